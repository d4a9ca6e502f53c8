"""Host build of the exact-mode deflate kernel's own code (test
infrastructure).

beast_amd/csrc/pmd_deflate_exact.hip runs one message's deflater as
wave-uniform code with lane-strided bulk loops; everything up to the kernel
entry (the Dx state machine and exact_msg) is plain C++ once the HIP
intrinsics are given one-lane meanings (lane 0, WAVE = 1, ballot of one
lane).  This module compiles that same source text for the host with
clang++ so its decisions can be checked against the oracle in the CPU suite
and debugged without a GPU.  It is not the oracle and not a product path.
"""
import ctypes
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
KSRC = os.path.join(HERE, "..", "..", "beast_amd", "csrc", "pmd_deflate_exact.hip")
BUILD = os.path.join(HERE, "_build")
GEN = os.path.join(BUILD, "exact_host.cpp")
LIB = os.path.join(BUILD, "libexact_host.so")
CLANG = os.environ.get("BPMD_HOST_CLANG", "/opt/rocm/lib/llvm/bin/clang++")
_L = None

SHIM = r"""
#include <stdint.h>
#include <stddef.h>
#define __device__
#define __forceinline__ inline
#define __constant__
#define __restrict__
namespace bpmd {
enum Status : int32_t { ST_OK = 0, ST_NEED_BUFFERS = 1 };
constexpr int WAVE = 1;
inline unsigned lane_id() { return 0; }
}
static inline uint64_t __ballot(bool b) { return b ? 1ull : 0ull; }
#define __builtin_amdgcn_fence(a, b) ((void)0)
#define __builtin_amdgcn_readfirstlane(v) (v)
"""

DRIVER = r"""
}  // namespace dx
}  // namespace bpmd

extern "C" int32_t dx_host(int level, int wbits, int mem, int strategy, const uint8_t* msg, uint32_t len,
                           uint8_t* out, uint32_t cap)
{
    using namespace bpmd::dx;
    if (level == -1) level = 6;
    if (wbits == 8) wbits = 9;
    Cfg c;
    c.level = level;
    c.strategy = strategy;
    c.wbits = (uint32_t)wbits;
    c.hbits = (uint32_t)mem + 7;
    c.lit_bufsize = 1u << (mem + 6);
    static thread_local Trees T;
    const size_t w = (size_t)1 << wbits;
    uint8_t* win = new uint8_t[2 * w + MAXM + 64]();
    uint16_t* prv = new uint16_t[w]();
    uint16_t* hd = new uint16_t[(size_t)1 << c.hbits]();
    uint8_t* syms = new uint8_t[3 * (size_t)c.lit_bufsize]();
    const int32_t r = exact_msg(&T, win, prv, hd, syms, (uint32_t)w, msg, len, out, cap, c);
    delete[] win;
    delete[] prv;
    delete[] hd;
    delete[] syms;
    return r;
}
"""


def build():
    os.makedirs(BUILD, exist_ok=True)
    if os.path.exists(LIB) and os.path.getmtime(LIB) >= max(os.path.getmtime(KSRC), os.path.getmtime(__file__)):
        return LIB
    src = open(KSRC).read()
    body = src[:src.index("// LDS tiers by message length")]
    body = body.replace('#include "pmd_common.h"', "")
    # per-process names and an atomic rename: parallel test workers (pytest -n)
    # may build at once, and one must never load a half-written library
    gen, tmp = "%s.%d.cpp" % (GEN[:-4], os.getpid()), "%s.%d.tmp" % (LIB, os.getpid())
    with open(gen, "w") as f:
        f.write(SHIM + body + DRIVER)
    subprocess.run([CLANG, "-O2", "-std=c++17", "-shared", "-fPIC", "-Wno-unused-function", gen, "-o", tmp],
                   check=True)
    os.replace(tmp, LIB)
    os.remove(gen)
    return LIB


def lib():
    global _L
    if _L is None:
        _L = ctypes.CDLL(build())
        _L.dx_host.restype = ctypes.c_int32
        _L.dx_host.argtypes = [ctypes.c_int] * 4 + [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_void_p,
                                                   ctypes.c_uint32]
    return _L


def deflate(msg: bytes, level=6, wbits=15, mem=4, strategy=0, cap=None):
    """(status, payload): status 0, or 1 (need_buffers) as the kernel reports."""
    if cap is None:
        cap = len(msg) + ((len(msg) + 7) >> 3) + ((len(msg) + 63) >> 6) + 11
    out = ctypes.create_string_buffer(max(cap, 1))
    r = lib().dx_host(level, wbits, mem, strategy, msg, len(msg), out, cap)
    return (1, b"") if r < 0 else (0, out.raw[:r])
