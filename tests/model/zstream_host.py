"""Host build of the per-stream inflate kernel's own code (test
infrastructure).

beast_amd/csrc/pmd_zstream.hip runs Beast's inflate_stream state machine as
wave-uniform code (zstream_run) with lane-strided bulk loops.  With
BPMD_ZSTREAM_HOST and one-lane meanings of the HIP intrinsics (lane 0,
WAVE = 1, readfirstlane = identity) that same source text is plain C++; the
wave-cooperative table builder is replaced by the serial builder it is
slot-for-slot equal to (huff_table.h; the equality is tests/test_gpu_tables.py).
This module compiles it for the host so the CPU suite can check every
write()'s z_params against the oracle without a GPU.  It is not the oracle
and not a product path.
"""
import ctypes
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "..", "..", "beast_amd", "csrc")
KSRC = os.path.join(CSRC, "pmd_zstream.hip")
BUILD = os.path.join(HERE, "_build")
SHIM = os.path.join(BUILD, "zstream_shim.h")
GEN = os.path.join(BUILD, "zstream_host.cpp")
LIB = os.path.join(BUILD, "libzstream_host.so")
CXX = os.environ.get("BPMD_HOST_CXX", "g++")
_L = None

SHIM_TEXT = r"""
#pragma once
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#include <stdlib.h>
#include <stdio.h>
#define __device__
#define __host__
#define __forceinline__ inline
#define __constant__
#define __global__
#define __builtin_amdgcn_readfirstlane(v) (v)
struct uint4 { uint32_t x, y, z, w; };
#include "huff_table.h"
namespace bpmd {
enum Status : int32_t {
    ST_OK = 0, ST_NEED_BUFFERS = 1, ST_END_OF_STREAM = 2, ST_NEED_DICT = 3, ST_STREAM_ERROR = 4,
    ST_INVALID_BLOCK_TYPE = 5, ST_INVALID_STORED_LENGTH = 6, ST_TOO_MANY_SYMBOLS = 7,
    ST_INVALID_CODE_LENGTHS = 8, ST_INVALID_BIT_LENGTH_REPEAT = 9, ST_MISSING_EOB = 10,
    ST_INVALID_LITERAL_LENGTH = 11, ST_INVALID_DISTANCE_CODE = 12, ST_INVALID_DISTANCE = 13,
    ST_OVER_SUBSCRIBED_LENGTH = 14, ST_INCOMPLETE_LENGTH_SET = 15, ST_GENERAL = 16,
};
constexpr int WAVE = 1;
inline unsigned lane_id() { return 0; }
inline void wave_sync() {}
static const uint16_t kLenBase[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31,
                                      35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
static const uint8_t kLenExtra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3,
                                      4, 4, 4, 4, 5, 5, 5, 5, 0};
static const uint16_t kDistBase[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193,
                                       257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145,
                                       8193, 12289, 16385, 24577};
static const uint8_t kDistExtra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8,
                                       9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
struct WaveTableScratch { uint16_t sorted[320]; };
// the serial builder the wave-cooperative one equals
template <int TYPE>
inline int build_table_wave(const uint8_t* lens, unsigned n, uint16_t* tab, unsigned req_root,
                            WaveTableScratch& S, unsigned& root_out, unsigned& used_out, unsigned& lmin_out)
{
    unsigned root = req_root, used = 0;
    const int r = build_table(TYPE, lens, n, tab, &root, &used, S.sorted, &lmin_out);
    if (r) return r;
    root_out = root;
    used_out = used;
    return 0;
}
}  // namespace bpmd
"""

DRIVER = r"""
extern "C" size_t zs_host_state_bytes(void) { return sizeof(bpmd::zst::State); }

extern "C" void zs_host_reset(void* st, int wbits)
{
    bpmd::zst::State* s = (bpmd::zst::State*)st;
    memset(&s->h, 0, sizeof s->h);
    s->h.mode = bpmd::zst::HEAD;
    s->h.wbits = (uint32_t)wbits;
}

// one write(): returns the zlib::error; res = {in_used, out_used, ec, data_type, published}
extern "C" int zs_host_write(void* st, const uint8_t* in, uint64_t n, uint8_t* out, uint64_t cap, int flush,
                             void* res)
{
    static thread_local bpmd::zst::Lds L;
    // BPMD_ZSTREAM_PAR=0: the serial inflate_fast loop (default: the parallel one, one lane)
    const char* e = getenv("BPMD_ZSTREAM_PAR");
    const char* hp = getenv("BPMD_ZSTREAM_HPAR");   // 0: the serial code-length loop
    const int par = (e ? atoi(e) != 0 : 1) | (hp && hp[0] == '0' ? 8 : 0);
    bpmd::zst::zstream_run(L, (bpmd::zst::State*)st, in, n, out, cap, flush, (bpmd::zst::Result*)res, par);
    return ((bpmd::zst::Result*)res)->ec;
}
"""


def build():
    os.makedirs(BUILD, exist_ok=True)
    deps = [KSRC, os.path.join(CSRC, "zstream.h"), os.path.join(CSRC, "huff_table.h"), __file__]
    if os.path.exists(LIB) and os.path.getmtime(LIB) >= max(os.path.getmtime(d) for d in deps):
        return LIB
    with open(SHIM, "w") as f:
        f.write(SHIM_TEXT)
    with open(GEN, "w") as f:
        f.write('#include "pmd_zstream.hip"\n' + DRIVER)
    cmd = [CXX, "-O1", "-g", *os.environ.get("ZS_HOST_FLAGS", "").split(), "-std=c++17", "-fPIC", "-shared", "-DBPMD_ZSTREAM_HOST", "-x", "c++",
           "-include", SHIM, "-I", CSRC, "-o", LIB, GEN]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("host build of pmd_zstream.hip failed:\n" + r.stderr)
    return LIB


class Result(ctypes.Structure):
    _fields_ = [("in_used", ctypes.c_uint64), ("out_used", ctypes.c_uint64), ("ec", ctypes.c_int32),
                ("data_type", ctypes.c_int32), ("published", ctypes.c_int32), ("pad", ctypes.c_int32)]


def lib():
    global _L
    if _L is None:
        L = ctypes.CDLL(build())
        vp = ctypes.c_void_p
        L.zs_host_state_bytes.restype = ctypes.c_size_t
        L.zs_host_reset.argtypes = [vp, ctypes.c_int]
        L.zs_host_write.argtypes = [vp, vp, ctypes.c_uint64, vp, ctypes.c_uint64, ctypes.c_int,
                                    ctypes.POINTER(Result)]
        _L = L
    return _L


class HostInflater:
    """Drives the host build exactly as pmd_stream.hip drives the kernel
    (same output-room bound, same z_params updates)."""

    def __init__(self, wbits=15):
        self.L = lib()
        self.st = ctypes.create_string_buffer(self.L.zs_host_state_bytes())
        self.L.zs_host_reset(self.st, wbits)

    def reset(self, wbits=15):
        self.L.zs_host_reset(self.st, wbits)

    def write(self, zs, flush):
        n = zs.avail_in
        cap = min(zs.avail_out, 1040 * n + 8192)
        src = ctypes.create_string_buffer(ctypes.string_at(zs.next_in, n) if n else b"", n + 64)
        dst = ctypes.create_string_buffer(cap + 64)
        res = Result()
        self.L.zs_host_write(self.st, src, n, dst, cap, flush, ctypes.byref(res))
        if res.out_used:
            ctypes.memmove(zs.next_out, dst, res.out_used)
        if res.published:
            zs.next_in = (zs.next_in or 0) + res.in_used
            zs.avail_in -= res.in_used
            zs.total_in += res.in_used
            zs.next_out = (zs.next_out or 0) + res.out_used
            zs.avail_out -= res.out_used
            zs.total_out += res.out_used
            zs.data_type = res.data_type
        return res.ec
