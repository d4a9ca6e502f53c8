"""Host model of the GPU deflate algorithm (tests/model/deflate_model.cpp).

Test infrastructure: it states, in plain serial C++, exactly the parse /
Huffman / block-choice / framing the HIP kernel implements, so GPU output can
be checked byte for byte.  It is not the oracle (the oracle restates
Beast's own zlib); round trips and size tolerances are checked against the
oracle separately.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "deflate_model.cpp")
CSRC = os.path.join(HERE, "..", "..", "beast_amd", "csrc")
LIB = os.path.join(HERE, "_build", "libdmodel.so")
_L = None

# kernel constants (beast_amd/csrc/pmd_deflate.hip)
CHUNK, HBITS, LANES, MIN_SEG = 4096, 11, 64, 16


def build():
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    deps = [SRC, os.path.join(CSRC, "lz_core.h")]
    if os.path.exists(LIB) and os.path.getmtime(LIB) >= max(os.path.getmtime(d) for d in deps):
        return LIB
    tmp = "%s.%d.tmp" % (LIB, os.getpid())   # atomic under parallel test workers
    subprocess.run(["g++", "-O2", "-shared", "-fPIC", "-I", CSRC, SRC, "-o", tmp], check=True)
    os.replace(tmp, LIB)
    return LIB


def lib():
    global _L
    if _L is None:
        _L = ctypes.CDLL(build())
        vp = ctypes.c_void_p
        _L.dmodel_batch.restype = ctypes.c_int64
        _L.dmodel_batch.argtypes = [vp, vp, vp, ctypes.c_uint32] + [ctypes.c_int] * 9 + [vp, ctypes.c_uint64, vp, vp]
    return _L


def encode(data, off, lens, level=6, wbits=15, strategy=0):
    """Model payloads for the messages (data[off[i]:off[i]+lens[i]])."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.uint32)
    n = len(lens)
    if level == -1:
        level = 6
    wbits = 9 if wbits == 8 else wbits
    cap = int(lens.astype(np.int64).sum()) * 2 + 64 * n + 64
    out = np.zeros(cap, np.uint8)
    oo = np.zeros(n, np.uint64)
    ol = np.zeros(n, np.uint32)
    hist = lib().dmodel_chunk_hist(level)   # lz::chunk_hist (lz_core.h): 2 KiB, 4 KiB at levels >= 7
    r = lib().dmodel_batch(data.ctypes.data, off.ctypes.data, lens.ctypes.data, n, level, wbits, strategy, CHUNK,
                           hist, HBITS, LANES, MIN_SEG, 0, out.ctypes.data, cap, oo.ctypes.data, ol.ctypes.data)
    assert r >= 0
    return [out[int(oo[i]):int(oo[i]) + int(ol[i])].tobytes() for i in range(n)]
