"""Seeded synthetic payload batches for the benches and tests.

Thin ctypes layer over csrc/synth.c ("Synthetic inputs").
A batch is the struct-of-arrays layout the C-ABI takes: one contiguous byte
buffer plus per-message uint64 offsets and uint32 lengths.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

KINDS = {"json": 0, "corpus1": 1, "random": 2, "binary": 3, "zeros": 4}


def _lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "libbpmd_synth.so")
        if not os.path.exists(path):
            subprocess.run(["gcc", "-O2", "-fPIC", "-shared", "-o", path,
                            os.path.join(_HERE, "csrc", "synth.c"), "-lm"], check=True)
        L = ctypes.CDLL(path)
        L.bpmd_synth_fill.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.bpmd_synth_zipf_sizes.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                                            ctypes.c_void_p]
        _LIB = L
    return _LIB


def offsets(lens: np.ndarray, align: int = 1) -> np.ndarray:
    """Exclusive prefix sum of lengths (each slot rounded up to `align`)."""
    lens = np.asarray(lens, dtype=np.uint64)
    if align > 1:
        lens = (lens + (align - 1)) // align * align
    off = np.zeros(len(lens), dtype=np.uint64)
    if len(lens):
        off[1:] = np.cumsum(lens[:-1])
    return off


def zipf_sizes(n: int, seed: int, first: int = 0) -> np.ndarray:
    out = np.zeros(n, dtype=np.uint32)
    _lib().bpmd_synth_zipf_sizes(seed, first, n, out.ctypes.data_as(ctypes.c_void_p))
    return out


def make_batch(kind: str, lens, seed: int, first: int = 0):
    """Returns (data uint8, off uint64, lens uint32) for messages
    [first, first + len(lens))."""
    lens = np.ascontiguousarray(lens, dtype=np.uint32)
    off = offsets(lens)
    total = int(lens.astype(np.uint64).sum())
    data = np.zeros(max(total, 1), dtype=np.uint8)
    r = _lib().bpmd_synth_fill(KINDS[kind], seed, first, len(lens), off.ctypes.data_as(ctypes.c_void_p),
                               lens.ctypes.data_as(ctypes.c_void_p), data.ctypes.data_as(ctypes.c_void_p))
    if r:
        raise ValueError(kind)
    return data, off, lens
