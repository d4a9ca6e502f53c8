"""Diagnostic: per-phase cycle counters of the deflate kernel (prof build).

    python beast_amd/build.py prof
    BPMD_LIB=beast_amd/libbeast_pmd_prof.so python scripts/diag_deflate.py
"""
import ctypes
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from beast_amd import pmd, synth  # noqa: E402

NAMES = {0: "window+head init", 1: "hash chains", 2: "parse", 3: "repair+histogram", 4: "keys+sort",
         5: "merge (serial)", 6: "depths", 7: "limit+scatter", 8: "canonical codes", 9: "rle+bl tree (lane0)",
         10: "costs", 11: "stored emit", 12: "token bit count", 13: "zero+header (lane0)", 14: "token emit",
         15: "global copy", 18: "#chunks", 19: "chain steps (sum lanes)", 20: "chain steps (max lane)",
         21: "find calls (sum lanes)", 22: "parse iterations (max lane)",
         23: "parse iterations (sum lanes)", 16: "active parse lanes"}


def main():
    n = int(os.environ.get("DIAG_MSGS", "8192"))
    kind = os.environ.get("DIAG_KIND", "json")
    size = int(os.environ.get("DIAG_SIZE", "4096"))
    level = int(os.environ.get("DIAG_LEVEL", "6"))
    lens = np.full(n, size, dtype=np.uint32)
    raw, off, ln = synth.make_batch(kind, lens, seed=0x5EED0003)
    src = pmd.Batch.from_arrays(raw, off.astype(np.int64), ln.astype(np.int32))
    L = pmd.lib()
    L.bpmd_diag_deflate_counters.argtypes = [ctypes.c_void_p, ctypes.c_int]
    L.bpmd_diag_set_grid.argtypes = [ctypes.c_uint]
    L.bpmd_diag_set_grid(int(os.environ.get("DIAG_GRID", "0")))
    c = (ctypes.c_ulonglong * 24)()
    pmd.deflate_batch(src, level=level)
    torch.cuda.synchronize()
    L.bpmd_diag_deflate_counters(c, 1)
    t0 = time.perf_counter()
    r = pmd.deflate_batch(src, level=level)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    L.bpmd_diag_deflate_counters(c, 1)
    assert int((r.status != 0).sum()) == 0
    print(f"{n} msgs x {size} B {kind} L{level}: {dt * 1e3:.2f} ms, ratio {int(r.out.len.sum()) / (n * size):.4f}")
    for i in range(24):
        if i in NAMES:
            print(f"  {NAMES[i]:>24}: {c[i] / n:14.1f} per msg")


if __name__ == "__main__":
    main()
