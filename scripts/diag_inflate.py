"""Diagnostic: per-phase cycle counters of the inflate kernel (prof build).

    python beast_amd/build.py prof
    BPMD_LIB=beast_amd/libbeast_pmd_prof.so python scripts/diag_inflate.py
"""
import ctypes
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from beast_amd import pmd, synth  # noqa: E402

NAMES = {0: "-", 1: "fixed/other hdr", 2: "passA", 3: "passB+fix", 4: "scan+passC", 5: "expand",
         6: "#rounds", 7: "#passB iters", 8: "#blocks", 9: "#ptrjump iters", 10: "window load", 11: "#window loads",
         12: "final flush", 13: "passA trips", 14: "passB trips", 15: "passC trips", 16: "clen table",
         17: "clen decode", 18: "lens table", 19: "dists table", 20: "hdr fields", 21: "-", 22: "-", 23: "-"}


def main():
    n = int(os.environ.get("DIAG_MSGS", "8192"))
    kind = os.environ.get("DIAG_KIND", "json")
    size = int(os.environ.get("DIAG_SIZE", "4096"))
    lens = np.full(n, size, dtype=np.uint32)
    raw, off, ln = synth.make_batch(kind, lens, seed=0x5EED0002)
    payloads = bench.pmd_compress_host(raw, off, ln)
    buf, coff, clen = bench.pack(payloads)
    dev = torch.device("cuda", 0)
    src = pmd.Batch(torch.from_numpy(buf).to(dev), torch.from_numpy(coff).to(dev), torch.from_numpy(clen).to(dev))
    L = pmd.lib()
    L.bpmd_diag_counters.argtypes = [ctypes.c_void_p, ctypes.c_int]
    L.bpmd_diag_set_grid.argtypes = [ctypes.c_uint]
    L.bpmd_diag_set_grid(int(os.environ.get("DIAG_GRID", "0")))
    c = (ctypes.c_ulonglong * 24)()
    r = pmd.inflate_batch(src, size)
    torch.cuda.synchronize()
    print("reset rc", L.bpmd_diag_counters(c, 1), flush=True)
    t0 = time.perf_counter()
    r = pmd.inflate_batch(src, size)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    L.bpmd_diag_counters(c, 1)
    assert int((r.status != 0).sum()) == 0
    print(f"{n} msgs x {size} B {kind}: {dt * 1e3:.2f} ms, ratio {clen.sum() / (n * size):.3f}")
    tot = 0
    for i in range(24):
        if NAMES[i] != "-":
            print(f"  {NAMES[i]:>16}: {c[i] / n:14.1f} per msg")
    d = (ctypes.c_ulonglong * 24)()
    L.bpmd_diag_counters(d, 2)
    print("debug record:", list(d)[:16])


if __name__ == "__main__":
    main()
