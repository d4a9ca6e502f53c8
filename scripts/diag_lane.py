"""Diagnostic: per-wave loop counters of the lane-per-message inflate kernel
(prof build).

    python beast_amd/build.py prof
    BPMD_LIB=beast_amd/libbeast_pmd_prof.so python scripts/diag_lane.py
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

NAMES = {0: "wave cycles", 1: "iterations", 2: "lanes alive/iter", 3: "iters w/ decode", 4: "lanes decoding/iter",
         5: "iters w/ copy", 6: "iters w/ header", 7: "lanes in header/iter", 8: "cyc A decode", 9: "cyc B store",
         10: "cyc C+D headers", 11: "cyc E copy", 12: "lanes decoding after copy issue", 13: "iters w/ pass1", 14: "iters w/ pass2", 15: "cyc loop top"}


def main():
    n = int(os.environ.get("DIAG_MSGS", "65536"))
    kind = os.environ.get("DIAG_KIND", "json")
    size = int(os.environ.get("DIAG_SIZE", "4096"))
    lens = np.full(n, size, dtype=np.uint32)
    raw, off, ln = synth.make_batch(kind, lens, seed=0x5EED0002)
    payloads = bench.pmd_compress_host(raw, off, ln)
    buf, coff, clen = bench.pack(payloads)
    dev = torch.device("cuda", 0)
    src = pmd.Batch(torch.from_numpy(buf).to(dev), torch.from_numpy(coff).to(dev), torch.from_numpy(clen).to(dev))
    L = pmd.lib()
    L.bpmd_diag_lane_counters.argtypes = [ctypes.c_void_p, ctypes.c_int]
    L.bpmd_set_inflate_kernel(1)
    c = (ctypes.c_ulonglong * 16)()
    r = pmd.inflate_batch(src, size)
    torch.cuda.synchronize()
    L.bpmd_diag_lane_counters(c, 1)
    t0 = time.perf_counter()
    r = pmd.inflate_batch(src, size)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    L.bpmd_diag_lane_counters(c, 1)
    assert int((r.status != 0).sum()) == 0
    waves = (n + 63) // 64
    it = c[1] / waves
    print(f"{n} msgs x {size} B {kind}: {dt * 1e3:.2f} ms, ratio {clen.sum() / (n * size):.3f}, waves {waves}")
    for i in range(16):
        if i in NAMES:
            v = c[i] / waves
            extra = f"  ({v / it:8.2f} per iter)" if i in (2, 4, 7, 8, 9, 10, 11, 15) else ""
            print(f"  {NAMES[i]:>22}: {v:14.1f} per wave{extra}")


if __name__ == "__main__":
    main()
