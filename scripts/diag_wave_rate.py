"""Per-message decode rate of the two inflate kernels on one GPU: batches of
n messages of `size` bytes (json or binary, Beast's pmd payloads at L6/mem4),
forced to the wave kernel (and its round modes) or the lane kernel.
    python scripts/diag_wave_rate.py
"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from beast_amd import pmd, synth  # noqa: E402


def run(kind, n, size, kernel, walk, level=6):
    lens = np.full(n, size, dtype=np.uint32)
    raw, off, ln = synth.make_batch(kind, lens, seed=0x5EED00D1)
    src = pmd.Batch.from_arrays(raw, off.astype(np.int64), ln.astype(np.int32))
    d = pmd.deflate_batch(src, level=level, mem_level=4, exact=True)   # Beast's own block structure
    torch.cuda.synchronize()
    comp = pmd.Batch(d.out.data, d.out.off, d.out.len)
    L = pmd.lib()
    L.bpmd_set_inflate_kernel(kernel)
    L.bpmd_diag_set_wave_walk(walk)
    r = pmd.inflate_batch(comp, size)
    torch.cuda.synchronize()
    ok = int((r.status != 0).sum()) == 0 and torch.equal(r.out.data[:n * size].view(n, size)[:, :size],
                                                         src.data[:n * size].view(n, size))
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        pmd.inflate_batch(comp, size)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    t = float(np.median(ts))
    L.bpmd_set_inflate_kernel(0)
    L.bpmd_diag_set_wave_walk(0)
    name = {1: "lane", 2: "wave"}[kernel] + ("" if kernel == 1 else {0: "/auto", 1: "/walk", 2: "/spec"}[walk])
    print(f"{kind:6s} n={n:6d} size={size:6d} L{level} {name:10s} {t * 1e3:8.3f} ms  "
          f"{n * size / t / 2**30:7.2f} GiB/s  per-msg-wave {t * 1e3 * 2304 / max(n, 1):.3f} ms  ok={ok}", flush=True)


if __name__ == "__main__":
    for kind, n, size in (("json", 2304, 40960), ("json", 9216, 40960), ("json", 16384, 4096),
                          ("binary", 2304, 65536), ("binary", 16384, 65536)):
        for kernel, walk in ((2, 0), (2, 2), (2, 1), (1, 0)):
            if kernel == 1 and n * size > 600 << 20:
                continue
            run(kind, n, size, kernel, walk)
    run("binary", 16384, 65536, 2, 0, level=1)
