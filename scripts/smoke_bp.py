"""A few block-parallel inflate calls (forced mode) with progress lines, to
check a new build quickly before the test suite."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from beast_amd import pmd, synth  # noqa: E402

L = pmd.lib()
for kind, n, size in (("json", 16, 40960), ("binary", 64, 65536), ("json", 2048, 16384)):
    lens = np.full(n, size, dtype=np.uint32)
    raw, off, ln = synth.make_batch(kind, lens, seed=7)
    src = pmd.Batch.from_arrays(raw, off.astype(np.int64), ln.astype(np.int32))
    d = pmd.deflate_batch(src, level=6, mem_level=4)
    torch.cuda.synchronize()
    print(f"{kind} {n}x{size}: deflated", flush=True)
    comp = pmd.Batch(d.out.data, d.out.off, d.out.len)
    L.bpmd_set_inflate_kernel(3)
    t0 = time.perf_counter()
    r = pmd.inflate_batch(comp, size)
    torch.cuda.synchronize()
    ok = int((r.status != 0).sum()) == 0 and torch.equal(r.out.data[:n * size].view(n, size), src.data[:n * size].view(n, size))
    print(f"  bp inflate {1e3 * (time.perf_counter() - t0):.2f} ms ok {ok}", flush=True)
    L.bpmd_set_inflate_kernel(0)
    assert ok
print("smoke_bp ok", flush=True)
