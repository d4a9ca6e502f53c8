"""C5-shaped deflate (64 KiB binary, L6) and a C4 slice, a few launches each, for
rocprofv3 --kernel-trace --stats (per-kernel times of the chunk-parallel path)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from beast_amd import pmd, synth  # noqa: E402


def run(kind, lens, seed, level, reps=4):
    raw, off, ln = synth.make_batch(kind, lens, seed=seed)
    src = pmd.Batch.from_arrays(raw, off.astype(np.int64), ln.astype(np.int32))
    for _ in range(reps):
        d = pmd.deflate_batch(src, level=level)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        d = pmd.deflate_batch(src, level=level)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    total = int(ln.astype(np.int64).sum())
    ms = float(np.median(ts))
    print(f"{kind} n={len(ln)} {total / 2**20:.0f} MiB  {ms:.3f} ms  {total / 2**30 / (ms / 1e3):.2f} GiB/s "
          f"ok={int((d.status != 0).sum()) == 0}", flush=True)


if __name__ == "__main__":
    run("binary", np.full(4096, 65536, dtype=np.uint32), 0x5EED0005, 6)
    run("json", synth.zipf_sizes(131072, 0x5EED0004), 0x5EED0004, 6)
