"""This library's own payloads (GPU deflate, sync markers) on one shard of
C4 (L6) or C5 (L1 / L6): timing per call and the block-parallel counters.
    python scripts/diag_own_shard.py c4 6 8 [reps]
"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from beast_amd import pmd, shard, synth  # noqa: E402


def main():
    leg, level, parts = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 3
    if leg == "c4":
        lens_all, kind, seed = synth.zipf_sizes(bench.C4_MSGS, bench.SEED_C4), "json", bench.SEED_C4
    else:
        lens_all, kind, seed = np.full(bench.C5_MSGS, 65536, np.uint32), "binary", bench.SEED_C5
    a, b = shard.byte_balanced_ranges(lens_all, parts)[0] if parts > 1 else (0, len(lens_all))
    lens = lens_all[a:b]
    raw, off, ln = synth.make_batch(kind, lens, seed=seed, first=a)
    src = pmd.Batch.from_arrays(raw, off.astype(np.int64), ln.astype(np.int32))
    d = pmd.deflate_batch(src, level=level, mem_level=4)
    torch.cuda.synchronize()
    comp = pmd.Batch(d.out.data, d.out.off, d.out.len)
    out = torch.empty_like(src.data)
    total = int(ln.astype(np.int64).sum())
    print(f"own {leg} L{level} 1/{parts}: {len(lens)} msgs, {total / 2**20:.1f} MiB", flush=True)
    for r in range(reps):
        pmd.bp_counters(reset=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res = pmd.inflate_batch(comp, src.len, out=out, out_off=src.off)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        c = pmd.bp_counters(reset=True)
        ok = int((res.status != 0).sum()) == 0 and torch.equal(out, src.data)
        print(f"  call {r}: {dt * 1e3:.3f} ms ({total / 2**30 / dt:.1f} GiB/s) ok={ok} bp resolved {c[0]} "
              f"segments {c[1]} fallback {c[2]} spill {c[3]}", flush=True)


if __name__ == "__main__":
    main()
