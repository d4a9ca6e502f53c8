"""Block-parallel scan counters (build with -DBPMD_BP_DIAG) on one 8-way C4
shard of this library's payloads:
    BPMD_LIB=beast_amd/libbeast_pmd_bpdiag.so python scripts/diag_bp_shard.py
"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from beast_amd import pmd, shard, synth  # noqa: E402


def main():
    lens_all = synth.zipf_sizes(bench.C4_MSGS, bench.SEED_C4)
    a, b = shard.byte_balanced_ranges(lens_all, 8)[0]
    lens = lens_all[a:b]
    raw, off, ln = synth.make_batch("json", lens, seed=bench.SEED_C4, first=a)
    src = pmd.Batch.from_arrays(raw, off.astype(np.int64), ln.astype(np.int32))
    d = pmd.deflate_batch(src, level=6, mem_level=4)
    torch.cuda.synchronize()
    comp = pmd.Batch(d.out.data, d.out.off, d.out.len)
    L = pmd.lib()
    c = (ctypes.c_ulonglong * 12)()
    pmd.inflate_batch(comp, src.len)
    torch.cuda.synchronize()
    L.bpmd_diag_bp_counters(c, 1)
    pmd.inflate_batch(comp, src.len)
    torch.cuda.synchronize()
    L.bpmd_diag_bp_counters(c, 1)
    names = ["payloads resolved", "segments on chains", "fallbacks", "-", "regions scanned", "stored found",
             "dynamic searches", "full header checks", "cyc stage", "cyc stored", "cyc dynamic", "-"]
    for i, nm in enumerate(names):
        print(f"  {nm:22s} {c[i]}")
    clen = d.out.len.cpu().numpy()
    print("compressed: max", clen.max(), "sum", clen.sum())


if __name__ == "__main__":
    main()
