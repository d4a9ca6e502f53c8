"""Which C5 payload falls back from block-parallel to the wave kernel, and why
(segment status / symbols / slot of the last fallback):
    python scripts/diag_bp_fallback.py [level]
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
    level = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    lens_all = np.full(bench.C5_MSGS, 65536, np.uint32)
    L = pmd.lib()
    L.bpmd_diag_bp_fallback.argtypes = [ctypes.c_void_p]
    for a, b in shard.byte_balanced_ranges(lens_all, 8):
        lens = lens_all[a:b]
        raw, off, ln = synth.make_batch("binary", lens, seed=bench.SEED_C5, first=a)
        src = pmd.Batch.from_arrays(raw, off.astype(np.int64), ln.astype(np.int32))
        d = pmd.deflate_batch(src, level=level, mem_level=4)
        torch.cuda.synchronize()
        comp = pmd.Batch(d.out.data, d.out.off, d.out.len)
        c = (ctypes.c_ulonglong * 12)()
        L.bpmd_diag_bp_counters(c, 1)
        r = pmd.inflate_batch(comp, src.len)
        torch.cuda.synchronize()
        L.bpmd_diag_bp_counters(c, 1)
        fb = (ctypes.c_uint32 * 8)()
        L.bpmd_diag_bp_fallback(fb)
        ok = int((r.status != 0).sum()) == 0
        print(f"shard [{a}, {b}) ok {ok} fallbacks {c[2]} last: msg {a + fb[0] if c[2] else '-'} seg {fb[1]} "
              f"status {fb[2]} nsym {fb[3]} cap {fb[4]} next {fb[5]} bit {fb[6]} kind {fb[7]} "
              f"comp_len {int(d.out.len[fb[0]]) if c[2] else '-'}", flush=True)


if __name__ == "__main__":
    main()
