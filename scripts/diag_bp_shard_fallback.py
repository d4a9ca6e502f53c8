"""Block-parallel fallbacks per call on the bench's virtual shards of a C5 leg,
the way bench.py runs them (whole batch deflated once, each shard's sub-batch
inflated: one warmup, then timed calls back to back), with the per-call wave-kernel
fallback count of the block-parallel path:
    python scripts/diag_bp_shard_fallback.py [level] [parts] [rounds]"""
import ctypes
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
    level = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    parts = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    lens = np.full(bench.C5_MSGS, 65536, np.uint32)
    raw, off, ln = synth.make_batch("binary", lens, seed=bench.SEED_C5)
    src = pmd.Batch.from_arrays(raw, off.astype(np.int64), ln.astype(np.int32))
    d = pmd.deflate_batch(src, level=level, mem_level=4)
    torch.cuda.synchronize()
    comp = pmd.Batch(d.out.data, d.out.off, d.out.len)
    rbuf = torch.empty_like(src.data)
    L = pmd.lib()
    L.bpmd_diag_bp_fallback.argtypes = [ctypes.c_void_p]
    c = (ctypes.c_ulonglong * 12)()
    r = pmd.inflate_batch(comp, src.len, out=rbuf, out_off=src.off)   # the whole batch first, as the bench
    torch.cuda.synchronize()
    for rnd in range(rounds):
        for k, (a, b) in enumerate(shard.byte_balanced_ranges(lens, parts)):
            sub = pmd.Batch(comp.data, comp.off[a:b], comp.len[a:b])
            line = []
            for call in range(4):   # warmup + 3
                L.bpmd_diag_bp_counters(c, 1)
                t0 = time.perf_counter()
                r = pmd.inflate_batch(sub, src.len[a:b], out=rbuf, out_off=src.off[a:b])
                torch.cuda.synchronize()
                dt = (time.perf_counter() - t0) * 1e3
                L.bpmd_diag_bp_counters(c, 1)
                ok = int((r.status != 0).sum()) == 0
                line.append(f"{dt:6.2f}ms fb{c[2]}{'' if ok else ' BAD'}")
            fb = (ctypes.c_uint32 * 8)()
            L.bpmd_diag_bp_fallback(fb)
            print(f"round {rnd} shard {k} [{a},{b}): " + "  ".join(line) +
                  f"  last fb: msg {fb[0]} seg {fb[1]} status {fb[2]} nsym {fb[3]} cap {fb[4]}", flush=True)


if __name__ == "__main__":
    main()
