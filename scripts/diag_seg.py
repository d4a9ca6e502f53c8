"""Lane-kernel role counters (prof build) for the long payloads of one 8-way
C4 shard, decoded by the lane kernel (mode 1) and block-parallel (mode 3):
    BPMD_LIB=beast_amd/libbeast_pmd_prof.so python scripts/diag_seg.py [min_len]
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
from beast_amd import pmd, shard, synth  # noqa: E402

NAMES = ["dec cycles", "dec iters", "dec sleeps", "dec hdr iters", "exp cycles", "exp iters", "exp sleeps",
         "lanes: header, ring not empty", "dec lap: input+tail", "dec lap: S_DATA", "dec lap: headers",
         "dec lap: publish+loop", "lanes: data, ring full", "lanes: data, room", "lanes: finished", "lanes: in headers"]


def main():
    min_len = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    lens_all = synth.zipf_sizes(bench.C4_MSGS, bench.SEED_C4)
    a, b = shard.byte_balanced_ranges(lens_all, 8)[0]
    lens = lens_all[a:b]
    keep = np.nonzero(lens >= min_len)[0]
    raw, off, ln = synth.make_batch("json", lens, seed=bench.SEED_C4, first=a)
    raw2 = np.concatenate([raw[int(off[i]):int(off[i]) + int(ln[i])] for i in keep])
    ln2 = ln[keep].astype(np.uint32)
    off2 = synth.offsets(ln2)
    dev = torch.device("cuda", 0)
    src = pmd.Batch.from_arrays(raw2, off2.astype(np.int64), ln2.astype(np.int32))
    d = pmd.deflate_batch(src, level=6, mem_level=4)
    torch.cuda.synchronize()
    comp = pmd.Batch(d.out.data, d.out.off, d.out.len)
    L = pmd.lib()
    c = (ctypes.c_ulonglong * 16)()
    total = int(ln2.astype(np.int64).sum())
    print(f"{len(keep)} payloads >= {min_len} B, {total / 2**20:.1f} MiB", flush=True)
    for mode, name in ((1, "lane"), (3, "bp")):
        L.bpmd_set_inflate_kernel(mode)
        rbuf = torch.empty_like(src.data)
        r = pmd.inflate_batch(comp, src.len, out=rbuf, out_off=src.off)
        torch.cuda.synchronize()
        ok = int((r.status != 0).sum()) == 0 and torch.equal(rbuf[:total], src.data[:total])
        L.bpmd_diag_lane3_counters(c, 1)
        t0 = time.perf_counter()
        pmd.inflate_batch(comp, src.len, out=rbuf, out_off=src.off)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        L.bpmd_diag_lane3_counters(c, 1)
        print(f"{name}: {dt * 1e3:.2f} ms ok {ok}", flush=True)
        for i in range(16):
            print(f"    {NAMES[i]:32s} {c[i]:16d}", flush=True)
    L.bpmd_set_inflate_kernel(0)


if __name__ == "__main__":
    main()
