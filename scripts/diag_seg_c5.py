"""Lane-kernel role counters (prof build) of the segment kernel on C5 (64 KiB
binary, L1): this library's payloads against a Beast peer's (host zlib,
memLevel 4), the whole batch or one 8-way shard:
    BPMD_LIB=beast_amd/libbeast_pmd_prof.so python scripts/diag_seg_c5.py [parts]
Counter sums over all waves of the call (bpmd_diag_lane3_counters24)."""
import ctypes
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("BPMD_LIB", os.path.join(ROOT, "beast_amd", "libbeast_pmd_prof.so"))
import bench  # noqa: E402
from beast_amd import pmd, shard, synth  # noqa: E402

NAMES = ["dec cycles", "dec iters", "dec sleeps", "dec hdr iters", "exp cycles", "exp iters", "exp sleeps",
         "lanes: header, ring not empty", "dec lap: input+tail", "dec lap: S_DATA", "dec lap: headers",
         "dec lap: publish+loop", "lanes: data, ring full", "lanes: data, room", "lanes: finished",
         "lanes: in headers", "hdr: type/stored/copy", "hdr: table+lenlens", "hdr: codelens", "hdr: build",
         "hdr: place"]


def main():
    parts = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    lens_all = np.full(bench.C5_MSGS, 65536, np.uint32)
    a, b = shard.byte_balanced_ranges(lens_all, parts)[0] if parts > 1 else (0, len(lens_all))
    lens = lens_all[a:b]
    raw, off, ln = synth.make_batch("binary", lens, seed=bench.SEED_C5, first=a)
    dev = torch.device("cuda", 0)
    src = pmd.Batch.from_arrays(raw, off.astype(np.int64), ln.astype(np.int32))
    total = int(ln.astype(np.int64).sum())
    d = pmd.deflate_batch(src, level=1, mem_level=4)
    torch.cuda.synchronize()
    own = pmd.Batch(d.out.data, d.out.off, d.out.len)
    bp_list, _ = bench.beast_payloads(raw, off, ln, 1)
    bbuf, boff, blen = bench.pack(bp_list)
    beast = pmd.Batch(torch.from_numpy(bbuf).to(dev), torch.from_numpy(boff).to(dev), torch.from_numpy(blen).to(dev))
    L = pmd.lib()
    c = (ctypes.c_ulonglong * 24)()
    rows = {}
    for name, comp in (("own", own), ("beast", beast)):
        rbuf = torch.empty_like(src.data)
        pmd.inflate_batch(comp, src.len, out=rbuf, out_off=src.off)
        torch.cuda.synchronize()
        L.bpmd_diag_lane3_counters24(c, 1)
        t0 = time.perf_counter()
        r = pmd.inflate_batch(comp, src.len, out=rbuf, out_off=src.off)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        L.bpmd_diag_lane3_counters24(c, 1)
        ok = int((r.status != 0).sum()) == 0 and torch.equal(rbuf[:total], src.data[:total])
        rows[name] = list(c)
        print(f"{name}: {len(lens)} msgs, {dt * 1e3:.3f} ms, exact {ok}", flush=True)
    print(f"{'counter':32s} {'own':>16s} {'beast':>16s} {'beast/own':>10s}")
    for i, nm in enumerate(NAMES):
        o, bv = rows["own"][i], rows["beast"][i]
        print(f"{nm:32s} {o:16d} {bv:16d} {bv / o if o else float('nan'):10.2f}")
    # per-task records (prof build, g_l3hprof[5-7]): the longest task by
    # lifetime and by decoder iterations (task index, its result), and the
    # 4-byte stored-copy steps of all tasks
    for name in ("own", "beast"):
        r = rows[name]
        t5, t6 = r[21], r[22]
        print(f"{name}: longest task {t5 & 0x1ffff} (result {(t5 >> 17) & 0x7f}) {t5 >> 24} cycles; "
              f"most iterations task {t6 & 0x1ffff} (result {(t6 >> 17) & 0x7f}) {t6 >> 24}; "
              f"stored-copy steps {r[23]}")


if __name__ == "__main__":
    main()
