"""Beast-produced payloads (host zlib = Beast's deflate_stream) on one shard
of C4 (L6) or C5 (L1 / L6): timing per call and the block-parallel counters.
Run under rocprofv3 --kernel-trace --stats for the per-kernel split.
    python scripts/diag_beast_shard.py c5 1 8 [reps] [shard]     (leg, level, parts)
    BPMD_LIB=beast_amd/libbeast_pmd_bpdiag.so ... for the scan counters
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


def main():
    leg, level, parts = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 3
    which = int(sys.argv[5]) if len(sys.argv) > 5 else 0   # the shard (of `parts`)
    if leg == "c4":
        lens_all, kind, seed = synth.zipf_sizes(bench.C4_MSGS, bench.SEED_C4), "json", bench.SEED_C4
    else:
        lens_all, kind, seed = np.full(bench.C5_MSGS, 65536, np.uint32), "binary", bench.SEED_C5
    a, b = shard.byte_balanced_ranges(lens_all, parts)[which] if parts > 1 else (0, len(lens_all))
    lens = lens_all[a:b]
    raw, off, ln = synth.make_batch(kind, lens, seed=seed, first=a)
    payloads, _ = bench.beast_payloads(raw, off, ln, level)
    buf, boff, blen = bench.pack(payloads)
    dev = torch.device("cuda", 0)
    src = pmd.Batch(torch.from_numpy(buf).to(dev), torch.from_numpy(boff).to(dev), torch.from_numpy(blen).to(dev))
    cap = torch.from_numpy(ln.astype(np.int32)).to(dev)
    ooff = torch.from_numpy(off.astype(np.int64)).to(dev)
    out = torch.empty(int(ln.astype(np.int64).sum()) + 64, dtype=torch.uint8, device=dev)
    ref = torch.from_numpy(raw).to(dev)
    print(f"{leg} L{level} 1/{parts}: {len(lens)} msgs, {ln.astype(np.int64).sum() / 2**20:.1f} MiB, "
          f"compressed {blen.astype(np.int64).sum() / 2**20:.1f} MiB", flush=True)
    for r in range(reps):
        pmd.bp_counters(reset=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res = pmd.inflate_batch(src, cap, out=out, out_off=ooff)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        c = pmd.bp_counters(reset=True)
        fb = (ctypes.c_uint32 * 8)()
        pmd.lib().bpmd_diag_bp_fallback(fb)
        ok = int((res.status != 0).sum()) == 0 and torch.equal(out[:ref.numel()], ref)
        print(f"  call {r}: {dt * 1e3:.3f} ms ({ln.astype(np.int64).sum() / 2**30 / dt:.1f} GiB/s) ok={ok} "
              f"bp resolved {c[0]} segments {c[1]} fallback {c[2]} spill {c[3]} | scan regions {c[4]} stored {c[5]} "
              f"dyn-searched {c[6]} full-checks {c[7]} cyc stage/stored/dyn {c[8]}/{c[9]}/{c[10]} | last fallback: "
              f"msg {fb[0]} seg {fb[1]} status {fb[2]} nsym {fb[3]} cap {fb[4]} next {fb[5]} bit {fb[6]} kind {fb[7]}",
              flush=True)


if __name__ == "__main__":
    main()
