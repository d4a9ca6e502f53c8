"""One op of one bench leg, alone, for rocprofv3 (scripts/profile_legs.sh):
the leg's inputs are built as bench.py builds them, the op runs once untimed
and then --steps times, and nothing else touches the GPU except the setup
(for an inflate op: one deflate of the same batch, whose kernels have other
names).  So the kernel trace and the FETCH_SIZE / WRITE_SIZE passes of this
process are the op's own.

    python scripts/leg_profile.py --leg c4_l6 --op inflate --steps 5
legs: c3 (deflate only), c4_l6, c5_l1, c5_l6; a suffix _s8 takes shard 0 of
the byte-balanced 8-way split (what one rank of an 8-GPU node runs)
"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from beast_amd import pmd, synth  # noqa: E402

LEGS = {"c4_l6": ("json", None, bench.SEED_C4, 6), "c5_l1": ("binary", 65536, bench.SEED_C5, 1),
        "c5_l6": ("binary", 65536, bench.SEED_C5, 6), "c3": ("json", 4096, bench.SEED_C3, 6)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--leg", required=True, choices=sorted(LEGS) + [k + "_s8" for k in LEGS if k != "c3"])
    ap.add_argument("--op", required=True, choices=["deflate", "inflate"])
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    base = a.leg[:-3] if a.leg.endswith("_s8") else a.leg
    kind, size, seed, level = LEGS[base]
    first = 0
    if base == "c4_l6":
        lens = synth.zipf_sizes(bench.C4_MSGS, seed)
    elif a.leg == "c3":
        lens = np.full(bench.N_MSGS, size, dtype=np.uint32)
    else:
        lens = np.full(bench.C5_MSGS, size, dtype=np.uint32)
    if a.leg.endswith("_s8"):
        from beast_amd import shard
        first, e = shard.byte_balanced_ranges(lens, 8)[0]
        lens = lens[first:e]
    dev = torch.device("cuda", 0)
    raw, off, ln = synth.make_batch(kind, lens, seed=seed, first=first)
    src = pmd.Batch(torch.from_numpy(raw).to(dev), torch.from_numpy(off.astype(np.int64)).to(dev),
                    torch.from_numpy(ln.astype(np.int32)).to(dev))
    del raw
    l64 = lens.astype(np.int64)
    cap = torch.from_numpy((l64 + (l64 + 7) // 8 + (l64 + 63) // 64 + 11).astype(np.int32)).to(dev)
    coff = pmd.slot_offsets(cap)
    cbuf = torch.empty(int(coff[-1].item()) + int(cap[-1].item()) + 64, dtype=torch.uint8, device=dev)

    def deflate():
        return pmd.deflate_batch(src, level=level, mem_level=4, out_cap=cap, out=cbuf, out_off=coff)

    d = deflate()
    torch.cuda.synchronize()
    if a.op == "deflate":
        for _ in range(a.steps):
            deflate()
        torch.cuda.synchronize()
        print("deflate steps", a.steps, "status_ok", int((d.status != 0).sum()) == 0)
        return
    comp = pmd.Batch(cbuf, coff, d.out.len.clone())
    rbuf = torch.empty_like(src.data)

    def inflate():
        return pmd.inflate_batch(comp, src.len, out=rbuf, out_off=src.off)

    import ctypes
    L = pmd.lib()
    c = (ctypes.c_ulonglong * 12)()
    L.bpmd_diag_bp_counters(c, 1)
    r = inflate()
    for _ in range(a.steps):
        inflate()
    torch.cuda.synchronize()
    L.bpmd_diag_bp_counters(c, 1)
    runs = a.steps + 1
    print(a.leg, "inflate steps", a.steps, "status_ok", int((r.status != 0).sum()) == 0, "msgs", len(lens),
          "bp payloads/run", c[0] // runs, "segments/run", c[1] // runs, "wave fallbacks/run", c[2] / runs)


if __name__ == "__main__":
    main()
