#!/usr/bin/env python3
"""Benchmark: device-resident permessage-deflate throughput on MI355X.

Workload (BASELINE.json configs[1], "C2"): 64 Ki independent 4 KiB JSON-like
WebSocket payloads per GPU, compressed with compLevel=6, memLevel=4,
windowBits=15 and Beast's pmd framing (impl_base.hpp:85-154), resident in HBM.
One step = one batched inflate launch over the whole batch.  The C3 round
trip (GPU deflate + GPU inflate of the same shape) is reported alongside.

Launch:  python bench.py [--gpus N --steps K --warmup W]
N > 1 runs under torch.distributed.run: every rank inflates its own 64 Ki
messages (messages are independent streams under no_context_takeover), so
there is no collective on the data path; scaling is weak.  Timing is
barrier + synchronize on both sides, max over ranks.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
import zlib

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from beast_amd import pmd, synth  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
N_MSGS = 1 << 16
MSG_BYTES = 4096
SEED = 0x5EED0002


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def pmd_compress_host(data, off, lens, level=6, wbits=15, mem=4):
    """Inputs for the inflate benchmark, produced the way a Beast peer's
    deflater produces them (Flush::none, Flush::block, Flush::sync, strip
    00 00 FF FF).  The system zlib is byte-identical to Beast at these
    settings (tests/test_oracle.py::test_python_zlib_agrees_at_pmd_defaults)."""
    out = []
    mv = memoryview(data)
    for i in range(len(lens)):
        o, n = int(off[i]), int(lens[i])
        c = zlib.compressobj(level, zlib.DEFLATED, -wbits, mem)
        p = c.compress(mv[o:o + n]) + c.flush(zlib.Z_BLOCK) + c.flush(zlib.Z_SYNC_FLUSH)
        out.append(p[:-4])
    return out


def pack(payloads, align=16):
    lens = np.fromiter((len(p) for p in payloads), dtype=np.int64, count=len(payloads))
    slot = (lens + align - 1) // align * align
    off = np.zeros(len(payloads), dtype=np.int64)
    off[1:] = np.cumsum(slot[:-1])
    buf = np.zeros(int(slot.sum()) + 64, dtype=np.uint8)
    for i, p in enumerate(payloads):
        buf[off[i]:off[i] + lens[i]] = np.frombuffer(p, dtype=np.uint8)
    return buf, off, lens.astype(np.int32)


def cpu_baseline(comp_buf, comp_off, comp_len, raw_lens, threads, budget_s=12.0):
    """Oracle (C restatement of Beast's zlib, byte-identical to it) inflating
    the same payloads on the host cores; bounded sample."""
    from oracle import oracle as O
    n = len(comp_len)
    # size the sample so one pass is ~1-2 s on the given threads
    t0 = time.perf_counter()
    k = min(n, 2048)
    O.inflate_batch(comp_buf, comp_off[:k], comp_len[:k], raw_lens[:k], threads=1)
    per_msg = (time.perf_counter() - t0) / k
    sample = int(min(n, max(4096, budget_s / 4 / max(per_msg, 1e-9) * threads)))
    times = []
    for _ in range(3):
        t0 = time.perf_counter()
        O.inflate_batch(comp_buf, comp_off[:sample], comp_len[:sample], raw_lens[:sample], threads=threads)
        times.append(time.perf_counter() - t0)
    t = sorted(times)[1]
    gib = float(raw_lens[:sample].astype(np.int64).sum()) / (1 << 30)
    return {"value": round(gib / t, 3), "unit": "GiB/s", "cores": threads, "kind": "port",
            "sample": f"{sample} x {MSG_BYTES} B C2 payloads, oracle inflate (Beast-equivalent C), "
                      f"{threads} threads, median of 3"}


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the newest committed rocprofv3
    PMC summary (profiles/rNN_*_pmc.csv, collected by scripts/profile.sh on
    this exact workload).  FETCH_SIZE is doubled and both counters are
    read in KiB, per MI355X_MICROARCH.md's gfx950 notes.  None if absent."""
    import csv
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc.csv")))
    for f in reversed(files):
        fetch, write = [], []
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if kernel not in r["kernel"]:
                    continue
                (fetch if r["counter"] == "FETCH_SIZE" else write).append(float(r["value_kB"]))
        if fetch and write:
            return int((2 * float(np.median(fetch)) + float(np.median(write))) * 1024), os.path.relpath(f, ROOT)
    return None, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--msgs", type=int, default=N_MSGS)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    n = args.msgs
    t0 = time.perf_counter()
    lens = np.full(n, MSG_BYTES, dtype=np.uint32)
    raw, raw_off, raw_len = synth.make_batch("json", lens, seed=SEED, first=rank * n)
    payloads = pmd_compress_host(raw, raw_off, raw_len)
    comp_buf, comp_off, comp_len = pack(payloads)
    log(f"[rank {rank}] inputs ready in {time.perf_counter() - t0:.1f}s, ratio "
        f"{comp_len.sum() / raw_len.astype(np.int64).sum():.4f}")

    dev = torch.device("cuda", local)
    src = pmd.Batch(torch.from_numpy(comp_buf).to(dev), torch.from_numpy(comp_off).to(dev),
                    torch.from_numpy(comp_len).to(dev))
    cap = torch.full((n,), MSG_BYTES, dtype=torch.int32, device=dev)
    out_off = pmd.slot_offsets(cap)
    out = torch.empty(n * MSG_BYTES + 64, dtype=torch.uint8, device=dev)

    def step():
        return pmd.inflate_batch(src, cap, out=out, out_off=out_off)

    # correctness gate (outside the timed region)
    r = step()
    torch.cuda.synchronize()
    ok = int((r.status != 0).sum()) == 0 and torch.equal(
        out[: n * MSG_BYTES].view(n, MSG_BYTES), torch.from_numpy(raw.reshape(n, MSG_BYTES)).to(dev))
    if not ok:
        log(f"[rank {rank}] PARITY FAILURE")
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t_start = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record()
        step()
        ev[i][1].record()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t_start
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    if dist:
        t = torch.tensor([wall, kern_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall, kern_ms = float(t[0]), float(t[1])

    uncomp = n * MSG_BYTES
    comp = int(comp_len.astype(np.int64).sum())
    total_uncomp = uncomp * world
    value = total_uncomp / (1 << 30) / (wall / args.steps)
    alg_bytes = comp + uncomp + 16 * n
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
    traffic, traffic_src = pmc_traffic("inflate_kernel") if n == N_MSGS else (None, None)
    result = {
        "metric": "GiB/s device-resident inflate+deflate over batched WS payloads, 1/2/4/8 GPU",
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(wall / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (seeded JSON-like text, compressed host-side with zlib L6/mem4/w15 + pmd framing)",
        "config": {"workload": "C2 inflate-only: 64Ki x 4KiB payloads/GPU, compLevel=6, memLevel=4, windowBits=15",
                   "msgs_per_gpu": n, "msg_bytes": MSG_BYTES, "compressed_bytes_per_gpu": comp,
                   "parallelism": f"dp{world} (independent message shards)"},
        "parity_ok": bool(ok),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                     "traffic_source": traffic_src,
                     "kernel": "inflate_kernel", "kernel_ms": round(kern_ms, 4),
                     "alg_bytes_per_launch": alg_bytes},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        threads = min(16, os.cpu_count() or 1)
        result["cpu_baseline"] = cpu_baseline(comp_buf, comp_off, comp_len, raw_len.astype(np.uint32), threads)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
