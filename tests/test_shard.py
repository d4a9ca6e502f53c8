"""CPU: multi-rank sharding of a message batch (byte-balanced contiguous
ranges, no payload exchange) and the control-plane collectives, exercised
with the gloo backend at world_size 2 -- the same code runs over RCCL on
GPUs in bench.py."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from beast_amd import shard, synth
from oracle import oracle as O


def test_ranges_cover_and_balance_bytes():
    rng = np.random.default_rng(1)
    r = np.arange(1, 257)
    p = r ** -1.1
    p /= p.sum()
    lens = 256 * rng.choice(r, size=20000, p=p)    # C4-style Zipf sizes
    for world in (1, 2, 3, 4, 8):
        rs = shard.byte_balanced_ranges(lens, world)
        assert rs[0][0] == 0 and rs[-1][1] == len(lens)
        assert all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))
        b = [int(lens[s:e].sum()) for s, e in rs]
        assert max(b) - min(b) <= 2 * int(lens.max()), b


def test_ranges_degenerate():
    assert shard.byte_balanced_ranges(np.array([], dtype=np.int64), 4) == [(0, 0)] * 4
    rs = shard.byte_balanced_ranges(np.array([5, 0, 0]), 2)
    assert rs[0][0] == 0 and rs[-1][1] == 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lens = np.array([100, 4096, 17, 9000, 0, 2500, 4096, 333], dtype=np.uint32)
    data, off, ln = synth.make_batch("json", lens, seed=9)
    rs = shard.byte_balanced_ranges(ln, world)
    d, o, l = shard.local_slice(data, off, ln, rs[rank])
    # each rank compresses only its own messages (the CPU oracle stands in
    # for the device here; this test covers the partitioning and collectives)
    local = [O.pmd_deflate(bytes(d[int(o[i]):int(o[i]) + int(l[i])]), 6, 15, 4) for i in range(len(l))]
    start, total = shard.global_output_offsets(sum(len(x) for x in local))
    t = shard.max_over_ranks(float(rank + 1))
    q.put((rank, rs[rank], start, total, t, b"".join(local)))
    dist.destroy_process_group()


def test_two_rank_gloo_shards_and_collectives():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    lens = np.array([100, 4096, 17, 9000, 0, 2500, 4096, 333], dtype=np.uint32)
    data, off, ln = synth.make_batch("json", lens, seed=9)
    expect = b"".join(O.pmd_deflate(bytes(data[int(off[i]):int(off[i]) + int(ln[i])]), 6, 15, 4)
                      for i in range(len(ln)))
    # ranges partition the batch, offsets place rank outputs back to back
    assert res[0][1][0] == 0 and res[0][1][1] == res[1][1][0] and res[1][1][1] == len(ln)
    assert res[0][2] == 0 and res[1][2] == len(res[0][5]) and res[0][3] == res[1][3] == len(expect)
    assert res[0][5] + res[1][5] == expect
    assert res[0][4] == res[1][4] == 2.0


def _bench_worker(rank, world, port, q):
    """bench.py's own partition code (shard_config + per-rank synthesis by
    global message index) on a C4-shaped batch under gloo."""
    import sys
    import torch.distributed as dist
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lens_all = synth.zipf_sizes(600, bench.SEED_C4)
    s0, e0, per_rank = bench.shard_config(lens_all, rank, world)
    data, off, ln = synth.make_batch("json", lens_all[s0:e0], seed=bench.SEED_C4, first=s0)
    local = [O.pmd_deflate(bytes(data[int(off[i]):int(off[i]) + int(ln[i])]), 6, 15, 4) for i in range(len(ln))]
    start, total = shard.global_output_offsets(sum(len(x) for x in local))
    q.put((rank, (s0, e0), per_rank, start, total, b"".join(local)))
    dist.destroy_process_group()


def test_two_rank_gloo_runs_bench_partition():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=180) for _ in range(world)])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    lens_all = synth.zipf_sizes(600, bench.SEED_C4)
    data, off, ln = synth.make_batch("json", lens_all, seed=bench.SEED_C4)
    expect = b"".join(O.pmd_deflate(bytes(data[int(off[i]):int(off[i]) + int(ln[i])]), 6, 15, 4)
                      for i in range(len(ln)))
    (r0, g0, b0, st0, tot0, out0), (r1, g1, b1, st1, tot1, out1) = res
    assert g0[0] == 0 and g0[1] == g1[0] and g1[1] == len(lens_all)
    assert b0 == b1 and sum(b0) == int(lens_all.astype(np.int64).sum())
    assert max(b0) - min(b0) <= 2 * int(lens_all.max())
    assert st0 == 0 and st1 == len(out0) and tot0 == tot1 == len(expect)
    assert out0 + out1 == expect   # per-rank synthesis by global index == the whole batch


def test_c_abi_shard_ranges_match_python():
    """bpmd_shard_ranges (the C++ server's split, pmd_multi.hip) cuts exactly
    where beast_amd/shard.py does."""
    from beast_amd import pmd, synth
    rng = np.random.default_rng(5)
    cases = [synth.zipf_sizes(20000, 0x5EED0004), np.full(1000, 65536, dtype=np.uint32),
             np.zeros(17, dtype=np.uint32), np.array([], dtype=np.uint32), np.array([7], dtype=np.uint32),
             rng.integers(0, 70000, 5000).astype(np.uint32)]
    for lens in cases:
        for world in (1, 2, 3, 4, 7, 8):
            assert pmd.shard_ranges(lens, world) == shard.byte_balanced_ranges(lens, world), (len(lens), world)
