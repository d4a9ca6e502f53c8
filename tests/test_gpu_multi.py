"""GPU: the one-process multi-device entry points (bpmd_*_batch_multi,
pmd_multi.hip).  The box has one GPU, so the shards are
"virtual devices": every shard on device 0 with a stream of its own, which
exercises the launch, the per-shard scratch and the output-size gather the
same way.  Results must equal one bpmd_*_batch over the whole batch, and the
gathered totals must place every shard in one global output."""
import numpy as np
import pytest
import torch

from beast_amd import pmd, synth
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _sub(b: pmd.Batch, a, e):
    return pmd.Batch(b.data, b.off[a:e], b.len[a:e])


@pytest.mark.parametrize("parts", [1, 2, 3, 8])
def test_multi_equals_single_batch(parts):
    lens = synth.zipf_sizes(3000, 0x5EED00A1)
    data, off, ln = synth.make_batch("json", lens, seed=0x5EED00A1)
    src = pmd.Batch.from_arrays(data, off, ln)
    ranges = pmd.shard_ranges(lens, parts)
    streams = [torch.cuda.Stream() for _ in ranges]
    dres, dtot = pmd.deflate_batch_multi([_sub(src, a, e) for a, e in ranges], level=6, streams=streams)
    torch.cuda.synchronize()
    one = pmd.deflate_batch(src, level=6)
    torch.cuda.synchronize()
    pays_one = one.out.to_host()
    pays = []
    for (a, e), r, t in zip(ranges, dres, dtot):
        assert int((r.status != 0).sum()) == 0
        got = r.out.to_host()
        assert int(t) == sum(len(p) for p in got)
        pays += got
    assert pays == pays_one   # the deflater is deterministic per message
    # inflate the shards' payloads back, again split
    comp = [pmd.Batch.from_host(pays[a:e]) for a, e in ranges]
    ires, itot = pmd.inflate_batch_multi(comp, [src.len[a:e] for a, e in ranges], streams=streams)
    torch.cuda.synchronize()
    back = []
    for r, t in zip(ires, itot):
        assert int((r.status != 0).sum()) == 0
        got = r.out.to_host()
        assert int(t) == sum(len(x) for x in got)
        back += got
    msgs = [bytes(data[int(off[i]):int(off[i]) + int(ln[i])]) for i in range(len(ln))]
    assert back == msgs
    # global layout from the gathered totals
    starts = np.concatenate([[0], np.cumsum(itot)])
    assert int(starts[-1]) == int(ln.astype(np.int64).sum())


def test_multi_rejects_bad_device():
    import ctypes
    L = pmd.lib()
    arr = (pmd._Shard * 1)()
    arr[0].device = 99
    cfg = pmd._Cfg(6, 15, 4, 0, 0)
    assert L.bpmd_inflate_batch_multi(ctypes.byref(cfg), arr, 1, None) == -1
    assert L.bpmd_deflate_batch_multi(ctypes.byref(cfg), arr, 1, None) == -1


def test_multi_deflate_pinned_memory_flat():
    """every shard runs on a host thread of its own, and the chunk
    count's pinned read-back word used to be thread_local, i.e. one pinned
    allocation leaked per shard thread and call.  It is now one word per
    (device, stream): repeated multi-shard deflates of long messages keep the
    count of pinned blocks flat."""
    import ctypes
    L = pmd.lib()
    L.bpmd_internal_pinned_count.restype = ctypes.c_size_t
    lens = np.full(64, 20000, dtype=np.uint32)   # > 4 KiB: the chunk-count read-back runs
    data, off, ln = synth.make_batch("json", lens, seed=0x5EED00A2)
    src = pmd.Batch.from_arrays(data, off, ln)
    ranges = pmd.shard_ranges(lens, 4)
    streams = [torch.cuda.Stream() for _ in ranges]
    pmd.deflate_batch_multi([_sub(src, a, e) for a, e in ranges], level=6, streams=streams)
    torch.cuda.synchronize()
    base = L.bpmd_internal_pinned_count()
    for _ in range(5):
        dres, _tot = pmd.deflate_batch_multi([_sub(src, a, e) for a, e in ranges], level=6, streams=streams)
        torch.cuda.synchronize()
        assert all(int((r.status != 0).sum()) == 0 for r in dres)
    assert L.bpmd_internal_pinned_count() == base
