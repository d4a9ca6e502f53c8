"""GPU parity on the shapes of BASELINE.json configs C4 and C5,
at sizes the oracle finishes in seconds.

C4: Zipf message sizes 256 B - 64 KiB (synth.zipf_sizes, P(r) ∝ r^-1.1,
size = 256·r), JSON-like text, L6 / memLevel 4.  C5: 64 KiB low-compressibility
binary messages at deflate levels 1 and 6.

Inflate: payloads made by the oracle (byte-identical to Beast's deflate) are
inflated on both GPU kernels and in the automatic per-message split; output, lengths and statuses must equal the
oracle's inflate (= the original messages).  Deflate: GPU payloads must inflate
back byte for byte through the oracle (Beast's inflate) and the GPU inflater,
stay within deflate_upper_bound, and stay within SIZE_TOLERANCE of Beast's
compressed size at the same level.
"""
import numpy as np
import pytest

from beast_amd import synth
from oracle import oracle as O

pytestmark = pytest.mark.gpu

SIZE_TOLERANCE = 1.10   # Σ GPU payload bytes / Σ Beast payload bytes, same level


def _c4(n=8192):
    lens = synth.zipf_sizes(n, 0x5EED0004)
    return synth.make_batch("json", lens, seed=0x5EED0004)


def _c5(n=2048):
    # 2048 messages: automatic mode sends them block-parallel, as the bench's
    # C5 batch (inflate_impl: batches of 2048 - 32 Ki messages, payloads over
    # 4 KiB compressed)
    lens = np.full(n, 65536, dtype=np.uint32)
    return synth.make_batch("binary", lens, seed=0x5EED0005)


def _gpu_inflate(comp, coff, clen, caps, kernel):
    import torch
    from beast_amd import pmd
    assert pmd.lib().bpmd_set_inflate_kernel(kernel) == 0
    try:
        src = pmd.Batch.from_arrays(comp, coff.astype(np.int64), clen.astype(np.int32))
        res = pmd.inflate_batch(src, torch.tensor(caps.astype(np.int32)))
        torch.cuda.synchronize()
        return res.status.cpu().numpy(), res.out
    finally:
        pmd.lib().bpmd_set_inflate_kernel(0)


def _equal_to_messages(out, data, off, lens):
    import torch
    got_len = out.len.cpu().numpy()
    assert (got_len == lens).all(), np.nonzero(got_len != lens)[0][:8]
    # gather the GPU slots into one contiguous buffer and compare on the device
    idx = torch.cat([torch.arange(int(o), int(o) + int(n), device=out.data.device)
                     for o, n in zip(out.off.cpu().numpy(), lens)])
    want = torch.from_numpy(data[: int(lens.astype(np.uint64).sum())]).to(out.data.device)
    assert torch.equal(out.data[idx], want)


@pytest.mark.parametrize("kernel", [0, 1, 2], ids=["auto", "lane", "wave"])
@pytest.mark.parametrize("cfg", ["c4", "c5_l1", "c5_l6"])
def test_inflate_of_beast_payloads(cfg, kernel):
    data, off, lens = _c4() if cfg == "c4" else _c5()
    level = {"c4": 6, "c5_l1": 1, "c5_l6": 6}[cfg]
    comp, coff, clen, cst = O.deflate_batch(data, off, lens, level=level, wbits=15, mem_level=4,
                                            threads=16)
    assert (cst == 0).all()
    st, out = _gpu_inflate(comp, coff, clen, lens, kernel)
    assert int((st != 0).sum()) == 0, np.nonzero(st)[0][:8]
    _equal_to_messages(out, data, off, lens)
    # one byte short of each message: need_buffers, exactly as the oracle reports
    short = np.maximum(lens.astype(np.int64) - 1, 0).astype(np.uint32)
    st2, _ = _gpu_inflate(comp, coff, clen, short, kernel)
    _, _, _, est = O.inflate_batch(comp, coff, clen, short, threads=16)
    assert (st2 == est).all(), np.nonzero(st2 != est)[0][:8]


@pytest.mark.parametrize("cfg", ["c4", "c5_l1", "c5_l6"])
def test_deflate_roundtrip_and_size(cfg):
    import torch
    from beast_amd import pmd
    data, off, lens = _c4() if cfg == "c4" else _c5()
    level = {"c4": 6, "c5_l1": 1, "c5_l6": 6}[cfg]
    src = pmd.Batch.from_arrays(data, off.astype(np.int64), lens.astype(np.int32))
    d = pmd.deflate_batch(src, level=level, mem_level=4)
    torch.cuda.synchronize()
    assert int((d.status != 0).sum()) == 0
    plen = d.out.len.cpu().numpy().astype(np.uint64)
    ub = np.array([O.upper_bound(int(x)) for x in lens], dtype=np.uint64)
    assert (plen <= ub).all()
    # Beast's inflate (oracle) of the GPU payloads gives the messages back
    comp = d.out.data.cpu().numpy()
    poff = d.out.off.cpu().numpy().astype(np.uint64)
    out, ooff, olen, ost = O.inflate_batch(comp, poff, plen.astype(np.uint32), lens, threads=16)
    assert (ost == 0).all() and (olen == lens).all()
    for i in range(len(lens)):
        a, b = int(ooff[i]), int(off[i])
        assert np.array_equal(out[a:a + int(lens[i])], data[b:b + int(lens[i])]), i
    # and so does the GPU inflater
    r = pmd.inflate_batch(pmd.Batch(d.out.data, d.out.off, d.out.len),
                          torch.tensor(lens.astype(np.int32)))
    torch.cuda.synchronize()
    assert int((r.status != 0).sum()) == 0
    _equal_to_messages(r.out, data, off, lens)
    # compressed size against Beast's at the same level
    _, _, clen, _ = O.deflate_batch(data, off, lens, level=level, wbits=15, mem_level=4, threads=16)
    ours, beast = int(plen.sum()), int(clen.astype(np.uint64).sum())
    assert ours <= SIZE_TOLERANCE * beast, (ours, beast, ours / beast)


def test_c4_work_queue_batch():
    """More messages than the chip's resident lanes (65 536): the lane kernel's
    work queue hands the rest out as lanes finish.  Oracle payloads of a
    C4-shaped batch (sizes capped at 8 KiB to keep the oracle quick), inflated
    on the GPU: every message equals the oracle's inflate."""
    import torch
    from beast_amd import pmd
    n = 70000
    lens = np.minimum(synth.zipf_sizes(n, 0x5EED0044), 8192).astype(np.uint32)
    raw, off, ln = synth.make_batch("json", lens, seed=0x5EED0044)
    comp, coff, clen, st = O.deflate_batch(raw, off, ln, level=6, mem_level=4, threads=16)
    assert (st == 0).all()
    for kernel in (0, 1):
        assert pmd.lib().bpmd_set_inflate_kernel(kernel) == 0
        try:
            src = pmd.Batch.from_arrays(comp, coff.astype(np.int64), clen.astype(np.int32))
            cap = torch.from_numpy(ln.astype(np.int32)).cuda()
            r = pmd.inflate_batch(src, cap)
            torch.cuda.synchronize()
            assert int((r.status != 0).sum()) == 0
            assert torch.equal(r.out.len.cpu(), torch.from_numpy(ln.astype(np.int32)))
            outs = r.out.data.cpu().numpy()
            o_off = r.out.off.cpu().numpy()
            got = np.concatenate([outs[int(o_off[i]):int(o_off[i]) + int(ln[i])] for i in range(n)])
            assert np.array_equal(got, raw[:int(ln.astype(np.int64).sum())])
        finally:
            pmd.lib().bpmd_set_inflate_kernel(0)


def test_c4_long_payloads_split_from_lanes():
    """A work-queue batch whose longest payloads exceed 125 % of the batch's
    compressed bytes per resident lane (and 2 KiB; the value lives in
    pmd_capi.hip inflate_impl, BPMD_LONG_SHARE_PCT): those are decoded
    block-parallel (pmd_inflate_bp.hip) on a side stream from the
    longest-first order while the lane kernel takes the rest (pmd_capi.hip
    inflate_impl, bpmd_internal_lane_long_split; the wave kernel when
    BPMD_INFLATE_BP=0).  Every message -- including corrupted long and short
    ones -- must equal the oracle's inflate in status and bytes."""
    import torch
    from beast_amd import pmd
    n = 70000
    lens = synth.zipf_sizes(n, 0x5EED0045)
    raw, off, ln = synth.make_batch("json", lens, seed=0x5EED0045)
    comp, coff, clen, st = O.deflate_batch(raw, off, ln, level=6, mem_level=4, threads=16)
    assert (st == 0).all()
    thr = max(4096, 2 * int(clen.astype(np.int64).sum()) // 65536)
    longs = np.nonzero(clen > thr)[0]
    assert len(longs) > 20, len(longs)   # the split is exercised
    comp = comp.copy()
    rng = np.random.default_rng(45)
    for i in list(longs[:8]) + list(rng.choice(n, 8, replace=False)):
        j = int(coff[i]) + int(rng.integers(int(clen[i]) // 2, int(clen[i])))
        comp[j] ^= 0x10
    cap = ln.astype(np.uint32)
    exp_out, exp_off, exp_len, exp_st = O.inflate_batch(comp, coff, clen, cap, threads=16)
    src = pmd.Batch.from_arrays(comp, coff.astype(np.int64), clen.astype(np.int32))
    r = pmd.inflate_batch(src, torch.from_numpy(cap.astype(np.int32)).cuda())
    torch.cuda.synchronize()
    got_st = r.status.cpu().numpy()
    got_len = r.out.len.cpu().numpy()
    assert np.array_equal(got_st, exp_st), np.nonzero(got_st != exp_st)[0][:10]
    assert np.array_equal(got_len, exp_len.astype(got_len.dtype))
    outs = r.out.data.cpu().numpy()
    o_off = r.out.off.cpu().numpy()
    for i in range(n):
        a, b = int(o_off[i]), int(exp_off[i])
        k = int(exp_len[i])
        assert np.array_equal(outs[a:a + k], exp_out[b:b + k]), i


def _full_roundtrip(kind, lens, seed, level):
    """The bench's own mixed-leg path at the bench's own size: the whole batch
    synthesized with the bench's seed, deflated on the GPU, inflated on the GPU
    in automatic mode (lanes + block-parallel side stream), compared with the
    original bytes on the device."""
    import torch
    from beast_amd import pmd
    data, off, ln = synth.make_batch(kind, lens, seed=seed)
    dev = torch.device("cuda", 0)
    src = pmd.Batch(torch.from_numpy(data).to(dev), torch.from_numpy(off.astype(np.int64)).to(dev),
                    torch.from_numpy(ln.astype(np.int32)).to(dev))
    d = pmd.deflate_batch(src, level=level, mem_level=4)
    torch.cuda.synchronize()
    assert int((d.status != 0).sum()) == 0
    cap = torch.from_numpy(ln.astype(np.int32)).to(dev)
    # output slots laid out as the input batch, so the whole buffer compares
    r = pmd.inflate_batch(pmd.Batch(d.out.data, d.out.off, d.out.len), cap, out_off=src.off)
    torch.cuda.synchronize()
    assert int((r.status != 0).sum()) == 0, np.nonzero(r.status.cpu().numpy())[0][:8]
    assert torch.equal(r.out.len, cap)
    assert torch.equal(r.out.data[: src.data.numel()], src.data)
    return int(d.out.len.sum()) / float(ln.astype(np.float64).sum())


def test_full_c4_batch_roundtrip():
    """configs[3] at full size: 1 Mi Zipf JSON messages (8.4 GiB), L6."""
    ratio = _full_roundtrip("json", synth.zipf_sizes(1 << 20, 0x5EED0004), 0x5EED0004, 6)
    assert 0.2 < ratio < 0.4


@pytest.mark.parametrize("level", [1, 6])
def test_full_c5_batch_roundtrip(level):
    """configs[4] at full size: 16 Ki x 64 KiB binary messages (1 GiB), L1 / L6."""
    ratio = _full_roundtrip("binary", np.full(16384, 65536, dtype=np.uint32), 0x5EED0005, level)
    assert 0.9 < ratio < 1.01
