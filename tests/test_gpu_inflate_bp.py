"""Block-parallel inflate of long payloads (pmd_inflate_bp.hip): payloads cut
at their dynamic-block headers, segments decoded one per lane as symbols,
resolved in stream order.  Bytes, lengths and statuses must equal the
oracle's serial inflate (oracle/bzo_inflate.c, inflate_stream.ipp) exactly,
including the first invalid distance, the output capacity and decode errors
wherever they fall relative to the segment boundaries."""
import random
import zlib

import numpy as np
import pytest

from beast_amd import synth
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _pmd():
    import torch  # noqa: F401
    from beast_amd import pmd
    return pmd


@pytest.fixture(params=["bp", "auto"])
def mode(request):
    pmd = _pmd()
    assert pmd.lib().bpmd_set_inflate_kernel({"bp": 3, "auto": 0}[request.param]) == 0
    yield request.param
    pmd.lib().bpmd_set_inflate_kernel(0)


def _run(payloads, caps, raw=False):
    import torch
    pmd = _pmd()
    src = pmd.Batch.from_host(payloads)
    c = caps if isinstance(caps, int) else torch.tensor(caps, dtype=torch.int32)
    res = pmd.inflate_batch(src, c, raw=raw)
    torch.cuda.synchronize()
    return res.status.cpu().numpy(), res.out.to_host()


def _check(payloads, caps, raw=False):
    st, outs = _run(payloads, caps, raw=raw)
    for i, p in enumerate(payloads):
        cap = caps if isinstance(caps, int) else caps[i]
        est, eout = O.pmd_inflate(p, cap=cap, raw=raw)
        assert int(st[i]) == est, (i, O.ERRORS[int(st[i])], O.ERRORS[est], len(p), cap)
        assert outs[i] == eout, (i, len(outs[i]), len(eout), cap)


def _data(kind, size, seed):
    d, _, _ = synth.make_batch(kind, [size], seed=seed)
    return bytes(d[:size])


@pytest.mark.parametrize("level", [1, 6, 9])
@pytest.mark.parametrize("mem", [1, 4, 9])
def test_long_payloads_beast_blocks(mode, level, mem):
    """Beast's own payloads (the oracle's deflate_stream): blocks every
    lit_bufsize - 1 symbols, stored / fixed / dynamic mixed."""
    payloads, caps = [], []
    for kind in ("json", "binary", "corpus1", "random"):
        for size in (9000, 40000, 65536, 150000):
            data = _data(kind, size, level * 1000 + mem * 10 + size)
            payloads.append(O.pmd_deflate(data, level, 15, mem))
            caps.append(size)
    _check(payloads, caps)
    _check(payloads, caps, raw=True)


def test_long_payloads_gpu_deflater(mode):
    """This library's chunk-parallel deflater (one block per 4 KiB chunk)."""
    import torch
    pmd = _pmd()
    sizes = [65536] * 24 + [30000] * 8 + [200000] * 2
    kinds = ["binary", "json", "corpus1"]
    payloads = []
    for i, size in enumerate(sizes):
        data = _data(kinds[i % 3], size, 77 + i)
        src = pmd.Batch.from_host([data])
        res = pmd.deflate_batch(src, level=1 + (i % 2) * 5)
        torch.cuda.synchronize()
        assert int(res.status[0]) == 0
        payloads.append(res.out.to_host()[0])
    _check(payloads, sizes)


def test_capacity_cuts_across_segments(mode):
    """The capacity rule at every kind of position: inside segments, at their
    boundaries, at the exact size and past it."""
    data = _data("json", 120000, 11)
    p = O.pmd_deflate(data, 6, 15, 1)   # 64-symbol blocks: many candidates
    rng = random.Random(3)
    caps = sorted({1, 4095, 4096, 4097, 65535, 65536, 119999, 120000, 120001} |
                  {rng.randrange(1, 120000) for _ in range(40)})
    _check([p] * len(caps), caps)
    _check([p] * len(caps), caps, raw=True)


def test_preset_dictionary_distances(mode):
    """Distances past the start of the message (a peer that used a preset
    dictionary): invalid_distance at the first such token, whichever segment
    holds it, and the capacity rule when the output is full first."""
    rng = random.Random(5)
    zd = rng.randbytes(32768)
    payloads, caps = [], []
    for lead in (0, 3000, 9000, 20000, 28000):
        data = bytearray(rng.randbytes(lead))
        while len(data) < 40000:
            k = rng.randrange(0, 32768 - 64)
            data += zd[k:k + rng.randrange(16, 64)] + rng.randbytes(rng.randrange(200, 2000))
        for level, mem in ((6, 4), (1, 1), (9, 8)):
            c = zlib.compressobj(level, zlib.DEFLATED, -15, mem, zdict=zd)
            comp = c.compress(bytes(data)) + c.flush(zlib.Z_SYNC_FLUSH)
            assert comp.endswith(b"\x00\x00\xff\xff")
            payloads.append(comp[:-4])
            caps.append(len(data))
            payloads.append(comp[:-4])
            caps.append(max(1, lead - 7))
    _check(payloads, caps)


def test_corrupted_long_payloads(mode):
    rng = random.Random(9)
    base = [O.pmd_deflate(_data(k, 50000, i), rng.choice([1, 6]), 15, 4)
            for i, k in enumerate(("json", "binary", "corpus1"))]
    payloads = []
    for _ in range(150):
        q = bytearray(rng.choice(base))
        if rng.randrange(2):
            for _ in range(rng.randrange(1, 4)):
                q[rng.randrange(len(q))] ^= 1 << rng.randrange(8)
        else:
            q = q[:rng.randrange(64, len(q))]
        payloads.append(bytes(q))
    _check(payloads, 60000)
    _check(payloads, 60000, raw=True)


def test_highly_compressible_falls_back(mode):
    """Output far above the per-segment estimate (zeros, runs): the segment
    slot fills and the payload is decoded again by the wave kernel."""
    payloads, caps = [], []
    for kind, size in (("zeros", 500000), ("corpus1", 300000), ("zeros", 70000)):
        data = _data(kind, size, size)
        payloads.append(O.pmd_deflate(data, 6, 15, 8))
        caps.append(size)
    _check(payloads, caps)


def test_auto_mixed_batch_takes_bp():
    """Automatic mode, 2 100 messages: the long ones go block-parallel, the
    rest to the lane kernel, all in one call."""
    pmd = _pmd()
    assert pmd.lib().bpmd_set_inflate_kernel(0) == 0
    rng = random.Random(13)
    payloads, caps = [], []
    for i in range(2100):
        if i % 7 == 0:
            size = rng.choice([20000, 65536])
            kind = rng.choice(["binary", "json"])
        else:
            size = rng.randrange(100, 4000)
            kind = "json"
        data = _data(kind, size, 1000 + i)
        payloads.append(O.pmd_deflate(data, rng.choice([1, 6]), 15, 4))
        caps.append(size)
    _check(payloads, caps)


@pytest.mark.parametrize("raw", [False, True])
def test_final_stored_block_keeps_end_of_stream(mode, raw):
    """zlib's Z_FINISH on incompressible data ends with a final (BFINAL=1)
    stored block, which the scan can also find as a stored candidate; the
    segment that reaches it must keep its BFINAL bit, so the message ends
    with end_of_stream (raw) or fails the pmd tail, as the serial decoder
    does (RFC 7692 allows a sender to finish a message that way)."""
    rng = random.Random(0xF1)
    payloads, caps = [], []
    for _ in range(12):
        size = rng.randrange(9000, 150000)
        data = rng.randbytes(size)
        c = zlib.compressobj(rng.choice([1, 6]), zlib.DEFLATED, -15)
        payloads.append(c.compress(data) + c.flush(zlib.Z_FINISH))
        caps.append(size + 16)
    _check(payloads, caps, raw=raw)


@pytest.mark.parametrize("level", [1, 6])
def test_c5_payload_with_false_stored_candidate(level):
    """The bench's C5 message 11145 (seed 0x5EED0005), as this library
    deflates it, holds a random LEN / NLEN pair at byte 53 863 whose LEN
    (6 857) lands exactly on a real block start, so the stored-block check
    passes it.  With slots sized to the next candidate only, the real segment
    before it outgrew its slot and the payload fell back to the wave kernel
    (f59740b: slots reach to the candidate after next).  Forced block-parallel,
    the payload must decode exactly and without a fallback."""
    import ctypes
    import torch
    pmd = _pmd()
    raw, off, ln = synth.make_batch("binary", np.full(1, 65536, np.uint32), seed=0x5EED0005, first=11145)
    src = pmd.Batch.from_arrays(raw, off.astype(np.int64), ln.astype(np.int32))
    d = pmd.deflate_batch(src, level=level, mem_level=4)
    torch.cuda.synchronize()
    assert int(d.status[0]) == 0
    c = (ctypes.c_ulonglong * 12)()
    pmd.lib().bpmd_diag_bp_counters(c, 1)
    assert pmd.lib().bpmd_set_inflate_kernel(3) == 0
    try:
        r = pmd.inflate_batch(pmd.Batch(d.out.data, d.out.off, d.out.len), torch.tensor([65536], dtype=torch.int32))
        torch.cuda.synchronize()
    finally:
        pmd.lib().bpmd_set_inflate_kernel(0)
    pmd.lib().bpmd_diag_bp_counters(c, 1)
    assert int(r.status[0]) == 0 and int(r.out.len[0]) == 65536
    assert torch.equal(r.out.data[:65536], src.data[:65536])
    assert c[0] == 1 and c[1] >= 8 and c[2] == 0, list(c)[:3]   # one payload, its segments, no fallback


def test_foreign_payload_with_one_early_flush():
    """A foreign encoder's payload whose only sync flush is near its start
    (CPython's zlib, raw deflate, memLevel 4: Z_SYNC_FLUSH after the first
    KiB, then ~1 KiB dynamic blocks without markers).  Pass 1 marks it (an
    empty stored block), but pass 2 still searches every region farther than
    MARK_SPAN from the last marker or stored block (pmd_inflate_bp.hip), so
    the payload is cut at its dynamic headers instead of decoding as one
    serial segment: exact output, many segments, no fallback."""
    import ctypes
    import zlib
    pmd = _pmd()
    msg = _data("json", 256 * 1024, 7)
    co = zlib.compressobj(6, zlib.DEFLATED, -15, 4)
    p = co.compress(msg[:1024]) + co.flush(zlib.Z_SYNC_FLUSH) + co.compress(msg[1024:]) + co.flush(zlib.Z_SYNC_FLUSH)
    assert p.endswith(b"\x00\x00\xff\xff")
    payloads = [p[:-4]] * 4
    c = (ctypes.c_ulonglong * 12)()
    pmd.lib().bpmd_diag_bp_counters(c, 1)
    assert pmd.lib().bpmd_set_inflate_kernel(3) == 0
    try:
        _check(payloads, len(msg) + 16)
    finally:
        pmd.lib().bpmd_set_inflate_kernel(0)
    pmd.lib().bpmd_diag_bp_counters(c, 1)
    assert c[0] == 4 and c[1] >= 4 * 16 and c[2] == 0, list(c)[:4]



def test_stored_block_ending_in_the_last_region():
    """the last region of a payload also takes the remainder past
    regions * R (region_of), so a stored block whose data ends inside it, past
    (k + 1) * R, may be followed by a block start in that region.  Pass 2 used
    to take (k + 1) * R as the region's end (skipping it as "inside the stored
    data") and searched only up to there; it now uses the real end, and the
    dynamic block after the stored data becomes a segment of its own.  Payload:
    17 hand-made stored blocks (random bytes) ending in the last region, then a
    small dynamic block (CPython zlib, BFINAL 0, sync-flushed; the pmd tail is
    stripped).  Exact output, 18 segments per payload (the start, 16 stored
    blocks found by pass 1, the dynamic block)."""
    import ctypes
    import zlib
    pmd = _pmd()
    R = 1024   # R_MIN: four ~68 KB payloads are far below a lane's share
    js = _data("json", 700, 11)
    co = zlib.compressobj(6, zlib.DEFLATED, -15, 4)
    dyn = co.compress(js) + co.flush(zlib.Z_SYNC_FLUSH)
    assert dyn.endswith(b"\x00\x00\xff\xff") and (dyn[0] >> 1) & 3 == 2 and not dyn[0] & 1
    dyn = dyn[:-4]
    D = len(dyn)
    assert D < R // 2 - 16
    K = 66   # regions: round((S + D) / R) == K, stored data ending past K * R
    S = K * R + 8
    rnd = random.Random(5)
    sizes = [4000] * 16
    sizes.append(S - sum(sizes) - 5 * 17)
    stored, plain = b"", b""
    for n in sizes:
        blk = bytes(rnd.getrandbits(8) for _ in range(n))
        stored += b"\x00" + n.to_bytes(2, "little") + (n ^ 0xFFFF).to_bytes(2, "little") + blk
        plain += blk
    assert len(stored) == S and round((S + D) / R) == K
    p = stored + dyn
    payloads = [p] * 4
    c = (ctypes.c_ulonglong * 12)()
    pmd.lib().bpmd_diag_bp_counters(c, 1)
    assert pmd.lib().bpmd_set_inflate_kernel(3) == 0
    try:
        _check(payloads, len(plain) + len(js) + 16)
    finally:
        pmd.lib().bpmd_set_inflate_kernel(0)
    pmd.lib().bpmd_diag_bp_counters(c, 1)
    assert c[0] == 4 and c[1] == 4 * 18 and c[2] == 0, list(c)[:4]


@pytest.mark.parametrize("raw", [False, True])
def test_stored_segments_copied_from_the_payload(raw):
    """Round 6: a stored block whose end is the next candidate's start is not
    decoded by a lane; the resolve copies its bytes from the payload
    (SEG_DIRECT, pmd_inflate_lane3.hip begin / bp_resolve_kernel).  Runs of
    hand-made stored blocks (random bytes, 3-5 KB) before a dynamic block,
    at output capacities that cut inside a stored block, exactly at a block's
    end, one byte before it, and at the full size: bytes and statuses equal
    the oracle's serial inflate; with room for the whole output no payload
    falls back (a small capacity sizes the symbol slots small, bp_stats_kernel,
    and the dynamic block's segment may then go to the wave kernel)."""
    import ctypes
    import zlib
    pmd = _pmd()
    rnd = random.Random(11)
    js = _data("json", 900, 12)
    co = zlib.compressobj(6, zlib.DEFLATED, -15, 4)
    dyn = co.compress(js) + co.flush(zlib.Z_SYNC_FLUSH)
    dyn = dyn[:-4]
    stored, plain, ends = b"", b"", []
    for _ in range(24):
        n = rnd.randrange(3000, 5000)
        blk = bytes(rnd.getrandbits(8) for _ in range(n))
        stored += b"\x00" + n.to_bytes(2, "little") + (n ^ 0xFFFF).to_bytes(2, "little") + blk
        plain += blk
        ends.append(len(plain))
    p = stored + dyn
    full = len(plain) + len(js)
    cuts = [ends[5], ends[5] - 1, ends[5] + 1, ends[11] + 1234, 77, ends[-1]]
    c = (ctypes.c_ulonglong * 12)()
    pmd.lib().bpmd_diag_bp_counters(c, 1)
    assert pmd.lib().bpmd_set_inflate_kernel(3) == 0
    try:
        _check([p] * 4, [full + 16, full, full + 16, full], raw=raw)
        pmd.lib().bpmd_diag_bp_counters(c, 1)
        assert c[0] == 4 and c[2] == 0, list(c)[:4]
        _check([p] * len(cuts), cuts, raw=raw)
    finally:
        pmd.lib().bpmd_set_inflate_kernel(0)


# ---------------------------------------------------- workspace sizing (r05)
# A stream's block-parallel decode workspace is sized on its first call (one
# read-back) or by bpmd_inflate_reserve; payloads over the capacity are
# spilled to the wave kernel (counter [3]) and the capacity grows for the
# next call; a workspace that cannot be allocated falls back to a smaller
# one.  Each test releases its stream's pools so the next one starts cold.

def _c5_like(n, seed, level=1):
    import torch
    pmd = _pmd()
    raw, off, ln = synth.make_batch("binary", np.full(n, 65536, np.uint32), seed=seed)
    src = pmd.Batch.from_arrays(raw, off.astype(np.int64), ln.astype(np.int32))
    d = pmd.deflate_batch(src, level=level)
    torch.cuda.synchronize()
    assert int((d.status != 0).sum()) == 0
    return src, pmd.Batch(d.out.data, d.out.off, d.out.len), torch.from_numpy(ln.astype(np.int32)).cuda()


def _on_fresh_stream(fn):
    import ctypes
    import torch
    pmd = _pmd()
    assert pmd.lib().bpmd_set_inflate_kernel(0) == 0
    st = torch.cuda.Stream()
    try:
        with torch.cuda.stream(st):
            return fn(st)
    finally:
        st.synchronize()
        pmd.lib().bpmd_internal_scratch_release(ctypes.c_void_p(st.cuda_stream))


def _call(st, comp, cap, src):
    import torch
    pmd = _pmd()
    out = torch.empty_like(src.data)
    pmd.bp_counters(reset=True)
    r = pmd.inflate_batch(comp, cap, out=out, out_off=src.off, stream=st)
    st.synchronize()
    c = pmd.bp_counters(reset=True)
    ok = int((r.status != 0).sum()) == 0 and torch.equal(r.out.len, src.len) and torch.equal(out, src.data)
    return ok, c


def test_first_call_on_a_fresh_stream_takes_no_fallback():
    """The stream's first C5-shaped call already decodes every long payload
    block-parallel: no capacity spill, no resolve fallback."""
    src, comp, cap = _c5_like(2048, 0x5EED0061)

    def body(st):
        ok, c = _call(st, comp, cap, src)
        assert ok
        assert c[0] == 2048 and c[2] == 0 and c[3] == 0, c[:4]
        ok, c = _call(st, comp, cap, src)
        assert ok and c[0] == 2048 and c[2] == 0 and c[3] == 0, c[:4]
    _on_fresh_stream(body)


def test_reserved_too_small_spills_then_grows():
    """A reserve far below the batch: the fitting prefix decodes
    block-parallel, the rest through the wave kernel, all exact; the next
    call has grown to the batch and spills nothing."""
    src, comp, cap = _c5_like(2048, 0x5EED0062)   # >= 2048: the lane/bp path, not the wave kernel
    pmd = _pmd()

    def body(st):
        pmd.inflate_reserve(65536, 65536, 1, stream=st)
        ok, c = _call(st, comp, cap, src)
        assert ok and c[3] > 0 and c[0] + c[3] == 2048, c[:4]
        ok, c = _call(st, comp, cap, src)
        assert ok and c[0] == 2048 and c[2] == 0 and c[3] == 0, c[:4]
    _on_fresh_stream(body)


def test_failed_workspace_allocation_falls_back():
    """The first three decode-workspace allocations fail: the call keeps a
    smaller workspace (exact output, spills to the wave kernel).  That
    capacity is then a ceiling for the next 8 calls (under memory
    pressure every call would otherwise sync, free and fail again): the two
    calls after it keep the same capacity -- no regrowth, so no allocation
    and no stream sync -- and spill exactly; once the hold has run out the
    capacity grows again and every payload decodes block-parallel."""
    import ctypes
    src, comp, cap = _c5_like(2048, 0x5EED0063)
    pmd = _pmd()

    def caps(st):
        v = (ctypes.c_ulonglong * 5)()
        assert pmd.lib().bpmd_diag_bp_caps(ctypes.c_void_p(st.cuda_stream), v) == 0
        return list(v)

    def body(st):
        pmd.lib().bpmd_diag_bp_fail_alloc(3)
        try:
            ok, c = _call(st, comp, cap, src)
        finally:
            pmd.lib().bpmd_diag_bp_fail_alloc(0)
        assert ok and c[3] > 0, c[:4]
        c0 = caps(st)
        assert c0[0] == c0[2] and c0[1] == c0[3] and c0[4] == 8, c0
        for k in range(2):
            ok, c = _call(st, comp, cap, src)
            assert ok and c[3] > 0, c[:4]
            ck = caps(st)
            assert ck[:4] == c0[:4] and ck[4] == 7 - k, (ck, c0)
        for _ in range(7):
            ok, c = _call(st, comp, cap, src)
            assert ok
        assert caps(st)[4] == 0
        ok, c = _call(st, comp, cap, src)
        assert ok and c[0] == 2048 and c[3] == 0, c[:4]
    _on_fresh_stream(body)


def test_deep_reference_chains(mode):
    """A 1 KiB pattern repeated with 5-10 % of its bytes changed each time:
    most bytes copy the byte one period back, which was itself copied, so a
    reference crosses many segments before it reaches a literal.  Chains
    deeper than the resolve's hop limit are finished segment by segment
    (pmd_inflate_bp.hip bp_resolve2_kernel pass 3); every byte must equal the
    oracle's."""
    rng = random.Random(0xDEE9)
    payloads, caps = [], []
    for size, rate in ((120000, 0.05), (65536, 0.10), (200000, 0.02)):
        per = bytearray(rng.randbytes(1024))
        data = bytearray()
        while len(data) < size:
            for _ in range(int(1024 * rate)):
                per[rng.randrange(1024)] = rng.randrange(256)
            data += per
        data = bytes(data[:size])
        for level, mem in ((6, 4), (1, 8)):
            payloads.append(O.pmd_deflate(data, level, 15, mem))
            caps.append(size)
    _check(payloads, caps)
    _check(payloads, caps, raw=True)


@pytest.mark.parametrize("level", [1, 6])
def test_fixed_block_skim(mode, level):
    """The fixed-block skim (off by default; bpmd_diag_set_bp_skim): Beast's
    near-random payloads are runs of stored and fixed blocks, and the walks
    from pass 1's stored candidates record every block start they pass.
    Results must stay the serial decoder's, including capacity cuts and
    corrupted payloads (a walk only ever adds candidates)."""
    pmd = _pmd()
    rng = random.Random(0x5C1 + level)
    payloads, caps = [], []
    for i in range(40):
        size = rng.choice([20000, 65536, 100000])
        data = _data(rng.choice(["binary", "random", "json"]), size, 500 + i)
        payloads.append(O.pmd_deflate(data, level, 15, rng.choice([1, 4, 8])))
        caps.append(size if i % 5 else rng.randrange(1, size))
    for i in range(0, 40, 7):   # a few corrupted ones
        q = bytearray(payloads[i])
        q[rng.randrange(len(q))] ^= 1 << rng.randrange(8)
        payloads[i] = bytes(q)
    pmd.lib().bpmd_diag_set_bp_skim(1)
    try:
        _check(payloads, caps)
        _check(payloads, caps, raw=True)
    finally:
        pmd.lib().bpmd_diag_set_bp_skim(0)
