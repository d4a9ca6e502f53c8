"""Which batch calls return before the device has run the work queued ahead
of them (include/beast_pmd.h, "Batch calls are asynchronous on stream").

A long device copy is queued on the caller's stream first; a call that does
not wait on the device returns while that copy is still running (the stream
is not idle and the call took a small part of the copy's time).  The
block-parallel inflate path reads its workspace totals back only on a
stream's first call, and not at all after bpmd_inflate_reserve: so
bpmd_inflate_batch returns at once on a batch of long payloads once the
stream is warm or reserved (a cold, unreserved stream's first call waits,
as the header states); bpmd_deflate_batch with a message over 4 KiB reads
back its chunk count and returns only after the copy."""
import numpy as np
import pytest

from beast_amd import synth

pytestmark = pytest.mark.gpu


def _setup():
    import torch
    from beast_amd import pmd
    dev = torch.device("cuda", 0)
    free, _ = torch.cuda.mem_get_info(dev)
    size = min(3 << 30, free // 4)
    if size < (256 << 20):
        pytest.skip(f"{free >> 20} MiB free: not enough for the queued copy")
    big = torch.empty(size, dtype=torch.uint8, device=dev)
    big2 = torch.empty_like(big)
    return torch, pmd, dev, big, big2


def _call_behind_copies(torch, fn, big, big2, copies=8):
    """Queue `copies` device copies, then fn(); True when the copies had
    finished by the time fn returned (checked on an event, not a clock)."""
    torch.cuda.synchronize()
    for _ in range(copies):
        big2.copy_(big)
    ev = torch.cuda.Event()
    ev.record()
    fn()
    done = ev.query()
    torch.cuda.synchronize()
    return done


def test_inflate_block_parallel_batch_does_not_wait():
    torch, pmd, dev, big, big2 = _setup()
    # C5-shaped long payloads in a 2 048-message batch: the block-parallel path
    raw, off, ln = synth.make_batch("binary", np.full(2048, 65536, np.uint32), seed=0x5EED0055)
    src = pmd.Batch.from_arrays(raw, off.astype(np.int64), ln.astype(np.int32))
    d = pmd.deflate_batch(src, level=1)
    comp = pmd.Batch(d.out.data, d.out.off, d.out.len)
    cap = torch.from_numpy(ln.astype(np.int32)).to(dev)
    out = torch.empty_like(src.data)

    def call():
        return pmd.inflate_batch(comp, cap, out=out, out_off=src.off)

    for _ in range(3):   # the stream's pools reach this batch's size
        r = call()
    torch.cuda.synchronize()
    assert int((r.status != 0).sum()) == 0 and torch.equal(out, src.data)
    assert not _call_behind_copies(torch, call, big, big2), "the call waited for the queued copies"


def test_first_inflate_after_reserve_does_not_wait():
    """on a fresh stream sized by bpmd_inflate_reserve the very
    first block-parallel inflate call enqueues only (no totals read-back)."""
    import ctypes
    torch, pmd, dev, big, big2 = _setup()
    raw, off, ln = synth.make_batch("binary", np.full(2048, 65536, np.uint32), seed=0x5EED0057)
    src = pmd.Batch.from_arrays(raw, off.astype(np.int64), ln.astype(np.int32))
    d = pmd.deflate_batch(src, level=1)
    comp = pmd.Batch(d.out.data, d.out.off, d.out.len)
    cap = torch.from_numpy(ln.astype(np.int32)).to(dev)
    out = torch.empty_like(src.data)
    torch.cuda.synchronize()
    st = torch.cuda.Stream()
    try:
        with torch.cuda.stream(st):
            pmd.inflate_reserve(int(d.out.len.sum()), int(ln.sum()), 2048, stream=st)

            def call():
                return pmd.inflate_batch(comp, cap, out=out, out_off=src.off, stream=st)

            torch.cuda.synchronize()
            for _ in range(8):
                big2.copy_(big)
            ev = torch.cuda.Event()
            ev.record(st)
            r = call()
            waited = ev.query()
            st.synchronize()
            assert int((r.status != 0).sum()) == 0 and torch.equal(out, src.data)
            assert not waited, "the first call after the reserve waited for the queued copies"
    finally:
        st.synchronize()
        pmd.lib().bpmd_internal_scratch_release(ctypes.c_void_p(st.cuda_stream))


def test_deflate_of_long_messages_waits_for_its_chunk_count():
    torch, pmd, dev, big, big2 = _setup()
    raw, off, ln = synth.make_batch("json", np.full(512, 65536, np.uint32), seed=0x5EED0056)
    src = pmd.Batch.from_arrays(raw, off.astype(np.int64), ln.astype(np.int32))
    ub = np.array([pmd.upper_bound(int(x)) for x in ln], dtype=np.int32)
    cap = torch.from_numpy(ub).to(dev)
    coff = pmd.slot_offsets(cap)
    cbuf = torch.empty(int(coff[-1]) + int(ub[-1]) + 64, dtype=torch.uint8, device=dev)

    def call():   # every buffer given: the wrapper itself never waits
        return pmd.deflate_batch(src, level=6, out_cap=cap, out=cbuf, out_off=coff)

    for _ in range(2):
        d = call()
    torch.cuda.synchronize()
    assert int((d.status != 0).sum()) == 0
    # documented: it waits for the work queued before it
    assert _call_behind_copies(torch, call, big, big2), "the call returned before the queued copies ran"
