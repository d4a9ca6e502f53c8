"""GPU: the micro-batcher behind the per-stream calls (pmd_stream.hip; SURVEY
8(f) N2).  Concurrent write() calls of different streams run as one launch,
each with exactly its single-call result.  Python threads drive the C ABI
through ctypes (the GIL is released during each call), so their calls
overlap on the device; every result is compared with the same connections
run one after another with the batcher off."""
import ctypes
import threading

import pytest

from beast_amd import synth
from tests.test_gpu_stream import SYNC, ZParams, _lib, ws_deflate_message, ws_inflate_message

pytestmark = pytest.mark.gpu


def _api():
    L = _lib()
    L.bpmd_stream_batching.argtypes = [ctypes.c_int, ctypes.c_int]
    L.bpmd_stream_batch_stats.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    return L


def _stats(L):
    c = (ctypes.c_ulonglong * 4)()
    assert L.bpmd_stream_batch_stats(c, 1) == 0
    return list(c)


def _msgs(conn, n):
    sizes = [(conn * 7919 + k * 104729) % 30000 for k in range(n)]
    sizes[0] = [0, 1, 700, 4096, 4097][conn % 5]
    raw, off, ln = synth.make_batch("json", sizes, seed=0x5EED0600 + conn)
    return [bytes(raw[int(off[i]):int(off[i]) + int(ln[i])]) for i in range(n)]


def _connection(L, cfg, msgs):
    """One connection: its deflater (level, memLevel; never reset under
    context takeover, reset after each message otherwise) and inflater."""
    level, mem, takeover = cfg
    zo, zi = ctypes.c_void_p(), ctypes.c_void_p()
    assert L.bpmd_deflate_stream_create(level, 15, mem, 0, ctypes.byref(zo)) == 0
    assert L.bpmd_inflate_stream_create(15, ctypes.byref(zi)) == 0
    pays, backs = [], []
    try:
        for m in msgs:
            p = ws_deflate_message(L, zo, m)
            if not takeover:
                assert L.bpmd_deflate_stream_reset(zo) == 0
            pays.append(p)
            backs.append(ws_inflate_message(L, zi, p))
    finally:
        L.bpmd_stream_destroy(zo)
        L.bpmd_stream_destroy(zi)
    return pays, backs


def _run(L, cfgs, msgs_of, threaded):
    res = [None] * len(cfgs)
    errs = []

    def work(i):
        try:
            res[i] = _connection(L, cfgs[i], msgs_of[i])
        except Exception as e:   # noqa: BLE001 (reported below)
            errs.append((i, repr(e)))

    if threaded:
        ts = [threading.Thread(target=work, args=(i,)) for i in range(len(cfgs))]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
    else:
        for i in range(len(cfgs)):
            work(i)
    assert not errs, errs
    return res


@pytest.mark.parametrize("max_calls,delay_us", [(256, 0), (8, 0), (64, 300)])
def test_batched_streams_equal_single_calls(max_calls, delay_us):
    """24 connections at three levels, two memLevels, with and without context
    takeover: every payload byte and every round trip of the concurrent,
    batched run equals the same connections run one by one unbatched (the
    deflate flushes of different parameters go to separate deflater calls of
    one batch), and the batched run makes fewer launches than calls."""
    L = _api()
    cfgs = [((1, 6, 9)[i % 3], (4, 8)[(i // 3) % 2], i % 4 != 0) for i in range(24)]
    msgs_of = [_msgs(i, 4) for i in range(24)]
    try:
        assert L.bpmd_stream_batching(0, 0) == 0
        ref = _run(L, cfgs, msgs_of, threaded=False)
        assert L.bpmd_stream_batching(max_calls, delay_us) == 0
        _stats(L)
        got = _run(L, cfgs, msgs_of, threaded=True)
        ic, il, dc, dl = _stats(L)
    finally:
        L.bpmd_stream_batching(256, 0)
    for i in range(24):
        assert got[i][0] == ref[i][0], i
        assert got[i][1] == msgs_of[i] == ref[i][1], i
    assert ic > 0 and dc > 0 and il < ic and dl <= dc, (ic, il, dc, dl)


def test_batched_inflate_error_stays_with_its_stream():
    """16 inflaters called at once, every fourth fed a corrupt block (BTYPE 3):
    those calls return invalid_block_type without advancing z_params (the
    reference's err()), the others inflate their payloads exactly, in the
    same batches."""
    L = _api()
    zo = ctypes.c_void_p()
    assert L.bpmd_deflate_stream_create(6, 15, 4, 0, ctypes.byref(zo)) == 0
    msg = _msgs(3, 1)[0] or b"x" * 500
    good = ws_deflate_message(L, zo, msg)
    L.bpmd_stream_destroy(zo)
    bad = b"\x07" + b"\x00" * 63   # BFINAL 1, BTYPE 3
    out = [None] * 16

    def work(i):
        zi = ctypes.c_void_p()
        assert L.bpmd_inflate_stream_create(15, ctypes.byref(zi)) == 0
        try:
            if i % 4 == 0:
                src = ctypes.create_string_buffer(bad, len(bad))
                buf = ctypes.create_string_buffer(4096)
                zs = ZParams(ctypes.addressof(src), len(bad), 0, ctypes.cast(buf, ctypes.c_void_p), 4096, 0, 2)
                r = L.bpmd_inflate_stream_write(zi, ctypes.byref(zs), SYNC)
                out[i] = (r, zs.total_in, zs.total_out)
            else:
                out[i] = ws_inflate_message(L, zi, good)
        finally:
            L.bpmd_stream_destroy(zi)

    assert L.bpmd_stream_batching(256, 200) == 0
    try:
        ts = [threading.Thread(target=work, args=(i,)) for i in range(16)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
    finally:
        L.bpmd_stream_batching(256, 0)
    for i in range(16):
        if i % 4 == 0:
            assert out[i] == (5, 0, 0), out[i]   # zlib::error::invalid_block_type
        else:
            assert out[i] == msg, i


def test_batching_settings_are_validated():
    L = _api()
    assert L.bpmd_stream_batching(-1, 0) != 0
    assert L.bpmd_stream_batching(5000, 0) != 0
    assert L.bpmd_stream_batching(16, -1) != 0
    assert L.bpmd_stream_batching(0, 0) == 0      # off
    assert L.bpmd_stream_batching(256, 0) == 0    # the default
    assert L.bpmd_stream_batch_stats(None, 0) != 0
