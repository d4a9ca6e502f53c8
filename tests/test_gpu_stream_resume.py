"""GPU: the per-stream inflater (bpmd_inflate_stream_*, behind the drop-in
zlib::inflate_stream) is a resumable decoder.  Checked call by call against
the oracle's streaming restatement of Beast's inflate_stream
(oracle/bzo_inflate.c = inflate_stream.ipp:74-535 + window.hpp:51-144):

* the same status and the same output bytes from every write(), whatever
  the input cuts, output room and flush (sync / block / trees);
* one inflater for a whole connection (Beast never resets zi between
  messages, impl_base.hpp:192-202, 277-309), with context takeover, so
  later messages copy from earlier ones through the window;
* the per-call window rule (a distance past the window the reference holds
  at the call's start is invalid_distance, inflate_stream.ipp:1046-1061);
* BAD and DONE modes (inflate_stream.ipp:516-529);
* configs[0]'s shape driven exactly as read.hpp:1284-1356 drives it, with the
  stream's memory bounded however long the connection runs.

The reference leaves input unconsumed when avail_out runs out first; the GPU
stream keeps those bytes and reports them consumed, so each side is offered
input from its own consumed position up to the same cut, which gives both the
same bytes to decode by the end of every call."""
import ctypes
import json
import os
import random

import numpy as np
import pytest

from beast_amd import synth
from oracle import oracle as O

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NONE, BLOCK, PARTIAL, SYNC, FULL, FINISH, TREES = range(7)
FLUSH_NAMES = {NONE: "none", BLOCK: "block", SYNC: "sync", FINISH: "finish", TREES: "trees"}
EB = b"\x00\x00\xff\xff"


class ZParams(ctypes.Structure):
    _fields_ = [("next_in", ctypes.c_void_p), ("avail_in", ctypes.c_size_t), ("total_in", ctypes.c_size_t),
                ("next_out", ctypes.c_void_p), ("avail_out", ctypes.c_size_t), ("total_out", ctypes.c_size_t),
                ("data_type", ctypes.c_int)]


def _lib():
    from beast_amd import pmd
    L = pmd.lib()
    vp = ctypes.c_void_p
    L.bpmd_inflate_stream_create.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
    L.bpmd_inflate_stream_write.argtypes = [vp, ctypes.POINTER(ZParams), ctypes.c_int]
    L.bpmd_inflate_stream_reset.argtypes = [vp, ctypes.c_int]
    L.bpmd_inflate_stream_footprint.argtypes = [vp, ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_size_t)]
    L.bpmd_stream_destroy.argtypes = [vp]
    return L


class GpuInflater:
    def __init__(self, wbits=15):
        self.L = _lib()
        self.h = ctypes.c_void_p()
        assert self.L.bpmd_inflate_stream_create(wbits, ctypes.byref(self.h)) == 0

    def write(self, zs, flush):
        r = self.L.bpmd_inflate_stream_write(self.h, ctypes.byref(zs), flush)
        assert r >= 0, f"C ABI error {r}"
        return r

    def footprint(self):
        hb, db = ctypes.c_size_t(), ctypes.c_size_t()
        assert self.L.bpmd_inflate_stream_footprint(self.h, ctypes.byref(hb), ctypes.byref(db)) == 0
        return hb.value, db.value

    def close(self):
        self.L.bpmd_stream_destroy(self.h)


class OracleInflater:
    def __init__(self, wbits=15):
        self.z = O.Inflater(wbits)

    def write(self, zs, flush):
        return self.z.write(zs, FLUSH_NAMES.get(flush, "sync"))


def drive(inf, stream: bytes, calls):
    """calls: [(cut, avail_out, flush)].  Each call offers input from the
    inflater's consumed position to max(cut, consumed).  Returns
    [(status, output bytes or None after an error)] and stops after an error
    or end_of_stream."""
    src = ctypes.create_string_buffer(stream, max(1, len(stream)))
    base = ctypes.addressof(src)
    consumed = 0
    res = []
    for cut, room, flush in calls:
        cut = max(cut, consumed)
        buf = ctypes.create_string_buffer(max(1, room))
        zs = ZParams(base + consumed if cut > consumed else None, cut - consumed, 0,
                     ctypes.addressof(buf), room, 0, 2)
        st = inf.write(zs, flush)
        err = st > 2
        res.append((st, None if err else buf.raw[:zs.total_out]))
        consumed += zs.total_in
        if err:
            break
    return res


def compare(stream, calls, wbits=15, label=""):
    g = GpuInflater(wbits)
    try:
        got = drive(g, stream, calls)
    finally:
        g.close()
    want = drive(OracleInflater(wbits), stream, calls)
    n = min(len(got), len(want))
    for i in range(n):
        assert got[i][0] == want[i][0], (label, i, O.ERRORS[got[i][0]], O.ERRORS[want[i][0]], calls[i])
        assert got[i][1] == want[i][1], (label, i, None if got[i][1] is None else len(got[i][1]),
                                         None if want[i][1] is None else len(want[i][1]), calls[i])
    assert len(got) == len(want), (label, len(got), len(want))
    return want


def connection_stream(msgs, level=6, wbits=15, mem=4, takeover=True):
    """What one connection's inflater receives: each payload followed by the
    00 00 FF FF that inflate_with_eb feeds (impl_base.hpp:179-190)."""
    if takeover:
        pays = O.pmd_deflate_stream(msgs, level, wbits, mem)
    else:
        pays = [O.pmd_deflate(m, level, wbits, mem) for m in msgs]
    return b"".join(p + EB for p in pays)


def _msgs(kind, sizes, seed):
    data, off, lens = synth.make_batch(kind, sizes, seed=seed)
    return [bytes(data[int(off[i]):int(off[i]) + int(lens[i])]) for i in range(len(sizes))]


def random_calls(rng, total, n_calls, rooms, flushes=(SYNC,)):
    cuts = sorted(rng.randrange(0, total + 1) for _ in range(n_calls - 1)) + [total]
    calls = [(c, rng.choice(rooms), rng.choice(flushes)) for c in cuts]
    # drain: keep calling with everything offered until nothing more comes out
    calls += [(total, 1 << 16, SYNC)] * 8
    return calls


@pytest.mark.parametrize("kind", ["json", "corpus1", "binary", "random"])
@pytest.mark.parametrize("level,mem", [(1, 4), (6, 4), (8, 4), (9, 9), (6, 1)])
def test_connection_random_cuts_match_reference(kind, level, mem):
    rng = random.Random(f"{kind}{level}{mem}")
    msgs = _msgs(kind, [rng.choice([0, 1, 100, 1024, 4096, 9000]) for _ in range(12)], seed=level * 10 + mem)
    stream = connection_stream(msgs, level=level, mem=mem)
    for trial in range(3):
        calls = random_calls(rng, len(stream), rng.choice([3, 20, 80]), [4096, 1 << 16, 300, 7])
        compare(stream, calls, label=f"{kind} L{level} m{mem} t{trial}")


def test_output_room_of_one_byte_and_big_blocks():
    # memLevel 9: blocks of up to 32 Ki symbols; output handed out a byte at a time
    msgs = _msgs("corpus1", [20000], seed=5)
    stream = connection_stream(msgs, level=9, mem=9)
    calls = [(len(stream), 1, SYNC)] * 3000 + [(len(stream), 1 << 16, SYNC)] * 4
    compare(stream, calls, label="room 1")


def test_flush_block_and_trees_mixed():
    rng = random.Random(11)
    msgs = _msgs("json", [3000, 50, 8000, 0, 700], seed=3)
    stream = connection_stream(msgs, level=6, mem=4)
    for trial in range(4):
        calls = random_calls(rng, len(stream), 40, [1 << 16, 500], flushes=(SYNC, BLOCK, TREES, NONE))
        compare(stream, calls, label=f"flush mix {trial}")


def test_flush_trees_known_answers():
    with open(os.path.join(GOLD, "inflate_kat.json")) as f:
        k = json.load(f)["flush_trees"]
    for name in ("fixed", "stored"):
        stream = bytes.fromhex(k[name])
        want = compare(stream, [(len(stream), 5, TREES), (len(stream), 5, SYNC)], label=name)
        assert want[1][1] == bytes.fromhex(k["expect_out"])


def test_known_answer_vectors_split():
    with open(os.path.join(GOLD, "inflate_kat.json")) as f:
        vecs = json.load(f)["vectors"]
    for v in vecs:
        d = bytes.fromhex(v["in"])
        if "prefix" in v:
            d = d[:v["prefix"]]
        w = v.get("wbits", 15)
        whole = compare(d, [(len(d), 1024, SYNC), (len(d), 1024, SYNC)], wbits=w, label=v["in"][:16])
        assert O.ERRORS[whole[0][0]] == v["expect"]
        for cut in range(1, len(d)):
            compare(d, [(cut, 1024, SYNC), (len(d), 1024, SYNC), (len(d), 1024, SYNC)], wbits=w,
                    label=f"{v['in'][:16]}@{cut}")


def test_small_window_call_split_rule():
    """Stream compressed with a 32 KiB window, inflated with windowBits 9..12:
    whether a long distance is invalid depends on where the calls split."""
    rng = random.Random(7)
    msgs = _msgs("corpus1", [6000, 6000], seed=9)
    stream = connection_stream(msgs, level=9, wbits=15, mem=8)
    seen_err = False
    for w in (9, 10, 12):
        for trial in range(6):
            calls = random_calls(rng, len(stream), rng.choice([2, 10, 40]), [1 << 16, 2000, 64])
            want = compare(stream, calls, wbits=w, label=f"w{w} t{trial}")
            seen_err |= any(s == O.ERROR_CODES["invalid_distance"] for s, _ in want)
    assert seen_err   # the rule was exercised


def test_end_of_stream_then_done_mode():
    import zlib
    c = zlib.compressobj(6, zlib.DEFLATED, -15, 8)
    stream = c.compress(b"hello world " * 300) + c.flush(zlib.Z_FINISH) + b"trailing garbage"
    for cuts in ([len(stream)], [10, 40, len(stream)], list(range(1, len(stream) + 1, 3))):
        calls = [(x, 1 << 16, SYNC) for x in cuts] + [(len(stream), 1 << 16, SYNC)] * 3
        want = compare(stream, calls, label=f"eos {len(cuts)}")
        assert want[-1][0] == O.ERROR_CODES["end_of_stream"]


def test_errors_then_bad_mode():
    rng = random.Random(3)
    msgs = _msgs("json", [4096] * 4, seed=4)
    good = bytearray(connection_stream(msgs, level=6, mem=4))
    for trial in range(12):
        bad = bytearray(good)
        at = rng.randrange(len(bad) // 3, len(bad))
        bad[at] ^= 1 << rng.randrange(8)
        calls = random_calls(rng, len(bad), rng.choice([1, 5, 30]), [4096, 1 << 16])
        compare(bytes(bad), calls, label=f"corrupt {trial}@{at}")


def ws_read_message(inf, payload: bytes, user_buf=4096, rd_buf=1536):
    """read.hpp:1284-1356: rd_buf slices with Flush::sync, then
    inflate_with_eb until a call produces nothing.  Returns (status, bytes)."""
    out = bytearray()
    pos = 0
    src = ctypes.create_string_buffer(payload, max(1, len(payload)))
    while pos < len(payload):
        buf = ctypes.create_string_buffer(user_buf)
        k = min(rd_buf, len(payload) - pos)
        zs = ZParams(ctypes.addressof(src) + pos, k, 0, ctypes.addressof(buf), user_buf, 0, 2)
        st = inf.write(zs, SYNC)
        if st:   # check_stop_now: any error (need_buffers included) fails the read
            return st, bytes(out)
        pos += zs.total_in
        out += buf.raw[:zs.total_out]
    eb = ctypes.create_string_buffer(EB, 4)
    used = 0
    while True:
        buf = ctypes.create_string_buffer(user_buf)
        zs = ZParams(ctypes.addressof(eb) + used, 4 - used, 0, ctypes.addressof(buf), user_buf, 0, 2)
        st = inf.write(zs, SYNC)
        if st == 1:
            st = 0
        if st:
            return st, bytes(out)
        used += zs.total_in
        out += buf.raw[:zs.total_out]
        if zs.total_out == 0:
            return 0, bytes(out)


def test_c1_connection_bounded_memory():
    """configs[0]'s shape: one connection, 1 Ki x 1 KiB text messages, default
    context takeover at compLevel 8 / memLevel 4 (option.hpp:61-64), read as
    read.hpp does; identical to the oracle's never-reset inflater, and the
    stream's memory does not grow with the connection's age."""
    msgs = _msgs("json", [1024] * 1024, seed=0x5EED0001)
    pays = O.pmd_deflate_stream(msgs, 8, 15, 4)
    want = O.pmd_inflate_stream(pays, cap=1 << 16)
    g = GpuInflater(15)
    feet = []
    try:
        for i, p in enumerate(pays):
            st, got = ws_read_message(g, p)
            assert (st, got) == want[i], (i, st, len(got))
            assert got == msgs[i]
            if i in (63, 1023):
                feet.append(g.footprint())
    finally:
        g.close()
    (h0, d0), (h1, d1) = feet
    assert h1 <= max(h0, 1) * 2 + 4096 and d1 == d0, feet
    assert h1 < 64 * 1024 and d1 < 1 << 20, feet


def test_many_small_writes_per_call_cost_bounded():
    """A 64 KiB message in 100-byte writes: every write decodes its own bytes
    plus at most one round again (the kept input stays small)."""
    msgs = _msgs("json", [65536], seed=21)
    stream = connection_stream(msgs, level=6, mem=4)
    g = GpuInflater(15)
    src = ctypes.create_string_buffer(stream, len(stream))
    out = bytearray()
    peak = 0
    try:
        pos = 0
        while pos < len(stream):
            k = min(100, len(stream) - pos)
            buf = ctypes.create_string_buffer(1 << 17)
            zs = ZParams(ctypes.addressof(src) + pos, k, 0, ctypes.addressof(buf), 1 << 17, 0, 2)
            assert g.write(zs, SYNC) == 0
            pos += zs.total_in
            out += buf.raw[:zs.total_out]
            peak = max(peak, g.footprint()[0])
    finally:
        g.close()
    assert bytes(out) == msgs[0]
    assert peak < 16 * 1024, peak
