"""Shared driver and cases for the per-stream inflater (zlib::inflate_stream
behind bpmd_inflate_stream_*): every write() is compared with the oracle's
restatement of Beast's inflate_stream (oracle/bzo_inflate.c =
inflate_stream.ipp:74-535 + bitstream.hpp + window.hpp) field by field --
status, next_in / avail_in / total_in, next_out / avail_out / total_out,
data_type, and the bytes in the caller's buffer (also after an error, which
returns without advancing z_params, inflate_stream.ipp:120-125).

Used by tests/test_gpu_zstream.py (the kernel, through the C ABI) and
tests/test_zstream_host.py (the kernel's own source built for the host)."""
import ctypes
import json
import os
import random

from beast_amd import synth
from oracle import oracle as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NONE, BLOCK, PARTIAL, SYNC, FULL, FINISH, TREES = range(7)
FLUSH_NAMES = {NONE: "none", BLOCK: "block", PARTIAL: "partial", SYNC: "sync", FULL: "full", FINISH: "finish",
               TREES: "trees"}
EB = b"\x00\x00\xff\xff"


class ZParams(ctypes.Structure):
    _fields_ = [("next_in", ctypes.c_void_p), ("avail_in", ctypes.c_size_t), ("total_in", ctypes.c_size_t),
                ("next_out", ctypes.c_void_p), ("avail_out", ctypes.c_size_t), ("total_out", ctypes.c_size_t),
                ("data_type", ctypes.c_int)]


class OracleInflater:
    def __init__(self, wbits=15):
        self.z = O.Inflater(wbits)

    def write(self, zs, flush):
        return self.z.write(zs, FLUSH_NAMES[flush])


def drive(inf, stream: bytes, calls):
    """calls: [(cut, avail_out, flush)].  Each call offers input from where
    the inflater's next_in stands to max(cut, that).  Returns one record per
    call: (status, total_in, avail_in, total_out, avail_out, data_type,
    in position, out position, the whole output buffer); stops after an
    error or end_of_stream."""
    src = ctypes.create_string_buffer(stream, max(1, len(stream)))
    base = ctypes.addressof(src)
    pos = 0
    recs = []
    for cut, room, flush in calls:
        cut = max(cut, pos)
        buf = ctypes.create_string_buffer(max(1, room))
        zs = ZParams(base + pos if cut > pos else None, cut - pos, 0, ctypes.addressof(buf), room, 0, 12345)
        st = inf.write(zs, flush)
        assert st >= 0, f"C ABI error {st}"
        in_at = (zs.next_in - base) if zs.next_in else pos
        out_at = (zs.next_out - ctypes.addressof(buf)) if zs.next_out else 0
        recs.append((st, zs.total_in, zs.avail_in, zs.total_out, zs.avail_out, zs.data_type, in_at, out_at,
                     buf.raw))
        pos += zs.total_in
        if st >= 2:
            break
    return recs


FIELDS = ("status", "total_in", "avail_in", "total_out", "avail_out", "data_type", "next_in", "next_out", "bytes")


def compare(make, stream, calls, wbits=15, label=""):
    """make(wbits) -> inflater under test.  Asserts every call equal to the
    oracle's; returns the oracle's records."""
    want = drive(OracleInflater(wbits), stream, calls)
    inf = make(wbits)
    try:
        got = drive(inf, stream, calls)
    finally:
        close = getattr(inf, "close", None)
        if close:
            close()
    for i in range(min(len(got), len(want))):
        for f, a, b in zip(FIELDS, got[i], want[i]):
            assert a == b, (label, "call", i, f, a if f != "bytes" else len(a), b if f != "bytes" else len(b),
                            calls[i], O.ERRORS[got[i][0]], O.ERRORS[want[i][0]])
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


def msgs_of(kind, sizes, seed):
    data, off, lens = synth.make_batch(kind, sizes, seed=seed)
    return [bytes(data[int(off[i]):int(off[i]) + int(lens[i])]) for i in range(len(sizes))]


def random_calls(rng, total, n_calls, rooms, flushes=(SYNC,)):
    cuts = sorted(rng.randrange(0, total + 1) for _ in range(n_calls - 1)) + [total]
    calls = [(c, rng.choice(rooms), rng.choice(flushes)) for c in cuts]
    # drain: keep calling with everything offered until nothing more comes out
    calls += [(total, 1 << 16, SYNC)] * 8
    return calls


def kat_vectors():
    with open(os.path.join(GOLD, "inflate_kat.json")) as f:
        return json.load(f)


# ------------------------------------------------------- websocket read path

class WsReader:
    """websocket::stream's sync read_some inflate branch
    (read.hpp:1284-1385) over one inflater: rd_buf filled from the socket up
    to its capacity, avail_in clamped to the frame's rd_remain, rd_buf and
    rd_remain advanced by exactly total_in, then inflate_with_eb
    (impl_base.hpp:179-190) with rd_eb_consumed until a call produces
    nothing; any error stops the read (check_stop_now).  Messages are given
    as their frames' payloads (headers parsed elsewhere)."""

    def __init__(self, inf, rd_buf_cap=1536):
        self.inf = inf
        self.cap = rd_buf_cap
        self.calls = []   # (status, total_in, total_out, data_type) of every write()

    def begin(self, frames):
        self.frames = list(frames)
        self.sock = bytearray()
        self.rd_buf = bytearray()
        self.rd_remain = 0
        self.fin = False
        self.rd_eb_consumed = 0   # rd_deflated(rsv1), impl_base.hpp:68-77
        self.rd_done = False
        for p in self.frames:
            self.sock += p
        self._next_frame()

    def _next_frame(self):
        p = self.frames.pop(0)
        self.rd_remain = len(p)
        self.fin = not self.frames

    def _write(self, data: bytes, room: int):
        src = ctypes.create_string_buffer(data, max(1, len(data)))
        buf = ctypes.create_string_buffer(max(1, room))
        zs = ZParams(ctypes.addressof(src) if data else None, len(data), 0, ctypes.addressof(buf), room, 0, 0)
        st = self.inf.write(zs, SYNC)
        self.calls.append((st, zs.total_in, zs.total_out, zs.data_type))
        return st, zs, buf.raw[:zs.total_out]

    def read_some(self, size):
        """One read_some into a `size`-byte buffer: (bytes, status)."""
        while self.rd_remain == 0 and not self.fin:
            self._next_frame()
        out = bytearray()
        did_read = False
        room = size
        while room > 0:
            if self.rd_remain > 0:
                if self.rd_buf:
                    data = bytes(self.rd_buf[:min(self.rd_remain, len(self.rd_buf))])
                elif not did_read:
                    k = min(self.cap - len(self.rd_buf), len(self.sock))
                    self.rd_buf += self.sock[:k]
                    del self.sock[:k]
                    data = bytes(self.rd_buf[:min(self.rd_remain, len(self.rd_buf))])
                    did_read = True
                else:
                    break
                st, zs, got = self._write(data, room)
                if st:
                    return bytes(out), st
                self.rd_remain -= zs.total_in
                del self.rd_buf[:zs.total_in]
            elif self.fin:
                st, zs, got = self._write(EB[self.rd_eb_consumed:], room)
                self.rd_eb_consumed += zs.total_in
                assert self.rd_eb_consumed <= 4
                if st == 1:   # need_buffers cleared
                    st = 0
                if st:
                    return bytes(out), st
                if zs.total_out == 0:
                    self.rd_done = True
                    break
            else:
                break
            out += got
            room -= zs.total_out
        return bytes(out), 0

    def read_message(self, frames, size):
        """do { read_some(size) } while (!is_message_done()) -- the shape of
        read3.cpp:1190-1200; returns (bytes, first error or 0)."""
        self.begin(frames)
        msg = bytearray()
        while True:
            got, st = self.read_some(size)
            msg += got
            if st:
                return bytes(msg), st
            if self.rd_done:
                return bytes(msg), 0


def ws_replay(make, messages, size, rd_buf_cap=1536, wbits=15):
    """Reads every message (a list of frame payloads) through WsReader on the
    inflater under test and on the oracle; asserts the same bytes, errors
    and per-write() z_params; returns the oracle side's messages."""
    a = WsReader(make(wbits), rd_buf_cap)
    b = WsReader(OracleInflater(wbits), rd_buf_cap)
    res = []
    try:
        for i, frames in enumerate(messages):
            ga = a.read_message(frames, size)
            gb = b.read_message(frames, size)
            assert ga == gb, (i, len(ga[0]), ga[1], len(gb[0]), gb[1])
            if a.calls != b.calls:
                k = next((k for k, (x, y) in enumerate(zip(a.calls, b.calls)) if x != y), None)
                raise AssertionError(("message", i, "write", k, a.calls[k] if k is not None else len(a.calls),
                                      b.calls[k] if k is not None else len(b.calls)))
            res.append(gb)
    finally:
        close = getattr(a.inf, "close", None)
        if close:
            close()
    return res


# ------------------------------------------------------------------- cases

def case_connection_random_cuts(make, kind, level, mem):
    rng = random.Random(f"{kind}{level}{mem}")
    msgs = msgs_of(kind, [rng.choice([0, 1, 100, 1024, 4096, 9000]) for _ in range(12)], seed=level * 10 + mem)
    stream = connection_stream(msgs, level=level, mem=mem)
    for trial in range(3):
        calls = random_calls(rng, len(stream), rng.choice([3, 20, 80]), [4096, 1 << 16, 300, 7, 1, 258, 257])
        compare(make, stream, calls, label=f"{kind} L{level} m{mem} t{trial}")


def case_foreign_payloads(make):
    """A connection whose peer is another encoder (CPython's zlib, no context
    takeover): payloads with mid-message none / block / sync / full flushes and
    zlib's strategies (tests/foreign.py), each followed by 00 00 FF FF, under
    random cuts and output rooms."""
    from tests.foreign import foreign_payloads
    rng = random.Random("foreign")
    pays, _, _ = foreign_payloads(21, 24)
    stream = b"".join(p + EB for p in pays)
    for trial in range(3):
        calls = random_calls(rng, len(stream), rng.choice([5, 40, 160]), [4096, 1 << 16, 300, 7, 1, 258])
        compare(make, stream, calls, label=f"foreign t{trial}")


def case_output_room_one_byte(make, n_calls=3000):
    # memLevel 9: blocks of up to 32 Ki symbols; output handed out a byte at a time
    msgs = msgs_of("corpus1", [20000], seed=5)
    stream = connection_stream(msgs, level=9, mem=9)
    calls = [(len(stream), 1, SYNC)] * n_calls + [(len(stream), 1 << 16, SYNC)] * 4
    compare(make, stream, calls, label="room 1")


def case_byte_at_a_time_input(make):
    msgs = msgs_of("json", [3000, 20], seed=6)
    stream = connection_stream(msgs, level=6, mem=4)
    calls = [(k, 1 << 16, SYNC) for k in range(1, len(stream) + 1)] + [(len(stream), 1 << 16, SYNC)] * 3
    compare(make, stream, calls, label="input 1")


def case_flush_mix(make):
    rng = random.Random(11)
    msgs = msgs_of("json", [3000, 50, 8000, 0, 700], seed=3)
    stream = connection_stream(msgs, level=6, mem=4)
    for trial in range(4):
        calls = random_calls(rng, len(stream), 40, [1 << 16, 500, 3],
                             flushes=(SYNC, BLOCK, TREES, NONE, FINISH, PARTIAL, FULL))
        compare(make, stream, calls, label=f"flush mix {trial}")


def case_flush_trees_kat(make):
    k = kat_vectors()["flush_trees"]
    for name in ("fixed", "stored"):
        stream = bytes.fromhex(k[name])
        want = compare(make, stream, [(len(stream), 5, TREES), (len(stream), 5, SYNC)], label=name)
        assert want[1][8][:want[1][3]] == bytes.fromhex(k["expect_out"])


def case_kat_split(make, every_cut=True):
    for v in kat_vectors()["vectors"]:
        d = bytes.fromhex(v["in"])
        if "prefix" in v:
            d = d[:v["prefix"]]
        w = v.get("wbits", 15)
        whole = compare(make, d, [(len(d), 1024, SYNC), (len(d), 1024, SYNC)], wbits=w, label=v["in"][:16])
        assert O.ERRORS[whole[0][0]] == v["expect"]
        cuts = range(1, len(d)) if every_cut else range(1, len(d), max(1, len(d) // 8))
        for cut in cuts:
            compare(make, d, [(cut, 1024, SYNC), (len(d), 1024, SYNC), (len(d), 1024, SYNC)], wbits=w,
                    label=f"{v['in'][:16]}@{cut}")


def case_small_window(make):
    """Stream compressed with a 32 KiB window, inflated with windowBits 9..12:
    whether a long distance is invalid depends on where the calls split."""
    rng = random.Random(7)
    msgs = msgs_of("corpus1", [6000, 6000], seed=9)
    stream = connection_stream(msgs, level=9, wbits=15, mem=8)
    seen_err = False
    for w in (9, 10, 12):
        for trial in range(6):
            calls = random_calls(rng, len(stream), rng.choice([2, 10, 40]), [1 << 16, 2000, 64])
            want = compare(make, stream, calls, wbits=w, label=f"w{w} t{trial}")
            seen_err |= any(r[0] == O.ERROR_CODES["invalid_distance"] for r in want)
    assert seen_err   # the rule was exercised


def case_end_of_stream(make):
    import zlib
    c = zlib.compressobj(6, zlib.DEFLATED, -15, 8)
    stream = c.compress(b"hello world " * 300) + c.flush(zlib.Z_FINISH) + b"trailing garbage"
    for cuts in ([len(stream)], [10, 40, len(stream)], list(range(1, len(stream) + 1, 3))):
        calls = [(x, 1 << 16, SYNC) for x in cuts] + [(len(stream), 1 << 16, SYNC)] * 3
        want = compare(make, stream, calls, label=f"eos {len(cuts)}")
        assert want[-1][0] == O.ERROR_CODES["end_of_stream"]


def case_stored_blocks(make):
    rng = random.Random(12)
    msgs = msgs_of("random", [70000, 5, 3000], seed=12)
    stream = connection_stream(msgs, level=0, mem=4)   # stored blocks
    for trial in range(4):
        calls = random_calls(rng, len(stream), rng.choice([3, 30]), [1 << 17, 4000, 1, 70000],
                             flushes=(SYNC, TREES, BLOCK))
        compare(make, stream, calls, label=f"stored {trial}")


def case_errors(make):
    rng = random.Random(3)
    msgs = msgs_of("json", [4096] * 4, seed=4)
    good = bytearray(connection_stream(msgs, level=6, mem=4))
    for trial in range(12):
        bad = bytearray(good)
        at = rng.randrange(len(bad) // 3, len(bad))
        bad[at] ^= 1 << rng.randrange(8)
        calls = random_calls(rng, len(bad), rng.choice([1, 5, 30]), [4096, 1 << 16, 100])
        calls += [(len(bad), 1 << 16, SYNC)] * 2   # BAD mode answers need_buffers
        compare(make, bytes(bad), calls, label=f"corrupt {trial}@{at}")


def issue3028_message() -> bytes:
    with open(os.path.join(GOLD, "ws_issues.json")) as f:
        return bytes.fromhex(json.load(f)["issue3028"]["message_hex"])


def issue1630_frames():
    """[(opcode, payload)] of the four packets' frames, read3.cpp:619-1009."""
    with open(os.path.join(GOLD, "ws_issues.json")) as f:
        packets = [bytes.fromhex(p) for p in json.load(f)["issue1630"]["packets_hex"]]
    out = []
    for p in packets:
        i = 0
        while i < len(p):
            b0, b1 = p[i], p[i + 1]
            assert b0 & 0x80 and b0 & 0x40 and not b1 & 0x80   # FIN, RSV1 (compressed), unmasked
            n = b1 & 0x7f
            i += 2
            if n == 126:
                n = int.from_bytes(p[i:i + 2], "big")
                i += 2
            elif n == 127:
                n = int.from_bytes(p[i:i + 8], "big")
                i += 8
            out.append((b0 & 0x0f, p[i:i + n]))
            i += n
    return out
