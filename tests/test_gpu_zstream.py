"""GPU: the per-stream inflater (bpmd_inflate_stream_*, behind the drop-in
zlib::inflate_stream) runs Beast's inflate_stream state machine on the
device (beast_amd/csrc/pmd_zstream.hip).  Every write() is checked against
the oracle's restatement (oracle/bzo_inflate.c = inflate_stream.ipp:74-535 +
bitstream.hpp + window.hpp) field by field -- status, next_in / avail_in /
total_in, next_out / avail_out / total_out, data_type and the bytes in the
caller's buffer (tests/zstream_cases.py):

* random input cuts and output rooms (1, 7, 257, 258, 300 ... bytes), one
  inflater for a whole connection with context takeover (Beast never resets
  zi between messages, impl_base.hpp:192-202);
* input a byte at a time, output a byte at a time, every Flush value, the
  Flush::trees known answers, the reference's inflate KATs split at every
  byte, stored blocks, small windows (the per-call window rule,
  inflate_stream.ipp:1046-1061), end of stream, corrupted input and BAD mode;
* websocket::stream's read path replayed on both sides (read.hpp:1284-1385:
  rd_buf advanced by total_in, inflate_with_eb with rd_eb_consumed): the
  reference's issue 3028 (three context-takeover messages read one byte per
  read_some, read3.cpp:1133-1226) and issue 1630 (four packets whose
  deflate blocks split UTF-8 characters, read3.cpp:619-1009);
* configs[0]'s shape (1 Ki x 1 KiB messages on one connection) with the
  stream's memory bounded."""
import ctypes

import pytest

from oracle import oracle as O
from tests import zstream_cases as Z

pytestmark = pytest.mark.gpu


def _lib():
    from beast_amd import pmd
    L = pmd.lib()
    vp = ctypes.c_void_p
    L.bpmd_inflate_stream_create.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
    L.bpmd_inflate_stream_write.argtypes = [vp, ctypes.POINTER(Z.ZParams), ctypes.c_int]
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

    def reset(self, wbits):
        assert self.L.bpmd_inflate_stream_reset(self.h, wbits) == 0

    def footprint(self):
        hb, db = ctypes.c_size_t(), ctypes.c_size_t()
        assert self.L.bpmd_inflate_stream_footprint(self.h, ctypes.byref(hb), ctypes.byref(db)) == 0
        return hb.value, db.value

    def close(self):
        self.L.bpmd_stream_destroy(self.h)


make = GpuInflater


@pytest.mark.parametrize("kind", ["json", "corpus1", "binary", "random"])
@pytest.mark.parametrize("level,mem", [(1, 4), (6, 4), (8, 4), (9, 9), (6, 1)])
def test_connection_random_cuts(kind, level, mem):
    Z.case_connection_random_cuts(make, kind, level, mem)


def test_foreign_encoder_connection():
    Z.case_foreign_payloads(make)


def test_output_room_one_byte():
    Z.case_output_room_one_byte(make, n_calls=1200)


def test_byte_at_a_time_input():
    Z.case_byte_at_a_time_input(make)


def test_flush_mix():
    Z.case_flush_mix(make)


def test_flush_trees_known_answers():
    Z.case_flush_trees_kat(make)


def test_known_answer_vectors_split():
    Z.case_kat_split(make)


def test_small_window_call_split_rule():
    Z.case_small_window(make)


def test_end_of_stream_then_done_mode():
    Z.case_end_of_stream(make)


def test_stored_blocks():
    Z.case_stored_blocks(make)


def test_errors_then_bad_mode():
    Z.case_errors(make)


@pytest.mark.parametrize("par", [0, 1, 8, 9])
def test_serial_and_parallel_fast_loops(par):
    """inflate_fast runs wave-parallel by default (pmd_zstream.hip pfast: the
    lanes decode every candidate bit offset of a window, the scalar unit
    replays inflate_fast on the chain of real token starts), and so do the
    dynamic header's code lengths (hdr_par); the serial loops they replay
    stay selectable (bpmd_diag_set_zstream_parallel bit 0 = pfast, bit 3 =
    the serial code-length loop; BPMD_ZSTREAM_PAR=0 / BPMD_ZSTREAM_HPAR=0).
    Every combination must give the oracle's write()s."""
    L = _lib()
    L.bpmd_diag_set_zstream_parallel.argtypes = [ctypes.c_int]
    L.bpmd_diag_set_zstream_parallel(par)
    try:
        for kind in ("json", "binary", "random"):
            Z.case_connection_random_cuts(make, kind, 6, 4)
        Z.case_foreign_payloads(make)
        Z.case_errors(make)
        Z.case_small_window(make)
        Z.case_byte_at_a_time_input(make)
        Z.case_kat_split(make, every_cut=False)
    finally:
        L.bpmd_diag_set_zstream_parallel(-1)


def test_reset_between_streams():
    """reset(windowBits) mid-stream: fresh state and window, new size."""
    msgs = Z.msgs_of("json", [5000, 5000], seed=31)
    s1 = Z.connection_stream(msgs[:1], level=6, mem=4)
    s2 = Z.connection_stream(msgs[1:], level=6, wbits=10, mem=4)
    g = GpuInflater(15)
    o = Z.OracleInflater(15)
    try:
        Z.drive(g, s1, [(len(s1) // 2, 1 << 16, Z.SYNC)])
        Z.drive(o, s1, [(len(s1) // 2, 1 << 16, Z.SYNC)])
        g.reset(10)
        o.z.reset(10)
        calls = [(len(s2) // 3, 100, Z.SYNC), (len(s2), 1 << 16, Z.SYNC), (len(s2), 1 << 16, Z.SYNC)]
        assert Z.drive(g, s2, calls) == Z.drive(o, s2, calls)
    finally:
        g.close()


def test_issue3028_one_byte_reads():
    """read3.cpp:1133-1226: the client writes the message three times with
    context takeover (default pmd options: compLevel 8, memLevel 4,
    option.hpp:61-64); the server reads each with read_some into a 1-byte
    buffer until is_message_done()."""
    msg = Z.issue3028_message()
    pays = O.pmd_deflate_stream([msg] * 3, 8, 15, 4)
    res = Z.ws_replay(make, [[p] for p in pays], size=1)
    assert all(r == (msg, 0) for r in res)


@pytest.mark.parametrize("size,rd_buf", [(4096, 1536), (1, 1536), (7, 64), (65536, 4096)])
def test_issue1630_packets(size, rd_buf):
    """read3.cpp:619-1009: four compressed text frames on one connection
    whose deflate blocks split multi-byte characters across calls; every
    message inflates without error and is valid UTF-8."""
    frames = Z.issue1630_frames()
    res = Z.ws_replay(make, [[p] for _, p in frames], size=size, rd_buf_cap=rd_buf)
    for got, st in res:
        assert st == 0 and O.utf8_check(got) == 0


def test_c1_connection_bounded_memory():
    """configs[0]'s shape: one connection, 1 Ki x 1 KiB text messages, default
    context takeover at compLevel 8 / memLevel 4 (option.hpp:61-64), read as
    read.hpp does; identical to the oracle's never-reset inflater call by
    call, and the stream's memory does not grow with the connection's age."""
    msgs = Z.msgs_of("json", [1024] * 1024, seed=0x5EED0001)
    pays = O.pmd_deflate_stream(msgs, 8, 15, 4)
    g = GpuInflater(15)
    a = Z.WsReader(g, 1536)
    b = Z.WsReader(Z.OracleInflater(15), 1536)
    feet = []
    try:
        for i, p in enumerate(pays):
            got = a.read_message([p], 4096)
            assert got == b.read_message([p], 4096) == (msgs[i], 0), i
            if i in (63, 1023):
                feet.append(g.footprint())
        assert a.calls == b.calls
    finally:
        g.close()
    (h0, d0), (h1, d1) = feet
    # host: only the pinned staging of the call's copies (no decoder state)
    assert h1 == h0 and h0 < 1 << 20 and d1 == d0 and d1 < 1 << 20, feet


def test_many_small_writes():
    """A 64 KiB message in 100-byte writes: the device state carries the
    reservoir, so nothing is re-decoded and nothing is kept on the host."""
    msgs = Z.msgs_of("json", [65536], seed=21)
    stream = Z.connection_stream(msgs, level=6, mem=4)
    calls = [(min(k, len(stream)), 1 << 17, Z.SYNC) for k in range(100, len(stream) + 100, 100)]
    calls += [(len(stream), 1 << 17, Z.SYNC)] * 2
    want = Z.compare(make, stream, calls, label="100-byte writes")
    assert b"".join(r[8][:r[3]] for r in want) == msgs[0]
