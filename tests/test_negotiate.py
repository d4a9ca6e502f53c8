"""permessage-deflate negotiation wire format, against
the expectations of the reference's own tests (test/beast/websocket/
handshake.cpp:306-552, testExtRead / testExtWrite / testExtNegotiate),
restated here as data.  Host code: no device needed."""
import ctypes

import pytest

from beast_amd import pmd


class Offer(ctypes.Structure):
    _fields_ = [("accept", ctypes.c_int), ("server_max_window_bits", ctypes.c_int),
                ("client_max_window_bits", ctypes.c_int), ("server_no_context_takeover", ctypes.c_int),
                ("client_no_context_takeover", ctypes.c_int)]


class Options(ctypes.Structure):
    _fields_ = [("server_enable", ctypes.c_int), ("client_enable", ctypes.c_int),
                ("server_max_window_bits", ctypes.c_int), ("client_max_window_bits", ctypes.c_int),
                ("server_no_context_takeover", ctypes.c_int), ("client_no_context_takeover", ctypes.c_int)]


def _read(s: str) -> Offer:
    o = Offer()
    b = s.encode()
    assert pmd.lib().bpmd_pmd_read(b, len(b), ctypes.byref(o)) == 0
    return o


def _write(o: Offer) -> str:
    buf = ctypes.create_string_buffer(512)
    n = pmd.lib().bpmd_pmd_write(ctypes.byref(o), buf, 512)
    assert n >= 0
    return buf.value.decode()


def _negotiate(opts: Options, offer: Offer):
    cfg = Offer()
    buf = ctypes.create_string_buffer(512)
    n = pmd.lib().bpmd_pmd_negotiate(ctypes.byref(opts), ctypes.byref(offer), ctypes.byref(cfg), buf, 512)
    assert n >= 0
    return cfg, buf.value.decode()


REJECT = [
    "permessage-deflate; server_max_window_bits=8; server_max_window_bits=8",
    "permessage-deflate; server_max_window_bits", "permessage-deflate; server_max_window_bits=",
    "permessage-deflate; server_max_window_bits=-1", "permessage-deflate; server_max_window_bits=7",
    "permessage-deflate; server_max_window_bits=16",
    "permessage-deflate; server_max_window_bits=999999999999999999999999",
    "permessage-deflate; server_max_window_bits=9a",
    "permessage-deflate; client_max_window_bits=8; client_max_window_bits=8",
    "permessage-deflate; client_max_window_bits=-1", "permessage-deflate; client_max_window_bits=7",
    "permessage-deflate; client_max_window_bits=16",
    "permessage-deflate; client_max_window_bits=999999999999999999999999",
    "permessage-deflate; server_no_context_takeover; server_no_context_takeover",
    "permessage-deflate; server_no_context_takeover=-1", "permessage-deflate; server_no_context_takeover=x",
    'permessage-deflate; server_no_context_takeover="yz"',
    "permessage-deflate; server_no_context_takeover=999999999999999999999999",
    "permessage-deflate; client_no_context_takeover; client_no_context_takeover",
    "permessage-deflate; client_no_context_takeover=-1", "permessage-deflate; client_no_context_takeover=x",
    'permessage-deflate; client_no_context_takeover="yz"',
    "permessage-deflate; client_no_context_takeover=999999999999999999999999",
    "permessage-deflate; unknown", "permessage-deflate; unknown=", "permessage-deflate; unknown=1",
    "permessage-deflate; unknown=x", 'permessage-deflate; unknown="xy"',
]


@pytest.mark.parametrize("s", REJECT)
def test_read_rejects(s):
    assert not _read(s).accept


def test_read_accepts():
    o = _read("permessage-deflate; client_max_window_bits")
    assert o.accept and o.client_max_window_bits == -1
    o = _read("permessage-deflate; client_max_window_bits=")
    assert o.accept and o.client_max_window_bits == -1
    for name in ("server_no_context_takeover", "client_no_context_takeover"):
        for s in (f"permessage-deflate; {name}", f"permessage-deflate; {name}="):
            o = _read(s)
            assert o.accept and getattr(o, name) == 1
    o = _read("x-other; a=1, permessage-deflate; server_max_window_bits=10; client_no_context_takeover")
    assert o.accept and o.server_max_window_bits == 10 and o.client_no_context_takeover


def test_write():
    o = Offer(1, 0, 0, 0, 0)
    assert _write(o) == "permessage-deflate"
    o.server_max_window_bits = 10
    assert _write(o) == "permessage-deflate; server_max_window_bits=10"
    o.server_max_window_bits = -1
    assert _write(o) == "permessage-deflate; server_max_window_bits"
    o.server_max_window_bits, o.client_max_window_bits = 0, 10
    assert _write(o) == "permessage-deflate; client_max_window_bits=10"
    o.client_max_window_bits = -1
    assert _write(o) == "permessage-deflate; client_max_window_bits"
    o.client_max_window_bits, o.server_no_context_takeover = 0, 1
    assert _write(o) == "permessage-deflate; server_no_context_takeover"
    o.server_no_context_takeover, o.client_no_context_takeover = 0, 1
    assert _write(o) == "permessage-deflate; client_no_context_takeover"


def test_negotiate():
    opts = Options(1, 0, 15, 15, 0, 0)

    def accept(offer, result):
        cfg, got = _negotiate(opts, _read(offer))
        assert got == result, (offer, got)
        poc = _read(got)
        pmd.lib().bpmd_pmd_normalize(ctypes.byref(poc))
        assert poc.accept
        assert cfg.server_max_window_bits != 0 and cfg.client_max_window_bits != 0

    def reject(offer):
        cfg, got = _negotiate(opts, _read(offer))
        assert not cfg.accept and got == ""

    accept("permessage-deflate", "permessage-deflate")
    accept("permessage-deflate; server_max_window_bits=14", "permessage-deflate; server_max_window_bits=14")
    accept("permessage-deflate; server_max_window_bits=15", "permessage-deflate")
    accept("permessage-deflate; server_max_window_bits=8", "permessage-deflate; server_max_window_bits=9")
    opts.server_max_window_bits = 10
    accept("permessage-deflate", "permessage-deflate; server_max_window_bits=10")
    accept("permessage-deflate; server_max_window_bits=14", "permessage-deflate; server_max_window_bits=10")
    opts.server_max_window_bits = 8
    accept("permessage-deflate; server_max_window_bits=14", "permessage-deflate; server_max_window_bits=9")
    opts.server_max_window_bits = 15
    accept("permessage-deflate; client_max_window_bits", "permessage-deflate")
    opts.client_max_window_bits = 10
    accept("permessage-deflate; client_max_window_bits", "permessage-deflate; client_max_window_bits=10")
    reject("permessage-deflate")
    # server_enable off: never accepted
    opts = Options(0, 0, 15, 15, 0, 0)
    reject("permessage-deflate")
