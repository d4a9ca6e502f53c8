"""Frame-adjacent byte passes, CPU side: the oracle's
masking and UTF-8 checker against the reference's own test expectations
(test/beast/websocket/utf8_checker.cpp, restated in tests/utf8_cases.py),
RFC 6455's masking example and CPython's UTF-8 decoder; and the argument
checks of the new C-ABI entry points (no device needed)."""
import codecs
import ctypes
import random

from beast_amd import pmd
from oracle import oracle as O
from tests import utf8_cases


def test_mask_rfc6455_example():
    # RFC 6455 §5.7: "Hello" masked with the key 37 fa 21 3d is 7f 9f 4d 51 58
    key = int.from_bytes(bytes.fromhex("37fa213d"), "little")
    assert O.mask(b"Hello", key) == bytes.fromhex("7f9f4d5158")


def test_mask_phase_and_involution():
    rng = random.Random(3)
    for _ in range(300):
        data = rng.randbytes(rng.randrange(0, 300))
        key = rng.getrandbits(32)
        cut = rng.randrange(0, len(data) + 1)
        whole = O.mask(data, key)
        # a prepared key carries its rotation from one buffer to the next (mask.ipp:53-58)
        assert O.mask(data[:cut], key) + O.mask(data[cut:], key, phase=cut % 4) == whole
        assert O.mask(whole, key) == data


def test_utf8_reference_cases_streaming():
    n = 0
    for segs, writes, fin in utf8_cases.cases():
        u = O.Utf8Checker()
        got = [u.write(s) for s in segs]
        assert got == writes, (b"|".join(segs).hex(), got, writes)
        if fin is not None:
            assert u.finish() == fin, b"|".join(segs).hex()
        n += 1
    assert n > 3000


def test_utf8_reference_cases_whole_prefix():
    """Each write() verdict equals that of one write() over the whole prefix so
    far -- the batch kernel's semantics."""
    for acc, verdict in utf8_cases.prefixes():
        v = O.utf8_check(acc)
        if verdict is None:
            assert v != 2, acc.hex()
        else:
            assert v == verdict, (acc.hex(), v, verdict)


def _py_verdict(b: bytes) -> int:
    try:
        codecs.getincrementaldecoder("utf-8")().decode(b, final=False)
    except UnicodeDecodeError:
        return 2
    try:
        b.decode("utf-8")
    except UnicodeDecodeError:
        return 1
    return 0


SPECIAL = [0x00, 0x41, 0x7f, 0x80, 0x8f, 0x90, 0x9f, 0xa0, 0xbf, 0xc0, 0xc1, 0xc2, 0xdf, 0xe0, 0xe1, 0xec, 0xed, 0xee,
           0xef, 0xf0, 0xf1, 0xf3, 0xf4, 0xf5, 0xf7, 0xf8, 0xfe, 0xff]
ALPHABET = ["a", "~", "é", "߿", "ࠀ", "ж", "語", "퟿", "", "�", "￿",
            "\U00010000", "\U0001f600", "\U0010ffff"]


def utf8_fuzz(rng, n):
    out = []
    for _ in range(n):
        kind = rng.randrange(5)
        if kind == 0:
            b = rng.randbytes(rng.randrange(0, 12))
        elif kind == 1:
            b = bytes(rng.choice(SPECIAL) for _ in range(rng.randrange(1, 9)))
        else:
            s = "".join(rng.choice(ALPHABET) for _ in range(rng.randrange(0, 30)))
            b = bytearray(s.encode())
            if kind == 2 and b:
                b[rng.randrange(len(b))] = rng.choice(SPECIAL)
            elif kind == 3:
                b = b[:rng.randrange(len(b) + 1)]
            b = bytes(b)
        out.append(b)
    return out


def test_utf8_oracle_matches_cpython_decoder():
    """Whole messages: valid exactly when CPython decodes them.  Prefixes:
    whatever CPython's incremental decoder already rejects is invalid here
    too (CPython 3.10 does not reject every invalid prefix early, e.g. ED A0;
    the reference's fail-fast cases pin those)."""
    rng = random.Random(11)
    for b in utf8_fuzz(rng, 20000):
        v, pv = O.utf8_check(b), _py_verdict(b)
        assert (v == 0) == (pv == 0), b.hex()
        if pv == 2:
            assert v == 2, b.hex()


def test_utf8_streaming_equals_whole():
    rng = random.Random(12)
    for b in utf8_fuzz(rng, 3000):
        cuts = sorted(rng.randrange(len(b) + 1) for _ in range(rng.randrange(0, 4)))
        u = O.Utf8Checker()
        prev, ok = 0, True
        for c in cuts + [len(b)]:
            ok = u.write(b[prev:c]) and ok
            prev = c
            if not ok:
                break
        v = 2 if not ok else (0 if u.finish() else 1)
        assert v == O.utf8_check(b), (b.hex(), cuts)


def test_frame_entry_points_validate_before_device_use():
    L = pmd.lib()
    assert L.bpmd_mask_batch(None, None, None, 0, None, None, None) == 0
    assert L.bpmd_mask_batch(None, None, None, 1, None, None, None) == -1
    assert L.bpmd_utf8_check_batch(None, None, None, 1, None, None) == -1
    cfg = pmd._Cfg(6, 7, 4, 0, 0)
    assert L.bpmd_read_batch(ctypes.byref(cfg), None, None, None, None, None, 1, None, None, None, None, None,
                             None) == -2
    cfg = pmd._Cfg(6, 15, 4, 0, 0)
    assert L.bpmd_read_batch(ctypes.byref(cfg), None, None, None, None, None, 1, None, None, None, None, None,
                             None) == -1
    assert L.bpmd_write_batch(ctypes.byref(pmd._Cfg(10, 15, 4, 0, 0)), None, None, None, None, 1, None, None, None,
                              None, None, None) == -1
    assert L.bpmd_inflate_takeover_batch(ctypes.byref(cfg), None, None, None, None, 1, None, None, None, None, None,
                                         None) == -1
    assert L.bpmd_slide_batch(None, None, None, None, 1, None) == -1
    assert L.bpmd_frame_batch(None, None, None, None, None, None, None, 4096, 0, None, None, None) == 0
    assert L.bpmd_frame_batch(None, None, None, None, None, None, None, 4096, 1, None, None, None) == -1


# RFC 6455 §5.7 and RFC 7692 §7.2.3 example frames: the header layout that
# websocket/detail/frame.hpp:134-175 writes (key little-endian on the wire)
_HELLO_DEFLATED = bytes([0xf2, 0x48, 0xcd, 0xc9, 0xc9, 0x07, 0x00])


def test_frame_headers_rfc_examples():
    assert O.frame_write(b"Hello", 1, False) == bytes([0x81, 0x05]) + b"Hello"
    assert O.frame_write(b"Hello", 1, False, keys=[0x3d21fa37]) == bytes(
        [0x81, 0x85, 0x37, 0xfa, 0x21, 0x3d, 0x7f, 0x9f, 0x4d, 0x51, 0x58])
    assert O.frame_write(b"Hello", 1, False, frame_max=3) == bytes([0x01, 0x03]) + b"Hel" + bytes([0x80, 0x02]) + b"lo"
    f = O.frame_write(bytes(256), 2, False)
    assert f[:4] == bytes([0x82, 0x7e, 0x01, 0x00]) and len(f) == 260
    f = O.frame_write(bytes(65536), 2, False, frame_max=1 << 20)
    assert f[:10] == bytes([0x82, 0x7f, 0, 0, 0, 0, 0, 1, 0, 0]) and len(f) == 65546
    # permessage-deflate: RSV1 on the first frame only
    assert O.frame_write(_HELLO_DEFLATED, 1, True) == bytes([0xc1, 0x07]) + _HELLO_DEFLATED
    f = O.frame_write(_HELLO_DEFLATED, 1, True, frame_max=3)
    assert f == bytes([0x41, 0x03]) + _HELLO_DEFLATED[:3] + bytes([0x00, 0x03]) + _HELLO_DEFLATED[3:6] + \
        bytes([0x80, 0x01]) + _HELLO_DEFLATED[6:]
    assert O.frame_write(b"", 2, True) == bytes([0xc2, 0x00])


def test_frame_wire_size_matches_oracle():
    import torch
    L = pmd.lib()
    rng = random.Random(16)
    lens = [0, 1, 124, 125, 126, 127, 4095, 4096, 4097, 65535, 65536, 65537, 200000] + \
        [rng.randrange(0, 300000) for _ in range(40)]
    for fm in (1, 3, 125, 126, 4096, 65535, 65536, 1 << 20):
        for masked in (0, 1):
            want = [len(O.frame_write(bytes(n), 2, True, keys=[0] * (max(1, -(-n // fm))) if masked else None,
                                      frame_max=fm)) for n in lens] if fm >= 125 else None
            got = [L.bpmd_frame_wire_size(n, fm, masked) for n in lens]
            if want is not None:
                assert got == want, (fm, masked)
            t = pmd.frame_wire_sizes(torch.tensor(lens), fm, bool(masked)).tolist()
            assert t == got, (fm, masked)
