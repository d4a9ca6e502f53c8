"""CPU tests of the oracle (the parity checker) against the reference's own
vectors: zlib 1.3.1 golden payloads and Beast's inflate known-answer tests."""
import hashlib
import json
import os
import random
import zlib

import numpy as np
import pytest

from beast_amd import synth
from oracle import oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _kat():
    with open(os.path.join(GOLD, "inflate_kat.json")) as f:
        return json.load(f)


def test_deflate_matches_reference_zlib_golden():
    with open(os.path.join(GOLD, "deflate_golden.json")) as f:
        doc = json.load(f)
    cache = {}
    for e in doc["entries"]:
        key = (e["kind"], e["seed"], e["size"])
        if key not in cache:
            data, _, _ = synth.make_batch(e["kind"], [e["size"]], seed=e["seed"])
            cache[key] = bytes(data[:e["size"]])
        msg = cache[key]
        assert hashlib.sha256(msg).hexdigest() == e["in_sha256"], "synthetic generator drifted"
        out = O.pmd_deflate(msg, e["level"], e["wbits"], e["mem"], e["strategy"])
        assert len(out) == e["out_len"] and hashlib.sha256(out).hexdigest() == e["out_sha256"], e
        if "out_hex" in e:
            assert out.hex() == e["out_hex"]
        st, back = O.pmd_inflate(out, cap=max(e["size"], 1))
        assert st == 0 and back == msg


@pytest.mark.parametrize("i", range(19))
def test_inflate_known_answers(i):
    v = _kat()["vectors"][i]
    data = bytes.fromhex(v["in"])
    if "prefix" in v:
        data = data[:v["prefix"]]
    st, _ = O.pmd_inflate(data, cap=1024, wbits=v["wbits"], raw=True)
    assert O.ERRORS[st] == v["expect"]


def test_flush_trees_vectors_decode_hello():
    k = _kat()["flush_trees"]
    for key in ("fixed", "stored"):
        st, out = O.pmd_inflate(bytes.fromhex(k[key]), cap=5, raw=True)
        assert st == 0 and out == bytes.fromhex(k["expect_out"])


def test_empty_message_is_single_zero_byte():
    # impl_base.hpp:124-148: Flush::block then Flush::sync on no input
    assert O.pmd_deflate(b"", 8, 15, 4) == b"\x00"
    st, out = O.pmd_inflate(b"\x00", cap=16)
    assert st == 0 and out == b""


@pytest.mark.parametrize("level", range(10))
def test_roundtrip_every_level(level):
    for kind in ("json", "corpus1", "random", "binary", "zeros"):
        for size in (0, 3, 1000, 5000, 70000):
            data, _, _ = synth.make_batch(kind, [size], seed=11)
            msg = bytes(data[:size])
            for mem in (1, 4, 9):
                p = O.pmd_deflate(msg, level, 15, mem)
                st, back = O.pmd_inflate(p, cap=max(size, 1))
                assert st == 0 and back == msg, (kind, size, level, mem)


def test_python_zlib_agrees_at_pmd_defaults():
    """Independent check: the system zlib equals the oracle at L1/L6/L9, mem 4."""
    data, _, _ = synth.make_batch("json", [20000], seed=3)
    msg = bytes(data)
    for lvl in (1, 6, 9):
        c = zlib.compressobj(lvl, zlib.DEFLATED, -15, 4)
        py = c.compress(msg) + c.flush(zlib.Z_BLOCK) + c.flush(zlib.Z_SYNC_FLUSH)
        assert O.pmd_deflate(msg, lvl, 15, 4) == py[:-4]


# a path check, not O.ref(): collecting this module (also under -m gpu) must
# not map the reference's compiled zlib into the process
_REF_SO = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "_ref", "libzref.so")


@pytest.mark.skipif(not os.path.exists(_REF_SO), reason="reference zlib not built here")
def test_random_configs_against_reference_zlib():
    rng = random.Random(5)
    for _ in range(150):
        kind = rng.choice(["json", "corpus1", "random", "binary"])
        size = rng.choice([0, 1, 2, 3, 10, 100, 259, 262, 1023, 4096, 33000, 70000])
        data, _, _ = synth.make_batch(kind, [size], seed=rng.randrange(1 << 30))
        msg = bytes(data[:size])
        lvl, wb, mem, st = rng.randrange(1, 10), rng.randrange(9, 16), rng.randrange(1, 10), rng.randrange(5)
        assert O.pmd_deflate(msg, lvl, wb, mem, st) == O.ref_pmd_deflate(msg, lvl, wb, mem, st)


def test_corrupt_streams_do_not_crash_and_match_python_on_valid_prefix():
    rng = random.Random(9)
    data, _, _ = synth.make_batch("json", [3000], seed=1)
    p = bytearray(O.pmd_deflate(bytes(data), 6, 15, 4))
    for _ in range(300):
        q = bytearray(p)
        for _ in range(rng.randrange(1, 4)):
            q[rng.randrange(len(q))] ^= 1 << rng.randrange(8)
        st, out = O.pmd_inflate(bytes(q), cap=4096)
        assert 0 <= st <= 16
        d = zlib.decompressobj(-15)
        try:
            ref = d.decompress(bytes(q) + b"\x00\x00\xff\xff", 4096)
            ok = True
        except zlib.error:
            ok = False
        if st == 0 and ok:
            assert out == ref[:len(out)]


def test_batch_threads_match_single():
    lens = np.array([100, 4096, 0, 7000, 1], dtype=np.uint32)
    data, off, lens = synth.make_batch("json", lens, seed=2)
    a = O.deflate_batch(data, off, lens, threads=1)
    b = O.deflate_batch(data, off, lens, threads=3)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    out, out_off, out_len, status = a
    assert (status == 0).all()
    inf = O.inflate_batch(out, out_off, out_len, lens.astype(np.uint32) + 1, threads=2)
    for i in range(len(lens)):
        o = int(inf[1][i])
        assert bytes(inf[0][o:o + inf[2][i]]) == bytes(data[int(off[i]):int(off[i]) + int(lens[i])])


def test_capacity_overflow_reports_need_buffers():
    data, _, _ = synth.make_batch("json", [5000], seed=4)
    p = O.pmd_deflate(bytes(data), 6, 15, 4)
    st, out = O.pmd_inflate(p, cap=4999)
    assert st == 1 and out == bytes(data[:4999])
    st, out = O.pmd_inflate(p, cap=5000)
    assert st == 0 and out == bytes(data)
