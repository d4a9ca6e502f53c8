"""CPU: the host model of the GPU deflate algorithm (tests/model) produces
payloads that Beast's inflate (oracle restatement) decodes back to the
message, within the size tolerance the GPU tests apply.  This pins the
algorithm the kernel is compared against byte for byte."""
import numpy as np
import pytest

from beast_amd import synth
from oracle import oracle as O
from tests.model import model as M


def _run(kind, sizes, level=6, wbits=15, strategy=0, seed=1):
    lens = np.array(sizes, dtype=np.uint32)
    data, off, ln = synth.make_batch(kind, lens, seed=seed)
    pl = M.encode(data, off, ln, level=level, wbits=wbits, strategy=strategy)
    msgs = [bytes(data[int(off[i]):int(off[i]) + int(ln[i])]) for i in range(len(sizes))]
    for i, m in enumerate(msgs):
        st, out = O.pmd_inflate(pl[i], cap=max(len(m), 1), wbits=wbits)
        assert st == 0 and out == m, (kind, sizes[i], level, strategy, O.ERRORS[st])
        assert len(pl[i]) <= O.upper_bound(len(m))
    return msgs, pl


@pytest.mark.parametrize("level", range(10))
def test_model_roundtrip_levels(level):
    for kind in ("json", "corpus1", "random", "binary", "zeros"):
        _run(kind, [0, 1, 3, 100, 4096, 4097, 20000], level=level, seed=level)


@pytest.mark.parametrize("strategy", range(5))
def test_model_roundtrip_strategies(strategy):
    for kind in ("json", "binary", "zeros"):
        _run(kind, [0, 2, 300, 4096, 9000], strategy=strategy, seed=strategy)


@pytest.mark.parametrize("wbits", [8, 9, 12, 15])
def test_model_roundtrip_window_bits(wbits):
    _run("json", [5000, 30000], level=9, wbits=wbits)


def test_model_size_within_tolerance_of_beast():
    msgs, pl = _run("json", [4096] * 256, level=6, seed=0x5EED0003)
    ours = sum(len(p) for p in pl)
    beast = sum(len(O.pmd_deflate(m, 6, 15, 4)) for m in msgs)
    assert ours <= 1.10 * beast, ours / beast


def test_runwise_code_length_coding_equals_serial_state_machine():
    """The kernel codes code-length runs independently (lz::rle_run); it must
    reproduce the reference's scan_tree/send_tree state machine
    (deflate_stream.ipp:978-1110) symbol for symbol."""
    import ctypes
    import random
    L = M.lib()
    rng = random.Random(3)
    out1 = (ctypes.c_uint32 * 400)()
    out2 = (ctypes.c_uint32 * 400)()
    na, nb = ctypes.c_int(), ctypes.c_int()
    for trial in range(3000):
        n = rng.randrange(1, 320)
        mode = trial % 3
        if mode == 0:
            lens = [rng.choice([0, 0, 0, 5, 6, 7, 8]) for _ in range(n)]
        elif mode == 1:
            lens = []
            while len(lens) < n:
                lens += [rng.randrange(0, 16)] * rng.randrange(1, 160)
            lens = lens[:n]
        else:
            lens = [rng.randrange(0, 16) for _ in range(n)]
        buf = (ctypes.c_uint8 * n)(*lens)
        ok = L.dmodel_rle_check(buf, n, out1, out2, ctypes.byref(na), ctypes.byref(nb))
        assert ok == 1, (lens, na.value, nb.value)


def _slightly_compressible(n, seed, frac):
    # random bytes; a fraction of the 64-byte units copies 16-47 bytes from up
    # to 1.5 KiB back (inside a chunk's 2 KiB history), like C5's binary kind
    rng = np.random.default_rng(seed)
    d = rng.integers(0, 256, n, dtype=np.uint8)
    for p in range(64, n, 64):
        if rng.random() < frac:
            span = int(rng.integers(16, 48))
            back = int(rng.integers(span, min(p, 1500) + 1))
            d[p:p + span] = d[p - back:p - back + span]
    return d


def test_minimum_gain_for_chunks_of_long_messages():
    """lz::chunk_stored (lz_core.h, BPMD_MIN_GAIN_SHIFT 4): a Huffman chunk of a
    multi-chunk message must save 1/16 of its bytes, else it is stored; a
    one-chunk message keeps Beast's rule (tr_flush_block,
    deflate_stream.ipp:1478: any saving keeps the Huffman block)."""
    data = _slightly_compressible(16384, 3, 1 / 16)
    (multi,) = M.encode(data, [0], [16384], level=1)
    st, out = O.pmd_inflate(multi, cap=16384)
    assert st == 0 and out == data.tobytes()
    assert len(multi) >= 16384   # every chunk saved < 256 bytes: all stored
    single = [M.encode(data[i * 4096:(i + 1) * 4096], [0], [4096], level=1)[0] for i in range(4)]
    assert sum(len(s) < 4096 for s in single) >= 2   # the same chunks alone: Huffman blocks
    # chunks that save more than 1/16 keep their Huffman blocks
    data = _slightly_compressible(16384, 3, 1 / 4)
    (multi,) = M.encode(data, [0], [16384], level=1)
    st, out = O.pmd_inflate(multi, cap=16384)
    assert st == 0 and out == data.tobytes()
    assert len(multi) < 16384 * 15 // 16 + 64
