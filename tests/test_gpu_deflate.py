"""GPU deflate through the C ABI.

Contract (BASELINE.json north_star): every payload inflates
back to the message byte for byte -- checked with the CPU oracle (the
restatement of Beast's own inflate) and with the GPU inflater -- and the
compressed size stays within the stated tolerance of Beast's deflate at the
same level (oracle, byte-identical to Beast).  The kernel's output is also
checked byte for byte against the host model of its algorithm
(tests/model/deflate_model.cpp).
"""
import random

import numpy as np
import pytest

from beast_amd import synth
from oracle import oracle as O
from tests.model import model as M

pytestmark = pytest.mark.gpu

SIZE_TOLERANCE = 1.10   # Σ GPU payload bytes / Σ Beast payload bytes, same level, JSON-like text


def _deflate(msgs, level=6, wbits=15, strategy=0, out_cap=None):
    import torch
    from beast_amd import pmd
    src = pmd.Batch.from_host(msgs)
    cap = None if out_cap is None else torch.tensor(out_cap, dtype=torch.int32)
    res = pmd.deflate_batch(src, level=level, window_bits=wbits, strategy=strategy, out_cap=cap)
    torch.cuda.synchronize()
    return res.status.cpu().numpy(), res.out.to_host()


def _msgs(kinds, sizes, seed):
    out = []
    for k in kinds:
        for s in sizes:
            d, _, _ = synth.make_batch(k, [s], seed=seed + s)
            out.append(bytes(d[:s]))
    return out


def _check_roundtrip(msgs, payloads, status, wbits=15):
    for i, m in enumerate(msgs):
        assert int(status[i]) == 0, (i, int(status[i]))
        assert len(payloads[i]) <= O.upper_bound(len(m)), (i, len(payloads[i]), len(m))
        st, out = O.pmd_inflate(payloads[i], cap=max(len(m), 1), wbits=wbits)
        assert st == 0 and out == m, (i, O.ERRORS[st], len(out), len(m))


def _check_model(msgs, payloads, level, wbits=15, strategy=0):
    data = np.frombuffer(b"".join(msgs) or b"\0", dtype=np.uint8)
    lens = np.array([len(m) for m in msgs], dtype=np.uint32)
    off = np.zeros(len(msgs), dtype=np.uint64)
    off[1:] = np.cumsum(lens[:-1].astype(np.uint64))
    exp = M.encode(data, off, lens, level=level, wbits=wbits, strategy=strategy)
    bad = [i for i in range(len(msgs)) if exp[i] != payloads[i]]
    assert not bad, (len(bad), bad[:8])


@pytest.mark.parametrize("level", [0, 1, 2, 4, 6, 9])
def test_roundtrip_corpora(level):
    msgs = _msgs(("json", "corpus1", "random", "binary", "zeros"), (0, 1, 2, 3, 17, 255, 1024, 4095, 4096, 4097,
                                                                     9000, 70000), seed=level)
    st, pl = _deflate(msgs, level=level)
    _check_roundtrip(msgs, pl, st)
    _check_model(msgs, pl, level)


@pytest.mark.parametrize("strategy", [1, 2, 3, 4])
def test_roundtrip_strategies(strategy):
    msgs = _msgs(("json", "binary", "zeros"), (0, 7, 300, 4096, 20000), seed=100 + strategy)
    st, pl = _deflate(msgs, level=6, strategy=strategy)
    _check_roundtrip(msgs, pl, st)
    _check_model(msgs, pl, 6, strategy=strategy)
    if strategy == 2:   # huffman only: no back-references, so never smaller than the order-0 entropy
        assert all(len(p) > 0 for p in pl)


@pytest.mark.parametrize("wbits", [9, 10, 12, 15])
def test_window_bits_limit_distances(wbits):
    msgs = _msgs(("json", "corpus1"), (1000, 4096, 30000), seed=wbits)
    st, pl = _deflate(msgs, level=9, wbits=wbits)
    _check_roundtrip(msgs, pl, st, wbits=wbits)
    _check_model(msgs, pl, 9, wbits=wbits)


def test_empty_message_is_one_zero_byte():
    st, pl = _deflate([b""])
    assert int(st[0]) == 0 and pl[0] == O.pmd_deflate(b"", 6, 15, 4) == b"\x00"


def test_capacity_too_small_reports_need_buffers():
    msgs = _msgs(("random",), (4096, 10000), seed=5)
    st, pl = _deflate(msgs, out_cap=[100, 5000])
    assert list(st) == [1, 1] and pl == [b"", b""]


def test_random_mixture():
    rng = random.Random(7)
    msgs = []
    for _ in range(300):
        k = rng.choice(["json", "corpus1", "random", "binary", "zeros"])
        s = rng.choice([0, 1, 40, 700, 4096, 5000, 16384, 65536])
        d, _, _ = synth.make_batch(k, [s], seed=rng.randrange(1 << 30))
        msgs.append(bytes(d[:s]))
    for level in (1, 6):
        st, pl = _deflate(msgs, level=level)
        _check_roundtrip(msgs, pl, st)
        _check_model(msgs, pl, level)


@pytest.mark.parametrize("level", [1, 6])
def test_minimum_gain_chunk_choice_equals_model(level):
    """lz::chunk_stored: chunks of long messages that save under 1/16 are stored,
    one-chunk messages keep Beast's rule; the kernel makes the host model's
    choice on data either side of the threshold (tests/test_model.py)."""
    from tests.test_model import _slightly_compressible
    msgs = []
    for seed, frac in ((3, 1 / 16), (4, 1 / 8), (5, 1 / 4), (6, 1 / 32)):
        d = _slightly_compressible(65536, seed, frac).tobytes()
        msgs += [d, d[:4096], d[:9000]]
    st, pl = _deflate(msgs, level=level)
    _check_roundtrip(msgs, pl, st)
    _check_model(msgs, pl, level)


@pytest.mark.parametrize("level", [1, 6, 9])
def test_size_tolerance_vs_beast(level):
    n = 2048
    lens = np.full(n, 4096, dtype=np.uint32)
    data, off, ln = synth.make_batch("json", lens, seed=0x5EED0003)
    msgs = [bytes(data[int(off[i]):int(off[i]) + 4096]) for i in range(n)]
    st, pl = _deflate(msgs, level=level)
    assert int((st != 0).sum()) == 0
    ours = sum(len(p) for p in pl)
    beast = sum(len(O.pmd_deflate(m, level, 15, 4)) for m in msgs)
    assert ours <= SIZE_TOLERANCE * beast, (ours, beast, ours / beast)


def test_gpu_inflate_of_gpu_deflate_full_batch():
    """C3 shape: 64 Ki x 4 KiB JSON, deflate then inflate on the device."""
    import torch
    from beast_amd import pmd
    n = 1 << 16
    lens = np.full(n, 4096, dtype=np.uint32)
    data, off, ln = synth.make_batch("json", lens, seed=0x5EED0003)
    src = pmd.Batch.from_arrays(data, off.astype(np.int64), ln.astype(np.int32))
    d = pmd.deflate_batch(src, level=6)
    assert int((d.status != 0).sum()) == 0
    comp = pmd.Batch(d.out.data, d.out.off, d.out.len)
    r = pmd.inflate_batch(comp, 4096)
    torch.cuda.synchronize()
    assert int((r.status != 0).sum()) == 0
    assert torch.equal(r.out.data[: n * 4096].view(n, 4096), src.data[: n * 4096].view(n, 4096))
