"""GPU parity of the HIP inflate path against the CPU oracle (bit-exact bytes,
lengths and zlib::error statuses), through the C ABI."""
import json
import os
import random

import numpy as np
import pytest

from beast_amd import synth
from oracle import oracle as O
from tests.foreign import foreign_payloads

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(autouse=True, params=["lane", "wave", "wave_walk", "wave_spec", "bp"])
def inflate_kernel(request):
    """Every inflate test runs on both kernels (pmd_inflate_lane3.hip and
    pmd_inflate.hip), forced through bpmd_set_inflate_kernel; the wave kernel
    also with every round a walk round and with speculative rounds only
    (bpmd_diag_set_wave_walk); and block-parallel (pmd_inflate_bp.hip: every
    payload of 64 bytes or more cut at its dynamic-block headers)."""
    pmd = _pmd()
    mode = {"lane": 1, "wave": 2, "wave_walk": 2, "wave_spec": 2, "bp": 3}[request.param]
    walk = {"wave_walk": 1, "wave_spec": 2}.get(request.param, 0)
    assert pmd.lib().bpmd_set_inflate_kernel(mode) == 0
    assert pmd.lib().bpmd_diag_set_wave_walk(walk) == 0
    yield request.param
    pmd.lib().bpmd_set_inflate_kernel(0)
    pmd.lib().bpmd_diag_set_wave_walk(0)


def _pmd():
    import torch  # noqa: F401
    from beast_amd import pmd
    return pmd


def _gpu_inflate(payloads, cap, raw=False, wbits=15):
    pmd = _pmd()
    src = pmd.Batch.from_host(payloads)
    caps = cap if isinstance(cap, int) else __import__("torch").tensor(cap, dtype=__import__("torch").int32)
    res = pmd.inflate_batch(src, caps, window_bits=wbits, raw=raw)
    __import__("torch").cuda.synchronize()
    st = res.status.cpu().numpy()
    outs = res.out.to_host()
    return st, outs


def _check_against_oracle(payloads, caps, raw=False, wbits=15):
    st, outs = _gpu_inflate(payloads, caps, raw=raw, wbits=wbits)
    for i, p in enumerate(payloads):
        cap = caps if isinstance(caps, int) else caps[i]
        est, eout = O.pmd_inflate(p, cap=cap, raw=raw, wbits=wbits)
        assert int(st[i]) == est, (i, O.ERRORS[int(st[i])], O.ERRORS[est], len(p))
        assert outs[i] == eout, (i, len(outs[i]), len(eout))


def test_known_answer_vectors_raw():
    with open(os.path.join(GOLD, "inflate_kat.json")) as f:
        kat = json.load(f)
    payloads, expect = [], []
    for v in kat["vectors"]:
        d = bytes.fromhex(v["in"])
        if "prefix" in v:
            d = d[:v["prefix"]]
        payloads.append(d)
        expect.append(v["expect"])
    st, _ = _gpu_inflate(payloads, 1024, raw=True)
    got = [O.ERRORS[int(s)] for s in st]
    assert got == expect
    k = kat["flush_trees"]
    st, outs = _gpu_inflate([bytes.fromhex(k["fixed"]), bytes.fromhex(k["stored"])], 5, raw=True)
    assert list(st) == [0, 0] and outs == [b"Hello", b"Hello"]


@pytest.mark.parametrize("level", [1, 6, 9])
@pytest.mark.parametrize("mem", [4, 8])
def test_parity_corpora(level, mem):
    payloads, caps = [], []
    for kind in ("json", "corpus1", "random", "binary", "zeros"):
        for size in (0, 1, 17, 255, 1024, 4096, 9000, 70000):
            data, _, _ = synth.make_batch(kind, [size], seed=level * 100 + mem + size)
            payloads.append(O.pmd_deflate(bytes(data[:size]), level, 15, mem))
            caps.append(max(size, 1))
    _check_against_oracle(payloads, caps)


def test_parity_levels_strategies_windows():
    payloads, caps = [], []
    rng = random.Random(1)
    for _ in range(120):
        kind = rng.choice(["json", "corpus1", "random", "binary", "zeros"])
        size = rng.choice([0, 5, 300, 4096, 12000, 40000])
        data, _, _ = synth.make_batch(kind, [size], seed=rng.randrange(1 << 30))
        lvl, wb, mem, st = rng.randrange(0, 10), rng.randrange(9, 16), rng.randrange(1, 10), rng.randrange(5)
        payloads.append(O.pmd_deflate(bytes(data[:size]), lvl, wb, mem, st))
        caps.append(max(size, 1))
    _check_against_oracle(payloads, caps)


def test_capacity_overflow_and_exact_fit():
    data, _, _ = synth.make_batch("json", [20000], seed=5)
    p = O.pmd_deflate(bytes(data), 6, 15, 4)
    caps = [1, 100, 4095, 4096, 8191, 8192, 8193, 19999, 20000, 20001]
    _check_against_oracle([p] * len(caps), caps)


def test_corrupted_and_truncated_payloads():
    rng = random.Random(7)
    base = []
    for kind in ("json", "corpus1", "binary"):
        data, _, _ = synth.make_batch(kind, [6000], seed=rng.randrange(1000))
        base.append(O.pmd_deflate(bytes(data), rng.choice([1, 6, 9]), 15, 4))
    payloads = []
    for _ in range(400):
        q = bytearray(rng.choice(base))
        op = rng.randrange(3)
        if op == 0:
            for _ in range(rng.randrange(1, 5)):
                q[rng.randrange(len(q))] ^= 1 << rng.randrange(8)
        elif op == 1:
            q = q[:rng.randrange(len(q))]
        else:
            q = bytearray(rng.randbytes(rng.randrange(1, 200)))
        payloads.append(bytes(q))
    _check_against_oracle(payloads, 7000)
    _check_against_oracle(payloads, 7000, raw=True)


def test_bfinal_inside_message_is_end_of_stream():
    # read3.cpp:529-610: a BFINAL block inside a message fails with end_of_stream
    import zlib
    c = zlib.compressobj(6, zlib.DEFLATED, -15)
    final = c.compress(b"hello hello hello") + c.flush(zlib.Z_FINISH)
    _check_against_oracle([final, final + b"\x01\x02"], 100)


def test_full_batch_roundtrip_property():
    """64 Ki x 4 KiB JSON (the C2 shape): GPU output == original input."""
    import torch
    pmd = _pmd()
    n = 1 << 16
    lens = np.full(n, 4096, dtype=np.uint32)
    data, off, lens = synth.make_batch("json", lens, seed=0x5EED0002)
    comp, coff, clen, cst = O.deflate_batch(data, off, lens, level=6, wbits=15, mem_level=4, threads=16)
    assert (cst == 0).all()
    src = pmd.Batch.from_arrays(comp, coff.astype(np.int64), clen.astype(np.int32))
    res = pmd.inflate_batch(src, 4096)
    torch.cuda.synchronize()
    assert int((res.status != 0).sum()) == 0
    assert int((res.out.len != 4096).sum()) == 0
    got = res.out.data[: n * 4096].view(n, 4096)
    want = torch.from_numpy(data.reshape(n, 4096)).cuda()
    assert torch.equal(got, want)


def test_parity_foreign_encoder_flush_mixes():
    """CPython zlib payloads with mid-payload flushes of every kind, in both
    framings, at exact, generous and short capacities, against the oracle
    (the oracle itself is pinned on the same payloads against CPython's
    inflate in tests/test_oracle_foreign.py)."""
    pmd_p, raw_p, orig = foreign_payloads(11, 160)
    rng = random.Random(12)
    caps = [max(1, rng.choice([len(o), len(o) + 77, len(o) // 2 + 1])) for o in orig]
    _check_against_oracle(pmd_p, caps)
    _check_against_oracle(raw_p, caps, raw=True)
