"""Exact mode of the batch deflater (BPMD_F_EXACT):
every payload must equal, byte for byte, the one Beast's deflate_stream
produces under impl_base's call sequence -- here the oracle's restatement,
which is itself byte-identical to the reference's zlib 1.3.1
(tests/test_oracle.py) -- for every level, memLevel, windowBits and strategy,
including empty, tiny, window-sliding and incompressible messages, and the
need_buffers verdict of a slot that is too small."""
import ctypes

import numpy as np
import pytest

from beast_amd import synth
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _msgs(kinds, sizes, seed):
    out = []
    for k in kinds:
        for s in sizes:
            d, _, _ = synth.make_batch(k, [s], seed=seed + 7 * s)
            out.append(bytes(d[:s]))
    return out


def _gpu(msgs, level, wbits=15, mem=4, strategy=0, out_cap=None, key=None):
    import torch
    from beast_amd import pmd
    src = pmd.Batch.from_host(msgs)
    if key is None:
        res = pmd.deflate_batch(src, level=level, window_bits=wbits, mem_level=mem, strategy=strategy,
                                out_cap=out_cap, exact=True)
    else:
        res = pmd.write_batch(src, key=key, level=level, window_bits=wbits, mem_level=mem, strategy=strategy,
                              out_cap=out_cap, exact=True)
    torch.cuda.synchronize()
    return [int(x) for x in res.status.cpu().numpy()], res.out.to_host()


def _check(msgs, level, wbits=15, mem=4, strategy=0):
    st, pl = _gpu(msgs, level, wbits, mem, strategy)
    bad = []
    for i, m in enumerate(msgs):
        exp = O.pmd_deflate(m, level, wbits, mem, strategy)
        if st[i] != 0 or pl[i] != exp:
            bad.append((i, len(m), st[i], len(pl[i]), len(exp)))
    assert not bad, bad[:6]


SIZES = (0, 1, 2, 3, 4, 17, 255, 256, 1000, 4096, 5000)


@pytest.mark.parametrize("level", list(range(10)))
def test_levels_json_and_binary(level):
    _check(_msgs(("json", "binary", "zeros"), SIZES, seed=level), level)


@pytest.mark.parametrize("mem", [1, 4, 8, 9])
@pytest.mark.parametrize("wbits", [9, 12, 15])
def test_mem_and_window(mem, wbits):
    _check(_msgs(("json", "corpus1"), (0, 3, 600, 3000, 9000), seed=mem * 16 + wbits), 6, wbits, mem)


@pytest.mark.parametrize("strategy", [1, 2, 3, 4])
@pytest.mark.parametrize("level", [1, 6])
def test_strategies(strategy, level):
    _check(_msgs(("json", "binary", "zeros"), (0, 5, 300, 4096, 7000), seed=40 + strategy), level, strategy=strategy)


@pytest.mark.parametrize("level", [1, 6, 9])
def test_window_slides_and_long_messages(level):
    # past 2 * 2^windowBits - 262 bytes the reference slides its window, and
    # near the end its comparisons read the bytes the slide left behind
    msgs = _msgs(("json", "binary"), (20000, 65536, 70000), seed=90 + level)
    _check(msgs, level, 15)
    _check(_msgs(("json",), (1500, 4000), seed=3), level, 9)


def test_c3_sample_exact():
    lens = np.full(512, 4096, dtype=np.uint32)
    d, off, ln = synth.make_batch("json", lens, seed=0x5EED0003)
    msgs = [bytes(d[int(off[i]):int(off[i]) + 4096]) for i in range(512)]
    _check(msgs, 6)


def test_need_buffers_matches_reference():
    L = O.lib()
    msgs = _msgs(("json", "random"), (0, 10, 500, 4096), seed=5)
    for m in msgs:
        full = len(O.pmd_deflate(m, 6))
        for cap in sorted({0, 1, 5, 6, max(full - 3, 0), full, full + 1, full + 5, full + 6, full + 7}):
            buf = ctypes.create_string_buffer(max(cap, 1))
            z = L.bzo_deflate_new()
            L.bzo_deflate_reset_params(z, 6, 15, 4, 0)
            src = ctypes.create_string_buffer(m, len(m)) if m else None
            r = L.bzo_pmd_deflate_msg(z, src, len(m), buf, cap)
            L.bzo_deflate_free(z)
            st, pl = _gpu([m], 6, out_cap=cap)
            if r < 0:
                assert st[0] == -r, (len(m), cap, r, st[0])
            else:
                assert st[0] == 0 and pl[0] == buf.raw[:r], (len(m), cap, r, st[0])


def test_client_mask_applied():
    msgs = _msgs(("json",), (0, 9, 700, 4096), seed=11)
    keys = [0x11223344, 0xdeadbeef, 0x01020304, 0xffffffff]
    st, pl = _gpu(msgs, 6, key=keys)
    for i, m in enumerate(msgs):
        exp = O.pmd_deflate(m, 6)
        k = keys[i].to_bytes(4, "little")
        assert st[i] == 0 and pl[i] == bytes(b ^ k[j & 3] for j, b in enumerate(exp)), i
