"""CPU check of the exact-mode deflate kernel's own logic (BPMD_F_EXACT,
beast_amd/csrc/pmd_deflate_exact.hip), compiled for the host by
tests/model/exact_host.py with one-lane meanings of the HIP intrinsics:
every payload must equal the oracle's (the restatement of Beast's
deflate_stream, itself byte-identical to the reference's zlib 1.3.1).  The
GPU build of the same code is checked in tests/test_gpu_deflate_exact.py."""
import pytest

from beast_amd import synth
from oracle import oracle as O
from tests.model import exact_host as X


def _msgs(kinds, sizes, seed):
    out = []
    for k in kinds:
        for s in sizes:
            d, _, _ = synth.make_batch(k, [s], seed=seed + 7 * s)
            out.append(bytes(d[:s]))
    return out


def _check(msgs, level, wbits=15, mem=4, strategy=0):
    for m in msgs:
        st, p = X.deflate(m, level, wbits, mem, strategy)
        assert st == 0 and p == O.pmd_deflate(m, level, wbits, mem, strategy), (len(m), level, wbits, mem, strategy)


@pytest.mark.parametrize("level", list(range(10)))
def test_levels(level):
    _check(_msgs(("json", "binary", "zeros"), (0, 1, 3, 17, 256, 1000, 4096, 5000), seed=level), level)


@pytest.mark.parametrize("mem,wbits", [(1, 9), (4, 12), (8, 15), (9, 9), (9, 15)])
def test_mem_window(mem, wbits):
    _check(_msgs(("json", "corpus1"), (0, 600, 3000, 9000), seed=mem + wbits), 6, wbits, mem)


@pytest.mark.parametrize("strategy", [1, 2, 3, 4])
def test_strategies(strategy):
    _check(_msgs(("json", "zeros"), (0, 5, 300, 4096), seed=strategy), 6, strategy=strategy)


def test_window_slide():
    _check(_msgs(("json", "binary"), (65536, 70000), seed=9), 6)
    _check(_msgs(("json",), (4000,), seed=3), 1, wbits=9)


def test_need_buffers_verdicts():
    import ctypes
    L = O.lib()
    for m in _msgs(("json", "random"), (0, 10, 500, 4096), seed=5):
        full = len(O.pmd_deflate(m, 6))
        for cap in sorted({0, 1, 5, 6, max(full - 3, 0), full, full + 1, full + 5, full + 6, full + 7}):
            buf = ctypes.create_string_buffer(max(cap, 1))
            z = L.bzo_deflate_new()
            L.bzo_deflate_reset_params(z, 6, 15, 4, 0)
            src = ctypes.create_string_buffer(m, len(m)) if m else None
            r = L.bzo_pmd_deflate_msg(z, src, len(m), buf, cap)
            L.bzo_deflate_free(z)
            st, p = X.deflate(m, 6, cap=cap)
            if r < 0:
                assert st == -r, (len(m), cap, r, st)
            else:
                assert st == 0 and p == buf.raw[:r], (len(m), cap, r, st)
