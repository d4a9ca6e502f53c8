"""The oracle's inflate on payloads from another encoder (CPython's zlib):
every flush kind mid-payload, zlib's strategies, memLevels and windows, in
both framings, checked against CPython's own inflate (CPU only; the GPU
kernels are checked against the oracle on the same payloads in
tests/test_gpu_inflate.py::test_parity_foreign_encoder_flush_mixes)."""
import zlib

from oracle import oracle as O
from tests.foreign import foreign_payloads


def test_oracle_inflate_matches_cpython_on_foreign_payloads():
    pmd_p, raw_p, orig = foreign_payloads(11, 160)
    for i, (p, r, o) in enumerate(zip(pmd_p, raw_p, orig)):
        cap = max(1, len(o))
        st, out = O.pmd_inflate(p, cap=cap)
        assert out == o, (i, len(out), len(o))
        assert O.ERRORS[st] in ("ok", "need_buffers"), (i, O.ERRORS[st])
        d = zlib.decompressobj(-15)
        assert d.decompress(p + b"\x00\x00\xff\xff") == o
        st, out = O.pmd_inflate(r, cap=cap + 16, raw=True)
        assert out == o, (i, "raw", len(out), len(o))
