"""The oracle's deflate_stream on the reference's CVE-2018-25032 inputs
(deflate_stream.cpp:610-636): end_of_stream within deflate_upper_bound, the
stream inflates back to the input, and the bytes equal the reference's
vendored zlib 1.3.1 (Z_FINISH, same level / memLevel / strategy) when it is
built.  The GPU paths are checked in tests/test_gpu_reference_pins.py."""
import zlib

import pytest

from oracle import oracle as O
from tests import cve_cases as C


@pytest.mark.parametrize("name,data,level,strategy", C.cases(), ids=lambda v: str(v)[:12])
def test_oracle_finishes_within_upper_bound(name, data, level, strategy):
    assert len(data) == 32768
    st, out, used = C.finish_once(O.Deflater(level, 15, 1, strategy), data)
    assert O.ERRORS[st] == "end_of_stream" and used == len(data)
    assert len(out) <= O.upper_bound(len(data))
    # (a Beast inflater would need bytes past the final EOB to see it: its
    # slow path asks for lenbits_ bits first, inflate_stream.ipp:374-375)
    assert zlib.decompress(out, -15) == data
    if O.ref() is not None:
        assert out == O.ref_pmd_deflate(data, level, 15, 1, strategy, mode=2)
