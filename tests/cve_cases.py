"""CVE-2018-25032 pins (test/beast/zlib/deflate_stream.cpp:610-636): a
deflate_stream at memLevel 1 with Strategy::fixed / normal, one
write(Flush::finish) into deflate_upper_bound bytes must return
end_of_stream without overflowing.  Inputs: tests/golden/cve_2018_25032.json
(generator: tests/golden/make_cve_2018_25032.py)."""
import ctypes
import json
import os

from oracle import oracle as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def cases():
    with open(os.path.join(GOLD, "cve_2018_25032.json")) as f:
        d = json.load(f)
    return [(name, d[name].encode("ascii"), level, O.STRATEGY[strat]) for name, level, strat in d["cases"]]


def finish_once(deflater, data: bytes):
    """testCVE's single write: returns (status, output bytes)."""
    n = O.upper_bound(len(data))
    src = ctypes.create_string_buffer(data, len(data))
    out = ctypes.create_string_buffer(n)
    zs = O.ZParams(ctypes.addressof(src), len(data), 0, ctypes.addressof(out), n, 0, 0)
    st = deflater.write(zs, "finish")
    return st, out.raw[:zs.total_out], zs.total_in
