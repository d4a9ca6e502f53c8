"""GPU checks against data the reference itself holds:

* CVE-2018-25032 (test/beast/zlib/deflate_stream.cpp:610-636): the
  per-stream deflate_stream at memLevel 1, Strategy::fixed / normal, one
  write(Flush::finish) into deflate_upper_bound bytes returns end_of_stream;
  the batch deflater stays within the bound and round-trips; exact mode
  equals the oracle (Beast's deflate restated) on the same inputs;
* the golden manifest tests/golden/deflate_golden.json -- payloads of the
  reference's vendored zlib 1.3.1 under impl_base's call pattern, made by
  tests/golden/make_golden.py -- read directly: exact mode must reproduce
  every entry's length and sha256 (and its bytes where stored)."""
import ctypes
import hashlib
import json
import os
import zlib

import numpy as np
import pytest

from beast_amd import synth
from oracle import oracle as O
from tests import cve_cases as C

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _gpu_deflate_stream(data, level, mem, strategy):
    from beast_amd import pmd
    L = pmd.lib()
    vp = ctypes.c_void_p
    L.bpmd_deflate_stream_create.argtypes = [ctypes.c_int] * 4 + [ctypes.POINTER(vp)]
    L.bpmd_deflate_stream_write.argtypes = [vp, ctypes.POINTER(O.ZParams), ctypes.c_int]
    L.bpmd_stream_destroy.argtypes = [vp]
    h = vp()
    assert L.bpmd_deflate_stream_create(level, 15, mem, strategy, ctypes.byref(h)) == 0
    try:
        class W:
            def write(self, zs, flush):
                return L.bpmd_deflate_stream_write(h, ctypes.byref(zs), O.FLUSH[flush])
        return C.finish_once(W(), data)
    finally:
        L.bpmd_stream_destroy(h)


@pytest.mark.parametrize("name,data,level,strategy", C.cases(), ids=lambda v: str(v)[:12])
def test_cve_2018_25032_deflate_stream(name, data, level, strategy):
    st, out, used = _gpu_deflate_stream(data, level, 1, strategy)
    assert O.ERRORS[st] == "end_of_stream" and used == len(data)
    assert len(out) <= O.upper_bound(len(data))
    assert zlib.decompress(out, -15) == data


def _batch(msgs, level, mem, strategy, exact):
    import torch
    from beast_amd import pmd
    res = pmd.deflate_batch(pmd.Batch.from_host(msgs), level=level, window_bits=15, mem_level=mem,
                            strategy=strategy, exact=exact)
    torch.cuda.synchronize()
    return [int(x) for x in res.status.cpu().numpy()], res.out.to_host()


@pytest.mark.parametrize("exact", [False, True])
def test_cve_2018_25032_batch(exact):
    for name, data, level, strategy in C.cases():
        st, pl = _batch([data, data[:4096], data[-777:]], level, 1, strategy, exact)
        for i, m in enumerate([data, data[:4096], data[-777:]]):
            assert st[i] == 0 and len(pl[i]) <= O.upper_bound(len(m)), (name, level, strategy, i)
            assert O.pmd_inflate(pl[i], cap=len(m) + 16) == (0, m)
            if exact:
                assert pl[i] == O.pmd_deflate(m, level, 15, 1, strategy), (name, level, strategy, i)


def test_exact_mode_reproduces_golden_manifest():
    with open(os.path.join(GOLD, "deflate_golden.json")) as f:
        entries = json.load(f)["entries"]
    groups = {}
    for e in entries:
        groups.setdefault((e["level"], e["wbits"], e["mem"], e["strategy"]), []).append(e)
    import torch
    from beast_amd import pmd
    checked = 0
    for (level, wbits, mem, strat), es in groups.items():
        msgs = []
        for e in es:
            data, _, _ = synth.make_batch(e["kind"], [e["size"]], seed=e["seed"])
            m = bytes(data[:e["size"]])
            assert hashlib.sha256(m).hexdigest() == e["in_sha256"], e
            msgs.append(m)
        res = pmd.deflate_batch(pmd.Batch.from_host(msgs), level=level, window_bits=wbits, mem_level=mem,
                                strategy=strat, exact=True)
        torch.cuda.synchronize()
        st = res.status.cpu().numpy()
        outs = res.out.to_host()
        for e, s, p in zip(es, st, outs):
            assert int(s) == 0 and len(p) == e["out_len"], (e["kind"], e["size"], level, wbits, mem, strat)
            assert hashlib.sha256(p).hexdigest() == e["out_sha256"], (e["kind"], e["size"], level, wbits, mem, strat)
            if "out_hex" in e:
                assert p.hex() == e["out_hex"]
            checked += 1
    assert checked == len(entries) == 336
