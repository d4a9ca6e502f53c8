"""GPU: the wave-cooperative decode-table builder equals the serial
restatement of the reference's inflate_table (inflate_stream.ipp:551-863)
slot for slot, including roots, sizes and error codes."""
import ctypes
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

KENOUGH = 852 + 592


def _random_complete(n_sym, rng, maxlen=15, nz=None):
    """Code lengths of a random complete prefix code over a random subset."""
    k = nz if nz is not None else rng.randrange(2, n_sym + 1)
    leaves = [0]
    while len(leaves) < k:
        cands = [i for i, d in enumerate(leaves) if d < maxlen]
        i = rng.choice(cands)
        d = leaves.pop(i)
        leaves += [d + 1, d + 1]
    syms = rng.sample(range(n_sym), k)
    lens = [0] * n_sym
    for s, d in zip(syms, leaves):
        lens[s] = d
    return lens


def _cases():
    rng = random.Random(42)
    cases = []
    for _ in range(300):
        t = rng.choice([0, 1, 2])
        n = {0: 19, 1: rng.randrange(257, 287), 2: rng.randrange(1, 31)}[t]
        mode = rng.random()
        maxlen = 7 if t == 0 else 15
        if mode < 0.6 and n >= 2:
            lens = _random_complete(n, rng, maxlen)
        elif mode < 0.7:
            lens = [0] * n
            lens[rng.randrange(n)] = 1          # single 1-bit code (accepted for lens/dists)
        elif mode < 0.75:
            lens = [0] * n                      # empty code
        else:
            lens = [rng.choice([0, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15][:maxlen + 3])
                    for _ in range(n)]          # arbitrary: over-subscribed / incomplete
        if t == 1 and mode < 0.6:
            lens[256] = lens[256] or 1 if sum(1 for x in lens if x) < 2 else lens[256]
        cases.append((t, n, lens))
    # deep codes that force many sub-tables
    for nz in (40, 120, 286):
        lens = _random_complete(286, rng, 15, nz=nz)
        cases.append((1, 286, lens))
    return cases


def test_wave_builder_matches_serial_builder():
    import torch
    from beast_amd import pmd
    L = pmd.lib()
    cases = _cases()
    n = len(cases)
    lens = np.zeros((n, 320), dtype=np.uint8)
    ns = np.zeros(n, dtype=np.uint32)
    ts = np.zeros(n, dtype=np.int32)
    for i, (t, k, l) in enumerate(cases):
        lens[i, :k] = l
        ns[i] = k
        ts[i] = t
    d_lens = torch.from_numpy(lens).cuda()
    d_n = torch.from_numpy(ns).cuda()
    d_t = torch.from_numpy(ts).cuda()
    wave = torch.empty(n * KENOUGH, dtype=torch.int16, device="cuda")
    serial = torch.empty(n * KENOUGH, dtype=torch.int16, device="cuda")
    meta = torch.empty(n * 8, dtype=torch.int32, device="cuda")
    vp = ctypes.c_void_p
    L.bpmd_diag_build_tables.argtypes = [vp] * 3 + [ctypes.c_uint32] + [vp] * 4
    r = L.bpmd_diag_build_tables(vp(d_lens.data_ptr()), vp(d_n.data_ptr()), vp(d_t.data_ptr()), n,
                                 vp(wave.data_ptr()), vp(serial.data_ptr()), vp(meta.data_ptr()),
                                 vp(torch.cuda.current_stream().cuda_stream))
    assert r == 0
    torch.cuda.synchronize()
    w = wave.cpu().numpy().view(np.uint16).reshape(n, KENOUGH)
    s = serial.cpu().numpy().view(np.uint16).reshape(n, KENOUGH)
    m = meta.cpu().numpy().reshape(n, 8)
    errs = 0
    for i in range(n):
        err_w, root_w, used_w, _, err_s, root_s, used_s, _ = m[i]
        assert err_w == err_s, (i, cases[i][0], err_w, err_s)
        if err_s == 0:
            assert root_w == root_s and used_w == used_s, (i, root_w, root_s, used_w, used_s)
            assert np.array_equal(w[i, :used_s], s[i, :used_s]), (i, np.nonzero(w[i, :used_s] != s[i, :used_s]))
            errs += 0
    assert n > 300
