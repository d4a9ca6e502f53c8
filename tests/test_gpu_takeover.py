"""Context-takeover streams on the GPU.

Without no_context_takeover, every connection's messages continue one deflate
stream: Beast's deflater is not reset between messages (impl_base.hpp:156-166)
and its inflater keeps its window (impl_base.hpp:192-202), so a message may
copy from earlier messages.  Each batch holds one message per connection; the
GPU must produce the oracle's bytes and statuses decoding the same stream
message by message."""
import random

import pytest

from beast_amd import synth
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _streams(rng, n_conn, rounds, level=6, wbits=15):
    msgs, pls = [], []
    for c in range(n_conn):
        kind = rng.choice(["json", "corpus1", "json"])
        ms = []
        for r in range(rounds):
            d, _, _ = synth.make_batch(kind, [rng.choice([0, 50, 700, 4096, 9000])], seed=c * 131 + r)
            ms.append(bytes(d))
        msgs.append(ms)
        pls.append(O.pmd_deflate_stream(ms, level, wbits, 4))
    return msgs, pls


@pytest.mark.parametrize("wbits", [15, 10])
def test_takeover_streams_match_oracle(wbits):
    import torch
    from beast_amd import pmd
    rng = random.Random(21 + wbits)
    n_conn, rounds = 200, 6
    msgs, pls = _streams(rng, n_conn, rounds, wbits=wbits)
    cap = 9000
    expect = [O.pmd_inflate_stream(p, cap=cap, wbits=wbits) for p in pls]
    tk = pmd.TakeoverInflater(n_conn, window_bits=wbits, max_msg=cap)
    uses_history = 0
    for r in range(rounds):
        batch = pmd.Batch.from_host([pls[c][r] for c in range(n_conn)])
        res = tk.inflate(batch, cap)
        torch.cuda.synchronize()
        st = res.status.cpu().tolist()
        outs = res.out.to_host()
        for c in range(n_conn):
            est, eout = expect[c][r]
            assert st[c] == est, (r, c, st[c], est)
            assert outs[c] == eout == msgs[c][r], (r, c)
        if r:
            fresh = [O.pmd_inflate(pls[c][r], cap=cap)[0] for c in range(n_conn)]
            uses_history += sum(1 for f in fresh if f != 0)
    assert uses_history > 0   # the streams really do reach into earlier messages


def test_distance_past_the_window_is_invalid():
    import torch
    from beast_amd import pmd
    rng = random.Random(5)
    # compressed with a 32 KiB window, decoded with a 512-byte one
    msgs, pls = _streams(rng, 64, 3, wbits=15)
    expect = [O.pmd_inflate_stream(p, cap=9000, wbits=9) for p in pls]
    tk = pmd.TakeoverInflater(64, window_bits=9, max_msg=9000)
    for r in range(3):
        res = tk.inflate(pmd.Batch.from_host([pls[c][r] for c in range(64)]), 9000)
        torch.cuda.synchronize()
        st = res.status.cpu().tolist()
        for c in range(64):
            if r == 0 or all(expect[c][k][0] == 0 for k in range(r)):
                assert st[c] == expect[c][r][0], (r, c, st[c], expect[c][r][0])


def test_takeover_deflate_round_trips_and_shrinks():
    """GPU deflate with context takeover: every connection's payload stream
    inflates (oracle, window kept) back to its messages, and reaching into
    earlier messages makes the payloads smaller than independent ones."""
    import torch
    from beast_amd import pmd
    rng = random.Random(31)
    n_conn, rounds = 150, 5
    msgs = []
    for c in range(n_conn):
        msgs.append([bytes(synth.make_batch("json", [rng.choice([1, 300, 2000, 4096, 6000])], seed=c * 7 + r)[0])
                     for r in range(rounds)])
    td = pmd.TakeoverDeflater(n_conn, level=6, max_msg=6000)
    pls = [[None] * rounds for _ in range(n_conn)]
    took = plain = 0
    for r in range(rounds):
        src = pmd.Batch.from_host([msgs[c][r] for c in range(n_conn)])
        res = td.deflate(src)
        ind = pmd.deflate_batch(src, level=6)
        torch.cuda.synchronize()
        assert res.status.cpu().tolist() == [0] * n_conn
        outs = res.out.to_host()
        for c in range(n_conn):
            pls[c][r] = outs[c]
        if r:
            took += sum(len(o) for o in outs)
            plain += sum(ind.out.len.cpu().tolist())
    for c in range(n_conn):
        got = O.pmd_inflate_stream(pls[c], cap=6000)
        assert [g[0] for g in got] == [0] * rounds, c
        assert [g[1] for g in got] == msgs[c], c
    assert took < plain, (took, plain)
