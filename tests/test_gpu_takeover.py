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
