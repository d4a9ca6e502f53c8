"""Cross-connection micro-batcher on the GPU: many
threads submit single messages; every completion must carry the oracle's
status and bytes, whether the batch was launched because it filled up, because
its oldest message waited max_delay_us, or by flush()."""
import random
import threading

import pytest

from beast_amd import synth
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _msgs(rng, n):
    out = []
    for i in range(n):
        d, _, _ = synth.make_batch(rng.choice(["json", "corpus1", "binary", "zeros"]),
                                   [rng.choice([0, 1, 200, 4096, 9000])], seed=i)
        out.append(bytes(d))
    return out


def test_inflate_from_many_threads():
    from beast_amd import pmd
    rng = random.Random(1)
    msgs = _msgs(rng, 1200)
    payloads = [O.pmd_deflate(m, 6, 15, 4) for m in msgs]
    payloads[7] = payloads[7][:len(payloads[7]) // 2]   # a truncated one
    b = pmd.Batcher("inflate", max_msgs=256, max_in_bytes=1 << 20, max_out_bytes=4 << 20, max_delay_us=500)
    comps = [None] * len(payloads)

    def worker(t):
        for i in range(t, len(payloads), 8):
            comps[i] = b.submit(payloads[i], 9000)

    ts = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    b.flush()
    for i, c in enumerate(comps):
        st, out = c.wait(10)
        est, eout = O.pmd_inflate(payloads[i], cap=9000)
        assert st == est and out == eout, i
    b.close()


def test_deflate_round_trip_and_small_buffers():
    from beast_amd import pmd
    rng = random.Random(2)
    msgs = _msgs(rng, 600)
    b = pmd.Batcher("deflate", level=6, max_msgs=128, max_in_bytes=1 << 20, max_out_bytes=2 << 20)
    comps = [b.submit(m, O.upper_bound(len(m))) for m in msgs]
    small = b.submit(msgs[3] if len(msgs[3]) > 100 else b"x" * 5000, 4)
    b.flush()
    for m, c in zip(msgs, comps):
        st, p = c.wait(10)
        assert st == 0
        est, out = O.pmd_inflate(p, cap=max(len(m), 1))
        assert est == 0 and out == m
    assert small.wait(10)[0] == 1   # need_buffers: the caller's buffer is too small
    b.close()


def test_delay_launches_without_flush():
    from beast_amd import pmd
    b = pmd.Batcher("inflate", max_msgs=4096, max_delay_us=2000)
    p = O.pmd_deflate(b"hello hello hello", 6, 15, 4)
    c = b.submit(p, 100)
    assert c.wait(30) == (0, b"hello hello hello")
    b.close()
