"""GPU: batch calls from several host threads on one HIP stream (the null
stream here) are serialised per stream (pmd_capi.hip stream_mutex), so their
work-queue counters and chunk workspaces never interleave: every thread's
results equal a single-threaded run's."""
import threading

import numpy as np
import pytest
import torch

from beast_amd import pmd, synth

pytestmark = pytest.mark.gpu


def test_two_threads_same_stream():
    # big enough for the work-queue and chunk paths (scratch blocks 0/1/2/5/7/9)
    lens = synth.zipf_sizes(70000, 0x5EED00C1)
    data, off, ln = synth.make_batch("json", lens, seed=0x5EED00C1)
    src = pmd.Batch.from_arrays(data, off, ln)
    ref = pmd.deflate_batch(src, level=6)
    torch.cuda.synchronize()
    ref_pay = ref.out.to_host()
    comp = pmd.Batch.from_host(ref_pay)
    errors = []

    def worker(k):
        try:
            for _ in range(3):
                d = pmd.deflate_batch(src, level=6)          # null stream, concurrently
                r = pmd.inflate_batch(comp, src.len)
                torch.cuda.synchronize()
                assert int((d.status != 0).sum()) == 0 and int((r.status != 0).sum()) == 0
                assert torch.equal(d.out.len, ref.out.len)
                assert torch.equal(r.out.len, src.len)
                tot = int(ln.astype(np.int64).sum())
                assert torch.equal(r.out.data[:tot], src.data[:tot])
        except Exception as e:   # noqa: BLE001 -- reported below
            errors.append((k, repr(e)))

    ts = [threading.Thread(target=worker, args=(k,)) for k in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors
