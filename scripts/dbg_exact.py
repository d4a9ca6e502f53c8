"""Exact-mode deflate bring-up: one message per launch, progress printed."""
import sys
import os
import time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from beast_amd import pmd, synth  # noqa: E402
from oracle import oracle as O  # noqa: E402

for level in (0, 6) if len(sys.argv) < 2 else (int(sys.argv[1]),):
    for kind in ("json", "zeros"):
        for n in (0, 1, 17, 4096):
            d, _, _ = synth.make_batch(kind, [max(n, 1)], seed=n)
            m = bytes(d[:n])
            t = time.time()
            res = pmd.deflate_batch(pmd.Batch.from_host([m]), level=level, exact=True)
            torch.cuda.synchronize()
            got = res.out.to_host()[0]
            print(level, kind, n, int(res.status[0]), got == O.pmd_deflate(m, level), f"{time.time() - t:.3f}s", flush=True)
