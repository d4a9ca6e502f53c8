"""Deflate rate and size against Beast's per level on a C4-shaped sample
(64 Ki Zipf JSON messages): levels >= 7 give each chunk 4 KiB of history
(lz::chunk_hist), the others 2 KiB.  Size ratio = GPU bytes / Beast bytes
(the oracle's port of Beast's deflate_stream, memLevel 4) on the first 400
messages.
    python scripts/deflate_levels.py [levels...]
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from beast_amd import pmd, synth  # noqa: E402
from oracle import oracle as O  # noqa: E402


def main():
    levels = [int(x) for x in sys.argv[1:]] or [6, 8, 9]
    raw, off, ln = synth.make_batch("json", synth.zipf_sizes(65536, 0x5EED0004), seed=0x5EED0004)
    src = pmd.Batch.from_arrays(raw, off.astype(np.int64), ln.astype(np.int32))
    total = int(ln.astype(np.int64).sum())
    k = 400
    for lv in levels:
        d = pmd.deflate_batch(src, level=lv)
        torch.cuda.synchronize()
        ts = []
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            d = pmd.deflate_batch(src, level=lv)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        ms = float(np.median(ts))
        beast = sum(len(O.pmd_deflate(bytes(raw[int(off[i]):int(off[i]) + int(ln[i])]), lv, 15, 4)) for i in range(k))
        gpu = int(d.out.len[:k].to(torch.int64).sum())
        print(f"level {lv}: {total / 2**30 / (ms / 1e3):6.2f} GiB/s, ratio {int(d.out.len.to(torch.int64).sum()) / total:.4f}, "
              f"size / Beast (first {k}) {gpu / beast:.4f}", flush=True)


if __name__ == "__main__":
    main()
