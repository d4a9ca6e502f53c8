"""Beast's compressed size on a sample of the C5 shape (the oracle's port of
Beast's deflate_stream, memLevel 4 = permessage_deflate's default, window 15),
for the ratio column of DESIGN.md section 6.  CPU only.
  python scripts/beast_ratio.py [messages]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from beast_amd import synth  # noqa: E402
from oracle import oracle as O  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
lens = np.full(n, 65536, dtype=np.uint32)
data, off, lens = synth.make_batch("binary", lens, seed=0x5EED0005)   # bench.py SEED_C5
for lvl in (1, 6):
    comp, coff, clen, cst = O.deflate_batch(data, off, lens, level=lvl, wbits=15, mem_level=4, threads=8)
    assert (cst == 0).all()
    print(f"C5 sample {n} x 64 KiB, level {lvl}, memLevel 4: Beast ratio {clen.sum() / lens.sum():.4f}")
