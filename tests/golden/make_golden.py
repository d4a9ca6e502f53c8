"""Regenerates tests/golden/deflate_golden.json (run in the build container).

Expected permessage-deflate payloads come from the reference's own vendored
zlib 1.3.1 (/root/reference/test/extern/zlib-1.3.1 compiled in place by
oracle/Makefile into oracle/_ref/libzref.so), driven with Beast's pmd call
pattern (websocket/detail/impl_base.hpp:85-154).  Beast's deflate equals zlib
1.3.1 at levels 1-9, so these vectors pin the C restatement
in oracle/ without needing the reference at test time.  Inputs are the seeded
synthetic corpora of beast_amd/synth.py; the manifest stores their sha256 and,
for small messages, the expected payload itself.
"""
import hashlib
import json
import os
import sys
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from beast_amd import synth  # noqa: E402
from oracle import oracle as O  # noqa: E402

SEED = 0x5EED0100
KINDS = ["json", "corpus1", "random", "zeros"]
SIZES = [0, 1, 17, 255, 1024, 4096, 65536]
CONFIGS = [(1, 15, 4), (6, 15, 4), (8, 15, 4), (9, 15, 4), (6, 15, 8), (6, 9, 4), (1, 9, 8), (6, 15, 9)]
STRATS = [(6, 15, 4, s) for s in (1, 2, 3, 4)]


def main():
    assert O.ref() is not None, "oracle/_ref/libzref.so missing: run make -C oracle"
    entries = []
    for ki, kind in enumerate(KINDS):
        for size in SIZES:
            data, _, _ = synth.make_batch(kind, [size], seed=SEED + ki)
            msg = bytes(data[:size])
            for (lvl, wb, mem, *st) in CONFIGS + STRATS:
                strat = st[0] if st else 0
                exp = O.ref_pmd_deflate(msg, lvl, wb, mem, strat)
                # independent cross-check with the system zlib at the pmd defaults
                if strat == 0 and wb == 15 and size:
                    c = zlib.compressobj(lvl, zlib.DEFLATED, -wb, mem, strat)
                    py = c.compress(msg) + c.flush(zlib.Z_BLOCK) + c.flush(zlib.Z_SYNC_FLUSH)
                    assert py[:-4] == exp, (kind, size, lvl, wb, mem)
                e = {"kind": kind, "seed": SEED + ki, "size": size, "level": lvl, "wbits": wb, "mem": mem,
                     "strategy": strat, "in_sha256": hashlib.sha256(msg).hexdigest(),
                     "out_len": len(exp), "out_sha256": hashlib.sha256(exp).hexdigest()}
                if len(exp) <= 160:
                    e["out_hex"] = exp.hex()
                entries.append(e)
    doc = {"source": __doc__.strip().splitlines()[0] + " See make_golden.py.", "entries": entries}
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "deflate_golden.json"), "w") as f:
        json.dump(doc, f, indent=0)
    print(len(entries), "entries")


if __name__ == "__main__":
    main()
