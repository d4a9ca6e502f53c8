"""Block-parallel inflate (pmd_inflate_bp.hip) against the wave kernel on
long payloads, for this library's deflater and Beast's own (exact mode):
    python scripts/diag_bp.py [quick]
"""
import ctypes
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from beast_amd import pmd, synth  # noqa: E402

MODES = {"auto": 0, "wave": 2, "bp": 3}


def run(kind, n, size, producer, level, modes):
    lens = np.full(n, size, dtype=np.uint32)
    raw, off, ln = synth.make_batch(kind, lens, seed=0x5EED00D5)
    src = pmd.Batch.from_arrays(raw, off.astype(np.int64), ln.astype(np.int32))
    d = pmd.deflate_batch(src, level=level, mem_level=4, exact=(producer == "beast"))
    torch.cuda.synchronize()
    comp = pmd.Batch(d.out.data, d.out.off, d.out.len)
    L = pmd.lib()
    c0 = (ctypes.c_ulonglong * 12)()
    L.bpmd_diag_bp_counters(c0, 1)
    for name in modes:
        L.bpmd_set_inflate_kernel(MODES[name])
        r = pmd.inflate_batch(comp, size)
        torch.cuda.synchronize()
        ok = int((r.status != 0).sum()) == 0 and torch.equal(r.out.data[:n * size].view(n, size),
                                                             src.data[:n * size].view(n, size))
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            pmd.inflate_batch(comp, size)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        t = float(np.median(ts))
        c = (ctypes.c_ulonglong * 12)()
        L.bpmd_diag_bp_counters(c, 1)
        runs = 6
        print(f"{kind:6s} {producer:5s} L{level} n={n:6d} size={size:6d} {name:5s} {t * 1e3:8.3f} ms "
              f"{n * size / t / 2**30:7.2f} GiB/s ok={ok}  bp: msgs {c[0] // runs} segs/msg "
              f"{c[1] / max(c[0], 1):.1f} fallbacks {c[2] // runs} regions {c[4] // runs} stored {c[5] // runs} "
              f"dynscan {c[6] // runs} deep {c[7] // runs} cyc/region stage {c[8] / max(c[4], 1):.0f} "
              f"stored {c[9] / max(c[4], 1):.0f} dyn {c[10] / max(c[6], 1):.0f}", flush=True)
    L.bpmd_set_inflate_kernel(0)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "case":   # case kind n size producer level mode
        k, n, sz, pr, lv, md = sys.argv[2:8]
        run(k, int(n), int(sz), pr, int(lv), [md])
        sys.exit(0)
    quick = len(sys.argv) > 1 and sys.argv[1] == "quick"
    cases = [("binary", 16384, 65536, "gpu", 1), ("binary", 16384, 65536, "gpu", 6),
             ("json", 9216, 40960, "gpu", 6), ("binary", 2048, 65536, "gpu", 1)]
    if not quick:
        cases += [("binary", 4096, 65536, "beast", 1), ("json", 4096, 40960, "beast", 6)]
    for kind, n, size, producer, level in cases:
        run(kind, n, size, producer, level, ["bp", "wave", "auto"])
