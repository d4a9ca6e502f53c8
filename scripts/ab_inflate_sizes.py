"""Times GPU inflate on the C4 (Zipf 256 B-64 KiB JSON, L6) and C5 (64 KiB binary,
L6) shapes with each inflate kernel forced (bpmd_set_inflate_kernel: 0 auto,
1 lane, 2 wave; SPLITS="1024 2048" adds auto runs at those BPMD_INFLATE_SPLIT values): median of 5 launches by HIP events, GiB/s of output.  The
payloads are the GPU deflater's (checked back against the messages)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from beast_amd import pmd, synth  # noqa: E402


def workloads():
    yield "C2-shape 4KiB", 6, synth.make_batch("json", np.full(65536, 4096, dtype=np.uint32), seed=0x5EED0002)
    lens = synth.zipf_sizes(int(os.environ.get("C4_MSGS", "65536")), 0x5EED0004)
    yield "C4 zipf L6", 6, synth.make_batch("json", lens, seed=0x5EED0004)
    n5 = int(os.environ.get("C5_MSGS", "4096"))
    yield "C5 binary L6", 6, synth.make_batch("binary", np.full(n5, 65536, dtype=np.uint32), seed=0x5EED0005)


def main():
    for name, level, (raw, off, ln) in workloads():
        src = pmd.Batch.from_arrays(raw, off.astype(np.int64), ln.astype(np.int32))
        d = pmd.deflate_batch(src, level=level)
        comp = pmd.Batch(d.out.data, d.out.off, d.out.len)
        cap = torch.from_numpy(ln.astype(np.int32)).cuda()
        total = int(ln.astype(np.int64).sum())
        runs = [(0, f"auto/{t}", t) for t in os.environ.get("SPLITS", "").split()]
        runs += [(0, "auto", None), (1, "lane", None), (2, "wave", None)]
        for mode, kname, split in runs:
            if split is None:
                os.environ.pop("BPMD_INFLATE_SPLIT", None)
            else:
                os.environ["BPMD_INFLATE_SPLIT"] = split
            assert pmd.lib().bpmd_set_inflate_kernel(mode) == 0
            r = pmd.inflate_batch(comp, cap)
            torch.cuda.synchronize()
            ok = int((r.status != 0).sum()) == 0 and torch.equal(r.out.len, src.len)
            ts = []
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                pmd.inflate_batch(comp, cap, out=r.out.data, out_off=r.out.off)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            ms = float(np.median(ts))
            print(f"{name:14s} {kname:10s} n={len(ln)} {total / 2**20:8.1f} MiB  {ms:8.3f} ms  "
                  f"{total / 2**30 / (ms / 1e3):7.2f} GiB/s  ok={ok}", flush=True)
        pmd.lib().bpmd_set_inflate_kernel(0)


if __name__ == "__main__":
    main()
