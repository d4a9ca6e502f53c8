"""Per-role loop counters of the pipelined lane kernel (prof build): runs the
C2 launch once on libbeast_pmd_prof.so and prints cycles and iterations per
wave for the decoder and the expander."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("BPMD_LIB", os.path.join(ROOT, "beast_amd", "libbeast_pmd_prof.so"))
import bench  # noqa: E402
from beast_amd import pmd, synth  # noqa: E402


def main():
    n = int(os.environ.get("DIAG_MSGS", "65536"))
    size = int(os.environ.get("DIAG_SIZE", "4096"))
    lens = np.full(n, size, dtype=np.uint32)
    raw, off, ln = synth.make_batch(os.environ.get("DIAG_KIND", "json"), lens, seed=0x5EED0002)
    buf, coff, clen = bench.pack(bench.pmd_compress_host(raw, off, ln))
    dev = torch.device("cuda", 0)
    src = pmd.Batch(torch.from_numpy(buf).to(dev), torch.from_numpy(coff).to(dev), torch.from_numpy(clen).to(dev))
    cap = torch.full((n,), size, dtype=torch.int32, device=dev)
    L = pmd.lib()
    c = (ctypes.c_ulonglong * 24)()
    pmd.inflate_batch(src, cap)
    torch.cuda.synchronize()
    L.bpmd_diag_lane3_counters24(c, 1)
    r = pmd.inflate_batch(src, cap)
    torch.cuda.synchronize()
    L.bpmd_diag_lane3_counters24(c, 1)
    ok = torch.equal(r.out.data[: n * size].view(n, size), torch.from_numpy(raw.reshape(n, size)).to(dev))
    w = n // 64
    names = ["dec cycles", "dec iters", "dec sleeps", "dec hdr iters", "exp cycles", "exp iters", "exp sleeps", "lanes: header, ring not empty",
             "dec lap: input+tail", "dec lap: S_DATA", "dec lap: headers", "dec lap: publish+loop",
             "lanes: data, ring full", "lanes: data, room", "lanes: finished", "lanes: in headers",
             "hdr: type/stored/copy", "hdr: table+lenlens", "hdr: codelens", "hdr: build", "hdr: place", "-", "-", "-"]
    for i, nm in enumerate(names):
        if nm == "-":
            continue
        print(f"{nm:14s} {c[i] / w:12.0f} per wave")
    print("exact", ok)


if __name__ == "__main__":
    main()
