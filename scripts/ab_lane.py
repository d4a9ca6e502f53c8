"""Times the C2 inflate launch for library variants (timing only; experiment
variants may produce wrong output).  VARIANTS="nostore noload" python scripts/ab_lane.py"""
import ctypes
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from beast_amd import synth  # noqa: E402


def main():
    n = int(os.environ.get("DIAG_MSGS", "65536"))
    lens = np.full(n, 4096, dtype=np.uint32)
    raw, off, ln = synth.make_batch("json", lens, seed=0x5EED0002)
    payloads = bench.pmd_compress_host(raw, off, ln)
    buf, coff, clen = bench.pack(payloads)
    dev = torch.device("cuda", 0)
    d_in = torch.from_numpy(buf).to(dev)
    d_off = torch.from_numpy(coff.astype(np.uint64).view(np.int64)).to(dev)
    d_len = torch.from_numpy(clen.astype(np.int32)).to(dev)
    cap = torch.full((n,), 4096, dtype=torch.int32, device=dev)
    o_off = torch.arange(n, dtype=torch.int64, device=dev) * 4096
    out = torch.empty(n * 4096 + 64, dtype=torch.uint8, device=dev)
    olen = torch.empty(n, dtype=torch.int32, device=dev)
    st = torch.empty(n, dtype=torch.int32, device=dev)

    class Cfg(ctypes.Structure):
        _fields_ = [("level", ctypes.c_int), ("window_bits", ctypes.c_int), ("mem_level", ctypes.c_int),
                    ("strategy", ctypes.c_int), ("flags", ctypes.c_uint32)]
    cfg = Cfg(0, 15, 8, 0, 0)
    ref = torch.from_numpy(raw.reshape(n, 4096)).to(dev)
    for v in ["default"] + os.environ.get("VARIANTS", "").split():
        path = os.path.join(ROOT, "beast_amd", "libbeast_pmd.so" if v == "default" else f"libbeast_pmd_{v}.so")
        L = ctypes.CDLL(path)
        L.bpmd_set_inflate_kernel(int(os.environ.get("KERNEL", "1")))
        p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        args = (ctypes.byref(cfg), p(d_in), p(d_off), p(d_len), ctypes.c_uint32(n), p(out), p(o_off), p(cap), p(olen),
                p(st), ctypes.c_void_p(0))
        assert L.bpmd_inflate_batch(*args) == 0
        torch.cuda.synchronize()
        ok = torch.equal(out[:n * 4096].view(n, 4096), ref)
        ts = []
        for _ in range(8):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            L.bpmd_inflate_batch(*args)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        ms = float(np.median(ts))
        print(f"{v:>10}: {ms:7.3f} ms  {n * 4096 / 2**30 / (ms / 1e3):7.2f} GiB/s  exact={ok}", flush=True)


if __name__ == "__main__":
    main()
