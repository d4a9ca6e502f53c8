"""Times GPU deflate on the C4 (Zipf 256 B-64 KiB JSON, L6) and C5 (64 KiB binary,
L1 and L6) shapes for library variants: median of 5 launches by HIP events on
the current stream, GiB/s of uncompressed input, and the compressed ratio.
VARIANTS="prev" python scripts/ab_deflate_sizes.py   (libbeast_pmd_<v>.so)
STATIC=1 adds the product library with the history kernel on a static grid
stride (bpmd_deflate_static_grid) instead of its work queue."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from beast_amd import synth  # noqa: E402


class Cfg(ctypes.Structure):
    _fields_ = [("level", ctypes.c_int), ("window_bits", ctypes.c_int), ("mem_level", ctypes.c_int),
                ("strategy", ctypes.c_int), ("flags", ctypes.c_uint32)]


def workloads():
    n4 = int(os.environ.get("C4_MSGS", "65536"))
    lens = synth.zipf_sizes(n4, 0x5EED0004)
    yield "C4 zipf L6", 6, synth.make_batch("json", lens, seed=0x5EED0004)
    n5 = int(os.environ.get("C5_MSGS", "4096"))
    b = synth.make_batch("binary", np.full(n5, 65536, dtype=np.uint32), seed=0x5EED0005)
    yield "C5 binary L1", 1, b
    yield "C5 binary L6", 6, b


def main():
    dev = torch.device("cuda", 0)
    libs = [("default", "libbeast_pmd.so")] + [(v, f"libbeast_pmd_{v}.so")
                                               for v in os.environ.get("VARIANTS", "").split()]
    libs = [(v, ctypes.CDLL(os.path.join(ROOT, "beast_amd", f))) for v, f in libs]
    if os.environ.get("STATIC"):
        libs.insert(1, ("static", libs[0][1]))
    for name, level, (raw, off, ln) in workloads():
        n = len(ln)
        d_in = torch.from_numpy(raw).to(dev)
        d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
        d_len = torch.from_numpy(ln.astype(np.int32)).to(dev)
        ub = ln.astype(np.int64) + (ln.astype(np.int64) + 7) // 8 + (ln.astype(np.int64) + 63) // 64 + 11
        slot = (ub + 15) // 16 * 16
        o_off_h = np.zeros(n, dtype=np.int64)
        o_off_h[1:] = np.cumsum(slot[:-1])
        o_off = torch.from_numpy(o_off_h).to(dev)
        cap = torch.from_numpy(ub.astype(np.int32)).to(dev)
        out = torch.empty(int(slot.sum()) + 64, dtype=torch.uint8, device=dev)
        olen = torch.empty(n, dtype=torch.int32, device=dev)
        st = torch.empty(n, dtype=torch.int32, device=dev)
        cfg = Cfg(level, 15, 4, 0, 0)
        p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        total = int(ln.astype(np.int64).sum())
        for v, L in libs:
            if v in ("default", "static"):
                ctypes.c_uint.in_dll(L, "bpmd_deflate_static_grid").value = 1 if v == "static" else 0
            s = torch.cuda.current_stream().cuda_stream
            args = (ctypes.byref(cfg), p(d_in), p(d_off), p(d_len), ctypes.c_uint32(n), p(out), p(o_off), p(cap),
                    p(olen), p(st), ctypes.c_void_p(s))
            assert L.bpmd_deflate_batch(*args) == 0
            torch.cuda.synchronize()
            ok = int((st != 0).sum()) == 0
            ratio = int(olen.to(torch.int64).sum()) / total
            ts = []
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                L.bpmd_deflate_batch(*args)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            ms = float(np.median(ts))
            print(f"{name:14s} {v:8s} n={n} {total / 2**20:8.1f} MiB  {ms:8.3f} ms  "
                  f"{total / 2**30 / (ms / 1e3):7.2f} GiB/s  ratio {ratio:.4f}  ok={ok}", flush=True)


if __name__ == "__main__":
    main()
