"""Times the C3 deflate launch (64 Ki x 4 KiB JSON, L6) for library variants and
reports each one's size against Beast's (oracle) on the first 8 Ki messages.
VARIANTS="chain16 chain8" python scripts/ab_deflate.py"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from beast_amd import synth  # noqa: E402
from oracle import oracle as O  # noqa: E402


def main():
    n = int(os.environ.get("DIAG_MSGS", "65536"))
    lens = np.full(n, 4096, dtype=np.uint32)
    raw, off, ln = synth.make_batch("json", lens, seed=0x5EED0003)
    k = min(n, 8192)
    _, _, blen, _ = O.deflate_batch(raw, off[:k], ln[:k], level=6, mem_level=4, threads=16)
    beast = int(blen.astype(np.int64).sum())
    dev = torch.device("cuda", 0)
    d_in = torch.from_numpy(raw).to(dev)
    d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
    d_len = torch.from_numpy(ln.astype(np.int32)).to(dev)
    ub = 4096 + 512 + 64 + 11
    slot = (ub + 15) // 16 * 16
    cap = torch.full((n,), ub, dtype=torch.int32, device=dev)
    o_off = torch.arange(n, dtype=torch.int64, device=dev) * slot
    out = torch.empty(n * slot + 64, dtype=torch.uint8, device=dev)
    olen = torch.empty(n, dtype=torch.int32, device=dev)
    st = torch.empty(n, dtype=torch.int32, device=dev)

    class Cfg(ctypes.Structure):
        _fields_ = [("level", ctypes.c_int), ("window_bits", ctypes.c_int), ("mem_level", ctypes.c_int),
                    ("strategy", ctypes.c_int), ("flags", ctypes.c_uint32)]
    cfg = Cfg(6, 15, 4, 0, 0)
    for v in ["default"] + os.environ.get("VARIANTS", "").split():
        path = os.path.join(ROOT, "beast_amd", "libbeast_pmd.so" if v == "default" else f"libbeast_pmd_{v}.so")
        L = ctypes.CDLL(path)
        p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        args = (ctypes.byref(cfg), p(d_in), p(d_off), p(d_len), ctypes.c_uint32(n), p(out), p(o_off), p(cap), p(olen),
                p(st), ctypes.c_void_p(0))
        assert L.bpmd_deflate_batch(*args) == 0
        torch.cuda.synchronize()
        ok = int((st != 0).sum()) == 0
        sizes = olen.cpu().numpy().astype(np.int64)
        # spot-check round trips with the oracle
        host = out.cpu().numpy()
        for i in range(0, n, n // 64):
            s0 = int(o_off[i])
            est, eo = O.pmd_inflate(host[s0:s0 + int(sizes[i])].tobytes(), cap=4096)
            ok = ok and est == 0 and eo == raw[int(off[i]):int(off[i]) + 4096].tobytes()
        ts = []
        for _ in range(6):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            L.bpmd_deflate_batch(*args)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        ms = float(np.median(ts))
        print(f"{v:>10}: {ms:7.3f} ms  {n * 4096 / 2**30 / (ms / 1e3):7.2f} GiB/s  size/beast="
              f"{sizes[:k].sum() / beast:.4f}  ok={ok}", flush=True)


if __name__ == "__main__":
    main()
