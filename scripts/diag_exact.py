"""Which C2 messages a library variant gets wrong, and where (diagnostics).
LIB=libbeast_pmd_lpw32.so python scripts/diag_exact.py"""
import ctypes
import os
import sys

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
    d_off = torch.from_numpy(coff.astype(np.int64)).to(dev)
    d_len = torch.from_numpy(clen.astype(np.int32)).to(dev)
    cap = torch.full((n,), 4096, dtype=torch.int32, device=dev)
    o_off = torch.arange(n, dtype=torch.int64, device=dev) * 4096
    ref = torch.from_numpy(raw.reshape(n, 4096)).to(dev)

    class Cfg(ctypes.Structure):
        _fields_ = [("level", ctypes.c_int), ("window_bits", ctypes.c_int), ("mem_level", ctypes.c_int),
                    ("strategy", ctypes.c_int), ("flags", ctypes.c_uint32)]
    cfg = Cfg(0, 15, 8, 0, 0)
    L = ctypes.CDLL(os.path.join(ROOT, "beast_amd", os.environ.get("LIB", "libbeast_pmd.so")))
    L.bpmd_set_inflate_kernel(1)
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    for rep in range(3):
        out = torch.zeros(n * 4096 + 64, dtype=torch.uint8, device=dev)
        olen = torch.full((n,), -1, dtype=torch.int32, device=dev)
        st = torch.full((n,), -7, dtype=torch.int32, device=dev)
        assert L.bpmd_inflate_batch(ctypes.byref(cfg), p(d_in), p(d_off), p(d_len), n, p(out), p(o_off), p(cap),
                                    p(olen), p(st), None) == 0
        torch.cuda.synchronize()
        got = out[:n * 4096].view(n, 4096)
        bad = (got != ref).any(dim=1) | (st != 0) | (olen != 4096)
        idx = torch.nonzero(bad).flatten().cpu().numpy()
        print(f"rep {rep}: {len(idx)} bad messages; status hist {np.unique(st.cpu().numpy(), return_counts=True)}",
              flush=True)
        if len(idx):
            lanes = np.bincount(idx % 64, minlength=64)
            print("  by lane%64:", lanes.tolist())
            print("  by block%8:", np.bincount((idx // 32) % 8, minlength=8).tolist())
            for i in idx[:4]:
                g = got[i].cpu().numpy()
                r = raw.reshape(n, 4096)[i]
                d = np.nonzero(g != r)[0]
                print(f"  msg {i}: st={int(st[i])} len={int(olen[i])} first diff at {d[0] if len(d) else None}, "
                      f"ndiff={len(d)} got={g[d[0]:d[0]+16].tobytes() if len(d) else b''} "
                      f"want={r[d[0]:d[0]+16].tobytes() if len(d) else b''}", flush=True)


if __name__ == "__main__":
    main()
