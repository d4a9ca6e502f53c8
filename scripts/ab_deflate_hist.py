import ctypes, os, sys, numpy as np, torch
sys.path.insert(0, '/root/repo')
from beast_amd import synth
from oracle import oracle as O
for v in ["default"] + os.environ["VARIANTS"].split():
    path = "/root/repo/beast_amd/libbeast_pmd.so" if v == "default" else f"/root/repo/beast_amd/libbeast_pmd_{v}.so"
    os.environ["BPMD_LIB"] = path
    import importlib
    from beast_amd import pmd
    pmd._LIB = None
    importlib.reload(pmd)
    for kind, lens, seed in (("binary", np.full(4096, 65536, dtype=np.uint32), 0x5EED0005), ("json", synth.zipf_sizes(65536, 0x5EED0004), 0x5EED0004)):
        raw, off, ln = synth.make_batch(kind, lens, seed=seed)
        src = pmd.Batch.from_arrays(raw, off.astype(np.int64), ln.astype(np.int32))
        d = pmd.deflate_batch(src, level=6)
        torch.cuda.synchronize()
        ts = []
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(); d = pmd.deflate_batch(src, level=6); e1.record(); torch.cuda.synchronize(); ts.append(e0.elapsed_time(e1))
        total = int(ln.astype(np.int64).sum()); ms = float(np.median(ts))
        comp = int(d.out.len.to(torch.int64).sum())
        # Beast's size on a sample
        k = 400 if kind == "json" else 40
        beast = sum(len(O.pmd_deflate(bytes(raw[int(off[i]):int(off[i])+int(ln[i])]), 6, 15, 4)) for i in range(k))
        gpu = int(d.out.len[:k].to(torch.int64).sum())
        print(f"{v:8s} {kind:6s} {total/2**30/(ms/1e3):6.2f} GiB/s ratio {comp/total:.4f} size/Beast(first {k}) {gpu/beast:.4f}", flush=True)
