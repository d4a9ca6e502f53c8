import os, sys, numpy as np, torch
sys.path.insert(0, '/root/repo')
from beast_amd import pmd, synth
from oracle import oracle as O
for n, kind in ((300, "json"), (300, "binary"), (300, "zeros")):
    lens = np.full(n, 4096, dtype=np.uint32)
    raw, off, ln = synth.make_batch(kind, lens, seed=5)
    comp, coff, clen, st = O.deflate_batch(raw, off, ln, level=6, mem_level=4, threads=8)
    pmd.lib().bpmd_set_inflate_kernel(1)
    src = pmd.Batch.from_arrays(comp, coff.astype(np.int64), clen.astype(np.int32))
    cap = torch.from_numpy(ln.astype(np.int32)).cuda()
    r = pmd.inflate_batch(src, cap)
    torch.cuda.synchronize()
    stt = r.status.cpu().numpy(); ol = r.out.len.cpu().numpy()
    bad = np.nonzero(stt)[0]
    outs = r.out.to_host()
    wrong = [i for i in range(n) if outs[i] != bytes(raw[int(off[i]):int(off[i]) + 4096])]
    print(kind, "bad status", len(bad), bad[:10], stt[bad[:10]], "wrong content", len(wrong), wrong[:10], ol[wrong[:5]] if wrong else "")
