import ctypes, random, sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from beast_amd import pmd
L = pmd.lib()
rng = random.Random(1)
n = 2000
steps = np.array([[rng.choice([1,2,2,3,3,4,5,7,9,11]) for _ in range(64)] for _ in range(n)], dtype=np.uint32)
d = torch.from_numpy(steps.reshape(-1)).cuda()
out = torch.zeros(n, dtype=torch.int64, device="cuda")
vp = ctypes.c_void_p
L.bpmd_diag_chain.argtypes = [vp, ctypes.c_uint32, vp, vp]
L.bpmd_diag_chain(vp(d.data_ptr()), n, vp(out.data_ptr()), None)
torch.cuda.synchronize()
got = out.cpu().numpy().view(np.uint64)
bad = 0
for c in range(n):
    m, o = 0, 0
    while o < 64:
        m |= 1 << o; o += int(steps[c][o])
    if int(got[c]) != m:
        bad += 1
        if bad < 3: print("case", c, bin(int(got[c])), bin(m))
print("bad", bad, "of", n)
