"""Debug helper: inflate one known payload with the prof library and dump
the kernel's debug record (g_prof_dbg)."""
import ctypes
import sys

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import torch  # noqa: E402

from beast_amd import pmd, synth  # noqa: E402
from oracle import oracle as O  # noqa: E402

d, _, _ = synth.make_batch("json", [255], seed=1 * 100 + 4 + 255)
p = O.pmd_deflate(bytes(d[:255]), 1, 15, 4)
L = pmd.lib()
L.bpmd_diag_counters.argtypes = [ctypes.c_void_p, ctypes.c_int]
c = (ctypes.c_ulonglong * 24)()
L.bpmd_diag_counters(c, 1)
res = pmd.inflate_batch(pmd.Batch.from_host([p]), 255)
torch.cuda.synchronize()
print("status", res.status.cpu().tolist())
dd = (ctypes.c_ulonglong * 16)()
L.bpmd_diag_counters(dd, 2)
for k in range(5):
    w, hv, sl = dd[3 * k], dd[3 * k + 1], dd[3 * k + 2]
    print("chain", bin(w), "have", hv >> 32, "->", hv & 0xffffffff, "stop_at", sl >> 32, "lastp", sl & 0xffffffff)
