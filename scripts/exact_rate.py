"""Exact-mode deflate rate (BPMD_F_EXACT) on the C3 batch (64 Ki x 4 KiB
JSON, L6/mem4/w15) and on a C4-shaped Zipf sample, by HIP events; payloads
of a sample checked against the oracle (Beast's deflater)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import bench  # noqa: E402
from beast_amd import pmd, synth  # noqa: E402
from oracle import oracle as O  # noqa: E402


def cpu(name, raw, off, lens, threads=32):
    """The same batch on the host: the reference's zlib 1.3.1 (oracle/_ref) and the port, `threads` threads."""
    cap = (lens.astype(np.uint64) + lens.astype(np.uint64) // 1000 + 64).astype(np.uint32)
    gib = float(lens.astype(np.int64).sum()) / 2**30
    for impl in ("reference", "port"):
        r = O.time_batch(impl, False, raw, off, lens, cap, threads=threads, reps=3)
        if r is not None:
            print(f"{name} CPU {impl} {threads} threads {r[0] * 1e3:.1f} ms {gib / r[0]:.2f} GiB/s", flush=True)


def run(name, raw, off, lens, check=512):
    dev = torch.device("cuda", 0)
    src = pmd.Batch(torch.from_numpy(raw).to(dev), torch.from_numpy(off.astype(np.int64)).to(dev),
                    torch.from_numpy(lens.astype(np.int32)).to(dev))
    for exact in (False, True):
        r = pmd.deflate_batch(src, level=6, exact=exact)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        r = pmd.deflate_batch(src, level=6, exact=exact)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        gib = float(lens.astype(np.int64).sum()) / 2**30
        outl = r.out.len.cpu().numpy()
        line = f"{name} exact={exact} {ms:.2f} ms {gib / (ms / 1e3):.2f} GiB/s ratio {outl.sum() / lens.sum():.4f}"
        if exact:
            pl = r.out.to_host()
            bad = sum(pl[i] != O.pmd_deflate(bytes(raw[off[i]:off[i] + lens[i]]), 6) for i in range(min(check, len(lens))))
            line += f" mismatches {bad}/{min(check, len(lens))}"
        print(line, flush=True)


lens = np.full(65536, 4096, dtype=np.uint32)
raw, off, ln = synth.make_batch("json", lens, seed=bench.SEED_C3)
if os.environ.get("EXACT_C3", "1") != "0":
    run("C3", raw, off, ln)
n4 = 65536
rng = np.random.default_rng(4)
r = np.arange(1, 257)
p = r ** -1.1
p /= p.sum()
zl = (256 * rng.choice(r, size=n4, p=p)).astype(np.uint32)
raw, off, ln = synth.make_batch("json", zl, seed=bench.SEED_C4)
run("C4-64Ki", raw, off, ln, check=256)
cpu("C4-64Ki", raw, off, ln)
