"""C4 at 8 GPUs, one shard on this GPU: inflate time of shard k (default the
first) with the long-payload split on/off and the wave kernel's round modes,
and the number of payloads the split sends to the wave kernel.
    python scripts/diag_c4_shard.py [--parts 8] [--shard 0]
"""
import argparse
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def child(args):
    import torch
    from beast_amd import pmd, shard, synth
    import bench
    lens_all = synth.zipf_sizes(bench.C4_MSGS, bench.SEED_C4)
    a, b = shard.byte_balanced_ranges(lens_all, args.parts)[args.shard]
    lens = lens_all[a:b]
    raw, off, ln = synth.make_batch("json", lens, seed=bench.SEED_C4, first=a)
    dev = torch.device("cuda", 0)
    src = pmd.Batch(torch.from_numpy(raw).to(dev), torch.from_numpy(off.astype(np.int64)).to(dev),
                    torch.from_numpy(ln.astype(np.int32)).to(dev))
    d = pmd.deflate_batch(src, level=6, mem_level=4)
    torch.cuda.synchronize()
    clen = d.out.len.cpu().numpy().astype(np.int64)
    thr = max(4096, 2 * int(clen.sum()) // 65536)
    thr64 = (thr + 63) >> 6
    nlong = int(((clen >> 6) > thr64).sum())
    comp = pmd.Batch(d.out.data, d.out.off, d.out.len)
    pmd.lib().bpmd_diag_set_wave_walk(int(os.environ.get("WALK", "0")))
    for _ in range(2):
        r = pmd.inflate_batch(comp, src.len)
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        r = pmd.inflate_batch(comp, src.len)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ok = int((r.status != 0).sum()) == 0
    print(f"parts {args.parts} shard {args.shard} msgs {len(lens)} long {nlong} (thr {thr} B, max comp {clen.max()}) "
          f"LONG={os.environ.get('BPMD_INFLATE_LONG', '1')} WALK={os.environ.get('WALK', '0')} "
          f"inflate {np.median(ts) * 1e3:.2f} ms ok {ok}", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--parts", type=int, default=8)
    ap.add_argument("--shard", type=int, default=0)
    ap.add_argument("--child", action="store_true")
    args = ap.parse_args()
    if args.child:
        return child(args)
    for env in ({"BPMD_INFLATE_LONG": "0"}, {"BPMD_INFLATE_LONG": "1"}, {"BPMD_INFLATE_LONG": "1", "WALK": "2"},
                {"BPMD_INFLATE_LONG": "1", "WALK": "1"}):
        e = dict(os.environ, **env)
        subprocess.run([sys.executable, __file__, "--child", "--parts", str(args.parts), "--shard", str(args.shard)],
                       env=e, check=True, timeout=300)


if __name__ == "__main__":
    main()
