"""Inflate time of one rank's shard of an 8-GPU split (shard 0 of 8) of
configs[3] (C4) and configs[4] (C5, L1), and of the whole batches, under
environment settings given as NAME=VALUE,... arguments (one child process
each, so the library reads them fresh):
    python scripts/diag_shards.py "" BPMD_LONG_SHARE_PCT=100 ...
"""
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def child(which):
    import torch
    import bench
    from beast_amd import pmd, shard, synth
    dev = torch.device("cuda", 0)
    for name in which.split(","):
        leg, part = name.split(":")
        if leg == "c4":
            lens_all, kind, seed, level = synth.zipf_sizes(bench.C4_MSGS, bench.SEED_C4), "json", bench.SEED_C4, 6
        else:
            lens_all, kind, seed, level = np.full(bench.C5_MSGS, 65536, np.uint32), "binary", bench.SEED_C5, 1
        a, b = (0, len(lens_all)) if part == "all" else shard.byte_balanced_ranges(lens_all, 8)[0]
        lens = lens_all[a:b]
        raw, off, ln = synth.make_batch(kind, lens, seed=seed, first=a)
        src = pmd.Batch(torch.from_numpy(raw).to(dev), torch.from_numpy(off.astype(np.int64)).to(dev),
                        torch.from_numpy(ln.astype(np.int32)).to(dev))
        del raw
        d = pmd.deflate_batch(src, level=level, mem_level=4)
        torch.cuda.synchronize()
        comp = pmd.Batch(d.out.data, d.out.off, d.out.len)
        rbuf = torch.empty_like(src.data)
        r = pmd.inflate_batch(comp, src.len, out=rbuf, out_off=src.off)
        torch.cuda.synchronize()
        total = int(lens.astype(np.int64).sum())
        ok = int((r.status != 0).sum()) == 0 and torch.equal(rbuf[:total], src.data[:total])
        ts = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            pmd.inflate_batch(comp, src.len, out=rbuf, out_off=src.off)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        t = float(np.median(ts))
        print(f"  {name:8s} msgs {len(lens):8d} inflate {t:8.3f} ms {total / 2**30 / (t / 1e3):8.2f} GiB/s ok {ok}",
              flush=True)
        del src, d, comp, rbuf, r
        torch.cuda.empty_cache()


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        return child(sys.argv[2])
    which = os.environ.get("WHICH", "c4:s8,c5:s8,c5:all")
    for spec in sys.argv[1:] or [""]:
        env = dict(os.environ)
        for kv in filter(None, spec.split(",")):
            k, v = kv.split("=")
            env[k] = v
        print(f"== {spec or 'default'}", flush=True)
        subprocess.run([sys.executable, __file__, "--child", which], env=env, check=True, timeout=400)


if __name__ == "__main__":
    main()
