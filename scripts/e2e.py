"""End-to-end (PCIe-inclusive) rate: the path starts and ends in host memory
(Boost.Asio socket buffers), so this times pinned host -> device copy,
kernel, device -> host copy for the C2 inflate batch and the C3 deflate
batch, pipelined in chunks: one H2D stream, --depth compute streams, one D2H stream
for the inflate batch; the deflate batch runs each chunk's H2D, call and D2H
on one of --ddepth streams (the copies of both directions and the kernels
overlap; nothing in the loop waits on the device).  Reported in DESIGN.md; never the bench `value`.

    python scripts/e2e.py [--chunks 8] [--reps 5]

`*_copy_only_GiBps`: the same copies with no kernel (the PCIe bound of the
pipeline).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from beast_amd import pmd, synth  # noqa: E402


def chunk_views(buf, off, lens, nchunks):
    n = len(lens)
    per = (n + nchunks - 1) // nchunks
    out = []
    for c in range(nchunks):
        s, e = c * per, min(n, (c + 1) * per)
        base, end = int(off[s]), int(off[e - 1] + lens[e - 1])
        out.append((torch.from_numpy(np.ascontiguousarray(buf[base:end])).pin_memory(),
                    torch.from_numpy((off[s:e] - base).astype(np.int64)).pin_memory(),
                    torch.from_numpy(lens[s:e].astype(np.int32)).pin_memory(), e - s))
    return out


def run_pipeline(chunks, kernel, out_bytes_of, reps, depth=2):
    """Three engines: one stream copies the chunks in (H2D), `depth` streams
    run the batch calls (chunk i on stream i % depth, after its input's
    event), one stream copies the outputs back (D2H, after the chunk's
    kernel event), so the D2H of chunk i runs while later chunks decode and
    the copies of both directions overlap each other and the kernels.
    (Round 5's first version ran each chunk's H2D, call and D2H on one of 3
    streams, so a chunk's call waited for the D2H before it on that stream:
    26 GiB/s against a 41 GiB/s copy bound.)  Every device buffer is
    allocated up front, one per chunk, so nothing in the timed loop waits on
    the device."""
    dev = torch.device("cuda", 0)
    h2d, d2h = torch.cuda.Stream(), torch.cuda.Stream()
    comp = [torch.cuda.Stream() for _ in range(depth)]
    slots = [dict(d=torch.empty(c[0].numel() + 64, dtype=torch.uint8, device=dev),
                  o=torch.empty(c[3], dtype=torch.int64, device=dev),
                  l=torch.empty(c[3], dtype=torch.int32, device=dev),
                  out=torch.empty(out_bytes_of(c[3]) + 64, dtype=torch.uint8, device=dev)) for c in chunks]
    outs_h = [torch.empty(out_bytes_of(c[3]), dtype=torch.uint8).pin_memory() for c in chunks]
    lens_h = [torch.empty(c[3], dtype=torch.int32).pin_memory() for c in chunks]
    times = []
    for _ in range(reps + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ev_in, ev_k = [], []
        for i, (hd, ho, hl, n) in enumerate(chunks):
            sl = slots[i]
            with torch.cuda.stream(h2d):
                sl["d"][: hd.numel()].copy_(hd, non_blocking=True)
                sl["o"].copy_(ho, non_blocking=True)
                sl["l"].copy_(hl, non_blocking=True)
                e = torch.cuda.Event()
                e.record(h2d)
                ev_in.append(e)
        for i, (hd, ho, hl, n) in enumerate(chunks):
            sl = slots[i]
            s = comp[i % depth]
            s.wait_event(ev_in[i])
            with torch.cuda.stream(s):
                src = pmd.Batch(sl["d"], sl["o"], sl["l"])
                res = kernel(src, s, sl["out"], n)
                sl["keep"] = res
                e = torch.cuda.Event()
                e.record(s)
                ev_k.append(e)
        for i, (hd, ho, hl, n) in enumerate(chunks):
            d2h.wait_event(ev_k[i])
            with torch.cuda.stream(d2h):
                res = slots[i]["keep"]
                outs_h[i].copy_(res.out.data[: outs_h[i].numel()], non_blocking=True)
                lens_h[i].copy_(res.out.len, non_blocking=True)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    return sorted(times[1:])[len(times[1:]) // 2], outs_h, lens_h


def run_pipeline_inorder(chunks, kernel, out_bytes_of, reps, depth=3):
    """(Deflate: measured faster than the three-engine form, 33.9 vs 22-23
    GiB/s, profiles/r05zzn_e2e.log.)  Chunk i runs on stream i % depth: its H2D, its batch call, its D2H of
    the output and lengths.  Every device buffer is allocated up front (per
    stream) and the batch calls get their output slots, so nothing in the
    timed loop waits on the device: the H2D of chunk i + 1 and the D2H of
    chunk i run on different streams, i.e. on the two copy directions at
    once, beside the kernels."""
    dev = torch.device("cuda", 0)
    streams = [torch.cuda.Stream() for _ in range(depth)]
    maxin = max(c[0].numel() for c in chunks)
    maxn = max(c[3] for c in chunks)
    maxout = max(out_bytes_of(c[3]) for c in chunks)
    slots = [dict(d=torch.empty(maxin + 64, dtype=torch.uint8, device=dev),
                  o=torch.empty(maxn, dtype=torch.int64, device=dev),
                  l=torch.empty(maxn, dtype=torch.int32, device=dev),
                  out=torch.empty(maxout + 64, dtype=torch.uint8, device=dev)) for _ in streams]
    outs_h = [torch.empty(out_bytes_of(c[3]), dtype=torch.uint8).pin_memory() for c in chunks]
    lens_h = [torch.empty(c[3], dtype=torch.int32).pin_memory() for c in chunks]
    times = []
    for _ in range(reps + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i, (hd, ho, hl, n) in enumerate(chunks):
            s = streams[i % depth]
            sl = slots[i % depth]
            with torch.cuda.stream(s):
                sl["d"][: hd.numel()].copy_(hd, non_blocking=True)
                sl["o"][:n].copy_(ho, non_blocking=True)
                sl["l"][:n].copy_(hl, non_blocking=True)
                src = pmd.Batch(sl["d"], sl["o"][:n], sl["l"][:n])
                res = kernel(src, s, sl["out"], n)
                outs_h[i].copy_(res.out.data[: outs_h[i].numel()], non_blocking=True)
                lens_h[i].copy_(res.out.len, non_blocking=True)
                sl["keep"] = res
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    return sorted(times[1:])[len(times[1:]) // 2], outs_h, lens_h


def copy_only(chunks, out_bytes_of, reps):
    """The same H2D and D2H bytes on the same two copy streams with no kernel:
    what the PCIe link alone allows this pipeline (the e2e rate's bound)."""
    dev = torch.device("cuda", 0)
    h2d, d2h = torch.cuda.Stream(), torch.cuda.Stream()
    ins = [torch.empty(c[0].numel() + 64, dtype=torch.uint8, device=dev) for c in chunks]
    outs = [torch.zeros(out_bytes_of(c[3]) + 64, dtype=torch.uint8, device=dev) for c in chunks]
    outs_h = [torch.empty(out_bytes_of(c[3]), dtype=torch.uint8).pin_memory() for c in chunks]
    times = []
    for _ in range(reps + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i, (hd, ho, hl, n) in enumerate(chunks):
            with torch.cuda.stream(h2d):
                ins[i][: hd.numel()].copy_(hd, non_blocking=True)
            with torch.cuda.stream(d2h):
                outs_h[i].copy_(outs[i][: outs_h[i].numel()], non_blocking=True)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    return sorted(times[1:])[len(times[1:]) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunks", type=int, default=4)
    ap.add_argument("--dchunks", type=int, default=8, help="deflate chunks")
    ap.add_argument("--ddepth", type=int, default=3, help="deflate streams (chunk i's copies and call on stream i % ddepth)")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--depth", type=int, default=4, help="inflate compute streams")
    ap.add_argument("--msgs", type=int, default=bench.N_MSGS)
    a = ap.parse_args()
    n, mb = a.msgs, bench.MSG_BYTES
    lens = np.full(n, mb, dtype=np.uint32)
    res = {}

    # C2 inflate: compressed payloads in, 4 KiB messages out
    raw, roff, rlen = synth.make_batch("json", lens, seed=bench.SEED_C2)
    comp, coff, clen = bench.pack(bench.pmd_compress_host(raw, roff, rlen))
    chunks = chunk_views(comp, coff, clen, a.chunks)
    per = max(c[3] for c in chunks)
    dev = torch.device("cuda", 0)
    icap = torch.full((per,), mb, dtype=torch.int32, device=dev)
    ioff = pmd.slot_offsets(icap)
    t, outs, _ = run_pipeline(chunks, lambda src, s, out, k: pmd.inflate_batch(src, icap[:k], stream=s, out=out,
                                                                             out_off=ioff[:k]),
                              lambda k: k * mb, a.reps, a.depth)
    got = np.concatenate([o.numpy() for o in outs])
    res["inflate_e2e_GiBps"] = round(n * mb / (1 << 30) / t, 3)
    res["inflate_e2e_ok"] = bool(np.array_equal(got, raw[: n * mb]))
    res["inflate_h2d_bytes"] = int(comp.nbytes)
    tc = copy_only(chunks, lambda k: k * mb, a.reps)
    res["inflate_copy_only_GiBps"] = round(n * mb / (1 << 30) / tc, 3)

    # C3 deflate: messages in, payloads out (slots of upper_bound bytes)
    raw3, off3, len3 = synth.make_batch("json", lens, seed=bench.SEED_C3)
    ub = pmd.upper_bound(mb)
    slot = (ub + 15) // 16 * 16
    chunks3 = chunk_views(raw3, off3, len3, a.dchunks)
    per3 = max(c[3] for c in chunks3)
    dcap = torch.full((per3,), ub, dtype=torch.int32, device=dev)
    doff = pmd.slot_offsets(dcap)
    t3, outs3, lens3 = run_pipeline_inorder(chunks3, lambda src, s, out, k: pmd.deflate_batch(src, level=6, stream=s,
                                                                                     out_cap=dcap[:k], out=out,
                                                                                     out_off=doff[:k]),
                                    lambda k: k * slot, a.reps, a.ddepth)
    rt = [pmd.Batch(torch.from_numpy(o.numpy()), doff[: len(l)].cpu(), l) for o, l in zip(outs3, lens3)]
    ok3 = True
    import zlib
    for c, b in enumerate(rt[:1]):   # spot check: the first chunk's first 64 payloads inflate back (host zlib)
        for j in range(64):
            o, k = int(b.off[j]), int(b.len[j])
            d = zlib.decompressobj(-15)
            m = d.decompress(bytes(b.data[o:o + k].numpy()) + b"\x00\x00\xff\xff")
            ok3 = ok3 and m == bytes(raw3[off3[j]:off3[j] + len3[j]])
    res["deflate_e2e_spot_ok"] = bool(ok3)
    res["deflate_e2e_GiBps"] = round(n * mb / (1 << 30) / t3, 3)
    res["deflate_d2h_bytes"] = int(sum(int(x.numpy().sum()) for x in lens3))
    tc3 = copy_only(chunks3, lambda k: k * slot, a.reps)
    res["deflate_copy_only_GiBps"] = round(n * mb / (1 << 30) / tc3, 3)
    res["chunks"] = a.chunks
    res["compute_streams"] = a.depth
    res["deflate_chunks"] = a.dchunks
    res["deflate_compute_streams"] = a.ddepth
    print(json.dumps(res))


if __name__ == "__main__":
    main()
