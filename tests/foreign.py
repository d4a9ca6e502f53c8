"""Payloads from a foreign encoder (CPython's zlib) for the inflate parity tests."""
import random

from beast_amd import synth


def foreign_payloads(seed, count):
    """Payloads from another encoder (CPython's zlib, not the oracle's port of
    Beast's deflater) built from 1-6 pieces, each ended by a random flush:
    none, Z_BLOCK, Z_SYNC_FLUSH (an empty stored block mid-payload, which the
    block-parallel scan takes for a chunk marker), Z_FULL_FLUSH (the same and
    a fresh window); zlib's own strategies (filtered, Huffman-only, RLE, fixed)
    and memLevel / window sizes.  Returns (pmd payloads: last piece sync-flushed
    with 00 00 FF FF removed, raw payloads: Z_FINISH, originals)."""
    import zlib
    rng = random.Random(seed)
    flushes = [zlib.Z_NO_FLUSH, zlib.Z_BLOCK, zlib.Z_SYNC_FLUSH, zlib.Z_FULL_FLUSH]
    strategies = [zlib.Z_DEFAULT_STRATEGY, zlib.Z_FILTERED, zlib.Z_HUFFMAN_ONLY, zlib.Z_RLE, zlib.Z_FIXED]
    pmd_p, raw_p, orig = [], [], []
    for _ in range(count):
        kind = rng.choice(["json", "corpus1", "random", "binary", "zeros"])
        wb, lvl, mem = rng.randrange(9, 16), rng.randrange(0, 10), rng.randrange(1, 10)
        strat = rng.choice(strategies)
        pieces = []
        for _ in range(rng.randrange(1, 7)):
            size = rng.choice([0, 1, 100, 1500, 4096, 9000, 20000])
            data, _, _ = synth.make_batch(kind, [size], seed=rng.randrange(1 << 30))
            pieces.append((bytes(data[:size]), rng.choice(flushes)))
        for mode in ("pmd", "raw"):
            c = zlib.compressobj(lvl, zlib.DEFLATED, -wb, mem, strat)
            out = b""
            for k, (d, fl) in enumerate(pieces):
                out += c.compress(d)
                last = k == len(pieces) - 1
                if last:
                    out += c.flush(zlib.Z_SYNC_FLUSH if mode == "pmd" else zlib.Z_FINISH)
                elif fl != zlib.Z_NO_FLUSH:
                    out += c.flush(fl)
            if mode == "pmd":
                assert out.endswith(b"\x00\x00\xff\xff")
                pmd_p.append(out[:-4])
            else:
                raw_p.append(out)
        orig.append(b"".join(d for d, _ in pieces))
    return pmd_p, raw_p, orig

