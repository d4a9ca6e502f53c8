"""Token statistics of the bench's C2 payloads (host only, no GPU).

Decodes a sample of C2 messages with a small pure-Python raw-DEFLATE walker
that counts blocks, literals, matches, code lengths and the bits they use,
to size the inflate kernel's per-symbol budget.
Usage: python scripts/c2_token_stats.py [n_msgs]
"""
import os
import sys
import zlib
from collections import Counter

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from beast_amd import synth  # noqa: E402

SEED_C2 = 0x5EED0002


class Bits:
    def __init__(self, b):
        self.v = int.from_bytes(b, "little")
        self.p = 0
        self.n = 8 * len(b)

    def get(self, k):
        r = (self.v >> self.p) & ((1 << k) - 1)
        self.p += k
        return r


def build(lens):
    # canonical decode dict: (len, code) -> sym
    bl = Counter(l for l in lens if l)
    code, nxt = 0, {}
    for L in range(1, 16):
        code = (code + bl.get(L - 1, 0)) << 1
        nxt[L] = code
    d = {}
    for s, L in enumerate(lens):
        if L:
            d[(L, nxt[L])] = s
            nxt[L] += 1
    return d


def dec(bs, d):
    c = 0
    for L in range(1, 16):
        c = (c << 1) | bs.get(1)
        if (L, c) in d:
            return d[(L, c)], L
    raise ValueError("bad code")


LBASE = [3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258]
LEXT = [0] * 8 + [1] * 4 + [2] * 4 + [3] * 4 + [4] * 4 + [5] * 4 + [0]
DBASE = [1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537, 2049, 3073,
         4097, 6145, 8193, 12289, 16385, 24577]
DEXT = [0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13]


def walk(p, st):
    bs = Bits(p)
    while bs.p + 3 <= bs.n:
        last = bs.get(1)
        t = bs.get(2)
        st["blocks"] += 1
        st["btype"][t] += 1
        if t == 0:
            bs.p = (bs.p + 7) & ~7
            if bs.p + 32 > bs.n:
                break
            n = bs.get(16)
            bs.get(16)
            bs.p += 8 * n
            st["stored_bytes"] += n
        elif t in (1, 2):
            if t == 1:
                ll = [8] * 144 + [9] * 112 + [7] * 24 + [8] * 8
                dl = [5] * 30
            else:
                hlit = bs.get(5) + 257
                hdist = bs.get(5) + 1
                hclen = bs.get(4) + 4
                order = [16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15]
                cl = [0] * 19
                for i in range(hclen):
                    cl[order[i]] = bs.get(3)
                cd = build(cl)
                lens = []
                while len(lens) < hlit + hdist:
                    s, _ = dec(bs, cd)
                    if s < 16:
                        lens.append(s)
                    elif s == 16:
                        lens += [lens[-1]] * (3 + bs.get(2))
                    elif s == 17:
                        lens += [0] * (3 + bs.get(3))
                    else:
                        lens += [0] * (11 + bs.get(7))
                ll, dl = lens[:hlit], lens[hlit:]
                st["hdr_bits"] += 0
            ld, dd = build(ll), build(dl)
            while True:
                s, L = dec(bs, ld)
                st["litlen_L"][L] += 1
                if s < 256:
                    st["lit"] += 1
                elif s == 256:
                    break
                else:
                    i = s - 257
                    ml = LBASE[i] + bs.get(LEXT[i])
                    ds, Ld = dec(bs, dd)
                    st["dist_L"][Ld] += 1
                    dist = DBASE[ds] + bs.get(DEXT[ds])
                    st["match"] += 1
                    st["mlen"] += ml
                    st["dist_lt8"] += dist < 8
                    st["dist_sum"] += dist
        else:
            raise ValueError("type 3")
        if last:
            break
        if bs.n - bs.p < 10:
            break
    # runs of literals before each match
    return st


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    lens = np.full(n, 4096, dtype=np.uint32)
    raw, off, ln = synth.make_batch("json", lens, seed=SEED_C2)
    st = {"blocks": 0, "btype": Counter(), "stored_bytes": 0, "lit": 0, "match": 0, "mlen": 0,
          "litlen_L": Counter(), "dist_L": Counter(), "dist_lt8": 0, "dist_sum": 0, "hdr_bits": 0}
    comp = 0
    per_msg_sym = []
    for i in range(n):
        o = int(off[i])
        c = zlib.compressobj(6, zlib.DEFLATED, -15, 4)
        p = c.compress(raw[o:o + 4096].tobytes()) + c.flush(zlib.Z_BLOCK) + c.flush(zlib.Z_SYNC_FLUSH)
        p = p[:-4]
        comp += len(p)
        before = st["lit"] + st["match"]
        walk(p, st)
        per_msg_sym.append(st["lit"] + st["match"] - before)
    print(f"messages {n}  comp bytes/msg {comp / n:.1f}")
    print(f"blocks/msg {st['blocks'] / n:.2f}  types {dict(st['btype'])}")
    print(f"literals/msg {st['lit'] / n:.1f}  matches/msg {st['match'] / n:.1f}  "
          f"symbols/msg {(st['lit'] + st['match']) / n:.1f}  (max {max(per_msg_sym)}, min {min(per_msg_sym)})")
    print(f"mean match len {st['mlen'] / max(st['match'], 1):.2f}  mean dist {st['dist_sum'] / max(st['match'], 1):.1f}"
          f"  dist<8 share {st['dist_lt8'] / max(st['match'], 1):.3f}")
    tot = sum(st["litlen_L"].values())
    print("lit/len code lengths:", {L: round(c / tot, 3) for L, c in sorted(st["litlen_L"].items())})
    totd = sum(st["dist_L"].values())
    print("dist code lengths:", {L: round(c / totd, 3) for L, c in sorted(st["dist_L"].items())})


if __name__ == "__main__":
    main()
