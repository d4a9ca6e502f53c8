// deflate_model.cpp -- host model of the GPU deflate algorithm (design tool
// and bit-exact expectation for the kernel).  Build:
//   g++ -O2 -shared -fPIC -I beast_amd/csrc scripts/deflate_model.cpp -o /tmp/libdmodel.so
//
// Per message: chunks of C bytes with H bytes of history in the window; per
// chunk, hash chains over the window, 64 lane segments parsed independently
// (greedy or lazy per the level table), segment-boundary repair by a prefix
// max of segment end positions, one block per chunk (stored / fixed /
// dynamic, smallest), pmd tail (empty stored block header bits 000 + pad).
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
#include <vector>

#include "lz_core.h"

using namespace lz;

struct Params {
    int level, wbits, strategy;     // strategy: 0 normal 1 filtered 2 huffman 3 rle 4 fixed
    int chunk, hist, hbits, lanes, min_seg;
    int chain_cap;                  // 0 = level table value
};

struct Tok { uint32_t pos, len, dist; };   // len 1 = literal

struct BitW {
    std::vector<uint8_t>* out;
    uint64_t acc = 0;
    int n = 0;
    void put(uint32_t v, int b)
    {
        acc |= (uint64_t)v << n;
        n += b;
        while (n >= 8) { out->push_back((uint8_t)acc); acc >>= 8; n -= 8; }
    }
    void align() { if (n) put(0, 8 - n); }
};

static unsigned match_len(const uint8_t* w, unsigned a, unsigned b, unsigned maxl)
{
    unsigned l = 0;
    while (l < maxl && w[a + l] == w[b + l]) ++l;
    return l;
}

// longest_match restatement (deflate_stream.ipp:1747-1844), window-relative
static unsigned longest(const uint8_t* w, const int32_t* prev, unsigned p, unsigned end, unsigned prev_len,
                        const Level& L, unsigned max_dist, unsigned chain_cap, unsigned& best_dist)
{
    unsigned chain = chain_cap ? chain_cap : L.chain;
    if (prev_len >= L.good) chain >>= 2;
    unsigned maxl = end - p < (unsigned)MAX_MATCH ? end - p : MAX_MATCH;
    unsigned nice = L.nice < maxl ? L.nice : maxl;
    unsigned best = prev_len;
    int c = prev[p];
    while (c >= 0 && p - (unsigned)c <= max_dist && chain-- > 0) {
        if (best < maxl && w[c + best] == w[p + best] && w[c] == w[p]) {
            unsigned l = match_len(w, c, p, maxl);
            if (l > best) {
                best = l;
                best_dist = p - c;
                if (l >= nice) break;
            }
        }
        c = prev[c];
    }
    return best;
}

static void parse_segment(const uint8_t* w, const int32_t* prev, unsigned a, unsigned b, unsigned end,
                          const Params& P, const Level& L, unsigned max_dist, std::vector<Tok>& toks)
{
    unsigned p = a;
    const bool lazy = L.parser == P_SLOW;
    auto find = [&](unsigned q, unsigned thr, unsigned& d) -> unsigned {
        if (P.strategy == 2 || q + MIN_MATCH > end) return thr;
        if (P.strategy == 3) {   // rle: distance 1 only
            if (q == 0) return thr;
            unsigned maxl = end - q < (unsigned)MAX_MATCH ? end - q : MAX_MATCH;
            unsigned l = 0;
            while (l < maxl && w[q + l] == w[q - 1]) ++l;
            if (l > thr && l >= MIN_MATCH) { d = 1; return l; }
            return thr;
        }
        unsigned l = longest(w, prev, q, end, thr, L, max_dist, P.chain_cap, d);
        if (l <= 5 && l > thr && (P.strategy == 1 || (l == MIN_MATCH && d > TOO_FAR))) return thr;
        return l;
    };
    unsigned d0 = 0;
    unsigned l0 = p < b ? find(p, MIN_MATCH - 1, d0) : 0;
    while (p < b) {
        if (l0 < MIN_MATCH) {
            toks.push_back({p, 1, 0});
            ++p;
            if (p < b) l0 = find(p, MIN_MATCH - 1, d0);
            continue;
        }
        if (lazy && l0 < L.lazy && p + 1 < end) {
            unsigned d1 = 0;
            unsigned l1 = find(p + 1, l0, d1);
            if (l1 > l0) {
                toks.push_back({p, 1, 0});
                ++p;
                l0 = l1;
                d0 = d1;
                continue;
            }
        }
        toks.push_back({p, l0, d0});
        p += l0;
        if (p < b) l0 = find(p, MIN_MATCH - 1, d0);
    }
}

struct Coder {
    uint8_t llen[N_LCODES + 2], dlen[N_DCODES];   // fixed code has 288 lit/len symbols
    uint16_t lcode[N_LCODES + 2], dcode[N_DCODES];
};

static void put_tokens(BitW& bw, const std::vector<Tok>& toks, const uint8_t* w, const Coder& c)
{
    for (const Tok& t : toks) {
        if (t.len == 1) { bw.put(c.lcode[w[t.pos]], c.llen[w[t.pos]]); continue; }
        unsigned s, nx, xv;
        len_code(t.len, s, nx, xv);
        bw.put(c.lcode[s], c.llen[s]);
        if (nx) bw.put(xv, nx);
        dist_code(t.dist, s, nx, xv);
        bw.put(c.dcode[s], c.dlen[s]);
        if (nx) bw.put(xv, nx);
    }
    bw.put(c.lcode[EOB], c.llen[EOB]);
}

// Encode one message; returns the pmd payload (tail stripped).
static std::vector<uint8_t> encode(const uint8_t* msg, unsigned n, const Params& P)
{
    std::vector<uint8_t> out;
    BitW bw;
    bw.out = &out;
    Level L = level_params(P.level);
    Params Q = P;   // the kernel's chain limit for this message
    if (!Q.chain_cap) Q.chain_cap = (int)gpu_chain(P.level, n <= (unsigned)P.chunk);
    unsigned wsize = 1u << (P.wbits < 9 ? 9 : P.wbits);
    unsigned max_dist = wsize - LOOKAHEAD_MIN;
    std::vector<int32_t> prev;
    std::vector<int32_t> head(1u << P.hbits);
    // the stitch's marker before every Huffman-coded chunk but the first, and
    // before chunk 1 whatever its kind: an empty stored block, so the block
    // starts on a byte
    auto marker = [&](unsigned base) {
        if (!base) return;
        bw.put(0, 3);
        bw.align();
        bw.put(0, 16);
        bw.put(0xFFFF, 16);
    };
    for (unsigned base = 0; base < n; base += P.chunk) {
        unsigned cend = base + P.chunk < n ? base + P.chunk : n;
        unsigned wb = base > (unsigned)P.hist ? base - P.hist : 0;
        const uint8_t* w = msg + wb;
        unsigned wn = cend - wb, a0 = base - wb;
        std::vector<Tok> toks;
        bool chunk_incomp = false;
        if (L.parser != P_STORED) {
            prev.assign(wn, -1);
            std::fill(head.begin(), head.end(), -1);
            for (unsigned q = 0; q + MIN_MATCH <= wn; ++q) {
                uint32_t x = w[q] | (w[q + 1] << 8) | (w[q + 2] << 16) | (q + 3 < wn ? (uint32_t)w[q + 3] << 24 : 0u);
                uint32_t h = chain_hash(x, wn - q, P.hbits);
                prev[q] = head[h];
                head[h] = (int32_t)q;
            }
            // incompressible chunk: all literals, no parse (lz_core.h incompressible)
            bool no_parse = false;
            if (INCOMP_DEN && P.strategy != 2 && P.strategy != 3) {
                unsigned hits = 0;
                for (unsigned q = a0; q + 4 <= wn; q += INCOMP_STRIDE)
                    hits += prev[q] >= 0 && memcmp(w + prev[q], w + q, 4) == 0;
                no_parse = incompressible(hits, wn - a0);
            }
            chunk_incomp = no_parse;
            unsigned len = wn - a0;
            unsigned seg = (len + P.lanes - 1) / P.lanes;
            const unsigned min_seg = a0 ? 32u : (unsigned)P.min_seg;   // (pmd_deflate.hip: history keeps 32)
            if (seg < min_seg) seg = min_seg;
            unsigned E = a0;
            for (unsigned s = a0; s < wn; s += seg) {
                unsigned b = s + seg < wn ? s + seg : wn;
                std::vector<Tok> lt;
                if (no_parse)
                    for (unsigned q = s; q < b; ++q) lt.push_back({q, 1, 0});
                else
                    parse_segment(w, prev.data(), s, b, wn, Q, L, max_dist, lt);
                // boundary repair against the previous segments' end E
                for (const Tok& t : lt) {
                    if (t.pos + t.len <= E) continue;
                    if (t.pos < E) {
                        unsigned r = t.pos + t.len - E;
                        if (t.len > 1 && r >= MIN_MATCH) toks.push_back({E, r, t.dist});
                        else for (unsigned q = E; q < t.pos + t.len; ++q) toks.push_back({q, 1, 0});
                    } else {
                        toks.push_back(t);
                    }
                }
                unsigned own = lt.empty() ? s : lt.back().pos + lt.back().len;
                if (own > E) E = own;
            }
        }
        // block choice (deflate_stream.ipp:1425-1518)
        uint32_t lf[N_LCODES] = {0}, df[N_DCODES] = {0};
        for (const Tok& t : toks) {
            if (t.len == 1) { lf[w[t.pos]]++; continue; }
            unsigned s, nx, xv;
            len_code(t.len, s, nx, xv);
            lf[s]++;
            dist_code(t.dist, s, nx, xv);
            df[s]++;
        }
        lf[EOB] = 1;
        Coder dyn, fix;
        HuffScratch S;
        huff_lengths_host(lf, N_LCODES, MAX_BITS, dyn.llen, S, true);
        huff_lengths_host(df, N_DCODES, MAX_BITS, dyn.dlen, S);
        int lcodes = N_LCODES, dcodes = N_DCODES;
        while (lcodes > 257 && dyn.llen[lcodes - 1] == 0) --lcodes;
        while (dcodes > 1 && dyn.dlen[dcodes - 1] == 0) --dcodes;
        // code-length alphabet
        std::vector<uint8_t> all(dyn.llen, dyn.llen + lcodes);
        all.insert(all.end(), dyn.dlen, dyn.dlen + dcodes);
        uint32_t bf[N_BLCODES] = {0};
        auto getl = [&](int i) { return (int)dyn.llen[i]; };
        auto getd = [&](int i) { return (int)dyn.dlen[i]; };
        auto cnt = [&](int s, int, int) { bf[s]++; };
        rle_lengths(getl, lcodes, cnt);
        rle_lengths(getd, dcodes, cnt);
        uint8_t bll[N_BLCODES];
        uint16_t blc[N_BLCODES];
        huff_lengths_host(bf, N_BLCODES, MAX_BL_BITS, bll, S);
        canonical_codes_host(bll, N_BLCODES, blc);
        int blcodes = N_BLCODES;
        while (blcodes > 4 && bll[bl_order(blcodes - 1)] == 0) --blcodes;
        uint64_t dyn_bits = 3 + 5 + 5 + 4 + 3 * blcodes, fix_bits = 3;
        for (int s = 0; s < N_BLCODES; ++s) dyn_bits += (uint64_t)bf[s] * (bll[s] + (s == 16 ? 2 : s == 17 ? 3 : s == 18 ? 7 : 0));
        for (int s = 0; s < N_LCODES; ++s) {
            unsigned x = s > 256 ? len_extra_bits(s) : 0;
            dyn_bits += (uint64_t)lf[s] * (dyn.llen[s] + x);
            fix_bits += (uint64_t)lf[s] * (fixed_lit_len(s) + x);
        }
        for (int s = 0; s < N_DCODES; ++s) {
            dyn_bits += (uint64_t)df[s] * (dyn.dlen[s] + dist_extra_bits(s));
            fix_bits += (uint64_t)df[s] * (5 + dist_extra_bits(s));
        }
        unsigned clen = cend - base;
        uint64_t opt_b = (dyn_bits + 7) >> 3, fix_b = (fix_bits + 7) >> 3;
        if (P.strategy == 4) opt_b = fix_b + 1;
        // an incompressible chunk of a multi-chunk message: stored outright
        // (lz_core.h INCOMP_STORED)
        if (L.parser == P_STORED || (INCOMP_STORED && chunk_incomp && n > (unsigned)P.chunk) ||
            chunk_stored(clen, opt_b < fix_b ? opt_b : fix_b, n > (unsigned)P.chunk)) {
            if (base == (unsigned)P.chunk) marker(base);   // chunk 1 carries a marker whatever its kind
            bw.put(0, 3);
            bw.align();
            bw.put(clen & 0xFFFF, 16);
            bw.put(~clen & 0xFFFF, 16);
            for (unsigned q = 0; q < clen; ++q) bw.put(msg[base + q], 8);
        } else if (fix_b <= opt_b) {
            marker(base);
            for (int s = 0; s < N_LCODES + 2; ++s) fix.llen[s] = (uint8_t)fixed_lit_len(s);
            for (int s = 0; s < N_DCODES; ++s) fix.dlen[s] = 5;
            canonical_codes_host(fix.llen, N_LCODES + 2, fix.lcode);
            canonical_codes_host(fix.dlen, N_DCODES, fix.dcode);
            bw.put(1 << 1, 3);
            put_tokens(bw, toks, w, fix);
        } else {
            canonical_codes_host(dyn.llen, N_LCODES, dyn.lcode);
            canonical_codes_host(dyn.dlen, N_DCODES, dyn.dcode);
            marker(base);
            bw.put(2 << 1, 3);
            bw.put(lcodes - 257, 5);
            bw.put(dcodes - 1, 5);
            bw.put(blcodes - 4, 4);
            for (int i = 0; i < blcodes; ++i) bw.put(bll[bl_order(i)], 3);
            auto emit = [&](int s, int nx, int xv) { bw.put(blc[s], bll[s]); if (nx) bw.put(xv, nx); };
            rle_lengths(getl, lcodes, emit);
            rle_lengths(getd, dcodes, emit);
            put_tokens(bw, toks, w, dyn);
        }
    }
    // pmd tail: Flush::sync's empty stored block minus 00 00 FF FF
    bw.put(0, 3);
    bw.align();
    return out;
}

extern "C" int64_t dmodel_batch(const uint8_t* data, const uint64_t* off, const uint32_t* len, uint32_t n,
                                int level, int wbits, int strategy, int chunk, int hist, int hbits, int lanes,
                                int min_seg, int chain_cap, uint8_t* out, uint64_t out_cap, uint64_t* out_off,
                                uint32_t* out_len)
{
    Params P{level, wbits, strategy, chunk, hist, hbits, lanes, min_seg, chain_cap};
    uint64_t pos = 0;
    for (uint32_t i = 0; i < n; ++i) {
        std::vector<uint8_t> e = encode(data + off[i], len[i], P);
        if (pos + e.size() > out_cap) return -1;
        memcpy(out + pos, e.data(), e.size());
        out_off[i] = pos;
        out_len[i] = (uint32_t)e.size();
        pos += e.size();
    }
    return (int64_t)pos;
}

// Self-check hook: code-length run-length coding of `lens[0..n)` by the
// serial state machine and by the per-run closed form the kernel uses;
// writes both symbol streams (sym | extra << 8) and returns 1 if equal.
extern "C" int dmodel_rle_check(const uint8_t* lens, int n, uint32_t* serial, uint32_t* runs, int* ns, int* nr)
{
    int a = 0, b = 0;
    auto get = [&](int i) { return (int)lens[i]; };
    rle_lengths(get, n, [&](int s, int, int x) { serial[a++] = (uint32_t)s | ((uint32_t)x << 8); });
    unsigned cnt = 0;
    for (int i = 0; i < n;) {
        int j = i + 1;
        while (j < n && lens[j] == lens[i]) ++j;
        cnt += rle_run_count(lens[i], (unsigned)(j - i));
        rle_run(lens[i], (unsigned)(j - i), [&](int s, int, int x) { runs[b++] = (uint32_t)s | ((uint32_t)x << 8); });
        i = j;
    }
    *ns = a;
    *nr = b;
    if (a != b || (unsigned)b != cnt) return 0;
    for (int i = 0; i < a; ++i)
        if (serial[i] != runs[i]) return 0;
    return 1;
}

// history bytes before each chunk of a long message (the kernel's value)
extern "C" int dmodel_chunk_hist(int level) { return (int)chunk_hist(level); }
