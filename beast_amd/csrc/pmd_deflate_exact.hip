// pmd_deflate_exact.hip -- exact mode of the batch deflater (BPMD_F_EXACT,
// SURVEY.md §8(f) N4): payloads bit-identical to Beast's deflate_stream
// (include/boost/beast/zlib/detail/deflate_stream.ipp) under the
// permessage-deflate call sequence of impl_base<true>::deflate
// (websocket/detail/impl_base.hpp:85-154: Flush::none over the message,
// Flush::block, Flush::sync, 00 00 FF FF dropped) with a reset per message.
//
// Exactness needs Beast's serial decisions: the lazy parse (each match
// decision depends on the previous one), hash chains in insertion order,
// blocks cut when the symbol buffer fills (lit_bufsize - 1 symbols),
// Huffman trees from zlib's heap with its depth tie-break, the
// stored/fixed/dynamic choice, and even the bytes a match comparison sees
// past the end of the data after a window slide.  So one WAVE runs one
// message's state machine as wave-uniform code, and the lanes share the
// bulk work inside it: the 256-byte match comparisons of longest_match
// (64 bytes per step, first mismatch by ballot), window fills and slides,
// table clears.  The window / prev / head arrays live in LDS for messages
// of up to 4 KiB and up to 8 KiB at memLevel <= 5 (tiers 0 and 1) and in a
// per-wave global workspace otherwise (tier 2); the code is the same
// through generic pointers.  Tree construction uses per-wave LDS in all.
//
// Reference map: level table deflate_stream.hpp:571-590; reset / init
// deflate_stream.ipp:227-265, 595-737; fill_window 1520-1669; longest_match
// 1747-1844; f_stored 1856-1924, f_fast 1932-2039, f_slow 2045-2184, f_rle
// 2190-2270, f_huff 2276-2324; tally 1396-1418; tr_flush_block 1425-1518;
// build_tree / gen_bitlen / gen_codes 115-141, 744-973; scan_tree /
// send_tree / build_bl_tree / send_all_trees 978-1180; compress_block
// 1184-1238; stored block / bi_windup 1284-1394; doWrite 357-499.
#include "pmd_common.h"

namespace bpmd {
namespace dx {

enum : int {
    NLIT = 256, NLENC = 29, NLC = NLIT + 1 + NLENC, NDC = 30, NBL = 19, HEAPN = 2 * NLC + 1,
    MAXB = 15, MAXBL = 7, MINM = 3, MAXM = 258, EOBS = 256, TOO_FAR = 4096, LOOK = MAXM + MINM + 1,
    WINIT = MAXM, REP36 = 16, REPZ310 = 17, REPZ11 = 18
};
enum : int { FL_NONE = 0, FL_BLOCK = 1, FL_SYNC = 3 };
enum : int { BS_NEED_MORE = 0, BS_BLOCK_DONE = 1 };
enum : int { PA_STORED = 0, PA_FAST = 1, PA_SLOW = 2 };

__constant__ static const uint8_t kXl[NLENC] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2,
                                                2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ static const uint8_t kXd[NDC] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6,
                                              6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
__constant__ static const uint8_t kXb[NBL] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 2, 3, 7};
__constant__ static const uint8_t kBlOrder[NBL] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

struct Lvl {
    uint32_t good, lazy, nice, chain;
    int parser;
};
__device__ __forceinline__ Lvl level_row(int l)
{
    switch (l) {
    case 0: return {0, 0, 0, 0, PA_STORED};
    case 1: return {4, 4, 8, 4, PA_FAST};
    case 2: return {4, 5, 16, 8, PA_FAST};
    case 3: return {4, 6, 32, 32, PA_FAST};
    case 4: return {4, 4, 16, 16, PA_SLOW};
    case 5: return {8, 16, 32, 32, PA_SLOW};
    case 6: return {8, 16, 128, 128, PA_SLOW};
    case 7: return {8, 32, 128, 256, PA_SLOW};
    case 8: return {32, 128, 258, 1024, PA_SLOW};
    default: return {32, 258, 258, 4096, PA_SLOW};
    }
}

// length code of (length - 3), distance code of (distance - 1), and their bases
__device__ __forceinline__ uint32_t len_code(uint32_t m)
{
    if (m < 8) return m;
    if (m == 255) return 28;
    const uint32_t x = 29u - __builtin_clz(m);   // floor(log2 m) - 2
    return 4 * x + 4 + ((m >> x) & 3u);
}
__device__ __forceinline__ uint32_t len_base(uint32_t c)
{
    if (c < 8) return c;
    if (c == 28) return 255;
    return (4u + (c & 3u)) << ((c - 4) >> 2);
}
__device__ __forceinline__ uint32_t dist_code(uint32_t d)
{
    if (d < 4) return d;
    const uint32_t e = 31u - __builtin_clz(d);
    return 2 * e + ((d >> (e - 1)) & 1u);
}
__device__ __forceinline__ uint32_t dist_base(uint32_t c) { return c < 4 ? c : (2u + (c & 1u)) << ((c >> 1) - 1); }
__device__ __forceinline__ uint32_t rev_bits(uint32_t code, uint32_t len) { return __builtin_bitreverse32(code) >> (32 - len); }

// the fixed trees (deflate_stream.ipp:143-225): lengths and bit-reversed codes
__device__ __forceinline__ uint32_t fix_llen(uint32_t n) { return n < 144 ? 8u : n < 256 ? 9u : n < 280 ? 7u : 8u; }
__device__ __forceinline__ uint32_t fix_lcode(uint32_t n)
{
    if (n < 144) return rev_bits(0x30u + n, 8);
    if (n < 256) return rev_bits(0x190u + n - 144, 9);
    if (n < 280) return rev_bits(n - 256, 7);
    return rev_bits(0xc0u + n - 280, 8);
}

struct Node {
    uint16_t f;   // frequency, then the (bit-reversed) code
    uint16_t l;   // parent, then the code length
};

// per-wave tree workspace (LDS)
struct Trees {
    Node lt[HEAPN];
    Node dt[2 * NDC + 1];
    Node bt[2 * NBL + 1];
    int16_t heap[HEAPN];
    uint8_t depth[HEAPN];
    uint16_t bl_count[MAXB + 1];
};

// tree descriptor: kind 0 literal/length, 1 distance, 2 bit lengths
struct TDesc {
    Node* dyn;
    int kind, elems, maxlen, max_code;
};

__device__ __forceinline__ void mem_fence() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); }
// Every lane holds the same deflater state; U() tells the compiler so (the
// first active lane's copy), which keeps the serial state machine on scalar
// registers and scalar branches instead of exec-masked divergent loops.
__device__ __forceinline__ uint32_t U(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }


// LSB-first bit sink into the output slot; bytes past cap are counted, not stored
struct Bits {
    uint8_t* out;
    uint32_t cap, key;
    uint64_t acc;
    uint32_t nacc, opos;
    __device__ void byte(uint32_t b)
    {
        if (lane_id() == 0 && opos < cap) out[opos] = (uint8_t)b;
        ++opos;
    }
    __device__ void put(uint32_t v, uint32_t n)
    {
        acc |= (uint64_t)v << nacc;
        nacc += n;
        while (nacc >= 8) {
            byte((uint32_t)acc & 0xffu);
            acc >>= 8;
            nacc -= 8;
        }
    }
    __device__ void windup()
    {
        if (nacc) byte((uint32_t)acc & 0xffu);
        acc = 0;
        nacc = 0;
    }
    __device__ uint32_t bytes_done() const { return opos; }   // whole bytes (nacc < 8)
};

struct Cfg {
    int level, strategy;
    uint32_t wbits, hbits, lit_bufsize;
};

// one block's Huffman coding and bit emission (tr_flush_block and below),
// called when the symbol buffer fills or a flush ends: out of line, on a
// private copy, so the parser's state stays in registers
struct Blk {
    Trees* T;
    uint8_t* syms;
    const uint8_t* win;
    int level, strategy;
    uint32_t sym_next;
    int32_t block_start;
    uint32_t opt_len, static_len;
    Bits bw;
    TDesc ld, dd, bd;

    // ------------------------------------------------------------ trees
    __device__ void reset_block()
    {
        for (int n = (int)lane_id(); n < NLC; n += WAVE) T->lt[n].f = 0;
        for (int n = (int)lane_id(); n < NDC; n += WAVE) T->dt[n].f = 0;
        for (int n = (int)lane_id(); n < NBL; n += WAVE) T->bt[n].f = 0;
        mem_fence();
        if (lane_id() == 0) T->lt[EOBS].f = 1;
        mem_fence();
        opt_len = static_len = 0;
    }
    __device__ uint32_t stat_len(const TDesc& d, int n) const { return d.kind == 0 ? fix_llen(n) : 5u; }
    __device__ uint32_t xbits(const TDesc& d, int n) const
    {
        if (d.kind == 0) return n >= NLIT + 1 ? kXl[n - (NLIT + 1)] : 0u;
        if (d.kind == 1) return kXd[n];
        return kXb[n];
    }
    __device__ bool smaller(const Node* t, int a, int b) const
    {
        const uint32_t fa = U(t[a].f), fb = U(t[b].f);
        return fa < fb || (fa == fb && U(T->depth[a]) <= U(T->depth[b]));
    }
    __device__ void sift(const Node* t, int k, int heap_len)
    {
        const int v = (int)U((uint32_t)(int)T->heap[k]);
        int j = k << 1;
        while (j <= heap_len) {
            if (j < heap_len && smaller(t, (int)U((uint32_t)(int)T->heap[j + 1]), (int)U((uint32_t)(int)T->heap[j]))) ++j;
            const int hj = (int)U((uint32_t)(int)T->heap[j]);
            if (smaller(t, v, hj)) break;
            T->heap[k] = (int16_t)hj;
            k = j;
            j <<= 1;
        }
        T->heap[k] = (int16_t)v;
    }
    // gen_bitlen (deflate_stream.ipp:786-873)
    __device__ void gen_bitlen(TDesc& d, int heap_max)
    {
        Node* t = d.dyn;
        for (int b = 0; b <= MAXB; ++b) T->bl_count[b] = 0;
        t[U((uint32_t)(int)T->heap[heap_max])].l = 0;
        int overflow = 0, h;
        for (h = heap_max + 1; h < HEAPN; ++h) {
            const int n = (int)U((uint32_t)(int)T->heap[h]);
            int bits = (int)U(t[U(t[n].l)].l) + 1;
            if (bits > d.maxlen) {
                bits = d.maxlen;
                ++overflow;
            }
            t[n].l = (uint16_t)bits;
            if (n > d.max_code) continue;
            T->bl_count[bits]++;
            const uint32_t xb = xbits(d, n);
            const uint32_t f = U(t[n].f);
            opt_len += f * ((uint32_t)bits + xb);
            if (d.kind != 2) static_len += f * (stat_len(d, n) + xb);
        }
        if (overflow == 0) return;
        do {
            int bits = d.maxlen - 1;
            while (U(T->bl_count[bits]) == 0) --bits;
            T->bl_count[bits]--;
            T->bl_count[bits + 1] += 2;
            T->bl_count[d.maxlen]--;
            overflow -= 2;
        } while (overflow > 0);
        for (int bits = d.maxlen; bits != 0; --bits) {
            int n = (int)U(T->bl_count[bits]);
            while (n != 0) {
                const int m = (int)U((uint32_t)(int)T->heap[--h]);
                if (m > d.max_code) continue;
                const int lm = (int)U(t[m].l);
                if (lm != bits) {
                    opt_len += (uint32_t)(((int32_t)bits - (int32_t)lm) * (int32_t)U(t[m].f));
                    t[m].l = (uint16_t)bits;
                }
                --n;
            }
        }
    }
    // gen_codes (deflate_stream.ipp:115-141)
    __device__ void gen_codes(Node* t, int max_code)
    {
        uint32_t next[MAXB + 1];
        uint32_t code = 0;
        for (int b = 1; b <= MAXB; ++b) {
            code = (code + U(T->bl_count[b - 1])) << 1;
            next[b] = code;
        }
        for (int n = 0; n <= max_code; ++n) {
            const uint32_t l = U(t[n].l);
            if (l == 0) continue;
            uint32_t c = 0;
#pragma unroll
            for (int b = 1; b <= MAXB; ++b)
                if ((uint32_t)b == l) c = next[b]++;
            t[n].f = (uint16_t)rev_bits(c, l);
        }
    }
    // build_tree (deflate_stream.ipp:888-973)
    __device__ void build_tree(TDesc& d)
    {
        Node* t = d.dyn;
        int heap_len = 0, heap_max = HEAPN, max_code = -1;
        for (int n = 0; n < d.elems; ++n) {
            if (U(t[n].f) != 0) {
                T->heap[++heap_len] = (int16_t)n;
                max_code = n;
                T->depth[n] = 0;
            } else {
                t[n].l = 0;
            }
        }
        while (heap_len < 2) {
            const int node = max_code < 2 ? ++max_code : 0;
            T->heap[++heap_len] = (int16_t)node;
            t[node].f = 1;
            T->depth[node] = 0;
            opt_len--;
            if (d.kind != 2) static_len -= stat_len(d, node);
        }
        d.max_code = max_code;
        for (int n = heap_len / 2; n >= 1; --n) sift(t, n, heap_len);
        int node = d.elems;
        do {
            const int n = (int)U((uint32_t)(int)T->heap[1]);
            T->heap[1] = (int16_t)U((uint32_t)(int)T->heap[heap_len--]);
            sift(t, 1, heap_len);
            const int m = (int)U((uint32_t)(int)T->heap[1]);
            T->heap[--heap_max] = (int16_t)n;
            T->heap[--heap_max] = (int16_t)m;
            t[node].f = (uint16_t)(U(t[n].f) + U(t[m].f));
            const uint32_t dn = U(T->depth[n]), dm = U(T->depth[m]);
            T->depth[node] = (uint8_t)((dn >= dm ? dn : dm) + 1);
            t[n].l = t[m].l = (uint16_t)node;
            T->heap[1] = (int16_t)node++;
            sift(t, 1, heap_len);
        } while (heap_len >= 2);
        T->heap[--heap_max] = (int16_t)U((uint32_t)(int)T->heap[1]);
        gen_bitlen(d, heap_max);
        gen_codes(t, max_code);
    }
    // scan_tree (deflate_stream.ipp:978-1042)
    __device__ void scan_tree(Node* t, int max_code)
    {
        int prevlen = -1, nextlen = (int)U(t[0].l), count = 0, max_count = 7, min_count = 4;
        if (nextlen == 0) {
            max_count = 138;
            min_count = 3;
        }
        t[max_code + 1].l = 0xffff;
        for (int n = 0; n <= max_code; ++n) {
            const int curlen = nextlen;
            nextlen = (int)U(t[n + 1].l);
            if (++count < max_count && curlen == nextlen) continue;
            if (count < min_count) T->bt[curlen].f = (uint16_t)(U(T->bt[curlen].f) + count);
            else if (curlen != 0) {
                if (curlen != prevlen) T->bt[curlen].f++;
                T->bt[REP36].f++;
            } else if (count <= 10) T->bt[REPZ310].f++;
            else T->bt[REPZ11].f++;
            count = 0;
            prevlen = curlen;
            if (nextlen == 0) {
                max_count = 138;
                min_count = 3;
            } else if (curlen == nextlen) {
                max_count = 6;
                min_count = 3;
            } else {
                max_count = 7;
                min_count = 4;
            }
        }
    }
    __device__ void send_code(const Node* t, int c) { bw.put(U(t[c].f), U(t[c].l)); }
    // send_tree (deflate_stream.ipp:1046-1110)
    __device__ void send_tree(const Node* t, int max_code)
    {
        int prevlen = -1, nextlen = (int)U(t[0].l), count = 0, max_count = 7, min_count = 4;
        if (nextlen == 0) {
            max_count = 138;
            min_count = 3;
        }
        for (int n = 0; n <= max_code; ++n) {
            const int curlen = nextlen;
            nextlen = (int)U(t[n + 1].l);
            if (++count < max_count && curlen == nextlen) continue;
            if (count < min_count) {
                do send_code(T->bt, curlen);
                while (--count != 0);
            } else if (curlen != 0) {
                if (curlen != prevlen) {
                    send_code(T->bt, curlen);
                    --count;
                }
                send_code(T->bt, REP36);
                bw.put((uint32_t)(count - 3), 2);
            } else if (count <= 10) {
                send_code(T->bt, REPZ310);
                bw.put((uint32_t)(count - 3), 3);
            } else {
                send_code(T->bt, REPZ11);
                bw.put((uint32_t)(count - 11), 7);
            }
            count = 0;
            prevlen = curlen;
            if (nextlen == 0) {
                max_count = 138;
                min_count = 3;
            } else if (curlen == nextlen) {
                max_count = 6;
                min_count = 3;
            } else {
                max_count = 7;
                min_count = 4;
            }
        }
    }
    // build_bl_tree (deflate_stream.ipp:1127-1155)
    __device__ int build_bl_tree()
    {
        scan_tree(T->lt, ld.max_code);
        scan_tree(T->dt, dd.max_code);
        build_tree(bd);
        int maxi;
        for (maxi = NBL - 1; maxi >= 3; --maxi)
            if (U(T->bt[kBlOrder[maxi]].l) != 0) break;
        opt_len += 3 * ((uint32_t)maxi + 1) + 5 + 5 + 4;
        return maxi;
    }
    // compress_block (deflate_stream.ipp:1184-1238); fixed = the static trees
    __device__ void compress_block(bool fixed)
    {
        for (uint32_t sx = 0; sx < sym_next; sx += 3) {
            const uint32_t dist = U((uint32_t)syms[sx] | ((uint32_t)syms[sx + 1] << 8));
            const uint32_t lc = U(syms[sx + 2]);
            if (dist == 0) {
                if (fixed) bw.put(fix_lcode(lc), fix_llen(lc));
                else send_code(T->lt, (int)lc);
            } else {
                const uint32_t code = len_code(lc);
                const uint32_t sym = code + NLIT + 1;
                if (fixed) bw.put(fix_lcode(sym), fix_llen(sym));
                else send_code(T->lt, (int)sym);
                const uint32_t xl = kXl[code];
                if (xl) bw.put(lc - len_base(code), xl);
                const uint32_t d = dist - 1;
                const uint32_t dc = dist_code(d);
                if (fixed) bw.put(rev_bits(dc, 5), 5);
                else send_code(T->dt, (int)dc);
                const uint32_t xd = kXd[dc];
                if (xd) bw.put(d - dist_base(dc), xd);
            }
        }
        if (fixed) bw.put(fix_lcode(EOBS), fix_llen(EOBS));
        else send_code(T->lt, EOBS);
    }
    // tr_stored_block (deflate_stream.ipp:1325-1344); data = window bytes or none
    __device__ void stored_block(int32_t from, uint32_t n, bool has_data, bool last)
    {
        bw.put(last ? 1u : 0u, 3);
        bw.windup();
        bw.put(n & 0xffffu, 16);
        bw.put(~n & 0xffffu, 16);
        if (!has_data) return;
        // the bytes go out whole (bw holds no partial byte here)
        const uint32_t base = bw.opos;
        for (uint32_t j = lane_id(); j < n; j += WAVE)
            if (base + j < bw.cap) bw.out[base + j] = win[(uint32_t)from + j];
        bw.opos += n;
    }
    // tr_flush_block (deflate_stream.ipp:1425-1518)
    __device__ __forceinline__ void close_inline(bool has_buf, uint32_t stored_len, bool last)
    {
        uint32_t opt_lenb, static_lenb;
        int max_blindex = 0;
        mem_fence();
        if (level > 0) {
            build_tree(ld);
            build_tree(dd);
            max_blindex = build_bl_tree();
            opt_lenb = (opt_len + 3 + 7) >> 3;
            static_lenb = (static_len + 3 + 7) >> 3;
            if (static_lenb <= opt_lenb) opt_lenb = static_lenb;
        } else {
            opt_lenb = static_lenb = stored_len + 5;
        }
        if (stored_len + 4 <= opt_lenb && has_buf) {
            stored_block(block_start, stored_len, true, last);
        } else if (strategy == 4 /* Strategy::fixed */ || static_lenb == opt_lenb) {
            bw.put(2u + (last ? 1u : 0u), 3);
            compress_block(true);
        } else {
            bw.put(4u + (last ? 1u : 0u), 3);
            const int lcodes = ld.max_code + 1, dcodes = dd.max_code + 1, blcodes = max_blindex + 1;
            bw.put((uint32_t)(lcodes - 257), 5);
            bw.put((uint32_t)(dcodes - 1), 5);
            bw.put((uint32_t)(blcodes - 4), 4);
            for (int r = 0; r < blcodes; ++r) bw.put(U(T->bt[kBlOrder[r]].l), 3);
            send_tree(T->lt, lcodes - 1);
            send_tree(T->dt, dcodes - 1);
            compress_block(false);
        }
        mem_fence();
        reset_block();
        if (last) bw.windup();
    }
    __device__ __attribute__((noinline)) void close_block(bool has_buf, uint32_t stored_len, bool last)
    {
        Blk L = *this;
        L.close_inline(has_buf, stored_len, last);
        *this = L;
    }
};

// one message's deflater (the fields of detail::deflate_stream this path uses)
struct Dx {
    Trees* T;
    uint8_t* win;
    uint16_t* prv;
    uint16_t* hd;
    uint8_t* syms;
    const uint8_t* msg;
    uint32_t len, in_pos;
    uint32_t wsize, wmask, window_size, hash_size, hash_mask, hash_shift, maxdist;
    int level, strategy, parser;
    Lvl L;
    uint32_t strstart, lookahead, insert, ins_h, high_water;
    int32_t block_start;
    uint32_t prev_length, match_length, prev_match, match_start;
    bool match_available;
    uint32_t sym_next, sym_end, lit_bufsize;
    Blk* B;

    __device__ void flush_block(bool last)
    {
        B->sym_next = sym_next;
        B->block_start = block_start;
        B->close_block(block_start >= 0, (uint32_t)((int32_t)strstart - block_start), last);
        sym_next = 0;
        block_start = (int32_t)strstart;
    }
    __device__ bool tally_lit(uint32_t c)
    {
        if (lane_id() == 0) {
            syms[sym_next] = 0;
            syms[sym_next + 1] = 0;
            syms[sym_next + 2] = (uint8_t)c;
            T->lt[c].f++;
        }
        mem_fence();
        sym_next += 3;
        return sym_next == sym_end;
    }
    __device__ bool tally_match(uint32_t dist, uint32_t lm3)
    {
        if (lane_id() == 0) {
            syms[sym_next] = (uint8_t)(dist & 0xffu);
            syms[sym_next + 1] = (uint8_t)(dist >> 8);
            syms[sym_next + 2] = (uint8_t)lm3;
            T->lt[len_code(lm3) + NLIT + 1].f++;
            T->dt[dist_code(dist - 1)].f++;
        }
        mem_fence();
        sym_next += 3;
        return sym_next == sym_end;
    }

    // --------------------------------------------------------- window
    __device__ uint32_t wb(uint32_t i) const { return U(win[i]); }   // a byte all lanes read
    __device__ uint32_t wl(uint32_t i) const { return win[i]; }      // each lane its own byte
    __device__ void hash_step(uint32_t c) { ins_h = ((ins_h << hash_shift) ^ c) & hash_mask; }
    __device__ uint32_t hash_insert(uint32_t str)
    {
        hash_step(wb(str + (MINM - 1)));
        const uint32_t h = U(hd[ins_h]);
        mem_fence();
        if (lane_id() == 0) {
            prv[str & wmask] = (uint16_t)h;
            hd[ins_h] = (uint16_t)str;
        }
        mem_fence();
        return h;
    }
    // fill_window (deflate_stream.ipp:1520-1669)
    __device__ void refill()
    {
        do {
            uint32_t more = window_size - lookahead - strstart;
            if (strstart >= wsize + maxdist) {
                mem_fence();
                for (uint32_t j = lane_id(); j < wsize; j += WAVE) {
                    const uint8_t v = win[wsize + j];
                    win[j] = v;
                }
                match_start -= wsize;
                strstart -= wsize;
                block_start -= (int32_t)wsize;
                if (insert > strstart) insert = strstart;
                for (uint32_t j = lane_id(); j < hash_size; j += WAVE) {
                    const uint32_t m = hd[j];
                    hd[j] = (uint16_t)(m >= wsize ? m - wsize : 0u);
                }
                for (uint32_t j = lane_id(); j < wsize; j += WAVE) {
                    const uint32_t m = prv[j];
                    prv[j] = (uint16_t)(m >= wsize ? m - wsize : 0u);
                }
                mem_fence();
                more += wsize;
            }
            const uint32_t avail_in = len - in_pos;
            if (avail_in == 0) break;
            const uint32_t n = avail_in < more ? avail_in : more;
            const uint32_t dst = strstart + lookahead;
            for (uint32_t j = lane_id(); j < n; j += WAVE) win[dst + j] = msg[in_pos + j];
            mem_fence();
            in_pos += n;
            lookahead += n;
            if (lookahead + insert >= MINM) {
                uint32_t str = strstart - insert;
                ins_h = wb(str);
                hash_step(wb(str + 1));
                while (insert) {
                    hash_step(wb(str + MINM - 1));
                    const uint32_t h = U(hd[ins_h]);
                    mem_fence();
                    if (lane_id() == 0) {
                        prv[str & wmask] = (uint16_t)h;
                        hd[ins_h] = (uint16_t)str;
                    }
                    mem_fence();
                    ++str;
                    --insert;
                    if (lookahead + insert < MINM) break;
                }
            }
        } while (lookahead < LOOK && in_pos != len);
        if (high_water < window_size) {
            const uint32_t curr = strstart + lookahead;
            uint32_t from = 0, cnt = 0;
            if (high_water < curr) {
                cnt = window_size - curr;
                if (cnt > WINIT) cnt = WINIT;
                from = curr;
                high_water = curr + cnt;
            } else if (high_water < curr + WINIT) {
                cnt = curr + WINIT - high_water;
                if (cnt > window_size - high_water) cnt = window_size - high_water;
                from = high_water;
                high_water += cnt;
            }
            for (uint32_t j = lane_id(); j < cnt; j += WAVE) win[from + j] = 0;
            mem_fence();
        }
    }
    // longest_match (deflate_stream.ipp:1747-1844): the candidate walk is
    // serial; each candidate's bytes 3..258 are compared 64 at a time
    __device__ uint32_t longest(uint32_t cur)
    {
        uint32_t chain = L.chain;
        const uint32_t scan = strstart;
        uint32_t best = prev_length;
        uint32_t nice = L.nice;
        const uint32_t limit = strstart > maxdist ? strstart - maxdist : 0u;
        uint32_t end1 = wb(scan + best - 1), end0 = wb(scan + best);
        const uint32_t s0 = wb(scan), s1 = wb(scan + 1);
        if (prev_length >= L.good) chain >>= 2;
        if (nice > lookahead) nice = lookahead;
        const uint32_t lane = lane_id();
        do {
            if (wb(cur + best) != end0 || wb(cur + best - 1) != end1 || wb(cur) != s0 || wb(cur + 1) != s1)
                continue;
            // bytes 3.. (byte 2 is equal by the hash, as the reference assumes)
            uint32_t mlen = MAXM;
            for (uint32_t b0 = 3; b0 < MAXM; b0 += WAVE) {
                const uint32_t i = b0 + lane;
                const bool ne = i < MAXM && wl(scan + i) != wl(cur + i);
                const uint64_t bal = __ballot(ne);
                if (bal) {
                    mlen = b0 + (uint32_t)__builtin_ctzll(bal);
                    break;
                }
            }
            if (mlen > best) {
                match_start = cur;
                best = mlen;
                if (mlen >= nice) break;
                end1 = wb(scan + best - 1);
                end0 = wb(scan + best);
            }
        } while ((cur = U(prv[cur & wmask])) > limit && --chain != 0);
        return best <= lookahead ? best : lookahead;
    }

    // --------------------------------------------------------- parsers
    // each returns BS_NEED_MORE (Flush::none ran out of input) or BS_BLOCK_DONE
    __device__ int parse_stored(int flush)
    {
        uint32_t max_block = 0xffff;
        if (max_block > lit_bufsize * 4 - 5) max_block = lit_bufsize * 4 - 5;
        for (;;) {
            if (lookahead <= 1) {
                refill();
                if (lookahead == 0 && flush == FL_NONE) return BS_NEED_MORE;
                if (lookahead == 0) break;
            }
            strstart += lookahead;
            lookahead = 0;
            const uint32_t max_start = (uint32_t)block_start + max_block;
            if (strstart == 0 || strstart >= max_start) {
                lookahead = strstart - max_start;
                strstart = max_start;
                flush_block(false);
            }
            if (strstart - (uint32_t)block_start >= maxdist) flush_block(false);
        }
        insert = 0;
        if ((int32_t)strstart > block_start) flush_block(false);
        return BS_BLOCK_DONE;
    }
    __device__ int parse_fast(int flush)
    {
        for (;;) {
            if (lookahead < LOOK) {
                refill();
                if (lookahead < LOOK && flush == FL_NONE) return BS_NEED_MORE;
                if (lookahead == 0) break;
            }
            uint32_t head = 0;
            if (lookahead >= MINM) head = hash_insert(strstart);
            if (head != 0 && strstart - head <= maxdist) match_length = longest(head);
            bool bflush;
            if (match_length >= MINM) {
                bflush = tally_match(strstart - match_start, match_length - MINM);
                lookahead -= match_length;
                if (match_length <= L.lazy && lookahead >= MINM) {
                    match_length--;
                    do {
                        strstart++;
                        hash_insert(strstart);
                    } while (--match_length != 0);
                    strstart++;
                } else {
                    strstart += match_length;
                    match_length = 0;
                    ins_h = wb(strstart);
                    hash_step(wb(strstart + 1));
                }
            } else {
                bflush = tally_lit(wb(strstart));
                lookahead--;
                strstart++;
            }
            if (bflush) flush_block(false);
        }
        insert = strstart < MINM - 1 ? strstart : MINM - 1;
        if (sym_next) flush_block(false);
        return BS_BLOCK_DONE;
    }
    __device__ int parse_slow(int flush)
    {
        for (;;) {
            if (lookahead < LOOK) {
                refill();
                if (lookahead < LOOK && flush == FL_NONE) return BS_NEED_MORE;
                if (lookahead == 0) break;
            }
            uint32_t head = 0;
            if (lookahead >= MINM) head = hash_insert(strstart);
            prev_length = match_length;
            prev_match = match_start;
            match_length = MINM - 1;
            if (head != 0 && prev_length < L.lazy && strstart - head <= maxdist) {
                match_length = longest(head);
                if (match_length <= 5 &&
                    (strategy == 1 /* filtered */ || (match_length == MINM && strstart - match_start > TOO_FAR)))
                    match_length = MINM - 1;
            }
            if (prev_length >= MINM && match_length <= prev_length) {
                const uint32_t max_insert = strstart + lookahead - MINM;
                const bool bflush = tally_match(strstart - 1 - prev_match, prev_length - MINM);
                lookahead -= prev_length - 1;
                prev_length -= 2;
                do {
                    if (++strstart <= max_insert) hash_insert(strstart);
                } while (--prev_length != 0);
                match_available = false;
                match_length = MINM - 1;
                strstart++;
                if (bflush) flush_block(false);
            } else if (match_available) {
                const bool bflush = tally_lit(wb(strstart - 1));
                if (bflush) flush_block(false);
                strstart++;
                lookahead--;
            } else {
                match_available = true;
                strstart++;
                lookahead--;
            }
        }
        if (match_available) {
            tally_lit(wb(strstart - 1));
            match_available = false;
        }
        insert = strstart < MINM - 1 ? strstart : MINM - 1;
        if (sym_next) flush_block(false);
        return BS_BLOCK_DONE;
    }
    __device__ int parse_rle(int flush)
    {
        for (;;) {
            if (lookahead <= MAXM) {
                refill();
                if (lookahead <= MAXM && flush == FL_NONE) return BS_NEED_MORE;
                if (lookahead == 0) break;
            }
            match_length = 0;
            if (lookahead >= MINM && strstart > 0) {
                const uint32_t p = wb(strstart - 1);
                if (p == wb(strstart) && p == wb(strstart + 1) && p == wb(strstart + 2)) {
                    // the reference compares 8 bytes per step from strstart + 3 up to
                    // strstart + MAXM (it may read one step past the match)
                    uint32_t mlen = MAXM;
                    for (uint32_t b0 = 3; b0 < MAXM; b0 += WAVE) {
                        const uint32_t i = b0 + lane_id();
                        const bool ne = i < MAXM && wl(strstart + i) != p;
                        const uint64_t bal = __ballot(ne);
                        if (bal) {
                            mlen = b0 + (uint32_t)__builtin_ctzll(bal);
                            break;
                        }
                    }
                    match_length = mlen > lookahead ? lookahead : mlen;
                }
            }
            bool bflush;
            if (match_length >= MINM) {
                bflush = tally_match(1, match_length - MINM);
                lookahead -= match_length;
                strstart += match_length;
                match_length = 0;
            } else {
                bflush = tally_lit(wb(strstart));
                lookahead--;
                strstart++;
            }
            if (bflush) flush_block(false);
        }
        insert = 0;
        if (sym_next) flush_block(false);
        return BS_BLOCK_DONE;
    }
    __device__ int parse_huff(int flush)
    {
        for (;;) {
            if (lookahead == 0) {
                refill();
                if (lookahead == 0) {
                    if (flush == FL_NONE) return BS_NEED_MORE;
                    break;
                }
            }
            match_length = 0;
            const bool bflush = tally_lit(wb(strstart));
            lookahead--;
            strstart++;
            if (bflush) flush_block(false);
        }
        insert = 0;
        if (sym_next) flush_block(false);
        return BS_BLOCK_DONE;
    }
    __device__ int run(int flush)
    {
        if (strategy == 2) return parse_huff(flush);
        if (strategy == 3) return parse_rle(flush);
        if (parser == PA_STORED) return parse_stored(flush);
        if (parser == PA_FAST) return parse_fast(flush);
        return parse_slow(flush);
    }
};

// One message under impl_base's call sequence (see the header).  Returns the
// payload length, or -1 with *status = need_buffers when the slot is too
// small for the reference's output (its checks after each write() call).
__device__ int32_t exact_msg(Trees* T, uint8_t* win, uint16_t* prv, uint16_t* hd, uint8_t* syms, uint32_t prv_n,
                             const uint8_t* msg, uint32_t len, uint8_t* out, uint32_t cap, const Cfg& c)
{
    Blk b;
    b.T = T;
    b.syms = syms;
    b.win = win;
    b.level = c.level;
    b.strategy = c.strategy;
    b.ld = TDesc{T->lt, 0, NLC, MAXB, 0};
    b.dd = TDesc{T->dt, 1, NDC, MAXB, 0};
    b.bd = TDesc{T->bt, 2, NBL, MAXBL, 0};
    b.bw.out = out;
    b.bw.cap = cap;
    b.bw.acc = 0;
    b.bw.nacc = 0;
    b.bw.opos = 0;
    b.reset_block();
    Dx s;
    s.B = &b;
    s.T = T;
    s.win = win;
    s.prv = prv;
    s.hd = hd;
    s.syms = syms;
    s.msg = msg;
    s.len = len;
    s.in_pos = 0;
    s.wsize = 1u << c.wbits;
    s.wmask = s.wsize - 1;
    s.window_size = 2 * s.wsize;
    s.hash_size = 1u << c.hbits;
    s.hash_mask = s.hash_size - 1;
    s.hash_shift = (c.hbits + MINM - 1) / MINM;
    s.maxdist = s.wsize - LOOK;
    s.level = c.level;
    s.strategy = c.strategy;
    s.L = level_row(c.level);
    s.parser = s.L.parser;
    s.lit_bufsize = c.lit_bufsize;
    s.sym_end = (c.lit_bufsize - 1) * 3;
    s.sym_next = 0;
    // init / lm_init (deflate_stream.ipp:595-718): prev_ and head cleared
    for (uint32_t j = lane_id(); j < prv_n; j += WAVE) prv[j] = 0;
    for (uint32_t j = lane_id(); j < s.hash_size; j += WAVE) hd[j] = 0;
    mem_fence();
    s.high_water = 0;
    s.strstart = 0;
    s.block_start = 0;
    s.lookahead = 0;
    s.insert = 0;
    s.match_length = s.prev_length = MINM - 1;
    s.match_available = false;
    s.match_start = s.prev_match = 0;
    s.ins_h = 0;
    // write(Flush::none) over the message (skipped for an empty one), then
    // write(Flush::block), then write(Flush::sync), with the reference's
    // checks after each: input left or no room after Flush::none, fewer than
    // 6 bytes of room after Flush::block -> need_buffers.  (One call site of
    // the parsers, so they are inlined once.)
    for (int ph = len ? 0 : 1; ph < 3; ++ph) {
        s.run(ph == 0 ? FL_NONE : ph == 1 ? FL_BLOCK : FL_SYNC);
        if (ph == 0 && b.bw.bytes_done() >= cap) return -1;
        if (ph == 1 && b.bw.bytes_done() + 6 > cap) return -1;
    }
    // Flush::sync's parser found no input and emitted nothing; the empty
    // stored block's header bits + pad stay, its 00 00 FF FF is dropped
    b.bw.put(0, 3);
    b.bw.windup();
    return (int32_t)b.bw.opos;
}

// LDS tiers by message length (memLevel <= 5): window bytes, prev_ entries.
// A tier's window holds the whole physical window (2^(windowBits+1)) or, when
// that is larger, the message plus the reference's look-ahead: then no slide
// can happen (it needs strstart >= 2 * w_size - 262), and no position reaches
// past the prev_ entries.  TIER 0: <= 4 KiB (6 waves per CU at memLevel 4),
// TIER 1: <= 8 KiB - 262, TIER 2: the per-wave global workspace.
template <int TIER> struct Tier;
template <> struct Tier<0> { static constexpr uint32_t MAX = 4096, WIN = 4096 + 512, PRV = 4096; };
template <> struct Tier<1> { static constexpr uint32_t MAX = 8192 - LOOK, WIN = 8192 + 512, PRV = 8192; };
__host__ __device__ constexpr int tier_of(uint32_t len, uint32_t hbits)
{
    return hbits > 12 ? 2 : len <= Tier<0>::MAX ? 0 : len <= Tier<1>::MAX ? 1 : 2;
}

// The workspace tier's waves wait on global memory most of the time, so its
// kernel is held to 4 waves per SIMD (<= 128 VGPRs) for more of them in
// flight (BPMD_EXACT_T2_OCC; 3 per SIMD unbounded)
#ifndef BPMD_EXACT_T2_OCC
#define BPMD_EXACT_T2_OCC 4
#endif
#ifndef BPMD_T2_LDS_HEAD
#define BPMD_T2_LDS_HEAD 2048
#endif
constexpr uint32_t T2_LDS_HEAD = BPMD_T2_LDS_HEAD;   // head entries the workspace tier keeps in LDS
template <int TIER>
__global__ void __launch_bounds__(64, TIER == 2 ? BPMD_EXACT_T2_OCC : 1)
deflate_exact_kernel(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                     const uint32_t* __restrict__ in_len, uint32_t n, uint8_t* __restrict__ out,
                     const uint64_t* __restrict__ out_off, const uint32_t* __restrict__ out_cap,
                     uint32_t* __restrict__ out_len, int32_t* __restrict__ status, const uint32_t* __restrict__ mask_key,
                     Cfg c, uint8_t* __restrict__ ws, size_t ws_per_wave, const uint32_t* __restrict__ order,
                     uint32_t* __restrict__ qctr)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    Trees* T = (Trees*)smem;
    const uint32_t wsize = 1u << c.wbits, hash_size = 1u << c.hbits;
    uint8_t *win, *syms;
    uint16_t *prv, *hd;
    uint32_t prv_n;
    if constexpr (TIER < 2) {
        uint8_t* p = smem + ((sizeof(Trees) + 15) & ~(size_t)15);
        win = p;
        p += Tier<TIER>::WIN;
        prv = (uint16_t*)p;
        prv_n = wsize < Tier<TIER>::PRV ? wsize : Tier<TIER>::PRV;
        p += 2 * Tier<TIER>::PRV;
        hd = (uint16_t*)p;
        p += 2 * hash_size;
        syms = p;
    } else {
        uint8_t* p = ws + (size_t)blockIdx.x * ws_per_wave;
        win = p;
        p += 2 * wsize + MAXM + 64;
        p = (uint8_t*)(((uintptr_t)p + 15) & ~(uintptr_t)15);
        prv = (uint16_t*)p;
        prv_n = wsize;
        p += 2 * wsize;
        hd = (uint16_t*)p;
        p += 2 * hash_size;
        syms = p;
        // head[] in LDS beside the trees when it is small (memLevel <= 4:
        // 4 KiB): one global round trip fewer per inserted position
        if (hash_size <= T2_LDS_HEAD) hd = (uint16_t*)(smem + ((sizeof(Trees) + 15) & ~(size_t)15));
    }
    // the workspace tier takes the messages longest first from a queue (the
    // order sorts by len >> 6), so the longest start at once and the waves
    // end together; the LDS tiers stride over the batch.  Each kernel leaves
    // the other tiers' messages.  (One call site of the message body: two
    // would inline it twice and double the registers.)
    uint32_t next = blockIdx.x;
    for (;;) {
        uint32_t i, len;
        if constexpr (TIER == 2) {
            uint32_t k = 0;
            if (lane_id() == 0) k = atomicAdd(qctr, 1u);
            k = U(k);
            if (k >= n) break;
            i = U(order[k]);
            len = U(in_len[i]);
            if (c.hbits <= 12 && len + 64 <= Tier<1>::MAX) break;   // every later one is shorter
        } else {
            if (next >= n) break;
            i = next;
            next += gridDim.x;
            len = in_len[i];
        }
        if (tier_of(len, c.hbits) != TIER) continue;
        uint8_t* o = out + out_off[i];
        const uint32_t cap = out_cap[i];
        const int32_t r = exact_msg(T, win, prv, hd, syms, prv_n, in + in_off[i], len, o, cap, c);
        mem_fence();
        if (r >= 0 && mask_key) {
            // client role: the payload masked on the way out (write.hpp:679-685)
            const uint32_t key = mask_key[i];
            for (uint32_t j = lane_id(); j < (uint32_t)r; j += WAVE) o[j] ^= (uint8_t)(key >> (8 * (j & 3)));
        }
        if (lane_id() == 0) {
            out_len[i] = r >= 0 ? (uint32_t)r : 0u;
            status[i] = r >= 0 ? ST_OK : ST_NEED_BUFFERS;
        }
        mem_fence();
    }
}

}  // namespace dx
}  // namespace bpmd

extern "C" void* bpmd_internal_scratch(hipStream_t s, size_t bytes, int which);
extern "C" const uint32_t* bpmd_internal_lane_order(const uint32_t* in_len, uint32_t n, hipStream_t stream,
                                                    const uint32_t** keys_out);

// cfg already validated (pmd_capi.hip deflate_impl)
extern "C" int bpmd_internal_deflate_exact(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                                           uint32_t n, uint8_t* out, const uint64_t* out_off,
                                           const uint32_t* out_cap, uint32_t* out_len, int32_t* status, int level,
                                           int window_bits, int mem_level, int strategy, const uint32_t* mask_key,
                                           hipStream_t stream)
{
    using namespace bpmd::dx;
    if (n == 0) return 0;
    Cfg c;
    c.level = level;
    c.strategy = strategy;
    c.wbits = (uint32_t)window_bits;
    c.hbits = (uint32_t)mem_level + 7;
    c.lit_bufsize = 1u << (mem_level + 6);
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    hipError_t e;
    const size_t trees = (sizeof(Trees) + 15) & ~(size_t)15;
    if (c.hbits <= 12) {
        const size_t tail = 2 * ((size_t)1 << c.hbits) + 3 * (size_t)c.lit_bufsize;
        hipLaunchKernelGGL(deflate_exact_kernel<0>, dim3(n), dim3(64), trees + Tier<0>::WIN + 2 * Tier<0>::PRV + tail,
                           stream, in, in_off, in_len, n, out, out_off, out_cap, out_len, status, mask_key, c,
                           (uint8_t*)nullptr, (size_t)0, (const uint32_t*)nullptr, (uint32_t*)nullptr);
        if ((e = hipGetLastError()) != hipSuccess) return (int)e;
        hipLaunchKernelGGL(deflate_exact_kernel<1>, dim3(n), dim3(64), trees + Tier<1>::WIN + 2 * Tier<1>::PRV + tail,
                           stream, in, in_off, in_len, n, out, out_off, out_cap, out_len, status, mask_key, c,
                           (uint8_t*)nullptr, (size_t)0, (const uint32_t*)nullptr, (uint32_t*)nullptr);
        if ((e = hipGetLastError()) != hipSuccess) return (int)e;
    }
    // the rest: window / prev / head / symbols in a per-wave workspace.  The
    // waves are latency-bound on it, so as many as the registers allow
    // (BPMD_EXACT_T2_OCC per SIMD; round 3 ran four per CU), taking the
    // messages longest first from a queue (BPMD_EXACT_WAVES_PER_CU overrides)
    static const unsigned wpc = [] {
        const char* ev = getenv("BPMD_EXACT_WAVES_PER_CU");
        const unsigned v = ev ? (unsigned)strtoul(ev, nullptr, 10) : 0u;
        return v ? v : 4u * BPMD_EXACT_T2_OCC;
    }();
    const size_t wsz = (size_t)1 << c.wbits;
    const size_t per = ((2 * wsz + MAXM + 64 + 15) & ~(size_t)15) + 2 * wsz + 2 * ((size_t)1 << c.hbits) +
                       3 * (size_t)c.lit_bufsize + 64;
    const unsigned grid = (unsigned)cus * wpc;
    uint8_t* ws = (uint8_t*)bpmd_internal_scratch(stream, per * grid, 4);
    uint32_t* qctr = (uint32_t*)bpmd_internal_scratch(stream, 256, 3);
    const uint32_t* order = bpmd_internal_lane_order(in_len, n, stream, nullptr);
    if (!ws || !qctr) return (int)hipErrorOutOfMemory;
    if (!order || hipMemsetAsync(qctr, 0, sizeof(uint32_t), stream) != hipSuccess) return (int)hipErrorUnknown;
    const size_t t2_lds = trees + (((size_t)1 << c.hbits) <= T2_LDS_HEAD ? 2 * ((size_t)1 << c.hbits) : 0);
    hipLaunchKernelGGL(deflate_exact_kernel<2>, dim3(grid < n ? grid : n), dim3(64), t2_lds, stream, in, in_off,
                       in_len, n, out, out_off, out_cap, out_len, status, mask_key, c, ws, per, order, qctr);
    return (int)hipGetLastError();
}
