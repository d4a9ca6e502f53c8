// huff_wave.h -- wave-cooperative construction of the decode tables of
// huff_table.h (same slots, same zlib-compatible layout, same errors).
//
// The serial builder (huff_table.h, a restatement of inflate_stream.ipp:
// 551-863) walks codes one by one.  Here the 64 lanes share the work:
//   counts     15 ballots per 64 symbols
//   sorting    rank within a length = prefix of the ballot (mbcnt)
//   root table one lane per slot: the slot's first `root` stream bits are a
//              left-justified code prefix; its length is the number of
//              canonical limits at or below it (codes of one length form one
//              contiguous range), its symbol an offset into the sorted list
//   sub-tables for a complete code every root prefix holding longer codes is
//              a full subtree whose depth is its longest code, which is the
//              size zlib's "left" loop arrives at; sub-tables are laid out in
//              canonical order of their prefixes, exactly as zlib does.
#pragma once

#include "huff_table.h"

namespace bpmd {

struct WaveTableScratch {
    uint16_t sorted[320];
    uint32_t offs[16];     // first sorted index of each length
    uint32_t first[16];    // first canonical code of each length
    uint32_t next[16];     // running sorted index while ranking
    uint32_t grp[320];     // per sub-table: (curr << 16) | offset
};

__device__ __forceinline__ uint32_t wave_prefix_count(uint64_t m)
{
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

template <int TYPE>
__device__ __forceinline__ uint16_t make_slot(unsigned sym, unsigned bits)
{
    if (TYPE == BUILD_CODES) return slot(K_VAL, bits, sym);
    if (TYPE == BUILD_LENS) {
        if (sym < 256) return slot(K_VAL, bits, sym);
        if (sym == 256) return slot(K_EOB, bits, 0);
        if (sym <= 285) return slot(K_LEN, bits, sym - 257);
        return slot(K_SPECIAL, bits, V_INVALID);
    }
    return sym <= 29 ? slot(K_VAL, bits, sym) : slot(K_SPECIAL, bits, V_INVALID);
}

// All 64 lanes must call.  Returns 0 / 14 / 15 / 16 (wave-uniform).
template <int TYPE>
__device__ int build_table_wave(const uint8_t* lens, unsigned n, uint16_t* tab, unsigned req_root,
                                WaveTableScratch& S, unsigned& root_out, unsigned& used_out, unsigned& lmin_out)
{
    const unsigned lane = __lane_id();
    uint32_t cnt[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) cnt[i] = 0;
    const unsigned chunks = (n + 63) / 64;
    for (unsigned c = 0; c < chunks; ++c) {
        const unsigned s = c * 64 + lane;
        const unsigned len = s < n ? lens[s] : 0u;
#pragma unroll
        for (int l = 1; l < 16; ++l) cnt[l] += (uint32_t)__builtin_popcountll(__ballot(len == (unsigned)l));
    }
    unsigned hi = 0, lo = 0;
#pragma unroll
    for (int l = 15; l >= 1; --l)
        if (!hi && cnt[l]) hi = l;
#pragma unroll
    for (int l = 1; l <= 15; ++l)
        if (!lo && cnt[l]) lo = l;
    if (hi == 0) {
        if (lane < 2) tab[lane] = slot(K_SPECIAL, 1, V_INVALID);
        root_out = 1;
        used_out = 2;
        lmin_out = 1;
        return 0;
    }
    lmin_out = lo;
    unsigned root = req_root;
    if (root > hi) root = hi;
    if (root < lo) root = lo;
    int avail = 1;
#pragma unroll
    for (int l = 1; l <= 15; ++l) {
        avail = (avail << 1) - (int)cnt[l];
        if (avail < 0) return 14;
    }
    if (avail > 0 && (TYPE == BUILD_CODES || hi != 1)) return 15;

    // offsets, canonical first codes, left-justified limits
    uint32_t offs[16], first[16], lim[16];
    {
        uint32_t o = 0, code = 0, prev = 0;
#pragma unroll
        for (int l = 1; l <= 15; ++l) {
            offs[l] = o;
            o += cnt[l];
            code = (code + prev) << 1;
            first[l] = code;
            prev = cnt[l];
        }
#pragma unroll
        for (int l = 1; l <= 15; ++l) lim[l] = l <= (int)root ? (first[l] + cnt[l]) << (root - l) : 0;
    }
    if (lane < 16) {
        // lane-indexed copies for per-lane lookups
        uint32_t vo = 0, vf = 0;
#pragma unroll
        for (int l = 1; l <= 15; ++l)
            if ((int)lane == l) { vo = offs[l]; vf = first[l]; }
        S.offs[lane] = vo;
        S.first[lane] = vf;
        S.next[lane] = vo;
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");

    // sort symbols by (length, symbol)
    for (unsigned c = 0; c < chunks; ++c) {
        const unsigned s = c * 64 + lane;
        const unsigned len = s < n ? lens[s] : 0u;
        uint64_t mine = 0;
        uint32_t adds[16];
#pragma unroll
        for (int l = 1; l < 16; ++l) {
            const uint64_t m = __ballot(len == (unsigned)l);
            adds[l] = (uint32_t)__builtin_popcountll(m);
            if (len == (unsigned)l) mine = m;
        }
        if (len) S.sorted[S.next[len] + wave_prefix_count(mine)] = (uint16_t)s;
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
        if (lane >= 1 && lane < 16) {
            uint32_t a = 0;
#pragma unroll
            for (int l = 1; l < 16; ++l)
                if ((int)lane == l) a = adds[l];
            S.next[lane] += a;
        }
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
    }

    // root table
    const unsigned nroot = 1u << root;
    for (unsigned idx = lane; idx < nroot; idx += 64) {
        const uint32_t prefix = __builtin_bitreverse32(idx) >> (32 - root);
        unsigned l = 1;
#pragma unroll
        for (int j = 1; j <= 15; ++j)
            if (j <= (int)root && prefix >= lim[j]) ++l;
        uint16_t sl;
        if (l <= root) {
            const uint32_t code = prefix >> (root - l);
            const unsigned sym = S.sorted[S.offs[l] + code - S.first[l]];
            sl = make_slot<TYPE>(sym, l);
        } else {
            // a sub-table link (filled below) or, for the one accepted
            // incomplete code (a single 1-bit code), an invalid slot
            sl = slot(K_SPECIAL, root, V_INVALID);
        }
        tab[idx] = sl;
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");

    // sub-tables for codes longer than root
    unsigned used = nroot;
    if (hi > root) {
        const unsigned kbeg = S.offs[root + 1];   // root < hi <= 15
        uint32_t nlong = 0;
#pragma unroll
        for (int l = 1; l <= 15; ++l)
            if (l > (int)root) nlong += cnt[l];
        // pass 1: group (= sub-table) boundaries, sizes and offsets.  Codes
        // are in canonical order, so each root prefix P is one run; its
        // sub-table size is 2^(len of its last, longest code - root).
        uint32_t carry_prefix = 0xffffffffu, carry_off = nroot, carry_groups = 0;
        const unsigned lchunks = (nlong + 63) / 64;
        for (unsigned c = 0; c < lchunks; ++c) {
            const unsigned k = kbeg + c * 64 + lane;
            const bool act = c * 64 + lane < nlong;
            unsigned len = 0, code = 0, P = 0;
            if (act) {
                const unsigned sym = S.sorted[k];
                len = lens[sym];
                code = S.first[len] + (k - S.offs[len]);
                P = code >> (len - root);
            }
            uint32_t prevP = __shfl_up(P, 1);
            if (lane == 0) prevP = carry_prefix;
            const uint32_t nextP = __shfl_down(P, 1);
            const bool nxt_act = (c * 64 + lane + 1) < nlong;
            const bool start = act && P != prevP;
            bool is_last = act && (!nxt_act || nextP != P);
            if (act && lane == 63 && nxt_act) {
                // the next code sits in the next chunk
                const unsigned k2 = k + 1;
                const unsigned sym2 = S.sorted[k2];
                const unsigned len2 = lens[sym2];
                const unsigned code2 = S.first[len2] + (k2 - S.offs[len2]);
                is_last = (code2 >> (len2 - root)) != P;
            }
            const uint32_t size = is_last ? (1u << (len - root)) : 0u;
            uint32_t incl = size;
#pragma unroll
            for (unsigned d = 1; d < 64; d <<= 1) {
                const uint32_t y = __shfl_up(incl, d);
                incl += lane >= d ? y : 0u;   // select: a shuffle must not sink under divergence
            }
            const uint32_t off = carry_off + incl - size;   // same for every code of a group
            const uint64_t sm = __ballot(start);
            const uint32_t my_g = carry_groups + (uint32_t)__builtin_popcountll(sm & ((2ull << lane) - 1ull)) - 1u;
            if (is_last) S.grp[my_g] = ((len - root) << 16) | off;
            carry_off = __builtin_amdgcn_readfirstlane(__shfl(off + size, 63));
            carry_prefix = __shfl(P, 63);
            carry_groups += (uint32_t)__builtin_popcountll(sm);
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");
        }
        used = carry_off;
        // pass 2: links and sub-table entries
        carry_prefix = 0xffffffffu;
        carry_groups = 0;
        for (unsigned c = 0; c < lchunks; ++c) {
            const unsigned k = kbeg + c * 64 + lane;
            const bool act = c * 64 + lane < nlong;
            unsigned len = 0, code = 0, P = 0, sym = 0;
            if (act) {
                sym = S.sorted[k];
                len = lens[sym];
                code = S.first[len] + (k - S.offs[len]);
                P = code >> (len - root);
            }
            uint32_t prevP = __shfl_up(P, 1);
            if (lane == 0) prevP = carry_prefix;
            const bool start = act && P != prevP;
            const uint64_t sm = __ballot(start);
            const uint32_t my_g = carry_groups + (uint32_t)__builtin_popcountll(sm & ((2ull << lane) - 1ull)) - 1u;
            if (act) {
                const uint32_t gi = S.grp[my_g];
                const unsigned curr = gi >> 16, off = gi & 0xffffu;
                if (start) tab[__builtin_bitreverse32(P) >> (32 - root)] = slot(K_SPECIAL, curr, off);
                const unsigned dl = len - root;
                const unsigned low = __builtin_bitreverse32(code & ((1u << dl) - 1u)) >> (32 - dl);
                const uint16_t sl = make_slot<TYPE>(sym, dl);
                for (unsigned e = low; e < (1u << curr); e += (1u << dl)) tab[off + e] = sl;
            }
            carry_prefix = __shfl(P, 63);
            carry_groups += (uint32_t)__builtin_popcountll(sm);
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");
        }
    }
    if ((TYPE == BUILD_LENS && used > kEnoughLens) || (TYPE == BUILD_DISTS && used > kEnoughDists)) return 16;
    root_out = root;
    used_out = used;
    return 0;
}

}  // namespace bpmd
