// canon.h -- table-free canonical Huffman decode shared by the lane kernel
// (pmd_inflate_lane3.hip) and the block-parallel scan (pmd_inflate_bp.hip).
//
// One register word per code length L: Q = lim_L << 15 | L << 11 | end_L,
// where lim_L is the left-justified end of the codes of length <= L and
// end_L the canonical index past them.  For the bit-reversed code c an
// unsigned min of Q - ((c + 1) << 15) over the words finds the smallest
// lim_L > c (inflate_stream.ipp:632-640 builds the same canonical order).
#pragma once
#include "pmd_common.h"

namespace bpmd {
namespace lp3 {

template <int NB>
struct Canon {
    uint32_t Q[NB];
    uint32_t root;   // the reference's (clamped) root table bits
};

template <int NB>
__device__ __forceinline__ uint32_t canon_min(const uint32_t (&Q)[NB], uint32_t c)
{
    // a chain of three-input mins (v_min3_u32): NB - 1 values fold in
    // (NB - 1) / 2 instructions
    const uint32_t k1 = (c + 1) << 15;
    uint32_t m = Q[0] - k1;
#pragma unroll
    for (int i = 1; i + 1 < NB; i += 2)
        m = __builtin_elementwise_min(__builtin_elementwise_min(m, Q[i] - k1), Q[i + 1] - k1);
    if (NB % 2 == 0) m = __builtin_elementwise_min(m, Q[NB - 1] - k1);
    return m;
}

struct Sym {
    uint32_t L;     // code length
    uint32_t idx;   // canonical index (0 when invalid)
    bool inval;
};

// NB words; BITS: the code width c is read at (the longest length, 15 for
// literal/length and distance codes, 7 for the code-length code) -- equal to
// NB except for the compact words below
template <int NB, int BITS = NB>
__device__ __forceinline__ Sym canon_decode(const uint32_t (&Q)[NB], uint32_t c)
{
    const uint32_t m = canon_min<NB>(Q, c);
    Sym r;
    r.inval = (m >> 31) != 0;
    const uint32_t q = m + ((c + 1) << 15);
    r.L = (q >> 11) & 15u;
    const int32_t below = (int32_t)(c - (q >> 15)) >> (BITS - (int32_t)r.L);   // in [-count_L, -1]
    r.idx = r.inval ? 0u : (uint32_t)((int32_t)(q & 0x7ffu) + below);
    return r;
}

// A code uses few distinct lengths (deflated JSON: about 8-10 for
// literal/length, 5-7 for distances), and a length with no codes adds a word
// that can never win the search (its lim equals the length before it).  The
// compact form keeps only the words of lengths that have codes, in order,
// padded with 0 (0 - (c + 1) << 15 wraps above 2^31, so padding never wins
// and an invalid code still reads as invalid): the same result as
// canon_min<15> in K - 1 instead of 14 subtractions and mins.  Returns false
// when the code has more than K distinct lengths (the caller keeps the full
// search for it).
template <int NB, int K>
__device__ __forceinline__ bool compact_canon(const uint32_t (&Q)[NB], uint32_t (&W)[K])
{
    uint32_t rank = 0, prev = 0;
#pragma unroll
    for (int j = 0; j < K; ++j) W[j] = 0;
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        const uint32_t lim = Q[i] >> 15;
        const bool used = lim != prev;
        prev = lim;
#pragma unroll
        for (int j = 0; j < K; ++j) W[j] = (used && rank == (uint32_t)j) ? Q[i] : W[j];
        rank += used ? 1u : 0u;
    }
    return rank <= (uint32_t)K;
}

// The reference's slow path asks for the root bits, or for root + sub-table
// index bits when the code is longer than the root: a sub-table covers one
// root prefix and is as deep as the longest code under it, i.e. the length
// of the last code of the prefix's range (inflate_stream.ipp:360-420, 688-709).
template <int NB>
__device__ __forceinline__ uint32_t canon_need(const Canon<NB>& t, const Sym& y, uint32_t c)
{
    if (y.inval || y.L <= t.root) return t.root;
    const uint32_t re = c | ((1u << (NB - t.root)) - 1u);
    return ((canon_min<NB>(t.Q, re) + ((re + 1) << 15)) >> 11) & 15u;
}

__device__ __forceinline__ uint32_t rev15(uint64_t bb) { return __builtin_bitreverse32((uint32_t)bb) >> 17; }
__device__ __forceinline__ uint32_t lowmask(uint32_t n) { return n >= 32 ? ~0u : ((1u << n) - 1u); }

// counts c[1..NB] -> canonical words; returns 0, 14 or 15 following
// inflate_table's acceptance rules (inflate_stream.ipp:574-617).
// type: 0 codes, 1 lens, 2 dists.  (The first canonical index of length l
// is the running sum of c[1..l-1]; callers that need it recompute it.)
template <int NB>
__device__ __forceinline__ int make_canon(const uint32_t (&c)[16], uint32_t R, int type, Canon<NB>& t)
{
    uint32_t lim = 0, cu = 0, nz = 0;   // nz: bit l set when some code has length l
#pragma unroll
    for (int l = 1; l <= NB; ++l) {
        cu += c[l];
        lim += c[l] << (NB - l);
        t.Q[l - 1] = (lim << 15) | ((uint32_t)l << 11) | cu;
        nz |= c[l] ? 1u << l : 0u;
    }
    if (nz == 0) {   // empty code: a 1-bit root of invalid slots
        t.root = 1;
        return 0;
    }
    const uint32_t lo = (uint32_t)__builtin_ctz(nz), hi = 31u - (uint32_t)__builtin_clz(nz);
    const uint32_t r = R < hi ? R : hi;
    t.root = r < lo ? lo : r;
    // The reference's running `left` (2^l minus the codes of length <= l)
    // ends at 2^NB - lim; a prefix can only be over-subscribed if the whole
    // Kraft sum is, since the partial sums only grow.
    if (lim > (1u << NB)) return ST_OVER_SUBSCRIBED_LENGTH;
    if (lim < (1u << NB) && (type == 0 || hi != 1)) return ST_INCOMPLETE_LENGTH_SET;
    return 0;
}

}  // namespace lp3
}  // namespace bpmd
