// lz_core.h -- encoder pieces shared by the HIP deflate kernel and the host
// model used to size its parameters (scripts/deflate_model.cpp).
//
// Everything here is plain integer code callable from host or device.  The
// encoder is NOT required to be bit-identical to Beast (the contract is a
// byte-identical round trip and a stated size tolerance), but the pieces
// follow the reference's design so ratios stay comparable:
//   level table (good/lazy/nice/chain, greedy vs lazy)   zlib/detail/deflate_stream.hpp:571-590
//   longest_match chain walk rules                       zlib/detail/deflate_stream.ipp:1747-1844
//   lazy evaluation (f_slow) incl. TOO_FAR / filtered     deflate_stream.ipp:2045-2184
//   length / distance codes and extra bits               deflate_stream.ipp:143-225 (get_lut)
//   code-length run-length coding (16/17/18)             deflate_stream.ipp:978-1110
//   block type choice (stored / fixed / dynamic)         deflate_stream.ipp:1425-1518
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#define LZ_HD __host__ __device__ __forceinline__
#else
#define LZ_HD static inline
#endif

namespace lz {

enum : int {
    MIN_MATCH = 3, MAX_MATCH = 258, TOO_FAR = 4096, LOOKAHEAD_MIN = MAX_MATCH + MIN_MATCH + 1,
    N_LIT = 256, EOB = 256, N_LCODES = 286, N_DCODES = 30, N_BLCODES = 19, MAX_BITS = 15, MAX_BL_BITS = 7,
};

enum Parser : int { P_STORED = 0, P_FAST = 1, P_SLOW = 2 };

struct Level { uint16_t good, lazy, nice, chain; int parser; };

// deflate_stream.hpp:571-590 (values of the reference's configuration table)
LZ_HD Level level_params(int level)
{
    switch (level) {
    case 0: return {0, 0, 0, 0, P_STORED};
    case 1: return {4, 4, 8, 4, P_FAST};
    case 2: return {4, 5, 16, 8, P_FAST};
    case 3: return {4, 6, 32, 32, P_FAST};
    case 4: return {4, 4, 16, 16, P_SLOW};
    case 5: return {8, 16, 32, 32, P_SLOW};
    case 7: return {8, 32, 128, 256, P_SLOW};
    case 8: return {32, 128, 258, 1024, P_SLOW};
    case 9: return {32, 258, 258, 4096, P_SLOW};
    default: return {8, 16, 128, 128, P_SLOW};   // 6 (and -1 = default)
    }
}

// Chain limit the GPU encoder uses: the level table's, capped at
// BPMD_CHAIN_CAP for messages of one 4 KiB chunk (C3 corpus at level 6 with
// 4-byte chain keys, round 3: cap 16 / 12 / 8 / 6 / 5 / 4 = 34.1 / 35.5 /
// 37.6 / 39.5 / 40.3 / 41.2 GiB/s at 0.991 / 0.994 / 1.001 / 1.006 / 1.011 /
// 1.016x Beast's size; 4 is the default: the fastest within
// 1.02x) and at BPMD_CHAIN_CAP_MULTI (0 = the table's value) for the chunks
// of longer messages, which see BPMD_CHUNK_HIST bytes of history before the
// chunk.  configs[3] (C4), whole batch, size against Beast at level 6 and
// deflate GiB/s:
//   history 4096, cap 16: 1.086x, 16.4 (the LDS holds 5 waves per CU)
//   history 2048, cap 16: 1.111x, 23.9 (6 waves per CU)
//   history 2048, cap 32: 1.089x, 20.9   <- default
#ifndef BPMD_CHAIN_CAP
#define BPMD_CHAIN_CAP 4
#endif
#ifndef BPMD_CHAIN_CAP_MULTI
#define BPMD_CHAIN_CAP_MULTI 32
#endif
#ifndef BPMD_CHUNK_HIST
#define BPMD_CHUNK_HIST 2048
#endif
// Levels >= BPMD_DEEP_LEVEL (zlib's slow levels 7-9) give each chunk 4 KiB of
// history instead (round 5; C4 at 4 KiB and chain cap 32: 1.038x Beast's size
// at 20.6 GiB/s against 1.059x at 30.5 with 2 KiB): the chunk
// kernel's LDS then holds 5 waves per CU instead of 6.
#ifndef BPMD_DEEP_LEVEL
#define BPMD_DEEP_LEVEL 7
#endif
constexpr unsigned CHUNK_HIST_DEEP = 4096;
LZ_HD unsigned chunk_hist(int level)
{
    return level >= BPMD_DEEP_LEVEL && CHUNK_HIST_DEEP > (unsigned)BPMD_CHUNK_HIST ? CHUNK_HIST_DEEP
                                                                                   : (unsigned)BPMD_CHUNK_HIST;
}
LZ_HD unsigned gpu_chain(int level, bool single_chunk)
{
    const unsigned c = level_params(level).chain;
    const unsigned cap = single_chunk ? (unsigned)BPMD_CHAIN_CAP : (unsigned)BPMD_CHAIN_CAP_MULTI;
    return cap && c > cap ? cap : c;
}

LZ_HD int ilog2(uint32_t v) { return 31 - __builtin_clz(v); }

// Length symbol (257..285), its extra-bit count and extra value for a match
// length 3..258.
LZ_HD void len_code(unsigned len, unsigned& sym, unsigned& nx, unsigned& xv)
{
    unsigned l = len - MIN_MATCH;
    if (l < 8) { sym = 257 + l; nx = 0; xv = 0; return; }
    if (len == MAX_MATCH) { sym = 285; nx = 0; xv = 0; return; }
    unsigned eb = (unsigned)ilog2(l) - 2;
    unsigned hi = (l >> eb) & 3;
    sym = 257 + 4 * (eb + 1) + hi;
    nx = eb;
    xv = l - ((4 | hi) << eb);
}

// Distance symbol (0..29), extra-bit count and extra value for 1..32768.
LZ_HD void dist_code(unsigned dist, unsigned& sym, unsigned& nx, unsigned& xv)
{
    unsigned d = dist - 1;
    if (d < 4) { sym = d; nx = 0; xv = 0; return; }
    unsigned eb = (unsigned)ilog2(d) - 1;
    unsigned hi = (d >> eb) & 1;
    sym = 2 * (eb + 1) + hi;
    nx = eb;
    xv = d - ((2 | hi) << eb);
}

LZ_HD unsigned len_extra_bits(unsigned sym) { return (sym >= 265 && sym < 285) ? (sym - 261) / 4 : 0; }
LZ_HD unsigned dist_extra_bits(unsigned sym) { return sym >= 4 ? (sym - 2) / 2 : 0; }

// Fixed-Huffman code lengths (RFC 1951 §3.2.6).
LZ_HD unsigned fixed_lit_len(unsigned sym) { return sym < 144 ? 8 : sym < 256 ? 9 : sym < 280 ? 7 : 8; }

LZ_HD uint32_t reverse_bits(uint32_t code, unsigned len)
{
#if defined(__clang__)
    return __builtin_bitreverse32(code) >> (32 - len);
#else
    uint32_t r = 0;
    for (unsigned i = 0; i < len; ++i, code >>= 1) r = (r << 1) | (code & 1);
    return r;
#endif
}

// Hash of the 3 bytes at a position (bytes packed little-endian in `w`).
// Hash-chain key of position q: its next 4 bytes (w, little-endian), or the
// 3 there are when q is 3 bytes from the window's end (avail = bytes from q
// to the end).  Beast's chains key on MIN_MATCH = 3 bytes (deflate_stream.ipp
// UPDATE_HASH); keying on 4 means every candidate a capped walk visits shares
// 4 bytes with the current string, so a 16-candidate walk finds longer
// matches than Beast's 128-candidate one on 3-byte chains, and 3-byte matches
// (worth 1-2 bits each) are found only at a window's end.  C3 at level 6:
// 33.1 -> 34.4 GiB/s, 1.020 -> 0.991x Beast's size.
// Incompressible chunks (round 5).  After the chains are built, every
// INCOMP_STRIDE-th position q of the chunk (q + 4 within the window) counts a
// hit when the head of its chain holds the same 4 bytes.  With fewer than one
// hit per INCOMP_DEN chunk bytes (sampled: hits * INCOMP_STRIDE * INCOMP_DEN <
// chunk bytes) the
// chunk is near-random and the parse would find almost no matches, so it is
// coded as literals without one (a dynamic or stored block as usual); 0 turns
// the test off.  Beast has no such test; the size change on C5's near-random
// bytes is in DESIGN.md 4.2.
#ifndef BPMD_INCOMP_DEN
#define BPMD_INCOMP_DEN 64
#endif
constexpr unsigned INCOMP_DEN = BPMD_INCOMP_DEN, INCOMP_STRIDE = 4;
LZ_HD bool incompressible(unsigned hits, unsigned chunk_bytes)
{
    return INCOMP_DEN && (unsigned long long)hits * INCOMP_STRIDE * INCOMP_DEN < chunk_bytes;
}
// Round 6: an incompressible chunk of a message longer than one chunk is a
// stored block outright (no parse, no trees).  A Huffman code over near-random
// bytes saved ~0.7 % of them (C5: 0.9932 of the input; stored: ~1.0001), and a
// stored block inflates as one copy: the block-parallel decoder takes it as a
// single token and a lane never decodes it symbol by symbol -- C5's 8-way
// shards were one Huffman chunk's serial decode.  Messages of one
// chunk keep the size-based choice.  0 restores round 5's rule.
#ifndef BPMD_INCOMP_STORED
#define BPMD_INCOMP_STORED 1
#endif
constexpr bool INCOMP_STORED = BPMD_INCOMP_STORED != 0;
// Round 6: the block choice of a chunk of a multi-chunk message.  Beast keeps
// a Huffman block whenever it is smaller than the stored one
// (tr_flush_block, deflate_stream.ipp:1478: stored_len + 4 <= opt_lenb).
// Here it must also save 1/2^BPMD_MIN_GAIN_SHIFT of the chunk (256 bytes of
// 4 KiB at 4): a stored chunk inflates as one copy (SEG_DIRECT),
// a Huffman chunk of near-random bytes one symbol at a time on one lane
// (~2 ms per 4 KiB), and a chunk that saves under ~6 % is that kind.  Messages
// of one chunk keep Beast's rule.  0 restores it everywhere.  C5 (near-random
// binary, profiles/r06m_ab_min_gain.log), shift 0 / 5 / 4 / 3: size 1.0077 /
// 1.0091 / 1.0128 / 1.0158x Beast's at L1, deflate 98.6 / 102.9 / 109.0 /
// 112.6 GiB/s, inflate 174 / 177 / 192 / 248 GiB/s.  JSON chunks save 60-70 %
// and never reach the rule.
#ifndef BPMD_MIN_GAIN_SHIFT
#define BPMD_MIN_GAIN_SHIFT 4
#endif
LZ_HD bool chunk_stored(unsigned clen, unsigned long long best_bytes, bool multi_chunk)
{
    const unsigned slack = (BPMD_MIN_GAIN_SHIFT && multi_chunk) ? clen >> BPMD_MIN_GAIN_SHIFT : 0u;
    return (unsigned long long)clen + 4 <= best_bytes + slack;
}

LZ_HD uint32_t chain_hash(uint32_t w, unsigned avail, unsigned hbits)
{
#ifdef BPMD_CHAIN_KEY3   // diagnostics: round 2's 3-byte keys
    (void)avail;
    return ((w & 0xFFFFFFu) * 0x9E3779B1u) >> (32 - hbits);
#else
    return ((avail >= 4 ? w : (w & 0xFFFFFFu)) * 0x9E3779B1u) >> (32 - hbits);
#endif
}

// ---------------------------------------------------------------- Huffman
//
// Shannon code lengths for wide alphabets (round 3).  When a block uses at
// least SHANNON_MIN literal/length symbols (near-random bytes: C5), the
// optimal Huffman lengths are nearly flat and the serial two-queue merge is
// the costliest step of the block (~150 K cycles of ~700 K per 4 KiB chunk).
// There the lengths come from the symbols' own frequencies instead: L(f) =
// the smallest L >= 1 with f * 2^L >= T (T = the alphabet's total, so the
// Kraft sum is <= 1), counted per length, the code completed by moving the
// longest codes up one level while the Kraft sum stays <= 1 (an incomplete
// literal/length code is an error for inflate_stream, ipp:574-617), and the
// lengths reassigned in frequency order as gen_bitlen does.  C5 (64 KiB
// binary): deflate 19.5 -> 23.7 GiB/s at L1, payloads 0.9909 -> 0.9890 of
// the input (the merge's 15-bit overflow repair costs more here than the
// Shannon lengths do); never used for narrower alphabets (JSON: 100-150).
#ifndef BPMD_SHANNON_MIN
#define BPMD_SHANNON_MIN 200
#endif
constexpr unsigned SHANNON_MIN = BPMD_SHANNON_MIN;

LZ_HD unsigned shannon_len(uint32_t f, uint32_t T, unsigned max_bits)
{
    unsigned L = (unsigned)(__builtin_clz(f) - __builtin_clz(T));   // f * 2^L in [T / 2, 2T)
    if (((uint64_t)f << L) < (uint64_t)T) ++L;
    L = L < 1 ? 1u : L;
    return L > max_bits ? max_bits : L;
}

// bl_count[1..max_bits] of a code with Kraft sum <= 1 -> a complete code
LZ_HD void complete_code(unsigned* bl_count, unsigned max_bits)
{
    uint32_t k = 0;
    for (unsigned b = 1; b <= max_bits; ++b) k += bl_count[b] << (max_bits - b);
    uint32_t slack = (1u << max_bits) - k;
    for (unsigned b = max_bits; b >= 2 && slack; --b) {
        const uint32_t unit = 1u << (max_bits - b);
        uint32_t n = slack / unit;
        n = n < bl_count[b] ? n : bl_count[b];
        bl_count[b] -= n;
        bl_count[b - 1] += n;
        slack -= n * unit;
    }
}
//
// Code lengths for one alphabet.  Deterministic restatement of the
// two-queue Huffman construction over leaves sorted by (freq, symbol), with
// the reference's length-limiting rule (deflate_stream.ipp:786-873): leaves
// deeper than max_bits are clamped, the Kraft overflow is repaid by moving
// leaves down from the deepest non-full level, and lengths are reassigned in
// frequency order (least frequent gets the longest code).  As in the
// reference, an alphabet with fewer than two used symbols gets dummy
// symbols so that a complete code always exists.
//
// Host reference version (serial); the kernel has a wave-parallel sort and
// runs the linear merge on one lane with identical results.
struct HuffScratch {
    uint32_t key[N_LCODES + 2];      // (freq << 9) | sym, sorted ascending
    uint32_t iw[N_LCODES + 2];       // internal node weights
    uint16_t parent[2 * N_LCODES + 4];
    uint8_t depth[2 * N_LCODES + 4];
};

#if !defined(__HIP_DEVICE_COMPILE__)
static inline void sort_u32(uint32_t* a, int n)
{
    for (int i = 1; i < n; ++i) {
        uint32_t v = a[i];
        int j = i - 1;
        while (j >= 0 && a[j] > v) { a[j + 1] = a[j]; --j; }
        a[j + 1] = v;
    }
}

// freq[0..n) -> lens[0..n); returns the number of used symbols after dummies.
// shannon: the literal/length tree, which takes Shannon lengths when wide.
static inline int huff_lengths_host(const uint32_t* freq, int n, int max_bits, uint8_t* lens, HuffScratch& S,
                                    bool shannon = false)
{
    int m = 0;
    uint32_t f2[N_LCODES + 2];
    for (int i = 0; i < n; ++i) { f2[i] = freq[i]; lens[i] = 0; }
    int used = 0;
    for (int i = 0; i < n; ++i) used += f2[i] != 0;
    // the reference forces at least two codes (deflate_stream.ipp:911-925):
    // dummy symbols 0 and 1 (or the first unused) with frequency 1
    for (int i = 0; used < 2 && i < n; ++i)
        if (f2[i] == 0) { f2[i] = 1; ++used; }
    for (int i = 0; i < n; ++i)
        if (f2[i]) S.key[m++] = (f2[i] << 9) | (uint32_t)i;
    sort_u32(S.key, m);
    if (shannon && m >= (int)SHANNON_MIN) {
        uint32_t T = 0;
        for (int i = 0; i < m; ++i) T += S.key[i] >> 9;
        unsigned bl[MAX_BITS + 2] = {0};
        for (int i = 0; i < m; ++i) bl[shannon_len(S.key[i] >> 9, T, (unsigned)max_bits)]++;
        complete_code(bl, (unsigned)max_bits);
        int i = m - 1;   // most frequent first gets the shortest
        for (int bits = 1; bits <= max_bits; ++bits)
            for (unsigned c = 0; c < bl[bits]; ++c) S.depth[i--] = (uint8_t)bits;
        for (int j = 0; j < m; ++j) lens[S.key[j] & 511] = S.depth[j];
        return m;
    }
    // two-queue merge: leaves 0..m-1, internal nodes m..2m-2
    int li = 0, ii = 0;
    for (int k = 0; k < m - 1; ++k) {
        uint32_t w[2];
        int id[2];
        for (int t = 0; t < 2; ++t) {
            bool take_leaf = li < m && (ii >= k || (S.key[li] >> 9) <= S.iw[ii]);
            if (take_leaf) { w[t] = S.key[li] >> 9; id[t] = li++; }
            else { w[t] = S.iw[ii]; id[t] = m + ii++; }
        }
        S.iw[k] = w[0] + w[1];
        S.parent[id[0]] = S.parent[id[1]] = (uint16_t)(m + k);
    }
    // depths top-down (root = m + m - 2)
    int root = 2 * m - 2;
    S.depth[root] = 0;
    for (int v = root - 1; v >= 0; --v) S.depth[v] = (uint8_t)(S.depth[S.parent[v]] + 1);
    // clamp + overflow repair (reference: gen_bitlen)
    unsigned bl_count[MAX_BITS + 2] = {0};
    int overflow = 0;
    for (int i = 0; i < m; ++i) {
        int d = S.depth[i];
        if (d > max_bits) { d = max_bits; ++overflow; }
        bl_count[d]++;
    }
    if (overflow) {
        do {
            int bits = max_bits - 1;
            while (bl_count[bits] == 0) --bits;
            bl_count[bits]--;
            bl_count[bits + 1] += 2;
            bl_count[max_bits]--;
            overflow -= 2;
        } while (overflow > 0);
        // reassign: most frequent leaves (end of the sorted list) get the
        // shortest lengths
        int i = m - 1;
        for (int bits = 1; bits <= max_bits; ++bits)
            for (unsigned c = 0; c < bl_count[bits]; ++c) S.depth[i--] = (uint8_t)bits;
    }
    for (int i = 0; i < m; ++i) lens[S.key[i] & 511] = S.depth[i];
    return m;
}

// Canonical codes (bit-reversed for LSB-first emission), deflate_stream.ipp:115-141.
static inline void canonical_codes_host(const uint8_t* lens, int n, uint16_t* codes)
{
    unsigned cnt[MAX_BITS + 1] = {0}, next[MAX_BITS + 1];
    for (int i = 0; i < n; ++i) cnt[lens[i]]++;
    cnt[0] = 0;
    unsigned code = 0;
    for (int b = 1; b <= MAX_BITS; ++b) { code = (code + cnt[b - 1]) << 1; next[b] = code; }
    for (int i = 0; i < n; ++i) codes[i] = lens[i] ? (uint16_t)reverse_bits(next[lens[i]]++, lens[i]) : 0;
}
#endif

// Run-length coding of a code-length sequence (16: repeat previous 3-6,
// 17: zeros 3-10, 18: zeros 11-138), the reference's scan_tree/send_tree
// state machine (deflate_stream.ipp:978-1110).  `emit(sym, extra_bits,
// extra_value)` is called per code-length symbol.  `nextlen` past the end is
// a sentinel that never matches.
template <class Get, class Emit>
LZ_HD void rle_lengths(Get get, int count_n, Emit emit)
{
    int prevlen = -1, nextlen = get(0), count = 0;
    int max_count = 7, min_count = 4;
    if (nextlen == 0) { max_count = 138; min_count = 3; }
    for (int i = 0; i < count_n; ++i) {
        int curlen = nextlen;
        nextlen = i + 1 < count_n ? get(i + 1) : 0xFFFF;
        if (++count < max_count && curlen == nextlen) continue;
        if (count < min_count) {
            do { emit(curlen, 0, 0); } while (--count != 0);
        } else if (curlen != 0) {
            if (curlen != prevlen) { emit(curlen, 0, 0); --count; }
            emit(16, 2, count - 3);
        } else if (count <= 10) {
            emit(17, 3, count - 3);
        } else {
            emit(18, 7, count - 11);
        }
        count = 0;
        prevlen = curlen;
        if (nextlen == 0) { max_count = 138; min_count = 3; }
        else if (curlen == nextlen) { max_count = 6; min_count = 3; }
        else { max_count = 7; min_count = 4; }
    }
}

// The same coding, run by run: the symbols for one maximal run of r equal
// code lengths v (a run starts at a tree's first element or after a
// different value, so the state machine above always enters it with
// max_count 138 for zeros, 7 otherwise, and prevlen != v).  Lets the kernel
// code every run independently.
template <class Emit>
LZ_HD void rle_run(unsigned v, unsigned r, Emit emit)
{
    if (v == 0) {
        for (; r >= 138; r -= 138) emit(18, 7, 127);
        if (r >= 11) emit(18, 7, r - 11);
        else if (r >= 3) emit(17, 3, r - 3);
        else for (; r; --r) emit(0, 0, 0);
        return;
    }
    if (r < 4) {
        for (; r; --r) emit((int)v, 0, 0);
        return;
    }
    emit((int)v, 0, 0);
    if (r <= 7) {
        emit(16, 2, (int)r - 4);
        return;
    }
    emit(16, 2, 3);
    for (r -= 7; r >= 6; r -= 6) emit(16, 2, 3);
    if (r >= 3) emit(16, 2, (int)r - 3);
    else for (; r; --r) emit((int)v, 0, 0);
}

LZ_HD unsigned rle_run_count(unsigned v, unsigned r)
{
    if (v == 0) {
        const unsigned rem = r % 138;
        return r / 138 + (rem >= 3 ? 1 : rem);
    }
    if (r < 4) return r;
    if (r <= 7) return 2;
    const unsigned rem = (r - 7) % 6;
    return 2 + (r - 7) / 6 + (rem >= 3 ? 1 : rem);
}

// Order in which code-length code lengths are sent (RFC 1951 §3.2.7).
LZ_HD unsigned bl_order(unsigned i)
{
    const uint8_t o[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
    return o[i];
}

}  // namespace lz
