// pmd_deflate.hip -- batched raw-DEFLATE encode of permessage-deflate
// messages on gfx950 (CDNA4, wave64).  One wavefront owns one message at a
// time; messages are independent streams (no_context_takeover, a4 in
// SURVEY.md §8).
//
// Output per message is what Beast's deflater emits for one message driven
// by impl_base<true>::deflate (websocket/detail/impl_base.hpp:85-154): the
// message's blocks with BFINAL = 0, then the header bits of Flush::sync's
// empty stored block (000) and byte padding, with the 00 00 FF FF tail
// stripped.  The block contents are this kernel's own parse (the contract is
// a byte-identical round trip and a compressed-size tolerance, not
// bit-identity with zlib); tests/model/deflate_model.cpp is the host model of
// exactly this algorithm.
//
// Per 4 KiB chunk of a message (small messages: one chunk, no history; large
// messages: each chunk sees the previous 2 KiB as history, BPMD_CHUNK_HIST):
//   1. window -> LDS with 16-byte loads;
//   2. hash chains: 64 positions per step (two steps per iteration); LDS
//      exchange on a 2^11 head table links every position to the previous
//      one with the same hash of its next 4 bytes (lz::chain_hash);
//   3. parse: the chunk is cut into 64 lane segments; each lane runs the
//      reference's greedy (levels 1-3) or lazy (4-9) matcher with its
//      chain / lazy / nice / good limits (deflate_stream.hpp:571-590) over
//      its segment, writing match tokens by position (literals are taken
//      from the window afterwards) and a token-start bitmap;
//   4. boundary repair: an exclusive prefix max of segment end positions
//      gives each lane the first position it owns; tokens covered by an
//      earlier lane's last match are dropped and a straddling token keeps
//      its tail (a match with the same distance, or literals);
//   5. histograms with LDS atomics, Huffman code lengths (bitonic sort of
//      the used keys in registers, linear two-queue merge on one lane per
//      tree, depths by pointer jumping, the reference's 15-bit limit
//      repair; Shannon lengths for wide alphabets), canonical codes;
//   6. block choice as the reference's tr_flush_block (stored / fixed /
//      dynamic, deflate_stream.ipp:1425-1518);
//   7. bit packing: per-lane bit counts, wave prefix sum, ds_or into an LDS
//      bit buffer, dword stores to the output slot.
#include <atomic>
#include <type_traits>

#include <mutex>

#include <hipcub/hipcub.hpp>

#include "pmd_common.h"
#include "wave_util.h"
#include "lz_core.h"

namespace bpmd {
namespace dfl {

constexpr unsigned CHUNK = 4096;
constexpr unsigned HB = 11;
constexpr unsigned HSIZE = 1u << HB;
#ifndef BPMD_MIN_SEG
#define BPMD_MIN_SEG 16
#endif
constexpr unsigned MIN_SEG = BPMD_MIN_SEG;   // parse segment floor (bytes per lane) of a chunk without history
// A lane whose finds have walked more than BPMD_CHAIN_BUDGET chain candidates
// per 64 bytes of its parse segment walks at most 4 per find from then on
// (0 = no budget): the busiest lane sets a chunk's parse time
#ifndef BPMD_CHAIN_BUDGET
#define BPMD_CHAIN_BUDGET 0
#endif
// BPMD_DUAL_TEST: an iteration of the parse's chain walk that rejects its
// candidate outright (no longer match, no byte run to extend) also tests the
// next candidate of the chain, with the same limits and in the same order
// (1), and in the chunk kernel (chain cap 32) a third after that (2; the
// single-chunk kernel's walks are capped at 4 and lose with three)
// BPMD_MIN_SEG_HIST: the parse segment floor of a chunk with history bytes
// before it (the host model's min_seg with history)
#ifndef BPMD_MIN_SEG_HIST
#define BPMD_MIN_SEG_HIST 32
#endif
#ifndef BPMD_DUAL_TEST
#define BPMD_DUAL_TEST 2
#endif
// lz::INCOMP_DEN (lz_core.h): a chunk whose sampled positions almost never
// repeat their 4-byte key at the head of their chain is coded as literals
// without the parse
constexpr uint32_t NONE = 0xFFFFu;
constexpr unsigned NODES = 576 + 64;          // lit tree nodes [0, 576), dist tree [576, 640)
constexpr unsigned NODES_PER_LANE = NODES / WAVE;
constexpr unsigned DIST_IDX = 288;            // dist symbol s lives at lens/codes[288 + s]

struct HuffLds {
    uint32_t lf[288];
    uint32_t df[32];
    uint32_t bf[20];
    union {
        uint32_t keys[512];          // sort buffer (tree build)
        struct {
            uint16_t sym[320];       // run-length coded code lengths: sym | extra << 5
            uint64_t start[6];       // run-start bitmap over the code-length sequence
            uint32_t tkey[24];       // code-length-code tree keys
        } r;
    };
    uint16_t iw[320];            // internal node weights: lit [0, 288), dist [288, 320)
    uint16_t parent[NODES];
    uint8_t depth[NODES];
    uint8_t lens[320];
    uint32_t codes[320];         // reversed code | len << 16
    uint32_t blcount[2][16];
    uint8_t bll[20];
    uint32_t blc[20];
    uint32_t misc[8];
};

template <int HIST>
struct alignas(16) DefLds {
    static constexpr unsigned W = HIST + CHUNK;
    // window bytes at byte offset `ws`; output bit buffer after the parse.  The
    // window has no slack (ws = 0): single-chunk 20480 B per wave, 8 waves per
    // CU, history kernel (2048 B of history) 26624 B, 6 waves per CU; reads past the data land in `a` and are clamped by the lookahead, and
    // the bit buffer's last words spill into lf[] only after lf is dead.
    uint32_t win[W / 4];
    union {
        uint16_t prev[W < 4096 ? 4096 : W];
        HuffLds h;
    } a;
    union {
        uint32_t head[HSIZE];
        uint16_t tok[CHUNK];
    } b;
};

static_assert(sizeof(DefLds<0>) == 160 * 1024 / 8, "single-chunk deflate LDS: 8 waves per CU");
static_assert(sizeof(DefLds<2048>) == 26624, "history deflate LDS: 6 waves per CU");
static_assert(offsetof(DefLds<0>, b) % 16 == 0 && offsetof(DefLds<2048>, b) % 16 == 0, "tok[] is cleared with 16-byte stores");
static_assert(offsetof(HuffLds, lf) == 0, "bit buffer spill lands in lf[] (dead while packing)");

struct Params {
    lz::Level L;
    int strategy;        // bpmd_strategy
    unsigned max_dist;   // w_size - MIN_LOOKAHEAD
    unsigned chain;      // chain limit (level table, capped for single-chunk messages)
    uint32_t* out_bits;  // optional: payload length in bits before the sync-marker tail
    const uint32_t* mask_key;   // optional: mask payload i with key i on the way out (write.hpp:679-685)
    const uint32_t* hist_len;   // optional (context takeover): plaintext bytes before message i usable as history
};

// Diagnostic build only (-DBPMD_PROF): per-phase wave cycles and counts.
__device__ unsigned long long g_dprof[24];
#ifdef BPMD_PROF
struct Prof {
    unsigned long long c[24];
    unsigned long long t;
    __device__ Prof() : t(__builtin_amdgcn_s_memtime()) { for (int i = 0; i < 24; ++i) c[i] = 0; }
    __device__ void lap(int i) { const unsigned long long t2 = __builtin_amdgcn_s_memtime(); c[i] += t2 - t; t = t2; }
    __device__ void cnt(int i, unsigned long long n) { c[i] += n; }
    __device__ void flush() { if (lane_id() == 0) for (int i = 0; i < 24; ++i) atomicAdd(&g_dprof[i], c[i]); }
};
#else
struct Prof {
    __device__ void lap(int) {}
    __device__ void cnt(int, unsigned long long) {}
    __device__ void flush() {}
};
#endif

// ------------------------------------------------------------------ window

struct Win {
    const uint32_t* w;
    const uint8_t* b;
    unsigned ws;
    __device__ __forceinline__ uint32_t byte(unsigned i) const { return b[ws + i]; }
    __device__ __forceinline__ uint32_t dw(unsigned i) const
    {
        const unsigned j = ws + i;
        const uint32_t lo = w[j >> 2], hi = w[(j >> 2) + 1];
        return __builtin_amdgcn_alignbit(hi, lo, (j & 3) * 8);
    }
    // 8 bytes starting at window byte i (little-endian)
    __device__ __forceinline__ uint64_t qw(unsigned i) const
    {
        const unsigned j = ws + i, k = j >> 2, sh = (j & 3) * 8;
        const uint32_t w0 = w[k], w1 = w[k + 1], w2 = w[k + 2];
        return ((uint64_t)__builtin_amdgcn_alignbit(w2, w1, sh) << 32) | __builtin_amdgcn_alignbit(w1, w0, sh);
    }
};

// a wave-uniform value moved into a VGPR (see the parse loop)
__device__ __forceinline__ unsigned to_vgpr(unsigned x)
{
    unsigned v;
    asm volatile("v_mov_b32 %0, %1" : "=v"(v) : "s"(x));
    return v;
}

// number of equal leading bytes of two 8-byte groups (8 = all)
__device__ __forceinline__ unsigned eq_bytes(uint64_t a, uint64_t b)
{
    const uint64_t x = a ^ b;
    return x ? (unsigned)__builtin_ctzll(x) >> 3 : 8u;
}

template <int HIST>
__device__ __forceinline__ unsigned load_window(DefLds<HIST>& S, const uint8_t* src, unsigned nbytes)
{
    const uintptr_t a = (uintptr_t)src;
    const unsigned s = (unsigned)(a & 15);
    const uint4* g = (const uint4*)(a - s);
    const unsigned units = (s + nbytes + 15) >> 4;
    uint4* l = (uint4*)S.win;
    // aligned 16-byte loads (never past the aligned unit holding the last
    // byte), shifted down by s bytes so the window starts at LDS byte 0
    const unsigned q = s >> 2, r = (s & 3) * 8;
    for (unsigned u = lane_id(); u < ((nbytes + 15) >> 4); u += WAVE) {
        const uint4 x = g[u];
        const uint4 y = u + 1 < units ? g[u + 1] : make_uint4(0, 0, 0, 0);
        const uint32_t d0 = q == 0 ? x.x : q == 1 ? x.y : q == 2 ? x.z : x.w;
        const uint32_t d1 = q == 0 ? x.y : q == 1 ? x.z : q == 2 ? x.w : y.x;
        const uint32_t d2 = q == 0 ? x.z : q == 1 ? x.w : q == 2 ? y.x : y.y;
        const uint32_t d3 = q == 0 ? x.w : q == 1 ? y.x : q == 2 ? y.y : y.z;
        const uint32_t d4 = q == 0 ? y.x : q == 1 ? y.y : q == 2 ? y.z : y.w;
        l[u] = make_uint4(__builtin_amdgcn_alignbit(d1, d0, r), __builtin_amdgcn_alignbit(d2, d1, r),
                          __builtin_amdgcn_alignbit(d3, d2, r), __builtin_amdgcn_alignbit(d4, d3, r));
    }
    return 0;
}

// ---------------------------------------------------------------- bit sink

struct BitOr {
    uint32_t* w;
    uint32_t wpos;
    unsigned nb;
    uint64_t acc;
    __device__ __forceinline__ void start(uint32_t* words, uint32_t bitpos)
    {
        w = words;
        wpos = bitpos >> 5;
        nb = bitpos & 31;
        acc = 0;
    }
    __device__ __forceinline__ void put(uint32_t v, unsigned n)
    {
        acc |= (uint64_t)v << nb;
        nb += n;
        if (nb >= 32) {
            atomicOr(&w[wpos], (uint32_t)acc);
            acc >>= 32;
            nb -= 32;
            ++wpos;
        }
    }
    __device__ __forceinline__ void flush()
    {
        if (nb) atomicOr(&w[wpos], (uint32_t)acc);
        nb = 0;
        acc = 0;
    }
};

// ------------------------------------------------------------- per-lane tokens

struct LaneToks {
    uint64_t kept;       // token starts (relative to a) owned after repair
    unsigned a, b;       // segment [a, b) in window coordinates
    unsigned lastdist;   // distance of a match starting at b - 1
    unsigned rem_kind;   // 0 none, 1 match, 2 literals
    unsigned rem_len, rem_dist, rem_b0, rem_b1;
};

// Calls f(is_match, lit_or_len, dist) for every owned token in order.
// SINGLE: one call site, for bodies that are cheap to run whole for either
// kind (a wave then runs one body per token instead of both, which pays off
// when matches are common); otherwise a literal and a match call site (the
// wave skips the match body when no lane has a match: binary data).
// Tokens are taken four at a time, their tok[] entries (and the distance
// slots after them) loaded together before the bodies run, so a lane waits
// for one LDS round trip per four tokens instead of one per token.
// FILL: the first pass after the parse, which leaves literal tokens zero in
// tok[]: their bytes come from the window and are stored for later passes.
// G: tokens whose entries are loaded together -- 4 in the single-chunk
// kernel (C3 deflate +2 %), 1 in the chunk kernel, where the grouped loop
// cost the parse's register allocation 8 % on C5
// (profiles/r04zb_ab_token_groups.log)
template <bool SINGLE = false, bool FILL = false, int G = 1, class F>
__device__ __forceinline__ void for_tokens(const LaneToks& T, uint16_t* tok, unsigned a0, F f,
                                           const uint8_t* wb = nullptr)
{
    if (T.rem_kind == 1) f(true, T.rem_len, T.rem_dist);
    else if (T.rem_kind == 2) {
        f(false, T.rem_b0, 0u);
        if (T.rem_len > 1) f(false, T.rem_b1, 0u);
    }
    uint64_t m = T.kept;
    while (m) {
        unsigned pos[G];
        bool v[G];
#pragma unroll
        for (int j = 0; j < G; ++j) {
            v[j] = m != 0;
            pos[j] = T.a + (v[j] ? (unsigned)__builtin_ctzll(m) : 0u);
            m &= m - 1;
        }
        uint32_t e[G], dn[G], lb[G];
#pragma unroll
        for (int j = 0; j < G; ++j) {
            e[j] = tok[pos[j] - a0];
            dn[j] = tok[(pos[j] + 1 < T.b ? pos[j] + 1 : pos[j]) - a0];
            if (FILL) lb[j] = wb[pos[j]];
        }
#pragma unroll
        for (int j = 0; j < G; ++j) {
            if (!v[j]) continue;
            const bool mt = (e[j] & 0x8000u) != 0;
            const unsigned d = pos[j] + 1 < T.b ? dn[j] + 1 : T.lastdist;
            uint32_t lit = e[j];
            if (FILL && !mt) {
                lit = lb[j];
                tok[pos[j] - a0] = (uint16_t)lit;
            }
            if (SINGLE) {
                f(mt, mt ? (e[j] & 0xFFu) + 3 : lit, d);
            } else if (mt) {
                f(true, (e[j] & 0xFFu) + 3, d);
            } else {
                f(false, lit, 0u);
            }
        }
    }
}

__device__ __forceinline__ uint32_t pack_code(uint32_t code, unsigned len)
{
    return (len ? lz::reverse_bits(code, len) : 0u) | (len << 16);
}

// --------------------------------------------------------------- Huffman

// Two-queue merge for one tree, run by one lane (lit on lane 0, dist on lane
// 1 at the same time).  Leaves are the sorted keys [kb, kb + m); internal
// node k is node m + k; parent[] gets node ids relative to the tree base.
// Branch-free: each queue's next TWO weights are held in registers, a pick
// is a compare and selects, and the weight two places ahead in the queue it
// took from is loaded for the pick after next (a lane-divergent branchy pick
// spent most of its instructions on exec masks and waited on every load).
__device__ __forceinline__ void merge_tree(HuffLds& H, unsigned kb, unsigned m, unsigned ib, unsigned pb)
{
    auto leaf = [&](unsigned i) -> uint32_t {   // weight of leaf i, 0 past the leaves
        const uint32_t k = H.keys[kb + (i < m ? i : m - 1)];
        return i < m ? (k >> 9) & 0x3FFFFFu : 0u;
    };
    unsigned li = 0, ii = 0;
    uint32_t kw = leaf(0), kw1 = leaf(1);   // leaves li, li + 1
    uint32_t iq = 0, iq1 = 0;               // internal ii, ii + 1 (valid below k)
    for (unsigned k = 0; k + 1 < m; ++k) {
        uint32_t w[2];
        unsigned id[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const bool have_i = ii < k;
            const bool take_leaf = li < m && (!have_i || kw <= iq);
            w[t] = take_leaf ? kw : iq;
            id[t] = take_leaf ? li : m + ii;
            // the queue that gave up its head: next weight moves up, the one
            // after it is loaded (internal weights past k - 1 are patched below)
            const uint32_t nl = leaf(li + 2);
            const uint32_t ni = H.iw[ib + (ii + 2 < 320 - ib ? ii + 2 : ii)];
            kw = take_leaf ? kw1 : kw;
            kw1 = take_leaf ? nl : kw1;
            iq = take_leaf ? iq : iq1;
            iq1 = take_leaf ? iq1 : (uint32_t)ni;
            li += take_leaf ? 1u : 0u;
            ii += take_leaf ? 0u : 1u;
        }
        const uint32_t ws = (uint16_t)(w[0] + w[1]);
        H.iw[ib + k] = (uint16_t)ws;
        H.parent[pb + id[0]] = (uint16_t)(m + k);
        H.parent[pb + id[1]] = (uint16_t)(m + k);
        // the new node is the queue's head or second when the queue had fewer
        iq = ii == k ? ws : iq;
        iq1 = ii + 1 == k ? ws : iq1;
    }
}

// The code-length code (19 symbols, lengths <= 7): Huffman lengths as
// lz::huff_lengths_host computes them, then canonical codes, the count of
// code-length code lengths sent (HCLEN + 4) and the dynamic header's size
// (deflate_stream.ipp:1396-1418 build_bl_tree, 1420-1438 send_all_trees).
// Wave-parallel: symbol s in lane s, ranks by comparing each key with every
// other key, the 18-step merge and the depths as wave-uniform loops over
// v_readlane (no LDS round trip per step).
__device__ void bl_tree_wave(HuffLds& H, uint32_t& hdr_bits, uint32_t& nbl_out)
{
    using namespace lz;
    const unsigned lane = lane_id();
    const bool sl = lane < (unsigned)N_BLCODES;
    const uint32_t f0 = sl ? H.bf[lane] : 0u;
    // at least two codes: the first unused symbols get frequency 1
    const unsigned used = (unsigned)__builtin_popcountll(ballot(f0 != 0));
    const uint64_t zero = ballot(sl && f0 == 0);
    const uint32_t f = (sl && f0 == 0 && used < 2 && popc_below(zero) < 2 - used) ? 1u : f0;
    const uint32_t key = f ? (f << 9) | lane : 0xFFFFFFFFu;
    const unsigned m = (unsigned)__builtin_popcountll(ballot(f != 0));
    // ascending rank of each used key (keys are distinct)
    unsigned rank = 0;
#pragma unroll
    for (unsigned j = 0; j < (unsigned)N_BLCODES; ++j) {
        const uint32_t kj = (uint32_t)__builtin_amdgcn_readlane((int)key, (int)j);
        rank += kj < key ? 1u : 0u;
    }
    if (f) H.r.tkey[rank] = key;
    wave_sync();
    const uint32_t sorted = lane < m ? H.r.tkey[lane] : 0u;   // lane r: the r-th smallest key
    const uint32_t sw = sorted >> 9;
    // two-queue merge (leaves 0..m-1, internal nodes m..2m-2)
    uint32_t iw = 0, par = 0;
    {
        unsigned li = 0, ii = 0;
        uint32_t kw = (uint32_t)__builtin_amdgcn_readlane((int)sw, 0);
        for (unsigned k = 0; k + 1 < m; ++k) {
            uint32_t w[2];
            unsigned id[2];
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                const uint32_t iwv = ii < k ? (uint32_t)__builtin_amdgcn_readlane((int)iw, (int)ii) : 0xFFFFFFFFu;
                if (li < m && (ii >= k || kw <= iwv)) {
                    w[t] = kw;
                    id[t] = li++;
                    kw = li < m ? (uint32_t)__builtin_amdgcn_readlane((int)sw, (int)li) : 0u;
                } else {
                    w[t] = iwv;
                    id[t] = m + ii++;
                }
            }
            iw = lane == k ? (uint32_t)(uint16_t)(w[0] + w[1]) : iw;
            par = (lane == id[0] || lane == id[1]) ? m + k : par;
        }
    }
    // depths top-down (root = 2m - 2; node v's parent is above it)
    uint32_t dep = 0;
    for (int v = (int)(2 * m) - 3; v >= 0; --v) {
        const unsigned p = (unsigned)__builtin_amdgcn_readlane((int)par, v);
        const uint32_t d = (uint32_t)__builtin_amdgcn_readlane((int)dep, (int)p) + 1u;
        dep = lane == (unsigned)v ? d : dep;
    }
    // length limit (deflate_stream.ipp gen_bitlen): clamp, repair the Kraft
    // overflow, reassign lengths in frequency order
    uint32_t len = dep;
    const uint64_t over_m = ballot(lane < m && dep > (uint32_t)MAX_BL_BITS);
    if (over_m) {
        int overflow = (int)__builtin_popcountll(over_m);
        uint32_t blc = 0;   // lane b: leaves of length b
#pragma unroll
        for (unsigned b2 = 1; b2 <= (unsigned)MAX_BL_BITS; ++b2) {
            const unsigned c = (unsigned)__builtin_popcountll(
                ballot(lane < m && (dep > (uint32_t)MAX_BL_BITS ? (uint32_t)MAX_BL_BITS : dep) == b2));
            blc = lane == b2 ? c : blc;
        }
        while (overflow > 0) {
            unsigned bits = MAX_BL_BITS - 1;
            while (__builtin_amdgcn_readlane((int)blc, (int)bits) == 0) --bits;
            blc = lane == bits ? blc - 1u : lane == bits + 1 ? blc + 2u : blc;
            blc = lane == (unsigned)MAX_BL_BITS ? blc - 1u : blc;
            overflow -= 2;
        }
        // the r-th most frequent leaf (leaf m - 1 - r) gets the r-th shortest length
        const unsigned r = m - 1 - lane;
        unsigned cum = 0, bits = MAX_BL_BITS;
        for (unsigned b2 = MAX_BL_BITS; b2 >= 1; --b2) {
            cum = 0;
            for (unsigned b3 = 1; b3 <= b2; ++b3) cum += (uint32_t)__builtin_amdgcn_readlane((int)blc, (int)b3);
            if (r < cum) bits = b2;
        }
        len = bits;
    }
    // lengths by symbol
    if (sl) H.bll[lane] = 0;
    wave_sync();
    if (lane < m) H.bll[sorted & 511] = (uint8_t)len;
    wave_sync();
    const uint32_t bl = sl ? H.bll[lane] : 0u;
    // canonical codes: next_code per length, then rank among equal lengths by symbol
    uint32_t code = 0, next = 0;
#pragma unroll
    for (unsigned b2 = 1; b2 <= (unsigned)MAX_BL_BITS; ++b2) {
        const uint64_t mb = ballot(sl && bl == b2);
        if (bl == b2) code = next + popc_below(mb);
        next = (next + (uint32_t)__builtin_popcountll(mb)) << 1;
    }
    if (sl) H.blc[lane] = bl ? pack_code(code, bl) : 0u;
    // code lengths sent: down to the last nonzero in bl_order, at least 4
    const bool nz = sl && H.bll[bl_order(sl ? lane : 0u)] != 0;
    const uint64_t nzm = ballot(nz);
    const unsigned nbl = nzm ? 64u - (unsigned)__builtin_clzll(nzm) : 0u;
    nbl_out = nbl < 4 ? 4u : nbl;
    const uint32_t xb = lane == 16 ? 2u : lane == 17 ? 3u : lane == 18 ? 7u : 0u;
    hdr_bits = 3 + 5 + 5 + 4 + 3 * nbl_out + wave_sum(sl ? f0 * (bl + xb) : 0u);
    wave_sync();
}

// Lit/len and distance code lengths + canonical codes for the current
// histograms (H.lf with EOB counted, H.df).  Whole wave.
// Bitonic sort (ascending) of the 64 * R keys at k[0, 64 R), element
// lane * R + r in register r of its lane: partners less than R apart are
// compare-exchanged in registers, the others across lanes by xor shuffles.
template <int R>
__device__ __forceinline__ void sort_keys_reg(uint32_t* keys)
{
    const unsigned lane = lane_id();
    uint32_t v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) v[r] = keys[lane * R + r];
#pragma unroll
    for (unsigned k = 2; k <= 64u * R; k <<= 1) {
#pragma unroll
        for (unsigned j = k >> 1; j > 0; j >>= 1) {
            if (j < (unsigned)R) {
#pragma unroll
                for (unsigned r = 0; r < (unsigned)R; ++r) {
                    if (r & j) continue;
                    const unsigned e = lane * R + r;
                    const bool up = (e & k) == 0;
                    const uint32_t x = v[r], y = v[r ^ j];
                    const bool sw = (x > y) == up;
                    v[r] = sw ? y : x;
                    v[r ^ j] = sw ? x : y;
                }
            } else {
                const unsigned lm = j / R;   // partner lane distance
                const bool lower = (lane & lm) == 0;
#pragma unroll
                for (unsigned r = 0; r < (unsigned)R; ++r) {
                    const unsigned e = lane * R + r;
                    const bool up = (e & k) == 0;
                    const uint32_t y = (uint32_t)__shfl_xor((int)v[r], (int)lm);
                    const uint32_t mn = v[r] < y ? v[r] : y, mx = v[r] < y ? y : v[r];
                    v[r] = (lower == up) ? mn : mx;
                }
            }
        }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) keys[lane * R + r] = v[r];
}

__device__ void build_trees(HuffLds& H, Prof& pf)
{
    const unsigned lane = lane_id();
    // --- keys, with the reference's "at least two codes" dummies
    unsigned used_l = 0, used_d = 0;
    for (unsigned i = lane; i < 320; i += WAVE) {
        used_l += (i < 286 && H.lf[i] != 0);
        used_d += (i >= DIST_IDX && i < DIST_IDX + 30 && H.df[i - DIST_IDX] != 0);
    }
    used_l = wave_sum(used_l);
    used_d = wave_sum(used_d);
    for (unsigned i = lane; i < 512; i += WAVE) {
        uint32_t k = 0xFFFFFFFFu;
        if (i < 286 && H.lf[i]) k = (H.lf[i] << 9) | i;
        else if (i >= DIST_IDX && i < DIST_IDX + 30 && H.df[i - DIST_IDX]) k = 0x80000000u | (H.df[i - DIST_IDX] << 9) | (i - DIST_IDX);
        H.keys[i] = k;
    }
    wave_sync();
    if (lane == 0) {
        for (unsigned i = 0; used_l < 2 && i < 286; ++i)
            if (H.lf[i] == 0) { H.keys[i] = (1u << 9) | i; ++used_l; }
        for (unsigned i = 0; used_d < 2 && i < 30; ++i)
            if (H.df[i] == 0) { H.keys[DIST_IDX + i] = 0x80000000u | (1u << 9) | i; ++used_d; }
    }
    used_l = used_l < 2 ? 2 : used_l;
    used_d = used_d < 2 ? 2 : used_d;
    wave_sync();
    // --- compact the used keys to the front (lit keys stay below dist keys:
    // bit 31) so the sort covers the next power of two >= their count, not 512
    const unsigned used = (unsigned)__builtin_amdgcn_readfirstlane((int)(used_l + used_d));
    const unsigned P = used <= 128 ? 128u : used <= 256 ? 256u : 512u;
    {
        uint32_t kv[5];
#pragma unroll
        for (unsigned t = 0; t < 5; ++t) kv[t] = H.keys[lane + t * WAVE];
        wave_sync();
        unsigned at = 0;
#pragma unroll
        for (unsigned t = 0; t < 5; ++t) {
            const bool v = kv[t] != 0xFFFFFFFFu;
            const uint64_t bm = ballot(v);
            if (v) H.keys[at + popc_below(bm)] = kv[t];
            at += (unsigned)__builtin_popcountll(bm);
        }
        for (unsigned i = at + lane; i < P; i += WAVE) H.keys[i] = 0xFFFFFFFFu;
        wave_sync();
    }
#ifdef BPMD_SORT_LDS   // diagnostics: round 3's bitonic sort through LDS
    // --- bitonic sort of P keys (P / 128 compare-exchanges per lane per stage)
    for (unsigned k = 2; k <= P; k <<= 1) {
        for (unsigned j = k >> 1; j > 0; j >>= 1) {
#pragma unroll
            for (unsigned t = 0; t < 4; ++t) {
                if (t >= P / 128) break;
                const unsigned i = lane + t * WAVE;
                const unsigned lo = ((i & ~(j - 1)) << 1) | (i & (j - 1)), hi = lo + j;
                const uint32_t x = H.keys[lo], y = H.keys[hi];
                const bool up = (lo & k) == 0;
                if ((x > y) == up) { H.keys[lo] = y; H.keys[hi] = x; }
            }
            wave_sync();
        }
    }
#else
    // --- bitonic sort of P keys in registers (P / 64 per lane)
    if (P == 128) sort_keys_reg<2>(H.keys);
    else if (P == 256) sort_keys_reg<4>(H.keys);
    else sort_keys_reg<8>(H.keys);
    wave_sync();
#endif
    pf.lap(4);
    const unsigned ml = used_l, md = used_d;
    // a wide literal/length alphabet takes Shannon lengths (lz_core.h), no merge
    const bool shan = ml >= lz::SHANNON_MIN;
    // --- merges (lane 0: lit, lane 1: dist)
    if (lane < 2) {
        if (lane == 0) { if (!shan) merge_tree(H, 0, ml, 0, 0); }
        else merge_tree(H, ml, md, 288, 576);
    }
    wave_sync();
    pf.lap(5);
    // --- depths by pointer jumping over both trees
    const unsigned root_l = 2 * ml - 2, root_d = 576 + 2 * md - 2;
    {
        uint32_t anc[NODES_PER_LANE], dep[NODES_PER_LANE];
#pragma unroll
        for (unsigned t = 0; t < NODES_PER_LANE; ++t) {
            const unsigned v = lane + t * WAVE;
            const bool lit = v < 576;
            const unsigned root = lit ? root_l : root_d;
            const bool valid = lit ? (!shan && v <= root_l) : (v >= 576 && v <= root_d);
            anc[t] = valid && v != root ? (unsigned)H.parent[v] + (lit ? 0u : 576u) : v;
            dep[t] = valid && v != root ? 1u : 0u;
            if (valid) {
                H.parent[v] = (uint16_t)anc[t];
                H.depth[v] = (uint8_t)dep[t];
            }
        }
        wave_sync();
        for (int round = 0; round < 10; ++round) {
            bool any = false;
#pragma unroll
            for (unsigned t = 0; t < NODES_PER_LANE; ++t) {
                const unsigned v = lane + t * WAVE;
                const unsigned a = anc[t];
                if (a != v) {
                    const unsigned aa = H.parent[a];
                    if (aa != a) any = true;
                    dep[t] += H.depth[a];
                    anc[t] = aa;
                }
            }
            wave_sync();
#pragma unroll
            for (unsigned t = 0; t < NODES_PER_LANE; ++t) {
                const unsigned v = lane + t * WAVE;
                const bool lit = v < 576;
                const bool valid = lit ? (!shan && v <= root_l) : (v >= 576 && v <= root_d);
                if (valid) {
                    H.parent[v] = (uint16_t)anc[t];
                    H.depth[v] = (uint8_t)dep[t];
                }
            }
            wave_sync();
            if (!ballot(any)) break;
        }
    }
    pf.lap(6);
    // --- length limit (15) and per-length counts
    for (unsigned i = lane; i < 32; i += WAVE) H.blcount[i >> 4][i & 15] = 0;
    wave_sync();
    uint32_t T = 0;   // Shannon lengths: the literal/length alphabet's total
    if (shan) {
        for (unsigned i = lane; i < ml; i += WAVE) T += H.keys[i] >> 9;
        T = wave_sum(T);
    }
    unsigned ovf_l = 0, ovf_d = 0;
    for (unsigned i = lane; i < ml + md; i += WAVE) {
        const bool lit = i < ml;
        const unsigned v = lit ? i : 576 + (i - ml);
        unsigned d = lit && shan ? lz::shannon_len(H.keys[i] >> 9, T, lz::MAX_BITS) : H.depth[v];
        if (d > lz::MAX_BITS) { d = lz::MAX_BITS; if (lit) ++ovf_l; else ++ovf_d; }
        atomicAdd(&H.blcount[lit ? 0 : 1][d], 1u);
    }
    ovf_l = wave_sum(ovf_l);
    ovf_d = wave_sum(ovf_d);
    wave_sync();
    if (ovf_l | ovf_d | (shan ? 1u : 0u)) {
        if (lane == 0 && shan) lz::complete_code(H.blcount[0], lz::MAX_BITS);
        if (lane < 2 && !(lane == 0 && shan)) {
            int overflow = (int)(lane == 0 ? ovf_l : ovf_d);
            uint32_t* bc = H.blcount[lane];
            while (overflow > 0) {
                unsigned bits = lz::MAX_BITS - 1;
                while (bc[bits] == 0) --bits;
                bc[bits]--;
                bc[bits + 1] += 2;
                bc[lz::MAX_BITS]--;
                overflow -= 2;
            }
        }
        wave_sync();
        // reassign: the r-th most frequent leaf gets the r-th shortest length
        for (unsigned i = lane; i < ml + md; i += WAVE) {
            const bool lit = i < ml;
            if ((lit ? (ovf_l || shan) : ovf_d) == 0) continue;
            const unsigned m = lit ? ml : md, leaf = lit ? i : i - ml;
            const unsigned r = m - 1 - leaf;
            const uint32_t* bc = H.blcount[lit ? 0 : 1];
            unsigned cum = 0, bits = 1;
            for (; bits <= lz::MAX_BITS; ++bits) {
                cum += bc[bits];
                if (r < cum) break;
            }
            H.depth[lit ? leaf : 576 + leaf] = (uint8_t)bits;
        }
        wave_sync();
    }
    // --- scatter lengths to symbols
    for (unsigned i = lane; i < 320; i += WAVE) H.lens[i] = 0;
    wave_sync();
    for (unsigned i = lane; i < ml + md; i += WAVE) {
        const bool lit = i < ml;
        const uint32_t key = H.keys[i];
        const unsigned sym = key & 511;
        H.lens[lit ? sym : DIST_IDX + sym] = H.depth[lit ? i : 576 + (i - ml)];
    }
    wave_sync();
}

// Canonical codes for lens[base, base + n) into codes[].
__device__ __forceinline__ void canonical_codes(HuffLds& H, unsigned base, unsigned n)
{
    const unsigned lane = lane_id();
    uint32_t next = 0;   // lane b (1..15) holds next_code[b]
    {
        // counts per length
        uint32_t cnt = 0;
        for (unsigned c = 0; c < n; c += WAVE) {
            const unsigned i = c + lane;
            const unsigned len = i < n ? H.lens[base + i] : 0;
            for (unsigned b = 1; b <= lz::MAX_BITS; ++b) {
                const unsigned k = (unsigned)__builtin_popcountll(ballot(len == b));
                if (lane == b) cnt += k;
            }
        }
        // next_code[b] = (next_code[b-1] + cnt[b-1]) << 1
        uint32_t code = 0;
        for (unsigned b = 1; b <= lz::MAX_BITS; ++b) {
            const uint32_t cprev = (uint32_t)__builtin_amdgcn_readlane((int)cnt, (int)(b - 1));
            code = (code + (b == 1 ? 0u : cprev)) << 1;
            if (lane == b) next = code;
        }
    }
    for (unsigned c = 0; c < n; c += WAVE) {
        const unsigned i = c + lane;
        const unsigned len = i < n ? H.lens[base + i] : 0;
        uint32_t code = 0;
        for (unsigned b = 1; b <= lz::MAX_BITS; ++b) {
            const uint64_t m = ballot(len == b);
            const uint32_t nb = (uint32_t)__builtin_amdgcn_readlane((int)next, (int)b);
            if (len == b) code = nb + popc_below(m);
            if (lane == b) next += (uint32_t)__builtin_popcountll(m);
        }
        if (i < n) H.codes[base + i] = pack_code(code, len);
    }
    wave_sync();
}

__device__ __forceinline__ unsigned fixed_code(unsigned sym, unsigned& len)
{
    if (sym < 144) { len = 8; return 0x30 + sym; }
    if (sym < 256) { len = 9; return 0x190 + (sym - 144); }
    if (sym < 280) { len = 7; return sym - 256; }
    len = 8;
    return 0xC0 + (sym - 280);
}

// ------------------------------------------------------------------ kernel

struct MsgOut {
    uint8_t* dst;
    uint32_t cap;
    uint32_t opos;     // bytes completed
    uint32_t carry;    // pending partial byte
    unsigned cbits;    // valid bits in carry
    bool overflow;
    uint32_t key;      // masking key, 0 = unmasked: payload byte j ^= key >> 8 (j % 4) (mask.ipp:38-59)
    bool stored;       // the last chunk was written as a stored block
};

__device__ __forceinline__ void put_bytes_global(MsgOut& o, const uint8_t* src_lds, unsigned ob, unsigned nbytes)
{
    // LDS byte ob + j -> dst[opos + j]; LDS word k <-> global dword (dst + opos - ob + 4k)
    const unsigned lane = lane_id();
    uint8_t* d = o.dst + o.opos;
    const unsigned end = ob + nbytes;
    const unsigned wfirst = (ob + 3) >> 2, wlast = end >> 2;   // whole words [wfirst, wlast)
    uint32_t* gw = (uint32_t*)(d - ob);
    const uint32_t* lw = (const uint32_t*)src_lds;
    // global dword k holds payload bytes opos - ob + 4k + t: key byte (opos - ob + t) % 4
    const uint32_t kw = __builtin_amdgcn_alignbit(o.key, o.key, 8u * ((o.opos - ob) & 3u));
    for (unsigned k = wfirst + lane; k < wlast; k += WAVE) gw[k] = lw[k] ^ kw;
    // edges
    if (lane < 4) {
        const unsigned j = ob + lane;
        if (j < end && j < wfirst * 4) d[j - ob] = src_lds[j] ^ (uint8_t)(kw >> (8 * (j & 3)));
    } else if (lane < 8) {
        const unsigned j = wlast * 4 + (lane - 4);
        if (j >= ob && j < end && j >= wfirst * 4) d[j - ob] = src_lds[j] ^ (uint8_t)(kw >> (8 * (j & 3)));
    }
}

template <int HIST>
__device__ void deflate_chunk(DefLds<HIST>& S, const uint8_t* msg, unsigned base, unsigned len, unsigned hist,
                              const Params& P, MsgOut& o, Prof& pf)
{
    constexpr int TOKG = HIST == 0 ? 4 : 1;
    using namespace lz;
    const unsigned lane = lane_id();
    const unsigned cend = base + CHUNK < len ? base + CHUNK : len;
    // the window reaches HIST bytes back; for the first chunk of a context-
    // takeover message those are the connection's earlier plaintext (hist
    // bytes before the message)
    const unsigned back = base + hist < (unsigned)HIST ? base + hist : (unsigned)HIST;
    const int wb = (int)base - (int)back;
    const unsigned wn = cend - base + back, a0 = back, clen = cend - base;
    const bool stored_only = P.L.parser == P_STORED;

    Win W;
    W.w = S.win;
    W.b = (const uint8_t*)S.win;
    W.ws = 0;
    HuffLds& H = S.a.h;
    unsigned kind = 0;   // 0 stored, 1 fixed, 2 dynamic
    LaneToks T;
    T.kept = 0;
    T.rem_kind = 0;
    T.rem_len = T.rem_dist = T.rem_b0 = T.rem_b1 = 0;
    T.lastdist = 0;
    T.a = T.b = 0;
    uint32_t hdr_bits = 0, blcodes = 0, lcodes = 0, dcodes = 0, nrle = 0;
    uint32_t n_tok = 0, n_match = 0;   // tokens and matches of the chunk (after the histogram pass: whole wave)

    if (!stored_only) {
        W.ws = load_window(S, msg + wb, wn);
        const bool chains = P.strategy != 2 && P.strategy != 3;
        if (chains) {
            uint4* h4 = (uint4*)S.b.head;
            for (unsigned i = lane; i < HSIZE / 4; i += WAVE) h4[i] = make_uint4(~0u, ~0u, ~0u, ~0u);
        }
        wave_sync();
        pf.lap(0);
        // ---- hash chains
        if (chains) {
            // 64 positions per step: link each position to the head of its
            // hash (or to a lower lane of the same step that exchanged first),
            // then raise the head to the step's highest position.  (Measured
            // and dropped: hashes first into prev[], then four steps' LDS
            // atomics in flight together -- 573 K -> 653 K cycles per C4
            // message, profiles/r04x_diag_deflate_phases.log.)
#ifdef BPMD_CHAIN1   // diagnostics: one step at a time
            for (unsigned g = 0; g < wn; g += WAVE) {
                const unsigned q = g + lane;
                uint32_t pv = NONE;
                if (q + MIN_MATCH <= wn) {
                    const uint32_t h = chain_hash(W.dw(q), wn - q, HB);
                    const uint32_t pre = S.b.head[h];
                    const uint32_t old = atomicExch(&S.b.head[h], q);
                    const uint32_t c = old < q ? old : pre;
                    atomicMax(&S.b.head[h], q);
                    pv = c < NONE ? c : NONE;
                }
                if (q < wn) S.a.prev[q] = (uint16_t)pv;
            }
#else
            // two steps per iteration: both steps' window loads and hashes
            // first, then their head operations in step order
            for (unsigned g = 0; g < wn; g += 2 * WAVE) {
                const unsigned q0 = g + lane, q1 = q0 + WAVE;
                const bool i0 = q0 + MIN_MATCH <= wn, i1 = q1 + MIN_MATCH <= wn;
                const uint32_t w0 = W.dw(i0 ? q0 : 0u), w1 = W.dw(i1 ? q1 : 0u);
                const uint32_t h0 = chain_hash(w0, wn - q0, HB), h1 = chain_hash(w1, wn - q1, HB);
                uint32_t pv0 = NONE, pv1 = NONE;
                if (i0) {
                    const uint32_t pre = S.b.head[h0];
                    const uint32_t old = atomicExch(&S.b.head[h0], q0);
                    const uint32_t c = old < q0 ? old : pre;
                    atomicMax(&S.b.head[h0], q0);
                    pv0 = c < NONE ? c : NONE;
                }
                if (i1) {
                    const uint32_t pre = S.b.head[h1];
                    const uint32_t old = atomicExch(&S.b.head[h1], q1);
                    const uint32_t c = old < q1 ? old : pre;
                    atomicMax(&S.b.head[h1], q1);
                    pv1 = c < NONE ? c : NONE;
                }
                if (q0 < wn) S.a.prev[q0] = (uint16_t)pv0;
                if (q1 < wn) S.a.prev[q1] = (uint16_t)pv1;
            }
#endif
        }
        wave_sync();
        // incompressible chunk (near-random bytes): every INCOMP_STRIDE-th
        // position of the chunk, is the head of its chain the same 4 bytes?
        // Under one in INCOMP_DEN, the parse would find almost nothing: all
        // literals.  64 samples per step; a chunk with repeats (JSON) has
        // passed the threshold after the first step and stops there.
        bool no_parse = false;
        if (INCOMP_DEN && chains) {
            unsigned hits = 0;
            no_parse = true;
            for (unsigned g = a0; g + 4 <= wn && no_parse; g += INCOMP_STRIDE * WAVE) {
                const unsigned q = g + INCOMP_STRIDE * lane;
                const uint32_t c = q + 4 <= wn ? S.a.prev[q] : NONE;
                const bool hit = c != NONE && W.dw(c) == W.dw(q);
                hits += (unsigned)__builtin_popcountll(__ballot(hit));
                no_parse = incompressible(hits, clen);
            }
        }
        pf.lap(1);
        if (INCOMP_STORED && no_parse && len > CHUNK) {
            kind = 0;   // stored outright (lz_core.h INCOMP_STORED)
            goto emit_block;
        }
        [[maybe_unused]] unsigned steps = 0, finds = 0, iters = 0;
        // ---- parse (head table dead from here; tok[] reuses it)
        unsigned seg = (clen + WAVE - 1) / WAVE;
        // (a chunk with history keeps 32: its matches reach back across more
        // segment boundaries -- C1's takeover messages 1.0438 -> 1.0516x
        // Beast's size at 16)
        const unsigned min_seg = a0 ? (unsigned)BPMD_MIN_SEG_HIST : MIN_SEG;
        seg = seg < min_seg ? min_seg : seg;
        const unsigned a = a0 + lane * seg;
        const unsigned b = a + seg < wn ? a + seg : wn;
        const bool active = a < wn;
        uint64_t bm = 0;
        unsigned own_end = 0, lastdist = 0;
        // literal tokens are not written by the parse (the histogram pass
        // takes them from the window): tok[] starts zeroed, matches set 0x8000.
        // (Measured and dropped: the literal's byte loaded with every
        // iteration's other loads and stored by the parse -- C4 26.2 -> 25.2
        // GiB/s, profiles/r04y_ab_literal_preload_rejected.log.)
        {
            uint4* t4 = (uint4*)S.b.tok;
            for (unsigned i = lane; i < CHUNK * 2 / 16; i += WAVE) t4[i] = make_uint4(0, 0, 0, 0);
        }
        wave_sync();
        if (active && no_parse) {
            own_end = b;
            bm = b - a >= 64 ? ~0ull : (1ull << (b - a)) - 1;
        } else if (active) {
            // The reference's parse loop (f_fast / f_slow) and longest_match
            // chain walk, flattened into one state machine so that every
            // iteration does one unit of work per lane (one chain candidate,
            // or 8 more bytes of a match) -- nested divergent loops would
            // multiply lane imbalance.  A find's setup (chain head, limits)
            // runs at the end of the iteration that finished the previous
            // find, so a find costs no iteration of its own.
            // The level's limits are wave-uniform, but kept in VGPRs here: in
            // scalar registers the loop's many lane masks push them out to
            // VGPR lanes, reloaded (v_readlane) every iteration.
            const unsigned max_dist = to_vgpr(P.max_dist), good = to_vgpr(P.L.good), nice_l = to_vgpr(P.L.nice),
                           lazy_l = to_vgpr(P.L.lazy), chain_max = to_vgpr(P.chain);
            const unsigned pflags = to_vgpr((P.L.parser == P_SLOW ? 1u : 0u) | (P.strategy == 2 ? 2u : 0u) |
                                            (P.strategy == 3 ? 4u : 0u) | (P.strategy == 1 ? 8u : 0u));
            const bool lazy = (pflags & 1u) != 0, no_match = (pflags & 2u) != 0, rle = (pflags & 4u) != 0,
                       filtered = (pflags & 8u) != 0;
            unsigned p = a, l0 = 0, d0 = 0;
            const unsigned budget = BPMD_CHAIN_BUDGET ? to_vgpr((BPMD_CHAIN_BUDGET * seg + 63) / 64) : ~0u;
            bool have0 = false;
            bool mt = false;   // match state (chain otherwise)
            unsigned q = p, thr = MIN_MATCH - 1, c = 0, chain_left = 0, best = thr, bd = 0, nice = 0, maxl = 0,
                     l = 0, cn = NONE;   // cn: the candidate after c
            // find setup at q: chain head and limits; no candidate (c = NONE)
            // ends the find at the next iteration with best = thr
            auto setup = [&]() {
                maxl = wn - q < (unsigned)MAX_MATCH ? wn - q : (unsigned)MAX_MATCH;
                uint32_t h = S.a.prev[q];
                asm volatile("" : "+v"(h));   // one load for every lane, not a branch on rle
                c = rle ? (q > 0 ? q - 1 : NONE) : h;
                c = (no_match || q + MIN_MATCH > wn) ? NONE : c;
                if (BPMD_DUAL_TEST) cn = S.a.prev[c < wn ? c : 0];
                chain_left = rle ? 1u : (thr >= good ? chain_max >> 2 : chain_max);
                if (BPMD_CHAIN_BUDGET) chain_left = steps > budget && chain_left > 4u ? 4u : chain_left;
                nice = rle ? maxl : (nice_l < maxl ? nice_l : maxl);
            };
            setup();
            while (p < b) {
                ++iters;
#if BPMD_DUAL_TEST
                // every load issued up front: candidate c, the next one cn (its
                // prev cnn, and cnn's prev for an iteration that uses both)
                const unsigned cc = c < wn ? c : 0, cc2 = cn < wn ? cn : 0;
                const uint32_t cnn = S.a.prev[cc2];
                const uint32_t cb = W.byte(cc + best), qb = W.byte(q + best), cb2 = W.byte(cc2 + best);
                const uint64_t cv = W.qw(cc + l), qv = W.qw(q + l), cv2 = W.qw(cc2);
                const unsigned cc3 = cnn < wn ? cnn : 0;
                const uint32_t cnnn = S.a.prev[cc3];
                constexpr bool T3 = BPMD_DUAL_TEST > 1 && HIST > 0;   // (unused loads fold away without)
                const uint32_t cb3 = T3 ? W.byte(cc3 + best) : 0u;
                const uint64_t cv3 = T3 ? W.qw(cc3) : 0ull;
                const uint32_t c4 = T3 ? S.a.prev[cnnn < wn ? cnnn : 0] : NONE;
                const unsigned k3 = eq_bytes(cv3, qv);
                constexpr bool T4 = BPMD_DUAL_TEST > 2 && HIST > 0;
                const unsigned cc4 = cnnn < wn ? cnnn : 0;
                const uint32_t cb4 = T4 ? W.byte(cc4 + best) : 0u;
                const uint64_t cv4 = T4 ? W.qw(cc4) : 0ull;
                const uint32_t c5 = T4 ? S.a.prev[c4 < wn ? c4 : 0] : NONE;
                const unsigned k4 = eq_bytes(cv4, qv);
                const unsigned k = eq_bytes(cv, qv), k2 = eq_bytes(cv2, qv);   // qv = qw(q) outside a match
                const bool ch = !mt;
                // bitwise, not short-circuit: no branches
                const bool term = ch & ((c == NONE) | (q - c > max_dist) | (chain_left == 0));
                const bool test = ch & !term;
                const bool quick = test & (best < maxl) & (cb == qb) & (k > 0);
                const bool go_match = quick & (k == 8) & (maxl > 8);
                const bool ext = mt & (k == 8) & (l + 8 < maxl);
                const bool have_len = (quick & !go_match) | (mt & !ext);
                const unsigned len = l + k < maxl ? l + k : maxl;
                const bool improve = have_len & (len > best);
                // c rejected with best unchanged: cn is tested as the next
                // iteration would (same best, chain_left one lower)
                const bool rej1 = test & !go_match & !improve;
                const unsigned cl1 = chain_left - test;
                const bool term2 = rej1 & ((cn == NONE) | (q - cn > max_dist) | (cl1 == 0));
                const bool test2 = rej1 & !term2;
                const bool quick2 = test2 & (best < maxl) & (cb2 == qb) & (k2 > 0);
                const bool go2 = quick2 & (k2 == 8) & (maxl > 8);
                const unsigned len2 = k2 < maxl ? k2 : maxl;
                const bool improve2 = quick2 & !go2 & (len2 > best);
                // and a third (cnn) when cn was rejected outright too
                const bool rej2 = T3 & test2 & !go2 & !improve2;
                const unsigned cl2 = cl1 - test2;
                const bool term3 = rej2 & ((cnn == NONE) | (q - cnn > max_dist) | (cl2 == 0));
                const bool test3 = rej2 & !term3;
                const bool quick3 = test3 & (best < maxl) & (cb3 == qb) & (k3 > 0);
                const bool go3 = quick3 & (k3 == 8) & (maxl > 8);
                const unsigned len3 = k3 < maxl ? k3 : maxl;
                const bool improve3 = quick3 & !go3 & (len3 > best);
                const bool rej3 = T4 & test3 & !go3 & !improve3;
                const unsigned cl3 = cl2 - test3;
                const bool term4 = rej3 & ((cnnn == NONE) | (q - cnnn > max_dist) | (cl3 == 0));
                const bool test4 = rej3 & !term4;
                const bool quick4 = test4 & (best < maxl) & (cb4 == qb) & (k4 > 0);
                const bool go4 = quick4 & (k4 == 8) & (maxl > 8);
                const unsigned len4 = k4 < maxl ? k4 : maxl;
                const bool improve4 = quick4 & !go4 & (len4 > best);
                best = improve ? len : improve2 ? len2 : improve3 ? len3 : improve4 ? len4 : best;
                bd = improve ? q - c : improve2 ? q - cn : improve3 ? q - cnn : improve4 ? q - cnnn : bd;
                const bool found = term | (improve & (len >= nice)) | term2 | (improve2 & (len2 >= nice)) | term3 |
                                   (improve3 & (len3 >= nice)) | term4 | (improve4 & (len4 >= nice));
                steps += test + test2 + test3 + test4;
                chain_left = cl3 - test4;
                const bool adv4 = rej3 & !found & !go4;               // c .. cnnn done
                const bool adv3 = rej2 & !rej3 & !found & !go3;       // c, cn, cnn done
                const bool adv2 = rej1 & !rej2 & !found & !go2;       // c and cn done
                const bool adv1 = !rej1 & !found & ((test & !go_match) | (mt & !ext));
                l = go_match || go2 || go3 || go4 ? 8u : ext ? l + 8 : 0u;
                const unsigned c_new = adv4 ? c4 : (adv3 || go4) ? cnnn : (adv2 || go3) ? cnn : (adv1 || go2) ? cn : c;
                cn = adv4 ? c5 : (adv3 || go4) ? c4 : (adv2 || go3) ? cnnn : (adv1 || go2) ? cnn : cn;
                c = c_new;
                mt = go_match || ext || go2 || go3 || go4;
#else
                // every load issued up front
                const unsigned cc = c < wn ? c : 0;
                const uint32_t pn = S.a.prev[cc];
                const uint32_t cb = W.byte(cc + best), qb = W.byte(q + best);
                const uint64_t cv = W.qw(cc + l), qv = W.qw(q + l);
                const unsigned k = eq_bytes(cv, qv);
                const bool ch = !mt;
                // bitwise, not short-circuit: no branches
                const bool term = ch & ((c == NONE) | (q - c > max_dist) | (chain_left == 0));
                const bool test = ch & !term;
                const bool quick = test & (best < maxl) & (cb == qb) & (k > 0);
                const bool go_match = quick & (k == 8) & (maxl > 8);
                const bool ext = mt & (k == 8) & (l + 8 < maxl);
                const bool have_len = (quick & !go_match) | (mt & !ext);
                const unsigned len = l + k < maxl ? l + k : maxl;
                const bool improve = have_len & (len > best);
                best = improve ? len : best;
                bd = improve ? q - c : bd;
                const bool found = term | (improve & (len >= nice));
                steps += test;
                chain_left -= test;
                const bool advance = !found & ((test & !go_match) | (mt & !ext));
                l = go_match ? 8u : ext ? l + 8 : 0u;
                c = advance ? pn : c;
                mt = go_match || ext;
#endif
                if (found) {
                    // f_slow / f_fast decision, as selects
                    const bool drop = best > thr && best <= 5 &&
                                      (filtered || (best == (unsigned)MIN_MATCH && bd > (unsigned)TOO_FAR));
                    const unsigned lr = drop ? thr : best;
                    const bool lit = have0 ? lr > l0 : lr < (unsigned)MIN_MATCH;
                    const bool emit1 = have0 && lr <= l0;          // the pending match wins
                    const bool take = have0 ? lr > l0 : lr >= (unsigned)MIN_MATCH;   // (lr, bd) pending
                    unsigned el = l0, ed = d0;
                    l0 = take ? lr : l0;
                    d0 = take ? bd : d0;
                    bm |= (uint64_t)lit << (p - a);
                    p += lit;
                    const bool emit2 = !emit1 && take && p < b && !(lazy && l0 < lazy_l && p + 1 < wn);
                    el = emit1 ? el : l0;
                    ed = emit1 ? ed : d0;
                    have0 = take && !emit2;
                    if (emit1 || emit2) {
                        S.b.tok[p - a0] = (uint16_t)(0x8000u | (el - MIN_MATCH));
                        if (p + 1 < b) S.b.tok[p + 1 - a0] = (uint16_t)(ed - 1);
                        else lastdist = ed;
                        bm |= 1ull << (p - a);
                        p += el;
                    }
                    q = have0 ? p + 1 : p;
                    thr = have0 ? l0 : (unsigned)(MIN_MATCH - 1);
                    best = thr;
                    bd = 0;
                    ++finds;
                    setup();
                }
            }
            own_end = p;
        }
        wave_sync();
        pf.lap(2);
#ifdef BPMD_PROF
        pf.cnt(19, wave_sum(steps));
        pf.cnt(20, wave_maxu(steps));
        pf.cnt(21, wave_sum(finds));
        pf.cnt(18, 1);
        pf.cnt(22, wave_maxu(iters));
        pf.cnt(23, wave_sum(iters));
        pf.cnt(16, wave_sum(active ? 1u : 0u));
#endif
        // ---- boundary repair
        const unsigned E = wave_scan_max_excl(own_end, a0);
        T.a = a;
        T.b = b;
        T.lastdist = lastdist;
        if (active) {
            const unsigned rel = E - a;
            const uint64_t below = rel >= 64 ? bm : (bm & ((1ull << rel) - 1));
            T.kept = rel >= 64 ? 0 : (bm & ~((1ull << rel) - 1));
            if (below) {
                const unsigned t = 63 - (unsigned)__builtin_clzll(below);
                const unsigned pos = a + t;
                const uint32_t e = S.b.tok[pos - a0];
                const unsigned tl = (e & 0x8000u) ? (e & 0xFFu) + MIN_MATCH : 1;
                if (pos + tl > E) {
                    const unsigned r = pos + tl - E;
                    if (tl > 1 && r >= (unsigned)MIN_MATCH) {
                        T.rem_kind = 1;
                        T.rem_len = r;
                        T.rem_dist = pos + 1 < b ? (unsigned)S.b.tok[pos + 1 - a0] + 1 : lastdist;
                    } else {
                        T.rem_kind = 2;
                        T.rem_len = r;
                        T.rem_b0 = W.byte(E);
                        T.rem_b1 = r > 1 ? W.byte(E + 1) : 0;
                    }
                }
            }
        }
        // ---- histograms (prev[] is dead: all lanes left the parse)
        for (unsigned i = lane; i < 288 + 32 + 20; i += WAVE) {
            if (i < 288) H.lf[i] = 0;
            else if (i < 320) H.df[i - 288] = 0;
            else H.bf[i - 320] = 0;
        }
        wave_sync();
        for_tokens<false, true, TOKG>(T, S.b.tok, a0, [&](bool is_match, unsigned v, unsigned dist) {
            ++n_tok;
            if (!is_match) { atomicAdd(&H.lf[v], 1u); return; }
            ++n_match;
            unsigned s, nx, xv;
            len_code(v, s, nx, xv);
            atomicAdd(&H.lf[s], 1u);
            dist_code(dist, s, nx, xv);
            atomicAdd(&H.df[s], 1u);
        }, W.b + W.ws);
        n_tok = wave_sum(n_tok);
        n_match = wave_sum(n_match);
        wave_sync();
        if (lane == 0) H.lf[EOB] = 1;
        wave_sync();
        pf.lap(3);
        build_trees(H, pf);
        pf.lap(7);
        canonical_codes(H, 0, N_LCODES);
        canonical_codes(H, DIST_IDX, N_DCODES);
        pf.lap(8);
        // ---- code-length code (lane 0) and block costs
        {
            unsigned ll = 0, dl = 0;
            for (unsigned i = lane; i < N_LCODES; i += WAVE)
                if (H.lens[i]) ll = i + 1;
            for (unsigned i = lane; i < N_DCODES; i += WAVE)
                if (H.lens[DIST_IDX + i]) dl = i + 1;
            lcodes = wave_maxu(ll);
            dcodes = wave_maxu(dl);
            lcodes = lcodes < 257 ? 257 : lcodes;
            dcodes = dcodes < 1 ? 1 : dcodes;
        }
        {
            // Code-length sequence (lit lens, then dist lens; runs never
            // cross the two) coded run by run (lz::rle_run == the reference's
            // scan_tree/send_tree): run starts by ballot, run lengths from
            // the start bitmap, symbol counts, prefix sum, symbols to
            // H.r.sym and their histogram to H.bf.
            const unsigned N = lcodes + dcodes;
            auto val = [&](unsigned i) -> unsigned { return i < lcodes ? H.lens[i] : H.lens[DIST_IDX + i - lcodes]; };
            for (unsigned c0 = 0; c0 < 320; c0 += WAVE) {
                const unsigned i = c0 + lane;
                const bool st = i == N || (i < N && (i == 0 || i == lcodes || val(i) != val(i - 1)));
                const uint64_t m = ballot(st);
                if (lane == 0) H.r.start[c0 >> 6] = m;
            }
            wave_sync();
            uint32_t run_carry = 0;
            for (unsigned c0 = 0; c0 < 320; c0 += WAVE) {
                const unsigned i = c0 + lane;
                const bool st = i < N && ((H.r.start[i >> 6] >> (i & 63)) & 1);
                unsigned v = 0, r = 0, ns = 0;
                if (st) {
                    v = val(i);
                    unsigned w = i >> 6;
                    uint64_t m = H.r.start[w] & ~((2ull << (i & 63)) - 1);
                    while (!m) m = H.r.start[++w];
                    r = (w << 6) + (unsigned)__builtin_ctzll(m) - i;
                    ns = rle_run_count(v, r);
                }
                const uint32_t incl = wave_scan_incl(ns);
                uint32_t pos = run_carry + incl - ns;
                if (st) {
                    rle_run(v, r, [&](int s, int, int x) {
                        H.r.sym[pos++] = (uint16_t)(s | (x << 5));
                        atomicAdd(&H.bf[s], 1u);
                    });
                }
                run_carry += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
            }
            nrle = run_carry;
            wave_sync();
        }
        bl_tree_wave(H, hdr_bits, blcodes);
        pf.lap(9);
        uint32_t dyn = 0, fix = 0;
        for (unsigned i = lane; i < N_LCODES; i += WAVE) {
            const uint32_t f = H.lf[i];
            const unsigned x = i > 256 ? len_extra_bits(i) : 0;
            dyn += f * (H.lens[i] + x);
            fix += f * (fixed_lit_len(i) + x);
        }
        if (lane < N_DCODES) {
            const uint32_t f = H.df[lane];
            dyn += f * (H.lens[DIST_IDX + lane] + dist_extra_bits(lane));
            fix += f * (5 + dist_extra_bits(lane));
        }
        dyn = wave_sum(dyn);
        fix = wave_sum(fix) + 3;
        wave_sync();
        dyn += hdr_bits;
        uint32_t opt_b = (dyn + 7) >> 3;
        const uint32_t fix_b = (fix + 7) >> 3;
        if (P.strategy == 4) opt_b = fix_b + 1;
        const uint32_t best = opt_b < fix_b ? opt_b : fix_b;
        kind = chunk_stored(clen, best, len > CHUNK) ? 0u : (fix_b <= opt_b ? 1u : 2u);
        pf.lap(10);
    }

emit_block:
    if (kind == 0) {
        // ---- stored block: 000, pad, LEN, NLEN, bytes (tr_stored_block)
        const unsigned hb = o.cbits + 3 > 8 ? 2u : 1u;
        const unsigned total = hb + 4 + clen;
        if (o.opos + total > o.cap) { o.overflow = true; return; }
        uint8_t* d = o.dst + o.opos;
        // payload byte opos + j takes key byte (opos + j) % 4 (0 = unmasked)
        const uint32_t kd = __builtin_amdgcn_alignbit(o.key, o.key, 8u * (o.opos & 3u));
        auto km = [&](unsigned j) { return (uint8_t)(kd >> (8 * (j & 3))); };
        if (lane == 0) {
            d[0] = (uint8_t)o.carry ^ km(0);
            if (hb == 2) d[1] = km(1);
            d[hb + 0] = (uint8_t)(clen & 0xFF) ^ km(hb);
            d[hb + 1] = (uint8_t)(clen >> 8) ^ km(hb + 1);
            d[hb + 2] = (uint8_t)(~clen & 0xFF) ^ km(hb + 2);
            d[hb + 3] = (uint8_t)((~clen >> 8) & 0xFF) ^ km(hb + 3);
        }
        for (unsigned i = lane; i < clen; i += WAVE) d[hb + 4 + i] = msg[base + i] ^ km(hb + 4 + i);
        o.opos += total;
        o.carry = 0;
        o.cbits = 0;
        o.stored = true;
        pf.lap(11);
        return;
    }

    // ---- Huffman block: codes table = fixed or dynamic
    o.stored = false;
    if (kind == 1) {
        for (unsigned i = lane; i < N_LCODES; i += WAVE) {
            unsigned l;
            const unsigned c = fixed_code(i, l);
            H.codes[i] = pack_code(c, l);
        }
        if (lane < N_DCODES) H.codes[DIST_IDX + lane] = pack_code(lane, 5);
        hdr_bits = 3;
    }
    wave_sync();
    // per-lane token bits
    uint32_t nbits = 0;
    // matches in at least a quarter of the tokens: one token body per step
    const bool dense = (unsigned)__builtin_amdgcn_readfirstlane((int)n_match) * 4 > n_tok;
    auto count_bits = [&](bool is_match, unsigned v, unsigned dist) {
        unsigned s, nx, xv;
        len_code(is_match ? v : 3u, s, nx, xv);
        nbits += (H.codes[is_match ? s : v] >> 16) + (is_match ? nx : 0u);
        if (is_match) {
            dist_code(dist, s, nx, xv);
            nbits += (H.codes[DIST_IDX + s] >> 16) + nx;
        }
    };
    if (dense) for_tokens<true, false, TOKG>(T, S.b.tok, a0, count_bits);
    else for_tokens<false, false, TOKG>(T, S.b.tok, a0, count_bits);
    const uint32_t incl = wave_scan_incl(nbits);
    const uint32_t tok_bits = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    const uint32_t eob_len = H.codes[EOB] >> 16;
    const unsigned ob = (unsigned)((uintptr_t)(o.dst + o.opos) & 3);
    const uint32_t start_bits = ob * 8 + o.cbits;
    const uint32_t total_bits = o.cbits + hdr_bits + tok_bits + eob_len;   // from the carry's first bit
    const unsigned nbytes = (total_bits + 7) >> 3;
    if (o.opos + nbytes > o.cap) { o.overflow = true; return; }
    // zero the bit buffer (win is dead: literals live in tok[])
    uint32_t* ow = S.win;
    pf.lap(12);
    const unsigned nwords = (ob + nbytes + 3) >> 2;
    for (unsigned i = lane; i < nwords + 1; i += WAVE) ow[i] = 0;
    wave_sync();
    if (lane == 0) {
        BitOr bw;
        bw.start(ow, ob * 8);
        bw.put(o.carry, o.cbits);
        if (kind == 1) {
            bw.put(1u << 1, 3);
        } else {
            bw.put(2u << 1, 3);
            bw.put(lcodes - 257, 5);
            bw.put(dcodes - 1, 5);
            bw.put(blcodes - 4, 4);
            for (unsigned i = 0; i < blcodes; ++i) bw.put(H.bll[bl_order(i)], 3);
        }
        // end of block after all tokens
        BitOr be;
        be.start(ow, start_bits + hdr_bits + tok_bits);
        const uint32_t c = H.codes[EOB];
        be.put(c & 0xFFFFu, c >> 16);
        be.flush();
        bw.flush();
    }
    if (kind == 2) {
        // run-length coded code lengths, one symbol per lane per step
        uint32_t at = start_bits + 3 + 5 + 5 + 4 + 3 * blcodes;
        for (unsigned c0 = 0; c0 < nrle; c0 += WAVE) {
            const unsigned k = c0 + lane;
            uint32_t nb = 0, v = 0;
            if (k < nrle) {
                const uint32_t e = H.r.sym[k], s = e & 31u, x = e >> 5;
                const uint32_t code = H.blc[s], cl = code >> 16;
                v = (code & 0xFFFFu) | (x << cl);
                nb = cl + (s == 16 ? 2u : s == 17 ? 3u : s == 18 ? 7u : 0u);
            }
            const uint32_t incl2 = wave_scan_incl(nb);
            if (nb) {
                const uint32_t bp = at + incl2 - nb, sh = bp & 31;
                atomicOr(&ow[bp >> 5], v << sh);
                if (sh + nb > 32) atomicOr(&ow[(bp >> 5) + 1], v >> (32 - sh));
            }
            at += (uint32_t)__builtin_amdgcn_readlane((int)incl2, 63);
        }
    }
    pf.lap(13);
    {
        BitOr bw;
        bw.start(ow, start_bits + hdr_bits + (incl - nbits));
        auto emit = [&](bool is_match, unsigned v, unsigned dist) {
            // literal: its code; match: length code + extra, then distance
            // code + extra (each <= 28 bits, one put each)
            unsigned s, nx, xv;
            len_code(is_match ? v : 3u, s, nx, xv);
            const uint32_t c = H.codes[is_match ? s : v];
            const unsigned l1 = c >> 16;
            bw.put((c & 0xFFFFu) | (is_match ? xv << l1 : 0u), l1 + (is_match ? nx : 0u));
            if (is_match) {
                dist_code(dist, s, nx, xv);
                const uint32_t c2 = H.codes[DIST_IDX + s];
                bw.put((c2 & 0xFFFFu) | (xv << (c2 >> 16)), (c2 >> 16) + nx);
            }
        };
        if (dense) for_tokens<true, false, TOKG>(T, S.b.tok, a0, emit);
        else for_tokens<false, false, TOKG>(T, S.b.tok, a0, emit);
        bw.flush();
    }
    wave_sync();
    pf.lap(14);
    put_bytes_global(o, (const uint8_t*)ow, ob, nbytes);
    const uint8_t* ob8 = (const uint8_t*)ow;
    o.opos += total_bits >> 3;
    o.cbits = total_bits & 7;
    o.carry = o.cbits ? ob8[ob + (total_bits >> 3)] : 0u;
    wave_sync();
    pf.lap(15);
}

// one wave per single-chunk message (<= CHUNK bytes, no takeover history)
__global__ void __launch_bounds__(64)
deflate_kernel(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off, const uint32_t* __restrict__ in_len,
               uint32_t n, uint8_t* __restrict__ out, const uint64_t* __restrict__ out_off,
               const uint32_t* __restrict__ out_cap, uint32_t* __restrict__ out_len, int32_t* __restrict__ status,
               Params P, uint32_t* __restrict__ qctr)
{
    __shared__ DefLds<0> S;
    const unsigned lane = lane_id();
    Prof pf;
    // messages from a counter when the batch outnumbers the waves (a wave
    // whose messages were short takes more), a fixed stride otherwise
    auto next = [&](uint32_t i) -> uint32_t {
        if (!qctr) return i + gridDim.x;
        uint32_t v = 0;
        if (lane == 0) v = atomicAdd(qctr, 1u);
        return gridDim.x + (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
    };
    for (uint32_t i = blockIdx.x; i < n; i = next(i)) {
        const uint32_t len = in_len[i];
        if (len > CHUNK) continue;   // chunk-parallel path (deflate_chunks_kernel + stitch_kernel)
        MsgOut o;
        o.dst = out + out_off[i];
        o.cap = out_cap[i];
        o.opos = 0;
        o.carry = 0;
        o.cbits = 0;
        o.overflow = false;
        o.key = P.mask_key ? P.mask_key[i] : 0u;
        o.stored = false;
        const uint8_t* msg = in + in_off[i];
        if (len) deflate_chunk<0>(S, msg, 0, len, 0u, P, o, pf);
        // Flush::sync's empty stored block header (000) + pad; 00 00 FF FF stripped
        const unsigned tb = o.cbits + 3 > 8 ? 2u : 1u;
        if (!o.overflow && o.opos + tb > o.cap) o.overflow = true;
        if (lane == 0) {
            if (!o.overflow) {
                o.dst[o.opos] = (uint8_t)(o.carry ^ (o.key >> (8 * (o.opos & 3))));
                if (tb == 2) o.dst[o.opos + 1] = (uint8_t)(o.key >> (8 * ((o.opos + 1) & 3)));
            }
            out_len[i] = o.overflow ? 0u : o.opos + tb;
            if (P.out_bits) P.out_bits[i] = o.overflow ? 0u : o.opos * 8 + o.cbits;
            status[i] = o.overflow ? ST_NEED_BUFFERS : ST_OK;
        }
        wave_sync();
    }
    pf.flush();
}

// ------------------------------------------------ chunk-parallel large messages
// A message longer than one chunk (or any message of a context-takeover
// batch) is encoded chunk by chunk IN PARALLEL: every 4 KiB chunk, with the
// BPMD_CHUNK_HIST (2 KiB) of input before it as history, becomes one block of its own in a
// scratch slot, starting at bit 0 (deflate_chunks_kernel); then one wave per
// message stitches the blocks together at their bit offsets, applies the
// client mask and appends Flush::sync's empty stored block header
// (stitch_kernel).  A block's contents and its stored/fixed/dynamic choice do
// not depend on where it starts, so the payload is bit for bit the one the
// serial walk over the chunks would produce; only a stored block's padding to a byte
// boundary depends on its start, and the stitch writes it there.
constexpr unsigned SLOT = 4736;   // >= bpmd_deflate_upper_bound(CHUNK) + 2, 16-byte multiple
constexpr int CHUNK_HIST = BPMD_CHUNK_HIST;   // (lz_core.h) history bytes before each chunk (and before a takeover message)

__device__ __forceinline__ uint32_t chunk_count(uint32_t len, bool all)
{
    return (all || len > CHUNK) ? (len + CHUNK - 1) / CHUNK : 0u;
}

struct ChunkCountOp {
    const uint32_t* len;
    uint32_t n;
    bool all;
    __host__ __device__ uint32_t operator()(uint32_t i) const
    {
        return i < n ? ((all || len[i] > CHUNK) ? (len[i] + CHUNK - 1) / CHUNK : 0u) : 0u;
    }
};

__global__ void __launch_bounds__(256) count_chunks_kernel(const uint32_t* __restrict__ in_len, uint32_t n, uint32_t all,
                                                           uint32_t* __restrict__ total)
{
    uint32_t c = 0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        c += chunk_count(in_len[i], all != 0);
    c = wave_sum(c);
    if (lane_id() == 0 && c) atomicAdd(total, c);
}

__global__ void __launch_bounds__(256) fill_items_kernel(const uint32_t* __restrict__ in_len, uint32_t n, uint32_t all,
                                                         const uint32_t* __restrict__ first, uint32_t* __restrict__ items)
{
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint32_t k = chunk_count(in_len[i], all != 0), f = first[i];
        for (uint32_t c = 0; c < k; ++c) items[f + c] = i;
    }
}

// One message whose chunk count the host knows (a stream's write): the work
// of the count, the scan and fill_items_kernel in one launch -- the counters
// zeroed, first = {0, total}, every item message 0
__global__ void __launch_bounds__(64) one_msg_setup_kernel(uint32_t* __restrict__ d_total, uint32_t* __restrict__ first,
                                                           uint32_t* __restrict__ items, uint32_t total)
{
    const uint32_t t = threadIdx.x;
    d_total[t] = t == 0 ? total : 0u;   // (the 256 bytes the memset clears otherwise)
    if (t < 2) first[t] = t ? total : 0u;
    for (uint32_t c = t; c < total; c += 64) items[c] = 0;
}

template <int HIST>
__global__ void __launch_bounds__(64)
deflate_chunks_kernel(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                      const uint32_t* __restrict__ in_len, const uint32_t* __restrict__ items,
                      const uint32_t* __restrict__ first, const uint32_t* __restrict__ n_items,
                      uint8_t* __restrict__ temp, uint32_t* __restrict__ bits, uint32_t* __restrict__ qctr, Params P)
{
    __shared__ DefLds<HIST> S;
    Prof pf;
    const uint32_t total = *n_items;
    // chunks from a counter: 6 waves per CU leave two SIMDs with two, whose
    // waves would set the end of a static stride
    auto next = [&]() -> uint32_t {
        uint32_t v = 0;
        if (lane_id() == 0) v = atomicAdd(qctr, 1u);
        return (uint32_t)__shfl((int)v, 0);
    };
    for (uint32_t k = next(); k < total; k = next()) {
        const uint32_t i = items[k];
        const uint32_t c = k - first[i];
        const uint32_t len = in_len[i];
        const unsigned hist = P.hist_len ? (P.hist_len[i] < (unsigned)HIST ? P.hist_len[i] : (unsigned)HIST) : 0u;
        MsgOut o;
        o.dst = temp + (size_t)k * SLOT;
        o.cap = SLOT;
        o.opos = 0;
        o.carry = 0;
        o.cbits = 0;
        o.overflow = false;
        o.key = 0;
        o.stored = false;
        deflate_chunk<HIST>(S, in + in_off[i], c * CHUNK, len, hist, P, o, pf);
        if (lane_id() == 0)
            bits[k] = o.overflow ? 0xFFFFFFFFu : ((o.stored ? 0x80000000u : 0u) | (o.opos * 8 + o.cbits));
        wave_sync();
    }
    pf.flush();
}

// one wave per large message: its chunk blocks at their bit offsets
__global__ void __launch_bounds__(64)
stitch_kernel(const uint32_t* __restrict__ in_len, uint32_t n, uint32_t all, const uint32_t* __restrict__ first,
              const uint8_t* __restrict__ temp, const uint32_t* __restrict__ bits, uint8_t* __restrict__ out,
              const uint64_t* __restrict__ out_off, const uint32_t* __restrict__ out_cap,
              uint32_t* __restrict__ out_len, int32_t* __restrict__ status, uint32_t* __restrict__ out_bits,
              const uint32_t* __restrict__ mask_key)
{
    const unsigned lane = lane_id();
    for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
        const uint32_t len = in_len[i];
        if (!all && len <= CHUNK) continue;
        const uint32_t nk = chunk_count(len, all != 0), f = first[i];
        uint8_t* o = out + out_off[i];
        const uint32_t cap = out_cap[i];
        const uint32_t key = mask_key ? mask_key[i] : 0u;
        auto km = [&](uint32_t p) { return (uint8_t)(key >> (8 * (p & 3))); };
        uint32_t bit = 0;   // output bits so far
        uint32_t cv = 0;    // the partial byte at bit >> 3 (its low bit & 7 bits)
        bool overflow = false;
        for (uint32_t c = 0; c < nk && !overflow; ++c) {
            const uint32_t k = f + c;
            const uint32_t w = bits[k];
            if (w == 0xFFFFFFFFu) { overflow = true; break; }
            const uint8_t* t = temp + (size_t)k * SLOT;
            const uint32_t L = w & 0x7FFFFFFFu;
            if (c == 1 && (w & 0x80000000u)) {
                // a stored chunk 1 gets the marker too, so every payload of two
                // or more chunks carries one and a block-parallel inflater
                // knows its Huffman blocks are all marked (pmd_inflate_bp.hip)
                const uint32_t B = bit >> 3, P = (bit + 3 + 7) >> 3;
                if (P + 4 + 1 > cap) { overflow = true; break; }
                if (lane == 0) {
                    o[B] = (uint8_t)cv ^ km(B);
                    if (P - B == 2) o[B + 1] = km(B + 1);
                }
                if (lane < 4) o[P + lane] = (uint8_t)(lane < 2 ? 0x00 : 0xff) ^ km(P + lane);
                bit = (P + 4) * 8;
                cv = 0;
            }
            const uint32_t B = bit >> 3, s = bit & 7;
            if (w & 0x80000000u) {
                // stored block: 000 at `bit`, pad to a byte, then LEN NLEN and the
                // bytes (in the slot from byte 1: header + pad took byte 0)
                const uint32_t P = (bit + 3 + 7) >> 3;
                const uint32_t nbytes = L / 8 - 1;
                if (P + nbytes + 1 > cap) { overflow = true; break; }
                if (lane == 0) {
                    o[B] = (uint8_t)cv ^ km(B);
                    if (P - B == 2) o[B + 1] = km(B + 1);
                }
                for (uint32_t j = lane; j < nbytes; j += WAVE) o[P + j] = t[1 + j] ^ km(P + j);
                bit = (P + nbytes) * 8;
                cv = 0;
            } else {
                if (c) {
                    // a marker before every Huffman-coded chunk but the first:
                    // an empty stored block (000, pad, 00 00 FF FF), so the
                    // block starts on a byte that a block-parallel inflater
                    // finds by a byte search (pmd_inflate_bp.hip); ~5 bytes
                    // per 4 KiB chunk
                    const uint32_t P = (bit + 3 + 7) >> 3;
                    if (P + 4 + 1 > cap) { overflow = true; break; }
                    if (lane == 0) {
                        o[B] = (uint8_t)cv ^ km(B);
                        if (P - B == 2) o[B + 1] = km(B + 1);
                    }
                    if (lane < 4) o[P + lane] = (uint8_t)(lane < 2 ? 0x00 : 0xff) ^ km(P + lane);
                    bit = (P + 4) * 8;
                    cv = 0;
                }
                const uint32_t B = bit >> 3, s = bit & 7;
                const uint32_t end = bit + L;
                if (((end + 7) >> 3) + 1 > cap) { overflow = true; break; }
                const uint32_t nb = (L + 7) >> 3;             // slot bytes
                const uint32_t full = (end >> 3) - B;         // output bytes completed by this block
                auto tb = [&](uint32_t j) -> uint32_t { return j < nb ? t[j] : 0u; };
                auto val = [&](uint32_t j) -> uint32_t {
                    const uint32_t lo = s == 0 ? 0u : (j == 0 ? cv : tb(j - 1) >> (8 - s));
                    return ((tb(j) << s) | lo) & 0xFFu;
                };
                for (uint32_t j = lane; j < full; j += WAVE) o[B + j] = (uint8_t)val(j) ^ km(B + j);
                cv = (end & 7) ? val(full) : 0u;
                bit = end;
            }
        }
        // Flush::sync's empty stored block header (000) + pad; 00 00 FF FF stripped
        const uint32_t tbytes = (bit & 7) + 3 > 8 ? 2u : 1u;
        const uint32_t olen = (bit >> 3) + tbytes;
        if (!overflow && olen > cap) overflow = true;
        if (lane == 0) {
            if (!overflow) {
                o[bit >> 3] = (uint8_t)cv ^ km(bit >> 3);
                if (tbytes == 2) o[(bit >> 3) + 1] = km((bit >> 3) + 1);
            }
            out_len[i] = overflow ? 0u : olen;
            if (out_bits) out_bits[i] = overflow ? 0u : bit;
            status[i] = overflow ? ST_NEED_BUFFERS : ST_OK;
        }
        wave_sync();
    }
}

}  // namespace dfl
}  // namespace bpmd

extern "C" unsigned bpmd_diag_grid_override;
extern "C" void* bpmd_internal_scratch(hipStream_t s, size_t bytes, int which);
extern "C" void* bpmd_internal_pinned(hipStream_t s, size_t bytes, int which);
#ifndef BPMD_DEFLATE_QUEUE
#define BPMD_DEFLATE_QUEUE 1
#endif

namespace {
// single-chunk messages: as many waves as the LDS holds, grid-strided or
// (BPMD_DEFLATE_QUEUE) drained from a counter
int launch_single(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint32_t n, uint8_t* out,
                  const uint64_t* out_off, const uint32_t* out_cap, uint32_t* out_len, int32_t* status,
                  const bpmd::dfl::Params& P, hipStream_t stream)
{
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const unsigned per_cu = (160u * 1024u) / (unsigned)sizeof(bpmd::dfl::DefLds<0>);
    unsigned grid = (unsigned)cus * (per_cu ? per_cu : 1u);
    if (bpmd_diag_grid_override) grid = bpmd_diag_grid_override;
    if (grid > n) grid = n;
    uint32_t* qctr = nullptr;
    if (BPMD_DEFLATE_QUEUE && n > grid) {   // scratch block 7: the single-chunk message counter
        qctr = (uint32_t*)bpmd_internal_scratch(stream, 256, 7);
        if (!qctr || hipMemsetAsync(qctr, 0, sizeof(uint32_t), stream) != hipSuccess) return (int)hipErrorOutOfMemory;
    }
    hipLaunchKernelGGL(bpmd::dfl::deflate_kernel, dim3(grid), dim3(64), 0, stream, in, in_off, in_len, n, out, out_off,
                       out_cap, out_len, status, P, qctr);
    return (int)hipGetLastError();
}
}  // namespace

namespace {
// tune: null, or deflate_stream::tune's (good_length, max_lazy, nice_length,
// max_chain) (deflate_stream.ipp:307-317) replacing the level's table row;
// the level still picks the parser, and the chain keeps the engine's caps
// host_chunks >= 0: the caller knows the batch's chunk count (the per-stream
// deflater, one message of known length), so nothing is read back
int deflate_impl(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint32_t n, uint8_t* out,
                 const uint64_t* out_off, const uint32_t* out_cap, uint32_t* out_len, int32_t* status,
                 uint32_t* out_bits, const uint32_t* mask_key, const uint32_t* hist_len, int level, int window_bits,
                 int strategy, hipStream_t stream, const int* tune = nullptr, int64_t host_chunks = -1)
{
    bpmd::dfl::Params P;
    P.L = lz::level_params(level);
    auto clamp16 = [](int v) { return (uint16_t)(v < 0 ? 0 : v > 65535 ? 65535 : v); };
    if (tune) {
        P.L.good = clamp16(tune[0]);
        P.L.lazy = clamp16(tune[1]);
        P.L.nice = clamp16(tune[2]);
        P.L.chain = clamp16(tune[3]);
    }
    auto chain = [&](bool single) {
        const unsigned cap = single ? (unsigned)BPMD_CHAIN_CAP : (unsigned)BPMD_CHAIN_CAP_MULTI;
        return cap && P.L.chain > cap ? cap : (unsigned)P.L.chain;
    };
    P.strategy = strategy;
    const unsigned wsize = 1u << window_bits;
    P.max_dist = wsize - lz::LOOKAHEAD_MIN;
    P.out_bits = out_bits;
    P.mask_key = mask_key;
    P.hist_len = hist_len;
    using namespace bpmd::dfl;
    const uint32_t all = hist_len ? 1u : 0u;   // context takeover: every message needs its history window
    // how many chunk blocks the large messages make (one small read back: it
    // sizes the workspace; the single-chunk kernel is enqueued right after it
    // and runs meanwhile)
    uint32_t* d_total = (uint32_t*)bpmd_internal_scratch(stream, 256, 1);   // [0] chunk count, [32] chunk queue
    if (!d_total) return (int)hipErrorOutOfMemory;
    // one message with its chunk count known (a stream's write): one setup
    // launch below instead of the memset, the count, the scan and the fill
    const bool one = n == 1 && host_chunks >= 0;
    hipError_t he = hipSuccess;
    if (!one) {
        he = hipMemsetAsync(d_total, 0, 256, stream);
        if (he != hipSuccess) return (int)he;
        hipLaunchKernelGGL(count_chunks_kernel, dim3(n < 256 * 256 ? (n + 255) / 256 : 256), dim3(256), 0, stream, in_len,
                           n, all, d_total);
    }
    uint32_t total = 0;
    P.chain = chain(true);
    if (host_chunks >= 0) {
        if (host_chunks > 0xFFFFFFFFll) return (int)hipErrorInvalidValue;
        total = (uint32_t)host_chunks;   // the device count above is the same number
        const int e = all ? 0 : launch_single(in, in_off, in_len, n, out, out_off, out_cap, out_len, status, P, stream);
        if (e) return e;
    } else {
    // a pinned word of the stream (the caller holds its launch lock), so the
    // copy is asynchronous and the event covers it
    uint32_t* h_total = (uint32_t*)bpmd_internal_pinned(stream, 64, 0);
    if (!h_total) return (int)hipErrorOutOfMemory;
    hipEvent_t ev = nullptr;
    if ((he = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) return (int)he;
    if ((he = hipMemcpyAsync(h_total, d_total, sizeof(uint32_t), hipMemcpyDeviceToHost, stream)) != hipSuccess ||
        (he = hipEventRecord(ev, stream)) != hipSuccess) {
        (void)hipEventDestroy(ev);
        return (int)he;
    }
    int e = all ? 0 : launch_single(in, in_off, in_len, n, out, out_off, out_cap, out_len, status, P, stream);
    he = hipEventSynchronize(ev);
    (void)hipEventDestroy(ev);
    if (e) return e;
    if (he != hipSuccess) return (int)he;
    total = *h_total;
    }
    const bool big = total > 0 || all;
    if (!big) {
        // the stitch also finishes zero-chunk messages only on the takeover path
        return 0;
    }
    // workspace: first[n + 1] | items[total] | bits[total] | slots[total] | scan temp
    // (round 5's single-write chunk kernel, which placed each chunk's block
    // without the stitch's second write, measured slower -- a chunk's wave
    // waits, holding its CU slot, for the chunk before it to finish encoding:
    // C4 26.6 -> 23.8, C5 L1 27.6 -> 25.5 GiB/s, profiles/r05k_ab_single_write.log
    // -- and was removed in round 6)
    size_t cub_bytes = 0;
    hipcub::CountingInputIterator<uint32_t> idx(0);
    hipcub::TransformInputIterator<uint32_t, ChunkCountOp, hipcub::CountingInputIterator<uint32_t>> counts(
        idx, ChunkCountOp{in_len, n, all != 0});
    if (!one &&
        (he = hipcub::DeviceScan::ExclusiveSum(nullptr, cub_bytes, counts, (uint32_t*)nullptr, n + 1, stream)) !=
            hipSuccess)
        return (int)he;
    auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t o_first = 0, o_items = up(o_first + 4ull * (n + 1)),
                 o_bits = up(o_items + 4ull * total),
                 o_slots = up(o_bits + 4ull * total),
                 o_cub = up(o_slots + (size_t)SLOT * total), bytes = up(o_cub + cub_bytes);
    uint8_t* ws = (uint8_t*)bpmd_internal_scratch(stream, bytes, 2);
    if (!ws) return (int)hipErrorOutOfMemory;
    uint32_t* first = (uint32_t*)(ws + o_first);
    uint32_t* items = (uint32_t*)(ws + o_items);
    uint32_t* bits = (uint32_t*)(ws + o_bits);
    uint8_t* slots = ws + o_slots;
    if (one) {
        hipLaunchKernelGGL(one_msg_setup_kernel, dim3(1), dim3(64), 0, stream, d_total, first, items, total);
    } else {
        if ((he = hipcub::DeviceScan::ExclusiveSum(ws + o_cub, cub_bytes, counts, first, n + 1, stream)) != hipSuccess)
            return (int)he;
        const unsigned fgrid = n < 256 * 1024 ? (n + 255) / 256 : 1024;
        hipLaunchKernelGGL(fill_items_kernel, dim3(fgrid), dim3(256), 0, stream, in_len, n, all, first, items);
    }
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    P.chain = chain(false);
    // the chunk kernel with the level's history (lz::chunk_hist: 2 KiB, or 4 KiB
    // at the slow levels)
    auto launch_chunks = [&](auto hist_tag) -> int {
        constexpr int H = decltype(hist_tag)::value;
        const unsigned per_cu = (160u * 1024u) / (unsigned)sizeof(DefLds<H>);
        const unsigned grid = total < (uint32_t)cus * per_cu ? total : (unsigned)cus * per_cu;
        hipLaunchKernelGGL(deflate_chunks_kernel<H>, dim3(grid), dim3(64), 0, stream, in, in_off, in_len, items,
                           first, d_total, slots, bits, d_total + 32, P);
        return 0;
    };
    if (total) {
        const int e = lz::chunk_hist(level) == lz::CHUNK_HIST_DEEP
                          ? launch_chunks(std::integral_constant<int, (int)lz::CHUNK_HIST_DEEP>{})
                          : launch_chunks(std::integral_constant<int, CHUNK_HIST>{});
        if (e) return e;
    }
    // the stitch: every chunked message (and the empty messages of a takeover batch)
    {
        const unsigned sgrid = n < (uint32_t)cus * 16 ? n : (unsigned)cus * 16;
        hipLaunchKernelGGL(stitch_kernel, dim3(sgrid), dim3(64), 0, stream, in_len, n, all, first, slots, bits, out,
                           out_off, out_cap, out_len, status, out_bits, mask_key);
    }
    return (int)hipGetLastError();
}
}  // namespace

extern "C" int bpmd_internal_deflate_bits(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                                          uint32_t n, uint8_t* out, const uint64_t* out_off, const uint32_t* out_cap,
                                          uint32_t* out_len, int32_t* status, uint32_t* out_bits, int level,
                                          int window_bits, int strategy, const int* tune, hipStream_t stream)
{
    return deflate_impl(in, in_off, in_len, n, out, out_off, out_cap, out_len, status, out_bits, nullptr, nullptr,
                        level, window_bits, strategy, stream, tune);
}

// the per-stream deflater's flush (pmd_stream.hip): exact bit lengths, and
// the stream's earlier plaintext before the message as history (context
// takeover), hist_len null for none
extern "C" int bpmd_internal_deflate_bits_hist(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                                               uint32_t n, uint8_t* out, const uint64_t* out_off,
                                               const uint32_t* out_cap, uint32_t* out_len, int32_t* status,
                                               uint32_t* out_bits, const uint32_t* hist_len, int level,
                                               int window_bits, int strategy, const int* tune, hipStream_t stream,
                                               int64_t host_chunks)
{
    return deflate_impl(in, in_off, in_len, n, out, out_off, out_cap, out_len, status, out_bits, nullptr, hist_len,
                        level, window_bits, strategy, stream, tune, host_chunks);
}

extern "C" int bpmd_internal_deflate_keyed(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                                           uint32_t n, uint8_t* out, const uint64_t* out_off, const uint32_t* out_cap,
                                           uint32_t* out_len, int32_t* status, int level, int window_bits,
                                           int strategy, const uint32_t* mask_key, hipStream_t stream)
{
    return deflate_impl(in, in_off, in_len, n, out, out_off, out_cap, out_len, status, nullptr, mask_key, nullptr,
                        level, window_bits, strategy, stream);
}

extern "C" int bpmd_internal_deflate_takeover(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                                              uint32_t n, uint8_t* out, const uint64_t* out_off,
                                              const uint32_t* out_cap, uint32_t* out_len, int32_t* status, int level,
                                              int window_bits, int strategy, const uint32_t* hist_len,
                                              hipStream_t stream)
{
    return deflate_impl(in, in_off, in_len, n, out, out_off, out_cap, out_len, status, nullptr, nullptr, hist_len,
                        level, window_bits, strategy, stream);
}

extern "C" int bpmd_internal_deflate(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint32_t n,
                                     uint8_t* out, const uint64_t* out_off, const uint32_t* out_cap,
                                     uint32_t* out_len, int32_t* status, int level, int window_bits, int strategy,
                                     hipStream_t stream)
{
    return bpmd_internal_deflate_bits(in, in_off, in_len, n, out, out_off, out_cap, out_len, status, nullptr, level,
                                      window_bits, strategy, nullptr, stream);
}

extern "C" int bpmd_diag_deflate_counters(unsigned long long* out, int reset)
{
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(bpmd::dfl::g_dprof), sizeof(unsigned long long) * 24) != hipSuccess)
        return -1;
    if (reset) {
        unsigned long long z[24] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(bpmd::dfl::g_dprof), z, sizeof z) != hipSuccess) return -1;
    }
    return 0;
}
