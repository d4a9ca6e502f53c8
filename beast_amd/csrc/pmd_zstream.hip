// pmd_zstream.hip -- the per-stream inflater behind zlib::inflate_stream
// (include/boost/beast/zlib/inflate_stream.hpp:63-213): one write() per
// launch, on the GPU, with the reference's state carried on the device.
//
// Why a state machine and not the batch decoders.  Beast's inflate_stream
// keeps everything between write() calls -- mode, the 32-bit bit reservoir,
// a half-decoded symbol, the code tables, the 2^windowBits window
// (inflate_stream.ipp:74-535, bitstream.hpp:49-194, window.hpp:51-144) --
// and websocket::stream advances its read buffer by exactly the total_in a
// call reports (read.hpp:1342-1343, impl_base.hpp:183-187).  How many bytes
// a call consumes depends on that state: the slow path pulls bytes one at a
// time until a lookup has the bits it asks for (root, or root + sub-table
// bits), inflate_fast pulls 16 bits at a time and hands whole bytes back when
// it returns (inflate_stream.ipp:1111-1112), and which of the two runs
// depends on how much input and output room is left.  The batch kernels
// decode whole messages and cannot reproduce that, so a per-stream call runs
// the reference's decoder itself: the same modes, the same fills, drops and
// rewinds, the same window rule, so next_in / avail_in / total_in / next_out
// / avail_out / total_out / data_type and the zlib::error are the
// reference's after every call, including calls that stop inside a symbol,
// a header or a stored block, and errors (which return without done()).
//
// Execution: one wave.  The decoder's control flow is wave-uniform (values
// read from LDS are made uniform with readfirstlane, so branches are scalar);
// the lanes share the bulk work -- code tables (huff_wave.h, slot-for-slot
// equal to inflate_table), match copies (64 bytes per step out of a 64 KiB
// LDS history ring), stored-block copies, loading the window into the ring
// the first time a distance reaches it, the window update, and the output
// stores.  Input is staged through LDS 4 KiB at a time.
// The decoder body (zstream_run) is plain wave-uniform C++; with
// BPMD_ZSTREAM_HOST the same text compiles for the host with one-lane
// meanings of the intrinsics (tests/model/zstream_host.py), so the CPU suite
// checks it against the oracle too.
#ifndef BPMD_ZSTREAM_HOST
#include "pmd_common.h"
#include "huff_table.h"
#include "huff_wave.h"
#include "wave_util.h"
#include <atomic>
#include <cstdlib>
#endif
#include "zstream.h"

namespace bpmd {
namespace zst {

constexpr uint32_t HR = 65536, HM = HR - 1;   // history ring: window + this call's output
constexpr uint32_t IST = 4096;               // input staging
constexpr uint64_t FLUSH_AT = 16384;          // unflushed output kept below this (ring room)
// wave-parallel inflate_fast (pfast): ZQ candidate bit offsets per lane per
// window, a window's accepted output bounded by ZWOUT (+ one match), its
// token-start bitmap ZBM words, input staged ZSPAN bytes past the window start
constexpr uint32_t ZQ = 4, ZWOUT = 8192, ZSPAN = 64;
constexpr uint32_t ZBM = (ZWOUT + 258 + 2 * 64) / 32 + 4;
// pfast is used while at least this much input / output room is left (the
// serial loop takes the last few tokens; both stop where inflate_fast stops)
constexpr uint64_t ZMIN_IN = 24, ZMIN_OUT = 512;

struct alignas(16) Lds {
    uint8_t hist[HR];
    uint8_t ist[IST];
    uint16_t tab[kCodes];
    uint8_t lens[kLens];
    uint8_t flens[288];   // fixed-block code lengths (fixedTables, inflate_stream.ipp:865-930)
    WaveTableScratch ts;
    uint32_t ptok[ZQ * WAVE];   // pfast: a window's accepted tokens, (olen << 16) | literal or distance
    uint32_t pbm[ZBM];          // pfast: their first output byte, one bit per output byte of the window
    uint32_t prec[ZQ * WAVE];   // pfast: the chain's tokens: candidate word A (bit fields, kind)
    uint16_t poend[ZQ * WAVE];  // pfast: the bit after each, from the window's first bit
};

// cross-lane steps of pfast (one-lane meanings in the host build)
#ifndef BPMD_ZSTREAM_HOST
__device__ __forceinline__ uint32_t rdlane(uint32_t v, uint32_t j) { return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)j); }
__device__ __forceinline__ uint64_t ballot64(bool p) { return __ballot(p); }
__device__ __forceinline__ uint32_t shfl32(uint32_t v, uint32_t from) { return (uint32_t)__shfl((int)v, (int)from); }
__device__ __forceinline__ uint32_t fsh(uint32_t hi, uint32_t lo, uint32_t sh) { return __builtin_amdgcn_alignbit(hi, lo, sh); }
__device__ __forceinline__ uint32_t shfl_up32(uint32_t v, uint32_t d) { return (uint32_t)__shfl_up((int)v, d); }
__device__ __forceinline__ uint32_t below64(uint64_t m)
{
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
#else
inline uint32_t rdlane(uint32_t v, uint32_t) { return v; }
inline uint64_t ballot64(bool p) { return p ? 1u : 0u; }
inline uint32_t shfl32(uint32_t v, uint32_t) { return v; }
inline uint32_t fsh(uint32_t hi, uint32_t lo, uint32_t sh) { return (uint32_t)((((uint64_t)hi << 32) | lo) >> (sh & 31)); }
inline void atomicOr(uint32_t* p, uint32_t v) { *p |= v; }
inline uint32_t shfl_up32(uint32_t v, uint32_t) { return v; }
inline uint32_t below64(uint64_t) { return 0; }
#endif
// pfast's byte-lag maps: fast()'s reservoir holds bn = r + 8 L bits at a token
// boundary, r fixed by the bit position, L in 0..3 the refill history; a
// token maps L before it to L after it (2 bits per entry, 4 entries)
__host__ __device__ constexpr uint32_t lag_compose(uint32_t first, uint32_t then)
{
    uint32_t r = 0;
    for (uint32_t x = 0; x < 4; ++x) r |= ((then >> (2 * ((first >> (2 * x)) & 3u))) & 3u) << (2 * x);
    return r;
}
#ifndef BPMD_ZST_SCAN
#define BPMD_ZST_SCAN 1   // 0: the scalar replay of round 5's first pfast
#endif
// a candidate token: A = c1 | x << 4 | c2 << 7 | dx << 11 | kind << 15 (bits of
// the literal/length code incl. a sub-table's, length extra, distance code,
// distance extra); B = (output bytes << 16) | literal or distance
enum : uint32_t { Z_LIT = 0, Z_MATCH = 1, Z_EOB = 2, Z_BADLIT = 3, Z_BADDIST = 4 };

// RFC 1951 §3.2.5's length and distance bases and extra bits in closed form,
// equal to the tables at every value a K_LEN slot (0..28) or a distance K_VAL
// slot (0..29) carries (huff_table.h); checked below at compile time.  Scalar
// arithmetic: the tables in constant memory cost four dependent vector-memory
// loads per match on this one-wave kernel (~60 % of a 1 KiB message's call)
__host__ __device__ constexpr uint32_t len_extra(uint32_t c) { return c < 8u || c == 28u ? 0u : (c >> 2) - 1u; }
__host__ __device__ constexpr uint32_t len_base(uint32_t c)
{
    return c < 8u ? 3u + c : c == 28u ? 258u : ((4u + (c & 3u)) << ((c >> 2) - 1u)) + 3u;
}
__host__ __device__ constexpr uint32_t dist_extra(uint32_t c) { return c < 4u ? 0u : (c >> 1) - 1u; }
__host__ __device__ constexpr uint32_t dist_base(uint32_t c) { return c < 4u ? 1u + c : ((2u + (c & 1u)) << ((c >> 1) - 1u)) + 1u; }
constexpr bool closed_forms_match()
{
    constexpr uint16_t lb[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
    constexpr uint8_t lx[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
    constexpr uint16_t db[30] = {1,   2,   3,   4,   5,   7,    9,    13,   17,   25,   33,   49,    65,    97,    129,
                                 193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
    for (uint32_t c = 0; c < 29; ++c)
        if (len_base(c) != lb[c] || len_extra(c) != lx[c]) return false;
    for (uint32_t c = 0; c < 30; ++c)
        if (dist_base(c) != db[c] || dist_extra(c) != (c < 4 ? 0u : c / 2 - 1)) return false;
    return true;
}
static_assert(closed_forms_match(), "length / distance closed forms");

__device__ __forceinline__ uint32_t uni(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
__device__ __forceinline__ bool is_link(uint32_t s) { return slot_kind(s) == K_SPECIAL && slot_val(s) != V_INVALID; }

__constant__ static const uint8_t kOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

enum : int { F_BLOCK = 1, F_FINISH = 5, F_TREES = 6 };   // zlib::Flush values that change doWrite

// Diagnostic build only (-DBPMD_PROF): cycles per phase and event counts,
// summed over calls (bpmd_diag_zstream_counters; scripts/diag_zstream.py).
// 0 entry (state in), 1 block header, 2 table builds, 3 inflate_fast, 4 window
// load, 5 match copies, 6 done() and state out, 7 whole call, 8 input
// staging; counts: 9 copies, 10 fast-loop tokens, 11 output bytes, 12
// stagings, 13 calls, 14 input bytes; inside inflate_fast: 15 bit refill +
// literal/length lookup, 16 literal store, 17 length extra + distance decode,
// 18 loop tail, 19 the cost of one lap (two clock reads); 24 symbols decoded
// by the slow path (LEN mode), 25 code-length symbols hdr_par committed, 26
// block headers (TYPEDO)
constexpr int ZPN = 32;
#ifndef BPMD_ZSTREAM_HOST
__device__ unsigned long long g_zprof[ZPN];
#endif
#if defined(BPMD_PROF) && !defined(BPMD_ZSTREAM_HOST)
#define ZP_NOW() ((unsigned long long)__builtin_amdgcn_s_memtime())
#define ZP_ADD(i, v) (zp[i] += (unsigned long long)(v))
#define ZP_DECL unsigned long long zp[ZPN] = {};
#define ZP_FLUSH() \
    do { \
        if (lane == 0 && !(par & 4)) \
            for (int i_ = 0; i_ < ZPN; ++i_) atomicAdd(&g_zprof[i_], zp[i_]); \
    } while (0)
#elif defined(BPMD_ZSTREAM_HOST) && defined(BPMD_ZS_HOST_COUNT)
// host model, counts only (tests/model/zstream_host.py, ZS_HOST_FLAGS)
extern "C" { unsigned long long zs_host_counts[ZPN]; }
#define ZP_NOW() 0ull
#define ZP_ADD(i, v) (zs_host_counts[i] += (unsigned long long)(v))
#define ZP_DECL
#define ZP_FLUSH() ((void)0)
#else
#define ZP_NOW() 0ull
#define ZP_ADD(i, v) ((void)0)
#define ZP_DECL
#define ZP_FLUSH() ((void)0)
#endif

__device__ void zstream_run(Lds& L, State* __restrict__ st, const uint8_t* __restrict__ in, uint64_t n_in,
                            uint8_t* __restrict__ out, uint64_t cap, int flush, Result* __restrict__ res, int par)
{
    const unsigned lane = lane_id();
    // par: bit 0 the wave-parallel inflate_fast, bit 3 the serial code-length
    // loop instead of hdr_par (diagnostics and tests; bits 1-2: prof build)
    const bool hpar = !(par & 8);
    ZP_DECL
    const unsigned long long zt0 = ZP_NOW();
    unsigned long long zth = zt0, ztd = 0;
    (void)zth;
    (void)ztd;
    Head h = st->h;
    const uint32_t wcap = 1u << h.wbits;

    // tables and code lengths the current mode still needs
    if (h.mode >= CODELENS && h.mode <= LIT)
        for (unsigned i = lane; i < kCodes; i += WAVE) L.tab[i] = st->codes[i];
    if (h.mode == LENLENS || h.mode == CODELENS)
        for (unsigned i = lane; i < kLens; i += WAVE) L.lens[i] = st->lens[i];
    bool tab_dirty = false, lens_dirty = false;
    ZP_ADD(0, ZP_NOW() - zt0);

    // ---- input: bytes [ib0, ib1) of this call's input are staged in LDS
    uint64_t ip = 0, ib0 = 0, ib1 = 0;
    auto stage = [&](uint64_t at) {
        const unsigned long long zs = ZP_NOW();
        (void)zs;
        wave_sync();
        ib0 = at & ~(uint64_t)15;
        ib1 = ib0 + IST < n_in ? ib0 + IST : n_in;
        for (uint32_t k = lane * 16; k < IST; k += WAVE * 16)
            if (ib0 + k < n_in) *(uint4*)(L.ist + k) = *(const uint4*)(in + ib0 + k);
        wave_sync();
        ZP_ADD(8, ZP_NOW() - zs);
        ZP_ADD(12, 1);
    };
    // bit reservoir, bitstream.hpp: v_ holds n_ bits, bytes enter at bit n_.
    // The bytes come from the staging buffer through a register prefetch of
    // up to 8 bytes (one LDS round trip per 5-8 bytes instead of one per
    // byte); only the reference's own ip / bn / bv are state, so the bytes
    // each call consumes are unchanged (the prefetch is refilled whenever ip
    // moves other than byte by byte: rewind, stored-block copies)
    uint32_t bv = h.bv, bn = h.bn;
    uint64_t pfv = 0, pfip = ~0ull;   // bytes [pfip, pfip + pfn) of the input in pfv
    uint32_t pfn = 0;
    auto pull = [&]() {
        if (ip != pfip || pfn == 0) {
            if (ip < ib0 || ip >= ib1) stage(ip);
            const uint32_t off = (uint32_t)(ip - ib0);
            const uint32_t a = off & ~3u;
            const uint32_t d0 = uni(*(const uint32_t*)(L.ist + a));
            const uint32_t d1 = a + 8 <= IST ? uni(*(const uint32_t*)(L.ist + a + 4)) : 0u;
            pfv = (((uint64_t)d1 << 32) | d0) >> (8 * (off & 3u));
            const uint64_t staged = ib1 - ip;
            const uint32_t have = (a + 8 <= IST ? 8u : 4u) - (off & 3u);
            pfn = (uint32_t)(staged < have ? staged : have);
            pfip = ip;
        }
        const uint32_t b = (uint32_t)pfv & 0xffu;
        pfv >>= 8;
        --pfn;
        ++pfip;
        ++ip;
        if (bn < 32) bv += b << bn;
        bn += 8;
    };
    auto fill = [&](uint32_t k) -> bool {   // bitstream::fill
        while (bn < k) {
            if (ip == n_in) return false;
            pull();
        }
        return true;
    };
    auto peek = [&](uint32_t k) -> uint32_t { return k >= 32 ? bv : (bv & ((1u << k) - 1u)); };
    auto drop = [&](uint32_t k) {
        bv = k >= 32 ? 0u : bv >> k;
        bn -= k;
    };
    auto take = [&](uint32_t k) -> uint32_t {
        const uint32_t r = peek(k);
        drop(k);
        return r;
    };
    auto rewind = [&]() {   // bitstream::rewind: whole bytes back to the input
        ip -= bn >> 3;
        bn &= 7;
        bv &= (1u << bn) - 1u;
    };

    // ---- output: this call's bytes go to the ring and out to `out`
    uint64_t op = 0, flushed = 0;
    auto flush_out = [&]() {
        wave_sync();
        for (uint64_t p = flushed + lane; p < op; p += WAVE) out[p] = L.hist[(uint32_t)p & HM];
        flushed = op;
        wave_sync();
    };
    auto put = [&](uint32_t b) {
        if (lane == 0) L.hist[(uint32_t)op & HM] = (uint8_t)b;
        ++op;
    };
    bool winld = false;
    auto load_window = [&]() {   // window byte k back sits at ring position -k
        // ring position HR - wsize + t takes window byte (wpos - wsize + t) mod
        // wcap: 16 bytes per lane per step from t0 on (t0: the first t whose
        // ring position is 16-byte aligned), single bytes before t0 and where
        // a 16-byte run wraps around the window's end
        const unsigned long long zw = ZP_NOW();
        (void)zw;
        wave_sync();
        const uint32_t ws = h.wsize, s0 = (h.wpos - ws) & (wcap - 1);
        const uint32_t t0 = ws & 15u;   // (all of it when ws < 16)
        for (uint32_t t = lane; t < t0; t += WAVE) L.hist[(HR - ws + t) & HM] = st->win[(s0 + t) & (wcap - 1)];
        for (uint32_t t = t0 + 16 * lane; t < ws; t += 16 * WAVE) {
            const uint32_t src = (s0 + t) & (wcap - 1);
            const uint32_t dst = (HR - ws + t) & HM;
            if (t + 16 <= ws && src + 16 <= wcap) {
                typedef uint4 uint4_un __attribute__((aligned(1)));
                *(uint4*)(L.hist + dst) = *(const uint4_un*)(st->win + src);
            } else {
                for (uint32_t j = 0; j < 16 && t + j < ws; ++j)
                    L.hist[(dst + j) & HM] = st->win[(src + j) & (wcap - 1)];
            }
        }
        winld = true;
        wave_sync();
        ZP_ADD(4, ZP_NOW() - zw);
    };
    // n bytes copied from `dist` back (window, then this call's output): the
    // history is contiguous, so byte j is history[op - dist + j mod dist]
    auto copy_back = [&](uint32_t dist, uint32_t n) {
        if (dist > op && !winld) load_window();
        const unsigned long long zc = ZP_NOW();
        (void)zc;
        wave_sync();
        for (uint32_t j0 = 0; j0 < n; j0 += WAVE) {
            const uint32_t j = j0 + lane;
            if (j < n) {
                const uint32_t k = dist >= n ? j : j % dist;
                const uint8_t b = L.hist[(uint32_t)(op - dist + k) & HM];
                L.hist[(uint32_t)(op + j) & HM] = b;
            }
        }
        op += n;
        wave_sync();
        ZP_ADD(5, ZP_NOW() - zc);
        ZP_ADD(9, 1);
    };
    auto copy_in = [&](uint32_t n) {   // a stored block's bytes
        for (uint32_t done = 0; done < n;) {
            const uint32_t piece = n - done < 8192u ? n - done : 8192u;
            wave_sync();
            for (uint32_t j = lane; j < piece; j += WAVE) L.hist[(uint32_t)(op + j) & HM] = in[ip + j];
            ip += piece;
            op += piece;
            done += piece;
            wave_sync();
            if (op - flushed >= FLUSH_AT) flush_out();
        }
    };
    // code tables into LDS; returns 0 or the zlib::error of inflate_table
    auto build = [&](int type, const uint8_t* lens, unsigned n, unsigned at, unsigned req, uint32_t& root,
                     uint32_t& used) -> int {
        const unsigned long long zb = ZP_NOW();
        (void)zb;
        wave_sync();
        unsigned r = 0, u = 0, lmin = 0;
        int e;
        if (type == BUILD_CODES) e = build_table_wave<BUILD_CODES>(lens, n, L.tab + at, req, L.ts, r, u, lmin);
        else if (type == BUILD_LENS) e = build_table_wave<BUILD_LENS>(lens, n, L.tab + at, req, L.ts, r, u, lmin);
        else e = build_table_wave<BUILD_DISTS>(lens, n, L.tab + at, req, L.ts, r, u, lmin);
        wave_sync();
        tab_dirty = true;
        ZP_ADD(2, ZP_NOW() - zb);
        root = uni(r);
        used = uni(u);
        return (int)uni((uint32_t)e);
    };

    // ---- inflate_fast (inflate_stream.ipp:979-1113); 0 or an error (mode BAD)
    auto fast = [&]() -> int32_t {
        const uint64_t in_last = n_in - 5, out_last = cap - 257;
        const uint32_t lmask = (1u << h.lroot) - 1u, dmask = (1u << h.droot) - 1u;
        int32_t err = 0;
        const unsigned long long zf = ZP_NOW();
        (void)zf;
        unsigned long long zl = ZP_NOW();
        (void)zl;
        do {
            ZP_ADD(10, 1);
#ifdef BPMD_ZSTREAM_LAPS
            { const unsigned long long a = ZP_NOW(), b = ZP_NOW(); ZP_ADD(19, b - a); }
#define ZLAP(i) do { const unsigned long long n_ = ZP_NOW(); ZP_ADD(i, n_ - zl); zl = n_; } while (0)
#else
#define ZLAP(i) ((void)0)
#endif
            ZLAP(18);
            if (bn < 15) {
                pull();
                pull();
            }
            uint32_t s = uni(L.tab[bv & lmask]);
            if (is_link(s)) {   // 2nd-level code: root bits, then the sub-table's index bits
                drop(h.lroot);
                s = uni(L.tab[slot_val(s) + (bv & ((1u << slot_bits(s)) - 1u))]);
            }
            drop(slot_bits(s));
            const uint32_t kind = slot_kind(s), val = slot_val(s);
            ZLAP(15);
            if (kind == K_VAL) {
                put(val);
                ZLAP(16);
            } else if (kind == K_LEN) {
                uint32_t len = len_base(val);
                const uint32_t x = len_extra(val);
                if (x) {
                    if (bn < x) pull();
                    len += bv & ((1u << x) - 1u);
                    drop(x);
                }
                if (bn < 15) {
                    pull();
                    pull();
                }
                uint32_t d = uni(L.tab[h.dtab + (bv & dmask)]);
                if (is_link(d)) {
                    drop(h.droot);
                    d = uni(L.tab[h.dtab + slot_val(d) + (bv & ((1u << slot_bits(d)) - 1u))]);
                }
                drop(slot_bits(d));
                if (slot_kind(d) != K_VAL) {
                    err = ST_INVALID_DISTANCE_CODE;
                    break;
                }
                uint32_t dist = dist_base(slot_val(d));
                const uint32_t dx = dist_extra(slot_val(d));
                if (bn < dx) {
                    pull();
                    if (bn < dx) pull();
                }
                dist += bv & ((1u << dx) - 1u);
                drop(dx);
                ZLAP(17);
                if (dist > op) {   // from the window
                    const uint64_t back = dist - op;
                    if (back > h.wsize) {
                        err = ST_INVALID_DISTANCE;
                        break;
                    }
                    const uint32_t n = len < back ? len : (uint32_t)back;
                    copy_back(dist, n);
                    len -= n;
                }
                if (len) copy_back(dist, len);   // from this call's output (room >= 258 here)
                ZLAP(23);
            } else if (kind == K_EOB) {
                h.mode = TYPE;
                break;
            } else {
                err = ST_INVALID_LITERAL_LENGTH;
                break;
            }
            if (op - flushed >= FLUSH_AT) flush_out();
        } while (ip < in_last && op < out_last);
        if (err) h.mode = BAD;
        rewind();
        ZP_ADD(3, ZP_NOW() - zf);
        return err;
    };

    // ---- inflate_fast, wave-parallel.  Per window of ZQ * WAVE bit offsets from
    // the next token's first bit, every lane decodes the token that would start
    // at each of its ZQ offsets (a token's symbols are a function of the bits:
    // every lookup of fast() sees >= 15 valid bits); the scalar unit follows
    // the chain of real token starts through those candidates and replays
    // fast() on it token by token -- its byte refills (so ip and bn are
    // fast()'s), its checks in fast()'s order and its loop condition -- and
    // the lanes then write the accepted tokens' bytes 64 at a time (a match
    // reaching into the same 64 bytes by pointer jumping).  So the tokens, the
    // stopping point, ip / bv / bn and the error are fast()'s.
    auto pfast = [&]() -> int32_t {
        const uint64_t in_last = n_in - 5, out_last = cap - 257;
        const uint32_t lroot = h.lroot, droot = h.droot, dtab = h.dtab;
        const uint32_t lmask = (1u << lroot) - 1u, dmask = (1u << droot) - 1u;
        const uint64_t wsize = h.wsize;
        const uint32_t* iw = (const uint32_t*)L.ist;
        int32_t err = 0;
        bool stop = false;
        const unsigned long long zp0 = ZP_NOW();
        unsigned long long zq = zp0;
        (void)zp0;
        (void)zq;
        int64_t sb = 0;   // L.ist[i] holds input byte sb + i
        bool virt = false;
        while (!stop) {
            if (bn > ip * 8) {
                if (virt) goto staged;   // (bv is the reservoir only on entry)
                // the reservoir still holds bits of an earlier call's input: a
                // window of its own, L.ist = the bn bits (padded in front to a
                // byte) followed by this call's input from ip on
                const uint32_t nb = (bn + 7) >> 3, k = 8 * nb - bn;
                const uint64_t pre = (uint64_t)bv << k;
                wave_sync();
                for (uint32_t i = lane; i < ZSPAN + 16; i += WAVE)
                    L.ist[i] = i < nb ? (uint8_t)(pre >> (8 * i)) : (ip + i - nb < n_in ? in[ip + i - nb] : (uint8_t)0);
                wave_sync();
                sb = (int64_t)ip - (int64_t)nb;
                ib0 = ib1 = ~0ull >> 1;   // the staging pull() uses is gone
                virt = true;
            } else {
                const uint64_t P = ip * 8 - bn;   // the next token's first bit
                if ((P >> 3) < ib0 || (P >> 3) >= ib1 || (P >> 3) + ZSPAN > ib0 + IST) stage(P >> 3);
                sb = (int64_t)ib0;
            }
        staged:
            const uint32_t rb = (uint32_t)((int64_t)(ip * 8) - (int64_t)bn - 8 * sb);
            ZP_ADD(15, ZP_NOW() - zq);
            zq = ZP_NOW();
            // candidates at bits rb + lane + WAVE q of the staged input
            const int64_t Ps = (int64_t)(ip * 8) - (int64_t)bn;   // the window's first bit (< 0: reservoir bits)
            uint32_t ca[ZQ], cb[ZQ], cj[ZQ];
#pragma unroll
            for (uint32_t q = 0; q < ZQ; ++q) {
                const uint32_t r = rb + lane + WAVE * q, w = r >> 5, sh = r & 31;
                const uint32_t d0 = iw[w], d1 = iw[w + 1], d2 = iw[w + 2];
                const uint64_t v = ((uint64_t)fsh(d2, d1, sh) << 32) | fsh(d1, d0, sh);
                uint32_t sl = L.tab[(uint32_t)v & lmask], c1;
                if (is_link(sl)) {
                    sl = L.tab[slot_val(sl) + ((uint32_t)(v >> lroot) & ((1u << slot_bits(sl)) - 1u))];
                    c1 = lroot + slot_bits(sl);
                } else {
                    c1 = slot_bits(sl);
                }
                const uint32_t kind = slot_kind(sl), val = slot_val(sl);
                uint32_t a = c1 | (kind == K_VAL ? Z_LIT : kind == K_EOB ? Z_EOB : Z_BADLIT) << 15, b = (1u << 16) | val;
                if (kind == K_LEN) {
                    const uint32_t x = len_extra(val);
                    const uint32_t len = len_base(val) + ((uint32_t)(v >> c1) & ((1u << x) - 1u));
                    const uint32_t u = c1 + x;
                    uint32_t d = L.tab[dtab + ((uint32_t)(v >> u) & dmask)], c2;
                    if (is_link(d)) {
                        d = L.tab[dtab + slot_val(d) + ((uint32_t)(v >> (u + droot)) & ((1u << slot_bits(d)) - 1u))];
                        c2 = droot + slot_bits(d);
                    } else {
                        c2 = slot_bits(d);
                    }
                    if (slot_kind(d) != K_VAL) {
                        a = c1 | x << 4 | c2 << 7 | Z_BADDIST << 15;
                    } else {
                        const uint32_t dx = dist_extra(slot_val(d));
                        const uint32_t dist = dist_base(slot_val(d)) + ((uint32_t)(v >> (u + c2)) & ((1u << dx) - 1u));
                        a = c1 | x << 4 | c2 << 7 | dx << 11 | Z_MATCH << 15;
                        b = (len << 16) | dist;
                    }
                }
                // the bits this candidate consumes before fast() stops or goes on
                const uint32_t k_ = a >> 15;
                const uint32_t nb_ = k_ == Z_MATCH ? (a & 15u) + ((a >> 4) & 7u) + ((a >> 7) & 15u) + ((a >> 11) & 15u)
                                                   : (a & 15u);
                ca[q] = a;
                cb[q] = b;
                cj[q] = k_ == Z_LIT || k_ == Z_MATCH ? nb_ : 255u;   // the chain ends at an event
            }
            for (uint32_t i = lane; i < ZBM; i += WAVE) L.pbm[i] = 0;
            wave_sync();
            ZP_ADD(16, ZP_NOW() - zq);
            zq = ZP_NOW();
            const uint64_t op0 = op;
            uint32_t acc = 0, wout = 0;
            bool needwin = false;
#if BPMD_ZST_SCAN
            // the chain of real token starts: one step per token on the scalar unit
            uint64_t mm[ZQ];
            {
                uint32_t o = 0;
#pragma unroll
                for (uint32_t q = 0; q < ZQ; ++q) {
                    uint64_t m = 0;
                    while (o < WAVE * (q + 1)) {
                        const uint32_t j = o - WAVE * q;
                        m |= 1ull << j;
                        o += rdlane(cj[q], j);
                    }
                    mm[q] = m;
                }
            }
            // its tokens in order
            uint32_t K = 0;
#pragma unroll
            for (uint32_t q = 0; q < ZQ; ++q) {
                if ((mm[q] >> lane) & 1ull) {
                    const uint32_t rk = K + below64(mm[q]), a = ca[q], k_ = (a >> 15) & 7u;
                    const uint32_t nb_ = k_ == Z_MATCH   ? (a & 15u) + ((a >> 4) & 7u) + ((a >> 7) & 15u) + ((a >> 11) & 15u)
                                         : k_ == Z_BADDIST ? (a & 15u) + ((a >> 4) & 7u) + ((a >> 7) & 15u)
                                                           : (a & 15u);
                    L.prec[rk] = a;
                    L.ptok[rk] = cb[q];
                    L.poend[rk] = (uint16_t)(lane + WAVE * q + nb_);
                }
                K += (uint32_t)__builtin_popcountll(mm[q]);
            }
            wave_sync();
            // fast() on them, 64 at a time: byte lags by a scan of lag maps,
            // output offsets by a prefix sum, fast()'s checks per token, and
            // the first token where fast() stops (or the window's output cap)
            uint32_t Lc = ((uint32_t)bn - ((uint32_t)(-Ps) & 7u)) >> 3;   // bn = r + 8 L at the window's start
            uint32_t wrel = 0;
            for (uint32_t g = 0; g < K; g += WAVE) {
                const uint32_t t = g + lane;
                const bool act = t < K;
                const uint32_t a = act ? L.prec[t] : 0u, b = act ? L.ptok[t] : 0u, oe = act ? L.poend[t] : 0u;
                const uint32_t kind = (a >> 15) & 7u;
                // the token's lag map: fast()'s refills for each byte lag before it
                const uint32_t c1_ = a & 15u, x_ = (a >> 4) & 7u, c2_ = (a >> 7) & 15u, dx_ = (a >> 11) & 15u;
                const uint32_t nb_ = kind == Z_MATCH ? c1_ + x_ + c2_ + dx_ : kind == Z_BADDIST ? c1_ + x_ + c2_ : c1_;
                const uint32_t r_out = (uint32_t)(-(Ps + (int64_t)oe)) & 7u, r_in = (r_out + nb_) & 7u;
                uint32_t f = 0;
#pragma unroll
                for (uint32_t lv = 0; lv < 4; ++lv) {
                    uint32_t bq = r_in + 8 * lv;
                    bq += bq < 15 ? 16u : 0u;
                    bq -= c1_;
                    if (kind == Z_MATCH || kind == Z_BADDIST) {
                        if (bq < x_) bq += 8;
                        bq -= x_;
                        bq += bq < 15 ? 16u : 0u;
                        bq -= c2_;
                        if (kind == Z_MATCH) {
                            if (bq < dx_) bq += 8;
                            if (bq < dx_) bq += 8;
                            bq -= dx_;
                        }
                    }
                    f |= (((bq - r_out) >> 3) & 3u) << (2 * lv);
                }
                f = act ? f : 0xe4u;   // (identity map)
#pragma unroll
                for (uint32_t d = 1; d < WAVE; d <<= 1) {
                    const uint32_t y = shfl_up32(f, d);
                    f = lane >= d ? lag_compose(y, f) : f;
                }
                const uint32_t La = (f >> (2 * Lc)) & 3u;
                uint32_t osum = act && (kind == Z_LIT || kind == Z_MATCH) ? b >> 16 : 0u;
                const uint32_t olen = osum;
#pragma unroll
                for (uint32_t d = 1; d < WAVE; d <<= 1) {
                    const uint32_t y = shfl_up32(osum, d);
                    osum += lane >= d ? y : 0u;
                }
                const uint32_t oafter = wrel + osum, obefore = oafter - olen;
                const uint64_t ipa = (uint64_t)(((Ps + (int64_t)oe + 7) >> 3) + (int64_t)La);
                const uint64_t dist = b & 0xffffu, opb = op0 + obefore;
                const bool ev = act && (kind == Z_EOB || kind == Z_BADLIT || kind == Z_BADDIST);
                const bool bdist = act && kind == Z_MATCH && dist > opb && dist - opb > wsize;
                const bool ok = act && !ev && !bdist;
                const bool lstop = ok && !(ipa < in_last && op0 + oafter < out_last);
                const bool wcap = ok && oafter >= ZWOUT;
                const uint64_t sm = ballot64(ev || bdist || lstop || wcap);
                const uint32_t first = sm ? (uint32_t)__builtin_ctzll(sm) : (uint32_t)WAVE;
                const bool okf = first < WAVE && rdlane(ok ? 1u : 0u, first) != 0;
                const bool take = act && (lane < first || (lane == first && okf));
                if (take) atomicOr(&L.pbm[obefore >> 5], 1u << (obefore & 31));
                needwin = needwin || ballot64(take && kind == Z_MATCH && dist > opb) != 0;
                const uint32_t last = first < WAVE ? first : (K - g < WAVE ? K - g : (uint32_t)WAVE) - 1;
                const int64_t Pe = Ps + (int64_t)rdlane(oe, last);
                const uint32_t Le = rdlane(La, last);
                acc = g + last + (first < WAVE && !okf ? 0u : 1u);
                wrel = rdlane(first < WAVE && !okf ? obefore : oafter, last);
                Lc = Le;
                if (first < WAVE || g + WAVE >= K) {
                    // fast()'s state after that token
                    ip = (uint64_t)((Pe + 7) >> 3) + Le;
                    bn = (uint32_t)((int64_t)(ip * 8) - Pe);
                    if (first < WAVE) {
                        const uint32_t kf = rdlane(kind, first);
                        if (kf == Z_EOB) {
                            h.mode = TYPE;
                            stop = true;
                        } else if (kf == Z_BADLIT) {
                            err = ST_INVALID_LITERAL_LENGTH;
                            stop = true;
                        } else if (kf == Z_BADDIST) {
                            err = ST_INVALID_DISTANCE_CODE;
                            stop = true;
                        } else if (rdlane(bdist ? 1u : 0u, first)) {
                            err = ST_INVALID_DISTANCE;
                            stop = true;
                        } else if (rdlane(lstop ? 1u : 0u, first)) {
                            stop = true;
                        }   // else the window's output cap: the next window goes on
                    }
                    break;
                }
            }
            wout = wrel;
#else
            // the chain, replaying fast() (inflate_stream.ipp:979-1113)
            uint32_t o = 0;
#pragma unroll
            for (uint32_t q = 0; q < ZQ; ++q) {
                while (!stop && o < WAVE * (q + 1) && wout < ZWOUT) {
                    const uint32_t a = rdlane(ca[q], o - WAVE * q);
                    const uint32_t c1 = a & 15u, x = (a >> 4) & 7u, c2 = (a >> 7) & 15u, dx = (a >> 11) & 15u,
                                   kind = (a >> 15) & 7u;
                    if (bn < 15) {   // pull(); pull();
                        ip += 2;
                        bn += 16;
                    }
                    bn -= c1;
                    if (kind == Z_EOB) {
                        h.mode = TYPE;
                        stop = true;
                        break;
                    }
                    if (kind == Z_BADLIT) {
                        err = ST_INVALID_LITERAL_LENGTH;
                        stop = true;
                        break;
                    }
                    const uint32_t b = rdlane(cb[q], o - WAVE * q);
                    if (kind != Z_LIT) {
                        if (x) {
                            if (bn < x) {
                                ip += 1;
                                bn += 8;
                            }
                            bn -= x;
                        }
                        if (bn < 15) {
                            ip += 2;
                            bn += 16;
                        }
                        bn -= c2;
                        if (kind == Z_BADDIST) {
                            err = ST_INVALID_DISTANCE_CODE;
                            stop = true;
                            break;
                        }
                        if (bn < dx) {
                            ip += 1;
                            bn += 8;
                            if (bn < dx) {
                                ip += 1;
                                bn += 8;
                            }
                        }
                        bn -= dx;
                        const uint64_t dist = b & 0xffffu, opc = op0 + wout;
                        if (dist > opc) {   // from the window
                            if (dist - opc > wsize) {
                                err = ST_INVALID_DISTANCE;
                                stop = true;
                                break;
                            }
                            needwin = true;
                        }
                    }
                    if (lane == 0) {
                        L.ptok[acc] = b;
                        atomicOr(&L.pbm[wout >> 5], 1u << (wout & 31));
                    }
                    ++acc;
                    wout += b >> 16;
                    o += c1 + x + c2 + dx;
                    if (!(ip < in_last && op0 + wout < out_last)) stop = true;
                }
            }
#endif
            ZP_ADD(21, 1);
            ZP_ADD(22, acc);
            ZP_ADD(17, ZP_NOW() - zq);
            zq = ZP_NOW();
            // the accepted tokens' bytes
            if (needwin && !winld) load_window();
            wave_sync();
            {
                int32_t tprev = -1;
                const uint64_t upto = lane == 63 ? ~0ull : ((2ull << lane) - 1);
                const uint64_t wmask = WAVE == 64 ? ~0ull : ((1ull << WAVE) - 1);
                for (uint32_t c = 0; c < wout; c += WAVE) {
                    const uint32_t w = c >> 5, sh = c & 31;
                    const uint64_t lo = L.pbm[w] | ((uint64_t)L.pbm[w + 1] << 32);
                    const uint64_t B = (sh ? (lo >> sh) | ((uint64_t)L.pbm[w + 2] << (64 - sh)) : lo) & wmask;
                    const uint32_t rel = c + lane;
                    const bool act = rel < wout;
                    const int32_t T = tprev + (int32_t)__builtin_popcountll(B & upto);
                    const uint32_t info = act ? L.ptok[T] : (1u << 16);
                    uint32_t val = info & 0xffu;
                    int32_t src = (int32_t)rel - (int32_t)(info & 0xffffu);   // relative to op0
                    bool pend = false;
                    if (act && (info >> 16) >= 3) {
                        if (src >= (int32_t)c) pend = true;
                        else val = L.hist[((uint32_t)op0 + (uint32_t)src) & HM];
                    }
                    while (ballot64(pend)) {   // a match reaching into these bytes
                        const uint32_t from = pend ? (uint32_t)src - c : lane;
                        const uint32_t v2 = shfl32(val, from);
                        const int32_t s2 = (int32_t)shfl32((uint32_t)src, from);
                        const bool p2 = shfl32(pend ? 1u : 0u, from) != 0;
                        if (pend) {
                            if (!p2) {
                                val = v2;
                                pend = false;
                            } else {
                                src = s2;
                            }
                        }
                    }
                    if (act) L.hist[((uint32_t)op0 + rel) & HM] = (uint8_t)val;
                    tprev += (int32_t)__builtin_popcountll(B);
                    wave_sync();
                }
            }
            op = op0 + wout;
            if (op - flushed >= FLUSH_AT) flush_out();
            ZP_ADD(18, ZP_NOW() - zq);
            zq = ZP_NOW();
        }
        // fast()'s reservoir holds the bn stream bits before ip
        pfip = ~0ull;
        pfn = 0;
        if (err) h.mode = BAD;
        ip -= bn >> 3;   // rewind()
        bn &= 7;
        bv = bn ? uni((uint32_t)L.ist[(uint32_t)((int64_t)ip - 1 - sb)]) >> (8 - bn) : 0u;
        ZP_ADD(20, ZP_NOW() - zp0);
        return err;
    };

    // ---- the dynamic header's code lengths, wave-parallel (CODELENS).  Per
    // window of ZQ * WAVE bit offsets from the next symbol's first bit, every
    // lane decodes the code-length symbol (and its repeat bits) that would
    // start at each of its offsets; the scalar unit follows the chain of real
    // symbol starts; the lanes then write the lengths (repeat counts by a
    // prefix sum, a 16's value from the last symbol before it that is not a
    // 16).  The bytes the reference's fill() calls pull are a running maximum
    // over the symbols (each pulls until it has max(root, code + repeat bits)),
    // so ip / bn / bv after the window are the serial loop's.  Only symbols the
    // serial loop would take without stopping are committed: one that lacks
    // input, a 16 with no length before it, or a repeat past the end leaves the
    // rest to the serial loop, which stops or fails exactly as the reference.
    // Returns the symbols committed (0: nothing done).
    auto hdr_par = [&](uint32_t want) -> uint32_t {
        const uint32_t lroot = h.lroot, lmask = (1u << lroot) - 1u;
        const uint32_t* iw = (const uint32_t*)L.ist;
        const uint64_t S = ip * 8 - bn;   // the next symbol's first bit (bn <= ip * 8)
        if ((S >> 3) < ib0 || (S >> 3) >= ib1 || (S >> 3) + ZSPAN > ib0 + IST) stage(S >> 3);
        const uint32_t rb = (uint32_t)(S - 8 * ib0);
        const uint32_t avail = (uint32_t)(8 * (ib1 - ib0));   // staged bits (ib1 <= n_in)
        // candidate word: len | val << 4 | need << 9 | rep << 13 | ok << 21
        uint32_t cw[ZQ];
#pragma unroll
        for (uint32_t q = 0; q < ZQ; ++q) {
            const uint32_t r = rb + lane + WAVE * q, w = r >> 5, sh = r & 31;
            const uint32_t d0 = iw[w], d1 = iw[w + 1];
            const uint32_t v = fsh(d1, d0, sh);   // >= 32 valid bits; a symbol needs <= 14
            const uint32_t sl = L.tab[v & lmask];
            const uint32_t cb = slot_bits(sl);
            const uint32_t val = slot_kind(sl) == K_SPECIAL ? 0u : slot_val(sl);
            const uint32_t x = val == 16 ? 2u : val == 17 ? 3u : val == 18 ? 7u : 0u;
            const uint32_t ev = (v >> cb) & ((1u << x) - 1u);
            const uint32_t rep = val < 16 ? 1u : val == 18 ? 11u + ev : 3u + ev;
            const uint32_t len = cb + x, need = len > lroot ? len : lroot;
            const bool ok = r + need <= avail;
            cw[q] = len | val << 4 | need << 9 | rep << 13 | (ok ? 1u : 0u) << 21;
        }
        // the chain, on the scalar unit
        uint64_t mm[ZQ];
        uint32_t have = h.have, o = 0, pulled = (uint32_t)(ip - ib0) * 8, n = 0;
        bool stop = false;
#pragma unroll
        for (uint32_t q = 0; q < ZQ; ++q) {
            uint64_t m = 0;
            while (!stop && o < WAVE * (q + 1)) {
                const uint32_t j = o - WAVE * q;
                const uint32_t c = rdlane(cw[q], j);
                const uint32_t val = (c >> 4) & 31u, rep = (c >> 13) & 255u;
                if (!((c >> 21) & 1u) || (val == 16 && have == 0) || have + rep > want) {
                    stop = true;
                    break;
                }
                m |= 1ull << j;
                have += rep;
                ++n;
                const uint32_t e = ((rb + o + ((c >> 9) & 15u) + 7u) & ~7u);   // bits pulled through this symbol
                pulled = e > pulled ? e : pulled;
                o += c & 15u;
                if (have == want) stop = true;
            }
            mm[q] = m;
        }
        if (n == 0) return 0;
        ZP_ADD(25, n);
        // the lengths: rank of each chain symbol, its first slot and its value
        uint32_t* rec = L.prec;   // rank -> val | rep << 8
        wave_sync();
        uint32_t K = 0;
#pragma unroll
        for (uint32_t q = 0; q < ZQ; ++q) {
            if ((mm[q] >> lane) & 1ull) rec[K + below64(mm[q])] = ((cw[q] >> 4) & 31u) | ((cw[q] >> 13) & 255u) << 8;
            K += (uint32_t)__builtin_popcountll(mm[q]);
        }
        wave_sync();
        uint32_t base = h.have;                                    // the first slot of this group
        uint32_t prev = base ? uni(L.lens[base - 1]) : 0u;         // the length before it
        for (uint32_t g = 0; g < n; g += WAVE) {
            const uint32_t t = g + lane;
            const uint32_t rv = t < n ? rec[t] : 0u, val = rv & 255u, rep = t < n ? rv >> 8 : 0u;
            // inclusive prefix sums: repeat counts, and the last rank (+1) whose value is not a 16's
            uint32_t sum = rep, last = t < n && val != 16 ? t + 1 : 0u;
            for (uint32_t d = 1; d < WAVE; d <<= 1) {
                const uint32_t s2 = shfl_up32(sum, d), l2 = shfl_up32(last, d);
                if (lane >= d) {
                    sum += s2;
                    last = l2 > last ? l2 : last;
                }
            }
            const uint32_t lastv = last ? rec[last - 1] & 255u : 0u;
            const uint32_t src = last ? (lastv < 16 ? lastv : 0u) : prev;   // 17 / 18 write zeros
            const uint32_t fv = val < 16 ? val : val == 16 ? src : 0u;
            if (t < n)
                for (uint32_t k = 0; k < rep; ++k) L.lens[base + sum - rep + k] = (uint8_t)fv;
            const uint32_t gl = n - g < WAVE ? n - g - 1 : WAVE - 1;   // the group's last lane
            const uint32_t tot = rdlane(sum, gl), fl = rdlane(fv, gl);
            base += tot;
            prev = fl;
        }
        wave_sync();
        lens_dirty = true;
        h.have = have;
        // the reservoir after the last symbol: bytes pulled so far, bits past it
        const uint32_t rend = rb + o;
        ip = ib0 + (pulled >> 3);
        bn = pulled - rend;
        {
            const uint32_t w = rend >> 5, sh = rend & 31;
            const uint32_t v = fsh(uni(iw[w + 1]), uni(iw[w]), sh);
            bv = bn >= 32 ? v : v & ((1u << bn) - 1u);
        }
        return n;
    };

    // ---- the code-length code's lengths (LENLENS) in one step when their bits
    // are staged: lane j takes the 3 bits of length j; fill(3) one length at a
    // time pulls ceil((first bit + 3 n) / 8) bytes in all, so ip / bn / bv
    // are the serial loop's.  Otherwise (input short) the serial loop runs.
    auto lenlens_par = [&]() {
        const uint32_t* iw = (const uint32_t*)L.ist;
        const uint64_t S = ip * 8 - bn;   // bn <= ip * 8
        if ((S >> 3) < ib0 || (S >> 3) >= ib1 || (S >> 3) + ZSPAN > ib0 + IST) stage(S >> 3);
        const uint32_t rb = (uint32_t)(S - 8 * ib0), nb = 3 * (h.ncode - h.have);
        if (rb + nb > (uint32_t)(8 * (ib1 - ib0))) return;
        wave_sync();
        for (uint32_t j = h.have + lane; j < h.ncode; j += WAVE) {
            const uint32_t r = rb + 3 * (j - h.have);
            L.lens[kOrder[j]] = (uint8_t)(fsh(iw[(r >> 5) + 1], iw[r >> 5], r & 31) & 7u);
        }
        wave_sync();
        const uint32_t rend = rb + nb, pulled = (rend + 7) & ~7u;
        if (ib0 + (pulled >> 3) > ip) ip = ib0 + (pulled >> 3);
        bn = (uint32_t)(ip - ib0) * 8 - rend;
        const uint32_t v = fsh(uni(iw[(rend >> 5) + 1]), uni(iw[rend >> 5]), rend & 31);
        bv = bn >= 32 ? v : v & ((1u << bn) - 1u);
        h.have = h.ncode;
        lens_dirty = true;
    };

    int32_t ec = 0;
    int32_t published = 0;
    int32_t data_type = 0;

    if (h.mode == TYPE) h.mode = TYPEDO;
    // prof build: cycles between trips through the switch, by the mode the
    // trip began in (27 type, 28 stored, 29 dynamic header, 30 LEN .. LIT)
    [[maybe_unused]] unsigned long long zsw = ZP_NOW();
    [[maybe_unused]] uint32_t zsm = h.mode;
    auto zbucket = [](uint32_t m) { return m <= TYPEDO ? 27 : m <= COPY ? 28 : m <= CODELENS ? 29 : m <= LIT ? 30 : 31; };
    (void)zbucket;
    for (;;) {
        {
            const unsigned long long n_ = ZP_NOW();
            ZP_ADD(zbucket(zsm), n_ - zsw);
            zsw = n_;
            zsm = h.mode;
        }
        switch (h.mode) {
        case HEAD:
            h.mode = TYPEDO;
            continue;
        case TYPE:
            if (flush == F_BLOCK || flush == F_TREES) goto done;
            [[fallthrough]];
        case TYPEDO: {
            if (h.last) {
                drop(bn % 8);
                h.mode = CHECK;
                continue;
            }
            ZP_ADD(26, 1);
            if (!fill(3)) goto done;
            h.last = take(1);
            const uint32_t t = take(2);
            if (t == 0) {
                h.mode = STORED;
            } else if (t == 1) {
                for (unsigned i = lane; i < 288; i += WAVE) L.flens[i] = i < 144 ? 8 : i < 256 ? 9 : i < 280 ? 7 : 8;
                uint32_t root, used;
                build(BUILD_LENS, L.flens, 288, 0, 9, root, used);
                h.lroot = root;
                for (unsigned i = lane; i < 32; i += WAVE) L.flens[i] = 5;
                uint32_t droot, dused;
                build(BUILD_DISTS, L.flens, 32, used, 5, droot, dused);
                h.droot = droot;
                h.dtab = used;
                h.mode = LEN_;
                if (flush == F_TREES) goto done;
            } else if (t == 2) {
                h.mode = TABLE;
            } else {
                ec = ST_INVALID_BLOCK_TYPE;
                h.mode = BAD;
                goto quiet;
            }
            continue;
        }
        case STORED: {
            drop(bn % 8);
            if (!fill(32)) goto done;
            const uint32_t v = peek(32);
            h.length = v & 0xffffu;
            if (h.length != ((v >> 16) ^ 0xffffu)) {
                ec = ST_INVALID_STORED_LENGTH;
                h.mode = BAD;
                goto quiet;
            }
            bv = 0;   // bitstream::flush
            bn = 0;
            h.mode = COPY_;
            if (flush == F_TREES) goto done;
        }
            [[fallthrough]];
        case COPY_:
            h.mode = COPY;
            [[fallthrough]];
        case COPY: {
            uint64_t n = h.length;
            if (n == 0) {
                h.mode = TYPE;
                continue;
            }
            if (n > n_in - ip) n = n_in - ip;
            if (n > cap - op) n = cap - op;
            if (n == 0) goto done;
            copy_in((uint32_t)n);
            h.length -= (uint32_t)n;
            continue;
        }
        case TABLE:
            zth = ZP_NOW();
            if (!fill(14)) goto done;
            h.nlen = take(5) + 257;
            h.ndist = take(5) + 1;
            h.ncode = take(4) + 4;
            if (h.nlen > 286 || h.ndist > 30) {
                ec = ST_TOO_MANY_SYMBOLS;
                h.mode = BAD;
                goto quiet;
            }
            h.have = 0;
            h.mode = LENLENS;
            [[fallthrough]];
        case LENLENS: {
            if (hpar && h.have < h.ncode && bn <= ip * 8) lenlens_par();
            while (h.have < h.ncode) {
                if (!fill(3)) goto done;
                const uint32_t v = take(3);
                if (lane == 0) L.lens[kOrder[h.have]] = (uint8_t)v;
                lens_dirty = true;
                ++h.have;
            }
            while (h.have < 19) {
                if (lane == 0) L.lens[kOrder[h.have]] = 0;
                ++h.have;
            }
            lens_dirty = true;
            uint32_t root, used;
            const int e = build(BUILD_CODES, L.lens, 19, 0, 7, root, used);
            if (e) {   // inflate_stream.ipp:255-261: BAD, then done() reports it
                ec = e;
                h.mode = BAD;
                continue;
            }
            h.lroot = root;
            h.have = 0;
            h.mode = CODELENS;
        }
            [[fallthrough]];
        case CODELENS: {
            const uint32_t want = h.nlen + h.ndist;
            bool hp = hpar;   // (off for the rest of the call once a window commits nothing)
            while (h.have < want) {
                if (hp && want - h.have >= 8 && bn <= ip * 8) {
                    if (hdr_par(want)) continue;
                    hp = false;
                }
                if (!fill(h.lroot)) goto done;
                const uint32_t s = uni(L.tab[peek(h.lroot)]);
                const uint32_t cb = slot_bits(s);
                // the empty code's slots are {op 64, bits 1, val 0} (ipp:574-584)
                const uint32_t val = slot_kind(s) == K_SPECIAL ? 0u : slot_val(s);
                if (val < 16) {
                    drop(cb);
                    if (lane == 0) L.lens[h.have] = (uint8_t)val;
                    ++h.have;
                    lens_dirty = true;
                    continue;
                }
                uint32_t rep, fv;
                if (val == 16) {
                    if (!fill(cb + 2)) goto done;
                    drop(cb);
                    if (h.have == 0) {
                        ec = ST_INVALID_BIT_LENGTH_REPEAT;
                        h.mode = BAD;
                        goto quiet;
                    }
                    rep = 3 + take(2);
                    wave_sync();
                    fv = uni(L.lens[h.have - 1]);
                } else if (val == 17) {
                    if (!fill(cb + 3)) goto done;
                    drop(cb);
                    rep = 3 + take(3);
                    fv = 0;
                } else {
                    if (!fill(cb + 7)) goto done;
                    drop(cb);
                    rep = 11 + take(7);
                    fv = 0;
                }
                if (h.have + rep > want) {
                    ec = ST_INVALID_BIT_LENGTH_REPEAT;
                    h.mode = BAD;
                    goto quiet;
                }
                wave_sync();
                for (uint32_t j = lane; j < rep; j += WAVE) L.lens[h.have + j] = (uint8_t)fv;
                h.have += rep;
                lens_dirty = true;
            }
            wave_sync();
            if (uni(L.lens[256]) == 0) {
                ec = ST_MISSING_EOB;
                h.mode = BAD;
                goto quiet;
            }
            uint32_t lroot, lused, droot, dused;
            int e = build(BUILD_LENS, L.lens, h.nlen, 0, 9, lroot, lused);
            if (!e) e = build(BUILD_DISTS, L.lens + h.nlen, h.ndist, lused, 6, droot, dused);
            if (e) {   // inflate_stream.ipp:336-349: BAD and return, without done()
                ec = e;
                h.mode = BAD;
                goto quiet;
            }
            h.lroot = lroot;
            h.droot = droot;
            h.dtab = lused;
            h.mode = LEN_;
            ZP_ADD(1, ZP_NOW() - zth);
            if (flush == F_TREES) goto done;
        }
            [[fallthrough]];
        case LEN_:
            h.mode = LEN;
            [[fallthrough]];
        case LEN: {
        len_again:   // (the next symbol without a trip through the switch)
            if (n_in - ip >= 6 && cap - op >= 258) {
                const int32_t e = (par & 1) && n_in - ip >= ZMIN_IN && cap - op >= ZMIN_OUT ? pfast() : fast();
                if (e) {
                    ec = e;
                    goto quiet;
                }
                continue;
            }
            ZP_ADD(24, 1);
            if (!fill(h.lroot)) goto done;
            uint32_t s = uni(L.tab[peek(h.lroot)]);
            if (is_link(s)) {
                const uint32_t w = h.lroot + slot_bits(s);
                if (!fill(w)) goto done;
                s = uni(L.tab[slot_val(s) + (peek(w) >> h.lroot)]);
                drop(h.lroot + slot_bits(s));
            } else {
                drop(slot_bits(s));
            }
            const uint32_t kind = slot_kind(s), val = slot_val(s);
            if (kind == K_VAL) {
                // LIT, in place: the byte, or LIT kept for the next call
                if (op == cap) {
                    h.length = val;
                    h.mode = LIT;
                    goto done;
                }
                put(val);
                goto len_again;
            }
            if (kind == K_EOB) {
                h.mode = TYPE;
                continue;
            }
            if (kind != K_LEN) {
                ec = ST_INVALID_LITERAL_LENGTH;
                h.mode = BAD;
                goto quiet;
            }
            h.length = len_base(val);
            h.extra = len_extra(val);
            h.mode = LENEXT;
        }
            [[fallthrough]];
        case LENEXT:
            if (h.extra) {
                if (!fill(h.extra)) goto done;
                h.length += take(h.extra);
            }
            h.was = h.length;
            h.mode = DIST;
            [[fallthrough]];
        case DIST: {
            if (!fill(h.droot)) goto done;
            uint32_t d = uni(L.tab[h.dtab + peek(h.droot)]);
            if (is_link(d)) {
                const uint32_t w = h.droot + slot_bits(d);
                if (!fill(w)) goto done;
                d = uni(L.tab[h.dtab + slot_val(d) + (peek(w) >> h.droot)]);
                drop(h.droot + slot_bits(d));
            } else {
                drop(slot_bits(d));
            }
            if (slot_kind(d) != K_VAL) {
                ec = ST_INVALID_DISTANCE_CODE;
                h.mode = BAD;
                goto quiet;
            }
            h.offset = dist_base(slot_val(d));
            h.extra = dist_extra(slot_val(d));
            h.mode = DISTEXT;
        }
            [[fallthrough]];
        case DISTEXT:
            if (h.extra) {
                if (!fill(h.extra)) goto done;
                h.offset += take(h.extra);
            }
            h.mode = MATCH;
            [[fallthrough]];
        case MATCH: {
            if (op == cap) goto done;
            uint64_t n = h.length;
            if (h.offset > op) {   // from the window as it was when the call began
                const uint32_t back = (uint32_t)(uint16_t)(h.offset - op);
                if (back > h.wsize) {
                    ec = ST_INVALID_DISTANCE;
                    h.mode = BAD;
                    goto quiet;
                }
                if (n > back) n = back;
            }
            if (n > cap - op) n = cap - op;
            copy_back(h.offset, (uint32_t)n);
            h.length -= (uint32_t)n;
            if (op - flushed >= FLUSH_AT) flush_out();
            if (h.length == 0) {
                h.mode = LEN;
                goto len_again;
            }
            continue;
        }
        case LIT:
            if (op == cap) goto done;
            put(h.length);
            h.mode = LEN;
            continue;
        case CHECK:
            h.mode = DONE;
            [[fallthrough]];
        case DONE:
            ec = ST_END_OF_STREAM;
            goto done;
        case BAD:
            goto done;
        default:   // SYNC: unreachable (the reference throws logic_error)
            ec = ST_STREAM_ERROR;
            goto quiet;
        }
    }

done:   // the done() lambda, inflate_stream.ipp:88-119
    ztd = ZP_NOW();
    ZP_ADD(zbucket(zsm), ztd - zsw);
    flush_out();
    if (op && h.mode < BAD && (h.mode < CHECK || flush != F_FINISH)) {
        // window::write (window.hpp:109-141): the last min(n, capacity) bytes
        const uint64_t k = op < wcap ? op : wcap;
        for (uint64_t j = op - k + lane; j < op; j += WAVE)
            st->win[(uint32_t)(h.wpos + j) & (wcap - 1)] = L.hist[(uint32_t)j & HM];
        h.wpos = (uint32_t)((h.wpos + op) & (wcap - 1));
        h.wsize = (uint32_t)((uint64_t)h.wsize + op < wcap ? h.wsize + op : wcap);
    }
    data_type = (int32_t)(bn + (h.last ? 64u : 0u) + (h.mode == TYPE ? 128u : 0u) +
                          (h.mode == LEN_ || h.mode == COPY_ ? 256u : 0u));
    if (((ip == 0 && op == 0) || flush == F_FINISH) && ec == 0) ec = ST_NEED_BUFFERS;
    published = 1;
quiet:
    if (!ztd) ztd = ZP_NOW();
    flush_out();
    h.bv = bv;
    h.bn = bn;
    if (tab_dirty)
        for (unsigned i = lane; i < kCodes; i += WAVE) st->codes[i] = L.tab[i];
    if (lens_dirty)
        for (unsigned i = lane; i < kLens; i += WAVE) st->lens[i] = L.lens[i];
    if (lane == 0) {
        st->h = h;
        res->in_used = ip;
        res->out_used = op;
        res->ec = ec;
        res->data_type = data_type;
        res->published = published;
    }
    ZP_ADD(6, ZP_NOW() - ztd);
    ZP_ADD(7, ZP_NOW() - zt0);
    ZP_ADD(11, op);
    ZP_ADD(13, 1);
    ZP_ADD(14, ip);
    ZP_FLUSH();
}

#ifndef BPMD_ZSTREAM_HOST
#ifdef BPMD_PROF
__device__ State g_warm_st;
__device__ uint8_t g_warm_out[1 << 16];
__device__ Result g_warm_res;
#endif
__global__ void __launch_bounds__(WAVE)
zstream_write_kernel(State* __restrict__ st, const uint8_t* __restrict__ in, uint64_t n_in, uint8_t* __restrict__ out,
                     uint64_t cap, int flush, Result* __restrict__ res, int par)
{
    __shared__ Lds L;
#ifdef BPMD_PROF
    // diagnostics (BPMD_ZSTREAM_WARM=1): the same call first on a copy of the
    // state, uncounted, so the counted call runs with warm caches
    if (par & 2) {
        static_assert(sizeof(State) % 4 == 0, "state copy in dwords");
        for (unsigned i = lane_id(); i < sizeof(State) / 4; i += WAVE)
            ((uint32_t*)&g_warm_st)[i] = ((const uint32_t*)st)[i];
        __syncthreads();
        zstream_run(L, &g_warm_st, in, n_in, g_warm_out, cap < sizeof g_warm_out ? cap : sizeof g_warm_out, flush,
                    &g_warm_res, (par & 9) | 4);
        __syncthreads();
    }
#endif
    zstream_run(L, st, in, n_in, out, cap, flush, res, par & 9);
}

// the micro-batcher's launch (pmd_stream.hip): one write() of a different
// stream per workgroup, each exactly the call zstream_write_kernel makes
__global__ void __launch_bounds__(WAVE)
zstream_write_batch_kernel(const ZCall* __restrict__ calls, int par)
{
    __shared__ Lds L;
    const ZCall c = calls[blockIdx.x];
    zstream_run(L, (State*)c.st, c.in, c.n_in, c.out, c.cap, c.flush, (Result*)c.res, par & 9);
}
#endif

}  // namespace zst
}  // namespace bpmd

#ifndef BPMD_ZSTREAM_HOST
// One inflate_stream::write() on `stream`: st is the stream's device state,
// in/out device buffers of n_in bytes and `cap` bytes of room.
// BPMD_ZSTREAM_PAR=0 (or bpmd_diag_set_zstream_parallel(0)): the serial
// inflate_fast loop instead of the wave-parallel one (same results)
static std::atomic<int> g_zst_par{-1};

// on: -1 the environment's default, else bit 0 the wave-parallel
// inflate_fast, bit 3 the serial code-length loop (BPMD_ZSTREAM_HPAR=0)
extern "C" int bpmd_diag_set_zstream_parallel(int on)
{
    g_zst_par.store(on < 0 ? -1 : (on & 9));
    return 0;
}

extern "C" int bpmd_internal_zstream_write(void* st, const uint8_t* in, uint64_t n_in, uint8_t* out, uint64_t cap,
                                           int flush, void* res, hipStream_t stream)
{
    using namespace bpmd::zst;
    static const int env_par = [] {
        const char* e = getenv("BPMD_ZSTREAM_PAR");
        const char* hp = getenv("BPMD_ZSTREAM_HPAR");
        return (e ? (atoi(e) ? 1 : 0) : 1) | (hp && hp[0] == '0' ? 8 : 0);
    }();
    const int o = g_zst_par.load();
    int par = o < 0 ? env_par : o;
#ifdef BPMD_PROF
    static const int env_warm = [] {
        const char* e = getenv("BPMD_ZSTREAM_WARM");
        return e && atoi(e) ? 2 : 0;
    }();
    par |= env_warm;
#endif
    hipLaunchKernelGGL(zstream_write_kernel, dim3(1), dim3(bpmd::WAVE), 0, stream, (State*)st, in, n_in, out, cap,
                       flush, (Result*)res, par);
    return (int)hipGetLastError();
}

// n write() calls of n different streams in one launch (calls: device array
// of bpmd::zst::ZCall)
extern "C" int bpmd_internal_zstream_write_batch(const void* calls, uint32_t n, hipStream_t stream)
{
    using namespace bpmd::zst;
    if (n == 0) return 0;
    static const int env_par = [] {
        const char* e = getenv("BPMD_ZSTREAM_PAR");
        const char* hp = getenv("BPMD_ZSTREAM_HPAR");
        return (e ? (atoi(e) ? 1 : 0) : 1) | (hp && hp[0] == '0' ? 8 : 0);
    }();
    const int o = g_zst_par.load();
    const int par = o < 0 ? env_par : o;
    hipLaunchKernelGGL(zstream_write_batch_kernel, dim3(n), dim3(bpmd::WAVE), 0, stream, (const ZCall*)calls, par);
    return (int)hipGetLastError();
}

// diagnostic counters (meaningful only in the -DBPMD_PROF build)
extern "C" int bpmd_diag_zstream_counters(unsigned long long* out, int reset)
{
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(bpmd::zst::g_zprof), sizeof(unsigned long long) * bpmd::zst::ZPN) != hipSuccess)
        return -1;
    if (reset) {
        unsigned long long z[bpmd::zst::ZPN] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(bpmd::zst::g_zprof), z, sizeof z) != hipSuccess) return -1;
    }
    return 0;
}
#endif
