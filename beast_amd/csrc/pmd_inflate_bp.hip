// pmd_inflate_bp.hip -- block-parallel inflate of long payloads (SURVEY.md
// 8(a) inflate path; VERDICT r2 "a fast decoder for one long message").
//
// One lane decodes one DEFLATE stream serially at the lane kernel's rate,
// but a 64 KiB payload is ~20 ms of one lane's time, and a batch of few long
// payloads fills few lanes.  Beast (like zlib) cuts a block every
// lit_bufsize - 1 symbols (deflate_stream.ipp:1406, :679), this library's
// deflater every 4 KiB chunk, so a long payload holds many blocks, and a
// dynamic block's header is self-validating: HLIT/HDIST ranges, a complete
// code-length code, code lengths that fill complete literal/length and
// distance codes with an end-of-block code (inflate_stream.ipp:222-354,
// 574-617).  So:
//
//   1. stats (bp_stats_kernel): per long payload a region size R (the
//      batch's long bytes over four segments per lane of the chip, 1-8 KiB),
//      its region count and symbol workspace; exclusive sums give every
//      payload's first task and workspace offset; bp_fit_kernel keeps the
//      payloads that fit the stream's workspace capacity (the rest go to the
//      wave kernel) -- no host read-back (see the driver below);
//   2. scan (bp_scan_kernel, two passes, one wave per region): region 0's
//      candidate is the payload's first bit; region k > 0 is searched for a
//      stored block (LEN / NLEN, then a look at the block after it), and a
//      region without one -- in a payload without empty stored blocks (sync
//      markers) -- for the first bit offset that passes a cheap filter
//      (block type 2, HLIT <= 29, HDIST <= 29, a complete code-length code by
//      Kraft sum) and then the full header check above.  Then
//      (bp_slots_kernel) each candidate gets a symbol slot sized by its
//      compressed span;
//   3. decode (pmd_inflate_lane3.hip, segment mode): one lane per candidate
//      from its header to the first block boundary that is the payload's
//      next candidate, as 16-bit symbols (bp.h); candidates that are not
//      real block starts are simply never reached;
//   4. resolve (bp_resolve_kernel): one wave per payload follows the chain
//      from the first segment (each segment names the candidate it handed
//      off to), turns references into the bytes already written, and applies
//      the reference's rules in stream order: the first invalid distance,
//      the output capacity, the first decode error or the end of the stream
//      (inflate_stream.ipp:475-514; out_len / status as pmd_inflate.hip);
//   5. a payload whose segment outgrew its slot (output far above the
//      region estimate) is decoded again by the wave kernel (pmd_inflate.hip),
//      from a device-side list.
//
// Results are those of the serial decoders bit for bit
// (tests/test_gpu_inflate_bp.py against the oracle).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <atomic>
#include <mutex>
#include <vector>

#include "bp.h"
#include "canon.h"
#include "pmd_common.h"

extern "C" void* bpmd_internal_scratch(hipStream_t s, size_t bytes, int which);
extern "C" int bpmd_internal_inflate_lane3_seg(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                                               uint32_t n_tasks, const void* tasks, uint16_t* sym, void* res,
                                               uint32_t raw, uint32_t* qctr, uint32_t grid_wgs, hipStream_t stream,
                                               const uint32_t* n_dev);
extern "C" int bpmd_internal_inflate_wave_ordered(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                                                  uint32_t n, uint8_t* out, const uint64_t* out_off,
                                                  const uint32_t* out_cap, uint32_t* out_len, int32_t* status,
                                                  uint32_t raw, const uint32_t* mask_key, const uint32_t* order,
                                                  const uint32_t* limit, hipStream_t stream);

namespace bpmd {
namespace bp {

constexpr uint32_t SEG_OUT = 4096;       // target output per region (a C2 message's worth)
constexpr uint32_t R_MIN = 1024, R_MAX = 8192;
constexpr uint32_t STAGE_EXTRA = 320;    // staged bytes past a region: the longest dynamic header (2 283 bits)
constexpr uint32_t STAGE_BYTES = R_MAX + STAGE_EXTRA + 16;   // + one dword before the region
constexpr uint32_t SLACK = 512;          // symbols of slack per slot
constexpr uint32_t SCAN_WAVES = 4;       // waves per scan workgroup (they share the Kraft table)

// per-payload stats (index i of the long list)
struct Stat {
    uint32_t regions;   // region count
    uint32_t R;         // region size, bytes
    uint32_t F16;       // slot symbols per compressed byte, 16.16 (1.25 x min(cap / len, 4))
    uint32_t pad;
};

__global__ void __launch_bounds__(256)
bp_sum_kernel(const uint32_t* __restrict__ in_len, const uint32_t* __restrict__ order,
              const uint32_t* __restrict__ nlong, uint32_t n, unsigned long long* __restrict__ total)
{
    unsigned long long acc = 0;
    const uint32_t nl = *nlong;
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < nl && i < n; i += gridDim.x * 256u) acc += in_len[order[i]];
    for (int d = 32; d >= 1; d >>= 1) acc += __shfl_down(acc, d);
    if ((threadIdx.x & 63) == 0 && acc) atomicAdd(total, acc);
}

// Region size: the batch's long bytes over 4 segments per lane of the chip
// (BPMD_BP_SEGS; finer regions balance the segment kernel's lanes better,
// at the cost of scanning more regions), within
// [R_MIN, R_MAX].  Round 3 never went below SEG_OUT of output at the
// payload's provisioned ratio (-DBPMD_BP_R_FLOOR), which left an 8-way shard
// of C5 with 4 KiB regions and half the chip's lanes idle.
__global__ void __launch_bounds__(256)
bp_stats_kernel(const uint32_t* __restrict__ in_len, const uint32_t* __restrict__ out_cap,
                const uint32_t* __restrict__ order, const uint32_t* __restrict__ nlong, uint32_t n,
                const unsigned long long* __restrict__ total, uint32_t lanes, uint32_t segs_per_lane,
                Stat* __restrict__ st, uint32_t* __restrict__ regions, unsigned long long* __restrict__ words)
{
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    uint32_t na = 0;
    unsigned long long w = 0;
    Stat s = {0, 0, 0, 0};
    if (i < *nlong && in_len[order[i]] < (1u << 28)) {   // bit positions fit 32 bits
        const uint32_t m = order[i];
        const uint32_t len = in_len[m], cap = out_cap[m];
        // output per compressed byte the caller provisioned, capped at 4
        const uint64_t e16 = cap >= 4ull * len ? (4ull << 16) : (((uint64_t)cap << 16) / (len ? len : 1u));
        uint64_t R = cap ? ((uint64_t)SEG_OUT * len) / cap : R_MAX;
        const uint64_t share = *total / ((uint64_t)segs_per_lane * (lanes ? lanes : 1u));
#ifdef BPMD_BP_R_FLOOR   // diagnostics: round 3's rule (never below SEG_OUT of output)
        R = R < share ? share : R;
#else
        // the share alone: a batch with fewer long bytes than the chip's lanes
        // want cuts its payloads finer, down to R_MIN (about one of Beast's
        // 1023-symbol blocks of near-random data; an 8-way shard of C5 has
        // 1 KiB a lane), not at SEG_OUT of output
        (void)R;
        R = share;
#endif
        R = R < R_MIN ? R_MIN : R > R_MAX ? R_MAX : R;
        R &= ~255ull;
        na = (uint32_t)((len + R / 2) / R);   // a last region shorter than R / 2 joins the one before
        na = na ? na : 1u;
        s.regions = na;
        s.R = (uint32_t)R;
        s.F16 = (uint32_t)((e16 * 5) >> 2);
        // slots: span to the third candidate after it (rounded up to bytes;
        // the spans add up to at most 3 (len + na)) x F16, plus SLACK each,
        // after the payload's guard
        w = ((((unsigned long long)3 * (len + na)) * s.F16) >> 16) + (unsigned long long)SLACK * na + SYM_GUARD + 64;
    }
    st[i] = s;
    regions[i] = na;
    words[i] = w;
}

struct Totals {
    unsigned long long tasks;
    unsigned long long words;
};

__global__ void bp_totals_kernel(const uint32_t* __restrict__ regions, const uint32_t* __restrict__ task_base,
                                 const unsigned long long* __restrict__ words,
                                 const unsigned long long* __restrict__ word_base, uint32_t n,
                                 Totals* __restrict__ tot)
{
    if (threadIdx.x == 0) {
        tot->tasks = (unsigned long long)task_base[n - 1] + regions[n - 1];
        tot->words = word_base[n - 1] + words[n - 1];
    }
}

// diagnostics (bpmd_diag_bp_counters): [0] payloads resolved, [1] segments
// on their chains, [2] payloads sent to the wave kernel by the resolve (a
// segment outgrew its slot), [3] payloads sent to it by bp_fit_kernel (over
// the stream's workspace capacity); with -DBPMD_BP_DIAG
// (contended atomics: timing changes) also [4] regions scanned, [5] found a
// stored block, [6] searched for dynamic headers, [7] full dynamic-header
// checks, [8-10] scan cycles staging / stored search / dynamic search
#ifdef BPMD_BP_DIAG
#define BP_DIAG(x) x
#else
#define BP_DIAG(x)
#endif
__device__ unsigned long long g_bp_diag[12];
// the last payload that fell back to the wave kernel (bpmd_diag_bp_fallback):
// message, segment (task - first task), segment status, symbols, slot symbols
__device__ uint32_t g_bp_fb[8];

// Without a read-back the decode workspace has a fixed capacity (tasks,
// symbol words): the long payloads that fit are a prefix of the order
// (the sums only grow), the rest go to the wave kernel's list.  fit[0] =
// payloads decoded block-parallel, fit[1] = their tasks; *tot = the totals
// the whole list would need (the host grows the capacity from them).
__global__ void __launch_bounds__(256)
bp_fit_kernel(const uint32_t* __restrict__ nlong, const uint32_t* __restrict__ regions,
              const uint32_t* __restrict__ task_base, const unsigned long long* __restrict__ words,
              const unsigned long long* __restrict__ word_base, uint32_t n, unsigned long long cap_tasks,
              unsigned long long cap_words, const uint32_t* __restrict__ order, uint32_t* __restrict__ fit,
              Totals* __restrict__ tot, uint32_t* __restrict__ fb_list, uint32_t* __restrict__ fb_count)
{
    const uint32_t nl = *nlong < n ? *nlong : n;
    auto fits = [&](uint32_t k) {   // the first k payloads fit
        return k == 0 || ((unsigned long long)task_base[k - 1] + regions[k - 1] <= cap_tasks &&
                          word_base[k - 1] + words[k - 1] <= cap_words);
    };
    uint32_t lo = 0, hi = nl;   // largest k <= nl with fits(k)
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (fits(mid)) lo = mid;
        else hi = mid - 1;
    }
    const uint32_t nfit = lo;
    if (threadIdx.x == 0) {
        fit[0] = nfit;
        fit[1] = nfit ? task_base[nfit - 1] + regions[nfit - 1] : 0u;
        tot->tasks = n ? (unsigned long long)task_base[n - 1] + regions[n - 1] : 0ull;
        tot->words = n ? word_base[n - 1] + words[n - 1] : 0ull;
    }
    for (uint32_t i = nfit + threadIdx.x; i < nl; i += blockDim.x) fb_list[atomicAdd(fb_count, 1u)] = order[i];
    // capacity spills (bpmd_diag_bp_counters [3]): payloads the workspace
    // could not take this call
    if (threadIdx.x == 0 && nl > nfit) atomicAdd(&g_bp_diag[3], (unsigned long long)(nl - nfit));
}


// ------------------------------------------------------------------ scan
__device__ __forceinline__ uint32_t wave_lane() { return threadIdx.x & 63u; }

static __constant__ const uint8_t kClenOrderBp[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// 32 bits of the staged region at LDS bit b (the stage is padded with zeros)
__device__ __forceinline__ uint32_t peek32(const uint32_t* S, uint32_t b)
{
    const uint32_t w = b >> 5;
    return __builtin_amdgcn_alignbit(S[w + 1], S[w], b & 31u);
}

// Bit sources for the header checks: the staged region (LDS) or the payload
// in global memory (stored candidates look at the block after them).
struct LdsBits {
    const uint32_t* S;
    __device__ __forceinline__ uint32_t peek(uint32_t b) const { return peek32(S, b); }
};
struct GlobalBits {
    const uint32_t* A;   // the payload's aligned base
    uint32_t E;          // dwords holding payload bytes
    __device__ __forceinline__ uint32_t peek(uint32_t b) const
    {
        const uint32_t w = b >> 5;
        const uint32_t lo = w < E ? A[w] : 0u, hi = w + 1 < E ? A[w + 1] : 0u;
        return __builtin_amdgcn_alignbit(hi, lo, b & 31u);
    }
};

// Is there a dynamic-block header at bit b (source bits, payload bits end at
// lim)?  The reference's header rules (inflate_stream.ipp:222-354: HLIT /
// HDIST ranges, a complete code-length code, the repeat rules) plus what
// every real encoder's Huffman trees satisfy and random bits almost never do
// (tests: no false candidate in real payloads): a complete literal/length
// code of at least 16 codes with an end-of-block code, and a complete,
// single or empty distance code.  A block this rejects is only not a
// segment start.
template <class Bits>
__device__ bool dyn_header_ok(const Bits& B, uint32_t b, uint32_t lim)
{
    if (b + 17 > lim) return false;
    const uint32_t h = B.peek(b + 3);
    const uint32_t nlen = (h & 31u) + 257, ndist = ((h >> 5) & 31u) + 1, ncode = ((h >> 10) & 15u) + 4;
    if (nlen > 286 || ndist > 30) return false;
    uint32_t p = b + 17;
    if (p + 3 * ncode > lim) return false;
    uint64_t clp = 0;   // code-length-code lengths, 3 bits per symbol
    {
        const uint32_t a = B.peek(p), c = B.peek(p + 30);
        const uint64_t x = (uint64_t)(a & 0x3fffffffu) | ((uint64_t)c << 30);   // 57 bits: fields 0-18
        for (uint32_t i = 0; i < ncode; ++i) clp |= ((x >> (3 * i)) & 7ull) << (3 * kClenOrderBp[i]);
    }
    p += 3 * ncode;
    uint64_t acc = 0;
#pragma unroll
    for (int i = 0; i < 19; ++i) acc += 1ull << (5 * ((clp >> (3 * i)) & 7u));
    uint32_t c[16];
#pragma unroll
    for (int l = 0; l < 16; ++l) c[l] = (l >= 1 && l <= 7) ? (uint32_t)(acc >> (5 * l)) & 31u : 0u;
    lp3::Canon<7> tc;
    if (lp3::make_canon<7>(c, 7, 0, tc)) return false;
    // symbols in canonical order, 5 bits each, in registers
    uint64_t cls0 = 0, cls1 = 0;
    {
        uint64_t offs = 0;
        uint32_t cu = 0;
#pragma unroll
        for (int l = 1; l <= 7; ++l) {
            offs |= (uint64_t)cu << (5 * l);
            cu += c[l];
        }
#pragma unroll
        for (int i = 0; i < 19; ++i) {
            const uint32_t l = (uint32_t)(clp >> (3 * i)) & 7u;
            const uint32_t at = (uint32_t)(offs >> (5 * l)) & 31u;
            offs += l ? 1ull << (5 * l) : 0ull;
            if (l) {
                if (at < 12) cls0 |= (uint64_t)i << (5 * at);
                else cls1 |= (uint64_t)i << (5 * (at - 12));
            }
        }
    }
    const uint32_t want = nlen + ndist;
    uint32_t have = 0, prev = 0, kl = 0, kd = 0, nl_codes = 0, nd_codes = 0, md = 0;
    bool eob = false;
    uint32_t rp = p;   // 64 bits from rp in r
    uint64_t r = (uint64_t)B.peek(p) | ((uint64_t)B.peek(p + 32) << 32);
    while (have < want) {
        if (p + 7 > lim) return false;
        if (p - rp >= 32) {
            rp = p;
            r = (uint64_t)B.peek(p) | ((uint64_t)B.peek(p + 32) << 32);
        }
        const uint32_t v = (uint32_t)(r >> (p - rp));
        const uint32_t c7 = __builtin_bitreverse32(v) >> 25;
        const lp3::Sym y = lp3::canon_decode<7>(tc.Q, c7);
        if (y.inval) return false;
        const uint32_t ix = y.idx < 19 ? y.idx : 0u;
        const uint32_t sym = ix < 12 ? (uint32_t)(cls0 >> (5 * ix)) & 31u : (uint32_t)(cls1 >> (5 * (ix - 12))) & 31u;
        uint32_t val = sym, rep = 1, used = y.L;
        if (sym >= 16) {
            const uint32_t xb = sym == 16 ? 2u : (sym == 17 ? 3u : 7u);
            const uint32_t x = (v >> y.L) & ((1u << xb) - 1u);
            used += xb;
            if (sym == 16) {
                if (have == 0) return false;
                val = prev;
                rep = 3 + x;
            } else {
                val = 0;
                rep = (sym == 17 ? 3u : 11u) + x;
            }
            if (have + rep > want) return false;
        }
        if (p + used > lim) return false;
        p += used;
        if (val) {
            const uint32_t a = have, e = have + rep;
            const uint32_t nl = (e < nlen ? e : nlen) > a ? (e < nlen ? e : nlen) - a : 0u;
            const uint32_t nd = rep - nl;
            kl += nl << (15 - val);
            kd += nd << (15 - val);
            nl_codes += nl;
            nd_codes += nd;
            md = nd && val > md ? val : md;
            if (a <= 256 && 256 < e) eob = true;
            if (kl > 32768u || kd > 32768u) return false;   // over-subscribed
        }
        prev = val;
        have += rep;
    }
    if (!eob || kl != 32768u || nl_codes < 16) return false;
    if (kd != 32768u && kd != 0u && !(nd_codes == 1 && md == 1)) return false;
    return true;
}

// Could a fixed-code block start at bit b?  BFINAL 0, BTYPE 1, then the
// first FW symbols of the fixed code (inflate_stream.ipp:865-930; RFC 1951
// 3.2.6) decoded arithmetically: no end of block among them (a Beast peer cuts
// a block every lit_bufsize - 1 = 1 023 symbols, deflate_stream.ipp:1406),
// no invalid literal/length (286, 287) or distance (30, 31) code, and at most
// FMAX length codes.  Random bits decode as ~22 % length codes (the 7-bit
// codes 257-279 and 8-bit 280-285), the near-random data a Beast peer codes
// in fixed blocks as 0-5 % (C5: tr_flush_block picks fixed for it,
// deflate_stream.ipp:1425-1518): the test tells a real block start from the
// ~4 random offsets per KiB that show a fixed header after seven zero bits
// (a fixed block's end-of-block code).  Random bits pass about 1 in 10^4
// (96 symbols, at most 6 lengths; 48 and 4 let ~0.3 % through, about one
// false start per Beast C5 payload: a segment before two of them gets a slot
// sized short, and 21-37 % of the payloads fell back to the wave kernel,
// profiles/r06l_beast_shard.log).  A block it rejects -- a fixed block of
// text with many matches, say -- is only not a segment start.  (FW * 9 bits
// fit in STAGE_EXTRA.)
#ifndef BPMD_BP_FIXED
// bit 0: a stored block followed by a fixed block that passes fixed_block_ok
// is a candidate (round 5: only an empty one); bit 1: pass 2 also searches
// fixed-block starts after a fixed block's end-of-block code, checked by
// fixed_block_ok and fixed_eob_at (without the latter, 21-37 % of C5's
// Beast payloads fell back: profiles/r06l_beast_shard.log)
#define BPMD_BP_FIXED 3
#endif
constexpr uint32_t FW = 96, FMAX = 6;
template <class Bits>
__device__ bool fixed_block_ok(const Bits& B, uint32_t b, uint32_t lim)
{
    if (b + 3 + FW * 9 > lim) return false;
    if ((B.peek(b) & 7u) != 2u) return false;   // BFINAL 0, BTYPE 1
    uint32_t p = b + 3, nm = 0;
    for (uint32_t k = 0; k < FW; ++k) {
        if (p + 32 > lim) return false;
        const uint32_t v = B.peek(p);
        const uint32_t c9 = __builtin_bitreverse32(v) >> 23;   // the next 9 code bits, first bit highest
        const uint32_t c7 = c9 >> 2, c8 = c9 >> 1;
        uint32_t sym, len;
        if (c7 <= 23u) { sym = 256u + c7; len = 7; }
        else if (c8 >= 48u && c8 <= 191u) { sym = c8 - 48u; len = 8; }
        else if (c8 >= 192u && c8 <= 199u) { sym = 280u + c8 - 192u; len = 8; }
        else { sym = 144u + c9 - 400u; len = 9; }
        if (sym == 256u || sym > 285u) return false;
        p += len;
        if (sym > 256u) {
            if (++nm > FMAX) return false;
            const uint32_t li = sym - 257u;
            const uint32_t xl = (li < 8u || li == 28u) ? 0u : ((li - 4u) >> 2);
            const uint32_t v2 = B.peek(p + xl);
            const uint32_t d5 = __builtin_bitreverse32(v2) >> 27;
            if (d5 >= 30u) return false;
            p += xl + 5u + (d5 < 4u ? 0u : (d5 >> 1) - 1u);
        }
    }
    return true;
}

// Pass 2's fixed-block starts follow a fixed block's end-of-block code
// (seven zero bits).  Inside a fixed block of literals the same ten bits
// show about 4 times per KiB (a literal code ending in zeros, the next one
// starting 010), and decoding from there resynchronises with the block's own
// codes within a few symbols, so fixed_block_ok cannot tell.  What tells is
// the stream before: parsed with the fixed code from FBACK bits earlier
// (also resynchronised by then), a real end-of-block code starts a symbol
// at t = b - 7; inside a block the symbol boundaries pass over t (the zeros
// are the tail of one code and the head of the next).
constexpr uint32_t FBACK = 480;
template <class Bits>
__device__ bool fixed_eob_at(const Bits& B, uint32_t from, uint32_t t)
{
    uint32_t p = from;
    for (uint32_t k = 0; k < 160 && p < t; ++k) {
        const uint32_t c9 = __builtin_bitreverse32(B.peek(p)) >> 23;
        const uint32_t c7 = c9 >> 2, c8 = c9 >> 1;
        uint32_t sym;
        if (c7 <= 23u) { sym = 256u + c7; p += 7; }
        else if (c8 >= 48u && c8 <= 191u) { sym = c8 - 48u; p += 8; }
        else if (c8 >= 192u && c8 <= 199u) { sym = 280u + c8 - 192u; p += 8; }
        else { sym = 144u; p += 9; }
        if (sym > 256u && sym <= 285u) {   // length extra bits, distance code, its extra bits
            const uint32_t li = sym - 257u;
            p += (li < 8u || li == 28u) ? 0u : ((li - 4u) >> 2);
            const uint32_t d5 = __builtin_bitreverse32(B.peek(p)) >> 27;
            p += 5u + (d5 < 4u ? 0u : d5 < 30u ? (d5 >> 1) - 1u : 0u);
        }
    }
    return p == t;
}

// Kraft sum x 128 of four 3-bit code-length-code lengths (0 = unused)
__device__ __forceinline__ uint32_t kraft4(uint32_t f)
{
    uint32_t k = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t l = (f >> (3 * j)) & 7u;
        k += l ? 128u >> l : 0u;
    }
    return k;
}

// Could a dynamic-block header start at bit b?  Block type 2, HLIT <= 29,
// HDIST <= 29 and a complete code-length code (about 1 in 1 000 random
// offsets pass).
template <class Bits>
__device__ __forceinline__ bool dyn_header_quick(const Bits& B, uint32_t b, uint32_t lim)
{
    if (b + 17 + 57 > lim) return false;
    const uint32_t h = B.peek(b);
    if (((h >> 1) & 3u) != 2u || ((h >> 3) & 31u) > 29u || ((h >> 8) & 31u) > 29u) return false;
    const uint32_t ncode = ((h >> 13) & 15u) + 4;
    const uint32_t a = B.peek(b + 17), c = B.peek(b + 47);
    const uint64_t x = (uint64_t)(a & 0x3fffffffu) | ((uint64_t)c << 30);
    uint32_t kr = 0;
    for (uint32_t i = 0; i < ncode; ++i) {
        const uint32_t l = (uint32_t)(x >> (3 * i)) & 7u;
        kr += l ? 128u >> l : 0u;
    }
    return kr == 128u;
}

// Is there a stored block whose LEN field is payload byte pb (LEN == ~NLEN,
// checked by the caller)?  The bits before it must be the zero padding and
// block type every encoder writes (checked by the caller), the block must end
// inside the payload, and what follows must look like a block: the payload's
// end, another stored block, a plausible dynamic header, or -- after an
// empty block (a sync-flush marker, 2^-34 per random byte) -- a fixed one.
// A false start would only cost a wasted lane (its slot is its own) ... and
// its rate here is below 1 in 10^12 per byte.
__device__ bool stored_ok(const GlobalBits& G, const LdsBits& Lb, uint32_t bias, uint32_t lim, uint32_t s,
                          uint32_t len, uint32_t pb, uint32_t L)
{
    const uint32_t q = pb + 4 + L;   // the next block's first byte
    if (q > len) return false;
    if (q == len) return true;
    const uint32_t lq = 8 * q + bias;   // the next header's LDS bit, when staged
    const bool staged = lq + 96 <= lim;
    const uint32_t h = staged ? Lb.peek(lq) : G.peek(8 * (s + q));
    const uint32_t type = (h >> 1) & 3u;
    // a dynamic header after it.  The quick filter passes ~1 in 4 000 random
    // offsets, which let about one false stored candidate per GiB of
    // near-random payload through (LEN / NLEN match 1 in 65 536 positions),
    // and a false candidate before a region's real one sizes the real
    // segment's slot short (the payload then falls back to the wave kernel).
    // An empty block (a sync marker, 00 00 FF FF: 1 in 2^32) keeps the quick
    // filter; any other length also passes the full header check.
    if (type == 2) {
        const bool quick = staged ? dyn_header_quick(Lb, lq, lim) : dyn_header_quick(G, 8 * (s + q), 8 * (s + len));
        return quick && (L == 0 || dyn_header_ok(G, 8 * (s + q), 8 * (s + len)));
    }
    if (type == 0) {
        if (q + 5 > len) return false;
        const uint32_t w = staged && lq + 8 + 32 <= lim ? Lb.peek(lq + 8) : G.peek(8 * (s + q + 1));
        return ((w & 0xffffu) ^ (w >> 16)) == 0xffffu;
    }
    // a fixed block after it: after an empty block, or (round 6) when its
    // first symbols read as a real fixed block does (fixed_block_ok): a Beast
    // peer's near-random payloads are runs of stored and fixed blocks
    if (type != 1) return false;
    if (L == 0) return true;
    if (!(BPMD_BP_FIXED & 1)) return false;
    return staged && lq + 3 + FW * 9 + 32 <= lim ? fixed_block_ok(Lb, lq, lim) : fixed_block_ok(G, 8 * (s + q), 8 * (s + len));
}

// the most compressed bytes from one of this library's markers (or a stored
// block, or the payload's start) to the next: a 4 KiB chunk's block (stored
// at worst: 4 096 + 5) plus the next marker
constexpr uint32_t MARK_SPAN = 4096 + 5 + 5 + 16;
#ifndef BPMD_BP_MARK_END
#define BPMD_BP_MARK_END 1   // 0: any marker marks the payload (round 5 until the ADVICE fix)
#endif
constexpr uint32_t LIST = 128;         // candidate offsets per wave and chunk
constexpr uint32_t CHUNK_STEPS = 4;    // 4 x 2048 bit offsets between deep-check rounds
constexpr uint32_t STORED_FLAG = 0x80000000u;

struct ScanLds {
    uint16_t kraft[4096];                       // kraft4 of every 12-bit field group
    uint32_t stage[SCAN_WAVES][STAGE_BYTES / 4 + 8];
    uint32_t list[SCAN_WAVES][LIST];
    uint32_t cnt[SCAN_WAVES];
};

// region -> long-list index, for the scan's per-region work items
__global__ void __launch_bounds__(256)
bp_region_map_kernel(const uint32_t* __restrict__ nlong, const uint32_t* __restrict__ regions,
                     const uint32_t* __restrict__ task_base, uint32_t* __restrict__ map)
{
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= *nlong) return;
    const uint32_t tb = task_base[i], nr = regions[i];
    for (uint32_t k = 0; k < nr; ++k) map[tb + k] = i;
}

// One wave per region (all regions of all long payloads in one index space,
// so a batch of few payloads still spreads over the chip).
// Two passes.  Pass 1 (DYN = false) searches every region for a stored
// block and marks the payload when it finds an empty one (a sync marker, as
// this library's deflater writes before every chunk of a long message);
// regions without a stored block are left KIND_PENDING.  Pass 2 (DYN = true)
// searches the pending regions for dynamic headers -- unless their payload
// has sync markers, whose chunk starts the stored search already found: a
// region without one lies inside a chunk, and its bit-offset search would
// only cost time (a missing candidate just lengthens the segment before it).
template <bool DYN>
__global__ void __launch_bounds__(64 * SCAN_WAVES)
bp_scan_kernel(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
               const uint32_t* __restrict__ in_len, const uint32_t* __restrict__ order,
               const uint32_t* __restrict__ region_map, const uint32_t* __restrict__ n_regions_dev,
               const Stat* __restrict__ stats, const uint32_t* __restrict__ task_base, SegTask* __restrict__ tasks,
               uint32_t* __restrict__ marked, uint32_t dyn_stride)
{
    __shared__ ScanLds L;
    const uint32_t n_regions = *n_regions_dev;
    for (uint32_t f = threadIdx.x; f < 4096; f += blockDim.x) L.kraft[f] = (uint16_t)kraft4(f);
    __syncthreads();
    const uint32_t lane = wave_lane(), wv = threadIdx.x >> 6;
    uint32_t* S = L.stage[wv];
    uint32_t* list = L.list[wv];
    uint32_t* cnt = &L.cnt[wv];
    // static grid stride: regions cost about the same, and one counter
    // taken per region serialises on its atomics (C5: 131 072 regions)
    const uint32_t waves = gridDim.x * SCAN_WAVES;
    // pass 2 screens 64 regions per step, one per lane (three dependent loads
    // per region, once per 64 instead of once per region: C4 8-way shard
    // 0.86 ms of screening), and runs the search on those still to do
    const uint32_t step = DYN ? 64u : 1u;
    for (uint32_t g0 = (blockIdx.x * SCAN_WAVES + wv) * step; g0 < n_regions; g0 += waves * step) {
    uint64_t todo = 1;
    if (DYN) {
        // only the regions pass 1 left pending, of unmarked payloads, and of
        // those every dyn_stride-th (a dynamic-header search costs a region's
        // whole bit-offset scan; BPMD_BP_SEGS sweep of Beast's payloads,
        // profiles/r05h_bp_segs_sweep.log)
        const uint32_t gl = g0 + lane;
        bool need = false;
        if (gl < n_regions && tasks[gl].kind == KIND_PENDING) {
            const uint32_t ri = region_map[gl];
            // (marked: bit 0 a sync marker, bit 1 a stored candidate within
            // MARK_SPAN + R of the payload's end -- a foreign encoder's payload
            // that flushed once near its start is searched; bit 2
            // a stored block with data, which turns on the fixed-block search)
            // The stride (BPMD_BP_DYN_STRIDE, else per payload): a payload with
            // stored data blocks (near-random data: a Beast peer's stored and
            // fixed runs, bit 2) is searched in one region per 4 KiB whatever
            // the region size, so a small batch's fine regions (R down to
            // R_MIN for an 8-way shard) do not multiply the search; the
            // other payloads in every region (C4's dynamic blocks of ~350
            // bytes need the candidates).  C5 8-way Beast shards L1 / L6 8.8 /
            // 16.0 -> 8.1 / 9.4 ms at stride 4 everywhere, while C4's rose
            // 16.1 -> 20.6 ms and the whole C5 batch (R = 4 KiB) fell 60 -> 48
            // GiB/s (profiles/r06w_stride_sweep.log)
            // (the last region, which also takes the payload's remainder, is
            // always searched)
            const uint32_t mk = marked[ri];
            const Stat sr = stats[ri];
            const uint32_t kr = gl - task_base[ri];
            const uint32_t ds = dyn_stride > 1 ? dyn_stride : (mk & 4u) && sr.R < 4096u ? 4096u / sr.R : 1u;
            // (a region the stride passes over still gets the fixed-block
            // search when the payload has it: that one is cheap)
            const bool fixed_only = kr % ds != 0 && kr + 1 != sr.regions;
            if (((mk & 3u) | (BPMD_BP_MARK_END ? 0u : 2u)) == 3u ||
                (fixed_only && !((BPMD_BP_FIXED & 2) && (mk & 4u)))) {
                tasks[gl].kind = KIND_NONE;
            } else {
                // a region inside the data of a stored block pass 1 found (one
                // of the 8 regions before it) holds no block start: no search
                // (this library's incompressible chunks go stored without a
                // marker; Beast's binary payloads are 35-60 % stored blocks)
                const uint32_t k = gl - task_base[ri], R = stats[ri].R;
                // the region's real end: the last region also takes the
                // payload's remainder (region_of), which may hold a block
                // start past the stored block's data
                const uint32_t rend = k + 1 == stats[ri].regions ? in_len[order[ri]] : (k + 1) * R;
                bool inside = false;
                for (uint32_t j = 1; j <= 8 && j <= k; ++j) {
                    const uint32_t kj = tasks[gl - j].kind;
                    const uint8_t* pm = in + in_off[order[ri]];
                    // (region 0 is the payload's start: a stored first block
                    // has its LEN field at byte 1)
                    if (kj == KIND_STORED || (j == k && ((pm[0] >> 1) & 3u) == 0)) {
                        const uint32_t pb = kj == KIND_STORED ? tasks[gl - j].bit >> 3 : 1u;
                        const uint32_t d0 = pb + 4, d1 = d0 + ((uint32_t)pm[pb] | (uint32_t)pm[pb + 1] << 8);
                        inside = d0 <= k * R && rend <= d1;
                        break;
                    }
                    if (kj != KIND_PENDING && kj != KIND_NONE) break;
                }
                if (inside) tasks[gl].kind = KIND_NONE;
                else need = true;
            }
        }
        todo = __ballot(need);
    }
    while (todo) {
        const uint32_t g = g0 + (uint32_t)__builtin_ctzll(todo);
        todo &= todo - 1;
        const uint32_t i = (uint32_t)__builtin_amdgcn_readfirstlane((int)region_map[g]);
        const uint32_t m = order[i];
        const Stat st = stats[i];
        const bool fixed_on = (BPMD_BP_FIXED & 2) && DYN && (marked[i] & 4u);   // pass 1's marks (an earlier launch)
        // the dynamic-header search only in every ds-th region of a payload
        // with stored data blocks (and its last); the others search fixed
        // starts only (the screening above)
        const uint32_t kq = g - task_base[i];
        const uint32_t dsq = dyn_stride > 1 ? dyn_stride : (marked[i] & 4u) && st.R < 4096u ? 4096u / st.R : 1u;
        const bool dyn_on = kq % dsq == 0 || kq + 1 == st.regions;
        const uint32_t len = in_len[m];
        const uint32_t tb = task_base[i];
        const uint8_t* p = in + in_off[m];
        const uint32_t s = (uint32_t)((uintptr_t)p & 3u);
        const uint32_t* A = (const uint32_t*)(p - s);
        const uint32_t E = (s + len + 3) >> 2;   // dwords holding payload bytes
        const GlobalBits G{A, E};
        {
            const uint32_t k = g - tb;
            uint32_t bit = 0, kind = KIND_START;
            // region 0's candidate is the payload's first bit, but pass 1 also
            // searches it for an empty stored block to mark the payload: a
            // short payload's only sync marker may lie there, and without the
            // mark pass 2 would run the bit-offset search on every later region
            // (C4 8-way shard: 1.06 ms)
            if (k || !DYN) {
                kind = KIND_NONE;
                BP_DIAG(const uint64_t t0 = __builtin_amdgcn_s_memtime());
                // stage payload bytes from the dword before the region's first
                // byte (so every offset has its previous byte) to STAGE_EXTRA
                // past its end, as dwords; bytes past the payload read as zeros
                const uint32_t q0 = ((s + k * st.R) >> 2) - 1;
                const uint32_t nwords = STAGE_BYTES / 4 + 8;
                const uint32_t tailm = ((s + len) & 3u) ? (1u << (8 * ((s + len) & 3u))) - 1u : ~0u;
                // only the words this region's size needs are loaded (the last
                // region also holds the payload's remainder, region_of: up to
                // 1.5 R, searched as far as the stage holds it)
                const uint32_t rlen = (k + 1 == st.regions ? len : (k + 1) * st.R) - k * st.R;
                const uint32_t nw = (rlen + STAGE_EXTRA + 64) / 4 < nwords ? (rlen + STAGE_EXTRA + 64) / 4 : nwords;
                {
                    // all loads in flight together (a load-store loop would
                    // wait out one memory latency per dword)
                    constexpr uint32_t U = (STAGE_BYTES / 4 + 8 + 63) / 64;
                    uint32_t v[U];
#pragma unroll
                    for (uint32_t u = 0; u < U; ++u) {
                        const uint32_t j = lane + 64u * u;
                        v[u] = j < nw && q0 + j < E ? A[q0 + j] : 0u;
                    }
                    // the words past the loaded ones (+ 2 for the peeks at
                    // the end) read as zeros; the rest of the stage is not
                    // touched (a 1 KiB region stages ~1.4 KiB, not 8.5)
#pragma unroll
                    for (uint32_t u = 0; u < U; ++u) {
                        const uint32_t j = lane + 64u * u;
                        if (j < nwords && j < nw + 8) S[j] = q0 + j == E - 1 ? v[u] & tailm : v[u];
                    }
                }
                if (lane == 0) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                __builtin_amdgcn_wave_barrier();
                asm volatile("" ::: "memory");
                // LDS bit of payload bit b: b + bias; payload bits end at lim
                // (and never past the staged words)
                const uint32_t bias = 8 * s - 32 * q0;
                const uint32_t lim0 = 8 * (s + len) - 32 * q0, slim = 32 * (nw - 2);
                const uint32_t lim = lim0 < slim ? lim0 : slim;
                const LdsBits Lb{S};
                BP_DIAG(__builtin_amdgcn_s_waitcnt(0); const uint64_t t1 = __builtin_amdgcn_s_memtime());
                const uint32_t b0 = 8 * k * st.R;                                     // region's first payload bit
                const uint32_t rs = 4 * nw - STAGE_EXTRA - 64 < rlen ? 4 * nw - STAGE_EXTRA - 64 : rlen;
                const uint32_t b1 = 8 * (k * st.R + rs) < 8 * len ? 8 * (k * st.R + rs) : 8 * len;   // past its last
                // 1. stored blocks, by their LEN / NLEN fields (a byte search
                // over the whole region; this library's deflater writes an
                // empty one before every chunk of a long message)
                uint32_t best = 0xffffffffu, best_len = 0;
                for (uint32_t base = b0; base < (DYN ? b0 : b1); base += 2048) {
                    const uint32_t first = base + 32 * lane;
                    const uint32_t lb = first + bias;
                    const uint32_t wp = peek32(S, lb - 8), w0 = peek32(S, lb), w1 = peek32(S, lb + 32);
                    uint32_t found = 0xffffffffu, flen = 0;
#pragma unroll
                    for (uint32_t j = 0; j < 4; ++j) {
                        const uint32_t x = __builtin_amdgcn_alignbit(w1, w0, 8 * j);
                        const uint32_t prevb = j ? (w0 >> (8 * (j - 1))) & 0xffu : wp & 0xffu;
                        const uint32_t pb = (first >> 3) + j;
                        const bool c = first + 8 * j < b1 && ((x & 0xffffu) ^ (x >> 16)) == 0xffffu &&
                                       (prevb & 0xc0u) == 0 && pb + 4 + (x & 0xffffu) <= len;
                        if (c && found == 0xffffffffu && stored_ok(G, Lb, bias, lim, s, len, pb, x & 0xffffu)) {
                            found = 8 * pb;
                            flen = x & 0xffffu;
                        }
                    }
                    const uint64_t fm = __ballot(found != 0xffffffffu);
                    if (fm) {
                        best = (uint32_t)__builtin_amdgcn_readlane((int)found, (int)__builtin_ctzll(fm));
                        best_len = (uint32_t)__builtin_amdgcn_readlane((int)flen, (int)__builtin_ctzll(fm));
                        break;
                    }
                }
                BP_DIAG(const uint64_t t2 = __builtin_amdgcn_s_memtime();
                        if (lane == 0) {
                            atomicAdd(&g_bp_diag[4], 1ull);
                            atomicAdd(&g_bp_diag[8], t1 - t0);
                            atomicAdd(&g_bp_diag[9], t2 - t1);
                        })
                // near the end: this library's deflater starts a block at least
                // every MARK_SPAN bytes, so its last regions hold a marker or a
                // stored block (or the payload is that short).  Two spans: a
                // last stored chunk is no candidate (Flush::sync's stripped
                // header follows it, not a whole block)
                const bool near_end = (k + 1) * st.R + st.R + 2 * MARK_SPAN >= len;
                if (k == 0) {
                    if (lane == 0) {
                        if (best != 0xffffffffu) atomicOr(&marked[i], best_len == 0 ? 1u : 4u);
                        if (len <= 2 * MARK_SPAN || (best != 0xffffffffu && near_end)) atomicOr(&marked[i], 2u);
                    }
                    kind = KIND_START;
                } else if (best != 0xffffffffu) {
                    bit = best;
                    kind = KIND_STORED;
                    if (lane == 0) atomicOr(&marked[i], (best_len == 0 ? 1u : 4u) | (near_end ? 2u : 0u));
                    BP_DIAG(if (lane == 0) atomicAdd(&g_bp_diag[5], 1ull));
                } else if (!DYN) {
                    kind = KIND_PENDING;
                } else {
                    BP_DIAG(if (lane == 0) atomicAdd(&g_bp_diag[6], 1ull));
                    // 2. dynamic headers: block type 2, HLIT / HDIST in range
                    // and a complete code-length code (Kraft sum, table), in
                    // chunks; then the full check, one candidate per lane
                    for (uint32_t cb = b0; cb < b1 && best == 0xffffffffu; cb += 2048 * CHUNK_STEPS) {
                        for (uint32_t base = cb; base < cb + 2048 * CHUNK_STEPS && base < b1; base += 2048) {
                            const uint32_t first = base + 32 * lane;
                            const uint32_t lb = first + bias;
                            const uint32_t w0 = peek32(S, lb), w1 = peek32(S, lb + 32), w2 = peek32(S, lb + 64),
                                           w3 = peek32(S, lb + 96);
                            const uint64_t lo = ((uint64_t)w1 << 32) | w0;
                            // BFINAL 0, BTYPE 2 (a final block is left to the
                            // segment before it: halves the offsets to check)
                            uint64_t mk = ~lo & ~(lo >> 1) & (lo >> 2);
                            mk &= ~((lo >> 4) & (lo >> 5) & (lo >> 6) & (lo >> 7));
                            mk &= ~((lo >> 9) & (lo >> 10) & (lo >> 11) & (lo >> 12));
                            uint32_t cand = dyn_on ? (uint32_t)mk : 0u;
                            if (first >= b1) cand = 0;
                            else if (b1 - first < 32) cand &= (1u << (b1 - first)) - 1u;
                            // fixed-block starts after a fixed block (round 6): seven zero
                            // bits (its end-of-block code), BFINAL 0, BTYPE 1 -- the bits
                            // o - 7 .. o + 2 around offset o read 0000000 0 1 0.  Only in
                            // payloads with a stored block of data (a Beast peer's
                            // near-random runs): in a dynamic-coded text stream ~1 in 2 000
                            // bits shows the pattern and ~0.6 % of those pass
                            // fixed_block_ok, about one false start per 40 KiB payload
                            // (each one sends the payload to the wave kernel)
                            if (fixed_on) {
                                const uint32_t wm = peek32(S, lb - 8);   // bits first - 8 ..
                                const uint64_t x = ((uint64_t)w0 << 8 | (wm & 0xffu)) | ((uint64_t)w1 << 40);
                                const uint64_t y = ~x;
                                const uint64_t t1 = y & (y >> 1), t2 = t1 & (t1 >> 2), t3 = t2 & (t2 >> 4);   // 8 zeros
                                uint32_t fm = (uint32_t)((t3 >> 1) & (x >> 9) & (y >> 10));
                                if (first >= b1) fm = 0;
                                else if (b1 - first < 32) fm &= (1u << (b1 - first)) - 1u;
                                if (first < 8) fm &= ~0u << (8 - first);   // the zero bits lie in the payload
                                while (fm) {
                                    const uint32_t o = (uint32_t)__builtin_ctz(fm);
                                    fm &= fm - 1;
                                    const uint32_t at = atomicAdd(cnt, 1u);
                                    if (at < LIST) list[at] = 0x80000000u | (first + o);
                                }
                            }
                            while (cand) {
                                const uint32_t o = (uint32_t)__builtin_ctz(cand);
                                cand &= cand - 1;
                                const uint32_t ncode = ((uint32_t)(lo >> (o + 13)) & 15u) + 4;
                                const uint32_t sh = o + 17;   // 17..48: the 57 field bits from w0..w3
                                uint32_t x0, x1;
                                if (sh < 32) {
                                    x0 = __builtin_amdgcn_alignbit(w1, w0, sh);
                                    x1 = __builtin_amdgcn_alignbit(w2, w1, sh);
                                } else {
                                    x0 = __builtin_amdgcn_alignbit(w2, w1, sh - 32);
                                    x1 = __builtin_amdgcn_alignbit(w3, w2, sh - 32);
                                }
                                uint64_t x = ((uint64_t)x1 << 32) | x0;
                                x &= (1ull << (3 * ncode)) - 1ull;
                                const uint32_t kr = L.kraft[x & 0xfff] + L.kraft[(x >> 12) & 0xfff] +
                                                    L.kraft[(x >> 24) & 0xfff] + L.kraft[(x >> 36) & 0xfff] +
                                                    L.kraft[(x >> 48) & 0x1ff];
                                if (kr == 128) {
                                    const uint32_t at = atomicAdd(cnt, 1u);
                                    if (at < LIST) list[at] = first + o;
                                }
                            }
                        }
                        __builtin_amdgcn_wave_barrier();
                        asm volatile("" ::: "memory");
                        const uint32_t c0 = __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        const uint32_t nc = c0 < LIST ? c0 : LIST;
                        BP_DIAG(if (lane == 0) atomicAdd(&g_bp_diag[7], (unsigned long long)nc));
                        asm volatile("" ::: "memory");
                        if (lane == 0) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        asm volatile("" ::: "memory");
                        for (uint32_t j0 = 0; j0 < nc; j0 += 64) {
                            // (candidate bit << 1 | 1 for a fixed block: the min is the
                            // first candidate, payload bits < 2^31)
                            uint32_t ok = 0xffffffffu;
                            if (j0 + lane < nc) {
                                const uint32_t e = list[j0 + lane], b = e & 0x7fffffffu;
                                bool good;
                                if (e >> 31) {
                                    good = fixed_block_ok(Lb, b + bias, lim);
                                    if (good) {
                                        // (from the stage when it holds bit `from`; the stage's
                                        // first bit is payload bit -bias)
                                        const uint32_t from = b > FBACK ? b - FBACK : 0u;
                                        good = (int32_t)(from + bias) >= 0
                                                   ? fixed_eob_at(Lb, from + bias, b + bias - 7u)
                                                   : fixed_eob_at(G, 8 * s + from, 8 * s + b - 7u);
                                    }
                                } else {
                                    good = dyn_header_ok(Lb, b + bias, lim);
                                }
                                if (good) ok = (b << 1) | (e >> 31);
                            }
                            for (uint32_t d = 32; d >= 1; d >>= 1) {
                                const uint32_t y = __shfl_xor(ok, d);
                                ok = y < ok ? y : ok;
                            }
                            best = ok < best ? ok : best;
                        }
                        __builtin_amdgcn_wave_barrier();
                    }
                    if (best != 0xffffffffu) {
                        bit = best >> 1;
                        kind = (best & 1u) ? KIND_FIXED : KIND_DYN;
                    }
                    BP_DIAG(if (lane == 0) atomicAdd(&g_bp_diag[10], __builtin_amdgcn_s_memtime() - t2));
                }
                __builtin_amdgcn_wave_barrier();
            }
            if (lane == 0) {
                SegTask t;
                t.msg = m;
                t.bit = bit;
                t.kind = kind;
                t.left = st.regions - 1 - k;
                t.sym_off = 0;
                t.sym_cap = 0;
                t.pad = 0;
                tasks[tb + k] = t;
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
    }
}

// ------------------------------------------------------------------- skim
// A Beast peer's long payloads carry no sync markers: tr_flush_block cuts a
// block every lit_bufsize - 1 symbols and picks stored, fixed or dynamic by
// size (deflate_stream.ipp:1406, :1425-1518), and near-random data gives
// runs of stored and FIXED blocks.  A fixed block's header is three bits
// that any bit offset can look like, so no scan finds it, and a run of them
// was one serial segment.  The skim starts one lane at every candidate pass
// 1 found (a stored block, or the payload's first bit) and walks the blocks
// after it: a stored block by its LEN field, a fixed block symbol by symbol
// with the fixed code (inflate_stream.ipp:865-930; no tables, no output),
// until a dynamic block, the next candidate, a final block or an error.
// Every block start it passes becomes its region's candidate when the region
// has none (a dynamic block's start too), and the regions it crossed without
// a block start are settled as candidate-free, so pass 2 searches only the
// regions no walk reached.  A walk that meets anything unexpected simply
// stops: candidates only ever cut the serial decode, which checks
// everything again (bit-exact results do not depend on the skim).
struct SkimBits {
    const uint32_t* A;   // the payload's aligned base
    uint32_t E;          // dwords holding payload bytes
    uint32_t sbits;      // 8 x the payload's offset in A[0]
    __device__ __forceinline__ uint32_t word(uint32_t w) const { return w < E ? A[w] : 0u; }
};

// the region of payload byte `byte` (bp_stats_kernel: na regions of R bytes,
// the last one taking the rest)
__device__ __forceinline__ uint32_t region_of(uint32_t byte, uint32_t R, uint32_t na)
{
    const uint32_t k = byte / R;
    return k < na ? k : na - 1;
}

__global__ void __launch_bounds__(256)
bp_skim_kernel(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
               const uint32_t* __restrict__ in_len, const uint32_t* __restrict__ order,
               const uint32_t* __restrict__ region_map, const uint32_t* __restrict__ n_regions_dev,
               const Stat* __restrict__ stats, const uint32_t* __restrict__ task_base, SegTask* __restrict__ tasks,
               const uint32_t* __restrict__ marked)
{
    const uint32_t n_regions = *n_regions_dev;
    for (uint32_t g = blockIdx.x * 256u + threadIdx.x; g < n_regions; g += gridDim.x * 256u) {
    const SegTask t0 = tasks[g];
    if (t0.kind != KIND_START && t0.kind != KIND_STORED) continue;
    const uint32_t i = region_map[g];
    if ((marked[i] & 3u) == 3u) continue;   // sync markers: pass 1 found the chunk starts
    const Stat st = stats[i];
    const uint32_t tb = task_base[i];
    const uint32_t k0 = g - tb;
    const uint32_t m = order[i];
    const uint32_t len = in_len[m];
    const uint8_t* p = in + in_off[m];
    const uint32_t s = (uint32_t)((uintptr_t)p & 3u);
    SkimBits B{(const uint32_t*)(p - s), (s + len + 3) >> 2, 8 * s};
    // the next candidate pass 1 found (stored: its LEN field's bit)
    uint32_t next_bit = 8 * len;
    for (uint32_t k = k0 + 1; k < st.regions; ++k) {
        const uint32_t kd = tasks[tb + k].kind;
        if (kd == KIND_STORED) {
            next_bit = tasks[tb + k].bit;
            break;
        }
    }
    const uint32_t end_bits = 8 * len;
    // bit reader: 64 bits at `pos` from the dwords at w0 (+ the next one)
    uint32_t pos;
    bool stored_now;
    if (t0.kind == KIND_STORED) {
        pos = t0.bit;   // the LEN field
        stored_now = true;
    } else {
        pos = 0;
        stored_now = false;
    }
    uint32_t last_k = k0;   // the region of the last block start recorded (or the walk's own)
    auto settle = [&](uint32_t kto) {   // regions after last_k up to kto (exclusive): no block start
        for (uint32_t k = last_k + 1; k < kto && k < st.regions; ++k)
            if (tasks[tb + k].kind == KIND_PENDING) tasks[tb + k].kind = KIND_NONE;
    };
    auto record = [&](uint32_t bit, uint32_t kind) {
        const uint32_t k = region_of(bit >> 3, st.R, st.regions);
        if (k <= last_k) return;   // a region that has its start already
        settle(k);
        SegTask& t = tasks[tb + k];
        if (t.kind == KIND_PENDING || t.kind == KIND_NONE) {
            t.bit = bit;
            t.kind = kind;
        }
        last_k = k;
    };
    // bit reader: bb holds nb bits; refills take dwords from the 16-byte
    // block q; the next three blocks are already loading (a fixed block of
    // near-random bytes uses a block every ~14 symbols, and one block ahead
    // left the walk waiting on memory at every block)
    uint4 q = make_uint4(0, 0, 0, 0), n1 = q, n2 = q, n3 = q;
    uint32_t qi = 0, bi = 0;   // dword index in q; block index of n3
    uint64_t bb = 0;
    uint32_t nb = 0;
    auto load_block = [&](uint32_t b) -> uint4 {   // 16-byte block b of A, zeros past the payload
        return 16 * b < 4 * B.E ? *(const uint4*)(B.A + 4 * b) : make_uint4(0, 0, 0, 0);
    };
    auto reset = [&](uint32_t at) {   // position the reader at payload bit `at`
        const uint32_t qb = B.sbits + at;
        const uint32_t blk = qb >> 7;
        q = load_block(blk);
        n1 = load_block(blk + 1);
        n2 = load_block(blk + 2);
        n3 = load_block(blk + 3);
        bi = blk + 3;
        qi = (qb >> 5) & 3u;
        const uint32_t d = qi == 0 ? q.x : qi == 1 ? q.y : qi == 2 ? q.z : q.w;
        bb = (uint64_t)(d >> (qb & 31u));
        nb = 32 - (qb & 31u);
        ++qi;
        pos = at;
    };
    auto fill = [&]() {
        if (nb <= 32) {
            if (qi == 4) {
                q = n1;
                n1 = n2;
                n2 = n3;
                n3 = load_block(++bi);
                qi = 0;
            }
            const uint32_t d = qi == 0 ? q.x : qi == 1 ? q.y : qi == 2 ? q.z : q.w;
            bb |= (uint64_t)d << nb;
            nb += 32;
            ++qi;
        }
    };
    auto take = [&](uint32_t n) {   // n <= 32 bits, after fill()
        const uint32_t v = (uint32_t)bb & (n >= 32 ? ~0u : ((1u << n) - 1u));
        bb >>= n;
        nb -= n;
        pos += n;
        return v;
    };
    reset(pos);
    for (uint32_t guard = 0; guard < 4096; ++guard) {
        if (stored_now) {
            // LEN NLEN at `pos` (byte aligned), then the bytes
            if (pos + 32 > end_bits) break;
            fill();
            const uint32_t v = take(32);
            const uint32_t L = v & 0xffffu;
            if (L != ((v >> 16) ^ 0xffffu)) break;
            const uint32_t nxt = pos + 8 * L;
            if (nxt >= end_bits) break;
            reset(nxt);
            stored_now = false;
        }
        // a block header at pos
        if (pos >= next_bit || pos + 3 > end_bits) break;
        fill();
        const uint32_t h = take(3);
        if (h & 1) break;   // a final block: nothing after it
        const uint32_t type = h >> 1;
        if (type == 0) {
            const uint32_t lb = (pos + 7) & ~7u;   // the LEN field
            if (lb >= next_bit) break;             // the next candidate's block: its walk
            record(lb, KIND_STORED);
            reset(lb);
            stored_now = true;
            continue;
        }
        if (type != 1) {   // dynamic (or invalid): a candidate, and the walk ends
            if (type == 2) record(pos - 3, KIND_DYN);
            break;
        }
        record(pos - 3, KIND_FIXED);
        // the fixed block's symbols up to its end-of-block
        bool ok = false;
        for (uint32_t n = 0; n < 65536; ++n) {
            fill();
            if (pos + 7 > end_bits) break;
            const uint32_t c9 = __builtin_bitreverse32((uint32_t)bb) >> 23;   // the next 9 code bits, first bit high
            uint32_t L, sym;
            if ((c9 >> 2) < 24) {
                L = 7;
                sym = 256 + (c9 >> 2);
            } else if ((c9 >> 1) < 192) {
                L = 8;
                sym = (c9 >> 1) - 48;
            } else if ((c9 >> 1) < 200) {
                L = 8;
                sym = 280 + (c9 >> 1) - 192;
            } else {
                L = 9;
                sym = 144 + c9 - 400;
            }
            take(L);
            if (sym == 256) {
                ok = true;
                break;
            }
            if (sym < 256) continue;
            if (sym > 285) break;   // invalid literal/length code
            const uint32_t li = sym - 257;
            const uint32_t xl = (li < 8 || li == 28) ? 0u : ((li - 4) >> 2);
            fill();
            take(xl);
            const uint32_t dsym = __builtin_bitreverse32((uint32_t)bb) >> 27;
            take(5);
            if (dsym >= 30) break;   // invalid distance code
            const uint32_t xd = dsym < 4 ? 0u : (dsym >> 1) - 1;
            fill();
            take(xd);
        }
        if (!ok || pos > end_bits) break;
    }
    // the regions the walk crossed up to where it stopped hold no other start
    settle(region_of((pos < end_bits ? pos : end_bits - 1) >> 3, st.R, st.regions));
    }
}

// Slots, one wave per long payload once every region is scanned: each
// candidate's span runs to the next candidate (or the end of the payload);
// slot = span x F16 + SLACK symbols, laid out in order.
__global__ void __launch_bounds__(256)
bp_slots_kernel(const uint32_t* __restrict__ in_len, const uint32_t* __restrict__ order,
                const uint32_t* __restrict__ nlong, const Stat* __restrict__ stats,
                const uint32_t* __restrict__ task_base, const unsigned long long* __restrict__ word_base,
                SegTask* __restrict__ tasks)
{
    const uint32_t lane = wave_lane();
    const uint32_t end = *nlong;
    for (uint32_t i = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; i < end; i += (gridDim.x * blockDim.x) >> 6) {
        const Stat st = stats[i];
        const uint32_t len = in_len[order[i]];
        const uint32_t tb = task_base[i];
        uint64_t run = word_base[i] + SYM_GUARD;
        // A slot reaches to the third candidate after it: a false candidate
        // (a random LEN / NLEN whose LEN happens to land on a real block
        // start, ~1 per GiB of binary payload; a fixed-block start the checks
        // let through) that precedes a region's real one must not size the
        // real segment's slot to its own short span.  (Round 5 reached to the
        // second: one 8-way C5 shard of Beast payloads in two then sent one
        // payload to the wave kernel, +4 to +7 ms, profiles/r06g_shard_fallbacks.log.)
        uint32_t n1 = 8 * len, n2 = 8 * len, n3 = 8 * len;   // the three next candidates' bits, from the chunks after
        const uint32_t nch = (st.regions + 63) / 64;
        // (a1, a2, a3) <- the three smallest of (a1, a2, a3) and (b1, b2, b3), ascending
        auto three_min = [](uint32_t& a1, uint32_t& a2, uint32_t& a3, uint32_t b1, uint32_t b2, uint32_t b3) {
            auto ins = [&](uint32_t v) {
                if (v < a3) a3 = v;
                if (a3 < a2) { const uint32_t t = a2; a2 = a3; a3 = t; }
                if (a2 < a1) { const uint32_t t = a1; a1 = a2; a2 = t; }
            };
            ins(b1);
            ins(b2);
            ins(b3);
        };
        // chunks from the last to the first (suffix scans of the three smallest
        // candidate bits), slot offsets assigned afterwards from the first
        SegTask* vt = tasks + tb;
        for (uint32_t c = nch; c-- > 0;) {
            const uint32_t k = c * 64 + lane;
            const bool v = k < st.regions && vt[k].kind != KIND_NONE;
            const uint32_t b = v ? vt[k].bit : 0xffffffffu;
            uint32_t s1 = b, s2 = 0xffffffffu, s3 = 0xffffffffu;   // inclusive suffix: the three smallest from k on
            for (uint32_t d = 1; d < 64; d <<= 1) {
                const uint32_t y1 = __shfl_down(s1, d), y2 = __shfl_down(s2, d), y3 = __shfl_down(s3, d);
                if (lane + d < 64) three_min(s1, s2, s3, y1, y2, y3);
            }
            // the three candidates after k: lane k + 1's suffix, then the chunks after
            uint32_t a1 = __shfl_down(s1, 1), a2 = __shfl_down(s2, 1), a3 = __shfl_down(s3, 1);
            if (lane == 63) a1 = a2 = a3 = 0xffffffffu;
            three_min(a1, a2, a3, n1, n2, n3);
            if (v) {
                const uint32_t after = a3 < 8 * len ? a3 : 8 * len;
                const uint32_t span = after > b ? (after - b + 7) >> 3 : 1u;
                vt[k].sym_cap = (uint32_t)(((uint64_t)span * st.F16) >> 16) + SLACK;
            }
            uint32_t c1 = __shfl(s1, 0), c2 = __shfl(s2, 0), c3 = __shfl(s3, 0);
            three_min(c1, c2, c3, n1, n2, n3);
            n1 = c1;
            n2 = c2;
            n3 = c3;
        }
        __builtin_amdgcn_s_waitcnt(0);
        __builtin_amdgcn_wave_barrier();
        for (uint32_t c = 0; c < nch; ++c) {
            const uint32_t k = c * 64 + lane;
            const bool v = k < st.regions && vt[k].kind != KIND_NONE;
            const uint32_t cap = v ? vt[k].sym_cap : 0u;
            uint32_t incl = cap;
            for (uint32_t d = 1; d < 64; d <<= 1) {
                const uint32_t y = __shfl_up(incl, d);
                incl += lane >= d ? y : 0u;
            }
            if (v) vt[k].sym_off = run + incl - cap;
            run += __shfl(incl, 63);
        }
        __builtin_amdgcn_s_waitcnt(0);
        __builtin_amdgcn_wave_barrier();
    }
}

// ---------------------------------------------------------------- resolve
typedef uint32_t uint32_ua __attribute__((aligned(1)));
typedef uint4 uint4_ua __attribute__((aligned(1)));


typedef uint2 uint2_sa __attribute__((aligned(2)));
// symbols per lane per step of the serial resolve (a step is one dependent
// round trip -- symbols, then the bytes references read).  32 measured the
// same as 16 on 8-way C4 / C5 shards (8.63 vs 8.65 ms, 2.41 vs 2.40 ms); a
// build with 64 did not finish its first C4 shard call within 180 s and was
// not pursued (profiles/r05n_resolve_width.log)
#ifndef BPMD_BP_RSYM
#define BPMD_BP_RSYM 16
#endif
constexpr uint32_t RSYM = BPMD_BP_RSYM;

__global__ void __launch_bounds__(256)
bp_resolve_kernel(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                  const uint32_t* __restrict__ order, const uint32_t* __restrict__ nlong,
                  const uint32_t* __restrict__ task_base, const SegTask* __restrict__ tasks,
                  const SegRes* __restrict__ res, const uint16_t* __restrict__ sym, uint8_t* __restrict__ out,
                  const uint64_t* __restrict__ out_off, const uint32_t* __restrict__ out_cap,
                  uint32_t* __restrict__ out_len, int32_t* __restrict__ status, uint32_t raw,
                  uint32_t* __restrict__ fb_list, uint32_t* __restrict__ fb_count, uint32_t* __restrict__ qctr,
                  const Stat* __restrict__ stats)
{
    const uint32_t lane = wave_lane();
    const uint32_t end = *nlong;
    const int32_t full_status = raw ? ST_OK : ST_NEED_BUFFERS;
    for (;;) {
        uint32_t i = 0;
        if (lane == 0) i = atomicAdd(qctr, 1u);
        i = (uint32_t)__builtin_amdgcn_readfirstlane((int)i);
        if (i >= end) break;
        const uint32_t m = order[i];
        const uint32_t cap = out_cap[m];
        uint8_t* o = out + out_off[m];
        uint32_t t = task_base[i];
        uint32_t P = 0;
        int32_t stv = ST_OK;
        uint32_t olen = 0;
        bool fallback = stats[i].regions == 0;
        uint32_t nseg = 0;
        while (!fallback) {
            ++nseg;
            const SegRes r = res[t];
            if (r.status == SEG_DIRECT && r.next > t && r.next != 0xffffffffu) {
                // a stored block: its bytes from the payload, 16 per lane per step
                const uint32_t n = r.nsym, room = cap - P;
                const uint32_t c = n < room ? n : room;
                const uint8_t* src = in + in_off[m] + (tasks[t].bit >> 3) + 4;
                uint8_t* dst = o + P;
                uint32_t j = 16 * lane;
                for (; j + 16 <= c; j += 1024) *(uint4_ua*)(dst + j) = *(const uint4_ua*)(src + j);
                for (; j < c; ++j) dst[j] = src[j];   // the last partial 16 bytes (one lane)
                if (n > room) {
                    stv = full_status;
                    olen = cap;
                    break;
                }
                P += n;
                __builtin_amdgcn_s_waitcnt(0);
                t = r.next;
                continue;
            }
            const uint16_t* sy = sym + tasks[t].sym_off;
            const uint32_t n = r.nsym;
            const uint32_t room = cap - P;   // P <= cap
            uint32_t bad = n;                // first symbol referring before the payload
            // RSYM symbols per lane per step, all loads in flight together
            for (uint32_t c = 0; c < n; c += 64 * RSYM) {
                const uint32_t j0 = c + RSYM * lane;
                uint32_t v[RSYM];
                if (j0 + RSYM <= n) {
#pragma unroll
                    for (int h = 0; h < (int)RSYM / 4; ++h) {
                        const uint2 w = *(const uint2_sa*)(sy + j0 + 4 * h);
                        v[4 * h] = w.x & 0xffffu; v[4 * h + 1] = w.x >> 16;
                        v[4 * h + 2] = w.y & 0xffffu; v[4 * h + 3] = w.y >> 16;
                    }
                } else {
#pragma unroll
                    for (int q = 0; q < (int)RSYM; ++q) v[q] = j0 + q < n ? sy[j0 + q] : 0u;
                }
                uint32_t lbad = 0xffffffffu;
                uint32_t bytes[RSYM];
#pragma unroll
                for (int q = 0; q < (int)RSYM; ++q) {
                    const uint32_t x = v[q];
                    bytes[q] = x & 0xffu;
                    if (j0 + q < n && (x & SYM_REF)) {
                        const uint32_t back = (x & 0x7fffu) + 1;   // bytes before the segment's start
                        if (back > P) {
                            lbad = lbad == 0xffffffffu ? j0 + q : lbad;
                        } else {
                            bytes[q] = o[P - back];
                        }
                    }
                }
                // the first invalid reference of the step (in stream order)
                uint32_t mb = lbad;
                for (uint32_t d = 32; d >= 1; d >>= 1) {
                    const uint32_t y = __shfl_xor(mb, d);
                    mb = y < mb ? y : mb;
                }
                const uint32_t upto = (mb < n ? mb : n) < room ? (mb < n ? mb : n) : room;
                if (j0 + RSYM <= upto) {
                    uint32_t d4[RSYM / 4];
#pragma unroll
                    for (int h = 0; h < (int)RSYM / 4; ++h)
                        d4[h] = bytes[4 * h] | (bytes[4 * h + 1] << 8) | (bytes[4 * h + 2] << 16) | (bytes[4 * h + 3] << 24);
                    #pragma unroll
                    for (int h = 0; h < (int)RSYM / 16; ++h)
                        *(uint4_ua*)(o + P + j0 + 16 * h) = make_uint4(d4[4 * h], d4[4 * h + 1], d4[4 * h + 2], d4[4 * h + 3]);
                } else {
#pragma unroll
                    for (int q = 0; q < (int)RSYM; ++q)
                        if (j0 + q < upto) o[P + j0 + q] = (uint8_t)bytes[q];
                }
                if (mb != 0xffffffffu) {
                    bad = mb;
                    break;
                }
                if (c + 64 * RSYM > room) break;   // the rest lies past the capacity
            }
            if (bad < n) {
                // the token at P + bad has a distance past the output so far
                // (the rule is checked before the capacity, except in raw mode
                // where output at or past the capacity stops first)
                const uint32_t X = P + bad;
                if (raw ? X < cap : X <= cap) {
                    stv = ST_INVALID_DISTANCE;
                    olen = X;
                } else {
                    stv = full_status;
                    olen = cap;
                }
                break;
            }
            if (n > room) {
                stv = full_status;
                olen = cap;
                break;
            }
            P += n;
            // the segment's bytes are out before the next segment refers to them
            __builtin_amdgcn_s_waitcnt(0);
            if (r.status == SEG_HANDOFF && r.next > t && r.next != 0xffffffffu) {
                t = r.next;
                continue;
            }
            if (r.status == SEG_FULL || r.status == SEG_SKIP || r.status == SEG_HANDOFF || r.status == SEG_DIRECT) {
                fallback = true;
                if (lane == 0) {
                    g_bp_fb[0] = m;
                    g_bp_fb[1] = t - task_base[i];
                    g_bp_fb[2] = (uint32_t)r.status;
                    g_bp_fb[3] = r.nsym;
                    g_bp_fb[4] = tasks[t].sym_cap;
                    g_bp_fb[5] = r.next;
                    g_bp_fb[6] = tasks[t].bit;
                    g_bp_fb[7] = tasks[t].kind;
                }
                break;
            }
            stv = r.status;
            olen = P;
            break;
        }
        if (lane == 0) {
            atomicAdd(&g_bp_diag[0], 1ull);
            atomicAdd(&g_bp_diag[1], (unsigned long long)nseg);
            if (fallback) atomicAdd(&g_bp_diag[2], 1ull);
            if (fallback) {
                fb_list[atomicAdd(fb_count, 1u)] = m;
            } else {
                out_len[m] = olen;
                status[m] = stv;
            }
        }
    }
}

// ------------------------------------------------- segment-parallel resolve
// Round 4's resolve walked each payload's segments in order on one wave,
// because a reference reads bytes the earlier segments write: a 64 KiB
// payload was 64 dependent steps, and the longest payloads set the kernel's
// end.  Now two kernels, the phase boundary between them a kernel boundary
// (no workgroup ever waits for another):
//   bp_chain_kernel   one lane per payload walks the chain of segment
//                     results only (no symbols): each on-chain segment's
//                     output start and slot, the capacity cut, the status,
//                     the fallbacks;
//   bp_resolve2_kernel one workgroup per payload (a queue over payloads)
//                     resolves all its segments at once: a reference is
//                     followed into the SYMBOLS of the segment that holds its
//                     target (found by a binary search over the chain's
//                     output starts in LDS) and on, while the target is itself
//                     a reference -- symbols never change after decoding, so
//                     no order between segments is needed.  The first
//                     reference before the payload's start (the reference's
//                     invalid_distance, inflate_stream.ipp:475-514) is found
//                     in a first pass, so no byte at or past it is written.
struct PayRes {
    uint32_t nseg;     // segments on the chain up to the terminating one
    uint32_t olen;     // output length by the chain alone (capacity / status)
    int32_t status;    // status by the chain alone
    uint32_t flags;    // 1 fallback (wave kernel), 2 capacity cut
};
static_assert(sizeof(PayRes) == 16, "PayRes layout");

__global__ void __launch_bounds__(256)
bp_chain_kernel(const uint32_t* __restrict__ order, const uint32_t* __restrict__ nlong,
                const uint32_t* __restrict__ task_base, const SegTask* __restrict__ tasks,
                const SegRes* __restrict__ res, const uint32_t* __restrict__ out_cap, uint32_t raw,
                const Stat* __restrict__ stats, uint32_t* __restrict__ chp, uint64_t* __restrict__ chs,
                PayRes* __restrict__ pay, uint32_t* __restrict__ out_len, int32_t* __restrict__ status,
                uint32_t* __restrict__ fb_list, uint32_t* __restrict__ fb_count)
{
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= *nlong) return;
    const uint32_t m = order[i];
    const uint32_t cap = out_cap[m];
    const uint32_t tb = task_base[i];
    const int32_t full_status = raw ? ST_OK : ST_NEED_BUFFERS;
    PayRes pr = {0, 0, ST_OK, 0};
    if (stats[i].regions == 0) {
        pr.flags = 1;
    } else {
        uint32_t t = tb, P = 0, k = 0;
        for (;;) {
            const SegRes r = res[t];
            if (r.status == SEG_DIRECT) {   // (no symbols: this form sends the payload to the wave kernel)
                pr.flags = 1;
                break;
            }
            chp[tb + k] = P;
            chs[tb + k] = tasks[t].sym_off;
            ++k;
            if (r.nsym > cap - P) {   // the capacity cuts this segment
                pr.status = full_status;
                pr.olen = cap;
                pr.flags = 2;
                break;
            }
            P += r.nsym;
            if (r.status == SEG_HANDOFF && r.next > t && r.next != 0xffffffffu) {
                t = r.next;
                continue;
            }
            if (r.status == SEG_FULL || r.status == SEG_SKIP || r.status == SEG_HANDOFF) {
                pr.flags = 1;
                {
                    g_bp_fb[0] = m;
                    g_bp_fb[1] = t - tb;
                    g_bp_fb[2] = (uint32_t)r.status;
                    g_bp_fb[3] = r.nsym;
                    g_bp_fb[4] = tasks[t].sym_cap;
                    g_bp_fb[5] = r.next;
                    g_bp_fb[6] = tasks[t].bit;
                    g_bp_fb[7] = tasks[t].kind;
                }
                break;
            }
            pr.status = r.status;
            pr.olen = P;
            break;
        }
        pr.nseg = k;
        atomicAdd(&g_bp_diag[1], (unsigned long long)k);
    }
    atomicAdd(&g_bp_diag[0], 1ull);
    if (pr.flags & 1) {
        atomicAdd(&g_bp_diag[2], 1ull);
        fb_list[atomicAdd(fb_count, 1u)] = m;
    }
    pay[i] = pr;
    (void)out_len;
    (void)status;
}

constexpr uint32_t RES_THREADS = 256;
constexpr uint32_t RES_LDS_SEGS = 1024;   // chains up to this length resolve from LDS
constexpr uint32_t RES_HOPS = 32;         // references followed per byte in pass 2

// the chain segment holding output position q (chp ascending, chp[0] = 0)
__device__ __forceinline__ uint32_t seg_of(const uint32_t* __restrict__ P, uint32_t K, uint32_t q)
{
    uint32_t lo = 0, hi = K - 1;   // largest k with P[k] <= q
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (P[mid] <= q) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

__global__ void __launch_bounds__(RES_THREADS)
bp_resolve2_kernel(const uint32_t* __restrict__ order, const uint32_t* __restrict__ nlong,
                   const uint32_t* __restrict__ task_base, const uint16_t* __restrict__ sym,
                   uint8_t* __restrict__ out, const uint64_t* __restrict__ out_off,
                   const uint32_t* __restrict__ out_cap, uint32_t* __restrict__ out_len,
                   int32_t* __restrict__ status, uint32_t raw, const uint32_t* __restrict__ chp,
                   const uint64_t* __restrict__ chs, const PayRes* __restrict__ pay, uint32_t* __restrict__ qctr)
{
    __shared__ uint32_t sP[RES_LDS_SEGS];
    __shared__ uint64_t sS[RES_LDS_SEGS];
    __shared__ uint32_t s_i, s_bad, s_deep;
    const uint32_t tid = threadIdx.x;
    const uint32_t end = *nlong;
    for (;;) {
        if (tid == 0) s_i = atomicAdd(qctr, 1u);
        __syncthreads();
        const uint32_t i = s_i;
        if (i >= end) break;
        const PayRes pr = pay[i];
        if (pr.flags & 1) {   // the wave kernel decodes it (bp_chain_kernel listed it)
            __syncthreads();
            continue;
        }
        const uint32_t m = order[i];
        const uint32_t cap = out_cap[m];
        uint8_t* o = out + out_off[m];
        const uint32_t tb = task_base[i];
        const uint32_t K = pr.nseg;
        const bool lds = K <= RES_LDS_SEGS;
        for (uint32_t k = tid; k < K && lds; k += RES_THREADS) {
            sP[k] = chp[tb + k];
            sS[k] = chs[tb + k];
        }
        if (tid == 0) {
            s_bad = 0xffffffffu;
            s_deep = 0;
        }
        __syncthreads();
        const uint32_t* P = lds ? sP : chp + tb;
        const uint64_t* S = lds ? sS : chs + tb;
        // positions whose references count: the output, plus (pmd mode) the
        // token at the capacity when the capacity cut the chain -- a bad
        // distance there is the reference's error, not need_buffers
        const uint32_t lim = pr.olen + ((pr.flags & 2) && !raw ? 1u : 0u);
        // pass 1: the first reference before the payload's start
        for (uint32_t k = 0; k < K; ++k) {
            const uint32_t p0 = P[k], p1 = k + 1 < K ? P[k + 1] : lim;
            const uint32_t n = p1 > p0 ? p1 - p0 : 0u;
            const uint16_t* sy = sym + S[k];
            for (uint32_t j = tid * 4; j < n; j += RES_THREADS * 4) {
#pragma unroll
                for (uint32_t q = 0; q < 4; ++q) {
                    if (j + q < n) {
                        const uint32_t v = sy[j + q];
                        if ((v & SYM_REF) && (v & 0x7fffu) + 1 > p0) atomicMin(&s_bad, p0 + j + q);
                    }
                }
            }
        }
        __syncthreads();
        const uint32_t bad = s_bad;
        const uint32_t olen = bad < lim ? bad : pr.olen;
        // pass 2: bytes [0, olen), 4 per thread per step; a reference is
        // followed through the symbols until a literal, at most RES_HOPS
        // times (a run of one byte repeated across many segments -- a
        // distance-1 match carried from segment to segment -- would take one
        // hop per segment for every byte: such a payload is finished by
        // pass 3 instead)
        bool deep = false;
        for (uint32_t k = 0; k < K; ++k) {
            const uint32_t p0 = P[k];
            if (p0 >= olen) break;
            const uint32_t p1 = k + 1 < K ? (P[k + 1] < olen ? P[k + 1] : olen) : olen;
            const uint16_t* sy = sym + S[k];
            for (uint32_t j = tid * 4; p0 + j < p1; j += RES_THREADS * 4) {
                uint32_t b[4];
#pragma unroll
                for (uint32_t q = 0; q < 4; ++q) {
                    b[q] = 0;
                    if (p0 + j + q < p1) {
                        uint32_t v = sy[j + q];
                        uint32_t base = p0;   // output start of the segment v belongs to
                        for (uint32_t h = 0; (v & SYM_REF) && h < RES_HOPS; ++h) {
                            const uint32_t t = base - ((v & 0x7fffu) + 1);   // >= 0 before `bad`
                            const uint32_t kk = seg_of(P, K, t);
                            base = P[kk];
                            v = sym[S[kk] + (t - base)];
                        }
                        deep = deep || (v & SYM_REF);
                        b[q] = v & 0xffu;
                    }
                }
                const uint32_t x = p0 + j;
                if (x + 4 <= p1) {
                    *(uint32_ua*)(o + x) = b[0] | (b[1] << 8) | (b[2] << 16) | (b[3] << 24);
                } else {
#pragma unroll
                    for (uint32_t q = 0; q < 4; ++q)
                        if (x + q < p1) o[x + q] = (uint8_t)b[q];
                }
            }
        }
        if (deep) s_deep = 1;
        __syncthreads();
        if (s_deep) {
            // pass 3: segment by segment in stream order, a reference reading
            // the byte the earlier segments wrote (round 4's resolve, with the
            // workgroup's four waves on each segment; the barrier makes the
            // bytes visible across them)
            for (uint32_t k = 0; k < K; ++k) {
                const uint32_t p0 = P[k];
                if (p0 >= olen) break;
                const uint32_t p1 = k + 1 < K ? (P[k + 1] < olen ? P[k + 1] : olen) : olen;
                const uint16_t* sy = sym + S[k];
                for (uint32_t j = tid * 4; p0 + j < p1; j += RES_THREADS * 4) {
#pragma unroll
                    for (uint32_t q = 0; q < 4; ++q) {
                        if (p0 + j + q < p1) {
                            const uint32_t v = sy[j + q];
                            o[p0 + j + q] = (v & SYM_REF) ? o[p0 - ((v & 0x7fffu) + 1)] : (uint8_t)v;
                        }
                    }
                }
                __syncthreads();
            }
        }
        if (tid == 0) {
            const bool inval = bad < lim;
            out_len[m] = olen;
            // (bad < lim: before the capacity in raw mode, at or before it in
            // pmd mode -- the serial decoder's order of the two checks)
            status[m] = inval ? ST_INVALID_DISTANCE : pr.status;
        }
        __syncthreads();
    }
}

}  // namespace bp
}  // namespace bpmd

// ------------------------------------------------------------------ driver
// Long payloads order[0, *nlong) of a batch (pmd_capi.hip inflate_impl); the
// rest of the batch is the caller's.  n: the batch's message count (bounds
// nlong).  The decode workspace has a per-(device, stream) capacity:
//   * the first call on a stream sizes it to that call's needs (one read-back
//     of the totals, the only wait of the path), or bpmd_inflate_reserve()
//     sets it beforehand with no wait at all;
//   * later calls only enqueue: long payloads that do not fit go to the wave
//     kernel (bp_fit_kernel, counted in bpmd_diag_bp_counters [3]) and each
//     call's totals are copied to pinned memory, so that a later call grows
//     the capacity to them once that copy has completed;
//   * growth is bounded by the device's free memory, and a workspace that
//     cannot be allocated falls back to the last capacity that could (or to
//     none: every long payload then takes the wave kernel), never an error.
namespace {
inline size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }
struct BpCaps {
    int dev;
    hipStream_t s;
    unsigned long long tasks, words;   // decode workspace capacity
    bpmd::bp::Totals* seen;            // pinned: the totals of the last call
    hipEvent_t ev;                     // recorded after that copy
    bool pending;                      // ev recorded, not yet consumed
    bool sized;                        // capacity set (first call or reserve)
    // after a workspace allocation failed: the capacity that could be had is
    // a ceiling for the next `hold` calls (8, doubling with every failure up
    // to 1024), so under memory pressure a call does not sync, free and fail
    // to allocate again every time
    unsigned long long ceil_tasks, ceil_words;
    uint32_t hold, backoff;
};
std::mutex g_bp_mu;
std::vector<BpCaps> g_bp_caps;
std::atomic<int> g_bp_fail{0};   // diagnostics: decode-workspace allocations to fail
std::atomic<int> g_bp_skim{-1};  // the skim: -1 from BPMD_BP_SKIM, 0 off, 1 on

uint8_t* dw_alloc(hipStream_t s, size_t bytes)
{
    if (g_bp_fail.load() > 0 && g_bp_fail.fetch_sub(1) > 0) return nullptr;
    return (uint8_t*)bpmd_internal_scratch(s, bytes, 11);
}

// the entry of (device, stream), created zeroed; nullptr when the pinned
// totals or the event cannot be made.  Caller holds g_bp_mu.
BpCaps* caps_for(int dev, hipStream_t s)
{
    for (auto& e : g_bp_caps)
        if (e.dev == dev && e.s == s) return &e;
    BpCaps e{dev, s, 0, 0, nullptr, nullptr, false, false, 0, 0, 0, 8};
    if (hipHostMalloc((void**)&e.seen, sizeof(bpmd::bp::Totals), hipHostMallocDefault) != hipSuccess) return nullptr;
    e.seen->tasks = e.seen->words = 0;
    if (hipEventCreateWithFlags(&e.ev, hipEventDisableTiming) != hipSuccess) {
        (void)hipHostFree(e.seen);
        return nullptr;
    }
    g_bp_caps.push_back(e);
    return &g_bp_caps.back();
}

// decode workspace layout for a capacity (n: the batch's message count):
// tasks, results, fallback list, region map, marks, the resolve's chains
// (output start and slot of every segment on a payload's chain, in chain
// order at the payload's first task; per payload: chain length, output
// length, status), symbols
struct DwLayout {
    size_t tasks, res, fb, map, mark, chp, chs, pay, sym, bytes;
    DwLayout(unsigned long long nt, unsigned long long words, uint32_t n)
    {
        using namespace bpmd::bp;
        tasks = 0;
        res = al256(tasks + sizeof(SegTask) * nt);
        fb = al256(res + sizeof(SegRes) * nt);
        map = al256(fb + 4ull * n);
        mark = al256(map + 4ull * nt);
        chp = al256(mark + 4ull * n);
        chs = al256(chp + 4ull * nt);
        pay = al256(chs + 8ull * nt);
        sym = al256(pay + sizeof(PayRes) * (size_t)n);
        bytes = al256(sym + 2ull * (words + SYM_GUARD + 64));
    }
};
inline size_t dw_bytes(unsigned long long tasks, unsigned long long words, uint32_t n)
{
    return DwLayout(tasks, words, n).bytes;
}

// a capacity of t tasks and w words plus a quarter, within half the free memory
void grow_to(BpCaps* c, unsigned long long t, unsigned long long w)
{
    unsigned long long nt = c->tasks, nw = c->words;
    if (t > nt) nt = t + t / 4;
    if (w > nw) nw = w + w / 4;
    if (nt > 0xffffffffull) nt = 0xffffffffull;
    size_t fr = 0, tot = 0;
    if ((nt != c->tasks || nw != c->words) && hipMemGetInfo(&fr, &tot) == hipSuccess) {
        // per task: the task, its result, the region map word and the
        // resolve's chain entries (DwLayout chp 4 B, chs 8 B)
        const unsigned long long budget = fr / 2,
                                 per_task = sizeof(bpmd::bp::SegTask) + sizeof(bpmd::bp::SegRes) + 4 + 4 + 8;
        if (nt * per_task > budget) nt = budget / per_task;
        if (2 * nw + nt * per_task > budget) nw = (budget - nt * per_task) / 2;
    }
    if (c->hold) {
        nt = nt < c->ceil_tasks ? nt : c->ceil_tasks;
        nw = nw < c->ceil_words ? nw : c->ceil_words;
    }
    c->tasks = nt > c->tasks ? nt : c->tasks;
    c->words = nw > c->words ? nw : c->words;
}
}  // namespace

// frees the pinned totals and event of a stream about to be destroyed
extern "C" void bpmd_internal_bp_release(hipStream_t s)
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return;
    std::lock_guard<std::mutex> lk(g_bp_mu);
    for (size_t i = 0; i < g_bp_caps.size(); ++i)
        if (g_bp_caps[i].dev == dev && g_bp_caps[i].s == s) {
            (void)hipEventSynchronize(g_bp_caps[i].ev);
            (void)hipHostFree(g_bp_caps[i].seen);
            (void)hipEventDestroy(g_bp_caps[i].ev);
            g_bp_caps[i] = g_bp_caps.back();
            g_bp_caps.pop_back();
            return;
        }
}

// bpmd_inflate_reserve (pmd_capi.hip): a capacity for batches whose long
// payloads total at most in_bytes of input, out_bytes of output capacity and
// msgs payloads -- bp_stats_kernel's bounds: regions of >= R_MIN bytes, at
// most one more per payload; slot words 2 (len + regions) x 1.25 x
// min(cap / len, 4) + SLACK per region + the guard per payload.
extern "C" int bpmd_internal_bp_reserve(hipStream_t s, unsigned long long in_bytes, unsigned long long out_bytes,
                                        unsigned long long msgs)
{
    using namespace bpmd::bp;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return (int)hipErrorNoDevice;
    const unsigned long long t = in_bytes / R_MIN + msgs;
    // (bp_stats_kernel: slots of 3 (len + regions) x F16 symbols, F16 = 1.25 x cap / len)
    const unsigned long long w = (15 * out_bytes) / 4 + (15ull + SLACK) * t + (SYM_GUARD + 64ull) * msgs;
    std::lock_guard<std::mutex> lk(g_bp_mu);
    BpCaps* c = caps_for(dev, s);
    if (!c) return (int)hipErrorOutOfMemory;
    grow_to(c, t, w);
    c->sized = true;
    return 0;
}

extern "C" int bpmd_internal_inflate_bp(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint32_t n,
                                        uint8_t* out, const uint64_t* out_off, const uint32_t* out_cap,
                                        uint32_t* out_len, int32_t* status, uint32_t raw, const uint32_t* order,
                                        const uint32_t* nlong, hipStream_t s)
{
    using namespace bpmd::bp;
    if (n == 0) return 0;
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    // this stream's capacity, grown to what an earlier call needed
    unsigned long long cap_tasks = 0, cap_words = 0;
    Totals* seen = nullptr;
    hipEvent_t ev = nullptr;
    bool cold = false;
    {
        std::lock_guard<std::mutex> lk(g_bp_mu);
        BpCaps* c = caps_for(dev, s);
        if (!c) return (int)hipErrorOutOfMemory;
        if (c->hold) --c->hold;   // the ceiling lifts after `hold` calls
        if (c->pending && hipEventQuery(c->ev) == hipSuccess) {
            c->pending = false;
            grow_to(c, c->seen->tasks, c->seen->words);
        }
        cold = !c->sized;
        cap_tasks = c->tasks;
        cap_words = c->words;
        seen = c->seen;
        ev = c->ev;
    }
    // per-payload workspace (scratch block 10): stats, regions, words, their
    // exclusive sums, totals, fit, queues, scan temp
    size_t tmp1 = 0, tmp2 = 0;
    if (hipcub::DeviceScan::ExclusiveSum(nullptr, tmp1, (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)n, s) !=
            hipSuccess ||
        hipcub::DeviceScan::ExclusiveSum(nullptr, tmp2, (const unsigned long long*)nullptr,
                                         (unsigned long long*)nullptr, (int)n, s) != hipSuccess)
        return (int)hipErrorUnknown;
    const size_t o_st = 0, o_reg = al256(o_st + sizeof(Stat) * (size_t)n), o_tb = al256(o_reg + 4ull * n),
                 o_w = al256(o_tb + 4ull * n), o_wb = al256(o_w + 8ull * n), o_tot = al256(o_wb + 8ull * n),
                 o_q = al256(o_tot + sizeof(Totals)), o_tmp = al256(o_q + 64),
                 sz = al256(o_tmp + (tmp1 > tmp2 ? tmp1 : tmp2));
    // q: [0] scan queue, [1] resolve queue, [2] fallback count, [3] seg queue,
    // [4-5] long bytes, [6] payloads that fit, [7] their tasks
    uint8_t* ws = (uint8_t*)bpmd_internal_scratch(s, sz, 10);
    if (!ws) return (int)hipErrorOutOfMemory;
    Stat* st = (Stat*)(ws + o_st);
    uint32_t* reg = (uint32_t*)(ws + o_reg);
    uint32_t* tbase = (uint32_t*)(ws + o_tb);
    unsigned long long* words = (unsigned long long*)(ws + o_w);
    unsigned long long* wbase = (unsigned long long*)(ws + o_wb);
    Totals* dtot = (Totals*)(ws + o_tot);
    uint32_t* q = (uint32_t*)(ws + o_q);
    void* tmp = ws + o_tmp;
    unsigned long long* total = (unsigned long long*)(q + 4);
    uint32_t* fit = q + 6;
    if (hipMemsetAsync(q, 0, 64, s) != hipSuccess) return (int)hipErrorUnknown;
    hipLaunchKernelGGL(bp_sum_kernel, dim3(n / 256 + 1 < 1024 ? n / 256 + 1 : 1024), dim3(256), 0, s, in_len, order,
                       nlong, n, total);
    // BPMD_BP_SEGS (diagnostics): target segments per lane of the chip
    static const uint32_t segs = [] {
        const char* e = getenv("BPMD_BP_SEGS");
        const uint32_t v = e ? (uint32_t)strtoul(e, nullptr, 10) : 0u;
        return v ? v : 4u;   // 2 / 4 / 8: C4 8-way shard 10.3 / 9.1 / 9.3 ms, C5 92 / 96 / 100 GiB/s
    }();
    hipLaunchKernelGGL(bp_stats_kernel, dim3((n + 255) / 256), dim3(256), 0, s, in_len, out_cap, order, nlong, n, total,
                       256u * (uint32_t)cus, segs, st, reg, words);
    if (hipGetLastError() != hipSuccess) return (int)hipErrorUnknown;
    size_t t1 = tmp1, t2 = tmp2;
    if (hipcub::DeviceScan::ExclusiveSum(tmp, t1, reg, tbase, (int)n, s) != hipSuccess ||
        hipcub::DeviceScan::ExclusiveSum(tmp, t2, words, wbase, (int)n, s) != hipSuccess)
        return (int)hipErrorUnknown;
    if (cold) {
        // the stream's first call: its own totals, read back once
        hipLaunchKernelGGL(bp_totals_kernel, dim3(1), dim3(64), 0, s, reg, tbase, words, wbase, n, dtot);
        if (hipGetLastError() != hipSuccess ||
            hipMemcpyAsync(seen, dtot, sizeof(Totals), hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            return (int)hipErrorUnknown;
        std::lock_guard<std::mutex> lk(g_bp_mu);
        BpCaps* c = caps_for(dev, s);
        if (!c) return (int)hipErrorOutOfMemory;
        grow_to(c, seen->tasks, seen->words);
        c->sized = true;
        cap_tasks = c->tasks;
        cap_words = c->words;
    }
    // decode workspace (scratch block 11), sized by the capacity: tasks,
    // results, fallback list, region map, marks, symbols.  A block that
    // cannot be had: the capacity it replaces, else none.
    uint8_t* dw = dw_alloc(s, dw_bytes(cap_tasks, cap_words, n));
    if (!dw) {
        (void)hipGetLastError();   // clear the allocation error
        unsigned long long pt = 0, pw = 0;
        {
            std::lock_guard<std::mutex> lk(g_bp_mu);
            BpCaps* c = caps_for(dev, s);
            if (c) {
                pt = c->tasks = c->tasks == cap_tasks ? c->tasks / 2 : c->tasks;
                pw = c->words = c->words == cap_words ? c->words / 2 : c->words;
            }
        }
        cap_tasks = pt;
        cap_words = pw;
        for (;;) {
            if (cap_words < (1ull << 16)) cap_tasks = cap_words = 0;
            dw = dw_alloc(s, dw_bytes(cap_tasks, cap_words, n));
            if (dw) break;
            (void)hipGetLastError();
            if (cap_words == 0) return (int)hipErrorOutOfMemory;   // not even the lists
            cap_tasks /= 2;
            cap_words /= 2;
        }
        std::lock_guard<std::mutex> lk(g_bp_mu);
        BpCaps* c = caps_for(dev, s);
        if (c) {
            c->tasks = cap_tasks;
            c->words = cap_words;
            c->ceil_tasks = cap_tasks;
            c->ceil_words = cap_words;
            c->hold = c->backoff;
            c->backoff = c->backoff < 1024 ? 2 * c->backoff : 1024u;
        }
    }
    const DwLayout D(cap_tasks, cap_words, n);
    SegTask* tasks = (SegTask*)(dw + D.tasks);
    SegRes* res = (SegRes*)(dw + D.res);
    uint32_t* fb = (uint32_t*)(dw + D.fb);
    uint16_t* sym = (uint16_t*)(dw + D.sym);
    uint32_t* rmap = (uint32_t*)(dw + D.map);
    uint32_t* marked = (uint32_t*)(dw + D.mark);
    uint32_t* chp = (uint32_t*)(dw + D.chp);
    uint64_t* chs = (uint64_t*)(dw + D.chs);
    PayRes* pay = (PayRes*)(dw + D.pay);
    if (hipMemsetAsync(marked, 0, 4ull * n, s) != hipSuccess) return (int)hipErrorUnknown;
    hipLaunchKernelGGL(bp_fit_kernel, dim3(1), dim3(256), 0, s, nlong, reg, tbase, words, wbase, n, cap_tasks,
                       cap_words, order, fit, dtot, fb, q + 2);
    // the totals for a later call (pinned, no wait here); the event counts
    // only once it is recorded
    if (hipGetLastError() != hipSuccess ||
        hipMemcpyAsync(seen, dtot, sizeof(Totals), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipEventRecord(ev, s) != hipSuccess)
        return (int)hipErrorUnknown;
    {
        std::lock_guard<std::mutex> lk(g_bp_mu);
        BpCaps* c = caps_for(dev, s);
        if (c) c->pending = true;
    }
    // scan: one wave per region, SCAN_WAVES waves per workgroup, ~3
    // workgroups per CU by LDS; then the slots, one wave per payload
    hipLaunchKernelGGL(bp_region_map_kernel, dim3((n + 255) / 256), dim3(256), 0, s, fit, reg, tbase, rmap);
    const uint32_t scan_wgs = 3u * cus;
    // BPMD_BP_DYN_STRIDE: pass 2 searches every n-th pending region (default
    // 1; 4 measured C4 8-way Beast shard 16.6 -> 17.8 ms, C5 17.6 -> 15.7 ms,
    // profiles/r05j_ab_compact_canon.log)
    static const uint32_t dyn_stride = [] {
        const char* e = getenv("BPMD_BP_DYN_STRIDE");
        const uint32_t v = e ? (uint32_t)strtoul(e, nullptr, 10) : 0u;
        return v ? v : 1u;   // 1: the per-payload stride (bp_scan_kernel)
    }();
    hipLaunchKernelGGL(bp_scan_kernel<false>, dim3(scan_wgs), dim3(64 * SCAN_WAVES), 0, s, in, in_off, in_len, order,
                       rmap, fit + 1, st, tbase, tasks, marked, dyn_stride);
    // the skim (payloads without sync markers), then pass 2 on the regions no
    // walk reached (BPMD_BP_SKIM=1; off by default: see the A/B in DESIGN 4.1d)
    int skim_mode = g_bp_skim.load();
    if (skim_mode < 0) {
        const char* e = getenv("BPMD_BP_SKIM");
        skim_mode = e && e[0] == '1' ? 1 : 0;
        g_bp_skim.store(skim_mode);
    }
    const bool skim = skim_mode == 1;
    if (skim)
        hipLaunchKernelGGL(bp_skim_kernel, dim3(4u * cus), dim3(256), 0, s, in, in_off, in_len, order, rmap, fit + 1, st,
                           tbase, tasks, marked);
    hipLaunchKernelGGL(bp_scan_kernel<true>, dim3(scan_wgs), dim3(64 * SCAN_WAVES), 0, s, in, in_off, in_len, order,
                       rmap, fit + 1, st, tbase, tasks, marked, dyn_stride);
    hipLaunchKernelGGL(bp_slots_kernel, dim3(4u * cus), dim3(256), 0, s, in_len, order, fit, st, tbase,
                       wbase, tasks);
    if (hipGetLastError() != hipSuccess) return (int)hipErrorUnknown;
    // segments: a work queue over the device-side task count
    const uint32_t wgs = 4u * cus;
    int e = bpmd_internal_inflate_lane3_seg(in, in_off, in_len, (uint32_t)cap_tasks, tasks, sym, res, raw, q + 3, wgs,
                                            s, fit + 1);
    if (e) return e;
    // resolve: the serial walk per payload (default), or the segment-parallel
    // form (BPMD_BP_RESOLVE=parallel; measured slower: a reference in
    // deflated JSON usually points at a byte that was itself copied from the
    // segment before, and so on back to the payload's first segment, so the
    // chase through symbols runs one hop per earlier segment -- C4 8-way
    // shard 8.6 -> 14.7 ms, profiles/r05e_resolve_ab.log)
    static const bool serial_resolve = [] {
        const char* e = getenv("BPMD_BP_RESOLVE");
        return !(e && !strcmp(e, "parallel"));
    }();
    if (serial_resolve) {
        hipLaunchKernelGGL(bp_resolve_kernel, dim3(8u * cus), dim3(256), 0, s, in, in_off, order, fit, tbase, tasks, res,
                           sym, out, out_off, out_cap, out_len, status, raw, fb, q + 2, q + 1, st);
        if (hipGetLastError() != hipSuccess) return (int)hipErrorUnknown;
    } else {
        hipLaunchKernelGGL(bp_chain_kernel, dim3(n / 256 + 1), dim3(256), 0, s, order, fit, tbase, tasks, res, out_cap,
                           raw, st, chp, chs, pay, out_len, status, fb, q + 2);
        hipLaunchKernelGGL(bp_resolve2_kernel, dim3(8u * cus), dim3(RES_THREADS), 0, s, order, fit, tbase, sym, out,
                           out_off, out_cap, out_len, status, raw, chp, chs, pay, q + 1);
        if (hipGetLastError() != hipSuccess) return (int)hipErrorUnknown;
    }
    // payloads over the capacity or whose output outgrew the slots: the wave
    // kernel, from the list
    return bpmd_internal_inflate_wave_ordered(in, in_off, in_len, n, out, out_off, out_cap, out_len, status, raw,
                                              nullptr, fb, q + 2, s);
}

// the fixed-block skim on (1) or off (0) for the following calls (tests, A/B)
extern "C" void bpmd_diag_set_bp_skim(int on) { g_bp_skim.store(on ? 1 : 0); }

// diagnostics (tests): the next k decode-workspace allocations fail
extern "C" void bpmd_diag_bp_fail_alloc(int k) { g_bp_fail.store(k); }

// diagnostics (tests): the stream's decode-workspace capacity and ceiling:
// out[0] tasks, [1] words, [2] ceiling tasks, [3] ceiling words, [4] calls
// the ceiling still holds; -1 when the stream has no entry
extern "C" int bpmd_diag_bp_caps(hipStream_t s, unsigned long long* out5)
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return -1;
    std::lock_guard<std::mutex> lk(g_bp_mu);
    for (auto& e : g_bp_caps)
        if (e.dev == dev && e.s == s) {
            out5[0] = e.tasks;
            out5[1] = e.words;
            out5[2] = e.ceil_tasks;
            out5[3] = e.ceil_words;
            out5[4] = e.hold;
            return 0;
        }
    return -1;
}

extern "C" int bpmd_diag_bp_fallback(uint32_t* out8)
{
    return hipMemcpyFromSymbol(out8, HIP_SYMBOL(bpmd::bp::g_bp_fb), sizeof(uint32_t) * 8) == hipSuccess ? 0 : -1;
}

// diagnostics: the 12 counters of g_bp_diag (out[12]); reset after reading
extern "C" int bpmd_diag_bp_counters(unsigned long long* out, int reset)
{
    unsigned long long v[12] = {};
    if (hipMemcpyFromSymbol(v, HIP_SYMBOL(bpmd::bp::g_bp_diag), sizeof v) != hipSuccess) return -1;
    for (int i = 0; i < 12; ++i) out[i] = v[i];
    if (reset) {
        const unsigned long long z[12] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(bpmd::bp::g_bp_diag), z, sizeof z) != hipSuccess) return -1;
    }
    return 0;
}
