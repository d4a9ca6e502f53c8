// pmd_inflate_lane3.hip -- batched raw-DEFLATE decode, one LANE per message,
// split across two waves that run side by side: a DECODER wave and an
// EXPANDER wave per 64 messages, joined by a per-message token ring in LDS.
//
// Every lane runs the reference's serial decoder (include/boost/beast/zlib/
// detail/inflate_stream.ipp:74-535) on its own message, but one wave doing
// both Huffman decoding and the output copies serialises two unrelated
// instruction streams: every iteration issues the decode code, the header
// code and the copy code for all 64 lanes, and a wave alone on its SIMD
// issues at most one instruction every ~4 cycles and stalls on each of its
// LDS and memory waits (MI355X_MICROARCH.md: "one wave alone: 4").  Here
// each workgroup has two waves over the same 64 messages:
//
//   decoder  (wave 0)  bit reader, block headers, canonical tables, symbol
//                      decode with the reference's checks; per iteration it
//                      emits one 8-byte token: up to 4 literal bytes and an
//                      optional match (length, distance); never touches the
//                      output slot
//   expander (wave 1)  takes tokens and writes the output: literal bytes,
//                      match copies from the lane's own earlier output in
//                      16/32-byte chunks (the slot is the window), the
//                      message's out_len / status at its END token
//
// so each wave runs one lean stream, and the SIMD interleaves the two: the
// expander's memory waits hide behind decoding, the decoder's LDS waits
// behind copying.  Two waves per SIMD need <= 256 VGPRs (this kernel: see
// the resource remark); 4 workgroups x 64 lanes x 632 B fit the 160 KiB LDS.
//
// Token ring: 32 entries of 8 B per message, stored in the per-lane LDS
// that only block headers use (code-length histogram, nibbles, code-length
// code symbols), so the decoder waits for the ring to drain before a
// dynamic block header.  head (written by the decoder) and tail (by the
// expander) sit after the lane's tables.  LDS operations of one wave are
// performed in issue order, so writing an entry before head (decoder) and
// reading head before the entry (expander) publishes it; the compiler is
// kept from reordering them by relaxed atomics and memory clobbers.
//
// Token word 1: bits 0-2 literal count, 3-11 match length (0 = none),
// 12-27 distance; bit 31 = END (word 0 = out_len, bits 0-7 = status).
// Output semantics per message are those of pmd_inflate.hip.
#include <hipcub/hipcub.hpp>

#include "pmd_common.h"
#include "canon.h"
#include "bp.h"
#include "lane_io.h"

namespace bpmd {
namespace lp3 {
using namespace lio;

// per-lane LDS layout (bytes)
constexpr unsigned O_LIT = 0;      // u8[288]  literal/length symbols, canonical order (low 8 bits)
constexpr unsigned O_DST = 288;    // u8[32]   distance symbols, canonical order
constexpr unsigned O_HIST = 320;   // u32[16]  pass 1: length histogram (lit | lit<256 << 10 | dist << 20)
                                   //          pass 2: placement cursors (lit | dist << 16)
                                   //          data: token ring entries 0-7
constexpr unsigned O_LE = 384;     // u16[16]  litend per code length
constexpr unsigned O_CLS = 416;    // u8[20]   code-length code symbols, canonical order  } data: token
constexpr unsigned O_NIB = 448;    // u8[160]  code lengths, one nibble per symbol       } ring 8-31
constexpr unsigned O_HEAD = 624;   // u32      tokens written (decoder)
constexpr unsigned O_TAIL = 628;   // u32      tokens taken (expander)
constexpr unsigned STRIDE = 632;   // x 64 lanes x 4 workgroups = 161 792 B per CU
#ifndef BPMD3_RING
#define BPMD3_RING 32
#endif
constexpr unsigned RING = BPMD3_RING;   // token ring entries per message (at most 32: the header scratch holds 32)
constexpr unsigned WG_MSGS = 64;
constexpr uint32_t TOK_END = 0x80000000u;   // word 0: out_len, bits 0-7: status
constexpr uint32_t TOK_NEW = 0x40000000u;   // word 0: the message the lane starts (work queue)
constexpr uint32_t TOK_EXIT = 0x20000000u;  // the queue is empty: the lane is done
constexpr uint32_t TOK_STORED = 0x10000000u;  // segment mode: bits 0-15 stored bytes, word 0 their payload offset

#ifndef BPMD3_KLIT
#define BPMD3_KLIT 4
#endif
#ifndef BPMD3_ESLEEP
#define BPMD3_ESLEEP 8
#endif
#ifndef BPMD3_KX
#define BPMD3_KX 4
#endif
#ifndef BPMD3_XSTEPS
#define BPMD3_XSTEPS 1
#endif
#ifndef BPMD3_XPIPE
#define BPMD3_XPIPE 0
#endif
constexpr int KX = BPMD3_KX;   // expander pieces per iteration
#ifndef BPMD3_DPRIO
#define BPMD3_DPRIO 3
#endif
constexpr int KLIT = BPMD3_KLIT;   // symbols decoded per iteration when literals lead (bytes queue in one u32)
#ifndef BPMD3_KCL
#define BPMD3_KCL 6
#endif
// compact canonical search (canon.h compact_canon): words per literal/length
// and distance table (0, the default: the full 15-word search only).
// Measured slower on C2 (11 / 8 words: 163-167, 9 / 7: 172, off: 190-191
// GiB/s, three interleaved runs, profiles/r05j_ab_compact_canon.log): the
// compact words are 27 more VGPRs live across the loop (208 vs 181) and a
// wave-uniform branch per decode, which cost more than the 9 subtractions
// and mins they save.
#ifndef BPMD3_CKL
#define BPMD3_CKL 0
#endif
#ifndef BPMD3_CKD
#define BPMD3_CKD 8
#endif
constexpr int CKL = BPMD3_CKL > 0 ? BPMD3_CKL : 1, CKD = BPMD3_CKD > 0 ? BPMD3_CKD : 1;
constexpr int KCL = BPMD3_KCL;   // code-length symbols per iteration (pass 1; a refill before each, <= 4 input dwords per iteration)
#ifndef BPMD3_KNIB
#define BPMD3_KNIB 32
#endif
constexpr int KNIB = BPMD3_KNIB;  // code lengths placed per iteration (pass 2; a multiple of 8, at most 32)

enum : uint32_t { S_TYPE, S_DATA, S_SHDR, S_SCOPY, S_DYN, S_PASS1, S_BUILD, S_PASS2, S_DONE };

__device__ __forceinline__ unsigned ring_at(uint32_t e)
{
    const uint32_t k = e % RING;
    return k < 8 ? O_HIST + 8 * k : O_CLS + 8 * (k - 8);
}

// Per-lane LDS addressing.  Default: one lane's area is contiguous, lanes
// STRIDE bytes apart (158 dwords, an even count: same-offset accesses of
// lanes l and l + 16 share a bank, and table lookups at lane-dependent
// offsets collide at random).  BPMD3_ILV=1 interleaves the 64 areas by
// dword -- dword w of lane l at 256 w + 4 l of the workgroup's block -- so
// every lane stays in bank l mod 32 whatever the offset (MI355X_MICROARCH.md
// LDS: ds_read_b32 serves lanes 0-31 and 32-63 one cycle each): C2's
// SQ_LDS_BANK_CONFLICT 36.5 M -> 0, but each table lookup's address costs two
// more VALU instructions (SQ_INSTS_VALU 471 M -> 501 M) and the decoder is
// issue-bound, not LDS-bound (SQ_WAIT_INST_LDS 1.4 M of 1 428 M wave
// cycles): C2 189.4-190.3 (contiguous) vs 184.4-185.3 GiB/s (interleaved),
// three interleaved runs on one box (profiles/r05b_ab_lds_interleave.log,
// r05b_c2_sq_interleaved.txt).
#ifndef BPMD3_ILV
#define BPMD3_ILV 0
#endif
__device__ __forceinline__ uint8_t* lane_area(uint8_t* smem, unsigned lane)
{
    return BPMD3_ILV ? smem + 4 * lane : smem + lane * STRIDE;
}
// byte b / dword w of the lane's area (T = lane_area())
__device__ __forceinline__ uint8_t* lb(uint8_t* T, uint32_t b)
{
    return BPMD3_ILV ? T + (((b >> 2) << 8) | (b & 3u)) : T + b;
}
__device__ __forceinline__ uint32_t* lw(uint8_t* T, uint32_t w)
{
    return BPMD3_ILV ? (uint32_t*)(T + (w << 8)) : (uint32_t*)T + w;
}
__device__ __forceinline__ uint2 ring_ld(uint8_t* T, uint32_t e)
{
    const uint32_t d = ring_at(e) >> 2;
    return make_uint2(*lw(T, d), *lw(T, d + 1));
}
__device__ __forceinline__ void ring_st(uint8_t* T, uint32_t e, uint2 v)
{
    const uint32_t d = ring_at(e) >> 2;
    *lw(T, d) = v.x;
    *lw(T, d + 1) = v.y;
}
// c ? b : a as bitwise selects the compiler cannot turn back into a
// dynamically indexed array (which it places in scratch memory)
__device__ __forceinline__ uint2 pick(uint2 a, uint2 b, bool c)
{
    uint32_t m = c ? ~0u : 0u;
    asm volatile("" : "+v"(m));
    return make_uint2((b.x & m) | (a.x & ~m), (b.y & m) | (a.y & ~m));
}
constexpr uint32_t W_HIST = O_HIST / 4, W_LE = O_LE / 4, W_NIB = O_NIB / 4, W_HEAD = O_HEAD / 4, W_TAIL = O_TAIL / 4;
// Diagnostic build only (-DBPMD_PROF): per-role loop counters, summed over waves:
// [0] decoder cycles [1] decoder iterations [2] decoder sleeps [3] decoder
// header iterations [4] expander cycles [5] expander iterations [6] expander sleeps
__device__ unsigned long long g_l3prof[16];
// [0-4] decoder cycles in the header section's parts (type / stored / copy,
// TABLE + LENLENS, CODELENS, BUILD, PLACE), [5-7] spare (prof build only)
__device__ unsigned long long g_l3hprof[8];
#ifdef BPMD_PROF
#define L3_DECL unsigned long long l3t0_ = __builtin_amdgcn_s_memtime(), l3c_[4] = {0, 0, 0, 0}
#define L3_CNT(i) (l3c_[i] += 1)
#define L3_LAPDECL unsigned long long l3l_ = __builtin_amdgcn_s_memtime(), l3lap_[4] = {0, 0, 0, 0}
#define L3_LAP(i) do { const unsigned long long t2_ = __builtin_amdgcn_s_memtime(); l3lap_[i] += t2_ - l3l_; l3l_ = t2_; } while (0)
#define L3_LAPFLUSH() do { if ((threadIdx.x & 63) == 0) { for (int i_ = 0; i_ < 4; ++i_) atomicAdd(&g_l3prof[8 + i_], l3lap_[i_]); \
    for (int i_ = 0; i_ < 5; ++i_) atomicAdd(&g_l3hprof[i_], l3h_[i_]); } } while (0)
#define L3_HSTART() unsigned long long l3hl_ = __builtin_amdgcn_s_memtime()
#define L3_HLAP(i) do { const unsigned long long t2_ = __builtin_amdgcn_s_memtime(); l3h_[i] += t2_ - l3hl_; l3hl_ = t2_; } while (0)
#define L3_FLUSH(base) do { if ((threadIdx.x & 63) == 0) { atomicAdd(&g_l3prof[base], __builtin_amdgcn_s_memtime() - l3t0_); \
    for (int i_ = 1; i_ < 4; ++i_) atomicAdd(&g_l3prof[base + i_], l3c_[i_]); } } while (0)
#else
#define L3_DECL
#define L3_CNT(i)
#define L3_FLUSH(base)
#define L3_LAPDECL
#define L3_LAP(i)
#define L3_LAPFLUSH()
#define L3_HSTART()
#define L3_HLAP(i)
#endif

static __constant__ const uint8_t kClenOrder2[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// ------------------------------------------------------------------ expander
// Up to KX pieces per iteration -- a token's literal bytes and one chunk of
// its match -- are taken from the ring, and every match chunk whose source
// lies wholly below the output already stored (F) is loaded in the same
// iteration, so the pieces' loads are in flight together; they are stored at
// the start of the next iteration, in output order (a store's spare bytes
// past its piece are overwritten by the next store).  A match whose source
// reaches into pieces not yet stored ends the batch.  Distances below 8
// become a pattern register built from the 8 bytes before the match.
__device__ __forceinline__ void expander(uint8_t* T, bool valid, uint32_t m, uint8_t* __restrict__ out,
                                         const uint64_t* __restrict__ out_off, const uint32_t* __restrict__ out_cap,
                                         uint32_t* __restrict__ out_len, int32_t* __restrict__ status,
                                         const uint32_t* __restrict__ hist_len, uint32_t hist_max, bool queue)
{
    uint8_t* o = out;
    uint32_t cap = 0, hist = 0;
    auto slot = [&](uint32_t mm) {
        o = out + out_off[mm];
        cap = out_cap[mm];
        hist = hist_len ? (hist_len[mm] < hist_max ? hist_len[mm] : hist_max) : 0u;
    };
    if (valid) slot(m);
    bool exited = !queue && !valid;   // no token will come any more
    uint32_t tail = 0, pos = 0;       // pos: output position after every piece taken
    // the match being copied: bytes left, distance, next output position
    uint32_t crem = 0, cdist = 0, cq = 0;
    uint64_t cpat = 0;
    uint32_t cpat_st = 0;   // dist < 8: 0 pattern not requested, 1 requested, 2 ready
    // pieces taken in the previous iteration, stored at the start of this one
    uint32_t l_dst[KX], l_val[KX], l_n[KX], m_dst[KX], m_sz[KX], m_pat[KX];
    uint4 m_w[KX];
#pragma unroll
    for (int j = 0; j < KX; ++j) {
        l_dst[j] = l_val[j] = l_n[j] = m_dst[j] = m_sz[j] = m_pat[j] = 0;
        m_w[j] = make_uint4(0, 0, 0, 0);
    }
    L3_DECL;
    for (;;) {
        bool pending = false;
#pragma unroll
        for (int j = 0; j < KX; ++j) pending = pending || l_n[j] != 0 || m_sz[j] != 0;
        if (!__ballot(!exited || crem != 0 || pending)) break;
        L3_CNT(1);
        bool worked = pending;
        // ================================================ stores, output order
        // (a store's bytes past its piece are overwritten by the next one)
#pragma unroll
        for (int j = 0; j < KX; ++j) {
            if (l_n[j]) {
                if (l_dst[j] + 4 <= cap) {
                    *(uint32_u*)(o + l_dst[j]) = l_val[j];
                } else {
#pragma unroll
                    for (uint32_t b = 0; b < 4; ++b)
                        if (b < l_n[j]) o[l_dst[j] + b] = (uint8_t)(l_val[j] >> (8 * b));
                }
            }
            if (m_sz[j]) {
                uint4 w = m_w[j];
                if (m_pat[j]) {
                    // the cpd bytes before the match, repeated with period cpd
                    const uint32_t cpd = m_pat[j] & 0xffu, csh = m_pat[j] >> 8;
                    uint64_t v = ((uint64_t)w.y << 32) | w.x;
                    v >>= 8 * csh;
                    v &= (1ull << (8 * cpd)) - 1;
                    if (cpd < 8) v |= v << (8 * cpd);
                    if (cpd < 4) v |= v << (16 * cpd);
                    if (cpd < 2) v |= v << (32 * cpd);
                    if (cpat_st == 1) {   // still the current match
                        cpat = v;
                        cpat_st = 2;
                    }
                    w = make_uint4((uint32_t)v, (uint32_t)(v >> 32), 0, 0);
                }
                store_bounded(o, m_dst[j], m_sz[j], cap, w);
            }
            l_n[j] = 0;
            m_sz[j] = 0;
            m_pat[j] = 0;
        }
        // ================================================ take pieces
        if (!exited) {
            const uint32_t head = lds_load((uint8_t*)lw(T, W_HEAD));
            compiler_fence();
            uint2 ent[KX];
#pragma unroll
            for (int j = 0; j < KX; ++j) ent[j] = ring_ld(T, tail + j);
            compiler_fence();
            const uint32_t F = crem ? cq : pos;   // everything before F is stored
            uint32_t k = 0;                       // entries taken this iteration
            bool stop = false;
#pragma unroll
            for (int j = 0; j < KX; ++j) {
                if (!stop && crem == 0) {
                    if (tail == head) {
                        stop = true;
                    } else {
                        uint2 e = ent[0];
#pragma unroll
                        for (int i = 1; i <= j; ++i) e = pick(e, ent[i], k == (uint32_t)i);
                        if (e.y & TOK_END) {
                            out_len[m] = e.x;
                            const int32_t stt = (int32_t)(int8_t)(e.y & 0xffu);
                            status[m] = stt;
                            exited = !queue;
                            ++tail;
                            ++k;
                            worked = true;
                            stop = true;
                        } else if (e.y & (TOK_NEW | TOK_EXIT)) {
                            // switches the output slot: only with no piece pending
                            if (j == 0) {
                                if (e.y & TOK_NEW) {
                                    m = e.x;
                                    slot(m);
                                    pos = 0;
                                } else {
                                    exited = true;
                                }
                                ++tail;
                                ++k;
                                worked = true;
                            }
                            stop = true;
                        } else {
                            const uint32_t nl = e.y & 7u, ml = (e.y >> 3) & 511u;
                            if (nl) {
                                l_dst[j] = pos;
                                l_val[j] = e.x;
                                l_n[j] = nl;
                                pos += nl;
                            }
                            if (ml) {
                                crem = ml;
                                cdist = (e.y >> 12) & 0xffffu;
                                cq = pos;
                                cpat_st = 0;
                                pos += ml;
                            }
                            ++tail;
                            ++k;
                            worked = true;
                        }
                    }
                }
                if (!stop && crem != 0) {
                    if (cdist >= 8) {
                        // a chunk whose source lies below F: loaded now, stored next iteration
                        const uint32_t C = cdist >= 16 ? 16u : 8u;
                        const uint32_t n = crem < C ? crem : C;
                        const int32_t src = (int32_t)cq - (int32_t)cdist;
                        if (src + (int32_t)n <= (int32_t)F) {
                            if (C == 16) {
                                m_w[j] = *(const uint4_u*)(o + src);
                            } else {
                                const uint2 v = *(const uint2_u*)(o + src);
                                m_w[j] = make_uint4(v.x, v.y, 0, 0);
                            }
                            m_dst[j] = cq;
                            m_sz[j] = C;
                            cq += n;
                            crem -= n;
                            worked = true;
                        } else {
                            stop = true;
                        }
                    } else {
                        const uint32_t adv0 = 8 - 8 % cdist;
                        const uint32_t adv = adv0 < crem ? adv0 : crem;
                        if (cpat_st == 2) {
                            m_w[j] = make_uint4((uint32_t)cpat, (uint32_t)(cpat >> 32), 0, 0);
                            m_dst[j] = cq;
                            m_sz[j] = 8;
                            cq += adv;
                            crem -= adv;
                            worked = true;
                        } else if (cpat_st == 0 && cq <= F) {
                            // the cdist bytes before cq, read as 8 bytes that never
                            // start before the slot's window
                            const int32_t src = max((int32_t)cq - 8, -(int32_t)hist);
                            const uint2 v = *(const uint2_u*)(o + src);
                            m_w[j] = make_uint4(v.x, v.y, 0, 0);
                            m_pat[j] = cdist | ((uint32_t)((int32_t)cq - (int32_t)cdist - src) << 8);
                            cpat_st = 1;
                            m_dst[j] = cq;
                            m_sz[j] = 8;
                            cq += adv;
                            crem -= adv;
                            worked = true;
                        } else {
                            stop = true;
                        }
                    }
                }
            }
            lds_store((uint8_t*)lw(T, W_TAIL), tail);
        }
        if (!__ballot(worked)) {   // the decoder is behind: leave it the SIMD
            L3_CNT(2);
            __builtin_amdgcn_s_sleep(BPMD3_ESLEEP);
        }
    }
    L3_FLUSH(4);
}

// --------------------------------------------------------- segment expander
// Segment mode (bp.h): the slot holds 16-bit symbols.  Match sources before
// the slot's start become references (SYM_REF | k: the byte k + 1 positions
// before the segment), so a chunk that straddles the start is loaded from
// the guard or the preceding slot and its early elements replaced; a chunk
// wholly before the start is not loaded at all.  Same pipeline as
// expander(): a chunk loaded in one memory section is stored in the next,
// stores go in output order, spare elements past a token are overwritten
// by later output, nothing is stored past the slot's capacity.
typedef uint2 uint2_s __attribute__((aligned(2)));
typedef uint4 uint4_s __attribute__((aligned(2)));

__device__ __forceinline__ uint32_t ref_pair(uint32_t w, int32_t a)   // elements a, a + 1 packed in w
{
    const uint32_t lo = a < 0 ? (bp::SYM_REF | (uint32_t)(-a - 1)) : (w & 0xffffu);
    const uint32_t hi = a + 1 < 0 ? (bp::SYM_REF | (uint32_t)(-a - 2)) : (w >> 16);
    return lo | (hi << 16);
}
__device__ __forceinline__ uint4 ref_fix(uint4 w, int32_t src)
{
    return make_uint4(ref_pair(w.x, src), ref_pair(w.y, src + 2), ref_pair(w.z, src + 4), ref_pair(w.w, src + 6));
}
// the 8 symbols before a match of distance p < 8, repeated with period p
__device__ __forceinline__ uint4 sym_pattern(uint4 w, uint32_t p)
{
    const uint32_t e[8] = {w.x & 0xffffu, w.x >> 16, w.y & 0xffffu, w.y >> 16,
                           w.z & 0xffffu, w.z >> 16, w.w & 0xffffu, w.w >> 16};
    uint32_t r[8];
    uint32_t idx = 8 - p;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        uint32_t v = e[0];
#pragma unroll
        for (int k = 1; k < 8; ++k) v = idx == (uint32_t)k ? e[k] : v;
        r[j] = v;
        idx = idx + 1 == 8 ? 8 - p : idx + 1;
    }
    return make_uint4(r[0] | (r[1] << 16), r[2] | (r[3] << 16), r[4] | (r[5] << 16), r[6] | (r[7] << 16));
}
__device__ __forceinline__ void store_syms8(uint16_t* o, uint32_t dst, uint32_t lim, uint4 w)
{
    if (dst + 8 <= lim) {
        *(uint4_s*)(o + dst) = w;
        return;
    }
    const uint32_t d[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j)
        if (dst + j < lim) o[dst + j] = (uint16_t)(d[j >> 1] >> (16 * (j & 1)));
}

// four payload bytes as four symbols (two dwords)
__device__ __forceinline__ uint32_t sym_lo(uint32_t d) { return __builtin_amdgcn_perm(0u, d, 0x0c010c00u); }
__device__ __forceinline__ uint32_t sym_hi(uint32_t d) { return __builtin_amdgcn_perm(0u, d, 0x0c030c02u); }

__device__ __forceinline__ void expander_seg(uint8_t* T, bool valid, uint32_t m, uint16_t* __restrict__ sym,
                                             const bp::SegTask* __restrict__ tasks, bp::SegRes* __restrict__ res,
                                             bool queue, const uint8_t* __restrict__ in,
                                             const uint64_t* __restrict__ in_off, const uint32_t* __restrict__ in_len)
{
    // The batched pipeline of expander(): up to KX pieces per iteration, a
    // piece being a token's literal symbols and one chunk -- of a match (8 or
    // 16 symbols whose source lies below F or before the segment), of its
    // pattern (distances below 8), or of a stored block's bytes (32, read from
    // the payload) -- loaded in one iteration and stored in the next.
    uint16_t* o = sym;
    uint32_t cap = 0;
    const uint8_t* pl = in;   // the task's payload, [pl, pl_end)
    const uint8_t* pl_end = in;
    auto slot = [&](uint32_t t) {
        const bp::SegTask tk = tasks[t];
        o = sym + tk.sym_off;
        cap = tk.sym_cap;
        const uint32_t mm = tk.kind == bp::KIND_NONE ? 0u : tk.msg;
        pl = in + in_off[mm];
        pl_end = pl + in_len[mm];
    };
    if (valid) slot(m);
    bool exited = !queue && !valid;
    uint32_t tail = 0, pos = 0;
    uint32_t crem = 0, cdist = 0, cq = 0;
    uint4 cpat = make_uint4(0, 0, 0, 0);
    uint32_t cpat_st = 0;   // dist < 8: 0 pattern not requested, 1 requested, 2 ready
    // stored block being copied: bytes left, next source, next symbol
    uint32_t srem = 0, sdst = 0;
    const uint8_t* ssrc = in;
    // pieces: literal symbols, and a chunk of kind 0 none, 1 match, 2 pattern
    // (ready), 3 pattern request, 4 stored bytes
    constexpr uint32_t CK_MATCH = 1, CK_PAT = 2, CK_PATREQ = 3, CK_STORED = 4;
    uint32_t l_dst[KX], l_val[KX], l_n[KX], c_kind[KX], c_dst[KX], c_sz[KX];
    int32_t c_src[KX];
    uint4 c_w0[KX], c_w1[KX];
#pragma unroll
    for (int j = 0; j < KX; ++j) {
        l_dst[j] = l_val[j] = l_n[j] = c_kind[j] = c_dst[j] = c_sz[j] = 0;
        c_src[j] = 0;
        c_w0[j] = c_w1[j] = make_uint4(0, 0, 0, 0);
    }
    L3_DECL;
    for (;;) {
        bool pending = false;
#pragma unroll
        for (int j = 0; j < KX; ++j) pending = pending || l_n[j] != 0 || c_kind[j] != 0;
        if (!__ballot(!exited || crem != 0 || srem != 0 || pending)) break;
        L3_CNT(1);
        bool worked = pending;
        // ================================================ stores, output order
#pragma unroll
        for (int j = 0; j < KX; ++j) {
            if (l_n[j]) {
                // the token's literal bytes as four symbols, one 8-byte store
                const uint32_t bval = l_val[j], bdst = l_dst[j];
                const uint2 w = make_uint2((bval & 0xffu) | ((bval & 0xff00u) << 8),
                                           ((bval >> 16) & 0xffu) | ((bval >> 8) & 0xff0000u));
                if (bdst + 4 <= cap) {
                    *(uint2_s*)(o + bdst) = w;
                } else {
#pragma unroll
                    for (uint32_t q = 0; q < 4; ++q)
                        if (q < l_n[j] && bdst + q < cap) o[bdst + q] = (uint16_t)((bval >> (8 * q)) & 0xffu);
                }
            }
            if (c_kind[j] == CK_STORED) {
                const uint4 w0 = c_w0[j], w1 = c_w1[j];
                const uint32_t d = c_dst[j];
                store_syms8(o, d, cap, make_uint4(sym_lo(w0.x), sym_hi(w0.x), sym_lo(w0.y), sym_hi(w0.y)));
                store_syms8(o, d + 8, cap, make_uint4(sym_lo(w0.z), sym_hi(w0.z), sym_lo(w0.w), sym_hi(w0.w)));
                store_syms8(o, d + 16, cap, make_uint4(sym_lo(w1.x), sym_hi(w1.x), sym_lo(w1.y), sym_hi(w1.y)));
                store_syms8(o, d + 24, cap, make_uint4(sym_lo(w1.z), sym_hi(w1.z), sym_lo(w1.w), sym_hi(w1.w)));
            } else if (c_kind[j] == CK_PAT) {
                store_syms8(o, c_dst[j], cap, c_w0[j]);
            } else if (c_kind[j]) {
                uint4 w = ref_fix(c_w0[j], c_src[j]);
                if (c_kind[j] == CK_PATREQ) {
                    w = sym_pattern(w, c_sz[j]);
                    if (cpat_st == 1) {   // still the current match
                        cpat = w;
                        cpat_st = 2;
                    }
                }
                store_syms8(o, c_dst[j], cap, w);
                if (c_kind[j] == CK_MATCH && c_sz[j] == 16) store_syms8(o, c_dst[j] + 8, cap, ref_fix(c_w1[j], c_src[j] + 8));
            }
            l_n[j] = 0;
            c_kind[j] = 0;
        }
        // ================================================ take pieces
        if (!exited || crem != 0 || srem != 0) {
            const uint32_t head = exited ? tail : lds_load((uint8_t*)lw(T, W_HEAD));
            compiler_fence();
            uint2 ent[KX];
#pragma unroll
            for (int j = 0; j < KX; ++j) ent[j] = ring_ld(T, tail + j);
            compiler_fence();
            const uint32_t F = crem ? cq : srem ? sdst : pos;   // every symbol before F is stored
            uint32_t k = 0;
            bool stop = false;
#pragma unroll
            for (int j = 0; j < KX; ++j) {
                if (!stop && crem == 0 && srem == 0) {
                    if (tail == head) {
                        stop = true;
                    } else {
                        uint2 e = ent[0];
#pragma unroll
                        for (int i = 1; i <= j; ++i) e = pick(e, ent[i], k == (uint32_t)i);
                        if (e.y & TOK_END) {
                            const uint32_t delta = (e.y >> 8) & 0x1fffffu;
                            bp::SegRes r;
                            r.nsym = e.x;
                            r.status = (int32_t)(int8_t)(e.y & 0xffu);
                            r.next = delta ? m + delta : 0xffffffffu;
                            r.pad = 0;
                            res[m] = r;
                            exited = !queue;
                            ++tail;
                            ++k;
                            worked = true;
                            stop = true;
                        } else if (e.y & (TOK_NEW | TOK_EXIT)) {
                            if (j == 0) {   // switches the slot: only with no piece pending
                                if (e.y & TOK_NEW) {
                                    m = e.x;
                                    slot(m);
                                    pos = 0;
                                } else {
                                    exited = true;
                                }
                                ++tail;
                                ++k;
                                worked = true;
                            }
                            stop = true;
                        } else if (e.y & TOK_STORED) {
                            srem = e.y & 0xffffu;
                            ssrc = pl + e.x;
                            sdst = pos;
                            pos += srem;
                            ++tail;
                            ++k;
                            worked = true;
                        } else {
                            const uint32_t nl = e.y & 7u, ml = (e.y >> 3) & 511u;
                            if (nl) {
                                l_dst[j] = pos;
                                l_val[j] = e.x;
                                l_n[j] = nl;
                                pos += nl;
                            }
                            if (ml) {
                                crem = ml;
                                cdist = (e.y >> 12) & 0xffffu;
                                cq = pos;
                                cpat_st = 0;
                                pos += ml;
                            }
                            ++tail;
                            ++k;
                            worked = true;
                        }
                    }
                }
                if (!stop && srem != 0) {
                    // 32 stored bytes (nothing past the payload's end is read)
                    const uint32_t kb = srem < 32 ? srem : 32u;
                    if (ssrc + 32 <= pl_end) {
                        c_w0[j] = *(const uint4_u*)ssrc;
                        c_w1[j] = *(const uint4_u*)(ssrc + 16);
                    } else {
                        uint32_t d[8] = {0, 0, 0, 0, 0, 0, 0, 0};
                        for (uint32_t q = 0; q < kb; ++q) d[q >> 2] |= (uint32_t)ssrc[q] << (8 * (q & 3));
                        c_w0[j] = make_uint4(d[0], d[1], d[2], d[3]);
                        c_w1[j] = make_uint4(d[4], d[5], d[6], d[7]);
                    }
                    c_kind[j] = CK_STORED;
                    c_dst[j] = sdst;
                    ssrc += kb;
                    sdst += kb;
                    srem -= kb;
                    worked = true;
                } else if (!stop && crem != 0) {
                    const uint32_t C = (cdist >= 16 && crem > 8) ? 16u : cdist >= 8 ? 8u : 0u;
                    if (C) {
                        const uint32_t n = crem < C ? crem : C;
                        const int32_t src = (int32_t)cq - (int32_t)cdist;
                        if (src + (int32_t)n <= (int32_t)F) {
                            uint4 w0 = make_uint4(0, 0, 0, 0), w1 = w0;
                            if (src + 8 > 0) w0 = *(const uint4_s*)(o + src);
                            if (C == 16 && src + 16 > 0) w1 = *(const uint4_s*)(o + src + 8);
                            c_w0[j] = w0;
                            c_w1[j] = w1;
                            c_src[j] = src;
                            c_kind[j] = CK_MATCH;
                            c_dst[j] = cq;
                            c_sz[j] = C;
                            cq += n;
                            crem -= n;
                            worked = true;
                        } else {
                            stop = true;
                        }
                    } else {
                        const uint32_t adv0 = 8 - 8 % cdist;
                        const uint32_t adv = adv0 < crem ? adv0 : crem;
                        if (cpat_st == 2) {
                            c_w0[j] = cpat;
                            c_kind[j] = CK_PAT;
                            c_dst[j] = cq;
                            cq += adv;
                            crem -= adv;
                            worked = true;
                        } else if (cpat_st == 0 && cq <= F) {
                            const int32_t src = (int32_t)cq - 8;
                            c_w0[j] = src + 8 > 0 ? *(const uint4_s*)(o + src) : make_uint4(0, 0, 0, 0);
                            c_src[j] = src;
                            c_kind[j] = CK_PATREQ;
                            c_sz[j] = cdist;   // the pattern's period
                            c_dst[j] = cq;
                            cpat_st = 1;
                            cq += adv;
                            crem -= adv;
                            worked = true;
                        } else {
                            stop = true;
                        }
                    }
                }
            }
            if (!exited || k) lds_store((uint8_t*)lw(T, W_TAIL), tail);
        }
        if (!__ballot(worked)) {
            L3_CNT(2);
            __builtin_amdgcn_s_sleep(BPMD3_ESLEEP);
        }
    }
    L3_FLUSH(4);
}

// ------------------------------------------------------------------- decoder
// SEG: segment mode (block-parallel inflate, bp.h): the "messages" are
// segment tasks; a lane starts at the task's bit, writes 16-bit symbols to
// the task's slot (no window or capacity rule of the message: matches may
// reach before the segment, the slot's end is SEG_FULL) and stops at the
// block boundary that is the message's next candidate (SEG_HANDOFF).
template <bool SEG>
__device__ __forceinline__ void decoder(uint8_t* T, bool valid, uint32_t m, const uint8_t* __restrict__ in,
                                        const uint64_t* __restrict__ in_off, const uint32_t* __restrict__ in_len,
                                        const uint32_t* __restrict__ out_cap, uint32_t raw,
                                        const uint32_t* __restrict__ mask_key, const uint32_t* __restrict__ hist_len,
                                        uint32_t hist_max, uint32_t n_msgs, const uint32_t* __restrict__ order,
                                        uint32_t* __restrict__ qctr, uint32_t s0,
                                        const bp::SegTask* __restrict__ tasks)
{
    const uint32_t tail = raw ? 0u : 4u;
    const int32_t full_status = SEG ? bp::SEG_FULL : raw ? ST_OK : ST_NEED_BUFFERS;
    // segment mode: payload bit of the view's first bit, the view's bits, and
    // the next candidate of the message (task index, bit, slots after it)
    uint32_t vbase = 0, vtot = 0, nk = 0, nk_bit = 0xffffffffu, nk_left = 0, nk_kind = 0;
    const uint8_t* pl = in;   // the segment's payload
    uint32_t pl_len = 0;
    auto next_cand = [&](uint32_t from, uint32_t left) {
        nk = 0;
        nk_bit = 0xffffffffu;
        nk_left = 0;
        nk_kind = bp::KIND_NONE;
        for (uint32_t j = 1; j <= left; ++j) {
            const bp::SegTask& c = tasks[from + j];
            if (c.kind != bp::KIND_NONE) {
                nk = from + j;
                nk_bit = c.bit;
                nk_left = left - j;
                nk_kind = c.kind;
                break;
            }
        }
    };
    // per-message state (set by begin())
    const uint8_t* A = in;
    uint32_t s = 0, n = 0, cap = 0, mk = 0, hist = 0;
    // bit reader: bb holds up to 64 bits; refills take 32-bit words from q
    // (a 16-byte block, shifted down as it is used), then from nx (the next
    // block, already in registers).  Blocks move nx <- sg <- memory only in
    // the loop's memory section, so decoding never waits on memory.
    uint4 q = make_uint4(0, 0, 0, 0), nx = q, sg = q;
    bool sg_ld = false;
    uint32_t blk = 3, qn = 4, sg_bi = 2;
    bool nx_used = false;
    uint64_t bb = 0;
    uint32_t nb = 0;
    int32_t tb = 0;   // stream bits not yet moved into bb
    auto refill = [&]() {   // branchless: in a wave some lane nearly always needs it
        const bool need = nb <= 32;
        const uint64_t add = (uint64_t)q.x << (nb & 63);
        bb |= need ? add : 0ull;
        nb += need ? 32u : 0u;
        tb -= need ? 32 : 0;
        q.x = need ? q.y : q.x;
        q.y = need ? q.z : q.y;
        q.z = need ? q.w : q.z;
        qn -= need ? 1u : 0u;
        const bool sw = qn == 0;
        q.x = sw ? nx.x : q.x;
        q.y = sw ? nx.y : q.y;
        q.z = sw ? nx.z : q.z;
        q.w = sw ? nx.w : q.w;
        qn = sw ? 4u : qn;
        nx_used = nx_used || sw;
    };
    // consume t <= 60 bits of the 64-bit window bb | q.x << nb (nb >= 33)
    auto drop_x = [&](uint32_t t) {
        const bool over = t > nb;
        const uint32_t r = (t - nb) & 31u;
        const uint64_t a = bb >> (t & 63u);
        const uint64_t b = (uint64_t)(q.x >> r);
        bb = over ? b : a;
        nb = over ? 32u - r : nb - t;
        tb -= over ? 32 : 0;
        q.x = over ? q.y : q.x;
        q.y = over ? q.z : q.y;
        q.z = over ? q.w : q.z;
        qn -= over ? 1u : 0u;
        const bool sw = qn == 0;
        q.x = sw ? nx.x : q.x;
        q.y = sw ? nx.y : q.y;
        q.z = sw ? nx.z : q.z;
        q.w = sw ? nx.w : q.w;
        qn = sw ? 4u : qn;
        nx_used = nx_used || sw;
    };
    auto drop = [&](uint32_t k) {
        bb >>= k;
        nb -= k;
    };
    uint32_t st = S_DONE;
    int32_t result = ST_OK;
    bool last = false, fin = true;   // fin: END token written
    uint32_t pos = 0, head = 0;
    Canon<15> tl, td;
    // the compact words of tl / td and whether they cover the whole code
    uint32_t WL[CKL], WD[CKD];
    bool wide = BPMD3_CKL == 0;
#pragma unroll
    for (int i = 0; i < CKL; ++i) WL[i] = 0;
#pragma unroll
    for (int i = 0; i < CKD; ++i) WD[i] = 0;
    Canon<7> tc;
    // header state
    uint32_t nlen = 0, ndist = 0, want = 0, have = 0, prev = 0;
    bool eob_seen = false, cl_empty = false;
    // stored block
    uint32_t srem = 0;
    bool sfull = false, sstarve = false;
    // work queue (qctr != null): a lane whose END token is out takes the next
    // message; its NEW token tells the expander which slot to write; a lane
    // that finds the queue empty sends EXIT
    uint32_t msg = m;
    bool send_new = false, send_exit = false, exhausted = qctr == nullptr;
#ifdef BPMD_PROF
    // per message / task (prof build): lifetime from begin() to its END token,
    // decoder iterations, and 4-byte stored-copy steps -> g_l3hprof[5-7]
    unsigned long long tk_t0_ = 0;
    uint32_t tk_it_ = 0, tk_sc_ = 0;
#endif
    const uint32_t first_slots = s0 + gridDim.x * WG_MSGS;
    // the bit reader over payload bytes [p, p + n) (+ the pmd tail)
    auto open_view = [&](const uint8_t* p, uint32_t nn) {
        n = nn;
        s = (uint32_t)((uintptr_t)p & 3);
        A = p - s;
        const uint4 b0w = issue_block(A, 0, s, n), b1w = issue_block(A, 1, s, n);
        q = finish_block(make_uint4(b0w.x ^ mk, b0w.y ^ mk, b0w.z ^ mk, b0w.w ^ mk), 0, s, n, tail);
        nx = finish_block(make_uint4(b1w.x ^ mk, b1w.y ^ mk, b1w.z ^ mk, b1w.w ^ mk), 1, s, n, tail);
        const uint32_t E_in = (s + n + 3) & ~3u;
        sg_ld = 32 < E_in;
        if (sg_ld) sg = *(const uint4*)(A + 32 - 4 * in_shift(32, E_in));
        blk = 3;
        qn = 4;
        sg_bi = 2;
        nx_used = false;
        bb = 0;
        nb = 0;
        tb = (int32_t)(8 * (s + n + tail));
        refill();
        refill();
    };
    auto begin = [&](uint32_t mm) {
        msg = mm;
#ifdef BPMD_PROF
        tk_t0_ = __builtin_amdgcn_s_memtime();
        tk_it_ = 0;
        tk_sc_ = 0;
#endif
        uint32_t byte0 = 0, bit0 = 0, kind = 0;
        bool skip = false;
        if (SEG) {
            // mm is a task: its message, first bit and slot
            const bp::SegTask tk = tasks[mm];
            skip = tk.kind == bp::KIND_NONE;
            kind = tk.kind;
            mm = skip ? 0u : tk.msg;
            byte0 = skip ? 0u : tk.bit >> 3;
            bit0 = skip ? 0u : tk.bit & 7u;
            cap = tk.sym_cap;
            next_cand(msg, skip ? 0u : tk.left);
            pl = in + in_off[mm];
            pl_len = in_len[mm];
        }
        if (!SEG) cap = out_cap[mm];
        {
            const uint8_t* p = in + in_off[mm] + byte0;
            const uint32_t s_ = (uint32_t)((uintptr_t)p & 3);
            // masked payloads (bpmd_read_batch): the dword at A + 4k holds payload
            // bytes 4k - s .. 4k - s + 3, masked with key bytes (j - s) % 4
            // (mask.ipp:38-59), so one rotation of the key unmasks every dword
            mk = mask_key ? __builtin_amdgcn_alignbit(mask_key[mm], mask_key[mm], 8u * ((0u - s_) & 3u)) : 0u;
            // context takeover (bpmd_inflate_takeover_batch): the hist bytes before
            // the slot are the window Beast's inflater keeps across messages
            hist = hist_len ? (hist_len[mm] < hist_max ? hist_len[mm] : hist_max) : 0u;
            open_view(p, in_len[mm] - byte0);
        }
        drop(8 * s + bit0);
        st = raw && n == 0 ? S_DONE : S_TYPE;
        result = raw && n == 0 ? ST_NEED_BUFFERS : ST_OK;
        if (SEG) {
            vtot = 8 * (s + n + tail);
            vbase = 8 * byte0 - 8 * s;
            // a stored candidate starts at its LEN field (byte aligned)
            st = skip ? S_DONE : kind == bp::KIND_STORED ? S_SHDR : st;
            result = skip ? bp::SEG_SKIP : result;
        }
        last = false;
        fin = false;
        pos = 0;
#pragma unroll
        for (int i = 0; i < 15; ++i) { tl.Q[i] = 0; td.Q[i] = 0; }
#pragma unroll
        for (int i = 0; i < CKL; ++i) WL[i] = 0;
#pragma unroll
        for (int i = 0; i < CKD; ++i) WD[i] = 0;
        tl.root = 9;
        td.root = 5;
#pragma unroll
        for (int i = 0; i < 7; ++i) tc.Q[i] = 0;
        tc.root = 1;
        srem = 0;
        if (SEG && kind == bp::KIND_STORED && !skip && nk_bit != 0xffffffffu) {
            // a stored block whose end is the next candidate's start (this
            // library's incompressible chunks; runs of Beast's stored blocks):
            // the resolve copies its bytes straight from the payload
            // (SEG_DIRECT), the lane decodes nothing.  The next candidate is a
            // dynamic or fixed header right at the end, or a stored block
            // whose header byte (BFINAL 0, type 0, padding) precedes its LEN.
            const uint8_t* pp = pl + byte0;
            const uint32_t L = (uint32_t)pp[0] | ((uint32_t)pp[1] << 8);
            const uint32_t NL = (uint32_t)pp[2] | ((uint32_t)pp[3] << 8);
            const uint32_t e = byte0 + 4 + L;   // the next block's first byte
            bool direct = (L ^ NL) == 0xffffu && e < pl_len;
            if (direct)
                direct = (nk_kind == bp::KIND_DYN || nk_kind == bp::KIND_FIXED)
                             ? nk_bit == 8 * e
                             : nk_kind == bp::KIND_STORED && nk_bit == 8 * e + 8 && (pl[e] & 7u) == 0;
            if (direct) {
                st = S_DONE;
                result = bp::SEG_DIRECT;
                pos = L;
            }
        }
    };
    // nx <- the staged block sg (unmasked, tail applied), and the next block
    // is staged (one 16-byte load)
    auto pipe = [&]() {
        // only a block that holds the payload's end needs finish_in's
        // shift and tail work: a wave-uniform test keeps it off the rest
        if (__ballot(sg_bi * 16 + 16 > s + n)) nx = finish_in(sg, sg_ld, sg_bi, s, n, tail, mk);
        else nx = make_uint4(sg.x ^ mk, sg.y ^ mk, sg.z ^ mk, sg.w ^ mk);
        const uint32_t b0 = blk * 16, E = (s + n + 3) & ~3u;
        sg_ld = b0 < E;
        if (sg_ld) sg = *(const uint4*)(A + b0 - 4 * in_shift(b0, E));
        sg_bi = blk++;
        nx_used = false;
    };
    // One token of a Huffman block: up to KLIT leading literals and a main
    // symbol (see data_step's body).  Called once per iteration, and a second
    // time for the lanes whose next input block is still unused.
    auto data_step = [&](uint32_t& enl, uint32_t& elit, uint32_t& emlen, uint32_t& edist) {
        // Up to KLIT symbols per iteration: while there is room for them
        // (input for KLIT - 1 literals plus a whole token, output for KLIT
        // literals, so no event can occur among them) leading literals are
        // taken directly; the first other symbol -- or, out of room, the
        // first symbol of any kind -- is the iteration's main token, handled
        // with the reference's checks below.  The KLIT code lengths come from
        // registers, so their KLIT symbol lookups go out together.
        refill();   // nb >= 33: with q.x, a 64-bit window
        const uint64_t w = nb >= 64 ? bb : (bb | ((uint64_t)q.x << nb));
        const bool multi = (tb + (int32_t)nb) >= 48 + 15 * (KLIT - 1) && pos + KLIT <= cap;
        uint32_t kp[KLIT + 1], kc[KLIT], kL[KLIT], kx[KLIT];
        bool kinv[KLIT];
        kp[0] = 0;
        // (a wave-uniform choice: the full search only while some lane's
        // tables have more distinct lengths than the compact words hold)
        const bool any_wide = BPMD3_CKL == 0 || __ballot(wide) != 0;
#pragma unroll
        for (int k = 0; k < KLIT; ++k) {
            kc[k] = rev15(w >> kp[k]);
            const Sym y = any_wide ? canon_decode<15>(tl.Q, kc[k]) : canon_decode<CKL, 15>(WL, kc[k]);
            kL[k] = y.L;
            kx[k] = y.idx;
            kinv[k] = y.inval;
            kp[k + 1] = kp[k] + (y.inval ? 15u : y.L);
        }
        uint32_t kle[KLIT], ksb[KLIT];
#pragma unroll
        for (int k = 0; k < KLIT; ++k) {
            kle[k] = *(const uint16_t*)lb(T, O_LE + 2 * kL[k]);
            ksb[k] = *lb(T, O_LIT + kx[k]);
        }
        uint32_t ks[KLIT];
#pragma unroll
        for (int k = 0; k < KLIT; ++k) ks[k] = ksb[k] + (kx[k] >= kle[k] ? 256u : 0u);
        // leading literals taken directly
        uint32_t nlit = 0, lbytes = 0;
#pragma unroll
        for (int k = 0; k < KLIT; ++k) {
            const bool take = multi && nlit == (uint32_t)k && !kinv[k] && ks[k] < 256;
            lbytes |= take ? ks[k] << (8 * k) : 0u;
            nlit += take ? 1u : 0u;
        }
        uint32_t lit_bits = 0;
#pragma unroll
        for (int k = 1; k <= KLIT; ++k) lit_bits = nlit == (uint32_t)k ? kp[k] : lit_bits;
        enl = nlit;
        elit = lbytes;
        pos += nlit;
        // the main token: symbol nlit (none when all KLIT were literals)
        uint32_t c15 = kc[0], L = kL[0], sym = ks[0];
        bool kinv_m = kinv[0];
#pragma unroll
        for (int k = 1; k < KLIT; ++k) {
            const bool here = nlit == (uint32_t)k;
            c15 = here ? kc[k] : c15;
            L = here ? kL[k] : L;
            sym = here ? ks[k] : sym;
            kinv_m = here ? kinv[k] : kinv_m;
        }
        const bool inval = kinv_m || sym >= 286;
        drop_x(lit_bits);
        // The main token, for the lanes that have one (nlit < KLIT), without
        // divergent branches: every outcome is a select (a branch costs the
        // wave its exec-mask instructions whether or not a lane takes it).
        const bool mt = nlit < (uint32_t)KLIT;
        refill();   // nb >= 33 again: the main token's <= 48 bits are in the window
        const uint64_t w2 = nb >= 64 ? bb : (bb | ((uint64_t)q.x << nb));
        const int32_t avail = tb + (int32_t)nb;
        Sym y;
        y.L = L;
        y.idx = 0;
        y.inval = inval;
        // the fill rule only bites within 48 bits of the end of the input:
        // a wave-uniform branch keeps its two canonical searches off the
        // common path
        const bool near_end = __ballot(mt && avail < 48) != 0;
        uint32_t need_l = 0;
        if (near_end && mt && avail < 48) need_l = canon_need<15>(tl, y, c15);
        const bool is_len = !inval && sym > 256;
        const uint32_t li = is_len ? sym - 257 : 0u;
        const uint32_t xl = (li < 8 || li == 28) ? 0u : ((li - 4) >> 2);
        uint32_t len = li < 8 ? li + 3 : (li == 28 ? 258u : (((4u + (li & 3)) << xl) + 3));
        len += (uint32_t)(w2 >> L) & lowmask(xl);
        const uint32_t used = L + (is_len ? xl : 0u);
        const uint32_t d15 = rev15(w2 >> used);
        const Sym yd = any_wide ? canon_decode<15>(td.Q, d15) : canon_decode<CKD, 15>(WD, d15);
        const uint32_t Ld = yd.L;
        const uint32_t dsym = *lb(T, O_DST + yd.idx);
        const bool invd = yd.inval || dsym >= 30;
        const uint32_t xd = dsym < 4 ? 0u : (dsym >> 1) - 1;
        uint32_t dist = dsym < 4 ? dsym + 1 : (((2u + (dsym & 1)) << xd) + 1);
        dist += (uint32_t)(w2 >> (used + Ld)) & lowmask(xd);
        uint32_t need_d = 0;
        if (near_end && mt && avail < 48 && is_len) need_d = canon_need<15>(td, yd, d15);
        // event, in the reference's order: 0 token, 1 eob, 2 starved, 3 error
        const bool s_m1 = (int32_t)used > avail || (int32_t)(used + need_d) > avail;
        const bool s_m2 = (int32_t)(used + Ld + xd) > avail;
        const uint32_t ev = (int32_t)need_l > avail ? 2u
                            : inval               ? 3u
                            : sym == 256          ? 1u
                            : !is_len             ? 0u
                            : s_m1                ? 2u
                            : invd                ? 3u
                            : s_m2                ? 2u
                                                  : 0u;
        const int32_t err = inval ? ST_INVALID_LITERAL_LENGTH : ST_INVALID_DISTANCE_CODE;
        const bool is_match = ev == 0 && is_len;
        drop_x(mt && ev < 2 ? (is_match ? used + Ld + xd : used) : 0u);
        // output checks in the reference's order (inflate_stream.ipp:475-514)
        const bool tok = mt && ev == 0;
        const bool c_raw = !SEG && raw && pos >= cap;
        const bool c_dist = !SEG && is_match && dist > pos + hist;
        const bool c_full = pos >= cap;
        uint32_t olen = is_match ? len : 1u;
        const bool c_trunc = pos + olen > cap;
        olen = c_trunc ? cap - pos : olen;
        const bool emit = tok && !c_raw && !c_dist && !c_full;
        const bool stop_full = tok && (c_raw || (!c_dist && (c_full || c_trunc)));
        const bool stop_dist = tok && !c_raw && c_dist;
        result = stop_full ? full_status : stop_dist ? ST_INVALID_DISTANCE : (mt && ev == 3) ? err : result;
        st = (stop_full || stop_dist || (mt && ev >= 2)) ? (uint32_t)S_DONE : (mt && ev == 1) ? (uint32_t)S_TYPE : st;
        emlen = emit && is_match ? olen : 0u;
        edist = emit && is_match ? dist : 0u;
        enl = emit && !is_match ? 1u : enl;
        elit = emit && !is_match ? sym : elit;
        pos += emit ? olen : 0u;
    };
    if (valid) begin(m);
    L3_DECL;
    L3_LAPDECL;
#ifdef BPMD_PROF
    unsigned long long l3x_[4] = {0, 0, 0, 0}, l3dyn_ = 0, l3h_[5] = {0, 0, 0, 0, 0};
#endif

    for (;;) {
        if (!exhausted) {
            const uint64_t idle = __ballot(fin && !send_new && !exhausted);
            // take new messages when a quarter of the wave waits or nothing else runs
            if (idle && (__builtin_popcountll(idle) * 4 >= 64 || __ballot(!fin) == 0)) {
                const unsigned leader = (unsigned)__builtin_ctzll(idle);
                uint32_t base = 0;
                if ((threadIdx.x & 63u) == leader) base = atomicAdd(qctr, (uint32_t)__builtin_popcountll(idle));
                base = __shfl(base, (int)leader);
                if ((idle >> (threadIdx.x & 63u)) & 1) {
                    const uint32_t k =
                        first_slots + base + (uint32_t)__builtin_popcountll(idle & ((1ull << (threadIdx.x & 63u)) - 1ull));
                    if (k < n_msgs) {
                        // the NEW token goes out first; the message begins once it is
                        // in the ring (its header may need the ring's LDS)
                        msg = order ? order[k] : k;
                        send_new = true;
                    } else {
                        exhausted = true;
                        send_exit = true;
                    }
                }
            }
        }
        if (!__ballot(!fin || send_new || send_exit)) break;
        L3_LAP(3);
        L3_CNT(1);
#ifdef BPMD_PROF
        if (__ballot(st != S_DATA && st != S_DONE && st != S_SCOPY && st != S_TYPE)) L3_CNT(3);
#endif
        // ---- the input pipeline (the only global memory the decoder touches)
        if (nx_used) pipe();
        const uint32_t taken = lds_load((uint8_t*)lw(T, W_TAIL));
        compiler_fence();
        const bool room = head - taken < RING;
        const bool ring_empty = head == taken;
#ifdef BPMD_PROF
        // lane states per iteration: [12] data lanes blocked by a full ring,
        // [13] data lanes with room, [14] finished lanes, [15] header lanes
        l3x_[0] += __builtin_popcountll(__ballot(st == S_DATA && !room));
        l3x_[1] += __builtin_popcountll(__ballot(st == S_DATA && room));
        l3x_[2] += __builtin_popcountll(__ballot(fin && !send_new));
        l3x_[3] += __builtin_popcountll(__ballot(st != S_DATA && st != S_DONE));
        l3dyn_ += __builtin_popcountll(__ballot(st == S_DYN && !ring_empty));   // [7]
#endif
        // this iteration's token
        uint32_t enl = 0, elit = 0, emlen = 0, edist = 0, estored = 0;
        const uint32_t st0 = st;
        const uint32_t head0 = head;
        L3_LAP(0);
        if (st == S_DATA && room) data_step(enl, elit, emlen, edist);


        L3_LAP(1);
        // ======================================= block headers, stored
        // (one wave-uniform branch skips the whole section while every lane
        // is in a block's data or finished: a wave issues every instruction
        // of the section's per-state tests otherwise, exec-mask work included)
        if (__ballot(st0 != S_DATA && st0 != S_DONE)) {
        L3_HSTART();
        if (SEG && st == S_TYPE && st0 == S_TYPE && !last) {
            // a block boundary: the next candidate's header starts here, or
            // candidates this segment has passed (not headers) are dropped
            const uint32_t cur = vbase + (uint32_t)((int32_t)vtot - (tb + (int32_t)nb));
            while (nk_bit < cur) next_cand(nk, nk_left);
            if (nk_bit == cur && (nk_kind == bp::KIND_DYN || nk_kind == bp::KIND_FIXED)) {
                result = bp::SEG_HANDOFF;
                st = S_DONE;
            }
        }
        if (st == S_TYPE && st0 == S_TYPE) {
            if (last) {
                result = ST_END_OF_STREAM;
                st = S_DONE;
            } else {
                refill();
                const int32_t avail = tb + (int32_t)nb;
                if (avail < 3) {
                    st = S_DONE;
                } else {
                    const uint32_t h = (uint32_t)bb & 7u;
                    drop(3);
                    last = (h & 1) != 0;
                    const uint32_t type = h >> 1;
                    if (type == 0) {
                        st = S_SHDR;
                    } else if (type == 1) {
                        // fixed tables (inflate_stream.ipp:865-930): canonical
                        // order is 256-279 | 0-143 280-287 | 144-255, distances 0-31
#pragma unroll 1
                        for (int k = 0; k < 20; ++k) {
#pragma unroll
                            for (int j = 0; j < 4; ++j) {
                                const int i = 16 * k + 4 * j;
                                const int v = i < 24 ? i : i < 168 ? i - 24 : i < 176 ? i - 144 : i < 288 ? i - 32 : i - 288;
                                *lw(T, 4 * k + j) = (uint32_t)v * 0x01010101u + 0x03020100u;
                            }
                        }
                        // litend: LE[7] = 0, LE[8] = 168, LE[9] = 288
                        *lw(T, W_LE + 3) = 0u << 16;
                        *lw(T, W_LE + 4) = 168u | (288u << 16);
                        // make_canon of the fixed counts (7: 24, 8: 152, 9: 112; distances 5: 32)
                        constexpr uint32_t kFixL[15] = {0x00000800u, 0x00001000u, 0x00001800u, 0x00002000u,
                                                        0x00002800u, 0x00003000u, 0x0c003818u, 0x320040b0u,
                                                        0x40004920u, 0x40005120u, 0x40005920u, 0x40006120u,
                                                        0x40006920u, 0x40007120u, 0x40007920u};
                        constexpr uint32_t kFixD[15] = {0x00000800u, 0x00001000u, 0x00001800u, 0x00002000u,
                                                        0x40002820u, 0x40003020u, 0x40003820u, 0x40004020u,
                                                        0x40004820u, 0x40005020u, 0x40005820u, 0x40006020u,
                                                        0x40006820u, 0x40007020u, 0x40007820u};
#pragma unroll
                        for (int i = 0; i < 15; ++i) {
                            tl.Q[i] = kFixL[i];
                            td.Q[i] = kFixD[i];
                        }
                        // fixed: literal/length lengths 7, 8, 9; distances 5
#pragma unroll
                        for (int i = 0; i < CKL; ++i) WL[i] = i < 3 ? kFixL[6 + i] : 0u;
#pragma unroll
                        for (int i = 0; i < CKD; ++i) WD[i] = i < 1 ? kFixD[4] : 0u;
                        wide = BPMD3_CKL == 0;
                        tl.root = 9;
                        td.root = 5;
                        st = S_DATA;
                    } else if (type == 2) {
                        st = S_DYN;
                    } else {
                        result = ST_INVALID_BLOCK_TYPE;
                        st = S_DONE;
                    }
                }
            }
        }
        if (st == S_SHDR) {
            // STORED (inflate_stream.ipp:184-204)
            refill();
            int32_t avail = tb + (int32_t)nb;
            drop((uint32_t)avail & 7u);
            avail &= ~7;
            refill();
            uint32_t cur = 0;
            if (SEG) {
                // the next candidate is this stored block (its LEN field)
                cur = vbase + (uint32_t)((int32_t)vtot - avail);
                // (not for a final stored block: the candidate's segment would
                // start without its BFINAL bit and miss the end of the stream)
                if (nk_bit == cur && nk_kind == bp::KIND_STORED && !last) {
                    result = bp::SEG_HANDOFF;
                    st = S_DONE;
                }
            }
            if (st != S_SHDR) {
            } else if (avail < 32) {
                st = S_DONE;
            } else {
                const uint32_t v = (uint32_t)bb & 0xffffu, nv = (uint32_t)(bb >> 16) & 0xffffu;
                if (v != (nv ^ 0xffffu)) {
                    result = ST_INVALID_STORED_LENGTH;
                    st = S_DONE;
                } else {
                    drop(32);
                    avail -= 32;
                    const uint32_t have_b = (uint32_t)avail >> 3;
                    uint32_t nc = v < have_b ? v : have_b;
                    sfull = false;
                    if (pos + nc > cap) {
                        nc = cap - pos;
                        sfull = true;
                    }
                    sstarve = nc < v;
                    srem = nc;
                    st = S_SCOPY;
                    if (SEG && room && (cur >> 3) + 4 + nc <= pl_len) {
                        // segment mode: the expander copies the block's bytes
                        // from the input (one token); the reader moves past
                        // them.  (Data reaching into the pmd tail goes the
                        // byte way: the tail is not in memory.)
                        const uint32_t from = (cur >> 3) + 4;   // payload byte of the data
                        estored = nc;
                        elit = from;
                        pos += nc;
                        srem = 0;
                        if (sfull) {
                            result = full_status;
                            st = S_DONE;
                        } else if (sstarve) {
                            st = S_DONE;
                        } else {
                            open_view(pl + from + nc, pl_len - from - nc);
                            drop(8 * s);
                            vtot = 8 * (s + n + tail);
                            vbase = 8 * (from + nc) - 8 * s;
                            st = S_TYPE;
                        }
                    }
                }
            }
        }
        if (st == S_SCOPY) {
            // COPY (inflate_stream.ipp:206-220): up to 4 bytes per iteration,
            // as a literal entry for the expander
            if (srem && room) {
#ifdef BPMD_PROF
                ++tk_sc_;
#endif
                refill();
                const uint32_t k = srem < 4 ? srem : 4u;
                elit = (uint32_t)bb;
                enl = k;
                drop(8 * k);
                pos += k;
                srem -= k;
            }
            if (srem == 0) {
                if (sfull) {
                    result = full_status;
                    st = S_DONE;
                } else if (sstarve) {
                    st = S_DONE;
                } else {
                    st = S_TYPE;
                }
            }
        }
        // ================================================== D. dynamic header
        // the code-length scratch shares LDS with the token ring: a dynamic
        // header starts once the expander has taken every entry
        L3_HLAP(0);
        if (st == S_DYN && ring_empty) {
            // TABLE / LENLENS (inflate_stream.ipp:222-262)
            refill();
            int32_t avail = tb + (int32_t)nb;
            if (avail < 14) {
                st = S_DONE;
            } else {
                nlen = ((uint32_t)bb & 31u) + 257;
                ndist = ((uint32_t)(bb >> 5) & 31u) + 1;
                const uint32_t ncode = ((uint32_t)(bb >> 10) & 15u) + 4;
                drop(14);
                avail -= 14;
                if (nlen > 286 || ndist > 30) {
                    result = ST_TOO_MANY_SYMBOLS;
                    st = S_DONE;
                } else if (avail < (int32_t)(3 * ncode)) {
                    st = S_DONE;
                } else {
                    // the 19 code-length-code lengths, 3 bits each by symbol
                    uint64_t clp = 0;
                    refill();
#pragma unroll
                    for (int i = 0; i < 10; ++i)
                        clp |= (uint64_t)((uint32_t)i < ncode ? ((uint32_t)(bb >> (3 * i)) & 7u) : 0u)
                               << (3 * kClenOrder2[i]);
                    drop(3 * (ncode < 10 ? ncode : 10u));
                    refill();
#pragma unroll
                    for (int i = 10; i < 19; ++i)
                        clp |= (uint64_t)((uint32_t)i < ncode ? ((uint32_t)(bb >> (3 * (i - 10))) & 7u) : 0u)
                               << (3 * kClenOrder2[i]);
                    drop(3 * (ncode > 10 ? ncode - 10 : 0u));
                    // code-length code (inflate_stream.ipp:249-262)
                    uint64_t acc = 0;
#pragma unroll
                    for (int i = 0; i < 19; ++i) acc += 1ull << (5 * ((clp >> (3 * i)) & 7u));
                    uint32_t c[16];
#pragma unroll
                    for (int l = 0; l < 16; ++l) c[l] = (l >= 1 && l <= 7) ? (uint32_t)(acc >> (5 * l)) & 31u : 0u;
                    const int e = make_canon<7>(c, 7, 0, tc);
                    cl_empty = c[1] + c[2] + c[3] + c[4] + c[5] + c[6] + c[7] == 0;
                    if (e) {
                        result = e;
                        st = S_DONE;
                    } else {
                        uint64_t offs = 0;   // first canonical index per length, 5 bits each
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
                            offs += 1ull << (5 * l);
                            if (l) *lb(T, O_CLS + at) = (uint8_t)i;
                        }
#pragma unroll
                        for (int k = 0; k < 40; ++k) *lw(T, W_NIB + k) = 0u;
#pragma unroll
                        for (int k = 0; k < 16; ++k) *lw(T, W_HIST + k) = 0u;
                        want = nlen + ndist;
                        have = 0;
                        prev = 0;
                        eob_seen = false;
                        st = S_PASS1;
                    }
                }
            }
        }
        L3_HLAP(1);
#pragma unroll
        for (int kc = 0; kc < KCL; ++kc) {
            if (st != S_PASS1 || st0 != S_PASS1) break;
                // CODELENS (inflate_stream.ipp:264-327), up to KCL symbols per iteration
                refill();
                const int32_t avail = tb + (int32_t)nb;
                uint32_t L = 1, csym = 0;
                if (!cl_empty) {
                    const uint32_t c7 = __builtin_bitreverse32((uint32_t)bb) >> 25;
                    const Sym yc = canon_decode<7>(tc.Q, c7);
                    L = yc.L;
                    csym = *lb(T, O_CLS + (yc.idx < 19 ? yc.idx : 0u));
                }
                if (avail < (int32_t)tc.root) {
                    st = S_DONE;
                } else {
                    uint32_t val = csym, rep = 1, used = L;
                    bool ok = true;
                    if (csym >= 16) {
                        const uint32_t xb = csym == 16 ? 2u : (csym == 17 ? 3u : 7u);
                        if (avail < (int32_t)(L + xb)) {
                            st = S_DONE;
                            ok = false;
                        } else {
                            const uint32_t x = (uint32_t)(bb >> L) & lowmask(xb);
                            used = L + xb;
                            if (csym == 16) {
                                if (have == 0) {
                                    result = ST_INVALID_BIT_LENGTH_REPEAT;
                                    st = S_DONE;
                                    ok = false;
                                }
                                val = prev;
                                rep = 3 + x;
                            } else {
                                val = 0;
                                rep = (csym == 17 ? 3u : 11u) + x;
                            }
                            if (ok && have + rep > want) {
                                result = ST_INVALID_BIT_LENGTH_REPEAT;
                                st = S_DONE;
                                ok = false;
                            }
                        }
                    }
                    if (ok) {
                        drop(used);
                        if (val) {
                            const uint32_t a = have, b = have + rep;
                            const uint64_t pat = ((uint64_t)val * 0x1111111111111111ull) & ((1ull << (4 * rep)) - 1);
                            const uint64_t v = pat << ((a & 7) * 4);
                            __hip_atomic_fetch_or(lw(T, W_NIB + (a >> 3)), (uint32_t)v, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_WORKGROUP);
                            if ((uint32_t)(v >> 32))
                                __hip_atomic_fetch_or(lw(T, W_NIB + (a >> 3) + 1), (uint32_t)(v >> 32), __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_WORKGROUP);
                            const uint32_t e_l = b < nlen ? b : nlen;
                            const uint32_t nl = e_l > a ? e_l - a : 0u;
                            const uint32_t e_o = b < 256 ? b : 256u;
                            const uint32_t nlo = e_o > a ? e_o - a : 0u;
                            const uint32_t s_d = a > nlen ? a : nlen;
                            const uint32_t nd = b > s_d ? b - s_d : 0u;
                            __hip_atomic_fetch_add(lw(T, W_HIST + val), nl | (nlo << 10) | (nd << 20), __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_WORKGROUP);
                            if (a <= 256 && 256 < b) eob_seen = true;
                        }
                        prev = val;
                        have += rep;
                        if (have == want) st = S_BUILD;
                    }
                }
        }
        L3_HLAP(2);
        if (st == S_BUILD) {
            if (!eob_seen) {
                result = ST_MISSING_EOB;
                st = S_DONE;
            } else {
                uint32_t h[16];
#pragma unroll
                for (int k = 0; k < 16; ++k) h[k] = *lw(T, W_HIST + k);
                uint32_t c[16];
                c[0] = 0;
#pragma unroll
                for (int l = 1; l < 16; ++l) c[l] = h[l] & 0x3ffu;
                int e = make_canon<15>(c, 9, 1, tl);
                if (!e) {
#pragma unroll
                    for (int l = 1; l < 16; ++l) c[l] = (h[l] >> 20) & 0x3ffu;
                    e = make_canon<15>(c, 6, 2, td);
                }
                if (!e && BPMD3_CKL) {
                    const bool okl = compact_canon<15, CKL>(tl.Q, WL);
                    const bool okd = compact_canon<15, CKD>(td.Q, WD);
                    wide = !(okl && okd);
                }
                if (e) {
                    result = e;
                    st = S_DONE;
                } else {
                    // litend (first canonical index past the literals of each length)
                    // and the placement cursors (first index of each length)
                    uint32_t cl_ = 0, cd_ = 0;
#pragma unroll
                    for (int l = 0; l < 16; l += 2) {
                        const uint32_t a0 = l ? h[l] : 0u, a1 = h[l + 1];
                        const uint32_t le0 = cl_ + ((a0 >> 10) & 0x3ffu);
                        *lw(T, W_HIST + l) = cl_ | (cd_ << 16);
                        cl_ += a0 & 0x3ffu;
                        cd_ += (a0 >> 20) & 0x3ffu;
                        const uint32_t le1 = cl_ + ((a1 >> 10) & 0x3ffu);
                        *lw(T, W_HIST + l + 1) = cl_ | (cd_ << 16);
                        cl_ += a1 & 0x3ffu;
                        cd_ += (a1 >> 20) & 0x3ffu;
                        *lw(T, W_LE + (l >> 1)) = le0 | (le1 << 16);
                    }
                    have = 0;
                    st = S_PASS2;
                }
            }
        }
        L3_HLAP(3);
        if (st == S_PASS2) {
            // place symbols in canonical order (inflate_stream.ipp:632-640)
#pragma unroll
            for (uint32_t h8 = 0; h8 < KNIB; h8 += 8) {
                const uint32_t w = *lw(T, W_NIB + ((have + h8) >> 3));
                uint32_t olds[8];
                // all fetch-adds first (no branch between them), then the
                // placements: one LDS round trip for the eight
#pragma unroll
                for (uint32_t k = 0; k < 8; ++k) {
                    const uint32_t i = have + h8 + k;
                    const uint32_t l = (w >> (4 * k)) & 15u;
                    const uint32_t inc = (l && i < want) ? (i < nlen ? 1u : 0x10000u) : 0u;
                    olds[k] = __hip_atomic_fetch_add(lw(T, W_HIST + l), inc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
#pragma unroll
                for (uint32_t k = 0; k < 8; ++k) {
                    const uint32_t i = have + h8 + k;
                    const uint32_t l = (w >> (4 * k)) & 15u;
                    if (l && i < want) {
                        if (i < nlen) *lb(T, O_LIT + (olds[k] & 0xffffu)) = (uint8_t)i;
                        else *lb(T, O_DST + (olds[k] >> 16)) = (uint8_t)(i - nlen);
                    }
                }
            }
            have += KNIB;
            if (have >= want) st = S_DATA;
        }

        L3_HLAP(4);
        }   // block headers, stored
        L3_LAP(2);
        // ---- publish the token (entry first, then head)
        // (selects rather than an if-chain: one predicated store, one head store)
        {
            const bool ctl = send_new || send_exit;       // NEW / EXIT (work queue)
            const bool data = !ctl && (enl || emlen || estored);   // produced only with room
            const bool endt = !ctl && !data && st == S_DONE && !fin;
            const bool adv = room && (ctl || data || endt);
            const uint32_t hand =
                SEG && (result == bp::SEG_HANDOFF || result == bp::SEG_DIRECT) ? (nk - msg) << 8 : 0u;
            const uint2 ent = ctl    ? make_uint2(msg, send_new ? TOK_NEW : TOK_EXIT)
                              : data ? make_uint2(elit, estored ? (TOK_STORED | estored)
                                                                : (enl | (emlen << 3) | (edist << 12)))
                                     : make_uint2(pos, TOK_END | hand | ((uint32_t)result & 0xffu));
            if (adv) ring_st(T, head, ent);
            compiler_fence();
            head += adv ? 1u : 0u;
            lds_store((uint8_t*)lw(T, W_HEAD), head);
            fin = fin || (adv && endt);
#ifdef BPMD_PROF
            ++tk_it_;
            if (adv && endt) {
                // low 24 bits: the task (17 bits) and its result (7 bits)
                const unsigned long long id = (msg & 0x1ffffu) | (((uint32_t)result & 0x7fu) << 17);
                atomicMax(&g_l3hprof[5], ((__builtin_amdgcn_s_memtime() - tk_t0_) << 24) | id);
                atomicMax(&g_l3hprof[6], ((unsigned long long)tk_it_ << 24) | id);
                atomicAdd(&g_l3hprof[7], (unsigned long long)tk_sc_);
            }
#endif
            if (adv && ctl) {
                if (send_new) begin(msg);
                send_new = false;
                send_exit = false;
            }
        }
        // ---- a second token for the lanes still in the same Huffman block
        // with room in the ring and their next input block unused (so this
        // step's refills cannot reach a block that is not loaded yet): the
        // loop's fixed work -- input pipeline, ring tail, header test,
        // publish and the wave's exit tests -- is then paid once per two
        // tokens (about half of the data lanes take it; a
        // third step, or refilling the input block first, measured neutral).
#pragma unroll
        for (int xs = 0; xs < BPMD3_XSTEPS; ++xs) {
            if (BPMD3_XPIPE && nx_used && st0 == S_DATA && st == S_DATA) pipe();
            if (!__ballot(st0 == S_DATA && st == S_DATA && !nx_used && head - taken < RING)) break;
            uint32_t enl2 = 0, elit2 = 0, emlen2 = 0, edist2 = 0;
            if (st0 == S_DATA && st == S_DATA && !nx_used && head - taken < RING)
                data_step(enl2, elit2, emlen2, edist2);
            const bool adv2 = enl2 != 0 || emlen2 != 0;
            if (adv2) ring_st(T, head, make_uint2(elit2, enl2 | (emlen2 << 3) | (edist2 << 12)));
            compiler_fence();
            head += adv2 ? 1u : 0u;
            lds_store((uint8_t*)lw(T, W_HEAD), head);
        }
        // blocked on a full ring in every lane: leave the SIMD to the expander
        if (!__ballot(head != head0 || st != st0 || (st != S_DATA && st != S_SCOPY && st != S_DONE))) {
            L3_CNT(2);
            __builtin_amdgcn_s_sleep(1);
        }
    }
    L3_FLUSH(0);
    L3_LAPFLUSH();
#ifdef BPMD_PROF
    if ((threadIdx.x & 63) == 0)
    {
        for (int i = 0; i < 4; ++i) atomicAdd(&g_l3prof[12 + i], l3x_[i]);
        atomicAdd(&g_l3prof[7], l3dyn_);
    }
#endif
}

// A workgroup is one decoder wave and one expander wave over 64 messages;
// four workgroups per CU (WG_MSGS).  (One workgroup of 4 decoders + 4
// expanders per CU, which pins a decoder and an expander to every SIMD,
// measured slower: 117 vs 130 GiB/s on C2.)
__global__ void __launch_bounds__(128, 2)
inflate_lane3_kernel(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                     const uint32_t* __restrict__ in_len, uint32_t n_msgs, uint8_t* __restrict__ out,
                     const uint64_t* __restrict__ out_off, const uint32_t* __restrict__ out_cap,
                     uint32_t* __restrict__ out_len, int32_t* __restrict__ status, uint32_t raw,
                     const uint32_t* __restrict__ mask_key, const uint32_t* __restrict__ hist_len, uint32_t hist_max,
                     uint32_t max_in, const uint32_t* __restrict__ order, uint32_t* __restrict__ qctr,
                     const uint32_t* __restrict__ skip)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const unsigned lane = threadIdx.x & 63u;
    const bool is_decoder = threadIdx.x < 64;
    uint8_t* T = lane_area(smem, lane);
    // skip: the first *skip entries of `order` belong to the wave kernel (the
    // long payloads of a work-queue batch, pmd_capi.hip inflate_impl)
    const uint32_t s0 = skip ? *skip : 0u;
    // first message: slot s0 + blockIdx.x * 64 + lane (of `order` when given)
    const uint32_t j = s0 + blockIdx.x * WG_MSGS + lane;
    bool valid = j < n_msgs;
    const uint32_t m = valid ? (order ? order[j] : j) : 0u;
    // max_in != 0: only payloads of at most max_in bytes (the rest go to the
    // wave kernel, see inflate_impl in pmd_capi.hip)
    if (valid && max_in && in_len[m] > max_in) valid = false;
    if (is_decoder) {
        *lw(T, W_HEAD) = 0u;
        *lw(T, W_TAIL) = 0u;
    }
    __syncthreads();
    if (is_decoder) {
        if (BPMD3_DPRIO) __builtin_amdgcn_s_setprio(BPMD3_DPRIO);   // the decoder sets the pace
        decoder<false>(T, valid, m, in, in_off, in_len, out_cap, raw, mask_key, hist_len, hist_max, n_msgs, order, qctr,
                       s0, nullptr);
    } else {
        expander(T, valid, m, out, out_off, out_cap, out_len, status, hist_len, hist_max, qctr != nullptr);
    }
}

// Segment mode (block-parallel inflate, pmd_inflate_bp.hip): the same
// decoder / expander pair over segment tasks.
__global__ void __launch_bounds__(128, 2)
inflate_lane3_seg_kernel(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                         const uint32_t* __restrict__ in_len, uint32_t n_tasks, const bp::SegTask* __restrict__ tasks,
                         uint16_t* __restrict__ sym, bp::SegRes* __restrict__ res, uint32_t raw,
                         uint32_t* __restrict__ qctr, const uint32_t* __restrict__ n_dev)
{
    // n_dev: the device-side task count (the block-parallel driver sizes
    // nothing on the host); n_tasks bounds it
    if (n_dev && *n_dev < n_tasks) n_tasks = *n_dev;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const unsigned lane = threadIdx.x & 63u;
    const bool is_decoder = threadIdx.x < 64;
    uint8_t* T = lane_area(smem, lane);
    const uint32_t j = blockIdx.x * WG_MSGS + lane;
    const bool valid = j < n_tasks;
    if (is_decoder) {
        *lw(T, W_HEAD) = 0u;
        *lw(T, W_TAIL) = 0u;
    }
    __syncthreads();
    if (is_decoder) {
        if (BPMD3_DPRIO) __builtin_amdgcn_s_setprio(BPMD3_DPRIO);
        decoder<true>(T, valid, valid ? j : 0u, in, in_off, in_len, nullptr, raw, nullptr, nullptr, 0u, n_tasks, nullptr,
                      qctr, 0u, tasks);
    } else {
        expander_seg(T, valid, valid ? j : 0u, sym, tasks, res, qctr != nullptr, in, in_off, in_len);
    }
}

}  // namespace lp3
}  // namespace bpmd

extern "C" int bpmd_internal_inflate_lane3_seg(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                                               uint32_t n_tasks, const void* tasks, uint16_t* sym, void* res,
                                               uint32_t raw, uint32_t* qctr, uint32_t grid_wgs, hipStream_t stream,
                                               const uint32_t* n_dev)
{
    using namespace bpmd::lp3;
    if (n_tasks == 0) return 0;
    unsigned grid = (n_tasks + WG_MSGS - 1) / WG_MSGS;
    if (qctr && grid_wgs && grid > grid_wgs) grid = grid_wgs;
    hipLaunchKernelGGL(inflate_lane3_seg_kernel, dim3(grid), dim3(128), WG_MSGS * STRIDE, stream, in, in_off, in_len,
                       n_tasks, (const bpmd::bp::SegTask*)tasks, sym, (bpmd::bp::SegRes*)res, raw, qctr, n_dev);
    return (int)hipGetLastError();
}

// order: NULL or the order messages are taken in (e.g. longest first);
// qctr: NULL (one message per lane) or a zeroed device counter: then the grid
// is at most grid_wgs workgroups and lanes take further messages from it.
extern "C" int bpmd_internal_inflate_lane3(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint32_t n,
                                           uint8_t* out, const uint64_t* out_off, const uint32_t* out_cap,
                                           uint32_t* out_len, int32_t* status, uint32_t raw, const uint32_t* mask_key,
                                           const uint32_t* hist_len, uint32_t hist_max, uint32_t max_in,
                                           const uint32_t* order, uint32_t* qctr, uint32_t grid_wgs,
                                           const uint32_t* skip, hipStream_t stream)
{
    using namespace bpmd::lp3;
    if (n == 0) return 0;
    unsigned grid = (n + WG_MSGS - 1) / WG_MSGS;
    if (qctr && grid_wgs && grid > grid_wgs) grid = grid_wgs;
    hipLaunchKernelGGL(inflate_lane3_kernel, dim3(grid), dim3(128), WG_MSGS * STRIDE, stream, in, in_off, in_len, n,
                       out, out_off, out_cap, out_len, status, raw, mask_key, hist_len, hist_max, max_in, order, qctr,
                       skip);
    return (int)hipGetLastError();
}

// ---------------------------------------------------------------- order
// Work-queue batches of mixed sizes (configs[3]): lanes take messages
// longest compressed payload first, so the long messages start while the
// short ones still fill the lanes that finish early, and no lane starts a
// 64 KiB message as the batch drains.  Keys are in_len >> 6 (coarse classes
// are enough for balance, and fewer radix passes), stable in message order.
namespace bpmd {
namespace lp3 {
__global__ void __launch_bounds__(256) order_keys_kernel(const uint32_t* __restrict__ in_len, uint32_t n,
                                                         uint32_t* __restrict__ key, uint32_t* __restrict__ idx)
{
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i < n) {
        key[i] = in_len[i] >> 6;
        idx[i] = i;
    }
}
}  // namespace lp3
}  // namespace bpmd

extern "C" void* bpmd_internal_scratch(hipStream_t s, size_t bytes, int which);

// order[0, n) = message indices, longest payload first; returns null on error.
// keys_out (optional): the sorted keys (in_len >> 6, descending).
extern "C" const uint32_t* bpmd_internal_lane_order(const uint32_t* in_len, uint32_t n, hipStream_t stream,
                                                    const uint32_t** keys_out)
{
    size_t temp = 0;
    if (hipcub::DeviceRadixSort::SortPairsDescending(nullptr, temp, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                                     (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)n, 0, 26,
                                                     stream) != hipSuccess)
        return nullptr;
    const size_t words = (size_t)n * 4;   // key in, key out, index in, index out
    uint8_t* p = (uint8_t*)bpmd_internal_scratch(stream, words * 4 + temp + 256, 5);
    if (!p) return nullptr;
    uint32_t* kin = (uint32_t*)p;
    uint32_t* kout = kin + n;
    uint32_t* iin = kout + n;
    uint32_t* iout = iin + n;
    void* tmp = (void*)(((uintptr_t)(iout + n) + 255) & ~(uintptr_t)255);
    hipLaunchKernelGGL(bpmd::lp3::order_keys_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, in_len, n, kin, iin);
    if (hipGetLastError() != hipSuccess) return nullptr;
    if (hipcub::DeviceRadixSort::SortPairsDescending(tmp, temp, kin, kout, iin, iout, (int)n, 0, 26, stream) !=
        hipSuccess)
        return nullptr;
    if (keys_out) *keys_out = kout;
    return iout;
}

// ------------------------------------------------------------ long payloads
// A lane decodes one message serially, so in a work-queue batch a payload
// that alone takes longer than the whole batch's share per lane sets the
// launch's end (at 8 GPUs, each rank's C4 shard ran ~20 ms on its 64 KiB
// messages against ~5 ms for the rest).  Those payloads go to the wave
// kernel, which decodes one message with 64 lanes, or to the block-parallel
// decoder, which cuts it at block starts.  "Longer than its share":
// compressed length above share_pct % of the batch's compressed bytes per
// resident lane (block-parallel: 125 % by default, BPMD_LONG_SHARE_PCT, so
// the work queue ends near the per-lane share; wave kernel: 200 %; the
// values live in pmd_capi.hip inflate_impl), and never below min_thr.  The count is computed on the device from the sorted keys, so the
// call stays asynchronous: split[0] = total compressed bytes (u64),
// split[2] = number of long payloads = a prefix of the longest-first order.
namespace bpmd {
namespace lp3 {
__global__ void __launch_bounds__(256) sum_in_kernel(const uint32_t* __restrict__ in_len, uint32_t n,
                                                     unsigned long long* __restrict__ total)
{
    unsigned long long acc = 0;
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) acc += in_len[i];
    for (int d = 32; d >= 1; d >>= 1) acc += __shfl_down(acc, d);
    if ((threadIdx.x & 63) == 0 && acc) atomicAdd(total, acc);
}
__global__ void long_count_kernel(const uint32_t* __restrict__ keys, uint32_t n, uint32_t lanes, uint32_t min_thr,
                                  uint32_t share_pct, unsigned long long* __restrict__ split)
{
    if (threadIdx.x != 0) return;
    if (min_thr == 0 && lanes == 0) {   // every payload
        ((uint32_t*)split)[2] = n;
        return;
    }
    const unsigned long long total = split[0];
    unsigned long long thr = lanes ? (unsigned long long)share_pct * total / (100ull * lanes) : 0ull;
    if (thr < min_thr) thr = min_thr;
    // long: key >= ceil(thr / 64), i.e. in_len >= thr when thr is a multiple
    // of 64 (every caller's), at least thr otherwise (keys descending)
    const uint32_t tk = (uint32_t)((thr + 63) >> 6);
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (keys[mid] >= tk) lo = mid + 1;
        else hi = mid;
    }
    ((uint32_t*)split)[2] = lo;
}
}  // namespace lp3
}  // namespace bpmd

// returns a device pointer to the number of long payloads (a prefix of the
// order bpmd_internal_lane_order returned with `keys`), or null on error.
// lanes == 0: a fixed threshold of min_thr compressed bytes (0: every payload).
extern "C" const uint32_t* bpmd_internal_lane_long_split(const uint32_t* in_len, const uint32_t* keys, uint32_t n,
                                                         uint32_t lanes, uint32_t min_thr, uint32_t share_pct,
                                                         hipStream_t stream)
{
    unsigned long long* split = (unsigned long long*)bpmd_internal_scratch(stream, 256, 9);
    if (!split || hipMemsetAsync(split, 0, 16, stream) != hipSuccess) return nullptr;
    const uint32_t blocks = n / 256 + 1 < 1024 ? n / 256 + 1 : 1024;
    hipLaunchKernelGGL(bpmd::lp3::sum_in_kernel, dim3(blocks), dim3(256), 0, stream, in_len, n, split);
    hipLaunchKernelGGL(bpmd::lp3::long_count_kernel, dim3(1), dim3(64), 0, stream, keys, n, lanes, min_thr, share_pct,
                       split);
    if (hipGetLastError() != hipSuccess) return nullptr;
    return (const uint32_t*)split + 2;
}

// diagnostic counters of the pipelined lane kernel (meaningful only in the
// -DBPMD_PROF build): out[0-15] g_l3prof, out[16-23] g_l3hprof when `out` has
// 24 entries (n24 != 0)
static int lane3_counters(unsigned long long* out, int reset, int n24)
{
    hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess) return (int)e;
    e = hipMemcpyFromSymbol(out, HIP_SYMBOL(bpmd::lp3::g_l3prof), sizeof(unsigned long long) * 16);
    if (e == hipSuccess && n24) e = hipMemcpyFromSymbol(out + 16, HIP_SYMBOL(bpmd::lp3::g_l3hprof), sizeof(unsigned long long) * 8);
    if (e != hipSuccess) return (int)e;
    if (reset) {
        unsigned long long z[16] = {0};
        e = hipMemcpyToSymbol(HIP_SYMBOL(bpmd::lp3::g_l3prof), z, sizeof z);
        if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(bpmd::lp3::g_l3hprof), z, sizeof(unsigned long long) * 8);
    }
    return (int)e;
}
extern "C" int bpmd_diag_lane3_counters(unsigned long long* out16, int reset) { return lane3_counters(out16, reset, 0); }
extern "C" int bpmd_diag_lane3_counters24(unsigned long long* out24, int reset) { return lane3_counters(out24, reset, 1); }
