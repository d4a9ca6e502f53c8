// pmd_inflate.hip -- batched raw-DEFLATE decode of permessage-deflate payloads
// on gfx950 (CDNA4, wave64).  One wavefront owns one message at a time.
//
// Reference semantics: Beast's decoder (include/boost/beast/zlib/detail/
// inflate_stream.ipp:74-535) driven as the websocket read path drives it
// (websocket/detail/impl_base.hpp:168-190, websocket/impl/read.hpp:1284-1356):
// the payload plus an appended 00 00 FF FF tail is decoded from a fresh
// state; decoding stops when the next step would need more bits than the
// input holds (the bitstream fill rule, bitstream.hpp:109-121), on BFINAL
// (end_of_stream), at the first data error (its zlib::error), or when the
// output would exceed the slot capacity (need_buffers, output truncated).
//
// Parallel decode.  Huffman decoding is serial within a stream, but a
// Huffman-coded bit stream re-synchronises when decoding starts at a wrong
// bit offset (on deflated JSON: 56 % of wrong starts within 8 tokens, 93 %
// within 32).  Each round of a block cuts the remaining bits into 64
// segments of ~32 tokens (estimated from the block's measured bits/token):
//   pass A  every lane decodes its segment from the segment start
//           (speculative for lanes >= 1) and records where it exits;
//   pass B  lane l restarts at lane l-1's exit -- the true token boundary
//           whenever lane l-1 re-synchronised -- and counts tokens/bytes;
//           lanes whose start disagrees with the predecessor's exit are
//           re-run until the chain is exact (lane 0 is exact by
//           construction, and each re-run makes the first bad lane exact);
//   pass C  after a prefix sum of the counts, lanes decode once more and
//           store their tokens straight into stream order, checking each
//           against its output position (invalid_distance, capacity).
// The first lane with an event (end of block, error, end of input,
// capacity) ends the round.  Tokens are then expanded 64 output bytes at a
// time: each lane finds its token with one popcount over a token-start
// bitmap, literal bytes are direct, match bytes read older output from the
// LDS ring (or global memory beyond it), and matches reaching into the same
// 64-byte chunk are resolved by pointer jumping across lanes (<= 6 steps).
//
// LDS per wave (~24 KiB): output ring, input window, round token list,
// bitmap / header scratch (union), decode tables (huff_table.h slots).
#include "pmd_common.h"
#include "huff_table.h"
#include "huff_wave.h"
#include "wave_util.h"

namespace bpmd {

#ifndef BPMD_RING
#define BPMD_RING 4096
#endif
#ifndef BPMD_TOT
#define BPMD_TOT 1024
#endif
// LDS per wave bounds the waves per CU, and the decode passes are latency
// bound (one wave alone runs its phases at the same speed as six sharing a
// CU), so the ring and token list are sized for occupancy: a 4 KiB ring and
// 1024 tokens per round still hold a whole 1023-symbol zlib block of text.
constexpr unsigned RING = BPMD_RING;     // output history ring (bytes)
constexpr unsigned RING_MASK = RING - 1;
constexpr unsigned R_MAX = RING - 256;   // output bytes per round, at most
#ifndef BPMD_IN_CAP
#define BPMD_IN_CAP 2560
#endif
// input window bytes (a round's segments need (64 * 300 + 160) / 8 + 16 =
// 2436).  2496 would bring WaveLds to 16 368 B, 10 waves per CU instead of 9:
// C5 inflate 33.9 -> 23.5 GiB/s with a fixed grid stride, even with the work
// queue (38.4 vs 38.7), so the window stays.
constexpr unsigned IN_CAP = BPMD_IN_CAP;
constexpr unsigned IN_PAD = 32;
constexpr unsigned WIN_WORDS = (IN_CAP + IN_PAD) / 4;
constexpr unsigned TOT = BPMD_TOT;       // tokens per round, at most
#ifndef BPMD_SEG_TOKENS
#define BPMD_SEG_TOKENS 20
#endif
constexpr unsigned SEG_TOKENS = BPMD_SEG_TOKENS;   // target tokens per lane segment
constexpr unsigned SEG_MAX_BITS = 300;   // keeps a round inside the window
constexpr unsigned BM_WORDS = (R_MAX + 128) / 32 + 2;

enum Ev : uint32_t { EV_NONE = 0, EV_EOB, EV_ERROR, EV_STARVED, EV_FULL, EV_PARTIAL, EV_LIMIT };

struct alignas(16) WaveLds {
    uint8_t ring[RING];
    uint32_t win[WIN_WORDS];
    uint32_t tok[TOT];
    union {
        uint32_t bitmap[BM_WORDS];
        struct {
            WaveTableScratch ts;
            uint8_t lens[320];
            alignas(4) uint8_t runval[320];   // code-length run starts: value + 1
        } h;
    } u;
    uint16_t tab[kEnough];
};
static_assert((WAVE * SEG_MAX_BITS + 160) / 8 + 16 <= IN_CAP, "a round's segments fit the input window");

__device__ uint16_t g_fixed_lens[512];
__device__ uint16_t g_fixed_dists[32];
// round mode (bpmd_diag_set_wave_walk, tests and A/B): 0 automatic, 1 walk
// rounds for every block, 2 speculative rounds for every block.  Walk rounds
// (lane j decodes the token at bit p0 + j + 64q, the chain followed through
// the candidates on the scalar unit) are exact without re-synchronisation;
// which mode is faster depends on the data (scripts/diag_wave_rate.py:
// Beast's own 64 KiB binary payloads, mostly fixed blocks of near-random
// literals, 21.2 vs 10.6 GiB/s for walk; JSON 38.6 vs 53.7 for speculative),
// so the automatic mode measures both on each message (s_memtime per round)
// and keeps the one with fewer cycles per token: a speculative round whose
// pass B needed more than WALK_PROBE re-runs is followed by a walk round, and
// every 16 rounds the mode not in use is measured again.
__device__ uint32_t g_wave_walk;

constexpr int WQ = 4;   // walk window: 64 x WQ candidate bit offsets
constexpr uint32_t WALK_PROBE = 4;

// Diagnostic build only (-DBPMD_PROF): per-phase cycle and event counters.
__device__ unsigned long long g_prof[24];
__device__ unsigned long long g_prof_dbg[16];
#ifdef BPMD_PROF
#define PROF_DECL unsigned long long prof_[24] = {0}; unsigned long long prof_t_ = __builtin_amdgcn_s_memtime()
#define PROF_MARK() (prof_t_ = __builtin_amdgcn_s_memtime())
#define PROF_LAP(i) do { unsigned long long t2_ = __builtin_amdgcn_s_memtime(); prof_[i] += t2_ - prof_t_; prof_t_ = t2_; } while (0)
#define PROF_CNT(i, n) (prof_[i] += (n))
#define PROF_FLUSH() do { if (lane_id() == 0) for (int i_ = 0; i_ < 24; ++i_) atomicAdd(&g_prof[i_], prof_[i_]); } while (0)
#else
#define PROF_DECL
#define PROF_MARK()
#define PROF_LAP(i)
#define PROF_CNT(i, n)
#define PROF_FLUSH()
#endif

struct Msg {
    const uint8_t* p;
    uint32_t n;       // payload bytes
    uint32_t total;   // payload + tail bytes
    uint32_t key;     // masking key (payload byte i ^= key >> 8 (i % 4), mask.ipp:38-59); 0 = unmasked
};

__device__ __forceinline__ uint32_t in_byte(const Msg& m, uint32_t i)
{
    if (i < m.n) return m.p[i] ^ ((m.key >> (8 * (i & 3))) & 0xffu);
    if (i < m.total) return (i - m.n) >= 2 ? 0xffu : 0u;   // 00 00 FF FF
    return 0;
}

// 4 bytes of payload || tail || zeros at byte offset i
__device__ __forceinline__ uint32_t in_word(const Msg& m, uint32_t i)
{
    if (i + 8 <= m.n) {
        uintptr_t a = (uintptr_t)(m.p + i);
        const uint32_t* w = (const uint32_t*)(a & ~(uintptr_t)3);
        const unsigned sh = (unsigned)(a & 3) * 8;
        const uint64_t v = ((uint64_t)w[1] << 32) | w[0];
        return (uint32_t)(v >> sh) ^ __builtin_amdgcn_alignbit(m.key, m.key, 8 * (i & 3));
    }
    return in_byte(m, i) | (in_byte(m, i + 1) << 8) | (in_byte(m, i + 2) << 16) | (in_byte(m, i + 3) << 24);
}

// Fill the LDS window with stream bytes [wbase, wbase + IN_CAP + IN_PAD).
// Every global load is issued before the first LDS store so their latencies
// overlap; only the word holding the payload's end and the tail past it take
// the byte path.
template <unsigned NW>
__device__ __forceinline__ void load_window(uint32_t* win, const Msg& m, uint32_t wbase)
{
    const unsigned lane = lane_id();
    constexpr unsigned PER_LANE = (NW + WAVE - 1) / WAVE;
    const uint32_t full = m.n >> 2;   // whole payload words
    const uint32_t w0 = wbase >> 2;
    uint32_t nfast = 0;               // window words served by plain loads
    if ((((uintptr_t)m.p) & 3) == 0 && full > w0) {
        nfast = full - w0 < NW ? full - w0 : NW;
        const uint32_t* p32 = (const uint32_t*)m.p + w0;
        uint32_t vals[PER_LANE];
#pragma unroll
        for (unsigned k = 0; k < PER_LANE; ++k) {
            const uint32_t i = lane + k * WAVE;
            vals[k] = p32[i < nfast ? i : 0];
        }
#pragma unroll
        for (unsigned k = 0; k < PER_LANE; ++k) {
            const uint32_t i = lane + k * WAVE;
            if (i < nfast) win[i] = vals[k] ^ m.key;   // aligned payload: byte j of a word takes key byte j
        }
    }
    for (uint32_t i = nfast + lane; i < NW; i += WAVE) win[i] = in_word(m, wbase + 4 * i);
}

// 64 stream bits starting at bit p_rel of the LDS window
__device__ __forceinline__ uint64_t peek64(const uint32_t* win, uint32_t p_rel)
{
    const uint32_t w = p_rel >> 5, sh = p_rel & 31;
    const uint32_t d0 = win[w], d1 = win[w + 1], d2 = win[w + 2];
    const uint32_t lo = __builtin_amdgcn_alignbit(d1, d0, sh);
    const uint32_t hi = __builtin_amdgcn_alignbit(d2, d1, sh);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint32_t lowbits(uint64_t v, unsigned n) { return (uint32_t)v & ((1u << n) - 1u); }

// byte of our own earlier output, read past the (non-coherent) L1
__device__ __forceinline__ uint32_t gbyte(const uint8_t* p)
{
    const uintptr_t a = (uintptr_t)p;
    uint32_t* w = (uint32_t*)(a & ~(uintptr_t)3);
    const uint32_t v = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return (v >> ((a & 3) * 8)) & 0xffu;
}


// ------------------------------------------------------------- token decode

struct Tok {
    uint32_t info;    // literal: byte;  match: (len << 16) | dist
    uint32_t nbits;
    uint32_t olen;    // output bytes
    uint32_t ev;      // EV_NONE, EV_EOB, EV_ERROR, EV_STARVED
    uint32_t err;
};

// One literal/length[/distance] token from the 64 stream bits v with Beast's
// fill rule: each step needs the bits the reference's slow path asks for
// (inflate_stream.ipp:360-474).  avail = bits left in the stream.
__device__ __forceinline__ Tok decode_tok(uint64_t v, uint32_t avail, const uint16_t* ltab, unsigned lroot,
                                          const uint16_t* dtab, unsigned droot)
{
    Tok t;
    t.info = 0;
    t.nbits = 0;
    t.olen = 0;
    t.ev = EV_NONE;
    t.err = 0;
    uint16_t s = ltab[lowbits(v, lroot)];
    unsigned need = lroot, used;
    if (slot_is_link(s)) {
        const unsigned sub = slot_bits(s);
        need = lroot + sub;
        s = ltab[slot_val(s) + lowbits(v >> lroot, sub)];
        used = lroot + slot_bits(s);
    } else {
        used = slot_bits(s);
    }
    if (avail < need) { t.ev = EV_STARVED; return t; }
    const unsigned kind = slot_kind(s);
    if (kind == K_VAL) {
        t.info = slot_val(s);
        t.nbits = used;
        t.olen = 1;
        return t;
    }
    if (kind == K_EOB) { t.ev = EV_EOB; t.nbits = used; return t; }
    if (kind == K_SPECIAL) { t.ev = EV_ERROR; t.err = ST_INVALID_LITERAL_LENGTH; return t; }
    // length (RFC 1951 3.2.5): base and extra bits from the symbol index
    const unsigned li = slot_val(s);
    const unsigned xl = (li < 8 || li == 28) ? 0u : ((li - 4) >> 2);
    unsigned len = li < 8 ? li + 3 : (li == 28 ? 258u : (((4u + (li & 3)) << xl) + 3));
    len += lowbits(v >> used, xl);
    used += xl;
    if (avail < used) { t.ev = EV_STARVED; return t; }
    uint16_t d = dtab[lowbits(v >> used, droot)];
    need = used + droot;
    unsigned dused;
    if (slot_is_link(d)) {
        const unsigned sub = slot_bits(d);
        need += sub;
        d = dtab[slot_val(d) + lowbits(v >> (used + droot), sub)];
        dused = used + droot + slot_bits(d);
    } else {
        dused = used + slot_bits(d);
    }
    if (avail < need) { t.ev = EV_STARVED; return t; }
    if (slot_kind(d) == K_SPECIAL) { t.ev = EV_ERROR; t.err = ST_INVALID_DISTANCE_CODE; return t; }
    const unsigned di = slot_val(d);
    const unsigned xd = di < 4 ? 0u : (di >> 1) - 1;
    unsigned dist = di < 4 ? di + 1 : (((2u + (di & 1)) << xd) + 1);
    dist += lowbits(v >> dused, xd);
    dused += xd;
    if (avail < dused) { t.ev = EV_STARVED; return t; }
    t.info = (len << 16) | dist;
    t.nbits = dused;
    t.olen = len;
    return t;
}

struct LaneRes {
    uint32_t exit, n, bytes, ev, err, trips;
};

__device__ __forceinline__ uint32_t wave_max(uint32_t x)
{
#pragma unroll
    for (unsigned d = 1; d < WAVE; d <<= 1) {
        const uint32_t y = __shfl_xor(x, d);
        x = x > y ? x : y;
    }
    return x;
}

struct Tables {
    const uint16_t* ltab;
    const uint16_t* dtab;
    unsigned lroot, droot;
};

// Count pass: decode tokens starting at `start` until a token would start
// at or beyond `end`, or an event.
__device__ __forceinline__ LaneRes decode_count(const WaveLds& L, uint32_t wb, uint32_t start, uint32_t end,
                                                uint32_t total_bits, const Tables& T)
{
    LaneRes r;
    r.n = 0;
    r.bytes = 0;
    r.ev = EV_NONE;
    r.err = 0;
    r.trips = 0;
    uint32_t p = start;
    while (p < end) {
        r.trips += 1;
        const uint64_t v = peek64(L.win, p - wb);
        const uint32_t avail = p < total_bits ? total_bits - p : 0;
        const Tok t = decode_tok(v, avail, T.ltab, T.lroot, T.dtab, T.droot);
        if (t.ev != EV_NONE) {
            r.ev = t.ev;
            r.err = t.err;
            if (t.ev == EV_EOB) p += t.nbits;
            break;
        }
        r.n += 1;
        r.bytes += t.olen;
        p += t.nbits;
    }
    r.exit = p;
    return r;
}

// Store pass: the same decode from an exact start, writing tokens at
// tok[P...] and their output offsets into the bitmap, with the checks the
// reference makes at each token's output position (inflate_stream.ipp:
// 475-514): a full buffer first when the capacity is exact (raw), then the
// distance, then the capacity.
// A whole message is decoded in one call from a fresh state, so a distance
// may reach back to the message's first output byte (inflate_stream.ipp:
// 475-496 with an empty window).
__device__ __forceinline__ LaneRes decode_store(WaveLds& L, uint32_t wb, uint32_t start, uint32_t end,
                                                uint32_t total_bits, const Tables& T, uint32_t P, uint32_t abs0,
                                                uint32_t round0, uint32_t cap, bool raw)
{
    LaneRes r;
    r.n = 0;
    r.bytes = 0;
    r.ev = EV_NONE;
    r.err = 0;
    r.trips = 0;
    uint32_t p = start;
    while (p < end) {
        r.trips += 1;
        const uint64_t v = peek64(L.win, p - wb);
        const uint32_t avail = p < total_bits ? total_bits - p : 0;
        const Tok t = decode_tok(v, avail, T.ltab, T.lroot, T.dtab, T.droot);
        if (t.ev != EV_NONE) {
            r.ev = t.ev;
            r.err = t.err;
            if (t.ev == EV_EOB) p += t.nbits;
            break;
        }
        const uint32_t abs = abs0 + r.bytes;
        if (raw && abs >= cap) { r.ev = EV_FULL; break; }
        if (t.olen > 1 || (t.info >> 16)) {
            if ((t.info & 0xffffu) > abs) { r.ev = EV_ERROR; r.err = ST_INVALID_DISTANCE; break; }
        }
        if (abs >= cap) { r.ev = EV_FULL; break; }
        L.tok[P + r.n] = t.info;
        const uint32_t rel = abs - round0;
        atomicOr(&L.u.bitmap[rel >> 5], 1u << (rel & 31));
        r.n += 1;
        p += t.nbits;
        if (abs + t.olen > cap) {
            r.bytes += cap - abs;
            r.ev = EV_PARTIAL;
            break;
        }
        r.bytes += t.olen;
    }
    r.exit = p;
    return r;
}

// --------------------------------------------------------------- wave utils

__device__ __forceinline__ uint32_t scan_incl(uint32_t x)
{
    const unsigned lane = lane_id();
#pragma unroll
    for (unsigned d = 1; d < WAVE; d <<= 1) {
        const uint32_t y = __shfl_up(x, d);
        x += lane >= d ? y : 0u;   // select: a shuffle must not sink under divergence
    }
    return x;
}

__device__ __forceinline__ uint32_t from_prev_lane(uint32_t x) { return __shfl_up(x, 1); }

__device__ __forceinline__ unsigned first_lane(uint64_t mask) { return mask ? (unsigned)__builtin_ctzll(mask) : WAVE; }

// set bits of m below this lane
__device__ __forceinline__ uint32_t popc_below_lane(uint64_t m)
{
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// ------------------------------------------------------------------- output

struct Out {
    uint8_t* g;       // message slot in global memory
    uint32_t cap;
    uint32_t pos;     // bytes produced
    uint32_t flushed; // bytes already stored to g
};

// store ring bytes [a, b) to global memory
__device__ void ring_flush(WaveLds& L, Out& o, uint32_t a, uint32_t b)
{
    if (b <= a) return;
    const unsigned lane = lane_id();
    if ((((uintptr_t)o.g) & 15) == 0) {
        const uint32_t a16 = (a + 15) & ~15u, b16 = b & ~15u;
        if (a16 < b16) {
            for (uint32_t i = a + lane; i < a16; i += WAVE) o.g[i] = L.ring[i & RING_MASK];
            for (uint32_t q = a16 + lane * 16; q < b16; q += WAVE * 16)
                *(uint4*)(o.g + q) = *(const uint4*)(L.ring + (q & RING_MASK));
            for (uint32_t i = b16 + lane; i < b; i += WAVE) o.g[i] = L.ring[i & RING_MASK];
            return;
        }
    }
    for (uint32_t i = a + lane; i < b; i += WAVE) o.g[i] = L.ring[i & RING_MASK];
}

// positions about to be overwritten in the ring must reach global memory
__device__ __forceinline__ void ring_reserve(WaveLds& L, Out& o, uint32_t n)
{
    const uint32_t need = o.pos + n;
    if (need > RING && need - RING > o.flushed) {
        ring_flush(L, o, o.flushed, need - RING);
        o.flushed = need - RING;
        __builtin_amdgcn_s_waitcnt(0);
        wave_sync();
    }
}

// expand the round's tokens into output bytes [o.pos, o.pos + nbytes)
__device__ __forceinline__ void expand_round(WaveLds& L, Out& o, uint32_t nbytes)
{
    const unsigned lane = lane_id();
    ring_reserve(L, o, nbytes);
    const uint32_t rs = o.pos, re = o.pos + nbytes;
    int32_t tprev = -1;
    const uint64_t upto = lane == 63 ? ~0ull : ((2ull << lane) - 1);
    for (uint32_t c = rs; c < re; c += WAVE) {
        const uint32_t rel = c - rs;   // multiple of 64
        const uint64_t B = ((uint64_t)L.u.bitmap[(rel >> 5) + 1] << 32) | L.u.bitmap[rel >> 5];
        const uint32_t q = c + lane;
        const bool act = q < re;
        // ring slots written by this chunk hold positions < wend - RING
        const uint32_t wend = c + WAVE < re ? c + WAVE : re;
        const int32_t T = tprev + (int32_t)__builtin_popcountll(B & upto);
        const uint32_t info = act ? L.tok[T] : 0u;
        const uint32_t len = info >> 16;
        uint32_t val = info & 0xffu;
        int32_t src = (int32_t)q - (int32_t)(info & 0xffffu);
        bool pend = false;
        if (act && len) {
            if (src >= (int32_t)c) pend = true;
            else if ((uint32_t)src + RING >= wend) val = L.ring[src & RING_MASK];
            else val = gbyte(o.g + src);
        }
        // matches reaching into this chunk: pointer jumping
        while (__ballot(pend)) {
            const unsigned from = pend ? src - c : lane;
            const uint32_t v2 = __shfl(val, from);
            const int32_t s2 = __shfl(src, from);
            const bool p2 = __shfl(pend ? 1 : 0, from) != 0;
            if (pend) {
                if (!p2) { val = v2; pend = false; }
                else src = s2;
            }
        }
        if (act) L.ring[q & RING_MASK] = (uint8_t)val;
        tprev += (int32_t)__builtin_popcountll(B);
        wave_sync();
    }
    o.pos = re;
}

// --------------------------------------------------------------- one message

static __constant__ const uint8_t kClenOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

__device__ void inflate_msg(WaveLds& L, const Msg& m, Out& o, bool raw, uint32_t& out_len, int32_t& status)
{
    const unsigned lane = lane_id();
    const uint32_t total_bits = m.total * 8;
    int32_t st = ST_OK;
    const int32_t full_status = raw ? ST_OK : ST_NEED_BUFFERS;
    if (m.total == 0) {   // raw mode, no input: no progress (inflate_stream.ipp:113-117)
        out_len = 0;
        status = ST_NEED_BUFFERS;
        return;
    }
    PROF_DECL;
    uint32_t wbase = 0;   // window start, bytes (multiple of 4)
    load_window<WIN_WORDS>(L.win, m, wbase);
    wave_sync();
    PROF_LAP(10);
    auto ensure = [&](uint32_t p, uint32_t nbytes) {
        const uint32_t b0 = p >> 3;
        if (b0 < wbase || b0 + nbytes > wbase + IN_CAP) {
            PROF_MARK();
            wbase = b0 & ~3u;
            wave_sync();
            load_window<WIN_WORDS>(L.win, m, wbase);
            wave_sync();
            PROF_LAP(10);
            PROF_CNT(11, 1);
        }
    };
    auto ubits = [&](uint32_t p, unsigned n) -> uint32_t { return lowbits(peek64(L.win, p - wbase * 8), n); };

    uint32_t pos = 0;   // stream bit position (wave-uniform)
    bool last = false;
    uint32_t est16 = 8 * 16;   // estimated bits per token, x16
    // round mode (g_wave_walk): forced, or chosen per message by the cycles
    // per token each mode measured on this message's recent rounds
    const uint32_t wmode = g_wave_walk;
    bool walk = wmode == 1;
    uint32_t cpt_spec = 0, cpt_walk = 0;   // cycles per token x16 of the last round of each mode (0: unknown)
    uint32_t rounds = 0;

    for (;;) {
        unsigned type;
        {
            // ---- TYPEDO (inflate_stream.ipp:146-182)
            if (last) { st = ST_END_OF_STREAM; break; }
            ensure(pos, 700);
            if (total_bits - pos < 3) break;
            const uint32_t hdr = ubits(pos, 3);
            pos += 3;
            last = (hdr & 1) != 0;
            type = hdr >> 1;
        }
        Tables T;
        T.ltab = L.tab;
        T.dtab = L.tab + 512;
        T.lroot = 9;
        T.droot = 5;

        if (type == 0) {
            // ---- STORED / COPY (ipp:184-220)
            pos = (pos + 7) & ~7u;
            if (pos > total_bits || total_bits - pos < 32) break;
            const uint32_t v = ubits(pos, 16);
            const uint32_t nv = ubits(pos + 16, 16);
            if (v != (nv ^ 0xffffu)) { st = ST_INVALID_STORED_LENGTH; break; }
            pos += 32;
            const uint32_t from = pos >> 3;
            const uint32_t have = m.total - from;
            uint32_t n = v < have ? v : have;
            bool full = false;
            if (o.pos + n > o.cap) { n = o.cap - o.pos; full = true; }
            for (uint32_t done = 0; done < n;) {
                const uint32_t piece = n - done < R_MAX ? n - done : R_MAX;
                ring_reserve(L, o, piece);
                for (uint32_t k = lane; k < piece; k += WAVE)
                    L.ring[(o.pos + k) & RING_MASK] = (uint8_t)in_byte(m, from + done + k);
                wave_sync();
                o.pos += piece;
                done += piece;
            }
            pos += n * 8;
            if (full) { st = full_status; break; }
            if (n < v) break;   // input ends inside the block
            continue;
        } else if (type == 1) {
            for (unsigned k = lane; k < 512; k += WAVE) L.tab[k] = g_fixed_lens[k];
            if (lane < 32) L.tab[512 + lane] = g_fixed_dists[lane];
            wave_sync();
        } else if (type == 2) {
            // ---- TABLE / LENLENS / CODELENS (ipp:222-354)
            if (total_bits - pos < 14) break;
            const unsigned nlen = ubits(pos, 5) + 257;
            const unsigned ndist = ubits(pos + 5, 5) + 1;
            const unsigned ncode = ubits(pos + 10, 4) + 4;
            pos += 14;
            if (nlen > 286 || ndist > 30) { st = ST_TOO_MANY_SYMBOLS; break; }
            // the code-length code lengths: lane i reads field i
            if (total_bits - pos < 3 * ncode) {
                // the reference reads them one by one and stops when starved
                break;
            }
            if (lane < 19) {
                uint32_t cl = 0;
                for (unsigned i = 0; i < ncode; ++i)
                    if (kClenOrder[i] == lane) cl = ubits(pos + 3 * i, 3);
                L.u.h.lens[lane] = (uint8_t)cl;
            }
            pos += 3 * ncode;
            wave_sync();
            unsigned croot = 0, cused = 0, cmin = 0;
            PROF_LAP(20);
            int r = build_table_wave<BUILD_CODES>(L.u.h.lens, 19, L.tab, 7, L.u.h.ts, croot, cused, cmin);
            wave_sync();
            PROF_LAP(16);
            if (r) { st = r; break; }
            // code lengths (ipp:264-327): every lane decodes a code-length
            // symbol at its own bit offset of a 64-bit window; a scalar walk
            // then follows the true chain through the window, applying the
            // reference's checks in order, and marks run starts; a final
            // fill-forward expands the runs.
            bool starved = false;
            const unsigned want = nlen + ndist;
            for (unsigned i = lane; i < 80; i += WAVE) ((uint32_t*)L.u.h.runval)[i] = 0;
            wave_sync();
            unsigned have = 0, prevlen = 0;
            while (have < want) {
                // Every lane decodes the symbol that would start at bit w +
                // lane; the true chain from w is found by pointer doubling
                // over reach masks, then the chain members are processed in
                // order with prefix sums -- the reference's per-symbol checks
                // (ipp:264-327) become "first member with an event".
                const uint32_t w = pos;
                const uint64_t v = peek64(L.win, w + lane - wbase * 8);
                const uint16_t s = L.tab[lowbits(v, croot)];
                const unsigned sym = slot_val(s), cb = slot_bits(s);
                const unsigned xb = sym < 16 ? 0u : (sym == 16 ? 2u : sym == 17 ? 3u : 7u);
                const unsigned x = lowbits(v >> cb, xb);
                const unsigned step = sym < 16 ? cb : cb + xb;
                // reach masks: R(o) = positions of the window reachable from o
                uint32_t J = lane + step;   // successor (>= 64: leaves the window)
                uint64_t R = (1ull << lane) | (J < WAVE ? (1ull << J) : 0ull);
#pragma unroll
                for (int k = 0; k < 6; ++k) {
                    const uint32_t jj = J < WAVE ? J : lane;
                    const uint32_t rlo = __shfl((uint32_t)R, jj), rhi = __shfl((uint32_t)(R >> 32), jj);
                    const uint32_t j2 = __shfl(J, jj);
                    // selects, not a branch: a shuffle sunk under divergence
                    // would read 0 from the switched-off lanes
                    const uint64_t keep = J < WAVE ? ~0ull : 0ull;
                    R |= (((uint64_t)rhi << 32) | rlo) & keep;
                    J = J < WAVE ? j2 : J;
                }
                const uint64_t chain = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(R >> 32)) << 32) |
                                       (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)R);   // returns int: no sign extension
                const bool mem = (chain >> lane) & 1;
                const unsigned rep = !mem ? 0u : sym < 16 ? 1u : sym == 16 ? 3u + x : (sym == 17 ? 3u : 11u) + x;
                const uint32_t incl = scan_incl(rep);
                const uint32_t hb = have + incl - rep;       // lengths decoded before this member
                const uint32_t av = total_bits - (w + lane);
                // events in the reference's order: starved (root bits, then
                // code + extra together), repeat without a previous length,
                // repeat past the end
                const unsigned ev = !mem ? 0u
                                  : av < croot ? 1u
                                  : sym < 16 ? 0u
                                  : av < cb + xb ? 1u
                                  : (sym == 16 && hb == 0) ? 2u
                                  : hb + rep > want ? 2u : 0u;
                const uint64_t m_done = __ballot(mem && hb >= want);
                const uint64_t m_ev = __ballot(ev != 0);
                const unsigned f_done = first_lane(m_done), f_ev = first_lane(m_ev);
                const unsigned stop_at = f_done < f_ev ? f_done : f_ev;   // first member not processed
                const bool proc = mem && lane < stop_at;
                // value of a repeat (16) = the last earlier non-16 member's
                const unsigned own = sym < 16 ? sym : 0u;
                const uint32_t src = (proc && sym != 16) ? lane + 1 : 0u;
                uint32_t lastsrc = src;
#pragma unroll
                for (unsigned d = 1; d < WAVE; d <<= 1) {
                    const uint32_t y = __shfl_up(lastsrc, d);
                    lastsrc = (lane >= d && y > lastsrc) ? y : lastsrc;
                }
                const uint32_t from = lastsrc ? lastsrc - 1 : 0u;
                const uint32_t vfrom = __shfl(own, from);
                const unsigned val = sym == 16 ? (lastsrc ? vfrom : prevlen) : own;
                if (proc) L.u.h.runval[hb] = (uint8_t)(val + 1);
                const uint64_t pm = __ballot(proc);
#ifdef BPMD_PROF
                const uint32_t have_in = have;
#endif
                if (pm) {
                    const unsigned lastp = 63u - (unsigned)__builtin_clzll(pm);
                    have = __shfl(hb + rep, lastp);
                    prevlen = __shfl(val, lastp);
                    pos = w + __shfl(lane + step, lastp);
                }
#ifdef BPMD_PROF
                if (lane == 0 && g_prof_dbg[15] < 5) {
                    const unsigned k5 = (unsigned)g_prof_dbg[15];
                    g_prof_dbg[3 * k5] = chain;
                    g_prof_dbg[3 * k5 + 1] = ((unsigned long long)have_in << 32) | have;
                    g_prof_dbg[3 * k5 + 2] = ((unsigned long long)stop_at << 32) | (63u - (unsigned)__builtin_clzll(pm | 1));
                    g_prof_dbg[15] = k5 + 1;
                }
#endif
                if (f_ev < f_done) {
                    if (__shfl(ev, f_ev) == 1) starved = true;
                    else st = ST_INVALID_BIT_LENGTH_REPEAT;
                    break;
                }
            }
            if (st) break;
            if (starved) break;
            wave_sync();
            {
                uint32_t carry = 0;
                const uint64_t upto = lane == 63 ? ~0ull : ((2ull << lane) - 1);
                for (unsigned c0 = 0; c0 < want; c0 += WAVE) {
                    const unsigned i = c0 + lane;
                    const uint32_t mk = i < want ? L.u.h.runval[i] : 0u;
                    const uint64_t mask = __ballot(mk != 0);
                    const uint64_t le = mask & upto;
                    const unsigned j = le ? 63u - (unsigned)__builtin_clzll(le) : 0u;
                    const uint32_t fromj = __shfl(mk, j);
                    const uint32_t val = le ? fromj : carry;
                    if (i < want) L.u.h.lens[i] = (uint8_t)(val - 1);
                    if (mask) carry = __shfl(mk, 63u - (unsigned)__builtin_clzll(mask));
                }
            }
            wave_sync();
            PROF_LAP(17);
            if (L.u.h.lens[256] == 0) { st = ST_MISSING_EOB; break; }
            unsigned lroot = 0, lused = 0, lmin = 0, droot = 0, dused = 0, dmin = 0;
            r = build_table_wave<BUILD_LENS>(L.u.h.lens, nlen, L.tab, 9, L.u.h.ts, lroot, lused, lmin);
            wave_sync();
            PROF_LAP(18);
            if (r) { st = r; break; }
            r = build_table_wave<BUILD_DISTS>(L.u.h.lens + nlen, ndist, L.tab + lused, 6, L.u.h.ts, droot, dused,
                                              dmin);
            wave_sync();
            PROF_LAP(19);
            if (r) { st = r; break; }
            T.lroot = lroot;
            T.droot = droot;
            T.dtab = L.tab + lused;
        } else {
            st = ST_INVALID_BLOCK_TYPE;
            break;
        }

        // ---- compressed data, in rounds (ipp:356-514)
        PROF_LAP(1);
        PROF_CNT(8, 1);
        bool stop = false, block_end = false;
        uint32_t shrink = 0;
        while (!stop && !block_end) {
            PROF_CNT(6, 1);
            const uint32_t S = pos;
            const uint64_t t_round = wmode == 0 ? __builtin_amdgcn_s_memtime() : 0ull;
            // every 16 rounds one round runs in the mode not in use, so its
            // measure stays current (the data may change character)
            if (wmode == 0 && (++rounds & 15) == 0 && cpt_spec && cpt_walk) walk = !walk;
            if (walk) {
                // ---- walk round: lane j decodes the tokens starting at bits
                // p0 + j + 64q (q < WQ); the true chain from p0 is then
                // followed on the scalar unit through those candidates
                // (v_readlane of their lengths), so every step is exact
                // whatever the code -- no re-synchronisation needed -- and
                // yields the tokens starting in [p0, p0 + 64 WQ).  The
                // reference's per-token checks apply to the chain members in
                // order, as in decode_store; the first member with an event
                // ends the round.
                for (unsigned i = lane; i < BM_WORDS; i += WAVE) L.u.bitmap[i] = 0;
                wave_sync();
                uint32_t p0 = S, ntok = 0, nbyte = 0, wev = EV_NONE, werr = 0;
                for (;;) {
                    ensure(p0, 8 * WQ + 16);
                    const uint32_t wbw = wbase * 8;
                    Tok t[WQ];
                    uint32_t nbq[WQ];
#pragma unroll
                    for (int q = 0; q < WQ; ++q) {
                        const uint32_t p = p0 + 64u * q + lane;
                        const uint32_t avail = p < total_bits ? total_bits - p : 0;
                        t[q] = decode_tok(peek64(L.win, p - wbw), avail, T.ltab, T.lroot, T.dtab, T.droot);
                        nbq[q] = t[q].ev == EV_NONE ? t[q].nbits : 0u;   // 0: an event ends the chain
                    }
                    // the chain, on scalar registers
                    uint64_t M[WQ];
                    uint32_t cur = 0;
                    bool ended = false;
#pragma unroll
                    for (int q = 0; q < WQ; ++q) {
                        M[q] = 0;
                        while (!ended && cur < 64u * (q + 1)) {
                            const uint32_t l = cur - 64u * q;
                            M[q] |= 1ull << l;
                            const uint32_t nb = (uint32_t)__builtin_amdgcn_readlane((int)nbq[q], (int)l);
                            if (nb == 0) ended = true;
                            else cur += nb;
                        }
                    }
                    // members in chain order: output offsets, events, stores
                    uint32_t base_tok = 0, base_byte = 0, fe = 64u * WQ, fev = EV_NONE;
                    uint32_t fe_before = 0, fe_abs = 0, fe_nb = 0, fe_err = 0;
#pragma unroll
                    for (int q = 0; q < WQ; ++q) {
                        const bool mem = (M[q] >> lane) & 1;
                        const uint32_t idx = base_tok + popc_below_lane(M[q]);
                        const uint32_t ol = mem && t[q].ev == EV_NONE ? t[q].olen : 0u;
                        const uint32_t ol_incl = base_byte + wave_scan_incl(ol);
                        const uint32_t abs = o.pos + nbyte + ol_incl - ol;
                        const bool is_match = t[q].olen > 1 || (t[q].info >> 16) != 0;
                        uint32_t e = EV_NONE;
                        if (mem && fe == 64u * WQ) {
                            if (t[q].ev != EV_NONE) e = t[q].ev;
                            else if (ntok + idx >= TOT || nbyte + ol_incl > R_MAX) e = EV_LIMIT;
                            else if (raw && abs >= o.cap) e = EV_FULL;
                            else if (is_match && (t[q].info & 0xffffu) > abs) e = EV_ERROR;
                            else if (abs >= o.cap) e = EV_FULL;
                            else if (abs + t[q].olen > o.cap) e = EV_PARTIAL;
                        }
                        const unsigned f = first_lane(__ballot(e != EV_NONE));
                        const bool store = mem && fe == 64u * WQ && (lane < f || (lane == f && e == EV_PARTIAL));
                        if (store) {
                            L.tok[ntok + idx] = t[q].info;
                            const uint32_t rel = abs - o.pos;
                            atomicOr(&L.u.bitmap[rel >> 5], 1u << (rel & 31));
                        }
                        if (fe == 64u * WQ && f < WAVE) {
                            fe = 64u * q + f;
                            fev = (uint32_t)__builtin_amdgcn_readlane((int)e, (int)f);
                            fe_before = (uint32_t)__builtin_amdgcn_readlane((int)(ol_incl - ol), (int)f);
                            fe_abs = (uint32_t)__builtin_amdgcn_readlane((int)abs, (int)f);
                            fe_nb = (uint32_t)__builtin_amdgcn_readlane((int)t[q].nbits, (int)f);
                            fe_err = (uint32_t)__builtin_amdgcn_readlane(
                                (int)(t[q].ev == EV_ERROR ? t[q].err : (uint32_t)ST_INVALID_DISTANCE), (int)f);
                        }
                        base_tok += (uint32_t)__builtin_popcountll(M[q]);
                        base_byte = (uint32_t)__builtin_amdgcn_readlane((int)ol_incl, 63);
                    }
                    if (fe == 64u * WQ) {   // the window's whole chain is in: the next window
                        ntok += base_tok;
                        nbyte += base_byte;
                        p0 += cur;
                        continue;
                    }
                    ntok += (uint32_t)__builtin_popcountll(M[0] & ((fe >= 64 ? ~0ull : ((1ull << fe) - 1ull))));
#pragma unroll
                    for (int q = 1; q < WQ; ++q) {
                        const uint32_t lo = 64u * q;
                        const uint64_t below = fe <= lo ? 0ull : fe >= lo + 64 ? ~0ull : ((1ull << (fe - lo)) - 1ull);
                        ntok += (uint32_t)__builtin_popcountll(M[q] & below);
                    }
                    if (fev == EV_PARTIAL) {
                        ntok += 1;
                        nbyte += fe_before + (o.cap - fe_abs);
                        p0 += fe + fe_nb;
                    } else {
                        nbyte += fe_before;
                        p0 += fe + (fev == EV_EOB ? fe_nb : 0u);
                    }
                    wev = fev == EV_LIMIT ? (uint32_t)EV_NONE : fev;
                    werr = fev == EV_ERROR ? fe_err : 0u;
                    break;
                }
                wave_sync();
                expand_round(L, o, nbyte);
                if (wmode == 0 && ntok >= 64) {
                    cpt_walk = (uint32_t)(((__builtin_amdgcn_s_memtime() - t_round) << 4) / ntok);
                    walk = !(cpt_spec && cpt_spec < cpt_walk);
                }
                switch (wev) {
                case EV_NONE: pos = p0; break;
                case EV_EOB: pos = p0; block_end = true; break;
                case EV_ERROR: st = (int32_t)werr; stop = true; break;
                case EV_STARVED: pos = p0; stop = true; break;
                default: st = full_status; pos = p0; stop = true; break;
                }
                continue;
            }
            const uint32_t rem = total_bits > S ? total_bits - S : 0;
            // segments keep ~SEG_TOKENS tokens even when the block is short:
            // shorter ones would rarely re-synchronise; lanes past the end of
            // the input simply starve
            uint32_t Lseg = (SEG_TOKENS * est16) >> 4;
            if (Lseg > SEG_MAX_BITS) Lseg = SEG_MAX_BITS;
            Lseg >>= shrink;
            if (Lseg == 0) Lseg = 1;
            (void)rem;
            ensure(S, (WAVE * Lseg + 160) / 8 + 16);
            const uint32_t wb = wbase * 8;
            const uint32_t seg0 = S + lane * Lseg, seg1 = seg0 + Lseg;

            PROF_MARK();
            const LaneRes a = decode_count(L, wb, seg0, seg1, total_bits, T);
            PROF_LAP(2);
            PROF_CNT(13, wave_max(a.trips));
            // cross-lane reads with every lane active (a ternary would run
            // the permute with lane 0 switched off and read 0 from it)
            const uint32_t a_prev = from_prev_lane(a.exit);
            uint32_t start = lane == 0 ? S : a_prev;
            LaneRes b = decode_count(L, wb, start, seg1, total_bits, T);
            PROF_CNT(14, wave_max(b.trips));
#ifdef BPMD_PROF
            if (b.trips > 200 && g_prof_dbg[0] == 0) {
                if (atomicCAS((unsigned long long*)&g_prof_dbg[0], 0ull, 2ull) == 0ull) {
                    g_prof_dbg[1] = lane; g_prof_dbg[2] = start; g_prof_dbg[3] = seg1; g_prof_dbg[4] = S;
                    g_prof_dbg[5] = Lseg; g_prof_dbg[6] = b.trips; g_prof_dbg[7] = b.ev; g_prof_dbg[8] = b.exit;
                    g_prof_dbg[9] = total_bits; g_prof_dbg[10] = a.exit; g_prof_dbg[11] = a.trips; g_prof_dbg[12] = b.n;
                    g_prof_dbg[13] = T.lroot; g_prof_dbg[14] = T.droot; g_prof_dbg[15] = est16;
                }
            }
#endif
            unsigned k;   // last lane of the round
            uint32_t reruns = 0;
            for (;;) {
                PROF_CNT(7, 1);
                ++reruns;
                const uint32_t prev_exit = from_prev_lane(b.exit);
                const bool bad = lane > 0 && start != prev_exit;
                const uint64_t evm = __ballot(b.ev != EV_NONE);
                const uint64_t badm = __ballot(bad);
                const unsigned fe = first_lane(evm), fb = first_lane(badm);
                if (fb > fe || fb == WAVE) {
                    k = fe == WAVE ? WAVE - 1 : fe;
                    break;
                }
                if (bad) {
                    start = prev_exit;
                    b = decode_count(L, wb, start, seg1, total_bits, T);
                }
                PROF_CNT(14, wave_max(bad ? b.trips : 0u));
#ifdef BPMD_PROF
                if (bad && b.trips > 200 && g_prof_dbg[0] == 0) {
                    if (atomicCAS((unsigned long long*)&g_prof_dbg[0], 0ull, 1ull) == 0ull) {
                        g_prof_dbg[1] = lane; g_prof_dbg[2] = start; g_prof_dbg[3] = seg1; g_prof_dbg[4] = S;
                        g_prof_dbg[5] = Lseg; g_prof_dbg[6] = b.trips; g_prof_dbg[7] = b.ev; g_prof_dbg[8] = b.exit;
                        g_prof_dbg[9] = total_bits; g_prof_dbg[10] = fe; g_prof_dbg[11] = fb; g_prof_dbg[12] = b.n;
                        g_prof_dbg[13] = T.lroot; g_prof_dbg[14] = T.droot; g_prof_dbg[15] = est16;
                    }
                }
#endif
            }
            PROF_LAP(3);
            // token and byte offsets within the round; keep the round within
            // the token list and the ring
            uint32_t nn = lane <= k ? b.n : 0, bb = lane <= k ? b.bytes : 0;
            uint32_t n_incl = scan_incl(nn), b_incl = scan_incl(bb);
            {
                const uint64_t over = __ballot(lane <= k && (n_incl > TOT || b_incl > R_MAX));
                const unsigned fo = first_lane(over);
                if (fo == 0) {          // one lane alone is too big: shorter segments
                    ++shrink;
                    continue;
                }
                if (fo <= k) k = fo - 1;
            }
            const uint32_t P = n_incl - nn, O = b_incl - bb;
            for (unsigned i = lane; i < BM_WORDS; i += WAVE) L.u.bitmap[i] = 0;
            wave_sync();
            LaneRes c;
            c.exit = start;
            c.n = 0;
            c.bytes = 0;
            c.ev = EV_NONE;
            c.err = 0;
            c.trips = 0;
            if (lane <= k)
                c = decode_store(L, wb, start, seg1, total_bits, T, P, o.pos + O, o.pos, o.cap, raw);
            wave_sync();
            const uint64_t evm2 = __ballot(lane <= k && c.ev != EV_NONE);
            const unsigned ke = first_lane(evm2);
            const unsigned kl = ke < WAVE ? ke : k;
            const uint32_t round_bytes = __shfl(O + c.bytes, kl);
            const uint32_t round_toks = __shfl(P + c.n, kl);
            const uint32_t kev = ke < WAVE ? __shfl(c.ev, kl) : (uint32_t)EV_NONE;
            const uint32_t kerr = __shfl(c.err, kl);
            const uint32_t kexit = __shfl(c.exit, kl);
            PROF_LAP(4);
            PROF_CNT(15, wave_max(c.trips));
            expand_round(L, o, round_bytes);
            PROF_LAP(5);
            if (round_toks) est16 = ((kexit - S) << 4) / round_toks;
            if (est16 < 16) est16 = 16;
            shrink = 0;
            if (wmode == 0 && round_toks >= 64) {
                cpt_spec = (uint32_t)(((__builtin_amdgcn_s_memtime() - t_round) << 4) / round_toks);
                // pass B ran (nearly) serially: measure a walk round, unless
                // one was measured slower
                walk = cpt_walk ? cpt_walk < cpt_spec : reruns > WALK_PROBE;
            }
            switch (kev) {
            case EV_NONE:
                pos = kexit;
                break;
            case EV_EOB:
                pos = kexit;
                block_end = true;
                break;
            case EV_ERROR:
                st = (int32_t)kerr;
                stop = true;
                break;
            case EV_STARVED:
                pos = kexit;
                stop = true;
                break;
            default:   // EV_FULL / EV_PARTIAL
                st = full_status;
                pos = kexit;
                stop = true;
                break;
            }
        }
        if (stop) break;
        PROF_MARK();
    }
    PROF_MARK();
    ring_flush(L, o, o.flushed, o.pos);
    PROF_LAP(12);
    PROF_FLUSH();
    out_len = o.pos;
    status = st;
}

__global__ void __launch_bounds__(WAVE)
inflate_kernel(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
               const uint32_t* __restrict__ in_len, uint32_t n_msgs, uint8_t* __restrict__ out,
               const uint64_t* __restrict__ out_off, const uint32_t* __restrict__ out_cap,
               uint32_t* __restrict__ out_len, int32_t* __restrict__ status, uint32_t raw,
               const uint32_t* __restrict__ mask_key, uint32_t min_in, uint32_t* __restrict__ qctr,
               const uint32_t* __restrict__ order, const uint32_t* __restrict__ limit)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    WaveLds& L = *reinterpret_cast<WaveLds*>(smem);
    auto run = [&](uint32_t msg) {
        Msg m;
        m.p = in + in_off[msg];
        m.n = in_len[msg];
        m.total = m.n + (raw ? 0u : 4u);
        m.key = mask_key ? mask_key[msg] : 0u;
        Out o;
        o.g = out + out_off[msg];
        o.cap = out_cap[msg];
        o.pos = 0;
        o.flushed = 0;
        uint32_t ol = 0;
        int32_t st = 0;
        inflate_msg(L, m, o, raw != 0, ol, st);
        if (lane_id() == 0) {
            out_len[msg] = ol;
            status[msg] = st;
        }
        wave_sync();
    };
    if (qctr) {
        // work queue: a wave takes the next message when its last one is
        // done, so waves that share a SIMD with more waves (9 per CU on 4
        // SIMDs) take fewer messages instead of setting the launch's end.
        // order/limit: the messages are order[0, *limit) (the long payloads
        // of a lane-kernel batch, pmd_capi.hip inflate_impl)
        const uint32_t end = limit ? *limit : n_msgs;
        for (;;) {
            uint32_t k = 0;
            if (lane_id() == 0) k = atomicAdd(qctr, 1u);
            k = (uint32_t)__builtin_amdgcn_readfirstlane((int)k);
            if (k >= end) break;
            const uint32_t msg = order ? order[k] : k;
            if (min_in && in_len[msg] <= min_in) continue;
            run(msg);
        }
        return;
    }
    // the wave's messages are blockIdx.x + k * gridDim.x; their lengths are
    // read 64 at a time (one per lane) so skipping costs no serial loads.
    // min_in != 0: only payloads longer than min_in (the lane kernel has the rest)
    for (uint64_t first = blockIdx.x; first < n_msgs; first += (uint64_t)WAVE * gridDim.x) {
    const uint64_t mine = first + (uint64_t)lane_id() * gridDim.x;
    uint64_t todo = __ballot(mine < n_msgs && (!min_in || in_len[mine] > min_in));
    while (todo) {
        const uint32_t msg = (uint32_t)(first + (uint64_t)__builtin_ctzll(todo) * gridDim.x);
        todo &= todo - 1;
        run(msg);
    }
    }
}

}  // namespace bpmd

// ---------------------------------------------------------------- launcher

extern "C" unsigned bpmd_diag_grid_override;   // pmd_capi.hip; 0 = size the grid by occupancy
extern "C" void* bpmd_internal_scratch(hipStream_t s, size_t bytes, int which);
#ifndef BPMD_WAVE_QUEUE
#define BPMD_WAVE_QUEUE 1
#endif

extern "C" int bpmd_internal_inflate_keyed_split(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                                           uint32_t n, uint8_t* out, const uint64_t* out_off, const uint32_t* out_cap,
                                           uint32_t* out_len, int32_t* status, uint32_t raw, const uint32_t* mask_key,
                                           uint32_t min_in, hipStream_t stream)
{
    using namespace bpmd;
    if (n == 0) return 0;
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const size_t lds = sizeof(WaveLds);
    const unsigned per_cu = (unsigned)(160 * 1024 / lds);
    unsigned grid = (unsigned)cus * (per_cu ? per_cu : 1);
    if (bpmd_diag_grid_override) grid = bpmd_diag_grid_override;
    if (grid > n) grid = n;
    // more messages than resident waves: a work queue (scratch block 6)
    uint32_t* qctr = nullptr;
    if (BPMD_WAVE_QUEUE && n > grid) {
        qctr = (uint32_t*)bpmd_internal_scratch(stream, 256, 6);
        if (!qctr || hipMemsetAsync(qctr, 0, sizeof(uint32_t), stream) != hipSuccess) return (int)hipErrorOutOfMemory;
    }
    hipLaunchKernelGGL(inflate_kernel, dim3(grid), dim3(WAVE), lds, stream, in, in_off, in_len, n, out, out_off,
                       out_cap, out_len, status, raw, mask_key, min_in, qctr, (const uint32_t*)nullptr,
                       (const uint32_t*)nullptr);
    return (int)hipGetLastError();
}

// The long payloads of a lane-kernel batch: messages order[0, *limit) (a
// device count, known only on the device), one wave each from the work queue.
extern "C" int bpmd_internal_inflate_wave_ordered(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                                                  uint32_t n, uint8_t* out, const uint64_t* out_off,
                                                  const uint32_t* out_cap, uint32_t* out_len, int32_t* status,
                                                  uint32_t raw, const uint32_t* mask_key, const uint32_t* order,
                                                  const uint32_t* limit, hipStream_t stream)
{
    using namespace bpmd;
    if (n == 0) return 0;
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const size_t lds = sizeof(WaveLds);
    const unsigned per_cu = (unsigned)(160 * 1024 / lds);
    unsigned grid = (unsigned)cus * (per_cu ? per_cu : 1);
    if (grid > n) grid = n;
    uint32_t* qctr = (uint32_t*)bpmd_internal_scratch(stream, 256, 6);
    if (!qctr || hipMemsetAsync(qctr, 0, sizeof(uint32_t), stream) != hipSuccess) return (int)hipErrorOutOfMemory;
    hipLaunchKernelGGL(inflate_kernel, dim3(grid), dim3(WAVE), lds, stream, in, in_off, in_len, n, out, out_off,
                       out_cap, out_len, status, raw, mask_key, 0u, qctr, order, limit);
    return (int)hipGetLastError();
}

extern "C" int bpmd_internal_inflate_keyed(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                                           uint32_t n, uint8_t* out, const uint64_t* out_off, const uint32_t* out_cap,
                                           uint32_t* out_len, int32_t* status, uint32_t raw, const uint32_t* mask_key,
                                           hipStream_t stream)
{
    return bpmd_internal_inflate_keyed_split(in, in_off, in_len, n, out, out_off, out_cap, out_len, status, raw,
                                             mask_key, 0u, stream);
}

extern "C" int bpmd_internal_inflate(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint32_t n,
                                     uint8_t* out, const uint64_t* out_off, const uint32_t* out_cap,
                                     uint32_t* out_len, int32_t* status, uint32_t raw, hipStream_t stream)
{
    return bpmd_internal_inflate_keyed(in, in_off, in_len, n, out, out_off, out_cap, out_len, status, raw, nullptr,
                                       stream);
}

extern "C" int bpmd_internal_init_fixed(void)
{
    using namespace bpmd;
    uint8_t lens[288];
    uint16_t sorted[288];
    uint16_t fl[512], fd[32];
    for (int i = 0; i < 144; ++i) lens[i] = 8;
    for (int i = 144; i < 256; ++i) lens[i] = 9;
    for (int i = 256; i < 280; ++i) lens[i] = 7;
    for (int i = 280; i < 288; ++i) lens[i] = 8;
    unsigned root = 9, used = 0;
    if (build_table(BUILD_LENS, lens, 288, fl, &root, &used, sorted) || root != 9) return -1;
    for (int i = 0; i < 32; ++i) lens[i] = 5;
    root = 5;
    if (build_table(BUILD_DISTS, lens, 32, fd, &root, &used, sorted) || root != 5) return -1;
    hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(g_fixed_lens), fl, sizeof fl);
    if (e != hipSuccess) return (int)e;
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_fixed_dists), fd, sizeof fd);
    return (int)e;
}

// round mode of the wave kernel (tests, A/B): 0 automatic, 1 walk rounds only,
// 2 speculative rounds only
extern "C" int bpmd_diag_set_wave_walk(int mode)
{
    using namespace bpmd;
    if (mode < 0 || mode > 2) return -1;
    const uint32_t v = (uint32_t)mode;
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_wave_walk), &v, sizeof v);
}

// diagnostic counters (meaningful only in the -DBPMD_PROF build)
extern "C" int bpmd_diag_counters(unsigned long long* out16, int reset)
{
    using namespace bpmd;
    hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess) return (int)e;
    // (the C++ overload takes the symbol by reference: pass the variable itself)
    if (reset == 2) return (int)hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_prof_dbg), sizeof(unsigned long long) * 16);
    e = hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_prof), sizeof(unsigned long long) * 24);
    if (e != hipSuccess) return (int)e;
    if (reset) {
        unsigned long long z[24] = {0};
        e = hipMemcpyToSymbol(HIP_SYMBOL(g_prof), z, sizeof z);
    }
    return (int)e;
}
