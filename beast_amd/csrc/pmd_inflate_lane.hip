// pmd_inflate_lane.hip -- batched raw-DEFLATE decode, one LANE per message.
//
// Throughput design for large batches of small independent messages (the
// no_context_takeover permessage-deflate case): every lane of a wave64 runs
// the reference's serial decoder (include/boost/beast/zlib/detail/
// inflate_stream.ipp:74-535) on its own message, so no work is speculative
// or repeated and the per-token instruction cost is shared by 64 messages.
// A batch of 64 Ki messages is 1024 waves = 4 per CU: every message of the
// batch is resident at once, and each lane's decode state has to fit in
// 160 KiB / 256 = 640 B of LDS.  That rules out zlib-style lookup tables
// (852 + 592 slots); instead:
//
//  * canonical decode: the 15 code bits, bit-reversed, are compared with the
//    left-justified first code of every length (14 register-resident words
//    per tree, each packing limit << 16 | length << 12 | first index), which
//    gives the code length and the symbol's index in canonical order; one
//    LDS byte read then gives the symbol (inflate_table's sorted[] array,
//    inflate_stream.ipp:632-640).  Literal/length symbols are stored as their
//    low 8 bits; a per-length "first non-literal index" (litend) restores
//    the ninth bit, because within one length canonical order puts literals
//    (< 256) first.
//  * code lengths (inflate_stream.ipp:264-327) are decoded once into a
//    nibble array and a packed length histogram in LDS (pass 1); the sorted
//    symbol arrays are then placed with LDS fetch-adds (pass 2).
//  * output goes straight to the message's slot in global memory and
//    matches read their source back from it: history is the lane's own
//    earlier stores, so no window is kept anywhere.  Match chunks are 16 B
//    (distance >= 16) or 8 B (shorter distances: an in-register repeating
//    pattern), the store of a chunk is issued one loop iteration after its
//    load so the load latency overlaps the next token's decode.
//
// The reference's fill rule (a step needs the bits the slow path would
// NEED, including root / sub-table index bits, bitstream.hpp:109-121) only
// matters within 48 bits of the end of the input; there the exact need is
// recomputed from the canonical limits (a sub-table spans one root prefix
// and is as deep as the longest code under it).
//
// Output semantics per message are those of pmd_inflate.hip (the wave
// kernel): same statuses, lengths and capacity rules.
#include "pmd_common.h"

namespace bpmd {
namespace lpm {

// per-lane LDS layout (bytes)
constexpr unsigned O_LIT = 0;      // u8[288]  literal/length symbols, canonical order (low 8 bits)
constexpr unsigned O_DST = 288;    // u8[32]   distance symbols, canonical order
constexpr unsigned O_HIST = 320;   // u32[16]  pass 1: length histogram (lit | lit<256 << 10 | dist << 20)
                                   //          pass 2: placement cursors (lit | dist << 16)
constexpr unsigned O_LE = 384;     // u16[16]  litend per code length
constexpr unsigned O_CLS = 416;    // u8[20]   code-length code symbols, canonical order
constexpr unsigned O_NIB = 448;    // u8[160]  code lengths, one nibble per symbol
constexpr unsigned STRIDE = 624;   // 64 * 624 = 39 936 B per wave: 4 waves per CU
// messages per wave: lanes past LPW idle, so that LPW = 32 puts two waves on
// every SIMD at 64 Ki messages (BPMD_WPS = 2 caps registers for that occupancy)
#ifndef BPMD_LPW
#define BPMD_LPW 64
#endif
#ifndef BPMD_WPS
#define BPMD_WPS 1
#endif
constexpr unsigned LPW = BPMD_LPW;
static_assert(LPW >= 1 && LPW <= 64, "lanes per wave");

#ifndef BPMD_KLIT
#define BPMD_KLIT 4
#endif
constexpr int KLIT = BPMD_KLIT;   // symbols decoded per iteration when literals lead
static_assert(KLIT >= 1 && KLIT <= 4, "literal bytes are queued in one 32-bit word");
// A second one-chunk match per iteration (decode loop, "One more match"):
// 109 -> 115 GiB/s on C2.  BPMD_NO_DUAL builds without it.
#ifndef BPMD_NO_DUAL
#define BPMD_DUAL
#endif
// ... with up to 3 literals between the two (114 -> 116.5 GiB/s)
#if defined(BPMD_DUAL) && !defined(BPMD_NO_SUFFIX)
#define BPMD_SUFFIX
#endif
#ifndef BPMD_KCL
#define BPMD_KCL 4
#endif
#ifndef BPMD_KNIB
#define BPMD_KNIB 16
#endif
constexpr int KCL = BPMD_KCL;     // code-length symbols per iteration (pass 1; <= 8: 8 x 14 bits fit the reader)
constexpr int KNIB = BPMD_KNIB;   // code lengths placed per iteration (pass 2; a multiple of 8)
static_assert(KCL >= 1 && KCL <= 8 && KNIB % 8 == 0 && KNIB <= 32, "header batching");

enum : uint32_t { S_TYPE, S_DATA, S_SHDR, S_SCOPY, S_DYN, S_PASS1, S_BUILD, S_PASS2, S_DONE };

// Canonical code of up to NB-bit codes, as one word per code length L:
//   Q[L-1] = lim_L << 15 | L << 11 | end_L
// lim_L = left-justified end of the codes of length <= L (NB-bit space),
// end_L = canonical index one past the last code of length L.  The code
// length of the NB-bit reversed code c is that of the smallest lim_L > c;
// an unsigned min of Q - ((c + 1) << 15) finds it without compares (words
// with lim_L <= c wrap to >= 2^31), and a result >= 2^31 means c lies past
// the used code space (an incomplete or empty code: invalid symbol).
template <int NB>
struct Canon {
    uint32_t Q[NB];
    uint32_t root;   // the reference's (clamped) root table bits
};

template <int NB>
__device__ __forceinline__ uint32_t canon_min(const uint32_t (&Q)[NB], uint32_t c)
{
    const uint32_t k1 = (c + 1) << 15;
    uint32_t m = Q[0] - k1;
#pragma unroll
    for (int i = 1; i + 1 < NB; i += 2) {
        const uint32_t x = Q[i] - k1, y = Q[i + 1] - k1;
        m = __builtin_elementwise_min(m, __builtin_elementwise_min(x, y));
    }
    if (NB % 2 == 0) m = __builtin_elementwise_min(m, Q[NB - 1] - k1);
    return m;
}

struct Sym {
    uint32_t L;     // code length
    uint32_t idx;   // canonical index (0 when invalid)
    bool inval;
};

template <int NB>
__device__ __forceinline__ Sym canon_decode(const uint32_t (&Q)[NB], uint32_t c)
{
    const uint32_t m = canon_min<NB>(Q, c);
    Sym r;
    r.inval = (m >> 31) != 0;
    const uint32_t q = m + ((c + 1) << 15);
    r.L = (q >> 11) & 15u;
    const int32_t below = (int32_t)(c - (q >> 15)) >> (NB - (int32_t)r.L);   // in [-count_L, -1]
    r.idx = r.inval ? 0u : (uint32_t)((int32_t)(q & 0x7ffu) + below);
    return r;
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
// type: 0 codes, 1 lens, 2 dists.  cum[l] = first canonical index of length l.
template <int NB>
__device__ __forceinline__ int make_canon(const uint32_t (&c)[16], uint32_t R, int type, Canon<NB>& t,
                                          uint32_t (&cum)[17])
{
    uint32_t hi = 0, lo = 0;
#pragma unroll
    for (int l = NB; l >= 1; --l)
        if (c[l]) lo = l;
#pragma unroll
    for (int l = 1; l <= NB; ++l)
        if (c[l]) hi = l;
    int left = 1;
    bool over = false;
#pragma unroll
    for (int l = 1; l <= NB; ++l) {
        left = 2 * left - (int)c[l];
        over |= left < 0;
    }
    uint32_t lim = 0, cu = 0;
    cum[0] = 0;
#pragma unroll
    for (int l = 1; l <= NB; ++l) {
        cum[l] = cu;
        cu += c[l];
        lim += c[l] << (NB - l);
        t.Q[l - 1] = (lim << 15) | ((uint32_t)l << 11) | cu;
    }
#pragma unroll
    for (int l = NB + 1; l <= 16; ++l) cum[l] = cu;
    if (hi == 0) {   // empty code: a 1-bit root of invalid slots
        t.root = 1;
        return 0;
    }
    const uint32_t r = R < hi ? R : hi;
    t.root = r < lo ? lo : r;
    if (over) return ST_OVER_SUBSCRIBED_LENGTH;
    if (left > 0 && (type == 0 || hi != 1)) return ST_INCOMPLETE_LENGTH_SET;
    return 0;
}

// Input blocks: 16 stream bytes at A + 16*bi, where the payload is
// [s, s+n) (A = payload & ~3).  issue_block() reads only dwords holding at
// least one payload byte -- an aligned dword lies in one page, so nothing
// past the payload's last page is touched -- and finish_block(), run after
// the data has arrived, turns the bytes past the payload into the
// 00 00 FF FF tail (pmd mode) and then zeros.
__device__ __forceinline__ uint4 issue_block(const uint8_t* A, uint32_t bi, uint32_t s, uint32_t n)
{
    const uint32_t b0 = bi * 16;
    if (b0 + 16 <= s + n) return *(const uint4*)(A + b0);
    const uint32_t* A32 = (const uint32_t*)(A + b0);
    uint4 w = make_uint4(0, 0, 0, 0);
    if (b0 + 4 > s && b0 < s + n) w.x = A32[0];
    if (b0 + 8 > s && b0 + 4 < s + n) w.y = A32[1];
    if (b0 + 12 > s && b0 + 8 < s + n) w.z = A32[2];
    if (b0 + 16 > s && b0 + 12 < s + n) w.w = A32[3];
    return w;
}
__device__ __forceinline__ uint32_t finish_dword(uint32_t d, int32_t r0, uint32_t n, uint32_t tail)
{
    // r0: payload index of the dword's first byte
    const int32_t valid = (int32_t)n - r0;
    if (valid >= 4) return d;
    d &= valid <= 0 ? 0u : ((1u << (8 * valid)) - 1u);
    if (tail) {
        const int32_t t2 = (int32_t)n + 2 - r0, t3 = t2 + 1;   // FF FF of 00 00 FF FF
        if (t2 >= 0 && t2 < 4) d |= 0xffu << (8 * t2);
        if (t3 >= 0 && t3 < 4) d |= 0xffu << (8 * t3);
    }
    return d;
}
__device__ __forceinline__ uint4 finish_block(uint4 w, uint32_t bi, uint32_t s, uint32_t n, uint32_t tail)
{
    const uint32_t b0 = bi * 16;
    if (b0 + 16 <= s + n) return w;
    const int32_t r0 = (int32_t)b0 - (int32_t)s;
    return make_uint4(finish_dword(w.x, r0, n, tail), finish_dword(w.y, r0 + 4, n, tail),
                      finish_dword(w.z, r0 + 8, n, tail), finish_dword(w.w, r0 + 12, n, tail));
}

// In-loop input block bi >= 2 (b0 >= 32): one 16-byte load, clamped to end
// at E = the end of the payload's last dword (so it never touches a page
// past the payload), or no load at all past E.  The block's dwords are the
// loaded ones shifted down by m; finish_in() applies that shift and the tail.
__device__ __forceinline__ uint32_t in_shift(uint32_t b0, uint32_t E) { return b0 + 16 > E ? (b0 + 16 - E) >> 2 : 0u; }
__device__ __forceinline__ uint4 finish_in(uint4 w, bool ld, uint32_t bi, uint32_t s, uint32_t n, uint32_t tail,
                                           uint32_t mk)
{
    const uint32_t b0 = bi * 16;
    const uint32_t E = (s + n + 3) & ~3u;
    w = ld ? make_uint4(w.x ^ mk, w.y ^ mk, w.z ^ mk, w.w ^ mk) : make_uint4(0, 0, 0, 0);   // unmask (mk: 0 or the key)
    const uint32_t m = ld ? in_shift(b0, E) : 0u;
    uint4 v = w;
    if (m == 1) v = make_uint4(w.y, w.z, w.w, 0);
    if (m == 2) v = make_uint4(w.z, w.w, 0, 0);
    if (m == 3) v = make_uint4(w.w, 0, 0, 0);
    return finish_block(v, bi, s, n, tail);
}

typedef uint4 uint4_u __attribute__((aligned(1)));
typedef uint2 uint2_u __attribute__((aligned(1)));

// Reads of the lane's own earlier output (match sources) are plain loads:
// within one wave the vector L1 is coherent with the wave's own stores
// (AMDGPU memory model, GFX90A/GFX942: no action is needed for coherence
// between the lanes of a wavefront).

// Store the first n of the sz (8 or 16) bytes of w at o + dst, never past
// o + lim: whole when it fits (spare bytes past n are overwritten by later
// output), byte by byte from registers at the end of the slot.
__device__ __forceinline__ void store_bounded(uint8_t* o, uint32_t dst, uint32_t sz, uint32_t lim, uint4 w)
{
    if (dst + sz <= lim) {
#ifdef BPMD_NT_OUT
        typedef unsigned v4s_ __attribute__((ext_vector_type(4), aligned(1)));
        if (sz == 16) __builtin_nontemporal_store((v4s_){w.x, w.y, w.z, w.w}, (v4s_*)(o + dst));
#else
        if (sz == 16) *(uint4_u*)(o + dst) = w;
#endif
        else *(uint2_u*)(o + dst) = make_uint2(w.x, w.y);
        return;
    }
    const uint32_t k = lim - dst;   // < sz
    const uint32_t d[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j)
        if (j < k) o[dst + j] = (uint8_t)(d[j >> 2] >> (8 * (j & 3)));
}

static __constant__ const uint8_t kClenOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// Diagnostic build only (-DBPMD_PROF): per-wave loop counters.
__device__ unsigned long long g_lprof[16];
#ifdef BPMD_PROF
#define LP_DECL unsigned long long lp_[16] = {0}; unsigned long long lpt_ = __builtin_amdgcn_s_memtime(), lpt0_ = lpt_
#define LP_LAP(i) do { unsigned long long t2_ = __builtin_amdgcn_s_memtime(); lp_[i] += t2_ - lpt_; lpt_ = t2_; } while (0)
#define LP_CNT(i, n) (lp_[i] += (n))
#define LP_FLUSH() do { lp_[0] = __builtin_amdgcn_s_memtime() - lpt0_; if (lane == 0) for (int i_ = 0; i_ < 16; ++i_) atomicAdd(&g_lprof[i_], lp_[i_]); } while (0)
#else
#define LP_DECL
#define LP_LAP(i)
#define LP_CNT(i, n)
#define LP_FLUSH()
#endif

__global__ void __launch_bounds__(64, BPMD_WPS)
inflate_lane_kernel(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                    const uint32_t* __restrict__ in_len, uint32_t n_msgs, uint8_t* __restrict__ out,
                    const uint64_t* __restrict__ out_off, const uint32_t* __restrict__ out_cap,
                    uint32_t* __restrict__ out_len, int32_t* __restrict__ status, uint32_t raw,
                    const uint32_t* __restrict__ mask_key, const uint32_t* __restrict__ hist_len, uint32_t hist_max,
                    uint32_t max_in)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const unsigned lane = threadIdx.x;
    const uint32_t msg = blockIdx.x * LPW + lane;
    uint8_t* T = smem + (lane % LPW) * STRIDE;
    uint32_t* H = (uint32_t*)(T + O_HIST);
    uint16_t* LE = (uint16_t*)(T + O_LE);

    // max_in != 0: only payloads of at most max_in bytes (the rest go to the
    // wave kernel, see inflate_impl in pmd_capi.hip)
    bool valid = lane < LPW && msg < n_msgs;
    if (valid && max_in && in_len[msg] > max_in) valid = false;
    if (__ballot(valid) == 0) return;
    const uint8_t* p = in;
    uint32_t n = 0, cap = 0;
    uint8_t* o = out;
    if (valid) {
        p = in + in_off[msg];
        n = in_len[msg];
        cap = out_cap[msg];
        o = out + out_off[msg];
    }
    const uint32_t tail = raw ? 0u : 4u;
    const int32_t full_status = raw ? ST_OK : ST_NEED_BUFFERS;

    // ---- bit reader.  bb holds up to 64 bits; refills take 32-bit words
    // from q (a 16-byte block, shifted down as it is used), then from nx
    // (the next block, already in registers).  Blocks move nx <- sg <- memory
    // only in the loop's memory section, so decoding never waits on memory.
    // (pointer arithmetic, not integer casts, keeps these global_ loads:
    // flat loads would also count on lgkmcnt and stall every LDS wait)
    const uint32_t s = (uint32_t)((uintptr_t)p & 3);
    const uint8_t* A = p - s;
    // masked payloads (bpmd_read_batch): the dword at A + 4k holds payload
    // bytes 4k - s .. 4k - s + 3, masked with key bytes (j - s) % 4
    // (mask.ipp:38-59), so one rotation of the key unmasks every dword
    const uint32_t mk =
        (valid && mask_key) ? __builtin_amdgcn_alignbit(mask_key[msg], mask_key[msg], 8u * ((0u - s) & 3u)) : 0u;
    // context takeover (bpmd_inflate_takeover_batch): the hist bytes before the
    // slot are the window Beast's inflater keeps across messages
    const uint32_t hist = (valid && hist_len) ? (hist_len[msg] < hist_max ? hist_len[msg] : hist_max) : 0u;
    uint4 q = make_uint4(0, 0, 0, 0), nx = q, sg = q;
    if (valid) {
        const uint4 b0w = issue_block(A, 0, s, n), b1w = issue_block(A, 1, s, n);
        q = finish_block(make_uint4(b0w.x ^ mk, b0w.y ^ mk, b0w.z ^ mk, b0w.w ^ mk), 0, s, n, tail);
        nx = finish_block(make_uint4(b1w.x ^ mk, b1w.y ^ mk, b1w.z ^ mk, b1w.w ^ mk), 1, s, n, tail);
    }
    // block 2 goes through the same clamped load and finish_in() as the loop's
    const uint32_t E_in = (s + n + 3) & ~3u;
    bool sg_ld = valid && 32 < E_in;
    if (sg_ld) sg = *(const uint4*)(A + 32 - 4 * in_shift(32, E_in));
    uint32_t blk = 3, qn = 4, sg_bi = 2;
    bool nx_used = false;   // nx moved into q: refill nx from sg in the next memory section
    uint64_t bb = 0;
    uint32_t nb = 0;
    int32_t tb = (int32_t)(8 * (s + n + tail));   // stream bits not yet moved into bb
    // branchless: in a wave some lane nearly always needs the refill
    auto refill = [&]() {
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
#ifdef BPMD_DUAL
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
#endif
    auto drop = [&](uint32_t k) {
        bb >>= k;
        nb -= k;
    };
    refill();
    refill();
    drop(8 * s);

    uint32_t st = valid ? (raw && n == 0 ? S_DONE : S_TYPE) : S_DONE;
    int32_t result = (valid && raw && n == 0) ? ST_NEED_BUFFERS : ST_OK;
    bool last = false;
    uint32_t pos = 0;

    Canon<15> tl, td;
#pragma unroll
    for (int i = 0; i < 15; ++i) { tl.Q[i] = 0; td.Q[i] = 0; }
    tl.root = 9;
    td.root = 5;

    // header state
    uint32_t nlen = 0, ndist = 0, want = 0, have = 0, prev = 0;
    bool eob_seen = false, cl_empty = false;
    Canon<7> tc;
#pragma unroll
    for (int i = 0; i < 7; ++i) tc.Q[i] = 0;
    tc.root = 1;
    // stored block
    uint32_t srem = 0;
    bool sfull = false, sstarve = false;
    // match copy: bytes left to issue, distance, next output position
    uint32_t crem = 0, cdist = 0, cq = 0;
    uint64_t cpat = 0;
    uint32_t cpat_st = 0;   // dist < 8: 0 pattern not requested, 1 source bytes in flight, 2 pattern ready
    // chunk loaded in the previous memory section, stored in the next one
    bool cst = false, cst_pat = false;
    uint32_t cdst = 0, csz = 0, cpd = 1, csh = 0;
    uint4 cw = make_uint4(0, 0, 0, 0);
#ifdef BPMD_DUAL
    // a second one-chunk match decoded in the same iteration: issued with the
    // first match's chunk, stored right after it
    bool m2 = false, cst2 = false;
    uint32_t m2_dst = 0, m2_len = 0, cdst2 = 0, csz2 = 0;
    int32_t m2_src = 0;
#ifdef BPMD_SUFFIX
    // literals between the two matches: stored after the first match's chunk
    // (two memory sections later), before the second's
    uint32_t l2cnt = 0, l2dst = 0, l2val = 0, l2rcnt = 0, l2rdst = 0, l2rval = 0;
#endif
    uint4 cw3 = cw, cw4 = cw;
#endif
#ifndef BPMD_NO_C32
#define BPMD_C32
#endif
#ifdef BPMD_C32
    uint4 cw2 = cw;   // second half of a 32-byte chunk
#endif
#ifdef BPMD_C64
    uint4 cw3 = cw, cw4 = cw;
#endif
    // byte stores decided by the previous compute section (literal or stored-block bytes)
    uint32_t bcnt = 0, bdst = 0, bval = 0;

    LP_DECL;
    for (;;) {
#ifdef BPMD_DUAL
#ifdef BPMD_SUFFIX
        const bool alive = st != S_DONE || crem != 0 || cst || bcnt != 0 || m2 || cst2 || l2cnt != 0 || l2rcnt != 0;
#else
        const bool alive = st != S_DONE || crem != 0 || cst || bcnt != 0 || m2 || cst2;
#endif
#else
        const bool alive = st != S_DONE || crem != 0 || cst || bcnt != 0;
#endif
        const uint64_t alive_m = __builtin_amdgcn_ballot_w64(alive);
        if (!alive_m) break;
        LP_CNT(1, 1);
        LP_CNT(2, __builtin_popcountll(alive_m));
        LP_CNT(3, __builtin_amdgcn_ballot_w64(st == S_DATA && crem == 0) != 0);
        LP_CNT(4, __builtin_popcountll(__builtin_amdgcn_ballot_w64(st == S_DATA && crem == 0)));
        LP_CNT(5, __builtin_amdgcn_ballot_w64(crem != 0) != 0);
        LP_CNT(6, __builtin_amdgcn_ballot_w64(st != S_DATA && st != S_DONE) != 0);
        LP_CNT(7, __builtin_popcountll(__builtin_amdgcn_ballot_w64(st != S_DATA && st != S_DONE)));
        LP_CNT(13, __builtin_amdgcn_ballot_w64(st == S_PASS1) != 0);
        LP_CNT(14, __builtin_amdgcn_ballot_w64(st == S_PASS2) != 0);
        LP_LAP(15);

        // ================================================ memory section
        // Every global load of the loop is issued here and its data is only
        // used in the next iteration's memory section, so the one wait per
        // iteration covers loads that had a whole decode step to land.
        // Stores go in output order (a chunk's spare tail bytes are always
        // overwritten by a later store), and every load of earlier output
        // is issued after the stores it reads.
        // consume what the previous memory section loaded (the one wait) ...
        // (each loaded variable has exactly one load site and is only read
        // here: a second site would merge into a register copy right after
        // the load, i.e. an immediate wait)
        if (nx_used) nx = finish_in(sg, sg_ld, sg_bi, s, n, tail, mk);
        if (cst) {
            uint4 w = cw;
            if (cst_pat) {
                // the cpd bytes before the match, repeated with period cpd (the
                // match that asked for them may be finished and a new one
                // decoded since: its distance is the request's own, cpd)
                uint64_t v = ((uint64_t)cw.y << 32) | cw.x;
                v >>= 8 * csh;
                v &= (1ull << (8 * cpd)) - 1;
                // (64-bit shifts of 64 or more wrap on the hardware: guard them)
                if (cpd < 8) v |= v << (8 * cpd);
                if (cpd < 4) v |= v << (16 * cpd);
                if (cpd < 2) v |= v << (32 * cpd);
                if (cpat_st == 1) {   // still the current match
                    cpat = v;
                    cpat_st = 2;
                }
                w = make_uint4((uint32_t)v, (uint32_t)(v >> 32), 0, 0);
            }
#ifndef BPMD_EXP_NOSTORE
#ifdef BPMD_C32
#ifdef BPMD_C64
            if (csz == 64) {
                store_bounded(o, cdst, 16, cap, w);
                store_bounded(o, cdst + 16, 16, cap, cw2);
                store_bounded(o, cdst + 32, 16, cap, cw3);
                store_bounded(o, cdst + 48, 16, cap, cw4);
            } else
#endif
            if (csz == 32) {
                // the chunk's used bytes pass cdst + 16, so both halves start inside the slot
                store_bounded(o, cdst, 16, cap, w);
                store_bounded(o, cdst + 16, 16, cap, cw2);
            } else
#endif
                store_bounded(o, cdst, csz, cap, w);
#endif
            cst = false;
            cst_pat = false;
        }
#ifdef BPMD_DUAL
#ifdef BPMD_SUFFIX
        if (l2rcnt) {
#pragma unroll
            for (uint32_t j = 0; j < 3; ++j)
                if (j < l2rcnt) o[l2rdst + j] = (uint8_t)(l2rval >> (8 * j));
            l2rcnt = 0;
        }
#endif
        if (cst2) {
            store_bounded(o, cdst2, 16, cap, cw3);
            if (csz2 == 32) store_bounded(o, cdst2 + 16, 16, cap, cw4);
            cst2 = false;
        }
#endif
        if (bcnt) {
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j)
#ifndef BPMD_EXP_NOSTORE
                if (j < bcnt) o[bdst + j] = (uint8_t)(bval >> (8 * j));
#else
                ;
#endif
            bcnt = 0;
        }
        // ... then issue this iteration's loads
        if (nx_used) {
            const uint32_t b0 = blk * 16, E = (s + n + 3) & ~3u;
            sg_ld = b0 < E;
#ifdef BPMD_NT_IN
            if (sg_ld) {
                typedef unsigned v4a_ __attribute__((ext_vector_type(4)));
                const v4a_ t_ = __builtin_nontemporal_load((const v4a_*)(A + b0 - 4 * in_shift(b0, E)));
                sg = make_uint4(t_.x, t_.y, t_.z, t_.w);
            }
#else
            if (sg_ld) sg = *(const uint4*)(A + b0 - 4 * in_shift(b0, E));
#endif
            sg_bi = blk++;
            nx_used = false;
        }
        LP_LAP(9);
        if (crem) {
#ifdef BPMD_C32
            // 32 bytes per iteration when the source lies a whole 32 back
#ifdef BPMD_C64
            const uint32_t C = (cdist >= 64 && crem > 48) ? 64u : (cdist >= 32 && crem > 16) ? 32u : cdist >= 16 ? 16u : 8u;
#else
            const uint32_t C = (cdist >= 32 && crem > 16) ? 32u : cdist >= 16 ? 16u : 8u;
#endif
#else
            const uint32_t C = cdist >= 16 ? 16u : 8u;
#endif
            bool ld = false;
            int32_t src = 0;   // < 0: in the window before the slot
            if (cdist < 8) {
                const uint32_t adv0 = 8 - 8 % cdist;
                const uint32_t adv = adv0 < crem ? adv0 : crem;
                if (cpat_st == 2) {
                    const uint4 pw = make_uint4((uint32_t)cpat, (uint32_t)(cpat >> 32), 0, 0);
                    store_bounded(o, cq, 8, cap, pw);
                    cq += adv;
                    crem -= adv;
#ifdef BPMD_PAT2
                    // adv0 is a whole number of periods: the same 8 bytes continue the run
                    if (crem) {
                        const uint32_t adv2 = adv0 < crem ? adv0 : crem;
                        store_bounded(o, cq, 8, cap, pw);
                        cq += adv2;
                        crem -= adv2;
                    }
#endif
                } else if (cpat_st == 0) {
                    // the cdist bytes before cq, read as 8 bytes that never
                    // start before the slot
                    ld = true;
                    src = max((int32_t)cq - 8, -(int32_t)hist);
                    csh = (uint32_t)((int32_t)cq - (int32_t)cdist - src);
                    cst_pat = true;
                    cpd = cdist;
                    csz = 8;
                    cpat_st = 1;
                    cdst = cq;
                    cq += adv;
                    crem -= adv;
                }
                // cpat_st == 1 cannot be seen here: the pattern is built in the
                // memory section that follows the one that requested it
            } else {
                ld = true;
                src = (int32_t)cq - (int32_t)cdist;
                csz = C;
                cdst = cq;
                const uint32_t adv = C < crem ? C : crem;
                cq += adv;
                crem -= adv;
            }
            if (ld) {
                // 16 bytes from src: the bytes used all lie in [src, cq); the
                // rest of the 16 may run into the next slot (never stored)
#ifdef BPMD_EXP_NOHLOAD
                cw = make_uint4(src, src + 1, src + 2, src + 3);   // timing experiment only
#else
#ifdef BPMD_NT_HIST
                {
                    typedef unsigned v4u_ __attribute__((ext_vector_type(4), aligned(1)));
                    const v4u_ t_ = __builtin_nontemporal_load((const v4u_*)(o + src));
                    cw = make_uint4(t_.x, t_.y, t_.z, t_.w);
                }
#else
                cw = *(const uint4_u*)(o + src);
#endif
#ifdef BPMD_C32
                if (C >= 32) cw2 = *(const uint4_u*)(o + src + 16);
#ifdef BPMD_C64
                if (C == 64) {
                    cw3 = *(const uint4_u*)(o + src + 32);
                    cw4 = *(const uint4_u*)(o + src + 48);
                }
#endif
#endif
#endif
                cst = true;
            }
        }
#ifdef BPMD_DUAL
#ifdef BPMD_SUFFIX
        if (l2cnt) {   // one section later they are stored, after the first chunk
            l2rcnt = l2cnt;
            l2rdst = l2dst;
            l2rval = l2val;
            l2cnt = 0;
        }
#endif
        if (m2) {
            cw3 = *(const uint4_u*)(o + m2_src);
            if (m2_len > 16) cw4 = *(const uint4_u*)(o + m2_src + 16);
            cst2 = true;
            cdst2 = m2_dst;
            csz2 = m2_len > 16 ? 32u : 16u;
            m2 = false;
        }
#endif
        LP_LAP(11);

        // Input bits per iteration stay <= 108 (the reader always holds >= 160
        // without touching memory): a state entered during an iteration runs
        // from the next one, except that a block header may run in the same
        // iteration as its type bits (<= 74 bits together).
        const uint32_t st0 = st;
        LP_CNT(12, __builtin_popcountll(__builtin_amdgcn_ballot_w64(st == S_DATA && crem == 0)));
        // ================================================ decode a token
        if (st == S_DATA && crem == 0) {
            // Up to KLIT symbols per iteration: while there is room for them
            // (input for KLIT - 1 literals plus a whole token, output for
            // KLIT literals, so no event can occur among them) leading
            // literals are taken directly; the first other symbol -- or, out
            // of room, the first symbol of any kind -- is the iteration's main
            // token, handled with the reference's checks below.  (Deflated
            // text: 65 % of tokens are literals, in runs of ~3.7.)
            refill();
            const bool multi = (tb + (int32_t)nb) >= 48 + 15 * (KLIT - 1) && pos + KLIT <= cap;
            bool found = false;
            uint32_t nlit = 0, lbytes = 0;
            int32_t avail = 0;
            uint32_t c15 = 0, L = 0, sym = 0;
            Sym y;
            bool inval = false;
#pragma unroll
            for (int k = 0; k < KLIT; ++k) {
                if (k > 0) refill();   // appends above the unconsumed bits only: harmless for finished lanes
                const bool act = !found && (k == 0 || multi);
                const uint32_t kc = rev15(bb);
                const Sym ky = canon_decode<15>(tl.Q, kc);
                const uint32_t kle = LE[ky.L];
                const uint32_t ks = T[O_LIT + ky.idx] + (ky.idx >= kle ? 256u : 0u);
                const bool kinv = ky.inval || ks >= 286;
                if (act && multi && !kinv && ks < 256) {
                    drop(ky.L);
                    lbytes |= ks << (8 * nlit);
                    ++nlit;
                } else if (act) {
                    found = true;
                    avail = tb + (int32_t)nb;
                    c15 = kc;
                    y = ky;
                    L = ky.L;
                    sym = ks;
                    inval = kinv;
                }
            }
            if (nlit) {
                bcnt = nlit;
                bdst = pos;
                bval = lbytes;
                pos += nlit;
            }
            if (found) {
                uint32_t need_l = 0;
                if (avail < 48) need_l = canon_need<15>(tl, y, c15);
                // length and distance are decoded for every lane (a wave nearly
                // always holds a match): no divergent branch around them
                const bool is_len = !inval && sym > 256;
                const uint32_t li = is_len ? sym - 257 : 0u;
                const uint32_t xl = (li < 8 || li == 28) ? 0u : ((li - 4) >> 2);
                uint32_t len = li < 8 ? li + 3 : (li == 28 ? 258u : (((4u + (li & 3)) << xl) + 3));
                len += (uint32_t)(bb >> L) & lowmask(xl);
                const uint32_t used = L + (is_len ? xl : 0u);
                drop(used);
                refill();
                const uint32_t d15 = rev15(bb);
                const Sym yd = canon_decode<15>(td.Q, d15);
                const uint32_t Ld = yd.L;
                const uint32_t dsym = T[O_DST + yd.idx];
                const bool invd = yd.inval || dsym >= 30;
                const uint32_t xd = dsym < 4 ? 0u : (dsym >> 1) - 1;
                uint32_t dist = dsym < 4 ? dsym + 1 : (((2u + (dsym & 1)) << xd) + 1);
                dist += (uint32_t)(bb >> Ld) & lowmask(xd);
                uint32_t need_d = 0;
                if (avail < 48 && is_len) need_d = canon_need<15>(td, yd, d15);
                bool is_match = false;
                uint32_t ev = 0;   // 0 token, 1 eob, 2 starved, 3 error
                int32_t err = 0;
                if ((int32_t)need_l > avail) {
                    ev = 2;
                } else if (inval) {
                    ev = 3;
                    err = ST_INVALID_LITERAL_LENGTH;
                } else if (sym == 256) {
                    ev = 1;
                } else if (sym > 256) {
                    if ((int32_t)used > avail || (int32_t)(used + need_d) > avail) {
                        ev = 2;
                    } else if (invd) {
                        ev = 3;
                        err = ST_INVALID_DISTANCE_CODE;
                    } else if ((int32_t)(used + Ld + xd) > avail) {
                        ev = 2;
                    } else {
                        drop(Ld + xd);
                        is_match = true;
                    }
                }
                if (ev == 0) {
                    // output checks in the reference's order (inflate_stream.ipp:475-514)
                    if (raw && pos >= cap) {
                        result = full_status;
                        st = S_DONE;
                    } else if (is_match && dist > pos + hist) {
                        result = ST_INVALID_DISTANCE;
                        st = S_DONE;
                    } else if (pos >= cap) {
                        result = full_status;
                        st = S_DONE;
                    } else {
                        uint32_t olen = is_match ? len : 1u;
                        if (pos + olen > cap) {
                            olen = cap - pos;
                            result = full_status;
                            st = S_DONE;
                        }
                        if (is_match) {
                            crem = olen;
                            cdist = dist;
                            cq = pos;
                            cpat_st = 0;
                        } else {
                            bcnt = 1;
                            bdst = pos;
                            bval = sym;
                        }
                        pos += olen;
#ifdef BPMD_DUAL
                        // One more match this iteration when both copies are one
                        // chunk and the second reads only bytes before the first
                        // (so neither waits for the other); its bits are taken only
                        // if it qualifies.  The reader must hold 48 more bits.
                        const bool one1 = (dist >= 32 && len <= 32) || (dist >= 16 && len <= 16);
                        uint32_t gap = 0;   // literals taken between the two matches
#ifdef BPMD_SUFFIX
                        if (is_match && st == S_DATA && olen == len && one1) {
                            l2val = 0;
#pragma unroll
                            for (int k = 0; k < 3; ++k) {
                                const uint32_t hk = nb + 32u * qn + (nx_used ? 0u : 128u);
                                if (!(hk >= 128 && tb + (int32_t)nb >= 63 && pos < cap && gap == (uint32_t)k)) break;
                                refill();
                                const uint64_t wk = nb >= 64 ? bb : (bb | ((uint64_t)q.x << nb));
                                const Sym yk = canon_decode<15>(tl.Q, rev15(wk));
                                const uint32_t sk = (uint32_t)T[O_LIT + yk.idx] + (yk.idx >= LE[yk.L] ? 256u : 0u);
                                if (yk.inval || sk >= 256) break;
                                drop_x(yk.L);
                                l2val |= sk << (8 * gap);
                                l2dst = gap ? l2dst : pos;
                                ++gap;
                                ++pos;
                            }
                            l2cnt = gap;
                        }
#endif
                        const uint32_t held = nb + 32u * qn + (nx_used ? 0u : 128u);
                        if (is_match && st == S_DATA && olen == len && one1 && held >= 80 &&
                            tb + (int32_t)nb >= 48) {
                            refill();   // nb >= 33: with q.x, a 64-bit window
                            const uint64_t w2 = nb >= 64 ? bb : (bb | ((uint64_t)q.x << nb));
                            const Sym y2 = canon_decode<15>(tl.Q, rev15(w2));
                            const uint32_t sym2 = (uint32_t)T[O_LIT + y2.idx] + (y2.idx >= LE[y2.L] ? 256u : 0u);
                            const bool len_ok = !y2.inval && sym2 > 256 && sym2 < 286;
                            const uint32_t li2 = len_ok ? sym2 - 257 : 0u;
                            const uint32_t xl2 = (li2 < 8 || li2 == 28) ? 0u : ((li2 - 4) >> 2);
                            uint32_t len2 = li2 < 8 ? li2 + 3 : (li2 == 28 ? 258u : (((4u + (li2 & 3)) << xl2) + 3));
                            len2 += (uint32_t)(w2 >> y2.L) & lowmask(xl2);
                            const uint32_t u2 = y2.L + xl2;
                            const uint64_t w2d = w2 >> u2;
                            const Sym yd2 = canon_decode<15>(td.Q, rev15(w2d));
                            const uint32_t dsym2 = T[O_DST + yd2.idx];
                            const uint32_t xd2 = dsym2 < 4 ? 0u : (dsym2 >> 1) - 1;
                            uint32_t dist2 = dsym2 < 4 ? dsym2 + 1 : (((2u + (dsym2 & 1)) << xd2) + 1);
                            dist2 += (uint32_t)(w2d >> yd2.L) & lowmask(xd2);
                            const uint32_t tot2 = u2 + yd2.L + xd2;
                            const uint32_t c2 = len2 <= 16 ? 16u : 32u;   // its one chunk
                            if (len_ok && !yd2.inval && dsym2 < 30 && len2 <= 32 && dist2 >= len + gap + c2 &&
                                dist2 <= pos + hist && pos + len2 <= cap && (int32_t)tot2 <= tb + (int32_t)nb) {
                                drop_x(tot2);
                                m2 = true;
                                m2_dst = pos;
                                m2_src = (int32_t)pos - (int32_t)dist2;
                                m2_len = len2;
                                pos += len2;
                            }
                        }
#endif
                    }
                } else if (ev == 1) {
                    st = S_TYPE;
                } else if (ev == 2) {
                    st = S_DONE;
                } else {
                    result = err;
                    st = S_DONE;
                }
            }
        }
        LP_LAP(8);

        // ======================================= block headers, stored
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
                        uint4* dst4 = (uint4*)T;
#pragma unroll
                        for (int k = 0; k < 20; ++k) {
                            uint32_t w4[4];
#pragma unroll
                            for (int j = 0; j < 4; ++j) {
                                const int i = 16 * k + 4 * j;
                                const int v = i < 24 ? i : i < 168 ? i - 24 : i < 176 ? i - 144 : i < 288 ? i - 32 : i - 288;
                                w4[j] = (uint32_t)v * 0x01010101u + 0x03020100u;
                            }
                            dst4[k] = make_uint4(w4[0], w4[1], w4[2], w4[3]);
                        }
                        LE[7] = 0;
                        LE[8] = 168;
                        LE[9] = 288;
                        uint32_t c[16], cum[17];
#pragma unroll
                        for (int l = 0; l < 16; ++l) c[l] = 0;
                        c[7] = 24;
                        c[8] = 152;
                        c[9] = 112;
                        make_canon<15>(c, 9, 1, tl, cum);
#pragma unroll
                        for (int l = 0; l < 16; ++l) c[l] = 0;
                        c[5] = 32;
                        make_canon<15>(c, 5, 2, td, cum);
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
            if (avail < 32) {
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
                }
            }
        }
        if (st == S_SCOPY) {
            // COPY (inflate_stream.ipp:206-220): up to 4 bytes per iteration,
            // stored by the next memory section (after any literals this
            // iteration already queued before its end of block)
            if (srem && bcnt == 0) {
                refill();
                const uint32_t k = srem < 4 ? srem : 4u;
                bval = (uint32_t)bb;
                bdst = pos;
                bcnt = k;
                drop(8 * k);
                pos += k;
                srem -= k;
            }
            if (srem == 0 && bcnt == 0) {
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
        if (st == S_DYN) {
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
                    uint32_t cl[19];
                    refill();
#pragma unroll
                    for (int i = 0; i < 10; ++i)
                        cl[kClenOrder[i]] = (uint32_t)i < ncode ? ((uint32_t)(bb >> (3 * i)) & 7u) : 0u;
                    drop(3 * (ncode < 10 ? ncode : 10u));
                    refill();
#pragma unroll
                    for (int i = 10; i < 19; ++i)
                        cl[kClenOrder[i]] = (uint32_t)i < ncode ? ((uint32_t)(bb >> (3 * (i - 10))) & 7u) : 0u;
                    drop(3 * (ncode > 10 ? ncode - 10 : 0u));
                    // code-length code (inflate_stream.ipp:249-262)
                    uint64_t acc = 0;
#pragma unroll
                    for (int i = 0; i < 19; ++i) acc += 1ull << (5 * cl[i]);
                    uint32_t c[16], cum[17];
#pragma unroll
                    for (int l = 0; l < 16; ++l) c[l] = (l >= 1 && l <= 7) ? (uint32_t)(acc >> (5 * l)) & 31u : 0u;
                    const int e = make_canon<7>(c, 7, 0, tc, cum);
                    cl_empty = c[1] + c[2] + c[3] + c[4] + c[5] + c[6] + c[7] == 0;
                    if (e) {
                        result = e;
                        st = S_DONE;
                    } else {
                        uint64_t offs = 0;
#pragma unroll
                        for (int l = 1; l <= 7; ++l) offs |= (uint64_t)cum[l] << (5 * l);
#pragma unroll
                        for (int i = 0; i < 19; ++i) {
                            const uint32_t l = cl[i];
                            const uint32_t at = (uint32_t)(offs >> (5 * l)) & 31u;
                            offs += 1ull << (5 * l);
                            if (l) T[O_CLS + at] = (uint8_t)i;
                        }
                        uint64_t* nib = (uint64_t*)(T + O_NIB);
#pragma unroll
                        for (int k = 0; k < 20; ++k) nib[k] = 0;
                        uint4* h4 = (uint4*)H;
#pragma unroll
                        for (int k = 0; k < 4; ++k) h4[k] = make_uint4(0, 0, 0, 0);
                        want = nlen + ndist;
                        have = 0;
                        prev = 0;
                        eob_seen = false;
                        st = S_PASS1;
                    }
                }
            }
        }
#ifdef BPMD_P1_BRANCHLESS
#pragma unroll
        for (int kc = 0; kc < KCL; ++kc) {
            if (st != S_PASS1 || st0 != S_PASS1) break;
            // CODELENS (inflate_stream.ipp:264-327) with the outcomes as selects
            refill();
            const int32_t avail = tb + (int32_t)nb;
            const uint32_t c7 = __builtin_bitreverse32((uint32_t)bb) >> 25;
            const Sym yc = canon_decode<7>(tc.Q, c7);
            const uint32_t L = cl_empty ? 1u : yc.L;
            const uint32_t csym = cl_empty ? 0u : (uint32_t)T[O_CLS + (yc.idx < 19 ? yc.idx : 0u)];
            const bool rpt = csym >= 16;
            const uint32_t xb = csym == 16 ? 2u : csym == 17 ? 3u : csym == 18 ? 7u : 0u;
            const uint32_t x = (uint32_t)(bb >> L) & lowmask(xb);
            const uint32_t used = L + xb;
            const uint32_t rep = csym == 16 ? 3u + x : csym == 17 ? 3u + x : csym == 18 ? 11u + x : 1u;
            const uint32_t val = csym == 16 ? prev : (rpt ? 0u : csym);
            const bool starve = avail < (int32_t)tc.root || (rpt && avail < (int32_t)used);
            const bool bad = !starve && rpt && ((csym == 16 && have == 0) || have + rep > want);
            const bool ok = !starve && !bad;
            result = bad ? ST_INVALID_BIT_LENGTH_REPEAT : result;
            st = ok ? st : S_DONE;
            drop(ok ? used : 0u);
            const bool wr = ok && val != 0;   // then rep <= 6
            const uint32_t a = have, rw = wr ? rep : 0u, b = have + rw;
            const uint64_t pat = ((uint64_t)val * 0x1111111111111111ull) & ((1ull << (4 * rw)) - 1);
            const uint64_t v = pat << ((a & 7) * 4);
            uint32_t* nw = (uint32_t*)(T + O_NIB) + (a >> 3);
            __hip_atomic_fetch_or(nw, (uint32_t)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __hip_atomic_fetch_or(nw + 1, (uint32_t)(v >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            const uint32_t e_l = b < nlen ? b : nlen;
            const uint32_t nl = e_l > a ? e_l - a : 0u;
            const uint32_t e_o = b < 256 ? b : 256u;
            const uint32_t nlo = e_o > a ? e_o - a : 0u;
            const uint32_t s_d = a > nlen ? a : nlen;
            const uint32_t nd = b > s_d ? b - s_d : 0u;
            __hip_atomic_fetch_add(H + val, nl | (nlo << 10) | (nd << 20), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WORKGROUP);
            eob_seen = eob_seen || (wr && a <= 256 && 256 < b);
            prev = ok ? val : prev;
            have += ok ? rep : 0u;
            st = (ok && have == want) ? S_BUILD : st;
        }
#else
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
                    csym = T[O_CLS + (yc.idx < 19 ? yc.idx : 0u)];
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
                            uint32_t* nw = (uint32_t*)(T + O_NIB) + (a >> 3);
                            __hip_atomic_fetch_or(nw, (uint32_t)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                            if ((uint32_t)(v >> 32))
                                __hip_atomic_fetch_or(nw + 1, (uint32_t)(v >> 32), __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_WORKGROUP);
                            const uint32_t e_l = b < nlen ? b : nlen;
                            const uint32_t nl = e_l > a ? e_l - a : 0u;
                            const uint32_t e_o = b < 256 ? b : 256u;
                            const uint32_t nlo = e_o > a ? e_o - a : 0u;
                            const uint32_t s_d = a > nlen ? a : nlen;
                            const uint32_t nd = b > s_d ? b - s_d : 0u;
                            __hip_atomic_fetch_add(H + val, nl | (nlo << 10) | (nd << 20), __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_WORKGROUP);
                            if (a <= 256 && 256 < b) eob_seen = true;
                        }
                        prev = val;
                        have += rep;
                        if (have == want) st = S_BUILD;
                    }
                }
        }
#endif
        if (st == S_BUILD) {
            if (!eob_seen) {
                result = ST_MISSING_EOB;
                st = S_DONE;
            } else {
                uint32_t h[16];
                const uint4* h4 = (const uint4*)H;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const uint4 v = h4[k];
                    h[4 * k] = v.x;
                    h[4 * k + 1] = v.y;
                    h[4 * k + 2] = v.z;
                    h[4 * k + 3] = v.w;
                }
                uint32_t c[16], cuml[17], cumd[17];
                c[0] = 0;
#pragma unroll
                for (int l = 1; l < 16; ++l) c[l] = h[l] & 0x3ffu;
                int e = make_canon<15>(c, 9, 1, tl, cuml);
                if (!e) {
#pragma unroll
                    for (int l = 1; l < 16; ++l) c[l] = (h[l] >> 20) & 0x3ffu;
                    e = make_canon<15>(c, 6, 2, td, cumd);
                }
                if (e) {
                    result = e;
                    st = S_DONE;
                } else {
                    uint32_t lev[16];
                    lev[0] = 0;
#pragma unroll
                    for (int l = 1; l < 16; ++l) lev[l] = cuml[l] + ((h[l] >> 10) & 0x3ffu);
                    uint4* le4 = (uint4*)LE;
                    le4[0] = make_uint4(lev[0] | (lev[1] << 16), lev[2] | (lev[3] << 16), lev[4] | (lev[5] << 16),
                                        lev[6] | (lev[7] << 16));
                    le4[1] = make_uint4(lev[8] | (lev[9] << 16), lev[10] | (lev[11] << 16),
                                        lev[12] | (lev[13] << 16), lev[14] | (lev[15] << 16));
                    uint4* h4w = (uint4*)H;
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        h4w[k] = make_uint4(cuml[4 * k] | (cumd[4 * k] << 16), cuml[4 * k + 1] | (cumd[4 * k + 1] << 16),
                                            cuml[4 * k + 2] | (cumd[4 * k + 2] << 16),
                                            cuml[4 * k + 3] | (cumd[4 * k + 3] << 16));
                    have = 0;
                    st = S_PASS2;
                }
            }
        }
        if (st == S_PASS2) {
            // place symbols in canonical order (inflate_stream.ipp:632-640)
#pragma unroll
            for (uint32_t h8 = 0; h8 < KNIB; h8 += 8) {
                const uint32_t w = ((const uint32_t*)(T + O_NIB))[(have + h8) >> 3];
                uint32_t olds[8];
                // all fetch-adds first (no branch between them), then the
                // placements: one LDS round trip for the eight
#pragma unroll
                for (uint32_t k = 0; k < 8; ++k) {
                    const uint32_t i = have + h8 + k;
                    const uint32_t l = (w >> (4 * k)) & 15u;
                    const uint32_t inc = (l && i < want) ? (i < nlen ? 1u : 0x10000u) : 0u;
                    olds[k] = __hip_atomic_fetch_add(H + l, inc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
#pragma unroll
                for (uint32_t k = 0; k < 8; ++k) {
                    const uint32_t i = have + h8 + k;
                    const uint32_t l = (w >> (4 * k)) & 15u;
#ifdef BPMD_P2_BRANCHLESS
                    // one store per symbol, no branch: unused placements land on
                    // a spare byte past the code-length symbols
                    const bool use = l && i < want, lit = i < nlen;
                    const uint32_t at = !use ? O_CLS + 31u : lit ? O_LIT + (olds[k] & 0xffffu) : O_DST + (olds[k] >> 16);
                    T[at] = (uint8_t)(lit ? i : i - nlen);
#else
                    if (l && i < want) {
                        if (i < nlen) T[O_LIT + (olds[k] & 0xffffu)] = (uint8_t)i;
                        else T[O_DST + (olds[k] >> 16)] = (uint8_t)(i - nlen);
                    }
#endif
                }
            }
            have += KNIB;
            if (have >= want) st = S_DATA;
        }

        LP_LAP(10);
    }
    LP_FLUSH();
    if (valid) {
        out_len[msg] = pos;
        status[msg] = result;
    }
}

}  // namespace lpm
}  // namespace bpmd

extern "C" int bpmd_internal_inflate_lane_split(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                                                uint32_t n, uint8_t* out, const uint64_t* out_off,
                                                const uint32_t* out_cap, uint32_t* out_len, int32_t* status,
                                                uint32_t raw, const uint32_t* mask_key, const uint32_t* hist_len,
                                                uint32_t hist_max, uint32_t max_in, hipStream_t stream)
{
    using namespace bpmd::lpm;
    if (n == 0) return 0;
    const unsigned grid = (n + LPW - 1) / LPW;
    hipLaunchKernelGGL(inflate_lane_kernel, dim3(grid), dim3(64), LPW * STRIDE, stream, in, in_off, in_len, n, out,
                       out_off, out_cap, out_len, status, raw, mask_key, hist_len, hist_max, max_in);
    return (int)hipGetLastError();
}

extern "C" int bpmd_internal_inflate_lane(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                                          uint32_t n, uint8_t* out, const uint64_t* out_off,
                                          const uint32_t* out_cap, uint32_t* out_len, int32_t* status, uint32_t raw,
                                          const uint32_t* mask_key, const uint32_t* hist_len, uint32_t hist_max,
                                          hipStream_t stream)
{
    return bpmd_internal_inflate_lane_split(in, in_off, in_len, n, out, out_off, out_cap, out_len, status, raw,
                                            mask_key, hist_len, hist_max, 0u, stream);
}

extern "C" int bpmd_internal_init_fixed_lane(void)
{
    // nothing to upload: the fixed tables are computed arithmetically (S_TYPE)
    return 0;
}

// diagnostic counters of the lane kernel (meaningful only in the -DBPMD_PROF build)
extern "C" int bpmd_diag_lane_counters(unsigned long long* out16, int reset)
{
    using namespace bpmd::lpm;
    hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess) return (int)e;
    e = hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_lprof), sizeof(unsigned long long) * 16);
    if (e != hipSuccess) return (int)e;
    if (reset) {
        unsigned long long z[16] = {0};
        e = hipMemcpyToSymbol(HIP_SYMBOL(g_lprof), z, sizeof z);
    }
    return (int)e;
}
