// pmd_inflate_lane4.hip -- batched raw-DEFLATE decode, one LANE per message,
// table-driven (round 4).  Same two-wave organisation as pmd_inflate_lane3.hip
// (a DECODER wave and an EXPANDER wave per group of messages, joined by a
// per-message token ring in LDS), but the decoder looks symbols up in
// per-message Huffman tables instead of running a canonical search:
//
//   lane3: a 15-word unsigned-min search per symbol (~34 VALU instructions,
//          ~170 of the ~600 issue slots of a data step) so that each message
//          needs only 632 B of LDS and all 64 Ki C2 messages are in flight;
//   lane4: one LDS read per symbol (root table indexed by the next RL code
//          bits, a uniform-depth sub-table for the longer codes), ~1.2 KiB of
//          LDS per message, so fewer messages are in flight (128 per CU) but
//          each decodes several times faster.
//
// Every decision the reference takes per symbol (inflate_stream.ipp:74-535:
// invalid codes, the fill rule near the end of the input, end of block,
// output capacity, distance too far back) is made exactly as in lane3, from
// the same (code length, symbol) pair: the canonical words are still built
// (make_canon validates the code lengths and gives the reference's fill rule
// near the end of the input), only the per-symbol decode reads a table.
//
// A block whose longer codes do not fit the sub-table budget (never seen on
// Beast's 4 KiB messages; possible for adversarial code lengths) ends the
// lane's message with the internal status FB4: the message is appended to a
// device-side list that the lane3 kernel decodes after this launch, so the
// result is always the exact one.
//
// The expander takes up to KX pieces (a token's literal bytes and one chunk
// of its match) per iteration and issues all their match loads before it
// waits for any: a match whose source lies wholly below the output already
// stored is independent of the pieces before it in the batch.  The loaded
// chunks are stored at the start of the next iteration, in output order.
#include <stdlib.h>
#include <string.h>

#include <atomic>

#include "pmd_common.h"
#include "canon.h"
#include "lane_io.h"

namespace bpmd {
namespace lp4 {
using namespace lio;
using lp3::Canon;
using lp3::Sym;
using lp3::canon_need;
using lp3::lowmask;
using lp3::make_canon;

#ifndef BPMD4_RL
#define BPMD4_RL 8
#endif
#ifndef BPMD4_RD
#define BPMD4_RD 5
#endif
#ifndef BPMD4_SUBL
#define BPMD4_SUBL 128
#endif
#ifndef BPMD4_SUBD
#define BPMD4_SUBD 16
#endif
#ifndef BPMD4_LANES
#define BPMD4_LANES 32
#endif
#ifndef BPMD4_KL
#define BPMD4_KL 2
#endif
#ifndef BPMD4_KX
#define BPMD4_KX 4
#endif
#ifndef BPMD4_KCL
#define BPMD4_KCL 6
#endif
#ifndef BPMD4_KNIB
#define BPMD4_KNIB 32
#endif

constexpr uint32_t RL = BPMD4_RL;      // literal/length root table bits
constexpr uint32_t RD = BPMD4_RD;      // distance root table bits
constexpr uint32_t SUBL = BPMD4_SUBL;  // literal/length sub-table entries (codes longer than RL)
constexpr uint32_t SUBD = BPMD4_SUBD;  // distance sub-table entries
constexpr uint32_t RING = 32;          // token ring entries per message
constexpr uint32_t LANES = BPMD4_LANES;   // messages per wave (active lanes)
constexpr int KL = BPMD4_KL;           // symbols decoded per data step when literals lead
constexpr int KX = BPMD4_KX;           // expander pieces per iteration
constexpr int KCL = BPMD4_KCL;         // code-length symbols per header iteration
constexpr int KNIB = BPMD4_KNIB;       // symbols placed per table-fill iteration

// per-lane LDS layout (bytes)
constexpr uint32_t O_LR = 0;                      // u16[1 << RL]  literal/length root
constexpr uint32_t O_LS = O_LR + (2u << RL);      // u16[SUBL]     literal/length sub-table
constexpr uint32_t O_DR = O_LS + 2u * SUBL;       // u32[1 << RD]  distance root
constexpr uint32_t O_DS = O_DR + (4u << RD);      // u32[SUBD]     distance sub-table
constexpr uint32_t O_RG = O_DS + 4u * SUBD;       // token ring; during a header the scratch below
constexpr uint32_t O_NIB = O_RG;                  //   u8[160]  code lengths, one nibble per symbol
constexpr uint32_t O_HIST = O_RG + 160;           //   u32[16]  length histogram, then fill cursors
constexpr uint32_t O_CLS = O_RG + 224;            //   u8[20]   code-length code symbols, canonical order
constexpr uint32_t O_HEAD = O_RG + 8u * RING;     // u32 tokens written (decoder)
constexpr uint32_t O_TAIL = O_HEAD + 4;           // u32 tokens taken (expander)
constexpr uint32_t STRIDE = (O_TAIL + 4 + 15) & ~15u;
static_assert(8 * RING >= 244, "the header scratch lives in the ring");
static_assert(O_LS % 16 == 0 && O_DR % 16 == 0 && O_DS % 16 == 0, "tables are filled with 16-byte stores");

// literal/length entry (u16): bits 0-3 code length, 4-7 kind, 8-15 value
constexpr uint32_t K_LIT = 6, K_EOB = 7, K_BAD = 8, K_SUB = 9;   // kind 0-5: length code, kind = extra bits, value = base - 3
// distance entry (u32): bits 0-3 code length, 4-7 extra bits (or kind), 8-23 base
constexpr uint32_t DK_BAD = 14, DK_SUB = 15;

constexpr int32_t ST_FB4 = 120;   // internal: re-decode this message with the lane3 kernel

constexpr uint32_t TOK_END = 0x80000000u;
constexpr uint32_t TOK_NEW = 0x40000000u;
constexpr uint32_t TOK_EXIT = 0x20000000u;

enum : uint32_t { S_TYPE, S_DATA, S_SHDR, S_SCOPY, S_DYN, S_FIX, S_PASS1, S_BUILD, S_PASS2, S_DONE };

__device__ __forceinline__ unsigned ring_at(uint32_t e) { return O_RG + 8u * (e % RING); }

__device__ __forceinline__ uint32_t lit_entry(uint32_t sym, uint32_t l)
{
    if (sym < 256) return l | (K_LIT << 4) | (sym << 8);
    if (sym == 256) return l | (K_EOB << 4);
    if (sym < 286) {
        const uint32_t li = sym - 257;
        const uint32_t xl = (li < 8 || li == 28) ? 0u : ((li - 4) >> 2);
        const uint32_t base = li < 8 ? li + 3 : (li == 28 ? 258u : (((4u + (li & 3)) << xl) + 3));
        return l | (xl << 4) | ((base - 3) << 8);
    }
    return l | (K_BAD << 4);
}
__device__ __forceinline__ uint32_t dist_entry(uint32_t ds, uint32_t l)
{
    if (ds >= 30) return l | (DK_BAD << 4);
    const uint32_t xd = ds < 4 ? 0u : (ds >> 1) - 1;
    const uint32_t base = ds < 4 ? ds + 1 : (((2u + (ds & 1)) << xd) + 1);
    return l | (xd << 4) | (base << 8);
}
// bytes (a power of two >= the entry size) of copies of the entry at p (aligned to bytes)
__device__ __forceinline__ void fill_entries(uint8_t* p, uint32_t bytes, uint32_t e32)
{
    if (bytes >= 16) {
        const uint4 r = make_uint4(e32, e32, e32, e32);
        for (uint32_t u = 0; u < bytes; u += 16) *(uint4*)(p + u) = r;
    } else if (bytes == 8) {
        *(uint2*)p = make_uint2(e32, e32);
    } else if (bytes == 4) {
        *(uint32_t*)p = e32;
    } else {
        *(uint16_t*)p = (uint16_t)e32;
    }
}

static __constant__ const uint8_t kClenOrder4[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// ------------------------------------------------------------------ expander
__device__ __forceinline__ void expander(uint8_t* T, bool valid, uint32_t m, uint8_t* __restrict__ out,
                                         const uint64_t* __restrict__ out_off, const uint32_t* __restrict__ out_cap,
                                         uint32_t* __restrict__ out_len, int32_t* __restrict__ status,
                                         const uint32_t* __restrict__ hist_len, uint32_t hist_max, bool queue,
                                         uint32_t* __restrict__ fb)
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
    for (;;) {
        bool pending = false;
#pragma unroll
        for (int j = 0; j < KX; ++j) pending = pending || l_n[j] != 0 || m_sz[j] != 0;
        if (!__ballot(!exited || crem != 0 || pending)) break;
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
            const uint32_t head = lds_load(T + O_HEAD);
            compiler_fence();
            uint2 ent[KX];
#pragma unroll
            for (int j = 0; j < KX; ++j) ent[j] = *(const uint2*)(T + ring_at(tail + j));
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
                        for (int i = 1; i <= j; ++i) e = k == (uint32_t)i ? ent[i] : e;
                        if (e.y & TOK_END) {
                            out_len[m] = e.x;
                            const int32_t stt = (int32_t)(int8_t)(e.y & 0xffu);
                            status[m] = stt;
                            if (stt == ST_FB4) fb[1 + atomicAdd(fb, 1u)] = m;
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
            lds_store(T + O_TAIL, tail);
        }
        if (!__ballot(worked)) __builtin_amdgcn_s_sleep(4);   // the decoder is behind
    }
}

// ------------------------------------------------------------------- decoder
__device__ __forceinline__ void decoder(uint8_t* T, bool valid, uint32_t m, const uint8_t* __restrict__ in,
                                        const uint64_t* __restrict__ in_off, const uint32_t* __restrict__ in_len,
                                        const uint32_t* __restrict__ out_cap, uint32_t raw,
                                        const uint32_t* __restrict__ mask_key, const uint32_t* __restrict__ hist_len,
                                        uint32_t hist_max, uint32_t n_msgs, const uint32_t* __restrict__ order,
                                        uint32_t* __restrict__ qctr, uint32_t s0, uint32_t subl_cap, uint32_t subd_cap)
{
    uint32_t* H = (uint32_t*)(T + O_HIST);
    const uint16_t* LR = (const uint16_t*)(T + O_LR);
    const uint16_t* LS = (const uint16_t*)(T + O_LS);
    const uint32_t* DR = (const uint32_t*)(T + O_DR);
    const uint32_t* DS = (const uint32_t*)(T + O_DS);
    const uint32_t tail = raw ? 0u : 4u;
    const int32_t full_status = raw ? ST_OK : ST_NEED_BUFFERS;
    // per-message state (set by begin())
    const uint8_t* A = in;
    uint32_t s = 0, n = 0, cap = 0, mk = 0, hist = 0;
    // bit reader (as lane3): bb holds up to 64 bits; refills take 32-bit
    // words from q, then from nx; blocks move nx <- sg <- memory only in
    // the loop's input pipeline, so decoding never waits on memory
    uint4 q = make_uint4(0, 0, 0, 0), nx = q, sg = q;
    bool sg_ld = false;
    uint32_t blk = 3, qn = 4, sg_bi = 2;
    bool nx_used = false;
    uint64_t bb = 0;
    uint32_t nb = 0;
    int32_t tb = 0;   // stream bits not yet moved into bb
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
    auto drop_x = [&](uint32_t t) {   // consume t <= 60 bits of bb | q.x << nb (nb >= 33)
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
    Canon<15> tl, td;   // canonical words: validation and the fill rule near the end
    Canon<7> tc;
    // table geometry of the current block: sub-table index = (code32 >> sh) - base
    uint32_t lsh = 0, lbase = 0, dsh = 0, dbase = 0, lmax = 0, dmax = 0;
    // header state
    uint32_t nlen = 0, ndist = 0, want = 0, have = 0, prev = 0;
    bool eob_seen = false, cl_empty = false;
    uint32_t srem = 0;
    bool sfull = false, sstarve = false;
    uint32_t msg = m;
    bool send_new = false, send_exit = false, exhausted = qctr == nullptr;
    const uint32_t first_slots = s0 + gridDim.x * LANES;
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
        cap = out_cap[mm];
        const uint8_t* p = in + in_off[mm];
        const uint32_t s_ = (uint32_t)((uintptr_t)p & 3);
        // masked payloads (bpmd_read_batch): one rotation of the key unmasks every dword (mask.ipp:38-59)
        mk = mask_key ? __builtin_amdgcn_alignbit(mask_key[mm], mask_key[mm], 8u * ((0u - s_) & 3u)) : 0u;
        // context takeover: the hist bytes before the slot are the inflater's window
        hist = hist_len ? (hist_len[mm] < hist_max ? hist_len[mm] : hist_max) : 0u;
        open_view(p, in_len[mm]);
        drop(8 * s);
        st = raw && n == 0 ? S_DONE : S_TYPE;
        result = raw && n == 0 ? ST_NEED_BUFFERS : ST_OK;
        last = false;
        fin = false;
        pos = 0;
        srem = 0;
    };
    auto pipe = [&]() {
        if (__ballot(sg_bi * 16 + 16 > s + n)) nx = finish_in(sg, sg_ld, sg_bi, s, n, tail, mk);
        else nx = make_uint4(sg.x ^ mk, sg.y ^ mk, sg.z ^ mk, sg.w ^ mk);
        const uint32_t b0 = blk * 16, E = (s + n + 3) & ~3u;
        sg_ld = b0 < E;
        if (sg_ld) sg = *(const uint4*)(A + b0 - 4 * in_shift(b0, E));
        sg_bi = blk++;
        nx_used = false;
    };
    // literal/length entry of the code whose first bit is the lsb of x
    auto lit_lookup = [&](uint32_t x) -> uint32_t {
        const uint32_t c = __builtin_bitreverse32(x);
        uint32_t e = LR[c >> (32 - RL)];
        if (__ballot(((e >> 4) & 15u) == K_SUB)) {
            if (((e >> 4) & 15u) == K_SUB) e = LS[(c >> lsh) - lbase];
        }
        return e;
    };
    auto dist_lookup = [&](uint32_t x) -> uint32_t {
        const uint32_t c = __builtin_bitreverse32(x);
        uint32_t e = DR[c >> (32 - RD)];
        if (__ballot(((e >> 4) & 15u) == DK_SUB)) {
            if (((e >> 4) & 15u) == DK_SUB) e = DS[(c >> dsh) - dbase];
        }
        return e;
    };
    // One token of a Huffman block: up to KL leading literals and a main
    // symbol, with lane3's checks (pmd_inflate_lane3.hip data_step).
    auto data_step = [&](uint32_t& enl, uint32_t& elit, uint32_t& emlen, uint32_t& edist) {
        refill();   // nb >= 33: with q.x, a 64-bit window
        const uint64_t w = nb >= 64 ? bb : (bb | ((uint64_t)q.x << nb));
        const bool multi = (tb + (int32_t)nb) >= 48 + 15 * (KL - 1) && pos + KL <= cap;
        uint32_t kp[KL + 1], ke[KL];
        kp[0] = 0;
#pragma unroll
        for (int k = 0; k < KL; ++k) {
            ke[k] = lit_lookup((uint32_t)(w >> kp[k]));
            const uint32_t kind = (ke[k] >> 4) & 15u;
            kp[k + 1] = kp[k] + (kind == K_BAD ? 15u : (ke[k] & 15u));
        }
        uint32_t nlit = 0, lbytes = 0;
#pragma unroll
        for (int k = 0; k < KL; ++k) {
            const bool take = multi && nlit == (uint32_t)k && ((ke[k] >> 4) & 15u) == K_LIT;
            lbytes |= take ? (ke[k] >> 8) << (8 * k) : 0u;
            nlit += take ? 1u : 0u;
        }
        uint32_t lit_bits = 0;
#pragma unroll
        for (int k = 1; k <= KL; ++k) lit_bits = nlit == (uint32_t)k ? kp[k] : lit_bits;
        enl = nlit;
        elit = lbytes;
        pos += nlit;
        // the main token: symbol nlit (none when all KL were literals)
        uint32_t e = ke[0], pm = 0;
#pragma unroll
        for (int k = 1; k < KL; ++k) {
            e = nlit == (uint32_t)k ? ke[k] : e;
            pm = nlit == (uint32_t)k ? kp[k] : pm;
        }
        const uint32_t c15 = __builtin_bitreverse32((uint32_t)(w >> pm)) >> 17;
        const uint32_t kind = (e >> 4) & 15u;
        const uint32_t L = e & 15u;
        const bool inval = kind == K_BAD;
        drop_x(lit_bits);
        const bool mt = nlit < (uint32_t)KL;
        refill();   // nb >= 33 again: the main token's <= 48 bits are in the window
        const uint64_t w2 = nb >= 64 ? bb : (bb | ((uint64_t)q.x << nb));
        const int32_t avail = tb + (int32_t)nb;
        const bool near_end = __ballot(mt && avail < 48) != 0;
        Sym y;
        y.L = L;
        y.idx = 0;
        y.inval = inval;
        uint32_t need_l = 0;
        if (near_end && mt && avail < 48) need_l = canon_need<15>(tl, y, c15);
        const bool is_len = kind <= 5u;
        const uint32_t xl = is_len ? kind : 0u;
        const uint32_t len = (e >> 8) + 3 + ((uint32_t)(w2 >> L) & lowmask(xl));
        const uint32_t used = L + xl;
        const uint32_t de = dist_lookup((uint32_t)(w2 >> used));
        const uint32_t Ld = de & 15u, dk = (de >> 4) & 15u;
        const bool invd = dk == DK_BAD;
        const uint32_t xd = invd ? 0u : dk;
        const uint32_t dist = (de >> 8) + ((uint32_t)(w2 >> (used + Ld)) & lowmask(xd));
        uint32_t need_d = 0;
        if (near_end && mt && avail < 48 && is_len) {
            Sym yd;
            yd.L = Ld;
            yd.idx = 0;
            yd.inval = invd;
            need_d = canon_need<15>(td, yd, __builtin_bitreverse32((uint32_t)(w2 >> used)) >> 17);
        }
        // event, in the reference's order: 0 token, 1 eob, 2 starved, 3 error
        const bool s_m1 = (int32_t)used > avail || (int32_t)(used + need_d) > avail;
        const bool s_m2 = (int32_t)(used + Ld + xd) > avail;
        const uint32_t ev = (int32_t)need_l > avail ? 2u
                            : inval               ? 3u
                            : kind == K_EOB       ? 1u
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
        const bool c_raw = raw && pos >= cap;
        const bool c_dist = is_match && dist > pos + hist;
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
        elit = emit && !is_match ? (e >> 8) : elit;
        pos += emit ? olen : 0u;
    };
    if (valid) begin(m);

    for (;;) {
        if (!exhausted) {
            const uint64_t idle = __ballot(fin && !send_new && !exhausted);
            // take new messages when a quarter of the wave waits or nothing else runs
            if (idle && (__builtin_popcountll(idle) * 4 >= LANES || __ballot(!fin) == 0)) {
                const unsigned leader = (unsigned)__builtin_ctzll(idle);
                uint32_t base = 0;
                if ((threadIdx.x & 63u) == leader) base = atomicAdd(qctr, (uint32_t)__builtin_popcountll(idle));
                base = __shfl(base, (int)leader);
                if ((idle >> (threadIdx.x & 63u)) & 1) {
                    const uint32_t k =
                        first_slots + base + (uint32_t)__builtin_popcountll(idle & ((1ull << (threadIdx.x & 63u)) - 1ull));
                    if (k < n_msgs) {
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
        // ---- the input pipeline (the only global memory the decoder touches)
        if (nx_used) pipe();
        const uint32_t taken = lds_load(T + O_TAIL);
        compiler_fence();
        const bool room = head - taken < RING;
        const bool ring_empty = head == taken;
        uint32_t enl = 0, elit = 0, emlen = 0, edist = 0;
        const uint32_t st0 = st;
        const uint32_t head0 = head;
        if (st == S_DATA && room) data_step(enl, elit, emlen, edist);

        // ======================================= block headers, stored
        if (__ballot(st0 != S_DATA && st0 != S_DONE)) {
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
                    st = type == 0 ? (uint32_t)S_SHDR : type == 1 ? (uint32_t)S_FIX : type == 2 ? (uint32_t)S_DYN : (uint32_t)S_DONE;
                    if (type == 3) result = ST_INVALID_BLOCK_TYPE;
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
            // COPY (inflate_stream.ipp:206-220): up to 4 bytes per iteration
            if (srem && room) {
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
        // ================================================== fixed tables
        // (inflate_stream.ipp:865-930): built by the same table fill from the
        // fixed code lengths; the scratch shares LDS with the ring, so the ring
        // drains first
        if (st == S_FIX && ring_empty) {
            uint4* nib4 = (uint4*)(T + O_NIB);
#pragma unroll
            for (int k = 0; k < 10; ++k) {
                uint32_t wv[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int wi = 4 * k + i;   // nibble word: symbols 8 wi .. 8 wi + 7
                    wv[i] = wi < 18 ? 0x88888888u : wi < 32 ? 0x99999999u : wi < 35 ? 0x77777777u : wi < 36 ? 0x88888888u : 0x55555555u;
                }
                nib4[k] = make_uint4(wv[0], wv[1], wv[2], wv[3]);
            }
            uint4* h4 = (uint4*)H;
            h4[0] = make_uint4(0, 0, 0, 0);
            h4[1] = make_uint4(0, 32u << 20, 0, 24u);
            h4[2] = make_uint4(152u | (144u << 10), 112u | (112u << 10), 0, 0);
            h4[3] = make_uint4(0, 0, 0, 0);
            nlen = 288;
            ndist = 32;
            want = 320;
            eob_seen = true;
            st = S_BUILD;
        }
        // ================================================== D. dynamic header
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
                    uint64_t clp = 0;
                    refill();
#pragma unroll
                    for (int i = 0; i < 10; ++i)
                        clp |= (uint64_t)((uint32_t)i < ncode ? ((uint32_t)(bb >> (3 * i)) & 7u) : 0u)
                               << (3 * kClenOrder4[i]);
                    drop(3 * (ncode < 10 ? ncode : 10u));
                    refill();
#pragma unroll
                    for (int i = 10; i < 19; ++i)
                        clp |= (uint64_t)((uint32_t)i < ncode ? ((uint32_t)(bb >> (3 * (i - 10))) & 7u) : 0u)
                               << (3 * kClenOrder4[i]);
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
                            offs += 1ull << (5 * l);
                            if (l) T[O_CLS + at] = (uint8_t)i;
                        }
                        uint4* nib4 = (uint4*)(T + O_NIB);
#pragma unroll
                        for (int k = 0; k < 10; ++k) nib4[k] = make_uint4(0, 0, 0, 0);
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
#pragma unroll
        for (int kc = 0; kc < KCL; ++kc) {
            if (st != S_PASS1 || st0 != S_PASS1) break;
            // CODELENS (inflate_stream.ipp:264-327), up to KCL symbols per iteration
            refill();
            const int32_t avail = tb + (int32_t)nb;
            uint32_t L = 1, csym = 0;
            if (!cl_empty) {
                const uint32_t c7 = __builtin_bitreverse32((uint32_t)bb) >> 25;
                const Sym yc = lp3::canon_decode<7>(tc.Q, c7);
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
                        const uint32_t s_d = a > nlen ? a : nlen;
                        const uint32_t nd = b > s_d ? b - s_d : 0u;
                        __hip_atomic_fetch_add(H + val, nl | (nd << 20), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        if (a <= 256 && 256 < b) eob_seen = true;
                    }
                    prev = val;
                    have += rep;
                    if (have == want) st = S_BUILD;
                }
            }
        }
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
                uint32_t c[16], cd[16];
                c[0] = cd[0] = 0;
                lmax = dmax = 0;
#pragma unroll
                for (int l = 1; l < 16; ++l) {
                    c[l] = h[l] & 0x3ffu;
                    cd[l] = (h[l] >> 20) & 0x3ffu;
                    lmax = c[l] ? (uint32_t)l : lmax;
                    dmax = cd[l] ? (uint32_t)l : dmax;
                }
                int e = make_canon<15>(c, 9, 1, tl);
                if (!e) e = make_canon<15>(cd, 6, 2, td);
                if (e) {
                    result = e;
                    st = S_DONE;
                } else {
                    // Table geometry.  lim(l) = left-justified (15-bit) end of the
                    // codes of length <= l (Q word bits 15+); codes of length l
                    // start at lim(l - 1).  Root slot of a code of length
                    // l <= R: its first R bits; sub-table slot of a longer code:
                    // its first lmax bits minus the first long code's.
                    const uint32_t lim_lr = tl.Q[RL - 1] >> 15, lim_dr = td.Q[RD - 1] >> 15;
                    const uint32_t lsub_n = lmax > RL ? (32768u - lim_lr) >> (15 - lmax) : 0u;
                    const uint32_t dsub_n = dmax > RD ? ((td.Q[14] >> 15) - lim_dr) >> (15 - dmax) : 0u;
                    lsh = 32 - lmax;
                    lbase = lmax > RL ? lim_lr >> (15 - lmax) : 0u;
                    dsh = 32 - dmax;
                    dbase = dmax > RD ? lim_dr >> (15 - dmax) : 0u;
                    if (lsub_n > subl_cap || dsub_n > subd_cap) {
                        result = ST_FB4;   // re-decoded by the lane3 kernel
                        st = S_DONE;
                    } else {
                        // fill cursors: first slot of each code length (lit | dist << 16)
#pragma unroll
                        for (int l = 1; l < 16; ++l) {
                            const uint32_t ll0 = l > 1 ? tl.Q[l - 2] >> 15 : 0u;
                            const uint32_t dl0 = l > 1 ? td.Q[l - 2] >> 15 : 0u;
                            const uint32_t sl = (uint32_t)l <= RL ? ll0 >> (15 - RL)
                                                                   : ((ll0 >> (15 - lmax)) - lbase) & 0xffffu;
                            const uint32_t sd = (uint32_t)l <= RD ? dl0 >> (15 - RD)
                                                                   : ((dl0 >> (15 - dmax)) - dbase) & 0xffffu;
                            H[l] = sl | (sd << 16);
                        }
                        // roots start as "longer code" (when the block has them) or invalid
                        const uint32_t lfill = lmax > RL ? (RL | (K_SUB << 4)) : (K_BAD << 4);
                        const uint4 lr4 = make_uint4(lfill * 0x10001u, lfill * 0x10001u, lfill * 0x10001u, lfill * 0x10001u);
#pragma unroll
                        for (uint32_t k = 0; k < (2u << RL) / 16; ++k) *(uint4*)(T + O_LR + 16 * k) = lr4;
                        const uint32_t dfill = dmax > RD ? (RD | (DK_SUB << 4)) : (DK_BAD << 4);
                        const uint4 dr4 = make_uint4(dfill, dfill, dfill, dfill);
#pragma unroll
                        for (uint32_t k = 0; k < (4u << RD) / 16; ++k) *(uint4*)(T + O_DR + 16 * k) = dr4;
                        have = 0;
                        st = S_PASS2;
                    }
                }
            }
        }
        if (st == S_PASS2) {
            // place each code's entries: 2^(depth - l) copies at its slot
#pragma unroll
            for (uint32_t h8 = 0; h8 < KNIB; h8 += 8) {
                const uint32_t i0 = have + h8;
                const uint32_t w = i0 < want ? ((const uint32_t*)(T + O_NIB))[i0 >> 3] : 0u;
                if (__ballot(w != 0)) {
                    uint32_t olds[8];
#pragma unroll
                    for (uint32_t k = 0; k < 8; ++k) {
                        const uint32_t i = i0 + k;
                        const uint32_t l = (w >> (4 * k)) & 15u;
                        const bool lit = i < nlen;
                        const uint32_t dep = lit ? (l <= RL ? RL : lmax) : (l <= RD ? RD : dmax);
                        const uint32_t inc = (l && i < want) ? (1u << (dep - l)) << (lit ? 0 : 16) : 0u;
                        olds[k] = __hip_atomic_fetch_add(H + l, inc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
#pragma unroll
                    for (uint32_t k = 0; k < 8; ++k) {
                        const uint32_t i = i0 + k;
                        const uint32_t l = (w >> (4 * k)) & 15u;
                        if (l && i < want) {
                            if (i < nlen) {
                                const uint32_t sl = olds[k] & 0xffffu;
                                const bool root = l <= RL;
                                const uint32_t at = (root ? O_LR : O_LS) + 2 * sl;
                                const uint32_t ent = lit_entry(i, l);
                                fill_entries(T + at, 2u << ((root ? RL : lmax) - l), ent * 0x10001u);
                            } else {
                                const uint32_t sd = olds[k] >> 16;
                                const bool root = l <= RD;
                                const uint32_t at = (root ? O_DR : O_DS) + 4 * sd;
                                fill_entries(T + at, 4u << ((root ? RD : dmax) - l), dist_entry(i - nlen, l));
                            }
                        }
                    }
                }
            }
            have += KNIB;
            if (have >= want) st = S_DATA;
        }
        }   // block headers, stored
        // ---- publish the token (entry first, then head)
        {
            const bool ctl = send_new || send_exit;
            const bool data = !ctl && (enl || emlen);
            const bool endt = !ctl && !data && st == S_DONE && !fin;
            const bool adv = room && (ctl || data || endt);
            const uint2 ent = ctl    ? make_uint2(msg, send_new ? TOK_NEW : TOK_EXIT)
                              : data ? make_uint2(elit, enl | (emlen << 3) | (edist << 12))
                                     : make_uint2(pos, TOK_END | ((uint32_t)result & 0xffu));
            if (adv) *(uint2*)(T + ring_at(head)) = ent;
            compiler_fence();
            head += adv ? 1u : 0u;
            lds_store(T + O_HEAD, head);
            fin = fin || (adv && endt);
            if (adv && ctl) {
                if (send_new) begin(msg);
                send_new = false;
                send_exit = false;
            }
        }
        // ---- a second token for the lanes still in the same Huffman block with
        // room in the ring and their next input block unused (lane3's DATA2)
        if (__ballot(st0 == S_DATA && st == S_DATA && !nx_used && head - taken < RING)) {
            uint32_t enl2 = 0, elit2 = 0, emlen2 = 0, edist2 = 0;
            if (st0 == S_DATA && st == S_DATA && !nx_used && head - taken < RING)
                data_step(enl2, elit2, emlen2, edist2);
            const bool adv2 = enl2 != 0 || emlen2 != 0;
            if (adv2) *(uint2*)(T + ring_at(head)) = make_uint2(elit2, enl2 | (emlen2 << 3) | (edist2 << 12));
            compiler_fence();
            head += adv2 ? 1u : 0u;
            lds_store(T + O_HEAD, head);
        }
        // blocked on a full ring in every lane: leave the SIMD to the expander
        if (!__ballot(head != head0 || st != st0 || (st != S_DATA && st != S_SCOPY && st != S_DONE)))
            __builtin_amdgcn_s_sleep(1);
    }
}

// A workgroup is one decoder wave and one expander wave over LANES messages
// (lanes LANES..63 of both waves leave at once).
__global__ void __launch_bounds__(128, 2)
inflate_lane4_kernel(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                     const uint32_t* __restrict__ in_len, uint32_t n_msgs, uint8_t* __restrict__ out,
                     const uint64_t* __restrict__ out_off, const uint32_t* __restrict__ out_cap,
                     uint32_t* __restrict__ out_len, int32_t* __restrict__ status, uint32_t raw,
                     const uint32_t* __restrict__ mask_key, const uint32_t* __restrict__ hist_len, uint32_t hist_max,
                     uint32_t max_in, const uint32_t* __restrict__ order, uint32_t* __restrict__ qctr,
                     const uint32_t* __restrict__ skip, uint32_t* __restrict__ fb, uint32_t subl_cap, uint32_t subd_cap)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const unsigned lane = threadIdx.x & 63u;
    const bool is_decoder = threadIdx.x < 64;
    if (lane >= LANES) return;
    uint8_t* T = smem + lane * STRIDE;
    // skip: the first *skip entries of `order` belong to another kernel
    const uint32_t s0 = skip ? *skip : 0u;
    const uint32_t j = s0 + blockIdx.x * LANES + lane;
    bool valid = j < n_msgs;
    const uint32_t m = valid ? (order ? order[j] : j) : 0u;
    // max_in != 0: only payloads of at most max_in bytes (the rest go to the wave kernel)
    if (valid && max_in && in_len[m] > max_in) valid = false;
    if (is_decoder) *(uint2*)(T + O_HEAD) = make_uint2(0, 0);
    __syncthreads();
    if (is_decoder) {
        __builtin_amdgcn_s_setprio(3);   // the decoder sets the pace
        decoder(T, valid, m, in, in_off, in_len, out_cap, raw, mask_key, hist_len, hist_max, n_msgs, order, qctr, s0,
                subl_cap < SUBL ? subl_cap : SUBL, subd_cap < SUBD ? subd_cap : SUBD);
    } else {
        expander(T, valid, m, out, out_off, out_cap, out_len, status, hist_len, hist_max, qctr != nullptr, fb);
    }
}

}  // namespace lp4
}  // namespace bpmd

extern "C" int bpmd_internal_inflate_lane3(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint32_t n,
                                           uint8_t* out, const uint64_t* out_off, const uint32_t* out_cap,
                                           uint32_t* out_len, int32_t* status, uint32_t raw, const uint32_t* mask_key,
                                           const uint32_t* hist_len, uint32_t hist_max, uint32_t max_in,
                                           const uint32_t* order, uint32_t* qctr, uint32_t grid_wgs,
                                           const uint32_t* skip, hipStream_t stream, const uint32_t* n_dev);
extern "C" void* bpmd_internal_scratch(hipStream_t s, size_t bytes, int which);

// sub-table budgets (literal/length | distance << 16); diagnostics and tests
// lower them (bpmd_diag_set_lane4_sub, BPMD_LANE4_SUB="l,d") so that the
// hand-back path runs: 0,0 hands back every block with a code longer than the
// root bits
static std::atomic<int64_t> g_lane4_caps{-1};
static uint32_t lane4_sub_caps()
{
    using namespace bpmd::lp4;
    int64_t v = g_lane4_caps.load();
    if (v < 0) {
        const char* e = getenv("BPMD_LANE4_SUB");
        uint32_t l = SUBL, d = SUBD;
        if (e) {
            l = (uint32_t)strtoul(e, nullptr, 10);
            const char* c = strchr(e, ',');
            d = c ? (uint32_t)strtoul(c + 1, nullptr, 10) : SUBD;
        }
        v = (int64_t)((l & 0xffffu) | (d << 16));
        g_lane4_caps.store(v);
    }
    return (uint32_t)v;
}
extern "C" int bpmd_diag_set_lane4_sub(int l, int d)
{
    using namespace bpmd::lp4;
    if (l < 0 || d < 0) {
        g_lane4_caps.store((int64_t)(SUBL | (SUBD << 16)));
        return 0;
    }
    g_lane4_caps.store((int64_t)(((uint32_t)l & 0xffffu) | ((uint32_t)d << 16)));
    return 0;
}

// messages one CU holds in flight (the work-queue threshold of inflate_impl)
extern "C" uint32_t bpmd_internal_lane4_per_cu(void)
{
    using namespace bpmd::lp4;
    return (160u * 1024u / (LANES * STRIDE)) * LANES;
}

// Lane4 decode of [s0, n) of `order` (or of the batch), then the lane3
// kernel over the messages lane4 handed back (device-side list; usually
// empty).  qctr / grid_wgs: as bpmd_internal_inflate_lane3.
extern "C" int bpmd_internal_inflate_lane4(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint32_t n,
                                           uint8_t* out, const uint64_t* out_off, const uint32_t* out_cap,
                                           uint32_t* out_len, int32_t* status, uint32_t raw, const uint32_t* mask_key,
                                           const uint32_t* hist_len, uint32_t hist_max, uint32_t max_in,
                                           const uint32_t* order, uint32_t* qctr, uint32_t grid_wgs,
                                           const uint32_t* skip, hipStream_t stream)
{
    using namespace bpmd::lp4;
    if (n == 0) return 0;
    const uint32_t caps = lane4_sub_caps();
    // fallback list: [count, message...]
    uint32_t* fb = (uint32_t*)bpmd_internal_scratch(stream, ((size_t)n + 64) * 4, 12);
    if (!fb || hipMemsetAsync(fb, 0, 4, stream) != hipSuccess) return (int)hipErrorOutOfMemory;
    unsigned grid = (n + LANES - 1) / LANES;
    if (qctr && grid_wgs && grid > grid_wgs) grid = grid_wgs;
    hipLaunchKernelGGL(inflate_lane4_kernel, dim3(grid), dim3(128), LANES * STRIDE, stream, in, in_off, in_len, n, out,
                       out_off, out_cap, out_len, status, raw, mask_key, hist_len, hist_max, max_in, order, qctr, skip, fb,
                       caps & 0xffffu, caps >> 16);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    // the handed-back messages: one lane3 workgroup per CU drains them from a queue
    uint32_t* q2 = (uint32_t*)bpmd_internal_scratch(stream, 256, 13);
    if (!q2 || hipMemsetAsync(q2, 0, 4, stream) != hipSuccess) return (int)hipErrorOutOfMemory;
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    return bpmd_internal_inflate_lane3(in, in_off, in_len, n, out, out_off, out_cap, out_len, status, raw, mask_key,
                                       hist_len, hist_max, 0u, fb + 1, q2, (uint32_t)cus, nullptr, stream, fb);
}
