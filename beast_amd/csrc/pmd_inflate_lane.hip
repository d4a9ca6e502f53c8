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

enum : uint32_t { S_TYPE, S_DATA, S_SHDR, S_SCOPY, S_DYN, S_PASS1, S_BUILD, S_PASS2, S_DONE };

struct Tree {
    uint32_t P[14];   // group of length i + 2: lim << 16 | (i + 2) << 12 | first index
    uint32_t limend;  // left-justified end of the used code space
    uint32_t root;    // the reference's (clamped) root table bits
};

template <int N>
__device__ __forceinline__ uint32_t selchain(const uint32_t (&P)[N], uint32_t key)
{
    uint32_t s = 1u << 12;   // length 1, limit 0, first index 0
#pragma unroll
    for (int i = 0; i < N; ++i) s = P[i] <= key ? P[i] : s;
    return s;
}

__device__ __forceinline__ uint32_t rev15(uint64_t bb) { return __builtin_bitreverse32((uint32_t)bb) >> 17; }
__device__ __forceinline__ uint32_t lowmask(uint32_t n) { return n >= 32 ? ~0u : ((1u << n) - 1u); }

// counts c[1..15] -> canonical group words; returns 0, 14 or 15 following
// inflate_table's acceptance rules (inflate_stream.ipp:574-617).
// type: 0 codes, 1 lens, 2 dists.  cum[l] = first canonical index of length l.
template <int NB>
__device__ __forceinline__ int make_tree(const uint32_t (&c)[16], uint32_t R, int type, uint32_t (&P)[NB - 1],
                                         uint32_t& limend, uint32_t& root, uint32_t (&cum)[17])
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
        if (l < NB) P[l - 1] = (lim << 16) | ((uint32_t)(l + 1) << 12) | cu;
    }
#pragma unroll
    for (int l = NB + 1; l <= 16; ++l) cum[l] = cu;
    limend = lim;
    if (hi == 0) {   // empty code: a 1-bit root of invalid slots
        root = 1;
        return 0;
    }
    uint32_t r = R < hi ? R : hi;
    root = r < lo ? lo : r;
    if (over) return ST_OVER_SUBSCRIBED_LENGTH;
    if (left > 0 && (type == 0 || hi != 1)) return ST_INCOMPLETE_LENGTH_SET;
    return 0;
}

// 16 stream bytes at A + 16*bi: payload bytes [s, s+n) of the lane's
// message, then the 00 00 FF FF tail (pmd mode), then zeros.  Only blocks
// wholly inside the payload are read with one 16-byte load; the edges never
// touch memory outside the payload.
__device__ __forceinline__ uint4 load_block(const uint8_t* A, uint32_t bi, uint32_t s, uint32_t n, uint32_t tail)
{
    const uint32_t b0 = bi * 16;
    if (b0 >= s && b0 + 16 <= s + n) return *(const uint4*)(A + b0);
    uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const int32_t r = (int32_t)(b0 + j) - (int32_t)s;
        uint32_t b = 0;
        if (r >= 0 && (uint32_t)r < n) b = A[b0 + j];
        else if (r >= 0 && (uint32_t)r - n < tail) b = ((uint32_t)r - n) >= 2 ? 0xffu : 0u;
        w[j >> 2] |= b << ((j & 3) * 8);
    }
    return make_uint4(w[0], w[1], w[2], w[3]);
}

typedef uint4 uint4_u __attribute__((aligned(1)));
typedef uint2 uint2_u __attribute__((aligned(1)));
typedef uint64_t u64_u __attribute__((aligned(1)));

static __constant__ const uint8_t kClenOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// fixed-code canonical symbol image (low 8 bits): lengths 7: 256-279,
// 8: 0-143 then 280-287, 9: 144-255; distances 0-31
__device__ __attribute__((aligned(16))) uint32_t g_fixed_img[80];

__global__ void __launch_bounds__(64)
inflate_lane_kernel(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                    const uint32_t* __restrict__ in_len, uint32_t n_msgs, uint8_t* __restrict__ out,
                    const uint64_t* __restrict__ out_off, const uint32_t* __restrict__ out_cap,
                    uint32_t* __restrict__ out_len, int32_t* __restrict__ status, uint32_t raw)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const unsigned lane = threadIdx.x;
    const uint32_t msg = blockIdx.x * 64 + lane;
    uint8_t* T = smem + lane * STRIDE;
    uint32_t* H = (uint32_t*)(T + O_HIST);
    uint16_t* LE = (uint16_t*)(T + O_LE);

    const bool valid = msg < n_msgs;
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

    // ---- bit reader: 64-bit buffer refilled 32 bits at a time from a
    // 16-byte block (q) with the next block (r) already in flight.
    const uint8_t* A = (const uint8_t*)((uintptr_t)p & ~(uintptr_t)3);
    const uint32_t s = (uint32_t)((uintptr_t)p & 3);
    uint4 q = make_uint4(0, 0, 0, 0), r = q;
    if (valid) {
        q = load_block(A, 0, s, n, tail);
        r = load_block(A, 1, s, n, tail);
    }
    uint32_t blk = 2, qn = 4;
    uint64_t bb = 0;
    uint32_t nb = 0;
    int32_t tb = (int32_t)(8 * (s + n + tail));   // stream bits not yet moved into bb
    auto refill = [&]() {
        if (nb <= 32) {
            bb |= (uint64_t)q.x << nb;
            nb += 32;
            tb -= 32;
            q.x = q.y;
            q.y = q.z;
            q.z = q.w;
            if (--qn == 0) {
                q = r;
                qn = 4;
                r = load_block(A, blk++, s, n, tail);
            }
        }
    };
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

    Tree tl, td;
#pragma unroll
    for (int i = 0; i < 14; ++i) { tl.P[i] = 0; td.P[i] = 0; }
    tl.limend = td.limend = 0;
    tl.root = 9;
    td.root = 5;

    // header state
    uint32_t nlen = 0, ndist = 0, want = 0, have = 0, prev = 0;
    bool eob_seen = false, cl_empty = false;
    uint32_t PC[6] = {0, 0, 0, 0, 0, 0};
    uint32_t croot = 1;
    // stored block
    uint32_t srem = 0;
    bool sfull = false, sstarve = false;
    // match copy: bytes left, distance, next output position, pattern
    uint32_t crem = 0, cdist = 0, cq = 0;
    uint64_t cpat = 0;
    bool cpat_ok = false;
    // deferred chunk store
    bool pend = false;
    uint32_t pdst = 0, psz = 0;
    uint4 pw = make_uint4(0, 0, 0, 0);

    for (;;) {
        const bool alive = st != S_DONE || crem != 0 || pend;
        if (!__builtin_amdgcn_ballot_w64(alive)) break;

        // ================================================ A. decode a token
        bool emit_lit = false;
        uint32_t lit_byte = 0, lit_pos = 0;
        if (st == S_DATA && crem == 0) {
            refill();
            const int32_t avail = tb + (int32_t)nb;
            const uint32_t c15 = rev15(bb);
            const uint32_t sel = selchain(tl.P, (c15 << 16) | 0xffffu);
            const uint32_t L = (sel >> 12) & 15u;
            bool inval = c15 >= tl.limend;
            uint32_t idx = (sel & 0xfffu) + ((c15 - (sel >> 16)) >> (15u - L));
            idx = inval ? 0u : idx;
            const uint32_t le = LE[L];
            uint32_t sym = T[O_LIT + idx] + (idx >= le ? 256u : 0u);
            inval |= sym >= 286;
            uint32_t need_l = 0;
            if (avail < 48) {
                need_l = tl.root;
                if (!inval && L > tl.root) {
                    const uint32_t re = c15 | lowmask(15u - tl.root);
                    need_l = (selchain(tl.P, (re << 16) | 0xffffu) >> 12) & 15u;
                }
            }
            uint32_t len = 0, dist = 0;
            bool is_match = false;
            uint32_t ev = 0;   // 0 token, 1 eob, 2 starved, 3 error
            int32_t err = 0;
            if ((int32_t)need_l > avail) {
                ev = 2;
            } else if (inval) {
                ev = 3;
                err = ST_INVALID_LITERAL_LENGTH;
            } else if (sym < 256) {
                drop(L);
                lit_byte = sym;
            } else if (sym == 256) {
                drop(L);
                ev = 1;
            } else {
                const uint32_t li = sym - 257;
                const uint32_t xl = (li < 8 || li == 28) ? 0u : ((li - 4) >> 2);
                len = li < 8 ? li + 3 : (li == 28 ? 258u : (((4u + (li & 3)) << xl) + 3));
                len += (uint32_t)(bb >> L) & lowmask(xl);
                const uint32_t used = L + xl;
                if ((int32_t)used > avail) {
                    ev = 2;
                } else {
                    drop(used);
                    refill();
                    const uint32_t d15 = rev15(bb);
                    const uint32_t seld = selchain(td.P, (d15 << 16) | 0xffffu);
                    const uint32_t Ld = (seld >> 12) & 15u;
                    bool invd = d15 >= td.limend;
                    uint32_t idd = (seld & 0xfffu) + ((d15 - (seld >> 16)) >> (15u - Ld));
                    idd = invd ? 0u : idd;
                    const uint32_t dsym = T[O_DST + idd];
                    invd |= dsym >= 30;
                    uint32_t need_d = 0;
                    if (avail < 48) {
                        need_d = td.root;
                        if (!invd && Ld > td.root) {
                            const uint32_t re = d15 | lowmask(15u - td.root);
                            need_d = (selchain(td.P, (re << 16) | 0xffffu) >> 12) & 15u;
                        }
                    }
                    if ((int32_t)(used + need_d) > avail) {
                        ev = 2;
                    } else if (invd) {
                        ev = 3;
                        err = ST_INVALID_DISTANCE_CODE;
                    } else {
                        const uint32_t xd = dsym < 4 ? 0u : (dsym >> 1) - 1;
                        dist = dsym < 4 ? dsym + 1 : (((2u + (dsym & 1)) << xd) + 1);
                        dist += (uint32_t)(bb >> Ld) & lowmask(xd);
                        if ((int32_t)(used + Ld + xd) > avail) ev = 2;
                        else {
                            drop(Ld + xd);
                            is_match = true;
                        }
                    }
                }
            }
            if (ev == 0) {
                // output checks in the reference's order (inflate_stream.ipp:475-514)
                if (raw && pos >= cap) {
                    result = full_status;
                    st = S_DONE;
                } else if (is_match && dist > pos) {
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
                        cpat_ok = false;
                    } else {
                        emit_lit = true;
                        lit_pos = pos;
                    }
                    pos += olen;
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

        // ========================================= B. deferred chunk store
        if (pend) {
            if (psz == 16) *(uint4_u*)(o + pdst) = pw;
            else *(uint2_u*)(o + pdst) = make_uint2(pw.x, pw.y);
            pend = false;
        }
        if (emit_lit) o[lit_pos] = (uint8_t)lit_byte;

        // ======================================= C. block headers, stored
        if (st == S_TYPE) {
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
                        // fixed tables (inflate_stream.ipp:865-930)
                        uint4* dst4 = (uint4*)T;
#pragma unroll
                        for (int k = 0; k < 20; ++k) dst4[k] = ((const uint4*)g_fixed_img)[k];
                        LE[7] = 0;
                        LE[8] = 168;
                        LE[9] = 288;
                        uint32_t c[16], cum[17];
#pragma unroll
                        for (int l = 0; l < 16; ++l) c[l] = 0;
                        c[7] = 24;
                        c[8] = 152;
                        c[9] = 112;
                        make_tree<15>(c, 9, 1, tl.P, tl.limend, tl.root, cum);
#pragma unroll
                        for (int l = 0; l < 16; ++l) c[l] = 0;
                        c[5] = 32;
                        make_tree<15>(c, 5, 2, td.P, td.limend, td.root, cum);
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
            if (srem) {
                refill();
                const uint32_t k = srem < 4 ? srem : 4u;
                const uint32_t w = (uint32_t)bb;
#pragma unroll
                for (uint32_t j = 0; j < 4; ++j)
                    if (j < k) o[pos + j] = (uint8_t)(w >> (8 * j));
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
                    uint32_t limend_c;
                    const int e = make_tree<7>(c, 7, 0, PC, limend_c, croot, cum);
                    (void)limend_c;
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
        if (st == S_PASS1) {
            // CODELENS (inflate_stream.ipp:264-327), one symbol per iteration
            refill();
            const int32_t avail = tb + (int32_t)nb;
            uint32_t L = 1, csym = 0;
            if (!cl_empty) {
                const uint32_t c7 = __builtin_bitreverse32((uint32_t)bb) >> 25;
                const uint32_t sel = selchain(PC, (c7 << 16) | 0xffffu);
                L = (sel >> 12) & 15u;
                const uint32_t idx = (sel & 0xfffu) + ((c7 - (sel >> 16)) >> (7u - L));
                csym = T[O_CLS + (idx < 19 ? idx : 0u)];
            }
            if (avail < (int32_t)croot) {
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
                int e = make_tree<15>(c, 9, 1, tl.P, tl.limend, tl.root, cuml);
                if (!e) {
#pragma unroll
                    for (int l = 1; l < 16; ++l) c[l] = (h[l] >> 20) & 0x3ffu;
                    e = make_tree<15>(c, 6, 2, td.P, td.limend, td.root, cumd);
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
            const uint32_t w = ((const uint32_t*)(T + O_NIB))[have >> 3];
#pragma unroll
            for (uint32_t k = 0; k < 8; ++k) {
                const uint32_t i = have + k;
                const uint32_t l = (w >> (4 * k)) & 15u;
                const bool isl = i < nlen;
                const uint32_t inc = (l && i < want) ? (isl ? 1u : 0x10000u) : 0u;
                if (inc) {
                    const uint32_t old = __hip_atomic_fetch_add(H + l, inc, __ATOMIC_RELAXED,
                                                                __HIP_MEMORY_SCOPE_WORKGROUP);
                    if (isl) T[O_LIT + (old & 0xffffu)] = (uint8_t)i;
                    else T[O_DST + (old >> 16)] = (uint8_t)(i - nlen);
                }
            }
            have += 8;
            if (have >= want) st = S_DATA;
        }

        // ======================================================= E. copy step
        if (crem) {
            const uint32_t C = cdist >= 16 ? 16u : 8u;
            if (cq + C > cap || (cdist < 8 && cq < 8)) {
                // slot edge: byte by byte, in order
                for (uint32_t j = 0; j < crem; ++j) o[cq + j] = o[cq + j - cdist];
                cq += crem;
                crem = 0;
            } else {
                uint32_t adv;
                if (cdist >= 16) {
                    pw = *(const uint4_u*)(o + cq - cdist);
                    adv = 16;
                } else if (cdist >= 8) {
                    const uint2 v = *(const uint2_u*)(o + cq - cdist);
                    pw = make_uint4(v.x, v.y, 0, 0);
                    adv = 8;
                } else {
                    if (!cpat_ok) {
                        // the cdist bytes before cq, repeated (period cdist)
                        uint64_t v = *(const u64_u*)(o + cq - 8);
                        v >>= 8 * (8 - cdist);
                        v &= (1ull << (8 * cdist)) - 1;
                        // (64-bit shifts of 64 or more wrap on the hardware: guard them)
                        if (cdist < 8) v |= v << (8 * cdist);
                        if (cdist < 4) v |= v << (16 * cdist);
                        if (cdist < 2) v |= v << (32 * cdist);
                        cpat = v;
                        cpat_ok = true;
                    }
                    pw = make_uint4((uint32_t)cpat, (uint32_t)(cpat >> 32), 0, 0);
                    adv = 8 - 8 % cdist;
                }
                pend = true;
                pdst = cq;
                psz = C;
                if (adv > crem) adv = crem;
                cq += adv;
                crem -= adv;
            }
        }
    }
    if (valid) {
        out_len[msg] = pos;
        status[msg] = result;
    }
}

}  // namespace lpm
}  // namespace bpmd

extern "C" int bpmd_internal_inflate_lane(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                                          uint32_t n, uint8_t* out, const uint64_t* out_off,
                                          const uint32_t* out_cap, uint32_t* out_len, int32_t* status, uint32_t raw,
                                          hipStream_t stream)
{
    using namespace bpmd::lpm;
    if (n == 0) return 0;
    const unsigned grid = (n + 63) / 64;
    hipLaunchKernelGGL(inflate_lane_kernel, dim3(grid), dim3(64), 64 * STRIDE, stream, in, in_off, in_len, n, out,
                       out_off, out_cap, out_len, status, raw);
    return (int)hipGetLastError();
}

extern "C" int bpmd_internal_init_fixed_lane(void)
{
    using namespace bpmd::lpm;
    uint8_t img[320];
    unsigned k = 0;
    for (unsigned v = 256; v < 280; ++v) img[k++] = (uint8_t)(v & 0xff);
    for (unsigned v = 0; v < 144; ++v) img[k++] = (uint8_t)v;
    for (unsigned v = 280; v < 288; ++v) img[k++] = (uint8_t)(v & 0xff);
    for (unsigned v = 144; v < 256; ++v) img[k++] = (uint8_t)v;
    for (unsigned v = 0; v < 32; ++v) img[k++] = (uint8_t)v;
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_fixed_img), img, sizeof img);
}
