// pmd_inflate.hip -- batched raw-DEFLATE decode for permessage-deflate
// payloads on gfx950 (CDNA4).  One wavefront owns one message at a time.
//
// Semantics follow Beast's decoder (include/boost/beast/zlib/detail/
// inflate_stream.ipp:74-535) driven the way the websocket read path drives
// it (websocket/detail/impl_base.hpp:168-190, websocket/impl/read.hpp:
// 1284-1356): the payload plus an appended 00 00 FF FF tail is decoded from a
// fresh state; decoding stops when the next step would need more bits than
// the input holds (Beast's bitstream fill rule), on BFINAL (end_of_stream),
// on the first data error (its zlib::error value), or when the output would
// exceed the message's capacity (need_buffers, output truncated to the
// capacity).
//
// Memory: per wave, LDS holds the decode tables (16-bit slots, huff_table.h),
// the code lengths and an output stage.  Messages whose output fits the stage
// never touch global memory except for one coalesced store at the end;
// larger ones flush the stage in STAGE-byte pieces and read older history
// back from global memory.
#include "pmd_common.h"
#include "huff_table.h"

namespace bpmd {

constexpr unsigned STAGE = 8192;          // output stage bytes per wave
constexpr unsigned WAVES_PER_BLOCK = 4;

struct alignas(16) WaveLds {
    uint8_t stage[STAGE];                   // 16-byte aligned (first member)
    uint16_t tab[kEnough];                  // lens table then dists table
    uint16_t sorted[320];
    uint8_t lens[320];
};

// fixed-Huffman tables built once on the host with the same builder
__device__ uint16_t g_fixed_lens[512];
__device__ uint16_t g_fixed_dists[32];

struct InMsg {
    const uint8_t* p;
    uint32_t n;        // payload bytes
    uint32_t total;    // payload + tail bytes (4 unless raw)
};

__device__ __forceinline__ uint32_t in_byte(const InMsg& m, uint32_t i)
{
    if (i < m.n) return m.p[i];
    if (i < m.total) return (i - m.n) >= 2 ? 0xffu : 0u;   // 00 00 FF FF
    return 0;
}

// 4 bytes of the virtual stream (payload || tail || zeros) at byte offset i
__device__ __forceinline__ uint32_t in_word(const InMsg& m, uint32_t i)
{
    if (i + 8 <= m.n) {
        uintptr_t a = (uintptr_t)(m.p + i);
        const uint32_t* w = (const uint32_t*)(a & ~(uintptr_t)3);
        unsigned sh = (unsigned)(a & 3) * 8;
        uint64_t v = ((uint64_t)w[1] << 32) | w[0];
        return (uint32_t)(v >> sh);
    }
    return in_byte(m, i) | (in_byte(m, i + 1) << 8) | (in_byte(m, i + 2) << 16) | (in_byte(m, i + 3) << 24);
}

// LSB-first bit reader over the virtual stream (wave-uniform state)
struct Bits {
    uint64_t buf;
    uint32_t cnt;      // valid bits in buf
    uint32_t next;     // next byte offset to load
    uint32_t total_bits;
    __device__ __forceinline__ void refill(const InMsg& m)
    {
        if (cnt <= 32) {
            buf |= (uint64_t)in_word(m, next) << cnt;
            next += 4;
            cnt += 32;
        }
    }
    __device__ __forceinline__ uint32_t pos() const { return next * 8 - cnt; }
    __device__ __forceinline__ uint32_t avail() const
    {
        uint32_t p = pos();
        return p < total_bits ? total_bits - p : 0;
    }
    __device__ __forceinline__ uint32_t peek(unsigned n) const { return (uint32_t)(buf & ((1ull << n) - 1)); }
    __device__ __forceinline__ void drop(unsigned n) { buf >>= n; cnt -= n; }
    __device__ __forceinline__ uint32_t take(unsigned n)
    {
        uint32_t v = peek(n);
        drop(n);
        return v;
    }
};

// Output: stage in LDS, history beyond the stage in global memory.
struct Out {
    uint8_t* g;          // message output slot
    uint32_t cap;
    uint32_t pos;        // bytes produced
    uint32_t base;       // absolute position of stage[0]
    uint8_t* stage;
};

__device__ void flush_stage(Out& o, uint32_t upto)
{
    // copy stage[0, upto-base) to global [base, upto)
    const unsigned lane = lane_id();
    uint32_t n = upto - o.base;
    uint8_t* dst = o.g + o.base;
    if ((((uintptr_t)dst) & 15) == 0) {
        uint32_t n16 = n & ~15u;
        for (uint32_t i = lane * 16; i < n16; i += WAVE * 16)
            *(uint4*)(dst + i) = *(const uint4*)(o.stage + i);
        for (uint32_t i = n16 + lane; i < n; i += WAVE) dst[i] = o.stage[i];
    } else {
        for (uint32_t i = lane; i < n; i += WAVE) dst[i] = o.stage[i];
    }
    __builtin_amdgcn_s_waitcnt(0);   // stores visible to this wave's later loads
    __threadfence_block();
}

__device__ __forceinline__ uint8_t out_read(const Out& o, uint32_t q)
{
    return q >= o.base ? o.stage[q - o.base] : o.g[q];
}

// make room so that [pos, pos+n) fits in the stage (n <= STAGE/2)
__device__ __forceinline__ void stage_room(Out& o, uint32_t n)
{
    if (o.pos + n - o.base > STAGE) {
        // keep the stage aligned to STAGE/2 so the tail stays resident
        uint32_t keep_from = o.pos & ~(STAGE / 2 - 1);
        if (keep_from > o.base) {
            flush_stage(o, keep_from);
            uint32_t shift = keep_from - o.base;
            uint32_t live = o.pos - keep_from;
            const unsigned lane = lane_id();
            for (uint32_t i = lane; i < live; i += WAVE) {
                uint8_t c = o.stage[shift + i];
                __builtin_amdgcn_wave_barrier();
                o.stage[i] = c;
            }
            __builtin_amdgcn_wave_barrier();
            o.base = keep_from;
        }
    }
}

// wave-parallel match copy: out[pos + k] = out[pos - dist + (k mod dist)]
__device__ __forceinline__ void copy_match(Out& o, uint32_t len, uint32_t dist)
{
    const unsigned lane = lane_id();
    uint32_t start = o.pos;
    if (dist >= len) {
        for (uint32_t k = lane; k < len; k += WAVE) {
            uint8_t c = out_read(o, start - dist + k);
            o.stage[start + k - o.base] = c;
        }
    } else {
        // overlapping: rounds of min(dist, 64) bytes, each round reads only
        // bytes finished by earlier rounds
        uint32_t step = dist < WAVE ? dist : WAVE;
        for (uint32_t k0 = 0; k0 < len; k0 += step) {
            uint32_t k = k0 + lane;
            uint8_t c = 0;
            if (lane < step && k < len) c = out_read(o, start - dist + k);
            __builtin_amdgcn_wave_barrier();
            if (lane < step && k < len) o.stage[start + k - o.base] = c;
            __builtin_amdgcn_wave_barrier();
        }
    }
    __builtin_amdgcn_wave_barrier();
    o.pos = start + len;
}

// Decode one symbol with Beast's fill rule.  Returns false when the input
// cannot supply the bits the reference would ask for.
__device__ __forceinline__ bool decode_sym(Bits& b, const InMsg& m, const uint16_t* tab, unsigned root,
                                           uint16_t& out)
{
    b.refill(m);
    uint32_t av = b.avail();
    if (av < root) return false;
    uint16_t s = tab[b.peek(root)];
    if (slot_is_link(s)) {
        unsigned sub = slot_bits(s);
        if (av < root + sub) return false;
        uint16_t t = tab[slot_val(s) + ((b.peek(root + sub)) >> root)];
        b.drop(root + slot_bits(t));
        out = t;
        return true;
    }
    b.drop(slot_bits(s));
    out = s;
    return true;
}

static const __constant__ uint8_t kClenOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// One message; all lanes run the same control flow (uniform state).
// raw: plain zlib::inflate_stream::write() semantics (no tail; a full output
// buffer ends the call without error).  Otherwise the pmd message semantics:
// producing byte cap+1 reports need_buffers.
__device__ void inflate_one(WaveLds& L, const InMsg& m, Out& o, uint32_t& out_len, int32_t& status, bool raw)
{
    const int32_t full_status = raw ? ST_OK : ST_NEED_BUFFERS;
    const unsigned lane = lane_id();
    Bits b;
    b.buf = 0;
    b.cnt = 0;
    b.next = 0;
    b.total_bits = m.total * 8;
    int st = ST_OK;
    bool last = false;

    if (m.total == 0) {            // raw mode, empty input: no progress
        out_len = 0;
        status = ST_NEED_BUFFERS;
        return;
    }

    for (;;) {
        // ---- TYPEDO (inflate_stream.ipp:146-182)
        if (last) { st = ST_END_OF_STREAM; break; }
        b.refill(m);
        if (b.avail() < 3) break;
        last = b.take(1) != 0;
        unsigned type = b.take(2);
        unsigned lroot = 9, droot = 6;
        const uint16_t* ltab = L.tab;
        const uint16_t* dtab = L.tab;
        if (type == 0) {
            // ---- STORED / COPY (ipp:184-220)
            b.drop(b.cnt & 7);
            if (b.avail() < 32) break;
            b.refill(m);
            uint32_t v = b.take(16);
            uint32_t nv = b.take(16);
            if (v != (nv ^ 0xffffu)) { st = ST_INVALID_STORED_LENGTH; break; }
            // bytes left in the reservoir are whole bytes; rewind them
            uint32_t from = b.next - b.cnt / 8;
            b.buf = 0;
            b.cnt = 0;
            uint32_t have = m.total > from ? m.total - from : 0;
            uint32_t n = v < have ? v : have;
            bool overflow = false;
            if (o.pos + n > o.cap) { n = o.cap - o.pos; overflow = true; }
            // copy in pieces that fit the stage
            uint32_t done = 0;
            while (done < n) {
                uint32_t piece = n - done;
                if (piece > STAGE / 2) piece = STAGE / 2;
                stage_room(o, piece);
                for (uint32_t k = lane; k < piece; k += WAVE)
                    o.stage[o.pos + k - o.base] = (uint8_t)in_byte(m, from + done + k);
                __builtin_amdgcn_wave_barrier();
                o.pos += piece;
                done += piece;
            }
            b.next = from + n;
            if (overflow) { st = full_status; break; }
            if (n < v) break;            // input ran out inside the block
            continue;
        } else if (type == 1) {
            // fixed tables: copy into the wave's table space
            for (unsigned k = lane; k < 512; k += WAVE) L.tab[k] = g_fixed_lens[k];
            for (unsigned k = lane; k < 32; k += WAVE) L.tab[512 + k] = g_fixed_dists[k];
            __builtin_amdgcn_wave_barrier();
            lroot = 9;
            droot = 5;
            dtab = L.tab + 512;
        } else if (type == 2) {
            // ---- TABLE / LENLENS / CODELENS (ipp:222-354)
            b.refill(m);
            if (b.avail() < 14) break;
            unsigned nlen = b.take(5) + 257;
            unsigned ndist = b.take(5) + 1;
            unsigned ncode = b.take(4) + 4;
            if (nlen > 286 || ndist > 30) { st = ST_TOO_MANY_SYMBOLS; break; }
            bool starved = false;
            if (lane < 19) L.lens[lane] = 0;
            __builtin_amdgcn_wave_barrier();
            for (unsigned i = 0; i < ncode; ++i) {
                b.refill(m);
                if (b.avail() < 3) { starved = true; break; }
                unsigned v = b.take(3);
                if (lane == 0) L.lens[kClenOrder[i]] = (uint8_t)v;
            }
            if (starved) break;
            __builtin_amdgcn_wave_barrier();
            unsigned croot = 7, used = 0;
            int r = 0;
            if (lane == 0) r = build_table(BUILD_CODES, L.lens, 19, L.tab, &croot, &used, L.sorted);
            r = __shfl(r, 0);
            croot = __shfl(croot, 0);
            __builtin_amdgcn_wave_barrier();
            if (r) { st = r; break; }
            unsigned have = 0;
            while (have < nlen + ndist) {
                uint16_t s;
                if (!decode_sym(b, m, L.tab, croot, s)) { starved = true; break; }
                unsigned sym = slot_val(s);
                if (sym < 16) {
                    if (lane == 0) L.lens[have] = (uint8_t)sym;
                    ++have;
                    continue;
                }
                // repeat codes: the reference asks for code+extra bits at once
                // (ipp:282-312); the code bits were already consumed above, so
                // ask for the extra bits only
                unsigned xb = sym == 16 ? 2 : sym == 17 ? 3 : 7;
                b.refill(m);
                if (b.avail() < xb) { starved = true; break; }
                unsigned rep, val;
                if (sym == 16) {
                    if (have == 0) { st = ST_INVALID_BIT_LENGTH_REPEAT; break; }
                    rep = 3 + b.take(2);
                    __builtin_amdgcn_wave_barrier();
                    val = L.lens[have - 1];
                } else if (sym == 17) {
                    rep = 3 + b.take(3);
                    val = 0;
                } else {
                    rep = 11 + b.take(7);
                    val = 0;
                }
                if (have + rep > nlen + ndist) { st = ST_INVALID_BIT_LENGTH_REPEAT; break; }
                for (unsigned k = lane; k < rep; k += WAVE) L.lens[have + k] = (uint8_t)val;
                __builtin_amdgcn_wave_barrier();
                have += rep;
            }
            if (st) break;
            if (starved) break;
            __builtin_amdgcn_wave_barrier();
            if (L.lens[256] == 0) { st = ST_MISSING_EOB; break; }
            lroot = 9;
            droot = 6;
            unsigned lused = 0, dused = 0;
            int r1 = 0, r2 = 0;
            if (lane == 0) {
                r1 = build_table(BUILD_LENS, L.lens, nlen, L.tab, &lroot, &lused, L.sorted);
                if (!r1) r2 = build_table(BUILD_DISTS, L.lens + nlen, ndist, L.tab + lused, &droot, &dused, L.sorted);
            }
            r1 = __shfl(r1, 0);
            r2 = __shfl(r2, 0);
            lroot = __shfl(lroot, 0);
            droot = __shfl(droot, 0);
            lused = __shfl(lused, 0);
            __builtin_amdgcn_wave_barrier();
            if (r1) { st = r1; break; }
            if (r2) { st = r2; break; }
            dtab = L.tab + lused;
        } else {
            st = ST_INVALID_BLOCK_TYPE;
            break;
        }

        // ---- LEN ... MATCH (ipp:356-514)
        bool block_end = false;
        for (;;) {
            uint16_t s;
            if (!decode_sym(b, m, ltab, lroot, s)) break;
            unsigned kind = slot_kind(s);
            if (kind == K_VAL) {
                if (o.pos >= o.cap) { st = full_status; break; }
                stage_room(o, 1);
                if (lane == 0) o.stage[o.pos - o.base] = (uint8_t)slot_val(s);
                __builtin_amdgcn_wave_barrier();
                o.pos += 1;
                continue;
            }
            if (kind == K_EOB) { block_end = true; break; }
            if (kind == K_SPECIAL) { st = ST_INVALID_LITERAL_LENGTH; break; }
            unsigned li = slot_val(s);
            unsigned len = kLenBase[li];
            unsigned xb = kLenExtra[li];
            if (xb) {
                b.refill(m);
                if (b.avail() < xb) break;
                len += b.take(xb);
            }
            if (!decode_sym(b, m, dtab, droot, s)) break;
            if (slot_kind(s) == K_SPECIAL) { st = ST_INVALID_DISTANCE_CODE; break; }
            unsigned di = slot_val(s);
            unsigned dist = kDistBase[di];
            xb = kDistExtra[di];
            if (xb) {
                b.refill(m);
                if (b.avail() < xb) break;
                dist += b.take(xb);
            }
            // a full buffer stops the reference before its distance check
            // (ipp:475-476) when the caller's capacity is exact (raw); the
            // pmd driver gives it one spare byte, so the check comes first
            if (raw && o.pos >= o.cap) break;
            if (dist > o.pos) { st = ST_INVALID_DISTANCE; break; }
            if (o.pos >= o.cap) { st = full_status; break; }
            bool overflow = false;
            if (o.pos + len > o.cap) { len = o.cap - o.pos; overflow = true; }
            stage_room(o, len);
            copy_match(o, len, dist);
            if (overflow) { st = full_status; break; }
        }
        if (!block_end) break;   // starved, error or overflow
    }
    if (o.pos > o.base) flush_stage(o, o.pos);
    out_len = o.pos;
    status = st;
}

__global__ void __launch_bounds__(WAVES_PER_BLOCK * WAVE)
inflate_kernel_v1(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                  const uint32_t* __restrict__ in_len, uint32_t n_msgs, uint8_t* __restrict__ out,
                  const uint64_t* __restrict__ out_off, const uint32_t* __restrict__ out_cap,
                  uint32_t* __restrict__ out_len, int32_t* __restrict__ status, uint32_t raw)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const unsigned wave = threadIdx.x / WAVE;
    WaveLds& L = reinterpret_cast<WaveLds*>(smem)[wave];
    const uint32_t msg = blockIdx.x * WAVES_PER_BLOCK + wave;
    if (msg >= n_msgs) return;
    InMsg m;
    m.p = in + in_off[msg];
    m.n = in_len[msg];
    m.total = m.n + (raw ? 0u : 4u);
    Out o;
    o.g = out + out_off[msg];
    o.cap = out_cap[msg];
    o.pos = 0;
    o.base = 0;
    o.stage = L.stage;
    uint32_t ol = 0;
    int32_t st = 0;
    inflate_one(L, m, o, ol, st, raw != 0);
    if (lane_id() == 0) {
        out_len[msg] = ol;
        status[msg] = st;
    }
}

}  // namespace bpmd

// ---------------------------------------------------------------- launcher

extern "C" int bpmd_internal_inflate_v1(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                                        uint32_t n, uint8_t* out, const uint64_t* out_off,
                                        const uint32_t* out_cap, uint32_t* out_len, int32_t* status,
                                        uint32_t raw, hipStream_t stream)
{
    using namespace bpmd;
    if (n == 0) return 0;
    dim3 grid((n + WAVES_PER_BLOCK - 1) / WAVES_PER_BLOCK);
    size_t lds = sizeof(WaveLds) * WAVES_PER_BLOCK;
    hipLaunchKernelGGL(inflate_kernel_v1, grid, dim3(WAVES_PER_BLOCK * WAVE), lds, stream, in, in_off, in_len, n,
                       out, out_off, out_cap, out_len, status, raw);
    return (int)hipGetLastError();
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
