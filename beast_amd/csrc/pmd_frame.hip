// pmd_frame.hip -- the byte passes either side of the codec on Beast's frame
// path:
//
//   * masking: payload byte j ^= prepared[(j + phase) % 4], prepared[i] =
//     key >> 8i (websocket/detail/mask.ipp:20-59); the key is the frame
//     header's, read little-endian (impl/stream_impl.hpp:866-870).  Masking
//     is an involution: one pass masks (write.hpp:679-685) or unmasks
//     (read.hpp:1324-1327).
//   * UTF-8 validation of text payloads (websocket/detail/utf8_checker.ipp:
//     39-315, called at read.hpp:1372-1384).  For one message fed as a
//     single write() the checker accepts exactly the well-formed UTF-8 of
//     RFC 3629 (valid(), utf8_checker.ipp:43-85: no overlongs, no
//     surrogates, nothing above U+10FFFF); a message that stops inside a
//     code point whose bytes so far are a valid prefix passes write() (the
//     fail-fast rule, :86-157) and fails finish() (:31-37).
//
// Both passes stream HBM: one wave per message, 16 bytes per lane per step,
// aligned 16-byte accesses (an aligned block holding a payload byte never
// leaves that byte's page).  The mask pass stores bytes one at a time only at
// a message's two ragged edges, so neighbouring messages are never
// read-modify-written.
//
// The fused forms -- unmasking inside inflate's input loads, masking inside
// deflate's output stores -- live in the codec kernels; bpmd_read_batch runs
// the UTF-8 pass right after inflate on the same stream (pmd_capi.hip).
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bpmd {
namespace frame {

constexpr unsigned WAVE = 64;
constexpr unsigned WPB = 4;   // waves (messages in flight) per block
constexpr uint32_t H = 0x80808080u;

// rotate right by 8*r bits: byte t of the result is byte (t + r) % 4 of k
__device__ __forceinline__ uint32_t rotr8(uint32_t k, uint32_t r) { return __builtin_amdgcn_alignbit(k, k, 8u * (r & 3u)); }

__global__ void __launch_bounds__(WAVE * WPB)
mask_kernel(uint8_t* __restrict__ data, const uint64_t* __restrict__ off, const uint32_t* __restrict__ len,
            const uint32_t* __restrict__ key, const uint8_t* __restrict__ phase, uint32_t n)
{
    const unsigned lane = threadIdx.x & (WAVE - 1);
    for (uint32_t m = blockIdx.x * WPB + (threadIdx.x / WAVE); m < n; m += gridDim.x * WPB) {
        const uint32_t nb = len[m];
        if (nb == 0) continue;
        uint8_t* p = data + off[m];
        const uint32_t s = (uint32_t)((uintptr_t)p & 15u);
        uint8_t* base = p - s;
        // byte base + a is payload byte a - s: prepared[(a - s + phase) % 4],
        // so every dword of an aligned block takes the same rotation of key
        const uint32_t kw = rotr8(key[m], (phase ? phase[m] : 0u) - s);
        const uint32_t units = (s + nb + 15u) >> 4;
        for (uint32_t u = lane; u < units; u += WAVE) {
            const uint32_t b0 = u * 16;
            if (b0 >= s && b0 + 16 <= s + nb) {
                uint4 w = *(uint4*)(base + b0);
                w.x ^= kw;
                w.y ^= kw;
                w.z ^= kw;
                w.w ^= kw;
                *(uint4*)(base + b0) = w;
            } else {
#pragma unroll
                for (uint32_t j = 0; j < 16; ++j) {
                    const uint32_t a = b0 + j;
                    if (a >= s && a < s + nb) base[a] ^= (uint8_t)(kw >> (8 * (j & 3)));
                }
            }
        }
    }
}

// byte flags (0x80 per byte) of the bytes [lo, hi) of a dword, lo/hi in bytes
// relative to the dword and clamped to 0..4
__device__ __forceinline__ uint32_t span_flags(int32_t lo, int32_t hi)
{
    lo = lo < 0 ? 0 : lo > 4 ? 4 : lo;
    hi = hi < 0 ? 0 : hi > 4 ? 4 : hi;
    if (hi <= lo) return 0u;
    const uint64_t m = (1ull << (8 * hi)) - (1ull << (8 * lo));
    return (uint32_t)m & H;
}

// the dword starting k bytes later (k = 1..3) in the byte stream lo, hi
__device__ __forceinline__ uint32_t sh(uint32_t lo, uint32_t hi, uint32_t k) { return __builtin_amdgcn_alignbit(hi, lo, 8u * k); }

// Verdict bits of one 16-byte unit: x[0..3] the unit, x[4] the next unit's
// first dword; v[0..4] the same bytes' in-message flags.  Each byte inside
// the message that starts a code point is checked against the bytes after it
// (at most 4 further on, hence x[4]):
//   invalid lead (C0, C1, F5..FF), a missing continuation, a continuation too
//   many (the byte after a complete code point), the second-byte ranges of
//   E0 / ED / F0 / F4 (overlong, surrogate, > U+10FFFF).
// A continuation byte that no lead claims is always the byte right after a
// complete code point (caught there) or the message's first byte (checked by
// the caller).  Bytes past the message count as "continuation still to come"
// for the missing-continuation test, which reports them as incomplete.
__device__ __forceinline__ void utf8_unit(const uint32_t (&x)[5], const uint32_t (&v)[5], bool& err, bool& inc)
{
    uint32_t Cx[5], Cy[5];
#pragma unroll
    for (int d = 0; d < 5; ++d) {
        const uint32_t c = x[d] & ~(x[d] << 1) & H;   // 10xxxxxx
        Cx[d] = c | (~v[d] & H);
        Cy[d] = c & v[d];
    }
    uint32_t e = 0, ic = 0;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        const uint32_t b = x[d];
        const uint32_t g0 = b & (b << 1) & H;   // 11xxxxxx
        const uint32_t g1 = g0 & (b << 2);      // 111xxxxx
        const uint32_t g2 = g1 & (b << 3);      // 1111xxxx
        const uint32_t g3 = g2 & (b << 4);      // 11111xxx
        const uint32_t a1 = ~b & H;             // 0xxxxxxx
        const uint32_t l2 = g0 & ~g1, l3 = g1 & ~g2, l4 = g2 & ~g3;
        const uint32_t lo4 = b & 0x0F0F0F0Fu, lo3 = b & 0x07070707u;
        const uint32_t z1e = ~((b & 0x1E1E1E1Eu) + 0x7F7F7F7Fu) & H;   // C0 / C1
        const uint32_t ge5 = (lo3 + 0x7B7B7B7Bu) & H;                   // F5..F7
        const uint32_t bad = g3 | (l2 & z1e) | (l4 & ge5);
        const uint32_t e0 = l3 & ~(lo4 + 0x7F7F7F7Fu);
        const uint32_t ed = l3 & ~((lo4 ^ 0x0D0D0D0Du) + 0x7F7F7F7Fu);
        const uint32_t f0 = l4 & ~(lo3 + 0x7F7F7F7Fu);
        const uint32_t f4 = l4 & ~((lo3 ^ 0x04040404u) + 0x7F7F7F7Fu);
        const uint32_t y = sh(x[d], x[d + 1], 1);                              // second bytes
        const uint32_t y20 = (y << 2) & H, y30 = ((y << 2) | (y << 3)) & H;   // >= A0, >= 90 for 10xxxxxx
        const uint32_t range = ((e0 & ~y20) | (ed & y20) | (f0 & ~y30) | (f4 & y30)) & sh(Cy[d], Cy[d + 1], 1);
        const uint32_t n2 = l2 | l3 | l4, n3 = l3 | l4;
        const uint32_t c1 = sh(Cx[d], Cx[d + 1], 1), c2 = sh(Cx[d], Cx[d + 1], 2), c3 = sh(Cx[d], Cx[d + 1], 3);
        const uint32_t t1 = sh(Cy[d], Cy[d + 1], 1), t2 = sh(Cy[d], Cy[d + 1], 2), t3 = sh(Cy[d], Cy[d + 1], 3);
        const uint32_t t4 = Cy[d + 1];
        const uint32_t ed_ =
            bad | (n2 & ~c1) | (n3 & ~c2) | (l4 & ~c3) | (a1 & t1) | (l2 & t2) | (l3 & t3) | (l4 & t4) | range;
        e |= ed_ & v[d];
        const uint32_t v1 = sh(v[d], v[d + 1], 1), v2 = sh(v[d], v[d + 1], 2), v3 = sh(v[d], v[d + 1], 3);
        ic |= ((n2 & ~v1) | (n3 & ~v2) | (l4 & ~v3)) & v[d];
    }
    err = err || e != 0;
    inc = inc || ic != 0;
}

// text == nullptr: result[m] = verdict (0 valid, 1 incomplete, 2 invalid)
// for every message.  text != nullptr: only messages with text[m] != 0 and
// result[m] == 0 are checked, and one that is not valid gets result[m] =
// fail_status (bpmd_read_batch: result holds the inflate status, data / off /
// len describe the inflated output).
__global__ void __launch_bounds__(WAVE * WPB)
utf8_kernel(const uint8_t* __restrict__ data, const uint64_t* __restrict__ off, const uint32_t* __restrict__ len,
            uint32_t n, int32_t* __restrict__ result, const uint8_t* __restrict__ text, int32_t fail_status)
{
    const unsigned lane = threadIdx.x & (WAVE - 1);
    for (uint32_t m = blockIdx.x * WPB + (threadIdx.x / WAVE); m < n; m += gridDim.x * WPB) {
        if (text && (text[m] == 0 || result[m] != 0)) continue;
        const uint32_t nb = len[m];
        const uint8_t* p = data + off[m];
        const uint32_t s = (uint32_t)((uintptr_t)p & 15u);
        const uint8_t* base = p - s;
        const uint32_t units = (s + nb + 15u) >> 4, end = s + nb;
        bool err = false, inc = false;
        for (uint32_t u0 = 0; u0 < units; u0 += WAVE) {
            const uint32_t u = u0 + lane, b0 = u * 16;
            uint4 w = make_uint4(0, 0, 0, 0);
            if (u < units) w = *(const uint4*)(base + b0);
            uint32_t nxt = __shfl_down(w.x, 1);
            if (lane == WAVE - 1) nxt = (b0 + 16 < end) ? *(const uint32_t*)(base + b0 + 16) : 0u;
            if (u >= units) continue;
            if (((w.x | w.y | w.z | w.w | nxt) & H) == 0) continue;   // all ASCII: nothing to reject
            const uint32_t x[5] = {w.x, w.y, w.z, w.w, nxt};
            if (b0 >= s && b0 + 20 <= end) {   // unit and look-ahead inside the message
                const uint32_t v[5] = {H, H, H, H, H};
                utf8_unit(x, v, err, inc);
            } else {
                uint32_t v[5];
#pragma unroll
                for (int d = 0; d < 5; ++d)
                    v[d] = span_flags((int32_t)s - (int32_t)(b0 + 4 * d), (int32_t)end - (int32_t)(b0 + 4 * d));
                utf8_unit(x, v, err, inc);
            }
            if (u == 0 && nb) {   // the first byte must start a code point
                const uint32_t f = x[s >> 2] >> (8 * (s & 3));
                err = err || (f & 0xC0u) == 0x80u;
            }
        }
        const bool any_err = __any(err), any_inc = __any(inc);
        if (lane == 0) {
            const int32_t verdict = any_err ? 2 : any_inc ? 1 : 0;
            if (!text) result[m] = verdict;
            else if (verdict) result[m] = fail_status;
        }
    }
}

// Context takeover (§8(f) N3) window maintenance: move the last keep[i]
// bytes before pos[i] of connection buffer i to its front.  The caller slides
// only when pos >= 2 * keep, so source and destination never overlap.
typedef uint4 uint4_u __attribute__((aligned(1)));

__global__ void __launch_bounds__(WAVE * WPB)
slide_kernel(uint8_t* __restrict__ buf, const uint64_t* __restrict__ base, const uint32_t* __restrict__ pos,
             const uint32_t* __restrict__ keep, uint32_t n)
{
    const unsigned lane = threadIdx.x & (WAVE - 1);
    for (uint32_t m = blockIdx.x * WPB + (threadIdx.x / WAVE); m < n; m += gridDim.x * WPB) {
        const uint32_t k = keep[m];
        uint8_t* dst = buf + base[m];
        const uint8_t* src = dst + pos[m] - k;
        for (uint32_t j = 16 * lane; j < k; j += 16 * WAVE) {
            if (j + 16 <= k) *(uint4_u*)(dst + j) = *(const uint4_u*)(src + j);
            else
                for (uint32_t t = j; t < k; ++t) dst[t] = src[t];
        }
    }
}


// ---------------------------------------------------------------- frames
// Send side of a message (write.hpp:463-545): the payload goes out in frames
// of at most frame_max bytes, each with its header (frame.hpp:134-175): FIN
// on the last, RSV1 and the opcode on the first (cont = 0 after), MASK and
// the frame's own key (little-endian on the wire) for a client, whose frame
// payload is then masked from the key's first byte.  One wave per message:
// lanes 0..13 write the header bytes, then 16 payload bytes per lane per step
// (a frame's 16-byte units start at frame offsets that are multiples of 4,
// so every dword of a unit takes the key as it is).
__device__ __forceinline__ uint32_t hdr_len(uint64_t len, bool masked)
{
    return (len <= 125 ? 2u : len <= 65535 ? 4u : 10u) + (masked ? 4u : 0u);
}

typedef uint4 uint4_fu __attribute__((aligned(1)));

__global__ void __launch_bounds__(WAVE * WPB)
frame_kernel(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off, const uint32_t* __restrict__ in_len,
             const uint8_t* __restrict__ op, const uint8_t* __restrict__ flags, const uint32_t* __restrict__ keys,
             const uint32_t* __restrict__ key_base, uint32_t frame_max, uint32_t n, uint8_t* __restrict__ wire,
             const uint64_t* __restrict__ wire_off)
{
    const unsigned lane = threadIdx.x & (WAVE - 1);
    for (uint32_t m = blockIdx.x * WPB + (threadIdx.x / WAVE); m < n; m += gridDim.x * WPB) {
        const uint32_t nb = in_len[m];
        const uint8_t* p = in + in_off[m];
        uint8_t* w = wire + wire_off[m];
        const uint32_t frames = nb == 0 ? 1u : (nb + frame_max - 1) / frame_max;
        const bool masked = keys != nullptr;
        const uint32_t kb = masked ? key_base[m] : 0u;
        const uint32_t opc = op ? op[m] & 15u : 2u;
        const bool rsv1 = flags ? (flags[m] & 1u) != 0 : true;
        uint64_t wp = 0;
        for (uint32_t f = 0; f < frames; ++f) {
            const uint32_t a = f * frame_max, len = f + 1 < frames ? frame_max : nb - a;
            const uint32_t key = masked ? keys[kb + f] : 0u;
            // header bytes 0-7 in h0, 8-13 in h1 (frame.hpp:134-175)
            const uint32_t b0 = (f + 1 == frames ? 0x80u : 0u) | (f == 0 && rsv1 ? 0x40u : 0u) | (f == 0 ? opc : 0u);
            uint64_t h0, h1 = 0;
            uint32_t hl;
            if (len <= 125) {
                h0 = b0 | (uint64_t)((masked ? 0x80u : 0u) | len) << 8;
                hl = 2;
            } else if (len <= 65535) {
                h0 = b0 | (uint64_t)((masked ? 0x80u : 0u) | 126u) << 8 | (uint64_t)(len >> 8) << 16 |
                     (uint64_t)(len & 0xffu) << 24;
                hl = 4;
            } else {
                // 64-bit big-endian length: bytes 2..9 = 0, 0, 0, 0, len >> 24 .. len
                h0 = b0 | (uint64_t)((masked ? 0x80u : 0u) | 127u) << 8 | (uint64_t)(len >> 24) << 48 |
                     (uint64_t)((len >> 16) & 0xffu) << 56;
                h1 = (uint64_t)((len >> 8) & 0xffu) | (uint64_t)(len & 0xffu) << 8;
                hl = 10;
            }
            if (masked) {
                if (hl == 10) h1 |= (uint64_t)key << 16;
                else h0 |= (uint64_t)key << (8 * hl);
                hl += 4;
            }
            if (lane < hl) w[wp + lane] = (uint8_t)((lane < 8 ? h0 >> (8 * lane) : h1 >> (8 * (lane - 8))) & 0xffu);
            uint8_t* dst = w + wp + hl;
            const uint8_t* src = p + a;
            const uint32_t full = len >> 4;
            for (uint32_t u = lane; u < full; u += WAVE) {
                uint4 v = *(const uint4_fu*)(src + 16 * u);
                v.x ^= key;
                v.y ^= key;
                v.z ^= key;
                v.w ^= key;
                *(uint4_fu*)(dst + 16 * u) = v;
            }
            const uint32_t t = 16 * full + lane;
            if (t < len) dst[t] = src[t] ^ (uint8_t)(key >> (8 * (t & 3u)));
            wp += hl + len;
        }
    }
}

}  // namespace frame
}  // namespace bpmd

namespace {
unsigned frame_grid(uint32_t n)
{
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const unsigned want = (n + bpmd::frame::WPB - 1) / bpmd::frame::WPB, cap = (unsigned)cus * 8u;
    return want < cap ? want : cap;
}
}  // namespace

extern "C" int bpmd_internal_mask(uint8_t* data, const uint64_t* off, const uint32_t* len, uint32_t n,
                                  const uint32_t* key, const uint8_t* phase, hipStream_t stream)
{
    if (n == 0) return 0;
    hipLaunchKernelGGL(bpmd::frame::mask_kernel, dim3(frame_grid(n)), dim3(bpmd::frame::WAVE * bpmd::frame::WPB), 0,
                       stream, data, off, len, key, phase, n);
    return (int)hipGetLastError();
}

extern "C" int bpmd_internal_utf8(const uint8_t* data, const uint64_t* off, const uint32_t* len, uint32_t n,
                                  int32_t* result, const uint8_t* text, int32_t fail_status, hipStream_t stream)
{
    if (n == 0) return 0;
    hipLaunchKernelGGL(bpmd::frame::utf8_kernel, dim3(frame_grid(n)), dim3(bpmd::frame::WAVE * bpmd::frame::WPB), 0,
                       stream, data, off, len, n, result, text, fail_status);
    return (int)hipGetLastError();
}

extern "C" int bpmd_internal_slide(uint8_t* buf, const uint64_t* base, const uint32_t* pos, const uint32_t* keep,
                                   uint32_t n, hipStream_t stream)
{
    if (n == 0) return 0;
    hipLaunchKernelGGL(bpmd::frame::slide_kernel, dim3(frame_grid(n)), dim3(bpmd::frame::WAVE * bpmd::frame::WPB), 0,
                       stream, buf, base, pos, keep, n);
    return (int)hipGetLastError();
}

extern "C" int bpmd_internal_frame(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, const uint8_t* op,
                                   const uint8_t* flags, const uint32_t* keys, const uint32_t* key_base,
                                   uint32_t frame_max, uint32_t n, uint8_t* wire, const uint64_t* wire_off,
                                   hipStream_t stream)
{
    if (n == 0) return 0;
    hipLaunchKernelGGL(bpmd::frame::frame_kernel, dim3(frame_grid(n)), dim3(bpmd::frame::WAVE * bpmd::frame::WPB), 0,
                       stream, in, in_off, in_len, op, flags, keys, key_base, frame_max, n, wire, wire_off);
    return (int)hipGetLastError();
}
