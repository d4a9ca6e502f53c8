// lane_io.h -- per-lane input and output helpers shared by the lane
// inflate kernels (pmd_inflate_lane3.hip, pmd_inflate_lane4.hip): relaxed
// LDS words between the two waves of a workgroup, 16-byte input blocks of a
// payload that never touch a page past it (with the pmd tail and the client
// mask applied), and output stores bounded by the slot's capacity.
#pragma once
#include "pmd_common.h"

namespace bpmd {
namespace lio {

__device__ __forceinline__ uint32_t lds_load(const uint8_t* p)
{
    return __hip_atomic_load((const uint32_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_store(uint8_t* p, uint32_t v)
{
    __hip_atomic_store((uint32_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void compiler_fence() { asm volatile("" ::: "memory"); }

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
typedef uint32_t uint32_u __attribute__((aligned(1)));

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
        if (sz == 16) *(uint4_u*)(o + dst) = w;
        else *(uint2_u*)(o + dst) = make_uint2(w.x, w.y);
        return;
    }
    const uint32_t k = lim - dst;   // < sz
    const uint32_t d[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j)
        if (j < k) o[dst + j] = (uint8_t)(d[j >> 2] >> (8 * (j & 3)));
}

}  // namespace lio
}  // namespace bpmd
