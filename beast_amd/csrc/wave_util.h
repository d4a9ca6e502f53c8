// wave_util.h -- wave64 collectives used by the pmd kernels.  All of these
// must be called with the whole wave active (cross-lane reads from an
// inactive lane return 0 on CDNA).
#pragma once

#include "pmd_common.h"

namespace bpmd {

__device__ __forceinline__ void wave_sync() { __builtin_amdgcn_wave_barrier(); asm volatile("" ::: "memory"); }

__device__ __forceinline__ uint32_t wave_sum(uint32_t x)
{
#pragma unroll
    for (unsigned d = 1; d < WAVE; d <<= 1) x += __shfl_xor(x, d);
    return x;
}

__device__ __forceinline__ uint32_t wave_maxu(uint32_t x)
{
#pragma unroll
    for (unsigned d = 1; d < WAVE; d <<= 1) {
        const uint32_t y = __shfl_xor(x, d);
        x = x > y ? x : y;
    }
    return x;
}

__device__ __forceinline__ uint32_t wave_scan_incl(uint32_t x)
{
    const unsigned lane = lane_id();
#pragma unroll
    for (unsigned d = 1; d < WAVE; d <<= 1) {
        const uint32_t y = __shfl_up(x, d);
        x += lane >= d ? y : 0u;   // select: a shuffle must not sink under divergence
    }
    return x;
}

// exclusive prefix max; lane 0 gets `ident`
__device__ __forceinline__ uint32_t wave_scan_max_excl(uint32_t x, uint32_t ident)
{
    const unsigned lane = lane_id();
#pragma unroll
    for (unsigned d = 1; d < WAVE; d <<= 1) {
        const uint32_t y = __shfl_up(x, d);
        x = (lane >= d && y > x) ? y : x;
    }
    const uint32_t e = __shfl_up(x, 1);
    return lane == 0 ? ident : (e > ident ? e : ident);
}

__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }

__device__ __forceinline__ unsigned popc_below(uint64_t m)
{
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
}

}  // namespace bpmd
