// wave_util.h -- wave64 collectives used by the pmd kernels.  All of these
// must be called with the whole wave active (cross-lane reads from an
// inactive lane return 0 on CDNA).
#pragma once

#include "pmd_common.h"

namespace bpmd {

__device__ __forceinline__ void wave_sync() { __builtin_amdgcn_wave_barrier(); asm volatile("" ::: "memory"); }

// DPP steps (GFX9 encodings): row_shr:n shifts within rows of 16 lanes,
// row_bcast:15 / row_bcast:31 carry a row's last lane into the next row(s);
// lanes with nothing to read take 0 (the identity of + and unsigned max).
template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ uint32_t dpp0(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROWS, 0xf, false);
}

// inclusive scans in 6 DPP steps (no LDS round trip, unlike shuffles)
__device__ __forceinline__ uint32_t wave_scan_incl(uint32_t x)
{
    x += dpp0<0x111>(x);        // row_shr:1
    x += dpp0<0x112>(x);        // row_shr:2
    x += dpp0<0x114>(x);        // row_shr:4
    x += dpp0<0x118>(x);        // row_shr:8
    x += dpp0<0x142, 0xa>(x);   // row_bcast:15 -> rows 1, 3
    x += dpp0<0x143, 0xc>(x);   // row_bcast:31 -> rows 2, 3
    return x;
}

__device__ __forceinline__ uint32_t wave_scan_maxu(uint32_t x)
{
    x = max(x, dpp0<0x111>(x));
    x = max(x, dpp0<0x112>(x));
    x = max(x, dpp0<0x114>(x));
    x = max(x, dpp0<0x118>(x));
    x = max(x, dpp0<0x142, 0xa>(x));
    x = max(x, dpp0<0x143, 0xc>(x));
    return x;
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t x)
{
    return (uint32_t)__builtin_amdgcn_readlane((int)wave_scan_incl(x), 63);
}

__device__ __forceinline__ uint32_t wave_maxu(uint32_t x)
{
    return (uint32_t)__builtin_amdgcn_readlane((int)wave_scan_maxu(x), 63);
}

// exclusive prefix max; lane 0 gets `ident`
__device__ __forceinline__ uint32_t wave_scan_max_excl(uint32_t x, uint32_t ident)
{
    const uint32_t e = __shfl_up(wave_scan_maxu(x), 1);
    return lane_id() == 0 ? ident : (e > ident ? e : ident);
}

__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }

__device__ __forceinline__ unsigned popc_below(uint64_t m)
{
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
}

}  // namespace bpmd
