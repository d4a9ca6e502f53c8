// pmd_multi.hip -- one process driving a batch split over several GPUs
// (SURVEY.md 8(b)/(e)): a C++ server holding impl_base's codecs for many
// connections can shard a batch without torch.distributed.
//
// With no_context_takeover every message is an independent DEFLATE stream,
// so a batch splits into contiguous, byte-balanced message ranges
// (bpmd_shard_ranges, the same cut as beast_amd/shard.py); each shard's
// payloads and output slots live on its own device and no payload crosses
// GPUs.  The *_multi calls launch every shard on its device and stream
// (asynchronously, one host thread), and when asked gather each shard's total
// output bytes -- a per-device reduction of d_out_len read back to the host
// -- so every shard's place in one global output layout is known
// (exclusive prefix sum).  That gather is the only exchange the path has;
// multi-process deployments (one process per GPU) do it with an RCCL
// all-gather instead (beast_amd/shard.py global_output_offsets).
#include <hip/hip_runtime.h>

#include <mutex>
#include <thread>
#include <vector>

#include "../../include/beast_pmd.h"

extern "C" void* bpmd_internal_scratch(hipStream_t s, size_t bytes, int which);

namespace {

__global__ void sum_lens_kernel(const uint32_t* __restrict__ len, uint32_t n, unsigned long long* __restrict__ total)
{
    unsigned long long acc = 0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) acc += len[i];
    // wave reduction, then one atomic per wave
    for (int d = 32; d >= 1; d >>= 1) acc += __shfl_down(acc, d);
    if ((threadIdx.x & 63) == 0 && acc) atomicAdd(total, acc);
}

typedef int (*batch_fn)(const bpmd_cfg*, const uint8_t*, const uint64_t*, const uint32_t*, uint32_t, uint8_t*,
                        const uint64_t*, const uint32_t*, uint32_t*, int32_t*, void*);

extern "C" void* bpmd_internal_stream_mutex(hipStream_t s);

// one shard: its batch call, then (out_bytes) the per-shard total on the
// shard's own stream, after its batch (scratch block 8), under the stream's
// launch lock like every scratch user
int run_shard(batch_fn fn, const bpmd_cfg* cfg, const bpmd_shard& s, bool want_total, unsigned long long** sum)
{
    if (hipSetDevice(s.device) != hipSuccess) return BPMD_R_HIP_ERROR;
    int r = fn(cfg, s.d_in, s.d_in_off, s.d_in_len, s.n_msgs, s.d_out, s.d_out_off, s.d_out_cap, s.d_out_len,
               s.d_status, s.stream);
    if (r || !want_total) return r;
    const hipStream_t hs = (hipStream_t)s.stream;
    std::mutex* mu = (std::mutex*)bpmd_internal_stream_mutex(hs);
    if (!mu) return BPMD_R_HIP_ERROR;
    std::lock_guard<std::mutex> launch(*mu);
    *sum = (unsigned long long*)bpmd_internal_scratch(hs, 256, 8);
    if (!*sum || hipMemsetAsync(*sum, 0, sizeof(unsigned long long), hs) != hipSuccess) return BPMD_R_HIP_ERROR;
    if (s.n_msgs) {
        const uint32_t blocks = s.n_msgs / 256 + 1 < 1024 ? s.n_msgs / 256 + 1 : 1024;
        hipLaunchKernelGGL(sum_lens_kernel, dim3(blocks), dim3(256), 0, hs, s.d_out_len, s.n_msgs, *sum);
        if (hipGetLastError() != hipSuccess) return BPMD_R_HIP_ERROR;
    }
    return BPMD_R_OK;
}

int run_multi(batch_fn fn, const bpmd_cfg* cfg, const bpmd_shard* shards, int n_shards, uint64_t* out_bytes)
{
    if (!cfg || n_shards < 0 || (n_shards && !shards)) return BPMD_R_INVALID_ARGUMENT;
    int cur = 0, count = 0;
    if (hipGetDevice(&cur) != hipSuccess || hipGetDeviceCount(&count) != hipSuccess || count == 0)
        return BPMD_R_NO_DEVICE;
    for (int i = 0; i < n_shards; ++i)
        if (shards[i].device < 0 || shards[i].device >= count) return BPMD_R_INVALID_ARGUMENT;
    std::vector<unsigned long long*> sums((size_t)n_shards, nullptr);
    std::vector<int> rs((size_t)n_shards, BPMD_R_OK);
    // every shard launched from a host thread of its own: a call that waits
    // on its stream (a deflate batch with messages over 4 KiB reads back its
    // chunk count) then waits beside the other shards' launches, not before
    // them (round 4 launched the shards one after another)
    if (n_shards == 1) {
        rs[0] = run_shard(fn, cfg, shards[0], out_bytes != nullptr, &sums[0]);
    } else {
        std::vector<std::thread> th;
        th.reserve((size_t)n_shards);
        for (int i = 0; i < n_shards; ++i)
            th.emplace_back([&, i] { rs[i] = run_shard(fn, cfg, shards[i], out_bytes != nullptr, &sums[i]); });
        for (auto& t : th) t.join();
    }
    int r = BPMD_R_OK;
    for (int i = 0; i < n_shards; ++i)
        if (rs[i] != BPMD_R_OK && r == BPMD_R_OK) r = rs[i];
    // gather the totals
    for (int i = 0; i < n_shards && r == BPMD_R_OK && out_bytes; ++i) {
        unsigned long long v = 0;
        if (hipSetDevice(shards[i].device) != hipSuccess ||
            hipMemcpyAsync(&v, sums[i], sizeof v, hipMemcpyDeviceToHost, (hipStream_t)shards[i].stream) !=
                hipSuccess ||
            hipStreamSynchronize((hipStream_t)shards[i].stream) != hipSuccess) {
            r = BPMD_R_HIP_ERROR;
            break;
        }
        out_bytes[i] = v;
    }
    (void)hipSetDevice(cur);
    return r;
}

}  // namespace

extern "C" int bpmd_shard_ranges(const uint32_t* lens, uint32_t n, int n_parts, uint32_t* starts)
{
    // beast_amd/shard.py byte_balanced_ranges: shard r ends at the first
    // message whose byte prefix sum reaches (r + 1) / n_parts of the total
    if (n_parts < 1 || !starts || (n && !lens)) return BPMD_R_INVALID_ARGUMENT;
    uint64_t total = 0;
    for (uint32_t i = 0; i < n; ++i) total += lens[i];
    starts[0] = 0;
    uint64_t csum = 0;
    uint32_t i = 0;
    for (int r = 1; r < n_parts; ++r) {
        uint32_t cut;
        if (total) {
            const double target = (double)(total * (uint64_t)r) / (double)n_parts;
            while (i < n && (double)(csum + lens[i]) < target) csum += lens[i++];
            cut = i < n ? i + 1 : n;   // the first prefix sum >= target, inclusive
        } else {
            cut = (uint32_t)(((uint64_t)n * (uint64_t)r) / (uint64_t)n_parts);
        }
        if (cut < starts[r - 1]) cut = starts[r - 1];
        starts[r] = cut < n ? cut : n;
    }
    starts[n_parts] = n;
    return BPMD_R_OK;
}

extern "C" int bpmd_inflate_batch_multi(const bpmd_cfg* cfg, const bpmd_shard* shards, int n_shards,
                                        uint64_t* out_bytes)
{
    return run_multi(bpmd_inflate_batch, cfg, shards, n_shards, out_bytes);
}

extern "C" int bpmd_deflate_batch_multi(const bpmd_cfg* cfg, const bpmd_shard* shards, int n_shards,
                                        uint64_t* out_bytes)
{
    return run_multi(bpmd_deflate_batch, cfg, shards, n_shards, out_bytes);
}
