// pmd_capi.hip -- extern "C" entry points declared in include/beast_pmd.h.
#include <hip/hip_runtime.h>

#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <mutex>
#include <new>
#include <vector>

#include "../../include/beast_pmd.h"

extern "C" int bpmd_internal_init_fixed(void);
extern "C" int bpmd_internal_inflate_keyed(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                                           uint32_t n, uint8_t* out, const uint64_t* out_off, const uint32_t* out_cap,
                                           uint32_t* out_len, int32_t* status, uint32_t raw, const uint32_t* mask_key,
                                           hipStream_t stream);

extern "C" int bpmd_internal_inflate_keyed_split(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                                                 uint32_t n, uint8_t* out, const uint64_t* out_off,
                                                 const uint32_t* out_cap, uint32_t* out_len, int32_t* status,
                                                 uint32_t raw, const uint32_t* mask_key, uint32_t min_in,
                                                 hipStream_t stream);
extern "C" int bpmd_internal_inflate_lane3(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint32_t n,
                                           uint8_t* out, const uint64_t* out_off, const uint32_t* out_cap,
                                           uint32_t* out_len, int32_t* status, uint32_t raw, const uint32_t* mask_key,
                                           const uint32_t* hist_len, uint32_t hist_max, uint32_t max_in,
                                           const uint32_t* order, uint32_t* qctr, uint32_t grid_wgs,
                                           const uint32_t* skip, hipStream_t stream);
extern "C" const uint32_t* bpmd_internal_lane_order(const uint32_t* in_len, uint32_t n, hipStream_t stream,
                                                    const uint32_t** keys_out);
extern "C" const uint32_t* bpmd_internal_lane_long_split(const uint32_t* in_len, const uint32_t* keys, uint32_t n,
                                                         uint32_t lanes, uint32_t min_thr, uint32_t share_pct,
                                                         hipStream_t stream);
extern "C" int bpmd_internal_inflate_bp(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint32_t n,
                                        uint8_t* out, const uint64_t* out_off, const uint32_t* out_cap,
                                        uint32_t* out_len, int32_t* status, uint32_t raw, const uint32_t* order,
                                        const uint32_t* nlong, hipStream_t s);
extern "C" void bpmd_internal_bp_release(hipStream_t s);
extern "C" int bpmd_internal_bp_reserve(hipStream_t s, unsigned long long in_bytes, unsigned long long out_bytes,
                                        unsigned long long msgs);
extern "C" int bpmd_internal_inflate_wave_ordered(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                                                  uint32_t n, uint8_t* out, const uint64_t* out_off,
                                                  const uint32_t* out_cap, uint32_t* out_len, int32_t* status,
                                                  uint32_t raw, const uint32_t* mask_key, const uint32_t* order,
                                                  const uint32_t* limit, hipStream_t stream);
extern "C" int bpmd_internal_deflate_keyed(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                                           uint32_t n, uint8_t* out, const uint64_t* out_off, const uint32_t* out_cap,
                                           uint32_t* out_len, int32_t* status, int level, int window_bits,
                                           int strategy, const uint32_t* mask_key, hipStream_t stream);

extern "C" int bpmd_internal_deflate_exact(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                                           uint32_t n, uint8_t* out, const uint64_t* out_off,
                                           const uint32_t* out_cap, uint32_t* out_len, int32_t* status, int level,
                                           int window_bits, int mem_level, int strategy, const uint32_t* mask_key,
                                           hipStream_t stream);

extern "C" int bpmd_internal_deflate_takeover(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                                              uint32_t n, uint8_t* out, const uint64_t* out_off,
                                              const uint32_t* out_cap, uint32_t* out_len, int32_t* status, int level,
                                              int window_bits, int strategy, const uint32_t* hist_len,
                                              hipStream_t stream);

extern "C" int bpmd_internal_mask(uint8_t* data, const uint64_t* off, const uint32_t* len, uint32_t n,
                                  const uint32_t* key, const uint8_t* phase, hipStream_t stream);
extern "C" int bpmd_internal_utf8(const uint8_t* data, const uint64_t* off, const uint32_t* len, uint32_t n,
                                  int32_t* result, const uint8_t* text, int32_t fail_status, hipStream_t stream);
extern "C" int bpmd_internal_slide(uint8_t* buf, const uint64_t* base, const uint32_t* pos, const uint32_t* keep,
                                   uint32_t n, hipStream_t stream);

namespace {
std::mutex g_init_mu;
uint64_t g_init_devices = 0;   // bit d: device d's symbols are initialised

// Per (device, stream) scratch for batch calls that need device workspace
// (work-queue counters, message order, chunk workspace).  Allocated on first
// use and grown when a larger batch arrives.  A batch call holds its
// stream's launch lock from its first enqueue to its last, so two host
// threads submitting on one stream (the null stream, say) cannot interleave
// their memsets and launches over the same counters and workspace; calls on
// different streams use different scratch.
struct Scratch {
    int dev;
    hipStream_t stream;
    int which;
    uint8_t* p;
    size_t cap;
};
struct StreamLock {
    int dev;
    hipStream_t stream;
    std::mutex* mu;
};
// A side stream per (device, stream): the long payloads of a work-queue
// batch decode block-parallel on it while the lane kernel runs the rest on
// the caller's stream (fork / join events; the caller's stream waits for the
// side stream before anything after the batch call).
struct Side {
    int dev;
    hipStream_t stream;
    hipStream_t side;
    hipEvent_t fork, join;
};
std::mutex g_scratch_mu;
std::vector<Scratch> g_scratch;
std::vector<Scratch> g_pinned;   // small pinned host blocks per (device, stream), same lifetime rules
std::vector<StreamLock> g_locks;
std::vector<Side> g_sides;

bool side_for(hipStream_t s, Side& out)
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return false;
    std::lock_guard<std::mutex> lk(g_scratch_mu);
    for (auto& e : g_sides)
        if (e.dev == dev && e.stream == s) {
            out = e;
            return true;
        }
    Side d{dev, s, nullptr, nullptr, nullptr};
    if (hipStreamCreateWithFlags(&d.side, hipStreamNonBlocking) != hipSuccess) return false;
    if (hipEventCreateWithFlags(&d.fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&d.join, hipEventDisableTiming) != hipSuccess) {
        (void)hipStreamDestroy(d.side);
        return false;
    }
    g_sides.push_back(d);
    out = d;
    return true;
}

std::mutex* stream_mutex(hipStream_t s)
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> lk(g_scratch_mu);
    for (auto& e : g_locks)
        if (e.dev == dev && e.stream == s) return e.mu;
    std::mutex* mu = new (std::nothrow) std::mutex();
    if (mu) g_locks.push_back(StreamLock{dev, s, mu});
    return mu;
}

// the caller holds the stream's launch lock, so nothing else enqueues work
// that could use the block while it is replaced
uint8_t* scratch_for(hipStream_t s, size_t bytes, int which = 0)
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    uint8_t* old = nullptr;
    {
        std::lock_guard<std::mutex> lk(g_scratch_mu);
        for (auto& e : g_scratch)
            if (e.dev == dev && e.stream == s && e.which == which) {
                if (e.cap >= bytes) return e.p;
                old = e.p;
                e.p = nullptr;
                e.cap = 0;
                break;
            }
    }
    // the stream may still use the old block: free it once the stream is idle
    if (old) {
        if (hipStreamSynchronize(s) != hipSuccess) return nullptr;
        (void)hipFree(old);
    }
    uint8_t* p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> lk(g_scratch_mu);
    for (auto& e : g_scratch)
        if (e.dev == dev && e.stream == s && e.which == which) {
            e.p = p;
            e.cap = bytes;
            return p;
        }
    g_scratch.push_back(Scratch{dev, s, which, p, bytes});
    return p;
}
}

// scratch block `which` (0 inflate queue, 1-2 deflate workspace, 3-4 exact
// deflate queue and workspace, 5 inflate message order, 6 wave inflate queue,
// 7 deflate chunk queue, 8 multi-device output totals, 9 long-payload split,
// 10-11 block-parallel inflate stats and decode workspace)
// for other translation units
extern "C" void* bpmd_internal_scratch(hipStream_t s, size_t bytes, int which)
{
    return scratch_for(s, bytes, which);
}

// A small pinned host block per (device, stream, which) -- the target of a
// read-back that an event then covers (0: the deflate chunk count).  Kept
// per stream, not per host thread: pmd_multi.hip launches each shard from a
// thread of its own, and a thread_local block would leak one pinned
// allocation per shard thread.  The caller holds the stream's
// launch lock; freed by bpmd_internal_scratch_release.
extern "C" void* bpmd_internal_pinned(hipStream_t s, size_t bytes, int which)
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || bytes > 4096) return nullptr;
    std::lock_guard<std::mutex> lk(g_scratch_mu);
    for (auto& e : g_pinned)
        if (e.dev == dev && e.stream == s && e.which == which) return e.p;
    uint8_t* p = nullptr;
    if (hipHostMalloc((void**)&p, 4096, hipHostMallocDefault) != hipSuccess) return nullptr;
    g_pinned.push_back(Scratch{dev, s, which, p, 4096});
    return p;
}
extern "C" size_t bpmd_internal_pinned_count(void)
{
    std::lock_guard<std::mutex> lk(g_scratch_mu);
    return g_pinned.size();
}

// Frees every scratch block and the launch lock of a stream that is about to
// be destroyed (per-stream codecs, batcher slots).  The caller has
// synchronised the stream and no other thread uses it.
extern "C" void bpmd_internal_scratch_release(hipStream_t s)
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return;
    bpmd_internal_bp_release(s);
    hipStream_t side = nullptr;
    {
    std::lock_guard<std::mutex> lk(g_scratch_mu);
    for (size_t i = 0; i < g_sides.size(); ++i)
        if (g_sides[i].dev == dev && g_sides[i].stream == s) {
            side = g_sides[i].side;
            (void)hipStreamSynchronize(side);
            (void)hipEventDestroy(g_sides[i].fork);
            (void)hipEventDestroy(g_sides[i].join);
            g_sides[i] = g_sides.back();
            g_sides.pop_back();
            break;
        }
    for (size_t i = 0; i < g_scratch.size();) {
        if (g_scratch[i].dev == dev && (g_scratch[i].stream == s || (side && g_scratch[i].stream == side))) {
            (void)hipFree(g_scratch[i].p);
            g_scratch[i] = g_scratch.back();
            g_scratch.pop_back();
        } else {
            ++i;
        }
    }
    for (size_t i = 0; i < g_pinned.size();) {
        if (g_pinned[i].dev == dev && (g_pinned[i].stream == s || (side && g_pinned[i].stream == side))) {
            (void)hipHostFree(g_pinned[i].p);
            g_pinned[i] = g_pinned.back();
            g_pinned.pop_back();
        } else {
            ++i;
        }
    }
    for (size_t i = 0; i < g_locks.size(); ++i)
        if (g_locks[i].dev == dev && g_locks[i].stream == s) {
            delete g_locks[i].mu;
            g_locks[i] = g_locks.back();
            g_locks.pop_back();
            break;
        }
    }
    if (side) {
        bpmd_internal_bp_release(side);
        (void)hipStreamDestroy(side);
    }
}

// the launch lock of a stream (pmd_multi.hip takes it around its own
// scratch use, as scratch_for requires)
extern "C" void* bpmd_internal_stream_mutex(hipStream_t s) { return stream_mutex(s); }

// Number of scratch blocks held (footprint tests)
extern "C" size_t bpmd_internal_scratch_count(void)
{
    std::lock_guard<std::mutex> lk(g_scratch_mu);
    return g_scratch.size();
}

extern "C" const char* bpmd_version(void) { return "beast_pmd 0.2 (gfx950)"; }

// Diagnostics only (scripts/diag_*.py): force the launch grid, e.g. one
// wave, to time a kernel's phases without other waves on the CU.
extern "C" unsigned bpmd_diag_grid_override = 0;
extern "C" void bpmd_diag_set_grid(unsigned grid) { bpmd_diag_grid_override = grid; }

// Kernel choice for a batch: one lane per message (pmd_inflate_lane3.hip)
// for throughput, one wave per message (pmd_inflate.hip) for latency when
// the batch is too small to fill the chip's lanes, and block-parallel decode
// (pmd_inflate_bp.hip) for the long payloads of large batches.
// BPMD_INFLATE=lane|wave|bp or bpmd_set_inflate_kernel() forces one (the
// tests run all three; "bp" sends every payload of 64 bytes or more through
// the block-parallel path).
static std::atomic<int> g_inflate_kernel{-1};   // -1 unset, 0 auto, 1 lane, 2 wave, 3 bp

extern "C" int bpmd_set_inflate_kernel(int mode)
{
    if (mode < 0 || mode > 3) return BPMD_R_INVALID_ARGUMENT;
    g_inflate_kernel.store(mode);
    return BPMD_R_OK;
}

static int inflate_mode()
{
    int m = g_inflate_kernel.load();
    if (m < 0) {
        const char* e = getenv("BPMD_INFLATE");
        m = (e && !strcmp(e, "lane")) ? 1 : (e && !strcmp(e, "wave")) ? 2 : (e && !strcmp(e, "bp")) ? 3 : 0;
        g_inflate_kernel.store(m);
    }
    return m;
}

// block-parallel decode of long payloads in automatic mode (BPMD_INFLATE_BP=0: off)
static bool inflate_bp_enabled()
{
    static const bool on = [] {
        const char* e = getenv("BPMD_INFLATE_BP");
        return !(e && e[0] == '0');
    }();
    return on;
}

// Automatic choice, per message: a lane-kernel wave lasts as long as its
// longest message and a batch of few messages leaves most lanes of the chip
// idle, so payloads longer than the split (compressed bytes; several 4 KiB
// chunks of output) go to the wave kernel and only batches of >= 2048
// messages use lanes at all; batches of >= 32 Ki messages use lanes only.  BPMD_INFLATE_SPLIT overrides the split.
static uint32_t inflate_split()
{
    const char* e = getenv("BPMD_INFLATE_SPLIT");
    return e ? (uint32_t)strtoul(e, nullptr, 10) : 4096u;
}

extern "C" int bpmd_init(void)
{
    int dev = -1;
    if (hipGetDevice(&dev) != hipSuccess) return BPMD_R_NO_DEVICE;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0) return BPMD_R_NO_DEVICE;
    std::lock_guard<std::mutex> lk(g_init_mu);
    const uint64_t bit = dev < 64 ? 1ull << dev : 0ull;
    if (g_init_devices & bit) return BPMD_R_OK;
    if (bpmd_internal_init_fixed() != 0) return BPMD_R_HIP_ERROR;
    g_init_devices |= bit;
    return BPMD_R_OK;
}

// The block-parallel path runs on the caller's stream (batches below 32 Ki
// messages, forced mode) or on its side stream (work-queue batches): both
// get the capacity.
extern "C" int bpmd_inflate_reserve(void* stream, uint64_t in_bytes, uint64_t out_bytes, uint32_t n_long)
{
    int r = bpmd_init();
    if (r) return r;
    const hipStream_t s = (hipStream_t)stream;
    std::mutex* mu = stream_mutex(s);
    if (!mu) return BPMD_R_HIP_ERROR;
    std::lock_guard<std::mutex> launch(*mu);
    Side sd;
    if (!side_for(s, sd)) return BPMD_R_HIP_ERROR;
    if (bpmd_internal_bp_reserve(s, in_bytes, out_bytes, n_long) ||
        bpmd_internal_bp_reserve(sd.side, in_bytes, out_bytes, n_long))
        return BPMD_R_HIP_ERROR;
    return BPMD_R_OK;
}

extern "C" size_t bpmd_deflate_upper_bound(size_t n)
{
    // zlib/deflate_stream.hpp:402-410
    return n + ((n + 7) >> 3) + ((n + 63) >> 6) + 11;
}

namespace {

// bpmd_inflate_batch and its fused / context-takeover forms.  key: masking
// keys or null; hist: window bytes before each slot (context takeover) or
// null -- only the lane kernel reads a window, so it always runs then.
int inflate_impl(const bpmd_cfg* cfg, const uint8_t* d_in, const uint64_t* d_in_off, const uint32_t* d_in_len,
                 uint32_t n_msgs, uint8_t* d_out, const uint64_t* d_out_off, const uint32_t* d_out_cap,
                 uint32_t* d_out_len, int32_t* d_status, const uint32_t* key, const uint32_t* hist, void* stream)
{
    if (!cfg) return BPMD_R_INVALID_ARGUMENT;
    // inflate_stream.ipp:57-61: windowBits outside 8..15 throws domain_error
    if (cfg->window_bits < 8 || cfg->window_bits > 15) return BPMD_R_DOMAIN_ERROR;
    if (n_msgs == 0) return BPMD_R_OK;
    if (!d_in || !d_in_off || !d_in_len || !d_out || !d_out_off || !d_out_cap || !d_out_len || !d_status)
        return BPMD_R_INVALID_ARGUMENT;
    int r = bpmd_init();
    if (r) return r;
    const uint32_t raw = (cfg->flags & BPMD_F_RAW) ? 1u : 0u;
    const hipStream_t s = (hipStream_t)stream;
    std::mutex* mu = stream_mutex(s);
    if (!mu) return BPMD_R_HIP_ERROR;
    std::lock_guard<std::mutex> launch(*mu);
    const int m = inflate_mode();
    // block-parallel decode applies to plain batches (no takeover window, no
    // masking key: the segment decoder starts mid-payload)
    const bool bp_ok = !hist && !key && ((m == 0 && inflate_bp_enabled()) || m == 3);
    if (m == 3 && bp_ok) {
        // forced (tests): every payload of 64 bytes or more, the rest on lanes
        const uint32_t* keys = nullptr;
        const uint32_t* order = bpmd_internal_lane_order(d_in_len, n_msgs, s, &keys);
        const uint32_t* nlong = order ? bpmd_internal_lane_long_split(d_in_len, keys, n_msgs, 0u, 64u, 0u, s) : nullptr;
        if (!nlong || bpmd_internal_inflate_bp(d_in, d_in_off, d_in_len, n_msgs, d_out, d_out_off, d_out_cap,
                                               d_out_len, d_status, raw, order, nlong, s) ||
            bpmd_internal_inflate_lane3(d_in, d_in_off, d_in_len, n_msgs, d_out, d_out_off, d_out_cap, d_out_len,
                                        d_status, raw, nullptr, nullptr, 1u << cfg->window_bits, 0u, order, nullptr,
                                        0u, nlong, s))
            return BPMD_R_HIP_ERROR;
        return BPMD_R_OK;
    }
    // lane-kernel share: everything (hist / forced lane), nothing (forced wave /
    // small batch), or the payloads of at most `split` bytes
    const bool lane = hist || m == 1 || (m == 0 && n_msgs >= 2048);
    // from 32 Ki messages on, the lanes fill the chip whatever the sizes: no
    // split, and no second launch (C2 +1.6 %, C4 lane-only 23.2 vs 22.6 GiB/s)
    const uint32_t split = (hist || m != 0 || n_msgs >= 32768) ? 0u : inflate_split();
    int e = 0;
    if (lane) {
        // more messages than the chip holds lanes: a work queue keeps every
        // lane busy until the batch is done (mixed sizes, configs[3])
        int dev = 0, cus = 256;
        if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        uint32_t wgs = 4u * (uint32_t)cus;   // 4 workgroups of 64 messages per CU are resident
        // diagnostics / tests: BPMD_QUEUE_WGS caps the grid so that small batches
        // run through the work queue too
        static const uint32_t q_override = [] {
            const char* e = getenv("BPMD_QUEUE_WGS");
            return e ? (uint32_t)strtoul(e, nullptr, 10) : 0u;
        }();
        if (q_override) wgs = q_override;
        uint32_t* qctr = nullptr;
        const uint32_t* order = nullptr;
        const uint32_t* nlong = nullptr;
        if (n_msgs > wgs * 64u && !split) {
            qctr = (uint32_t*)scratch_for(s, 256);
            if (!qctr || hipMemsetAsync(qctr, 0, sizeof(uint32_t), s) != hipSuccess) return BPMD_R_HIP_ERROR;
            // longest first, so no lane starts a long message as the batch drains
            // (BPMD_INFLATE_ORDER=0: batch order)
            static const bool ordered = [] {
                const char* e = getenv("BPMD_INFLATE_ORDER");
                return !(e && e[0] == '0');
            }();
            // payloads too long for one lane go to the wave kernel first
            // (automatic mode, no takeover window; BPMD_INFLATE_LONG=0: off)
            static const bool long_split = [] {
                const char* e = getenv("BPMD_INFLATE_LONG");
                return !(e && e[0] == '0');
            }();
            const uint32_t* keys = nullptr;
            if (ordered && !(order = bpmd_internal_lane_order(d_in_len, n_msgs, s, &keys))) return BPMD_R_HIP_ERROR;
            if (ordered && long_split && m == 0 && !hist) {
                // long payloads: block-parallel, or one wave each
                // (block-parallel: above 1.25 lanes' share of the batch, from 2 KiB
                // compressed; DESIGN.md 4.1c.  One 8-way C4 shard at 50 / 100 /
                // 150 / 200 %: 9.2 / 8.4-8.9 / 8.3 / 10.5 ms; C4 projected 4- and
                // 8-way speedups at 100 / 125 / 150 %: 3.29-3.30 and 5.29 / 3.36-3.46
                // and 5.30-5.36 / 2.81-2.95 and 5.39-5.45, round 4)
                static const uint32_t share_pct = [] {
                    const char* e = getenv("BPMD_LONG_SHARE_PCT");
                    return e ? (uint32_t)strtoul(e, nullptr, 10) : 125u;
                }();
                if (!(nlong = bp_ok ? bpmd_internal_lane_long_split(d_in_len, keys, n_msgs, wgs * 64u, 2048u, share_pct, s)
                                    : bpmd_internal_lane_long_split(d_in_len, keys, n_msgs, wgs * 64u, 4096u, 200u, s)))
                    return BPMD_R_HIP_ERROR;
                if (bp_ok) {
                    // the lane kernel on the caller's stream (it skips the long
                    // prefix of the order) and the long payloads block-parallel
                    // on the side stream at the same time: each fills the CUs
                    // the other's tail leaves idle
                    Side sd;
                    if (!side_for(s, sd) || hipEventRecord(sd.fork, s) != hipSuccess ||
                        hipStreamWaitEvent(sd.side, sd.fork, 0) != hipSuccess)
                        return BPMD_R_HIP_ERROR;
                    // (both enqueue only, except the stream's first
                    // block-parallel call without bpmd_inflate_reserve: it
                    // reads its workspace totals back once, on the side
                    // stream, so it waits for the work queued before it --
                    // and cannot run under stream capture)
                    const int eb = bpmd_internal_inflate_bp(d_in, d_in_off, d_in_len, n_msgs, d_out, d_out_off,
                                                            d_out_cap, d_out_len, d_status, raw, order, nlong, sd.side);
                    e = bpmd_internal_inflate_lane3(d_in, d_in_off, d_in_len, n_msgs, d_out, d_out_off, d_out_cap,
                                                    d_out_len, d_status, raw, key, hist, 1u << cfg->window_bits, 0u,
                                                    order, qctr, wgs, nlong, s);
                    if (hipEventRecord(sd.join, sd.side) != hipSuccess || hipStreamWaitEvent(s, sd.join, 0) != hipSuccess)
                        return BPMD_R_HIP_ERROR;
                    return e || eb ? BPMD_R_HIP_ERROR : BPMD_R_OK;
                }
                if (bpmd_internal_inflate_wave_ordered(d_in, d_in_off, d_in_len, n_msgs, d_out, d_out_off, d_out_cap,
                                                       d_out_len, d_status, raw, key, order, nlong, s))
                    return BPMD_R_HIP_ERROR;
            }
        } else if (split && bp_ok) {
            // payloads over the split: block-parallel; the rest on lanes, in
            // the same longest-first order after them
            const uint32_t* keys = nullptr;
            if (!(order = bpmd_internal_lane_order(d_in_len, n_msgs, s, &keys)) ||
                !(nlong = bpmd_internal_lane_long_split(d_in_len, keys, n_msgs, 0u, split, 0u, s)) ||
                bpmd_internal_inflate_bp(d_in, d_in_off, d_in_len, n_msgs, d_out, d_out_off, d_out_cap, d_out_len,
                                         d_status, raw, order, nlong, s))
                return BPMD_R_HIP_ERROR;
            e = bpmd_internal_inflate_lane3(d_in, d_in_off, d_in_len, n_msgs, d_out, d_out_off, d_out_cap, d_out_len,
                                            d_status, raw, key, hist, 1u << cfg->window_bits, 0u, order, nullptr, wgs,
                                            nlong, s);
            return e ? BPMD_R_HIP_ERROR : BPMD_R_OK;
        }
        e = bpmd_internal_inflate_lane3(d_in, d_in_off, d_in_len, n_msgs, d_out, d_out_off, d_out_cap, d_out_len,
                                        d_status, raw, key, hist, 1u << cfg->window_bits, split, order, qctr, wgs,
                                        nlong, s);
    }
    if (!e && (!lane || split))
        e = bpmd_internal_inflate_keyed_split(d_in, d_in_off, d_in_len, n_msgs, d_out, d_out_off, d_out_cap,
                                              d_out_len, d_status, raw, key, lane ? split : 0u, s);
    return e ? BPMD_R_HIP_ERROR : BPMD_R_OK;
}

int deflate_impl(const bpmd_cfg* cfg, const uint8_t* d_in, const uint64_t* d_in_off, const uint32_t* d_in_len,
                 uint32_t n_msgs, uint8_t* d_out, const uint64_t* d_out_off, const uint32_t* d_out_cap,
                 uint32_t* d_out_len, int32_t* d_status, const uint32_t* key, const uint32_t* hist, void* stream)
{
    if (!cfg) return BPMD_R_INVALID_ARGUMENT;
    // deflate_stream.ipp:235-253: level -1 means 6; windowBits 8 becomes 9;
    // anything outside level 0..9, windowBits 8..15, memLevel 1..9 throws
    // std::invalid_argument.
    int level = cfg->level == -1 ? 6 : cfg->level;
    int wbits = cfg->window_bits == 8 ? 9 : cfg->window_bits;
    if (level < 0 || level > 9 || wbits < 8 || wbits > 15 || cfg->mem_level < 1 || cfg->mem_level > 9)
        return BPMD_R_INVALID_ARGUMENT;
    if (cfg->strategy < BPMD_STRATEGY_NORMAL || cfg->strategy > BPMD_STRATEGY_FIXED) return BPMD_R_INVALID_ARGUMENT;
    if (n_msgs == 0) return BPMD_R_OK;
    if (!d_in || !d_in_off || !d_in_len || !d_out || !d_out_off || !d_out_cap || !d_out_len || !d_status)
        return BPMD_R_INVALID_ARGUMENT;
    int r = bpmd_init();
    if (r) return r;
    std::mutex* mu = stream_mutex((hipStream_t)stream);
    if (!mu) return BPMD_R_HIP_ERROR;
    std::lock_guard<std::mutex> launch(*mu);
    if (cfg->flags & BPMD_F_EXACT) {
        // the reference's own algorithm, message by message (pmd_deflate_exact.hip)
        if (hist) return BPMD_R_INVALID_ARGUMENT;
        return bpmd_internal_deflate_exact(d_in, d_in_off, d_in_len, n_msgs, d_out, d_out_off, d_out_cap, d_out_len,
                                           d_status, level, wbits, cfg->mem_level, cfg->strategy, key,
                                           (hipStream_t)stream)
                   ? BPMD_R_HIP_ERROR
                   : BPMD_R_OK;
    }
    int e = hist ? bpmd_internal_deflate_takeover(d_in, d_in_off, d_in_len, n_msgs, d_out, d_out_off, d_out_cap,
                                                  d_out_len, d_status, level, wbits, cfg->strategy, hist,
                                                  (hipStream_t)stream)
                 : bpmd_internal_deflate_keyed(d_in, d_in_off, d_in_len, n_msgs, d_out, d_out_off, d_out_cap,
                                               d_out_len, d_status, level, wbits, cfg->strategy, key,
                                               (hipStream_t)stream);
    return e ? BPMD_R_HIP_ERROR : BPMD_R_OK;
}

}  // namespace

extern "C" int bpmd_inflate_batch(const bpmd_cfg* cfg, const uint8_t* d_in, const uint64_t* d_in_off,
                                  const uint32_t* d_in_len, uint32_t n_msgs, uint8_t* d_out,
                                  const uint64_t* d_out_off, const uint32_t* d_out_cap,
                                  uint32_t* d_out_len, int32_t* d_status, void* stream)
{
    return inflate_impl(cfg, d_in, d_in_off, d_in_len, n_msgs, d_out, d_out_off, d_out_cap, d_out_len, d_status,
                        nullptr, nullptr, stream);
}

extern "C" int bpmd_deflate_batch(const bpmd_cfg* cfg, const uint8_t* d_in, const uint64_t* d_in_off,
                                  const uint32_t* d_in_len, uint32_t n_msgs, uint8_t* d_out,
                                  const uint64_t* d_out_off, const uint32_t* d_out_cap,
                                  uint32_t* d_out_len, int32_t* d_status, void* stream)
{
    return deflate_impl(cfg, d_in, d_in_off, d_in_len, n_msgs, d_out, d_out_off, d_out_cap, d_out_len, d_status,
                        nullptr, nullptr, stream);
}

// ------------------------------------------------ frame passes (§8(f) N1)

extern "C" int bpmd_mask_batch(uint8_t* d_data, const uint64_t* d_off, const uint32_t* d_len, uint32_t n_msgs,
                               const uint32_t* d_key, const uint8_t* d_phase, void* stream)
{
    if (n_msgs == 0) return BPMD_R_OK;
    if (!d_data || !d_off || !d_len || !d_key) return BPMD_R_INVALID_ARGUMENT;
    int r = bpmd_init();
    if (r) return r;
    return bpmd_internal_mask(d_data, d_off, d_len, n_msgs, d_key, d_phase, (hipStream_t)stream) ? BPMD_R_HIP_ERROR
                                                                                                 : BPMD_R_OK;
}

extern "C" int bpmd_internal_frame(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, const uint8_t* op,
                                   const uint8_t* flags, const uint32_t* keys, const uint32_t* key_base,
                                   uint32_t frame_max, uint32_t n, uint8_t* wire, const uint64_t* wire_off,
                                   hipStream_t stream);

// frame.hpp:134-175 header sizes over the write.hpp:463-545 frame loop
extern "C" uint64_t bpmd_frame_wire_size(uint64_t payload_len, uint32_t frame_max, int masked)
{
    if (frame_max == 0) return 0;
    const uint64_t frames = payload_len == 0 ? 1 : (payload_len + frame_max - 1) / frame_max;
    const uint64_t last = payload_len - (frames - 1) * frame_max;
    auto hdr = [&](uint64_t len) -> uint64_t { return (len <= 125 ? 2u : len <= 65535 ? 4u : 10u) + (masked ? 4u : 0u); };
    return payload_len + (frames - 1) * hdr(frame_max) + hdr(last);
}

extern "C" int bpmd_frame_batch(const uint8_t* d_in, const uint64_t* d_in_off, const uint32_t* d_in_len,
                                const uint8_t* d_op, const uint8_t* d_flags, const uint32_t* d_keys,
                                const uint32_t* d_key_base, uint32_t frame_max, uint32_t n_msgs, uint8_t* d_wire,
                                const uint64_t* d_wire_off, void* stream)
{
    if (n_msgs == 0) return BPMD_R_OK;
    if (!d_in || !d_in_off || !d_in_len || !d_wire || !d_wire_off || frame_max == 0 || (d_keys && !d_key_base))
        return BPMD_R_INVALID_ARGUMENT;
    int r = bpmd_init();
    if (r) return r;
    return bpmd_internal_frame(d_in, d_in_off, d_in_len, d_op, d_flags, d_keys, d_key_base, frame_max, n_msgs, d_wire,
                               d_wire_off, (hipStream_t)stream)
               ? BPMD_R_HIP_ERROR
               : BPMD_R_OK;
}

extern "C" int bpmd_utf8_check_batch(const uint8_t* d_data, const uint64_t* d_off, const uint32_t* d_len,
                                     uint32_t n_msgs, int32_t* d_result, void* stream)
{
    if (n_msgs == 0) return BPMD_R_OK;
    if (!d_data || !d_off || !d_len || !d_result) return BPMD_R_INVALID_ARGUMENT;
    int r = bpmd_init();
    if (r) return r;
    return bpmd_internal_utf8(d_data, d_off, d_len, n_msgs, d_result, nullptr, 0, (hipStream_t)stream)
               ? BPMD_R_HIP_ERROR
               : BPMD_R_OK;
}

extern "C" int bpmd_read_batch(const bpmd_cfg* cfg, const uint8_t* d_in, const uint64_t* d_in_off,
                               const uint32_t* d_in_len, const uint32_t* d_key, const uint8_t* d_text,
                               uint32_t n_msgs, uint8_t* d_out, const uint64_t* d_out_off,
                               const uint32_t* d_out_cap, uint32_t* d_out_len, int32_t* d_status, void* stream)
{
    int r = inflate_impl(cfg, d_in, d_in_off, d_in_len, n_msgs, d_out, d_out_off, d_out_cap, d_out_len, d_status,
                         d_key, nullptr, stream);
    if (r || n_msgs == 0 || !d_text) return r;
    // read.hpp:1372-1384: text whose inflated bytes are not UTF-8 fails with bad_frame_payload
    return bpmd_internal_utf8(d_out, d_out_off, d_out_len, n_msgs, d_status, d_text, BPMD_BAD_FRAME_PAYLOAD,
                              (hipStream_t)stream)
               ? BPMD_R_HIP_ERROR
               : BPMD_R_OK;
}

extern "C" int bpmd_write_batch(const bpmd_cfg* cfg, const uint8_t* d_in, const uint64_t* d_in_off,
                                const uint32_t* d_in_len, const uint32_t* d_key, uint32_t n_msgs, uint8_t* d_out,
                                const uint64_t* d_out_off, const uint32_t* d_out_cap, uint32_t* d_out_len,
                                int32_t* d_status, void* stream)
{
    return deflate_impl(cfg, d_in, d_in_off, d_in_len, n_msgs, d_out, d_out_off, d_out_cap, d_out_len, d_status,
                        d_key, nullptr, stream);
}

// ---------------------------------------------- context takeover (§8(f) N3)

extern "C" int bpmd_inflate_takeover_batch(const bpmd_cfg* cfg, const uint8_t* d_in, const uint64_t* d_in_off,
                                           const uint32_t* d_in_len, const uint32_t* d_hist_len, uint32_t n_msgs,
                                           uint8_t* d_out, const uint64_t* d_out_off, const uint32_t* d_out_cap,
                                           uint32_t* d_out_len, int32_t* d_status, void* stream)
{
    if (n_msgs && !d_hist_len) return BPMD_R_INVALID_ARGUMENT;
    return inflate_impl(cfg, d_in, d_in_off, d_in_len, n_msgs, d_out, d_out_off, d_out_cap, d_out_len, d_status,
                        nullptr, d_hist_len, stream);
}

extern "C" int bpmd_deflate_takeover_batch(const bpmd_cfg* cfg, const uint8_t* d_in, const uint64_t* d_in_off,
                                           const uint32_t* d_in_len, const uint32_t* d_hist_len, uint32_t n_msgs,
                                           uint8_t* d_out, const uint64_t* d_out_off, const uint32_t* d_out_cap,
                                           uint32_t* d_out_len, int32_t* d_status, void* stream)
{
    if (n_msgs && !d_hist_len) return BPMD_R_INVALID_ARGUMENT;
    return deflate_impl(cfg, d_in, d_in_off, d_in_len, n_msgs, d_out, d_out_off, d_out_cap, d_out_len, d_status,
                        nullptr, d_hist_len, stream);
}

extern "C" int bpmd_slide_batch(uint8_t* d_buf, const uint64_t* d_base, const uint32_t* d_pos, const uint32_t* d_keep,
                                uint32_t n, void* stream)
{
    if (n == 0) return BPMD_R_OK;
    if (!d_buf || !d_base || !d_pos || !d_keep) return BPMD_R_INVALID_ARGUMENT;
    int r = bpmd_init();
    if (r) return r;
    return bpmd_internal_slide(d_buf, d_base, d_pos, d_keep, n, (hipStream_t)stream) ? BPMD_R_HIP_ERROR : BPMD_R_OK;
}
