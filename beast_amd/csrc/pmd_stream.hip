// pmd_stream.hip -- per-stream entry points behind the C++ compatibility
// facade (include/beast_amd/zlib.hpp, include/boost/beast/zlib/*.hpp):
// zlib::deflate_stream / zlib::inflate_stream write() semantics, executed by
// the GPU kernels.  Host code only.
//
// deflate: input is buffered until a flush; each flush compresses the
//   buffered bytes on the GPU (blocks with BFINAL = 0, exact bit length
//   returned by the kernel) and appends the flush's own bits the way the
//   reference's doWrite does (deflate_stream.ipp:357-499): Flush::block
//   leaves the last partial byte pending, partial adds tr_align's empty
//   static block, sync/full add the empty stored block 000 + pad +
//   00 00 FF FF, finish adds a final empty block and reports end_of_stream.
//   Pending output, duplicate-flush need_buffers, stream_error and
//   invalid_argument follow doWrite.
// inflate: the reference's decoder state lives on the device (zstream.h) and
//   each write() is one launch of the per-stream kernel (pmd_zstream.hip),
//   which runs inflate_stream.ipp's state machine with its bit reservoir and
//   window: the call uploads the caller's input, the kernel decodes exactly
//   what the reference would, and the host copies the output back and
//   advances z_params by the kernel's done() record -- the reference's
//   total_in (input left unconsumed stays with the caller), total_out and
//   data_type; an error returns without advancing them, as err() does.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <new>
#include <vector>

#include "../../include/beast_pmd.h"
#include "lz_core.h"
#include "zstream.h"

extern "C" int bpmd_internal_zstream_write(void* st, const uint8_t* in, uint64_t n_in, uint8_t* out, uint64_t cap,
                                           int flush, void* res, hipStream_t stream);
extern "C" void bpmd_internal_scratch_release(hipStream_t stream);
extern "C" int bpmd_internal_deflate_bits_hist(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                                               uint32_t n, uint8_t* out, const uint64_t* out_off,
                                               const uint32_t* out_cap, uint32_t* out_len, int32_t* status,
                                               uint32_t* out_bits, const uint32_t* hist_len, int level,
                                               int window_bits, int strategy, const int* tune, hipStream_t stream,
                                               int64_t host_chunks);
extern "C" int bpmd_internal_zstream_write_batch(const void* calls, uint32_t n, hipStream_t stream);

struct bpmd_stream {
    bool is_deflate = true;
    // deflate parameters
    int level = 6, wbits = 15, mem_level = 9, strategy = 0;
    // inflate: windowBits, device state (zstream.h State + Result), call buffers
    int inf_wbits = 15;
    void* zst = nullptr;
    bool zreset = true;         // a reset() to apply before the next write()
    uint8_t* din = nullptr;
    size_t din_cap = 0;
    uint8_t* dout = nullptr;
    size_t dout_cap = 0;
    // deflate: buffered message bytes; the plaintext already compressed since
    // the last reset (its last BPMD_CHUNK_HIST bytes: the history the next
    // flush's matches may reach into, as Beast's window does across flushes
    // and, under context takeover, across messages)
    std::vector<uint8_t> in;
    std::vector<uint8_t> hist;
    // deflate: output not yet handed out, plus < 8 pending bits
    std::vector<uint8_t> pend;
    size_t pend_pos = 0;
    uint32_t bits = 0;
    unsigned nbits = 0;
    int last_flush = -1;        // boost::none
    bool finished = false;      // finish_state
    bool inited = false;        // inited_ (deflate_stream.hpp:252): set by the first write after a reset
    bool tuned = false;         // tune() values in force (until reset / a level change)
    int tune4[4] = {0, 0, 0, 0};
    // device scratch
    hipStream_t hs = nullptr;
    uint8_t* dmem = nullptr;
    size_t dcap = 0;
    // pinned host staging for the call's copies (a copy from pageable memory
    // is staged by the runtime and waits; from pinned memory it is one DMA)
    uint8_t* hpin = nullptr;
    size_t hpin_cap = 0;
};

namespace {

// the stream's pinned staging buffer, at least `need` bytes
uint8_t* pinned(bpmd_stream* s, size_t need)
{
    if (need <= s->hpin_cap) return s->hpin;
    if (s->hpin) (void)hipHostFree(s->hpin);
    s->hpin = nullptr;
    s->hpin_cap = 0;
    const size_t c = std::max<size_t>(need + need / 2, 1 << 16);
    if (hipHostMalloc((void**)&s->hpin, c, hipHostMallocDefault) != hipSuccess) {
        s->hpin = nullptr;
        return nullptr;
    }
    s->hpin_cap = c;
    return s->hpin;
}

int ensure_device(bpmd_stream* s, size_t need)
{
    if (!s->hs && hipStreamCreateWithFlags(&s->hs, hipStreamNonBlocking) != hipSuccess) return BPMD_R_HIP_ERROR;
    if (need <= s->dcap) return BPMD_R_OK;
    if (s->dmem) (void)hipFree(s->dmem);
    s->dmem = nullptr;
    s->dcap = 0;
    size_t cap = std::max<size_t>(need, 1 << 16);
    if (hipMalloc(&s->dmem, cap) != hipSuccess) return BPMD_R_HIP_ERROR;
    s->dcap = cap;
    return BPMD_R_OK;
}

struct Meta {
    uint64_t in_off, out_off;
    uint32_t in_len, out_cap, out_len, bits;
    int32_t status;
    uint32_t hist_len;
    uint32_t pad[5];
};
static_assert(sizeof(Meta) == 64, "meta block");

// one flush's bytes through the deflate kernels with the stream's history in
// front of them; returns 0 or a negative bpmd_result.  Device block:
// [meta 64 B][output][history + input]; the host stages meta and input in
// pinned memory, so the call is two H2D copies, the kernels (the chunk count
// is known here, so the deflater reads nothing back), one D2H of meta and
// output together and one wait.
int run_one(bpmd_stream* s, const uint8_t* in, size_t n, size_t out_cap, std::vector<uint8_t>& out, int32_t& status,
            uint32_t& bits)
{
    const size_t hn = s->hist.size();
    if (n + hn > 0xFFFFFFFFu || out_cap > 0xFFFFFFFFu) return BPMD_R_INVALID_ARGUMENT;
    int r = bpmd_init();
    if (r) return r;
    const size_t out_at = 64, in_at = (out_at + out_cap + 15) & ~size_t(15), total = in_at + hn + n;
    if ((r = ensure_device(s, total + 16)) != 0) return r;
    uint8_t* h = pinned(s, total + 16);
    if (!h) return BPMD_R_HIP_ERROR;
    Meta m{};
    m.in_off = hn;
    m.out_off = 0;
    m.in_len = (uint32_t)n;
    m.out_cap = (uint32_t)out_cap;
    m.hist_len = (uint32_t)hn;
    std::memcpy(h, &m, sizeof m);
    if (hn) std::memcpy(h + in_at, s->hist.data(), hn);
    if (n) std::memcpy(h + in_at + hn, in, n);
    uint8_t* d = s->dmem;
    // after the first copy from the pinned buffer is queued, every error
    // return first waits for the stream: the next call refills (or frees)
    // that buffer while the DMA could still read it
    auto fail = [&]() {
        (void)hipStreamSynchronize(s->hs);
        return BPMD_R_HIP_ERROR;
    };
    if (hipMemcpyAsync(d, h, sizeof m, hipMemcpyHostToDevice, s->hs) != hipSuccess) return fail();
    if (hn + n && hipMemcpyAsync(d + in_at, h + in_at, hn + n, hipMemcpyHostToDevice, s->hs) != hipSuccess)
        return fail();
    Meta* dm = (Meta*)d;
    // chunks of the chunk-parallel path: every chunk with a history window,
    // else only messages over one chunk (pmd_deflate.hip chunk_count)
    const int64_t chunks = hn ? (int64_t)((n + 4095) / 4096) : (n > 4096 ? (int64_t)((n + 4095) / 4096) : 0);
    const int e = bpmd_internal_deflate_bits_hist(d + in_at, &dm->in_off, &dm->in_len, 1, d + out_at, &dm->out_off,
                                                  &dm->out_cap, &dm->out_len, &dm->status, &dm->bits,
                                                  hn ? &dm->hist_len : nullptr, s->level, s->wbits, s->strategy,
                                                  s->tuned ? s->tune4 : nullptr, s->hs, chunks);
    if (e) return fail();
    if (hipMemcpyAsync(h, d, out_at + out_cap, hipMemcpyDeviceToHost, s->hs) != hipSuccess) return fail();
    if (hipStreamSynchronize(s->hs) != hipSuccess) return BPMD_R_HIP_ERROR;
    std::memcpy(&m, h, sizeof m);
    if (m.out_len > out_cap) return BPMD_R_HIP_ERROR;
    out.assign(h + out_at, h + out_at + m.out_len);
    status = m.status;
    bits = m.bits;
    return BPMD_R_OK;
}

// the flushed bytes become history; only the last lz::chunk_hist(level) are
// used (kept: the most any level uses)
void add_history(bpmd_stream* s, const uint8_t* p, size_t n)
{
    constexpr size_t keep = lz::CHUNK_HIST_DEEP > BPMD_CHUNK_HIST ? lz::CHUNK_HIST_DEEP : BPMD_CHUNK_HIST;
    if (n >= keep) {
        s->hist.assign(p + n - keep, p + n);
        return;
    }
    s->hist.insert(s->hist.end(), p, p + n);
    if (s->hist.size() > keep) s->hist.erase(s->hist.begin(), s->hist.end() - (ptrdiff_t)keep);
}

// ------------------------------------------------------------ deflate bits

void put_bits(bpmd_stream* s, uint32_t v, unsigned n)
{
    s->bits |= v << s->nbits;
    s->nbits += n;
    while (s->nbits >= 8) {
        s->pend.push_back((uint8_t)s->bits);
        s->bits >>= 8;
        s->nbits -= 8;
    }
}

// append `nb` bits of the little-endian bit string p
void put_bitstring(bpmd_stream* s, const uint8_t* p, uint64_t nb)
{
    uint64_t i = 0;
    if (s->nbits == 0) {
        const size_t whole = (size_t)(nb >> 3);
        s->pend.insert(s->pend.end(), p, p + whole);
        i = (uint64_t)whole * 8;
    }
    for (; i + 8 <= nb; i += 8) put_bits(s, p[i >> 3], 8);
    if (i < nb) put_bits(s, p[i >> 3] & ((1u << (nb - i)) - 1), (unsigned)(nb - i));
}

void align_bits(bpmd_stream* s)
{
    if (s->nbits) put_bits(s, 0, 8 - s->nbits);
}

void drain(bpmd_stream* s, bpmd_zparams* zs)
{
    const size_t avail = s->pend.size() - s->pend_pos;
    const size_t k = std::min(avail, zs->avail_out);
    if (k) {
        std::memcpy(zs->next_out, s->pend.data() + s->pend_pos, k);
        zs->next_out = (uint8_t*)zs->next_out + k;
        zs->avail_out -= k;
        zs->total_out += k;
        s->pend_pos += k;
    }
    if (s->pend_pos == s->pend.size()) {
        s->pend.clear();
        s->pend_pos = 0;
    }
}

bool has_pending(const bpmd_stream* s) { return s->pend_pos < s->pend.size(); }

void reset_deflate(bpmd_stream* s)
{
    s->in.clear();
    s->hist.clear();
    s->pend.clear();
    s->pend_pos = 0;
    s->bits = 0;
    s->nbits = 0;
    s->last_flush = -1;
    s->finished = false;
    s->inited = false;   // the next write's init() -> lm_init() restores the level's table row
    s->tuned = false;
}

// one flush's compression: through the micro-batcher when it is on (below)
int run_flush(bpmd_stream* s, size_t out_cap, std::vector<uint8_t>& out, int32_t& status, uint32_t& bits);

}  // namespace

extern "C" int bpmd_deflate_stream_create(int level, int window_bits, int mem_level, int strategy,
                                          bpmd_stream** out)
{
    if (!out) return BPMD_R_INVALID_ARGUMENT;
    *out = nullptr;
    // deflate_stream.ipp:235-253
    if (level == -1) level = 6;
    if (window_bits == 8) window_bits = 9;
    if (level < 0 || level > 9 || window_bits < 8 || window_bits > 15 || mem_level < 1 || mem_level > 9 ||
        strategy < BPMD_STRATEGY_NORMAL || strategy > BPMD_STRATEGY_FIXED)
        return BPMD_R_INVALID_ARGUMENT;
    bpmd_stream* s = new (std::nothrow) bpmd_stream();
    if (!s) return BPMD_R_INVALID_ARGUMENT;
    s->is_deflate = true;
    s->level = level;
    s->wbits = window_bits;
    s->mem_level = mem_level;
    s->strategy = strategy;
    *out = s;
    return BPMD_R_OK;
}

extern "C" int bpmd_deflate_stream_reset(bpmd_stream* s)
{
    if (!s || !s->is_deflate) return BPMD_R_INVALID_ARGUMENT;
    reset_deflate(s);
    return BPMD_R_OK;
}

extern "C" int bpmd_deflate_stream_write(bpmd_stream* s, bpmd_zparams* zs, int flush)
{
    if (!s || !s->is_deflate || !zs || flush < BPMD_FLUSH_NONE || flush > BPMD_FLUSH_TREES)
        return BPMD_R_INVALID_ARGUMENT;
    if (!zs->next_in && zs->avail_in) return BPMD_R_INVALID_ARGUMENT;   // throws invalid_argument
    if (!zs->next_out || (s->finished && flush != BPMD_FLUSH_FINISH)) return BPMD_STREAM_ERROR;
    if (zs->avail_out == 0) return BPMD_NEED_BUFFERS;
    s->inited = true;   // maybe_init() (deflate_stream.ipp:361)
    const int old = s->last_flush;
    s->last_flush = flush;
    if (has_pending(s)) {
        drain(s, zs);
        if (zs->avail_out == 0) {
            s->last_flush = -1;
            return BPMD_OK;
        }
    } else if (zs->avail_in == 0 && old >= 0 && flush <= old && flush != BPMD_FLUSH_FINISH) {
        return BPMD_NEED_BUFFERS;
    }
    if (s->finished && zs->avail_in) return BPMD_NEED_BUFFERS;
    if (zs->avail_in) {
        const uint8_t* p = (const uint8_t*)zs->next_in;
        s->in.insert(s->in.end(), p, p + zs->avail_in);
        zs->next_in = p + zs->avail_in;
        zs->total_in += zs->avail_in;
        zs->avail_in = 0;
    }
    if (flush != BPMD_FLUSH_NONE && !s->finished) {
        if (!s->in.empty()) {
            std::vector<uint8_t> out;
            int32_t st = 0;
            uint32_t nb = 0;
            const size_t cap = bpmd_deflate_upper_bound(s->in.size()) + 16;
            int r = run_flush(s, cap, out, st, nb);
            if (r) return r;
            if (st != BPMD_OK) return BPMD_STREAM_ERROR;
            put_bitstring(s, out.data(), nb);
            add_history(s, s->in.data(), s->in.size());
            s->in.clear();
        }
        switch (flush) {
        case BPMD_FLUSH_PARTIAL:     // tr_align: empty static block
            put_bits(s, 1u << 1, 3);
            put_bits(s, 0, 7);
            break;
        case BPMD_FLUSH_SYNC:
        case BPMD_FLUSH_FULL:        // tr_stored_block(nullptr, 0): 000, pad, 00 00 FF FF
            put_bits(s, 0, 3);
            align_bits(s);
            put_bits(s, 0x0000, 16);
            put_bits(s, 0xFFFF, 16);
            break;
        case BPMD_FLUSH_FINISH:      // last block: empty fixed block with BFINAL = 1
            put_bits(s, 1u | (1u << 1), 3);
            put_bits(s, 0, 7);
            align_bits(s);
            s->finished = true;
            break;
        default:                     // block / trees: the block is complete, bits stay pending
            break;
        }
        drain(s, zs);
        if (zs->avail_out == 0) s->last_flush = -1;
    }
    if (flush == BPMD_FLUSH_FINISH) return has_pending(s) ? BPMD_OK : BPMD_END_OF_STREAM;
    return BPMD_OK;
}

extern "C" int bpmd_deflate_stream_params(bpmd_stream* s, bpmd_zparams* zs, int level, int strategy)
{
    // deflate_stream::params (deflate_stream.ipp:307-338): buffered input is
    // compressed with the old parameters first, as a Flush::block
    if (!s || !s->is_deflate || !zs) return BPMD_R_INVALID_ARGUMENT;
    if (level == -1) level = 6;
    if (level < 0 || level > 9 || strategy < BPMD_STRATEGY_NORMAL || strategy > BPMD_STRATEGY_FIXED)
        return BPMD_STREAM_ERROR;
    int r = BPMD_OK;
    if (!s->in.empty() && (level != s->level || strategy != s->strategy)) {
        r = bpmd_deflate_stream_write(s, zs, BPMD_FLUSH_BLOCK);
        if (r == BPMD_NEED_BUFFERS) r = BPMD_OK;
    }
    if (r == BPMD_OK) {
        if (level != s->level) s->tuned = false;   // doParams reloads the level's table row
        s->level = level;
        s->strategy = strategy;
    }
    return r;
}

extern "C" int bpmd_deflate_stream_tune(bpmd_stream* s, int good_length, int max_lazy, int nice_length, int max_chain)
{
    // deflate_stream::tune (deflate_stream.hpp:163-181, deflate_stream.ipp:307-317).
    // Before the stream's first write the values are overwritten by the lazy
    // init()'s lm_init() (deflate_stream.ipp:688, 697-710), so they only take
    // effect on an initialised stream, until the next reset.
    if (!s || !s->is_deflate) return BPMD_R_INVALID_ARGUMENT;
    if (!s->inited) return BPMD_R_OK;
    s->tune4[0] = good_length;
    s->tune4[1] = max_lazy;
    s->tune4[2] = nice_length;
    s->tune4[3] = max_chain;
    s->tuned = true;
    return BPMD_R_OK;
}

extern "C" int bpmd_deflate_stream_pending(bpmd_stream* s, unsigned* value, int* bits)
{
    // deflate_stream::pending (deflate_stream.hpp:344-348)
    if (!s || !s->is_deflate) return BPMD_R_INVALID_ARGUMENT;
    if (value) *value = (unsigned)(s->pend.size() - s->pend_pos);
    if (bits) *bits = (int)s->nbits;
    return BPMD_OK;
}

extern "C" int bpmd_deflate_stream_prime(bpmd_stream* s, int bits, int value)
{
    // deflate_stream::prime (deflate_stream.ipp:340-355): insert up to 16 bits
    if (!s || !s->is_deflate) return BPMD_R_INVALID_ARGUMENT;
    if (bits < 0 || bits > 16) return BPMD_NEED_BUFFERS;
    if (bits) put_bits(s, (uint32_t)value & ((1u << bits) - 1u), (unsigned)bits);
    return BPMD_OK;
}

extern "C" int bpmd_inflate_stream_create(int window_bits, bpmd_stream** out)
{
    if (!out) return BPMD_R_INVALID_ARGUMENT;
    *out = nullptr;
    if (window_bits < 8 || window_bits > 15) return BPMD_R_DOMAIN_ERROR;   // inflate_stream.ipp:57-61
    bpmd_stream* s = new (std::nothrow) bpmd_stream();
    if (!s) return BPMD_R_INVALID_ARGUMENT;
    s->is_deflate = false;
    s->inf_wbits = window_bits;
    *out = s;
    return BPMD_R_OK;
}

namespace {

using bpmd::zst::Head;
using bpmd::zst::Result;
using bpmd::zst::State;

// inflate_stream::doReset (inflate_stream.ipp:55-72): HEAD, empty reservoir,
// empty window of 2^windowBits
Head fresh_head(int window_bits)
{
    Head h{};
    h.mode = bpmd::zst::HEAD;
    h.wbits = (uint32_t)window_bits;
    return h;
}

// the stream's device state (reset if a reset() is pending)
int ensure_zhead(bpmd_stream* s)
{
    if (!s->zst) {
        if (hipMalloc(&s->zst, sizeof(State) + sizeof(Result)) != hipSuccess) {
            s->zst = nullptr;
            return BPMD_R_HIP_ERROR;
        }
        s->zreset = true;
    }
    if (s->zreset) {
        const Head h = fresh_head(s->inf_wbits);
        if (hipMemcpy(s->zst, &h, sizeof h, hipMemcpyHostToDevice) != hipSuccess) return BPMD_R_HIP_ERROR;
        s->zreset = false;
    }
    return BPMD_R_OK;
}

// ... and the single-call path's stream and input / output buffers
int ensure_zbuf(bpmd_stream* s, size_t n_in, size_t cap)
{
    if (!s->hs && hipStreamCreateWithFlags(&s->hs, hipStreamNonBlocking) != hipSuccess) return BPMD_R_HIP_ERROR;
    // input and output buffers, with slack for the 16-byte input staging loads
    if (n_in + 64 > s->din_cap) {
        if (s->din) (void)hipFree(s->din);
        s->din = nullptr;
        s->din_cap = 0;
        const size_t c = std::max<size_t>(n_in + n_in / 2 + 64, 4096);
        if (hipMalloc(&s->din, c) != hipSuccess) return BPMD_R_HIP_ERROR;
        s->din_cap = c;
    }
    if (cap + 128 > s->dout_cap) {   // [result 64 B][output]
        if (s->dout) (void)hipFree(s->dout);
        s->dout = nullptr;
        s->dout_cap = 0;
        const size_t c = std::max<size_t>(cap + cap / 2 + 128, 4096);
        if (hipMalloc(&s->dout, c) != hipSuccess) return BPMD_R_HIP_ERROR;
        s->dout_cap = c;
    }
    return BPMD_R_OK;
}

// one write() on the stream's own HIP stream: the input is uploaded, the
// kernel runs, and the result record and output come back (the output
// lands in the caller's buffer whether or not done() publishes it)
int inflate_one(bpmd_stream* s, const uint8_t* in, size_t n, uint8_t* out, size_t cap, int flush, Result& res)
{
    int r = ensure_zbuf(s, n, cap);
    if (r) return r;
    const hipStream_t hs = s->hs;
    // the result record and the output share one device block, so one D2H
    // brings both back when the output is at most `spec` bytes (pinned
    // staging for both directions: each copy is one DMA)
    constexpr size_t RES_AT = 64;
    const size_t spec = std::min<size_t>(cap, 16384);
    uint8_t* h = pinned(s, std::max(n, RES_AT + spec) + 64);
    if (!h) return BPMD_R_HIP_ERROR;
    if (n) std::memcpy(h, in, n);
    bool ok = (n == 0 || hipMemcpyAsync(s->din, h, n, hipMemcpyHostToDevice, hs) == hipSuccess) &&
              bpmd_internal_zstream_write(s->zst, s->din, n, s->dout + RES_AT, cap, flush, s->dout, hs) == 0 &&
              hipMemcpyAsync(h, s->dout, RES_AT + spec, hipMemcpyDeviceToHost, hs) == hipSuccess &&
              hipStreamSynchronize(hs) == hipSuccess;
    if (ok) std::memcpy(&res, h, sizeof res);
    ok = ok && res.out_used <= cap;
    if (ok && res.out_used) {
        std::memcpy(out, h + RES_AT, std::min<size_t>(res.out_used, spec));
        if (res.out_used > spec)
            ok = hipMemcpy(out + spec, s->dout + RES_AT + spec, res.out_used - spec, hipMemcpyDeviceToHost) ==
                 hipSuccess;
    }
    if (!ok) {
        // the pinned staging buffer may still be a DMA's source or target
        (void)hipStreamSynchronize(hs);
        return BPMD_R_HIP_ERROR;   // the device state is unchanged only if the kernel never ran
    }
    return BPMD_R_OK;
}

}  // namespace

// ------------------------------------------------------------ micro-batcher
// write() calls of different streams made at the same time
// -- a server's connections, each reading and writing on its own thread or
// strand (impl_base.hpp:85-190 inflate / deflate calls, write.hpp:463-545)
// -- run as one launch.  A call queues itself; if no batch is running it
// becomes the leader: it takes up to max_calls queued calls (one per stream),
// runs them together and wakes their callers.  Calls that arrive while a
// batch runs form the next one (a group commit: no added latency when a
// stream is alone -- its batch is one call), and
// max_delay_us > 0 lets a leader wait that long for more.  Every call's
// result is its single-call result: the inflate launch runs the same
// per-stream state machine for each stream (one workgroup per call,
// pmd_zstream.hip), the deflate launch the same per-message kernels, whose
// bytes do not depend on the batch's other messages.
namespace {

struct Job {
    bpmd_stream* s = nullptr;
    // inflate: the caller's input and output room
    const uint8_t* in = nullptr;
    size_t n = 0;
    uint8_t* out = nullptr;
    size_t cap = 0;
    int flush = 0;
    Result res{};
    // deflate: the stream's buffered input (s->in) and where its output goes
    size_t out_cap = 0;
    std::vector<uint8_t>* dout = nullptr;
    int32_t status = 0;
    uint32_t bits = 0;
    int rc = 0;
    bool done = false;
};

// a leader's device block, its pinned mirror and the HIP stream they use
struct Arena {
    hipStream_t hs = nullptr;
    uint8_t* d = nullptr;
    uint8_t* h = nullptr;
    size_t cap = 0;
    bool reserve(size_t need)
    {
        if (!hs && hipStreamCreateWithFlags(&hs, hipStreamNonBlocking) != hipSuccess) {
            hs = nullptr;
            return false;
        }
        if (need <= cap) return true;
        if (d) (void)hipFree(d);
        if (h) (void)hipHostFree(h);
        d = h = nullptr;
        cap = 0;
        const size_t c = std::max<size_t>(need + need / 2, 1 << 20);
        if (hipMalloc((void**)&d, c) != hipSuccess) {
            d = nullptr;
            return false;
        }
        if (hipHostMalloc((void**)&h, c, hipHostMallocDefault) != hipSuccess) {
            (void)hipFree(d);
            d = h = nullptr;
            return false;
        }
        cap = c;
        return true;
    }
};

// settings: max_calls < 2 is off
std::atomic<int> g_bmax{-1}, g_bdelay{-1};
// [0] inflate calls, [1] inflate launches, [2] deflate flushes, [3] deflate launches
std::atomic<unsigned long long> g_bstat[4];

int batch_max()
{
    int m = g_bmax.load();
    if (m < 0) {
        const char* e = getenv("BPMD_STREAM_BATCH");
        m = e ? std::max(0, std::min(atoi(e), 4096)) : 256;
        const char* d = getenv("BPMD_STREAM_BATCH_DELAY_US");
        g_bdelay.store(d ? std::max(0, atoi(d)) : 0);
        g_bmax.store(m);
    }
    return m;
}

class Coalescer {
  public:
    explicit Coalescer(int dev) : dev_(dev) {}
    template <class Exec>
    void run(Job* j, int max_calls, Exec&& exec)
    {
        std::unique_lock<std::mutex> lk(mu_);
        q_.push_back(j);
        if (busy_) arrive_.notify_one();
        while (!j->done) {
            if (busy_) {
                done_.wait(lk);
                continue;
            }
            busy_ = true;
            const int delay = g_bdelay.load();
            if (delay > 0 && q_.size() < (size_t)max_calls)
                arrive_.wait_for(lk, std::chrono::microseconds(delay), [&] { return q_.size() >= (size_t)max_calls; });
            // in arrival order, one call per stream (a stream's calls are
            // its owner's sequence: a second one waits for the next batch)
            std::vector<Job*> take;
            for (auto it = q_.begin(); it != q_.end() && take.size() < (size_t)max_calls;) {
                bool dup = false;
                for (const Job* t : take) dup = dup || t->s == (*it)->s;
                if (dup) {
                    ++it;
                    continue;
                }
                take.push_back(*it);
                it = q_.erase(it);
            }
            lk.unlock();
            // the coalescer's device (its streams' state lives there), whatever
            // this thread had current
            int prev = -1;
            (void)hipGetDevice(&prev);
            if (prev != dev_) (void)hipSetDevice(dev_);
            exec(arena_, take);
            if (prev != dev_ && prev >= 0) (void)hipSetDevice(prev);
            lk.lock();
            for (Job* t : take) t->done = true;
            busy_ = false;
            done_.notify_all();
        }
    }

  private:
    std::mutex mu_;
    std::condition_variable done_, arrive_;
    std::deque<Job*> q_;
    bool busy_ = false;
    Arena arena_;
    int dev_;
};

// one pair per device: a stream's device state lives on the device its
// owner had current, and calls only batch with calls of the same device.
// Process-lifetime objects (never destroyed: HIP may be torn down first).
constexpr int MAX_DEV = 64;
Coalescer* coalescer(int dev, bool inflate)
{
    static std::mutex mu;
    static Coalescer* tab[2][MAX_DEV] = {};
    if (dev < 0 || dev >= MAX_DEV) return nullptr;
    std::lock_guard<std::mutex> lk(mu);
    Coalescer*& c = tab[inflate ? 0 : 1][dev];
    if (!c) c = new (std::nothrow) Coalescer(dev);
    return c;
}

constexpr size_t up256(size_t x) { return (x + 255) & ~(size_t)255; }

void fail_all(std::vector<Job*>& jobs, hipStream_t hs)
{
    if (hs) (void)hipStreamSynchronize(hs);   // no DMA may still use the pinned mirror
    for (Job* j : jobs) j->rc = BPMD_R_HIP_ERROR;
}

// k inflate write() calls as one launch.  Block: [ZCall k][inputs]
// [Result k][outputs]; one H2D of calls + inputs, the launch, one D2H of the
// results and outputs (of the results alone, then each call's used output,
// when the output room is over 4 MiB).
void inflate_batch(Arena& A, std::vector<Job*>& jobs)
{
    using bpmd::zst::ZCall;
    const uint32_t k = (uint32_t)jobs.size();
    std::vector<size_t> ioff(k), ooff(k);
    size_t o = up256(sizeof(ZCall) * k);
    for (uint32_t i = 0; i < k; ++i) {
        ioff[i] = o;
        o = up256(o + jobs[i]->n + 64);   // + the staging loads' slack
    }
    const size_t res_at = o;
    o = up256(res_at + 64ull * k);
    for (uint32_t i = 0; i < k; ++i) {
        ooff[i] = o;
        o = up256(o + jobs[i]->cap);
    }
    const size_t total = o;
    if (!A.reserve(total)) return fail_all(jobs, A.hs);
    ZCall* zc = (ZCall*)A.h;
    for (uint32_t i = 0; i < k; ++i) {
        const Job* j = jobs[i];
        if (j->n) std::memcpy(A.h + ioff[i], j->in, j->n);
        ZCall c{};
        c.st = j->s->zst;
        c.in = A.d + ioff[i];
        c.n_in = j->n;
        c.out = A.d + ooff[i];
        c.cap = j->cap;
        c.res = A.d + res_at + 64ull * i;
        c.flush = j->flush;
        zc[i] = c;
    }
    const bool whole = total - res_at <= (4u << 20);
    bool ok = hipMemcpyAsync(A.d, A.h, res_at, hipMemcpyHostToDevice, A.hs) == hipSuccess &&
              bpmd_internal_zstream_write_batch(A.d, k, A.hs) == 0 &&
              hipMemcpyAsync(A.h + res_at, A.d + res_at, (whole ? total : res_at + 64ull * k) - res_at,
                             hipMemcpyDeviceToHost, A.hs) == hipSuccess &&
              hipStreamSynchronize(A.hs) == hipSuccess;
    if (!ok) return fail_all(jobs, A.hs);
    for (uint32_t i = 0; i < k && ok; ++i) {
        Job* j = jobs[i];
        std::memcpy(&j->res, A.h + res_at + 64ull * i, sizeof(Result));
        ok = j->res.out_used <= j->cap;
        if (ok && !whole && j->res.out_used)
            ok = hipMemcpyAsync(A.h + ooff[i], A.d + ooff[i], j->res.out_used, hipMemcpyDeviceToHost, A.hs) ==
                 hipSuccess;
    }
    if (ok && !whole) ok = hipStreamSynchronize(A.hs) == hipSuccess;
    if (!ok) return fail_all(jobs, A.hs);
    for (uint32_t i = 0; i < k; ++i) {
        Job* j = jobs[i];
        if (j->res.out_used) std::memcpy(j->out, A.h + ooff[i], j->res.out_used);
        j->rc = BPMD_R_OK;
    }
}

// (a batch of one too: with the batcher on, streams use the leaders'
// buffers and HIP stream and allocate none of their own -- creating a HIP
// stream or pinned buffer per connection serializes in the runtime)
void inflate_exec(Arena& A, std::vector<Job*>& jobs)
{
    g_bstat[1].fetch_add(1);
    inflate_batch(A, jobs);
}

// deflate flushes with the same parameters (level, windowBits, strategy,
// tune values, history or not) as one call of the deflater.  Block:
// [SoA meta][outputs][history + input, per flush]; H2D of meta and inputs,
// the kernels (the chunk count is known here: nothing is read back), one D2H
// of meta + outputs (meta, then each flush's output, past 4 MiB of room).
void deflate_group(Arena& A, std::vector<Job*>& jobs)
{
    const uint32_t k = (uint32_t)jobs.size();
    const bpmd_stream* s0 = jobs[0]->s;
    const bool hist = !s0->hist.empty();
    const size_t m_in_off = 0, m_out_off = 8ull * k, m_in_len = 16ull * k, m_out_cap = 20ull * k,
                 m_hist = 24ull * k, m_out_len = 28ull * k, m_bits = 32ull * k, m_status = 36ull * k;
    const size_t out_at = up256(40ull * k);
    std::vector<uint64_t> oo(k), io(k);
    size_t o = 0;
    for (uint32_t i = 0; i < k; ++i) {
        oo[i] = o;
        o = up256(o + jobs[i]->out_cap);
    }
    const size_t in_at = out_at + o;
    size_t ib = 0;
    int64_t chunks = 0;
    for (uint32_t i = 0; i < k; ++i) {
        const bpmd_stream* s = jobs[i]->s;
        const size_t hn = s->hist.size(), n = s->in.size();
        if (n + hn > 0xFFFFFFFFu || jobs[i]->out_cap > 0xFFFFFFFFu) {
            for (Job* j : jobs) j->rc = BPMD_R_INVALID_ARGUMENT;
            return;
        }
        io[i] = ib;
        ib = up256(ib + hn + n);
        // run_one's count (pmd_deflate.hip chunk_count)
        chunks += hn ? (int64_t)((n + 4095) / 4096) : (n > 4096 ? (int64_t)((n + 4095) / 4096) : 0);
    }
    const size_t total = in_at + ib + 16;
    if (!A.reserve(total)) return fail_all(jobs, A.hs);
    uint8_t* h = A.h;
    std::memset(h, 0, out_at);
    for (uint32_t i = 0; i < k; ++i) {
        const bpmd_stream* s = jobs[i]->s;
        const size_t hn = s->hist.size(), n = s->in.size();
        ((uint64_t*)(h + m_in_off))[i] = io[i] + hn;
        ((uint64_t*)(h + m_out_off))[i] = oo[i];
        ((uint32_t*)(h + m_in_len))[i] = (uint32_t)n;
        ((uint32_t*)(h + m_out_cap))[i] = (uint32_t)jobs[i]->out_cap;
        ((uint32_t*)(h + m_hist))[i] = (uint32_t)hn;
        if (hn) std::memcpy(h + in_at + io[i], s->hist.data(), hn);
        if (n) std::memcpy(h + in_at + io[i] + hn, s->in.data(), n);
    }
    uint8_t* d = A.d;
    const bool whole = in_at <= (4u << 20);
    bool ok = hipMemcpyAsync(d, h, out_at, hipMemcpyHostToDevice, A.hs) == hipSuccess &&
              (ib == 0 || hipMemcpyAsync(d + in_at, h + in_at, ib, hipMemcpyHostToDevice, A.hs) == hipSuccess) &&
              bpmd_internal_deflate_bits_hist(d + in_at, (const uint64_t*)(d + m_in_off),
                                              (const uint32_t*)(d + m_in_len), k, d + out_at,
                                              (const uint64_t*)(d + m_out_off), (const uint32_t*)(d + m_out_cap),
                                              (uint32_t*)(d + m_out_len), (int32_t*)(d + m_status),
                                              (uint32_t*)(d + m_bits), hist ? (const uint32_t*)(d + m_hist) : nullptr,
                                              s0->level, s0->wbits, s0->strategy, s0->tuned ? s0->tune4 : nullptr,
                                              A.hs, chunks) == 0 &&
              hipMemcpyAsync(h, d, whole ? in_at : out_at, hipMemcpyDeviceToHost, A.hs) == hipSuccess &&
              hipStreamSynchronize(A.hs) == hipSuccess;
    if (!ok) return fail_all(jobs, A.hs);
    for (uint32_t i = 0; i < k && ok; ++i) {
        const uint32_t len = ((const uint32_t*)(h + m_out_len))[i];
        ok = len <= jobs[i]->out_cap;
        if (ok && !whole && len)
            ok = hipMemcpyAsync(h + out_at + oo[i], d + out_at + oo[i], len, hipMemcpyDeviceToHost, A.hs) ==
                 hipSuccess;
    }
    if (ok && !whole) ok = hipStreamSynchronize(A.hs) == hipSuccess;
    if (!ok) return fail_all(jobs, A.hs);
    for (uint32_t i = 0; i < k; ++i) {
        Job* j = jobs[i];
        const uint32_t len = ((const uint32_t*)(h + m_out_len))[i];
        j->dout->assign(h + out_at + oo[i], h + out_at + oo[i] + len);
        j->status = ((const int32_t*)(h + m_status))[i];
        j->bits = ((const uint32_t*)(h + m_bits))[i];
        j->rc = BPMD_R_OK;
    }
}

bool same_params(const bpmd_stream* a, const bpmd_stream* b)
{
    return a->level == b->level && a->wbits == b->wbits && a->strategy == b->strategy && a->tuned == b->tuned &&
           (!a->tuned || std::memcmp(a->tune4, b->tune4, sizeof a->tune4) == 0) &&
           a->hist.empty() == b->hist.empty();
}

void deflate_exec(Arena& A, std::vector<Job*>& jobs)
{
    std::vector<bool> used(jobs.size(), false);
    for (size_t i = 0; i < jobs.size(); ++i) {
        if (used[i]) continue;
        std::vector<Job*> g{jobs[i]};
        for (size_t j = i + 1; j < jobs.size(); ++j)
            if (!used[j] && same_params(jobs[i]->s, jobs[j]->s)) {
                used[j] = true;
                g.push_back(jobs[j]);
            }
        g_bstat[3].fetch_add(1);
        deflate_group(A, g);   // (a group of one too, as inflate_exec)
    }
}

// the inflate write()'s call, batched or not
int inflate_call(bpmd_stream* s, const uint8_t* in, size_t n, uint8_t* out, size_t cap, int flush, Result& res)
{
    const int mx = batch_max();
    if (mx < 2) return inflate_one(s, in, n, out, cap, flush, res);
    g_bstat[0].fetch_add(1);
    Job j;
    j.s = s;
    j.in = in;
    j.n = n;
    j.out = out;
    j.cap = cap;
    j.flush = flush;
    int dev = 0;
    Coalescer* c = hipGetDevice(&dev) == hipSuccess ? coalescer(dev, true) : nullptr;
    if (!c) return inflate_one(s, in, n, out, cap, flush, res);
    c->run(&j, mx, inflate_exec);
    res = j.res;
    return j.rc;
}

int run_flush(bpmd_stream* s, size_t out_cap, std::vector<uint8_t>& out, int32_t& status, uint32_t& bits)
{
    const int mx = batch_max();
    if (mx < 2) return run_one(s, s->in.data(), s->in.size(), out_cap, out, status, bits);
    g_bstat[2].fetch_add(1);
    Job j;
    j.s = s;
    j.out_cap = out_cap;
    j.dout = &out;
    int dev = 0;
    Coalescer* c = hipGetDevice(&dev) == hipSuccess ? coalescer(dev, false) : nullptr;
    if (!c) return run_one(s, s->in.data(), s->in.size(), out_cap, out, status, bits);
    c->run(&j, mx, deflate_exec);
    status = j.status;
    bits = j.bits;
    return j.rc;
}

}  // namespace

extern "C" int bpmd_stream_batching(int max_calls, int max_delay_us)
{
    if (max_calls < 0 || max_calls > 4096 || max_delay_us < 0) return BPMD_R_INVALID_ARGUMENT;
    (void)batch_max();   // the environment's defaults read first, then replaced
    g_bdelay.store(max_delay_us);
    g_bmax.store(max_calls);
    return BPMD_R_OK;
}

extern "C" int bpmd_stream_batch_stats(unsigned long long* out, int reset)
{
    if (!out) return BPMD_R_INVALID_ARGUMENT;
    for (int i = 0; i < 4; ++i) out[i] = reset ? g_bstat[i].exchange(0) : g_bstat[i].load();
    return BPMD_R_OK;
}

extern "C" int bpmd_inflate_stream_reset(bpmd_stream* s, int window_bits)
{
    if (!s || s->is_deflate) return BPMD_R_INVALID_ARGUMENT;
    if (window_bits < 8 || window_bits > 15) return BPMD_R_DOMAIN_ERROR;
    s->inf_wbits = window_bits;
    s->zreset = true;   // applied before the next write()
    return BPMD_R_OK;
}

extern "C" int bpmd_inflate_stream_clear(bpmd_stream* s)
{
    // inflate_stream::clear -> doClear is empty in the reference
    // (inflate_stream.ipp:49-53): state and window persist
    return (!s || s->is_deflate) ? BPMD_R_INVALID_ARGUMENT : BPMD_R_OK;
}

extern "C" int bpmd_inflate_stream_write(bpmd_stream* s, bpmd_zparams* zs, int flush)
{
    if (!s || s->is_deflate || !zs || flush < BPMD_FLUSH_NONE || flush > BPMD_FLUSH_TREES)
        return BPMD_R_INVALID_ARGUMENT;
    if ((!zs->next_in && zs->avail_in) || (!zs->next_out && zs->avail_out)) return BPMD_STREAM_ERROR;
    int r = bpmd_init();
    if (r) return r;
    const size_t n = zs->avail_in;
    // Output room handed to the kernel.  A call cannot produce more than the
    // pending match (<= 258) plus 258 bytes per 2 bits of the input and the
    // reservoir (<= 32 bits), so a room of at least that plus 258 leaves the
    // reference's "avail_out >= 258" fast-path test unchanged.
    const size_t bound = 1040 * n + 8192;
    const size_t cap = std::min<size_t>(zs->avail_out, bound);
    if ((r = ensure_zhead(s)) != 0) return r;
    Result res{};
    if ((r = inflate_call(s, (const uint8_t*)zs->next_in, n, (uint8_t*)zs->next_out, cap, flush, res)) != 0) return r;
    if (res.published) {
        zs->next_in = (const uint8_t*)zs->next_in + res.in_used;
        zs->avail_in -= res.in_used;
        zs->total_in += res.in_used;
        zs->next_out = (uint8_t*)zs->next_out + res.out_used;
        zs->avail_out -= res.out_used;
        zs->total_out += res.out_used;
        zs->data_type = res.data_type;
    }
    return res.ec;
}

extern "C" int bpmd_inflate_stream_footprint(const bpmd_stream* s, size_t* host_bytes, size_t* device_bytes)
{
    if (!s || s->is_deflate) return BPMD_R_INVALID_ARGUMENT;
    if (device_bytes)
        *device_bytes = (s->zst ? sizeof(State) + sizeof(Result) : 0) + s->din_cap + s->dout_cap;
    if (host_bytes) *host_bytes = s->hpin_cap;   // pinned staging only
    return BPMD_R_OK;
}

extern "C" void bpmd_stream_destroy(bpmd_stream* s)
{
    if (!s) return;
    if (s->hs) (void)hipStreamSynchronize(s->hs);
    if (s->dmem) (void)hipFree(s->dmem);
    if (s->zst) (void)hipFree(s->zst);
    if (s->din) (void)hipFree(s->din);
    if (s->dout) (void)hipFree(s->dout);
    if (s->hpin) (void)hipHostFree(s->hpin);
    if (s->hs) {
        bpmd_internal_scratch_release(s->hs);
        (void)hipStreamDestroy(s->hs);
    }
    delete s;
}
