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
#include <cstring>
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
            int r = run_one(s, s->in.data(), s->in.size(), cap, out, st, nb);
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

// the stream's device state, its result record and call buffers
int ensure_zstate(bpmd_stream* s, size_t n_in, size_t cap)
{
    if (!s->hs && hipStreamCreateWithFlags(&s->hs, hipStreamNonBlocking) != hipSuccess) return BPMD_R_HIP_ERROR;
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

}  // namespace

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
    if ((r = ensure_zstate(s, n, cap)) != 0) return r;
    const hipStream_t hs = s->hs;
    Result res{};
    // the result record and the output share one device block, so one D2H
    // brings both back when the output is at most `spec` bytes (pinned
    // staging for both directions: each copy is one DMA)
    constexpr size_t RES_AT = 64;
    const size_t spec = std::min<size_t>(cap, 16384);
    uint8_t* h = pinned(s, std::max(n, RES_AT + spec) + 64);
    if (!h) return BPMD_R_HIP_ERROR;
    if (n) std::memcpy(h, zs->next_in, n);
    bool ok = (n == 0 || hipMemcpyAsync(s->din, h, n, hipMemcpyHostToDevice, hs) == hipSuccess) &&
              bpmd_internal_zstream_write(s->zst, s->din, n, s->dout + RES_AT, cap, flush, s->dout, hs) == 0 &&
              hipMemcpyAsync(h, s->dout, RES_AT + spec, hipMemcpyDeviceToHost, hs) == hipSuccess &&
              hipStreamSynchronize(hs) == hipSuccess;
    if (ok) std::memcpy(&res, h, sizeof res);
    // the bytes are in the caller's buffer whether or not done() publishes them
    ok = ok && res.out_used <= cap;
    if (ok && res.out_used) {
        std::memcpy(zs->next_out, h + RES_AT, std::min<size_t>(res.out_used, spec));
        if (res.out_used > spec)
            ok = hipMemcpy((uint8_t*)zs->next_out + spec, s->dout + RES_AT + spec, res.out_used - spec,
                           hipMemcpyDeviceToHost) == hipSuccess;
    }
    if (!ok) {
        // the pinned staging buffer may still be a DMA's source or target
        (void)hipStreamSynchronize(hs);
        return BPMD_R_HIP_ERROR;   // the device state is unchanged only if the kernel never ran
    }
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
