// pmd_stream.hip -- per-stream entry points behind the C++ compatibility
// facade (include/beast_amd/zlib.hpp, include/boost/beast/zlib/*.hpp):
// zlib::deflate_stream / zlib::inflate_stream write() semantics, executed by
// the GPU kernels (a batch of one).  Host code only.
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
// inflate: a resumable decoder (inflate_resume.h).  Each write() appends its
//   input to the bytes kept since the last checkpoint, resumes the wave
//   kernel there with the window (the last 2^windowBits output bytes before
//   the checkpoint) in front of the output slot, hands out the bytes past
//   those already delivered, then drops the input before the new checkpoint
//   and slides the window on the device.  Per call the GPU decodes the new
//   input plus at most one round again, and the stream holds O(window +
//   one round + the caller's buffers) whatever the connection's age.  The
//   reference's per-call rules are kept: the window check of a distance
//   depends on the call boundaries (bpmd_resume_call), BAD mode answers
//   need_buffers, DONE answers end_of_stream, Flush::block / Flush::trees stop
//   at block boundaries / after a block header.  Input is reported consumed
//   whole (the reference can leave input unconsumed when avail_out runs out
//   first; here those bytes are kept and decoded by later calls).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/beast_pmd.h"
#include "inflate_resume.h"

extern "C" int bpmd_internal_inflate_resume(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                                            uint8_t* out, const uint64_t* out_off, const uint32_t* out_cap,
                                            uint32_t* out_len, int32_t* status, bpmd_resume_call rc,
                                            hipStream_t stream);
extern "C" int bpmd_internal_deflate_bits(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                                          uint32_t n, uint8_t* out, const uint64_t* out_off, const uint32_t* out_cap,
                                          uint32_t* out_len, int32_t* status, uint32_t* out_bits, int level,
                                          int window_bits, int strategy, const int* tune, hipStream_t stream);

struct bpmd_stream {
    bool is_deflate = true;
    // deflate parameters
    int level = 6, wbits = 15, mem_level = 9, strategy = 0;
    // inflate parameters and decoder state (inflate_resume.h)
    int inf_wbits = 15;
    int inf_mode = 0;           // 0 decoding, 1 DONE (end_of_stream), 2 BAD
    bpmd_resume ck{};           // checkpoint; ck.bit counts from in[0]
    uint32_t hist = 0;          // window bytes = min(output before the checkpoint, 2^wbits)
    uint64_t in_abs = 0;        // stream offset of in[0]
    uint64_t ref_pos = 0;       // input bytes the reference would have consumed so far
    uint32_t wcur = 0;          // which device window/output buffer holds the window
    uint8_t* dwo[2] = {nullptr, nullptr};   // [2^15 window][output slot] each
    size_t dwo_cap = 0;         // output slot bytes of each
    uint8_t* dctl = nullptr;    // meta + checkpoint in/out
    uint8_t* din = nullptr;     // pending input
    size_t din_cap = 0;
    // buffered input (deflate: message bytes; inflate: compressed bytes since the checkpoint)
    std::vector<uint8_t> in;
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
    // inflate: bytes decoded past the checkpoint and already handed out
    size_t delivered = 0;
    // device scratch
    hipStream_t hs = nullptr;
    uint8_t* dmem = nullptr;
    size_t dcap = 0;
};

namespace {

// device block layout: [meta 64 B][input][output]
struct DevLayout {
    size_t in_off, out_off, total;
};

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
    uint32_t pad[6];
};
static_assert(sizeof(Meta) == 64, "meta block");

// one message through a batch kernel; returns 0 or a negative bpmd_result
int run_one(bpmd_stream* s, bool deflate, const uint8_t* in, size_t n, size_t out_cap, std::vector<uint8_t>& out,
            int32_t& status, uint32_t& bits)
{
    if (n > 0xFFFFFFFFu || out_cap > 0xFFFFFFFFu) return BPMD_R_INVALID_ARGUMENT;
    int r = bpmd_init();
    if (r) return r;
    const size_t in_at = 64, out_at = (in_at + n + 15) & ~size_t(15);
    if ((r = ensure_device(s, out_at + out_cap + 16)) != 0) return r;
    Meta m{};
    m.in_off = 0;
    m.out_off = 0;
    m.in_len = (uint32_t)n;
    m.out_cap = (uint32_t)out_cap;
    uint8_t* d = s->dmem;
    if (hipMemcpyAsync(d, &m, sizeof m, hipMemcpyHostToDevice, s->hs) != hipSuccess) return BPMD_R_HIP_ERROR;
    if (n && hipMemcpyAsync(d + in_at, in, n, hipMemcpyHostToDevice, s->hs) != hipSuccess) return BPMD_R_HIP_ERROR;
    Meta* dm = (Meta*)d;
    int e;
    (void)deflate;
    e = bpmd_internal_deflate_bits(d + in_at, &dm->in_off, &dm->in_len, 1, d + out_at, &dm->out_off, &dm->out_cap,
                                   &dm->out_len, &dm->status, &dm->bits, s->level, s->wbits, s->strategy,
                                   s->tuned ? s->tune4 : nullptr, s->hs);
    if (e) return BPMD_R_HIP_ERROR;
    if (hipMemcpyAsync(&m, d, sizeof m, hipMemcpyDeviceToHost, s->hs) != hipSuccess) return BPMD_R_HIP_ERROR;
    if (hipStreamSynchronize(s->hs) != hipSuccess) return BPMD_R_HIP_ERROR;
    out.resize(m.out_len);
    if (m.out_len && hipMemcpy(out.data(), d + out_at, m.out_len, hipMemcpyDeviceToHost) != hipSuccess)
        return BPMD_R_HIP_ERROR;
    status = m.status;
    bits = m.bits;
    return BPMD_R_OK;
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
            int r = run_one(s, true, s->in.data(), s->in.size(), cap, out, st, nb);
            if (r) return r;
            if (st != BPMD_OK) return BPMD_STREAM_ERROR;
            put_bitstring(s, out.data(), nb);
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

constexpr size_t kWinMax = size_t(1) << 15;   // window area in front of each output slot
constexpr size_t kCtlMeta = 0, kCtlIn = 512, kCtlOut = 1024, kCtlBytes = 2048;

void reset_inflate(bpmd_stream* s, int window_bits)
{
    // inflate_stream::reset (inflate_stream.ipp:55-72): fresh state, empty window
    s->inf_wbits = window_bits;
    s->inf_mode = 0;
    s->ck = bpmd_resume{};
    s->hist = 0;
    s->in_abs = 0;
    s->ref_pos = 0;
    s->delivered = 0;
    s->in.clear();
    s->in.shrink_to_fit();
}

// device buffers for one call: pending input of n bytes, output slot of cap
int ensure_inflate_device(bpmd_stream* s, size_t n, size_t cap)
{
    if (!s->hs && hipStreamCreateWithFlags(&s->hs, hipStreamNonBlocking) != hipSuccess) return BPMD_R_HIP_ERROR;
    if (!s->dctl && hipMalloc(&s->dctl, kCtlBytes) != hipSuccess) return BPMD_R_HIP_ERROR;
    if (n > s->din_cap) {
        if (s->din) (void)hipFree(s->din);
        s->din = nullptr;
        s->din_cap = 0;
        const size_t c = std::max<size_t>(n + n / 2, 4096);
        if (hipMalloc(&s->din, c + 64) != hipSuccess) return BPMD_R_HIP_ERROR;
        s->din_cap = c;
    }
    if (cap > s->dwo_cap || !s->dwo[0]) {
        // grow both; the window moves to the new current buffer
        const size_t c = std::max<size_t>(cap + cap / 2, 1 << 16);
        uint8_t* nb[2] = {nullptr, nullptr};
        for (int k = 0; k < 2; ++k)
            if (hipMalloc(&nb[k], kWinMax + c + 64) != hipSuccess) {
                if (nb[0]) (void)hipFree(nb[0]);
                return BPMD_R_HIP_ERROR;
            }
        if (s->hist && s->dwo[s->wcur] &&
            hipMemcpyAsync(nb[0] + kWinMax - s->hist, s->dwo[s->wcur] + kWinMax - s->hist, s->hist,
                           hipMemcpyDeviceToDevice, s->hs) != hipSuccess)
            return BPMD_R_HIP_ERROR;
        if (hipStreamSynchronize(s->hs) != hipSuccess) return BPMD_R_HIP_ERROR;
        for (int k = 0; k < 2; ++k)
            if (s->dwo[k]) (void)hipFree(s->dwo[k]);
        s->dwo[0] = nb[0];
        s->dwo[1] = nb[1];
        s->wcur = 0;
        s->dwo_cap = c;
    }
    return BPMD_R_OK;
}

struct InfMeta {
    uint64_t in_off, out_off;
    uint32_t in_len, out_cap, out_len;
    int32_t status;
};

}  // namespace

extern "C" int bpmd_inflate_stream_reset(bpmd_stream* s, int window_bits)
{
    if (!s || s->is_deflate) return BPMD_R_INVALID_ARGUMENT;
    if (window_bits < 8 || window_bits > 15) return BPMD_R_DOMAIN_ERROR;
    reset_inflate(s, window_bits);
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
    zs->data_type = 2;   // unknown until a call decodes
    // DONE: end_of_stream without touching the buffers; BAD: no progress
    // (inflate_stream.ipp:516-529, done() at :88-119)
    if (s->inf_mode == 1) return BPMD_END_OF_STREAM;
    if (s->inf_mode == 2) return BPMD_NEED_BUFFERS;
    int r = bpmd_init();
    if (r) return r;
    const size_t n_in = zs->avail_in;
    const size_t kept = s->in.size();
    if (n_in) {
        const uint8_t* p = (const uint8_t*)zs->next_in;
        s->in.insert(s->in.end(), p, p + n_in);
    }
    const size_t n = s->in.size();
    const uint32_t W = 1u << s->inf_wbits;
    // output slot: what is re-decoded (delivered) plus this call's room, which
    // the pending input could not exceed anyway (<= 258 bytes per 2 bits)
    const size_t room = std::min<size_t>(zs->avail_out, 1040 * n + 1024);
    const size_t cap = s->delivered + room;
    if (n > 0xFFFFFFF0u || cap > 0xFFFFFFF0u) {
        s->in.resize(kept);
        return BPMD_R_INVALID_ARGUMENT;
    }
    size_t fresh = 0;
    int32_t st = BPMD_OK;
    bpmd_resume out_ck{};
    const uint64_t ref_before = s->ref_pos;
    if (n == 0) {
        st = BPMD_NEED_BUFFERS;   // nothing to decode (raw mode, no input)
        out_ck = s->ck;
    } else {
        if ((r = ensure_inflate_device(s, n, cap)) != 0) {
            s->in.resize(kept);
            return r;
        }
        uint8_t* wo = s->dwo[s->wcur];
        InfMeta m{};
        m.in_off = 0;
        m.out_off = kWinMax;
        m.in_len = (uint32_t)n;
        m.out_cap = (uint32_t)cap;
        const hipStream_t hs = s->hs;
        bool ok = hipMemcpyAsync(s->dctl + kCtlMeta, &m, sizeof m, hipMemcpyHostToDevice, hs) == hipSuccess &&
                  hipMemcpyAsync(s->dctl + kCtlIn, &s->ck, sizeof s->ck, hipMemcpyHostToDevice, hs) == hipSuccess &&
                  hipMemcpyAsync(s->din, s->in.data(), n, hipMemcpyHostToDevice, hs) == hipSuccess;
        bpmd_resume_call rc;
        rc.rin = (const bpmd_resume*)(s->dctl + kCtlIn);
        rc.rout = (bpmd_resume*)(s->dctl + kCtlOut);
        rc.hist = s->hist;
        rc.D = (uint32_t)s->delivered;
        rc.cw = (uint32_t)std::min<size_t>(s->hist + s->delivered, W);
        rc.flush = flush == BPMD_FLUSH_BLOCK ? BPMD_RF_BLOCK : flush == BPMD_FLUSH_TREES ? BPMD_RF_TREES
                                                                                         : BPMD_RF_SYNC;
        InfMeta* dm = (InfMeta*)(s->dctl + kCtlMeta);
        ok = ok && bpmd_internal_inflate_resume(s->din, &dm->in_off, &dm->in_len, wo, &dm->out_off, &dm->out_cap,
                                                &dm->out_len, &dm->status, rc, hs) == 0;
        ok = ok && hipMemcpyAsync(&m, s->dctl + kCtlMeta, sizeof m, hipMemcpyDeviceToHost, hs) == hipSuccess &&
             hipMemcpyAsync(&out_ck, s->dctl + kCtlOut, sizeof out_ck, hipMemcpyDeviceToHost, hs) == hipSuccess &&
             hipStreamSynchronize(hs) == hipSuccess;
        if (!ok) {
            s->in.resize(kept);
            return BPMD_R_HIP_ERROR;
        }
        st = m.status;
        fresh = m.out_len > s->delivered ? m.out_len - s->delivered : 0;
        if (fresh && hipMemcpy(zs->next_out, wo + kWinMax + s->delivered, fresh, hipMemcpyDeviceToHost) != hipSuccess)
            return BPMD_R_HIP_ERROR;
        // advance the checkpoint: window <- the last W bytes before it
        const uint32_t K = out_ck.out;
        const uint32_t nh = (uint32_t)std::min<size_t>((size_t)s->hist + K, W);
        if (K && st < BPMD_END_OF_STREAM) {
            uint8_t* nw = s->dwo[s->wcur ^ 1];
            if (hipMemcpyAsync(nw + kWinMax - nh, wo + kWinMax + K - nh, nh, hipMemcpyDeviceToDevice, hs) !=
                hipSuccess)
                return BPMD_R_HIP_ERROR;
            s->wcur ^= 1;
        }
        const size_t used_bytes = out_ck.bit >> 3;
        if (st == BPMD_END_OF_STREAM) {
            // consumed up to the byte holding the last bit of the final block
            const size_t end = (out_ck.bit + 7) >> 3;
            const size_t take = end > kept ? std::min(end - kept, n_in) : 0;
            zs->next_in = (const uint8_t*)zs->next_in + take;
            zs->avail_in -= take;
            zs->total_in += take;
            zs->next_out = (uint8_t*)zs->next_out + fresh;
            zs->avail_out -= fresh;
            zs->total_out += fresh;
            s->inf_mode = 1;
            s->in.clear();
            s->in.shrink_to_fit();
            return BPMD_END_OF_STREAM;
        }
        if (st > BPMD_END_OF_STREAM) {
            // a data error: the reference's err() returns without done(), so
            // the bytes are in the caller's buffer but zs is not advanced
            // (inflate_stream.ipp:121-125); the stream is BAD from now on
            s->inf_mode = 2;
            s->in.clear();
            s->in.shrink_to_fit();
            return st;
        }
        // the reference's consumption: an exhausted input is taken whole; a
        // call that stopped early (Flush::block / trees, a full output)
        // leaves the bytes past where it stopped (bits held < 8 after
        // inflate_fast's rewind, inflate_stream.ipp:1101-1112)
        const uint64_t stop_at = s->in_abs + ((out_ck.end_bit + 7) >> 3);
        if (out_ck.why == BPMD_RW_STARVED) s->ref_pos = s->in_abs + n;
        else if (stop_at > s->ref_pos) s->ref_pos = std::min<uint64_t>(stop_at, s->in_abs + n);
        s->hist = nh;
        s->delivered = s->delivered + fresh - K;
        s->in.erase(s->in.begin(), s->in.begin() + (ptrdiff_t)used_bytes);
        s->in_abs += used_bytes;
        out_ck.bit -= (uint32_t)(8 * used_bytes);
        // data_type (inflate_stream.ipp:108-112): bits held, last block, block boundary, after a header
        const uint32_t held = out_ck.end_bit >= 8 * used_bytes ? (uint32_t)(8 * n - out_ck.end_bit) : 0u;
        zs->data_type = (int)((held < 64 ? held : 0u) + (out_ck.last ? 64u : 0u) + (out_ck.at_type ? 128u : 0u) +
                              (out_ck.at_hdr ? 256u : 0u));
        s->ck = out_ck;
        if (s->in.capacity() > 4 * s->in.size() + 65536) s->in.shrink_to_fit();
    }
    zs->next_in = (const uint8_t*)zs->next_in + n_in;
    zs->avail_in = 0;
    zs->total_in += n_in;
    zs->next_out = (uint8_t*)zs->next_out + fresh;
    zs->avail_out -= fresh;
    zs->total_out += fresh;
    // done(): no progress -- nothing the reference would have consumed, nothing produced
    if ((s->ref_pos == ref_before && fresh == 0) || flush == BPMD_FLUSH_FINISH) return BPMD_NEED_BUFFERS;
    return BPMD_OK;
}

extern "C" int bpmd_inflate_stream_footprint(const bpmd_stream* s, size_t* host_bytes, size_t* device_bytes)
{
    if (!s || s->is_deflate) return BPMD_R_INVALID_ARGUMENT;
    if (host_bytes) *host_bytes = s->in.capacity();
    if (device_bytes)
        *device_bytes = (s->dctl ? kCtlBytes : 0) + (s->din ? s->din_cap + 64 : 0) +
                        (s->dwo[0] ? 2 * (kWinMax + s->dwo_cap + 64) : 0);
    return BPMD_R_OK;
}

extern "C" void bpmd_stream_destroy(bpmd_stream* s)
{
    if (!s) return;
    if (s->dmem) (void)hipFree(s->dmem);
    if (s->dctl) (void)hipFree(s->dctl);
    if (s->din) (void)hipFree(s->din);
    for (int k = 0; k < 2; ++k)
        if (s->dwo[k]) (void)hipFree(s->dwo[k]);
    if (s->hs) (void)hipStreamDestroy(s->hs);
    delete s;
}
