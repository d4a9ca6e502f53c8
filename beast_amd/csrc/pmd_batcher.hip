// pmd_batcher.hip -- cross-connection micro-batcher.
// Host code only.
//
// Beast drives its codec once per message from each connection's own async
// operation (write_some_op, websocket/impl/write.hpp:463-545; the read side,
// read.hpp:522-610 and 1284-1385, through impl_base.hpp:85-190), so a server
// with thousands of connections makes thousands of tiny codec calls.  The
// batcher is the seam that turns them into batch launches: any thread submits
// one message (host bytes) with a completion callback -- the completion-
// handler model of those async operations -- and the batcher packs messages
// into pinned staging; a launcher thread starts a batch (H2D, one kernel
// launch, D2H on the slot's stream) when max_msgs or the staging bytes are
// reached or the oldest message has waited max_delay_us; a completion thread
// waits for it, copies each output to its submitter's buffer and runs the
// callbacks.  Two staging slots alternate, so submissions fill one while the
// GPU works on the other.
#include <hip/hip_runtime.h>

#include <chrono>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "../../include/beast_pmd.h"

namespace {

using clk = std::chrono::steady_clock;

size_t a16(size_t n) { return (n + 15) & ~size_t(15); }

struct Item {
    void* out;
    size_t out_cap;
    bpmd_done_fn fn;
    void* user;
};

struct Slot {
    uint8_t *h_in = nullptr, *h_out = nullptr, *d_in = nullptr, *d_out = nullptr;
    uint64_t *h_in_off = nullptr, *h_out_off = nullptr, *d_in_off = nullptr, *d_out_off = nullptr;
    uint32_t *h_in_len = nullptr, *h_out_cap = nullptr, *d_in_len = nullptr, *d_out_cap = nullptr;
    uint32_t *h_out_len = nullptr, *d_out_len = nullptr;
    int32_t *h_status = nullptr, *d_status = nullptr;
    hipStream_t stream = nullptr;
    std::vector<Item> items;
    size_t in_bytes = 0, out_bytes = 0;
    bool sealed = false;     // full: launch as soon as possible
    bool inflight = false;   // launched, not yet delivered
    int launch_err = 0;
    clk::time_point first;
};

template <class T>
bool host_alloc(T*& p, size_t n)
{
    return hipHostMalloc((void**)&p, n * sizeof(T) + 16, 0) == hipSuccess;
}
template <class T>
bool dev_alloc(T*& p, size_t n)
{
    return hipMalloc((void**)&p, n * sizeof(T) + 16) == hipSuccess;
}

}  // namespace

struct bpmd_batcher {
    bpmd_cfg cfg{};
    int op = BPMD_OP_INFLATE;
    uint32_t max_msgs = 0;
    size_t max_in = 0, max_out = 0;
    clk::duration delay{};
    int device = 0;
    Slot slot[2];
    int cur = 0;           // slot taking submissions
    int fifo[2] = {0, 0};  // launched slots, oldest first
    int nfifo = 0;
    std::mutex mu;
    std::condition_variable cv_work;   // launcher: something to launch, or stop
    std::condition_variable cv_done;   // completer: something launched, or stop
    std::condition_variable cv_room;   // submitters: a slot became free
    std::condition_variable cv_idle;   // flushers: deliveries caught up
    bool stop = false, launcher_done = false;
    unsigned flushers = 0;
    uint64_t submitted = 0, completed = 0;
    int error = 0;
    std::thread launcher, completer;
};

extern "C" void bpmd_internal_scratch_release(hipStream_t stream);

namespace {

void free_slot(Slot& s)
{
    for (void* p : {(void*)s.h_in, (void*)s.h_out, (void*)s.h_in_off, (void*)s.h_out_off, (void*)s.h_in_len,
                    (void*)s.h_out_cap, (void*)s.h_out_len, (void*)s.h_status})
        if (p) (void)hipHostFree(p);
    for (void* p : {(void*)s.d_in, (void*)s.d_out, (void*)s.d_in_off, (void*)s.d_out_off, (void*)s.d_in_len,
                    (void*)s.d_out_cap, (void*)s.d_out_len, (void*)s.d_status})
        if (p) (void)hipFree(p);
    if (s.stream) {
        (void)hipStreamSynchronize(s.stream);
        bpmd_internal_scratch_release(s.stream);
        (void)hipStreamDestroy(s.stream);
    }
    s = Slot();
}

bool alloc_slot(bpmd_batcher* b, Slot& s)
{
    const size_t m = b->max_msgs;
    bool ok = host_alloc(s.h_in, b->max_in) && host_alloc(s.h_out, b->max_out) && host_alloc(s.h_in_off, m) &&
              host_alloc(s.h_out_off, m) && host_alloc(s.h_in_len, m) && host_alloc(s.h_out_cap, m) &&
              host_alloc(s.h_out_len, m) && host_alloc(s.h_status, m);
    ok = ok && dev_alloc(s.d_in, b->max_in) && dev_alloc(s.d_out, b->max_out) && dev_alloc(s.d_in_off, m) &&
         dev_alloc(s.d_out_off, m) && dev_alloc(s.d_in_len, m) && dev_alloc(s.d_out_cap, m) &&
         dev_alloc(s.d_out_len, m) && dev_alloc(s.d_status, m);
    ok = ok && hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking) == hipSuccess;
    if (ok) s.items.reserve(m);
    return ok;
}

// Copies and the batch launch of slot s, all asynchronous on its stream.
int launch(bpmd_batcher* b, Slot& s)
{
    const size_t n = s.items.size();
    hipStream_t st = s.stream;
    const auto H2D = hipMemcpyHostToDevice, D2H = hipMemcpyDeviceToHost;
    bool ok = hipMemcpyAsync(s.d_in, s.h_in, s.in_bytes ? s.in_bytes : 1, H2D, st) == hipSuccess &&
              hipMemcpyAsync(s.d_in_off, s.h_in_off, n * 8, H2D, st) == hipSuccess &&
              hipMemcpyAsync(s.d_in_len, s.h_in_len, n * 4, H2D, st) == hipSuccess &&
              hipMemcpyAsync(s.d_out_off, s.h_out_off, n * 8, H2D, st) == hipSuccess &&
              hipMemcpyAsync(s.d_out_cap, s.h_out_cap, n * 4, H2D, st) == hipSuccess;
    if (!ok) return BPMD_R_HIP_ERROR;
    const int r = b->op == BPMD_OP_INFLATE
                      ? bpmd_inflate_batch(&b->cfg, s.d_in, s.d_in_off, s.d_in_len, (uint32_t)n, s.d_out, s.d_out_off,
                                           s.d_out_cap, s.d_out_len, s.d_status, st)
                      : bpmd_deflate_batch(&b->cfg, s.d_in, s.d_in_off, s.d_in_len, (uint32_t)n, s.d_out, s.d_out_off,
                                           s.d_out_cap, s.d_out_len, s.d_status, st);
    if (r) return r;
    ok = hipMemcpyAsync(s.h_out_len, s.d_out_len, n * 4, D2H, st) == hipSuccess &&
         hipMemcpyAsync(s.h_status, s.d_status, n * 4, D2H, st) == hipSuccess &&
         hipMemcpyAsync(s.h_out, s.d_out, s.out_bytes ? s.out_bytes : 1, D2H, st) == hipSuccess;
    return ok ? BPMD_R_OK : BPMD_R_HIP_ERROR;
}

// Wait for slot s, hand each result to its submitter (no lock held).
int deliver(Slot& s)
{
    int err = s.launch_err;
    if (!err && hipStreamSynchronize(s.stream) != hipSuccess) err = BPMD_R_HIP_ERROR;
    for (size_t i = 0; i < s.items.size(); ++i) {
        const Item& it = s.items[i];
        int32_t status = err ? err : s.h_status[i];
        size_t len = err ? 0 : s.h_out_len[i];
        if (!err && len > it.out_cap) {   // deflate payload larger than the caller's buffer
            status = BPMD_NEED_BUFFERS;
            len = 0;
        }
        if (len) std::memcpy(it.out, s.h_out + s.h_out_off[i], len);
        it.fn(it.user, status, len);
    }
    return err;
}

void launcher_main(bpmd_batcher* b)
{
    (void)hipSetDevice(b->device);
    std::unique_lock<std::mutex> lk(b->mu);
    for (;;) {
        Slot& s = b->slot[b->cur];
        const bool have = !s.inflight && !s.items.empty();
        if (have && (s.sealed || b->stop || b->flushers || clk::now() >= s.first + b->delay)) {
            const int k = b->cur;
            s.inflight = true;
            b->cur ^= 1;
            lk.unlock();
            const int e = launch(b, s);
            lk.lock();
            s.launch_err = e;
            b->fifo[b->nfifo++] = k;
            b->cv_done.notify_all();
            b->cv_room.notify_all();
            continue;
        }
        if (b->stop && !have) break;
        if (have)
            b->cv_work.wait_until(lk, s.first + b->delay);
        else
            b->cv_work.wait(lk);
    }
    b->launcher_done = true;
    b->cv_done.notify_all();
}

void completer_main(bpmd_batcher* b)
{
    (void)hipSetDevice(b->device);
    std::unique_lock<std::mutex> lk(b->mu);
    for (;;) {
        if (b->nfifo == 0) {
            if (b->launcher_done) break;
            b->cv_done.wait(lk);
            continue;
        }
        Slot& s = b->slot[b->fifo[0]];
        lk.unlock();
        const int err = deliver(s);
        lk.lock();
        b->completed += s.items.size();
        s.items.clear();
        s.in_bytes = s.out_bytes = 0;
        s.sealed = s.inflight = false;
        s.launch_err = 0;
        if (err && !b->error) b->error = err;
        b->fifo[0] = b->fifo[1];
        --b->nfifo;
        b->cv_room.notify_all();
        b->cv_work.notify_all();
        b->cv_idle.notify_all();
    }
}

}  // namespace

extern "C" int bpmd_batcher_create(const bpmd_cfg* cfg, int op, uint32_t max_msgs, size_t max_in_bytes,
                                   size_t max_out_bytes, uint32_t max_delay_us, bpmd_batcher** out)
{
    if (!cfg || !out || (op != BPMD_OP_INFLATE && op != BPMD_OP_DEFLATE) || max_msgs == 0 || max_in_bytes == 0 ||
        max_out_bytes == 0)
        return BPMD_R_INVALID_ARGUMENT;
    *out = nullptr;
    // parameters are validated exactly as the batch calls do (zero messages: no device use)
    const int v = op == BPMD_OP_INFLATE
                      ? bpmd_inflate_batch(cfg, nullptr, nullptr, nullptr, 0, nullptr, nullptr, nullptr, nullptr,
                                           nullptr, nullptr)
                      : bpmd_deflate_batch(cfg, nullptr, nullptr, nullptr, 0, nullptr, nullptr, nullptr, nullptr,
                                           nullptr, nullptr);
    if (v) return v;
    int r = bpmd_init();
    if (r) return r;
    bpmd_batcher* b = new (std::nothrow) bpmd_batcher;
    if (!b) return BPMD_R_INVALID_ARGUMENT;
    b->cfg = *cfg;
    b->op = op;
    b->max_msgs = max_msgs;
    b->max_in = a16(max_in_bytes);
    b->max_out = a16(max_out_bytes);
    b->delay = std::chrono::microseconds(max_delay_us);
    (void)hipGetDevice(&b->device);
    if (!alloc_slot(b, b->slot[0]) || !alloc_slot(b, b->slot[1])) {
        free_slot(b->slot[0]);
        free_slot(b->slot[1]);
        delete b;
        return BPMD_R_HIP_ERROR;
    }
    b->launcher = std::thread(launcher_main, b);
    b->completer = std::thread(completer_main, b);
    *out = b;
    return BPMD_R_OK;
}

extern "C" int bpmd_batcher_submit(bpmd_batcher* b, const void* in, size_t n, void* out, size_t out_cap,
                                   bpmd_done_fn fn, void* user)
{
    if (!b || !fn || (n && !in) || (out_cap && !out)) return BPMD_R_INVALID_ARGUMENT;
    const size_t slot_cap = b->op == BPMD_OP_DEFLATE ? bpmd_deflate_upper_bound(n) : out_cap;
    if (n > 0xFFFFFFFFu || slot_cap > 0xFFFFFFFFu || a16(n) > b->max_in || a16(slot_cap) > b->max_out)
        return BPMD_R_INVALID_ARGUMENT;
    std::unique_lock<std::mutex> lk(b->mu);
    for (;;) {
        if (b->error) return b->error;
        if (b->stop) return BPMD_R_INVALID_ARGUMENT;
        Slot& s = b->slot[b->cur];
        if (!s.inflight) {
            if (s.items.size() < b->max_msgs && s.in_bytes + a16(n) <= b->max_in &&
                s.out_bytes + a16(slot_cap) <= b->max_out)
                break;
            if (!s.sealed) {
                s.sealed = true;
                b->cv_work.notify_all();
            }
        }
        b->cv_room.wait(lk);
    }
    Slot& s = b->slot[b->cur];
    const size_t k = s.items.size();
    if (k == 0) {
        s.first = clk::now();
        b->cv_work.notify_all();
    }
    if (n) std::memcpy(s.h_in + s.in_bytes, in, n);
    s.h_in_off[k] = s.in_bytes;
    s.h_in_len[k] = (uint32_t)n;
    s.h_out_off[k] = s.out_bytes;
    s.h_out_cap[k] = (uint32_t)slot_cap;
    s.in_bytes += a16(n);
    s.out_bytes += a16(slot_cap);
    s.items.push_back(Item{out, out_cap, fn, user});
    ++b->submitted;
    if (s.items.size() == b->max_msgs) {
        s.sealed = true;
        b->cv_work.notify_all();
    }
    return BPMD_R_OK;
}

extern "C" int bpmd_batcher_flush(bpmd_batcher* b)
{
    if (!b) return BPMD_R_INVALID_ARGUMENT;
    std::unique_lock<std::mutex> lk(b->mu);
    const uint64_t target = b->submitted;
    ++b->flushers;
    b->cv_work.notify_all();
    b->cv_idle.wait(lk, [&] { return b->completed >= target || b->error != 0; });
    --b->flushers;
    return b->error;
}

extern "C" void bpmd_batcher_destroy(bpmd_batcher* b)
{
    if (!b) return;
    {
        std::lock_guard<std::mutex> lk(b->mu);
        b->stop = true;
    }
    b->cv_work.notify_all();
    b->cv_room.notify_all();
    b->cv_done.notify_all();
    if (b->launcher.joinable()) b->launcher.join();
    if (b->completer.joinable()) b->completer.join();
    free_slot(b->slot[0]);
    free_slot(b->slot[1]);
    delete b;
}
