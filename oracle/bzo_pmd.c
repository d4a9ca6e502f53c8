/*
 * bzo_pmd.c -- CPU ORACLE (test infrastructure only, see bzo.h).
 *
 * permessage-deflate framing around the restated codec:
 *   compress one message       websocket/detail/impl_base.hpp:85-154
 *   no_context_takeover reset  impl_base.hpp:156-166
 *   inflate + 00 00 FF FF tail impl_base.hpp:168-190, websocket/impl/read.hpp:1343-1356
 * plus multi-threaded batch drivers used as the CPU baseline (one deflater and
 * one inflater per thread, contiguous message ranges, reset per message --
 * the shape of test/bench/zlib/{deflate,inflate}_stream.cpp).
 */
#include "bzo.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

long bzo_pmd_deflate_msg(bzo_deflater* z, const uint8_t* in, size_t n, uint8_t* out, size_t cap)
{
    bzo_zparams zs;
    memset(&zs, 0, sizeof zs);
    zs.data_type = 2;
    zs.next_out = out;
    zs.avail_out = cap;
    int ec;
    if (n != 0) {                       /* empty buffers are skipped */
        zs.next_in = in;
        zs.avail_in = n;
        ec = bzo_deflate_write(z, &zs, BZO_FLUSH_NONE);
        if (ec && ec != BZO_NEED_BUFFERS) return -(long)(ec < 0 ? BZO_GENERAL : ec);
        if (zs.avail_in != 0 || zs.avail_out == 0) return -(long)BZO_NEED_BUFFERS;
    }
    zs.next_in = NULL;
    zs.avail_in = 0;
    ec = bzo_deflate_write(z, &zs, BZO_FLUSH_BLOCK);
    if (ec && ec != BZO_NEED_BUFFERS) return -(long)ec;
    if (zs.avail_out < 6) return -(long)BZO_NEED_BUFFERS;
    ec = bzo_deflate_write(z, &zs, BZO_FLUSH_SYNC);
    if (ec) return -(long)ec;
    /* drop the 00 00 FF FF of the empty stored block */
    return (long)zs.total_out - 4;
}

/* per-thread scratch so the decoder can run one byte past the caller's
 * capacity: producing byte cap+1 is how "capacity exceeded" is detected */
static __thread uint8_t* scratch_buf = NULL;
static __thread size_t scratch_cap = 0;

static uint8_t* scratch(size_t need)
{
    if (scratch_cap < need) {
        free(scratch_buf);
        scratch_cap = need < 65536 ? 65536 : need;
        scratch_buf = (uint8_t*)malloc(scratch_cap);
    }
    return scratch_buf;
}

size_t bzo_inflate_last_out(const bzo_inflater* z);

int bzo_pmd_inflate_msg(bzo_inflater* z, const uint8_t* in, size_t n, uint8_t* out, size_t cap,
                        size_t* out_len, int raw)
{
    static const uint8_t tail[4] = {0x00, 0x00, 0xff, 0xff};
    uint8_t* buf = scratch(cap + 1);
    size_t made = 0;
    int ec = 0, st = BZO_OK;
    bzo_zparams zs;

    if (n != 0 || raw) {
        /* impl.inflate(): zi.write(zs, Flush::sync) over the payload */
        memset(&zs, 0, sizeof zs);
        zs.next_in = in;
        zs.avail_in = n;
        zs.next_out = buf;
        /* raw: exactly one inflate_stream::write() into cap bytes */
        zs.avail_out = raw ? cap : cap + 1;
        ec = bzo_inflate_write(z, &zs, BZO_FLUSH_SYNC);
        made = bzo_inflate_last_out(z);
        if (raw) { st = ec < 0 ? BZO_GENERAL : ec; goto done; }
        if (made > cap) { made = cap; st = BZO_NEED_BUFFERS; goto done; }
        if (ec && ec != BZO_NEED_BUFFERS) { st = ec < 0 ? BZO_GENERAL : ec; goto done; }
    }
    {
        /* inflate_with_eb() until a call produces no output */
        size_t eb_used = 0;
        for (;;) {
            memset(&zs, 0, sizeof zs);
            zs.next_in = tail + eb_used;
            zs.avail_in = 4 - eb_used;
            zs.next_out = buf + made;
            zs.avail_out = cap + 1 - made;
            ec = bzo_inflate_write(z, &zs, BZO_FLUSH_SYNC);
            size_t got = bzo_inflate_last_out(z);
            eb_used += zs.total_in;
            made += got;
            if (made > cap) { made = cap; st = BZO_NEED_BUFFERS; goto done; }
            if (ec == BZO_NEED_BUFFERS) ec = 0;
            if (ec) { st = ec < 0 ? BZO_GENERAL : ec; goto done; }
            if (got == 0) break;
        }
    }
done:
    memcpy(out, buf, made);
    *out_len = made;
    return st;
}

/* ------------------------------------------------------------- batches */

typedef struct {
    int kind;   /* 0 deflate, 1 inflate */
    int level, wbits, mem_level, strategy, raw;
    const uint8_t* in; const uint64_t* in_off; const uint32_t* in_len;
    uint8_t* out; const uint64_t* out_off; const uint32_t* out_cap;
    uint32_t* out_len; int32_t* status;
    uint32_t lo, hi;
} job_t;

static void* run_job(void* arg)
{
    job_t* j = (job_t*)arg;
    if (j->kind == 0) {
        bzo_deflater* z = bzo_deflate_new();
        int r = bzo_deflate_reset_params(z, j->level, j->wbits, j->mem_level, j->strategy);
        for (uint32_t i = j->lo; i < j->hi; ++i) {
            if (r) { j->status[i] = BZO_STREAM_ERROR; j->out_len[i] = 0; continue; }
            bzo_deflate_reset(z);
            long got = bzo_pmd_deflate_msg(z, j->in + j->in_off[i], j->in_len[i],
                                           j->out + j->out_off[i], j->out_cap[i]);
            if (got < 0) { j->status[i] = (int32_t)(-got); j->out_len[i] = 0; }
            else { j->status[i] = 0; j->out_len[i] = (uint32_t)got; }
        }
        bzo_deflate_free(z);
    } else {
        bzo_inflater* z = bzo_inflate_new();
        for (uint32_t i = j->lo; i < j->hi; ++i) {
            size_t got = 0;
            if (bzo_inflate_reset(z, j->wbits)) { j->status[i] = BZO_STREAM_ERROR; j->out_len[i] = 0; continue; }
            int st = bzo_pmd_inflate_msg(z, j->in + j->in_off[i], j->in_len[i],
                                         j->out + j->out_off[i], j->out_cap[i], &got, j->raw);
            j->status[i] = st;
            j->out_len[i] = (uint32_t)got;
        }
        bzo_inflate_free(z);
    }
    return NULL;
}

static int run_batch(job_t proto, uint32_t n, int threads)
{
    if (threads <= 0) threads = 1;
    if ((uint32_t)threads > n) threads = n ? (int)n : 1;
    job_t* jobs = (job_t*)calloc((size_t)threads, sizeof(job_t));
    pthread_t* tid = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    uint32_t per = (n + (uint32_t)threads - 1) / (uint32_t)threads;
    for (int t = 0; t < threads; ++t) {
        jobs[t] = proto;
        jobs[t].lo = (uint32_t)t * per < n ? (uint32_t)t * per : n;
        jobs[t].hi = jobs[t].lo + per < n ? jobs[t].lo + per : n;
        if (threads == 1) run_job(&jobs[t]);
        else pthread_create(&tid[t], NULL, run_job, &jobs[t]);
    }
    if (threads > 1)
        for (int t = 0; t < threads; ++t) pthread_join(tid[t], NULL);
    free(jobs);
    free(tid);
    return 0;
}

int bzo_pmd_deflate_batch(int level, int wbits, int mem_level, int strategy, const uint8_t* in,
                          const uint64_t* in_off, const uint32_t* in_len, uint32_t n, uint8_t* out,
                          const uint64_t* out_off, const uint32_t* out_cap, uint32_t* out_len,
                          int32_t* status, int threads)
{
    job_t p;
    memset(&p, 0, sizeof p);
    p.kind = 0; p.level = level; p.wbits = wbits; p.mem_level = mem_level; p.strategy = strategy;
    p.in = in; p.in_off = in_off; p.in_len = in_len; p.out = out; p.out_off = out_off;
    p.out_cap = out_cap; p.out_len = out_len; p.status = status;
    return run_batch(p, n, threads);
}

int bzo_pmd_inflate_batch(int wbits, int raw, const uint8_t* in, const uint64_t* in_off,
                          const uint32_t* in_len, uint32_t n, uint8_t* out, const uint64_t* out_off,
                          const uint32_t* out_cap, uint32_t* out_len, int32_t* status, int threads)
{
    job_t p;
    memset(&p, 0, sizeof p);
    p.kind = 1; p.wbits = wbits; p.raw = raw;
    p.in = in; p.in_off = in_off; p.in_len = in_len; p.out = out; p.out_off = out_off;
    p.out_cap = out_cap; p.out_len = out_len; p.status = status;
    return run_batch(p, n, threads);
}
