/*
 * zref_shim.c -- TEST INFRASTRUCTURE.  A thin C wrapper, linked against the
 * reference's vendored zlib 1.3.1 (/root/reference/test/extern/zlib-1.3.1,
 * compiled in place by oracle/Makefile with Z_PREFIX into
 * oracle/_ref/libzref.so).  It reproduces the permessage-deflate call pattern
 * of websocket/detail/impl_base.hpp:85-154 on real zlib so that the C
 * restatement in bzo_deflate.c can be checked byte-for-byte (Beast == zlib
 * 1.3.1 at levels 1-9).
 */
#ifndef ZREF_SYSTEM
#define Z_PREFIX 1   /* libzref.so: the vendored zlib, prefixed; libzsys.so: the image's -lz */
#endif
#include "zlib.h"

#include <string.h>

/* Returns the pmd payload length, or -1 on failure.  flush_mode 0 = pmd
 * framing (NO_FLUSH, BLOCK, SYNC, strip 4); 1 = one Z_FULL_FLUSH call (the
 * shape of test/bench/zlib/deflate_stream.cpp:90-118); 2 = Z_FINISH. */
long zref_deflate(int level, int wbits, int mem_level, int strategy, int flush_mode,
                  const unsigned char* in, unsigned long n, unsigned char* out, unsigned long cap)
{
    z_stream zs;
    memset(&zs, 0, sizeof zs);
    if (deflateInit2(&zs, level, Z_DEFLATED, -wbits, mem_level, strategy) != Z_OK) return -1;
    zs.next_out = out;
    zs.avail_out = (uInt)cap;
    long result = -1;
    if (flush_mode == 0) {
        if (n) {
            zs.next_in = (unsigned char*)in;
            zs.avail_in = (uInt)n;
            if (deflate(&zs, Z_NO_FLUSH) == Z_STREAM_ERROR) goto out;
            if (zs.avail_in) goto out;
        }
        if (deflate(&zs, Z_BLOCK) == Z_STREAM_ERROR) goto out;
        if (zs.avail_out < 6) goto out;
        if (deflate(&zs, Z_SYNC_FLUSH) != Z_OK) goto out;
        result = (long)zs.total_out - 4;
    } else {
        zs.next_in = (unsigned char*)in;
        zs.avail_in = (uInt)n;
        int r = deflate(&zs, flush_mode == 1 ? Z_FULL_FLUSH : Z_FINISH);
        if (r == Z_STREAM_ERROR) goto out;
        result = (long)zs.total_out;
    }
out:
    deflateEnd(&zs);
    return result;
}

/* Raw inflate of a complete stream; returns output length or -1. */
long zref_inflate(int wbits, const unsigned char* in, unsigned long n, unsigned char* out,
                  unsigned long cap, int* zret)
{
    z_stream zs;
    memset(&zs, 0, sizeof zs);
    if (inflateInit2(&zs, -wbits) != Z_OK) return -1;
    zs.next_in = (unsigned char*)in;
    zs.avail_in = (uInt)n;
    zs.next_out = out;
    zs.avail_out = (uInt)cap;
    int r = inflate(&zs, Z_SYNC_FLUSH);
    if (zret) *zret = r;
    long got = (long)zs.total_out;
    inflateEnd(&zs);
    return got;
}

/* ------------------------------------------------------------------------
 * Batches for the CPU baseline (bench.py / scripts/calibrate_cpu.py): the
 * reference's zlib over contiguous message ranges, one z_stream per thread,
 * re-initialised per message as Beast re-inits its codec per message under
 * no_context_takeover (impl_base.hpp:156-166).  Inflate feeds the payload
 * plus the 00 00 FF FF tail with Z_SYNC_FLUSH (impl_base.hpp:168-190). */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>

typedef struct {
    int inflate, level, wbits, mem_level;
    const unsigned char* in;
    const uint64_t* in_off;
    const uint32_t* in_len;
    unsigned char* out;
    const uint64_t* out_off;
    const uint32_t* out_cap;
    uint32_t* out_len;
    uint32_t lo, hi;
} zref_job;

static void* zref_run(void* arg)
{
    zref_job* j = (zref_job*)arg;
    static const unsigned char tail[4] = {0x00, 0x00, 0xff, 0xff};
    /* one codec per thread, reset per message (as Beast's per-connection
     * codec is reset, without freeing its buffers) */
    z_stream zs;
    memset(&zs, 0, sizeof zs);
    if (j->inflate ? inflateInit2(&zs, -j->wbits) != Z_OK
                   : deflateInit2(&zs, j->level, Z_DEFLATED, -j->wbits, j->mem_level, 0) != Z_OK)
        return NULL;
    for (uint32_t i = j->lo; i < j->hi; ++i) {
        const unsigned char* p = j->in + j->in_off[i];
        unsigned char* o = j->out + j->out_off[i];
        if (j->inflate) {
            inflateReset(&zs);
            zs.next_in = (unsigned char*)p;
            zs.avail_in = j->in_len[i];
            zs.next_out = o;
            zs.avail_out = j->out_cap[i];
            inflate(&zs, Z_SYNC_FLUSH);
            zs.next_in = (unsigned char*)tail;
            zs.avail_in = 4;
            inflate(&zs, Z_SYNC_FLUSH);
            j->out_len[i] = (uint32_t)zs.total_out;
        } else {
            /* impl_base.hpp:85-154: Flush::none, block, sync, strip 4 */
            deflateReset(&zs);
            zs.next_out = o;
            zs.avail_out = j->out_cap[i];
            if (j->in_len[i]) {
                zs.next_in = (unsigned char*)p;
                zs.avail_in = j->in_len[i];
                deflate(&zs, Z_NO_FLUSH);
            }
            deflate(&zs, Z_BLOCK);
            deflate(&zs, Z_SYNC_FLUSH);
            j->out_len[i] = zs.total_out >= 4 ? (uint32_t)zs.total_out - 4 : 0u;
        }
    }
    if (j->inflate) inflateEnd(&zs);
    else deflateEnd(&zs);
    return NULL;
}

int zref_batch(int inflate_, int level, int wbits, int mem_level, const unsigned char* in, const uint64_t* in_off,
               const uint32_t* in_len, uint32_t n, unsigned char* out, const uint64_t* out_off,
               const uint32_t* out_cap, uint32_t* out_len, int threads)
{
    if (threads < 1) threads = 1;
    if ((uint32_t)threads > n) threads = n ? (int)n : 1;
    zref_job* jobs = (zref_job*)calloc((size_t)threads, sizeof(zref_job));
    pthread_t* tid = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    if (!jobs || !tid) return -1;
    const uint32_t per = (n + (uint32_t)threads - 1) / (uint32_t)threads;
    for (int t = 0; t < threads; ++t) {
        zref_job* j = &jobs[t];
        j->inflate = inflate_;
        j->level = level;
        j->wbits = wbits;
        j->mem_level = mem_level;
        j->in = in;
        j->in_off = in_off;
        j->in_len = in_len;
        j->out = out;
        j->out_off = out_off;
        j->out_cap = out_cap;
        j->out_len = out_len;
        j->lo = per * (uint32_t)t < n ? per * (uint32_t)t : n;
        j->hi = j->lo + per < n ? j->lo + per : n;
        if (threads == 1) zref_run(j);
        else pthread_create(&tid[t], NULL, zref_run, j);
    }
    if (threads > 1)
        for (int t = 0; t < threads; ++t) pthread_join(tid[t], NULL);
    free(jobs);
    free(tid);
    return 0;
}

/* the zlib this shim was built against (1.3.1 for libzref, the image's for libzsys) */
const char* zref_version(void) { return zlibVersion(); }
