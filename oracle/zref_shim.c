/*
 * zref_shim.c -- TEST INFRASTRUCTURE.  A thin C wrapper, linked against the
 * reference's vendored zlib 1.3.1 (/root/reference/test/extern/zlib-1.3.1,
 * compiled in place by oracle/Makefile with Z_PREFIX into
 * oracle/_ref/libzref.so).  It reproduces the permessage-deflate call pattern
 * of websocket/detail/impl_base.hpp:85-154 on real zlib so that the C
 * restatement in bzo_deflate.c can be checked byte-for-byte (Beast == zlib
 * 1.3.1 at levels 1-9).
 */
#define Z_PREFIX 1
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
