/*
 * oracle_backend.c -- TEST INFRASTRUCTURE.  The per-stream entry points of
 * include/beast_pmd.h that the drop-in boost::beast::zlib headers call,
 * implemented on the CPU oracle (oracle/bzo_*.c, the C restatement of
 * Beast's zlib).  Linking tests/cpp/ws_echo.cpp against this library
 * instead of libbeast_pmd.so runs the same C1 harness with Beast's CPU
 * codec, so the GPU facade's echo time has a CPU number measured the same
 * way beside it (tests/test_facade.py).  Not a product path: nothing under
 * beast_amd/ loads it.
 */
#include <stdlib.h>
#include <string.h>

#include "../../include/beast_pmd.h"
#include "../../oracle/bzo.h"

struct bpmd_stream {
    int is_deflate;
    bzo_deflater* zo;
    bzo_inflater* zi;
};

static bzo_zparams to_bzo(const bpmd_zparams* z)
{
    bzo_zparams b;
    b.next_in = (const uint8_t*)z->next_in;
    b.avail_in = z->avail_in;
    b.total_in = z->total_in;
    b.next_out = (uint8_t*)z->next_out;
    b.avail_out = z->avail_out;
    b.total_out = z->total_out;
    b.data_type = z->data_type;
    return b;
}

static void from_bzo(bpmd_zparams* z, const bzo_zparams* b)
{
    z->next_in = b->next_in;
    z->avail_in = b->avail_in;
    z->total_in = b->total_in;
    z->next_out = b->next_out;
    z->avail_out = b->avail_out;
    z->total_out = b->total_out;
    z->data_type = b->data_type;
}

static int result(int r)
{
    return r == BZO_THROW_INVALID_ARGUMENT ? BPMD_R_INVALID_ARGUMENT
         : r == BZO_THROW_DOMAIN_ERROR     ? BPMD_R_DOMAIN_ERROR
         : r < 0                           ? BPMD_R_HIP_ERROR
                                           : r;
}

size_t bpmd_deflate_upper_bound(size_t n) { return bzo_deflate_upper_bound_free(n); }

int bpmd_deflate_stream_create(int level, int window_bits, int mem_level, int strategy, bpmd_stream** out)
{
    if (!out) return BPMD_R_INVALID_ARGUMENT;
    bpmd_stream* s = (bpmd_stream*)calloc(1, sizeof *s);
    s->is_deflate = 1;
    s->zo = bzo_deflate_new();
    int r = bzo_deflate_reset_params(s->zo, level, window_bits, mem_level, strategy);
    if (r) {
        bzo_deflate_free(s->zo);
        free(s);
        *out = NULL;
        return result(r);
    }
    *out = s;
    return BPMD_R_OK;
}

int bpmd_deflate_stream_reset(bpmd_stream* s)
{
    if (!s || !s->is_deflate) return BPMD_R_INVALID_ARGUMENT;
    bzo_deflate_reset(s->zo);
    return BPMD_R_OK;
}

int bpmd_deflate_stream_write(bpmd_stream* s, bpmd_zparams* zs, int flush)
{
    if (!s || !s->is_deflate || !zs) return BPMD_R_INVALID_ARGUMENT;
    bzo_zparams b = to_bzo(zs);
    int r = bzo_deflate_write(s->zo, &b, flush);
    from_bzo(zs, &b);
    return result(r);
}

int bpmd_deflate_stream_params(bpmd_stream* s, bpmd_zparams* zs, int level, int strategy)
{
    if (!s || !s->is_deflate || !zs) return BPMD_R_INVALID_ARGUMENT;
    bzo_zparams b = to_bzo(zs);
    int r = bzo_deflate_params(s->zo, &b, level, strategy);
    from_bzo(zs, &b);
    return result(r);
}

int bpmd_deflate_stream_tune(bpmd_stream* s, int good, int lazy, int nice, int chain)
{
    if (!s || !s->is_deflate) return BPMD_R_INVALID_ARGUMENT;
    bzo_deflate_tune(s->zo, good, lazy, nice, chain);
    return BPMD_R_OK;
}

int bpmd_deflate_stream_pending(bpmd_stream* s, unsigned* value, int* bits)
{
    if (!s || !s->is_deflate) return BPMD_R_INVALID_ARGUMENT;
    return result(bzo_deflate_pending(s->zo, value, bits));
}

int bpmd_deflate_stream_prime(bpmd_stream* s, int bits, int value)
{
    if (!s || !s->is_deflate) return BPMD_R_INVALID_ARGUMENT;
    return result(bzo_deflate_prime(s->zo, bits, value));
}

int bpmd_inflate_stream_create(int window_bits, bpmd_stream** out)
{
    if (!out) return BPMD_R_INVALID_ARGUMENT;
    bpmd_stream* s = (bpmd_stream*)calloc(1, sizeof *s);
    s->zi = bzo_inflate_new();
    int r = bzo_inflate_reset(s->zi, window_bits);
    if (r) {
        bzo_inflate_free(s->zi);
        free(s);
        *out = NULL;
        return result(r);
    }
    *out = s;
    return BPMD_R_OK;
}

int bpmd_inflate_stream_reset(bpmd_stream* s, int window_bits)
{
    if (!s || s->is_deflate) return BPMD_R_INVALID_ARGUMENT;
    return result(bzo_inflate_reset(s->zi, window_bits));
}

int bpmd_inflate_stream_clear(bpmd_stream* s)
{
    if (!s || s->is_deflate) return BPMD_R_INVALID_ARGUMENT;
    bzo_inflate_clear(s->zi);
    return BPMD_R_OK;
}

int bpmd_inflate_stream_write(bpmd_stream* s, bpmd_zparams* zs, int flush)
{
    if (!s || s->is_deflate || !zs) return BPMD_R_INVALID_ARGUMENT;
    bzo_zparams b = to_bzo(zs);
    int r = bzo_inflate_write(s->zi, &b, flush);
    from_bzo(zs, &b);
    return result(r);
}

void bpmd_stream_destroy(bpmd_stream* s)
{
    if (!s) return;
    if (s->zo) bzo_deflate_free(s->zo);
    if (s->zi) bzo_inflate_free(s->zi);
    free(s);
}

/* the C ABI's init: the oracle needs no device */
int bpmd_init(void) { return BPMD_R_OK; }
