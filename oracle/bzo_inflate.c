/*
 * bzo_inflate.c -- CPU ORACLE (test infrastructure only, see bzo.h).
 *
 * Restates Beast's raw-DEFLATE decoder:
 *   state machine        include/boost/beast/zlib/detail/inflate_stream.ipp:74-535
 *   table construction   inflate_stream.ipp:551-863
 *   fixed tables         inflate_stream.ipp:865-930
 *   fast decode loop     inflate_stream.ipp:979-1113
 *   bit reservoir        include/boost/beast/zlib/detail/bitstream.hpp:49-194
 *   history window       include/boost/beast/zlib/detail/window.hpp:51-144
 */
#include "bzo.h"

#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------- tables */

/* A decode-table slot.  kind: 0 literal, 16+n base value with n extra bits,
 * 96 end-of-block, 64 invalid, 1..15 link to a second-level table of that
 * many index bits (val = offset of the sub-table from the root). */
typedef struct { uint8_t kind; uint8_t nbits; uint16_t val; } slot_t;

enum { LENS_ROOT = 9, DISTS_ROOT = 6, CODES_ROOT = 7 };
enum { ENOUGH_LENS = 852, ENOUGH_DISTS = 592, ENOUGH = ENOUGH_LENS + ENOUGH_DISTS };
enum { BUILD_CODES = 0, BUILD_LENS = 1, BUILD_DISTS = 2 };

/* RFC 1951 §3.2.5 length/distance bases.  The "kind" column is 16 + extra
 * bits; 64 marks symbols that may not appear (286/287 and 30/31). */
static const uint16_t len_base[31] = {
    3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31,
    35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258, 0, 0};
static const uint8_t len_kind[31] = {
    16, 16, 16, 16, 16, 16, 16, 16, 17, 17, 17, 17, 18, 18, 18, 18,
    19, 19, 19, 19, 20, 20, 20, 20, 21, 21, 21, 21, 16, 64, 64};
static const uint16_t dist_base[32] = {
    1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193,
    257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145,
    8193, 12289, 16385, 24577, 0, 0};
static const uint8_t dist_kind[32] = {
    16, 16, 16, 16, 17, 17, 18, 18, 19, 19, 20, 20, 21, 21, 22, 22,
    23, 23, 24, 24, 25, 25, 26, 26, 27, 27, 28, 28, 29, 29, 64, 64};

/* Canonical-Huffman table builder, same acceptance rules and the same
 * two-level layout as inflate_stream.ipp:551-863 (root size clamped to
 * [min,max] code length; over-subscribed codes rejected; incomplete codes
 * accepted only for a single 1-bit lens/dists code; an empty code yields a
 * two-entry table of invalid slots). */
static int build_table(int type, const uint16_t* lens, unsigned ncodes,
                       slot_t** cursor, unsigned* root_io, uint16_t* sorted)
{
    uint16_t cnt[16], first[16];
    unsigned i, lo, hi;
    for (i = 0; i < 16; ++i) cnt[i] = 0;
    for (i = 0; i < ncodes; ++i) cnt[lens[i]]++;

    unsigned root = *root_io;
    hi = 15;
    while (hi >= 1 && cnt[hi] == 0) --hi;
    if (root > hi) root = hi;
    if (hi == 0) {
        slot_t bad = {64, 1, 0};
        (*cursor)[0] = bad;
        (*cursor)[1] = bad;
        *cursor += 2;
        *root_io = 1;
        return BZO_OK;
    }
    lo = 1;
    while (lo < hi && cnt[lo] == 0) ++lo;
    if (root < lo) root = lo;

    int avail = 1;
    for (i = 1; i <= 15; ++i) {
        avail = (avail << 1) - cnt[i];
        if (avail < 0) return BZO_OVER_SUBSCRIBED_LENGTH;
    }
    if (avail > 0 && (type == BUILD_CODES || hi != 1))
        return BZO_INCOMPLETE_LENGTH_SET;

    first[1] = 0;
    for (i = 1; i < 15; ++i) first[i + 1] = (uint16_t)(first[i] + cnt[i]);
    for (i = 0; i < ncodes; ++i)
        if (lens[i] != 0) sorted[first[lens[i]]++] = (uint16_t)i;

    /* symbols below 'special' are plain values; at or above use the tables */
    const uint16_t* vbase = NULL;
    const uint8_t* vkind = NULL;
    unsigned special;
    if (type == BUILD_CODES) { special = 20; }
    else if (type == BUILD_LENS) { vbase = len_base; vkind = len_kind; special = 257; }
    else { vbase = dist_base; vkind = dist_kind; special = 0; }

    slot_t* base_tab = *cursor;   /* root table */
    slot_t* tab = base_tab;       /* table currently being filled */
    unsigned code = 0;            /* current code, bit-reversed counter */
    unsigned k = 0;               /* index into sorted[] */
    unsigned len = lo;            /* current code length */
    unsigned idx_bits = root;     /* index bits of the current table */
    unsigned skip = 0;            /* low code bits consumed by the root */
    unsigned cur_low = ~0u;       /* root index of the open sub-table */
    unsigned total = 1u << root;  /* slots allocated so far */
    const unsigned low_mask = total - 1;

    if ((type == BUILD_LENS && total > ENOUGH_LENS) ||
        (type == BUILD_DISTS && total > ENOUGH_DISTS))
        return BZO_THROW_LOGIC_ERROR;

    for (;;) {
        slot_t s;
        unsigned sym = sorted[k];
        s.nbits = (uint8_t)(len - skip);
        if (sym + 1u < special) { s.kind = 0; s.val = (uint16_t)sym; }
        else if (sym >= special) { s.kind = vkind[sym - special]; s.val = vbase[sym - special]; }
        else { s.kind = 96; s.val = 0; }      /* end of block */

        /* replicate across every index whose low (len-skip) bits match */
        unsigned step = 1u << (len - skip);
        unsigned span = 1u << idx_bits;
        unsigned next_span = span;
        do {
            span -= step;
            tab[(code >> skip) + span] = s;
        } while (span != 0);

        /* advance the bit-reversed code */
        unsigned bit = 1u << (len - 1);
        while (code & bit) bit >>= 1;
        if (bit != 0) { code &= bit - 1; code += bit; }
        else code = 0;

        ++k;
        if (--cnt[len] == 0) {
            if (len == hi) break;
            len = lens[sorted[k]];
        }

        if (len > root && (code & low_mask) != cur_low) {
            if (skip == 0) skip = root;
            tab += next_span;
            /* size the sub-table to hold every remaining code sharing it */
            idx_bits = len - skip;
            int room = 1 << idx_bits;
            while (idx_bits + skip < hi) {
                room -= cnt[idx_bits + skip];
                if (room <= 0) break;
                ++idx_bits;
                room <<= 1;
            }
            total += 1u << idx_bits;
            if ((type == BUILD_LENS && total > ENOUGH_LENS) ||
                (type == BUILD_DISTS && total > ENOUGH_DISTS))
                return BZO_THROW_LOGIC_ERROR;
            cur_low = code & low_mask;
            base_tab[cur_low].kind = (uint8_t)idx_bits;
            base_tab[cur_low].nbits = (uint8_t)root;
            base_tab[cur_low].val = (uint16_t)(tab - base_tab);
        }
    }
    if (code != 0) {              /* incomplete 1-bit code: one invalid slot */
        slot_t bad;
        bad.kind = 64;
        bad.nbits = (uint8_t)(len - skip);
        bad.val = 0;
        tab[code] = bad;
    }
    *cursor += total;
    *root_io = root;
    return BZO_OK;
}

/* fixed-Huffman tables, inflate_stream.ipp:865-920 */
static slot_t fixed_lens[512];
static slot_t fixed_dists[32];
static unsigned fixed_lens_root, fixed_dists_root;
static int fixed_ready = 0;

static void build_fixed(void)
{
    uint16_t lens[320];
    uint16_t sorted[320];
    unsigned i;
    if (fixed_ready) return;
    for (i = 0; i < 144; ++i) lens[i] = 8;
    for (; i < 256; ++i) lens[i] = 9;
    for (; i < 280; ++i) lens[i] = 7;
    for (; i < 288; ++i) lens[i] = 8;
    slot_t* p = fixed_lens;
    fixed_lens_root = 9;
    build_table(BUILD_LENS, lens, 288, &p, &fixed_lens_root, sorted);
    /* symbols 286/287 are reachable through the fixed code: mark invalid */
    fixed_lens[99].kind = 64;
    fixed_lens[227].kind = 64;
    fixed_lens[355].kind = 64;
    fixed_lens[483].kind = 64;
    for (i = 0; i < 32; ++i) lens[i] = 5;
    p = fixed_dists;
    fixed_dists_root = 5;
    build_table(BUILD_DISTS, lens, 32, &p, &fixed_dists_root, sorted);
    fixed_ready = 1;
}

/* ------------------------------------------------------------ bit source */

typedef struct { uint32_t v; unsigned n; } bits_t;

/* ensure at least need bits; false when input runs out (bitstream.hpp fill) */
static int bits_need(bits_t* b, unsigned need, const uint8_t** in, const uint8_t* end)
{
    while (b->n < need) {
        if (*in == end) return 0;
        b->v += (uint32_t)(*(*in)++) << b->n;
        b->n += 8;
    }
    return 1;
}
static unsigned bits_peek(const bits_t* b, unsigned n) { return (unsigned)(b->v & ((1ull << n) - 1)); }
static void bits_drop(bits_t* b, unsigned n) { b->v >>= n; b->n -= n; }
static unsigned bits_take(bits_t* b, unsigned n)
{
    unsigned r = bits_peek(b, n);
    bits_drop(b, n);
    return r;
}

/* ---------------------------------------------------------------- window */

typedef struct {
    uint8_t* buf;
    unsigned pos, fill, cap, wbits;
} hist_t;

static void hist_reset(hist_t* w, unsigned wbits)
{
    if (w->wbits != wbits) {
        free(w->buf);
        w->buf = NULL;
        w->wbits = wbits;
        w->cap = 1u << wbits;
    }
    w->pos = 0;
    w->fill = 0;
}
static void hist_read(const hist_t* w, uint8_t* out, unsigned back, unsigned n)
{
    if (w->pos >= w->fill) { memcpy(out, w->buf + (w->pos - back), n); return; }
    unsigned i = (w->pos - back + w->cap) % w->cap;
    unsigned m = w->cap - i;
    if (n <= m) { memcpy(out, w->buf + i, n); return; }
    memcpy(out, w->buf + i, m);
    memcpy(out + m, w->buf, n - m);
}
static void hist_write(hist_t* w, const uint8_t* in, size_t n)
{
    if (!w->buf) w->buf = (uint8_t*)malloc(w->cap);
    if (n >= w->cap) {
        w->pos = 0;
        w->fill = w->cap;
        memcpy(w->buf, in + (n - w->cap), w->cap);
        return;
    }
    if (w->pos + n <= w->cap) {
        memcpy(w->buf + w->pos, in, n);
        w->fill = (w->fill >= w->cap - n) ? w->cap : (unsigned)(w->fill + n);
        w->pos = (unsigned)((w->pos + n) % w->cap);
        return;
    }
    unsigned m = w->cap - w->pos;
    memcpy(w->buf + w->pos, in, m);
    w->pos = (unsigned)(n - m);
    memcpy(w->buf, in + m, w->pos);
    w->fill = w->cap;
}

/* --------------------------------------------------------------- decoder */

enum {
    M_HEAD, M_TYPE, M_TYPEDO, M_STORED, M_COPY_, M_COPY, M_TABLE, M_LENLENS,
    M_CODELENS, M_LEN_, M_LEN, M_LENEXT, M_DIST, M_DISTEXT, M_MATCH, M_LIT,
    M_CHECK, M_DONE, M_BAD, M_SYNC
};

struct bzo_inflater {
    hist_t hist;
    bits_t bits;
    int mode;
    int last;
    unsigned length, offset, extra, was;
    unsigned nlen, ndist, ncode, have;
    const slot_t* lcode;
    const slot_t* dcode;
    unsigned lroot, droot;
    slot_t* next;
    uint16_t lens[320];
    uint16_t work[288];
    slot_t codes[ENOUGH];
    int back;
    size_t last_out;   /* bytes written by the latest write(), even when the
                          reference returns without publishing them in zs */
};

bzo_inflater* bzo_inflate_new(void)
{
    bzo_inflater* s = (bzo_inflater*)calloc(1, sizeof(bzo_inflater));
    build_fixed();
    bzo_inflate_reset(s, 15);
    return s;
}

void bzo_inflate_free(bzo_inflater* s)
{
    if (!s) return;
    free(s->hist.buf);
    free(s);
}

/* inflate_stream.ipp:55-71 */
int bzo_inflate_reset(bzo_inflater* s, int wbits)
{
    if (wbits < 8 || wbits > 15) return BZO_THROW_DOMAIN_ERROR;
    hist_reset(&s->hist, (unsigned)wbits);
    s->bits.v = 0;
    s->bits.n = 0;
    s->mode = M_HEAD;
    s->last = 0;
    s->lcode = s->codes;
    s->dcode = s->codes;
    s->next = s->codes;
    s->back = -1;
    return BZO_OK;
}

/* inflate_stream.ipp:49-53: intentionally empty */
void bzo_inflate_clear(bzo_inflater* s) { (void)s; }

typedef struct {
    const uint8_t* in0; const uint8_t* in; const uint8_t* in_end;
    uint8_t* out0; uint8_t* out; uint8_t* out_end;
} cursor_t;

/* inflate_stream.ipp:979-1113; returns error or 0 */
static int decode_fast(bzo_inflater* s, cursor_t* c)
{
    const uint8_t* in_last = c->in + (c->in_end - c->in - 5);
    uint8_t* out_last = c->out + (c->out_end - c->out - 257);
    const unsigned lmask = (1u << s->lroot) - 1;
    const unsigned dmask = (1u << s->droot) - 1;
    bits_t* b = &s->bits;
    int err = 0;

    do {
        if (b->n < 15) {
            b->v += (uint32_t)(*c->in++) << b->n; b->n += 8;
            b->v += (uint32_t)(*c->in++) << b->n; b->n += 8;
        }
        const slot_t* e = &s->lcode[b->v & lmask];
        for (;;) {
            bits_drop(b, e->nbits);
            unsigned k = e->kind;
            if (k == 0) { *c->out++ = (uint8_t)e->val; break; }
            if (k & 16) {
                unsigned len = e->val;
                k &= 15;
                if (k) {
                    if (b->n < k) { b->v += (uint32_t)(*c->in++) << b->n; b->n += 8; }
                    len += b->v & ((1u << k) - 1);
                    bits_drop(b, k);
                }
                if (b->n < 15) {
                    b->v += (uint32_t)(*c->in++) << b->n; b->n += 8;
                    b->v += (uint32_t)(*c->in++) << b->n; b->n += 8;
                }
                const slot_t* d = &s->dcode[b->v & dmask];
                for (;;) {
                    bits_drop(b, d->nbits);
                    unsigned dk = d->kind;
                    if (dk & 16) {
                        unsigned dist = d->val;
                        dk &= 15;
                        if (b->n < dk) {
                            b->v += (uint32_t)(*c->in++) << b->n; b->n += 8;
                            if (b->n < dk) { b->v += (uint32_t)(*c->in++) << b->n; b->n += 8; }
                        }
                        dist += b->v & ((1u << dk) - 1);
                        bits_drop(b, dk);
                        unsigned made = (unsigned)(c->out - c->out0);
                        if (dist > made) {
                            unsigned back = dist - made;
                            if (back > s->hist.fill) { err = BZO_INVALID_DISTANCE; goto bad; }
                            unsigned n = len < back ? len : back;
                            hist_read(&s->hist, c->out, back, n);
                            c->out += n;
                            len -= n;
                        }
                        if (len > 0) {
                            const uint8_t* from = c->out - dist;
                            size_t room = (size_t)(c->out_end - c->out);
                            unsigned n = len < room ? len : (unsigned)room;
                            while (n--) *c->out++ = *from++;
                        }
                        break;
                    } else if ((dk & 64) == 0) {
                        d = &s->dcode[d->val + (b->v & ((1u << dk) - 1))];
                        continue;
                    } else { err = BZO_INVALID_DISTANCE_CODE; goto bad; }
                }
                break;
            } else if ((k & 64) == 0) {
                e = &s->lcode[e->val + (b->v & ((1u << k) - 1))];
                continue;
            } else if (k & 32) {
                s->mode = M_TYPE;
                goto out;
            } else { err = BZO_INVALID_LITERAL_LENGTH; goto bad; }
        }
    } while (c->in < in_last && c->out < out_last);
out:
    /* give back whole unused bytes (bitstream.hpp rewind) */
    c->in -= b->n >> 3;
    b->n &= 7;
    b->v &= (1u << b->n) - 1;
    return 0;
bad:
    s->mode = M_BAD;
    c->in -= b->n >> 3;
    b->n &= 7;
    b->v &= (1u << b->n) - 1;
    return err;
}

static const uint8_t clen_order[19] = {
    16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

/* Error exits -- err() (inflate_stream.ipp:120-125), the table errors at
 * :336-349 and inflate_fast's at :362-369 -- return without the done()
 * bookkeeping: zs and the window are left untouched. */
static int quiet_fail(bzo_inflater* s, cursor_t* c, int err)
{
    s->mode = M_BAD;
    s->last_out = (size_t)(c->out - c->out0);
    return err;
}

/* done() lambda, inflate_stream.ipp:89-119 */
static int finish_call(bzo_inflater* s, bzo_zparams* zs, cursor_t* c, int flush, int ec)
{
    size_t used_out = (size_t)(c->out - c->out0);
    s->last_out = used_out;
    size_t used_in = (size_t)(c->in - c->in0);
    if (used_out && s->mode < M_BAD && (s->mode < M_CHECK || flush != BZO_FLUSH_FINISH))
        hist_write(&s->hist, c->out0, used_out);
    zs->next_in = c->in;
    zs->avail_in = (size_t)(c->in_end - c->in);
    zs->next_out = c->out;
    zs->avail_out = (size_t)(c->out_end - c->out);
    zs->total_in += used_in;
    zs->total_out += used_out;
    zs->data_type = (int)s->bits.n + (s->last ? 64 : 0) + (s->mode == M_TYPE ? 128 : 0) +
                    (s->mode == M_LEN_ || s->mode == M_COPY_ ? 256 : 0);
    if (((!used_in && !used_out) || flush == BZO_FLUSH_FINISH) && !ec)
        ec = BZO_NEED_BUFFERS;
    return ec;
}

/* inflate_stream.ipp:74-535 */
int bzo_inflate_write(bzo_inflater* s, bzo_zparams* zs, int flush)
{
    s->last_out = 0;
    cursor_t c;
    c.in0 = c.in = zs->next_in;
    c.in_end = zs->next_in + zs->avail_in;
    c.out0 = c.out = zs->next_out;
    c.out_end = zs->next_out + zs->avail_out;
    bits_t* b = &s->bits;
    int ec = 0;

#define NEED(n) do { if (!bits_need(b, (n), &c.in, c.in_end)) return finish_call(s, zs, &c, flush, ec); } while (0)
/* err() (inflate_stream.ipp:120-125) sets BAD and returns without done():
 * z_params are not advanced, though the bytes are in the caller's buffer */
#define FAIL(e) return quiet_fail(s, &c, (e))

    if (s->mode == M_TYPE) s->mode = M_TYPEDO;
    for (;;) {
        switch (s->mode) {
        case M_HEAD:
            s->mode = M_TYPEDO;
            break;
        case M_TYPE:
            if (flush == BZO_FLUSH_BLOCK || flush == BZO_FLUSH_TREES)
                return finish_call(s, zs, &c, flush, ec);
            /* fall through */
        case M_TYPEDO: {
            if (s->last) {
                bits_drop(b, b->n % 8);
                s->mode = M_CHECK;
                break;
            }
            NEED(3);
            s->last = bits_take(b, 1) != 0;
            switch (bits_take(b, 2)) {
            case 0: s->mode = M_STORED; break;
            case 1:
                s->lcode = fixed_lens; s->lroot = fixed_lens_root;
                s->dcode = fixed_dists; s->droot = fixed_dists_root;
                s->mode = M_LEN_;
                if (flush == BZO_FLUSH_TREES) return finish_call(s, zs, &c, flush, ec);
                break;
            case 2: s->mode = M_TABLE; break;
            default: FAIL(BZO_INVALID_BLOCK_TYPE);
            }
            break;
        }
        case M_STORED: {
            bits_drop(b, b->n % 8);
            NEED(32);
            uint32_t v = (uint32_t)bits_peek(b, 32);
            s->length = v & 0xffff;
            if (s->length != ((v >> 16) ^ 0xffff)) FAIL(BZO_INVALID_STORED_LENGTH);
            b->v = 0;
            b->n = 0;
            s->mode = M_COPY_;
            if (flush == BZO_FLUSH_TREES) return finish_call(s, zs, &c, flush, ec);
        }   /* fall through */
        case M_COPY_:
            s->mode = M_COPY;
            /* fall through */
        case M_COPY: {
            size_t n = s->length;
            if (n == 0) { s->mode = M_TYPE; break; }
            if (n > (size_t)(c.in_end - c.in)) n = (size_t)(c.in_end - c.in);
            if (n > (size_t)(c.out_end - c.out)) n = (size_t)(c.out_end - c.out);
            if (n == 0) return finish_call(s, zs, &c, flush, ec);
            memcpy(c.out, c.in, n);
            c.in += n;
            c.out += n;
            s->length -= (unsigned)n;
            break;
        }
        case M_TABLE:
            NEED(14);
            s->nlen = bits_take(b, 5) + 257;
            s->ndist = bits_take(b, 5) + 1;
            s->ncode = bits_take(b, 4) + 4;
            if (s->nlen > 286 || s->ndist > 30) FAIL(BZO_TOO_MANY_SYMBOLS);
            s->have = 0;
            s->mode = M_LENLENS;
            /* fall through */
        case M_LENLENS: {
            while (s->have < s->ncode) {
                NEED(3);
                s->lens[clen_order[s->have++]] = (uint16_t)bits_take(b, 3);
            }
            while (s->have < 19) s->lens[clen_order[s->have++]] = 0;
            s->next = s->codes;
            s->lcode = s->next;
            s->lroot = CODES_ROOT;
            int r = build_table(BUILD_CODES, s->lens, 19, &s->next, &s->lroot, s->work);
            if (r) {
                ec = r;
                s->mode = M_BAD;
                if (r < 0) return r;
                break;
            }
            s->have = 0;
            s->mode = M_CODELENS;
        }   /* fall through */
        case M_CODELENS: {
            while (s->have < s->nlen + s->ndist) {
                NEED(s->lroot);
                const slot_t* e = &s->lcode[bits_peek(b, s->lroot)];
                if (e->val < 16) {
                    bits_drop(b, e->nbits);
                    s->lens[s->have++] = e->val;
                } else {
                    unsigned rep, fillv;
                    if (e->val == 16) {
                        NEED(e->nbits + 2u);
                        bits_drop(b, e->nbits);
                        if (s->have == 0) FAIL(BZO_INVALID_BIT_LENGTH_REPEAT);
                        rep = 3 + bits_take(b, 2);
                        fillv = s->lens[s->have - 1];
                    } else if (e->val == 17) {
                        NEED(e->nbits + 3u);
                        bits_drop(b, e->nbits);
                        rep = 3 + bits_take(b, 3);
                        fillv = 0;
                    } else {
                        NEED(e->nbits + 7u);
                        bits_drop(b, e->nbits);
                        rep = 11 + bits_take(b, 7);
                        fillv = 0;
                    }
                    if (s->have + rep > s->nlen + s->ndist) FAIL(BZO_INVALID_BIT_LENGTH_REPEAT);
                    while (rep--) s->lens[s->have++] = (uint16_t)fillv;
                }
            }
            if (s->mode == M_BAD) break;
            if (s->lens[256] == 0) FAIL(BZO_MISSING_EOB);
            s->next = s->codes;
            s->lcode = s->next;
            s->lroot = LENS_ROOT;
            int r = build_table(BUILD_LENS, s->lens, s->nlen, &s->next, &s->lroot, s->work);
            if (r) return quiet_fail(s, &c, r);
            s->dcode = s->next;
            s->droot = DISTS_ROOT;
            r = build_table(BUILD_DISTS, s->lens + s->nlen, s->ndist, &s->next, &s->droot, s->work);
            if (r) return quiet_fail(s, &c, r);
            s->mode = M_LEN_;
            if (flush == BZO_FLUSH_TREES) return finish_call(s, zs, &c, flush, ec);
        }   /* fall through */
        case M_LEN_:
            s->mode = M_LEN;
            /* fall through */
        case M_LEN: {
            if (c.in_end - c.in >= 6 && c.out_end - c.out >= 258) {
                int r = decode_fast(s, &c);
                if (r) return quiet_fail(s, &c, r);
                if (s->mode == M_TYPE) s->back = -1;
                break;
            }
            NEED(s->lroot);
            s->back = 0;
            const slot_t* e = &s->lcode[bits_peek(b, s->lroot)];
            if (e->kind && (e->kind & 0xf0) == 0) {
                const slot_t* link = e;
                NEED((unsigned)link->nbits + link->kind);
                e = &s->lcode[link->val + (bits_peek(b, link->nbits + link->kind) >> link->nbits)];
                bits_drop(b, link->nbits + e->nbits);
                s->back += link->nbits + e->nbits;
            } else {
                bits_drop(b, e->nbits);
                s->back += e->nbits;
            }
            s->length = e->val;
            if (e->kind == 0) { s->mode = M_LIT; break; }
            if (e->kind & 32) { s->back = -1; s->mode = M_TYPE; break; }
            if (e->kind & 64) FAIL(BZO_INVALID_LITERAL_LENGTH);
            s->extra = e->kind & 15;
            s->mode = M_LENEXT;
        }   /* fall through */
        case M_LENEXT:
            if (s->extra) {
                NEED(s->extra);
                s->length += bits_take(b, s->extra);
                s->back += (int)s->extra;
            }
            s->was = s->length;
            s->mode = M_DIST;
            /* fall through */
        case M_DIST: {
            NEED(s->droot);
            const slot_t* e = &s->dcode[bits_peek(b, s->droot)];
            if ((e->kind & 0xf0) == 0) {
                const slot_t* link = e;
                NEED((unsigned)link->nbits + link->kind);
                e = &s->dcode[link->val + (bits_peek(b, link->nbits + link->kind) >> link->nbits)];
                bits_drop(b, link->nbits + e->nbits);
                s->back += link->nbits + e->nbits;
            } else {
                bits_drop(b, e->nbits);
                s->back += e->nbits;
            }
            if (e->kind & 64) FAIL(BZO_INVALID_DISTANCE_CODE);
            s->offset = e->val;
            s->extra = e->kind & 15;
            s->mode = M_DISTEXT;
        }   /* fall through */
        case M_DISTEXT:
            if (s->extra) {
                NEED(s->extra);
                s->offset += bits_take(b, s->extra);
                s->back += (int)s->extra;
            }
            s->mode = M_MATCH;
            /* fall through */
        case M_MATCH: {
            if (c.out == c.out_end) return finish_call(s, zs, &c, flush, ec);
            size_t made = (size_t)(c.out - c.out0);
            if (s->offset > made) {
                unsigned back = (unsigned)(uint16_t)(s->offset - made);
                if (back > s->hist.fill) FAIL(BZO_INVALID_DISTANCE);
                size_t n = s->length;
                if (n > back) n = back;
                if (n > (size_t)(c.out_end - c.out)) n = (size_t)(c.out_end - c.out);
                hist_read(&s->hist, c.out, back, (unsigned)n);
                c.out += n;
                s->length -= (unsigned)n;
            } else {
                const uint8_t* from = c.out - s->offset;
                size_t n = s->length;
                if (n > (size_t)(c.out_end - c.out)) n = (size_t)(c.out_end - c.out);
                s->length -= (unsigned)n;
                while (n--) *c.out++ = *from++;
            }
            if (s->length == 0) s->mode = M_LEN;
            break;
        }
        case M_LIT:
            if (c.out == c.out_end) return finish_call(s, zs, &c, flush, ec);
            *c.out++ = (uint8_t)s->length;
            s->mode = M_LEN;
            break;
        case M_CHECK:
            s->mode = M_DONE;
            /* fall through */
        case M_DONE:
            ec = BZO_END_OF_STREAM;
            return finish_call(s, zs, &c, flush, ec);
        case M_BAD:
            return finish_call(s, zs, &c, flush, ec);
        default:
            return BZO_THROW_LOGIC_ERROR;
        }
    }
#undef NEED
#undef FAIL
}

size_t bzo_inflate_last_out(const bzo_inflater* s) { return s->last_out; }
