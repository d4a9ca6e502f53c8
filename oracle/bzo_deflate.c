/*
 * bzo_deflate.c -- CPU ORACLE (test infrastructure only, see bzo.h).
 *
 * Restates Beast's raw-DEFLATE encoder (a port of zlib deflate.c/trees.c):
 *   parameters / reset     include/boost/beast/zlib/detail/deflate_stream.ipp:227-265
 *   upper bound            deflate_stream.ipp:283-305
 *   write() state machine  deflate_stream.ipp:357-499
 *   init / lm_init         deflate_stream.ipp:595-718
 *   Huffman trees          deflate_stream.ipp:115-141, 744-1180
 *   block emission         deflate_stream.ipp:1184-1518
 *   window / matching      deflate_stream.ipp:1520-1844
 *   parsers                deflate_stream.ipp:1856-2324 (stored/fast/slow/rle/huff)
 *   level table            include/boost/beast/zlib/detail/deflate_stream.hpp:571-590
 */
#include "bzo.h"

#include <stdlib.h>
#include <string.h>

enum {
    N_LIT = 256, N_LENCODE = 29, N_LCODES = N_LIT + 1 + N_LENCODE, N_DCODES = 30,
    N_BLCODES = 19, HEAP_N = 2 * N_LCODES + 1, MAXBITS = 15, MAXBLBITS = 7,
    MINM = 3, MAXM = 258, EOB = 256, TOO_FAR = 4096,
    LOOKAHEAD_MIN = MAXM + MINM + 1, WIN_INIT = MAXM,
    REP_3_6 = 16, REPZ_3_10 = 17, REPZ_11_138 = 18
};

/* ---------------------------------------------------------- static tables */

static const uint8_t xbits_len[N_LENCODE] = {
    0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
static const uint8_t xbits_dist[N_DCODES] = {
    0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
static const uint8_t xbits_bl[N_BLCODES] = {
    0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 2, 3, 7};
static const uint8_t bl_rank[N_BLCODES] = {
    16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

/* tree node: f = frequency, later the (bit-reversed) code; l = parent, later
 * the code length */
typedef struct { uint16_t f; uint16_t l; } node_t;

static node_t stat_ltree[N_LCODES + 2];
static node_t stat_dtree[N_DCODES];
static uint8_t lcode_of[MAXM - MINM + 1];   /* match length-3 -> length code */
static uint8_t dcode_of[512];               /* distance-1 -> distance code */
static uint8_t lbase_of[N_LENCODE];
static uint16_t dbase_of[N_DCODES];
static int tables_ready = 0;

static unsigned reverse_bits(unsigned code, int len)
{
    unsigned r = 0;
    do { r |= code & 1; code >>= 1; r <<= 1; } while (--len > 0);
    return r >> 1;
}

/* deflate_stream.ipp:115-141 */
static void assign_codes(node_t* tree, int max_code, const uint16_t* bl_count)
{
    uint16_t next[MAXBITS + 1];
    unsigned code = 0;
    for (int bits = 1; bits <= MAXBITS; ++bits) {
        code = (code + bl_count[bits - 1]) << 1;
        next[bits] = (uint16_t)code;
    }
    for (int n = 0; n <= max_code; ++n) {
        int len = tree[n].l;
        if (len == 0) continue;
        tree[n].f = (uint16_t)reverse_bits(next[len]++, len);
    }
}

/* deflate_stream.ipp:143-225 */
static void init_tables(void)
{
    if (tables_ready) return;
    unsigned length = 0;
    for (int code = 0; code < N_LENCODE - 1; ++code) {
        lbase_of[code] = (uint8_t)length;
        for (unsigned n = 0; n < (1u << xbits_len[code]); ++n) lcode_of[length++] = (uint8_t)code;
    }
    lcode_of[255] = N_LENCODE - 1;
    unsigned dist = 0;
    int code;
    for (code = 0; code < 16; ++code) {
        dbase_of[code] = (uint16_t)dist;
        for (unsigned n = 0; n < (1u << xbits_dist[code]); ++n) dcode_of[dist++] = (uint8_t)code;
    }
    dist >>= 7;
    for (; code < N_DCODES; ++code) {
        dbase_of[code] = (uint16_t)(dist << 7);
        for (unsigned n = 0; n < (1u << (xbits_dist[code] - 7)); ++n) dcode_of[256 + dist++] = (uint8_t)code;
    }
    uint16_t bl_count[MAXBITS + 1];
    memset(bl_count, 0, sizeof bl_count);
    unsigned n = 0;
    while (n <= 143) stat_ltree[n++].l = 8;
    bl_count[8] += 144;
    while (n <= 255) stat_ltree[n++].l = 9;
    bl_count[9] += 112;
    while (n <= 279) stat_ltree[n++].l = 7;
    bl_count[7] += 24;
    while (n <= 287) stat_ltree[n++].l = 8;
    bl_count[8] += 8;
    assign_codes(stat_ltree, N_LCODES + 1, bl_count);
    for (n = 0; n < N_DCODES; ++n) {
        stat_dtree[n].l = 5;
        stat_dtree[n].f = (uint16_t)reverse_bits(n, 5);
    }
    tables_ready = 1;
}

static unsigned dist_code(unsigned d) { return d < 256 ? dcode_of[d] : dcode_of[256 + (d >> 7)]; }

/* ----------------------------------------------------------------- state */

typedef struct {
    node_t* dyn;
    const node_t* stat;       /* static tree or NULL */
    const uint8_t* xbits;
    int xbase, elems, maxlen;
    int max_code;
} tdesc_t;

typedef struct { uint16_t good, lazy, nice, chain; int parser; } level_t;
enum { P_STORED, P_FAST, P_SLOW };
/* deflate_stream.hpp:571-590 */
static const level_t levels[10] = {
    {0, 0, 0, 0, P_STORED}, {4, 4, 8, 4, P_FAST}, {4, 5, 16, 8, P_FAST},
    {4, 6, 32, 32, P_FAST}, {4, 4, 16, 16, P_SLOW}, {8, 16, 32, 32, P_SLOW},
    {8, 16, 128, 128, P_SLOW}, {8, 32, 128, 256, P_SLOW},
    {32, 128, 258, 1024, P_SLOW}, {32, 258, 258, 4096, P_SLOW}};

enum { BS_NEED_MORE, BS_BLOCK_DONE, BS_FINISH_STARTED, BS_FINISH_DONE };
enum { ST_BUSY = 0, ST_FINISH = 1 };

struct bzo_deflater {
    /* parameters */
    int level, wbits, hbits, strategy;
    unsigned lit_bufsize;
    int inited;
    int status;
    int last_flush;            /* -1 == not set (boost::none) */

    /* buffers */
    uint8_t* mem; size_t mem_size;
    uint8_t* window; uint16_t* prev; uint16_t* head;
    uint8_t* pend; uint32_t pend_size; uint8_t* pend_out; uint32_t pending;
    uint8_t* syms; unsigned sym_next, sym_end;

    unsigned w_size, w_mask, window_size;
    unsigned hash_size, hash_mask, hash_shift, ins_h;
    uint32_t high_water;

    long block_start;
    unsigned strstart, match_start, lookahead, prev_length, match_length, prev_match;
    int match_available;
    unsigned insert;
    unsigned good, lazy, nice, chain;

    /* trees */
    node_t dyn_ltree[HEAP_N];
    node_t dyn_dtree[2 * N_DCODES + 1];
    node_t bl_tree[2 * N_BLCODES + 1];
    tdesc_t ldesc, ddesc, bldesc;
    uint16_t bl_count[MAXBITS + 1];
    int heap[2 * N_LCODES + 1];
    int heap_len, heap_max;
    uint8_t depth[2 * N_LCODES + 1];
    uint32_t opt_len, static_len;
    unsigned matches;

    uint16_t bi_buf;
    int bi_valid;
};

static unsigned max_dist(const bzo_deflater* s) { return s->w_size - LOOKAHEAD_MIN; }

/* --------------------------------------------------------------- bit sink */

static void put_byte(bzo_deflater* s, uint8_t c) { s->pend[s->pending++] = c; }
static void put_short(bzo_deflater* s, unsigned w)
{
    put_byte(s, (uint8_t)(w & 0xff));
    put_byte(s, (uint8_t)((w >> 8) & 0xff));
}
/* 16-bit bit buffer, LSB first (detail/deflate_stream.hpp:436-474) */
static void send_bits(bzo_deflater* s, unsigned value, int length)
{
    if (s->bi_valid > 16 - length) {
        s->bi_buf |= (uint16_t)(value << s->bi_valid);
        put_short(s, s->bi_buf);
        s->bi_buf = (uint16_t)(value >> (16 - s->bi_valid));
        s->bi_valid += length - 16;
    } else {
        s->bi_buf |= (uint16_t)(value << s->bi_valid);
        s->bi_valid += length;
    }
}
#define SEND_CODE(s, c, tree) send_bits((s), (tree)[c].f, (tree)[c].l)

static void bi_windup(bzo_deflater* s)
{
    if (s->bi_valid > 8) put_short(s, s->bi_buf);
    else if (s->bi_valid > 0) put_byte(s, (uint8_t)s->bi_buf);
    s->bi_buf = 0;
    s->bi_valid = 0;
}
static void bi_flush(bzo_deflater* s)
{
    if (s->bi_valid == 16) {
        put_short(s, s->bi_buf);
        s->bi_buf = 0;
        s->bi_valid = 0;
    } else if (s->bi_valid >= 8) {
        put_byte(s, (uint8_t)s->bi_buf);
        s->bi_buf >>= 8;
        s->bi_valid -= 8;
    }
}

/* ------------------------------------------------------------ tree build */

static void reset_block(bzo_deflater* s)
{
    for (int n = 0; n < N_LCODES; ++n) s->dyn_ltree[n].f = 0;
    for (int n = 0; n < N_DCODES; ++n) s->dyn_dtree[n].f = 0;
    for (int n = 0; n < N_BLCODES; ++n) s->bl_tree[n].f = 0;
    s->dyn_ltree[EOB].f = 1;
    s->opt_len = 0;
    s->static_len = 0;
    s->sym_next = 0;
    s->matches = 0;
}

static int node_less(const bzo_deflater* s, const node_t* t, int a, int b)
{
    return t[a].f < t[b].f || (t[a].f == t[b].f && s->depth[a] <= s->depth[b]);
}

static void sift_down(bzo_deflater* s, const node_t* t, int k)
{
    int v = s->heap[k];
    int j = k << 1;
    while (j <= s->heap_len) {
        if (j < s->heap_len && node_less(s, t, s->heap[j + 1], s->heap[j])) ++j;
        if (node_less(s, t, v, s->heap[j])) break;
        s->heap[k] = s->heap[j];
        k = j;
        j <<= 1;
    }
    s->heap[k] = v;
}

/* deflate_stream.ipp:786-873 (length assignment with depth limiting) */
static void assign_lengths(bzo_deflater* s, tdesc_t* d)
{
    node_t* t = d->dyn;
    int h, n, m, bits, overflow = 0;
    for (bits = 0; bits <= MAXBITS; ++bits) s->bl_count[bits] = 0;
    t[s->heap[s->heap_max]].l = 0;
    for (h = s->heap_max + 1; h < HEAP_N; ++h) {
        n = s->heap[h];
        bits = t[t[n].l].l + 1;
        if (bits > d->maxlen) { bits = d->maxlen; ++overflow; }
        t[n].l = (uint16_t)bits;
        if (n > d->max_code) continue;
        s->bl_count[bits]++;
        int xb = (n >= d->xbase) ? d->xbits[n - d->xbase] : 0;
        uint16_t f = t[n].f;
        s->opt_len += (uint32_t)f * (uint32_t)(bits + xb);
        if (d->stat) s->static_len += (uint32_t)f * (uint32_t)(d->stat[n].l + xb);
    }
    if (overflow == 0) return;
    do {
        bits = d->maxlen - 1;
        while (s->bl_count[bits] == 0) --bits;
        s->bl_count[bits]--;
        s->bl_count[bits + 1] += 2;
        s->bl_count[d->maxlen]--;
        overflow -= 2;
    } while (overflow > 0);
    for (bits = d->maxlen; bits != 0; --bits) {
        n = s->bl_count[bits];
        while (n != 0) {
            m = s->heap[--h];
            if (m > d->max_code) continue;
            if ((unsigned)t[m].l != (unsigned)bits) {
                s->opt_len += (uint32_t)(((long)bits - (long)t[m].l) * (long)t[m].f);
                t[m].l = (uint16_t)bits;
            }
            --n;
        }
    }
}

/* deflate_stream.ipp:888-973 */
static void make_tree(bzo_deflater* s, tdesc_t* d)
{
    node_t* t = d->dyn;
    int n, m, node, max_code = -1;
    s->heap_len = 0;
    s->heap_max = HEAP_N;
    for (n = 0; n < d->elems; ++n) {
        if (t[n].f != 0) {
            s->heap[++s->heap_len] = max_code = n;
            s->depth[n] = 0;
        } else {
            t[n].l = 0;
        }
    }
    while (s->heap_len < 2) {
        node = s->heap[++s->heap_len] = (max_code < 2 ? ++max_code : 0);
        t[node].f = 1;
        s->depth[node] = 0;
        s->opt_len--;
        if (d->stat) s->static_len -= d->stat[node].l;
    }
    d->max_code = max_code;
    for (n = s->heap_len / 2; n >= 1; --n) sift_down(s, t, n);
    node = d->elems;
    do {
        n = s->heap[1];
        s->heap[1] = s->heap[s->heap_len--];
        sift_down(s, t, 1);
        m = s->heap[1];
        s->heap[--s->heap_max] = n;
        s->heap[--s->heap_max] = m;
        t[node].f = (uint16_t)(t[n].f + t[m].f);
        s->depth[node] = (uint8_t)((s->depth[n] >= s->depth[m] ? s->depth[n] : s->depth[m]) + 1);
        t[n].l = t[m].l = (uint16_t)node;
        s->heap[1] = node++;
        sift_down(s, t, 1);
    } while (s->heap_len >= 2);
    s->heap[--s->heap_max] = s->heap[1];
    assign_lengths(s, d);
    assign_codes(t, max_code, s->bl_count);
}

/* deflate_stream.ipp:978-1042: count code-length symbols */
static void scan_lengths(bzo_deflater* s, node_t* t, int max_code)
{
    int prevlen = -1, curlen, nextlen = t[0].l, count = 0, max_count = 7, min_count = 4;
    if (nextlen == 0) { max_count = 138; min_count = 3; }
    t[max_code + 1].l = 0xffff;
    for (int n = 0; n <= max_code; ++n) {
        curlen = nextlen;
        nextlen = t[n + 1].l;
        if (++count < max_count && curlen == nextlen) continue;
        if (count < min_count) s->bl_tree[curlen].f = (uint16_t)(s->bl_tree[curlen].f + count);
        else if (curlen != 0) {
            if (curlen != prevlen) s->bl_tree[curlen].f++;
            s->bl_tree[REP_3_6].f++;
        } else if (count <= 10) s->bl_tree[REPZ_3_10].f++;
        else s->bl_tree[REPZ_11_138].f++;
        count = 0;
        prevlen = curlen;
        if (nextlen == 0) { max_count = 138; min_count = 3; }
        else if (curlen == nextlen) { max_count = 6; min_count = 3; }
        else { max_count = 7; min_count = 4; }
    }
}

/* deflate_stream.ipp:1046-1110: emit run-length coded code lengths */
static void emit_lengths(bzo_deflater* s, node_t* t, int max_code)
{
    int prevlen = -1, curlen, nextlen = t[0].l, count = 0, max_count = 7, min_count = 4;
    if (nextlen == 0) { max_count = 138; min_count = 3; }
    for (int n = 0; n <= max_code; ++n) {
        curlen = nextlen;
        nextlen = t[n + 1].l;
        if (++count < max_count && curlen == nextlen) continue;
        if (count < min_count) {
            do { SEND_CODE(s, curlen, s->bl_tree); } while (--count != 0);
        } else if (curlen != 0) {
            if (curlen != prevlen) { SEND_CODE(s, curlen, s->bl_tree); --count; }
            SEND_CODE(s, REP_3_6, s->bl_tree);
            send_bits(s, (unsigned)(count - 3), 2);
        } else if (count <= 10) {
            SEND_CODE(s, REPZ_3_10, s->bl_tree);
            send_bits(s, (unsigned)(count - 3), 3);
        } else {
            SEND_CODE(s, REPZ_11_138, s->bl_tree);
            send_bits(s, (unsigned)(count - 11), 7);
        }
        count = 0;
        prevlen = curlen;
        if (nextlen == 0) { max_count = 138; min_count = 3; }
        else if (curlen == nextlen) { max_count = 6; min_count = 3; }
        else { max_count = 7; min_count = 4; }
    }
}

/* deflate_stream.ipp:1127-1155 */
static int make_bl_tree(bzo_deflater* s)
{
    int maxi;
    scan_lengths(s, s->dyn_ltree, s->ldesc.max_code);
    scan_lengths(s, s->dyn_dtree, s->ddesc.max_code);
    make_tree(s, &s->bldesc);
    for (maxi = N_BLCODES - 1; maxi >= 3; --maxi)
        if (s->bl_tree[bl_rank[maxi]].l != 0) break;
    s->opt_len += 3 * ((uint32_t)maxi + 1) + 5 + 5 + 4;
    return maxi;
}

/* deflate_stream.ipp:1164-1180 */
static void send_header_trees(bzo_deflater* s, int lcodes, int dcodes, int blcodes)
{
    send_bits(s, (unsigned)(lcodes - 257), 5);
    send_bits(s, (unsigned)(dcodes - 1), 5);
    send_bits(s, (unsigned)(blcodes - 4), 4);
    for (int r = 0; r < blcodes; ++r) send_bits(s, s->bl_tree[bl_rank[r]].l, 3);
    emit_lengths(s, s->dyn_ltree, lcodes - 1);
    emit_lengths(s, s->dyn_dtree, dcodes - 1);
}

/* deflate_stream.ipp:1184-1238 */
static void emit_symbols(bzo_deflater* s, const node_t* lt, const node_t* dt)
{
    unsigned sx = 0;
    if (s->sym_next != 0) {
        do {
            unsigned dist = s->syms[sx++];
            dist += (unsigned)s->syms[sx++] << 8;
            int lc = s->syms[sx++];
            if (dist == 0) {
                SEND_CODE(s, lc, lt);
            } else {
                unsigned code = lcode_of[lc];
                SEND_CODE(s, code + N_LIT + 1, lt);
                int extra = xbits_len[code];
                if (extra != 0) send_bits(s, (unsigned)(lc - lbase_of[code]), extra);
                --dist;
                code = dist_code(dist);
                SEND_CODE(s, code, dt);
                extra = xbits_dist[code];
                if (extra != 0) send_bits(s, dist - dbase_of[code], extra);
            }
        } while (sx < s->sym_next);
    }
    SEND_CODE(s, EOB, lt);
}

/* deflate_stream.ipp:1252-1280 */
static int guess_text(const bzo_deflater* s)
{
    unsigned long mask = 0xf3ffc07fUL;
    int n;
    for (n = 0; n <= 31; ++n, mask >>= 1)
        if ((mask & 1) && s->dyn_ltree[n].f != 0) return 0;
    if (s->dyn_ltree[9].f != 0 || s->dyn_ltree[10].f != 0 || s->dyn_ltree[13].f != 0) return 1;
    for (n = 32; n < N_LIT; ++n)
        if (s->dyn_ltree[n].f != 0) return 1;
    return 0;
}

/* deflate_stream.ipp:1325-1394 */
static void stored_block(bzo_deflater* s, const uint8_t* buf, uint32_t len, int last)
{
    send_bits(s, (0u << 1) + (unsigned)last, 3);
    bi_windup(s);
    put_short(s, (uint16_t)len);
    put_short(s, (uint16_t)~len);
    if (buf) memcpy(s->pend + s->pending, buf, len);
    s->pending += len;
}
static void align_block(bzo_deflater* s)
{
    send_bits(s, 1u << 1, 3);
    SEND_CODE(s, EOB, stat_ltree);
    bi_flush(s);
}

/* deflate_stream.ipp:1425-1518 (Beast's ordering of the fixed-strategy test) */
static void close_block(bzo_deflater* s, bzo_zparams* zs, const uint8_t* buf, uint32_t stored_len, int last)
{
    uint32_t opt_lenb, static_lenb;
    int max_blindex = 0;
    if (s->level > 0) {
        if (zs->data_type == 2) zs->data_type = guess_text(s);
        make_tree(s, &s->ldesc);
        make_tree(s, &s->ddesc);
        max_blindex = make_bl_tree(s);
        opt_lenb = (s->opt_len + 3 + 7) >> 3;
        static_lenb = (s->static_len + 3 + 7) >> 3;
        if (static_lenb <= opt_lenb) opt_lenb = static_lenb;
    } else {
        opt_lenb = static_lenb = stored_len + 5;
    }
    if (stored_len + 4 <= opt_lenb && buf != NULL) {
        stored_block(s, buf, stored_len, last);
    } else if (s->strategy == BZO_STRATEGY_FIXED || static_lenb == opt_lenb) {
        send_bits(s, (1u << 1) + (unsigned)last, 3);
        emit_symbols(s, stat_ltree, stat_dtree);
    } else {
        send_bits(s, (2u << 1) + (unsigned)last, 3);
        send_header_trees(s, s->ldesc.max_code + 1, s->ddesc.max_code + 1, max_blindex + 1);
        emit_symbols(s, s->dyn_ltree, s->dyn_dtree);
    }
    reset_block(s);
    if (last) bi_windup(s);
}

static int tally_lit(bzo_deflater* s, uint8_t c)
{
    s->syms[s->sym_next++] = 0;
    s->syms[s->sym_next++] = 0;
    s->syms[s->sym_next++] = c;
    s->dyn_ltree[c].f++;
    return s->sym_next == s->sym_end;
}
static int tally_match(bzo_deflater* s, unsigned dist, unsigned lenm3)
{
    s->syms[s->sym_next++] = (uint8_t)(dist & 0xff);
    s->syms[s->sym_next++] = (uint8_t)(dist >> 8);
    s->syms[s->sym_next++] = (uint8_t)lenm3;
    --dist;
    s->dyn_ltree[lcode_of[lenm3] + N_LIT + 1].f++;
    s->dyn_dtree[dist_code(dist)].f++;
    return s->sym_next == s->sym_end;
}

/* --------------------------------------------------------- output pump */

/* deflate_stream.ipp:1676-1694 */
static void drain(bzo_deflater* s, bzo_zparams* zs)
{
    bi_flush(s);
    size_t len = s->pending;
    if (len > zs->avail_out) len = zs->avail_out;
    if (len == 0) return;
    memcpy(zs->next_out, s->pend_out, len);
    zs->next_out += len;
    s->pend_out += len;
    zs->total_out += len;
    zs->avail_out -= len;
    s->pending -= (uint32_t)len;
    if (s->pending == 0) s->pend_out = s->pend;
}

/* deflate_stream.ipp:1699-1711 */
static void flush_block(bzo_deflater* s, bzo_zparams* zs, int last)
{
    close_block(s, zs, s->block_start >= 0L ? s->window + (unsigned)s->block_start : NULL,
                (uint32_t)((long)s->strstart - s->block_start), last);
    s->block_start = (long)s->strstart;
    drain(s, zs);
}

/* deflate_stream.ipp:1719-1734 */
static unsigned read_input(bzo_deflater* s, bzo_zparams* zs, uint8_t* dst, unsigned size)
{
    (void)s;
    size_t len = zs->avail_in < size ? zs->avail_in : size;
    if (len == 0) return 0;
    zs->avail_in -= len;
    memcpy(dst, zs->next_in, len);
    zs->next_in += len;
    zs->total_in += len;
    return (unsigned)len;
}

static void hash_step(const bzo_deflater* s, unsigned* h, uint8_t c)
{
    *h = ((*h << s->hash_shift) ^ c) & s->hash_mask;
}
/* insert window[str..str+2]; returns the previous chain head */
static unsigned hash_insert(bzo_deflater* s, unsigned str)
{
    hash_step(s, &s->ins_h, s->window[str + (MINM - 1)]);
    unsigned h = s->head[s->ins_h];
    s->prev[str & s->w_mask] = (uint16_t)h;
    s->head[s->ins_h] = (uint16_t)str;
    return h;
}
static void clear_heads(bzo_deflater* s) { memset(s->head, 0, (size_t)s->hash_size * sizeof(uint16_t)); }

/* deflate_stream.ipp:1520-1669 */
static void refill(bzo_deflater* s, bzo_zparams* zs)
{
    unsigned n, m, more;
    uint16_t* p;
    unsigned wsize = s->w_size;
    do {
        more = s->window_size - s->lookahead - s->strstart;
        if (s->strstart >= wsize + max_dist(s)) {
            memcpy(s->window, s->window + wsize, wsize);
            s->match_start -= wsize;
            s->strstart -= wsize;
            s->block_start -= (long)wsize;
            if (s->insert > s->strstart) s->insert = s->strstart;
            n = s->hash_size;
            p = &s->head[n];
            do { m = *--p; *p = (uint16_t)(m >= wsize ? m - wsize : 0); } while (--n);
            n = wsize;
            p = &s->prev[n];
            do { m = *--p; *p = (uint16_t)(m >= wsize ? m - wsize : 0); } while (--n);
            more += wsize;
        }
        if (zs->avail_in == 0) break;
        n = read_input(s, zs, s->window + s->strstart + s->lookahead, more);
        s->lookahead += n;
        if (s->lookahead + s->insert >= MINM) {
            unsigned str = s->strstart - s->insert;
            s->ins_h = s->window[str];
            hash_step(s, &s->ins_h, s->window[str + 1]);
            while (s->insert) {
                hash_step(s, &s->ins_h, s->window[str + MINM - 1]);
                s->prev[str & s->w_mask] = s->head[s->ins_h];
                s->head[s->ins_h] = (uint16_t)str;
                ++str;
                --s->insert;
                if (s->lookahead + s->insert < MINM) break;
            }
        }
    } while (s->lookahead < LOOKAHEAD_MIN && zs->avail_in != 0);

    if (s->high_water < s->window_size) {
        uint32_t curr = s->strstart + s->lookahead;
        uint32_t winit;
        if (s->high_water < curr) {
            winit = s->window_size - curr;
            if (winit > WIN_INIT) winit = WIN_INIT;
            memset(s->window + curr, 0, winit);
            s->high_water = curr + winit;
        } else if (s->high_water < curr + WIN_INIT) {
            winit = curr + WIN_INIT - s->high_water;
            if (winit > s->window_size - s->high_water) winit = s->window_size - s->high_water;
            memset(s->window + s->high_water, 0, winit);
            s->high_water += winit;
        }
    }
}

/* deflate_stream.ipp:1747-1844 */
static unsigned longest(bzo_deflater* s, unsigned cur)
{
    unsigned chain = s->chain;
    uint8_t* scan = s->window + s->strstart;
    uint8_t* match;
    int len;
    int best = (int)s->prev_length;
    int nice = (int)s->nice;
    unsigned limit = s->strstart > max_dist(s) ? s->strstart - max_dist(s) : 0;
    const uint16_t* prev = s->prev;
    unsigned wmask = s->w_mask;
    uint8_t* strend = s->window + s->strstart + MAXM;
    uint8_t end1 = scan[best - 1];
    uint8_t end0 = scan[best];

    if (s->prev_length >= s->good) chain >>= 2;
    if ((unsigned)nice > s->lookahead) nice = (int)s->lookahead;
    do {
        match = s->window + cur;
        if (match[best] != end0 || match[best - 1] != end1 || *match != *scan || *++match != scan[1])
            continue;
        scan += 2;
        ++match;
        do {
        } while (*++scan == *++match && *++scan == *++match && *++scan == *++match &&
                 *++scan == *++match && *++scan == *++match && *++scan == *++match &&
                 *++scan == *++match && *++scan == *++match && scan < strend);
        len = MAXM - (int)(strend - scan);
        scan = strend - MAXM;
        if (len > best) {
            s->match_start = cur;
            best = len;
            if (len >= nice) break;
            end1 = scan[best - 1];
            end0 = scan[best];
        }
    } while ((cur = prev[cur & wmask]) > limit && --chain != 0);
    if ((unsigned)best <= s->lookahead) return (unsigned)best;
    return s->lookahead;
}

/* --------------------------------------------------------------- parsers */

#define EMIT_BLOCK(s, zs, last)                                               \
    do {                                                                      \
        flush_block((s), (zs), (last));                                       \
        if ((zs)->avail_out == 0) return (last) ? BS_FINISH_STARTED : BS_NEED_MORE; \
    } while (0)

/* deflate_stream.ipp:1856-1924 (the pre-1.2.11 stored algorithm) */
static int parse_stored(bzo_deflater* s, bzo_zparams* zs, int flush)
{
    uint32_t max_block = 0xffff;
    if (max_block > s->pend_size - 5) max_block = s->pend_size - 5;
    for (;;) {
        if (s->lookahead <= 1) {
            refill(s, zs);
            if (s->lookahead == 0 && flush == BZO_FLUSH_NONE) return BS_NEED_MORE;
            if (s->lookahead == 0) break;
        }
        s->strstart += s->lookahead;
        s->lookahead = 0;
        uint32_t max_start = (uint32_t)s->block_start + max_block;
        if (s->strstart == 0 || (uint32_t)s->strstart >= max_start) {
            s->lookahead = (unsigned)(s->strstart - max_start);
            s->strstart = (unsigned)max_start;
            EMIT_BLOCK(s, zs, 0);
        }
        if (s->strstart - (unsigned)s->block_start >= max_dist(s)) EMIT_BLOCK(s, zs, 0);
    }
    s->insert = 0;
    if (flush == BZO_FLUSH_FINISH) {
        EMIT_BLOCK(s, zs, 1);
        return BS_FINISH_DONE;
    }
    if ((long)s->strstart > s->block_start) EMIT_BLOCK(s, zs, 0);
    return BS_BLOCK_DONE;
}

/* deflate_stream.ipp:1932-2039 (greedy, levels 1-3) */
static int parse_fast(bzo_deflater* s, bzo_zparams* zs, int flush)
{
    unsigned head;
    int bflush;
    for (;;) {
        if (s->lookahead < LOOKAHEAD_MIN) {
            refill(s, zs);
            if (s->lookahead < LOOKAHEAD_MIN && flush == BZO_FLUSH_NONE) return BS_NEED_MORE;
            if (s->lookahead == 0) break;
        }
        head = 0;
        if (s->lookahead >= MINM) head = hash_insert(s, s->strstart);
        if (head != 0 && s->strstart - head <= max_dist(s)) s->match_length = longest(s, head);
        if (s->match_length >= MINM) {
            bflush = tally_match(s, s->strstart - s->match_start, s->match_length - MINM);
            s->lookahead -= s->match_length;
            if (s->match_length <= s->lazy && s->lookahead >= MINM) {
                s->match_length--;
                do {
                    s->strstart++;
                    head = hash_insert(s, s->strstart);
                } while (--s->match_length != 0);
                s->strstart++;
            } else {
                s->strstart += s->match_length;
                s->match_length = 0;
                s->ins_h = s->window[s->strstart];
                hash_step(s, &s->ins_h, s->window[s->strstart + 1]);
            }
        } else {
            bflush = tally_lit(s, s->window[s->strstart]);
            s->lookahead--;
            s->strstart++;
        }
        if (bflush) EMIT_BLOCK(s, zs, 0);
    }
    s->insert = s->strstart < MINM - 1 ? s->strstart : MINM - 1;
    if (flush == BZO_FLUSH_FINISH) {
        EMIT_BLOCK(s, zs, 1);
        return BS_FINISH_DONE;
    }
    if (s->sym_next) EMIT_BLOCK(s, zs, 0);
    return BS_BLOCK_DONE;
}

/* deflate_stream.ipp:2045-2184 (lazy evaluation, levels 4-9) */
static int parse_slow(bzo_deflater* s, bzo_zparams* zs, int flush)
{
    unsigned head;
    int bflush;
    for (;;) {
        if (s->lookahead < LOOKAHEAD_MIN) {
            refill(s, zs);
            if (s->lookahead < LOOKAHEAD_MIN && flush == BZO_FLUSH_NONE) return BS_NEED_MORE;
            if (s->lookahead == 0) break;
        }
        head = 0;
        if (s->lookahead >= MINM) head = hash_insert(s, s->strstart);
        s->prev_length = s->match_length;
        s->prev_match = s->match_start;
        s->match_length = MINM - 1;
        if (head != 0 && s->prev_length < s->lazy && s->strstart - head <= max_dist(s)) {
            s->match_length = longest(s, head);
            if (s->match_length <= 5 &&
                (s->strategy == BZO_STRATEGY_FILTERED ||
                 (s->match_length == MINM && s->strstart - s->match_start > TOO_FAR)))
                s->match_length = MINM - 1;
        }
        if (s->prev_length >= MINM && s->match_length <= s->prev_length) {
            unsigned max_insert = s->strstart + s->lookahead - MINM;
            bflush = tally_match(s, s->strstart - 1 - s->prev_match, s->prev_length - MINM);
            s->lookahead -= s->prev_length - 1;
            s->prev_length -= 2;
            do {
                if (++s->strstart <= max_insert) head = hash_insert(s, s->strstart);
            } while (--s->prev_length != 0);
            s->match_available = 0;
            s->match_length = MINM - 1;
            s->strstart++;
            if (bflush) EMIT_BLOCK(s, zs, 0);
        } else if (s->match_available) {
            bflush = tally_lit(s, s->window[s->strstart - 1]);
            if (bflush) flush_block(s, zs, 0);
            s->strstart++;
            s->lookahead--;
            if (zs->avail_out == 0) return BS_NEED_MORE;
        } else {
            s->match_available = 1;
            s->strstart++;
            s->lookahead--;
        }
    }
    if (s->match_available) {
        tally_lit(s, s->window[s->strstart - 1]);
        s->match_available = 0;
    }
    s->insert = s->strstart < MINM - 1 ? s->strstart : MINM - 1;
    if (flush == BZO_FLUSH_FINISH) {
        EMIT_BLOCK(s, zs, 1);
        return BS_FINISH_DONE;
    }
    if (s->sym_next) EMIT_BLOCK(s, zs, 0);
    return BS_BLOCK_DONE;
}

/* deflate_stream.ipp:2190-2270 */
static int parse_rle(bzo_deflater* s, bzo_zparams* zs, int flush)
{
    int bflush;
    for (;;) {
        if (s->lookahead <= MAXM) {
            refill(s, zs);
            if (s->lookahead <= MAXM && flush == BZO_FLUSH_NONE) return BS_NEED_MORE;
            if (s->lookahead == 0) break;
        }
        s->match_length = 0;
        if (s->lookahead >= MINM && s->strstart > 0) {
            uint8_t* scan = s->window + s->strstart - 1;
            uint8_t prev = *scan;
            if (prev == *++scan && prev == *++scan && prev == *++scan) {
                uint8_t* strend = s->window + s->strstart + MAXM;
                do {
                } while (prev == *++scan && prev == *++scan && prev == *++scan &&
                         prev == *++scan && prev == *++scan && prev == *++scan &&
                         prev == *++scan && prev == *++scan && scan < strend);
                s->match_length = MAXM - (unsigned)(strend - scan);
                if (s->match_length > s->lookahead) s->match_length = s->lookahead;
            }
        }
        if (s->match_length >= MINM) {
            bflush = tally_match(s, 1, s->match_length - MINM);
            s->lookahead -= s->match_length;
            s->strstart += s->match_length;
            s->match_length = 0;
        } else {
            bflush = tally_lit(s, s->window[s->strstart]);
            s->lookahead--;
            s->strstart++;
        }
        if (bflush) EMIT_BLOCK(s, zs, 0);
    }
    s->insert = 0;
    if (flush == BZO_FLUSH_FINISH) {
        EMIT_BLOCK(s, zs, 1);
        return BS_FINISH_DONE;
    }
    if (s->sym_next) EMIT_BLOCK(s, zs, 0);
    return BS_BLOCK_DONE;
}

/* deflate_stream.ipp:2276-2324 */
static int parse_huff(bzo_deflater* s, bzo_zparams* zs, int flush)
{
    int bflush;
    for (;;) {
        if (s->lookahead == 0) {
            refill(s, zs);
            if (s->lookahead == 0) {
                if (flush == BZO_FLUSH_NONE) return BS_NEED_MORE;
                break;
            }
        }
        s->match_length = 0;
        bflush = tally_lit(s, s->window[s->strstart]);
        s->lookahead--;
        s->strstart++;
        if (bflush) EMIT_BLOCK(s, zs, 0);
    }
    s->insert = 0;
    if (flush == BZO_FLUSH_FINISH) {
        EMIT_BLOCK(s, zs, 1);
        return BS_FINISH_DONE;
    }
    if (s->sym_next) EMIT_BLOCK(s, zs, 0);
    return BS_BLOCK_DONE;
}

/* ------------------------------------------------------------ public API */

bzo_deflater* bzo_deflate_new(void)
{
    bzo_deflater* s = (bzo_deflater*)calloc(1, sizeof(bzo_deflater));
    init_tables();
    bzo_deflate_reset_params(s, 6, 15, 9, BZO_STRATEGY_NORMAL);
    return s;
}

void bzo_deflate_free(bzo_deflater* s)
{
    if (!s) return;
    free(s->mem);
    free(s);
}

/* deflate_stream.ipp:227-265 */
int bzo_deflate_reset_params(bzo_deflater* s, int level, int wbits, int mem_level, int strategy)
{
    if (level == -1) level = 6;
    if (wbits == 8) wbits = 9;
    if (level < 0 || level > 9) return BZO_THROW_INVALID_ARGUMENT;
    if (wbits < 8 || wbits > 15) return BZO_THROW_INVALID_ARGUMENT;
    if (mem_level < 1 || mem_level > 9) return BZO_THROW_INVALID_ARGUMENT;
    s->wbits = wbits;
    s->hbits = mem_level + 7;
    s->lit_bufsize = 1u << (mem_level + 6);
    s->level = level;
    s->strategy = strategy;
    s->inited = 0;
    return BZO_OK;
}

void bzo_deflate_reset(bzo_deflater* s) { s->inited = 0; }

void bzo_deflate_clear(bzo_deflater* s)
{
    s->inited = 0;
    free(s->mem);
    s->mem = NULL;
    s->mem_size = 0;
}

size_t bzo_deflate_upper_bound(const bzo_deflater* s, size_t n)
{
    size_t complen = n + ((n + 7) >> 3) + ((n + 63) >> 6) + 5;
    if (s->wbits != 15 || s->hbits != 8 + 7) return complen;
    return n + (n >> 12) + (n >> 14) + (n >> 25) + 13 - 6;
}

size_t bzo_deflate_upper_bound_free(size_t n)
{
    return n + ((n + 7) >> 3) + ((n + 63) >> 6) + 11;
}

void bzo_deflate_tune(bzo_deflater* s, int good, int lazy, int nice, int chain)
{
    s->good = (unsigned)good;
    s->lazy = (unsigned)lazy;
    s->nice = (unsigned)nice;
    s->chain = (unsigned)chain;
}

/* deflate_stream.ipp:595-691 */
static void lazy_init(bzo_deflater* s)
{
    s->w_size = 1u << s->wbits;
    s->w_mask = s->w_size - 1;
    s->hash_size = 1u << s->hbits;
    s->hash_mask = s->hash_size - 1;
    s->hash_shift = (unsigned)((s->hbits + MINM - 1) / MINM);
    size_t nwin = (size_t)s->w_size * 2;
    size_t nprev = (size_t)s->w_size * sizeof(uint16_t);
    size_t nhead = (size_t)s->hash_size * sizeof(uint16_t);
    size_t npend = (size_t)s->lit_bufsize * (sizeof(uint16_t) + 2);
    size_t need = nwin + nprev + nhead + npend;
    if (!s->mem || s->mem_size != need) {
        free(s->mem);
        s->mem = (uint8_t*)malloc(need);
        s->mem_size = need;
    }
    s->window = s->mem;
    s->prev = (uint16_t*)(s->mem + nwin);
    memset(s->prev, 0, nprev);
    s->head = (uint16_t*)(s->mem + nwin + nprev);
    s->high_water = 0;
    s->pend = s->mem + nwin + nprev + nhead;
    s->pend_size = (uint32_t)s->lit_bufsize * 4;
    s->syms = s->pend + s->lit_bufsize;
    s->sym_end = (s->lit_bufsize - 1) * 3;
    s->pending = 0;
    s->pend_out = s->pend;
    s->status = ST_BUSY;
    s->last_flush = BZO_FLUSH_NONE;

    s->ldesc.dyn = s->dyn_ltree; s->ldesc.stat = stat_ltree; s->ldesc.xbits = xbits_len;
    s->ldesc.xbase = N_LIT + 1; s->ldesc.elems = N_LCODES; s->ldesc.maxlen = MAXBITS;
    s->ddesc.dyn = s->dyn_dtree; s->ddesc.stat = stat_dtree; s->ddesc.xbits = xbits_dist;
    s->ddesc.xbase = 0; s->ddesc.elems = N_DCODES; s->ddesc.maxlen = MAXBITS;
    s->bldesc.dyn = s->bl_tree; s->bldesc.stat = NULL; s->bldesc.xbits = xbits_bl;
    s->bldesc.xbase = 0; s->bldesc.elems = N_BLCODES; s->bldesc.maxlen = MAXBLBITS;
    s->bi_buf = 0;
    s->bi_valid = 0;
    reset_block(s);

    s->window_size = 2u * s->w_size;
    clear_heads(s);
    s->lazy = levels[s->level].lazy;
    s->good = levels[s->level].good;
    s->nice = levels[s->level].nice;
    s->chain = levels[s->level].chain;
    s->strstart = 0;
    s->block_start = 0L;
    s->lookahead = 0;
    s->insert = 0;
    s->match_length = s->prev_length = MINM - 1;
    s->match_available = 0;
    s->ins_h = 0;
    s->inited = 1;
}

static int run_parser(bzo_deflater* s, bzo_zparams* zs, int flush)
{
    if (s->strategy == BZO_STRATEGY_HUFFMAN) return parse_huff(s, zs, flush);
    if (s->strategy == BZO_STRATEGY_RLE) return parse_rle(s, zs, flush);
    switch (levels[s->level].parser) {
    case P_STORED: return parse_stored(s, zs, flush);
    case P_FAST: return parse_fast(s, zs, flush);
    default: return parse_slow(s, zs, flush);
    }
}

/* deflate_stream.ipp:357-499 */
int bzo_deflate_write(bzo_deflater* s, bzo_zparams* zs, int flush)
{
    if (!s->inited) lazy_init(s);
    if (zs->next_in == NULL && zs->avail_in != 0) return BZO_THROW_INVALID_ARGUMENT;
    if (zs->next_out == NULL || (s->status == ST_FINISH && flush != BZO_FLUSH_FINISH))
        return BZO_STREAM_ERROR;
    if (zs->avail_out == 0) return BZO_NEED_BUFFERS;

    int old_flush = s->last_flush;
    s->last_flush = flush;

    if (s->pending != 0) {
        drain(s, zs);
        if (zs->avail_out == 0) {
            s->last_flush = -1;
            return BZO_OK;
        }
    } else if (zs->avail_in == 0 && old_flush >= 0 && flush <= old_flush && flush != BZO_FLUSH_FINISH) {
        return BZO_NEED_BUFFERS;
    }
    if (s->status == ST_FINISH && zs->avail_in != 0) return BZO_NEED_BUFFERS;

    if (zs->avail_in != 0 || s->lookahead != 0 || (flush != BZO_FLUSH_NONE && s->status != ST_FINISH)) {
        int bs = run_parser(s, zs, flush);
        if (bs == BS_FINISH_STARTED || bs == BS_FINISH_DONE) s->status = ST_FINISH;
        if (bs == BS_NEED_MORE || bs == BS_FINISH_STARTED) {
            if (zs->avail_out == 0) s->last_flush = -1;
            return BZO_OK;
        }
        if (bs == BS_BLOCK_DONE) {
            if (flush == BZO_FLUSH_PARTIAL) {
                align_block(s);
            } else if (flush != BZO_FLUSH_BLOCK) {
                stored_block(s, NULL, 0, 0);
                if (flush == BZO_FLUSH_FULL) {
                    clear_heads(s);
                    if (s->lookahead == 0) {
                        s->strstart = 0;
                        s->block_start = 0L;
                        s->insert = 0;
                    }
                }
            }
            drain(s, zs);
            if (zs->avail_out == 0) {
                s->last_flush = -1;
                return BZO_OK;
            }
        }
    }
    if (flush == BZO_FLUSH_FINISH) return BZO_END_OF_STREAM;
    return BZO_OK;
}

/* deflate_stream.ipp:307-345 */
int bzo_deflate_params(bzo_deflater* s, bzo_zparams* zs, int level, int strategy)
{
    int ec = 0;
    if (level == -1) level = 6;
    if (level < 0 || level > 9) return BZO_STREAM_ERROR;
    int func = levels[s->level].parser;
    if ((strategy != s->strategy || func != levels[level].parser) && zs->total_in != 0) {
        ec = bzo_deflate_write(s, zs, BZO_FLUSH_BLOCK);
        if (ec == BZO_NEED_BUFFERS && s->pending == 0) ec = 0;
    }
    if (s->level != level) {
        s->level = level;
        s->lazy = levels[level].lazy;
        s->good = levels[level].good;
        s->nice = levels[level].nice;
        s->chain = levels[level].chain;
    }
    s->strategy = strategy;
    return ec;
}

/* deflate_stream.ipp:582-590 */
int bzo_deflate_pending(bzo_deflater* s, unsigned* bytes, int* bits)
{
    if (bytes) *bytes = s->pending;
    if (bits) *bits = s->bi_valid;
    return 0;
}

/* deflate_stream.ipp:556-580 */
int bzo_deflate_prime(bzo_deflater* s, int bits, int value)
{
    if (!s->inited) lazy_init(s);
    if ((uint8_t*)(s->syms) < s->pend_out + 2) return BZO_NEED_BUFFERS;
    do {
        int put = 16 - s->bi_valid;
        if (put > bits) put = bits;
        s->bi_buf |= (uint16_t)((value & ((1 << put) - 1)) << s->bi_valid);
        s->bi_valid += put;
        bi_flush(s);
        value >>= put;
        bits -= put;
    } while (bits);
    return 0;
}
