/*
 * synth.c -- seeded synthetic WebSocket payload generators for the benches
 * and tests (SURVEY.md §8(d) "Synthetic inputs").  Host-only C, no oracle
 * code.  Every message i is generated independently from the xorshift64*
 * state S ^ (i * 0x9E3779B97F4A7C15), so shards on different ranks produce
 * identical bytes for the same global message index.
 *
 * kinds:
 *   0 JSON-like text: objects drawn from a 32-key vocabulary with integer,
 *     decimal and short-string values, truncated to the message size (C1-C4)
 *   1 corpus1: runs of 1..5 repeats over a 62-character alphabet (the shape
 *     of test/bench/zlib/inflate_stream.cpp:28-48)
 *   2 corpus2: uniformly random bytes (inflate_stream.cpp:50-60)
 *   3 low-compressibility binary: per 64-byte unit, 7/8 random bytes and 1/8
 *     copies of an earlier 16..64-byte span within 32 KiB (C5)
 *   4 zeros
 */
#include <stdint.h>
#include <math.h>
#include <string.h>

static inline uint64_t xs_next(uint64_t* s)
{
    uint64_t x = *s;
    x ^= x >> 12;
    x ^= x << 25;
    x ^= x >> 27;
    *s = x;
    return x * 0x2545F4914F6CDD1DULL;
}

static uint64_t seed_for(uint64_t seed, uint64_t i)
{
    uint64_t s = seed ^ (i * 0x9E3779B97F4A7C15ULL);
    if (s == 0) s = 0x9E3779B97F4A7C15ULL;
    /* decorrelate nearby seeds */
    for (int k = 0; k < 4; ++k) xs_next(&s);
    return s;
}

static const char* const keys[32] = {
    "id", "type", "user", "name", "email", "created_at", "updated_at", "status",
    "price", "quantity", "currency", "tags", "score", "rank", "latitude", "longitude",
    "session", "event", "payload", "version", "region", "channel", "seq", "timestamp",
    "active", "count", "ratio", "message", "source", "target", "level", "op"};
static const char* const words[24] = {
    "alpha", "bravo", "charlie", "delta", "echo", "foxtrot", "golf", "hotel",
    "ok", "error", "pending", "done", "EUR", "USD", "buy", "sell",
    "eu-west", "us-east", "ap-south", "trade", "quote", "book", "ticker", "heartbeat"};

static size_t put_str(char* dst, size_t cap, size_t pos, const char* s)
{
    while (*s && pos < cap) dst[pos++] = *s++;
    return pos;
}
static size_t put_uint(char* dst, size_t cap, size_t pos, uint64_t v)
{
    char tmp[24];
    int n = 0;
    do { tmp[n++] = (char)('0' + v % 10); v /= 10; } while (v);
    while (n && pos < cap) dst[pos++] = tmp[--n];
    return pos;
}

static void gen_json(uint8_t* out, size_t n, uint64_t* s)
{
    char* d = (char*)out;
    size_t p = 0;
    while (p < n) {
        p = put_str(d, n, p, p == 0 ? "{" : ",\n{");
        unsigned fields = 3 + (unsigned)(xs_next(s) % 7);
        for (unsigned f = 0; f < fields && p < n; ++f) {
            uint64_t r = xs_next(s);
            if (f) p = put_str(d, n, p, ", ");
            p = put_str(d, n, p, "\"");
            p = put_str(d, n, p, keys[r & 31]);
            p = put_str(d, n, p, "\": ");
            switch ((r >> 5) & 3) {
            case 0: p = put_uint(d, n, p, (r >> 8) % 100000); break;
            case 1:
                p = put_uint(d, n, p, (r >> 8) % 1000);
                p = put_str(d, n, p, ".");
                p = put_uint(d, n, p, (r >> 20) % 100);
                break;
            case 2:
                p = put_str(d, n, p, "\"");
                p = put_str(d, n, p, words[(r >> 8) % 24]);
                if ((r >> 14) & 1) { p = put_str(d, n, p, "-"); p = put_uint(d, n, p, (r >> 16) % 1000); }
                p = put_str(d, n, p, "\"");
                break;
            default: p = put_str(d, n, p, ((r >> 8) & 1) ? "true" : "null"); break;
            }
        }
        p = put_str(d, n, p, "}");
    }
}

static void gen_corpus1(uint8_t* out, size_t n, uint64_t* s)
{
    static const char alpha[] = "0123456789ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz";
    size_t p = 0;
    while (p < n) {
        uint64_t r = xs_next(s);
        unsigned rep = 1 + (unsigned)(r % 5);
        char c = alpha[(r >> 8) % 62];
        while (rep-- && p < n) out[p++] = (uint8_t)c;
    }
}

static void gen_random(uint8_t* out, size_t n, uint64_t* s)
{
    size_t p = 0;
    while (p + 8 <= n) {
        uint64_t r = xs_next(s);
        memcpy(out + p, &r, 8);
        p += 8;
    }
    if (p < n) {
        uint64_t r = xs_next(s);
        memcpy(out + p, &r, n - p);
    }
}

static void gen_binary(uint8_t* out, size_t n, uint64_t* s)
{
    size_t p = 0;
    while (p < n) {
        size_t unit = n - p < 64 ? n - p : 64;
        uint64_t r = xs_next(s);
        if ((r & 7) == 0 && p >= 64) {
            size_t span = 16 + (size_t)((r >> 3) % 49);
            if (span > unit) span = unit;
            size_t window = p < 32768 ? p : 32768;
            size_t back = span + (size_t)((r >> 16) % (window - span + 1));
            if (back > p) back = p;
            for (size_t k = 0; k < span; ++k) out[p + k] = out[p - back + k];
            gen_random(out + p + span, unit - span, s);
        } else {
            gen_random(out + p, unit, s);
        }
        p += unit;
    }
}

/* Fill messages [first, first+count) of a batch whose message i has
 * length len[i] at out + off[i].  Global index = first + local index. */
int bpmd_synth_fill(int kind, uint64_t seed, uint64_t first, uint32_t count,
                    const uint64_t* off, const uint32_t* len, uint8_t* out)
{
    for (uint32_t i = 0; i < count; ++i) {
        uint64_t s = seed_for(seed, first + i);
        uint8_t* dst = out + off[i];
        size_t n = len[i];
        switch (kind) {
        case 0: gen_json(dst, n, &s); break;
        case 1: gen_corpus1(dst, n, &s); break;
        case 2: gen_random(dst, n, &s); break;
        case 3: gen_binary(dst, n, &s); break;
        case 4: memset(dst, 0, n); break;
        default: return -1;
        }
    }
    return 0;
}

/* Zipf message sizes for C4: rank r in [1,256], P(r) ~ r^-1.1, size 256*r. */
int bpmd_synth_zipf_sizes(uint64_t seed, uint64_t first, uint32_t count, uint32_t* len)
{
    static double cdf[256];
    static int ready = 0;
    if (!ready) {
        double acc = 0.0;
        for (int r = 1; r <= 256; ++r) {
            double w = pow((double)r, -1.1);
            acc += w;
            cdf[r - 1] = acc;
        }
        for (int r = 0; r < 256; ++r) cdf[r] /= acc;
        ready = 1;
    }
    for (uint32_t i = 0; i < count; ++i) {
        uint64_t s = seed_for(seed ^ 0x5A5A5A5AULL, first + i);
        double u = (double)(xs_next(&s) >> 11) * (1.0 / 9007199254740992.0);
        int lo = 0, hi = 255;
        while (lo < hi) {
            int mid = (lo + hi) / 2;
            if (cdf[mid] < u) lo = mid + 1; else hi = mid;
        }
        len[i] = 256u * (uint32_t)(lo + 1);
    }
    return 0;
}
