/*
 * bzo_frame.c -- CPU ORACLE (test infrastructure only; see bzo.h) for the
 * byte passes either side of the codec on Beast's frame path (SURVEY.md
 * §8(f) N1): masking and UTF-8 validation.
 *
 * Restates
 *   websocket/detail/mask.ipp:20-59            prepare_key, rol, mask_inplace
 *   websocket/detail/frame.hpp:134-175         write(DynamicBuffer&, frame_header)
 *   websocket/impl/write.hpp:463-545           the compressed-message frame loop
 *                                               (op / rsv1 on the first frame,
 *                                               cont after, fin on the last,
 *                                               a key per frame)
 *   websocket/detail/utf8_checker.ipp:22-324   utf8_checker::reset / finish /
 *                                               write, check_utf8
 * The checker is restated by its rules rather than its loops: the
 * reference's alignment loop, 8-byte ASCII loop and slow loop all apply
 * valid() to whole code points and differ only in speed; the tail keeps a
 * partial code point (needed(), :158-172) and answers with the fail-fast test
 * (:86-157), and the next write() completes it first (:176-206).
 *
 * Pinned by the expectations of the reference's own tests
 * (test/beast/websocket/utf8_checker.cpp, restated as data in
 * tests/utf8_cases.py), by CPython's UTF-8 decoder on random input
 * (tests/test_frame.py) and, for masking and frame headers, by the example
 * frames of RFC 6455 §5.7 and RFC 7692 §7.2.3 (tests/test_frame.py).
 */
#include <string.h>

#include "bzo.h"

unsigned bzo_mask(uint8_t* p, size_t n, uint32_t key, unsigned phase)
{
    /* prepare_key (mask.ipp:20-27): byte i of the key is key >> 8i; a prepared
     * key that already masked `phase` bytes is rotated by phase (rol,
     * :29-36).  mask_inplace XORs byte j with prepared[j % 4] and rotates by
     * the n % 4 bytes of a ragged tail (:38-59). */
    uint8_t k[4];
    for (unsigned i = 0; i < 4; ++i) k[i] = (uint8_t)(key >> (8 * ((i + phase) & 3u)));
    for (size_t j = 0; j < n; ++j) p[j] ^= k[j & 3];
    return (unsigned)((phase + n) & 3u);
}

/* needed() (utf8_checker.ipp:158-172): bytes of the code point a byte starts */
static size_t needed(uint8_t v)
{
    if (v < 0x80) return 1;
    if (v < 0xc0) return 0;
    if (v < 0xe0) return 2;
    if (v < 0xf0) return 3;
    if (v < 0xf8) return 4;
    return 0;
}

/* valid() (utf8_checker.ipp:43-85) as ranges: the lead's allowed values and
 * the range of its second byte (C0/C1 and E0 80..9F and F0 80..8F overlong,
 * ED A0..BF surrogates, F4 90..BF and F5..FF above U+10FFFF); the later
 * bytes are 80..BF.  starts_ok() tests the first k bytes of a code point, so
 * it is valid() for a whole one and !fail_fast() for a partial one. */
static int starts_ok(const uint8_t* p, size_t k)
{
    const uint8_t b = p[0];
    uint8_t lo = 0x80, hi = 0xbf;
    size_t len;
    if (b < 0x80) len = 1;
    else if (b < 0xc2) return 0;
    else if (b < 0xe0) len = 2;
    else if (b < 0xf0) {
        len = 3;
        if (b == 0xe0) lo = 0xa0;
        if (b == 0xed) hi = 0x9f;
    } else if (b < 0xf5) {
        len = 4;
        if (b == 0xf0) lo = 0x90;
        if (b == 0xf4) hi = 0x8f;
    } else
        return 0;
    for (size_t i = 1; i < k && i < len; ++i) {
        const uint8_t a = i == 1 ? lo : 0x80, z = i == 1 ? hi : 0xbf;
        if (p[i] < a || p[i] > z) return 0;
    }
    return 1;
}

void bzo_utf8_reset(bzo_utf8* u)
{
    u->need = 0;
    u->have = 0;
}

int bzo_utf8_finish(bzo_utf8* u)
{
    const int ok = u->need == 0;   /* utf8_checker.ipp:31-37 */
    bzo_utf8_reset(u);
    return ok;
}

int bzo_utf8_write(bzo_utf8* u, const uint8_t* in, size_t n)
{
    if (u->need) {
        /* complete the code point the previous write left open (:176-206) */
        const size_t k = n < u->need ? n : u->need;
        memcpy(u->cp + u->have, in, k);
        u->have += k;
        u->need -= k;
        in += k;
        n -= k;
        if (u->need) return starts_ok(u->cp, u->have);   /* still open: fail fast */
        if (!starts_ok(u->cp, u->have)) return 0;
        u->have = 0;
    }
    while (n) {
        const size_t need = needed(in[0]);
        if (!need) return 0;
        if (need > n) {
            /* the code point continues in the next write (:296-311) */
            memcpy(u->cp, in, n);
            u->have = n;
            u->need = need - n;
            return starts_ok(u->cp, u->have);
        }
        if (!starts_ok(in, need)) return 0;
        in += need;
        n -= need;
    }
    return 1;
}

int bzo_utf8_check(const uint8_t* p, size_t n)
{
    /* check_utf8 (:317-324), keeping write()'s verdict apart from finish()'s */
    bzo_utf8 u;
    bzo_utf8_reset(&u);
    if (!bzo_utf8_write(&u, p, n)) return 2;
    return bzo_utf8_finish(&u) ? 0 : 1;
}

int bzo_utf8_check_batch(const uint8_t* in, const uint64_t* off, const uint32_t* len, uint32_t n, int32_t* result)
{
    for (uint32_t i = 0; i < n; ++i) result[i] = bzo_utf8_check(in + off[i], len[i]);
    return 0;
}

/* frame.hpp:134-175: FIN | RSV1 | opcode, MASK | 7-bit length (126: 16-bit,
 * 127: 64-bit big-endian), then the key in little-endian byte order */
static size_t frame_header(uint8_t* b, int fin, int rsv1, unsigned op, int mask, uint64_t len, uint32_t key)
{
    size_t n;
    b[0] = (uint8_t)((fin ? 0x80u : 0u) | (rsv1 ? 0x40u : 0u) | (op & 15u));
    b[1] = mask ? 0x80u : 0u;
    if (len <= 125) {
        b[1] |= (uint8_t)len;
        n = 2;
    } else if (len <= 65535) {
        b[1] |= 126;
        b[2] = (uint8_t)(len >> 8);
        b[3] = (uint8_t)len;
        n = 4;
    } else {
        b[1] |= 127;
        for (int i = 0; i < 8; ++i) b[2 + i] = (uint8_t)(len >> (8 * (7 - i)));
        n = 10;
    }
    if (mask) {
        for (int i = 0; i < 4; ++i) b[n + i] = (uint8_t)(key >> (8 * i));
        n += 4;
    }
    return n;
}

size_t bzo_frame_wire_size(uint64_t n, uint64_t frame_max, int masked)
{
    const uint64_t frames = n == 0 ? 1 : (n + frame_max - 1) / frame_max;
    size_t total = (size_t)n;
    for (uint64_t f = 0; f < frames; ++f) {
        const uint64_t len = f + 1 < frames ? frame_max : n - f * frame_max;
        total += (len <= 125 ? 2 : len <= 65535 ? 4 : 10) + (masked ? 4 : 0);
    }
    return total;
}

/* write.hpp:463-545: the payload goes out in frames of at most frame_max
 * bytes (the wr_buf the deflater fills); the first frame carries the opcode
 * and RSV1 (a compressed message), later ones opcode cont (0) and no RSV1;
 * FIN on the last; a client masks each frame with its own key (keys[f]). */
size_t bzo_frame_write(uint8_t* out, const uint8_t* payload, uint64_t n, unsigned op, int rsv1, const uint32_t* keys,
                       uint64_t frame_max)
{
    const uint64_t frames = n == 0 ? 1 : (n + frame_max - 1) / frame_max;
    size_t w = 0;
    for (uint64_t f = 0; f < frames; ++f) {
        const uint64_t a = f * frame_max, len = f + 1 < frames ? frame_max : n - a;
        const uint32_t key = keys ? keys[f] : 0u;
        w += frame_header(out + w, f + 1 == frames, f == 0 && rsv1, f == 0 ? op : 0u, keys != NULL, len, key);
        memcpy(out + w, payload + a, (size_t)len);
        if (keys) bzo_mask(out + w, (size_t)len, key, 0);
        w += (size_t)len;
    }
    return w;
}
