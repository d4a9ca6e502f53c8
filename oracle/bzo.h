/*
 * bzo.h -- CPU ORACLE for the permessage-deflate hot path.  TEST
 * INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py, never by the product path (beast_amd/).
 *
 * A clean-room C restatement of Boost.Beast's header-only zlib
 * (include/boost/beast/zlib/, Beast v361) plus the RFC 7692 framing that the
 * websocket stream wraps around it (websocket/detail/impl_base.hpp:85-202).
 * Behaviour follows the reference file:line cited at each function in bzo.c.
 *
 * Parity pinning: (1) deflate output is compared byte-for-byte with zlib
 * 1.3.1 built from the reference's vendored sources
 * (/root/reference/test/extern/zlib-1.3.1, recipe oracle/Makefile ->
 * oracle/_ref/libzref.so), which Beast matches at levels 1-9 (SURVEY.md
 * §0.4); (2) inflate error semantics are pinned by the reference's own
 * known-answer vectors (test/beast/zlib/inflate_stream.cpp:505-586), kept as
 * data in tests/golden/inflate_kat.json.
 */
#ifndef BZO_H
#define BZO_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* zlib::z_params (zlib/zlib.hpp:78-144) */
typedef struct bzo_zparams {
    const uint8_t* next_in;
    size_t avail_in;
    size_t total_in;
    uint8_t* next_out;
    size_t avail_out;
    size_t total_out;
    int data_type;           /* 0 binary, 1 text, 2 unknown */
} bzo_zparams;

/* zlib::Flush (zlib/zlib.hpp:159-183); order matters */
enum {
    BZO_FLUSH_NONE = 0, BZO_FLUSH_BLOCK, BZO_FLUSH_PARTIAL, BZO_FLUSH_SYNC,
    BZO_FLUSH_FULL, BZO_FLUSH_FINISH, BZO_FLUSH_TREES
};

/* zlib::Strategy (zlib/zlib.hpp:209-246) */
enum {
    BZO_STRATEGY_NORMAL = 0, BZO_STRATEGY_FILTERED, BZO_STRATEGY_HUFFMAN,
    BZO_STRATEGY_RLE, BZO_STRATEGY_FIXED
};

/* zlib::error (zlib/error.hpp:48-138).  Negative values stand for the C++
 * exceptions the reference throws (invalid_argument / domain_error /
 * logic_error). */
enum {
    BZO_OK = 0,
    BZO_NEED_BUFFERS = 1, BZO_END_OF_STREAM, BZO_NEED_DICT, BZO_STREAM_ERROR,
    BZO_INVALID_BLOCK_TYPE, BZO_INVALID_STORED_LENGTH, BZO_TOO_MANY_SYMBOLS,
    BZO_INVALID_CODE_LENGTHS, BZO_INVALID_BIT_LENGTH_REPEAT, BZO_MISSING_EOB,
    BZO_INVALID_LITERAL_LENGTH, BZO_INVALID_DISTANCE_CODE,
    BZO_INVALID_DISTANCE, BZO_OVER_SUBSCRIBED_LENGTH,
    BZO_INCOMPLETE_LENGTH_SET, BZO_GENERAL,
    BZO_THROW_INVALID_ARGUMENT = -1,
    BZO_THROW_DOMAIN_ERROR = -2,
    BZO_THROW_LOGIC_ERROR = -3
};

typedef struct bzo_inflater bzo_inflater;
typedef struct bzo_deflater bzo_deflater;

/* ---- inflate_stream (zlib/inflate_stream.hpp:63-213) ---- */
bzo_inflater* bzo_inflate_new(void);
void bzo_inflate_free(bzo_inflater*);
int  bzo_inflate_reset(bzo_inflater*, int window_bits);
void bzo_inflate_clear(bzo_inflater*);
int  bzo_inflate_write(bzo_inflater*, bzo_zparams*, int flush);

/* ---- deflate_stream (zlib/deflate_stream.hpp:59-369) ---- */
bzo_deflater* bzo_deflate_new(void);   /* default ctor: (6, 15, 9, normal) */
void   bzo_deflate_free(bzo_deflater*);
int    bzo_deflate_reset_params(bzo_deflater*, int level, int window_bits,
                                int mem_level, int strategy);
void   bzo_deflate_reset(bzo_deflater*);
void   bzo_deflate_clear(bzo_deflater*);
size_t bzo_deflate_upper_bound(const bzo_deflater*, size_t source_len);
void   bzo_deflate_tune(bzo_deflater*, int good, int lazy, int nice, int chain);
int    bzo_deflate_params(bzo_deflater*, bzo_zparams*, int level, int strategy);
int    bzo_deflate_pending(bzo_deflater*, unsigned* bytes, int* bits);
int    bzo_deflate_prime(bzo_deflater*, int bits, int value);
int    bzo_deflate_write(bzo_deflater*, bzo_zparams*, int flush);

/* free-function deflate_upper_bound (zlib/deflate_stream.hpp:402-410) */
size_t bzo_deflate_upper_bound_free(size_t n);

/* ---- permessage-deflate framing (websocket/detail/impl_base.hpp) ---- */
/* One message: Flush::none over the input, then Flush::block, then
 * Flush::sync, and drop the trailing 00 00 FF FF (impl_base.hpp:85-154).
 * Returns the payload length, or -(error) on failure / insufficient cap. */
long bzo_pmd_deflate_msg(bzo_deflater*, const uint8_t* in, size_t n,
                         uint8_t* out, size_t cap);
/* One message: inflate the payload with Flush::sync, then append the
 * 00 00 FF FF tail (impl_base.hpp:168-190, read.hpp:1343-1356).  When
 * raw != 0 no tail is appended (plain zlib::inflate_stream semantics, used by
 * the reference's known-answer tests).  Writes at most cap bytes; status is
 * 0, an error code, or BZO_NEED_BUFFERS when the output exceeded cap. */
int  bzo_pmd_inflate_msg(bzo_inflater*, const uint8_t* in, size_t n,
                         uint8_t* out, size_t cap, size_t* out_len, int raw);

/* Batch helpers used by tests/bench (threads <= 0 means 1).  Every message is
 * an independent stream (no_context_takeover: reset per message). */
int bzo_pmd_deflate_batch(int level, int window_bits, int mem_level,
                          int strategy, const uint8_t* in,
                          const uint64_t* in_off, const uint32_t* in_len,
                          uint32_t n_msgs, uint8_t* out,
                          const uint64_t* out_off, const uint32_t* out_cap,
                          uint32_t* out_len, int32_t* status, int threads);
int bzo_pmd_inflate_batch(int window_bits, int raw, const uint8_t* in,
                          const uint64_t* in_off, const uint32_t* in_len,
                          uint32_t n_msgs, uint8_t* out,
                          const uint64_t* out_off, const uint32_t* out_cap,
                          uint32_t* out_len, int32_t* status, int threads);

/* ---- frame-adjacent byte passes (bzo_frame.c) ---- */
/* mask_inplace (websocket/detail/mask.ipp:38-59) with a key already rotated
 * by `phase` bytes; returns the rotation afterwards */
unsigned bzo_mask(uint8_t* p, size_t n, uint32_t key, unsigned phase);
/* frame headers (websocket/detail/frame.hpp:134-175) and the frame loop of a
 * message (websocket/impl/write.hpp:463-545); keys NULL = unmasked */
size_t bzo_frame_wire_size(uint64_t n, uint64_t frame_max, int masked);
size_t bzo_frame_write(uint8_t* out, const uint8_t* payload, uint64_t n, unsigned op, int rsv1, const uint32_t* keys,
                       uint64_t frame_max);
/* utf8_checker (websocket/detail/utf8_checker.hpp/.ipp) */
typedef struct bzo_utf8 {
    size_t need;   /* bytes still needed by the open code point */
    size_t have;   /* bytes of it seen */
    uint8_t cp[4];
} bzo_utf8;
void bzo_utf8_reset(bzo_utf8*);
int  bzo_utf8_write(bzo_utf8*, const uint8_t* in, size_t n);
int  bzo_utf8_finish(bzo_utf8*);
/* one write() + finish(): 0 valid, 1 write ok but finish fails, 2 write fails */
int  bzo_utf8_check(const uint8_t* p, size_t n);
int  bzo_utf8_check_batch(const uint8_t* in, const uint64_t* off, const uint32_t* len, uint32_t n,
                          int32_t* result);

#ifdef __cplusplus
}
#endif
#endif
