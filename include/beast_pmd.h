/*
 * beast_pmd.h -- C ABI of the MI355X permessage-deflate engine.
 *
 * Drop-in boundary for Boost.Beast's WebSocket permessage-deflate path.  In
 * Beast the only caller of the codec is websocket::stream<..., true> through
 * impl_base<true> (include/boost/beast/websocket/detail/impl_base.hpp:85-202),
 * which calls exactly:
 *     zo.reset(level, wbits, memLevel, Strategy::normal)   impl_base.hpp:295-307
 *     zo.write(zs, Flush::{none,block,sync}, ec)            impl_base.hpp:104-141
 *     zo.reset()                                            impl_base.hpp:156-166
 *     zi.reset(wbits)  zi.write(zs, Flush::sync, ec)        impl_base.hpp:168-190, 295-305
 * Each entry point below names the reference interface it replaces.
 *
 * Conventions: plain pointers and sizes only.  All functions are noexcept and
 * return 0 on success or a negative bpmd_result; per-message outcomes are
 * Beast's zlib::error values (include/boost/beast/zlib/error.hpp:48-138) in
 * the status array.  Device pointers refer to memory of the current HIP
 * device; `stream` is a hipStream_t (0 = default stream).  Batch calls are
 * asynchronous on `stream`: they enqueue their kernels and return without
 * waiting for the device (bpmd_inflate_batch / bpmd_read_batch of every size,
 * the block-parallel path of long payloads included; deflate of messages of
 * at most 4 KiB), with two exceptions, both waits on `stream`:
 *   - bpmd_deflate_batch / bpmd_write_batch with a message longer than
 *     4 KiB (or any context-takeover deflate) read back a 4-byte chunk count
 *     that sizes their chunk workspace, so they return only once the work
 *     queued on `stream` before them has run (the short messages' kernel is
 *     enqueued before the wait and runs meanwhile);
 *   - a call that needs more device workspace than its stream's pool holds
 *     (work queues, chunk scratch, block-parallel decode workspace) grows
 *     the pool, and freeing the smaller block waits for `stream` to drain;
 *     a stream that repeats one batch shape grows it only on the first calls;
 *   - the first inflate call on a stream that decodes long payloads
 *     block-parallel reads back that batch's workspace totals once (so the
 *     first call already runs the fast path), unless bpmd_inflate_reserve()
 *     sized the stream before.  That read-back waits for the work queued on
 *     the stream before the call, so a stream that is being captured into a
 *     graph (hipStreamBeginCapture) must be reserved first.
 * Concurrent calls from several host threads on one stream are serialised
 * per stream.
 */
#ifndef BEAST_PMD_H
#define BEAST_PMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* zlib::error (zlib/error.hpp:48-138) */
enum bpmd_status {
    BPMD_OK = 0,
    BPMD_NEED_BUFFERS = 1,
    BPMD_END_OF_STREAM = 2,
    BPMD_NEED_DICT = 3,
    BPMD_STREAM_ERROR = 4,
    BPMD_INVALID_BLOCK_TYPE = 5,
    BPMD_INVALID_STORED_LENGTH = 6,
    BPMD_TOO_MANY_SYMBOLS = 7,
    BPMD_INVALID_CODE_LENGTHS = 8,
    BPMD_INVALID_BIT_LENGTH_REPEAT = 9,
    BPMD_MISSING_EOB = 10,
    BPMD_INVALID_LITERAL_LENGTH = 11,
    BPMD_INVALID_DISTANCE_CODE = 12,
    BPMD_INVALID_DISTANCE = 13,
    BPMD_OVER_SUBSCRIBED_LENGTH = 14,
    BPMD_INCOMPLETE_LENGTH_SET = 15,
    BPMD_GENERAL = 16
};

/* call-level results (negative) */
enum bpmd_result {
    BPMD_R_OK = 0,
    BPMD_R_INVALID_ARGUMENT = -1,   /* reference throws std::invalid_argument */
    BPMD_R_DOMAIN_ERROR = -2,       /* reference throws std::domain_error */
    BPMD_R_HIP_ERROR = -3,
    BPMD_R_NO_DEVICE = -4
};

/* zlib::Strategy (zlib/zlib.hpp:209-246) */
enum bpmd_strategy {
    BPMD_STRATEGY_NORMAL = 0, BPMD_STRATEGY_FILTERED = 1, BPMD_STRATEGY_HUFFMAN = 2,
    BPMD_STRATEGY_RLE = 3, BPMD_STRATEGY_FIXED = 4
};

/* flags */
#define BPMD_F_RAW 1u   /* inflate: plain inflate_stream::write() semantics, no 00 00 FF FF tail */
#define BPMD_F_EXACT 2u /* deflate: payloads bit-identical to Beast's deflate_stream (the
                           reference's parse, block splits and trees; slower). Not with
                           context takeover. */

/* Codec configuration: the subset of websocket::permessage_deflate
 * (websocket/option.hpp:34-67) that reaches the codec after negotiation
 * (impl_base.hpp:277-309). */
typedef struct bpmd_cfg {
    int level;        /* compLevel 0..9 (-1 = 6) */
    int window_bits;  /* 9..15 for deflate (8 is bumped to 9), 8..15 for inflate */
    int mem_level;    /* 1..9 */
    int strategy;     /* bpmd_strategy */
    uint32_t flags;
} bpmd_cfg;

/* Library / device bring-up.  Idempotent.  Returns BPMD_R_NO_DEVICE when no
 * HIP device is visible (the engine has no CPU fallback). */
int bpmd_init(void);
/* Library version string. */
const char* bpmd_version(void);

/* Batched inflate of independent permessage-deflate payloads (replaces one
 * zi.reset(wbits) + zi.write(zs, Flush::sync) + inflate_with_eb() sequence
 * per message: impl_base.hpp:168-190, websocket/impl/read.hpp:1284-1356).
 *   d_in + d_in_off[i], d_in_len[i]   payload i without the 00 00 FF FF tail
 *   d_out + d_out_off[i], d_out_cap[i] output slot i
 *   d_out_len[i]  bytes produced;  d_status[i]  zlib::error of message i
 *                 (need_buffers = output exceeded d_out_cap[i]) */
int bpmd_inflate_batch(const bpmd_cfg* cfg, const uint8_t* d_in, const uint64_t* d_in_off,
                       const uint32_t* d_in_len, uint32_t n_msgs, uint8_t* d_out,
                       const uint64_t* d_out_off, const uint32_t* d_out_cap,
                       uint32_t* d_out_len, int32_t* d_status, void* stream);

/* Workspace for the block-parallel decode of long payloads on `stream`
 * (no Beast counterpart: the reference decodes on the caller's thread).  Sizes
 * the stream's capacity for batches whose long payloads total at most
 * in_bytes of compressed input, out_bytes of output capacity and n_long
 * payloads, so that no later call on the stream waits to size it; a long
 * payload that does not fit a stream's capacity is still decoded exactly, by
 * the slower wave kernel.  The capacity never exceeds half the device's free
 * memory.  Optional: without it the stream's first such call sizes it. */
int bpmd_inflate_reserve(void* stream, uint64_t in_bytes, uint64_t out_bytes, uint32_t n_long);

/* Batched deflate of independent messages into permessage-deflate payloads
 * (replaces one zo.write(zs, Flush::none) ... zo.write(zs, Flush::block),
 * zo.write(zs, Flush::sync), strip 00 00 FF FF, zo.reset() sequence per
 * message under no_context_takeover: impl_base.hpp:85-166,
 * websocket/impl/write.hpp:655-703).  cfg->level / window_bits / mem_level
 * are validated as deflate_stream::reset (deflate_stream.ipp:227-265);
 * strategy selects the parser as zlib::Strategy does.  The payload is a
 * valid raw-DEFLATE stream whose blocks all have BFINAL = 0, ending with
 * the header bits of an empty stored block padded to a byte, exactly the
 * framing Beast produces; the block contents are this engine's own parse
 * (byte-identical round trip, compressed size within the tolerance stated
 * in DESIGN.md).
 *   d_in + d_in_off[i], d_in_len[i]     message i
 *   d_out + d_out_off[i], d_out_cap[i]  output slot i (bpmd_deflate_upper_bound(len) always suffices)
 *   d_out_len[i]  payload bytes;  d_status[i]  0, or need_buffers if the
 *                 slot was too small (d_out_len[i] = 0, slot contents undefined) */
int bpmd_deflate_batch(const bpmd_cfg* cfg, const uint8_t* d_in, const uint64_t* d_in_off,
                       const uint32_t* d_in_len, uint32_t n_msgs, uint8_t* d_out,
                       const uint64_t* d_out_off, const uint32_t* d_out_cap,
                       uint32_t* d_out_len, int32_t* d_status, void* stream);

/* Inflate kernel selection (no reference counterpart; tuning and tests):
 * 0 automatic (one lane per message for batches of >= 2048 messages, one
 * wave per message below), 1 always lane-per-message, 2 always
 * wave-per-message.  Both produce identical results.  Initial value from
 * the BPMD_INFLATE environment variable ("lane" / "wave"). */
int bpmd_set_inflate_kernel(int mode);

/* deflate_upper_bound (zlib/deflate_stream.hpp:402-410): size a d_out slot. */
size_t bpmd_deflate_upper_bound(size_t n);

/* ---------------------------------------------------------------------
 * One process, several GPUs.  Messages are
 * independent streams, so a batch splits into contiguous, byte-balanced
 * message ranges, one per device; every shard's buffers live on its own
 * device and no payload crosses GPUs.
 * ------------------------------------------------------------------- */

/* Byte-balanced contiguous ranges (beast_amd/shard.py): shard p is messages
 * [starts[p], starts[p+1]), starts has n_parts + 1 entries; shard r ends at
 * the first message whose byte prefix sum reaches (r + 1) / n_parts of the
 * total.  Host only. */
int bpmd_shard_ranges(const uint32_t* lens, uint32_t n, int n_parts, uint32_t* starts);

/* One shard: device pointers of `device`, launched on `stream` (a
 * hipStream_t of that device, 0 = its default stream). */
typedef struct bpmd_shard {
    int device;
    void* stream;
    const uint8_t* d_in;
    const uint64_t* d_in_off;
    const uint32_t* d_in_len;
    uint32_t n_msgs;
    uint8_t* d_out;
    const uint64_t* d_out_off;
    const uint32_t* d_out_cap;
    uint32_t* d_out_len;
    int32_t* d_status;
} bpmd_shard;

/* bpmd_inflate_batch / bpmd_deflate_batch on every shard, each on its own
 * device and stream, asynchronously; each shard is launched from a host
 * thread of its own, so a shard whose call waits on its stream (deflate of
 * messages over 4 KiB) does not hold back the others.  out_bytes (n_shards entries, or NULL):
 * each shard's total output bytes (sum of its d_out_len), gathered to the
 * host -- the call then waits for every shard -- so each shard's offset in
 * one global output is the exclusive prefix sum.  The current device is
 * restored. */
int bpmd_inflate_batch_multi(const bpmd_cfg* cfg, const bpmd_shard* shards, int n_shards, uint64_t* out_bytes);
int bpmd_deflate_batch_multi(const bpmd_cfg* cfg, const bpmd_shard* shards, int n_shards, uint64_t* out_bytes);

/* ---------------------------------------------------------------------
 * Frame-adjacent byte passes.  Masking keys are the
 * frame header's 32-bit key as Beast reads it, little-endian from the wire
 * (stream_impl.hpp:866-870): payload byte j is XORed with byte (j + phase) % 4
 * of the key (prepare_key / mask_inplace, websocket/detail/mask.ipp:20-59).
 * ------------------------------------------------------------------- */

/* Batched mask_inplace (mask.ipp:38-59), in place.  d_phase[i] is the key
 * rotation a prepared_key carries after masking the frame's earlier bytes
 * (rol, mask.ipp:29-36), i.e. their count mod 4; NULL = 0.  Masking is an
 * involution: the same call masks (write.hpp:679-685) and unmasks
 * (read.hpp:1324-1327). */
int bpmd_mask_batch(uint8_t* d_data, const uint64_t* d_off, const uint32_t* d_len, uint32_t n_msgs,
                    const uint32_t* d_key, const uint8_t* d_phase, void* stream);

/* utf8_checker verdicts (websocket/detail/utf8_checker.ipp) */
enum bpmd_utf8 {
    BPMD_UTF8_VALID = 0,       /* write() and finish() succeed */
    BPMD_UTF8_INCOMPLETE = 1,  /* write() succeeds, finish() fails: ends inside a code point */
    BPMD_UTF8_INVALID = 2      /* write() fails */
};

/* Batched check_utf8 (utf8_checker.ipp:317-324) keeping the verdict of one
 * utf8_checker::write() over each whole message: d_result[i] = bpmd_utf8.
 * Feeding a message in pieces gives the same verdicts: the fail-fast rule
 * (utf8_checker.ipp:86-157) rejects exactly the invalid prefixes. */
int bpmd_utf8_check_batch(const uint8_t* d_data, const uint64_t* d_off, const uint32_t* d_len, uint32_t n_msgs,
                          int32_t* d_result, void* stream);

/* websocket::error::bad_frame_payload (websocket/error.hpp): the per-message
 * status bpmd_read_batch reports for a text message that is not UTF-8. */
#define BPMD_BAD_FRAME_PAYLOAD 256

/* Receive side of a batch of permessage-deflate messages, fused
 * (read.hpp:1284-1385): unmask the payload inside inflate's input loads
 * (server role, read.hpp:1324-1327; d_key NULL = unmasked), inflate as
 * bpmd_inflate_batch, then check the inflated bytes of text messages
 * (d_text[i] != 0; NULL = all binary) as read.hpp:1372-1384 does.
 * d_status[i]: inflate's zlib::error if nonzero, else BPMD_BAD_FRAME_PAYLOAD
 * for a text message that is not valid UTF-8, else 0.  d_in is not
 * modified. */
int bpmd_read_batch(const bpmd_cfg* cfg, const uint8_t* d_in, const uint64_t* d_in_off, const uint32_t* d_in_len,
                    const uint32_t* d_key, const uint8_t* d_text, uint32_t n_msgs, uint8_t* d_out,
                    const uint64_t* d_out_off, const uint32_t* d_out_cap, uint32_t* d_out_len, int32_t* d_status,
                    void* stream);

/* Send side, fused (write.hpp:655-703): deflate as bpmd_deflate_batch and
 * mask each payload with d_key[i] inside the kernel's output stores (client
 * role, write.hpp:679-685; d_key NULL = unmasked). */
int bpmd_write_batch(const bpmd_cfg* cfg, const uint8_t* d_in, const uint64_t* d_in_off, const uint32_t* d_in_len,
                     const uint32_t* d_key, uint32_t n_msgs, uint8_t* d_out, const uint64_t* d_out_off,
                     const uint32_t* d_out_cap, uint32_t* d_out_len, int32_t* d_status, void* stream);

/* Frames of a batch of messages on the send side, as write_some sends a
 * compressed message (websocket/impl/write.hpp:463-545) with headers written
 * by detail::write (websocket/detail/frame.hpp:134-175): message i's payload
 * d_in + d_in_off[i] (d_in_len[i] bytes, e.g. bpmd_deflate_batch's output)
 * goes out in frames of at most frame_max bytes (Beast's wr_buf_size; one
 * empty frame for an empty payload).  Frame f: FIN on the last, RSV1 on the
 * first when d_flags[i] & 1 (compressed; NULL = all compressed), opcode
 * d_op[i] on the first (NULL = binary, 2) and cont (0) after; with d_keys
 * (client role) the MASK bit, key d_keys[d_key_base[i] + f] in the header
 * (little-endian) and the frame's payload masked with it (a fresh
 * prepare_key per frame).  The wire bytes go to d_wire + d_wire_off[i];
 * bpmd_frame_wire_size gives their count.  Any split is a valid RFC 6455
 * message; Beast's own split also depends on when its deflater flushes. */
uint64_t bpmd_frame_wire_size(uint64_t payload_len, uint32_t frame_max, int masked);
int bpmd_frame_batch(const uint8_t* d_in, const uint64_t* d_in_off, const uint32_t* d_in_len, const uint8_t* d_op,
                     const uint8_t* d_flags, const uint32_t* d_keys, const uint32_t* d_key_base, uint32_t frame_max,
                     uint32_t n_msgs, uint8_t* d_wire, const uint64_t* d_wire_off, void* stream);

/* ---------------------------------------------------------------------
 * Context takeover: when no_context_takeover is not
 * negotiated, Beast's inflater keeps its window from message to message
 * (do_context_takeover_read -> inflate_stream::clear() is a no-op,
 * impl_base.hpp:192-202, inflate_stream.ipp:49-53), so a message may copy
 * from the connection's earlier output.  Each connection keeps its output in
 * one device buffer; message i is decoded into d_out + d_out_off[i], right
 * after that connection's earlier output, whose last d_hist_len[i] bytes
 * (clamped to 2^windowBits) are the window.  One message per connection per
 * batch; connections run in parallel.  Statuses as bpmd_inflate_batch
 * (invalid_distance for a distance past the window).
 * ------------------------------------------------------------------- */
int bpmd_inflate_takeover_batch(const bpmd_cfg* cfg, const uint8_t* d_in, const uint64_t* d_in_off,
                                const uint32_t* d_in_len, const uint32_t* d_hist_len, uint32_t n_msgs,
                                uint8_t* d_out, const uint64_t* d_out_off, const uint32_t* d_out_cap,
                                uint32_t* d_out_len, int32_t* d_status, void* stream);

/* Send side of the same connections: Beast's deflater is not reset between
 * messages (do_context_takeover_write resets only under no_context_takeover,
 * impl_base.hpp:156-166), so its payloads may copy from earlier messages.
 * Message i's bytes at d_in + d_in_off[i] are preceded in d_in by
 * d_hist_len[i] bytes of that connection's earlier plaintext; a match reaches
 * at most BPMD_CHUNK_HIST bytes (beast_amd/csrc/lz_core.h) before the 4 KiB
 * chunk it is in and never more than 2^window_bits back, so the stream is
 * valid for any inflater whose windowBits >= cfg->window_bits.  Otherwise as
 * bpmd_deflate_batch. */
int bpmd_deflate_takeover_batch(const bpmd_cfg* cfg, const uint8_t* d_in, const uint64_t* d_in_off,
                                const uint32_t* d_in_len, const uint32_t* d_hist_len, uint32_t n_msgs,
                                uint8_t* d_out, const uint64_t* d_out_off, const uint32_t* d_out_cap,
                                uint32_t* d_out_len, int32_t* d_status, void* stream);

/* ---------------------------------------------------------------------
 * Cross-connection micro-batcher.  Beast runs one codec
 * call per message inside each connection's async operation
 * (write_some_op, write.hpp:463-545; read.hpp:522-610 via impl_base.hpp:85-190);
 * the batcher coalesces those calls across connections: any thread submits
 * one message (host bytes, copied at submit) with a completion callback;
 * batches launch when max_msgs or the staging bytes fill up, or when the
 * oldest message has waited max_delay_us.  Two pinned staging slots
 * alternate, so submissions continue while the GPU works.
 * ------------------------------------------------------------------- */
enum bpmd_op { BPMD_OP_INFLATE = 0, BPMD_OP_DEFLATE = 1 };
typedef struct bpmd_batcher bpmd_batcher;
/* One message done (on the batcher's completion thread; it must not call
 * bpmd_batcher_flush or _destroy).  status: the message's zlib::error
 * (need_buffers: out_cap too small), or a negative bpmd_result when its batch
 * failed; out_len: bytes written to the submitter's out buffer. */
typedef void (*bpmd_done_fn)(void* user, int32_t status, size_t out_len);
/* cfg as for bpmd_inflate_batch / bpmd_deflate_batch (validated the same
 * way); max_in_bytes / max_out_bytes size each staging slot (input bytes; for
 * inflate the sum of out_cap, for deflate of deflate_upper_bound(n)). */
int bpmd_batcher_create(const bpmd_cfg* cfg, int op, uint32_t max_msgs, size_t max_in_bytes, size_t max_out_bytes,
                        uint32_t max_delay_us, bpmd_batcher** out);
/* Queue one message.  `out` must stay valid until fn runs. */
int bpmd_batcher_submit(bpmd_batcher* b, const void* in, size_t n, void* out, size_t out_cap, bpmd_done_fn fn,
                        void* user);
/* Launch what is queued and wait until every message submitted so far has
 * completed. */
int bpmd_batcher_flush(bpmd_batcher* b);
/* Completes everything queued, then frees the batcher. */
void bpmd_batcher_destroy(bpmd_batcher* b);

/* ---------------------------------------------------------------------
 * permessage-deflate negotiation (wire format only), for
 * a facade that owns the handshake: the Sec-WebSocket-Extensions logic of
 * websocket/detail/pmd_extension.hpp/.ipp.  Host code, no device use.
 * ------------------------------------------------------------------- */
/* detail::pmd_offer (pmd_extension.hpp:27-42) */
typedef struct bpmd_pmd_offer {
    int accept;
    int server_max_window_bits;      /* 0 absent, or 8..15 (-1 present without value when writing) */
    int client_max_window_bits;      /* -1 present without value, 0 absent, or 8..15 */
    int server_no_context_takeover;
    int client_no_context_takeover;
} bpmd_pmd_offer;
/* websocket::permessage_deflate (option.hpp:34-67); the codec fields
 * (compLevel, memLevel, msg_size_threshold) live in bpmd_cfg */
typedef struct bpmd_pmd_options {
    int server_enable, client_enable;
    int server_max_window_bits, client_max_window_bits;
    int server_no_context_takeover, client_no_context_takeover;
} bpmd_pmd_options;
/* pmd_read (pmd_extension.ipp:45-166): the first permessage-deflate offer of
 * a Sec-WebSocket-Extensions value; offer->accept = 0 when it must be declined */
int bpmd_pmd_read(const char* ext, size_t n, bpmd_pmd_offer* offer);
/* pmd_write (pmd_extension.ipp:168-208): the header value of an offer into
 * out (NUL-terminated); returns its length */
int bpmd_pmd_write(const bpmd_pmd_offer* offer, char* out, size_t cap);
/* pmd_negotiate (pmd_extension.hpp:95-111, .ipp:210-290): the server's
 * configuration and response value for a client offer (empty when declined);
 * returns the response length */
int bpmd_pmd_negotiate(const bpmd_pmd_options* o, const bpmd_pmd_offer* offer, bpmd_pmd_offer* config, char* out,
                       size_t cap);
/* pmd_normalize (pmd_extension.ipp:292-305) */
void bpmd_pmd_normalize(bpmd_pmd_offer* offer);

/* Window maintenance for the buffers above: move the d_keep[i] bytes before
 * d_pos[i] of the buffer at d_buf + d_base[i] to its front (the caller slides
 * only when d_pos[i] >= 2 * d_keep[i], so the ranges never overlap). */
int bpmd_slide_batch(uint8_t* d_buf, const uint64_t* d_base, const uint32_t* d_pos, const uint32_t* d_keep,
                     uint32_t n, void* stream);

/* ---------------------------------------------------------------------
 * Per-stream API behind the C++ compatibility facade
 * (include/boost/beast/zlib/ headers).  Host buffers; each call runs on the
 * current device (deflate: the batch kernels on one message; inflate: the
 * per-stream kernel) and synchronises.
 * Throughput comes from the batch API above; these calls exist so code
 * written against zlib::deflate_stream / zlib::inflate_stream (the calls
 * impl_base<true> makes, impl_base.hpp:85-190) runs unchanged.
 * ------------------------------------------------------------------- */

/* z_params (zlib/zlib.hpp:78-144) */
typedef struct bpmd_zparams {
    const void* next_in;
    size_t avail_in;
    size_t total_in;
    void* next_out;
    size_t avail_out;
    size_t total_out;
    int data_type;
} bpmd_zparams;

/* zlib::Flush (zlib/zlib.hpp:159-183); the order matters */
enum bpmd_flush {
    BPMD_FLUSH_NONE = 0, BPMD_FLUSH_BLOCK, BPMD_FLUSH_PARTIAL, BPMD_FLUSH_SYNC, BPMD_FLUSH_FULL,
    BPMD_FLUSH_FINISH, BPMD_FLUSH_TREES
};

typedef struct bpmd_stream bpmd_stream;

/* deflate_stream::reset(level, windowBits, memLevel, strategy)
 * (deflate_stream.ipp:227-265); BPMD_R_INVALID_ARGUMENT where it throws */
int bpmd_deflate_stream_create(int level, int window_bits, int mem_level, int strategy, bpmd_stream** out);
/* deflate_stream::reset() (deflate_stream.hpp:123-127) */
int bpmd_deflate_stream_reset(bpmd_stream* s);
/* deflate_stream::write(zs, flush, ec) (deflate_stream.ipp:357-499): returns
 * the zlib::error value (0 = none) or BPMD_R_INVALID_ARGUMENT where it throws */
int bpmd_deflate_stream_write(bpmd_stream* s, bpmd_zparams* zs, int flush);
/* deflate_stream::params(zs, level, strategy, ec) (deflate_stream.ipp:307-338) */
int bpmd_deflate_stream_params(bpmd_stream* s, bpmd_zparams* zs, int level, int strategy);
/* deflate_stream::tune(good_length, max_lazy, nice_length, max_chain)
 * (deflate_stream.hpp:163-181, deflate_stream.ipp:307-317): replaces the
 * level's good/lazy/nice/chain limits for the following writes (the GPU
 * parser still caps the chain walk); like the reference, a
 * tune before the stream's first write is undone by its lazy init. */
int bpmd_deflate_stream_tune(bpmd_stream* s, int good_length, int max_lazy, int nice_length, int max_chain);
/* deflate_stream::pending(value, bits) (deflate_stream.hpp:344-348) */
int bpmd_deflate_stream_pending(bpmd_stream* s, unsigned* value, int* bits);
/* deflate_stream::prime(bits, value, ec) (deflate_stream.ipp:340-355) */
int bpmd_deflate_stream_prime(bpmd_stream* s, int bits, int value);
/* inflate_stream::reset(windowBits) (inflate_stream.ipp:55-72);
 * BPMD_R_DOMAIN_ERROR where it throws */
int bpmd_inflate_stream_create(int window_bits, bpmd_stream** out);
int bpmd_inflate_stream_reset(bpmd_stream* s, int window_bits);
/* inflate_stream::clear() -- a no-op in the reference (inflate_stream.ipp:49-53) */
int bpmd_inflate_stream_clear(bpmd_stream* s);
/* inflate_stream::write(zs, flush, ec) (inflate_stream.ipp:74-535).  The
 * reference's decoder state (mode, bit reservoir, tables, 2^windowBits
 * window) lives on the device and each call runs its state machine there
 * (beast_amd/csrc/pmd_zstream.hip), so the status, the output bytes and
 * every z_params field -- next_in/avail_in/total_in included: input the
 * reference leaves unconsumed stays with the caller -- equal Beast's after
 * every call.  A data error returns without advancing z_params, as the
 * reference's err() does (inflate_stream.ipp:120-125). */
int bpmd_inflate_stream_write(bpmd_stream* s, bpmd_zparams* zs, int flush);
/* Memory an inflate stream holds (host: the pinned staging buffer of the
 * call's copies, no decoder state; device: state + window and the call's
 * input/output buffers); no reference counterpart, for bounded-memory tests. */
int bpmd_inflate_stream_footprint(const bpmd_stream* s, size_t* host_bytes, size_t* device_bytes);
void bpmd_stream_destroy(bpmd_stream* s);

/* The micro-batcher behind the two write() calls above (no reference
 * counterpart; SURVEY §8(f) N2, for the call sites impl_base.hpp:85-190 and
 * write.hpp:463-545): calls of different streams made at the same time run
 * as one launch, each with exactly its single-call result (status, output
 * bytes, every z_params field).  A call that finds no batch running takes
 * up to max_calls queued calls (one per stream) and runs them; calls that
 * arrive meanwhile form the next batch, so a lone stream waits for nothing
 * (its batch is one call; with the batcher on, streams keep no HIP stream or staging buffers of their own).  max_delay_us > 0: a batch's
 * first call also waits up to that long for more.  max_calls < 2 turns it
 * off.  Default: 256 calls, no delay (environment: BPMD_STREAM_BATCH,
 * BPMD_STREAM_BATCH_DELAY_US). */
int bpmd_stream_batching(int max_calls, int max_delay_us);
/* out[0] inflate write() calls through the batcher, out[1] their launches,
 * out[2] deflate flushes, out[3] their deflater calls; reset != 0 zeroes them. */
int bpmd_stream_batch_stats(unsigned long long* out, int reset);

#ifdef __cplusplus
}
#endif
#endif
