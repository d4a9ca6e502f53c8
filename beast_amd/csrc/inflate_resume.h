// inflate_resume.h -- decoder checkpoint of the per-stream inflater
// (bpmd_inflate_stream_write, pmd_stream.hip), shared by host and device.
//
// Beast's inflate_stream keeps its mode, bit reservoir, code tables and a
// 2^windowBits window across write() calls (zlib/detail/inflate_stream.ipp:
// 74-535, detail/window.hpp:51-144).  The GPU decoder is not resident between
// calls, so each call ends by saving the last TOKEN BOUNDARY it reached -- a
// block boundary, the start of a decode round inside a Huffman block (with
// the block's code lengths, from which the tables are rebuilt), or a position
// inside a stored block -- and the next call resumes there.  Input before the
// checkpoint is dropped and output before it goes into the window, so a
// write() decodes its own input plus at most one round (<= 3840 output bytes)
// again, whatever the age of the connection.
#pragma once

#include <stdint.h>

// checkpoint modes
enum : uint32_t {
    BPMD_RM_TYPE = 0,     // block boundary (reference mode TYPE / TYPEDO)
    BPMD_RM_FIXED = 1,    // inside a fixed-Huffman block's data (LEN)
    BPMD_RM_DYN = 2,      // inside a dynamic block's data (LEN), lens[] valid
    BPMD_RM_STORED = 3,   // inside a stored block's data (COPY), srem valid
};

// why a call stopped (the host models the reference's input consumption
// from it: an exhausted input is consumed whole, an early stop leaves the
// bytes past the stop position)
enum : uint32_t { BPMD_RW_STARVED = 0, BPMD_RW_FLUSH = 1, BPMD_RW_FULL = 2, BPMD_RW_END = 3 };

// which flush the call was made with, as far as the decoder cares
// (inflate_stream.ipp:138-141, 166-168, 194-196, 350-352)
enum : uint32_t { BPMD_RF_SYNC = 0, BPMD_RF_BLOCK = 1, BPMD_RF_TREES = 2 };

struct bpmd_resume {
    uint32_t bit;      // stream bit of the checkpoint, from the call's first input byte
    uint32_t out;      // output bytes before the checkpoint, from the call's output start
    uint32_t mode;     // BPMD_RM_*
    uint32_t last;     // BFINAL of the current (or last finished) block
    uint32_t nlen;     // dynamic block: literal/length code count (257..286)
    uint32_t ndist;    // dynamic block: distance code count (1..30)
    uint32_t srem;     // stored block: bytes still to copy
    uint32_t end_bit;  // (out) stream bit where the call's decoding stopped
    uint32_t at_type;  // (out) the call stopped at a block boundary
    uint32_t at_hdr;   // (out) Flush::trees stopped it right after a block header
    uint32_t why;      // (out) BPMD_RW_*: why the call's decoding stopped
    uint32_t pad;
    uint8_t lens[320]; // dynamic block: nlen + ndist code lengths
};
static_assert(sizeof(bpmd_resume) == 368, "resume layout");

// per-call window rule (inflate_stream.ipp:1046-1061, 475-496): a match whose
// output starts at position p of this decode may reach back
//   p < D : hist + p                (checked when an earlier call made it)
//   p >= D: cw + (p - D)            (this call's window + this call's output)
// and a match that began before D and continues at D also needs dist <= cw
// (MATCH state re-entered with no output yet).  D = output bytes of the decode
// already delivered by earlier calls, hist = window bytes before the output
// slot = min(total output before the checkpoint, 2^wbits), cw = the window the
// reference holds at this call's start = min(total output before it, 2^wbits).
struct bpmd_resume_call {
    const bpmd_resume* rin;
    bpmd_resume* rout;
    uint32_t hist, D, cw, flush;
};
