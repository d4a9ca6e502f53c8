// bp.h -- block-parallel inflate of long payloads (pmd_inflate_bp.hip): the
// segment records shared by the candidate scan, the lane kernel's segment
// mode (pmd_inflate_lane3.hip) and the resolve pass.
//
// A long payload is cut at dynamic-block headers found by a bit-offset scan
// (plus the payload's first bit).  Each piece ("segment") is decoded by one
// lane of the lane kernel, from its first block header up to the first block
// boundary that is the next candidate's start, as 16-bit symbols: a literal
// byte (0-255), or -- for output a match copies from before the segment's
// start, where the bytes are not known yet -- a reference 0x8000 | k to the
// byte k + 1 positions before the segment's start.  In-segment copies copy
// symbols, so references propagate.  The resolve pass walks each payload's
// segments in stream order (segment -> the candidate it handed off to),
// replaces references by the bytes already written and applies the
// reference's output rules (inflate_stream.ipp:475-514) at message level.
#pragma once
#include <stdint.h>

namespace bpmd {
namespace bp {

// segment statuses beside the inflate ST_* codes (int8 in the END token)
constexpr int32_t SEG_HANDOFF = 100;   // stopped at the next candidate's header
constexpr int32_t SEG_FULL = 101;      // the symbol slot is full
constexpr int32_t SEG_SKIP = 102;      // no candidate in this region
// a stored block that ends where the next candidate starts: nothing decoded,
// the resolve copies its nsym bytes from the payload (after its LEN / NLEN)
constexpr int32_t SEG_DIRECT = 103;

constexpr uint32_t KIND_START = 0;    // the payload's first bit
constexpr uint32_t KIND_DYN = 1;      // a validated dynamic-block header (bit = its first bit)
constexpr uint32_t KIND_STORED = 2;   // a validated stored block (bit = 8 x its LEN field's byte)
constexpr uint32_t KIND_FIXED = 3;    // a fixed-code block reached by the skim (bit = its first bit)
constexpr uint32_t KIND_NONE = 0xffu; // region without a candidate
constexpr uint32_t KIND_PENDING = 0xfeu;  // scan pass 1: no stored block, the dynamic search pending

constexpr uint16_t SYM_REF = 0x8000u;   // symbol bit 15: reference before the segment

struct SegTask {
    uint32_t msg;       // message index
    uint32_t bit;       // first bit of the segment (payload-relative)
    uint32_t kind;      // KIND_*
    uint32_t left;      // task slots of the same message after this one
    uint64_t sym_off;   // first symbol of the slot (uint16 units)
    uint32_t sym_cap;   // slot capacity (symbols)
    uint32_t pad;
};
static_assert(sizeof(SegTask) == 32, "SegTask layout");

struct SegRes {
    uint32_t nsym;     // symbols produced
    int32_t status;    // ST_* or SEG_*
    uint32_t next;     // SEG_HANDOFF: the task it handed off to
    uint32_t pad;
};
static_assert(sizeof(SegRes) == 16, "SegRes layout");

// symbols of guard space before the first slot: a straddling 16-symbol load
// of a match source starts at most 15 symbols before its slot
constexpr uint32_t SYM_GUARD = 64;

}  // namespace bp
}  // namespace bpmd
