// zstream.h -- device-resident state of one zlib::inflate_stream and the
// result record of one write(), shared by the per-stream kernel
// (pmd_zstream.hip) and its host side (pmd_stream.hip).
//
// The fields are the members of Beast's inflate_stream that survive a
// write() call (include/boost/beast/zlib/detail/inflate_stream.hpp:87-140,
// bitstream.hpp:49-56, window.hpp:51-57).
#pragma once

#include <stdint.h>

namespace bpmd {
namespace zst {

// inflate_stream.hpp:87-118, in the reference's order (done() compares modes)
enum Mode : uint32_t {
    HEAD, TYPE, TYPEDO, STORED, COPY_, COPY, TABLE, LENLENS, CODELENS, LEN_, LEN, LENEXT, DIST, DISTEXT,
    MATCH, LIT, CHECK, DONE, BAD, SYNC
};

struct Head {
    uint32_t mode, last;
    uint32_t bv, bn;                    // bitstream v_ / n_
    uint32_t length, offset, extra, was;
    uint32_t nlen, ndist, ncode, have;
    uint32_t lroot, droot, dtab;        // lenbits_, distbits_, distcode_ - codes_
    uint32_t wbits, wsize, wpos;        // window bits_, size_, i_
    uint32_t pad[14];
};
static_assert(sizeof(Head) == 128, "head");

constexpr unsigned kLens = 320;
constexpr unsigned kCodes = 1444;       // kEnoughLens + kEnoughDists (huff_table.h)
constexpr unsigned kWin = 32768;

struct State {
    Head h;
    uint8_t lens[kLens];                // lens_ (values 0..15)
    uint16_t codes[kCodes];             // codes_ (huff_table.h slots)
    uint8_t pad[8];
    uint8_t win[kWin];                  // window p_, 2^wbits bytes used
};

// one write(): what done() publishes, or an error that skipped it
struct Result {
    uint64_t in_used, out_used;
    int32_t ec;          // zlib::error value (0 = none)
    int32_t data_type;   // inflate_stream.ipp:110-112
    int32_t published;   // 1: done() ran and zs advances; 0: err() returned without it
    int32_t pad;
};

// one write() of a batched launch (pmd_stream.hip's micro-batcher): the
// stream's device State, its input, output room and Result record
struct ZCall {
    void* st;
    const uint8_t* in;
    uint64_t n_in;
    uint8_t* out;
    uint64_t cap;
    void* res;
    int32_t flush;
    int32_t pad[3];
};
static_assert(sizeof(ZCall) == 64, "call record");

}  // namespace zst
}  // namespace bpmd
