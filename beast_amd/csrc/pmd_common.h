// pmd_common.h -- shared device definitions for the permessage-deflate
// kernels (gfx950 / CDNA4, wave64).
//
// Status values are Beast's zlib::error (include/boost/beast/zlib/error.hpp:48-138).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bpmd {

enum Status : int32_t {
    ST_OK = 0,
    ST_NEED_BUFFERS = 1,
    ST_END_OF_STREAM = 2,
    ST_NEED_DICT = 3,
    ST_STREAM_ERROR = 4,
    ST_INVALID_BLOCK_TYPE = 5,
    ST_INVALID_STORED_LENGTH = 6,
    ST_TOO_MANY_SYMBOLS = 7,
    ST_INVALID_CODE_LENGTHS = 8,
    ST_INVALID_BIT_LENGTH_REPEAT = 9,
    ST_MISSING_EOB = 10,
    ST_INVALID_LITERAL_LENGTH = 11,
    ST_INVALID_DISTANCE_CODE = 12,
    ST_INVALID_DISTANCE = 13,
    ST_OVER_SUBSCRIBED_LENGTH = 14,
    ST_INCOMPLETE_LENGTH_SET = 15,
    ST_GENERAL = 16,
};

constexpr int WAVE = 64;

__device__ __forceinline__ unsigned lane_id() { return __lane_id(); }

// RFC 1951 §3.2.5 tables (index = symbol - 257 / distance symbol)
__constant__ static const uint16_t kLenBase[29] = {
    3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31,
    35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ static const uint8_t kLenExtra[29] = {
    0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ static const uint16_t kDistBase[30] = {
    1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193,
    257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
__constant__ static const uint8_t kDistExtra[30] = {
    0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};

}  // namespace bpmd
