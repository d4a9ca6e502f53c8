// boost/beast/zlib/zlib.hpp -- drop-in replacement of Beast's zlib common
// types (reference: include/boost/beast/zlib/zlib.hpp:44-246) for the MI355X
// permessage-deflate engine.  With this repository's include/ directory
// ahead of Boost's on the include path, Beast's websocket layer
// (websocket/detail/impl_base.hpp:21-22, 45-55) compiles its pmd_type
// { zlib::deflate_stream zo; zlib::inflate_stream zi; } against the GPU
// engine without edits.  Same names, values and enum order as the reference.
#ifndef BOOST_BEAST_ZLIB_ZLIB_HPP
#define BOOST_BEAST_ZLIB_ZLIB_HPP

#include <cstddef>

namespace boost {
namespace beast {
namespace zlib {

using Byte = unsigned char;   // 8 bits
using uInt = unsigned int;    // 16 bits or more

// Possible values of the data_type field (zlib.hpp:54-59)
enum kind
{
    binary = 0,
    text = 1,
    unknown = 2
};

// Deflate codec parameters (zlib.hpp:78-144)
struct z_params
{
    void const* next_in;
    std::size_t avail_in;
    std::size_t total_in = 0;
    void* next_out;
    std::size_t avail_out;
    std::size_t total_out = 0;
    int data_type = unknown;
};

// Flush option (zlib.hpp:159-183); the order matters
enum class Flush
{
    none,
    block,
    partial,
    sync,
    full,
    finish,
    trees
};

// Compression levels (zlib.hpp:197-203)
enum compression
{
    none = 0,
    best_speed = 1,
    best_size = 9,
    default_size = -1
};

// Compression strategy (zlib.hpp:209-246)
enum class Strategy
{
    normal,
    filtered,
    huffman,
    rle,
    fixed
};

}  // namespace zlib
}  // namespace beast
}  // namespace boost

#endif
