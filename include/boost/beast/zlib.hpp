// boost/beast/zlib.hpp -- drop-in replacement of Beast's zlib umbrella
// header (reference: include/boost/beast/zlib.hpp) backed by the MI355X engine.
#ifndef BOOST_BEAST_ZLIB_HPP
#define BOOST_BEAST_ZLIB_HPP

#include <boost/beast/zlib/deflate_stream.hpp>
#include <boost/beast/zlib/error.hpp>
#include <boost/beast/zlib/inflate_stream.hpp>
#include <boost/beast/zlib/zlib.hpp>

#endif
