// beast_amd/zlib.hpp -- the C++ facade under the engine's own namespace:
// beast_amd::zlib is boost::beast::zlib of the drop-in headers in
// include/boost/beast/zlib/ (same classes; see those headers and
// INTEGRATION.md).  Header only; link libbeast_pmd.so.
#ifndef BEAST_AMD_ZLIB_HPP
#define BEAST_AMD_ZLIB_HPP

#include <boost/beast/zlib.hpp>

namespace beast_amd {
namespace zlib = ::boost::beast::zlib;
}  // namespace beast_amd

#endif
