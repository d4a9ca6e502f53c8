// boost/beast/zlib/inflate_stream.hpp -- drop-in zlib::inflate_stream
// (reference: include/boost/beast/zlib/inflate_stream.hpp:63-213) backed by
// the MI355X engine's per-stream decoder (bpmd_inflate_stream_*,
// include/beast_pmd.h; the state machine runs on the device,
// beast_amd/csrc/pmd_zstream.hip).  Output bytes, zlib::error values and
// every z_params field after each write() are the reference's; reset() throws std::domain_error
// for windowBits outside 8..15 (inflate_stream.ipp:57-61); clear() keeps
// the window and state as the reference's (empty) doClear does.
#ifndef BOOST_BEAST_ZLIB_INFLATE_STREAM_HPP
#define BOOST_BEAST_ZLIB_INFLATE_STREAM_HPP

#include <boost/beast/zlib/deflate_stream.hpp>
#include <boost/beast/zlib/error.hpp>
#include <boost/beast/zlib/zlib.hpp>

namespace boost {
namespace beast {
namespace zlib {

class inflate_stream
{
public:
    inflate_stream() { reset(15); }
    ~inflate_stream() { bpmd_stream_destroy(s_); }
    inflate_stream(inflate_stream const&) = delete;
    inflate_stream& operator=(inflate_stream const&) = delete;

    // inflate_stream.hpp:79-84
    void reset() { reset(15); }

    // inflate_stream.hpp:91-96, inflate_stream.ipp:55-72
    void reset(int windowBits)
    {
        if (!s_) {
            int r = bpmd_inflate_stream_create(windowBits, &s_);
            if (r == BPMD_R_DOMAIN_ERROR) throw std::domain_error("windowBits out of range");
            if (r) throw std::runtime_error("inflate_stream::reset");
            return;
        }
        if (bpmd_inflate_stream_reset(s_, windowBits) == BPMD_R_DOMAIN_ERROR)
            throw std::domain_error("windowBits out of range");
    }

    // inflate_stream.hpp:101-105
    void clear() { bpmd_inflate_stream_clear(s_); }

    // inflate_stream.hpp:208-212
    void write(z_params& zs, Flush flush, boost::beast::error_code& ec)
    {
        bpmd_zparams c = detail::to_c(zs);
        int r = bpmd_inflate_stream_write(s_, &c, static_cast<int>(flush));
        detail::assign(ec, r, "inflate_stream::write");
        detail::from_c(zs, c);
    }

private:
    bpmd_stream* s_ = nullptr;
};

}  // namespace zlib
}  // namespace beast
}  // namespace boost

#endif
