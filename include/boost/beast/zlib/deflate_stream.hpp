// boost/beast/zlib/deflate_stream.hpp -- drop-in zlib::deflate_stream
// (reference: include/boost/beast/zlib/deflate_stream.hpp:59-410) backed by
// the MI355X engine's per-stream C ABI (include/beast_pmd.h,
// bpmd_deflate_stream_*).  Same members, signatures and error behaviour:
// reset() throws std::invalid_argument on bad parameters
// (deflate_stream.ipp:235-253), write() reports zlib::error through ec and
// throws std::invalid_argument for a null next_in with avail_in > 0
// (deflate_stream.ipp:363-364).  Output is this engine's own parse: a valid
// stream with the reference's flush framing, round-tripping byte for byte,
// within the size tolerance stated in DESIGN.md.  Link libbeast_pmd.so; with
// no GPU, calls throw std::runtime_error (there is no CPU fallback).
#ifndef BOOST_BEAST_ZLIB_DEFLATE_STREAM_HPP
#define BOOST_BEAST_ZLIB_DEFLATE_STREAM_HPP

#include <boost/beast/zlib/error.hpp>
#include <boost/beast/zlib/zlib.hpp>

#include <cstddef>
#include <stdexcept>
#include <string>

#include "../../../beast_pmd.h"

namespace boost {
namespace beast {
namespace zlib {

namespace detail {

inline bpmd_zparams to_c(const z_params& zs)
{
    return bpmd_zparams{zs.next_in, zs.avail_in, zs.total_in, zs.next_out, zs.avail_out, zs.total_out, zs.data_type};
}

inline void from_c(z_params& zs, const bpmd_zparams& c)
{
    zs.next_in = c.next_in;
    zs.avail_in = c.avail_in;
    zs.total_in = c.total_in;
    zs.next_out = c.next_out;
    zs.avail_out = c.avail_out;
    zs.total_out = c.total_out;
    zs.data_type = c.data_type;
}

// a C ABI result into the reference's reporting: throws where it throws,
// BOOST_BEAST_ASSIGN_EC where it assigns
inline void assign(boost::beast::error_code& ec, int r, const char* what)
{
    if (r == BPMD_R_INVALID_ARGUMENT) throw std::invalid_argument(what);
    if (r == BPMD_R_DOMAIN_ERROR) throw std::domain_error(what);
    if (r < 0) throw std::runtime_error(std::string(what) + ": GPU engine unavailable");
    if (r) ec = make_error_code(static_cast<error>(r));
}

}  // namespace detail

// deflate_stream.hpp:402-410
inline std::size_t deflate_upper_bound(std::size_t bytes) { return bpmd_deflate_upper_bound(bytes); }

// deflate_stream.hpp:59-369
class deflate_stream
{
public:
    // deflate_stream.hpp:80-83: (6, 15, def_mem_level = 9, normal)
    deflate_stream() { reset(6, 15, 9, Strategy::normal); }
    ~deflate_stream() { bpmd_stream_destroy(s_); }
    deflate_stream(deflate_stream const&) = delete;
    deflate_stream& operator=(deflate_stream const&) = delete;

    // deflate_stream.hpp:107-116, deflate_stream.ipp:227-265
    void reset(int level, int windowBits, int memLevel, Strategy strategy)
    {
        bpmd_stream* n = nullptr;
        int r = bpmd_deflate_stream_create(level, windowBits, memLevel, static_cast<int>(strategy), &n);
        if (r == BPMD_R_INVALID_ARGUMENT) throw std::invalid_argument("invalid level, windowBits or memLevel");
        if (r) throw std::runtime_error("deflate_stream::reset");
        bpmd_stream_destroy(s_);
        s_ = n;
    }

    // deflate_stream.hpp:126-131
    void reset() { bpmd_deflate_stream_reset(s_); }

    // deflate_stream.hpp:141-146 (frees the buffers; the stream stays usable)
    void clear() { bpmd_deflate_stream_reset(s_); }

    // deflate_stream.hpp:157-161
    std::size_t upper_bound(std::size_t sourceLen) const { return deflate_upper_bound(sourceLen); }

    // deflate_stream.hpp:173-181
    void tune(int good_length, int max_lazy, int nice_length, int max_chain)
    {
        bpmd_deflate_stream_tune(s_, good_length, max_lazy, nice_length, max_chain);
    }

    // deflate_stream.hpp:293-300
    void write(z_params& zs, Flush flush, boost::beast::error_code& ec)
    {
        bpmd_zparams c = detail::to_c(zs);
        int r = bpmd_deflate_stream_write(s_, &c, static_cast<int>(flush));
        detail::assign(ec, r, "invalid input");
        detail::from_c(zs, c);
    }

    // deflate_stream.hpp:321-329
    void params(z_params& zs, int level, Strategy strategy, boost::beast::error_code& ec)
    {
        bpmd_zparams c = detail::to_c(zs);
        int r = bpmd_deflate_stream_params(s_, &c, level, static_cast<int>(strategy));
        detail::assign(ec, r, "params");
        detail::from_c(zs, c);
    }

    // deflate_stream.hpp:344-348
    void pending(unsigned* value, int* bits) { bpmd_deflate_stream_pending(s_, value, bits); }

    // deflate_stream.hpp:363-368
    void prime(int bits, int value, boost::beast::error_code& ec)
    {
        detail::assign(ec, bpmd_deflate_stream_prime(s_, bits, value), "prime");
    }

private:
    bpmd_stream* s_ = nullptr;
};

}  // namespace zlib
}  // namespace beast
}  // namespace boost

#endif
