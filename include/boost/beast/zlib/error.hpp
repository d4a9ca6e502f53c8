// boost/beast/zlib/error.hpp -- drop-in zlib::error (reference:
// include/boost/beast/zlib/error.hpp:48-138, impl/error.hpp, impl/error.ipp:
// 15-122): same enumerators and values, category name "boost.beast.zlib".
//
// The error code type is boost::beast::error_code.  Where Beast's own
// core/error.hpp is on the include path (a real Boost.Beast build) it is
// boost::system::error_code, as in the reference; a build without Boost (this
// repository's tests) gets std::error_code under the same names.
#ifndef BOOST_BEAST_ZLIB_ERROR_HPP
#define BOOST_BEAST_ZLIB_ERROR_HPP

#include <cstddef>
#include <string>
#include <system_error>
#include <type_traits>

#if defined(__has_include)
#if __has_include(<boost/beast/core/error.hpp>) && __has_include(<boost/system/error_code.hpp>)
#define BPMD_ZLIB_BOOST_SYSTEM 1
#endif
#endif

#ifdef BPMD_ZLIB_BOOST_SYSTEM
#include <boost/beast/core/error.hpp>
#else
namespace boost {
namespace beast {
using error_code = std::error_code;
using error_category = std::error_category;
using error_condition = std::error_condition;
}  // namespace beast
}  // namespace boost
#endif

namespace boost {
namespace beast {
namespace zlib {

// error.hpp:48-138
enum class error
{
    need_buffers = 1,
    end_of_stream,
    need_dict,
    stream_error,
    invalid_block_type,
    invalid_stored_length,
    too_many_symbols,
    invalid_code_lengths,
    invalid_bit_length_repeat,
    missing_eob,
    invalid_literal_length,
    invalid_distance_code,
    invalid_distance,
    over_subscribed_length,
    incomplete_length_set,
    general
};

namespace detail {

// impl/error.ipp:47-115.  boost::system::error_category has the buffer form
// of message() as a virtual; std::error_category does not, so there it is a
// plain member with the same meaning.
#ifdef BPMD_ZLIB_BOOST_SYSTEM
#define BPMD_ZLIB_MESSAGE_BUF_OVERRIDE override
#else
#define BPMD_ZLIB_MESSAGE_BUF_OVERRIDE
#endif

class error_codes : public boost::beast::error_category
{
public:
    const char* name() const noexcept override { return "boost.beast.zlib"; }

    // impl/error.ipp:57-86
    char const* message(int ev, char*, std::size_t) const noexcept BPMD_ZLIB_MESSAGE_BUF_OVERRIDE
    {
        switch (static_cast<error>(ev)) {
        case error::need_buffers: return "need buffers";
        case error::end_of_stream: return "unexpected end of deflate stream";
        case error::need_dict: return "need dict";
        case error::stream_error: return "stream error";
        case error::invalid_block_type: return "invalid block type";
        case error::invalid_stored_length: return "invalid stored block length";
        case error::too_many_symbols: return "too many symbols";
        case error::invalid_code_lengths: return "invalid code lengths";
        case error::invalid_bit_length_repeat: return "invalid bit length repeat";
        case error::missing_eob: return "missing end of block code";
        case error::invalid_literal_length: return "invalid literal/length code";
        case error::invalid_distance_code: return "invalid distance code";
        case error::invalid_distance: return "invalid distance";
        case error::over_subscribed_length: return "over-subscribed length";
        case error::incomplete_length_set: return "incomplete length set";
        case error::general:
        default: return "beast.zlib error";
        }
    }

    // impl/error.ipp:88-92
    std::string message(int ev) const override { return message(ev, nullptr, 0); }

    // impl/error.ipp:94-98
    boost::beast::error_condition default_error_condition(int ev) const noexcept override
    {
        return boost::beast::error_condition{ev, *this};
    }

    // impl/error.ipp:100-106
    bool equivalent(int ev, boost::beast::error_condition const& condition) const noexcept override
    {
        return condition.value() == ev && &condition.category() == this;
    }

    // impl/error.ipp:108-113
    bool equivalent(boost::beast::error_code const& error, int ev) const noexcept override
    {
        return error.value() == ev && &error.category() == this;
    }
};

inline const boost::beast::error_category& get_error_category()
{
    static const error_codes cat{};
    return cat;
}

}  // namespace detail

inline boost::beast::error_code make_error_code(error ev)
{
    return boost::beast::error_code{static_cast<int>(ev), detail::get_error_category()};
}

}  // namespace zlib
}  // namespace beast
}  // namespace boost

#ifdef BPMD_ZLIB_BOOST_SYSTEM
namespace boost {
namespace system {
template <>
struct is_error_code_enum<::boost::beast::zlib::error> { static bool const value = true; };
}  // namespace system
}  // namespace boost
#else
template <>
struct std::is_error_code_enum<::boost::beast::zlib::error> : std::true_type {};
#endif

#endif
