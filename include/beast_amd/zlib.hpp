// beast_amd/zlib.hpp -- C++ compatibility facade with the surface of
// boost::beast::zlib (include/boost/beast/zlib/{zlib,error,deflate_stream,
// inflate_stream}.hpp), backed by the MI355X engine through the per-stream
// C ABI of include/beast_pmd.h.  Header only; link libbeast_pmd.so.
//
// Names, enum order and member signatures follow the reference so code
// written against boost::beast::zlib compiles after a namespace change.
// Differences:
//   * error codes are std::error_code (category name "boost.beast.zlib",
//     same values) instead of boost::system::error_code;
//   * deflate output is this engine's own parse: a valid stream with
//     Beast's flush framing, not byte-identical to zlib's;
//   * deflate_stream::tune is accepted and ignored (the GPU parser keeps
//     its level's limits);
//   * each write() that has to produce output runs one GPU launch for the
//     buffered message; the batch API (beast_pmd.h) is the throughput path.
#ifndef BEAST_AMD_ZLIB_HPP
#define BEAST_AMD_ZLIB_HPP

#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <system_error>

#include "../beast_pmd.h"

namespace beast_amd {
namespace zlib {

// zlib.hpp:78-144
struct z_params {
    void const* next_in = nullptr;
    std::size_t avail_in = 0;
    std::size_t total_in = 0;
    void* next_out = nullptr;
    std::size_t avail_out = 0;
    std::size_t total_out = 0;
    int data_type = 2;   // unknown
};

// zlib.hpp:159-183 (order matters)
enum class Flush { none, block, partial, sync, full, finish, trees };

// zlib.hpp:197-203
enum compression { none = 0, best_speed = 1, best_size = 9, default_size = -1 };

// zlib.hpp:209-246
enum class Strategy { normal, filtered, huffman, rle, fixed };

// error.hpp:48-138
enum class error {
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
class error_category_impl : public std::error_category {
public:
    const char* name() const noexcept override { return "boost.beast.zlib"; }
    std::string message(int ev) const override
    {
        // impl/error.ipp:41-122
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
};
}  // namespace detail

inline const std::error_category& error_category()
{
    static const detail::error_category_impl cat;
    return cat;
}

inline std::error_code make_error_code(error e) { return std::error_code(static_cast<int>(e), error_category()); }

// deflate_stream.hpp:402-410
inline std::size_t deflate_upper_bound(std::size_t bytes) { return bpmd_deflate_upper_bound(bytes); }

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
inline void assign(std::error_code& ec, int r, const char* what)
{
    if (r == BPMD_R_INVALID_ARGUMENT) throw std::invalid_argument(what);
    if (r == BPMD_R_DOMAIN_ERROR) throw std::domain_error(what);
    if (r < 0) throw std::runtime_error(std::string(what) + ": GPU engine unavailable");
    ec = r ? make_error_code(static_cast<error>(r)) : std::error_code();
}
}  // namespace detail

// deflate_stream.hpp:59-369
class deflate_stream {
public:
    deflate_stream() { reset(6, 15, 9, Strategy::normal); }   // reference default ctor: (6, 15, 9, normal)
    ~deflate_stream() { bpmd_stream_destroy(s_); }
    deflate_stream(const deflate_stream&) = delete;
    deflate_stream& operator=(const deflate_stream&) = delete;

    void reset(int level, int windowBits, int memLevel, Strategy strategy)
    {
        bpmd_stream* n = nullptr;
        int r = bpmd_deflate_stream_create(level, windowBits, memLevel, static_cast<int>(strategy), &n);
        if (r == BPMD_R_INVALID_ARGUMENT) throw std::invalid_argument("invalid level, windowBits or memLevel");
        if (r) throw std::runtime_error("deflate_stream::reset");
        bpmd_stream_destroy(s_);
        s_ = n;
    }
    void reset() { bpmd_deflate_stream_reset(s_); }
    void clear() { bpmd_deflate_stream_reset(s_); }
    std::size_t upper_bound(std::size_t sourceLen) const { return deflate_upper_bound(sourceLen); }
    void tune(int, int, int, int) {}
    void write(z_params& zs, Flush flush, std::error_code& ec)
    {
        bpmd_zparams c = detail::to_c(zs);
        int r = bpmd_deflate_stream_write(s_, &c, static_cast<int>(flush));
        detail::assign(ec, r, "invalid input");
        detail::from_c(zs, c);
    }
    void params(z_params& zs, int level, Strategy strategy, std::error_code& ec)
    {
        bpmd_zparams c = detail::to_c(zs);
        int r = bpmd_deflate_stream_params(s_, &c, level, static_cast<int>(strategy));
        detail::assign(ec, r, "params");
        detail::from_c(zs, c);
    }
    void pending(unsigned* value, int* bits) { bpmd_deflate_stream_pending(s_, value, bits); }
    void prime(int bits, int value, std::error_code& ec) { detail::assign(ec, bpmd_deflate_stream_prime(s_, bits, value), "prime"); }

private:
    bpmd_stream* s_ = nullptr;
};

// inflate_stream.hpp:63-213
class inflate_stream {
public:
    inflate_stream() { reset(15); }
    ~inflate_stream() { bpmd_stream_destroy(s_); }
    inflate_stream(const inflate_stream&) = delete;
    inflate_stream& operator=(const inflate_stream&) = delete;

    void reset() { reset(15); }
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
    void clear() { bpmd_inflate_stream_clear(s_); }
    void write(z_params& zs, Flush flush, std::error_code& ec)
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
}  // namespace beast_amd

template <>
struct std::is_error_code_enum<beast_amd::zlib::error> : std::true_type {};

#endif
