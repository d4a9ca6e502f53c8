// impl_base_codec.cpp -- compile-only check (tests/test_facade.py) that the
// drop-in zlib headers under include/boost/beast/ accept every use Beast's
// websocket layer makes of the codec.  websocket/detail/impl_base.hpp cannot
// be compiled here (Boost is absent), so its codec calls are restated below
// with the same types, members, enumerators and expressions, each citing the
// line it mirrors; buffers are plain pointers instead of net:: buffers.
#include <boost/beast/zlib.hpp>

#include <cstddef>
#include <cstdint>
#include <string>
#include <system_error>
#include <type_traits>

namespace zlib = boost::beast::zlib;
using boost::beast::error_code;

namespace {

enum class role_type { client, server };

// impl_base.hpp:44-51
struct pmd_type {
    bool rd_set = false;
    std::size_t rd_eb_consumed = 0;
    zlib::deflate_stream zo;
    zlib::inflate_stream zi;
};

struct options {   // the permessage_deflate fields open_pmd reads (option.hpp:34-67)
    int compLevel = 8, memLevel = 4, client_max_window_bits = 15, server_max_window_bits = 15;
    bool client_no_context_takeover = false, server_no_context_takeover = false;
};

struct codec {
    pmd_type pmd;
    options opts;

    // impl_base.hpp:277-305
    void open_pmd(role_type role)
    {
        if (role == role_type::client) {
            pmd.zi.reset(opts.server_max_window_bits);
            pmd.zo.reset(opts.compLevel, opts.client_max_window_bits, opts.memLevel, zlib::Strategy::normal);
        } else {
            pmd.zi.reset(opts.client_max_window_bits);
            pmd.zo.reset(opts.compLevel, opts.server_max_window_bits, opts.memLevel, zlib::Strategy::normal);
        }
    }

    // impl_base.hpp:84-154, one input buffer
    bool deflate(std::uint8_t* out, std::size_t& out_size, const std::uint8_t* in, std::size_t in_size, bool fin,
                 std::size_t& total_in, error_code& ec)
    {
        auto& zo = pmd.zo;
        zlib::z_params zs;
        zs.avail_in = 0;
        zs.next_in = nullptr;
        zs.avail_out = out_size;
        zs.next_out = out;
        if (in_size) {
            zs.avail_in = in_size;
            zs.next_in = in;
            zo.write(zs, zlib::Flush::none, ec);
            if (ec) {
                if (ec != zlib::error::need_buffers) return false;
                ec = {};
            }
        }
        total_in = zs.total_in;
        if (zs.avail_out > 0 && fin && total_in == in_size) {
            zo.write(zs, zlib::Flush::block, ec);
            if (ec == zlib::error::need_buffers) ec = {};
            if (ec) return false;
            if (zs.avail_out >= 6) {
                zo.write(zs, zlib::Flush::sync, ec);
                zs.total_out -= 4;   // remove flush marker
                out_size = zs.total_out;
                return false;
            }
        }
        ec = {};
        out_size = zs.total_out;
        return true;
    }

    // impl_base.hpp:156-166
    void do_context_takeover_write(role_type role)
    {
        if ((role == role_type::client && opts.client_no_context_takeover) ||
            (role == role_type::server && opts.server_no_context_takeover))
            pmd.zo.reset();
    }

    // impl_base.hpp:168-174
    void inflate(zlib::z_params& zs, error_code& ec) { pmd.zi.write(zs, zlib::Flush::sync, ec); }

    // impl_base.hpp:176-190
    void inflate_with_eb(zlib::z_params& zs, error_code& ec)
    {
        const std::uint8_t eb[4] = {0x00, 0x00, 0xff, 0xff};
        zs.next_in = eb + pmd.rd_eb_consumed;
        zs.avail_in = sizeof(eb) - pmd.rd_eb_consumed;
        inflate(zs, ec);
        pmd.rd_eb_consumed += zs.total_in;
        if (ec == zlib::error::need_buffers) ec.clear();
    }

    // impl_base.hpp:192-202
    void do_context_takeover_read(role_type role)
    {
        if ((role == role_type::client && opts.server_no_context_takeover) ||
            (role == role_type::server && opts.client_no_context_takeover))
            pmd.zi.clear();
    }

    // read.hpp:1295-1345: the fields the read loop reads back
    std::size_t read_step(std::uint8_t* out, std::size_t n, const std::uint8_t* in, std::size_t avail, error_code& ec)
    {
        zlib::z_params zs;
        zs.next_out = out;
        zs.avail_out = n;
        zs.avail_in = avail;
        zs.next_in = in;
        inflate(zs, ec);
        return zs.total_in + zs.total_out;
    }
};

// zlib.hpp:78-144, 159-246 and error.hpp: the names and values the
// websocket layer and users rely on
static_assert(std::is_same<decltype(zlib::z_params{}.avail_in), std::size_t>::value, "z_params::avail_in");
static_assert(std::is_same<decltype(zlib::z_params{}.total_out), std::size_t>::value, "z_params::total_out");
static_assert(std::is_same<decltype(zlib::z_params{}.data_type), int>::value, "z_params::data_type");
static_assert(static_cast<int>(zlib::Flush::none) == 0 && static_cast<int>(zlib::Flush::block) == 1 &&
                  static_cast<int>(zlib::Flush::sync) == 3 && static_cast<int>(zlib::Flush::trees) == 6,
              "Flush order");
static_assert(static_cast<int>(zlib::error::need_buffers) == 1 && static_cast<int>(zlib::error::general) == 16,
              "error values");
static_assert(static_cast<int>(zlib::Strategy::normal) == 0 && static_cast<int>(zlib::Strategy::fixed) == 4,
              "Strategy values");

// error.ipp:47-115: the category's observable behaviour
bool category_behaves()
{
    const error_code ec = zlib::make_error_code(zlib::error::invalid_distance);
    const auto& cat = ec.category();
    char buf[8];
    return std::string(cat.name()) == "boost.beast.zlib" && ec.message() == "invalid distance" &&
           std::string(zlib::detail::error_codes{}.message(13, buf, sizeof buf)) == "invalid distance" &&
           cat.default_error_condition(13).value() == 13 && &cat.default_error_condition(13).category() == &cat &&
           cat.equivalent(13, cat.default_error_condition(13)) && cat.equivalent(ec, 13) &&
           ec == zlib::error::invalid_distance && ec != zlib::error::need_buffers;
}

}  // namespace

int impl_base_codec_uses(std::uint8_t* buf, std::size_t n)
{
    codec c;
    c.open_pmd(role_type::server);
    error_code ec;
    std::size_t out_size = n, total_in = 0;
    c.deflate(buf, out_size, buf, n / 2, true, total_in, ec);
    c.do_context_takeover_write(role_type::server);
    zlib::z_params zs;
    zs.next_out = buf;
    zs.avail_out = n;
    c.inflate_with_eb(zs, ec);
    c.do_context_takeover_read(role_type::server);
    return (int)(c.read_step(buf, n, buf, n, ec) + zlib::deflate_upper_bound(n)) + (category_behaves() ? 1 : 0);
}
