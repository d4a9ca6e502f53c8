// Drop-in check of the C++ facade: the exact call sequence of
// impl_base<true>::deflate (impl_base.hpp:85-154) and of the sync read path
// with inflate_with_eb (read.hpp:1284-1356, impl_base.hpp:168-190), written
// against boost::beast::zlib exactly as Beast writes it, compiled against the
// drop-in headers (include/boost/beast/zlib/).  One inflater for all messages,
// never reset (Beast resets zi only in open_pmd, impl_base.hpp:277-309).
// Exit 0 = round trip ok; 3 = no GPU engine available.
#include <beast_amd/permessage_deflate.hpp>
#include <boost/beast/zlib.hpp>

#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace zlib = boost::beast::zlib;

static std::vector<unsigned char> ws_deflate(zlib::deflate_stream& zo, const std::string& msg, std::size_t wr_buf)
{
    std::vector<unsigned char> payload;
    std::size_t consumed = 0;
    for (;;) {
        std::vector<unsigned char> out(wr_buf);
        zlib::z_params zs;
        zs.avail_out = out.size();
        zs.next_out = out.data();
        boost::beast::error_code ec;
        while (consumed + zs.total_in < msg.size()) {
            zs.next_in = msg.data() + consumed + zs.total_in;
            zs.avail_in = std::min<std::size_t>(1000, msg.size() - consumed - zs.total_in);
            zo.write(zs, zlib::Flush::none, ec);
            if (ec) { if (ec != zlib::error::need_buffers) throw std::runtime_error("deflate"); ec = {}; break; }
            if (zs.avail_out == 0) break;
        }
        consumed += zs.total_in;
        if (zs.avail_out > 0 && consumed == msg.size()) {
            zo.write(zs, zlib::Flush::block, ec);
            if (ec == zlib::error::need_buffers) ec = {};
            if (ec) throw std::runtime_error("block");
            if (zs.avail_out >= 6) {
                zo.write(zs, zlib::Flush::sync, ec);
                if (ec) throw std::runtime_error("sync");
                zs.total_out -= 4;   // remove flush marker
                payload.insert(payload.end(), out.begin(), out.begin() + zs.total_out);
                return payload;
            }
        }
        payload.insert(payload.end(), out.begin(), out.begin() + zs.total_out);
    }
}

static std::string ws_inflate(zlib::inflate_stream& zi, const std::vector<unsigned char>& p)
{
    std::string out;
    std::size_t pos = 0;
    std::vector<char> buf(4096);
    boost::beast::error_code ec;
    while (pos < p.size()) {
        zlib::z_params zs;
        zs.next_in = p.data() + pos;
        zs.avail_in = std::min<std::size_t>(1536, p.size() - pos);
        zs.next_out = buf.data();
        zs.avail_out = buf.size();
        zi.write(zs, zlib::Flush::sync, ec);
        if (ec && ec != zlib::error::need_buffers) throw std::runtime_error("inflate " + ec.message());
        pos += zs.total_in;
        out.append(buf.data(), zs.total_out);
    }
    const unsigned char eb[4] = {0x00, 0x00, 0xff, 0xff};
    std::size_t eb_used = 0;
    for (;;) {
        zlib::z_params zs;
        zs.next_in = eb + eb_used;
        zs.avail_in = 4 - eb_used;
        zs.next_out = buf.data();
        zs.avail_out = buf.size();
        zi.write(zs, zlib::Flush::sync, ec);
        if (ec == zlib::error::need_buffers) ec = {};
        if (ec) throw std::runtime_error("inflate_with_eb " + ec.message());
        eb_used += zs.total_in;
        out.append(buf.data(), zs.total_out);
        if (zs.total_out == 0) break;
    }
    return out;
}

int main()
{
    beast_amd::websocket::permessage_deflate o;
    o.server_enable = true;
    o.compLevel = 6;
    o.server_no_context_takeover = true;
    beast_amd::websocket::validate(o);
    try {
        bool threw = false;
        try { beast_amd::websocket::permessage_deflate b = o; b.memLevel = 0; beast_amd::websocket::validate(b); }
        catch (const std::invalid_argument&) { threw = true; }
        if (!threw) return 1;
        zlib::deflate_stream zo;
        zlib::inflate_stream zi;
        const bpmd_cfg c = beast_amd::websocket::deflate_cfg(o, true);
        zo.reset(c.level, c.window_bits, c.mem_level, zlib::Strategy::normal);
        zi.reset(beast_amd::websocket::inflate_cfg(o, true).window_bits);
        for (int m = 0; m < 4; ++m) {
            std::string msg;
            for (int i = 0; msg.size() < (std::size_t)(1000 + 3000 * m); ++i)
                msg += "{\"id\":" + std::to_string(i * 7 + m) + ",\"name\":\"user" + std::to_string(i % 13) + "\"},";
            auto payload = ws_deflate(zo, msg, 4096);
            zo.reset();   // do_context_takeover_write under server_no_context_takeover
            std::string back = ws_inflate(zi, payload);
            if (back != msg) {
                std::fprintf(stderr, "mismatch on message %d: %zu vs %zu bytes\n", m, back.size(), msg.size());
                return 1;
            }
            std::printf("message %d: %zu -> %zu bytes ok\n", m, msg.size(), payload.size());
        }
    } catch (const std::runtime_error& e) {
        std::fprintf(stderr, "engine unavailable: %s\n", e.what());
        return 3;
    }
    return 0;
}
