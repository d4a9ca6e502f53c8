// C1 (BASELINE.json configs[0]): a WebSocket echo over loopback with
// permessage-deflate on, 1 Ki x 1 KiB text messages, driven through the
// drop-in boost::beast::zlib headers (include/boost/beast/zlib/) -- i.e. the
// GPU engine -- by a socketpair harness that restates the websocket layer's
// pmd data path (Boost.Asio is not in this image):
//
//   write side   impl_base<true>::deflate (impl_base.hpp:85-154) with a
//                4096-byte wr_buf, frames with RSV1 on the first frame
//                (write.hpp:655-703), masked by the client (write.hpp:679-685)
//   read side    frame header parse, unmask (read.hpp:1324-1327), inflate in
//                rd_buf slices of <= 1536 bytes with Flush::sync, then
//                inflate_with_eb until a call produces nothing
//                (read.hpp:1284-1356, impl_base.hpp:168-190), UTF-8 check of
//                the text (read.hpp:1372-1384)
//   takeover     the default: no *_no_context_takeover, so neither side ever
//                resets its deflater or inflater (impl_base.hpp:156-202)
//
// The client sends each message, the server echoes what it received, the
// client checks the echo byte for byte.  Exit 0 = all messages echoed
// exactly; 1 = mismatch / protocol error; 3 = no GPU engine.
#include <boost/beast/zlib.hpp>

#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace zlib = boost::beast::zlib;

namespace {

struct Fail : std::runtime_error {
    using std::runtime_error::runtime_error;
};

void write_all(int fd, const void* p, size_t n)
{
    const char* c = static_cast<const char*>(p);
    while (n) {
        ssize_t k = ::write(fd, c, n);
        if (k <= 0) throw Fail("socket write");
        c += k;
        n -= (size_t)k;
    }
}

void read_all(int fd, void* p, size_t n)
{
    char* c = static_cast<char*>(p);
    while (n) {
        ssize_t k = ::read(fd, c, n);
        if (k <= 0) throw Fail("socket read");
        c += k;
        n -= (size_t)k;
    }
}

// mask_inplace (websocket/detail/mask.ipp:38-59) for a frame that starts at key phase 0
void mask(unsigned char* p, size_t n, uint32_t key)
{
    for (size_t i = 0; i < n; ++i) p[i] ^= (unsigned char)(key >> (8 * (i & 3)));
}

// utf8_checker (websocket/detail/utf8_checker.ipp) for a whole message
bool utf8_ok(const std::string& s)
{
    size_t i = 0;
    const auto* u = reinterpret_cast<const unsigned char*>(s.data());
    while (i < s.size()) {
        const unsigned c = u[i];
        size_t need;
        unsigned lo = 0x80, hi = 0xBF;
        if (c < 0x80) { ++i; continue; }
        else if (c >= 0xC2 && c <= 0xDF) need = 1;
        else if (c >= 0xE0 && c <= 0xEF) { need = 2; if (c == 0xE0) lo = 0xA0; if (c == 0xED) hi = 0x9F; }
        else if (c >= 0xF0 && c <= 0xF4) { need = 3; if (c == 0xF0) lo = 0x90; if (c == 0xF4) hi = 0x8F; }
        else return false;
        for (size_t k = 1; k <= need; ++k) {
            if (i + k >= s.size()) return false;
            const unsigned d = u[i + k];
            const unsigned l = k == 1 ? lo : 0x80, h = k == 1 ? hi : 0xBF;
            if (d < l || d > h) return false;
        }
        i += need + 1;
    }
    return true;
}

// One side of a connection: its own deflater and inflater (pmd_type,
// impl_base.hpp:45-55), opened as open_pmd does (impl_base.hpp:277-309).
class Endpoint {
public:
    Endpoint(int fd, bool client, int level, int mem_level) : fd_(fd), client_(client), key_(0x9e3779b9u)
    {
        zo_.reset(level, 15, mem_level, zlib::Strategy::normal);
        zi_.reset(15);
    }

    // write.hpp:621-703 (sync write_some with fin = true) over impl_base::deflate
    void send_text(const std::string& msg)
    {
        std::vector<unsigned char> wr_buf(4096);
        size_t consumed = 0;
        bool first = true;
        for (;;) {
            zlib::z_params zs;
            zs.next_in = nullptr;
            zs.avail_in = 0;
            zs.next_out = wr_buf.data();
            zs.avail_out = wr_buf.size();
            boost::beast::error_code ec;
            // impl_base.hpp:96-120: every input buffer with Flush::none
            while (consumed + zs.total_in < msg.size()) {
                zs.next_in = msg.data() + consumed + zs.total_in;
                zs.avail_in = msg.size() - consumed - zs.total_in;
                zo_.write(zs, zlib::Flush::none, ec);
                if (ec) {
                    if (ec != zlib::error::need_buffers) throw Fail("deflate: " + ec.message());
                    ec = {};
                    break;
                }
                if (zs.avail_out == 0) break;
            }
            consumed += zs.total_in;
            bool fin = false;
            // impl_base.hpp:121-148: at the end, Flush::block then Flush::sync and strip 00 00 FF FF
            if (zs.avail_out > 0 && consumed == msg.size()) {
                zo_.write(zs, zlib::Flush::block, ec);
                if (ec == zlib::error::need_buffers) ec = {};
                if (ec) throw Fail("deflate block: " + ec.message());
                if (zs.avail_out >= 6) {
                    zo_.write(zs, zlib::Flush::sync, ec);
                    if (ec) throw Fail("deflate sync: " + ec.message());
                    zs.total_out -= 4;
                    fin = true;
                }
            }
            send_frame(first ? 1 : 0, first, fin, wr_buf.data(), zs.total_out);
            first = false;
            if (fin) return;
        }
    }

    // read.hpp:989-1040 / 1063-1385: one whole message
    std::string recv_text()
    {
        std::string out;
        bool fin = false, first = true;
        while (!fin) {
            unsigned char h[2];
            read_all(fd_, h, 2);
            fin = (h[0] & 0x80) != 0;
            const bool rsv1 = (h[0] & 0x40) != 0;
            const unsigned op = h[0] & 0x0F;
            if (first && (op != 1 || !rsv1)) throw Fail("expected a compressed text frame");
            if (!first && (op != 0 || rsv1)) throw Fail("expected a continuation frame");
            first = false;
            const bool masked = (h[1] & 0x80) != 0;
            uint64_t len = h[1] & 0x7F;
            if (len == 126) {
                unsigned char e[2];
                read_all(fd_, e, 2);
                len = ((uint64_t)e[0] << 8) | e[1];
            } else if (len == 127) {
                unsigned char e[8];
                read_all(fd_, e, 8);
                len = 0;
                for (int i = 0; i < 8; ++i) len = (len << 8) | e[i];
            }
            uint32_t key = 0;
            if (masked) {
                unsigned char k[4];
                read_all(fd_, k, 4);
                key = (uint32_t)k[0] | ((uint32_t)k[1] << 8) | ((uint32_t)k[2] << 16) | ((uint32_t)k[3] << 24);
            }
            if (masked == client_) throw Fail("masking direction");
            // rd_buf slices of <= 1536 bytes, each fed with Flush::sync
            uint64_t done = 0;
            unsigned char rd_buf[1536];
            while (done < len) {
                const size_t k = (size_t)std::min<uint64_t>(sizeof rd_buf, len - done);
                read_all(fd_, rd_buf, k);
                if (masked) {   // the frame's key phase after `done` bytes
                    const unsigned ph = (unsigned)(done & 3);
                    const uint32_t rk = ph ? ((key >> (8 * ph)) | (key << (32 - 8 * ph))) : key;
                    mask(rd_buf, k, rk);
                }
                size_t used = 0;
                while (used < k) {
                    used += inflate_some(rd_buf + used, k - used, out);
                }
                done += k;
            }
        }
        // inflate_with_eb until a call produces nothing (read.hpp:1345-1356)
        const unsigned char eb[4] = {0x00, 0x00, 0xff, 0xff};
        size_t eb_used = 0;
        for (;;) {
            std::vector<char> buf(4096);
            zlib::z_params zs;
            zs.next_in = eb + eb_used;
            zs.avail_in = 4 - eb_used;
            zs.next_out = buf.data();
            zs.avail_out = buf.size();
            boost::beast::error_code ec;
            zi_.write(zs, zlib::Flush::sync, ec);
            if (ec == zlib::error::need_buffers) ec = {};
            if (ec) throw Fail("inflate_with_eb: " + ec.message());
            eb_used += zs.total_in;
            out.append(buf.data(), zs.total_out);
            if (zs.total_out == 0) break;
        }
        zi_.clear();   // do_context_takeover_read: a no-op here too
        if (!utf8_ok(out)) throw Fail("bad_frame_payload");
        return out;
    }

    size_t frames = 0, wire_bytes = 0;

private:
    // impl_base::inflate (impl_base.hpp:168-174): one zi.write into the user's buffer
    size_t inflate_some(const unsigned char* p, size_t n, std::string& out)
    {
        std::vector<char> buf(4096);
        zlib::z_params zs;
        zs.next_in = p;
        zs.avail_in = n;
        zs.next_out = buf.data();
        zs.avail_out = buf.size();
        boost::beast::error_code ec;
        zi_.write(zs, zlib::Flush::sync, ec);
        if (ec) throw Fail("inflate: " + ec.message());   // check_stop_now (read.hpp:1337)
        out.append(buf.data(), zs.total_out);
        if (zs.total_in == 0 && zs.total_out == 0) throw Fail("inflate made no progress");
        return zs.total_in;
    }

    void send_frame(unsigned op, bool rsv1, bool fin, unsigned char* p, size_t n)
    {
        unsigned char h[14];
        size_t hn = 2;
        h[0] = (unsigned char)((fin ? 0x80 : 0) | (rsv1 ? 0x40 : 0) | op);
        const unsigned char m = client_ ? 0x80 : 0;
        if (n < 126) {
            h[1] = (unsigned char)(m | n);
        } else if (n < 65536) {
            h[1] = (unsigned char)(m | 126);
            h[2] = (unsigned char)(n >> 8);
            h[3] = (unsigned char)n;
            hn = 4;
        } else {
            h[1] = (unsigned char)(m | 127);
            for (int i = 0; i < 8; ++i) h[2 + i] = (unsigned char)((uint64_t)n >> (56 - 8 * i));
            hn = 10;
        }
        if (client_) {
            key_ = key_ * 1103515245u + 12345u;
            for (int i = 0; i < 4; ++i) h[hn + i] = (unsigned char)(key_ >> (8 * i));
            hn += 4;
            mask(p, n, key_);
        }
        write_all(fd_, h, hn);
        write_all(fd_, p, n);
        ++frames;
        wire_bytes += hn + n;
    }

    int fd_;
    bool client_;
    uint32_t key_;
    zlib::deflate_stream zo_;
    zlib::inflate_stream zi_;
};

std::string make_message(unsigned i, size_t n)
{
    // JSON-like text with a little UTF-8, so the text check has work to do
    static const char* keys[] = {"id", "user", "ts", "price", "qty", "side", "venue", "note"};
    std::string s = "{";
    uint64_t x = 0x5EED0001ull ^ (i * 0x9E3779B97F4A7C15ull);
    while (s.size() < n) {
        x ^= x >> 12;
        x ^= x << 25;
        x ^= x >> 27;
        const uint64_t r = x * 0x2545F4914F6CDD1Dull;
        s += "\"";
        s += keys[r % 8];
        s += "\":";
        if ((r >> 8) % 3 == 0) s += std::to_string((r >> 16) % 100000);
        else if ((r >> 8) % 3 == 1) s += std::to_string((r >> 20) % 1000) + "." + std::to_string((r >> 40) % 100);
        else s += "\"caf\xc3\xa9-" + std::to_string((r >> 24) % 97) + "\"";
        s += ",";
    }
    // cut at a character boundary, then pad to exactly n bytes
    size_t cut = n;
    while (cut > 0 && cut < s.size() && ((unsigned char)s[cut] & 0xC0) == 0x80) --cut;
    s.resize(cut);
    s.append(n - cut, ' ');
    return s;
}

}  // namespace

int main(int argc, char** argv)
{
    const unsigned n_msgs = argc > 1 ? (unsigned)std::stoul(argv[1]) : 1024u;
    const size_t msg_bytes = argc > 2 ? (size_t)std::stoul(argv[2]) : 1024u;
    int sv[2];
    if (socketpair(AF_UNIX, SOCK_STREAM, 0, sv) != 0) return 1;
    int rc = 0;
    bool no_engine = false;
    std::string err;
    size_t wire_c2s = 0, wire_s2c = 0;
    const auto t0 = std::chrono::steady_clock::now();
    // websocket::permessage_deflate defaults (option.hpp:61-64): compLevel 8, memLevel 4
    std::thread server([&] {
        try {
            Endpoint srv(sv[1], false, 8, 4);
            for (unsigned i = 0; i < n_msgs; ++i) srv.send_text(srv.recv_text());
            wire_s2c = srv.wire_bytes;
        } catch (const Fail& e) {
            err = std::string("server: ") + e.what();
        } catch (const std::runtime_error& e) {
            no_engine = true;
        }
        ::shutdown(sv[1], SHUT_RDWR);
    });
    try {
        Endpoint client(sv[0], true, 8, 4);
        for (unsigned i = 0; i < n_msgs; ++i) {
            const std::string m = make_message(i, msg_bytes);
            client.send_text(m);
            const std::string back = client.recv_text();
            if (back != m) {
                std::fprintf(stderr, "echo mismatch on message %u (%zu vs %zu bytes)\n", i, back.size(), m.size());
                rc = 1;
                break;
            }
        }
        wire_c2s = client.wire_bytes;
    } catch (const Fail& e) {
        std::fprintf(stderr, "client: %s\n", e.what());
        rc = 1;
    } catch (const std::runtime_error& e) {
        std::fprintf(stderr, "engine unavailable: %s\n", e.what());
        no_engine = true;
    }
    ::shutdown(sv[0], SHUT_RDWR);
    server.join();
    if (no_engine) return 3;
    if (!err.empty()) {
        std::fprintf(stderr, "%s\n", err.c_str());
        rc = 1;
    }
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (rc == 0)
        std::printf("echo ok: %u messages x %zu B, wire %zu B client->server, %zu B server->client, %.3f s\n", n_msgs,
                    msg_bytes, wire_c2s, wire_s2c, s);
    ::close(sv[0]);
    ::close(sv[1]);
    return rc;
}
