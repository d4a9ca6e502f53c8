// write_threshold.cpp -- the reference's "intelligent compression" tests
// (test/beast/websocket/write.cpp:659-807, issues 226, 227 and 1666) over
// the drop-in surface: begin_msg's decision (stream_impl.hpp:225-231,
// impl_base.hpp:321-324: pmd enabled, compress(true), size >= the
// msg_size_threshold option) via beast_amd::websocket::compress_message,
// then the frame the server writes for one 256-byte message of '*' -- raw,
// or the payload impl_base::deflate produces through zlib::deflate_stream
// (GPU) -- counted as write.cpp's nwrite_bytes delta counts it.
// Usage: write_threshold [cpu|gpu].  Exit 0 = every expectation holds,
// 1 = one failed, 3 = no GPU engine (gpu mode).
#include <beast_amd/permessage_deflate.hpp>
#include <boost/beast/zlib.hpp>

#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

namespace zlib = boost::beast::zlib;
using beast_amd::websocket::permessage_deflate;

// impl_base.hpp:84-154 for a message that fits one 4 KiB write buffer
static long deflate_payload(const std::string& msg)
{
    zlib::deflate_stream zo;
    zo.reset(8, 15, 4, zlib::Strategy::normal);   // option.hpp:61-64 defaults, open_pmd
    std::vector<unsigned char> out(4096);
    zlib::z_params zs;
    zs.next_in = msg.data();
    zs.avail_in = msg.size();
    zs.next_out = out.data();
    zs.avail_out = out.size();
    boost::beast::error_code ec;
    zo.write(zs, zlib::Flush::none, ec);
    if (ec && ec != zlib::error::need_buffers) return ec.value() == 0 ? -1 : -ec.value();
    zo.write(zs, zlib::Flush::block, ec);
    if (ec == zlib::error::need_buffers) ec = {};
    if (ec || zs.avail_out < 6) return -100;
    zo.write(zs, zlib::Flush::sync, ec);
    if (ec) return -101;
    return (long)zs.total_out - 4;
}

// bytes the server's write puts on the wire for one message
static long write_bytes(std::size_t threshold, bool compress_opt, const std::string& s)
{
    permessage_deflate pmd;
    pmd.client_enable = true;
    pmd.server_enable = true;
    pmd.msg_size_threshold = threshold;
    beast_amd::websocket::validate(pmd);
    if (!beast_amd::websocket::compress_message(pmd, true, compress_opt, s.size()))
        return (long)bpmd_frame_wire_size(s.size(), 4096, 0);
    const long p = deflate_payload(s);
    return p < 0 ? p : (long)bpmd_frame_wire_size((uint64_t)p, 4096, 0);
}

int main(int argc, char** argv)
{
    const bool gpu = argc > 1 && std::strcmp(argv[1], "gpu") == 0;
    const std::string s(256, '*');
    int bad = 0;
    // issue 226: threshold 5, compress(false) for this message -> sent raw
    const long n226 = write_bytes(5, false, s);
    bad += !(n226 > (long)s.size());
    // issue 227: threshold 260 > 256 -> sent raw
    const long n227 = write_bytes(260, true, s);
    bad += !(n227 > (long)s.size());
    std::printf("issue226 %ld issue227 %ld\n", n226, n227);
    if (gpu) {
        if (bpmd_init() != BPMD_R_OK) {
            std::printf("no GPU engine\n");
            return 3;
        }
        // issue 1666: default threshold 0 -> compressed, fewer bytes than the message
        const long n1666 = write_bytes(0, true, s);
        bad += !(n1666 > 0 && n1666 < (long)s.size());
        std::printf("issue1666 %ld\n", n1666);
    }
    std::printf(bad ? "FAILED\n" : "ok\n");
    return bad ? 1 : 0;
}
