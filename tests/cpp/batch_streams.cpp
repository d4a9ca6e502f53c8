// SURVEY §8(f) N2 through the drop-in headers: T threads, each one
// connection's codec pair (a never-reset zlib::deflate_stream and
// zlib::inflate_stream, context takeover on, as the default negotiation
// leaves them), run impl_base<true>'s deflate call sequence
// (impl_base.hpp:85-154) and the read path's inflate + inflate_with_eb
// (read.hpp:1284-1356, impl_base.hpp:168-190) on M messages each, all at the
// same time.  The GPU build runs that twice -- the micro-batcher off, then on
// (bpmd_stream_batching) -- and checks every payload byte and every round
// trip; it prints both times and the batcher's call and launch counts.  Built
// against tests/cpp/oracle_backend.c (-DBPMD_CPU_BACKEND) it times the same
// threads on Beast's codec restated in C, on the CPU.
// Usage: batch_streams [threads=64] [messages=32] [bytes=1024]
// Exit 0 = ok; 1 = mismatch; 3 = no GPU engine available.
#include <boost/beast/zlib.hpp>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace zlib = boost::beast::zlib;

using Bytes = std::vector<unsigned char>;

static Bytes ws_deflate(zlib::deflate_stream& zo, const std::string& msg, std::size_t wr_buf)
{
    Bytes payload;
    std::size_t consumed = 0;
    for (;;) {
        Bytes out(wr_buf);
        zlib::z_params zs;
        zs.next_in = nullptr;
        zs.avail_in = 0;
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

static std::string ws_inflate(zlib::inflate_stream& zi, const Bytes& p)
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

// connection t's message m: JSON records, sizes varying around `bytes`
static std::string message(int t, int m, std::size_t bytes)
{
    const std::size_t n = bytes / 2 + (std::size_t)((t * 131 + m * 977) % (int)(bytes + 1));
    std::string s;
    for (int i = 0; s.size() < n; ++i)
        s += "{\"conn\":" + std::to_string(t) + ",\"seq\":" + std::to_string(m * 1000 + i) + ",\"v\":\"" +
             std::to_string((i * 2654435761u + (unsigned)t) % 100000) + "\"},";
    s.resize(n);
    return s;
}

struct Run {
    std::vector<std::vector<Bytes>> payloads;   // [thread][message]
    double seconds = 0;
    std::size_t bytes = 0;
    bool ok = true;
    bool engine = true;
};

static Run run_all(int T, int M, std::size_t bytes)
{
    Run r;
    r.payloads.resize(T);
    std::atomic<int> ready{0}, bad{0}, noeng{0};
    std::atomic<bool> go{false};
    std::vector<std::size_t> sent(T, 0);
    // each thread's finish time, taken before its codecs are destroyed (a
    // stream's teardown frees HIP resources: not part of the messages' time)
    std::vector<std::chrono::steady_clock::time_point> fin(T);
    std::vector<std::thread> ts;
    for (int t = 0; t < T; ++t)
        ts.emplace_back([&, t] {
            try {
                zlib::deflate_stream zo;
                zlib::inflate_stream zi;
                zo.reset(6, 15, 8, zlib::Strategy::normal);
                zi.reset(15);
                std::vector<std::string> msgs;
                for (int m = 0; m < M; ++m) msgs.push_back(message(t, m, bytes));
                // one untimed message first: the streams' device state, HIP
                // streams and staging buffers are allocated by their first call
                const std::string w = message(t, M + 1, bytes);
                if (ws_inflate(zi, ws_deflate(zo, w, 4096)) != w) bad.fetch_add(1);
                ready.fetch_add(1);
                while (!go.load()) std::this_thread::yield();
                for (int m = 0; m < M; ++m) {
                    Bytes p = ws_deflate(zo, msgs[m], 4096);
                    if (ws_inflate(zi, p) != msgs[m]) bad.fetch_add(1);
                    sent[t] += msgs[m].size();
                    r.payloads[t].push_back(std::move(p));
                }
                fin[t] = std::chrono::steady_clock::now();
            } catch (const std::runtime_error& e) {
                if (noeng.fetch_add(1) == 0) std::fprintf(stderr, "thread %d: %s\n", t, e.what());
                ready.fetch_add(1);
            }
        });
    while (ready.load() < T) std::this_thread::yield();
    const auto t0 = std::chrono::steady_clock::now();
    go.store(true);
    for (auto& th : ts) th.join();
    auto t1 = t0;
    for (const auto& f : fin) t1 = std::max(t1, f);
    r.seconds = std::chrono::duration<double>(t1 - t0).count();
    for (std::size_t b : sent) r.bytes += b;
    r.ok = bad.load() == 0;
    r.engine = noeng.load() == 0;
    return r;
}

int main(int argc, char** argv)
{
    const int T = argc > 1 ? std::atoi(argv[1]) : 64;
    const int M = argc > 2 ? std::atoi(argv[2]) : 32;
    const std::size_t bytes = argc > 3 ? (std::size_t)std::atoll(argv[3]) : 1024;
    auto rate = [](const Run& r) { return r.bytes / r.seconds / 1e6; };
#ifdef BPMD_CPU_BACKEND
    const Run c = run_all(T, M, bytes);
    if (!c.engine) return 3;
    if (!c.ok) return 1;
    std::printf("cpu codec: %d threads x %d messages, %zu B, %.3f s, %.1f MB/s round trip\n", T, M, c.bytes,
                c.seconds, rate(c));
    return 0;
#else
    unsigned long long st[4];
    // BATCH_STREAMS_ONLY_BATCHED=1 (profiling): the batched run alone
    const char* ob = std::getenv("BATCH_STREAMS_ONLY_BATCHED");
    const bool only_batched = ob && ob[0] == '1';
    bpmd_stream_batching(0, 0);
    const Run a = only_batched ? Run{} : run_all(T, M, bytes);
    if (!a.engine) return 3;
    bpmd_stream_batch_stats(st, 1);
    bpmd_stream_batching(256, 0);
    const Run b = run_all(T, M, bytes);
    if (!b.engine) return 3;
    bpmd_stream_batch_stats(st, 1);
    bpmd_stream_batching(256, 0);   // the default again
    if (!a.ok || !b.ok) {
        std::fprintf(stderr, "round trip mismatch: unbatched %d batched %d\n", (int)a.ok, (int)b.ok);
        return 1;
    }
    for (int t = 0; t < T && !only_batched; ++t)
        if (a.payloads[t] != b.payloads[t]) {
            std::fprintf(stderr, "thread %d: batched payloads differ from unbatched\n", t);
            return 1;
        }
    std::printf("unbatched: %d threads x %d messages, %zu B, %.3f s, %.1f MB/s round trip\n", T, M, a.bytes,
                a.seconds, rate(a));
    std::printf("batched: %.3f s, %.1f MB/s round trip; inflate calls %llu launches %llu; deflate flushes %llu "
                "launches %llu\n",
                b.seconds, rate(b), st[0], st[1], st[2], st[3]);
    std::printf("payloads equal: %d x %d\n", T, M);
    return 0;
#endif
}
