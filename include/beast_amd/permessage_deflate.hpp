// beast_amd/permessage_deflate.hpp -- websocket::permessage_deflate options
// (include/boost/beast/websocket/option.hpp:34-67) and their validation
// (websocket/detail/impl_base.hpp:230-250), plus the mapping from
// negotiated options to the codec configuration the batch API takes
// (impl_base.hpp:277-309).
#ifndef BEAST_AMD_PERMESSAGE_DEFLATE_HPP
#define BEAST_AMD_PERMESSAGE_DEFLATE_HPP

#include <cstddef>
#include <stdexcept>

#include "../beast_pmd.h"

namespace beast_amd {
namespace websocket {

struct permessage_deflate {
    bool server_enable = false;
    bool client_enable = false;
    int server_max_window_bits = 15;
    int client_max_window_bits = 15;
    bool server_no_context_takeover = false;
    bool client_no_context_takeover = false;
    int compLevel = 8;
    int memLevel = 4;
    std::size_t msg_size_threshold = 0;
};

// set_option_pmd (impl_base.hpp:230-250)
inline void validate(const permessage_deflate& o)
{
    if (o.server_max_window_bits > 15 || o.server_max_window_bits < 9)
        throw std::invalid_argument{"invalid server_max_window_bits"};
    if (o.client_max_window_bits > 15 || o.client_max_window_bits < 9)
        throw std::invalid_argument{"invalid client_max_window_bits"};
    if (o.compLevel < 0 || o.compLevel > 9)
        throw std::invalid_argument{"invalid compLevel"};
    if (o.memLevel < 1 || o.memLevel > 9)
        throw std::invalid_argument{"invalid memLevel"};
}

// open_pmd (impl_base.hpp:277-309): the deflater uses our own window bits,
// the inflater the peer's.  `server` is our role.
inline bpmd_cfg deflate_cfg(const permessage_deflate& negotiated, bool server)
{
    bpmd_cfg c{};
    c.level = negotiated.compLevel;
    c.window_bits = server ? negotiated.server_max_window_bits : negotiated.client_max_window_bits;
    c.mem_level = negotiated.memLevel;
    c.strategy = BPMD_STRATEGY_NORMAL;
    c.flags = 0;
    return c;
}

inline bpmd_cfg inflate_cfg(const permessage_deflate& negotiated, bool server)
{
    bpmd_cfg c{};
    c.level = 0;
    c.window_bits = server ? negotiated.client_max_window_bits : negotiated.server_max_window_bits;
    c.mem_level = 8;
    c.strategy = BPMD_STRATEGY_NORMAL;
    c.flags = 0;
    return c;
}

// begin_msg (stream_impl.hpp:225-252): compress this message?
inline bool compress_message(const permessage_deflate& negotiated, bool pmd_enabled, bool wr_compress_opt,
                             std::size_t n)
{
    return pmd_enabled && wr_compress_opt && n >= negotiated.msg_size_threshold;
}

}  // namespace websocket
}  // namespace beast_amd

#endif
