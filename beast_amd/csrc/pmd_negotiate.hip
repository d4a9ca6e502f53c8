// pmd_negotiate.hip -- permessage-deflate extension negotiation (SURVEY.md
// §8(f) N4, second half): the Sec-WebSocket-Extensions wire format Beast's
// handshake reads and writes (websocket/detail/pmd_extension.hpp/.ipp), for
// a facade that owns the handshake.  Host code only; no device use.
//
//   bpmd_pmd_read       pmd_read / pmd_read_impl       pmd_extension.ipp:45-166
//   bpmd_pmd_write      pmd_write / pmd_write_impl     pmd_extension.ipp:168-208
//   bpmd_pmd_negotiate  pmd_negotiate(_impl)           pmd_extension.hpp:95-111, .ipp:210-290
//   bpmd_pmd_normalize  pmd_normalize                  pmd_extension.ipp:292-305
//
// The header value is split as Beast's http::ext_list does (RFC 7230
// extension lists: comma-separated extensions, ';'-separated parameters,
// token or quoted-string values; "name=" is a parameter with an empty value).
#include <stddef.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../include/beast_pmd.h"

namespace {

struct Param {
    std::string name, value;
};
struct Ext {
    std::string name;
    std::vector<Param> params;
};

bool is_ows(char c) { return c == ' ' || c == '\t'; }

bool is_tchar(char c)
{
    if ((c >= '0' && c <= '9') || (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z')) return true;
    return strchr("!#$%&'*+-.^_`|~", c) != nullptr && c != 0;
}

bool iequals(const std::string& a, const char* b)
{
    const size_t n = strlen(b);
    if (a.size() != n) return false;
    for (size_t i = 0; i < n; ++i) {
        char x = a[i], y = b[i];
        if (x >= 'A' && x <= 'Z') x = (char)(x - 'A' + 'a');
        if (y >= 'A' && y <= 'Z') y = (char)(y - 'A' + 'a');
        if (x != y) return false;
    }
    return true;
}

// ext-list = *( "," OWS ) ext *( OWS "," [ OWS ext ] ); ext = token *( OWS ";" OWS param );
// param = token OWS [ "=" OWS ( token / quoted-string ) ].  Parsing stops at
// the first malformed element, as the reference's iterators do.
std::vector<Ext> parse_ext_list(const char* s, size_t n)
{
    std::vector<Ext> out;
    size_t i = 0;
    auto skip_ows = [&] { while (i < n && is_ows(s[i])) ++i; };
    auto token = [&](std::string& t) {
        const size_t b = i;
        while (i < n && is_tchar(s[i])) ++i;
        t.assign(s + b, i - b);
        return i > b;
    };
    for (;;) {
        while (i < n && (s[i] == ',' || is_ows(s[i]))) ++i;
        if (i >= n) break;
        Ext e;
        if (!token(e.name)) break;
        bool bad = false;
        for (;;) {
            skip_ows();
            if (i >= n || s[i] != ';') break;
            ++i;
            skip_ows();
            Param p;
            if (!token(p.name)) { bad = true; break; }
            skip_ows();
            if (i < n && s[i] == '=') {
                ++i;
                skip_ows();
                if (i < n && s[i] == '"') {
                    ++i;
                    bool closed = false;
                    while (i < n) {
                        if (s[i] == '\\' && i + 1 < n) { p.value += s[i + 1]; i += 2; continue; }
                        if (s[i] == '"') { ++i; closed = true; break; }
                        p.value += s[i++];
                    }
                    if (!closed) { bad = true; break; }
                } else {
                    token(p.value);   // may be empty: "name="
                }
            }
            e.params.push_back(p);
        }
        out.push_back(e);
        if (bad) break;
        skip_ows();
        if (i < n && s[i] != ',') break;
    }
    return out;
}

// parse_bits (pmd_extension.ipp:21-43): 1-2 digits, no leading zero
int parse_bits(const std::string& s)
{
    if (s.empty() || s.size() > 2 || s[0] < '1' || s[0] > '9') return -1;
    int v = 0;
    for (char c : s) {
        if (c < '0' || c > '9') return -1;
        v = 10 * v + (c - '0');
    }
    return v;
}

int put(char* out, size_t cap, const std::string& s)
{
    if (!out || cap < s.size() + 1) return BPMD_R_INVALID_ARGUMENT;
    memcpy(out, s.data(), s.size());
    out[s.size()] = 0;
    return (int)s.size();
}

}  // namespace

extern "C" int bpmd_pmd_read(const char* ext, size_t n, bpmd_pmd_offer* offer)
{
    if (!offer || (n && !ext)) return BPMD_R_INVALID_ARGUMENT;
    bpmd_pmd_offer o{};
    *offer = o;
    // the reference fills the offer as it goes and leaves it declined on any defect
    auto decline = [&] {
        o.accept = 0;
        *offer = o;
        return BPMD_R_OK;
    };
    for (const Ext& e : parse_ext_list(ext, n)) {
        if (!iequals(e.name, "permessage-deflate")) continue;
        // the first permessage-deflate offer decides
        for (const Param& p : e.params) {
            if (iequals(p.name, "server_max_window_bits")) {
                if (o.server_max_window_bits != 0 || p.value.empty()) return decline();
                o.server_max_window_bits = parse_bits(p.value);
                if (o.server_max_window_bits < 8 || o.server_max_window_bits > 15) return decline();
            } else if (iequals(p.name, "client_max_window_bits")) {
                if (o.client_max_window_bits != 0) return decline();
                if (p.value.empty()) {
                    o.client_max_window_bits = -1;
                } else {
                    o.client_max_window_bits = parse_bits(p.value);
                    if (o.client_max_window_bits < 8 || o.client_max_window_bits > 15) return decline();
                }
            } else if (iequals(p.name, "server_no_context_takeover")) {
                if (o.server_no_context_takeover || !p.value.empty()) return decline();
                o.server_no_context_takeover = 1;
            } else if (iequals(p.name, "client_no_context_takeover")) {
                if (o.client_no_context_takeover || !p.value.empty()) return decline();
                o.client_no_context_takeover = 1;
            } else {
                return decline();   // a parameter not defined for an offer
            }
        }
        o.accept = 1;
        *offer = o;
        return BPMD_R_OK;
    }
    return BPMD_R_OK;
}

extern "C" int bpmd_pmd_write(const bpmd_pmd_offer* offer, char* out, size_t cap)
{
    if (!offer) return BPMD_R_INVALID_ARGUMENT;
    std::string s = "permessage-deflate";
    auto bits = [&](const char* name, int v) {
        if (v == 0) return;
        s += "; ";
        s += name;
        if (v != -1) s += "=" + std::to_string(v);
    };
    bits("server_max_window_bits", offer->server_max_window_bits);
    bits("client_max_window_bits", offer->client_max_window_bits);
    if (offer->server_no_context_takeover) s += "; server_no_context_takeover";
    if (offer->client_no_context_takeover) s += "; client_no_context_takeover";
    return put(out, cap, s);
}

extern "C" int bpmd_pmd_negotiate(const bpmd_pmd_options* o, const bpmd_pmd_offer* offer, bpmd_pmd_offer* config,
                                  char* out, size_t cap)
{
    if (!o || !offer || !config) return BPMD_R_INVALID_ARGUMENT;
    bpmd_pmd_offer c{};
    if (!(offer->accept && o->server_enable)) {
        *config = c;
        return put(out, cap, "") < 0 ? BPMD_R_INVALID_ARGUMENT : 0;
    }
    c.accept = 1;
    std::string s = "permessage-deflate";
    c.server_no_context_takeover = offer->server_no_context_takeover || o->server_no_context_takeover;
    if (c.server_no_context_takeover) s += "; server_no_context_takeover";
    c.client_no_context_takeover = o->client_no_context_takeover || offer->client_no_context_takeover;
    if (c.client_no_context_takeover) s += "; client_no_context_takeover";
    c.server_max_window_bits = offer->server_max_window_bits != 0
                                   ? (offer->server_max_window_bits < o->server_max_window_bits
                                          ? offer->server_max_window_bits
                                          : o->server_max_window_bits)
                                   : o->server_max_window_bits;
    if (c.server_max_window_bits < 15) {
        // deflate cannot use 8 (zlib's deflateInit treats it as 9): answer 9
        if (c.server_max_window_bits < 9) c.server_max_window_bits = 9;
        s += "; server_max_window_bits=" + std::to_string(c.server_max_window_bits);
    }
    switch (offer->client_max_window_bits) {
    case -1:   // present without a value: our setting
        c.client_max_window_bits = o->client_max_window_bits;
        if (c.client_max_window_bits < 15) s += "; client_max_window_bits=" + std::to_string(c.client_max_window_bits);
        break;
    case 0:    // absent: the response must not carry it, so only 15 works
        if (o->client_max_window_bits == 15) c.client_max_window_bits = 15;
        else c.accept = 0;
        break;
    default:   // 8..15
        c.client_max_window_bits = o->client_max_window_bits < offer->client_max_window_bits
                                       ? o->client_max_window_bits
                                       : offer->client_max_window_bits;
        s += "; client_max_window_bits=" + std::to_string(c.client_max_window_bits);
        break;
    }
    *config = c;
    return put(out, cap, c.accept ? s : std::string());
}

extern "C" void bpmd_pmd_normalize(bpmd_pmd_offer* offer)
{
    if (!offer || !offer->accept) return;
    if (offer->server_max_window_bits == 0) offer->server_max_window_bits = 15;
    if (offer->client_max_window_bits == 0 || offer->client_max_window_bits == -1) offer->client_max_window_bits = 15;
}
