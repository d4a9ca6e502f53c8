// huff_table.h -- canonical-Huffman decode tables for raw DEFLATE.
//
// The table layout and acceptance rules are those of Beast's inflate_table
// (include/boost/beast/zlib/detail/inflate_stream.ipp:551-863): a root table
// of `root` index bits (requested 9 for literal/length, 6 for distance, 7 for
// code-length codes; clamped to [shortest, longest] code), second-level
// tables for longer codes, over-subscribed codes rejected, incomplete codes
// accepted only for a single 1-bit literal/length or distance code, and an
// empty code turned into a 2-slot table of invalid entries.  Keeping the
// same root/sub-table sizes matters: Beast's slow path asks for `root` (or
// `root + sub`) bits before it decodes a symbol, which decides where a
// truncated stream stops (inflate_stream.ipp:360-420).
//
// Slots are 16 bits so a whole worst-case table set (852 + 592 slots) costs
// 2.9 KiB of LDS per wave:  [15:6] value  [5:4] kind  [3:0] bits
#pragma once

#include <stdint.h>

#ifndef BPMD_HD
#define BPMD_HD __host__ __device__
#endif

namespace bpmd {

enum SlotKind : unsigned { K_VAL = 0, K_LEN = 1, K_EOB = 2, K_SPECIAL = 3 };
constexpr unsigned V_INVALID = 0x3FF;
enum BuildType { BUILD_CODES = 0, BUILD_LENS = 1, BUILD_DISTS = 2 };
constexpr unsigned kEnoughLens = 852, kEnoughDists = 592;
constexpr unsigned kEnough = kEnoughLens + kEnoughDists;

BPMD_HD inline uint16_t slot(unsigned kind, unsigned bits, unsigned val)
{
    return (uint16_t)((val << 6) | (kind << 4) | bits);
}
BPMD_HD inline unsigned slot_bits(uint16_t s) { return s & 15u; }
BPMD_HD inline unsigned slot_kind(uint16_t s) { return (s >> 4) & 3u; }
BPMD_HD inline unsigned slot_val(uint16_t s) { return s >> 6; }
BPMD_HD inline bool slot_is_link(uint16_t s) { return slot_kind(s) == K_SPECIAL && slot_val(s) != V_INVALID; }

// Builds one table at `tab`.  Returns 0, 14 (over-subscribed), 15
// (incomplete) or 16 (table overflow, a logic error in the reference).
// *root_io: requested root bits in, actual root bits out; *used: slots used.
// `lens` values are 0..15; `sorted` needs room for ncodes entries.
template <typename LenT, typename SlotT>
BPMD_HD inline int build_table(int type, const LenT* lens, unsigned ncodes, SlotT* tab,
                               unsigned* root_io, unsigned* used, uint16_t* sorted,
                               unsigned* min_len = nullptr)
{
    uint16_t cnt[16], first[16];
    for (unsigned i = 0; i < 16; ++i) cnt[i] = 0;
    for (unsigned i = 0; i < ncodes; ++i) cnt[lens[i]]++;

    unsigned root = *root_io;
    unsigned hi = 15;
    while (hi >= 1 && cnt[hi] == 0) --hi;
    if (root > hi) root = hi;
    if (hi == 0) {
        tab[0] = slot(K_SPECIAL, 1, V_INVALID);
        tab[1] = slot(K_SPECIAL, 1, V_INVALID);
        *root_io = 1;
        *used = 2;
        if (min_len) *min_len = 1;
        return 0;
    }
    unsigned lo = 1;
    while (lo < hi && cnt[lo] == 0) ++lo;
    if (min_len) *min_len = lo;
    if (root < lo) root = lo;

    int avail = 1;
    for (unsigned i = 1; i <= 15; ++i) {
        avail = (avail << 1) - cnt[i];
        if (avail < 0) return 14;
    }
    if (avail > 0 && (type == BUILD_CODES || hi != 1)) return 15;

    first[1] = 0;
    for (unsigned i = 1; i < 15; ++i) first[i + 1] = (uint16_t)(first[i] + cnt[i]);
    for (unsigned i = 0; i < ncodes; ++i)
        if (lens[i] != 0) sorted[first[lens[i]]++] = (uint16_t)i;

    unsigned code = 0, k = 0, len = lo, idx_bits = root, skip = 0;
    unsigned cur_low = ~0u, total = 1u << root;
    const unsigned low_mask = total - 1;
    unsigned tab_off = 0;   // offset of the table being filled
    const unsigned limit = type == BUILD_LENS ? kEnoughLens : type == BUILD_DISTS ? kEnoughDists : 0xffffu;
    if (total > limit) return 16;

    for (;;) {
        unsigned sym = sorted[k];
        uint16_t s;
        unsigned b = len - skip;
        if (type == BUILD_CODES) {
            s = slot(K_VAL, b, sym);
        } else if (type == BUILD_LENS) {
            if (sym < 256) s = slot(K_VAL, b, sym);
            else if (sym == 256) s = slot(K_EOB, b, 0);
            else if (sym <= 285) s = slot(K_LEN, b, sym - 257);
            else s = slot(K_SPECIAL, b, V_INVALID);
        } else {
            s = sym <= 29 ? slot(K_VAL, b, sym) : slot(K_SPECIAL, b, V_INVALID);
        }
        unsigned step = 1u << b;
        unsigned span = 1u << idx_bits;
        const unsigned this_span = span;
        do {
            span -= step;
            tab[tab_off + (code >> skip) + span] = s;
        } while (span != 0);

        unsigned bit = 1u << (len - 1);
        while (code & bit) bit >>= 1;
        if (bit != 0) { code &= bit - 1; code += bit; }
        else code = 0;

        ++k;
        if (--cnt[len] == 0) {
            if (len == hi) break;
            len = lens[sorted[k]];
        }
        if (len > root && (code & low_mask) != cur_low) {
            if (skip == 0) skip = root;
            tab_off += this_span;
            idx_bits = len - skip;
            int room = 1 << idx_bits;
            while (idx_bits + skip < hi) {
                room -= cnt[idx_bits + skip];
                if (room <= 0) break;
                ++idx_bits;
                room <<= 1;
            }
            total += 1u << idx_bits;
            if (total > limit) return 16;
            cur_low = code & low_mask;
            tab[cur_low] = slot(K_SPECIAL, idx_bits, tab_off);
        }
    }
    if (code != 0) tab[tab_off + code] = slot(K_SPECIAL, len - skip, V_INVALID);
    *root_io = root;
    *used = total;
    return 0;
}

}  // namespace bpmd
