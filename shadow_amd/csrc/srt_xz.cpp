// srt_xz.cpp -- the graph file sources of load_network_graph in the library:
// a plain GML file, or an .xz-compressed one decompressed here, then parsed by
// srt_gml_parse.
//
// Reference: load_network_graph (src/main/network/graph/mod.rs:494-509) and
// read_xz (:479-492), which calls lzma-rs 0.3.0 `xz_decompress` (not vendored
// in the reference tree; its published algorithm is the .xz container format
// 1.0.4 + LZMA2 + the LZMA decoder of the LZMA SDK, restated below).  The
// decoder is written for the whole-file case Shadow has: the compressed file
// is in memory and the output grows in one buffer that is also the LZMA
// dictionary (a match copies from earlier output).
//
// Container (per stream; streams may be concatenated with zero padding):
//   header  FD 37 7A 58 5A 00 | flags (00, check type) | CRC32(flags)
//   blocks  header (size byte, flags, optional sizes, filter list = LZMA2
//           only, CRC32) | LZMA2 data | padding to 4 | check (CRC32 / CRC64 /
//           SHA-256 / none, per the stream flags)
//   index   00 | record count | (unpadded size, uncompressed size)* | pad | CRC32
//   footer  CRC32 | backward size | flags | "YZ"
// Every size, CRC and check is verified; a mismatch is the reference's
// "Failed to decompress file".
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "srt_internal.h"

namespace {

struct XzError {
    const char *why;
};
[[noreturn]] void fail(const char *why) { throw XzError{why}; }

// ------------------------------------------------------------- checksums
uint32_t crc32_table[256];
uint64_t crc64_table[256];
struct CrcInit {
    CrcInit() {
        for (uint32_t i = 0; i < 256; ++i) {
            uint32_t c = i;
            uint64_t d = i;
            for (int k = 0; k < 8; ++k) {
                c = c & 1 ? (c >> 1) ^ 0xEDB88320u : c >> 1;                  // CRC-32 (IEEE 802.3)
                d = d & 1 ? (d >> 1) ^ 0xC96C5795D7870F42ull : d >> 1;        // CRC-64 (ECMA-182)
            }
            crc32_table[i] = c;
            crc64_table[i] = d;
        }
    }
} crc_init;

uint32_t crc32(const uint8_t *p, size_t n, uint32_t crc = 0) {
    crc = ~crc;
    for (size_t i = 0; i < n; ++i) crc = crc32_table[(crc ^ p[i]) & 0xff] ^ (crc >> 8);
    return ~crc;
}
uint64_t crc64(const uint8_t *p, size_t n) {
    uint64_t crc = ~0ull;
    for (size_t i = 0; i < n; ++i) crc = crc64_table[(crc ^ p[i]) & 0xff] ^ (crc >> 8);
    return ~crc;
}

// FIPS 180-4 SHA-256 (the .xz check type 0x0A)
void sha256(const uint8_t *msg, size_t len, uint8_t out[32]) {
    static const uint32_t K[64] = {
        0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
        0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
        0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
        0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
        0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
        0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
        0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
        0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
    uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    auto rotr = [](uint32_t x, int k) { return (x >> k) | (x << (32 - k)); };
    auto block = [&](const uint8_t *b) {
        uint32_t w[64];
        for (int i = 0; i < 16; ++i)
            w[i] = (uint32_t)b[4 * i] << 24 | (uint32_t)b[4 * i + 1] << 16 | (uint32_t)b[4 * i + 2] << 8 | b[4 * i + 3];
        for (int i = 16; i < 64; ++i) {
            const uint32_t s0 = rotr(w[i - 15], 7) ^ rotr(w[i - 15], 18) ^ (w[i - 15] >> 3);
            const uint32_t s1 = rotr(w[i - 2], 17) ^ rotr(w[i - 2], 19) ^ (w[i - 2] >> 10);
            w[i] = w[i - 16] + s0 + w[i - 7] + s1;
        }
        uint32_t a = h[0], bb = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
        for (int i = 0; i < 64; ++i) {
            const uint32_t t1 = hh + (rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25)) + ((e & f) ^ (~e & g)) + K[i] + w[i];
            const uint32_t t2 = (rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22)) + ((a & bb) ^ (a & c) ^ (bb & c));
            hh = g;
            g = f;
            f = e;
            e = d + t1;
            d = c;
            c = bb;
            bb = a;
            a = t1 + t2;
        }
        h[0] += a; h[1] += bb; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
    };
    size_t i = 0;
    for (; i + 64 <= len; i += 64) block(msg + i);
    uint8_t tail[128] = {};
    const size_t rest = len - i;
    std::memcpy(tail, msg + i, rest);
    tail[rest] = 0x80;
    const size_t tl = rest + 9 <= 64 ? 64 : 128;
    const uint64_t bits = (uint64_t)len * 8;
    for (int k = 0; k < 8; ++k) tail[tl - 1 - k] = (uint8_t)(bits >> (8 * k));
    block(tail);
    if (tl == 128) block(tail + 64);
    for (int k = 0; k < 8; ++k)
        for (int j = 0; j < 4; ++j) out[4 * k + j] = (uint8_t)(h[k] >> (24 - 8 * j));
}

// ------------------------------------------------------------ input cursor
struct In {
    const uint8_t *p;
    size_t n, pos = 0;
    uint8_t byte() {
        if (pos >= n) fail("truncated input");
        return p[pos++];
    }
    const uint8_t *take(size_t k) {
        if (n - pos < k) fail("truncated input");
        const uint8_t *r = p + pos;
        pos += k;
        return r;
    }
    // .xz variable-length integer (7 bits a byte, at most 9 bytes)
    uint64_t vli() {
        uint64_t v = 0;
        for (int i = 0; i < 9; ++i) {
            const uint8_t b = byte();
            v |= (uint64_t)(b & 0x7f) << (7 * i);
            if (!(b & 0x80)) {
                if (i > 0 && b == 0) fail("non-minimal integer");
                return v;
            }
        }
        fail("integer too long");
    }
};

uint32_t le32(const uint8_t *p) { return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24; }

// ------------------------------------------------------------------ LZMA
constexpr int NUM_STATES = 12, POS_STATES_MAX = 16, LEN_TO_POS_STATES = 4, END_POS_MODEL = 14,
              FULL_DISTANCES = 128, ALIGN_BITS = 4;

struct RangeDec {
    const uint8_t *p = nullptr;
    size_t n = 0, pos = 0;
    uint32_t range = 0, code = 0;
    void init(const uint8_t *b, size_t len) {
        p = b;
        n = len;
        pos = 0;
        if (len < 5 || b[0] != 0) fail("bad range coder start");
        range = 0xffffffffu;
        code = (uint32_t)b[1] << 24 | (uint32_t)b[2] << 16 | (uint32_t)b[3] << 8 | b[4];
        pos = 5;
    }
    void normalize() {
        if (range < (1u << 24)) {
            if (pos >= n) fail("LZMA chunk overran its compressed size");
            range <<= 8;
            code = code << 8 | p[pos++];
        }
    }
    uint32_t bit(uint16_t &prob) {
        const uint32_t bound = (range >> 11) * prob;
        uint32_t b;
        if (code < bound) {
            range = bound;
            prob += (2048 - prob) >> 5;
            b = 0;
        } else {
            range -= bound;
            code -= bound;
            prob -= prob >> 5;
            b = 1;
        }
        normalize();
        return b;
    }
    uint32_t tree(uint16_t *probs, int bits) {
        uint32_t m = 1;
        for (int i = 0; i < bits; ++i) m = (m << 1) | bit(probs[m]);
        return m - (1u << bits);
    }
    uint32_t tree_rev(uint16_t *probs, int bits) {
        uint32_t m = 1, sym = 0;
        for (int i = 0; i < bits; ++i) {
            const uint32_t b = bit(probs[m]);
            m = (m << 1) | b;
            sym |= b << i;
        }
        return sym;
    }
    uint32_t direct(int bits) {
        uint32_t r = 0;
        for (int i = 0; i < bits; ++i) {
            range >>= 1;
            uint32_t b = 0;
            if (code >= range) {
                code -= range;
                b = 1;
            }
            r = (r << 1) | b;
            normalize();
        }
        return r;
    }
};

struct LenDec {
    uint16_t choice, choice2, low[POS_STATES_MAX][8], mid[POS_STATES_MAX][8], high[256];
    void reset() {
        choice = choice2 = 1024;
        for (auto &a : low) for (auto &x : a) x = 1024;
        for (auto &a : mid) for (auto &x : a) x = 1024;
        for (auto &x : high) x = 1024;
    }
    uint32_t decode(RangeDec &rc, uint32_t ps) {
        if (!rc.bit(choice)) return 2 + rc.tree(low[ps], 3);
        if (!rc.bit(choice2)) return 10 + rc.tree(mid[ps], 3);
        return 18 + rc.tree(high, 8);
    }
};

struct Lzma {
    uint32_t lc = 0, lp = 0, pb = 0;
    uint32_t state = 0, rep[4] = {};
    uint16_t is_match[NUM_STATES][POS_STATES_MAX], is_rep[NUM_STATES], is_rep0[NUM_STATES], is_rep1[NUM_STATES],
        is_rep2[NUM_STATES], is_rep0_long[NUM_STATES][POS_STATES_MAX], dist_slot[LEN_TO_POS_STATES][64],
        dist_special[FULL_DISTANCES - END_POS_MODEL], align[1 << ALIGN_BITS];
    LenDec match_len, rep_len;
    std::vector<uint16_t> lit;
    void set_props(uint8_t d) {
        if (d >= 9 * 5 * 5) fail("bad LZMA properties");
        lc = d % 9;
        d /= 9;
        lp = d % 5;
        pb = d / 5;
        if (lc + lp > 4) fail("LZMA2 needs lc + lp <= 4");
        lit.assign((size_t)0x300 << (lc + lp), 1024);
    }
    void reset() {
        state = 0;
        rep[0] = rep[1] = rep[2] = rep[3] = 0;
        for (auto &a : is_match) for (auto &x : a) x = 1024;
        for (auto &a : is_rep0_long) for (auto &x : a) x = 1024;
        for (auto &a : dist_slot) for (auto &x : a) x = 1024;
        for (int i = 0; i < NUM_STATES; ++i) is_rep[i] = is_rep0[i] = is_rep1[i] = is_rep2[i] = 1024;
        for (auto &x : dist_special) x = 1024;
        for (auto &x : align) x = 1024;
        match_len.reset();
        rep_len.reset();
        std::fill(lit.begin(), lit.end(), (uint16_t)1024);
    }
    // one LZMA chunk: exactly `unpacked` bytes appended to out (which holds
    // the dictionary from dict_start on); written in place into the grown buffer
    void chunk(RangeDec &rc, std::vector<uint8_t> &out, size_t dict_start, uint64_t unpacked) {
        uint64_t pos = out.size();
        const uint64_t end = pos + unpacked;
        if (out.capacity() < end) out.reserve(std::max<uint64_t>(end, out.capacity() * 2));
        out.resize(end);
        uint8_t *o = out.data();
        const uint32_t pb_mask = (1u << pb) - 1, lp_mask = (1u << lp) - 1;
        while (pos < end) {
            // position bits count from the last dictionary reset (the SDK's processedPos)
            const uint32_t rel = (uint32_t)(pos - dict_start);
            const uint32_t ps = rel & pb_mask;
            if (!rc.bit(is_match[state][ps])) {
                // literal
                const uint32_t prev = pos > dict_start ? o[pos - 1] : 0;
                uint16_t *probs = lit.data() + 0x300 * (((rel & lp_mask) << lc) + (prev >> (8 - lc)));
                uint32_t sym = 1;
                if (state >= 7) {
                    if (pos - dict_start <= rep[0]) fail("match distance beyond the dictionary");
                    uint32_t mb = o[pos - rep[0] - 1];
                    do {
                        const uint32_t m = (mb >> 7) & 1;
                        mb <<= 1;
                        const uint32_t b = rc.bit(probs[0x100 + (m << 8) + sym]);
                        sym = (sym << 1) | b;
                        if (m != b) break;
                    } while (sym < 0x100);
                }
                while (sym < 0x100) sym = (sym << 1) | rc.bit(probs[sym]);
                o[pos++] = (uint8_t)sym;
                state = state < 4 ? 0 : state < 10 ? state - 3 : state - 6;
                continue;
            }
            uint32_t len;
            if (!rc.bit(is_rep[state])) {
                // a new match
                rep[3] = rep[2];
                rep[2] = rep[1];
                rep[1] = rep[0];
                len = match_len.decode(rc, ps);
                state = state < 7 ? 7 : 10;
                const uint32_t ls = len - 2 < LEN_TO_POS_STATES - 1 ? len - 2 : LEN_TO_POS_STATES - 1;
                const uint32_t slot = rc.tree(dist_slot[ls], 6);
                if (slot < 4) {
                    rep[0] = slot;
                } else {
                    const int nd = (int)(slot >> 1) - 1;
                    uint32_t dist = (2 | (slot & 1)) << nd;
                    if (slot < END_POS_MODEL) {
                        dist += rc.tree_rev(dist_special + dist - slot - 1, nd);
                    } else {
                        dist += rc.direct(nd - ALIGN_BITS) << ALIGN_BITS;
                        dist += rc.tree_rev(align, ALIGN_BITS);
                    }
                    rep[0] = dist;
                }
                if (rep[0] == 0xffffffffu) fail("end marker inside an LZMA2 chunk");
            } else {
                if (!rc.bit(is_rep0[state])) {
                    if (!rc.bit(is_rep0_long[state][ps])) {
                        // short rep: one byte at rep0
                        state = state < 7 ? 9 : 11;
                        if (pos - dict_start <= rep[0]) fail("match distance beyond the dictionary");
                        o[pos] = o[pos - rep[0] - 1];
                        ++pos;
                        continue;
                    }
                } else {
                    uint32_t d;
                    if (!rc.bit(is_rep1[state])) {
                        d = rep[1];
                    } else {
                        if (!rc.bit(is_rep2[state])) {
                            d = rep[2];
                        } else {
                            d = rep[3];
                            rep[3] = rep[2];
                        }
                        rep[2] = rep[1];
                    }
                    rep[1] = rep[0];
                    rep[0] = d;
                }
                len = rep_len.decode(rc, ps);
                state = state < 7 ? 8 : 11;
            }
            if (pos - dict_start <= rep[0]) fail("match distance beyond the dictionary");
            if (len > end - pos) fail("match runs past the chunk");
            const uint8_t *src = o + pos - rep[0] - 1;
            uint8_t *dst = o + pos;
            if (rep[0] + 1 >= len) {
                std::memcpy(dst, src, len);
            } else {
                for (uint32_t k = 0; k < len; ++k) dst[k] = src[k];  // overlapping: byte order matters
            }
            pos += len;
        }
    }
};

// LZMA2 (one block's compressed data): chunks until the end byte; returns the
// bytes it consumed
size_t lzma2_decode(const uint8_t *p, size_t n, std::vector<uint8_t> &out) {
    In in{p, n};
    Lzma lz;
    size_t dict_start = out.size();
    bool need_dict_reset = true, need_props = true;
    for (;;) {
        const uint8_t c = in.byte();
        if (c == 0x00) return in.pos;
        if (c >= 0xE0 || c == 0x01) {
            need_props = true;
            need_dict_reset = false;
            dict_start = out.size();
        } else if (need_dict_reset) {
            fail("LZMA2 stream does not start with a dictionary reset");
        }
        if (c >= 0x80) {
            const uint64_t unpacked = ((uint64_t)(c & 0x1f) << 16) + ((uint64_t)in.byte() << 8) + in.byte() + 1;
            const uint64_t packed = ((uint64_t)in.byte() << 8) + in.byte() + 1;
            if (c >= 0xC0) {
                lz.set_props(in.byte());
                need_props = false;
                lz.reset();
            } else if (need_props) {
                fail("LZMA2 chunk without properties");
            } else if (c >= 0xA0) {
                lz.reset();
            }
            RangeDec rc;
            rc.init(in.take(packed), packed);
            lz.chunk(rc, out, dict_start, unpacked);
            if (rc.code != 0 || rc.pos != rc.n) fail("LZMA chunk size mismatch");
        } else {
            if (c > 0x02) fail("bad LZMA2 control byte");
            const uint64_t size = ((uint64_t)in.byte() << 8) + in.byte() + 1;
            const uint8_t *d = in.take(size);
            out.insert(out.end(), d, d + size);
        }
    }
}

size_t check_size(uint32_t t) {
    static const uint8_t sz[16] = {0, 4, 4, 4, 8, 8, 8, 16, 16, 16, 32, 32, 32, 64, 64, 64};
    return sz[t & 15];
}

// one .xz stream starting at in.pos
void xz_stream(In &in, std::vector<uint8_t> &out) {
    static const uint8_t magic[6] = {0xFD, '7', 'z', 'X', 'Z', 0x00};
    const uint8_t *h = in.take(12);
    if (std::memcmp(h, magic, 6) != 0) fail("not an .xz stream (bad magic)");
    if (crc32(h + 6, 2) != le32(h + 8)) fail("stream header CRC32 mismatch");
    if (h[6] != 0 || (h[7] & 0xf0)) fail("unsupported stream flags");
    const uint32_t check = h[7];
    if (check != 0 && check != 1 && check != 4 && check != 10) fail("unsupported check type");
    struct Rec {
        uint64_t unpadded, uncompressed;
    };
    std::vector<Rec> recs;
    for (;;) {
        const size_t bh = in.pos;
        const uint8_t sb = in.byte();
        if (sb == 0x00) break;  // the index indicator
        const size_t hsize = ((size_t)sb + 1) * 4;
        in.pos = bh;
        const uint8_t *hb = in.take(hsize);
        if (crc32(hb, hsize - 4) != le32(hb + hsize - 4)) fail("block header CRC32 mismatch");
        In hi{hb + 1, hsize - 5};
        const uint8_t flags = hi.byte();
        if (flags & 0x3c) fail("reserved block flags");
        const uint32_t nfilt = (flags & 3) + 1;
        uint64_t csize = ~0ull, usize = ~0ull;
        if (flags & 0x40) csize = hi.vli();
        if (flags & 0x80) usize = hi.vli();
        for (uint32_t f = 0; f < nfilt; ++f) {
            const uint64_t id = hi.vli(), psz = hi.vli();
            if (id != 0x21 || nfilt != 1) fail("unsupported filter (LZMA2 only, as lzma-rs)");
            if (psz != 1) fail("bad LZMA2 filter properties");
            const uint8_t dp = hi.byte();
            if (dp > 40) fail("bad LZMA2 dictionary size");
        }
        while (hi.pos < hi.n)
            if (hi.byte() != 0) fail("non-zero block header padding");
        const size_t cstart = in.pos, ustart = out.size();
        const size_t used = lzma2_decode(in.p + in.pos, in.n - in.pos, out);
        in.pos += used;
        if (csize != ~0ull && csize != used) fail("block compressed size mismatch");
        if (usize != ~0ull && usize != out.size() - ustart) fail("block uncompressed size mismatch");
        while ((in.pos - cstart) & 3)
            if (in.byte() != 0) fail("non-zero block padding");
        const uint8_t *ck = in.take(check_size(check));
        const uint8_t *ud = out.data() + ustart;
        const size_t ul = out.size() - ustart;
        if (check == 1 && crc32(ud, ul) != le32(ck)) fail("block CRC32 mismatch");
        if (check == 4) {
            const uint64_t c = crc64(ud, ul);
            uint64_t want = 0;
            for (int k = 0; k < 8; ++k) want |= (uint64_t)ck[k] << (8 * k);
            if (c != want) fail("block CRC64 mismatch");
        }
        if (check == 10) {
            uint8_t d[32];
            sha256(ud, ul, d);
            if (std::memcmp(d, ck, 32) != 0) fail("block SHA-256 mismatch");
        }
        recs.push_back({(uint64_t)hsize + used + check_size(check), (uint64_t)ul});
    }
    // index (the indicator byte was read)
    const size_t ix = in.pos - 1;
    if (in.vli() != recs.size()) fail("index record count mismatch");
    for (const Rec &r : recs) {
        if (in.vli() != r.unpadded) fail("index unpadded size mismatch");
        if (in.vli() != r.uncompressed) fail("index uncompressed size mismatch");
    }
    while ((in.pos - ix) & 3)
        if (in.byte() != 0) fail("non-zero index padding");
    const size_t ilen = in.pos - ix;
    if (crc32(in.p + ix, ilen) != le32(in.take(4))) fail("index CRC32 mismatch");
    const uint8_t *ft = in.take(12);
    if (crc32(ft + 4, 6) != le32(ft)) fail("stream footer CRC32 mismatch");
    if (((uint64_t)le32(ft + 4) + 1) * 4 != ilen + 4) fail("backward size mismatch");
    if (ft[8] != h[6] || ft[9] != h[7]) fail("stream footer flags differ from the header");
    if (ft[10] != 'Y' || ft[11] != 'Z') fail("bad footer magic");
}

void set(srt_err *err, int code, const std::string &msg) {
    if (!err) return;
    err->code = code;
    std::snprintf(err->msg, sizeof err->msg, "%s", msg.c_str());
}

// String::from_utf8 (mod.rs:490): the decompressed graph must be UTF-8
bool valid_utf8(const uint8_t *s, size_t n) {
    size_t i = 0;
    while (i < n) {
        const uint8_t c = s[i];
        if (c < 0x80) {
            ++i;
            continue;
        }
        int k;
        uint32_t cp;
        if ((c & 0xe0) == 0xc0) k = 1, cp = c & 0x1f;
        else if ((c & 0xf0) == 0xe0) k = 2, cp = c & 0x0f;
        else if ((c & 0xf8) == 0xf0) k = 3, cp = c & 0x07;
        else return false;
        if (n - i <= (size_t)k) return false;
        for (int j = 1; j <= k; ++j) {
            if ((s[i + j] & 0xc0) != 0x80) return false;
            cp = cp << 6 | (s[i + j] & 0x3f);
        }
        if ((k == 1 && cp < 0x80) || (k == 2 && cp < 0x800) || (k == 3 && cp < 0x10000) || cp > 0x10ffff ||
            (cp >= 0xd800 && cp <= 0xdfff))
            return false;
        i += k + 1;
    }
    return true;
}

bool read_file(const char *path, std::vector<uint8_t> *buf) {
    FILE *f = std::fopen(path, "rb");
    if (!f) return false;
    std::fseek(f, 0, SEEK_END);
    const long sz = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    if (sz < 0) {
        std::fclose(f);
        return false;
    }
    buf->resize((size_t)sz);
    const bool ok = std::fread(buf->data(), 1, (size_t)sz, f) == (size_t)sz;
    std::fclose(f);
    return ok;
}

}  // namespace

extern "C" {

srt_status srt_xz_decompress(const uint8_t *in, size_t len, uint8_t **out, size_t *out_len, srt_err *err) {
    if (err) std::memset(err, 0, sizeof *err);
    if ((!in && len) || !out || !out_len) {
        set(err, SRT_ERR_INVALID, "null argument");
        return SRT_ERR_INVALID;
    }
    *out = nullptr;
    *out_len = 0;
    try {
        std::vector<uint8_t> buf;
        In s{in, len};
        bool any = false;
        while (s.pos < s.n) {
            // stream padding: zero bytes in multiples of four between streams
            if (any && s.p[s.pos] == 0) {
                const uint8_t *z = s.take(4);
                if (z[1] | z[2] | z[3]) fail("bad stream padding");
                continue;
            }
            xz_stream(s, buf);
            any = true;
        }
        if (!any) fail("empty input");
        uint8_t *r = static_cast<uint8_t *>(std::malloc(buf.size() + 1));
        if (!r) {
            set(err, SRT_ERR_OOM, "out of host memory");
            return SRT_ERR_OOM;
        }
        if (!buf.empty()) std::memcpy(r, buf.data(), buf.size());
        r[buf.size()] = 0;
        *out = r;
        *out_len = buf.size();
        return SRT_OK;
    } catch (const XzError &e) {
        // read_xz's context (mod.rs:488); the decoder's reason after it
        set(err, SRT_ERR_INVALID, std::string("Failed to decompress file: ") + e.why);
        return SRT_ERR_INVALID;
    } catch (...) {
        set(err, SRT_ERR_OOM, "out of host memory");
        return SRT_ERR_OOM;
    }
}

void srt_free(void *p) { std::free(p); }

srt_status srt_gml_parse_file(const char *path, int xz, srt_gml **out, srt_err *err) {
    if (err) std::memset(err, 0, sizeof *err);
    if (!path || !out) {
        set(err, SRT_ERR_INVALID, "null argument");
        return SRT_ERR_INVALID;
    }
    *out = nullptr;
    std::vector<uint8_t> raw;
    if (!read_file(path, &raw)) {
        // mod.rs:487 (xz) / :501 (plain); Rust's {path:?} quotes the path
        set(err, SRT_ERR_INVALID,
            xz ? std::string("Failed to open file: \"") + path + "\"" : std::string("Failed to read file: ") + path);
        return SRT_ERR_INVALID;
    }
    const uint8_t *text = raw.data();
    size_t tlen = raw.size();
    uint8_t *dec = nullptr;
    if (xz) {
        if (srt_status st = srt_xz_decompress(raw.data(), raw.size(), &dec, &tlen, err); st != SRT_OK) return st;
        text = dec;
    }
    if (!valid_utf8(text, tlen)) {
        srt_free(dec);
        set(err, SRT_ERR_INVALID, xz ? "invalid utf-8 in the decompressed graph"
                                     : std::string("Failed to read file: ") + path);
        return SRT_ERR_INVALID;
    }
    const srt_status st = srt_gml_parse(reinterpret_cast<const char *>(text), tlen, out, err);
    srt_free(dec);
    return st;
}

}  // extern "C"
