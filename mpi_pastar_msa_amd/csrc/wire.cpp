// wire.cpp -- the reference's inter-rank wire frame, for an MPI-compatible
// multi-node mode.
//
// The reference moves every message between ranks (node vectors, the
// sequences, the stats sync, the backtrace hand-overs) as one frame
// (lz4sup.cpp:13-43, decoded by :45-70):
//
//   u32 total    = compressed bytes + 12
//   u32 bound    = LZ4_compressBound(orig)
//   u32 orig     = payload bytes + 1 (the std::string's terminating NUL
//                  is compressed with it: lz4sup.cpp:16)
//   LZ4 block    (LZ4_compress, i.e. LZ4_compress_default at acceleration 1)
//
// The block is produced by our own compressor, which makes the same parsing
// decisions as liblz4 1.9.3's one-shot compressor (LZ4_compress_generic with
// no dictionary: a 4096-entry 16-bit index table hashed on 4 bytes below
// 64 KB + 11 of input, a 4096-entry 32-bit one hashed on 5 bytes above it,
// the skip-trigger search acceleration, backward catch-up and the
// "test next position" shortcut), so a frame is byte-identical to the one
// the reference emits for the same payload (tests/test_wire.py checks it
// against the reference's lz4sup.cpp compiled in place, oracle/Makefile).
// The decoder accepts any valid LZ4 block, as LZ4_decompress_fast does, but
// bounds-checks every read and write.
//
// The payload the reference frames is a Boost binary archive; Boost is not
// in this image, so the archive layer is not reproduced.
// Node records use the field order Node<N>::serialize writes
// (Node.h:57-64: m_g, m_f, pos, parenti), little-endian and packed.
#include <cstdint>
#include <cstring>
#include <vector>

#include "pastar_gpu.h"

namespace {

constexpr int kMinMatch = 4;
constexpr int kMfLimit = 12;      // the last match starts >= 12 bytes before the end
constexpr int kLastLiterals = 5;  // the last 5 bytes are always literals
constexpr int kMinLength = kMfLimit + 1;
constexpr int kHashLog = 12;      // LZ4_MEMORY_USAGE 14
constexpr uint32_t kLimit64k = 65536 + kMfLimit - 1;
constexpr uint32_t kMaxDistance = 65535;
constexpr int kSkipTrigger = 6;
constexpr uint32_t kMaxInput = 0x7E000000;
constexpr int kFrameHeader = 12;

inline uint32_t rd32(const uint8_t *p)
{
    uint32_t v;
    std::memcpy(&v, p, 4);
    return v;
}

inline uint64_t rd64(const uint8_t *p)
{
    uint64_t v;
    std::memcpy(&v, p, 8);
    return v;
}

inline int64_t compress_bound(int64_t n) { return n > kMaxInput ? 0 : n + n / 255 + 16; }

struct Table {
    bool small;  // 16-bit indices, 4-byte hash (input below 64 KB + 11)
    std::vector<uint32_t> idx;
    explicit Table(bool s) : small(s), idx((size_t)1 << (kHashLog + (s ? 1 : 0)), 0) {}
    uint32_t hash(const uint8_t *p) const
    {
        if (small)
            return (rd32(p) * 2654435761u) >> (32 - (kHashLog + 1));
        return (uint32_t)(((rd64(p) << 24) * 889523592379ull) >> (64 - kHashLog));
    }
    uint32_t get(uint32_t h) const { return small ? (idx[h] & 0xFFFF) : idx[h]; }
    void put(uint32_t h, uint32_t i) { idx[h] = small ? (i & 0xFFFF) : i; }
};

// number of equal bytes of a and b, a stopping at limit
inline uint32_t count_equal(const uint8_t *a, const uint8_t *b, const uint8_t *limit)
{
    const uint8_t *s = a;
    while (a < limit && *a == *b) {
        a++;
        b++;
    }
    return (uint32_t)(a - s);
}

inline uint8_t *put_length(uint8_t *op, uint32_t len)
{
    for (; len >= 255; len -= 255)
        *op++ = 255;
    *op++ = (uint8_t)len;
    return op;
}

// LZ4 block of src[0, n) into dst (capacity >= compress_bound(n)); returns
// the block's size.  Mirrors the decisions of liblz4 1.9.3's
// LZ4_compress_generic(noDict, noDictIssue, acceleration 1).
size_t lz4_block(const uint8_t *src, uint32_t n, uint8_t *dst)
{
    uint8_t *op = dst;
    if (n == 0) {
        *op++ = 0;
        return 1;
    }
    const uint8_t *ip = src, *anchor = src;
    const uint8_t *const iend = src + n;
    const uint8_t *const mflimit_plus_one = iend - kMfLimit + 1;
    const uint8_t *const matchlimit = iend - kLastLiterals;
    Table t(n < kLimit64k);
    if (n >= (uint32_t)kMinLength) {
        t.put(t.hash(ip), 0);
        ip++;
        uint32_t forward_h = t.hash(ip);
        for (;;) {
            const uint8_t *match;
            uint8_t *token;
            // find a match, stepping faster the longer none is found
            {
                const uint8_t *forward_ip = ip;
                uint32_t step = 1, search_nb = 1u << kSkipTrigger;
                for (;;) {
                    const uint32_t h = forward_h;
                    const uint32_t cur = (uint32_t)(forward_ip - src);
                    const uint32_t mi = t.get(h);
                    ip = forward_ip;
                    forward_ip += step;
                    step = search_nb++ >> kSkipTrigger;
                    if (forward_ip > mflimit_plus_one)
                        goto last_literals;
                    match = src + mi;
                    forward_h = t.hash(forward_ip);
                    t.put(h, cur);
                    if (!t.small && mi + kMaxDistance < cur)
                        continue;  // too far
                    if (rd32(match) == rd32(ip))
                        break;
                }
            }
            // catch up backwards
            while (ip > anchor && match > src && ip[-1] == match[-1]) {
                ip--;
                match--;
            }
            {
                const uint32_t lit = (uint32_t)(ip - anchor);
                token = op++;
                if (lit >= 15) {
                    *token = 15 << 4;
                    op = put_length(op, lit - 15);
                } else {
                    *token = (uint8_t)(lit << 4);
                }
                std::memcpy(op, anchor, lit);
                op += lit;
            }
            for (;;) {  // next_match
                const uint32_t off = (uint32_t)(ip - match);
                *op++ = (uint8_t)off;
                *op++ = (uint8_t)(off >> 8);
                uint32_t ml = count_equal(ip + kMinMatch, match + kMinMatch, matchlimit);
                ip += ml + kMinMatch;
                if (ml >= 15) {
                    *token += 15;
                    op = put_length(op, ml - 15);
                } else {
                    *token += (uint8_t)ml;
                }
                anchor = ip;
                if (ip >= mflimit_plus_one)
                    goto last_literals;
                t.put(t.hash(ip - 2), (uint32_t)(ip - 2 - src));
                // test the next position for an immediate match
                const uint32_t h = t.hash(ip);
                const uint32_t cur = (uint32_t)(ip - src);
                const uint32_t mi = t.get(h);
                match = src + mi;
                t.put(h, cur);
                if ((t.small || mi + kMaxDistance >= cur) && rd32(match) == rd32(ip)) {
                    token = op++;
                    *token = 0;
                    continue;
                }
                break;
            }
            forward_h = t.hash(++ip);
        }
    }
last_literals:
    {
        const uint32_t last = (uint32_t)(iend - anchor);
        if (last >= 15) {
            *op++ = 15 << 4;
            op = put_length(op, last - 15);
        } else {
            *op++ = (uint8_t)(last << 4);
        }
        std::memcpy(op, anchor, last);
        op += last;
    }
    return (size_t)(op - dst);
}

// decode an LZ4 block of exactly `n` output bytes; false on any malformed
// or out-of-bounds sequence
bool lz4_unblock(const uint8_t *src, size_t slen, uint8_t *dst, size_t n)
{
    const uint8_t *ip = src, *const iend = src + slen;
    uint8_t *op = dst, *const oend = dst + n;
    for (;;) {
        if (ip >= iend)
            return false;
        const uint8_t token = *ip++;
        size_t lit = token >> 4;
        if (lit == 15) {
            uint8_t b;
            do {
                if (ip >= iend)
                    return false;
                b = *ip++;
                lit += b;
            } while (b == 255);
        }
        if ((size_t)(iend - ip) < lit || (size_t)(oend - op) < lit)
            return false;
        std::memcpy(op, ip, lit);
        ip += lit;
        op += lit;
        if (op == oend)
            return ip == iend;  // the block ends on its last literals
        if (iend - ip < 2)
            return false;
        const size_t off = (size_t)ip[0] | ((size_t)ip[1] << 8);
        ip += 2;
        if (off == 0 || off > (size_t)(op - dst))
            return false;
        size_t ml = (token & 15);
        if (ml == 15) {
            uint8_t b;
            do {
                if (ip >= iend)
                    return false;
                b = *ip++;
                ml += b;
            } while (b == 255);
        }
        ml += kMinMatch;
        if ((size_t)(oend - op) < ml)
            return false;
        const uint8_t *m = op - off;
        for (size_t i = 0; i < ml; i++)  // overlapping copies repeat the pattern
            op[i] = m[i];
        op += ml;
    }
}

void put32(uint8_t *p, uint32_t v) { std::memcpy(p, &v, 4); }

}  // namespace

extern "C" {

int pastar_wire_frame_bound(int64_t len, int64_t *bound)
{
    if (!bound || len < 0 || len + 1 > (int64_t)kMaxInput)
        return PASTAR_EINVAL;
    *bound = kFrameHeader + compress_bound(len + 1);
    return PASTAR_OK;
}

int pastar_wire_frame_encode(const void *payload, int64_t len, void *out, int64_t cap, int64_t *out_len)
{
    int64_t bound = 0;
    if ((!payload && len) || !out || !out_len || pastar_wire_frame_bound(len, &bound) != PASTAR_OK || cap < bound)
        return PASTAR_EINVAL;
    // the reference compresses the string with its terminating NUL
    std::vector<uint8_t> src((size_t)len + 1, 0);
    if (len)
        std::memcpy(src.data(), payload, (size_t)len);
    uint8_t *o = static_cast<uint8_t *>(out);
    const size_t clen = lz4_block(src.data(), (uint32_t)(len + 1), o + kFrameHeader);
    put32(o, (uint32_t)(clen + kFrameHeader));
    put32(o + 4, (uint32_t)compress_bound(len + 1));
    put32(o + 8, (uint32_t)(len + 1));
    *out_len = (int64_t)clen + kFrameHeader;
    return PASTAR_OK;
}

int pastar_wire_frame_decode(const void *frame, int64_t frame_len, void *out, int64_t cap, int64_t *out_len)
{
    if (!frame || !out || !out_len || frame_len < kFrameHeader + 1)
        return PASTAR_EINVAL;
    const uint8_t *f = static_cast<const uint8_t *>(frame);
    const uint32_t total = rd32(f), orig = rd32(f + 8);
    if (total < (uint32_t)kFrameHeader + 1 || (int64_t)total > frame_len || orig == 0 || (int64_t)orig > cap ||
        orig > kMaxInput)
        return PASTAR_EINVAL;
    if (!lz4_unblock(f + kFrameHeader, total - kFrameHeader, static_cast<uint8_t *>(out), orig))
        return PASTAR_EINVAL;
    *out_len = orig;
    return PASTAR_OK;
}

int pastar_wire_pack_nodes(const pastar_node *nodes, int count, int n, void *out, int64_t cap, int64_t *out_len)
{
    if (n < 2 || n > PASTAR_MAX_SEQ || count < 0 || (count && !nodes) || !out_len)
        return PASTAR_EINVAL;
    const int64_t rec = 12 + 2 * (int64_t)n;
    if (cap < rec * count || (count && !out))
        return PASTAR_EINVAL;
    uint8_t *o = static_cast<uint8_t *>(out);
    for (int i = 0; i < count; i++) {
        const pastar_node &x = nodes[i];
        std::memcpy(o, &x.g, 4);
        std::memcpy(o + 4, &x.f, 4);
        std::memcpy(o + 8, x.pos, 2 * (size_t)n);
        std::memcpy(o + 8 + 2 * n, &x.parent_mask, 4);
        o += rec;
    }
    *out_len = rec * count;
    return PASTAR_OK;
}

int pastar_wire_unpack_nodes(const void *in, int64_t len, int n, pastar_node *out, int cap, int *count)
{
    if (n < 2 || n > PASTAR_MAX_SEQ || len < 0 || (len && !in) || !count)
        return PASTAR_EINVAL;
    const int64_t rec = 12 + 2 * (int64_t)n;
    if (len % rec || len / rec > cap || (len && !out))
        return PASTAR_EINVAL;
    const uint8_t *p = static_cast<const uint8_t *>(in);
    const int c = (int)(len / rec);
    for (int i = 0; i < c; i++) {
        pastar_node &x = out[i];
        std::memset(&x, 0, sizeof(x));
        std::memcpy(&x.g, p, 4);
        std::memcpy(&x.f, p + 4, 4);
        std::memcpy(x.pos, p + 8, 2 * (size_t)n);
        std::memcpy(&x.parent_mask, p + 8 + 2 * n, 4);
        p += rec;
    }
    *count = c;
    return PASTAR_OK;
}

}  // extern "C"
