// fm_layout.h — GPU-resident bidirectional FM-index layout (host + device).
//
// Replaces, for the device, the rank dictionary that sahara instantiates as
// fmc::BiFMIndex<Sigma, fmc::string::InterleavedBitvector16>
// (/root/reference/src/sahara/search.cpp:162, index.cpp:87).
//
// One 64-byte line per 64 BWT positions, one line array per direction:
//   cnt[c-1]  occurrences of symbol c (1..5) in BWT[0, 64*b)   (u32: n < 2^32)
//   srank     sampled rows in BWT[0, 64*b)                      (forward only)
//   plane[3]  bit j of plane p = bit p of the 3-bit symbol code at 64*b + j
//   sampled   bit j set if row 64*b + j carries an SA sample    (forward only)
// So rank-all-symbols at any position, the BWT symbol of a row and the
// "is this row sampled / which sample" question of locate each cost exactly
// one 64-B line. lb and lb+len share a line whenever their blocks coincide.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define SH_HD __host__ __device__ __forceinline__
#else
#define SH_HD inline
#endif

namespace sahara {

struct alignas(64) OccLine {
    uint32_t cnt[5];
    uint32_t srank;
    uint64_t plane[3];
    uint64_t sampled;
    uint64_t reserved;
};
static_assert(sizeof(OccLine) == 64, "OccLine must be one 64-byte line");

// Symbol codes follow ivsigma's delimited alphabets:
// d_dna4 = {$=0, A=1, C=2, G=3, T=4} (sigma 5), d_dna5 = {$=0, A=1, C=2, G=3, N=4, T=5} (sigma 6).
SH_HD uint64_t symMask(const uint64_t p[3], uint32_t c) {
    const uint64_t m0 = (c & 1u) ? p[0] : ~p[0];
    const uint64_t m1 = (c & 2u) ? p[1] : ~p[1];
    const uint64_t m2 = (c & 4u) ? p[2] : ~p[2];
    return m0 & m1 & m2;
}

SH_HD uint64_t lowMask(uint32_t off) {  // bits [0, off)
    return off ? (~0ull >> (64u - off)) : 0ull;
}

SH_HD uint32_t symAt(const uint64_t p[3], uint32_t off) {
    return (uint32_t)(((p[0] >> off) & 1u) | (((p[1] >> off) & 1u) << 1) | (((p[2] >> off) & 1u) << 2));
}

// Node of the search-scheme DFS, packed in 16 bytes (uint4 on device):
//   FM node:   x = lb (forward SA interval), y = lbRev (reverse), z = len
//   text node: x = first text position of the matched string t, y = one past
//              its last, z = 1 (a singleton interval resolved through SA)
//   w = pos | e << 16 | lastL << 20 | lastR << 22 | text << 24 | (|t| - pos + 16) << 25
// |t| - pos = #D - #I on the path, in [-15, 15].
enum : uint32_t { OP_NONE = 0, OP_MS = 1, OP_I = 2, OP_D = 3 };
constexpr uint32_t kTextBit = 1u << 24;
constexpr uint32_t kDeltaZero = 16u << 25;

SH_HD uint32_t packMeta(uint32_t pos, uint32_t e, uint32_t lastL, uint32_t lastR) {
    return pos | (e << 16) | (lastL << 20) | (lastR << 22) | kDeltaZero;
}
SH_HD uint32_t metaDelta(uint32_t w) { return w >> 25; }  // |t| - pos + 16

// Hit record flag: the cursor is already a text position (x), len 1.
constexpr uint32_t kPosKnown = 1u << 31;

// One expanded scheme position, packed in a u32 for LDS:
//   pi (16 bits) | l << 16 (4) | u << 20 (4) | dirRight << 24
SH_HD uint32_t packScheme(uint32_t pi, uint32_t l, uint32_t u, uint32_t right) {
    return pi | (l << 16) | (u << 20) | (right << 24);
}

constexpr uint32_t kMaxErrors = 15;     // 4-bit e / bounds
constexpr uint32_t kMaxPatternLen = 65535;

}  // namespace sahara
