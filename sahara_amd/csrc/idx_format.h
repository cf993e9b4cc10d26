// idx_format.h — the `.idx` file written by `sahara index` and read by
// `sahara search` (host side).
//
// Reference: index.cpp:96-100 writes `cereal::BinaryOutputArchive{ofs}` with
// archive(Sigma); archive(index); search.cpp:162-169 / :278-283 read the
// leading size_t sigma and dispatch on it. Only that first field is pinned by
// the reference; the BiFMIndex payload below is this build's own, written with
// cereal BinaryArchive conventions (host-endian scalars, u64 element count
// before every vector, std::array without a count):
//
//   u64 sigma | u64 magic | u64 n | u64 C[sigma+1] | vec<u64> recLens |
//   u64 samplingRate | vec<u8> bwtFwd | vec<u8> bwtRev | vec<u64> sampledBits |
//   vec<u32> samples
//
// bwtRev is the BWT of the records reversed one by one (record order kept),
// which makes the bidirectional update exact across delimiters.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace sahara {

constexpr uint64_t kIdxMagic = 0x3178646961726173ull;
// A text of 2^32 - 2 symbols or more is indexed in parts (records split at
// record boundaries, device_index.h splitRecords), each a complete index:
//
//   u64 sigma | u64 partsMagic | u64 nparts | nparts x (u64 bytes | the part
//   as a single-part image above, its own leading sigma included)
//
// A text that fits one part keeps the single-part layout byte for byte.
constexpr uint64_t kIdxPartsMagic = 0x7374726170616873ull;

struct IdxParts {
    uint32_t sigma = 0;
    uint64_t n = 0;
    uint32_t rate = 16;
    uint64_t C[8] = {0};
    std::vector<uint64_t> recLens;
    const uint8_t* bwtF = nullptr;
    const uint8_t* bwtR = nullptr;
    const uint64_t* sampled = nullptr;
    const uint32_t* samples = nullptr;
    uint64_t nsamples = 0;
};

std::vector<uint8_t> readFile(const std::string& path);
IdxParts parseIdx(const uint8_t* buf, size_t bytes);   // pointers alias buf
// single- or multi-part image -> its parts in record order (pointers alias buf)
std::vector<IdxParts> parseIdxAll(const uint8_t* buf, size_t bytes);
void writeIdx(const std::string& path, const IdxParts& p);
void writeIdxAll(const std::string& path, const std::vector<IdxParts>& parts);  // one part: writeIdx
uint64_t readIdxSigma(const std::string& path);         // search.cpp:278-283

void synthReads(const uint8_t* ranks, const uint64_t* recLens, uint64_t nrec, uint32_t sigma, uint64_t nreads,
                uint32_t len, uint32_t subs, uint32_t ins, uint32_t dels, uint32_t errors, uint64_t seed, uint8_t* out,
                uint64_t* origin);

}  // namespace sahara
