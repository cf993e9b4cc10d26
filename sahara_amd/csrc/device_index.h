// device_index.h — host-side handle of a GPU-resident bidirectional FM-index.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <functional>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "fm_layout.h"

namespace sahara {

struct Error : std::runtime_error {
    using std::runtime_error::runtime_error;
};

#define SH_HIP(expr)                                                                         \
    do {                                                                                     \
        hipError_t _e = (expr);                                                              \
        if (_e != hipSuccess)                                                                \
            throw ::sahara::Error(std::string("HIP error '") + hipGetErrorString(_e) +       \
                                  "' at " __FILE__ ":" + std::to_string(__LINE__) + ": " #expr); \
    } while (0)

// (test hook, SAHARA_TEST_HIGH_ADDR=1) every DevBuf starts at an address
// whose low 32-bit word has bit 31 set, 2 GiB more allocated for the shift:
// a kernel that rebuilds a 64-bit address from a sign-extended 32-bit half
// (the round-5 fault) then faults or reads the wrong memory
// in the GPU tests instead of depending on where the allocator puts things.
inline bool highAddrHook() {
    static const bool on = [] {
        const char* e = std::getenv("SAHARA_TEST_HIGH_ADDR");
        return e && std::atoi(e) == 1;
    }();
    return on;
}

template <typename T>
struct DevBuf {  // minimal owning device buffer that only ever grows
    T* ptr = nullptr;
    size_t cap = 0;
    void* base = nullptr;  // the allocation (ptr, unless highAddrHook)
    void reserve(size_t n) {
        if (n <= cap) return;
        release();
        if (n) {
            const bool high = highAddrHook();
            SH_HIP(hipMalloc(&base, n * sizeof(T) + (high ? (size_t)1 << 31 : 0)));
            const uint32_t lo = (uint32_t)reinterpret_cast<uintptr_t>(base);
            const size_t off = !high || (lo & 0x80000000u) ? 0 : (size_t)(0x80000000u - lo);
            ptr = reinterpret_cast<T*>(static_cast<char*>(base) + off);
        }
        cap = n;
    }
    void release() {
        if (base) (void)hipFree(base);
        base = nullptr;
        ptr = nullptr;
        cap = 0;
    }
    ~DevBuf() { release(); }
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    DevBuf(DevBuf&& o) noexcept : ptr(o.ptr), cap(o.cap), base(o.base) { o.ptr = nullptr; o.cap = 0; o.base = nullptr; }
    DevBuf& operator=(DevBuf&& o) noexcept {
        if (this != &o) {
            release();
            ptr = o.ptr;
            cap = o.cap;
            base = o.base;
            o.ptr = nullptr;
            o.cap = 0;
            o.base = nullptr;
        }
        return *this;
    }
};

// Text (and patterns) for the text phase as 3-bit-plane blocks: block i holds
// symbols [32i, 32i+32) as {plane0, plane1, plane2, 0}, bit j of plane b =
// bit b of symbol 32i+j. One 16-B load per 32 symbols, and per-symbol masks of
// 32 symbols come out of 3 word operations (search.hip, kSearchTextBatch).
constexpr uint64_t kTextPadBlocks = 4096;  // zero blocks after the text (text-phase windows)
inline uint64_t text3Blocks(uint64_t n) { return (n + 31) / 32 + kTextPadBlocks; }

struct DeviceIndex {
    int device = 0;
    uint32_t sigma = 6;
    uint32_t rate = 16;
    uint64_t n = 0;                 // text length incl. delimiters
    std::vector<uint64_t> recLens;
    std::vector<uint64_t> recStarts;
    uint64_t C[8] = {0};
    DevBuf<OccLine> occF, occR;     // n/64 + 1 lines each
    DevBuf<uint32_t> samples;       // text position per sampled row, row order
    uint64_t nsamples = 0;
    DevBuf<uint64_t> dRecStarts;
    // Resident for the search (HBM is 288 GB; at 3 Gbp these are 12 + 1.5 GB):
    DevBuf<uint32_t> saFull;        // SA[row] for every row: locate = one read
    DevBuf<uint4> text3;            // text as 3-bit-plane blocks of 32 symbols, '$' = 0, kTextPadBlocks zero blocks after
    // k-mer table: the bidirectional cursor {lb, lbRev, len, pos} of every
    // ACGT string of length kmerK (2 bits per symbol, first symbol most
    // significant). A search whose first kmerK steps admit no error starts
    // at depth kmerK with one lookup instead of kmerK rank steps.
    DevBuf<uint4> kmer;
    uint32_t kmerK = 0;
    bool kmerPos = false;           // an entry with len 1 holds SA[lb] in its fourth word
    uint64_t deviceBytes() const {
        return (occF.cap + occR.cap) * sizeof(OccLine) + samples.cap * 4 + dRecStarts.cap * 8 + saFull.cap * 4 +
               text3.cap * sizeof(uint4) + kmer.cap * sizeof(uint4);
    }
};

// index_build.hip
// withKmer = false leaves the k-mer table out (a multi-part index builds the
// tables of all its parts at one depth afterwards)
void buildFromText(DeviceIndex& I, const uint8_t* hostRanks, const uint64_t* recLens, uint64_t nrec,
                   uint32_t sigma, uint32_t rate, hipStream_t st, bool withKmer = true);
// host bytes -> device on a stream (an .idx image's arrays; default: hipMemcpyAsync)
using HostUpload = std::function<void(void* dst, const void* src, size_t bytes, hipStream_t st)>;
void buildFromParts(DeviceIndex& I, uint32_t sigma, uint64_t n, const uint64_t* recLens, uint64_t nrec,
                    uint32_t rate, const uint8_t* bwtF, const uint8_t* bwtR, const uint64_t* sampledBits,
                    const uint32_t* samples, uint64_t nsamples, hipStream_t st, bool withKmer = true,
                    const HostUpload* up = nullptr);
// depth of the k-mer table for a text of n symbols: floor(log4 n) + 1, at
// most 16 (a 68.7 GB table at 3 Gbp, where the mean 16-mer occurs 0.7 times:
// most exact first parts of a search then start as a text task), and at most
// what fits in half of the free HBM (`tables` tables of that depth: the parts
// of a multi-part index); SAHARA_KMER overrides (0 = no table)
uint32_t kmerDepth(uint64_t n, uint32_t tables = 1);
// Texts of 2^32 - 2 symbols or more are split into parts at record
// boundaries (rows, SA entries and cursors are 32-bit): first record of each
// part, then nrec. At most SAHARA_PART_SYMBOLS symbols (with delimiters) per
// part when set (tests). A record that alone needs 2^32 - 2 rows is refused.
std::vector<uint64_t> splitRecords(const uint64_t* recLens, uint64_t nrec);
void buildKmerTable(DeviceIndex& I, uint32_t K, hipStream_t st);
void exportParts(const DeviceIndex& I, uint8_t* bwtF, uint8_t* bwtR, uint64_t* sampledBits,
                 uint32_t* samples, hipStream_t st);

}  // namespace sahara
