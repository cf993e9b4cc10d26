// search.h — host-side launch interface of the search / locate kernels.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/sahara_hip.h"
#include "device_index.h"

namespace sahara {

struct SearchArgs {
    const OccLine* occF;
    const OccLine* occR;
    uint32_t C[8];
    uint32_t n;              // text length incl. delimiters (root interval length)
    const uint8_t* pats;     // npat * m ranks
    uint32_t m;
    uint32_t nsearch;
    uint32_t nitems;         // npat * nsearch
    const uint32_t* scheme;  // nsearch * m packed entries (packScheme)
    uint32_t* work;          // item counter
    uint4* stack;            // (stackCap - 4) * (grid threads) spilled nodes, [depth][lane]
    uint32_t stackCap;
    uint4* hits;             // (qid, lb, len, e)
    uint32_t hitCap;
    uint32_t* hitCount;      // reserved slots (waves reserve ranges; unused slots have len 0)
    uint32_t* filled;        // cursors actually written
    uint32_t* flags;         // 1 = stack overflow, 2 = hit-buffer overflow, 4 = corrupt locate
    unsigned long long* counters;  // nodes, rank nodes, lines, -, -, text nodes, conversions
    const uint32_t* sa;      // full SA (text mode / verify)
    const uint8_t* text4;    // 4-bit packed text
    uint32_t verify;         // 1: continue singleton intervals against the text
};

struct LocateArgs {
    const uint4* hits;
    uint64_t nhits;
    const uint64_t* rowOff;
    const OccLine* occF;
    uint32_t C[8];
    const uint32_t* samples;
    uint32_t rate;
    uint64_t* keys;
    uint32_t* flags;
    unsigned long long* counters;  // lf steps
    const uint32_t* sa;            // full SA: locate = one read (when useSA)
    uint32_t useSA;
};

int searchBlocksPerCU(uint32_t sigma, bool edit, size_t lds);
void launchSearch(const SearchArgs& a, uint32_t sigma, bool edit, bool count, uint32_t blocks, size_t lds,
                  hipStream_t st);
size_t rowOffsetsTempBytes(uint64_t nhits);
void rowOffsets(const uint4* hits, uint64_t nhits, uint64_t* off, void* tmp, size_t tmpBytes, hipStream_t st);
void launchLocate(const LocateArgs& a, bool count, hipStream_t st);
size_t sortTempBytes(uint64_t n);
uint64_t* sortKeys(uint64_t* k0, uint64_t* k1, uint64_t n, unsigned endBit, void* tmp, size_t tmpBytes,
                   hipStream_t st);
void launchDecode(const uint64_t* keys, uint64_t n, uint64_t qidBase, const uint64_t* starts, uint32_t nrec,
                  sahara_hit* out, hipStream_t st);
void launchDigest(const sahara_hit* h, uint64_t n, unsigned long long* out, hipStream_t st);

}  // namespace sahara
