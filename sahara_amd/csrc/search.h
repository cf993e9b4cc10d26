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
    const uint32_t* pats;    // npat * patWords 4-bit packed pattern words
    uint32_t patWords;
    uint32_t m;
    uint32_t nsearch;
    uint32_t nitems;         // npat * nsearch
    const uint4* seeds;      // starting cursors (kSeedItems), *seedCount of them
    const uint32_t* seedItem;  // their items (pattern * nsearch + search)
    const uint32_t* seedCount;
    const uint32_t* scheme;  // nsearch * m packed entries (packScheme)
    uint32_t* work;          // item counter
    uint4* stack;            // spilled DFS levels beyond the LDS part, [depth][grid thread]
    uint32_t stackCap;       // most entries a lane's stack holds (the DFS bound)
    uint32_t stackLevels;    // levels per lane, a ring (>= stackCap: work stealing moves a stack's bottom up)
    uint32_t stealAt;        // once the seed queue is dry: idle lanes take the bottom stack entry of a busy
                             // lane of their wave once this many are idle (0: off)
    uint4* hits;             // (qid, lb, len, e) or (qid, text pos, 1, e | kPosKnown)
    uint32_t hitCap;
    uint32_t* hitCount;      // reserved slots (waves reserve ranges; unused slots have len 0)
    uint32_t* filled;        // records actually written
    uint32_t* flags;         // 1 stack, 2 hits, 4 locate, 8 tasks, 16 text window
    unsigned long long* counters;  // nodes, rank nodes, lines, lf steps, digest, text nodes, tasks
    uint4* tasks;            // text tasks (row, |t|, qid, meta | search << 24)
    uint32_t taskCap;
    uint32_t* taskCount;
    uint32_t split;          // intervals of <= split rows go to the text phase (0: never)
    uint32_t ldsDepth;       // DFS levels kept in LDS (after the scheme table; the rest spill to HBM)
    // rows ranked where the hits are written: rank[slot] = the hit's first
    // row in its query's segment, qcnt[qid] += len (the batch's per-query row
    // counts, zero on entry; the locate chain's scan reads and clears them)
    uint32_t* qcnt;
    uint32_t* rank;
};

struct SeedArgs {
    const uint32_t* pats;
    uint32_t patWords;
    uint32_t nsearch;
    uint32_t itemBegin;         // items [itemBegin, nitems) of the batch (a batch's seeds in parts)
    uint32_t nitems;
    uint32_t n;
    const uint4* kmer;          // k-mer table (DeviceIndex::kmer), nullptr = start every item at the root
    uint32_t kmerK;
    uint32_t kmerPos;           // the table holds SA[lb] of single-row entries: their tasks carry text positions
    const uint32_t* kmerStart;  // per search: pattern offset of its error-free first kmerK steps, ~0u = n/a
    uint4* seeds;
    uint32_t* seedItem;
    uint32_t* seedCount;
    // a seed whose k-mer occurs once is already a text task: written straight
    // to the task list (the FM kernel's record format) instead of the seeds
    uint32_t m;
    uint32_t toText;            // 1: convert single-row seeds (the text phase runs, split >= 1)
    uint4* tasks;
    uint32_t taskCap;
    uint32_t* taskCount;
    uint32_t* flags;            // 8: task buffer too small
    unsigned long long* counters;  // count mode: text tasks (+6), else nullptr
};

// Text phase LDS: the scheme table comes first and takes at least one block of
// lane words (3 planes x 256 lanes), so that a read of a lane's window block -1
// (left reads near the window start) stays inside the workgroup's LDS.
constexpr uint32_t kTextTableMin = 3u * 256u;

// work counters of count mode (sahara_stats): [0..15] as SearchArgs::counters
// lists them, [16] text tasks that came with their text position (kTaskPos),
// [17..19] text-kernel cycles idle / in grab / whole wave lives
constexpr uint32_t kCounters = 56;
// a task record whose x is already a text position (a k-mer seed with one
// occurrence: DeviceIndex::kmerPos), not an SA row: bit 31 of its y (|t|)
constexpr uint32_t kTaskPos = 0x80000000u;

// One launch of the text phase over one batch's tasks [*taskBegin, *taskCount)
// (kSearchTextBatch)
struct TextBatchArgs {
    const uint32_t* sa;      // full SA: task records carry SA rows (unless kTaskPos), the kernel reads their positions
    const uint4* text3;      // text as 3-bit-plane blocks of 32 symbols (device_index.h)
    const uint4* pats3;      // the batch's patterns as 3-bit-plane blocks, patBlocks per pattern
    uint32_t patBlocks;
    uint32_t text3Bytes;     // bytes of text3 / of the batch's pats3 (buffer-load bounds; < 4 GiB)
    uint32_t pats3Bytes;
    uint32_t m;
    uint32_t nsearch;
    const uint2* table;      // nsearch * m: {packScheme | run << 25, a | b << 12} (capi.cpp textTable)
    const uint4* tasks;
    const uint32_t* taskCount;  // tasks written by the seed / FM kernels (device-side: no host round trip)
    const uint32_t* taskBegin;  // first task of this launch (device-side; nullptr: 0)
    uint32_t taskCap;
    uint32_t* work;          // the launch's striped queue counters (zero)
    uint4* hits;
    uint32_t hitCap;
    uint32_t* hitCount;
    uint32_t* filled;
    uint32_t* flags;
    unsigned long long* counters;
    uint32_t winBlocks;      // window blocks per lane (32 symbols each)
    uint32_t exactWindow;    // 1: the window starts at its first symbol (funnel-shifted copy), else block-aligned
    uint32_t stackCap;       // text DFS stack entries per lane
    uint32_t tableWords;     // LDS words before the lane slots: max(2 * nsearch * m, kTextTableMin)
    uint32_t steps;          // node expansions per lane between wave-level bookkeeping
    uint32_t refillAt;       // refill idle lanes once this many are idle
    uint32_t stealAt;        // once the task queue is dry: idle lanes take the bottom stack entry of a busy
                             // lane of their wave (with its window and pattern) once this many are idle (0: off)
    uint32_t* qcnt;          // as SearchArgs: rows ranked where the hits are written (the FM phase's counts)
    uint32_t* rank;
    uint32_t probe;          // (count mode) wave lives on the wall clock into counters [30..49] ...
    uint32_t isFirst;        // ... for the pass's first launch only
};

struct LocateArgs {
    const uint4* hits;
    uint64_t nhits;
    const uint64_t* qoff;          // per-query row segments (querySegments)
    const uint32_t* rank;          // per cursor: slot of its first row in the segment (querySegments)
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
int textBlocksPerCU(uint32_t sigma, bool edit, bool count, int shape, size_t lds);
int textShapeOf(uint32_t winBlocks, uint32_t patBlocks, bool exactWindow);
// the text phase of one batch (kSearchTextBatch)
void launchTextBatch(const TextBatchArgs& a, uint32_t sigma, bool edit, bool count, uint32_t blocks, size_t lds,
                     hipStream_t st);
void launchSeeds(const SeedArgs& a, uint32_t sigma, uint32_t blocks, hipStream_t st);
void launchPackPatterns(const uint8_t* src, uint64_t npat, uint32_t m, uint32_t patWords, uint32_t sigma,
                        uint32_t* dst, uint32_t* bad, hipStream_t st);
// n symbols, two per byte of nib (low nibble first) -> one per byte of dst
void launchUnpackNibbles(const uint8_t* nib, uint8_t* dst, uint64_t n, hipStream_t st);
void launchOffsetSeq(const sahara_hit* in, uint64_t n, uint64_t rec0, sahara_hit* out, hipStream_t st);
// --max_hits on the device: one batch's hits limited in place, kept rows returned
uint64_t limitBatch(sahara_hit* out, uint64_t rows, const uint64_t* qoff, uint32_t nq, uint32_t n,
                    DevBuf<uint32_t>& kcnt, DevBuf<uint64_t>& koff, DevBuf<sahara_hit>& buf, DevBuf<char>& tmp,
                    uint64_t* hostKept, hipStream_t st);
// key / index buffers of the multi-part merge (kept by the context)
struct MergeBufs {
    DevBuf<uint64_t> k0, k1;
    DevBuf<uint32_t> v0, v1;
};
void sortHitsByQid(const sahara_hit* in, uint64_t n, uint64_t nqid, sahara_hit* out, MergeBufs& B, DevBuf<char>& tmp,
                   hipStream_t st);
void launchCompactHits(const sahara_hit* h, uint64_t n, uint64_t qidBase, const uint64_t* starts, uint64_t* out,
                       hipStream_t st, uint32_t maxBlocks = 8192);
// a streamed chunk of 2-bit codes (read r0's first symbol at symbol `so` of
// src, 0..3) straight into both pattern forms of the patterns [p0, p1)
void launchPackFrom2(const uint8_t* src, uint32_t so, const uint32_t* exc, uint32_t nExc, uint64_t r0, uint64_t p0,
                     uint64_t p1, uint32_t m, bool rc, uint32_t sigma, uint32_t patWords, uint32_t patBlocks,
                     uint32_t* pats, uint4* pats3, hipStream_t st);
// reads [r0, r1) (m bytes each) -> patterns [2 r0, min(2 r1, pEnd)): read, reverse complement, ...
void launchInterleaveRC(const uint8_t* reads, uint64_t r0, uint64_t r1, uint32_t m, uint32_t sigma, uint64_t pEnd,
                        uint8_t* pats, hipStream_t st);
void launchSearch(const SearchArgs& a, uint32_t sigma, bool edit, bool count, uint32_t blocks, size_t lds,
                  hipStream_t st);
// locate + canonical order, per batch: querySegments (rows per query ->
// segments; long segments listed in big, their count in *nbig, read back by
// the host), launchLocate (keys into the segments), sortDecode (short
// segments in registers, medium across a wave, long in LDS, huge by segmented
// radix sort).
uint32_t scanTiles(uint32_t nq);  // u64 partials querySegments needs
// qcnt: the batch's per-query row counts, which the search kernels add up
// as they write the hits (SearchArgs::qcnt); all zero on return
void querySegments(uint32_t* qcnt, uint32_t nq, uint64_t* qoff, uint64_t* partial, uint32_t* big, uint32_t* nbig,
                   uint32_t* huge, uint32_t* nhuge, hipStream_t st);
void launchLocate(const LocateArgs& a, bool count, hipStream_t st);
// a batch's totals into pinned host memory in one launch: out[0..8) = the
// slot's counters (small), out[8..10) = the row total (u64), out[10..12) =
// the long / huge segment counts
void launchBatchTotals(const uint32_t* small, const uint64_t* rowTotal, const uint32_t* segCounts, uint32_t* out,
                       hipStream_t st);
size_t bigSortTempBytes(uint64_t rows, uint32_t nbig);
// long segments (> 64 rows, listed in big) are sorted in LDS, huge ones
// (> 2048, listed in huge) by the segmented radix sort
void sortDecode(uint64_t* k0, uint64_t* k1, uint64_t rows, const uint64_t* qoff, uint32_t nq, const uint32_t* big,
                uint32_t nbig, const uint32_t* huge, uint32_t nhuge, uint64_t qidBase, const uint64_t* starts,
                uint32_t nrec, sahara_hit* out, void* tmp, size_t tmpBytes, hipStream_t st);
void launchPackPatterns3(const uint8_t* src, uint64_t npat, uint32_t m, uint32_t patBlocks, uint4* dst,
                         hipStream_t st);
void launchDigest(const sahara_hit* h, uint64_t n, unsigned long long* out, hipStream_t st);
void launchCopyHits(const sahara_hit* h, uint64_t n, uint64_t qidOffset, sahara_hit* dst, hipStream_t st);

}  // namespace sahara
