// pass.cpp — one pass of the search over the staged patterns: batches
// through seeds, FM phase, text phase, locate, sort and decode on the
// context's streams, and the pass over every part of a
// multi-part index.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <chrono>
#include <exception>
#include <thread>

#include <sys/prctl.h>

#include "ctx.h"

namespace sahara {

// One pass over the staged patterns in batches of <= 4M. Per batch:
//   stream stD: chunk unpack (streamed upload), kSeedItems
//   stream st : kSearchFM                    -> hits, tasks of its slot
//   stream stB: kSearchTextBatch             -> hits of its slot
//   stream stC: row counts + ranks, scan, locate, sort, decode
//   stream stF: the batch's hits to the host sink (streamed calls)
// Ctx::kSlots slots rotate, so the seeds and FM phase of later batches
// (memory-latency bound) overlap the text phase of batch i (ALU bound), the
// text phases run back to back, and locate and sort of batch i-1 fill the
// gaps on stream stC. The issuing thread runs seeds, FM(i), text(i) as soon as
// slot i % kSlots is free; the finisher thread runs finish(i) (locate, sort,
// download), which frees it. Buffer overflow is detected after the fact from
// each batch's flags; the whole pass is then redone on one stream with grown
// buffers (`serial`), re-running a batch until it fits.
void runPass(Ctx* c, bool count, bool serial, sahara_stats& S, bool& overflow);

void runOne(Ctx* c, bool count);

DeviceIndex& partOf(Ctx* c, uint32_t p) { return p == 0 ? c->I : c->more.at(p - 1); }

// Search over a multi-part index: the pass runs over every part in turn (the
// staged patterns and scheme are shared; every part has the same k-mer
// depth), its hits get the part's record offset, and one stable sort by qid
// restores the canonical (qid, seq_id, pos, err) order, since part p's
// records all follow part p - 1's. Exact under P-strict: a DFS node exists in
// the whole index iff its interval is non-empty in some part, and its rows
// are the union of its rows over the parts. Hits reach the
// host after the last part (no per-batch sink).
void run(Ctx* c, bool count) {
    if (c->more.empty()) return runOne(c, count);
    sahara_hit* sink = c->sink;
    c->sink = nullptr;
    sahara_stats T{};
    uint64_t total = 0;
    const auto t0 = std::chrono::steady_clock::now();
    try {
        for (uint32_t p = 0; p <= c->more.size(); ++p) {
            if (p) std::swap(c->I, c->more[p - 1]);
            try {
                runOne(c, count);
            } catch (...) {
                if (p) std::swap(c->I, c->more[p - 1]);
                throw;
            }
            if (p) std::swap(c->I, c->more[p - 1]);
            if (c->outAll.cap < total + c->nout) {  // grow, keeping the parts so far
                DevBuf<sahara_hit> grown;
                grown.reserve(std::max<uint64_t>((total + c->nout) + (total + c->nout) / 4, 1024));
                if (total)
                    SH_HIP(hipMemcpyAsync(grown.ptr, c->outAll.ptr, total * sizeof(sahara_hit), hipMemcpyDeviceToDevice,
                                          c->st));
                SH_HIP(hipStreamSynchronize(c->st));
                c->outAll = std::move(grown);
            }
            launchOffsetSeq(c->out.ptr, c->nout, c->partRec0[p], c->outAll.ptr + total, c->st);
            total += c->nout;
            const sahara_stats& S = c->stats;  // the parts' work adds up
            T.patterns = S.patterns;
            T.search_grid = S.search_grid;
            T.text_grid = S.text_grid;
            T.pipelined = S.pipelined;
            for (uint64_t sahara_stats::*f :
                 {&sahara_stats::batches, &sahara_stats::cursors, &sahara_stats::nodes, &sahara_stats::rank_nodes,
                  &sahara_stats::ext_lines, &sahara_stats::lf_steps, &sahara_stats::text_nodes,
                  &sahara_stats::conversions, &sahara_stats::fm_iterations, &sahara_stats::text_iterations,
                  &sahara_stats::text_active, &sahara_stats::text_refills, &sahara_stats::text_cycles_refill,
                  &sahara_stats::text_cycles_step, &sahara_stats::text_cycles_emit, &sahara_stats::text_compare_steps,
                  &sahara_stats::text_steps, &sahara_stats::text_launches,
                  &sahara_stats::text_pos_tasks, &sahara_stats::text_stolen})
                T.*f += S.*f;
            for (double sahara_stats::*f : {&sahara_stats::search_ms, &sahara_stats::locate_ms, &sahara_stats::sort_ms,
                                            &sahara_stats::text_ms, &sahara_stats::seed_ms})
                T.*f += S.*f;
            T.search_launches += S.search_launches;
        }
        if (c->out.cap < total) {
            c->out.release();
            c->out.reserve(std::max<uint64_t>(total, 1024));
        }
        sortHitsByQid(c->outAll.ptr, total, c->npat, c->out.ptr, c->merge, c->tmp, c->st);
        SH_HIP(hipStreamSynchronize(c->st));
    } catch (...) {
        c->sink = sink;
        throw;
    }
    c->sink = sink;
    c->sinkDone = 0;
    c->nout = total;
    T.hits = total;
    T.total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    T.stage_ms = c->stageMs;
    for (int b = 0; b < 3; ++b) T.upload_chunks[b] = c->stats.upload_chunks[b];
    c->stats = T;
}

void runOne(Ctx* c, bool count) {
    if (!c->staged) throw Error("sahara_gpu_run: nothing staged");
    auto t0 = std::chrono::steady_clock::now();
    // SAHARA_PIPELINE=0 (profiling hook): batch after batch on one stream, so
    // that a kernel trace shows each kernel's stand-alone duration
    if (const char* e = std::getenv("SAHARA_PIPELINE")) c->pipeline = std::atol(e) != 0;
    sahara_stats S{};
    bool overflow = false;
    runPass(c, count, !c->pipeline, S, overflow);
    if (overflow) {
        S = sahara_stats{};
        runPass(c, count, true, S, overflow);
    }
    S.total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    S.stage_ms = c->stageMs;
    c->stats = S;
}

// The hit and task buffers' first sizes (SAHARA_HITCAP / SAHARA_TASKCAP in
// tests), for batches of maxBatch patterns; a pass grows them on overflow.
// sahara_gpu_prepare sizes them the same way.
void initWorkCaps(Ctx* c, uint64_t maxBatch) {
    if (c->hitCap == 0) {
        c->hitCap = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(1u << 20, 8 * maxBatch), 1u << 30);
        if (const char* e = std::getenv("SAHARA_HITCAP")) c->hitCap = (uint32_t)std::max(1L, std::atol(e));
    }
    if (c->taskCap == 0) {
        c->taskCap = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(1u << 20, 8 * maxBatch), 1u << 30);
        if (const char* e = std::getenv("SAHARA_TASKCAP")) c->taskCap = (uint32_t)std::max(1L, std::atol(e));
    }
}

void growCap(uint32_t& cap, uint32_t seen) {
    const uint64_t want = (uint64_t)seen + seen / 4 + 1024;
    if (want >= (1ull << 32) - 2) throw Error("a work buffer would exceed 2^32 entries in one batch");
    cap = std::max<uint32_t>(cap, (uint32_t)want);
}

// The finisher's waits in a streamed call. A blocking-sync wait sleeps in
// the driver until an interrupt wakes it, which took up to ~0.4 ms here (C2:
// the row total after a 50 us scan waited 0.07 ms in one call, 0.37 ms in the
// next); polling the event every pollUs microseconds keeps the thread asleep
// almost all the time and wakes within one period. pollUs 0: blocking sync.
static void waitSleepy(hipEvent_t e, uint32_t pollUs) {
    if (!pollUs) {
        SH_HIP(hipEventSynchronize(e));
        return;
    }
    for (;;) {
        const hipError_t r = hipEventQuery(e);
        if (r == hipSuccess) return;
        if (r != hipErrorNotReady) SH_HIP(r);
        std::this_thread::sleep_for(std::chrono::microseconds(pollUs));
    }
}

void runPass(Ctx* c, bool count, bool serial, sahara_stats& S, bool& overflow) {
    overflow = false;
    S.patterns = c->npat;
    const uint32_t sigma = c->I.sigma;
    // FM LDS: the scheme table, then the bottom fmLdsDepth DFS levels (16 B
    // per lane each; SAHARA_FM_LDS_DEPTH). None by default: with a depth-16
    // k-mer table the FM phase is light, its stack lives in L2, and its 1.2 KB
    // fit beside four text workgroups per CU (measured: depth 0 846M, 1 845M,
    // 4 817M reads/s at C3)
    // In the reference execution (verify off) every node is ranked from the
    // root, the DFS runs ~100x deeper trees and nothing else needs the LDS:
    // the bottom four levels there took C3 from 44.4M to 53.3M reads/s
    // (2: 49.9M, 8: 53.1M; profiles/r02_v1_sweep_ref_fm_lds_depth.txt).
    uint32_t fmLdsDepth = c->verify ? 0u : 4u;
    if (const char* e = std::getenv("SAHARA_FM_LDS_DEPTH")) fmLdsDepth = (uint32_t)std::max(0, std::min(8, std::atoi(e)));
    const size_t lds = (size_t)((c->nsearch * c->m + 3u) & ~3u) * 4 + (size_t)fmLdsDepth * 256 * 16;
    const int fullBpc = searchBlocksPerCU(sigma, c->edit, lds);
    int bpc = fullBpc;
    // Overlapped with the text phase of the previous batch, the FM phase
    // (memory-latency bound) runs one workgroup per CU beside three text
    // workgroups; alone it takes all that fit. (Measured at C3 with pruned
    // text steps: text 3 + FM 2 846-873M reads/s, text 4 + FM 1 845-847M;
    // after the atomic-free locate chain, text 3 + FM 1 917-957M against
    // text 3 + FM 2 883-905M and FM 3 847-890M, alternating runs on one box:
    // 115-131 VGPRs per FM wave leave the SIMDs' registers to the text waves
    // and the locate chain.)
    // patterns per batch: 4M (2M in a streamed call: its first batch waits
    // for the host to pack and upload it, its last one's hits for the
    // download, so smaller ones shorten both ends; C3 compact reads path
    // 584-615M -> 668-689M reads/s, profiles/r03_pcie_batch_sweep.txt),
    // fewer for schemes with many searches (work items must fit 2^31);
    // SAHARA_BATCH sets it (tests of the pipeline)
    uint64_t maxBatch = std::min<uint64_t>(c->streaming ? 1ull << 21 : 1ull << 22, (1ull << 31) / c->nsearch);
    if (const char* e = std::getenv("SAHARA_BATCH"))
        maxBatch = std::max<uint64_t>(1, std::min<uint64_t>((1ull << 31) / c->nsearch, std::atoll(e)));
    if (c->blockRecs) maxBatch = std::min<uint64_t>(maxBatch, 1ull << 27);  // compact records: qid - q0 < 2^28
    const uint64_t batchesHere = (c->npat + maxBatch - 1) / maxBatch;
    if (!serial && batchesHere > 1 && c->verify) bpc = 1;
    if (const char* e = std::getenv("SAHARA_FM_BPC")) bpc = std::max(1, std::min(searchBlocksPerCU(sigma, c->edit, lds), std::atoi(e)));
    const uint32_t blocks = (uint32_t)(c->numCU * bpc);
    // the first batch's FM phase has nothing to overlap with: full occupancy
    const uint32_t firstBlocks = std::getenv("SAHARA_FM_BPC") ? blocks : (uint32_t)(c->numCU * fullBpc);
    const uint64_t T = (uint64_t)std::max(blocks, firstBlocks) * 256;
    const uint32_t stackCap = std::max<uint32_t>(c->maxErr, 1) * (2 * sigma - 2) + 2;
    // a ring of stackCap levels per lane (work stealing moves a stack's bottom up)
    const uint32_t stackLevels = stackCap;
    c->stack.reserve((size_t)stackLevels * T);  // levels beyond the LDS part
    S.search_grid = blocks;

    // text phase geometry (LDS per lane: window | pattern | stack)
    // window: |t| + what both sides can still consume <= m + 2k symbols, plus
    // the block alignment of its start (31 symbols); 3 words per block
    // (exact start: m + 2k symbols in whole blocks, copied funnel-shifted from
    // one block more, where both fit the copy's 8 loads; else the block-aligned
    // start below it)
    const uint32_t exactBlocks = (c->m + 2 * c->maxErr + 31) / 32;
    const bool exactWindow = exactBlocks + 1 <= 8 && c->patBlocks <= 8;
    const uint32_t winBlocks = exactWindow ? exactBlocks : (c->m + 2 * c->maxErr + 31 + 31) / 32;
    const uint32_t textStack = 2 * c->maxErr + 2;
    const uint32_t tableWords = std::max<uint32_t>(2 * c->nsearch * c->m, kTextTableMin);
    const size_t textLds = (size_t)tableWords * 4 + (size_t)256 * (3 * (winBlocks + c->patBlocks) + 2 * textStack) * 4;
    if (const char* e = std::getenv("SAHARA_SPLIT")) c->split = (uint32_t)std::max(0L, std::atol(e));
    // read on every pass, so unsetting them restores the defaults (in-process A/Bs)
    const char* eSteps = std::getenv("SAHARA_TEXT_STEPS");
    const char* eRefill = std::getenv("SAHARA_REFILL_AT");
    c->textSteps = eSteps ? (uint32_t)std::max(1L, std::atol(eSteps)) : kTextStepsDefault;
    c->refillAt = eRefill ? (uint32_t)std::min(64L, std::max(1L, std::atol(eRefill))) : kRefillAtDefault;
    int tbpc = 0;
    // the text phase addresses text and a batch's patterns with 32-bit buffer offsets
    const bool textFits = text3Blocks(c->I.n) * 16 <= 0xFFFFFF00ull &&
                          maxBatch * c->patBlocks * 16 <= 0xFFFFFF00ull;
    const int textShape = textShapeOf(winBlocks, c->patBlocks, exactWindow);
    if (c->verify && c->m <= 2047 && textLds <= 160 * 1024 && textFits)
        tbpc = textBlocksPerCU(sigma, c->edit, count, textShape, textLds);
    // overlapped with the FM phase, three text workgroups per CU beside its one
    // (four would fit: r2 v8 measured text 4 against 3 in alternating pairs,
    // C3 914-943M vs 880-952M on one box and 873-914M vs 953-956M on another,
    // C2 950-1013M vs 956-1026M: the sign flips with the box)
    if (!serial && batchesHere > 1) tbpc = std::min(tbpc, 3);
    if (const char* e = std::getenv("SAHARA_TEXT_BPC"); e && tbpc > 0)
        tbpc = std::max(1, std::min(textBlocksPerCU(sigma, c->edit, count, textShape, textLds), std::atoi(e)));
    if (std::getenv("SAHARA_DUMP_COUNTERS"))
        std::fprintf(stderr, "text geometry: shape %d lds %zu blocks/CU %d (alone %d) serial %d\n", textShape, textLds, tbpc,
                     textBlocksPerCU(sigma, c->edit, count, textShape, textLds), (int)serial);
    const uint32_t split = tbpc > 0 ? c->split : 0u;
    // (pipelined) the first batch's text phase starts on its seed tasks while
    // its FM phase runs; a device-resident lone batch does not: its FM phase
    // runs at full occupancy, and its text phase split in two measured 45M
    // against 68M reads/s at C5 (r1)
    // A streamed call seeds its first batch in two parts, the first chunk's
    // as soon as that chunk is up, and starts the text phase on their tasks
    // while the rest of the batch uploads, seeds and runs its FM phase, also
    // when the call is one batch (C5 95.2M -> 100.2M, C2 500M -> 503M, C3
    // 792M -> 805M; without the split seeds a lone batch's early text phase
    // lost: C5 89.9M, C2 475M; profiles/r04_chunk_seeds_ab.txt).
    // SAHARA_CHUNK_SEEDS=0: one seed launch per batch
    const char* csEnv = std::getenv("SAHARA_CHUNK_SEEDS");
    const bool chunkSeeds = c->streaming && !serial && split && !(csEnv && std::atoi(csEnv) == 0);
    const bool early = !serial && split && (batchesHere > 1 || chunkSeeds);
    const bool chunked0 = early && chunkSeeds;
    const uint32_t textBlocks = (uint32_t)(c->numCU * std::max(tbpc, 1));
    S.text_grid = split ? textBlocks : 0u;
    S.pipelined = serial ? 0u : 1u;

    initWorkCaps(c, maxBatch);
    // batch boundaries: equal batches of <= maxBatch patterns, or (pipelined,
    // SAHARA_RAMP / SAHARA_RAMP_END: lists of pattern counts, ',' or ':') given
    // first and last batches around equal middle ones
    std::vector<uint64_t> bstart{0};
    {
        auto list = [](const char* e) {
            std::vector<uint64_t> v;
            for (const char* p = e; p && *p;) {
                char* end = nullptr;
                const unsigned long long x = std::strtoull(p, &end, 10);
                if (end == p) break;
                if (x) v.push_back(x);
                p = (*end == ',' || *end == ':') ? end + 1 : end;
            }
            return v;
        };
        std::vector<uint64_t> head = list(std::getenv("SAHARA_RAMP")), tail = list(std::getenv("SAHARA_RAMP_END"));
        uint64_t edges = 0;
        for (auto& x : head) edges += x = std::min(x, maxBatch);
        for (auto& x : tail) edges += x = std::min(x, maxBatch);
        if (serial || c->npat < edges + maxBatch) head.clear(), tail.clear(), edges = 0;
        for (uint64_t x : head) bstart.push_back(bstart.back() + x);
        const uint64_t mid = c->npat - edges, q0 = bstart.back(), nmid = (mid + maxBatch - 1) / maxBatch;
        for (uint64_t i = 1; i <= nmid; ++i) bstart.push_back(q0 + mid * i / nmid);
        for (uint64_t x : tail) bstart.push_back(bstart.back() + x);
    }
    const uint64_t nbatch = bstart.size() - 1;
    // per batch, 16 words of pinned host memory: the slot's counters (0-6),
    // the locate flags (7), the row total (8-9), the long / huge segment
    // counts (10, 11) and the rows --max_hits keeps (12-13). Pinned, so that their copies are plain DMA writes: a
    // copy into pageable memory waited behind the streamed upload's copies
    // (4.5 ms for batch 0's row total at C3 over PCIe, r3)
    if (c->pinnedCap < nbatch * 16) {
        if (c->pinned) SH_HIP(hipHostFree(c->pinned));
        c->pinned = nullptr;
        c->pinnedCap = nbatch * 16;
        SH_HIP(hipHostMalloc(&c->pinned, c->pinnedCap * sizeof(uint32_t)));
    }
    if (c->qoff.cap < maxBatch + 1) {
        c->qoff.reserve(maxBatch + 1);
        c->big.reserve(maxBatch);
        c->huge.reserve(maxBatch);
    }
    // The search kernels rank each hit's rows in its query's segment as they
    // write it (an atomic add on the slot's per-query count), so the locate
    // chain starts at the scan. Until r4 a pass of scattered atomics in the
    // chain (kCountRows) did it, beside the next batches' search, where the
    // chain lagged behind them: C3 805M -> 843M, C2 482M -> 503M, C5 94.2M ->
    // 95.6M reads/s (profiles/r04_emit_rank_ab.txt)
    for (auto& sl : c->slot) {
        sl.qcnt.reserve(maxBatch + 1);
        SH_HIP(hipMemsetAsync(sl.qcnt.ptr, 0, (maxBatch + 1) * sizeof(uint32_t), c->st));
    }
    hipStream_t sA = c->st, sB = serial ? c->st : c->stB, sC = serial ? c->st : c->stC, sD = serial ? c->st : c->stD;
    c->mark("pass", 0);
    SH_HIP(hipStreamSynchronize(c->st));
    SH_HIP(hipStreamSynchronize(c->stB));
    SH_HIP(hipStreamSynchronize(c->stC));
    SH_HIP(hipStreamSynchronize(c->stD));
    c->mark("pass synced", 0);
    // (profiling hook, count mode) the first text launch's wave lives
    const bool probe = count && std::getenv("SAHARA_DUMP_COUNTERS") != nullptr;
    if (count) {
        SH_HIP(hipMemsetAsync(c->counters.ptr, 0, kCounters * sizeof(unsigned long long), sA));
        SH_HIP(hipMemsetAsync(c->counters.ptr + 33, 0xFF, sizeof(unsigned long long), sA));  // (minima)
        SH_HIP(hipMemsetAsync(c->counters.ptr + 37, 0xFF, sizeof(unsigned long long), sA));
        SH_HIP(hipMemsetAsync(c->counters.ptr + 38, 0xFF, sizeof(unsigned long long), sA));
    }
    c->nout = 0;
    c->sinkDone = 0;
    c->sinkOk = c->sink != nullptr || c->blockRecs != nullptr;
    c->batchQ0.clear();
    c->batchEnd.clear();
    // a slot's counters and queues are zero when its `free` event fires:
    // here for the first use, after its locate (finish) for the next
    auto resetSlot = [&](Ctx::Slot& sl, hipStream_t s) {
        SH_HIP(hipMemsetAsync(sl.small.ptr, 0, 8 * sizeof(uint32_t), s));
        SH_HIP(hipMemsetAsync(sl.queues.ptr, 0, 768 * sizeof(uint32_t), s));
        SH_HIP(hipEventRecord(sl.free, s));
    };
    for (auto& sl : c->slot) resetSlot(sl, sA);

    // the batch's seed tasks are all written (stream sD): the first batch's
    // text phase launches on them (the count snapshot in small[5]) before its
    // FM phase ends
    auto seedTasksDone = [&](Ctx::Slot& sl) {
        SH_HIP(hipMemcpyAsync(sl.small.ptr + 5, sl.small.ptr + 4, 4, hipMemcpyDeviceToDevice, sD));
    };
    auto issueFM = [&](uint64_t b) {
        Ctx::Slot& sl = c->slot[b % Ctx::kSlots];
        const uint64_t q0 = bstart[b], nb = bstart[b + 1] - q0;
        sl.hits.reserve((size_t)c->hitCap + 1);
        sl.rank.reserve((size_t)c->hitCap + 1);
        sl.tasks.reserve((size_t)c->taskCap);
        SH_HIP(hipStreamWaitEvent(sA, sl.free, 0));  // the slot's previous batch is fully consumed
        SearchArgs a{};
        a.occF = c->I.occF.ptr;
        a.occR = c->I.occR.ptr;
        for (int i = 0; i < 8; ++i) a.C[i] = (uint32_t)c->I.C[i];
        a.n = (uint32_t)c->I.n;
        a.pats = c->pats.ptr + q0 * c->patWords;
        a.patWords = c->patWords;
        a.m = c->m;
        a.nsearch = c->nsearch;
        a.nitems = (uint32_t)(nb * c->nsearch);
        a.scheme = c->scheme.ptr;
        a.work = sl.queues.ptr;
        a.hitCount = sl.small.ptr + 1;
        a.flags = sl.small.ptr + 2;
        a.filled = sl.small.ptr + 3;
        a.taskCount = sl.small.ptr + 4;
        a.stack = c->stack.ptr;
        a.stackCap = stackCap;
        a.stackLevels = stackLevels;
        // in-wave work stealing at the launch's end: in the reference execution
        // (verify off) the FM phase is the whole search and its tail idles half
        // the lanes (C5 2.7M -> 5.3M reads/s, C3 52.7M -> 62.7M); beside the
        // text phase it changed nothing measurable (C5 93.4M vs 94.8M, C3
        // within the spread; profiles/r04_fm_steal_ab.txt)
        a.stealAt = c->verify ? 0u : 8u;
        if (const char* e = std::getenv("SAHARA_FM_STEAL_AT")) a.stealAt = (uint32_t)std::max(0, std::min(64, std::atoi(e)));
        a.hits = sl.hits.ptr;
        a.hitCap = c->hitCap;
        a.counters = c->counters.ptr;
        a.tasks = sl.tasks.ptr;
        a.taskCap = c->taskCap;
        a.split = split;
        a.ldsDepth = fmLdsDepth;
        a.qcnt = sl.qcnt.ptr;
        a.rank = sl.rank.ptr;
        // starting cursors; reference execution (verify off) ranks every node
        // from the root, so it does not use the k-mer table
        SeedArgs sd{};
        sd.pats = a.pats;
        sd.patWords = c->patWords;
        sd.nsearch = c->nsearch;
        sd.nitems = a.nitems;
        sd.n = a.n;
        sd.kmer = c->verify && c->I.kmerK ? c->I.kmer.ptr : nullptr;
        sd.kmerK = c->I.kmerK;
        sd.kmerPos = c->I.kmerPos ? 1u : 0u;
        if (const char* e = std::getenv("SAHARA_KMER_POS"); e && std::atoi(e) == 0) sd.kmerPos = 0;  // (A/B)
        sd.kmerStart = c->kmerStart.ptr;
        sl.seeds.reserve(a.nitems);
        sl.seedItem.reserve(a.nitems);
        sd.seeds = sl.seeds.ptr;
        sd.seedItem = sl.seedItem.ptr;
        sd.seedCount = sl.small.ptr + 6;
        sd.m = c->m;
        const char* seedTasks = std::getenv("SAHARA_SEED_TASKS");  // 0: every seed goes through the FM kernel
        sd.toText = split >= 1 && (!seedTasks || std::atoi(seedTasks) != 0) ? 1u : 0u;
        sd.tasks = sl.tasks.ptr;
        sd.taskCap = c->taskCap;
        sd.taskCount = sl.small.ptr + 4;
        sd.flags = sl.small.ptr + 2;
        sd.counters = count ? c->counters.ptr : nullptr;
        a.seeds = sl.seeds.ptr;
        a.seedItem = sl.seedItem.ptr;
        a.seedCount = sl.small.ptr + 6;
        // seeds on their own stream (sD), so that they run ahead of the FM
        // phase of the batch before (both are HBM-latency bound and light)
        SH_HIP(hipStreamWaitEvent(sD, sl.free, 0));
        // streamed upload: the batch's patterns (packed here on the host while
        // the batches before it search; unpacked on sD ahead of its seeds)
        auto seeds = [&](uint32_t i0, uint32_t i1) {
            sd.itemBegin = i0;
            sd.nitems = i1;
            launchSeeds(sd, sigma, std::max<uint32_t>(1, std::min<uint32_t>((i1 - i0 + 1023) / 1024, (uint32_t)c->numCU * 8)), sD);
        };
        if (chunked0 && b == 0) {
            // (streamed, early text) the first chunk's seeds as soon as it is
            // up; the text phase starts on their tasks while the rest of the
            // batch uploads; the other chunks' seeds as each arrives (a lone
            // batch is four chunks: staging.cpp), then the FM phase
            const uint64_t step = c->up.rc ? 2 * c->up.chunk : c->up.chunk;
            const uint64_t p1 = std::min<uint64_t>(bstart[1], step);
            ensureUploaded(c, p1, sD);
            SH_HIP(hipEventRecord(sl.fmStart, sD));
            seeds(0, (uint32_t)(p1 * c->nsearch));
            seedTasksDone(sl);
            SH_HIP(hipEventRecord(sl.seedDone0, sD));
            // each later part's seed launch timed on its own (not the upload waits between)
            uint32_t part = 0;
            for (uint64_t p0 = p1; p0 < bstart[1]; p0 += step, ++part) {
                const uint64_t pe = std::min<uint64_t>(bstart[1], p0 + step);
                ensureUploaded(c, pe, sD);
                while (c->partEv.size() < 2 * (size_t)(part + 1)) {
                    hipEvent_t e;
                    SH_HIP(hipEventCreate(&e));
                    c->partEv.push_back(e);
                }
                SH_HIP(hipEventRecord(c->partEv[2 * part], sD));
                seeds((uint32_t)(p0 * c->nsearch), (uint32_t)(pe * c->nsearch));
                SH_HIP(hipEventRecord(c->partEv[2 * part + 1], sD));
            }
            sl.seedParts = part;
            sl.seedsInParts = true;
        } else {
            sl.seedsInParts = false;
            ensureUploaded(c, bstart[b + 1], sD);
            SH_HIP(hipEventRecord(sl.fmStart, sD));
            seeds(0, a.nitems);
            // the seed tasks end here: the text phase may start on them (a
            // lone device-resident batch's text phase waits for its FM phase:
            // published after it below)
            if (split && early) seedTasksDone(sl);
            SH_HIP(hipEventRecord(sl.seedDone0, sD));
        }
        SH_HIP(hipEventRecord(sl.seedDone, sD));
        SH_HIP(hipStreamWaitEvent(sA, sl.seedDone, 0));
        SH_HIP(hipEventRecord(sl.fmBegin, sA));
        launchSearch(a, sigma, c->edit, count, b == 0 && !early ? firstBlocks : blocks, lds, sA);
        SH_HIP(hipEventRecord(sl.fmDone, sA));
        ++S.search_launches;
    };
    // in-wave work stealing while no task is in hand, once SAHARA_STEAL_AT
    // lanes of a wave are idle (0: off). Measured in one process, alternating:
    // C5 80.4M (off) -> 124.3M (1) / 129.5M (8) reads/s, lanes busy 0.656 ->
    // 0.890; C3 948M -> 1045M / 1056M, 0.787 -> 0.900
    uint32_t stealAt = 8;
    if (const char* e = std::getenv("SAHARA_STEAL_AT")) stealAt = (uint32_t)std::max(0, std::min(64, std::atoi(e)));
    auto issueText = [&](uint64_t b) {
        Ctx::Slot& sl = c->slot[b % Ctx::kSlots];
        // one launch per batch (kSearchTextBatch) after its FM phase; the
        // first batch of an early pass in two: its seed tasks while its FM
        // phase runs, then the tasks the FM phase appended after them
        const bool split0 = early && b == 0;
        sl.twoText = split && split0;
        SH_HIP(hipStreamWaitEvent(sB, split0 ? sl.seedDone0 : sl.fmDone, 0));
        SH_HIP(hipEventRecord(sl.textStart, sB));
        if (split) {
            const uint64_t q0 = bstart[b];
            TextBatchArgs t{};
            t.sa = c->I.saFull.ptr;
            t.text3 = c->I.text3.ptr;
            t.pats3 = c->pats3.ptr + q0 * c->patBlocks;
            t.patBlocks = c->patBlocks;
            t.text3Bytes = (uint32_t)std::min<uint64_t>(text3Blocks(c->I.n) * 16, 0xFFFFFF00ull);
            t.pats3Bytes = (uint32_t)std::min<uint64_t>((bstart[b + 1] - q0) * c->patBlocks * 16, 0xFFFFFF00ull);
            t.m = c->m;
            t.nsearch = c->nsearch;
            t.table = reinterpret_cast<const uint2*>(c->cover.ptr);
            t.tasks = sl.tasks.ptr;
            t.taskCount = sl.small.ptr + 4;
            t.taskCap = c->taskCap;
            t.work = sl.queues.ptr + 256;
            t.hits = sl.hits.ptr;
            t.hitCap = c->hitCap;
            t.hitCount = sl.small.ptr + 1;
            t.filled = sl.small.ptr + 3;
            t.flags = sl.small.ptr + 2;
            t.counters = c->counters.ptr;
            t.winBlocks = winBlocks;
            t.exactWindow = exactWindow ? 1u : 0u;
            t.stackCap = textStack;
            t.tableWords = tableWords;
            t.steps = c->textSteps;
            t.refillAt = c->refillAt;
            t.stealAt = stealAt;
            t.qcnt = sl.qcnt.ptr;
            t.rank = sl.rank.ptr;
            t.probe = probe ? 1u : 0u;
            t.isFirst = b == 0 ? 1u : 0u;
            if (split0) {
                t.taskCount = sl.small.ptr + 5;
                launchTextBatch(t, sigma, c->edit, count, textBlocks, textLds, sB);
                SH_HIP(hipEventRecord(sl.textMid0, sB));
                SH_HIP(hipStreamWaitEvent(sB, sl.fmDone, 0));
                SH_HIP(hipEventRecord(sl.textMid1, sB));
                t.taskBegin = sl.small.ptr + 5;
                t.taskCount = sl.small.ptr + 4;
                t.work = sl.queues.ptr + 512;
                ++S.text_launches;
            }
            launchTextBatch(t, sigma, c->edit, count, textBlocks, textLds, sB);
            ++S.text_launches;
        }
        SH_HIP(hipEventRecord(sl.textDone, sB));
    };
    // locate: row offsets (exclusive scan of len), SA / LF locate, canonical
    // sort, decode into the device-resident output, on stream sC. Needs the
    // batch's counts (host waits for its text phase). Returns false on
    // overflow; `finishCheck` then reads the locate flags and timings.
    uint32_t seenTask = 0, seenHit = 0;  // pipelined overflow: the caps the re-run needs
    // a streamed call's finisher sleeps in its waits while the calling thread
    // and the pool pack (device-resident runs spin)
    const bool sleepy = c->streaming && !serial;
    uint32_t pollUs = 20;
    if (const char* e = std::getenv("SAHARA_POLL_US")) pollUs = (uint32_t)std::max(0, std::atoi(e));
    unsigned long timerSlackNs = 1000;  // the finisher's timer slack (0: the process default)
    if (const char* e = std::getenv("SAHARA_TIMER_SLACK_NS")) timerSlackNs = (unsigned long)std::max(0L, std::atol(e));
    auto finish = [&](uint64_t b) {
        Ctx::Slot& sl = c->slot[b % Ctx::kSlots];
        const uint64_t q0 = bstart[b], nb = bstart[b + 1] - q0;
        c->mark("finish", b);
        // After the text phase, on sC (work on sB would wait for CU slots
        // between two text phases): the per-query row counts are scanned into
        // segment offsets right away, and one small kernel then writes the
        // batch's counters, its row total and its long-segment counts into
        // pinned host memory: one host round trip per batch, not two (until
        // r5 the counters went up first, and the scan waited for the host to
        // check them). A batch whose buffers overflowed is redone anyway, so
        // its scan is wasted work, not wrong work.
        SH_HIP(hipStreamWaitEvent(sC, sl.textDone, 0));
        SH_HIP(hipEventRecord(c->ev[2], sC));
        SH_HIP(hipMemsetAsync(c->small.ptr, 0, 8 * sizeof(uint32_t), sC));
        c->partial.reserve(scanTiles((uint32_t)nb));
        querySegments(sl.qcnt.ptr, (uint32_t)nb, c->qoff.ptr, c->partial.ptr, c->big.ptr, c->small.ptr + 4, c->huge.ptr,
                      c->small.ptr + 5, sC);
        uint32_t* pr = c->pinned + b * 16;
        launchBatchTotals(sl.small.ptr, c->qoff.ptr + nb, c->small.ptr + 4, pr, sC);
        SH_HIP(hipEventRecord(sleepy ? c->evSleep[0] : c->ev[6], sC));
        if (sleepy) waitSleepy(c->evSleep[0], pollUs);
        else SH_HIP(hipEventSynchronize(c->ev[6]));
        c->mark("text done, rows", b);
        const uint32_t* hs = pr;
        float ms = 0;
        if (sl.seedsInParts) {  // the seed launches, not the upload waits between them
            SH_HIP(hipEventElapsedTime(&ms, sl.fmStart, sl.seedDone0));
            for (uint32_t i = 0; i < sl.seedParts; ++i) {
                S.seed_ms += ms;
                SH_HIP(hipEventElapsedTime(&ms, c->partEv[2 * i], c->partEv[2 * i + 1]));
            }
        } else {
            SH_HIP(hipEventElapsedTime(&ms, sl.fmStart, sl.seedDone));
        }
        S.seed_ms += ms;
        SH_HIP(hipEventElapsedTime(&ms, sl.fmBegin, sl.fmDone));
        S.search_ms += ms;
        if (sl.twoText) {  // the two launches, not the wait for the FM phase between them
            SH_HIP(hipEventElapsedTime(&ms, sl.textStart, sl.textMid0));
            S.text_ms += ms;
            SH_HIP(hipEventElapsedTime(&ms, sl.textMid1, sl.textDone));
        } else {
            SH_HIP(hipEventElapsedTime(&ms, sl.textStart, sl.textDone));
        }
        S.text_ms += ms;
        if (hs[2] & 1u) throw Error("search stack overflow (internal bound violated)");
        if (hs[2] & 16u) throw Error("text phase: internal stack bound violated");
        if (hs[2] & (2u | 8u)) {  // hit or task buffer too small
            // (pipelined: issueFM may be reading the caps on the other host
            // thread; they grow after the pass, before the serial re-run)
            if (hs[2] & 8u) growCap(serial ? c->taskCap : seenTask, hs[4]);
            if (hs[2] & 2u) growCap(serial ? c->hitCap : seenHit, hs[1]);
            overflow = true;  // (the scan zeroed the slot's per-query counts)
            resetSlot(sl, sC);
            return false;
        }
        // reserved slots incl. len-0 holes; a wave's last range may reach past
        // the capacity without having written there (no overflow flag)
        const uint64_t nh = std::min<uint64_t>(hs[1], c->hitCap);
        S.cursors += hs[3];
        uint64_t rows = 0;
        std::memcpy(&rows, pr + 8, 8);
        const uint32_t nbig2[2] = {pr[10], pr[11]};
        if (rows >= (1ull << 32)) throw Error("more than 2^32 located hits in one batch of patterns");
        const uint32_t nbig = nbig2[0], nhuge = nbig2[1];
        const uint32_t* hugeList = c->huge.ptr;
        c->k0.reserve(std::max<uint64_t>(rows, 1));
        if (nhuge) c->k1.reserve(std::max<uint64_t>(rows, 1));
        LocateArgs la{};
        la.hits = sl.hits.ptr;
        la.nhits = nh;
        la.qoff = c->qoff.ptr;
        la.rank = sl.rank.ptr;
        la.occF = c->I.occF.ptr;
        for (int i = 0; i < 8; ++i) la.C[i] = (uint32_t)c->I.C[i];
        la.samples = c->I.samples.ptr;
        la.rate = c->I.rate;
        la.keys = c->k0.ptr;
        la.flags = c->small.ptr + 2;
        la.counters = c->counters.ptr + 3;
        la.sa = c->I.saFull.ptr;
        la.useSA = c->locateSA ? 1u : 0u;
        launchLocate(la, count, sC);
        SH_HIP(hipEventRecord(c->ev[3], sC));
        resetSlot(sl, sC);  // the slot's hits are consumed
        if (nhuge) c->tmp.reserve(bigSortTempBytes(rows, nhuge) + 256);
        if (c->nout + rows > c->out.cap) {  // grow the device-resident output
            const size_t want = std::max<size_t>((c->nout + rows) + (c->nout + rows) / 2, 1024);
            sahara_hit* np = nullptr;
            SH_HIP(hipMalloc(&np, want * sizeof(sahara_hit)));
            if (c->nout) SH_HIP(hipMemcpyAsync(np, c->out.ptr, c->nout * sizeof(sahara_hit), hipMemcpyDeviceToDevice, sC));
            SH_HIP(hipStreamSynchronize(sC));
            SH_HIP(hipStreamSynchronize(c->stF));  // sink copies may still read the old buffer
            c->out.release();
            c->out.ptr = np;
            c->out.base = np;
            c->out.cap = want;
        }
        sortDecode(c->k0.ptr, c->k1.ptr, rows, c->qoff.ptr, (uint32_t)nb, c->big.ptr, nbig, hugeList, nhuge, q0,
                   c->I.dRecStarts.ptr, (uint32_t)c->I.recStarts.size(), c->out.ptr + c->nout, c->tmp.ptr, c->tmp.cap,
                   sC);
        if (c->limitN)  // --max_hits: this batch's queries keep their n best positions (search_n)
            rows = limitBatch(c->out.ptr + c->nout, rows, c->qoff.ptr, (uint32_t)nb, c->limitN, c->limitCnt,
                              c->limitOff, c->limitBuf, c->tmp, reinterpret_cast<uint64_t*>(pr + 12), sC);
        SH_HIP(hipEventRecord(c->ev[4], sC));
        // sahara_gpu_search's host sink: the batch's hits go to host memory
        // on stF while later batches search (while they fit the sink)
        c->batchQ0.push_back(q0);
        c->batchEnd.push_back(c->nout + rows);
        if (c->sinkOk && c->nout + rows <= c->sinkCap) {
            const bool compact = c->compactSink && rows * sizeof(uint64_t) <= Ctx::kDownSlot && nb < (1ull << 28);
            if (rows && c->blockRecs) {
                // compact records made in HBM on sC (full grid, ~20 us), then
                // one D2H copy on stF: a copy engine moves them, no workgroup
                // waits on PCIe writes beside the text phase
                launchCompactHits(c->out.ptr + c->nout, rows, q0, c->I.dRecStarts.ptr, c->outRecs.ptr + c->nout, sC,
                                  1u << 16);
                SH_HIP(hipEventRecord(c->ev[7], sC));
                SH_HIP(hipStreamWaitEvent(c->stF, c->ev[7], 0));
                SH_HIP(hipMemcpyAsync(c->blockRecs + c->nout, c->outRecs.ptr + c->nout, rows * sizeof(uint64_t),
                                      hipMemcpyDeviceToHost, c->stF));
            } else if (rows && compact) {  // 8-B records, expanded on the host (Expander)
                const uint64_t j = c->downJobs++;
                const size_t slot = (size_t)(j % Ctx::kDownSlots);
                if (j >= Ctx::kDownSlots) c->expander->waitFor(j + 1 - Ctx::kDownSlots);  // the slot is read
                if (c->downEv.size() <= slot) {
                    const size_t had = c->downEv.size();
                    c->downEv.resize(Ctx::kDownSlots);
                    for (size_t i = had; i < Ctx::kDownSlots; ++i)
                        SH_HIP(hipEventCreateWithFlags(&c->downEv[i], hipEventDisableTiming));
                }
                uint64_t* stage = c->downRing + slot * (Ctx::kDownSlot / sizeof(uint64_t));
                c->outC.reserve(Ctx::kDownSlots * (Ctx::kDownSlot / sizeof(uint64_t)));
                uint64_t* dev = c->outC.ptr + slot * (Ctx::kDownSlot / sizeof(uint64_t));
                launchCompactHits(c->out.ptr + c->nout, rows, q0, c->I.dRecStarts.ptr, dev, sC);
                SH_HIP(hipEventRecord(c->ev[7], sC));
                SH_HIP(hipStreamWaitEvent(c->stF, c->ev[7], 0));
                SH_HIP(hipMemcpyAsync(stage, dev, rows * sizeof(uint64_t), hipMemcpyDeviceToHost, c->stF));
                SH_HIP(hipEventRecord(c->downEv[slot], c->stF));
                c->expander->submit({c->downEv[slot], stage, c->sink + c->nout, rows, q0});
            } else if (rows && c->sinkPinned) {
                SH_HIP(hipStreamWaitEvent(c->stF, c->ev[4], 0));
                SH_HIP(hipMemcpyAsync(c->sink + c->nout, c->out.ptr + c->nout, rows * sizeof(sahara_hit),
                                      hipMemcpyDeviceToHost, c->stF));
            } else if (rows) {  // neither fits: the rest goes after the pass
                c->sinkOk = false;
            }
            if (c->sinkOk) c->sinkDone = c->nout + rows;
        } else {
            c->sinkOk = false;
        }
        SH_HIP(hipMemcpyAsync(c->pinned + b * 16 + 7, c->small.ptr + 2, 4, hipMemcpyDeviceToHost, sC));
        SH_HIP(hipEventRecord(c->ev[5], sC));
        if (sleepy) SH_HIP(hipEventRecord(c->evSleep[2], sC));
        c->nout += rows;
        S.hits += rows;
        return true;
    };
    auto finishCheck = [&](uint64_t b) {
        if (sleepy) waitSleepy(c->evSleep[2], pollUs);  // recorded beside ev[5]
        SH_HIP(hipEventSynchronize(c->ev[5]));
        if (c->pinned[b * 16 + 7] & 4u) throw Error("locate walked off the SA samples (corrupt index)");
        float ms = 0;
        SH_HIP(hipEventElapsedTime(&ms, c->ev[2], c->ev[3]));
        S.locate_ms += ms;
        SH_HIP(hipEventElapsedTime(&ms, c->ev[3], c->ev[4]));
        S.sort_ms += ms;
        c->mark("checked", b);
    };

    if (!serial) {
        // Two host threads. This one packs the queries of a streamed upload
        // and issues seeds, FM(b) and text(b) as soon as batch b's slot is
        // free; a finisher thread waits for each batch's text phase and
        // issues its locate, sort and hit download, so that batch b's hits
        // leave while later batches are still being packed and searched.
        // FM(b) reuses the slot that finish(b - kSlots) released.
        std::mutex mu;
        std::condition_variable cv;
        uint64_t issued = 0, released = 0;  // batches issued; batches whose slot is released
        bool stop = false;
        std::exception_ptr finErr;
        std::thread finisher([&] {
            c->place.bind();
            // its polls sleep 20 us (SAHARA_POLL_US); Linux stretches a sleep
            // by the thread's timer slack (50 us by default), which a lone
            // batch's locate chain waited for twice (C2: ~70 us per wait)
            if (timerSlackNs) prctl(PR_SET_TIMERSLACK, timerSlackNs, 0, 0, 0);
            try {
                SH_HIP(hipSetDevice(c->device));
                bool pending = false;  // finishCheck owed for batch `owed`
                uint64_t owed = 0;
                for (uint64_t f = 0; f < nbatch; ++f) {
                    {
                        std::unique_lock<std::mutex> lk(mu);
                        cv.wait(lk, [&] { return issued > f || stop; });
                        if (issued <= f) break;
                    }
                    if (pending) finishCheck(owed);
                    pending = finish(f);
                    owed = f;
                    {
                        std::lock_guard<std::mutex> g(mu);
                        released = f + 1;
                        if (overflow) stop = true;  // the caller redoes the pass serially
                    }
                    cv.notify_all();
                    if (overflow) break;
                }
                if (pending) finishCheck(owed);
            } catch (...) {
                finErr = std::current_exception();
            }
            std::lock_guard<std::mutex> g(mu);
            stop = true;
            cv.notify_all();
        });
        std::exception_ptr issueErr;
        try {
            for (uint64_t b = 0; b < nbatch; ++b) {
                {
                    std::unique_lock<std::mutex> lk(mu);
                    cv.wait(lk, [&] { return b < released + Ctx::kSlots || stop; });
                    if (stop) break;
                }
                c->mark("issue", b);
                issueFM(b);
                issueText(b);
                c->mark("issued", b);
                ++S.batches;
                {
                    std::lock_guard<std::mutex> g(mu);
                    issued = b + 1;
                }
                cv.notify_all();
            }
        } catch (...) {
            issueErr = std::current_exception();
        }
        {
            std::lock_guard<std::mutex> g(mu);
            if (issueErr) stop = true;
        }
        cv.notify_all();
        finisher.join();
        c->mark("finisher joined", 0);
        SH_HIP(hipStreamSynchronize(sA));
        SH_HIP(hipStreamSynchronize(sB));
        SH_HIP(hipStreamSynchronize(sC));
        SH_HIP(hipStreamSynchronize(sD));
        SH_HIP(hipStreamSynchronize(c->stF));
        c->mark("streams synced", 0);
        if (issueErr) std::rethrow_exception(issueErr);
        if (finErr) std::rethrow_exception(finErr);
        if (overflow) {
            c->taskCap = std::max(c->taskCap, seenTask);
            c->hitCap = std::max(c->hitCap, seenHit);
        }
        if (overflow) return;  // the caller redoes the pass serially with the grown buffers
    } else {
        for (uint64_t b = 0; b < nbatch; ++b) {
            ++S.batches;
            for (;;) {  // re-run the batch until its buffers suffice
                overflow = false;
                issueFM(b);
                issueText(b);
                if (finish(b)) {
                    finishCheck(b);
                    break;
                }
            }
        }
        overflow = false;
        SH_HIP(hipStreamSynchronize(c->stF));
    }
    if (probe) {
        unsigned long long h[kCounters];
        SH_HIP(hipMemcpy(h, c->counters.ptr, sizeof(h), hipMemcpyDeviceToHost));
        std::fprintf(stderr, "text wave lives (first launch, us): last start %.1f first end %.1f last end %.1f mean %.1f; "
                     "tasks all taken seen first %.1f last %.1f by %llu waves, which ran on %.1f on average\n",
                     (h[34] - h[33]) / 100.0, (h[37] - h[33]) / 100.0, (h[35] - h[33]) / 100.0,
                     h[36] / 100.0 / std::max<double>(1, S.text_grid * 4.0), (h[38] - h[33]) / 100.0,
                     (h[39] - h[33]) / 100.0, h[31], h[30] / 100.0 / std::max<double>(1, (double)h[31]));
        std::fprintf(stderr, "text iterations before / after: %llu (busy lanes %.1f) / %llu (busy lanes %.1f); "
                     "nodes stolen %llu\n",
                     h[40], h[41] / std::max(1.0, (double)h[40]), h[42], h[43] / std::max(1.0, (double)h[42]), h[45]);
        std::fprintf(stderr, "text wall per iteration (us) before: refill %.2f steps+emit %.2f; after: refill %.2f steps+emit %.2f\n",
                     h[46] / 100.0 / std::max(1.0, (double)h[40]), h[47] / 100.0 / std::max(1.0, (double)h[40]),
                     h[48] / 100.0 / std::max(1.0, (double)h[42]), h[49] / 100.0 / std::max(1.0, (double)h[42]));
    }
    if (count) {
        unsigned long long h[kCounters];
        SH_HIP(hipMemcpyAsync(h, c->counters.ptr, sizeof(h), hipMemcpyDeviceToHost, sC));
        SH_HIP(hipStreamSynchronize(sC));
        S.nodes = h[0];
        S.rank_nodes = h[1];
        S.ext_lines = h[2];
        S.lf_steps = h[3];
        S.text_nodes = h[5];
        S.conversions = h[6];  // text tasks
        S.fm_iterations = h[7];
        S.text_iterations = h[8];
        S.text_active = h[9];
        S.text_refills = h[10];
        S.text_cycles_refill = h[11];
        S.text_cycles_step = h[12];
        S.text_cycles_emit = h[13];
        S.text_compare_steps = h[14];
        S.text_steps = h[15];
        S.text_pos_tasks = h[16];
        S.text_stolen = h[45];
        if (std::getenv("SAHARA_DUMP_COUNTERS")) {  // (profiling hook: the raw count-mode counters)
            for (uint32_t i = 0; i < kCounters; ++i) std::fprintf(stderr, "%s%llu", i ? " " : "counters ", h[i]);
            std::fprintf(stderr, "\n");
        }
    }
}

}  // namespace sahara
