// ctx.h — the per-device context of libsahara_hip.so and what the C ABI
// (capi.cpp), the query staging (staging.cpp) and the batch pipeline
// (pass.cpp) share.
#pragma once
#include <hip/hip_runtime.h>
#include <pthread.h>
#include <sched.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/sahara_hip.h"
#include "device_index.h"
#include "search.h"

namespace sahara {

extern thread_local std::string g_err;  // sahara_gpu_last_error

// NUMA placement of a context's own host threads that touch its pinned
// buffers (the pass's finisher, the hit expander, the ring pinning): the CPUs
// of the NUMA node the GPU hangs off (/sys/bus/pci/devices/<bdf>/numa_node),
// as far as the process may use them. The packing pool reads the caller's
// buffers, wherever those are, and stays unbound (staging.cpp hostPool).
// node = -1 (unknown, or SAHARA_NUMA=0): threads stay where the OS puts them.
struct Placement {
    int node = -1;
    int ncpus = 0;      // CPUs the context's threads are bound to (0: not bound)
    cpu_set_t cpus;
    Placement() { CPU_ZERO(&cpus); }
    void bind() const {
        if (ncpus > 0) (void)pthread_setaffinity_np(pthread_self(), sizeof(cpus), &cpus);
    }
};

// Host worker threads of a context (pattern packing for the upload), started
// once: a streamed upload packs several chunks per call, and fresh threads per
// chunk measured slower than the link.
class HostPool {
public:
    explicit HostPool(unsigned workers, const Placement* pl = nullptr) {
        for (unsigned i = 1; i <= workers; ++i)
            ts_.emplace_back([this, i, pl] {
                if (pl) pl->bind();
                loop(i);
            });
    }
    ~HostPool() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : ts_) t.join();
    }
    unsigned size() const { return (unsigned)ts_.size() + 1; }
    // f(t) for every t in [0, size()), t = 0 on the calling thread; f must not throw
    void run(const std::function<void(unsigned)>& f) {
        {
            std::lock_guard<std::mutex> g(mu_);
            job_ = &f;
            pending_ = (unsigned)ts_.size();
            ++gen_;
        }
        cv_.notify_all();
        f(0);
        std::unique_lock<std::mutex> lk(mu_);
        done_.wait(lk, [&] { return pending_ == 0; });
        job_ = nullptr;
    }

private:
    void loop(unsigned id) {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(unsigned)>* f;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
                f = job_;
            }
            (*f)(id);
            std::lock_guard<std::mutex> g(mu_);
            if (--pending_ == 0) done_.notify_all();
        }
    }
    std::vector<std::thread> ts_;
    std::mutex mu_;
    std::condition_variable cv_, done_;
    const std::function<void(unsigned)>* job_ = nullptr;
    uint64_t gen_ = 0;
    unsigned pending_ = 0;
    bool stop_ = false;
};

// Host threads that pack the streamed upload (staging.cpp): a FIFO of tasks
// rather than fork-join rounds, so that the pieces of several chunks are in
// flight at once. A fork-join round per chunk (13 pieces of 4M symbols on 16
// threads at C3) left threads idle at every chunk's end and stopped packing
// whenever the issuing thread was not inside it; queued chunks keep every
// thread busy while the issuing thread enqueues kernels or waits for a slot.
class TaskPool {
public:
    explicit TaskPool(unsigned workers, const Placement* pl = nullptr) {
        for (unsigned i = 0; i < std::max(workers, 1u); ++i)
            ts_.emplace_back([this, pl] {
                if (pl) pl->bind();
                loop();
            });
    }
    ~TaskPool() {  // tasks still queued are dropped (callers wait for theirs first)
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : ts_) t.join();
    }
    unsigned size() const { return (unsigned)ts_.size(); }
    void post(std::function<void()> f) {
        {
            std::lock_guard<std::mutex> g(mu_);
            q_.push_back(std::move(f));
        }
        cv_.notify_one();
    }
    void postMany(std::vector<std::function<void()>>& fs) {
        {
            std::lock_guard<std::mutex> g(mu_);
            for (auto& f : fs) q_.push_back(std::move(f));
        }
        cv_.notify_all();
        fs.clear();
    }

private:
    void loop() {
        for (;;) {
            std::function<void()> f;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
                if (stop_) return;
                f = std::move(q_.front());
                q_.pop_front();
            }
            f();
        }
    }
    std::vector<std::thread> ts_;
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<std::function<void()>> q_;
    bool stop_ = false;
};

// A group of tasks posted to a TaskPool that the poster waits for.
struct TaskGroup {
    std::atomic<uint64_t> left{0};
    std::mutex mu;
    std::condition_variable cv;
    void begin(uint64_t n) { left.store(n, std::memory_order_relaxed); }
    void oneDone() {
        if (left.fetch_sub(1, std::memory_order_acq_rel) == 1) {
            std::lock_guard<std::mutex> g(mu);
            cv.notify_all();
        }
    }
    void wait() {
        if (left.load(std::memory_order_acquire) == 0) return;
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return left.load(std::memory_order_acquire) == 0; });
    }
};

// Host side of sahara_gpu_search's compact hit download: batch by batch, the
// 8-B records (search.hip kCompactHits) land in pinned staging memory on
// stream stF, and this thread expands them into the caller's sahara_hit
// buffer (record id by binary search over the record starts) on a few worker
// threads while later batches still search. Cuts the PCIe download to a third
// (8 of 24 B per hit).
class Expander {
public:
    struct Job {
        hipEvent_t ev;           // the batch's download is done
        const uint64_t* src;     // compact records (pinned staging)
        sahara_hit* dst;
        uint64_t n, q0;          // records; the batch's first qid
    };
    Expander(int device, unsigned workers, const Placement* pl) : device_(device), pool_(workers, pl) {
        th_ = std::thread([this, pl] {
            if (pl) pl->bind();
            loop();
        });
    }
    ~Expander() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        th_.join();
    }
    void setStarts(const std::vector<uint64_t>* starts) { starts_ = starts; }
    std::function<void(const char*, uint64_t)> mark;  // SAHARA_TIMING=2 trace
    void submit(const Job& j) {
        {
            std::lock_guard<std::mutex> g(mu_);
            q_.push_back(j);
            ++submitted_;
        }
        cv_.notify_all();
    }
    // waits until the first n jobs submitted since reset() are expanded
    void waitFor(uint64_t n) {
        std::unique_lock<std::mutex> lk(mu_);
        idle_.wait(lk, [&] { return done_ >= n || err_; });
    }
    void reset() {
        drain();
        std::lock_guard<std::mutex> g(mu_);
        submitted_ = done_ = 0;
    }
    // waits until every submitted batch is expanded; rethrows the first failure
    void drain() {
        std::unique_lock<std::mutex> lk(mu_);
        idle_.wait(lk, [&] { return q_.empty() && !busy_; });
        if (err_) {
            std::exception_ptr e = err_;
            err_ = nullptr;
            std::rethrow_exception(e);
        }
    }

private:
    void loop() {
        (void)hipSetDevice(device_);
        for (;;) {
            Job j{};
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
                if (q_.empty()) return;
                j = q_.front();
                q_.erase(q_.begin());
                busy_ = true;
            }
            try {
                SH_HIP(hipEventSynchronize(j.ev));
                if (mark) mark("expand", done_);
                expand(j);
                if (mark) mark("expanded", done_);
            } catch (...) {
                std::lock_guard<std::mutex> g(mu_);
                if (!err_) err_ = std::current_exception();
            }
            std::lock_guard<std::mutex> g(mu_);
            busy_ = false;
            ++done_;
            idle_.notify_all();
        }
    }
    void expand(const Job& j) {
        const std::vector<uint64_t>& S = *starts_;
        const unsigned nt = pool_.size();
        const uint64_t per = (j.n + nt - 1) / nt;
        pool_.run([&](unsigned t) {
            const uint64_t b = std::min(j.n, (uint64_t)t * per), e = std::min(j.n, b + per);
            uint32_t seq = 0;
            uint64_t lo = 1, hi = 0;  // the current record's [start, next start): empty
            for (uint64_t i = b; i < e; ++i) {
                const uint64_t v = j.src[i], g = (v >> 4) & 0xFFFFFFFFull;
                if (g < lo || g >= hi) {  // hits come sorted by (qid, seq_id, pos): mostly the same record
                    seq = (uint32_t)(std::upper_bound(S.begin(), S.end(), g) - S.begin() - 1);
                    lo = S[seq];
                    hi = seq + 1 < S.size() ? S[seq + 1] : UINT64_MAX;
                }
                sahara_hit& h = j.dst[i];
                h.qid = j.q0 + (v >> 36);
                h.seq_id = seq;
                h.err = (uint32_t)(v & 15u);
                h.pos = g - lo;
            }
        });
    }
    int device_;
    HostPool pool_;
    const std::vector<uint64_t>* starts_ = nullptr;
    std::thread th_;
    std::mutex mu_;
    std::condition_variable cv_, idle_;
    std::vector<Job> q_;
    bool stop_ = false, busy_ = false;
    uint64_t submitted_ = 0, done_ = 0;
    std::exception_ptr err_;
};

// Text-phase scheduling defaults (SAHARA_TEXT_STEPS / SAHARA_REFILL_AT override
// them per pass). Two micro-steps per iteration beat four by 5% on C3 and 2% on
// C5, C2 within noise (profiles/r05_text_steps_ab.txt).
constexpr uint32_t kTextStepsDefault = 2;
constexpr uint32_t kRefillAtDefault = 8;
struct Ctx {
    int device = 0;
    Placement place;                      // NUMA node of the device; the context's threads run there
    hipStream_t st = nullptr;
    int numCU = 0;
    DeviceIndex I;
    // A text of 2^32 - 2 symbols or more is indexed in parts (splitRecords):
    // part 0 is I, parts 1.. are `more`; a search runs over each part in turn
    // (swapped into I) and merges the hits (run). partRec0[p] = the global id
    // of part p's first record. exportPart selects the part the export test
    // hooks read (sahara_gpu_select_part).
    std::vector<DeviceIndex> more;
    std::vector<uint64_t> partRec0{0};
    uint32_t exportPart = 0;
    DevBuf<sahara_hit> outAll;            // multi-part: hits of the parts so far
    MergeBufs merge;                      // multi-part: sort keys of the merge by qid

    // staged inputs
    DevBuf<uint32_t> pats;                // 4-bit packed patterns, patWords per pattern (FM phase)
    DevBuf<uint4> pats3;                  // 3-bit-plane blocks, patBlocks per pattern (text phase)
    uint64_t npat = 0;
    uint32_t m = 0, patWords = 0, patBlocks = 0;
    DevBuf<uint32_t> scheme, cover, kmerStart;        // FM scheme table; text table (textTable)
    uint32_t nsearch = 0;
    uint32_t maxErr = 0;
    bool edit = true;
    bool staged = false;
    bool verify = true;
    bool locateSA = true;
    uint32_t split = 1;                   // text-phase threshold (rows per interval)
    uint32_t textSteps = kTextStepsDefault;  // text-phase micro-steps per lane per wave iteration
    uint32_t refillAt = kRefillAtDefault;    // text-phase batch refill threshold (idle lanes)

    // work buffers. Batches rotate over kSlots slots so that seeds and the FM
    // phase run batches ahead (streams `stD`, `st`) of the text phase (stream
    // `stB`), while earlier batches run their locate and sort (stream `stC`).
    static constexpr int kSlots = 5;
    struct Slot {
        DevBuf<uint4> hits, tasks, seeds;  // seeds: starting cursors (kSeedItems -> kSearchFM)
        DevBuf<uint32_t> seedItem;
        DevBuf<uint32_t> qcnt, rank;      // rows ranked at emission: per-query row counts (zero between
                                          // batches), per hit slot its first row's place in its segment
        DevBuf<uint32_t> small;           // -, hitCount, flags, filled, taskCount, seed tasks, seedCount
        DevBuf<uint32_t> queues;          // striped work counters: FM seeds [0, 256), text tasks: the seed
                                          // tasks [256, 512), the FM phase's [512, 768)
        // kernel spans, each recorded on the kernel's own stream right around
        // its launch(es): seeds fmStart..seedDone (sD), FM fmBegin..fmDone
        // (sA), text textStart..textDone (sB); seedDone0: the batch's first
        // seed tasks are written
        hipEvent_t fmStart = nullptr, seedDone = nullptr, seedDone0 = nullptr, seedMid = nullptr, fmBegin = nullptr,
                   fmDone = nullptr, textStart = nullptr, textDone = nullptr, free = nullptr;
        // the first batch of an early pass launches its text phase twice:
        // textStart..textMid0, then textMid1..textDone (not the wait between)
        hipEvent_t textMid0 = nullptr, textMid1 = nullptr;
        bool twoText = false;
        bool seedsInParts = false;        // seeds in parts: fmStart..seedDone0, then Ctx::partEv's pairs
        uint32_t seedParts = 0;           // (the later parts: Ctx::partEv[2 i], [2 i + 1] around part i)
    } slot[kSlots];
    hipStream_t stB = nullptr, stC = nullptr, stD = nullptr;  // text, locate / sort, seeds
    std::vector<hipEvent_t> partEv;  // around the first batch's later seed launches (created on demand)
    uint32_t* pinned = nullptr;           // host copies of the slots' small counters (8 u32 per batch)
    // two pinned staging chunks for handing hits to pageable host memory: the
    // DMA of one chunk overlaps the host copy out of the other (copyOut)
    static constexpr size_t kOutChunk = 32u << 20;
    void* outStage[2] = {nullptr, nullptr};
    size_t pinnedCap = 0;
    bool pipeline = true;
    DevBuf<uint4> stack;                  // FM spill stack (stream st only)
    DevBuf<uint8_t> rawPats;              // staged pattern bytes before packing
    DevBuf<uint8_t> nibPats;              // the same, two symbols per byte as uploaded (stageIn)
    bool nibbleUpload = true;             // SAHARA_NIBBLE_UPLOAD=0: pattern bytes go up as given
    uint8_t* nibHost = nullptr;           // pinned: the packed patterns on their way up (stage)
    size_t nibHostCap = 0;
    DevBuf<uint32_t> small;               // scratch counters for single-stream helpers
    DevBuf<unsigned long long> counters;  // nodes, rank nodes, lines, lf steps, digest, text nodes, tasks
    DevBuf<uint64_t> qoff, k0, k1;        // per-query row segments of a batch; locate keys
    DevBuf<uint64_t> partial;             // tile sums of the segment scan
    DevBuf<uint32_t> big, huge;           // long / huge segments
    DevBuf<char> tmp;
    DevBuf<sahara_hit> out;
    uint64_t nout = 0;
    double stageMs = 0;                   // wall time of the last stage(): H2D, pack, validation
    uint32_t hitCap = 0, taskCap = 0;
    sahara_stats stats{};
    hipEvent_t ev[8] = {};
    // the finisher's waits in a streamed call (text done, row total, batch
    // checked): blocking-sync events, so that it sleeps instead of spinning a
    // CPU that the packing threads need (a 16-CPU quota on the GPU box)
    hipEvent_t evSleep[3] = {};

    // Streamed query upload (sahara_gpu_search, sahara_gpu_search_reads): the
    // source rows go up in chunks, each packed on the host (two symbols per
    // byte, ranks checked) into a slot of a pinned ring and copied on stream
    // stE when the first batch that needs it is issued, so that the upload of
    // later batches overlaps the search of earlier ones. ringEv[s] fires once
    // slot s's last DMA is done: the device-side unpacking waits for it, and
    // the host waits for it before packing into the slot again. The ring is
    // pinned once per context, in the background while the index loads.
    struct Upload {
        const uint8_t* src = nullptr;  // host symbols: the patterns, or the reads (rc); prepacked: 2-bit codes
        bool rc = false;               // reads: reverse complements interleaved on the device
        uint32_t bits = 4;             // 2: ACGT codes + N list, 4: nibbles, 8: bytes as given
        uint64_t rows = 0;             // source rows
        uint64_t chunk = 0;            // source rows per chunk (even: chunks start at even symbols)
        uint64_t done = 0;             // source rows enqueued
        uint64_t submitted = 0;        // chunks whose packing is posted to the pool (2 bits)
        uint32_t ahead = 6;            // chunks packed ahead of the issued ones (SAHARA_PACK_AHEAD)
        bool bad = false;              // a chunk held a byte that is no rank of this index
        double hostMs = 0;             // host time spent packing and enqueueing
        uint64_t chunks[3] = {0, 0, 0};  // chunks sent at 2 / 4 / 8 bits per symbol
        // reads that arrive two bits per symbol (sahara_gpu_search_packed):
        // chunks are copied into the ring, not packed; source symbol s of
        // the call is stream symbol sym0 + s; the N positions of the call's
        // reads are on the device (nList, relative to each chunk's first
        // whole byte), chunk j's from entry nFirst[j]
        bool prepacked = false;
        bool srcPinned = false;        // prepacked codes in page-locked memory: DMA'd from there, no copy
        uint64_t sym0 = 0;
        std::vector<uint64_t> nFirst;
    } up;
    DevBuf<uint32_t> nList;
    // the packed reads' N list last checked whole (strictly ascending): a
    // stream processed shard by shard is checked once, not once per shard
    const uint64_t* nPosChecked = nullptr;
    uint64_t nCountChecked = 0;
    bool streaming = false;
    hipStream_t stE = nullptr, stF = nullptr;  // pattern upload; hit download (sink)
    // SAHARA_TIMING=2: timing events around each chunk's DMA (bytes, events)
    std::vector<std::pair<uint64_t, std::pair<hipEvent_t, hipEvent_t>>> dmaEv;
    size_t dmaUsed = 0;
    static constexpr size_t kRingSlots = 8, kRingSlot = 32u << 20;  // 256 MB pinned
    uint8_t* ring = nullptr;
    hipEvent_t ringEv[kRingSlots] = {};
    // Chunks packed ahead (2-bit upload): chunk j packs into ring slot
    // j % kRingSlots on the pool's threads while the issuing thread still
    // enqueues earlier batches; uploadChunk waits for its pieces, then lists
    // the N positions and enqueues the DMA (staging.cpp packAhead).
    struct PackJob {
        uint64_t chunk = UINT64_MAX;               // in flight or finished: chunk index
        uint64_t pieces = 0, pieceSyms = 0;
        std::atomic<int> bad{0};
        std::vector<std::vector<uint32_t>> exc;    // per piece: N positions (chunk-relative symbols)
        TaskGroup group;
    } packJobs[kRingSlots];
    std::thread ringInit;                 // pins the ring (started by newCtx)
    uint64_t ringLoadNext = 0;            // uploadViaRing's next slot
    bool ringFailed = false;
    DevBuf<uint32_t> badFlag;             // device rank check of streamed chunks
    DevBuf<uint8_t> readRaw;              // streamed reads before the reverse-complement interleave
    std::unique_ptr<TaskPool> pool;       // declared after packJobs: its threads end first
    unsigned poolCap = 0;
    Placement packPlace;                  // the pool's CPUs when bound
    int poolNode = -2;                    // NUMA node the pool is bound to (-1: unbound)
    // host sink of sahara_gpu_search: each batch's sorted hits go to host
    // memory (pinned) on stF while later batches search
    sahara_hit* sink = nullptr;
    uint64_t sinkCap = 0, sinkDone = 0;
    bool sinkOk = false;
    uint64_t lastHits = 0;                // hits of the previous sahara_gpu_search (sink size estimate)
    // compact download into the sink (Expander): device records of the
    // pass, their pinned host staging, one event per batch's download
    // (batch b's records land in slot b % kDownSlots of a pinned ring,
    // pinned with the upload ring; the slot is reused once batch b is expanded)
    bool compactSink = false, sinkPinned = false;
    DevBuf<uint64_t> outC;
    static constexpr size_t kDownSlots = 3, kDownSlot = 64u << 20;  // 8M records per batch
    uint64_t* downRing = nullptr;
    uint64_t downJobs = 0;                // batches handed to the expander this call
    std::vector<hipEvent_t> downEv;
    std::unique_ptr<Expander> expander;
    // sahara_gpu_search_reads_compact: each batch's hits as 8-B records,
    // made by kCompactHits in HBM (outRecs, sinkCap entries) and copied by a
    // copy engine on stF into this pinned host buffer (sinkCap records); per
    // batch its first qid and one past its last record (the blocks of
    // sahara_hit_blocks). (Written by the kernel straight into the sink over
    // PCIe, the records held CU slots beside the text phase: C3 592M against
    // 632M reads/s with the copy engine, profiles/r03_pcie_compact_dma.txt.)
    uint64_t* blockRecs = nullptr;
    DevBuf<uint64_t> outRecs;
    std::vector<uint64_t> batchQ0, batchEnd;
    std::vector<uint64_t> recStartsEnd;   // record starts + the text length (sahara_hit_blocks.rec_starts)
    // --max_hits n applied per batch on the device (single-part indexes;
    // limitBatch), 0: off
    uint32_t limitN = 0;
    DevBuf<uint32_t> limitCnt;
    DevBuf<uint64_t> limitOff;
    DevBuf<sahara_hit> limitBuf;
    // SAHARA_TIMING=2: host-side marks of one call (ms since its start, what)
    bool traceOn = false;
    std::chrono::steady_clock::time_point traceT0;
    std::mutex traceMu;
    std::vector<std::pair<double, std::string>> trace;
    void mark(const char* what, uint64_t i) {
        if (!traceOn) return;
        const double t = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - traceT0).count();
        std::lock_guard<std::mutex> g(traceMu);
        trace.emplace_back(t, std::string(what) + " " + std::to_string(i));
    }

    ~Ctx() {
        // the pinning thread assigns ring and downRing: it must be done before
        // either is read (a context closed or failed right after newCtx)
        if (ringInit.joinable()) ringInit.join();
        expander.reset();
        for (hipEvent_t e : downEv) (void)hipEventDestroy(e);
        for (hipEvent_t e : partEv) (void)hipEventDestroy(e);
        if (downRing) (void)hipHostFree(downRing);
        for (auto& e : ev)
            if (e) (void)hipEventDestroy(e);
        for (auto& e : evSleep)
            if (e) (void)hipEventDestroy(e);
        for (auto& e : ringEv)
            if (e) (void)hipEventDestroy(e);
        if (ring) (void)hipHostFree(ring);
        if (stE) (void)hipStreamDestroy(stE);
        for (auto& d : dmaEv) {
            (void)hipEventDestroy(d.second.first);
            (void)hipEventDestroy(d.second.second);
        }
        if (stF) (void)hipStreamDestroy(stF);
        for (auto& sl : slot)
            for (hipEvent_t e : {sl.fmStart, sl.seedDone, sl.seedDone0, sl.seedMid, sl.fmBegin, sl.fmDone, sl.textStart,
                                 sl.textDone, sl.free, sl.textMid0, sl.textMid1})
                if (e) (void)hipEventDestroy(e);
        if (pinned) (void)hipHostFree(pinned);
        if (nibHost) (void)hipHostFree(nibHost);
        for (void* p : outStage)
            if (p) (void)hipHostFree(p);
        if (stB) (void)hipStreamDestroy(stB);
        if (stC) (void)hipStreamDestroy(stC);
        if (stD) (void)hipStreamDestroy(stD);
        if (st) (void)hipStreamDestroy(st);
    }
};

template <typename F>
int guarded(F&& f) {
    try {
        f();
        return 0;
    } catch (const std::exception& e) {
        g_err = e.what();
    } catch (...) {
        g_err = "unknown error";
    }
    return -1;
}

bool hitLess(const sahara_hit& a, const sahara_hit& b);
void limitHits(std::vector<sahara_hit>& v, uint32_t n);
void handOver(const std::vector<sahara_hit>& v, sahara_hit** hits, uint64_t* n_hits);
Ctx* newCtx(int device);
unsigned hostThreads(const Ctx* c, unsigned cap);
Ctx* ctxOf(void* p);
TaskPool& hostPool(Ctx* c);
Placement placementOfNode(int node);
// host bytes -> device through the pinned upload ring, copied into it by the
// pool's threads (an index image's arrays: staging.cpp)
void uploadViaRing(Ctx* c, void* dst, const void* src, size_t bytes, hipStream_t st);
// every pack job posted by the streamed upload is finished (the caller's
// source buffer is no longer read): before a new call stages, after a failed one
void drainPacking(Ctx* c);

// staging.cpp: scheme tables, the query packers, the streamed upload
void packSchemeTable(const uint32_t* pi, const uint32_t* l, const uint32_t* u, uint32_t ns, uint32_t m,
                     std::vector<uint32_t>& out, uint32_t& maxErr);
void textTable(const uint32_t* pi, const uint32_t* l, const uint32_t* u, uint32_t ns, uint32_t m,
               const std::vector<uint32_t>& packed, std::vector<uint32_t>& out);
bool hostHasAvx2();
bool hostHasAvx512();
uint64_t pack2Best(const uint8_t* in, uint8_t* out, uint64_t count, uint32_t sigma, uint64_t base,
                   std::vector<uint32_t>& exc);
uint64_t pack2Avx512(const uint8_t* in, uint8_t* out, uint64_t count, uint32_t sigma, uint64_t base,
                     std::vector<uint32_t>& exc);
uint64_t pack2Scalar(const uint8_t* in, uint8_t* out, uint64_t count, uint32_t sigma, uint64_t base,
                     std::vector<uint32_t>& exc);
uint64_t pack2Avx2(const uint8_t* in, uint8_t* out, uint64_t count, uint32_t sigma, uint64_t base,
                   std::vector<uint32_t>& exc);
void uploadChunk(Ctx* c, hipStream_t kst);
void ensureUploaded(Ctx* c, uint64_t patEnd, hipStream_t kst);
void stageScheme(Ctx* c, uint64_t npat, uint32_t m, const uint32_t* pi, const uint32_t* l, const uint32_t* u,
                 uint32_t ns, int edit);
// reads given two bits per symbol (sahara_gpu_search_packed[_compact])
struct PackedReads {
    uint64_t sym0;          // stream position of the first read's first symbol
    const uint64_t* nPos;   // stream positions of N, ascending (any outside the reads are ignored)
    uint64_t nCount;
};
void stageStreamed(Ctx* c, const uint8_t* src, uint64_t rows, bool rc, uint64_t npat, uint32_t m,
                   const uint32_t* pi, const uint32_t* l, const uint32_t* u, uint32_t ns, int edit,
                   const PackedReads* packed = nullptr);
void stage(Ctx* c, const uint8_t* ranks, uint64_t npat, uint32_t m, const uint32_t* pi, const uint32_t* l,
           const uint32_t* u, uint32_t ns, int edit);

// pass.cpp: one pass over the staged patterns (every part of the index)
DeviceIndex& partOf(Ctx* c, uint32_t p);
void run(Ctx* c, bool count);
void runOne(Ctx* c, bool count);
void runPass(Ctx* c, bool count, bool serial, sahara_stats& S, bool& overflow);
void growCap(uint32_t& cap, uint32_t seen);
void initWorkCaps(Ctx* c, uint64_t maxBatch);

}  // namespace sahara
