// capi.cpp — the C ABI of libsahara_hip.so (include/sahara_hip.h).
//
// The drop-in boundary for sahara's hot path: index residency
// (search.cpp:162-169), GPU index construction (index.cpp:87-100), and
// search + locate (search.cpp:218-250). No C++ types or exceptions cross it.

#include <hip/hip_runtime.h>
#include <immintrin.h>
#include <sys/mman.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <memory>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <random>
#include <unordered_map>
#include <string>
#include <atomic>
#include <thread>
#include <vector>

#include "../../include/sahara_hip.h"
#include "device_index.h"
#include "idx_format.h"
#include "search.h"

using namespace sahara;

namespace {

thread_local std::string g_err;

// Host worker threads of a context (pattern packing for the upload), started
// once: a streamed upload packs several chunks per call, and fresh threads per
// chunk measured slower than the link.
class HostPool {
public:
    explicit HostPool(unsigned workers) {
        for (unsigned i = 1; i <= workers; ++i) ts_.emplace_back([this, i] { loop(i); });
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
    Expander(int device, unsigned workers) : device_(device), pool_(workers) {
        th_ = std::thread([this] { loop(); });
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

struct Ctx {
    int device = 0;
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
    uint32_t textSteps = 4;               // text-phase micro-steps per lane per wave iteration
    uint32_t refillAt = 8;                // text-phase batch refill threshold (idle lanes)

    // work buffers. Batches rotate over three slots so that the FM phase runs
    // up to two batches ahead (stream `st`) of the text phase (stream `stB`),
    // while batch i-1 runs its locate and sort (stream `stC`).
    static constexpr int kSlots = 5;
    struct Slot {
        DevBuf<uint4> hits, tasks, seeds;  // seeds: starting cursors (kSeedItems -> kSearchFM)
        DevBuf<uint32_t> seedItem;
        DevBuf<uint32_t> small;           // -, hitCount, flags, filled, taskCount, seed tasks, seedCount
        DevBuf<uint32_t> queues;          // striped work counters: FM seeds [0, 256), text tasks [256, 512), [512, 768)
        hipEvent_t fmStart = nullptr, seedDone = nullptr, fmDone = nullptr, textStart = nullptr, textDone = nullptr,
                   free = nullptr;
    } slot[kSlots];
    hipStream_t stB = nullptr, stC = nullptr, stD = nullptr;  // text, locate / sort, seeds
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
    DevBuf<uint32_t> qcnt, big;           // per-query row counts (zero between batches); long segments
    DevBuf<char> tmp;
    DevBuf<sahara_hit> out;
    uint64_t nout = 0;
    double stageMs = 0;                   // wall time of the last stage(): H2D, pack, validation
    uint32_t hitCap = 0, taskCap = 0;
    sahara_stats stats{};
    hipEvent_t ev[8] = {};

    // Streamed query upload (sahara_gpu_search, sahara_gpu_search_reads): the
    // source rows go up in chunks, each packed on the host (two symbols per
    // byte, ranks checked) into a slot of a pinned ring and copied on stream
    // stE when the first batch that needs it is issued, so that the upload of
    // later batches overlaps the search of earlier ones. ringEv[s] fires once
    // slot s's last DMA is done: the device-side unpacking waits for it, and
    // the host waits for it before packing into the slot again. The ring is
    // pinned once per context, in the background while the index loads.
    struct Upload {
        const uint8_t* src = nullptr;  // host symbols: the patterns, or the reads (rc)
        bool rc = false;               // reads: reverse complements interleaved on the device
        uint32_t bits = 4;             // 2: ACGT codes + N list, 4: nibbles, 8: bytes as given
        uint64_t rows = 0;             // source rows
        uint64_t chunk = 0;            // source rows per chunk (even: chunks start at even symbols)
        uint64_t done = 0;             // source rows enqueued
        bool bad = false;              // a chunk held a byte that is no rank of this index
        double hostMs = 0;             // host time spent packing and enqueueing
        uint64_t chunks[3] = {0, 0, 0};  // chunks sent at 2 / 4 / 8 bits per symbol
    } up;
    std::vector<std::vector<uint32_t>> excParts;  // per packing thread: N positions of a 2-bit chunk
    bool streaming = false;
    hipStream_t stE = nullptr, stF = nullptr;  // pattern upload; hit download (sink)
    static constexpr size_t kRingSlots = 8, kRingSlot = 32u << 20;  // 256 MB pinned
    uint8_t* ring = nullptr;
    hipEvent_t ringEv[kRingSlots] = {};
    std::thread ringInit;                 // pins the ring (started by newCtx)
    bool ringFailed = false;
    DevBuf<uint32_t> badFlag;             // device rank check of streamed chunks
    DevBuf<uint8_t> readRaw;              // streamed reads before the reverse-complement interleave
    std::unique_ptr<HostPool> pool;
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
        expander.reset();
        for (hipEvent_t e : downEv) (void)hipEventDestroy(e);
        if (downRing) (void)hipHostFree(downRing);
        for (auto& e : ev)
            if (e) (void)hipEventDestroy(e);
        if (ringInit.joinable()) ringInit.join();
        for (auto& e : ringEv)
            if (e) (void)hipEventDestroy(e);
        if (ring) (void)hipHostFree(ring);
        if (stE) (void)hipStreamDestroy(stE);
        if (stF) (void)hipStreamDestroy(stF);
        for (auto& sl : slot)
            for (hipEvent_t e : {sl.fmStart, sl.seedDone, sl.fmDone, sl.textStart, sl.textDone, sl.free})
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

bool hitLess(const sahara_hit& a, const sahara_hit& b) {
    if (a.qid != b.qid) return a.qid < b.qid;
    if (a.seq_id != b.seq_id) return a.seq_id < b.seq_id;
    if (a.pos != b.pos) return a.pos < b.pos;
    return a.err < b.err;
}

// --max_hits n (search_n / search_best_n, search.cpp:228,231,240). Upstream's
// counting rule is unverifiable offline; policy here: per query,
// the n distinct text positions (seq_id, pos) with the fewest errors, ties by
// (seq_id, pos), each reported once with its minimum error count. Input and
// output are in canonical (qid, seq_id, pos, err) order.
void limitHits(std::vector<sahara_hit>& v, uint32_t n) {
    size_t w = 0;
    std::vector<sahara_hit> q;
    for (size_t i = 0; i < v.size();) {
        size_t j = i;
        q.clear();
        for (; j < v.size() && v[j].qid == v[i].qid; ++j)
            if (q.empty() || q.back().seq_id != v[j].seq_id || q.back().pos != v[j].pos) q.push_back(v[j]);
        if (q.size() > n) {
            std::stable_sort(q.begin(), q.end(), [](const sahara_hit& a, const sahara_hit& b) { return a.err < b.err; });
            q.resize(n);
            std::sort(q.begin(), q.end(), hitLess);
        }
        for (auto& h : q) v[w++] = h;
        i = j;
    }
    v.resize(w);
}

void handOver(const std::vector<sahara_hit>& v, sahara_hit** hits, uint64_t* n_hits) {
    auto* buf = static_cast<sahara_hit*>(std::malloc(std::max<size_t>(v.size(), 1) * sizeof(sahara_hit)));
    if (!buf) throw Error("out of host memory for hits");
    if (!v.empty()) std::memcpy(buf, v.data(), v.size() * sizeof(sahara_hit));
    *hits = buf;
    *n_hits = v.size();
}

Ctx* newCtx(int device) {
    int n = 0;
    SH_HIP(hipGetDeviceCount(&n));
    if (device < 0 || device >= n)
        throw Error("no HIP device " + std::to_string(device) + " (found " + std::to_string(n) + ")");
    SH_HIP(hipSetDevice(device));
    auto c = std::make_unique<Ctx>();
    c->device = device;
    hipDeviceProp_t prop;
    SH_HIP(hipGetDeviceProperties(&prop, device));
    if (std::string(prop.gcnArchName).find("gfx950") == std::string::npos)
        throw Error(std::string("libsahara_hip is built for gfx950 (MI355X); device is ") + prop.gcnArchName);
    c->numCU = prop.multiProcessorCount;
    SH_HIP(hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking));
    SH_HIP(hipStreamCreateWithFlags(&c->stB, hipStreamNonBlocking));
    SH_HIP(hipStreamCreateWithFlags(&c->stC, hipStreamNonBlocking));
    SH_HIP(hipStreamCreateWithFlags(&c->stD, hipStreamNonBlocking));
    SH_HIP(hipStreamCreateWithFlags(&c->stE, hipStreamNonBlocking));
    SH_HIP(hipStreamCreateWithFlags(&c->stF, hipStreamNonBlocking));
    for (auto& e : c->ev) SH_HIP(hipEventCreate(&e));
    for (auto& e : c->ringEv) SH_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    // the streamed upload's pinned ring, pinned while the caller builds or
    // loads the index (pinning 256 MB takes ~50 ms)
    Ctx* raw = c.get();
    raw->ringInit = std::thread([raw] {
        (void)hipSetDevice(raw->device);
        if (hipHostMalloc(reinterpret_cast<void**>(&raw->ring), Ctx::kRingSlots * Ctx::kRingSlot, hipHostMallocPortable) !=
            hipSuccess) {
            raw->ring = nullptr;
            raw->ringFailed = true;
        }
        if (hipHostMalloc(reinterpret_cast<void**>(&raw->downRing), Ctx::kDownSlots * Ctx::kDownSlot,
                          hipHostMallocPortable) != hipSuccess)
            raw->downRing = nullptr;  // no compact download: hits go to a pinned sink whole
    });
    for (auto& sl : c->slot) {
        for (hipEvent_t* e : {&sl.fmStart, &sl.seedDone, &sl.fmDone, &sl.textStart, &sl.textDone, &sl.free})
            SH_HIP(hipEventCreate(e));
        sl.small.reserve(8);
        sl.queues.reserve(768);
    }
    for (void*& p : c->outStage) SH_HIP(hipHostMalloc(&p, Ctx::kOutChunk));
    c->small.reserve(8);
    c->counters.reserve(16);
    SH_HIP(hipMemset(c->counters.ptr, 0, 16 * sizeof(unsigned long long)));
    return c.release();
}

Ctx* ctxOf(void* p) {
    if (!p) throw Error("null context");
    Ctx* c = static_cast<Ctx*>(p);
    SH_HIP(hipSetDevice(c->device));
    return c;
}

void packSchemeTable(const uint32_t* pi, const uint32_t* l, const uint32_t* u, uint32_t ns, uint32_t m,
                std::vector<uint32_t>& out, uint32_t& maxErr) {
    if (ns == 0) throw Error("empty search scheme");
    if (m == 0 || m > kMaxPatternLen) throw Error("pattern length out of range");
    out.resize((size_t)ns * m);
    maxErr = 0;
    for (uint32_t s = 0; s < ns; ++s) {
        const uint32_t* P = pi + (size_t)s * m;
        uint32_t lo = P[0], hi = P[0];
        if (P[0] >= m) throw Error("scheme pi out of range");
        for (uint32_t p = 0; p < m; ++p) {
            const uint32_t L = l[(size_t)s * m + p], U = u[(size_t)s * m + p];
            if (L > U || U > kMaxErrors) throw Error("scheme bounds must satisfy l <= u <= 15");
            if (p > 0) {
                if (P[p] == hi + 1) hi = P[p];
                else if (lo > 0 && P[p] == lo - 1) lo = P[p];
                else throw Error("scheme pi is not a connected order (search.cpp:191 expand)");
            }
            maxErr = std::max(maxErr, U);
        }
        for (uint32_t p = 0; p < m; ++p) {
            uint32_t right;
            if (p > 0) right = P[p] > P[p - 1];
            else right = m > 1 ? (P[1] > P[0]) : 1u;
            out[(size_t)s * m + p] = packScheme(P[p], l[(size_t)s * m + p], u[(size_t)s * m + p], right);
        }
    }
}

// Text-phase table, two words per (search, pos):
//   x = packScheme(...) | run << 25 — run = number of consecutive positions
//       from pos (<= 127) on the same side with u == u[pos] and l <= u[pos]:
//       a node at pos with e == u[pos] has no error child anywhere in that
//       run, so the DFS is a forced chain of matches through it;
//   y = a | b << 12 | same << 24 — pattern positions [a, b) covered before
//       step pos; `same` (<= run) positions from pos share pos's l as well,
//       so a chain of matches through them branches the same way at each.
void textTable(const uint32_t* pi, const uint32_t* l, const uint32_t* u, uint32_t ns, uint32_t m,
               const std::vector<uint32_t>& packed, std::vector<uint32_t>& out) {
    out.assign((size_t)ns * m * 2, 0);
    for (uint32_t s = 0; s < ns; ++s) {
        const uint32_t* P = pi + (size_t)s * m;
        const uint32_t* L = l + (size_t)s * m;
        const uint32_t* U = u + (size_t)s * m;
        const uint32_t* Q = packed.data() + (size_t)s * m;
        uint32_t a = P[0], b = P[0];
        for (uint32_t p = 0; p < m; ++p) {
            const uint32_t right = (Q[p] >> 24) & 1u;
            uint32_t run = 1, same = 1;
            while (run < 127 && p + run < m && ((Q[p + run] >> 24) & 1u) == right && U[p + run] == U[p] &&
                   L[p + run] <= U[p])
                ++run;
            while (same < run && L[p + same] == L[p]) ++same;
            out[((size_t)s * m + p) * 2] = Q[p] | (run << 25);
            out[((size_t)s * m + p) * 2 + 1] = a | (b << 12) | (same << 24);
            a = std::min(a, P[p]);
            b = std::max(b, P[p] + 1);
        }
    }
}

// Host pattern bytes -> device, one symbol per byte. Patterns cross PCIe as
// two symbols per byte: host threads each pack a slice, 4 MB at a time, into
// one pinned buffer and queue each piece's DMA as soon as it is packed, and
// kUnpackNibbles expands them on the device. At C3 this halves the 2 GB
// upload, which runs at the link's rate. Returns false when a byte is >= 16
// (no rank of any alphabet; smaller out-of-range ranks are found by the
// device check against this index's sigma).
static bool stageIn(Ctx* c, uint8_t* dst, const uint8_t* src, size_t n) {
    if (const char* e = std::getenv("SAHARA_NIBBLE_UPLOAD")) c->nibbleUpload = std::atoi(e) != 0;
    if (!c->nibbleUpload || n < (64u << 20)) {
        SH_HIP(hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, c->st));
        return true;
    }
    const size_t nb = (n + 1) / 2;  // packed bytes
    if (c->nibHostCap < nb) {
        if (c->nibHost) SH_HIP(hipHostFree(c->nibHost));
        c->nibHost = nullptr;
        c->nibHostCap = 0;
        SH_HIP(hipHostMalloc(reinterpret_cast<void**>(&c->nibHost), nb));
        c->nibHostCap = nb;
    }
    c->nibPats.reserve(nb + 8);
    SH_HIP(hipStreamSynchronize(c->st));  // the pinned buffer may still feed the last call's DMA
    uint8_t* out = c->nibHost;
    const unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    constexpr size_t kPiece = 4u << 20;
    const size_t pieces = (nb + kPiece - 1) / kPiece;
    std::atomic<uint64_t> orAll{0};
    std::atomic<int> failed{0};
    auto pack = [&](size_t lo, size_t hi) {  // packed bytes [lo, hi)
        uint64_t acc = 0;
        const uint8_t* in = src + 2 * lo;
        const size_t full = std::min(hi, n / 2);  // bytes with both symbols
        size_t i = lo;
        for (; i + 4 <= full; i += 4, in += 8) {  // 8 symbols -> 4 bytes
            uint64_t v;
            std::memcpy(&v, in, 8);
            acc |= v;
            v = (v | (v >> 4)) & 0x00FF00FF00FF00FFull;
            v = (v | (v >> 8)) & 0x0000FFFF0000FFFFull;
            const uint32_t w = (uint32_t)(v | (v >> 16));
            std::memcpy(out + i, &w, 4);
        }
        for (; i < full; ++i, in += 2) {
            out[i] = (uint8_t)(in[0] | (in[1] << 4));
            acc |= (uint64_t)(in[0] | in[1]);
        }
        for (; i < hi; ++i, in += 2) {  // the odd last symbol
            out[i] = in[0];
            acc |= in[0];
        }
        if (acc & 0xF0F0F0F0F0F0F0F0ull) orAll.fetch_or(1, std::memory_order_relaxed);
        if (hipMemcpyAsync(c->nibPats.ptr + lo, out + lo, hi - lo, hipMemcpyHostToDevice, c->st) != hipSuccess)
            failed.store(1);
    };
    auto worker = [&](unsigned t) {  // pieces t, t + nt, ...: the DMA queue fills front to back
        for (size_t k = t; k < pieces; k += nt) pack(k * kPiece, std::min(nb, (k + 1) * kPiece));
    };
    std::vector<std::thread> ts;
    for (unsigned t = 1; t < nt && t < pieces; ++t) ts.emplace_back(worker, t);
    worker(0);
    for (auto& t : ts) t.join();
    if (failed.load()) throw Error("pattern upload failed");
    launchUnpackNibbles(c->nibPats.ptr, dst, n, c->st);
    return orAll.load() == 0;
}

// Any byte of 8 that is no rank of a sigma-letter alphabet (0, or >= sigma;
// ivs::verify_rank, search.cpp:118-120): nonzero high bits. Exact: with every
// byte in [1, 16) the subtraction borrows nowhere and the addition carries
// out of no byte.
static inline uint64_t badRanks8(uint64_t v, uint64_t big) {
    constexpr uint64_t ones = 0x0101010101010101ull, highs = 0x8080808080808080ull;
    return (v & 0xF0F0F0F0F0F0F0F0ull) | ((v - ones) & ~v & highs) | ((v + big) & highs);
}

// 2 * count symbols of `in` (one per byte) -> count bytes of `out`, two per
// byte (low nibble first); the bytes from `full` on hold one symbol each (the
// odd last symbol of an upload). Returns nonzero if any symbol is no rank in
// [1, sigma).
static uint64_t packNibblesScalar(const uint8_t* in, uint8_t* out, uint64_t full, uint64_t count, uint32_t sigma) {
    const uint64_t big = (uint64_t)(0x80u - sigma) * 0x0101010101010101ull;
    uint64_t acc = 0, i = 0;
    for (; i + 4 <= full; i += 4, in += 8) {  // 8 symbols -> 4 bytes
        uint64_t v;
        std::memcpy(&v, in, 8);
        acc |= badRanks8(v, big);
        v = (v | (v >> 4)) & 0x00FF00FF00FF00FFull;
        v = (v | (v >> 8)) & 0x0000FFFF0000FFFFull;
        const uint32_t w = (uint32_t)(v | (v >> 16));
        std::memcpy(out + i, &w, 4);
    }
    for (; i < full; ++i, in += 2) {
        out[i] = (uint8_t)(in[0] | (in[1] << 4));
        acc |= (uint64_t)(in[0] == 0 || in[0] >= sigma || in[1] == 0 || in[1] >= sigma);
    }
    for (; i < count; ++i, in += 2) {  // the odd last symbol
        out[i] = in[0];
        acc |= (uint64_t)(in[0] == 0 || in[0] >= sigma);
    }
    return acc;
}

// The same with AVX2, 64 symbols per step: pairs combined by one multiply-add
// (lo * 1 + hi * 16), packed to bytes; ranks checked as max(v - 1, sigma - 2)
// == sigma - 2. About a tenth of the scalar instructions per byte, so that
// 16 host threads pack faster than the GPU searches (the streamed upload).
__attribute__((target("avx2"))) static uint64_t packNibblesAvx2(const uint8_t* in, uint8_t* out, uint64_t full,
                                                                uint64_t count, uint32_t sigma) {
    const __m256i mult = _mm256_set1_epi16(0x1001), one = _mm256_set1_epi8(1);
    const __m256i lim = _mm256_set1_epi8((char)(sigma - 2));
    __m256i bad = _mm256_setzero_si256();
    uint64_t i = 0;
    for (; i + 32 <= full; i += 32) {
        const __m256i a = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(in + 2 * i));
        const __m256i b = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(in + 2 * i + 32));
        const __m256i ta = _mm256_sub_epi8(a, one), tb = _mm256_sub_epi8(b, one);
        bad = _mm256_or_si256(bad, _mm256_xor_si256(_mm256_max_epu8(ta, lim), lim));
        bad = _mm256_or_si256(bad, _mm256_xor_si256(_mm256_max_epu8(tb, lim), lim));
        const __m256i pa = _mm256_maddubs_epi16(a, mult), pb = _mm256_maddubs_epi16(b, mult);
        _mm256_storeu_si256(reinterpret_cast<__m256i*>(out + i),
                            _mm256_permute4x64_epi64(_mm256_packus_epi16(pa, pb), 0xD8));
    }
    return (uint64_t)!_mm256_testz_si256(bad, bad) |
           packNibblesScalar(in + 2 * i, out + i, full - i, count - i, sigma);
}

// Nonzero if any byte of [p, p + n) is no rank in [1, sigma).
static uint64_t badRanksScalar(const uint8_t* p, uint64_t n, uint32_t sigma) {
    const uint64_t big = (uint64_t)(0x80u - sigma) * 0x0101010101010101ull;
    uint64_t acc = 0, i = 0;
    for (; i + 8 <= n; i += 8) {
        uint64_t v;
        std::memcpy(&v, p + i, 8);
        acc |= badRanks8(v, big);
    }
    for (; i < n; ++i) acc |= (uint64_t)(p[i] == 0 || p[i] >= sigma);
    return acc;
}

__attribute__((target("avx2"))) static uint64_t badRanksAvx2(const uint8_t* p, uint64_t n, uint32_t sigma) {
    const __m256i one = _mm256_set1_epi8(1), lim = _mm256_set1_epi8((char)(sigma - 2));
    __m256i bad = _mm256_setzero_si256();
    uint64_t i = 0;
    for (; i + 32 <= n; i += 32) {
        const __m256i t = _mm256_sub_epi8(_mm256_loadu_si256(reinterpret_cast<const __m256i*>(p + i)), one);
        bad = _mm256_or_si256(bad, _mm256_xor_si256(_mm256_max_epu8(t, lim), lim));
    }
    return (uint64_t)!_mm256_testz_si256(bad, bad) | badRanksScalar(p + i, n - i, sigma);
}

// Two bits per symbol (SAHARA_UPLOAD_BITS=2, the default for DNA): `count`
// symbols of `in` -> (count + 3) / 4 bytes of `out`, symbol i at bits
// 2 (i % 4) of byte i / 4, coded A C G T = 0 1 2 3. dna5's N (rank 4 of
// sigma 6) is coded 0 and its position (`base` + i) appended to `exc`; the
// device unpacks through a 4-entry table and patches the listed N positions
// (kUnpack2, kPatchRank). Returns nonzero if any symbol is no rank in [1, sigma).
static uint64_t pack2Scalar(const uint8_t* in, uint8_t* out, uint64_t count, uint32_t sigma, uint64_t base,
                            std::vector<uint32_t>& exc) {
    uint64_t bad = 0;
    for (uint64_t i = 0; i < count; i += 4) {
        uint32_t b = 0;
        for (uint32_t q = 0; q < 4 && i + q < count; ++q) {
            const uint32_t r = in[i + q];
            bad |= (uint64_t)(r == 0 || r >= sigma);
            uint32_t code = (r - 1u) & 3u;
            if (sigma == 6 && r >= 4) {
                if (r == 4) exc.push_back((uint32_t)(base + i + q));
                code = r == 5 ? 3u : 0u;
            }
            b |= code << (2 * q);
        }
        out[i / 4] = (uint8_t)b;
    }
    return bad;
}

// The same with AVX2, 128 symbols -> 32 bytes per step: codes t = rank - 1
// (dna5: T 4 -> 3, N 3 -> 0 and listed from a byte mask), pairs combined by
// one multiply-add (t0 + 4 t1), pairs of pairs by another (+ 16), packed to
// bytes and put back in order with one cross-lane permute.
__attribute__((target("avx2"))) static uint64_t pack2Avx2(const uint8_t* in, uint8_t* out, uint64_t count,
                                                          uint32_t sigma, uint64_t base, std::vector<uint32_t>& exc) {
    const __m256i one = _mm256_set1_epi8(1), three = _mm256_set1_epi8(3), four = _mm256_set1_epi8(4);
    const __m256i lim = _mm256_set1_epi8((char)(sigma - 2));
    const __m256i m14 = _mm256_set1_epi16(0x0401), m116 = _mm256_set1_epi32(0x00100001);
    const __m256i order = _mm256_setr_epi32(0, 4, 1, 5, 2, 6, 3, 7);
    const bool dna5 = sigma == 6;
    __m256i bad = _mm256_setzero_si256();
    uint64_t i = 0;
    for (; i + 128 <= count; i += 128) {
        __m256i d[4];
        for (int q = 0; q < 4; ++q) {
            __m256i t = _mm256_sub_epi8(_mm256_loadu_si256(reinterpret_cast<const __m256i*>(in + i + 32 * q)), one);
            bad = _mm256_or_si256(bad, _mm256_xor_si256(_mm256_max_epu8(t, lim), lim));
            if (dna5) {
                const __m256i isN = _mm256_cmpeq_epi8(t, three);
                uint32_t msk = (uint32_t)_mm256_movemask_epi8(isN);
                while (msk) {
                    exc.push_back((uint32_t)(base + i + 32 * q + (uint32_t)__builtin_ctz(msk)));
                    msk &= msk - 1u;
                }
                t = _mm256_andnot_si256(isN, _mm256_add_epi8(t, _mm256_cmpeq_epi8(t, four)));
            }
            t = _mm256_and_si256(t, three);
            d[q] = _mm256_madd_epi16(_mm256_maddubs_epi16(t, m14), m116);
        }
        const __m256i b = _mm256_packus_epi16(_mm256_packus_epi32(d[0], d[1]), _mm256_packus_epi32(d[2], d[3]));
        _mm256_storeu_si256(reinterpret_cast<__m256i*>(out + i / 4), _mm256_permutevar8x32_epi32(b, order));
    }
    return (uint64_t)!_mm256_testz_si256(bad, bad) | pack2Scalar(in + i, out + i / 4, count - i, sigma, base + i, exc);
}

static bool hostHasAvx2() {
    static const bool has = __builtin_cpu_supports("avx2");
    return has;
}

HostPool& hostPool(Ctx* c) {
    if (!c->pool) c->pool = std::make_unique<HostPool>(std::max(1u, std::min(16u, std::thread::hardware_concurrency())) - 1);
    return *c->pool;
}

// Packs the next chunk of the streamed upload (Ctx::Upload) on the host into
// its ring slot, enqueues the slot's DMA on stE (nothing else: the DMAs run
// back to back at the link's rate) and, on stream `kst` after the DMA's event,
// the unpack (and reverse-complement interleave) kernel and both pattern
// packings. A chunk with a byte that is no rank sets up.bad and enqueues
// nothing.
void uploadChunk(Ctx* c, hipStream_t kst) {
    Ctx::Upload& U = c->up;
    const auto t0 = std::chrono::steady_clock::now();
    c->mark("pack", U.done / std::max<uint64_t>(U.chunk, 1));
    const uint64_t r0 = U.done, r1 = std::min(U.rows, r0 + U.chunk);
    const uint32_t m = c->m, sigma = c->I.sigma;
    const uint64_t s0 = r0 * m, s1 = r1 * m, nsym = U.rows * m;  // symbols
    uint8_t* raw = U.rc ? c->readRaw.ptr : c->rawPats.ptr;
    HostPool& P = hostPool(c);
    const unsigned nt = P.size();
    std::atomic<int> bad{0};
    // pieces of 1 MB of packed bytes spread over the pool (a chunk at C3 is
    // ~25 MB packed); one DMA per chunk, overlapping the next chunk's packing
    constexpr uint64_t kPiece = 1u << 20;
    const bool avx2 = hostHasAvx2();
    const uint64_t j = r0 / U.chunk;
    const size_t slot = (size_t)(j % Ctx::kRingSlots);
    // a chunk owns bytes [s0 / 2, (s1 + 1) / 2) of the ring slot and of the
    // device staging buffer at any encoding (s0 is even)
    const uint64_t b0 = s0 / 2, b1 = (s1 + 1) / 2;
    uint32_t bits = U.bits;
    uint64_t nExc = 0, excOff = 0;  // 2 bits: the N list, at byte excOff of the chunk's region
    if (bits != 8) SH_HIP(hipEventSynchronize(c->ringEv[slot]));  // the slot's previous DMA is done
    uint8_t* out = c->ring + slot * Ctx::kRingSlot;
    if (bits == 2) {
        const uint64_t n = s1 - s0, pieces = (n + 4 * kPiece - 1) / (4 * kPiece);
        // one N list per piece: concatenated in piece order they are sorted
        if (c->excParts.size() < pieces) c->excParts.resize(pieces);
        for (auto& v : c->excParts) v.clear();
        P.run([&](unsigned t) {
            for (uint64_t k = t; k < pieces; k += nt) {  // pieces of 4 MB of symbols (1 MB packed)
                const uint64_t lo = k * 4 * kPiece, hi = std::min(n, lo + 4 * kPiece);
                const uint8_t* in = U.src + s0 + lo;
                const uint64_t acc = avx2 ? pack2Avx2(in, out + lo / 4, hi - lo, sigma, lo, c->excParts[k])
                                          : pack2Scalar(in, out + lo / 4, hi - lo, sigma, lo, c->excParts[k]);
                if (acc) bad.store(1, std::memory_order_relaxed);
            }
        });
        for (auto& v : c->excParts) nExc += v.size();
        excOff = ((b0 + (n + 3) / 4 + 3) & ~uint64_t(3)) - b0;  // 4-aligned on the device
        if (excOff + 4 * nExc > b1 - b0) {
            bits = 4;  // N-rich chunk: the list would not fit, go as nibbles
        } else if (!bad.load()) {
            uint8_t* e = out + excOff;
            for (auto& v : c->excParts) {
                if (!v.empty()) std::memcpy(e, v.data(), v.size() * 4);
                e += v.size() * 4;
            }
            SH_HIP(hipMemcpyAsync(c->nibPats.ptr + b0, out, excOff + 4 * nExc, hipMemcpyHostToDevice, c->stE));
        }
    }
    if (bits == 4 && !bad.load()) {
        const uint64_t pieces = (b1 - b0 + kPiece - 1) / kPiece;
        P.run([&](unsigned t) {
            for (uint64_t k = t; k < pieces; k += nt) {
                const uint64_t lo = b0 + k * kPiece, hi = std::min(b1, lo + kPiece);
                const uint64_t full = std::min(hi, std::max(lo, nsym / 2)) - lo;  // bytes with two symbols
                const uint8_t* in = U.src + 2 * lo;
                const uint64_t acc = avx2 ? packNibblesAvx2(in, out + (lo - b0), full, hi - lo, sigma)
                                          : packNibblesScalar(in, out + (lo - b0), full, hi - lo, sigma);
                if (acc) bad.store(1, std::memory_order_relaxed);
            }
        });
        if (!bad.load()) SH_HIP(hipMemcpyAsync(c->nibPats.ptr + b0, out, b1 - b0, hipMemcpyHostToDevice, c->stE));
    } else if (bits == 8) {  // one byte per symbol (SAHARA_UPLOAD_BITS=8): check, then copy as given
        const uint64_t pieces = (s1 - s0 + kPiece - 1) / kPiece;
        P.run([&](unsigned t) {
            for (uint64_t k = t; k < pieces; k += nt) {
                const uint64_t lo = s0 + k * kPiece, hi = std::min(s1, lo + kPiece);
                const uint64_t acc = avx2 ? badRanksAvx2(U.src + lo, hi - lo, sigma)
                                          : badRanksScalar(U.src + lo, hi - lo, sigma);
                if (acc) bad.store(1, std::memory_order_relaxed);
            }
        });
        if (!bad.load()) SH_HIP(hipMemcpyAsync(raw + s0, U.src + s0, s1 - s0, hipMemcpyHostToDevice, c->stE));
    }
    U.hostMs += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (bad.load()) {
        U.bad = true;
        return;
    }
    SH_HIP(hipEventRecord(c->ringEv[slot], c->stE));  // the chunk's DMA
    SH_HIP(hipStreamWaitEvent(kst, c->ringEv[slot], 0));
    if (bits == 4) launchUnpackNibbles(c->nibPats.ptr + b0, raw + s0, s1 - s0, kst);
    U.chunks[bits == 2 ? 0 : bits == 4 ? 1 : 2]++;
    const uint64_t p0 = U.rc ? 2 * r0 : r0, p1 = U.rc ? std::min(2 * r1, c->npat) : r1;
    if (bits == 2) {  // straight into both pattern forms (no byte pass); SAHARA_UPLOAD_BYTES=1: via bytes
        if (!std::getenv("SAHARA_UPLOAD_BYTES")) {
            launchPackFrom2(c->nibPats.ptr + b0, reinterpret_cast<const uint32_t*>(c->nibPats.ptr + b0 + excOff),
                            (uint32_t)nExc, r0, p0, p1, m, U.rc, sigma, c->patWords, c->patBlocks,
                            c->pats.ptr + 0, c->pats3.ptr + 0, kst);
            U.done = r1;
            c->mark("packed", r0 / U.chunk);
            return;
        }
        launchUnpack2(c->nibPats.ptr + b0, raw + s0, s1 - s0, sigma, kst);
        if (nExc) launchPatchRank(reinterpret_cast<const uint32_t*>(c->nibPats.ptr + b0 + excOff), nExc, raw + s0, 4, kst);
    }
    if (U.rc) launchInterleaveRC(c->readRaw.ptr, r0, r1, m, sigma, c->npat, c->rawPats.ptr, kst);
    if (p1 > p0) {
        launchPackPatterns(c->rawPats.ptr + p0 * m, p1 - p0, m, c->patWords, sigma, c->pats.ptr + p0 * c->patWords,
                           c->badFlag.ptr, kst);
        launchPackPatterns3(c->rawPats.ptr + p0 * m, p1 - p0, m, c->patBlocks, c->pats3.ptr + p0 * c->patBlocks, kst);
    }
    U.done = r1;
    c->mark("packed", r0 / U.chunk);
}

// Streamed upload: makes sure the patterns [0, patEnd) are enqueued, their
// device-side packing on stream kst (a no-op when the patterns were staged
// whole).
void ensureUploaded(Ctx* c, uint64_t patEnd, hipStream_t kst) {
    if (!c->streaming) return;
    Ctx::Upload& U = c->up;
    auto covered = [&] { return U.rc ? std::min(2 * U.done, c->npat) : U.done; };
    while (covered() < patEnd) {
        uploadChunk(c, kst);
        if (U.bad) throw Error("pattern rank out of range for this index");
    }
}

// The scheme half of staging: host tables, their upload, the k-mer starts.
void stageScheme(Ctx* c, uint64_t npat, uint32_t m, const uint32_t* pi, const uint32_t* l, const uint32_t* u,
                 uint32_t ns, int edit) {
    if (npat == 0) throw Error("no patterns");
    std::vector<uint32_t> packed, cover;
    packSchemeTable(pi, l, u, ns, m, packed, c->maxErr);
    if ((size_t)ns * m * 4 > 60 * 1024) throw Error("scheme too large for LDS (searches * len > 15360)");
    if (ns > 255) throw Error("at most 255 searches per scheme");
    textTable(pi, l, u, ns, m, packed, cover);
    c->scheme.reserve(packed.size());
    SH_HIP(hipMemcpyAsync(c->scheme.ptr, packed.data(), packed.size() * 4, hipMemcpyHostToDevice, c->st));
    c->cover.reserve(cover.size());
    SH_HIP(hipMemcpyAsync(c->cover.ptr, cover.data(), cover.size() * 4, hipMemcpyHostToDevice, c->st));
    // searches whose first kmerK steps admit no error start from the k-mer table
    std::vector<uint32_t> kst(ns, 0xFFFFFFFFu);
    const uint32_t K = c->I.kmerK;
    for (uint32_t s = 0; K && K <= m && s < ns; ++s) {
        bool exact = true;
        uint32_t lo = pi[(size_t)s * m];
        for (uint32_t p = 0; p < K; ++p) {
            exact = exact && u[(size_t)s * m + p] == 0;
            lo = std::min(lo, pi[(size_t)s * m + p]);
        }
        if (exact) kst[s] = lo;
    }
    c->kmerStart.reserve(ns);
    SH_HIP(hipMemcpyAsync(c->kmerStart.ptr, kst.data(), ns * 4, hipMemcpyHostToDevice, c->st));
    SH_HIP(hipStreamSynchronize(c->st));
    c->nsearch = ns;
    c->edit = edit != 0;
}

// Staging for a streamed search: the scheme now, the patterns chunk by chunk
// during the pass (uploadChunk). src holds `rows` rows of m symbols: the
// patterns, or (rc) the reads whose interleave with their reverse
// complements, cut to npat, is the query list.
void stageStreamed(Ctx* c, const uint8_t* src, uint64_t rows, bool rc, uint64_t npat, uint32_t m,
                   const uint32_t* pi, const uint32_t* l, const uint32_t* u, uint32_t ns, int edit) {
    c->staged = c->streaming = false;
    if (m == 0 || m > kMaxPatternLen) throw Error("pattern length out of range");
    stageScheme(c, npat, m, pi, l, u, ns, edit);
    c->m = m;
    c->npat = npat;
    c->patWords = (m + 7) / 8;
    c->patBlocks = (m + 31) / 32;
    c->rawPats.reserve(npat * m);
    c->pats.reserve(npat * c->patWords + 4);  // + tail words read by paired loads
    c->pats3.reserve(npat * c->patBlocks);
    if (rc) c->readRaw.reserve(rows * m);
    c->badFlag.reserve(1);
    Ctx::Upload& U = c->up;
    U = Ctx::Upload{};
    U.src = src;
    U.rc = rc;
    U.rows = rows;
    // symbols cross PCIe at 2 bits (DNA: A C G T codes, N positions listed),
    // 4 bits (any alphabet) or 8 (as given): SAHARA_UPLOAD_BITS, or
    // SAHARA_NIBBLE_UPLOAD=0 for 8
    if (const char* e = std::getenv("SAHARA_NIBBLE_UPLOAD")) c->nibbleUpload = std::atoi(e) != 0;
    U.bits = !c->nibbleUpload ? 8u : (c->I.sigma == 5 || c->I.sigma == 6) ? 2u : 4u;
    if (const char* e = std::getenv("SAHARA_UPLOAD_BITS")) {
        const int b = std::atoi(e);
        if (b == 2 || b == 4 || b == 8) U.bits = (uint32_t)b;
    }
    if (U.bits == 2 && c->I.sigma != 5 && c->I.sigma != 6) U.bits = 4;
    // 1M patterns per chunk (SAHARA_UPLOAD_CHUNK), at most one ring slot of nibbles
    uint64_t chunkPats = 1u << 20;
    if (const char* e = std::getenv("SAHARA_UPLOAD_CHUNK")) chunkPats = std::max<uint64_t>(2, std::atoll(e));
    uint64_t chunk = rc ? chunkPats / 2 : chunkPats;
    if (U.bits != 8) chunk = std::min<uint64_t>(chunk, Ctx::kRingSlot * 2 / m);
    U.chunk = std::max<uint64_t>(2, chunk & ~uint64_t(1));
    if (c->ringInit.joinable()) c->ringInit.join();
    if (U.bits != 8 && !c->ring) throw Error("could not pin the upload ring buffer");
    for (hipEvent_t e : c->ringEv) SH_HIP(hipEventSynchronize(e));  // the last call's DMAs
    if (U.bits != 8) c->nibPats.reserve((rows * m + 1) / 2 + 16);  // + the 12 B the 2-bit packer's last loads may touch
    SH_HIP(hipMemsetAsync(c->badFlag.ptr, 0, sizeof(uint32_t), c->stE));
    c->stageMs = 0;
    c->staged = c->streaming = true;
}

void stage(Ctx* c, const uint8_t* ranks, uint64_t npat, uint32_t m, const uint32_t* pi, const uint32_t* l,
           const uint32_t* u, uint32_t ns, int edit) {
    if (npat == 0) throw Error("no patterns");
    c->staged = c->streaming = false;
    std::vector<uint32_t> packed, cover;
    packSchemeTable(pi, l, u, ns, m, packed, c->maxErr);
    if ((size_t)ns * m * 4 > 60 * 1024) throw Error("scheme too large for LDS (searches * len > 15360)");
    if (ns > 255) throw Error("at most 255 searches per scheme");
    const auto t0 = std::chrono::steady_clock::now();
    textTable(pi, l, u, ns, m, packed, cover);
    c->patWords = (m + 7) / 8;
    {
        DevBuf<uint8_t>& raw = c->rawPats;  // kept: no 2 GB allocate / free per call at C3
        raw.reserve(npat * m);
        if (!stageIn(c, raw.ptr, ranks, npat * m)) {
            c->staged = false;
            throw Error("pattern rank out of range for this index");
        }
        c->pats.reserve(npat * c->patWords + 4);  // + tail words read by paired loads
        SH_HIP(hipMemsetAsync(c->small.ptr, 0, sizeof(uint32_t), c->st));
        launchPackPatterns(raw.ptr, npat, m, c->patWords, c->I.sigma, c->pats.ptr, c->small.ptr, c->st);
        c->patBlocks = (m + 31) / 32;
        c->pats3.reserve(npat * c->patBlocks);
        launchPackPatterns3(raw.ptr, npat, m, c->patBlocks, c->pats3.ptr, c->st);
        uint32_t bad = 0;
        SH_HIP(hipMemcpyAsync(&bad, c->small.ptr, sizeof(uint32_t), hipMemcpyDeviceToHost, c->st));
        SH_HIP(hipStreamSynchronize(c->st));
        if (bad) {
            c->staged = false;
            throw Error("pattern rank out of range for this index");
        }
    }
    c->scheme.reserve(packed.size());
    SH_HIP(hipMemcpyAsync(c->scheme.ptr, packed.data(), packed.size() * 4, hipMemcpyHostToDevice, c->st));
    c->cover.reserve(cover.size());
    SH_HIP(hipMemcpyAsync(c->cover.ptr, cover.data(), cover.size() * 4, hipMemcpyHostToDevice, c->st));
    // searches whose first kmerK steps admit no error start from the k-mer table
    std::vector<uint32_t> kst(ns, 0xFFFFFFFFu);
    const uint32_t K = c->I.kmerK;
    for (uint32_t s = 0; K && K <= m && s < ns; ++s) {
        bool exact = true;
        uint32_t lo = pi[(size_t)s * m];
        for (uint32_t p = 0; p < K; ++p) {
            exact = exact && u[(size_t)s * m + p] == 0;
            lo = std::min(lo, pi[(size_t)s * m + p]);
        }
        if (exact) kst[s] = lo;
    }
    c->kmerStart.reserve(ns);
    SH_HIP(hipMemcpyAsync(c->kmerStart.ptr, kst.data(), ns * 4, hipMemcpyHostToDevice, c->st));
    SH_HIP(hipStreamSynchronize(c->st));
    c->npat = npat;
    c->m = m;
    c->nsearch = ns;
    c->edit = edit != 0;
    c->staged = true;
    c->stageMs = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}


// One pass over the staged patterns in batches of <= 4M. Per batch:
//   stream st : kSeedItems, kSearchFM        -> hits, tasks of its slot
//   stream stB: kResolveTasks, kSearchText   -> hits of its slot
//   stream stC: row offsets, locate, sort, decode
// Three slots rotate, so the FM phase of batches i+1, i+2 (memory-latency
// bound) overlaps the text phase of batch i (ALU bound), and both phases run
// back to back while locate and sort of batch i-1 fill the gaps on stream
// stC. Host order: finish(i-3), FM(i), text(i) — FM(i) reuses the slot that
// locate(i-3) frees. Buffer overflow is detected
// after the fact from each batch's flags; the whole pass is then redone on one
// stream with grown buffers (`serial`), re-running a batch until it fits.
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
                  &sahara_stats::text_steps, &sahara_stats::text_launches})
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
        sortHitsByQid(c->outAll.ptr, total, c->out.ptr, c->tmp, c->st);
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

void growCap(uint32_t& cap, uint32_t seen) {
    const uint64_t want = (uint64_t)seen + seen / 4 + 1024;
    if (want >= (1ull << 32) - 2) throw Error("a work buffer would exceed 2^32 entries in one batch");
    cap = std::max<uint32_t>(cap, (uint32_t)want);
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
    // (memory-latency bound) runs two workgroups per CU beside three text
    // workgroups; alone it takes all that fit. (Measured at C3 with pruned
    // text steps: text 3 + FM 2 846-873M reads/s, text 4 + FM 1 845-847M.)
    // patterns per batch: 4M, fewer for schemes with many searches (work
    // items must fit 2^31); SAHARA_BATCH lowers it (tests of the pipeline)
    uint64_t maxBatch = std::min<uint64_t>(1ull << 22, (1ull << 31) / c->nsearch);
    if (const char* e = std::getenv("SAHARA_BATCH"))
        maxBatch = std::max<uint64_t>(1, std::min<uint64_t>((1ull << 31) / c->nsearch, std::atoll(e)));
    const uint64_t batchesHere = (c->npat + maxBatch - 1) / maxBatch;
    if (!serial && batchesHere > 1 && c->verify) bpc = 2;
    if (const char* e = std::getenv("SAHARA_FM_BPC")) bpc = std::max(1, std::min(searchBlocksPerCU(sigma, c->edit, lds), std::atoi(e)));
    const uint32_t blocks = (uint32_t)(c->numCU * bpc);
    // the first batch's FM phase has nothing to overlap with: full occupancy
    const uint32_t firstBlocks = std::getenv("SAHARA_FM_BPC") ? blocks : (uint32_t)(c->numCU * fullBpc);
    const uint64_t T = (uint64_t)std::max(blocks, firstBlocks) * 256;
    const uint32_t stackCap = std::max<uint32_t>(c->maxErr, 1) * (2 * sigma - 2) + 2;
    c->stack.reserve((size_t)std::max<uint32_t>(stackCap, 5) * T);  // levels beyond the LDS part
    S.search_grid = blocks;

    // text phase geometry (LDS per lane: window | pattern | stack)
    // window: |t| + what both sides can still consume <= m + 2k symbols, plus
    // the block alignment of its start (31 symbols); 3 words per block
    // (exact start: m + 2k symbols in whole blocks, copied funnel-shifted from
    // one block more; SAHARA_EXACT_WINDOW=0: the block-aligned start below it)
    const char* exactEnv = std::getenv("SAHARA_EXACT_WINDOW");
    const uint32_t exactBlocks = (c->m + 2 * c->maxErr + 31) / 32;
    const bool exactWindow = (!exactEnv || std::atoi(exactEnv) != 0) && exactBlocks + 1 <= 8 && c->patBlocks <= 8;
    const uint32_t winBlocks = exactWindow ? exactBlocks : (c->m + 2 * c->maxErr + 31 + 31) / 32;
    const uint32_t textStack = 2 * c->maxErr + 2;
    // one-word stack entries where a node fits 30 bits (search.hip packNode)
    // (SAHARA_PACKED_STACK; off by default: at m = 100 it buys a fourth text
    // workgroup per CU, but costs a pack / unpack per micro-step, and three
    // workgroups leave LDS for an FM workgroup beside them)
    const bool packedStack = c->m <= 127 && winBlocks <= 7 && c->maxErr <= 7 && std::getenv("SAHARA_PACKED_STACK") &&
                             std::atoi(std::getenv("SAHARA_PACKED_STACK")) != 0;
    const uint32_t tableWords = std::max<uint32_t>(2 * c->nsearch * c->m, kTextTableMin);
    const size_t textLds = (size_t)tableWords * 4 +
                           (size_t)256 * (3 * (winBlocks + c->patBlocks) + (packedStack ? 1 : 2) * textStack) * 4;
    if (const char* e = std::getenv("SAHARA_SPLIT")) c->split = (uint32_t)std::max(0L, std::atol(e));
    if (const char* e = std::getenv("SAHARA_TEXT_STEPS")) c->textSteps = (uint32_t)std::max(1L, std::atol(e));
    if (const char* e = std::getenv("SAHARA_REFILL_AT")) c->refillAt = (uint32_t)std::min(64L, std::max(1L, std::atol(e)));
    int tbpc = 0;
    // the text phase addresses text and a batch's patterns with 32-bit buffer offsets
    const bool textFits = text3Blocks(c->I.n) * 16 <= 0xFFFFFF00ull &&
                          maxBatch * c->patBlocks * 16 <= 0xFFFFFF00ull;
    if (c->verify && c->m <= 2047 && textLds <= 160 * 1024 && textFits)
        tbpc = textBlocksPerCU(sigma, c->edit, packedStack, textLds);
    // overlapped with the FM phase, three text workgroups per CU leave room
    // for two FM workgroups beside them (the FM chain of seeds and FM launches
    // is the other critical path once the text phase prunes dead children)
    if (!serial && batchesHere > 1) tbpc = std::min(tbpc, 3);
    if (const char* e = std::getenv("SAHARA_TEXT_BPC"); e && tbpc > 0) tbpc = std::max(1, std::min(textBlocksPerCU(sigma, c->edit, packedStack, textLds), std::atoi(e)));
    const uint32_t split = tbpc > 0 ? c->split : 0u;
    // where a task's SA row becomes its text position: 2 = inside the text
    // kernel, a chunk of task records ahead (default: no pass between the FM
    // and text phases); 1 = kResolveTasks after the FM phase on its stream;
    // 0 = kResolveTasks before the text phase (SAHARA_RESOLVE)
    uint32_t fmPrio = 0;
    if (const char* e = std::getenv("SAHARA_FM_PRIO")) fmPrio = (uint32_t)std::max(0, std::min(3, std::atoi(e)));
    int resolveMode = 2;
    if (const char* e = std::getenv("SAHARA_RESOLVE")) resolveMode = std::max(0, std::min(2, std::atoi(e)));
    // (pipelined, in-kernel task resolve) the first batch's text phase starts
    // on its seed tasks while its FM phase runs (SAHARA_EARLY_TEXT=0: after it)
    const char* earlyEnv = std::getenv("SAHARA_EARLY_TEXT");
    // (only with several batches: a lone batch's FM phase runs at full
    // occupancy, and its text phase split in two measured 45M against 68M
    // reads/s at C5)
    const bool early = !serial && split && resolveMode == 2 && batchesHere > 1 &&
                       (!earlyEnv || std::atoi(earlyEnv) != 0);
    const uint32_t textBlocks = (uint32_t)(c->numCU * std::max(tbpc, 1));
    S.text_grid = split ? textBlocks : 0u;
    S.pipelined = serial ? 0u : 1u;

    if (c->hitCap == 0) {
        c->hitCap = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(1u << 20, 8 * maxBatch), 1u << 30);
        if (const char* e = std::getenv("SAHARA_HITCAP")) c->hitCap = (uint32_t)std::max(1L, std::atol(e));
    }
    if (c->taskCap == 0) {
        c->taskCap = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(1u << 20, 8 * maxBatch), 1u << 30);
        if (const char* e = std::getenv("SAHARA_TASKCAP")) c->taskCap = (uint32_t)std::max(1L, std::atol(e));
    }
    // batch boundaries. SAHARA_RAMP (pipelined only): 1 makes the first two
    // batches smaller (1/4, 1/2 of the others) so that the FM phase of the
    // first, which overlaps nothing, is short; 2 also the last two
    std::vector<uint64_t> bstart{0};
    {
        const int rampMode = std::getenv("SAHARA_RAMP") ? std::atoi(std::getenv("SAHARA_RAMP")) : 0;
        const bool up = !serial && rampMode >= 1 && c->npat > 3 * maxBatch;
        const bool down = up && rampMode >= 2;
        const uint64_t edge[2] = {std::max<uint64_t>(maxBatch / 4, 1), std::max<uint64_t>(maxBatch / 2, 1)};
        const uint64_t mid = c->npat - (up ? edge[0] + edge[1] : 0) - (down ? edge[0] + edge[1] : 0);
        if (up) {
            bstart.push_back(edge[0]);
            bstart.push_back(edge[0] + edge[1]);
        }
        const uint64_t nmid = (mid + maxBatch - 1) / maxBatch, q0 = bstart.back();
        for (uint64_t i = 1; i <= nmid; ++i) bstart.push_back(q0 + mid * i / nmid);
        if (down) {
            bstart.push_back(bstart.back() + edge[1]);
            bstart.push_back(bstart.back() + edge[0]);
        }
    }
    const uint64_t nbatch = bstart.size() - 1;
    if (c->pinnedCap < nbatch * 8) {
        if (c->pinned) SH_HIP(hipHostFree(c->pinned));
        c->pinned = nullptr;
        SH_HIP(hipHostMalloc(&c->pinned, nbatch * 8 * sizeof(uint32_t)));
        c->pinnedCap = nbatch * 8;
    }
    if (c->qcnt.cap < maxBatch + 1) {
        c->qcnt.reserve(maxBatch + 1);
        c->qoff.reserve(maxBatch + 1);
        c->big.reserve(maxBatch);
    }
    SH_HIP(hipMemsetAsync(c->qcnt.ptr, 0, (maxBatch + 1) * sizeof(uint32_t), c->st));
    hipStream_t sA = c->st, sB = serial ? c->st : c->stB, sC = serial ? c->st : c->stC, sD = serial ? c->st : c->stD;
    SH_HIP(hipStreamSynchronize(c->st));
    SH_HIP(hipStreamSynchronize(c->stB));
    SH_HIP(hipStreamSynchronize(c->stC));
    SH_HIP(hipStreamSynchronize(c->stD));
    if (count) SH_HIP(hipMemsetAsync(c->counters.ptr, 0, 16 * sizeof(unsigned long long), sA));
    c->nout = 0;
    c->sinkDone = 0;
    c->sinkOk = c->sink != nullptr;
    // a slot's counters and queues are zero when its `free` event fires:
    // here for the first use, after its locate (finish) for the next
    auto resetSlot = [&](Ctx::Slot& sl, hipStream_t s) {
        SH_HIP(hipMemsetAsync(sl.small.ptr, 0, 8 * sizeof(uint32_t), s));
        SH_HIP(hipMemsetAsync(sl.queues.ptr, 0, 768 * sizeof(uint32_t), s));
        SH_HIP(hipEventRecord(sl.free, s));
    };
    for (auto& sl : c->slot) resetSlot(sl, sA);

    auto issueFM = [&](uint64_t b) {
        Ctx::Slot& sl = c->slot[b % Ctx::kSlots];
        const uint64_t q0 = bstart[b], nb = bstart[b + 1] - q0;
        sl.hits.reserve((size_t)c->hitCap + 1);
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
        a.hits = sl.hits.ptr;
        a.hitCap = c->hitCap;
        a.counters = c->counters.ptr;
        a.tasks = sl.tasks.ptr;
        a.taskCap = c->taskCap;
        a.split = split;
        a.ldsDepth = fmLdsDepth;
        a.prio = serial ? 0u : fmPrio;
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
        ensureUploaded(c, bstart[b + 1], sD);
        SH_HIP(hipEventRecord(sl.fmStart, sD));
        launchSeeds(sd, sigma, std::min<uint32_t>((a.nitems + 1023) / 1024, (uint32_t)c->numCU * 8), sD);
        if (early && b == 0)  // the seed tasks end here: the text phase may start on them
            SH_HIP(hipMemcpyAsync(sl.small.ptr + 5, sl.small.ptr + 4, 4, hipMemcpyDeviceToDevice, sD));
        SH_HIP(hipEventRecord(sl.seedDone, sD));
        SH_HIP(hipStreamWaitEvent(sA, sl.seedDone, 0));
        launchSearch(a, sigma, c->edit, count, b == 0 && !early ? firstBlocks : blocks, lds, sA);
        if (split && resolveMode == 1)
            launchResolveTasks(sl.tasks.ptr, sl.small.ptr + 4, c->taskCap, c->I.saFull.ptr, c->numCU * 8, sA);
        SH_HIP(hipEventRecord(sl.fmDone, sA));
        ++S.search_launches;
    };
    auto issueText = [&](uint64_t b) {
        Ctx::Slot& sl = c->slot[b % Ctx::kSlots];
        const uint64_t q0 = bstart[b];
        const bool split0 = early && b == 0;
        SH_HIP(hipStreamWaitEvent(sB, split0 ? sl.seedDone : sl.fmDone, 0));
        SH_HIP(hipEventRecord(sl.textStart, sB));
        if (split) {
            TextArgs t{};
            t.sa = c->I.saFull.ptr;
            t.text3 = c->I.text3.ptr;
            t.pats3 = c->pats3.ptr + q0 * c->patBlocks;
            t.patBlocks = c->patBlocks;
            t.text3Bytes = (uint32_t)std::min<uint64_t>(text3Blocks(c->I.n) * 16, 0xFFFFFF00ull);
            t.pats3Bytes = (uint32_t)std::min<uint64_t>((c->npat - q0) * c->patBlocks * 16, 0xFFFFFF00ull);
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
            // (SAHARA_PRUNE=0 turns it off; C3: 43 -> 28 micro-steps per read,
            // C5: 439 -> 303 and 68M -> 82M reads/s)
            const char* pruneEnv = std::getenv("SAHARA_PRUNE");
            t.prune = !pruneEnv || std::atoi(pruneEnv) != 0 ? 1u : 0u;
            t.stackCap = textStack;
            t.packedStack = packedStack ? 1u : 0u;
            t.tableWords = tableWords;
            t.resolveRows = resolveMode == 2 ? 1u : 0u;
            t.steps = c->textSteps;
            t.refillAt = c->refillAt;
            if (resolveMode == 0)
                launchResolveTasks(sl.tasks.ptr, sl.small.ptr + 4, c->taskCap, c->I.saFull.ptr, c->numCU * 8, sB);
            if (split0) {
                // the first batch's seed tasks while its FM phase runs, then the
                // tasks the FM phase appended after them
                t.taskCount = sl.small.ptr + 5;
                launchText(t, sigma, c->edit, count, textBlocks, textLds, sB);
                SH_HIP(hipStreamWaitEvent(sB, sl.fmDone, 0));
                t.taskBegin = sl.small.ptr + 5;
                t.taskCount = sl.small.ptr + 4;
                t.work = sl.queues.ptr + 512;
                ++S.text_launches;
            }
            launchText(t, sigma, c->edit, count, textBlocks, textLds, sB);
            ++S.text_launches;
        }
        SH_HIP(hipEventRecord(sl.textDone, sB));
    };
    // locate: row offsets (exclusive scan of len), SA / LF locate, canonical
    // sort, decode into the device-resident output, on stream sC. Needs the
    // batch's counts (host waits for its text phase). Returns false on
    // overflow; `finishCheck` then reads the locate flags and timings.
    uint32_t seenTask = 0, seenHit = 0;  // pipelined overflow: the caps the re-run needs
    auto finish = [&](uint64_t b) {
        Ctx::Slot& sl = c->slot[b % Ctx::kSlots];
        const uint64_t q0 = bstart[b], nb = bstart[b + 1] - q0;
        c->mark("finish", b);
        // the batch's counters, copied on sC (a copy on sB would wait for CU
        // slots between two text phases)
        SH_HIP(hipStreamWaitEvent(sC, sl.textDone, 0));
        SH_HIP(hipMemcpyAsync(c->pinned + b * 8, sl.small.ptr, 8 * sizeof(uint32_t), hipMemcpyDeviceToHost, sC));
        SH_HIP(hipEventRecord(c->ev[6], sC));
        SH_HIP(hipEventSynchronize(c->ev[6]));
        c->mark("text done", b);
        const uint32_t* hs = c->pinned + b * 8;
        float ms = 0;
        SH_HIP(hipEventElapsedTime(&ms, sl.fmStart, sl.seedDone));
        S.seed_ms += ms;
        SH_HIP(hipEventElapsedTime(&ms, sl.seedDone, sl.fmDone));
        S.search_ms += ms;
        SH_HIP(hipEventElapsedTime(&ms, sl.textStart, sl.textDone));
        S.text_ms += ms;
        if (hs[2] & 1u) throw Error("search stack overflow (internal bound violated)");
        if (hs[2] & 16u) throw Error("text phase: internal stack bound violated");
        if (hs[2] & (2u | 8u)) {  // hit or task buffer too small
            // (pipelined: issueFM may be reading the caps on the other host
            // thread; they grow after the pass, before the serial re-run)
            if (hs[2] & 8u) growCap(serial ? c->taskCap : seenTask, hs[4]);
            if (hs[2] & 2u) growCap(serial ? c->hitCap : seenHit, hs[1]);
            overflow = true;
            resetSlot(sl, sC);
            return false;
        }
        // reserved slots incl. len-0 holes; a wave's last range may reach past
        // the capacity without having written there (no overflow flag)
        const uint64_t nh = std::min<uint64_t>(hs[1], c->hitCap);
        S.cursors += hs[3];
        SH_HIP(hipEventRecord(c->ev[2], sC));
        SH_HIP(hipMemsetAsync(c->small.ptr, 0, 8 * sizeof(uint32_t), sC));
        c->partial.reserve(scanTiles((uint32_t)nb));
        querySegments(sl.hits.ptr, nh, c->qcnt.ptr, (uint32_t)nb, c->qoff.ptr, c->partial.ptr, c->big.ptr,
                      c->small.ptr + 4, sC);
        uint64_t rows = 0;
        uint32_t nbig = 0;
        SH_HIP(hipMemcpyAsync(&rows, c->qoff.ptr + nb, 8, hipMemcpyDeviceToHost, sC));
        SH_HIP(hipMemcpyAsync(&nbig, c->small.ptr + 4, 4, hipMemcpyDeviceToHost, sC));
        SH_HIP(hipStreamSynchronize(sC));
        c->mark("rows", b);
        if (rows >= (1ull << 32)) throw Error("more than 2^32 located hits in one batch of patterns");
        c->k0.reserve(std::max<uint64_t>(rows, 1));
        if (nbig) c->k1.reserve(std::max<uint64_t>(rows, 1));
        LocateArgs la{};
        la.hits = sl.hits.ptr;
        la.nhits = nh;
        la.qoff = c->qoff.ptr;
        la.qcnt = c->qcnt.ptr;
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
        if (nbig) c->tmp.reserve(bigSortTempBytes(rows, nbig) + 256);
        if (c->nout + rows > c->out.cap) {  // grow the device-resident output
            const size_t want = std::max<size_t>((c->nout + rows) + (c->nout + rows) / 2, 1024);
            sahara_hit* np = nullptr;
            SH_HIP(hipMalloc(&np, want * sizeof(sahara_hit)));
            if (c->nout) SH_HIP(hipMemcpyAsync(np, c->out.ptr, c->nout * sizeof(sahara_hit), hipMemcpyDeviceToDevice, sC));
            SH_HIP(hipStreamSynchronize(sC));
            SH_HIP(hipStreamSynchronize(c->stF));  // sink copies may still read the old buffer
            c->out.release();
            c->out.ptr = np;
            c->out.cap = want;
        }
        sortDecode(c->k0.ptr, c->k1.ptr, rows, c->qoff.ptr, (uint32_t)nb, c->big.ptr, nbig, q0, c->I.dRecStarts.ptr,
                   (uint32_t)c->I.recStarts.size(), c->out.ptr + c->nout, c->tmp.ptr, c->tmp.cap, sC);
        SH_HIP(hipEventRecord(c->ev[4], sC));
        // sahara_gpu_search's host sink: the batch's hits go to host memory
        // on stF while later batches search (while they fit the sink)
        if (c->sinkOk && c->nout + rows <= c->sinkCap) {
            const bool compact = c->compactSink && rows * sizeof(uint64_t) <= Ctx::kDownSlot && nb < (1ull << 28);
            if (rows && compact) {  // 8-B records, expanded on the host (Expander)
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
        SH_HIP(hipMemcpyAsync(c->pinned + b * 8 + 7, c->small.ptr + 2, 4, hipMemcpyDeviceToHost, sC));
        SH_HIP(hipEventRecord(c->ev[5], sC));
        c->nout += rows;
        S.hits += rows;
        return true;
    };
    auto finishCheck = [&](uint64_t b) {
        SH_HIP(hipEventSynchronize(c->ev[5]));
        if (c->pinned[b * 8 + 7] & 4u) throw Error("locate walked off the SA samples (corrupt index)");
        float ms = 0;
        SH_HIP(hipEventElapsedTime(&ms, c->ev[2], c->ev[3]));
        S.locate_ms += ms;
        SH_HIP(hipEventElapsedTime(&ms, c->ev[3], c->ev[4]));
        S.sort_ms += ms;
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
        if (issueErr) std::rethrow_exception(issueErr);
        if (finErr) std::rethrow_exception(finErr);
        if (overflow) {
            c->taskCap = std::max(c->taskCap, seenTask);
            c->hitCap = std::max(c->hitCap, seenHit);
        }
        SH_HIP(hipStreamSynchronize(sA));
        SH_HIP(hipStreamSynchronize(sB));
        SH_HIP(hipStreamSynchronize(sC));
        SH_HIP(hipStreamSynchronize(sD));
        SH_HIP(hipStreamSynchronize(c->stF));
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
    if (count) {
        unsigned long long h[16];
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
    }
}

}  // namespace

extern "C" {

const char* sahara_gpu_last_error(void) { return g_err.c_str(); }

int sahara_gpu_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int sahara_gpu_build(int device, const uint8_t* ranks, const uint64_t* rec_lens, uint64_t n_records, uint32_t sigma,
                     uint32_t sampling_rate, void** ctx) {
    return guarded([&] {
        std::unique_ptr<Ctx> c(newCtx(device));
        const std::vector<uint64_t> first = splitRecords(rec_lens, n_records);
        if (first.size() == 2) {
            buildFromText(c->I, ranks, rec_lens, n_records, sigma, sampling_rate, c->st);
        } else {  // parts at record boundaries, then their k-mer tables at one common depth
            uint64_t off = 0, nmax = 0;
            for (size_t p = 0; p + 1 < first.size(); ++p) {
                uint64_t syms = 0, n = 0;
                for (uint64_t r = first[p]; r < first[p + 1]; ++r) syms += rec_lens[r];
                n = syms + (first[p + 1] - first[p]);
                nmax = std::max(nmax, n);
                if (p) c->more.emplace_back();
                buildFromText(partOf(c.get(), (uint32_t)p), ranks + off, rec_lens + first[p], first[p + 1] - first[p],
                              sigma, sampling_rate, c->st, false);
                off += syms;
            }
            c->partRec0.assign(first.begin(), first.end() - 1);
            const uint32_t K = kmerDepth(nmax, (uint32_t)first.size() - 1);
            for (uint32_t p = 0; p + 1 < first.size(); ++p) buildKmerTable(partOf(c.get(), p), K, c->st);
        }
        *ctx = c.release();
    });
}

// an .idx image (one part or several) -> a context holding every part
Ctx* openImage(int device, const uint8_t* buf, size_t bytes) {
    const std::vector<IdxParts> parts = parseIdxAll(buf, bytes);
    std::unique_ptr<Ctx> c(newCtx(device));
    uint64_t rec0 = 0, nmax = 0;
    c->partRec0.clear();
    for (size_t p = 0; p < parts.size(); ++p) {
        const IdxParts& P = parts[p];
        if (p) c->more.emplace_back();
        buildFromParts(partOf(c.get(), (uint32_t)p), P.sigma, P.n, P.recLens.data(), P.recLens.size(), P.rate, P.bwtF,
                       P.bwtR, P.sampled, P.samples, P.nsamples, c->st, parts.size() == 1);
        c->partRec0.push_back(rec0);
        rec0 += P.recLens.size();
        nmax = std::max(nmax, P.n);
    }
    if (parts.size() > 1) {
        const uint32_t K = kmerDepth(nmax, (uint32_t)parts.size());
        for (uint32_t p = 0; p < parts.size(); ++p) buildKmerTable(partOf(c.get(), p), K, c->st);
    }
    return c.release();
}

int sahara_gpu_open(int device, const void* idx_image, size_t idx_bytes, void** ctx) {
    return guarded([&] { *ctx = openImage(device, static_cast<const uint8_t*>(idx_image), idx_bytes); });
}

int sahara_gpu_open_file(int device, const char* path, void** ctx) {
    return guarded([&] {
        std::vector<uint8_t> buf = readFile(path);
        *ctx = openImage(device, buf.data(), buf.size());
    });
}

int sahara_gpu_index_info(void* ctx, sahara_index_info* info) {
    return guarded([&] {
        Ctx* c = ctxOf(ctx);
        info->sigma = c->I.sigma;
        info->sampling_rate = c->I.rate;
        info->n = info->n_records = info->n_samples = info->device_bytes = 0;
        for (uint32_t p = 0; p <= c->more.size(); ++p) {  // totals over the parts
            const DeviceIndex& D = partOf(c, p);
            info->n += D.n;
            info->n_records += D.recLens.size();
            info->n_samples += D.nsamples;
            info->device_bytes += D.deviceBytes();
        }
        info->n_parts = (uint32_t)c->more.size() + 1;
        info->kmer_depth = c->I.kmerK;
    });
}

int sahara_gpu_export(void* ctx, uint8_t* bwt_f, uint8_t* bwt_r, uint64_t* sampled_bits, uint32_t* samples,
                      uint64_t* C, uint64_t* rec_lens) {
    return guarded([&] {
        Ctx* c = ctxOf(ctx);
        DeviceIndex& D = partOf(c, c->exportPart);
        exportParts(D, bwt_f, bwt_r, sampled_bits, samples, c->st);
        if (C) std::memcpy(C, D.C, (D.sigma + 1) * 8);
        if (rec_lens) std::memcpy(rec_lens, D.recLens.data(), D.recLens.size() * 8);
    });
}

int sahara_gpu_export_sa(void* ctx, uint32_t* sa) {
    return guarded([&] {
        const DeviceIndex& D = partOf(ctxOf(ctx), ctxOf(ctx)->exportPart);
        SH_HIP(hipMemcpy(sa, D.saFull.ptr, D.n * 4, hipMemcpyDeviceToHost));
    });
}

int sahara_gpu_export_text(void* ctx, uint8_t* text) {
    return guarded([&] {
        const DeviceIndex& D = partOf(ctxOf(ctx), ctxOf(ctx)->exportPart);
        std::vector<uint32_t> t3(((D.n + 31) / 32) * 4);
        SH_HIP(hipMemcpy(t3.data(), D.text3.ptr, t3.size() * 4, hipMemcpyDeviceToHost));
        for (uint64_t i = 0; i < D.n; ++i) {
            const uint32_t* b = &t3[(i / 32) * 4];
            const uint32_t j = (uint32_t)(i & 31);
            text[i] = (uint8_t)(((b[0] >> j) & 1u) | (((b[1] >> j) & 1u) << 1) | (((b[2] >> j) & 1u) << 2));
        }
    });
}

int sahara_gpu_part_info(void* ctx, uint32_t part, sahara_index_info* info) {
    return guarded([&] {
        Ctx* c = ctxOf(ctx);
        if (part > c->more.size()) throw Error("no index part " + std::to_string(part));
        const DeviceIndex& D = partOf(c, part);
        info->sigma = D.sigma;
        info->sampling_rate = D.rate;
        info->n = D.n;
        info->n_records = D.recLens.size();
        info->n_samples = D.nsamples;
        info->device_bytes = D.deviceBytes();
        info->n_parts = (uint32_t)c->more.size() + 1;
        info->kmer_depth = D.kmerK;
    });
}

int sahara_gpu_select_part(void* ctx, uint32_t part) {
    return guarded([&] {
        Ctx* c = ctxOf(ctx);
        if (part > c->more.size()) throw Error("no index part " + std::to_string(part));
        c->exportPart = part;
    });
}

int sahara_gpu_set_mode(void* ctx, int verify, int locate_sa) {
    return guarded([&] {
        Ctx* c = ctxOf(ctx);
        c->verify = verify != 0;
        c->locateSA = locate_sa != 0;
    });
}

int sahara_gpu_save(void* ctx, const char* path) {
    return guarded([&] {
        Ctx* c = ctxOf(ctx);
        const size_t np = c->more.size() + 1;
        std::vector<std::vector<uint8_t>> bf(np), br(np);
        std::vector<std::vector<uint64_t>> sb(np);
        std::vector<std::vector<uint32_t>> smp(np);
        std::vector<IdxParts> parts(np);
        for (uint32_t p = 0; p < np; ++p) {
            const DeviceIndex& D = partOf(c, p);
            const uint64_t n = D.n;
            bf[p].resize(n);
            br[p].resize(n);
            sb[p].resize(n / 64 + 1);
            smp[p].resize(D.nsamples);
            exportParts(D, bf[p].data(), br[p].data(), sb[p].data(), smp[p].data(), c->st);
            IdxParts& P = parts[p];
            P.sigma = D.sigma;
            P.n = n;
            P.rate = D.rate;
            std::copy(D.C, D.C + 8, P.C);
            P.recLens = D.recLens;
            P.bwtF = bf[p].data();
            P.bwtR = br[p].data();
            P.sampled = sb[p].data();
            P.samples = smp[p].data();
            P.nsamples = smp[p].size();
        }
        writeIdxAll(path, parts);
    });
}

int sahara_gpu_stage(void* ctx, const uint8_t* ranks, uint64_t n_patterns, uint32_t len, const uint32_t* pi,
                     const uint32_t* l, const uint32_t* u, uint32_t n_searches, int edit) {
    return guarded([&] { stage(ctxOf(ctx), ranks, n_patterns, len, pi, l, u, n_searches, edit); });
}

int sahara_gpu_run(void* ctx, int count, uint64_t* n_hits) {
    return guarded([&] {
        Ctx* c = ctxOf(ctx);
        run(c, count != 0);
        if (n_hits) *n_hits = c->nout;
    });
}

int sahara_gpu_fetch(void* ctx, sahara_hit* out, uint64_t capacity, uint64_t* n_hits) {
    return guarded([&] {
        Ctx* c = ctxOf(ctx);
        if (n_hits) *n_hits = c->nout;
        if (capacity < c->nout) throw Error("sahara_gpu_fetch: capacity too small");
        if (c->nout) SH_HIP(hipMemcpy(out, c->out.ptr, c->nout * sizeof(sahara_hit), hipMemcpyDeviceToHost));
    });
}

int sahara_gpu_copy_hits(void* ctx, void* dst_device, uint64_t capacity, uint64_t qid_offset, uint64_t* n_hits) {
    return guarded([&] {
        Ctx* c = ctxOf(ctx);
        if (n_hits) *n_hits = c->nout;
        if (capacity < c->nout) throw Error("sahara_gpu_copy_hits: capacity too small");
        if (c->nout && !dst_device) throw Error("sahara_gpu_copy_hits: null destination");
        launchCopyHits(c->out.ptr, c->nout, qid_offset, static_cast<sahara_hit*>(dst_device), c->st);
        SH_HIP(hipStreamSynchronize(c->st));
    });
}

int sahara_gpu_digest(void* ctx, uint64_t* digest) {
    return guarded([&] {
        Ctx* c = ctxOf(ctx);
        SH_HIP(hipMemsetAsync(c->counters.ptr + 4, 0, 8, c->st));
        launchDigest(c->out.ptr, c->nout, c->counters.ptr + 4, c->st);
        unsigned long long d = 0;
        SH_HIP(hipMemcpyAsync(&d, c->counters.ptr + 4, 8, hipMemcpyDeviceToHost, c->st));
        SH_HIP(hipStreamSynchronize(c->st));
        *digest = d;
    });
}

int sahara_gpu_stats(void* ctx, sahara_stats* stats) {
    return guarded([&] { *stats = ctxOf(ctx)->stats; });
}

// Hit buffers handed to the caller. Buffers of >= 64 MB are page-locked
// (hipHostMalloc), so the device-to-host copy runs at the link's rate straight
// into them, and sahara_gpu_free hands them back to a small pool instead of
// unpinning them: pinning (and first-touching) 0.6 GB costs more than copying
// into it, and a fresh box without transparent huge pages paid 28.6 ms for
// the page faults of a pageable buffer against 13 ms for the copy.
struct HitPool {
    std::mutex mu;
    std::unordered_map<void*, size_t> live;       // pinned buffers the callers hold
    std::vector<std::pair<void*, size_t>> idle;   // pinned buffers ready for reuse
    static constexpr size_t kKeep = 2;
};
static HitPool& hitPool() {
    static HitPool* p = new HitPool;  // never destroyed: callers may free after static destructors ran
    return *p;
}

// Host buffer for n hits (released with sahara_gpu_free); *pinned tells
// whether the device can copy into it directly.
static void* allocHits(uint64_t n, bool* pinned, uint64_t* capHits = nullptr, bool mayPin = true) {
    const size_t bytes = std::max<uint64_t>(n, 1) * sizeof(sahara_hit);
    *pinned = false;
    if (capHits) *capHits = std::max<uint64_t>(n, 1);
    size_t pinMin = 64u << 20;  // SAHARA_PIN_MIN: smallest pinned buffer in bytes (tests pin every size)
    if (const char* e = std::getenv("SAHARA_PIN_MIN")) pinMin = (size_t)std::atoll(e);
    if (bytes < pinMin) return std::malloc(bytes);
    HitPool& P = hitPool();
    std::vector<void*> unpin;
    void* p = nullptr;
    {
        std::lock_guard<std::mutex> g(P.mu);
        size_t best = SIZE_MAX;
        for (size_t i = 0; i < P.idle.size(); ++i)
            if (P.idle[i].second >= bytes && (best == SIZE_MAX || P.idle[i].second < P.idle[best].second)) best = i;
        if (best != SIZE_MAX) {
            p = P.idle[best].first;
            P.live[p] = P.idle[best].second;
            if (capHits) *capHits = P.idle[best].second / sizeof(sahara_hit);
            P.idle.erase(P.idle.begin() + (long)best);
        } else {  // none fits: the smaller idle ones will not fit later calls of this size either
            for (auto& e : P.idle) unpin.push_back(e.first);
            P.idle.clear();
        }
    }
    for (void* q : unpin) (void)hipHostFree(q);
    if (p) {
        *pinned = true;
        return p;
    }
    if (!mayPin) return std::malloc(bytes);  // a one-off caller: pinning would cost more than it saves
    const size_t huge = 2u << 20, cap = (bytes + bytes / 8 + huge - 1) / huge * huge;  // room for a run with more hits
    if (hipHostMalloc(&p, cap, hipHostMallocPortable) == hipSuccess && p) {
        std::lock_guard<std::mutex> g(P.mu);
        P.live[p] = cap;
        *pinned = true;
        if (capHits) *capHits = cap / sizeof(sahara_hit);
        return p;
    }
    (void)hipGetLastError();
    p = std::aligned_alloc(huge, (bytes + huge - 1) / huge * huge);  // pageable fallback
    if (p) (void)madvise(p, (bytes + huge - 1) / huge * huge, MADV_HUGEPAGE);
    return p;
}

static void freeHits(void* p) {
    if (!p) return;
    HitPool& P = hitPool();
    void* drop = nullptr;
    {
        std::lock_guard<std::mutex> g(P.mu);
        auto it = P.live.find(p);
        if (it == P.live.end()) {
            std::free(p);
            return;
        }
        P.idle.emplace_back(p, it->second);
        P.live.erase(it);
        if (P.idle.size() > HitPool::kKeep) {
            drop = P.idle.front().first;
            P.idle.erase(P.idle.begin());
        }
    }
    if (drop) (void)hipHostFree(drop);
}

// memcpy from several threads (host copies out of the pinned staging chunks)
static void parallelCopy(void* dst, const void* src, size_t bytes) {
    const unsigned nt = std::max(1u, std::min(8u, std::thread::hardware_concurrency()));
    if (bytes < (4u << 20) || nt == 1) {
        std::memcpy(dst, src, bytes);
        return;
    }
    std::vector<std::thread> ts;
    const size_t per = (bytes / nt + 4095) & ~size_t(4095);
    for (unsigned i = 0; i < nt; ++i) {
        const size_t b = i * per, e = std::min(bytes, b + per);
        if (b >= e) break;
        ts.emplace_back([=] { std::memcpy(static_cast<char*>(dst) + b, static_cast<const char*>(src) + b, e - b); });
    }
    for (auto& t : ts) t.join();
}

// Device hits -> pageable host memory through two pinned chunks: chunk k's
// DMA runs while the host copies chunk k-1 out (a direct copy to pageable
// memory runs at ~10 GB/s).
static void copyOut(Ctx* c, void* dst, const void* src, size_t bytes) {
    if (bytes < (8u << 20)) {
        SH_HIP(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
        return;
    }
    for (void*& p : c->outStage)
        if (!p) SH_HIP(hipHostMalloc(&p, Ctx::kOutChunk));
    const size_t n = (bytes + Ctx::kOutChunk - 1) / Ctx::kOutChunk;
    auto len = [&](size_t k) { return std::min(Ctx::kOutChunk, bytes - k * Ctx::kOutChunk); };
    for (size_t k = 0; k <= n; ++k) {
        if (k < n) {
            SH_HIP(hipMemcpyAsync(c->outStage[k & 1], static_cast<const char*>(src) + k * Ctx::kOutChunk, len(k),
                                  hipMemcpyDeviceToHost, c->st));
            SH_HIP(hipEventRecord(c->ev[k & 1], c->st));
        }
        if (k > 0) {
            SH_HIP(hipEventSynchronize(c->ev[(k - 1) & 1]));
            parallelCopy(static_cast<char*>(dst) + (k - 1) * Ctx::kOutChunk, c->outStage[(k - 1) & 1], len(k - 1));
        }
    }
}

// Waits for every stream of the context (after a failed streamed search: the
// issued batches may still run and copy into the sink).
static void drainAll(Ctx* c) {
    for (hipStream_t s : {c->st, c->stB, c->stC, c->stD, c->stE, c->stF}) (void)hipStreamSynchronize(s);
}

// sahara_gpu_search / sahara_gpu_search_reads: streamed upload, the pipelined
// pass, the hits streamed into a pinned host sink batch by batch, then handed
// to the caller (search.cpp:218-250 from host queries to host hits).
static void searchStreamed(Ctx* c, const uint8_t* src, uint64_t rows, bool rc, uint64_t npat, uint32_t len,
                           const uint32_t* pi, const uint32_t* l, const uint32_t* u, uint32_t n_searches, int edit,
                           uint32_t max_hits, sahara_hit** hits, uint64_t* n_hits) {
    using clk = std::chrono::steady_clock;
    const auto tA = clk::now();
    {
        const char* te = std::getenv("SAHARA_TIMING");
        c->traceOn = te && std::atoi(te) >= 2;
        c->traceT0 = tA;
        c->trace.clear();
    }
    stageStreamed(c, src, rows, rc, npat, len, pi, l, u, n_searches, edit);
    const auto tB = clk::now();
    c->sink = nullptr;
    c->sinkCap = 0;
    c->compactSink = c->sinkPinned = false;
    if (!max_hits) {  // sized from the last call (the bench's steady state), else 2 hits per pattern
        // a first call takes a pooled buffer if there is one, but pins none:
        // pinning ~1 GB costs ~200 ms, ten times the pageable copy-out
        const uint64_t est = c->lastHits ? c->lastHits + c->lastHits / 8 + 1024 : 2 * npat + 1024;
        bool pinned = false;
        void* p = allocHits(est, &pinned, &c->sinkCap, c->lastHits != 0);
        // hits go whole into a pinned sink (DMA; no host CPU or memory traffic
        // beyond the write), or, into pageable memory, as 8-B records that
        // host threads expand (Expander): a third of the PCIe bytes, but the
        // expansion reads and writes host memory the packing also needs
        // (at C3 it took ~4 ms per batch beside the packing, 300M against
        // 330M reads/s). SAHARA_COMPACT_DOWNLOAD=1 / SAHARA_FULL_DOWNLOAD=1 force one.
        const bool compactOk = c->downRing && c->maxErr < 16 && c->I.n < (1ull << 32);
        const char* fe = std::getenv("SAHARA_FULL_DOWNLOAD");
        const char* ce = std::getenv("SAHARA_COMPACT_DOWNLOAD");
        const bool compact = compactOk && !(fe && std::atoi(fe)) && (!pinned || (ce && std::atoi(ce)));
        if (p && (pinned || compact)) {
            c->sink = static_cast<sahara_hit*>(p);
            c->sinkPinned = pinned;
            c->compactSink = compact;
        } else {
            freeHits(p);
            c->sinkCap = 0;
        }
        if (c->compactSink) {
            if (!c->expander)
                c->expander = std::make_unique<Expander>(c->device, std::max(1u, std::min(8u, std::thread::hardware_concurrency())) - 1);
            c->expander->setStarts(&c->I.recStarts);
            c->expander->mark = [c](const char* w, uint64_t i) { c->mark(w, i); };
            c->expander->reset();
            c->downJobs = 0;
        }
    }
    const auto tC = clk::now();
    try {
        run(c, false);
        uint32_t bad = 0;
        SH_HIP(hipMemcpy(&bad, c->badFlag.ptr, sizeof(uint32_t), hipMemcpyDeviceToHost));
        if (bad) throw Error("pattern rank out of range for this index");
    } catch (...) {
        drainAll(c);
        if (c->compactSink) {
            try {
                c->expander->drain();  // nothing may write into the sink once it is freed
            } catch (...) {
            }
        }
        freeHits(c->sink);
        c->sink = nullptr;
        c->staged = c->streaming = false;
        throw;
    }
    if (c->compactSink) {
        try {
            c->expander->drain();
        } catch (...) {
            freeHits(c->sink);
            c->sink = nullptr;
            throw;
        }
    }
    c->mark("run end", 0);
    c->streaming = false;  // every chunk is up: sahara_gpu_run may re-run the staged patterns
    c->stats.stage_ms = c->up.hostMs;
    for (int b = 0; b < 3; ++b) c->stats.upload_chunks[b] = c->up.chunks[b];
    const auto t0 = std::chrono::steady_clock::now();
    sahara_hit* buf = c->sink;
    c->sink = nullptr;
    try {
        if (max_hits) {
            std::vector<sahara_hit> v(c->nout);
            if (c->nout) SH_HIP(hipMemcpy(v.data(), c->out.ptr, c->nout * sizeof(sahara_hit), hipMemcpyDeviceToHost));
            limitHits(v, max_hits);
            handOver(v, hits, n_hits);
        } else {
            if (buf && c->nout > c->sinkCap) {  // more hits than the sink holds: a bigger buffer, copied whole
                freeHits(buf);
                buf = nullptr;
                c->sinkDone = 0;
            }
            bool pinned = buf != nullptr && c->sinkPinned;
            if (!buf) {
                c->sinkDone = 0;
                buf = static_cast<sahara_hit*>(allocHits(c->nout, &pinned, nullptr, c->lastHits != 0));
                if (!buf) throw Error("out of host memory for hits");
            }
            if (c->nout > c->sinkDone) {  // the rest (or all) of the hits
                const size_t bytes = (c->nout - c->sinkDone) * sizeof(sahara_hit);
                if (pinned) {
                    SH_HIP(hipMemcpyAsync(buf + c->sinkDone, c->out.ptr + c->sinkDone, bytes, hipMemcpyDeviceToHost,
                                          c->st));
                    SH_HIP(hipStreamSynchronize(c->st));
                } else {
                    copyOut(c, buf + c->sinkDone, c->out.ptr + c->sinkDone, bytes);
                }
            }
            *hits = buf;
            *n_hits = c->nout;
            buf = nullptr;
        }
    } catch (...) {
        freeHits(buf);
        throw;
    }
    freeHits(buf);  // the sink of a max_hits call
    c->lastHits = c->nout;
    c->stats.output_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (std::getenv("SAHARA_TIMING")) {  // where a call's wall time goes (stderr)
        auto ms = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
        std::fprintf(stderr, "[sahara] stage %.1f ms, sink %.1f ms, pass %.1f ms (host packing %.1f ms), output %.1f ms\n",
                     ms(tA, tB), ms(tB, tC), ms(tC, t0), c->up.hostMs, c->stats.output_ms);
        std::sort(c->trace.begin(), c->trace.end());
        for (auto& m : c->trace) std::fprintf(stderr, "[sahara]   %8.2f %s\n", m.first, m.second.c_str());
        c->traceOn = false;
    }
}

int sahara_gpu_search(void* ctx, const uint8_t* ranks, uint64_t n_patterns, uint32_t len, const uint32_t* pi,
                      const uint32_t* l, const uint32_t* u, uint32_t n_searches, int edit, uint32_t max_hits,
                      sahara_hit** hits, uint64_t* n_hits) {
    return guarded([&] {
        searchStreamed(ctxOf(ctx), ranks, n_patterns, false, n_patterns, len, pi, l, u, n_searches, edit, max_hits,
                       hits, n_hits);
    });
}

int sahara_gpu_search_reads(void* ctx, const uint8_t* reads, uint64_t n_reads, uint32_t len, int reverse,
                            uint64_t limit, const uint32_t* pi, const uint32_t* l, const uint32_t* u,
                            uint32_t n_searches, int edit, uint32_t max_hits, sahara_hit** hits, uint64_t* n_hits) {
    return guarded([&] {
        Ctx* c = ctxOf(ctx);
        if (c->I.sigma != 5 && c->I.sigma != 6) throw Error("reverse complements need a dna4 or dna5 index");
        uint64_t npat = reverse ? 2 * n_reads : n_reads;
        if (limit && limit < npat) npat = limit;  // --limit_queries cuts the interleaved list (search.cpp:125-127)
        if (npat == 0) throw Error("no patterns");
        const uint64_t rows = reverse ? (npat + 1) / 2 : npat;
        searchStreamed(c, reads, rows, reverse != 0, npat, len, pi, l, u, n_searches, edit, max_hits, hits, n_hits);
    });
}

int sahara_gpu_search_best(void* ctx, const uint8_t* ranks, uint64_t n_patterns, uint32_t len, const uint32_t* pi,
                           const uint32_t* l, const uint32_t* u, const uint32_t* n_searches, uint32_t n_schemes,
                           uint32_t max_hits, sahara_hit** hits, uint64_t* n_hits) {
    return guarded([&] {
        Ctx* c = ctxOf(ctx);
        if (!n_schemes) throw Error("sahara_gpu_search_best: no schemes");
        // search_ng21::search_best (search.cpp:233-241): scheme j holds exactly j
        // errors; a pattern leaves the work list at the first j that reports.
        std::vector<uint64_t> todo(n_patterns);
        for (uint64_t i = 0; i < n_patterns; ++i) todo[i] = i;
        std::vector<uint8_t> sub;
        std::vector<sahara_hit> all;
        sahara_stats acc{};
        uint64_t off = 0;
        for (uint32_t j = 0; j < n_schemes && !todo.empty(); off += (uint64_t)n_searches[j] * len, ++j) {
            const uint8_t* src = ranks;
            if (todo.size() != n_patterns) {
                sub.resize(todo.size() * len);
                for (size_t i = 0; i < todo.size(); ++i)
                    std::memcpy(sub.data() + i * len, ranks + todo[i] * len, len);
                src = sub.data();
            }
            stage(c, src, todo.size(), len, pi + off, l + off, u + off, n_searches[j], 1);
            run(c, false);
            std::vector<sahara_hit> v(c->nout);
            if (c->nout) SH_HIP(hipMemcpy(v.data(), c->out.ptr, c->nout * sizeof(sahara_hit), hipMemcpyDeviceToHost));
            acc.search_ms += c->stats.search_ms;
            acc.locate_ms += c->stats.locate_ms;
            acc.sort_ms += c->stats.sort_ms;
            acc.total_ms += c->stats.total_ms;
            acc.hits += c->stats.hits;
            acc.patterns += c->stats.patterns;
            std::vector<char> found(todo.size(), 0);
            for (auto& h : v) {
                found[h.qid] = 1;
                h.qid = todo[h.qid];
            }
            all.insert(all.end(), v.begin(), v.end());
            size_t w = 0;
            for (size_t i = 0; i < todo.size(); ++i)
                if (!found[i]) todo[w++] = todo[i];
            todo.resize(w);
        }
        c->stats = acc;
        std::sort(all.begin(), all.end(), hitLess);
        if (max_hits) limitHits(all, max_hits);
        handOver(all, hits, n_hits);
    });
}

void sahara_gpu_free(void* p) { freeHits(p); }

void sahara_gpu_close(void* ctx) {
    if (!ctx) return;
    Ctx* c = static_cast<Ctx*>(ctx);
    (void)hipSetDevice(c->device);
    delete c;
}

// ------------------------------------------------------------ synthetic ----

int sahara_synth_reference(uint64_t seed, uint32_t sigma, const uint64_t* rec_lens, uint64_t n_records,
                           uint8_t* out) {
    return guarded([&] {
        if (sigma != 5 && sigma != 6) throw Error("sigma must be 5 or 6");
        const uint8_t code[4] = {1, 2, 3, (uint8_t)(sigma == 6 ? 5 : 4)};
        uint64_t total = 0;
        for (uint64_t r = 0; r < n_records; ++r) total += rec_lens[r];
        std::mt19937_64 gen(seed);
        uint64_t i = 0;
        for (; i + 32 <= total; i += 32) {
            uint64_t x = gen();
            for (int j = 0; j < 32; ++j) out[i + j] = code[(x >> (2 * j)) & 3u];
        }
        if (i < total) {
            uint64_t x = gen();
            for (int j = 0; i < total; ++i, ++j) out[i] = code[(x >> (2 * j)) & 3u];
        }
    });
}

int sahara_synth_reads(const uint8_t* ranks, const uint64_t* rec_lens, uint64_t n_records, uint32_t sigma,
                       uint64_t n_reads, uint32_t len, uint32_t errors, uint64_t seed, uint8_t* out,
                       uint64_t* origin) {
    return guarded([&] { synthReads(ranks, rec_lens, n_records, sigma, n_reads, len, 0, 0, 0, errors, seed, out, origin); });
}

int sahara_synth_reads_typed(const uint8_t* ranks, const uint64_t* rec_lens, uint64_t n_records, uint32_t sigma,
                             uint64_t n_reads, uint32_t len, uint32_t substitutions, uint32_t insertions,
                             uint32_t deletions, uint32_t errors, uint64_t seed, uint8_t* out, uint64_t* origin) {
    return guarded([&] {
        synthReads(ranks, rec_lens, n_records, sigma, n_reads, len, substitutions, insertions, deletions, errors, seed,
                   out, origin);
    });
}

int sahara_pack_2bit(const uint8_t* ranks, uint64_t n, uint32_t sigma, int scalar, uint8_t* out, uint32_t* n_pos,
                     uint64_t pos_cap, uint64_t* n_count) {
    int bad = 0;
    const int rc = guarded([&] {
        if (sigma != 5 && sigma != 6) throw Error("sigma must be 5 or 6");
        if (n >= (1ull << 32)) throw Error("at most 2^32 - 1 symbols per chunk");
        std::vector<uint32_t> pos;
        const uint64_t acc = (!scalar && hostHasAvx2()) ? pack2Avx2(ranks, out, n, sigma, 0, pos)
                                                        : pack2Scalar(ranks, out, n, sigma, 0, pos);
        bad = acc ? 1 : 0;
        *n_count = pos.size();
        if (n_pos && !pos.empty()) std::memcpy(n_pos, pos.data(), std::min<uint64_t>(pos.size(), pos_cap) * 4);
    });
    return rc ? rc : bad;
}

int sahara_interleave_rc(const uint8_t* reads, uint64_t n_reads, uint32_t len, uint32_t sigma, uint8_t* out) {
    return guarded([&] {
        if (sigma != 5 && sigma != 6) throw Error("sigma must be 5 or 6");
        uint8_t comp[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (sigma == 6) { comp[1] = 5; comp[2] = 3; comp[3] = 2; comp[4] = 4; comp[5] = 1; }
        else            { comp[1] = 4; comp[2] = 3; comp[3] = 2; comp[4] = 1; }
        for (uint64_t i = 0; i < n_reads; ++i) {
            const uint8_t* r = reads + i * len;
            uint8_t* f = out + (2 * i) * len;
            uint8_t* b = out + (2 * i + 1) * len;
            std::memcpy(f, r, len);
            for (uint32_t j = 0; j < len; ++j) b[j] = comp[r[len - 1 - j] & 7];
        }
    });
}

}  // extern "C"
