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
#include <cctype>
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
#include <sys/syscall.h>
#include <unistd.h>

#include "ctx.h"
#include "search.h"

using namespace sahara;

namespace sahara {

thread_local std::string g_err;

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

// SAHARA_DEVICE_MAP=a,b,c (test hook): context device d opens HIP device
// list[d], so that `sahara search --gpus N` and concurrent contexts run their
// multi-device code path on one GPU (tests/test_multi_device.py)
static int mapDevice(int device) {
    const char* e = std::getenv("SAHARA_DEVICE_MAP");
    if (!e || !*e) return device;
    std::vector<int> map;
    for (const char* p = e; *p;) {
        char* end = nullptr;
        const long v = std::strtol(p, &end, 10);
        if (end == p) throw Error(std::string("SAHARA_DEVICE_MAP: not a list of device numbers: ") + e);
        map.push_back((int)v);
        p = *end == ',' ? end + 1 : end;
        if (*end && *end != ',') throw Error(std::string("SAHARA_DEVICE_MAP: not a list of device numbers: ") + e);
    }
    if (device < 0 || (size_t)device >= map.size())
        throw Error("SAHARA_DEVICE_MAP has no entry for device " + std::to_string(device));
    return map[(size_t)device];
}

// The CPUs of NUMA node `node` that this process may run on.
Placement placementOfNode(int node) {
    Placement pl;
    pl.node = node;
    if (node < 0) return pl;
    std::FILE* f = std::fopen(("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist").c_str(), "r");
    if (!f) return pl;
    char buf[8192] = {0};
    const size_t got = std::fread(buf, 1, sizeof(buf) - 1, f);
    std::fclose(f);
    buf[got] = 0;
    cpu_set_t allowed;
    CPU_ZERO(&allowed);
    if (sched_getaffinity(0, sizeof(allowed), &allowed) != 0) return pl;
    cpu_set_t set;
    CPU_ZERO(&set);
    for (const char* p = buf; *p && *p != '\n';) {  // "0-15,64-79"
        char* end = nullptr;
        const long a = std::strtol(p, &end, 10);
        if (end == p) break;
        long b = a;
        if (*end == '-') b = std::strtol(end + 1, &end, 10);
        for (long i = a; i <= b && i < CPU_SETSIZE; ++i)
            if (CPU_ISSET(i, &allowed)) CPU_SET(i, &set);
        p = *end == ',' ? end + 1 : end;
    }
    pl.cpus = set;
    pl.ncpus = CPU_COUNT(&set);
    return pl;
}

// The CPUs of the device's NUMA node that this process may run on (Placement).
static void placeNear(Ctx* c) {
    const char* e = std::getenv("SAHARA_NUMA");
    if (e && std::atoi(e) == 0) return;
    char bdf[64] = {0};
    if (hipDeviceGetPCIBusId(bdf, sizeof(bdf), c->device) != hipSuccess) {
        (void)hipGetLastError();
        return;
    }
    std::string id(bdf);
    for (char& ch : id) ch = (char)std::tolower((unsigned char)ch);
    int node = -1;
    if (std::FILE* f = std::fopen(("/sys/bus/pci/devices/" + id + "/numa_node").c_str(), "r")) {
        if (std::fscanf(f, "%d", &node) != 1) node = -1;
        std::fclose(f);
    }
    c->place = placementOfNode(node);
}

// host threads a context uses for one job: its node's allowed CPUs (or the
// process's), at most cap
unsigned hostThreads(const Ctx* c, unsigned cap) {
    unsigned n = (unsigned)c->place.ncpus;
    if (n == 0) {
        cpu_set_t s;
        CPU_ZERO(&s);
        n = sched_getaffinity(0, sizeof(s), &s) == 0 ? (unsigned)CPU_COUNT(&s) : std::thread::hardware_concurrency();
    }
    return std::max(1u, std::min(cap, n));
}

Ctx* newCtx(int device) {
    int n = 0;
    SH_HIP(hipGetDeviceCount(&n));
    const int hipDev = mapDevice(device);
    if (hipDev < 0 || hipDev >= n)
        throw Error("no HIP device " + std::to_string(hipDev) + " (found " + std::to_string(n) + ")");
    SH_HIP(hipSetDevice(hipDev));
    auto c = std::make_unique<Ctx>();
    c->device = hipDev;
    placeNear(c.get());
    hipDeviceProp_t prop;
    SH_HIP(hipGetDeviceProperties(&prop, hipDev));
    if (std::string(prop.gcnArchName).find("gfx950") == std::string::npos)
        throw Error(std::string("libsahara_hip is built for gfx950 (MI355X); device is ") + prop.gcnArchName);
    c->numCU = prop.multiProcessorCount;
    SH_HIP(hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking));
    // (No stream gets a CU mask: with a CU-masked stream in the process the
    // memory-bound kernels on the other streams ran 1.4-1.8x longer, r5.)
    SH_HIP(hipStreamCreateWithFlags(&c->stB, hipStreamNonBlocking));
    SH_HIP(hipStreamCreateWithFlags(&c->stC, hipStreamNonBlocking));
    SH_HIP(hipStreamCreateWithFlags(&c->stD, hipStreamNonBlocking));
    SH_HIP(hipStreamCreateWithFlags(&c->stE, hipStreamNonBlocking));
    SH_HIP(hipStreamCreateWithFlags(&c->stF, hipStreamNonBlocking));
    for (auto& e : c->ev) SH_HIP(hipEventCreate(&e));
    for (auto& e : c->evSleep) SH_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventBlockingSync));
    for (auto& e : c->ringEv) SH_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    // the streamed upload's pinned ring, pinned while the caller builds or
    // loads the index (pinning 256 MB takes ~50 ms)
    Ctx* raw = c.get();
    raw->ringInit = std::thread([raw] {
        raw->place.bind();  // pinned pages first touched on the device's node
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
        for (hipEvent_t* e : {&sl.fmStart, &sl.seedDone, &sl.seedDone0, &sl.seedMid, &sl.fmBegin, &sl.fmDone,
                              &sl.textStart, &sl.textDone, &sl.free, &sl.textMid0, &sl.textMid1})
            SH_HIP(hipEventCreate(e));
        sl.small.reserve(8);
        sl.queues.reserve(768);
    }
    for (void*& p : c->outStage) SH_HIP(hipHostMalloc(&p, Ctx::kOutChunk));
    c->small.reserve(8);
    c->counters.reserve(kCounters);
    SH_HIP(hipMemset(c->counters.ptr, 0, kCounters * sizeof(unsigned long long)));
    return c.release();
}

Ctx* ctxOf(void* p) {
    if (!p) throw Error("null context");
    Ctx* c = static_cast<Ctx*>(p);
    SH_HIP(hipSetDevice(c->device));
    return c;
}

// an .idx image (one part or several) -> a context holding every part
Ctx* openImage(int device, const uint8_t* buf, size_t bytes) {
    const auto t0 = std::chrono::steady_clock::now();
    auto since = [&t0] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); };
    const std::vector<IdxParts> parts = parseIdxAll(buf, bytes);
    const double tParse = since();
    std::unique_ptr<Ctx> c(newCtx(device));
    const double tCtx = since();
    if (std::getenv("SAHARA_TIMING"))  // (the parts' own steps follow from buildFromParts)
        std::fprintf(stderr, "[sahara] open: parse %.1f ms, context %.1f ms\n", tParse, tCtx - tParse);
    uint64_t rec0 = 0, nmax = 0;
    c->partRec0.clear();
    // the image's arrays through the pinned ring (SAHARA_LOAD_RING=0: pageable copies)
    Ctx* raw = c.get();
    const HostUpload viaRing = [raw](void* dst, const void* src, size_t n, hipStream_t s) {
        uploadViaRing(raw, dst, src, n, s);
    };
    const char* lr = std::getenv("SAHARA_LOAD_RING");
    const HostUpload* up = lr && std::atoi(lr) == 0 ? nullptr : &viaRing;
    for (size_t p = 0; p < parts.size(); ++p) {
        const IdxParts& P = parts[p];
        if (p) c->more.emplace_back();
        buildFromParts(partOf(c.get(), (uint32_t)p), P.sigma, P.n, P.recLens.data(), P.recLens.size(), P.rate, P.bwtF,
                       P.bwtR, P.sampled, P.samples, P.nsamples, c->st, parts.size() == 1, up);
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

}  // namespace sahara

extern "C" {

const char* sahara_gpu_last_error(void) { return g_err.c_str(); }

const char* sahara_build_id(void) { return SAHARA_BUILD_ID; }

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

int sahara_gpu_open(int device, const void* idx_image, size_t idx_bytes, void** ctx) {
    return guarded([&] { *ctx = openImage(device, static_cast<const uint8_t*>(idx_image), idx_bytes); });
}

int sahara_gpu_open_file(int device, const char* path, void** ctx) {
    return guarded([&] {
        const std::vector<uint8_t> buf = readFile(path);
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
        const char* te = std::getenv("SAHARA_TIMING");  // 2: host-side marks of the call (stderr)
        c->traceOn = te && std::atoi(te) >= 2;
        if (c->traceOn) {
            c->trace.clear();
            c->traceT0 = std::chrono::steady_clock::now();
        }
        run(c, count != 0);
        if (n_hits) *n_hits = c->nout;
        if (c->traceOn) {
            c->mark("run returns", 0);
            std::sort(c->trace.begin(), c->trace.end());
            for (auto& m : c->trace) std::fprintf(stderr, "[sahara]   %8.3f %s\n", m.first, m.second.c_str());
            c->traceOn = false;
        }
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

int sahara_gpu_placement(void* ctx, int* device, int* numa_node, int* n_cpus) {
    return guarded([&] {
        Ctx* c = ctxOf(ctx);
        if (device) *device = c->device;
        if (numa_node) *numa_node = c->place.node;
        if (n_cpus) *n_cpus = c->place.ncpus;
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

// Host buffer of `bytes` (released with sahara_gpu_free); *pinned tells
// whether the device can copy (or write) into it directly; *capBytes its size.
static void* allocPinned(size_t bytes, bool* pinned, size_t* capBytes, bool mayPin, bool always = false);

// Host buffer for n hits (released with sahara_gpu_free).
static void* allocHits(uint64_t n, bool* pinned, uint64_t* capHits = nullptr, bool mayPin = true) {
    size_t cap = 0;
    void* p = allocPinned(std::max<uint64_t>(n, 1) * sizeof(sahara_hit), pinned, &cap, mayPin);
    if (capHits) *capHits = cap / sizeof(sahara_hit);
    return p;
}

// always: pinned whatever the size (a sink the device writes into)
static void* allocPinned(size_t bytes, bool* pinned, size_t* capBytes, bool mayPin, bool always) {
    bytes = std::max<size_t>(bytes, 1);
    *pinned = false;
    *capBytes = bytes;
    size_t pinMin = 64u << 20;  // SAHARA_PIN_MIN: smallest pinned buffer in bytes (tests pin every size)
    if (const char* e = std::getenv("SAHARA_PIN_MIN")) pinMin = (size_t)std::atoll(e);
    if (bytes < pinMin && !always) return std::malloc(bytes);
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
            *capBytes = P.idle[best].second;
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
        *capBytes = cap;
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
    drainPacking(c);  // chunks packed ahead: nothing reads the caller's buffer after the call
    for (hipStream_t s : {c->st, c->stB, c->stC, c->stD, c->stE, c->stF})
        if (s) (void)hipStreamSynchronize(s);
}

// SAHARA_TIMING=2: each chunk DMA's duration and rate from its events
static void printDmaTimes(Ctx* c) {
    for (size_t i = 0; i < c->dmaUsed; ++i) {
        float ms = 0;
        auto& d = c->dmaEv[i];
        if (hipEventElapsedTime(&ms, d.second.first, d.second.second) == hipSuccess)
            std::fprintf(stderr, "[sahara]   dma %zu: %.1f MB in %.3f ms, %.1f GB/s\n", i, d.first / 1e6, ms,
                         ms > 0 ? d.first / (ms * 1e6) : 0.0);
    }
    c->dmaUsed = 0;
}

// sahara_gpu_search / sahara_gpu_search_reads: streamed upload, the pipelined
// pass, the hits streamed into a pinned host sink batch by batch, then handed
// to the caller (search.cpp:218-250 from host queries to host hits).
static void searchStreamed(Ctx* c, const uint8_t* src, uint64_t rows, bool rc, uint64_t npat, uint32_t len,
                           const uint32_t* pi, const uint32_t* l, const uint32_t* u, uint32_t n_searches, int edit,
                           uint32_t max_hits, sahara_hit** hits, uint64_t* n_hits,
                           const PackedReads* packed = nullptr) {
    using clk = std::chrono::steady_clock;
    const auto tA = clk::now();
    {
        const char* te = std::getenv("SAHARA_TIMING");
        c->traceOn = te && std::atoi(te) >= 2;
        c->traceT0 = tA;
        c->trace.clear();
    }
    stageStreamed(c, src, rows, rc, npat, len, pi, l, u, n_searches, edit, packed);
    const auto tB = clk::now();
    c->sink = nullptr;
    c->sinkCap = 0;
    c->compactSink = c->sinkPinned = false;
    // --max_hits: per batch on the device (limitBatch), so the limited hits
    // stream to the host like any others; a multi-part index limits after
    // its parts merge, on the host (limitHits)
    const bool hostLimit = max_hits && !c->more.empty();
    c->limitN = hostLimit ? 0u : max_hits;
    if (!hostLimit) {  // sized from the last call (the bench's steady state), else 2 hits per pattern
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
                c->expander = std::make_unique<Expander>(c->device, hostThreads(c, 8) - 1, &c->place);
            c->expander->setStarts(&c->I.recStarts);
            c->expander->mark = [c](const char* w, uint64_t i) { c->mark(w, i); };
            c->expander->reset();
            c->downJobs = 0;
        }
    }
    const auto tC = clk::now();
    try {
        run(c, false);
        c->limitN = 0;
        uint32_t bad = 0;
        SH_HIP(hipMemcpy(&bad, c->badFlag.ptr, sizeof(uint32_t), hipMemcpyDeviceToHost));
        if (bad) throw Error("pattern rank out of range for this index");
    } catch (...) {
        c->limitN = 0;
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
        if (hostLimit) {
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
        printDmaTimes(c);
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

// sahara_gpu_search_reads_compact: the streamed pass with every batch's hits
// written as 8-B records by the device into a pinned host sink (pass.cpp
// finish), handed over as blocks (one per batch).
static void searchReadsCompact(Ctx* c, const uint8_t* reads, uint64_t n_reads, uint32_t len, int reverse,
                               uint64_t limit, const uint32_t* pi, const uint32_t* l, const uint32_t* u,
                               uint32_t n_searches, int edit, sahara_hit_blocks* out,
                               const PackedReads* packed = nullptr) {
    using clk = std::chrono::steady_clock;
    const auto tA = clk::now();
    if (c->I.sigma != 5 && c->I.sigma != 6) throw Error("reverse complements need a dna4 or dna5 index");
    if (!c->more.empty()) throw Error("compact hit records need a single-part index (text < 2^32 symbols)");
    uint64_t npat = reverse ? 2 * n_reads : n_reads;
    if (limit && limit < npat) npat = limit;  // --limit_queries (search.cpp:125-127)
    if (npat == 0) throw Error("no patterns");
    const uint64_t rows = reverse ? (npat + 1) / 2 : npat;
    {
        const char* te = std::getenv("SAHARA_TIMING");
        c->traceOn = te && std::atoi(te) >= 2;
        c->traceT0 = tA;
        c->trace.clear();
    }
    for (uint64_t i = 0; i < (uint64_t)n_searches * len; ++i)  // before staging: a refused call stages nothing
        if (u[i] > 15) throw Error("compact hit records hold at most 15 errors");
    stageStreamed(c, reads, rows, reverse != 0, npat, len, pi, l, u, n_searches, edit, packed);
    c->sink = nullptr;
    c->compactSink = c->sinkPinned = false;
    // the sink, sized from the last call (else 2 hits per pattern), always
    // page-locked: the device writes into it
    const uint64_t est = c->lastHits ? c->lastHits + c->lastHits / 8 + 1024 : 2 * npat + 1024;
    bool pinned = false;
    size_t capBytes = 0;
    void* sinkMem = nullptr;
    try {
        sinkMem = allocPinned(est * 8, &pinned, &capBytes, true, true);
        if (!sinkMem) throw Error("out of host memory for hits");
        c->blockRecs = pinned ? static_cast<uint64_t*>(sinkMem) : nullptr;
        c->sinkCap = pinned ? capBytes / 8 : 0;
        if (c->sinkCap) c->outRecs.reserve(c->sinkCap);
    } catch (...) {  // nothing may stream from the caller's reads after the call
        drainPacking(c);
        freeHits(sinkMem);
        c->blockRecs = nullptr;
        c->staged = c->streaming = false;
        throw;
    }
    auto* recs = static_cast<uint64_t*>(sinkMem);
    uint64_t recCap = capBytes / 8;
    try {
        run(c, false);
        uint32_t bad = 0;
        SH_HIP(hipMemcpy(&bad, c->badFlag.ptr, sizeof(uint32_t), hipMemcpyDeviceToHost));
        if (bad) throw Error("pattern rank out of range for this index");
        const auto t0 = clk::now();
        if (!c->blockRecs || c->sinkDone < c->nout) {
            // the sink held too few (or is not pinned): the records of every
            // batch again, from the device-resident hits, into one that fits
            if (c->nout > recCap) {
                freeHits(recs);
                recs = nullptr;
                recs = static_cast<uint64_t*>(allocPinned(c->nout * 8, &pinned, &capBytes, true, true));
                if (!recs) throw Error("out of host memory for hits");
                recCap = capBytes / 8;
            }
            uint64_t* dst = recs;
            if (!pinned) {
                c->outC.reserve(std::max<uint64_t>(c->nout, 1));
                dst = c->outC.ptr;
            }
            uint64_t b0 = 0;
            for (size_t b = 0; b < c->batchQ0.size(); ++b) {
                launchCompactHits(c->out.ptr + b0, c->batchEnd[b] - b0, c->batchQ0[b], c->I.dRecStarts.ptr, dst + b0,
                                  c->st, pinned ? 256u : 8192u);
                b0 = c->batchEnd[b];
            }
            if (!pinned && c->nout) SH_HIP(hipMemcpyAsync(recs, dst, c->nout * 8, hipMemcpyDeviceToHost, c->st));
            SH_HIP(hipStreamSynchronize(c->st));
        }
        c->stats.output_ms = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
    } catch (...) {
        drainAll(c);
        c->blockRecs = nullptr;
        freeHits(recs);
        c->staged = c->streaming = false;
        throw;
    }
    c->blockRecs = nullptr;
    c->streaming = false;
    c->stats.stage_ms = c->up.hostMs;
    for (int b = 0; b < 3; ++b) c->stats.upload_chunks[b] = c->up.chunks[b];
    const size_t nb = c->batchQ0.size();
    auto* q0 = static_cast<uint64_t*>(std::malloc(std::max<size_t>(nb, 1) * 8));
    auto* end = static_cast<uint64_t*>(std::malloc(std::max<size_t>(nb, 1) * 8));
    if (!q0 || !end) {
        std::free(q0);
        std::free(end);
        freeHits(recs);
        throw Error("out of host memory for hit blocks");
    }
    for (size_t b = 0; b < nb; ++b) {
        q0[b] = c->batchQ0[b];
        end[b] = c->batchEnd[b];
    }
    if (c->recStartsEnd.size() != c->I.recStarts.size() + 1) {
        c->recStartsEnd = c->I.recStarts;
        c->recStartsEnd.push_back(c->I.n);
    }
    out->recs = recs;
    out->n_hits = c->nout;
    out->block_qid0 = q0;
    out->block_end = end;
    out->n_blocks = nb;
    out->rec_starts = c->recStartsEnd.data();
    out->n_records = c->I.recStarts.size();
    c->lastHits = c->nout;
    if (std::getenv("SAHARA_TIMING")) {
        auto ms = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
        std::fprintf(stderr, "[sahara] compact call %.1f ms (host packing %.1f ms), output %.1f ms\n", ms(tA, clk::now()),
                     c->up.hostMs, c->stats.output_ms);
        std::sort(c->trace.begin(), c->trace.end());
        for (auto& m : c->trace) std::fprintf(stderr, "[sahara]   %8.2f %s\n", m.first, m.second.c_str());
        printDmaTimes(c);
        c->traceOn = false;
    }
}

int sahara_gpu_search_reads_compact(void* ctx, const uint8_t* reads, uint64_t n_reads, uint32_t len, int reverse,
                                    uint64_t limit, const uint32_t* pi, const uint32_t* l, const uint32_t* u,
                                    uint32_t n_searches, int edit, sahara_hit_blocks* out) {
    return guarded([&] {
        if (!out) throw Error("sahara_gpu_search_reads_compact: null output");
        *out = sahara_hit_blocks{};
        searchReadsCompact(ctxOf(ctx), reads, n_reads, len, reverse, limit, pi, l, u, n_searches, edit, out);
    });
}

int sahara_gpu_search_packed(void* ctx, const uint8_t* codes, uint64_t sym0, const uint64_t* n_pos, uint64_t n_count,
                             uint64_t n_reads, uint32_t len, int reverse, uint64_t limit, const uint32_t* pi,
                             const uint32_t* l, const uint32_t* u, uint32_t n_searches, int edit, uint32_t max_hits,
                             sahara_hit** hits, uint64_t* n_hits) {
    return guarded([&] {
        Ctx* c = ctxOf(ctx);
        if (!codes || (n_count && !n_pos)) throw Error("sahara_gpu_search_packed: null input");
        uint64_t npat = reverse ? 2 * n_reads : n_reads;
        if (limit && limit < npat) npat = limit;  // --limit_queries cuts the interleaved list (search.cpp:125-127)
        if (npat == 0) throw Error("no patterns");
        const uint64_t rows = reverse ? (npat + 1) / 2 : npat;
        const PackedReads pk{sym0, n_pos, n_count};
        searchStreamed(c, codes, rows, reverse != 0, npat, len, pi, l, u, n_searches, edit, max_hits, hits, n_hits,
                       &pk);
    });
}

int sahara_gpu_search_packed_compact(void* ctx, const uint8_t* codes, uint64_t sym0, const uint64_t* n_pos,
                                     uint64_t n_count, uint64_t n_reads, uint32_t len, int reverse, uint64_t limit,
                                     const uint32_t* pi, const uint32_t* l, const uint32_t* u, uint32_t n_searches,
                                     int edit, sahara_hit_blocks* out) {
    return guarded([&] {
        if (!out) throw Error("sahara_gpu_search_packed_compact: null output");
        *out = sahara_hit_blocks{};
        if (!codes || (n_count && !n_pos)) throw Error("sahara_gpu_search_packed_compact: null input");
        const PackedReads pk{sym0, n_pos, n_count};
        searchReadsCompact(ctxOf(ctx), codes, n_reads, len, reverse, limit, pi, l, u, n_searches, edit, out, &pk);
    });
}

int sahara_gpu_prepare(void* ctx, uint64_t n_patterns, uint32_t len) {
    return guarded([&] {
        if (n_patterns == 0) return;
        Ctx* c = ctx ? ctxOf(ctx) : nullptr;
        if (c) SH_HIP(hipSetDevice(c->device));
        // the sink the first compact call asks the pool for (searchReadsCompact),
        // pinned now and handed back to the pool, where the call finds it
        const uint64_t est = c && c->lastHits ? c->lastHits + c->lastHits / 8 + 1024 : 2 * n_patterns + 1024;
        bool pinned = false;
        size_t capBytes = 0;
        {
            HitPool& P = hitPool();
            std::lock_guard<std::mutex> g(P.mu);
            for (auto& e : P.idle)
                if (e.second >= est * 8) {  // pinned already (a NULL-context call before)
                    pinned = true;
                    capBytes = e.second;
                }
        }
        if (!pinned) {
            void* p = allocPinned(est * 8, &pinned, &capBytes, true, true);
            if (!p) throw Error("out of host memory for hits");
            freeHits(p);
        }
        if (!c) return;  // (NULL context: the host part only, e.g. beside the index load)
        if (pinned) c->outRecs.reserve(capBytes / 8);
        c->out.reserve(est);
        // the slots of a streamed pass (pass.cpp runPass: 2M-pattern batches),
        // sized as that pass sizes them
        const uint64_t maxBatch = 1ull << 21;
        initWorkCaps(c, maxBatch);
        const uint64_t nb = std::min<uint64_t>((n_patterns + maxBatch - 1) / maxBatch, Ctx::kSlots);
        // the locate chain's per-batch buffers (pass.cpp; the keys sized for a
        // batch's rows at four per pattern, grown by the pass if short)
        c->qoff.reserve(maxBatch + 1);
        c->big.reserve(maxBatch);
        c->huge.reserve(maxBatch);
        c->partial.reserve(scanTiles((uint32_t)maxBatch));
        c->k0.reserve(std::min<uint64_t>(n_patterns, maxBatch) * 4);
        for (uint64_t i = 0; i < nb; ++i) {
            Ctx::Slot& sl = c->slot[i];
            sl.hits.reserve((size_t)c->hitCap + 1);
            sl.rank.reserve((size_t)c->hitCap + 1);
            sl.tasks.reserve((size_t)c->taskCap);
            sl.qcnt.reserve(maxBatch + 1);  // per-query row counts (pass.cpp)
        }
        if (len) {
            const uint64_t patWords = (len + 7) / 8, patBlocks = (len + 31) / 32;
            c->rawPats.reserve(n_patterns * len);
            c->pats.reserve(n_patterns * patWords + 4);
            c->pats3.reserve(n_patterns * patBlocks);
            c->readRaw.reserve((n_patterns + 1) / 2 * len);
            c->nibPats.reserve((n_patterns * len + 1) / 2 + 16);  // the streamed upload's staging (staging.cpp)
        }
    });
}

void sahara_gpu_free_blocks(sahara_hit_blocks* b) {
    if (!b) return;
    freeHits(b->recs);
    std::free(b->block_qid0);
    std::free(b->block_end);
    *b = sahara_hit_blocks{};
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
            // --max_hits per batch on the device (single part; the host pass
            // below is then a no-op on what is left)
            c->limitN = c->more.empty() ? max_hits : 0u;
            try {
                run(c, false);
            } catch (...) {
                c->limitN = 0;
                throw;
            }
            c->limitN = 0;
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

void* sahara_host_alloc(size_t bytes) {
    void* p = nullptr;
    if (hipHostMalloc(&p, std::max<size_t>(bytes, 1), hipHostMallocPortable) != hipSuccess) {
        (void)hipGetLastError();
        g_err = "could not allocate " + std::to_string(bytes) + " bytes of page-locked host memory";
        return nullptr;
    }
    return p;
}

void sahara_host_free(void* p) {
    if (p) (void)hipHostFree(p);
}

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
        // scalar: 0 the widest the host has (AVX-512 / AVX2), 1 scalar, 2 AVX2 at most
        const uint64_t acc = scalar == 1 ? pack2Scalar(ranks, out, n, sigma, 0, pos)
                             : scalar == 2 ? (hostHasAvx2() ? pack2Avx2(ranks, out, n, sigma, 0, pos)
                                                            : pack2Scalar(ranks, out, n, sigma, 0, pos))
                                           : pack2Best(ranks, out, n, sigma, 0, pos);
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
