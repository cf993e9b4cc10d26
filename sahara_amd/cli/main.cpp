// main.cpp — the `sahara` command line, MI355X build.
//
// Drop-in for the reference CLI on the search hot path:
//   sahara index <fasta> [--ignore_unknown] [--dna4]          (src/sahara/index.cpp:20-121)
//   sahara search -q <fasta> -i <idx> [-o out] [-g gen] [-e k] [--no-reverse]
//                 [-m all|besthits] [-d ham|lev] [--max_hits n] [--limit_queries n]
//                                                            (src/sahara/search.cpp:22-291)
// Same flag spellings, defaults, stdout blocks, output format and exit codes
// (errors print their message and exit 1, main.cpp:13). Additions, all
// optional: --gpus N (query shards over N devices), --emit-errors (fourth
// output column e), --fm-only (reference execution: no text phase, LF-walk
// locate). The compute goes through the C ABI of libsahara_hip.so only.

#include <algorithm>
#include <atomic>
#include <charconv>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstdarg>
#include <cstring>
#include <fstream>
#include <functional>
#include <future>
#include <map>
#include <stdexcept>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "../../include/sahara_hip.h"
#include "../csrc/fasta.h"
#include "shard.h"

using namespace sahara_cli;
using namespace sahara_io;

namespace sahara_cli {
struct ReadSimulatorArgs {
    std::string input, output;
    size_t lineLength = 80, readLength = 150, nreads = 1000, sub = 0, ins = 0, del = 0, errors = 0;
    uint32_t seed = 0;
    bool haveInput = false;
};
int runReadSimulator(const ReadSimulatorArgs& a);  // read_simulator.cpp
}  // namespace sahara_cli

namespace {

struct CliError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

std::string fmtStr(const char* f, ...) __attribute__((format(printf, 1, 2)));
std::string fmtStr(const char* f, ...) {
    char buf[4096];
    va_list ap;
    va_start(ap, f);
    std::vsnprintf(buf, sizeof(buf), f, ap);
    va_end(ap);
    return buf;
}

// utils/StopWatch.h:8-28
struct StopWatch {
    std::chrono::steady_clock::time_point start = std::chrono::steady_clock::now();
    double reset() {
        auto t = std::chrono::steady_clock::now();
        double d = std::chrono::duration<double>(t - start).count();
        start = t;
        return d;
    }
};

void check(int rc, const char* what) {
    if (rc != 0) throw CliError(std::string(what) + ": " + sahara_gpu_last_error());
}

// ------------------------------------------------------------- options ----

struct Opt {
    std::vector<std::string> names;
    bool flag = false;
    std::string value;
    bool given = false;
};

struct Parser {
    std::map<std::string, Opt*> byName;
    std::vector<std::string> positional;
    void add(Opt& o) {
        for (auto& n : o.names) byName[n] = &o;
    }
    void parse(int argc, char** argv, int first) {
        for (int i = first; i < argc; ++i) {
            std::string a = argv[i];
            std::string val;
            bool hasVal = false;
            if (a.size() > 2 && a[0] == '-' && a.find('=') != std::string::npos) {
                val = a.substr(a.find('=') + 1);
                a = a.substr(0, a.find('='));
                hasVal = true;
            }
            auto it = byName.find(a);
            if (it == byName.end()) {
                if (!a.empty() && a[0] == '-' && a.size() > 1 && !std::isdigit((unsigned char)a[1]))
                    throw CliError("unknown option " + a);
                positional.push_back(a);
                continue;
            }
            Opt& o = *it->second;
            o.given = true;
            if (o.flag) continue;
            if (!hasVal) {
                if (i + 1 >= argc) throw CliError("option " + a + " expects a value");
                val = argv[++i];
            }
            o.value = val;
        }
    }
};

uint64_t toU64(const std::string& s, const char* what) {
    uint64_t v = 0;
    auto r = std::from_chars(s.data(), s.data() + s.size(), v);
    if (r.ec != std::errc() || r.ptr != s.data() + s.size()) throw CliError(std::string("invalid value for ") + what + ": " + s);
    return v;
}

// ---------------------------------------------------------------- index ----

int cmdIndex(int argc, char** argv) {
    Opt ignore{{"--ignore_unknown"}, true}, dna4{{"--dna4"}, true}, gpu{{"--gpu"}, false, "0"};
    Parser p;
    p.add(ignore);
    p.add(dna4);
    p.add(gpu);
    p.parse(argc, argv, 2);
    if (p.positional.size() != 1) throw CliError("sahara index expects exactly one FASTA file");
    const std::string path = p.positional[0];
    const uint32_t sigma = dna4.given ? 5 : 6;

    std::printf("constructing an index for %s\n", path.c_str());
    std::vector<std::tuple<std::string, double>> timing;
    StopWatch sw;

    // parallel whole-file ingest (fasta.h parseFastaParallel): records, ranks, first invalid character
    const unsigned nt = hostThreads();
    FastaData D = parseFastaParallel(path, sigma, nt);
    const uint64_t totalSize = D.ranks.size();
    if (ignore.given) {  // index.cpp:56-68: unknown characters become N (dna5) or a random base (dna4)
        if (dna4.given) {
            for (auto& v : D.ranks)
                if (v == 255 || v == 0 || v >= sigma) v = (uint8_t)(1 + std::rand() % 4);
        } else {
            parallelFor(nt, nt, [&](size_t t) {
                for (size_t i = D.ranks.size() * t / nt; i < D.ranks.size() * (t + 1) / nt; ++i)
                    if (D.ranks[i] == 255 || D.ranks[i] == 0 || D.ranks[i] >= sigma) D.ranks[i] = 4;
            });
        }
    } else if (D.bad) {
        const unsigned char ch = D.badChar;
        throw CliError(fmtStr("ref '%s' (%zu) has invalid character '%c' (0x%02x) at position %ld", D.badId.c_str(),
                              D.badRecord + 1, ch, ch, (long)D.badPos));
    }
    std::vector<uint64_t> lens(D.records());
    for (size_t r = 0; r < lens.size(); ++r) lens[r] = D.offs[r + 1] - D.offs[r];
    std::vector<uint8_t>& ranks = D.ranks;
    if (lens.empty()) throw CliError("reference file " + path + " was empty - abort\n");
    std::printf("config:\n");
    std::printf("  file: %s\n", path.c_str());
    std::printf("  sigma: %u\n", sigma);
    std::printf("  references: %zu\n", lens.size());
    std::printf("  totalSize: %llu\n", (unsigned long long)totalSize);
    timing.emplace_back("ld queries", sw.reset());

    void* ctx = nullptr;
    check(sahara_gpu_build((int)toU64(gpu.value, "--gpu"), ranks.data(), lens.data(), lens.size(), sigma, 16, &ctx),
          "index construction");
    timing.emplace_back("index creation", sw.reset());

    const std::string out = path + (dna4.given ? ".dna4.idx" : ".idx");
    check(sahara_gpu_save(ctx, out.c_str()), "saving index");
    sahara_gpu_close(ctx);
    timing.emplace_back("saving to disk", sw.reset());

    std::printf("stats:\n");
    double total = 0;
    for (auto& [k, t] : timing) {
        std::printf("  %-20s %10.2fs\n", (k + " time:").c_str(), t);
        total += t;
    }
    std::printf("  total time:          %10.2fs\n", total);
    return 0;
}

// --------------------------------------------------------------- search ----

// One device's hits as the library hands them over: qids local to its shard.
// Either whole records (hits) or compact ones (blocks, sahara_hit_blocks).
struct HitPart {
    sahara_hit* hits = nullptr;
    sahara_hit_blocks blocks{};
    bool compact = false;
    uint64_t n = 0;
    uint64_t qidOffset = 0;
    void release() {
        if (compact) sahara_gpu_free_blocks(&blocks);
        else sahara_gpu_free(hits);
        hits = nullptr;
        compact = false;
    }
};

// Text output of hits: "qid seqId pos[ e]\n" (search.cpp:254-261). Blocks of
// hits are formatted by nt threads, each taking the next block in order; a
// block's file offset is the previous block's end, published as soon as that
// block is formatted, so each thread writes its own block (pwrite) while the
// others format theirs: formatting and writing both run on every thread.
// Compact records are decoded right here, in the formatting loop that runs
// anyway: record id by the record starts (usually the previous hit's record),
// position, errors.
void writeHits(const std::string& path, const std::vector<HitPart>& parts, bool emitErrors, unsigned nt) {
    const int fd = ::open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
    if (fd < 0) throw CliError("can not open output file " + path);
    struct CloseFd {  // closed on every path out (formatting may throw, e.g. bad_alloc)
        int fd;
        bool closed = false;
        int close() { closed = true; return ::close(fd); }
        ~CloseFd() { if (!closed) (void)::close(fd); }
    } closer{fd};
    struct Block {
        const HitPart* part;
        uint64_t lo, hi;
    };
    std::vector<Block> blocks;
    constexpr uint64_t kBlock = 1u << 18;  // hits per block (~7 MB of text)
    for (const auto& hp : parts)
        for (uint64_t lo = 0; lo < hp.n; lo += kBlock) blocks.push_back({&hp, lo, std::min(hp.n, lo + kBlock)});
    std::vector<std::atomic<int64_t>> ends(blocks.size());
    for (auto& e : ends) e.store(-1, std::memory_order_relaxed);
    std::atomic<size_t> next{0};
    std::atomic<bool> failed{false};
    parallelFor(nt, nt, [&](size_t) {
        std::vector<char> buf;
        for (;;) {
            const size_t bi = next.fetch_add(1, std::memory_order_relaxed);
            if (bi >= blocks.size()) return;
            // A block that fails to format still publishes its end (as an
            // empty block), so that the blocks after it do not wait forever;
            // the call then fails.
            auto publishEmpty = [&] {
                int64_t off = 0;
                if (bi > 0)
                    while ((off = ends[bi - 1].load(std::memory_order_acquire)) < 0) std::this_thread::yield();
                ends[bi].store(off, std::memory_order_release);
            };
            const Block& B = blocks[bi];
            try {
                buf.resize((B.hi - B.lo) * 96);
            } catch (...) {
                failed.store(true);
                publishEmpty();
                continue;
            }
            char* o = buf.data();
            char* e = o + buf.size();
            auto line = [&](uint64_t qid, uint64_t seq, uint64_t pos, uint32_t err) {
                o = std::to_chars(o, e, qid).ptr;
                *o++ = ' ';
                o = std::to_chars(o, e, seq).ptr;
                *o++ = ' ';
                o = std::to_chars(o, e, pos).ptr;
                if (emitErrors) {
                    *o++ = ' ';
                    o = std::to_chars(o, e, err).ptr;
                }
                *o++ = '\n';
            };
            const HitPart& P = *B.part;
            if (!P.compact) {
                for (uint64_t k = B.lo; k < B.hi; ++k) {
                    const sahara_hit& h = P.hits[k];
                    line(h.qid + P.qidOffset, h.seq_id, h.pos, h.err);
                }
            } else {
                const sahara_hit_blocks& H = P.blocks;
                const uint64_t* S = H.rec_starts;
                uint64_t blk = (uint64_t)(std::upper_bound(H.block_end, H.block_end + H.n_blocks, B.lo) - H.block_end);
                uint64_t seq = 0, lo = 1, hi = 0;  // the current record's [start, next start): empty
                for (uint64_t k = B.lo; k < B.hi; ++k) {
                    while (k >= H.block_end[blk]) ++blk;
                    const uint64_t v = H.recs[k], g = (v >> 4) & 0xFFFFFFFFull;
                    if (g < lo || g >= hi) {
                        seq = (uint64_t)(std::upper_bound(S, S + H.n_records + 1, g) - S) - 1;
                        lo = S[seq];
                        hi = S[seq + 1];
                    }
                    line(H.block_qid0[blk] + (v >> 36) + P.qidOffset, seq, g - lo, (uint32_t)(v & 15u));
                }
            }
            const int64_t size = (int64_t)(o - buf.data());
            int64_t off = 0;
            if (bi > 0)
                while ((off = ends[bi - 1].load(std::memory_order_acquire)) < 0) std::this_thread::yield();
            ends[bi].store(off + size, std::memory_order_release);
            for (int64_t done = 0; done < size && !failed.load(std::memory_order_relaxed);) {
                const ssize_t w = ::pwrite(fd, buf.data() + done, (size_t)(size - done), off + done);
                if (w <= 0) failed.store(true);
                else done += w;
            }
        }
    });
    if (closer.close() != 0 || failed.load()) throw CliError("can not write output file " + path);
}

// A read-only mapping of a whole file (the .idx image every device loads).
struct MappedFile {
    const void* data = nullptr;
    size_t size = 0;
    explicit MappedFile(const std::string& path) {
        const int fd = ::open(path.c_str(), O_RDONLY);
        if (fd < 0) throw CliError("no valid index path at " + path);
        struct stat sb {};
        if (::fstat(fd, &sb) != 0 || sb.st_size == 0) {
            ::close(fd);
            throw CliError("can not read index " + path);
        }
        size = (size_t)sb.st_size;
        void* p = ::mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0);
        ::close(fd);
        if (p == MAP_FAILED) throw CliError("can not map index " + path);
        (void)::madvise(p, size, MADV_WILLNEED);
        data = p;
    }
    ~MappedFile() {
        if (data) ::munmap(const_cast<void*>(data), size);
    }
    MappedFile(const MappedFile&) = delete;
    MappedFile& operator=(const MappedFile&) = delete;
};

// Reads in a FASTA file and their length, estimated from its first 256 KB
// and its size (sahara_gpu_prepare's sizes; 0 when unknown). Errs high.
struct QueryEstimate {
    uint64_t reads = 0;
    uint32_t len = 0;
};
QueryEstimate estimateQueries(const std::string& path) {
    QueryEstimate q;
    struct stat sb {};
    if (::stat(path.c_str(), &sb) != 0 || sb.st_size <= 0) return q;
    std::ifstream f(path, std::ios::binary);
    std::vector<char> buf(256u << 10);
    f.read(buf.data(), (std::streamsize)buf.size());
    const size_t n = (size_t)f.gcount();
    std::vector<size_t> heads;  // '>' at line starts
    for (size_t i = 0; i < n; ++i)
        if (buf[i] == '>' && (i == 0 || buf[i - 1] == '\n')) heads.push_back(i);
    if (heads.size() < 2) return q;
    const double perRec = (double)(heads.back() - heads[0]) / (double)(heads.size() - 1);
    size_t i = heads[0];
    while (i < heads[1] && buf[i] != '\n') ++i;  // the first header line
    for (; i < heads[1]; ++i)
        if (buf[i] != '\n' && buf[i] != '\r') ++q.len;
    q.reads = (uint64_t)((double)sb.st_size / perRec * 1.05) + 16;
    return q;
}

uint64_t readSigma(const std::string& path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw CliError("no valid index path at " + path);
    uint64_t s = 0;
    f.read(reinterpret_cast<char*>(&s), 8);
    if (!f) throw CliError("can not read index " + path);
    return s;
}

// fmt's "{}" for a double: shortest round-trip representation
std::string shortest(double v) {
    char b[64];
    auto r = std::to_chars(b, b + sizeof(b), v);
    return std::string(b, r.ptr);
}

struct Scheme {
    std::vector<uint32_t> pi, l, u;
    uint32_t n = 0;
};

Scheme makeScheme(const std::string& gen, int minK, int maxK, uint32_t len, bool hamming) {
    Scheme s;
    int n = sahara_scheme(gen.c_str(), minK, maxK, len, hamming ? 1 : 0, nullptr, nullptr, nullptr, 0);
    if (n < 0) throw CliError("cannot expand search scheme " + gen + " to length " + std::to_string(len));
    s.n = (uint32_t)n;
    s.pi.resize((size_t)n * len);
    s.l.resize((size_t)n * len);
    s.u.resize((size_t)n * len);
    if (sahara_scheme(gen.c_str(), minK, maxK, len, hamming ? 1 : 0, s.pi.data(), s.l.data(), s.u.data(), n) != n)
        throw CliError("cannot expand search scheme " + gen + " to length " + std::to_string(len));
    return s;
}

int cmdSearch(int argc, char** argv) {
    Opt query{{"-q", "--query"}}, index{{"-i", "--index"}}, output{{"-o", "--output"}, false, "sahara-output.txt"};
    Opt gen{{"-g", "--generator"}, false, "h2-k2"}, dyn{{"--dynamic_generator"}, true};
    Opt errors{{"-e", "--errors"}, false, "0"}, noRev{{"--no-reverse"}, true};
    Opt mode{{"-m", "--search_mode"}, false, "all"}, dist{{"-d", "--distance-metric"}, false, "lev"};
    Opt maxHits{{"--max_hits"}, false, "0"}, limit{{"--limit_queries"}};
    Opt gpus{{"--gpus"}, false, "1"}, emitErr{{"--emit-errors"}, true}, fmOnly{{"--fm-only"}, true};
    Parser p;
    for (Opt* o : {&query, &index, &output, &gen, &dyn, &errors, &noRev, &mode, &dist, &maxHits, &limit, &gpus,
                   &emitErr, &fmOnly})
        p.add(*o);
    p.parse(argc, argv, 2);
    if (!p.positional.empty()) throw CliError("unexpected argument " + p.positional[0]);
    if (!query.given) throw CliError("option -q/--query is required");
    if (!index.given) throw CliError("option -i/--index is required");
    if (mode.value != "all" && mode.value != "besthits") throw CliError("invalid value for --search_mode: " + mode.value);
    if (dist.value != "ham" && dist.value != "lev") throw CliError("invalid value for --distance-metric: " + dist.value);
    const bool besthits = mode.value == "besthits";
    const bool edit = dist.value == "lev";
    const int k = (int)toU64(errors.value, "--errors");
    const long mh = std::strtol(maxHits.value.c_str(), nullptr, 10);
    const uint32_t ngpu = (uint32_t)std::max<uint64_t>(1, toU64(gpus.value, "--gpus"));

    // sigma dispatch (search.cpp:276-291)
    const uint64_t sigma = readSigma(index.value);
    if (sigma != 5 && sigma != 6) throw CliError("unknown index with " + std::to_string(sigma) + " letters");

    std::vector<std::tuple<std::string, double>> timing;
    StopWatch sw;

    // index residency (search.cpp:162-169): one context per device, the
    // devices loading the one mapped .idx image side by side, beside the query
    // ingest below (the ingest runs on host threads, the load is DMA)
    std::vector<void*> ctx(ngpu, nullptr);
    std::vector<double> devLoad(ngpu, 0.0);
    std::vector<std::string> loadErrs(ngpu);
    struct Loaders {
        MappedFile img;
        std::vector<std::thread> th;
        std::vector<void*>& ctx;
        Loaders(const std::string& path, std::vector<void*>& c) : img(path), ctx(c) {}
        void join() {
            for (auto& t : th)
                if (t.joinable()) t.join();
        }
        ~Loaders() {  // also on an exception: the contexts close after their loads end
            join();
            for (void*& c : ctx) {
                sahara_gpu_close(c);
                c = nullptr;
            }
        }
    } L(index.value, ctx);
    // The search call's one-time work (the pinned hit sink, the pass's device
    // buffers) happens here too, beside the ingest, sized by an estimate of
    // the queries (sahara_gpu_prepare): the sink is pinned while the index
    // loads, the buffers once it is resident. Compact records only, <= 2
    // devices (the library's pool keeps two idle sinks).
    const bool prepare = !besthits && mh <= 0 && ngpu <= 2;
    const QueryEstimate qe = prepare ? estimateQueries(query.value) : QueryEstimate{};
    uint64_t npatEst = (noRev.given ? 1 : 2) * qe.reads;
    if (limit.given) npatEst = std::min<uint64_t>(npatEst, toU64(limit.value, "--limit_queries"));
    npatEst = (npatEst + ngpu - 1) / ngpu + 2;
    std::shared_future<void> pinned;
    if (qe.reads) pinned = std::async(std::launch::async, [npatEst] { (void)sahara_gpu_prepare(nullptr, npatEst, 0); }).share();
    const auto loadStart = std::chrono::steady_clock::now();
    for (uint32_t g = 0; g < ngpu; ++g)
        L.th.emplace_back([&, g] {
            if (sahara_gpu_open((int)g, L.img.data, L.img.size, &ctx[g]) != 0) loadErrs[g] = sahara_gpu_last_error();
            devLoad[g] = std::chrono::duration<double>(std::chrono::steady_clock::now() - loadStart).count();
            if (qe.reads && ctx[g]) {
                pinned.wait();
                (void)sahara_gpu_prepare(ctx[g], npatEst, qe.len);  // a failure only costs the call its time
            }
        });

    // queries (search.cpp:111-130): parsed and verified on the host (parallel
    // whole-file ingest) straight into two bits per symbol with the N
    // positions listed (besthits: one rank per byte); the reverse-complement
    // interleave and --limit_queries cut happen on the device
    // (sahara_gpu_search_packed[_compact]), so only the packed reads cross
    // PCIe. Query numbers in messages count the interleaved list.
    // (the library's ingest, sahara_read_fasta: the 2-bit form lands in
    // page-locked memory, which the search calls DMA without a copy)
    const unsigned nt = hostThreads();
    const bool packedIn = !besthits;
    struct Queries {
        sahara_fasta f{};
        ~Queries() { sahara_free_fasta(&f); }
        size_t records() const { return f.n_records; }
    } Q;
    check(sahara_read_fasta(query.value.c_str(), (uint32_t)sigma, packedIn ? 2 : 1, nt, &Q.f), "reading queries");
    const size_t nrec = Q.records();
    const size_t per = noRev.given ? 1 : 2;  // patterns per read
    if (Q.f.bad) {
        const unsigned char ch = (unsigned char)Q.f.bad_char;
        throw CliError(fmtStr("query '%s' (%zu) has invalid character at position %ld '%c'(%x)", Q.f.bad_id,
                              per * (size_t)Q.f.bad_record + 1, (long)Q.f.bad_pos, ch, ch));
    }
    size_t nq = per * nrec;  // the interleaved query list, cut by --limit_queries
    if (limit.given) nq = std::min<size_t>(toU64(limit.value, "--limit_queries"), nq);
    if (nq == 0) throw CliError("query file " + query.value + " was empty - abort\n");
    const size_t nreads = (nq + per - 1) / per;  // reads that contribute a query
    timing.emplace_back("ld queries", sw.reset());

    std::printf(
        "config:\n"
        "  query:               %s\n"
        "  index:               %s\n"
        "  generator:           %s\n"
        "  dynamic expansion:   %s\n"
        "  allowed errors:      %d\n"
        "  reverse complements: %s\n"
        "  search mode:         %s\n"
        "  max hits:            %ld\n"
        "  output path:         %s\n",
        query.value.c_str(), index.value.c_str(), gen.value.c_str(), dyn.given ? "true" : "false", k,
        noRev.given ? "false" : "true", besthits ? "besthits" : "all", mh, output.value.c_str());
    {
        const size_t fwd = nq / per;
        std::printf("fwd queries: %zu\nbwd queries: %zu\n", fwd, nq - fwd);
    }
    std::fflush(stdout);

    // the index: whatever of its load the ingest did not hide
    L.join();
    for (uint32_t g = 0; g < ngpu; ++g)
        if (!loadErrs[g].empty()) throw CliError("loading index: " + loadErrs[g]);
    if (fmOnly.given)
        for (void* c : ctx) check(sahara_gpu_set_mode(c, 0, 0), "set mode");
    sahara_index_info info{};
    check(sahara_gpu_index_info(ctx[0], &info), "index info");
    timing.emplace_back("ld index", sw.reset());

    // scheme (search.cpp:174-212): one expansion for queries[0].size()
    {
        const char* names[64];
        int ng = sahara_scheme_generators(names, nullptr, 64);
        // the reference lists generator::all's keys, a map: sorted by name (search.cpp:177-181)
        std::vector<std::string> sorted(names, names + ng);
        std::sort(sorted.begin(), sorted.end());
        bool known = false;
        std::string all;
        for (size_t i = 0; i < sorted.size(); ++i) {
            known = known || gen.value == sorted[i];
            all += (i ? ", " : "") + sorted[i];
        }
        if (!known)
            throw CliError("unknown search scheme generetaror \"" + gen.value + "\", valid generators are: " + all);
    }
    const uint64_t* qoffs = Q.f.offs;
    const uint32_t len = (uint32_t)(qoffs[1] - qoffs[0]);
    for (size_t r = 0; r < nreads; ++r)
        if (qoffs[r + 1] - qoffs[r] != len)
            throw CliError(fmtStr("query %zu has length %zu, but all queries must have the length of the first "
                                  "(%u): sahara expands one search scheme for queries[0].size()",
                                  per * r, (size_t)(qoffs[r + 1] - qoffs[r]), len));
    const uint8_t* reads = Q.f.data;  // nreads x len, back to back (packedIn: 2-bit codes)

    std::vector<Scheme> schemes;  // all: [0..k]; besthits: one per exact error count j
    // --dynamic_generator: part sizes by weighted node count (search.cpp:192-195, 202-205)
    auto build = [&](int minK, int maxK, bool hamming, bool printPartition) {
        if (!dyn.given) return makeScheme(gen.value, minK, maxK, len, hamming);
        Scheme s;
        const int n = sahara_scheme_dynamic(gen.value.c_str(), minK, maxK, len, 0, edit ? 1 : 0, (int)sigma,
                                            (double)info.n, nullptr, 0, nullptr, nullptr, nullptr, 0);
        if (n < 0) throw CliError("cannot expand search scheme " + gen.value);
        std::vector<uint32_t> sizes(64);
        s.n = (uint32_t)n;
        s.pi.resize((size_t)n * len);
        s.l.resize((size_t)n * len);
        s.u.resize((size_t)n * len);
        if (sahara_scheme_dynamic(gen.value.c_str(), minK, maxK, len, hamming ? 1 : 0, edit ? 1 : 0, (int)sigma,
                                  (double)info.n, sizes.data(), 64, s.pi.data(), s.l.data(), s.u.data(), n) != n)
            throw CliError("cannot expand search scheme " + gen.value + " to length " + std::to_string(len));
        if (printPartition) {
            int P = 0;
            sahara_scheme_parts(gen.value.c_str(), minK, maxK, &P, nullptr, nullptr, nullptr, 0);
            std::string part = "[";
            for (int t = 0; t < P; ++t) part += (t ? ", " : "") + std::to_string(sizes[t]);
            std::printf("partition: %s]\n", part.c_str());
        }
        return s;
    };
    // each scheme's node counts right after it, as loadSearchScheme prints them
    // (search.cpp:186-212): on the expanded scheme, before limitToHamming
    auto add = [&](Scheme sch) {
        double nc = 0, wnc = 0;
        sahara_scheme_counts(sch.l.data(), sch.u.data(), sch.n, len, edit ? 1 : 0, (int)sigma, (double)info.n, &nc,
                             &wnc);
        std::printf("node count: %s\n", shortest(nc).c_str());
        std::printf("weighted node count: %s\n", shortest(wnc).c_str());
        schemes.push_back(std::move(sch));
    };
    if (!besthits) {
        add(build(0, k, false, true));
        // -d ham: the search runs on limitToHamming of that scheme (search.cpp:226)
        if (!edit) schemes.back() = build(0, k, true, false);
    } else {
        for (int j = 0; j <= k; ++j) add(build(j, j, false, true));
    }
    timing.emplace_back("searchScheme", sw.reset());

    // hits as compact records where they apply (all mode without --max_hits,
    // one index part, <= 15 errors; SAHARA_CLI_FULL_HITS=1: whole records)
    const char* fullEnv = std::getenv("SAHARA_CLI_FULL_HITS");
    const bool compactOut = !besthits && mh <= 0 && info.n_parts == 1 && k <= 15 && !(fullEnv && std::atoi(fullEnv));
    // search + locate (search.cpp:218-250), reads sharded over the devices
    // (a read and its reverse complement stay together; qids stay global)
    std::vector<HitPart> parts(ngpu);
    std::vector<double> devLocate(ngpu, 0.0), devSearch(ngpu, 0.0);
    std::vector<std::string> errs(ngpu);
    {
        std::vector<std::thread> th;
        for (uint32_t g = 0; g < ngpu; ++g) {
            th.emplace_back([&, g] {
                const QueryShard sh = queryShard(nq, per, ngpu, g);
                const size_t r0 = sh.r0, r1 = sh.r1, q0 = sh.q0, q1 = sh.q1;
                if (r0 == r1) return;
                const auto t0 = std::chrono::steady_clock::now();
                sahara_hit* hits = nullptr;
                uint64_t nh = 0;
                int rc;
                const uint32_t cap = (uint32_t)std::max(0L, mh);
                HitPart part;
                // the shard's reads: stream symbols [r0 * len, r1 * len) of the packed codes
                const uint64_t* npos = Q.f.n_count ? Q.f.n_pos : nullptr;
                const uint64_t ncount = Q.f.n_count;
                if (!besthits && compactOut) {  // 8-B records straight into host memory, decoded by writeHits
                    const Scheme& s = schemes[0];
                    rc = sahara_gpu_search_packed_compact(ctx[g], reads, (uint64_t)r0 * len, npos, ncount,
                                                          r1 - r0, len, noRev.given ? 0 : 1, q1 - q0, s.pi.data(),
                                                          s.l.data(), s.u.data(), s.n, edit ? 1 : 0, &part.blocks);
                    part.compact = rc == 0;
                    nh = part.blocks.n_hits;
                } else if (!besthits) {
                    const Scheme& s = schemes[0];
                    rc = sahara_gpu_search_packed(ctx[g], reads, (uint64_t)r0 * len, npos, ncount, r1 - r0, len,
                                                  noRev.given ? 0 : 1, q1 - q0, s.pi.data(), s.l.data(), s.u.data(),
                                                  s.n, edit ? 1 : 0, cap, &hits, &nh);
                } else {  // search_best takes the interleaved patterns
                    std::vector<uint8_t> pats((q1 - q0) * len);
                    for (size_t q = q0; q < q1; ++q) {
                        const uint8_t* src = reads + (q / per) * len;
                        uint8_t* dst = pats.data() + (q - q0) * len;
                        if (per == 2 && (q & 1)) {
                            for (uint32_t j = 0; j < len; ++j) dst[j] = complementRank(src[len - 1 - j], (uint32_t)sigma);
                        } else {
                            std::memcpy(dst, src, len);
                        }
                    }
                    std::vector<uint32_t> pi, l, u, ns;
                    for (const Scheme& s : schemes) {
                        pi.insert(pi.end(), s.pi.begin(), s.pi.end());
                        l.insert(l.end(), s.l.begin(), s.l.end());
                        u.insert(u.end(), s.u.begin(), s.u.end());
                        ns.push_back(s.n);
                    }
                    rc = sahara_gpu_search_best(ctx[g], pats.data(), q1 - q0, len, pi.data(), l.data(), u.data(),
                                                ns.data(), (uint32_t)ns.size(), cap, &hits, &nh);
                }
                if (rc != 0) {
                    errs[g] = sahara_gpu_last_error();
                    return;
                }
                sahara_stats st{};
                sahara_gpu_stats(ctx[g], &st);
                devLocate[g] = (st.locate_ms + st.sort_ms) / 1e3;
                devSearch[g] = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
                part.hits = hits;
                part.n = nh;
                part.qidOffset = q0;
                parts[g] = part;  // released after writing
            });
        }
        for (auto& t : th) t.join();
    }
    for (auto& e : errs)
        if (!e.empty()) {
            for (auto& hp : parts) hp.release();
            throw CliError("search: " + e);
        }
    double wall = sw.reset();
    const double loc = *std::max_element(devLocate.begin(), devLocate.end());
    timing.emplace_back("search", std::max(0.0, wall - loc));
    timing.emplace_back("locate", loc);

    uint64_t nhits = 0;
    for (auto& hp : parts) nhits += hp.n;
    writeHits(output.value, parts, emitErr.given, nt);
    for (auto& hp : parts) hp.release();
    timing.emplace_back("result", sw.reset());
    for (void*& c : ctx) {
        sahara_gpu_close(c);
        c = nullptr;
    }

    std::printf("stats:\n");
    double total = 0;
    for (auto& [key, t] : timing) {
        std::printf("  %-20s %10.2fs\n", (key + " time:").c_str(), t);
        total += t;
    }
    std::printf("  total time:          %10.2fs\n", total);
    std::printf("  queries per second:  %10.0fq/s\n", (double)nq / total);
    std::printf("  number of hits:      %10llu\n", (unsigned long long)nhits);
    // the index loads beside the query ingest: "ld index" above is the part of
    // its load the ingest did not hide; this is its whole load
    std::printf("  index load:          %10.2fs (beside ld queries)\n",
                *std::max_element(devLoad.begin(), devLoad.end()));
    if (ngpu > 1)  // --gpus N: each device's index load and search (an imbalance shows by name)
        for (uint32_t g = 0; g < ngpu; ++g)
            std::printf("  device %u:            ld index %.2fs, search %.2fs, hits %llu\n", g, devLoad[g],
                        devSearch[g], (unsigned long long)parts[g].n);
    return 0;
}

// `sahara read_simulator` (src/sahara/read_simulator.cpp:13-82)
int cmdReadSimulator(int argc, char** argv) {
    Opt input{{"-i", "--input"}}, output{{"-o", "--output"}}, width{{"--fasta_line_length"}, false, "80"};
    Opt len{{"-l", "--read_length"}, false, "150"}, n{{"-n", "--number_of_reads"}, false, "1000"};
    Opt sub{{"--substitution_errors"}, false, "0"}, ins{{"--insertion_errors"}, false, "0"};
    Opt del{{"--deletion_errors"}, false, "0"}, err{{"-e", "--errors"}, false, "0"}, seed{{"--seed"}, false, "0"};
    Parser p;
    for (Opt* o : {&input, &output, &width, &len, &n, &sub, &ins, &del, &err, &seed}) p.add(*o);
    p.parse(argc, argv, 2);
    if (!p.positional.empty()) throw CliError("unexpected argument " + p.positional[0]);
    if (!output.given) throw CliError("option -o/--output is required");
    ReadSimulatorArgs a;
    a.haveInput = input.given;
    a.input = input.value;
    a.output = output.value;
    a.lineLength = toU64(width.value, "--fasta_line_length");
    a.readLength = toU64(len.value, "--read_length");
    a.nreads = toU64(n.value, "--number_of_reads");
    a.sub = toU64(sub.value, "--substitution_errors");
    a.ins = toU64(ins.value, "--insertion_errors");
    a.del = toU64(del.value, "--deletion_errors");
    a.errors = toU64(err.value, "--errors");
    a.seed = (uint32_t)toU64(seed.value, "--seed");
    return runReadSimulator(a);
}

void help() {
    std::printf(
        "sahara - readmapper (MI355X build)\n"
        "  sahara index <fasta> [--ignore_unknown] [--dna4] [--gpu N]\n"
        "  sahara search -q <fasta> -i <index> [-o <out>] [-g <generator>] [-e <k>] [--no-reverse]\n"
        "                [-m all|besthits] [-d ham|lev] [--max_hits <n>] [--limit_queries <n>]\n"
        "                [--gpus <N>] [--emit-errors] [--fm-only]\n"
        "  sahara read_simulator -o <fasta> [-i <reference>] [-l <len>] [-n <reads>] [-e <errors>]\n"
        "                [--substitution_errors n] [--insertion_errors n] [--deletion_errors n]\n"
        "                [--fasta_line_length n] [--seed s]\n"
        "  sahara search_scheme list-generators\n");
}

}  // namespace

int main(int argc, char** argv) {
    // six streams per device context: their own hardware queues (HIP's default
    // is 4 per process), set before the first HIP call
    setenv("GPU_MAX_HW_QUEUES", "8", 0);
    try {
        if (argc < 2 || !std::strcmp(argv[1], "--help") || !std::strcmp(argv[1], "-h")) {
            help();
            return argc < 2 ? 1 : 0;
        }
        const std::string cmd = argv[1];
        if (cmd == "index") return cmdIndex(argc, argv);
        if (cmd == "search") return cmdSearch(argc, argv);
        if (cmd == "read_simulator") return cmdReadSimulator(argc, argv);
        if (cmd == "search_scheme" && argc >= 3 && std::string(argv[2]) == "list-generators") {
            const char* names[64];
            const char* descs[64];
            int n = sahara_scheme_generators(names, descs, 64);
            for (int i = 0; i < n; ++i) std::printf("%15s - %s\n", names[i], descs[i]);
            return 0;
        }
        throw CliError("unknown command " + cmd);
    } catch (const std::exception& e) {
        std::fflush(stdout);
        std::fprintf(stderr, "%s\n", e.what());
        return 1;
    }
}
