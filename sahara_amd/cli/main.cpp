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
#include <charconv>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstdarg>
#include <cstring>
#include <fstream>
#include <functional>
#include <map>
#include <stdexcept>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "../../include/sahara_hip.h"
#include "fasta.h"

using namespace sahara_cli;

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

    std::vector<uint8_t> ranks;
    std::vector<uint64_t> lens;
    uint64_t totalSize = 0;
    {
        FastaReader rd(path);
        Record rec;
        size_t n = 0;
        while (rd.next(rec)) {
            ++n;
            totalSize += rec.seq.size();
            std::vector<uint8_t> r = toRanks(rec.seq, sigma);
            if (ignore.given) {  // index.cpp:56-68
                for (auto& v : r) {
                    if (v != 255 && v != 0 && v < sigma) continue;
                    v = dna4.given ? (uint8_t)(1 + std::rand() % 4) : (uint8_t)4;
                }
            }
            if (long pos = firstInvalid(r, sigma); pos >= 0) {
                const unsigned char ch = (unsigned char)rec.seq[(size_t)pos];
                throw CliError(fmtStr("ref '%s' (%zu) has invalid character '%c' (0x%02x) at position %ld",
                                      rec.id.c_str(), n, ch, ch, pos));
            }
            ranks.insert(ranks.end(), r.begin(), r.end());
            lens.push_back(r.size());
        }
    }
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

// Fast text output of hits: "qid seqId pos[ e]\n" (search.cpp:254-261).
void writeHits(const std::string& path, const std::vector<std::vector<sahara_hit>>& parts, bool emitErrors) {
    std::FILE* f = std::fopen(path.c_str(), "w");
    if (!f) throw CliError("can not open output file " + path);
    std::vector<char> buf(1 << 22);
    size_t used = 0;
    auto put = [&](uint64_t v) {
        auto r = std::to_chars(buf.data() + used, buf.data() + buf.size(), v);
        used = (size_t)(r.ptr - buf.data());
    };
    for (const auto& hits : parts) {
        for (const sahara_hit& h : hits) {
            if (used + 96 > buf.size()) {
                std::fwrite(buf.data(), 1, used, f);
                used = 0;
            }
            put(h.qid);
            buf[used++] = ' ';
            put(h.seq_id);
            buf[used++] = ' ';
            put(h.pos);
            if (emitErrors) {
                buf[used++] = ' ';
                put(h.err);
            }
            buf[used++] = '\n';
        }
    }
    std::fwrite(buf.data(), 1, used, f);
    std::fclose(f);
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

    // queries (search.cpp:111-130): ranks, verification, RC interleave, limit
    std::vector<std::vector<uint8_t>> queries;
    {
        FastaReader rd(query.value);
        Record rec;
        while (rd.next(rec)) {
            queries.emplace_back(toRanks(rec.seq, (uint32_t)sigma));
            if (long pos = firstInvalid(queries.back(), (uint32_t)sigma); pos >= 0) {
                const unsigned char ch = (unsigned char)rec.seq[(size_t)pos];
                throw CliError(fmtStr("query '%s' (%zu) has invalid character at position %ld '%c'(%x)",
                                      rec.id.c_str(), queries.size(), pos, ch, ch));
            }
            if (!noRev.given) queries.emplace_back(reverseComplement(queries.back(), (uint32_t)sigma));
        }
    }
    if (limit.given) queries.resize(std::min<size_t>(toU64(limit.value, "--limit_queries"), queries.size()));
    if (queries.empty()) throw CliError("query file " + query.value + " was empty - abort\n");
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
        const size_t fwd = queries.size() / (noRev.given ? 1 : 2);
        std::printf("fwd queries: %zu\nbwd queries: %zu\n", fwd, queries.size() - fwd);
    }
    std::fflush(stdout);

    // index residency (search.cpp:162-169): one context per device
    std::vector<void*> ctx(ngpu, nullptr);
    for (uint32_t g = 0; g < ngpu; ++g) check(sahara_gpu_open_file((int)g, index.value.c_str(), &ctx[g]), "loading index");
    if (fmOnly.given)
        for (void* c : ctx) check(sahara_gpu_set_mode(c, 0, 0), "set mode");
    sahara_index_info info{};
    check(sahara_gpu_index_info(ctx[0], &info), "index info");
    timing.emplace_back("ld index", sw.reset());

    // scheme (search.cpp:174-212): one expansion for queries[0].size()
    {
        const char* names[64];
        int ng = sahara_scheme_generators(names, nullptr, 64);
        bool known = false;
        std::string all;
        for (int i = 0; i < ng; ++i) {
            known = known || gen.value == names[i];
            all += (i ? ", " : "") + std::string(names[i]);
        }
        if (!known)
            throw CliError("unknown search scheme generetaror \"" + gen.value + "\", valid generators are: " + all);
    }
    const uint32_t len = (uint32_t)queries[0].size();
    for (size_t i = 0; i < queries.size(); ++i)
        if (queries[i].size() != len)
            throw CliError(fmtStr("query %zu has length %zu, but all queries must have the length of the first "
                                  "(%u): sahara expands one search scheme for queries[0].size()",
                                  i, queries[i].size(), len));
    std::vector<uint8_t> flat;
    flat.reserve(queries.size() * len);
    for (auto& q : queries) flat.insert(flat.end(), q.begin(), q.end());
    const size_t nq = queries.size();
    std::vector<std::vector<uint8_t>>().swap(queries);

    std::vector<Scheme> schemes;  // all: [0..k]; besthits: one per exact error count j
    // --dynamic_generator: part sizes by weighted node count (search.cpp:192-195, 202-205)
    auto build = [&](int minK, int maxK, bool hamming) {
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
        int P = 0;
        sahara_scheme_parts(gen.value.c_str(), minK, maxK, &P, nullptr, nullptr, nullptr, 0);
        std::string part = "[";
        for (int t = 0; t < P; ++t) part += (t ? ", " : "") + std::to_string(sizes[t]);
        std::printf("partition: %s]\n", part.c_str());
        return s;
    };
    // each scheme's node counts right after it, as loadSearchScheme prints them (search.cpp:186-212)
    auto add = [&](Scheme sch) {
        double nc = 0, wnc = 0;
        sahara_scheme_counts(sch.l.data(), sch.u.data(), sch.n, len, edit ? 1 : 0, (int)sigma, (double)info.n, &nc,
                             &wnc);
        std::printf("node count: %s\n", shortest(nc).c_str());
        std::printf("weighted node count: %s\n", shortest(wnc).c_str());
        schemes.push_back(std::move(sch));
    };
    if (!besthits) add(build(0, k, !edit));
    else
        for (int j = 0; j <= k; ++j) add(build(j, j, false));
    timing.emplace_back("searchScheme", sw.reset());

    // search + locate (search.cpp:218-250), queries sharded over the devices
    std::vector<std::vector<sahara_hit>> parts(ngpu);
    std::vector<double> devLocate(ngpu, 0.0);
    std::vector<std::string> errs(ngpu);
    {
        std::vector<std::thread> th;
        for (uint32_t g = 0; g < ngpu; ++g) {
            th.emplace_back([&, g] {
                const size_t q0 = nq * g / ngpu, q1 = nq * (g + 1) / ngpu;
                if (q0 == q1) return;
                sahara_hit* hits = nullptr;
                uint64_t nh = 0;
                int rc;
                const uint32_t cap = (uint32_t)std::max(0L, mh);
                if (!besthits) {
                    const Scheme& s = schemes[0];
                    rc = sahara_gpu_search(ctx[g], flat.data() + q0 * len, q1 - q0, len, s.pi.data(), s.l.data(),
                                           s.u.data(), s.n, edit ? 1 : 0, cap, &hits, &nh);
                } else {
                    std::vector<uint32_t> pi, l, u, ns;
                    for (const Scheme& s : schemes) {
                        pi.insert(pi.end(), s.pi.begin(), s.pi.end());
                        l.insert(l.end(), s.l.begin(), s.l.end());
                        u.insert(u.end(), s.u.begin(), s.u.end());
                        ns.push_back(s.n);
                    }
                    rc = sahara_gpu_search_best(ctx[g], flat.data() + q0 * len, q1 - q0, len, pi.data(), l.data(),
                                                u.data(), ns.data(), (uint32_t)ns.size(), cap, &hits, &nh);
                }
                if (rc != 0) {
                    errs[g] = sahara_gpu_last_error();
                    return;
                }
                sahara_stats st{};
                sahara_gpu_stats(ctx[g], &st);
                std::vector<sahara_hit> got(hits, hits + nh);
                sahara_gpu_free(hits);
                for (auto& h : got) h.qid += q0;
                devLocate[g] = (st.locate_ms + st.sort_ms) / 1e3;
                parts[g] = std::move(got);
            });
        }
        for (auto& t : th) t.join();
    }
    for (auto& e : errs)
        if (!e.empty()) throw CliError("search: " + e);
    double wall = sw.reset();
    const double loc = *std::max_element(devLocate.begin(), devLocate.end());
    timing.emplace_back("search", std::max(0.0, wall - loc));
    timing.emplace_back("locate", loc);

    uint64_t nhits = 0;
    for (auto& p2 : parts) nhits += p2.size();
    writeHits(output.value, parts, emitErr.given);
    timing.emplace_back("result", sw.reset());
    for (void* c : ctx) sahara_gpu_close(c);

    std::printf("stats:\n");
    double total = 0;
    for (auto& [key, t] : timing) {
        std::printf("  %-20s %10.2fs\n", (key + " time:").c_str(), t);
        total += t;
    }
    std::printf("  total time:          %10.2fs\n", total);
    std::printf("  queries per second:  %10.0fq/s\n", (double)nq / total);
    std::printf("  number of hits:      %10llu\n", (unsigned long long)nhits);
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
