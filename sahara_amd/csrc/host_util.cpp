// host_util.cpp — .idx I/O, the synthetic read generator and the FASTA
// query ingest (host side).
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <mutex>
#include <thread>
#include <unordered_set>

#include <hip/hip_runtime.h>

#include "../../include/sahara_hip.h"
#include "device_index.h"
#include "fasta.h"
#include "idx_format.h"

namespace sahara {

std::vector<uint8_t> readFile(const std::string& path) {
    std::ifstream f(path, std::ios::binary | std::ios::ate);
    if (!f) throw Error("no valid index path at " + path);
    const std::streamsize sz = f.tellg();
    f.seekg(0);
    std::vector<uint8_t> buf((size_t)sz);
    if (sz && !f.read(reinterpret_cast<char*>(buf.data()), sz)) throw Error("cannot read " + path);
    return buf;
}

namespace {
struct Reader {
    const uint8_t* p;
    const uint8_t* end;
    template <typename T> T get() {
        if ((size_t)(end - p) < sizeof(T)) throw Error("truncated .idx file");
        T v;
        std::memcpy(&v, p, sizeof(T));
        p += sizeof(T);
        return v;
    }
    template <typename T> const T* vec(uint64_t& n) {
        n = get<uint64_t>();
        if (n > (uint64_t)(end - p) / sizeof(T)) throw Error("truncated .idx file");
        const T* r = reinterpret_cast<const T*>(p);
        p += n * sizeof(T);
        return r;
    }
};
}  // namespace

IdxParts parseIdx(const uint8_t* buf, size_t bytes) {
    Reader r{buf, buf + bytes};
    IdxParts P;
    const uint64_t sigma = r.get<uint64_t>();
    if (sigma != 5 && sigma != 6) throw Error("unknown index with " + std::to_string(sigma) + " letters");
    if (r.get<uint64_t>() != kIdxMagic) throw Error("not a sahara-amd .idx file (payload magic mismatch)");
    P.sigma = (uint32_t)sigma;
    P.n = r.get<uint64_t>();
    for (uint64_t c = 0; c <= sigma; ++c) P.C[c] = r.get<uint64_t>();
    uint64_t nrec = 0, nf = 0, nr = 0, ns = 0;
    const uint64_t* rl = r.vec<uint64_t>(nrec);
    P.recLens.assign(rl, rl + nrec);
    P.rate = (uint32_t)r.get<uint64_t>();
    P.bwtF = r.vec<uint8_t>(nf);
    P.bwtR = r.vec<uint8_t>(nr);
    // the u64/u32 vectors follow the n-byte BWTs, so they are in general NOT
    // 8/4-aligned in the image (nor is a part of a multi-part file): treat
    // sampled / samples as raw bytes — they are only ever memcpy'd / copied to
    // the device (buildFromParts, cpuParts), never dereferenced as typed
    P.sampled = r.vec<uint64_t>(ns);
    P.samples = r.vec<uint32_t>(P.nsamples);
    if (nf != P.n || nr != P.n || ns != P.n / 64 + 1) throw Error("inconsistent .idx payload sizes");
    uint64_t tot = 0;
    for (uint64_t x : P.recLens) tot += x + 1;
    if (tot != P.n) throw Error("record lengths do not match index size");
    return P;
}

std::vector<IdxParts> parseIdxAll(const uint8_t* buf, size_t bytes) {
    Reader r{buf, buf + bytes};
    const uint64_t sigma = r.get<uint64_t>();
    if (sigma != 5 && sigma != 6) throw Error("unknown index with " + std::to_string(sigma) + " letters");
    const uint64_t magic = r.get<uint64_t>();
    if (magic == kIdxMagic) return {parseIdx(buf, bytes)};
    if (magic != kIdxPartsMagic) throw Error("not a sahara-amd .idx file (payload magic mismatch)");
    const uint64_t np = r.get<uint64_t>();
    if (np == 0 || np > 4096) throw Error("implausible number of index parts: " + std::to_string(np));
    std::vector<IdxParts> out;
    for (uint64_t i = 0; i < np; ++i) {
        const uint64_t len = r.get<uint64_t>();
        if (len > (uint64_t)(r.end - r.p)) throw Error("truncated .idx file");
        out.push_back(parseIdx(r.p, len));
        if (out.back().sigma != sigma) throw Error("index parts disagree on sigma");
        r.p += len;
    }
    if (r.p != r.end) throw Error("trailing bytes after the index parts");
    return out;
}

namespace {
uint64_t idxBytes(const IdxParts& P) {
    // sigma, magic, n, C[], recLens (count + entries), rate; both BWTs, sampled bits, samples (count + data)
    return 8 * (3 + (P.sigma + 1) + 1 + P.recLens.size() + 1) + 2 * (8 + P.n) + 8 + 8 * (P.n / 64 + 1) + 8 +
           4 * P.nsamples;
}
void writeIdxTo(std::ostream& o, const IdxParts& P);
}  // namespace

void writeIdxAll(const std::string& path, const std::vector<IdxParts>& parts) {
    if (parts.size() == 1) return writeIdx(path, parts[0]);
    std::ofstream o(path, std::ios::binary);
    if (!o) throw Error("cannot write " + path);
    auto put = [&](uint64_t v) { o.write(reinterpret_cast<const char*>(&v), 8); };
    put(parts.at(0).sigma);
    put(kIdxPartsMagic);
    put(parts.size());
    for (const IdxParts& P : parts) {
        put(idxBytes(P));
        writeIdxTo(o, P);
    }
    if (!o) throw Error("write failed: " + path);
}

void writeIdx(const std::string& path, const IdxParts& P) {
    std::ofstream o(path, std::ios::binary);
    if (!o) throw Error("cannot write " + path);
    writeIdxTo(o, P);
    if (!o) throw Error("write failed: " + path);
}

namespace {
void writeIdxTo(std::ostream& o, const IdxParts& P) {
    auto put = [&](uint64_t v) { o.write(reinterpret_cast<const char*>(&v), 8); };
    put(P.sigma);
    put(kIdxMagic);
    put(P.n);
    for (uint32_t c = 0; c <= P.sigma; ++c) put(P.C[c]);
    put(P.recLens.size());
    o.write(reinterpret_cast<const char*>(P.recLens.data()), (std::streamsize)(P.recLens.size() * 8));
    put(P.rate);
    put(P.n);
    o.write(reinterpret_cast<const char*>(P.bwtF), (std::streamsize)P.n);
    put(P.n);
    o.write(reinterpret_cast<const char*>(P.bwtR), (std::streamsize)P.n);
    put(P.n / 64 + 1);
    o.write(reinterpret_cast<const char*>(P.sampled), (std::streamsize)((P.n / 64 + 1) * 8));
    put(P.nsamples);
    o.write(reinterpret_cast<const char*>(P.samples), (std::streamsize)(P.nsamples * 4));
}
}  // namespace

uint64_t readIdxSigma(const std::string& path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw Error("no valid index path at " + path);
    uint64_t s = 0;
    f.read(reinterpret_cast<char*>(&s), 8);
    if (!f) throw Error("cannot read " + path);
    return s;
}

// --------------------------------------------------------------- reads ----
// read_simulator.cpp:119-240 restated with a counter-based generator so reads
// can be produced in parallel and still depend only on (seed, read index):
//   per error, the type is S/I/D with probability 1/3 each (:258-267);
//   S turns a random 'M' of the transcript into 'S' (:129-136), I turns a
//   random 'M' into 'I' (:138-145), D inserts a 'D' at a random slot (:147-150);
//   the reference span (len - #I + #D) is sampled uniformly inside one record;
//   S writes one of the three other bases, I a random base, D skips a
//   reference base (:204-240). Reads therefore always have exactly `len` bases.
namespace {
struct Xoshiro {
    uint64_t s[4];
    static uint64_t splitmix(uint64_t& x) {
        uint64_t z = (x += 0x9e3779b97f4a7c15ull);
        z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
        z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
        return z ^ (z >> 31);
    }
    explicit Xoshiro(uint64_t seed) {
        for (auto& v : s) v = splitmix(seed);
    }
    static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
    uint64_t operator()() {
        const uint64_t r = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
        s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3]; s[2] ^= t; s[3] = rotl(s[3], 45);
        return r;
    }
    uint64_t below(uint64_t n) { return n ? (*this)() % n : 0; }
};
}  // namespace

void synthReads(const uint8_t* ranks, const uint64_t* recLens, uint64_t nrec, uint32_t sigma, uint64_t nreads,
                uint32_t len, uint32_t subs, uint32_t ins, uint32_t dels, uint32_t errors, uint64_t seed, uint8_t* out,
                uint64_t* origin) {
    if (sigma != 5 && sigma != 6) throw Error("sigma must be 5 or 6");
    if (len == 0) throw Error("read length must be > 0");
    const uint8_t code[4] = {1, 2, 3, (uint8_t)(sigma == 6 ? 5 : 4)};
    auto toIdx = [&](uint8_t r) -> int { return r == 1 ? 0 : r == 2 ? 1 : r == 3 ? 2 : 3; };
    std::vector<uint64_t> starts(nrec + 1, 0);
    for (uint64_t r = 0; r < nrec; ++r) starts[r + 1] = starts[r] + recLens[r];
    const uint64_t total = starts[nrec];
    if (total == 0) throw Error("empty reference");
    const unsigned nth = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::vector<std::thread> th;
    std::vector<std::string> errs(nth);
    for (unsigned t = 0; t < nth; ++t) {
        th.emplace_back([&, t] {
            std::vector<char> tr;
            for (uint64_t i = nreads * t / nth; i < nreads * (t + 1) / nth; ++i) {
                Xoshiro g(seed * 0x100000001b3ull + i);
                uint32_t ns = subs, ni = ins, nd = dels;
                for (uint32_t e = 0; e < errors; ++e) {
                    const uint64_t k = g.below(3);
                    ns += k == 0; ni += k == 1; nd += k == 2;
                }
                if (ns + ni > len) { errs[t] = "more substitutions+insertions than read length"; return; }
                tr.assign(len, 'M');
                auto pickM = [&](char to) {
                    for (;;) {
                        const uint64_t p = g.below(tr.size());
                        if (tr[p] == 'M') { tr[p] = to; return; }
                    }
                };
                for (uint32_t k = 0; k < ns; ++k) pickM('S');
                for (uint32_t k = 0; k < ni; ++k) pickM('I');
                for (uint32_t k = 0; k < nd; ++k) tr.insert(tr.begin() + (long)g.below(tr.size() + 1), 'D');
                const uint64_t span = (uint64_t)len - ni + nd;
                uint64_t rec = 0, pos = 0;
                for (int tries = 0;; ++tries) {
                    if (tries > 1000000) { errs[t] = "no record long enough for the reads"; return; }
                    const uint64_t gp = g.below(total);
                    rec = (uint64_t)(std::upper_bound(starts.begin(), starts.end(), gp) - starts.begin()) - 1;
                    pos = gp - starts[rec];
                    if (pos + span <= recLens[rec]) break;
                }
                const uint8_t* ref = ranks + starts[rec] + pos;
                uint8_t* o = out + i * len;
                uint64_t p = 0, w = 0;
                for (char c : tr) {
                    switch (c) {
                        case 'M': o[w++] = ref[p++]; break;
                        case 'S': o[w++] = code[(toIdx(ref[p++]) + 1 + (int)g.below(3)) % 4]; break;
                        case 'I': o[w++] = code[g.below(4)]; break;
                        default: ++p; break;  // 'D'
                    }
                }
                if (origin) { origin[2 * i] = rec; origin[2 * i + 1] = pos; }
            }
        });
    }
    for (auto& x : th) x.join();
    for (auto& e : errs)
        if (!e.empty()) throw Error(e);
}

}  // namespace sahara

namespace sahara {
extern thread_local std::string g_err;  // sahara_gpu_last_error (capi.cpp)
}

// ------------------------------------------------------------ FASTA ingest --
// sahara_read_fasta: search.cpp:111-130's query ingest (ivio::fasta::reader,
// ivs::convert_char_to_rank, ivs::verify_rank) on the host's threads, in one
// of the two forms the search calls take (fasta.h parseFastaParallel).
namespace {
template <typename T>
T* copyOut(const std::vector<T>& v) {
    T* p = static_cast<T*>(std::malloc(std::max<size_t>(v.size(), 1) * sizeof(T)));
    if (!p) throw sahara::Error("out of host memory for FASTA data");
    if (!v.empty()) std::memcpy(p, v.data(), v.size() * sizeof(T));
    return p;
}
// the form-2 buffers sahara_read_fasta page-locked (hipHostMalloc), so that
// sahara_free_fasta frees each the way it was allocated without asking HIP
std::mutex g_pinnedFastaMu;
std::unordered_set<void*> g_pinnedFasta;
void rememberPinnedFasta(void* p) {
    std::lock_guard<std::mutex> g(g_pinnedFastaMu);
    g_pinnedFasta.insert(p);
}
bool forgetPinnedFasta(void* p) {
    std::lock_guard<std::mutex> g(g_pinnedFastaMu);
    return g_pinnedFasta.erase(p) != 0;
}
}  // namespace

extern "C" {

int sahara_read_fasta(const char* path, uint32_t sigma, int form, uint32_t threads, sahara_fasta* out) {
    try {
        if (!out || !path) throw sahara::Error("sahara_read_fasta: null argument");
        *out = sahara_fasta{};
        if (sigma != 5 && sigma != 6) throw sahara::Error("sigma must be 5 or 6");
        if (form != 1 && form != 2) throw sahara::Error("form must be 1 (ranks) or 2 (two bits per symbol)");
        const unsigned nt = threads ? threads : sahara_io::hostThreads();
        // the two-bit form is written straight into page-locked memory (the
        // packed search calls DMA it as it is), pinned beside the parse's
        // first pass; pageable if pinning fails (the calls then copy it
        // through their staging ring)
        sahara_io::CodesAlloc pinnedCodes;
        pinnedCodes.alloc = [](size_t bytes) -> uint8_t* {
            void* p = nullptr;
            if (hipHostMalloc(&p, std::max<size_t>(bytes, 1), hipHostMallocPortable) != hipSuccess || !p) {
                (void)hipGetLastError();
                return static_cast<uint8_t*>(std::malloc(std::max<size_t>(bytes, 1)));
            }
            rememberPinnedFasta(p);
            return static_cast<uint8_t*>(p);
        };
        pinnedCodes.release = [](uint8_t* p) {
            if (forgetPinnedFasta(p)) (void)hipHostFree(p);
            else std::free(p);
        };
        sahara_io::FastaData D = sahara_io::parseFastaParallel(
            path, sigma, nt, 8u << 20, form == 2 ? sahara_io::FastaForm::kCodes2 : sahara_io::FastaForm::kRanks,
            form == 2 ? &pinnedCodes : nullptr);
        if (form == 2) {
            out->data = D.codes ? D.codes : copyOut(D.ranks);
        } else {
            out->data = copyOut(D.ranks);
        }
        out->offs = copyOut(D.offs);
        out->n_pos = copyOut(D.nPos);
        out->n_symbols = D.symbols;
        out->n_records = D.records();
        out->n_count = D.nPos.size();
        out->bad = D.bad ? 1 : 0;
        out->bad_record = D.badRecord;
        out->bad_pos = D.badPos;
        out->bad_char = D.badChar;
        std::vector<char> id(D.badId.begin(), D.badId.end());
        id.push_back(0);
        out->bad_id = copyOut(id);
        return 0;
    } catch (const std::exception& e) {
        if (out) sahara_free_fasta(out);
        sahara::g_err = e.what();
    }
    return -1;
}

void sahara_free_fasta(sahara_fasta* f) {
    if (!f) return;
    // freed the way sahara_read_fasta allocated it (recorded there): no HIP
    // call for a rank-form (CPU-only) ingest
    if (f->data && forgetPinnedFasta(f->data)) (void)hipHostFree(f->data);
    else std::free(f->data);
    std::free(f->offs);
    std::free(f->n_pos);
    std::free(f->bad_id);
    *f = sahara_fasta{};
}

}  // extern "C"
