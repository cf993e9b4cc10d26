// fasta.h — FASTA reading and rank conversion: the library's query ingest
// (sahara_read_fasta) and the `sahara` CLI's reference reader.
//
// Restates what the reference takes from ivio / ivsigma on this path:
//   ivio::fasta::reader            (search.cpp:115, index.cpp:53)
//   ivs::convert_char_to_rank<A>   (search.cpp:117, index.cpp:55)
//   ivs::verify_rank               (search.cpp:118, index.cpp:69)
//   ivs::reverse_complement_rank   (search.cpp:122)
// Alphabets: d_dna5 = {$, A, C, G, N, T} (sigma 6),
// d_dna4 = {$, A, C, G, T} (sigma 5); lower case maps like upper case; every
// other character is invalid (rank 255).
#pragma once
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <stdexcept>
#include <string>
#include <thread>
#include <utility>
#include <vector>

namespace sahara_io {

struct Record {
    std::string id;
    std::string seq;
};

// Streaming reader: multi-line records, '>' headers, CR/LF tolerant.
class FastaReader {
   public:
    explicit FastaReader(const std::string& path) : f_(std::fopen(path.c_str(), "rb")), path_(path) {
        if (!f_) throw std::runtime_error("can not open file " + path);
        buf_.resize(1 << 20);
    }
    ~FastaReader() {
        if (f_) std::fclose(f_);
    }
    FastaReader(const FastaReader&) = delete;
    FastaReader& operator=(const FastaReader&) = delete;

    bool next(Record& r) {
        r.id.clear();
        r.seq.clear();
        std::string line;
        if (!havePending_) {
            while (readLine(line)) {
                if (!line.empty() && line[0] == '>') { pending_ = line; havePending_ = true; break; }
                if (!line.empty()) throw std::runtime_error("malformed FASTA (sequence before header) in " + path_);
            }
            if (!havePending_) return false;
        }
        r.id = pending_.substr(1);
        havePending_ = false;
        while (readLine(line)) {
            if (!line.empty() && line[0] == '>') { pending_ = line; havePending_ = true; break; }
            r.seq += line;
        }
        return true;
    }

   private:
    bool readLine(std::string& out) {
        out.clear();
        for (;;) {
            if (pos_ >= len_) {
                len_ = std::fread(buf_.data(), 1, buf_.size(), f_);
                pos_ = 0;
                if (len_ == 0) return !out.empty();
            }
            const char* start = buf_.data() + pos_;
            const char* nl = static_cast<const char*>(std::memchr(start, '\n', len_ - pos_));
            if (!nl) {
                out.append(start, len_ - pos_);
                pos_ = len_;
                continue;
            }
            out.append(start, (size_t)(nl - start));
            pos_ += (size_t)(nl - start) + 1;
            if (!out.empty() && out.back() == '\r') out.pop_back();
            return true;
        }
    }

    std::FILE* f_;
    std::string path_;
    std::vector<char> buf_;
    size_t pos_ = 0, len_ = 0;
    std::string pending_;
    bool havePending_ = false;
};

inline uint8_t charToRank(char c, uint32_t sigma) {
    switch (c) {
        case 'A': case 'a': return 1;
        case 'C': case 'c': return 2;
        case 'G': case 'g': return 3;
        case 'T': case 't': return sigma == 6 ? 5 : 4;
        case 'N': case 'n': return sigma == 6 ? 4 : 255;
        default: return 255;
    }
}

// index of the first invalid rank, or -1 (ivs::verify_rank)
inline long firstInvalid(const std::vector<uint8_t>& r, uint32_t sigma) {
    for (size_t i = 0; i < r.size(); ++i)
        if (r[i] == 0 || r[i] >= sigma) return (long)i;
    return -1;
}

inline std::vector<uint8_t> toRanks(const std::string& s, uint32_t sigma) {
    std::vector<uint8_t> r(s.size());
    for (size_t i = 0; i < s.size(); ++i) r[i] = charToRank(s[i], sigma);
    return r;
}

// ----------------------------------------------------------------------------
// Whole-file FASTA ingest on several threads: the same records, ranks and
// validation as FastaReader + toRanks + firstInvalid, for the 3 Gbp reference
// of `sahara index` and the 10M-read query files of `sahara search`
// (single-threaded parsing dominates at that scale).
// The file is mapped and cut into pieces of ~8 MB that start at line starts.
// A line starting with '>' is a header (a new record), any other line is
// sequence. Pass 1 counts each piece's sequence characters and notes where
// its records start; pass 2 converts them at the prefix-summed offsets into
// one flat array, in one of two forms:
//   kRanks: one rank per byte (255 = no rank of the alphabet);
//   kCodes2: two bits per symbol, symbol s at bits 2 (s % 4) of byte s / 4,
//            A C G T coded 0 1 2 3, and the positions of dna5's N listed in
//            ascending order (their code is 0) — the packed reads that
//            sahara_gpu_search_packed[_compact] take, written without an
//            intermediate rank array (a quarter of the bytes).
enum class FastaForm { kRanks = 1, kCodes2 = 2 };

struct FastaData {
    std::vector<uint64_t> offs;     // record i = symbols [offs[i], offs[i+1])
    std::vector<uint8_t> ranks;     // kRanks: one per symbol; kCodes2: (symbols + 3) / 4 bytes
    uint8_t* codes = nullptr;       // kCodes2 with a CodesAlloc: the codes there instead (the caller's to free)
    uint64_t codesBytes = 0;        // kCodes2: (symbols + 3) / 4
    std::vector<uint64_t> nPos;     // kCodes2: symbols that are N (dna5), ascending
    uint64_t symbols = 0;
    // the first byte that is no rank of the alphabet, if any
    bool bad = false;
    size_t badRecord = 0;
    uint64_t badPos = 0;            // position in its record
    unsigned char badChar = 0;
    std::string badId;              // its record's header text after '>'
    size_t records() const { return offs.empty() ? 0 : offs.size() - 1; }
};

template <typename F>
inline void parallelFor(unsigned nt, size_t n, F&& f) {  // f(i) for i in [0, n), interleaved over nt threads
    if (nt <= 1 || n < 2) {
        for (size_t i = 0; i < n; ++i) f(i);
        return;
    }
    std::vector<std::thread> ts;
    for (unsigned t = 0; t < nt && t < n; ++t)
        ts.emplace_back([&, t] {
            for (size_t i = t; i < n; i += nt) f(i);
        });
    for (auto& t : ts) t.join();
}

inline unsigned hostThreads() {
    const char* e = std::getenv("OMP_NUM_THREADS");  // the GPU box's CPU share (16 per GPU)
    unsigned n = e ? (unsigned)std::atoi(e) : 0;
    if (n == 0) n = std::thread::hardware_concurrency();
    return std::max(1u, std::min(n, 32u));
}

// kCodes2 may go straight into a caller's buffer (the page-locked memory the
// search calls DMA): alloc(bytes) returns it, uninitialised, on a thread of
// its own while pass 1 runs (bytes >= the codes' size); the result is then in
// D.codes (the caller's to free) instead of D.ranks. release(p) frees it when
// the parse fails.
struct CodesAlloc {
    std::function<uint8_t*(size_t)> alloc;
    std::function<void(uint8_t*)> release;
};

inline FastaData parseFastaParallel(const std::string& path, uint32_t sigma, unsigned nt,
                                    size_t kPiece = 8u << 20, FastaForm form = FastaForm::kRanks,
                                    const CodesAlloc* codesAlloc = nullptr) {
    const int fd = ::open(path.c_str(), O_RDONLY);
    if (fd < 0) throw std::runtime_error("can not open file " + path);
    struct stat sb {};
    if (::fstat(fd, &sb) != 0) {
        ::close(fd);
        throw std::runtime_error("can not stat file " + path);
    }
    const size_t n = (size_t)sb.st_size;
    FastaData D;
    if (n == 0) {
        ::close(fd);
        return D;
    }
    void* mp = ::mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
    ::close(fd);
    if (mp == MAP_FAILED) throw std::runtime_error("can not map file " + path);
    (void)::madvise(mp, n, MADV_WILLNEED);
    const char* b = static_cast<const char*>(mp);
    struct Unmap {
        void* p;
        size_t n;
        ~Unmap() { ::munmap(p, n); }
    } unmap{mp, n};
    const bool codes = form == FastaForm::kCodes2;
    // the caller's output buffer, allocated beside pass 1 (symbols <= n)
    struct Alloc {
        std::thread t;
        uint8_t* p = nullptr;
        const CodesAlloc* a = nullptr;
        uint8_t* take() {  // joined; the buffer is the caller's from here on
            if (t.joinable()) t.join();
            uint8_t* q = p;
            p = nullptr;
            return q;
        }
        ~Alloc() {
            if (t.joinable()) t.join();
            if (p && a && a->release) a->release(p);  // (the parse failed)
        }
    } ext;
    if (codes && codesAlloc && codesAlloc->alloc) {
        ext.a = codesAlloc;
        ext.t = std::thread([&ext, codesAlloc, n] { ext.p = codesAlloc->alloc(n / 4 + 16); });
    }
    // pieces of ~kPiece bytes starting at line starts
    std::vector<size_t> bound{0};
    for (size_t p = kPiece; p < n;) {
        const void* nl = std::memchr(b + p, '\n', n - p);
        if (!nl) break;
        const size_t q = (size_t)(static_cast<const char*>(nl) - b) + 1;
        if (q >= n) break;
        bound.push_back(q);
        p = q + kPiece;
    }
    bound.push_back(n);
    const size_t P = bound.size() - 1;
    struct Piece {
        uint64_t seq = 0;                                    // sequence characters
        uint64_t lead = 0;                                   // ... before its first header
        std::vector<std::pair<uint64_t, uint64_t>> heads;    // (header position, sequence characters before it)
        uint64_t badAt = UINT64_MAX;                         // first invalid rank (piece-local sequence index)
        unsigned char badChar = 0;
        std::vector<uint64_t> nPos;                          // kCodes2: its N symbols (global positions)
        uint8_t head = 0, tail = 0;                          // kCodes2: its bits of the bytes it shares
    };
    std::vector<Piece> pc(P);
    // a line's sequence bytes end before its '\n', and before a '\r' right
    // in front of it (FastaReader::readLine; not at a last line without '\n')
    auto lineEnd = [&](size_t p, size_t eol, bool hasNl) { return hasNl && eol > p && b[eol - 1] == '\r' ? eol - 1 : eol; };
    // pass 1: count
    parallelFor(nt, P, [&](size_t i) {
        Piece& c = pc[i];
        uint64_t k = 0;
        for (size_t p = bound[i], e = bound[i + 1]; p < e;) {
            const void* nl = std::memchr(b + p, '\n', e - p);
            const size_t eol = nl ? (size_t)(static_cast<const char*>(nl) - b) : e;
            if (b[p] == '>') {
                if (c.heads.empty()) c.lead = k;
                c.heads.emplace_back(p, k);
            } else {
                k += lineEnd(p, eol, nl != nullptr) - p;
            }
            p = eol + 1;
        }
        c.seq = k;
        if (c.heads.empty()) c.lead = k;
    });
    // records and offsets: each piece writes its records' offsets at the
    // prefix-summed record and symbol counts (in parallel: 10M records)
    std::vector<uint64_t> base(P + 1, 0), rbase(P + 1, 0);
    for (size_t i = 0; i < P; ++i) {
        base[i + 1] = base[i] + pc[i].seq;
        rbase[i + 1] = rbase[i] + pc[i].heads.size();
    }
    uint64_t lead = 0;  // sequence characters before the first header
    for (size_t i = 0; i < P; ++i) {
        lead += pc[i].lead;
        if (!pc[i].heads.empty()) break;
    }
    if (lead > 0) throw std::runtime_error("malformed FASTA (sequence before header) in " + path);
    if (rbase[P] == 0) {
        D.codes = ext.take();
        return D;
    }
    D.offs.resize(rbase[P] + 1);
    parallelFor(nt, P, [&](size_t i) {
        uint64_t* o = D.offs.data() + rbase[i];
        for (const auto& h : pc[i].heads) *o++ = base[i] + h.second;
    });
    D.offs[rbase[P]] = base[P];
    D.symbols = base[P];
    // pass 2: convert
    uint8_t table[256];
    for (int c = 0; c < 256; ++c) table[c] = charToRank((char)c, sigma);
    uint8_t* out = nullptr;
    if (!codes) {
        D.ranks.resize(base[P]);
    } else {
        D.codes = ext.take();
        if (!D.codes) D.ranks.resize((base[P] + 3) / 4);
        out = D.codes ? D.codes : D.ranks.data();
        D.codesBytes = (base[P] + 3) / 4;
    }
    // per character: bits 0-1 its 2-bit code (A C G T = 0 1 2 3, N and
    // invalid characters 0), bit 2 N (dna5: listed), bit 3 no rank of the alphabet
    uint8_t cls[256];
    for (int c = 0; c < 256; ++c) {
        const uint8_t r = table[c];
        cls[c] = r >= sigma ? 8 : (sigma == 6 && r == 4) ? 4 : r == 1 ? 0 : r == 2 ? 1 : r == 3 ? 2 : 3;
    }
    parallelFor(nt, P, [&](size_t i) {
        Piece& c = pc[i];
        if (!codes) {
            uint8_t* const o0 = D.ranks.data() + base[i];
            uint8_t* o = o0;
            for (size_t p = bound[i], e = bound[i + 1]; p < e;) {
                const void* nl = std::memchr(b + p, '\n', e - p);
                const size_t eol = nl ? (size_t)(static_cast<const char*>(nl) - b) : e;
                if (b[p] != '>') {
                    for (size_t q = p, qe = lineEnd(p, eol, nl != nullptr); q < qe; ++q) {
                        const unsigned char ch = (unsigned char)b[q];
                        const uint8_t v = table[ch];
                        if (v >= sigma && c.badAt == UINT64_MAX) {
                            c.badAt = (uint64_t)(o - o0);
                            c.badChar = ch;
                        }
                        *o++ = v;
                    }
                }
                p = eol + 1;
            }
            return;
        }
        // two bits per symbol: whole bytes inside the piece are stored, the
        // partial first and last bytes (shared with the neighbours) kept in
        // head / tail and or-ed in afterwards
        const uint64_t g0 = base[i];
        uint64_t g = g0;
        uint32_t acc = 0;
        auto one = [&](unsigned char ch) {
            const uint8_t v = cls[ch];
            if (v & 12u) {
                if ((v & 8u) && c.badAt == UINT64_MAX) {
                    c.badAt = g - g0;
                    c.badChar = ch;
                }
                if (v & 4u) c.nPos.push_back(g);
            }
            acc |= (uint32_t)(v & 3u) << (2u * (uint32_t)(g & 3u));
            if ((g & 3u) == 3u) {
                if (g / 4 == g0 / 4 && (g0 & 3u)) c.head = (uint8_t)acc;
                else out[g / 4] = (uint8_t)acc;
                acc = 0;
            }
            ++g;
        };
        for (size_t p = bound[i], e = bound[i + 1]; p < e;) {
            const void* nl = std::memchr(b + p, '\n', e - p);
            const size_t eol = nl ? (size_t)(static_cast<const char*>(nl) - b) : e;
            if (b[p] != '>') {
                size_t q = p;
                const size_t qe = lineEnd(p, eol, nl != nullptr);
                while (q < qe && (g & 3u)) one((unsigned char)b[q++]);
                // whole bytes, four characters at a time (g % 4 == 0 here, so
                // the byte is the piece's own)
                for (; q + 4 <= qe; q += 4) {
                    const uint8_t v0 = cls[(unsigned char)b[q]], v1 = cls[(unsigned char)b[q + 1]];
                    const uint8_t v2 = cls[(unsigned char)b[q + 2]], v3 = cls[(unsigned char)b[q + 3]];
                    if ((v0 | v1 | v2 | v3) & 12u) {  // N or an invalid character: one at a time
                        for (size_t j = 0; j < 4; ++j) one((unsigned char)b[q + j]);
                        continue;
                    }
                    out[g / 4] = (uint8_t)(v0 | (v1 << 2) | (v2 << 4) | (v3 << 6));
                    g += 4;
                }
                while (q < qe) one((unsigned char)b[q++]);
            }
            p = eol + 1;
        }
        if (g & 3u) {  // a partial last byte
            if (g / 4 == g0 / 4 && (g0 & 3u)) c.head |= (uint8_t)acc;  // the piece lies inside one byte
            else c.tail = (uint8_t)acc;
        }
    });
    if (codes) {
        // the bytes pieces share were written by none of them: zero, then or in
        uint64_t nN = 0;
        for (size_t i = 0; i < P; ++i) {
            const uint64_t g0 = base[i], g1 = base[i + 1];
            if (g1 == g0) continue;
            if (g0 & 3u) out[g0 / 4] = 0;
            if (g1 & 3u) out[g1 / 4] = 0;
        }
        for (size_t i = 0; i < P; ++i) {
            const uint64_t g0 = base[i], g1 = base[i + 1];
            if (g1 == g0) continue;
            if (g0 & 3u) out[g0 / 4] |= pc[i].head;
            if ((g1 & 3u) && !(g1 / 4 == g0 / 4 && (g0 & 3u))) out[g1 / 4] |= pc[i].tail;
            nN += pc[i].nPos.size();
        }
        D.nPos.reserve(nN);
        for (size_t i = 0; i < P; ++i) D.nPos.insert(D.nPos.end(), pc[i].nPos.begin(), pc[i].nPos.end());
    }
    for (size_t i = 0; i < P; ++i)
        if (pc[i].badAt != UINT64_MAX) {
            const uint64_t at = base[i] + pc[i].badAt;
            D.bad = true;
            D.badRecord = (size_t)(std::upper_bound(D.offs.begin(), D.offs.end(), at) - D.offs.begin()) - 1;
            D.badPos = at - D.offs[D.badRecord];
            D.badChar = pc[i].badChar;
            // the record's header: piece j holds records [rbase[j], rbase[j + 1])
            const size_t j = (size_t)(std::upper_bound(rbase.begin(), rbase.end(), (uint64_t)D.badRecord) - rbase.begin()) - 1;
            const size_t h = pc[j].heads[D.badRecord - rbase[j]].first + 1;
            const void* nl = std::memchr(b + h, '\n', n - h);
            size_t eol = nl ? (size_t)(static_cast<const char*>(nl) - b) : n;
            if (eol > h && b[eol - 1] == '\r') --eol;
            D.badId.assign(b + h, eol - h);
            break;
        }
    return D;
}

// ivs::reverse_complement_rank of one rank: A<->T, C<->G, N->N
inline uint8_t complementRank(uint8_t c, uint32_t sigma) {
    if (sigma == 6) return c == 1 ? 5 : c == 2 ? 3 : c == 3 ? 2 : c == 5 ? 1 : c;
    return c == 1 ? 4 : c == 2 ? 3 : c == 3 ? 2 : c == 4 ? 1 : c;
}

inline std::vector<uint8_t> reverseComplement(const std::vector<uint8_t>& r, uint32_t sigma) {
    std::vector<uint8_t> o(r.size());
    for (size_t i = 0; i < r.size(); ++i) {
        const uint8_t c = r[r.size() - 1 - i];
        uint8_t x = c;
        if (sigma == 6) x = c == 1 ? 5 : c == 2 ? 3 : c == 3 ? 2 : c == 5 ? 1 : c;  // A<->T, C<->G, N->N
        else            x = c == 1 ? 4 : c == 2 ? 3 : c == 3 ? 2 : c == 4 ? 1 : c;
        o[i] = x;
    }
    return o;
}

}  // namespace sahara_io
