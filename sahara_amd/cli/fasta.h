// fasta.h — FASTA reading and rank conversion for the `sahara` CLI.
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
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace sahara_cli {

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

}  // namespace sahara_cli
