// read_simulator.cpp — `sahara read_simulator`: the reference's input
// generator (src/sahara/read_simulator.cpp), restated. Host only.
//
// Same flags and defaults (read_simulator.cpp:19-82), the same random
// engines in the same call order — rand() seeded by --seed for the error
// types and for replacing non-ACGT reference characters, one
// default-seeded std::mt19937_64 for the transcripts and another for the read
// positions and the inserted/substituted bases (:95-231) — and the same
// FASTA header "simulated-{i} (seqid:{s}, pos:{p}, trans:{t})" (:274). Built
// with the same standard library, the output is the reference's byte for
// byte. Quirks kept on purpose: --seed does not seed the mt19937 engines, and
// a read that would cross a record end is redrawn (:180-196).

#include <algorithm>
#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <limits>
#include <random>
#include <stdexcept>
#include <string>
#include <string_view>
#include <tuple>
#include <vector>

#include "../csrc/fasta.h"

namespace sahara_cli {
using namespace sahara_io;
namespace {

std::mt19937_64 g_transcriptEngine;  // the reference's global `generator` (read_simulator.cpp:114)

char randomPick() {
    switch (std::rand() % 4) {
        case 0: return 'A';
        case 1: return 'C';
        case 2: return 'G';
        default: return 'T';
    }
}

int rank4(char c) { return c == 'A' ? 0 : c == 'C' ? 1 : c == 'G' ? 2 : 3; }
char char4(int r) { return "ACGT"[r & 3]; }

// edit transcript of `len` read positions (read_simulator.cpp:117-166)
struct Transcript {
    std::string t;
    size_t matches;
    Transcript(size_t len, size_t sub, size_t ins, size_t del) : t(len, 'M'), matches(len) {
        for (size_t i = 0; i < sub; ++i) mark('S');
        for (size_t i = 0; i < ins; ++i) mark('I');
        for (size_t i = 0; i < del; ++i) {
            const size_t pos = std::uniform_int_distribution<size_t>{0, t.size()}(g_transcriptEngine);
            t.insert(t.begin() + (long)pos, 'D');
        }
    }
    void mark(char op) {
        if (matches == 0) throw std::runtime_error("no more matches for this transcript possible");
        auto pos = std::uniform_int_distribution<size_t>{0, t.size() - 1}(g_transcriptEngine);
        while (t[pos] != 'M') pos = std::uniform_int_distribution<size_t>{0, t.size() - 1}(g_transcriptEngine);
        t[pos] = op;
        matches -= 1;
    }
    size_t lengthOfRef() const { return t.size() - (size_t)std::count(t.begin(), t.end(), 'I'); }
};

// read positions and base draws (read_simulator.cpp:169-231)
struct ReadGenerator {
    const std::vector<std::string>& seqs;
    size_t readLength;
    size_t total;
    std::mt19937_64 engine;
    std::uniform_int_distribution<size_t> uniformPos;

    ReadGenerator(const std::vector<std::string>& s, size_t rl)
        : seqs(s), readLength(rl), total(sumLen(s)), uniformPos(0, sumLen(s) - 1) {}
    static size_t sumLen(const std::vector<std::string>& s) {
        size_t l = 0;
        for (auto& x : s) l += x.size();
        if (l == 0) throw std::runtime_error("reference is empty");
        return l;
    }

    std::tuple<size_t, size_t, std::string_view> generate(size_t len) {
        for (;;) {
            size_t pos = uniformPos(engine);
            size_t seqId = 0;
            for (std::string_view seq : seqs) {
                if (pos + len > seq.size()) break;
                if (pos < seq.size()) return {seqId, pos, seq.substr(pos, len)};
                seqId += 1;
                pos = pos + readLength - seq.size() - 1;
            }
        }
    }

    std::string apply(std::string_view v, const std::string& transcript) {
        std::string res;
        size_t p = 0;
        std::uniform_int_distribution<size_t> u02{0, 2}, u03{0, 3};
        for (char t : transcript) {
            switch (t) {
                case 'M': res.push_back(v[p]); ++p; break;
                case 'S': res.push_back(char4((int)((rank4(v[p]) + u02(engine) + 1) % 4))); ++p; break;
                case 'I': res.push_back(char4((int)u03(engine))); break;
                case 'D': ++p; break;
                default: throw std::runtime_error(std::string("Invalid transcript \"") + t + "\"");
            }
        }
        return res;
    }
};

void writeRecord(std::FILE* f, const std::string& id, const std::string& seq, size_t width) {
    std::fprintf(f, ">%s\n", id.c_str());
    for (size_t i = 0; i < seq.size(); i += width) {
        const size_t n = std::min(width, seq.size() - i);
        std::fwrite(seq.data() + i, 1, n, f);
        std::fputc('\n', f);
    }
    if (seq.empty()) std::fputc('\n', f);
}

}  // namespace

struct ReadSimulatorArgs {  // mirrored in main.cpp
    std::string input, output;
    size_t lineLength = 80, readLength = 150, nreads = 1000, sub = 0, ins = 0, del = 0, errors = 0;
    uint32_t seed = 0;
    bool haveInput = false;
};

int runReadSimulator(const ReadSimulatorArgs& a) {
    std::srand(a.seed);
    std::FILE* f = std::fopen(a.output.c_str(), "w");
    if (!f) throw std::runtime_error("can not open output file " + a.output);
    const size_t width = a.lineLength == 0 ? (size_t)std::numeric_limits<int>::max() : a.lineLength;
    if (a.haveInput) {
        std::vector<std::string> seqs;
        {
            FastaReader rd(a.input);
            Record rec;
            while (rd.next(rec)) {
                std::string s;
                s.reserve(rec.seq.size());
                for (char c : rec.seq) {
                    c = (char)std::toupper((unsigned char)c);  // dna4 normalisation
                    if (c != 'A' && c != 'C' && c != 'G' && c != 'T') c = randomPick();
                    s.push_back(c);
                }
                seqs.emplace_back(std::move(s));
            }
        }
        std::printf("loaded fasta file - start simulating\n");
        ReadGenerator gen(seqs, a.readLength);
        for (size_t i = 0; i < a.nreads; ++i) {
            size_t sub = a.sub, ins = a.ins, del = a.del;
            for (size_t k = 0; k < a.errors; ++k) {
                switch (std::rand() % 3) {
                    case 0: sub += 1; break;
                    case 1: ins += 1; break;
                    default: del += 1; break;
                }
            }
            Transcript tr(a.readLength, sub, ins, del);
            auto [seqId, pos, read] = gen.generate(tr.lengthOfRef());
            const std::string faulty = gen.apply(read, tr.t);
            writeRecord(f,
                        "simulated-" + std::to_string(i) + " (seqid:" + std::to_string(seqId) +
                            ", pos:" + std::to_string(pos) + ", trans:" + tr.t + ")",
                        faulty, width);
        }
    } else {
        std::printf("no fasta file - start pure random simulating\n");
        for (size_t i = 0; i < a.nreads; ++i) {
            std::string s;
            s.reserve(a.readLength);
            for (size_t k = 0; k < a.readLength; ++k) s.push_back(randomPick());
            writeRecord(f, "simulated-" + std::to_string(i), s, 80);
        }
    }
    std::fclose(f);
    return 0;
}

}  // namespace sahara_cli
