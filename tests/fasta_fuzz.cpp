// Fuzz check of the CLI's parallel FASTA ingest (sahara_amd/cli/fasta.h):
// parseFastaParallel must give the records, ranks and first invalid
// character of the sequential FastaReader + toRanks, for random FASTA-like
// files (CRLF, blank lines, '>' inside lines, empty records, invalid bytes),
// any piece size and thread count. Built and run by tests/test_fasta_parallel.py.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>

#include "../sahara_amd/csrc/fasta.h"

using namespace sahara_io;

int main(int argc, char** argv) {
    const std::string path = argc > 1 ? argv[1] : "/tmp/fasta_fuzz.fa";
    std::mt19937_64 g(12345);
    const char alpha[] = "ACGTNacgtnACGTACGTX>\r\n ";
    int failures = 0;
    for (int it = 0; it < 400; ++it) {
        std::string f;
        const int lines = (int)(g() % 40);
        if (g() % 5 == 0) f += "\n\r\n";  // blank lines before the first header
        for (int l = 0; l < lines; ++l) {
            if (g() % 4 == 0 || l == 0) {
                f += ">id" + std::to_string(l) + (g() % 3 ? " a>b" : "");
            } else {
                const int w = (int)(g() % 30);
                for (int k = 0; k < w; ++k) f += alpha[g() % (g() % 7 ? 12 : sizeof(alpha) - 1)];
            }
            f += g() % 5 ? "\n" : "\r\n";
        }
        if (g() % 3 == 0 && !f.empty()) f.pop_back();  // no final line break
        if (g() % 9 == 0) f = "AC\n" + f;               // sequence before the first header
        std::FILE* o = std::fopen(path.c_str(), "wb");
        std::fwrite(f.data(), 1, f.size(), o);
        std::fclose(o);
        const uint32_t sigma = g() % 2 ? 6 : 5;
        // sequential reference
        std::vector<std::vector<uint8_t>> want;
        std::vector<std::string> ids;
        std::string werr;
        try {
            FastaReader rd(path);
            Record r;
            while (rd.next(r)) {
                want.push_back(toRanks(r.seq, sigma));
                ids.push_back(r.id);
            }
        } catch (const std::exception& e) {
            werr = e.what();
        }
        for (size_t piece : {size_t(1), size_t(7), size_t(64), size_t(8) << 20}) {
            for (unsigned nt : {1u, 3u}) {
                std::string gerr;
                FastaData D;
                try {
                    D = parseFastaParallel(path, sigma, nt, piece);
                } catch (const std::exception& e) {
                    gerr = e.what();
                }
                bool ok = werr.empty() == gerr.empty();
                if (ok && werr.empty()) {
                    ok = D.records() == want.size();
                    long badRec = -1, badPos = -1;
                    for (size_t r = 0; ok && r < want.size(); ++r) {
                        ok = D.offs[r + 1] - D.offs[r] == want[r].size() &&
                             std::equal(want[r].begin(), want[r].end(), D.ranks.begin() + (long)D.offs[r]);
                        if (badRec < 0)
                            if (long p = firstInvalid(want[r], sigma); p >= 0) badRec = (long)r, badPos = p;
                    }
                    ok = ok && D.bad == (badRec >= 0);
                    if (ok && D.bad)
                        ok = (long)D.badRecord == badRec && (long)D.badPos == badPos && D.badId == ids[(size_t)badRec];
                    // the 2-bit form: the same records, codes of the valid
                    // symbols (A C G T = 0 1 2 3, N = 0), N listed, same first
                    // invalid character
                    FastaData E = parseFastaParallel(path, sigma, nt, piece, FastaForm::kCodes2);
                    ok = ok && E.offs == D.offs && E.bad == D.bad && E.badRecord == D.badRecord &&
                         E.badPos == D.badPos && E.badId == D.badId && E.ranks.size() == (D.ranks.size() + 3) / 4;
                    std::vector<uint64_t> wantN;
                    for (uint64_t q = 0; ok && q < D.ranks.size(); ++q) {
                        const uint8_t r = D.ranks[q];
                        if (r >= sigma) continue;  // invalid: code unspecified
                        const uint32_t code = (E.ranks[q / 4] >> (2 * (q % 4))) & 3u;
                        const uint32_t want2 = r == 1 ? 0 : r == 2 ? 1 : r == 3 ? 2 : (sigma == 6 && r == 4) ? 0 : 3;
                        ok = code == want2;
                        if (sigma == 6 && r == 4) wantN.push_back(q);
                    }
                    ok = ok && E.nPos == wantN && E.symbols == D.ranks.size();
                    // the same into a caller's buffer (uninitialised: filled
                    // with a pattern first), byte for byte
                    CodesAlloc A;
                    A.alloc = [](size_t b) {
                        uint8_t* p = static_cast<uint8_t*>(std::malloc(b));
                        std::memset(p, 0xA5, b);
                        return p;
                    };
                    A.release = [](uint8_t* p) { std::free(p); };
                    FastaData X = parseFastaParallel(path, sigma, nt, piece, FastaForm::kCodes2, &A);
                    ok = ok && X.ranks.empty() && X.codesBytes == E.ranks.size() && X.offs == E.offs &&
                         X.nPos == E.nPos && X.bad == E.bad && X.badRecord == E.badRecord && X.badPos == E.badPos &&
                         (E.ranks.empty() || std::equal(E.ranks.begin(), E.ranks.end(), X.codes));
                    std::free(X.codes);
                }
                if (!ok) {
                    std::printf("mismatch: iteration %d piece %zu threads %u (%s | %s)\n", it, piece, nt, werr.c_str(),
                                gerr.c_str());
                    ++failures;
                }
            }
        }
    }
    std::printf("%s\n", failures ? "FAIL" : "OK");
    return failures ? 1 : 0;
}
