// oracle.cpp — CPU restatement of sahara's search hot path (TEST INFRASTRUCTURE).
//
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
// this library. It is the checker and the timed CPU baseline, never the product.
//
// Reference anchors (paths relative to /root/reference):
//   index build  : src/sahara/index.cpp:41-112 (BiFMIndex{ref, samplingRate=16, threadNbr=1} at :87)
//   query ingest : src/sahara/search.cpp:111-130 (RC interleave :121-123)
//   scheme build : src/sahara/search.cpp:186-212 (generator, expand), :226 (limitToHamming)
//   search DFS   : src/sahara/search.cpp:227/230 (fmc::search_ng24::search<Edit>) [upstream]
//   locate       : src/sahara/search.cpp:244-250 (fmc::LocateLinear) [upstream]
// The upstream library (fmindex-collection v1.1.0) is absent; the semantics
// implemented are policy P0, written out in docs/semantics.md.
//
// Data structures deliberately differ from the GPU product's so that the two
// implementations cross-check each other: the oracle ranks with one one-hot
// bitvector per symbol (InterleavedBitvector-style, 64-position blocks with
// absolute u32 counts), the GPU with 3 bit-planes per 64-position line.

#include "oracle.h"

#include <algorithm>
#include <initializer_list>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <functional>
#include <map>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace orc {

// ---------------------------------------------------------------- index ----

struct Line {                 // 64 positions of one BWT
    uint32_t cnt[5];          // occurrences of symbol c+1 before the block
    uint32_t pad;
    uint64_t bits[5];         // one-hot bitvector of symbol c+1 inside the block
};

struct Index {
    uint32_t sigma = 6;
    uint64_t n = 0;                         // text length incl. one '$' per record
    std::vector<uint64_t> C;                // sigma+1 entries: C[c] = #symbols < c
    std::vector<uint64_t> recLen, recStart; // recStart[r] = first text position of record r
    uint32_t rate = 16;
    std::vector<uint8_t> bwtF, bwtR;
    std::vector<Line> occF, occR;
    std::vector<uint64_t> sampled;          // bit i: row i is sampled
    std::vector<uint64_t> sampledRank;      // #sampled rows before block b
    std::vector<uint32_t> samples;          // text position of each sampled row, row order
    std::vector<uint32_t> sa;               // full SA (only when built here)
};

static std::vector<Line> makeLines(const std::vector<uint8_t>& bwt, uint32_t sigma) {
    const uint64_t n = bwt.size();
    const uint64_t nb = n / 64 + 1;
    std::vector<Line> L(nb);
    uint64_t run[5] = {0, 0, 0, 0, 0};
    for (uint64_t b = 0; b < nb; ++b) {
        Line& ln = L[b];
        std::memset(&ln, 0, sizeof(ln));
        for (int c = 0; c < 5; ++c) ln.cnt[c] = (uint32_t)run[c];
        for (uint64_t j = 0; j < 64 && b * 64 + j < n; ++j) {
            uint8_t s = bwt[b * 64 + j];
            if (s >= 1 && s < sigma) {
                ln.bits[s - 1] |= 1ull << j;
                run[s - 1]++;
            }
        }
    }
    return L;
}

static inline uint64_t rankOf(const std::vector<Line>& L, uint32_t c, uint64_t i) {
    const Line& ln = L[i >> 6];
    const uint64_t o = i & 63;
    const uint64_t mask = o ? (~0ull >> (64 - o)) : 0ull;
    return ln.cnt[c - 1] + (uint64_t)__builtin_popcountll(ln.bits[c - 1] & mask);
}

static void finishIndex(Index& I) {
    I.occF = makeLines(I.bwtF, I.sigma);
    I.occR = makeLines(I.bwtR, I.sigma);
    const uint64_t nb = I.n / 64 + 1;
    I.sampledRank.assign(nb, 0);
    uint64_t run = 0;
    for (uint64_t b = 0; b < nb; ++b) {
        I.sampledRank[b] = run;
        if (b < I.sampled.size()) run += (uint64_t)__builtin_popcountll(I.sampled[b]);
    }
    I.recStart.resize(I.recLen.size());
    uint64_t s = 0;
    for (size_t r = 0; r < I.recLen.size(); ++r) {
        I.recStart[r] = s;
        s += I.recLen[r] + 1;
    }
}

// Suffix array by prefix doubling (Manber-Myers style with std::sort). '$' is
// rank 0 and compares like any symbol; a suffix that ends is smaller than
// every extension of it.
static std::vector<uint32_t> suffixArray(const std::vector<uint8_t>& T) {
    const uint64_t n = T.size();
    std::vector<uint32_t> sa(n), rk(n), tmp(n);
    for (uint64_t i = 0; i < n; ++i) { sa[i] = (uint32_t)i; rk[i] = T[i] + 1u; }
    for (uint64_t h = 1;; h <<= 1) {
        auto key2 = [&](uint32_t i) -> uint32_t { return i + h < n ? rk[i + h] : 0u; };
        std::sort(sa.begin(), sa.end(), [&](uint32_t a, uint32_t b) {
            if (rk[a] != rk[b]) return rk[a] < rk[b];
            return key2(a) < key2(b);
        });
        tmp[sa[0]] = 1;
        for (uint64_t i = 1; i < n; ++i) {
            bool diff = rk[sa[i]] != rk[sa[i - 1]] || key2(sa[i]) != key2(sa[i - 1]);
            tmp[sa[i]] = tmp[sa[i - 1]] + (diff ? 1u : 0u);
        }
        rk.swap(tmp);
        if (rk[sa[n - 1]] == n) break;
    }
    return sa;
}

static Index* build(const uint8_t* ranks, const uint64_t* recLens, uint64_t nrec, uint32_t sigma,
                    uint32_t rate) {
    auto* I = new Index();
    I->sigma = sigma;
    I->rate = rate;
    I->recLen.assign(recLens, recLens + nrec);
    std::vector<uint8_t> T, R;
    uint64_t total = 0;
    for (uint64_t r = 0; r < nrec; ++r) total += recLens[r] + 1;
    T.reserve(total);
    R.reserve(total);
    uint64_t off = 0;
    for (uint64_t r = 0; r < nrec; ++r) {
        for (uint64_t j = 0; j < recLens[r]; ++j) T.push_back(ranks[off + j]);
        T.push_back(0);
        for (uint64_t j = recLens[r]; j-- > 0;) R.push_back(ranks[off + j]);
        R.push_back(0);
        off += recLens[r];
    }
    const uint64_t n = T.size();
    I->n = n;
    I->C.assign(sigma + 1, 0);
    for (uint8_t c : T) I->C[c + 1]++;
    for (uint32_t c = 1; c <= sigma; ++c) I->C[c] += I->C[c - 1];
    I->sa = suffixArray(T);
    std::vector<uint32_t> saR = suffixArray(R);
    I->bwtF.resize(n);
    I->bwtR.resize(n);
    for (uint64_t i = 0; i < n; ++i) {
        I->bwtF[i] = T[(I->sa[i] + n - 1) % n];
        I->bwtR[i] = R[(saR[i] + n - 1) % n];
    }
    // recStart for sampling decisions
    std::vector<uint64_t> starts(nrec);
    uint64_t s = 0;
    for (uint64_t r = 0; r < nrec; ++r) { starts[r] = s; s += recLens[r] + 1; }
    I->sampled.assign(n / 64 + 1, 0);
    for (uint64_t i = 0; i < n; ++i) {
        uint64_t p = I->sa[i];
        uint64_t r = (uint64_t)(std::upper_bound(starts.begin(), starts.end(), p) - starts.begin()) - 1;
        // sampled: in-record offsets that are multiples of the rate, and every
        // delimiter (so no LF walk ever has to step through a '$')
        if ((p - starts[r]) % rate == 0 || p - starts[r] == recLens[r]) {
            I->sampled[i >> 6] |= 1ull << (i & 63);
            I->samples.push_back((uint32_t)p);
        }
    }
    finishIndex(*I);
    return I;
}

// ------------------------------------------------------------- cursor ----

struct Cur { uint64_t lb, lbr, len; };

// All sigma-1 children of `c` extended on the left (forward BWT) or on the
// right (reverse BWT). Bidirectional update: the other side's lower bound is
// shifted by the number of occurrences of smaller symbols, '$' included.
static inline void extendAll(const Index& I, const Cur& c, bool right, Cur* out,
                             uint64_t* linesTouched) {
    const std::vector<Line>& L = right ? I.occR : I.occF;
    const uint64_t lo = right ? c.lbr : c.lb;
    const uint64_t hi = lo + c.len;
    if (linesTouched) *linesTouched += ((lo >> 6) == (hi >> 6)) ? 1 : 2;
    uint64_t occSum = 0;
    uint64_t rlo[6], occ[6];
    for (uint32_t s = 1; s < I.sigma; ++s) {
        rlo[s] = rankOf(L, s, lo);
        occ[s] = rankOf(L, s, hi) - rlo[s];
        occSum += occ[s];
    }
    uint64_t acc = (right ? c.lb : c.lbr) + (c.len - occSum);  // '$' first
    for (uint32_t s = 1; s < I.sigma; ++s) {
        if (right) out[s] = Cur{acc, I.C[s] + rlo[s], occ[s]};
        else       out[s] = Cur{I.C[s] + rlo[s], acc, occ[s]};
        acc += occ[s];
    }
}

// ------------------------------------------------------------ schemes ----

struct PSearch { std::vector<int> pi, l, u; };
using PScheme = std::vector<PSearch>;

static std::vector<int> orderFrom(int P, int j, bool rightFirst) {
    std::vector<int> o{j};
    if (rightFirst) {
        for (int t = j + 1; t < P; ++t) o.push_back(t);
        for (int t = j - 1; t >= 0; --t) o.push_back(t);
    } else {
        for (int t = j - 1; t >= 0; --t) o.push_back(t);
        for (int t = j + 1; t < P; ++t) o.push_back(t);
    }
    return o;
}

static void enumDist(int P, int minK, int maxK, std::vector<int>& cur,
                     std::vector<std::vector<int>>& out) {
    if ((int)cur.size() == P) {
        int s = 0;
        for (int v : cur) s += v;
        if (s >= minK && s <= maxK) out.push_back(cur);
        return;
    }
    int s = 0;
    for (int v : cur) s += v;
    for (int e = 0; s + e <= maxK; ++e) {
        cur.push_back(e);
        enumDist(P, minK, maxK, cur, out);
        cur.pop_back();
    }
}

// Greedy box construction ("h2" family restatement): candidate searches start
// at each part and go right-first or left-first; every error distribution is
// assigned to a candidate whose first part is error-free and that sees the
// errors as late as possible; bounds are the tightest box around the assigned
// cumulative error vectors. Complete by construction.
static PScheme genBox(int P, int minK, int maxK) {
    std::vector<std::vector<int>> cands;
    for (int j = 0; j < P; ++j)
        for (int rf = 1; rf >= 0; --rf) {
            auto o = orderFrom(P, j, rf);
            if (std::find(cands.begin(), cands.end(), o) == cands.end()) cands.push_back(o);
        }
    std::vector<std::vector<int>> dists, cur;
    std::vector<int> tmp;
    enumDist(P, minK, maxK, tmp, dists);
    std::vector<std::vector<int>> lo(cands.size(), std::vector<int>(P, 1 << 20)),
        hi(cands.size(), std::vector<int>(P, -1));
    std::vector<bool> used(cands.size(), false);
    for (auto& d : dists) {
        int best = -1;
        long bestCost = 0;
        for (size_t ci = 0; ci < cands.size(); ++ci) {
            auto& o = cands[ci];
            if (d[o[0]] != 0 && P > maxK) continue;
            long cost = 0;
            int cum = 0;
            for (int i = 0; i < P; ++i) { cum += d[o[i]]; cost += cum; }
            if (best < 0 || cost < bestCost) { best = (int)ci; bestCost = cost; }
        }
        auto& o = cands[best];
        int cum = 0;
        for (int i = 0; i < P; ++i) {
            cum += d[o[i]];
            lo[best][i] = std::min(lo[best][i], cum);
            hi[best][i] = std::max(hi[best][i], cum);
        }
        used[best] = true;
    }
    PScheme s;
    for (size_t ci = 0; ci < cands.size(); ++ci)
        if (used[ci]) s.push_back(PSearch{cands[ci], lo[ci], hi[ci]});
    return s;
}

// A published table: per search the 1-based part order, lower and upper
// cumulative bounds as digit strings, for errors in [0, K]; minK lifts the
// last lower bound.
struct TableRow { const char *pi, *l, *u; };
static PScheme fromTable(std::initializer_list<TableRow> rows, int minK) {
    PScheme out;
    for (const TableRow& r : rows) {
        PSearch s;
        for (const char* c = r.pi; *c; ++c) s.pi.push_back(*c - '1');
        for (const char* c = r.l; *c; ++c) s.l.push_back(*c - '0');
        for (const char* c = r.u; *c; ++c) s.u.push_back(*c - '0');
        s.l.back() = std::max(s.l.back(), minK);
        out.push_back(s);
    }
    return out;
}

// PEX hierarchical partition (Navarro and Raffinot 2002; Kärkkäinen and Na
// 2007) as a search scheme, restated with parent links: nodes over leaf
// ranges [lo, hi) with budget hi - lo - 1; top-down splits a node of budget e
// after floor(e / 2) + 1 leaves, bottom-up pairs neighbours level by level
// (an odd last node moves up as it is). Search of leaf j: leaf j exact, then
// for each ancestor, from the leaf's parent up, the parts of the ancestor not
// yet covered (the side the other child lies on, outward), cumulative errors
// <= the ancestor's budget; with lower bounds, a leaf under the right child
// requires the ancestor to hold more errors than the left child's budget.
static PScheme genPex(int K, int minK, bool bottomUp, bool lower) {
    struct N { int lo, hi, parent, leftChild; };
    std::vector<N> nd;
    std::vector<int> leafNode(K + 1, -1);
    if (!bottomUp) {
        std::vector<int> todo{0};
        nd.push_back({0, K + 1, -1, -1});
        while (!todo.empty()) {
            const int id = todo.back();
            todo.pop_back();
            const int lo = nd[id].lo, hi = nd[id].hi;
            if (hi - lo == 1) { leafNode[lo] = id; continue; }
            const int cut = lo + (hi - lo - 1) / 2 + 1;
            const int a = (int)nd.size();
            nd.push_back({lo, cut, id, -1});
            nd.push_back({cut, hi, id, -1});
            nd[id].leftChild = a;
            todo.push_back(a);
            todo.push_back(a + 1);
        }
    } else {
        std::vector<int> cur;
        for (int j = 0; j <= K; ++j) { leafNode[j] = (int)nd.size(); cur.push_back((int)nd.size()); nd.push_back({j, j + 1, -1, -1}); }
        while (cur.size() > 1) {
            std::vector<int> nxt;
            size_t i = 0;
            for (; i + 1 < cur.size(); i += 2) {
                const int id = (int)nd.size();
                nd.push_back({nd[cur[i]].lo, nd[cur[i + 1]].hi, -1, cur[i]});
                nd[cur[i]].parent = nd[cur[i + 1]].parent = id;
                nxt.push_back(id);
            }
            if (i < cur.size()) nxt.push_back(cur[i]);
            cur = nxt;
        }
    }
    PScheme out;
    for (int j = 0; j <= K; ++j) {
        PSearch s{{j}, {0}, {0}};
        int child = leafNode[j];
        for (int a = nd[child].parent; a >= 0; child = a, a = nd[a].parent) {
            const int budget = nd[a].hi - nd[a].lo - 1;
            const int last = s.l.back();
            if (nd[child].hi < nd[a].hi)
                for (int t = nd[child].hi; t < nd[a].hi; ++t) { s.pi.push_back(t); s.l.push_back(last); s.u.push_back(budget); }
            else
                for (int t = nd[child].lo - 1; t >= nd[a].lo; --t) { s.pi.push_back(t); s.l.push_back(last); s.u.push_back(budget); }
            const bool underRight = nd[a].leftChild != child;
            if (lower && underRight) {
                const N& L = nd[nd[a].leftChild];
                s.l.back() = std::max(s.l.back(), L.hi - L.lo);
            }
        }
        s.l.back() = std::max(s.l.back(), minK);
        out.push_back(s);
    }
    return out;
}

static bool makeScheme(const std::string& name, int minK, int maxK, PScheme& out) {
    if (minK < 0 || maxK < minK) return false;
    if (name == "pex-td" || name == "pex-td-l" || name == "pex-bu" || name == "pex-bu-l") {
        out = genPex(maxK, minK, name[4] == 'b', name.size() == 8);
        return true;
    }
    if (name == "kianfar") {  // Kianfar et al. 2018, the paper's optimum schemes for K <= 2
        if (maxK > 2) return false;
        if (maxK == 0) out = {PSearch{{0}, {0}, {0}}};
        else if (maxK == 1) out = fromTable({{"12", "00", "01"}, {"21", "01", "01"}}, minK);
        else out = fromTable({{"1234", "0011", "0022"}, {"3214", "0000", "1122"}, {"4321", "0002", "0122"}}, minK);
        return true;
    }
    const bool tableFamily = name == "lam" || name == "kucherov-k1" || name == "kucherov-k2";
    if (tableFamily && maxK > 2) return false;  // tables for k <= 2 only
    if (tableFamily && maxK == 0) {             // one exact search over the family's parts
        const int P = name == "kucherov-k2" ? 2 : 1;
        out = {PSearch{orderFrom(P, 0, true), std::vector<int>(P, 0), std::vector<int>(P, 0)}};
        return true;
    }
    if (name == "lam") {  // Lam et al. 2009 (as Kucherov, Salikhov, Tsur 2016 give it)
        out = maxK == 1 ? fromTable({{"12", "00", "01"}, {"21", "00", "01"}}, minK)
                        : fromTable({{"123", "000", "022"}, {"321", "000", "012"}, {"213", "001", "012"}}, minK);
        return true;
    }
    if (name == "kucherov-k1") {
        out = maxK == 1 ? fromTable({{"12", "00", "01"}, {"21", "01", "01"}}, minK)
                        : fromTable({{"123", "000", "022"}, {"321", "000", "012"}, {"213", "001", "012"}}, minK);
        return true;
    }
    if (name == "kucherov-k2") {
        out = maxK == 1 ? fromTable({{"123", "000", "011"}, {"321", "001", "001"}}, minK)
                        : fromTable({{"1234", "0000", "0122"}, {"4321", "0001", "0122"}, {"2341", "0012", "0012"}},
                                    minK);
        return true;
    }
    if (name == "pigeon_opt" || name == "suffix") {
        // both: K + 1 parts, search j = part j, then the parts right of it,
        // then the parts left of it (nearest first)
        const int P = maxK + 1;
        out.clear();
        for (int j = 0; j < P; ++j) {
            PSearch s;
            s.pi = orderFrom(P, j, true);
            for (int i = 0; i < P; ++i) {
                const bool rightSweep = i < P - j;          // part j itself and the parts right of it
                const int r = rightSweep ? 0 : i - (P - j) + 1;  // r-th part of the left sweep
                if (name == "pigeon_opt") {   // parts left of the lowest error-free part j: >= 1 error each
                    s.l.push_back(i == 0 ? 0 : r);
                    s.u.push_back(i == 0 ? 0 : (rightSweep ? maxK - j : maxK - j + r));
                } else {                      // suffix filter: t + 1 parts of the suffix hold <= t errors
                    s.l.push_back(0);
                    s.u.push_back(rightSweep ? i : maxK);
                }
            }
            s.l[P - 1] = std::max(s.l[P - 1], minK);
            out.push_back(s);
        }
        return true;
    }
    if (name == "01*0") {  // K + 2 parts; one search per seed 0 1^t 0 (Vroland et al. 2016)
        const int P = maxK + 2;
        out.clear();
        for (int i = 0; i < P; ++i)
            for (int t = 0; t <= maxK && i + t + 2 <= P; ++t) {
                PSearch s;
                s.pi = orderFrom(P, i, true);
                for (int x = 0; x < P; ++x) {
                    if (x == 0) { s.l.push_back(0); s.u.push_back(0); }
                    else if (x <= t) { s.l.push_back(x); s.u.push_back(x); }    // one error per middle part
                    else if (x == t + 1) { s.l.push_back(t); s.u.push_back(t); } // the closing error-free part
                    else { s.l.push_back(t); s.u.push_back(maxK); }
                }
                s.l[P - 1] = std::max(s.l[P - 1], minK);
                out.push_back(s);
            }
        return true;
    }
    if (name == "backtracking") {
        out = {PSearch{{0}, {minK}, {maxK}}};
        return true;
    }
    if (name == "pigeon") {
        const int P = maxK + 1;
        out.clear();
        for (int j = 0; j < P; ++j) {
            PSearch s;
            s.pi = orderFrom(P, j, true);
            for (int i = 0; i < P; ++i) {
                s.l.push_back(i == P - 1 ? minK : 0);
                s.u.push_back(i == 0 ? 0 : maxK);
            }
            out.push_back(s);
        }
        return true;
    }
    if (name == "h2-k1" || name == "h2-k2" || name == "h2-k3") {
        const int extra = name[4] - '0';
        out = genBox(maxK + extra, minK, maxK);
        return true;
    }
    return false;
}

static bool coversDist(const PSearch& s, const std::vector<int>& d) {
    int cum = 0;
    for (size_t i = 0; i < s.pi.size(); ++i) {
        cum += d[s.pi[i]];
        if (cum < s.l[i] || cum > s.u[i]) return false;
    }
    return true;
}

struct ESearch { std::vector<uint32_t> pi, l, u; };

static bool expandSearch(const PSearch& s, uint32_t len, ESearch& e) {
    const int P = (int)s.pi.size();
    if (len < (uint32_t)P) return false;
    std::vector<uint32_t> cnt(P), start(P);
    for (int t = 0; t < P; ++t) cnt[t] = len / P + ((uint32_t)t < len % P ? 1 : 0);
    uint32_t acc = 0;
    for (int t = 0; t < P; ++t) { start[t] = acc; acc += cnt[t]; }
    e = ESearch{};
    for (int i = 0; i < P; ++i) {
        const int t = s.pi[i];
        const bool asc = (i == 0) ? (P == 1 || s.pi[1] > s.pi[0]) : (s.pi[i] > s.pi[i - 1]);
        for (uint32_t j = 0; j < cnt[t]; ++j) {
            e.pi.push_back(asc ? start[t] + j : start[t] + cnt[t] - 1 - j);
            e.u.push_back((uint32_t)s.u[i]);
            e.l.push_back((uint32_t)(j + 1 == cnt[t] ? s.l[i] : (i > 0 ? s.l[i - 1] : 0)));
        }
    }
    return true;
}

static void limitHamming(ESearch& e) {
    const size_t m = e.pi.size();
    for (size_t p = 0; p < m; ++p) e.u[p] = std::min<uint32_t>(e.u[p], (uint32_t)p + 1);
    for (size_t p = m - 1; p-- > 0;)
        if (e.l[p + 1] > 0) e.l[p] = std::max<uint32_t>(e.l[p], e.l[p + 1] - 1);
}

// --------------------------------------------------------------- search ----

enum : uint8_t { OP_NONE = 0, OP_MS = 1, OP_I = 2, OP_D = 3 };

struct Leaf { uint64_t qid, lb, len, e; };

struct Searcher {
    const Index& I;
    const uint8_t* P;
    uint32_t m;
    const uint32_t *pi, *l, *u;
    const uint8_t* dir;  // 1 = extend right
    bool edit;
    uint64_t qid;
    std::vector<Leaf>* leaves;
    orc_counters* cnt;

    void visit(const Cur& cur, uint32_t pos, uint32_t e, uint8_t lastL, uint8_t lastR) {
        if (pos == m) {
            leaves->push_back(Leaf{qid, cur.lb, cur.len, e});
            return;
        }
        cnt->nodes++;
        const uint32_t q = pi[pos];
        const bool right = dir[pos];
        const uint8_t cq = P[q];
        const uint8_t side = right ? lastR : lastL;
        const bool matchOK = l[pos] <= e && e <= u[pos];
        const bool misOK = l[pos] <= e + 1 && e + 1 <= u[pos];
        const bool delOK = edit && pos > 0 && e + 1 <= u[pos] && side != OP_I;
        const bool insOK = edit && misOK && side != OP_D;
        auto nl = [&](uint8_t op) { return pos == 0 ? op : (right ? lastL : op); };
        auto nr = [&](uint8_t op) { return pos == 0 ? op : (right ? op : lastR); };
        if (matchOK || misOK || delOK) {
            Cur ch[6];
            cnt->rank_nodes++;
            extendAll(I, cur, right, ch, &cnt->ext_lines);
            for (uint32_t c = 1; c < I.sigma; ++c) {
                if (ch[c].len == 0) continue;
                if (c == cq) {
                    if (matchOK) visit(ch[c], pos + 1, e, nl(OP_MS), nr(OP_MS));
                } else if (misOK) {
                    visit(ch[c], pos + 1, e + 1, nl(OP_MS), nr(OP_MS));
                }
                if (delOK) visit(ch[c], pos, e + 1, nl(OP_D), nr(OP_D));
            }
        }
        if (insOK) visit(cur, pos + 1, e + 1, nl(OP_I), nr(OP_I));
    }
};

static inline bool isSampled(const Index& I, uint64_t row) {
    return (I.sampled[row >> 6] >> (row & 63)) & 1ull;
}

static uint64_t locateRow(const Index& I, uint64_t row, uint64_t& steps) {
    uint64_t st = 0;
    while (!isSampled(I, row)) {
        const uint8_t c = I.bwtF[row];
        row = I.C[c] + rankOf(I.occF, c, row);
        ++st;
    }
    const uint64_t o = row & 63;
    const uint64_t mask = o ? (~0ull >> (64 - o)) : 0ull;
    const uint64_t k = I.sampledRank[row >> 6] + (uint64_t)__builtin_popcountll(I.sampled[row >> 6] & mask);
    steps += st;
    return (uint64_t)I.samples[k] + st;
}

static void toSeq(const Index& I, uint64_t gpos, uint64_t& seqId, uint64_t& seqPos) {
    auto it = std::upper_bound(I.recStart.begin(), I.recStart.end(), gpos);
    seqId = (uint64_t)(it - I.recStart.begin()) - 1;
    seqPos = gpos - I.recStart[seqId];
}

static std::vector<uint8_t> dirsOf(const uint32_t* pi, uint32_t m) {
    std::vector<uint8_t> d(m);
    for (uint32_t p = 1; p < m; ++p) d[p] = pi[p] > pi[p - 1];
    d[0] = m > 1 ? d[1] : 1;
    return d;
}

static void searchRange(const Index& I, const uint8_t* pats, uint64_t q0, uint64_t q1, uint32_t m,
                        const uint32_t* pi, const uint32_t* l, const uint32_t* u, uint32_t nsearch,
                        bool edit, bool locate, std::vector<uint64_t>& out, orc_counters& cnt) {
    std::vector<std::vector<uint8_t>> dirs(nsearch);
    for (uint32_t s = 0; s < nsearch; ++s) dirs[s] = dirsOf(pi + (size_t)s * m, m);
    std::vector<Leaf> leaves;
    for (uint64_t q = q0; q < q1; ++q) {
        leaves.clear();
        for (uint32_t s = 0; s < nsearch; ++s) {
            Searcher S{I, pats + q * m, m, pi + (size_t)s * m, l + (size_t)s * m, u + (size_t)s * m,
                       dirs[s].data(), edit, q, &leaves, &cnt};
            S.visit(Cur{0, 0, I.n}, 0, 0, OP_NONE, OP_NONE);
        }
        cnt.leaves += leaves.size();
        for (const Leaf& lf : leaves) {
            if (!locate) {
                out.insert(out.end(), {lf.qid, lf.lb, lf.len, lf.e});
                continue;
            }
            for (uint64_t r = lf.lb; r < lf.lb + lf.len; ++r) {
                uint64_t gpos = locateRow(I, r, cnt.lf_steps), sid, sp;
                toSeq(I, gpos, sid, sp);
                out.insert(out.end(), {lf.qid, sid, sp, lf.e});
                cnt.rows++;
            }
        }
    }
}

// ---------------------------------------------------------- brute force ----

static int64_t bruteforce(const uint8_t* ranks, const uint64_t* recLens, uint64_t nrec,
                          const uint8_t* pats, uint64_t npat, uint32_t m, uint32_t k, bool edit,
                          std::vector<uint64_t>& out) {
    const int INF = 1 << 28;
    for (uint64_t q = 0; q < npat; ++q) {
        const uint8_t* P = pats + q * m;
        uint64_t off = 0;
        for (uint64_t r = 0; r < nrec; ++r) {
            const uint8_t* T = ranks + off;
            const uint64_t L = recLens[r];
            for (uint64_t p = 0; p < L; ++p) {
                int best = INF;
                if (!edit) {
                    if (p + m <= L) {
                        int mm = 0;
                        for (uint32_t i = 0; i < m && mm <= (int)k; ++i) mm += P[i] != T[p + i];
                        best = mm;
                    }
                } else {
                    const uint64_t W = std::min<uint64_t>((uint64_t)m + k, L - p);
                    // A: last text char consumed diagonally; B: horizontally (D).
                    std::vector<int> A((m + 1) * (W + 1), INF), B((m + 1) * (W + 1), INF);
                    auto at = [&](uint32_t i, uint64_t j) { return i * (W + 1) + j; };
                    for (uint64_t j = 1; j <= W; ++j) {
                        for (uint32_t i = 0; i <= m; ++i) {
                            int a = INF, b = INF;
                            if (i > 0) {
                                int prev = (j == 1) ? (int)(i - 1)
                                                    : std::min(A[at(i - 1, j - 1)], B[at(i - 1, j - 1)]);
                                a = prev + (P[i - 1] != T[p + j - 1] ? 1 : 0);
                                a = std::min(a, A[at(i - 1, j)] + 1);
                                b = B[at(i - 1, j)] + 1;
                            }
                            if (j >= 2) b = std::min(b, std::min(A[at(i, j - 1)], B[at(i, j - 1)]) + 1);
                            A[at(i, j)] = std::min(a, INF);
                            B[at(i, j)] = std::min(b, INF);
                        }
                        best = std::min(best, A[at(m, j)]);
                    }
                }
                if (best <= (int)k) out.insert(out.end(), {q, r, p, (uint64_t)best});
            }
            off += L;
        }
    }
    return (int64_t)(out.size() / 4);
}

// ------------------------------------------------------------- idx file ----
// Layout (cereal BinaryArchive conventions: host-endian scalars, containers
// prefixed by a u64 element count, std::array without prefix). The first
// field, size_t sigma, is the one the reference pins (index.cpp:98,
// search.cpp:278-283). The payload is this build's own (docs/idx_format.md).

static const uint64_t IDX_MAGIC = 0x3178646961726173ull;  // "sarahidx1" tag, little-endian

template <typename T> static void wr(std::ofstream& o, const T& v) { o.write((const char*)&v, sizeof(T)); }
template <typename T> static void wrVec(std::ofstream& o, const std::vector<T>& v) {
    uint64_t n = v.size();
    wr(o, n);
    o.write((const char*)v.data(), (std::streamsize)(n * sizeof(T)));
}
template <typename T> static void rd(std::ifstream& i, T& v) { i.read((char*)&v, sizeof(T)); }
template <typename T> static void rdVec(std::ifstream& i, std::vector<T>& v) {
    uint64_t n = 0;
    rd(i, n);
    v.resize(n);
    i.read((char*)v.data(), (std::streamsize)(n * sizeof(T)));
}

}  // namespace orc

using namespace orc;

struct orc_index : Index {};

extern "C" {

orc_index* orc_build(const uint8_t* ranks, const uint64_t* rec_lens, uint64_t nrec, uint32_t sigma,
                     uint32_t sampling_rate) {
    if ((sigma != 5 && sigma != 6) || nrec == 0 || sampling_rate == 0) return nullptr;
    Index* I = build(ranks, rec_lens, nrec, sigma, sampling_rate);
    auto* o = new orc_index();
    static_cast<Index&>(*o) = std::move(*I);
    delete I;
    return o;
}

orc_index* orc_from_parts(uint32_t sigma, uint64_t n, const uint64_t* rec_lens, uint64_t nrec,
                          uint32_t sampling_rate, const uint8_t* bwt_f, const uint8_t* bwt_r,
                          const uint64_t* sampled_bits, const uint32_t* samples, uint64_t nsamples) {
    auto* I = new orc_index();
    I->sigma = sigma;
    I->n = n;
    I->rate = sampling_rate;
    I->recLen.assign(rec_lens, rec_lens + nrec);
    I->bwtF.assign(bwt_f, bwt_f + n);
    I->bwtR.assign(bwt_r, bwt_r + n);
    I->sampled.assign(sampled_bits, sampled_bits + (n / 64 + 1));
    I->samples.assign(samples, samples + nsamples);
    I->C.assign(sigma + 1, 0);
    for (uint64_t i = 0; i < n; ++i) I->C[bwt_f[i] + 1]++;
    for (uint32_t c = 1; c <= sigma; ++c) I->C[c] += I->C[c - 1];
    finishIndex(*I);
    return I;
}

void orc_free(orc_index* idx) { delete idx; }
uint64_t orc_size(const orc_index* idx) { return idx->n; }
uint64_t orc_nsamples(const orc_index* idx) { return idx->samples.size(); }

int orc_export(const orc_index* I, uint8_t* bwt_f, uint8_t* bwt_r, uint32_t* sa,
               uint64_t* sampled_bits, uint32_t* samples, uint64_t* C) {
    if (bwt_f) std::memcpy(bwt_f, I->bwtF.data(), I->n);
    if (bwt_r) std::memcpy(bwt_r, I->bwtR.data(), I->n);
    if (sa) {
        if (I->sa.size() != I->n) return -1;
        std::memcpy(sa, I->sa.data(), I->n * 4);
    }
    if (sampled_bits) std::memcpy(sampled_bits, I->sampled.data(), I->sampled.size() * 8);
    if (samples) std::memcpy(samples, I->samples.data(), I->samples.size() * 4);
    if (C) std::memcpy(C, I->C.data(), I->C.size() * 8);
    return 0;
}

int orc_write_idx(const orc_index* I, const char* path) {
    std::ofstream o(path, std::ios::binary);
    if (!o) return -1;
    uint64_t sigma = I->sigma;
    wr(o, sigma);
    wr(o, IDX_MAGIC);
    wr(o, I->n);
    for (uint32_t c = 0; c <= I->sigma; ++c) wr(o, I->C[c]);
    wrVec(o, I->recLen);
    uint64_t rate = I->rate;
    wr(o, rate);
    wrVec(o, I->bwtF);
    wrVec(o, I->bwtR);
    wrVec(o, I->sampled);
    wrVec(o, I->samples);
    return o ? 0 : -1;
}

orc_index* orc_read_idx(const char* path) {
    std::ifstream i(path, std::ios::binary);
    if (!i) return nullptr;
    uint64_t sigma = 0, magic = 0, n = 0, rate = 0;
    rd(i, sigma);
    rd(i, magic);
    if (magic != IDX_MAGIC || (sigma != 5 && sigma != 6)) return nullptr;
    rd(i, n);
    std::vector<uint64_t> C(sigma + 1), recLen, sampled;
    std::vector<uint8_t> bf, br;
    std::vector<uint32_t> samples;
    for (auto& c : C) rd(i, c);
    rdVec(i, recLen);
    rd(i, rate);
    rdVec(i, bf);
    rdVec(i, br);
    rdVec(i, sampled);
    rdVec(i, samples);
    if (!i || bf.size() != n || br.size() != n) return nullptr;
    return orc_from_parts((uint32_t)sigma, n, recLen.data(), recLen.size(), (uint32_t)rate, bf.data(),
                          br.data(), sampled.data(), samples.data(), samples.size());
}

int orc_scheme(const char* generator, int min_k, int max_k, uint32_t len, int hamming, uint32_t* pi,
               uint32_t* l, uint32_t* u, int max_searches) {
    PScheme ps;
    if (!makeScheme(generator, min_k, max_k, ps)) return -1;
    if (!pi) return (int)ps.size();
    if ((int)ps.size() > max_searches) return -2;
    for (size_t s = 0; s < ps.size(); ++s) {
        ESearch e;
        if (!expandSearch(ps[s], len, e)) return -3;
        if (hamming) limitHamming(e);
        std::copy(e.pi.begin(), e.pi.end(), pi + s * len);
        std::copy(e.l.begin(), e.l.end(), l + s * len);
        std::copy(e.u.begin(), e.u.end(), u + s * len);
    }
    return (int)ps.size();
}

int orc_scheme_complete(const char* generator, int min_k, int max_k) {
    PScheme ps;
    if (!makeScheme(generator, min_k, max_k, ps)) return -1;
    const int P = (int)ps[0].pi.size();
    std::vector<std::vector<int>> dists;
    std::vector<int> tmp;
    enumDist(P, min_k, max_k, tmp, dists);
    for (auto& d : dists) {
        bool ok = false;
        for (auto& s : ps) ok = ok || coversDist(s, d);
        if (!ok) return 0;
    }
    return 1;
}

static int64_t runSearch(const orc_index* I, const uint8_t* pats, uint64_t npat, uint32_t m,
                         const uint32_t* pi, const uint32_t* l, const uint32_t* u, uint32_t nsearch,
                         int edit, int nthreads, bool locate, uint64_t** out, orc_counters* counters) {
    if (nthreads < 1) nthreads = 1;
    if ((uint64_t)nthreads > npat) nthreads = npat ? (int)npat : 1;
    std::vector<std::vector<uint64_t>> parts(nthreads);
    std::vector<orc_counters> cnts(nthreads);
    for (auto& c : cnts) std::memset(&c, 0, sizeof(c));
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t) {
        uint64_t q0 = npat * t / nthreads, q1 = npat * (t + 1) / nthreads;
        th.emplace_back([&, t, q0, q1] {
            searchRange(*I, pats, q0, q1, m, pi, l, u, nsearch, edit != 0, locate, parts[t], cnts[t]);
        });
    }
    for (auto& t : th) t.join();
    uint64_t total = 0;
    for (auto& p : parts) total += p.size();
    auto* buf = (uint64_t*)std::malloc(std::max<uint64_t>(total, 1) * 8);
    uint64_t o = 0;
    for (auto& p : parts) { std::memcpy(buf + o, p.data(), p.size() * 8); o += p.size(); }
    *out = buf;
    if (counters) {
        std::memset(counters, 0, sizeof(*counters));
        for (auto& c : cnts) {
            counters->nodes += c.nodes;
            counters->rank_nodes += c.rank_nodes;
            counters->ext_lines += c.ext_lines;
            counters->leaves += c.leaves;
            counters->rows += c.rows;
            counters->lf_steps += c.lf_steps;
        }
    }
    return (int64_t)(total / 4);
}

int64_t orc_search(const orc_index* I, const uint8_t* pats, uint64_t npat, uint32_t m,
                   const uint32_t* pi, const uint32_t* l, const uint32_t* u, uint32_t nsearch, int edit,
                   int nthreads, uint64_t** out, orc_counters* counters) {
    return runSearch(I, pats, npat, m, pi, l, u, nsearch, edit, nthreads, true, out, counters);
}

int64_t orc_search_cursors(const orc_index* I, const uint8_t* pats, uint64_t npat, uint32_t m,
                           const uint32_t* pi, const uint32_t* l, const uint32_t* u, uint32_t nsearch,
                           int edit, uint64_t** out) {
    return runSearch(I, pats, npat, m, pi, l, u, nsearch, edit, 1, false, out, nullptr);
}

int64_t orc_bruteforce(const uint8_t* ranks, const uint64_t* rec_lens, uint64_t nrec, const uint8_t* pats,
                       uint64_t npat, uint32_t m, uint32_t k, int edit, uint64_t** out) {
    std::vector<uint64_t> v;
    int64_t n = bruteforce(ranks, rec_lens, nrec, pats, npat, m, k, edit != 0, v);
    auto* buf = (uint64_t*)std::malloc(std::max<size_t>(v.size(), 1) * 8);
    std::memcpy(buf, v.data(), v.size() * 8);
    *out = buf;
    return n;
}

void orc_free_buf(void* p) { std::free(p); }

}  // extern "C"
