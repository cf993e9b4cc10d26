// scheme.cpp — search-scheme generation for the product (host side).
//
// Restates what sahara's `loadSearchScheme` needs from fmindex-collection
// (/root/reference/src/sahara/search.cpp:174-212, :226):
//   generator::all[name](minK, maxK, sigma, N)   part-level {pi, l, u}
//   expand(oss, len)                            per-position bounds
//   limitToHamming(scheme)                      Hamming tightening
//   nodeCount / weightedNodeCount               printed by search.cpp:197-198
// The upstream generator tables are not in the container,
// so the generators are this build's own, each complete for every error
// distribution in [minK, maxK] (tests/test_scheme.py checks that, and checks
// this file against the oracle's independent restatement).

#include <stdint.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <functional>
#include <initializer_list>
#include <string>
#include <vector>

namespace {

struct Part {
    std::vector<int> pi, l, u;
};

// connected orders starting at part `start`
std::vector<int> connected(int P, int start, bool rightFirst) {
    std::vector<int> o;
    o.reserve(P);
    o.push_back(start);
    int lo = start, hi = start;
    while ((int)o.size() < P) {
        const bool canR = hi + 1 < P, canL = lo > 0;
        if (canR && (rightFirst || !canL)) o.push_back(++hi);
        else o.push_back(--lo);
    }
    return o;
}

void distributions(int P, int minK, int maxK, std::vector<std::vector<int>>& out) {
    std::vector<int> d(P, 0);
    for (;;) {
        int s = 0;
        for (int v : d) s += v;
        if (s >= minK && s <= maxK) out.push_back(d);
        int i = P - 1;  // odometer over [0, maxK]^P, pruned by the sum
        while (i >= 0) {
            ++d[i];
            int t = 0;
            for (int v : d) t += v;
            if (t <= maxK) break;
            d[i] = 0;
            --i;
        }
        if (i < 0) break;
    }
}

// "h2" family: greedy box construction over connected candidate searches.
std::vector<Part> boxScheme(int P, int minK, int maxK) {
    std::vector<std::vector<int>> cand;
    for (int s = 0; s < P; ++s)
        for (bool rf : {true, false}) {
            auto o = connected(P, s, rf);
            if (std::find(cand.begin(), cand.end(), o) == cand.end()) cand.push_back(o);
        }
    std::vector<std::vector<int>> dist;
    distributions(P, minK, maxK, dist);
    const int INF = 1 << 20;
    std::vector<Part> box(cand.size());
    std::vector<char> used(cand.size(), 0);
    for (size_t c = 0; c < cand.size(); ++c) {
        box[c].pi = cand[c];
        box[c].l.assign(P, INF);
        box[c].u.assign(P, -1);
    }
    for (const auto& d : dist) {
        int best = -1;
        long bestCost = 0;
        for (size_t c = 0; c < cand.size(); ++c) {
            if (P > maxK && d[cand[c][0]] != 0) continue;  // first part error-free
            long cost = 0, acc = 0;
            for (int i = 0; i < P; ++i) cost += (acc += d[cand[c][i]]);
            if (best < 0 || cost < bestCost) { best = (int)c; bestCost = cost; }
        }
        long acc = 0;
        for (int i = 0; i < P; ++i) {
            acc += d[cand[best][i]];
            box[best].l[i] = std::min<int>(box[best].l[i], (int)acc);
            box[best].u[i] = std::max<int>(box[best].u[i], (int)acc);
        }
        used[best] = 1;
    }
    std::vector<Part> out;
    for (size_t c = 0; c < cand.size(); ++c)
        if (used[c]) out.push_back(box[c]);
    return out;
}

// A published table {pi (1-based digits), l, u} per search, for errors in
// [0, K]; minK raises the last lower bound (a search then reports only
// alignments with >= minK errors; completeness holds, the total is the last
// cumulative count).
std::vector<Part> table(std::initializer_list<const char*> rows, int minK) {
    std::vector<Part> out;
    for (const char* r : rows) {  // "123,000,022"
        Part p;
        const char* f[3] = {r, std::strchr(r, ',') + 1, std::strrchr(r, ',') + 1};
        for (const char* c = f[0]; *c != ','; ++c) p.pi.push_back(*c - '1');
        for (const char* c = f[1]; *c != ','; ++c) p.l.push_back(*c - '0');
        for (const char* c = f[2]; *c; ++c) p.u.push_back(*c - '0');
        p.l.back() = std::max(p.l.back(), minK);
        out.push_back(p);
    }
    return out;
}

// the order that starts at part j, sweeps right to the end, then left to 0
std::vector<int> rightThenLeft(int P, int j) {
    std::vector<int> o{j};
    for (int t = j + 1; t < P; ++t) o.push_back(t);
    for (int t = j - 1; t >= 0; --t) o.push_back(t);
    return o;
}

// K = 0 for a table family: one exact search over its P parts
std::vector<Part> exactOnly(int P) { return {Part{connected(P, 0, true), std::vector<int>(P, 0), std::vector<int>(P, 0)}}; }

// PEX: the hierarchical partition of Navarro and Baeza-Yates' filter (as
// Navarro and Raffinot, "Flexible Pattern Matching in Strings", 2002, and
// Kärkkäinen and Na state it), written as a search scheme. The K + 1 parts
// are the leaves of a binary tree; a node over leaves [a, b) may hold
// e = b - a - 1 errors, and its two children e1 and e2 with e1 + e2 + 1 = e,
// so one child of a node within its budget is within its own: some leaf is
// error-free and every node above it is within its budget. One search per
// leaf: the leaf exactly, then each ancestor's other child, nearest part
// first, bounded by that ancestor's budget. The tree is built top-down
// (a node of budget e splits into floor(e / 2) + 1 leaves on the left and the
// rest on the right) or bottom-up (leaves merged pairwise from the left,
// level by level, an odd last node carried up). With lower bounds (the -l
// names), ties go to the left child: a search whose leaf lies in the right
// child of a node sees the left child over its budget, so the node holds
// at least e1 + 1 errors once the search has covered it.
struct PexNode {
    int a, b;           // leaves [a, b)
    int left, right;    // children (-1: a leaf)
};

int pexTopDown(std::vector<PexNode>& t, int a, int b) {
    const int id = (int)t.size();
    t.push_back({a, b, -1, -1});
    if (b - a > 1) {
        const int e = b - a - 1, mid = a + e / 2 + 1;
        const int l = pexTopDown(t, a, mid);
        const int r = pexTopDown(t, mid, b);
        t[id].left = l;
        t[id].right = r;
    }
    return id;
}

int pexBottomUp(std::vector<PexNode>& t, int P) {
    std::vector<int> level;
    for (int j = 0; j < P; ++j) {
        level.push_back((int)t.size());
        t.push_back({j, j + 1, -1, -1});
    }
    while (level.size() > 1) {
        std::vector<int> up;
        for (size_t i = 0; i + 1 < level.size(); i += 2) {
            up.push_back((int)t.size());
            t.push_back({t[level[i]].a, t[level[i + 1]].b, level[i], level[i + 1]});
        }
        if (level.size() % 2) up.push_back(level.back());
        level.swap(up);
    }
    return level[0];
}

std::vector<Part> pexScheme(int maxK, int minK, bool bottomUp, bool lower) {
    const int P = maxK + 1;
    std::vector<PexNode> t;
    const int root = bottomUp ? pexBottomUp(t, P) : pexTopDown(t, 0, P);
    std::vector<Part> out;
    // depth-first over the tree with the path of (node, came from the right child)
    std::vector<std::pair<int, bool>> path;
    auto leafSearch = [&](int j) {
        Part p;
        p.pi = {j};
        p.l = {0};
        p.u = {0};
        int lo = j, hi = j + 1;  // parts covered
        for (size_t k = path.size(); k-- > 0;) {
            const PexNode& A = t[path[k].first];
            const int e = A.b - A.a - 1;
            const bool fromRight = path[k].second;
            const int before = (int)p.pi.size();
            for (; hi < A.b; ++hi) p.pi.push_back(hi);
            for (; lo > A.a; --lo) p.pi.push_back(lo - 1);
            for (int i = before; i < (int)p.pi.size(); ++i) {
                p.l.push_back(p.l.back());
                p.u.push_back(e);
            }
            if (lower && fromRight) {
                const PexNode& L = t[A.left];
                p.l.back() = std::max(p.l.back(), L.b - L.a);  // left child's budget + 1
            }
        }
        p.l.back() = std::max(p.l.back(), minK);
        out.push_back(p);
    };
    std::function<void(int)> walk = [&](int id) {
        const PexNode& n = t[id];
        if (n.left < 0) {
            leafSearch(n.a);
            return;
        }
        path.push_back({id, false});
        walk(n.left);
        path.back().second = true;
        walk(n.right);
        path.pop_back();
    };
    walk(root);
    return out;
}

bool generate(const std::string& name, int minK, int maxK, std::vector<Part>& out) {
    if (minK < 0 || maxK < minK || maxK > 15) return false;
    // Lam et al. 2009 (bidirectional BWT, k <= 2), as Kucherov, Salikhov and
    // Tsur (2016) state it: halves / thirds searched exactly first
    if (name == "lam") {
        if (maxK == 0) out = exactOnly(1);
        else if (maxK == 1) out = table({"12,00,01", "21,00,01"}, minK);
        else if (maxK == 2) out = table({"123,000,022", "321,000,012", "213,001,012"}, minK);
        else return false;
        return true;
    }
    // Kucherov, Salikhov and Tsur's search shapes (2016), K + 1 parts (k1) and
    // K + 2 parts (k2), K <= 2, with this build's bounds: k1 at K = 1 is
    // their non-redundant scheme, k1 at K = 2 is Lam's table as they print
    // it, and the K + 2 tables are this build's tightest bounds for their
    // three shapes (forward, backward, bidirectional from part 2). Upstream's
    // kucherov tables are not in the container: hits and node counts of these
    // names are unpinned against it
    if (name == "kucherov-k1") {
        if (maxK == 0) out = exactOnly(1);
        else if (maxK == 1) out = table({"12,00,01", "21,01,01"}, minK);
        else if (maxK == 2) out = table({"123,000,022", "321,000,012", "213,001,012"}, minK);
        else return false;
        return true;
    }
    if (name == "kucherov-k2") {
        if (maxK == 0) out = exactOnly(2);
        else if (maxK == 1) out = table({"123,000,011", "321,001,001"}, minK);
        else if (maxK == 2) out = table({"1234,0000,0122", "4321,0001,0122", "2341,0012,0012"}, minK);
        else return false;
        return true;
    }
    // pigeonhole with fewer redundant searches: search j starts at part j,
    // taken as the lowest error-free part, so the parts left of it hold >= 1
    // error each (swept last: cumulative >= r after r of them; cumulative
    // bounds cannot say "each", so some overlap stays) and the right sweep
    // <= K - j
    if (name == "pigeon_opt") {
        const int P = maxK + 1;
        out.clear();
        for (int j = 0; j < P; ++j) {
            Part p;
            p.pi = rightThenLeft(P, j);
            p.l.push_back(0);
            p.u.push_back(0);
            for (int t = j + 1; t < P; ++t) { p.l.push_back(0); p.u.push_back(maxK - j); }
            for (int r = 1; r <= j; ++r) { p.l.push_back(r); p.u.push_back(maxK - (j - r)); }
            p.l.back() = std::max(p.l.back(), minK);
            out.push_back(p);
        }
        return true;
    }
    // suffix filter (Karkkainen and Na 2007): with <= K errors in K + 1 parts
    // some part j starts a suffix whose first t + 1 parts hold <= t errors;
    // search j checks that prefix bound on its right sweep, then goes left
    if (name == "suffix") {
        const int P = maxK + 1;
        out.clear();
        for (int j = 0; j < P; ++j) {
            Part p;
            p.pi = rightThenLeft(P, j);
            for (int t = 0; t < P - j; ++t) { p.l.push_back(0); p.u.push_back(t); }
            for (int r = 0; r < j; ++r) { p.l.push_back(0); p.u.push_back(maxK); }
            p.l.back() = std::max(p.l.back(), minK);
            out.push_back(p);
        }
        return true;
    }
    // 01*0 seeds (Vroland et al. 2016): <= K errors in K + 2 parts leave two
    // error-free parts with only one-error parts between them; one search per
    // such seed (start part i, s - 2 one-error parts), seed first, then right,
    // then left
    if (name == "01*0") {
        const int P = maxK + 2;
        out.clear();
        for (int i = 0; i < P; ++i)
            for (int sl = 2; i + sl <= P; ++sl) {
                const int mid = sl - 2;
                if (mid > maxK) continue;
                Part p;
                for (int t = i; t < P; ++t) p.pi.push_back(t);
                for (int t = i - 1; t >= 0; --t) p.pi.push_back(t);
                p.l.push_back(0);
                p.u.push_back(0);
                for (int t = 1; t <= mid; ++t) { p.l.push_back(t); p.u.push_back(t); }
                p.l.push_back(mid);
                p.u.push_back(mid);
                while ((int)p.l.size() < P) { p.l.push_back(mid); p.u.push_back(maxK); }
                p.l.back() = std::max(p.l.back(), minK);
                out.push_back(p);
            }
        return true;
    }
    // Kianfar et al. 2018's optimum search schemes (ILP optimum for K = 1,
    // 2), as the paper tabulates them (1-based): K + 1 and K + 2 parts.
    // Restated for K <= 2 only (unpinned against upstream's table)
    if (name == "kianfar") {
        if (maxK == 0) out = exactOnly(1);
        else if (maxK == 1) out = table({"12,00,01", "21,01,01"}, minK);
        else if (maxK == 2) out = table({"1234,0011,0022", "3214,0000,1122", "4321,0002,0122"}, minK);
        else return false;
        return true;
    }
    if (name == "pex-td" || name == "pex-td-l" || name == "pex-bu" || name == "pex-bu-l") {
        out = pexScheme(maxK, minK, name.compare(0, 6, "pex-bu") == 0, name.size() == 8);
        return true;
    }
    if (name == "backtracking") {
        out = {Part{{0}, {minK}, {maxK}}};
        return true;
    }
    if (name == "pigeon") {
        out.clear();
        const int P = maxK + 1;
        for (int s = 0; s < P; ++s) {
            Part p;
            p.pi = connected(P, s, true);
            p.l.assign(P, 0);
            p.l[P - 1] = minK;
            p.u.assign(P, maxK);
            p.u[0] = 0;
            out.push_back(p);
        }
        return true;
    }
    if (name.size() == 5 && name.compare(0, 4, "h2-k") == 0 && name[4] >= '1' && name[4] <= '3') {
        out = boxScheme(maxK + (name[4] - '0'), minK, maxK);
        return true;
    }
    return false;
}

// in the reference's listing order (search_scheme.cpp:192). Every table here
// is this build's restatement of a published construction; upstream's tables
// are not in the container, so each is unpinned against upstream (hits under
// P-set are not: a complete scheme finds the same positions, tests/
// test_scheme.py). The names it lists beyond these (optimum, 01*0_opt, hato)
// have no published construction restatable offline and stay unknown
// (search.cpp:181's error).
const char* kNames[] = {"backtracking", "01*0", "pigeon", "pigeon_opt", "suffix", "h2-k1", "h2-k2", "h2-k3",
                        "kianfar", "kucherov-k1", "kucherov-k2", "lam", "pex-td", "pex-td-l", "pex-bu", "pex-bu-l"};
const char* kDescs[] = {"single part, errors anywhere",
                        "k+2 parts, one search per 0 1* 0 seed (Vroland et al.; this build's bounds)",
                        "k+1 parts, one exact part per search (pigeonhole)",
                        "k+1 parts, pigeonhole with this build's tightened bounds",
                        "k+1 parts, suffix filter (Karkkainen and Na; this build's bounds)",
                        "k+1 parts, this build's greedy-box scheme",
                        "k+2 parts, this build's greedy-box scheme (default)",
                        "k+3 parts, this build's greedy-box scheme",
                        "Kianfar et al. optimum search schemes (k <= 2, the paper's table)",
                        "k+1 parts, Kucherov, Salikhov and Tsur shapes, this build's bounds (k <= 2)",
                        "k+2 parts, Kucherov, Salikhov and Tsur shapes, this build's bounds (k <= 2)",
                        "Lam et al. bidirectional scheme (k <= 2)",
                        "k+1 parts, PEX hierarchical partition, tree built top-down",
                        "k+1 parts, PEX top-down with lower bounds (left child preferred)",
                        "k+1 parts, PEX hierarchical partition, tree built bottom-up",
                        "k+1 parts, PEX bottom-up with lower bounds (left child preferred)"};

// expand(oss, len) with explicit part sizes: inside a part the order follows
// the search direction; upper bounds hold for the whole part, lower bounds
// apply at the part's last position.
bool expandSizes(const Part& s, const std::vector<unsigned>& sizes, std::vector<unsigned>& pi,
                 std::vector<unsigned>& l, std::vector<unsigned>& u) {
    const unsigned P = (unsigned)s.pi.size();
    if (sizes.size() != P) return false;
    std::vector<unsigned> first(P + 1, 0);
    for (unsigned t = 0; t < P; ++t) {
        if (sizes[t] == 0) return false;
        first[t + 1] = first[t] + sizes[t];
    }
    pi.clear(); l.clear(); u.clear();
    for (unsigned i = 0; i < P; ++i) {
        const unsigned t = (unsigned)s.pi[i];
        const bool asc = i == 0 ? (P == 1 || s.pi[1] > s.pi[0]) : (s.pi[i] > s.pi[i - 1]);
        const unsigned a = first[t], b = first[t + 1];
        for (unsigned j = a; j < b; ++j) {
            pi.push_back(asc ? j : a + b - 1 - j);
            u.push_back((unsigned)s.u[i]);
            l.push_back(j + 1 == b ? (unsigned)s.l[i] : (i ? (unsigned)s.l[i - 1] : 0u));
        }
    }
    return true;
}

// uniform part sizes: len/P, +1 for the first len%P parts
std::vector<unsigned> uniformSizes(unsigned P, unsigned len) {
    std::vector<unsigned> z(P);
    for (unsigned t = 0; t < P; ++t) z[t] = len / P + (t < len % P ? 1u : 0u);
    return z;
}

bool expand(const Part& s, unsigned len, std::vector<unsigned>& pi, std::vector<unsigned>& l,
            std::vector<unsigned>& u) {
    const unsigned P = (unsigned)s.pi.size();
    if (len < P) return false;
    return expandSizes(s, uniformSizes(P, len), pi, l, u);
}

void toHamming(std::vector<unsigned>& l, std::vector<unsigned>& u) {
    const size_t m = l.size();
    for (size_t p = 0; p < m; ++p) u[p] = std::min<unsigned>(u[p], (unsigned)p + 1);
    for (size_t p = m - 1; p-- > 0;)
        if (l[p + 1] > 0) l[p] = std::max(l[p], l[p + 1] - 1);
}

// Tree size of one expanded search when every symbol exists (the reference
// prints nodeCount<Edit>(oss, sigma), search.cpp:197): DP over (pos, e) with
// (sigma-1) M/S edges, and for Edit one I edge and (sigma-1) D edges.
// weightedNodeCount additionally weights a node at text depth d by
// min(1, N / (sigma-1)^d), its expected number of occurrences in N random
// symbols (search.cpp:198).
void counts(const std::vector<unsigned>& l, const std::vector<unsigned>& u, bool edit, int sigma, double N,
            double& nodes, double& weighted) {
    const size_t m = l.size();
    const int A = std::max(1, sigma - 1);
    const unsigned K = 16;
    // f[pos][e][depth] would be large; depth only matters through the weight,
    // so track weighted and unweighted sums per (e, depth) on the fly.
    const size_t D = m + 16;
    std::vector<double> cur(K * D, 0.0), nxt(K * D, 0.0);
    cur[0] = 1.0;  // root: pos 0, e 0, depth 0
    nodes = 0;
    weighted = 0;
    auto w = [&](size_t d) { return std::min(1.0, N / std::pow((double)A, (double)d)); };
    for (size_t pos = 0; pos < m; ++pos) {
        // deletions stay at pos: propagate within the layer in increasing e
        if (edit) {
            for (unsigned e = 0; e + 1 <= u[pos] && e + 1 < K; ++e)
                for (size_t d = 0; d + 1 < D; ++d)
                    if (cur[e * D + d] > 0 && pos > 0) cur[(e + 1) * D + d + 1] += cur[e * D + d] * A;
        }
        std::fill(nxt.begin(), nxt.end(), 0.0);
        for (unsigned e = 0; e < K; ++e)
            for (size_t d = 0; d < D; ++d) {
                const double c = cur[e * D + d];
                if (c == 0) continue;
                nodes += c;
                weighted += c * w(d);
                if (d + 1 < D) {
                    if (l[pos] <= e && e <= u[pos]) nxt[e * D + d + 1] += c;               // M
                    if (l[pos] <= e + 1 && e + 1 <= u[pos] && e + 1 < K) {
                        nxt[(e + 1) * D + d + 1] += c * (A - 1);                         // S
                        if (edit) nxt[(e + 1) * D + d] += c;                             // I
                    }
                }
            }
        cur.swap(nxt);
    }
    for (double c : cur) nodes += c;  // leaves
}

// --dynamic_generator (expandByWNCTopDown, search.cpp:192-195,202-205): part
// sizes chosen to minimise the summed weighted node count of the scheme.
// The upstream optimiser is not in the container; this one starts
// from the uniform split and moves part boundaries (by 8, 4, 2, 1 positions)
// while the weighted node count drops. Hits do not depend on the sizes.
std::vector<unsigned> optimizeSizes(const std::vector<Part>& parts, unsigned len, bool edit, int sigma, double N) {
    const unsigned P = (unsigned)parts[0].pi.size();
    std::vector<unsigned> z = uniformSizes(P, len);
    auto cost = [&](const std::vector<unsigned>& sz) {
        double total = 0;
        std::vector<unsigned> pi, l, u;
        for (const Part& s : parts) {
            if (!expandSizes(s, sz, pi, l, u)) return 1e300;
            double a = 0, b = 0;
            counts(l, u, edit, sigma, N, a, b);
            total += b;
        }
        return total;
    };
    double best = cost(z);
    for (unsigned step : {8u, 4u, 2u, 1u}) {
        for (int iter = 0; iter < 4 * (int)len; ++iter) {
            double bestMove = best;
            std::vector<unsigned> bestZ;
            for (unsigned b = 0; b + 1 < P; ++b)
                for (int dir : {-1, 1}) {
                    std::vector<unsigned> t = z;
                    const unsigned from = dir > 0 ? b : b + 1, to = dir > 0 ? b + 1 : b;
                    if (t[from] <= step) continue;
                    t[from] -= step;
                    t[to] += step;
                    const double c = cost(t);
                    if (c < bestMove * (1 - 1e-6)) { bestMove = c; bestZ = t; }  // real gains only
                }
            if (bestZ.empty()) break;
            z = bestZ;
            best = bestMove;
        }
    }
    return z;
}

}  // namespace

extern "C" {

int sahara_scheme_dynamic(const char* generator, int min_k, int max_k, uint32_t len, int hamming, int edit,
                          int sigma, double text_len, uint32_t* part_sizes, int max_parts, uint32_t* pi,
                          uint32_t* l, uint32_t* u, int max_searches) {
    std::vector<Part> parts;
    if (!generator || !generate(generator, min_k, max_k, parts)) return -1;
    const int P = (int)parts[0].pi.size();
    if (!pi) return (int)parts.size();
    if ((int)parts.size() > max_searches || P > max_parts) return -2;
    if (len < (uint32_t)P) return -3;
    const std::vector<unsigned> z = optimizeSizes(parts, len, edit != 0, sigma, text_len);
    for (int t = 0; t < P; ++t) part_sizes[t] = z[t];
    std::vector<unsigned> PI, L, U;
    for (size_t s = 0; s < parts.size(); ++s) {
        if (!expandSizes(parts[s], z, PI, L, U)) return -3;
        if (hamming) toHamming(L, U);
        for (uint32_t j = 0; j < len; ++j) {
            pi[s * len + j] = PI[j];
            l[s * len + j] = L[j];
            u[s * len + j] = U[j];
        }
    }
    return (int)parts.size();
}


int sahara_scheme_generators(const char** names, const char** descs, int cap) {
    const int n = (int)(sizeof(kNames) / sizeof(kNames[0]));
    for (int i = 0; i < n && i < cap; ++i) {
        if (names) names[i] = kNames[i];
        if (descs) descs[i] = kDescs[i];
    }
    return n;
}

int sahara_scheme(const char* generator, int min_k, int max_k, uint32_t len, int hamming, uint32_t* pi,
                  uint32_t* l, uint32_t* u, int max_searches) {
    std::vector<Part> parts;
    if (!generator || !generate(generator, min_k, max_k, parts)) return -1;
    if (!pi) return (int)parts.size();
    if ((int)parts.size() > max_searches) return -2;
    std::vector<unsigned> P, L, U;
    for (size_t s = 0; s < parts.size(); ++s) {
        if (!expand(parts[s], len, P, L, U)) return -3;
        if (hamming) toHamming(L, U);
        for (uint32_t j = 0; j < len; ++j) {
            pi[s * len + j] = P[j];
            l[s * len + j] = L[j];
            u[s * len + j] = U[j];
        }
    }
    return (int)parts.size();
}

int sahara_scheme_parts(const char* generator, int min_k, int max_k, int* parts_out, int* pi, int* l, int* u,
                        int max_entries) {
    std::vector<Part> parts;
    if (!generator || !generate(generator, min_k, max_k, parts)) return -1;
    const int P = (int)parts[0].pi.size();
    if (parts_out) *parts_out = P;
    if (pi) {
        if ((int)parts.size() * P > max_entries) return -2;
        for (size_t s = 0; s < parts.size(); ++s)
            for (int i = 0; i < P; ++i) {
                pi[s * P + i] = parts[s].pi[i];
                l[s * P + i] = parts[s].l[i];
                u[s * P + i] = parts[s].u[i];
            }
    }
    return (int)parts.size();
}

int sahara_scheme_counts(const uint32_t* l, const uint32_t* u, uint32_t n_searches, uint32_t len, int edit,
                         int sigma, double text_len, double* node_count, double* weighted_node_count) {
    double nc = 0, wc = 0;
    for (uint32_t s = 0; s < n_searches; ++s) {
        std::vector<unsigned> L(l + (size_t)s * len, l + (size_t)(s + 1) * len),
            U(u + (size_t)s * len, u + (size_t)(s + 1) * len);
        double a = 0, b = 0;
        counts(L, U, edit != 0, sigma, text_len, a, b);
        nc += a;
        wc += b;
    }
    *node_count = nc;
    *weighted_node_count = wc;
    return 0;
}

}  // extern "C"
