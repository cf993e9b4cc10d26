// shard.h — how `sahara search --gpus N` splits the query list over devices.
//
// The reference builds one query list (search.cpp:111-127): per read its
// forward pattern and, unless --no-reverse, its reverse complement, then cuts
// the list at --limit_queries. Device g gets a contiguous range of reads, so
// a read and its reverse complement stay on one device and the qids of all
// devices concatenate in order; sahara_gpu_search_reads cuts
// its own share of the list at `limit`.
#pragma once
#include <algorithm>
#include <cstddef>

namespace sahara_cli {

struct QueryShard {
    size_t r0 = 0, r1 = 0;  // reads [r0, r1)
    size_t q0 = 0, q1 = 0;  // their queries [q0, q1) of the interleaved list: qid offset q0, limit q1 - q0
};

// nq = queries after the cut, per = patterns per read (2 with reverse complements, else 1)
inline QueryShard queryShard(size_t nq, size_t per, unsigned devices, unsigned g) {
    const size_t nreads = (nq + per - 1) / per;  // reads that contribute a query
    QueryShard s;
    s.r0 = nreads * g / devices;
    s.r1 = nreads * (g + 1) / devices;
    s.q0 = std::min(nq, per * s.r0);
    s.q1 = std::min(nq, per * s.r1);
    return s;
}

}  // namespace sahara_cli
