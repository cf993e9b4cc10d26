/*
 * oracle.h — CPU restatement of sahara's search hot path.
 *
 * TEST INFRASTRUCTURE ONLY. Nothing in the product (sahara_amd/, include/,
 * the `sahara` CLI) links, loads or calls this code. Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg use it, and only
 * as the checker / the timed CPU baseline.
 *
 * What it restates (reference = /root/reference, seqan/sahara):
 *   - `sahara index` (src/sahara/index.cpp:41-112): FASTA ranks -> bidirectional
 *     FM-index, sampling rate 16 (index.cpp:87).
 *   - `sahara search` (src/sahara/search.cpp:104-274): search-scheme DFS
 *     (`fmc::search_ng24::search<Edit>`, search.cpp:227/230) and locate
 *     (`fmc::LocateLinear`, search.cpp:244-250).
 * The arithmetic lives in fmindex-collection v1.1.0 (cpm.dependencies:21-22),
 * which is not in the container; the semantics fixed here are the documented
 * policy P0 of docs/semantics.md. Parity against upstream is therefore
 * UNPINNED for the exact multiset; the hit set (P-set) is pinned by the
 * scheme-independent brute-force DP (orc_bruteforce) in this file.
 */
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_index orc_index;

typedef struct orc_counters {
    uint64_t nodes;      /* DFS nodes expanded (pos < len) */
    uint64_t rank_nodes; /* nodes that needed a rank (M/S/D allowed) */
    uint64_t ext_lines;  /* distinct 64-position Occ blocks touched by those ranks */
    uint64_t leaves;     /* reported (qid, cursor, e) records */
    uint64_t rows;       /* located SA rows (= hits) */
    uint64_t lf_steps;   /* LF steps taken during locate */
} orc_counters;

/* Build the bidirectional index from concatenated record ranks (no
 * delimiters; values 1..sigma-1) and per-record lengths. */
orc_index* orc_build(const uint8_t* ranks, const uint64_t* rec_lens, uint64_t nrec,
                     uint32_t sigma, uint32_t sampling_rate);
/* Build from exported parts (BWT of text and of the per-record reversed text,
 * sampled-row bitvector, SA samples in row order). */
orc_index* orc_from_parts(uint32_t sigma, uint64_t n, const uint64_t* rec_lens, uint64_t nrec,
                          uint32_t sampling_rate, const uint8_t* bwt_f, const uint8_t* bwt_r,
                          const uint64_t* sampled_bits, const uint32_t* samples, uint64_t nsamples);
void     orc_free(orc_index* idx);
uint64_t orc_size(const orc_index* idx);      /* n = text length incl. delimiters */
uint64_t orc_nsamples(const orc_index* idx);
/* Any pointer may be NULL. sa needs n entries (only for orc_build indexes). */
int orc_export(const orc_index* idx, uint8_t* bwt_f, uint8_t* bwt_r, uint32_t* sa,
               uint64_t* sampled_bits, uint32_t* samples, uint64_t* C);
int        orc_write_idx(const orc_index* idx, const char* path);
orc_index* orc_read_idx(const char* path);

/* Search schemes. Part-level generator output expanded to `len` positions.
 * Writes nsearch*len entries into each of pi/l/u (pass NULL to query the
 * count). Returns the number of searches or a negative error. */
int orc_scheme(const char* generator, int min_k, int max_k, uint32_t len, int hamming,
               uint32_t* pi, uint32_t* l, uint32_t* u, int max_searches);
/* 1 if the expanded scheme covers every error distribution in [min_k, max_k]
 * over `parts` parts (checked at part granularity, using the unexpanded scheme). */
int orc_scheme_complete(const char* generator, int min_k, int max_k);

/* Search + locate. Hits are written as 4 x uint64 (qid, seq_id, seq_pos, e),
 * unsorted, into *out (free with orc_free_buf). Returns the hit count. */
int64_t orc_search(const orc_index* idx, const uint8_t* pats, uint64_t npat, uint32_t m,
                   const uint32_t* pi, const uint32_t* l, const uint32_t* u, uint32_t nsearch,
                   int edit, int nthreads, uint64_t** out, orc_counters* counters);
/* Search only (no locate): leaves as 4 x uint64 (qid, lb, len, e). */
int64_t orc_search_cursors(const orc_index* idx, const uint8_t* pats, uint64_t npat, uint32_t m,
                           const uint32_t* pi, const uint32_t* l, const uint32_t* u, uint32_t nsearch,
                           int edit, uint64_t** out);

/* Scheme-independent brute force: for every (qid, seq_id, seq_pos) whose best
 * alignment has <= k errors, one record (qid, seq_id, seq_pos, min_e). */
int64_t orc_bruteforce(const uint8_t* ranks, const uint64_t* rec_lens, uint64_t nrec,
                       const uint8_t* pats, uint64_t npat, uint32_t m, uint32_t k, int edit,
                       uint64_t** out);

void orc_free_buf(void* p);

#ifdef __cplusplus
}
#endif
