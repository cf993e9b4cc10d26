/*
 * sahara_hip.h — C ABI of libsahara_hip.so, the MI355X (gfx950) drop-in for
 * sahara's search hot path.
 *
 * Reference interfaces this ABI replaces (paths under /root/reference):
 *   - fmc::BiFMIndex<Sigma, InterleavedBitvector16> load
 *       src/sahara/search.cpp:162-169           -> sahara_gpu_open / sahara_gpu_open_file
 *   - fmc::BiFMIndex{ref, samplingRate, threadNbr} construction + cereal save
 *       src/sahara/index.cpp:87-100             -> sahara_gpu_build / sahara_gpu_save
 *   - fmc::search_ng24::search<Edit>(index, queries, scheme, res_cb)
 *       src/sahara/search.cpp:218-231           -> sahara_gpu_search (search half)
 *   - fmc::LocateLinear{index, cursor}
 *       src/sahara/search.cpp:244-250           -> sahara_gpu_search (locate half)
 *   - search_n (--max_hits)  src/sahara/search.cpp:228,231 -> max_hits argument of sahara_gpu_search
 *   - search_ng21::search_best[_n]  src/sahara/search.cpp:233-241 -> sahara_gpu_search_best
 *
 * Conventions: plain C types only; 0 on success, negative on error with a
 * thread-local message from sahara_gpu_last_error(); no exceptions cross the
 * boundary. The caller owns every input buffer; the library owns `*hits`
 * until sahara_gpu_free. One context per device, used from one host thread.
 * Patterns are rank-encoded (ivsigma d_dna4/d_dna5 codes, 1..sigma-1), all of
 * the same length `len` (search.cpp:187 assumes this too), laid out
 * back-to-back. Qid i is the i-th pattern, exactly as in the reference's
 * `queries` vector (reverse complements interleaved by the caller,
 * search.cpp:121-123).
 *
 * Hits come back in canonical order: sorted by (qid, seq_id, pos, err). The
 * multiset equals the reference restatement's (one record per reported
 * cursor per located SA row; duplicates kept).
 */
#ifndef SAHARA_HIP_H
#define SAHARA_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* One located hit: query id, record id, 0-based position in the record,
 * number of errors of the reported alignment (search.cpp:246-248). 24 B. */
typedef struct sahara_hit {
    uint64_t qid;
    uint32_t seq_id;
    uint32_t err;
    uint64_t pos;
} sahara_hit;

typedef struct sahara_index_info {
    uint32_t sigma;          /* 5 (d_dna4) or 6 (d_dna5) */
    uint32_t sampling_rate;  /* SA sampling rate (16 in index.cpp:87) */
    uint64_t n;              /* text length incl. one delimiter per record */
    uint64_t n_records;
    uint64_t n_samples;
    uint64_t device_bytes;   /* HBM held by the resident index */
    uint32_t n_parts;        /* 1, or the parts of a text of >= 2^32 - 2 symbols (split at record boundaries) */
    uint32_t kmer_depth;     /* k-mer table depth (0: none) */
} sahara_index_info;

/* Per-run statistics of the last sahara_gpu_search / sahara_gpu_run call. */
typedef struct sahara_stats {
    uint64_t patterns;
    uint64_t batches;
    uint64_t cursors;        /* reported (qid, cursor, e) records */
    uint64_t hits;           /* located rows = hit records */
    double   search_ms;      /* device time of the search kernels (HIP events) */
    double   locate_ms;      /* device time of locate (incl. row-offset scan) */
    double   sort_ms;        /* device time of the canonical sort + decode */
    double   total_ms;       /* wall time of the whole call */
    /* Filled only by sahara_gpu_run(..., count=1): algorithmic work counters. */
    uint64_t nodes;          /* DFS nodes expanded */
    uint64_t rank_nodes;     /* nodes that ranked (M/S/D allowed) */
    uint64_t ext_lines;      /* distinct 64-position Occ lines those ranks touched */
    uint64_t lf_steps;       /* LF steps in locate */
    uint32_t search_launches;
    uint32_t search_grid;    /* workgroups per search launch */
    uint64_t text_nodes;     /* nodes expanded against the resident text (verify mode) */
    uint64_t conversions;    /* text tasks: rows of small intervals handed to the text phase */
    double   text_ms;        /* device time of the text-phase kernels (HIP events) */
    uint64_t fm_iterations;  /* wave iterations of the FM kernel (count=1) */
    uint64_t text_iterations;/* wave iterations of the text kernel (count=1) */
    uint64_t text_active;    /* sum of active lanes over text-kernel iterations (count=1) */
    uint64_t text_refills;   /* text-kernel iterations that refilled lanes (count=1) */
    uint64_t text_cycles_refill; /* shader cycles summed over text-kernel waves: task starts (count=1) */
    uint64_t text_cycles_step;   /* ... node / compare micro-steps (count=1) */
    uint64_t text_cycles_emit;   /* ... leaf emission (count=1) */
    uint64_t text_compare_steps; /* forced-run micro-steps, lane count (count=1) */
    uint32_t text_grid;          /* text-kernel workgroups per launch */
    uint32_t pipelined;          /* 1 if FM and text phases of consecutive batches overlapped */
    double   seed_ms;            /* starting cursors (k-mer table lookups) */
    uint64_t text_steps;         /* text-kernel micro-steps, lane count (count=1) */
    double   stage_ms;           /* host time of staging the patterns: 2- / 4-bit packing, rank check, H2D enqueue */
    double   output_ms;          /* sahara_gpu_search: wall time of handing the hits to the host */
    uint64_t text_launches;      /* text-phase kernel launches in the pass */
    uint64_t upload_chunks[3];   /* streamed upload chunks sent at 2 / 4 / 8 bits per symbol */
    uint64_t text_pos_tasks;     /* text tasks that came with their text position from the k-mer table (count=1) */
    uint64_t text_stolen;        /* nodes taken by idle lanes from busy lanes of their wave (count=1) */
    uint64_t reserved[8];        /* zero: room for counters added later without changing the struct's size */
} sahara_stats;

const char* sahara_gpu_last_error(void);
int  sahara_gpu_device_count(void);
/* The build id compiled into this library: the first 16 hex digits of the
 * SHA-256 over its sources (tools/build_id.py). Profiles record it, so that
 * a measurement can be matched to the build it measured. */
const char* sahara_build_id(void);

/* --- index residency (replaces the cereal load at search.cpp:162-169) --- */
/* idx_image: the bytes of a `.idx` file as written by `sahara index`. */
int  sahara_gpu_open(int device, const void* idx_image, size_t idx_bytes, void** ctx);
int  sahara_gpu_open_file(int device, const char* idx_path, void** ctx);
/* GPU index construction (replaces index.cpp:87): ranks = records
 * concatenated without delimiters, rec_lens[n_records]. */
int  sahara_gpu_build(int device, const uint8_t* ranks, const uint64_t* rec_lens, uint64_t n_records,
                      uint32_t sigma, uint32_t sampling_rate, void** ctx);
int  sahara_gpu_save(void* ctx, const char* path);          /* .idx writer (index.cpp:92-100) */
int  sahara_gpu_index_info(void* ctx, sahara_index_info* info);
/* Copy out the index parts (any pointer may be NULL): BWT of the text and of
 * the per-record reversed text (n bytes each), sampled-row bitvector
 * (n/64+1 words), SA samples (n_samples u32 text positions, row order),
 * C array (sigma+1 u64) and record lengths (n_records u64). */
int  sahara_gpu_export(void* ctx, uint8_t* bwt_f, uint8_t* bwt_r, uint64_t* sampled_bits,
                       uint32_t* samples, uint64_t* C, uint64_t* rec_lens);
/* Full suffix array and text (one symbol per byte, n entries) resident on the
 * device: built with the index or densified from the .idx samples (test hooks). */
int  sahara_gpu_export_sa(void* ctx, uint32_t* sa);
int  sahara_gpu_export_text(void* ctx, uint8_t* text);
/* Multi-part index (n_parts > 1): the part the export hooks above read
 * (default 0). Its records are the part's own, numbered from 0. */
int  sahara_gpu_select_part(void* ctx, uint32_t part);
/* sahara_gpu_index_info of one part (sahara_gpu_index_info: totals). */
int  sahara_gpu_part_info(void* ctx, uint32_t part, sahara_index_info* info);
/* Execution mode of the search (default verify = 1, locate_sa = 1):
 *   verify    1: once a DFS node's interval is a single row (SAHARA_SPLIT rows),
 *             resolve its text position through the resident SA and continue
 *             the identical DFS against the resident text (text phase);
 *             0: rank every node on the FM-index.
 *   locate_sa 1: locate rows by one read of the resident SA; 0: LF walk to
 *             the SA samples (fmc::LocateLinear, search.cpp:246).
 * The multiset of hits is the same in every mode. */
int  sahara_gpu_set_mode(void* ctx, int verify, int locate_sa);

/* --- search + locate (replaces search.cpp:218-250) ---
 * pi/l/u: the expanded search scheme, n_searches rows of len entries each
 * (fmc::search_scheme::expand output, search.cpp:191; limitToHamming already
 * applied by the caller for edit == 0, search.cpp:226).
 * max_hits > 0 is search_n (search.cpp:228,231): per query at most max_hits
 * distinct (seq_id, pos), fewest errors first, each once with its minimum e
 * (upstream's counting rule is unverified), applied per batch
 * on the device before the download. Hits come back sorted by
 * (qid, seq_id, pos, err) in a buffer released with sahara_gpu_free. */
int  sahara_gpu_search(void* ctx, const uint8_t* ranks, uint64_t n_patterns, uint32_t len,
                       const uint32_t* pi, const uint32_t* l, const uint32_t* u, uint32_t n_searches,
                       int edit, uint32_t max_hits, sahara_hit** hits, uint64_t* n_hits);
/* The same search from the reads themselves: query ingest's reverse-complement
 * interleave (search.cpp:121-127) runs on the device, so only the reads cross
 * PCIe. Qid 2i = read i, 2i + 1 = its reverse complement, as in the
 * reference's `queries`; reverse == 0 (--no-reverse) searches the reads as
 * given (qid i = read i). limit > 0 cuts the query list after the interleave
 * (--limit_queries). Requires a dna4 / dna5 index. Same hits, order and
 * ownership as sahara_gpu_search over the interleaved patterns. */
int  sahara_gpu_search_reads(void* ctx, const uint8_t* reads, uint64_t n_reads, uint32_t len, int reverse,
                             uint64_t limit, const uint32_t* pi, const uint32_t* l, const uint32_t* u,
                             uint32_t n_searches, int edit, uint32_t max_hits, sahara_hit** hits, uint64_t* n_hits);
/* Compact hit records: the same hits in 8 B each instead of 24, for callers
 * that turn them into text anyway (`sahara search` writes "qid seqId pos"):
 * a third of the device-to-host bytes, written by the device straight into
 * page-locked host memory batch by batch while later batches search. Record
 * i of block b (block_end[b-1] <= i < block_end[b], block_end[-1] = 0):
 *   qid    = block_qid0[b] + (recs[i] >> 36)
 *   text   = (recs[i] >> 4) & 0xFFFFFFFF   (position in the concatenated text)
 *   err    = recs[i] & 15
 *   seq_id = the r with rec_starts[r] <= text < rec_starts[r + 1]
 *   pos    = text - rec_starts[seq_id]
 * in canonical (qid, seq_id, pos, err) order. rec_starts (n_records + 1
 * entries, the last = the text length) belongs to the context and stays valid
 * until sahara_gpu_close; the rest is released by sahara_gpu_free_blocks. */
typedef struct sahara_hit_blocks {
    uint64_t* recs;
    uint64_t n_hits;
    uint64_t* block_qid0;
    uint64_t* block_end;
    uint64_t n_blocks;
    const uint64_t* rec_starts;
    uint64_t n_records;
} sahara_hit_blocks;
/* sahara_gpu_search_reads (max_hits = 0) with the hits as compact records.
 * Needs a single-part index (text < 2^32 symbols) and at most 15 errors. */
int  sahara_gpu_search_reads_compact(void* ctx, const uint8_t* reads, uint64_t n_reads, uint32_t len, int reverse,
                                     uint64_t limit, const uint32_t* pi, const uint32_t* l, const uint32_t* u,
                                     uint32_t n_searches, int edit, sahara_hit_blocks* out);
void sahara_gpu_free_blocks(sahara_hit_blocks* blocks);
/* The same searches from reads already two bits per symbol — the form
 * `sahara search`'s FASTA ingest produces (sahara_read_fasta form 2;
 * sahara_pack_2bit's layout): stream symbol s is bits 2 (s % 4) of
 * codes[s / 4], A C G T coded 0 1 2 3. Read i is the stream symbols
 * [sym0 + i * len, sym0 + (i + 1) * len) (sym0: a shard of a larger stream
 * may start inside a byte). dna5's N symbols are listed by stream position in
 * n_pos, strictly ascending (entries outside the reads are ignored; their
 * codes are ignored); a dna4 index takes none. The codes cross PCIe as given
 * (a quarter of the rank bytes) and the host does no per-symbol work; hits,
 * order, ownership and max_hits as sahara_gpu_search_reads[_compact]. */
int  sahara_gpu_search_packed(void* ctx, const uint8_t* codes, uint64_t sym0, const uint64_t* n_pos,
                              uint64_t n_count, uint64_t n_reads, uint32_t len, int reverse, uint64_t limit,
                              const uint32_t* pi, const uint32_t* l, const uint32_t* u, uint32_t n_searches,
                              int edit, uint32_t max_hits, sahara_hit** hits, uint64_t* n_hits);
int  sahara_gpu_search_packed_compact(void* ctx, const uint8_t* codes, uint64_t sym0, const uint64_t* n_pos,
                                      uint64_t n_count, uint64_t n_reads, uint32_t len, int reverse, uint64_t limit,
                                      const uint32_t* pi, const uint32_t* l, const uint32_t* u,
                                      uint32_t n_searches, int edit, sahara_hit_blocks* out);
/* Optional: a context's first search call does one-time work later calls
 * skip — the page-locked hit sink, the device buffers of the streamed pass.
 * A one-shot process (`sahara search`) can do it ahead, beside other work
 * (reading its queries): a sink for the hits of n_patterns patterns (as the
 * first compact call sizes it: two per pattern) pinned into the library's
 * pool, and the pass's device buffers for n_patterns patterns of length len
 * (0: unknown, those are left to the call). ctx NULL: the sink only (it
 * needs no device, so it can be pinned while the index loads). Results never
 * depend on it. */
int  sahara_gpu_prepare(void* ctx, uint64_t n_patterns, uint32_t len);
/* --search_mode besthits (search_ng21::search_best[_n], search.cpp:233-241):
 * n_schemes expanded schemes, scheme j covering exactly j errors, stored one
 * after another in pi/l/u (n_searches[j] rows of len entries each). A pattern's
 * hits are those of the first j that reports any; edit operations always on
 * (ng21 is the edit-distance search regardless of -d). max_hits as above. */
int  sahara_gpu_search_best(void* ctx, const uint8_t* ranks, uint64_t n_patterns, uint32_t len,
                            const uint32_t* pi, const uint32_t* l, const uint32_t* u,
                            const uint32_t* n_searches, uint32_t n_schemes, uint32_t max_hits,
                            sahara_hit** hits, uint64_t* n_hits);

/* Device-resident form of the same path for benchmarking: stage patterns and
 * scheme once, run search+locate+sort with results left in HBM, fetch later. */
int  sahara_gpu_stage(void* ctx, const uint8_t* ranks, uint64_t n_patterns, uint32_t len,
                      const uint32_t* pi, const uint32_t* l, const uint32_t* u, uint32_t n_searches,
                      int edit);
int  sahara_gpu_run(void* ctx, int count, uint64_t* n_hits);
int  sahara_gpu_fetch(void* ctx, sahara_hit* out, uint64_t capacity, uint64_t* n_hits);
/* The last run's hits, copied on the device into dst_device (device memory of
 * the context's GPU, >= capacity records) with qid_offset added to every qid:
 * rank-local -> global qids, ready for a gather of hit records across GPUs
 * (the reference is single-process, search.cpp:218-261). */
int  sahara_gpu_copy_hits(void* ctx, void* dst_device, uint64_t capacity, uint64_t qid_offset, uint64_t* n_hits);
/* Order-independent digest of the last run's hits (sum of a 64-bit mix of
 * each record) computed on the device. */
int  sahara_gpu_digest(void* ctx, uint64_t* digest);
int  sahara_gpu_stats(void* ctx, sahara_stats* stats);
/* Where a context runs: the HIP device it opened (SAHARA_DEVICE_MAP may remap
 * the device argument of sahara_gpu_open / _build, a test hook), the NUMA node
 * of that device (-1 unknown) and the number of host CPUs of that node the
 * context's own threads that touch its pinned buffers (finisher, hit
 * expander, ring pinning) are bound to (0: not bound; SAHARA_NUMA=0 turns
 * binding off). The packing threads read the caller's buffers and stay
 * unbound (SAHARA_PACK_BIND=1 binds them too). Any pointer may be NULL. */
int  sahara_gpu_placement(void* ctx, int* device, int* numa_node, int* n_cpus);

/* Releases a hit buffer returned by sahara_gpu_search / sahara_gpu_search_best.
 * Large buffers (>= 64 MB) are page-locked host memory; freeing one hands it
 * back to a small process-wide pool, so the next search of a similar size
 * writes into memory that is already pinned and faulted in. */
void sahara_gpu_free(void* p);
void sahara_gpu_close(void* ctx);
/* Page-locked host memory any context's DMA can read (NULL on failure, see
 * sahara_gpu_last_error). Packed reads kept in it (sahara_read_fasta's form 2
 * is) go up straight from there in sahara_gpu_search_packed[_compact],
 * without being copied through the library's staging ring: a quarter of the
 * host memory traffic of a rank-per-byte call. */
void* sahara_host_alloc(size_t bytes);
void sahara_host_free(void* p);

/* --- search schemes (replaces generator::all / expand / limitToHamming,
 * search.cpp:174-212, :226) --- */
/* Registered generator names/descriptions; returns the count. */
int  sahara_scheme_generators(const char** names, const char** descs, int cap);
/* Expanded scheme for `len`-long patterns: n_searches rows of len entries in
 * pi/l/u (pass pi == NULL to get the number of searches). hamming != 0 applies
 * limitToHamming. Returns the number of searches, -1 unknown generator/k,
 * -2 capacity, -3 len shorter than the number of parts. */
int  sahara_scheme(const char* generator, int min_k, int max_k, uint32_t len, int hamming,
                   uint32_t* pi, uint32_t* l, uint32_t* u, int max_searches);
/* --dynamic_generator (expandByWNCTopDown, search.cpp:192-195, 202-205):
 * like sahara_scheme, but the part sizes (written to part_sizes, one per part)
 * minimise the summed weighted node count for `sigma` and a text of text_len
 * symbols (edit != 0: counted with I/D edges). Returns the number of
 * searches; -1 unknown generator, -2 capacity, -3 len < parts. */
int  sahara_scheme_dynamic(const char* generator, int min_k, int max_k, uint32_t len, int hamming, int edit,
                           int sigma, double text_len, uint32_t* part_sizes, int max_parts, uint32_t* pi,
                           uint32_t* l, uint32_t* u, int max_searches);
/* Part-level (unexpanded) scheme: *parts = number of parts P; n_searches*P
 * entries per array. Returns the number of searches. */
int  sahara_scheme_parts(const char* generator, int min_k, int max_k, int* parts, int* pi, int* l, int* u,
                         int max_entries);
/* Node count / weighted node count of an expanded scheme (search.cpp:197-198). */
int  sahara_scheme_counts(const uint32_t* l, const uint32_t* u, uint32_t n_searches, uint32_t len, int edit,
                          int sigma, double text_len, double* node_count, double* weighted_node_count);

/* --- query ingest (replaces ivio::fasta::reader + ivs::convert_char_to_rank +
 * ivs::verify_rank, search.cpp:111-130; index.cpp:53-72) --- */
/* A FASTA file on `threads` host threads (0: OMP_NUM_THREADS, else all), in
 * form 1 (one rank per byte of data, 255 = no rank of the alphabet) or form 2
 * (two bits per symbol as sahara_gpu_search_packed takes them, N positions in
 * n_pos; data in page-locked memory, so the search calls DMA it directly). Records: symbols [offs[i], offs[i+1]). bad != 0: the first character
 * that is no rank of the alphabet is character bad_pos of record bad_record
 * (header bad_id), bad_char. Release with sahara_free_fasta. */
typedef struct sahara_fasta {
    uint8_t* data;
    uint64_t n_symbols;
    uint64_t* offs;
    uint64_t n_records;
    uint64_t* n_pos;
    uint64_t n_count;
    int bad;
    uint32_t bad_char;
    uint64_t bad_record;
    uint64_t bad_pos;
    char* bad_id;
} sahara_fasta;
int  sahara_read_fasta(const char* path, uint32_t sigma, int form, uint32_t threads, sahara_fasta* out);
void sahara_free_fasta(sahara_fasta* f);

/* --- synthetic inputs (host-side generators, BASELINE.md §2 / SURVEY §8(d)) --- */
/* Uniform i.i.d. ACGT records (ranks 1,2,3 and 4 (dna4) / 5 (dna5) for T),
 * std::mt19937_64(seed), 32 bases per draw. */
int  sahara_synth_reference(uint64_t seed, uint32_t sigma, const uint64_t* rec_lens, uint64_t n_records,
                            uint8_t* out_ranks);
/* read_simulator.cpp:119-240 restated: n_reads reads of exactly `len`
 * symbols sampled from the records with exactly `errors` transcript errors of
 * uniformly chosen type S/I/D each; read origin (record, pos) written to
 * origin[2*i], origin[2*i+1] when origin != NULL. */
int  sahara_synth_reads(const uint8_t* ranks, const uint64_t* rec_lens, uint64_t n_records, uint32_t sigma,
                        uint64_t n_reads, uint32_t len, uint32_t errors, uint64_t seed, uint8_t* out,
                        uint64_t* origin);
/* The same with the error types given as in `sahara read_simulator`
 * (--substitution_errors, --insertion_errors, --deletion_errors, -e):
 * fixed counts of S, I, D plus `errors` of uniformly chosen type. */
int  sahara_synth_reads_typed(const uint8_t* ranks, const uint64_t* rec_lens, uint64_t n_records, uint32_t sigma,
                              uint64_t n_reads, uint32_t len, uint32_t substitutions, uint32_t insertions,
                              uint32_t deletions, uint32_t errors, uint64_t seed, uint8_t* out, uint64_t* origin);
/* Host half of the streamed upload at two bits per symbol (test hook; the
 * search calls do this themselves): n ranks -> (n + 3) / 4 bytes in out,
 * symbol i at bits 2 (i % 4) of byte i / 4, A C G T coded 0 1 2 3; dna5's N
 * (rank 4 of sigma 6) is coded 0 and its position listed in n_pos (first
 * pos_cap of them), *n_count = how many. scalar: 0 the widest SIMD packer the
 * host has (AVX-512BW, else AVX2), 1 the scalar one, 2 AVX2 at most.
 * Returns 1 if a symbol is no rank in [1, sigma), 0 if all are, -1 on error. */
int  sahara_pack_2bit(const uint8_t* ranks, uint64_t n, uint32_t sigma, int scalar, uint8_t* out, uint32_t* n_pos,
                      uint64_t pos_cap, uint64_t* n_count);
/* Reverse complement interleave of search.cpp:121-123: out[2i] = read i,
 * out[2i+1] = its reverse complement (A<->T, C<->G, N->N). */
int  sahara_interleave_rc(const uint8_t* reads, uint64_t n_reads, uint32_t len, uint32_t sigma, uint8_t* out);

#ifdef __cplusplus
}
#endif
#endif /* SAHARA_HIP_H */
