/*
 * ragmi.h — C ABI of libragmi.so, the MI355X-native (gfx950) two-stage retrieval hot path.
 *
 * This is the drop-in boundary that replaces, for the reference
 * (pythonmailer/financial-rag-system, read-only at /root/reference):
 *   - the Qdrant server behind `QdrantClient.query_points` / `upsert` / `create_collection`
 *       main.py:92-95    get_qdrant()            -> rag_index_create
 *       main.py:215-239  retrieve_from_qdrant()  -> rag_index_search (one query per call, B=1)
 *       main2.py:160-163 retrieve_from_qdrant()  -> rag_index_search
 *       main2.py:281-295 batch_processor()       -> rag_index_search (B=32 in one call)
 *       ingest.py:86-96  ensure_collection()     -> rag_index_create (dim=384, COSINE)
 *       ingest.py:148-175 PointStruct + upsert   -> rag_index_upsert (row slots assigned by host)
 *       database.py:111-143 init_qdrant()        -> rag_index_create
 *   - the sentence-transformers encoders (see ragmi_bert.h).
 *
 * Conventions
 *   - All functions return 0 on success and a negative RAG_E* code on failure;
 *     rag_last_error() returns a thread-local message for the last failure on this thread.
 *   - "_dev" pointers are HIP device pointers (e.g. torch.Tensor.data_ptr() of a cuda tensor);
 *     "_host" pointers are host memory. Host buffers are caller-owned; device storage made by
 *     rag_index_create is handle-owned.
 *   - `stream` is a hipStream_t (torch.cuda.current_stream().cuda_stream); NULL = default stream.
 *     Device-pointer calls are asynchronous on `stream`; *_host calls are synchronous.
 *   - Handles are re-entrant: calls on one handle from several threads are serialised
 *     internally and each search uses its own workspace slot guarded by a HIP event, so
 *     concurrent searches on different streams are safe (main2.py runs up to 25 requests
 *     in flight through asyncio.to_thread, main2.py:52-53,218,228).
 *
 * Semantics (Qdrant COSINE collection, restated; see DESIGN.md §2 and oracle/scan_ref.c)
 *   - upsert: every vector is L2-normalised (canonical fp64 norm) to fp32,
 *     rounded to fp16 (RNE) and stored at its row slot; an existing slot is overwritten
 *     (md5 point ids make re-ingest idempotent, ingest.py:151-154).
 *   - search: the query is normalised the same way; score(row) = fp32(sum_k fp64(c_k)*fp64(q_k))
 *     with the canonical fp64 summation order (oracle/scan_ref.c); result = top-k rows by
 *     (score desc, row asc), optionally restricted per query to rows whose tag satisfies
 *     (tag & tag_mask) == tag_value (the payload `must` filter, main.py:218-236).
 *     Missing results (fewer than k matching rows) are reported as id -1, score -inf.
 */
#ifndef RAGMI_H
#define RAGMI_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  RAG_OK = 0,
  RAG_EINVAL = -1,   /* bad argument */
  RAG_EHIP = -2,     /* HIP runtime error */
  RAG_ENOMEM = -3,   /* device allocation failed */
  RAG_ERANGE = -4,   /* row slot beyond capacity, k too large, ... */
};

/* Largest k a single search may ask for (the reference uses limit=15, main.py:215).
 * Exactness is unconditional for every k <= RAG_MAX_K: the result is always the exact top-k
 * by (canonical score desc, row asc). The scan ranks rows by MFMA score (fp16 query, fp32
 * accumulation) and re-scores its approximate top-32 exactly; a per-query bound eps on
 * |MFMA score - exact score| (computed at query prep) certifies the result when the k-th
 * exact score exceeds the 32nd approximate score + eps. When it does not (near-duplicate
 * rows, k close to 32), every row whose MFMA score is >= (k-th exact score - eps) is
 * re-scored exactly, from the scan's per-wave lists when they provably hold all of them,
 * otherwise by a second pass over the shard (see rag_index_exactness_stats). */
#define RAG_MAX_K 32
/* Largest k of the large-k pass (round 5; Qdrant's query_points takes any `limit`,
 * main.py:215,232-237). RAG_MAX_K < k <= RAG_MAX_K_LARGE runs a separate exact pass per 32
 * queries: a sampled certified lower bound of each query's k-th best score, every row whose
 * MFMA score can reach it collected, all of those re-scored exactly, the k best by (score
 * desc, row asc) emitted — the same exact result and canonical scores as the k <= 32 path
 * (scan_kernels.hip, "Exact top-k for RAG_MAX_K < k"). rag_index_search_packed accepts k
 * up to this. rag_index_search itself takes ANY k >= 1: k > RAG_MAX_K_LARGE runs the full
 * exact pass (rag_index_search_full, round 6), and rag_merge_topk[_packed] merge any k (past
 * this by three stable radix sorts per query). */
#define RAG_MAX_K_LARGE 4096
/* Queries handled per scan pass; larger batches run ceil(B/32) passes. */
#define RAG_QUERY_TILE 32

typedef struct rag_index rag_index_t;

/* Last error message of the calling thread ("" if none). */
const char* rag_last_error(void);
/* Library version string. */
const char* rag_version(void);

/* Create an empty flat index of `dim`-dimensional vectors (dim % 32 == 0; 384 and 1024 are
 * built) with room for `capacity_rows` rows on HIP device `device`.
 * Replaces QdrantClient.create_collection(vectors_config=VectorParams(size, COSINE)),
 * ingest.py:86-96. */
int rag_index_create(int dim, int64_t capacity_rows, int device, rag_index_t** out);

/* Vector storage of an index. RAG_STORE_FP16: the normalised rows rounded to fp16 (RNE) —
 * the scan's operand, 2 B per element; scores are exact on the fp16 rows. RAG_STORE_FP32
 * (Qdrant's default Float32 datatype: VectorParams without `datatype`, database.py:124-130,
 * ingest.py:89-95): the normalised fp32 rows are kept as well (4 B more per element) and the
 * exact scores read them — score(row) = fp32(sum_k fp64(y_k) fp64(q_k)) over the fp32 row y,
 * ranking identical to an fp32 store — while the scan still streams the fp16 copy (the
 * certified select's error bound grows by ||fp16(y) - y|| <= 2^-11 ||y||). */
enum { RAG_STORE_FP16 = 0, RAG_STORE_FP32 = 1 };
/* Flag OR-ed into rag_index_create_ex's `storage` (and rag_encoder_create_ex's `flags`): the
 * process then honours the RAGMI_* environment knobs that switch kernels for A/B measurements
 * (scan / rescan grids, seed sample, GEMM and attention variants). Without it every knob reads
 * as its production default and a set knob is reported once on stderr. Diagnostic only:
 * several knobs trade the worst-case latency or the certificate's fallback for timing. */
#define RAG_CREATE_DIAGNOSTIC 0x100
/* The value the library uses for the integer knob `name` (a RAGMI_* variable): the variable's
 * value when it is set and diagnostics are on, else `dflt` (reporting an ignored variable
 * once on stderr). Runs the same code path as every knob site; for tests. */
int rag_knob_probe(const char* name, int dflt);
/* 1 in a diagnostic build of the library (-DRAGMI_DIAG_BUILD, out of tree: `python
 * ragmi/_build.py OUT.so -DRAGMI_DIAG_BUILD`), whose rag_bench_scan / rag_bert_attention also
 * carry the measured timing probes and kernel variants; 0 in the production libragmi.so
 * (rag_bench_scan variants 0 / 7, rag_bert_attention -1 / 42 / 10 only). */
int rag_diagnostic_build(void);
/* rag_index_create with an explicit storage (rag_index_create = RAG_STORE_FP16). */
int rag_index_create_ex(int dim, int64_t capacity_rows, int device, int storage,
                        rag_index_t** out);
/* RAG_STORE_FP16 / RAG_STORE_FP32 of an index (-1 for NULL). */
int rag_index_storage(const rag_index_t* index);
int rag_index_destroy(rag_index_t* index);

/* Grow capacity (keeps contents). */
int rag_index_reserve(rag_index_t* index, int64_t capacity_rows);
int64_t rag_index_capacity(const rag_index_t* index);
int64_t rag_index_count(const rag_index_t* index);
int rag_index_dim(const rag_index_t* index);

/* Write n vectors (fp32 [n][dim], device) into the row slots rows_dev[i] (int64, device);
 * tags_dev (uint32 [n], device) may be NULL (tag 0). `new_count` is the number of valid rows
 * after this upsert (rows >= new_count are ignored by search). Replaces qdrant.upsert,
 * ingest.py:171-175. */
int rag_index_upsert(rag_index_t* index, const float* vecs_dev, const int64_t* rows_dev,
                     const uint32_t* tags_dev, int64_t n, int64_t new_count, void* stream);
/* Same, host pointers, synchronous. */
int rag_index_upsert_host(rag_index_t* index, const float* vecs_host, const int64_t* rows_host,
                          const uint32_t* tags_host, int64_t n, int64_t new_count);

/* Top-k search of B queries (fp32 [B][dim], device). Outputs: out_scores_dev fp32 [B][k],
 * out_ids_dev int64 [B][k] (row + id_offset, or -1). filters_dev is NULL (no filter) or
 * uint32 [B][2] = (tag_mask, tag_value) per query: row r qualifies for query b iff
 * (tag[r] & tag_mask) == tag_value ((0,0) = every row). One scan serves a whole micro-batch
 * whose requests filter on different tickers (main2.py:228 per request).
 * Replaces QdrantClient.query_points, main.py:232-237. */
int rag_index_search(rag_index_t* index, const float* queries_dev, int B, int k,
                     const uint32_t* filters_dev, int64_t id_offset,
                     float* out_scores_dev, int64_t* out_ids_dev, void* stream);
/* rag_index_search by the full exact pass, for any k >= 1: per query every row is scored
 * exactly (the canonical fp64 order), the (score, row) pairs are radix-sorted (stable, score
 * descending, so ties stay row-ascending) and the first k emitted, -1 / -inf past the
 * matching rows. The same result as rag_index_search at every k; ~ms per query at 10M rows.
 * rag_index_search takes it for k > RAG_MAX_K_LARGE; callers take it to re-answer a query a
 * large-k pass left unanswered (rag_index_unanswered). No reference counterpart beyond
 * query_points(limit) itself (main.py:232-237). */
int rag_index_search_full(rag_index_t* index, const float* queries_dev, int B, int k,
                          const uint32_t* filters_dev, int64_t id_offset,
                          float* out_scores_dev, int64_t* out_ids_dev, void* stream);
/* Same, host pointers (filters_host may be NULL), synchronous. */
int rag_index_search_host(rag_index_t* index, const float* queries_host, int B, int k,
                          const uint32_t* filters_host, int64_t id_offset,
                          float* out_scores_host, int64_t* out_ids_host);

/* Multi-GPU exchange form of rag_index_search: the result is written as ONE array
 * out_packed [B][k][2] int32 = (fp32 score bits, global row id = local row + id_offset; -1
 * where fewer than k rows match), so the per-shard lists travel in a single all-gather.
 * Global row ids must stay below 2^31. */
int rag_index_search_packed(rag_index_t* index, const float* queries_dev, int B, int k,
                            const uint32_t* filters_dev, int64_t id_offset, int32_t* out_packed_dev,
                            void* stream);

/* Copy stored rows [row0, row0+n) out as row-major fp16 bits ([n][dim] uint16, host). */
int rag_index_export_rows(rag_index_t* index, int64_t row0, int64_t n, uint16_t* out_host);
/* Load already-stored rows back (persistence): row-major fp16 bits [n][dim] (host) are
 * written to rows [row0, row0+n) unchanged (no renormalisation), tags (host, may be NULL)
 * likewise; `new_count` = valid rows afterwards. Synchronous. */
int rag_index_import_rows(rag_index_t* index, int64_t row0, int64_t n, const uint16_t* rows_host,
                          const uint32_t* tags_host, int64_t new_count);
/* fp32 storage: copy the stored fp32 rows [row0, row0+n) out ([n][dim] float, host), and
 * load saved fp32 rows back (their fp16 scan copy is re-derived by the same RNE rounding, so
 * a reloaded index is bit-identical). rag_index_import_rows is refused on fp32 storage. */
int rag_index_export_rows32(rag_index_t* index, int64_t row0, int64_t n, float* out_host);
int rag_index_import_rows32(rag_index_t* index, int64_t row0, int64_t n, const float* rows_host,
                            const uint32_t* tags_host, int64_t new_count);
/* Copy stored tags of rows [row0, row0+n) to host. */
int rag_index_export_tags(rag_index_t* index, int64_t row0, int64_t n, uint32_t* out_host);

/* Merge n_lists per-shard result lists (each [B][k] sorted by (score desc, id asc), device;
 * laid out [n_lists][B][k]; padding: id -1) into the global top-k [B][k] (device) by (score
 * desc, id asc), padding -inf / -1 past the valid entries. Any k >= 1 (k > RAG_MAX_K_LARGE:
 * stream-ordered scratch of ~36 B per entry). Used after the RCCL all-gather of per-shard
 * results. */
int rag_merge_topk(const float* in_scores_dev, const int64_t* in_ids_dev, int n_lists, int B,
                   int k, float* out_scores_dev, int64_t* out_ids_dev, void* stream);
/* Same merge over the packed exchange form ([n_lists][B][k][2] int32, see
 * rag_index_search_packed) gathered from all shards. */
int rag_merge_topk_packed(const int32_t* in_packed_dev, int n_lists, int B, int k,
                          float* out_scores_dev, int64_t* out_ids_dev, void* stream);

/* Exactness bookkeeping (tests, bench): tier1 / tier2 = number of queries, since the index
 * was created, whose top-k was certified by the list re-scoring fallback / needed the second
 * pass over the shard (all other queries passed the error-bound check directly).
 * last_tiers (host, may be NULL when n_last == 0) receives, for the first n_last queries of
 * the most recent search PASS, 0 / 1 / 2 = the path that certified them (3 = marked for the
 * second pass but left unanswered, see rag_index_unanswered; -1 past the pass's
 * query count). Scope: a pass is one scan of <= 32 queries (<= 128 on the D = 1024 wide
 * scan); a search of more queries runs several passes and only its last one is reported, and
 * the state is per handle, so searches issued concurrently on several streams overwrite each
 * other's record (the tier1 / tier2 totals are exact in every case). Synchronises the device. */
int rag_index_exactness_stats(rag_index_t* index, int64_t* tier1, int64_t* tier2,
                              int32_t* last_tiers, int n_last);

/* Number of queries, since the index was created, that received NO result (-1 ids; their
 * last_tiers entry reads 3): k <= RAG_MAX_K passes whose second pass was skipped
 * (RAGMI_RESCAN_WG=0, honoured only under RAG_CREATE_DIAGNOSTIC), and large-k passes
 * (RAG_MAX_K < k <= RAG_MAX_K_LARGE) where more than 16384 rows tie within the MFMA error band
 * of a query's k-th best after the last collection round — possible in production (thousands
 * of identical chunks). Re-answer such queries with rag_index_search_full (the QdrantClient
 * front end does). Synchronises the device. */
int rag_index_unanswered(rag_index_t* index, int64_t* n);

/* Scan order across streams. serial = 1: each search pass's scan launch waits for the
 * previous pass's scan, whichever stream that ran on (one HIP event per handle), so passes
 * issued on several streams overlap their query prep, seed sampling and select with another
 * pass's scan while the HBM-bound scans themselves run one at a time (measured effective with
 * 2 streams; with 4 the traced scans still overlap). serial = 2: every pass hands
 * its scan to the handle's own scan stream and waits for it before select (two event hops
 * per pass; strictly one scan at a time). serial = 0 (default): passes on different streams
 * are unordered. No reference counterpart: the reference issues one HTTP search per query
 * (main.py:232-237); this is serving-loop plumbing for main2.py:281-295's batch processor
 * with several batches in flight. */
int rag_index_set_scan_order(rag_index_t* index, int serial);
/* Spatial partition of the batches in flight (serving option): a HIP stream restricted to CU
 * share `part` of `parts` (contiguous CU ids, hipExtStreamCreateWithCUMask). Searches issued
 * on such a stream size their scan grids to the stream's CUs (one scan workgroup per CU), so
 * `parts` batches in flight on `parts` partition streams scan side by side on disjoint CUs.
 * Results are identical on any stream. Destroy with rag_stream_destroy. (The reference has no
 * counterpart: Qdrant serves concurrent searches from one server process, main2.py:281-295.) */
int rag_stream_create_cu_partition(int device, int part, int parts, void** stream);
/* The same with an explicit CU mask (`words` 32-bit words, bit i = CU id i as
 * hipExtStreamCreateWithCUMask numbers them). On MI355X bit i is a CU of XCD i % 8, and an
 * XCD whose bits are all clear runs on ALL its CUs, so the mask must enable at least one CU
 * of every XCD (else RAG_EINVAL); likewise rag_stream_create_cu_partition takes at most
 * n_cu / 8 parts. Round 6. */
int rag_stream_create_cu_mask(int device, const uint32_t* mask, int words, void** stream);
int rag_stream_destroy(void* stream);
/* Diagnostic build only (else RAG_EINVAL): n_wg one-wave workgroups on `stream`, each writing
 * its (XCC_ID, HW_ID) hardware registers to out_dev[2 * wg .. +1] — where a CU mask's
 * workgroups actually run. */
int rag_diag_cu_probe(void* stream, int n_wg, int32_t* out_dev);

/* Kernel timing hook for bench.py: average device time (ms) of `rag_index_search` scan-kernel
 * launches measured with HIP events on the launch stream. enable = 0 off; enable = n > 0 records
 * an event pair around every n-th scan launch (each record costs a few us of device idle
 * time, so bench.py samples instead of timing every pass). */
int rag_profile_enable(rag_index_t* index, int enable);
int rag_profile_scan_ms(rag_index_t* index, double* total_ms, int64_t* launches);
/* The same event pairs as intervals: start_ms[i] / end_ms[i] of the i-th recorded launch,
 * relative to the first recorded launch's start (cap entries at most; *launches = how many
 * were recorded), then clears them like rag_profile_scan_ms. With several batches in flight
 * the launches of different streams overlap in time; bench.py takes the union of these
 * intervals as the time the scan kernel occupied the device. */
int rag_profile_scan_intervals(rag_index_t* index, double* start_ms, double* end_ms, int64_t cap,
                               int64_t* launches);

/* Diagnostic: average device ms of `reps` launches of scan variant `variant` on the current
 * corpus with the first min(B,32) queries (dim 384 only). Variants: 0 production (seeded
 * thresholds), 1 unseeded, 2 contiguous per-wave tile ranges, 3 MFMA without top-k,
 * 4 loads only, 5 without non-temporal loads, 6 without the load sched-barrier, 7 production
 * with every seed at +inf (top-k compares only), 8 the VALU ablation: v_dot2_f32_f16 instead
 * of MFMA over a row-group-major copy of the corpus, same top-k; 9 / 10 / 11 the dynamic tile
 * queue with chunks of 2 / 1 / 4 tiles, 12 dynamic (2) loads only, 13 / 14 static production
 * / loads only (9-14 time every launch on its own event pair), 15 production without the
 * end-of-scan sort of pending-only queries (timing probe), 16 production with the round-1
 * end-of-scan sort (A/B). dim 1024: variants 0-4 of
 * the wide (33-128 query) scan. The production library accepts variants 0 and 7 only (dim
 * 1024: 0); the others are compiled into the diagnostic build (rag_diagnostic_build). */
int rag_bench_scan(rag_index_t* index, const float* queries_dev, int B, int variant, int reps,
                   double* avg_ms);

#ifdef __cplusplus
}
#endif

#endif /* RAGMI_H */
