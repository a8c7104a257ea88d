// index_capi.hip — extern "C" boundary of the flat index (declared in include/ragmi.h).
//
// Host side of the Qdrant replacement: handle lifetime, capacity growth, workspace ring,
// kernel launch sequence of one search (qprep -> scan -> select). No compute runs
// on the host; every entry point either enqueues on the caller's stream or (for *_host)
// stages through device memory and synchronises.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdlib>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/ragmi.h"
#include "common_host.hpp"
#include "scan_kernels.hip"

#include <hipcub/hipcub.hpp>

using ragmi::half8;

namespace {

// Per-pass workspace slots. A slot is bound to the stream of its last pass: passes on the
// same stream are ordered by the stream itself, so the hot path records no events at all (an
// event record idles the queue for ~5 us between kernels). Up to kRing streams search
// concurrently without interference; a further stream drains the device once and rebinds
// the least recently used slot. (Round 4: 8 slots. With 4, a fifth stream in flight rebinds on
// every pass: 1.25M rows, 5-8 streams 137-141K qps; with 8, 5 / 6 / 8 streams 186-205K, and
// 4 streams stay the fastest at 209-210K, profiles/r04t_streams_hwqueues.jsonl.)
constexpr int kRing = 8;
constexpr int kMaxGroups = 4;   // query groups of 32 per pass (wide rows)

struct Workspace {
  float* qn = nullptr;
  half8* qfrag = nullptr;
  uint32_t* filt = nullptr;
  float* smax = nullptr;      // [kMaxLists][32] per-sample-wave maxima
  float* seed = nullptr;      // [32] seed thresholds
  float* part_s = nullptr;
  int* part_i = nullptr;
  float* heads_s = nullptr;   // [32][n_lists]
  int* heads_i = nullptr;
  int* heads_n = nullptr;
  int* progress = nullptr;      // [lists][groups] shared-group scan throttle words
  float* eps = nullptr;         // [groups][32] per-query |MFMA - exact| score bound (qprep)
  int* fb_tier = nullptr;       // [groups][32] certifying path per query of the last pass
  unsigned long long* fb_cnt = nullptr;   // [3] tier-1 / tier-2 / unanswered totals since creation
  int* tileq = nullptr;         // [8][kTileQStride] per-XCD tile-queue heads (dynamic scan)
  // tier-2 hand-off select -> rescan_kernel: (L, e_k) per query, the rescan workgroups' lists
  // [query][kRescanMaxWG][32] and the launch's arrival ticket (zero between passes)
  float* t2 = nullptr;
  float* t2_s = nullptr;
  int* t2_i = nullptr;
  int* t2_tk = nullptr;
  // large-k path (k > RAG_MAX_K; lk_* kernels), allocated on first use: sample maxima
  // [32][kLkSampleMax], per query thr / count / round flag, round flags, candidates
  // [32][kLkCap]
  float* lk_smax = nullptr;
  float* lk_thr = nullptr;
  int* lk_cnt = nullptr;
  int* lk_again = nullptr;
  int* lk_need = nullptr;
  int* lk_cand = nullptr;
  float* lk_es = nullptr;       // [32][kLkCap] exact scores of the candidates (lk_rescore)
  hipEvent_t ev_in = nullptr;   // scan-stream order: caller stream -> scan stream -> caller
  hipEvent_t ev_out = nullptr;
  hipStream_t owner = nullptr;  // stream of the last pass that used this slot
  int cus = 0;                  // CUs the owner stream may use (its CU mask; stream_cus)
  uint64_t cus_gen = 0;         // g_stream_gen when `cus` was read
  bool used = false;
  uint64_t tick = 0;            // last use (LRU rebinding)
};

struct ProfPair {
  hipEvent_t a, b;
};

}  // namespace

struct rag_index {
  int dim = 0;
  bool diagnostic = false;   // counted in ragmi::diagnostic_handles() (common_host.hpp)
  int device = 0;
  int64_t cap_rows = 0;   // multiple of 16
  int64_t count = 0;
  half8* corpus = nullptr;
  uint32_t* tags = nullptr;
  // storage (rag_index_create_ex): RAG_STORE_FP16 keeps only the scan's fp16 tile16 rows;
  // RAG_STORE_FP32 also the normalised fp32 rows (row-major [cap][dim]), which the exact
  // rescoring reads — Qdrant's default Float32 datatype
  int storage = RAG_STORE_FP16;
  float* rows32 = nullptr;
  int n_cu = 256;
  int max_wgs = 0;        // scan workgroups at full occupancy
  int scan_wgs = 0;       // D <= 384 scan grid cap: 3/4 of the CUs (launch_search_pass)
  int groups = 1;         // query groups of 32 per search pass
  std::mutex mu;
  Workspace ws[kRing];
  uint64_t ws_tick = 0;
  Workspace* last_ws = nullptr;   // workspace of the most recent search pass
  int last_bq = 0;                // its query count
  // host staging for *_host entry points
  void* stage = nullptr;
  size_t stage_bytes = 0;
  // profiling
  // scan order (rag_index_set_scan_order): when set, every scan launch waits for the
  // previous one (on whichever stream it ran), so passes on several streams overlap their
  // query prep / seeding / select with another pass's scan but never two scans
  // 0 free, 1 serial (event chain across the callers' streams), 2 serial on the handle's own
  // scan stream (each pass hands its scan to it and waits for it before select)
  int serial_scans = 0;
  hipStream_t scan_stream = nullptr;
  hipEvent_t scan_done = nullptr;
  hipStream_t scan_last = nullptr;
  bool scan_any = false;       // a scan has been chained since set_scan_order (scan_last may be
                               // the null stream, whose handle is nullptr)
  int prof = 0;                // 0 off; n > 0: time every n-th scan launch
  int64_t prof_seq = 0;
  std::vector<ProfPair> prof_pairs;
};

namespace {

int64_t round16(int64_t n) { return (n + 15) & ~int64_t(15); }

int alloc_corpus(rag_index* h, int64_t cap_rows, half8** corpus, uint32_t** tags) {
  const size_t cbytes = (size_t)cap_rows * h->dim * 2;
  RAG_HIP(hipMalloc(reinterpret_cast<void**>(corpus), std::max<size_t>(cbytes, 16)));
  if (hipMalloc(reinterpret_cast<void**>(tags), std::max<size_t>(cap_rows * 4, 16)) !=
      hipSuccess) {
    (void)hipFree(*corpus);
    return ragmi::fail(RAG_ENOMEM, "hipMalloc(tags) failed");
  }
  RAG_HIP(hipMemset(*corpus, 0, std::max<size_t>(cbytes, 16)));
  RAG_HIP(hipMemset(*tags, 0, std::max<size_t>(cap_rows * 4, 16)));
  return RAG_OK;
}

int ensure_stage(rag_index* h, size_t bytes) {
  if (h->stage_bytes >= bytes) return RAG_OK;
  if (h->stage) (void)hipFree(h->stage);
  h->stage = nullptr;
  h->stage_bytes = 0;
  RAG_HIP(hipMalloc(&h->stage, bytes));
  h->stage_bytes = bytes;
  return RAG_OK;
}

template <int D>
void launch_upsert(rag_index* h, const float* v, const int64_t* rows, const uint32_t* tags,
                   int64_t n, hipStream_t st) {
  ragmi::upsert_kernel<D><<<dim3((unsigned)n), dim3(64), 0, st>>>(
      v, rows, tags, h->corpus, h->tags, n, h->cap_rows, h->rows32);
}

// qprep's extra error-bound term for fp32 storage (scan_kernels.hip qprep_kernel): the exact
// score reads the fp32 row c32, the scan its fp16 rounding c: |sum (c - c32) qn| <=
// ||c - c32|| ||qn|| <= (2^-11 ||c32|| + 2^-25 sqrt(D)) (1 + 2^-20), ||c32|| <= 1 + 2^-20
double store_eps(const rag_index* h) {
  if (h->storage != RAG_STORE_FP32) return 0.0;
  return (0x1p-11 * (1.0 + 0x1p-20) + 0x1p-25 * std::sqrt((double)h->dim)) * (1.0 + 0x1p-20);
}

// Bumped by every rag_stream_create_cu_partition / rag_stream_destroy: a workspace's cached CU
// count is re-read when it changed, so a stream created later at a destroyed partition
// stream's address (with another mask, or none) never inherits the old count.
std::atomic<uint64_t> g_stream_gen{1};

// CUs a stream may run on: its CU mask (rag_stream_create_cu_partition gives each of the
// batches in flight its own share of the CUs), popcounted once per workspace binding; the null
// stream and unmasked streams -> every CU. The scan grids are sized to it (launch_search_pass).
int stream_cus(const rag_index* h, hipStream_t st) {
  if (!st) return h->n_cu;
  uint32_t mask[32] = {};
  const uint32_t words = (uint32_t)std::min(32, (h->n_cu + 31) / 32);
  if (hipExtStreamGetCUMask(st, words, mask) != hipSuccess) {
    (void)hipGetLastError();
    return h->n_cu;
  }
  int n = 0;
  for (uint32_t i = 0; i < words; ++i) n += __builtin_popcount(mask[i]);
  return n > 0 && n < h->n_cu ? n : h->n_cu;
}

// sample + thresh: seed thresholds for the scan (see sample_kernel). ~0.8% of the shard's
// tiles, spread evenly, at least 256 tiles (all of them for small shards).
// D <= 384 (one query group): qprep fused into the sample launch (qprep_sample_kernel);
// RAGMI_FUSED_PREP=0 (diagnostic A/B, ragmi::Knob) keeps the separate qprep launch
bool fused_prep() {
  static ragmi::Knob k("RAGMI_FUSED_PREP");
  return k.get(1) != 0;
}

// Workgroups of the tier-2 rescan launch: ~128 tiles each, at most one per CU. A marked pass
// streams the shard at the chip's rate with that many, and the idle launch (every pass) costs
// one dispatch per workgroup, each needing a CU with the rescan's 79 KB of LDS free beside the
// other streams' scans. Round 4 sweep (profiles/r04m_rescan_grid.jsonl), 1.25M rows, 4 in
// flight, qps / 4 marked queries' added ms at 1.25M / 10M rows: 512 workgroups (two per CU)
// 209.3K / 0.45 / 1.36, 256: 210.4K / 0.53 / 1.21, 128: 210.7K / 0.80 / 2.18.
// Round 6 A/B (profiles/r06_legs/r06af_*, r06ag_*): capped at the 64 CUs the 10M-row scan
// leaves free, the idle launch no longer waits beside the other batch's scan — 10M rows 29.03
// / 29.03K qps vs 28.93 / 28.21K — but the 1.25M-row line (partitioned streams) lost 0.7%
// (222.5 / 224.4K vs 223.1 / 226.9K) and a marked pass took 1.45 / 4.37 ms instead of 0.51 /
// 1.23 ms at 1.25M / 10M rows: the default stays.
// RAGMI_RESCAN_WG (diagnostic A/B) caps it; 0 = skip (queries left tier 3, unanswered).
int rescan_grid(const rag_index* h) {
  static ragmi::Knob k("RAGMI_RESCAN_WG");
  const int cap = k.get(ragmi::kRescanMaxWG);
  if (cap <= 0) return 0;
  const int64_t n_tiles = (h->count + 15) / 16;
  return (int)std::max<int64_t>(1, std::min<int64_t>({(int64_t)cap, (int64_t)ragmi::kRescanMaxWG,
                                                      (int64_t)h->n_cu, n_tiles / 128}));
}

// RAGMI_SAMPLE_DIV (diagnostic A/B): 1 / the sampled fraction of the shard's tiles
int sample_div() {
  static ragmi::Knob k("RAGMI_SAMPLE_DIV");
  return std::max(1, k.get(128));
}

template <int D, bool FILTER>
void launch_seed(rag_index* h, Workspace& w, int groups, hipStream_t st,
                 const float* q = nullptr, int Bq = 0, const uint32_t* filt_in = nullptr) {
  using namespace ragmi;
  const int n_tiles = (int)((h->count + 15) / 16);
  if (q) {     // fused: qprep inside the sample launch (also when there is nothing to sample)
    if constexpr (D <= 384) {
      const int div_f = sample_div();
      const int n_sample = n_tiles == 0 ? 0 : std::min({n_tiles, std::max(256, n_tiles / div_f),
                                                        kMaxSample});
      qprep_sample_kernel<D, FILTER><<<dim3(std::max(1, (n_sample + 7) / 8)), dim3(256), 0, st>>>(
          q, Bq, filt_in, w.qn, w.qfrag, w.filt, w.eps, store_eps(h), h->corpus, h->tags,
          (int)h->count, n_tiles, n_sample, w.smax);
      if (n_sample > 0)
        thresh_kernel<kMaxSample><<<dim3(kQ, 1), dim3(256), 0, st>>>(w.smax, n_sample, w.eps,
                                                                    w.seed);
    }
    return;
  }
  if (n_tiles == 0) return;   // the scan visits no tile; seeds are never read
  const int div = sample_div();
  // D = 1024 tiles are 32 KB and config 5 shards hold up to 3.1M of them: a 4096-tile cap
  // would sample 0.13% of a 50M-row shard and let ~25K rows per query past the seed
  constexpr int kCap = D > 384 ? kMaxSampleWide : kMaxSample;
  const int n_sample = std::min({n_tiles, std::max(256, n_tiles / div), kCap});
  if constexpr (D > 384)   // every query group in one pass over each sample tile
    sample_wide_kernel<D, FILTER><<<dim3((n_sample + 7) / 8), dim3(256), 0, st>>>(
        h->corpus, h->tags, w.filt, w.qfrag, (int)h->count, n_tiles, n_sample, w.smax, groups);
  else
    sample_kernel<D, FILTER><<<dim3((n_sample + 7) / 8, groups), dim3(256), 0, st>>>(
        h->corpus, h->tags, w.filt, w.qfrag, (int)h->count, n_tiles, n_sample, w.smax);
  thresh_kernel<kCap><<<dim3(kQ, groups), dim3(256), 0, st>>>(w.smax, n_sample, w.eps, w.seed);
}

template <int D>
int launch_search_pass(rag_index* h, Workspace& w, const float* q, int Bq, int k,
                       const uint32_t* filt, int64_t id_offset, float* out_s, int64_t* out_i,
                       int32_t* out_packed, hipStream_t st) {
  using namespace ragmi;
  // Bq <= 32 * h->groups queries: `groups` query groups of 32 (one for D <= 384)
  const int groups = (Bq + kQ - 1) / kQ;
  // fused qprep + sample only in free scan order (small shards, several scans overlapping):
  // there it is +1.1% (1.25M rows, 4 in flight, profiles/r03d_fused_prep_ab.jsonl); with the
  // scans chained (>= 4M rows) its 256-thread workgroups of ~180 registers, which cannot share a
  // CU with scan workgroups, landed between a scan's workgroups and stretched the scan launch
  // (10M rows: scan 0.76 vs 0.83 of the roofline, same qps, profiles/r03i_headline_prep_ab.jsonl)
  if (D <= 384 && groups == 1 && fused_prep() && h->serial_scans == 0) {
    if (filt)
      launch_seed<D, true>(h, w, groups, st, q, Bq, filt);
    else
      launch_seed<D, false>(h, w, groups, st, q, Bq, nullptr);
  } else {
    qprep_kernel<D><<<dim3(groups * kQ), dim3(64), 0, st>>>(q, Bq, filt, w.qn, w.qfrag, w.filt,
                                                            w.eps, store_eps(h));
    if (filt)
      launch_seed<D, true>(h, w, groups, st);
    else
      launch_seed<D, false>(h, w, groups, st);
  }
  const int64_t n_tiles = (h->count + 15) / 16;
  // D <= 384: queries in VGPRs, 2 workgroups per CU; wider rows: queries in LDS, 1 per CU,
  // R workgroups per query group (R % 8 == 0: XCD pairing of the groups, scan_lds_kernel)
  constexpr bool kLdsQ = D > 384;
  int grid;
  // a CU-partitioned stream (w.cus < n_cu): the same per-CU occupancy over its CUs only
  const bool part = w.cus > 0 && w.cus < h->n_cu;
  const int max_wgs = part ? 2 * w.cus : h->max_wgs;
  if constexpr (kLdsQ) {
    const int per_group = std::max(8, (max_wgs / 2 / groups) & ~7);
    const int need = (int)std::min<int64_t>(
        per_group, ((n_tiles + kLdsWaves - 1) / kLdsWaves + 7) & ~int64_t(7));
    grid = std::max(8, std::min(need, kMaxLists / kLdsWaves));
  } else {
    // One scan workgroup on 3/4 of the CUs (h->scan_wgs), not two on every CU: measured on
    // one MI355X (profiles/r03j_scan_wgs_*.jsonl, interleaved processes, 2 reps each) 10M rows
    // 27.19K qps / 83.0% of the HBM roofline at 512 workgroups -> 28.67-28.82K / 86.2-86.7% at
    // 192 (224: 86.0-86.6%, 256: 85.6-86.1%, 288: 66.2% — one CU in eight with a second
    // workgroup makes the launch wait on them —, 160: 82.9%, 128: 72.5%); 2.5M rows 99.3K ->
    // 103.1K; 1.25M rows with 4 in flight 189K -> 199K (union 0.71 -> 0.76). Fewer, longer
    // wave streams keep HBM as busy as twice as many, each wave's fixed start / end-of-scan
    // list work is paid by 768 waves instead of 2048 (select merges that many fewer lists), and
    // the free CUs take the other streams' query prep, sampling and select beside the scan
    // instead of behind it. RAGMI_SCAN_WGS overrides the cap (diagnostic A/B).
    static ragmi::Knob k_wgs("RAGMI_SCAN_WGS");
    const int wg_env = k_wgs.get(0) > 0 ? std::max(8, k_wgs.get(0)) : 0;
    // Filtered scans (a tag load and compare per row) keep two workgroups per CU: 10M rows,
    // per-query ticker filter, serial order: 26.8 / 27.0K qps at 512 vs 25.7 / 26.1K at 192
    // (scan 1.170 vs 1.21-1.24 ms, profiles/r03u_filtered_wgs.jsonl)
    // On a CU-partitioned stream (the batches in flight on disjoint CU sets) one workgroup per
    // CU of its share: 1.25M rows, 4 batches in flight on quarter-CU streams, 64 workgroups
    // 222-223K qps vs 205K at 48, 210-218K at 128, and 206-208K for 4 unpartitioned streams at
    // the default grid (scripts/diag/cu_partition.py, profiles/r05c_cu_partition.jsonl; bench lines
    // 222.7-223.3K vs 207.0-207.6K, profiles/r05d_partition_lines.jsonl)
    const int wg_cap = wg_env ? wg_env : filt ? max_wgs : part ? w.cus : h->scan_wgs;
    grid = (int)std::min<int64_t>(std::min(max_wgs, wg_cap),
                                  std::max<int64_t>(1, (n_tiles + 3) / 4));
    grid = std::min(grid, kMaxLists / kWavesPerWG);
  }
  const hipStream_t caller = st;
  if (h->serial_scans == 1) {
    if (!h->scan_done) RAG_HIP(hipEventCreateWithFlags(&h->scan_done, hipEventDisableTiming));
    // (keyed on scan_any, not on scan_last being non-null: a scan on the null stream leaves
    // scan_last == nullptr, and testing the handle let the next pass on another stream skip
    // its wait — the filtered 10M line's scans overlapped, traced: 2.2 ms launches, 1.24 ms
    // apart)
    if (h->scan_any && h->scan_last != st) RAG_HIP(hipStreamWaitEvent(st, h->scan_done, 0));
  } else if (h->serial_scans == 2) {
    if (!h->scan_stream) RAG_HIP(hipStreamCreateWithFlags(&h->scan_stream, hipStreamNonBlocking));
    if (!w.ev_in) RAG_HIP(hipEventCreateWithFlags(&w.ev_in, hipEventDisableTiming));
    if (!w.ev_out) RAG_HIP(hipEventCreateWithFlags(&w.ev_out, hipEventDisableTiming));
    RAG_HIP(hipEventRecord(w.ev_in, st));
    RAG_HIP(hipStreamWaitEvent(h->scan_stream, w.ev_in, 0));
    st = h->scan_stream;
  }
  ProfPair pp{};
  const bool timed = h->prof > 0 && (h->prof_seq++ % h->prof) == 0;
  if (timed) {
    RAG_HIP(hipEventCreate(&pp.a));
    RAG_HIP(hipEventCreate(&pp.b));
    // the LDS-query / wide scans (a memset + launch, or one launch): marker events around them;
    // the 384-d scan times its own dispatch (launch_fixed_timed below)
    if constexpr (kLdsQ) RAG_HIP(hipEventRecord(pp.a, st));
  }
#define RAG_SCAN_ARGS                                                                    \
  h->corpus, h->tags, w.filt, w.qfrag, (int)h->count, (int)n_tiles, w.seed, w.part_s, w.part_i, \
      w.heads_s, w.heads_i, w.heads_n
  const bool wide = kLdsQ && groups > 1 && !filt;
  if (wide) {
    // RAGMI_WIDE_WGS (diagnostic A/B): workgroup cap of the wide scan (default one per CU)
    static ragmi::Knob k_wide("RAGMI_WIDE_WGS");
    const int wide_env = k_wide.get(0) > 0 ? std::max(8, k_wide.get(0)) : 0;
    const int cap = wide_env ? std::min(wide_env, max_wgs / 2) : max_wgs / 2;
    grid = (int)std::min<int64_t>(cap, std::max<int64_t>(1, n_tiles));
  }
  if constexpr (kLdsQ) {
    const dim3 g3(grid * groups);
    if (wide) {
      // all groups in every workgroup, one pass over the corpus (scan_wide_kernel)
      // ring loads non-temporal (the corpus is read once per pass): 50M x 1024, B = 128
      // 70.3% -> 71.2% of the HBM roofline, loads-only 80.1% -> 85.8%
      // (profiles/r01h_wide_nt.jsonl). The diagnostic variants run only via rag_bench_scan.
      launch_fixed<kWideBlock>(scan_wide_kernel<D, 0, true>, dim3(grid), 0, st, h->corpus,
                               w.qfrag, (int)h->count, (int)n_tiles, w.seed, w.part_s,
                               w.part_i, w.heads_s, w.heads_i, w.heads_n, groups);
    } else if (groups == 1) {
      if (filt)
        launch_fixed<kLdsBlock>(scan_lds_kernel<D, true, true>, g3, 0, st, RAG_SCAN_ARGS, groups,
                                w.progress);
      else
        launch_fixed<kLdsBlock>(scan_lds_kernel<D, false, true>, g3, 0, st, RAG_SCAN_ARGS, groups,
                                w.progress);
    } else {
      RAG_HIP(hipMemsetAsync(w.progress, 0, (size_t)grid * kLdsWaves * groups * 4, st));
      if (filt)
        launch_fixed<kLdsBlock>(scan_lds_kernel<D, true, false>, g3, 0, st, RAG_SCAN_ARGS, groups,
                                w.progress);
      else
        launch_fixed<kLdsBlock>(scan_lds_kernel<D, false, false>, g3, 0, st, RAG_SCAN_ARGS, groups,
                                w.progress);
    }
  } else if (timed) {
    // the timed launch carries its own start / end timestamps (launch_fixed_timed)
    if (filt)
      RAG_HIP(launch_fixed_timed<kScanBlock>(scan_kernel<D, true>, dim3(grid), 0, st, pp.a, pp.b,
                                             RAG_SCAN_ARGS, nullptr));
    else
      RAG_HIP(launch_fixed_timed<kScanBlock>(scan_kernel<D, false>, dim3(grid), 0, st, pp.a, pp.b,
                                             RAG_SCAN_ARGS, nullptr));
  } else {
    if (filt)
      launch_fixed<kScanBlock>(scan_kernel<D, true>, dim3(grid), 0, st, RAG_SCAN_ARGS, nullptr);
    else
      launch_fixed<kScanBlock>(scan_kernel<D, false>, dim3(grid), 0, st, RAG_SCAN_ARGS, nullptr);
  }
#undef RAG_SCAN_ARGS
  if (timed) {
    if constexpr (kLdsQ) RAG_HIP(hipEventRecord(pp.b, st));
    h->prof_pairs.push_back(pp);
  }
  if (h->serial_scans == 1) {
    RAG_HIP(hipEventRecord(h->scan_done, st));
    h->scan_last = st;
    h->scan_any = true;
  } else if (h->serial_scans == 2) {
    RAG_HIP(hipEventRecord(w.ev_out, st));
    RAG_HIP(hipStreamWaitEvent(caller, w.ev_out, 0));
    st = caller;
  }
  const int n_lists = wide ? grid : grid * (kLdsQ ? kLdsWaves : kWavesPerWG);   // per group
  const ExactStats fb{w.fb_tier, w.fb_cnt, w.t2};
  // select certifies every query's top-k; its fallbacks (list re-scoring, a workgroup-local
  // second pass over the shard) run inside the same launch
#define RAG_SELECT(F)                                                                          \
  select_kernel<D, F><<<dim3(Bq), dim3(256), 0, st>>>(                                         \
      w.part_s, w.part_i, w.heads_s, w.heads_i, w.heads_n, n_lists, h->corpus, h->tags,      \
      w.filt, w.qfrag, (int)h->count, w.qn, k, w.eps, w.seed, fb, id_offset, out_s, out_i,   \
      out_packed, h->rows32)
  if (filt)
    RAG_SELECT(true);
  else
    RAG_SELECT(false);
#undef RAG_SELECT
  // tier 2 of the certificate (rescan_kernel): returns at once unless select marked a query
  // of the pass; otherwise its R workgroups stream the shard once per 16 marked queries.
  // RAGMI_RESCAN_WG (diagnostic A/B) caps R; 0 skips the launch, and mark_unanswered_kernel
  // then records the marked queries as unanswered (tier 3, rag_index_unanswered): timing only
  const int R = std::min(rescan_grid(h), part ? w.cus : h->n_cu);
  if (R > 0) {
#define RAG_RESCAN(F)                                                                   \
  launch_fixed<kScanBlock>(rescan_kernel<D, F>, dim3(R), 0, st, w.fb_tier, w.t2, Bq, h->corpus,  \
                           h->tags, w.filt, w.qfrag, (int)h->count, w.qn, k, w.eps, w.t2_s,  \
                           w.t2_i, w.t2_tk, id_offset, out_s, out_i, out_packed, h->rows32)
    if (filt)
      RAG_RESCAN(true);
    else
      RAG_RESCAN(false);
#undef RAG_RESCAN
  } else {
    mark_unanswered_kernel<<<dim3(1), dim3(64), 0, st>>>(w.fb_tier, Bq, w.fb_cnt);
  }
  RAG_HIP(hipGetLastError());
  return RAG_OK;
}

// One search pass of <= 32 queries for RAG_MAX_K < k <= RAG_MAX_K_LARGE (scan_kernels.hip,
// "Exact top-k for RAG_MAX_K < k"): qprep, a sample of the shard's tiles for the bound, then
// kLkRounds (collect, final) launch pairs; rounds after the first return at once unless a
// query's candidate list overflowed in the previous one.
int ensure_lk(Workspace& w) {
  using namespace ragmi;
  if (w.lk_cand) return RAG_OK;
  const size_t Q = kQ;
  // all seven or none: each buffer is allocated into a local and the workspace takes them only
  // when every allocation succeeded (a partial set would be re-allocated, and leaked, by the
  // next large-k call)
  void* p[7] = {};
  const size_t bytes[7] = {Q * kLkSampleMax * 4, Q * 4, Q * 4, Q * 4, 64, Q * kLkCap * 4,
                           Q * kLkCap * 4};
  for (int i = 0; i < 7; ++i) {
    if (hipMalloc(&p[i], bytes[i]) != hipSuccess) {
      (void)hipGetLastError();
      for (int j = 0; j < i; ++j) (void)hipFree(p[j]);
      return ragmi::fail(RAG_ENOMEM, "large-k workspace allocation failed");
    }
  }
  w.lk_smax = static_cast<float*>(p[0]);
  w.lk_thr = static_cast<float*>(p[1]);
  w.lk_cnt = static_cast<int*>(p[2]);
  w.lk_again = static_cast<int*>(p[3]);
  w.lk_need = static_cast<int*>(p[4]);
  w.lk_cand = static_cast<int*>(p[5]);
  w.lk_es = static_cast<float*>(p[6]);
  return RAG_OK;
}

// One search pass of <= 32 queries by the full exact path (scan_kernels.hip "Exact top-k
// for ANY k"): k > RAG_MAX_K_LARGE, or rag_index_search_full. Per query: exact scores of every
// row, a stable descending radix sort of (key, row), the first k emitted. The sort buffers
// (16 B per row + hipcub's scratch) are stream-ordered allocations released at the pass's end.
template <int D>
int launch_full_pass(rag_index* h, Workspace& w, const float* q, int Bq, int k,
                     const uint32_t* filt, int64_t id_offset, float* out_s, int64_t* out_i,
                     int32_t* out_packed, hipStream_t st) {
  using namespace ragmi;
  qprep_kernel<D><<<dim3(kQ), dim3(64), 0, st>>>(q, Bq, filt, w.qn, w.qfrag, w.filt, w.eps,
                                                  store_eps(h));
  RAG_HIP(hipGetLastError());
  const int n = (int)h->count;
  auto emit_grid = [&]() { return dim3((unsigned)std::min<int64_t>(1024, (k + 255) / 256)); };
  if (n == 0) {
    int* zero = nullptr;
    RAG_HIP(hipMallocAsync(reinterpret_cast<void**>(&zero), 4, st));
    RAG_HIP(hipMemsetAsync(zero, 0, 4, st));
    for (int j = 0; j < Bq; ++j)
      full_emit_kernel<<<emit_grid(), dim3(256), 0, st>>>(
          nullptr, nullptr, zero, k, id_offset, out_s ? out_s + (int64_t)j * k : nullptr,
          out_i ? out_i + (int64_t)j * k : nullptr,
          out_packed ? out_packed + (int64_t)j * k * 2 : nullptr);
    RAG_HIP(hipGetLastError());
    RAG_HIP(hipFreeAsync(zero, st));
    return RAG_OK;
  }
  size_t tmp_bytes = 0;
  RAG_HIP(hipcub::DeviceRadixSort::SortPairsDescending(
      nullptr, tmp_bytes, static_cast<const uint32_t*>(nullptr), static_cast<uint32_t*>(nullptr),
      static_cast<const int*>(nullptr), static_cast<int*>(nullptr), n, 0, 32, st));
  const size_t nb = (size_t)n * 4;
  char* buf = nullptr;
  const size_t m_off = 4 * nb, t_off = m_off + 256;
  RAG_HIP(hipMallocAsync(reinterpret_cast<void**>(&buf), t_off + tmp_bytes, st));
  uint32_t* k_in = reinterpret_cast<uint32_t*>(buf);
  uint32_t* k_out = reinterpret_cast<uint32_t*>(buf + nb);
  int* v_in = reinterpret_cast<int*>(buf + 2 * nb);
  int* v_out = reinterpret_cast<int*>(buf + 3 * nb);
  int* n_match = reinterpret_cast<int*>(buf + m_off);
  void* tmp = buf + t_off;
  RAG_HIP(hipMemsetAsync(n_match, 0, 4 * kQ, st));
  // one wave per 8 rows per step; up to 8 workgroups per CU
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(8 * h->n_cu, (n + 31) / 32));
  int rc = RAG_OK;
  for (int j = 0; j < Bq && rc == RAG_OK; ++j) {
    if (filt)
      full_score_kernel<D, true><<<dim3(grid), dim3(256), 0, st>>>(
          h->corpus, h->tags, w.filt + 2 * j, w.qn + (int64_t)j * D, n, h->rows32, k_in, v_in,
          n_match + j);
    else
      full_score_kernel<D, false><<<dim3(grid), dim3(256), 0, st>>>(
          h->corpus, h->tags, nullptr, w.qn + (int64_t)j * D, n, h->rows32, k_in, v_in,
          n_match + j);
    if (hipGetLastError() != hipSuccess ||
        hipcub::DeviceRadixSort::SortPairsDescending(tmp, tmp_bytes,
                                                     static_cast<const uint32_t*>(k_in), k_out,
                                                     static_cast<const int*>(v_in), v_out, n, 0,
                                                     32, st) != hipSuccess) {
      rc = ragmi::fail(RAG_EHIP, "full exact pass: score / sort launch failed");
      break;
    }
    full_emit_kernel<<<emit_grid(), dim3(256), 0, st>>>(
        k_out, v_out, n_match + j, k, id_offset, out_s ? out_s + (int64_t)j * k : nullptr,
        out_i ? out_i + (int64_t)j * k : nullptr,
        out_packed ? out_packed + (int64_t)j * k * 2 : nullptr);
    if (hipGetLastError() != hipSuccess) rc = ragmi::fail(RAG_EHIP, "full exact pass: emit");
  }
  // the pass certifies every query (tier 0) by construction
  (void)hipMemsetAsync(w.fb_tier, 0, 4 * kQ, st);
  (void)hipFreeAsync(buf, st);
  return rc;
}

// k > RAG_MAX_K_LARGE: per query, three stable radix sorts over the n_lists * k entries
// (scan_kernels.hip merge_any_*; the full pass's SortPairsDescending<uint32, int>, no other
// hipcub instantiation); stream-ordered scratch released at the end
template <bool PACKED>
int merge_any_k(const float* in_s, const int64_t* in_i, int n_lists, int B, int k, float* out_s,
                int64_t* out_i, hipStream_t st) {
  const int64_t n64 = (int64_t)n_lists * k;
  if (n64 > 0x7fffffff) return ragmi::fail(RAG_ERANGE, "merge: n_lists * k too large");
  const int n = (int)n64;
  size_t tmp = 0;
  RAG_HIP(hipcub::DeviceRadixSort::SortPairsDescending(
      nullptr, tmp, static_cast<const uint32_t*>(nullptr), static_cast<uint32_t*>(nullptr),
      static_cast<const int*>(nullptr), static_cast<int*>(nullptr), n, 0, 32, st));
  // keys in/out + positions in/out: 16 B per entry, + scratch (256-B aligned)
  const size_t nb = (size_t)n;
  char* buf = nullptr;
  const size_t t_off = (nb * 16 + 255) & ~(size_t)255;
  RAG_HIP(hipMallocAsync(reinterpret_cast<void**>(&buf), t_off + tmp, st));
  uint32_t* ka = reinterpret_cast<uint32_t*>(buf);
  uint32_t* kb = ka + nb;
  int* pa = reinterpret_cast<int*>(kb + nb);
  int* pb = pa + nb;
  void* scratch = buf + t_off;
  const dim3 g((unsigned)std::min<int64_t>(1024, (n64 + 255) / 256));
  const dim3 ge((unsigned)std::min<int64_t>(1024, ((int64_t)k + 255) / 256));
  auto sort = [&]() {   // (ka, pa) -> (kb, pb), stable, keys descending
    size_t t = tmp;
    return hipcub::DeviceRadixSort::SortPairsDescending(scratch, t,
                                                        static_cast<const uint32_t*>(ka), kb,
                                                        static_cast<const int*>(pa), pb, n, 0, 32,
                                                        st) == hipSuccess;
  };
  int rc = RAG_OK;
  for (int b = 0; b < B && rc == RAG_OK; ++b) {
    bool ok = true;
    for (int word = 0; word < 2 && ok; ++word) {   // id ascending: low word, then high word
      ragmi::merge_any_ids_kernel<PACKED><<<g, dim3(256), 0, st>>>(
          in_s, in_i, n_lists, B, k, b, word ? pb : nullptr, word, ka, pa);
      ok = hipGetLastError() == hipSuccess && sort();
    }
    if (ok) {
      ragmi::merge_any_scores_kernel<PACKED><<<g, dim3(256), 0, st>>>(in_s, in_i, n_lists, B, k,
                                                                      b, pb, ka, pa);
      ok = hipGetLastError() == hipSuccess && sort();
    }
    if (ok) {
      ragmi::merge_any_emit_kernel<PACKED><<<ge, dim3(256), 0, st>>>(in_s, in_i, B, k, b, kb, pb,
                                                                     out_s, out_i);
      ok = hipGetLastError() == hipSuccess;
    }
    if (!ok) rc = ragmi::fail(RAG_EHIP, "merge: sort / launch failed");
  }
  (void)hipFreeAsync(buf, st);
  return rc;
}

template <int D>
int launch_large_k_pass(rag_index* h, Workspace& w, const float* q, int Bq, int k,
                        const uint32_t* filt, int64_t id_offset, float* out_s, int64_t* out_i,
                        int32_t* out_packed, hipStream_t st) {
  using namespace ragmi;
  int rc = ensure_lk(w);
  if (rc) return rc;
  qprep_kernel<D><<<dim3(kQ), dim3(64), 0, st>>>(q, Bq, filt, w.qn, w.qfrag, w.filt, w.eps,
                                                  store_eps(h));
  const int n_tiles = (int)((h->count + 15) / 16);
  // bound sample: >= 4k tiles (so k distinct-row maxima exist with margin), >= 1/32 of the
  // shard, at most kLkSampleMax
  const int n_sample = n_tiles == 0 ? 0 : std::min({n_tiles, std::max(4 * k, n_tiles / 32),
                                                    kLkSampleMax});
  if (n_sample > 0) {
    if (filt)
      sample_kernel<D, true><<<dim3((n_sample + 7) / 8, 1), dim3(256), 0, st>>>(
          h->corpus, h->tags, w.filt, w.qfrag, (int)h->count, n_tiles, n_sample, w.lk_smax);
    else
      sample_kernel<D, false><<<dim3((n_sample + 7) / 8, 1), dim3(256), 0, st>>>(
          h->corpus, h->tags, w.filt, w.qfrag, (int)h->count, n_tiles, n_sample, w.lk_smax);
  }
  lk_bound_kernel<<<dim3(Bq), dim3(256), 0, st>>>(w.lk_smax, n_sample, k, w.eps, w.lk_thr,
                                                  w.lk_cnt, w.lk_again, w.lk_need);
  // collection grid: two workgroups per CU (10M rows, k = 33: 1.54-1.55 ms per pass vs
  // 1.57-1.64 at four, 2.37 at one; k = 100 1.64 either way; profiles/r05q_large_k_grid.jsonl)
  const int cgrid = (int)std::max<int64_t>(1, std::min<int64_t>(2 * h->n_cu, (n_tiles + 3) / 4));
  for (int r = 0; r < kLkRounds; ++r) {
    if (filt)
      lk_collect_kernel<D, true><<<dim3(cgrid), dim3(256), 0, st>>>(
          h->corpus, h->tags, w.filt, w.qfrag, (int)h->count, n_tiles, Bq, w.lk_thr, w.lk_cnt,
          w.lk_cand, w.lk_again, w.lk_need, r);
    else
      lk_collect_kernel<D, false><<<dim3(cgrid), dim3(256), 0, st>>>(
          h->corpus, h->tags, w.filt, w.qfrag, (int)h->count, n_tiles, Bq, w.lk_thr, w.lk_cnt,
          w.lk_cand, w.lk_again, w.lk_need, r);
    lk_rescore_kernel<D><<<dim3(kLkCap / 256, Bq), dim3(256), 0, st>>>(
        h->corpus, w.qn, w.lk_cnt, w.lk_cand, w.lk_again, w.lk_need, r, w.lk_es, h->rows32);
    lk_final_kernel<D><<<dim3(Bq), dim3(256), 0, st>>>(
        h->corpus, w.qn, k, w.lk_cnt, w.lk_cand, w.lk_es, w.eps, w.lk_thr, w.lk_again, w.lk_need, r,
        w.fb_tier, w.fb_cnt, id_offset, out_s, out_i, out_packed, h->rows32);
  }
  RAG_HIP(hipGetLastError());
  return RAG_OK;
}

template <int D>
void launch_import(rag_index* h, const half8* in, int64_t row0, int64_t n, hipStream_t st) {
  const int64_t total = n * (D / 8);
  ragmi::import_kernel<D><<<dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st>>>(
      in, row0, n, h->corpus);
}

template <int D>
void launch_import32(rag_index* h, const float* in, int64_t row0, int64_t n, hipStream_t st) {
  const int64_t total = n * (D / 8);
  ragmi::import32_kernel<D><<<dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st>>>(
      in, row0, n, h->corpus, h->rows32);
}

template <int D>
void launch_export(rag_index* h, int64_t row0, int64_t n, half8* out, hipStream_t st) {
  const int64_t total = n * (D / 8);
  const int blocks = (int)((total + 255) / 256);
  ragmi::export_kernel<D><<<dim3(blocks), dim3(256), 0, st>>>(h->corpus, row0, n, out);
}

#define RAG_DISPATCH_DIM(dim, FN, ...)                                   \
  do {                                                                   \
    if ((dim) == 384)                                                    \
      FN<384>(__VA_ARGS__);                                              \
    else if ((dim) == 1024)                                              \
      FN<1024>(__VA_ARGS__);                                             \
    else                                                                 \
      return ragmi::fail(RAG_EINVAL, "unsupported dim (built: 384, 1024)"); \
  } while (0)

int upsert_locked(rag_index* h, const float* vecs, const int64_t* rows, const uint32_t* tags,
                  int64_t n, int64_t new_count, hipStream_t st) {
  if (n < 0 || (n > 0 && (!vecs || !rows))) return ragmi::fail(RAG_EINVAL, "bad upsert args");
  if (new_count < 0 || new_count > h->cap_rows)
    return ragmi::fail(RAG_ERANGE, "new_count exceeds capacity (call rag_index_reserve)");
  if (n > 0x7fffffff) return ragmi::fail(RAG_ERANGE, "n too large for one upsert");
  RAG_HIP(hipSetDevice(h->device));
  if (n > 0) {
    RAG_DISPATCH_DIM(h->dim, launch_upsert, h, vecs, rows, tags, n, st);
    RAG_HIP(hipGetLastError());
  }
  h->count = new_count;
  return RAG_OK;
}

// full: the full exact path for every query (rag_index_search_full); it is also taken for
// k > RAG_MAX_K_LARGE (unpacked output only: the exchange merge holds at most that many)
int search_locked(rag_index* h, const float* q, int B, int k, const uint32_t* filt,
                  int64_t id_offset, float* out_s, int64_t* out_i, int32_t* out_packed,
                  hipStream_t st, bool full = false) {
  if (B < 0 || (B > 0 && (!q || (!out_packed && (!out_s || !out_i)))))
    return ragmi::fail(RAG_EINVAL, "bad search args");
  if (k < 1) return ragmi::fail(RAG_ERANGE, "k must be >= 1");
  if (out_packed && k > RAG_MAX_K_LARGE)
    return ragmi::fail(RAG_ERANGE, "packed (exchange) search: k must be <= RAG_MAX_K_LARGE=4096");
  full = full || k > RAG_MAX_K_LARGE;
  RAG_HIP(hipSetDevice(h->device));
  const bool large = k > RAG_MAX_K || full;
  const int per_pass = large ? ragmi::kQ : ragmi::kQ * h->groups;
  for (int b0 = 0; b0 < B; b0 += per_pass) {
    const int Bq = std::min(per_pass, B - b0);
    Workspace* wp = nullptr;
    for (auto& s : h->ws)
      if (s.used && s.owner == st) { wp = &s; break; }
    if (!wp)
      for (auto& s : h->ws)
        if (!s.used) { wp = &s; break; }
    if (!wp) {
      // every slot is bound to another stream whose last pass may still be running
      RAG_HIP(hipDeviceSynchronize());
      wp = &h->ws[0];
      for (auto& s : h->ws)
        if (s.tick < wp->tick) wp = &s;
    }
    Workspace& w = *wp;
    const uint64_t gen = g_stream_gen.load(std::memory_order_acquire);
    if (!w.used || w.owner != st || w.cus == 0 || w.cus_gen != gen) {
      w.cus = stream_cus(h, st);
      w.cus_gen = gen;
    }
    w.used = true;
    w.owner = st;
    w.tick = ++h->ws_tick;
    int rc;
    h->last_ws = &w;
    h->last_bq = Bq;
    if (large) {
      float* os = out_packed ? nullptr : out_s + (int64_t)b0 * k;
      int64_t* oi = out_packed ? nullptr : out_i + (int64_t)b0 * k;
      int32_t* op = out_packed ? out_packed + (int64_t)b0 * k * 2 : nullptr;
      const uint32_t* fq = filt ? filt + 2 * b0 : nullptr;
      if (full) {
        rc = h->dim == 384
                 ? launch_full_pass<384>(h, w, q + (int64_t)b0 * h->dim, Bq, k, fq, id_offset, os,
                                         oi, op, st)
                 : launch_full_pass<1024>(h, w, q + (int64_t)b0 * h->dim, Bq, k, fq, id_offset,
                                          os, oi, op, st);
        if (rc) return rc;
        continue;
      }
      rc = h->dim == 384
               ? launch_large_k_pass<384>(h, w, q + (int64_t)b0 * h->dim, Bq, k, fq, id_offset, os,
                                          oi, op, st)
               : launch_large_k_pass<1024>(h, w, q + (int64_t)b0 * h->dim, Bq, k, fq, id_offset,
                                           os, oi, op, st);
      if (rc) return rc;
      continue;
    }
    if (h->dim == 384)
      rc = launch_search_pass<384>(
          h, w, q + (int64_t)b0 * h->dim, Bq, k, filt ? filt + 2 * b0 : nullptr, id_offset,
          out_packed ? nullptr : out_s + (int64_t)b0 * k,
          out_packed ? nullptr : out_i + (int64_t)b0 * k,
          out_packed ? out_packed + (int64_t)b0 * k * 2 : nullptr, st);
    else
      rc = launch_search_pass<1024>(
          h, w, q + (int64_t)b0 * h->dim, Bq, k, filt ? filt + 2 * b0 : nullptr, id_offset,
          out_packed ? nullptr : out_s + (int64_t)b0 * k,
          out_packed ? nullptr : out_i + (int64_t)b0 * k,
          out_packed ? out_packed + (int64_t)b0 * k * 2 : nullptr, st);
    if (rc) return rc;
  }
  return RAG_OK;
}


// Diagnostic A/B of scan variants (see scan_kernel's knobs). Returns avg device ms/launch.
template <int D, int V>
void launch_variant(rag_index* h, Workspace& w, int grid, hipStream_t st) {
  using namespace ragmi;
  const int n_tiles = (int)((h->count + 15) / 16);
  // 0 prod (seeded) | 1 unseeded | 2 contiguous | 3 mfma-only | 4 loads-only | 5 no-nt
  // 6 no-sb | 9 / 10 / 11 dynamic tile queue, chunks of 2 / 1 / 4 tiles | 12 dynamic (2),
  // loads only | 13 / 14 static production / loads only (9-14: each launch timed on its own,
  // the queue heads zeroed between launches outside the timed window) | 15 production without
  // the end-of-scan sort of pending-only queries (results invalid) | 16 production with the
  // round-1 end-of-scan sort (two pending-only queries per 32-lane pass)
  constexpr int MODE = V == 3 ? 1 : V == 4 || V == 12 || V == 14 ? 2 : V == 15 ? 3 : V == 16 ? 4 : 0;
  constexpr bool STRIDED = V != 2;
  constexpr bool NT = V != 5;
  constexpr bool SB = V != 6;
  constexpr int DYN = V == 9 || V == 12 ? 2 : V == 10 ? 1 : V == 11 ? 4 : 0;
  launch_fixed<kScanBlock>(scan_kernel<D, false, MODE, STRIDED, NT, SB, DYN>, dim3(grid), 0, st,
                           h->corpus, h->tags, w.filt, w.qfrag, (int)h->count, n_tiles,
                           V == 1 ? nullptr : w.seed, w.part_s, w.part_i, w.heads_s, w.heads_i,
                           w.heads_n, w.tileq);
}

template <int D>
int bench_scan(rag_index* h, const float* q, int B, int variant, int reps, double* avg_ms) {
  using namespace ragmi;
  Workspace& w = h->ws[0];
  RAG_HIP(hipDeviceSynchronize());
  qprep_kernel<D><<<dim3(kQ), dim3(64), 0, nullptr>>>(q, std::min(B, kQ), nullptr, w.qn,
                                                      w.qfrag, w.filt, w.eps, store_eps(h));
  launch_seed<D, false>(h, w, 1, nullptr);
  // variant 7: the production kernel with every seed threshold at +inf, i.e. the top-k's
  // per-tile compares and branches with no candidate ever taken (its fixed cost)
  if (variant == 7)
    RAG_HIP(hipMemsetD32(reinterpret_cast<hipDeviceptr_t>(w.seed), 0x7f800000, kQ));
  const int64_t n_tiles = (h->count + 15) / 16;
  // the production grid (launch_search_pass: 3/4 of the CUs); RAGMI_SCAN_WGS overrides
  static ragmi::Knob k_wgs("RAGMI_SCAN_WGS");
  const int cap = k_wgs.get(0) > 0 ? std::max(8, k_wgs.get(0)) : h->scan_wgs;
  int grid = (int)std::min<int64_t>(std::min(h->max_wgs, cap), std::max<int64_t>(1, (n_tiles + 3) / 4));
  grid = std::min(grid, kMaxLists / kWavesPerWG);
  // variant 8: the v_dot2 VALU ablation over a row-group-major copy of the corpus
  half8* rows64 = nullptr;
  half8* qc = nullptr;
  const int n_groups = (int)((h->count + 63) / 64);
#ifdef RAGMI_DIAG_BUILD
  if (variant == 8) {
    RAG_HIP(hipMalloc(reinterpret_cast<void**>(&rows64), (size_t)n_groups * 64 * D * 2));
    RAG_HIP(hipMalloc(reinterpret_cast<void**>(&qc), (size_t)kQ * D * 2));
    RAG_HIP(hipMemset(rows64, 0, (size_t)n_groups * 64 * D * 2));
    const int64_t total = h->count * (D / 8);
    rows64_kernel<D><<<dim3((unsigned)((total + 255) / 256)), dim3(256), 0, nullptr>>>(
        h->corpus, h->count, rows64);
    qchunk_kernel<D><<<dim3(kQ), dim3(64), 0, nullptr>>>(w.qn, qc);
  }
#endif
  const int vgrid = std::min(h->max_wgs, std::max(1, (n_groups + 3) / 4));
  (void)vgrid;
  hipEvent_t a, b;
  RAG_HIP(hipEventCreate(&a));
  RAG_HIP(hipEventCreate(&b));
  auto one = [&]() {
#ifndef RAGMI_DIAG_BUILD
    // production library: the production scan only (variants 0 and 7); the MODE / DYN /
    // VALU probes are instantiated in the diagnostic build alone
    launch_variant<D, 0>(h, w, grid, nullptr);
#else
    if (variant == 8) {
      scan_valu_kernel<D><<<dim3(vgrid), dim3(256), 0, nullptr>>>(
          rows64, qc, (int)h->count, n_groups, w.seed, w.part_s, w.part_i, w.heads_s,
          w.heads_i, w.heads_n);
      return;
    }
    switch (variant) {
      case 0: launch_variant<D, 0>(h, w, grid, nullptr); break;
      case 1: launch_variant<D, 1>(h, w, grid, nullptr); break;
      case 2: launch_variant<D, 2>(h, w, grid, nullptr); break;
      case 3: launch_variant<D, 3>(h, w, grid, nullptr); break;
      case 4: launch_variant<D, 4>(h, w, grid, nullptr); break;
      case 5: launch_variant<D, 5>(h, w, grid, nullptr); break;
      case 7: launch_variant<D, 0>(h, w, grid, nullptr); break;
      case 15: launch_variant<D, 15>(h, w, grid, nullptr); break;
      case 16: launch_variant<D, 16>(h, w, grid, nullptr); break;
      default: launch_variant<D, 6>(h, w, grid, nullptr); break;
    }
#endif
  };
  float ms = 0.f;
#ifdef RAGMI_DIAG_BUILD
  if (variant >= 9 && variant <= 14) {
    // one launch per event pair; the tile-queue heads are zeroed before each, outside it
    for (int r = -1; r < reps; ++r) {
      RAG_HIP(hipMemsetAsync(w.tileq, 0, 8 * kTileQStride * 4, nullptr));
      RAG_HIP(hipEventRecord(a, nullptr));
      switch (variant) {
        case 9: launch_variant<D, 9>(h, w, grid, nullptr); break;
        case 10: launch_variant<D, 10>(h, w, grid, nullptr); break;
        case 11: launch_variant<D, 11>(h, w, grid, nullptr); break;
        case 12: launch_variant<D, 12>(h, w, grid, nullptr); break;
        case 13: launch_variant<D, 0>(h, w, grid, nullptr); break;
        default: launch_variant<D, 14>(h, w, grid, nullptr); break;
      }
      RAG_HIP(hipEventRecord(b, nullptr));
      RAG_HIP(hipEventSynchronize(b));
      float m1 = 0.f;
      RAG_HIP(hipEventElapsedTime(&m1, a, b));
      if (r >= 0) ms += m1;   // r = -1: warm-up
    }
  } else
#endif
  {
    one();  // warm
    RAG_HIP(hipEventRecord(a, nullptr));
    for (int r = 0; r < reps; ++r) one();
    RAG_HIP(hipEventRecord(b, nullptr));
    RAG_HIP(hipEventSynchronize(b));
    RAG_HIP(hipEventElapsedTime(&ms, a, b));
  }
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  if (rows64) (void)hipFree(rows64);
  if (qc) (void)hipFree(qc);
  RAG_HIP(hipGetLastError());
  *avg_ms = ms / reps;
  return RAG_OK;
}

// Diagnostic A/B of the wide (D = 1024, 33..128 queries, unfiltered) scan's variants
// (scan_wide_kernel MODE 0..4; 0 is production). Returns avg device ms/launch.
template <int D>
int bench_wide(rag_index* h, const float* q, int B, int mode, int reps, double* avg_ms) {
  using namespace ragmi;
  Workspace& w = h->ws[0];
  const int groups = (std::min(B, kQ * kMaxGroups) + kQ - 1) / kQ;
  if (groups < 2) return ragmi::fail(RAG_EINVAL, "wide scan variants need 33..128 queries");
  RAG_HIP(hipDeviceSynchronize());
  qprep_kernel<D><<<dim3(groups * kQ), dim3(64), 0, nullptr>>>(
      q, std::min(B, groups * kQ), nullptr, w.qn, w.qfrag, w.filt, w.eps, store_eps(h));
  launch_seed<D, false>(h, w, groups, nullptr);
  const int64_t n_tiles = (h->count + 15) / 16;
  const int grid = (int)std::min<int64_t>(h->max_wgs / 2, std::max<int64_t>(1, n_tiles));
  auto one = [&]() {
#define RAG_WIDE(MODE)                                                                     \
  launch_fixed<kWideBlock>(scan_wide_kernel<D, MODE, true>, dim3(grid), 0, nullptr,          \
                           h->corpus, w.qfrag, (int)h->count, (int)n_tiles, w.seed, w.part_s, \
                           w.part_i, w.heads_s, w.heads_i, w.heads_n, groups)
#ifdef RAGMI_DIAG_BUILD
    switch (mode) {
      case 1: RAG_WIDE(1); break;
      case 2: RAG_WIDE(2); break;
      case 3: RAG_WIDE(3); break;
      case 4: RAG_WIDE(4); break;
      default: RAG_WIDE(0); break;
    }
#else
    RAG_WIDE(0);
#endif
#undef RAG_WIDE
  };
  hipEvent_t a, b;
  RAG_HIP(hipEventCreate(&a));
  RAG_HIP(hipEventCreate(&b));
  one();  // warm
  RAG_HIP(hipEventRecord(a, nullptr));
  for (int r = 0; r < reps; ++r) one();
  RAG_HIP(hipEventRecord(b, nullptr));
  RAG_HIP(hipEventSynchronize(b));
  float ms = 0.f;
  RAG_HIP(hipEventElapsedTime(&ms, a, b));
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  RAG_HIP(hipGetLastError());
  *avg_ms = ms / reps;
  return RAG_OK;
}

}  // namespace

extern "C" {

const char* rag_last_error(void) { return ragmi::last_error().c_str(); }
const char* rag_version(void) { return "ragmi 0.1.0 (gfx950)"; }

int rag_index_create(int dim, int64_t capacity_rows, int device, rag_index_t** out) {
  return rag_index_create_ex(dim, capacity_rows, device, RAG_STORE_FP16, out);
}

int rag_index_create_ex(int dim, int64_t capacity_rows, int device, int storage,
                        rag_index_t** out) {
  ragmi::clear_error();
  if (!out) return ragmi::fail(RAG_EINVAL, "out is NULL");
  *out = nullptr;
  if (dim != 384 && dim != 1024) return ragmi::fail(RAG_EINVAL, "dim must be 384 or 1024");
  const bool diag = (storage & RAG_CREATE_DIAGNOSTIC) != 0;
  storage &= ~RAG_CREATE_DIAGNOSTIC;
  if (storage != RAG_STORE_FP16 && storage != RAG_STORE_FP32)
    return ragmi::fail(RAG_EINVAL, "storage must be RAG_STORE_FP16 or RAG_STORE_FP32");
  if (capacity_rows < 0 || capacity_rows > (int64_t(1) << 31) - 16)
    return ragmi::fail(RAG_ERANGE, "capacity_rows out of range [0, 2^31-16]");
  RAG_HIP(hipSetDevice(device));
  auto* h = new rag_index();
  h->dim = dim;
  h->device = device;
  h->cap_rows = round16(std::max<int64_t>(capacity_rows, 16));
  h->storage = storage;
  int rc = alloc_corpus(h, h->cap_rows, &h->corpus, &h->tags);
  if (rc) {
    delete h;
    return rc;
  }
  if (storage == RAG_STORE_FP32) {
    const size_t b32 = (size_t)h->cap_rows * dim * 4;
    if (hipMalloc(reinterpret_cast<void**>(&h->rows32), b32) != hipSuccess ||
        hipMemset(h->rows32, 0, b32) != hipSuccess) {
      rag_index_destroy(h);
      return ragmi::fail(RAG_ENOMEM, "hipMalloc(rows32) failed");
    }
  }
  int n_cu = 0;
  if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, device) !=
          hipSuccess ||
      n_cu <= 0)
    n_cu = 256;
  h->n_cu = n_cu;
  h->max_wgs = n_cu * 2;  // 2 x 256-thread workgroups per CU (__launch_bounds__(256, 2))
  h->scan_wgs = std::max(8, (n_cu * 3 / 4) & ~7);
  // wide rows (LDS-query scan) take up to 4 query groups (128 queries) per pass
  h->groups = dim > 384 ? kMaxGroups : 1;
  const size_t G = (size_t)h->groups, Q = ragmi::kQ;
  const int max_lists = std::min(h->max_wgs * ragmi::kWavesPerWG, ragmi::kMaxLists);
  for (auto& w : h->ws) {
    bool ok = hipMalloc(reinterpret_cast<void**>(&w.qn), G * Q * dim * 4) == hipSuccess &&
              hipMalloc(reinterpret_cast<void**>(&w.qfrag), G * 2 * (dim / 32) * 64 * 16) ==
                  hipSuccess &&
              hipMalloc(reinterpret_cast<void**>(&w.filt), G * Q * 2 * 4) == hipSuccess &&
              hipMalloc(reinterpret_cast<void**>(&w.smax),
                        G * (dim > 384 ? ragmi::kMaxSampleWide : ragmi::kMaxSample) * Q * 4) ==
                  hipSuccess &&
              hipMalloc(reinterpret_cast<void**>(&w.heads_s),
                        G * ragmi::kMaxLists * Q * 4) == hipSuccess &&
              hipMalloc(reinterpret_cast<void**>(&w.heads_i),
                        G * ragmi::kMaxLists * Q * 4) == hipSuccess &&
              hipMalloc(reinterpret_cast<void**>(&w.heads_n),
                        G * ragmi::kMaxLists * Q * 4) == hipSuccess &&
              hipMalloc(reinterpret_cast<void**>(&w.seed), G * Q * 4) == hipSuccess &&
              hipMalloc(reinterpret_cast<void**>(&w.part_s),
                        G * max_lists * Q * ragmi::kKS * 4) == hipSuccess &&
              hipMalloc(reinterpret_cast<void**>(&w.part_i),
                        G * max_lists * Q * ragmi::kKS * 4) == hipSuccess &&
              hipMalloc(reinterpret_cast<void**>(&w.progress),
                        G * ragmi::kMaxLists * 4) == hipSuccess &&
              hipMalloc(reinterpret_cast<void**>(&w.eps), G * Q * 4) == hipSuccess &&
              hipMalloc(reinterpret_cast<void**>(&w.fb_tier), G * Q * 4) == hipSuccess &&
              hipMalloc(reinterpret_cast<void**>(&w.fb_cnt), 32) == hipSuccess &&
              hipMalloc(reinterpret_cast<void**>(&w.tileq), 8 * ragmi::kTileQStride * 4) ==
                  hipSuccess &&
              hipMalloc(reinterpret_cast<void**>(&w.t2), G * Q * 2 * 4) == hipSuccess &&
              hipMalloc(reinterpret_cast<void**>(&w.t2_s),
                        G * Q * ragmi::kRescanMaxWG * 32 * 4) == hipSuccess &&
              hipMalloc(reinterpret_cast<void**>(&w.t2_i),
                        G * Q * ragmi::kRescanMaxWG * 32 * 4) == hipSuccess &&
              hipMalloc(reinterpret_cast<void**>(&w.t2_tk), 64) == hipSuccess &&
              hipMemset(w.t2_tk, 0, 64) == hipSuccess &&
              hipMemset(w.tileq, 0, 8 * ragmi::kTileQStride * 4) == hipSuccess &&
              hipMemset(w.fb_cnt, 0, 32) == hipSuccess &&
              hipMemset(w.fb_tier, 0, G * Q * 4) == hipSuccess;
    if (!ok) {
      rag_index_destroy(h);
      return ragmi::fail(RAG_ENOMEM, "workspace allocation failed");
    }
  }
  if (diag) {
    h->diagnostic = true;
    ragmi::diagnostic_acquire();
  }
  *out = h;
  return RAG_OK;
}

int rag_diagnostic_build(void) {
#ifdef RAGMI_DIAG_BUILD
  return 1;
#else
  return 0;
#endif
}

int rag_knob_probe(const char* name, int dflt) {
  if (!name) return dflt;
  ragmi::Knob k(name);
  return k.get(dflt);
}

int rag_index_destroy(rag_index_t* h) {
  ragmi::clear_error();
  if (!h) return RAG_OK;
  if (h->diagnostic) ragmi::diagnostic_release();
  (void)hipSetDevice(h->device);
  (void)hipDeviceSynchronize();
  for (auto& w : h->ws) {
    if (w.qn) (void)hipFree(w.qn);
    if (w.qfrag) (void)hipFree(w.qfrag);
    if (w.filt) (void)hipFree(w.filt);
    if (w.smax) (void)hipFree(w.smax);
    if (w.heads_s) (void)hipFree(w.heads_s);
    if (w.heads_i) (void)hipFree(w.heads_i);
    if (w.heads_n) (void)hipFree(w.heads_n);
    if (w.seed) (void)hipFree(w.seed);
    if (w.part_s) (void)hipFree(w.part_s);
    if (w.part_i) (void)hipFree(w.part_i);
    if (w.progress) (void)hipFree(w.progress);
    if (w.eps) (void)hipFree(w.eps);
    if (w.fb_tier) (void)hipFree(w.fb_tier);
    if (w.fb_cnt) (void)hipFree(w.fb_cnt);
    if (w.tileq) (void)hipFree(w.tileq);
    for (void* p : {(void*)w.t2, (void*)w.t2_s, (void*)w.t2_i, (void*)w.t2_tk})
      if (p) (void)hipFree(p);
    for (void* p : {(void*)w.lk_smax, (void*)w.lk_thr, (void*)w.lk_cnt, (void*)w.lk_again,
                    (void*)w.lk_need, (void*)w.lk_cand, (void*)w.lk_es})
      if (p) (void)hipFree(p);
    if (w.ev_in) (void)hipEventDestroy(w.ev_in);
    if (w.ev_out) (void)hipEventDestroy(w.ev_out);
  }
  for (auto& p : h->prof_pairs) {
    (void)hipEventDestroy(p.a);
    (void)hipEventDestroy(p.b);
  }
  if (h->scan_done) (void)hipEventDestroy(h->scan_done);
  if (h->scan_stream) (void)hipStreamDestroy(h->scan_stream);
  if (h->corpus) (void)hipFree(h->corpus);
  if (h->tags) (void)hipFree(h->tags);
  if (h->rows32) (void)hipFree(h->rows32);
  if (h->stage) (void)hipFree(h->stage);
  delete h;
  return RAG_OK;
}

int rag_index_reserve(rag_index_t* h, int64_t capacity_rows) {
  ragmi::clear_error();
  if (!h) return ragmi::fail(RAG_EINVAL, "index is NULL");
  if (capacity_rows > (int64_t(1) << 31) - 16)
    return ragmi::fail(RAG_ERANGE, "capacity_rows out of range");
  std::lock_guard<std::mutex> lk(h->mu);
  const int64_t cap = round16(capacity_rows);
  if (cap <= h->cap_rows) return RAG_OK;
  RAG_HIP(hipSetDevice(h->device));
  half8* nc = nullptr;
  uint32_t* nt = nullptr;
  float* n32 = nullptr;
  // the new buffers are freed on every error return below; released once the handle owns them
  struct Guard {
    half8** c; uint32_t** t; float** f;
    ~Guard() {
      if (*c) (void)hipFree(*c);
      if (*t) (void)hipFree(*t);
      if (*f) (void)hipFree(*f);
    }
  } guard{&nc, &nt, &n32};
  int rc = alloc_corpus(h, cap, &nc, &nt);
  if (rc) return rc;
  if (h->rows32) {
    const size_t b32 = (size_t)cap * h->dim * 4;
    if (hipMalloc(reinterpret_cast<void**>(&n32), b32) != hipSuccess) {
      n32 = nullptr;
      return ragmi::fail(RAG_ENOMEM, "hipMalloc(rows32) failed");
    }
    RAG_HIP(hipMemset(n32, 0, b32));
  }
  RAG_HIP(hipDeviceSynchronize());
  RAG_HIP(hipMemcpy(nc, h->corpus, (size_t)h->cap_rows * h->dim * 2, hipMemcpyDeviceToDevice));
  RAG_HIP(hipMemcpy(nt, h->tags, (size_t)h->cap_rows * 4, hipMemcpyDeviceToDevice));
  if (n32)
    RAG_HIP(hipMemcpy(n32, h->rows32, (size_t)h->cap_rows * h->dim * 4, hipMemcpyDeviceToDevice));
  (void)hipFree(h->corpus);
  (void)hipFree(h->tags);
  if (h->rows32) (void)hipFree(h->rows32);
  h->corpus = nc;
  h->tags = nt;
  h->rows32 = n32;
  h->cap_rows = cap;
  nc = nullptr;                                  // owned by the handle now
  nt = nullptr;
  n32 = nullptr;
  return RAG_OK;
}

int64_t rag_index_capacity(const rag_index_t* h) { return h ? h->cap_rows : -1; }
int64_t rag_index_count(const rag_index_t* h) { return h ? h->count : -1; }
int rag_index_dim(const rag_index_t* h) { return h ? h->dim : -1; }

int rag_index_upsert(rag_index_t* h, const float* vecs, const int64_t* rows,
                     const uint32_t* tags, int64_t n, int64_t new_count, void* stream) {
  ragmi::clear_error();
  if (!h) return ragmi::fail(RAG_EINVAL, "index is NULL");
  std::lock_guard<std::mutex> lk(h->mu);
  return upsert_locked(h, vecs, rows, tags, n, new_count, static_cast<hipStream_t>(stream));
}

int rag_index_upsert_host(rag_index_t* h, const float* vecs, const int64_t* rows,
                          const uint32_t* tags, int64_t n, int64_t new_count) {
  ragmi::clear_error();
  if (!h) return ragmi::fail(RAG_EINVAL, "index is NULL");
  if (n < 0 || (n > 0 && (!vecs || !rows))) return ragmi::fail(RAG_EINVAL, "bad upsert args");
  for (int64_t i = 0; i < n; ++i)
    if (rows[i] < 0 || rows[i] >= h->cap_rows)
      return ragmi::fail(RAG_ERANGE, "row slot beyond capacity (call rag_index_reserve)");
  std::lock_guard<std::mutex> lk(h->mu);
  RAG_HIP(hipSetDevice(h->device));
  const size_t vb = (size_t)n * h->dim * 4, rb = (size_t)n * 8, tb = (size_t)n * 4;
  int rc = ensure_stage(h, vb + rb + tb + 64);
  if (rc) return rc;
  char* base = static_cast<char*>(h->stage);
  RAG_HIP(hipDeviceSynchronize());
  if (n > 0) {
    RAG_HIP(hipMemcpy(base, vecs, vb, hipMemcpyHostToDevice));
    RAG_HIP(hipMemcpy(base + vb, rows, rb, hipMemcpyHostToDevice));
    if (tags) RAG_HIP(hipMemcpy(base + vb + rb, tags, tb, hipMemcpyHostToDevice));
  }
  rc = upsert_locked(h, reinterpret_cast<float*>(base), reinterpret_cast<int64_t*>(base + vb),
                     tags ? reinterpret_cast<uint32_t*>(base + vb + rb) : nullptr, n, new_count,
                     nullptr);
  if (rc) return rc;
  RAG_HIP(hipDeviceSynchronize());
  return RAG_OK;
}

int rag_index_search(rag_index_t* h, const float* q, int B, int k, const uint32_t* filters,
                     int64_t id_offset, float* out_s, int64_t* out_i, void* stream) {
  ragmi::clear_error();
  if (!h) return ragmi::fail(RAG_EINVAL, "index is NULL");
  std::lock_guard<std::mutex> lk(h->mu);
  return search_locked(h, q, B, k, filters, id_offset, out_s, out_i, nullptr,
                       static_cast<hipStream_t>(stream));
}

int rag_index_search_full(rag_index_t* h, const float* q, int B, int k, const uint32_t* filters,
                          int64_t id_offset, float* out_s, int64_t* out_i, void* stream) {
  ragmi::clear_error();
  if (!h) return ragmi::fail(RAG_EINVAL, "index is NULL");
  std::lock_guard<std::mutex> lk(h->mu);
  return search_locked(h, q, B, k, filters, id_offset, out_s, out_i, nullptr,
                       static_cast<hipStream_t>(stream), true);
}

int rag_index_search_packed(rag_index_t* h, const float* q, int B, int k,
                            const uint32_t* filters, int64_t id_offset, int32_t* out_packed,
                            void* stream) {
  ragmi::clear_error();
  if (!h || (B > 0 && !out_packed)) return ragmi::fail(RAG_EINVAL, "bad packed search args");
  if (id_offset < 0 || id_offset + h->count > INT32_MAX)
    return ragmi::fail(RAG_ERANGE, "packed ids are int32: global rows must stay below 2^31");
  std::lock_guard<std::mutex> lk(h->mu);
  return search_locked(h, q, B, k, filters, id_offset, nullptr, nullptr, out_packed,
                       static_cast<hipStream_t>(stream));
}

int rag_index_search_host(rag_index_t* h, const float* q, int B, int k,
                          const uint32_t* filters, int64_t id_offset, float* out_s,
                          int64_t* out_i) {
  ragmi::clear_error();
  if (!h) return ragmi::fail(RAG_EINVAL, "index is NULL");
  if (B < 0 || (B > 0 && (!q || !out_s || !out_i))) return ragmi::fail(RAG_EINVAL, "bad search args");
  if (k < 1) return ragmi::fail(RAG_ERANGE, "k must be >= 1");
  if (B == 0) return RAG_OK;
  std::lock_guard<std::mutex> lk(h->mu);
  RAG_HIP(hipSetDevice(h->device));
  // staging offsets rounded to 16 B (the int64 ids must be 8-B aligned for any B * k)
  auto up16 = [](size_t x) { return (x + 15) & ~size_t(15); };
  const size_t qb = up16((size_t)B * h->dim * 4), sb = up16((size_t)B * k * 4);
  const size_t ib = up16((size_t)B * k * 8), fb = (size_t)B * 8;
  int rc = ensure_stage(h, qb + sb + ib + fb + 64);
  if (rc) return rc;
  char* base = static_cast<char*>(h->stage);
  RAG_HIP(hipDeviceSynchronize());
  RAG_HIP(hipMemcpy(base, q, (size_t)B * h->dim * 4, hipMemcpyHostToDevice));
  if (filters) RAG_HIP(hipMemcpy(base + qb + sb + ib, filters, fb, hipMemcpyHostToDevice));
  rc = search_locked(h, reinterpret_cast<float*>(base), B, k,
                     filters ? reinterpret_cast<uint32_t*>(base + qb + sb + ib) : nullptr,
                     id_offset, reinterpret_cast<float*>(base + qb),
                     reinterpret_cast<int64_t*>(base + qb + sb), nullptr, nullptr);
  if (rc) return rc;
  RAG_HIP(hipDeviceSynchronize());
  RAG_HIP(hipMemcpy(out_s, base + qb, (size_t)B * k * 4, hipMemcpyDeviceToHost));
  RAG_HIP(hipMemcpy(out_i, base + qb + sb, (size_t)B * k * 8, hipMemcpyDeviceToHost));
  return RAG_OK;
}

int rag_index_export_rows(rag_index_t* h, int64_t row0, int64_t n, uint16_t* out) {
  ragmi::clear_error();
  if (!h || !out || row0 < 0 || n < 0 || row0 + n > h->cap_rows)
    return ragmi::fail(RAG_EINVAL, "bad export range");
  if (n == 0) return RAG_OK;
  std::lock_guard<std::mutex> lk(h->mu);
  RAG_HIP(hipSetDevice(h->device));
  const size_t bytes = (size_t)n * h->dim * 2;
  int rc = ensure_stage(h, bytes);
  if (rc) return rc;
  RAG_HIP(hipDeviceSynchronize());
  RAG_DISPATCH_DIM(h->dim, launch_export, h, row0, n, static_cast<half8*>(h->stage), nullptr);
  RAG_HIP(hipGetLastError());
  RAG_HIP(hipDeviceSynchronize());
  RAG_HIP(hipMemcpy(out, h->stage, bytes, hipMemcpyDeviceToHost));
  return RAG_OK;
}

int rag_index_import_rows(rag_index_t* h, int64_t row0, int64_t n, const uint16_t* rows,
                          const uint32_t* tags, int64_t new_count) {
  ragmi::clear_error();
  if (!h || (n > 0 && !rows) || row0 < 0 || n < 0 || row0 + n > h->cap_rows)
    return ragmi::fail(RAG_EINVAL, "bad import range (reserve capacity first)");
  if (h->rows32)
    return ragmi::fail(RAG_EINVAL, "fp32-storage index: load its fp32 rows (rag_index_import_rows32)");
  if (new_count < 0 || new_count > h->cap_rows)
    return ragmi::fail(RAG_ERANGE, "new_count exceeds capacity");
  std::lock_guard<std::mutex> lk(h->mu);
  RAG_HIP(hipSetDevice(h->device));
  if (n > 0) {
    const size_t bytes = (size_t)n * h->dim * 2;
    int rc = ensure_stage(h, bytes);
    if (rc) return rc;
    RAG_HIP(hipDeviceSynchronize());
    RAG_HIP(hipMemcpy(h->stage, rows, bytes, hipMemcpyHostToDevice));
    RAG_DISPATCH_DIM(h->dim, launch_import, h, static_cast<const half8*>(h->stage), row0, n,
                     nullptr);
    RAG_HIP(hipGetLastError());
    if (tags)
      RAG_HIP(hipMemcpy(h->tags + row0, tags, (size_t)n * 4, hipMemcpyHostToDevice));
    RAG_HIP(hipDeviceSynchronize());
  }
  h->count = new_count;
  return RAG_OK;
}

int rag_index_storage(const rag_index_t* h) { return h ? h->storage : -1; }

int rag_index_export_rows32(rag_index_t* h, int64_t row0, int64_t n, float* out) {
  ragmi::clear_error();
  if (!h || !out || row0 < 0 || n < 0 || row0 + n > h->cap_rows)
    return ragmi::fail(RAG_EINVAL, "bad export range");
  if (!h->rows32) return ragmi::fail(RAG_EINVAL, "index has fp16 storage (no fp32 rows)");
  if (n == 0) return RAG_OK;
  std::lock_guard<std::mutex> lk(h->mu);
  RAG_HIP(hipSetDevice(h->device));
  RAG_HIP(hipDeviceSynchronize());
  RAG_HIP(hipMemcpy(out, h->rows32 + row0 * h->dim, (size_t)n * h->dim * 4,
                    hipMemcpyDeviceToHost));
  return RAG_OK;
}

int rag_index_import_rows32(rag_index_t* h, int64_t row0, int64_t n, const float* rows,
                            const uint32_t* tags, int64_t new_count) {
  ragmi::clear_error();
  if (!h || (n > 0 && !rows) || row0 < 0 || n < 0 || row0 + n > h->cap_rows)
    return ragmi::fail(RAG_EINVAL, "bad import range (reserve capacity first)");
  if (!h->rows32) return ragmi::fail(RAG_EINVAL, "index has fp16 storage (no fp32 rows)");
  if (new_count < 0 || new_count > h->cap_rows)
    return ragmi::fail(RAG_ERANGE, "new_count exceeds capacity");
  std::lock_guard<std::mutex> lk(h->mu);
  RAG_HIP(hipSetDevice(h->device));
  if (n > 0) {
    const size_t bytes = (size_t)n * h->dim * 4;
    int rc = ensure_stage(h, bytes);
    if (rc) return rc;
    RAG_HIP(hipDeviceSynchronize());
    RAG_HIP(hipMemcpy(h->stage, rows, bytes, hipMemcpyHostToDevice));
    RAG_DISPATCH_DIM(h->dim, launch_import32, h, static_cast<const float*>(h->stage), row0, n,
                     nullptr);
    RAG_HIP(hipGetLastError());
    if (tags)
      RAG_HIP(hipMemcpy(h->tags + row0, tags, (size_t)n * 4, hipMemcpyHostToDevice));
    RAG_HIP(hipDeviceSynchronize());
  }
  h->count = new_count;
  return RAG_OK;
}

int rag_index_export_tags(rag_index_t* h, int64_t row0, int64_t n, uint32_t* out) {
  ragmi::clear_error();
  if (!h || !out || row0 < 0 || n < 0 || row0 + n > h->cap_rows)
    return ragmi::fail(RAG_EINVAL, "bad export range");
  if (n == 0) return RAG_OK;
  std::lock_guard<std::mutex> lk(h->mu);
  RAG_HIP(hipSetDevice(h->device));
  RAG_HIP(hipDeviceSynchronize());
  RAG_HIP(hipMemcpy(out, h->tags + row0, (size_t)n * 4, hipMemcpyDeviceToHost));
  return RAG_OK;
}

int rag_merge_topk(const float* in_s, const int64_t* in_i, int n_lists, int B, int k,
                   float* out_s, int64_t* out_i, void* stream) {
  ragmi::clear_error();
  if (n_lists < 1 || B < 0 || k < 1)
    return ragmi::fail(RAG_EINVAL, "bad merge args");
  if (B == 0) return RAG_OK;
  if (k > RAG_MAX_K_LARGE)
    return merge_any_k<false>(in_s, in_i, n_lists, B, k, out_s, out_i,
                              static_cast<hipStream_t>(stream));
  if (k > RAG_MAX_K)
    ragmi::merge_large_kernel<false><<<dim3(B), dim3(256), 0, static_cast<hipStream_t>(stream)>>>(
        in_s, in_i, n_lists, B, k, out_s, out_i);
  else
    ragmi::merge_exact_kernel<false><<<dim3(B), dim3(64), 0, static_cast<hipStream_t>(stream)>>>(
        in_s, in_i, n_lists, B, k, out_s, out_i);
  RAG_HIP(hipGetLastError());
  return RAG_OK;
}

int rag_merge_topk_packed(const int32_t* in_packed, int n_lists, int B, int k, float* out_s,
                          int64_t* out_i, void* stream) {
  ragmi::clear_error();
  if (n_lists < 1 || B < 0 || k < 1 || (B > 0 && !in_packed))
    return ragmi::fail(RAG_EINVAL, "bad merge args");
  if (B == 0) return RAG_OK;
  if (k > RAG_MAX_K_LARGE)
    return merge_any_k<true>(reinterpret_cast<const float*>(in_packed), nullptr, n_lists, B, k,
                             out_s, out_i, static_cast<hipStream_t>(stream));
  if (k > RAG_MAX_K)
    ragmi::merge_large_kernel<true><<<dim3(B), dim3(256), 0, static_cast<hipStream_t>(stream)>>>(
        reinterpret_cast<const float*>(in_packed), nullptr, n_lists, B, k, out_s, out_i);
  else
    ragmi::merge_exact_kernel<true><<<dim3(B), dim3(64), 0, static_cast<hipStream_t>(stream)>>>(
        reinterpret_cast<const float*>(in_packed), nullptr, n_lists, B, k, out_s, out_i);
  RAG_HIP(hipGetLastError());
  return RAG_OK;
}

int rag_bench_scan(rag_index_t* h, const float* queries_dev, int B, int variant, int reps,
                   double* avg_ms) {
  ragmi::clear_error();
#ifndef RAGMI_DIAG_BUILD
  if (variant != 0 && (variant != 7 || (h && h->dim != 384)))
    return ragmi::fail(RAG_EINVAL, "variant: 0 (production) or 7 (dim 384: seeds at +inf); the "
                                   "scan's timing probes are in the diagnostic build only");
#endif
  if (!h || !queries_dev || B < 1 || reps < 1 || !avg_ms || variant < 0 || variant > 16)
    return ragmi::fail(RAG_EINVAL, "bad bench args");
  std::lock_guard<std::mutex> lk(h->mu);
  RAG_HIP(hipSetDevice(h->device));
  if (h->dim == 1024) {
    if (variant > 4) return ragmi::fail(RAG_EINVAL, "dim 1024: wide scan variants 0..4");
    return bench_wide<1024>(h, queries_dev, B, variant, reps, avg_ms);
  }
  return bench_scan<384>(h, queries_dev, B, variant, reps, avg_ms);
}

int rag_index_exactness_stats(rag_index_t* h, int64_t* tier1, int64_t* tier2,
                               int32_t* last_tiers, int n_last) {
  ragmi::clear_error();
  if (!h || !tier1 || !tier2 || n_last < 0 || (n_last > 0 && !last_tiers))
    return ragmi::fail(RAG_EINVAL, "bad exactness stats args");
  std::lock_guard<std::mutex> lk(h->mu);
  RAG_HIP(hipSetDevice(h->device));
  RAG_HIP(hipDeviceSynchronize());
  unsigned long long t1 = 0, t2 = 0;
  for (auto& w : h->ws) {
    unsigned long long c[2];
    RAG_HIP(hipMemcpy(c, w.fb_cnt, sizeof(c), hipMemcpyDeviceToHost));
    t1 += c[0];
    t2 += c[1];
  }
  *tier1 = (int64_t)t1;
  *tier2 = (int64_t)t2;
  if (n_last > 0) {
    const int n = h->last_ws ? std::min(n_last, h->last_bq) : 0;
    for (int i = n; i < n_last; ++i) last_tiers[i] = -1;
    if (n > 0)
      RAG_HIP(hipMemcpy(last_tiers, h->last_ws->fb_tier, (size_t)n * 4, hipMemcpyDeviceToHost));
  }
  return RAG_OK;
}

int rag_index_unanswered(rag_index_t* h, int64_t* n) {
  ragmi::clear_error();
  if (!h || !n) return ragmi::fail(RAG_EINVAL, "bad args");
  std::lock_guard<std::mutex> lk(h->mu);
  RAG_HIP(hipSetDevice(h->device));
  RAG_HIP(hipDeviceSynchronize());
  unsigned long long tot = 0;
  for (auto& w : h->ws) {
    unsigned long long c[3];
    RAG_HIP(hipMemcpy(c, w.fb_cnt, sizeof(c), hipMemcpyDeviceToHost));
    tot += c[2];
  }
  *n = (int64_t)tot;
  return RAG_OK;
}

int rag_profile_enable(rag_index_t* h, int enable) {
  ragmi::clear_error();
  if (!h) return ragmi::fail(RAG_EINVAL, "index is NULL");
  std::lock_guard<std::mutex> lk(h->mu);
  h->prof = enable < 0 ? 0 : enable;
  h->prof_seq = 0;
  return RAG_OK;
}

int rag_index_set_scan_order(rag_index_t* h, int serial) {
  ragmi::clear_error();
  if (!h) return ragmi::fail(RAG_EINVAL, "index is NULL");
  std::lock_guard<std::mutex> lk(h->mu);
  h->serial_scans = serial < 0 || serial > 2 ? 1 : serial;
  h->scan_last = nullptr;
  h->scan_any = false;
  return RAG_OK;
}

int rag_stream_create_cu_partition(int device, int part, int parts, void** out) {
  ragmi::clear_error();
  if (!out || parts < 1 || part < 0 || part >= parts)
    return ragmi::fail(RAG_EINVAL, "need 0 <= part < parts and an output pointer");
  *out = nullptr;
  int n_cu = 0;
  RAG_HIP(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, device));
  // a part of >= 8 consecutive CU ids holds a CU of every XCD (bit i is on XCD i % 8); a
  // smaller one would leave XCDs without a bit, and those run on ALL their CUs
  if (parts > n_cu / 8) return ragmi::fail(RAG_EINVAL, "at most n_cu / 8 parts (8 CUs each)");
  // contiguous CU ids [part n / parts, (part + 1) n / parts)
  std::vector<uint32_t> mask((size_t)(n_cu + 31) / 32, 0u);
  const int c0 = (int)((int64_t)part * n_cu / parts), c1 = (int)((int64_t)(part + 1) * n_cu / parts);
  for (int c = c0; c < c1; ++c) mask[(size_t)c / 32] |= 1u << (c % 32);
  // (the stream belongs to the current device: switch to `device` for the call only)
  int prev = 0;
  RAG_HIP(hipGetDevice(&prev));
  RAG_HIP(hipSetDevice(device));
  hipStream_t st = nullptr;
  const hipError_t e = hipExtStreamCreateWithCUMask(&st, (uint32_t)mask.size(), mask.data());
  (void)hipSetDevice(prev);
  if (e != hipSuccess)
    return ragmi::fail(RAG_EHIP, std::string("hipExtStreamCreateWithCUMask: ") + hipGetErrorString(e));
  *out = st;
  g_stream_gen.fetch_add(1, std::memory_order_acq_rel);
  return RAG_OK;
}

int rag_stream_create_cu_mask(int device, const uint32_t* mask, int words, void** out) {
  ragmi::clear_error();
  if (!out || !mask || words < 1 || words > 32)
    return ragmi::fail(RAG_EINVAL, "need a mask of 1..32 words and an output pointer");
  *out = nullptr;
  int n = 0;
  for (int i = 0; i < words; ++i) n += __builtin_popcount(mask[i]);
  if (n == 0) return ragmi::fail(RAG_EINVAL, "empty CU mask");
  // bit i is a CU of XCD i % 8, and an XCD left with no bit runs on ALL its CUs (measured,
  // profiles/r06_cu_mask/r06s_cu_mask_probe.jsonl): such a mask would not restrict anything
  // there, so it is refused
  uint32_t xcds = 0;
  for (int i = 0; i < words * 32; ++i)
    if (mask[i / 32] >> (i % 32) & 1u) xcds |= 1u << (i % 8);
  if (xcds != 0xffu)
    return ragmi::fail(RAG_EINVAL, "CU mask must enable at least one CU of every XCD (bit i "
                                   "is on XCD i % 8)");
  int prev = 0;
  RAG_HIP(hipGetDevice(&prev));
  RAG_HIP(hipSetDevice(device));
  hipStream_t st = nullptr;
  const hipError_t e = hipExtStreamCreateWithCUMask(&st, (uint32_t)words, mask);
  (void)hipSetDevice(prev);
  if (e != hipSuccess)
    return ragmi::fail(RAG_EHIP, std::string("hipExtStreamCreateWithCUMask: ") + hipGetErrorString(e));
  *out = st;
  g_stream_gen.fetch_add(1, std::memory_order_acq_rel);
  return RAG_OK;
}

#ifdef RAGMI_DIAG_BUILD
// where a stream's workgroups run (diagnostic): per workgroup (XCC_ID, HW_ID) hardware
// registers, for mapping CU-mask bits to XCDs / shader engines / CUs
__global__ void cu_probe_kernel(int32_t* out) {
  uint32_t x, hw;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  // hold the CU a little so later workgroups spread over the allowed CUs
  const long long t0 = clock64();
  while (clock64() - t0 < 20000) {
  }
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = (int32_t)x;
    out[2 * blockIdx.x + 1] = (int32_t)hw;
  }
}
#endif

int rag_diag_cu_probe(void* stream, int n_wg, int32_t* out_dev) {
  ragmi::clear_error();
#ifdef RAGMI_DIAG_BUILD
  if (n_wg < 1 || !out_dev) return ragmi::fail(RAG_EINVAL, "n_wg >= 1 and an output buffer");
  cu_probe_kernel<<<dim3(n_wg), dim3(64), 0, static_cast<hipStream_t>(stream)>>>(out_dev);
  RAG_HIP(hipGetLastError());
  return RAG_OK;
#else
  (void)stream; (void)n_wg; (void)out_dev;
  return ragmi::fail(RAG_EINVAL, "rag_diag_cu_probe: diagnostic build only");
#endif
}

int rag_stream_destroy(void* stream) {
  ragmi::clear_error();
  if (!stream) return RAG_OK;
  g_stream_gen.fetch_add(1, std::memory_order_acq_rel);
  RAG_HIP(hipStreamDestroy(static_cast<hipStream_t>(stream)));
  return RAG_OK;
}

int rag_profile_scan_ms(rag_index_t* h, double* total_ms, int64_t* launches) {
  ragmi::clear_error();
  if (!h || !total_ms || !launches) return ragmi::fail(RAG_EINVAL, "bad args");
  std::lock_guard<std::mutex> lk(h->mu);
  double tot = 0.0;
  for (auto& p : h->prof_pairs) {
    RAG_HIP(hipEventSynchronize(p.b));
    float ms = 0.f;
    RAG_HIP(hipEventElapsedTime(&ms, p.a, p.b));
    tot += ms;
    (void)hipEventDestroy(p.a);
    (void)hipEventDestroy(p.b);
  }
  *launches = (int64_t)h->prof_pairs.size();
  *total_ms = tot;
  h->prof_pairs.clear();
  return RAG_OK;
}

int rag_profile_scan_intervals(rag_index_t* h, double* start_ms, double* end_ms, int64_t cap,
                               int64_t* launches) {
  ragmi::clear_error();
  if (!h || !launches || cap < 0 || (cap > 0 && (!start_ms || !end_ms)))
    return ragmi::fail(RAG_EINVAL, "bad args");
  std::lock_guard<std::mutex> lk(h->mu);
  const int64_t n = (int64_t)h->prof_pairs.size();
  for (int64_t i = 0; i < n; ++i) RAG_HIP(hipEventSynchronize(h->prof_pairs[(size_t)i].b));
  // every interval relative to the first recorded launch's start event (events of different
  // streams on one device share the device clock; an earlier launch reads negative)
  for (int64_t i = 0; i < n && i < cap; ++i) {
    const ProfPair& p = h->prof_pairs[(size_t)i];
    float a = 0.f, b = 0.f;
    RAG_HIP(hipEventElapsedTime(&a, h->prof_pairs[0].a, p.a));
    RAG_HIP(hipEventElapsedTime(&b, h->prof_pairs[0].a, p.b));
    start_ms[i] = a;
    end_ms[i] = b;
  }
  for (auto& p : h->prof_pairs) {
    (void)hipEventDestroy(p.a);
    (void)hipEventDestroy(p.b);
  }
  h->prof_pairs.clear();
  *launches = n;
  return RAG_OK;
}

}  // extern "C"
