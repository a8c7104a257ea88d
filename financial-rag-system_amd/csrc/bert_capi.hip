// bert_capi.hip — extern "C" boundary of the encoders (include/ragmi_bert.h): weight upload
// (fp32 HF layout -> fp16 GEMM weights with fused Q|K|V), workspace, forward launch sequence.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <type_traits>
#include <vector>

#include "../../include/ragmi_bert.h"
#include "bert_kernels.hip"
#include "common_host.hpp"

namespace {

using namespace ragmi::bert;
using ragmi::launch_fixed;

// largest static fp16 range bound accepted (fp16 max 65504; see range_bounds)
constexpr double kF16Safe = 60000.0;
// split-K of the small-batch fp32-output GEMMs (small_ksplit): most parts, and the workspace
// rows up to which y keeps room for them
constexpr int kMaxKSplit = 4;
static_assert(kMaxKSplit <= 4, "add_ln384_kernel sums at most 4 split-K parts");
constexpr int64_t kSplitMaxRows = 8192;

struct Layer {
  _Float16 *wqkv = nullptr, *wo = nullptr, *w1 = nullptr, *w2 = nullptr;
  _Float16 *wqkv_l = nullptr, *wo_l = nullptr, *w1_l = nullptr, *w2_l = nullptr;  // fp16x3
  float *bqkv = nullptr, *bo = nullptr, *g1 = nullptr, *be1 = nullptr, *bi1 = nullptr,
        *bi2 = nullptr, *g2 = nullptr, *be2 = nullptr;
  // deferred LayerNorm (fp16x3, hidden 384; DlArgs in bert_kernels.hip): the consumers of a
  // pending LN with its gamma folded into the weights — QKV (the previous layer's output LN;
  // layers >= 1) and FFN1 (this layer's attention-output LN) — and per output column c1 (the
  // folded planes' row sums) and c2 (bias + W beta)
  _Float16 *wqkv_f = nullptr, *wqkv_fl = nullptr, *w1_f = nullptr, *w1_fl = nullptr;
  float *qkv_c1 = nullptr, *qkv_c2 = nullptr, *w1_c1 = nullptr, *w1_c2 = nullptr;
};

__global__ void f32_to_f16_kernel(const float* __restrict__ in, _Float16* __restrict__ out,
                                  _Float16* __restrict__ out_lo, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    _Float16 h, l;
    { const half2 s16_ = split16(in[i]); h = s16_[0]; l = s16_[1]; }
    out[i] = h;
    if (out_lo) out_lo[i] = l;
  }
}

// c1[n] = sum_k (hi + lo)[n][k] in fp64 (the folded weights exactly as the GEMM sees them)
__global__ void fold_c1_kernel(const _Float16* __restrict__ hi, const _Float16* __restrict__ lo,
                               int N, int K, float* __restrict__ c1) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  double s = 0.0;
  for (int k = 0; k < K; ++k)
    s += (double)(float)hi[(int64_t)n * K + k] + (double)(float)lo[(int64_t)n * K + k];
  c1[n] = (float)s;
}

}  // namespace

// Activations of one forward in flight (grown on demand). One per HIP stream that calls the
// encoder: forwards on different streams run concurrently on the GPU (e.g. query batches of
// a serving loop pipelined over streams), so they must not share activation buffers; forwards
// on one stream are ordered by the stream and reuse its workspace.
struct EncWorkspace {
  hipStream_t stream = nullptr;
  uint64_t last_use = 0;
  int64_t cap_t = 0;
  int64_t y_rows = 0, yc_rows = 0;   // rows y / yc hold (room for split-K parts at small T)
  float *x = nullptr, *y = nullptr;
  _Float16 *xh = nullptr, *qkv = nullptr, *ctx = nullptr, *ff = nullptr;
  _Float16 *xl = nullptr, *qkv_l = nullptr, *ctx_l = nullptr, *ff_l = nullptr;  // fp16x3
  // last layer on the CLS rows only (B rows; see gather_cls_kernel)
  int64_t cap_b = 0;
  float *xc = nullptr, *yc = nullptr;
  _Float16 *xch = nullptr, *xcl = nullptr, *cc = nullptr, *ccl = nullptr, *ffc = nullptr,
           *ffcl = nullptr;
  // deferred LayerNorm: row statistics of z after the attention block (sa) / the FFN (sb)
  float *sa = nullptr, *sb = nullptr;

  // hipGraph replay of small-batch forwards (forward_graph): executable graphs keyed by the
  // padded shape (B, T, max_len), the padded inputs they read ([ids T | types T | cu B+1])
  // and the rows they write. A graph holds this workspace's buffer addresses: any regrowth
  // drops them (drop_graphs).
  struct Graph {
    int B = 0, T = 0, L = 0;
    hipGraphExec_t exec = nullptr;
    uint64_t last = 0;
  };
  std::vector<Graph> graphs;
  int32_t* g_in = nullptr;
  int64_t g_in_cap = 0;     // int32 elements
  float* g_out = nullptr;
  int64_t g_out_cap = 0;    // floats
  // private capture stream: capturing on the caller's stream in relaxed mode would
  // record any other thread's launches on that stream into the graph
  hipStream_t cstream = nullptr;

  void drop_graphs() {   // (a replay may still run on the workspace's stream: wait for it —
    // device-wide, since the caller may have destroyed that stream since its last forward)
    if (!graphs.empty()) (void)hipDeviceSynchronize();
    for (auto& g : graphs)
      if (g.exec) (void)hipGraphExecDestroy(g.exec);
    graphs.clear();
  }

  void release() {
    drop_graphs();
    for (void* p : {(void*)x, (void*)y, (void*)xh, (void*)qkv, (void*)ctx, (void*)ff, (void*)xl,
                    (void*)qkv_l, (void*)ctx_l, (void*)ff_l, (void*)xc, (void*)yc, (void*)xch,
                    (void*)xcl, (void*)cc, (void*)ccl, (void*)ffc, (void*)ffcl, (void*)sa,
                    (void*)sb, (void*)g_in, (void*)g_out})
      if (p) (void)hipFree(p);
    if (cstream) (void)hipStreamDestroy(cstream);
    *this = EncWorkspace{};
  }
};

struct rag_encoder {
  rag_bert_config cfg{};
  int device = 0;
  bool diagnostic = false;   // counted in ragmi::diagnostic_handles() (common_host.hpp)
  std::mutex mu;
  std::vector<void*> allocs;
  float *wemb = nullptr, *pemb = nullptr, *temb = nullptr, *eg = nullptr, *eb = nullptr;
  std::vector<Layer> layers;
  float *wp = nullptr, *bp = nullptr, *wc = nullptr, *bc = nullptr;
  // per-stream activation workspaces (at most kMaxWorkspaces; see workspace_for)
  std::vector<EncWorkspace> ws;
  uint64_t uses = 0;
  // residual + LayerNorm fused into the output projections: -1 auto, 0 off, 1 on
  int fuse_ln = -1;
  // deferred LayerNorm on the token rows (fp16x3, hidden 384): -1 auto, 0 off, 1 on
  int defer_ln = -1;
  // the deferred-LN FFN as one fused launch (ffn_fused_kernel): -1 auto, 0 off, 1 on
  int ffn_fused = -1;
  // hipGraph replay of small-batch forwards: -1 auto, 0 off, 1 on. A call on the null stream
  // replays on the encoder's own stream, ordered by two events (gstream, gev_*)
  int graphs = -1;
  hipStream_t gstream = nullptr;
  hipEvent_t gev_in = nullptr, gev_out = nullptr;
  // static fp16 range analysis of the weights (range_bounds): the largest |value| any fp16
  // (hi) plane of the forward can hold, for any input — without / with the deferred LayerNorm
  // (whose z planes hold the un-normalised residual sums)
  double bound_plain = 0.0, bound_defer = 0.0;
  // host-entry staging
  void* stage = nullptr;
  size_t stage_bytes = 0;
};

namespace {

template <typename T>
int dalloc(rag_encoder* e, T** p, size_t n) {
  RAG_HIP(hipMalloc(reinterpret_cast<void**>(p), std::max<size_t>(n * sizeof(T), 16)));
  e->allocs.push_back(*p);
  return RAG_OK;
}

int up_f32(rag_encoder* e, float** dst, const float* src, size_t n) {
  int rc = dalloc(e, dst, n);
  if (rc) return rc;
  RAG_HIP(hipMemcpy(*dst, src, n * 4, hipMemcpyHostToDevice));
  return RAG_OK;
}

// fp16 copy (and, for fp16x3, the fp16 residual lo = fp16(w - hi)) of one or more host fp32
// blocks laid end to end ([rows][K] each)
int up_f16(rag_encoder* e, _Float16** dst, _Float16** dst_lo,
           std::initializer_list<std::pair<const float*, size_t>> parts) {
  size_t n = 0;
  for (auto& p : parts) n += p.second;
  int rc = dalloc(e, dst, n);
  if (rc) return rc;
  if (dst_lo) {
    rc = dalloc(e, dst_lo, n);
    if (rc) return rc;
  }
  float* tmp = nullptr;
  RAG_HIP(hipMalloc(reinterpret_cast<void**>(&tmp), n * 4));
  size_t off = 0;
  for (auto& p : parts) {
    if (hipMemcpy(tmp + off, p.first, p.second * 4, hipMemcpyHostToDevice) != hipSuccess) {
      (void)hipFree(tmp);
      return ragmi::fail(RAG_EHIP, "weight upload failed");
    }
    off += p.second;
  }
  f32_to_f16_kernel<<<dim3((unsigned)((n + 255) / 256)), dim3(256)>>>(
      tmp, *dst, dst_lo ? *dst_lo : nullptr, (int64_t)n);
  RAG_HIP(hipDeviceSynchronize());
  (void)hipFree(tmp);
  return RAG_OK;
}

// deferred LayerNorm's folded consumer weights (see Layer): W' = W diag(gamma) (fp32 products,
// then fp16x3 planes), c1 = the planes' row sums (fold_c1_kernel), c2 = b + W beta (fp64).
// parts: (W [rows][K], b [rows]) blocks laid end to end (Q | K | V for the fused QKV)
int fold_ln(rag_encoder* e, std::initializer_list<std::pair<const float*, const float*>> parts,
            size_t rows, size_t K, const float* gam, const float* bet, _Float16** wf,
            _Float16** wfl, float** c1, float** c2) {
  const size_t N = parts.size() * rows;
  std::vector<float> wv(N * K), b2(N);
  size_t n = 0;
  for (auto& p : parts)
    for (size_t r = 0; r < rows; ++r, ++n) {
      double acc = p.second[r];
      for (size_t k = 0; k < K; ++k) {
        wv[n * K + k] = p.first[r * K + k] * gam[k];
        acc += (double)p.first[r * K + k] * (double)bet[k];
      }
      b2[n] = (float)acc;
    }
  int rc = up_f16(e, wf, wfl, {{wv.data(), N * K}});
  if (!rc) rc = up_f32(e, c2, b2.data(), N);
  if (!rc) rc = dalloc(e, c1, N);
  if (rc) return rc;
  fold_c1_kernel<<<dim3((unsigned)((N + 255) / 256)), dim3(256)>>>(*wf, *wfl, (int)N, (int)K, *c1);
  RAG_HIP(hipDeviceSynchronize());
  return RAG_OK;
}

int ensure_ws(const rag_bert_config& cfg, EncWorkspace* w, int64_t T) {
  if (T <= w->cap_t) return RAG_OK;
  w->drop_graphs();
  const int64_t cap = std::max<int64_t>(T, std::max<int64_t>(2 * w->cap_t, 1024));
  for (void* p : {(void*)w->x, (void*)w->y, (void*)w->xh, (void*)w->qkv, (void*)w->ctx,
                  (void*)w->ff, (void*)w->xl, (void*)w->qkv_l, (void*)w->ctx_l, (void*)w->ff_l,
                  (void*)w->sa, (void*)w->sb})
    if (p) (void)hipFree(p);
  w->x = w->y = w->sa = w->sb = nullptr;
  w->xh = w->qkv = w->ctx = w->ff = nullptr;
  w->xl = w->qkv_l = w->ctx_l = w->ff_l = nullptr;
  w->cap_t = 0;
  const int64_t H = cfg.hidden, FF = cfg.intermediate;
  if (cfg.precision == RAG_PREC_FP16X3) {
    RAG_HIP(hipMalloc(reinterpret_cast<void**>(&w->xl), cap * H * 2));
    RAG_HIP(hipMalloc(reinterpret_cast<void**>(&w->qkv_l), cap * 3 * H * 2));
    RAG_HIP(hipMalloc(reinterpret_cast<void**>(&w->ctx_l), cap * H * 2));
    RAG_HIP(hipMalloc(reinterpret_cast<void**>(&w->ff_l), cap * FF * 2));
    if (H == kDlH) {
      RAG_HIP(hipMalloc(reinterpret_cast<void**>(&w->sa), cap * kDlParts * 8));
      RAG_HIP(hipMalloc(reinterpret_cast<void**>(&w->sb), cap * kDlParts * 8));
    }
  }
  RAG_HIP(hipMalloc(reinterpret_cast<void**>(&w->x), cap * H * 4));
  w->y_rows = cap <= kSplitMaxRows ? cap * kMaxKSplit : cap;
  RAG_HIP(hipMalloc(reinterpret_cast<void**>(&w->y), w->y_rows * H * 4));
  RAG_HIP(hipMalloc(reinterpret_cast<void**>(&w->xh), cap * H * 2));
  RAG_HIP(hipMalloc(reinterpret_cast<void**>(&w->qkv), cap * 3 * H * 2));
  RAG_HIP(hipMalloc(reinterpret_cast<void**>(&w->ctx), cap * H * 2));
  RAG_HIP(hipMalloc(reinterpret_cast<void**>(&w->ff), cap * FF * 2));
  w->cap_t = cap;
  return RAG_OK;
}

constexpr size_t kMaxWorkspaces = 8;

// the workspace of `st` (created on first use); beyond kMaxWorkspaces streams the least
// recently used one is taken over after a device synchronize (its stream may still be
// running work that reads it; the stream itself may be gone, so it is not waited on)
EncWorkspace* workspace_for(rag_encoder* e, hipStream_t st) {
  ++e->uses;
  for (auto& w : e->ws)
    if (w.stream == st) {
      w.last_use = e->uses;
      return &w;
    }
  if (e->ws.size() < kMaxWorkspaces) {
    e->ws.emplace_back();
  } else {
    auto lru = std::min_element(e->ws.begin(), e->ws.end(),
                                [](const EncWorkspace& a, const EncWorkspace& b) {
                                  return a.last_use < b.last_use;
                                });
    if (hipDeviceSynchronize() != hipSuccess) return nullptr;
    std::iter_swap(lru, e->ws.end() - 1);
  }
  EncWorkspace& w = e->ws.back();
  w.stream = st;
  w.last_use = e->uses;
  return &w;
}

// GEMM variants: RAG_GEMM_TILE (gemm_kernel: one 128x128 tile per workgroup, 2 per CU),
// RAG_GEMM_SMALL (gemm_pipe_kernel<PipeSmall>: 64x64 tiles, the K panel in flight at once) and
// RAG_GEMM_WS (gemm_ws_kernel<PipeLarge>: persistent, one workgroup per CU, 8 MFMA waves fed
// by 4 loader waves through an LDS-DMA ring of 256x128 tiles); AUTO's choice is in gemm().
int cu_count() {
  static int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      v = 256;
    return std::max(8, v / 8 * 8);
  }();
  return n;
}

// RAGMI_* knobs below: diagnostic A/B only, honoured under RAG_CREATE_DIAGNOSTIC (ragmi::Knob)
int gemm_variant_default() {
  static ragmi::Knob k("RAGMI_GEMM");
  const char* s = k.str();
  if (s && std::strcmp(s, "tile") == 0) return (int)RAG_GEMM_TILE;
  if (s && std::strcmp(s, "ws") == 0) return (int)RAG_GEMM_WS;
  if (s && std::strcmp(s, "small") == 0) return (int)RAG_GEMM_SMALL;
  return (int)RAG_GEMM_AUTO;
}

// the DMA kernels address each operand and the output through 32-bit buffer extents
bool pipe_ok(int M, int N, int K) {
  return N % PBN == 0 && K % 64 == 0 && N <= kPipeBiasMax &&
         (int64_t)M * K * 2 < (int64_t(1) << 31) && (int64_t)M * N * 4 < (int64_t(1) << 31);
}

template <int EPI, bool SPLIT, typename CFG>
void launch_pipe(const _Float16* A, const _Float16* Al, const _Float16* W, const _Float16* Wl,
                 const float* bias, int M, int N, int K, void* C, _Float16* Clo, hipStream_t st,
                 int max_wg, const LnArgs& ln = LnArgs{}, int ksplit = 1) {
  const int tiles = (N / CFG::BN) * ((M + CFG::BM - 1) / CFG::BM) * ksplit;
  const dim3 grid((unsigned)std::min(max_wg, (tiles + 7) / 8 * 8));   // multiple of 8
  launch_fixed<kPipeBlock<CFG>>(gemm_pipe_kernel<EPI, SPLIT, CFG>, grid, 0, st, A, Al, W,
                                Wl, bias, M, N, K, C, Clo, ln, ksplit);
}

// split-K of the small-batch fp32-output GEMMs (O-proj, FFN2 of query batches: 64x64 tiles,
// one serial K loop per tile): K parts per tile, a function of K only, so a sequence's output
// never depends on what else is in its batch (tests/test_encoders_gpu.py batch independence).
// The parts are summed in order by add_ln_kernel. 0 = no split for this shape.
int small_ksplit(int K, int BK) {
  static ragmi::Knob k("RAGMI_KSPLIT");                     // diagnostic: 1 = off, n = force
  const int force = k.get(0);
  const int nk = K / BK;
  int s = force > 0 ? force : K >= 1536 ? 3 : K >= 384 ? 2 : 1;
  s = std::min(s, kMaxKSplit);
  while (s > 1 && nk % s) --s;
  return s;
}

// CUs a stream may use (its CU mask, rag_stream_create_cu_mask / _partition), rounded down to
// a multiple of 8 (the WS kernel's XCD-aware tile order assumes G % 8 == 0); the null stream,
// unmasked streams and a failed query -> every CU. The persistent WS grid is one workgroup per
// allowed CU: sized to the device, a masked stream would queue the extra workgroups behind
// the first ones and run a second round.
int stream_cus_enc(hipStream_t st) {
  if (!st) return cu_count();
  uint32_t mask[32] = {};
  const int words = std::min(32, (cu_count() + 31) / 32);
  if (hipExtStreamGetCUMask(st, (uint32_t)words, mask) != hipSuccess) {
    (void)hipGetLastError();
    return cu_count();
  }
  int n = 0;
  for (int i = 0; i < words; ++i) n += __builtin_popcount(mask[i]);
  n = n / 8 * 8;
  return n >= 8 && n < cu_count() ? n : cu_count();
}

template <int EPI, bool SPLIT, typename CFG, int PROBE = 0, int AUX = 0>
void launch_ws(const _Float16* A, const _Float16* Al, const _Float16* W, const _Float16* Wl,
               const float* bias, int M, int N, int K, void* C, _Float16* Clo, hipStream_t st,
               const DlArgs& dl = DlArgs{}) {
  const int tiles = (N / CFG::BN) * ((M + CFG::BM - 1) / CFG::BM);
  const dim3 grid((unsigned)std::min(stream_cus_enc(st), (tiles + 7) / 8 * 8));   // one per CU
  launch_fixed<kWsBlock<CFG>>(gemm_ws_kernel<EPI, SPLIT, CFG, PROBE, AUX>, grid, 0, st, A, Al, W,
                              Wl, bias, M, N, K, C, Clo, dl);
}

// the large-batch GEMMs (the WS kernel on PipeLarge: 8 MFMA waves of 64 x 64 + 4 loader waves)
template <int EPI, bool SPLIT, int AUX = 0>
void launch_ws_large(const _Float16* A, const _Float16* Al, const _Float16* W, const _Float16* Wl,
                     const float* bias, int M, int N, int K, void* C, _Float16* Clo,
                     hipStream_t st, const DlArgs& dl = DlArgs{}) {
  launch_ws<EPI, SPLIT, PipeLarge, 0, AUX>(A, Al, W, Wl, bias, M, N, K, C, Clo, st, dl);
}

// the 2-wave attention workgroups for query batches of sequences <= 32 tokens (attn_kernel
// THREADS = 128); RAGMI_ATTN_SHORT=0 (diagnostic A/B) keeps the 8-wave ones
bool attn_short(int hd, int max_len) {
  static ragmi::Knob k("RAGMI_ATTN_SHORT");
  return hd == 32 && max_len <= 32 && k.get(1) != 0;
}

// RAGMI_CLS_ATTN=0 (diagnostic A/B): the last layer's all-token QKV + attention instead of
// the K|V projection + CLS-only attention (round 4: rerank forward 9.17-9.19 vs 9.30-9.32 ms,
// profiles/r04aa_cls_attention_ab.jsonl)
bool cls_attn_on() {
  static ragmi::Knob k("RAGMI_CLS_ATTN");
  return k.get(1) != 0;
}

// shapes the deferred-LayerNorm WS GEMMs take: Ln* (K = 384 input rows; c1 | c2 staged in the
// 4096-float bias area) and ResLn (N = 384 output rows; bias | gamma | beta)
bool dl_gemm_ok(int epi, int M, int N, int K) {
  if (!pipe_ok(M, N, K)) return false;
  if (epi == kEpiResLn) return N == kDlH;
  return K == kDlH && 2 * N <= kPipeBiasMax;
}

#ifdef RAGMI_DIAG_BUILD
// the fused deferred-LN FFN (ffn_fused_kernel): hidden 384, intermediate 1536 (bge-small,
// MiniLM-L6), inside the deferred-LayerNorm forward. Auto: once the 128-row tiles fill every
// CU at least twice (round 6 measurements)
bool ffn_fused_for(const rag_encoder* e, int T, int FF) {
  if (FF != kFfnFF || e->ffn_fused == 0) return false;
  if (e->ffn_fused > 0) return true;
  return false;
}
// chunk width of the fused FFN (FfnRing): mode 1 -> V 0 (128 columns of H per pass), mode 2
// -> V 1 (256)
// (A/B modes 3 / 4 / 5: chunk 256 + the next stage's DMA issued mid-step / + s_setprio 1 on
// waves 4-7 / both)
int ffn_ring(const rag_encoder* e) {
  switch (e->ffn_fused) {
    case 2: return 1;
    case 3: return 3;
    case 4: return 5;
    case 5: return 7;
    default: return 0;
  }
}

void launch_ffn_fused(_Float16* zh, _Float16* zl, int M, const FfnArgs& a, hipStream_t st,
                      int ring) {
  const int tiles = (M + kFfnBM - 1) / kFfnBM;
  const dim3 grid((unsigned)std::max(1, std::min(cu_count(), tiles)));   // one per CU
  switch (ring) {
    case 1: launch_fixed<kFfnThreads>(ffn_fused_kernel<1>, grid, 0, st, zh, zl, M, a); break;
    case 3: launch_fixed<kFfnThreads>(ffn_fused_kernel<3>, grid, 0, st, zh, zl, M, a); break;
    case 5: launch_fixed<kFfnThreads>(ffn_fused_kernel<5>, grid, 0, st, zh, zl, M, a); break;
    case 7: launch_fixed<kFfnThreads>(ffn_fused_kernel<7>, grid, 0, st, zh, zl, M, a); break;
    default: launch_fixed<kFfnThreads>(ffn_fused_kernel<0>, grid, 0, st, zh, zl, M, a); break;
  }
}

#endif

// deferred-LayerNorm mode of the forward: -1 auto, 0 off, 1 on (where the shapes allow)
int defer_ln_default() {
  static ragmi::Knob k("RAGMI_DEFER_LN");
  return k.get(-1);
}

// the fused output projection + residual + LayerNorm (kEpiAddLn on PipeRow tiles)
bool add_ln_ok(int M, int N, int K) {
  return N == PipeRow::BN && K % 64 == 0 && (int64_t)M * K * 2 < (int64_t(1) << 31) &&
         (int64_t)M * N * 4 < (int64_t(1) << 31);
}

// x[M,N] = LN(x + A . W^T + bias) * gamma + beta (fp32, in place), xh = fp16(x)
// [, xl = fp16(x - xh)]: BertSelfOutput / BertOutput (dense + dropout(eval) + LayerNorm of
// the sum with the residual) in one pass over the rows
void gemm_add_ln(const _Float16* A, const _Float16* Al, const _Float16* W, const _Float16* Wl,
                 const float* bias, const float* gamma, const float* beta, float eps, int M,
                 int N, int K, float* x, _Float16* xh, _Float16* xl, hipStream_t st) {
  LnArgs ln;
  ln.gamma = gamma;
  ln.beta = beta;
  ln.xh = xh;
  ln.eps = eps;
  if (Al)
    launch_pipe<kEpiAddLn, true, PipeRow>(A, Al, W, Wl, bias, M, N, K, x, xl, st, cu_count(), ln);
  else
    launch_pipe<kEpiAddLn, false, PipeRow>(A, nullptr, W, nullptr, bias, M, N, K, x, nullptr, st,
                                           cu_count(), ln);
}

// fusion mode of the forward: -1 auto (once the 128-row bands cover the CUs), 0 off, 1 on
int fuse_ln_default() {
  static ragmi::Knob k("RAGMI_FUSE_LN");
  return k.get(-1);
}

int ensure_cls(const rag_bert_config& cfg, EncWorkspace* w, int64_t B) {
  if (B <= w->cap_b) return RAG_OK;
  w->drop_graphs();
  for (void* p : {(void*)w->xc, (void*)w->yc, (void*)w->xch, (void*)w->xcl, (void*)w->cc,
                  (void*)w->ccl, (void*)w->ffc, (void*)w->ffcl})
    if (p) (void)hipFree(p);
  w->xc = w->yc = nullptr;
  w->xch = w->xcl = w->cc = w->ccl = w->ffc = w->ffcl = nullptr;
  w->cap_b = 0;
  const int64_t cap = std::max<int64_t>(B, 256), H = cfg.hidden, FF = cfg.intermediate;
  RAG_HIP(hipMalloc(reinterpret_cast<void**>(&w->xc), cap * H * 4));
  w->yc_rows = cap * kMaxKSplit;
  RAG_HIP(hipMalloc(reinterpret_cast<void**>(&w->yc), w->yc_rows * H * 4));
  RAG_HIP(hipMalloc(reinterpret_cast<void**>(&w->xch), cap * H * 2));
  RAG_HIP(hipMalloc(reinterpret_cast<void**>(&w->cc), cap * H * 2));
  RAG_HIP(hipMalloc(reinterpret_cast<void**>(&w->ffc), cap * FF * 2));
  if (cfg.precision == RAG_PREC_FP16X3) {
    RAG_HIP(hipMalloc(reinterpret_cast<void**>(&w->xcl), cap * H * 2));
    RAG_HIP(hipMalloc(reinterpret_cast<void**>(&w->ccl), cap * H * 2));
    RAG_HIP(hipMalloc(reinterpret_cast<void**>(&w->ffcl), cap * FF * 2));
  }
  w->cap_b = cap;
  return RAG_OK;
}

// ksplit_io: in = the split-K parts the caller's C can hold (1 = no split; kEpiF32 only),
// out = the parts written (the caller sums them: add_ln_kernel)
template <int EPI>
void gemm(const _Float16* A, const _Float16* Al, const _Float16* W, const _Float16* Wl,
          const float* bias, int M, int N, int K, void* C, _Float16* Clo, hipStream_t st,
          int variant = RAG_GEMM_AUTO, int* ksplit_io = nullptr) {
  const int ks_room = ksplit_io ? *ksplit_io : 1;
  if (ksplit_io) *ksplit_io = 1;
  if (variant == RAG_GEMM_AUTO) variant = gemm_variant_default();
  const int pipe_tiles = (N / PBN) * ((M + PBM - 1) / PBM);
  // SMALL while its 64x64 tiles fit about two per CU (every query-batch GEMM; the N = 384
  // ones up to ~5K tokens), then WS (the loader-specialised pipe) once its 256x128 tiles reach
  // half the CUs, TILE in between. Measured per layer (QKV + O + FFN1 + FFN2, scripts/
  // bench_gemm.py, profiles/r02_gemm_ws.jsonl): 117K tokens fp16x3 WS 1.337 ms vs PIPE 1.447,
  // WIDE 1.416, TILE 1.547; 14.8K fp16x3 0.190 vs 0.216 / 0.223 / 0.216; at 4K tokens the
  // N = 384 GEMMs (48 tiles) run faster as TILE
  const int small_tiles = (N / 64) * ((M + 63) / 64);
  if (variant == RAG_GEMM_AUTO)
    variant = !pipe_ok(M, N, K)                  ? RAG_GEMM_TILE
              : small_tiles <= 2 * cu_count()    ? RAG_GEMM_SMALL
              : 2 * pipe_tiles >= cu_count()     ? RAG_GEMM_WS
                                                 : RAG_GEMM_TILE;
  if (variant != RAG_GEMM_TILE && !pipe_ok(M, N, K)) variant = RAG_GEMM_TILE;
  // (the small-batch A/B forms — BK-64 tiles, 64 x 128 tiles, loader-specialised small tiles —
  // and the PIPE / WIDE / BIG large-batch forms were measured and removed in round 5:
  // DESIGN.md §R5 lists their numbers)
  if (variant == RAG_GEMM_WS || variant == RAG_GEMM_WS_MFMA_ONLY ||
      variant == RAG_GEMM_WS_NO_STORE || variant == RAG_GEMM_WS_DMA_ONLY) {
    // non-temporal stores for the fp16 outputs (QKV / FFN1: 117K x 1152 fp16x3 0.354 ->
    // 0.310 ms, the streamed 540 MB no longer evicting the A panels the n-tiles of an XCD
    // share); the fp32 ones (O / FFN2, read back at once by add_ln) keep the default policy.
    // The probes keep production's store policy.
    constexpr int AX = EPI == kEpiF32 ? 0 : 2;
    auto go = [&](auto pc) {
      constexpr int P = decltype(pc)::value;
      if (Al) launch_ws<EPI, true, PipeLarge, P, AX>(A, Al, W, Wl, bias, M, N, K, C, Clo, st);
      else launch_ws<EPI, false, PipeLarge, P, AX>(A, nullptr, W, nullptr, bias, M, N, K, C, nullptr, st);
    };
    if (variant == RAG_GEMM_WS) go(std::integral_constant<int, 0>{});
    else if (variant == RAG_GEMM_WS_MFMA_ONLY) go(std::integral_constant<int, 7>{});
    else if (variant == RAG_GEMM_WS_NO_STORE) go(std::integral_constant<int, 6>{});
    else go(std::integral_constant<int, 8>{});
    return;
  }
  // split-K parts for the small fp32-output GEMMs (small_ksplit), where the caller has room
  auto ks_for = [&](int BK) {
    if constexpr (EPI != kEpiF32) return 1;
    if (ks_room <= 1 || N > kPipeBiasMax / 2) return 1;
    return std::min(ks_room, small_ksplit(K, BK));
  };
  if (variant == RAG_GEMM_SMALL) {
    // BK-32 tiles (64 KB LDS: 2 workgroups per CU; round 3: 782-token bge-small forward 0.628
    // vs 0.637 ms with BK-64 tiles at 1 per CU, and the config-2 line at 3 batches in flight
    // 71.1K vs 65.9K qps, where a 1-per-CU GEMM keeps the other batches' kernels off its CUs)
    const int ks = ks_for(Al ? kBK<true> : kBK<false>);
    // fp16x3 up to N = 2048: the 40 KB form, four workgroups per CU (PipeSmallR2; RAGMI_
    // SMALL_RING=3 on a diagnostic handle keeps the 3-stage one for A/Bs)
    static ragmi::Knob ring_knob("RAGMI_SMALL_RING");
    if (Al && ring_knob.get(2) == 2 && N <= PipeSmallR2::BIAS &&
        (ks == 1 || N <= PipeSmallR2::BIAS / 2)) {
      launch_pipe<EPI, true, PipeSmallR2>(A, Al, W, Wl, bias, M, N, K, C, Clo, st,
                                          4 * cu_count(), LnArgs{}, ks);
      if (ksplit_io) *ksplit_io = ks;
      return;
    }
    if (Al)   // 48 KB ring + 16 KB bias area: two workgroups per CU
      launch_pipe<EPI, true, PipeSmall<true>>(A, Al, W, Wl, bias, M, N, K, C, Clo, st,
                                              2 * cu_count(), LnArgs{}, ks);
    else
      launch_pipe<EPI, false, PipeSmall<false>>(A, nullptr, W, nullptr, bias, M, N, K, C,
                                                nullptr, st, 2 * cu_count(), LnArgs{}, ks);
    if (ksplit_io) *ksplit_io = ks;
    return;
  }
  const unsigned tiles = (unsigned)((N / BN) * ((M + BM - 1) / BM));
  const dim3 grid((tiles + 7) / 8 * 8);          // multiple of 8: XCD-aware tile order
  if (Al)
    gemm_kernel<EPI, true><<<grid, dim3(256), 0, st>>>(A, Al, W, Wl, bias, M, N, K, C, Clo);
  else
    gemm_kernel<EPI, false><<<grid, dim3(256), 0, st>>>(A, nullptr, W, nullptr, bias, M, N, K,
                                                        C, nullptr);
}

template <int H, int HD>
int forward_graph(rag_encoder* e, EncWorkspace* w, const int32_t* ids, const int32_t* types,
                  const int32_t* cu, int B, int T, int max_len, float* out, hipStream_t st);

// graph replay for this call? (small token batches on a non-null stream: the ~90 launches
// of a forward cost ~260 us of host time against ~620 us of device time at 32 queries,
// profiles/r03f_host_launch.jsonl; a replay is three host calls)
constexpr int kGraphMaxT = 8192;
constexpr int kGraphCache = 16;    // graphs per workspace (LRU)
bool use_graphs(const rag_encoder* e, hipStream_t st, int T, bool null_ok = false) {
  static ragmi::Knob k("RAGMI_ENC_GRAPH");
  const int env = k.get(-1);
  const int mode = e->graphs >= 0 ? e->graphs : env;
  if (mode == 0 || (st == nullptr && !null_ok)) return false;
  return mode > 0 || T <= kGraphMaxT;
}

template <int H, int HD>
int forward_t(rag_encoder* e, const int32_t* ids, const int32_t* types, const int32_t* cu,
              int B, int T, int max_len, float* out, hipStream_t st, bool capturing = false,
              EncWorkspace* w_in = nullptr) {
  const rag_bert_config& c = e->cfg;
  const int NH = H / HD, FF = c.intermediate;
  EncWorkspace* w = w_in ? w_in : workspace_for(e, st);
  if (!w) return ragmi::fail(RAG_EHIP, "device synchronize failed");
  if (!capturing && use_graphs(e, st, T))
    return forward_graph<H, HD>(e, w, ids, types, cu, B, T, max_len, out, st);
  int rc = ensure_ws(c, w, T);
  if (rc) return rc;
  rc = ensure_cls(c, w, B);
  if (rc) return rc;
  // fused: the output projections' epilogue adds the residual and normalises whole 384-wide
  // rows (saves the fp32 y round trip and add_ln's extra pass). Auto: fp16 mode once the
  // 128-row bands fill the CUs (rerank batch, 117K tokens: 5.25 -> 4.92 ms). In fp16x3 the
  // 128x384 two-stage ring loses to the 256x128 three-stage one by what the fusion saves
  // (10.63 vs 10.67 ms), so auto leaves it off there.
  auto fuse_for = [&](int R) {
    return add_ln_ok(R, H, FF) && add_ln_ok(R, H, H) &&
           (e->fuse_ln > 0 || (e->fuse_ln < 0 && !w->xl &&
                               (R + PipeRow::BM - 1) / PipeRow::BM >= cu_count()));
  };
  // fp16x3 with the two-kernel projections: the token rows' residual stream is kept as the
  // operand planes xh + xl alone (add_ln_kernel<XF>), no fp32 copy
  // deferred LayerNorm (DlArgs): auto once every token-row GEMM is a WS one (AUTO's choice:
  // the 384-wide projections' 256 x 128 tiles reach half the CUs, ~11K tokens)
  const bool dl_shapes = [&] {
    if (e->defer_ln == 0 || H != kDlH || !w->xl || !w->sa || !e->layers[0].w1_f ||
        e->bound_defer > kF16Safe)
      return false;
    return dl_gemm_ok(kEpiLnF16, T, 3 * H, H) && dl_gemm_ok(kEpiLnGeluF16, T, FF, H) &&
           dl_gemm_ok(kEpiResLn, T, H, H) && dl_gemm_ok(kEpiResLn, T, H, FF);
  }();
  const bool dl = [&] {
    if (!dl_shapes) return false;
    if (e->defer_ln > 0) return true;
    const int tiles384 = (H / PBN) * ((T + PBM - 1) / PBM);
    return gemm_variant_default() == RAG_GEMM_AUTO && 2 * tiles384 >= cu_count() &&
           (H / 64) * ((T + 63) / 64) > 2 * cu_count();
  }();
  const bool xf = dl || (w->xl && !fuse_for(T));
  embed_ln_kernel<H><<<dim3((max_len + 3) / 4, B), dim3(256), 0, st>>>(
      ids, types, cu, e->wemb, e->pemb, e->temb, e->eg, e->eb, c.layer_norm_eps, c.vocab,
      c.type_vocab, c.max_position, xf ? nullptr : w->x, w->xh, w->xl);
  const float scale = 1.0f / sqrtf((float)HD);
  // 1-D grid of (sequence, head) pairs, padded to a multiple of 8 (XCD-aware order in the
  // kernel; gridDim.x / NH = B after the padding is removed there)
  const dim3 agrid((unsigned)((NH * B + 7) / 8 * 8));
  const int planes = w->xl ? 2 : 1;
  const int kc = attn_chunk_keys<HD>(max_len, planes);
  const size_t alds = (size_t)attn_lds_bytes<HD>(kc, planes);
  const int nl = (int)e->layers.size();
  bool head_done = false;   // the bge head ran inside the last LayerNorm
  for (int l = 0; l < nl; ++l) {
    const Layer& L = e->layers[l];
    const bool last = l == nl - 1;                  // CLS rows only after the attention
    const Layer* P = l > 0 ? &e->layers[l - 1] : nullptr;
    // Last layer, deferred LayerNorm (fp16x3 large batches): only the [CLS] rows leave the
    // layer, so only their Q is needed. K|V for every token (the folded QKV weights' rows
    // H .. 3H-1, N = 2H), the CLS rows gathered with their pending LN2 applied, their Q by a
    // B-row GEMM, and a CLS-only attention (attn_cls_kernel) straight into the CLS context.
    // RAGMI_CLS_ATTN=0 (diagnostic A/B): the all-token QKV + attention path.
    if (last && dl && P && H == kDlH && HD == 32 && cls_attn_on()) {
      DlArgs a;
      a.st_in = w->sb;
      a.c1 = L.qkv_c1 + H;
      a.eps = c.layer_norm_eps;
      launch_ws_large<kEpiLnF16, true, 2>(w->xh, w->xl, L.wqkv_f + (int64_t)H * H,
                                    L.wqkv_fl + (int64_t)H * H, L.qkv_c2 + H, T, 2 * H, H,
                                    w->qkv, w->qkv_l, st, a);
      gather_cls_kernel<H><<<dim3(B), dim3(64), 0, st>>>(
          nullptr, w->xh, w->xl, nullptr, nullptr, cu, w->xc, nullptr, nullptr, w->sb, P->g2,
          P->be2, c.layer_norm_eps, w->xch, w->xcl);
      // Q of the CLS rows into the CLS FFN buffers (free until this layer's FFN1)
      gemm<kEpiF16>(w->xch, w->xcl, L.wqkv, L.wqkv_l, L.bqkv, B, H, H, w->ffc, w->ffcl, st);
      constexpr int kGroups = (H / HD) / kAttnClsHeads;
      launch_fixed<kAttnClsBlock>(attn_cls_kernel<H, HD>, dim3((unsigned)(B * kGroups)), 0, st,
                                  w->qkv, w->qkv_l, w->ffc, w->ffcl, cu, B, max_len, scale,
                                  w->cc, w->ccl);
    } else if (dl && P) {
      // LN2 of layer l-1 pending on z: folded into QKV (kEpiLnF16)
      DlArgs a;
      a.st_in = w->sb;
      a.c1 = L.qkv_c1;
      a.eps = c.layer_norm_eps;
      launch_ws_large<kEpiLnF16, true, 2>(w->xh, w->xl, L.wqkv_f, L.wqkv_fl, L.qkv_c2, T,
                                    3 * H, H, w->qkv, w->qkv_l, st, a);
    } else {
      gemm<kEpiF16>(w->xh, w->xl, L.wqkv, L.wqkv_l, L.bqkv, T, 3 * H, H, w->qkv, w->qkv_l, st);
    }
    const bool cls_done = last && dl && P && H == kDlH && HD == 32 && cls_attn_on();
    const int max_qb = last ? 1 : 1 << 20;
    if (cls_done) {
      // (the CLS context is in w->cc / w->ccl already)
    } else if (w->xl && attn_short(HD, max_len))
      launch_fixed<128>(attn_kernel<H, HD, true, kAttnVar, 128>, agrid, alds, st,
          w->qkv, w->qkv_l, cu, max_len, kc, scale, w->ctx, w->ctx_l, max_qb);
    else if (w->xl)
      launch_fixed<kAttnThreads<true>>(attn_kernel<H, HD, true>, agrid, alds, st,
          w->qkv, w->qkv_l, cu, max_len, kc, scale, w->ctx, w->ctx_l, max_qb);
    else if (attn_short(HD, max_len))
      launch_fixed<128>(attn_kernel<H, HD, false, kAttnVar, 128>, agrid, alds, st,
          w->qkv, nullptr, cu, max_len, kc, scale, w->ctx, nullptr, max_qb);
    else
      launch_fixed<kAttnThreads<false>>(attn_kernel<H, HD, false>, agrid, alds, st,
          w->qkv, nullptr, cu, max_len, kc, scale, w->ctx, nullptr, max_qb);
    if (dl && !last) {
      // z1 = LN2_{l-1}(z) + O-proj (stats -> sa); FFN1 with LN1 folded; z2 = LN1(z1) + FFN2
      // (stats -> sb); z lives in xh + xl throughout (updated in place)
      DlArgs o;
      o.st_in = P ? w->sb : nullptr;
      o.gamma = P ? P->g2 : nullptr;
      o.beta = P ? P->be2 : nullptr;
      o.st_out = w->sa;
      o.eps = c.layer_norm_eps;
      launch_ws_large<kEpiResLn, true>(w->ctx, w->ctx_l, L.wo, L.wo_l, L.bo, T, H, H, w->xh,
                                 w->xl, st, o);
#ifdef RAGMI_DIAG_BUILD
      if (ffn_fused_for(e, T, FF)) {
        // FFN1 + GELU + FFN2 + residual + LN statistics in one launch, H kept on the CU
        FfnArgs fa;
        fa.w1 = L.w1_f;
        fa.w1l = L.w1_fl;
        fa.c1 = L.w1_c1;
        fa.c2 = L.w1_c2;
        fa.w2 = L.w2;
        fa.w2l = L.w2_l;
        fa.b2 = L.bi2;
        fa.gamma = L.g1;
        fa.beta = L.be1;
        fa.st_in = w->sa;
        fa.st_out = w->sb;
        fa.eps = c.layer_norm_eps;
        launch_ffn_fused(w->xh, w->xl, T, fa, st, ffn_ring(e));
        continue;
      }
#endif
      DlArgs f;
      f.st_in = w->sa;
      f.c1 = L.w1_c1;
      f.eps = c.layer_norm_eps;
      launch_ws_large<kEpiLnGeluF16, true, 2>(w->xh, w->xl, L.w1_f, L.w1_fl, L.w1_c2, T, FF,
                                        H, w->ff, w->ff_l, st, f);
      DlArgs r;
      r.st_in = w->sa;
      r.gamma = L.g1;
      r.beta = L.be1;
      r.st_out = w->sb;
      r.eps = c.layer_norm_eps;
      launch_ws_large<kEpiResLn, true>(w->ff, w->ff_l, L.w2, L.w2_l, L.bi2, T, H, FF, w->xh,
                                 w->xl, st, r);
      continue;
    }
    // rows the rest of the layer runs on: all T tokens, or the B gathered CLS rows
    int R = T;
    float *x = xf ? nullptr : w->x, *y = w->y;
    int64_t y_rows = w->y_rows;
    _Float16 *xh = w->xh, *xl = w->xl, *ctx = w->ctx, *ctxl = w->ctx_l, *ff = w->ff,
             *ffl = w->ff_l;
    bool row_xf = xf;
    if (last) {
      // (deferred LayerNorm: x_cls = LN2_{l-1}(z) of the CLS rows; the CLS-only path
      // gathered them before its attention)
      const bool dlp = dl && P;
      if (!cls_done)
        gather_cls_kernel<H><<<dim3(B), dim3(64), 0, st>>>(
            x, w->xh, w->xl, w->ctx, w->ctx_l, cu, w->xc, w->cc, w->xl ? w->ccl : nullptr,
            dlp ? w->sb : nullptr, dlp ? P->g2 : nullptr, dlp ? P->be2 : nullptr,
            c.layer_norm_eps);
      row_xf = false;                                 // the B CLS rows keep an fp32 copy
      R = B;
      x = w->xc;
      y = w->yc;
      y_rows = w->yc_rows;
      xh = w->xch;
      xl = w->xl ? w->xcl : nullptr;
      ctx = w->cc;
      ctxl = w->xl ? w->ccl : nullptr;
      ff = w->ffc;
      ffl = w->xl ? w->ffcl : nullptr;
    }
    const unsigned lg = (unsigned)((R + 3) / 4);
    const bool fuse = !row_xf && fuse_for(R);
    // split-K parts y can hold for R rows (the small-batch GEMMs' K split, summed by add_ln)
    const int ks_room = (int)std::max<int64_t>(1, std::min<int64_t>(kMaxKSplit, y_rows / R));
    // bge head fused into the last residual + LayerNorm (add_ln384_kernel<false, true>: one
    // dispatch fewer per forward; cls_normalize_kernel's arithmetic)
    const bool l2_fused = H == 384 && last && !row_xf && c.head == RAG_HEAD_CLS_L2;
    auto add_ln = [&](const float* gam, const float* bet, int parts, bool final_ln = false) {
      const int64_t ps = (int64_t)R * H;
      if constexpr (H == 384) {
        // 16-B accesses and DPP / permlane reductions (round 3)
        if (final_ln && l2_fused) {
          add_ln384_kernel<false, true><<<dim3(lg), dim3(256), 0, st>>>(
              x, y, gam, bet, c.layer_norm_eps, xh, xl, R, parts, ps, out);
          return;
        }
        if (row_xf)
          add_ln384_kernel<true><<<dim3(lg), dim3(256), 0, st>>>(nullptr, y, gam, bet,
                                                                c.layer_norm_eps, xh, xl, R,
                                                                parts, ps);
        else
          add_ln384_kernel<false><<<dim3(lg), dim3(256), 0, st>>>(x, y, gam, bet,
                                                                 c.layer_norm_eps, xh, xl, R,
                                                                 parts, ps);
        return;
      }
      if (row_xf)
        add_ln_kernel<H, true><<<dim3(lg), dim3(256), 0, st>>>(nullptr, y, gam, bet,
                                                              c.layer_norm_eps, xh, xl, R,
                                                              parts, ps);
      else
        add_ln_kernel<H><<<dim3(lg), dim3(256), 0, st>>>(x, y, gam, bet, c.layer_norm_eps, xh,
                                                        xl, R, parts, ps);
    };
    if (fuse) {
      gemm_add_ln(ctx, ctxl, L.wo, L.wo_l, L.bo, L.g1, L.be1, c.layer_norm_eps, R, H, H, x, xh,
                  xl, st);
    } else {
      int ks = ks_room;
      gemm<kEpiF32>(ctx, ctxl, L.wo, L.wo_l, L.bo, R, H, H, y, nullptr, st, RAG_GEMM_AUTO, &ks);
      add_ln(L.g1, L.be1, ks);
    }
    gemm<kEpiGeluF16>(xh, xl, L.w1, L.w1_l, L.bi1, R, FF, H, ff, ffl, st);
    if (fuse) {
      gemm_add_ln(ff, ffl, L.w2, L.w2_l, L.bi2, L.g2, L.be2, c.layer_norm_eps, R, H, FF, x, xh,
                  xl, st);
      head_done = false;
    } else {
      int ks = ks_room;
      gemm<kEpiF32>(ff, ffl, L.w2, L.w2_l, L.bi2, R, H, FF, y, nullptr, st, RAG_GEMM_AUTO, &ks);
      add_ln(L.g2, L.be2, ks, true);
      head_done = l2_fused;
    }
  }
  // the final hidden states of the CLS tokens are rows 0 .. B-1 of w->xc (cu = null)
  if (c.head == RAG_HEAD_CLS_L2) {
    if (!head_done) cls_normalize_kernel<H><<<dim3(B), dim3(64), 0, st>>>(w->xc, nullptr, out);
  } else {
    ce_head_kernel<H><<<dim3(B), dim3(256), 0, st>>>(w->xc, nullptr, e->wp, e->bp, e->wc, e->bc,
                                                     out);
  }
  RAG_HIP(hipGetLastError());
  return RAG_OK;
}

// padded copy of a call's inputs into the graph's staging: ids / types past T are token 0 /
// type 0 (the pad rows [T, Tp) belong to no sequence: cu ends at T, so attention, the CLS
// gather and every row-wise kernel leave the real rows' values as without them)
__global__ void graph_stage_kernel(const int32_t* __restrict__ ids,
                                   const int32_t* __restrict__ types,
                                   const int32_t* __restrict__ cu, int B, int T, int Tp,
                                   int32_t* __restrict__ g) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < Tp) {
    g[i] = i < T ? ids[i] : 0;
    g[Tp + i] = i < T ? types[i] : 0;
  }
  if (i <= B) g[2 * Tp + i] = cu[i];
}

// Small-batch forward by graph replay: stage the inputs (one kernel), replay the graph captured
// for the padded shape (T up to a multiple of 64, max_len up to a multiple of 32 — the
// attention's key chunking depends on max_len only through that rounding, attn_chunk_keys),
// copy the B output rows out. The graph is captured on first use of its shape from the same
// eager code path (forward_t), so it launches the same kernels with the same arguments. The
// capture runs on the workspace's private capture stream (nothing executes during a capture;
// the caller's stream stays free for other threads, whose launches would otherwise be
// recorded into the graph), and a shape whose capture or instantiation fails runs eagerly on
// the caller's stream instead of failing the call.
template <int H, int HD>
int forward_graph(rag_encoder* e, EncWorkspace* w, const int32_t* ids, const int32_t* types,
                  const int32_t* cu, int B, int T, int max_len, float* out, hipStream_t st) {
  const rag_bert_config& c = e->cfg;
  const int Tp = (T + 63) / 64 * 64;
  const int Lp = std::min((max_len + 31) / 32 * 32, c.max_position);
  const int od = c.head == RAG_HEAD_CLS_L2 ? H : 1;
  int rc = ensure_ws(c, w, Tp);
  if (rc) return rc;
  rc = ensure_cls(c, w, B);
  if (rc) return rc;
  if (w->g_in_cap < 2 * (int64_t)Tp + B + 1 || w->g_out_cap < (int64_t)B * od) {
    w->drop_graphs();
    if (w->g_in) (void)hipFree(w->g_in);
    if (w->g_out) (void)hipFree(w->g_out);
    w->g_in = nullptr;
    w->g_out = nullptr;
    w->g_in_cap = w->g_out_cap = 0;
    const int64_t ni = std::max<int64_t>(2 * (int64_t)Tp + B + 1, 2 * 4096 + 257);
    const int64_t no = std::max<int64_t>((int64_t)B * od, 256 * (int64_t)od);
    RAG_HIP(hipMalloc(reinterpret_cast<void**>(&w->g_in), ni * 4));
    RAG_HIP(hipMalloc(reinterpret_cast<void**>(&w->g_out), no * 4));
    w->g_in_cap = ni;
    w->g_out_cap = no;
  }
  int32_t* g = w->g_in;
  graph_stage_kernel<<<dim3((unsigned)((std::max(Tp, B + 1) + 255) / 256)), dim3(256), 0, st>>>(
      ids, types, cu, B, T, Tp, g);
  RAG_HIP(hipGetLastError());
  EncWorkspace::Graph* hit = nullptr;
  for (auto& gr : w->graphs)
    if (gr.B == B && gr.T == Tp && gr.L == Lp) hit = &gr;
  if (!hit) {
    if ((int)w->graphs.size() >= kGraphCache) {
      auto lru = std::min_element(w->graphs.begin(), w->graphs.end(),
                                  [](const EncWorkspace::Graph& a, const EncWorkspace::Graph& b) {
                                    return a.last < b.last;
                                  });
      RAG_HIP(hipStreamSynchronize(st));      // its last replay was on this stream
      if (lru->exec) (void)hipGraphExecDestroy(lru->exec);
      w->graphs.erase(lru);
    }
    if (!w->cstream) RAG_HIP(hipStreamCreateWithFlags(&w->cstream, hipStreamNonBlocking));
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
    bool ok = hipStreamBeginCapture(w->cstream, hipStreamCaptureModeRelaxed) == hipSuccess;
    if (ok) {
      // (recorded on the private stream, but into THIS workspace's buffers)
      rc = forward_t<H, HD>(e, g, g + Tp, g + 2 * Tp, B, Tp, Lp, w->g_out, w->cstream, true, w);
      ok = hipStreamEndCapture(w->cstream, &graph) == hipSuccess && rc == RAG_OK && graph;
      ok = ok && hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0) == hipSuccess;
      if (graph) (void)hipGraphDestroy(graph);
    }
    if (!ok) {
      // a failed capture can leave its stream unusable: drop it (a new one next time). The
      // shape is remembered as eager (exec = null), so it is not captured again on every call,
      // and the first failure of the process is reported once on stderr.
      const hipError_t err = hipGetLastError();
      static std::atomic<bool> said{false};
      if (!said.exchange(true))
        std::fprintf(stderr, "ragmi: encoder graph capture failed (%s%s%s); shape B=%d T=%d "
                     "runs eagerly\n", hipGetErrorString(err), rc ? ": " : "",
                     rc ? rag_last_error() : "", B, Tp);
      (void)hipStreamDestroy(w->cstream);
      w->cstream = nullptr;
      ragmi::clear_error();
      w->graphs.push_back(EncWorkspace::Graph{B, Tp, Lp, nullptr, e->uses});
      return forward_t<H, HD>(e, ids, types, cu, B, T, max_len, out, st, true, w);
    }
    w->graphs.push_back(EncWorkspace::Graph{B, Tp, Lp, exec, 0});
    hit = &w->graphs.back();
  }
  hit->last = e->uses;
  if (!hit->exec)     // a shape whose capture failed: eager on the caller's stream
    return forward_t<H, HD>(e, ids, types, cu, B, T, max_len, out, st, true, w);
  RAG_HIP(hipGraphLaunch(hit->exec, st));
  RAG_HIP(hipMemcpyAsync(out, w->g_out, (size_t)B * od * 4, hipMemcpyDeviceToDevice, st));
  return RAG_OK;
}

// fp16 range guard. Every activation the forward stores as an fp16 plane is bounded, for ANY
// input, by the weights alone (interval arithmetic, modeling_bert.py's layer, restated):
//   LayerNorm output  |y_i| <= |gamma_i| sqrt(H - 1) + |beta_i|   (a standardised entry of H
//                     values is at most sqrt(H - 1) in magnitude; eps only shrinks it)
//   Linear output     |(W x + b)_j| <= sum_i |W_ji| bound(x_i) + |b_j|
//   attention context a convex combination of V rows: <= bound(V) per dimension
//   erf-GELU          |gelu(y)| <= max(|y|, 0.17)
// The plain forward stores LN outputs (xh/xl), Q|K|V, the attention context and the FFN
// intermediate in fp16 planes; the O-proj / FFN2 outputs and every pre-LN residual sum stay
// fp32. The deferred-LayerNorm forward (DlArgs) stores the pre-LN sums z = x + sublayer
// output as planes too. fp16 overflows above 65504; kF16Safe leaves margin for the fp32
// rounding of the bounded quantities themselves. So:
//   bound_plain > kF16Safe -> rag_encoder_create refuses the weights (RAG_ERANGE);
//   bound_defer > kF16Safe -> the deferred LayerNorm is never used (auto skips it, forcing it
//                             on fails).
// Real BERT checkpoints are far inside: the stress profile of ragmi.synth (outlier
// dimensions with gammas up to 20, |hidden| ~ 100-400) gives 790 / 15.6K.
void range_bounds(const rag_bert_config& c, const float* const* w, double* plain,
                  double* defer) {
  const int H = c.hidden, FF = c.intermediate;
  const double s = std::sqrt((double)(H - 1));
  auto ln = [&](const float* g, const float* b, std::vector<double>& out) {
    out.resize(H);
    for (int i = 0; i < H; ++i) out[i] = std::fabs((double)g[i]) * s + std::fabs((double)b[i]);
  };
  auto lin = [&](const float* W, const float* b, int N, int K, const std::vector<double>& x,
                 std::vector<double>& out) {
    out.resize(N);
    for (int n = 0; n < N; ++n) {
      double a = std::fabs((double)b[n]);
      const float* r = W + (size_t)n * K;
      for (int k = 0; k < K; ++k) a += std::fabs((double)r[k]) * x[k];
      out[n] = a;
    }
  };
  auto mx = [](const std::vector<double>& v) {
    double m = 0.0;
    for (double x : v) m = std::max(m, x);
    return m;
  };
  std::vector<double> g, q, k, v, a, g1, f, o, g2;
  ln(w[3], w[4], g);
  double bp = mx(g), bd = 0.0;
  for (int l = 0; l < c.layers; ++l) {
    const float* const* p = w + 5 + 16 * l;
    lin(p[0], p[1], H, H, g, q);
    lin(p[2], p[3], H, H, g, k);
    lin(p[4], p[5], H, H, g, v);                       // context <= V per dimension
    lin(p[6], p[7], H, H, v, a);                       // O-proj (fp32)
    for (int i = 0; i < H; ++i) bd = std::max(bd, g[i] + a[i]);          // z1
    ln(p[8], p[9], g1);
    lin(p[10], p[11], FF, H, g1, f);
    for (double& x : f) x = std::max(x, 0.17);         // erf-GELU
    lin(p[12], p[13], H, FF, f, o);                    // FFN2 (fp32)
    for (int i = 0; i < H; ++i) bd = std::max(bd, g1[i] + o[i]);         // z2
    ln(p[14], p[15], g2);
    bp = std::max({bp, mx(q), mx(k), mx(v), mx(g1), mx(f), mx(g2)});
    g.swap(g2);
  }
  *plain = bp;
  *defer = std::max(bp, bd);
}

// Built (hidden, head_dim) shapes: 384/32 (bge-small, MiniLM-L6), 768/64 (bge-base),
// 1024/64 (bge-large, SURVEY config 5).
bool shape_supported(int hidden, int heads) {
  return (hidden == 384 && heads == 12) || (hidden == 768 && heads == 12) ||
         (hidden == 1024 && heads == 16);
}

template <int H, int HD>
int set_attn_lds_attr() {
  RAG_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&attn_kernel<H, HD, true>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, kAttnLdsMax));
  RAG_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&attn_kernel<H, HD, false>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, kAttnLdsMax));
  RAG_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&attn_kernel<H, HD, true, kAttnVar, 128>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, kAttnLdsMax));
  RAG_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&attn_kernel<H, HD, false, kAttnVar, 128>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, kAttnLdsMax));
  return RAG_OK;
}

int forward_locked(rag_encoder* e, const int32_t* ids, const int32_t* types, const int32_t* cu,
                   int B, int T, int max_len, float* out, hipStream_t st) {
  switch (e->cfg.hidden) {
    case 384: return forward_t<384, 32>(e, ids, types, cu, B, T, max_len, out, st);
    case 768: return forward_t<768, 64>(e, ids, types, cu, B, T, max_len, out, st);
    default: return forward_t<1024, 64>(e, ids, types, cu, B, T, max_len, out, st);
  }
}

}  // namespace

extern "C" {

int rag_encoder_num_weights(const rag_bert_config* cfg) {
  if (!cfg) return -1;
  return 5 + 16 * cfg->layers + (cfg->head == RAG_HEAD_POOLER_CLS ? 4 : 0);
}

int rag_encoder_create_ex(const rag_bert_config* cfg, const float* const* w, int n_weights,
                          int device, int flags, rag_encoder_t** out) {
  ragmi::clear_error();
  if (flags & ~RAG_CREATE_DIAGNOSTIC) return ragmi::fail(RAG_EINVAL, "unknown encoder flags");
  const int rc = rag_encoder_create(cfg, w, n_weights, device, out);
  if (rc == RAG_OK && (flags & RAG_CREATE_DIAGNOSTIC)) {
    (*out)->diagnostic = true;
    ragmi::diagnostic_acquire();
    // knobs read at create time (the LayerNorm modes) see the handle as diagnostic
    (*out)->fuse_ln = fuse_ln_default();
    (*out)->defer_ln = defer_ln_default();
  }
  return rc;
}

int rag_encoder_create(const rag_bert_config* cfg, const float* const* w, int n_weights,
                       int device, rag_encoder_t** out) {
  ragmi::clear_error();
  if (!cfg || !w || !out) return ragmi::fail(RAG_EINVAL, "NULL argument");
  *out = nullptr;
  if (!shape_supported(cfg->hidden, cfg->heads) || cfg->intermediate < 128 ||
      cfg->intermediate % 128 != 0)
    return ragmi::fail(RAG_EINVAL,
                       "built for hidden/heads 384/12, 768/12, 1024/16 and intermediate a "
                       "multiple of 128");
  if (cfg->layers < 1 || cfg->layers > 64 || cfg->vocab < 1 || cfg->type_vocab < 1 ||
      cfg->max_position < 1 || cfg->max_position > 4096)
    return ragmi::fail(RAG_EINVAL, "bad config");
  if (cfg->head != RAG_HEAD_CLS_L2 && cfg->head != RAG_HEAD_POOLER_CLS)
    return ragmi::fail(RAG_EINVAL, "unknown head");
  if (cfg->precision != RAG_PREC_FP16 && cfg->precision != RAG_PREC_FP16X3)
    return ragmi::fail(RAG_EINVAL, "unknown precision");
  if (n_weights != rag_encoder_num_weights(cfg))
    return ragmi::fail(RAG_EINVAL, "wrong number of weight tensors");
  for (int i = 0; i < n_weights; ++i)
    if (!w[i]) return ragmi::fail(RAG_EINVAL, "NULL weight tensor");
  double b_plain = 0.0, b_defer = 0.0;
  range_bounds(*cfg, w, &b_plain, &b_defer);
  if (!(b_plain <= kF16Safe))
    return ragmi::fail(RAG_ERANGE,
                       "weights can drive an fp16 activation plane past 65504 (static bound " +
                           std::to_string(b_plain) +
                           "; see rag_encoder_range_bounds): refusing rather than returning inf");
  RAG_HIP(hipSetDevice(device));
  // attention stages K/V in dynamic LDS (up to 160 KB)
  {
    const int arc = cfg->hidden == 384    ? set_attn_lds_attr<384, 32>()
                    : cfg->hidden == 768 ? set_attn_lds_attr<768, 64>()
                                         : set_attn_lds_attr<1024, 64>();
    if (arc) return arc;
  }
  auto* e = new rag_encoder();
  e->cfg = *cfg;
  e->device = device;
  e->fuse_ln = fuse_ln_default();
  e->defer_ln = defer_ln_default();
  e->bound_plain = b_plain;
  e->bound_defer = b_defer;
  int rc = RAG_OK;
  auto chk = [&](int r) {
    if (r && !rc) rc = r;
  };
  const size_t Hs = cfg->hidden, H = cfg->hidden, FF = cfg->intermediate;
  chk(up_f32(e, &e->wemb, w[0], (size_t)cfg->vocab * Hs));
  chk(up_f32(e, &e->pemb, w[1], (size_t)cfg->max_position * Hs));
  chk(up_f32(e, &e->temb, w[2], (size_t)cfg->type_vocab * Hs));
  chk(up_f32(e, &e->eg, w[3], Hs));
  chk(up_f32(e, &e->eb, w[4], Hs));
  e->layers.resize(cfg->layers);
  for (int l = 0; l < cfg->layers && !rc; ++l) {
    const float* const* p = w + 5 + 16 * l;
    Layer& L = e->layers[l];
    const bool sp = cfg->precision == RAG_PREC_FP16X3;
    chk(up_f16(e, &L.wqkv, sp ? &L.wqkv_l : nullptr,
               {{p[0], Hs * H}, {p[2], Hs * H}, {p[4], Hs * H}}));
    {
      std::vector<float> b(3 * H);
      std::copy(p[1], p[1] + H, b.begin());
      std::copy(p[3], p[3] + H, b.begin() + H);
      std::copy(p[5], p[5] + H, b.begin() + 2 * H);
      chk(up_f32(e, &L.bqkv, b.data(), 3 * Hs));
    }
    chk(up_f16(e, &L.wo, sp ? &L.wo_l : nullptr, {{p[6], Hs * H}}));
    chk(up_f32(e, &L.bo, p[7], Hs));
    chk(up_f32(e, &L.g1, p[8], Hs));
    chk(up_f32(e, &L.be1, p[9], Hs));
    chk(up_f16(e, &L.w1, sp ? &L.w1_l : nullptr, {{p[10], (size_t)FF * H}}));
    chk(up_f32(e, &L.bi1, p[11], FF));
    chk(up_f16(e, &L.w2, sp ? &L.w2_l : nullptr, {{p[12], Hs * FF}}));
    chk(up_f32(e, &L.bi2, p[13], Hs));
    chk(up_f32(e, &L.g2, p[14], Hs));
    chk(up_f32(e, &L.be2, p[15], Hs));
    if (sp && H == kDlH && 2 * FF <= kPipeBiasMax && !rc) {
      if (l > 0) {
        const float* const* pp = p - 16;               // the previous layer's output LN
        chk(fold_ln(e, {{p[0], p[1]}, {p[2], p[3]}, {p[4], p[5]}}, H, H, pp[14], pp[15],
                    &L.wqkv_f, &L.wqkv_fl, &L.qkv_c1, &L.qkv_c2));
      }
      chk(fold_ln(e, {{p[10], p[11]}}, FF, H, p[8], p[9], &L.w1_f, &L.w1_fl, &L.w1_c1,
                  &L.w1_c2));
    }
  }
  if (cfg->head == RAG_HEAD_POOLER_CLS && !rc) {
    const float* const* p = w + 5 + 16 * cfg->layers;
    chk(up_f32(e, &e->wp, p[0], Hs * H));
    chk(up_f32(e, &e->bp, p[1], Hs));
    chk(up_f32(e, &e->wc, p[2], Hs));
    chk(up_f32(e, &e->bc, p[3], 1));
  }
  if (rc) {
    rag_encoder_destroy(e);
    return rc;
  }
  *out = e;
  return RAG_OK;
}

int rag_encoder_destroy(rag_encoder_t* e) {
  ragmi::clear_error();
  if (!e) return RAG_OK;
  if (e->diagnostic) ragmi::diagnostic_release();
  (void)hipSetDevice(e->device);
  (void)hipDeviceSynchronize();
  for (void* p : e->allocs) (void)hipFree(p);
  for (auto& w : e->ws) w.release();
  if (e->stage) (void)hipFree(e->stage);
  if (e->gev_in) (void)hipEventDestroy(e->gev_in);
  if (e->gev_out) (void)hipEventDestroy(e->gev_out);
  if (e->gstream) (void)hipStreamDestroy(e->gstream);
  delete e;
  return RAG_OK;
}

int rag_encoder_forward(rag_encoder_t* e, const int32_t* ids, const int32_t* types,
                        const int32_t* cu, int B, int T, int max_len, float* out, void* stream) {
  ragmi::clear_error();
  if (!e || !ids || !types || !cu || !out) return ragmi::fail(RAG_EINVAL, "NULL argument");
  if (B < 1 || T < B || max_len < 1 || max_len > e->cfg.max_position)
    return ragmi::fail(RAG_EINVAL, "bad batch shape (max_len must be <= max_position)");
  std::lock_guard<std::mutex> lk(e->mu);
  RAG_HIP(hipSetDevice(e->device));
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (st == nullptr && use_graphs(e, st, T, true)) {
    // null stream (graphs cannot be captured on it): replay on the encoder's own stream,
    // after everything queued on the null stream so far and before anything queued after
    if (!e->gstream) {
      RAG_HIP(hipStreamCreateWithFlags(&e->gstream, hipStreamNonBlocking));
      RAG_HIP(hipEventCreateWithFlags(&e->gev_in, hipEventDisableTiming));
      RAG_HIP(hipEventCreateWithFlags(&e->gev_out, hipEventDisableTiming));
    }
    RAG_HIP(hipEventRecord(e->gev_in, nullptr));
    RAG_HIP(hipStreamWaitEvent(e->gstream, e->gev_in, 0));
    const int rc = forward_locked(e, ids, types, cu, B, T, max_len, out, e->gstream);
    RAG_HIP(hipEventRecord(e->gev_out, e->gstream));
    RAG_HIP(hipStreamWaitEvent(nullptr, e->gev_out, 0));
    return rc;
  }
  return forward_locked(e, ids, types, cu, B, T, max_len, out, st);
}

int rag_bert_gemm(int variant, int epilogue, const void* A, const void* A_lo, const void* W,
                  const void* W_lo, const float* bias, int M, int N, int K, void* C,
                  void* C_lo, void* stream) {
  ragmi::clear_error();
  if (!A || !W || !bias || !C) return ragmi::fail(RAG_EINVAL, "NULL argument");
  if (M < 1 || N < BN || K < 64 || N % BN != 0 || K % 64 != 0)
    return ragmi::fail(RAG_EINVAL, "M >= 1, N and K multiples of 128 / 64 required");
  if ((A_lo == nullptr) != (W_lo == nullptr))
    return ragmi::fail(RAG_EINVAL, "A_lo and W_lo: both (fp16x3) or neither (fp16)");
  if (A_lo && epilogue != kEpiF32 && !C_lo)
    return ragmi::fail(RAG_EINVAL, "fp16x3 fp16-output GEMM needs C_lo");
  const bool known = variant == RAG_GEMM_AUTO || variant == RAG_GEMM_TILE ||
                     variant == RAG_GEMM_SMALL || variant == RAG_GEMM_WS ||
                     variant == RAG_GEMM_WS_MFMA_ONLY || variant == RAG_GEMM_WS_NO_STORE ||
                     variant == RAG_GEMM_WS_DMA_ONLY;
  if (!known) return ragmi::fail(RAG_EINVAL, "unknown GEMM variant");
  if ((variant == RAG_GEMM_SMALL || variant >= RAG_GEMM_WS) && !pipe_ok(M, N, K))
    return ragmi::fail(RAG_EINVAL, "SMALL / WS variants need N % 128 == 0, K % 64 == 0, "
                                   "N <= 4096, M*K*2 and M*N*4 < 2^31");
  auto* a = static_cast<const _Float16*>(A);
  auto* al = static_cast<const _Float16*>(A_lo);
  auto* w = static_cast<const _Float16*>(W);
  auto* wl = static_cast<const _Float16*>(W_lo);
  auto* clo = static_cast<_Float16*>(C_lo);
  auto st = static_cast<hipStream_t>(stream);
  switch (epilogue) {
    case kEpiF16: gemm<kEpiF16>(a, al, w, wl, bias, M, N, K, C, clo, st, variant); break;
    case kEpiGeluF16: gemm<kEpiGeluF16>(a, al, w, wl, bias, M, N, K, C, clo, st, variant); break;
    case kEpiF32: gemm<kEpiF32>(a, al, w, wl, bias, M, N, K, C, clo, st, variant); break;
    default: return ragmi::fail(RAG_EINVAL, "unknown epilogue");
  }
  RAG_HIP(hipGetLastError());
  return RAG_OK;
}

int rag_bert_gemm_splitk(int variant, const void* A, const void* A_lo, const void* W,
                         const void* W_lo, const float* bias, int M, int N, int K, float* C,
                         int max_parts, int* parts, void* stream) {
  ragmi::clear_error();
  if (!A || !W || !bias || !C || !parts) return ragmi::fail(RAG_EINVAL, "NULL argument");
  if ((A_lo == nullptr) != (W_lo == nullptr))
    return ragmi::fail(RAG_EINVAL, "A_lo and W_lo: both (fp16x3) or neither (fp16)");
  if (variant != RAG_GEMM_AUTO && variant != RAG_GEMM_SMALL)
    return ragmi::fail(RAG_EINVAL, "split-K runs on the SMALL GEMMs (AUTO, SMALL)");
  if (M < 1 || max_parts < 1 || N % BN != 0 || K % 64 != 0 || !pipe_ok(M, N, K))
    return ragmi::fail(RAG_EINVAL, "bad shape");
  int ks = std::min(max_parts, kMaxKSplit);
  gemm<kEpiF32>(static_cast<const _Float16*>(A), static_cast<const _Float16*>(A_lo),
                static_cast<const _Float16*>(W), static_cast<const _Float16*>(W_lo), bias, M, N,
                K, C, nullptr, static_cast<hipStream_t>(stream), variant, &ks);
  *parts = ks;
  RAG_HIP(hipGetLastError());
  return RAG_OK;
}

int rag_bert_gemm_add_ln(const void* A, const void* A_lo, const void* W, const void* W_lo,
                         const float* bias, const float* gamma, const float* beta, float eps,
                         int M, int N, int K, float* x, void* xh, void* xl, void* stream) {
  ragmi::clear_error();
  if (!A || !W || !bias || !gamma || !beta || !x || !xh)
    return ragmi::fail(RAG_EINVAL, "NULL argument");
  if ((A_lo == nullptr) != (W_lo == nullptr) || (A_lo != nullptr) != (xl != nullptr))
    return ragmi::fail(RAG_EINVAL, "A_lo, W_lo and xl: all three (fp16x3) or none (fp16)");
  if (M < 1 || !add_ln_ok(M, N, K))
    return ragmi::fail(RAG_EINVAL, "N == 384, K % 64 == 0, M*K*2 and M*N*4 < 2^31 required");
  gemm_add_ln(static_cast<const _Float16*>(A), static_cast<const _Float16*>(A_lo),
              static_cast<const _Float16*>(W), static_cast<const _Float16*>(W_lo), bias, gamma,
              beta, eps, M, N, K, x, static_cast<_Float16*>(xh), static_cast<_Float16*>(xl),
              static_cast<hipStream_t>(stream));
  RAG_HIP(hipGetLastError());
  return RAG_OK;
}

// attention alone (bge-small / MiniLM shape: hidden 384, head_dim 32), variant = the
// attn_kernel VAR bit mask (0..7; kAttnVar is the forward's): for A/B timing and tests
int rag_bert_attention(int variant, const void* qkv, const void* qkv_lo, const int32_t* cu,
                       int B, int max_len, void* ctx, void* ctx_lo, void* stream) {
  ragmi::clear_error();
  if (!qkv || !cu || !ctx || B < 1 || max_len < 1 || max_len > 512)
    return ragmi::fail(RAG_EINVAL, "qkv, cu, ctx required; 1 <= B, 1 <= max_len <= 512");
  if ((qkv_lo == nullptr) != (ctx_lo == nullptr))
    return ragmi::fail(RAG_EINVAL, "qkv_lo and ctx_lo: both (fp16x3) or neither (fp16)");
  if (variant == -1) variant = kAttnVar;
#ifdef RAGMI_DIAG_BUILD
  if ((variant < 0 || variant > 15) && variant != 18 && variant != 26 &&
      (variant < 40 || variant > 46 || variant % 2) && variant != 43 && variant != 106 &&
      variant != 107 && variant != 170 && variant != 298 && variant != 554 &&
      variant != 1066 && variant != 2090)
    return ragmi::fail(RAG_EINVAL,
                       "variant: -1, 0..15, 18, 26, 40, 42, 43, 44, 46, 106, 107, 170, 298, 554, 1066 or 2090");
#else
  // the production library carries the forward's variant and one A/B slot (round 6, VERDICT
  // r5 item 6); the measured family lives in the diagnostic build (-DRAGMI_DIAG_BUILD)
  if (variant != kAttnVar && variant != kAttnVarAB)
    return ragmi::fail(RAG_EINVAL, "variant: -1, 42 (the forward's) or 10 (A/B slot); the "
                                   "other VAR masks are in the diagnostic build only");
#endif
  constexpr int H = 384, HD = 32, NH = H / HD;
  const int planes = qkv_lo ? 2 : 1;
  const int kc = attn_chunk_keys<HD>(max_len, planes);
  const size_t alds = (size_t)attn_lds_bytes<HD>(kc, planes);
  const dim3 agrid((unsigned)((NH * B + 7) / 8 * 8));
  const float scale = 1.0f / sqrtf((float)HD);
  auto st = static_cast<hipStream_t>(stream);
  auto q = static_cast<const _Float16*>(qkv);
  auto ql = static_cast<const _Float16*>(qkv_lo);
  auto c = static_cast<_Float16*>(ctx);
  auto cl = static_cast<_Float16*>(ctx_lo);
  auto go = [&](auto vc) -> int {
    constexpr int V = decltype(vc)::value;
    if (qkv_lo) {
      RAG_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&attn_kernel<H, HD, true, V>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, kAttnLdsMax));
      launch_fixed<kAttnThreads<true>>(attn_kernel<H, HD, true, V>, agrid, alds, st,
          q, ql, cu, max_len, kc, scale, c, cl, 1 << 20);
    } else {
      RAG_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&attn_kernel<H, HD, false, V>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, kAttnLdsMax));
      launch_fixed<kAttnThreads<false>>(attn_kernel<H, HD, false, V>, agrid, alds, st,
          q, nullptr, cu, max_len, kc, scale, c, nullptr, 1 << 20);
    }
    RAG_HIP(hipGetLastError());
    return RAG_OK;
  };
#ifndef RAGMI_DIAG_BUILD
  if (variant == kAttnVarAB) return go(std::integral_constant<int, kAttnVarAB>{});
  return go(std::integral_constant<int, kAttnVar>{});
#else
  switch (variant) {
    case 0: return go(std::integral_constant<int, 0>{});
    case 1: return go(std::integral_constant<int, 1>{});
    case 2: return go(std::integral_constant<int, 2>{});
    case 3: return go(std::integral_constant<int, 3>{});
    case 4: return go(std::integral_constant<int, 4>{});
    case 5: return go(std::integral_constant<int, 5>{});
    case 6: return go(std::integral_constant<int, 6>{});
    case 7: return go(std::integral_constant<int, 7>{});
    case 8: return go(std::integral_constant<int, 8>{});
    case 9: return go(std::integral_constant<int, 9>{});
    case 10: return go(std::integral_constant<int, 10>{});
    case 11: return go(std::integral_constant<int, 11>{});
    case 12: return go(std::integral_constant<int, 12>{});
    case 13: return go(std::integral_constant<int, 13>{});
    case 14: return go(std::integral_constant<int, 14>{});
    case 18: return go(std::integral_constant<int, 18>{});   // 16 = paired query blocks
    case 26: return go(std::integral_constant<int, 26>{});
    case 40: return go(std::integral_constant<int, 40>{});   // 32 = peeled, prefetched blocks
    case 42: return go(std::integral_constant<int, 42>{});
    case 44: return go(std::integral_constant<int, 44>{});
    case 46: return go(std::integral_constant<int, 46>{});
    case 43: return go(std::integral_constant<int, 43>{});   // + 1 = rolling Q prefetch
    case 106: return go(std::integral_constant<int, 106>{});  // + 64 = staging loads first
    case 107: return go(std::integral_constant<int, 107>{});
    case 42 + 128: return go(std::integral_constant<int, 42 + 128>{});   // probes (round 6)
    case 42 + 256: return go(std::integral_constant<int, 42 + 256>{});
    case 42 + 512: return go(std::integral_constant<int, 42 + 512>{});   // scalar P scaling
    case 42 + 1024: return go(std::integral_constant<int, 42 + 1024>{});  // Q one block ahead
    case 42 + 2048: return go(std::integral_constant<int, 42 + 2048>{});  // LDS-DMA staging
    default: return go(std::integral_constant<int, 15>{});
  }
#endif
}

int rag_encoder_set_fusion(rag_encoder_t* e, int mode) {
  ragmi::clear_error();
  if (!e || mode < -1 || mode > 1) return ragmi::fail(RAG_EINVAL, "mode: -1 auto, 0 off, 1 on");
  std::lock_guard<std::mutex> lk(e->mu);
  e->fuse_ln = mode;
  for (auto& w : e->ws) w.drop_graphs();   // captured with the old mode's kernels
  return RAG_OK;
}

int rag_encoder_set_graphs(rag_encoder_t* e, int mode) {
  ragmi::clear_error();
  if (!e || mode < -1 || mode > 1) return ragmi::fail(RAG_EINVAL, "mode: -1 auto, 0 off, 1 on");
  std::lock_guard<std::mutex> lk(e->mu);
  e->graphs = mode;
  return RAG_OK;
}

int rag_encoder_set_ffn_fused(rag_encoder_t* e, int mode) {
  ragmi::clear_error();
#ifdef RAGMI_DIAG_BUILD
  if (!e || mode < -1 || mode > 5)
    return ragmi::fail(RAG_EINVAL, "mode: -1 auto, 0 off, 1 on (2-5: A/B shapes)");
#else
  if (!e || mode < -1 || mode > 0)
    return ragmi::fail(RAG_EINVAL, "mode: -1 auto or 0 off; the fused FFN (measured slower) is "
                                   "in the diagnostic build only");
#endif
  std::lock_guard<std::mutex> lk(e->mu);
  e->ffn_fused = mode;
  for (auto& w : e->ws) w.drop_graphs();
  return RAG_OK;
}

int rag_encoder_set_defer_ln(rag_encoder_t* e, int mode) {
  ragmi::clear_error();
  if (!e || mode < -1 || mode > 1) return ragmi::fail(RAG_EINVAL, "mode: -1 auto, 0 off, 1 on");
  if (mode == 1 && !(e->bound_defer <= kF16Safe))
    return ragmi::fail(RAG_ERANGE, "deferred LayerNorm refused: these weights can drive its "
                                   "un-normalised residual planes past fp16 range (static "
                                   "bound " + std::to_string(e->bound_defer) + ")");
  std::lock_guard<std::mutex> lk(e->mu);
  e->defer_ln = mode;
  for (auto& w : e->ws) w.drop_graphs();
  return RAG_OK;
}

int rag_encoder_range_bounds(const rag_encoder_t* e, double* plain, double* deferred) {
  ragmi::clear_error();
  if (!e) return ragmi::fail(RAG_EINVAL, "encoder is NULL");
  if (plain) *plain = e->bound_plain;
  if (deferred) *deferred = e->bound_defer;
  return RAG_OK;
}

int rag_encoder_weight_bounds(const rag_bert_config* cfg, const float* const* weights,
                              int n_weights, double* plain, double* deferred) {
  ragmi::clear_error();
  if (!cfg || !weights || n_weights != rag_encoder_num_weights(cfg))
    return ragmi::fail(RAG_EINVAL, "bad config / weights");
  for (int i = 0; i < n_weights; ++i)
    if (!weights[i]) return ragmi::fail(RAG_EINVAL, "NULL weight tensor");
  double p = 0.0, d = 0.0;
  range_bounds(*cfg, weights, &p, &d);
  if (plain) *plain = p;
  if (deferred) *deferred = d;
  return RAG_OK;
}

int rag_bert_gemm_dl(int epilogue, const void* A, const void* A_lo, const void* W,
                     const void* W_lo, const float* bias, const float* c1, const float* st_in,
                     const float* gamma, const float* beta, float eps, int M, int N, int K,
                     void* C, void* C_lo, float* st_out, void* stream) {
  ragmi::clear_error();
  if (!A || !A_lo || !W || !W_lo || !bias || !C || !C_lo)
    return ragmi::fail(RAG_EINVAL, "NULL argument");
  if (epilogue != RAG_EPI_LN_F16 && epilogue != RAG_EPI_LN_GELU_F16 &&
      epilogue != RAG_EPI_RES_LN)
    return ragmi::fail(RAG_EINVAL, "epilogue: RAG_EPI_LN_F16, RAG_EPI_LN_GELU_F16 or RAG_EPI_RES_LN");
  if (M < 1 || !dl_gemm_ok(epilogue, M, N, K))
    return ragmi::fail(RAG_EINVAL, "Ln*: K == 384, N % 128 == 0, N <= 2048; ResLn: N == 384");
  if (epilogue == RAG_EPI_RES_LN ? (!st_out || (st_in && (!gamma || !beta))) : (!c1 || !st_in))
    return ragmi::fail(RAG_EINVAL, "Ln*: c1 and st_in; ResLn: st_out (+ gamma, beta with st_in)");
  DlArgs d;
  d.st_in = st_in;
  d.st_out = st_out;
  d.gamma = gamma;
  d.beta = beta;
  d.c1 = c1;
  d.eps = eps;
  auto* a = static_cast<const _Float16*>(A);
  auto* al = static_cast<const _Float16*>(A_lo);
  auto* w = static_cast<const _Float16*>(W);
  auto* wl = static_cast<const _Float16*>(W_lo);
  auto* cl = static_cast<_Float16*>(C_lo);
  const auto st = static_cast<hipStream_t>(stream);
  if (epilogue == RAG_EPI_LN_F16)
    launch_ws_large<kEpiLnF16, true, 2>(a, al, w, wl, bias, M, N, K, C, cl, st, d);
  else if (epilogue == RAG_EPI_LN_GELU_F16)
    launch_ws_large<kEpiLnGeluF16, true, 2>(a, al, w, wl, bias, M, N, K, C, cl, st, d);
  else
    launch_ws_large<kEpiResLn, true>(a, al, w, wl, bias, M, N, K, C, cl, st, d);
  RAG_HIP(hipGetLastError());
  return RAG_OK;
}

int rag_build_pairs(const int32_t* q_ids, const int32_t* q_cu, int B, const int64_t* rows, int K,
                    const int16_t* c_toks, int lmax, const int32_t* c_lens, int max_len,
                    int32_t* ids, int32_t* types, int32_t* cu, int32_t* stats, void* stream) {
  ragmi::clear_error();
  if (!q_ids || !q_cu || !rows || !c_toks || !c_lens || !ids || !types || !cu || !stats)
    return ragmi::fail(RAG_EINVAL, "NULL argument");
  if (B < 1 || K < 1 || B * K > kPairsMax || lmax < 1 || max_len < 3 || max_len > 4096)
    return ragmi::fail(RAG_EINVAL, "need 1 <= B*K <= 1024, lmax >= 1, 3 <= max_len <= 4096");
  auto st = static_cast<hipStream_t>(stream);
  const int P = B * K;
  pairs_len_kernel<<<dim3(1), dim3(kPairsMax), 0, st>>>(q_cu, rows, c_lens, P, K, max_len, cu,
                                                         stats);
  pairs_fill_kernel<<<dim3(P), dim3(256), 0, st>>>(q_ids, q_cu, rows, c_toks, lmax, c_lens, cu,
                                                   K, max_len, ids, types);
  RAG_HIP(hipGetLastError());
  return RAG_OK;
}

int rag_encoder_forward_host(rag_encoder_t* e, const int32_t* ids, const int32_t* types,
                             const int32_t* cu, int B, int T, float* out) {
  ragmi::clear_error();
  if (!e || !ids || !types || !cu || !out || B < 1) return ragmi::fail(RAG_EINVAL, "bad args");
  if (cu[0] != 0 || cu[B] != T) return ragmi::fail(RAG_EINVAL, "cu_seqlens must span [0, T]");
  int max_len = 0;
  for (int b = 0; b < B; ++b) {
    const int L = cu[b + 1] - cu[b];
    if (L < 1) return ragmi::fail(RAG_EINVAL, "empty sequence");
    max_len = std::max(max_len, L);
  }
  if (max_len > e->cfg.max_position) return ragmi::fail(RAG_EINVAL, "sequence longer than max_position");
  for (int t = 0; t < T; ++t)
    if (ids[t] < 0 || ids[t] >= e->cfg.vocab || types[t] < 0 || types[t] >= e->cfg.type_vocab)
      return ragmi::fail(RAG_EINVAL, "token id / type out of range");
  const size_t ob = (size_t)B * (e->cfg.head == RAG_HEAD_CLS_L2 ? e->cfg.hidden : 1) * 4;
  const size_t need = (size_t)T * 8 + (size_t)(B + 1) * 4 + ob + 64;
  std::lock_guard<std::mutex> lk(e->mu);
  RAG_HIP(hipSetDevice(e->device));
  if (e->stage_bytes < need) {
    if (e->stage) (void)hipFree(e->stage);
    e->stage = nullptr;
    e->stage_bytes = 0;
    RAG_HIP(hipMalloc(&e->stage, need));
    e->stage_bytes = need;
  }
  char* s = static_cast<char*>(e->stage);
  int32_t* d_ids = reinterpret_cast<int32_t*>(s);
  int32_t* d_ty = d_ids + T;
  int32_t* d_cu = d_ty + T;
  float* d_out = reinterpret_cast<float*>(s + (((size_t)T * 8 + (size_t)(B + 1) * 4 + 15) & ~size_t(15)));
  RAG_HIP(hipMemcpy(d_ids, ids, (size_t)T * 4, hipMemcpyHostToDevice));
  RAG_HIP(hipMemcpy(d_ty, types, (size_t)T * 4, hipMemcpyHostToDevice));
  RAG_HIP(hipMemcpy(d_cu, cu, (size_t)(B + 1) * 4, hipMemcpyHostToDevice));
  int rc = forward_locked(e, d_ids, d_ty, d_cu, B, T, max_len, d_out, nullptr);
  if (rc) return rc;
  RAG_HIP(hipDeviceSynchronize());
  RAG_HIP(hipMemcpy(out, d_out, ob, hipMemcpyDeviceToHost));
  return RAG_OK;
}

}  // extern "C"
