/*
 * ragmi_bert.h — C ABI of the two BERT-small encoders on the retrieval hot path (libragmi.so).
 *
 * Replaces, for the reference (pythonmailer/financial-rag-system):
 *   main.py:80-84 / main2.py:88-96  get_embedder() -> SentenceTransformer("BAAI/bge-small-en-v1.5")
 *       .encode(str | list[str])  (main.py:144-149 /embed, 211-213 embed_query; main2.py:170-171
 *       embed_query_batch)                                   -> rag_encoder_create(head = RAG_HEAD_CLS_L2)
 *                                                              + rag_encoder_forward
 *   main.py:86-90 / main2.py:98-103 get_reranker() -> CrossEncoder("cross-encoder/ms-marco-MiniLM-L-6-v2")
 *       .predict([[q, t], ...])  (main.py:241-247 rerank_documents) -> head = RAG_HEAD_POOLER_CLS
 * Tokenisation (WordPiece) stays on the host (ragmi.encoders, `tokenizers` + a local vocab).
 *
 * Inputs are PACKED sequences: token ids / token-type ids of all B sequences back to back
 * (int32 [T]) and cu_seqlens (int32 [B+1], cu[0] = 0, cu[B] = T). Right padding in the
 * reference never changes a valid token's output, so packing is exact.
 * Outputs: RAG_HEAD_CLS_L2 -> fp32 [B][hidden] (L2-normalised CLS vector);
 *          RAG_HEAD_POOLER_CLS -> fp32 [B] (raw logit, identity activation).
 * Built shapes: hidden/heads 384/12 (bge-small, MiniLM-L6), 768/12 (bge-base) and 1024/16
 * (bge-large, config 5); head_dim 32 or 64; intermediate = 4 x hidden; max_pos <= 512.
 * Numerics: fp16 (or split fp16x3) GEMM/attention operands, fp32 accumulation / residual
 * stream / LayerNorm / softmax statistics.
 */
#ifndef RAGMI_BERT_H
#define RAGMI_BERT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { RAG_HEAD_CLS_L2 = 0, RAG_HEAD_POOLER_CLS = 1 };

enum { RAG_PREC_FP16 = 0, RAG_PREC_FP16X3 = 1 };

typedef struct {
  int vocab, hidden, layers, heads, intermediate, max_position, type_vocab;
  float layer_norm_eps;
  int head;      /* RAG_HEAD_* */
  int precision; /* RAG_PREC_FP16: fp16 GEMM/attention operands (fastest);
                    RAG_PREC_FP16X3: every product as a_hi*b_hi + a_hi*b_lo + a_lo*b_hi on the
                    fp16 MFMA pipe (~fp32 accuracy, 3x the MFMA work) */
} rag_bert_config;

typedef struct rag_encoder rag_encoder_t;

/* Number of weight tensors rag_encoder_create expects for `cfg`:
 * 5 + 16 * layers (+ 4 for RAG_HEAD_POOLER_CLS). */
int rag_encoder_num_weights(const rag_bert_config* cfg);

/* weights: host fp32 tensors in HF state-dict layout (Linear weight = [out][in]), order:
 *   embeddings.word_embeddings [vocab][H], .position_embeddings [max_pos][H],
 *   .token_type_embeddings [type_vocab][H], .LayerNorm.weight [H], .LayerNorm.bias [H];
 *   per layer l: attention.self.query.{weight [H][H], bias}, .key.{w,b}, .value.{w,b},
 *     attention.output.dense.{w,b}, attention.output.LayerNorm.{weight,bias},
 *     intermediate.dense.{weight [I][H], bias [I]}, output.dense.{weight [H][I], bias [H]},
 *     output.LayerNorm.{weight,bias};
 *   RAG_HEAD_POOLER_CLS: pooler.dense.{weight [H][H], bias}, classifier.{weight [1][H], bias [1]}. */
int rag_encoder_create(const rag_bert_config* cfg, const float* const* weights, int n_weights,
                       int device, rag_encoder_t** out);
/* rag_encoder_create with flags: RAG_CREATE_DIAGNOSTIC (ragmi.h) makes the process honour the
 * RAGMI_* kernel A/B knobs (GEMM / attention variants, split-K, fusion modes) — bench and
 * profiling scripts only. */
int rag_encoder_create_ex(const rag_bert_config* cfg, const float* const* weights, int n_weights,
                          int device, int flags, rag_encoder_t** out);
int rag_encoder_destroy(rag_encoder_t* enc);

/* Device pointers, asynchronous on `stream` (hipStream_t). max_len must be >= the longest
 * sequence (it sizes the attention kernel's LDS; a longer sequence is truncated to max_len
 * instead of overrunning it). */
int rag_encoder_forward(rag_encoder_t* enc, const int32_t* ids_dev, const int32_t* types_dev,
                        const int32_t* cu_seqlens_dev, int B, int T, int max_len,
                        float* out_dev, void* stream);
/* Host pointers, synchronous. */
int rag_encoder_forward_host(rag_encoder_t* enc, const int32_t* ids, const int32_t* types,
                             const int32_t* cu_seqlens, int B, int T, float* out);

/* Host-native WordPiece tokenisation of ASCII text (sentence-transformers' encode(list[str]) /
 * CrossEncoder.predict tokenise every call: main2.py:170-171, main.py:245). Exactly the rules
 * of the Rust tokenizers BertWordPieceTokenizer (clean_text, lowercase, punctuation split,
 * greedy longest-match WordPiece with "##" continuations, 100-char words -> [UNK],
 * [CLS] a [SEP] (b [SEP]) with token types 0 / 1, 'longest_first' truncation to max_length).
 * vocab_txt: the checkpoint's vocab.txt bytes (line i = id i, trailing whitespace trimmed,
 * later duplicates win). Texts (and optional pairs) are byte blobs with n+1 offsets; a text or
 * pair holding any byte >= 0x80 is skipped (fallback[j] = 1, zero tokens): the caller encodes
 * it with the Unicode-complete tokenizer. Outputs: ids / types [<= cap], cu [n+1] (packed).
 * Host memory, synchronous, thread-safe for concurrent encodes on one handle. */
typedef struct rag_wordpiece rag_wordpiece_t;
int rag_wordpiece_create(const char* vocab_txt, int64_t nbytes, int max_length, int lowercase,
                         rag_wordpiece_t** out);
int rag_wordpiece_destroy(rag_wordpiece_t* t);
int rag_wordpiece_encode(const rag_wordpiece_t* t, const char* texts, const int64_t* text_off,
                         const char* pairs, const int64_t* pair_off, int n, int32_t* ids,
                         int32_t* types, int32_t* cu, int64_t cap, uint8_t* fallback);

/* Cross-encoder batch assembly on the device (the batched rerank stage without a host round
 * trip: main.py:241-247 CrossEncoder.predict([[q, t] ...]) pair encoding
 * "[CLS] q [SEP] t [SEP]", token types 0/1, chunk truncated to fit max_len). Device pointers,
 * async on `stream`. q_ids/q_cu: the packed query batch (each query [CLS] ... [SEP]);
 * rows int64 [B][K]: search hits (-1 = none: row 0 is used, the caller masks); c_toks int16
 * [rows][lmax] cached chunk WordPiece ids (read as uint16), c_lens int32 [rows].
 * Outputs: ids/types int32 [<= B*K*max_len], cu int32 [B*K+1], stats int32 [2] = {T, longest
 * pair}. B*K <= 1024. */
int rag_build_pairs(const int32_t* q_ids, const int32_t* q_cu, int B, const int64_t* rows, int K,
                    const int16_t* c_toks, int lmax, const int32_t* c_lens, int max_len,
                    int32_t* ids, int32_t* types, int32_t* cu, int32_t* stats, void* stream);

/* Diagnostic entry (parity tests and the GEMM benchmark; not called by the reference path):
 * one encoder GEMM C[M,N] = A[M,K] . W[N,K]^T + bias[N] (the nn.Linear of modeling_bert.py
 * BertSelfAttention/BertIntermediate/BertOutput), device pointers, async on `stream`.
 * A, W fp16 row-major; A_lo/W_lo the fp16x3 residual planes (both NULL = plain fp16).
 * epilogue: RAG_EPI_F16 (C fp16 [+ C_lo]), RAG_EPI_GELU_F16 (erf-GELU, fp16 [+ C_lo]),
 * RAG_EPI_F32 (C fp32). variant: RAG_GEMM_AUTO (what the forward uses: SMALL for query
 * batches, WS once its 256x128 tiles reach half the CUs, TILE in between), _TILE (128x128
 * tiles, 2 workgroups per CU), _SMALL (64x64 tiles, the K panel in flight), _WS (persistent
 * 256x128 tiles, 4 loader waves feeding 8 MFMA waves through an LDS-DMA ring).
 * Timing probes of _WS (results meaningless; scripts/bench_gemm.py): _WS_NO_STORE (the
 * epilogue without its stores), _WS_MFMA_ONLY (no DMAs, no stores), _WS_DMA_ONLY (the DMA
 * ring alone). The round 1-5 A/B forms (PIPE, WIDE, BIG, SMALL_BK64, WS_BIG128, the ping-pong
 * GEMM, ...) were removed in round 5; their ids stay unassigned and are refused.
 * N % 128 == 0, K % 64 == 0 (SMALL / WS also N <= 4096). */
enum { RAG_EPI_F16 = 0, RAG_EPI_GELU_F16 = 1, RAG_EPI_F32 = 2 };
/* deferred-LayerNorm epilogues (rag_bert_gemm_dl) */
enum { RAG_EPI_LN_F16 = 4, RAG_EPI_LN_GELU_F16 = 5, RAG_EPI_RES_LN = 6 };
enum { RAG_GEMM_AUTO = 0, RAG_GEMM_TILE = 1, RAG_GEMM_SMALL = 5, RAG_GEMM_WS = 19,
       RAG_GEMM_WS_MFMA_ONLY = 20, RAG_GEMM_WS_NO_STORE = 21, RAG_GEMM_WS_DMA_ONLY = 22 };
int rag_bert_gemm(int variant, int epilogue, const void* A, const void* A_lo, const void* W,
                  const void* W_lo, const float* bias, int M, int N, int K, void* C,
                  void* C_lo, void* stream);

/* Diagnostic (parity tests, GEMM benchmark): the fp32-output GEMM with the split-K the forward
 * uses for small token batches — C holds max_parts x [M][N] floats and receives `*parts`
 * partial products (part 0 carries the bias) whose sum is A . W^T + bias; the forward sums
 * them in order inside its residual + LayerNorm pass. variant: AUTO or SMALL
 * (AUTO outside the small-batch regime writes one part). */
int rag_bert_gemm_splitk(int variant, const void* A, const void* A_lo, const void* W,
                         const void* W_lo, const float* bias, int M, int N, int K, float* C,
                         int max_parts, int* parts, void* stream);

/* the output projection of an encoder layer with its residual + LayerNorm fused
 * (modeling_bert.py BertSelfOutput / BertOutput: LayerNorm(dense(h) + x), eval mode), in place
 * on the fp32 residual rows: x[M,N] = LN(x + A . W^T + bias) * gamma + beta, xh = fp16(x),
 * xl = fp16(x - xh) (fp16x3: A_lo, W_lo and xl all given, else all NULL). N == 384 (whole
 * rows per tile), K % 64 == 0. What rag_encoder_forward runs for large fp16-mode token
 * counts (rag_encoder_set_fusion); exported for parity tests. */
int rag_bert_gemm_add_ln(const void* A, const void* A_lo, const void* W, const void* W_lo,
                         const float* bias, const float* gamma, const float* beta, float eps,
                         int M, int N, int K, float* x, void* xh, void* xl, void* stream);

/* Encoder attention alone, hidden 384 / head_dim 32 (bge-small, MiniLM-L6): ctx[T][384] =
 * per (sequence, head) softmax(Q K^T / sqrt(32)) V over the packed rows of qkv[T][1152]
 * (Q | K | V), cu[B+1] row offsets, max_len >= every sequence length (<= 512). qkv_lo /
 * ctx_lo: the fp16x3 lo planes (both or neither). variant: the kernel's VAR bit mask, 0..15
 * (1 rolling Q prefetch, 2 fp16x3 row sums by MFMA, 4 software-pipelined scores, 8 lean
 * block), 18 or 26 (16 = two query blocks per wave side by side), or -1 for the one the
 * forward runs (42). For A/B timing and parity tests. The production library carries -1 / 42
 * and the A/B slot 10 only; the rest of the family is in the diagnostic build
 * (rag_diagnostic_build, ragmi.h). */
int rag_bert_attention(int variant, const void* qkv, const void* qkv_lo, const int32_t* cu,
                       int B, int max_len, void* ctx, void* ctx_lo, void* stream);

/* forward's use of rag_bert_gemm_add_ln: -1 auto (default; env RAGMI_FUSE_LN overrides at
 * create), 0 never (separate GEMM + add-LayerNorm kernels), 1 always where the shape allows */
int rag_encoder_set_fusion(rag_encoder_t* e, int mode);

/* hipGraph replay of small-batch forwards: -1 auto (default; env RAGMI_ENC_GRAPH=0/1
 * overrides auto): calls with T <= 8192 tokens stage their inputs into
 * the stream's workspace (one kernel), replay the graph captured for the padded shape (T to a
 * multiple of 64, max_len to a multiple of 32; captured on first use from the eager path) and
 * copy the output rows out — three host calls instead of ~90 kernel launches; 0 never; 1 for
 * every call. A call on the null stream replays on the encoder's own stream, ordered after the
 * null stream's earlier work and before its later work by two events. Results are those of the
 * eager forward at the padded T. */
int rag_encoder_set_graphs(rag_encoder_t* e, int mode);

/* Deferred LayerNorm (fp16x3, hidden 384): the token rows' residual stream is kept
 * un-normalised between sublayers — z = x + sublayer output as fp16 hi + lo planes, plus per row
 * six {mean, centred sum of squares} statistics of its 64-column blocks — and LN(z) is applied
 * inside the GEMMs: a consumer (QKV, FFN1) multiplies z by W' = W diag(gamma) and corrects each
 * row in its epilogue, LN(z) W^T + b = rstd (z W'^T - mean c1) + c2 (c1 = row sums of W',
 * c2 = b + W beta, folded at rag_encoder_create), and the next residual add recomputes
 * LN(z) = (z - mean) rstd gamma + beta per element (modeling_bert.py BertSelfOutput /
 * BertOutput: LayerNorm(dense(h) + x), restated). Replaces the separate add-LayerNorm passes
 * on large token batches. Forward use: -1 auto (default, env RAGMI_DEFER_LN overrides at
 * create: once every token-row GEMM is the WS kernel, ~11K tokens), 0 never, 1 always where
 * the model allows (fp16x3, hidden 384). */
int rag_encoder_set_defer_ln(rag_encoder_t* e, int mode);

/* The deferred-LayerNorm forward's FFN (modeling_bert.py BertIntermediate + BertOutput) as ONE
 * launch per layer (round 6): FFN1 + GELU + FFN2 + residual + LayerNorm statistics over
 * 128-row tiles, the 1536-wide intermediate kept on the CU instead of written to and re-read
 * from HBM. Every output bit equals the two-GEMM form's at >= 16,384 tokens (the WS GEMMs'
 * natural K order). Measured 8-21% slower than the two GEMMs, so only the
 * diagnostic build (rag_diagnostic_build) carries it: there -1 auto (= off), 0 never, 1 / 2
 * on with 128- / 256-column chunks of the intermediate, 3-5 further A/B shapes; the
 * production library accepts -1 and 0. */
int rag_encoder_set_ffn_fused(rag_encoder_t* e, int mode);

/* fp16 range guard (no reference counterpart: the reference's torch forward is fp32). Every
 * activation the forward keeps as an fp16 plane is bounded by the weights alone, for any input
 * (interval arithmetic over the layer: |LN_i| <= |gamma_i| sqrt(H-1) + |beta_i|,
 * |W x + b|_j <= sum |W_ji| bound(x_i) + |b_j|, context <= bound(V), |gelu(y)| <= |y|).
 * plain: the largest such bound over the LN outputs, Q|K|V, attention context and FFN
 * intermediate; deferred: also over the un-normalised residual sums z the deferred
 * LayerNorm stores as planes. rag_encoder_create fails with RAG_ERANGE when plain > 60000
 * (fp16 max 65504), and the deferred LayerNorm is never used when deferred > 60000
 * (rag_encoder_set_defer_ln(1) then fails with RAG_ERANGE): no forward can return inf from an
 * fp16 overflow. rag_encoder_weight_bounds computes the same from host weights (no device). */
int rag_encoder_range_bounds(const rag_encoder_t* e, double* plain, double* deferred);
int rag_encoder_weight_bounds(const rag_bert_config* cfg, const float* const* weights,
                              int n_weights, double* plain, double* deferred);

/* the deferred-LayerNorm GEMM epilogues alone (parity tests), on the WS kernel (fp16x3: A_lo,
 * W_lo, C_lo required): st_in / st_out are [M][6][2] floats ({mean, M2} of columns 64j..64j+63).
 *  RAG_EPI_LN_F16 / RAG_EPI_LN_GELU_F16 (K == 384, N % 128 == 0, N <= 2048): per row r with
 *    (mean, rstd) from st_in, C = [gelu](rstd (A W^T - mean c1) + bias) as hi + lo planes;
 *  RAG_EPI_RES_LN (N == 384): z = (A W^T + bias) + x, x = (C - mean) rstd gamma + beta from
 *    the planes C / C_lo read in place (st_in NULL: x = C as is), written back to C / C_lo
 *    with its block statistics to st_out. */
int rag_bert_gemm_dl(int epilogue, const void* A, const void* A_lo, const void* W,
                     const void* W_lo, const float* bias, const float* c1, const float* st_in,
                     const float* gamma, const float* beta, float eps, int M, int N, int K,
                     void* C, void* C_lo, float* st_out, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* RAGMI_BERT_H */
