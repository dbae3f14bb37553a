/*
 * kwhisper -- C ABI of the MI355X (gfx950) Whisper teacher hot path.
 *
 * Drop-in boundary: the Python host (kotoba-whisper_amd/kwhisper) binds these entry points with
 * ctypes and exposes HF's WhisperForConditionalGeneration.generate() / WhisperFeatureExtractor API
 * (SURVEY.md §8b).  Every pointer below is a DEVICE pointer unless stated; the caller owns all
 * memory (kernels never allocate); every call is asynchronous on `stream` (a hipStream_t, 0 =
 * null stream) and is safe to capture in a hipGraph.  Return value: KW_OK or a KW_E* code;
 * kw_last_error() gives the message.  Nothing throws across the ABI.
 *
 * Element types: KW_DT_F32 = float32, KW_DT_BF16 = bfloat16 (raw uint16 storage).
 * Reference interfaces each entry point replaces are cited as TF/<file>:<line>, where
 * TF = transformers 5.15.0 (the arithmetic of kotoba-whisper's hot path, run_pseudo_labelling.py:338).
 */
#ifndef KWHISPER_H
#define KWHISPER_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* kw_stream_t;

enum { KW_OK = 0, KW_EINVAL = 1, KW_EHIP = 2, KW_EUNSUPPORTED = 3 };
enum { KW_DT_F32 = 0, KW_DT_BF16 = 1 };
enum { KW_EPI_STORE = 0, KW_EPI_RESID = 1, KW_EPI_HEADSPLIT = 2 };

/* ABI version (major*100 + minor) and the last error message of this thread. */
int kw_version(void);  /* 112 */
const char* kw_last_error(void);

/* A new non-blocking stream of its own (hipStreamCreateWithFlags), for callers that must not share one: the streams a
 * hipGraph capture forks into (PyTorch hands out streams from a fixed pool, so two host threads can be given the same
 * one, and a thread's launches on a stream another thread's capture has forked into join that capture). */
int kw_stream_create(kw_stream_t* out);
int kw_stream_destroy(kw_stream_t stream);

/* a1 -- log-mel spectrogram.
 * Replaces WhisperFeatureExtractor._torch_extract_fbank_features (TF/models/whisper/
 * feature_extraction_whisper.py:135-168): stft(n_fft 400, hop 160, periodic hann, center, reflect)
 * -> |X|^2 -> drop last frame -> mel_filters.T @ P -> log10(clamp 1e-10) -> per-clip max(x, max-8)
 * -> (x+4)/4.   audio: [batch][audio_stride] f32 (first n_samples used, n_samples % 160 == 0,
 * already padded/truncated as in __call__ :300-307); mel_filters: [201][n_mels] f32;
 * out: [batch][n_mels][n_samples/160] f32; workspace: >= 4*batch bytes. */
int kw_log_mel(const float* audio, int64_t batch, int64_t n_samples, int64_t audio_stride,
               const float* mel_filters, int n_mels, float* out, void* workspace, kw_stream_t stream);

/* Conv stem input re-layout: mel [B][C][T] f32 -> time-major, zero-padded [B][T+2][c_pad] (dtype),
 * so that Conv1d(k=3, p=1) is a GEMM whose im2col row t is the contiguous 3*c_pad slice at row t
 * (TF/models/whisper/modeling_whisper.py:566-567,618-619). */
int kw_mel_to_time_major(const float* mel, int64_t B, int64_t C, int64_t T, int64_t c_pad,
                         void* out, int out_dtype, kw_stream_t stream);

/* Linear / conv-as-GEMM:  C = epilogue(A . W^T + bias)  (nn.Linear, TF modeling_whisper.py:279-282,
 * 375-376, 444-445, 499-503, 566-567, 1080).
 * Row maps: logical row r of A lives at A + (r / a_rows_per_batch)*a_batch_stride
 * + (r % a_rows_per_batch)*lda (elements); the same for C.  W: [N][K] (or packed, kw_gemv).
 * Epilogues: STORE  C = act(acc + bias) * (col < scale_cols ? scale : 1) (+ row_add[r % period][col])
 *            RESID  C(f32) += acc + bias           (residual add, TF modeling_whisper.py:398,407)
 *            HEADSPLIT  as STORE, written to C[part][b][h][t][d] with part = col / (heads*head_dim),
 *                       b = r / hs_seq, t = r % hs_seq  (q/k/v and cross-K/V cache layout). */
typedef struct {
  int dtype;                 /* A and W element type */
  int c_dtype;               /* C element type (RESID: must be KW_DT_F32) */
  const void* A;
  int64_t lda, a_rows_per_batch, a_batch_stride;
  const void* W;
  const float* bias;         /* [N] or NULL */
  void* C;
  int64_t ldc, c_rows_per_batch, c_batch_stride;
  int64_t M, N, K;
  int epilogue;              /* KW_EPI_* */
  int gelu;                  /* exact-erf GELU after bias */
  float scale;               /* applied to columns [0, scale_cols) after bias/GELU */
  int64_t scale_cols;
  const float* row_add;      /* [period][N] f32 added after the activation, or NULL */
  int64_t row_add_period;
  int64_t hs_seq, hs_heads, hs_head_dim;
} kw_gemm_args;

int kw_gemm(const kw_gemm_args* args, kw_stream_t stream);

/* ---- decode step (bf16 engine) --------------------------------------------------------------- */

/* Decode-step linear over packed weights, any M (launched in 32-row chunks):
 *   A = x (bf16 [M][ldx]) or, if ln != 0, the LayerNorm (x - mean) * rstd (eps ln_eps) of each row of it,
 *   with gamma/beta folded into W / bias by the caller (W' = W diag(gamma), b' = b + W beta) and
 *   ln_colsum[n] = sum_k W'[n][k] (f32, of the bf16 values packed); computed as
 *   rstd * (x W'^T - mean * ln_colsum) with each row's statistics taken from x itself
 *   (TF modeling_whisper.py:446,476,500 + 469-503, proj_out :1080);
 *   STORE: C[m][n] = act(acc + bias) * (n < scale_cols ? scale : 1), C f32 or bf16;
 *   RESID: h[m][n] += acc + bias (f32 residual, modeling_whisper.py:482,495,503) and hb = bf16(h), the
 *          bf16 mirror the next LayerNorm-fused linear reads.
 * W: packed by kw_pack_weight.  workspace: >= kw_dec_linear_workspace_bytes(N, K) bytes, zero-filled
 * before first use (calls leave it zeroed); one workspace may serve all calls on one stream.
 * Results are bitwise deterministic (fixed-order reductions, no float atomics). */
typedef struct {
  const void* x;
  int64_t ldx;
  int ln;                    /* fuse the LayerNorm of x (STORE only) */
  float ln_eps;
  const float* ln_colsum;    /* [N], required with ln */
  const void* W;
  const float* bias;         /* [N] f32 or NULL */
  int epilogue;              /* KW_EPI_STORE or KW_EPI_RESID */
  void* C;                   /* STORE output [M][ldc] */
  int64_t ldc;
  int c_dtype;
  int gelu;
  float scale;
  int64_t scale_cols;
  float* h;                  /* RESID: f32 residual [M][ldh] (in/out) */
  void* hb;                  /* RESID: bf16 mirror [M][ldh] (out) */
  int64_t ldh;
  int64_t M, N, K;
  void* workspace;
  size_t ws_bytes;
} kw_dec_linear_args;

int kw_dec_linear(const kw_dec_linear_args* args, kw_stream_t stream);
size_t kw_dec_linear_workspace_bytes(int64_t N, int64_t K);
/* W [N][K] bf16 -> packed [ceil(N/32)*2][K/32][64 lanes][8] bf16 (columns >= N zero); K % 32 == 0. */
int kw_pack_weight(const void* W, int64_t N, int64_t K, void* packed, kw_stream_t stream);
size_t kw_packed_weight_bytes(int64_t N, int64_t K);

/* LayerNorm (eps) over the last dim of x [rows][dim] f32 -> y [rows][dim] (y_dtype);
 * TF modeling_whisper.py:371,377,434,443,446,642,790. dim % 4 == 0, dim <= 2048.  delta (bf16
 * [rows][dim] or NULL): the producing linear's output, added to x in place first (the residual add
 * of :398,407 fused in front of the next LayerNorm). */
int kw_layernorm(float* x, int64_t rows, int64_t dim, const float* gamma, const float* beta,
                 float eps, void* y, int y_dtype, const void* delta, kw_stream_t stream);
/* The same over a bf16 residual stream x [rows][dim] (the encoder's bf16 path): x += delta is rounded
 * to bf16, as the reference's residual add in a bf16 model is. dim % 8 == 0, dim <= 2048, x/y/delta
 * 16-B aligned. */
int kw_layernorm_bf16res(void* x, int64_t rows, int64_t dim, const float* gamma, const float* beta,
                         float eps, void* y, int y_dtype, const void* delta, kw_stream_t stream);

/* Encoder self-attention softmax(Q K^T) V (q pre-scaled; TF sdpa_attention.py:79-166, non-causal).
 * qkv: [3][B][H][T][hd] (dtype), out: [B][T][H*hd] (dtype). hd == 64.  dtype | KW_ATTN_Q_LOG2 (bf16 only):
 * q also carries log2(e) (scores in log2 units -- the producer folds it into its q scale), which saves the
 * softmax one multiply-add per score. */
#define KW_ATTN_Q_LOG2 0x100
int kw_attention(int dtype, const void* qkv, int64_t B, int64_t H, int64_t T, int64_t hd, void* out,
                 kw_stream_t stream);

/* Decoder input embedding: h[b*q_len+i] = tok_emb[ids[b][L-q_len+i]] + pos_emb[L-q_len+i]
 * with L = *cur_len read on device (TF modeling_whisper.py:737-762; no embed scale); hb (optional,
 * bf16, may be NULL) receives bf16(h) for the bf16 engine's LayerNorm-fused linears. */
int kw_embed(int dtype, const int64_t* ids, int64_t ids_stride, int64_t B, int64_t q_len,
             const int32_t* cur_len, const void* tok_emb, const void* pos_emb, int64_t d, float* h,
             void* hb, kw_stream_t stream);

/* Decoder self-attention over a static cache (TF modeling_whisper.py:469-480, cache_utils.py:127-145):
 * appends k/v of the q_len newest positions [L-q_len, L) to k_cache/v_cache [B][H][t_max][hd],
 * then causal attention for those positions. qkv: [B*q_len][3*H*hd]; out [B*q_len][H*hd]; t_max <= 512.
 * q_len == 1 needs workspace >= kw_self_attn_workspace(B, H, t_max) bytes, zero-filled before first use
 * (arrival counters every call leaves at zero); q_len > 1 ignores it.  bp (q_len == 1 only, or NULL):
 * beam-search slot table [B][bp_stride] int32 -- key/value position k < L-1 of row b is read from
 * cache row bp[b][k] (beams share their prefix; the reorder of cache_utils.py:2035-2038 moves no K/V). */
int kw_self_attn_step(int dtype, const void* qkv, int64_t B, int64_t q_len, int64_t H, int64_t hd,
                      void* k_cache, void* v_cache, int64_t t_max, const int32_t* cur_len,
                      const int32_t* bp, int64_t bp_stride, void* out, void* workspace, size_t ws_bytes,
                      kw_stream_t stream);
size_t kw_self_attn_workspace(int64_t B, int64_t H, int64_t t_max);

/* The self-attention block of one greedy decode step in ONE launch (bf16): the LayerNorm-fused QKV projection
 * (TF modeling_whisper.py:446,469-471; q * head_dim^-0.5 :309) and the self-attention step over the static
 * cache with the new key / value appended (:469-480, cache_utils.py:127-145) -- kw_dec_linear(qkv) followed by
 * kw_self_attn_step(q_len 1) without the kernel boundary (the projection and caches bitwise the same, the
 * attention output within bf16 rounding: its keys are summed in 16-slot passes): the projection's output is
 * handed to the attention in-launch as 8-byte {bf16 x 2, tag} granules while the cached K/V rows load.
 * cur_len outside [1, min(256, t_max)] sets the workspace status word (kw_dec_qkv_self_status_offset) and writes NaN.
 *   x: hb [M][ldx] bf16 (the residual mirror; LayerNorm applied as kw_dec_linear's ln); W: packed [3d][d] with
 *   gamma folded (kw_pack_weight); ln_colsum / bias: [3d] f32; scale multiplies the q columns (< d);
 *   k_cache / v_cache: one layer's [M][H][t_max][64] bf16; cur_len: L on device (positions [0, L-1) cached,
 *   L-1 new), L <= 256; out: [M][d] bf16.  M <= 32, d = 64 H, d <= 1280.
 * workspace >= kw_dec_qkv_self_workspace(M, d) bytes, ZERO-FILLED before first use (every call re-arms it).
 * Every in-launch wait is on work dispatched before it (no co-residency assumption: safe beside other work on
 * the GPU).  kw_dec_qkv_self_supported(): 1 when the shape is covered. */
typedef struct {
  const void* x;
  int64_t ldx;
  float ln_eps;
  const float* ln_colsum;
  const void* W;
  const float* bias;
  float scale;
  int64_t M, d, H;
  void* k_cache;
  void* v_cache;
  int64_t t_max;
  const int32_t* cur_len;
  void* out;
  void* workspace;
  size_t ws_bytes;
} kw_dec_qkv_self_args;

int kw_dec_qkv_self(const kw_dec_qkv_self_args* args, kw_stream_t stream);
size_t kw_dec_qkv_self_workspace(int64_t M, int64_t d);
int kw_dec_qkv_self_supported(int64_t M, int64_t d, int64_t H);

/* The cross-attention block's query projection and attention step of one greedy decode step in ONE launch
 * (bf16): the LayerNorm-fused q projection (TF modeling_whisper.py:483; q * head_dim^-0.5 :309) and the
 * attention over the item's encoder K / V (:323-356) -- kw_dec_linear(xq) followed by kw_cross_attn_step
 * (q_len 1) without the kernel boundary, bit for bit: the projection hands the query to the attention
 * in-launch as 8-byte {bf16 x 2, tag} granules while the chunks' K / V streams are already in flight.
 *   x: hb [M][ldx] bf16; W: packed [d][d] with gamma folded (kw_pack_weight); ln_colsum / bias: [d] f32; scale
 *   multiplies every column; k / v: one layer's [M][H][S][64] bf16 (item m's K / V); out: [M][d] bf16.
 *   M <= 32, d = 64 H <= 1280, S such that kw_cross_attn_step's chunks hold 225..256 keys (e.g. 1500).
 * workspace >= kw_dec_xq_cross_workspace(M, d, H, S) bytes, ZERO-FILLED before first use (every call re-arms
 * it).  Every in-launch wait is on work dispatched before it (no co-residency assumption: safe beside other
 * work on the GPU).  kw_dec_xq_cross_supported(): 1 when the shape is covered. */
typedef struct {
  const void* x;
  int64_t ldx;
  float ln_eps;
  const float* ln_colsum;
  const void* W;
  const float* bias;
  float scale;
  int64_t M, d, H;
  const void* k;
  const void* v;
  int64_t S;
  void* out;
  void* workspace;
  size_t ws_bytes;
} kw_dec_xq_cross_args;

int kw_dec_xq_cross(const kw_dec_xq_cross_args* args, kw_stream_t stream);
size_t kw_dec_xq_cross_workspace(int64_t M, int64_t d, int64_t H, int64_t S);
int kw_dec_xq_cross_supported(int64_t M, int64_t d, int64_t H, int64_t S);

/* Which grid a bf16 one-row cross-attention of `rows` = B * H (row, head) pairs over S keys launches (for
 * profilers naming kernels): 1 = one workgroup per pair streaming its chunks (cross_attn_row_kernel; used when
 * the pairs fill the CUs and fit at once and S = 1500), 0 = one workgroup per (pair, chunk).  fused: the
 * kw_dec_xq_cross variant.  Both give bitwise the same rows. */
int kw_cross_attn_pair_kernel(int64_t rows, int64_t S, int fused);

/* Decoder cross-attention against cached encoder K/V [B][H][S][hd] (TF modeling_whisper.py:323-326).
 * q: [B*q_len][H*hd]; out: [B*q_len][H*hd]; S <= 2048; workspace >= kw_cross_attn_workspace(...) bytes and
 * ZERO-FILLED before its first use (it holds arrival counters that every call leaves at zero). */
int kw_cross_attn_step(int dtype, const void* q, int64_t B, int64_t q_len, int64_t H, int64_t hd,
                       const void* k, const void* v, int64_t S, void* out, void* workspace,
                       size_t ws_bytes, kw_stream_t stream);
size_t kw_cross_attn_workspace(int64_t B, int64_t q_len, int64_t H, int64_t hd, int64_t S);

/* Hand-off status of kw_dec_qkv_self / kw_dec_xq_cross / kw_cross_attn_step: the byte offset, inside the
 * caller's workspace of that entry point (same dimensions), of an int32 STATUS word.  A launch whose in-launch
 * hand-off poll timed out (a protocol failure, never expected) -- or, for kw_dec_qkv_self, whose cur_len was
 * outside [1, min(256, t_max)] -- sets it nonzero and writes NaN into the rows concerned; no kernel clears it.
 * The caller reads it after synchronizing the stream and, when it is set, rejects that work's results and
 * zero-fills the whole workspace (a late producer may have left granules armed) before the next launch
 * (failures surface as errors, not as tokens; kwhisper.decode raises KWError).
 * The int32 after the status word of kw_dec_qkv_self / kw_dec_xq_cross is a FAULT-INJECTION word for tests:
 * while it is nonzero, the next launch's first projection workgroup skips its publish and clears it, so
 * that launch's consumers of the projection's columns [0, 16) time out and set the status word. */
size_t kw_dec_qkv_self_status_offset(int64_t M, int64_t d);
size_t kw_dec_xq_cross_status_offset(int64_t M, int64_t d, int64_t H, int64_t S);
size_t kw_cross_attn_status_offset(int64_t B, int64_t q_len, int64_t H, int64_t hd, int64_t S);

/* One greedy decoding step on f32 logits [B][V] (TF generation/utils.py:2894-2937):
 * SuppressTokens -> SuppressTokensAtBegin (when L == begin_index) -> WhisperTimeStamp (if
 * return_timestamps; TF generation/logits_process.py:1816-2047) -> argmax (first max) ->
 * finished rows emit pad -> ids[b][L] = token; unfinished[b] updated (EOS / L+1 >= max_length);
 * the last workgroup advances *cur_len and writes *n_unfinished.  suppress_mask: [V] uint8 (1 = suppressed).
 * scores_out: optional [B][V] f32 copy of the processed scores (NULL to skip). */
typedef struct {
  float* logits;
  int64_t B, V;
  const uint8_t* suppress_mask;
  const int32_t* begin_suppress;
  int32_t n_begin_suppress;
  int32_t return_timestamps;
  int32_t ts_begin, no_ts_id, eos_id, pad_id;
  int32_t max_initial_ts;     /* -1 = None */
  int64_t* ids;               /* [B][ids_stride] */
  int64_t ids_stride;
  int32_t* cur_len;
  int32_t max_length, begin_index;
  int32_t* unfinished;        /* [B] */
  int32_t* counter;           /* [1] scratch, zero before first use */
  int32_t* n_unfinished;      /* [1] rows still unfinished after this step (written by the last workgroup) */
  float* scores_out;
  void* workspace;            /* optional, zero-filled once, >= kw_greedy_step_workspace(B) bytes: without
                                 timestamps / scores_out each row is split over several workgroups whose
                                 partial argmaxes the row's last arriver combines (NULL: one workgroup per row) */
  size_t ws_bytes;
} kw_sampler_args;

int kw_greedy_step(const kw_sampler_args* args, kw_stream_t stream);
size_t kw_greedy_step_workspace(int64_t B);

/* The LM head and the greedy step of one decode step in ONE launch (no timestamps): kw_dec_linear(lm) -- the final
 * LayerNorm folded, proj_out (TF modeling_whisper.py:790,1080) -- followed by kw_greedy_step (TF generation/
 * utils.py:2894-2937: SuppressTokens, SuppressTokensAtBegin, argmax, finished rows emit pad, stopping) without the
 * kernel boundary: every workgroup of the LM head's weight stream publishes, per row, the processed arg-max of its
 * run of columns, and the last one to arrive merges them and finishes the step.  The token is kw_greedy_step's
 * (first index among equal maxima; a NaN logit never wins).
 *   lm: a kw_dec_linear LM head -- LayerNorm-fused (ln = 1) STORE, M = B <= 32 rows; lm->C: f32 logits [B][ldc], or
 *       NULL to skip storing them (the greedy step needs only the arg-max);
 *   g:  a kw_sampler_args of the same B x V with return_timestamps = 0 and scores_out = NULL; g->logits and
 *       g->counter are not used; g->workspace >= kw_dec_lm_greedy_workspace(B, V) bytes, ZERO-FILLED before first
 *       use (every launch re-arms it).
 * kw_dec_lm_greedy_supported(B, V, d): 1 when the shape is covered (else use kw_dec_linear + kw_greedy_step). */
int kw_dec_lm_greedy(const kw_dec_linear_args* lm, const kw_sampler_args* g, kw_stream_t stream);
size_t kw_dec_lm_greedy_workspace(int64_t B, int64_t V);
int kw_dec_lm_greedy_supported(int64_t B, int64_t V, int64_t d);

/* ---- beam search step (a10: TF/generation/utils.py:3208-3527), num_return_sequences = 1 ----------
 * Running rows are R = B * num_beams, item-major (row = b * num_beams + beam).  One step is
 * kw_beam_logprobs then kw_beam_select; both read the device cur_len and do nothing once *done != 0,
 * so the step can be replayed from a hipGraph past the end of the search. */

/* log_softmax of each row's raw f32 logits (utils.py:3380), the Whisper processors on the log-probs
 * (as kw_greedy_step, with the row's own history ids[r][0..L) ), and the row's k best processed
 * log-probs, descending, ties to the lower token id: cand_val/cand_idx [R][k], k <= 16. */
typedef struct {
  const float* logits;
  int64_t R, V;
  const uint8_t* suppress_mask;
  const int32_t* begin_suppress;
  int32_t n_begin_suppress;
  int32_t return_timestamps;
  int32_t ts_begin, no_ts_id, eos_id;
  int32_t max_initial_ts;     /* -1 = None */
  const int64_t* ids;         /* [R][ids_stride] running histories */
  int64_t ids_stride;
  const int32_t* cur_len;
  int32_t begin_index;
  int32_t k;
  float* cand_val;
  int32_t* cand_idx;
  const int32_t* done;
  void* workspace;            /* optional, zero-filled once, >= kw_beam_logprobs_workspace(R) bytes: each row
                                 over several workgroups + a last-arriver merge (NULL: one workgroup per row) */
  size_t ws_bytes;
} kw_beam_logprobs_args;

int kw_beam_logprobs(const kw_beam_logprobs_args* args, kw_stream_t stream);
size_t kw_beam_logprobs_workspace(int64_t R);

/* Selection for one step (utils.py:3077-3205, 3008-3075): top 2*num_beams continuations over
 * beams x vocab of (log-prob + running score), MaxLength / EOS criteria, the next running beams
 * (ids rows rewritten in place: parent history + token; bp rows: parent slot table + own slot),
 * the finished set (fin_seq/fin_score/fin_len/fin_flag, length_penalty, early_stopping 0 = False,
 * 1 = True, 2 = "never"), the early-stop heuristic (unsat) and, from the last item, *go (1 = the
 * reference loop continues) / *done, and *cur_len += 1.  Initial state: ids rows = prompt, bp rows =
 * own row for p < P (or bp NULL when the K/V cache is not shared), run_scores = [0, -1e9, ...] per
 * item, fin_seq = fill_id, fin_score = -1e9, fin_len = fin_flag = 0, unsat = 1, counter = go = done = 0.
 * 2 <= num_beams <= 8, max_length <= 512, fin_stride / ids_stride / bp_stride >= max_length. */
typedef struct {
  int64_t B;
  int32_t num_beams;
  int64_t V;
  const float* cand_val;
  const int32_t* cand_idx;
  int64_t* ids;
  int64_t ids_stride;
  int32_t* bp;
  int64_t bp_stride;
  float* run_scores;          /* [R] */
  int64_t* fin_seq;           /* [B][num_beams][fin_stride] */
  int64_t fin_stride;
  float* fin_score;           /* [B][num_beams] */
  int32_t* fin_len;           /* generated tokens of each finished sequence */
  int32_t* fin_flag;
  int32_t* unsat;             /* [B] */
  int32_t* cur_len;
  int32_t begin_index;        /* prompt length */
  int32_t max_length;
  int32_t eos_id;
  int32_t fill_id;            /* pad_token_id (or eos when there is none) */
  float length_penalty;
  int32_t early_stopping;
  int32_t* counter;
  int32_t* go;
  int32_t* done;
  int32_t* item_flags;        /* [B][3] scratch */
} kw_beam_select_args;

int kw_beam_select(const kw_beam_select_args* args, kw_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* KWHISPER_H */
