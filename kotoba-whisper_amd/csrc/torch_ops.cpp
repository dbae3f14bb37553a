// PyTorch-ROCm custom ops over the kwhisper C ABI (include/kwhisper.h): torch.ops.kw.*
//
// "Torch custom ops (torch.ops.kw.*) wrap the ABI".  Each op takes device tensors plus
// plain integers, fills the ABI's argument block, and launches on torch's CURRENT HIP stream (so the
// kernels order with torch's own work and are captured by torch.cuda.graph like any torch op).  The ops
// mutate their output tensors in place (schema annotations Tensor(a!)) and return nothing; there is no
// CPU kernel and no fallback: a non-HIP tensor is rejected.  Error behaviour mirrors the ctypes binding:
// KW_EINVAL -> ValueError, any other code -> RuntimeError, both with kw_last_error()'s message.
//
// The C ABI stays the boundary beneath (libkwhisper.so, linked, not re-implemented here).
#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <cstdint>
#include <string>
#include <vector>

#include "kwhisper.h"

namespace {

using at::Tensor;
using std::optional;

void* stream_of(const Tensor& t) { return (void*)c10::hip::getCurrentHIPStream(t.device().index()).stream(); }

void check(int rc, const char* what) {
  if (rc == KW_OK) return;
  const char* msg = kw_last_error();
  TORCH_CHECK_VALUE(rc != KW_EINVAL, what, ": ", msg ? msg : "");
  TORCH_CHECK(false, what, " failed (code ", rc, "): ", msg ? msg : "");
}

void dev(const Tensor& t, const char* what) {
  TORCH_CHECK_VALUE(t.is_cuda(), what, ": kwhisper ops take device (HIP) tensors");
}
void dev(const optional<Tensor>& t, const char* what) {
  if (t.has_value()) dev(*t, what);
}

int dt_of(const Tensor& t) {
  if (t.scalar_type() == at::kFloat) return KW_DT_F32;
  if (t.scalar_type() == at::kBFloat16) return KW_DT_BF16;
  TORCH_CHECK_VALUE(false, "unsupported dtype ", t.scalar_type(), "; expected float32 or bfloat16");
}

template <typename T = void>
T* ptr(const Tensor& t, int64_t offset_elems = 0) {
  return reinterpret_cast<T*>(reinterpret_cast<char*>(t.data_ptr()) + offset_elems * t.element_size());
}
template <typename T = void>
T* optr(const optional<Tensor>& t) {
  return t.has_value() ? ptr<T>(*t) : nullptr;
}

int64_t at_(const std::vector<int64_t>& v, size_t i, const char* what) {
  TORCH_CHECK_VALUE(i < v.size(), what, ": argument list too short");
  return v[i];
}

// ---- a1 log-mel ---------------------------------------------------------------------------------------
void log_mel(const Tensor& audio, const Tensor& mel_filters, Tensor& out, Tensor& workspace) {
  dev(audio, "kw_log_mel");
  dev(mel_filters, "kw_log_mel");
  dev(out, "kw_log_mel");
  dev(workspace, "kw_log_mel");
  TORCH_CHECK_VALUE(audio.dim() == 2 && audio.scalar_type() == at::kFloat && audio.stride(1) == 1,
                    "audio must be a (B, n_samples) float32 tensor with unit inner stride");
  c10::DeviceGuard g(audio.device());
  check(kw_log_mel(ptr<const float>(audio), audio.size(0), audio.size(1), audio.stride(0), ptr<const float>(mel_filters),
                   (int)mel_filters.size(1), ptr<float>(out), ptr(workspace), stream_of(audio)),
        "kw_log_mel");
}

void mel_to_time_major(const Tensor& mel, int64_t c_pad, Tensor& out) {
  dev(mel, "kw_mel_to_time_major");
  dev(out, "kw_mel_to_time_major");
  TORCH_CHECK_VALUE(mel.dim() == 3 && mel.is_contiguous() && mel.scalar_type() == at::kFloat,
                    "mel must be a contiguous (B, C, T) float32 tensor");
  c10::DeviceGuard g(mel.device());
  check(kw_mel_to_time_major(ptr<const float>(mel), mel.size(0), mel.size(1), mel.size(2), c_pad, ptr(out), dt_of(out),
                             stream_of(mel)),
        "kw_mel_to_time_major");
}

// ---- linear / conv-as-GEMM ----------------------------------------------------------------------------
// geo = [a_offset, lda, a_rows_per_batch, a_batch_stride, c_offset, ldc, c_rows_per_batch, c_batch_stride,
//        M, N, K, epilogue, gelu, scale_cols, row_add_period, hs_seq, hs_heads, hs_head_dim]
void gemm(const Tensor& A, const Tensor& W, const optional<Tensor>& bias, Tensor& C, const optional<Tensor>& row_add,
          std::vector<int64_t> geo, double scale, int64_t dtype) {
  const char* w = "kw_gemm";
  dev(A, w), dev(W, w), dev(bias, w), dev(C, w), dev(row_add, w);
  TORCH_CHECK_VALUE(geo.size() == 18, "kw_gemm: geo must hold 18 integers");
  kw_gemm_args a{};
  a.dtype = dtype >= 0 ? (int)dtype : dt_of(W);
  a.c_dtype = dt_of(C);
  a.A = ptr(A, geo[0]);
  a.lda = geo[1], a.a_rows_per_batch = geo[2], a.a_batch_stride = geo[3];
  a.W = ptr(W);
  a.bias = optr<const float>(bias);
  a.C = ptr(C, geo[4]);
  a.ldc = geo[5], a.c_rows_per_batch = geo[6], a.c_batch_stride = geo[7];
  a.M = geo[8], a.N = geo[9], a.K = geo[10];
  a.epilogue = (int)geo[11];
  a.gelu = (int)geo[12];
  a.scale = (float)scale;
  a.scale_cols = geo[13];
  a.row_add = optr<const float>(row_add);
  a.row_add_period = geo[14];
  a.hs_seq = geo[15], a.hs_heads = geo[16], a.hs_head_dim = geo[17];
  c10::DeviceGuard g(W.device());
  check(kw_gemm(&a, stream_of(W)), w);
}

// ---- decode-step linear over packed weights -----------------------------------------------------------
// geo = [x_offset, ldx, ln, c_offset, ldc, gelu, scale_cols, resid_row0, ldh, M, N, K]
void dec_linear(const Tensor& x, const Tensor& W, const optional<Tensor>& bias, const optional<Tensor>& ln_colsum,
                optional<Tensor> C, optional<Tensor> h, optional<Tensor> hb, Tensor& workspace,
                std::vector<int64_t> geo, double ln_eps, double scale) {
  const char* w = "kw_dec_linear";
  dev(x, w), dev(W, w), dev(bias, w), dev(ln_colsum, w), dev(C, w), dev(h, w), dev(hb, w), dev(workspace, w);
  TORCH_CHECK_VALUE(geo.size() == 12, "kw_dec_linear: geo must hold 12 integers");
  TORCH_CHECK_VALUE(x.scalar_type() == at::kBFloat16 && W.scalar_type() == at::kBFloat16,
                    "kw_dec_linear takes bf16 activations and packed bf16 weights");
  kw_dec_linear_args a{};
  a.x = ptr(x, geo[0]);
  a.ldx = geo[1];
  a.ln = (int)geo[2];
  a.ln_eps = (float)ln_eps;
  a.ln_colsum = optr<const float>(ln_colsum);
  a.W = ptr(W);
  a.bias = optr<const float>(bias);
  if (h.has_value()) {
    TORCH_CHECK_VALUE(hb.has_value() && h->scalar_type() == at::kFloat && hb->scalar_type() == at::kBFloat16,
                      "RESID needs an f32 residual and a bf16 mirror");
    a.epilogue = KW_EPI_RESID;
    a.h = ptr<float>(*h, geo[7] * geo[8]);
    a.hb = ptr(*hb, geo[7] * geo[8]);
    a.ldh = geo[8];
  } else {
    TORCH_CHECK_VALUE(C.has_value(), "STORE needs C");
    a.epilogue = KW_EPI_STORE;
    a.C = ptr(*C, geo[3]);
    a.ldc = geo[4];
    a.c_dtype = dt_of(*C);
  }
  a.gelu = (int)geo[5];
  a.scale = (float)scale;
  a.scale_cols = geo[6];
  a.M = geo[9], a.N = geo[10], a.K = geo[11];
  a.workspace = ptr(workspace);
  a.ws_bytes = (size_t)workspace.numel() * workspace.element_size();
  c10::DeviceGuard g(W.device());
  check(kw_dec_linear(&a, stream_of(W)), w);
}

void pack_weight(const Tensor& W, Tensor& out) {
  dev(W, "kw_pack_weight");
  dev(out, "kw_pack_weight");
  TORCH_CHECK_VALUE(W.dim() == 2 && W.is_contiguous() && W.scalar_type() == at::kBFloat16,
                    "pack_weight expects a contiguous 2-D bfloat16 tensor");
  TORCH_CHECK_VALUE((size_t)out.numel() * out.element_size() >= kw_packed_weight_bytes(W.size(0), W.size(1)),
                    "pack_weight: output too small");
  c10::DeviceGuard g(W.device());
  check(kw_pack_weight(ptr(W), W.size(0), W.size(1), ptr(out), stream_of(W)), "kw_pack_weight");
}

// ---- LayerNorm (residual stream f32 or bf16) ----------------------------------------------------------
void layernorm(Tensor& x, const Tensor& gamma, const Tensor& beta, double eps, Tensor& y, const optional<Tensor>& delta) {
  const char* w = "kw_layernorm";
  dev(x, w), dev(gamma, w), dev(beta, w), dev(y, w), dev(delta, w);
  TORCH_CHECK_VALUE(x.is_contiguous() && (x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16),
                    "layernorm input must be contiguous float32 or bfloat16");
  const int64_t dim = x.size(-1), rows = x.numel() / dim;
  c10::DeviceGuard g(x.device());
  if (x.scalar_type() == at::kBFloat16)
    check(kw_layernorm_bf16res(ptr(x), rows, dim, ptr<const float>(gamma), ptr<const float>(beta), (float)eps, ptr(y),
                               dt_of(y), optr<const void>(delta), stream_of(x)),
          "kw_layernorm_bf16res");
  else
    check(kw_layernorm(ptr<float>(x), rows, dim, ptr<const float>(gamma), ptr<const float>(beta), (float)eps, ptr(y),
                       dt_of(y), optr<const void>(delta), stream_of(x)),
          w);
}

// ---- attention ----------------------------------------------------------------------------------------
void attention(const Tensor& qkv, int64_t B, int64_t H, int64_t T, int64_t hd, Tensor& out, int64_t flags) {
  dev(qkv, "kw_attention");
  dev(out, "kw_attention");
  c10::DeviceGuard g(qkv.device());
  check(kw_attention(dt_of(qkv) | (int)flags, ptr(qkv), B, H, T, hd, ptr(out), stream_of(qkv)), "kw_attention");
}

void embed(const Tensor& ids, int64_t B, int64_t q_len, const Tensor& cur_len, const Tensor& tok_emb,
           const Tensor& pos_emb, Tensor& h, optional<Tensor> hb) {
  const char* w = "kw_embed";
  dev(ids, w), dev(cur_len, w), dev(tok_emb, w), dev(pos_emb, w), dev(h, w), dev(hb, w);
  c10::DeviceGuard g(ids.device());
  check(kw_embed(dt_of(tok_emb), ptr<const int64_t>(ids), ids.stride(0), B, q_len, ptr<const int32_t>(cur_len),
                 ptr(tok_emb), ptr(pos_emb), tok_emb.size(1), ptr<float>(h), optr<void>(hb), stream_of(ids)),
        w);
}

void self_attn_step(const Tensor& qkv, int64_t B, int64_t q_len, int64_t H, int64_t hd, Tensor& k_cache,
                    Tensor& v_cache, int64_t t_max, const Tensor& cur_len, Tensor& out, optional<Tensor> workspace,
                    const optional<Tensor>& bp) {
  const char* w = "kw_self_attn_step";
  dev(qkv, w), dev(k_cache, w), dev(v_cache, w), dev(cur_len, w), dev(out, w), dev(workspace, w), dev(bp, w);
  const size_t nb = workspace.has_value() ? (size_t)workspace->numel() * workspace->element_size() : 0;
  c10::DeviceGuard g(qkv.device());
  check(kw_self_attn_step(dt_of(qkv), ptr(qkv), B, q_len, H, hd, ptr(k_cache), ptr(v_cache), t_max,
                          ptr<const int32_t>(cur_len), optr<const int32_t>(bp), bp.has_value() ? bp->stride(0) : 0,
                          ptr(out), optr<void>(workspace), nb, stream_of(qkv)),
        w);
}

// ---- fused decode cross-attention query + step -----------------------------------------------------------
// dims = [ldx, M, d, H, S]
void dec_xq_cross(const Tensor& x, const Tensor& W, const optional<Tensor>& bias, const Tensor& ln_colsum,
                  const Tensor& k, const Tensor& v, Tensor& out, Tensor& workspace, std::vector<int64_t> dims,
                  double ln_eps, double scale) {
  const char* w = "kw_dec_xq_cross";
  dev(x, w), dev(W, w), dev(bias, w), dev(ln_colsum, w), dev(k, w), dev(v, w), dev(out, w), dev(workspace, w);
  TORCH_CHECK_VALUE(dims.size() == 5, "kw_dec_xq_cross: dims must hold 5 integers");
  TORCH_CHECK_VALUE(x.scalar_type() == at::kBFloat16 && W.scalar_type() == at::kBFloat16 &&
                        out.scalar_type() == at::kBFloat16 && k.scalar_type() == at::kBFloat16 &&
                        v.scalar_type() == at::kBFloat16,
                    "kw_dec_xq_cross takes bf16 activations, packed bf16 weights, bf16 K / V and output");
  kw_dec_xq_cross_args a{};
  a.x = ptr(x);
  a.ldx = dims[0];
  a.ln_eps = (float)ln_eps;
  a.ln_colsum = ptr<const float>(ln_colsum);
  a.W = ptr(W);
  a.bias = optr<const float>(bias);
  a.scale = (float)scale;
  a.M = dims[1], a.d = dims[2], a.H = dims[3];
  a.k = ptr(k);
  a.v = ptr(v);
  a.S = dims[4];
  a.out = ptr(out);
  a.workspace = ptr(workspace);
  a.ws_bytes = (size_t)workspace.numel() * workspace.element_size();
  c10::DeviceGuard g(x.device());
  check(kw_dec_xq_cross(&a, stream_of(x)), w);
}

// ---- fused decode self-attention block (LayerNorm-fused QKV projection + self-attention step) ------------
// dims = [ldx, M, d, H, t_max]
void dec_qkv_self(const Tensor& x, const Tensor& W, const optional<Tensor>& bias, const Tensor& ln_colsum,
                  Tensor& k_cache, Tensor& v_cache, const Tensor& cur_len, Tensor& out, Tensor& workspace,
                  std::vector<int64_t> dims, double ln_eps, double scale) {
  const char* w = "kw_dec_qkv_self";
  dev(x, w), dev(W, w), dev(bias, w), dev(ln_colsum, w), dev(k_cache, w), dev(v_cache, w), dev(cur_len, w),
      dev(out, w), dev(workspace, w);
  TORCH_CHECK_VALUE(dims.size() == 5, "kw_dec_qkv_self: dims must hold 5 integers");
  TORCH_CHECK_VALUE(x.scalar_type() == at::kBFloat16 && W.scalar_type() == at::kBFloat16 &&
                        out.scalar_type() == at::kBFloat16 && k_cache.scalar_type() == at::kBFloat16,
                    "kw_dec_qkv_self takes bf16 activations, packed bf16 weights, bf16 caches and output");
  kw_dec_qkv_self_args a{};
  a.x = ptr(x);
  a.ldx = dims[0];
  a.ln_eps = (float)ln_eps;
  a.ln_colsum = ptr<const float>(ln_colsum);
  a.W = ptr(W);
  a.bias = optr<const float>(bias);
  a.scale = (float)scale;
  a.M = dims[1], a.d = dims[2], a.H = dims[3];
  a.k_cache = ptr(k_cache);
  a.v_cache = ptr(v_cache);
  a.t_max = dims[4];
  a.cur_len = ptr<const int32_t>(cur_len);
  a.out = ptr(out);
  a.workspace = ptr(workspace);
  a.ws_bytes = (size_t)workspace.numel() * workspace.element_size();
  c10::DeviceGuard g(x.device());
  check(kw_dec_qkv_self(&a, stream_of(x)), w);
}

void cross_attn_step(const Tensor& q, int64_t B, int64_t q_len, int64_t H, int64_t hd, const Tensor& k, const Tensor& v,
                     int64_t S, Tensor& out, Tensor& workspace) {
  const char* w = "kw_cross_attn_step";
  dev(q, w), dev(k, w), dev(v, w), dev(out, w), dev(workspace, w);
  c10::DeviceGuard g(q.device());
  check(kw_cross_attn_step(dt_of(q), ptr(q), B, q_len, H, hd, ptr(k), ptr(v), S, ptr(out), ptr(workspace),
                           (size_t)workspace.numel() * workspace.element_size(), stream_of(q)),
        w);
}

// ---- greedy step (processors + argmax + stopping) -----------------------------------------------------
// cfg = [return_timestamps, ts_begin, no_ts_id, eos_id, pad_id, max_initial_ts, max_length, begin_index]
void greedy_step(Tensor& logits, const Tensor& suppress_mask, const optional<Tensor>& begin_suppress, Tensor& ids,
                 Tensor& cur_len, Tensor& unfinished, Tensor& counter, Tensor& n_unfinished, optional<Tensor> scores_out,
                 optional<Tensor> workspace, std::vector<int64_t> cfg) {
  const char* w = "kw_greedy_step";
  dev(logits, w), dev(suppress_mask, w), dev(begin_suppress, w), dev(ids, w), dev(cur_len, w), dev(unfinished, w);
  dev(counter, w), dev(n_unfinished, w), dev(scores_out, w), dev(workspace, w);
  TORCH_CHECK_VALUE(cfg.size() == 8, "kw_greedy_step: cfg must hold 8 integers");
  kw_sampler_args a{};
  a.logits = ptr<float>(logits);
  a.B = logits.size(0), a.V = logits.size(1);
  a.suppress_mask = ptr<const uint8_t>(suppress_mask);
  a.begin_suppress = optr<const int32_t>(begin_suppress);
  a.n_begin_suppress = begin_suppress.has_value() ? (int32_t)begin_suppress->numel() : 0;
  a.return_timestamps = (int32_t)cfg[0];
  a.ts_begin = (int32_t)cfg[1], a.no_ts_id = (int32_t)cfg[2], a.eos_id = (int32_t)cfg[3], a.pad_id = (int32_t)cfg[4];
  a.max_initial_ts = (int32_t)cfg[5];
  a.ids = ptr<int64_t>(ids);
  a.ids_stride = ids.stride(0);
  a.cur_len = ptr<int32_t>(cur_len);
  a.max_length = (int32_t)cfg[6], a.begin_index = (int32_t)cfg[7];
  a.unfinished = ptr<int32_t>(unfinished);
  a.counter = ptr<int32_t>(counter);
  a.n_unfinished = ptr<int32_t>(n_unfinished);
  a.scores_out = optr<float>(scores_out);
  a.workspace = optr<void>(workspace);
  a.ws_bytes = workspace.has_value() ? (size_t)workspace->numel() * workspace->element_size() : 0;
  c10::DeviceGuard g(logits.device());
  check(kw_greedy_step(&a, stream_of(logits)), w);
}

// ---- LM head + greedy step in one launch (no timestamps) ------------------------------------------------
// lm_geo = [x_offset, ldx, M, N, K]; cfg = [eos_id, pad_id, max_length, begin_index]
void dec_lm_greedy(const Tensor& x, const Tensor& W, const optional<Tensor>& bias, const Tensor& ln_colsum,
                   optional<Tensor> logits, const Tensor& suppress_mask, const optional<Tensor>& begin_suppress,
                   Tensor& ids, Tensor& cur_len, Tensor& unfinished, Tensor& n_unfinished, Tensor& workspace,
                   std::vector<int64_t> lm_geo, double ln_eps, std::vector<int64_t> cfg) {
  const char* w = "kw_dec_lm_greedy";
  dev(x, w), dev(W, w), dev(bias, w), dev(ln_colsum, w), dev(logits, w), dev(suppress_mask, w), dev(begin_suppress, w);
  dev(ids, w), dev(cur_len, w), dev(unfinished, w), dev(n_unfinished, w), dev(workspace, w);
  TORCH_CHECK_VALUE(lm_geo.size() == 5 && cfg.size() == 4, "kw_dec_lm_greedy: lm_geo holds 5, cfg 4 integers");
  TORCH_CHECK_VALUE(x.scalar_type() == at::kBFloat16 && W.scalar_type() == at::kBFloat16,
                    "kw_dec_lm_greedy takes bf16 activations and packed bf16 weights");
  kw_dec_linear_args a{};
  a.x = ptr(x, lm_geo[0]);
  a.ldx = lm_geo[1];
  a.ln = 1;
  a.ln_eps = (float)ln_eps;
  a.ln_colsum = ptr<const float>(ln_colsum);
  a.W = ptr(W);
  a.bias = optr<const float>(bias);
  a.epilogue = KW_EPI_STORE;
  a.C = optr<void>(logits);
  a.ldc = logits.has_value() ? logits->stride(0) : lm_geo[3];
  a.c_dtype = KW_DT_F32;
  a.scale = 1.f;
  a.M = lm_geo[2], a.N = lm_geo[3], a.K = lm_geo[4];
  kw_sampler_args g{};
  g.B = a.M, g.V = a.N;
  g.suppress_mask = ptr<const uint8_t>(suppress_mask);
  g.begin_suppress = optr<const int32_t>(begin_suppress);
  g.n_begin_suppress = begin_suppress.has_value() ? (int32_t)begin_suppress->numel() : 0;
  g.eos_id = (int32_t)cfg[0], g.pad_id = (int32_t)cfg[1], g.max_length = (int32_t)cfg[2], g.begin_index = (int32_t)cfg[3];
  g.max_initial_ts = -1;
  g.ids = ptr<int64_t>(ids);
  g.ids_stride = ids.stride(0);
  g.cur_len = ptr<int32_t>(cur_len);
  g.unfinished = ptr<int32_t>(unfinished);
  g.n_unfinished = ptr<int32_t>(n_unfinished);
  g.workspace = ptr(workspace);
  g.ws_bytes = (size_t)workspace.numel() * workspace.element_size();
  c10::DeviceGuard dg(x.device());
  check(kw_dec_lm_greedy(&a, &g, stream_of(x)), w);
}

// ---- beam search step ---------------------------------------------------------------------------------
// cfg = [return_timestamps, ts_begin, no_ts_id, eos_id, max_initial_ts, begin_index, k]
void beam_logprobs(const Tensor& logits, const Tensor& suppress_mask, const optional<Tensor>& begin_suppress,
                   const Tensor& ids, const Tensor& cur_len, Tensor& cand_val, Tensor& cand_idx, const Tensor& done,
                   optional<Tensor> workspace, std::vector<int64_t> cfg) {
  const char* w = "kw_beam_logprobs";
  dev(logits, w), dev(suppress_mask, w), dev(begin_suppress, w), dev(ids, w), dev(cur_len, w);
  dev(cand_val, w), dev(cand_idx, w), dev(done, w), dev(workspace, w);
  TORCH_CHECK_VALUE(cfg.size() == 7, "kw_beam_logprobs: cfg must hold 7 integers");
  kw_beam_logprobs_args a{};
  a.logits = ptr<const float>(logits);
  a.R = logits.size(0), a.V = logits.size(1);
  a.suppress_mask = ptr<const uint8_t>(suppress_mask);
  a.begin_suppress = optr<const int32_t>(begin_suppress);
  a.n_begin_suppress = begin_suppress.has_value() ? (int32_t)begin_suppress->numel() : 0;
  a.return_timestamps = (int32_t)cfg[0];
  a.ts_begin = (int32_t)cfg[1], a.no_ts_id = (int32_t)cfg[2], a.eos_id = (int32_t)cfg[3];
  a.max_initial_ts = (int32_t)cfg[4];
  a.ids = ptr<const int64_t>(ids);
  a.ids_stride = ids.stride(0);
  a.cur_len = ptr<const int32_t>(cur_len);
  a.begin_index = (int32_t)cfg[5];
  a.k = (int32_t)cfg[6];
  a.cand_val = ptr<float>(cand_val);
  a.cand_idx = ptr<int32_t>(cand_idx);
  a.done = ptr<const int32_t>(done);
  a.workspace = optr<void>(workspace);
  a.ws_bytes = workspace.has_value() ? (size_t)workspace->numel() * workspace->element_size() : 0;
  c10::DeviceGuard g(logits.device());
  check(kw_beam_logprobs(&a, stream_of(logits)), w);
}

// cfg = [B, num_beams, V, begin_index, max_length, eos_id, fill_id, early_stopping]
void beam_select(const Tensor& cand_val, const Tensor& cand_idx, Tensor& ids, optional<Tensor> bp, Tensor& run_scores,
                 Tensor& fin_seq, Tensor& fin_score, Tensor& fin_len, Tensor& fin_flag, Tensor& unsat, Tensor& cur_len,
                 Tensor& counter, Tensor& go, Tensor& done, Tensor& item_flags, std::vector<int64_t> cfg,
                 double length_penalty) {
  const char* w = "kw_beam_select";
  dev(cand_val, w), dev(cand_idx, w), dev(ids, w), dev(bp, w), dev(run_scores, w), dev(fin_seq, w), dev(fin_score, w);
  dev(fin_len, w), dev(fin_flag, w), dev(unsat, w), dev(cur_len, w), dev(counter, w), dev(go, w), dev(done, w);
  dev(item_flags, w);
  TORCH_CHECK_VALUE(cfg.size() == 8, "kw_beam_select: cfg must hold 8 integers");
  kw_beam_select_args a{};
  a.B = cfg[0], a.num_beams = (int32_t)cfg[1], a.V = cfg[2];
  a.cand_val = ptr<const float>(cand_val);
  a.cand_idx = ptr<const int32_t>(cand_idx);
  a.ids = ptr<int64_t>(ids);
  a.ids_stride = ids.stride(0);
  a.bp = optr<int32_t>(bp);
  a.bp_stride = bp.has_value() ? bp->stride(0) : 0;
  a.run_scores = ptr<float>(run_scores);
  a.fin_seq = ptr<int64_t>(fin_seq);
  a.fin_stride = fin_seq.size(-1);
  a.fin_score = ptr<float>(fin_score);
  a.fin_len = ptr<int32_t>(fin_len);
  a.fin_flag = ptr<int32_t>(fin_flag);
  a.unsat = ptr<int32_t>(unsat);
  a.cur_len = ptr<int32_t>(cur_len);
  a.begin_index = (int32_t)cfg[3], a.max_length = (int32_t)cfg[4], a.eos_id = (int32_t)cfg[5];
  a.fill_id = (int32_t)cfg[6];
  a.length_penalty = (float)length_penalty;
  a.early_stopping = (int32_t)cfg[7];
  a.counter = ptr<int32_t>(counter);
  a.go = ptr<int32_t>(go);
  a.done = ptr<int32_t>(done);
  a.item_flags = ptr<int32_t>(item_flags);
  c10::DeviceGuard g(ids.device());
  check(kw_beam_select(&a, stream_of(ids)), w);
}

// ---- workspace / packing sizes (host queries) ---------------------------------------------------------
int64_t workspace_bytes(std::string kind, std::vector<int64_t> d) {
  auto n = [&](size_t i) { return at_(d, i, "kw::workspace_bytes"); };
  if (kind == "dec_linear") return (int64_t)kw_dec_linear_workspace_bytes(n(0), n(1));
  if (kind == "packed_weight") return (int64_t)kw_packed_weight_bytes(n(0), n(1));
  if (kind == "self_attn") return (int64_t)kw_self_attn_workspace(n(0), n(1), n(2));
  if (kind == "cross_attn") return (int64_t)kw_cross_attn_workspace(n(0), n(1), n(2), n(3), n(4));
  if (kind == "greedy_step") return (int64_t)kw_greedy_step_workspace(n(0));
  if (kind == "lm_greedy") return (int64_t)kw_dec_lm_greedy_workspace(n(0), n(1));
  if (kind == "qkv_self") return (int64_t)kw_dec_qkv_self_workspace(n(0), n(1));
  if (kind == "xq_cross") return (int64_t)kw_dec_xq_cross_workspace(n(0), n(1), n(2), n(3));
  if (kind == "beam_logprobs") return (int64_t)kw_beam_logprobs_workspace(n(0));
  // byte offsets of the hand-off status words inside those workspaces (include/kwhisper.h)
  if (kind == "qkv_self_status") return (int64_t)kw_dec_qkv_self_status_offset(n(0), n(1));
  if (kind == "xq_cross_status") return (int64_t)kw_dec_xq_cross_status_offset(n(0), n(1), n(2), n(3));
  if (kind == "cross_attn_status") return (int64_t)kw_cross_attn_status_offset(n(0), n(1), n(2), n(3), n(4));
  TORCH_CHECK_VALUE(false, "kw::workspace_bytes: unknown kind ", kind);
}

int64_t version() { return kw_version(); }

}  // namespace

TORCH_LIBRARY(kw, m) {
  m.def("version() -> int", &version);
  m.def("workspace_bytes(str kind, int[] dims) -> int", &workspace_bytes);
  m.def("log_mel(Tensor audio, Tensor mel_filters, Tensor(a!) out, Tensor(b!) workspace) -> ()");
  m.def("mel_to_time_major(Tensor mel, int c_pad, Tensor(a!) out) -> ()");
  m.def("gemm(Tensor A, Tensor W, Tensor? bias, Tensor(a!) C, Tensor? row_add, int[] geo, float scale, int dtype) -> ()");
  m.def("dec_linear(Tensor x, Tensor W, Tensor? bias, Tensor? ln_colsum, Tensor(a!)? C, Tensor(b!)? h, "
        "Tensor(c!)? hb, Tensor(d!) workspace, int[] geo, float ln_eps, float scale) -> ()");
  m.def("pack_weight(Tensor W, Tensor(a!) out) -> ()");
  m.def("layernorm(Tensor(a!) x, Tensor gamma, Tensor beta, float eps, Tensor(b!) y, Tensor? delta) -> ()");
  m.def("attention(Tensor qkv, int B, int H, int T, int hd, Tensor(a!) out, int flags=0) -> ()");
  m.def("embed(Tensor ids, int B, int q_len, Tensor cur_len, Tensor tok_emb, Tensor pos_emb, Tensor(a!) h, "
        "Tensor(b!)? hb) -> ()");
  m.def("self_attn_step(Tensor qkv, int B, int q_len, int H, int hd, Tensor(a!) k_cache, Tensor(b!) v_cache, "
        "int t_max, Tensor cur_len, Tensor(c!) out, Tensor(d!)? workspace, Tensor? bp) -> ()");
  m.def("dec_qkv_self(Tensor x, Tensor W, Tensor? bias, Tensor ln_colsum, Tensor(a!) k_cache, Tensor(b!) v_cache, "
        "Tensor cur_len, Tensor(c!) out, Tensor(d!) workspace, int[] dims, float ln_eps, float scale) -> ()");
  m.def("dec_xq_cross(Tensor x, Tensor W, Tensor? bias, Tensor ln_colsum, Tensor k, Tensor v, Tensor(a!) out, "
        "Tensor(b!) workspace, int[] dims, float ln_eps, float scale) -> ()");
  m.def("cross_attn_step(Tensor q, int B, int q_len, int H, int hd, Tensor k, Tensor v, int S, Tensor(a!) out, "
        "Tensor(b!) workspace) -> ()");
  m.def("greedy_step(Tensor(a!) logits, Tensor suppress_mask, Tensor? begin_suppress, Tensor(b!) ids, "
        "Tensor(c!) cur_len, Tensor(d!) unfinished, Tensor(e!) counter, Tensor(f!) n_unfinished, "
        "Tensor(g!)? scores_out, Tensor(h!)? workspace, int[] cfg) -> ()");
  m.def("dec_lm_greedy(Tensor x, Tensor W, Tensor? bias, Tensor ln_colsum, Tensor(a!)? logits, Tensor suppress_mask, "
        "Tensor? begin_suppress, Tensor(b!) ids, Tensor(c!) cur_len, Tensor(d!) unfinished, Tensor(e!) n_unfinished, "
        "Tensor(f!) workspace, int[] lm_geo, float ln_eps, int[] cfg) -> ()");
  m.def("beam_logprobs(Tensor logits, Tensor suppress_mask, Tensor? begin_suppress, Tensor ids, Tensor cur_len, "
        "Tensor(a!) cand_val, Tensor(b!) cand_idx, Tensor done, Tensor(c!)? workspace, int[] cfg) -> ()");
  m.def("beam_select(Tensor cand_val, Tensor cand_idx, Tensor(a!) ids, Tensor(b!)? bp, Tensor(c!) run_scores, "
        "Tensor(d!) fin_seq, Tensor(e!) fin_score, Tensor(f!) fin_len, Tensor(g!) fin_flag, Tensor(h!) unsat, "
        "Tensor(i!) cur_len, Tensor(j!) counter, Tensor(k!) go, Tensor(l!) done, Tensor(m!) item_flags, int[] cfg, "
        "float length_penalty) -> ()");
}

TORCH_LIBRARY_IMPL(kw, CUDA, m) {
  m.impl("log_mel", &log_mel);
  m.impl("mel_to_time_major", &mel_to_time_major);
  m.impl("gemm", &gemm);
  m.impl("dec_linear", &dec_linear);
  m.impl("pack_weight", &pack_weight);
  m.impl("layernorm", &layernorm);
  m.impl("attention", &attention);
  m.impl("embed", &embed);
  m.impl("self_attn_step", &self_attn_step);
  m.impl("cross_attn_step", &cross_attn_step);
  m.impl("dec_qkv_self", &dec_qkv_self);
  m.impl("dec_xq_cross", &dec_xq_cross);
  m.impl("greedy_step", &greedy_step);
  m.impl("dec_lm_greedy", &dec_lm_greedy);
  m.impl("beam_logprobs", &beam_logprobs);
  m.impl("beam_select", &beam_select);
}
