/* Lab-only ABI (not in libkwhisper.so): the fused decode feed-forward block, built by
 *   bash tools/lab/mlp_lab_build.sh "-DKW_LAB_MLP"   (product sources + tools/lab/lab_switches.diff)
 * and driven by tools/lab/mlp_coresident.py.  It lost to the two kw_dec_linear launches in rounds 4 and 5
 * (profiles/r05b_mlp_decomposition.txt), so the product library does not carry it. */
#pragma once
#include "../../include/kwhisper.h"
#ifdef __cplusplus
extern "C" {
#endif

/* The feed-forward block of one greedy decode step in ONE launch (bf16): the LayerNorm-fused fc1 with GELU (TF
 * modeling_whisper.py:499-501, activations.py:70-89) and fc2 with the residual add (:502-505) -- kw_dec_linear(fc1,
 * ln, gelu, bf16 C) followed by kw_dec_linear(fc2, RESID) without the kernel boundary, h and hb within f32 summation
 * order of the two launches': fc1's workgroups hand each 32-column block of the GELU output to fc2 in-launch (write-through
 * fragment tiles + one flag each) while fc2's workgroups, one per 16 output columns, already hold their weights.
 *   x: hb [M][ldx] bf16 (the residual mirror, fc1's LayerNorm input); fc1_w: packed [F][d] with gamma folded,
 *   fc1_colsum / fc1_bias: [F] f32; fc2_w: packed [d][F], fc2_bias: [d] f32; h [M][ldh] f32 (+= fc2(...)) and its
 *   bf16 mirror hb (x may be hb).  M <= 32; the shapes of kw_dec_mlp_supported() (large-v3 / kotoba-whisper:
 *   d 1280, F 5120).
 * workspace >= kw_dec_mlp_workspace(M, d, F) bytes, ZERO-FILLED before first use (every call re-arms it); its
 * status word (kw_dec_mlp_status_offset) and the fault-injection word after it work as kw_dec_qkv_self's (a
 * poll timeout writes NaN rows).  Every in-launch wait is on a workgroup dispatched before it. */
typedef struct {
  const void* x;
  int64_t ldx;
  float ln_eps;
  const float* fc1_colsum;
  const void* fc1_w;
  const float* fc1_bias;
  const void* fc2_w;
  const float* fc2_bias;
  float* h;
  void* hb;
  int64_t ldh;
  int64_t M, d, F;
  void* workspace;
  size_t ws_bytes;
} kw_dec_mlp_args;

int kw_dec_mlp(const kw_dec_mlp_args* args, kw_stream_t stream);
size_t kw_dec_mlp_workspace(int64_t M, int64_t d, int64_t F);
int kw_dec_mlp_supported(int64_t M, int64_t d, int64_t F);
size_t kw_dec_mlp_status_offset(int64_t M, int64_t d, int64_t F);

#ifdef __cplusplus
}
#endif
