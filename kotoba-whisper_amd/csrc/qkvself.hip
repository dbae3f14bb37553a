// The decoder self-attention block of one greedy decode step in ONE launch (bf16 engine, gfx950):
// the LayerNorm-fused QKV projection (TF/models/whisper/modeling_whisper.py:446 self_attn_layer_norm,
// :469-471 q/k/v with q * head_dim^-0.5 :309) and the self-attention step over the static cache with the
// new key/value appended (:469-480, TF/cache_utils.py:127-145, TF/integrations/sdpa_attention.py:79-166) --
// what kw_dec_linear(qkv) followed by kw_self_attn_step computes in two launches: the projection bitwise the
// same (so the K/V caches are), the attention within bf16 rounding (its keys are summed in another grouping).
//
//  * workgroups [0, n_lin): the projection, 16 columns each -- dec_linear_kernel<5, 1, LN, STORE, bf16>'s
//    arithmetic on 4 waves (decproj.h: its 8 waves as virtual waves, reduced in the same order), the bf16
//    results handed over as 8-byte {bf16 x 2, tag} granules [M][3d/2] instead of stored;
//  * workgroups [n_lin, n_lin + M H / 2): two (row, head) pairs each, two waves per pair.  A pair's first 128
//    cached K/V rows are loaded at launch -- while the projection runs, where the unfused step loads them
//    only after a kernel boundary -- and rows 128..255 (L = *cur_len <= 256) right after; it polls its 96
//    granules (the q, k, v of its head) and re-arms them (tag 0: each granule has exactly one consumer),
//    appends k, v at position L - 1 and attends with attention.hip's bf16 row arithmetic (wave_row_bf16 with
//    16 key slots per pass, an online exp2 merge of the two passes, then of the two waves).  At 256 threads
//    and <= 3 workgroups per CU, all n_lin + M H / 2 <= 12 H + 16 H workgroups of large-v3 are resident in one
//    round on 256 CUs.
//
// Deadlock freedom: the projection workgroups wait for nothing and lead the dispatch order; a pair waits only
// for them, i.e. for work dispatched before it -- resident or finished, whatever else shares the GPU (no
// co-residency assumption).  Polls are bounded: a timeout sets the error word and writes NaN (loud).
#include "attn_common.h"
#include "decproj.h"

// development hook (tools/lab/qkv_stamps.hip defines it to record s_memrealtime per workgroup phase); no-op here
#ifndef KW_QS_STAMP
#define KW_QS_STAMP(slot)
#endif

namespace {

constexpr int QS_SPIN_LIMIT = 1 << 22;
constexpr int QS_PAIRS = 2;      // (row, head) pairs per attention workgroup, two waves each
constexpr int QS_MAX_LEN = 256;  // key positions per step: two 128-key passes

struct QSP {
  const bf16_t* x;
  int64_t ldx;
  float ln_eps;
  const float* ln_colsum;
  const bf16x8* W;
  const float* bias;
  float scale;
  int M, d, H, n_lin;
  bf16_t* kc;
  bf16_t* vc;
  int t_max;
  const int32_t* cur_len;
  unsigned long long* gran;  // [M][3d/2]
  int* err;
  bf16_t* out;
};

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void qkv_self_kernel(QSP p) {
  __shared__ __attribute__((aligned(16))) char scratch[PROJ_SCRATCH];  // projection workgroups
  __shared__ float ared[QS_PAIRS][2][64];
  __shared__ float astat[QS_PAIRS][4];
  __shared__ uint32_t stage[QS_PAIRS][96];
  const int d = p.d, H = p.H, M = p.M;
  if ((int)blockIdx.x < p.n_lin) {
    proj_publish_granules<true>(ProjArgs{p.x, p.ldx, M, d, 3 * d, p.ln_eps, p.ln_colsum, p.W, p.bias, p.scale, d, p.err + 1},
                          blockIdx.x, scratch, p.gran);
    return;
  }
  KW_QS_STAMP(4);
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform (scalar branches)
  const int ps = wave >> 1, pw = wave & 1, ptid = tid & 127;  // pair slot (2 waves each), wave within it
  const int L = *p.cur_len;  // positions [0, L - 1) cached, L - 1 new
  const bool len_ok = L >= 1 && L <= QS_MAX_LEN && L <= p.t_max;
  const int Lc = len_ok ? L : 1;
  const int p0 = Lc - 1;

  // ---- 1. this slot's pair: its first 128 cached K/V rows in flight before anything else (rows past L - 1
  //         clamped; the row at L - 1 is replaced by the new key / value below).  Lane (slot, sub) holds 16 B of
  //         the rows 128 pass + slot + 16 j, slot in [0, 16) across the pair's two waves.
  const int pair = ((int)blockIdx.x - p.n_lin) * QS_PAIRS + ps;
  const bool has_pair = pair < M * H;  // wave-uniform
  const int b = has_pair ? pair / H : 0, h = has_pair ? pair - (pair / H) * H : 0;
  const int sub = lane & 7, slot = pw * 8 + (lane >> 3);
  bf16_t* kb = p.kc + ((int64_t)b * H + h) * p.t_max * HD;
  bf16_t* vb = p.vc + ((int64_t)b * H + h) * p.t_max * HD;
  const int nj0 = min((Lc + 15) >> 4, 8), nj1 = max(min((Lc - 128 + 15) >> 4, 8), 0);
  u32x4 kr[8], vr[8];
  if (has_pair) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (j < nj0) kr[j] = ld_row8<bf16_t>(kb + (int64_t)min(slot + 16 * j, p0) * HD + sub * 8).u[0];
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (j < nj0) vr[j] = ld_row8<bf16_t>(vb + (int64_t)min(slot + 16 * j, p0) * HD + sub * 8).u[0];
  }

  // ---- 2. the pair's q, k, v granules (one poller per granule, re-armed after), then the softmax over the
  //         first 128 positions and, for L > 128, an online merge of positions 128..255 (loaded after the first
  //         pass: steps past 128 are outside the bench's 128-token decode)
  if (has_pair && ptid < 96) {
    const int part = ptid >> 5, c = ptid & 31;  // part 0 q, 1 k, 2 v; c = column pair within the head
    unsigned long long* g = p.gran + (int64_t)b * (3 * d / 2) + part * (d / 2) + h * 32 + c;
    unsigned long long x = 0;
    int it = 0;
    for (;; ++it) {
      x = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((x >> 32) == 1ull || it >= QS_SPIN_LIMIT) break;
      __builtin_amdgcn_s_sleep(KW_POLL_SLEEP);
    }
    if ((x >> 32) != 1ull || !len_ok) {
      x = 0x7fc07fc0ull;  // bf16 NaN pair: the failure propagates to the output
      __hip_atomic_store(p.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    stage[ps][ptid] = (uint32_t)x;
    __hip_atomic_store(g, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm (single consumer)
  }
  __syncthreads();
  KW_QS_STAMP(5);
  if (has_pair) {
    const uint32_t* st = stage[ps];
    const u32x4 qraw = {st[sub * 4], st[sub * 4 + 1], st[sub * 4 + 2], st[sub * 4 + 3]};
    const u32x4 knew = {st[32 + sub * 4], st[32 + sub * 4 + 1], st[32 + sub * 4 + 2], st[32 + sub * 4 + 3]};
    const u32x4 vnew = {st[64 + sub * 4], st[64 + sub * 4 + 1], st[64 + sub * 4 + 2], st[64 + sub * 4 + 3]};
    float ql[8];
    {
      Row8<bf16_t> qr;
      qr.u[0] = qraw;
      unpack8<bf16_t>(qr, ql);
#pragma unroll
      for (int i = 0; i < 8; ++i) ql[i] *= LOG2E;
    }
    const int pn = p0 >> 7, jn = (p0 & 127) >> 4, sn = p0 & 15;
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (pn == 0 && j == jn && slot == sn) {
        kr[j] = knew;
        vr[j] = vnew;
      }
    float mw, lw, acc[8];
    wave_row_bf16<16>(ql, kr, vr, 0, Lc, slot, nj0, mw, lw, acc);
    if (nj1 > 0) {  // online merge of the second pass (pass 0 is full, so mw is finite; a wave with no valid key
                    // in pass 1 has m1 = -inf and contributes exp2(-inf) = 0)
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (j < nj1) kr[j] = ld_row8<bf16_t>(kb + (int64_t)min(128 + slot + 16 * j, p0 - 1) * HD + sub * 8).u[0];
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (j < nj1) vr[j] = ld_row8<bf16_t>(vb + (int64_t)min(128 + slot + 16 * j, p0 - 1) * HD + sub * 8).u[0];
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (pn == 1 && j == jn && slot == sn) {
          kr[j] = knew;
          vr[j] = vnew;
        }
      float m1, l1, a1[8];
      wave_row_bf16<16>(ql, kr, vr, 128, Lc, slot, nj1, m1, l1, a1);
      const float mn = fmaxf(mw, m1);
      const float f0 = __builtin_amdgcn_exp2f(mw - mn), f1 = __builtin_amdgcn_exp2f(m1 - mn);
      lw = fmaf(lw, f0, l1 * f1);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] = fmaf(acc[i], f0, a1[i] * f1);
      mw = mn;
    }
    if (slot == sn && len_ok) {  // append position L - 1 to the cache (cache_utils.py:127-145 without the copy),
                                 // after every load of this pair's rows
      *reinterpret_cast<u32x4*>(kb + (int64_t)p0 * HD + sub * 8) = knew;
      *reinterpret_cast<u32x4*>(vb + (int64_t)p0 * HD + sub * 8) = vnew;
    }
    if (lane < 8) {
#pragma unroll
      for (int i = 0; i < 8; ++i) ared[ps][pw][lane * 8 + i] = acc[i];
    }
    if (lane == 0) {
      astat[ps][pw] = mw;
      astat[ps][2 + pw] = lw;
    }
  }
  KW_QS_STAMP(6);
  __syncthreads();
  if (has_pair && ptid < HD) {
    const float* st = astat[ps];
    const float m = fmaxf(st[0], st[1]);
    const float f0 = __builtin_amdgcn_exp2f(st[0] - m), f1 = __builtin_amdgcn_exp2f(st[1] - m);  // -inf wave -> 0
    const float l = fmaf(st[2], f0, st[3] * f1);
    const float o = fmaf(ared[ps][0][ptid], f0, ared[ps][1][ptid] * f1);
    p.out[(int64_t)b * d + h * HD + ptid] = f2bf(o / l);
  }
  KW_QS_STAMP(7);
}

size_t qs_gran_bytes(int64_t M, int64_t d) { return (size_t)M * (size_t)(3 * d / 2) * sizeof(unsigned long long); }

bool qs_shape_ok(int64_t M, int64_t d, int64_t H) {
  return proj_shape_ok(M, d) && H >= 1 && d == 64 * H;
}

}  // namespace

extern "C" size_t kw_dec_qkv_self_workspace(int64_t M, int64_t d) {
  return (M >= 1 && d > 0) ? qs_gran_bytes(M, d) + 64 : 0;
}

extern "C" size_t kw_dec_qkv_self_status_offset(int64_t M, int64_t d) {
  return (M >= 1 && d > 0) ? qs_gran_bytes(M, d) : 0;  // status word, then the fault-injection word
}

extern "C" int kw_dec_qkv_self_supported(int64_t M, int64_t d, int64_t H) {
  return qs_shape_ok(M, d, H) ? 1 : 0;  // (every wait is on earlier-dispatched work: no residency condition)
}

extern "C" int kw_dec_qkv_self(const kw_dec_qkv_self_args* a, kw_stream_t stream) {
  if (!a || !a->x || !a->W || !a->ln_colsum || !a->k_cache || !a->v_cache || !a->cur_len || !a->out || !a->workspace)
    return kw_set_error_msg(KW_EINVAL, "kw_dec_qkv_self: null pointer");
  if (!qs_shape_ok(a->M, a->d, a->H) || a->ldx < a->d || a->ldx % 8 || (uintptr_t)a->x % 16 || a->t_max < 1 ||
      a->t_max > 4096)
    return kw_set_error_msg(KW_EINVAL, "kw_dec_qkv_self: M <= 32 rows, d = 64 H <= 1280, ldx % 8 == 0, 16-B aligned x");
  if (a->ws_bytes < kw_dec_qkv_self_workspace(a->M, a->d))
    return kw_set_error_msg(KW_EINVAL, "kw_dec_qkv_self: needs a zero-filled workspace of kw_dec_qkv_self_workspace()");
  QSP p;
  p.x = reinterpret_cast<const bf16_t*>(a->x);
  p.ldx = a->ldx;
  p.ln_eps = a->ln_eps;
  p.ln_colsum = a->ln_colsum;
  p.W = reinterpret_cast<const bf16x8*>(a->W);
  p.bias = a->bias;
  p.scale = a->scale;
  p.M = (int)a->M;
  p.d = (int)a->d;
  p.H = (int)a->H;
  p.n_lin = (int)(3 * a->d / 16);
  p.kc = reinterpret_cast<bf16_t*>(a->k_cache);
  p.vc = reinterpret_cast<bf16_t*>(a->v_cache);
  p.t_max = (int)a->t_max;
  p.cur_len = a->cur_len;
  p.gran = reinterpret_cast<unsigned long long*>(a->workspace);
  p.err = reinterpret_cast<int*>(reinterpret_cast<char*>(a->workspace) + qs_gran_bytes(a->M, a->d));
  p.out = reinterpret_cast<bf16_t*>(a->out);
  const int grid = p.n_lin + (int)((a->M * a->H + QS_PAIRS - 1) / QS_PAIRS);
  hipLaunchKernelGGL(qkv_self_kernel, dim3((unsigned)grid), dim3(256), 0, (hipStream_t)stream, p);
  KW_CHECK_LAUNCH();
  return KW_OK;
}
