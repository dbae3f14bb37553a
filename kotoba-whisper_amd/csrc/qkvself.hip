// The decoder self-attention block of one greedy decode step in ONE launch (bf16 engine, gfx950):
// the LayerNorm-fused QKV projection (TF/models/whisper/modeling_whisper.py:446 self_attn_layer_norm,
// :469-471 q/k/v with q * head_dim^-0.5 :309) and the self-attention step over the static cache with the
// new key/value appended (:469-480, TF/cache_utils.py:127-145, TF/integrations/sdpa_attention.py:79-166) --
// what kw_dec_linear(qkv) followed by kw_self_attn_step computes in two launches, bitwise the same.
//
//  * workgroups [0, n_lin): dec_linear_kernel<5, 1, LN, STORE, bf16>'s arithmetic for 16 projection
//    columns each (the same fragments, MFMA order, LayerNorm statistics, wave-ordered reduction and
//    epilogue), the bf16 results handed over as 8-byte {bf16 x 2, tag} granules [M][3d/2] instead of
//    stored (MI355X_MICROARCH price list, handoff-1to1: one sc1 store per granule, sc1 polls, untorn);
//  * every workgroup: two (row, head) pairs, one per 4-wave half (pair = 2 * blockIdx.x + half).  A pair's
//    cached K/V rows (positions < L - 1, L = *cur_len <= 256) are loaded at launch -- while the projection
//    runs, where the unfused step loads them only after a kernel boundary; the pair then polls its 96
//    granules (the q, k, v of its head), re-arms them (tag 0: each granule has exactly one consumer),
//    appends k, v at position L - 1 and attends with attention.hip's bf16 row arithmetic (wave_row_bf16,
//    merge_waves_bf16).
//
// Deadlock freedom: a workgroup waits only for granules of workgroups [0, n_lin), and those publish before
// they wait for anything; the host launches only when n_lin workgroups fit on the device at once
// (kw_dec_qkv_self_supported), so every publisher is resident.  Polls are bounded: a timeout sets the error
// word and writes NaN (loud, never silent).
#include "attn_common.h"

namespace {

constexpr int QS_KTM = 5;    // k-tiles per wave: dec_linear's geometry for K <= 1280 (8 waves x 5)
constexpr int QS_WAVES = 8;  // 512 threads: the projection's 8 waves, then two 4-wave attention halves
constexpr int QS_SPIN_LIMIT = 1 << 22;

__device__ __forceinline__ void qs_glds16(const void* g, char* lds_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}

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

__global__ __launch_bounds__(512) void qkv_self_kernel(QSP p) {
  extern __shared__ __attribute__((aligned(16))) char xs[];  // activation image (projection workgroups)
  __shared__ f32x4 red[QS_WAVES][2][64];
  __shared__ float rpart[QS_WAVES][32][2];
  __shared__ float rstat[32][2];
  __shared__ float ared[2][4][64];
  __shared__ float astat[2][8];
  __shared__ uint32_t stage[2][96];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int half = wave >> 2, hw = wave & 3, htid = tid & 255;
  const int d = p.d, H = p.H, M = p.M;
  const int L = *p.cur_len;  // positions [0, L - 1) cached, L - 1 new
  const int p0 = L - 1;

  // ---- 0. this half's pair: its cached K/V rows in flight before anything else (rows past L - 1 clamped;
  //         the row at L - 1 is replaced by the new key / value below)
  const int pair = 2 * blockIdx.x + half;
  const bool has_pair = pair < M * H;  // wave-uniform
  const int b = has_pair ? pair / H : 0, h = has_pair ? pair - (pair / H) * H : 0;
  const int sub = lane & 7, slot = hw * 8 + (lane >> 3);
  const int nj = (L + 31) / 32;  // key groups holding positions < L (<= 8)
  bf16_t* kb = p.kc + ((int64_t)b * H + h) * p.t_max * HD;
  bf16_t* vb = p.vc + ((int64_t)b * H + h) * p.t_max * HD;
  u32x4 kr[8], vr[8];
  if (has_pair) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (j < nj) kr[j] = ld_row8<bf16_t>(kb + (int64_t)min(slot + 32 * j, L - 1) * HD + sub * 8).u[0];
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (j < nj) vr[j] = ld_row8<bf16_t>(vb + (int64_t)min(slot + 32 * j, L - 1) * HD + sub * 8).u[0];
  }

  // ---- 1. the projection: dec_linear_kernel<5, 1, true, KW_EPI_STORE, bf16_t>, 16 columns per workgroup
  if (blockIdx.x < p.n_lin) {
    const int cg = blockIdx.x;
    const int K = d, N = 3 * d;
    const int nkt = K >> 5;
    // dec_linear's wave count for this K (choose(): 5 k-tiles per wave): waves past it only stage activations
    const int nwl = (nkt + QS_KTM - 1) / QS_KTM;
    const bool lin = wave < nwl;
    const int nsl = nwl, sl = lin ? wave : nwl - 1;
    const int kt0 = lin ? (nkt * sl) / nsl : 0, kt1 = lin ? (nkt * (sl + 1)) / nsl : 0;
    const int ktl = max(kt1 - 1, kt0);
    const int arow = lane & 15;
    bf16x8 w[QS_KTM], a0[QS_KTM], a1[QS_KTM];
    if (lin) {
#pragma unroll
      for (int u = 0; u < QS_KTM; ++u)
        w[u] = __builtin_nontemporal_load(p.W + ((int64_t)cg * nkt + min(kt0 + u, ktl)) * 64 + lane);
    }
    const int cpr = nkt * 4, cprp = cpr + 1;
    {
      const int ninst = (32 * cprp + 63) / 64;
      const float inv = 1.0f / (float)cprp;
      for (int j = wave; j < ninst; j += QS_WAVES) {
        const int pidx = j * 64 + lane;
        int row = (int)(((float)pidx + 0.5f) * inv);
        int cs = pidx - row * cprp;
        if (cs < 0) { --row; cs += cprp; }
        if (cs >= cprp) { ++row; cs -= cprp; }
        if (row > 31) { row = 31; cs = 0; }
        if (cs >= cpr) cs = cpr - 1;
        qs_glds16(p.x + (int64_t)min(row, M - 1) * p.ldx + cs * 8, xs + j * 1024);
      }
    }
    const int n_e = min(cg * 16 + (lane & 15), N - 1);
    const float ebias = p.bias ? p.bias[n_e] : 0.f;
    const float ecsum = p.ln_colsum[n_e];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
#pragma unroll
    for (int u = 0; u < QS_KTM; ++u) {
      const int pos = (arow * cprp) + (min(kt0 + u, ktl)) * 4 + (lane >> 4);
      a0[u] = *reinterpret_cast<const bf16x8*>(xs + pos * 16);
      a1[u] = *reinterpret_cast<const bf16x8*>(xs + (pos + 16 * cprp) * 16);
    }
    f32x4 c0 = f32x4{0.f, 0.f, 0.f, 0.f}, c1 = c0;
#pragma unroll
    for (int u = 0; u < QS_KTM; ++u) {
      if (kt0 + u < kt1) {
        c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[u], w[u], c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[u], w[u], c1, 0, 0, 0);
      }
    }
    {
      bf16x8 ones;
#pragma unroll
      for (int e = 0; e < 8; ++e) ones[e] = (__bf16)1.0f;
      f32x4 s0 = f32x4{0.f, 0.f, 0.f, 0.f}, s1 = s0, q0 = s0, q1 = s0;
#pragma unroll
      for (int u = 0; u < QS_KTM; ++u)
        if (kt0 + u < kt1) {
          s0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[u], ones, s0, 0, 0, 0);
          s1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[u], ones, s1, 0, 0, 0);
          q0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[u], a0[u], q0, 0, 0, 0);
          q1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[u], a1[u], q1, 0, 0, 0);
        }
      if ((lane & 15) == 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          rpart[wave][4 * (lane >> 4) + i][0] = s0[i];
          rpart[wave][16 + 4 * (lane >> 4) + i][0] = s1[i];
        }
      }
      const int di = (lane & 15) - 4 * (lane >> 4);
      if (di >= 0 && di < 4) {
        rpart[wave][lane & 15][1] = q0[di];
        rpart[wave][16 + (lane & 15)][1] = q1[di];
      }
    }
    if (lin) {
      red[wave][0][lane] = c0;
      red[wave][1][lane] = c1;
    }
    __syncthreads();
    if (wave == 0) {
      for (int w2 = 1; w2 < nwl; ++w2) {
        c0 += red[w2][0][lane];
        c1 += red[w2][1][lane];
      }
      if (lane < 32) {
        float sx = 0.f, sq = 0.f;
        for (int w2 = 0; w2 < nwl; ++w2) {
          sx += rpart[w2][lane][0];
          sq += rpart[w2][lane][1];
        }
        const float inv = 1.f / (float)K;
        const float mean = sx * inv;
        rstat[lane][0] = mean;
        rstat[lane][1] = rsqrtf(fmaxf(sq * inv - mean * mean, 0.f) + p.ln_eps);
      }
      // epilogue: dec_linear's STORE value, rounded to bf16, paired with the neighbouring column's (lane ^ 1)
      // and published as one granule per column pair by the even column's lane
      const int n = cg * 16 + (lane & 15);
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = 16 * hh + 4 * (lane >> 4) + r;
          float v = hh ? c1[r] : c0[r];
          v = rstat[m][1] * (v - rstat[m][0] * ecsum);
          v += ebias;
          if (n < d) v *= p.scale;
          const uint32_t mine = f2bf(v);
          const uint32_t other = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)mine, 0xB1, 0xF, 0xF, false);  // lane ^ 1
          if ((lane & 1) == 0 && m < M && n < N)
            __hip_atomic_store(p.gran + (int64_t)m * (N / 2) + (n >> 1), (1ull << 32) | (mine | (other << 16)),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
  }

  // ---- 2. the pair: its head's q, k, v from the granules (one poller per granule), then the attention
  if (has_pair && htid < 96) {
    const int part = htid >> 5, c = htid & 31;  // part 0 q, 1 k, 2 v; c = column pair within the head
    unsigned long long* g = p.gran + (int64_t)b * (3 * d / 2) + part * (d / 2) + h * 32 + c;
    unsigned long long x = 0;
    int it = 0;
    for (;; ++it) {
      x = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((x >> 32) == 1ull || it >= QS_SPIN_LIMIT) break;
      __builtin_amdgcn_s_sleep(1);
    }
    if ((x >> 32) != 1ull) {
      x = 0x7fc07fc0ull;  // bf16 NaN pair: the failure propagates to the output
      __hip_atomic_store(p.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    stage[half][htid] = (uint32_t)x;
    __hip_atomic_store(g, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm (single consumer)
  }
  __syncthreads();
  if (has_pair) {
    const u32x4 qraw = {stage[half][sub * 4], stage[half][sub * 4 + 1], stage[half][sub * 4 + 2], stage[half][sub * 4 + 3]};
    const u32x4 knew = {stage[half][32 + sub * 4], stage[half][32 + sub * 4 + 1], stage[half][32 + sub * 4 + 2],
                        stage[half][32 + sub * 4 + 3]};
    const u32x4 vnew = {stage[half][64 + sub * 4], stage[half][64 + sub * 4 + 1], stage[half][64 + sub * 4 + 2],
                        stage[half][64 + sub * 4 + 3]};
    float ql[8];
    {
      Row8<bf16_t> qr;
      qr.u[0] = qraw;
      unpack8<bf16_t>(qr, ql);
#pragma unroll
      for (int i = 0; i < 8; ++i) ql[i] *= LOG2E;
    }
    const int jn = p0 >> 5, sn = p0 & 31;
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (j == jn && slot == sn) {
        kr[j] = knew;
        vr[j] = vnew;
      }
    if (slot == sn) {  // append position L - 1 to the cache (cache_utils.py:127-145 without the copy)
      *reinterpret_cast<u32x4*>(kb + (int64_t)p0 * HD + sub * 8) = knew;
      *reinterpret_cast<u32x4*>(vb + (int64_t)p0 * HD + sub * 8) = vnew;
    }
    float mw, lw, acc[8];
    wave_row_bf16(ql, kr, vr, 0, L, slot, nj, mw, lw, acc);
    if (lane < 8) {
#pragma unroll
      for (int i = 0; i < 8; ++i) ared[half][hw][lane * 8 + i] = acc[i];
    }
    if (lane == 0) {
      astat[half][hw] = mw;
      astat[half][4 + hw] = lw;
    }
  }
  __syncthreads();
  if (has_pair && htid < HD) {
    float m, l, o;
    merge_waves_bf16(astat[half], ared[half], htid, m, l, o);
    p.out[(int64_t)b * d + h * HD + htid] = f2bf(o / l);
  }
}

size_t qs_lds_bytes(int64_t d) {  // dec_linear's activation image for K = d: 32 rows x (4 k-tiles... + 1 pad) chunks
  const int tiles = (int)(d / 32);
  return (size_t)((32 * (4 * tiles + 1) + 63) / 64) * 1024;
}

size_t qs_gran_bytes(int64_t M, int64_t d) { return (size_t)M * (size_t)(3 * d / 2) * sizeof(unsigned long long); }

bool qs_shape_ok(int64_t M, int64_t d, int64_t H) {
  return M >= 1 && M <= 32 && H >= 1 && d == 64 * H && d % 32 == 0 && d / 32 <= QS_WAVES * QS_KTM;
}

}  // namespace

extern "C" size_t kw_dec_qkv_self_workspace(int64_t M, int64_t d) {
  return (M >= 1 && d > 0) ? qs_gran_bytes(M, d) + 64 : 0;
}

extern "C" int kw_dec_qkv_self_supported(int64_t M, int64_t d, int64_t H) {
  if (!qs_shape_ok(M, d, H)) return 0;
  const int n_lin = (int)(3 * d / 16);
  int dev = 0, ncu = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 0;
  const size_t shm = qs_lds_bytes(d);
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(&qkv_self_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)shm) != hipSuccess)
    return 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(&qkv_self_kernel), 512, shm) !=
      hipSuccess)
    return 0;
  return (int64_t)per_cu * ncu >= n_lin ? 1 : 0;  // every publishing workgroup resident at once
}

extern "C" int kw_dec_qkv_self(const kw_dec_qkv_self_args* a, kw_stream_t stream) {
  if (!a || !a->x || !a->W || !a->ln_colsum || !a->k_cache || !a->v_cache || !a->cur_len || !a->out || !a->workspace)
    return kw_set_error_msg(KW_EINVAL, "kw_dec_qkv_self: null pointer");
  if (!qs_shape_ok(a->M, a->d, a->H) || a->ldx < a->d || a->ldx % 8 || (uintptr_t)a->x % 16 || a->t_max < 1 ||
      a->t_max > 4096)
    return kw_set_error_msg(KW_EINVAL, "kw_dec_qkv_self: M <= 32 rows, d = 64 H <= 1280, ldx % 8 == 0, 16-B aligned x");
  if (a->ws_bytes < kw_dec_qkv_self_workspace(a->M, a->d))
    return kw_set_error_msg(KW_EINVAL, "kw_dec_qkv_self: needs a zero-filled workspace of kw_dec_qkv_self_workspace()");
  static int64_t checked_d = -1;  // co-residency of the publishing workgroups (deadlock freedom), per width
  static int checked = 0;
  if (checked_d != a->d) {
    checked = kw_dec_qkv_self_supported(a->M, a->d, a->H);
    checked_d = a->d;
  }
  if (!checked)
    return kw_set_error_msg(KW_EUNSUPPORTED, "kw_dec_qkv_self: the projection workgroups do not fit on the device at once");
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
  const int pairs_wg = (int)((a->M * a->H + 1) / 2);
  const int grid = p.n_lin > pairs_wg ? p.n_lin : pairs_wg;
  hipLaunchKernelGGL(qkv_self_kernel, dim3((unsigned)grid), dim3(512), qs_lds_bytes(a->d), (hipStream_t)stream, p);
  KW_CHECK_LAUNCH();
  return KW_OK;
}
