// a1 -- Whisper log-mel spectrogram on gfx950.
//
// Replaces WhisperFeatureExtractor._torch_extract_fbank_features
// (TF/models/whisper/feature_extraction_whisper.py:135-168).  Per workgroup: FT consecutive STFT
// frames of one clip.  The reflect-padded audio span of those frames is staged once in LDS
// (coalesced 16-B loads), the windowed 400-point DFT is evaluated against an LDS twiddle table,
// |X|^2 stays in LDS, the slaney mel projection reads the (L2-resident) filter bank, and log10 is
// written time-contiguous.  The per-clip maximum is an order-preserving integer atomicMax; a second
// light pass applies max(x, max-8) and (x+4)/4.
//
// Roofline: 1.12 GFLOP and 1.92 MB in / 1.54 MB out per clip -> compute-light; the
// DFT runs on the VALU with f64 accumulation.
#include <math.h>

#include "kw_common.h"

namespace {

constexpr int N_FFT = 400;
constexpr int HOP = 160;
constexpr int N_BINS = N_FFT / 2 + 1;  // 201
constexpr int FT = 16;                 // frames per workgroup
constexpr int SPAN = (FT - 1) * HOP + N_FFT;  // 5360 samples
constexpr int THREADS = 256;

__device__ __forceinline__ uint32_t f2key(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key2f(uint32_t k) {
  uint32_t u = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;
  return __uint_as_float(u);
}

__global__ __launch_bounds__(THREADS) void logmel_kernel(const float* __restrict__ audio, int64_t n_samples,
                                                         int64_t audio_stride, const float* __restrict__ fb,
                                                         int n_mels, float* __restrict__ out, int n_out,
                                                         uint32_t* __restrict__ clip_max) {
  // the staged audio span is dead once the windowed frames are built: it shares memory with |X|^2
  union SpanOrPower {
    float xs[SPAN];
    float pw[FT][N_BINS + 3];
  };
  __shared__ SpanOrPower u;
  __shared__ double win[N_FFT];
  __shared__ double xw[N_FFT][FT];  // windowed frames, sample-major: one broadcast read per (n, frame)
  float* const xs = u.xs;
  auto& pw = u.pw;
  __shared__ uint32_t red[THREADS / 64];
  __shared__ short mrange[512][2];  // mel m's nonzero filter bins [lo, hi) (slaney triangles: one contiguous run)

  const int b = blockIdx.y;
  const int f0 = blockIdx.x * FT;
  const float* x = audio + (int64_t)b * audio_stride;
  const int tid = threadIdx.x;
  const float two_pi_n = 6.283185307179586476925 / N_FFT;

  for (int i = tid; i < N_FFT; i += THREADS) {
    double a = 6.283185307179586476925 * (double)i / N_FFT;
    win[i] = (double)(float)(0.5 - 0.5 * cos(a));  // torch.hann_window(400) (periodic), f32 values
  }
  // each mel filter's nonzero bins: the projection below sums only those, in the same bin order -- for FINITE power
  // spectra bitwise the dense sum (a zero weight adds +0 to the f32 accumulator) at a fraction of its 201
  // multiply-adds per output.  Non-finite audio differs: the dense sum's 0 * Inf terms make every mel bin NaN (as
  // the reference's mel_filters.T @ magnitudes does), the sparse sum keeps bins whose filter range avoids the bad
  // frequency bins finite (parity on non-finite input is unpinned)
  for (int m = tid; m < n_mels; m += THREADS) {
    int lo = N_BINS, hi = 0;
    for (int k0 = 0; k0 < N_BINS; k0 += 8) {
      float w[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) w[u] = fb[min(k0 + u, N_BINS - 1) * n_mels + m];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (k0 + u < N_BINS && w[u] != 0.f) {
          lo = min(lo, k0 + u);
          hi = k0 + u + 1;
        }
    }
    mrange[m][0] = (short)lo;
    mrange[m][1] = (short)max(hi, lo);
  }
  (void)two_pi_n;
  // reflect-padded span: padded index p = f0*HOP + i  ->  original index j = p - 200
  const int64_t base = (int64_t)f0 * HOP - N_FFT / 2;
  for (int i = tid; i < SPAN; i += THREADS) {
    int64_t j = base + i;
    if (j < 0) j = -j;
    if (j >= n_samples) j = 2 * (n_samples - 1) - j;
    if (j < 0) j = 0;  // only for absurdly short inputs (guarded on the host)
    xs[i] = x[j];
  }
  __syncthreads();

  // |DFT|^2 for FT frames x 201 bins.  Thread k owns bin k of every frame: per sample n it reads its
  // twiddle pair once and the FT windowed samples by broadcast, so the LDS traffic per f64 FMA is
  // ~1/2 read instead of 2.  The accumulation order over n is the same as a per-(frame, bin) loop.
  const int n_frames_here = min(FT, n_out + 1 - f0);  // frames computed (last global frame dropped below)
  for (int i = tid; i < N_FFT * FT; i += THREADS) {
    const int n = i / FT, f = i - n * FT;
    xw[n][f] = f < n_frames_here ? (double)xs[f * HOP + n] * win[n] : 0.0;
  }
  __syncthreads();
  if (tid < N_BINS) {
    const int k = tid;
    double re[FT], im[FT];
#pragma unroll
    for (int f = 0; f < FT; ++f) re[f] = im[f] = 0.0;
    // twiddle e^{i 2 pi n k / 400} by f64 rotation (relative drift ~1e-14 over 400 steps, far below the
    // f32 result), re-anchored to the exact value every 50 samples
    const double th = 6.283185307179586476925 * (double)k / N_FFT;
    const double cr = cos(th), sr = sin(th);
    double c = 1.0, sn = 0.0;
    for (int n = 0; n < N_FFT; ++n) {
      if (n % 50 == 0) {
        const double a = 6.283185307179586476925 * (double)((n * k) % N_FFT) / N_FFT;
        c = cos(a);
        sn = sin(a);
      }
#pragma unroll
      for (int f = 0; f < FT; ++f) {
        const double v = xw[n][f];
        re[f] = fma(v, c, re[f]);
        im[f] = fma(v, sn, im[f]);
      }
      const double c2 = c * cr - sn * sr;
      sn = fma(c, sr, sn * cr);
      c = c2;
    }
#pragma unroll
    for (int f = 0; f < FT; ++f) pw[f][k] = (float)(re[f] * re[f] + im[f] * im[f]);
  }
  __syncthreads();

  // mel projection + log10; thread -> (mel, frame), frame fastest (time-contiguous stores)
  float local_max = -INFINITY;
  for (int o = tid; o < FT * n_mels; o += THREADS) {
    const int m = o / FT;
    const int f = o - m * FT;
    const int t = f0 + f;
    if (t >= n_out) continue;
    float acc = 0.f;
    const int k1 = mrange[m][1];
    for (int k = mrange[m][0]; k < k1; ++k) acc = fmaf(fb[k * n_mels + m], pw[f][k], acc);
    const float lg = log10f(fmaxf(acc, 1e-10f));
    out[((int64_t)b * n_mels + m) * n_out + t] = lg;
    local_max = fmaxf(local_max, lg);
  }
  local_max = wave_max(local_max);
  if ((tid & 63) == 0) red[tid >> 6] = f2key(local_max);
  __syncthreads();
  if (tid == 0) {
    uint32_t k = red[0];
    for (int i = 1; i < THREADS / 64; ++i) k = max(k, red[i]);
    atomicMax(clip_max + b, k);
  }
}

__global__ void logmel_norm_kernel(float* __restrict__ out, int64_t per_clip, const uint32_t* __restrict__ clip_max) {
  const int b = blockIdx.y;
  const float mx = key2f(clip_max[b]) - 8.0f;
  float* o = out + (int64_t)b * per_clip;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < per_clip; i += (int64_t)gridDim.x * blockDim.x) {
    o[i] = (fmaxf(o[i], mx) + 4.0f) / 4.0f;
  }
}

}  // namespace

extern "C" int kw_log_mel(const float* audio, int64_t batch, int64_t n_samples, int64_t audio_stride,
                          const float* mel_filters, int n_mels, float* out, void* workspace, kw_stream_t stream) {
  if (!audio || !mel_filters || !out || !workspace || batch <= 0 || n_mels <= 0 || n_mels > 512)
    return kw_set_error_msg(KW_EINVAL, "kw_log_mel: invalid arguments");
  if (n_samples < N_FFT || n_samples % HOP != 0 || audio_stride < n_samples)
    return kw_set_error_msg(KW_EINVAL, "kw_log_mel: n_samples must be >= 400, a multiple of 160, <= audio_stride");
  hipStream_t s = (hipStream_t)stream;
  const int n_out = (int)(n_samples / HOP);  // frames after dropping the last one
  hipError_t e = hipMemsetAsync(workspace, 0, sizeof(uint32_t) * batch, s);
  if (e != hipSuccess) return kw_set_error(e);
  dim3 grid((n_out + FT - 1) / FT, (unsigned)batch);
  hipLaunchKernelGGL(logmel_kernel, grid, dim3(THREADS), 0, s, audio, n_samples, audio_stride, mel_filters, n_mels,
                     out, n_out, (uint32_t*)workspace);
  KW_CHECK_LAUNCH();
  hipLaunchKernelGGL(logmel_norm_kernel, dim3(64, (unsigned)batch), dim3(256), 0, s, out, (int64_t)n_mels * n_out,
                     (const uint32_t*)workspace);
  KW_CHECK_LAUNCH();
  return KW_OK;
}
