// stft_psd.hip — batched spectrogram (scipy.signal.spectrogram PSD semantics) for gfx950.
//
// Replaces spec_denoising/pipeline_data.py:32-35 (scipy.signal.spectrogram ->
// log(S+eps) -> per-spectrogram min-max -> drop Nyquist row), i.e. the arithmetic of
// scipy/signal/_spectral_py.py:1863-2204 (frames, per-frame detrend, window, rfft,
// |X|^2 * scale, one-sided x2) for power-of-two nperseg.
//
// Work decomposition (one workgroup = one tile of TF consecutive frames of one shot):
//  * Two real frames share one complex FFT (z = a + i b; "two-for-one"): the
//    separation A_k = (Z_k + conj Z_{N-k})/2, B_k = (Z_k - conj Z_{N-k})/(2i) needs
//    no twiddles.
//  * One FFT is owned by G lanes of one wave (G = 8..64), N/G points per lane, so
//    every inter-pass exchange is wave-local (no workgroup barrier inside the FFT).
//  * Pass 1 reads the raw samples straight from HBM (coalesced across the G lanes),
//    computes the per-frame linear-detrend sums while the samples sit in registers,
//    reduces them across the lane group, detrends + windows in place and runs an
//    in-register radix-R1 DIF; later passes are Stockham passes through a padded
//    per-FFT LDS buffer (radix R2, R3) with twiddles from an LDS table.
//  * The epilogue forms |A|^2, |B|^2, the one-sided scale, log2(P+eps) and the
//    running min/max, and stages the (bins x frames) tile in LDS so the final store
//    writes whole frequency rows of the freq-major [F][T] output.
//  * Per-spectrogram min/max: one pair of order-preserving uint atomics per
//    workgroup; a second light kernel applies (L - min)/(max - min).
//    log2 is used instead of ln for the normalised output: the ratio is invariant.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <algorithm>
#include <string>
#include <vector>

#include "fft_common.hpp"
#include "specenh.h"

namespace specenh {

thread_local std::string g_last_error;

int set_error(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

#define SPECENH_HIP_CHECK(expr)                                                          \
  do {                                                                                   \
    hipError_t _e = (expr);                                                              \
    if (_e != hipSuccess)                                                                \
      return set_error(SPECENH_EHIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

struct StftArgs {
  const float* x;
  long long x_stride;
  int T;
  int hop;
  float scale;     // density or spectrum scale
  float eps;
  float inv_kk;    // 1 / sum_n (n - (N-1)/2)^2
  int detrend;
  int flags;
  float* out;
  int F_out;
  unsigned* minmax;  // [batch][2] order-preserving keys
  const float* window;
  const float2* twiddle;  // W_N^m, m in [0, N)
  const double* dc_coef;  // c_n: DC bin of the detrended, windowed frame = <x, c> (fp64)
};

// Per-N decomposition: G lanes per FFT, WAVES per workgroup, Stockham radices.
template <int N>
struct Cfg;
template <> struct Cfg<64>   { static constexpr int G = 8,  WAVES = 4, R1 = 8,  R2 = 8,  R3 = 1; };
template <> struct Cfg<128>  { static constexpr int G = 8,  WAVES = 4, R1 = 16, R2 = 8,  R3 = 1; };
template <> struct Cfg<256>  { static constexpr int G = 16, WAVES = 4, R1 = 16, R2 = 16, R3 = 1; };
template <> struct Cfg<512>  { static constexpr int G = 16, WAVES = 4, R1 = 32, R2 = 16, R3 = 1; };
template <> struct Cfg<1024> { static constexpr int G = 32, WAVES = 4, R1 = 32, R2 = 32, R3 = 1; };
template <> struct Cfg<2048> { static constexpr int G = 64, WAVES = 4, R1 = 32, R2 = 8,  R3 = 8; };
template <> struct Cfg<4096> { static constexpr int G = 64, WAVES = 2, R1 = 32, R2 = 16, R3 = 8; };

template <int N>
struct Layout {
  using C = Cfg<N>;
  static constexpr int G = C::G;
  static constexpr int THREADS = 64 * C::WAVES;
  static constexpr int FFTS = C::WAVES * (64 / G);  // concurrent FFTs per workgroup
  static constexpr int TF = 2 * FFTS;                // frames per workgroup tile
  static constexpr int TS = TF + 1;                  // tile row stride (odd: conflict-free)
  static constexpr int NBINS = N / 2 + 1;
  static constexpr int BUF = N + N / 32;             // padded complex entries per FFT
  // byte offsets into dynamic LDS (all multiples of 16)
  static constexpr int OFF_TW = 0;
  static constexpr int OFF_WIN = OFF_TW + N * 8;
  static constexpr int OFF_BUF = OFF_WIN + N * 4;
  static constexpr int OFF_TILE = OFF_BUF + FFTS * BUF * 8;
  static constexpr int OFF_RED = OFF_TILE + ((NBINS * TS * 4 + 15) / 16) * 16;
  static constexpr int BYTES = OFF_RED + 2 * C::WAVES * 4 + 16;
  static_assert(BYTES <= 160 * 1024, "LDS budget");
  static_assert(C::R1 * C::R2 * C::R3 == N, "radix product");
};

__device__ __forceinline__ int pad(int e) { return e + (e >> 5); }

// Stockham pass NS>1 through the LDS buffer (all butterflies of the lane read first,
// then written back in place: legal because the whole FFT lives in one wave).
template <int N, int G, int R, int NS>
__device__ __forceinline__ void stockham_pass(float2* buf, const float2* tw, int gl) {
  constexpr int NB = N / R;
  constexpr int BPL = NB / G;
  constexpr int LOGR = ilog2(R);
  static_assert(BPL >= 1 && NB % G == 0, "butterflies per lane");
  float2 v[BPL][R];
#pragma unroll
  for (int i = 0; i < BPL; ++i) {
    const int b = gl + i * G;
#pragma unroll
    for (int r = 0; r < R; ++r) v[i][r] = buf[pad(b + r * NB)];
  }
  wave_lds_sync();
#pragma unroll
  for (int i = 0; i < BPL; ++i) {
    const int b = gl + i * G;
    const int k = b % NS;
#pragma unroll
    for (int r = 1; r < R; ++r) v[i][r] = cmul(v[i][r], tw[r * k * (N / (NS * R))]);
    fft_dif<R>(v[i]);
    const int base = (b / NS) * NS * R + k;
#pragma unroll
    for (int r = 0; r < R; ++r) buf[pad(base + bitrev(r, LOGR) * NS)] = v[i][r];
  }
  wave_lds_sync();
}

template <int N>
__global__ __launch_bounds__(Layout<N>::THREADS) void stft_psd_kernel(StftArgs a) {
  using C = Cfg<N>;
  using Lo = Layout<N>;
  constexpr int G = C::G;
  constexpr int R1 = C::R1;
  constexpr int NB1 = N / R1;
  constexpr int BPL1 = NB1 / G;
  constexpr int LOGR1 = ilog2(R1);
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float2* s_tw = reinterpret_cast<float2*>(smem + Lo::OFF_TW);
  float* s_win = reinterpret_cast<float*>(smem + Lo::OFF_WIN);
  float* s_tile = reinterpret_cast<float*>(smem + Lo::OFF_TILE);
  float* s_red = reinterpret_cast<float*>(smem + Lo::OFF_RED);

  const int tid = threadIdx.x;
  const int shot = blockIdx.y;
  const int t0 = blockIdx.x * Lo::TF;

  for (int i = tid; i < N; i += Lo::THREADS) {
    s_tw[i] = a.twiddle[i];
    s_win[i] = a.window[i];
  }
  __syncthreads();

  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int gl = lane % G;                          // lane within the FFT group
  const int fi = wave * (64 / G) + lane / G;        // FFT index within the tile
  float2* buf = reinterpret_cast<float2*>(smem + Lo::OFF_BUF) + fi * Lo::BUF;
  const int fa = t0 + 2 * fi;                       // frame index of the real part
  const bool va = fa < a.T;
  const bool vb = fa + 1 < a.T;
  // Invalid frames (tail of the last tile) read frame 0 of the same shot and are
  // zeroed after the load: loads stay unconditional (no per-element branch/wait).
  const float* xs = a.x + (long long)shot * a.x_stride;
  const float* xa = xs + (long long)(va ? fa : 0) * a.hop;
  const float* xb = xs + (long long)(vb ? fa + 1 : 0) * a.hop;

  // ---- pass 1: load, detrend, window, radix-R1 DIF, store to LDS ----
  // Detrend in two sweeps over the register-resident samples: a rough mean m1
  // (division by N = 2^k is exact), then mean/slope of the residuals x - m1. The
  // rounding of m1 then never enters y coherently: the post-detrend DC bin (tiny by
  // construction, and the usual argmin of the spectrogram) keeps fp32-rounding
  // accuracy instead of inheriting |mean| * eps * sum(w).
  float2 v[BPL1][R1];
  constexpr float kmid = 0.5f * float(N - 1);
  constexpr float invN = 1.0f / float(N);
  float s0a = 0.f, s0b = 0.f;
  // DC bin in fp64: X_0 = sum_n w_n y_n = <x, c> with c = w - mean(w) - kc * sum(w kc)/sum(kc^2)
  // (c is orthogonal to constants and ramps, so the detrend cancellation happens exactly
  // in the coefficients, not in the data). After detrending X_0 is tiny by construction;
  // in fp32 it would sit at the rounding floor eps*||w y|| and, being the usual
  // spectrogram minimum under 'spectrum' scaling, would shift every normalised value.
  double dca = 0.0, dcb = 0.0;
#pragma unroll
  for (int i = 0; i < BPL1; ++i) {
    const int b = gl + i * G;
#pragma unroll
    for (int r = 0; r < R1; ++r) {
      const int n = b + r * NB1;
      const float la = xa[n], lb = xb[n];
      const float xa_n = va ? la : 0.f;
      const float xb_n = vb ? lb : 0.f;
      v[i][r] = make_float2(xa_n, xb_n);
      s0a += xa_n;
      s0b += xb_n;
      const double c = a.dc_coef[n];
      dca = fma((double)xa_n, c, dca);
      dcb = fma((double)xb_n, c, dcb);
    }
  }
#pragma unroll
  for (int m = G / 2; m >= 1; m >>= 1) {
    dca += __shfl_xor(dca, m);
    dcb += __shfl_xor(dcb, m);
  }
  float lo_a = 0.f, lo_b = 0.f, slope_a = 0.f, slope_b = 0.f;
  if (a.detrend != SPECENH_DETREND_NONE) {
#pragma unroll
    for (int m = G / 2; m >= 1; m >>= 1) {
      s0a += __shfl_xor(s0a, m);
      s0b += __shfl_xor(s0b, m);
    }
    const float m1a = s0a * invN, m1b = s0b * invN;
    float r0a = 0.f, r0b = 0.f, r1a = 0.f, r1b = 0.f;
#pragma unroll
    for (int i = 0; i < BPL1; ++i) {
      const int b = gl + i * G;
#pragma unroll
      for (int r = 0; r < R1; ++r) {
        const float kc = float(b + r * NB1) - kmid;
        const float ra = v[i][r].x - m1a, rb = v[i][r].y - m1b;
        v[i][r] = make_float2(ra, rb);
        r0a += ra;
        r0b += rb;
        r1a = fmaf(kc, ra, r1a);
        r1b = fmaf(kc, rb, r1b);
      }
    }
#pragma unroll
    for (int m = G / 2; m >= 1; m >>= 1) {
      r0a += __shfl_xor(r0a, m);
      r0b += __shfl_xor(r0b, m);
      r1a += __shfl_xor(r1a, m);
      r1b += __shfl_xor(r1b, m);
    }
    lo_a = r0a * invN;
    lo_b = r0b * invN;
    if (a.detrend == SPECENH_DETREND_LINEAR) {
      slope_a = r1a * a.inv_kk;
      slope_b = r1b * a.inv_kk;
    }
  }
#pragma unroll
  for (int i = 0; i < BPL1; ++i) {
    const int b = gl + i * G;
#pragma unroll
    for (int r = 0; r < R1; ++r) {
      const int n = b + r * NB1;
      const float kc = float(n) - kmid;
      const float w = s_win[n];
      const float ya = fmaf(-slope_a, kc, v[i][r].x - lo_a);
      const float yb = fmaf(-slope_b, kc, v[i][r].y - lo_b);
      v[i][r] = make_float2(w * ya, w * yb);
    }
    fft_dif<R1>(v[i]);
#pragma unroll
    for (int r = 0; r < R1; ++r) buf[pad(b * R1 + bitrev(r, LOGR1))] = v[i][r];
  }
  wave_lds_sync();

  // ---- remaining Stockham passes in LDS ----
  stockham_pass<N, G, C::R2, R1>(buf, s_tw, gl);
  if constexpr (C::R3 > 1) stockham_pass<N, G, C::R3, R1 * C::R2>(buf, s_tw, gl);

  // ---- epilogue: separate the two frames, PSD, log, min/max, stage the tile ----
  const bool want_log = (a.flags & (SPECENH_STFT_LOG | SPECENH_STFT_NORMALIZE)) != 0;
  const bool log2_out = (a.flags & SPECENH_STFT_NORMALIZE) != 0;
  float lmin = INFINITY, lmax = -INFINITY;
  const int fl = 2 * fi;
  constexpr int IB = (Lo::NBINS + G - 1) / G;
#pragma unroll 4
  for (int i = 0; i < IB; ++i) {
    const int k = gl + i * G;
    if (k < Lo::NBINS) {
      const float2 zk = buf[pad(k)];
      const float2 zm = buf[pad((N - k) & (N - 1))];
      const float ar = zk.x + zm.x, ai = zk.y - zm.y;
      const float br = zk.x - zm.x, bi = zk.y + zm.y;
      const float s = (k == 0 || k == N / 2) ? 0.25f * a.scale : 0.5f * a.scale;
      float pa = fmaf(ar, ar, ai * ai) * s;
      float pb = fmaf(br, br, bi * bi) * s;
      if (k == 0) {
        pa = (float)(dca * dca * (double)a.scale);
        pb = (float)(dcb * dcb * (double)a.scale);
      }
      if (want_log) {
        pa = __log2f(pa + a.eps);
        pb = __log2f(pb + a.eps);
        if (!log2_out) {
          pa *= 0.69314718055994530942f;
          pb *= 0.69314718055994530942f;
        }
      }
      if (va) { lmin = fminf(lmin, pa); lmax = fmaxf(lmax, pa); }
      if (vb) { lmin = fminf(lmin, pb); lmax = fmaxf(lmax, pb); }
      s_tile[k * Lo::TS + fl] = pa;
      s_tile[k * Lo::TS + fl + 1] = pb;
    }
  }
  __syncthreads();

  // ---- per-spectrogram min/max (one atomic pair per workgroup) ----
  if (a.flags & SPECENH_STFT_NORMALIZE) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
      lmin = fminf(lmin, __shfl_xor(lmin, m));
      lmax = fmaxf(lmax, __shfl_xor(lmax, m));
    }
    if (lane == 0) {
      s_red[wave] = lmin;
      s_red[C::WAVES + wave] = lmax;
    }
    __syncthreads();
    if (tid == 0) {
      float mn = s_red[0], mx = s_red[C::WAVES];
      for (int w = 1; w < C::WAVES; ++w) {
        mn = fminf(mn, s_red[w]);
        mx = fmaxf(mx, s_red[C::WAVES + w]);
      }
      atomicMin(&a.minmax[2 * shot], f2key(mn));
      atomicMax(&a.minmax[2 * shot + 1], f2key(mx));
    }
  }

  // ---- store whole frequency rows of the tile: out[shot][k][t0 : t0+TFv] ----
  const int tfv = min(Lo::TF, a.T - t0);
  float* o = a.out + (long long)shot * a.F_out * a.T + t0;
  const int total = a.F_out * tfv;
  for (int e = tid; e < total; e += Lo::THREADS) {
    const int k = e / tfv;
    const int f = e - k * tfv;
    o[(long long)k * a.T + f] = s_tile[k * Lo::TS + f];
  }
}

__global__ void minmax_init_kernel(unsigned* mm, long long batch) {
  long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i < batch) {
    mm[2 * i] = 0xffffffffu;
    mm[2 * i + 1] = 0u;
  }
}

// out[b] = (L - min_b) / (max_b - min_b) over one spectrogram's F*T values.
__global__ __launch_bounds__(256) void normalize_kernel(float* out, const unsigned* mm,
                                                        long long per_shot) {
  const long long shot = blockIdx.y;
  const float mn = key2f(mm[2 * shot]);
  const float mx = key2f(mm[2 * shot + 1]);
  const float inv = 1.0f / (mx - mn);
  float* o = out + shot * per_shot;
  for (long long e = blockIdx.x * 256ll + threadIdx.x; e < per_shot; e += 256ll * gridDim.x)
    o[e] = (o[e] - mn) * inv;
}

template <int N>
hipError_t launch_stft(const StftArgs& a, long long batch, hipStream_t stream) {
  using Lo = Layout<N>;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)stft_psd_kernel<N>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, Lo::BYTES);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  dim3 grid((a.T + Lo::TF - 1) / Lo::TF, (unsigned)batch);
  hipLaunchKernelGGL(stft_psd_kernel<N>, grid, dim3(Lo::THREADS), Lo::BYTES, stream, a);
  return hipGetLastError();
}

}  // namespace specenh

using namespace specenh;

struct specenh_stft_plan {
  int nperseg, noverlap, hop;
  double fs, eps, scale;
  int scaling, detrend;
  int device;
  float* d_window;
  float2* d_twiddle;
  double* d_dc;
};

extern "C" {

const char* specenh_last_error(void) { return g_last_error.c_str(); }
const char* specenh_version(void) { return "specenh 0.1.0 gfx950"; }

long long specenh_stft_frames(long long length, int nperseg, int noverlap) {
  if (nperseg <= 0 || noverlap < 0 || noverlap >= nperseg)
    return set_error(SPECENH_EINVAL, "noverlap must be less than nperseg.");
  if (length < nperseg) return set_error(SPECENH_EINVAL, "signal shorter than nperseg");
  return (length - nperseg) / (nperseg - noverlap) + 1;
}

int specenh_stft_plan_create(specenh_stft_plan** plan, int nperseg, int noverlap,
                             const double* window_host, double fs, int scaling, int detrend,
                             double eps) {
  if (!plan || !window_host) return set_error(SPECENH_EINVAL, "null plan/window pointer");
  *plan = nullptr;
  if (noverlap < 0 || noverlap >= nperseg)
    return set_error(SPECENH_EINVAL, "noverlap must be less than nperseg.");
  if (nperseg < 64 || nperseg > 4096 || (nperseg & (nperseg - 1)))
    return set_error(SPECENH_EUNSUPPORTED,
                     "nperseg must be a power of two in [64, 4096] on the GPU path");
  if (scaling != SPECENH_SCALING_DENSITY && scaling != SPECENH_SCALING_SPECTRUM)
    return set_error(SPECENH_EINVAL, "Unknown scaling");
  if (detrend < SPECENH_DETREND_NONE || detrend > SPECENH_DETREND_LINEAR)
    return set_error(SPECENH_EINVAL, "Trend type must be 'linear' or 'constant'.");
  if (!(fs > 0)) return set_error(SPECENH_EINVAL, "fs must be positive");
  const int N = nperseg;
  double s1 = 0, s2 = 0;
  std::vector<float> win(N);
  for (int i = 0; i < N; ++i) {
    s1 += window_host[i];
    s2 += window_host[i] * window_host[i];
    win[i] = float(window_host[i]);
  }
  // DC coefficients c_n (fp64): the detrend folded into the window (see kernel).
  std::vector<double> dc(N);
  {
    const double kmid = 0.5 * (N - 1);
    double sk2 = 0, swk = 0;
    for (int i = 0; i < N; ++i) {
      sk2 += (i - kmid) * (i - kmid);
      swk += window_host[i] * (i - kmid);
    }
    const double wbar = s1 / N;
    for (int i = 0; i < N; ++i) {
      double c = window_host[i];
      if (detrend != SPECENH_DETREND_NONE) c -= wbar;
      if (detrend == SPECENH_DETREND_LINEAR) c -= (i - kmid) * (swk / sk2);
      dc[i] = c;
    }
  }
  std::vector<float2> tw(N);
  for (int m = 0; m < N; ++m) {
    ct::CS cs = ct::cossin_frac(m, N);
    tw[m] = make_float2(float(cs.c), float(-cs.s));
  }
  auto* p = new specenh_stft_plan{};
  p->nperseg = N;
  p->noverlap = noverlap;
  p->hop = N - noverlap;
  p->fs = fs;
  p->eps = eps;
  p->scaling = scaling;
  p->detrend = detrend;
  p->scale = scaling == SPECENH_SCALING_DENSITY ? 1.0 / (fs * s2) : 1.0 / (s1 * s1);
  hipError_t e = hipGetDevice(&p->device);
  if (e == hipSuccess) e = hipMalloc(&p->d_window, N * sizeof(float));
  if (e == hipSuccess) e = hipMalloc(&p->d_twiddle, N * sizeof(float2));
  if (e == hipSuccess) e = hipMalloc(&p->d_dc, N * sizeof(double));
  if (e == hipSuccess) e = hipMemcpy(p->d_dc, dc.data(), N * sizeof(double), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(p->d_window, win.data(), N * sizeof(float), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(p->d_twiddle, tw.data(), N * sizeof(float2), hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    (void)hipFree(p->d_window);
    (void)hipFree(p->d_twiddle);
    (void)hipFree(p->d_dc);
    delete p;
    return set_error(SPECENH_EHIP, std::string("plan allocation: ") + hipGetErrorString(e));
  }
  *plan = p;
  return SPECENH_OK;
}

int specenh_stft_plan_destroy(specenh_stft_plan* plan) {
  if (!plan) return SPECENH_OK;
  (void)hipFree(plan->d_window);
  (void)hipFree(plan->d_twiddle);
  (void)hipFree(plan->d_dc);
  delete plan;
  return SPECENH_OK;
}

size_t specenh_stft_workspace_bytes(const specenh_stft_plan* plan, long long batch) {
  (void)plan;
  return (size_t)(batch > 0 ? batch : 0) * 2 * sizeof(unsigned);
}

int specenh_stft_psd(const specenh_stft_plan* plan, const float* x, long long batch,
                     long long length, long long x_stride, float* out, int flags,
                     void* workspace, void* stream) {
  if (!plan) return set_error(SPECENH_EINVAL, "null plan");
  if (batch < 0) return set_error(SPECENH_EINVAL, "batch must be >= 0");
  if (batch == 0) return SPECENH_OK;
  if (!x || !out) return set_error(SPECENH_EINVAL, "null x/out");
  const int N = plan->nperseg;
  long long T = specenh_stft_frames(length, N, plan->noverlap);
  if (T < 0) return (int)T;
  if (x_stride < length) return set_error(SPECENH_EINVAL, "x_stride < length");
  if (T > (1ll << 30)) return set_error(SPECENH_EINVAL, "too many frames");
  if (flags & SPECENH_STFT_NORMALIZE) {
    if (!workspace) return set_error(SPECENH_EINVAL, "NORMALIZE needs a workspace");
  }
  hipStream_t st = (hipStream_t)stream;
  StftArgs a{};
  a.x = x;
  a.x_stride = x_stride;
  a.T = (int)T;
  a.hop = plan->hop;
  a.scale = (float)plan->scale;
  a.eps = (float)plan->eps;
  a.inv_kk = (float)(12.0 / ((double)N * ((double)N * N - 1.0)));
  a.detrend = plan->detrend;
  a.flags = flags;
  a.out = out;
  a.F_out = (flags & SPECENH_STFT_DROP_NYQUIST) ? N / 2 : N / 2 + 1;
  a.minmax = (unsigned*)workspace;
  a.window = plan->d_window;
  a.twiddle = plan->d_twiddle;
  a.dc_coef = plan->d_dc;
  const long long F_out = a.F_out;
  for (long long b0 = 0; b0 < batch; b0 += 65535) {
    const long long nb = std::min<long long>(65535, batch - b0);
    StftArgs c = a;
    c.x = x + b0 * x_stride;
    c.out = out + b0 * F_out * T;
    c.minmax = a.minmax ? a.minmax + 2 * b0 : nullptr;
    if (flags & SPECENH_STFT_NORMALIZE) {
      hipLaunchKernelGGL(minmax_init_kernel, dim3((unsigned)((nb + 255) / 256)), dim3(256), 0,
                         st, c.minmax, nb);
      SPECENH_HIP_CHECK(hipGetLastError());
    }
    hipError_t e;
    switch (N) {
      case 64: e = launch_stft<64>(c, nb, st); break;
      case 128: e = launch_stft<128>(c, nb, st); break;
      case 256: e = launch_stft<256>(c, nb, st); break;
      case 512: e = launch_stft<512>(c, nb, st); break;
      case 1024: e = launch_stft<1024>(c, nb, st); break;
      case 2048: e = launch_stft<2048>(c, nb, st); break;
      case 4096: e = launch_stft<4096>(c, nb, st); break;
      default: return set_error(SPECENH_EUNSUPPORTED, "unsupported nperseg");
    }
    if (e != hipSuccess)
      return set_error(SPECENH_EHIP, std::string("stft launch: ") + hipGetErrorString(e));
    if (flags & SPECENH_STFT_NORMALIZE) {
      const long long per_shot = F_out * T;
      unsigned gx = (unsigned)std::min<long long>((per_shot + 255) / 256, 64);
      hipLaunchKernelGGL(normalize_kernel, dim3(gx, (unsigned)nb), dim3(256), 0, st, c.out,
                         c.minmax, per_shot);
      SPECENH_HIP_CHECK(hipGetLastError());
    }
  }
  return SPECENH_OK;
}

}  // extern "C"
