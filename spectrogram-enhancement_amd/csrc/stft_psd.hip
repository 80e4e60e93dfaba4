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
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <string>
#include <vector>

#include "fft_common.hpp"
#include "specenh.h"

// Development-only flag bit (not part of the public header): skip the output store,
// to separate compute from store cost when profiling.
#define SPECENH_STFT_DEV_NOSTORE (1 << 16)

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
  const float* window;
  const float2* twiddle;  // per-pass [r-1][k] tables (TwOff<N>)
  const double* dc_coef;  // c_n: DC bin of the detrended, windowed frame = <x, c> (fp64)
};

// Per-N decomposition: G lanes per FFT, WAVES per workgroup, Stockham radices.
template <int N>
struct Cfg;
// G lanes own one FFT (two frames); WAVES per workgroup (one workgroup per CU: the
// LDS footprint is sized for that); R1 x R2 (x R3) Stockham radices; PF = prefetch the
// next tile's samples into registers while the current tile computes.
template <> struct Cfg<64>   { static constexpr int G = 8,  WAVES = 8, R1 = 8,  R2 = 8,  R3 = 1, PF = 1; };
template <> struct Cfg<128>  { static constexpr int G = 8,  WAVES = 8, R1 = 16, R2 = 8,  R3 = 1, PF = 1; };
template <> struct Cfg<256>  { static constexpr int G = 16, WAVES = 8, R1 = 16, R2 = 16, R3 = 1, PF = 1; };
template <> struct Cfg<512>  { static constexpr int G = 16, WAVES = 8, R1 = 32, R2 = 16, R3 = 1, PF = 1; };
template <> struct Cfg<1024> { static constexpr int G = 32, WAVES = 8, R1 = 32, R2 = 32, R3 = 1, PF = 1; };
template <> struct Cfg<2048> { static constexpr int G = 64, WAVES = 4, R1 = 32, R2 = 8,  R3 = 8, PF = 1; };
template <> struct Cfg<4096> { static constexpr int G = 64, WAVES = 2, R1 = 32, R2 = 16, R3 = 8, PF = 0; };

// Stockham pass p >= 2 of radix R at stride NS uses twiddles W_N^{r k N/(NS R)} for
// r in [1, R), k in [0, NS); stored as a [r-1][k] table so the lanes of a group read
// consecutive k (conflict-free). TwOff<N>::P2 / P3 are the per-pass table offsets.
template <int N>
struct TwOff {
  using C = Cfg<N>;
  static constexpr int P2 = 0;
  static constexpr int P3 = P2 + (C::R2 - 1) * C::R1;
  static constexpr int TOTAL = P3 + (C::R3 > 1 ? (C::R3 - 1) * C::R1 * C::R2 : 0);
};

template <int N>
struct Layout {
  using C = Cfg<N>;
  static constexpr int G = C::G;
  static constexpr int THREADS = 64 * C::WAVES;
  static constexpr int WPE = C::WAVES >= 8 ? C::WAVES / 4 : 1;  // waves per SIMD
  static constexpr int FFTS = C::WAVES * (64 / G);  // concurrent FFTs per workgroup
  static constexpr int TF = 2 * FFTS;                // frames per tile (power of two)
  static constexpr int LOG_TF = ilog2(TF);
  static constexpr int TS = TF + 1;                  // tile row stride (odd: conflict-free)
  static constexpr int NBINS = N / 2 + 1;
  static constexpr int IB = (NBINS + G - 1) / G;     // bins per lane in the epilogue
  static constexpr int BUF = N + N / 32;             // padded complex entries per FFT
  static constexpr int BUF_BYTES = FFTS * BUF * 8;
  static constexpr int TILE_BYTES = NBINS * TS * 4;  // aliases the FFT buffers
  static constexpr int TWN = TwOff<N>::TOTAL;
  // byte offsets into dynamic LDS (all multiples of 16)
  static constexpr int OFF_DC = 0;
  static constexpr int OFF_TW = OFF_DC + N * 8;
  static constexpr int OFF_WIN = OFF_TW + ((TWN * 8 + 15) / 16) * 16;
  static constexpr int OFF_BUF = OFF_WIN + N * 4;
  static constexpr int OFF_RED = OFF_BUF + (BUF_BYTES > TILE_BYTES ? BUF_BYTES : TILE_BYTES);
  static constexpr int BYTES = OFF_RED + 4 * C::WAVES * 4;
  static_assert(BYTES <= 160 * 1024, "LDS budget");
  static_assert(C::R1 * C::R2 * C::R3 == N, "radix product");
  static_assert((TF & (TF - 1)) == 0, "tile width must be a power of two");
};

__device__ __forceinline__ int pad(int e) { return e + (e >> 5); }

// min/max of three floats as one instruction each (plain fminf/fmaxf get NaN-quieting
// canonicalisation v_max ops on every operand). Operands are finite here or NaN only
// when the input itself is NaN.
__device__ __forceinline__ float fmin3(float a, float b, float c) {
  float r;
  asm("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ float fmax3(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// Workgroup barrier that orders LDS only: waits for this wave's LDS ops (lgkmcnt) and
// meets the other waves, but leaves global loads (the register prefetch) and global
// stores in flight. __syncthreads() would add s_waitcnt vmcnt(0) and serialise both.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// ---------------------------------------------------------------- lane-group sums
// Sum over aligned groups of G lanes, result in every lane of the group. DPP
// (quad_perm, row half-mirror, row mirror) inside a 16-lane row; ds_swizzle / a
// 32-lane shuffle above that.
template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, true));
}
template <int CTRL>
__device__ __forceinline__ double dppd(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xF, 0xF, true);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
template <int G, typename T>
__device__ __forceinline__ T group_sum(T v) {
  static_assert(G >= 4 && G <= 64, "group size");
  if constexpr (sizeof(T) == 4) {
    v += dppf<0xB1>(v);  // quad_perm [1,0,3,2]
    v += dppf<0x4E>(v);  // quad_perm [2,3,0,1]
    if constexpr (G >= 8) v += dppf<0x141>(v);   // row_half_mirror
    if constexpr (G >= 16) v += dppf<0x140>(v);  // row_mirror
  } else {
    v += dppd<0xB1>(v);
    v += dppd<0x4E>(v);
    if constexpr (G >= 8) v += dppd<0x141>(v);
    if constexpr (G >= 16) v += dppd<0x140>(v);
  }
  if constexpr (G >= 32) v += __shfl_xor(v, 16);
  if constexpr (G >= 64) v += __shfl_xor(v, 32);
  return v;
}

// Stockham pass NS>1 through the LDS buffer (all butterflies of the lane read first,
// then written back in place: legal because the whole FFT lives in one wave).
template <int N, int G, int R, int NS>
__device__ __forceinline__ void stockham_pass(float2* buf, const float2* tw /* [R-1][NS] */,
                                              int gl) {
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
    for (int r = 1; r < R; ++r) v[i][r] = cmul(v[i][r], tw[(r - 1) * NS + k]);
    fft_dif<R>(v[i]);
    const int base = (b / NS) * NS * R + k;
#pragma unroll
    for (int r = 0; r < R; ++r) buf[pad(base + bitrev(r, LOGR) * NS)] = v[i][r];
  }
  wave_lds_sync();
}

// acc += (double)x * c, as one opaque statement: hipcc otherwise converts all N/G
// samples to fp64 up front (2 VGPRs each) before running the FMA chain.
// v_cvt_f64_f32 -> v_fma_f64 is an ordinary VALU RAW dependency (interlocked).
__device__ __forceinline__ void dc_fma(double& acc, float x, double c) {
  double t;
  asm volatile("v_cvt_f64_f32 %1, %2\n\tv_fma_f64 %0, %1, %3, %0"
               : "+v"(acc), "=&v"(t)
               : "v"(x), "v"(c));
}

// Raw samples of one FFT pair as this lane holds them: x[.][r] = (frame a, frame b)
// at n = gl + i*G + r*NB1.
template <int N>
struct PairSamples {
  static constexpr int R1 = Cfg<N>::R1;
  static constexpr int BPL1 = (N / R1) / Cfg<N>::G;
  float2 x[BPL1][R1];
};

// Shot-local buffer descriptor (wave-uniform base, 32-bit offsets): every sample load
// and row store is then one VGPR offset + an immediate, not a 64-bit address pair.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0,
                                           (int)(bytes < 0x7fffffffll ? bytes : 0x7fffffffll),
                                           0x00020000);
}

// XH: the samples are fp16 (the C5 stream's shots), widened to fp32 on load (exact).
template <int N, bool XH = false>
__device__ __forceinline__ void load_pair(PairSamples<N>& s, __amdgpu_buffer_rsrc_t xr, int hop,
                                          int fa, int T, int gl) {
  constexpr int G = Cfg<N>::G;
  constexpr int NB1 = N / Cfg<N>::R1;
  constexpr int ES = XH ? 2 : 4;  // bytes per sample
  // Frames past the end duplicate the last frame: their spectra equal a valid one, so
  // they cannot move the min/max and need no masking; they are never stored.
  const int oa = ((fa < T ? fa : T - 1) * hop + gl) * ES;
  const int ob = ((fa + 1 < T ? fa + 1 : T - 1) * hop + gl) * ES;
#pragma unroll
  for (int i = 0; i < PairSamples<N>::BPL1; ++i)
#pragma unroll
    for (int r = 0; r < PairSamples<N>::R1; ++r) {
      const int o = (i * G + r * NB1) * ES;
      if constexpr (XH) {
        const unsigned short ha = __builtin_amdgcn_raw_buffer_load_b16(xr, oa + o, 0, 0);
        const unsigned short hb = __builtin_amdgcn_raw_buffer_load_b16(xr, ob + o, 0, 0);
        s.x[i][r] = make_float2((float)__builtin_bit_cast(_Float16, ha),
                                (float)__builtin_bit_cast(_Float16, hb));
      } else {
        s.x[i][r] = make_float2(
            __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, oa + o, 0, 0)),
            __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, ob + o, 0, 0)));
      }
    }
}

// Detrend + window + all FFT passes for one pair; leaves Z (natural order) in `buf`
// and returns the fp64 DC bins of both frames.
template <int N, bool XH = false>
__device__ __forceinline__ void fft_pair(const StftArgs& a, PairSamples<N>& in, bool va,
                                         bool vb, const float2* s_tw, const float* s_win,
                                         const double* s_dc, float2* buf, int gl, double& dca,
                                         double& dcb, __amdgpu_buffer_rsrc_t xr, int fa_next,
                                         bool prefetch) {
  using C = Cfg<N>;
  constexpr int G = C::G;
  constexpr int R1 = C::R1;
  constexpr int NB1 = N / R1;
  constexpr int BPL1 = NB1 / G;
  constexpr int LOGR1 = ilog2(R1);
  constexpr float kmid = 0.5f * float(N - 1);
  constexpr float invN = 1.0f / float(N);

  // DC bin in fp64: X_0 = sum_n w_n y_n = <x, c> with c = w - mean(w) - kc*sum(w kc)/sum(kc^2)
  // (c is orthogonal to constants and ramps, so the detrend cancellation happens exactly
  // in the coefficients, not in the data). After detrending X_0 is tiny by construction;
  // in fp32 it would sit at the rounding floor eps*||w y|| and, being the usual
  // spectrogram minimum under 'spectrum' scaling, would shift every normalised value.
  float2 v[BPL1][R1];
  float s0a = 0.f, s0b = 0.f, s1a = 0.f, s1b = 0.f;
  // 4 independent fp64 partial sums per frame: a single chain of R1 dependent
  // v_fma_f64 would be latency-bound.
  constexpr int NDC = 4;
  double pda[NDC] = {}, pdb[NDC] = {};
  const double* dcp = s_dc + gl;
#pragma unroll
  for (int i = 0; i < BPL1; ++i)
#pragma unroll
    for (int r = 0; r < R1; ++r) {
      const int j = i * G + r * NB1;
      const float xa_n = in.x[i][r].x, xb_n = in.x[i][r].y;
      v[i][r] = in.x[i][r];
      s0a += xa_n;
      s0b += xb_n;
      s1a = fmaf(float(j), xa_n, s1a);
      s1b = fmaf(float(j), xb_n, s1b);
      const double c = dcp[j];
      dc_fma(pda[(i * R1 + r) % NDC], xa_n, c);
      dc_fma(pdb[(i * R1 + r) % NDC], xb_n, c);
    }
  dca = (pda[0] + pda[1]) + (pda[2] + pda[3]);
  dcb = (pdb[0] + pdb[1]) + (pdb[2] + pdb[3]);
  // `in` is consumed: refill it with the next tile's samples now, so their HBM latency
  // hides under this pair's FFT (the fences keep the loads after the reads above).
  __builtin_amdgcn_sched_barrier(0);
  if (prefetch) load_pair<N, XH>(in, xr, a.hop, fa_next, a.T, gl);
  __builtin_amdgcn_sched_barrier(0);
  dca = group_sum<G>(dca);
  dcb = group_sum<G>(dcb);

  // Linear detrend in one sweep: mean and least-squares slope from the lane sums
  // S0 = sum x, S1 = sum j x (kc_n = kc0 + j with the lane base kc0 = gl - (N-1)/2 and
  // j = i*G + r*NB1 a compile-time offset, so per-register factors are immediates).
  // Only the DC bin is sensitive to the fp32 rounding of the fitted line (a coherent
  // error times sum(w)); it is taken from the fp64 path above instead.
  const float kc0 = float(gl) - kmid;
  float A_a = 0.f, A_b = 0.f, B_a = 0.f, B_b = 0.f;  // y = x - A - B*j
  if (a.detrend != SPECENH_DETREND_NONE) {
    s1a = fmaf(kc0, s0a, s1a);  // lane sums of kc*x
    s1b = fmaf(kc0, s0b, s1b);
    s0a = group_sum<G>(s0a);
    s0b = group_sum<G>(s0b);
    A_a = s0a * invN;
    A_b = s0b * invN;
    if (a.detrend == SPECENH_DETREND_LINEAR) {
      s1a = group_sum<G>(s1a);
      s1b = group_sum<G>(s1b);
      const float sa = s1a * a.inv_kk, sb = s1b * a.inv_kk;
      A_a = fmaf(sa, kc0, A_a);
      A_b = fmaf(sb, kc0, A_b);
      B_a = sa;
      B_b = sb;
    }
  }
  const float* win = s_win + gl;
#pragma unroll
  for (int i = 0; i < BPL1; ++i) {
    const int b = gl + i * G;
#pragma unroll
    for (int r = 0; r < R1; ++r) {
      const int j = i * G + r * NB1;
      const float w = win[j];
      const float ya = fmaf(-B_a, float(j), v[i][r].x - A_a);
      const float yb = fmaf(-B_b, float(j), v[i][r].y - A_b);
      v[i][r] = make_float2(w * ya, w * yb);
    }
    fft_dif<R1>(v[i]);
#pragma unroll
    for (int r = 0; r < R1; ++r) buf[pad(b * R1 + bitrev(r, LOGR1))] = v[i][r];
  }
  wave_lds_sync();
  stockham_pass<N, G, C::R2, R1>(buf, s_tw + TwOff<N>::P2, gl);
  if constexpr (C::R3 > 1) stockham_pass<N, G, C::R3, R1 * C::R2>(buf, s_tw + TwOff<N>::P3, gl);
}

// Separate the two frames of this lane group's FFT pair (Z in `buf`), PSD (+log2 / ln) of
// bins gl + i*G in registers, running min/max. DC bins come from the fp64 path.
template <int N>
__device__ __forceinline__ void pair_psd(const StftArgs& a, const float2* buf, int gl, double dca,
                                         double dcb, bool want_log, bool log2_out,
                                         float (&pv)[Layout<N>::IB][2], float& lmin, float& lmax) {
  using Lo = Layout<N>;
  constexpr int G = Cfg<N>::G;
  constexpr int IB = Lo::IB;
  const float scale_mid = 0.5f * a.scale, scale_end = 0.25f * a.scale;
#pragma unroll
  for (int i = 0; i < IB; ++i) {
    // bins k = gl + i*G: only i == 0 holds k = 0 (gl == 0), only i == IB-1 can hold
    // k = N/2 and k > N/2 (clamped to a duplicate of bin gl), all compile-time known.
    const int k = gl + i * G;
    const int kk = (i == IB - 1 && k >= Lo::NBINS) ? gl : k;
    const float2 zk = buf[pad(kk)];
    const float2 zm = buf[pad((N - kk) & (N - 1))];
    const float ar = zk.x + zm.x, ai = zk.y - zm.y;
    const float br = zk.x - zm.x, bi = zk.y + zm.y;
    float qa = fmaf(ar, ar, ai * ai);
    float qb = fmaf(br, br, bi * bi);
    float sc = scale_mid;
    if (i == IB - 1 && (N / 2) % G == 0) sc = (kk == N / 2) ? scale_end : scale_mid;
    float pa, pb;
    if (want_log) {
      pa = __log2f(fmaf(qa, sc, a.eps));
      pb = __log2f(fmaf(qb, sc, a.eps));
    } else {
      pa = qa * sc;
      pb = qb * sc;
    }
    if (i == 0) {  // DC of both frames from the fp64 path (lane gl == 0 only)
      const float da = (float)(dca * dca * (double)a.scale);
      const float db = (float)(dcb * dcb * (double)a.scale);
      if (gl == 0) {
        pa = want_log ? __log2f(da + a.eps) : da;
        pb = want_log ? __log2f(db + a.eps) : db;
      }
    }
    if (want_log && !log2_out) {
      pa *= 0.69314718055994530942f;
      pb *= 0.69314718055994530942f;
    }
    lmin = fmin3(lmin, pa, pb);
    lmax = fmax3(lmax, pa, pb);
    pv[i][0] = pa;
    pv[i][1] = pb;
  }
}

// The workgroup's (bins x TF frames) tile through LDS (it aliases the FFT buffers) and out
// as frequency-row segments out[k][t0 : t0 + tfv]; with `norm` each value is rescaled
// (v - mn) * inv on the way. Starts and ends with a workgroup LDS barrier.
template <int N>
__device__ __forceinline__ void tile_store(const StftArgs& a, float* s_tile,
                                           const float (&pv)[Layout<N>::IB][2], int gl, int fi,
                                           int tid, __amdgpu_buffer_rsrc_t orr, int t0, float mn,
                                           float inv, bool norm) {
  using Lo = Layout<N>;
  constexpr int G = Cfg<N>::G;
  constexpr int IB = Lo::IB;
  lds_barrier();  // every group is done with its FFT buffer: reuse as the tile
  const int fl = 2 * fi;
#pragma unroll
  for (int i = 0; i < IB; ++i) {
    const int k = gl + i * G;
    if (k < Lo::NBINS) {
      s_tile[k * Lo::TS + fl] = norm ? (pv[i][0] - mn) * inv : pv[i][0];
      s_tile[k * Lo::TS + fl + 1] = norm ? (pv[i][1] - mn) * inv : pv[i][1];
    }
  }
  lds_barrier();
  // ---- store frequency-row segments: out[shot][k][t0 : t0+tfv] ----
  // Compile-time trip count: the compiler can then count these stores in its partial
  // vmcnt waits for the prefetched samples instead of draining everything.
  const int tfv = min(Lo::TF, a.T - t0);
  if (!(a.flags & SPECENH_STFT_DEV_NOSTORE)) {
    constexpr int ST = (Lo::NBINS * Lo::TF + Lo::THREADS - 1) / Lo::THREADS;
    constexpr int ROWS_PER_IT = Lo::THREADS >> Lo::LOG_TF;
    const int k0 = tid >> Lo::LOG_TF;
    const int f = tid & (Lo::TF - 1);
    // one VGPR offset for all stores of this tile; the row step is a scalar soffset
    const int voff = (k0 * a.T + t0 + f) * 4;
    const int sstep = ROWS_PER_IT * a.T * 4;
    int soff = 0;
    asm volatile("" : "+s"(soff));  // opaque: keeps the 33 offsets from being hoisted
                                    // out of the tile loop into (spilled) SGPRs
#pragma unroll
    for (int it = 0; it < ST; ++it) {
      const int k = k0 + it * ROWS_PER_IT;
      if (k < a.F_out && f < tfv)
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(s_tile[k * Lo::TS + f]), orr,
                                              voff, soff, 0);
      soff += sstep;
    }
  }
  lds_barrier();  // tile (= FFT buffers) free for the next tile's FFTs
}

// One workgroup per spectrogram (shot): loops over tiles of TF frames. Tables are
// staged in LDS once per shot; each lane group's next-tile samples are prefetched
// into registers while the current tile computes. Per tile every lane group runs one
// FFT pair and keeps its PSD / log2-PSD values (IB bins x 2 frames) in registers;
// the FFT buffers are then reused as the (bins x frames) tile so the store writes
// frequency-row segments of TF frames. With NORMALIZE the workgroup knows the whole
// spectrogram's min/max at the end and rescales its own output in a final sweep
// (the rows were written moments ago and are re-read from the on-die caches).
template <int N, bool XH = false>
__global__ __launch_bounds__(Layout<N>::THREADS, Layout<N>::WPE) void stft_psd_kernel(
    StftArgs a) {
  using C = Cfg<N>;
  using Lo = Layout<N>;
  constexpr int G = C::G;
  constexpr int IB = Lo::IB;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* s_dc = reinterpret_cast<double*>(smem + Lo::OFF_DC);
  float2* s_tw = reinterpret_cast<float2*>(smem + Lo::OFF_TW);
  float* s_win = reinterpret_cast<float*>(smem + Lo::OFF_WIN);
  float* s_tile = reinterpret_cast<float*>(smem + Lo::OFF_BUF);
  float* s_red = reinterpret_cast<float*>(smem + Lo::OFF_RED);

  const int tid = threadIdx.x;
  const long long shot = blockIdx.x;
  for (int i = tid; i < Lo::TWN; i += Lo::THREADS) s_tw[i] = a.twiddle[i];
  for (int i = tid; i < N; i += Lo::THREADS) {
    s_win[i] = a.window[i];
    s_dc[i] = a.dc_coef[i];
  }

  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int gl = lane % G;                          // lane within the FFT group
  const int fi = wave * (64 / G) + lane / G;        // FFT index within the tile
  float2* buf = reinterpret_cast<float2*>(smem + Lo::OFF_BUF) + fi * Lo::BUF;
  constexpr int ES = XH ? 2 : 4;
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(
      reinterpret_cast<const char*>(a.x) + shot * a.x_stride * ES, a.x_stride * ES);
  const bool want_log = (a.flags & (SPECENH_STFT_LOG | SPECENH_STFT_NORMALIZE)) != 0;
  const bool log2_out = (a.flags & SPECENH_STFT_NORMALIZE) != 0;
  const int ntiles = (a.T + Lo::TF - 1) / Lo::TF;
  float* o_shot = a.out + shot * (long long)a.F_out * a.T;
  float lmin = INFINITY, lmax = -INFINITY;

  const __amdgpu_buffer_rsrc_t orr = make_rsrc(o_shot, (long long)a.F_out * a.T * 4);
  PairSamples<N> nxt;
  if constexpr (C::PF) load_pair<N, XH>(nxt, xr, a.hop, 2 * fi, a.T, gl);
  __syncthreads();

  for (int tile = 0; tile < ntiles; ++tile) {
    const int t0 = tile * Lo::TF;
    const int fa = t0 + 2 * fi;
    const bool va = true, vb = true;  // tail frames are clamped duplicates (load_pair)
    if constexpr (!C::PF) load_pair<N, XH>(nxt, xr, a.hop, fa, a.T, gl);
    double dca, dcb;
    fft_pair<N, XH>(a, nxt, va, vb, s_tw, s_win, s_dc, buf, gl, dca, dcb, xr, fa + Lo::TF,
                C::PF && tile + 1 < ntiles);

    // ---- separate the two frames, PSD (+log2/ln), running min/max; values in registers ----
    float pv[IB][2];
    pair_psd<N>(a, buf, gl, dca, dcb, want_log, log2_out, pv, lmin, lmax);
    tile_store<N>(a, s_tile, pv, gl, fi, tid, orr, t0, 0.f, 1.f, false);
  }

  if (a.flags & SPECENH_STFT_NORMALIZE) {
    // ---- whole-spectrogram min/max, then rescale this shot's rows in place ----
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
      lmin = fminf(lmin, __shfl_xor(lmin, m));
      lmax = fmaxf(lmax, __shfl_xor(lmax, m));
    }
    if (lane == 0) {
      s_red[wave] = lmin;
      s_red[C::WAVES + wave] = lmax;
    }
    __syncthreads();  // also orders this workgroup's row stores before the re-reads
    float mn = s_red[0], mx = s_red[C::WAVES];
#pragma unroll
    for (int w = 1; w < C::WAVES; ++w) {
      mn = fminf(mn, s_red[w]);
      mx = fmaxf(mx, s_red[C::WAVES + w]);
    }
    const float inv = 1.0f / (mx - mn);  // max == min -> NaN, as the reference's 0/0
    const long long total = (long long)a.F_out * a.T;
    const long long head = ((16 - ((size_t)o_shot & 15)) & 15) / 4;  // to 16-B alignment
    const long long h = head < total ? head : total;
    for (long long e = tid; e < h; e += Lo::THREADS) o_shot[e] = (o_shot[e] - mn) * inv;
    float4* o4 = reinterpret_cast<float4*>(o_shot + h);
    const long long n4 = (total - h) / 4;
    for (long long e = tid; e < n4; e += Lo::THREADS) {
      float4 q = o4[e];
      q.x = (q.x - mn) * inv;
      q.y = (q.y - mn) * inv;
      q.z = (q.z - mn) * inv;
      q.w = (q.w - mn) * inv;
      o4[e] = q;
    }
    for (long long e = h + 4 * n4 + tid; e < total; e += Lo::THREADS)
      o_shot[e] = (o_shot[e] - mn) * inv;
  }
}

template <int N, bool XH = false>
hipError_t launch_stft(const StftArgs& a, long long batch, hipStream_t stream) {
  using Lo = Layout<N>;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)stft_psd_kernel<N, XH>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, Lo::BYTES);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  hipLaunchKernelGGL((stft_psd_kernel<N, XH>), dim3((unsigned)batch), dim3(Lo::THREADS),
                     Lo::BYTES, stream, a);
  return hipGetLastError();
}


// ---------------------------------------------------------------- team schedule (NORMALIZE)
// The min-max normalisation (pipeline_data.py:34) needs a spectrogram's extremes before
// any of its values can be stored. stft_psd_kernel (one workgroup per shot) therefore
// re-reads and rewrites its whole output once (518 KB per C2 shot, mostly from beyond
// L2). Here a shot's frame tiles are computed by a TEAM of M workgroups, one tile each:
// a member keeps its tile in registers, publishes its local extremes as ONE 8-byte
// granule {maxkey, ~minkey} (an agent-scope store; both halves are nonzero for any
// non-NaN value, so the granule is its own ready flag), and stores its normalised tile
// once the team's M granules are in — every output byte is written exactly once.
// The grid is persistent and no larger than the device's resident capacity, so all
// members of a team are co-resident; tasks are pipelined: a workgroup publishes task i,
// computes task i+1, and only then waits for task i's team (deadlock-free by induction
// over i: every publish precedes the same workgroup's next wait). Correctness does not
// rest on co-residency (kernels on other streams or processes can break it): spins are
// bounded, and a member that gives up stores its tile un-normalised (raw log values),
// marks the tile in a flag array and sets the (sticky) timeout word, after which no
// member of the launch waits any more. team_fixup_kernel, launched behind the team kernel
// on the same stream, normalises exactly the marked tiles from the then-complete
// granules with the same arithmetic ((v - mn) * inv): bit-identical to the in-kernel path.
constexpr int TEAM_MAX = 64;           // one wave polls a team's granules
constexpr int STFT_DEV_NOTEAM = 1 << 17;     // development flag: force stft_psd_kernel
constexpr int STFT_DEV_FORCETEAM = 1 << 18;  // development flag: team even for small shots
constexpr int STFT_DEV_GIVEUP = 1 << 19;     // test flag: every team wait gives up at once

// Wave-wide: the team's extremes once all M granules are in (returns true), or false when
// the wait gave up (bounded spins, or another member already timed out in this launch).
__device__ __forceinline__ bool team_minmax(const unsigned long long* g, int M, int lane,
                                            unsigned* tmo, float& mn, float& mx,
                                            bool give_up) {
  unsigned long long v = 0;
  bool complete = true;
  if (give_up) {  // (test flag) exercise the raw-store + fixup path
    if (lane == 0) __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    complete = false;
  }
  for (unsigned spins = 0; complete; ++spins) {
    if (lane < M) v = __hip_atomic_load(g + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool ok = lane >= M || ((unsigned)v != 0u && (unsigned)(v >> 32) != 0u);
    if (__all(ok)) break;
    if (spins >= (1u << 20) ||
        __hip_atomic_load(tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) {
      if (lane == 0) __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      complete = false;
      break;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  unsigned kmax = lane < M ? (unsigned)v : 0u;
  unsigned kinv = lane < M ? (unsigned)(v >> 32) : 0u;
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    kmax = max(kmax, (unsigned)__shfl_xor((int)kmax, m));
    kinv = max(kinv, (unsigned)__shfl_xor((int)kinv, m));
  }
  mx = key2f(kmax);
  mn = key2f(~kinv);
  return complete;
}

template <int N>
__global__ __launch_bounds__(Layout<N>::THREADS, Layout<N>::WPE) void stft_team_kernel(
    StftArgs a, unsigned long long* gran, long long batch, int M, int Q, unsigned* tmo,
    unsigned char* tile_flag) {
  using C = Cfg<N>;
  using Lo = Layout<N>;
  constexpr int G = C::G;
  constexpr int IB = Lo::IB;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* s_dc = reinterpret_cast<double*>(smem + Lo::OFF_DC);
  float2* s_tw = reinterpret_cast<float2*>(smem + Lo::OFF_TW);
  float* s_win = reinterpret_cast<float*>(smem + Lo::OFF_WIN);
  float* s_tile = reinterpret_cast<float*>(smem + Lo::OFF_BUF);
  float* s_red = reinterpret_cast<float*>(smem + Lo::OFF_RED);  // [2*WAVES] + team {mn, mx}

  if ((int)blockIdx.x >= Q * M) return;  // whole workgroup: spare slots of the grid
  const int tid = threadIdx.x;
  const int q = blockIdx.x / M, mem = blockIdx.x - (blockIdx.x / M) * M;
  for (int i = tid; i < Lo::TWN; i += Lo::THREADS) s_tw[i] = a.twiddle[i];
  for (int i = tid; i < N; i += Lo::THREADS) {
    s_win[i] = a.window[i];
    s_dc[i] = a.dc_coef[i];
  }
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int gl = lane % G;
  const int fi = wave * (64 / G) + lane / G;
  float2* buf = reinterpret_cast<float2*>(smem + Lo::OFF_BUF) + fi * Lo::BUF;
  const int t0 = mem * Lo::TF;  // this member's tile: frames [t0, t0 + TF)
  const int fa = t0 + 2 * fi;
  const long long ntask = (batch - q + Q - 1) / Q;  // shots q, q + Q, ... < batch
  const long long plane = (long long)a.F_out * a.T;
  const long long xbytes = a.x_stride * 4;

  PairSamples<N> nxt;
  load_pair<N>(nxt, make_rsrc(a.x + q * a.x_stride, xbytes), a.hop, fa, a.T, gl);
  float pvp[IB][2];
#pragma unroll
  for (int i = 0; i < IB; ++i) pvp[i][0] = pvp[i][1] = 0.f;
  __syncthreads();

  for (long long it = 0; it <= ntask; ++it) {
    const long long shot = q + it * Q;
    const bool cur = it < ntask;
    float pvc[IB][2];
    float lmin = INFINITY, lmax = -INFINITY;
    if (cur) {
      const bool pf = it + 1 < ntask;
      const __amdgpu_buffer_rsrc_t xn = make_rsrc(a.x + (pf ? shot + Q : shot) * a.x_stride, xbytes);
      double dca, dcb;
      fft_pair<N>(a, nxt, true, true, s_tw, s_win, s_dc, buf, gl, dca, dcb, xn, fa, pf);
      float dmin = INFINITY, dmax = -INFINITY;  // (pair_psd's running extremes: unused)
      pair_psd<N>(a, buf, gl, dca, dcb, true, true, pvc, dmin, dmax);
      // the tile's extremes from the held values themselves (the v_min3/v_max3 running
      // pair in pair_psd came out wrong in this kernel's schedule: measured on gfx950)
#pragma unroll
      for (int i = 0; i < IB; ++i) {
        lmin = fminf(lmin, fminf(pvc[i][0], pvc[i][1]));
        lmax = fmaxf(lmax, fmaxf(pvc[i][0], pvc[i][1]));
      }
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
      lmin = fminf(lmin, __shfl_xor(lmin, m));
      lmax = fmaxf(lmax, __shfl_xor(lmax, m));
    }
    if (lane == 0) {
      s_red[wave] = lmin;
      s_red[C::WAVES + wave] = lmax;
    }
    lds_barrier();  // s_red complete; every lane is done reading its FFT buffer
    if (cur && tid == 0) {
      float mn = s_red[0], mx = s_red[C::WAVES];
#pragma unroll
      for (int w = 1; w < C::WAVES; ++w) {
        mn = fminf(mn, s_red[w]);
        mx = fmaxf(mx, s_red[C::WAVES + w]);
      }
      const unsigned long long gv =
          ((unsigned long long)(~f2key(mn)) << 32) | (unsigned long long)f2key(mx);
      __hip_atomic_store(gran + shot * M + mem, gv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (it > 0) {  // the previous task's tile: team extremes, normalise, store
      const long long sp = shot - Q;
      if (wave == 0) {
        float mn, mx;
        const bool done = team_minmax(gran + sp * M, M, lane, tmo, mn, mx,
                                      (a.flags & STFT_DEV_GIVEUP) != 0);
        if (lane == 0) {
          s_red[2 * C::WAVES] = mn;
          s_red[2 * C::WAVES + 1] = mx;
          s_red[2 * C::WAVES + 2] = done ? 1.f : 0.f;
          if (!done) tile_flag[sp * M + mem] = 1;  // raw tile: team_fixup_kernel finishes it
        }
      }
      lds_barrier();
      const float mn = s_red[2 * C::WAVES];
      const float inv = 1.0f / (s_red[2 * C::WAVES + 1] - mn);  // max == min -> NaN (0/0)
      const bool done = s_red[2 * C::WAVES + 2] != 0.f;
      const __amdgpu_buffer_rsrc_t orr = make_rsrc(a.out + sp * plane, plane * 4);
      tile_store<N>(a, s_tile, pvp, gl, fi, tid, orr, t0, mn, inv, done);
    } else {
      lds_barrier();  // s_red is rewritten by the next task only after thread 0 read it
    }
    if (cur) {
#pragma unroll
      for (int i = 0; i < IB; ++i) {
        pvp[i][0] = pvc[i][0];
        pvp[i][1] = pvc[i][1];
      }
    }
  }
}

// Normalises the tiles a team kernel stored raw (tile_flag set), from the granules, which
// are complete once that kernel has finished. Returns at once when no wait timed out.
__global__ __launch_bounds__(256) void team_fixup_kernel(float* out, int F_out, int T, int TF,
                                                         const unsigned long long* gran,
                                                         const unsigned char* tile_flag,
                                                         long long batch, int M,
                                                         const unsigned* tmo) {
  if (*tmo == 0u) return;  // uniform: the common case, every tile normalised in-kernel
  const long long plane = (long long)F_out * T;
  for (long long task = blockIdx.x; task < batch * M; task += gridDim.x) {
    if (!tile_flag[task]) continue;  // uniform per workgroup
    const long long shot = task / M;
    const int mem = (int)(task - shot * M);
    unsigned kmax = 0u, kinv = 0u;
    for (int j = 0; j < M; ++j) {
      const unsigned long long v = gran[shot * M + j];
      kmax = max(kmax, (unsigned)v);
      kinv = max(kinv, (unsigned)(v >> 32));
    }
    const float mx = key2f(kmax), mn = key2f(~kinv);
    const float inv = 1.0f / (mx - mn);
    const int t0 = mem * TF, tw = min(TF, T - t0);
    float* o = out + shot * plane + t0;
    for (int e = threadIdx.x; e < F_out * tw; e += blockDim.x) {
      const int k = e / tw, t = e - (e / tw) * tw;
      o[(long long)k * T + t] = (o[(long long)k * T + t] - mn) * inv;
    }
  }
}

// Launch the team schedule when it applies (NORMALIZE, workspace given, team size <=
// TEAM_MAX and <= the resident capacity). *launched = false: the caller falls back.
template <int N>
hipError_t launch_team(const StftArgs& a, long long batch, void* workspace, hipStream_t stream,
                       bool* launched) {
  using Lo = Layout<N>;
  *launched = false;
  const int M = (a.T + Lo::TF - 1) / Lo::TF;
  if (M > TEAM_MAX) return hipSuccess;
  static int cap[64] = {};  // resident workgroups per device (0 = not queried)
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  if (dev < 0 || dev >= 64) return hipSuccess;
  if (cap[dev] == 0) {
    e = hipFuncSetAttribute((const void*)stft_team_kernel<N>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, Lo::BYTES);
    if (e != hipSuccess) return e;
    int per_cu = 0, cus = 0;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)stft_team_kernel<N>,
                                                     Lo::THREADS, Lo::BYTES);
    if (e != hipSuccess) return e;
    e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (e != hipSuccess) return e;
    // never trust the occupancy answer alone (co-residency is a correctness condition
    // here): bound it by the register file (512 VGPR+AGPR per lane and SIMD, 8-register
    // granules, 4 SIMDs per CU) and by LDS as well
    hipFuncAttributes fa{};
    e = hipFuncGetAttributes(&fa, (const void*)stft_team_kernel<N>);
    if (e != hipSuccess) return e;
    const int regs = ((fa.numRegs + 7) / 8) * 8;
    const int waves_per_simd = regs > 0 ? std::min(8, 512 / regs) : 8;
    const int by_regs = waves_per_simd * 4 / Cfg<N>::WAVES;
    const int by_lds = (160 * 1024) / Lo::BYTES;
    per_cu = std::min(per_cu, std::min(by_regs, by_lds));
    cap[dev] = per_cu * cus > 0 ? per_cu * cus : -1;
  }
  if (cap[dev] < M) return hipSuccess;
  long long Q = cap[dev] / M;
  if (Q > batch) Q = batch;
  // workspace: [timeout word, 16 B][granules: batch x M x 8 B][tile flags: batch x M B],
  // zeroed every call (specenh_stft_workspace_bytes sizes it for M = TEAM_MAX)
  unsigned* tmo = reinterpret_cast<unsigned*>(workspace);
  unsigned long long* gran =
      reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(workspace) + 16);
  unsigned char* tflag = reinterpret_cast<unsigned char*>(gran + (size_t)batch * M);
  const size_t zero = 16 + (size_t)batch * M * 9;
  e = hipMemsetAsync(workspace, 0, zero, stream);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(stft_team_kernel<N>, dim3((unsigned)(Q * M)), dim3(Lo::THREADS), Lo::BYTES,
                     stream, a, gran, batch, M, (int)Q, tmo, tflag);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(team_fixup_kernel, dim3(1024), dim3(256), 0, stream, a.out, a.F_out, a.T,
                     Lo::TF, gran, tflag, batch, M, tmo);
  e = hipGetLastError();
  *launched = e == hipSuccess;
  return e;
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
  std::vector<float2> tw;
  auto add_pass = [&](int R, int NS) {  // [r-1][k] = W_N^{r k N/(NS R)}
    for (int r = 1; r < R; ++r)
      for (int k = 0; k < NS; ++k) {
        ct::CS cs = ct::cossin_frac((long long)r * k * (N / (NS * R)), N);
        tw.push_back(make_float2(float(cs.c), float(-cs.s)));
      }
  };
  switch (N) {
#define SPECENH_TW_CASE(NN)                                                              \
  case NN:                                                                               \
    add_pass(Cfg<NN>::R2, Cfg<NN>::R1);                                                  \
    if (Cfg<NN>::R3 > 1) add_pass(Cfg<NN>::R3, Cfg<NN>::R1 * Cfg<NN>::R2);               \
    break;
    SPECENH_TW_CASE(64) SPECENH_TW_CASE(128) SPECENH_TW_CASE(256) SPECENH_TW_CASE(512)
    SPECENH_TW_CASE(1024) SPECENH_TW_CASE(2048) SPECENH_TW_CASE(4096)
#undef SPECENH_TW_CASE
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
  if (e == hipSuccess) e = hipMalloc(&p->d_twiddle, tw.size() * sizeof(float2));
  if (e == hipSuccess) e = hipMalloc(&p->d_dc, N * sizeof(double));
  if (e == hipSuccess) e = hipMemcpy(p->d_dc, dc.data(), N * sizeof(double), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(p->d_window, win.data(), N * sizeof(float), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(p->d_twiddle, tw.data(), tw.size() * sizeof(float2), hipMemcpyHostToDevice);
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
  if (batch <= 0) return 16;
  return 16 + (size_t)batch * TEAM_MAX * 9;  // team schedule: timeout word, granules, flags
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
  a.window = plan->d_window;
  a.twiddle = plan->d_twiddle;
  a.dc_coef = plan->d_dc;
  const long long F_out = a.F_out;
  // team schedule for large spectrograms (C2: 518 KB each); small ones (C5: 64 KB) are
  // re-read from L2 by the sweep for less than the team's hand-off costs (measured)
  const bool team = (F_out * T * 4 >= (256ll << 10)) || (flags & STFT_DEV_FORCETEAM);
  if ((flags & SPECENH_STFT_NORMALIZE) && workspace && !(flags & STFT_DEV_NOTEAM) && team &&
      batch <= (1ll << 30)) {
    bool launched = false;
    hipError_t e = hipSuccess;
    switch (N) {
      case 64: e = launch_team<64>(a, batch, workspace, st, &launched); break;
      case 128: e = launch_team<128>(a, batch, workspace, st, &launched); break;
      case 256: e = launch_team<256>(a, batch, workspace, st, &launched); break;
      case 512: e = launch_team<512>(a, batch, workspace, st, &launched); break;
      case 1024: e = launch_team<1024>(a, batch, workspace, st, &launched); break;
      default: break;  // 2048 / 4096: the held tile would spill; one workgroup per shot
    }
    if (e != hipSuccess)
      return set_error(SPECENH_EHIP, std::string("stft team launch: ") + hipGetErrorString(e));
    if (launched) return SPECENH_OK;
  }
  for (long long b0 = 0; b0 < batch; b0 += 1 << 30) {
    const long long nb = std::min<long long>(1 << 30, batch - b0);
    StftArgs c = a;
    c.x = x + b0 * x_stride;
    c.out = out + b0 * F_out * T;
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
  }
  return SPECENH_OK;
}

int specenh_stft_psd_f16(const specenh_stft_plan* plan, const void* x, long long batch,
                         long long length, long long x_stride, float* out, int flags,
                         void* stream) {
  if (!plan) return set_error(SPECENH_EINVAL, "null plan");
  if (batch < 0) return set_error(SPECENH_EINVAL, "batch must be >= 0");
  if (batch == 0) return SPECENH_OK;
  if (!x || !out) return set_error(SPECENH_EINVAL, "null x/out");
  const int N = plan->nperseg;
  long long T = specenh_stft_frames(length, N, plan->noverlap);
  if (T < 0) return (int)T;
  if (x_stride < length) return set_error(SPECENH_EINVAL, "x_stride < length");
  if (T > (1ll << 30)) return set_error(SPECENH_EINVAL, "too many frames");
  if (N > 1024) return set_error(SPECENH_EUNSUPPORTED, "fp16 samples need nperseg <= 1024");
  StftArgs a{};
  a.x = reinterpret_cast<const float*>(x);  // reinterpreted as fp16 by stft_psd_kernel<N, true>
  a.x_stride = x_stride;
  a.T = (int)T;
  a.hop = plan->hop;
  a.scale = (float)plan->scale;
  a.eps = (float)plan->eps;
  a.inv_kk = (float)(12.0 / ((double)N * ((double)N * N - 1.0)));
  a.detrend = plan->detrend;
  a.flags = flags;
  a.F_out = (flags & SPECENH_STFT_DROP_NYQUIST) ? N / 2 : N / 2 + 1;
  a.window = plan->d_window;
  a.twiddle = plan->d_twiddle;
  a.dc_coef = plan->d_dc;
  hipStream_t st = (hipStream_t)stream;
  const long long F_out = a.F_out;
  for (long long b0 = 0; b0 < batch; b0 += 1 << 30) {
    const long long nb = std::min<long long>(1 << 30, batch - b0);
    StftArgs c = a;
    c.x = reinterpret_cast<const float*>(reinterpret_cast<const _Float16*>(x) + b0 * x_stride);
    c.out = out + b0 * F_out * T;
    hipError_t e;
    switch (N) {
      case 64: e = launch_stft<64, true>(c, nb, st); break;
      case 128: e = launch_stft<128, true>(c, nb, st); break;
      case 256: e = launch_stft<256, true>(c, nb, st); break;
      case 512: e = launch_stft<512, true>(c, nb, st); break;
      case 1024: e = launch_stft<1024, true>(c, nb, st); break;
      default: return set_error(SPECENH_EUNSUPPORTED, "unsupported nperseg");
    }
    if (e != hipSuccess)
      return set_error(SPECENH_EHIP, std::string("stft launch: ") + hipGetErrorString(e));
  }
  return SPECENH_OK;
}

}  // extern "C"
