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

#ifndef SPECENH_C1024_WAVES
#define SPECENH_C1024_WAVES 4
#define SPECENH_C1024_OCC 3
#endif
#ifndef SPECENH_C1024_PF
#define SPECENH_C1024_PF 1
#endif
#ifndef SPECENH_STFT_WIDE_EMIT
#define SPECENH_STFT_WIDE_EMIT 1
#endif
#ifndef SPECENH_STFT_STORE_AUX
#define SPECENH_STFT_STORE_AUX 0  // cache-policy bits of the spectrogram stores
#endif
#ifndef SPECENH_STFT_PF_AFTER_WAIT
#define SPECENH_STFT_PF_AFTER_WAIT 1
#endif
#ifndef SPECENH_STFT_BUFPAD
#define SPECENH_STFT_BUFPAD 1  // bank offset between the FFT buffers of one 32-lane half
#endif
#ifndef SPECENH_STFT_PF_EARLY
#define SPECENH_STFT_PF_EARLY 0
#endif
#include "specenh.h"
#include "runtime.hpp"

// Development-only flag bit (not part of the public header): skip the output store,
// to separate compute from store cost when profiling.
#define SPECENH_STFT_DEV_NOSTORE (1 << 16)
// Profiling only: every prefetch re-reads frames 0-1 of its shot (L2 hits, no HBM reads).
#define SPECENH_STFT_DEV_NOLOAD (1 << 21)

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
  // DC bin of the detrended, windowed frame = <x, c> in fp64 with
  // c_n = w_n - dc_alpha - dc_beta (n - (N-1)/2), w the fp32 window (see pair_spectrum)
  double dc_alpha;
  double dc_beta;
  const double* dc_coef;  // the same c_n as a table (fp64), staged in LDS when it fits
  // cross spectrum (stft_team_kernel MODE 3): the second signal of each pair
  const float* y;
  long long y_stride;
};

// Per-N decomposition: G lanes per FFT, WAVES per workgroup, Stockham radices.
template <int N>
struct Cfg;
// G lanes own one FFT (two frames); WAVES per workgroup; OCC = resident workgroups per CU
// the LDS and register budgets are sized for; R1 x R2 (x R3) Stockham radices; PF =
// prefetch the next tile's samples into registers while the current tile computes.
// N = 1024 (C2): 4-wave workgroups, 3 per CU (168 VGPRs, 47 KB LDS each), so one
// workgroup's barriers, team wait and store burst overlap two others' FFTs.
template <> struct Cfg<64>   { static constexpr int G = 8,  WAVES = 8, OCC = 1, R1 = 8,  R2 = 8,  R3 = 1, PF = 1; };
template <> struct Cfg<128>  { static constexpr int G = 8,  WAVES = 8, OCC = 1, R1 = 16, R2 = 8,  R3 = 1, PF = 1; };
template <> struct Cfg<256>  { static constexpr int G = 16, WAVES = 8, OCC = 1, R1 = 16, R2 = 16, R3 = 1, PF = 1; };
template <> struct Cfg<512>  { static constexpr int G = 16, WAVES = 8, OCC = 1, R1 = 32, R2 = 16, R3 = 1, PF = 1; };
template <> struct Cfg<1024> { static constexpr int G = 32, WAVES = SPECENH_C1024_WAVES, OCC = SPECENH_C1024_OCC, R1 = 32, R2 = 32, R3 = 1, PF = SPECENH_C1024_PF; };
template <> struct Cfg<2048> { static constexpr int G = 64, WAVES = 4, OCC = 1, R1 = 32, R2 = 8,  R3 = 8, PF = 1; };
template <> struct Cfg<4096> { static constexpr int G = 64, WAVES = 2, OCC = 1, R1 = 32, R2 = 16, R3 = 8, PF = 0; };

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

constexpr int align16(int b) { return (b + 15) / 16 * 16; }
constexpr int lds_granules(int b) { return (b + 2047) / 2048 * 2048; }

template <int N>
struct Layout {
  using C = Cfg<N>;
  static constexpr int G = C::G;
  static constexpr int THREADS = 64 * C::WAVES;
  static constexpr int WPE = C::OCC * C::WAVES >= 4 ? C::OCC * C::WAVES / 4 : 1;  // waves/SIMD
  static constexpr int FFTS = C::WAVES * (64 / G);  // concurrent FFTs per workgroup
  static constexpr int TF = 2 * FFTS;                // frames per tile (power of two)
  static constexpr int LOG_TF = ilog2(TF);
  // Tile rows: odd stride TF + 1 (conflict-free 4-B writes), or for G = 32 unpadded
  // (TS = TF) with an XOR swizzle of the frame index, element (k, f) at
  // k TS + (f ^ swz(k)), swz(k) = ((k / (64/TF)) & (TF/2 - 1)) << 1: each lane's two
  // frames go out as one 8-B write, writes (rows gl + 32 i) and row reads (64/TF rows x
  // TF frames per wave) are conflict-free, and the tile is no larger than the FFT buffers.
  static constexpr bool TILE_SWZ = G == 32 && (TF == 16 || TF == 32);
  static constexpr int TS = TILE_SWZ ? TF : TF + 1;
  static constexpr int NBINS = N / 2 + 1;
  static constexpr int IB = (NBINS + G - 1) / G;     // bins per lane in the epilogue
  // per-FFT exchange buffer: N padded FLOATS (real and imaginary parts take turns), plus a
  // bank offset between the FFTs that share a 32-lane half (G = 8, 16): at BUF = N + N/32 the
  // neighbouring FFTs' contiguous 16-element reads overlapped on 8 banks (2-way conflicts in
  // every exchange read); the extra 4 / 8 floats put them on disjoint banks (tools/lds_banks.py:
  // N = 256 exchange reads 284 -> 160 LDS cycles per FFT pass pair, writes unchanged)
  static constexpr int BUF =
      N + N / 32 + (SPECENH_STFT_BUFPAD ? (G == 16 ? 8 : (G == 8 ? 4 : 0)) : 0);
  static constexpr int BUF_BYTES = FFTS * BUF * 4;
  static constexpr int TILE_BYTES = NBINS * TS * 4;  // aliases the FFT buffers
  static constexpr int TWN = TwOff<N>::TOTAL;
  // + 16 B: the mirror read of lane 0 (see pair_spectrum) may touch one float past the
  // last FFT buffer
  static constexpr int REGION = align16((BUF_BYTES > TILE_BYTES ? BUF_BYTES : TILE_BYTES) + 16);
  static constexpr int RED_BYTES = 4 * C::WAVES * 4;  // [2*WAVES] + team {mn, mx, done}
  static constexpr int BASE_BYTES = align16(TWN * 8) + align16(N * 4) + REGION + RED_BYTES;
  // the fp64 DC coefficient table goes to LDS when OCC workgroups still fit with it;
  // otherwise pair_spectrum forms the coefficients from the window (3 more fp64 ops/sample)
  // (budget in 2-KB allocation granules: a table that only fits to the byte cost one
  // resident workgroup per CU when measured, 1.44 -> 1.79 ms at C2)
  static constexpr bool DC_TABLE = lds_granules(BASE_BYTES + N * 8) * C::OCC <= 160 * 1024;
  // byte offsets into dynamic LDS (all multiples of 16)
  static constexpr int OFF_TW = 0;
  static constexpr int OFF_WIN = OFF_TW + align16(TWN * 8);
  static constexpr int OFF_DC = OFF_WIN + align16(N * 4);
  static constexpr int OFF_BUF = OFF_DC + (DC_TABLE ? N * 8 : 0);
  static constexpr int OFF_RED = OFF_BUF + REGION;
  static constexpr int BYTES = OFF_RED + RED_BYTES;
  static_assert(lds_granules(BYTES) * C::OCC <= 160 * 1024, "LDS budget");
  static_assert(C::R1 * C::R2 * C::R3 == N, "radix product");
  static_assert((TF & (TF - 1)) == 0, "tile width must be a power of two");
  static_assert(4 * C::WAVES >= 2 * C::WAVES + 3, "reduction scratch");
};

__device__ __forceinline__ int pad(int e) { return e + (e >> 5); }

template <int N>
__device__ __forceinline__ int tile_swz(int k) {
  using Lo = Layout<N>;
  if constexpr (Lo::TILE_SWZ) return ((k / (64 / Lo::TF)) & (Lo::TF / 2 - 1)) << 1;
  return 0;
}

// min/max of three floats as one instruction each (plain fminf/fmaxf get NaN-quieting
// canonicalisation v_max ops on every operand). Operands are finite here or NaN only
// when the input itself is NaN. hipcc pads no hazard inside an asm statement, and the
// operands come straight from v_log_f32 (a transcendental: a VALU read of its result
// needs wait states), so the pad is in the string: without it the max read a stale
// register in some schedules (the held-tile kernel's extremes came out O(1) wrong).
__device__ __forceinline__ float fmin3(float a, float b, float c) {
  float r;
  asm("s_nop 1\n\tv_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ float fmax3(float a, float b, float c) {
  float r;
  asm("s_nop 1\n\tv_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
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

// Split exchange through one per-FFT float buffer: the register array `w` of one stage
// (element (i, r) holds FFT index WI(i, r)) becomes the next stage's `v` (element (i, r)
// = FFT index RI(i, r)); real parts first, then imaginary parts, so the buffer is N
// floats instead of N complex values. Wave-local (the FFT lives in one wave).
template <int WB, int WR, int RB, int RR, class WI, class RI>
__device__ __forceinline__ void split_exchange(float* buf, const f2v (&w)[WB][WR], f2v (&v)[RB][RR],
                                               WI wi, RI ri) {
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int i = 0; i < WB; ++i)
#pragma unroll
      for (int r = 0; r < WR; ++r) buf[pad(wi(i, r))] = w[i][r][h];
    wave_lds_sync();
#pragma unroll
    for (int i = 0; i < RB; ++i)
#pragma unroll
      for (int r = 0; r < RR; ++r) v[i][r][h] = buf[pad(ri(i, r))];
    wave_lds_sync();
  }
}

// Stockham pass of radix R at stride NS on registers loaded by split_exchange from FFT
// indices b + r*N/R (b = gl + i*G): twiddles from the LDS table, then the in-register DIF.
// Element (i, r) then holds FFT index stockham_out<N, G, R, NS>(gl, i, r).
template <int N, int G, int R, int NS>
__device__ __forceinline__ int stockham_out(int gl, int i, int r) {
  const int b = gl + i * G;
  return (b / NS) * NS * R + b % NS + bitrev(r, ilog2(R)) * NS;
}
template <int N, int G, int R, int NS>
__device__ __forceinline__ void stockham_compute(f2v (&v)[(N / R) / G][R], const f2v* tw, int gl) {
  constexpr int BPL = (N / R) / G;
#pragma unroll
  for (int i = 0; i < BPL; ++i) {
    const int k = (gl + i * G) % NS;
#pragma unroll
    for (int r = 1; r < R; ++r) {
      v[i][r] = pk::cmul(v[i][r], tw[(r - 1) * NS + k]);
      // twiddles in chunks of 8: the scheduler would otherwise hoist all R-1 table reads
      // (2 VGPRs each) ahead of the multiplies
      if (r % 8 == 7) __builtin_amdgcn_sched_barrier(0);
    }
    fft_dif<R>(v[i]);
  }
}

// acc += (double)x * c, as one opaque statement: hipcc otherwise converts all N/G
// samples to fp64 up front (2 VGPRs each) before running the FMA chain.
// v_cvt_f64_f32 -> v_fma_f64 is an ordinary VALU RAW dependency (interlocked).
__device__ __forceinline__ void dc_fma(double& acc, float x, double c) {
  double t;
  asm("v_cvt_f64_f32 %1, %2\n\tv_fma_f64 %0, %1, %3, %0" : "+v"(acc), "=&v"(t) : "v"(x), "v"(c));
}

// Raw samples of one FFT pair as this lane holds them: x[.][r] = (frame a, frame b)
// at n = gl + i*G + r*NB1.
template <int N>
struct PairSamples {
  static constexpr int R1 = Cfg<N>::R1;
  static constexpr int BPL1 = (N / R1) / Cfg<N>::G;
  f2v x[BPL1][R1];  // {frame a, frame b} sample pairs
};

// Shot-local buffer descriptor (wave-uniform base, 32-bit offsets): every sample load
// and row store is then one VGPR offset + an immediate, not a 64-bit address pair.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0,
                                           (int)(bytes < 0x7fffffffll ? bytes : 0x7fffffffll),
                                           0x00020000);
}

// XH: the samples are fp16 (the C5 stream's shots), widened to fp32 on load (exact).
// XY: the pair is frame fa of two signals (x from xr, y from yr: the cross spectrum);
// otherwise frames fa and fa + 1 of one signal (yr is unused).
template <int N, bool XH = false, bool XY = false>
__device__ __forceinline__ void load_pair(PairSamples<N>& s, __amdgpu_buffer_rsrc_t xr,
                                          __amdgpu_buffer_rsrc_t yr, int hop, int fa, int T,
                                          int gl) {
  constexpr int G = Cfg<N>::G;
  constexpr int NB1 = N / Cfg<N>::R1;
  constexpr int ES = XH ? 2 : 4;  // bytes per sample
  // Frames past the end duplicate the last frame: their spectra equal a valid one, so
  // they cannot move the min/max and need no masking; they are never stored.
  const int oa = ((fa < T ? fa : T - 1) * hop + gl) * ES;
  const int ob = XY ? oa : ((fa + 1 < T ? fa + 1 : T - 1) * hop + gl) * ES;
  const __amdgpu_buffer_rsrc_t br = XY ? yr : xr;
  // The per-register offset o goes in the scalar soffset operand (an SGPR constant): as a
  // VGPR add it would cost one VALU op per load (the compiler does not fold it into the
  // instruction's immediate offset).
  // (opaque base: the N/G constants are re-formed by SALU adds here rather than hoisted
  // out of the tile loop into N/G live SGPRs)
  int sbase = 0;
  asm volatile("" : "+s"(sbase));
#pragma unroll
  for (int i = 0; i < PairSamples<N>::BPL1; ++i)
#pragma unroll
    for (int r = 0; r < PairSamples<N>::R1; ++r) {
      const int o = sbase + (i * G + r * NB1) * ES;
      if constexpr (XH) {
        const unsigned short ha = __builtin_amdgcn_raw_buffer_load_b16(xr, oa, o, 0);
        const unsigned short hb = __builtin_amdgcn_raw_buffer_load_b16(br, ob, o, 0);
        s.x[i][r] = f2v{(float)__builtin_bit_cast(_Float16, ha),
                        (float)__builtin_bit_cast(_Float16, hb)};
      } else {
        s.x[i][r] = f2v{__uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, oa, o, 0)),
                        __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(br, ob, o, 0))};
      }
    }
}

// One FFT pair end to end: detrend + window + all FFT passes (split exchanges through the
// lane group's float buffer `buf`), then the two frames' separation, PSD (+ log2 / ln) of
// bins gl + i*G into pv[i] = (frame a, frame b) and the running min/max. DC bins come
// from the fp64 path. With `prefetch`, the next tile's samples are loaded into `nxt` while
// this pair computes (`in` and `nxt` may be the same set: `in` is consumed first).
template <int N, bool XH = false, bool XY = false>
__device__ __forceinline__ void pair_spectrum(const StftArgs& a, const PairSamples<N>& in,
                                              PairSamples<N>& nxt, const f2v* s_tw,
                                              const float* s_win, const double* s_dc,
                                              float* buf, int gl,
                                              double dc_base, __amdgpu_buffer_rsrc_t xr,
                                              __amdgpu_buffer_rsrc_t yr, int fa_next, bool prefetch, bool want_log,
                                              bool log2_out, f2v (&pv)[Layout<N>::IB],
                                              float& lmin, float& lmax) {
  using C = Cfg<N>;
  using Lo = Layout<N>;
  constexpr int G = C::G;
  constexpr int R1 = C::R1;
  constexpr int NB1 = N / R1;
  constexpr int BPL1 = NB1 / G;
  constexpr int LOGR1 = ilog2(R1);
  constexpr float kmid = 0.5f * float(N - 1);
  constexpr float invN = 1.0f / float(N);
  constexpr int IB = Lo::IB;
  constexpr bool PF_EARLY = SPECENH_STFT_PF_EARLY;

  // DC bin in fp64: X_0 = sum_n w_n y_n = <x, c> with c = w - mean(w) - kc*sum(w kc)/sum(kc^2)
  // (c is orthogonal to constants and ramps, so the detrend cancellation happens exactly
  // in the coefficients, not in the data). After detrending X_0 is tiny by construction;
  // in fp32 it would sit at the rounding floor eps*||w y|| and, being the usual
  // spectrogram minimum under 'spectrum' scaling, would shift every normalised value.
  // c_n comes from the LDS table (Layout::DC_TABLE) or is formed here from the fp32
  // window as c_n = (w_n - dc_base) - beta * j (dc_base = alpha + beta * (gl - kmid) per
  // lane); both are the same fp64 coefficients up to fp64 rounding.
  f2v s0 = {0.f, 0.f}, s1 = {0.f, 0.f};  // per frame (a, b): sum x, sum j x
  // 4 independent fp64 partial sums per frame: a single chain of R1 dependent
  // v_fma_f64 would be latency-bound.
  constexpr int NDC = 4;
  double pda[NDC] = {}, pdb[NDC] = {};
  const float* win = s_win + gl;
#pragma unroll
  for (int i = 0; i < BPL1; ++i)
#pragma unroll
    for (int r = 0; r < R1; ++r) {
      const int j = i * G + r * NB1;
      const f2v xv = in.x[i][r];
      s0 += xv;
      s1 = __builtin_elementwise_fma(f2v{float(j), float(j)}, xv, s1);
      double c;
      if constexpr (Lo::DC_TABLE)
        c = s_dc[gl + j];
      else
        c = __builtin_fma(-a.dc_beta, double(j), (double)win[j] - dc_base);
      dc_fma(pda[(i * R1 + r) % NDC], xv.x, c);
      dc_fma(pdb[(i * R1 + r) % NDC], xv.y, c);
      if ((i * R1 + r) % 8 == 7) __builtin_amdgcn_sched_barrier(0);
    }
  // memory clobber: the windowing below re-reads win[j] from LDS instead of keeping the
  // N/G values read above live across the detrend sums (CSE would add N/G VGPRs)
  asm volatile("" ::: "memory");
  double dca = (pda[0] + pda[1]) + (pda[2] + pda[3]);
  double dcb = (pdb[0] + pdb[1]) + (pdb[2] + pdb[3]);
  dca = group_sum<G>(dca);
  dcb = group_sum<G>(dcb);

  // Linear detrend in one sweep: mean and least-squares slope from the lane sums
  // S0 = sum x, S1 = sum j x (kc_n = kc0 + j with the lane base kc0 = gl - (N-1)/2 and
  // j = i*G + r*NB1 a compile-time offset, so per-register factors are immediates).
  // Only the DC bin is sensitive to the fp32 rounding of the fitted line (a coherent
  // error times sum(w)); it is taken from the fp64 path above instead.
  const float kc0 = float(gl) - kmid;
  f2v A = {0.f, 0.f}, nB = {0.f, 0.f};  // y = x - A - B*j (nB = -B)
  if (a.detrend != SPECENH_DETREND_NONE) {
    s1 = __builtin_elementwise_fma(f2v{kc0, kc0}, s0, s1);  // lane sums of kc*x
    s0 = f2v{group_sum<G>(s0.x), group_sum<G>(s0.y)};
    A = s0 * invN;
    if (a.detrend == SPECENH_DETREND_LINEAR) {
      const f2v sl = f2v{group_sum<G>(s1.x), group_sum<G>(s1.y)} * a.inv_kk;
      A = __builtin_elementwise_fma(sl, f2v{kc0, kc0}, A);
      nB = -sl;
    }
  }
  f2v v1[BPL1][R1];
#pragma unroll
  for (int i = 0; i < BPL1; ++i) {
#pragma unroll
    for (int r = 0; r < R1; ++r) {
      const int j = i * G + r * NB1;
      const f2v y = __builtin_elementwise_fma(nB, f2v{float(j), float(j)}, in.x[i][r] - A);
      v1[i][r] = y * win[j];
    }
    fft_dif<R1>(v1[i]);
  }
  // `in` is consumed; the next tile's samples are loaded once the Stockham passes are
  // done (below): issued earlier, the 64 in-flight sample registers on top of a pass's
  // 64 data registers spill under the 168-VGPR budget of Cfg<1024>::OCC = 3

  // `prefetch` is compile-time per configuration and unconditional at run time: a
  // conditional load would keep the consumed samples live (the "not loaded" path) when
  // `nxt` is `in`. Past the last tile the clamped frames / repeated shot are re-read.
  auto issue_prefetch = [&]() {  // fences keep the loads after the FFT's reads of `in`
    __builtin_amdgcn_sched_barrier(0);
    if (prefetch)
      load_pair<N, XH, XY>(nxt, xr, yr, a.hop, (a.flags & SPECENH_STFT_DEV_NOLOAD) ? 0 : fa_next,
                           a.T, gl);
    __builtin_amdgcn_sched_barrier(0);
  };
  // ---- Stockham passes 2 (and 3) ----
  constexpr int R2 = C::R2, R3 = C::R3;
  if constexpr (PF_EARLY) issue_prefetch();
  f2v v2[(N / R2) / G][R2];
  split_exchange(buf, v1, v2, [&](int i, int r) { return (gl + i * G) * R1 + bitrev(r, LOGR1); },
                 [&](int i, int r) { return gl + i * G + r * (N / R2); });
  stockham_compute<N, G, R2, R1>(v2, s_tw + TwOff<N>::P2, gl);

  // ---- final split exchange: Z[k] and Z[N - k] for bins k = gl + i*G ----
  // Mirror-bin index pad((N - k) & (N - 1)). For G a multiple of 32 it is affine in i:
  // zmb - (G + G/32) i, so all IB reads share one address register (otherwise the
  // compiler hoists IB lane-dependent addresses out of the tile loop and spills them).
  // Lane gl == 0 at i == 0 reads one slot past its FFT buffer (still inside the LDS
  // allocation, Layout::OFF_RED): that value is bin 0's, which the fp64 DC path replaces.
  const int zmb = N + N / 32 - gl + ((-gl) >> 5);
  auto kk_of = [&](int i) {  // bins k > N/2 (only at i == IB-1) duplicate bin gl
    const int k = gl + i * G;
    return (i == IB - 1 && k >= Lo::NBINS) ? gl : k;
  };
  auto mi_of = [&](int i) {
    const int k = gl + i * G;
    const bool dup = i == IB - 1 && k >= Lo::NBINS;
    if constexpr (G % 32 == 0) return dup ? zmb : zmb - (G + G / 32) * i;
    return pad((N - kk_of(i)) & (N - 1));
  };
  // The two frames' powers accumulate across the real and imaginary halves of the
  // exchange: q = ((Re Z_k + Re Z_m)^2 + (Im Z_k - Im Z_m)^2,
  //                (Re Z_k - Re Z_m)^2 + (Im Z_k + Im Z_m)^2) = 4 (|A_k|^2, |B_k|^2)
  // (m = N - k), so only IB pairs stay live between the halves, not 2 IB complex values.
  f2v q[IB];
  auto final_exchange = [&](const auto& vf, auto out_index) {
    constexpr int FB = sizeof(vf) / sizeof(vf[0]);
    constexpr int FR = sizeof(vf[0]) / sizeof(vf[0][0]);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int i = 0; i < FB; ++i)
#pragma unroll
        for (int r = 0; r < FR; ++r) buf[pad(out_index(i, r))] = vf[i][r][h];
      wave_lds_sync();
#pragma unroll
      for (int i = 0; i < IB; ++i) {
        const float zk = buf[pad(kk_of(i))], zm = buf[mi_of(i)];
        const f2v t = h == 0 ? f2v{zk + zm, zk - zm} : f2v{zk - zm, zk + zm};
        q[i] = h == 0 ? t * t : __builtin_elementwise_fma(t, t, q[i]);
      }
      wave_lds_sync();
    }
  };
  if constexpr (R3 > 1) {
    f2v v3[(N / R3) / G][R3];
    split_exchange(buf, v2, v3,
                   [&](int i, int r) { return stockham_out<N, G, R2, R1>(gl, i, r); },
                   [&](int i, int r) { return gl + i * G + r * (N / R3); });
    stockham_compute<N, G, R3, R1 * R2>(v3, s_tw + TwOff<N>::P3, gl);
    if constexpr (!PF_EARLY) issue_prefetch();
    final_exchange(v3, [&](int i, int r) { return stockham_out<N, G, R3, R1 * R2>(gl, i, r); });
  } else {
    if constexpr (!PF_EARLY) issue_prefetch();
    final_exchange(v2, [&](int i, int r) { return stockham_out<N, G, R2, R1>(gl, i, r); });
  }

  // ---- separate the two frames, PSD (+log2/ln), running min/max ----
  const float scale_mid = 0.5f * a.scale, scale_end = 0.25f * a.scale;
#pragma unroll
  for (int i = 0; i < IB; ++i) {
    // bins k = gl + i*G: only i == 0 holds k = 0 (gl == 0), only i == IB-1 can hold
    // k = N/2 and k > N/2 (clamped to a duplicate of bin gl), all compile-time known.
    const int kk = kk_of(i);
    float sc = scale_mid;
    if (i == IB - 1 && (N / 2) % G == 0) sc = (kk == N / 2) ? scale_end : scale_mid;
    float pa, pb;
    if (want_log) {
      pa = __log2f(fmaf(q[i].x, sc, a.eps));
      pb = __log2f(fmaf(q[i].y, sc, a.eps));
    } else {
      pa = q[i].x * sc;
      pb = q[i].y * sc;
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
    pv[i] = f2v{pa, pb};
  }
}

// The workgroup's (bins x TF frames) tile through LDS (it aliases the FFT buffers): each
// lane group writes its bins for its two frames (raw, or rescaled (v - mn) * inv with
// `norm`); no barriers here.
template <int N>
__device__ __forceinline__ void tile_write(float* s_tile, const f2v (&pv)[Layout<N>::IB], int gl,
                                           int fi, float mn, float inv, bool norm) {
  using Lo = Layout<N>;
  constexpr int G = Cfg<N>::G;
  constexpr int IB = Lo::IB;
  const int fl = 2 * fi;
#pragma unroll
  for (int i = 0; i < IB; ++i) {
    const int k = gl + i * G;
    if (k < Lo::NBINS) {
      const f2v t = norm ? (pv[i] - mn) * inv : pv[i];
      if constexpr (Lo::TILE_SWZ) {
        *reinterpret_cast<f2v*>(s_tile + k * Lo::TS + (fl ^ tile_swz<N>(k))) = t;
      } else {
        s_tile[k * Lo::TS + fl] = t.x;
        s_tile[k * Lo::TS + fl + 1] = t.y;
      }
    }
  }
}

// The tile out as frequency-row segments out[k][t0 : t0 + tfv]; with `norm` each value is
// rescaled (v - mn) * inv on the way (the same arithmetic as tile_write's). No barriers.
// Branch-free: rows k >= F_out land past the end of the shot's buffer descriptor
// (num_records = F_out * T * 4) and frames past T get an offset beyond it, so the
// hardware drops exactly those stores (the host keeps a plane below 2^30 bytes).
// Compile-time trip count: the compiler can then count these stores in its partial
// vmcnt waits for the prefetched samples instead of draining everything.
template <int N>
__device__ __forceinline__ void tile_emit(const StftArgs& a, const float* s_tile, int tid,
                                          __amdgpu_buffer_rsrc_t orr, int t0, float mn, float inv,
                                          bool norm) {
  using Lo = Layout<N>;
  const int tfv = min(Lo::TF, a.T - t0);
  if (a.flags & SPECENH_STFT_DEV_NOSTORE) return;
  constexpr int ST = (Lo::NBINS * Lo::TF + Lo::THREADS - 1) / Lo::THREADS;
  constexpr int ROWS_PER_IT = Lo::THREADS >> Lo::LOG_TF;
  constexpr int GRP = 12;  // LDS reads issued ahead of their stores
  const int k0 = tid >> Lo::LOG_TF;
  const int f = tid & (Lo::TF - 1);
  // one VGPR offset for all stores of this tile; the row step is a scalar soffset
  const int voff = f < tfv ? (k0 * a.T + t0 + f) * 4 : (1 << 30);
  const int sstep = ROWS_PER_IT * a.T * 4;
  // With the swizzled tile, rows k0 + it * ROWS_PER_IT take two swizzle values that
  // alternate with `it` (the row step moves the swizzle key by half its range).
  constexpr int SWZ_STEP =
      Lo::TILE_SWZ ? ((ROWS_PER_IT / (64 / Lo::TF)) & (Lo::TF / 2 - 1)) << 1 : 0;
  static_assert(!Lo::TILE_SWZ || ((2 * (ROWS_PER_IT / (64 / Lo::TF))) % (Lo::TF / 2)) == 0,
                "swizzle must alternate over row groups");
  const float* src0 = s_tile + k0 * Lo::TS + (f ^ tile_swz<N>(k0));
  const float* src1 = s_tile + k0 * Lo::TS + (f ^ (tile_swz<N>(k0) ^ SWZ_STEP));
#pragma unroll
  for (int g0 = 0; g0 < ST; g0 += GRP) {
    float v[GRP];
#pragma unroll
    for (int u = 0; u < GRP; ++u) {
      const int it = g0 + u;
      if (it < ST && it * ROWS_PER_IT < Lo::NBINS) {
        if ((it + 1) * ROWS_PER_IT <= Lo::NBINS) {
          v[u] = ((it & 1) ? src1 : src0)[it * ROWS_PER_IT * Lo::TS];
        } else {  // last, partial row group: rows past the tile re-read its last row (their
                  // stores fall past the descriptor's end anyway)
          const int k = min(k0 + it * ROWS_PER_IT, Lo::NBINS - 1);
          v[u] = s_tile[k * Lo::TS + (f ^ tile_swz<N>(k))];
        }
        if (norm) v[u] = (v[u] - mn) * inv;
      }
    }
#pragma unroll
    for (int u = 0; u < GRP; ++u)
      if (g0 + u < ST && (g0 + u) * ROWS_PER_IT < Lo::NBINS)
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v[u]), orr, voff, (g0 + u) * sstep,
                                              SPECENH_STFT_STORE_AUX);
  }
}

// tile_emit for the swizzled 16-frame tile (G = 32, TF = 16: nperseg 1024) with 16-byte
// stores: lane (row k, quad q) reads frames 4q .. 4q + 3 of row k as one ds_read_b128 and
// writes them with one buffer_store_dwordx4 (dword-aligned: rows are T = 253 floats apart),
// instead of four ds_read_b32 + four 4-byte stores. The tile's XOR swizzle moves frame f of
// row k to f ^ s(k), s even: the quad lands at quad q ^ (s >> 2), its two pairs swapped when
// s & 2. A quad with frames past T (the row's last member tile) goes out as dwords, the
// invalid ones past the descriptor (dropped). Same arithmetic as tile_emit.
template <int N>
__device__ __forceinline__ void tile_emit4(const StftArgs& a, const float* s_tile, int tid,
                                           __amdgpu_buffer_rsrc_t orr, int t0, float mn,
                                           float inv, bool norm) {
  using Lo = Layout<N>;
  static_assert(Lo::TILE_SWZ && Lo::TF == 16, "16-frame swizzled tile");
  const int tfv = min(Lo::TF, a.T - t0);
  if (a.flags & SPECENH_STFT_DEV_NOSTORE) return;
  constexpr int ROWS_PER_IT = Lo::THREADS / 4;
  constexpr int ST = (Lo::NBINS + ROWS_PER_IT - 1) / ROWS_PER_IT;
  const int q = tid & 3, k0 = tid >> 2;
  const bool whole = 4 * q + 3 < tfv;
  const int voff = (k0 * a.T + t0 + 4 * q) * 4;
  const int sstep = ROWS_PER_IT * a.T * 4;
#pragma unroll
  for (int it = 0; it < ST; ++it) {
    const int k = min(k0 + it * ROWS_PER_IT, Lo::NBINS - 1);  // rows past the tile: re-read
    const int sw = tile_swz<N>(k);
    const float4 r = *reinterpret_cast<const float4*>(s_tile + k * Lo::TS + 4 * (q ^ (sw >> 2)));
    float v[4];
    const bool swp = (sw & 2) != 0;
    v[0] = swp ? r.z : r.x;
    v[1] = swp ? r.w : r.y;
    v[2] = swp ? r.x : r.z;
    v[3] = swp ? r.y : r.w;
    if (norm) {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = (v[j] - mn) * inv;
    }
    // rows k >= F_out fall past the descriptor (num_records = F_out T 4 bytes): dropped
    const int row_ok = k0 + it * ROWS_PER_IT < Lo::NBINS;
    const int off = row_ok ? voff : (1 << 30);
    if (whole) {
      typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
      __builtin_amdgcn_raw_buffer_store_b128(
          u32x4{__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]),
                __float_as_uint(v[3])},
          orr, off, it * sstep, SPECENH_STFT_STORE_AUX);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v[j]), orr,
                                              4 * q + j < tfv ? off + 4 * j : (1 << 30),
                                              it * sstep, SPECENH_STFT_STORE_AUX);
    }
  }
}

// tile_write + tile_emit between workgroup LDS barriers: starts with one (every group is
// done with its FFT buffer) unless the caller has just passed one, ends with one (the
// tile = FFT buffers free for the next tile's FFTs).
template <int N>
__device__ __forceinline__ void tile_store(const StftArgs& a, float* s_tile,
                                           const f2v (&pv)[Layout<N>::IB], int gl, int fi,
                                           int tid, __amdgpu_buffer_rsrc_t orr, int t0, float mn,
                                           float inv, bool norm, bool lead_barrier = true) {
  if (lead_barrier) lds_barrier();
  tile_write<N>(s_tile, pv, gl, fi, mn, inv, norm);
  lds_barrier();
  tile_emit<N>(a, s_tile, tid, orr, t0, 0.f, 1.f, false);
  lds_barrier();
}

// Cross-spectrum tiles (stft_team_kernel MODE 3): one frame per lane group, so the tile is
// FFTS = TF / 2 frames wide, NBINS rows at an odd stride TS1 (the 4-B writes of a lane
// group's bins k = gl + i G land in distinct banks). Same barrier discipline as tile_store.
template <int N>
struct Tile1 {
  using Lo = Layout<N>;
  static constexpr int TF1 = Lo::FFTS;
  static constexpr int LOG_TF1 = ilog2(TF1);
  static constexpr int TS1 = TF1 + 1;
  static_assert(Lo::NBINS * TS1 * 4 <= Lo::REGION - 16, "one-frame tile fits the FFT buffers");
  static_assert(Lo::THREADS % TF1 == 0, "row groups");
};

template <int N>
__device__ __forceinline__ void tile_store1(const StftArgs& a, float* s_tile,
                                            const float (&pv)[Layout<N>::IB], int gl, int fi,
                                            int tid, __amdgpu_buffer_rsrc_t orr, int t0) {
  using Lo = Layout<N>;
  using T1 = Tile1<N>;
  constexpr int G = Cfg<N>::G;
  lds_barrier();  // every group is done with its FFT buffer
#pragma unroll
  for (int i = 0; i < Lo::IB; ++i) {
    const int k = gl + i * G;
    if (k < Lo::NBINS) s_tile[k * T1::TS1 + fi] = pv[i];
  }
  lds_barrier();
  // rows out as segments out[k][t0 : t0 + TF1]; rows past F_out and frames past T fall
  // outside the descriptor (dropped), as in tile_emit
  const int tfv = min(T1::TF1, a.T - t0);
  constexpr int ROWS_PER_IT = Lo::THREADS >> T1::LOG_TF1;
  constexpr int ST = (Lo::NBINS + ROWS_PER_IT - 1) / ROWS_PER_IT;
  constexpr int GRP = 9;
  const int k0 = tid >> T1::LOG_TF1;
  const int f = tid & (T1::TF1 - 1);
  const int voff = f < tfv ? (k0 * a.T + t0 + f) * 4 : (1 << 30);
  const int sstep = ROWS_PER_IT * a.T * 4;
#pragma unroll
  for (int g0 = 0; g0 < ST; g0 += GRP) {
    float v[GRP];
#pragma unroll
    for (int u = 0; u < GRP; ++u)
      if (g0 + u < ST) v[u] = s_tile[min(k0 + (g0 + u) * ROWS_PER_IT, Lo::NBINS - 1) * T1::TS1 + f];
#pragma unroll
    for (int u = 0; u < GRP; ++u)
      if (g0 + u < ST)
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v[u]), orr, voff, (g0 + u) * sstep, 0);
  }
  lds_barrier();  // tile (= FFT buffers) free for the next tile's FFTs
}

// Per-lane base of the DC coefficients: alpha + beta * (gl - (N-1)/2).
template <int N>
__device__ __forceinline__ double dc_lane_base(const StftArgs& a, int gl) {
  return a.dc_alpha + a.dc_beta * (double(gl) - 0.5 * double(N - 1));
}

// One workgroup per spectrogram (shot): loops over tiles of TF frames. Tables are
// staged in LDS once per shot; each lane group's next-tile samples are prefetched
// into registers while the current tile computes. Per tile every lane group runs one
// FFT pair and keeps its PSD / log2-PSD values (IB bins x 2 frames) in registers;
// the FFT buffers are then reused as the (bins x frames) tile so the store writes
// frequency-row segments of TF frames. With NORMALIZE the workgroup knows the whole
// spectrogram's min/max at the end and rescales its own output in a final sweep
// (the rows were written moments ago and are re-read from the on-die caches).
// HOLD (NORMALIZE, a spectrogram of HOLD <= 2 tiles: the C5 stream's 128 frames at
// nperseg 256): every tile's values stay in the lane groups' registers (HOLD x IB pairs)
// until the extremes are known, and each tile is stored once, normalised on its way through
// the LDS tile — no raw store, no re-read, no second write. PMC had the sweep at 454 MB per
// 2048 C5 shots for 202 MB of algorithmic traffic: the raw rows of the 2 x 32 resident shots
// per XCD (4 MB) do not stay in its 4 MB L2. Same arithmetic ((v - mn) * inv); the two
// instantiations' FFT code is scheduled differently, so values agree to an ulp or so of the
// log2 PSD (<= 1e-6 on [0, 1], measured; N = 512 bitwise), not bit for bit.
//
// EXACT (SPECENH_STFT_EXACT, the numpy-compat entries specgr / specgr_array): one real frame
// per complex FFT, its partner the zero frame (the loads go through a zero-length buffer
// descriptor, which returns 0). A lane group runs its tile's two frames as two FFTs, so the
// tile layout, the normalising sweep and the stores are unchanged. The two-for-one
// separation hands bin k of frame a the partner frame's fp32 rounding at the same bin, which
// at a spectral null of frame a is relatively large (tools/stft_pair_error.py: ln-PSD error
// 1.5e-4 paired, 3.7e-5 against a zero partner). Twice the FFT work: not a throughput path.
template <int N, bool XH = false, int HOLD = 0, bool EXACT = false>
__global__ __launch_bounds__(Layout<N>::THREADS, Layout<N>::WPE) void stft_psd_kernel(
    StftArgs a) {
  using C = Cfg<N>;
  using Lo = Layout<N>;
  constexpr int G = C::G;
  constexpr int IB = Lo::IB;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  f2v* s_tw = reinterpret_cast<f2v*>(smem + Lo::OFF_TW);
  float* s_win = reinterpret_cast<float*>(smem + Lo::OFF_WIN);
  float* s_tile = reinterpret_cast<float*>(smem + Lo::OFF_BUF);
  float* s_red = reinterpret_cast<float*>(smem + Lo::OFF_RED);

  const int tid = threadIdx.x;
  const long long shot = blockIdx.x;
  for (int i = tid; i < Lo::TWN; i += Lo::THREADS) s_tw[i] = f2v{a.twiddle[i].x, a.twiddle[i].y};
  for (int i = tid; i < N; i += Lo::THREADS) s_win[i] = a.window[i];
  double* s_dc = reinterpret_cast<double*>(smem + Lo::OFF_DC);
  if constexpr (Lo::DC_TABLE)
    for (int i = tid; i < N; i += Lo::THREADS) s_dc[i] = a.dc_coef[i];

  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int gl = lane % G;                          // lane within the FFT group
  const int fi = wave * (64 / G) + lane / G;        // FFT index within the tile
  float* buf = reinterpret_cast<float*>(smem + Lo::OFF_BUF) + fi * Lo::BUF;
  constexpr int ES = XH ? 2 : 4;
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(
      reinterpret_cast<const char*>(a.x) + shot * a.x_stride * ES, a.x_stride * ES);
  const bool want_log = (a.flags & (SPECENH_STFT_LOG | SPECENH_STFT_NORMALIZE)) != 0;
  const bool log2_out = (a.flags & SPECENH_STFT_NORMALIZE) != 0;
  const int ntiles = (a.T + Lo::TF - 1) / Lo::TF;
  float* o_shot = a.out + shot * (long long)a.F_out * a.T;
  float lmin = INFINITY, lmax = -INFINITY;
  const double dcb = dc_lane_base<N>(a, gl);

  const __amdgpu_buffer_rsrc_t orr = make_rsrc(o_shot, (long long)a.F_out * a.T * 4);
  PairSamples<N> s0;
  const __amdgpu_buffer_rsrc_t zr = make_rsrc(a.x, 0);  // EXACT: the zero partner frame
  if constexpr (EXACT) {
    if constexpr (C::PF) load_pair<N, XH, true>(s0, xr, zr, a.hop, 2 * fi, a.T, gl);
  } else if constexpr (C::PF) {
    load_pair<N, XH>(s0, xr, xr, a.hop, 2 * fi, a.T, gl);
  }
  __syncthreads();

  if constexpr (EXACT) {
    static_assert(HOLD == 0, "exact mode runs the sweep schedule");
    for (int tile = 0; tile < ntiles; ++tile) {
      const int t0 = tile * Lo::TF;
      const int fa = t0 + 2 * fi;  // frames fa, fa + 1: one FFT each
      f2v pv[IB], pw[IB];
      float dmn = INFINITY, dmx = -INFINITY;  // (the zero frame's values: unused)
      if constexpr (!C::PF) load_pair<N, XH, true>(s0, xr, zr, a.hop, fa, a.T, gl);
      pair_spectrum<N, XH, true>(a, s0, s0, s_tw, s_win, s_dc, buf, gl, dcb, xr, zr, fa + 1,
                                 C::PF != 0, want_log, log2_out, pv, dmn, dmx);
      if constexpr (!C::PF) load_pair<N, XH, true>(s0, xr, zr, a.hop, fa + 1, a.T, gl);
      // the second FFT re-uses the lane group's buffer: its first exchange writes only after
      // the group's own reads of the first (wave-local, ordered by wave_lds_sync)
      pair_spectrum<N, XH, true>(a, s0, s0, s_tw, s_win, s_dc, buf, gl, dcb, xr, zr,
                                 fa + Lo::TF, C::PF != 0, want_log, log2_out, pw, dmn, dmx);
#pragma unroll
      for (int i = 0; i < IB; ++i) {
        pv[i].y = pw[i].x;
        lmin = fminf(lmin, fminf(pv[i].x, pv[i].y));
        lmax = fmaxf(lmax, fmaxf(pv[i].x, pv[i].y));
      }
      tile_store<N>(a, s_tile, pv, gl, fi, tid, orr, t0, 0.f, 1.f, false);
    }
  } else if constexpr (HOLD > 0) {  // (host-checked: NORMALIZE, ntiles == HOLD)
    f2v pv[HOLD][IB];
#pragma unroll
    for (int tile = 0; tile < HOLD; ++tile) {
      const int fa = tile * Lo::TF + 2 * fi;
      if constexpr (!C::PF) load_pair<N, XH>(s0, xr, xr, a.hop, fa, a.T, gl);
      pair_spectrum<N, XH>(a, s0, s0, s_tw, s_win, s_dc, buf, gl, dcb, xr, xr, fa + Lo::TF,
                           C::PF != 0 && tile + 1 < HOLD, want_log, log2_out, pv[tile], lmin,
                           lmax);
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
    __syncthreads();  // s_red complete; every group is done with its FFT buffer
    float mn = s_red[0], mx = s_red[C::WAVES];
#pragma unroll
    for (int w = 1; w < C::WAVES; ++w) {
      mn = fminf(mn, s_red[w]);
      mx = fmaxf(mx, s_red[C::WAVES + w]);
    }
    const float inv = 1.0f / (mx - mn);  // max == min -> NaN, as the reference's 0/0
#pragma unroll
    for (int tile = 0; tile < HOLD; ++tile)
      tile_store<N>(a, s_tile, pv[tile], gl, fi, tid, orr, tile * Lo::TF, mn, inv, true,
                    tile > 0);
    return;
  }
  if constexpr (!EXACT) {
    for (int tile = 0; tile < ntiles; ++tile) {
      const int t0 = tile * Lo::TF;
      const int fa = t0 + 2 * fi;  // tail frames are clamped duplicates (load_pair)
      if constexpr (!C::PF) load_pair<N, XH>(s0, xr, xr, a.hop, fa, a.T, gl);
      f2v pv[IB];
      pair_spectrum<N, XH>(a, s0, s0, s_tw, s_win, s_dc, buf, gl, dcb, xr, xr, fa + Lo::TF,
                           C::PF != 0, want_log, log2_out, pv, lmin, lmax);
      tile_store<N>(a, s_tile, pv, gl, fi, tid, orr, t0, 0.f, 1.f, false);
    }
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
    if (e == hipSuccess)
      e = hipFuncSetAttribute((const void*)stft_psd_kernel<N, XH, 0, true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, Lo::BYTES);
    if constexpr (N <= 512)
      for (const void* k : {(const void*)stft_psd_kernel<N, XH, 1>, (const void*)stft_psd_kernel<N, XH, 2>})
        if (e == hipSuccess)
          e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, Lo::BYTES);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  if (a.flags & SPECENH_STFT_EXACT) {
    SPECENH_LAUNCH((stft_psd_kernel<N, XH, 0, true>), dim3((unsigned)batch), dim3(Lo::THREADS),
                   Lo::BYTES, stream, a);
    return hipGetLastError();
  }
  // held tiles: normalised spectrograms of one or two tiles (larger N hold more bins per
  // lane: the second tile's values would spill)
  if constexpr (N <= 512) {
    const int ntiles = (a.T + Lo::TF - 1) / Lo::TF;
    const bool hold = (a.flags & SPECENH_STFT_NORMALIZE) && !(a.flags & SPECENH_STFT_DEV_NOSTORE) &&
                      ntiles <= 2 && variant(V_STFT_NO_HOLD) == 0;
    if (hold) {
      if (ntiles == 2)
        SPECENH_LAUNCH((stft_psd_kernel<N, XH, 2>), dim3((unsigned)batch), dim3(Lo::THREADS),
                       Lo::BYTES, stream, a);
      else
        SPECENH_LAUNCH((stft_psd_kernel<N, XH, 1>), dim3((unsigned)batch), dim3(Lo::THREADS),
                       Lo::BYTES, stream, a);
      return hipGetLastError();
    }
  }
  SPECENH_LAUNCH((stft_psd_kernel<N, XH>), dim3((unsigned)batch), dim3(Lo::THREADS),
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
constexpr int STFT_DEV_NOWAIT = 1 << 20;     // profiling flag: skip the team wait (wrong output)

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
    int ln = lane;  // opaque: the per-lane 64-bit address is re-formed here each poll
    asm volatile("" : "+v"(ln));  // instead of being hoisted out of the task loop (spilled)
    if (lane < M) v = __hip_atomic_load(g + ln, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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

// MODE (compile time, so each schedule keeps its own register allocation): 0 = plain
// PSD, 1 = log PSD (independent tiles: no granules, no waits), 2 = NORMALIZE (teams),
// 3 = cross-spectrum amplitude |Pxy| of the signal pairs (x[b], y[b]) (independent tiles).
// MODE 3 runs the same FFT pairs with the two frames of a pair taken from x and y at one
// time t: the separated spectra are X_t and Y_t, and |Pxy| = |conj(X) Y| * scale * (2 off
// DC/Nyquist) = sqrt(PSD_x * PSD_y), from the two PSD values pair_spectrum forms anyway
// (DC from the fp64 path as for the PSD). A lane group runs one pair per tile, so a
// member's tile is TF / 2 frames (tile_store1). (Two pairs per group for a TF-wide tile
// held one frame's amplitudes across the second FFT: 88 VGPRs spilled at 3 waves per SIMD,
// and at 2 waves per SIMD it ran 1.61 ms at C2.)
template <int N, int MODE>
__global__ __launch_bounds__(Layout<N>::THREADS, Layout<N>::WPE) void stft_team_kernel(
    StftArgs a, unsigned long long* gran, long long batch, int M, int Q, unsigned* tmo,
    unsigned char* tile_flag, int xcd_teams) {
  using C = Cfg<N>;
  using Lo = Layout<N>;
  constexpr int G = C::G;
  constexpr int IB = Lo::IB;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  f2v* s_tw = reinterpret_cast<f2v*>(smem + Lo::OFF_TW);
  float* s_win = reinterpret_cast<float*>(smem + Lo::OFF_WIN);
  float* s_tile = reinterpret_cast<float*>(smem + Lo::OFF_BUF);
  float* s_red = reinterpret_cast<float*>(smem + Lo::OFF_RED);  // [2*WAVES] + team {mn, mx, done}

  if ((int)blockIdx.x >= Q * M) return;  // whole workgroup: spare slots of the grid
  const int tid = threadIdx.x;
  // xcd_teams: a team's members are blocks b, b + 8, b + 16, ... (dealt to one XCD), so the
  // row segments two neighbouring members write into one 32-B sector meet in one L2, and
  // the frames their sample windows share are read once (a speed choice only: nothing
  // here depends on where the blocks actually run)
  const int b = blockIdx.x;
  const int s8 = xcd_teams ? (b >> 3) : b;
  const int q = xcd_teams ? (s8 / M) * 8 + (b & 7) : s8 / M;
  const int mem = s8 - (s8 / M) * M;
  for (int i = tid; i < Lo::TWN; i += Lo::THREADS) s_tw[i] = f2v{a.twiddle[i].x, a.twiddle[i].y};
  for (int i = tid; i < N; i += Lo::THREADS) s_win[i] = a.window[i];
  double* s_dc = reinterpret_cast<double*>(smem + Lo::OFF_DC);
  if constexpr (Lo::DC_TABLE)
    for (int i = tid; i < N; i += Lo::THREADS) s_dc[i] = a.dc_coef[i];
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int gl = lane % G;
  const int fi = wave * (64 / G) + lane / G;
  float* buf = reinterpret_cast<float*>(smem + Lo::OFF_BUF) + fi * Lo::BUF;
  const int t0 = mem * Lo::TF;  // this member's tile: frames [t0, t0 + TF)
  const int fa = t0 + 2 * fi;
  const long long ntask = (batch - q + Q - 1) / Q;  // shots q, q + Q, ... < batch
  const long long plane = (long long)a.F_out * a.T;
  const long long xbytes = a.x_stride * 4;
  const double dcb = dc_lane_base<N>(a, gl);
  // Without NORMALIZE the tiles are independent: the same persistent tile-parallel
  // schedule, no granules and no waits (log or plain PSD values stored as computed).
  constexpr bool normalize = MODE == 2;
  constexpr bool want_log = MODE == 1 || MODE == 2;
  constexpr bool xy = MODE == 3;

  PairSamples<N> s0;
  if constexpr (xy) {
    // one frame per lane group: tile frames [mem * TF1, + TF1), frame t1 + fi per group
    const int t1 = mem * Tile1<N>::TF1;
    const int f1 = t1 + fi;
    const long long ybytes = a.y_stride * 4;
    load_pair<N, false, true>(s0, make_rsrc(a.x + q * a.x_stride, xbytes),
                              make_rsrc(a.y + q * a.y_stride, ybytes), a.hop, f1, a.T, gl);
    __syncthreads();
    for (long long it = 0; it < ntask; ++it) {
      const long long shot = q + it * Q;
      const long long nshot = it + 1 < ntask ? shot + Q : shot;
      float dmin = INFINITY, dmax = -INFINITY;  // (pair_spectrum's running extremes: unused)
      f2v pv[IB];
      pair_spectrum<N, false, true>(a, s0, s0, s_tw, s_win, s_dc, buf, gl, dcb,
                                    make_rsrc(a.x + nshot * a.x_stride, xbytes),
                                    make_rsrc(a.y + nshot * a.y_stride, ybytes), f1, true, false,
                                    false, pv, dmin, dmax);
      float amp[IB];
#pragma unroll
      for (int i = 0; i < IB; ++i) amp[i] = __builtin_sqrtf(pv[i].x) * __builtin_sqrtf(pv[i].y);
      tile_store1<N>(a, s_tile, amp, gl, fi, tid, make_rsrc(a.out + shot * plane, plane * 4), t1);
    }
    return;
  }
  // C::PF = 0: no register prefetch; each task loads its own samples at its start (the
  // other resident waves cover the latency)
  if constexpr (C::PF)
    load_pair<N>(s0, make_rsrc(a.x + q * a.x_stride, xbytes), make_rsrc(a.x, 0), a.hop, fa, a.T, gl);
  __syncthreads();

  // Per task: the tile's spectrum (next task's samples prefetched meanwhile), publish the
  // tile's extremes, wait for the team's, store the normalised tile. No software
  // pipelining across tasks: the other resident workgroups of the CU (Cfg::OCC) fill
  // the waits.
  for (long long it = 0; it < ntask; ++it) {
    const long long shot = q + it * Q;
    const bool pf = it + 1 < ntask;
    const __amdgpu_buffer_rsrc_t xn = make_rsrc(a.x + (pf ? shot + Q : shot) * a.x_stride, xbytes);
    f2v pv[IB];
    float dmin = INFINITY, dmax = -INFINITY;  // (pair_spectrum's running extremes: unused)
    // NORMALIZE: the next task's samples are requested after the team wait, not inside
    // pair_spectrum: vmcnt is in order, so the wave polling the granules would otherwise
    // first wait for its whole prefetch to land while the workgroup idles at the barrier
    constexpr bool pf_inside = C::PF && (!normalize || !SPECENH_STFT_PF_AFTER_WAIT);
    if constexpr (!C::PF)
      load_pair<N>(s0, make_rsrc(a.x + shot * a.x_stride, xbytes), make_rsrc(a.x, 0), a.hop, fa, a.T,
                   gl);
    pair_spectrum<N>(a, s0, s0, s_tw, s_win, s_dc, buf, gl, dcb, xn, xn, fa, pf_inside, want_log, normalize,
                     pv, dmin, dmax);
    const __amdgpu_buffer_rsrc_t orr = make_rsrc(a.out + shot * plane, plane * 4);
    if constexpr (!normalize) {
      tile_store<N>(a, s_tile, pv, gl, fi, tid, orr, t0, 0.f, 1.f, false);
      continue;
    }
    // the tile's extremes from the held values themselves (the v_min3/v_max3 running
    // pair came out wrong in this kernel's schedule: measured on gfx950)
    float lmin = INFINITY, lmax = -INFINITY;
#pragma unroll
    for (int i = 0; i < IB; ++i) {
      lmin = fminf(lmin, fminf(pv[i].x, pv[i].y));
      lmax = fmaxf(lmax, fmaxf(pv[i].x, pv[i].y));
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
    // the raw tile goes to LDS now (normalised on its way out), overlapping the team wait
    tile_write<N>(s_tile, pv, gl, fi, 0.f, 1.f, false);
    if (tid == 0) {
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
    if (wave == 0) {
      float mn = 0.f, mx = 1.f;
      const bool done = (a.flags & STFT_DEV_NOWAIT) ||
                        team_minmax(gran + shot * M, M, lane, tmo, mn, mx,
                                    (a.flags & STFT_DEV_GIVEUP) != 0);
      if (lane == 0) {
        s_red[2 * C::WAVES] = mn;
        s_red[2 * C::WAVES + 1] = mx;
        s_red[2 * C::WAVES + 2] = done ? 1.f : 0.f;
        if (!done) tile_flag[shot * M + mem] = 1;  // raw tile: team_fixup_kernel finishes it
      }
    }
    lds_barrier();
    if constexpr (C::PF && !pf_inside) {
      __builtin_amdgcn_sched_barrier(0);
      load_pair<N>(s0, xn, xn, a.hop, (a.flags & SPECENH_STFT_DEV_NOLOAD) ? 0 : fa, a.T, gl);
      __builtin_amdgcn_sched_barrier(0);
    }
    const float mn = s_red[2 * C::WAVES];
    const float inv = 1.0f / (s_red[2 * C::WAVES + 1] - mn);  // max == min -> NaN (0/0)
    const bool done = s_red[2 * C::WAVES + 2] != 0.f;
    if constexpr (Lo::TILE_SWZ && Lo::TF == 16 && SPECENH_STFT_WIDE_EMIT)
      tile_emit4<N>(a, s_tile, tid, orr, t0, mn, inv, done);
    else
      tile_emit<N>(a, s_tile, tid, orr, t0, mn, inv, done);
    lds_barrier();  // tile (= FFT buffers) free for the next task's FFTs
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
template <int N, int MODE>
hipError_t launch_team_mode(const StftArgs& a, long long batch, void* workspace, hipStream_t stream,
                            bool* launched) {
  using Lo = Layout<N>;
  *launched = false;
  const int TFM = MODE == 3 ? Tile1<N>::TF1 : Lo::TF;  // frames per member tile
  const int M = (a.T + TFM - 1) / TFM;
  if (M > TEAM_MAX) return hipSuccess;
  static int cap[64] = {};  // resident workgroups per device (0 = not queried)
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  if (dev < 0 || dev >= 64) return hipSuccess;
  if (cap[dev] == 0) {
    e = hipFuncSetAttribute((const void*)stft_team_kernel<N, MODE>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, Lo::BYTES);
    if (e != hipSuccess) return e;
    int per_cu = 0, cus = 0;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)stft_team_kernel<N, MODE>,
                                                     Lo::THREADS, Lo::BYTES);
    if (e != hipSuccess) return e;
    e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (e != hipSuccess) return e;
    // never trust the occupancy answer alone (co-residency is a correctness condition
    // here): bound it by the register file (512 VGPR+AGPR per lane and SIMD, 8-register
    // granules, 4 SIMDs per CU) and by LDS as well
    hipFuncAttributes fa{};
    e = hipFuncGetAttributes(&fa, (const void*)stft_team_kernel<N, MODE>);
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
  const int xcd_teams = Q >= 8;
  if (xcd_teams) Q &= ~7ll;  // Q / 8 teams per XCD
  constexpr bool normalize = MODE == 2;
  unsigned* tmo = nullptr;
  unsigned long long* gran = nullptr;
  unsigned char* tflag = nullptr;
  if constexpr (normalize) {
    // workspace: [timeout word, 16 B][granules: batch x M x 8 B][tile flags: batch x M B],
    // zeroed every call (specenh_stft_workspace_bytes sizes it for M = TEAM_MAX)
    tmo = reinterpret_cast<unsigned*>(workspace);
    gran = reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(workspace) + 16);
    tflag = reinterpret_cast<unsigned char*>(gran + (size_t)batch * M);
    const size_t zero = 16 + (size_t)batch * M * 9;
    e = hipMemsetAsync(workspace, 0, zero, stream);
    if (e != hipSuccess) return e;
  }
  SPECENH_LAUNCH((stft_team_kernel<N, MODE>), dim3((unsigned)(Q * M)), dim3(Lo::THREADS), Lo::BYTES,
                     stream, a, gran, batch, M, (int)Q, tmo, tflag, xcd_teams);
  e = hipGetLastError();
  if (e != hipSuccess || !normalize) {
    *launched = e == hipSuccess;
    return e;
  }
  SPECENH_LAUNCH(team_fixup_kernel, dim3(1024), dim3(256), 0, stream, a.out, a.F_out, a.T,
                     Lo::TF, gran, tflag, batch, M, tmo);
  e = hipGetLastError();
  *launched = e == hipSuccess;
  return e;
}

template <int N>
hipError_t launch_team(const StftArgs& a, long long batch, void* workspace, hipStream_t stream,
                       bool* launched) {
  if (a.flags & SPECENH_STFT_NORMALIZE)
    return launch_team_mode<N, 2>(a, batch, workspace, stream, launched);
  if (a.flags & SPECENH_STFT_LOG) return launch_team_mode<N, 1>(a, batch, workspace, stream, launched);
  return launch_team_mode<N, 0>(a, batch, workspace, stream, launched);
}

}  // namespace specenh

using namespace specenh;

struct specenh_stft_plan;

namespace specenh {
// Cross-spectrum amplitude |Pxy| [batch][N/2 + 1][T] of the signal pairs (x[b], y[b]) on the
// team schedule (stft_team_kernel MODE 3), with the tables of an STFT plan of the same
// window / detrend / scaling (eps unused). *launched = false when it does not apply
// (nperseg > 1024, a plane of 1 GiB or more, more tiles than resident workgroups): the
// caller (specenh_csd) then runs csd_kernel.
int stft_csd_amplitude(const specenh_stft_plan* plan, const float* x, const float* y,
                       long long batch, long long length, long long x_stride, long long y_stride,
                       float* out, hipStream_t stream, bool* launched);
}  // namespace specenh

struct specenh_stft_plan {
  int nperseg, noverlap, hop;
  double fs, eps, scale;
  int scaling, detrend;
  int device;
  float* d_window;
  float2* d_twiddle;
  double dc_alpha, dc_beta;  // DC coefficients from the fp32 window (StftArgs)
  double* d_dc;              // c_n = w_n - alpha - beta (n - kmid), fp64
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
  // DC coefficients c_n = w_n - alpha - beta (n - kmid) (fp64): the detrend folded into
  // the window the kernel applies (the fp32 one), so c stays orthogonal to constants and
  // ramps to fp64 precision (see pair_spectrum).
  double dc_alpha = 0, dc_beta = 0;
  {
    const double kmid = 0.5 * (N - 1);
    double sk2 = 0, swk = 0, sw = 0;
    for (int i = 0; i < N; ++i) {
      sk2 += (i - kmid) * (i - kmid);
      swk += double(win[i]) * (i - kmid);
      sw += double(win[i]);
    }
    if (detrend != SPECENH_DETREND_NONE) dc_alpha = sw / N;
    if (detrend == SPECENH_DETREND_LINEAR) dc_beta = swk / sk2;
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
  p->dc_alpha = dc_alpha;
  p->dc_beta = dc_beta;
  hipError_t e = hipGetDevice(&p->device);
  if (e == hipSuccess) e = hipMalloc(&p->d_window, N * sizeof(float));
  if (e == hipSuccess) e = hipMalloc(&p->d_twiddle, tw.size() * sizeof(float2));
  if (e == hipSuccess) e = hipMalloc(&p->d_dc, N * sizeof(double));
  if (e == hipSuccess) {
    std::vector<double> dc(N);
    for (int i = 0; i < N; ++i) dc[i] = (double(win[i]) - dc_alpha) - dc_beta * (i - 0.5 * (N - 1));
    e = hipMemcpy(p->d_dc, dc.data(), N * sizeof(double), hipMemcpyHostToDevice);
  }
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
  if ((long long)(N / 2 + 1) * T * 4 >= (1ll << 30))
    return set_error(SPECENH_EUNSUPPORTED, "one spectrogram must stay below 1 GiB");
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
  a.dc_alpha = plan->dc_alpha;
  a.dc_beta = plan->dc_beta;
  a.dc_coef = plan->d_dc;
  const long long F_out = a.F_out;
  // team (tile-parallel) schedule for large spectrograms (C2: 518 KB each); small ones (C5:
  // 64 KB) are re-read from L2 by the sweep for less than the team's hand-off costs
  // (measured). Without NORMALIZE it needs no workspace.
  const bool team = (F_out * T * 4 >= (256ll << 10)) || (flags & STFT_DEV_FORCETEAM);
  const bool norm = (flags & SPECENH_STFT_NORMALIZE) != 0;
  // EXACT: one frame per FFT on the sweep schedule (launch_stft)
  if ((workspace || !norm) && !(flags & (STFT_DEV_NOTEAM | SPECENH_STFT_EXACT)) && team &&
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
  if ((long long)(N / 2 + 1) * T * 4 >= (1ll << 30))
    return set_error(SPECENH_EUNSUPPORTED, "one spectrogram must stay below 1 GiB");
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
  a.dc_alpha = plan->dc_alpha;
  a.dc_beta = plan->dc_beta;
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

namespace specenh {

int stft_csd_amplitude(const specenh_stft_plan* plan, const float* x, const float* y,
                       long long batch, long long length, long long x_stride, long long y_stride,
                       float* out, hipStream_t stream, bool* launched) {
  *launched = false;
  const int N = plan->nperseg;
  const long long T = specenh_stft_frames(length, N, plan->noverlap);
  if (T < 0) return (int)T;
  if (N > 1024 || batch > (1ll << 30) || (long long)(N / 2 + 1) * T * 4 >= (1ll << 30) ||
      x_stride * 4 >= (1ll << 31) || y_stride * 4 >= (1ll << 31))
    return SPECENH_OK;
  StftArgs a{};
  a.x = x;
  a.x_stride = x_stride;
  a.y = y;
  a.y_stride = y_stride;
  a.T = (int)T;
  a.hop = plan->hop;
  a.scale = (float)plan->scale;
  a.eps = 0.f;
  a.inv_kk = (float)(12.0 / ((double)N * ((double)N * N - 1.0)));
  a.detrend = plan->detrend;
  a.flags = 0;
  a.out = out;
  a.F_out = N / 2 + 1;
  a.window = plan->d_window;
  a.twiddle = plan->d_twiddle;
  a.dc_alpha = plan->dc_alpha;
  a.dc_beta = plan->dc_beta;
  a.dc_coef = plan->d_dc;
  hipError_t e = hipSuccess;
  switch (N) {
    case 64: e = launch_team_mode<64, 3>(a, batch, nullptr, stream, launched); break;
    case 128: e = launch_team_mode<128, 3>(a, batch, nullptr, stream, launched); break;
    case 256: e = launch_team_mode<256, 3>(a, batch, nullptr, stream, launched); break;
    case 512: e = launch_team_mode<512, 3>(a, batch, nullptr, stream, launched); break;
    case 1024: e = launch_team_mode<1024, 3>(a, batch, nullptr, stream, launched); break;
    default: break;
  }
  if (e != hipSuccess)
    return set_error(SPECENH_EHIP, std::string("csd team launch: ") + hipGetErrorString(e));
  return SPECENH_OK;
}

}  // namespace specenh
