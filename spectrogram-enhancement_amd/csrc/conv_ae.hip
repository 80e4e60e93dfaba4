// conv_ae.hip — the convolutional autoencoder's kernels for gfx950 (NHWC, MFMA).
//
// Replaces the Keras/TensorFlow layers of VAE/manual_scan_3layers.py:186-212
// (Conv2D / MaxPooling2D / Conv2DTranspose, padding="same", relu/sigmoid, Adam +
// binary_crossentropy).
//
// One implicit GEMM serves every convolution of the model:
//   out[m][co] = sum_k A[m][k] * Bt[co][k],   m = output pixel, k = (ky, kx, ci)
// with A gathered from the NHWC input (include/specenh.h, specenh_conv2d). Conv2D
// forward is a stride-1 conv, the input gradient of Conv2DTranspose is a stride-2 conv,
// and Conv2DTranspose forward / Conv2D input gradient are convs over a zero-dilated
// input. The dilated case is never materialised: it is split into in_dil^2 output
// phases, each a dense stride-1 conv over the undilated input with the sub-kernel of the
// taps that hit real samples (no MFMA work or gather spent on the holes). One launch
// carries every phase (blockIdx.z).
//
// Weights are N-major ("OHWI"): Bt[co][(ky, kx, ci)], so a B fragment row is contiguous.
//
//   conv_fwd_kernel     MFMA 16x16x32 bf16 (fp32 accumulate) or 16x16x4 f32. Workgroup =
//                       4 waves, 16*MT output pixels x 16*NT channels per wave; the next
//                       slab's gathers are in flight during the current slab's MFMAs (LDS-
//                       only barriers); 160-byte LDS rows make every ds_read_b128 fragment
//                       read bank-conflict free. Epilogue: + bias, optional fp32 pre-
//                       activation store, optional ReLU mask of another tensor (backward
//                       through a ReLU), relu / sigmoid.
//   conv_wgrad_kernel   dBt[co][k] = sum_m dOut[m][co] A[m][k]: the same gather, 64 pixels
//                       per step staged transposed in LDS (pixel pairs packed per 32-bit
//                       write), split over pixel chunks into a workspace and reduced in a
//                       fixed order (bit-reproducible); the bias gradient rides along.
//   maxpool2 fwd/bwd, bce_logits (Keras graph-mode BCE from logits), adam (Keras form),
//   flip_transpose (dgrad weights), cast.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <string>

#include "specenh.h"
#include "runtime.hpp"

namespace specenh {
int set_error(int code, const std::string& msg);  // stft_psd.hip
int launch_conv_narrow(int dtype, const void* in, int N, int IH, int IW, int C, const void* w,
                       int KH, int KW, int CO, const float* bias, int pad_t, int pad_l, int OH,
                       int OW, int act, void* out, int out_f32, float* logits, int pool,
                       unsigned char* argmax, const void* mask, hipStream_t st);  // conv_narrow.hip
int launch_conv_c1_mfma(int dtype, const void* in, int N, int IH, int IW, int C, const void* w,
                        int KH, int KW, int CO, const float* bias, int pad_t, int pad_l, int OH,
                        int OW, int act, void* out, int out_f32, float* logits, int pool,
                        unsigned char* argmax, const void* mask, hipStream_t st);  // conv_c1_mfma.hip

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float to_f(float x) { return x; }
__device__ __forceinline__ float to_f(__bf16 x) { return (float)x; }
__device__ __forceinline__ float to_f(_Float16 x) { return (float)x; }
template <typename T>
__device__ __forceinline__ T from_f(float x);
template <>
__device__ __forceinline__ float from_f<float>(float x) { return x; }
template <>
__device__ __forceinline__ __bf16 from_f<__bf16>(float x) { return (__bf16)x; }
template <>
__device__ __forceinline__ _Float16 from_f<_Float16>(float x) { return (_Float16)x; }

// Barrier for LDS hand-off only: does not drain outstanding global loads (the prefetch).
__device__ __forceinline__ void lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// ------------------------------------------------------------------ geometry
// One dense implicit GEMM (one output phase):
//   A[m][(jy, jx, ci)] = in[n][oy*stride - pad_t + jy][ox*stride - pad_l + jx][ci]
//   weight column of (jy, jx, ci) = ((ky0 + kstep*jy)*KWf + kx0 + kstep*jx)*C + ci
//   result stored at pixel (oy*oys + oy0, ox*oxs + ox0) of an OHs x OWs image.
struct Geo {
  int N, IH, IW, C;
  int OH, OW, CO;
  int KH, KW;
  int stride, pad_t, pad_l;
  int ky0, kx0, kstep, KWf, Kf;
  int oys, oy0, oxs, ox0, OHs, OWs;
};
constexpr int MAXPH = 4;

__device__ __forceinline__ int wcol(const Geo& g, int tap, int ci) {
  const int jy = tap / g.KW, jx = tap - (tap / g.KW) * g.KW;
  return ((g.ky0 + g.kstep * jy) * g.KWf + g.kx0 + g.kstep * jx) * g.C + ci;
}

template <typename T>
struct Tile;
template <>
struct Tile<__bf16> {
  static constexpr int BK = 64, LD = 80;  // 160-byte LDS rows
};
template <>
struct Tile<_Float16> {
  static constexpr int BK = 64, LD = 80;
};
template <>
struct Tile<float> {
  static constexpr int BK = 32, LD = 40;
};

// 8 consecutive elements of T as raw 32-bit words.
template <typename T>
struct V8 {
  uint32_t w[sizeof(T) * 2];
};

template <typename T>
__device__ __forceinline__ V8<T> ld8(const T* p) {
  V8<T> v;
  const uint4 a = reinterpret_cast<const uint4*>(p)[0];
  v.w[0] = a.x; v.w[1] = a.y; v.w[2] = a.z; v.w[3] = a.w;
  if constexpr (sizeof(T) == 4) {
    const uint4 b = reinterpret_cast<const uint4*>(p)[1];
    v.w[4] = b.x; v.w[5] = b.y; v.w[6] = b.z; v.w[7] = b.w;
  }
  return v;
}

template <typename T>
__device__ __forceinline__ void st8(T* p, const V8<T>& v) {
  reinterpret_cast<uint4*>(p)[0] = uint4{v.w[0], v.w[1], v.w[2], v.w[3]};
  if constexpr (sizeof(T) == 4)
    reinterpret_cast<uint4*>(p)[1] = uint4{v.w[4], v.w[5], v.w[6], v.w[7]};
}

template <typename T>
__device__ __forceinline__ void zero8(V8<T>& v) {
#pragma unroll
  for (int i = 0; i < (int)(sizeof(T) * 2); ++i) v.w[i] = 0u;
}

__device__ __forceinline__ uint32_t bits(float x) { return __float_as_uint(x); }
__device__ __forceinline__ uint32_t bits(__bf16 x) {
  return (uint32_t)__builtin_bit_cast(unsigned short, x);
}
__device__ __forceinline__ uint32_t bits(_Float16 x) {
  return (uint32_t)__builtin_bit_cast(unsigned short, x);
}

// element j of a V8 (as raw bits)
template <typename T>
__device__ __forceinline__ uint32_t elem_bits(const V8<T>& v, int j) {
  if constexpr (sizeof(T) == 4) return v.w[j];
  else return (v.w[j >> 1] >> (16 * (j & 1))) & 0xffffu;
}

template <typename T>
__device__ __forceinline__ void set_elem(V8<T>& v, int j, T x) {
  if constexpr (sizeof(T) == 4) {
    v.w[j] = bits(x);
  } else {
    const uint32_t b = bits(x) << (16 * (j & 1));
    v.w[j >> 1] = (v.w[j >> 1] & (0xffff0000u >> (16 * (j & 1)))) | b;
  }
}

// Two floats rounded to T (round to nearest even) and packed into one 32-bit word, element
// a in the low half: v_cvt_pk_bf16_f32 / two v_cvt_f16_f32 + v_pack_b32_f16 (no mask ops).
template <typename T>
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  if constexpr (__is_same(T, __bf16)) {
    typedef __bf16 b2 __attribute__((ext_vector_type(2)));
    return __builtin_bit_cast(uint32_t, b2{(__bf16)a, (__bf16)b});
  } else {
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
    return __builtin_bit_cast(uint32_t, h2{(_Float16)a, (_Float16)b});
  }
}

// max(a, b) without the NaN-quieting canonicalisation fmaxf gets (operands are
// accumulators: finite unless the inputs hold NaN/Inf) as v_med3_f32(a, b, +inf): a
// builtin, not inline asm, so the compiler's hazard recognizer sees the read of an MFMA
// result and pads the XDL-write -> VALU-read wait states (inside an asm statement it
// does not)
__device__ __forceinline__ float vmax(float a, float b) {
  return __builtin_amdgcn_fmed3f(a, b, __builtin_inff());
}

// 8 GEMM-K elements k .. k+7 of one output pixel (by, bx = top-left of its window, nb =
// n*IH). Out-of-range rows have by far below zero.
template <typename T>
__device__ __forceinline__ V8<T> gather_a8(const T* __restrict__ in, const Geo& g, int K, int k,
                                           int by, int bx, int nb) {
  V8<T> v;
  if ((g.C & 7) == 0) {
    const int tap = k / g.C, ci = k - (k / g.C) * g.C;
    const int jy = tap / g.KW, jx = tap - (tap / g.KW) * g.KW;
    const int iy = by + jy, ix = bx + jx;
    const bool ok = k < K && (unsigned)iy < (unsigned)g.IH && (unsigned)ix < (unsigned)g.IW;
    v = ld8(in + (ok ? ((nb + iy) * g.IW + ix) * g.C + ci : 0));
    if (!ok) zero8(v);
  } else {
    zero8(v);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int kk = k + j;
      const int tap = kk / g.C, ci = kk - (kk / g.C) * g.C;
      const int jy = tap / g.KW, jx = tap - (tap / g.KW) * g.KW;
      const int iy = by + jy, ix = bx + jx;
      const bool ok = kk < K && (unsigned)iy < (unsigned)g.IH && (unsigned)ix < (unsigned)g.IW;
      const T x = in[ok ? ((nb + iy) * g.IW + ix) * g.C + ci : 0];
      if (ok) set_elem(v, j, x);
    }
  }
  return v;
}

// 8 GEMM-K elements k .. k+7 of weight row co (Bt[co][Kf]).
template <typename T>
__device__ __forceinline__ V8<T> gather_b8(const T* __restrict__ W, const Geo& g, int K, int k,
                                           int co) {
  V8<T> v;
  if ((g.C & 7) == 0) {
    const bool ok = co < g.CO && k < K;
    const int tap = k / g.C, ci = k - (k / g.C) * g.C;
    v = ld8(W + (ok ? co * g.Kf + wcol(g, tap, ci) : 0));
    if (!ok) zero8(v);
  } else {
    zero8(v);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int kk = k + j;
      const bool ok = co < g.CO && kk < K;
      const int tap = kk / g.C, ci = kk - (kk / g.C) * g.C;
      const T x = W[ok ? co * g.Kf + wcol(g, tap, ci) : 0];
      if (ok) set_elem(v, j, x);
    }
  }
  return v;
}

// acc += A_tile(16 rows at sa) x B_tile(16 rows at sb)^T over one BK slab.
template <typename T>
__device__ __forceinline__ f32x4 mfma_slab(const T* sa, const T* sb, f32x4 acc, int lane) {
  constexpr int BK = Tile<T>::BK, LD = Tile<T>::LD;
  if constexpr (__is_same(T, __bf16)) {
#pragma unroll
    for (int s = 0; s < BK / 32; ++s) {
      const bf16x8 a = *reinterpret_cast<const bf16x8*>(sa + (lane & 15) * LD + 32 * s + 8 * (lane >> 4));
      const bf16x8 b = *reinterpret_cast<const bf16x8*>(sb + (lane & 15) * LD + 32 * s + 8 * (lane >> 4));
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
    }
  } else if constexpr (__is_same(T, _Float16)) {
#pragma unroll
    for (int s = 0; s < BK / 32; ++s) {
      const f16x8 a = *reinterpret_cast<const f16x8*>(sa + (lane & 15) * LD + 32 * s + 8 * (lane >> 4));
      const f16x8 b = *reinterpret_cast<const f16x8*>(sb + (lane & 15) * LD + 32 * s + 8 * (lane >> 4));
      acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc, 0, 0, 0);
    }
  } else {
#pragma unroll
    for (int s = 0; s < BK / 4; ++s) {
      const float a = sa[(lane & 15) * LD + 4 * s + (lane >> 4)];
      const float b = sb[(lane & 15) * LD + 4 * s + (lane >> 4)];
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
    }
  }
  return acc;
}

struct ConvArgs {
  Geo g[MAXPH];
  const void* in;
  const void* w;      // Bt [CO][Kf]
  const float* bias;  // [CO] or null
  void* out;          // [N][OHs][OWs][CO], float if out_f32 else T
  const void* mask;   // same shape, T, or null: v *= (mask > 0)
  float* logits;      // same shape, fp32 pre-activation, or null
  int out_f32;
  int act;            // 0 none, 1 relu, 2 sigmoid
  int nph;            // output phases (1, or in_dil^2)
  int pool;           // 1: fused 2x2/2 max-pool, out is [N][OH/2][OW/2][CO]
  unsigned char* argmax;  // pooled argmax (dy*2+dx), or null
  // LDS-patch kernel, all phases in one workgroup: union patch origin/extent
  int ph_shared, upt, upl, PH, PW;
  // conv_patch_kernel<..., WL>: the workgroup's weight rows staged in LDS at byte offset
  // wl_off, row stride wl_rs elements (wl_rs / 2 = 8 mod 64 dwords: conflict-free fragments)
  int wl_off, wl_rs;
  // conv_patch_kernel (specenh_conv2d_pooled_in): the input is the full-resolution gradient of
  // a ReLU + MaxPooling2D((2,2)), formed from the pool's gradient rpd [N][IH/2][IW/2][C], its
  // argmax ram and pooled output rpy (null: no ReLU mask) while the patch is staged
  const void* rpd;
  const unsigned char* ram;
  const void* rpy;
};

// 8 channels of the full-resolution gradient a MaxPooling2D((2,2)) backward would write at a
// pixel of parity sel = 2 (y & 1) + (x & 1): the pool's gradient dv where the argmax bytes am
// name sel and the pooled output yv > 0 (the ReLU mask of the pool's input at its argmax;
// > 0 as 16-bit bits: sign clear and nonzero), else 0 (specenh_maxpool2_bwd's arithmetic)
__device__ __forceinline__ uint4 pool_route8(uint4 dv, uint2 am, uint4 yv, uint32_t sel) {
  const uint32_t d4[4] = {dv.x, dv.y, dv.z, dv.w}, y4[4] = {yv.x, yv.y, yv.z, yv.w};
  uint32_t o4[4];
#pragma unroll
  for (int h = 0; h < 4; ++h) {
    const uint32_t amw = h < 2 ? am.x : am.y;
    uint32_t r = 0u;
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const uint32_t y16 = (y4[h] >> (16 * b)) & 0xffffu;
      const bool keep = ((amw >> (8 * (2 * (h & 1) + b))) & 0xffu) == sel && !(y16 & 0x8000u) &&
                        y16 != 0u;
      r |= keep ? (d4[h] & (0xffffu << (16 * b))) : 0u;
    }
    o4[h] = r;
  }
  return uint4{o4[0], o4[1], o4[2], o4[3]};
}
constexpr uint32_t POOL_ROUTE_POS = 0x3f803f80u;  // two 16-bit values > 0 (no ReLU mask)

// ------------------------------------------------------------------ forward / dgrad
template <typename T, int MT, int NT>
__global__ __launch_bounds__(256) void conv_fwd_kernel(ConvArgs a) {
  constexpr int BK = Tile<T>::BK, LD = Tile<T>::LD;
  constexpr int BM = 64 * MT, BN = 16 * NT;
  constexpr int KG = BK / 8;          // 8-element groups per k-slab
  constexpr int RSTEP = 256 / KG;     // rows between a thread's gather rows
  constexpr int ROWS = BM / RSTEP;    // gather rows per thread
  constexpr int BG = BN * KG;         // B groups per slab
  constexpr int BPER = (BG + 255) / 256;
  __shared__ __attribute__((aligned(16))) T sA[BM * LD];
  __shared__ __attribute__((aligned(16))) T sB[BN * LD];

  const Geo& g = a.g[blockIdx.z];
  const int M = g.N * g.OH * g.OW;
  const int m0 = blockIdx.x * BM;
  if (m0 >= M) return;
  const int n0 = blockIdx.y * BN;
  const int K = g.KH * g.KW * g.C;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const T* __restrict__ in = reinterpret_cast<const T*>(a.in);
  const T* __restrict__ W = reinterpret_cast<const T*>(a.w);

  const int kg = tid % KG, r0 = tid / KG;
  const int hw = g.OH * g.OW;
  int by[ROWS], bx[ROWS], nb[ROWS];
#pragma unroll
  for (int i = 0; i < ROWS; ++i) {
    const int m = m0 + r0 + RSTEP * i;
    if (m < M) {
      const int n = m / hw, rem = m - (m / hw) * hw;
      const int oy = rem / g.OW, ox = rem - (rem / g.OW) * g.OW;
      by[i] = oy * g.stride - g.pad_t;
      bx[i] = ox * g.stride - g.pad_l;
      nb[i] = n * g.IH;
    } else {
      by[i] = -(1 << 29);
      bx[i] = 0;
      nb[i] = 0;
    }
  }

  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  V8<T> ra[ROWS], rb[BPER];
  auto fetch = [&](int k0) {
#pragma unroll
    for (int i = 0; i < ROWS; ++i) ra[i] = gather_a8<T>(in, g, K, k0 + 8 * kg, by[i], bx[i], nb[i]);
#pragma unroll
    for (int j = 0; j < BPER; ++j) {
      const int idx = tid + 256 * j;
      const int co_l = idx / KG, kgb = idx - (idx / KG) * KG;
      if (idx < BG) rb[j] = gather_b8<T>(W, g, K, k0 + 8 * kgb, n0 + co_l);
    }
  };

  if (K > 0) fetch(0);
  for (int k0 = 0; k0 < K; k0 += BK) {
#pragma unroll
    for (int i = 0; i < ROWS; ++i) st8(sA + (r0 + RSTEP * i) * LD + 8 * kg, ra[i]);
#pragma unroll
    for (int j = 0; j < BPER; ++j) {
      const int idx = tid + 256 * j;
      const int co_l = idx / KG, kgb = idx - (idx / KG) * KG;
      if (idx < BG) st8(sB + co_l * LD + 8 * kgb, rb[j]);
    }
    lds_sync();
    if (k0 + BK < K) fetch(k0 + BK);  // in flight during the MFMAs below
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j)
        acc[i][j] = mfma_slab<T>(sA + 16 * (wave * MT + i) * LD, sB + 16 * j * LD, acc[i][j], lane);
    lds_sync();
  }

  // epilogue: D[row][col], col = lane & 15, row = 4*(lane >> 4) + reg
#pragma unroll
  for (int i = 0; i < MT; ++i) {
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
      const int m = m0 + 16 * (wave * MT + i) + 4 * (lane >> 4) + reg;
      if (m >= M) continue;
      const int n = m / hw, rem = m - (m / hw) * hw;
      const int oy = rem / g.OW, ox = rem - (rem / g.OW) * g.OW;
      const long long pix =
          ((long long)n * g.OHs + oy * g.oys + g.oy0) * g.OWs + ox * g.oxs + g.ox0;
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int col = n0 + 16 * j + (lane & 15);
        if (col >= g.CO) continue;
        const long long idx = pix * g.CO + col;
        float v = acc[i][j][reg] + (a.bias ? a.bias[col] : 0.f);
        if (a.logits) a.logits[idx] = v;
        if (a.mask && !(to_f(reinterpret_cast<const T*>(a.mask)[idx]) > 0.f)) v = 0.f;
        if (a.act == 1) v = fmaxf(v, 0.f);
        else if (a.act == 2) v = 1.f / (1.f + __expf(-v));
        if (a.out_f32) reinterpret_cast<float*>(a.out)[idx] = v;
        else reinterpret_cast<T*>(a.out)[idx] = from_f<T>(v);
      }
    }
  }
}

// ------------------------------------------------------------------ LDS-patch forward
// Stride-1 convolutions in bf16/f16 (every Conv2D forward, every Conv2DTranspose phase,
// Conv2D input gradients): the workgroup's 16x16 output tile needs a (16+KH-1) x (16+KW-1)
// input patch, staged in LDS once per channel chunk; A fragments are read from the patch
// (ds_read_b128, bank-conflict-free pixel strides), so each input element is fetched
// about (20/16)^2 times instead of KH*KW times. B fragments (the small, L2-resident
// weights) go straight to registers, one k-step ahead.
// CC = channels per chunk: 64 or 32 (C % 32 == 0), 16 (C == 16: two taps per MFMA), 1
// (C == 1: all <= 32 taps in one MFMA).
// Epilogue: the tile goes through LDS and leaves as 16-byte stores; with POOL the 2x2
// max-pool (+argmax) is taken in registers first — a wave's 4 output rows and a lane's
// 4 consecutive pixels are exactly 2x2 windows — so the full-resolution tensor is never
// written. Phases of a dilated conv (Conv2DTranspose) run in workgroups on the same XCD
// one after the other (blockIdx.x % 8 picks the XCD): they share the input patch and
// interleave into the same output lines in that XCD's L2.
template <int CC>
struct Patch;
template <>
struct Patch<64> { static constexpr int PST = 80; };  // 160-byte pixels
template <>
struct Patch<32> { static constexpr int PST = 48; };  // 96-byte pixels
template <>
struct Patch<16> { static constexpr int PST = 16; };  // 32-byte pixels
template <>
struct Patch<1> { static constexpr int PST = 1; };

// 8 consecutive 16-bit weights through a buffer descriptor: the lane's row offset stays in
// one VGPR for the whole k-loop and the k-step's column offset is a wave-uniform soffset, so
// a weight-ring refill costs no VALU address arithmetic (and no temporaries whose reuse
// would make the compiler drain the ring's other in-flight loads).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t weight_rsrc(const void* base, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0,
                                           (int)(bytes < 0x7fffffffll ? bytes : 0x7fffffffll),
                                           0x00020000);
}
template <typename T>
__device__ __forceinline__ V8<T> ldw(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  static_assert(sizeof(T) == 2, "16-bit weights");
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0);
  V8<T> v;
  v.w[0] = a.x; v.w[1] = a.y; v.w[2] = a.z; v.w[3] = a.w;
  return v;
}

template <typename T>
__device__ __forceinline__ f32x4 mfma32(const V8<T>& a, const V8<T>& b, f32x4 acc) {
  if constexpr (__is_same(T, __bf16)) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                   __builtin_bit_cast(bf16x8, b), acc, 0, 0, 0);
  } else {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a),
                                                  __builtin_bit_cast(f16x8, b), acc, 0, 0, 0);
  }
}

__device__ __forceinline__ float apply_act(float v, int act) {
  if (act == 1) return fmaxf(v, 0.f);
  if (act == 2) return 1.f / (1.f + __expf(-v));
  return v;
}

// PAIR (Conv2DTranspose, stride 2): the workgroup owns one output-row phase py of a tile
// and computes its two column phases (py, 0) and (py, 1) over one staged patch. Phase
// (py, 0) waits in registers, packed to T; after (py, 1) the patch is dead, so both are
// interleaved into an LDS image of the 16 output rows x 32 pixels x CO channels that
// aliases the patch, and leave as 16-byte stores of whole rows, so no 128-B output line is
// completed by two phase stores microseconds apart. Opt-in (SPECENH_CONVT_PAIR=1): with
// all four phases in one workgroup (ph_shared, the default) the measured convT write
// traffic is 1.02-1.25x algorithmic (profiles/pmc_traffic.json). The two row phases of a
// tile run on one XCD back to back and share its input lines in L2.

// waves per SIMD the register budget is sized for (4 -> 128 VGPRs, 3 -> 168, 2 -> 256)
#ifndef SPECENH_PATCH_WPE
#define SPECENH_PATCH_WPE(PAIR, NT, CC) \
  ((PAIR && NT == 1) || (CC == 16 && NT == 2) ? 4 : ((CC == 32 && NT == 4) || CC == 64 ? 3 : 1))
#endif
// weight-ring depth of the wave-split kernel (k-steps of loads in flight per wave); 8 for
// NT = 1 measured 5 % slower on convT1/convT2, 4 for NT = 2 spills
#ifndef SPECENH_WS_PD1
#define SPECENH_WS_PD1 4
#endif
#ifndef SPECENH_WS_PD2
#define SPECENH_WS_PD2 2
#endif
// S2 (stride-2 conv, CC == 16, one phase: the input gradient of a Conv2DTranspose): the
// 35 x 35 input patch of a 16 x 16 output tile is staged de-interleaved into its four
// (row, column) parity sub-patches of 18 x 18, so tap (jy, jx) of output pixel (y, x) is
// pixel (y + jy/2, x + jx/2) of sub-patch (jy&1, jx&1): the lanes' fragment reads stay
// unit-stride and the k-step loop is the stride-1 one.
// RT (round 6, specenh_conv2d_pooled_in): the input patch is routed from a pool's gradient
// (ConvArgs::rpd / ram / rpy) while it is staged; a template argument, not a run-time test, so
// the other instantiations' register allocation is untouched (as a run-time branch it cost
// them 20-40 VGPRs and SGPR spills)
template <typename T, int NT, int CC, bool POOL, bool PAIR = false, bool S2 = false, bool WS = false,
          bool WL = false, bool K5 = false, bool RT = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WS ? 3 : SPECENH_PATCH_WPE(PAIR, NT, CC))))
void conv_patch_kernel(ConvArgs a) {
  static_assert(!RT || (!S2 && !PAIR && !POOL && CC >= 16), "routed input: a plain stride-1 conv");
  static_assert(!S2 || (CC == 16 && !POOL && !PAIR), "stride-2 patches: CC 16, plain epilogue");
  static_assert(!WL || (CC == 16 && !PAIR && !WS), "LDS weights: the 16-channel single-chunk kernel");
  // K5: a plain stride-1 5 x 5 conv of one phase and one channel chunk (host-checked), so
  // every tap offset is a compile-time immediate of the fully unrolled k-loop
  static_assert(!K5 || (WL && !S2), "compile-time taps: with LDS weights");
  static_assert(!WS || !PAIR, "wave split: not with the row-phase pair epilogue");
  constexpr int TILE = 16;
  constexpr int PST = Patch<CC>::PST;
  // output rows per wave: 4 (waves stacked over the 16 rows, each wave all 16 NT channels),
  // or 8 with WS (2 x 2 waves: row halves x channel halves of a 32 NT-channel workgroup;
  // each weight fragment feeds 8 MFMAs instead of 4 and the waves load different weights)
  constexpr int MT = WS ? 8 : 4;
  // the patch (and PAIR's output stage) in dynamic LDS sized by the launch for the actual
  // patch (patch_lds_bytes): a Conv2DTranspose's 4 phases share an 18 x 18 patch, not 20 x 20
  // (CC = 64: 52 KB -> 3 workgroups per CU instead of 2)
  extern __shared__ __attribute__((aligned(16))) unsigned char sP_raw[];
  T* const sP = reinterpret_cast<T*>(sP_raw);
  constexpr int MAXTAP = 64;         // taps per phase (k <= 7: 49)
  __shared__ int sTap[MAXPH][MAXTAP];  // patch offset of tap t (elements), -1 past the last tap
  __shared__ int sCol[MAXPH][MAXTAP];  // weight column of tap t at ci = 0

  // the per-tile program; K5 workgroups run it persistently over tiles blockIdx.x,
  // + gridDim.x, ... with the weight rows staged once (first)
  auto body = [&](const int bx_in, const bool first) {
  if (!first) lds_sync();  // every wave is done with the previous tile's patch

  // ---- phases of this workgroup: all of them over one shared patch, a row-phase pair
  // (PAIR), or blockIdx.z ----
  int bx = bx_in, pyp = 0;
  if constexpr (PAIR) {  // blocks 16q + 8py + x: tile 8q + x, row phase py, XCD x
    const int j = bx >> 3;
    pyp = j & 1;
    bx = (j >> 1) * 8 + (bx & 7);
  }
  const bool shared = PAIR || a.ph_shared != 0;
  const int ph_lo = PAIR ? 2 * pyp : (shared ? 0 : (int)blockIdx.z);
  const int ph_hi = PAIR ? ph_lo + 2 : (shared ? a.nph : ph_lo + 1);
  const Geo& g0 = a.g[ph_lo];
  const int ntx = (g0.OW + TILE - 1) / TILE, nty = (g0.OH + TILE - 1) / TILE;
  if (bx >= g0.N * nty * ntx) return;
  const int n = bx / (nty * ntx);
  const int trem = bx - n * (nty * ntx);
  const int ty = trem / ntx, tx = trem - (trem / ntx) * ntx;
  const int oy0 = ty * TILE, ox0 = tx * TILE;
  const int upt = shared ? a.upt : g0.pad_t, upl = shared ? a.upl : g0.pad_l;
  const int PH = shared ? a.PH : (S2 ? 2 * TILE - 2 : TILE - 1) + g0.KH;
  const int PW = shared ? a.PW : (S2 ? 2 * TILE - 2 : TILE - 1) + g0.KW;
  const int SPH = S2 ? (PH + 1) / 2 : PH, SPW = S2 ? (PW + 1) / 2 : PW;  // S2 sub-patches
  const int iy0 = (S2 ? 2 : 1) * oy0 - upt, ix0 = (S2 ? 2 : 1) * ox0 - upl;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wrow = WS ? (wave >> 1) : wave;
  const int n0 = blockIdx.y * 16 * NT * (WS ? 2 : 1) + (WS ? (wave & 1) * 16 * NT : 0);
  const int kgrp = lane >> 4, px = lane & 15;
  const T* __restrict__ in = reinterpret_cast<const T*>(a.in);
  const T* __restrict__ W = reinterpret_cast<const T*>(a.w);

  for (int e = tid; e < MAXTAP * (ph_hi - ph_lo); e += 256) {
    const int p = ph_lo + e / MAXTAP, t = e % MAXTAP;
    const Geo& g = a.g[p];
    const int jy = t / g.KW, jx = t - (t / g.KW) * g.KW;
    const int dy = upt - g.pad_t, dx = upl - g.pad_l;  // this phase's shift in the patch
    sTap[p][t] = t < g.KH * g.KW ? ((jy + dy) * PW + jx + dx) * PST : -1;
    sCol[p][t] = t < g.KH * g.KW ? ((g.ky0 + g.kstep * jy) * g.KWf + g.kx0 + g.kstep * jx) * g.C : 0;
  }

  int rbase[MT];  // this lane's pixel (row i of the wave, column px) in the patch
#pragma unroll
  for (int i = 0; i < MT; ++i) rbase[i] = ((wrow * MT + i) * SPW + px) * PST;

  auto stage = [&](int c) {
    if constexpr (CC == 1) {
      for (int e = tid; e < PH * PW; e += 256) {
        const int py = e / PW, pxx = e - (e / PW) * PW;
        const int iy = iy0 + py, ix = ix0 + pxx;
        const bool ok = (unsigned)iy < (unsigned)g0.IH && (unsigned)ix < (unsigned)g0.IW;
        const T v = in[ok ? (n * g0.IH + iy) * g0.IW + ix : 0];
        sP[e] = ok ? v : from_f<T>(0.f);
      }
    } else {
      constexpr int GP = CC / 8;  // 8-channel groups per pixel
      // pix / PW as a multiply-shift (exact: pix * (PW - 1) < 2^16), 32-bit offsets
      // (check_sizes bounds every tensor below 2^31 elements)
      const int pwinv = (65536 + PW - 1) / PW;
      const int IHl = g0.IH, IWl = g0.IW, Cl = g0.C;
      const T* __restrict__ inb = in + n * IHl * IWl * Cl + c * CC;
      // batches of NB loads in flight per thread (a load-wait-store loop would pay the full
      // memory latency once per element); out-of-image pixels load a valid address and are
      // zeroed, so the loads are unconditional
      constexpr int NB = (SPECENH_PATCH_WPE(PAIR, NT, CC) >= 4 || NT >= 4) ? 4 : 8;  // VGPR budget
      const int total = PH * PW * GP;
      if constexpr (RT) {
        {  // routed from the pool's gradient (specenh_conv2d_pooled_in)
          // one element per (pooled pixel, 8-channel group) covering the patch: its gradient,
          // argmax bytes and pooled value are loaded ONCE and give the 2 x 2 full-resolution
          // pixels (those inside the patch; even IH / IW: all in the image or all out)
          const int PHl = IHl >> 1, PWl = IWl >> 1;
          const int qy0 = iy0 >> 1, qx0 = ix0 >> 1;  // (floor: arithmetic shifts)
          const int QH = ((iy0 + PH - 1) >> 1) - qy0 + 1, QW = ((ix0 + PW - 1) >> 1) - qx0 + 1;
          const int qwinv = (65536 + QW - 1) / QW;  // exact: qpix * (QW - 1) < 2^16
          const int pbase = n * PHl * PWl * Cl + c * CC;
          const T* __restrict__ dpb = reinterpret_cast<const T*>(a.rpd) + pbase;
          const T* __restrict__ ypb = a.rpy ? reinterpret_cast<const T*>(a.rpy) + pbase : nullptr;
          const unsigned char* __restrict__ amb = a.ram + pbase;
          const int qtotal = QH * QW * GP;
          constexpr int NR = NB / 2;  // three loads per element
          for (int e0 = tid; e0 < qtotal; e0 += NR * 256) {
            uint4 dv[NR], yv[NR];
            uint2 am[NR];
            int qy[NR], qx[NR], cg[NR];
#pragma unroll
            for (int k = 0; k < NR; ++k) {
              const int e = min(e0 + 256 * k, qtotal - 1);
              const int qpix = e / GP;
              cg[k] = e - qpix * GP;
              const int r = (qpix * qwinv) >> 16;
              qy[k] = qy0 + r;
              qx[k] = qx0 + qpix - r * QW;
              const bool ok = (unsigned)qy[k] < (unsigned)PHl && (unsigned)qx[k] < (unsigned)PWl;
              const int po = (ok ? qy[k] * PWl + qx[k] : 0) * Cl + 8 * cg[k];
              dv[k] = *reinterpret_cast<const uint4*>(dpb + po);
              am[k] = *reinterpret_cast<const uint2*>(amb + po);
              yv[k] = ypb ? *reinterpret_cast<const uint4*>(ypb + po)
                          : uint4{POOL_ROUTE_POS, POOL_ROUTE_POS, POOL_ROUTE_POS, POOL_ROUTE_POS};
              if (!ok) dv[k] = uint4{0u, 0u, 0u, 0u};
            }
#pragma unroll
            for (int k = 0; k < NR; ++k) {
              if (e0 + 256 * k >= qtotal) continue;
#pragma unroll
              for (int sub = 0; sub < 4; ++sub) {
                const int py = 2 * qy[k] + (sub >> 1) - iy0, pxx = 2 * qx[k] + (sub & 1) - ix0;
                if ((unsigned)py < (unsigned)PH && (unsigned)pxx < (unsigned)PW)
                  *reinterpret_cast<uint4*>(sP + (py * PW + pxx) * PST + 8 * cg[k]) =
                      pool_route8(dv[k], am[k], yv[k], (uint32_t)sub);
              }
            }
          }
          return;
        }
      }
      for (int e0 = tid; e0 < total; e0 += NB * 256) {
        uint4 v[NB];
        int dst[NB];
#pragma unroll
        for (int k = 0; k < NB; ++k) {
          const int e = min(e0 + 256 * k, total - 1);
          const int pix = e / GP, cg = e - (e / GP) * GP;
          const int py = (pix * pwinv) >> 16, pxx = pix - py * PW;
          const int iy = iy0 + py, ix = ix0 + pxx;
          const bool ok = (unsigned)iy < (unsigned)IHl && (unsigned)ix < (unsigned)IWl;
          v[k] = *reinterpret_cast<const uint4*>(inb + (ok ? (iy * IWl + ix) * Cl : 0) + 8 * cg);
          if (!ok) v[k] = uint4{0u, 0u, 0u, 0u};
          const int spix = S2 ? ((py & 1) * 2 + (pxx & 1)) * SPH * SPW + (py >> 1) * SPW + (pxx >> 1) : pix;
          dst[k] = spix * PST + 8 * cg;
        }
#pragma unroll
        for (int k = 0; k < NB; ++k)
          if (e0 + 256 * k < total) *reinterpret_cast<uint4*>(sP + dst[k]) = v[k];
      }
    }
  };

  const int nchunk = CC == 1 ? 1 : g0.C / CC;
  uint32_t hold[MT][NT][2];  // PAIR: phase (py, 0), packed to T
  for (int p = ph_lo; p < ph_hi; ++p) {
    const Geo& g = a.g[p];
    const int ntap = g.KH * g.KW;
    f32x4 acc[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    for (int c = 0; c < nchunk; ++c) {
      if (p == ph_lo || nchunk > 1) {
        if (c > 0 || p > ph_lo) lds_sync();  // previous chunk's fragment reads are done
        stage(c);
        if constexpr (WL) {
          if (p == ph_lo && first) {  // this workgroup's 16 NT weight rows (all phases), once
            const int Kf = K5 ? 400 : g0.Kf, kv = Kf / 8, nv = 16 * NT * kv;
            T* sWt = reinterpret_cast<T*>(sP_raw + a.wl_off);
            for (int e0 = tid; e0 < nv; e0 += 4 * 256) {
              uint4 v[4];
              int dst[4];
#pragma unroll
              for (int k = 0; k < 4; ++k) {
                const int e = min(e0 + 256 * k, nv - 1);
                const int rr = e / kv, q = e - rr * kv;
                v[k] = *reinterpret_cast<const uint4*>(W + (long long)min(n0 + rr, g0.CO - 1) * Kf + 8 * q);
                dst[k] = rr * a.wl_rs + 8 * q;
              }
#pragma unroll
              for (int k = 0; k < 4; ++k)
                if (e0 + 256 * k < nv) *reinterpret_cast<uint4*>(sWt + dst[k]) = v[k];
            }
          }
        }
        lds_sync();
      }
      if constexpr (CC >= 32) {
        // ---- k-steps: one MFMA K=32 slab each; weights are the A operand (rows = output
        // channels), the patch the B operand (columns = pixels): D[channel][pixel]. Tap
        // geometry is wave-uniform scalar arithmetic; weight loads are unconditional from
        // clamped rows (a clamped row only feeds output channels >= CO, never stored), so
        // the prefetch ring has no branches and no WAW waits on in-flight loads ----
        constexpr int SUB = CC / 32;  // 32-channel slabs per tap
        const int KWl = g.KW, Kfl = g.Kf, Cl = g.C, KWf = g.KWf, ks = g.kstep;
        const int ky0 = g.ky0, kx0 = g.kx0;
        const int dy = upt - g.pad_t, dx = upl - g.pad_l;  // this phase's shift in the patch
        const int kwinv = (65536 + KWl - 1) / KWl;         // t / KW == (t * kwinv) >> 16, t < 32
        const int nsteps = ntap * SUB;
        const __amdgpu_buffer_rsrc_t wrs = weight_rsrc(W, (long long)g.CO * Kfl * sizeof(T));
        int wv[NT];  // byte offset of this lane's weight row (+ chunk, k group)
#pragma unroll
        for (int j = 0; j < NT; ++j)
          wv[j] = (int)(((long long)min(n0 + 16 * j + px, g.CO - 1) * Kfl + c * CC + 8 * kgrp) * sizeof(T));
        auto wcol_of = [&](int st) {  // wave-uniform: scalar
          const int t = st / SUB, h = st - (st / SUB) * SUB;
          const int jy = (t * kwinv) >> 16, jx = t - jy * KWl;
          return ((ky0 + ks * jy) * KWf + kx0 + ks * jx) * Cl + 32 * h;
        };
        auto aoff_of = [&](int st) {
          const int t = st / SUB, h = st - (st / SUB) * SUB;
          const int jy = (t * kwinv) >> 16, jx = t - jy * KWl;
          return ((jy + dy) * PW + jx + dx) * PST + 32 * h;
        };
        // ring of PD weight fragments consumed in place (no copies) and refilled PD steps ahead
        constexpr int PD = WS ? (NT == 1 ? SPECENH_WS_PD1 : SPECENH_WS_PD2) : (NT >= 3 ? (CC == 64 ? 1 : 2) : (NT == 2 ? 2 : 8));
        V8<T> wring[PD][NT];
#pragma unroll
        for (int u = 0; u < PD; ++u)
          if (u < nsteps) {
            const int col = wcol_of(u);
#pragma unroll
            for (int j = 0; j < NT; ++j) wring[u][j] = ldw<T>(wrs, wv[j], col * (int)sizeof(T));
          }
        // whole rounds of PD steps with unconditional refills (the last PD refills re-load
        // the last step's column, unused), so every ring slot is refilled exactly once per
        // round and the compiler keeps the slots in place: a step waits only for its own
        // slot's load, PD - 1 rounds old. A conditional refill had the slots rotated through
        // register copies and every step waiting for the youngest load (vmcnt(0)).
        int s0 = 0;
        for (; s0 + PD <= nsteps; s0 += PD)
#pragma unroll
        for (int u = 0; u < PD; ++u) {
          const int st = s0 + u;
          const int aoff = aoff_of(st) + 8 * kgrp;
          V8<T> pv[MT];
#pragma unroll
          for (int i = 0; i < MT; ++i) {
            const uint4 q = *reinterpret_cast<const uint4*>(sP + rbase[i] + aoff);  // ds_read_b128
            pv[i].w[0] = q.x; pv[i].w[1] = q.y; pv[i].w[2] = q.z; pv[i].w[3] = q.w;
          }
#pragma unroll
          for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int j = 0; j < NT; ++j) acc[i][j] = mfma32<T>(wring[u][j], pv[i], acc[i][j]);
          const int col = wcol_of(min(st + PD, nsteps - 1));
#pragma unroll
          for (int j = 0; j < NT; ++j) wring[u][j] = ldw<T>(wrs, wv[j], col * (int)sizeof(T));
        }
#pragma unroll
        for (int u = 0; u < PD - 1; ++u) {  // the remaining nsteps % PD steps: slots 0, 1, ..
          const int st = s0 + u;
          if (st >= nsteps) break;
          const int aoff = aoff_of(st) + 8 * kgrp;
          V8<T> pv[MT];
#pragma unroll
          for (int i = 0; i < MT; ++i) {
            const uint4 q = *reinterpret_cast<const uint4*>(sP + rbase[i] + aoff);
            pv[i].w[0] = q.x; pv[i].w[1] = q.y; pv[i].w[2] = q.z; pv[i].w[3] = q.w;
          }
#pragma unroll
          for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int j = 0; j < NT; ++j) acc[i][j] = mfma32<T>(wring[u][j], pv[i], acc[i][j]);
        }
      } else if constexpr (CC == 16) {
        // ---- 16 channels: one MFMA K=32 slab = two taps (lane groups kgrp 0-1: tap 2st,
        // 2-3: tap 2st+1). Same branch-free scheme as above; the missing second tap of an
        // odd tap count is a zeroed weight fragment on the last step ----
        const int KWl = g.KW, Kfl = g.Kf, Cl = g.C, KWf = g.KWf, ks = g.kstep;
        const int ky0 = g.ky0, kx0 = g.kx0;
        const int dy = upt - g.pad_t, dx = upl - g.pad_l;
        const int kwinv = (65536 + KWl - 1) / KWl;
        const int nsteps = (ntap + 1) / 2;
        const bool second = (kgrp >> 1) != 0;
        const __amdgpu_buffer_rsrc_t wrs = weight_rsrc(W, (long long)g.CO * Kfl * sizeof(T));
        int wv[NT];
#pragma unroll
        for (int j = 0; j < NT; ++j)
          wv[j] = (int)(((long long)min(n0 + 16 * j + px, g.CO - 1) * Kfl + c * CC + 8 * (kgrp & 1)) * sizeof(T));
        auto wcol_t = [&](int t) {
          const int jy = (t * kwinv) >> 16, jx = t - jy * KWl;
          return ((ky0 + ks * jy) * KWf + kx0 + ks * jx) * Cl;
        };
        auto aoff_t = [&](int t) {
          const int jy = (t * kwinv) >> 16, jx = t - jy * KWl;
          if constexpr (S2)
            return (((jy & 1) * 2 + (jx & 1)) * SPH * SPW + (jy >> 1) * SPW + (jx >> 1)) * PST;
          else
            return ((jy + dy) * PW + jx + dx) * PST;
        };
        // the two taps' columns are wave-uniform: the first as the soffset, the second as a
        // per-lane delta (lane groups 2-3 take tap 2st + 1)
        auto wload = [&](int st, V8<T> (&dst)[NT]) {
          const int c0 = wcol_t(2 * st), c1 = wcol_t(min(2 * st + 1, ntap - 1));
          const int dl = second ? (c1 - c0) * (int)sizeof(T) : 0;
#pragma unroll
          for (int j = 0; j < NT; ++j) dst[j] = ldw<T>(wrs, wv[j] + dl, c0 * (int)sizeof(T));
        };
        if constexpr (K5) {
          // 13 steps of two taps, all offsets immediates: tap t = (jy, jx) sits at patch
          // offset (jy * 20 + jx) * 16 and weight column 16 t. Lane groups 2-3 read tap
          // 2st + 1: +16 elements in the weight row, and in the patch +16 (same kernel row)
          // or +(20 - 4) * 16 (tap 2st ends a row) -- two per-lane bases, chosen per step
          // at compile time.
          constexpr int PWc = TILE - 1 + 5;
          const T* wb = reinterpret_cast<const T*>(sP_raw + a.wl_off) + px * a.wl_rs +
                        8 * (kgrp & 1) + (second ? 16 : 0);
          // the last step has no tap 25: lane groups 2-3 re-read tap 24's weights (their
          // patch operand is zero); past the last weight row is unallocated LDS, whose
          // stale bits could be Inf/NaN (and 0 x Inf is NaN)
          const T* wbl = wb - (second ? 16 : 0);
          int pb0[MT], pb1[MT];
#pragma unroll
          for (int i = 0; i < MT; ++i) {
            pb0[i] = rbase[i] + 8 * (kgrp & 1) + (second ? PST : 0);
            pb1[i] = rbase[i] + 8 * (kgrp & 1) + (second ? (PWc - 4) * PST : 0);
          }
#pragma unroll
          for (int st = 0; st < 13; ++st) {
            const int t0 = 2 * st, jy = t0 / 5, jx = t0 % 5;
            const int ao = (jy * PWc + jx) * PST;
            V8<T> wf[NT], pv[MT];
#pragma unroll
            for (int j = 0; j < NT; ++j) {
              const uint4 q = *reinterpret_cast<const uint4*>((st == 12 ? wbl : wb) + 16 * j * a.wl_rs + 16 * t0);
              wf[j].w[0] = q.x; wf[j].w[1] = q.y; wf[j].w[2] = q.z; wf[j].w[3] = q.w;
            }
#pragma unroll
            for (int i = 0; i < MT; ++i) {
              const uint4 q = *reinterpret_cast<const uint4*>(sP + (jx == 4 ? pb1[i] : pb0[i]) + ao);
              pv[i].w[0] = q.x; pv[i].w[1] = q.y; pv[i].w[2] = q.z; pv[i].w[3] = q.w;
            }
            if (st == 12 && second) {  // tap 25 does not exist
#pragma unroll
              for (int i = 0; i < MT; ++i) zero8(pv[i]);
            }
#pragma unroll
            for (int i = 0; i < MT; ++i)
#pragma unroll
              for (int j = 0; j < NT; ++j) acc[i][j] = mfma32<T>(wf[j], pv[i], acc[i][j]);
          }
        } else if constexpr (WL) {
          // weights from the LDS copy: no global loads (and no vmcnt waits) in the k-loop
          const T* sWt = reinterpret_cast<const T*>(sP_raw + a.wl_off) + px * a.wl_rs + 8 * (kgrp & 1);
          for (int st = 0; st < nsteps; ++st) {
            const int a0 = aoff_t(2 * st), a1 = aoff_t(min(2 * st + 1, ntap - 1));
            const int aoff = (second ? a1 : a0) + 8 * (kgrp & 1);
            const int c0 = wcol_t(2 * st), c1 = wcol_t(min(2 * st + 1, ntap - 1));
            const int wo = second ? c1 : c0;
            V8<T> wf[NT], pv[MT];
#pragma unroll
            for (int j = 0; j < NT; ++j) {
              const uint4 q = *reinterpret_cast<const uint4*>(sWt + 16 * j * a.wl_rs + wo);
              wf[j].w[0] = q.x; wf[j].w[1] = q.y; wf[j].w[2] = q.z; wf[j].w[3] = q.w;
            }
#pragma unroll
            for (int i = 0; i < MT; ++i) {
              const uint4 q = *reinterpret_cast<const uint4*>(sP + rbase[i] + aoff);
              pv[i].w[0] = q.x; pv[i].w[1] = q.y; pv[i].w[2] = q.z; pv[i].w[3] = q.w;
            }
            if (__builtin_expect(2 * st + 1 >= ntap, 0)) {
              if (second) {
#pragma unroll
                for (int i = 0; i < MT; ++i) zero8(pv[i]);
              }
              __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
            for (int i = 0; i < MT; ++i)
#pragma unroll
              for (int j = 0; j < NT; ++j) acc[i][j] = mfma32<T>(wf[j], pv[i], acc[i][j]);
          }
        } else {
        constexpr int PD = WS ? (NT == 1 ? 4 : 2) : (NT >= 3 ? 2 : (NT == 2 ? 2 : 8));
        V8<T> wring[PD][NT];
#pragma unroll
        for (int u = 0; u < PD; ++u)
          if (u < nsteps) wload(u, wring[u]);
        for (int s0 = 0; s0 < nsteps; s0 += PD)
#pragma unroll
        for (int u = 0; u < PD; ++u) {
          const int st = s0 + u;
          if (st >= nsteps) break;
          const int a0 = aoff_t(2 * st), a1 = aoff_t(min(2 * st + 1, ntap - 1));
          const int aoff = (second ? a1 : a0) + 8 * (kgrp & 1);
          V8<T> pv[MT];
#pragma unroll
          for (int i = 0; i < MT; ++i) {
            const uint4 q = *reinterpret_cast<const uint4*>(sP + rbase[i] + aoff);  // ds_read_b128
            pv[i].w[0] = q.x; pv[i].w[1] = q.y; pv[i].w[2] = q.z; pv[i].w[3] = q.w;
          }
          if (__builtin_expect(2 * st + 1 >= ntap, 0)) {  // last step of an odd tap count:
            // no second tap (a wave-uniform branch: the zeroing stays out of the other steps)
            if (second) {
#pragma unroll
              for (int i = 0; i < MT; ++i) zero8(pv[i]);
            }
            __builtin_amdgcn_sched_barrier(0);
          }
#pragma unroll
          for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int j = 0; j < NT; ++j) acc[i][j] = mfma32<T>(wring[u][j], pv[i], acc[i][j]);
          if (st + PD < nsteps) wload(st + PD, wring[u]);
        }
        }  // !WL
      } else {
        // ---- k-steps: one MFMA K=32 slab each; weights are the A operand (rows = output
        // channels), the patch the B operand (columns = pixels): D[channel][pixel] ----
        constexpr int SUB = CC >= 32 ? CC / 32 : 1;  // 32-channel slabs per tap
        const int nsteps = CC >= 32 ? ntap * SUB : (CC == 16 ? (ntap + 1) / 2 : 1);
        auto load_w = [&](int st, V8<T> (&b)[NT]) {
  #pragma unroll
          for (int j = 0; j < NT; ++j) {
            const int co = n0 + 16 * j + px;
            zero8(b[j]);
            if constexpr (CC >= 32) {
              const int t = st / SUB, h = st - (st / SUB) * SUB;
              if (co < g.CO) b[j] = ld8(W + co * g.Kf + sCol[p][t] + c * CC + 32 * h + 8 * kgrp);
            } else if constexpr (CC == 16) {
              const int t = 2 * st + (kgrp >> 1);
              if (co < g.CO && t < ntap) b[j] = ld8(W + co * g.Kf + sCol[p][t] + 8 * (kgrp & 1));
            } else {
  #pragma unroll
              for (int q = 0; q < 8; ++q) {
                const int t = 8 * kgrp + q;
                if (co < g.CO && t < ntap) set_elem(b[j], q, W[co * g.Kf + sCol[p][t]]);
              }
            }
          }
        };
        // weight fragments PD k-steps ahead in a register ring: they come from L2, and one
        // k-step of MFMA work (4*NT MFMAs, 64-256 cycles) does not cover that latency
        constexpr int PD = NT >= 3 ? (CC == 64 ? 1 : 2) : (NT == 2 ? 2 : 8);
        V8<T> wring[PD][NT];
  #pragma unroll
        for (int u = 0; u < PD; ++u)
          if (u < nsteps) load_w(u, wring[u]);
        for (int s0 = 0; s0 < nsteps; s0 += PD)
  #pragma unroll
        for (int u = 0; u < PD; ++u) {
          const int st = s0 + u;
          if (st >= nsteps) break;
          V8<T> wcur[NT];
  #pragma unroll
          for (int j = 0; j < NT; ++j) wcur[j] = wring[u][j];
          if (st + PD < nsteps) load_w(st + PD, wring[u]);
          int aoff = 0;
          bool aon = true;
          if constexpr (CC >= 32) {
            const int t = st / SUB, h = st - (st / SUB) * SUB;
            aoff = sTap[p][t] + 32 * h + 8 * kgrp;
          } else if constexpr (CC == 16) {
            const int t = 2 * st + (kgrp >> 1);
            aon = t < ntap;
            aoff = (aon ? sTap[p][t] : 0) + 8 * (kgrp & 1);
          }
  #pragma unroll
          for (int i = 0; i < MT; ++i) {
            V8<T> pv;
            if constexpr (CC == 1) {
              zero8(pv);
  #pragma unroll
              for (int q = 0; q < 8; ++q) {
                const int off = sTap[p][8 * kgrp + q];
                if (off >= 0) set_elem(pv, q, sP[rbase[i] + off]);
              }
            } else {
              const uint4 u = *reinterpret_cast<const uint4*>(sP + rbase[i] + aoff);  // ds_read_b128
              pv.w[0] = u.x; pv.w[1] = u.y; pv.w[2] = u.z; pv.w[3] = u.w;
              if (!aon) zero8(pv);
            }
  #pragma unroll
            for (int j = 0; j < NT; ++j) acc[i][j] = mfma32<T>(wcur[j], pv, acc[i][j]);
          }
        }
      }
    }

    // ---- epilogue: lane holds channels n0 + 16j + 4*kgrp + r (r = 0..3) of output
    // pixel (row oy0 + 4*wave + i, column ox0 + px) — 4 consecutive NHWC channels ----
    float bv[NT][4];
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ch = n0 + 16 * j + 4 * kgrp + r;
        bv[j][r] = (a.bias && ch < g.CO) ? a.bias[ch] : 0.f;
      }
    const int ox = ox0 + px;
    if constexpr (POOL) {
      // 2x2 windows: rows (2ip, 2ip+1) of this wave in registers, columns (px, px^1) across
      // the lane pair; values compared as stored (rounded to T), first max wins
      const int PHo = g.OH / 2, PWo = g.OW / 2;
      if (!a.argmax && (g.CO & 3) == 0 && a.act <= 1) {
        // inference: the pooled value only. x -> round_T(act(x + b)) is monotone, so the
        // max of the four stored values is that map of the max accumulator: max first
        // (in-lane rows, then the lane pair), one bias add / ReLU / rounding per output.
        const bool relu = a.act == 1;
#pragma unroll
        for (int ip = 0; ip < MT / 2; ++ip) {
          const int oy = oy0 + wrow * MT + 2 * ip;
          const int py = oy / 2, pxo = ox / 2;
          const bool store = (px & 1) == 0 && py < PHo && pxo < PWo;
#pragma unroll
          for (int j = 0; j < NT; ++j) {
            float m[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float m1 = vmax(acc[2 * ip][j][r], acc[2 * ip + 1][j][r]);
              float v = vmax(m1, __shfl_xor(m1, 1)) + bv[j][r];
              m[r] = relu ? vmax(v, 0.f) : v;
            }
            const int ch0 = n0 + 16 * j + 4 * kgrp;
            if (store && ch0 < g.CO) {
              const long long o = (((long long)n * PHo + py) * PWo + pxo) * g.CO + ch0;
              *reinterpret_cast<uint2*>(reinterpret_cast<T*>(a.out) + o) =
                  uint2{pack2<T>(m[0], m[1]), pack2<T>(m[2], m[3])};
            }
          }
        }
      } else
#pragma unroll
      for (int ip = 0; ip < MT / 2; ++ip) {
        const int oy = oy0 + wrow * MT + 2 * ip;
        const int py = oy / 2, pxo = ox / 2;
        const bool store = (px & 1) == 0 && py < PHo && pxo < PWo;
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          float best[4];
          unsigned arg4 = 0;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float v00 = to_f(from_f<T>(apply_act(acc[2 * ip][j][r] + bv[j][r], a.act)));
            const float v10 = to_f(from_f<T>(apply_act(acc[2 * ip + 1][j][r] + bv[j][r], a.act)));
            const float v01 = __shfl_xor(v00, 1);
            const float v11 = __shfl_xor(v10, 1);
            float b = v00;
            unsigned q = 0;
            if (v01 > b) { b = v01; q = 1; }
            if (v10 > b) { b = v10; q = 2; }
            if (v11 > b) { b = v11; q = 3; }
            best[r] = b;
            arg4 |= q << (8 * r);
          }
          const int ch0 = n0 + 16 * j + 4 * kgrp;
          if (store && ch0 < g.CO) {
            const long long o = (((long long)n * PHo + py) * PWo + pxo) * g.CO + ch0;
            T* dst = reinterpret_cast<T*>(a.out) + o;
            if ((g.CO & 3) == 0) {
              V8<T> pk;
              zero8(pk);
#pragma unroll
              for (int r = 0; r < 4; ++r) set_elem(pk, r, from_f<T>(best[r]));
              *reinterpret_cast<uint2*>(dst) = uint2{pk.w[0], pk.w[1]};
              if (a.argmax) *reinterpret_cast<unsigned*>(a.argmax + o) = arg4;
            } else {
#pragma unroll
              for (int r = 0; r < 4; ++r)
                if (ch0 + r < g.CO) {
                  dst[r] = from_f<T>(best[r]);
                  if (a.argmax) a.argmax[o + r] = (unsigned char)(arg4 >> (8 * r));
                }
            }
          }
        }
      }
    } else if constexpr (PAIR) {
      uint32_t pk[MT][NT][2];
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          V8<T> q;
          zero8(q);
#pragma unroll
          for (int r = 0; r < 4; ++r) set_elem(q, r, from_f<T>(apply_act(acc[i][j][r] + bv[j][r], a.act)));
          pk[i][j][0] = q.w[0];
          pk[i][j][1] = q.w[1];
        }
      if (p == ph_lo) {
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
          for (int j = 0; j < NT; ++j) {
            hold[i][j][0] = pk[i][j][0];
            hold[i][j][1] = pk[i][j][1];
          }
      } else {
        constexpr int CO = 16 * NT;  // the workgroup holds every channel (host-checked)
        constexpr int PS = 2 * CO + 8;  // a pixel pair + 16 B: spreads the lanes' 8-B writes
        constexpr int QV = 2 * CO / 8;  // 16-byte vectors per pixel pair
        lds_sync();  // every wave's fragment reads of the patch are done
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
          for (int j = 0; j < NT; ++j) {
            const int o = ((wrow * MT + i) * 16 + px) * PS + 16 * j + 4 * kgrp;
            *reinterpret_cast<uint2*>(sP + o) = uint2{hold[i][j][0], hold[i][j][1]};
            *reinterpret_cast<uint2*>(sP + o + CO) = uint2{pk[i][j][0], pk[i][j][1]};
          }
        lds_sync();
        T* __restrict__ out = reinterpret_cast<T*>(a.out);
        const int obase = ((n * g.OHs + pyp) * g.OWs + 2 * ox0) * CO;
        for (int e = tid; e < 16 * 16 * QV; e += 256) {
          const int r = e / (16 * QV), c = e - r * (16 * QV);  // row, vector in the row
          const int q = c / QV;                                 // pixel pair = input column
          if (oy0 + r >= g.OH || ox0 + q >= g.OW) continue;
          const int o = obase + 2 * (oy0 + r) * g.OWs * CO + 8 * c;
          *reinterpret_cast<uint4*>(out + o) =
              *reinterpret_cast<const uint4*>(sP + (r * 16 + q) * PS + 8 * (c - q * QV));
        }
      }
    } else if (!a.logits && !a.out_f32 && (g.CO & 3) == 0 && a.act <= 1) {
      // the inference/activation-store path: 32-bit offsets, branch-free ReLU, 8-byte stores;
      // the backward pass's ReLU mask as 8-byte loads at the same offsets (act(0) = 0 here)
      const bool relu = a.act == 1;
      const int CO = g.CO, OWs = g.OWs;
      const int pbase = (n * g.OHs + g.oy0) * OWs + g.ox0 + ox * g.oxs;
      T* __restrict__ out = reinterpret_cast<T*>(a.out);
      const T* __restrict__ mk = reinterpret_cast<const T*>(a.mask);
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const int oy = oy0 + wrow * MT + i;
        if (oy >= g.OH || ox >= g.OW) continue;
        const int o = (pbase + oy * g.oys * OWs) * CO;
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          const int ch0 = n0 + 16 * j + 4 * kgrp;
          if (ch0 >= CO) continue;
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float x = acc[i][j][r] + bv[j][r];
            v[r] = relu ? vmax(x, 0.f) : x;
          }
          if (mk) {
            const uint2 m = *reinterpret_cast<const uint2*>(mk + o + ch0);
            const uint32_t mw[2] = {m.x, m.y};
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const T mv = __builtin_bit_cast(T, (unsigned short)(mw[r >> 1] >> (16 * (r & 1))));
              v[r] = to_f(mv) > 0.f ? v[r] : 0.f;
            }
          }
          *reinterpret_cast<uint2*>(out + o + ch0) = uint2{pack2<T>(v[0], v[1]), pack2<T>(v[2], v[3])};
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const int oy = oy0 + wrow * MT + i;
        if (oy >= g.OH || ox >= g.OW) continue;
        const long long pix =
            ((long long)n * g.OHs + oy * g.oys + g.oy0) * g.OWs + ox * g.oxs + g.ox0;
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          const int ch0 = n0 + 16 * j + 4 * kgrp;
          if (ch0 >= g.CO) continue;
          const long long o = pix * g.CO + ch0;
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r] + bv[j][r];
          if (a.mask || a.logits || (g.CO & 3) != 0) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              if (ch0 + r >= g.CO) continue;
              float x = v[r];
              if (a.logits) a.logits[o + r] = x;
              if (a.mask && !(to_f(reinterpret_cast<const T*>(a.mask)[o + r]) > 0.f)) x = 0.f;
              x = apply_act(x, a.act);
              if (a.out_f32) reinterpret_cast<float*>(a.out)[o + r] = x;
              else reinterpret_cast<T*>(a.out)[o + r] = from_f<T>(x);
            }
          } else if (a.out_f32) {
            *reinterpret_cast<float4*>(reinterpret_cast<float*>(a.out) + o) =
                float4{apply_act(v[0], a.act), apply_act(v[1], a.act), apply_act(v[2], a.act),
                       apply_act(v[3], a.act)};
          } else {
            V8<T> pk;
            zero8(pk);
#pragma unroll
            for (int r = 0; r < 4; ++r) set_elem(pk, r, from_f<T>(apply_act(v[r], a.act)));
            *reinterpret_cast<uint2*>(reinterpret_cast<T*>(a.out) + o) = uint2{pk.w[0], pk.w[1]};
          }
        }
      }
    }
  }
  };
  if constexpr (K5) {
    // persistent: the weight rows stay in LDS for all of the workgroup's tiles
    const Geo& gk = a.g[0];
    const int total = gk.N * ((gk.OH + 15) / 16) * ((gk.OW + 15) / 16);
    bool first = true;
    for (int t = (int)blockIdx.x; t < total; t += (int)gridDim.x) {
      body(t, first);
      first = false;
    }
  } else {
    body((int)blockIdx.x, true);
  }
}

// ------------------------------------------------------------------ weight gradient
struct WgradArgs {
  Geo g[MAXPH];
  int chunk[MAXPH];  // pixels per z-slice of each phase (multiple of the pixel step)
  int Z;             // z-slices per phase
  const void* in;
  const void* dout;  // [N][OHs][OWs][CO]
  float* part;       // [Z][CO][Kf]
  float* bpart;      // [nphase][Z][CO] (bias) or null
  // dOut given as the gradient of the following MaxPooling2D((2,2)) (specenh_conv2d_wgrad_pooled):
  // dOut[y][x][c] = pd[y/2][x/2][c] where argmax pam == 2 (y&1) + (x&1) and pooled py > 0
  const void* pd = nullptr;
  const unsigned char* pam = nullptr;
  const void* py = nullptr;  // or null: no ReLU mask
  bool overwrite = false;    // dw / dbias = the gradient (specenh_conv2d_wgrad_pooled)
};

// Workgroup: 64 GEMM-K columns (blockIdx.x) x 16*NT channels (blockIdx.y) x one pixel
// chunk (blockIdx.z = phase*Z + z). Wave w owns k-columns 16w .. 16w+15.
template <typename T, int NT>
__global__ __launch_bounds__(256) void conv_wgrad_kernel(WgradArgs a) {
  constexpr int BP = Tile<T>::BK;  // pixels per step
  constexpr int LD = Tile<T>::LD;
  constexpr int BN = 16 * NT;
  __shared__ __attribute__((aligned(16))) T sA[64 * LD];  // [k][pixel]
  __shared__ __attribute__((aligned(16))) T sG[BN * LD];  // [co][pixel]
  const int ph = blockIdx.z / a.Z, z = blockIdx.z - (blockIdx.z / a.Z) * a.Z;
  const Geo& g = a.g[ph];
  const int K = g.KH * g.KW * g.C;
  const int k0 = blockIdx.x * 64;
  if (k0 >= K) return;
  const int n0 = blockIdx.y * BN;
  const int M = g.N * g.OH * g.OW;
  const int p_begin = z * a.chunk[ph];
  const int p_end = min(M, p_begin + a.chunk[ph]);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int hw = g.OH * g.OW;
  const T* __restrict__ in = reinterpret_cast<const T*>(a.in);
  const T* __restrict__ dout = reinterpret_cast<const T*>(a.dout);

  // bf16: thread = (pixel pair, 8-group); f32: thread = (pixel, 8-group)
  constexpr int PP = sizeof(T) == 2 ? 2 : 1;
  const int grp = tid & 7, pslot = (tid >> 3) * PP;  // pslot < BP
  const bool g_on = 8 * grp < BN;

  auto pix_geom = [&](int m, int& by, int& bx, int& nb, long long& orow) {
    if (m < p_end) {
      const int n = m / hw, rem = m - (m / hw) * hw;
      const int oy = rem / g.OW, ox = rem - (rem / g.OW) * g.OW;
      by = oy * g.stride - g.pad_t;
      bx = ox * g.stride - g.pad_l;
      nb = n * g.IH;
      orow = (((long long)n * g.OHs + oy * g.oys + g.oy0) * g.OWs + ox * g.oxs + g.ox0) * g.CO;
    } else {
      by = -(1 << 29); bx = 0; nb = 0; orow = -1;
    }
  };
  V8<T> va[PP], vg[PP];
  auto fetch = [&](int p0) {
#pragma unroll
    for (int q = 0; q < PP; ++q) {
      int by, bx, nb;
      long long orow;
      pix_geom(p0 + pslot + q, by, bx, nb, orow);
      va[q] = gather_a8<T>(in, g, K, k0 + 8 * grp, by, bx, nb);
      zero8(vg[q]);
      if (g_on && orow >= 0) {
        const int co = n0 + 8 * grp;
        if ((g.CO & 7) == 0 && co + 8 <= g.CO) {
          vg[q] = ld8(dout + orow + co);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (co + j < g.CO) set_elem(vg[q], j, dout[orow + co + j]);
        }
      }
    }
  };
  auto stage = [&]() {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if constexpr (PP == 2) {
        *reinterpret_cast<uint32_t*>(sA + (8 * grp + j) * LD + pslot) =
            elem_bits(va[0], j) | (elem_bits(va[1], j) << 16);
        if (g_on)
          *reinterpret_cast<uint32_t*>(sG + (8 * grp + j) * LD + pslot) =
              elem_bits(vg[0], j) | (elem_bits(vg[1], j) << 16);
      } else {
        *reinterpret_cast<uint32_t*>(sA + (8 * grp + j) * LD + pslot) = elem_bits(va[0], j);
        if (g_on) *reinterpret_cast<uint32_t*>(sG + (8 * grp + j) * LD + pslot) = elem_bits(vg[0], j);
      }
    }
  };

  f32x4 acc[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bacc = 0.f;
  const bool do_bias = a.bpart && blockIdx.x == 0 && tid < BN;

  if (p_begin < p_end) fetch(p_begin);
  for (int p0 = p_begin; p0 < p_end; p0 += BP) {
    stage();
    lds_sync();
    if (p0 + BP < p_end) fetch(p0 + BP);
#pragma unroll
    for (int j = 0; j < NT; ++j)
      acc[j] = mfma_slab<T>(sG + 16 * j * LD, sA + 16 * wave * LD, acc[j], lane);
    if (do_bias) {
#pragma unroll 8
      for (int p = 0; p < BP; ++p) bacc += to_f(sG[tid * LD + p]);
    }
    lds_sync();
  }

  // D[co][k]: col = lane & 15 -> k, row = 4*(lane >> 4) + reg -> co
  const int kc = k0 + 16 * wave + (lane & 15);
  if (kc < K) {
    const int tap = kc / g.C, ci = kc - (kc / g.C) * g.C;
    const int col = wcol(g, tap, ci);
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const int co = n0 + 16 * j + 4 * (lane >> 4) + reg;
        if (co < g.CO) a.part[((long long)z * g.CO + co) * g.Kf + col] = acc[j][reg];
      }
  }
  if (do_bias && n0 + tid < g.CO) a.bpart[((long long)ph * a.Z + z) * g.CO + n0 + tid] = bacc;
}

// ------------------------------------------------------------------ weight gradient, C % 16 == 0
// dW[co][(tap, ci)] = sum_p dOut[p][co] * in[p + tap][ci] as MFMA 16x16x32 with the 32 pixels
// as the reduction: A = dOut^T (16 co x 32 px), B = input window (32 px x 16 ci). A workgroup
// owns one phase, 16 input channels, 16*NTW output channels and a run of 16x16 output tiles;
// per tile the dOut tile ([pixel][co]) and the input patch ([pixel][16 ci]) are staged in LDS
// as plain NHWC rows (16-B copies) and the fragments come out with ds_read_b64_tr_b16
// (the transpose is free), so one staged dOut fragment feeds every tap: wave w owns taps
// w, w+4, ... (<= 7 of 25) and keeps 7 x NTW accumulators; the bias gradient is one more
// MFMA per co-block against a ones fragment. Partial sums per pixel run (blockIdx.x) go to
// part[z] and are reduced in a fixed order (ordered_sum_kernel): bit-reproducible.
struct WgradTrArgs {
  Geo g[MAXPH];
  int Z;     // tile runs per phase (blockIdx.x)
  int ncog;  // co groups of 16 * NTW (blockIdx.y = chunk * ncog + cog)
  int ntg;   // wgrad_tr_kernel: groups of 28 taps (blockIdx.z = phase * ntg + group; k 7: 2)
  const void* in;
  const void* dout;  // [N][OHs][OWs][CO]
  float* part;       // [Z][CO][Kf]
  float* bpart;      // [nphase][Z][CO] or null
  int upt, upl, PH, PW;  // phase-shared launches (wgrad_trp_kernel): the union patch
  const void* pd;        // dOut from the pool's gradient (WgradArgs::pd), or null
  const unsigned char* pam;
  const void* py;
};

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));

// rows q = 0..3 of a 4 x 16 block of 16-bit elements, transposed across a 16-lane group
__device__ __forceinline__ s16x4 lds_tr16(const void* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(const_cast<void*>(p)));
}

template <typename T>
__device__ __forceinline__ f32x4 mfma_s16(s16x8 a, s16x8 b, f32x4 acc) {
  if constexpr (__is_same(T, __bf16))
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                   __builtin_bit_cast(bf16x8, b), acc, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a),
                                                  __builtin_bit_cast(f16x8, b), acc, 0, 0, 0);
}

// C1 (one input channel, the first Conv2D): the B tile is an im2col block built in LDS per tile
// ([256 pixels][32 taps], taps >= KH*KW zero, tap 31 = 1 so column 31 of D is the bias
// gradient); waves w take k-block w & 1 over pixel groups of parity w >> 1 and pairs of waves
// are summed in a fixed order at the end. The next tile's global data is prefetched into
// registers while the current tile computes.
#ifndef SPECENH_WGRAD_SWZ
#define SPECENH_WGRAD_SWZ 1
#endif
// PD: dOut routed from a pool's gradient (WgradTrArgs::pd) — compiled in for C1 (the model's
// first Conv2D, run-time test) and the PD instantiations (round 6: the pooled Conv2Ds after it)
// only, so the other layers' kernels keep their registers
template <typename T, int NTW, bool C1, bool PD = false>
__global__ __launch_bounds__(256) void wgrad_tr_kernel(WgradTrArgs a) {
  constexpr int CH = 16;             // input channels per workgroup: one k-block per tap
  constexpr int COT = 16 * NTW;      // output channels per workgroup
  // SWZ (round 5): a half-wave's transposed reads cover 8 CONSECUTIVE pixels (K element k of
  // lane group g4: pixel 4 (g4 & 1) + (k & 3) + 8 (k >> 2) of its tile row; round 4 read
  // columns 0-3 and 8-11 together) from unpadded 32-byte pixel rows: 256 B = all 64 banks,
  // whatever the tap offset; 64-byte dOut rows (32 channels) swap their two 32-byte chunks on
  // pixel bit 2. PMC had SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE 0.50 with padded rows.
  constexpr bool SWZ = SPECENH_WGRAD_SWZ != 0;
  constexpr int DST = SWZ ? COT : COT + 8;  // dOut tile row stride (elements)
  constexpr int PST = C1 ? 40 : (SWZ ? CH : CH + 8);  // B rows: im2col taps (C1) or patch pixel channels
  constexpr int HI = SWZ ? 8 : 4;           // pixel step of a fragment's second 4 K elements
  constexpr int MAXT = C1 ? 1 : 7;   // taps (k-blocks) per wave
  constexpr int PROWS = C1 ? 256 : 484;  // the 22 x 22 patch of a 7 x 7 kernel
  constexpr int NDV = COT / 8;       // dOut uint4 per thread (256 pixels x COT channels)
  constexpr int NPV = C1 ? 2 : 4;    // patch elements (C1: T) / uint4 per thread
  __shared__ __attribute__((aligned(16))) T sD[256 * DST];
  __shared__ __attribute__((aligned(16))) T sP[PROWS * PST];
  __shared__ __attribute__((aligned(16))) T sIn[C1 ? 20 * 20 : 8];
  const int ph = blockIdx.z / a.ntg, tb = 28 * (blockIdx.z - ph * a.ntg);  // first tap
  const Geo& g = a.g[ph];
  const int chunk = blockIdx.y / a.ncog, cog = blockIdx.y - (blockIdx.y / a.ncog) * a.ncog;
  const int c0 = chunk * CH, co0 = cog * COT;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ntx = (g.OW + 15) / 16, nty = (g.OH + 15) / 16;
  const long long ntiles = (long long)g.N * nty * ntx;
  const long long t_begin = blockIdx.x * ntiles / a.Z, t_end = (blockIdx.x + 1) * ntiles / a.Z;
  const int ntap = g.KH * g.KW;
  const int PW = 16 + g.KW - 1, PH = 16 + g.KH - 1;
  const T* __restrict__ in = reinterpret_cast<const T*>(a.in);
  const T* __restrict__ dout = reinterpret_cast<const T*>(a.dout);
  const bool co_vec = (g.CO & 7) == 0, co_one = g.CO == 1;

  f32x4 acc[MAXT][NTW];
#pragma unroll
  for (int t = 0; t < MAXT; ++t)
#pragma unroll
    for (int j = 0; j < NTW; ++j) acc[t][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 bacc[NTW];
#pragma unroll
  for (int j = 0; j < NTW; ++j) bacc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bool do_bias = !C1 && a.bpart && chunk == 0 && wave == 0 && tb == 0;
  s16x8 ones;
  const short one = __builtin_bit_cast(short, from_f<T>(1.f));
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = one;

  // tr-read lane roles: group g4 = lane >> 4 owns MFMA K-elements 8 g4 .. 8 g4 + 7 = pixels
  // (row 2 pg + (g4 >> 1), columns 8 (g4 & 1) .. + 7) of pixel group pg; lane 4q + p of the
  // group addresses row q (pixel column + q, + 4 for the upper half) and elements 4p .. 4p+3
  const int g4 = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  const int prow = g4 >> 1, pcol = (SWZ ? 4 : 8) * (g4 & 1) + q;
  // dOut chunk slot of 16-channel chunk j at pixel P (element offset 16 dch(P, j))
  auto dch = [](int P, int j) { return (SWZ && COT == 32) ? (j ^ ((P >> 2) & 1)) : j; };
  // C1: the im2col taps t < 31 as offsets jy PW + jx into the staged patch (uniform)
  int c1off[C1 ? 31 : 1];
#pragma unroll
  for (int t = 0; t < (C1 ? 31 : 1); ++t) {
    const int tc = min(t, ntap - 1);
    c1off[t] = (tc / g.KW) * PW + tc - (tc / g.KW) * g.KW;
  }
  // this wave's taps t = wave + 4 tt as patch offsets (elements), formed once; taps past the
  // kernel repeat the last one (their MFMAs run, their sums are never stored)
  int toff[C1 ? 1 : MAXT];
#pragma unroll
  for (int tt = 0; tt < (C1 ? 1 : MAXT); ++tt) {
    const int t = min(tb + wave + 4 * tt, ntap - 1);
    const int jy = t / g.KW, jx = t - (t / g.KW) * g.KW;
    toff[tt] = (jy * PW + jx) * PST;
  }

  // ---- per-thread prefetch registers of one tile ----
  uint4 rd[NDV];
  T rd1;               // CO == 1: this thread's pixel
  uint4 rp[C1 ? 1 : NPV];
  T rp1[C1 ? NPV : 1];
  auto tile_org = [&](long long tile, int& n, int& oyt, int& oxt) {
    // 32-bit unsigned divisions (the host keeps N x tiles below 2^31): the 64-bit divide
    // routine had cost ~200 SALU per tile
    const unsigned tu = (unsigned)tile, per = (unsigned)(nty * ntx);
    n = (int)(tu / per);
    const unsigned trem = tu - (unsigned)n * per;
    oyt = (int)(trem / (unsigned)ntx) * 16;
    oxt = (int)(trem - (trem / (unsigned)ntx) * (unsigned)ntx) * 16;
  };
  // dOut element u of this thread: (tile pixel, 8-channel vector). Routed from a pool's
  // gradient with 4 vectors per pixel, a thread takes ONE pooled (pixel, vector) and its 2 x 2
  // full-resolution block (u = 2 dy + dx), so each pooled value is loaded once, not 4 times
  const bool rblk = PD && NDV == 4;
  auto dmap = [&](int u, int& pix, int& v) {
    if (rblk) {
      const int qp = tid >> 2;
      v = tid & 3;
      pix = ((2 * (qp >> 3) + (u >> 1)) << 4) + 2 * (qp & 7) + (u & 1);
    } else {
      const int e = tid + 256 * u;
      pix = e / NDV;
      v = e - pix * NDV;
    }
  };
  auto fetch = [&](long long tile) {
    int n, oyt, oxt;
    tile_org(tile, n, oyt, oxt);
    if (PD && co_vec && rblk) {
      const int qp = tid >> 2;
      const int oy = oyt + 2 * (qp >> 3), ox = oxt + 2 * (qp & 7);  // the block's top left
      const int co = co0 + 8 * (tid & 3);
      uint4 dv = uint4{0u, 0u, 0u, 0u};
      uint4 yv = uint4{POOL_ROUTE_POS, POOL_ROUTE_POS, POOL_ROUTE_POS, POOL_ROUTE_POS};
      uint2 am = uint2{0u, 0u};
      const bool ok = oy < g.OH && ox < g.OW && co < g.CO;  // (even OH, OW: whole block)
      if (ok) {
        const long long po = (((long long)n * (g.OH >> 1) + (oy >> 1)) * (g.OW >> 1) + (ox >> 1)) * g.CO + co;
        dv = *reinterpret_cast<const uint4*>(reinterpret_cast<const T*>(a.pd) + po);
        am = *reinterpret_cast<const uint2*>(a.pam + po);
        if (a.py) yv = *reinterpret_cast<const uint4*>(reinterpret_cast<const T*>(a.py) + po);
      }
#pragma unroll
      for (int u = 0; u < NDV; ++u) rd[u] = pool_route8(dv, am, yv, (uint32_t)u);
    } else if (co_vec) {
#pragma unroll
      for (int u = 0; u < NDV; ++u) {
        const int e = tid + 256 * u;
        const int pix = e / NDV, v = e - (e / NDV) * NDV;
        const int oy = oyt + (pix >> 4), ox = oxt + (pix & 15);
        const int co = co0 + 8 * v;
        rd[u] = uint4{0u, 0u, 0u, 0u};
        if ((C1 || PD) && a.pd) {  // routed from the pool's gradient: argmax select + ReLU mask
          if (oy < g.OH && ox < g.OW && co < g.CO) {
            const long long po = (((long long)n * (g.OH >> 1) + (oy >> 1)) * (g.OW >> 1) + (ox >> 1)) * g.CO + co;
            const uint4 dv = *reinterpret_cast<const uint4*>(reinterpret_cast<const T*>(a.pd) + po);
            const uint2 am = *reinterpret_cast<const uint2*>(a.pam + po);
            uint4 yv = uint4{POOL_ROUTE_POS, POOL_ROUTE_POS, POOL_ROUTE_POS, POOL_ROUTE_POS};
            if (a.py) yv = *reinterpret_cast<const uint4*>(reinterpret_cast<const T*>(a.py) + po);
            rd[u] = pool_route8(dv, am, yv, (uint32_t)(((oy & 1) << 1) | (ox & 1)));
          }
          continue;
        }
        if (oy < g.OH && ox < g.OW && co < g.CO)
          rd[u] = *reinterpret_cast<const uint4*>(
              dout + (((long long)n * g.OHs + oy * g.oys + g.oy0) * g.OWs + ox * g.oxs + g.ox0) * g.CO + co);
      }
    } else if (co_one) {
      const int oy = oyt + (tid >> 4), ox = oxt + (tid & 15);
      rd1 = from_f<T>(0.f);
      if (oy < g.OH && ox < g.OW)
        rd1 = dout[((long long)n * g.OHs + oy * g.oys + g.oy0) * g.OWs + ox * g.oxs + g.ox0];
    }
#pragma unroll
    for (int u = 0; u < NPV; ++u) {
      const int e = tid + 256 * u;
      if constexpr (C1) {
        const int py = e / PW, px = e - (e / PW) * PW;
        const int iy = oyt - g.pad_t + py, ix = oxt - g.pad_l + px;
        rp1[u] = from_f<T>(0.f);
        if (e < PH * PW && (unsigned)iy < (unsigned)g.IH && (unsigned)ix < (unsigned)g.IW)
          rp1[u] = in[((long long)n * g.IH + iy) * g.IW + ix];
      } else {
        const int pix = e >> 1, v = e & 1;
        const int py = pix / PW, px = pix - (pix / PW) * PW;
        const int iy = oyt - g.pad_t + py, ix = oxt - g.pad_l + px;
        rp[u] = uint4{0u, 0u, 0u, 0u};
        if (pix < PH * PW && (unsigned)iy < (unsigned)g.IH && (unsigned)ix < (unsigned)g.IW)
          rp[u] = *reinterpret_cast<const uint4*>(in + (((long long)n * g.IH + iy) * g.IW + ix) * g.C + c0 + 8 * v);
      }
    }
  };
  auto stage = [&](long long tile) {
    if (co_vec) {
#pragma unroll
      for (int u = 0; u < NDV; ++u) {
        int pix, v;
        dmap(u, pix, v);
        *reinterpret_cast<uint4*>(sD + pix * DST + 16 * dch(pix, v >> 1) + 8 * (v & 1)) = rd[u];
      }
    } else if (co_one) {
      const uint32_t w0 = __builtin_bit_cast(unsigned short, rd1);
#pragma unroll
      for (int v = 0; v < COT / 8; ++v)
        *reinterpret_cast<uint4*>(sD + tid * DST + 16 * dch(tid, v >> 1) + 8 * (v & 1)) =
            uint4{v == 0 ? w0 : 0u, 0u, 0u, 0u};
    } else {  // other narrow CO: element-wise, not prefetched
      int n, oyt, oxt;
      tile_org(tile, n, oyt, oxt);
      for (int e = tid; e < 256 * COT; e += 256) {
        const int pix = e / COT, c = e - (e / COT) * COT;
        const int oy = oyt + (pix >> 4), ox = oxt + (pix & 15);
        T val = from_f<T>(0.f);
        if (oy < g.OH && ox < g.OW && co0 + c < g.CO)
          val = dout[(((long long)n * g.OHs + oy * g.oys + g.oy0) * g.OWs + ox * g.oxs + g.ox0) * g.CO + co0 + c];
        sD[pix * DST + 16 * dch(pix, c >> 4) + (c & 15)] = val;
      }
    }
    if constexpr (C1) {
#pragma unroll
      for (int u = 0; u < NPV; ++u) {
        const int e = tid + 256 * u;
        if (e < PH * PW) sIn[e] = rp1[u];
      }
      lds_sync();
      // im2col row of this thread's pixel: taps (ky, kx) -> column ky*KW + kx; 31 = ones
      // (tap offsets from c1off, formed once: a run-time division per tap and tile had made
      // this kernel SALU-bound, 22 M SALU for 0.13 M MFMAs per C4 step)
      const T* const srow = sIn + (tid >> 4) * PW + (tid & 15);
#pragma unroll
      for (int t4 = 0; t4 < 8; ++t4) {
        uint32_t w[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          uint32_t pk = 0u;
#pragma unroll
          for (int e2 = 0; e2 < 2; ++e2) {
            const int t = 4 * t4 + 2 * h + e2;
            unsigned short b = 0;
            if (t == 31) {
              b = (unsigned short)one;
            } else if (t < ntap) {
              b = __builtin_bit_cast(unsigned short, srow[c1off[t]]);
            }
            pk |= (uint32_t)b << (16 * e2);
          }
          w[h] = pk;
        }
        *reinterpret_cast<uint2*>(sP + tid * PST + 4 * t4) = uint2{w[0], w[1]};
      }
    } else {
#pragma unroll
      for (int u = 0; u < NPV; ++u) {
        const int e = tid + 256 * u;
        const int pix = e >> 1, v = e & 1;
        if (pix < PH * PW) *reinterpret_cast<uint4*>(sP + pix * PST + 8 * v) = rp[u];
      }
    }
  };

  if (t_begin < t_end) fetch(t_begin);
  for (long long tile = t_begin; tile < t_end; ++tile) {
    lds_sync();  // the previous tile's fragment reads are done
    stage(tile);
    lds_sync();
    if (tile + 1 < t_end) fetch(tile + 1);  // in flight while this tile computes
    if constexpr (C1) {
      // wave w: k-block kb = w & 1 (taps 16 kb .. 16 kb + 15), pixel groups of parity w >> 1
      const int kb = wave & 1;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int pg = 2 * i + (wave >> 1);
        const int r = 2 * pg + prow;
        const T* da = sD + (r * 16 + pcol) * DST + 4 * pp;
        const T* pb = sP + (r * 16 + pcol) * PST + 16 * kb + 4 * pp;
        const s16x4 blo = lds_tr16(pb), bhi = lds_tr16(pb + HI * PST);
        const s16x8 bf = s16x8{blo[0], blo[1], blo[2], blo[3], bhi[0], bhi[1], bhi[2], bhi[3]};
#pragma unroll
        for (int j = 0; j < NTW; ++j) {
          const int jc = 16 * dch(pcol, j);
          const s16x4 lo = lds_tr16(da + jc), hi = lds_tr16(da + HI * DST + jc);
          const s16x8 af = s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          acc[0][j] = mfma_s16<T>(af, bf, acc[0][j]);
        }
      }
    } else {
      // Per pixel group: every fragment read is issued before the MFMAs that use it, and the
      // MFMAs run unconditionally (a tap past the kernel reads a clamped, valid offset; its
      // accumulator is never stored): round 4's loop read each tap's B fragment, waited
      // lgkmcnt(0) and formed the next tap's offset with a run-time division, serialising
      // ~15 SALU, an LDS round trip and two MFMAs per tap.
#pragma unroll 2
      for (int pg = 0; pg < 8; ++pg) {
        const int r = 2 * pg + prow;
        s16x8 af[NTW], bf[MAXT];
        const T* da = sD + (r * 16 + pcol) * DST + 4 * pp;
#pragma unroll
        for (int j = 0; j < NTW; ++j) {
          const int jc = 16 * dch(pcol, j);
          const s16x4 lo = lds_tr16(da + jc), hi = lds_tr16(da + HI * DST + jc);
          af[j] = s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        }
        const T* pr = sP + (r * PW + pcol) * PST + 4 * pp;
#pragma unroll
        for (int tt = 0; tt < MAXT; ++tt) {
          const s16x4 lo = lds_tr16(pr + toff[tt]), hi = lds_tr16(pr + toff[tt] + HI * PST);
          bf[tt] = s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        }
#pragma unroll
        for (int tt = 0; tt < MAXT; ++tt)
#pragma unroll
          for (int j = 0; j < NTW; ++j) acc[tt][j] = mfma_s16<T>(af[j], bf[tt], acc[tt][j]);
        if (do_bias) {
#pragma unroll
          for (int j = 0; j < NTW; ++j) bacc[j] = mfma_s16<T>(af[j], ones, bacc[j]);
        }
      }
    }
  }
  // ---- partial sums: D[co][n], lane column n = lane & 15, rows co = 4 (lane >> 4) + r ----
  const long long z = blockIdx.x;
  if constexpr (C1) {
    // waves 2, 3 hand their sums to waves 0, 1 (same k-block): fixed-order pair sums
    float* red = reinterpret_cast<float*>(sD);
    lds_sync();
    if (wave >= 2) {
#pragma unroll
      for (int j = 0; j < NTW; ++j)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) red[(((wave - 2) * NTW + j) * 4 + rr) * 64 + lane] = acc[0][j][rr];
    }
    lds_sync();
    if (wave < 2) {
      const int t = 16 * wave + (lane & 15);
#pragma unroll
      for (int j = 0; j < NTW; ++j)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const float v = acc[0][j][rr] + red[((wave * NTW + j) * 4 + rr) * 64 + lane];
          const int co = co0 + 16 * j + 4 * (lane >> 4) + rr;
          if (co >= g.CO) continue;
          if (t < ntap) a.part[(z * g.CO + co) * g.Kf + wcol(g, t, 0)] = v;
          else if (t == 31 && a.bpart) a.bpart[((long long)ph * a.Z + z) * g.CO + co] = v;
        }
    }
    return;
  }
  const int ci = c0 + (lane & 15);
#pragma unroll
  for (int tt = 0; tt < MAXT; ++tt) {
    const int t = tb + wave + 4 * tt;
    if (t >= ntap) break;
    const int col = wcol(g, t, ci);
#pragma unroll
    for (int j = 0; j < NTW; ++j)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int co = co0 + 16 * j + 4 * (lane >> 4) + rr;
        if (co < g.CO) a.part[(z * g.CO + co) * g.Kf + col] = acc[tt][j][rr];
      }
  }
  if (do_bias && (lane & 15) == 0) {
#pragma unroll
    for (int j = 0; j < NTW; ++j)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int co = co0 + 16 * j + 4 * (lane >> 4) + rr;
        if (co < g.CO) a.bpart[((long long)ph * a.Z + z) * g.CO + co] = bacc[j][rr];
      }
  }
}

// Conv2DTranspose stride 2 (four output phases (oy0, ox0) = (p >> 1, p & 1) over one tile
// grid): a workgroup owns a 16 x 16 phase tile of ALL four phases, i.e. the 32 x 32 dOut
// region, staged de-interleaved per phase ([phase][256 pixels][16 co], the wgrad_tr_kernel
// layout), and ONE union input patch serves every phase's taps. The (phase, tap) blocks
// (25 for a 5 x 5 kernel) are split into contiguous runs of <= 7 per wave, so a wave reloads
// its dOut fragment only when the run crosses into the next phase; wave w also owns the
// bias gradient of phase w (bpart[w][z]). Same fixed-order partial sums as wgrad_tr_kernel.
template <typename T>
__global__ __launch_bounds__(256) void wgrad_trp_kernel(WgradTrArgs a) {
  constexpr int CH = 16, COT = 16, DST = COT + 8, PST = CH + 8, MAXT = 7;
  __shared__ __attribute__((aligned(16))) T sD[4 * 256 * DST];
  __shared__ __attribute__((aligned(16))) T sP[400 * PST];
  const Geo& g0 = a.g[0];
  const int chunk = blockIdx.y / a.ncog, cog = blockIdx.y - (blockIdx.y / a.ncog) * a.ncog;
  const int c0 = chunk * CH, co0 = cog * COT;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ntx = (g0.OW + 15) / 16, nty = (g0.OH + 15) / 16;
  const long long ntiles = (long long)g0.N * nty * ntx;
  const long long t_begin = blockIdx.x * ntiles / a.Z, t_end = (blockIdx.x + 1) * ntiles / a.Z;
  const int PW = a.PW, PH = a.PH;
  const T* __restrict__ in = reinterpret_cast<const T*>(a.in);
  const T* __restrict__ dout = reinterpret_cast<const T*>(a.dout);
  const int CO = g0.CO, OHs = g0.OHs, OWs = g0.OWs;

  // this wave's run of (phase, tap) blocks: u in [ub, ue) over the phases' taps in order;
  // blocks past the run repeat its last block (their MFMAs run, their sums are never
  // stored). A run spans at most two phases (host-checked, wgrad_trp_runs_ok): blocks
  // tt < split use phase pa's dOut fragment, the others phase pb's.
  int U = 0;
#pragma unroll
  for (int p = 0; p < 4; ++p) U += a.g[p].KH * a.g[p].KW;
  const int ub = wave * U / 4, ue = (wave + 1) * U / 4;
  int boff[MAXT], tph[MAXT], ttap[MAXT];
#pragma unroll
  for (int tt = 0; tt < MAXT; ++tt) {
    int u = min(ub + tt, ue - 1), p = 0;
    while (p < 3 && u >= a.g[p].KH * a.g[p].KW) { u -= a.g[p].KH * a.g[p].KW; ++p; }
    const Geo& g = a.g[p];
    const int jy = u / max(g.KW, 1), jx = u - (u / max(g.KW, 1)) * g.KW;
    tph[tt] = p;
    ttap[tt] = u;
    boff[tt] = ((a.upt - g.pad_t + jy) * PW + a.upl - g.pad_l + jx) * PST;
  }
  const int pa = tph[0], pb = tph[MAXT - 1];
  int split = MAXT;
#pragma unroll
  for (int tt = MAXT - 1; tt >= 1; --tt)
    if (tph[tt] != pa) split = tt;
  const int aoffa = pa * 256 * DST, aoffb = pb * 256 * DST;

  f32x4 acc[MAXT];
#pragma unroll
  for (int t = 0; t < MAXT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 bacc = f32x4{0.f, 0.f, 0.f, 0.f};
  const bool do_bias = a.bpart && chunk == 0;
  s16x8 ones;
  const short one = __builtin_bit_cast(short, from_f<T>(1.f));
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = one;
  const int g4 = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  const int prow = g4 >> 1, pcol = 8 * (g4 & 1) + q;

  uint4 rd[8];  // 32 x 32 dOut pixels x 16 co: 2048 uint4
  uint4 rp[4];  // <= 20 x 20 patch pixels x 16 ci: 800 uint4
  auto tile_org = [&](long long tile, int& n, int& oyt, int& oxt) {
    // 32-bit unsigned divisions (the host keeps N x tiles below 2^31): the 64-bit divide
    // routine had cost ~200 SALU per tile
    const unsigned tu = (unsigned)tile, per = (unsigned)(nty * ntx);
    n = (int)(tu / per);
    const unsigned trem = tu - (unsigned)n * per;
    oyt = (int)(trem / (unsigned)ntx) * 16;
    oxt = (int)(trem - (trem / (unsigned)ntx) * (unsigned)ntx) * 16;
  };
  auto fetch = [&](long long tile) {
    int n, oyt, oxt;
    tile_org(tile, n, oyt, oxt);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = tid + 256 * u;
      const int pix = e >> 1, v = e & 1;
      const int y = 2 * oyt + (pix >> 5), x = 2 * oxt + (pix & 31);
      rd[u] = uint4{0u, 0u, 0u, 0u};
      if (y < OHs && x < OWs)
        rd[u] = *reinterpret_cast<const uint4*>(dout + (((long long)n * OHs + y) * OWs + x) * CO + co0 + 8 * v);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = tid + 256 * u;
      const int pix = e >> 1, v = e & 1;
      const int py = pix / PW, px = pix - (pix / PW) * PW;
      const int iy = oyt - a.upt + py, ix = oxt - a.upl + px;
      rp[u] = uint4{0u, 0u, 0u, 0u};
      if (pix < PH * PW && (unsigned)iy < (unsigned)g0.IH && (unsigned)ix < (unsigned)g0.IW)
        rp[u] = *reinterpret_cast<const uint4*>(in + (((long long)n * g0.IH + iy) * g0.IW + ix) * g0.C + c0 + 8 * v);
    }
  };
  auto stage = [&]() {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = tid + 256 * u;
      const int pix = e >> 1, v = e & 1;
      const int y = pix >> 5, x = pix & 31;
      const int p = 2 * (y & 1) + (x & 1);
      *reinterpret_cast<uint4*>(sD + (p * 256 + (y >> 1) * 16 + (x >> 1)) * DST + 8 * v) = rd[u];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = tid + 256 * u;
      const int pix = e >> 1, v = e & 1;
      if (pix < PH * PW) *reinterpret_cast<uint4*>(sP + pix * PST + 8 * v) = rp[u];
    }
  };
  auto afrag = [&](const T* da) {
    const s16x4 lo = lds_tr16(da), hi = lds_tr16(da + 4 * DST);
    return s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  };

  if (t_begin < t_end) fetch(t_begin);
  for (long long tile = t_begin; tile < t_end; ++tile) {
    lds_sync();
    stage();
    lds_sync();
    if (tile + 1 < t_end) fetch(tile + 1);
    // per pixel group: both dOut fragments and every B fragment read before the MFMAs, which
    // then run back to back (round 4 waited lgkmcnt(0) before each one and branched around
    // the run's end and phase changes, moving accumulators through VGPRs)
#pragma unroll 2
    for (int pg = 0; pg < 8; ++pg) {
      const int r = 2 * pg + prow;
      const int pix = r * 16 + pcol, ppix = r * PW + pcol;
      const s16x8 a0 = afrag(sD + aoffa + pix * DST + 4 * pp);
      const s16x8 a1 = afrag(sD + aoffb + pix * DST + 4 * pp);
      s16x8 bf[MAXT];
#pragma unroll
      for (int tt = 0; tt < MAXT; ++tt) {
        const T* pb_ = sP + ppix * PST + boff[tt] + 4 * pp;
        const s16x4 lo = lds_tr16(pb_), hi = lds_tr16(pb_ + 4 * PST);
        bf[tt] = s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int tt = 0; tt < MAXT; ++tt) acc[tt] = mfma_s16<T>(tt < split ? a0 : a1, bf[tt], acc[tt]);
      if (do_bias) bacc = mfma_s16<T>(afrag(sD + wave * 256 * DST + pix * DST + 4 * pp), ones, bacc);
    }
  }
  const long long z = blockIdx.x;
  const int ci = c0 + (lane & 15);
#pragma unroll
  for (int tt = 0; tt < MAXT; ++tt) {
    if (ub + tt >= ue) break;
    const int col = wcol(a.g[tph[tt]], ttap[tt], ci);
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int co = co0 + 4 * (lane >> 4) + rr;
      if (co < CO) a.part[(z * CO + co) * g0.Kf + col] = acc[tt][rr];
    }
  }
  if (do_bias && (lane & 15) == 0) {
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int co = co0 + 4 * (lane >> 4) + rr;
      if (co < CO) a.bpart[((long long)wave * a.Z + z) * CO + co] = bacc[rr];
    }
  }
}

// One output channel, 16 input channels (the last Conv2D, VAE/manual_scan_3layers.py:199):
//   dW[jy][jx][ci] = sum_p dOut[p] in[p + (jy, jx) - pad][ci]
//                  = sum_q in[q + (jy, 0) - pad][ci] * dOut[q - (0, jx)]       (q = p + (0, jx))
// so with the pixels q of a tile (16 rows x 24 columns) as the MFMA reduction, A = the input
// patch shifted by jy (rows = ci, ds_read_b64_tr_b16 from [pixel][ci] rows) and B = dOut
// shifted by jx (columns = jx): one MFMA per (32 pixels, jy) yields all KW taps of a kernel
// row, 5x fewer MFMAs than one per tap with 15 of 16 rows idle. The KW shifted copies of
// the 16 x 16 dOut tile live in LDS with their zero margins written once. A workgroup is
// ONE wave over a run of tiles (no barriers beyond the wave's own LDS ordering), the next
// tile prefetched in registers; the bias gradient is the lanes' fp32 sums of dOut, reduced
// in a fixed order. Partial sums per run go to part[z] / bpart[z] (ordered_sum_kernel).
template <typename T>
__global__ __launch_bounds__(64) void wgrad_co1_kernel(WgradTrArgs a) {
  constexpr int QC = 24;       // q columns per tile row (16 + KW - 1 <= 20, 3 groups of 8)
  constexpr int PSTC = 24;     // patch pixel stride (16 ci + 8: tr reads 2-way at most)
  constexpr int PR = 20;       // patch rows (16 + KH - 1, KH <= 5)
  constexpr int NPV = (PR * QC * 2 + 63) / 64;  // patch uint4 per lane (15)
  __shared__ __attribute__((aligned(16))) T sP[PR * QC * PSTC];
  __shared__ __attribute__((aligned(16))) T sB[5 * 16 * QC];
  const Geo& g = a.g[0];
  const int lane = threadIdx.x;
  const int KH = g.KH, KW = g.KW;
  const int ntx = (g.OW + 15) / 16, nty = (g.OH + 15) / 16;
  const long long ntiles = (long long)g.N * nty * ntx;
  const long long t_begin = blockIdx.x * ntiles / a.Z, t_end = (blockIdx.x + 1) * ntiles / a.Z;
  const T* __restrict__ in = reinterpret_cast<const T*>(a.in);
  const T* __restrict__ dout = reinterpret_cast<const T*>(a.dout);

  // zero margins of the shifted dOut copies (columns outside [s, s + 16) stay zero)
  for (int e = lane; e < 5 * 16 * QC / 8; e += 64)
    reinterpret_cast<uint4*>(sB)[e] = uint4{0u, 0u, 0u, 0u};

  f32x4 acc[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bsum = 0.f;

  const int g4 = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3, n16 = lane & 15;
  const int sft = min(n16, KW - 1);  // B column jx (columns >= KW are never stored)

  uint4 rp[NPV];
  uint2 rd;
  auto tile_org = [&](long long tile, int& n, int& oyt, int& oxt) {
    // 32-bit unsigned divisions (the host keeps N x tiles below 2^31): the 64-bit divide
    // routine had cost ~200 SALU per tile
    const unsigned tu = (unsigned)tile, per = (unsigned)(nty * ntx);
    n = (int)(tu / per);
    const unsigned trem = tu - (unsigned)n * per;
    oyt = (int)(trem / (unsigned)ntx) * 16;
    oxt = (int)(trem - (trem / (unsigned)ntx) * (unsigned)ntx) * 16;
  };
  auto fetch = [&](long long tile) {
    int n, oyt, oxt;
    tile_org(tile, n, oyt, oxt);
    {  // dOut: lane = (row lane >> 2, columns 4 (lane & 3) .. + 3)
      const int oy = oyt + (lane >> 2), ox = oxt + 4 * (lane & 3);
      const bool full = oy < g.OH && ox + 3 < g.OW && (g.OW & 3) == 0;
      const long long o = ((long long)n * g.OH + min(oy, g.OH - 1)) * g.OW;
      if (full) {
        rd = *reinterpret_cast<const uint2*>(dout + o + ox);
      } else {
        uint32_t w[2] = {0u, 0u};
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (oy < g.OH && ox + k < g.OW)
            w[k >> 1] |= (uint32_t)__builtin_bit_cast(unsigned short, dout[o + ox + k]) << (16 * (k & 1));
        rd = uint2{w[0], w[1]};
      }
    }
#pragma unroll
    for (int u = 0; u < NPV; ++u) {
      const int e = min(lane + 64 * u, PR * QC * 2 - 1);
      const int pix = e >> 1, v = e & 1;
      const int py = pix / QC, px = pix - (pix / QC) * QC;
      const int iy = oyt - g.pad_t + py, ix = oxt - g.pad_l + px;
      const bool ok = (unsigned)iy < (unsigned)g.IH && (unsigned)ix < (unsigned)g.IW;
      rp[u] = *reinterpret_cast<const uint4*>(in + (ok ? (((long long)n * g.IH + iy) * g.IW + ix) * 16 : 0) + 8 * v);
      if (!ok) rp[u] = uint4{0u, 0u, 0u, 0u};
    }
  };

  if (t_begin < t_end) fetch(t_begin);
  for (long long tile = t_begin; tile < t_end; ++tile) {
    lds_sync();  // the previous tile's fragment reads are done
#pragma unroll
    for (int u = 0; u < NPV; ++u) {
      const int e = lane + 64 * u;
      if (e < PR * QC * 2) *reinterpret_cast<uint4*>(sP + (e >> 1) * PSTC + 8 * (e & 1)) = rp[u];
    }
    {
      const int row = lane >> 2, c0 = 4 * (lane & 3);
      const uint32_t w[2] = {rd.x, rd.y};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const unsigned short b = (unsigned short)(w[k >> 1] >> (16 * (k & 1)));
        bsum += to_f(__builtin_bit_cast(T, b));
        for (int s = 0; s < KW; ++s) sB[(s * 16 + row) * QC + c0 + k + s] = __builtin_bit_cast(T, b);
      }
    }
    lds_sync();
    if (tile + 1 < t_end) fetch(tile + 1);
    // 12 chunks of 32 pixels: lane group g4 takes the 8-column run (row, cg) = pair 4 c + g4
#pragma unroll 2
    for (int c = 0; c < 12; ++c) {
      const int idx = 4 * c + g4, row = idx / 3, cg = idx - (idx / 3) * 3;
      const uint4 bq = *reinterpret_cast<const uint4*>(sB + (sft * 16 + row) * QC + 8 * cg);
      const s16x8 bf = __builtin_bit_cast(s16x8, bq);
#pragma unroll
      for (int jy = 0; jy < 5; ++jy) {
        if (jy >= KH) break;  // uniform
        const T* pa = sP + ((row + jy) * QC + 8 * cg + q) * PSTC + 4 * pp;
        const s16x4 lo = lds_tr16(pa), hi = lds_tr16(pa + 4 * PSTC);
        const s16x8 af = s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        acc[jy] = mfma_s16<T>(af, bf, acc[jy]);
      }
    }
  }
  // D[m = ci][n = jx]: lane holds ci = 4 (lane >> 4) + r, jx = lane & 15
  const long long z = blockIdx.x;
  if (n16 < KW) {
#pragma unroll
    for (int jy = 0; jy < 5; ++jy) {
      if (jy >= KH) break;
#pragma unroll
      for (int r = 0; r < 4; ++r)
        a.part[z * g.Kf + (jy * KW + n16) * 16 + 4 * g4 + r] = acc[jy][r];
    }
  }
  if (a.bpart) {
    // fixed-order tree over the 64 lanes
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) bsum += __shfl_down(bsum, off);
    if (lane == 0) a.bpart[z] = bsum;
  }
}

// dst[e] += sum_{z < nz} part[z * n + e], always in the same order (bit-reproducible). One
// launch carries two such sums (the weight and the bias gradient): blocks [0, nb0) do job 0.
// A 1024-thread workgroup owns 64 consecutive e (a wave's loads are one 256-byte run) and 16
// z-lanes (its waves); lane zl sums z = zl, zl + 16, ... in order with 8 loads in flight, then
// the 16 lane sums meet in a fixed pairwise tree. (Round 4 gave a workgroup 16 e x 16 z-lanes:
// 64-byte runs per wave load and up to 16 serial round trips per lane, 8.7 us per launch.)
struct SumJob {
  const float* part;
  float* dst;
  long long n;
  int nz, ew;
  int overwrite;  // dst = sum instead of dst += sum
};

constexpr int SUM_EW = 64, SUM_ZL = 16;

__global__ __launch_bounds__(SUM_EW * SUM_ZL) void ordered_sum_kernel(SumJob j0, SumJob j1,
                                                                      unsigned nb0) {
  __shared__ float red[SUM_EW * SUM_ZL];
  const bool second = blockIdx.x >= nb0;
  const SumJob j = second ? j1 : j0;
  const long long blk = second ? blockIdx.x - nb0 : blockIdx.x;
  const int el = threadIdx.x & (SUM_EW - 1), zl = threadIdx.x / SUM_EW;
  const long long e = blk * SUM_EW + el;
  float t = 0.f;
  if (e < j.n) {
    const float* p = j.part + e;
    int z = zl;
    for (; z + 7 * SUM_ZL < j.nz; z += 8 * SUM_ZL) {
      float v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = p[(long long)(z + k * SUM_ZL) * j.n];
#pragma unroll
      for (int k = 0; k < 8; ++k) t += v[k];
    }
    for (; z < j.nz; z += SUM_ZL) t += p[(long long)z * j.n];
  }
  red[threadIdx.x] = t;
  __syncthreads();
  for (int w = SUM_ZL / 2; w >= 1; w >>= 1) {
    if (zl < w) red[threadIdx.x] += red[threadIdx.x + w * SUM_EW];
    __syncthreads();
  }
  if (zl == 0 && e < j.n) j.dst[e] = j.overwrite ? red[threadIdx.x] : j.dst[e] + red[threadIdx.x];
}

// the sums of one weight-gradient launch: dw over nz slices, db (if any) over nzb slices
inline SumJob sum_job(const float* part, int nz, long long n, float* dst, bool overwrite) {
  return SumJob{part, dst, n, nz, SUM_EW, overwrite ? 1 : 0};
}
inline unsigned sum_blocks(const SumJob& j) { return (unsigned)((j.n + SUM_EW - 1) / SUM_EW); }
inline void launch_ordered_sums(const float* part, int nz, long long n, float* dw, const float* bpart,
                                int nzb, long long nb, float* db, hipStream_t st,
                                bool overwrite = false) {
  const SumJob j0 = sum_job(part, nz, n, dw, overwrite);
  SumJob j1{};
  unsigned blocks = sum_blocks(j0);
  if (db) {
    j1 = sum_job(bpart, nzb, nb, db, overwrite);
    blocks += sum_blocks(j1);
  }
  SPECENH_LAUNCH(ordered_sum_kernel, dim3(blocks), dim3(SUM_EW * SUM_ZL), 0, st, j0, j1,
                 sum_blocks(j0));
}

// ------------------------------------------------------------------ elementwise
template <typename T>
__global__ void maxpool2_fwd_kernel(const T* __restrict__ in, int N, int H, int W, int C,
                                    T* __restrict__ out, unsigned char* __restrict__ am) {
  const long long total = (long long)N * (H / 2) * (W / 2) * C;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    long long r = i / C;
    const int x = (int)(r % (W / 2));
    r /= (W / 2);
    const int y = (int)(r % (H / 2));
    const int n = (int)(r / (H / 2));
    const T* p = in + (((long long)n * H + 2 * y) * W + 2 * x) * C + c;
    float best = to_f(p[0]);
    int arg = 0;
    const float v1 = to_f(p[C]), v2 = to_f(p[(long long)W * C]), v3 = to_f(p[(long long)W * C + C]);
    if (v1 > best) { best = v1; arg = 1; }
    if (v2 > best) { best = v2; arg = 2; }
    if (v3 > best) { best = v3; arg = 3; }
    out[i] = from_f<T>(best);
    if (am) am[i] = (unsigned char)arg;
  }
}

// dIn = dOut routed to the argmax, times (pooled > 0) — the ReLU mask of the pool's input
// at its argmax; dIn fully written.
template <typename T>
__global__ void maxpool2_bwd_kernel(const T* __restrict__ dout, const unsigned char* __restrict__ am,
                                    const T* __restrict__ pooled, int N, int H, int W, int C,
                                    T* __restrict__ din) {
  const long long total = (long long)N * (H / 2) * (W / 2) * C;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    long long r = i / C;
    const int x = (int)(r % (W / 2));
    r /= (W / 2);
    const int y = (int)(r % (H / 2));
    const int n = (int)(r / (H / 2));
    const float gv = (!pooled || to_f(pooled[i]) > 0.f) ? to_f(dout[i]) : 0.f;
    const int arg = am[i];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const long long o = (((long long)n * H + 2 * y + (q >> 1)) * W + 2 * x + (q & 1)) * C + c;
      din[o] = from_f<T>(q == arg ? gv : 0.f);
    }
  }
}

// 16-bit, C % 8 == 0: one thread per (pooled pixel, 8 channels): 16-byte loads of dout and
// the pooled values (ReLU mask), 8 argmax bytes, four 16-byte stores; 32-bit indexing
// (check_sizes bounds every tensor below 2^31 elements)
template <typename T>
__global__ __launch_bounds__(256) void maxpool2_bwd_vec_kernel(const T* __restrict__ dout,
                                                               const unsigned char* __restrict__ am,
                                                               const T* __restrict__ pooled, int N,
                                                               int H, int W, int C,
                                                               T* __restrict__ din) {
  const int C8 = C >> 3, PW = W >> 1, PH = H >> 1;
  const int i = blockIdx.x * 256 + threadIdx.x;  // (n, y, x, c8)
  if (i >= N * PH * PW * C8) return;
  const int c8 = i % C8, r = i / C8;
  const int x = r % PW, r2 = r / PW;
  const int y = r2 % PH, n = r2 / PH;
  const int e = r * C + 8 * c8;  // pooled element index
  const uint4 g = *reinterpret_cast<const uint4*>(dout + e);
  const uint2 a2 = *reinterpret_cast<const uint2*>(am + e);
  uint32_t gw[4] = {g.x, g.y, g.z, g.w};
  if (pooled) {
    const uint4 pv = *reinterpret_cast<const uint4*>(pooled + e);
    const uint32_t pw[4] = {pv.x, pv.y, pv.z, pv.w};
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float m = to_f(__builtin_bit_cast(T, (unsigned short)(pw[k >> 1] >> (16 * (k & 1)))));
      if (!(m > 0.f)) gw[k >> 1] &= 0xffff0000u >> (16 * (k & 1));
    }
  }
  const uint32_t aw[2] = {a2.x, a2.y};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint32_t o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      // channels 2k, 2k+1: keep the gradient half whose argmax is q
      const uint32_t b0 = (aw[(2 * k) >> 2] >> (8 * ((2 * k) & 3))) & 0xffu;
      const uint32_t b1 = (aw[(2 * k + 1) >> 2] >> (8 * ((2 * k + 1) & 3))) & 0xffu;
      o[k] = gw[k] & ((b0 == (uint32_t)q ? 0x0000ffffu : 0u) | (b1 == (uint32_t)q ? 0xffff0000u : 0u));
    }
    const int oo = ((n * H + 2 * y + (q >> 1)) * W + 2 * x + (q & 1)) * C + 8 * c8;
    *reinterpret_cast<uint4*>(din + oo) = uint4{o[0], o[1], o[2], o[3]};
  }
}

// Keras BCE after a sigmoid (graph mode): sigmoid_cross_entropy_with_logits; the grad of
// the mean is (sigmoid(z) - t) / n. One fp64 atomic per workgroup.
template <typename TT, typename TG>
__global__ __launch_bounds__(256) void bce_logits_kernel(const float* __restrict__ z,
                                                          const TT* __restrict__ t, long long n,
                                                          TG* __restrict__ grad,
                                                          double* __restrict__ loss) {
  __shared__ double red[4];
  double acc = 0.0;
  const float inv = 1.0f / (float)n;
  // BCE_U elements per thread per pass with all their loads issued first (a grid-stride loop
  // of one element waited a full round trip per element: 22 us at C4's 2 M elements).
  // log1p(e) for e = exp(-|z|) in (0, 1] by Goldberg's form u = 1 + e, log(u) e / (u - 1)
  // (e when u rounds to 1), the sigmoid by the hardware reciprocal: the library log1pf and
  // IEEE division were ~190 instructions per element (round 4: 21 us per C4 step).
  // The grid is at most 256 workgroups: each ends in one device-scope fp64 atomic on the
  // same word and those serialise at the memory side (~18 ns each, measured: 1024 of them
  // were 19 us).
  constexpr int BCE_U = 16;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i0 = blockIdx.x * (long long)blockDim.x + threadIdx.x; i0 < n;
       i0 += BCE_U * stride) {
    float zv[BCE_U], tv[BCE_U];
    // unconditional loads from clamped indices (a guarded load is a branch per element, and
    // the loads then went out one at a time); out-of-range values are masked below
#pragma unroll
    for (int u = 0; u < BCE_U; ++u) {
      const long long i = i0 + u * stride;
      const long long ic = i < n ? i : n - 1;
      zv[u] = z[ic];
      tv[u] = to_f(t[ic]);
    }
    float part = 0.f;
#pragma unroll
    for (int u = 0; u < BCE_U; ++u) {
      const long long i = i0 + u * stride;
      const float zi = zv[u], ti = tv[u];
      const float e = __expf(-fabsf(zi));
      const float w = 1.f + e;
      const float l1p = w == 1.f ? e : __logf(w) * (e * __builtin_amdgcn_rcpf(w - 1.f));
      const float li = fmaxf(zi, 0.f) - zi * ti + l1p;
      part += i < n ? li : 0.f;
      // sigmoid(z) = 1 / (1 + exp(-z)): exp(-z) = e for z >= 0, 1 / e otherwise
      const float sg = zi >= 0.f ? __builtin_amdgcn_rcpf(w) : e * __builtin_amdgcn_rcpf(w);
      if (grad && i < n) grad[i] = from_f<TG>((sg - ti) * inv);
    }
    acc += (double)part;
  }
  for (int m = 32; m >= 1; m >>= 1) acc += __shfl_xor(acc, m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0 && loss) atomicAdd(loss, (red[0] + red[1]) + (red[2] + red[3]));
}

template <typename T>
__global__ void adam_kernel(float* __restrict__ w, const float* __restrict__ g, float* __restrict__ m,
                            float* __restrict__ v, long long n, float lr_t, float b1, float b2,
                            float eps, float gscale, T* __restrict__ w_lowp) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const float gi = g[i] * gscale;
    const float mi = b1 * m[i] + (1.f - b1) * gi;
    const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    const float wi = w[i] - lr_t * mi / (sqrtf(vi) + eps);
    w[i] = wi;
    if (w_lowp) w_lowp[i] = from_f<T>(wi);
  }
}

// Adam (as adam_kernel) with the input-gradient GEMM weights of up to 8 layers written from
// the updated weights in the same pass: element i of segment s (w[off .. off + k k ci co) =
// bt[co][ky][kx][ci]) also goes to bd[ci][k-1-ky][k-1-kx][co] (flip_transpose_kernel's map),
// as T — the value w_lowp receives, or fp32 for fp32 training. Replaces the per-layer
// flip_transpose launches that followed every optimizer step.
struct FlipSegs {
  long long off[8];
  int k[8], ci[8], co[8];
  void* dst[8];
  int n;
};

template <typename T, bool LOWP>
__global__ void adam_flip_kernel(float* __restrict__ w, const float* __restrict__ g,
                                 float* __restrict__ m, float* __restrict__ v, long long n,
                                 float lr_t, float b1, float b2, float eps, float gscale,
                                 T* __restrict__ w_lowp, FlipSegs fs) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const float gi = g[i] * gscale;
    const float mi = b1 * m[i] + (1.f - b1) * gi;
    const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    const float wi = w[i] - lr_t * mi / (sqrtf(vi) + eps);
    w[i] = wi;
    const T wt = from_f<T>(wi);
    if (LOWP) w_lowp[i] = wt;
    for (int s = 0; s < fs.n; ++s) {
      const int k = fs.k[s], CI = fs.ci[s], CO = fs.co[s];
      const long long r = i - fs.off[s];
      if (r < 0 || r >= (long long)k * k * CI * CO) continue;
      const int ci = (int)(r % CI);
      long long t = r / CI;
      const int kx = (int)(t % k);
      t /= k;
      const int ky = (int)(t % k);
      const int co = (int)(t / k);
      reinterpret_cast<T*>(fs.dst[s])[(((long long)ci * k + (k - 1 - ky)) * k + (k - 1 - kx)) * CO + co] = wt;
    }
  }
}

// bd[ci][a][b][co] = bt[co][k-1-a][k-1-b][ci]
template <typename T>
__global__ void flip_transpose_kernel(const T* __restrict__ bt, int k, int CI, int CO,
                                      T* __restrict__ bd) {
  const long long total = (long long)k * k * CI * CO;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int co = (int)(i % CO);
    long long r = i / CO;
    const int b = (int)(r % k);
    r /= k;
    const int aa = (int)(r % k);
    const int ci = (int)(r / k);
    bd[i] = bt[(((long long)co * k + (k - 1 - aa)) * k + (k - 1 - b)) * CI + ci];
  }
}

template <typename TS, typename TD>
__global__ void cast_kernel(const TS* __restrict__ s, TD* __restrict__ d, long long n) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x)
    d[i] = from_f<TD>(to_f(s[i]));
}

inline unsigned grid1d(long long n) {
  return (unsigned)std::max<long long>(1, std::min<long long>((n + 255) / 256, 65536));
}

// ------------------------------------------------------------------ host planning
// Split a conv over an in_dil-dilated input (stride 1) into in_dil^2 dense output phases.
int plan_phases(int N, int IH, int IW, int C, int CO, int KH, int KW, int stride, int pad_t,
                int pad_l, int in_dil, int OH, int OW, Geo* g, int* nph) {
  const int Kf = KH * KW * C;
  if (in_dil == 1) {
    g[0] = Geo{N, IH, IW, C, OH, OW, CO, KH, KW, stride, pad_t, pad_l,
               0, 0, 1, KW, Kf, 1, 0, 1, 0, OH, OW};
    *nph = 1;
    return SPECENH_OK;
  }
  if (in_dil != 2 || stride != 1)
    return set_error(SPECENH_EUNSUPPORTED, "dilated input supports in_dil 2 with stride 1");
  const int d = in_dil;
  int n = 0;
  for (int py = 0; py < d; ++py) {
    for (int px = 0; px < d; ++px) {
      const int OHq = OH > py ? (OH - py + d - 1) / d : 0;
      const int OWq = OW > px ? (OW - px + d - 1) / d : 0;
      if (OHq == 0 || OWq == 0) continue;
      const int ky0 = ((pad_t - py) % d + d) % d, kx0 = ((pad_l - px) % d + d) % d;
      const int ny = ky0 < KH ? (KH - ky0 + d - 1) / d : 0;
      const int nx = kx0 < KW ? (KW - kx0 + d - 1) / d : 0;
      const int offy = (py - pad_t + ky0) / d, offx = (px - pad_l + kx0) / d;  // exact
      g[n++] = Geo{N, IH, IW, C, OHq, OWq, CO, ny, nx, 1, -offy, -offx,
                   ky0, kx0, d, KW, Kf, d, py, d, px, OH, OW};
    }
  }
  *nph = n;
  return SPECENH_OK;
}

int check_sizes(long long N, long long IH, long long IW, long long C, long long OH, long long OW,
                long long CO) {
  if (N <= 0 || IH <= 0 || IW <= 0 || C <= 0 || OH <= 0 || OW <= 0 || CO <= 0)
    return set_error(SPECENH_EINVAL, "bad convolution geometry");
  if (N * IH * IW * C >= (1LL << 31) || N * OH * OW * CO >= (1LL << 31))
    return set_error(SPECENH_EUNSUPPORTED, "tensor too large for one launch (split the batch)");
  return SPECENH_OK;
}

// dynamic LDS of conv_patch_kernel<T, NT, CC, *, PAIR>: the staged patch (largest phase, or
// the shared patch of all phases) and, for PAIR, the output stage it aliases
template <typename T, int CC>
size_t patch_lds_bytes(const ConvArgs& a, int nph, int NT, bool pair) {
  size_t px = 0;
  if (a.ph_shared) {
    px = (size_t)a.PH * a.PW;
  } else {
    for (int i = 0; i < nph; ++i)
      px = std::max(px, (size_t)(16 + a.g[i].KH - 1) * (16 + a.g[i].KW - 1));
  }
  size_t elems = px * Patch<CC>::PST;
  if (pair) elems = std::max(elems, (size_t)16 * 16 * (32 * NT + 8));
  return (elems * sizeof(T) + 15) / 16 * 16;
}

// output-channel blocks of 16 per workgroup: all of them (up to 4) unless that leaves fewer
// than 2 workgroups per CU (a small batch at 16 x 16 output: 128 tiles), then narrower
// blocks over more workgroups (each re-stages the patch, an L2 hit)
inline int patch_nt(int CO, unsigned tiles) {
  int nt = std::min(4, (CO + 15) / 16);
  const unsigned long long want = (unsigned long long)std::max(1, variant(V_PATCH_MIN_WG));
  while (nt > 1 && (unsigned long long)tiles * ((CO + 16 * nt - 1) / (16 * nt)) < want) nt = (nt + 1) / 2;
  return nt;
}

template <typename T, int CC, bool RT = false>
int launch_patch(ConvArgs a, int nph, hipStream_t st) {
  // all phases of a dilated conv in one workgroup when they share a tile grid and the
  // input fits one channel chunk: one staged patch serves every phase, and the phases'
  // interleaved output lines are completed by the same workgroup
  a.ph_shared = 0;
  const int nchunk = CC == 1 ? 1 : a.g[0].C / CC;
  if (nph > 1 && nchunk == 1) {
    bool same = true;
    int upt = -1 << 20, upl = -1 << 20, lo_y = 1 << 20, hi_y = -(1 << 20), lo_x = 1 << 20,
        hi_x = -(1 << 20);
    for (int i = 0; i < nph; ++i) {
      const Geo& g = a.g[i];
      same = same && g.OH == a.g[0].OH && g.OW == a.g[0].OW;
      upt = std::max(upt, g.pad_t);
      upl = std::max(upl, g.pad_l);
      lo_y = std::min(lo_y, -g.pad_t);
      hi_y = std::max(hi_y, 15 - g.pad_t + g.KH - 1);
      lo_x = std::min(lo_x, -g.pad_l);
      hi_x = std::max(hi_x, 15 - g.pad_l + g.KW - 1);
    }
    if (same && hi_y - lo_y + 1 <= 20 && hi_x - lo_x + 1 <= 20) {
      a.ph_shared = 1;
      a.upt = upt;
      a.upl = upl;
      a.PH = hi_y - lo_y + 1;
      a.PW = hi_x - lo_x + 1;
    }
  }
  unsigned tiles = 0;
  for (int i = 0; i < nph; ++i)
    tiles = std::max(tiles, (unsigned)(a.g[i].N * ((a.g[i].OH + 15) / 16) * ((a.g[i].OW + 15) / 16)));
  const int CO = a.g[0].CO;
  const int nt = patch_nt(CO, tiles);
  // Conv2DTranspose stride 2: (tile, row phase) workgroups with whole-row stores
  bool pair = a.ph_shared && nph == 4 && !a.pool && !a.mask && !a.logits && !a.out_f32 &&
              CO == 16 * nt && (variant(V_CONVT_PAIR) != 0);
  for (int i = 0; pair && i < nph; ++i) {
    const Geo& g = a.g[i];
    pair = g.oys == 2 && g.oxs == 2 && g.oy0 == i / 2 && g.ox0 == i % 2 && g.OHs == 2 * g.OH &&
           g.OWs == 2 * g.OW;
  }
  if (pair && !RT) {
    const dim3 grid2((tiles + 7) / 8 * 16, 1, 1);
    const size_t lds = patch_lds_bytes<T, CC>(a, nph, nt, true);
#define SPECENH_PAIR(NT) SPECENH_LAUNCH((conv_patch_kernel<T, NT, CC, false, !RT>), grid2, dim3(256), lds, st, a)
    if (nt == 1) SPECENH_PAIR(1);
    else if (nt == 2) SPECENH_PAIR(2);
    else if (nt == 3) SPECENH_PAIR(3);
    else SPECENH_PAIR(4);
#undef SPECENH_PAIR
    return hipGetLastError() == hipSuccess ? SPECENH_OK : set_error(SPECENH_EHIP, "conv launch");
  }
  // 16-channel single-chunk convs (the model's conv2, 16 -> 32): the workgroup's weight rows
  // are staged in LDS next to the patch, so the k-loop issues no global loads. With the
  // weights streamed from L2 into a register ring the compiler drained every in-flight ring
  // load at each k-step (s_waitcnt vmcnt(0)); SPECENH_PATCH_NO_WL=1 restores that path.
  if constexpr (CC == 16 && !RT) {
    const int Kf = a.g[0].Kf;
    if (nph == 1 && !a.ph_shared && a.g[0].C == 16 && Kf % 8 == 0 &&
        !(variant(V_PATCH_NO_WL) != 0)) {
      const int rs_dw = (Kf / 2 - 8 + 63) / 64 * 64 + 8;  // >= Kf / 2 and = 8 mod 64
      a.wl_rs = 2 * rs_dw;
      const size_t pl = patch_lds_bytes<T, CC>(a, nph, nt, false);
      a.wl_off = (int)pl;
      const size_t lds = pl + (size_t)16 * nt * a.wl_rs * sizeof(T);
      const Geo& g = a.g[0];
      const bool k5 = g.KH == 5 && g.KW == 5 && g.ky0 == 0 && g.kx0 == 0 && g.kstep == 1 &&
                      g.KWf == 5 && Kf == 400 && !(variant(V_PATCH_NO_K5) != 0);
      // LDS weights only with the persistent K5 kernel: restaged per tile (any other
      // 16-channel geometry) they measured slower than the L2 weight ring
      if (k5 && lds <= 48 * 1024) {
        const dim3 grid(tiles, (unsigned)((CO + 16 * nt - 1) / (16 * nt)), 1);
        // persistent K5 grid: 4 workgroups per CU (LDS and registers)
        const dim3 gridk(std::min<unsigned>(tiles, 4u * (unsigned)device_cus()), grid.y, 1);
#define SPECENH_PATCHL(NT, P)                                                                       \
  if (k5) SPECENH_LAUNCH((conv_patch_kernel<T, NT, 16, P, false, false, false, true, true>), gridk, \
                             dim3(256), lds, st, a);                                                 \
  else SPECENH_LAUNCH((conv_patch_kernel<T, NT, 16, P, false, false, false, true>), grid, dim3(256), lds, st, a)
        if (a.pool) {
          if (nt == 1) SPECENH_PATCHL(1, true);
          else if (nt == 2) SPECENH_PATCHL(2, true);
          else if (nt == 3) SPECENH_PATCHL(3, true);
          else SPECENH_PATCHL(4, true);
        } else {
          if (nt == 1) SPECENH_PATCHL(1, false);
          else if (nt == 2) SPECENH_PATCHL(2, false);
          else if (nt == 3) SPECENH_PATCHL(3, false);
          else SPECENH_PATCHL(4, false);
        }
#undef SPECENH_PATCHL
        return hipGetLastError() == hipSuccess ? SPECENH_OK : set_error(SPECENH_EHIP, "conv launch");
      }
    }
  }
  // wave split (2 x 2 waves, 8 rows x 16 NTW channels each, 32 NTW channels per workgroup):
  // each weight fragment feeds 8 MFMAs instead of 4 and the waves load different weights,
  // so the weight loads' L2 latency has twice the MFMA work to hide behind. Register budget
  // held at 3 waves per SIMD. Per 2048 shots (tools/layer_ab.py HIP events, 4x1 -> 2x2):
  // conv3+pool 0.26 -> 0.21, convT1 0.27 -> 0.22, convT2 0.56 -> 0.46 ms.
  // Default wherever the channels allow and the grid keeps >= 2 workgroups per CU;
  // SPECENH_PATCH_WSPLIT=1 forces it, =0 turns it off. The accumulation order per output
  // is unchanged: bitwise the same results.
  const int ntw = nt >= 4 && CC == 32 ? 2 : 1;  // (2 with 64-channel chunks spills)
  const int wsm = variant(V_PATCH_WSPLIT);
  // not with 16-channel chunks: conv2+pool (C 16 -> 32) runs 0.48 ms with the split vs
  // 0.38 without per 2048 shots (tools/layer_ab.py); 32/64-channel chunks gain 20-25 %
  const bool ws_shape = CC >= 32 && nt >= 2 && CO % (32 * ntw) == 0;
  const bool ws_auto =
      (unsigned long long)tiles * (CO / (32 * ntw)) * (a.ph_shared ? 1 : nph) >= 512;
  if (ws_shape && (wsm == 1 || (wsm < 0 && ws_auto))) {
    const dim3 gridw(tiles, (unsigned)(CO / (32 * ntw)), a.ph_shared ? 1 : nph);
    const size_t ldsw = patch_lds_bytes<T, CC>(a, nph, ntw, false);
#define SPECENH_PATCHW(NT, P) SPECENH_LAUNCH((conv_patch_kernel<T, NT, CC, P && !RT, false, false, true, false, false, RT>), gridw, dim3(256), ldsw, st, a)
    if (a.pool) {
      if (ntw == 1) SPECENH_PATCHW(1, true);
      else SPECENH_PATCHW(2, true);
    } else {
      if (ntw == 1) SPECENH_PATCHW(1, false);
      else SPECENH_PATCHW(2, false);
    }
#undef SPECENH_PATCHW
    return hipGetLastError() == hipSuccess ? SPECENH_OK : set_error(SPECENH_EHIP, "conv launch");
  }
  const dim3 grid(tiles, (unsigned)((CO + 16 * nt - 1) / (16 * nt)), a.ph_shared ? 1 : nph);
  const size_t lds = patch_lds_bytes<T, CC>(a, nph, nt, false);
#define SPECENH_PATCH(NT, P) SPECENH_LAUNCH((conv_patch_kernel<T, NT, CC, P && !RT, false, false, false, false, false, RT>), grid, dim3(256), lds, st, a)
  if (a.pool) {
    if (nt == 1) SPECENH_PATCH(1, true);
    else if (nt == 2) SPECENH_PATCH(2, true);
    else if (nt == 3) SPECENH_PATCH(3, true);
    else SPECENH_PATCH(4, true);
  } else {
    if (nt == 1) SPECENH_PATCH(1, false);
    else if (nt == 2) SPECENH_PATCH(2, false);
    else if (nt == 3) SPECENH_PATCH(3, false);
    else SPECENH_PATCH(4, false);
  }
#undef SPECENH_PATCH
  return hipGetLastError() == hipSuccess ? SPECENH_OK : set_error(SPECENH_EHIP, "conv launch");
}

// stride-2 conv (Conv2DTranspose input gradient) over de-interleaved 16-channel patches. At
// least 2 N tiles per workgroup (SPECENH_S2_MIN_NT, default 2): with C > 16 every N tile
// re-stages all channel chunks, and the C4 step's 16 x 16 convT1 gradient (128 tiles) ran 512
// one-tile workgroups: 0.737 -> 0.716 ms per step with 2 (profiles/r05_c4_s2_nt_ab.txt)
template <typename T>
int launch_patch_s2(const ConvArgs& a, hipStream_t st) {
  const Geo& g = a.g[0];
  const unsigned tiles = (unsigned)(g.N * ((g.OH + 15) / 16) * ((g.OW + 15) / 16));
  const int nt = std::min(std::max(patch_nt(g.CO, tiles), variant(V_S2_MIN_NT)),
                          std::min(4, (g.CO + 15) / 16));
  const int sph = (30 + g.KH + 1) / 2, spw = (30 + g.KW + 1) / 2;
  const size_t lds = ((size_t)4 * sph * spw * Patch<16>::PST * sizeof(T) + 15) / 16 * 16;
  const dim3 grid(tiles, (unsigned)((g.CO + 16 * nt - 1) / (16 * nt)), 1);
#define SPECENH_S2(NT) SPECENH_LAUNCH((conv_patch_kernel<T, NT, 16, false, false, true>), grid, dim3(256), lds, st, a)
  if (nt == 1) SPECENH_S2(1);
  else if (nt == 2) SPECENH_S2(2);
  else if (nt == 3) SPECENH_S2(3);
  else SPECENH_S2(4);
#undef SPECENH_S2
  return hipGetLastError() == hipSuccess ? SPECENH_OK : set_error(SPECENH_EHIP, "conv launch");
}

// which LDS-patch chunking applies (0 = none: use the generic gather kernel; -2: the
// stride-2 16-channel patch kernel)
int patch_cc(const ConvArgs& a, int nph) {
  if (nph == 1 && a.g[0].stride == 2 && a.g[0].C % 16 == 0 && a.g[0].KH <= 5 && a.g[0].KW <= 5 &&
      !a.pool && !(variant(V_CONV_NO_S2) != 0))
    return -2;
  if (nph != 1 && nph != 4) return 0;
  for (int i = 0; i < nph; ++i) {
    const Geo& g = a.g[i];
    // (k <= 7: the 7 x 7 convs of hyperparam_scan.py:153-161 take the patch kernel too, a 22 x 22
    // patch; round 4 stopped at 5 x 5 and sent them to the gather kernel, 2.5 ms per 512)
    if (g.stride != 1 || g.KH > 7 || g.KW > 7 || g.KH * g.KW > 64) return 0;
  }
  const int C = a.g[0].C;
  if (C % 64 == 0) return 64;
  if (C % 32 == 0) return 32;
  if (C == 16) return 16;
  if (C == 1) {  // one MFMA k-step holds all taps: at most 32 (k <= 5)
    for (int i = 0; i < nph; ++i)
      if (a.g[i].KH > 5 || a.g[i].KW > 5 || a.g[i].KH * a.g[i].KW > 32) return 0;
    return 1;
  }
  return 0;
}

// conv_rows.hip: inference Conv2D(5, relu, same) + MaxPooling2D(2) and Conv2DTranspose(5,
// s2, relu, same) on 64 channels as row sweeps
int conv_rows_pool(int dtype, const void* x, int N, int H, int W, int CI, const void* w,
                   const float* b, int CO, int K, void* out, hipStream_t st, bool* launched);
int convt_rows(int dtype, const void* x, int N, int H, int W, int CI, const void* w,
               const float* b, int CO, int K, void* out, hipStream_t st, bool* launched);
int conv1_rows_pool(int dtype, const void* x, int N, int H, int W, const void* w,
                    const float* b, int CO, void* out, hipStream_t st, bool* launched);

template <typename T>
int launch_fwd(const ConvArgs& a, int nph, hipStream_t st) {
  if constexpr (!__is_same(T, float)) {
    const Geo& g = a.g[0];
    if (nph == 1 && a.pool && !a.argmax && !a.mask && !a.logits && !a.out_f32 && a.act == 1 &&
        a.bias && g.stride == 1 && (g.KH == 5 || g.KH == 3) && g.KW == g.KH &&
        g.pad_t == g.KH / 2 && g.pad_l == g.KH / 2 &&
        g.OH == g.IH && g.OW == g.IW && g.ky0 == 0 && g.kx0 == 0 && g.kstep == 1 &&
        g.KWf == g.KH && g.Kf == g.KH * g.KH * g.C && g.oys == 1 && g.oxs == 1 && g.oy0 == 0 &&
        g.ox0 == 0) {
      bool launched = false;
      const int rc = conv_rows_pool(__is_same(T, _Float16) ? SPECENH_DTYPE_F16 : SPECENH_DTYPE_BF16,
                                    a.in, g.N, g.IH, g.IW, g.C, a.w, a.bias, g.CO, g.KH, a.out,
                                    st, &launched);
      if (rc != SPECENH_OK || launched) return rc;
    }
    if (!(variant(V_CONV_NO_PATCH) != 0)) {
      switch (patch_cc(a, nph)) {
        case -2: return launch_patch_s2<T>(a, st);
        case 64: return launch_patch<T, 64>(a, nph, st);
        case 32: return launch_patch<T, 32>(a, nph, st);
        case 16: return launch_patch<T, 16>(a, nph, st);
        case 1: return launch_patch<T, 1>(a, nph, st);
        default: break;
      }
    }
  }
  if (a.pool) return set_error(SPECENH_EUNSUPPORTED, "fused max-pool needs the LDS-patch path");
  int maxM = 0;
  for (int i = 0; i < nph; ++i) maxM = std::max(maxM, a.g[i].N * a.g[i].OH * a.g[i].OW);
  const int CO = a.g[0].CO;
  const int nt = std::min(4, (CO + 15) / 16);
  const int mt = nt >= 3 ? 2 : 4;
  const unsigned gx = (unsigned)((maxM + 64 * mt - 1) / (64 * mt));
  const unsigned gy = (unsigned)((CO + 16 * nt - 1) / (16 * nt));
  const dim3 grid(gx, gy, nph);
#define SPECENH_FWD(MT, NT) SPECENH_LAUNCH((conv_fwd_kernel<T, MT, NT>), grid, dim3(256), 0, st, a)
  if (nt == 1) SPECENH_FWD(4, 1);
  else if (nt == 2) SPECENH_FWD(4, 2);
  else if (nt == 3) SPECENH_FWD(2, 3);
  else SPECENH_FWD(2, 4);
#undef SPECENH_FWD
  return hipGetLastError() == hipSuccess ? SPECENH_OK : set_error(SPECENH_EHIP, "conv launch");
}

struct WgradPlan {
  int Z, nt;
  unsigned gx, gy;
};

// tile runs of the MFMA path (wgrad_tr_kernel): at most this many partial slices
// (small weight tensors may take more runs: a layer with one workgroup per run would
// otherwise leave one workgroup per CU, latency-bound)
inline int wgrad_tr_zmax(long long CO, long long Kf) { return CO * Kf <= 8192 ? 2048 : 256; }

WgradPlan wgrad_plan(int Kf, int CO) {
  WgradPlan p{};
  p.nt = std::min(4, (CO + 15) / 16);
  p.gx = (unsigned)((Kf + 63) / 64);
  p.gy = (unsigned)((CO + 16 * p.nt - 1) / (16 * p.nt));
  const long long want = 2048 / std::max<long long>(1, (long long)p.gx * p.gy);
  p.Z = (int)std::min<long long>(256, std::max<long long>(1, want));
  return p;
}

// the MFMA path: bf16/f16, every phase stride 1 with C % 16 == 0 and <= 28 taps in a 20 x 20
// patch (SPECENH_WGRAD_GENERIC=1 forces the generic gather kernel)
template <typename T>
bool wgrad_tr_applies(const WgradArgs& a, int nph) {
  if constexpr (__is_same(T, float)) return false;
  if ((variant(V_WGRAD_GENERIC) != 0)) return false;
  for (int i = 0; i < nph; ++i) {
    const Geo& g = a.g[i];
    if ((g.C % 16 != 0 && g.C != 1) || g.stride != 1 || g.KH > 7 || g.KW > 7)
      return false;
    if (g.C == 1 && (g.KH * g.KW > 31 || g.KH > 5 || g.KW > 5))
      return false;  // im2col columns 0..30 (+ the ones column)
  }
  return true;
}

template <typename T>
int launch_wgrad_tr(const WgradArgs& w, int nph, float* dw, float* db, hipStream_t st) {
  const Geo& g0 = w.g[0];
  WgradTrArgs a{};
  // (C == 1: workspace sized like the MFMA path, see specenh_conv2d_wgrad_workspace_bytes)
  for (int i = 0; i < nph; ++i) a.g[i] = w.g[i];
  a.in = w.in;
  a.dout = w.dout;
  a.part = w.part;
  a.bpart = w.bpart;
  a.pd = w.pd;
  a.pam = w.pam;
  a.py = w.py;
  const int nt = std::min(4, (g0.CO + 15) / 16);
  const int ntw = nt >= 2 ? 2 : 1;
  a.ncog = (g0.CO + 16 * ntw - 1) / (16 * ntw);
  a.ntg = 1;
  for (int i = 0; i < nph; ++i) a.ntg = std::max(a.ntg, (w.g[i].KH * w.g[i].KW + 27) / 28);
  const bool c1 = g0.C == 1;
  const int nchunk = c1 ? 1 : g0.C / 16;
  long long tiles = 1;
  for (int i = 0; i < nph; ++i)
    tiles = std::max(tiles, (long long)w.g[i].N * ((w.g[i].OH + 15) / 16) * ((w.g[i].OW + 15) / 16));
  // ~4096 workgroups, at least 4 tiles each
  const long long wg_target = std::max(1, variant(V_WGRAD_WG));
  long long z = wg_target / std::max(1LL, (long long)nchunk * a.ncog * nph * a.ntg);
  z = std::min<long long>(z, std::max(1LL, tiles / (c1 ? std::max(1, variant(V_WGRAD_C1_TILES)) : 4)));
  a.Z = (int)std::max(1LL, std::min<long long>(z, wgrad_tr_zmax(g0.CO, g0.Kf)));
  // one output channel over 16 input channels: jy-shifted input x jx-shifted dOut
  if (nph == 1 && g0.CO == 1 && g0.C == 16 && g0.KH <= 5 && g0.KW <= 5 &&
      !(variant(V_WGRAD_NO_CO1) != 0)) {
    a.Z = (int)std::max(1LL, std::min<long long>({tiles / 2, (long long)wgrad_tr_zmax(1, g0.Kf), wg_target}));
    SPECENH_LAUNCH(wgrad_co1_kernel<T>, dim3((unsigned)a.Z), dim3(64), 0, st, a);
    launch_ordered_sums(a.part, a.Z, g0.Kf, dw, a.bpart, a.Z, 1, db, st, w.overwrite);
    return hipGetLastError() == hipSuccess ? SPECENH_OK : set_error(SPECENH_EHIP, "wgrad launch");
  }
  // Conv2DTranspose stride 2: all four phases per workgroup over one union patch
  if (!c1 && nph == 4 && g0.CO % 16 == 0 && a.ntg == 1 && !(variant(V_WGRAD_PERPHASE) != 0)) {
    bool ok = true;
    int upt = -1 << 20, upl = -1 << 20, lo_y = 1 << 20, hi_y = -(1 << 20), lo_x = 1 << 20,
        hi_x = -(1 << 20), U = 0;
    for (int i = 0; i < nph; ++i) {
      const Geo& g = w.g[i];
      ok = ok && g.OH == g0.OH && g.OW == g0.OW && g.oys == 2 && g.oxs == 2 && g.oy0 == i / 2 &&
           g.ox0 == i % 2 && g.OHs == 2 * g.OH && g.OWs == 2 * g.OW;
      upt = std::max(upt, g.pad_t);
      upl = std::max(upl, g.pad_l);
      lo_y = std::min(lo_y, -g.pad_t);
      hi_y = std::max(hi_y, 15 - g.pad_t + g.KH - 1);
      lo_x = std::min(lo_x, -g.pad_l);
      hi_x = std::max(hi_x, 15 - g.pad_l + g.KW - 1);
      U += g.KH * g.KW;
    }
    // each wave's run of (phase, tap) blocks (wgrad_trp_kernel) spans at most two phases
    auto phase_of = [&](int u) {
      int p = 0;
      while (p < 3 && u >= w.g[p].KH * w.g[p].KW) { u -= w.g[p].KH * w.g[p].KW; ++p; }
      return p;
    };
    for (int wv = 0; wv < 4 && ok && U > 0; ++wv) {
      const int ub = wv * U / 4, ue = (wv + 1) * U / 4;
      if (ue > ub && phase_of(ue - 1) - phase_of(ub) > 1) ok = false;
    }
    if (ok && hi_y - lo_y + 1 <= 20 && hi_x - lo_x + 1 <= 20 && U <= 28) {
      a.upt = upt;
      a.upl = upl;
      a.PH = hi_y - lo_y + 1;
      a.PW = hi_x - lo_x + 1;
      a.ncog = g0.CO / 16;
      long long zp = wg_target / std::max(1LL, (long long)nchunk * a.ncog);
      zp = std::min<long long>(zp, std::max(1LL, tiles / 4));
      a.Z = (int)std::max(1LL, std::min<long long>(zp, wgrad_tr_zmax(g0.CO, g0.Kf)));
      SPECENH_LAUNCH(wgrad_trp_kernel<T>, dim3((unsigned)a.Z, (unsigned)(nchunk * a.ncog)), dim3(256), 0,
                         st, a);
      launch_ordered_sums(a.part, a.Z, (long long)g0.CO * g0.Kf, dw, a.bpart, nph * a.Z, g0.CO, db, st,
                          w.overwrite);
      return hipGetLastError() == hipSuccess ? SPECENH_OK : set_error(SPECENH_EHIP, "wgrad launch");
    }
  }
  const dim3 grid((unsigned)a.Z, (unsigned)(nchunk * a.ncog), (unsigned)(nph * a.ntg));
  if (c1) {
    if (ntw == 1) SPECENH_LAUNCH((wgrad_tr_kernel<T, 1, true>), grid, dim3(256), 0, st, a);
    else SPECENH_LAUNCH((wgrad_tr_kernel<T, 2, true>), grid, dim3(256), 0, st, a);
  } else {
    if (a.pd) {
      if (ntw == 1) SPECENH_LAUNCH((wgrad_tr_kernel<T, 1, false, true>), grid, dim3(256), 0, st, a);
      else SPECENH_LAUNCH((wgrad_tr_kernel<T, 2, false, true>), grid, dim3(256), 0, st, a);
    } else {
      if (ntw == 1) SPECENH_LAUNCH((wgrad_tr_kernel<T, 1, false>), grid, dim3(256), 0, st, a);
      else SPECENH_LAUNCH((wgrad_tr_kernel<T, 2, false>), grid, dim3(256), 0, st, a);
    }
  }
  launch_ordered_sums(a.part, a.Z, (long long)g0.CO * g0.Kf, dw, a.bpart, nph * a.Z, g0.CO, db, st,
                      w.overwrite);
  return hipGetLastError() == hipSuccess ? SPECENH_OK : set_error(SPECENH_EHIP, "wgrad launch");
}

template <typename T>
int launch_wgrad(WgradArgs& a, int nph, float* dw, float* db, hipStream_t st) {
  if constexpr (!__is_same(T, float))
    if (wgrad_tr_applies<T>(a, nph)) return launch_wgrad_tr<T>(a, nph, dw, db, st);
  const Geo& g0 = a.g[0];
  const WgradPlan p = wgrad_plan(g0.Kf, g0.CO);
  constexpr int BP = Tile<T>::BK;
  a.Z = p.Z;
  for (int i = 0; i < nph; ++i) {
    const long long M = (long long)a.g[i].N * a.g[i].OH * a.g[i].OW;
    long long ch = (M + p.Z - 1) / p.Z;
    a.chunk[i] = (int)(((ch + BP - 1) / BP) * BP);
  }
  unsigned gx = 0;
  for (int i = 0; i < nph; ++i)
    gx = std::max(gx, (unsigned)((a.g[i].KH * a.g[i].KW * a.g[i].C + 63) / 64));
  const dim3 grid(gx, p.gy, (unsigned)(nph * p.Z));
#define SPECENH_WG(NT) SPECENH_LAUNCH((conv_wgrad_kernel<T, NT>), grid, dim3(256), 0, st, a)
  if (p.nt == 1) SPECENH_WG(1);
  else if (p.nt == 2) SPECENH_WG(2);
  else if (p.nt == 3) SPECENH_WG(3);
  else SPECENH_WG(4);
#undef SPECENH_WG
  launch_ordered_sums(a.part, p.Z, (long long)g0.CO * g0.Kf, dw, a.bpart, nph * p.Z, g0.CO, db, st,
                      a.overwrite);
  return hipGetLastError() == hipSuccess ? SPECENH_OK : set_error(SPECENH_EHIP, "wgrad launch");
}

}  // namespace specenh

using namespace specenh;

extern "C" {

int specenh_conv2d(int dtype, const void* in, int N, int IH, int IW, int C, const void* w_gemm,
                   int KH, int KW, int CO, const float* bias, int stride, int pad_t, int pad_l,
                   int in_dil, int OH, int OW, int act, const void* mask, float* logits,
                   void* out, int out_f32, int pool2, unsigned char* argmax, void* stream) {
  if (int e = check_sizes(N, IH, IW, C, OH, OW, CO)) return e;
  if (KH <= 0 || KW <= 0 || stride <= 0 || in_dil <= 0)
    return set_error(SPECENH_EINVAL, "bad convolution geometry");
  if (!in || !w_gemm || !out) return set_error(SPECENH_EINVAL, "null pointer");
  if (act < 0 || act > 2) return set_error(SPECENH_EINVAL, "bad activation");
  if (dtype < 0 || dtype > 2) return set_error(SPECENH_EINVAL, "dtype must be f32, bf16 or f16");
  ConvArgs a{};
  int nph = 0;
  if (int e = plan_phases(N, IH, IW, C, CO, KH, KW, stride, pad_t, pad_l, in_dil, OH, OW, a.g, &nph))
    return e;
  a.in = in; a.w = w_gemm; a.bias = bias; a.out = out; a.out_f32 = out_f32;
  a.mask = mask; a.act = act; a.logits = logits; a.nph = nph;
  a.pool = pool2 ? 1 : 0;
  a.argmax = argmax;
  if (a.pool && (nph != 1 || (OH & 1) || (OW & 1) || mask || logits || out_f32))
    return set_error(SPECENH_EUNSUPPORTED, "fused max-pool: plain conv with even output only");
  hipStream_t st = (hipStream_t)stream;
  // Conv2DTranspose(K, s2, relu, same) on 64 channels (K = 5) or 32 (K = 3 / 5 / 7): the row
  // sweeps (conv_rows.hip); pad = K - 1 - (K - 2) / 2 of the dilated-input conv
  if (dtype != SPECENH_DTYPE_F32 && stride == 1 && in_dil == 2 && KH == KW &&
      (KH == 3 || KH == 5 || KH == 7) && pad_t == KH - 1 - (KH - 2) / 2 && pad_l == pad_t &&
      OH == 2 * IH && OW == 2 * IW && act == 1 && !mask && !logits && !out_f32 && !pool2 &&
      bias) {
    bool launched = false;
    const int rc = convt_rows(dtype, in, N, IH, IW, C, w_gemm, bias, CO, KH, out, st, &launched);
    if (rc != SPECENH_OK || launched) return rc;
  }
  // 1 input channel, pooled inference on 128-wide images: the row sweep (conv_rows.hip)
  if (stride == 1 && in_dil == 1 && C == 1 && KH == 5 && KW == 5 && pad_t == 2 && pad_l == 2 &&
      OH == IH && OW == IW && act == 1 && pool2 && !argmax && !mask && !logits && !out_f32 &&
      bias && dtype != SPECENH_DTYPE_F32) {
    bool launched = false;
    const int rc = conv1_rows_pool(dtype, in, N, IH, IW, w_gemm, bias, CO, out, st, &launched);
    if (rc != SPECENH_OK || launched) return rc;
  }
  // 1 input channel: window rows as MFMA K runs (conv_c1_mfma.hip)
  if (stride == 1 && in_dil == 1 && C == 1 && !(variant(V_CONV_NO_C1MFMA) != 0)) {
    const int r = launch_conv_c1_mfma(dtype, in, N, IH, IW, C, w_gemm, KH, KW, CO, bias, pad_t,
                                      pad_l, OH, OW, act, out, out_f32, logits, pool2, argmax, mask, st);
    if (r != 0) return r < 0 ? r : SPECENH_OK;
  }
  // 1 input or 1 output channel: direct VALU convolution (conv_narrow.hip)
  if (stride == 1 && in_dil == 1 && !(variant(V_CONV_NO_NARROW) != 0)) {
    const int r = launch_conv_narrow(dtype, in, N, IH, IW, C, w_gemm, KH, KW, CO, bias, pad_t,
                                     pad_l, OH, OW, act, out, out_f32, logits, pool2, argmax, mask, st);
    if (r != 0) return r < 0 ? r : SPECENH_OK;
  }
  if (dtype == SPECENH_DTYPE_F32) return launch_fwd<float>(a, nph, st);
  if (dtype == SPECENH_DTYPE_BF16) return launch_fwd<__bf16>(a, nph, st);
  return launch_fwd<_Float16>(a, nph, st);
}

size_t specenh_conv2d_wgrad_workspace_bytes(int N, int OH, int OW, int KH, int KW, int C,
                                            int CO) {
  if (N <= 0 || OH <= 0 || OW <= 0 || KH <= 0 || KW <= 0 || C <= 0 || CO <= 0) return 0;
  const WgradPlan p = wgrad_plan(KH * KW * C, CO);
  // room for the generic plan's slices and, when C % 16 == 0, the MFMA path's
  const size_t Z = (C % 16 == 0 || C == 1)
                       ? std::max<size_t>(p.Z, wgrad_tr_zmax(CO, (long long)KH * KW * C))
                       : (size_t)p.Z;
  return (Z * CO * KH * KW * C + (size_t)MAXPH * Z * CO) * sizeof(float);
}

int specenh_conv2d_wgrad(int dtype, const void* in, int N, int IH, int IW, int C, const void* dout,
                         int KH, int KW, int CO, int stride, int pad_t, int pad_l, int in_dil,
                         int OH, int OW, float* dw, float* dbias, void* workspace, void* stream) {
  return specenh_conv2d_wgrad_ex(dtype, in, N, IH, IW, C, dout, KH, KW, CO, stride, pad_t, pad_l,
                                 in_dil, OH, OW, dw, dbias, 0, workspace, stream);
}

int specenh_conv2d_wgrad_ex(int dtype, const void* in, int N, int IH, int IW, int C,
                            const void* dout, int KH, int KW, int CO, int stride, int pad_t,
                            int pad_l, int in_dil, int OH, int OW, float* dw, float* dbias,
                            int overwrite, void* workspace, void* stream) {
  if (int e = check_sizes(N, IH, IW, C, OH, OW, CO)) return e;
  if (KH <= 0 || KW <= 0 || stride <= 0 || in_dil <= 0)
    return set_error(SPECENH_EINVAL, "bad convolution geometry");
  if (!in || !dout || !dw || !workspace) return set_error(SPECENH_EINVAL, "null pointer");
  if (in_dil > KH || in_dil > KW)
    return set_error(SPECENH_EUNSUPPORTED, "wgrad needs kernel_size >= in_dil");
  if (dtype < 0 || dtype > 2) return set_error(SPECENH_EINVAL, "dtype must be f32, bf16 or f16");
  WgradArgs a{};
  int nph = 0;
  if (int e = plan_phases(N, IH, IW, C, CO, KH, KW, stride, pad_t, pad_l, in_dil, OH, OW, a.g, &nph))
    return e;
  const WgradPlan p = wgrad_plan(KH * KW * C, CO);
  a.in = in;
  a.dout = dout;
  a.overwrite = overwrite != 0;
  a.part = (float*)workspace;
  const size_t Zws = (C % 16 == 0 || C == 1)
                         ? std::max<size_t>(p.Z, wgrad_tr_zmax(CO, (long long)KH * KW * C))
                         : (size_t)p.Z;
  a.bpart = dbias ? a.part + Zws * CO * KH * KW * C : nullptr;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == SPECENH_DTYPE_F32) return launch_wgrad<float>(a, nph, dw, dbias, st);
  if (dtype == SPECENH_DTYPE_BF16) return launch_wgrad<__bf16>(a, nph, dw, dbias, st);
  return launch_wgrad<_Float16>(a, nph, dw, dbias, st);
}

int specenh_conv2d_wgrad_pooled(int dtype, const void* in, int N, int IH, int IW, int C,
                                const void* dpool, const unsigned char* argmax, const void* pooled,
                                int KH, int KW, int CO, int stride, int pad_t, int pad_l,
                                int in_dil, int OH, int OW, float* dw, float* dbias,
                                void* workspace, void* stream) {
  if (int e = check_sizes(N, IH, IW, C, OH, OW, CO)) return e;
  if (KH <= 0 || KW <= 0 || stride <= 0 || in_dil <= 0)
    return set_error(SPECENH_EINVAL, "bad convolution geometry");
  if (!in || !dpool || !argmax || !dw || !workspace) return set_error(SPECENH_EINVAL, "null pointer");
  if (dtype != SPECENH_DTYPE_BF16 && dtype != SPECENH_DTYPE_F16)
    return set_error(SPECENH_EUNSUPPORTED, "pooled wgrad: bf16 / f16");
  if ((C != 1 && C % 16 != 0) || stride != 1 || in_dil != 1 || (OH & 1) || (OW & 1) || (CO & 7) ||
      ((uintptr_t)dpool & 15) || ((uintptr_t)argmax & 7) || ((uintptr_t)pooled & 15))
    return set_error(SPECENH_EUNSUPPORTED,
                     "pooled wgrad: C = 1 or C % 16 == 0, stride 1, even output, CO % 8 == 0");
  WgradArgs a{};
  int nph = 0;
  if (int e = plan_phases(N, IH, IW, C, CO, KH, KW, stride, pad_t, pad_l, in_dil, OH, OW, a.g, &nph))
    return e;
  if (nph != 1 || a.g[0].oys != 1 || a.g[0].oxs != 1 || a.g[0].oy0 != 0 || a.g[0].ox0 != 0 ||
      a.g[0].CO != CO || a.g[0].OHs != OH || a.g[0].OWs != OW)
    return set_error(SPECENH_EUNSUPPORTED, "pooled wgrad: a plain stride-1 convolution");
  const WgradPlan p = wgrad_plan(KH * KW * C, CO);
  a.in = in;
  a.dout = nullptr;
  a.pd = dpool;
  a.pam = argmax;
  a.py = pooled;
  a.overwrite = true;
  a.part = (float*)workspace;
  const size_t Zws = std::max<size_t>(p.Z, wgrad_tr_zmax(CO, (long long)KH * KW * C));
  a.bpart = dbias ? a.part + Zws * CO * KH * KW * C : nullptr;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == SPECENH_DTYPE_BF16) {
    if (!wgrad_tr_applies<__bf16>(a, nph)) return set_error(SPECENH_EUNSUPPORTED, "pooled wgrad: shape");
    return launch_wgrad_tr<__bf16>(a, nph, dw, dbias, st);
  }
  if (!wgrad_tr_applies<_Float16>(a, nph)) return set_error(SPECENH_EUNSUPPORTED, "pooled wgrad: shape");
  return launch_wgrad_tr<_Float16>(a, nph, dw, dbias, st);
}

int specenh_conv2d_pooled_in(int dtype, const void* dpool, const unsigned char* argmax,
                             const void* pooled, int N, int IH, int IW, int C, const void* w_gemm,
                             int KH, int KW, int CO, const float* bias, int pad_t, int pad_l,
                             int OH, int OW, int act, const void* mask, void* out, void* stream) {
  if (int e = check_sizes(N, IH, IW, C, OH, OW, CO)) return e;
  if (KH <= 0 || KW <= 0) return set_error(SPECENH_EINVAL, "bad convolution geometry");
  if (!dpool || !argmax || !w_gemm || !out) return set_error(SPECENH_EINVAL, "null pointer");
  if (act < 0 || act > 2) return set_error(SPECENH_EINVAL, "bad activation");
  if (dtype != SPECENH_DTYPE_BF16 && dtype != SPECENH_DTYPE_F16)
    return set_error(SPECENH_EUNSUPPORTED, "pool-routed conv: bf16 / f16");
  if ((IH & 1) || (IW & 1) || C % 16 != 0 || ((uintptr_t)dpool & 15) || ((uintptr_t)argmax & 7) ||
      ((uintptr_t)pooled & 15))
    return set_error(SPECENH_EUNSUPPORTED, "pool-routed conv: even input, C % 16 == 0");
  ConvArgs a{};
  int nph = 0;
  if (int e = plan_phases(N, IH, IW, C, CO, KH, KW, 1, pad_t, pad_l, 1, OH, OW, a.g, &nph)) return e;
  a.in = dpool; a.w = w_gemm; a.bias = bias; a.out = out; a.mask = mask; a.act = act; a.nph = nph;
  a.rpd = dpool; a.ram = argmax; a.rpy = pooled;
  const int cc = variant(V_CONV_NO_PATCH) != 0 ? 0 : patch_cc(a, nph);
  if (nph != 1 || (cc != 16 && cc != 32 && cc != 64))
    return set_error(SPECENH_EUNSUPPORTED, "pool-routed conv: a stride-1 conv on the LDS-patch path");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == SPECENH_DTYPE_BF16)
    return cc == 64 ? launch_patch<__bf16, 64, true>(a, nph, st)
                    : (cc == 32 ? launch_patch<__bf16, 32, true>(a, nph, st)
                                : launch_patch<__bf16, 16, true>(a, nph, st));
  return cc == 64 ? launch_patch<_Float16, 64, true>(a, nph, st)
                  : (cc == 32 ? launch_patch<_Float16, 32, true>(a, nph, st)
                              : launch_patch<_Float16, 16, true>(a, nph, st));
}

int specenh_maxpool2_fwd(int dtype, const void* in, int N, int H, int W, int C, void* out,
                         unsigned char* argmax, void* stream) {
  if (N <= 0 || H <= 0 || W <= 0 || C <= 0 || (H & 1) || (W & 1))
    return set_error(SPECENH_EINVAL, "maxpool2 needs even H, W");
  if (!in || !out) return set_error(SPECENH_EINVAL, "null pointer");
  const long long n = (long long)N * (H / 2) * (W / 2) * C;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == 0)
    SPECENH_LAUNCH(maxpool2_fwd_kernel<float>, dim3(grid1d(n)), dim3(256), 0, st,
                       (const float*)in, N, H, W, C, (float*)out, argmax);
  else if (dtype == 1)
    SPECENH_LAUNCH(maxpool2_fwd_kernel<__bf16>, dim3(grid1d(n)), dim3(256), 0, st,
                       (const __bf16*)in, N, H, W, C, (__bf16*)out, argmax);
  else if (dtype == 2)
    SPECENH_LAUNCH(maxpool2_fwd_kernel<_Float16>, dim3(grid1d(n)), dim3(256), 0, st,
                       (const _Float16*)in, N, H, W, C, (_Float16*)out, argmax);
  else
    return set_error(SPECENH_EINVAL, "dtype");
  return hipGetLastError() == hipSuccess ? SPECENH_OK : set_error(SPECENH_EHIP, "maxpool fwd");
}

int specenh_maxpool2_bwd(int dtype, const void* dout, const unsigned char* argmax,
                         const void* pooled, int N, int H, int W, int C, void* din,
                         void* stream) {
  if (N <= 0 || H <= 0 || W <= 0 || C <= 0 || (H & 1) || (W & 1))
    return set_error(SPECENH_EINVAL, "maxpool2 needs even H, W");
  if (!dout || !argmax || !din) return set_error(SPECENH_EINVAL, "null pointer");
  const long long n = (long long)N * (H / 2) * (W / 2) * C;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == 0)
    SPECENH_LAUNCH(maxpool2_bwd_kernel<float>, dim3(grid1d(n)), dim3(256), 0, st,
                       (const float*)dout, argmax, (const float*)pooled, N, H, W, C, (float*)din);
  else if ((dtype == 1 || dtype == 2) && (C & 7) == 0 && 4 * n < (1LL << 31)) {
    const unsigned blocks = (unsigned)((n / 8 + 255) / 256);
    if (dtype == 1)
      SPECENH_LAUNCH(maxpool2_bwd_vec_kernel<__bf16>, dim3(blocks), dim3(256), 0, st,
                         (const __bf16*)dout, argmax, (const __bf16*)pooled, N, H, W, C, (__bf16*)din);
    else
      SPECENH_LAUNCH(maxpool2_bwd_vec_kernel<_Float16>, dim3(blocks), dim3(256), 0, st,
                         (const _Float16*)dout, argmax, (const _Float16*)pooled, N, H, W, C,
                         (_Float16*)din);
  } else if (dtype == 1)
    SPECENH_LAUNCH(maxpool2_bwd_kernel<__bf16>, dim3(grid1d(n)), dim3(256), 0, st,
                       (const __bf16*)dout, argmax, (const __bf16*)pooled, N, H, W, C,
                       (__bf16*)din);
  else if (dtype == 2)
    SPECENH_LAUNCH(maxpool2_bwd_kernel<_Float16>, dim3(grid1d(n)), dim3(256), 0, st,
                       (const _Float16*)dout, argmax, (const _Float16*)pooled, N, H, W, C,
                       (_Float16*)din);
  else
    return set_error(SPECENH_EINVAL, "dtype");
  return hipGetLastError() == hipSuccess ? SPECENH_OK : set_error(SPECENH_EHIP, "maxpool bwd");
}

int specenh_bce_logits(const float* z, const void* target, int target_dtype, long long n,
                       void* grad, int grad_dtype, double* loss_sum, void* stream) {
  if (!z || !target || n <= 0) return set_error(SPECENH_EINVAL, "bce args");
  hipStream_t st = (hipStream_t)stream;
  const unsigned gx = (unsigned)std::max<long long>(1, std::min<long long>((n + 256 * 16 - 1) / (256 * 16), 256));
#define SPECENH_BCE(TT, TG)                                                                   \
  SPECENH_LAUNCH((bce_logits_kernel<TT, TG>), dim3(gx), dim3(256), 0, st, z,             \
                     (const TT*)target, n, (TG*)grad, loss_sum)
  if (target_dtype == 0 && grad_dtype == 0) SPECENH_BCE(float, float);
  else if (target_dtype == 0 && grad_dtype == 1) SPECENH_BCE(float, __bf16);
  else if (target_dtype == 1 && grad_dtype == 0) SPECENH_BCE(__bf16, float);
  else if (target_dtype == 1 && grad_dtype == 1) SPECENH_BCE(__bf16, __bf16);
  else if (target_dtype == 0 && grad_dtype == 2) SPECENH_BCE(float, _Float16);
  else if (target_dtype == 2 && grad_dtype == 0) SPECENH_BCE(_Float16, float);
  else if (target_dtype == 2 && grad_dtype == 2) SPECENH_BCE(_Float16, _Float16);
  else return set_error(SPECENH_EINVAL, "dtype");
#undef SPECENH_BCE
  return hipGetLastError() == hipSuccess ? SPECENH_OK : set_error(SPECENH_EHIP, "bce");
}

int specenh_adam_step(float* w, const float* g, float* m, float* v, long long n, float lr_t,
                      float b1, float b2, float eps, float grad_scale, void* w_lowp,
                      int lowp_dtype, void* stream) {
  if (!w || !g || !m || !v || n <= 0) return set_error(SPECENH_EINVAL, "adam args");
  hipStream_t st = (hipStream_t)stream;
  if (lowp_dtype == SPECENH_DTYPE_F16)
    SPECENH_LAUNCH(adam_kernel<_Float16>, dim3(grid1d(n)), dim3(256), 0, st, w, g, m, v, n,
                       lr_t, b1, b2, eps, grad_scale, (_Float16*)w_lowp);
  else if (lowp_dtype == SPECENH_DTYPE_BF16 || !w_lowp)
    SPECENH_LAUNCH(adam_kernel<__bf16>, dim3(grid1d(n)), dim3(256), 0, st, w, g, m, v, n,
                       lr_t, b1, b2, eps, grad_scale, (__bf16*)w_lowp);
  else
    return set_error(SPECENH_EINVAL, "adam: low-precision copy must be bf16 or f16");
  return hipGetLastError() == hipSuccess ? SPECENH_OK : set_error(SPECENH_EHIP, "adam");
}

int specenh_adam_step_flip(float* w, const float* g, float* m, float* v, long long n, float lr_t,
                           float b1, float b2, float eps, float grad_scale, void* w_lowp,
                           int lowp_dtype, int nseg, const long long* seg_off, const int* seg_kcc,
                           void* const* seg_dst, void* stream) {
  if (!w || !g || !m || !v || n <= 0) return set_error(SPECENH_EINVAL, "adam args");
  if (nseg < 0 || nseg > 8 || (nseg > 0 && (!seg_off || !seg_kcc || !seg_dst)))
    return set_error(SPECENH_EINVAL, "adam_flip: 0..8 segments");
  FlipSegs fs{};
  fs.n = nseg;
  for (int s = 0; s < nseg; ++s) {
    const long long sz = (long long)seg_kcc[3 * s] * seg_kcc[3 * s] * seg_kcc[3 * s + 1] *
                         seg_kcc[3 * s + 2];
    if (!seg_dst[s] || sz <= 0 || seg_off[s] < 0 || seg_off[s] + sz > n)
      return set_error(SPECENH_EINVAL, "adam_flip: segment outside w");
    fs.off[s] = seg_off[s];
    fs.k[s] = seg_kcc[3 * s];
    fs.ci[s] = seg_kcc[3 * s + 1];
    fs.co[s] = seg_kcc[3 * s + 2];
    fs.dst[s] = seg_dst[s];
  }
  hipStream_t st = (hipStream_t)stream;
  if (!w_lowp)
    SPECENH_LAUNCH((adam_flip_kernel<float, false>), dim3(grid1d(n)), dim3(256), 0, st, w, g, m, v,
                   n, lr_t, b1, b2, eps, grad_scale, (float*)nullptr, fs);
  else if (lowp_dtype == SPECENH_DTYPE_F16)
    SPECENH_LAUNCH((adam_flip_kernel<_Float16, true>), dim3(grid1d(n)), dim3(256), 0, st, w, g, m,
                   v, n, lr_t, b1, b2, eps, grad_scale, (_Float16*)w_lowp, fs);
  else if (lowp_dtype == SPECENH_DTYPE_BF16)
    SPECENH_LAUNCH((adam_flip_kernel<__bf16, true>), dim3(grid1d(n)), dim3(256), 0, st, w, g, m,
                   v, n, lr_t, b1, b2, eps, grad_scale, (__bf16*)w_lowp, fs);
  else
    return set_error(SPECENH_EINVAL, "adam: low-precision copy must be bf16 or f16");
  return hipGetLastError() == hipSuccess ? SPECENH_OK : set_error(SPECENH_EHIP, "adam_flip");
}

int specenh_weight_flip_transpose(int dtype, const void* bt, int k, int ci, int co, void* bd,
                                  void* stream) {
  const long long n = (long long)k * k * ci * co;
  if (!bt || !bd || n <= 0) return set_error(SPECENH_EINVAL, "flip args");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == 0)
    SPECENH_LAUNCH(flip_transpose_kernel<float>, dim3(grid1d(n)), dim3(256), 0, st,
                       (const float*)bt, k, ci, co, (float*)bd);
  else if (dtype == 1)
    SPECENH_LAUNCH(flip_transpose_kernel<__bf16>, dim3(grid1d(n)), dim3(256), 0, st,
                       (const __bf16*)bt, k, ci, co, (__bf16*)bd);
  else if (dtype == 2)
    SPECENH_LAUNCH(flip_transpose_kernel<_Float16>, dim3(grid1d(n)), dim3(256), 0, st,
                       (const _Float16*)bt, k, ci, co, (_Float16*)bd);
  else
    return set_error(SPECENH_EINVAL, "dtype");
  return hipGetLastError() == hipSuccess ? SPECENH_OK : set_error(SPECENH_EHIP, "flip");
}

int specenh_cast(int src_dtype, const void* src, int dst_dtype, void* dst, long long n,
                 void* stream) {
  if (!src || !dst || n < 0) return set_error(SPECENH_EINVAL, "cast args");
  if (n == 0) return SPECENH_OK;
  hipStream_t st = (hipStream_t)stream;
  const dim3 g(grid1d(n)), b(256);
#define SPECENH_CAST(TS, TD) \
  SPECENH_LAUNCH((cast_kernel<TS, TD>), g, b, 0, st, (const TS*)src, (TD*)dst, n)
  const int key = src_dtype * 3 + dst_dtype;
  switch (src_dtype < 0 || src_dtype > 2 || dst_dtype < 0 || dst_dtype > 2 ? -1 : key) {
    case 0 * 3 + 1: SPECENH_CAST(float, __bf16); break;
    case 0 * 3 + 2: SPECENH_CAST(float, _Float16); break;
    case 1 * 3 + 0: SPECENH_CAST(__bf16, float); break;
    case 2 * 3 + 0: SPECENH_CAST(_Float16, float); break;
    case 1 * 3 + 2: SPECENH_CAST(__bf16, _Float16); break;
    case 2 * 3 + 1: SPECENH_CAST(_Float16, __bf16); break;
    default: return set_error(SPECENH_EINVAL, "cast: dtypes must differ, each f32/bf16/f16");
  }
#undef SPECENH_CAST
  return hipGetLastError() == hipSuccess ? SPECENH_OK : set_error(SPECENH_EHIP, "cast");
}

}  // extern "C"
