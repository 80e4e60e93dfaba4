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

namespace specenh {
int set_error(int code, const std::string& msg);  // stft_psd.hip

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
};

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

template <typename T, int NT, int CC>
struct PatchSmem {
  static constexpr int PMAX = 20;
  static constexpr int PATCH = PMAX * PMAX * Patch<CC>::PST * (int)sizeof(T);
  // plain output tile [256 px][16*NT]: fp32 only when NT <= 2 (patch_cc rejects CO > 32)
  static constexpr int OUT = 256 * 16 * NT * (NT <= 2 ? 4 : (int)sizeof(T));
  static constexpr int BYTES = PATCH > OUT ? PATCH : OUT;
};

template <typename T, int NT, int CC, bool POOL>
__global__ __launch_bounds__(256) void conv_patch_kernel(ConvArgs a) {
  constexpr int TILE = 16, PMAX = 20;
  constexpr int PST = Patch<CC>::PST;
  constexpr int MT = 4;  // output rows per wave
  constexpr int COT = 16 * NT;
  __shared__ __attribute__((aligned(16))) char smem[PatchSmem<T, NT, CC>::BYTES];
  __shared__ int sTap[32];  // patch offset of tap t (elements), -1 past the last tap
  __shared__ int sCol[32];  // weight column of tap t at ci = 0
  T* sP = reinterpret_cast<T*>(smem);

  // ---- which tile and phase (the phases of a tile share an XCD) ----
  int phase = 0, tile = blockIdx.x;
  if (a.nph > 1) {
    const int r = blockIdx.x & 31;
    phase = r >> 3;
    tile = (blockIdx.x >> 5) * 8 + (r & 7);
    if (phase >= a.nph) return;
  }
  const Geo& g = a.g[phase];
  const int ntx = (g.OW + TILE - 1) / TILE, nty = (g.OH + TILE - 1) / TILE;
  if (tile >= g.N * nty * ntx) return;
  const int n = tile / (nty * ntx);
  const int trem = tile - n * (nty * ntx);
  const int ty = trem / ntx, tx = trem - (trem / ntx) * ntx;
  const int oy0 = ty * TILE, ox0 = tx * TILE;
  const int iy0 = oy0 - g.pad_t, ix0 = ox0 - g.pad_l;
  const int PW = TILE + g.KW - 1, PH = TILE + g.KH - 1;
  const int ntap = g.KH * g.KW;
  const int n0 = blockIdx.y * COT;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const T* __restrict__ in = reinterpret_cast<const T*>(a.in);
  const T* __restrict__ W = reinterpret_cast<const T*>(a.w);

  if (tid < 32) {
    const int jy = tid / g.KW, jx = tid - (tid / g.KW) * g.KW;
    sTap[tid] = tid < ntap ? (jy * PW + jx) * PST : -1;
    sCol[tid] = tid < ntap ? ((g.ky0 + g.kstep * jy) * g.KWf + g.kx0 + g.kstep * jx) * g.C : 0;
  }

  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  int rbase[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) rbase[i] = ((wave * MT + i) * PW + (lane & 15)) * PST;
  const int kgrp = lane >> 4;

  const int nchunk = CC == 1 ? 1 : g.C / CC;
  for (int c = 0; c < nchunk; ++c) {
    // ---- stage the patch of channel chunk c ----
    if constexpr (CC == 1) {
      for (int e = tid; e < PH * PW; e += 256) {
        const int py = e / PW, px = e - (e / PW) * PW;
        const int iy = iy0 + py, ix = ix0 + px;
        const bool ok = (unsigned)iy < (unsigned)g.IH && (unsigned)ix < (unsigned)g.IW;
        const T v = in[ok ? (n * g.IH + iy) * g.IW + ix : 0];
        sP[e] = ok ? v : from_f<T>(0.f);
      }
    } else {
      constexpr int GP = CC / 8;  // 8-channel groups per pixel
      for (int e = tid; e < PH * PW * GP; e += 256) {
        const int pix = e / GP, cg = e - (e / GP) * GP;
        const int py = pix / PW, px = pix - (pix / PW) * PW;
        const int iy = iy0 + py, ix = ix0 + px;
        const bool ok = (unsigned)iy < (unsigned)g.IH && (unsigned)ix < (unsigned)g.IW;
        V8<T> v = ld8(in + (ok ? ((n * g.IH + iy) * g.IW + ix) * g.C + c * CC + 8 * cg : 0));
        if (!ok) zero8(v);
        st8(sP + pix * PST + 8 * cg, v);
      }
    }
    lds_sync();

    // ---- k-steps: one MFMA K=32 slab each ----
    constexpr int SUB = CC >= 32 ? CC / 32 : 1;  // 32-channel slabs per tap
    const int nsteps = CC >= 32 ? ntap * SUB : (CC == 16 ? (ntap + 1) / 2 : 1);
    auto load_b = [&](int s, V8<T> (&b)[NT]) {
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int co = n0 + 16 * j + (lane & 15);
        zero8(b[j]);
        if constexpr (CC >= 32) {
          const int t = s / SUB, h = s - (s / SUB) * SUB;
          if (co < g.CO) b[j] = ld8(W + co * g.Kf + sCol[t] + c * CC + 32 * h + 8 * kgrp);
        } else if constexpr (CC == 16) {
          const int t = 2 * s + (kgrp >> 1);
          if (co < g.CO && t < ntap) b[j] = ld8(W + co * g.Kf + sCol[t] + 8 * (kgrp & 1));
        } else {
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const int t = 8 * kgrp + q;
            if (co < g.CO && t < ntap) set_elem(b[j], q, W[co * g.Kf + sCol[t]]);
          }
        }
      }
    };
    V8<T> bcur[NT], bnxt[NT];
    load_b(0, bcur);
    for (int s = 0; s < nsteps; ++s) {
      if (s + 1 < nsteps) load_b(s + 1, bnxt);
      int aoff = 0;
      bool aon = true;
      if constexpr (CC >= 32) {
        const int t = s / SUB, h = s - (s / SUB) * SUB;
        aoff = sTap[t] + 32 * h + 8 * kgrp;
      } else if constexpr (CC == 16) {
        const int t = 2 * s + (kgrp >> 1);
        aon = t < ntap;
        aoff = (aon ? sTap[t] : 0) + 8 * (kgrp & 1);
      }
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        V8<T> av;
        if constexpr (CC == 1) {
          zero8(av);
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const int off = sTap[8 * kgrp + q];
            if (off >= 0) set_elem(av, q, sP[rbase[i] + off]);
          }
        } else {
          av = *reinterpret_cast<const V8<T>*>(sP + rbase[i] + aoff);
          if (!aon) zero8(av);
        }
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = mfma32<T>(av, bcur[j], acc[i][j]);
      }
#pragma unroll
      for (int j = 0; j < NT; ++j) bcur[j] = bnxt[j];
    }
    lds_sync();  // the patch is overwritten by the next chunk / the output tile
  }

  // ---- epilogue. D element (i, j, reg): output row oy0 + 4*wave + i, column
  // ox0 + 4*(lane>>4) + reg, channel n0 + 16*j + (lane&15) ----
  const int colv = (int)min(COT, g.CO - n0);  // valid channels of this tile
  if (a.mask || a.logits) {
    // training paths (dgrad with a ReLU mask / last layer's logits): direct stores
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const int oy = oy0 + wave * MT + i;
      if (oy >= g.OH) continue;
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const int ox = ox0 + 4 * (lane >> 4) + reg;
        if (ox >= g.OW) continue;
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
          v = apply_act(v, a.act);
          if (a.out_f32) reinterpret_cast<float*>(a.out)[idx] = v;
          else reinterpret_cast<T*>(a.out)[idx] = from_f<T>(v);
        }
      }
    }
    return;
  }

  if constexpr (POOL) {
    // 2x2 windows: rows (2*ip, 2*ip+1) of this wave, columns (2*rp, 2*rp+1) of this lane
    T* sO = sP;                                                   // [64 px][COT]
    unsigned char* sAm = reinterpret_cast<unsigned char*>(smem) + 64 * COT * sizeof(T);
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int ch = 16 * j + (lane & 15);
      const float bv = (a.bias && n0 + ch < g.CO) ? a.bias[n0 + ch] : 0.f;
#pragma unroll
      for (int ip = 0; ip < 2; ++ip)
#pragma unroll
        for (int rp = 0; rp < 2; ++rp) {
          // compare the values the layer would store (rounded to T), first max wins: the
          // same argmax as MaxPooling2D on the stored activation
          float best = to_f(from_f<T>(apply_act(acc[2 * ip][j][2 * rp] + bv, a.act)));
          int arg = 0;
#pragma unroll
          for (int q = 1; q < 4; ++q) {
            const float v =
                to_f(from_f<T>(apply_act(acc[2 * ip + (q >> 1)][j][2 * rp + (q & 1)] + bv, a.act)));
            if (v > best) { best = v; arg = q; }
          }
          const int pp = (2 * wave + ip) * 8 + 2 * (lane >> 4) + rp;  // pooled pixel in 8x8
          sO[pp * COT + ch] = from_f<T>(best);
          sAm[pp * COT + ch] = (unsigned char)arg;
        }
    }
    lds_sync();
    const int PHo = g.OH / 2, PWo = g.OW / 2;
    const int py0 = oy0 / 2, px0 = ox0 / 2;
    if (colv == COT && (g.CO & 7) == 0) {
      constexpr int GPP = COT / 8;  // 16-byte chunks per pooled pixel
      for (int e = tid; e < 64 * GPP; e += 256) {
        const int pp = e / GPP, cg = e - (e / GPP) * GPP;
        const int py = py0 + pp / 8, px = px0 + (pp & 7);
        if (py >= PHo || px >= PWo) continue;
        const long long o = (((long long)n * PHo + py) * PWo + px) * g.CO + n0 + 8 * cg;
        *reinterpret_cast<uint4*>(reinterpret_cast<T*>(a.out) + o) =
            *reinterpret_cast<const uint4*>(sO + pp * COT + 8 * cg);
        if (a.argmax)
          *reinterpret_cast<uint2*>(a.argmax + o) =
              *reinterpret_cast<const uint2*>(sAm + pp * COT + 8 * cg);
      }
    } else {
      for (int e = tid; e < 64 * COT; e += 256) {
        const int pp = e / COT, ch = e - (e / COT) * COT;
        const int py = py0 + pp / 8, px = px0 + (pp & 7);
        if (ch >= colv || py >= PHo || px >= PWo) continue;
        const long long o = (((long long)n * PHo + py) * PWo + px) * g.CO + n0 + ch;
        reinterpret_cast<T*>(a.out)[o] = sO[pp * COT + ch];
        if (a.argmax) a.argmax[o] = sAm[pp * COT + ch];
      }
    }
    return;
  } else {
    // plain tile [256 px][COT] through LDS, in the output dtype
    const bool f32o = a.out_f32 != 0;
    float* sOf = reinterpret_cast<float*>(smem);
    T* sOt = sP;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int ch = 16 * j + (lane & 15);
      const float bv = (a.bias && n0 + ch < g.CO) ? a.bias[n0 + ch] : 0.f;
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {
          const int px = (wave * MT + i) * 16 + 4 * (lane >> 4) + reg;
          const float v = apply_act(acc[i][j][reg] + bv, a.act);
          if (f32o) sOf[px * COT + ch] = v;
          else sOt[px * COT + ch] = from_f<T>(v);
        }
    }
    lds_sync();
    const int esz = f32o ? 4 : (int)sizeof(T);
    const int cpc = 16 / esz;  // channels per 16-byte chunk
    if (colv == COT && (g.CO % cpc) == 0) {
      const int gpp = COT / cpc;
      for (int e = tid; e < 256 * gpp; e += 256) {
        const int px = e / gpp, cg = e - (e / gpp) * gpp;
        const int oy = oy0 + px / 16, ox = ox0 + (px & 15);
        if (oy >= g.OH || ox >= g.OW) continue;
        const long long o =
            (((long long)n * g.OHs + oy * g.oys + g.oy0) * g.OWs + ox * g.oxs + g.ox0) * g.CO +
            n0 + cpc * cg;
        const char* src = smem + ((long long)px * COT + cpc * cg) * esz;
        char* dst = reinterpret_cast<char*>(a.out) + o * esz;
        *reinterpret_cast<uint4*>(dst) = *reinterpret_cast<const uint4*>(src);
      }
    } else {
      for (int e = tid; e < 256 * COT; e += 256) {
        const int px = e / COT, ch = e - (e / COT) * COT;
        const int oy = oy0 + px / 16, ox = ox0 + (px & 15);
        if (ch >= colv || oy >= g.OH || ox >= g.OW) continue;
        const long long o =
            (((long long)n * g.OHs + oy * g.oys + g.oy0) * g.OWs + ox * g.oxs + g.ox0) * g.CO +
            n0 + ch;
        if (f32o) reinterpret_cast<float*>(a.out)[o] = sOf[px * COT + ch];
        else reinterpret_cast<T*>(a.out)[o] = sOt[px * COT + ch];
      }
    }
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

// dst[e] += sum_{z < nz} part[z * n + e], always in the same order (bit-reproducible).
__global__ void ordered_sum_kernel(const float* __restrict__ part, int nz, long long n,
                                   float* __restrict__ dst) {
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n;
       e += (long long)gridDim.x * blockDim.x) {
    float t0 = 0.f, t1 = 0.f, t2 = 0.f, t3 = 0.f;
    int z = 0;
    for (; z + 4 <= nz; z += 4) {
      t0 += part[(long long)z * n + e];
      t1 += part[(long long)(z + 1) * n + e];
      t2 += part[(long long)(z + 2) * n + e];
      t3 += part[(long long)(z + 3) * n + e];
    }
    for (; z < nz; ++z) t0 += part[(long long)z * n + e];
    dst[e] += (t0 + t1) + (t2 + t3);
  }
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
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const float zi = z[i], ti = to_f(t[i]);
    acc += (double)(fmaxf(zi, 0.f) - zi * ti + log1pf(__expf(-fabsf(zi))));
    if (grad) grad[i] = from_f<TG>((1.f / (1.f + __expf(-zi)) - ti) * inv);
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

// Developer switch read once per process (A/B of kernel variants on the GPU box).
inline bool getenv_flag(const char* name) {
  const char* v = std::getenv(name);
  return v && *v && *v != '0';
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

template <typename T, int CC>
int launch_patch(const ConvArgs& a, int nph, hipStream_t st) {
  unsigned tiles = 0;
  for (int i = 0; i < nph; ++i)
    tiles = std::max(tiles, (unsigned)(a.g[i].N * ((a.g[i].OH + 15) / 16) * ((a.g[i].OW + 15) / 16)));
  const unsigned gx = nph == 1 ? tiles : ((tiles + 7) / 8) * 32;  // phases: 4 x 8-tile groups
  const int CO = a.g[0].CO;
  const int nt = std::min(4, (CO + 15) / 16);
  const dim3 grid(gx, (unsigned)((CO + 16 * nt - 1) / (16 * nt)), 1);
#define SPECENH_PATCH(NT, P) hipLaunchKernelGGL((conv_patch_kernel<T, NT, CC, P>), grid, dim3(256), 0, st, a)
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

// which LDS-patch chunking applies (0 = none: use the generic gather kernel)
int patch_cc(const ConvArgs& a, int nph) {
  if (nph != 1 && nph != 4) return 0;
  for (int i = 0; i < nph; ++i) {
    const Geo& g = a.g[i];
    if (g.stride != 1 || g.KH > 5 || g.KW > 5 || g.KH * g.KW > 32) return 0;
    if (a.out_f32 && a.g[0].CO > 32) return 0;  // fp32 output tile must fit the LDS union
  }
  const int C = a.g[0].C;
  if (C % 64 == 0) return 64;
  if (C % 32 == 0) return 32;
  if (C == 16) return 16;
  if (C == 1) return 1;
  return 0;
}

template <typename T>
int launch_fwd(const ConvArgs& a, int nph, hipStream_t st) {
  if constexpr (!__is_same(T, float)) {
    if (!getenv_flag("SPECENH_CONV_NO_PATCH")) {
      switch (patch_cc(a, nph)) {
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
#define SPECENH_FWD(MT, NT) hipLaunchKernelGGL((conv_fwd_kernel<T, MT, NT>), grid, dim3(256), 0, st, a)
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

WgradPlan wgrad_plan(int Kf, int CO) {
  WgradPlan p{};
  p.nt = std::min(4, (CO + 15) / 16);
  p.gx = (unsigned)((Kf + 63) / 64);
  p.gy = (unsigned)((CO + 16 * p.nt - 1) / (16 * p.nt));
  const long long want = 2048 / std::max<long long>(1, (long long)p.gx * p.gy);
  p.Z = (int)std::min<long long>(256, std::max<long long>(1, want));
  return p;
}

template <typename T>
int launch_wgrad(WgradArgs& a, int nph, float* dw, float* db, hipStream_t st) {
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
#define SPECENH_WG(NT) hipLaunchKernelGGL((conv_wgrad_kernel<T, NT>), grid, dim3(256), 0, st, a)
  if (p.nt == 1) SPECENH_WG(1);
  else if (p.nt == 2) SPECENH_WG(2);
  else if (p.nt == 3) SPECENH_WG(3);
  else SPECENH_WG(4);
#undef SPECENH_WG
  const long long n = (long long)g0.CO * g0.Kf;
  hipLaunchKernelGGL(ordered_sum_kernel, dim3(grid1d(n)), dim3(256), 0, st, a.part, p.Z, n, dw);
  if (db)
    hipLaunchKernelGGL(ordered_sum_kernel, dim3(1), dim3(256), 0, st, a.bpart, nph * p.Z,
                       (long long)g0.CO, db);
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
  if (dtype == SPECENH_DTYPE_F32) return launch_fwd<float>(a, nph, st);
  if (dtype == SPECENH_DTYPE_BF16) return launch_fwd<__bf16>(a, nph, st);
  return launch_fwd<_Float16>(a, nph, st);
}

size_t specenh_conv2d_wgrad_workspace_bytes(int N, int OH, int OW, int KH, int KW, int C,
                                            int CO) {
  if (N <= 0 || OH <= 0 || OW <= 0 || KH <= 0 || KW <= 0 || C <= 0 || CO <= 0) return 0;
  const WgradPlan p = wgrad_plan(KH * KW * C, CO);
  return ((size_t)p.Z * CO * KH * KW * C + (size_t)MAXPH * p.Z * CO) * sizeof(float);
}

int specenh_conv2d_wgrad(int dtype, const void* in, int N, int IH, int IW, int C, const void* dout,
                         int KH, int KW, int CO, int stride, int pad_t, int pad_l, int in_dil,
                         int OH, int OW, float* dw, float* dbias, void* workspace, void* stream) {
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
  a.part = (float*)workspace;
  a.bpart = dbias ? a.part + (size_t)p.Z * CO * KH * KW * C : nullptr;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == SPECENH_DTYPE_F32) return launch_wgrad<float>(a, nph, dw, dbias, st);
  if (dtype == SPECENH_DTYPE_BF16) return launch_wgrad<__bf16>(a, nph, dw, dbias, st);
  return launch_wgrad<_Float16>(a, nph, dw, dbias, st);
}

int specenh_maxpool2_fwd(int dtype, const void* in, int N, int H, int W, int C, void* out,
                         unsigned char* argmax, void* stream) {
  if (N <= 0 || H <= 0 || W <= 0 || C <= 0 || (H & 1) || (W & 1))
    return set_error(SPECENH_EINVAL, "maxpool2 needs even H, W");
  if (!in || !out) return set_error(SPECENH_EINVAL, "null pointer");
  const long long n = (long long)N * (H / 2) * (W / 2) * C;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == 0)
    hipLaunchKernelGGL(maxpool2_fwd_kernel<float>, dim3(grid1d(n)), dim3(256), 0, st,
                       (const float*)in, N, H, W, C, (float*)out, argmax);
  else if (dtype == 1)
    hipLaunchKernelGGL(maxpool2_fwd_kernel<__bf16>, dim3(grid1d(n)), dim3(256), 0, st,
                       (const __bf16*)in, N, H, W, C, (__bf16*)out, argmax);
  else if (dtype == 2)
    hipLaunchKernelGGL(maxpool2_fwd_kernel<_Float16>, dim3(grid1d(n)), dim3(256), 0, st,
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
    hipLaunchKernelGGL(maxpool2_bwd_kernel<float>, dim3(grid1d(n)), dim3(256), 0, st,
                       (const float*)dout, argmax, (const float*)pooled, N, H, W, C, (float*)din);
  else if (dtype == 1)
    hipLaunchKernelGGL(maxpool2_bwd_kernel<__bf16>, dim3(grid1d(n)), dim3(256), 0, st,
                       (const __bf16*)dout, argmax, (const __bf16*)pooled, N, H, W, C,
                       (__bf16*)din);
  else if (dtype == 2)
    hipLaunchKernelGGL(maxpool2_bwd_kernel<_Float16>, dim3(grid1d(n)), dim3(256), 0, st,
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
  const unsigned gx = std::min<unsigned>(grid1d(n), 1024);
#define SPECENH_BCE(TT, TG)                                                                   \
  hipLaunchKernelGGL((bce_logits_kernel<TT, TG>), dim3(gx), dim3(256), 0, st, z,             \
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
    hipLaunchKernelGGL(adam_kernel<_Float16>, dim3(grid1d(n)), dim3(256), 0, st, w, g, m, v, n,
                       lr_t, b1, b2, eps, grad_scale, (_Float16*)w_lowp);
  else if (lowp_dtype == SPECENH_DTYPE_BF16 || !w_lowp)
    hipLaunchKernelGGL(adam_kernel<__bf16>, dim3(grid1d(n)), dim3(256), 0, st, w, g, m, v, n,
                       lr_t, b1, b2, eps, grad_scale, (__bf16*)w_lowp);
  else
    return set_error(SPECENH_EINVAL, "adam: low-precision copy must be bf16 or f16");
  return hipGetLastError() == hipSuccess ? SPECENH_OK : set_error(SPECENH_EHIP, "adam");
}

int specenh_weight_flip_transpose(int dtype, const void* bt, int k, int ci, int co, void* bd,
                                  void* stream) {
  const long long n = (long long)k * k * ci * co;
  if (!bt || !bd || n <= 0) return set_error(SPECENH_EINVAL, "flip args");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == 0)
    hipLaunchKernelGGL(flip_transpose_kernel<float>, dim3(grid1d(n)), dim3(256), 0, st,
                       (const float*)bt, k, ci, co, (float*)bd);
  else if (dtype == 1)
    hipLaunchKernelGGL(flip_transpose_kernel<__bf16>, dim3(grid1d(n)), dim3(256), 0, st,
                       (const __bf16*)bt, k, ci, co, (__bf16*)bd);
  else if (dtype == 2)
    hipLaunchKernelGGL(flip_transpose_kernel<_Float16>, dim3(grid1d(n)), dim3(256), 0, st,
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
  hipLaunchKernelGGL((cast_kernel<TS, TD>), g, b, 0, st, (const TS*)src, (TD*)dst, n)
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
