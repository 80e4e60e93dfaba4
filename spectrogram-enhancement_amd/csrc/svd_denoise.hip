// svd_denoise.hip — batched SVD low-rank denoiser for gfx950.
//
// Replaces spec_denoising/denoising_by_svd.ipynb:188-229 (denoiseSignal):
//   u, s, vh = np.linalg.svd(A, full_matrices=False)
//   out = u[:, start:stop] @ diag(s[start:stop]) @ vh[start:stop, :]
// for a batch of matrices. Identity used: s_i u_i v_i^T = A v_i v_i^T, so
//   out = A * (V_sel V_sel^T)                       (m >= n, V right singular vectors)
//   out = (U_sel U_sel^T) * A                       (m <  n, U left singular vectors)
// and with V_K = the top-K vectors:
//   [start, stop) with stop <  r : out = A V_stop V_stop^T - A V_start V_start^T
//   [start, stop) with stop == r : out = A - A V_start V_start^T      (e.g. the default 1..r)
// so only a top-K subspace of the Gram matrix is ever needed (K = stop or start).
//
// Pipeline (all HIP, one stream):
//   1. gram_kernel     G = X^T X per matrix, X = A (m>=n) or A^T (m<n); fp32 MFMA
//                      v_mfma_f32_32x32x2_f32 (bit-exact fp32 FMA chains), 32x32 tile per wave.
//   2. subspace_kernel one workgroup per matrix: Y = G*Omega, then q rounds of
//                      {CholeskyQR2 in fp64, Y = G*Z}; Rayleigh-Ritz H = Z^T G Z;
//                      cyclic Jacobi on H (one wave); V = Z*Q sorted by Ritz value.
//   3. recon_kernel    out = X P or X - X P with P = V_K V_K^T restricted to the selected
//                      columns (written back in A's orientation).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <string>
#include <vector>

#include "fft_common.hpp"
#include "specenh.h"
#include "runtime.hpp"

namespace specenh {
int set_error(int code, const std::string& msg);  // stft_psd.hip

typedef float f32x16 __attribute__((ext_vector_type(16)));

// Element (k, i) of X for matrix b: X = A (k = row, i = col) or X = A^T.
struct XView {
  const float* base;
  long long batch_stride;
  long long sk, si;  // strides of k and i
};

// ---------------------------------------------------------------- 1. Gram
// Each wave computes one 32x32 tile (ti <= tj) of G = X^T X over K rows of X.
// MFMA 32x32x2 f32: lane l supplies A[i = l&31][k = l>>5] and B[k = l>>5][j = l&31];
// D[row][col] with col = l&31, row = (reg&3) + 8*(reg>>2) + 4*(l>>5).
__global__ __launch_bounds__(256) void gram_kernel(XView x, int K, int r, float* G,
                                                   int ntiles_side) {
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int ntri = ntiles_side * (ntiles_side + 1) / 2;
  const int t = blockIdx.x * 4 + wave;
  if (t >= ntri) return;  // wave-uniform
  // t -> (ti, tj), ti <= tj, row-major over the upper triangle
  int ti = 0, rem = t;
  while (rem >= ntiles_side - ti) {
    rem -= ntiles_side - ti;
    ++ti;
  }
  const int tj = ti + rem;
  const long long b = blockIdx.y;
  const float* X = x.base + b * x.batch_stride;
  const int ci = ti * 32 + (lane & 31), cj = tj * 32 + (lane & 31);
  const int kh = lane >> 5;
  const bool vi = ci < r, vj = cj < r;
  const float* pi = X + (vi ? ci : 0) * x.si + kh * x.sk;
  const float* pj = X + (vj ? cj : 0) * x.si + kh * x.sk;
  f32x16 acc = {};
  int k = 0;
  for (; k + 2 <= K; k += 2) {
    const float a = vi ? pi[(long long)k * x.sk] : 0.f;
    const float bb = vj ? pj[(long long)k * x.sk] : 0.f;
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bb, acc, 0, 0, 0);
  }
  if (k < K) {  // odd K: last row paired with a zero row
    const float a = (vi && kh == 0) ? pi[(long long)k * x.sk] : 0.f;
    const float bb = (vj && kh == 0) ? pj[(long long)k * x.sk] : 0.f;
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bb, acc, 0, 0, 0);
  }
  float* Gb = G + b * (long long)r * r;
#pragma unroll
  for (int reg = 0; reg < 16; ++reg) {
    const int row = ti * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5);
    const int col = tj * 32 + (lane & 31);
    if (row < r && col < r) {
      Gb[(long long)row * r + col] = acc[reg];
      Gb[(long long)col * r + row] = acc[reg];
    }
  }
}

// r <= 128: one workgroup per matrix. X is staged through LDS in chunks of 32 rows
// (coalesced 16-byte loads, the next chunk in registers while the current one is used);
// the upper triangle of 16x16 tiles (36 at r = 128) is dealt round-robin to the 4 waves,
// v_mfma_f32_16x16x4_f32 reads both operands from the chunk (ds_read_b32, row pitch
// r + 16 words: conflict-free). Same fp32 products as gram_kernel, in another order.
constexpr int GL_KC = 32;
__global__ __launch_bounds__(256) void gram_lds_kernel(XView x, int K, int r, float* G) {
  __shared__ float sX[GL_KC * (128 + 16)];
  const int ld = r + 16;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const float* X = x.base + (long long)blockIdx.x * x.batch_stride;
  const int nt = (r + 15) / 16, ntri = nt * (nt + 1) / 2;
  typedef float f32x4v __attribute__((ext_vector_type(4)));
  f32x4v acc[9];
  int tI[9], tJ[9];
#pragma unroll
  for (int q = 0; q < 9; ++q) {
    acc[q] = f32x4v{0.f, 0.f, 0.f, 0.f};
    int t = wave + 4 * q, ti = 0;
    if (t >= ntri) t = -1;
    if (t >= 0) {
      while (t >= nt - ti) { t -= nt - ti; ++ti; }
      tI[q] = ti; tJ[q] = ti + t;
    } else {
      tI[q] = -1; tJ[q] = -1;
    }
  }
  // staging: GL_KC x r elements; row-major X (si == 1): float4 along i, else along k
  const bool rowmaj = x.si == 1;
  const int nvec = GL_KC * r / 4;  // r % 4 == 0 (host-checked)
  float4 reg[4];
  auto fetch = [&](int k0) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = tid + 256 * u;
      reg[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (e < nvec) {
        if (rowmaj) {
          const int kk = e / (r / 4), i4 = e - (e / (r / 4)) * (r / 4);
          if (k0 + kk < K)
            reg[u] = *reinterpret_cast<const float4*>(X + (long long)(k0 + kk) * x.sk + 4 * i4);
        } else {  // X[k][i] = base[k + i * si]: 4 consecutive k of one column i
          const int i = e / (GL_KC / 4), k4 = e - (e / (GL_KC / 4)) * (GL_KC / 4);
          const float* src = X + (long long)i * x.si + k0 + 4 * k4;
          if (k0 + 4 * k4 + 3 < K) {
            reg[u] = make_float4(src[0], src[1], src[2], src[3]);
          } else {
            float v[4] = {0.f, 0.f, 0.f, 0.f};
            for (int c = 0; c < 4; ++c)
              if (k0 + 4 * k4 + c < K) v[c] = src[c];
            reg[u] = make_float4(v[0], v[1], v[2], v[3]);
          }
        }
      }
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = tid + 256 * u;
      if (e >= nvec) continue;
      if (rowmaj) {
        const int kk = e / (r / 4), i4 = e - (e / (r / 4)) * (r / 4);
        *reinterpret_cast<float4*>(sX + kk * ld + 4 * i4) = reg[u];
      } else {
        const int i = e / (GL_KC / 4), k4 = e - (e / (GL_KC / 4)) * (GL_KC / 4);
        sX[(4 * k4 + 0) * ld + i] = reg[u].x;
        sX[(4 * k4 + 1) * ld + i] = reg[u].y;
        sX[(4 * k4 + 2) * ld + i] = reg[u].z;
        sX[(4 * k4 + 3) * ld + i] = reg[u].w;
      }
    }
  };
  // columns r .. 16*nt - 1 of the chunk stay zero
  for (int e = tid; e < GL_KC * (16 * nt - r); e += 256) {
    const int kk = e / (16 * nt - r), i = r + e - kk * (16 * nt - r);
    sX[kk * ld + i] = 0.f;
  }
  fetch(0);
  const int kr = lane >> 4, cl = lane & 15;
  for (int k0 = 0; k0 < K; k0 += GL_KC) {
    __syncthreads();  // previous chunk fully consumed
    store();
    __syncthreads();
    if (k0 + GL_KC < K) fetch(k0 + GL_KC);
#pragma unroll
    for (int s4 = 0; s4 < GL_KC / 4; ++s4) {
      const float* row = sX + (4 * s4 + kr) * ld + cl;
#pragma unroll
      for (int q = 0; q < 9; ++q) {
        if (tI[q] < 0) continue;  // wave-uniform
        const float a = row[16 * tI[q]], b = row[16 * tJ[q]];
        acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[q], 0, 0, 0);
      }
    }
  }
  float* Gb = G + (long long)blockIdx.x * r * r;
#pragma unroll
  for (int q = 0; q < 9; ++q) {
    if (tI[q] < 0) continue;
#pragma unroll
    for (int reg4 = 0; reg4 < 4; ++reg4) {
      const int row = 16 * tI[q] + 4 * kr + reg4, col = 16 * tJ[q] + cl;
      if (row < r && col < r) {
        Gb[(long long)row * r + col] = acc[q][reg4];
        Gb[(long long)col * r + row] = acc[q][reg4];
      }
    }
  }
}

// 128 < r <= 256 (r % 4 == 0; C3: 513 x 256): one workgroup of 4 waves per matrix, X read
// from HBM once. gram_kernel (one wave per 32x32 tile, operands straight from global) read
// every X element 9 times, 5.5x the input from HBM by PMC (11.9 GB per 4096 C3 matrices).
// Here X is staged through LDS in chunks of G2_KC rows (the next chunk in registers while
// the current one is used; row pitch G2_LD = 288 words: the two half-waves' rows land 32
// banks apart); the 36 upper-triangle 32x32 tiles of G go 9 to each wave. Per pair of rows a
// wave reads the 8 column-panel fragments once: tile (ti, tj) takes fragment ti as the MFMA's
// A operand and fragment tj as its B operand (same v_mfma_f32_32x32x2_f32 as gram_kernel,
// whose lane layout is documented there), so 8 LDS reads feed 9 MFMAs. Columns r .. 255 of
// the chunk stay zero; rows past K are fetched as zeros (exact +0 products).
constexpr int G2_KC = 16, G2_LD = 288;
// row-major upper triangle of the 8 x 8 tile grid: tile t -> (ti, tj)
__device__ constexpr int kG2TI[36] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 1, 1, 1, 2, 2, 2,
                                      2, 2, 2, 3, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 6, 6, 7};
__device__ constexpr int kG2TJ[36] = {0, 1, 2, 3, 4, 5, 6, 7, 1, 2, 3, 4, 5, 6, 7, 2, 3, 4,
                                      5, 6, 7, 3, 4, 5, 6, 7, 4, 5, 6, 7, 5, 6, 7, 6, 7, 7};

template <int W>  // the wave's tiles are W, W + 4, ..., W + 32: compile-time panel indices
__device__ __forceinline__ void gram256_wave(const XView& x, int K, int r, float* sX,
                                             float* Gb) {
  const int tid = threadIdx.x, lane = tid & 63;
  const float* X = x.base + (long long)blockIdx.x * x.batch_stride;
  const bool rowmaj = x.si == 1;
  const int nvec = G2_KC * r / 4;
  constexpr int NV = G2_KC * 256 / 4 / 256;  // float4 per thread per chunk (r = 256)
  float4 reg[NV];
  auto fetch = [&](int k0) {
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      const int e = tid + 256 * u;
      reg[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (e < nvec) {
        if (rowmaj) {
          const int kk = e / (r / 4), i4 = e - kk * (r / 4);
          if (k0 + kk < K)
            reg[u] = *reinterpret_cast<const float4*>(X + (long long)(k0 + kk) * x.sk + 4 * i4);
        } else {  // X[k][i] = base[k + i * si]: 4 consecutive k of one column i
          const int i = e / (G2_KC / 4), k4 = e - i * (G2_KC / 4);
          const float* src = X + (long long)i * x.si + k0 + 4 * k4;
          float v[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int c = 0; c < 4; ++c)
            if (k0 + 4 * k4 + c < K) v[c] = src[c];
          reg[u] = make_float4(v[0], v[1], v[2], v[3]);
        }
      }
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      const int e = tid + 256 * u;
      if (e >= nvec) continue;
      if (rowmaj) {
        const int kk = e / (r / 4), i4 = e - kk * (r / 4);
        *reinterpret_cast<float4*>(sX + kk * G2_LD + 4 * i4) = reg[u];
      } else {
        const int i = e / (G2_KC / 4), k4 = e - i * (G2_KC / 4);
        sX[(4 * k4 + 0) * G2_LD + i] = reg[u].x;
        sX[(4 * k4 + 1) * G2_LD + i] = reg[u].y;
        sX[(4 * k4 + 2) * G2_LD + i] = reg[u].z;
        sX[(4 * k4 + 3) * G2_LD + i] = reg[u].w;
      }
    }
  };
  f32x16 acc[9];
#pragma unroll
  for (int q = 0; q < 9; ++q) acc[q] = f32x16{};
  const int c = lane & 31, kh = lane >> 5;
  fetch(0);
  for (int k0 = 0; k0 < K; k0 += G2_KC) {
    __syncthreads();  // previous chunk fully consumed
    store();
    __syncthreads();
    if (k0 + G2_KC < K) fetch(k0 + G2_KC);
#pragma unroll 4
    for (int s2 = 0; s2 < G2_KC / 2; ++s2) {
      const float* row = sX + (2 * s2 + kh) * G2_LD + c;
      float f[8];
#pragma unroll
      for (int p = 0; p < 8; ++p) f[p] = row[32 * p];
#pragma unroll
      for (int q = 0; q < 9; ++q)
        acc[q] = __builtin_amdgcn_mfma_f32_32x32x2f32(f[kG2TI[W + 4 * q]], f[kG2TJ[W + 4 * q]],
                                                      acc[q], 0, 0, 0);
    }
  }
#pragma unroll
  for (int q = 0; q < 9; ++q) {
    const int ti = kG2TI[W + 4 * q], tj = kG2TJ[W + 4 * q];
#pragma unroll
    for (int reg16 = 0; reg16 < 16; ++reg16) {
      const int row = ti * 32 + (reg16 & 3) + 8 * (reg16 >> 2) + 4 * kh;
      const int col = tj * 32 + c;
      if (row < r && col < r) {
        Gb[(long long)row * r + col] = acc[q][reg16];
        Gb[(long long)col * r + row] = acc[q][reg16];
      }
    }
  }
}

__global__ __launch_bounds__(256, 2) void gram256_kernel(XView x, int K, int r, float* G) {
  __shared__ __attribute__((aligned(16))) float sX[G2_KC * G2_LD];
  // columns r .. 255 stay zero (the stores only write i < r)
  for (int e = threadIdx.x; e < G2_KC * (256 - r); e += 256) {
    const int kk = e / (256 - r), i = r + e - kk * (256 - r);
    sX[kk * G2_LD + i] = 0.f;
  }
  float* Gb = G + (long long)blockIdx.x * r * r;
  switch (threadIdx.x >> 6) {
    case 0: gram256_wave<0>(x, K, r, sX, Gb); break;
    case 1: gram256_wave<1>(x, K, r, sX, Gb); break;
    case 2: gram256_wave<2>(x, K, r, sX, Gb); break;
    default: gram256_wave<3>(x, K, r, sX, Gb); break;
  }
}

// 128 < r <= 256, on the fp16 matrix cores. gram256_kernel runs at ~0.5 of the fp32 MFMA
// peak (1.9 ms per 4096 C3 matrices, 7x the HBM time of reading X). Here every element is
// split as 2^e x = hi + lo, two fp16 numbers (hi = fp16(2^e x), lo = fp16(2^e x - hi): 22
// significant bits, the residual below 2^-22 |x|), and each 32x32 tile of G takes three
// v_mfma_f32_32x32x16_f16 products per 16 rows, hi^T hi + hi^T lo + lo^T hi (the dropped
// lo^T lo is below 2^-22 of the product), fp32 accumulation: the products' error is ~20x
// below the fp32 Gram's own rounding (tools/gram_split_sim.py), at 16x the fp32 MFMA rate.
// Scale: e is one per matrix, the running minimum of 15 - exponent(chunk max |x|), so every
// scaled value stays below 2^15 (fp16 max 65504); when a chunk lowers e, the accumulators are
// rescaled by 2^(2 de) (exact), and G = acc * 2^-2e at the end. Chunk = GS_KC = 16 rows of X:
// thread t stages column t (16 values; rows past K and columns past r are zero), its wave's
// max goes to LDS before the barrier that precedes the chunk's conversion, so the scale costs
// no extra barrier. LDS holds hi and lo as [k-half][column][8 halves]: lane l's MFMA operand
// for column panel p (A[i][k] = X[k][32p + i], B[k][j] = X[k][32p + j], the same fragment)
// is one ds_read_b128 at [l >> 5][32p + (l & 31)], and the staging writes are 16 B per thread
// at consecutive addresses (both conflict-free). Tiles: with panels A = 0..3 and B = 4..7,
// wave 0 takes A x A (10 upper-triangle tiles), wave 1 B x B (10), waves 2 and 3 {0,1} x B
// and {2,3} x B (8 each), so a wave holds 4 or 6 panels' fragments (32 / 48 VGPRs) instead
// of all 8 (64: the 9-per-wave deal spilled at two waves per SIMD).
constexpr int GS_KC = 16;
__device__ constexpr int kGSTI[4][10] = {{0, 0, 0, 0, 1, 1, 1, 2, 2, 3},
                                         {4, 4, 4, 4, 5, 5, 5, 6, 6, 7},
                                         {0, 0, 0, 0, 1, 1, 1, 1, 0, 0},
                                         {2, 2, 2, 2, 3, 3, 3, 3, 0, 0}};
__device__ constexpr int kGSTJ[4][10] = {{0, 1, 2, 3, 1, 2, 3, 2, 3, 3},
                                         {4, 5, 6, 7, 5, 6, 7, 6, 7, 7},
                                         {4, 5, 6, 7, 4, 5, 6, 7, 0, 0},
                                         {4, 5, 6, 7, 4, 5, 6, 7, 0, 0}};
typedef _Float16 gs_f16x8 __attribute__((ext_vector_type(8)));
typedef float gs_f32x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ float wave_max64(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

template <int W>  // NT = tiles of this wave
__device__ __forceinline__ void gram256s_wave(const XView& x, int K, int r, gs_f16x8* sH,
                                              gs_f16x8* sL, float* sMax, float* Gb) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float* X = x.base + (long long)blockIdx.x * x.batch_stride;
  const bool rowmaj = x.si == 1;
  const bool vec4 = !rowmaj && x.sk == 1 && (x.si & 3) == 0 && (x.batch_stride & 3) == 0 &&
                    (reinterpret_cast<uintptr_t>(x.base) & 15) == 0;
  const bool col_ok = tid < r;
  const float* pc = X + (long long)(col_ok ? tid : 0) * x.si;
  float v[GS_KC];
  auto fetch = [&](int k0) {
    if (!col_ok) {
#pragma unroll
      for (int kk = 0; kk < GS_KC; ++kk) v[kk] = 0.f;
      return;
    }
    const float* p = pc + (long long)k0 * x.sk;
    if (k0 + GS_KC <= K) {
      if (vec4) {
#pragma unroll
        for (int u = 0; u < GS_KC / 4; ++u) {
          const float4 q = *reinterpret_cast<const float4*>(p + 4 * u);
          v[4 * u] = q.x; v[4 * u + 1] = q.y; v[4 * u + 2] = q.z; v[4 * u + 3] = q.w;
        }
      } else {
#pragma unroll
        for (int kk = 0; kk < GS_KC; ++kk) v[kk] = p[(long long)kk * x.sk];
      }
    } else {
#pragma unroll
      for (int kk = 0; kk < GS_KC; ++kk) v[kk] = k0 + kk < K ? p[(long long)kk * x.sk] : 0.f;
    }
  };
  auto post_max = [&]() {
    float m = 0.f;
#pragma unroll
    for (int kk = 0; kk < GS_KC; ++kk) m = fmaxf(m, fabsf(v[kk]));
    m = wave_max64(m);
    if (lane == 0) sMax[wave] = m;
  };
  constexpr int NT = W < 2 ? 10 : 8;
  f32x16 acc[NT];
#pragma unroll
  for (int q = 0; q < NT; ++q) acc[q] = f32x16{};
  int e_run = 110;  // lowered by the first chunk with a nonzero finite max
  const int c = lane & 31, kh = lane >> 5;
  fetch(0);
  post_max();
  for (int k0 = 0; k0 < K; k0 += GS_KC) {
    __syncthreads();  // previous chunk consumed; the chunk's wave maxima visible
    {
      const float4 mw = *reinterpret_cast<const float4*>(sMax);
      const float M = fmaxf(fmaxf(mw.x, mw.y), fmaxf(mw.z, mw.w));
      if (M > 0.f && M <= 3.0e38f) {  // (Inf / NaN chunks keep the scale)
        const int et = 15 - __builtin_amdgcn_frexp_expf(M);  // M * 2^et in [2^14, 2^15)
        if (et < e_run) {  // wave-uniform
          const int d = 2 * (max(et, -110) - e_run);
#pragma unroll
          for (int q = 0; q < NT; ++q)
#pragma unroll
            for (int j = 0; j < 16; ++j) acc[q][j] = __builtin_ldexpf(acc[q][j], d);
          e_run = max(et, -110);
        }
      }
      gs_f32x8 y0, y1;
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) {
        y0[kk] = __builtin_ldexpf(v[kk], e_run);
        y1[kk] = __builtin_ldexpf(v[8 + kk], e_run);
      }
      const gs_f16x8 h0 = __builtin_convertvector(y0, gs_f16x8);
      const gs_f16x8 h1 = __builtin_convertvector(y1, gs_f16x8);
      const gs_f16x8 l0 = __builtin_convertvector(y0 - __builtin_convertvector(h0, gs_f32x8), gs_f16x8);
      const gs_f16x8 l1 = __builtin_convertvector(y1 - __builtin_convertvector(h1, gs_f32x8), gs_f16x8);
      sH[tid] = h0;
      sH[256 + tid] = h1;
      sL[tid] = l0;
      sL[256 + tid] = l1;
    }
    __syncthreads();  // chunk visible; sMax read by every wave
    const bool more = k0 + GS_KC < K;
    if (more) fetch(k0 + GS_KC);
    gs_f16x8 fh[8], fl[8];
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      fh[p] = sH[256 * kh + 32 * p + c];
      fl[p] = sL[256 * kh + 32 * p + c];
    }
#pragma unroll
    for (int q = 0; q < NT; ++q)
      acc[q] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fh[kGSTI[W][q]], fh[kGSTJ[W][q]],
                                                      acc[q], 0, 0, 0);
#pragma unroll
    for (int q = 0; q < NT; ++q)
      acc[q] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fh[kGSTI[W][q]], fl[kGSTJ[W][q]],
                                                      acc[q], 0, 0, 0);
#pragma unroll
    for (int q = 0; q < NT; ++q)
      acc[q] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fl[kGSTI[W][q]], fh[kGSTJ[W][q]],
                                                      acc[q], 0, 0, 0);
    if (more) post_max();  // (after the MFMAs: the loads had their time to land)
  }
  // D[row][col]: col = c, rows 4 kh + (reg & 3) + 8 (reg >> 2). The mirrored tile is stored as
  // float4 runs: regs 4g .. 4g + 3 of a lane are four consecutive rows = four consecutive
  // columns of G's row `col` (4 wide stores per tile instead of 16 single-word scatters).
  const int ex = -2 * e_run;
#pragma unroll
  for (int q = 0; q < NT; ++q) {
    const int ti = kGSTI[W][q], tj = kGSTJ[W][q];
    const int col = tj * 32 + c;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int row0 = ti * 32 + 8 * g + 4 * kh;
      float4 o;
      o.x = __builtin_ldexpf(acc[q][4 * g], ex);
      o.y = __builtin_ldexpf(acc[q][4 * g + 1], ex);
      o.z = __builtin_ldexpf(acc[q][4 * g + 2], ex);
      o.w = __builtin_ldexpf(acc[q][4 * g + 3], ex);
      if (col < r) {
        if (row0 + 3 < r && (r & 3) == 0) {
          *reinterpret_cast<float4*>(Gb + (long long)col * r + row0) = o;
        } else {
          if (row0 < r) Gb[(long long)col * r + row0] = o.x;
          if (row0 + 1 < r) Gb[(long long)col * r + row0 + 1] = o.y;
          if (row0 + 2 < r) Gb[(long long)col * r + row0 + 2] = o.z;
          if (row0 + 3 < r) Gb[(long long)col * r + row0 + 3] = o.w;
        }
        if (ti != tj) {
          if (row0 < r) Gb[(long long)row0 * r + col] = o.x;
          if (row0 + 1 < r) Gb[(long long)(row0 + 1) * r + col] = o.y;
          if (row0 + 2 < r) Gb[(long long)(row0 + 2) * r + col] = o.z;
          if (row0 + 3 < r) Gb[(long long)(row0 + 3) * r + col] = o.w;
        }
      }
    }
  }
}

__global__ __launch_bounds__(256, 2) void gram256s_kernel(XView x, int K, int r, float* G) {
  __shared__ __attribute__((aligned(16))) gs_f16x8 sH[2 * 256];
  __shared__ __attribute__((aligned(16))) gs_f16x8 sL[2 * 256];
  __shared__ __attribute__((aligned(16))) float sMax[4];
  float* Gb = G + (long long)blockIdx.x * r * r;
  switch (threadIdx.x >> 6) {
    case 0: gram256s_wave<0>(x, K, r, sH, sL, sMax, Gb); break;
    case 1: gram256s_wave<1>(x, K, r, sH, sL, sMax, Gb); break;
    case 2: gram256s_wave<2>(x, K, r, sH, sL, sMax, Gb); break;
    default: gram256s_wave<3>(x, K, r, sH, sL, sMax, Gb); break;
  }
}

// ---------------------------------------------------------------- 2. subspace
constexpr int SS_THREADS = 256;
#ifndef SPECENH_SS_SINGLE_QR
#define SPECENH_SS_SINGLE_QR 1  // single CholeskyQR in the intermediate subspace rounds
#endif
constexpr int PMAX = 48;  // max subspace width (LDS: r=256 -> 2 x 48 KB + tables)

// deterministic pseudo-random start vectors
__device__ __forceinline__ float hash_unit(unsigned i, unsigned j) {
  unsigned h = i * 0x9E3779B1u ^ (j + 0x7F4A7C15u) * 0x85EBCA77u;
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  h ^= h >> 12;
  h *= 0x297A2D39u;
  h ^= h >> 15;
  return (float)(h & 0xFFFFFF) * (1.0f / 16777216.0f) - 0.5f;
}

#ifndef SPECENH_GZ_GB
#define SPECENH_GZ_GB 8
#endif

// Y = G Z for symmetric G (global, r x r) and Z (LDS, r x P): Y[i][:] = sum_j G[j][i] Z[j][:].
// One row i per thread; at each j the threads read row j of G coalesced and Z[j][:] is an
// LDS broadcast.
template <int P>
__device__ __forceinline__ void gemm_GZ(const float* G, int r, const float* sZ, float* sY) {
  for (int i = threadIdx.x; i < r; i += SS_THREADS) {
    float acc[P];
#pragma unroll
    for (int c = 0; c < P; ++c) acc[c] = 0.f;
    // G rows in batches of GB loads in flight (G comes from L2 / HBM: one batch per round
    // trip), then the batch's FMAs in the same j order
    // G loads per batch: 8 for P <= 24 (C3 rank-16 5.05 -> 4.84 ms vs 16; 32: 6.2 ms, 64:
    // slower still — more rows in flight per thread congest L2 / the memory pipeline)
    constexpr int GB = P <= 24 ? SPECENH_GZ_GB : 16;
    const int nb = r / GB;
    for (int q = 0; q < nb; ++q) {
      const int j = GB * q;
      float g[GB];
#pragma unroll
      for (int u = 0; u < GB; ++u) g[u] = G[(long long)(j + u) * r + i];
#pragma unroll
      for (int u = 0; u < GB; ++u) {
        const float4* zj = reinterpret_cast<const float4*>(sZ + (j + u) * P);
#pragma unroll
        for (int c4 = 0; c4 < P / 4; ++c4) {
          const float4 z = zj[c4];
          acc[4 * c4 + 0] = fmaf(g[u], z.x, acc[4 * c4 + 0]);
          acc[4 * c4 + 1] = fmaf(g[u], z.y, acc[4 * c4 + 1]);
          acc[4 * c4 + 2] = fmaf(g[u], z.z, acc[4 * c4 + 2]);
          acc[4 * c4 + 3] = fmaf(g[u], z.w, acc[4 * c4 + 3]);
        }
      }
    }
    for (int j = nb * GB; j < r; ++j) {
      const float g = G[(long long)j * r + i];
      const float4* zj = reinterpret_cast<const float4*>(sZ + j * P);
#pragma unroll
      for (int c4 = 0; c4 < P / 4; ++c4) {
        const float4 z = zj[c4];
        acc[4 * c4 + 0] = fmaf(g, z.x, acc[4 * c4 + 0]);
        acc[4 * c4 + 1] = fmaf(g, z.y, acc[4 * c4 + 1]);
        acc[4 * c4 + 2] = fmaf(g, z.z, acc[4 * c4 + 2]);
        acc[4 * c4 + 3] = fmaf(g, z.w, acc[4 * c4 + 3]);
      }
    }
    float4* yi = reinterpret_cast<float4*>(sY + i * P);
#pragma unroll
    for (int c4 = 0; c4 < P / 4; ++c4)
      yi[c4] = make_float4(acc[4 * c4], acc[4 * c4 + 1], acc[4 * c4 + 2], acc[4 * c4 + 3]);
  }
}

// Y = G Z with FOUR rows per thread (r % 4 == 0, G 16-byte aligned): thread (quad q = lane,
// wave w) takes rows 4q .. 4q + 3 of Y over the w-th quarter of the j range, so one
// float4 load per lane moves a whole 1 KB row of G per wave instruction (gemm_GZ's dword
// loads move 256 B) and each broadcast Z[j] read feeds 4 P FMAs instead of P. The four
// quarter sums meet in sY in wave order (fixed: the result does not depend on timing).
// C3 rank-16 5.11 -> 4.48 ms, default 3.40 -> 3.22 ms (profiles/r05_svd_ab_gzquad.txt);
// SVD_GZ_ROWS=1 keeps one row per thread.
template <int P>
__device__ __forceinline__ void gemm_GZ4(const float* G, int r, const float* sZ, float* sY) {
  constexpr int GB = 8;  // float4 loads in flight per batch
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int nq = r >> 2, jq = (r + 3) >> 2;
  const int j0 = min(r, w * jq), j1 = min(r, j0 + jq);
  const float4* __restrict__ G4 = reinterpret_cast<const float4*>(G);
  for (int base = 0; base < nq; base += 64) {  // uniform trip count (barriers inside)
    const int qd = base + lane;
    const bool act = qd < nq;
    const int qc = act ? qd : 0;  // inactive lanes load a valid row and discard it
    float acc[4][P];
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int c = 0; c < P; ++c) acc[k][c] = 0.f;
    int j = j0;
    for (; j + GB <= j1; j += GB) {
      float4 g[GB];
#pragma unroll
      for (int u = 0; u < GB; ++u) g[u] = G4[(long long)(j + u) * nq + qc];
#pragma unroll
      for (int u = 0; u < GB; ++u) {
        const float4* zj = reinterpret_cast<const float4*>(sZ + (j + u) * P);
        const float gv[4] = {g[u].x, g[u].y, g[u].z, g[u].w};
#pragma unroll
        for (int c4 = 0; c4 < P / 4; ++c4) {
          const float4 z = zj[c4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            acc[k][4 * c4 + 0] = fmaf(gv[k], z.x, acc[k][4 * c4 + 0]);
            acc[k][4 * c4 + 1] = fmaf(gv[k], z.y, acc[k][4 * c4 + 1]);
            acc[k][4 * c4 + 2] = fmaf(gv[k], z.z, acc[k][4 * c4 + 2]);
            acc[k][4 * c4 + 3] = fmaf(gv[k], z.w, acc[k][4 * c4 + 3]);
          }
        }
      }
    }
    for (; j < j1; ++j) {
      const float4 g = G4[(long long)j * nq + qc];
      const float gv[4] = {g.x, g.y, g.z, g.w};
      const float4* zj = reinterpret_cast<const float4*>(sZ + j * P);
#pragma unroll
      for (int c4 = 0; c4 < P / 4; ++c4) {
        const float4 z = zj[c4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          acc[k][4 * c4 + 0] = fmaf(gv[k], z.x, acc[k][4 * c4 + 0]);
          acc[k][4 * c4 + 1] = fmaf(gv[k], z.y, acc[k][4 * c4 + 1]);
          acc[k][4 * c4 + 2] = fmaf(gv[k], z.z, acc[k][4 * c4 + 2]);
          acc[k][4 * c4 + 3] = fmaf(gv[k], z.w, acc[k][4 * c4 + 3]);
        }
      }
    }
    // quarter sums into sY: wave 0 stores, waves 1, 2, 3 add in turn
#pragma unroll
    for (int s = 0; s < SS_THREADS / 64; ++s) {
      if (w == s && act) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          float4* yi = reinterpret_cast<float4*>(sY + (4 * qd + k) * P);
#pragma unroll
          for (int c4 = 0; c4 < P / 4; ++c4) {
            float4 v = make_float4(acc[k][4 * c4], acc[k][4 * c4 + 1], acc[k][4 * c4 + 2],
                                   acc[k][4 * c4 + 3]);
            if (s > 0) {
              const float4 o = yi[c4];
              v = make_float4(o.x + v.x, o.y + v.y, o.z + v.z, o.w + v.w);
            }
            yi[c4] = v;
          }
        }
      }
      __syncthreads();
    }
  }
}

// P = 8 (the default K = 1 subspace) ------------------------------------------------
// The generic helpers above give each output to one thread, which then walks all r rows:
// latency chains of r dependent LDS reads (cholqr's Gram, Rayleigh-Ritz) or of r/8
// batches of L2 loads (G Z). With P = 8 every thread of the workgroup takes part instead.

// out[a][b] = sum_i A[i][a] B[i][b] in fp64 for all 8 x 8 (a, b). Lane (row i, quarter q)
// forms the 16 products of rows a in {2q, 2q + 1}; the 16 lanes of a quarter sum by
// butterflies, the 4 waves through sPart[4][64]. Ends with the result visible to all.
__device__ void prod8(const float* sA, const float* sB, int r, double* sPart, double* out) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, q = lane >> 4;
  double acc[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) acc[k] = 0.0;
  for (int i = 16 * wave + (lane & 15); i < r; i += 16 * (SS_THREADS / 64)) {
    const float2 a = *reinterpret_cast<const float2*>(sA + i * 8 + 2 * q);
    const float4 b0 = *reinterpret_cast<const float4*>(sB + i * 8);
    const float4 b1 = *reinterpret_cast<const float4*>(sB + i * 8 + 4);
    const float bv[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
    for (int k = 0; k < 16; ++k) acc[k] = fma((double)(k < 8 ? a.x : a.y), (double)bv[k & 7], acc[k]);
  }
#pragma unroll
  for (int m = 1; m < 16; m <<= 1)
#pragma unroll
    for (int k = 0; k < 16; ++k) acc[k] += __shfl_xor(acc[k], m);
  if ((lane & 15) == 0)
#pragma unroll
    for (int k = 0; k < 16; ++k) sPart[wave * 64 + 16 * q + k] = acc[k];
  __syncthreads();
  if (tid < 64) {
    double v = 0.0;
#pragma unroll
    for (int w = 0; w < SS_THREADS / 64; ++w) v += sPart[w * 64 + tid];
    out[tid] = v;
  }
  __syncthreads();
}

// Y = G Z for P = 8: thread (row i, j-half) sums over half of the rows of G with 16 loads
// in flight; the two halves meet in sT (r x 8).
__device__ void gemm_GZ8(const float* G, int r, const float* sZ, float* sY, float* sT) {
  const int tid = threadIdx.x, jh = tid >> 7;
  const int half = (r + 1) / 2, j0 = jh * half, j1 = jh ? r : half;
  for (int i = tid & 127; i < r; i += 128) {
    float acc[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) acc[c] = 0.f;
    const int nb = (j1 - j0) / 16;
    for (int q = 0; q < nb; ++q) {
      const int j = j0 + 16 * q;
      float g[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) g[u] = G[(long long)(j + u) * r + i];
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const float4 z0 = *reinterpret_cast<const float4*>(sZ + (j + u) * 8);
        const float4 z1 = *reinterpret_cast<const float4*>(sZ + (j + u) * 8 + 4);
        acc[0] = fmaf(g[u], z0.x, acc[0]); acc[1] = fmaf(g[u], z0.y, acc[1]);
        acc[2] = fmaf(g[u], z0.z, acc[2]); acc[3] = fmaf(g[u], z0.w, acc[3]);
        acc[4] = fmaf(g[u], z1.x, acc[4]); acc[5] = fmaf(g[u], z1.y, acc[5]);
        acc[6] = fmaf(g[u], z1.z, acc[6]); acc[7] = fmaf(g[u], z1.w, acc[7]);
      }
    }
    for (int j = j0 + 16 * nb; j < j1; ++j) {
      const float gj = G[(long long)j * r + i];
#pragma unroll
      for (int c = 0; c < 8; ++c) acc[c] = fmaf(gj, sZ[j * 8 + c], acc[c]);
    }
    float* dst = jh ? sT : sY;
    *reinterpret_cast<float4*>(dst + i * 8) = make_float4(acc[0], acc[1], acc[2], acc[3]);
    *reinterpret_cast<float4*>(dst + i * 8 + 4) = make_float4(acc[4], acc[5], acc[6], acc[7]);
  }
  __syncthreads();
  for (int idx = tid; idx < r * 8; idx += SS_THREADS) sY[idx] += sT[idx];
  __syncthreads();
}

// out[a][c] = sum_i A[i][a] B[i][c] in fp64 for all P x P (a, c); A, B r x P fp32 in LDS.
// On the fp64 matrix cores: (P rounded up to 16)^2 / 256 tiles of v_mfma_f64_16x16x4_f64,
// dealt to the 4 waves, r / 4 MFMAs each (the fp32 values are exact in fp64, products exact,
// sums in fp64). A per-thread walk over all r rows was a serial chain of r dependent fp64
// adds per entry (the subspace kernel's Rayleigh-Ritz and CholeskyQR Grams). Lane l supplies
// A[i = i0 + (l >> 4)][a = 16 ta + (l & 15)] and B[i][c = 16 tb + (l & 15)]; D holds
// (row (l >> 4) + 4 reg, col l & 15) of the tile. Ends with out visible to all threads.
typedef double f64x4 __attribute__((ext_vector_type(4)));
template <int P>
__device__ __forceinline__ void prodP(const float* sA, const float* sB, int r, double* out) {
  constexpr int NT = (P + 15) / 16;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m = lane & 15, kq = lane >> 4;
  for (int t = wave; t < NT * NT; t += SS_THREADS / 64) {  // wave-uniform
    const int ta = t / NT, tb = t % NT;
    const int a = 16 * ta + m, c = 16 * tb + m;
    // 16 rows per iteration into two accumulators, every read of an iteration (and, with
    // the unroll, of the next) issued ahead of its MFMAs: the one-accumulator loop was a
    // chain of r / 4 LDS reads -> convert -> MFMA round trips (~24 k clocks per Gram at
    // r = 256, P = 24; SS_STATS build)
    const bool va = a < P, vb = c < P;
    const int ac = va ? a : 0, cc = vb ? c : 0;
    f64x4 acc = {0.0, 0.0, 0.0, 0.0}, acc1 = {0.0, 0.0, 0.0, 0.0};
    int i0 = 0;
    for (; i0 + 16 <= r; i0 += 16) {
      double av[4], bv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = i0 + 4 * u + kq;
        const float xa = sA[i * P + ac], xb = sB[i * P + cc];
        av[u] = va ? (double)xa : 0.0;
        bv[u] = vb ? (double)xb : 0.0;
      }
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[0], bv[0], acc, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(av[1], bv[1], acc1, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[2], bv[2], acc, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(av[3], bv[3], acc1, 0, 0, 0);
    }
    for (; i0 < r; i0 += 4) {
      const int i = i0 + kq;
      const double av = (i < r && va) ? (double)sA[i * P + ac] : 0.0;
      const double bv = (i < r && vb) ? (double)sB[i * P + cc] : 0.0;
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
    }
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) acc[reg] += acc1[reg];
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
      const int row = 16 * ta + kq + 4 * reg, col = 16 * tb + m;
      if (row < P && col < P) out[row * P + col] = acc[reg];
    }
  }
  __syncthreads();
}

// prod8 on the fp64 matrix cores: one 16 x 16 tile (the 8 x 8 block valid), the r rows
// split over the four waves (16-row steps, two accumulators, as prodP), the four partial
// 8 x 8 blocks summed in wave order through sPart[4][64]. prod8's butterflies were 64
// cross-lane fp64 exchanges per call. Ends with out visible to all threads.
#ifndef SPECENH_SS_PROD8_VALU
#define SPECENH_SS_PROD8_VALU 0
#endif
__device__ __forceinline__ void prod8m(const float* sA, const float* sB, int r, double* sPart,
                                       double* out) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m = lane & 15, kq = lane >> 4;
  const bool v = m < 8;
  const int mc = v ? m : 0;
  const int rq = ((r + 15) / 16 + 3) / 4 * 16;  // rows per wave, a multiple of 16
  const int i_lo = min(r, wave * rq), i_hi = min(r, i_lo + rq);
  f64x4 acc = {0.0, 0.0, 0.0, 0.0}, acc1 = {0.0, 0.0, 0.0, 0.0};
  int i0 = i_lo;
  for (; i0 + 16 <= i_hi; i0 += 16) {
    double av[4], bv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = i0 + 4 * u + kq;
      const float xa = sA[i * 8 + mc], xb = sB[i * 8 + mc];
      av[u] = v ? (double)xa : 0.0;
      bv[u] = v ? (double)xb : 0.0;
    }
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[0], bv[0], acc, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(av[1], bv[1], acc1, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[2], bv[2], acc, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(av[3], bv[3], acc1, 0, 0, 0);
  }
  for (; i0 < i_hi; i0 += 4) {
    const int i = i0 + kq;
    const double av = (i < i_hi && v) ? (double)sA[i * 8 + mc] : 0.0;
    const double bv = (i < i_hi && v) ? (double)sB[i * 8 + mc] : 0.0;
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
  }
#pragma unroll
  for (int reg = 0; reg < 4; ++reg) {
    const int row = kq + 4 * reg;  // D row (a), column m (c)
    if (row < 8 && v) sPart[wave * 64 + row * 8 + m] = acc[reg] + acc1[reg];
  }
  __syncthreads();
  if (tid < 64) out[tid] = (sPart[tid] + sPart[64 + tid]) + (sPart[128 + tid] + sPart[192 + tid]);
  __syncthreads();
}

// lane `src`'s v (wave-uniform src, a compile-time constant at the call sites)
__device__ __forceinline__ double readlane_f64(double v, int src) {
  const long long u = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_readlane((int)u, src);
  const int hi = __builtin_amdgcn_readlane((int)(u >> 32), src);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (long long)(unsigned)lo);
}

// fp64 1/x and 1/sqrt(x) from v_rcp_f64 / v_rsq_f64 and two Newton steps (full fp64
// precision for finite x != 0 / x > 0): the IEEE division and sqrt sequences sat on the
// critical path of every Jacobi round (the angle is computed once per pair, then rounded to
// fp32 for the rotation).
#ifndef SPECENH_SS_EXACT_ANGLE
#define SPECENH_SS_EXACT_ANGLE 0
#endif
__device__ __forceinline__ double rcp64_2(double x) {
  double r = __builtin_amdgcn_rcp(x);
  r = fma(r, fma(-x, r, 1.0), r);
  return fma(r, fma(-x, r, 1.0), r);
}
__device__ __forceinline__ double rsq64_2(double x) {
  double r = __builtin_amdgcn_rsq(x);
  r = fma(r * fma(-0.5 * x, r * r, 0.5), 1.0, r);      // r (1 + (1 - x r^2) / 2)
  return fma(r * fma(-0.5 * x, r * r, 0.5), 1.0, r);
}
// Orthonormalise the columns of Y (r x P, LDS) into Z with CholeskyQR in fp64:
// S = Y^T Y, S = R^T R, Z = Y R^-1. fp64 keeps the Gram of Y (condition up to ~1e12
// here) factorisable; callers run it twice (CholeskyQR2) for fp32-level orthogonality.
template <int P>
__device__ __forceinline__ void cholqr(const float* sY, float* sZ, int r, double* sS, double* sRi,
                                       long long* sub = nullptr) {
  const int tid = threadIdx.x;
#ifdef SPECENH_SS_STATS  // sub-phase clocks: Gram, Cholesky, forward substitution
  long long t_ = __builtin_amdgcn_s_memtime();
#define CQ_MARK(q)                                              \
  do {                                                          \
    const long long n_ = __builtin_amdgcn_s_memtime();          \
    if (sub) sub[q] += n_ - t_;                                 \
    t_ = n_;                                                    \
  } while (0)
#else
#define CQ_MARK(q) \
  do {             \
  } while (0)
#endif
  if constexpr (P == 8) {
    if (SPECENH_SS_PROD8_VALU) prod8(sY, sY, r, sS + 2 * P * P, sS);  // scratch [4][64] past sS, sRi
    else prod8m(sY, sY, r, sS + 2 * P * P, sS);
  } else {
    prodP<P>(sY, sY, r, sS);  // (full P x P; the factorisation reads the upper triangle)
  }
  __syncthreads();
  CQ_MARK(0);
  if (tid < 64 && P > 24) {  // Cholesky S = R^T R (R upper, in place), one wave, in LDS
    for (int k = 0; k < P; ++k) {
      double d = sS[k * P + k];
      d = d > 0.0 ? sqrt(d) : 1e-300;  // rank-deficient: keep going, column ~ 0
      wave_lds_sync();
      if (tid == 0) sS[k * P + k] = d;
      for (int j = k + 1 + tid; j < P; j += 64) sS[k * P + j] /= d;
      wave_lds_sync();
      constexpr int W = P;  // trailing block <= P x P
      for (int idx = tid; idx < W * W; idx += 64) {
        const int i2 = idx / W, j2 = idx % W;
        if (i2 > k && j2 >= i2) sS[i2 * P + j2] -= sS[k * P + i2] * sS[k * P + j2];
      }
      wave_lds_sync();
    }
  } else if (tid < 64) {  // P <= 24: the same factorisation in registers, lane j holding
                          // column j of S; row k of R reaches the lanes by readlane (no LDS
                          // round trips or wave syncs per pivot; larger P would spill)
    const int j = tid;
    double col[P];
#pragma unroll
    for (int i = 0; i < P; ++i) col[i] = (j < P && i <= j) ? sS[i * P + j] : 0.0;
#pragma unroll
    for (int k = 0; k < P; ++k) {
      double d = readlane_f64(col[k], k);
      if (SPECENH_SS_EXACT_ANGLE) {
        d = d > 0.0 ? sqrt(d) : 1e-300;  // rank-deficient: keep going, column ~ 0
        col[k] = j == k ? d : col[k] / d;  // row k of R (lanes j > k; j < k hold zeros)
      } else {  // the same from one v_rsq_f64 + Newton steps (the pivot's critical path)
        const double ri = d > 0.0 ? rsq64_2(d) : 1e300;
        col[k] = j == k ? (d > 0.0 ? d * ri : 1e-300) : col[k] * ri;
      }
#pragma unroll
      for (int i = k + 1; i < P; ++i) {  // trailing S[i][j] -= R[k][i] R[k][j], j >= i
        const double rki = readlane_f64(col[k], i);
        if (j >= i) col[i] -= rki * col[k];
      }
    }
    if (j < P)
#pragma unroll
      for (int i = 0; i < P; ++i)
        if (i <= j) sS[i * P + j] = col[i];
  }
  // Z = Y R^-1 row by row as the forward substitution z R = y (R upper):
  //   z_c = (y_c - sum_{d<c} z_d R[d][c]) / R[c][c],
  // P (P - 1) / 2 fp64 FMAs per row on broadcast LDS reads of R. Round 3 formed R^-1 first
  // with one wave (a serial chain of dependent fp64 LDS round trips per column) and then
  // multiplied by it (P^2 FMAs per row).
  if (tid < P) sRi[tid] = 1.0 / sS[tid * P + tid];
  __syncthreads();
  CQ_MARK(1);
  for (int i = tid; i < r; i += SS_THREADS) {
    // Column by column (z_c from the finished z_0 .. z_{c-1}): each z_c is consumed by the
    // next columns, so the FMAs stay in order. The pivot-row form (eliminate z_d from every
    // later column) let the compiler sink each pivot's FMAs to the end and keep every R
    // entry live: at P = 24 ~270 scratch spills per row and 512 registers per lane. R is
    // the same for every row: the opaque zero offset, renewed per column, keeps its reads
    // from being hoisted out of the row loop.
    int opq = 0;
    double z[P];
#pragma unroll
    for (int c = 0; c < P; ++c) {
      asm volatile("" : "+v"(opq));
      const double* rc = sS + c + opq;  // column c of R: rc[d * P]
      double t = sY[i * P + c];
#pragma unroll
      for (int d = 0; d < c; ++d) t = fma(-z[d], rc[d * P], t);
      z[c] = t * sRi[c + opq];
    }
#pragma unroll
    for (int c = 0; c < P; ++c) sZ[i * P + c] = (float)z[c];
  }
  __syncthreads();
  CQ_MARK(2);
#undef CQ_MARK
}

// rotation annihilating hab: tau = (hbb - haa) / (2 hab), t = sign(tau) / (|tau| +
// sqrt(1 + tau^2)), c = 1 / sqrt(1 + t^2), s = t c (|hab| > 1e-37)
__device__ __forceinline__ void jacobi_angle(double haa, double hbb, double hab, double& c,
                                             double& s) {
  if (SPECENH_SS_EXACT_ANGLE) {
    const double tau = (hbb - haa) / (2.0 * hab);
    const double tt = (tau >= 0 ? 1.0 : -1.0) / (fabs(tau) + sqrt(1.0 + tau * tau));
    c = 1.0 / sqrt(1.0 + tt * tt);
    s = tt * c;
    return;
  }
  const double tau = (hbb - haa) * rcp64_2(2.0 * hab);
  const double u = fma(tau, tau, 1.0);
  const double tt = copysign(rcp64_2(fabs(tau) + u * rsq64_2(u)), tau >= 0 ? 1.0 : -1.0);
  c = rsq64_2(fma(tt, tt, 1.0));
  s = tt * c;
}

// Parallel (round-robin / Brent-Luk) cyclic Jacobi on the symmetric P x P matrix H in
// LDS, one wave: each round rotates P/2 disjoint (a, b) pairs at once; Q accumulates
// the eigenvectors. Angles in fp64.
template <int P>
__device__ __forceinline__ int jacobi(float* sH, float* sQ, float* sCS, int* sPair) {  // -> sweeps run
  const int lane = threadIdx.x;  // wave 0
  for (int idx = lane; idx < P * P; idx += 64) sQ[idx] = (idx / P == idx % P) ? 1.f : 0.f;
  wave_lds_sync();
  int sweep = 0;
  for (; sweep < 15; ++sweep) {
    // The pairings of the unrolled rounds are the same every sweep: an opaque zero keeps
    // the compiler from hoisting all (round, item) index sets out of the sweep loop, where
    // they stayed live across the whole kernel and spilled (~270 VGPRs at P = 24)
    int opq = 0;
    asm volatile("" : "+v"(opq));
    double off = 0.0, diag = 0.0;
    for (int idx = lane; idx < P * P; idx += 64) {
      const double h = sH[idx];
      if (idx / P != idx % P) off += h * h; else diag += h * h;
    }
    for (int m = 32; m >= 1; m >>= 1) {
      off += __shfl_xor(off, m);
      diag += __shfl_xor(diag, m);
    }
    // uniform; H is stored in fp32, so an off-diagonal mass ~1e-13 of the diagonal (entries
    // ~3e-7 relative) is its rounding floor: converged
    if (off <= 1e-13 * diag) break;
    for (int round = 0; round < P - 1; ++round) {
      if (lane < P / 2) {  // tournament pairing: player 0 fixed, others rotate
        auto player = [&](int k) { return k == 0 ? 0 : 1 + (k - 1 + round + opq) % (P - 1); };
        int a = player(lane), b = player(P - 1 - lane);
        if (a > b) { const int t = a; a = b; b = t; }
        const double hab = sH[a * P + b];
        double c = 1.0, s = 0.0;
        if (fabs(hab) > 1e-37) {
          const double haa = sH[a * P + a], hbb = sH[b * P + b];
          jacobi_angle(haa, hbb, hab, c, s);
        }
        sCS[2 * lane] = (float)c;
        sCS[2 * lane + 1] = (float)s;
        sPair[2 * lane] = a;
        sPair[2 * lane + 1] = b;
      }
      wave_lds_sync();
      // The two updates below: a lane's pair (a, b) is recomputed in registers (the same
      // tournament formula) rather than read back from sPair, and the fixed trip count is
      // unrolled, so each pass is one round of independent LDS reads, not a dependent chain
      // of sPair -> sH round trips per item.
      constexpr int NIT = ((P / 2) * P + 63) / 64;
      // (P = 8, one item per lane: measured 1.37 ms with the sPair reads, 1.61 ms with the
      // recomputation per C3 default pass, so it keeps the table)
      auto pair_of = [&](int j, int& a, int& b) {
        if constexpr (P == 8) {
          a = sPair[2 * j];
          b = sPair[2 * j + 1];
        } else {
          auto player = [&](int k) { return k == 0 ? 0 : 1 + (k - 1 + round + opq) % (P - 1); };
          a = player(j);
          b = player(P - 1 - j);
          if (a > b) { const int t = a; a = b; b = t; }
        }
      };
      // (each pass reads all its items before writing any: the items touch disjoint
      // elements, and the compiler, unable to prove that, kept every item's reads behind
      // the previous item's writes — NIT dependent LDS round trips per pass)
      int ia[NIT], ib[NIT], ik[NIT];
      float cc[NIT], ss[NIT], xa[NIT], xb[NIT], qa[NIT], qb[NIT];
#pragma unroll
      for (int u = 0; u < NIT; ++u) {  // rows a, b of every pair
        const int idx = lane + 64 * u;
        const int j = idx < (P / 2) * P ? idx / P : 0;
        ik[u] = idx % P;
        pair_of(j, ia[u], ib[u]);
        cc[u] = sCS[2 * j];
        ss[u] = sCS[2 * j + 1];
        xa[u] = sH[ia[u] * P + ik[u]];
        xb[u] = sH[ib[u] * P + ik[u]];
      }
#pragma unroll
      for (int u = 0; u < NIT; ++u)
        if (lane + 64 * u < (P / 2) * P) {
          sH[ia[u] * P + ik[u]] = cc[u] * xa[u] - ss[u] * xb[u];
          sH[ib[u] * P + ik[u]] = ss[u] * xa[u] + cc[u] * xb[u];
        }
      wave_lds_sync();
#pragma unroll
      for (int u = 0; u < NIT; ++u) {  // columns a, b; Q columns
        xa[u] = sH[ik[u] * P + ia[u]];
        xb[u] = sH[ik[u] * P + ib[u]];
        qa[u] = sQ[ik[u] * P + ia[u]];
        qb[u] = sQ[ik[u] * P + ib[u]];
      }
#pragma unroll
      for (int u = 0; u < NIT; ++u)
        if (lane + 64 * u < (P / 2) * P) {
          sH[ik[u] * P + ia[u]] = cc[u] * xa[u] - ss[u] * xb[u];
          sH[ik[u] * P + ib[u]] = ss[u] * xa[u] + cc[u] * xb[u];
          sQ[ik[u] * P + ia[u]] = cc[u] * qa[u] - ss[u] * qb[u];
          sQ[ik[u] * P + ib[u]] = ss[u] * qa[u] + cc[u] * qb[u];
        }
      wave_lds_sync();
    }
  }
  return sweep;
}

// The same cyclic Jacobi with the lanes grouped by pair (default): L lanes per pair, lane
// (pair j, sub) covering columns NC sub .. of rows (a, b) in the row pass and rows NC sub ..
// of columns (a, b) in the column pass. Each lane computes its own pair's angle from the
// reads of the row pass, so a round is two read -> write phases and two wave syncs; the
// table form above (P / 2 angle lanes write (c, s) to LDS, sync, every lane reads them
// back) adds a third dependent LDS round trip. The pair indices advance by one tournament
// step per round in registers (no modulo per item and round).
#ifndef SPECENH_SS_JACOBI_TABLE
#define SPECENH_SS_JACOBI_TABLE 0
#endif
template <int P>
__device__ __forceinline__ int jacobi_grouped(float* sH, float* sQ) {  // -> sweeps run
  constexpr int NP = P / 2;                                   // pairs per round
  constexpr int L = (128 / P) < P ? (128 / P) : P;            // lanes per pair
  constexpr int NC = (P + L - 1) / L;                         // columns (rows) per lane
  static_assert(L * NP <= 64, "lanes");
  const int lane = threadIdx.x;  // wave 0
  for (int idx = lane; idx < P * P; idx += 64) sQ[idx] = (idx / P == idx % P) ? 1.f : 0.f;
  const int j = lane / L, sub = lane - j * L;
  const bool live = j < NP;
  const int k0 = NC * sub;
  // tournament players of pair j: kA = j (player 0 never moves), kB = P - 1 - j; player
  // k > 0 sits at 1 + (k - 1 + round) mod (P - 1)
  const int kA = live ? j : 0, kB = live ? P - 1 - j : P - 1;
  int ra0 = kA == 0 ? 0 : kA - 1, rb0 = kB - 1;  // round-0 offsets
  wave_lds_sync();
  int sweep = 0;
  for (; sweep < 15; ++sweep) {
    double off = 0.0, diag = 0.0;
    for (int idx = lane; idx < P * P; idx += 64) {
      const double h = sH[idx];
      if (idx / P != idx % P) off += h * h; else diag += h * h;
    }
    for (int m = 32; m >= 1; m >>= 1) {
      off += __shfl_xor(off, m);
      diag += __shfl_xor(diag, m);
    }
    if (off <= 1e-13 * diag) break;  // (uniform; see jacobi)
    int ra = ra0, rb = rb0;
    for (int round = 0; round < P - 1; ++round) {
      int a = kA == 0 ? 0 : 1 + ra, b = 1 + rb;
      if (a > b) { const int t = a; a = b; b = t; }
      // row pass: the pair's 2 x 2 entries and this lane's columns of rows a, b
      const float haa = sH[a * P + a], hbb = sH[b * P + b], hab = sH[a * P + b];
      float xa[NC], xb[NC];
#pragma unroll
      for (int u = 0; u < NC; ++u) {
        const int k = min(k0 + u, P - 1);
        xa[u] = sH[a * P + k];
        xb[u] = sH[b * P + k];
      }
      double cd = 1.0, sd = 0.0;
      if (fabs((double)hab) > 1e-37) jacobi_angle(haa, hbb, hab, cd, sd);
      const float c = (float)cd, sn = (float)sd;
      if (live) {
#pragma unroll
        for (int u = 0; u < NC; ++u)
          if (k0 + u < P) {
            sH[a * P + k0 + u] = c * xa[u] - sn * xb[u];
            sH[b * P + k0 + u] = sn * xa[u] + c * xb[u];
          }
      }
      wave_lds_sync();
      // column pass: rows k0 .. of columns a, b of H and Q
      float qa[NC], qb[NC];
#pragma unroll
      for (int u = 0; u < NC; ++u) {
        const int k = min(k0 + u, P - 1);
        xa[u] = sH[k * P + a];
        xb[u] = sH[k * P + b];
        qa[u] = sQ[k * P + a];
        qb[u] = sQ[k * P + b];
      }
      if (live) {
#pragma unroll
        for (int u = 0; u < NC; ++u)
          if (k0 + u < P) {
            const int k = k0 + u;
            sH[k * P + a] = c * xa[u] - sn * xb[u];
            sH[k * P + b] = sn * xa[u] + c * xb[u];
            sQ[k * P + a] = c * qa[u] - sn * qb[u];
            sQ[k * P + b] = sn * qa[u] + c * qb[u];
          }
      }
      wave_lds_sync();
      ra = ra + 1 == P - 1 ? 0 : ra + 1;
      rb = rb + 1 == P - 1 ? 0 : rb + 1;
    }
  }
  return sweep;
}

// P = 8 adds the prod8 scratch ([4][64] doubles after sRi) and gemm_GZ8's sT (r x 8).
template <int P>
struct SsLayout {
  static constexpr int part = P == 8 ? 4 * 64 : 0;  // doubles
  static size_t bytes(int r) {
    return (size_t)2 * r * P * 4 + (size_t)(2 * P * P + part) * 8 + (size_t)2 * P * P * 4 +
           P * 4 + P * 8 + 64 + (P == 8 ? (size_t)r * 8 * 4 : 0);
  }
};

// One workgroup per matrix: top-K eigenpairs of G (r x r) -> V[b] (r x K), theta[b] (K).
// With flags, the boundary Ritz pairs of the kept range (component K-1, and cut2 when the
// range starts inside the subspace) are checked: sqrt(theta_c) * ||G v_c - theta_c v_c|| /
// (theta_c - theta_{c+1}) bounds the reconstruction error their angle causes (Davis-Kahan);
// above tolv * ||X||_F (tolv = 5e-6: half the 1e-5 parity contract, and above the fp32
// floor of the residual itself on gapped inputs) the matrix is flagged for the fp64 eigen
// path (a cut with no spectral gap, e.g. inside a noise bulk, where subspace iteration does
// not converge).
template <int P>
// Waves per SIMD the register budget is sized for (P = 16, 24: 256 VGPRs, 2 workgroups per CU)
#ifndef SPECENH_SS_WPE
#define SPECENH_SS_WPE 2
#endif
#ifndef SPECENH_SS8_WPE
#define SPECENH_SS8_WPE 4  // (C3 default 3.22 -> 3.16 ms vs 2)
#endif
__global__ __launch_bounds__(SS_THREADS)
__attribute__((amdgpu_waves_per_eu(P == 8 ? SPECENH_SS8_WPE : P <= 24 ? SPECENH_SS_WPE : 1)))
void subspace_kernel(const float* G, int r, int K,
                                                              int iters, float* V,
                                                              float* theta, int cut2,
                                                              float tolv, int* flags, int seed,
                                                              const int* only, int gz_quad) {
  __shared__ double sRed[4];
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* sS = reinterpret_cast<double*>(smem);            // P x P
  double* sRi = sS + P * P;                                  // P x P
  double* sPart = sRi + P * P;                               // SsLayout<P>::part
  float* sZ = reinterpret_cast<float*>(sPart + SsLayout<P>::part);  // r x P
  float* sY = sZ + r * P;                                    // r x P
  float* sH = sY + r * P;                                    // P x P
  float* sQ = sH + P * P;                                    // P x P
  float* sCS = sQ + P * P;                                   // P (c, s per pair)
  int* sPair = reinterpret_cast<int*>(sCS + P);              // P
  int* sOrd = sPair + P;                                     // P
  float* sT = reinterpret_cast<float*>(sOrd + P + 16);      // r x 8 (P = 8)
  const long long b = blockIdx.x;
  const float* Gb = G + b * (long long)r * r;
  const int tid = threadIdx.x;
#ifdef SPECENH_SS_STATS  // development build (tools/ss_stats.py): shader clocks per phase
  long long tacc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tlast = __builtin_amdgcn_s_memtime();
  long long csub[3] = {0, 0, 0};
#define CQ_SUB csub
  int sweeps = 0;
#define SS_MARK(slot)                                    \
  do {                                                   \
    const long long now_ = __builtin_amdgcn_s_memtime(); \
    tacc[slot] += now_ - tlast;                          \
    tlast = now_;                                        \
  } while (0)
#else
#define SS_MARK(slot) \
  do {                \
  } while (0)
#define CQ_SUB nullptr
#endif

  // (gz_quad: the host checked r % 4 == 0 and a 16-byte aligned G, r^2 floats per matrix)
  auto GZ = [&](const float* z, float* y) {
    if (P <= 24 && gz_quad) gemm_GZ4<P <= 24 ? P : 8>(Gb, r, z, y);
    else if constexpr (P == 8) gemm_GZ8(Gb, r, z, y, sT);
    else gemm_GZ<P>(Gb, r, z, y);
  };
  if (only && !only[b]) return;  // (second pass: only the matrices the first one flagged)
  for (int idx = tid; idx < r * P; idx += SS_THREADS)
    sZ[idx] = hash_unit(idx / P + 7919u * seed, idx % P);
  __syncthreads();
  GZ(sZ, sY);
  __syncthreads();
  SS_MARK(0);
  auto bsum = [&](double v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
    __syncthreads();
    if ((tid & 63) == 0) sRed[tid >> 6] = v;
    __syncthreads();
    return (sRed[0] + sRed[1]) + (sRed[2] + sRed[3]);
  };
  double tr = 0.0;  // tr(G) = ||X||_F^2, for the flag's tolerance
  if (flags) {
    for (int i = tid; i < r; i += SS_THREADS) tr += Gb[(long long)i * r + i];
    tr = bsum(tr);
  }
  // Staged first pass: 2 rounds, Rayleigh-Ritz and the convergence check; only a matrix
  // the check flags runs the remaining rounds (from the current basis) and a second
  // Rayleigh-Ritz. For the default K = 1 (P = 8, 5 rounds) log-spectrograms (a dominant
  // first component) converge in 2 rounds, while a small gap (the gapped C3 set,
  // s2/s1 = 0.8) takes all 5; an oversampled top-K block (3 rounds) mostly converges in 2.
  const int stage1 = (flags && !only && iters > 2) ? 2 : iters;
  int bad = 0;
  for (int stage = 0; stage < 2; ++stage) {
    const int nit = stage == 0 ? stage1 : iters - stage1;
    for (int it = 0; it < nit; ++it) {
      if (it + 1 < nit && (SPECENH_SS_SINGLE_QR)) {
        // Intermediate rounds only have to keep the block well conditioned (G Z
        // re-amplifies the dominant directions anyway): one CholeskyQR pass. The basis
        // that feeds the Rayleigh-Ritz step below gets the full CholeskyQR2.
        cholqr<P>(sY, sZ, r, sS, sRi, CQ_SUB);  // Z = orth(Y) to ~cond(Y) * eps
        SS_MARK(1);
        GZ(sZ, sY);                     // Y = G Z
        __syncthreads();
        SS_MARK(2);
        continue;
      }
      cholqr<P>(sY, sZ, r, sS, sRi, CQ_SUB);  // Z = orth(Y)
      cholqr<P>(sZ, sY, r, sS, sRi, CQ_SUB);  // second pass into Y ...
      SS_MARK(1);
      GZ(sY, sZ);                     // ... Z = G * orth(Y)
      __syncthreads();
      SS_MARK(2);
      // swap names: basis in sY, product in sZ -> keep (Y := product, Z := basis)
      float* t = sY;
      sY = sZ;
      sZ = t;
    }
    // Rayleigh-Ritz: H = Z^T (G Z) = Z^T Y
    if constexpr (P == 8) {
      if (SPECENH_SS_PROD8_VALU) prod8(sZ, sY, r, sPart, sS);
      else prod8m(sZ, sY, r, sPart, sS);
      if (tid < 64) sH[tid] = (float)sS[tid];
    } else {
      prodP<P>(sZ, sY, r, sS);
      for (int q = tid; q < P * P; q += SS_THREADS) sH[q] = (float)sS[q];
    }
    __syncthreads();
    for (int q = tid; q < P * P; q += SS_THREADS) {  // symmetrise
      const int a = q / P, c = q % P;
      if (a < c) {
        const float m = 0.5f * (sH[a * P + c] + sH[c * P + a]);
        sH[a * P + c] = m;
        sH[c * P + a] = m;
      }
    }
    __syncthreads();
    SS_MARK(3);
    if (tid < 64) {
      const int sw = SPECENH_SS_JACOBI_TABLE ? jacobi<P>(sH, sQ, sCS, sPair)
                                             : jacobi_grouped<P>(sH, sQ);
#ifdef SPECENH_SS_STATS
      sweeps += sw;
#else
      (void)sw;
#endif
      // Ritz values descending, ties in index order (a stable sort), as ranks: lane c counts
      // the values ahead of its own (thread 0's insertion sort was a serial chain of LDS
      // reads); NaN sorts last
      wave_lds_sync();
      if (tid < P) {
        auto key = [&](int c) {
          const float v = sH[c * P + c];
          return v == v ? v : -INFINITY;
        };
        const float t = key(tid);
        int rank = 0;
#pragma unroll
        for (int d = 0; d < P; ++d) {
          const float u = key(d);
          rank += (u > t || (u == t && d < tid)) ? 1 : 0;
        }
        sOrd[rank] = tid;
      }
    }
    __syncthreads();
    SS_MARK(4);
    bad = 0;
    if (flags) {
      for (int which = 0; which < 2; ++which) {
        const int c = which == 0 ? K - 1 : cut2;  // uniform
        if (c < 0 || c >= K) continue;
        const int col = sOrd[c];
        const double th = sH[col * P + col];
        double acc = 0.0;
        for (int i = tid; i < r; i += SS_THREADS) {
          double ri = 0.0;
#pragma unroll
          for (int d = 0; d < P; ++d)
            ri = fma((double)sY[i * P + d] - th * (double)sZ[i * P + d], (double)sQ[d * P + col], ri);
          acc = fma(ri, ri, acc);
        }
        const double res = sqrt(bsum(acc));
        if (c + 1 >= P) {
          if (P < r) bad = 1;  // no Ritz value past the cut to measure the gap against
          continue;
        }
        const double gap = th - (double)sH[sOrd[c + 1] * P + sOrd[c + 1]];
        if (!(sqrt(fmax(th, 0.0)) * res <= (double)tolv * gap * sqrt(fmax(tr, 0.0)))) bad = 1;
      }
    }
    SS_MARK(5);
    if (!bad || stage1 >= iters) break;  // uniform: converged, or no second stage
  }
  if (flags && tid == 0) flags[b] = bad;
  float* Vb = V + b * (long long)r * K;  // V[:, c] = Z Q[:, ord[c]], c < K
  for (int idx = tid; idx < r * K; idx += SS_THREADS) {
    const int i = idx / K, c = idx % K;
    const int col = sOrd[c];
    double s = 0.0;
#pragma unroll
    for (int d = 0; d < P; ++d) s += (double)sZ[i * P + d] * sQ[d * P + col];
    Vb[(long long)i * K + c] = (float)s;
  }
  if (tid < K) theta[b * K + tid] = sH[sOrd[tid] * P + sOrd[tid]];
#ifdef SPECENH_SS_STATS  // (into this matrix's Gram: dead once V is out, no flagged reruns here)
  SS_MARK(6);
  __syncthreads();
  if (tid == 0) {
    long long* o = reinterpret_cast<long long*>(const_cast<float*>(Gb));
    for (int q = 0; q < 7; ++q) o[q] = tacc[q];
    o[7] = sweeps;
    for (int q = 0; q < 3; ++q) o[8 + q] = csub[q];
  }
#endif
#undef SS_MARK
#undef CQ_SUB
}

// Workgroup barrier that orders LDS only: waits for this wave's LDS operations, not for
// its global loads (__syncthreads' release fence would also drain vmcnt, i.e. wait for the
// next matrix's prefetch at the first barrier after it is issued).
__device__ __forceinline__ void lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// ---------------------------------------------------------------- 3. reconstruction
// Workgroup = (matrix, block of RB X-rows). With X_blk (RB x r), V (r x K):
//   Y = X_blk V_K                       (RB x K)      phase 1
//   out = Y[:, lo:hi] V[:, lo:hi]^T     (RB x r)      phase 2 (complement: X_blk - ...)
constexpr int RB = 32;

// only (optional, device int[batch]): reconstruct only the matrices with only[b] != 0.
template <typename TO>
__device__ __forceinline__ TO to_out(float v) { return (TO)v; }

// TO: output element type (float, or _Float16 / __bf16 when the consumer computes in half
// precision: the cast rides on the reconstruction's store, no separate pass)
template <int KP, typename TO>
__global__ __launch_bounds__(256) void recon_kernel(XView x, int Kr, int r, const float* V,
                                                    int K, int lo, int hi, int complement,
                                                    const int* only, TO* out,
                                                    long long out_bstride, long long osk,
                                                    long long osi) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* sV = reinterpret_cast<float*>(smem);  // r x KP (zero-padded columns)
  float* sX = sV + r * KP;                      // RB x (r + 1)
  float* sY = sX + RB * (r + 1);                // RB x KP
  const long long b = blockIdx.y;
  if (only && !only[b]) return;
  const int k0 = blockIdx.x * RB;
  const int tid = threadIdx.x;
  const float* X = x.base + b * x.batch_stride;
  const float* Vb = V + b * (long long)r * K;
  // Staging in batches of loads per thread, all in flight before their LDS writes (a
  // plain strided loop waits for each load in turn: ~50 HBM round trips per workgroup).
  // (batches of 16 for V and 32 for X: one round trip each at C3's r = 256, K = 16)
  constexpr int UB = 16, UBX = 32;
  for (int i0 = tid; i0 < r * KP; i0 += 256 * UB) {
    float t[UB];
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const int idx = i0 + 256 * u, i = idx / KP, c = idx % KP;
      t[u] = (idx < r * KP && c >= lo && c < hi) ? Vb[(long long)i * K + c] : 0.f;  // used columns
    }
#pragma unroll
    for (int u = 0; u < UB; ++u)
      if (i0 + 256 * u < r * KP) sV[i0 + 256 * u] = t[u];
  }
  const int rows = min(RB, Kr - k0);
  const bool tr = x.si != 1;  // transposed view: walk the contiguous k direction
  for (int i0 = tid; i0 < RB * r; i0 += 256 * UBX) {
    float t[UBX];
#pragma unroll
    for (int u = 0; u < UBX; ++u) {
      const int idx = i0 + 256 * u;
      const int kk = tr ? idx % RB : idx / r, i = tr ? idx / RB : idx % r;
      t[u] = (idx < RB * r && kk < rows) ? X[(long long)(k0 + kk) * x.sk + (long long)i * x.si] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < UBX; ++u) {
      const int idx = i0 + 256 * u;
      const int kk = tr ? idx % RB : idx / r, i = tr ? idx / RB : idx % r;
      if (idx < RB * r) sX[kk * (r + 1) + i] = t[u];
    }
  }
  __syncthreads();
  // phase 1: RB x KP entries of Y, a quad of columns per thread (one X read and one 16-byte
  // V read per 4 FMAs; unused columns of sV are zero, so their Y entries are +0)
  for (int e = tid; e < RB * (KP / 4); e += 256) {
    const int kk = e / (KP / 4), c4 = e % (KP / 4);
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    if (4 * c4 + 3 >= lo && 4 * c4 < hi)
      for (int i = 0; i < r; ++i) {
        const float xv = sX[kk * (r + 1) + i];
        const float4 v = *reinterpret_cast<const float4*>(sV + i * KP + 4 * c4);
        s.x = fmaf(xv, v.x, s.x);
        s.y = fmaf(xv, v.y, s.y);
        s.z = fmaf(xv, v.z, s.z);
        s.w = fmaf(xv, v.w, s.w);
      }
    *reinterpret_cast<float4*>(sY + kk * KP + 4 * c4) = s;
  }
  __syncthreads();
  // phase 2: out rows, thread per column i (coalesced along i for m >= n)
  TO* Ob = out + b * out_bstride;
  if (osi == 1) {  // column i's V row stays in registers over the block's rows; Y rows are
                   // wave-wide broadcasts
    for (int i = tid; i < r; i += 256) {
      float v[KP];
#pragma unroll
      for (int c4 = 0; c4 < KP / 4; ++c4) {
        const float4 t = *reinterpret_cast<const float4*>(sV + i * KP + 4 * c4);
        v[4 * c4] = t.x; v[4 * c4 + 1] = t.y; v[4 * c4 + 2] = t.z; v[4 * c4 + 3] = t.w;
      }
      for (int kk = 0; kk < rows; ++kk) {
        float s = 0.f;
#pragma unroll
        for (int c4 = 0; c4 < KP / 4; ++c4) {
          const float4 y = *reinterpret_cast<const float4*>(sY + kk * KP + 4 * c4);
          s = fmaf(y.x, v[4 * c4], s);
          s = fmaf(y.y, v[4 * c4 + 1], s);
          s = fmaf(y.z, v[4 * c4 + 2], s);
          s = fmaf(y.w, v[4 * c4 + 3], s);
        }
        const float o = complement ? sX[kk * (r + 1) + i] - s : s;
        Ob[(long long)(k0 + kk) * osk + i] = to_out<TO>(o);
      }
    }
    return;
  }
  for (int e = tid; e < RB * r; e += 256) {
    int kk, i;
    if (osi == 1) { kk = e / r; i = e % r; } else { i = e / RB; kk = e % RB; }
    if (kk >= rows) continue;
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < KP; ++c) s = fmaf(sY[kk * KP + c], sV[i * KP + c], s);
    const float v = complement ? sX[kk * (r + 1) + i] - s : s;
    Ob[(long long)(k0 + kk) * osk + (long long)i * osi] = to_out<TO>(v);
  }
}

// recon_mfma_kernel: the same reconstruction with both products on the fp32 matrix cores
// (v_mfma_f32_16x16x4_f32). recon_kernel's scalar FMAs needed one or two LDS reads per four
// FMAs plus their address arithmetic: 954 M VALU instructions for C3's rank-16 pass, 3.6x the
// FMAs themselves (PMC, profiles/pmc_r04.json). Per workgroup (matrix, RB = 32 rows):
//   phase 1  Y (32 x KPP) = X_blk (32 x RP) V (RP x KPP): 2 x NT tiles of 16 x 16, the r-long
//            K loop split over two waves when there are fewer than four tiles (partials summed
//            in LDS);
//   phase 2  out (32 x RP) = [X_blk -] Y V^T: 2 x RP/16 tiles dealt to the 4 waves, K = KPP.
// Operand layout (16x16x4 f32): lane l supplies A[l & 15][l >> 4] and B[l >> 4][l & 15], and
// holds D[4 (l >> 4) + j][l & 15]. LDS pitches: X rows RP + 2 words (A reads: 16 rows x 2 k per
// 32-lane group on distinct banks), V rows KPP + 1 (odd: conflict-free both as phase 1's B, rows
// k, and as phase 2's B, rows i), Y rows KPP + 1. Columns r .. RP - 1 and K .. KPP - 1 are zero.
template <int KP, typename TO>
__global__ __launch_bounds__(256) void recon_mfma_kernel(XView x, int Kr, int r, const float* V,
                                                         int K, int lo, int hi, int complement,
                                                         const int* only, TO* out,
                                                         long long out_bstride, long long osk,
                                                         long long osi) {
  constexpr int NT = (KP + 15) / 16, KPP = 16 * NT, PV = KPP + 1, PY = KPP + 1;
  constexpr int KS = 2 * NT < 4 ? 2 : 1;  // K split of phase 1
  typedef float f4 __attribute__((ext_vector_type(4)));
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int RP = (r + 15) & ~15, PX = RP + 2;
  float* sV = reinterpret_cast<float*>(smem);  // RP x PV
  float* sX = sV + RP * PV;                     // RB x PX
  float* sY = sX + RB * PX;                     // KS x RB x PY
  const long long b = blockIdx.y;
  if (only && !only[b]) return;
  const int k0 = blockIdx.x * RB;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int cl = lane & 15, kr = lane >> 4;
  const float* X = x.base + b * x.batch_stride;
  const float* Vb = V + b * (long long)r * K;
  constexpr int UB = 16, UBX = 32;
  for (int i0 = tid; i0 < RP * KPP; i0 += 256 * UB) {
    float t[UB];
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const int idx = i0 + 256 * u, i = idx / KPP, c = idx % KPP;
      t[u] = (idx < RP * KPP && i < r && c >= lo && c < hi) ? Vb[(long long)i * K + c] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const int idx = i0 + 256 * u;
      if (idx < RP * KPP) sV[(idx / KPP) * PV + idx % KPP] = t[u];
    }
  }
  const int rows = min(RB, Kr - k0);
  const bool tr = x.si != 1;
  for (int i0 = tid; i0 < RB * RP; i0 += 256 * UBX) {
    float t[UBX];
#pragma unroll
    for (int u = 0; u < UBX; ++u) {
      const int idx = i0 + 256 * u;
      const int kk = tr ? idx % RB : idx / RP, i = tr ? idx / RB : idx % RP;
      t[u] = (idx < RB * RP && kk < rows && i < r)
                 ? X[(long long)(k0 + kk) * x.sk + (long long)i * x.si] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < UBX; ++u) {
      const int idx = i0 + 256 * u;
      const int kk = tr ? idx % RB : idx / RP, i = tr ? idx / RB : idx % RP;
      if (idx < RB * RP) sX[kk * PX + i] = t[u];
    }
  }
  __syncthreads();
  // ---- phase 1: Y = X_blk V
  {
    const int klen = RP / KS;
    for (int t = wave; t < 2 * NT * KS; t += 4) {
      const int tile = t % (2 * NT), part = t / (2 * NT);
      const int rt = tile & 1, ct = tile >> 1;
      const float* a_p = sX + (16 * rt + cl) * PX + part * klen + kr;
      const float* b_p = sV + (part * klen + kr) * PV + 16 * ct + cl;
      f4 acc = f4{0.f, 0.f, 0.f, 0.f};
      for (int k = 0; k < klen; k += 4)
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a_p[k], b_p[k * PV], acc, 0, 0, 0);
      float* yp = sY + part * RB * PY + (16 * rt + 4 * kr) * PY + 16 * ct + cl;
#pragma unroll
      for (int j = 0; j < 4; ++j) yp[j * PY] = acc[j];
    }
  }
  __syncthreads();
  if constexpr (KS == 2) {
    for (int e = tid; e < RB * KPP; e += 256) {
      const int row = e / KPP, c = e % KPP;
      sY[row * PY + c] += sY[RB * PY + row * PY + c];
    }
    __syncthreads();
  }
  // ---- phase 2: out = [X_blk -] Y V^T
  TO* Ob = out + b * out_bstride;
  const int nit = RP / 16;
  for (int t = wave; t < 2 * nit; t += 4) {
    const int rt = t & 1, it = t >> 1;
    const float* a_p = sY + (16 * rt + cl) * PY + kr;
    const float* b_p = sV + (16 * it + cl) * PV + kr;
    f4 acc = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < KPP; k += 4)
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a_p[k], b_p[k], acc, 0, 0, 0);
    const int col = 16 * it + cl;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = 16 * rt + 4 * kr + j;
      if (row < rows && col < r) {
        const float v = complement ? sX[row * PX + col] - acc[j] : acc[j];
        Ob[(long long)(k0 + row) * osk + (long long)col * osi] = to_out<TO>(v);
      }
    }
  }
}

// V (r x K, the kept columns [lo, hi)) into LDS as RP x KPP with row pitch PV, zero-padded:
// batches of 16 loads per thread in flight before their LDS writes (a plain strided loop
// waited a full round trip for each of its RP KPP / 256 loads)
template <int KPP, int PV>
__device__ __forceinline__ void stage_v(const float* Vb, int r, int K, int lo, int hi, int RP,
                                        float* sV) {
  constexpr int UB = 16;
  for (int i0 = threadIdx.x; i0 < RP * KPP; i0 += 256 * UB) {
    float t[UB];
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const int idx = i0 + 256 * u, i = idx / KPP, c = idx % KPP;
      t[u] = (idx < RP * KPP && i < r && c >= lo && c < hi) ? Vb[(long long)i * K + c] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const int idx = i0 + 256 * u;
      if (idx < RP * KPP) sV[(idx / KPP) * PV + idx % KPP] = t[u];
    }
  }
}

// recon_stream_kernel: recon_mfma_kernel's two products, with a workgroup walking a run of
// `bps` consecutive row blocks of one matrix (all of them when the batch fills the chip:
// C3's 4096 matrices, 17 blocks each). recon_mfma_kernel's workgroups each staged V (16 KB at
// K = 16, half the X block's bytes) and one X block, then computed, then stored: nothing in
// flight while computing, ~2 workgroups per CU, 4.3x the HBM time of reading X and writing
// the output. Here V is staged once per run, and the next X block's loads are issued before
// the current block's products, so they are in flight behind the MFMAs and the stores.
// Staging without run-time divisions: row-major X (TRANS = false) as float4s, thread t ->
// float4 column t & 63 of rows t >> 6, + 4, ... (8 per block; columns >= r zero); transposed X
// (TRANS, X[k][i] = base[k + i si]) as thread t -> column t, 32 consecutive k (float4s when
// aligned). Phase 2's tiles put the output's contiguous direction along the lanes: D = Y V^T
// tiles for row-major output, D = V Y^T (the same two LDS operands, swapped) for transposed.
template <int KP, typename TO, bool TRANS>
__global__ __launch_bounds__(256, 2) void recon_stream_kernel(
    XView x, int Kr, int r, const float* V, int K, int lo, int hi, int complement,
    const int* only, TO* out, long long out_bstride, long long osk, long long osi, int bps) {
  constexpr int NT = (KP + 15) / 16, KPP = 16 * NT, PV = KPP + 1, PY = KPP + 1;
  constexpr int KS = 2 * NT < 4 ? 2 : 1;  // K split of phase 1
  typedef float f4 __attribute__((ext_vector_type(4)));
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int RP = (r + 15) & ~15, PX = RP + 2;
  float* sV = reinterpret_cast<float*>(smem);  // RP x PV
  float* sX = sV + RP * PV;                     // RB x PX
  float* sY = sX + RB * PX;                     // KS x RB x PY
  const long long b = blockIdx.y;
  if (only && !only[b]) return;
  const int nblk = (Kr + RB - 1) / RB;
  const int blk0 = blockIdx.x * bps, blk1 = min(nblk, blk0 + bps);
  if (blk0 >= blk1) return;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int cl = lane & 15, kr = lane >> 4;
  const float* X = x.base + b * x.batch_stride;
  const float* Vb = V + b * (long long)r * K;
  stage_v<KPP, PV>(Vb, r, K, lo, hi, RP, sV);
  float4 stA[8], stB[8];  // two blocks in flight: the next two blocks' X
  const bool vec_t = TRANS && (x.si & 3) == 0 && (x.batch_stride & 3) == 0 &&
                     (reinterpret_cast<uintptr_t>(x.base) & 15) == 0;
  // rows = 0: no loads (zeros), so a refill past the run is a predicated no-op rather than
  // a branch around the loads (a conditional refill keeps the batches out of registers)
  auto fetch = [&](float4 (&st)[8], int k0, int rows) {
    if constexpr (!TRANS) {
      const int c4 = tid & 63, rs = tid >> 6;
      const bool cv = 4 * c4 < r;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int kk = rs + 4 * u;
        st[u] = (cv && kk < rows)
                    ? *reinterpret_cast<const float4*>(X + (long long)(k0 + kk) * x.sk + 4 * c4)
                    : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    } else {
      const float* p = X + (long long)(tid < r ? tid : 0) * x.si + k0;
      if (vec_t && rows == RB && tid < r) {
#pragma unroll
        for (int u = 0; u < 8; ++u) st[u] = *reinterpret_cast<const float4*>(p + 4 * u);
      } else {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          float e[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) e[q] = (tid < r && 4 * u + q < rows) ? p[4 * u + q] : 0.f;
          st[u] = make_float4(e[0], e[1], e[2], e[3]);
        }
      }
    }
  };
  auto stage = [&](const float4 (&st)[8]) {
    if constexpr (!TRANS) {
      const int c4 = tid & 63, rs = tid >> 6;
      if (4 * c4 < RP) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          float* d = sX + (rs + 4 * u) * PX + 4 * c4;  // (PX even: 8-byte aligned)
          *reinterpret_cast<float2*>(d) = make_float2(st[u].x, st[u].y);
          *reinterpret_cast<float2*>(d + 2) = make_float2(st[u].z, st[u].w);
        }
      }
    } else if (tid < RP) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        sX[(4 * u) * PX + tid] = st[u].x;
        sX[(4 * u + 1) * PX + tid] = st[u].y;
        sX[(4 * u + 2) * PX + tid] = st[u].z;
        sX[(4 * u + 3) * PX + tid] = st[u].w;
      }
    }
  };
  TO* Ob = out + b * out_bstride;
  const int nit = RP / 16;
  auto block = [&](int blk, float4 (&st)[8]) {
    const int k0 = blk * RB, rows = min(RB, Kr - k0);
    // (LDS-only barriers: __syncthreads' release fence drains vmcnt, i.e. it waited for the
    // prefetched blocks at the first barrier after their loads were issued)
    lds_sync();  // the previous block's products are done with sX / sY (and sV staged)
    stage(st);
    lds_sync();
    // block blk + 2 into the registers just staged: in flight behind two blocks' products
    fetch(st, k0 + 2 * RB, blk + 2 < blk1 ? min(RB, Kr - k0 - 2 * RB) : 0);
    // ---- phase 1: Y = X_blk V
    {
      const int klen = RP / KS;
      for (int t = wave; t < 2 * NT * KS; t += 4) {
        const int tile = t % (2 * NT), part = t / (2 * NT);
        const int rt = tile & 1, ct = tile >> 1;
        const float* a_p = sX + (16 * rt + cl) * PX + part * klen + kr;
        const float* b_p = sV + (part * klen + kr) * PV + 16 * ct + cl;
        // two accumulators, 8 k-steps per batch of LDS reads (one dependent chain of
        // read -> MFMA -> MFMA per k-step left the chain's latency exposed); klen % 32 == 0
        // when RP % 64 == 0 (C3), else the tail loop
        f4 acc = f4{0.f, 0.f, 0.f, 0.f}, acc2 = f4{0.f, 0.f, 0.f, 0.f};
        int k = 0;
        for (; k + 32 <= klen; k += 32) {
          float av[8], bv[8];
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            av[q] = a_p[k + 4 * q];
            bv[q] = b_p[(k + 4 * q) * PV];
          }
#pragma unroll
          for (int q = 0; q < 8; q += 2) {
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[q], bv[q], acc, 0, 0, 0);
            acc2 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[q + 1], bv[q + 1], acc2, 0, 0, 0);
          }
        }
        for (; k < klen; k += 4)
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a_p[k], b_p[k * PV], acc, 0, 0, 0);
        acc += acc2;
        float* yp = sY + part * RB * PY + (16 * rt + 4 * kr) * PY + 16 * ct + cl;
#pragma unroll
        for (int j = 0; j < 4; ++j) yp[j * PY] = acc[j];
      }
    }
    lds_sync();
    if constexpr (KS == 2) {
      for (int e = tid; e < RB * KPP; e += 256) {
        const int row = e / KPP, c = e % KPP;
        sY[row * PY + c] += sY[RB * PY + row * PY + c];
      }
      lds_sync();
    }
    // ---- phase 2: out = [X_blk -] Y V^T
    for (int t = wave; t < 2 * nit; t += 4) {
      const int rt = t & 1, it = t >> 1;
      const float* y_p = sY + (16 * rt + cl) * PY + kr;
      const float* v_p = sV + (16 * it + cl) * PV + kr;
      f4 acc = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < KPP; k += 4)
        acc = TRANS ? __builtin_amdgcn_mfma_f32_16x16x4f32(v_p[k], y_p[k], acc, 0, 0, 0)
                    : __builtin_amdgcn_mfma_f32_16x16x4f32(y_p[k], v_p[k], acc, 0, 0, 0);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = TRANS ? 16 * rt + cl : 16 * rt + 4 * kr + j;
        const int col = TRANS ? 16 * it + 4 * kr + j : 16 * it + cl;
        if (row < rows && col < r) {
          const float v = complement ? sX[row * PX + col] - acc[j] : acc[j];
          Ob[(long long)(k0 + row) * osk + (long long)col * osi] = to_out<TO>(v);
        }
      }
    }
  };
  fetch(stA, blk0 * RB, min(RB, Kr - blk0 * RB));
  fetch(stB, (blk0 + 1) * RB, blk0 + 1 < blk1 ? min(RB, Kr - (blk0 + 1) * RB) : 0);
  for (int blk = blk0; blk < blk1; blk += 2) {
    block(blk, stA);
    if (blk + 1 < blk1) block(blk + 1, stB);
  }
}

// ---------------------------------------------------------------- 2'. top-1 complement
// The default kept range of denoiseSignal (denoising_by_svd.ipynb:188-229 with start = 1,
// stop = None: every component but the first) is out = X - (X v1) v1^T. For Kr, r <= 128
// one workgroup per matrix does it in one pass over HBM: X (zero-padded to 128 x 128) is
// resident in LDS and block power iteration with 4 vectors runs on it directly,
//   U = X Z,  Y = X^T U (= G Z),  Z <- Y R^-1 (CholeskyQR, fp64 Gram of Y),
// so the Gram matrix G is never formed. From the second round on, Rayleigh-Ritz in span(Z)
// (generalised, with the basis Gram M = Z^T Z: H q = theta M q, H = U^T U = Z^T G Z) gives
// theta_1 >= theta_2 and v = Z q_1, u = U q_1 = X v, and the same residual test as the
// subspace kernel: sqrt(theta_1) ||G v - theta_1 v|| <= tolv (theta_1 - theta_2) ||X||_F
// with G v = Y q_1. A matrix that fails it after TOP1_MAX_ROUNDS is flagged for the fp64
// eigen path (its output is overwritten there).
#ifndef SPECENH_TOP1_SWZ
#define SPECENH_TOP1_SWZ 1  // round 6: bank-conflict-free LDS layouts (tools/lds_banks.py)
#endif
namespace top1 {
constexpr int N = 128;              // X tile (rows k, columns i), zero-padded
constexpr int LD = N + 4;           // LDS row pitch in words: conflict-free row walks
constexpr int MAX_ROUNDS = 24;
// Zt row pitch and element offset. With SPECENH_TOP1_SWZ 4 pad words follow every 64
// columns, so the X Z phase's basis reads of chunks c and c + 16 (one ds_read_b128 lane
// group) land 4 banks apart instead of on the same 4 banks.
constexpr int ZP = SPECENH_TOP1_SWZ ? N + 8 : N;
__host__ __device__ constexpr int zt(int p, int k) {
  return p * ZP + k + (SPECENH_TOP1_SWZ ? 4 * (k >> 6) : 0);
}
// The per-wave partial sums of Y = X^T U: row i at slot pos(i). The writers (lane (cc, h):
// rows 4 cc + 2 h + {0, 1}, two ds_write_b128) were 4-way conflicted at slot = i; the XOR of
// bits 3-5 into bits 0-2 keeps every 8-lane write group on 8 distinct 16-byte slots and stays
// inside the row's 8-row block (the same wave's range for the reduction's readers).
__device__ __forceinline__ int ppos(int i) { return SPECENH_TOP1_SWZ ? i ^ ((i >> 3) & 7) : i; }
// X Z phase: the float4 column chunk of lane column group g (0..7) in k-step j (0..3). Each
// ds_read_b128 lane group holds g in {0..3} or {4..7} with 4 rows kb each; the chunks of
// g = 0, 1 share a 16-bank quarter, g = 2, 3 the opposite one, all four the same chunk
// residue mod 4: 64 distinct banks per group (the old mapping 8 (g & 1) + (g >> 1) + ... put
// two addresses on one bank in every group).
__device__ __forceinline__ int xz_chunk(int g, int j) {
  if (SPECENH_TOP1_SWZ)
    return 2 * (j >> 1) + (g >> 2) + 4 * ((j & 1) + 2 * ((g >> 1) & 1)) + 16 * (g & 1);
  return 8 * (g & 1) + (g >> 1) + 16 * (j & 1) + 4 * (j >> 1);
}
// X | Zt (4 x ZP, basis transposed) | U (N x 4) | part (4 waves x N x 4) | reduction scratch
constexpr size_t LDS_BYTES = (size_t)N * LD * 4 + 4 * ZP * 4 + N * 4 * 4 + 4 * N * 4 * 4 + 64 * 8;


// 1/sqrt(d) for d > 0: v_rsq_f64 plus one Newton step (the factors below only need to be
// consistent with each other, not correctly rounded)
__device__ __forceinline__ double rsq64(double d) {
  const double r = __builtin_amdgcn_rsq(d);
  return r * fma(-0.5 * d * r, r, 1.5);
}

// 4 x 4 Cholesky M = L L^T (lower) in fp64, returned as the strictly lower part of L and
// rinv = 1 / diag(L). A pivot below 1e-20 of its diagonal entry marks the column dead (its
// vector lies in the span of the earlier ones, or is zero): rinv = 0, column of L zero.
__device__ __forceinline__ void chol4(const double (&M)[4][4], double (&L)[4][4], double (&rinv)[4]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    double d = M[j][j];
#pragma unroll
    for (int l = 0; l < j; ++l) d = fma(-L[j][l], L[j][l], d);
    const bool live = d > 1e-20 * M[j][j] && d > 0.0;
    rinv[j] = live ? rsq64(d) : 0.0;
    L[j][j] = 0.0;
#pragma unroll
    for (int k = j + 1; k < 4; ++k) {
      double s = M[k][j];
#pragma unroll
      for (int l = 0; l < j; ++l) s = fma(-L[k][l], L[j][l], s);
      L[k][j] = s * rinv[j];
      L[j][k] = 0.0;
    }
  }
}

// solve z L^T = y for the row vector z (z = y R^-1 with R = L^T); dead columns -> 0
__device__ __forceinline__ void solve_row(const double (&L)[4][4], const double (&rinv)[4],
                                          const double (&y)[4], double (&z)[4]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    double s = y[j];
#pragma unroll
    for (int l = 0; l < j; ++l) s = fma(-z[l], L[j][l], s);
    z[j] = s * rinv[j];
  }
}

// cyclic Jacobi on a symmetric 4 x 4 in registers, fp32 (only the top eigenvector's
// direction and the second Ritz value are taken from it: the Rayleigh quotient and the
// residual test are redone in fp64). A -> diag, Q accumulates.
__device__ __forceinline__ void jacobi4(float (&A)[4][4], float (&Q)[4][4]) {
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) Q[a][b] = a == b ? 1.f : 0.f;
  for (int sweep = 0; sweep < 6; ++sweep) {
    float off = 0.f, dg = 0.f;
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      dg = fmaf(A[a][a], A[a][a], dg);
#pragma unroll
      for (int b = a + 1; b < 4; ++b) off = fmaf(A[a][b], A[a][b], off);
    }
    if (!(off > 1e-14f * dg)) break;  // uniform (every thread holds the same matrix)
#pragma unroll
    for (int pr = 0; pr < 6; ++pr) {
      const int p = pr < 3 ? 0 : (pr < 5 ? 1 : 2);
      const int q = pr < 3 ? pr + 1 : (pr < 5 ? pr - 1 : 3);
      const float apq = A[p][q];
      if (apq == 0.f) continue;
      const float tau = 0.5f * (A[q][q] - A[p][p]) * __builtin_amdgcn_rcpf(apq);
      const float t = copysignf(__builtin_amdgcn_rcpf(fabsf(tau) + __builtin_amdgcn_sqrtf(fmaf(tau, tau, 1.f))), tau);
      const float c = __builtin_amdgcn_rsqf(fmaf(t, t, 1.f)), s = t * c;
#pragma unroll
      for (int k = 0; k < 4; ++k) {  // columns p, q
        const float akp = A[k][p], akq = A[k][q];
        A[k][p] = c * akp - s * akq;
        A[k][q] = s * akp + c * akq;
        const float qkp = Q[k][p], qkq = Q[k][q];
        Q[k][p] = c * qkp - s * qkq;
        Q[k][q] = s * qkp + c * qkq;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {  // rows p, q
        const float apk = A[p][k], aqk = A[q][k];
        A[p][k] = c * apk - s * aqk;
        A[q][k] = s * apk + c * aqk;
      }
    }
  }
}

template <int CTRL>
__device__ __forceinline__ double dpp64(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xF, 0xF, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double readlane64(double v, int l) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, l);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
// sum over the 64 lanes of a wave (every lane active): DPP inside rows of 16 (quad
// swaps, half-row and row mirrors), then the four row sums; no LDS traffic
__device__ __forceinline__ double wave_sum64(double v) {
  v += dpp64<0xB1>(v);   // quad_perm [1, 0, 3, 2]
  v += dpp64<0x4E>(v);   // quad_perm [2, 3, 0, 1]
  v += dpp64<0x141>(v);  // row_half_mirror
  v += dpp64<0x140>(v);  // row_mirror
  return (readlane64(v, 0) + readlane64(v, 16)) + (readlane64(v, 32) + readlane64(v, 48));
}

// Sum NV doubles over the 128 threads of waves 0 and 1 (waves 2, 3 skip the wave sums);
// every thread returns the totals. One barrier; the caller separates reuse of sR.
template <int NV>
__device__ __forceinline__ void bsum128(double (&v)[NV], double* sR) {
  const int tid = threadIdx.x, w = tid >> 6;
  if (w < 2) {
#pragma unroll
    for (int j = 0; j < NV; ++j) v[j] = wave_sum64(v[j]);
    if ((tid & 63) == 0)
#pragma unroll
      for (int j = 0; j < NV; ++j) sR[w * NV + j] = v[j];
  }
  lds_sync();
#pragma unroll
  for (int j = 0; j < NV; ++j) v[j] = sR[j] + sR[NV + j];
}

// Gram entries of the 128-row blocks, fp64: value j < NV is sum_i A[i][a] A[i][b] for the
// pair n = j % 10 of the upper triangle of block j / 10 (0: Y, 1: Z, 2: U). Thread
// (j, c) sums 16 rows, the 8 partial sums meet through DPP inside each 8-lane group; every
// thread returns all NV sums. Y and U are row-major N x 4, Z transposed (4 x ZP). With
// SPECENH_TOP1_SWZ thread c takes rows 8 i + c (the 8 lanes of one j on 8 banks); the
// contiguous 16-row chunks (rows 16 c + i) put them on ONE bank of the row-major blocks
// (8-way: 1,936 of 2,192 LDS cycles of a check round, tools/lds_banks.py).
template <int NV>
__device__ __forceinline__ void gram_sums(const float* sY, const float* sZt, const float* sU,
                                          double* sRed) {
  const int t = threadIdx.x, j = t >> 3, c = t & 7;
  double s = 0.0;
  if (j < NV) {
    const int n = j % 10, src = j / 10;
    const int a = (int)((0x3221110000ULL >> (4 * n)) & 15);
    const int b = (int)((0x3323213210ULL >> (4 * n)) & 15);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int row = SPECENH_TOP1_SWZ ? 8 * i + c : 16 * c + i;
      const float va = src == 0 ? sY[4 * row + a] : (src == 1 ? sZt[zt(a, row)] : sU[4 * row + a]);
      const float vb = src == 0 ? sY[4 * row + b] : (src == 1 ? sZt[zt(b, row)] : sU[4 * row + b]);
      s = fma((double)va, (double)vb, s);
    }
  }
  s += dpp64<0xB1>(s);   // quad_perm [1, 0, 3, 2]
  s += dpp64<0x4E>(s);   // quad_perm [2, 3, 0, 1]
  s += dpp64<0x141>(s);  // row_half_mirror: the two quads of each 8-lane group
  if (c == 0 && j < NV) sRed[j] = s;
  lds_sync();
}

// symmetric 4 x 4 from the 10 upper-triangle sums at p (gram_sums order)
__device__ __forceinline__ void sym4(const double* p, double (&M)[4][4]) {
  int n = 0;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int c = a; c < 4; ++c) {
      M[a][c] = M[c][a] = p[n];
      ++n;
    }
}
}  // namespace top1

template <typename TO>
__global__ __launch_bounds__(256, 2) void top1_kernel(XView x, int Kr, int r, float tolv,
                                                       int* flags, TO* out, long long ob,
                                                       long long osk, long long osi,
                                                       long long batch, long long* phase_clk) {
  using namespace top1;
#ifdef SPECENH_TOP1_STATS  // development build: shader clocks per phase (thread 0)
  long long tacc[8], tlast;
#define T1_MARK(slot)                                      \
  do {                                                     \
    const long long now_ = __builtin_amdgcn_s_memtime();   \
    tacc[slot] += now_ - tlast;                            \
    tlast = now_;                                          \
  } while (0)
#else
#define T1_MARK(slot) \
  do {                \
  } while (0)
#endif
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* sX = reinterpret_cast<float*>(smem);  // N x LD
  float* sZt = sX + N * LD;                     // 4 x ZP
  float* sU = sZt + 4 * ZP;                     // N x 4
  float* sP = sU + 4 * N;                       // 4 x N x 4
  double* sR = reinterpret_cast<double*>(sP + 16 * N);  // 64
  double* vd = reinterpret_cast<double*>(sP);  // N: final v (fp64), after the iteration
  double* ud = vd + N;                            // N: u = X v
  double* hd = ud + N;                            // N: half sums
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
#ifdef SPECENH_TOP1_STATS
  for (int q = 0; q < 8; ++q) tacc[q] = 0;
  tlast = __builtin_amdgcn_s_memtime();
#endif
  const long long b = blockIdx.x;
  if (b >= batch) return;
  const float* X = x.base + b * x.batch_stride;

  // ---- stage X into LDS (zero-padded), ||X||_F^2 in fp64
  double fro = 0.0;
  if (x.si == 1) {  // rows of X contiguous: 16-byte loads along i, all in flight
    constexpr int NLD = N * N / 4 / 256;
    float4 v[NLD];
#pragma unroll
    for (int u = 0; u < NLD; ++u) {
      const int e = tid + 256 * u, k = e >> 5, i = 4 * (e & 31);
      v[u] = (k < Kr && i < r) ? *reinterpret_cast<const float4*>(X + (long long)k * x.sk + i)
                               : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < NLD; ++u) {
      const int e = tid + 256 * u, k = e >> 5, i = 4 * (e & 31);
      *reinterpret_cast<float4*>(sX + k * LD + i) = v[u];
      fro += (double)v[u].x * v[u].x + (double)v[u].y * v[u].y + (double)v[u].z * v[u].z +
             (double)v[u].w * v[u].w;
    }
  } else {  // X = A^T: contiguous along k
    for (int e = tid; e < N * N / 4; e += 256) {
      const int i = e >> 5, k = 4 * (e & 31);
      const float4 v = (k < Kr && i < r)
                           ? *reinterpret_cast<const float4*>(X + (long long)i * x.si + k)
                           : make_float4(0.f, 0.f, 0.f, 0.f);
      sX[k * LD + i] = v.x;
      sX[(k + 1) * LD + i] = v.y;
      sX[(k + 2) * LD + i] = v.z;
      sX[(k + 3) * LD + i] = v.w;
      fro += (double)v.x * v.x + (double)v.y * v.y + (double)v.z * v.z + (double)v.w * v.w;
    }
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) fro += __shfl_xor(fro, m);
  if (lane == 0) sR[32 + w] = fro;
  if (tid < N)
#pragma unroll
    for (int p = 0; p < 4; ++p)  // column 0 all ones (close to v1 for the non-negative
                                   // log spectrograms), the others pseudo-random
      sZt[zt(p, tid)] = tid < r ? (p == 0 ? 1.f : hash_unit(tid, p)) : 0.f;
  lds_sync();
  const double tr = (sR[32] + sR[33]) + (sR[34] + sR[35]);
  T1_MARK(0);

  // XZ: lane (row group kb, column group g): rows kb + 32 m (m < 4), 4 float4 column chunks
  // c(g, j) chosen so that the two groups of a 16-lane LDS window sit 32 banks apart
  const int kb = 8 * w + (lane & 7), g = lane >> 3;
  // XtU: lane (chunk cc = 4 columns, half h of the wave's 32 rows)
  const int cc = lane & 31, h = lane >> 5;
  float y[4], z[4], uk[4];  // thread i < N: row i of Y = G Z, of Z, and row k = i of U
  int bad = 1, t_used = 0;
  for (int t = 1;; ++t) {
    {  // U = X Z
      float a[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) a[q] = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = xz_chunk(g, j);
        float4 zv[4];
#pragma unroll
        for (int p = 0; p < 4; ++p) zv[p] = *reinterpret_cast<const float4*>(sZt + zt(p, 4 * c));
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const float4 xv = *reinterpret_cast<const float4*>(sX + (kb + 32 * m) * LD + 4 * c);
#pragma unroll
          for (int p = 0; p < 4; ++p) {
            float s = a[4 * m + p];
            s = fmaf(xv.x, zv[p].x, s);
            s = fmaf(xv.y, zv[p].y, s);
            s = fmaf(xv.z, zv[p].z, s);
            s = fmaf(xv.w, zv[p].w, s);
            a[4 * m + p] = s;
          }
        }
      }
      // reduce-scatter over the 8 column groups (lane bits 5, 4, 3): the lane keeps
      // rows m = g >> 1, columns p = 2 (g & 1) + {0, 1}
      const int b5 = (g >> 2) & 1, b4 = (g >> 1) & 1, b3 = g & 1;
      float a8[8], a4[4], a2[2];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float keep = b5 ? a[8 + q] : a[q], send = b5 ? a[q] : a[8 + q];
        a8[q] = keep + __shfl_xor(send, 32);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float keep = b4 ? a8[4 + q] : a8[q], send = b4 ? a8[q] : a8[4 + q];
        a4[q] = keep + __shfl_xor(send, 16);
      }
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const float keep = b3 ? a4[2 + q] : a4[q], send = b3 ? a4[q] : a4[2 + q];
        a2[q] = keep + __shfl_xor(send, 8);
      }
      *reinterpret_cast<float2*>(sU + 4 * (kb + 32 * (g >> 1)) + 2 * b3) = make_float2(a2[0], a2[1]);
    }
    lds_sync();
    T1_MARK(1);
    {  // Y = X^T U: wave w sums its 32 rows, lane halves 16 each
      float a[16];  // [column q][p]
#pragma unroll
      for (int q = 0; q < 16; ++q) a[q] = 0.f;
      const int k0 = 32 * w + 16 * h;
#pragma unroll 4
      for (int kk = 0; kk < 16; ++kk) {
        const float4 xv = *reinterpret_cast<const float4*>(sX + (k0 + kk) * LD + 4 * cc);
        const float4 uv = *reinterpret_cast<const float4*>(sU + 4 * (k0 + kk));
        const float xs[4] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          a[4 * q + 0] = fmaf(xs[q], uv.x, a[4 * q + 0]);
          a[4 * q + 1] = fmaf(xs[q], uv.y, a[4 * q + 1]);
          a[4 * q + 2] = fmaf(xs[q], uv.z, a[4 * q + 2]);
          a[4 * q + 3] = fmaf(xs[q], uv.w, a[4 * q + 3]);
        }
      }
      float a8[8];  // halves meet: h keeps columns 2h, 2h + 1
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float keep = h ? a[8 + q] : a[q], send = h ? a[q] : a[8 + q];
        a8[q] = keep + __shfl_xor(send, 32);
      }
      float* dst = sP + w * 4 * N;
      *reinterpret_cast<float4*>(dst + 4 * ppos(4 * cc + 2 * h)) = make_float4(a8[0], a8[1], a8[2], a8[3]);
      *reinterpret_cast<float4*>(dst + 4 * ppos(4 * cc + 2 * h + 1)) = make_float4(a8[4], a8[5], a8[6], a8[7]);
    }
    lds_sync();
    if (tid < N) {
      const int pt = ppos(tid);
      float4 s = *reinterpret_cast<const float4*>(sP + 4 * pt);
#pragma unroll
      for (int ww = 1; ww < 4; ++ww) {
        const float4 o = *reinterpret_cast<const float4*>(sP + ww * 4 * N + 4 * pt);
        s.x += o.x; s.y += o.y; s.z += o.z; s.w += o.w;
      }
      y[0] = s.x; y[1] = s.y; y[2] = s.z; y[3] = s.w;
      *reinterpret_cast<float4*>(sP + 4 * tid) = s;  // Y in place of wave 0's partials
      const float4 u4 = *reinterpret_cast<const float4*>(sU + 4 * tid);
      uk[0] = u4.x; uk[1] = u4.y; uk[2] = u4.z; uk[3] = u4.w;
#pragma unroll
      for (int p = 0; p < 4; ++p) z[p] = sZt[zt(p, tid)];
    } else {
#pragma unroll
      for (int p = 0; p < 4; ++p) y[p] = z[p] = uk[p] = 0.f;
    }
    lds_sync();
    // Rayleigh-Ritz + residual test at rounds 2, 3, 4, then every second round
    T1_MARK(2);
    const bool check = t >= 2 && (t <= 4 || t % 2 == 0 || t == MAX_ROUNDS);  // uniform
    // Gram sums in sR: [0, 10) Y^T Y (every round), [10, 20) Z^T Z, [20, 30) U^T U (checks)
    if (check) {
      gram_sums<30>(sP, sZt, sU, sR);
      double L[4][4], ri[4];
      {
        double M[4][4];
        sym4(sR + 10, M);
        chol4(M, L, ri);
      }
      double H[4][4];
      sym4(sR + 20, H);
      // C = L^-1 H L^-T with M = L L^T (dead basis columns: rows / columns of C zero)
      double W[4][4];
      float C[4][4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {  // W = L^-1 H, column by column
#pragma unroll
        for (int a = 0; a < 4; ++a) {
          double s = H[a][c];
#pragma unroll
          for (int l = 0; l < a; ++l) s = fma(-L[a][l], W[l][c], s);
          W[a][c] = s * ri[a];
        }
      }
#pragma unroll
      for (int c = 0; c < 4; ++c) {  // C = L^-1 W^T (lower triangle, mirrored)
        double col[4];
#pragma unroll
        for (int a = 0; a < 4; ++a) {
          double s = W[c][a];
#pragma unroll
          for (int l = 0; l < a; ++l) s = fma(-L[a][l], col[l], s);
          col[a] = s * ri[a];
        }
#pragma unroll
        for (int a = c; a < 4; ++a) C[a][c] = C[c][a] = (float)col[a];
      }
      float Q[4][4];
      jacobi4(C, Q);
      // top Ritz pair and the second Ritz value, without indexing registers dynamically
      float th1f = C[0][0], th2f = -3.0e38f, qt[4] = {Q[0][0], Q[1][0], Q[2][0], Q[3][0]};
#pragma unroll
      for (int a = 1; a < 4; ++a) {
        const bool gt = C[a][a] > th1f;
        th2f = fmaxf(th2f, gt ? th1f : C[a][a]);
        th1f = gt ? C[a][a] : th1f;
#pragma unroll
        for (int c = 0; c < 4; ++c) qt[c] = gt ? Q[c][a] : qt[c];
      }
      double q1[4];  // L^T q1 = qt (back substitution): v = Z q1 (unit norm up to fp32)
#pragma unroll
      for (int a = 3; a >= 0; --a) {
        double s = qt[a];
#pragma unroll
        for (int l = a + 1; l < 4; ++l) s = fma(-L[l][a], q1[l], s);
        q1[a] = s * ri[a];
      }
      double vi = 0.0, gv = 0.0;
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        vi = fma((double)z[p], q1[p], vi);
        gv = fma((double)y[p], q1[p], gv);  // (G v)_i
      }
      double rs[3] = {gv * vi, vi * vi, gv * gv};
      lds_sync();  // sR reuse
      bsum128<3>(rs, sR + 40);
      // fp64 Rayleigh quotient theta = v^T G v / v^T v and the residual of the normalised
      // v: ||G v - theta v||^2 / ||v||^2 = (g.g - theta g.v) / v.v
      const double vv = fmax(rs[1], 1e-300);
      const double th1 = rs[0] / vv;
      const double res2 = fmax(rs[2] - th1 * rs[0], 0.0) / vv;
      const double th2 = fmin((double)th2f, th1);
      // Accuracy target on the OUTPUT: after the fp64 power step below, the error of v is
      // at most f * res / gap with f = theta_2 / theta_1 <= (tr - theta_1) / theta_1, and
      // the output error ~ sqrt(theta_1) * that, against tolv * ||out||_F where
      // ||out||_F^2 = tr - theta_1 (floored at 1e-4 tr: 1% of ||X||_F, rank-1 inputs)
      const double rest = fmax(tr - th1, 1e-4 * fmax(tr, 0.0));
      const double f = fmin(1.0, rest / fmax(th1, 1e-300));
      const bool conv = sqrt(fmax(th1, 0.0) * res2) * f <= (double)tolv * (th1 - th2) * sqrt(rest);
      if (conv || t >= MAX_ROUNDS) {  // uniform
        bad = conv ? 0 : 1;
        t_used = t;
        if (tid < N) vd[tid] = vi * rsq64(vv);  // v / ||v|| (partials were read above)
        T1_MARK(4);
        break;
      }
      T1_MARK(4);
    } else {
      gram_sums<10>(sP, sZt, sU, sR);
    }
    // Z = Y R^-1 (CholeskyQR, S = R^T R): each thread rewrites its own column of Zt
    double L[4][4], ri[4], yd[4], zd[4];
    {
      double S[4][4];
      sym4(sR, S);
      chol4(S, L, ri);
    }
    if (tid < N) {
#pragma unroll
      for (int p = 0; p < 4; ++p) yd[p] = y[p];
      solve_row(L, ri, yd, zd);
#pragma unroll
      for (int p = 0; p < 4; ++p) sZt[zt(p, tid)] = (float)zd[p];
    }
    lds_sync();
    T1_MARK(3);
  }
  // ---- one power step in fp64 from the converged v: v <- X^T X v / ||X^T X v||, then
  // u = X v, so that fp32 rounding in the iteration (relative ~1e-6, amplified by
  // sigma_1 / ||out||_F in the output) is damped by theta_2 / theta_1
  auto Xv = [&]() {  // ud = X vd: thread (row k, column half h)
    const int k = tid & (N - 1), h = tid >> 7;
    const float* xr = sX + k * LD + 64 * h;
    const double* vv = vd + 64 * h;
    double s0 = 0.0, s1 = 0.0;
#pragma unroll 4
    for (int j = 0; j < 16; ++j) {
      const float4 x4 = *reinterpret_cast<const float4*>(xr + 4 * j);
      const double2 v01 = *reinterpret_cast<const double2*>(vv + 4 * j);
      const double2 v23 = *reinterpret_cast<const double2*>(vv + 4 * j + 2);
      s0 = fma((double)x4.x, v01.x, s0);
      s1 = fma((double)x4.y, v01.y, s1);
      s0 = fma((double)x4.z, v23.x, s0);
      s1 = fma((double)x4.w, v23.y, s1);
    }
    if (h) hd[k] = s0 + s1;
    lds_sync();
    if (!h) ud[k] = (s0 + s1) + hd[k];
    lds_sync();
  };
  lds_sync();
  Xv();
  {  // w = X^T u: thread (column i, row half h); v = w / ||w||
    const int i = tid & (N - 1), h = tid >> 7;
    double s0 = 0.0, s1 = 0.0;
#pragma unroll 8
    for (int kk = 0; kk < 64; kk += 2) {
      const int k = 64 * h + kk;
      s0 = fma((double)sX[k * LD + i], ud[k], s0);
      s1 = fma((double)sX[(k + 1) * LD + i], ud[k + 1], s1);
    }
    if (h) hd[i] = s0 + s1;
    lds_sync();
    const double w = h ? 0.0 : (s0 + s1) + hd[i];
    double nn[1] = {w * w};
    bsum128<1>(nn, sR + 40);
    if (!h) vd[i] = nn[0] > 0.0 ? w * rsq64(nn[0]) : 0.0;
    lds_sync();
  }
  Xv();
  T1_MARK(5);
#ifdef SPECENH_TOP1_STATS  // development build (tools/top1_stats.py): rounds in the flag word
  if (flags && tid == 0) flags[b] = bad + 2 * t_used;
#else
  if (flags && tid == 0) flags[b] = bad;
#endif
  // ---- out = X - u v^T (fp64, rounded once to fp32) in A's orientation
  TO* Ob = out + b * ob;
  if (osi == 1) {
    for (int e = tid; e < Kr * (r / 4); e += 256) {
      const int k = e / (r / 4), i = 4 * (e % (r / 4));
      const float4 xv = *reinterpret_cast<const float4*>(sX + k * LD + i);
      const double2 v01 = *reinterpret_cast<const double2*>(vd + i);
      const double2 v23 = *reinterpret_cast<const double2*>(vd + i + 2);
      const double u = ud[k];
      TO* o = Ob + (long long)k * osk + i;
      o[0] = to_out<TO>((float)fma(-u, v01.x, (double)xv.x));
      o[1] = to_out<TO>((float)fma(-u, v01.y, (double)xv.y));
      o[2] = to_out<TO>((float)fma(-u, v23.x, (double)xv.z));
      o[3] = to_out<TO>((float)fma(-u, v23.y, (double)xv.w));
    }
  } else {  // contiguous along k
    for (int e = tid; e < r * (Kr / 4); e += 256) {
      const int i = e / (Kr / 4), k = 4 * (e % (Kr / 4));
      const double vi = vd[i];
      TO* o = Ob + (long long)i * osi + k;
#pragma unroll
      for (int c = 0; c < 4; ++c)
        o[c] = to_out<TO>((float)fma(-ud[k + c], vi, (double)sX[(k + c) * LD + i]));
    }
  }
  T1_MARK(6);
#ifdef SPECENH_TOP1_STATS
  if (phase_clk && tid == 0)
    for (int q = 0; q < 8; ++q) phase_clk[b * 8 + q] = tacc[q];
#endif
#undef T1_MARK
}


// ---------------------------------------------------------------- optimal hard threshold
// use_optimal / computeSignal (denoising_by_svd.ipynb:174-181, 210-217) need the median of
// ALL singular values and how many exceed omega(beta) * median. They come from the
// eigenvalues of the Gram matrix in fp64 (the noise singular values sit ~1e-3 below the
// largest; an fp32 Gram would bury their squares in its rounding): Householder reduction
// to tridiagonal form, then Sturm-count bisection for exactly the three numbers needed
// (the two middle order statistics and the count above the threshold).

// fp64 Gram G = X^T X: 64x64 tile per workgroup (upper-triangle tiles, mirrored), 16 rows
// of X per LDS stage, 4x4 outputs per thread. Products of fp32 inputs are exact in fp64.
__device__ __forceinline__ void gram64_one(XView x, int K, int r, double* G, int nts,
                                           long long b, int tile) {
  __shared__ double sa[16][65], sb[16][65];
  int t = tile, ti = 0;
  while (t >= nts - ti) {
    t -= nts - ti;
    ++ti;
  }
  const int tj = ti + t;
  const float* X = x.base + b * x.batch_stride;
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  double acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = 0.0;
  for (int k0 = 0; k0 < K; k0 += 16) {
    for (int idx = tid; idx < 16 * 64; idx += 256) {
      int kk, c;
      if (x.si == 1) {  // rows of X contiguous: coalesce along the column index
        kk = idx >> 6;
        c = idx & 63;
      } else {
        c = idx >> 4;
        kk = idx & 15;
      }
      const int k = k0 + kk, ci = ti * 64 + c, cj = tj * 64 + c;
      sa[kk][c] = (k < K && ci < r) ? (double)X[(long long)k * x.sk + (long long)ci * x.si] : 0.0;
      sb[kk][c] = (k < K && cj < r) ? (double)X[(long long)k * x.sk + (long long)cj * x.si] : 0.0;
    }
    __syncthreads();
#pragma unroll 4
    for (int kk = 0; kk < 16; ++kk) {
      double av[4], bv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        av[i] = sa[kk][ty * 4 + i];
        bv[i] = sb[kk][tx * 4 + i];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fma(av[i], bv[j], acc[i][j]);
    }
    __syncthreads();
  }
  double* Gb = G + b * (long long)r * r;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = ti * 64 + ty * 4 + i, col = tj * 64 + tx * 4 + j;
      if (row < r && col < r) {
        Gb[(long long)row * r + col] = acc[i][j];
        Gb[(long long)col * r + row] = acc[i][j];
      }
    }
}

// The fallback kernels below loop over matrices b = blockIdx.y (.x), + gridDim: as the fp64
// path behind top1 / the subspace kernels (`only`: the few flagged matrices) they launch a
// small grid, not one workgroup per matrix that mostly returns at once (four such launches
// cost ~25 us per 4096-matrix C5 step); without `only` the grid covers every matrix.
__global__ __launch_bounds__(256) void gram64_kernel(XView x, int K, int r, double* G, int nts,
                                                     const int* only, long long nmat) {
  for (long long b = blockIdx.y; b < nmat; b += gridDim.y) {
    if (only && !only[b]) continue;  // uniform: matrix not selected
    gram64_one(x, K, r, G, nts, b, blockIdx.x);
    __syncthreads();  // (LDS reused by the next matrix)
  }
}


__device__ __forceinline__ double block_sum256(double v, double* red) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
  __syncthreads();  // red is reused call after call
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

// Householder tridiagonalisation of the symmetric n x n fp64 matrix A (in place, global,
// n <= 256, one workgroup per matrix; thread i owns column i of the trailing block):
// d = diagonal, e = off-diagonal. Step k: v from A[k+1:, k], p = tau A22 v,
// w = p - (tau/2)(p.v) v, A22 -= v w^T + w v^T (LAPACK dsytd2 / dlarfg arithmetic).
// With taug, the reflectors are kept for the eigenvector back-transform: v_k (v_k[0] = 1
// implicit) overwrites row k right of the diagonal (never read again), tau_k -> taug[k];
// G = Q T Q^T with Q = H_0 H_1 ... H_{n-3}.
__device__ __forceinline__ void tridiag_one(double* G, int n, double* dg, double* eg,
                                            double* taug, long long b) {
  __shared__ double sv[256], sw[256], red[4];
  double* A = G + b * (long long)n * n;
  double* d = dg + b * n;
  double* e = eg + b * n;
  double* taub = taug ? taug + b * n : nullptr;
  const int tid = threadIdx.x;
  for (int k = 0; k + 2 < n; ++k) {
    const int len = n - k - 1;
    double* rowk = A + (long long)k * n + k + 1;  // = column k below the diagonal
    const double xv = tid < len ? rowk[tid] : 0.0;
    const double s2 = block_sum256(tid >= 1 && tid < len ? xv * xv : 0.0, red);
    const double alpha = rowk[0];
    if (tid == 0) d[k] = A[(long long)k * n + k];
    if (s2 == 0.0) {  // uniform: already tridiagonal in this column
      if (tid == 0) {
        e[k] = alpha;
        if (taub) taub[k] = 0.0;
      }
      continue;
    }
    const double beta = -copysign(sqrt(alpha * alpha + s2), alpha);
    const double tau = (beta - alpha) / beta;
    const double scal = 1.0 / (alpha - beta);
    if (tid == 0) {
      e[k] = beta;
      if (taub) taub[k] = tau;
    }
    const double vi = tid == 0 ? 1.0 : (tid < len ? xv * scal : 0.0);
    if (tid < len) sv[tid] = vi;
    if (taub && tid >= 1 && tid < len) rowk[tid] = vi;  // rowk[0] (alpha) is read above
    __syncthreads();
    double p = 0.0;
    if (tid < len) {
      const double* col = A + (long long)(k + 1) * n + (k + 1) + tid;
#pragma unroll 8
      for (int j = 0; j < len; ++j) p = fma(col[(long long)j * n], sv[j], p);
      p *= tau;
    }
    const double pv = block_sum256(tid < len ? p * vi : 0.0, red);
    const double w = p - 0.5 * tau * pv * vi;
    if (tid < len) sw[tid] = w;
    __syncthreads();
    if (tid < len) {
      double* col = A + (long long)(k + 1) * n + (k + 1) + tid;
#pragma unroll 8
      for (int j = 0; j < len; ++j) col[(long long)j * n] -= sv[j] * w + sw[j] * vi;
    }
    __syncthreads();  // the next step reads what other threads just wrote (same CU)
  }
  if (tid == 0) {
    if (n >= 2) {
      d[n - 2] = A[(long long)(n - 2) * n + n - 2];
      e[n - 2] = A[(long long)(n - 2) * n + n - 1];
    }
    d[n - 1] = A[(long long)(n - 1) * n + n - 1];
  }
}

__global__ __launch_bounds__(256) void tridiag_kernel(double* G, int n, double* dg, double* eg,
                                                      double* taug, const int* only,
                                                      long long nmat) {
  for (long long b = blockIdx.x; b < nmat; b += gridDim.x) {
    if (only && !only[b]) continue;
    tridiag_one(G, n, dg, eg, taug, b);
    __syncthreads();
  }
}


// Number of eigenvalues < x of the symmetric tridiagonal (d, e2 = e^2) (Sturm sequence,
// LAPACK dstebz pivmin guard).
__device__ int sturm_count(const double* d, const double* e2, int n, double x, double pivmin) {
  double q = d[0] - x;
  if (fabs(q) < pivmin) q = -pivmin;
  int c = q < 0.0;
  for (int i = 1; i < n; ++i) {
    q = d[i] - x - e2[i - 1] / q;
    if (fabs(q) < pivmin) q = -pivmin;
    c += q < 0.0;
  }
  return c;
}

// k-th smallest eigenvalue (0-based) by 65-way multisection: each lane counts at one point.
__device__ double kth_eig(const double* d, const double* e2, int n, int k, double lo, double hi,
                          double pivmin, int lane) {
  for (int it = 0; it < 16 && hi > lo; ++it) {
    const double x = lo + (hi - lo) * (double)(lane + 1) / 65.0;
    const int c = sturm_count(d, e2, n, x, pivmin);
    const unsigned long long m = __ballot(c > k);
    const int first = m ? __ffsll((long long)m) - 1 : 64;
    const double nlo = first == 0 ? lo : lo + (hi - lo) * (double)first / 65.0;
    const double nhi = first == 64 ? hi : lo + (hi - lo) * (double)(first + 1) / 65.0;
    if (!(nhi < hi) && !(nlo > lo)) break;  // no progress at double resolution
    lo = nlo;
    hi = nhi;
  }
  return 0.5 * (lo + hi);
}

// One wave per matrix: median singular value and num_sing = #(s > omega * median)
// (s = sqrt(max(lambda, 0)), lambda the Gram eigenvalues; numpy's median of r values).
__global__ __launch_bounds__(64) void optimal_rank_kernel(const double* dg, const double* eg,
                                                          int n, double omega, int* num_sing,
                                                          double* median) {
  __shared__ double sd[256], se2[256];
  const long long b = blockIdx.x;
  const int lane = threadIdx.x;
  double lo = INFINITY, hi = -INFINITY, emax = 0.0;
  for (int i = lane; i < n; i += 64) {
    const double di = dg[b * n + i];
    const double el = i > 0 ? fabs(eg[b * n + i - 1]) : 0.0;
    const double er = i + 1 < n ? fabs(eg[b * n + i]) : 0.0;
    sd[i] = di;
    if (i + 1 < n) se2[i] = er * er;
    lo = fmin(lo, di - el - er);
    hi = fmax(hi, di + el + er);
    emax = fmax(emax, er * er);
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    lo = fmin(lo, __shfl_xor(lo, m));
    hi = fmax(hi, __shfl_xor(hi, m));
    emax = fmax(emax, __shfl_xor(emax, m));
  }
  __syncthreads();
  const double span = fmax(hi - lo, fmax(fabs(hi), fabs(lo))) * 4e-16 + 1e-300;
  lo -= span;
  hi += span;
  const double pivmin = 2.2250738585072014e-308 * fmax(1.0, emax);
  double med;
  if (n & 1) {
    med = sqrt(fmax(kth_eig(sd, se2, n, n / 2, lo, hi, pivmin, lane), 0.0));
  } else {
    const double a1 = kth_eig(sd, se2, n, n / 2 - 1, lo, hi, pivmin, lane);
    const double a2 = kth_eig(sd, se2, n, n / 2, lo, hi, pivmin, lane);
    med = 0.5 * (sqrt(fmax(a1, 0.0)) + sqrt(fmax(a2, 0.0)));
  }
  const double t = omega * med;
  const int below = sturm_count(sd, se2, n, t * t, pivmin);  // s < t (s == t: measure zero)
  if (lane == 0) {
    num_sing[b] = n - below;
    if (median) median[b] = med;
  }
}

// ---------------------------------------------------------------- any kept range
// A kept range [lo, hi) that would need more than a top-40 subspace, or the bottom of the
// spectrum (a negative stop, use_optimal with num_sing == 0: denoising_by_svd.ipynb:216-228),
// is reconstructed from eigenvectors of the fp64 Gram matrix: Householder tridiagonal form
// (tridiag_kernel, reflectors kept), Sturm bisection for each selected eigenvalue, inverse
// iteration on the tridiagonal (LU with partial pivoting, LAPACK dlagtf/dlagts arithmetic;
// near-degenerate eigenvalues are iterated in sequence and orthogonalised against each other
// as dstein does), the reflectors applied back, then out = X V V^T for the kept set, or
// out = X - X V V^T for its complement, whichever set is smaller (<= r/2 vectors).
constexpr int EIG_MAXN = 256;
constexpr int EIG_ITERS = 4;

// Kept components [lo, hi) (descending singular values) -> selected ascending eigen-indices
// [p0, p1) u [q0, q1) and the complement flag.
__device__ __forceinline__ void eig_select(int r, int lo, int hi, int& p0, int& p1, int& q0,
                                           int& q1, int& comp) {
  lo = max(lo, 0);
  hi = min(hi, r);
  p0 = p1 = q0 = q1 = 0;
  comp = 0;
  if (hi <= lo) return;
  if (lo + (r - hi) < hi - lo) {
    comp = 1;
    p1 = r - hi;
    q0 = r - lo;
    q1 = r;
  } else {
    p0 = r - hi;
    p1 = r - lo;
  }
}

// lambda_idx (ascending, 0-based) by bisection on the Sturm count, to an absolute width of
// a few ulps of ||T|| (what inverse iteration needs).
__device__ double eig_bisect(const double* d, const double* e2, int n, int idx, double lo,
                             double hi, double pivmin, double atol) {
  for (int it = 0; it < 96; ++it) {
    const double mid = 0.5 * (lo + hi);
    if (hi - lo <= atol || !(mid > lo && mid < hi)) break;
    if (sturm_count(d, e2, n, mid, pivmin) > idx) hi = mid;
    else lo = mid;
  }
  return 0.5 * (lo + hi);
}

// y <- (T - lam I)^{-1} y, arrays strided by ld. dlagtf's factorisation (partial pivoting,
// U with two super-diagonals kept in ua/ub/ud) fused with the forward application of L,
// then back substitution with pivots below tol perturbed to +-tol (dlagts job = -1).
__device__ void tri_inverse_solve(const double* d, const double* e, int n, double lam,
                                  double tol, double* y, double* ua, double* ub, double* ud,
                                  long long ld) {
  double a = d[0] - lam, bsup = n > 1 ? e[0] : 0.0, yk = y[0];
  for (int k = 0; k + 1 < n; ++k) {
    const double c = e[k], an = d[k + 1] - lam, bn = k + 2 < n ? e[k + 1] : 0.0;
    const double yn = y[(long long)(k + 1) * ld];
    if (fabs(a) >= fabs(c)) {  // row k pivots: [a, bsup] over [c, an, bn]
      const double mult = a != 0.0 ? c / a : 0.0;
      ua[k * ld] = a;
      ub[k * ld] = bsup;
      ud[k * ld] = 0.0;
      y[k * ld] = yk;
      a = an - mult * bsup;
      bsup = bn;
      yk = yn - mult * yk;
    } else {  // interchange: row k+1 pivots
      const double mult = a / c;
      ua[k * ld] = c;
      ub[k * ld] = an;
      ud[k * ld] = bn;
      y[k * ld] = yn;
      a = bsup - mult * an;
      bsup = -mult * bn;
      yk = yk - mult * yn;
    }
  }
  ua[(long long)(n - 1) * ld] = a;
  y[(long long)(n - 1) * ld] = yk;
  double x1 = 0.0, x2 = 0.0;  // x[k+1], x[k+2]
  for (int k = n - 1; k >= 0; --k) {
    double piv = ua[k * ld];
    if (fabs(piv) < tol) piv = piv < 0.0 ? -tol : tol;
    const double u1 = k + 1 < n ? ub[k * ld] : 0.0, u2 = k + 2 < n ? ud[k * ld] : 0.0;
    const double xk = (y[k * ld] - u1 * x1 - u2 * x2) / piv;
    y[k * ld] = xk;
    x2 = x1;
    x1 = xk;
  }
}

__device__ void col_normalize(double* y, int n, long long ld) {
  double mx = 0.0;
  for (int i = 0; i < n; ++i) mx = fmax(mx, fabs(y[i * ld]));
  if (!(mx > 0.0) || !isfinite(mx)) {  // degenerate solve: restart from a unit vector
    for (int i = 0; i < n; ++i) y[i * ld] = i == 0 ? 1.0 : 0.0;
    return;
  }
  double s = 0.0;
  for (int i = 0; i < n; ++i) {
    const double v = y[i * ld] / mx;
    s = fma(v, v, s);
  }
  const double inv = 1.0 / (mx * sqrt(s));
  for (int i = 0; i < n; ++i) y[i * ld] *= inv;
}

// One workgroup per matrix. ranges (device int[2 * batch]) gives a per-matrix kept [lo, hi),
// else the uniform (lo, hi). Writes the selected eigenvectors of G (Q z, fp64) to
// Z[b][i][j] (row stride ld) and kinfo[b] = {count, complement}.
__device__ __forceinline__ void eigvec_one(const double* G, const double* dg,
                                                     const double* eg, const double* taug, int n,
                                                     int lo, int hi, const int* ranges, double* Z,
                                                     double* fac, long long ld, int* kinfo,
                                                     long long b) {
  __shared__ double sd[EIG_MAXN], se[EIG_MAXN], se2[EIG_MAXN], slam[EIG_MAXN], sv[EIG_MAXN];
  __shared__ int sidx[EIG_MAXN], slead[EIG_MAXN];
  __shared__ double red[4];
  const int tid = threadIdx.x;
  if (ranges) {
    lo = ranges[2 * b];
    hi = ranges[2 * b + 1];
  }
  int p0, p1, q0, q1, comp;
  eig_select(n, lo, hi, p0, p1, q0, q1, comp);
  const int np = p1 - p0, k = np + (q1 - q0);
  if (tid == 0) {
    kinfo[2 * b] = k;
    kinfo[2 * b + 1] = comp;
  }
  if (k == 0) return;  // uniform per workgroup
  double gl = INFINITY, gu = -INFINITY, emax = 0.0;
  for (int i = tid; i < n; i += 256) {
    const double di = dg[b * n + i];
    const double el = i > 0 ? fabs(eg[b * n + i - 1]) : 0.0;
    const double er = i + 1 < n ? fabs(eg[b * n + i]) : 0.0;
    sd[i] = di;
    se[i] = i + 1 < n ? eg[b * n + i] : 0.0;
    se2[i] = er * er;
    gl = fmin(gl, di - el - er);
    gu = fmax(gu, di + el + er);
    emax = fmax(emax, er * er);
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    gl = fmin(gl, __shfl_xor(gl, m));
    gu = fmax(gu, __shfl_xor(gu, m));
    emax = fmax(emax, __shfl_xor(emax, m));
  }
  __syncthreads();
  if ((tid & 63) == 0) {
    red[tid >> 6] = gl;
  }
  __syncthreads();
  gl = fmin(fmin(red[0], red[1]), fmin(red[2], red[3]));
  __syncthreads();
  if ((tid & 63) == 0) red[tid >> 6] = gu;
  __syncthreads();
  gu = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
  __syncthreads();
  if ((tid & 63) == 0) red[tid >> 6] = emax;
  __syncthreads();
  emax = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
  const double tnorm = fmax(fabs(gl), fabs(gu)) + 1e-300;
  const double eps = 2.220446049250313e-16;
  gl -= 4.0 * eps * tnorm;
  gu += 4.0 * eps * tnorm;
  const double pivmin = 2.2250738585072014e-308 * fmax(1.0, emax);
  // 1. eigenvalues of the selected indices (ascending)
  for (int j = tid; j < k; j += 256) {
    const int idx = j < np ? p0 + j : q0 + (j - np);
    sidx[j] = idx;
    slam[j] = eig_bisect(sd, se2, n, idx, gl, gu, pivmin, 2.0 * eps * tnorm);
  }
  __syncthreads();
  // 2. clusters: consecutive indices closer than 1e-9 ||T|| share one sequential chain
  const double ctol = 1e-9 * tnorm;
  for (int j = tid; j < k; j += 256)
    slead[j] = (j == 0 || sidx[j] != sidx[j - 1] + 1 || slam[j] - slam[j - 1] > ctol) ? 1 : 0;
  __syncthreads();
  double* Zb = Z + b * (long long)n * ld;
  double* fa = fac + b * (long long)n * ld * 3;
  // 3. inverse iteration; a chain leader runs its whole cluster in order (dstein)
  const double tol = eps * tnorm;
  for (int j0 = tid; j0 < k; j0 += 256) {
    if (!slead[j0]) continue;
    for (int j = j0; j < k && (j == j0 || !slead[j]); ++j) {
      double* y = Zb + j;
      for (int i = 0; i < n; ++i)
        y[i * ld] = hash_unit((unsigned)i, (unsigned)(sidx[j] * 7919 + 17)) + (i == sidx[j] % n ? 0.25 : 0.0);
      for (int it = 0; it < EIG_ITERS; ++it) {
        for (int q = j0; q < j; ++q) {  // orthogonalise against the cluster's earlier vectors
          const double* z = Zb + q;
          double dot = 0.0;
          for (int i = 0; i < n; ++i) dot = fma(z[i * ld], y[i * ld], dot);
          for (int i = 0; i < n; ++i) y[i * ld] = fma(-dot, z[i * ld], y[i * ld]);
        }
        col_normalize(y, n, ld);
        tri_inverse_solve(sd, se, n, slam[j], tol, y, fa + j, fa + ld * n + j,
                          fa + 2 * ld * n + j, ld);
        col_normalize(y, n, ld);
      }
      for (int q = j0; q < j; ++q) {  // final orthogonalisation within the cluster
        const double* z = Zb + q;
        double dot = 0.0;
        for (int i = 0; i < n; ++i) dot = fma(z[i * ld], y[i * ld], dot);
        for (int i = 0; i < n; ++i) y[i * ld] = fma(-dot, z[i * ld], y[i * ld]);
      }
      col_normalize(y, n, ld);
    }
  }
  __syncthreads();
  // 4. back-transform: z <- H_0 (H_1 (... H_{n-3} z)), reflector k lives in row k of G
  const double* Gb = G + b * (long long)n * n;
  const double* taub = taug + b * n;
  for (int kk = n - 3; kk >= 0; --kk) {
    const double tau = taub[kk];
    if (tau == 0.0) continue;  // uniform
    const int len = n - kk - 1;
    for (int t = tid; t < len; t += 256) sv[t] = t == 0 ? 1.0 : Gb[(long long)kk * n + kk + 1 + t];
    __syncthreads();
    for (int j = tid; j < k; j += 256) {
      double* z = Zb + (long long)(kk + 1) * ld + j;
      double dot = 0.0;
      for (int t = 0; t < len; ++t) dot = fma(sv[t], z[t * ld], dot);
      dot *= tau;
      for (int t = 0; t < len; ++t) z[t * ld] = fma(-dot, sv[t], z[t * ld]);
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void eigvec_kernel(const double* G, const double* dg,
                                                     const double* eg, const double* taug, int n,
                                                     int lo, int hi, const int* ranges, double* Z,
                                                     double* fac, long long ld, int* kinfo,
                                                     const int* only, long long nmat) {
  for (long long b = blockIdx.x; b < nmat; b += gridDim.x) {
    if (only && !only[b]) continue;
    eigvec_one(G, dg, eg, taug, n, lo, hi, ranges, Z, fac, ld, kinfo, b);
    __syncthreads();
  }
}


// Per-matrix kept ranges of the optimal modes from num_sing, with the notebook's slicing:
// use_optimal keeps u[:, 0:num_sing-1] (:216-228; num_sing == 0 -> stop = -1 -> [0, r-1)),
// computeSignal keeps [1, 2 num_sing) (:181-185; 2 num_sing > r is an IndexError, flagged).
__global__ void optimal_ranges_kernel(const int* num, long long batch, int r, int mode,
                                      int* ranges, int* bad) {
  const long long b = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (b >= batch) return;
  const int ns = num[b];
  int lo, hi;
  if (mode == SPECENH_SVD_OPTIMAL) {
    lo = 0;
    hi = ns - 1;
    if (hi < 0) hi = max(hi + r, 0);  // Python slice bound
  } else {
    lo = 1;
    hi = 2 * ns;
    if (ns > 0 && hi > r) {
      atomicOr(bad, 1);
      hi = r;
    }
  }
  ranges[2 * b] = min(lo, r);
  ranges[2 * b + 1] = min(hi, r);
}

// out = X V V^T (complement = 0) or X - X V V^T, V = the count selected columns of Z[b]
// (fp64, cast to fp32 in LDS). Workgroup = (matrix, RB rows of X); thread i owns column i
// of the row block (r <= 256), V streams through LDS 32 columns at a time.
template <typename TO>
__device__ __forceinline__ void recon_eig_one(XView x, int Kr, int r, const double* Z,
                                              long long ld, const int* kinfo, TO* out,
                                              long long out_bstride, long long osk,
                                              long long osi, long long b, int kb) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* sX = reinterpret_cast<float*>(smem);  // RB x (r + 1)
  float* sV = sX + RB * (r + 1);                // r x 33
  float* sY = sV + r * 33;                      // RB x 33
  const int kc = kinfo[2 * b], comp = kinfo[2 * b + 1];
  const int k0 = kb * RB, tid = threadIdx.x;
  const int rows = min(RB, Kr - k0);
  const float* X = x.base + b * x.batch_stride;
  if (x.si == 1) {
    for (int idx = tid; idx < RB * r; idx += 256) {
      const int kk = idx / r, i = idx % r;
      sX[kk * (r + 1) + i] = kk < rows ? X[(long long)(k0 + kk) * x.sk + i] : 0.f;
    }
  } else {
    for (int idx = tid; idx < RB * r; idx += 256) {
      const int i = idx / RB, kk = idx % RB;
      sX[kk * (r + 1) + i] = kk < rows ? X[(long long)(k0 + kk) * x.sk + (long long)i * x.si] : 0.f;
    }
  }
  float acc[RB];
#pragma unroll
  for (int kk = 0; kk < RB; ++kk) acc[kk] = 0.f;
  const double* Zb = Z + b * (long long)r * ld;
  for (int c0 = 0; c0 < kc; c0 += 32) {
    __syncthreads();  // sX staged / previous chunk consumed
    for (int idx = tid; idx < r * 32; idx += 256) {
      const int i = idx >> 5, c = idx & 31;
      sV[i * 33 + c] = c0 + c < kc ? (float)Zb[(long long)i * ld + c0 + c] : 0.f;
    }
    __syncthreads();
    for (int e = tid; e < RB * 32; e += 256) {
      const int kk = e >> 5, c = e & 31;
      float s = 0.f;
      for (int i = 0; i < r; ++i) s = fmaf(sX[kk * (r + 1) + i], sV[i * 33 + c], s);
      sY[kk * 33 + c] = s;
    }
    __syncthreads();
    if (tid < r) {
#pragma unroll
      for (int kk = 0; kk < RB; ++kk) {
        float s = acc[kk];
#pragma unroll 8
        for (int c = 0; c < 32; ++c) s = fmaf(sY[kk * 33 + c], sV[tid * 33 + c], s);
        acc[kk] = s;
      }
    }
  }
  __syncthreads();
  if (tid < r) {
    TO* Ob = out + b * out_bstride;
#pragma unroll
    for (int kk = 0; kk < RB; ++kk) {
      if (kk >= rows) break;
      const float v = comp ? sX[kk * (r + 1) + tid] - acc[kk] : acc[kk];
      Ob[(long long)(k0 + kk) * osk + (long long)tid * osi] = to_out<TO>(v);
    }
  }
}

template <typename TO>
__global__ __launch_bounds__(256) void recon_eig_kernel(XView x, int Kr, int r, const double* Z,
                                                        long long ld, const int* kinfo, TO* out,
                                                        long long out_bstride, long long osk,
                                                        long long osi, const int* only,
                                                        long long nmat) {
  for (long long b = blockIdx.y; b < nmat; b += gridDim.y) {
    if (only && !only[b]) continue;
    recon_eig_one<TO>(x, Kr, r, Z, ld, kinfo, out, out_bstride, osk, osi, b, blockIdx.x);
    __syncthreads();
  }
}


}  // namespace specenh

using namespace specenh;

namespace {

// G = X^T X for every matrix: the LDS-chunked kernel for r <= 128 (r % 4 == 0), else
// one wave per 32x32 tile.
void launch_gram(const XView& xv, int Kr, int r, float* G, long long batch, hipStream_t st) {
  // float4 row loads need 16-B aligned rows when X is row-major
  const bool vec_ok = xv.si != 1 || (xv.sk % 4 == 0 && xv.batch_stride % 4 == 0 &&
                                     (reinterpret_cast<uintptr_t>(xv.base) & 15) == 0);
  const bool lds = r <= 128 && r % 4 == 0 && variant(V_SVD_GRAM_TILES) == 0;
  const bool split = r > 128 && r <= 256 && variant(V_SVD_GRAM_TILES) == 0 &&
                     variant(V_SVD_GRAM_F32) == 0;
  const bool lds256 = r > 128 && r <= 256 && r % 4 == 0 && vec_ok &&
                      variant(V_SVD_GRAM_TILES) == 0;
  const int nts = (r + 31) / 32;
  const int ntri = nts * (nts + 1) / 2;
  for (long long b0 = 0; b0 < batch; b0 += 65535) {
    const long long nb = std::min<long long>(65535, batch - b0);
    XView xb = xv;
    xb.base = xv.base + b0 * xv.batch_stride;
    if (split)
      SPECENH_LAUNCH(gram256s_kernel, dim3((unsigned)nb), dim3(256), 0, st, xb, Kr, r,
                     G + b0 * (long long)r * r);
    else if (lds)
      SPECENH_LAUNCH(gram_lds_kernel, dim3((unsigned)nb), dim3(256), 0, st, xb, Kr, r,
                         G + b0 * (long long)r * r);
    else if (lds256)
      SPECENH_LAUNCH(gram256_kernel, dim3((unsigned)nb), dim3(256), 0, st, xb, Kr, r,
                     G + b0 * (long long)r * r);
    else
      SPECENH_LAUNCH(gram_kernel, dim3((ntri + 3) / 4, (unsigned)nb), dim3(256), 0, st, xb,
                         Kr, r, G + b0 * (long long)r * r, nts);
  }
}

template <int P>
hipError_t launch_subspace_t(const float* G, int r, int K, float* V, float* theta,
                             long long batch, hipStream_t st, int cut2, int* flags, int seed,
                             const int* only) {
  const size_t lds = SsLayout<P>::bytes(r);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  hipError_t e = hipFuncSetAttribute((const void*)subspace_kernel<P>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  // 3 rounds when the subspace oversamples the wanted K by >= 8 columns, else 5
  // (a second pass over flagged matrices starts elsewhere and iterates 4x longer)
  const int iters = (P >= K + 8 ? 3 : 5) * (seed ? 4 : 1);
  const int quad = P <= 24 && r % 4 == 0 && (reinterpret_cast<uintptr_t>(G) & 15) == 0 &&
                   variant(V_SVD_GZ_ROWS) == 0;
  SPECENH_LAUNCH(subspace_kernel<P>, dim3((unsigned)batch), dim3(SS_THREADS), lds, st, G, r,
                     K, iters, V, theta, cut2, 5e-6f, flags, seed, only, quad);
  return hipGetLastError();
}

hipError_t launch_subspace(int p, const float* G, int r, int K, float* V, float* theta,
                           long long batch, hipStream_t st, int cut2 = -1, int* flags = nullptr,
                           int seed = 0, const int* only = nullptr) {
  switch (p) {
#define SPECENH_SS(n) \
    case n: return launch_subspace_t<n>(G, r, K, V, theta, batch, st, cut2, flags, seed, only);
    SPECENH_SS(8) SPECENH_SS(16) SPECENH_SS(24) SPECENH_SS(32) SPECENH_SS(40) SPECENH_SS(48)
#undef SPECENH_SS
    default: return hipErrorInvalidValue;
  }
}

template <int KP, typename TO>
hipError_t launch_recon_t(XView xb, int Kr, int r, const float* V, int K, int lo, int hi,
                          int comp, const int* only, void* out, long long ob, long long osk,
                          long long osi, long long nb, hipStream_t st) {
  if (variant(V_SVD_RECON_VALU) == 0) {  // the matrix-core reconstruction
    constexpr int NT = (KP + 15) / 16, KPP = 16 * NT, KS = 2 * NT < 4 ? 2 : 1;
    const int RP = (r + 15) & ~15;
    const size_t lm = ((size_t)RP * (KPP + 1) + (size_t)RB * (RP + 2) +
                       (size_t)KS * RB * (KPP + 1)) * 4;
    // runs of row blocks per workgroup: row-major X with 16-byte rows, or transposed X
    const bool rowmaj16 = xb.si == 1 && r % 4 == 0 && xb.sk % 4 == 0 &&
                          xb.batch_stride % 4 == 0 && (reinterpret_cast<uintptr_t>(xb.base) & 15) == 0;
    const bool trans = xb.sk == 1 && xb.si != 1;
    if (lm <= 160 * 1024 && r <= 256 && (rowmaj16 || trans) &&
        variant(V_SVD_RECON_BLOCKS) == 0) {
      const int nblk = (Kr + RB - 1) / RB;
      // enough workgroups for ~4 per CU, each a run of consecutive blocks of one matrix
      const long long want = 4LL * device_cus();
      const int segs = (int)std::max(1LL, std::min<long long>(nblk, (want + nb - 1) / nb));
      const int bps = (nblk + segs - 1) / segs;
      const int grid_x = (nblk + bps - 1) / bps;
      const void* kfn = trans ? (const void*)recon_stream_kernel<KP, TO, true>
                              : (const void*)recon_stream_kernel<KP, TO, false>;
      hipError_t e = hipFuncSetAttribute(kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lm);
      if (e != hipSuccess) return e;
      if (trans)
        SPECENH_LAUNCH((recon_stream_kernel<KP, TO, true>), dim3(grid_x, (unsigned)nb), dim3(256),
                       lm, st, xb, Kr, r, V, K, lo, hi, comp, only, reinterpret_cast<TO*>(out),
                       ob, osk, osi, bps);
      else
        SPECENH_LAUNCH((recon_stream_kernel<KP, TO, false>), dim3(grid_x, (unsigned)nb), dim3(256),
                       lm, st, xb, Kr, r, V, K, lo, hi, comp, only, reinterpret_cast<TO*>(out),
                       ob, osk, osi, bps);
      return hipGetLastError();
    }
    if (lm <= 160 * 1024) {
      hipError_t e = hipFuncSetAttribute((const void*)recon_mfma_kernel<KP, TO>,
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lm);
      if (e != hipSuccess) return e;
      SPECENH_LAUNCH((recon_mfma_kernel<KP, TO>), dim3((Kr + RB - 1) / RB, (unsigned)nb),
                     dim3(256), lm, st, xb, Kr, r, V, K, lo, hi, comp, only,
                     reinterpret_cast<TO*>(out), ob, osk, osi);
      return hipGetLastError();
    }
  }
  const size_t lds = (size_t)r * KP * 4 + (size_t)RB * (r + 1) * 4 + (size_t)RB * KP * 4;
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  hipError_t e = hipFuncSetAttribute((const void*)recon_kernel<KP, TO>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  SPECENH_LAUNCH((recon_kernel<KP, TO>), dim3((Kr + RB - 1) / RB, (unsigned)nb), dim3(256),
                     lds, st, xb, Kr, r, V, K, lo, hi, comp, only, reinterpret_cast<TO*>(out),
                     ob, osk, osi);
  return hipGetLastError();
}

template <typename TO>
hipError_t launch_recon_k(int KP, XView xb, int Kr, int r, const float* V, int K, int lo,
                          int hi, int comp, const int* only, void* out, long long ob,
                          long long osk, long long osi, long long nb, hipStream_t st) {
  switch (KP) {
#define SPECENH_RC(n)                                                                          \
  case n:                                                                                      \
    return launch_recon_t<n, TO>(xb, Kr, r, V, K, lo, hi, comp, only, out, ob, osk, osi, nb, \
                                 st);
    SPECENH_RC(8) SPECENH_RC(16) SPECENH_RC(24) SPECENH_RC(32) SPECENH_RC(40) SPECENH_RC(48)
#undef SPECENH_RC
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_recon(int KP, XView xb, int Kr, int r, const float* V, int K, int lo, int hi,
                        int comp, const int* only, void* out, long long ob, long long osk,
                        long long osi, long long nb, hipStream_t st, int odt = SPECENH_DTYPE_F32) {
  if (odt == SPECENH_DTYPE_F16)
    return launch_recon_k<_Float16>(KP, xb, Kr, r, V, K, lo, hi, comp, only, out, ob, osk, osi, nb, st);
  if (odt == SPECENH_DTYPE_BF16)
    return launch_recon_k<__bf16>(KP, xb, Kr, r, V, K, lo, hi, comp, only, out, ob, osk, osi, nb, st);
  return launch_recon_k<float>(KP, xb, Kr, r, V, K, lo, hi, comp, only, out, ob, osk, osi, nb, st);
}

size_t dtype_size(int dt) { return dt == SPECENH_DTYPE_F32 ? 4 : 2; }

// ---- eigen path (any kept range, r <= 256): workspace per matrix and chunking
struct EigLayout {
  int r;
  long long ld;  // row stride of Z / the factor arrays: >= r/2 selected vectors
  size_t per_matrix() const {
    return (size_t)r * r * 8 + 3 * (size_t)r * 8 + 4 * (size_t)r * ld * 8 + 4 * 4 + 8;
  }
  // matrices per pass, <= 1 GiB of workspace (the caller allocates it on every call, so it
  // is bounded independently of the batch). Every pass is 4 launches even when the pass
  // only re-does flagged matrices (the fallback after top1 / subspace: the others return at
  // once, ~5 us per mostly-empty pass measured): C3's 4096 x 513 x 256 takes 7 passes
  // (650 matrices of 1.6 MB each), the C5 stream's 2048 x 128 x 128 slices one. Round 4 ran
  // an 8 GB cap (one pass for C3): 60 us faster at C3 for 6.5 GB of workspace per call.
  static constexpr size_t kCapBytes = 1ull << 30;
  long long chunk(long long batch) const {
    const long long c = (long long)(kCapBytes / per_matrix());
    return std::max(1LL, std::min(batch, c));
  }
  size_t bytes(long long batch) const { return (size_t)chunk(batch) * per_matrix() + 256; }
};
EigLayout eig_layout(int r) { return EigLayout{r, (long long)(r / 2 + 2)}; }

// The flagged-matrix fallback in ONE launch (`only` given, no optimal-rank step): a
// workgroup takes a flagged matrix through the Gram tiles, the tridiagonalisation, the
// eigenvectors and the reconstruction blocks in turn (device-scope fences between the
// phases: each reads the previous one's global results). The four launches it replaces
// cost ~4.8 us each even with nothing flagged (grids of 512-1536 workgroups that return at
// once): ~39 us per 4096-shot C5 step.
#ifndef SPECENH_EIG_MERGED
#define SPECENH_EIG_MERGED 1
#endif
template <typename TO>
__global__ __launch_bounds__(256) void eig_fallback_kernel(
    XView x, int Kr, int r, double* G, int nts, double* dg, double* eg, double* taug, int lo,
    int hi, double* Z, double* fac, long long ld, int* kinfo, TO* out, long long out_bstride,
    long long osk, long long osi, const int* only, long long nmat) {
  const int ntri = nts * (nts + 1) / 2, nkb = (Kr + RB - 1) / RB;
  for (long long b = blockIdx.x; b < nmat; b += gridDim.x) {
    if (!only[b]) continue;  // uniform
    for (int t = 0; t < ntri; ++t) {
      gram64_one(x, Kr, r, G, nts, b, t);
      __syncthreads();
    }
    __threadfence();
    __syncthreads();
    tridiag_one(G, r, dg, eg, taug, b);
    __threadfence();
    __syncthreads();
    eigvec_one(G, dg, eg, taug, r, lo, hi, nullptr, Z, fac, ld, kinfo, b);
    __threadfence();
    __syncthreads();
    for (int kb = 0; kb < nkb; ++kb) {
      recon_eig_one<TO>(x, Kr, r, Z, ld, kinfo, out, out_bstride, osk, osi, b, kb);
      __syncthreads();
    }
  }
}

template <typename TO>
hipError_t launch_recon_eig_t(XView xb, int Kr, int r, const double* Z, long long ld,
                              const int* kinfo, void* out, long long ob, long long osk,
                              long long osi, long long nb, hipStream_t st, const int* only) {
  const size_t lds = (size_t)RB * (r + 1) * 4 + (size_t)r * 33 * 4 + (size_t)RB * 33 * 4;
  hipError_t e = hipFuncSetAttribute((const void*)recon_eig_kernel<TO>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  const unsigned gm = only ? (unsigned)std::min<long long>(nb, 2LL * device_cus()) : (unsigned)nb;
  SPECENH_LAUNCH(recon_eig_kernel<TO>, dim3((Kr + RB - 1) / RB, gm), dim3(256), lds, st, xb, Kr,
                 r, Z, ld, kinfo, reinterpret_cast<TO*>(out), ob, osk, osi, only, nb);
  return hipGetLastError();
}

hipError_t launch_recon_eig(int odt, XView xb, int Kr, int r, const double* Z, long long ld,
                            const int* kinfo, void* out, long long ob, long long osk,
                            long long osi, long long nb, hipStream_t st, const int* only) {
  if (odt == SPECENH_DTYPE_F16)
    return launch_recon_eig_t<_Float16>(xb, Kr, r, Z, ld, kinfo, out, ob, osk, osi, nb, st, only);
  if (odt == SPECENH_DTYPE_BF16)
    return launch_recon_eig_t<__bf16>(xb, Kr, r, Z, ld, kinfo, out, ob, osk, osi, nb, st, only);
  return launch_recon_eig_t<float>(xb, Kr, r, Z, ld, kinfo, out, ob, osk, osi, nb, st, only);
}

template <typename TO>
hipError_t launch_eig_fallback_t(XView xb, int Kr, int r, double* G, int nts, double* dg,
                                 double* eg, double* taug, int lo, int hi, double* Z,
                                 double* fac, long long ld, int* kinfo, void* out, long long ob,
                                 long long osk, long long osi, const int* only, long long nb,
                                 unsigned gm, hipStream_t st) {
  const size_t lds = (size_t)RB * (r + 1) * 4 + (size_t)r * 33 * 4 + (size_t)RB * 33 * 4;
  hipError_t e = hipFuncSetAttribute((const void*)eig_fallback_kernel<TO>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  SPECENH_LAUNCH(eig_fallback_kernel<TO>, dim3(gm), dim3(256), lds, st, xb, Kr, r, G, nts, dg,
                 eg, taug, lo, hi, Z, fac, ld, kinfo, reinterpret_cast<TO*>(out), ob, osk, osi,
                 only, nb);
  return hipGetLastError();
}

hipError_t launch_eig_fallback(int odt, XView xb, int Kr, int r, double* G, int nts, double* dg,
                               double* eg, double* taug, int lo, int hi, double* Z, double* fac,
                               long long ld, int* kinfo, void* out, long long ob, long long osk,
                               long long osi, const int* only, long long nb, unsigned gm,
                               hipStream_t st) {
  if (odt == SPECENH_DTYPE_F16)
    return launch_eig_fallback_t<_Float16>(xb, Kr, r, G, nts, dg, eg, taug, lo, hi, Z, fac, ld,
                                           kinfo, out, ob, osk, osi, only, nb, gm, st);
  if (odt == SPECENH_DTYPE_BF16)
    return launch_eig_fallback_t<__bf16>(xb, Kr, r, G, nts, dg, eg, taug, lo, hi, Z, fac, ld,
                                         kinfo, out, ob, osk, osi, only, nb, gm, st);
  return launch_eig_fallback_t<float>(xb, Kr, r, G, nts, dg, eg, taug, lo, hi, Z, fac, ld, kinfo,
                                      out, ob, osk, osi, only, nb, gm, st);
}

// The eigen path over the whole batch, chunk by chunk (stream-ordered, no host sync).
// Uniform kept range (lo, hi), or with opt_mode >= 0 the per-matrix optimal-threshold range
// (num_sing / median / bad flag written to the optional outputs).
int eig_denoise(const float* A, long long batch, int m, int n, long long a_stride, int lo,
                int hi, int opt_mode, void* out, int odt, int* num_out, double* med_out,
                int* bad, void* workspace, hipStream_t st, const int* only = nullptr) {
  const int r = std::min(m, n);
  if (r > EIG_MAXN)
    return set_error(SPECENH_EUNSUPPORTED,
                     "kept range needs the eigen path, which handles min(m, n) <= 256");
  const EigLayout L = eig_layout(r);
  const long long ch = L.chunk(batch);
  char* w = (char*)workspace;
  double* G64 = (double*)w;
  double* dd = G64 + ch * (long long)r * r;
  double* ee = dd + ch * r;
  double* tau = ee + ch * r;
  double* Z = tau + ch * r;
  double* fac = Z + ch * (long long)r * L.ld;
  int* kinfo = (int*)(fac + 3 * ch * (long long)r * L.ld);
  int* ranges = kinfo + 2 * ch;
  int* num = ranges + 2 * ch;
  double* med = (double*)(((uintptr_t)(num + ch) + 7) & ~(uintptr_t)7);
  XView xv;
  xv.batch_stride = a_stride;
  int Kr;
  long long osk, osi;
  if (m >= n) {
    xv.sk = n; xv.si = 1; Kr = m; osk = n; osi = 1;
  } else {
    xv.sk = 1; xv.si = n; Kr = n; osk = 1; osi = n;
  }
  const long long ob = (long long)m * n;
  const size_t osz = dtype_size(odt);
  const int nts64 = (r + 63) / 64, ntri64 = nts64 * (nts64 + 1) / 2;
  const double beta = (double)r / (double)std::max(m, n);
  // omega(beta), denoising_by_svd.ipynb:155-159: sum of coef * beta**(3 - i), Python's order
  const double omega = ((0.0 + 0.56 * std::pow(beta, 3.0)) + -0.95 * std::pow(beta, 2.0)) +
                       1.82 * std::pow(beta, 1.0) + 1.43 * std::pow(beta, 0.0);
  for (long long b0 = 0; b0 < batch; b0 += ch) {
    const long long nb = std::min(ch, batch - b0);
    xv.base = A + b0 * a_stride;
    const int* on = only ? only + b0 : nullptr;
    // fallback (on: the flagged few): a grid of at most two workgroups per CU looping over
    // the matrices instead of one per matrix (gram64_kernel's comment). The merged launch
    // takes 32 workgroups (SPECENH_EIG_GRID): in the two-stream C5 step its 58 KB-LDS
    // workgroups wait for CU slots held by the other stream's autoencoder kernels, and 512 of
    // them that return at once still cost 0.65 % of the step (2.142 -> 2.128 ms at 16, 2.132
    // at 64, profiles/r06_eig_grid_ab.txt); a batch with many flagged matrices loops 32-wide.
    const long long gcap = variant(V_EIG_GRID) > 0 ? variant(V_EIG_GRID) : 2LL * device_cus();
    const unsigned gm = on ? (unsigned)std::min<long long>(nb, gcap) : (unsigned)nb;
    // The merged one-workgroup-per-matrix fallback was A/B'd at C5's size (128 x 128, a few
    // flagged matrices); a large matrix (C3: 513 x 256) puts its whole Gram, tridiagonal
    // solve and reconstruction on one workgroup per CU, which loses to the split launches'
    // tile-parallel grids once many matrices are flagged. Merged only while r * Kr is small.
    const bool merged_fits = (long long)r * Kr <= 128LL * 128;
    if (on && opt_mode < 0 && merged_fits && SPECENH_EIG_MERGED && variant(V_EIG_SPLIT) == 0) {
      const hipError_t e = launch_eig_fallback(odt, xv, Kr, r, G64, nts64, dd, ee, tau, lo, hi,
                                               Z, fac, L.ld, kinfo,
                                               static_cast<char*>(out) + (size_t)(b0 * ob) * osz,
                                               ob, osk, osi, on, nb, gm, st);
      if (e != hipSuccess) return set_error(SPECENH_EHIP, std::string("eigen fallback: ") + hipGetErrorString(e));
      continue;
    }
    SPECENH_LAUNCH(gram64_kernel, dim3(ntri64, gm), dim3(256), 0, st, xv, Kr, r, G64, nts64, on,
                   nb);
    SPECENH_LAUNCH(tridiag_kernel, dim3(gm), dim3(256), 0, st, G64, r, dd, ee, tau, on, nb);
    const int* rg = nullptr;
    if (opt_mode >= 0) {
      SPECENH_LAUNCH(optimal_rank_kernel, dim3((unsigned)nb), dim3(64), 0, st, dd, ee, r,
                         omega, num, med);
      SPECENH_LAUNCH(optimal_ranges_kernel, dim3((unsigned)((nb + 255) / 256)), dim3(256), 0,
                         st, num, nb, r, opt_mode, ranges, bad);
      if (num_out && hipMemcpyAsync(num_out + b0, num, (size_t)nb * 4, hipMemcpyDeviceToDevice,
                                    st) != hipSuccess)
        return set_error(SPECENH_EHIP, "num_sing copy");
      if (med_out && hipMemcpyAsync(med_out + b0, med, (size_t)nb * 8, hipMemcpyDeviceToDevice,
                                    st) != hipSuccess)
        return set_error(SPECENH_EHIP, "median copy");
      rg = ranges;
    }
    SPECENH_LAUNCH(eigvec_kernel, dim3(gm), dim3(256), 0, st, G64, dd, ee, tau, r, lo, hi, rg,
                   Z, fac, L.ld, kinfo, on, nb);
    if (hipGetLastError() != hipSuccess) return set_error(SPECENH_EHIP, "eigen path launch");
    const hipError_t e = launch_recon_eig(odt, xv, Kr, r, Z, L.ld, kinfo,
                                          static_cast<char*>(out) + (size_t)(b0 * ob) * osz, ob,
                                          osk, osi, nb, st, on);
    if (e != hipSuccess) return set_error(SPECENH_EHIP, std::string("recon: ") + hipGetErrorString(e));
  }
  return SPECENH_OK;
}

// top1_kernel's shapes: both dimensions <= 128 and multiples of 4 (16-byte rows / columns),
// 16-byte aligned matrices
bool top1_fits(const float* A, int m, int n, long long a_stride) {
  return m <= top1::N && n <= top1::N && m % 4 == 0 && n % 4 == 0 && a_stride % 4 == 0 &&
         ((uintptr_t)A & 15) == 0;
}

template <typename TO>
hipError_t launch_top1_t(const float* A, long long batch, int m, int n, long long a_stride,
                         int* flags, void* out, hipStream_t st, long long* phase_clk) {
  const hipError_t attr = hipFuncSetAttribute(
      (const void*)top1_kernel<TO>, hipFuncAttributeMaxDynamicSharedMemorySize,
      (int)top1::LDS_BYTES);
  if (attr != hipSuccess) return attr;
  XView xv;
  xv.base = A;
  xv.batch_stride = a_stride;
  int Kr, r = std::min(m, n);
  long long osk, osi;
  if (m >= n) {
    xv.sk = n; xv.si = 1; Kr = m; osk = n; osi = 1;
  } else {
    xv.sk = 1; xv.si = n; Kr = n; osk = 1; osi = n;
  }
  for (long long b0 = 0; b0 < batch; b0 += 1LL << 30) {  // one workgroup per matrix
    const long long nb = std::min<long long>(1LL << 30, batch - b0);
    XView xb = xv;
    xb.base = A + b0 * a_stride;
    SPECENH_LAUNCH(top1_kernel<TO>, dim3((unsigned)nb), dim3(256), top1::LDS_BYTES, st, xb, Kr,
                   r, 5e-6f, flags + b0, reinterpret_cast<TO*>(out) + b0 * (long long)m * n,
                   (long long)m * n, osk, osi, nb, phase_clk ? phase_clk + 8 * b0 : nullptr);
  }
  return hipGetLastError();
}

hipError_t launch_top1(const float* A, long long batch, int m, int n, long long a_stride,
                       int* flags, void* out, int odt, hipStream_t st, long long* phase_clk) {
  if (odt == SPECENH_DTYPE_F16)
    return launch_top1_t<_Float16>(A, batch, m, n, a_stride, flags, out, st, phase_clk);
  if (odt == SPECENH_DTYPE_BF16)
    return launch_top1_t<__bf16>(A, batch, m, n, a_stride, flags, out, st, phase_clk);
  return launch_top1_t<float>(A, batch, m, n, a_stride, flags, out, st, phase_clk);
}

// denoising_by_svd.ipynb:224-228: clamp start < 0 and stop > r, then Python slicing
// u[:, start:stop] (a negative stop counts from the end) -> kept [lo, hi), hi <= lo empty.
void resolve_slice(int r, int start, int stop, int& lo, int& hi) {
  if (start < 0) start = 0;
  if (stop > r) stop = r;
  lo = std::min(start, r);
  hi = stop < 0 ? std::max(stop + r, 0) : stop;
  if (hi < lo) hi = lo;
}

// Which path a uniform kept range takes: 0 = zeros/copy (no workspace), 1 = top-K subspace
// (K returned), 2 = eigen path.
int range_path(int r, int lo, int hi, int& K) {
  K = 0;
  if (hi <= lo || (lo == 0 && hi == r)) return 0;
  K = hi == r ? lo : hi;
  return (K <= PMAX - 8 && std::max(8, ((K + 7 + 7) / 8) * 8) <= std::max(8, (r / 8) * 8) &&
          ((r / 8) * 8 >= K))
             ? 1
             : 2;
}
}  // namespace

extern "C" {

size_t specenh_svd_workspace_bytes(long long batch, int m, int n, int kmax) {
  const long long r = std::min(m, n);
  if (batch <= 0 || r <= 0) return 16;
  if (kmax > PMAX - 8 && r <= EIG_MAXN) return eig_layout((int)r).bytes(batch);
  // subspace path: G, V, theta; for r <= 256 also the per-matrix convergence flags of the
  // two subspace passes and the eigen-path workspace that redoes what stays flagged
  size_t off = (size_t)(batch * r * r + batch * r * kmax + batch * kmax) * sizeof(float);
  if (r > EIG_MAXN) return off;
  off = (off + 255) / 256 * 256 + 2 * (size_t)batch * 4;
  off = (off + 255) / 256 * 256;
  return off + eig_layout((int)r).bytes(batch);
}

size_t specenh_svd_denoise_workspace_bytes(long long batch, int m, int n, int start, int stop) {
  if (batch <= 0 || m <= 0 || n <= 0) return 16;
  const int r = std::min(m, n);
  int lo, hi, K;
  resolve_slice(r, start, stop, lo, hi);
  switch (range_path(r, lo, hi, K)) {
    case 1: return specenh_svd_workspace_bytes(batch, m, n, K);
    case 2:  // (+ top1_kernel's flags for the default range)
      return r <= EIG_MAXN ? eig_layout(r).bytes(batch) + (lo == 1 && hi == r ? batch * 4 + 256 : 0)
                           : 16;
    default: return 16;
  }
}

int specenh_svd_denoise(const float* A, long long batch, int m, int n, long long a_stride,
                        int start, int stop, float* out, void* workspace, void* stream) {
  return specenh_svd_denoise_ex(A, batch, m, n, a_stride, start, stop, out, SPECENH_DTYPE_F32,
                                workspace, stream);
}

int specenh_svd_denoise_ex(const float* A, long long batch, int m, int n, long long a_stride,
                           int start, int stop, void* out, int out_dtype, void* workspace,
                           void* stream) {
  if (out_dtype != SPECENH_DTYPE_F32 && out_dtype != SPECENH_DTYPE_F16 &&
      out_dtype != SPECENH_DTYPE_BF16)
    return set_error(SPECENH_EINVAL, "svd output dtype must be f32, bf16 or f16");
  if (batch < 0 || m <= 0 || n <= 0) return set_error(SPECENH_EINVAL, "bad matrix shape");
  if (batch == 0) return SPECENH_OK;
  if (!A || !out || !workspace) return set_error(SPECENH_EINVAL, "null pointer");
  if (a_stride < (long long)m * n) return set_error(SPECENH_EINVAL, "a_stride < m*n");
  const int r = std::min(m, n);
  int lo, hi, K;
  resolve_slice(r, start, stop, lo, hi);  // denoising_by_svd.ipynb:224-228
  hipStream_t st = (hipStream_t)stream;
  const long long ob = (long long)m * n;
  const size_t osz = dtype_size(out_dtype);
  const int path = range_path(r, lo, hi, K);
  if (path == 0 && hi <= lo) {  // empty slice: zeros (u[:, s:s] @ ... = 0)
    if (hipMemsetAsync(out, 0, (size_t)batch * ob * osz, st) != hipSuccess)
      return set_error(SPECENH_EHIP, "memset");
    return SPECENH_OK;
  }
  if (path == 0) {  // whole range: out = A (u s vh reproduces A)
    if (out_dtype == SPECENH_DTYPE_F32) {
      if (hipMemcpy2DAsync(out, ob * sizeof(float), A, a_stride * sizeof(float),
                           ob * sizeof(float), batch, hipMemcpyDeviceToDevice, st) != hipSuccess)
        return set_error(SPECENH_EHIP, "copy");
      return SPECENH_OK;
    }
    for (long long b = 0; b < batch; ++b) {  // cast (one call when A is dense)
      const long long nb = a_stride == ob ? batch : 1;
      const int rc = specenh_cast(SPECENH_DTYPE_F32, A + b * a_stride, out_dtype,
                                  static_cast<char*>(out) + (size_t)(b * ob) * osz, nb * ob, stream);
      if (rc != SPECENH_OK) return rc;
      b += nb - 1;
    }
    return SPECENH_OK;
  }
  if (lo == 1 && hi == r && top1_fits(A, m, n, a_stride) && variant(V_SVD_NO_TOP1) == 0) {
    // one pass: top1_kernel writes every output and flags the matrices without a converged
    // gap at the cut; the fp64 eigen path redoes those (its kernels return at once for the
    // others). Workspace: the flags and eigen-path regions of the subspace layout, or for
    // r too small for a subspace the eigen-path layout followed by the flags.
    size_t off, eoff;
    if (path == 1) {
      off = (size_t)(batch * r * r + batch * (long long)r * K + batch * K) * sizeof(float);
      off = (off + 255) / 256 * 256;
      eoff = (off + 2 * (size_t)batch * 4 + 255) / 256 * 256;
    } else {
      eoff = 0;
      off = eig_layout(r).bytes(batch);
    }
    int* flags = (int*)((char*)workspace + off);
#ifdef SPECENH_TOP1_STATS  // development build: phase clocks into the (unused) Gram region
    long long* phase_clk = path == 1 ? (long long*)workspace : nullptr;
#else
    long long* phase_clk = nullptr;
#endif
    const hipError_t e = launch_top1(A, batch, m, n, a_stride, flags, out, out_dtype, st, phase_clk);
    if (e != hipSuccess) return set_error(SPECENH_EHIP, std::string("top1: ") + hipGetErrorString(e));
    return eig_denoise(A, batch, m, n, a_stride, 1, r, -1, out, out_dtype, nullptr, nullptr,
                       nullptr, (char*)workspace + eoff, st, flags);
  }
  if (path == 2)  // wide or bottom-of-spectrum range: fp64 eigenvectors (r <= 256)
    return eig_denoise(A, batch, m, n, a_stride, lo, hi, -1, out, out_dtype, nullptr, nullptr,
                       nullptr, workspace, st);
  // Top-K subspace: [lo, hi) = V_hi V_hi^T - V_lo V_lo^T (K = hi), or X - X V_lo V_lo^T when
  // hi == r (K = lo). Subspace width: K + 7 oversampling rounded up to a multiple of 8 (8 for
  // the default K = 1), <= r (rounded down to 8).
  const bool complement = (hi == r);
  int p = std::max(8, ((K + 7 + 7) / 8) * 8);
  if (p > r) p = (r / 8) * 8;
  // X orientation: Gram over the smaller dimension
  XView xv;
  xv.base = A;
  xv.batch_stride = a_stride;
  int Kr;  // rows of X
  long long osk, osi;
  if (m >= n) {
    xv.sk = n; xv.si = 1; Kr = m; osk = n; osi = 1;
  } else {
    xv.sk = 1; xv.si = n; Kr = n; osk = 1; osi = n;
  }
  if (complement) {  // columns [0, lo) of the top-lo subspace, subtracted from X
    hi = lo;
    lo = 0;
  }
  float* G = (float*)workspace;
  float* V = G + batch * (long long)r * r;
  float* theta = V + batch * (long long)r * K;
  int* flags = nullptr;   // first subspace pass: cut without a converged gap
  int* flags2 = nullptr;  // still so after the second pass
  void* eig_ws = nullptr;
  if (r <= EIG_MAXN) {
    size_t off = (size_t)(batch * r * r + batch * (long long)r * K + batch * K) * sizeof(float);
    off = (off + 255) / 256 * 256;
    flags = (int*)((char*)workspace + off);
    flags2 = flags + batch;
    off = (off + 2 * (size_t)batch * 4 + 255) / 256 * 256;
    eig_ws = (char*)workspace + off;
  }
  launch_gram(xv, Kr, r, G, batch, st);
  if (hipGetLastError() != hipSuccess) return set_error(SPECENH_EHIP, "gram launch");
  const int KP = (K + 7) / 8 * 8;
  hipError_t e = launch_subspace(p, G, r, K, V, theta, batch, st,
                                 (!complement && lo > 0) ? lo - 1 : -1, flags);
  if (e != hipSuccess) return set_error(SPECENH_EHIP, std::string("subspace: ") + hipGetErrorString(e));
  for (long long b0 = 0; b0 < batch; b0 += 65535) {
    const long long nb = std::min<long long>(65535, batch - b0);
    XView xb = xv;
    xb.base = A + b0 * a_stride;
    e = launch_recon(KP, xb, Kr, r, V + b0 * (long long)r * K, K, lo, hi, complement ? 1 : 0,
                     nullptr, static_cast<char*>(out) + (size_t)(b0 * ob) * osz, ob, osk, osi, nb,
                     st, out_dtype);
    if (e != hipSuccess) return set_error(SPECENH_EHIP, std::string("recon: ") + hipGetErrorString(e));
  }
  if (hipGetLastError() != hipSuccess) return set_error(SPECENH_EHIP, "recon launch");
  if (!flags) return SPECENH_OK;
  // Flagged matrices: a second subspace pass (other start vectors, 4x the rounds) catches
  // an unlucky start; what is still flagged has no spectral gap at the cut and is redone by
  // the fp64 eigen path. Every kernel of both returns at once for unflagged matrices.
  if (hipMemsetAsync(flags2, 0, (size_t)batch * 4, st) != hipSuccess)
    return set_error(SPECENH_EHIP, "memset");
  e = launch_subspace(p, G, r, K, V, theta, batch, st, (!complement && lo > 0) ? lo - 1 : -1,
                      flags2, 1, flags);
  if (e != hipSuccess) return set_error(SPECENH_EHIP, std::string("subspace: ") + hipGetErrorString(e));
  for (long long b0 = 0; b0 < batch; b0 += 65535) {
    const long long nb = std::min<long long>(65535, batch - b0);
    XView xb = xv;
    xb.base = A + b0 * a_stride;
    e = launch_recon(KP, xb, Kr, r, V + b0 * (long long)r * K, K, lo, hi, complement ? 1 : 0,
                     flags + b0, static_cast<char*>(out) + (size_t)(b0 * ob) * osz, ob, osk, osi,
                     nb, st, out_dtype);
    if (e != hipSuccess) return set_error(SPECENH_EHIP, std::string("recon: ") + hipGetErrorString(e));
  }
  if (complement) {  // back to the kept range [start, r)
    lo = hi;
    hi = r;
  }
  return eig_denoise(A, batch, m, n, a_stride, lo, hi, -1, out, out_dtype, nullptr, nullptr,
                     nullptr, eig_ws, st, flags2);
}

size_t specenh_svd_optimal_workspace_bytes(long long batch, int m, int n) {
  if (batch <= 0 || m <= 0 || n <= 0) return 16;
  const int r = std::min(m, n);
  if (r > EIG_MAXN) return 16;
  return eig_layout(r).bytes(batch) + 256;  // + the IndexError flag
}

int specenh_svd_denoise_optimal(const float* A, long long batch, int m, int n,
                                long long a_stride, int mode, float* out, int* num_sing,
                                double* median_sv, void* workspace, void* stream) {
  if (batch < 0 || m <= 0 || n <= 0) return set_error(SPECENH_EINVAL, "bad matrix shape");
  if (mode != SPECENH_SVD_OPTIMAL && mode != SPECENH_SVD_COMPUTE)
    return set_error(SPECENH_EINVAL, "mode must be SPECENH_SVD_OPTIMAL or SPECENH_SVD_COMPUTE");
  if (batch == 0) return SPECENH_OK;
  if (!A || !out || !workspace) return set_error(SPECENH_EINVAL, "null pointer");
  if (a_stride < (long long)m * n) return set_error(SPECENH_EINVAL, "a_stride < m*n");
  const int r = std::min(m, n);
  if (r > EIG_MAXN)
    return set_error(SPECENH_EUNSUPPORTED, "optimal threshold path needs min(m, n) <= 256");
  hipStream_t st = (hipStream_t)stream;
  // the IndexError flag sits past the eigen-path workspace
  int* bad = (int*)((char*)workspace + eig_layout(r).bytes(batch));
  if (mode == SPECENH_SVD_COMPUTE && hipMemsetAsync(bad, 0, sizeof(int), st) != hipSuccess)
    return set_error(SPECENH_EHIP, "memset");
  const int rc = eig_denoise(A, batch, m, n, a_stride, 0, 0, mode, out, SPECENH_DTYPE_F32,
                             num_sing, median_sv, bad, workspace, st);
  if (rc != SPECENH_OK || mode != SPECENH_SVD_COMPUTE) return rc;  // use_optimal: no host sync
  // computeSignal raises IndexError when 2 num_sing > r (:181-185, s[idx] out of bounds):
  // that needs the counts on the host, one stream sync.
  int hbad = 0;
  if (hipMemcpyAsync(&hbad, bad, sizeof(int), hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return set_error(SPECENH_EHIP, "IndexError flag readback");
  if (hbad)
    return set_error(SPECENH_ERANGE, "index out of bounds for axis 0 with size " +
                                         std::to_string(r) + " (2 * num_sing > min(m, n))");
  return SPECENH_OK;
}

}  // extern "C"
