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

// Y = G Z for symmetric G (global, r x r) and Z (LDS, r x P): Y[i][:] = sum_j G[j][i] Z[j][:].
// One row i per thread; at each j the threads read row j of G coalesced and Z[j][:] is an
// LDS broadcast.
template <int P>
__device__ void gemm_GZ(const float* G, int r, const float* sZ, float* sY) {
  for (int i = threadIdx.x; i < r; i += SS_THREADS) {
    float acc[P];
#pragma unroll
    for (int c = 0; c < P; ++c) acc[c] = 0.f;
#pragma unroll 8
    for (int j = 0; j < r; ++j) {
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
    int j = j0;
    for (; j + 16 <= j1; j += 16) {
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
    for (; j < j1; ++j) {
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

// Orthonormalise the columns of Y (r x P, LDS) into Z with CholeskyQR in fp64:
// S = Y^T Y, S = R^T R, Z = Y R^-1. fp64 keeps the Gram of Y (condition up to ~1e12
// here) factorisable; callers run it twice (CholeskyQR2) for fp32-level orthogonality.
template <int P>
__device__ void cholqr(const float* sY, float* sZ, int r, double* sS, double* sRi) {
  const int tid = threadIdx.x;
  constexpr int NPAIRS = P * (P + 1) / 2;
  if constexpr (P == 8) {
    prod8(sY, sY, r, sS + 2 * P * P, sS);  // scratch [4][64] past sS, sRi (SsLayout)
  } else
  for (int q = tid; q < NPAIRS; q += SS_THREADS) {
    int a = 0, rem = q;
    while (rem >= P - a) {
      rem -= P - a;
      ++a;
    }
    const int bcol = a + rem;
    double s = 0.0;
    for (int i = 0; i < r; ++i) s += (double)sY[i * P + a] * (double)sY[i * P + bcol];
    sS[a * P + bcol] = s;
  }
  __syncthreads();
  if (tid < 64) {  // Cholesky S = R^T R (R upper, in place), one wave
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
  }
  // R^-1 (upper) into sRi, one wave, one column per lane:
  //   Rinv[j][j] = 1/R[j][j];  Rinv[i][j] = -(sum_{k=i+1..j} R[i][k] Rinv[k][j]) / R[i][i]
  // (lane j reads only R and its own column of Rinv).
  if (tid < 64) {
    for (int idx = tid; idx < P * P; idx += 64) sRi[idx] = 0.0;
    wave_lds_sync();
    for (int j = tid; j < P; j += 64) {
      sRi[j * P + j] = 1.0 / sS[j * P + j];
      for (int i = j - 1; i >= 0; --i) {
        double acc = 0.0;
        for (int k = i + 1; k <= j; ++k) acc += sS[i * P + k] * sRi[k * P + j];
        sRi[i * P + j] = -acc / sS[i * P + i];
      }
    }
  }
  __syncthreads();
  for (int i = tid; i < r; i += SS_THREADS) {  // z = y R^-1 (row times upper triangle)
    double z[P];
#pragma unroll
    for (int c = 0; c < P; ++c) z[c] = 0.0;
#pragma unroll 1
    for (int d = 0; d < P; ++d) {
      const double yd = sY[i * P + d];
      const double* rd = sRi + d * P;
#pragma unroll
      for (int c = 0; c < P; ++c) z[c] = fma(yd, rd[c], z[c]);  // rd[c] = 0 for c < d
    }
#pragma unroll
    for (int c = 0; c < P; ++c) sZ[i * P + c] = (float)z[c];
  }
  __syncthreads();
}

// Parallel (round-robin / Brent-Luk) cyclic Jacobi on the symmetric P x P matrix H in
// LDS, one wave: each round rotates P/2 disjoint (a, b) pairs at once; Q accumulates
// the eigenvectors. Angles in fp64.
template <int P>
__device__ void jacobi(float* sH, float* sQ, float* sCS, int* sPair) {
  const int lane = threadIdx.x;  // wave 0
  for (int idx = lane; idx < P * P; idx += 64) sQ[idx] = (idx / P == idx % P) ? 1.f : 0.f;
  wave_lds_sync();
  for (int sweep = 0; sweep < 15; ++sweep) {
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
        auto player = [&](int k) { return k == 0 ? 0 : 1 + (k - 1 + round) % (P - 1); };
        int a = player(lane), b = player(P - 1 - lane);
        if (a > b) { const int t = a; a = b; b = t; }
        const double hab = sH[a * P + b];
        double c = 1.0, s = 0.0;
        if (fabs(hab) > 1e-37) {
          const double haa = sH[a * P + a], hbb = sH[b * P + b];
          const double tau = (hbb - haa) / (2.0 * hab);
          const double tt = (tau >= 0 ? 1.0 : -1.0) / (fabs(tau) + sqrt(1.0 + tau * tau));
          c = 1.0 / sqrt(1.0 + tt * tt);
          s = tt * c;
        }
        sCS[2 * lane] = (float)c;
        sCS[2 * lane + 1] = (float)s;
        sPair[2 * lane] = a;
        sPair[2 * lane + 1] = b;
      }
      wave_lds_sync();
      for (int idx = lane; idx < (P / 2) * P; idx += 64) {  // rows a, b of every pair
        const int j = idx / P, k = idx % P;
        const int a = sPair[2 * j], b = sPair[2 * j + 1];
        const float c = sCS[2 * j], s = sCS[2 * j + 1];
        const float xa = sH[a * P + k], xb = sH[b * P + k];
        sH[a * P + k] = c * xa - s * xb;
        sH[b * P + k] = s * xa + c * xb;
      }
      wave_lds_sync();
      for (int idx = lane; idx < (P / 2) * P; idx += 64) {  // columns a, b; Q columns
        const int j = idx / P, k = idx % P;
        const int a = sPair[2 * j], b = sPair[2 * j + 1];
        const float c = sCS[2 * j], s = sCS[2 * j + 1];
        const float xa = sH[k * P + a], xb = sH[k * P + b];
        sH[k * P + a] = c * xa - s * xb;
        sH[k * P + b] = s * xa + c * xb;
        const float qa = sQ[k * P + a], qb = sQ[k * P + b];
        sQ[k * P + a] = c * qa - s * qb;
        sQ[k * P + b] = s * qa + c * qb;
      }
      wave_lds_sync();
    }
  }
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
template <int P>
__global__ __launch_bounds__(SS_THREADS) void subspace_kernel(const float* G, int r, int K,
                                                              int iters, float* V,
                                                              float* theta) {
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

  auto GZ = [&](const float* z, float* y) {
    if constexpr (P == 8) gemm_GZ8(Gb, r, z, y, sT);
    else gemm_GZ<P>(Gb, r, z, y);
  };
  for (int idx = tid; idx < r * P; idx += SS_THREADS) sZ[idx] = hash_unit(idx / P, idx % P);
  __syncthreads();
  GZ(sZ, sY);
  __syncthreads();
  for (int it = 0; it < iters; ++it) {
    if (it + 1 < iters && (SPECENH_SS_SINGLE_QR)) {
      // Intermediate rounds only have to keep the block well conditioned (G Z re-amplifies
      // the dominant directions anyway): one CholeskyQR pass. The basis that feeds the
      // Rayleigh-Ritz step below gets the full CholeskyQR2.
      cholqr<P>(sY, sZ, r, sS, sRi);  // Z = orth(Y) to ~cond(Y) * eps
      GZ(sZ, sY);                     // Y = G Z
      __syncthreads();
      continue;
    }
    cholqr<P>(sY, sZ, r, sS, sRi);  // Z = orth(Y)
    cholqr<P>(sZ, sY, r, sS, sRi);  // second pass into Y ...
    GZ(sY, sZ);                     // ... Z = G * orth(Y)
    __syncthreads();
    // swap names: basis in sY, product in sZ -> keep (Y := product, Z := basis)
    float* t = sY;
    sY = sZ;
    sZ = t;
  }
  // Rayleigh-Ritz: H = Z^T (G Z) = Z^T Y
  if constexpr (P == 8) {
    prod8(sZ, sY, r, sPart, sS);
    if (tid < 64) sH[tid] = (float)sS[tid];
  } else {
    for (int q = tid; q < P * P; q += SS_THREADS) {
      const int a = q / P, c = q % P;
      double s = 0.0;
      for (int i = 0; i < r; ++i) s += (double)sZ[i * P + a] * (double)sY[i * P + c];
      sH[q] = (float)s;
    }
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
  if (tid < 64) {
    jacobi<P>(sH, sQ, sCS, sPair);
    if (tid == 0) {  // sort Ritz values descending (insertion sort, P <= 64)
      for (int c = 0; c < P; ++c) sOrd[c] = c;
      for (int c = 1; c < P; ++c) {
        const int key = sOrd[c];
        int d = c - 1;
        while (d >= 0 && sH[sOrd[d] * P + sOrd[d]] < sH[key * P + key]) {
          sOrd[d + 1] = sOrd[d];
          --d;
        }
        sOrd[d + 1] = key;
      }
    }
  }
  __syncthreads();
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
}

// ---------------------------------------------------------------- 3. reconstruction
// Workgroup = (matrix, block of RB X-rows). With X_blk (RB x r), V (r x K):
//   Y = X_blk V_K                       (RB x K)      phase 1
//   out = Y[:, lo:hi] V[:, lo:hi]^T     (RB x r)      phase 2 (complement: X_blk - ...)
constexpr int RB = 32;

// ranges (optional, device int[2 * batch]): a per-matrix [lo, hi) replacing the uniform
// one (always the direct, non-complement form); hi <= lo gives zeros.
template <typename TO>
__device__ __forceinline__ TO to_out(float v) { return (TO)v; }

// TO: output element type (float, or _Float16 / __bf16 when the consumer computes in half
// precision: the cast rides on the reconstruction's store, no separate pass)
template <int KP, typename TO>
__global__ __launch_bounds__(256) void recon_kernel(XView x, int Kr, int r, const float* V,
                                                    int K, int lo, int hi, int complement,
                                                    const int* ranges, TO* out,
                                                    long long out_bstride, long long osk,
                                                    long long osi) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* sV = reinterpret_cast<float*>(smem);  // r x KP (zero-padded columns)
  float* sX = sV + r * KP;                      // RB x (r + 1)
  float* sY = sX + RB * (r + 1);                // RB x KP
  const long long b = blockIdx.y;
  if (ranges) {
    lo = ranges[2 * b];
    hi = ranges[2 * b + 1];
    complement = 0;
  }
  const int k0 = blockIdx.x * RB;
  const int tid = threadIdx.x;
  const float* X = x.base + b * x.batch_stride;
  const float* Vb = V + b * (long long)r * K;
  for (int idx = tid; idx < r * KP; idx += 256) {
    const int i = idx / KP, c = idx % KP;
    sV[idx] = (c >= lo && c < hi) ? Vb[(long long)i * K + c] : 0.f;  // only used columns
  }
  const int rows = min(RB, Kr - k0);
  if (x.si == 1) {
    for (int idx = tid; idx < RB * r; idx += 256) {
      const int kk = idx / r, i = idx % r;
      sX[kk * (r + 1) + i] = kk < rows ? X[(long long)(k0 + kk) * x.sk + i] : 0.f;
    }
  } else {  // transposed view: read along the contiguous k direction
    for (int idx = tid; idx < RB * r; idx += 256) {
      const int i = idx / RB, kk = idx % RB;
      sX[kk * (r + 1) + i] = kk < rows ? X[(long long)(k0 + kk) * x.sk + (long long)i * x.si] : 0.f;
    }
  }
  __syncthreads();
  // phase 1: RB x KP entries of Y, 256 threads
  for (int e = tid; e < RB * KP; e += 256) {
    const int kk = e / KP, c = e % KP;
    float s = 0.f;
    if (c >= lo && c < hi)
      for (int i = 0; i < r; ++i) s = fmaf(sX[kk * (r + 1) + i], sV[i * KP + c], s);
    sY[e] = s;
  }
  __syncthreads();
  // phase 2: out rows, thread per column i (coalesced along i for m >= n)
  TO* Ob = out + b * out_bstride;
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


// ---------------------------------------------------------------- optimal hard threshold
// use_optimal / computeSignal (denoising_by_svd.ipynb:174-181, 210-217) need the median of
// ALL singular values and how many exceed omega(beta) * median. They come from the
// eigenvalues of the Gram matrix in fp64 (the noise singular values sit ~1e-3 below the
// largest; an fp32 Gram would bury their squares in its rounding): Householder reduction
// to tridiagonal form, then Sturm-count bisection for exactly the three numbers needed
// (the two middle order statistics and the count above the threshold).

// fp64 Gram G = X^T X: 64x64 tile per workgroup (upper-triangle tiles, mirrored), 16 rows
// of X per LDS stage, 4x4 outputs per thread. Products of fp32 inputs are exact in fp64.
__global__ __launch_bounds__(256) void gram64_kernel(XView x, int K, int r, double* G, int nts) {
  __shared__ double sa[16][65], sb[16][65];
  int t = blockIdx.x, ti = 0;
  while (t >= nts - ti) {
    t -= nts - ti;
    ++ti;
  }
  const int tj = ti + t;
  const long long b = blockIdx.y;
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
__global__ __launch_bounds__(256) void tridiag_kernel(double* G, int n, double* dg, double* eg) {
  __shared__ double sv[256], sw[256], red[4];
  const long long b = blockIdx.x;
  double* A = G + b * (long long)n * n;
  double* d = dg + b * n;
  double* e = eg + b * n;
  const int tid = threadIdx.x;
  for (int k = 0; k + 2 < n; ++k) {
    const int len = n - k - 1;
    const double* rowk = A + (long long)k * n + k + 1;  // = column k below the diagonal
    const double xv = tid < len ? rowk[tid] : 0.0;
    const double s2 = block_sum256(tid >= 1 && tid < len ? xv * xv : 0.0, red);
    const double alpha = rowk[0];
    if (tid == 0) d[k] = A[(long long)k * n + k];
    if (s2 == 0.0) {  // uniform: already tridiagonal in this column
      if (tid == 0) e[k] = alpha;
      continue;
    }
    const double beta = -copysign(sqrt(alpha * alpha + s2), alpha);
    const double tau = (beta - alpha) / beta;
    const double scal = 1.0 / (alpha - beta);
    if (tid == 0) e[k] = beta;
    const double vi = tid == 0 ? 1.0 : (tid < len ? xv * scal : 0.0);
    if (tid < len) sv[tid] = vi;
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

}  // namespace specenh

using namespace specenh;

namespace {
bool getenv_set(const char* name) {
  const char* v = std::getenv(name);
  return v && *v && *v != '0';
}

// G = X^T X for every matrix: the LDS-chunked kernel for r <= 128 (r % 4 == 0), else
// one wave per 32x32 tile.
void launch_gram(const XView& xv, int Kr, int r, float* G, long long batch, hipStream_t st) {
  const bool lds = r <= 128 && r % 4 == 0 && !getenv_set("SPECENH_SVD_GRAM_TILES");
  const int nts = (r + 31) / 32;
  const int ntri = nts * (nts + 1) / 2;
  for (long long b0 = 0; b0 < batch; b0 += 65535) {
    const long long nb = std::min<long long>(65535, batch - b0);
    XView xb = xv;
    xb.base = xv.base + b0 * xv.batch_stride;
    if (lds)
      hipLaunchKernelGGL(gram_lds_kernel, dim3((unsigned)nb), dim3(256), 0, st, xb, Kr, r,
                         G + b0 * (long long)r * r);
    else
      hipLaunchKernelGGL(gram_kernel, dim3((ntri + 3) / 4, (unsigned)nb), dim3(256), 0, st, xb,
                         Kr, r, G + b0 * (long long)r * r, nts);
  }
}

template <int P>
hipError_t launch_subspace_t(const float* G, int r, int K, float* V, float* theta,
                             long long batch, hipStream_t st) {
  const size_t lds = SsLayout<P>::bytes(r);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  hipError_t e = hipFuncSetAttribute((const void*)subspace_kernel<P>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  // 3 rounds when the subspace oversamples the wanted K by >= 8 columns, else 5
  const int iters = P >= K + 8 ? 3 : 5;
  hipLaunchKernelGGL(subspace_kernel<P>, dim3((unsigned)batch), dim3(SS_THREADS), lds, st, G, r,
                     K, iters, V, theta);
  return hipGetLastError();
}

hipError_t launch_subspace(int p, const float* G, int r, int K, float* V, float* theta,
                           long long batch, hipStream_t st) {
  switch (p) {
    case 8: return launch_subspace_t<8>(G, r, K, V, theta, batch, st);
    case 16: return launch_subspace_t<16>(G, r, K, V, theta, batch, st);
    case 24: return launch_subspace_t<24>(G, r, K, V, theta, batch, st);
    case 32: return launch_subspace_t<32>(G, r, K, V, theta, batch, st);
    case 40: return launch_subspace_t<40>(G, r, K, V, theta, batch, st);
    case 48: return launch_subspace_t<48>(G, r, K, V, theta, batch, st);
    default: return hipErrorInvalidValue;
  }
}

template <int KP, typename TO>
hipError_t launch_recon_t(XView xb, int Kr, int r, const float* V, int K, int lo, int hi,
                          int comp, const int* ranges, void* out, long long ob, long long osk,
                          long long osi, long long nb, hipStream_t st) {
  const size_t lds = (size_t)r * KP * 4 + (size_t)RB * (r + 1) * 4 + (size_t)RB * KP * 4;
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  hipError_t e = hipFuncSetAttribute((const void*)recon_kernel<KP, TO>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((recon_kernel<KP, TO>), dim3((Kr + RB - 1) / RB, (unsigned)nb), dim3(256),
                     lds, st, xb, Kr, r, V, K, lo, hi, comp, ranges, reinterpret_cast<TO*>(out),
                     ob, osk, osi);
  return hipGetLastError();
}

template <typename TO>
hipError_t launch_recon_k(int KP, XView xb, int Kr, int r, const float* V, int K, int lo,
                          int hi, int comp, const int* ranges, void* out, long long ob,
                          long long osk, long long osi, long long nb, hipStream_t st) {
  switch (KP) {
#define SPECENH_RC(n)                                                                          \
  case n:                                                                                      \
    return launch_recon_t<n, TO>(xb, Kr, r, V, K, lo, hi, comp, ranges, out, ob, osk, osi, nb, \
                                 st);
    SPECENH_RC(8) SPECENH_RC(16) SPECENH_RC(24) SPECENH_RC(32) SPECENH_RC(40) SPECENH_RC(48)
#undef SPECENH_RC
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_recon(int KP, XView xb, int Kr, int r, const float* V, int K, int lo, int hi,
                        int comp, const int* ranges, void* out, long long ob, long long osk,
                        long long osi, long long nb, hipStream_t st, int odt = SPECENH_DTYPE_F32) {
  if (odt == SPECENH_DTYPE_F16)
    return launch_recon_k<_Float16>(KP, xb, Kr, r, V, K, lo, hi, comp, ranges, out, ob, osk, osi, nb, st);
  if (odt == SPECENH_DTYPE_BF16)
    return launch_recon_k<__bf16>(KP, xb, Kr, r, V, K, lo, hi, comp, ranges, out, ob, osk, osi, nb, st);
  return launch_recon_k<float>(KP, xb, Kr, r, V, K, lo, hi, comp, ranges, out, ob, osk, osi, nb, st);
}

size_t dtype_size(int dt) { return dt == SPECENH_DTYPE_F32 ? 4 : 2; }
}  // namespace

extern "C" {

size_t specenh_svd_workspace_bytes(long long batch, int m, int n, int kmax) {
  const long long r = std::min(m, n);
  return (size_t)(batch * r * r + batch * r * kmax + batch * kmax) * sizeof(float);
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
  // denoising_by_svd.ipynb:224-227 clamping
  if (start < 0) start = 0;
  if (stop > r) stop = r;
  hipStream_t st = (hipStream_t)stream;
  const long long ob = (long long)m * n;
  const size_t osz = dtype_size(out_dtype);
  if (stop <= start) {  // empty range: zeros (u[:, s:s] @ ... = 0)
    if (hipMemsetAsync(out, 0, (size_t)batch * ob * osz, st) != hipSuccess)
      return set_error(SPECENH_EHIP, "memset");
    return SPECENH_OK;
  }
  // Needed top-K subspace: complement form when stop == r.
  const bool complement = (stop == r);
  const int K = complement ? start : stop;
  if (complement && start == 0) {  // whole range: out = A (u s vh reproduces A)
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
  if (K > PMAX - 8 || K > r)
    return set_error(SPECENH_EUNSUPPORTED,
                     "GPU SVD denoiser needs a top-K subspace with K <= 40 (K = stop, or start "
                     "when stop == r)");
  // subspace width: K + 7 oversampling rounded up to a multiple of 8 (8 for the default
  // K = 1), <= r (rounded down to 8)
  int p = std::max(8, ((K + 7 + 7) / 8) * 8);
  if (p > r) p = (r / 8) * 8;
  if (p < K || p < 8)
    return set_error(SPECENH_EUNSUPPORTED, "matrix too small for the GPU subspace solver");
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
  const int lo = complement ? 0 : start, hi = complement ? start : stop;
  float* G = (float*)workspace;
  float* V = G + batch * (long long)r * r;
  float* theta = V + batch * (long long)r * K;
  launch_gram(xv, Kr, r, G, batch, st);
  if (hipGetLastError() != hipSuccess) return set_error(SPECENH_EHIP, "gram launch");
  const int KP = ((hi - lo > 0 ? K : 1) + 7) / 8 * 8;
  hipError_t e = launch_subspace(p, G, r, K, V, theta, batch, st);
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
  return SPECENH_OK;
}


size_t specenh_svd_optimal_workspace_bytes(long long batch, int m, int n) {
  if (batch <= 0 || m <= 0 || n <= 0) return 16;
  const size_t r = (size_t)std::min(m, n);
  size_t off = (size_t)batch * r * r * 8 + 2 * (size_t)batch * r * 8;  // G64, d, e
  off += (size_t)batch * (4 + 4 + 8);                                  // num, ranges, median
  off = (off + 255) / 256 * 256;
  return off + specenh_svd_workspace_bytes(batch, m, n, PMAX - 8);
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
  if (r > 256)
    return set_error(SPECENH_EUNSUPPORTED, "optimal threshold path needs min(m, n) <= 256");
  hipStream_t st = (hipStream_t)stream;
  // workspace carve (specenh_svd_optimal_workspace_bytes)
  char* w = (char*)workspace;
  double* G64 = (double*)w;
  double* dd = G64 + batch * (long long)r * r;
  double* ee = dd + batch * (long long)r;
  int* num = (int*)(ee + batch * (long long)r);
  int* ranges = num + batch;
  double* med = (double*)(ranges + 2 * batch);
  size_t off = (size_t)batch * r * r * 8 + 2 * (size_t)batch * r * 8 + (size_t)batch * 16;
  off = (off + 255) / 256 * 256;
  float* G = (float*)(w + off);
  XView xv;
  xv.base = A;
  xv.batch_stride = a_stride;
  int Kr;
  long long osk, osi;
  if (m >= n) {
    xv.sk = n; xv.si = 1; Kr = m; osk = n; osi = 1;
  } else {
    xv.sk = 1; xv.si = n; Kr = n; osk = 1; osi = n;
  }
  // 1-3: fp64 Gram, tridiagonal form, median and count above the threshold
  const int nts64 = (r + 63) / 64;
  const int ntri64 = nts64 * (nts64 + 1) / 2;
  for (long long b0 = 0; b0 < batch; b0 += 65535) {
    const long long nb = std::min<long long>(65535, batch - b0);
    XView xb = xv;
    xb.base = A + b0 * a_stride;
    hipLaunchKernelGGL(gram64_kernel, dim3(ntri64, (unsigned)nb), dim3(256), 0, st, xb, Kr, r,
                       G64 + b0 * (long long)r * r, nts64);
  }
  hipLaunchKernelGGL(tridiag_kernel, dim3((unsigned)batch), dim3(256), 0, st, G64, r, dd, ee);
  const double beta = (double)r / (double)std::max(m, n);
  // omega(beta), denoising_by_svd.ipynb:155-159: sum of coef * beta**(3 - i), Python's order
  const double omega = ((0.0 + 0.56 * std::pow(beta, 3.0)) + -0.95 * std::pow(beta, 2.0)) +
                       1.82 * std::pow(beta, 1.0) + 1.43 * std::pow(beta, 0.0);
  hipLaunchKernelGGL(optimal_rank_kernel, dim3((unsigned)batch), dim3(64), 0, st, dd, ee, r,
                     omega, num, med);
  if (hipGetLastError() != hipSuccess) return set_error(SPECENH_EHIP, "optimal rank launch");
  // 4: the kept range per matrix decides the subspace width: one host round trip
  std::vector<int> hn((size_t)batch);
  if (hipMemcpyAsync(hn.data(), num, (size_t)batch * sizeof(int), hipMemcpyDeviceToHost, st) !=
          hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return set_error(SPECENH_EHIP, "num_sing readback");
  if (num_sing &&
      hipMemcpyAsync(num_sing, num, (size_t)batch * sizeof(int), hipMemcpyDeviceToDevice, st) !=
          hipSuccess)
    return set_error(SPECENH_EHIP, "num_sing copy");
  if (median_sv &&
      hipMemcpyAsync(median_sv, med, (size_t)batch * sizeof(double), hipMemcpyDeviceToDevice,
                     st) != hipSuccess)
    return set_error(SPECENH_EHIP, "median copy");
  std::vector<int> hr(2 * (size_t)batch);
  int K = 0;
  for (long long b = 0; b < batch; ++b) {
    const int ns = hn[b];
    int lo, hi;
    if (mode == SPECENH_SVD_OPTIMAL) {  // :216-217 start = 0, stop = num_sing - 1
      lo = 0;
      hi = ns - 1;
    } else {  // computeSignal :181-185: s[idx] for idx in range(1, 2 num_sing)
      if (2 * ns - 1 > r - 1 && ns > 0)
        return set_error(SPECENH_ERANGE, "index " + std::to_string(2 * ns - 1) +
                                             " is out of bounds for axis 0 with size " +
                                             std::to_string(r));
      lo = 1;
      hi = 2 * ns;
    }
    if (lo < 0) lo = 0;  // :224-227 clamping
    if (hi > r) hi = r;
    hr[2 * b] = lo;
    hr[2 * b + 1] = hi;
    if (hi > lo) K = std::max(K, hi);
  }
  if (K == 0) {
    if (hipMemsetAsync(out, 0, (size_t)batch * m * n * sizeof(float), st) != hipSuccess)
      return set_error(SPECENH_EHIP, "memset");
    return SPECENH_OK;
  }
  if (K > PMAX - 8 || K > r)
    return set_error(SPECENH_EUNSUPPORTED,
                     "the kept range needs a top-" + std::to_string(K) +
                         " singular subspace; the GPU subspace solver handles K <= 40");
  if (hipMemcpy(ranges, hr.data(), hr.size() * sizeof(int), hipMemcpyHostToDevice) != hipSuccess)
    return set_error(SPECENH_EHIP, "ranges upload");
  int p = std::max(8, ((K + 7 + 7) / 8) * 8);
  if (p > r) p = (r / 8) * 8;
  if (p < K || p < 8)
    return set_error(SPECENH_EUNSUPPORTED, "matrix too small for the GPU subspace solver");
  // 5: fp32 Gram, top-K subspace, per-matrix reconstruction
  float* V = G + batch * (long long)r * r;
  float* theta = V + batch * (long long)r * K;
  launch_gram(xv, Kr, r, G, batch, st);
  hipError_t e = launch_subspace(p, G, r, K, V, theta, batch, st);
  if (e != hipSuccess)
    return set_error(SPECENH_EHIP, std::string("subspace: ") + hipGetErrorString(e));
  const int KP = (K + 7) / 8 * 8;
  const long long ob = (long long)m * n;
  for (long long b0 = 0; b0 < batch; b0 += 65535) {
    const long long nb = std::min<long long>(65535, batch - b0);
    XView xb = xv;
    xb.base = A + b0 * a_stride;
    e = launch_recon(KP, xb, Kr, r, V + b0 * (long long)r * K, K, 0, 0, 0, ranges + 2 * b0,
                     out + b0 * ob, ob, osk, osi, nb, st);
    if (e != hipSuccess)
      return set_error(SPECENH_EHIP, std::string("recon: ") + hipGetErrorString(e));
  }
  return SPECENH_OK;
}

}  // extern "C"
