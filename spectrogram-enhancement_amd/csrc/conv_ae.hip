// conv_ae.hip — the convolutional autoencoder's kernels for gfx950 (NHWC, MFMA).
//
// Replaces the Keras/TensorFlow layers of VAE/manual_scan_3layers.py:186-212
// (Conv2D / MaxPooling2D / Conv2DTranspose, padding="same", relu/sigmoid, Adam +
// binary_crossentropy) with:
//   * conv_igemm_kernel   ONE implicit-GEMM convolution: out[m][co] = sum_k A[m][k] B[k][co]
//                         with A gathered from the NHWC input (k = (ky, kx, ci)):
//                           vy = oy*stride - pad_t + ky, iy = vy / in_dil (valid if exact)
//                         Conv2D fwd (stride 1), Conv2D dgrad (flipped/transposed B),
//                         Conv2DTranspose fwd (in_dil = 2 over a flipped B) and
//                         Conv2DTranspose dgrad (stride 2) are all this kernel.
//                         Epilogue: + bias, optional pre-activation store, optional ReLU
//                         mask of another tensor (the backward ReLU), relu / sigmoid.
//                         MFMA 16x16x32 bf16 (fp32 accumulate) or 16x16x4 f32.
//   * conv_wgrad_kernel   dB[k][co] += sum_m A[m][k] dOut[m][co] (same gather), split over
//                         pixel chunks, fp32 atomics into the gradient.
//   * maxpool2 fwd/bwd    2x2/2 with argmax; backward fuses the ReLU mask of its input.
//   * bce_logits_kernel   Keras graph-mode BCE after a sigmoid = sigmoid_cross_entropy
//                         _with_logits, mean over elements; grad = (sigmoid(z) - t) / n.
//   * adam_kernel         Keras Adam (w -= lr_t m / (sqrt(v) + eps)), refreshes the bf16
//                         GEMM copy of the weights.
//   * flip_transpose      Bd[(a,b,co)][ci] = Bf[(k-1-a, k-1-b, ci)][co] (dgrad weights).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <string>

#include "specenh.h"

namespace specenh {
int set_error(int code, const std::string& msg);  // stft_psd.hip

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

struct ConvGeom {
  int N, IH, IW, C;  // input NHWC
  int OH, OW, CO;    // output NHWC
  int KH, KW;
  int stride, pad_t, pad_l, in_dil;
};

__device__ __forceinline__ float to_f(float x) { return x; }
__device__ __forceinline__ float to_f(__bf16 x) { return (float)x; }
template <typename T>
__device__ __forceinline__ T from_f(float x);
template <>
__device__ __forceinline__ float from_f<float>(float x) { return x; }
template <>
__device__ __forceinline__ __bf16 from_f<__bf16>(float x) { return (__bf16)x; }

// Input coordinate of a (output pixel, tap) pair; -1 if the tap reads padding or a hole
// of the dilated input.
__device__ __forceinline__ int in_coord(int base, int kk, int dil, int extent) {
  const int v = base + kk;
  if (v < 0) return -1;
  int i = v;
  if (dil > 1) {
    if (v % dil) return -1;
    i = v / dil;
  }
  return i < extent ? i : -1;
}

// Load 8 consecutive GEMM-K elements of row (n, base_y, base_x) starting at k.
template <typename T>
__device__ __forceinline__ void gather8(const T* __restrict__ in, const ConvGeom& g, int K,
                                        int n, int by, int bx, int k, bool vm, T (&v)[8]) {
  if ((g.C & 7) == 0) {  // one tap, 8 contiguous channels
    bool ok = vm && k < K;
    int iy = -1, ix = -1, ci = 0;
    if (ok) {
      const int tap = k / g.C;
      ci = k - tap * g.C;
      const int ky = tap / g.KW, kx = tap - ky * g.KW;
      iy = in_coord(by, ky, g.in_dil, g.IH);
      ix = in_coord(bx, kx, g.in_dil, g.IW);
      ok = iy >= 0 && ix >= 0;
    }
    if (ok) {
      const T* p = in + (((long long)n * g.IH + iy) * g.IW + ix) * g.C + ci;
      if constexpr (sizeof(T) == 2) {
        const uint4 q = *reinterpret_cast<const uint4*>(p);
        const T* e = reinterpret_cast<const T*>(&q);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = e[j];
      } else {
        const float4 q0 = reinterpret_cast<const float4*>(p)[0];
        const float4 q1 = reinterpret_cast<const float4*>(p)[1];
        v[0] = q0.x; v[1] = q0.y; v[2] = q0.z; v[3] = q0.w;
        v[4] = q1.x; v[5] = q1.y; v[6] = q1.z; v[7] = q1.w;
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = from_f<T>(0.f);
    }
  } else {  // generic (e.g. the 1-channel first layer)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int kk = k + j;
      T x = from_f<T>(0.f);
      if (vm && kk < K) {
        const int tap = kk / g.C, ci = kk - (kk / g.C) * g.C;
        const int ky = tap / g.KW, kx = tap - ky * g.KW;
        const int iy = in_coord(by, ky, g.in_dil, g.IH), ix = in_coord(bx, kx, g.in_dil, g.IW);
        if (iy >= 0 && ix >= 0) x = in[(((long long)n * g.IH + iy) * g.IW + ix) * g.C + ci];
      }
      v[j] = x;
    }
  }
}

// Load 8 consecutive output channels [co, co+8) of GEMM row r of a [rows][CO] matrix.
template <typename T>
__device__ __forceinline__ void load_row8(const T* __restrict__ p, int rows, int CO, int r, int co,
                                          T (&v)[8]) {
  if (r < rows && (CO & 7) == 0 && co + 8 <= CO) {
    const T* q = p + (long long)r * CO + co;
    if constexpr (sizeof(T) == 2) {
      const uint4 u = *reinterpret_cast<const uint4*>(q);
      const T* e = reinterpret_cast<const T*>(&u);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = e[j];
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = q[j];
    }
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      v[j] = (r < rows && co + j < CO) ? p[(long long)r * CO + co + j] : from_f<T>(0.f);
  }
}

constexpr int BM = 64, BK = 32, KPAD = 8, LDK = BK + KPAD;

// MFMA over one BK=32 slice: a/b rows (16 x 32 each) from LDS with row stride LDK.
template <typename T>
__device__ __forceinline__ f32x4 mfma_slice(const T* sa, const T* sb, f32x4 acc, int lane) {
  if constexpr (sizeof(T) == 2) {
    const bf16x8 a = *reinterpret_cast<const bf16x8*>(sa + (lane & 15) * LDK + 8 * (lane >> 4));
    const bf16x8 b = *reinterpret_cast<const bf16x8*>(sb + (lane & 15) * LDK + 8 * (lane >> 4));
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
  } else {
#pragma unroll
    for (int s = 0; s < BK / 4; ++s) {
      const float a = sa[(lane & 15) * LDK + 4 * s + (lane >> 4)];
      const float b = sb[(lane & 15) * LDK + 4 * s + (lane >> 4)];
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
    }
    return acc;
  }
}

struct ConvFwdArgs {
  ConvGeom g;
  const void* in;
  const void* w;        // GEMM B [K][CO]
  const float* bias;    // [CO] or null
  void* out;            // [M][CO], float if out_f32 else T
  int out_f32;
  const void* mask;     // [M][CO] T or null: v *= (mask > 0)
  int act;              // 0 none, 1 relu, 2 sigmoid
  float* logits;        // [M][CO] fp32 pre-activation store or null
};

// Workgroup: 64 output pixels x (16*NT) output channels; wave w owns rows 16w..16w+15.
template <typename T, int NT>
__global__ __launch_bounds__(256) void conv_igemm_kernel(ConvFwdArgs a) {
  constexpr int BN = 16 * NT;
  __shared__ __attribute__((aligned(16))) T sA[BM * LDK];
  __shared__ __attribute__((aligned(16))) T sB[BN * LDK];
  const ConvGeom& g = a.g;
  const T* __restrict__ in = reinterpret_cast<const T*>(a.in);
  const T* __restrict__ W = reinterpret_cast<const T*>(a.w);
  const int K = g.KH * g.KW * g.C;
  const long long M = (long long)g.N * g.OH * g.OW;
  const long long m0 = (long long)blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

  // this thread's gather row (tid>>2) and k-group (tid&3)
  const int ml = tid >> 2, kg = tid & 3;
  const long long m = m0 + ml;
  const bool vm = m < M;
  int n = 0, by = 0, bx = 0;
  if (vm) {
    const int hw = g.OH * g.OW;
    n = (int)(m / hw);
    const int rem = (int)(m - (long long)n * hw);
    const int oy = rem / g.OW, ox = rem - (rem / g.OW) * g.OW;
    by = oy * g.stride - g.pad_t;
    bx = ox * g.stride - g.pad_l;
  }
  f32x4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int k0 = 0; k0 < K; k0 += BK) {
    T va[8];
    gather8<T>(in, g, K, n, by, bx, k0 + 8 * kg, vm, va);
#pragma unroll
    for (int j = 0; j < 8; ++j) sA[ml * LDK + 8 * kg + j] = va[j];
    // B tile [BK][BN] -> sB[co][k]
    constexpr int GROUPS = BN / 8;
    if (tid < BK * GROUPS) {
      const int kk = tid / GROUPS, cg = tid - kk * GROUPS;
      T vb[8];
      load_row8<T>(W, K, g.CO, k0 + kk, n0 + 8 * cg, vb);
#pragma unroll
      for (int j = 0; j < 8; ++j) sB[(8 * cg + j) * LDK + kk] = vb[j];
    }
    __syncthreads();
#pragma unroll
    for (int t = 0; t < NT; ++t)
      acc[t] = mfma_slice<T>(sA + 16 * wave * LDK, sB + 16 * t * LDK, acc[t], lane);
    __syncthreads();
  }

  // epilogue: D[row][col], col = lane&15, row = 4*(lane>>4) + reg
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int col = n0 + 16 * t + (lane & 15);
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
      const long long mm = m0 + 16 * wave + 4 * (lane >> 4) + reg;
      if (mm >= M || col >= g.CO) continue;
      const long long idx = mm * g.CO + col;
      float v = acc[t][reg] + (a.bias ? a.bias[col] : 0.f);
      if (a.logits) a.logits[idx] = v;
      if (a.mask && !(to_f(reinterpret_cast<const T*>(a.mask)[idx]) > 0.f)) v = 0.f;
      if (a.act == 1) v = fmaxf(v, 0.f);
      else if (a.act == 2) v = 1.f / (1.f + __expf(-v));
      if (a.out_f32) reinterpret_cast<float*>(a.out)[idx] = v;
      else reinterpret_cast<T*>(a.out)[idx] = from_f<T>(v);
    }
  }
}

// part[z][k][co] = sum over pixel chunk z of A[m][k] * dOut[m][co] (deterministic split-K:
// the chunks are summed in order by wgrad_reduce_kernel).
// Workgroup: 64 GEMM-K rows x (16*NT) channels x `chunk` pixels (multiple of 32).
template <typename T, int NT>
__global__ __launch_bounds__(256) void conv_wgrad_kernel(ConvGeom g, const T* __restrict__ in,
                                                          const T* __restrict__ dout,
                                                          float* __restrict__ part, int chunk) {
  constexpr int BN = 16 * NT;
  constexpr int BMK = 64, BP = 32, LDP = BP + KPAD;
  __shared__ __attribute__((aligned(16))) T sA[BMK * LDP];  // [k][m]
  __shared__ __attribute__((aligned(16))) T sG[BN * LDP];   // [co][m]
  const int K = g.KH * g.KW * g.C;
  const long long M = (long long)g.N * g.OH * g.OW;
  const int k0 = blockIdx.x * BMK;
  const int n0 = blockIdx.y * BN;
  const long long p0 = (long long)blockIdx.z * chunk;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int hw = g.OH * g.OW;
  f32x4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int pc = 0; pc < chunk; pc += BP) {
    // gather: thread -> pixel (tid & 31), k-group (tid >> 5): 8 k of one pixel
    {
      const int ml = tid & 31, kgp = tid >> 5;
      const long long m = p0 + pc + ml;
      const bool vm = m < M;
      int n = 0, by = 0, bx = 0;
      if (vm) {
        n = (int)(m / hw);
        const int rem = (int)(m - (long long)n * hw);
        const int oy = rem / g.OW, ox = rem - (rem / g.OW) * g.OW;
        by = oy * g.stride - g.pad_t;
        bx = ox * g.stride - g.pad_l;
      }
      T va[8];
      gather8<T>(in, g, K, n, by, bx, k0 + 8 * kgp, vm, va);
#pragma unroll
      for (int j = 0; j < 8; ++j) sA[(8 * kgp + j) * LDP + ml] = va[j];
    }
    {  // dOut tile [32 pixels][BN] -> sG[co][m]
      constexpr int GROUPS = BN / 8;
      if (tid < BP * GROUPS) {
        const int ml = tid / GROUPS, cg = tid - ml * GROUPS;
        const long long m = p0 + pc + ml;
        T vg[8];
        if (m < M) {
          load_row8<T>(dout + m * g.CO, 1, g.CO, 0, n0 + 8 * cg, vg);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) vg[j] = from_f<T>(0.f);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) sG[(8 * cg + j) * LDP + ml] = vg[j];
      }
    }
    __syncthreads();
#pragma unroll
    for (int t = 0; t < NT; ++t)
      acc[t] = mfma_slice<T>(sA + 16 * wave * LDP, sG + 16 * t * LDP, acc[t], lane);
    __syncthreads();
  }
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int col = n0 + 16 * t + (lane & 15);
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
      const int kk = k0 + 16 * wave + 4 * (lane >> 4) + reg;
      if (kk < K && col < g.CO)
        part[((long long)blockIdx.z * K + kk) * g.CO + col] = acc[t][reg];
    }
  }
}

// part[block][co] = sum over the block's rows of dOut[m][co]
template <typename T>
__global__ __launch_bounds__(256) void bias_grad_kernel(const T* __restrict__ dout, long long M,
                                                         int CO, float* __restrict__ bpart,
                                                         int rows_per_block) {
  __shared__ float s[256];
  const long long r0 = (long long)blockIdx.x * rows_per_block;
  const int co = threadIdx.x % CO;
  const int lanes_per_co = 256 / CO;
  const int part = threadIdx.x / CO;
  float acc = 0.f;
  if (part < lanes_per_co)
    for (long long r = r0 + part; r < std::min<long long>(M, r0 + rows_per_block); r += lanes_per_co)
      acc += to_f(dout[r * CO + co]);
  s[threadIdx.x] = (part < lanes_per_co) ? acc : 0.f;
  __syncthreads();
  if (threadIdx.x < CO) {
    float t = 0.f;
    for (int p = 0; p < lanes_per_co; ++p) t += s[p * CO + threadIdx.x];
    bpart[(long long)blockIdx.x * CO + threadIdx.x] = t;
  }
}

// dst[e] += sum_{z < nz} part[z * n + e], in order (bit-reproducible).
__global__ void ordered_sum_kernel(const float* __restrict__ part, int nz, long long n,
                                   float* __restrict__ dst) {
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n;
       e += (long long)gridDim.x * blockDim.x) {
    float t = 0.f;
    for (int z = 0; z < nz; ++z) t += part[(long long)z * n + e];
    dst[e] += t;
  }
}

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
    am[i] = (unsigned char)arg;
  }
}

// dIn = scatter(dOut to argmax) * (relu_in > 0), dIn fully written.
template <typename T>
__global__ void maxpool2_bwd_kernel(const T* __restrict__ dout, const unsigned char* __restrict__ am,
                                    const T* __restrict__ relu_in, int N, int H, int W, int C,
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
    const float gv = to_f(dout[i]);
    const int arg = am[i];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const long long o = (((long long)n * H + 2 * y + (q >> 1)) * W + 2 * x + (q & 1)) * C + c;
      const bool on = q == arg && (!relu_in || to_f(relu_in[o]) > 0.f);
      din[o] = from_f<T>(on ? gv : 0.f);
    }
  }
}

// Keras BCE after a sigmoid (graph mode): sigmoid_cross_entropy_with_logits, mean.
template <typename TT, typename TG>
__global__ void bce_logits_kernel(const float* __restrict__ z, const TT* __restrict__ t,
                                  long long n, TG* __restrict__ grad, double* __restrict__ loss) {
  double acc = 0.0;
  const float inv = 1.0f / (float)n;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const float zi = z[i], ti = to_f(t[i]);
    acc += (double)(fmaxf(zi, 0.f) - zi * ti + log1pf(__expf(-fabsf(zi))));
    if (grad) grad[i] = from_f<TG>((1.f / (1.f + __expf(-zi)) - ti) * inv);
  }
  for (int m = 32; m >= 1; m >>= 1) acc += __shfl_xor(acc, m);
  if ((threadIdx.x & 63) == 0 && loss) atomicAdd(loss, acc);
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

// Bd[((a*k + b)*CO + co)*CI + ci] = Bf[(((k-1-a)*k + (k-1-b))*CI + ci)*CO + co]
template <typename T>
__global__ void flip_transpose_kernel(const T* __restrict__ bf, int k, int CI, int CO,
                                      T* __restrict__ bd) {
  const long long total = (long long)k * k * CI * CO;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int ci = (int)(i % CI);
    long long r = i / CI;
    const int co = (int)(r % CO);
    r /= CO;
    const int b = (int)(r % k), aa = (int)(r / k);
    bd[i] = bf[(((long long)(k - 1 - aa) * k + (k - 1 - b)) * CI + ci) * CO + co];
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

template <typename T>
int launch_conv(const ConvFwdArgs& a, hipStream_t st) {
  const long long M = (long long)a.g.N * a.g.OH * a.g.OW;
  const unsigned gx = (unsigned)((M + BM - 1) / BM);
  const int nt = std::min(4, (a.g.CO + 15) / 16);
  const unsigned gy = (unsigned)((a.g.CO + 16 * nt - 1) / (16 * nt));
  switch (nt) {
    case 1: hipLaunchKernelGGL((conv_igemm_kernel<T, 1>), dim3(gx, gy), dim3(256), 0, st, a); break;
    case 2: hipLaunchKernelGGL((conv_igemm_kernel<T, 2>), dim3(gx, gy), dim3(256), 0, st, a); break;
    case 3: hipLaunchKernelGGL((conv_igemm_kernel<T, 3>), dim3(gx, gy), dim3(256), 0, st, a); break;
    default: hipLaunchKernelGGL((conv_igemm_kernel<T, 4>), dim3(gx, gy), dim3(256), 0, st, a); break;
  }
  return hipGetLastError() == hipSuccess ? SPECENH_OK : set_error(SPECENH_EHIP, "conv launch");
}

struct WgradPlan {
  int nt;
  unsigned gx, gy, gz;
  long long chunk;
  unsigned nbias;  // bias-grad blocks
  size_t part_elems, bias_elems;
};
constexpr int BIAS_ROWS = 4096;

WgradPlan wgrad_plan(long long M, int K, int CO) {
  WgradPlan p{};
  p.nt = std::min(4, (CO + 15) / 16);
  p.gx = (unsigned)((K + 63) / 64);
  p.gy = (unsigned)((CO + 16 * p.nt - 1) / (16 * p.nt));
  // pixel chunks: ~4 workgroups per CU overall, chunk a multiple of 32 pixels
  const long long want = std::max<long long>(1, 1024 / (long long)(p.gx * p.gy));
  long long chunk = (M + want - 1) / want;
  p.chunk = std::max<long long>(256, ((chunk + 31) / 32) * 32);
  p.gz = (unsigned)((M + p.chunk - 1) / p.chunk);
  p.nbias = (unsigned)((M + BIAS_ROWS - 1) / BIAS_ROWS);
  p.part_elems = (size_t)p.gz * K * CO;
  p.bias_elems = (size_t)p.nbias * CO;
  return p;
}

template <typename T>
int launch_wgrad(const ConvGeom& g, const T* in, const T* dout, float* dw, float* db,
                 float* ws, hipStream_t st) {
  const long long M = (long long)g.N * g.OH * g.OW;
  const int K = g.KH * g.KW * g.C;
  const WgradPlan p = wgrad_plan(M, K, g.CO);
  const dim3 grid(p.gx, p.gy, p.gz);
  const int ch = (int)p.chunk;
  switch (p.nt) {
    case 1: hipLaunchKernelGGL((conv_wgrad_kernel<T, 1>), grid, dim3(256), 0, st, g, in, dout, ws, ch); break;
    case 2: hipLaunchKernelGGL((conv_wgrad_kernel<T, 2>), grid, dim3(256), 0, st, g, in, dout, ws, ch); break;
    case 3: hipLaunchKernelGGL((conv_wgrad_kernel<T, 3>), grid, dim3(256), 0, st, g, in, dout, ws, ch); break;
    default: hipLaunchKernelGGL((conv_wgrad_kernel<T, 4>), grid, dim3(256), 0, st, g, in, dout, ws, ch); break;
  }
  const long long n = (long long)K * g.CO;
  hipLaunchKernelGGL(ordered_sum_kernel, dim3(grid1d(n)), dim3(256), 0, st, ws, (int)p.gz, n, dw);
  if (db) {
    float* bpart = ws + p.part_elems;
    hipLaunchKernelGGL(bias_grad_kernel<T>, dim3(p.nbias), dim3(256), 0, st, dout, M, g.CO,
                       bpart, BIAS_ROWS);
    hipLaunchKernelGGL(ordered_sum_kernel, dim3(1), dim3(256), 0, st, bpart, (int)p.nbias,
                       (long long)g.CO, db);
  }
  return hipGetLastError() == hipSuccess ? SPECENH_OK : set_error(SPECENH_EHIP, "wgrad launch");
}

int check_geom(const ConvGeom& g) {
  if (g.N <= 0 || g.IH <= 0 || g.IW <= 0 || g.C <= 0 || g.OH <= 0 || g.OW <= 0 || g.CO <= 0 ||
      g.KH <= 0 || g.KW <= 0 || g.stride <= 0 || g.in_dil <= 0)
    return set_error(SPECENH_EINVAL, "bad convolution geometry");
  return SPECENH_OK;
}

}  // namespace specenh

using namespace specenh;

extern "C" {

int specenh_conv2d(int dtype, const void* in, int N, int IH, int IW, int C, const void* w_gemm,
                   int KH, int KW, int CO, const float* bias, int stride, int pad_t, int pad_l,
                   int in_dil, int OH, int OW, int act, const void* mask, float* logits,
                   void* out, int out_f32, void* stream) {
  ConvFwdArgs a{};
  a.g = ConvGeom{N, IH, IW, C, OH, OW, CO, KH, KW, stride, pad_t, pad_l, in_dil};
  if (int e = check_geom(a.g)) return e;
  if (!in || !w_gemm || !out) return set_error(SPECENH_EINVAL, "null pointer");
  if (act < 0 || act > 2) return set_error(SPECENH_EINVAL, "bad activation");
  a.in = in; a.w = w_gemm; a.bias = bias; a.out = out; a.out_f32 = out_f32;
  a.mask = mask; a.act = act; a.logits = logits;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == 0) return launch_conv<float>(a, st);
  if (dtype == 1) return launch_conv<__bf16>(a, st);
  return set_error(SPECENH_EINVAL, "dtype must be 0 (f32) or 1 (bf16)");
}

size_t specenh_conv2d_wgrad_workspace_bytes(int N, int OH, int OW, int KH, int KW, int C,
                                            int CO) {
  if (N <= 0 || OH <= 0 || OW <= 0 || KH <= 0 || KW <= 0 || C <= 0 || CO <= 0) return 0;
  const WgradPlan p = wgrad_plan((long long)N * OH * OW, KH * KW * C, CO);
  return (p.part_elems + p.bias_elems) * sizeof(float);
}

int specenh_conv2d_wgrad(int dtype, const void* in, int N, int IH, int IW, int C, const void* dout,
                         int KH, int KW, int CO, int stride, int pad_t, int pad_l, int in_dil,
                         int OH, int OW, float* dw, float* dbias, void* workspace, void* stream) {
  ConvGeom g{N, IH, IW, C, OH, OW, CO, KH, KW, stride, pad_t, pad_l, in_dil};
  if (int e = check_geom(g)) return e;
  if (!in || !dout || !dw || !workspace) return set_error(SPECENH_EINVAL, "null pointer");
  if (dbias && CO > 256) return set_error(SPECENH_EUNSUPPORTED, "bias grad supports CO <= 256");
  hipStream_t st = (hipStream_t)stream;
  float* ws = (float*)workspace;
  if (dtype == 0)
    return launch_wgrad<float>(g, (const float*)in, (const float*)dout, dw, dbias, ws, st);
  if (dtype == 1)
    return launch_wgrad<__bf16>(g, (const __bf16*)in, (const __bf16*)dout, dw, dbias, ws, st);
  return set_error(SPECENH_EINVAL, "dtype must be 0 (f32) or 1 (bf16)");
}

int specenh_maxpool2_fwd(int dtype, const void* in, int N, int H, int W, int C, void* out,
                         unsigned char* argmax, void* stream) {
  if (N <= 0 || H <= 0 || W <= 0 || C <= 0 || (H & 1) || (W & 1))
    return set_error(SPECENH_EINVAL, "maxpool2 needs even H, W");
  const long long n = (long long)N * (H / 2) * (W / 2) * C;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == 0)
    hipLaunchKernelGGL(maxpool2_fwd_kernel<float>, dim3(grid1d(n)), dim3(256), 0, st,
                       (const float*)in, N, H, W, C, (float*)out, argmax);
  else if (dtype == 1)
    hipLaunchKernelGGL(maxpool2_fwd_kernel<__bf16>, dim3(grid1d(n)), dim3(256), 0, st,
                       (const __bf16*)in, N, H, W, C, (__bf16*)out, argmax);
  else
    return set_error(SPECENH_EINVAL, "dtype");
  return hipGetLastError() == hipSuccess ? SPECENH_OK : set_error(SPECENH_EHIP, "maxpool fwd");
}

int specenh_maxpool2_bwd(int dtype, const void* dout, const unsigned char* argmax,
                         const void* relu_in, int N, int H, int W, int C, void* din,
                         void* stream) {
  if (N <= 0 || H <= 0 || W <= 0 || C <= 0 || (H & 1) || (W & 1))
    return set_error(SPECENH_EINVAL, "maxpool2 needs even H, W");
  const long long n = (long long)N * (H / 2) * (W / 2) * C;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == 0)
    hipLaunchKernelGGL(maxpool2_bwd_kernel<float>, dim3(grid1d(n)), dim3(256), 0, st,
                       (const float*)dout, argmax, (const float*)relu_in, N, H, W, C, (float*)din);
  else if (dtype == 1)
    hipLaunchKernelGGL(maxpool2_bwd_kernel<__bf16>, dim3(grid1d(n)), dim3(256), 0, st,
                       (const __bf16*)dout, argmax, (const __bf16*)relu_in, N, H, W, C,
                       (__bf16*)din);
  else
    return set_error(SPECENH_EINVAL, "dtype");
  return hipGetLastError() == hipSuccess ? SPECENH_OK : set_error(SPECENH_EHIP, "maxpool bwd");
}

int specenh_bce_logits(const float* z, const void* target, int target_dtype, long long n,
                       void* grad, int grad_dtype, double* loss_sum, void* stream) {
  if (!z || !target || n <= 0) return set_error(SPECENH_EINVAL, "bce args");
  hipStream_t st = (hipStream_t)stream;
  const unsigned gx = std::min<unsigned>(grid1d(n), 2048);
#define SPECENH_BCE(TT, TG)                                                                   \
  hipLaunchKernelGGL((bce_logits_kernel<TT, TG>), dim3(gx), dim3(256), 0, st, z,             \
                     (const TT*)target, n, (TG*)grad, loss_sum)
  if (target_dtype == 0 && grad_dtype == 0) SPECENH_BCE(float, float);
  else if (target_dtype == 0 && grad_dtype == 1) SPECENH_BCE(float, __bf16);
  else if (target_dtype == 1 && grad_dtype == 0) SPECENH_BCE(__bf16, float);
  else if (target_dtype == 1 && grad_dtype == 1) SPECENH_BCE(__bf16, __bf16);
  else return set_error(SPECENH_EINVAL, "dtype");
#undef SPECENH_BCE
  return hipGetLastError() == hipSuccess ? SPECENH_OK : set_error(SPECENH_EHIP, "bce");
}

int specenh_adam_step(float* w, const float* g, float* m, float* v, long long n, float lr_t,
                      float b1, float b2, float eps, float grad_scale, void* w_bf16,
                      void* stream) {
  if (!w || !g || !m || !v || n <= 0) return set_error(SPECENH_EINVAL, "adam args");
  hipLaunchKernelGGL(adam_kernel<__bf16>, dim3(grid1d(n)), dim3(256), 0, (hipStream_t)stream, w,
                     g, m, v, n, lr_t, b1, b2, eps, grad_scale, (__bf16*)w_bf16);
  return hipGetLastError() == hipSuccess ? SPECENH_OK : set_error(SPECENH_EHIP, "adam");
}

int specenh_weight_flip_transpose(int dtype, const void* bf, int k, int ci, int co, void* bd,
                                  void* stream) {
  const long long n = (long long)k * k * ci * co;
  if (!bf || !bd || n <= 0) return set_error(SPECENH_EINVAL, "flip args");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == 0)
    hipLaunchKernelGGL(flip_transpose_kernel<float>, dim3(grid1d(n)), dim3(256), 0, st,
                       (const float*)bf, k, ci, co, (float*)bd);
  else if (dtype == 1)
    hipLaunchKernelGGL(flip_transpose_kernel<__bf16>, dim3(grid1d(n)), dim3(256), 0, st,
                       (const __bf16*)bf, k, ci, co, (__bf16*)bd);
  else
    return set_error(SPECENH_EINVAL, "dtype");
  return hipGetLastError() == hipSuccess ? SPECENH_OK : set_error(SPECENH_EHIP, "flip");
}

int specenh_cast(int src_dtype, const void* src, int dst_dtype, void* dst, long long n,
                 void* stream) {
  if (!src || !dst || n < 0) return set_error(SPECENH_EINVAL, "cast args");
  if (n == 0) return SPECENH_OK;
  hipStream_t st = (hipStream_t)stream;
  if (src_dtype == 0 && dst_dtype == 1)
    hipLaunchKernelGGL((cast_kernel<float, __bf16>), dim3(grid1d(n)), dim3(256), 0, st,
                       (const float*)src, (__bf16*)dst, n);
  else if (src_dtype == 1 && dst_dtype == 0)
    hipLaunchKernelGGL((cast_kernel<__bf16, float>), dim3(grid1d(n)), dim3(256), 0, st,
                       (const __bf16*)src, (float*)dst, n);
  else
    return set_error(SPECENH_EINVAL, "cast supports f32<->bf16");
  return hipGetLastError() == hipSuccess ? SPECENH_OK : set_error(SPECENH_EHIP, "cast");
}

}  // extern "C"
