// conv_narrow.hip — the autoencoder's narrow-channel convolutions on the VALU (gfx950).
//
// The first Conv2D of the reference model (1 -> 16 channels, VAE/manual_scan_3layers.py:187)
// and the last one (16 -> 1, sigmoid, :199) have a GEMM dimension of 1: on the MFMA path
// (conv_ae.hip) they fill 1/16 of a 16x16 tile and their fragments are gathered element by
// element. Here they are direct convolutions with packed dot products (v_dot2_f32_f16 /
// v_dot2c_f32_bf16: two products + fp32 accumulate per lane and instruction), the input
// patch staged once per workgroup in LDS and the weights read as LDS broadcasts:
//
//   conv_c1_kernel<T, K, POOL>   C == 1, any CO (16-channel blocks): each lane computes a
//       2x2 output block x 16 channels; the K taps of a kernel row are paired along x
//       ((kx, kx+1) -> one dot2), the odd column shift is one v_alignbit. POOL fuses the
//       following MaxPooling2D((2,2)) (+ argmax) exactly like the MFMA path does (values
//       compared as stored in T, first max wins), so fused and unfused results are equal.
//   conv_co1_kernel<T, C, K>     CO == 1, C in {16, 32}: each lane computes P consecutive
//       output pixels of a row (P = 64 / C) and reuses every loaded input column for the K
//       taps it meets; channels pair naturally in NHWC (one 32-bit word = 2 channels). The
//       patch is stored in groups of P pixels padded by 16 bytes (group stride 144 B), which
//       makes the lanes' ds_read_b128 conflict-free.
// Accumulation is fp32 in both (products of two 16-bit values are exact in fp32).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <string>

#include "specenh.h"
#include "runtime.hpp"

namespace specenh {
int set_error(int code, const std::string& msg);  // stft_psd.hip

namespace {

typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

struct NarrowArgs {
  const void* in;
  const void* w;  // w_gemm [CO][K][K][C]
  const float* bias;
  void* out;
  float* logits;
  unsigned char* argmax;
  int N, IH, IW, C, OH, OW, CO;
  int pad_t, pad_l;
  int act, out_f32;
  const void* mask;  // conv_c1_kernel, no pool: out = 0 where mask <= 0 (backward of a ReLU)
  int band_steps;  // conv_co1_kernel: TR-row steps per workgroup (blockIdx.y = band)
};

__device__ __forceinline__ float act_f(float v, int act) {
  if (act == SPECENH_ACT_RELU) return fmaxf(v, 0.f);
  if (act == SPECENH_ACT_SIGMOID) return 1.f / (1.f + __expf(-v));
  return v;
}

template <typename T>
__device__ __forceinline__ uint32_t tbits(T x) {
  return (uint32_t)__builtin_bit_cast(unsigned short, x);
}
template <typename T>
__device__ __forceinline__ T from_bits(uint32_t b) {
  return __builtin_bit_cast(T, (unsigned short)b);
}

// c + a.lo*b.lo + a.hi*b.hi for two packed 16-bit values of T
template <typename T>
__device__ __forceinline__ float dot2(uint32_t a, uint32_t b, float c) {
  if constexpr (__is_same(T, _Float16)) {
    return __builtin_amdgcn_fdot2(__builtin_bit_cast(f16x2, a), __builtin_bit_cast(f16x2, b), c,
                                  false);
  } else {  // v_dot2c_f32_bf16 (gfx950)
    typedef __bf16 b2 __attribute__((ext_vector_type(2)));
    return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(b2, a), __builtin_bit_cast(b2, b), c,
                                          false);
  }
}

// ------------------------------------------------------------------ C == 1
constexpr int C1_TILE = 32;  // output rows and columns per workgroup (16 x 16 lanes x 2 x 2)

template <typename T, int K, bool POOL>
__global__ __launch_bounds__(256) void conv_c1_kernel(NarrowArgs a) {
  constexpr int NPX = (K + 1) / 2;                    // tap pairs per kernel row
  constexpr int NQ = K * NPX;                         // tap pairs per output channel
  constexpr int NQ4 = (NQ + 3) / 4 * 4;
  constexpr int WR = K + 1;                           // window rows/columns of a 2x2 block
  constexpr int PST = C1_TILE + K + (K & 1 ? 1 : 0);  // patch row stride (even)
  constexpr int PH = C1_TILE + K - 1;
  __shared__ __attribute__((aligned(16))) T sP[PH * PST];
  __shared__ __attribute__((aligned(16))) uint32_t sW[16][NQ4];
  __shared__ float sB[16];

  const int tid = threadIdx.x;
  const int ntx = (a.OW + C1_TILE - 1) / C1_TILE, nty = (a.OH + C1_TILE - 1) / C1_TILE;
  const int n = blockIdx.x / (ntx * nty);
  const int trem = blockIdx.x - n * (ntx * nty);
  const int oy0 = (trem / ntx) * C1_TILE, ox0 = (trem % ntx) * C1_TILE;
  const int cb = blockIdx.y * 16;
  const int iy0 = oy0 - a.pad_t, ix0 = ox0 - a.pad_l;
  const T* __restrict__ in = reinterpret_cast<const T*>(a.in);
  const T* __restrict__ W = reinterpret_cast<const T*>(a.w);

  {
    // every load of the patch in flight at once (unconditional, from a clamped address)
    constexpr int NE = (PH * PST + 255) / 256;
    T v[NE];
#pragma unroll
    for (int k = 0; k < NE; ++k) {
      const int e = tid + 256 * k;
      const int py = e / PST, px = e - (e / PST) * PST;
      const int iy = iy0 + py, ix = ix0 + px;
      const bool ok = e < PH * PST && px < C1_TILE + K - 1 && (unsigned)iy < (unsigned)a.IH &&
                      (unsigned)ix < (unsigned)a.IW;
      v[k] = in[ok ? ((long long)n * a.IH + iy) * a.IW + ix : 0];
      if (!ok) v[k] = (T)0.f;
    }
#pragma unroll
    for (int k = 0; k < NE; ++k)
      if (tid + 256 * k < PH * PST) sP[tid + 256 * k] = v[k];
  }
  for (int e = tid; e < 16 * NQ4; e += 256) {
    const int cl = e / NQ4, q = e - (e / NQ4) * NQ4;
    const int ky = q / NPX, j = q - (q / NPX) * NPX;
    const int co = cb + cl;
    uint32_t v = 0;
    if (co < a.CO && q < NQ) {
      const T* wr = W + (long long)co * K * K + ky * K;
      v = tbits(wr[2 * j]);
      if (2 * j + 1 < K) v |= tbits(wr[2 * j + 1]) << 16;
    }
    sW[cl][q] = v;
  }
  if (tid < 16) sB[tid] = (a.bias && cb + tid < a.CO) ? a.bias[cb + tid] : 0.f;
  __syncthreads();

  const int tx = tid & 15, ty = tid >> 4;
  // pairs of window row r: pa = columns (2m, 2m+1), pb = columns (2m+1, 2m+2); a pair's
  // second tap past the kernel edge meets a zero weight (inputs are finite)
  uint32_t pa[WR][NPX], pb[WR][NPX];
#pragma unroll
  for (int r = 0; r < WR; ++r) {
    uint32_t raw[NPX + 1];
    const T* row = sP + (2 * ty + r) * PST + 2 * tx;
#pragma unroll
    for (int m = 0; m <= NPX; ++m)
      raw[m] = (2 * m < WR) ? *reinterpret_cast<const uint32_t*>(row + 2 * m) : 0u;
#pragma unroll
    for (int m = 0; m < NPX; ++m) {
      pa[r][m] = raw[m];
      pb[r][m] = __builtin_amdgcn_alignbit(raw[m + 1], raw[m], 16);
    }
  }

  // per output channel: accumulate the 2x2 block, then pool / pack it at once (no
  // 64-float accumulator array stays live)
  const int oy = oy0 + 2 * ty, ox = ox0 + 2 * tx;
  const int nco = min(16, a.CO - cb);
  uint32_t pk[2][2][8], am[4];
#pragma unroll
  for (int i = 0; i < 8; ++i) pk[0][0][i] = pk[0][1][i] = pk[1][0][i] = pk[1][1][i] = 0u;
#pragma unroll
  for (int i = 0; i < 4; ++i) am[i] = 0u;
  long long opix[2][2];
  bool okpix[2][2];
#pragma unroll
  for (int dy = 0; dy < 2; ++dy)
#pragma unroll
    for (int dx = 0; dx < 2; ++dx) {
      okpix[dy][dx] = oy + dy < a.OH && ox + dx < a.OW;
      opix[dy][dx] = (((long long)n * a.OH + oy + dy) * a.OW + ox + dx) * a.CO + cb;
    }
#pragma unroll
  for (int cl = 0; cl < 16; ++cl) {
    uint32_t wq[NQ4];
#pragma unroll
    for (int q4 = 0; q4 < NQ4 / 4; ++q4) {
      const uint4 u = *reinterpret_cast<const uint4*>(&sW[cl][4 * q4]);  // broadcast
      wq[4 * q4] = u.x;
      wq[4 * q4 + 1] = u.y;
      wq[4 * q4 + 2] = u.z;
      wq[4 * q4 + 3] = u.w;
    }
    float s[2][2];
#pragma unroll
    for (int dy = 0; dy < 2; ++dy) {
      float s0 = 0.f, s1 = 0.f;
#pragma unroll
      for (int ky = 0; ky < K; ++ky)
#pragma unroll
        for (int j = 0; j < NPX; ++j) {
          s0 = dot2<T>(pa[dy + ky][j], wq[ky * NPX + j], s0);
          s1 = dot2<T>(pb[dy + ky][j], wq[ky * NPX + j], s1);
        }
      s[dy][0] = s0;
      s[dy][1] = s1;
    }
    const float bb = sB[cl];
    if constexpr (POOL) {
      const float v00 = (float)(T)act_f(s[0][0] + bb, a.act);
      const float v01 = (float)(T)act_f(s[0][1] + bb, a.act);
      const float v10 = (float)(T)act_f(s[1][0] + bb, a.act);
      const float v11 = (float)(T)act_f(s[1][1] + bb, a.act);
      float b = v00;
      uint32_t q = 0;
      if (v01 > b) { b = v01; q = 1; }
      if (v10 > b) { b = v10; q = 2; }
      if (v11 > b) { b = v11; q = 3; }
      pk[0][0][cl >> 1] |= tbits((T)b) << (16 * (cl & 1));
      am[cl >> 2] |= q << (8 * (cl & 3));
    } else {
#pragma unroll
      for (int dy = 0; dy < 2; ++dy)
#pragma unroll
        for (int dx = 0; dx < 2; ++dx) {
          const float v = act_f(s[dy][dx] + bb, a.act);
          if (a.out_f32) {
            if (okpix[dy][dx] && cl < nco) reinterpret_cast<float*>(a.out)[opix[dy][dx] + cl] = v;
          } else {
            pk[dy][dx][cl >> 1] |= tbits((T)v) << (16 * (cl & 1));
          }
        }
    }
    // keep the scheduler from hoisting every channel's weight reads (register pressure)
    __builtin_amdgcn_sched_barrier(0);
  }

  if constexpr (POOL) {
    const int PHo = a.OH / 2, PWo = a.OW / 2, py = oy / 2, px = ox / 2;
    if (py >= PHo || px >= PWo) return;
    const long long o = (((long long)n * PHo + py) * PWo + px) * a.CO + cb;
    T* dst = reinterpret_cast<T*>(a.out) + o;
    if (nco == 16 && (a.CO & 7) == 0) {
      reinterpret_cast<uint4*>(dst)[0] = uint4{pk[0][0][0], pk[0][0][1], pk[0][0][2], pk[0][0][3]};
      reinterpret_cast<uint4*>(dst)[1] = uint4{pk[0][0][4], pk[0][0][5], pk[0][0][6], pk[0][0][7]};
    } else {
      for (int cl = 0; cl < nco; ++cl)
        dst[cl] = from_bits<T>(pk[0][0][cl >> 1] >> (16 * (cl & 1)));
    }
    if (a.argmax) {
      if (nco == 16 && (a.CO & 15) == 0)
        *reinterpret_cast<uint4*>(a.argmax + o) = uint4{am[0], am[1], am[2], am[3]};
      else
        for (int cl = 0; cl < nco; ++cl)
          a.argmax[o + cl] = (unsigned char)(am[cl >> 2] >> (8 * (cl & 3)));
    }
  } else if (!a.out_f32) {
#pragma unroll
    for (int dy = 0; dy < 2; ++dy)
#pragma unroll
      for (int dx = 0; dx < 2; ++dx) {
        if (!okpix[dy][dx]) continue;
        T* dst = reinterpret_cast<T*>(a.out) + opix[dy][dx];
        uint32_t* w8 = pk[dy][dx];
        if (a.mask) {
          const T* mk = reinterpret_cast<const T*>(a.mask) + opix[dy][dx];
          uint32_t m8[8];
          if (nco == 16 && (a.CO & 7) == 0) {
            const uint4 m0 = reinterpret_cast<const uint4*>(mk)[0], m1 = reinterpret_cast<const uint4*>(mk)[1];
            m8[0] = m0.x; m8[1] = m0.y; m8[2] = m0.z; m8[3] = m0.w;
            m8[4] = m1.x; m8[5] = m1.y; m8[6] = m1.z; m8[7] = m1.w;
          } else {
#pragma unroll
            for (int i = 0; i < 8; ++i) m8[i] = 0u;
            for (int cl = 0; cl < nco; ++cl) m8[cl >> 1] |= tbits(mk[cl]) << (16 * (cl & 1));
          }
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const uint32_t lo = (float)from_bits<T>(m8[i] & 0xffffu) > 0.f ? 0x0000ffffu : 0u;
            const uint32_t hi = (float)from_bits<T>(m8[i] >> 16) > 0.f ? 0xffff0000u : 0u;
            w8[i] &= lo | hi;
          }
        }
        if (nco == 16 && (a.CO & 7) == 0) {
          reinterpret_cast<uint4*>(dst)[0] = uint4{w8[0], w8[1], w8[2], w8[3]};
          reinterpret_cast<uint4*>(dst)[1] = uint4{w8[4], w8[5], w8[6], w8[7]};
        } else {
          for (int cl = 0; cl < nco; ++cl) dst[cl] = from_bits<T>(w8[cl >> 1] >> (16 * (cl & 1)));
        }
      }
  }
}

// ------------------------------------------------------------------ CO == 1
// One workgroup streams a band of a 128-column strip of one image top to bottom (bands of
// band_steps x TR output rows, so that a batch of 128 x 128 images still spreads over the
// whole chip; a band re-reads the K - 1 halo rows above it), TR output rows per step. The
// input rows live in an LDS ring of TR + K - 1 rows: each step reads only its TR
// new rows from HBM (no halo re-reads), and they are loaded into registers one step ahead,
// while the current rows compute.
template <int C>
struct Co1 {
  static constexpr int P = 64 / C;            // output pixels per lane
  static constexpr int TW = 128;              // output columns per workgroup
  static constexpr int TR = 256 / (TW / P);   // output rows per step (8 or 4)
  static constexpr int GS = P * C * 2 + 16;   // bytes per group of P patch pixels (144)
};

template <int C, int K>
struct Co1Ring {
  using G = Co1<C>;
  static constexpr int NG = (G::TW + K - 1 + G::P - 1) / G::P;  // groups per ring row
  static constexpr int RB = NG * G::GS;                          // bytes per ring row
  static constexpr int RN = G::TR + K - 1;                       // ring rows
  static constexpr int C8 = C / 8;                               // 16-byte pieces per pixel
  static constexpr int PIECES = G::TR * NG * G::P * C8;          // per step (new rows)
  static constexpr int PPT = (PIECES + 255) / 256;               // pieces per thread
  static constexpr int LDS = RN * RB + K * K * (C / 2) * 4;
};

template <typename T, int C, int K>
__global__ __launch_bounds__(256) void conv_co1_kernel(NarrowArgs a) {
  using G = Co1<C>;
  using Rg = Co1Ring<C, K>;
  constexpr int P = G::P, TR = G::TR, TW = G::TW, GS = G::GS;
  constexpr int NG = Rg::NG, RB = Rg::RB, RN = Rg::RN, C8 = Rg::C8;
  constexpr int CW = C / 2;  // 32-bit words per pixel
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* sP = smem;                                    // RN x RB ring
  uint32_t* sW = reinterpret_cast<uint32_t*>(smem + RN * RB);  // [K][K][CW]

  const int tid = threadIdx.x;
  const int ntx = (a.OW + TW - 1) / TW;
  const int n = blockIdx.x / ntx;
  const int ox0 = (blockIdx.x - n * ntx) * TW;
  const int ix0 = ox0 - a.pad_l;
  const int step0 = blockIdx.y * a.band_steps;
  const int nsteps = min((a.OH + TR - 1) / TR, step0 + a.band_steps);
  const T* __restrict__ in = reinterpret_cast<const T*>(a.in);
  const T* __restrict__ img = in + (long long)n * a.IH * a.IW * C;

  // piece e of input row iy: pixel px = e / C8 of the strip, 16-byte piece h = e % C8
  auto fetch = [&](int iy, int e) -> uint4 {
    const int px = e / C8, h = e - (e / C8) * C8;
    const int ix = ix0 + px;
    const bool ok = px < NG * P && (unsigned)iy < (unsigned)a.IH && (unsigned)ix < (unsigned)a.IW;
    return ok ? *reinterpret_cast<const uint4*>(img + ((long long)iy * a.IW + ix) * C + 8 * h)
              : uint4{0u, 0u, 0u, 0u};
  };
  auto put = [&](int iy, int e, uint4 v) {
    const int px = e / C8, h = e - (e / C8) * C8;
    const int slot = (iy + a.pad_t) % RN;
    if (px < NG * P)
      *reinterpret_cast<uint4*>(sP + slot * RB + (px / P) * GS + (px % P) * (2 * C) + 16 * h) = v;
  };
  constexpr int ROWP = NG * P * C8;  // pieces per input row

  // prologue: the first step's RN rows
  for (int e = tid; e < RN * ROWP; e += 256) {
    const int rr = e / ROWP, pe = e - rr * ROWP;
    const int iy = step0 * TR - a.pad_t + rr;
    put(iy, pe, fetch(iy, pe));
  }
  for (int e = tid; e < K * K * CW; e += 256)
    sW[e] = reinterpret_cast<const uint32_t*>(a.w)[e];  // [ky][kx][ci pairs] (CO == 1)
  __syncthreads();

  const int g = tid % (TW / P), r = tid / (TW / P);
  const float bb = a.bias ? a.bias[0] : 0.f;
  for (int step = step0; step < nsteps; ++step) {
    // next step's TR new rows into registers (their latency hides under this step)
    const int ny0 = (step + 1) * TR - a.pad_t + K - 1;  // first new input row of step + 1
    uint4 nx[Rg::PPT];
    const bool more = step + 1 < nsteps;
#pragma unroll
    for (int j = 0; j < Rg::PPT; ++j) {
      const int e = tid + j * 256;
      nx[j] = uint4{0u, 0u, 0u, 0u};
      if (more && e < Rg::PIECES) nx[j] = fetch(ny0 + e / ROWP, e % ROWP);
    }

    float acc[P];
#pragma unroll
    for (int p = 0; p < P; ++p) acc[p] = 0.f;
    const int iyb = step * TR - a.pad_t + r;  // input row of (r, ky = 0)
#pragma unroll 1
    for (int ky = 0; ky < K; ++ky) {
      const unsigned char* row = sP + ((iyb + ky + a.pad_t) % RN) * RB + g * GS;
#pragma unroll
      for (int c = 0; c < P + K - 1; ++c) {
        uint32_t col[CW];
        const unsigned char* src = row + (c / P) * GS + (c % P) * (2 * C);
#pragma unroll
        for (int h = 0; h < C8; ++h) {
          const uint4 u = *reinterpret_cast<const uint4*>(src + 16 * h);
          col[4 * h] = u.x;
          col[4 * h + 1] = u.y;
          col[4 * h + 2] = u.z;
          col[4 * h + 3] = u.w;
        }
#pragma unroll
        for (int kx = 0; kx < K; ++kx) {
          const int p = c - kx;
          if (p < 0 || p >= P) continue;  // compile-time
          const uint32_t* wr = sW + (ky * K + kx) * CW;
#pragma unroll
          for (int h = 0; h < C8; ++h) {
            const uint4 w4 = *reinterpret_cast<const uint4*>(wr + 4 * h);  // broadcast
            acc[p] = dot2<T>(col[4 * h], w4.x, acc[p]);
            acc[p] = dot2<T>(col[4 * h + 1], w4.y, acc[p]);
            acc[p] = dot2<T>(col[4 * h + 2], w4.z, acc[p]);
            acc[p] = dot2<T>(col[4 * h + 3], w4.w, acc[p]);
          }
        }
        __builtin_amdgcn_sched_barrier(0);  // one input column live at a time
      }
    }

    // epilogue: bias, logits, activation, P consecutive pixels of one row
    const int oy = step * TR + r, ox = ox0 + g * P;
    if (oy < a.OH && ox < a.OW) {
      const long long o = ((long long)n * a.OH + oy) * a.OW + ox;
      float v[P];
#pragma unroll
      for (int p = 0; p < P; ++p) v[p] = acc[p] + bb;
      const bool full = ox + P <= a.OW && (a.OW % P) == 0;
      if (a.logits) {
        if (full && P == 4) {
          *reinterpret_cast<float4*>(a.logits + o) = float4{v[0], v[1], v[P > 2 ? 2 : 0], v[P - 1]};
        } else {
          for (int p = 0; p < P; ++p)
            if (ox + p < a.OW) a.logits[o + p] = v[p];
        }
      }
#pragma unroll
      for (int p = 0; p < P; ++p) v[p] = act_f(v[p], a.act);
      if (a.out_f32) {
        float* dst = reinterpret_cast<float*>(a.out) + o;
        if (full && P == 4) {
          *reinterpret_cast<float4*>(dst) = float4{v[0], v[1], v[P > 2 ? 2 : 0], v[P - 1]};
        } else if (full && P == 2) {
          *reinterpret_cast<float2*>(dst) = float2{v[0], v[1]};
        } else {
          for (int p = 0; p < P; ++p)
            if (ox + p < a.OW) dst[p] = v[p];
        }
      } else {
        T* dst = reinterpret_cast<T*>(a.out) + o;
        for (int p = 0; p < P; ++p)
          if (ox + p < a.OW) dst[p] = (T)v[p];
      }
    }
    if (!more) break;
    __syncthreads();  // every lane is done with the ring rows the new ones replace
#pragma unroll
    for (int j = 0; j < Rg::PPT; ++j) {
      const int e = tid + j * 256;
      if (e < Rg::PIECES) put(ny0 + e / ROWP, e % ROWP, nx[j]);
    }
    __syncthreads();
  }
}

template <typename T, int C, int K>
int launch_co1(const NarrowArgs& a, hipStream_t st) {
  using Rg = Co1Ring<C, K>;
  static_assert(Rg::LDS <= 160 * 1024, "LDS budget");
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute((const void*)conv_co1_kernel<T, C, K>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, Rg::LDS) != hipSuccess)
      return set_error(SPECENH_EHIP, "conv_co1 attribute");
    attr = true;
  }
  const long long strips = (long long)a.N * ((a.OW + Co1<C>::TW - 1) / Co1<C>::TW);
  // bands: ~1024 workgroups (every CU busy) unless the halo re-reads would exceed ~25%
  const int steps = (a.OH + Co1<C>::TR - 1) / Co1<C>::TR;
  const int min_steps = std::max(1, (4 * (K - 1) + Co1<C>::TR - 1) / Co1<C>::TR);
  long long bands = std::max(1LL, std::min<long long>(steps, (1024 + strips - 1) / strips));
  NarrowArgs b = a;
  b.band_steps = std::max<int>(min_steps, (int)((steps + bands - 1) / bands));
  bands = (steps + b.band_steps - 1) / b.band_steps;
  SPECENH_LAUNCH((conv_co1_kernel<T, C, K>), dim3((unsigned)strips, (unsigned)bands), dim3(256),
                     Rg::LDS, st, b);
  return hipGetLastError() == hipSuccess ? 1 : set_error(SPECENH_EHIP, "conv_co1 launch");
}

// ---------------------------------------------------------------- CO == 1 on the MFMA
// conv_co1m_kernel<T, NKS, K>: one output channel from C = 32 NKS input channels (the last
// Conv2D of the reference's 64/32-channel variants, VAE/manual_scan.py:199,
// hyperparam_scan.py:161) as D[kx][x'] = sum_(ky, ci) w[ky][kx][ci] in[y + ky - p][x'][ci]
// on v_mfma_f32_16x16x32 (A = the weights, rows kx < K of 16; B = 16 input positions x'),
// then out[y][x] = sum_kx D[kx][x + kx - p] through a per-wave LDS scratch. The 16 x 16 tile
// keeps K of its 16 rows (5 / 16 at K = 5) where a 16-channel output tile keeps 1 / 16, and
// the K taps of a kernel row cost one MFMA per 32 channels. A wave owns 16 output columns x R
// output rows: each input row's B fragments (two tiles, x' = x0 - 8 .. x0 + 23) are loaded
// once and feed the K output rows that use it.
#ifndef SPECENH_CO1M_R
#define SPECENH_CO1M_R 8
#endif
typedef _Float16 f16x8m __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8m __attribute__((ext_vector_type(8)));
typedef float f32x4m __attribute__((ext_vector_type(4)));
template <typename T>
__device__ __forceinline__ f32x4m mfma16(const uint4& a, const uint4& b, f32x4m acc) {
  if constexpr (__is_same(T, _Float16))
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8m, a),
                                                  __builtin_bit_cast(f16x8m, b), acc, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8m, a),
                                                   __builtin_bit_cast(bf16x8m, b), acc, 0, 0, 0);
}

template <typename T, int NKS, int K>
__global__ __launch_bounds__(256) void conv_co1m_kernel(NarrowArgs a) {
  constexpr int C = 32 * NKS, R = SPECENH_CO1M_R, P = K / 2, NIR = R + K - 1;
  __shared__ __attribute__((aligned(16))) float scr[4][32][16];  // per wave: [x' - x0 + 8][kx]
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int m = lane & 15, kg = lane >> 4;
  const int nstrip = (a.OW + 15) / 16, ngrp = (nstrip + 3) / 4, nband = (a.OH + R - 1) / R;
  int bid = blockIdx.x;
  const int grp = bid % ngrp;
  bid /= ngrp;
  const int band = bid % nband, n = bid / nband;
  const int strip = grp * 4 + wv;
  if (strip >= nstrip) return;  // (whole wave: no barriers below)
  const int x0 = 16 * strip, y0 = band * R;
  const T* __restrict__ in = reinterpret_cast<const T*>(a.in) + (long long)n * a.IH * a.IW * C;
  // weights: A fragment of (ky, k-step): row kx = m (< K), channels 32 ks + 8 kg .. + 7
  uint4 wf[K][NKS];
  {
    const T* __restrict__ W = reinterpret_cast<const T*>(a.w);  // [1][K][K][C]
#pragma unroll
    for (int ky = 0; ky < K; ++ky)
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks)
        wf[ky][ks] = m < K ? *reinterpret_cast<const uint4*>(W + ((ky * K + m) * C) + 32 * ks + 8 * kg)
                           : uint4{0u, 0u, 0u, 0u};
  }
  f32x4m acc[R][2];
#pragma unroll
  for (int o = 0; o < R; ++o) acc[o][0] = acc[o][1] = f32x4m{0.f, 0.f, 0.f, 0.f};
  // B fragments of input row iy: tile t, position x' = x0 - 8 + 16 t + m, channels of k-step
  auto load_row = [&](int iy, uint4 (&b)[2][NKS]) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int xp = x0 - 8 + 16 * t + m;
      const bool ok = (unsigned)iy < (unsigned)a.IH && (unsigned)xp < (unsigned)a.IW;
      const T* src = in + ((long long)(ok ? iy : 0) * a.IW + (ok ? xp : 0)) * C + 8 * kg;
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        const uint4 v = *reinterpret_cast<const uint4*>(src + 32 * ks);
        b[t][ks] = ok ? v : uint4{0u, 0u, 0u, 0u};
      }
    }
  };
  uint4 bc[2][NKS], bn[2][NKS];
  load_row(y0 - P, bc);
#pragma unroll
  for (int ir = 0; ir < NIR; ++ir) {
    if (ir + 1 < NIR) load_row(y0 - P + ir + 1, bn);  // next row's loads behind these MFMAs
#pragma unroll
    for (int ky = 0; ky < K; ++ky) {
      const int o = ir - ky;  // output row y0 + o reads input row y0 + o + ky - P
      if (o < 0 || o >= R) continue;  // compile-time
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) acc[o][t] = mfma16<T>(wf[ky][ks], bc[t][ks], acc[o][t]);
    }
    if (ir + 1 < NIR) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) bc[t][ks] = bn[t][ks];
    }
  }
  // out[y][x0 + j] = sum_kx D[kx][x0 + j + kx - P]: lane (x' = m, rows kx = 4 kg + i) writes its
  // four D values of each tile as one 16-byte run of scr[x'][kx]; lanes 0-15 sum the diagonal
  const float bb = a.bias ? a.bias[0] : 0.f;
  float (*sw)[16] = scr[wv];
#pragma unroll
  for (int o = 0; o < R; ++o) {
    const int oy = y0 + o;
#pragma unroll
    for (int t = 0; t < 2; ++t)
      *reinterpret_cast<float4*>(&sw[16 * t + m][4 * kg]) =
          float4{acc[o][t][0], acc[o][t][1], acc[o][t][2], acc[o][t][3]};
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (LDS is in order per wave; this
                                                          // also keeps the compiler's order)
    float v = bb;
#pragma unroll
    for (int kx = 0; kx < K; ++kx) v += sw[m + kx - P + 8][kx];
    const int ox = x0 + m;
    if (lane < 16 && oy < a.OH && ox < a.OW) {
      const long long oi = ((long long)n * a.OH + oy) * a.OW + ox;
      if (a.logits) a.logits[oi] = v;
      const float r = act_f(v, a.act);
      if (a.out_f32) reinterpret_cast<float*>(a.out)[oi] = r;
      else reinterpret_cast<T*>(a.out)[oi] = (T)r;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads before the next row's writes
  }
}

template <typename T, int NKS, int K>
int launch_co1m(const NarrowArgs& a, hipStream_t st) {
  constexpr int R = SPECENH_CO1M_R;
  const long long nstrip = (a.OW + 15) / 16, ngrp = (nstrip + 3) / 4;
  const long long blocks = (long long)a.N * ((a.OH + R - 1) / R) * ngrp;
  if (blocks > 0x7fffffffLL) return 0;
  SPECENH_LAUNCH((conv_co1m_kernel<T, NKS, K>), dim3((unsigned)blocks), dim3(256), 0, st, a);
  return hipGetLastError() == hipSuccess ? 1 : set_error(SPECENH_EHIP, "conv_co1m launch");
}

template <typename T, int K>
int launch_c1(const NarrowArgs& a, bool pool, hipStream_t st) {
  const long long tiles = (long long)a.N * ((a.OH + C1_TILE - 1) / C1_TILE) *
                          ((a.OW + C1_TILE - 1) / C1_TILE);
  const dim3 grid((unsigned)tiles, (unsigned)((a.CO + 15) / 16));
  if (pool) SPECENH_LAUNCH((conv_c1_kernel<T, K, true>), grid, dim3(256), 0, st, a);
  else SPECENH_LAUNCH((conv_c1_kernel<T, K, false>), grid, dim3(256), 0, st, a);
  return hipGetLastError() == hipSuccess ? 1 : set_error(SPECENH_EHIP, "conv_c1 launch");
}

template <typename T>
int dispatch(const NarrowArgs& a, int K, bool pool, hipStream_t st) {
  if (a.mask && (a.C != 1 || pool || a.out_f32 || a.act == SPECENH_ACT_SIGMOID)) return 0;  // act(0) = 0
  if (a.C == 1) {
    if (a.logits) return 0;
    switch (K) {
      case 3: return launch_c1<T, 3>(a, pool, st);
      case 5: return launch_c1<T, 5>(a, pool, st);
      case 7: return launch_c1<T, 7>(a, pool, st);
      default: return 0;
    }
  }
  if (a.CO == 1 && !pool) {
    // C = 64, or 32 at K >= 5, "same" padding: the MFMA kernel (CO1_VALU=1 keeps
    // conv_co1_kernel for 32). Per 512 x 256 x 128 launch: C 64 / K 5 1.85 ms (16-channel
    // MFMA patch tile) -> 0.84, C 32 / K 7 1.15 (VALU) -> 0.57, C 32 / K 5 -> 0.39; C 32 / K 3
    // stays on the VALU kernel (0.30 vs 0.35 ms).
    const bool same = a.pad_t == K / 2 && a.pad_l == K / 2 && a.OH == a.IH && a.OW == a.IW;
    if (same && (a.C == 64 || (a.C == 32 && K >= 5 && variant(V_CO1_VALU) == 0))) {
      if (a.C == 64) {
        switch (K) {
          case 3: return launch_co1m<T, 2, 3>(a, st);
          case 5: return launch_co1m<T, 2, 5>(a, st);
          case 7: return launch_co1m<T, 2, 7>(a, st);
          default: return 0;
        }
      }
      switch (K) {
        case 5: return launch_co1m<T, 1, 5>(a, st);
        case 7: return launch_co1m<T, 1, 7>(a, st);
        default: return 0;
      }
    }
    if (a.C == 16) {
      switch (K) {
        case 3: return launch_co1<T, 16, 3>(a, st);
        case 5: return launch_co1<T, 16, 5>(a, st);
        case 7: return launch_co1<T, 16, 7>(a, st);
        default: return 0;
      }
    }
    if (a.C == 32) {
      switch (K) {
        case 3: return launch_co1<T, 32, 3>(a, st);
        case 5: return launch_co1<T, 32, 5>(a, st);
        case 7: return launch_co1<T, 32, 7>(a, st);
        default: return 0;
      }
    }
  }
  return 0;
}

}  // namespace

// Narrow-channel direct convolution (C == 1, or CO == 1 with C in {16, 32, 64}), bf16/f16,
// stride 1, undilated, square odd kernel <= 7 (a ReLU mask only for C == 1 without pooling
// or fp32 output). Returns 1 when launched, 0
// when the shape is not covered (the caller takes the MFMA path), < 0 on error.
int launch_conv_narrow(int dtype, const void* in, int N, int IH, int IW, int C, const void* w,
                       int KH, int KW, int CO, const float* bias, int pad_t, int pad_l, int OH,
                       int OW, int act, void* out, int out_f32, float* logits, int pool,
                       unsigned char* argmax, const void* mask, hipStream_t st) {
  if (dtype == SPECENH_DTYPE_F32 || KH != KW || (KH & 1) == 0 || KH > 7) return 0;
  if (C != 1 && CO != 1) return 0;
  if (pool && ((OH & 1) || (OW & 1))) return 0;
  NarrowArgs a{in, w, bias, out, logits, argmax, N, IH, IW, C, OH, OW, CO,
               pad_t, pad_l, act, out_f32, mask, 0};
  if (dtype == SPECENH_DTYPE_BF16) return dispatch<__bf16>(a, KH, pool != 0, st);
  return dispatch<_Float16>(a, KH, pool != 0, st);
}

}  // namespace specenh
