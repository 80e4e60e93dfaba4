// conv_c1_mfma.hip — one-input-channel convolutions on MFMA (gfx950).
//
// The first Conv2D of the reference model (1 -> 16 channels, k 5, relu, then
// MaxPooling2D((2,2)); VAE/manual_scan_3layers.py:187-188). The masked epilogue below also
// serves the input gradient of the last conv, 16 -> 1 through the previous ReLU, :199 (round 6
// default: with the C4 weight gradients on two side streams the C4 step is 0.688 -> 0.671 ms
// against the VALU kernel, which round 5 had kept; SPECENH_C1_MASK_MFMA=0 selects it). With
// C == 1 the GEMM-K of a pixel is its K x K window. The window
// rows are contiguous runs of the input row, so the MFMA K index is laid out as (ky, kx)
// with kx padded to 8: a lane's 8 K-elements are ONE 8-element run of an input row, and
// one 16x16x32 MFMA covers 4 kernel rows of 16 pixels x 16 output channels (2 MFMAs for
// K <= 8 rows). The staged rows are kept twice in LDS as 32-bit words, as loaded and
// shifted by one element, so every run starts on a word of one copy and a B fragment is
// four word reads (no per-pixel record building). Weights (the A operand: rows = output
// channels, kx >= K zero) stay in registers for the whole workgroup.
//
// Workgroup: a 32 x 32 output tile x 16 output channels (blockIdx.y), 4 waves of 8 output
// rows x 2 column blocks: block cb holds the pixels x = 2 l16 + cb, so the 2x2 max-pool
// window of a lane's pooled pixel is in its own accumulators (no cross-lane exchange, every
// lane stores). Epilogues as in conv_patch_kernel (csrc/conv_ae.hip):
// fused 2x2 max-pool (+ argmax; values compared as stored in T, first max wins; without
// argmax the max accumulator is taken first, a monotone map, bitwise the same), or plain
// stores with the optional ReLU mask of the backward pass (act(0) = 0 there).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <string>

#include "specenh.h"
#include "runtime.hpp"

namespace specenh {
int set_error(int code, const std::string& msg);  // stft_psd.hip

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

struct C1mArgs {
  const void* in;    // [N][IH][IW] (C == 1)
  const void* w;     // w_gemm [CO][K][K]
  const float* bias;
  void* out;         // [N][OH][OW][CO] or pooled [N][OH/2][OW/2][CO]
  const void* mask;  // plain epilogue only: out = 0 where mask <= 0
  unsigned char* argmax;
  int N, IH, IW, OH, OW, CO, K, pad_t, pad_l, act;
};

constexpr int TILE = 32;
constexpr int PRS = 40;  // patch rows (32 + K - 1 <= 39), + 1 for clamped reads
constexpr int RW = 20;   // staged row: 20 words = 40 elements (runs start at <= 32, 8 long)
constexpr int RDW = 48;  // LDS row pitch in words: the 4 kernel-row lane groups of a
                         // fragment read sit 48 = -16 (mod 64) banks apart: conflict-free

template <typename T>
__device__ __forceinline__ float tof(T x) { return (float)x; }

template <typename T>
__device__ __forceinline__ f32x4 mfma(uint4 a, uint4 b, f32x4 c) {
  if constexpr (__is_same(T, __bf16))
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                   __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a),
                                                  __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}

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

__device__ __forceinline__ float act_f(float v, int act) {
  if (act == SPECENH_ACT_RELU) return fmaxf(v, 0.f);
  if (act == SPECENH_ACT_SIGMOID) return 1.f / (1.f + __expf(-v));
  return v;
}

template <typename T, bool POOL, int PAR>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void conv_c1_mfma_kernel(C1mArgs a) {
  // Staged rows as 32-bit words: P0[r][j] = elements (2j, 2j+1) of staged row r, and the
  // copy shifted by one element P1[r][j] = (2j+1, 2j+2). Every 8-element run a fragment
  // needs then starts on a word of one of them (even start: P0, odd start: P1).
  __shared__ uint32_t sP0[PRS * RDW], sP1[PRS * RDW];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ntx = (a.OW + TILE - 1) / TILE, nty = (a.OH + TILE - 1) / TILE;
  const int tpi = ntx * nty;  // tiles per image; gridDim.x is a multiple of it
  const int co0 = blockIdx.y * 16;
  const int K = a.K, PR = TILE + K - 1;
  // PAR = pad_l & 1: staged rows start at the even element ix0 - PAR
  // this workgroup's tile position (fixed) and images n0, n0 + nstep, ...
  const int trem = blockIdx.x % tpi, n0 = blockIdx.x / tpi, nstep = gridDim.x / tpi;
  const int oy0 = (trem / ntx) * TILE, ox0 = (trem % ntx) * TILE;
  const int iy0 = oy0 - a.pad_t, ix0 = ox0 - a.pad_l - PAR;
  const T* __restrict__ in = reinterpret_cast<const T*>(a.in);
  const T* __restrict__ W = reinterpret_cast<const T*>(a.w);

  // a tile's patch rows -> registers as words (all loads in flight, zero outside the image;
  // IW even and the word start even, so a word is entirely inside or outside). The
  // per-thread (row, word) slots and their in-image test are the same for every image.
  constexpr int NW = (PRS * RW + 255) / 256;
  uint32_t v[NW];
  int woff[NW];  // element offset of the word in an image, -1: zero
  int soff[NW];  // LDS word index, -1: none
#pragma unroll
  for (int k = 0; k < NW; ++k) {
    const int e = tid + 256 * k;
    const int r = e / RW, j = e - (e / RW) * RW;
    const int iy = iy0 + r, ix = ix0 + 2 * j;
    const bool ok = e < PRS * RW && r < PR && (unsigned)iy < (unsigned)a.IH &&
                    (unsigned)ix < (unsigned)a.IW;
    woff[k] = ok ? iy * a.IW + ix : -1;
    soff[k] = e < PRS * RW ? r * RDW + j : -1;
  }
  const long long img = (long long)a.IH * a.IW;
  auto fetch = [&](int n) {
    const T* src = in + n * img;
#pragma unroll
    for (int k = 0; k < NW; ++k) {
      v[k] = *reinterpret_cast<const uint32_t*>(src + (woff[k] >= 0 ? woff[k] : 0));
      if (woff[k] < 0) v[k] = 0u;
    }
  };
  // ---- weights (A operand): lane = (co = lane & 15, kernel row 4 s + (lane >> 4)) ----
  const int g4 = lane >> 4, l16 = lane & 15;
  uint4 wf[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int ky = 4 * s + g4, co = co0 + l16;
    uint32_t w4[4] = {0u, 0u, 0u, 0u};
    if (ky < K && co < a.CO) {
      const T* wr = W + ((long long)co * K + ky) * K;
#pragma unroll
      for (int kx = 0; kx < 8; ++kx)
        if (kx < K) w4[kx >> 1] |= (uint32_t)__builtin_bit_cast(unsigned short, wr[kx]) << (16 * (kx & 1));
    }
    wf[s] = uint4{w4[0], w4[1], w4[2], w4[3]};
  }

  float bv[4];  // biases of this lane's channels co0 + 4 g4 + r
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int ch = co0 + 4 * g4 + r;
    bv[r] = (a.bias && ch < a.CO) ? a.bias[ch] : 0.f;
  }
  // weights and biases are in registers before the loop: a wait for them inside the loop
  // would also wait for the prefetch and (CDNA4 vmcnt counts stores) the previous stores
  __builtin_amdgcn_s_waitcnt(0x0F70);  // s_waitcnt vmcnt(0)

  // persistent over images n0, n0 + nstep, ... at a fixed tile position: the next image's
  // rows are loaded into registers while this one's MFMAs and stores run
  if (n0 < a.N) fetch(n0);
  for (int n = n0; n < a.N; n += nstep) {
  __syncthreads();  // the previous tile's fragment reads are done
#pragma unroll
  for (int k = 0; k < NW; ++k)
    if (soff[k] >= 0) sP0[soff[k]] = v[k];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NW; ++k)  // the shifted copy (word RW of a row, element 40, unused)
    if (soff[k] >= 0) sP1[soff[k]] = __builtin_amdgcn_alignbit(sP0[soff[k] + 1], sP0[soff[k]], 16);
  __syncthreads();
  if (n + nstep < a.N) fetch(n + nstep);

  // ---- MFMAs: wave rows 8 wave + 4 hf + i (two halves of 4 rows: half the accumulator
  // registers live at a time). Column block cb holds the pixels x = 2 l16 + cb, so a 2x2
  // pooling window is (acc[2ip][0..1], acc[2ip+1][0..1]) of ONE lane. Pixel x's run starts
  // at staged element x + PAR: P0 word l16 + PAR when cb == PAR, else P1 word l16.
  const int nks = (K + 3) / 4;
#pragma unroll 1
  for (int hf = 0; hf < 2; ++hf) {
  const int rw0 = 8 * wave + 4 * hf;  // first tile row of this half
  f32x4 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i][0] = acc[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        if (s >= nks) break;  // uniform
        const int r = rw0 + i + 4 * s + g4;  // <= 38 < PRS; rows past K meet zero weights
        const uint32_t* q = (cb == PAR ? sP0 + PAR : sP1) + r * RDW + l16;
        acc[i][cb] = mfma<T>(wf[s], uint4{q[0], q[1], q[2], q[3]}, acc[i][cb]);
      }

  // ---- epilogue: lane holds channels co0 + 4 g4 + r of pixels (rw0 + i, 2 l16 + cb) ----
  const int ch0 = co0 + 4 * g4;
  const bool vec = (a.CO & 3) == 0;
  if constexpr (POOL) {
    const int PHo = a.OH / 2, PWo = a.OW / 2;
#pragma unroll
    for (int ip = 0; ip < 2; ++ip) {
      const int py = (oy0 + rw0 + 2 * ip) / 2, px = ox0 / 2 + l16;
      const bool store = py < PHo && px < PWo && ch0 < a.CO;
      const long long o = (((long long)n * PHo + py) * PWo + px) * a.CO + ch0;
      T* dst = reinterpret_cast<T*>(a.out) + o;
      float m[4];
      unsigned arg4 = 0;
      if (!a.argmax && a.act <= 1) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = vmax(vmax(acc[2 * ip][0][r], acc[2 * ip][1][r]),
                               vmax(acc[2 * ip + 1][0][r], acc[2 * ip + 1][1][r])) + bv[r];
          m[r] = a.act == 1 ? vmax(v, 0.f) : v;
        }
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v00 = tof((T)act_f(acc[2 * ip][0][r] + bv[r], a.act));
          const float v01 = tof((T)act_f(acc[2 * ip][1][r] + bv[r], a.act));
          const float v10 = tof((T)act_f(acc[2 * ip + 1][0][r] + bv[r], a.act));
          const float v11 = tof((T)act_f(acc[2 * ip + 1][1][r] + bv[r], a.act));
          float b = v00;
          unsigned q = 0;
          if (v01 > b) { b = v01; q = 1; }
          if (v10 > b) { b = v10; q = 2; }
          if (v11 > b) { b = v11; q = 3; }
          m[r] = b;
          arg4 |= q << (8 * r);
        }
      }
      if (!store) continue;
      if (vec) {
        *reinterpret_cast<uint2*>(dst) = uint2{pack2<T>(m[0], m[1]), pack2<T>(m[2], m[3])};
        if (a.argmax) *reinterpret_cast<unsigned*>(a.argmax + o) = arg4;
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (ch0 + r < a.CO) {
            dst[r] = (T)m[r];
            if (a.argmax) a.argmax[o + r] = (unsigned char)(arg4 >> (8 * r));
          }
      }
    }
  } else {
    const T* __restrict__ mk = reinterpret_cast<const T*>(a.mask);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        const int oy = oy0 + rw0 + i, ox = ox0 + 2 * l16 + cb;
        if (oy >= a.OH || ox >= a.OW || ch0 >= a.CO) continue;
        const long long o = (((long long)n * a.OH + oy) * a.OW + ox) * a.CO + ch0;
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = act_f(acc[i][cb][r] + bv[r], a.act);
        if (vec) {
          if (mk) {
            const uint2 mm = *reinterpret_cast<const uint2*>(mk + o);
            const uint32_t mw[2] = {mm.x, mm.y};
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const T mv = __builtin_bit_cast(T, (unsigned short)(mw[r >> 1] >> (16 * (r & 1))));
              v[r] = tof(mv) > 0.f ? v[r] : 0.f;
            }
          }
          *reinterpret_cast<uint2*>(reinterpret_cast<T*>(a.out) + o) =
              uint2{pack2<T>(v[0], v[1]), pack2<T>(v[2], v[3])};
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            if (ch0 + r >= a.CO) continue;
            float x = v[r];
            if (mk && !(tof(mk[o + r]) > 0.f)) x = 0.f;
            reinterpret_cast<T*>(a.out)[o + r] = (T)x;
          }
        }
      }
  }
  }  // row halves
  }  // images
}

template <typename T, bool POOL>
int launch_t(const C1mArgs& a, hipStream_t st) {
  const long long tpi = (long long)((a.OH + TILE - 1) / TILE) * ((a.OW + TILE - 1) / TILE);
  const int cus = device_cus();
  const bool par = a.pad_l & 1;
  const void* fn = par ? (const void*)conv_c1_mfma_kernel<T, POOL, 1>
                       : (const void*)conv_c1_mfma_kernel<T, POOL, 0>;
  static int per_cu[2] = {0, 0};
  int& pc = per_cu[POOL ? 1 : 0];
  if (pc == 0 && (hipOccupancyMaxActiveBlocksPerMultiprocessor(&pc, fn, 256, 0) != hipSuccess || pc <= 0))
    pc = 2;
  const unsigned cob = (unsigned)((a.CO + 15) / 16);
  // persistent: each workgroup keeps one tile position and walks the images; as many
  // image groups as fill the resident slots (at least one)
  const long long groups = std::max<long long>(1, std::min<long long>(a.N, (long long)pc * cus / cob / tpi));
  const dim3 grid((unsigned)(groups * tpi), cob);
  if (par) SPECENH_LAUNCH((conv_c1_mfma_kernel<T, POOL, 1>), grid, dim3(256), 0, st, a);
  else SPECENH_LAUNCH((conv_c1_mfma_kernel<T, POOL, 0>), grid, dim3(256), 0, st, a);
  return hipGetLastError() == hipSuccess ? 1 : set_error(SPECENH_EHIP, "conv_c1_mfma launch");
}

template <typename T>
int launch(const C1mArgs& a, bool pool, hipStream_t st) {
  return pool ? launch_t<T, true>(a, st) : launch_t<T, false>(a, st);
}

}  // namespace

// C == 1, 16-bit, stride 1, undilated, square kernel <= 8, T output (no fp32 logits /
// output, no mask). Returns 1 when launched, 0 when not covered.
int launch_conv_c1_mfma(int dtype, const void* in, int N, int IH, int IW, int C, const void* w,
                        int KH, int KW, int CO, const float* bias, int pad_t, int pad_l, int OH,
                        int OW, int act, void* out, int out_f32, float* logits, int pool,
                        unsigned char* argmax, const void* mask, hipStream_t st) {
  if (C != 1 || (dtype != SPECENH_DTYPE_BF16 && dtype != SPECENH_DTYPE_F16)) return 0;
  if (KH != KW || KH > 8 || out_f32 || logits) return 0;
  // the masked full-resolution store (the C4 input gradient of the last conv): here by default
  // (round 6, see the file comment; SPECENH_C1_MASK_MFMA=0: the VALU kernel)
  if (mask && variant(V_C1_MASK_MFMA) == 0) return 0;
  if (pool && ((OH & 1) || (OW & 1))) return 0;
  if ((IW & 1) || ((uintptr_t)in & 3)) return 0;  // staged as 32-bit words
  if ((long long)((OH + TILE - 1) / TILE) * ((OW + TILE - 1) / TILE) >= (1LL << 24) ||
      (long long)IH * IW >= (1LL << 31))
    return 0;
  C1mArgs a{in, w, bias, out, mask, argmax, N, IH, IW, OH, OW, CO, KH, pad_t, pad_l, act};
  if (dtype == SPECENH_DTYPE_BF16) return launch<__bf16>(a, pool != 0, st);
  return launch<_Float16>(a, pool != 0, st);
}

}  // namespace specenh
