// conv_rows.hip — the encoder's pooled 5 x 5 convolutions as a row sweep (gfx950).
//
// VAE/manual_scan_3layers.py:188-193: Conv2D(32, 5, relu, same) + MaxPooling2D(2) on the
// 64 x 64 x 16 map, Conv2D(64, 5, relu, same) + MaxPooling2D(2) on the 32 x 32 x 32 map.
// conv_patch_kernel (conv_ae.hip) runs these as 16 x 16 output tiles: every patch fragment
// feeds the MFMAs of ONE (tap, output row) and every tile re-stages a 2-pixel halo; PMC put
// both layers at 0.31-0.41 of the MFMA peak with ~5 VALU + 2.5 SALU instructions per MFMA.
// Here a workgroup walks whole images DOWN, two input rows per step:
//  * wave (window wx, channel block nb) owns 16 output columns x 16 output channels. Its 25
//    (CIN = 32) or 13 (CIN = 16, two taps per K = 32 step) weight fragments stay in registers
//    for the whole launch (the MFMA A operand: 16 output channels x 32 K).
//  * input row r is read ONCE per (window, tap column): that B fragment (32 K x 16 pixels)
//    feeds the MFMAs of all five kernel rows, i.e. output rows r + 2 - ky (5 MFMAs per LDS
//    read). Six accumulators (output rows 2q - 2 .. 2q + 3) rotate down the image.
//  * CIN = 16 pairs taps (kx, kx + 1) of one input row in a K step (columns 0-1, 2-3); the
//    fifth column pairs rows: F(r) = (row r, row r + 1) at kx = 4 feeds output rows r + 2
//    (weights w[0][4], w[1][4]), r (w[2][4], w[3][4]) and r - 2 (w[4][4], 0): 13 MFMAs per
//    input row for 12.5 taps of work (plus F(-1) once per image for output row 1).
//  * when output rows 2p, 2p + 1 are complete, the 2 x 2 max-pool runs in registers (rows in
//    lane, columns across the lane pair m, m ^ 1 by DPP); the bias is the accumulators'
//    start value and ReLU / rounding commute with the max, so pooled row p is
//    round_T(relu(max)) and is stored as 8 bytes per even lane.
//  * input rows arrive by LDS-DMA (global_load_lds, 16 B per lane) into an 8-row ring,
//    three steps ahead; rows outside the image are zero-filled, as is the 2-pixel halo of
//    every ring row. One workgroup barrier per step. Workgroups are persistent: the row
//    stream runs on across the workgroup's images (image i, rows 0 .. H + 1, the last two
//    zero), so the pipeline never drains between images.
// 64-byte pixels (CIN = 32) are stored with their 16-byte groups swizzled, g ^ ((p >> 1) & 3)
// (conflict-free B-fragment reads under the ds_read_b128 lane groups); 32-byte pixels need
// no swizzle. Host-checked shapes: (CIN, COUT, W) = (16, 32, 64) and (32, 64, 32), H even.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <mutex>
#include <string>
#include <type_traits>

#include "lds_dma.hpp"
#include "specenh.h"
#include "runtime.hpp"

namespace specenh {
int set_error(int code, const std::string& msg);  // stft_psd.hip

namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <typename T>
__device__ __forceinline__ f32x4 mfma(const uint4& a, const uint4& b, f32x4 acc) {
  if constexpr (__is_same(T, _Float16))
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a),
                                                  __builtin_bit_cast(f16x8, b), acc, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                   __builtin_bit_cast(bf16x8, b), acc, 0, 0, 0);
}

// two fp32 -> one packed pair of T (round to nearest even) as ONE v_cvt_pk_{f16,bf16}_f32;
// the element-wise form became two converts plus a shift and an or
template <typename T>
__device__ __forceinline__ uint32_t pack2(float lo, float hi) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  typedef T t2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f2{lo, hi}, t2));
}

__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}


// max with the neighbouring lane (m ^ 1): DPP quad_perm [1, 0, 3, 2]
__device__ __forceinline__ float max_pair(float v) {
  const float o = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, true));
  return fmaxf(v, o);
}

template <int CIN, int COUT, int W, int K = 5>
struct RC {
  static constexpr int NWIN = W / 16;                 // 16-column windows
  static constexpr int NNB = COUT / 16;               // 16-channel blocks
  static constexpr int WAVES = NWIN * NNB;
  static constexpr int THREADS = 64 * WAVES;
  static constexpr int PIX = CIN * 2;                 // bytes per pixel
  static constexpr int ROWB = (W + 4) * PIX;          // ring row: 2 zero pixels each side
  static constexpr int RING = 8;                      // rows (4 steps)
  static constexpr int LDS = RING * ROWB;
  static constexpr int NW = CIN == 16 ? 13 : K * K;   // resident weight fragments
  static_assert(K == 5 || (CIN == 32 && (K == 3 || K == 5)), "kernel size");
  static constexpr int CPP = CIN / 8;                 // 16-byte groups per pixel
  static constexpr int CHUNKS = W * CPP;              // 16-byte chunks per row
  static constexpr int WPR = CHUNKS / 64;             // waves moving one row (1 KB each)
  static constexpr int DMA_WAVES = 2 * WPR;           // waves moving a step's two rows
  static_assert(WAVES == 8 && CHUNKS % 64 == 0 && DMA_WAVES <= WAVES, "shape");
  // waves per SIMD the register budget is sized for (CIN = 32 holds K^2 fragments)
  static constexpr int WPE = CIN == 16 || K == 3 ? 4 : 2;
};

struct CRArgs {
  const void* x;     // [N][H][W][CIN]
  const void* w;     // forward GEMM weights [COUT][5][5][CIN]
  const float* b;    // [COUT]
  void* out;         // [N][H/2][W/2][COUT]
  int N, H;
  int lgb;           // convT row sweeps: log2 of the row bands per image (0: whole images)
};

// K (CIN = 32 only): the kernel size, 5 (the reference model) or 3 (hyperparam_scan.py's
// k = 3 model): K^2 resident tap fragments, K B fragments per input row, output rows
// r + K/2 - ky; the accumulator ring of 6 rows and the pooling lag are the same.
template <typename T, int CIN, int COUT, int W, int K = 5>
__global__ __launch_bounds__((RC<CIN, COUT, W, K>::THREADS))
__attribute__((amdgpu_waves_per_eu(RC<CIN, COUT, W, K>::WPE)))
void conv_rows_pool_kernel(CRArgs a) {
  using C = RC<CIN, COUT, W, K>;
  extern __shared__ __attribute__((aligned(16))) unsigned char ring[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int m = lane & 15, kg = lane >> 4;
  const int wx = wv % C::NWIN, nb = wv / C::NWIN;
  const int x0 = 16 * wx;
  const int H = a.H, SPI = H / 2 + 1;  // steps per image: rows (2q, 2q + 1), q = 0 .. H/2
  const int G = gridDim.x;
  const int nimg = ((int)a.N - (int)blockIdx.x + G - 1) / G;
  const int S = nimg * SPI + 1;  // + 1: the last pair is stored one step after its rows

  {
    uint4* z = reinterpret_cast<uint4*>(ring);
    for (int e = tid; e < C::LDS / 16; e += C::THREADS) z[e] = uint4{0u, 0u, 0u, 0u};
  }

  // ---- resident weights: A operand, lane (m, kg) = output channel 16 nb + m, K 8 kg .. ----
  uint4 wf[C::NW];
  {
    const T* __restrict__ Wg = reinterpret_cast<const T*>(a.w);
    const int co = 16 * nb + m;
    auto tap = [&](int ky, int kx, int c8) {
      return *reinterpret_cast<const uint4*>(Wg + ((co * K + ky) * K + kx) * CIN + c8);
    };
    if constexpr (CIN == 32) {
#pragma unroll
      for (int t = 0; t < K * K; ++t) wf[t] = tap(t / K, t % K, 8 * kg);
    } else {
      const int hi = kg >> 1, c8 = 8 * (kg & 1);
#pragma unroll
      for (int ky = 0; ky < 5; ++ky) {
        wf[ky] = tap(ky, hi, c8);          // columns (0, 1)
        wf[5 + ky] = tap(ky, 2 + hi, c8);  // columns (2, 3)
      }
      wf[10] = tap(hi, 4, c8);             // F: (w[0][4], w[1][4])
      wf[11] = tap(2 + hi, 4, c8);         //    (w[2][4], w[3][4])
      wf[12] = hi ? uint4{0u, 0u, 0u, 0u} : tap(4, 4, c8);  // (w[4][4], 0)
    }
  }
  const f32x4 bias = f32x4{a.b[16 * nb + 4 * kg], a.b[16 * nb + 4 * kg + 1],
                           a.b[16 * nb + 4 * kg + 2], a.b[16 * nb + 4 * kg + 3]};

  // ---- this lane's B-fragment byte offsets within a ring row ----
  int boff[CIN == 32 ? K : 1];
  int foff = 0, foffw = 0, fo0 = 0;  // CIN = 16: F fragment (next row in the next slot /
                                     // wrapped), and its offset within one row
  if constexpr (CIN == 32) {
#pragma unroll
    for (int kx = 0; kx < K; ++kx) {
      const int ps = x0 + m + kx + 2 - K / 2;  // stored pixel (x + 2)
      boff[kx] = ps * 64 + 16 * (kg ^ ((ps >> 1) & 3));
    }
  } else {
    boff[0] = (x0 + m + (kg >> 1)) * 32 + 16 * (kg & 1);  // columns (0, 1); (2, 3) at + 64
    const int fo = (x0 + m + 4) * 32 + 16 * (kg & 1);
    fo0 = fo;
    foff = fo + (kg >> 1) * C::ROWB;
    foffw = fo - (kg >> 1) * 7 * C::ROWB;  // row r in slot 7: row r + 1 in slot 0
  }

  // ---- row DMA: waves 0 .. DMA_WAVES - 1, wave w moves part w % WPR of row w / WPR ----
  const T* __restrict__ X = reinterpret_cast<const T*>(a.x);
  const bool dma_wave = wv < C::DMA_WAVES;
  int dsrc = 0, ddst = 0;
  if (dma_wave) {
    const int c = (wv % C::WPR) * 64 + lane;  // chunk of the row
    const int ps = 2 + c / C::CPP, gs = c % C::CPP;
    const int g = CIN == 32 ? (gs ^ ((ps >> 1) & 3)) : gs;
    dsrc = (ps - 2) * CIN + 8 * g;  // element offset within the image row
    ddst = 2 * C::PIX + (wv % C::WPR) * 1024;
  }
  // rows of global step s: image (s / SPI) of this workgroup, rows 2q, 2q + 1 (q = s % SPI)
  // rows of global step s = il SPI + q (the caller keeps (il, q) as scalar counters: a
  // run-time division per use cost ~25 SALU and a VALU reciprocal, three per step)
  auto stage_at = [&](int s, int il, int q) -> bool {  // whether this wave issued an LDS-DMA
    if (!dma_wave) return false;
    const int r = 2 * q + wv / C::WPR;
    unsigned char* dst = ring + ((2 * s + wv / C::WPR) & 7) * C::ROWB + ddst;
    if (s < S && il < nimg && r < H) {
      const long long n = (long long)blockIdx.x + (long long)il * G;
      lds_dma16_s(X + ((n * H + r) * W) * CIN, 2u * dsrc, dst);
      return true;
    }
    *reinterpret_cast<uint4*>(dst + 16 * lane) = uint4{0u, 0u, 0u, 0u};
    return false;
  };
  auto stage = [&](int s) { return stage_at(s, s / SPI, s - (s / SPI) * SPI); };  // (prologue)
  __syncthreads();  // ring zeroed
  stage(0);
  stage(1);
  stage(2);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  lds_barrier();

  f32x4 acc[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) acc[i] = bias;
  T* __restrict__ O = reinterpret_cast<T*>(a.out);
  const int PW = W / 2, PHh = H / 2;

  // (image, step in image) of steps s - 2 (pool), s (conv), s + 3 (DMA), advanced per step
  int ilA = -1, qA = SPI - 2, ilC = 0, qC = 0, ilS = 3 / SPI, qS = 3 - (3 / SPI) * SPI;
  auto adv = [&](int& il, int& q) {
    if (++q == SPI) { q = 0; ++il; }
  };
  // step s with I = s % 3 compile-time (the accumulator ring: output row 2q + d -> slot
  // (2 I + d) mod 6)
  auto step = [&](auto ic, const int s) {
    constexpr int I = decltype(ic)::value;
    auto slot = [](int d) { return (2 * I + d + 12) % 6; };
    // (1) pair s - 2 (output rows 2q - 4, 2q - 3) is complete: pool, store, reset
    {
      f32x4& r0 = acc[slot(-4)];
      f32x4& r1 = acc[slot(-3)];
      {
        const int il = ilA, q = qA;  // pair s - 2
        if (il >= 0 && il < nimg && q < PHh) {
          float v[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) v[i] = fmaxf(max_pair(fmaxf(r0[i], r1[i])), 0.f);
          // lanes m, m ^ 1 hold the same pooled values: both store them (no exec-mask branch)
          const long long n = (long long)blockIdx.x + (long long)il * G;
          const long long o = ((n * PHh + q) * PW + (x0 + m) / 2) * COUT + 16 * nb + 4 * kg;
          *reinterpret_cast<uint2*>(O + o) = uint2{pack2<T>(v[0], v[1]), pack2<T>(v[2], v[3])};
        }
      }
      r0 = bias;
      r1 = bias;
    }
    // (2) rows of step s + 3 into the ring
    const bool issued = stage_at(s + 3, ilS, qS);
    // (3) this step's input rows
    const int il = ilC, q = qC;
    if (il < nimg && 2 * q < H) {
      // every B fragment of the step first (one LDS latency per step, not one per row or
      // tap column: sched_barrier keeps the compiler from sinking the reads to their MFMAs)
      constexpr int NB = CIN == 32 ? K : 3;
      uint4 bf[2][NB];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int rs = (2 * s + j) & 7;
        const unsigned char* rb = ring + rs * C::ROWB;
        if constexpr (CIN == 32) {
#pragma unroll
          for (int kx = 0; kx < K; ++kx) bf[j][kx] = *reinterpret_cast<const uint4*>(rb + boff[kx]);
        } else {
          bf[j][0] = *reinterpret_cast<const uint4*>(rb + boff[0]);
          bf[j][1] = *reinterpret_cast<const uint4*>(rb + boff[0] + 64);
          bf[j][2] = *reinterpret_cast<const uint4*>(rb + (rs == 7 ? foffw : foff));
        }
      }
      uint4 bT = uint4{0u, 0u, 0u, 0u};
      if constexpr (CIN == 16) {
        if (q == 0) {
          // F(-1) = (row -1, row 0): output row 1 gets w[1][4] x row 0. Row -1 is zero
          // padding (not read: its ring slot is being refilled by this step's stage)
          bT = *reinterpret_cast<const uint4*>(ring + ((2 * s) & 7) * C::ROWB + fo0);
          if (kg < 2) bT = uint4{0u, 0u, 0u, 0u};
        }
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        if constexpr (CIN == 32) {
#pragma unroll
          for (int kx = 0; kx < K; ++kx)
#pragma unroll
            for (int ky = 0; ky < K; ++ky) {
              f32x4& ac = acc[slot(j + K / 2 - ky)];
              ac = mfma<T>(wf[ky * K + kx], bf[j][kx], ac);
            }
        } else {
          // consecutive MFMAs into different accumulators (no back-to-back dependency)
#pragma unroll
          for (int ky = 0; ky < 5; ++ky) {
            f32x4& ac = acc[slot(j + 2 - ky)];
            ac = mfma<T>(wf[ky], bf[j][0], ac);
          }
#pragma unroll
          for (int ky = 0; ky < 5; ++ky) {
            f32x4& ac = acc[slot(j + 2 - ky)];
            ac = mfma<T>(wf[5 + ky], bf[j][1], ac);
          }
          acc[slot(j + 2)] = mfma<T>(wf[10], bf[j][2], acc[slot(j + 2)]);
          acc[slot(j)] = mfma<T>(wf[11], bf[j][2], acc[slot(j)]);
          acc[slot(j - 2)] = mfma<T>(wf[12], bf[j][2], acc[slot(j - 2)]);
          if (j == 0 && q == 0) acc[slot(1)] = mfma<T>(wf[10], bT, acc[slot(1)]);
        }
      }
    }
    // (4) rows of step s + 2 (DMA issued at step s - 1) have landed; this step's stores are
    // older than its DMA and complete too
    if (issued) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    adv(ilA, qA);
    adv(ilC, qC);
    adv(ilS, qS);
    lds_barrier();
  };
  int s = 0;
  for (; s + 3 <= S; s += 3) {
    step(std::integral_constant<int, 0>{}, s);
    step(std::integral_constant<int, 1>{}, s + 1);
    step(std::integral_constant<int, 2>{}, s + 2);
  }
  if (s < S) step(std::integral_constant<int, 0>{}, s);
  if (s + 1 < S) step(std::integral_constant<int, 1>{}, s + 1);
}

template <typename T, int CIN, int COUT, int W, int K = 5>
hipError_t launch_rows(const CRArgs& a, hipStream_t st) {
  using C = RC<CIN, COUT, W, K>;
  const void* k = reinterpret_cast<const void*>(&conv_rows_pool_kernel<T, CIN, COUT, W, K>);
  static int per_cu[64] = {};
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  if (dev < 0 || dev >= 64) dev = 0;
  if (per_cu[dev] == 0) {
    int pc = 0;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&pc, k, C::THREADS, C::LDS);
    if (e != hipSuccess) return e;
    per_cu[dev] = std::max(1, pc);
  }
  const long long grid = std::min<long long>(a.N, (long long)per_cu[dev] * device_cus());
  SPECENH_LAUNCH((conv_rows_pool_kernel<T, CIN, COUT, W, K>), dim3((unsigned)grid),
                 dim3(C::THREADS), C::LDS, st, a);
  return hipGetLastError();
}

// ============================================================================ convT rows
// Conv2DTranspose(CO, 5, strides=2, relu, same) on 64-channel inputs as a row sweep
// (VAE/manual_scan_3layers.py:196-197: the decoder's 64 -> 64 at 16 x 16 -> 32 x 32 and,
// outside the fused decoder, 64 -> 32 at 32 x 32 -> 64 x 64). conv_patch_kernel runs the
// four output phases as dense convs over 16 x 16 tiles (0.20 of the MFMA peak). Here, as in
// decoder3's producer waves (decoder_tail.hip), input position row s yields output rows
// 2s, 2s + 1: for each of the 9 neighbourhood offsets (dy, dx) one B fragment pair (input
// row s + dy shifted by dx, 16 positions x 64 channels, two K = 32 halves) feeds every
// phase that has the tap — 50 MFMAs from 18 LDS reads per (row, 16 positions, 16 output
// channels). Output phase (py, px) of position (s, x) is pixel (2s + py, 2x + px), its tap
// (ky, kx) = (2 dy + 3 - py, 2 dx + 3 - px) when inside the 5 x 5 kernel (pad 3 of the
// dilated-input conv): 4 / 6 / 6 / 9 taps, exactly the 25 useful ones.
//  * wave (window wx, channel block nb) holds its 50 tap fragments (A operand) in registers
//    for the launch; the four phase accumulators start at the bias.
//  * the input rows are one stream per persistent workgroup: position p = il (H + 1) + 1 + r
//    holds row r of the workgroup's image il, position il (H + 1) the zero row between
//    images, so step g (image g / (H + 1), row s = g % (H + 1), s = H a bubble) reads
//    positions g .. g + 2 and the ring refill is one position per step (LDS-DMA, 3 steps
//    ahead, 8-row ring).
//  * the packed outputs of step g are stored at the start of step g + 1, ahead of that
//    step's DMA, so the end-of-step vmcnt wait (everything but that DMA) never waits on a
//    store younger than the DMA it needs.
// Input pixels are 128 B with their 16-byte groups swizzled, g ^ (p & 7) (decoder3's x1_off:
// conflict-free fragment reads).
template <int CO, int W>
struct TC {
  static constexpr int CI = 64;
  static constexpr int NWIN = W / 16, NNB = CO / 16;
  static constexpr int WAVES = NWIN * NNB;
  static constexpr int THREADS = 64 * WAVES;
  static constexpr int ROWB = (W + 2) * CI * 2;  // one zero position each side
  static constexpr int RING = 8;
  static constexpr int LDS = RING * ROWB;
  static constexpr int DMA_WAVES = W * CI * 2 / 1024;  // one 1-KB DMA per wave and row
  static_assert(WAVES == 4 && DMA_WAVES <= WAVES, "shape");
};

__device__ __forceinline__ constexpr int tky(int py, int dy) { return 2 * dy + 3 - py; }
__device__ __forceinline__ constexpr bool ttap(int ph, int dy, int dx) {
  return tky(ph >> 1, dy) >= 0 && tky(ph >> 1, dy) < 5 && tky(ph & 1, dx) >= 0 &&
         tky(ph & 1, dx) < 5;
}

// bias + ReLU of four fp32 accumulators -> four T in 8 bytes. ReLU commutes with the monotone
// rounding, so it runs on the packed 16-bit pairs: v_pk_max_f16 for fp16; for bf16 each half's
// sign is spread over the half by a packed arithmetic shift and cleared with one bitfield select
// (-0 -> +0 as max(x, 0) gives it). fmaxf on the fp32 accumulators cost 32 VALU per 16 values
// (the max and a NaN-quieting max per element), these 4-6.
template <typename T>
__device__ __forceinline__ uint32_t relu2(uint32_t p) {
  if constexpr (__is_same(T, _Float16)) {
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
    const h2 z = h2{(_Float16)0.f, (_Float16)0.f};
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(h2, p), z));
  } else {
    typedef short s2 __attribute__((ext_vector_type(2)));
    const uint32_t neg = __builtin_bit_cast(uint32_t, __builtin_bit_cast(s2, p) >> (short)15);
    return p & ~neg;
  }
}
template <typename T>
__device__ __forceinline__ uint2 relu_pack4(const f32x4& v) {
  return uint2{relu2<T>(pack2<T>(v[0], v[1])), relu2<T>(pack2<T>(v[2], v[3]))};
}

// LEAD: ring refills in flight beyond the one a step waits for. Step g needs positions
// g + 1 .. g + 3 after its barrier, so it waits for the DMA of position g + 3 only, issued LEAD
// steps earlier; the wave's ledger of its vector-memory ops (LDS-DMAs, and the output stores,
// which vmcnt counts too on gfx9) turns that into the count of younger ops. Round 3 waited
// with vmcnt(1) for everything but the DMA just issued, i.e. for the previous step's DMA and
// this step's own stores.
template <typename T, int CO, int W, int LEAD>
__global__ __launch_bounds__((TC<CO, W>::THREADS)) __attribute__((amdgpu_waves_per_eu(2)))
void convt_rows_kernel(CRArgs a) {
  static_assert(LEAD >= 1 && LEAD <= 4, "8-row ring: positions g .. g + 3 + LEAD live");
  using C = TC<CO, W>;
  extern __shared__ __attribute__((aligned(16))) unsigned char ring[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int m = lane & 15, kg = lane >> 4;
  const int wx = wv % C::NWIN, nb = wv / C::NWIN;
  // the stream's units: whole images (lgb = 0) or row bands of HB rows (small batches)
  const int H = a.H, lgb = a.lgb, HB = H >> lgb, bmask = (1 << lgb) - 1;
  const int SPI = HB + (lgb ? 2 : 1);
  const int G = gridDim.x;
  const int nimg = (((int)a.N << lgb) - (int)blockIdx.x + G - 1) / G;
  const int S = nimg * SPI;

  {
    uint4* z = reinterpret_cast<uint4*>(ring);
    for (int e = tid; e < C::LDS / 16; e += C::THREADS) z[e] = uint4{0u, 0u, 0u, 0u};
  }
  // tap fragments [phase][(dy, dx) taps][K half]
  uint4 wf[50];
  {
    const T* __restrict__ Wg = reinterpret_cast<const T*>(a.w);
    int u = 0;
#pragma unroll
    for (int ph = 0; ph < 4; ++ph)
#pragma unroll
      for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
        for (int dx = -1; dx <= 1; ++dx) {
          if (!ttap(ph, dy, dx)) continue;
#pragma unroll
          for (int kh = 0; kh < 2; ++kh)
            wf[u++] = *reinterpret_cast<const uint4*>(
                Wg + (((16 * nb + m) * 5 + tky(ph >> 1, dy)) * 5 + tky(ph & 1, dx)) * 64 +
                32 * kh + 8 * kg);
        }
  }
  const f32x4 bias = f32x4{a.b[16 * nb + 4 * kg], a.b[16 * nb + 4 * kg + 1],
                           a.b[16 * nb + 4 * kg + 2], a.b[16 * nb + 4 * kg + 3]};
  resident_loads_landed();
  int xo[3];  // byte offset of pixel 16 wx + m + dx (stored + 1), group kg, in a ring row
#pragma unroll
  for (int dx = -1; dx <= 1; ++dx) {
    const int ps = 16 * wx + m + dx + 1;
    xo[dx + 1] = ps * 128 + 16 * (kg ^ (ps & 7));
  }
  // ring refill: wave w < DMA_WAVES moves chunks 64 w .. 64 w + 63 of a row
  const T* __restrict__ X = reinterpret_cast<const T*>(a.x);
  const bool dma_wave = wv < C::DMA_WAVES;
  int dsrc = 0;
  if (dma_wave) {
    const int c = 64 * wv + lane;
    const int ps = 1 + c / 8, gs = c & 7;
    dsrc = (ps - 1) * 64 + 8 * (gs ^ (ps & 7));
  }
  // stream position p = il SPI + q -> ring slot p & 7: row r0 + q - 1 of the workgroup's unit
  // il (unit v = blockIdx.x + il G: image v >> lgb, first row r0 = (v & bmask) HB); rows
  // outside the image are the zero rows (one between whole images, two between bands)
  auto stage_at = [&](int p, int il, int q) -> bool {
    if (!dma_wave) return false;
    unsigned char* dst = ring + (p & 7) * C::ROWB + 128 + 1024 * wv;
    const int v = (int)blockIdx.x + il * G;
    const int r = (v & bmask) * HB + q - 1;
    if (il < nimg && r >= 0 && r < H) {
      const long long n = (long long)(v >> lgb);
      lds_dma16_s(X + ((n * H + r) * W) * 64, 2u * dsrc, dst);
      return true;
    }
    *reinterpret_cast<uint4*>(dst + 16 * lane) = uint4{0u, 0u, 0u, 0u};
    return false;
  };
  auto stage = [&](int p) -> bool {  // (prologue)
    const int il = p / SPI;
    return stage_at(p, il, p - il * SPI);
  };
  __syncthreads();  // ring zeroed
#pragma unroll
  for (int p = 0; p < 3 + LEAD; ++p) stage(p);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  lds_barrier();

  T* __restrict__ O = reinterpret_cast<T*>(a.out);
  const int OW = 2 * W;
  uint2 pk[4];
  long long po = 0;   // element offset of the held outputs' (2s, 2x) pixel
  bool held = false;  // (wave-uniform, as convt_rows_pw_kernel's)
  int vmn = 0;        // this wave's vector-memory ops issued in the loop
  int mk[LEAD + 1];   // vmn right after the DMA of position g + 3 + i (-1: none in flight)
#pragma unroll
  for (int i = 0; i <= LEAD; ++i) mk[i] = -1;
  auto store_held = [&]() {
    if (held) {
#pragma unroll
      for (int ph = 0; ph < 4; ++ph)
        gstore8(O + po + ((ph >> 1) * OW + (ph & 1)) * CO, pk[ph]);
      vmn += 4;
    }
  };
  // scalar counters (image, step in image) of step g and of its refill position g + 3 + LEAD
  int il = 0, s = 0;
  int ilp = (3 + LEAD) / SPI, sp = 3 + LEAD - ilp * SPI;
  for (int g = 0; g < S; ++g) {
    store_held();
    held = false;
    mk[LEAD] = stage_at(g + 3 + LEAD, ilp, sp) ? ++vmn : -1;
    if (s < HB) {
      f32x4 acc[4] = {bias, bias, bias, bias};
      int u0[4] = {0, 8, 20, 32};
#pragma unroll
      for (int dy = -1; dy <= 1; ++dy) {
        const unsigned char* src = ring + ((g + 1 + dy) & 7) * C::ROWB;
#pragma unroll
        for (int dx = -1; dx <= 1; ++dx) {
          // K half 1 (groups kg + 4) sits at the half-0 offset ^ 64 bytes (swizzle bit 2)
          const uint4 b0 = *reinterpret_cast<const uint4*>(src + xo[dx + 1]);
          const uint4 b1 = *reinterpret_cast<const uint4*>(src + (xo[dx + 1] ^ 64));
#pragma unroll
          for (int ph = 0; ph < 4; ++ph)
            if (ttap(ph, dy, dx)) acc[ph] = mfma<T>(wf[u0[ph]], b0, acc[ph]);
#pragma unroll
          for (int ph = 0; ph < 4; ++ph)
            if (ttap(ph, dy, dx)) {
              acc[ph] = mfma<T>(wf[u0[ph] + 1], b1, acc[ph]);
              u0[ph] += 2;
            }
        }
      }
#pragma unroll
      for (int ph = 0; ph < 4; ++ph) pk[ph] = relu_pack4<T>(acc[ph]);
      const int v = (int)blockIdx.x + il * G;
      const long long n = (long long)(v >> lgb);
      po = ((n * 2 * H + 2 * ((v & bmask) * HB + s)) * OW + 2 * (16 * wx + m)) * CO + 16 * nb + 4 * kg;
      held = true;
    }
    if (mk[0] >= 0) wait_vmcnt_ss<15>(vmn - mk[0]);  // position g + 3 has landed
    lds_barrier();
#pragma unroll
    for (int i = 0; i < LEAD; ++i) mk[i] = mk[i + 1];
    if (++s == SPI) { s = 0; ++il; }
    if (++sp == SPI) { sp = 0; ++ilp; }
  }
  store_held();
}

// convt_rows_pw_kernel: convT1 (CO = 64 on 16-position rows), every wave with its OWN input
// ring. The four waves of convt_rows_kernel<T, 64, 16> (one per 16-channel block) all read the
// whole input row, so they shared one ring filled by two of them and met at a workgroup barrier
// every step. Here each wave LDS-DMAs the row (2 x 1 KB) into its own 8-row ring (18 KB; 72 KB
// per workgroup, two workgroups per CU) and waits only for its own refill: no barrier in the
// step loop, the two waves of a SIMD drift freely against each other. The input is read from
// L2 four times instead of once (it is 32 KB per image against 128 KB of output).
template <typename T, int LEAD>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))
void convt_rows_pw_kernel(CRArgs a) {
  static_assert(LEAD >= 1 && LEAD <= 4, "8-row ring: positions g .. g + 3 + LEAD live");
  using C = TC<64, 16>;
  constexpr int CO = 64, W = 16;
  constexpr int WR = C::RING * C::ROWB;  // bytes per wave ring
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_pw[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int m = lane & 15, kg = lane >> 4;
  const int nb = wv;
  unsigned char* const ring = lds_pw + wv * WR;
  // units: whole images or row bands, as convt_rows_kernel's
  const int H = a.H, lgb = a.lgb, HB = H >> lgb, bmask = (1 << lgb) - 1;
  const int SPI = HB + (lgb ? 2 : 1);
  const int G = gridDim.x;
  const int nimg = (((int)a.N << lgb) - (int)blockIdx.x + G - 1) / G;
  const int S = nimg * SPI;

  for (int e = lane; e < WR / 16; e += 64) reinterpret_cast<uint4*>(ring)[e] = uint4{0u, 0u, 0u, 0u};
  // the zero fill's ds_writes and the prologue's LDS-DMA writes into the same ring take
  // different paths with no mutual ordering: the writes complete before any DMA is issued
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  uint4 wf[50];  // tap fragments [phase][(dy, dx) taps][K half]
  {
    const T* __restrict__ Wg = reinterpret_cast<const T*>(a.w);
    int u = 0;
#pragma unroll
    for (int ph = 0; ph < 4; ++ph)
#pragma unroll
      for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
        for (int dx = -1; dx <= 1; ++dx) {
          if (!ttap(ph, dy, dx)) continue;
#pragma unroll
          for (int kh = 0; kh < 2; ++kh)
            wf[u++] = *reinterpret_cast<const uint4*>(
                Wg + (((16 * nb + m) * 5 + tky(ph >> 1, dy)) * 5 + tky(ph & 1, dx)) * 64 +
                32 * kh + 8 * kg);
        }
  }
  const f32x4 bias = f32x4{a.b[16 * nb + 4 * kg], a.b[16 * nb + 4 * kg + 1],
                           a.b[16 * nb + 4 * kg + 2], a.b[16 * nb + 4 * kg + 3]};
  resident_loads_landed();
  int xo[3];  // byte offset of pixel m + dx (stored + 1), group kg, in a ring row
#pragma unroll
  for (int dx = -1; dx <= 1; ++dx) {
    const int ps = m + dx + 1;
    xo[dx + 1] = ps * 128 + 16 * (kg ^ (ps & 7));
  }
  // refill: 16-byte chunks c = lane and 64 + lane of a row (pixel 1 + c / 8, swizzled group)
  const T* __restrict__ X = reinterpret_cast<const T*>(a.x);
  int dsrc[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int c = 64 * h + lane;
    const int ps = 1 + c / 8, gs = c & 7;
    dsrc[h] = (ps - 1) * 64 + 8 * (gs ^ (ps & 7));
  }
  // stream position p = il SPI + q -> ring slot p & 7 (row r0 + q - 1 of unit il, as
  // convt_rows_kernel's); returns the DMAs issued
  auto stage_at = [&](int p, int il, int q) -> int {
    unsigned char* dst = ring + (p & 7) * C::ROWB + 128;
    const int v = (int)blockIdx.x + il * G;
    const int r = (v & bmask) * HB + q - 1;
    if (il < nimg && r >= 0 && r < H) {
      const long long n = (long long)(v >> lgb);
      const T* src = X + ((n * H + r) * W) * 64;
      lds_dma16_s(src, 2u * dsrc[0], dst);
      lds_dma16_s(src, 2u * dsrc[1], dst + 1024);
      return 2;
    }
    *reinterpret_cast<uint4*>(dst + 16 * lane) = uint4{0u, 0u, 0u, 0u};
    *reinterpret_cast<uint4*>(dst + 1024 + 16 * lane) = uint4{0u, 0u, 0u, 0u};
    return 0;
  };
#pragma unroll
  for (int p = 0; p < 3 + LEAD; ++p) {
    const int il = p / SPI;
    stage_at(p, il, p - il * SPI);
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");

  T* __restrict__ O = reinterpret_cast<T*>(a.out);
  constexpr int OW = 2 * W;
  uint2 pk[4];
  long long po = 0;    // element offset of the held outputs' (2s, 2x) pixel
  bool held = false;   // (wave-uniform: a per-lane "po >= 0" test had made the ledger below
                       // per-lane VGPRs, the stores an exec-masked region and the wait a ladder)
  int vmn = 0;         // this wave's vector-memory ops issued in the loop
  int mk[LEAD + 1];    // vmn right after the DMAs of position g + 3 + i (-1: none in flight)
#pragma unroll
  for (int i = 0; i <= LEAD; ++i) mk[i] = -1;
  auto store_held = [&]() {
    if (held) {
#pragma unroll
      for (int ph = 0; ph < 4; ++ph)
        gstore8(O + po + ((ph >> 1) * OW + (ph & 1)) * CO, pk[ph]);
      vmn += 4;
    }
  };
  int il = 0, s = 0;
  int ilp = (3 + LEAD) / SPI, sp = 3 + LEAD - ilp * SPI;
  for (int g = 0; g < S; ++g) {
    store_held();
    held = false;
    const int nd = stage_at(g + 3 + LEAD, ilp, sp);
    vmn += nd;
    mk[LEAD] = nd ? vmn : -1;
    if (s < HB) {
      f32x4 acc[4] = {bias, bias, bias, bias};
      int u0[4] = {0, 8, 20, 32};
#pragma unroll
      for (int dy = -1; dy <= 1; ++dy) {
        const unsigned char* src = ring + ((g + 1 + dy) & 7) * C::ROWB;
#pragma unroll
        for (int dx = -1; dx <= 1; ++dx) {
          const uint4 b0 = *reinterpret_cast<const uint4*>(src + xo[dx + 1]);
          const uint4 b1 = *reinterpret_cast<const uint4*>(src + (xo[dx + 1] ^ 64));
#pragma unroll
          for (int ph = 0; ph < 4; ++ph)
            if (ttap(ph, dy, dx)) acc[ph] = mfma<T>(wf[u0[ph]], b0, acc[ph]);
#pragma unroll
          for (int ph = 0; ph < 4; ++ph)
            if (ttap(ph, dy, dx)) {
              acc[ph] = mfma<T>(wf[u0[ph] + 1], b1, acc[ph]);
              u0[ph] += 2;
            }
        }
      }
#pragma unroll
      for (int ph = 0; ph < 4; ++ph) pk[ph] = relu_pack4<T>(acc[ph]);
      const int v = (int)blockIdx.x + il * G;
      const long long n = (long long)(v >> lgb);
      po = ((n * 2 * H + 2 * ((v & bmask) * HB + s)) * OW + 2 * m) * CO + 16 * nb + 4 * kg;
      held = true;
    }
    // this wave's refill of position g + 3 (both DMAs) has landed; LDS reads are in order
    // within a wave, so the zero-filled rows need no wait. Steady state: 3 steps of 4 stores
    // + 2 DMAs younger than it, i.e. >= 15
    if (mk[0] >= 0) wait_vmcnt_ss<15>(vmn - mk[0]);
    asm volatile("" ::: "memory");
#pragma unroll
    for (int i = 0; i < LEAD; ++i) mk[i] = mk[i + 1];
    if (++s == SPI) { s = 0; ++il; }
    if (++sp == SPI) { sp = 0; ++ilp; }
  }
  store_held();
}

// convt_rows_pg_kernel (variant CONVT_PG; measured SLOWER than convt_rows_pw_kernel, 0.148 vs
// 0.130 ms per 2048 shots, profiles/r05_convt1_pg_ab.txt: kept for the record of the trial):
// convT1 with the four output phases split over two waves per 16-channel
// block (8 waves, one workgroup per CU): wave group A runs phases (0,0) and (1,1) (4 + 9 taps),
// group B phases (0,1) and (1,0) (6 + 6), so a wave holds 26 or 24 tap fragments (~100 VGPRs)
// instead of 50 and has the registers to read all of a step's B fragments (18 / 16) before its
// MFMAs: convt_rows_pw_kernel read them in pairs right before use, exposing an LDS round trip
// per neighbourhood offset (PMC: MFMA busy 0.35). Each wave keeps its own input ring (LDS-DMA,
// no barrier in the step loop), as convt_rows_pw_kernel.
template <typename T, int LEAD>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2)))
void convt_rows_pg_kernel(CRArgs a) {
  static_assert(LEAD >= 1 && LEAD <= 4, "8-row ring: positions g .. g + 3 + LEAD live");
  using C = TC<64, 16>;
  constexpr int CO = 64, W = 16;
  constexpr int WR = C::RING * C::ROWB;  // bytes per wave ring
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_pg[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int m = lane & 15, kg = lane >> 4;
  const int nb = wv & 3;
  unsigned char* const ring = lds_pg + wv * WR;
  const int H = a.H, SPI = H + 1;
  const int G = gridDim.x;
  const int nimg = ((int)a.N - (int)blockIdx.x + G - 1) / G;
  const int S = nimg * SPI;

  for (int e = lane; e < WR / 16; e += 64) reinterpret_cast<uint4*>(ring)[e] = uint4{0u, 0u, 0u, 0u};
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // zero fill before the DMAs (other path)
  const f32x4 bias = f32x4{a.b[16 * nb + 4 * kg], a.b[16 * nb + 4 * kg + 1],
                           a.b[16 * nb + 4 * kg + 2], a.b[16 * nb + 4 * kg + 3]};
  int xo[3];  // byte offset of pixel m + dx (stored + 1), group kg, in a ring row
#pragma unroll
  for (int dx = -1; dx <= 1; ++dx) {
    const int ps = m + dx + 1;
    xo[dx + 1] = ps * 128 + 16 * (kg ^ (ps & 7));
  }
  const T* __restrict__ X = reinterpret_cast<const T*>(a.x);
  int dsrc[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int c = 64 * h + lane;
    const int ps = 1 + c / 8, gs = c & 7;
    dsrc[h] = (ps - 1) * 64 + 8 * (gs ^ (ps & 7));
  }
  auto stage_at = [&](int p, int il, int r) -> int {
    unsigned char* dst = ring + (p & 7) * C::ROWB + 128;
    if (il < nimg && r >= 0) {
      const long long n = (long long)blockIdx.x + (long long)il * G;
      const T* src = X + ((n * H + r) * W) * 64;
      lds_dma16_s(src, 2u * dsrc[0], dst);
      lds_dma16_s(src, 2u * dsrc[1], dst + 1024);
      return 2;
    }
    *reinterpret_cast<uint4*>(dst + 16 * lane) = uint4{0u, 0u, 0u, 0u};
    *reinterpret_cast<uint4*>(dst + 1024 + 16 * lane) = uint4{0u, 0u, 0u, 0u};
    return 0;
  };
  T* __restrict__ O = reinterpret_cast<T*>(a.out);
  constexpr int OW = 2 * W;

  // the wave group's program: phases PA, PB (compile time)
  auto run = [&](auto pa_c, auto pb_c) {
    constexpr int PA = decltype(pa_c)::value, PB = decltype(pb_c)::value;
    constexpr int PHS[2] = {PA, PB};
    // (dy, dx) offsets either phase uses, and the fragments: [phase slot][taps][K half]
    constexpr int NF = 2 * (((PA >> 1) + 2) * ((PA & 1) + 2) + ((PB >> 1) + 2) * ((PB & 1) + 2));
    uint4 wf[NF];
    {
      const T* __restrict__ Wg = reinterpret_cast<const T*>(a.w);
      int u = 0;
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
          for (int dx = -1; dx <= 1; ++dx) {
            const int ph = PHS[q];
            if (!ttap(ph, dy, dx)) continue;
#pragma unroll
            for (int kh = 0; kh < 2; ++kh)
              wf[u++] = *reinterpret_cast<const uint4*>(
                  Wg + (((16 * nb + m) * 5 + tky(ph >> 1, dy)) * 5 + tky(ph & 1, dx)) * 64 +
                  32 * kh + 8 * kg);
          }
    }
    resident_loads_landed();
#pragma unroll
    for (int p = 0; p < 3 + LEAD; ++p) {
      const int il = p / SPI;
      stage_at(p, il, p - il * SPI - 1);
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    uint2 pk[2];
    long long po = 0;   // element offset of the held outputs' (2s, 2x) pixel
    bool held = false;  // (wave-uniform, as convt_rows_pw_kernel's)
    int vmn = 0;        // this wave's vector-memory ops issued in the loop
    int mk[LEAD + 1];   // vmn right after the DMAs of position g + 3 + i (-1: none in flight)
#pragma unroll
    for (int i = 0; i <= LEAD; ++i) mk[i] = -1;
    auto store_held = [&]() {
      if (held) {
#pragma unroll
        for (int q = 0; q < 2; ++q)
          gstore8(O + po + ((PHS[q] >> 1) * OW + (PHS[q] & 1)) * CO, pk[q]);
        vmn += 2;
      }
    };
    int il = 0, s = 0;
    int ilp = (3 + LEAD) / SPI, sp = 3 + LEAD - ilp * SPI;
    for (int g = 0; g < S; ++g) {
      store_held();
      held = false;
      const int nd = stage_at(g + 3 + LEAD, ilp, sp - 1);
      vmn += nd;
      mk[LEAD] = nd ? vmn : -1;
      if (s < H) {
        uint4 bq[9][2];
#pragma unroll
        for (int dy = -1; dy <= 1; ++dy) {
          const unsigned char* src = ring + ((g + 1 + dy) & 7) * C::ROWB;
#pragma unroll
          for (int dx = -1; dx <= 1; ++dx) {
            if (!ttap(PA, dy, dx) && !ttap(PB, dy, dx)) continue;
            bq[3 * (dy + 1) + dx + 1][0] = *reinterpret_cast<const uint4*>(src + xo[dx + 1]);
            bq[3 * (dy + 1) + dx + 1][1] = *reinterpret_cast<const uint4*>(src + (xo[dx + 1] ^ 64));
          }
        }
        __builtin_amdgcn_sched_barrier(0);
        f32x4 acc[2] = {bias, bias};
        int u0[2] = {0, NF / 2 - 0};
        u0[1] = 2 * ((PA >> 1) + 2) * ((PA & 1) + 2);
#pragma unroll
        for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
          for (int dx = -1; dx <= 1; ++dx)
#pragma unroll
            for (int q = 0; q < 2; ++q)
              if (ttap(PHS[q], dy, dx)) {
                acc[q] = mfma<T>(wf[u0[q]], bq[3 * (dy + 1) + dx + 1][0], acc[q]);
                acc[q] = mfma<T>(wf[u0[q] + 1], bq[3 * (dy + 1) + dx + 1][1], acc[q]);
                u0[q] += 2;
              }
#pragma unroll
        for (int q = 0; q < 2; ++q) pk[q] = relu_pack4<T>(acc[q]);
        const long long n = (long long)blockIdx.x + (long long)il * G;
        po = ((n * 2 * H + 2 * s) * OW + 2 * m) * CO + 16 * nb + 4 * kg;
        held = true;
      }
      if (mk[0] >= 0) wait_vmcnt(vmn - mk[0]);
      asm volatile("" ::: "memory");
#pragma unroll
      for (int i = 0; i < LEAD; ++i) mk[i] = mk[i + 1];
      if (++s == SPI) { s = 0; ++il; }
      if (++sp == SPI) { sp = 0; ++ilp; }
    }
    store_held();
  };
  if (wv < 4)
    run(std::integral_constant<int, 0>{}, std::integral_constant<int, 3>{});
  else
    run(std::integral_constant<int, 1>{}, std::integral_constant<int, 2>{});
}

template <typename T>
hipError_t launch_convt_rows_pg(const CRArgs& a, hipStream_t st) {
  using C = TC<64, 16>;
  constexpr int LDS = 8 * C::RING * C::ROWB;
  const void* k = reinterpret_cast<const void*>(&convt_rows_pg_kernel<T, 3>);
  static bool attr[2] = {false, false};
  if (!attr[__is_same(T, __bf16)]) {
    (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    attr[__is_same(T, __bf16)] = true;
  }
  const long long grid = std::min<long long>(a.N, (long long)device_cus());
  SPECENH_LAUNCH((convt_rows_pg_kernel<T, 3>), dim3((unsigned)grid), dim3(512), LDS, st, a);
  return hipGetLastError();
}

// log2 of the row bands per image for the convT row sweeps: whole images while the batch
// fills the resident workgroup slots; a small batch (C4's 128 images: 128 workgroups for 512
// slots) is cut into up to 8 bands of >= 4 rows (two bubble steps and two halo rows each)
int convt_row_bands_lg(int N, int H, long long slots) {
  const int forced = variant(V_ROWS_BANDS);
  int lg = 0;
  while (lg < 3 && (H % (2 << lg)) == 0 && (H >> (lg + 1)) >= 4 &&
         (forced >= 0 ? lg < forced : ((long long)N << (lg + 1)) <= slots))
    ++lg;
  return lg;
}

template <typename T>
hipError_t launch_convt_rows_pw(const CRArgs& a0, hipStream_t st) {
  using C = TC<64, 16>;
  constexpr int LDS = 4 * C::RING * C::ROWB;
  const void* k = reinterpret_cast<const void*>(&convt_rows_pw_kernel<T, 3>);
  static int per_cu[64] = {};
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  if (dev < 0 || dev >= 64) dev = 0;
  if (per_cu[dev] == 0) {
    (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    int pc = 0;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&pc, k, 256, LDS);
    if (e != hipSuccess) return e;
    per_cu[dev] = std::max(1, pc);
  }
  const long long slots = (long long)per_cu[dev] * device_cus();
  CRArgs a = a0;
  a.lgb = convt_row_bands_lg(a.N, a.H, slots);
  const long long grid = std::min<long long>((long long)a.N << a.lgb, slots);
  SPECENH_LAUNCH((convt_rows_pw_kernel<T, 3>), dim3((unsigned)grid), dim3(256), LDS, st, a);
  return hipGetLastError();
}

template <typename T, int CO, int W, int LEAD>
hipError_t launch_convt_rows_lead(const CRArgs& a0, hipStream_t st) {
  using C = TC<CO, W>;
  const void* k = reinterpret_cast<const void*>(&convt_rows_kernel<T, CO, W, LEAD>);
  static int per_cu[64] = {};
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  if (dev < 0 || dev >= 64) dev = 0;
  if (per_cu[dev] == 0) {
    int pc = 0;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&pc, k, C::THREADS, C::LDS);
    if (e != hipSuccess) return e;
    per_cu[dev] = std::max(1, pc);
  }
  const long long slots = (long long)per_cu[dev] * device_cus();
  CRArgs a = a0;
  a.lgb = convt_row_bands_lg(a.N, a.H, slots);
  const long long grid = std::min<long long>((long long)a.N << a.lgb, slots);
  SPECENH_LAUNCH((convt_rows_kernel<T, CO, W, LEAD>), dim3((unsigned)grid), dim3(C::THREADS),
                 C::LDS, st, a);
  return hipGetLastError();
}

template <typename T, int CO, int W>
hipError_t launch_convt_rows(const CRArgs& a, hipStream_t st) {
  return variant(V_ROWS_SHORT_LEAD) ? launch_convt_rows_lead<T, CO, W, 1>(a, st)
                               : launch_convt_rows_lead<T, CO, W, 3>(a, st);
}

// ============================================================================ convT rows, 32 in
// convt_rows32_kernel: Conv2DTranspose(CO, K, strides=2, relu, same) on 32-channel inputs as a
// row sweep, K = 3 / 5 / 7 — the decoders' first Conv2DTranspose of the reference's scan models
// (VAE/hyperparam_scan.py:160 and manual_scan.py:197: 32 -> 32 at 64 x 32 -> 128 x 64 for their
// 256 x 128 inputs), which conv_patch_kernel ran at 0.06-0.19 of the MFMA peak. The schedule of
// convt_rows_kernel with the kernel size generalised: output phase (py, px) of position (s, x)
// reads input row s + dy with tap ky = 2 dy + PT - py (PT = K - 1 - (K - 2) / 2, the dilated
// conv's pad), so each neighbourhood offset's ONE B fragment (32 channels: one K step) feeds
// every phase that has the tap, exactly the K^2 useful taps per (row, 16 positions, 16 output
// channels). Positions: row r of the workgroup's image il at il SPI + r - DY0, SPI = H +
// max(DY1, -DY0) (zero rows between images), so step g reads positions g .. g + NDY - 1.
// Input pixels are 64 B with their 16-byte groups swizzled by (p >> 1) & 3 (conflict-free
// fragment reads at any offset, tools/lds_banks.py).
template <int CO, int W, int K>
struct TC32 {
  static constexpr int CI = 32;
  static constexpr int NWIN = W / 16, NNB = CO / 16;
  static constexpr int WAVES = NWIN * NNB;
  static constexpr int THREADS = 64 * WAVES;
  static constexpr int PT = K - 1 - (K - 2) / 2;
  static constexpr int ky_of(int py, int dy) { return 2 * dy + PT - py; }
  static constexpr bool tap(int ph, int dy, int dx) {
    return ky_of(ph >> 1, dy) >= 0 && ky_of(ph >> 1, dy) < K && ky_of(ph & 1, dx) >= 0 &&
           ky_of(ph & 1, dx) < K;
  }
  static constexpr bool any_tap(int dy, int dx) {
    return tap(0, dy, dx) || tap(1, dy, dx) || tap(2, dy, dx) || tap(3, dy, dx);
  }
  static constexpr int DY0 = -(PT / 2), DY1 = (K - PT) / 2;  // neighbourhood rows (and columns)
  static constexpr int NDY = DY1 - DY0 + 1;
  static constexpr int GAP = DY1 > -DY0 ? DY1 : -DY0;       // zero rows between images
  static constexpr int tap_index(int ph, int dy, int dx) {  // phase-major, (dy, dx) row-major
    int u = 0;
    for (int p = 0; p < 4; ++p)
      for (int a = DY0; a <= DY1; ++a)
        for (int b = DY0; b <= DY1; ++b) {
          if (p == ph && a == dy && b == dx) return u;
          if (tap(p, a, b)) ++u;
        }
    return -1;
  }
  static constexpr int ROWB = (W + NDY - 1) * CI * 2;  // pixels x = DY0 .. W - 1 + DY1
  static constexpr int RING = 8;
  static constexpr int LDS = RING * ROWB;
  static constexpr int DMA_WAVES = W * CI * 2 / 1024;  // one 1-KB DMA per wave and row
  static_assert(WAVES == 4 && DMA_WAVES <= WAVES && (W * CI * 2) % 1024 == 0, "shape");
  static_assert(tap(3, DY0, DY0) || tap(0, DY0, DY0) || any_tap(DY0, 0), "neighbourhood");
};

__device__ __forceinline__ int x32off(int ps, int g) { return ps * 64 + 16 * (g ^ ((ps >> 1) & 3)); }

template <typename T, int CO, int W, int K, int LEAD>
__global__ __launch_bounds__((TC32<CO, W, K>::THREADS)) __attribute__((amdgpu_waves_per_eu(2)))
void convt_rows32_kernel(CRArgs a) {
  using C = TC32<CO, W, K>;
  constexpr int DY0 = C::DY0, DY1 = C::DY1, NDY = C::NDY;
  static_assert(LEAD >= 1 && NDY + LEAD + 1 <= C::RING, "ring: positions g .. g + NDY + LEAD live");
  extern __shared__ __attribute__((aligned(16))) unsigned char ring[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int m = lane & 15, kg = lane >> 4;
  const int wx = wv % C::NWIN, nb = wv / C::NWIN;
  const int H = a.H, SPI = H + C::GAP;
  const int G = gridDim.x;
  const int nimg = ((int)a.N - (int)blockIdx.x + G - 1) / G;
  const int S = nimg * SPI;

  {
    uint4* z = reinterpret_cast<uint4*>(ring);
    for (int e = tid; e < C::LDS / 16; e += C::THREADS) z[e] = uint4{0u, 0u, 0u, 0u};
  }
  uint4 wf[K * K];  // tap fragments, phase-major
  {
    const T* __restrict__ Wg = reinterpret_cast<const T*>(a.w);
#pragma unroll
    for (int ph = 0; ph < 4; ++ph)
#pragma unroll
      for (int dy = DY0; dy <= DY1; ++dy)
#pragma unroll
        for (int dx = DY0; dx <= DY1; ++dx)
          if (C::tap(ph, dy, dx))
            wf[C::tap_index(ph, dy, dx)] = *reinterpret_cast<const uint4*>(
                Wg + (((16 * nb + m) * K + C::ky_of(ph >> 1, dy)) * K + C::ky_of(ph & 1, dx)) * 32 +
                8 * kg);
  }
  const f32x4 bias = f32x4{a.b[16 * nb + 4 * kg], a.b[16 * nb + 4 * kg + 1],
                           a.b[16 * nb + 4 * kg + 2], a.b[16 * nb + 4 * kg + 3]};
  resident_loads_landed();
  int xo[NDY];  // byte offset of pixel 16 wx + m + dx (stored x - DY0), group kg, in a ring row
#pragma unroll
  for (int dx = DY0; dx <= DY1; ++dx) xo[dx - DY0] = x32off(16 * wx + m + dx - DY0, kg);
  // ring refill: wave w < DMA_WAVES moves chunks 64 w .. 64 w + 63 (pixels 16 w .. 16 w + 15)
  const T* __restrict__ X = reinterpret_cast<const T*>(a.x);
  const bool dma_wave = wv < C::DMA_WAVES;
  int dsrc = 0;
  if (dma_wave) {
    const int c = 64 * wv + lane;
    const int x = c / 4, gs = c & 3, ps = x - DY0;
    dsrc = x * 32 + 8 * (gs ^ ((ps >> 1) & 3));
  }
  // stream position p = il SPI + r - DY0 -> ring slot p & 7 (a zero row unless 0 <= r < H)
  auto stage_at = [&](int p, int il, int r) -> bool {
    if (!dma_wave) return false;
    unsigned char* dst = ring + (p & 7) * C::ROWB + (-DY0) * 64 + 1024 * wv;
    if (il < nimg && r >= 0 && r < H) {
      const long long n = (long long)blockIdx.x + (long long)il * G;
      lds_dma16_s(X + ((n * H + r) * W) * 32, 2u * dsrc, dst);
      return true;
    }
    *reinterpret_cast<uint4*>(dst + 16 * lane) = uint4{0u, 0u, 0u, 0u};
    return false;
  };
  auto stage = [&](int p) -> bool {  // (prologue)
    const int il = p / SPI;
    return stage_at(p, il, p - il * SPI + DY0);
  };
  __syncthreads();  // ring zeroed
#pragma unroll
  for (int p = 0; p < NDY + LEAD; ++p) stage(p);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  lds_barrier();

  T* __restrict__ O = reinterpret_cast<T*>(a.out);
  const int OW = 2 * W;
  uint2 pk[4];
  long long po = 0;   // element offset of the held outputs' (2s, 2x) pixel
  bool held = false;  // (wave-uniform, as convt_rows_pw_kernel's)
  int vmn = 0;        // this wave's vector-memory ops issued in the loop
  int mk[LEAD + 1];   // vmn right after the DMA of position g + NDY + i (-1: none in flight)
#pragma unroll
  for (int i = 0; i <= LEAD; ++i) mk[i] = -1;
  auto store_held = [&]() {
    if (held) {
#pragma unroll
      for (int ph = 0; ph < 4; ++ph)
        gstore8(O + po + ((ph >> 1) * OW + (ph & 1)) * CO, pk[ph]);
      vmn += 4;
    }
  };
  // scalar counters (image, step in image) of step g and of its refill position g + NDY + LEAD
  int il = 0, s = 0;
  int ilp = (NDY + LEAD) / SPI, sp = NDY + LEAD - ilp * SPI;
  for (int g = 0; g < S; ++g) {
    store_held();
    held = false;
    mk[LEAD] = stage_at(g + NDY + LEAD, ilp, sp + DY0) ? ++vmn : -1;
    if (s < H) {
      f32x4 acc[4] = {bias, bias, bias, bias};
#pragma unroll
      for (int dy = DY0; dy <= DY1; ++dy) {
        const unsigned char* src = ring + ((g + dy - DY0) & 7) * C::ROWB;
#pragma unroll
        for (int dx = DY0; dx <= DY1; ++dx) {
          if (!C::any_tap(dy, dx)) continue;
          const uint4 b = *reinterpret_cast<const uint4*>(src + xo[dx - DY0]);
#pragma unroll
          for (int ph = 0; ph < 4; ++ph)
            if (C::tap(ph, dy, dx)) acc[ph] = mfma<T>(wf[C::tap_index(ph, dy, dx)], b, acc[ph]);
        }
      }
#pragma unroll
      for (int ph = 0; ph < 4; ++ph) pk[ph] = relu_pack4<T>(acc[ph]);
      const long long n = (long long)blockIdx.x + (long long)il * G;
      po = ((n * 2 * H + 2 * s) * OW + 2 * (16 * wx + m)) * CO + 16 * nb + 4 * kg;
      held = true;
    }
    if (mk[0] >= 0) wait_vmcnt_ss<15>(vmn - mk[0]);  // position g + NDY has landed
    lds_barrier();
#pragma unroll
    for (int i = 0; i < LEAD; ++i) mk[i] = mk[i + 1];
    if (++s == SPI) { s = 0; ++il; }
    if (++sp == SPI) { sp = 0; ++ilp; }
  }
  store_held();
}

template <typename T, int CO, int W, int K>
hipError_t launch_convt_rows32(const CRArgs& a, hipStream_t st) {
  using C = TC32<CO, W, K>;
  constexpr int LEAD = 8 - C::NDY - 1 < 3 ? 8 - C::NDY - 1 : 3;
  const void* k = reinterpret_cast<const void*>(&convt_rows32_kernel<T, CO, W, K, LEAD>);
  static int per_cu[64] = {};
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  if (dev < 0 || dev >= 64) dev = 0;
  if (per_cu[dev] == 0) {
    int pc = 0;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&pc, k, C::THREADS, C::LDS);
    if (e != hipSuccess) return e;
    per_cu[dev] = std::max(1, pc);
  }
  const long long grid = std::min<long long>(a.N, (long long)per_cu[dev] * device_cus());
  SPECENH_LAUNCH((convt_rows32_kernel<T, CO, W, K, LEAD>), dim3((unsigned)grid),
                 dim3(C::THREADS), C::LDS, st, a);
  return hipGetLastError();
}

// ============================================================================ C = 1 rows
// The first Conv2D(16, 5, relu, same) + MaxPooling2D(2) (VAE/manual_scan_3layers.py:187-188)
// on W = 128 one-channel images, as a row sweep. As in conv_c1_mfma.hip the MFMA K index is
// (ky, kx) with kx padded to 8: lane group kg's 8 K-elements are one 8-element run of input
// row y - 2 + kg, so B(r) = rows r .. r + 3 and output row y = A0 x B(y - 2) + A1 x B'(y + 2)
// (A0: kernel rows 0-3, A1: row 4 in lane group 0; B' = B with lane groups 1-3 zeroed).
// Lane m of wave w owns output columns x = 32 w + 2 m + cb (cb = 0, 1): the 2 x 2 pool of
// pooled pixel 16 w + m is in the lane's own four accumulators (rows 2p, 2p + 1 x cb), so a
// step (pooled row p) is 8 MFMAs per wave, no cross-lane exchange, 8-byte stores of whole
// 512-byte pixel runs per wave. conv_c1_mfma tiles 32 x 32 with a halo and re-read the
// input 3.3x (PMC); here every row is read once.
//  * a staged row holds elements x = -8 .. W + 5 (zero outside the image) twice, as 32-bit
//    words as loaded (copy 0) and shifted by one element (copy 1), so every run starts on
//    a word of one copy: a B fragment is 4 word reads (the run of column cb comes from
//    copy cb);
//  * the rows are one stream per workgroup: position il (H + 4) + r + 2 holds row r of the
//    workgroup's image il (two zero rows above and below each image), step g = il (H/2 + 2)
//    + p reads positions 2g .. 2g + 5 (p >= H/2: bubbles); LDS-DMA 5 steps ahead into a
//    16-row ring (waited for two steps later), copy 1 built one step ahead of use.
constexpr int C1W = 128;       // image width
constexpr int C1CW = 72;       // words per copy (elements x = -8 .. W + 5, even count)
constexpr int C1ROW = 2 * C1CW;  // words per staged row (copy 0, copy 1): 144 = 16 (mod 32)
constexpr int C1RING = 16;
constexpr int C1LDS = C1RING * C1ROW * 4;

template <typename T>
__global__ __launch_bounds__(256) void conv1_rows_pool_kernel(CRArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char ring_raw[];
  uint32_t* const ring = reinterpret_cast<uint32_t*>(ring_raw);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int m = lane & 15, kg = lane >> 4;
  const int H = a.H, SPI = H / 2 + 2, PPI = H + 4;
  const int G = gridDim.x;
  const int nimg = ((int)a.N - (int)blockIdx.x + G - 1) / G;
  const int S = nimg * SPI;

  for (int e = tid; e < C1RING * C1ROW; e += 256) ring[e] = 0u;
  // A operand: lane (m, kg) = channel m, K = (kernel row kg, kx 0..7) / (row 4 in group 0)
  uint4 w0, w1;
  {
    const T* __restrict__ Wg = reinterpret_cast<const T*>(a.w);
    uint32_t q0[4], q1[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float v[4];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int kx = 2 * i + h;
        v[2 * h] = kx < 5 ? (float)Wg[(m * 5 + kg) * 5 + kx] : 0.f;
        v[2 * h + 1] = kx < 5 && kg == 0 ? (float)Wg[(m * 5 + 4) * 5 + kx] : 0.f;
      }
      q0[i] = pack2<T>(v[0], v[2]);
      q1[i] = pack2<T>(v[1], v[3]);
    }
    w0 = uint4{q0[0], q0[1], q0[2], q0[3]};
    w1 = uint4{q1[0], q1[1], q1[2], q1[3]};
  }
  const f32x4 bias = f32x4{a.b[4 * kg], a.b[4 * kg + 1], a.b[4 * kg + 2], a.b[4 * kg + 3]};

  // ring refill (wave 0): positions pp, pp + 1 by LDS-DMA, 16 B (8 elements) per lane from
  // lanes 0-15, into copy 0 words 4 .. 67 (x = 0 .. W - 1); returns the DMAs issued
  const T* __restrict__ X = reinterpret_cast<const T*>(a.x);
  auto stage = [&](int pp) -> int {
    if (wv != 0) return 0;
    int nd = 0;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int pos = pp + j;
      const int il = pos / PPI, r = pos - il * PPI - 2;
      uint32_t* dst = ring + (pos & (C1RING - 1)) * C1ROW + 4;  // x = 0 is word 4
      if (il < nimg && r >= 0 && r < H) {
        const long long n = (long long)blockIdx.x + (long long)il * G;
        if (lane < 16) lds_dma16(X + (n * H + r) * C1W + 8 * lane, dst);
        ++nd;
      } else if (lane < 16) {
        *reinterpret_cast<uint4*>(dst + 4 * lane) = uint4{0u, 0u, 0u, 0u};
      }
    }
    return nd;
  };
  // copy 1 of positions pp, pp + 1: word i = elements (2i + 1, 2i + 2) of copy 0
  auto shift = [&](int pp) {
    if (tid < 2 * C1CW) {
      const int j = tid / C1CW, i = tid - j * C1CW;
      uint32_t* row = ring + ((pp + j) & (C1RING - 1)) * C1ROW;
      const uint32_t lo = row[i], hi = row[i + 1];  // i = 71 reads copy 1 word 0: unused
      row[C1CW + i] = __builtin_amdgcn_alignbit(hi, lo, 16);
    }
  };
  __syncthreads();  // ring zeroed
  for (int pp = 0; pp < 10; pp += 2) stage(pp);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  lds_barrier();
  shift(0); shift(2); shift(4);
  lds_barrier();

  // B fragment of position pos (rows pos .. pos + 3 in lane groups 0..3), column block cb:
  // words 16 w + m + 3 .. + 6 of copy cb of row pos + kg
  const int wbase = 16 * wv + m + 3;
  auto bfrag = [&](int pos, int cb) -> uint4 {
    const uint32_t* row = ring + ((pos + kg) & (C1RING - 1)) * C1ROW + cb * C1CW + wbase;
    return uint4{row[0], row[1], row[2], row[3]};
  };
  T* __restrict__ O = reinterpret_cast<T*>(a.out);
  const int PW = C1W / 2, PH = H / 2;
  for (int g = 0; g < S; ++g) {
    // positions 2g + 10, 2g + 11 into the ring (their slots held 2g - 6, 2g - 5: done)
    const int nd = stage(2 * g + 10);
    shift(2 * g + 6);  // copy 1 for step g + 1 (positions landed at the end of step g - 1)
    const int il = g / SPI, p = g - il * SPI;
    if (p < PH) {
      const int pb = 2 * g;  // position of input row 2p - 2
      f32x4 acc[2][2];
#pragma unroll
      for (int dy = 0; dy < 2; ++dy)
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          // output row y = 2p + dy: B(y - 2) at position pb + dy, B'(y + 2) at pb + dy + 4
          const uint4 b = bfrag(pb + dy, cb);
          uint4 b4 = bfrag(pb + dy + 4, cb);
          if (kg != 0) b4 = uint4{0u, 0u, 0u, 0u};
          acc[dy][cb] = mfma<T>(w0, b, bias);
          acc[dy][cb] = mfma<T>(w1, b4, acc[dy][cb]);
        }
      float v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        v[i] = fmaxf(fmaxf(fmaxf(acc[0][0][i], acc[0][1][i]), fmaxf(acc[1][0][i], acc[1][1][i])),
                     0.f);
      const long long n = (long long)blockIdx.x + (long long)il * G;
      *reinterpret_cast<uint2*>(O + ((n * PH + p) * PW + 16 * wv + m) * 16 + 4 * kg) =
          uint2{pack2<T>(v[0], v[1]), pack2<T>(v[2], v[3])};
    }
    // wave 0: the DMAs of step g - 1 (positions 2g + 8, 2g + 9, shifted at step g + 1) must
    // land before the barrier; this step's DMAs and its store are the youngest vector-memory
    // ops, so wait for all but those. The other waves issue only stores: no wait.
    if (wv == 0) {
      const int younger = nd + (p < PH ? 1 : 0);
      if (younger == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      else if (younger == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
      else if (younger == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    }
    lds_barrier();
  }
}

template <typename T>
hipError_t launch_conv1_rows(const CRArgs& a, hipStream_t st) {
  const void* k = reinterpret_cast<const void*>(&conv1_rows_pool_kernel<T>);
  static int per_cu[64] = {};
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  if (dev < 0 || dev >= 64) dev = 0;
  if (per_cu[dev] == 0) {
    int pc = 0;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&pc, k, 256, C1LDS);
    if (e != hipSuccess) return e;
    per_cu[dev] = std::max(1, pc);
  }
  const long long grid = std::min<long long>(a.N, (long long)per_cu[dev] * device_cus());
  SPECENH_LAUNCH(conv1_rows_pool_kernel<T>, dim3((unsigned)grid), dim3(256), C1LDS, st, a);
  return hipGetLastError();
}

// ============================================================================ encoder 1+2
// The encoder's first two layers in one launch (VAE/manual_scan_3layers.py:187-191):
// Conv2D(16, 5, relu) + MaxPooling2D(2) on 128 x 128 one-channel images, then Conv2D(32, 5,
// relu) + MaxPooling2D(2). The 64 x 64 x 16 map between them (128 KB per image, written and
// read once each by the two-launch path) is produced in conv2's LDS ring and never reaches
// HBM. The conv2 part is conv_rows_pool_kernel<T, 16, 32, 64> step for step; instead of an
// LDS-DMA of its input rows, step s computes the two conv2 input rows of step s + 2 with
// the conv1 row sweep (conv1_rows_pool_kernel: waves 0-3 the first row, 4-7 the second,
// 16 pooled pixels each) from a 32-row stream of the images' rows (4 per step: H + 4 =
// 4 (H/4 + 1) positions per image), LDS-DMA 8 steps ahead, copy 1 built 4 steps later.
struct E2Args {
  const void* x;    // [N][H][128] (C = 1)
  const void* w1;   // conv1 GEMM weights [16][5][5]
  const float* b1;  // [16]
  const void* w2;   // conv2 GEMM weights [32][5][5][16]
  const float* b2;  // [32]
  void* out;        // [N][H/4][32][32]
  int N, H;
};

constexpr int E2R1 = 32;  // conv1 input ring rows (positions)
// Staged image rows: SPECENH_ENC2_COPIES element-shifted copies of C1CW words each. With 2
// (copy c = the row shifted by c elements) a lane's 8-element B run starts on a word, so
// it is read as two ds_read2_b32 (16 LDS cycles per fragment); with 4 (c = 0 .. 3) every
// run starts on an even word and is read as two ds_read_b64 (8 cycles with their 2-way
// conflicts: tools-free brute force over copy / row strides found no conflict-free even
// layout). The conv1 B fragments are 8 of each step's 14 LDS reads per wave.
#ifndef SPECENH_ENC2_COPIES
#define SPECENH_ENC2_COPIES 4
#endif
constexpr int E2NC = SPECENH_ENC2_COPIES;
// copy c at word E2CB(c) of a staged row. A half-wave's b64 reads cover copies (cb, cb + 2)
// at words w .. w + 17 of one and w + 2 .. w + 19 of the other, for two ring rows: with
// E2CB(cb) - E2CB(cb + 2) = 14 (mod 64) and a row stride of 32 (mod 64) those are 64
// distinct banks (conflict-free; the plain 72-word stride was 2-way).
__host__ __device__ constexpr int E2CB(int c) {
  return E2NC == 4 ? (c == 0 ? 0 : c == 1 ? 72 : c == 2 ? 178 : 250) : c * C1CW;
}
constexpr int E2ROW = E2NC == 4 ? 352 : 2 * C1CW;  // words per staged row
constexpr int E2RROWS = E2R1 + 2;                  // ring + two zero rows (parities)
#ifndef SPECENH_ENC2_STAGGER
#define SPECENH_ENC2_STAGGER 0
#endif

// WPE: waves per SIMD the register budget is cut for (4: two workgroups per CU, 128 VGPRs;
// 2: one workgroup, 256 VGPRs)
template <typename T, int WPE>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(WPE)))
void enc2_rows_kernel(E2Args a) {
  using C = RC<16, 32, 64>;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  unsigned char* const ring = lds;                                        // conv2 input rows
  uint32_t* const ring1 = reinterpret_cast<uint32_t*>(lds + C::LDS);     // image rows
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int m = lane & 15, kg = lane >> 4;
  const int wx = wv % C::NWIN, nb = wv / C::NWIN;
  const int x0 = 16 * wx;
  const int H1 = a.H, H = H1 / 2;           // conv1 / conv2 input heights
  const int SPI = H / 2 + 1, PPI = H1 + 4;  // conv2 steps and image-row positions per image
  const int G = gridDim.x;
  const int nimg = ((int)a.N - (int)blockIdx.x + G - 1) / G;
  const int S = nimg * SPI + 1;

  for (int e = tid; e < (C::LDS + E2RROWS * E2ROW * 4) / 16; e += 512)
    reinterpret_cast<uint4*>(lds)[e] = uint4{0u, 0u, 0u, 0u};
  // both layers' biases in LDS (read where used: as resident f32x4s they cost the 8 VGPRs
  // that made the 4-waves-per-SIMD build spill)
  float* const btab = reinterpret_cast<float*>(lds + C::LDS + E2RROWS * E2ROW * 4);
  if (tid < 16) btab[tid] = a.b1[tid];
  else if (tid < 48) btab[tid] = a.b2[tid - 16];
  auto bias2_ld = [&]() { return *reinterpret_cast<const f32x4*>(btab + 16 + 16 * nb + 4 * kg); };

  // ---- conv2: resident weight fragments (as conv_rows_pool_kernel, CIN = 16) ----
  uint4 wf[13];
  {
    const T* __restrict__ Wg = reinterpret_cast<const T*>(a.w2);
    const int co = 16 * nb + m, hi = kg >> 1, c8 = 8 * (kg & 1);
    auto tap = [&](int ky, int kx) {
      return *reinterpret_cast<const uint4*>(Wg + ((co * 5 + ky) * 5 + kx) * 16 + c8);
    };
#pragma unroll
    for (int ky = 0; ky < 5; ++ky) {
      wf[ky] = tap(ky, hi);
      wf[5 + ky] = tap(ky, 2 + hi);
    }
    wf[10] = tap(hi, 4);
    wf[11] = tap(2 + hi, 4);
    wf[12] = hi ? uint4{0u, 0u, 0u, 0u} : tap(4, 4);
  }

  const int boff = (x0 + m + (kg >> 1)) * 32 + 16 * (kg & 1);
  const int fo = (x0 + m + 4) * 32 + 16 * (kg & 1);
  const int foff = fo + (kg >> 1) * C::ROWB, foffw = fo - (kg >> 1) * 7 * C::ROWB;

  // ---- conv1: A fragments (kernel rows 0-3 / row 4 in lane group 0) ----
  uint4 v0, v1;
  {
    const T* __restrict__ W1 = reinterpret_cast<const T*>(a.w1);
    uint32_t q0[4], q1[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float v[4];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int kx = 2 * i + h;
        v[2 * h] = kx < 5 ? (float)W1[(m * 5 + kg) * 5 + kx] : 0.f;
        v[2 * h + 1] = kx < 5 && kg == 0 ? (float)W1[(m * 5 + 4) * 5 + kx] : 0.f;
      }
      q0[i] = pack2<T>(v[0], v[2]);
      q1[i] = pack2<T>(v[1], v[3]);
    }
    v0 = uint4{q0[0], q0[1], q0[2], q0[3]};
    v1 = uint4{q1[0], q1[1], q1[2], q1[3]};
  }
  resident_loads_landed();
  const int w1x = wv & 3, jr = wv >> 2;  // conv1 pixel block, conv2 input row of the pair
  const int wbase = 16 * w1x + m + 3;
  // 4 copies: the run of pooled pixel p = 16 w1x + m at column parity cb starts at element
  // 2 p + cb + 6 of copy 0; copy c = that element mod 4 holds it at the even word w4
  const int p1 = 16 * w1x + m;
  const int c4hi = 2 * ((p1 + 3) & 1), w4 = p1 + 3 - ((p1 + 3) & 1);
  const int cbase0 = E2CB(c4hi) + w4, cbase1 = E2CB(1 + c4hi) + w4;  // column parity 0 / 1

  // image-row stream: position pp = il (H1 + 4) + y + 2; waves 0-3 move positions pp + wv.
  // The loop keeps (image, row) of its positions and steps as scalar counters advanced per
  // step (a run-time division per use had cost ~25 SALU + a VALU reciprocal each).
  const T* __restrict__ X = reinterpret_cast<const T*>(a.x);
  auto stage1_at = [&](int pos, int il, int y) -> int {  // position pos = il PPI + y + 2
    uint32_t* dst = ring1 + (pos & (E2R1 - 1)) * E2ROW + 4;
    if (il < nimg && y >= 0 && y < H1) {
      const long long n = (long long)blockIdx.x + (long long)il * G;
      // wave-uniform row base + 16 B per lane (SGPR base, no 64-bit lane address to keep)
      if (lane < 16) lds_dma16_s(X + (n * H1 + y) * C1W, 16u * lane, dst);
      return 1;
    }
    // a zero formed at the store: as a loop-invariant uint4 it was hoisted and spilled
    int z = 0;
    asm volatile("" : "+v"(z));
    if (lane < 16) *reinterpret_cast<uint4*>(dst + 4 * lane) = uint4{(uint32_t)z, (uint32_t)z, (uint32_t)z, (uint32_t)z};
    return 0;
  };
  auto stage1 = [&](int pp) -> int {  // (prologue)
    if (wv >= 4) return 0;
    const int pos = pp + wv;
    const int il = pos / PPI;
    return stage1_at(pos, il, pos - il * PPI - 2);
  };
  auto shift1 = [&](int pp) {  // copies 1 .. E2NC - 1 of positions pp .. pp + 3
    constexpr int NW = E2NC == 4 ? C1CW - 2 : C1CW;  // (copy 0 words read: i .. i + 2)
    if (tid < 4 * NW) {
      const int j = tid / NW, i = tid - j * NW;
      uint32_t* row = ring1 + ((pp + j) & (E2R1 - 1)) * E2ROW;
      const uint32_t r0 = row[i], r1 = row[i + 1];
      row[E2CB(1) + i] = __builtin_amdgcn_alignbit(r1, r0, 16);
      if constexpr (E2NC == 4) {
        const uint32_t r2 = row[i + 2];
        row[E2CB(2) + i] = r1;
        row[E2CB(3) + i] = __builtin_amdgcn_alignbit(r2, r1, 16);
      }
    }
  };
  auto run_at = [&](const uint32_t* row, int cb) -> uint4 {  // row: staged row start
    if constexpr (E2NC == 4) {
      // volatile: two separate ds_read_b64 (2 LDS cycles each); the compiler otherwise pairs
      // reads into ds_read2_b64, which costs 8
      typedef __attribute__((address_space(3))) const volatile unsigned long long lds_u64;
      const lds_u64* r = (const lds_u64*)(row + (cb ? cbase1 : cbase0));
      const unsigned long long lo = r[0], hi = r[1];
      return uint4{(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)};
    } else {
      const uint32_t* r = row + cb * C1CW + wbase;
      return uint4{r[0], r[1], r[2], r[3]};
    }
  };
  auto bfrag = [&](int pos, int cb) -> uint4 {
    return run_at(ring1 + ((pos + kg) & (E2R1 - 1)) * E2ROW, cb);
  };
  // B' (kernel row 4 only): lane group 0 reads row pos, groups 1-3 the zero row past the ring
  // (an address select instead of zeroing 4 data registers)
  // (two zero rows: the one an odd number of rows from pos, so its banks miss lane group 0's)
  auto bfrag4 = [&](int pos, int cb) -> uint4 {
    const uint32_t* zrow = ring1 + (E2NC == 4 ? E2R1 + 1 - (pos & 1) : E2R1) * E2ROW;
    return run_at(kg == 0 ? ring1 + (pos & (E2R1 - 1)) * E2ROW : zrow, cb);
  };
  // conv2 input row 2 q2 + jr of conv2 step g2 (image g2 / SPI) into its ring slot: pooled
  // pixels 16 w1x + m, channels 4 kg .. 4 kg + 3 (zero rows outside the image)
  auto produce = [&](int g2, int il, int q2) {  // g2 = il SPI + q2
    const int r = 2 * q2 + jr;
    // branch-free (the step stays one basic block, so the scheduler can interleave these
    // MFMAs with conv2's): rows past the image are computed from whatever finite rows the
    // ring holds and replaced by zeros
    const int pb = 4 * g2 + 2 * jr;  // position of image row 2r - 2
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    const f32x4 bias1 = *reinterpret_cast<const f32x4*>(btab + 4 * kg);
#pragma unroll
    for (int dy = 0; dy < 2; ++dy)
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        const uint4 b = bfrag(pb + dy, cb);
        const uint4 b4 = bfrag4(pb + dy + 4, cb);
        f32x4 acc1 = mfma<T>(v0, b, bias1);
        acc1 = mfma<T>(v1, b4, acc1);
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = fmaxf(v[i], acc1[i]);  // (>= 0: relu folded)
      }
    const bool real = il < nimg && r < H;
    const uint2 pk = real ? uint2{pack2<T>(v[0], v[1]), pack2<T>(v[2], v[3])} : uint2{0u, 0u};
    *reinterpret_cast<uint2*>(ring + ((2 * g2 + jr) & 7) * C::ROWB + (16 * w1x + m + 2) * 32 +
                              8 * kg) = pk;
  };

  __syncthreads();  // rings zeroed
  for (int pp = 0; pp < 32; pp += 4) stage1(pp);  // positions 0 .. 31 (steps -8 .. -1)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  lds_barrier();
  for (int pp = 0; pp < 16; pp += 4) shift1(pp);
  lds_barrier();
  produce(0, 0, 0);
  produce(1, 1 / SPI, 1 % SPI);
  lds_barrier();

  f32x4 acc[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) acc[i] = bias2_ld();
  T* __restrict__ O = reinterpret_cast<T*>(a.out);
  const int PW = 32, PHh = H / 2;
  int c_1 = 0, c_2 = 0;  // this wave's vector-memory ops (store + LDS-DMA) of steps s - 1, s - 2
  // scalar counters: steps s - 2 (pool), s (conv2), s + 2 (conv1) as (image, step in image),
  // and this wave's stage-1 position 4 s + 32 + wv as (image, row); floor division once here
  auto fdiv = [](int x, int d) { return x >= 0 ? x / d : -((-x + d - 1) / d); };
  int ilA = fdiv(-2, SPI), qA = -2 - ilA * SPI;
  int qC = 0;
  int ilB = 2 / SPI, qB = 2 - ilB * SPI;
  int ilD = (32 + wv) / PPI, rD = 32 + wv - ilD * PPI;  // row y = rD - 2
  auto adv = [](int& il, int& q, int by, int per) {
    q += by;
    if (q >= per) { q -= per; ++il; }
  };

  auto step = [&](auto ic, const int s) {
    constexpr int I = decltype(ic)::value;
    auto slot = [](int d) { return (2 * I + d + 12) % 6; };
    int ns = 0;  // stores issued by this wave in this step
    {  // conv2 pair s - 2: pool, store, reset
      f32x4& r0 = acc[slot(-4)];
      f32x4& r1 = acc[slot(-3)];
      {
        const int il = ilA, q = qA;
        if (il >= 0 && il < nimg && q < PHh) {
          ns = 1;
          float v[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) v[i] = fmaxf(max_pair(fmaxf(r0[i], r1[i])), 0.f);
          // lanes m and m ^ 1 hold the same pooled values (max_pair) and store them to the same
          // pixel: no exec-mask branch around the store
          const long long n = (long long)blockIdx.x + (long long)il * G;
          const long long o = ((n * PHh + q) * PW + (x0 + m) / 2) * 32 + 16 * nb + 4 * kg;
          *reinterpret_cast<uint2*>(O + o) = uint2{pack2<T>(v[0], v[1]), pack2<T>(v[2], v[3])};
        }
      }
      const f32x4 bias = bias2_ld();
      r0 = bias;
      r1 = bias;
    }
    // image rows 8 steps ahead (positions 4s + 32 .. 4s + 35: slots of 4s .. 4s + 3, whose
    // last readers were this step's predecessors), copy 1 of positions 4s + 16 .. 4s + 19
    // (landed: DMA of step s - 4, waited at the end of step s - 1), conv2 input rows of
    // step s + 2 (positions 4s + 8 .. 4s + 15)
    const int nd = wv < 4 ? stage1_at(4 * s + 32 + wv, ilD, rD - 2) : 0;
    shift1(4 * s + 16);
    // this step's conv2 rows, unconditionally: past an image they are the zero rows the
    // conv1 stage stored (adding nothing)
    const int q = qC;
    auto conv2_rows = [&]() {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int rs = (2 * s + j) & 7;
      const unsigned char* rb = ring + rs * C::ROWB;
      const uint4 b0 = *reinterpret_cast<const uint4*>(rb + boff);
      const uint4 b2 = *reinterpret_cast<const uint4*>(rb + boff + 64);
      uint4 bF = *reinterpret_cast<const uint4*>(rb + (rs == 7 ? foffw : foff));
      // the bubble step's F(H + 1) would pair the zero row H + 1 with the NEXT image's row 0
      // (the next ring slot) and add it to that image's output rows 1 / -1 (pair s + 1 is
      // the next image's rows 0, 1): zero it (the next image's F(-1) adds that term)
      if (j == 1 && q == SPI - 1) bF = uint4{0u, 0u, 0u, 0u};
#pragma unroll
      for (int ky = 0; ky < 5; ++ky) {
        f32x4& ac = acc[slot(j + 2 - ky)];
        ac = mfma<T>(wf[ky], b0, ac);
      }
#pragma unroll
      for (int ky = 0; ky < 5; ++ky) {
        f32x4& ac = acc[slot(j + 2 - ky)];
        ac = mfma<T>(wf[5 + ky], b2, ac);
      }
      acc[slot(j + 2)] = mfma<T>(wf[10], bF, acc[slot(j + 2)]);
      acc[slot(j)] = mfma<T>(wf[11], bF, acc[slot(j)]);
      acc[slot(j - 2)] = mfma<T>(wf[12], bF, acc[slot(j - 2)]);
      if (j == 0) {  // F(-1) at the top of an image (q == 0), zero otherwise
        uint4 bT = *reinterpret_cast<const uint4*>(ring + ((2 * s) & 7) * C::ROWB + fo);
        if (kg < 2 || q != 0) bT = uint4{0u, 0u, 0u, 0u};
        acc[slot(1)] = mfma<T>(wf[10], bT, acc[slot(1)]);
      }
    }
    };
    // The two waves of a SIMD (w, w + 4) run the same program and meet at one barrier per
    // step; run in the same order, both would read conv1's LDS-heavy B fragments, then both
    // issue conv2's MFMAs. Waves 4-7 take the two halves in the other order (they are
    // independent: produce writes the ring slots of step s + 2, conv2 reads those of steps s,
    // s + 1), so each SIMD pairs one wave's conv1 with the other's conv2 (MI355X_MICROARCH.md,
    // two waves per SIMD, item 9: a stagger). Measured slower (0.337 vs 0.311 ms per 2048,
    // profiles/r05_enc2_stagger_ab.txt; its VGPR spills rose 5 -> 20), so off by default.
    if (SPECENH_ENC2_STAGGER && wv >= 4) {
      conv2_rows();
      produce(s + 2, ilB, qB);
    } else {
      produce(s + 2, ilB, qB);
      conv2_rows();
    }
    // the DMA of step s - 3 (copy-1 shifted at step s + 1) must have landed: wait for all
    // but this wave's vector-memory ops of steps s - 2 .. s (each step: its store, then its
    // DMA). Only the DMA waves wait; stores alone are never waited for.
    if (wv < 4) {
      const int younger = c_2 + c_1 + ns + nd;
      if (younger >= 6) {  // (steady state: store + DMA in each of the three steps)
        asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      } else switch (younger) {
        case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
        case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
        case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
        case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
        case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
        case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
      }
    }
    c_2 = c_1;
    c_1 = ns + nd;
    adv(ilA, qA, 1, SPI);
    qC = qC + 1 == SPI ? 0 : qC + 1;
    adv(ilB, qB, 1, SPI);
    adv(ilD, rD, 4, PPI);
    lds_barrier();
  };
  int s = 0;
  for (; s + 3 <= S; s += 3) {
    step(std::integral_constant<int, 0>{}, s);
    step(std::integral_constant<int, 1>{}, s + 1);
    step(std::integral_constant<int, 2>{}, s + 2);
  }
  if (s < S) step(std::integral_constant<int, 0>{}, s);
  if (s + 1 < S) step(std::integral_constant<int, 1>{}, s + 1);
}

constexpr int E2LDS = RC<16, 32, 64>::LDS + E2RROWS * E2ROW * 4 + 48 * 4;

template <typename T, int WPE>
hipError_t launch_enc2_wpe(const E2Args& a, hipStream_t st) {
  const void* k = reinterpret_cast<const void*>(&enc2_rows_kernel<T, WPE>);
  static int per_cu[64] = {};
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  if (dev < 0 || dev >= 64) dev = 0;
  if (per_cu[dev] == 0) {
    int pc = 0;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&pc, k, 512, E2LDS);
    if (e != hipSuccess) return e;
    per_cu[dev] = std::max(1, pc);
  }
  const long long grid = std::min<long long>(a.N, (long long)per_cu[dev] * device_cus());
  SPECENH_LAUNCH((enc2_rows_kernel<T, WPE>), dim3((unsigned)grid), dim3(512), E2LDS, st, a);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_enc2(const E2Args& a, hipStream_t st) {
  return variant(V_ENC2_WPE2) ? launch_enc2_wpe<T, 2>(a, st) : launch_enc2_wpe<T, 4>(a, st);
}

}  // namespace

// The row-sweep kernel for an inference Conv2D(5, relu, same) + MaxPooling2D(2) when the
// shape is one it is built for; *launched = false otherwise (the caller runs
// conv_patch_kernel).
int conv_rows_pool(int dtype, const void* x, int N, int H, int W, int CI, const void* w,
                   const float* b, int CO, int K, void* out, hipStream_t st, bool* launched) {
  *launched = false;
  if (variant(V_CONV_NO_ROWS) != 0 || N <= 0 || H < 2 || (H & 1) || !b) return SPECENH_OK;
  if ((long long)N * H * W * CI >= (1ll << 31)) return SPECENH_OK;
  CRArgs a{};
  a.x = x; a.w = w; a.b = b; a.out = out; a.N = N; a.H = H;
  hipError_t e = hipSuccess;
  const bool f16 = dtype == SPECENH_DTYPE_F16;
  if (dtype != SPECENH_DTYPE_F16 && dtype != SPECENH_DTYPE_BF16) return SPECENH_OK;
  if (CI == 16 && CO == 32 && W == 64 && K == 5)
    e = f16 ? launch_rows<_Float16, 16, 32, 64>(a, st) : launch_rows<__bf16, 16, 32, 64>(a, st);
  else if (CI == 32 && CO == 64 && W == 32 && K == 5)
    e = f16 ? launch_rows<_Float16, 32, 64, 32>(a, st) : launch_rows<__bf16, 32, 64, 32>(a, st);
  else if (CI == 32 && CO == 32 && W == 64 && K == 5)  // hyperparam_scan.py, 256 x 128 inputs
    e = f16 ? launch_rows<_Float16, 32, 32, 64>(a, st) : launch_rows<__bf16, 32, 32, 64>(a, st);
  else if (CI == 32 && CO == 32 && W == 64 && K == 3)
    e = f16 ? launch_rows<_Float16, 32, 32, 64, 3>(a, st) : launch_rows<__bf16, 32, 32, 64, 3>(a, st);
  else
    return SPECENH_OK;
  if (e != hipSuccess) return set_error(SPECENH_EHIP, std::string("conv_rows: ") + hipGetErrorString(e));
  *launched = true;
  return SPECENH_OK;
}

}  // namespace specenh

namespace specenh {

// The row-sweep kernel for Conv2DTranspose(CO, 5, s2, relu, same) on 64-channel inputs of
// width 16 (CO 64) or 32 (CO 32), forward (any batch); *launched = false otherwise.
int convt_rows(int dtype, const void* x, int N, int H, int W, int CI, const void* w,
               const float* b, int CO, int K, void* out, hipStream_t st, bool* launched) {
  *launched = false;
  if (variant(V_CONVT_NO_ROWS) != 0 || N <= 0 || H <= 0 || !b) return SPECENH_OK;
  if (dtype != SPECENH_DTYPE_F16 && dtype != SPECENH_DTYPE_BF16) return SPECENH_OK;
  if ((long long)N * 4 * H * W * CO >= (1ll << 31)) return SPECENH_OK;
  CRArgs a{};
  a.x = x; a.w = w; a.b = b; a.out = out; a.N = N; a.H = H;
  const bool f16 = dtype == SPECENH_DTYPE_F16;
  hipError_t e;
  if (CI == 32) {  // the scan models' first Conv2DTranspose (32 -> 32 on 32-position rows)
    if (CO != 32 || W != 32) return SPECENH_OK;
    if (K == 3) e = f16 ? launch_convt_rows32<_Float16, 32, 32, 3>(a, st) : launch_convt_rows32<__bf16, 32, 32, 3>(a, st);
    else if (K == 5) e = f16 ? launch_convt_rows32<_Float16, 32, 32, 5>(a, st) : launch_convt_rows32<__bf16, 32, 32, 5>(a, st);
    else if (K == 7) e = f16 ? launch_convt_rows32<_Float16, 32, 32, 7>(a, st) : launch_convt_rows32<__bf16, 32, 32, 7>(a, st);
    else return SPECENH_OK;
    if (e != hipSuccess) return set_error(SPECENH_EHIP, std::string("convt_rows32: ") + hipGetErrorString(e));
    *launched = true;
    return SPECENH_OK;
  }
  if (CI != 64 || K != 5) return SPECENH_OK;
  if (CO == 64 && W == 16 && variant(V_CONVT_SHARED_RING) == 0 && variant(V_CONVT_PG) != 0)
    e = f16 ? launch_convt_rows_pg<_Float16>(a, st) : launch_convt_rows_pg<__bf16>(a, st);
  else if (CO == 64 && W == 16 && variant(V_CONVT_SHARED_RING) == 0)
    e = f16 ? launch_convt_rows_pw<_Float16>(a, st) : launch_convt_rows_pw<__bf16>(a, st);
  else if (CO == 64 && W == 16)
    e = f16 ? launch_convt_rows<_Float16, 64, 16>(a, st) : launch_convt_rows<__bf16, 64, 16>(a, st);
  else if (CO == 32 && W == 32)
    e = f16 ? launch_convt_rows<_Float16, 32, 32>(a, st) : launch_convt_rows<__bf16, 32, 32>(a, st);
  else
    return SPECENH_OK;
  if (e != hipSuccess) return set_error(SPECENH_EHIP, std::string("convt_rows: ") + hipGetErrorString(e));
  *launched = true;
  return SPECENH_OK;
}

}  // namespace specenh

namespace specenh {

// The C = 1 row sweep for an inference Conv2D(16, 5, relu, same) + MaxPooling2D(2) on
// 128-wide images; *launched = false otherwise (the caller runs conv_c1_mfma).
int conv1_rows_pool(int dtype, const void* x, int N, int H, int W, const void* w,
                    const float* b, int CO, void* out, hipStream_t st, bool* launched) {
  *launched = false;
  if (variant(V_CONV1_NO_ROWS) != 0 || N <= 0 || H < 2 || (H & 1) || W != C1W || CO != 16 || !b)
    return SPECENH_OK;
  if (dtype != SPECENH_DTYPE_F16 && dtype != SPECENH_DTYPE_BF16) return SPECENH_OK;
  if (((uintptr_t)x & 15) || (long long)N * H * W >= (1ll << 31)) return SPECENH_OK;
  CRArgs a{};
  a.x = x; a.w = w; a.b = b; a.out = out; a.N = N; a.H = H;
  const hipError_t e = dtype == SPECENH_DTYPE_F16 ? launch_conv1_rows<_Float16>(a, st)
                                                  : launch_conv1_rows<__bf16>(a, st);
  if (e != hipSuccess) return set_error(SPECENH_EHIP, std::string("conv1_rows: ") + hipGetErrorString(e));
  *launched = true;
  return SPECENH_OK;
}

}  // namespace specenh

// Conv2D(16, 5, relu, same) + MaxPooling2D(2) + Conv2D(32, 5, relu, same) + MaxPooling2D(2)
// on [N][H][128][1] 16-bit images (H a multiple of 4) in one launch (enc2_rows_kernel).
extern "C" int specenh_encoder2(int dtype, const void* x, int N, int H, int W, const void* w1_gemm,
                                const float* b1, int CO1, const void* w2_gemm, const float* b2,
                                int CO2, int k, void* out, void* stream) {
  using namespace specenh;
  if (N < 0 || H <= 0 || W <= 0) return set_error(SPECENH_EINVAL, "bad input shape");
  if (dtype != SPECENH_DTYPE_F16 && dtype != SPECENH_DTYPE_BF16)
    return set_error(SPECENH_EUNSUPPORTED, "fused encoder: fp16 / bf16 only");
  if (W != C1W || CO1 != 16 || CO2 != 32 || k != 5 || (H & 3))
    return set_error(SPECENH_EUNSUPPORTED,
                     "fused encoder: Conv2D(16, 5) + pool + Conv2D(32, 5) + pool on 128-wide "
                     "one-channel images, height a multiple of 4");
  if (N == 0) return SPECENH_OK;
  if (!x || !w1_gemm || !b1 || !w2_gemm || !b2 || !out) return set_error(SPECENH_EINVAL, "null pointer");
  if (((uintptr_t)x & 15) || (long long)N * H * W >= (1ll << 31))
    return set_error(SPECENH_EINVAL, "input must be 16-byte aligned and below 2^31 elements");
  E2Args a{};
  a.x = x; a.w1 = w1_gemm; a.b1 = b1; a.w2 = w2_gemm; a.b2 = b2; a.out = out; a.N = N; a.H = H;
  hipStream_t st = (hipStream_t)stream;
  static std::once_flag once;
  std::call_once(once, [] {
    const void* const ks[4] = {reinterpret_cast<const void*>(&enc2_rows_kernel<_Float16, 4>),
                               reinterpret_cast<const void*>(&enc2_rows_kernel<__bf16, 4>),
                               reinterpret_cast<const void*>(&enc2_rows_kernel<_Float16, 2>),
                               reinterpret_cast<const void*>(&enc2_rows_kernel<__bf16, 2>)};
    for (const void* k : ks)
      (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, E2LDS);
  });
  const hipError_t e = dtype == SPECENH_DTYPE_F16 ? launch_enc2<_Float16>(a, st)
                                                  : launch_enc2<__bf16>(a, st);
  if (e != hipSuccess) return set_error(SPECENH_EHIP, std::string("encoder2: ") + hipGetErrorString(e));
  return SPECENH_OK;
}
