// tail_rows_g.hip — the decoder tail of the reference's OTHER autoencoders as one row-sweep
// launch (gfx950): Conv2DTranspose(CO, KT, strides=2, relu, same) on 64-position-wide
// 32-channel inputs, then Conv2D(1, KO, sigmoid, same) — VAE/hyperparam_scan.py:160-161
// (32 -> 32 at kernel 3 / 5 / 7, 256 x 128 inputs: a 128 x 64 x 32 map into this pair) and
// VAE/manual_scan.py:198-199 (32 -> conv1 = 64 at kernel 5 or 3).
// Run as two launches, the CO-channel map between them (2 MB per 256 x 128 image at CO = 32)
// is written and read once through HBM and the Conv2D(1) ran on the VALU; here it only ever
// exists as LDS rows. (decoder_tail.hip's tail_rows_kernel is the CO = 16, k = 5 case of the
// 3-layer model; this file generalises the channel count and the kernel sizes.)
//
// One workgroup per image walks DOWN it one input-position row q per step:
//  a. Conv2DTranspose: wave (position block w = 16 positions, channel group cg) holds the
//     KT^2 tap fragments of its CPW 16-channel blocks in registers (A operand: 16 output
//     channels x 32 input channels per tap). For each neighbourhood offset (dy, dx) ONE B
//     fragment (input row q + dy shifted by dx: 32 channels x 16 positions) feeds every
//     output phase (py, px) that has the tap (ky, kx) = (2 dy + PT - py, 2 dx + PT - px):
//     exactly the KT^2 useful taps, no work on dilation holes. + bias, ReLU, round to T ->
//     map rows 2q, 2q + 1 of an LDS ring.
//  b. Conv2D(CO -> 1) for the output row pair Y = 2q - 2L, Y + 1 on MFMA:
//       D[x'][(r, kx)] = sum_{p, dr, ci} map[Y - HO + 2p + dr][x'][ci] w[2p + dr - r][kx][ci]
//     (A = map fragments, B = the weights as resident fragments; N = (r, kx), 2 KO of 16
//     columns), over this wave's channels only: a partial per channel group, into an LDS
//     scratch. A wave reads exactly the map columns and channels it wrote itself, so the map
//     needs no barrier.
//  c. input row q + DY1 + 1 (loaded into registers two steps earlier) -> the input ring.
//  d. one barrier, then out[Y + r][x] = bo + sum_{cg, kx} D_cg[x + kx - HO][(r, kx)],
//     sigmoid, fp32 stores of whole 128-column rows.
// Ring slots are compile-time at every access: the step loop is unrolled by a period UU that
// both rings divide (TG::plan).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <mutex>
#include <string>

#include "lds_dma.hpp"
#include "specenh.h"
#include "runtime.hpp"

#ifndef SPECENH_TAILG_PYSPLIT
#define SPECENH_TAILG_PYSPLIT 0
#endif

namespace specenh {
int set_error(int code, const std::string& msg);  // stft_psd.hip

namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
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

template <typename T>
__device__ __forceinline__ uint32_t pack2(float lo, float hi) {
  const T a = (T)lo, b = (T)hi;
  return (uint32_t)__builtin_bit_cast(unsigned short, a) |
         ((uint32_t)__builtin_bit_cast(unsigned short, b) << 16);
}

// bias'd accumulators -> ReLU -> four T in 8 bytes (ReLU commutes with the rounding; fp16
// runs it on the packed halves)
template <typename T>
__device__ __forceinline__ uint2 relu_pack(const f32x4& v) {
  if constexpr (__is_same(T, _Float16)) {
    const f16x2 lo = f16x2{(_Float16)v[0], (_Float16)v[1]};
    const f16x2 hi = f16x2{(_Float16)v[2], (_Float16)v[3]};
    const f16x2 z = f16x2{(_Float16)0.f, (_Float16)0.f};
    return uint2{__builtin_bit_cast(uint32_t, __builtin_elementwise_max(lo, z)),
                 __builtin_bit_cast(uint32_t, __builtin_elementwise_max(hi, z))};
  } else {
    return uint2{pack2<T>(fmaxf(v[0], 0.f), fmaxf(v[1], 0.f)),
                 pack2<T>(fmaxf(v[2], 0.f), fmaxf(v[3], 0.f))};
  }
}

// workgroup barrier ordering LDS only (the register prefetch loads stay in flight)
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

constexpr int gcd_c(int a, int b) { return b ? gcd_c(b, a % b) : a; }
constexpr int lcm_c(int a, int b) { return a / gcd_c(a, b) * b; }
constexpr int pmod(int a, int m) { return ((a % m) + m) % m; }

template <int CO, int KT, int KO>
struct TG {
  static constexpr int CI = 32, QW = 64, MW = 2 * QW;
  static constexpr int PT = KT - 1 - (KT - 2) / 2;  // pad of the dilated-input conv (Keras SAME)
  static constexpr int ky_of(int py, int dy) { return 2 * dy + PT - py; }
  static constexpr bool tap(int ph, int dy, int dx) {
    return ky_of(ph >> 1, dy) >= 0 && ky_of(ph >> 1, dy) < KT && ky_of(ph & 1, dx) >= 0 &&
           ky_of(ph & 1, dx) < KT;
  }
  static constexpr bool any_tap(int dy, int dx) {
    return tap(0, dy, dx) || tap(1, dy, dx) || tap(2, dy, dx) || tap(3, dy, dx);
  }
  static constexpr int dy_min() {
    for (int d = -8; d <= 8; ++d)
      for (int e = -8; e <= 8; ++e)
        if (any_tap(d, e)) return d;
    return 0;
  }
  static constexpr int dy_max() {
    for (int d = 8; d >= -8; --d)
      for (int e = -8; e <= 8; ++e)
        if (any_tap(d, e)) return d;
    return 0;
  }
  static constexpr int DY0 = dy_min(), DY1 = dy_max();  // the same range for dx
  static constexpr int NDY = DY1 - DY0 + 1;
  // register index of phase ph's tap (dy, dx): phase-major, (dy, dx) row-major
  static constexpr int tap_index(int ph, int dy, int dx) {
    int u = 0;
    for (int p = 0; p < 4; ++p)
      for (int a = DY0; a <= DY1; ++a)
        for (int b = DY0; b <= DY1; ++b) {
          if (p == ph && a == dy && b == dx) return u;
          if (tap(p, a, b)) ++u;
        }
    return -1;
  }
  static constexpr int NTAP = KT * KT;
  static constexpr int NCB = CO / 16;                      // 16-channel blocks
  // blocks per wave: all of them while their taps fit ~100 VGPRs, else two channel groups
  // (8 waves; CO = 64 at k = 5: 2 blocks x 25 taps = 200 VGPRs per wave)
  static constexpr int CPW = NTAP * NCB <= 25 ? NCB : NCB / 2;
  static constexpr int NCW = NCB / CPW;                    // channel groups
  static constexpr int NW = 4 * NCW;                       // waves (4 position blocks each)
  static constexpr int THREADS = 64 * NW;
  static constexpr int HO = KO / 2;
  static constexpr int L = (HO + 1) / 2;  // output pair Y = 2q - 2L: map rows Y - HO .. Y + 1 + HO <= 2q + 1
  static constexpr int P = HO + 1;        // map-row pairs of one output pair
  // input staging: LDS-DMA two rows ahead when the tap fragments leave no registers for a
  // prefetch (CO = 64, k = 5: 36 instead of 46 spilled VGPRs; the others ran 4-13 % slower
  // with it, profiles/r06_ae_layers_variants_b.txt), else a register prefetch two rows ahead
  // stored one row ahead
  static constexpr bool DMA = CO == 64 && NTAP * CPW > 40;
  static constexpr int NEED_X = NDY + (DMA ? 2 : 1);  // input rows live in a step
  static constexpr int NEED_M = 2 * L + HO + 2;  // map rows live in a step
  // input pixel stride: dense 64 B with swizzled groups (DMA: lane-linear rows), else 96 B
  // (conflict-free unswizzled reads, the dx shifts then immediates)
  static constexpr int XST = DMA ? CI : 48;
  static constexpr int XROW = (QW + NDY - 1) * XST;
  static constexpr int MROW = MW * CO;
  static constexpr int NSC = 2 * KO;  // scratch rows n = KO r + kx
  static constexpr int SCW = MW + 8;  // scratch row (floats): 4 zero pads each side
  static constexpr int SC_BYTES = NCW * 2 * NSC * SCW * 4;
  // Conv2D(1) weight fragments: in registers unless the tap fragments leave no room
  static constexpr bool WO_LDS = NTAP * CPW * 4 + P * CPW * 4 > 200;
  static constexpr int WO_BYTES = WO_LDS ? NCB * P * 64 * 16 : 0;
  static constexpr int BIAS_BYTES = CO * 4;
  // ring sizes and the unroll period: input ring NXR (| UU), map ring NMR (| 2 UU), within LDS
  struct Plan {
    int nx, nm, u;
  };
  static constexpr Plan plan() {
    Plan best{0, 0, 1 << 30};
    long best_lds = 1L << 40;
    for (int nx = NEED_X; nx <= NEED_X + 4; ++nx)
      for (int nm2 = (NEED_M + 1) / 2; nm2 <= (NEED_M + 1) / 2 + 4; ++nm2) {
        const long lds = (long)nx * XROW * 2 + 2L * nm2 * MROW * 2 + SC_BYTES + WO_BYTES + BIAS_BYTES;
        if (lds > 160L * 1024) continue;
        int u = lcm_c(nx, nm2);
        if (!DMA && u % 2) u *= 2;  // even: the two prefetch register sets alternate with q
        if (u < best.u || (u == best.u && lds < best_lds)) {
          best = Plan{nx, 2 * nm2, u};
          best_lds = lds;
        }
      }
    return best;
  }
  static constexpr int NXR = plan().nx, NMR = plan().nm, UU = plan().u;
  static constexpr int LDS_X = NXR * XROW * 2, LDS_M = NMR * MROW * 2;
  static constexpr int OFF_SC = LDS_X + LDS_M;
  static constexpr int OFF_WO = OFF_SC + SC_BYTES;
  static constexpr int OFF_BIAS = OFF_WO + WO_BYTES;
  static constexpr int LDS_BYTES = OFF_BIAS + BIAS_BYTES;
  static_assert(NXR > 0 && UU <= 12, "no ring plan fits the LDS");
  static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");
  static_assert(CO % 16 == 0 && NCB % CPW == 0, "channel blocks");
  static_assert(2 * KO <= 16, "Conv2D(1) N columns (r, kx)");
  static constexpr int SWM = CO / 8 - 1;
  static constexpr bool PYSPLIT = SPECENH_TAILG_PYSPLIT ? NTAP * CPW * 4 > 150 : DMA;
};

// input ring pixel P (stored x - DY0), 8-channel group g (16 B): g XOR ((P >> 1) & 3), so the
// B-fragment reads (16 consecutive pixels, one group) are conflict-free at any pixel offset
// (tools/lds_banks.py); the rows arrive by LDS-DMA (lane-linear) with the swizzle applied on
// the source side
template <bool DMA>
__device__ __forceinline__ int xoff(int P, int g) {
  return DMA ? P * 32 + 8 * (g ^ ((P >> 1) & 3)) : P * 48 + 8 * g;
}

// map pixel col, 4-channel group g (8 B): g XOR 2 ((col >> 1) & (CO/8 - 1)) keeps the 16-byte
// pairs (2k, 2k + 1) the Conv2D(1) A reads take together and spreads both the epilogue's
// 8-byte writes (16 lanes, columns 2 positions apart) and those reads over the banks
// (tools/lds_banks.py: CO = 32 conflict-free both ways; CO = 64 reads conflict-free, writes
// 2-way)
template <int CO>
__device__ __forceinline__ int moff(int col, int g) {
  return col * CO + 4 * (g ^ (2 * ((col >> 1) & (CO / 8 - 1))));
}

struct TGArgs {
  const void* x;    // [N][H][64][32]
  const void* wt;   // Conv2DTranspose forward GEMM weights [CO][KT][KT][32]
  const float* bt;  // [CO]
  const void* wo;   // Conv2D(1) GEMM weights [KO][KO][CO]
  const float* bo;  // [1]
  float* out;       // [N][2H][128], sigmoid
  int N, H;
};

template <typename T, int CO, int KT, int KO>
__global__ __launch_bounds__((TG<CO, KT, KO>::THREADS)) void tailg_kernel(TGArgs a) {
  using C = TG<CO, KT, KO>;
  constexpr int CPW = C::CPW, NTAP = C::NTAP, P = C::P, DY0 = C::DY0, DY1 = C::DY1;
  constexpr int NXR = C::NXR, NMR = C::NMR, UU = C::UU, CI = C::CI;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  T* const xr = reinterpret_cast<T*>(lds);
  T* const mr = reinterpret_cast<T*>(lds + C::LDS_X);
  float* const sc = reinterpret_cast<float*>(lds + C::OFF_SC);
  uint4* const wol = reinterpret_cast<uint4*>(lds + C::OFF_WO);
  float* const sbias = reinterpret_cast<float*>(lds + C::OFF_BIAS);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int w = wv & 3, cg = wv >> 2;
  const int m = lane & 15, kg = lane >> 4;
  const int n = blockIdx.x;
  const int H = a.H;
  const T* __restrict__ X = reinterpret_cast<const T*>(a.x) + (long long)n * H * C::QW * CI;
  float* __restrict__ O = a.out + (long long)n * (2 * H) * C::MW;

  // ---- resident fragments ----
  uint4 wt[CPW][NTAP];
  {
    const T* __restrict__ Wt = reinterpret_cast<const T*>(a.wt);
#pragma unroll
    for (int cb = 0; cb < CPW; ++cb) {
      const int co = 16 * (cg * CPW + cb) + m;
#pragma unroll
      for (int ph = 0; ph < 4; ++ph)
#pragma unroll
        for (int dy = DY0; dy <= DY1; ++dy)
#pragma unroll
          for (int dx = DY0; dx <= DY1; ++dx)
            if (C::tap(ph, dy, dx))
              wt[cb][C::tap_index(ph, dy, dx)] = *reinterpret_cast<const uint4*>(
                  Wt + ((co * KT + C::ky_of(ph >> 1, dy)) * KT + C::ky_of(ph & 1, dx)) * CI + 8 * kg);
    }
  }
  // Conv2D(1) B fragment of map-row pair p, channel block cbabs: n = m = KO r + kx,
  // k = (dr = kg >> 1, channel 16 cbabs + 8 (kg & 1) + j)
  auto wo_frag = [&](int p, int cbabs) -> uint4 {
    const int r = m / KO, kx = m - (m / KO) * KO, ky = 2 * p + (kg >> 1) - r;
    if (m >= 2 * KO || ky < 0 || ky >= KO) return uint4{0u, 0u, 0u, 0u};
    return *reinterpret_cast<const uint4*>(reinterpret_cast<const T*>(a.wo) +
                                           (ky * KO + kx) * CO + 16 * cbabs + 8 * (kg & 1));
  };
  uint4 wo[C::WO_LDS ? 1 : P][C::WO_LDS ? 1 : CPW];
  if constexpr (!C::WO_LDS) {
#pragma unroll
    for (int p = 0; p < P; ++p)
#pragma unroll
      for (int cb = 0; cb < CPW; ++cb) wo[p][cb] = wo_frag(p, cg * CPW + cb);
  }
  const float bo = a.bo[0];

  // ---- zero every ring (the conv's zero padding, the halo pixels, rows above the image) ----
  for (int e = tid; e < C::LDS_BYTES / 16; e += C::THREADS)
    reinterpret_cast<uint4*>(lds)[e] = uint4{0u, 0u, 0u, 0u};
  __syncthreads();
  if constexpr (C::WO_LDS) {  // [cbabs][p][lane] fragments, written after the zeroing
    for (int f = wv; f < C::NCB * P; f += C::NW) wol[f * 64 + lane] = wo_frag(f % P, f / P);
  }
  for (int c = tid; c < CO; c += C::THREADS) sbias[c] = a.bt[c];
  // the launch-resident loads have landed (otherwise their wait sits inside the step loop and
  // drains the ring's LDS-DMAs every step)
  __builtin_amdgcn_s_waitcnt(0x0F70);

  // input staging, waves 0-3: one row (64 pixels x 64 B) as one 1-KB LDS-DMA per wave (DMA:
  // lane i -> pixel 16 wv + i / 4, stored group i & 3, source group swizzled), or as 16 B per
  // thread from the register prefetch; rows outside the image are zero rows. stage() returns
  // whether this wave issued a DMA (its vector-memory ledger).
  const bool stager = wv < 4;
  const int sx = C::DMA ? 16 * wv + (lane >> 2) : tid >> 2;  // (stager threads: tid < 256)
  const int sP = sx - DY0;
  const int sg = C::DMA ? (lane & 3) ^ ((sP >> 1) & 3) : (tid & 3);
  const int xso = C::DMA ? 0 : xoff<false>(sP, sg);  // register staging: this thread's 16 B
  auto stage = [&](int row, int slot) -> int {
    T* dst = xr + slot * C::XROW + (16 * wv - DY0) * C::XST;  // wave-uniform, 16-B aligned
    if (row >= 0 && row < H) {
      lds_dma16_s(X + (long long)row * C::QW * CI, 2u * (sx * CI + 8 * sg), dst);
      return 1;
    }
    *reinterpret_cast<uint4*>(dst + 8 * lane) = uint4{0u, 0u, 0u, 0u};
    return 0;
  };
  auto gload = [&](int row) -> uint4 {
    const int rr = min(max(row, 0), H - 1);
    uint4 v = *reinterpret_cast<const uint4*>(X + ((long long)rr * C::QW + sx) * CI + 8 * sg);
    if (row < 0 || row >= H) v = uint4{0u, 0u, 0u, 0u};
    return v;
  };
  uint4 pre[C::DMA ? 1 : 2];
  if (stager) {
    if constexpr (C::DMA) {
#pragma unroll
      for (int row = 0; row <= DY1 + 1; ++row) stage(row, pmod(row, NXR));
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
#pragma unroll
      for (int row = 0; row <= DY1; ++row)
        *reinterpret_cast<uint4*>(xr + pmod(row, NXR) * C::XROW + xso) = gload(row);
      pre[0] = gload(DY1 + 1);
      pre[1] = gload(DY1 + 2);
    }
  }
  lds_barrier();

  // this lane's B-fragment offsets (pixel 16 w + m + dx, group kg) in an input ring row
  int xo[C::DMA ? C::NDY : 1];
  if constexpr (C::DMA) {
#pragma unroll
    for (int dx = DY0; dx <= DY1; ++dx) xo[dx - DY0] = xoff<true>(16 * w + m + dx - DY0, kg);
  } else {
    xo[0] = xoff<false>(16 * w + m - DY0, kg);  // + dx * XST: an immediate
  }
  // scratch: D of column block b at [cg][buf][n = m][4 + 16 b + 4 kg]; sums of waves 0-3
  const int ox = 32 * w + (lane & 31), orow = lane >> 5;
  const int NS = H + C::L;  // steps: output pairs Y = 0 .. 2H - 2
  int st_prev = 0;          // this wave's output stores of the previous step (vmcnt ledger)

  auto step = [&](auto ic, const int q) {
    constexpr int I = decltype(ic)::value;
    if (q >= NS) return;  // uniform
    // input row q + DY1 + 2 into its ring slot (needed from step q + 2 on; the slot held row
    // q + DY1 + 2 - NXR < q + DY0: no step still running reads it)
    int nd = 0;
    if constexpr (C::DMA) nd = stager ? stage(q + DY1 + 2, pmod(I + DY1 + 2, NXR)) : 0;
    // ---- a. Conv2DTranspose of input row q -> map rows 2q, 2q + 1 ----
    T* const m0 = mr + pmod(2 * I, NMR) * C::MROW;
    T* const m1 = mr + pmod(2 * I + 1, NMR) * C::MROW;
    if (q < H) {
      // output row phases py = 0, 1 together (one B read per neighbourhood offset feeds all
      // four phases), or one after the other when the taps leave no room for all 4 CPW
      // accumulators (C::PYSPLIT: half the accumulators, the B fragments read twice)
#pragma unroll
      for (int half = 0; half < (C::PYSPLIT ? 2 : 1); ++half) {
        constexpr int NPH = C::PYSPLIT ? 2 : 4;
        const int ph0 = C::PYSPLIT ? 2 * half : 0;
        f32x4 acc[CPW][NPH];
#pragma unroll
        for (int cb = 0; cb < CPW; ++cb)
#pragma unroll
          for (int j = 0; j < NPH; ++j)
            acc[cb][j] = *reinterpret_cast<const f32x4*>(sbias + 16 * (cg * CPW + cb) + 4 * kg);
#pragma unroll
        for (int dy = DY0; dy <= DY1; ++dy) {
          const T* src = xr + pmod(I + dy, NXR) * C::XROW;
#pragma unroll
          for (int dx = DY0; dx <= DY1; ++dx) {
            bool any = false;
#pragma unroll
            for (int j = 0; j < NPH; ++j) any = any || C::tap(ph0 + j, dy, dx);
            if (!any) continue;
            const uint4 b = *reinterpret_cast<const uint4*>(
                src + (C::DMA ? xo[C::DMA ? dx - DY0 : 0] : xo[0] + dx * C::XST));
#pragma unroll
            for (int j = 0; j < NPH; ++j) {
              if (!C::tap(ph0 + j, dy, dx)) continue;
#pragma unroll
              for (int cb = 0; cb < CPW; ++cb)
                acc[cb][j] = mfma<T>(wt[cb][C::tap_index(ph0 + j, dy, dx)], b, acc[cb][j]);
            }
          }
        }
#pragma unroll
        for (int cb = 0; cb < CPW; ++cb)
#pragma unroll
          for (int j = 0; j < NPH; ++j) {
            const int ph = ph0 + j;
            const int col = 2 * (16 * w + m) + (ph & 1);
            *reinterpret_cast<uint2*>(((ph >> 1) ? m1 : m0) +
                                      moff<CO>(col, 4 * (cg * CPW + cb) + kg)) = relu_pack<T>(acc[cb][j]);
          }
      }
    } else {  // below the image: the Conv2D(1) zero padding
#pragma unroll
      for (int cb = 0; cb < CPW; ++cb)
#pragma unroll
        for (int ph = 0; ph < 4; ++ph) {
          const int col = 2 * (16 * w + m) + (ph & 1);
          *reinterpret_cast<uint2*>(((ph >> 1) ? m1 : m0) + moff<CO>(col, 4 * (cg * CPW + cb) + kg)) =
              uint2{0u, 0u};
        }
    }
    // ---- b. Conv2D(1) partial D (this wave's channels) of output pair Y = 2q - 2L ----
    const int Y = 2 * q - 2 * C::L;
    const bool emit = Y >= 0;  // uniform
    float* const scb = sc + ((cg * 2 + (I & 1)) * C::NSC) * C::SCW;
    if (emit) {
#pragma unroll
      for (int blk = 0; blk < 2; ++blk) {
        const int col = 32 * w + 16 * blk + m;
        f32x4 d = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int p = 0; p < P; ++p) {
          // map row Y - HO + 2p + dr (dr = kg >> 1): compile-time slots, a lane select
          const int s0 = pmod(2 * I - 2 * C::L - C::HO + 2 * p, NMR);
          const int s1 = s0 + 1 == NMR ? 0 : s0 + 1;
          const T* mrow = mr + ((kg >> 1) ? s1 : s0) * C::MROW;
#pragma unroll
          for (int cb = 0; cb < CPW; ++cb) {
            const int cbabs = cg * CPW + cb;
            const uint4 av = *reinterpret_cast<const uint4*>(mrow + moff<CO>(col, 4 * cbabs + 2 * (kg & 1)));
            uint4 bw;
            if constexpr (C::WO_LDS) bw = wol[(cbabs * P + p) * 64 + lane];
            else bw = wo[p][cb];
            d = mfma<T>(av, bw, d);
          }
        }
        if (m < C::NSC)  // D[x' = 32 w + 16 blk + 4 kg + i][n = m]
          *reinterpret_cast<f32x4*>(scb + m * C::SCW + 4 + 32 * w + 16 * blk + 4 * kg) = d;
      }
    }
    // ---- c. the DMA of step q - 1 (row q + DY1 + 1, read from step q + 1 on) has landed: wait
    // for all but this wave's younger vector-memory ops (the previous step's store, this step's
    // DMA) ----
    if constexpr (C::DMA) {
      if (stager) wait_vmcnt(st_prev + nd);
    } else if (stager) {  // input row q + DY1 + 1 (loaded two steps ago) into its ring slot
      *reinterpret_cast<uint4*>(xr + pmod(I + DY1 + 1, NXR) * C::XROW + xso) = pre[I & 1];
    }
    lds_barrier();
    // ---- d. diagonal sums over the channel groups' partials, sigmoid, stores ----
    if (emit && wv < 4) {
      float s = bo;
#pragma unroll
      for (int g = 0; g < C::NCW; ++g) {
        const float* sp = sc + ((g * 2 + (I & 1)) * C::NSC + orow * KO) * C::SCW + 4 + ox - C::HO;
#pragma unroll
        for (int kx = 0; kx < KO; ++kx) s += sp[kx * C::SCW + kx];
      }
      O[(long long)(Y + orow) * C::MW + ox] = __builtin_amdgcn_rcpf(1.f + __expf(-s));
    }
    if constexpr (C::DMA) st_prev = emit && wv < 4 ? 1 : 0;
    else if (stager) pre[I & 1] = gload(q + DY1 + 3);
  };

  for (int q0 = 0; q0 < NS; q0 += UU) {
    step(std::integral_constant<int, 0>{}, q0);
    if constexpr (UU > 1) step(std::integral_constant<int, 1>{}, q0 + 1);
    if constexpr (UU > 2) step(std::integral_constant<int, 2>{}, q0 + 2);
    if constexpr (UU > 3) step(std::integral_constant<int, 3>{}, q0 + 3);
    if constexpr (UU > 4) step(std::integral_constant<int, 4>{}, q0 + 4);
    if constexpr (UU > 5) step(std::integral_constant<int, 5>{}, q0 + 5);
    if constexpr (UU > 6) step(std::integral_constant<int, 6>{}, q0 + 6);
    if constexpr (UU > 7) step(std::integral_constant<int, 7>{}, q0 + 7);
    if constexpr (UU > 8) step(std::integral_constant<int, 8>{}, q0 + 8);
    if constexpr (UU > 9) step(std::integral_constant<int, 9>{}, q0 + 9);
    if constexpr (UU > 10) step(std::integral_constant<int, 10>{}, q0 + 10);
    if constexpr (UU > 11) step(std::integral_constant<int, 11>{}, q0 + 11);
  }
}

template <typename T, int CO, int KT, int KO>
hipError_t launch_tailg(const TGArgs& a, hipStream_t st) {
  using C = TG<CO, KT, KO>;
  static std::once_flag once;
  static hipError_t attr = hipSuccess;
  std::call_once(once, [] {
    attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&tailg_kernel<T, CO, KT, KO>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS_BYTES);
  });
  if (attr != hipSuccess) return attr;
  SPECENH_LAUNCH((tailg_kernel<T, CO, KT, KO>), dim3((unsigned)a.N), dim3(C::THREADS),
                 C::LDS_BYTES, st, a);
  return hipGetLastError();
}

template <typename T>
hipError_t dispatch(const TGArgs& a, int CO, int kt, int ko, hipStream_t st, bool* launched) {
  *launched = true;
  if (CO == 32 && kt == 3 && ko == 3) return launch_tailg<T, 32, 3, 3>(a, st);
  if (CO == 32 && kt == 5 && ko == 5) return launch_tailg<T, 32, 5, 5>(a, st);
  if (CO == 32 && kt == 7 && ko == 7) return launch_tailg<T, 32, 7, 7>(a, st);
  if (CO == 64 && kt == 3 && ko == 3) return launch_tailg<T, 64, 3, 3>(a, st);
  if (CO == 64 && kt == 5 && ko == 5) return launch_tailg<T, 64, 5, 5>(a, st);
  *launched = false;
  return hipSuccess;
}

}  // namespace

// The general row-sweep tail for (C, CO, kt, ko) other than the 3-layer model's (32, 16, 5, 5)
// at 64-position-wide inputs (inference, fp32 sigmoid output); *launched = false when the
// configuration is not built here.
bool tail_rows_general_supported(int C, int CO, int kt, int ko, int W) {
  if (C != 32 || W != 64 || kt != ko) return false;
  return (CO == 32 && (kt == 3 || kt == 5 || kt == 7)) || (CO == 64 && (kt == 3 || kt == 5));
}

int tail_rows_general(int dtype, const void* x, int N, int H, int W, int C, const void* wt,
                      const float* bt, int CO, int kt, const void* wo, const float* bo, int ko,
                      float* out, hipStream_t st, bool* launched) {
  *launched = false;
  if (!tail_rows_general_supported(C, CO, kt, ko, W)) return SPECENH_OK;
  if (dtype != SPECENH_DTYPE_F16 && dtype != SPECENH_DTYPE_BF16) return SPECENH_OK;
  if (N <= 0 || H <= 0) return SPECENH_OK;
  if ((long long)N * H * W * C >= (1ll << 31) || (long long)N * 4 * H * W >= (1ll << 31))
    return set_error(SPECENH_EINVAL, "tensor too large (2^31 elements)");
  if (!x || !wt || !bt || !wo || !bo || !out) return set_error(SPECENH_EINVAL, "null pointer");
  TGArgs a{x, wt, bt, wo, bo, out, N, H};
  const hipError_t e = dtype == SPECENH_DTYPE_F16 ? dispatch<_Float16>(a, CO, kt, ko, st, launched)
                                                  : dispatch<__bf16>(a, CO, kt, ko, st, launched);
  if (e != hipSuccess)
    return set_error(SPECENH_EHIP, std::string("tail_rows_general: ") + hipGetErrorString(e));
  return SPECENH_OK;
}

}  // namespace specenh
