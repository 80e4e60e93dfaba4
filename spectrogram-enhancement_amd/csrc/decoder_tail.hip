// decoder_tail.hip — the autoencoder's last two layers fused, for inference (gfx950).
//
// VAE/manual_scan_3layers.py:197-199 ends the model with
//   Conv2DTranspose(16, 5, strides=2, activation="relu", padding="same")   32 -> 16 channels
//   Conv2D(1, 5, activation="sigmoid", padding="same")                     16 -> 1
// Run as two launches (conv_ae.hip + conv_narrow.hip), the 16-channel map between them —
// 128 x 128 x 16 fp16 per image, 2.15 GB per 4,096 shots written once and read once — is
// the largest tensor of the C5 stream. Here one workgroup produces a 32 x 32 tile of the
// final output and that map never leaves the CU:
//
//  1. Conv2DTranspose as ONE implicit GEMM over input positions. Output pixel
//     (2q + py, 2r + px) of a stride-2 "same" transposed conv reads input rows q + dy with
//     ky = 2 dy + p - py (p = k - 1 - (k - 2) / 2, the dilated conv's pad; 0 <= ky < k), so
//     a position (q, r) and its 3 x 3 input neighbourhood yield the whole 2 x 2 output block:
//     four phases, each a 16-channel MFMA N-block over its own taps (4 / 6 / 6 / 9 of the
//     9 neighbourhood taps for k = 5: exactly the 25 useful taps, no work on dilation holes).
//     The tile needs 18 x 18 positions (a one-position halo for the 5 x 5 conv that follows)
//     = 21 M-blocks of 16, from a 20 x 20 x 32 input patch staged in LDS (zero outside the
//     image). v_mfma_f32_16x16x32_{f16,bf16}: weights as the A operand (16 output channels
//     x 32 input channels of one tap), the patch as B (32 channels x 16 positions), fp32
//     accumulation. Each wave owns one phase and half of its M-blocks (convt_conv_out_kernel
//     balances the phases over the SIMDs); its tap weights sit in registers, loaded while
//     the patch is staged.
//  2. Epilogue: + bias, ReLU, round to T (exactly what the unfused layer stores), into a
//     36 x 36 x 16 LDS image of the map (48-byte pixels: conflict-free reads below) that
//     aliases the dead input patch; pixels outside the image are the conv's zero padding.
//  3. Conv2D 16 -> 1, 5 x 5, on MFMA: per output row y, D[x'][kx] = sum_{ky,ci}
//     map[y + ky][x'][ci] w[ky][kx][ci] (A = map rows from LDS, B = the weights as fragments
//     held in registers), then out[y][x] = sum_kx D[x + kx][kx] through a per-wave scratch;
//     + bias, sigmoid, fp32 store (coalesced 128-byte row segments).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <mutex>
#include <cstdlib>
#include <cstdint>
#include <string>
#include <type_traits>
#include <vector>

#include "lds_dma.hpp"
#include "specenh.h"
#include "runtime.hpp"

namespace specenh {
int set_error(int code, const std::string& msg);  // stft_psd.hip

namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int TO = 32;                 // final output pixels per tile side
constexpr int NP = TO / 2 + 2;         // 18 input positions per side (one-position halo)
constexpr int NPOS = NP * NP;          // 324
constexpr int NBLK = (NPOS + 15) / 16;  // 21 M-blocks
constexpr int XW = NP + 2;             // 20: input patch side (3 x 3 neighbourhood)
constexpr int CI = 32, CO = 16, KT = 5, KO = 5;
constexpr int XPST = 48;               // patch pixel stride (elements): 32 channels + pad
constexpr int YW = 2 * NP;             // 36: map region side
constexpr int PT = KT - 1 - (KT - 2) / 2;  // 3: pad of the dilated-input conv
constexpr int PXW = 48;                // Conv2D(1) scratch: positions x' per row (3 blocks)

struct TailArgs {
  const void* x;      // [N][H][W][CI]
  const void* wt;     // convT forward GEMM weights [CO][KT][KT][CI]
  const float* bt;    // [CO]
  const void* wo;     // conv_out GEMM weights [1][KO][KO][CO]
  const float* bo;    // [1]
  float* out;         // [N][2H][2W]
  int N, H, W, tiles_y, tiles_x;
};

// tap row ky of neighbourhood offset dy for output row phase py (-1 <= dy <= 1; valid when
// 0 <= ky < KT)
__host__ __device__ constexpr int ky_of(int py, int dy) { return 2 * dy + PT - py; }

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
__device__ __forceinline__ float dot2(uint32_t a, uint32_t b, float c) {
  if constexpr (__is_same(T, _Float16)) {
    return __builtin_amdgcn_fdot2(__builtin_bit_cast(f16x2, a), __builtin_bit_cast(f16x2, b), c,
                                  false);
  } else {  // v_dot2c_f32_bf16 (gfx950)
    return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, a),
                                           __builtin_bit_cast(bf16x2, b), c, false);
  }
}

template <typename T>
__device__ __forceinline__ uint32_t pack2(float lo, float hi) {
  const T a = (T)lo, b = (T)hi;
  return (uint32_t)__builtin_bit_cast(unsigned short, a) |
         ((uint32_t)__builtin_bit_cast(unsigned short, b) << 16);
}

__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Phase PH = py * 2 + px: its taps in (dy, dx) order, compile-time (static register indices).
template <int PH>
struct Taps {
  static constexpr bool ok(int dy, int dx) {
    return ky_of(PH >> 1, dy) >= 0 && ky_of(PH >> 1, dy) < KT && ky_of(PH & 1, dx) >= 0 &&
           ky_of(PH & 1, dx) < KT;
  }
};

template <typename T, int PH>
__device__ __forceinline__ void load_taps(uint4 (&wr)[9], const T* __restrict__ Wt, int m,
                                          int kg) {
  int u = 0;
#pragma unroll
  for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
    for (int dx = -1; dx <= 1; ++dx)
      if (Taps<PH>::ok(dy, dx)) {
        wr[u] = *reinterpret_cast<const uint4*>(
            Wt + ((m * KT + ky_of(PH >> 1, dy)) * KT + ky_of(PH & 1, dx)) * CI + 8 * kg);
        ++u;
      }
}

template <typename T, int PH>
__device__ __forceinline__ f32x4 item_mfma(const uint4 (&wr)[9], const T* sp, f32x4 acc) {
  int u = 0;
#pragma unroll
  for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
    for (int dx = -1; dx <= 1; ++dx)
      if (Taps<PH>::ok(dy, dx)) {
        const uint4 b = *reinterpret_cast<const uint4*>(sp + (dy * XW + dx) * XPST);
        acc = mfma<T>(wr[u], b, acc);
        ++u;
      }
  return acc;
}

constexpr int MAXBLK = (NBLK + 1) / 2;  // 11: M-blocks per wave (two waves per phase)
constexpr int XV = XW * XW * (CI / 8);   // 16-byte vectors of one input patch
constexpr int XPF = (XV + 511) / 512;    // of them per thread

// map pixel p's 8-channel half h lives at half h ^ bit 3 of p: conflict-free reads in the
// Conv2D(1) phase with 32-byte pixels (bank search over the ds_read_b128 lane groups)
__device__ __forceinline__ int ymap(int pix, int h) { return pix * CO + 8 * (h ^ ((pix >> 3) & 1)); }

struct TileGeo {
  int n, oy0, ox0;
};
__device__ __forceinline__ TileGeo tile_geo(const TailArgs& a, int tile) {
  const int tiles = a.tiles_y * a.tiles_x;
  TileGeo g;
  g.n = tile / tiles;
  const int t = tile - g.n * tiles;
  const int ty = t / a.tiles_x;
  g.oy0 = ty * TO;
  g.ox0 = (t - ty * a.tiles_x) * TO;
  return g;
}

// this thread's part of tile's input patch (zero outside the image) -> registers
template <typename T>
__device__ __forceinline__ void load_patch(const TailArgs& a, int tile, uint4 (&v)[XPF]) {
  const TileGeo g = tile_geo(a, tile);
  const int xa = g.oy0 / 2 - 2, xb = g.ox0 / 2 - 2;  // first input pixel of the patch
  const T* __restrict__ X = reinterpret_cast<const T*>(a.x) + (long long)g.n * a.H * a.W * CI;
#pragma unroll
  for (int u = 0; u < XPF; ++u) {
    const int e = threadIdx.x + 512 * u;
    const int pix = e >> 2, cg = e & 3;
    const int py = pix / XW, pxx = pix - py * XW;
    const int iy = xa + py, ix = xb + pxx;
    v[u] = uint4{0u, 0u, 0u, 0u};
    if (e < XV && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W)
      v[u] = *reinterpret_cast<const uint4*>(X + ((long long)iy * a.W + ix) * CI + 8 * cg);
  }
}

template <typename T>
__device__ __forceinline__ void store_patch(T* sx, const uint4 (&v)[XPF]) {
#pragma unroll
  for (int u = 0; u < XPF; ++u) {
    const int e = threadIdx.x + 512 * u;
    if (e < XV) *reinterpret_cast<uint4*>(sx + (e >> 2) * XPST + 8 * (e & 3)) = v[u];
  }
}

// A persistent workgroup's program for a wave whose phase is PH (compile-time: its taps and
// weight registers are static), over tiles blockIdx.x, + gridDim.x, ...: the next tile's
// input patch is loaded into registers during this tile's Conv2D(1) (the patch and the map
// have LDS regions of their own) and written to LDS behind it.
template <typename T, int PH>
__device__ __forceinline__ void tail_body(const TailArgs& a, T* sx, T* sy, int wave, int half) {
  const int lane = threadIdx.x & 63;
  const int kg = lane >> 4, m = lane & 15;
  const int total = a.N * a.tiles_y * a.tiles_x;
  const int H2 = 2 * a.H, W2 = 2 * a.W;
  const int G = gridDim.x;

  uint4 wr[9];  // this phase's tap weights (A fragments)
  load_taps<T, PH>(wr, reinterpret_cast<const T*>(a.wt), m, kg);
  float bias[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) bias[r] = a.bt[4 * kg + r];
  const float bo = a.bo[0];
  // Conv2D(1) weights as MFMA B fragments: k = (kernel row 2 s + (kg >> 1), 8 channels
  // 8 (kg & 1) ..), n = kx = m (zero for kx >= KO or row >= KO)
  uint4 wo_frag[3];
#pragma unroll
  for (int s2 = 0; s2 < 3; ++s2) {
    const int ky = 2 * s2 + (kg >> 1);
    wo_frag[s2] = uint4{0u, 0u, 0u, 0u};
    if (ky < KO && m < KO)
      wo_frag[s2] = *reinterpret_cast<const uint4*>(reinterpret_cast<const T*>(a.wo) +
                                                    (ky * KO + m) * CO + 8 * (kg & 1));
  }
  // the weights and biases are in registers before the tile loop starts: otherwise the
  // compiler's wait for them sits inside the loop, and on CDNA4 vmcnt also counts the
  // previous tile's output stores, so every tile would wait for its predecessor's writes
  __builtin_amdgcn_s_waitcnt(0x0F70);  // s_waitcnt vmcnt(0)
  const int b0 = half * MAXBLK, nb = min(MAXBLK, NBLK - b0);

  uint4 pf[XPF];
  int tile = blockIdx.x;
  if (tile < total) {
    load_patch<T>(a, tile, pf);
    store_patch<T>(sx, pf);
  }
  lds_barrier();
  for (; tile < total; tile += G) {
    const TileGeo g = tile_geo(a, tile);
    // opaque per tile: keeps the tile-invariant block addresses (11 blocks x 9 taps) from
    // being hoisted out of the loop into registers
    int mm = m;
    asm volatile("" : "+v"(mm));
    // ---- MFMA per M-block of phase PH over the patch, then its epilogue: + bias, ReLU,
    // round to T -> the map (zero outside the image; the map has its own LDS region, so a
    // block's results leave registers at once) ----
#pragma unroll
    for (int j = 0; j < MAXBLK; ++j) {
      if (j >= nb) continue;
      const int pos = (b0 + j) * 16 + mm;
      const int pq = pos < NPOS ? pos / NP : 0, pr = pos < NPOS ? pos - (pos / NP) * NP : 0;
      const f32x4 acc = item_mfma<T, PH>(wr, sx + ((pq + 1) * XW + pr + 1) * XPST + 8 * kg,
                                         f32x4{0.f, 0.f, 0.f, 0.f});
      if (pos >= NPOS) continue;
      const int yy = 2 * pq + (PH >> 1), yx = 2 * pr + (PH & 1);
      const int gy = g.oy0 - 2 + yy, gx = g.ox0 - 2 + yx;
      const bool in = (unsigned)gy < (unsigned)H2 && (unsigned)gx < (unsigned)W2;
      uint2 v;
      v.x = in ? pack2<T>(fmaxf(acc[0] + bias[0], 0.f), fmaxf(acc[1] + bias[1], 0.f)) : 0u;
      v.y = in ? pack2<T>(fmaxf(acc[2] + bias[2], 0.f), fmaxf(acc[3] + bias[3], 0.f)) : 0u;
      *reinterpret_cast<uint2*>(sy + ymap(yy * YW + yx, kg >> 1) + 4 * (kg & 1)) = v;
    }
    lds_barrier();  // the map is complete; every patch read is done
    // the next tile's patch: loads in flight during this tile's Conv2D(1)
    const bool next = tile + G < total;
    if (next) load_patch<T>(a, tile + G, pf);

    // ---- Conv2D(1, 5x5) + sigmoid on MFMA: per output row y,
    //   D[x'][kx] = sum_{ky, ci} map[y + ky][x'][ci] w[ky][kx][ci]   (A = map, B = weights)
    //   out[y][x] = sum_kx D[x + kx][kx]
    // 3 MFMAs (kernel-row pairs) per 16 positions x', 3 position blocks per row; the
    // diagonal sums go through a per-wave scratch in the dead patch region ----
    {
      float* sp = reinterpret_cast<float*>(sx) + wave * (2 * KO * PXW);
      const int x = lane & 31, hh = lane >> 5;
      float* __restrict__ O = a.out + (long long)g.n * H2 * W2;
      const int gx = g.ox0 + x;
#pragma unroll 1
      for (int j = 0; j < 2; ++j) {  // rows 4 wave + 2 j + {0, 1}
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int yrow = 4 * wave + 2 * j + h;
#pragma unroll
          for (int xb = 0; xb < 3; ++xb) {
            f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
            const int xc = min(16 * xb + m, YW - 1);  // columns >= 36 feed no output
#pragma unroll
            for (int s2 = 0; s2 < 3; ++s2) {
              const int row = min(yrow + 2 * s2 + (kg >> 1), YW - 1);  // row 5: zero weights
              const uint4 av = *reinterpret_cast<const uint4*>(sy + ymap(row * YW + xc, kg & 1));
              acc = mfma<T>(av, wo_frag[s2], acc);
            }
            if (m < KO)  // D[x' = 16 xb + 4 kg + r][kx = m]
              *reinterpret_cast<f32x4*>(sp + (h * KO + m) * PXW + 16 * xb + 4 * kg) = acc;
          }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // wave-local: D in the scratch
        float sum = bo;
#pragma unroll
        for (int kx = 0; kx < KO; ++kx) sum += sp[(hh * KO + kx) * PXW + x + kx];
        const int gy = g.oy0 + 4 * wave + 2 * j + hh;
        if (gx < W2 && gy < H2) O[(long long)gy * W2 + gx] = 1.f / (1.f + __expf(-sum));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads done before the next D
      }
    }
    lds_barrier();  // every wave's scratch use is over before the next patch lands there
    if (next) store_patch<T>(sx, pf);  // the patch is dead since the first barrier
    lds_barrier();                      // next patch in; this tile's map reads done
  }
}

// Waves of a 512-thread workgroup go to the CU's SIMDs in the order 0 -> 2 -> 1 -> 3
// (MI355X_MICROARCH.md §Two waves per SIMD): waves w and w + 4 share a SIMD. The heavy
// phase (1,1) (9 taps) goes to waves 0, 1 and the light (0,0) (4 taps) to their SIMD
// partners 4, 5; (0,1) and (1,0) (6 taps) to waves 2, 3 and 6, 7: per SIMD 136 / 136 / 126 /
// 126 MFMAs per tile. Each phase's 21 M-blocks split 11 / 10 between its two waves.
template <typename T>
__global__ __launch_bounds__(512, 4) void convt_conv_out_kernel(TailArgs a) {
  __shared__ __attribute__((aligned(16))) T sx[XW * XW * XPST];  // input patch
  static_assert(8 * 2 * KO * PXW * sizeof(float) <= sizeof(sx), "Conv2D(1) scratch in the patch");
  __shared__ __attribute__((aligned(16))) T sy[YW * YW * CO];    // 16-channel map
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  switch (wave) {
    case 0: tail_body<T, 3>(a, sx, sy, wave, 0); break;
    case 1: tail_body<T, 3>(a, sx, sy, wave, 1); break;
    case 2: tail_body<T, 1>(a, sx, sy, wave, 0); break;
    case 3: tail_body<T, 2>(a, sx, sy, wave, 0); break;
    case 4: tail_body<T, 0>(a, sx, sy, wave, 0); break;
    case 5: tail_body<T, 0>(a, sx, sy, wave, 1); break;
    case 6: tail_body<T, 1>(a, sx, sy, wave, 1); break;
    default: tail_body<T, 2>(a, sx, sy, wave, 1); break;
  }
}

int resident_grid() { return 2 * device_cus(); }  // 2 workgroups per CU (LDS and registers)

// ============================================================================ row sweep
// tail_rows_kernel: the same two layers for 64-position-wide inputs (the model's 128-wide
// spectrogram strips and C5 images), walked DOWN the image one input-position row at a
// time instead of in 2-D tiles with halos. A workgroup owns a band of output rows of one
// image; its 4 waves own 16 position columns each (64 = the input width: no column halo).
//
// Step q (input-position row q):
//  a. Conv2DTranspose: for each of the 9 neighbourhood offsets (dy, dx) ONE B fragment
//     (32 channels x 16 positions of input row q + dy, shifted by dx) feeds every phase
//     that has the tap: 25 MFMAs from 9 LDS reads (the 2-D tile kernel: one read per
//     MFMA). The A operands (16 output channels x 32 input channels per tap, 25 taps) stay
//     in registers for the whole launch. Epilogue + bias, ReLU, round to T -> map rows
//     2q, 2q+1 of a 6-row LDS ring. A wave writes exactly the 32 map columns its own
//     Conv2D(1) blocks read, so the map needs no barrier.
//  b. Conv2D(16 -> 1, 5x5) for output rows 2q-2, 2q-1 (map rows 2q-4 .. 2q+1), on MFMA:
//     D[x'][(r, kx)] = sum_{p, dr, ci} map[2q-4+2p+dr][x'][ci] w[2p+dr-r][kx][ci], three
//     MFMAs (map-row pairs p) per 16 columns x' give 2 output rows x 5 kx (10 of 16 N
//     columns; the tile kernel's per-row form used 5), then out[y][x] = sum_kx D[x+kx-2]
//     [(r, kx)] through an LDS scratch (double-buffered).
//  c. input row q + 2 (loaded into registers two steps earlier) -> the 4-row LDS ring.
//  d. one barrier (ring slot and scratch), then the diagonal sums, sigmoid, fp32 stores,
//     and the load of input row q + 4.
// Map rows outside the image are the Conv2D(1) zero padding: the ring starts zeroed and
// steps past the last position row write zero rows.
namespace rows {
constexpr int QW = 64;               // input positions per row (the kernel's input width)
constexpr int XST = 48;              // input pixel stride (elements): 96 B, conflict-free
constexpr int XROW = (QW + 2) * XST;  // input ring row: pixels x = -1 .. 64
constexpr int NXR = 4;               // input ring rows
constexpr int MW = 2 * QW;           // 128 map / output columns
constexpr int MROW = MW * CO;        // map ring row (elements): 32-B pixels
constexpr int NMR = 8;               // map ring rows (a step writes 2, the Conv2D(1) reads 6)
constexpr int SCW = MW + 8;          // scratch row (floats): 4 zero pads each side
constexpr int SCR = 10;              // scratch rows (n = 5 r + kx)
constexpr int LDS_X = NXR * XROW * 2;          // bytes
constexpr int LDS_M = NMR * MROW * 2;
constexpr int LDS_S = 2 * SCR * SCW * 4;
constexpr int LDS_BYTES = LDS_X + LDS_M + LDS_S;  // 69,056 B: 2 workgroups per CU
}  // namespace rows

// map pixel p, 4-channel group g (8 B): the two 16-B halves of a pixel swap when bit 2 of p
// is set. The Conv2DTranspose epilogue writes 8 B per lane at 64-B pixel steps (plain
// layout: 8-way bank conflicts on ds_write_b64, 4-way with the swap) and the Conv2D(1) A
// reads (16 B = groups 2h, 2h + 1 of consecutive pixels) stay conflict-free.
__device__ __forceinline__ int map_off(int p, int g) { return p * CO + 4 * (g ^ (2 * ((p >> 2) & 1))); }

struct RowsArgs {
  const void* x;    // [N][H][64][32]
  const void* wt;   // convT forward GEMM weights [CO][KT][KT][CI]
  const float* bt;  // [CO]
  const void* wo;   // conv_out GEMM weights [KO][KO][CO]
  const float* bo;  // [1]
  float* out;       // [N][2H][128] (inference: sigmoid)
  void* map;        // TRAIN: the ReLU'd map [N][2H][128][CO] (T)
  float* logits;    // TRAIN: pre-sigmoid [N][2H][128]
  void* out_t;      // TRAIN: sigmoid [N][2H][128] (T)
  int N, H, R, nb;  // R: output rows per band (even), nb: bands per image
};

// bias + ReLU of four fp32 accumulators -> four T packed in 8 bytes. The accumulators start
// at the bias (folded into the MFMA chain); ReLU commutes with the monotone rounding, so for
// fp16 it runs on the packed halves (v_pk_max_f16: 2 instead of 4 VALU).
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

// The last two layers' per-wave state and steps, shared by tail_rows_kernel and
// decoder3_kernel: lane (m = lane & 15, kg = lane >> 4) of wave w (0..3) owns input
// positions 16 w + m of a position row, i.e. map columns 32 w .. 32 w + 31. Ring slots are
// passed as values that are compile-time constants at every call site (the step loops are
// unrolled by the ring period), so every LDS access is a per-lane base + an immediate.
template <typename T>
struct TailWave {
  uint4 wt[25];  // Conv2DTranspose taps (A: co = m, ci = 8 kg ..), phase-major, (dy, dx) order
  f32x4 bias;    // the accumulators' start
  float bo;
  uint4 wo[3];   // Conv2D(1) B fragments per map-row pair p: k = (dr, ci), n = 5 r + kx
  int mw[2];     // map write offset (elements, in a row) of this lane's pixel, px = 0, 1
  int gw[2];     // the same in a plain [128][CO] HBM row (training: the stored map)
  int mrd[2];    // map read offset of this lane's A row (pair row dr = kg >> 1), block 0, 1
  int scw[2];    // scratch write offset, block 0, 1
  int scr;       // scratch read offset of this lane's output (r, x), kx = 0
  int ox;        // this lane's output column x = 32 w + (lane & 31) (row r = lane >> 5)

  __device__ __forceinline__ void load(const void* wt_gemm, const float* bt, const void* wo_gemm,
                                       const float* b_o, int w, int lane) {
    using namespace rows;
    const int m = lane & 15, kg = lane >> 4;
    const T* __restrict__ Wt = reinterpret_cast<const T*>(wt_gemm);
    int u = 0;
#pragma unroll
    for (int ph = 0; ph < 4; ++ph)
#pragma unroll
      for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
        for (int dx = -1; dx <= 1; ++dx) {
          const int ky = ky_of(ph >> 1, dy), kx = ky_of(ph & 1, dx);
          if (ky < 0 || ky >= KT || kx < 0 || kx >= KT) continue;
          wt[u++] = *reinterpret_cast<const uint4*>(Wt + ((m * KT + ky) * KT + kx) * CI + 8 * kg);
        }
    bias = f32x4{bt[4 * kg], bt[4 * kg + 1], bt[4 * kg + 2], bt[4 * kg + 3]};
    bo = b_o[0];
    const T* __restrict__ Wo = reinterpret_cast<const T*>(wo_gemm);
    const int r = m / 5, kx = m - 5 * (m / 5), dr = kg >> 1;
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      const int ky = 2 * p + dr - r;
      wo[p] = uint4{0u, 0u, 0u, 0u};
      if (m < 10 && ky >= 0 && ky < KO)
        wo[p] = *reinterpret_cast<const uint4*>(Wo + (ky * KO + kx) * CO + 8 * (kg & 1));
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      mw[i] = map_off(2 * (16 * w + m) + i, kg);
      gw[i] = (2 * (16 * w + m) + i) * CO + 4 * kg;
      mrd[i] = (kg >> 1) * MROW + map_off(32 * w + 16 * i + m, 2 * (kg & 1));
      scw[i] = min(m, SCR - 1) * SCW + 4 + 32 * w + 16 * i + 4 * kg;
    }
    scr = 5 * (lane >> 5) * SCW + 4 + 32 * w + (lane & 31) - 2;
    ox = 32 * w + (lane & 31);
  }

  // Conv2DTranspose of one position row. xin: this lane's B-fragment address of input
  // row q - 1 (pixel 16 w + m - 1, group kg); xrow: elements between ring rows q+dy; xo(dx):
  // offset of the dx-shifted pixel; -> map rows at mrow0 / mrow1 (rows 2q, 2q + 1), and with
  // GST to the HBM rows g01 / g01 + 128 CO (training; null: a row outside the band).
  template <bool GST = false, typename RowOff, typename Xo>
  __device__ __forceinline__ void convt(const T* xin, RowOff xrow, Xo xo, T* mrow0,
                                        T* mrow1, T* __restrict__ g01 = nullptr) const {
    f32x4 acc[4] = {bias, bias, bias, bias};
    int u0[4] = {0, 4, 10, 16};  // first tap register of each phase (4 / 6 / 6 / 9 taps)
#pragma unroll
    for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
      for (int dx = -1; dx <= 1; ++dx) {
        const uint4 b = *reinterpret_cast<const uint4*>(xin + xrow(dy) + xo(dx));
#pragma unroll
        for (int ph = 0; ph < 4; ++ph) {
          const int ky = ky_of(ph >> 1, dy), kx = ky_of(ph & 1, dx);
          if (ky < 0 || ky >= KT || kx < 0 || kx >= KT) continue;
          acc[ph] = mfma<T>(wt[u0[ph]++], b, acc[ph]);
        }
      }
#pragma unroll
    for (int ph = 0; ph < 4; ++ph) {
      const uint2 v = relu_pack<T>(acc[ph]);
      *reinterpret_cast<uint2*>(((ph >> 1) ? mrow1 : mrow0) + mw[ph & 1]) = v;
      if constexpr (GST)
        if (g01) *reinterpret_cast<uint2*>(g01 + (ph >> 1) * (rows::MW * CO) + gw[ph & 1]) = v;
    }
  }

  __device__ __forceinline__ void zero_rows(T* mrow0, T* mrow1) const {
#pragma unroll
    for (int ph = 0; ph < 4; ++ph)
      *reinterpret_cast<uint2*>(((ph >> 1) ? mrow1 : mrow0) + mw[ph & 1]) = uint2{0u, 0u};
  }

  // Conv2D(1) MFMAs for output rows 2q - 2, 2q - 1: mrow(j) = map row 2q - 4 + j (j even;
  // row j + 1 is the next ring slot: the ring has an even row count and j is even) -> D into
  // the scratch scb
  template <typename MapRow>
  __device__ __forceinline__ void conv_out_d(MapRow mrow, float* scb, int m) const {
#pragma unroll
    for (int blk = 0; blk < 2; ++blk) {
      f32x4 d = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        // map row 2q - 4 + 2p + dr: lane groups kg >> 1 = 0 / 1 read the pair's two rows
        const uint4 av = *reinterpret_cast<const uint4*>(mrow(2 * p) + mrd[blk]);
        d = mfma<T>(av, wo[p], d);
      }
      if (m < rows::SCR)  // D[x' = 32 w + 16 blk + 4 kg + i][n = m]
        *reinterpret_cast<f32x4*>(scb + scw[blk]) = d;
    }
  }

  // diagonal sums of the scratch -> sigmoid -> output rows y0, y0 + 1 (O: the image's rows)
  __device__ __forceinline__ void conv_out_sums(const float* scb, float* __restrict__ O, int y0,
                                                int lane) const {
    float s = bo;
#pragma unroll
    for (int kx = 0; kx < KO; ++kx) s += scb[scr + kx * rows::SCW + kx];
    O[(long long)(y0 + (lane >> 5)) * rows::MW + ox] = __builtin_amdgcn_rcpf(1.f + __expf(-s));
  }

  // training: the same sums -> fp32 logits and the sigmoid in T
  __device__ __forceinline__ void conv_out_sums_train(const float* scb, float* __restrict__ L,
                                                      T* __restrict__ Ot, int y0, int lane) const {
    float s = bo;
#pragma unroll
    for (int kx = 0; kx < KO; ++kx) s += scb[scr + kx * rows::SCW + kx];
    const long long o = (long long)(y0 + (lane >> 5)) * rows::MW + ox;
    L[o] = s;
    Ot[o] = (T)__builtin_amdgcn_rcpf(1.f + __expf(-s));
  }
};

template <int I>
using IC = std::integral_constant<int, I>;

// v (this lane's value) moved within 16-lane rows by the DPP control CTRL (0 where the source
// lane is outside the row). The value first passes through an empty asm statement: applied
// directly to an element of an MFMA result vector, hipcc (ROCm 7.2) folds the DPP move into its
// user with the vector's FIRST register as the source (element 1 or 2 read element 0: the
// map-free decoder3 was wrong in every column but the first until this; the same happens with
// __builtin_amdgcn_mov_dpp). A plain 32-bit VGPR source is folded correctly.
template <int CTRL>
__device__ __forceinline__ float dpp_shift(float v) {
  int x = __builtin_bit_cast(int, v);
  asm volatile("" : "+v"(x));
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, x, CTRL, 0xf, 0xf, false));
}

template <typename T, bool TRAIN>
__global__ __launch_bounds__(256, 2) void tail_rows_kernel(RowsArgs a) {
  using namespace rows;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  T* const xr = reinterpret_cast<T*>(lds_raw);                  // input ring
  T* const mr = reinterpret_cast<T*>(lds_raw + LDS_X);          // map ring
  float* const sc = reinterpret_cast<float*>(lds_raw + LDS_X + LDS_M);  // D scratch x2

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int m = lane & 15, kg = lane >> 4;
  const int n = blockIdx.x / a.nb, band = blockIdx.x - n * a.nb;
  const int H = a.H, H2 = 2 * H;
  const int Y0 = band * a.R, Y1 = min(H2, Y0 + a.R);
  const int qa = max(0, Y0 / 2 - 1), qe = Y1 / 2;  // steps qa .. qe inclusive
  const T* __restrict__ X = reinterpret_cast<const T*>(a.x) + (long long)n * H * QW * CI;
  float* __restrict__ O = TRAIN ? nullptr : a.out + (long long)n * H2 * MW;
  float* __restrict__ L = TRAIN ? a.logits + (long long)n * H2 * MW : nullptr;
  T* __restrict__ Ot = TRAIN ? reinterpret_cast<T*>(a.out_t) + (long long)n * H2 * MW : nullptr;
  T* __restrict__ G = TRAIN ? reinterpret_cast<T*>(a.map) + (long long)n * H2 * MW * CO : nullptr;

  TailWave<T> tw;
  tw.load(a.wt, a.bt, a.wo, a.bo, w, lane);

  // ---- zero the rings and the scratch pads, then stage input rows qa-1 .. qa+1 ----
  {
    uint4* z = reinterpret_cast<uint4*>(lds_raw);
    for (int e = tid; e < LDS_BYTES / 16; e += 256) z[e] = uint4{0u, 0u, 0u, 0u};
  }
  __syncthreads();
  // ring slots relative to the band: input row qa - 1 + j in slot j & 3, map row 2 qa + j in
  // slot j & 7 (rows 2 qa - 4 .. 2 qa - 1 are the zeroed slots 4 .. 7 for the first band)
  const int spix = tid >> 2, scg = tid & 3;  // this thread's 16 B of a staged row
  T* const xst = xr + (spix + 1) * XST + 8 * scg;
  auto gload = [&](int row) -> uint4 {
    const int rr = min(max(row, 0), H - 1);
    uint4 v = *reinterpret_cast<const uint4*>(X + ((long long)rr * QW + spix) * CI + 8 * scg);
    if (row < 0 || row >= H) v = uint4{0u, 0u, 0u, 0u};
    return v;
  };
#pragma unroll
  for (int j = 0; j < 3; ++j) *reinterpret_cast<uint4*>(xst + j * XROW) = gload(qa - 1 + j);
  uint4 pa = gload(qa + 2), pb = gload(qa + 3);  // rows q+2 (even steps), q+3 (odd steps)
  lds_barrier();
  const T* const xin = xr + (16 * w + m) * XST + 8 * kg;  // pixel 16 w + m - 1 (stored + 1)

  // step i (q = qa + i) with I = i & 3 compile-time
  auto step = [&](auto ic, const int i, uint4& pre) {
    constexpr int I = decltype(ic)::value;
    const int q = qa + i;
    T* const m0 = mr + ((2 * I) & 7) * MROW;
    T* const m1 = mr + ((2 * I + 1) & 7) * MROW;
    if (q < H) {
      if constexpr (TRAIN)  // map rows 2q, 2q + 1 to HBM when they are this band's
        tw.template convt<true>(xin, [](int dy) { return ((I + 1 + dy) & 3) * XROW; },
                                [](int dx) { return (dx + 1) * XST; }, m0, m1,
                                2 * q >= Y0 && 2 * q < Y1 ? G + (long long)2 * q * MW * CO : nullptr);
      else
        tw.convt(xin, [](int dy) { return ((I + 1 + dy) & 3) * XROW; },
                 [](int dx) { return (dx + 1) * XST; }, m0, m1);
    } else  // below the image: the Conv2D(1) zero padding
      tw.zero_rows(m0, m1);
    const bool emit = 2 * q - 2 >= Y0;
    float* const scb = sc + (I & 1) * (SCR * SCW);
    if (emit)
      tw.conv_out_d([&](int j) { return mr + ((2 * I - 4 + j + 8) & 7) * MROW; }, scb, m);
    *reinterpret_cast<uint4*>(xst + ((I + 3) & 3) * XROW) = pre;  // input row q + 2
    lds_barrier();  // lgkmcnt only: the prefetch loads stay in flight across it
    if (emit) {
      if constexpr (TRAIN) tw.conv_out_sums_train(scb, L, Ot, 2 * q - 2, lane);
      else tw.conv_out_sums(scb, O, 2 * q - 2, lane);
    }
    pre = gload(q + 4);
  };

  const int ns = qe - qa + 1;
  int i = 0;
  for (; i + 4 <= ns; i += 4) {
    step(IC<0>{}, i, pa);
    step(IC<1>{}, i + 1, pb);
    step(IC<2>{}, i + 2, pa);
    step(IC<3>{}, i + 3, pb);
  }
  if (i < ns) step(IC<0>{}, i, pa);
  if (i + 1 < ns) step(IC<1>{}, i + 1, pb);
  if (i + 2 < ns) step(IC<2>{}, i + 2, pa);
}

// ============================================================================ decoder3
// decoder3_kernel: the model's last THREE layers in one launch, for 32-position-wide inputs
// (the C5 images: 32 x 32 x 64 -> 128 x 128):
//   Conv2DTranspose(32, 5, s2, relu) -> Conv2DTranspose(16, 5, s2, relu) -> Conv2D(1, 5,
//   sigmoid)  (VAE/manual_scan_3layers.py:196-199)
// The 64 x 64 x 32 map between the two Conv2DTransposes — 256 KB per image, the largest
// tensor of the unfused decoder after the tail's own map — is produced and consumed in LDS
// rows and never reaches HBM. One workgroup per image, 8 waves in two roles that share
// nothing but LDS rings and one barrier per macro step:
//  * producer waves 0-3 (one per (16-position window, 16-channel block) of the 32 x 32
//    channel output): Conv2DTranspose(64 -> 32) one input row s per macro step, every
//    neighbourhood offset's B fragment (2 K-steps) feeding all phases, 50 tap fragments
//    resident in registers -> rows 2s, 2s + 1 of the tail's input ring (64 positions x 32
//    channels, 64-byte pixels with a 16-byte group swizzle: conflict-free tail reads);
//  * consumer waves 4-7: two steps of the row-sweep tail (TailWave) per macro step, two
//    rows behind the producer.
// Waves w and w + 4 share a SIMD (MI355X_MICROARCH.md, two waves per SIMD): each SIMD pairs
// one producer and one consumer. Macro steps are unrolled by 4, the rings' period.
// the output emission (bias, edge word, sigmoid, store) of each tail step runs on the producer
// waves (idle 0.34 of a macro step, tools/d3_stats.py) from per-lane partial sums the consumer
// leaves in LDS; the consumer (0.95 busy) keeps only the two DPP adds and one LDS write.
// Measured 8 % SLOWER per launch (0.429 vs 0.398 ms per 2048, 3 interleaved rounds,
// profiles/r06_d3_producer_emit_ab.txt): the producers' added sigmoid, stores and LDS reads
// take issue slots from the consumer on the shared SIMD. Off; kept for the record.
#ifndef SPECENH_D3_PEMIT
#define SPECENH_D3_PEMIT 0
#endif
namespace d3 {
constexpr int CI1 = 64, CO1 = 32;     // the first Conv2DTranspose
constexpr int W1 = 32;                // its input positions per row
constexpr int X1ST = CI1;             // its input pixels: dense 128 B, 16-B groups swizzled
constexpr int X1ROW = (W1 + 2) * X1ST;
constexpr int NX1 = 8;                // input ring rows (positions g .. g + 3 + LEAD live)
constexpr int X2ST = 32;              // tail input pixel stride (elements): dense 64 B, swizzled
constexpr int X2ROW = (2 * W1 + 2) * X2ST;
constexpr int NX2 = 8;
constexpr int LDS_X1 = NX1 * X1ROW * 2;
constexpr int LDS_X2 = NX2 * X2ROW * 2;
constexpr int LDS_M = rows::NMR * rows::MROW * 2;
constexpr int LDS_S = 4 * rows::SCR * rows::SCW * 4;
constexpr int LDS_BYTES = LDS_X1 + LDS_X2 + LDS_M + LDS_S;  // 123,136 B: one workgroup per CU
// map-free consumer: per (macro-step parity, tail step of the pair) the column-boundary sums
// of the 4 consumer waves, slots 1 .. 4 (0 and 5: the image's zero borders), 2 sides x 4
// lane groups
constexpr int NBND = 6 * 2 * 4;
constexpr int BSTR = NBND + 64;  // exchange buffer stride: the slots + one dump word per lane
// SPECENH_D3_PEMIT: the consumer's per-lane partial sums of a tail step (parity, step, wave,
// lane) for the producer waves to finish and store
constexpr int LDS_ES = SPECENH_D3_PEMIT ? 2 * 2 * 4 * 64 * 4 : 0;
constexpr int LDS_BYTES_NM = LDS_X1 + LDS_X2 + 4 * BSTR * 4 + LDS_ES;  // 70,400 B (+ 4 KB PEMIT)
}  // namespace d3

// first Conv2DTranspose input pixel ps (x = ps - 1), 16-byte group g of its 8: group g sits
// at g ^ (ps & 7), so the producers' fragment reads (16 consecutive pixels, one group) are
// conflict-free; the rows arrive by LDS-DMA (lane-linear), the swizzle applied on the source
__device__ __forceinline__ int x1_off(int ps, int g) { return ps * d3::X1ST + 8 * (g ^ (ps & 7)); }

// tail input pixel p (-1 .. 64 stored at p + 1), 16-byte group g: groups swizzled by bits 1-2
// of the stored pixel (producer 8-byte writes at 2-pixel steps 4-way instead of 8-way;
// consumer 16-byte reads of consecutive pixels conflict-free)
__device__ __forceinline__ int x2_off(int ps, int g) { return ps * d3::X2ST + 8 * (g ^ ((ps >> 1) & 3)); }


#ifndef SPECENH_D3_CPRIO
// round 4: +4 % (profiles/r04_d3_ab.txt); round 6, with the zero-map steps skipped and the
// consumer at 0.95 of the macro step vs the producers' 0.66 (tools/d3_stats.py): -1.3 % per
// launch over 3 interleaved rounds (profiles/r06_d3_cprio_ab.txt)
#define SPECENH_D3_CPRIO 1
#endif
#ifndef SPECENH_D3_BRANCHFREE
#define SPECENH_D3_BRANCHFREE 1
#endif

struct D3Args {
  const void* x;     // [N][H][32][64]
  const void* w1;    // first Conv2DTranspose forward GEMM weights [32][5][5][64]
  const float* b1;   // [32]
  const void* wt;    // second [16][5][5][32]
  const float* bt;   // [16]
  const void* wo;    // Conv2D(1) [5][5][16]
  const float* bo;   // [1]
  void* out;         // [N][4H][128], fp32 or (out_f16) fp16
  int N, H;
  int out_f16;       // store the sigmoid outputs as fp16 (the C5 stream's 32,768 B per shot)
};

#ifdef SPECENH_D3_STATS  // development build (tools/d3_stats.py): per-wave barrier clocks
__device__ unsigned long long d3_stats[1024 * 8 * 4];
struct D3Clock {
  long long last = 0, busy = 0, wait = 0, n = 0;
  __device__ __forceinline__ void barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const long long t0 = __builtin_amdgcn_s_memtime();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const long long t1 = __builtin_amdgcn_s_memtime();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (last) busy += t0 - last;
    wait += t1 - t0;
    ++n;
    last = t1;
  }
  __device__ void flush(int wv) {
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 1024) {
      unsigned long long* p = d3_stats + (blockIdx.x * 8 + wv) * 4;
      p[0] = busy; p[1] = wait; p[2] = n; p[3] = 0;
    }
  }
};
#define D3_BARRIER() clk.barrier()
#else
#define D3_BARRIER() lds_barrier()
#endif

// MAP = false (the default since round 4): the consumer never writes the 16-channel map. Its
// Conv2D(1) runs as MFMAs on the Conv2DTranspose's own packed accumulators (the B operand of
// v_mfma_f32_16x16x32 is exactly what the ReLU-packed 16x16 accumulators of one phase pair hold:
// 8 channels-by-column values of one position per lane), into three rolling accumulators of
// output-row PAIRS; only the column shifts of the 5 x 5 window cross lanes (DPP row shifts) and,
// at the 16-position block edges, waves (8 floats through LDS per tail step). MAP = true keeps
// the round-3 consumer (map ring + D scratch + diagonal sums; V_D3_MAP) for A/B.
// LEAD: the producer's input-ring refills in flight beyond the one a macro step waits for
// (step g needs position g + 3 after its barrier and waits for that DMA only, issued LEAD steps
// earlier; round 3: LEAD 0, the DMA issued by the same step).
template <typename T, bool MAP, int LEAD, bool OUT16 = false>
__global__ __launch_bounds__(512, 2) void decoder3_kernel(D3Args a) {
  static_assert(LEAD >= 0 && LEAD <= 4, "8-row input ring");
  using namespace d3;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  constexpr int LB = MAP ? LDS_BYTES : LDS_BYTES_NM;
  T* const x1r = reinterpret_cast<T*>(lds_raw);
  T* const x2r = reinterpret_cast<T*>(lds_raw + LDS_X1);
  T* const mr = reinterpret_cast<T*>(lds_raw + LDS_X1 + LDS_X2);
  float* const sc = reinterpret_cast<float*>(lds_raw + LDS_X1 + LDS_X2 + LDS_M);
  float* const bnd = reinterpret_cast<float*>(lds_raw + LDS_X1 + LDS_X2);  // !MAP
  float* const es = bnd + 4 * BSTR;                                          // !MAP, PEMIT

  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int m = lane & 15, kg = lane >> 4;
  const int H1 = a.H, H2 = 2 * H1, H3 = 4 * H1;
#ifdef SPECENH_D3_STATS
  D3Clock clk;
#endif
  // Persistent workgroups: one continuous row stream over the workgroup's images
  // n = blockIdx.x + i G. Per image SPI = H1 + 1 macro steps: producer step s = 0 .. H1 - 1
  // turns input row s into tail-input rows 2s, 2s + 1, step s = H1 writes the two zero rows
  // that separate images; the consumer's tail steps then run on, 2 per macro step, with
  // per-image tail step t = 0 .. 2 H1 + 1 (t >= 2 H1: zero map rows). The input stream has
  // one zero row between images (position i SPI), so producer step g reads positions
  // g .. g + 2. Ring slots are global (macro step g, tail steps 2g - 4 / 2g - 3; the MAP
  // consumer 2g - 3 / 2g - 2), so the
  // compile-time slot offsets of the unrolled loops are the single-image ones. Round 2/3
  // launched one workgroup per image: per image the LDS clear, the 50 + 28 fragment loads
  // and the pipeline fill and drain (3 of 35 macro steps) were paid again.
  const int SPI = H1 + 1, TPI = 2 * SPI;
  const int G = gridDim.x;
  const int nimg = ((int)a.N - (int)blockIdx.x + G - 1) / G;
  const int S = nimg * SPI + 2;  // + 2: the consumer's last tail steps
  {
    uint4* z = reinterpret_cast<uint4*>(lds_raw);
    for (int e = tid; e < LB / 16; e += 512) z[e] = uint4{0u, 0u, 0u, 0u};
  }
  __syncthreads();

  if (wv < 4) {
    // ======================= producer: Conv2DTranspose(64 -> 32), input rows s - 1 .. s + 1
    const int wx = wv & 1, nb = wv >> 1;
    uint4 w1[50];  // [phase taps][k-step]
    {
      const T* __restrict__ Wg = reinterpret_cast<const T*>(a.w1);
      int u = 0;
#pragma unroll
      for (int ph = 0; ph < 4; ++ph)
#pragma unroll
        for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
          for (int dx = -1; dx <= 1; ++dx) {
            const int ky = ky_of(ph >> 1, dy), kx = ky_of(ph & 1, dx);
            if (ky < 0 || ky >= KT || kx < 0 || kx >= KT) continue;
#pragma unroll
            for (int kh = 0; kh < 2; ++kh)
              w1[u++] = *reinterpret_cast<const uint4*>(
                  Wg + (((16 * nb + m) * KT + ky) * KT + kx) * CI1 + 32 * kh + 8 * kg);
          }
    }
    const f32x4 bias = f32x4{a.b1[16 * nb + 4 * kg], a.b1[16 * nb + 4 * kg + 1],
                             a.b1[16 * nb + 4 * kg + 2], a.b1[16 * nb + 4 * kg + 3]};
    resident_loads_landed();
    const T* __restrict__ X = reinterpret_cast<const T*>(a.x);
    // input stream position p (image p / SPI, row p % SPI - 1; row -1 is the zero row) ->
    // ring slot p & 3 by LDS-DMA: wave wv moves stored pixels 1 + 8 wv .. 8 + 8 wv (1 KB,
    // lane-linear); lane i takes stored group i & 7, i.e. source group (i & 7) ^ (ps & 7)
    const int dps = 1 + 8 * wv + (lane >> 3);
    const int dsrc = (dps - 1) * CI1 + 8 * ((lane & 7) ^ (dps & 7));
    unsigned char* const ddst = lds_raw + (1 + 8 * wv) * X1ST * 2;
    // position p = il SPI + row + 1; returns whether this wave issued an LDS-DMA
    auto stage_at = [&](int p, int il, int row) -> bool {
      unsigned char* dst = ddst + (p & (NX1 - 1)) * X1ROW * 2;
      if (il < nimg && row >= 0 && row < H1) {
        const long long n = (long long)blockIdx.x + (long long)il * G;
        lds_dma16_s(X + ((n * H1 + row) * W1) * CI1, 2u * dsrc, dst);
        return true;
      }
      // between / after the images: the zero padding rows
      *reinterpret_cast<uint4*>(dst + 16 * lane) = uint4{0u, 0u, 0u, 0u};
      return false;
    };
    auto stage = [&](int p) -> bool {  // (prologue)
      const int il = p / SPI;
      return stage_at(p, il, p - il * SPI - 1);
    };
    // this lane's B-fragment offsets (pixel 16 wx + m + dx, group kg) in an input ring row,
    // and its 16-byte tail-input write offset: after the row-pair swap (store_pair below) a
    // lane of an even row kg holds phase px = 0's channels 16 nb + 4 kg .. + 7 and a lane of an
    // odd row phase px = 1's channels 16 nb + 4 (kg - 1) .. + 7, i.e. 16-byte group
    // 2 nb + kg / 2 of pixel 2 (16 wx + m) + 1 + (kg & 1)
    int xo[3];
#pragma unroll
    for (int dx = -1; dx <= 1; ++dx) xo[dx + 1] = x1_off(16 * wx + m + dx + 1, kg);
    const int x2w16 = x2_off(2 * (16 * wx + m) + 1 + (kg & 1), 2 * nb + (kg >> 1));
    // One tail-input row's two phases (px = 0, 1) as ONE ds_write_b128 per lane instead of two
    // 4-way conflicted ds_write_b64: v_permlane16_swap exchanges odd rows of the first operand
    // with even rows of the second, so rows kg, kg ^ 1 trade the halves they do not keep (PMC
    // round 4: the 8-byte writes were 0.24 of the LDS-array cycles in bank conflicts; the
    // 16-byte writes are 2-way at most, under their transfer cycles)
    auto store_pair = [&](T* row, uint2 p0, uint2 p1) {
      const auto sx = __builtin_amdgcn_permlane16_swap(p0.x, p1.x, false, false);
      const auto sy = __builtin_amdgcn_permlane16_swap(p0.y, p1.y, false, false);
      *reinterpret_cast<uint4*>(row + x2w16) = uint4{sx[0], sy[0], sx[1], sy[1]};
    };
#pragma unroll
    for (int p = 0; p < 3 + LEAD; ++p) stage(p);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    D3_BARRIER();  // (macro step -1: the consumers' matching barrier is below)
    int vmn = 0;       // this wave's LDS-DMAs issued in the loop (its only vector-memory ops)
    int mk[LEAD + 1];  // vmn right after the DMA of position g + 3 + i (-1: none in flight)
#pragma unroll
    for (int i = 0; i <= LEAD; ++i) mk[i] = -1;

    // the consumer's emission (SPECENH_D3_PEMIT): its lane layout for consumer wave wv, and the
    // (image, tail step) counters of its tail steps 2g - 4, 2g - 3
    int eil_p = -1, etl_p = TPI - 4;
    const int orow_p = kg >> 1, ocol_p = 32 * wv + 2 * m + (kg & 1);
    const int bri_p = m == 0 ? (wv * 2 + 0) * 4 + kg : (m == 15 ? ((wv + 2) * 2 + 1) * 4 + kg : 0);
    // scalar counters (image, step in image) of macro step g and of its refill position
    int ilg = 0, sg = 0;
    int ilp = (3 + LEAD) / SPI, sp = 3 + LEAD - ilp * SPI;
    auto pstep = [&](auto ic, const int g) {
      constexpr int I = decltype(ic)::value;  // g & 7 (the input ring's period)
      mk[LEAD] = stage_at(g + 3 + LEAD, ilp, sp - 1) ? ++vmn : -1;
      T* const r0 = x2r + ((2 * I) & 7) * X2ROW;  // (tail ring: period 4 macro steps)
      T* const r1 = x2r + ((2 * I + 1) & 7) * X2ROW;
      if (ilg < nimg && sg < H1) {
        f32x4 acc[4] = {bias, bias, bias, bias};
        int u0[4] = {0, 8, 20, 32};
#pragma unroll
        for (int dy = -1; dy <= 1; ++dy) {
          const T* src = x1r + ((I + 1 + dy + NX1) & (NX1 - 1)) * X1ROW;  // position g + 1 + dy
#pragma unroll
          for (int dx = -1; dx <= 1; ++dx) {
            // group kg + 4 (the second K-step) sits at the first's offset ^ 32 elements:
            // the swizzle XORs the group index, whose bit 2 is element-offset bit 5
            const uint4 b0 = *reinterpret_cast<const uint4*>(src + xo[dx + 1]);
            const uint4 b1 = *reinterpret_cast<const uint4*>(src + (xo[dx + 1] ^ 32));
#pragma unroll
            for (int ph = 0; ph < 4; ++ph) {
              const int ky = ky_of(ph >> 1, dy), kx = ky_of(ph & 1, dx);
              if (ky < 0 || ky >= KT || kx < 0 || kx >= KT) continue;
              acc[ph] = mfma<T>(w1[u0[ph]], b0, acc[ph]);
              acc[ph] = mfma<T>(w1[u0[ph] + 1], b1, acc[ph]);
              u0[ph] += 2;
            }
          }
        }
        store_pair(r0, relu_pack<T>(acc[0]), relu_pack<T>(acc[1]));
        store_pair(r1, relu_pack<T>(acc[2]), relu_pack<T>(acc[3]));
      } else {  // tail-input rows 2 H1, 2 H1 + 1 (and past the last image): zero padding
        *reinterpret_cast<uint4*>(r0 + x2w16) = uint4{0u, 0u, 0u, 0u};
        *reinterpret_cast<uint4*>(r1 + x2w16) = uint4{0u, 0u, 0u, 0u};
      }
      if (mk[0] >= 0) wait_vmcnt_ss<LEAD>(vmn - mk[0]);  // input position g + 3 has landed
      D3_BARRIER();
#pragma unroll
      for (int i = 0; i < LEAD; ++i) mk[i] = mk[i + 1];
      if (++sg == SPI) { sg = 0; ++ilg; }
      if (++sp == SPI) { sp = 0; ++ilp; }
      if constexpr (!MAP && SPECENH_D3_PEMIT) {
#pragma unroll
        for (int k = 0; k < 2; ++k) {  // the consumer's tail steps 2g - 4 + k of this macro step
          const int eil = eil_p, etl = etl_p;
          if (++etl_p == TPI) { etl_p = 0; ++eil_p; }
          if (eil >= 0 && eil < nimg && etl >= 1 && etl <= H2) {
            const float sp_ = es[(((I & 1) * 2 + k) * 4 + wv) * 64 + lane] +
                              bnd[((I & 1) * 2 + k) * BSTR + bri_p];
            const long long n = (long long)blockIdx.x + (long long)eil * G;
            const long long o = (n * H3 + 2 * (etl - 1) + orow_p) * rows::MW + ocol_p;
            const float y = __builtin_amdgcn_rcpf(1.f + __expf(-sp_));
            if constexpr (OUT16)
              reinterpret_cast<_Float16*>(a.out)[o] = (_Float16)y;
            else
              reinterpret_cast<float*>(a.out)[o] = y;
          }
        }
      }
    };
    int g = 0;
    for (; g + 8 <= S; g += 8) {
      pstep(IC<0>{}, g);
      pstep(IC<1>{}, g + 1);
      pstep(IC<2>{}, g + 2);
      pstep(IC<3>{}, g + 3);
      pstep(IC<4>{}, g + 4);
      pstep(IC<5>{}, g + 5);
      pstep(IC<6>{}, g + 6);
      pstep(IC<7>{}, g + 7);
    }
    if (g < S) pstep(IC<0>{}, g);
    if (g + 1 < S) pstep(IC<1>{}, g + 1);
    if (g + 2 < S) pstep(IC<2>{}, g + 2);
    if (g + 3 < S) pstep(IC<3>{}, g + 3);
    if (g + 4 < S) pstep(IC<4>{}, g + 4);
    if (g + 5 < S) pstep(IC<5>{}, g + 5);
    if (g + 6 < S) pstep(IC<6>{}, g + 6);
#ifdef SPECENH_D3_STATS
    clk.flush(wv);
#endif
  } else if constexpr (!MAP) {
    // ======================= map-free consumer, tail steps t = 2g - 4, 2g - 3 per macro step g
    // Tail step t (per-image tl) turns tail-input rows t - 1 .. t + 1 into the Conv2DTranspose
    // accumulators of map rows 2tl, 2tl + 1 (16 positions x 16 channels x 4 phases per wave),
    // packs them after bias + ReLU exactly as the map would hold them, and adds their Conv2D(1)
    // contributions to output-row pairs tl - 1, tl, tl + 1 (P0, P1, P2). Pair tl - 1 is then
    // complete (map rows 2tl - 4 .. 2tl + 1) and is emitted after the macro step's barrier.
    const int w = wv - 4;
    uint4 wt[25];  // Conv2DTranspose taps (A: co = m, ci = 8 kg ..), phase-major, (dy, dx) order
    {
      const T* __restrict__ Wt = reinterpret_cast<const T*>(a.wt);
      int u = 0;
#pragma unroll
      for (int ph = 0; ph < 4; ++ph)
#pragma unroll
        for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
          for (int dx = -1; dx <= 1; ++dx) {
            const int ky = ky_of(ph >> 1, dy), kx = ky_of(ph & 1, dx);
            if (ky < 0 || ky >= KT || kx < 0 || kx >= KT) continue;
            wt[u++] = *reinterpret_cast<const uint4*>(Wt + ((m * KT + ky) * KT + kx) * CI + 8 * kg);
          }
    }
    const f32x4 bias = f32x4{a.bt[4 * kg], a.bt[4 * kg + 1], a.bt[4 * kg + 2], a.bt[4 * kg + 3]};
    // Conv2D(1) A fragments wd[d][py] for pair tl + d - 1 and map row 2tl + py. Result row
    // i = 4 gO + j (gO = i >> 2: output row r = gO >> 1 of the pair, column parity o = gO & 1)
    // holds output column 2 m' + ox of position m', ox = o + {0, 2, -2}[j] (j = 3 unused), so
    // lane group g of the result owns output (r, o) = (g >> 1, g & 1) of its position and
    // receives the ox = o + 2 / o - 2 parts from positions m - 1 / m + 1. K = 8 kA + 4 px + c:
    // channel 4 kA + c of map column 2 m' + px (the packed B layout below).
    // ky = py + 2 - 2 (d - 1) - r, kx = px + 2 - ox.
    uint4 wd[3][2];
    {
      const T* __restrict__ Wo = reinterpret_cast<const T*>(a.wo);
      const int i = lane & 15, kA = lane >> 4;
      const int gO = i >> 2, j = i & 3, r = gO >> 1, o = gO & 1;
      const int ox = o + (j == 1 ? 2 : (j == 2 ? -2 : 0));
#pragma unroll
      for (int d = 0; d < 3; ++d)
#pragma unroll
        for (int py = 0; py < 2; ++py) {
          const int ky = py + 2 - 2 * (d - 1) - r;
          uint32_t e[4];
#pragma unroll
          for (int h = 0; h < 4; ++h) {
            uint32_t v2 = 0;
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
              const int el = 2 * h + s2, px = el >> 2, c = el & 3, kx = px + 2 - ox;
              unsigned short bits = 0;
              if (j < 3 && ky >= 0 && ky < KO && kx >= 0 && kx < KO)
                bits = __builtin_bit_cast(unsigned short, Wo[(ky * KO + kx) * CO + 4 * kA + c]);
              v2 |= (uint32_t)bits << (16 * s2);
            }
            e[h] = v2;
          }
          wd[d][py] = uint4{e[0], e[1], e[2], e[3]};
        }
    }
    const float bo = a.bo[0];
    resident_loads_landed();
    int xo[3];  // element offset of pixel 16 w + m + dx (stored + 1), group kg, in a ring row
#pragma unroll
    for (int dx = -1; dx <= 1; ++dx) xo[dx + 1] = x2_off(16 * w + m + dx + 1, kg);
    // this lane's output pixel of a pair: row kg >> 1, column 32 w + 2 m + (kg & 1); block-edge
    // exchange: lane m = 15 publishes E[1] (column 2 m + o + 2: the next wave's m = 0) in slot
    // w + 1 side 0, lane m = 0 publishes E[2] in side 1; m = 0 / 15 read the neighbours' slots,
    // every other lane a never-written zero word
    const int orow = kg >> 1, ocol = 32 * w + 2 * m + (kg & 1);
    // every lane stores its word each tail step (no exec-mask branch): lanes other than
    // m = 0 / 15 into their own word of the buffer's dump area (one lane-constant index: a
    // per-buffer pointer select had compiled to exec-mask branches every tail step)
    const int bwi = (m == 0 || m == 15) ? ((w + 1) * 2 + (m == 0 ? 1 : 0)) * 4 + kg : NBND + lane;
    const int bri = m == 0 ? (w * 2 + 0) * 4 + kg : (m == 15 ? ((w + 2) * 2 + 1) * 4 + kg : 0);
#if SPECENH_D3_CPRIO
    // the consumer waves are the macro step's critical path (barrier clocks, tools/d3_stats.py:
    // busy 95 % of the step vs the producers' 81 %): they win the SIMD's issue arbitration
    __builtin_amdgcn_s_setprio(1);
#endif
    D3_BARRIER();  // macro step -1

    f32x4 P0 = f32x4{0.f, 0.f, 0.f, 0.f}, P1 = P0, P2 = P0;
    // tail steps t = 2g - 4, 2g - 3 per macro step g (round 6; round 5: 2g - 3, 2g - 2): the
    // per-image steps pair as (even, odd), so the two zero-map steps 2 H1, 2 H1 + 1 of an image
    // share one macro step, which skips their MFMAs (tskip) instead of masking them
    int il = -1, tl = TPI - 4;  // tail step t = -4
    // the nine B fragments of tail step t (ring slot T8 = t & 7): rows t - 1 .. t + 1, pixel
    // shifts dx = -1 .. 1
    auto frags = [&](auto ic, uint4 (&bq)[9]) {
      constexpr int T8 = decltype(ic)::value;
#pragma unroll
      for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
        for (int dx = -1; dx <= 1; ++dx)
          bq[3 * (dy + 1) + dx + 1] =
              *reinterpret_cast<const uint4*>(x2r + ((T8 + dy + 8) & 7) * X2ROW + xo[dx + 1]);
    };
    auto tstep = [&](auto ic, const uint4 (&bq)[9], float* bb, f32x4& E, int& eil,
                     int& etl) -> bool {
      constexpr int T8 = decltype(ic)::value;  // t & 7: the tail-input ring slot of row t
      (void)T8;
      eil = il;
      etl = tl;
      if (++tl == TPI) { tl = 0; ++il; }
      const bool img = eil >= 0 && eil < nimg;
#if !SPECENH_D3_BRANCHFREE
      if (!img) return false;
#endif
      // (branch-free: before the first / past the last image the ring rows are zero rows and
      // the results are masked, so both tail steps of a macro step form one basic block and
      // the scheduler can interleave their MFMA chains)
      f32x4 acc[4] = {bias, bias, bias, bias};
      int u0[4] = {0, 4, 10, 16};  // first tap register of each phase (4 / 6 / 6 / 9 taps)
      // all nine B fragments first (frags, by the caller), then the 25 MFMAs: read in pairs
      // just ahead of their MFMAs (the compiler's schedule), each pair's LDS latency was exposed
#pragma unroll
      for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
        for (int dx = -1; dx <= 1; ++dx) {
          const uint4 b = bq[3 * (dy + 1) + dx + 1];
#pragma unroll
          for (int ph = 0; ph < 4; ++ph) {
            const int ky = ky_of(ph >> 1, dy), kx = ky_of(ph & 1, dx);
            if (ky < 0 || ky >= KT || kx < 0 || kx >= KT) continue;
            acc[ph] = mfma<T>(wt[u0[ph]++], b, acc[ph]);
          }
        }
      // map rows 2tl, 2tl + 1 as the Conv2D(1)'s B operands (zero below the image)
      const uint32_t keep = img && etl < H2 ? 0xffffffffu : 0u;
      uint4 bv[2];
#pragma unroll
      for (int py = 0; py < 2; ++py) {
        const uint2 lo = relu_pack<T>(acc[2 * py]), hi = relu_pack<T>(acc[2 * py + 1]);
        bv[py] = uint4{lo.x & keep, lo.y & keep, hi.x & keep, hi.y & keep};
      }
#pragma unroll
      for (int py = 0; py < 2; ++py) {
        P0 = mfma<T>(wd[0][py], bv[py], P0);
        P1 = mfma<T>(wd[1][py], bv[py], P1);
        P2 = mfma<T>(wd[2][py], bv[py], P2);
      }
      E = P0;
      P0 = P1;
      P1 = P2;
      P2 = f32x4{0.f, 0.f, 0.f, 0.f};
#if SPECENH_D3_BRANCHFREE
      bb[bwi] = m == 0 ? E[2] : E[1];
      return img && etl >= 1 && etl <= H2;  // pair tl - 1 is an output row pair
#else
      if (etl < 1 || etl > H2) return false;  // pair tl - 1 is not an output row pair
      if (m == 0 || m == 15) bb[bwi] = m == 0 ? E[2] : E[1];
      return true;
#endif
    };
    // a tail step without MFMAs (zero map rows: the image's steps 2 H1, 2 H1 + 1 and the
    // pipeline's fill / drain): the pair rotation, exchange store and emit test of tstep
    auto tskip = [&](float* bb, f32x4& E, int& eil, int& etl) -> bool {
      eil = il;
      etl = tl;
      if (++tl == TPI) { tl = 0; ++il; }
      E = P0;
      P0 = P1;
      P1 = P2;
      P2 = f32x4{0.f, 0.f, 0.f, 0.f};
      bb[bwi] = m == 0 ? E[2] : E[1];
      return eil >= 0 && eil < nimg && etl >= 1 && etl <= H2;
    };
    auto emit = [&](const f32x4& E, float edge, int eil, int etl) {  // edge: bb[bri]
      float s = bo + E[0];
      s += dpp_shift<0x111>(E[1]);  // row_shr:1: lane m reads lane m - 1
      s += dpp_shift<0x101>(E[2]);  // row_shl:1: lane m reads lane m + 1
      s += edge;
      const long long n = (long long)blockIdx.x + (long long)eil * G;
      const long long o = (n * H3 + 2 * (etl - 1) + orow) * rows::MW + ocol;
      const float y = __builtin_amdgcn_rcpf(1.f + __expf(-s));
      // (the output dtype as a template argument: a run-time test of out_f16 split the macro
      // step into blocks, and the LDS waits after the join were conservative; 1.1 % per launch)
      if constexpr (OUT16)
        reinterpret_cast<_Float16*>(a.out)[o] = (_Float16)y;
      else
        reinterpret_cast<float*>(a.out)[o] = y;
    };
    auto cstep = [&](auto ic) {
      constexpr int I = decltype(ic)::value;  // g & 3
      float* const b0 = bnd + ((I & 1) * 2) * BSTR;
      float* const b1 = b0 + BSTR;
      f32x4 E0, E1;
      int il0, tl0, il1, tl1;
      bool e0, e1;
      if (il >= 0 && il < nimg && tl < H2) {  // (wave-uniform) both steps inside an image
        uint4 bq[9];
        frags(IC<(2 * I + 4) & 7>{}, bq);  // (2g - 4) & 7
        __builtin_amdgcn_sched_barrier(0);
        e0 = tstep(IC<(2 * I + 4) & 7>{}, bq, b0, E0, il0, tl0);
        frags(IC<(2 * I + 5) & 7>{}, bq);
        __builtin_amdgcn_sched_barrier(0);
        e1 = tstep(IC<(2 * I + 5) & 7>{}, bq, b1, E1, il1, tl1);
      } else {
        e0 = tskip(b0, E0, il0, tl0);
        e1 = tskip(b1, E1, il1, tl1);
      }
#if SPECENH_D3_PEMIT
      (void)e0;
      (void)e1;
      float* const ep = es + ((I & 1) * 2 * 4 + w) * 64 + lane;
      // (emit's summation order: bo + E[0], the two shifted terms, then the edge word)
      ep[0] = ((bo + E0[0]) + dpp_shift<0x111>(E0[1])) + dpp_shift<0x101>(E0[2]);
      ep[4 * 64] = ((bo + E1[0]) + dpp_shift<0x111>(E1[1])) + dpp_shift<0x101>(E1[2]);
      D3_BARRIER();
#else
      D3_BARRIER();
      // (emitting these in the next macro step, after its first fragment reads, to overlap the
      // two LDS latencies: measured neutral, profiles/r06_d3_out16_ab.txt)
      if (e0) emit(E0, b0[bri], il0, tl0);
      if (e1) emit(E1, b1[bri], il1, tl1);
#endif
    };
    int g = 0;
    for (; g + 4 <= S; g += 4) {
      cstep(IC<0>{});
      cstep(IC<1>{});
      cstep(IC<2>{});
      cstep(IC<3>{});
    }
    if (g < S) cstep(IC<0>{});
    if (g + 1 < S) cstep(IC<1>{});
    if (g + 2 < S) cstep(IC<2>{});
#ifdef SPECENH_D3_STATS
    clk.flush(wv);
#endif
  } else {
    // ======================= consumer: the row-sweep tail, tail steps t = 2g - 3, 2g - 2
    const int w = wv - 4;
    TailWave<T> tw;
    tw.load(a.wt, a.bt, a.wo, a.bo, w, lane);
    int xo[3];  // element offset of pixel 16 w + m + dx (stored + 1), group kg, in a ring row
#pragma unroll
    for (int dx = -1; dx <= 1; ++dx) xo[dx + 1] = x2_off(16 * w + m + dx + 1, kg);
    D3_BARRIER();  // macro step -1
    // global tail step t (image t / TPI, per-image step tl = t % TPI) with T8 = t & 7
    // compile-time from g & 3. The Conv2D(1) of step tl is for output rows 2tl - 4, 2tl - 3
    // (map rows 2tl - 6 .. 2tl - 1, all written by earlier steps: the 8-row map ring holds
    // 2t - 6 .. 2t + 1), so it does not wait for this step's Conv2DTranspose and the two MFMA
    // streams interleave. It is issued first: its map reads then precede this step's map
    // writes into the slots of rows 2t - 8, 2t - 7. Map rows of per-image steps tl >= 2 H1
    // are zero (the Conv2D(1) padding below one image and above the next).
    auto tstep = [&](auto ic, const int t, float* scb) {
      constexpr int T8 = decltype(ic)::value;  // t & 7: the tail-input ring slot of row t
      constexpr int T4 = T8 & 3;                // the map ring: rows 2t, 2t + 1 in slots 2 T4 ..
      if (t < 0) return;
      const int il = t / TPI, tl = t - il * TPI;
      if (il >= nimg) return;
      if (tl >= 2)
        tw.conv_out_d([&](int j) { return mr + ((2 * T4 - 6 + j + 8) & 7) * rows::MROW; }, scb,
                      m);
      T* const m0 = mr + ((2 * T4) & 7) * rows::MROW;
      T* const m1 = mr + ((2 * T4 + 1) & 7) * rows::MROW;
      if (tl < H2)
        tw.convt(x2r, [](int dy) { return ((T8 + dy + 8) & 7) * X2ROW; },
                 [&](int dx) { return xo[dx + 1]; }, m0, m1);
      else
        tw.zero_rows(m0, m1);
    };
    auto sums = [&](const float* scb, int t) {
      if (t < 0) return;
      const int il = t / TPI, tl = t - il * TPI;
      if (il >= nimg || tl < 2) return;
      const long long n = (long long)blockIdx.x + (long long)il * G;
      tw.conv_out_sums(scb, reinterpret_cast<float*>(a.out) + n * H3 * rows::MW, 2 * tl - 4,
                       lane);  // (fp32 output only: the host refuses out_f16 with V_D3_MAP)
    };
    auto cstep = [&](auto ic, const int g) {
      constexpr int I = decltype(ic)::value;  // g & 3
      float* const sc0 = sc + ((I & 1) * 2) * (rows::SCR * rows::SCW);
      float* const sc1 = sc0 + rows::SCR * rows::SCW;
      tstep(IC<(2 * I + 5) & 7>{}, 2 * g - 3, sc0);  // (2g - 3) & 7 = (2 I - 3) & 7
      tstep(IC<(2 * I + 6) & 7>{}, 2 * g - 2, sc1);
      D3_BARRIER();
      sums(sc0, 2 * g - 3);
      sums(sc1, 2 * g - 2);
    };
    int g = 0;
    for (; g + 4 <= S; g += 4) {
      cstep(IC<0>{}, g);
      cstep(IC<1>{}, g + 1);
      cstep(IC<2>{}, g + 2);
      cstep(IC<3>{}, g + 3);
    }
    if (g < S) cstep(IC<0>{}, g);
    if (g + 1 < S) cstep(IC<1>{}, g + 1);
    if (g + 2 < S) cstep(IC<2>{}, g + 2);
#ifdef SPECENH_D3_STATS
    clk.flush(wv);
#endif
  }
}

}  // namespace
}  // namespace specenh

using namespace specenh;

namespace {
// the row sweep over bands of output rows per image: one band (no recomputed halo rows)
// unless the batch leaves fewer than 2 workgroups per CU
template <bool TRAIN>
int launch_tail_rows(int dtype, RowsArgs& r, hipStream_t st) {
  const int N = r.N, H = r.H;
  int nb = 1;
  while (nb < 8 && (long long)N * nb < 2ll * device_cus() && 2 * H / (2 * nb) >= 8) nb *= 2;
  r.R = ((2 * H + nb - 1) / nb + 1) & ~1;
  r.nb = (2 * H + r.R - 1) / r.R;
  const long long grid = (long long)N * r.nb;
  if (grid >= (1ll << 31)) return set_error(SPECENH_EINVAL, "too many workgroups");
  if (dtype == SPECENH_DTYPE_F16)
    SPECENH_LAUNCH((tail_rows_kernel<_Float16, TRAIN>), dim3((unsigned)grid), dim3(256), rows::LDS_BYTES, st, r);
  else
    SPECENH_LAUNCH((tail_rows_kernel<__bf16, TRAIN>), dim3((unsigned)grid), dim3(256), rows::LDS_BYTES, st, r);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(SPECENH_EHIP, std::string("tail_rows: ") + hipGetErrorString(e));
  return SPECENH_OK;
}
}  // namespace

extern "C" int specenh_convt_conv_out_train(int dtype, const void* x, int N, int H, int W, int C,
                                            const void* wt_gemm, const float* bt, int CO_, int kt,
                                            const void* wo_gemm, const float* bo, int ko,
                                            void* map, float* logits, void* out, void* stream) {
  if (N < 0 || H <= 0 || W <= 0) return set_error(SPECENH_EINVAL, "bad input shape");
  if (dtype != SPECENH_DTYPE_F16 && dtype != SPECENH_DTYPE_BF16)
    return set_error(SPECENH_EUNSUPPORTED, "fused decoder tail: fp16 / bf16 only");
  if (C != CI || CO_ != CO || kt != KT || ko != KO || W != rows::QW)
    return set_error(SPECENH_EUNSUPPORTED,
                     "fused decoder tail (training): Conv2DTranspose(16, 5) on 64-wide "
                     "32-channel inputs + Conv2D(1, 5)");
  if (N == 0) return SPECENH_OK;
  if (!x || !wt_gemm || !bt || !wo_gemm || !bo || !map || !logits || !out)
    return set_error(SPECENH_EINVAL, "null pointer");
  if ((long long)N * H * W * C >= (1ll << 31) || (long long)N * 4 * H * W * CO >= (1ll << 31))
    return set_error(SPECENH_EINVAL, "tensor too large (2^31 elements)");
  RowsArgs r{};
  r.x = x; r.wt = wt_gemm; r.bt = bt; r.wo = wo_gemm; r.bo = bo;
  r.map = map; r.logits = logits; r.out_t = out;
  r.N = N; r.H = H;
  return launch_tail_rows<true>(dtype, r, (hipStream_t)stream);
}

namespace specenh {
// tail_rows_g.hip: the reference's other autoencoders' tails (CO = 32, k = 3 / 5 / 7)
bool tail_rows_general_supported(int C, int CO, int kt, int ko, int W);
int tail_rows_general(int dtype, const void* x, int N, int H, int W, int C, const void* wt,
                      const float* bt, int CO, int kt, const void* wo, const float* bo, int ko,
                      float* out, hipStream_t st, bool* launched);
}  // namespace specenh

extern "C" int specenh_convt_conv_out(int dtype, const void* x, int N, int H, int W, int C,
                                      const void* wt_gemm, const float* bt, int CO_, int kt,
                                      const void* wo_gemm, const float* bo, int ko, float* out,
                                      void* stream) {
  if (N < 0 || H <= 0 || W <= 0) return set_error(SPECENH_EINVAL, "bad input shape");
  if (dtype != SPECENH_DTYPE_F16 && dtype != SPECENH_DTYPE_BF16)
    return set_error(SPECENH_EUNSUPPORTED, "fused decoder tail: fp16 / bf16 only");
  hipStream_t st = (hipStream_t)stream;
  if (tail_rows_general_supported(C, CO_, kt, ko, W)) {
    if (N == 0) return SPECENH_OK;
    bool launched = false;
    const int rc = tail_rows_general(dtype, x, N, H, W, C, wt_gemm, bt, CO_, kt, wo_gemm, bo, ko,
                                     out, st, &launched);
    if (rc != SPECENH_OK || launched) return rc;
  }
  if (C != CI || CO_ != CO || kt != KT || ko != KO)
    return set_error(SPECENH_EUNSUPPORTED,
                     "fused decoder tail: Conv2DTranspose(16, 5) on 32 channels + Conv2D(1, 5), "
                     "or Conv2DTranspose(32, k) + Conv2D(1, k), k = 3 / 5 / 7, on 64-wide inputs");
  if (N == 0) return SPECENH_OK;
  if (W == rows::QW && variant(V_TAIL_TILES) == 0) {  // the row-sweep kernel
    if (!x || !wt_gemm || !bt || !wo_gemm || !bo || !out) return set_error(SPECENH_EINVAL, "null pointer");
    if ((long long)N * H * W * C >= (1ll << 31) || (long long)N * 4 * H * W >= (1ll << 31))
      return set_error(SPECENH_EINVAL, "tensor too large (2^31 elements)");
    RowsArgs r{};
    r.x = x; r.wt = wt_gemm; r.bt = bt; r.wo = wo_gemm; r.bo = bo; r.out = out;
    r.N = N; r.H = H;
    return launch_tail_rows<false>(dtype, r, st);
  }
  if (!x || !wt_gemm || !bt || !wo_gemm || !bo || !out) return set_error(SPECENH_EINVAL, "null pointer");
  if ((long long)N * H * W * C >= (1ll << 31) || (long long)N * 4 * H * W >= (1ll << 31))
    return set_error(SPECENH_EINVAL, "tensor too large (2^31 elements)");
  TailArgs a{};
  a.x = x;
  a.wt = wt_gemm;
  a.bt = bt;
  a.wo = wo_gemm;
  a.bo = bo;
  a.out = out;
  a.N = N;
  a.H = H;
  a.W = W;
  a.tiles_y = (2 * H + TO - 1) / TO;
  a.tiles_x = (2 * W + TO - 1) / TO;
  const long long tiles = (long long)N * a.tiles_y * a.tiles_x;
  if (tiles >= (1ll << 31)) return set_error(SPECENH_EINVAL, "too many tiles");
  const unsigned grid = (unsigned)std::min<long long>(tiles, resident_grid());
  if (dtype == SPECENH_DTYPE_F16)
    SPECENH_LAUNCH(convt_conv_out_kernel<_Float16>, dim3(grid), dim3(512), 0, st, a);
  else
    SPECENH_LAUNCH(convt_conv_out_kernel<__bf16>, dim3(grid), dim3(512), 0, st, a);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(SPECENH_EHIP, std::string("convt_conv_out: ") +
                                                          hipGetErrorString(e));
  return SPECENH_OK;
}

#ifdef SPECENH_D3_STATS
extern "C" int specenh_d3_stats(void* host, int bytes) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(d3_stats), bytes) == hipSuccess ? 0 : -1;
}
#endif

extern "C" int specenh_decoder3_ex(int dtype, const void* x, int N, int H, int W, int C,
                                   const void* w1_gemm, const float* b1, int CO1,
                                   const void* wt_gemm, const float* bt, int CO2,
                                   const void* wo_gemm, const float* bo, int k, void* out,
                                   int out_dtype, void* stream) {
  if (out_dtype != SPECENH_DTYPE_F32 && out_dtype != SPECENH_DTYPE_F16)
    return set_error(SPECENH_EUNSUPPORTED, "fused decoder: fp32 or fp16 output");
  if (N < 0 || H <= 0 || W <= 0) return set_error(SPECENH_EINVAL, "bad input shape");
  if (dtype != SPECENH_DTYPE_F16 && dtype != SPECENH_DTYPE_BF16)
    return set_error(SPECENH_EUNSUPPORTED, "fused decoder: fp16 / bf16 only");
  if (W != d3::W1 || C != d3::CI1 || CO1 != d3::CO1 || CO2 != CO || k != KT)
    return set_error(SPECENH_EUNSUPPORTED,
                     "fused decoder: Conv2DTranspose(32, 5) on 32-wide 64-channel inputs + "
                     "Conv2DTranspose(16, 5) + Conv2D(1, 5)");
  if (N == 0) return SPECENH_OK;
  if (!x || !w1_gemm || !b1 || !wt_gemm || !bt || !wo_gemm || !bo || !out)
    return set_error(SPECENH_EINVAL, "null pointer");
  if ((long long)N * H * W * C >= (1ll << 31) || (long long)N * 16 * H * W >= (1ll << 31))
    return set_error(SPECENH_EINVAL, "tensor too large (2^31 elements)");
  D3Args a{};
  a.x = x; a.w1 = w1_gemm; a.b1 = b1; a.wt = wt_gemm; a.bt = bt; a.wo = wo_gemm; a.bo = bo;
  a.out = out; a.N = N; a.H = H;
  a.out_f16 = out_dtype == SPECENH_DTYPE_F16;
  hipStream_t st = (hipStream_t)stream;
  // (the kernels are named here, outside the lambda, so the device compilation instantiates
  // them)
  const void* const k16 = reinterpret_cast<const void*>(&decoder3_kernel<_Float16, true, 0>);
  const void* const kb16 = reinterpret_cast<const void*>(&decoder3_kernel<__bf16, true, 0>);
  static std::once_flag attr_once;
  std::call_once(attr_once, [k16, kb16] {
    (void)hipFuncSetAttribute(k16, hipFuncAttributeMaxDynamicSharedMemorySize, d3::LDS_BYTES);
    (void)hipFuncSetAttribute(kb16, hipFuncAttributeMaxDynamicSharedMemorySize, d3::LDS_BYTES);
    const void* const nm[8] = {
        reinterpret_cast<const void*>(&decoder3_kernel<_Float16, false, 3>),
        reinterpret_cast<const void*>(&decoder3_kernel<__bf16, false, 3>),
        reinterpret_cast<const void*>(&decoder3_kernel<_Float16, false, 0>),
        reinterpret_cast<const void*>(&decoder3_kernel<__bf16, false, 0>),
        reinterpret_cast<const void*>(&decoder3_kernel<_Float16, false, 3, true>),
        reinterpret_cast<const void*>(&decoder3_kernel<__bf16, false, 3, true>),
        reinterpret_cast<const void*>(&decoder3_kernel<_Float16, false, 0, true>),
        reinterpret_cast<const void*>(&decoder3_kernel<__bf16, false, 0, true>)};
    for (const void* k : nm)
      (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, d3::LDS_BYTES_NM);
  });
  // persistent: one workgroup per CU (256 VGPRs at 2 waves per SIMD; 68 KB of LDS, 120 KB with
  // the map ring)
  const unsigned grid = (unsigned)std::min<long long>(N, device_cus());
  const bool map = variant(V_D3_MAP) != 0, short_lead = variant(V_ROWS_SHORT_LEAD) != 0;
  if (map && a.out_f16)
    return set_error(SPECENH_EUNSUPPORTED, "fused decoder: the map consumer stores fp32 only");
  const dim3 gd(grid), bd(512);
  // the map-free kernels by (input dtype, output dtype) as a compile-time pair
  auto launch_nm = [&](auto t, auto o16) {
    using TT = decltype(t);
    constexpr bool O16 = decltype(o16)::value;
    if (short_lead)
      SPECENH_LAUNCH((decoder3_kernel<TT, false, 0, O16>), gd, bd, d3::LDS_BYTES_NM, st, a);
    else
      SPECENH_LAUNCH((decoder3_kernel<TT, false, 3, O16>), gd, bd, d3::LDS_BYTES_NM, st, a);
  };
  using F16OUT = std::integral_constant<bool, true>;
  using F32OUT = std::integral_constant<bool, false>;
  if (dtype == SPECENH_DTYPE_F16) {
    if (map)
      SPECENH_LAUNCH((decoder3_kernel<_Float16, true, 0>), gd, bd, d3::LDS_BYTES, st, a);
    else if (a.out_f16)
      launch_nm(_Float16{}, F16OUT{});
    else
      launch_nm(_Float16{}, F32OUT{});
  } else {
    if (map)
      SPECENH_LAUNCH((decoder3_kernel<__bf16, true, 0>), gd, bd, d3::LDS_BYTES, st, a);
    else if (a.out_f16)
      launch_nm(__bf16{}, F16OUT{});
    else
      launch_nm(__bf16{}, F32OUT{});
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(SPECENH_EHIP, std::string("decoder3: ") + hipGetErrorString(e));
  return SPECENH_OK;
}

extern "C" int specenh_decoder3(int dtype, const void* x, int N, int H, int W, int C,
                                const void* w1_gemm, const float* b1, int CO1, const void* wt_gemm,
                                const float* bt, int CO2, const void* wo_gemm, const float* bo,
                                int k, float* out, void* stream) {
  return specenh_decoder3_ex(dtype, x, N, H, W, C, w1_gemm, b1, CO1, wt_gemm, bt, CO2, wo_gemm, bo,
                             k, out, SPECENH_DTYPE_F32, stream);
}
