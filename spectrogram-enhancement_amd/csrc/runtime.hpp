// runtime.hpp — host-side runtime shared by the kernel files: kernel-variant switches,
// the per-device CU count for persistent grids, and the record of the last launched kernel.
//
// Variant switches select between kernels that compute the same result (A/B tests and the
// per-layer tools). They are read from the environment ONCE per process (SPECENH_<NAME>,
// first use) and can be changed afterwards only through specenh_set_variant() — a launch
// reads one atomic, never the environment.
#pragma once

#include <hip/hip_runtime.h>

namespace specenh {

enum Variant : int {
  V_CONVT_PAIR = 0,   // Conv2DTranspose forward in (tile, row-phase) workgroups (opt-in)
  V_PATCH_NO_WL,      // 16-channel conv: weights from the L2 ring instead of LDS
  V_PATCH_NO_K5,      // 16-channel conv: no compile-time 5x5 taps / persistent grid
  V_PATCH_WSPLIT,     // 2x2 wave split: -1 auto (default), 0 off, 1 forced
  V_CONV_NO_S2,       // stride-2 conv: generic gather kernel instead of the S2 patch kernel
  V_CONV_NO_PATCH,    // every conv through the generic gather kernel
  V_CONV_NO_C1MFMA,   // C = 1 conv on the VALU kernel instead of MFMA
  V_CONV_NO_NARROW,   // no VALU narrow kernels (1 in / 1 out channel)
  V_WGRAD_GENERIC,    // weight gradients through the generic gather kernel
  V_WGRAD_NO_CO1,     // CO = 1 weight gradient through the general MFMA kernel
  V_WGRAD_PERPHASE,   // Conv2DTranspose weight gradient one phase per workgroup
  V_SVD_GRAM_TILES,   // Gram matrix through the triangle-tile kernel instead of LDS rows
  V_TAIL_TILES,       // fused decoder tail: 2-D tile kernel instead of the row sweep
  V_DECODER_UNFUSED,  // engine (Python): no three-layer decoder launch (specenh_decoder3)
  V_SVD_NO_TOP1,      // default kept range [1, r): Gram + subspace + recon instead of top1_kernel
  V_CONV_NO_ROWS,     // pooled encoder convs: conv_patch_kernel tiles instead of the row sweep
  V_CONVT_NO_ROWS,    // Conv2DTranspose on 64 channels: conv_patch_kernel instead of the row sweep
  V_CONV1_NO_ROWS,    // C = 1 pooled conv: conv_c1_mfma tiles instead of the row sweep
  V_ENCODER_UNFUSED,  // engine (Python): no two-layer encoder launch (specenh_encoder2)
  V_STFT_NO_HOLD,     // per-shot normalised STFT: raw rows + re-read sweep, not held tiles
  V_D3_MAP,           // decoder3: Conv2D(1) from a 16-channel map ring in LDS (round-3 consumer)
  V_ENC2_WPE2,        // fused encoder: one workgroup per CU (256 VGPRs) instead of two
  V_CONVT_SHARED_RING, // convT1 row sweep: one shared input ring + per-step barrier (round 3)
  V_SVD_RECON_VALU,   // SVD reconstruction with scalar FMAs (round 3) instead of fp32 MFMA
  V_ROWS_SHORT_LEAD,  // convT rows / decoder3 producer: the round-3 ring refill lead (1 / 0 steps, not 3)
  V_SVD_GRAM_F32,     // 128 < r <= 256 Gram on fp32 MFMA (round 3) instead of the fp16 hi/lo split
  V_SVD_RECON_BLOCKS, // SVD reconstruction one workgroup per row block (recon_mfma_kernel), not runs
  V_CONVT_PG,         // convT1 row sweep: phases split over 8 waves (round 5 trial, slower) instead of 4 x 50 taps
  V_SVD_GZ_ROWS,      // subspace G Z one row per thread (round 4) instead of four
  V_EIG_SPLIT,        // flagged-matrix fp64 fallback as four launches instead of one
  V_CO1_VALU,         // one-output-channel conv on 32 channels: VALU dot2 kernel instead of MFMA
  V_C1_MASK_MFMA,     // masked C = 1 conv (C4 input gradient of the last conv) on MFMA (1, round 6) or the VALU (0)
  V_S2_MIN_NT,        // stride-2 input-gradient patch kernel: at least this many 16-channel N tiles
  V_PATCH_MIN_WG,     // patch kernels: fewer output-channel tiles per workgroup until this many workgroups
  V_WGRAD_WG,         // weight-gradient MFMA kernels: workgroups per launch aimed at (tile runs)
  V_WGRAD_C1_TILES,   // one-input-channel weight gradient: at least this many tiles per workgroup
  V_EIG_GRID,         // flagged-matrix fallback: workgroups per launch (<= 0: two per CU)
  V_ROWS_BANDS,       // convT row sweeps: log2 row bands per image (-1: auto, small batches)
  V_COUNT
};

// current value of a switch (0 = the shipped default path; V_PATCH_WSPLIT: -1)
int variant(Variant v);

// CU count of the calling thread's current HIP device, queried once per device
int device_cus();

// record `kernel` (the host stub a launch used) as the calling thread's last launch:
// specenh_last_kernel_name() reports its symbol, so a measurement can key PMC counters by
// the exact kernel it timed
void note_launch(const void* kernel);

}  // namespace specenh

// hipLaunchKernelGGL + note_launch. K may be parenthesised (a template-id with commas).
#define SPECENH_LAUNCH(K, ...)                                        \
  do {                                                                \
    ::specenh::note_launch(reinterpret_cast<const void*>(&K));        \
    hipLaunchKernelGGL(K, __VA_ARGS__);                               \
  } while (0)
