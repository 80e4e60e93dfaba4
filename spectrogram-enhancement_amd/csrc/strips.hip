// strips.hip — the strip glue between the spectrogram and the autoencoder.
//
// Reference (VAE/manual_scan_3layers.py:28-54):
//   patch:   patchify(S, (256, 128), step=128)[0][x], x < 30  ==  S[:256, 128x : 128x+128]
//   unpatch: unpatchify of 30 strips back to (256, 3840)
//   reshape: (N, 256, 128) -> (N, 256, 128, 1)
// On the GPU the three are one strided copy each way; pack also casts to the AE's compute
// dtype, so specgr's fp32 output becomes the AE's NHWC (C = 1) input in one pass.
// Each thread moves 4 consecutive columns (16-byte fp32 loads when aligned).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>

#include "specenh.h"
#include "runtime.hpp"

namespace specenh {
int set_error(int code, const std::string& msg);  // stft_psd.hip

namespace {

__device__ __forceinline__ void put(float* p, float v) { *p = v; }
__device__ __forceinline__ void put(__bf16* p, float v) { *p = (__bf16)v; }
__device__ __forceinline__ void put(_Float16* p, float v) { *p = (_Float16)v; }
__device__ __forceinline__ float get(const float* p) { return *p; }
__device__ __forceinline__ float get(const __bf16* p) { return (float)*p; }
__device__ __forceinline__ float get(const _Float16* p) { return (float)*p; }

// out[(b*n + x)][r][c] = S[b][r][x*width + c]
template <typename TD>
__global__ void pack_kernel(const float* __restrict__ S, long long batch, int T, long long s_stride,
                            int rows, int width, int n, TD* __restrict__ out) {
  const int qw = width / 4;  // quads per strip row
  const long long total = batch * n * rows * qw;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int q = (int)(i % qw);
    long long t = i / qw;
    const int r = (int)(t % rows);
    t /= rows;
    const int x = (int)(t % n);
    const long long b = t / n;
    const float* src = S + b * s_stride + (long long)r * T + (long long)x * width + 4 * q;
    TD* dst = out + ((b * n + x) * rows + r) * (long long)width + 4 * q;
#pragma unroll
    for (int j = 0; j < 4; ++j) put(dst + j, src[j]);
  }
}

// out[b][r][x*width + c] = strips[(b*n + x)][r][c]
template <typename TS>
__global__ void unpack_kernel(const TS* __restrict__ strips, long long batch, int rows, int width,
                              int n, float* __restrict__ out) {
  const int qw = width / 4;
  const long long total = batch * n * rows * qw;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int q = (int)(i % qw);
    long long t = i / qw;
    const int r = (int)(t % rows);
    t /= rows;
    const int x = (int)(t % n);
    const long long b = t / n;
    const TS* src = strips + ((b * n + x) * rows + r) * (long long)width + 4 * q;
    float* dst = out + (b * rows + r) * (long long)n * width + (long long)x * width + 4 * q;
#pragma unroll
    for (int j = 0; j < 4; ++j) dst[j] = get(src + j);
  }
}

unsigned blocks_for(long long n) {
  return (unsigned)std::max<long long>(1, std::min<long long>((n + 255) / 256, 1 << 16));
}

}  // namespace
}  // namespace specenh

using namespace specenh;

extern "C" {

int specenh_strips_pack(int dst_dtype, const float* S, long long batch, int F, int T,
                        long long s_stride, int rows, int width, int n_strips, void* out,
                        void* stream) {
  if (!S || !out || batch <= 0 || rows <= 0 || width <= 0 || n_strips <= 0)
    return set_error(SPECENH_EINVAL, "strips_pack: bad arguments");
  if (rows > F || (long long)n_strips * width > T || s_stride < (long long)F * T)
    return set_error(SPECENH_EINVAL, "strips_pack: strips exceed the spectrogram");
  if (width % 4) return set_error(SPECENH_EUNSUPPORTED, "strips_pack: width % 4 != 0");
  const long long total = batch * n_strips * rows * (width / 4);
  hipStream_t st = (hipStream_t)stream;
  if (dst_dtype == SPECENH_DTYPE_F32)
    SPECENH_LAUNCH(pack_kernel<float>, dim3(blocks_for(total)), dim3(256), 0, st, S, batch, T,
                       s_stride, rows, width, n_strips, (float*)out);
  else if (dst_dtype == SPECENH_DTYPE_BF16)
    SPECENH_LAUNCH(pack_kernel<__bf16>, dim3(blocks_for(total)), dim3(256), 0, st, S, batch,
                       T, s_stride, rows, width, n_strips, (__bf16*)out);
  else if (dst_dtype == SPECENH_DTYPE_F16)
    SPECENH_LAUNCH(pack_kernel<_Float16>, dim3(blocks_for(total)), dim3(256), 0, st, S,
                       batch, T, s_stride, rows, width, n_strips, (_Float16*)out);
  else
    return set_error(SPECENH_EINVAL, "strips_pack: dtype");
  return hipGetLastError() == hipSuccess ? SPECENH_OK : set_error(SPECENH_EHIP, "strips_pack");
}

int specenh_strips_unpack(int src_dtype, const void* strips, long long batch, int rows, int width,
                          int n_strips, float* out, void* stream) {
  if (!strips || !out || batch <= 0 || rows <= 0 || width <= 0 || n_strips <= 0)
    return set_error(SPECENH_EINVAL, "strips_unpack: bad arguments");
  if (width % 4) return set_error(SPECENH_EUNSUPPORTED, "strips_unpack: width % 4 != 0");
  const long long total = batch * n_strips * rows * (width / 4);
  hipStream_t st = (hipStream_t)stream;
  if (src_dtype == SPECENH_DTYPE_F32)
    SPECENH_LAUNCH(unpack_kernel<float>, dim3(blocks_for(total)), dim3(256), 0, st,
                       (const float*)strips, batch, rows, width, n_strips, out);
  else if (src_dtype == SPECENH_DTYPE_BF16)
    SPECENH_LAUNCH(unpack_kernel<__bf16>, dim3(blocks_for(total)), dim3(256), 0, st,
                       (const __bf16*)strips, batch, rows, width, n_strips, out);
  else if (src_dtype == SPECENH_DTYPE_F16)
    SPECENH_LAUNCH(unpack_kernel<_Float16>, dim3(blocks_for(total)), dim3(256), 0, st,
                       (const _Float16*)strips, batch, rows, width, n_strips, out);
  else
    return set_error(SPECENH_EINVAL, "strips_unpack: dtype");
  return hipGetLastError() == hipSuccess ? SPECENH_OK : set_error(SPECENH_EHIP, "strips_unpack");
}

}  // extern "C"
