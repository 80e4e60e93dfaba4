// filters.hip — the label-generator helpers of spec_denoising/pipeline_data.py:38-61 on the
// GPU: norm, rescale, meansub and quantfilt over a batch of spectrograms.
//
// Each spectrogram is one rows x cols block (row-major, like the reference's F x T arrays);
// statistics are per spectrogram and accumulated in fp64. T = float or double: the numpy
// API uploads the reference's float64 arrays unchanged, so the double path reproduces
// numpy up to the order of its fp64 sums; elementwise results follow numpy's formulas in T.
// quantfilt's per-column quantile is numpy's 'linear' method exactly: the virtual index
// n*q + (1 - q) - 1 (numpy's alpha = beta = 1 expression, evaluated on the host), the two
// neighbouring order statistics found by stable rank counting in LDS, numpy's two-sided
// _lerp in fp64 (explicitly rounded operations, no contraction), then x < q ? 0 : x.
#include <hip/hip_runtime.h>

#include <cmath>
#include <string>
#include <utility>
#include <vector>

#include "specenh.h"
#include "runtime.hpp"

namespace specenh {
int set_error(int code, const std::string& msg);  // stft_psd.hip

namespace {

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
  return v;
}

__device__ double block_sum(double v, double* red) {
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

__device__ void block_minmax(double& mn, double& mx, double* red) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    mn = fmin(mn, __shfl_xor(mn, m));
    mx = fmax(mx, __shfl_xor(mx, m));
  }
  __syncthreads();
  if ((threadIdx.x & 63) == 0) {
    red[threadIdx.x >> 6] = mn;
    red[4 + (threadIdx.x >> 6)] = mx;
  }
  __syncthreads();
  mn = fmin(fmin(red[0], red[1]), fmin(red[2], red[3]));
  mx = fmax(fmax(red[4], red[5]), fmax(red[6], red[7]));
}

// mean of every row (meansub, :59): one wave per row
template <typename T>
__global__ __launch_bounds__(256) void rowmean_kernel(const T* S, long long batch, int rows,
                                                      int cols, long long stride, double* rm) {
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= batch * rows) return;
  const long long b = row / rows;
  const int r = (int)(row - b * rows);
  const T* p = S + b * stride + (long long)r * cols;
  double acc = 0.0;
  for (int c = threadIdx.x & 63; c < cols; c += 64) acc += (double)p[c];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) rm[row] = acc / (double)cols;
}

// per-spectrogram statistics: NORM {mean, std}; RESCALE {min, max}; MEANSUB {min, max} of
// |x - rowmean| (as T, like numpy's array of that dtype)
template <typename T>
__global__ __launch_bounds__(256) void stats_kernel(const T* S, int rows, int cols,
                                                    long long stride, int op, const double* rm,
                                                    double* stats) {
  __shared__ double red[8];
  const long long b = blockIdx.x;
  const T* s = S + b * stride;
  const long long n = (long long)rows * cols;
  if (op == SPECENH_FILTER_NORM) {
    double acc = 0.0;
    for (long long e = threadIdx.x; e < n; e += 256) acc += (double)s[e];
    const double mean = block_sum(acc, red) / (double)n;
    double a2 = 0.0;
    for (long long e = threadIdx.x; e < n; e += 256) {
      const double d = (double)s[e] - mean;
      a2 += d * d;
    }
    const double var = block_sum(a2, red) / (double)n;
    if (threadIdx.x == 0) {
      stats[2 * b] = mean;
      stats[2 * b + 1] = sqrt(var);
    }
    return;
  }
  double mn = INFINITY, mx = -INFINITY;
  for (long long e = threadIdx.x; e < n; e += 256) {
    double v = (double)s[e];
    if (op == SPECENH_FILTER_MEANSUB)
      v = (double)(T)fabs((double)s[e] - rm[b * rows + e / cols]);
    mn = fmin(mn, v);
    mx = fmax(mx, v);
  }
  block_minmax(mn, mx, red);
  if (threadIdx.x == 0) {
    stats[2 * b] = mn;
    stats[2 * b + 1] = mx;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void apply_kernel(const T* S, T* out, long long batch, int rows,
                                                    int cols, long long stride, int op,
                                                    const double* rm, const double* stats) {
  const long long n = (long long)rows * cols;
  const long long total = batch * n;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < total;
       i += (long long)gridDim.x * 256) {
    const long long b = i / n, e = i - b * n;
    const T x = S[b * stride + e];
    const double s0 = stats[2 * b], s1 = stats[2 * b + 1];
    T y;
    if (op == SPECENH_FILTER_NORM) {  // (data - mn) / std
      y = (T)(x - (T)s0) / (T)s1;
    } else if (op == SPECENH_FILTER_RESCALE) {  // (data - min) / (max - min)
      y = (T)(x - (T)s0) / (T)((T)s1 - (T)s0);
    } else {  // rescale(|src - mn|)
      const T d = (T)fabs((double)x - rm[b * rows + e / cols]);
      y = (T)(d - (T)s0) / (T)((T)s1 - (T)s0);
    }
    out[b * stride + e] = y;
  }
}

constexpr int QF_COLS = 16;  // columns per workgroup

// quantfilt: order statistics lo/hi of each column by stable rank counting, numpy's lerp,
// threshold. Columns of the tile live column-major in LDS.
template <typename T>
__global__ __launch_bounds__(256) void quantfilt_kernel(const T* S, T* out, int rows, int cols,
                                                        long long stride, int lo, int hi,
                                                        double gamma) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  T* col = reinterpret_cast<T*>(smem);  // [QF_COLS][rows]
  __shared__ double sel[QF_COLS][2];
  const long long b = blockIdx.y;
  const int c0 = blockIdx.x * QF_COLS;
  const int nc = min(QF_COLS, cols - c0);
  const T* s = S + b * stride;
  for (int idx = threadIdx.x; idx < rows * QF_COLS; idx += 256) {
    const int r = idx / QF_COLS, c = idx - (idx / QF_COLS) * QF_COLS;
    col[c * rows + r] = c < nc ? s[(long long)r * cols + c0 + c] : (T)0;
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < rows * nc; idx += 256) {
    const int c = idx / rows, i = idx - (idx / rows) * rows;
    const T* v = col + c * rows;
    const T vi = v[i];
    int rank = 0;
    for (int j = 0; j < rows; ++j) {
      const T vj = v[j];
      rank += (vj < vi) || (vj == vi && j < i);
    }
    if (rank == lo) sel[c][0] = (double)vi;
    if (rank == hi) sel[c][1] = (double)vi;
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < rows * nc; idx += 256) {
    const int r = idx / nc, c = idx - (idx / nc) * nc;
    const double a = sel[c][0], bb = sel[c][1];
    const double diff = __dsub_rn(bb, a);  // numpy _lerp, :4653-4657
    const double q = gamma >= 0.5 ? __dsub_rn(bb, __dmul_rn(diff, __dsub_rn(1.0, gamma)))
                                  : __dadd_rn(a, __dmul_rn(diff, gamma));
    const T x = col[c * rows + r];
    out[b * stride + (long long)r * cols + c0 + c] = ((double)x < q) ? (T)0 : x;
  }
}


// ---------------------------------------------------------------- cv2 steps on uint8
// gaussblr (:52-55) and morph (:64-72): the image is quantised to uint8 exactly as
// (rescale(src)*255).astype('uint8') (T arithmetic, truncation), filtered with OpenCV's
// 8-bit algorithms restated (integer arithmetic: Gaussian taps in Q8 summing to 256, rows
// then columns, (v + 2^15) >> 16, BORDER_REFLECT_101; rect dilate/erode with the anchor at
// k/2 and outside pixels ignored), and rescaled as numpy evaluates rescale() on a uint8
// array: (u - min) / (max - min) as a true (fp64) division. OpenCV is absent, so the
// restatement is oracle/filters.py and parity with cv2 itself is unpinned.
constexpr int MAX_TAPS = 127;
struct GaussTaps {
  int kw, kh;
  unsigned short kx[MAX_TAPS], ky[MAX_TAPS];
};

__device__ __forceinline__ int reflect101(int p, int n) {
  if (n == 1) return 0;
  while (p < 0 || p >= n) {
    if (p < 0) p = -p;
    if (p >= n) p = 2 * n - 2 - p;
  }
  return p;
}

template <typename T>
__global__ __launch_bounds__(256) void quant_u8_kernel(const T* S, long long batch, int rows,
                                                       int cols, long long stride,
                                                       const double* stats, unsigned char* q) {
  const long long n = (long long)rows * cols, total = batch * n;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < total;
       i += (long long)gridDim.x * 256) {
    const long long b = i / n, e = i - b * n;
    const T mn = (T)stats[2 * b], mx = (T)stats[2 * b + 1];
    const T r = (T)((T)(S[b * stride + e] - mn) / (T)(mx - mn)) * (T)255;
    q[i] = (r >= (T)0 && r < (T)256) ? (unsigned char)(int)r : (unsigned char)0;
  }
}

__global__ __launch_bounds__(256) void gauss_rows_kernel(const unsigned char* q, long long batch,
                                                         int rows, int cols, GaussTaps tp,
                                                         unsigned short* h) {
  const long long n = (long long)rows * cols, total = batch * n;
  const int half = tp.kw / 2;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < total;
       i += (long long)gridDim.x * 256) {
    const long long rowbase = i - i % cols;
    const int c = (int)(i - rowbase);
    unsigned acc = 0;
    for (int j = 0; j < tp.kw; ++j)
      acc += (unsigned)tp.kx[j] * q[rowbase + reflect101(c + j - half, cols)];
    h[i] = (unsigned short)acc;  // <= 255 * 256
  }
}

__global__ __launch_bounds__(256) void gauss_cols_kernel(const unsigned short* h, long long batch,
                                                         int rows, int cols, GaussTaps tp,
                                                         unsigned char* o) {
  const long long n = (long long)rows * cols, total = batch * n;
  const int half = tp.kh / 2;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < total;
       i += (long long)gridDim.x * 256) {
    const long long b = i / n, e = i - b * n;
    const int r = (int)(e / cols), c = (int)(e - (long long)r * cols);
    const unsigned short* hb = h + b * n + c;
    unsigned acc = 0;
    for (int k = 0; k < tp.kh; ++k)
      acc += (unsigned)tp.ky[k] * hb[(long long)reflect101(r + k - half, rows) * cols];
    const unsigned v = (acc + (1u << 15)) >> 16;
    o[i] = (unsigned char)(v > 255u ? 255u : v);
  }
}

// rect dilate (IS_MAX) / erode over src(r + i - kh/2, c + j - kw/2); outside pixels ignored
template <bool IS_MAX>
__global__ __launch_bounds__(256) void morph_u8_kernel(const unsigned char* a, long long batch,
                                                       int rows, int cols, int kh, int kw,
                                                       unsigned char* o) {
  const long long n = (long long)rows * cols, total = batch * n;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < total;
       i += (long long)gridDim.x * 256) {
    const long long b = i / n, e = i - b * n;
    const int r = (int)(e / cols), c = (int)(e - (long long)r * cols);
    const unsigned char* ab = a + b * n;
    unsigned v = IS_MAX ? 0u : 255u;
    for (int y = max(r - kh / 2, 0); y < min(r - kh / 2 + kh, rows); ++y)
      for (int x = max(c - kw / 2, 0); x < min(c - kw / 2 + kw, cols); ++x) {
        const unsigned s = ab[(long long)y * cols + x];
        v = IS_MAX ? max(v, s) : min(v, s);
      }
    o[i] = (unsigned char)v;
  }
}

__global__ __launch_bounds__(256) void u8_stats_kernel(const unsigned char* u, int rows, int cols,
                                                       double* stats) {
  __shared__ double red[8];
  const long long b = blockIdx.x, n = (long long)rows * cols;
  const unsigned char* s = u + b * n;
  double mn = INFINITY, mx = -INFINITY;
  for (long long e = threadIdx.x; e < n; e += 256) {
    const double v = (double)s[e];
    mn = fmin(mn, v);
    mx = fmax(mx, v);
  }
  block_minmax(mn, mx, red);
  if (threadIdx.x == 0) {
    stats[2 * b] = mn;
    stats[2 * b + 1] = mx;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void u8_rescale_kernel(const unsigned char* u, long long batch,
                                                         int rows, int cols, long long stride,
                                                         const double* stats, T* out) {
  const long long n = (long long)rows * cols, total = batch * n;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < total;
       i += (long long)gridDim.x * 256) {
    const long long b = i / n, e = i - b * n;
    const double mn = stats[2 * b], mx = stats[2 * b + 1];
    out[b * stride + e] = (T)(((double)u[i] - mn) / (mx - mn));
  }
}

inline unsigned grid_for(long long n) {
  const long long g = (n + 255) / 256;
  return (unsigned)(g < 1 ? 1 : (g > 65536 ? 65536 : g));
}

template <typename T>
int run_filter(int op, const T* S, long long batch, int rows, int cols, long long stride, T* out,
               double* ws, hipStream_t st) {
  double* stats = ws;
  double* rm = ws + 2 * batch;
  if (op == SPECENH_FILTER_MEANSUB)
    SPECENH_LAUNCH(rowmean_kernel<T>, dim3(grid_for(batch * rows * 64)), dim3(256), 0, st, S,
                       batch, rows, cols, stride, rm);
  SPECENH_LAUNCH(stats_kernel<T>, dim3((unsigned)batch), dim3(256), 0, st, S, rows, cols,
                     stride, op, rm, stats);
  SPECENH_LAUNCH(apply_kernel<T>, dim3(grid_for(batch * rows * cols)), dim3(256), 0, st, S,
                     out, batch, rows, cols, stride, op, rm, stats);
  return hipGetLastError() == hipSuccess ? SPECENH_OK : set_error(SPECENH_EHIP, "filter launch");
}

template <typename T>
int run_quantfilt(const T* S, long long batch, int rows, int cols, long long stride, int lo,
                  int hi, double gamma, T* out, hipStream_t st) {
  const size_t lds = (size_t)rows * QF_COLS * sizeof(T);
  if (hipFuncSetAttribute((const void*)quantfilt_kernel<T>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
    return set_error(SPECENH_EHIP, "quantfilt attribute");
  for (long long b0 = 0; b0 < batch; b0 += 65535) {
    const long long nb = std::min<long long>(65535, batch - b0);
    SPECENH_LAUNCH(quantfilt_kernel<T>, dim3((cols + QF_COLS - 1) / QF_COLS, (unsigned)nb),
                       dim3(256), lds, st, S + b0 * stride, out + b0 * stride, rows, cols, stride,
                       lo, hi, gamma);
  }
  return hipGetLastError() == hipSuccess ? SPECENH_OK
                                         : set_error(SPECENH_EHIP, "quantfilt launch");
}


// OpenCV's 8-bit Gaussian taps (oracle/filters.py gaussian_taps_q8): sigma from ksize when
// sigma <= 0, fixed small tables for n <= 7, normalise, Q8 by error diffusion with the
// centre tap taking the remainder (sum exactly 256).
int gauss_taps_q8(int n, double sigma, unsigned short* out) {
  if (n < 1 || n % 2 != 1 || n > MAX_TAPS)
    return set_error(SPECENH_EINVAL, "Gaussian kernel size must be odd, positive and <= 127");
  static const double small[4][7] = {{1.0},
                                     {0.25, 0.5, 0.25},
                                     {0.0625, 0.25, 0.375, 0.25, 0.0625},
                                     {0.03125, 0.109375, 0.21875, 0.28125, 0.21875, 0.109375,
                                      0.03125}};
  std::vector<double> k(n);
  const int half = n / 2;
  if (n <= 7 && sigma <= 0) {
    for (int i = 0; i < n; ++i) k[i] = small[half][i];
  } else {
    const double s = sigma > 0 ? sigma : ((n - 1) * 0.5 - 1) * 0.3 + 0.8;
    const double scale2 = -0.5 / (s * s);
    double tot = 0.0;
    for (int i = 0; i < half; ++i) {
      const double x = i - (n - 1) * 0.5;
      k[i] = std::exp(scale2 * x * x);
      tot += k[i];
    }
    tot = 2.0 * tot + 1.0;
    for (int i = 0; i < half; ++i) k[i] /= tot;
    k[half] = 1.0 / tot;
  }
  double err = 0.0;
  int sum = 0;
  for (int i = 0; i < half; ++i) {
    const double adj = k[i] * 256.0 + err;
    const int q = (int)std::nearbyint(adj);
    err = adj - q;
    out[i] = out[n - 1 - i] = (unsigned short)q;
    sum += q;
  }
  out[half] = (unsigned short)(256 - 2 * sum);
  return SPECENH_OK;
}

struct U8Work {
  double* stats;
  unsigned char* a;
  unsigned char* b;
  unsigned short* h;
};

inline U8Work u8_work(void* ws, long long batch, long long n) {
  char* p = (char*)ws;
  U8Work w;
  w.stats = (double*)p;
  p += ((size_t)batch * 16 + 255) / 256 * 256;
  w.h = (unsigned short*)p;
  p += ((size_t)n * 2 + 255) / 256 * 256;
  w.a = (unsigned char*)p;
  p += ((size_t)n + 255) / 256 * 256;
  w.b = (unsigned char*)p;
  return w;
}

template <typename T>
int run_u8_filter(bool gauss, const T* S, long long batch, int rows, int cols, long long stride,
                  const GaussTaps* tp, T* out, void* ws, hipStream_t st) {
  const long long n = batch * rows * cols;
  U8Work w = u8_work(ws, batch, n);
  const unsigned g = grid_for(n);
  SPECENH_LAUNCH(stats_kernel<T>, dim3((unsigned)batch), dim3(256), 0, st, S, rows, cols,
                     stride, (int)SPECENH_FILTER_RESCALE, (const double*)nullptr, w.stats);
  SPECENH_LAUNCH(quant_u8_kernel<T>, dim3(g), dim3(256), 0, st, S, batch, rows, cols, stride,
                     w.stats, w.a);
  if (gauss) {
    SPECENH_LAUNCH(gauss_rows_kernel, dim3(g), dim3(256), 0, st, w.a, batch, rows, cols, *tp,
                       w.h);
    SPECENH_LAUNCH(gauss_cols_kernel, dim3(g), dim3(256), 0, st, w.h, batch, rows, cols, *tp,
                       w.b);
  } else {  // MORPH_CLOSE 4x4 (dilate, erode) then MORPH_OPEN 3x1 (erode, dilate)
    SPECENH_LAUNCH(morph_u8_kernel<true>, dim3(g), dim3(256), 0, st, w.a, batch, rows, cols,
                       4, 4, w.b);
    SPECENH_LAUNCH(morph_u8_kernel<false>, dim3(g), dim3(256), 0, st, w.b, batch, rows, cols,
                       4, 4, w.a);
    SPECENH_LAUNCH(morph_u8_kernel<false>, dim3(g), dim3(256), 0, st, w.a, batch, rows, cols,
                       1, 3, w.b);
    SPECENH_LAUNCH(morph_u8_kernel<true>, dim3(g), dim3(256), 0, st, w.b, batch, rows, cols,
                       1, 3, w.a);
    std::swap(w.a, w.b);
  }
  SPECENH_LAUNCH(u8_stats_kernel, dim3((unsigned)batch), dim3(256), 0, st, w.b, rows, cols,
                     w.stats);
  SPECENH_LAUNCH(u8_rescale_kernel<T>, dim3(g), dim3(256), 0, st, w.b, batch, rows, cols,
                     stride, w.stats, out);
  return hipGetLastError() == hipSuccess ? SPECENH_OK : set_error(SPECENH_EHIP, "u8 filter launch");
}

int check_common(int dtype, const void* S, long long batch, int rows, int cols, long long stride,
                 const void* out) {
  if (dtype != SPECENH_DTYPE_F32 && dtype != SPECENH_DTYPE_F64)
    return set_error(SPECENH_EINVAL, "filters take float32 or float64 spectrograms");
  if (batch < 0 || rows <= 0 || cols <= 0) return set_error(SPECENH_EINVAL, "bad shape");
  if (stride < (long long)rows * cols) return set_error(SPECENH_EINVAL, "stride < rows*cols");
  if (batch > 0 && (!S || !out)) return set_error(SPECENH_EINVAL, "null pointer");
  return SPECENH_OK;
}

}  // namespace
}  // namespace specenh

using namespace specenh;

extern "C" {

size_t specenh_filter_workspace_bytes(long long batch, int rows) {
  if (batch <= 0 || rows <= 0) return 16;
  return (size_t)batch * (2 + (size_t)rows) * sizeof(double);
}

int specenh_filter(int op, int dtype, const void* S, long long batch, int rows, int cols,
                   long long stride, void* out, void* workspace, void* stream) {
  if (int e = check_common(dtype, S, batch, rows, cols, stride, out)) return e;
  if (op != SPECENH_FILTER_NORM && op != SPECENH_FILTER_RESCALE && op != SPECENH_FILTER_MEANSUB)
    return set_error(SPECENH_EINVAL, "unknown filter op");
  if (batch == 0) return SPECENH_OK;
  if (!workspace) return set_error(SPECENH_EINVAL, "null workspace");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == SPECENH_DTYPE_F64)
    return run_filter<double>(op, (const double*)S, batch, rows, cols, stride, (double*)out,
                              (double*)workspace, st);
  return run_filter<float>(op, (const float*)S, batch, rows, cols, stride, (float*)out,
                           (double*)workspace, st);
}

int specenh_quantfilt(int dtype, const void* S, long long batch, int rows, int cols,
                      long long stride, double thr, void* out, void* stream) {
  if (int e = check_common(dtype, S, batch, rows, cols, stride, out)) return e;
  if (!(thr >= 0.0 && thr <= 1.0)) return set_error(SPECENH_EINVAL, "Quantiles must be in the range [0, 1]");
  if ((size_t)rows * QF_COLS * (dtype == SPECENH_DTYPE_F64 ? 8 : 4) > 160 * 1024 - 512)
    return set_error(SPECENH_EUNSUPPORTED, "quantfilt on the GPU needs rows <= 1264");
  if (batch == 0) return SPECENH_OK;
  // numpy 'linear' (alpha = beta = 1): virtual index, neighbours, gamma (_quantile)
  const double vi = (double)rows * thr + (1.0 + thr * (1.0 - 1.0 - 1.0)) - 1.0;
  int lo, hi;
  double gamma;
  if (vi >= rows - 1) {
    lo = hi = rows - 1;
    gamma = 0.0;  // a == b: the lerp returns the maximum
  } else if (vi < 0) {
    lo = hi = 0;
    gamma = 0.0;
  } else {
    const double fl = std::floor(vi);
    lo = (int)fl;
    hi = lo + 1;
    gamma = vi - fl;
  }
  hipStream_t st = (hipStream_t)stream;
  if (dtype == SPECENH_DTYPE_F64)
    return run_quantfilt<double>((const double*)S, batch, rows, cols, stride, lo, hi, gamma,
                                 (double*)out, st);
  return run_quantfilt<float>((const float*)S, batch, rows, cols, stride, lo, hi, gamma,
                              (float*)out, st);
}

size_t specenh_u8filter_workspace_bytes(long long batch, int rows, int cols) {
  if (batch <= 0 || rows <= 0 || cols <= 0) return 16;
  const size_t n = (size_t)batch * rows * cols;
  return ((size_t)batch * 16 + 255) / 256 * 256 + (n * 2 + 255) / 256 * 256 +
         2 * ((n + 255) / 256 * 256);
}

int specenh_gaussblr(int dtype, const void* S, long long batch, int rows, int cols,
                     long long stride, int kw, int kh, double sigma, void* out, void* workspace,
                     void* stream) {
  if (int e = check_common(dtype, S, batch, rows, cols, stride, out)) return e;
  GaussTaps tp{};
  tp.kw = kw;
  tp.kh = kh;
  if (int e = gauss_taps_q8(kw, sigma, tp.kx)) return e;
  if (int e = gauss_taps_q8(kh, sigma, tp.ky)) return e;
  if (batch == 0) return SPECENH_OK;
  if (!workspace) return set_error(SPECENH_EINVAL, "null workspace");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == SPECENH_DTYPE_F64)
    return run_u8_filter<double>(true, (const double*)S, batch, rows, cols, stride, &tp,
                                 (double*)out, workspace, st);
  return run_u8_filter<float>(true, (const float*)S, batch, rows, cols, stride, &tp, (float*)out,
                              workspace, st);
}

int specenh_morph(int dtype, const void* S, long long batch, int rows, int cols, long long stride,
                  void* out, void* workspace, void* stream) {
  if (int e = check_common(dtype, S, batch, rows, cols, stride, out)) return e;
  if (batch == 0) return SPECENH_OK;
  if (!workspace) return set_error(SPECENH_EINVAL, "null workspace");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == SPECENH_DTYPE_F64)
    return run_u8_filter<double>(false, (const double*)S, batch, rows, cols, stride, nullptr,
                                 (double*)out, workspace, st);
  return run_u8_filter<float>(false, (const float*)S, batch, rows, cols, stride, nullptr,
                              (float*)out, workspace, st);
}

}  // extern "C"
