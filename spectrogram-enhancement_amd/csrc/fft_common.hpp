// fft_common.hpp — in-register FFT building blocks for gfx950 (wave64).
//
// A radix-R DFT whose R points live in one lane's VGPRs, fully unrolled, with
// every twiddle a compile-time constant (computed by constexpr double-precision
// trig below, rounded once to fp32). Trivial twiddles (1, -i, (1-i)/sqrt2, ...)
// are special-cased at compile time so no multiply is emitted for them.
#pragma once

#include <hip/hip_runtime.h>

namespace specenh {

// ----------------------------------------------------------------- constexpr trig
namespace ct {
constexpr double kPi = 3.14159265358979323846264338327950288;

constexpr double taylor_sin(double x) {  // |x| <= pi/4
  double x2 = x * x, term = x, sum = x;
  for (int n = 1; n < 14; ++n) {
    term *= -x2 / ((2.0 * n) * (2.0 * n + 1.0));
    sum += term;
  }
  return sum;
}
constexpr double taylor_cos(double x) {  // |x| <= pi/4
  double x2 = x * x, term = 1.0, sum = 1.0;
  for (int n = 1; n < 14; ++n) {
    term *= -x2 / ((2.0 * n - 1.0) * (2.0 * n));
    sum += term;
  }
  return sum;
}
// cos / sin of 2*pi*k/M with exact octant reduction (k, M integers).
struct CS {
  double c, s;
};
constexpr CS cossin_frac(long long k, long long M) {
  k %= M;
  if (k < 0) k += M;
  // 8k = q*M + r, angle = (q*M + r) * pi / (4M) = q*pi/4 + r*pi/(4M)
  long long q = (8 * k) / M;
  long long r = 8 * k - q * M;  // 0 <= r < M
  double a = kPi * double(r) / (4.0 * double(M));  // in [0, pi/4)
  double c0 = taylor_cos(a), s0 = taylor_sin(a);
  // rotate by q * 45 degrees
  const double h = 0.70710678118654752440084436210484903;
  double c = c0, s = s0;
  switch (q & 7) {
    case 0: c = c0; s = s0; break;
    case 1: c = h * (c0 - s0); s = h * (c0 + s0); break;
    case 2: c = -s0; s = c0; break;
    case 3: c = -h * (c0 + s0); s = h * (c0 - s0); break;
    case 4: c = -c0; s = -s0; break;
    case 5: c = -h * (c0 - s0); s = -h * (c0 + s0); break;
    case 6: c = s0; s = -c0; break;
    default: c = h * (c0 + s0); s = -h * (c0 - s0); break;
  }
  // exact values at multiples of 45 degrees
  if (r == 0) {
    const double ex_c[8] = {1.0, h, 0.0, -h, -1.0, -h, 0.0, h};
    const double ex_s[8] = {0.0, h, 1.0, h, 0.0, -h, -1.0, -h};
    c = ex_c[q & 7];
    s = ex_s[q & 7];
  }
  return CS{c, s};
}
}  // namespace ct

// Forward DFT twiddle W_M^k = exp(-2*pi*i*k/M) as fp32 constants.
template <int M>
struct Twiddles {
  float re[M > 1 ? M : 1];
  float im[M > 1 ? M : 1];
  constexpr Twiddles() : re{}, im{} {
    for (int k = 0; k < M; ++k) {
      ct::CS cs = ct::cossin_frac(k, M);
      re[k] = float(cs.c);
      im[k] = float(-cs.s);
    }
  }
};

constexpr int ilog2(int n) { return n <= 1 ? 0 : 1 + ilog2(n >> 1); }
constexpr int bitrev(int v, int bits) {
  int r = 0;
  for (int i = 0; i < bits; ++i) r |= ((v >> i) & 1) << (bits - 1 - i);
  return r;
}

__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmul(float2 a, float2 w) {
  return make_float2(fmaf(a.x, w.x, -a.y * w.y), fmaf(a.x, w.y, a.y * w.x));
}

// ------------------------------------------------------------ complex arithmetic
// A complex value as a two-float vector {re, im}. The library is built without packed
// fp32 codegen (build.py: on CDNA4 a v_pk_*_f32 issues as two scalar ops and only adds
// register-pair moves), so these are plain scalar VALU ops; rotations by -i are free
// (operand renaming).
typedef float f2v __attribute__((ext_vector_type(2)));

namespace pk {
__device__ __forceinline__ f2v add(f2v a, f2v b) { return a + b; }
__device__ __forceinline__ f2v sub(f2v a, f2v b) { return a - b; }
// -i (a - b) = (a.y - b.y, b.x - a.x)
__device__ __forceinline__ f2v sub_mi(f2v a, f2v b) { return f2v{a.y - b.y, b.x - a.x}; }
__device__ __forceinline__ f2v cmul(f2v d, f2v w) {
  return f2v{fmaf(d.x, w.x, -d.y * w.y), fmaf(d.x, w.y, d.y * w.x)};
}
}  // namespace pk

// In-register radix-2 DIF butterflies of one stage (span H), unrolled by recursion; the
// difference's twiddle W_{2H}^K is a compile-time constant (1 and -i cost nothing extra).
template <int R, int H, int S, int K>
struct DifStage {
  __device__ __forceinline__ static void run(f2v (&v)[R]) {
    if constexpr (S < R) {
      if constexpr (K < H) {
        constexpr int M = 2 * H;
        const f2v a = v[S + K], b = v[S + K + H];
        v[S + K] = pk::add(a, b);
        if constexpr (K == 0) {
          v[S + K + H] = pk::sub(a, b);
        } else if constexpr (4 * K == M) {
          v[S + K + H] = pk::sub_mi(a, b);
        } else {
          constexpr Twiddles<M> tw{};
          v[S + K + H] = pk::cmul(pk::sub(a, b), f2v{tw.re[K], tw.im[K]});
        }
        DifStage<R, H, S, K + 1>::run(v);
      } else {
        DifStage<R, H, S + 2 * H, 0>::run(v);
      }
    }
  }
};

template <int R, int H>
struct DifAll {
  __device__ __forceinline__ static void run(f2v (&v)[R]) {
    if constexpr (H >= 1) {
      DifStage<R, H, 0, 0>::run(v);
      DifAll<R, H / 2>::run(v);
    }
  }
};

// Radix-R forward DFT in registers. Input natural order; on return v[r] holds
// output bin bitrev(r) (log2 R bits) — callers fold that permutation into their
// store addresses at compile time.
template <int R>
__device__ __forceinline__ void fft_dif(f2v (&v)[R]) {
  DifAll<R, R / 2>::run(v);
}

// Wave-scope ordering point between LDS phases of one wave-resident FFT:
// keeps the compiler from moving LDS accesses across it and waits for them.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Order-preserving float <-> uint32 key (for atomic min/max of floats).
__device__ __forceinline__ unsigned f2key(float f) {
  unsigned b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float key2f(unsigned k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

}  // namespace specenh
