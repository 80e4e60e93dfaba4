// VALU issue-rate microbenchmark (gfx950): cycles per wave64 instruction for v_fma_f32,
// v_pk_fma_f32, v_fma_f64, v_add_f32, v_log_f32, measured with enough waves to fill
// every SIMD. Build: hipcc -O3 --offload-arch=gfx950 -o valu_rate valu_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP 256
#define CH 8

template <int OP>
__global__ __launch_bounds__(256) void k(float* out, int iters) {
  float a[CH];
  double d[CH];
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 p[CH];
  for (int c = 0; c < CH; ++c) {
    a[c] = threadIdx.x * 1e-3f + c;
    d[c] = a[c];
    p[c] = f2{a[c], a[c] + 1};
  }
  const float m = 0.999f, b = 1e-3f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < REP; ++r)
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        if constexpr (OP == 0) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[c]) : "v"(m), "v"(b));
        if constexpr (OP == 1) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(p[c]) : "v"(p[0]), "v"(p[1]));
        if constexpr (OP == 2) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(d[c]) : "v"(d[0]), "v"(d[1]));
        if constexpr (OP == 3) asm volatile("v_add_f32 %0, %0, %1" : "+v"(a[c]) : "v"(m));
        if constexpr (OP == 4) asm volatile("v_log_f32 %0, %0" : "+v"(a[c]));
        if constexpr (OP == 5) asm volatile("v_cvt_f64_f32 %0, %1" : "=v"(d[c]) : "v"(a[c]));
      }
  }
  float s = 0;
  for (int c = 0; c < CH; ++c) s += a[c] + (float)d[c] + p[c].x + p[c].y;
  if (s == 12345.f) out[0] = s;
}

int main() {
  float* out;
  hipMalloc(&out, 4);
  int dev = 0, cus = 0, clk = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev);
  const int blocks = cus * 8;  // 8 x 4 waves per CU = 8 waves per SIMD
  const int iters = 40;
  const char* names[] = {"v_fma_f32", "v_pk_fma_f32", "v_fma_f64", "v_add_f32", "v_log_f32", "v_cvt_f64_f32"};
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int op = 0; op < 6; ++op) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(e0);
      switch (op) {
        case 0: k<0><<<blocks, 256>>>(out, iters); break;
        case 1: k<1><<<blocks, 256>>>(out, iters); break;
        case 2: k<2><<<blocks, 256>>>(out, iters); break;
        case 3: k<3><<<blocks, 256>>>(out, iters); break;
        case 4: k<4><<<blocks, 256>>>(out, iters); break;
        case 5: k<5><<<blocks, 256>>>(out, iters); break;
      }
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (rep == 1) {
        const double waves_per_simd = blocks * 4.0 / (cus * 4.0);
        const double instr_per_simd = waves_per_simd * (double)iters * REP * CH;
        const double cyc = ms * 1e-3 * clk * 1e3;  // clockRate in kHz
        printf("%-14s %8.3f ms  %.2f cycles per wave64 instruction per SIMD (clock %d MHz)\n",
               names[op], ms, cyc / instr_per_simd, clk / 1000);
      }
    }
  }
  return 0;
}
