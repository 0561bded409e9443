// Microbenchmark: how v_exp_f32 (transcendental) and plain VALU share a SIMD with a stream of
// v_mfma_f32_32x32x16_bf16 -- the question behind K1's d = 40 ceiling (16 v_exp per 7 MFMAs).
// Each wave loops over a hand-written asm block of 8 independent MFMAs, each followed by E v_exp
// and F v_fma_f32 (independent registers), and reports shader cycles (s_memtime) per MFMA.
// Build: hipcc --offload-arch=gfx950 -O3 tools/issue_bench.hip -o tools/issue_bench
// Run:   tools/issue_bench   (prints one JSON line per configuration)
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

#define STR2(x) #x
#define STR(x) STR2(x)

typedef float f32x2 __attribute__((ext_vector_type(2)));

// the instruction mix of a packed polynomial exp2 of 2 values on the plain VALU pipe (3 v_pk_add_f32,
// 2 v_pk_fma_f32, 2 v_lshl_add_u32): t = x + 1.5*2^23, n = t - 1.5*2^23, f = x - n, 2^f ~ c0 + f(c1 +
// c2 f), exponent += n.  Throughput only: the registers are arbitrary.
__device__ __forceinline__ void pexp2_mix(f32x2& a, f32x2& b, f32x2& c, float& u, float& v) {
  asm volatile(
      "v_pk_add_f32 %0, %0, %1\n\t"
      "v_pk_add_f32 %1, %0, %2\n\t"
      "v_pk_add_f32 %2, %1, %0\n\t"
      "v_pk_fma_f32 %0, %2, %1, %0\n\t"
      "v_pk_fma_f32 %1, %2, %0, %1\n\t"
      "v_lshl_add_u32 %3, %3, 23, %4\n\t"
      "v_lshl_add_u32 %4, %4, 23, %3"
      : "+v"(a), "+v"(b), "+v"(c), "+v"(u), "+v"(v));
}

template <int E, int F, int TE, int PX = 0>
__global__ __launch_bounds__(512) void bench(long long* out, int iters) {
  f32x16 acc[4];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 16; ++j) acc[i][j] = 0.f;
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = (__bf16)(0.01f * (threadIdx.x + j));
    b[j] = (__bf16)(0.02f * j);
  }
  float x0 = threadIdx.x * 1e-3f, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5;
  float y0 = 0, y1 = 0, y2 = 0, y3 = 0, y4 = 0, y5 = 0;
  f32x2 pa = {x0, x1}, pb = {x2, x3}, pc = {x4, x5}, qa = pa, qb = pb, qc = pc;
  float pu = x0, pv = x1, qu = x2, qv = x3;
  __syncthreads();
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc[u & 3]) : "v"(a), "v"(b));
      if (E >= 1) asm volatile("v_exp_f32 %0, %1" : "=v"(y0) : "v"(x0));
      if (E >= 2) asm volatile("v_exp_f32 %0, %1" : "=v"(y1) : "v"(x1));
      if (E >= 3) asm volatile("v_exp_f32 %0, %1" : "=v"(y2) : "v"(x2));
      if (E >= 4) asm volatile("v_exp_f32 %0, %1" : "=v"(y3) : "v"(x3));
      if (TE >= 1) asm volatile("v_exp_f32 %0, %1" : "=v"(y0) : "v"(x0));
      if (F >= 1) asm volatile("v_fma_f32 %0, %1, %1, %0" : "+v"(y4) : "v"(x4));
      if (F >= 2) asm volatile("v_fma_f32 %0, %1, %1, %0" : "+v"(y5) : "v"(x5));
      if (F >= 3) asm volatile("v_fma_f32 %0, %1, %1, %0" : "+v"(y1) : "v"(x1));
      if (F >= 4) asm volatile("v_fma_f32 %0, %1, %1, %0" : "+v"(y2) : "v"(x2));
      if (F >= 5) asm volatile("v_fma_f32 %0, %1, %1, %0" : "+v"(y3) : "v"(x3));
      if (F >= 6) asm volatile("v_fma_f32 %0, %1, %1, %0" : "+v"(y4) : "v"(x0));
      if (F >= 7) asm volatile("v_fma_f32 %0, %1, %1, %0" : "+v"(y5) : "v"(x1));
      if (F >= 8) asm volatile("v_fma_f32 %0, %1, %1, %0" : "+v"(y1) : "v"(x2));
      if (PX >= 1) pexp2_mix(pa, pb, pc, pu, pv);
      if (PX >= 2) pexp2_mix(qa, qb, qc, qu, qv);
    }
  }
  asm volatile("s_nop 15\n\ts_nop 15");
  long long t1 = __builtin_amdgcn_s_memtime();
  float s = y0 + y1 + y2 + y3 + y4 + y5 + pa[0] + pb[1] + pc[0] + qa[1] + qb[0] + qc[1] + pu + pv + qu + qv;
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 16; ++j) s += acc[i][j];
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
  if (s == 12345.f) out[0] = 0;
}

template <int E, int F, int TE = 0, int PX = 0>
void run(int threads, const char* name) {
  const int iters = 2000, nblk = 256;
  long long* d;
  const int nw = nblk * threads / 64;
  hipMalloc(&d, nw * sizeof(long long));
  hipLaunchKernelGGL((bench<E, F, TE, PX>), dim3(nblk), dim3(threads), 0, 0, d, iters);   // warm-up
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL((bench<E, F, TE, PX>), dim3(nblk), dim3(threads), 0, 0, d, iters);
  hipEventRecord(e1);
  hipDeviceSynchronize();
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  long long* h = new long long[nw];
  hipMemcpy(h, d, nw * sizeof(long long), hipMemcpyDeviceToHost);
  double sum = 0;
  for (int i = 0; i < nw; ++i) sum += h[i];
  const double cyc = sum / nw / (iters * 8.0);
  const double mfma = (double)nblk * threads / 64 * iters * 8;
  printf("{\"case\": \"%s\", \"waves_per_simd\": %d, \"exp_per_mfma\": %d, \"fma_per_mfma\": %d, "
         "\"poly_pairs_per_mfma\": %d, \"cycles_per_mfma\": %.2f, \"ms\": %.4f, \"tflops\": %.1f, \"clock_ghz\": %.3f}\n",
         name, threads / 256, E + TE, F, PX, cyc, ms, mfma * 32768 / ms / 1e9, cyc * iters * 8 / (ms * 1e-3) / 1e9);
  delete[] h;
  hipFree(d);
}

int main() {
  for (int threads : {256, 512}) {
    run<0, 0>(threads, "mfma");
    run<1, 0>(threads, "mfma+1exp");
    run<2, 0>(threads, "mfma+2exp");
    run<3, 0>(threads, "mfma+3exp");
    run<4, 0>(threads, "mfma+4exp");
    run<0, 2>(threads, "mfma+2fma");
    run<0, 4>(threads, "mfma+4fma");
    run<0, 6>(threads, "mfma+6fma");
    run<0, 8>(threads, "mfma+8fma");
    run<2, 2>(threads, "mfma+2exp+2fma");
    run<2, 4>(threads, "mfma+2exp+4fma");
    run<1, 4>(threads, "mfma+1exp+4fma");
    run<1, 6>(threads, "mfma+1exp+6fma");
    run<0, 0, 0, 1>(threads, "mfma+1poly");
    run<1, 0, 0, 1>(threads, "mfma+1exp+1poly");
    run<2, 0, 0, 1>(threads, "mfma+2exp+1poly");
    run<0, 0, 0, 2>(threads, "mfma+2poly");
    run<1, 2>(threads, "mfma+1exp+2fma");
  }
  return 0;
}
