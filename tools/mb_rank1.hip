// Microbenchmark (diagnostic): cycles per rank-1 update of a 24x24 column-per-lane matrix
// (the IPM kernel's U' diag(d) U loop, Go2 sizes) in three forms, one wave per SIMD:
//   dpp   : v_fmac_f64_dpp row_newbcast (the product's form), u broadcast from the lane holding it
//   lds   : u row read from LDS as 16-byte broadcast reads, plain v_fma_f64
//   plain : v_fma_f64 only, operands already in registers (issue-rate floor)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

constexpr int NY = 24, NQ = 12, REPS = 64;

template <int K, bool NOP>
__device__ __forceinline__ void fmac2(double& a, double& b, double src, double ma, double mb) {
  if constexpr (NOP)
    asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %2, %3 row_newbcast:%5 row_mask:0xf bank_mask:0xf\n\t"
                 "v_fmac_f64_dpp %1, %2, %4 row_newbcast:%5 row_mask:0xf bank_mask:0xf"
                 : "+v"(a), "+v"(b) : "v"(src), "v"(ma), "v"(mb), "n"(K));
  else
    asm volatile("v_fmac_f64_dpp %0, %2, %3 row_newbcast:%5 row_mask:0xf bank_mask:0xf\n\t"
                 "v_fmac_f64_dpp %1, %2, %4 row_newbcast:%5 row_mask:0xf bank_mask:0xf"
                 : "+v"(a), "+v"(b) : "v"(src), "v"(ma), "v"(mb), "n"(K));
}

template <int I, int N, class F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    sfor<I + 1, N>(f);
  }
}

template <int MODE>
__global__ __launch_bounds__(64, 1) void k(double* out, long long* cyc, double seed) {
  __shared__ __attribute__((aligned(16))) double sU[NQ * 32];
  const int l = threadIdx.x & 15;
  for (int i = threadIdx.x; i < NQ * 32; i += 64) sU[i] = seed * (i + 1);
  __syncthreads();
  double c0[NY], c1[NY];
  for (int i = 0; i < NY; ++i) c0[i] = c1[i] = seed + i + l;
  const long long t0 = clock64();
  for (int rep = 0; rep < REPS; ++rep) {
#pragma unroll 1
    for (int q = 0; q < NQ; ++q) {
      const double u0 = sU[q * 32 + l], u1 = sU[q * 32 + 16 + l];
      const double t0v = u0 * 1.0001, t1v = u1 * 0.9999;
      if constexpr (MODE == 0) {
        sfor<0, NY>([&](auto ic) {
          constexpr int i = decltype(ic)::value;
          fmac2<i % 16, i % 16 == 0>(c0[i], c1[i], i < 16 ? u0 : u1, t0v, t1v);
        });
      } else if constexpr (MODE == 1) {
        const double2* row = reinterpret_cast<const double2*>(sU + q * 32);
#pragma unroll
        for (int i = 0; i < NY; i += 2) {
          const double2 v = row[i / 2];
          c0[i] = fma(v.x, t0v, c0[i]);
          c1[i] = fma(v.x, t1v, c1[i]);
          c0[i + 1] = fma(v.y, t0v, c0[i + 1]);
          c1[i + 1] = fma(v.y, t1v, c1[i + 1]);
        }
      } else {
#pragma unroll
        for (int i = 0; i < NY; ++i) {
          c0[i] = fma(u0, t0v, c0[i]);
          c1[i] = fma(u1, t1v, c1[i]);
        }
      }
    }
  }
  const long long t1 = clock64();
  double s = 0.0;
  for (int i = 0; i < NY; ++i) s += c0[i] + c1[i];
  out[blockIdx.x * 64 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main(int argc, char** argv) {
  const int blocks = argc > 1 ? atoi(argv[1]) : 1024;   // 1024: one wave per SIMD
  double* out;
  long long* cyc;
  hipMalloc(&out, blocks * 64 * sizeof(double));
  hipMalloc(&cyc, blocks * sizeof(long long));
  static long long h[65536];
  const char* names[3] = {"dpp", "lds", "plain"};
  for (int mode = 0; mode < 3; ++mode) {
    for (int w = 0; w < 2; ++w) {
      if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(64), 0, 0, out, cyc, 1.0);
      if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(64), 0, 0, out, cyc, 1.0);
      if (mode == 2) hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(64), 0, 0, out, cyc, 1.0);
      hipDeviceSynchronize();
    }
    hipMemcpy(h, cyc, blocks * sizeof(long long), hipMemcpyDeviceToHost);
    double avg = 0;
    for (int b = 0; b < blocks; ++b) avg += h[b];
    avg /= blocks;
    const double per_q = avg / (REPS * NQ);
    printf("%-6s cycles/rank-1 (q) %.1f  per f64 FMA instr %.2f\n", names[mode], per_q,
           per_q / (2 * NY));
  }
  return 0;
}
