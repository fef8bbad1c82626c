// Microbenchmark / check (GPU): the exact-order wave butterfly sum of osc_setup.hpp (permlane32 /
// permlane16 swaps and DPP for the six xor levels) against the shuffle butterfly it replaces --
// bitwise equality on random data, and the clocks of each.
//   hipcc --offload-arch=gfx950 -O3 -I operational-space-control_amd/csrc tools/mb_wave_sum.hip -o /tmp/mb_wave_sum
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include "osc_device.hpp"

__device__ __forceinline__ double sum_shfl(double v) {
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return __shfl(v, 0, 64);
}
#include "osc_wave_sum.hpp"

__global__ void check(const double* in, double* out, unsigned long long* clk, int reps) {
  const double v = in[blockIdx.x * 64 + threadIdx.x];
  double a = 0.0, b = 0.0;
  unsigned long long t0 = clock64();
  for (int r = 0; r < reps; ++r) a += sum_shfl(v + r);
  unsigned long long t1 = clock64();
  for (int r = 0; r < reps; ++r) b += osc::wave_sum_fast(v + r);
  unsigned long long t2 = clock64();
  out[2 * (blockIdx.x * 64 + threadIdx.x)] = sum_shfl(v);
  out[2 * (blockIdx.x * 64 + threadIdx.x) + 1] = osc::wave_sum_fast(v);
  if (threadIdx.x == 0) {
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = t2 - t1;
  }
  if (a != b && threadIdx.x == 0) out[0] = -1.0;   // (keeps both loops live)
}

int main() {
  const int nb = 256, n = nb * 64, reps = 64;
  double* h = (double*)malloc(sizeof(double) * n);
  srand(7);
  for (int i = 0; i < n; ++i) h[i] = (rand() / (double)RAND_MAX - 0.5) * pow(10.0, rand() % 12 - 6);
  double *din, *dout;
  unsigned long long* dclk;
  hipMalloc(&din, sizeof(double) * n);
  hipMalloc(&dout, sizeof(double) * 2 * n);
  hipMalloc(&dclk, sizeof(unsigned long long) * 2 * nb);
  hipMemcpy(din, h, sizeof(double) * n, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(check, dim3(nb), dim3(64), 0, 0, din, dout, dclk, reps);
  double* o = (double*)malloc(sizeof(double) * 2 * n);
  unsigned long long* c = (unsigned long long*)malloc(sizeof(unsigned long long) * 2 * nb);
  hipMemcpy(o, dout, sizeof(double) * 2 * n, hipMemcpyDeviceToHost);
  hipMemcpy(c, dclk, sizeof(unsigned long long) * 2 * nb, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < n; ++i)
    if (memcmp(&o[2 * i], &o[2 * i + 1], 8) != 0) ++bad;
  double cs = 0, cf = 0;
  for (int b = 0; b < nb; ++b) { cs += c[2 * b]; cf += c[2 * b + 1]; }
  printf("{\"lanes\": %d, \"bitwise_mismatches\": %d, \"clocks_per_sum_shfl\": %.1f, \"clocks_per_sum_fast\": %.1f}\n",
         n, bad, cs / nb / reps, cf / nb / reps);
  return bad != 0;
}
