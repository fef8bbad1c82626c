// Microbenchmark / layout check (diagnostic): v_mfma_f64_16x16x4f64 operand and result layout
// as the setup kernel uses it, and its issue cost at 1 wave per SIMD.
//   A (16x4):  lane l holds A[l & 15][l >> 4]
//   B (4x16):  lane l holds B[l >> 4][l & 15]
//   C (16x16): lane l, register r holds C[(l >> 4) + 4 r][l & 15]
// Build: hipcc -O3 --offload-arch=gfx950 tools/mb_mfma64.hip -o tools/build/mb_mfma64
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

__global__ void layout(const double* A, const double* B, double* C) {
  const int l = threadIdx.x;
  d4 acc = {0.0, 0.0, 0.0, 0.0};
  for (int q = 0; q < 4; ++q) {   // K = 16 as four k-steps of 4
    const double a = A[(l & 15) * 16 + 4 * q + (l >> 4)];
    const double b = B[(4 * q + (l >> 4)) * 16 + (l & 15)];
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
  }
  for (int r = 0; r < 4; ++r) C[((l >> 4) + 4 * r) * 16 + (l & 15)] = acc[r];
}

// chained: T = A B (16x16), then D = A' T with T's registers as the B operand
__global__ void chain(const double* A, const double* B, double* D) {
  const int l = threadIdx.x;
  d4 t = {0.0, 0.0, 0.0, 0.0};
  for (int q = 0; q < 4; ++q) {
    const double a = A[(l & 15) * 16 + 4 * q + (l >> 4)];
    const double b = B[(4 * q + (l >> 4)) * 16 + (l & 15)];
    t = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, t, 0, 0, 0);
  }
  d4 d = {0.0, 0.0, 0.0, 0.0};
  for (int r = 0; r < 4; ++r) {   // k-step r covers rows (l >> 4) + 4 r of T
    const double a = A[((l >> 4) + 4 * r) * 16 + (l & 15)];   // A'[i = l & 15][k = (l>>4) + 4r]
    d = __builtin_amdgcn_mfma_f64_16x16x4f64(a, t[r], d, 0, 0, 0);
  }
  for (int r = 0; r < 4; ++r) D[((l >> 4) + 4 * r) * 16 + (l & 15)] = d[r];
}

__global__ void rate(double* out, double a, int iters) {
  const int l = threadIdx.x;
  d4 c0 = {0.0, 0.0, 0.0, 0.0}, c1 = c0, c2 = c0, c3 = c0;
  double x = a + l;
  for (int it = 0; it < iters; ++it) {
    c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, a, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, a, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, a, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, a, c3, 0, 0, 0);
  }
  out[blockIdx.x * 64 + l] = c0[0] + c1[1] + c2[2] + c3[3];
}

int main() {
  double hA[256], hB[256], hC[256], hD[256];
  for (int i = 0; i < 256; ++i) {
    hA[i] = std::sin(0.37 * i + 0.1);
    hB[i] = std::cos(0.21 * i - 0.3);
  }
  double *dA, *dB, *dC, *dD, *dO;
  hipMalloc(&dA, 2048); hipMalloc(&dB, 2048); hipMalloc(&dC, 2048); hipMalloc(&dD, 2048);
  hipMalloc(&dO, 1024 * 64 * 8);
  hipMemcpy(dA, hA, 2048, hipMemcpyHostToDevice);
  hipMemcpy(dB, hB, 2048, hipMemcpyHostToDevice);
  layout<<<1, 64>>>(dA, dB, dC);
  chain<<<1, 64>>>(dA, dB, dD);
  hipMemcpy(hC, dC, 2048, hipMemcpyDeviceToHost);
  hipMemcpy(hD, dD, 2048, hipMemcpyDeviceToHost);
  double e1 = 0.0, e2 = 0.0, T[256];
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      double s = 0.0;
      for (int k = 0; k < 16; ++k) s += hA[i * 16 + k] * hB[k * 16 + j];
      T[i * 16 + j] = s;
      e1 = std::fmax(e1, std::fabs(s - hC[i * 16 + j]));
    }
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      double s = 0.0;
      for (int k = 0; k < 16; ++k) s += hA[k * 16 + i] * T[k * 16 + j];
      e2 = std::fmax(e2, std::fabs(s - hD[i * 16 + j]));
    }
  printf("layout max err %.3e  chain max err %.3e\n", e1, e2);
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  const int iters = 20000;
  for (int w : {1, 2, 4}) {
    rate<<<1024 * w, 64>>>(dO, 1.0001, 100);
    hipEventRecord(a);
    rate<<<1024 * w, 64>>>(dO, 1.0001, iters);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    // 256 CUs x 4 SIMDs; clocks at ~2.4 GHz
    printf("waves/SIMD %d: %.1f ns per MFMA per wave (%.1f clk @2.4GHz), %.1f TFLOP/s\n", w,
           ms * 1e6 / (4.0 * iters), ms * 1e6 / (4.0 * iters) * 2.4,
           2.0 * 16 * 16 * 4 * 4.0 * iters * 1024 * w / (ms * 1e-3) / 1e12);
  }
  return (e1 < 1e-12 && e2 < 1e-12) ? 0 : 1;
}
