// Micro-check of the DPP forms used by the LDL^T pivot chain (osc_device.hpp recip1_bcast):
// v_rcp_f64_dpp row_newbcast, v_fmac_f64_dpp with a negated DPP source.  One wave; prints the
// lanes whose results differ from the plain-arithmetic reference.  Diagnostic only.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int K>
__device__ double rcp_b(double v) {
  double r;
  asm volatile("s_nop 1\n\tv_rcp_f64_dpp %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf"
               : "=&v"(r) : "v"(v), "n"(K));
  return r;
}
template <int K>
__device__ double mov_b(double v) {
  double r;
  asm volatile("s_nop 1\n\tv_mov_b64_dpp %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf"
               : "=&v"(r) : "v"(v), "n"(K));
  return r;
}
template <int K>
__device__ double fmac_neg_b(double acc, double v, double m) {
  asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, -%1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
               : "+v"(acc) : "v"(v), "v"(m), "n"(K));
  return acc;
}

__global__ void k(double* out) {
  const int l = threadIdx.x;
  const double v = 1.5 + l * 0.25;
  const double m = 0.5 + l;
  const double b = mov_b<3>(v);
  out[0 * 64 + l] = b;
  out[1 * 64 + l] = rcp_b<3>(v);
  out[2 * 64 + l] = __builtin_amdgcn_rcp(b);
  out[3 * 64 + l] = fmac_neg_b<3>(1.0, v, m);
  out[4 * 64 + l] = fma(-b, m, 1.0);
}

int main() {
  double* d;
  hipMalloc(&d, 5 * 64 * sizeof(double));
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  double h[5 * 64];
  hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int l = 0; l < 64; ++l) {
    if (h[64 + l] != h[128 + l] || h[192 + l] != h[256 + l]) {
      ++bad;
      if (bad < 10)
        printf("lane %d bcast %.17g rcp_dpp %.17g rcp %.17g fmac_dpp %.17g ref %.17g\n", l, h[l],
               h[64 + l], h[128 + l], h[192 + l], h[256 + l]);
    }
  }
  printf("lane 5: bcast %.17g rcp_dpp %.17g rcp %.17g fmac_dpp %.17g ref %.17g\n", h[5], h[69],
         h[133], h[197], h[261]);
  printf("%d bad lanes\n", bad);
  return 0;
}
