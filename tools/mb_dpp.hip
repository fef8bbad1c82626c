// Semantics check of 64-bit DPP FMA forms on gfx950 (v_fmac_f64_dpp row_newbcast).
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_fmac(double* out) {
  int l = threadIdx.x;
  double c = 1000.0 * l, src = l + 0.5, m = 2.0;
  asm volatile("s_nop 4");
  asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf"
               : "+v"(c) : "v"(src), "v"(m));
  out[l] = c;
  double c2 = 1000.0 * l + 0.25;
  asm volatile("s_nop 4");
  asm volatile("v_fmac_f64_dpp %0, %0, %1 row_newbcast:5 row_mask:0xf bank_mask:0xf"
               : "+v"(c2) : "v"(m));
  out[64 + l] = c2;
  double d = 0.0;
  asm volatile("s_nop 4");
  asm volatile("v_mov_b64_dpp %0, %1 row_newbcast:3 row_mask:0xf bank_mask:0xf"
               : "=v"(d) : "v"(src));
  out[128 + l] = d;
  double e = 1000.0 * l;
  asm volatile("s_nop 4");
  asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(e) : "v"(d), "v"(m));
  out[192 + l] = e;
}

int main() {
  double* d;
  hipMalloc(&d, 256 * sizeof(double));
  k_fmac<<<1, 64>>>(d);
  double h[256];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  int bad = 0;
  for (int l = 0; l < 64; ++l) {
    int r = l / 16 * 16;
    double e0 = 1000.0 * l + (r + 3 + 0.5) * 2.0;
    double e1 = 1000.0 * l + 0.25 + (1000.0 * (r + 5) + 0.25) * 2.0;
    double e2 = r + 3 + 0.5;
    if (h[l] != e0 || h[64 + l] != e1 || h[128 + l] != e2 || h[192 + l] != e0) {
      if (bad < 8) printf("lane %d: fmac %g (exp %g)  self %g (exp %g)  mov %g (exp %g)  fma %g\n",
                          l, h[l], e0, h[64 + l], e1, h[128 + l], e2, h[192 + l]);
      ++bad;
    }
  }
  printf("%s (%d bad lanes)\n", bad ? "MISMATCH" : "OK", bad);
  return bad != 0;
}
