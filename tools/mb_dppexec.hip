// Does a 64-bit DPP row_newbcast read the source lane's VGPR when that lane is disabled in EXEC?
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(double* out) {
  int l = threadIdx.x;
  double c = 1000.0 * l, src = l + 0.5, m = 2.0;
  // EXEC = lanes with (l % 16) > 3  (source lane 3 of each row disabled)
  asm volatile(
      "s_mov_b64 s[20:21], exec\n\t"
      "s_mov_b32 s22, 0xfff0fff0\n\t"
      "s_mov_b32 s23, 0xfff0fff0\n\t"
      "s_and_b64 exec, s[20:21], s[22:23]\n\t"
      "s_nop 4\n\t"
      "v_fmac_f64_dpp %0, %1, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
      "s_mov_b64 exec, s[20:21]"
      : "+v"(c) : "v"(src), "v"(m) : "s20", "s21", "s22", "s23");
  out[l] = c;
}
int main() {
  double* d; (void)hipMalloc(&d, 64 * 8);
  k<<<1, 64>>>(d);
  double h[64]; (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int l = 0; l < 20; ++l) {
    int r = l / 16 * 16;
    printf("lane %2d: %g  (if source read: %g, untouched: %g)\n", l, h[l], 1000.0 * l + (r + 3.5) * 2, 1000.0 * l);
  }
  return 0;
}
