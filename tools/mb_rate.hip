// Microbenchmark (diagnostic): per-wave issue cost of v_fma_f64, v_mov_b64_dpp row_newbcast,
// ds_swizzle and v_readlane on MI355X, at 1/2/4/8 waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#define NACC 16
#define ITERS 4096
__global__ void fma64(double* out, double a, double b) {
  double acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = threadIdx.x + i;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = fma(acc[i], a, b);
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void dppmov(double* out, double a, double b) {
  double acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = threadIdx.x + i;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) {
      long long x = __double_as_longlong(acc[i]);
      acc[i] = __longlong_as_double(__builtin_amdgcn_mov_dpp(x, 0x150 + 3, 0xf, 0xf, false));
    }
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void dppfma(double* out, double a, double b) {
  double acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = threadIdx.x + i;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) {
      long long x = __double_as_longlong(acc[(i + 1) % NACC]);
      double bb = __longlong_as_double(__builtin_amdgcn_mov_dpp(x, 0x150 + 3, 0xf, 0xf, false));
      acc[i] = fma(bb, a, acc[i]);
    }
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void fma32(double* out, double a, double b) {
  float acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = threadIdx.x + i;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = fmaf(acc[i], (float)a, (float)b);
  }
  float s = 0;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void fmacdpp(double* out, double a, double b) {
  double acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = threadIdx.x + i;
  double src = a + threadIdx.x;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i)
      asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf"
                   : "+v"(acc[i]) : "v"(src), "v"(b));
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void fmadep(double* out, double a, double b) {   // one dependent chain
  double acc = threadIdx.x;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc = fma(acc, a, b);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}
__global__ void rcp64(double* out, double a, double b) {
  double acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = threadIdx.x + i + 1.0;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_rcp(acc[i]);
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void cnd64(double* out, double a, double b) {
  double acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = threadIdx.x + i + 1.0;
  int l = threadIdx.x;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) {
      asm volatile("" : "+v"(l));
      acc[i] = (l == i) ? a : acc[i];
    }
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void nop0(double* out, double a, double b) {
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) asm volatile("s_nop 0");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a;
}
__global__ void ldsb(double* out, double a, double b) {   // broadcast ds_read_b128
  __shared__ double sm[256];
  sm[threadIdx.x] = a + threadIdx.x;
  __syncthreads();
  double acc0 = 0, acc1 = 0;
  for (int it = 0; it < ITERS; ++it) {
    int base = (it * 2) & 127;
    asm volatile("" : "+v"(base));
#pragma unroll
    for (int i = 0; i < NACC; ++i) {
      double2 v = *reinterpret_cast<const double2*>(&sm[(base + 2 * i) & 254]);
      acc0 += v.x; acc1 += v.y;
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc0 + acc1;
}
template <class F>
void run(const char* name, F kern, double* out) {
  for (int wps : {1, 2, 4, 8}) {
    int blocks = 256 * 4 * wps;   // one 64-thread block per wave; waves per SIMD = wps
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(64), 0, 0, out, 1.0000001, 1e-9);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(64), 0, 0, out, 1.0000001, 1e-9);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    double instr_per_wave = double(ITERS) * NACC;
    // cycles per instruction per SIMD at 2.4 GHz nominal
    double cyc = ms * 1e-3 * 2.4e9 / (instr_per_wave * wps);
    printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.3f, \"simd_cycles_per_wave_instr\": %.2f}\n",
           name, wps, ms, cyc);
  }
}
int main() {
  double* out;
  (void)hipMalloc(&out, sizeof(double) * 256 * 4 * 8 * 64);
  run("v_fma_f64", fma64, out);
  run("v_fma_f32", fma32, out);
  run("v_mov_b64_dpp_newbcast", dppmov, out);
  run("dpp_mov+fma_f64 pair", dppfma, out);
  run("v_fmac_f64_dpp (asm)", fmacdpp, out);
  run("v_fma_f64 dependent chain", fmadep, out);
  run("v_rcp_f64", rcp64, out);
  run("cndmask f64 (2x b32 + cmp)", cnd64, out);
  run("s_nop 0", nop0, out);
  run("ds_read_b128 bcast + 2 add_f64", ldsb, out);
  return 0;
}
