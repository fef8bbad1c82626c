// Micro-check (diagnostic): issue cost of instruction classes for ONE wavefront alone on the GPU
// (the straggler's situation at 4,096 Go2 envs).  Each kernel runs a fixed unrolled block in a
// loop; cycles per block from s_memtime; printed as clocks per instruction of the block.
#include <hip/hip_runtime.h>
#include <cstdio>
#define ITERS 2000

#define FMA8                                                                       \
  "v_fma_f64 v[0:1], v[0:1], v[16:17], v[18:19]\n\t"                               \
  "v_fma_f64 v[2:3], v[2:3], v[16:17], v[18:19]\n\t"                               \
  "v_fma_f64 v[4:5], v[4:5], v[16:17], v[18:19]\n\t"                               \
  "v_fma_f64 v[6:7], v[6:7], v[16:17], v[18:19]\n\t"                               \
  "v_fma_f64 v[8:9], v[8:9], v[16:17], v[18:19]\n\t"                               \
  "v_fma_f64 v[10:11], v[10:11], v[16:17], v[18:19]\n\t"                           \
  "v_fma_f64 v[12:13], v[12:13], v[16:17], v[18:19]\n\t"                           \
  "v_fma_f64 v[14:15], v[14:15], v[16:17], v[18:19]\n\t"

template <int KIND>
__global__ void k(unsigned long long* out) {
  unsigned long long t0 = 0, t1 = 0;
  asm volatile("v_mov_b32 v16, 0\n\tv_mov_b32 v17, 0x3ff00000\n\tv_mov_b32 v18, 0\n\tv_mov_b32 v19, 0" ::
                   : "v16", "v17", "v18", "v19");
  for (int w = 0; w < 2; ++w) {
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
    for (int it = 0; it < ITERS; ++it) {
      if constexpr (KIND == 0) {   // 8 independent f64 FMAs
        asm volatile(FMA8 ::: "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10",
                     "v11", "v12", "v13", "v14", "v15");
      } else if constexpr (KIND == 1) {   // 8 FMAs + 8 s_mov_b32
        asm volatile(
            "v_fma_f64 v[0:1], v[0:1], v[16:17], v[18:19]\n\ts_mov_b32 s40, 0x10001\n\t"
            "v_fma_f64 v[2:3], v[2:3], v[16:17], v[18:19]\n\ts_mov_b32 s41, 0x10001\n\t"
            "v_fma_f64 v[4:5], v[4:5], v[16:17], v[18:19]\n\ts_mov_b32 s40, 0x20002\n\t"
            "v_fma_f64 v[6:7], v[6:7], v[16:17], v[18:19]\n\ts_mov_b32 s41, 0x20002\n\t"
            "v_fma_f64 v[8:9], v[8:9], v[16:17], v[18:19]\n\ts_mov_b32 s40, 0x30003\n\t"
            "v_fma_f64 v[10:11], v[10:11], v[16:17], v[18:19]\n\ts_mov_b32 s41, 0x30003\n\t"
            "v_fma_f64 v[12:13], v[12:13], v[16:17], v[18:19]\n\ts_mov_b32 s40, 0x40004\n\t"
            "v_fma_f64 v[14:15], v[14:15], v[16:17], v[18:19]\n\ts_mov_b32 s41, 0x40004\n\t" ::
                : "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12",
                  "v13", "v14", "v15", "s40", "s41");
      } else if constexpr (KIND == 2) {   // 8 FMAs + 8 s_nop 0
        asm volatile(
            "v_fma_f64 v[0:1], v[0:1], v[16:17], v[18:19]\n\ts_nop 0\n\t"
            "v_fma_f64 v[2:3], v[2:3], v[16:17], v[18:19]\n\ts_nop 0\n\t"
            "v_fma_f64 v[4:5], v[4:5], v[16:17], v[18:19]\n\ts_nop 0\n\t"
            "v_fma_f64 v[6:7], v[6:7], v[16:17], v[18:19]\n\ts_nop 0\n\t"
            "v_fma_f64 v[8:9], v[8:9], v[16:17], v[18:19]\n\ts_nop 0\n\t"
            "v_fma_f64 v[10:11], v[10:11], v[16:17], v[18:19]\n\ts_nop 0\n\t"
            "v_fma_f64 v[12:13], v[12:13], v[16:17], v[18:19]\n\ts_nop 0\n\t"
            "v_fma_f64 v[14:15], v[14:15], v[16:17], v[18:19]\n\ts_nop 0\n\t" ::
                : "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12",
                  "v13", "v14", "v15");
      } else if constexpr (KIND == 3) {   // 8 FMAs + 8 v_cndmask_b32 (independent)
        asm volatile(
            "v_fma_f64 v[0:1], v[0:1], v[16:17], v[18:19]\n\tv_cndmask_b32 v20, v21, v22, vcc\n\t"
            "v_fma_f64 v[2:3], v[2:3], v[16:17], v[18:19]\n\tv_cndmask_b32 v23, v21, v22, vcc\n\t"
            "v_fma_f64 v[4:5], v[4:5], v[16:17], v[18:19]\n\tv_cndmask_b32 v24, v21, v22, vcc\n\t"
            "v_fma_f64 v[6:7], v[6:7], v[16:17], v[18:19]\n\tv_cndmask_b32 v25, v21, v22, vcc\n\t"
            "v_fma_f64 v[8:9], v[8:9], v[16:17], v[18:19]\n\tv_cndmask_b32 v26, v21, v22, vcc\n\t"
            "v_fma_f64 v[10:11], v[10:11], v[16:17], v[18:19]\n\tv_cndmask_b32 v27, v21, v22, vcc\n\t"
            "v_fma_f64 v[12:13], v[12:13], v[16:17], v[18:19]\n\tv_cndmask_b32 v28, v21, v22, vcc\n\t"
            "v_fma_f64 v[14:15], v[14:15], v[16:17], v[18:19]\n\tv_cndmask_b32 v29, v21, v22, vcc\n\t" ::
                : "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12",
                  "v13", "v14", "v15", "v20", "v23", "v24", "v25", "v26", "v27", "v28", "v29");
      } else if constexpr (KIND == 4) {   // 8 independent v_fmac_f64_dpp row_newbcast
        asm volatile(
            "v_fmac_f64_dpp v[0:1], v[16:17], v[18:19] row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
            "v_fmac_f64_dpp v[2:3], v[16:17], v[18:19] row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
            "v_fmac_f64_dpp v[4:5], v[16:17], v[18:19] row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
            "v_fmac_f64_dpp v[6:7], v[16:17], v[18:19] row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
            "v_fmac_f64_dpp v[8:9], v[16:17], v[18:19] row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
            "v_fmac_f64_dpp v[10:11], v[16:17], v[18:19] row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
            "v_fmac_f64_dpp v[12:13], v[16:17], v[18:19] row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
            "v_fmac_f64_dpp v[14:15], v[16:17], v[18:19] row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t" ::
                : "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12",
                  "v13", "v14", "v15");
      } else if constexpr (KIND == 5) {   // 8 FMAs + 4 v_cndmask_b32_e64 on an SGPR mask
        asm volatile(
            "v_fma_f64 v[0:1], v[0:1], v[16:17], v[18:19]\n\tv_cndmask_b32_e64 v20, v21, v22, s[40:41]\n\t"
            "v_fma_f64 v[2:3], v[2:3], v[16:17], v[18:19]\n\t"
            "v_fma_f64 v[4:5], v[4:5], v[16:17], v[18:19]\n\tv_cndmask_b32_e64 v23, v21, v22, s[40:41]\n\t"
            "v_fma_f64 v[6:7], v[6:7], v[16:17], v[18:19]\n\t"
            "v_fma_f64 v[8:9], v[8:9], v[16:17], v[18:19]\n\tv_cndmask_b32_e64 v24, v21, v22, s[40:41]\n\t"
            "v_fma_f64 v[10:11], v[10:11], v[16:17], v[18:19]\n\t"
            "v_fma_f64 v[12:13], v[12:13], v[16:17], v[18:19]\n\tv_cndmask_b32_e64 v25, v21, v22, s[40:41]\n\t"
            "v_fma_f64 v[14:15], v[14:15], v[16:17], v[18:19]\n\t" ::
                : "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12",
                  "v13", "v14", "v15", "v20", "v23", "v24", "v25");
      } else if constexpr (KIND == 6) {   // 8 s_nop 0 alone
        asm volatile("s_nop 0\n\ts_nop 0\n\ts_nop 0\n\ts_nop 0\n\ts_nop 0\n\ts_nop 0\n\ts_nop 0\n\ts_nop 0\n\t");
      } else if constexpr (KIND == 7) {   // 8 s_mov_b32 alone
        asm volatile(
            "s_mov_b32 s40, 1\n\ts_mov_b32 s41, 2\n\ts_mov_b32 s42, 3\n\ts_mov_b32 s43, 4\n\t"
            "s_mov_b32 s44, 1\n\ts_mov_b32 s45, 2\n\ts_mov_b32 s46, 3\n\ts_mov_b32 s47, 4\n\t" ::
                : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47");
      } else if constexpr (KIND == 8) {   // 8 dependent FMAs (one chain)
        asm volatile(
            "v_fma_f64 v[0:1], v[0:1], v[16:17], v[18:19]\n\t"
            "v_fma_f64 v[0:1], v[0:1], v[16:17], v[18:19]\n\t"
            "v_fma_f64 v[0:1], v[0:1], v[16:17], v[18:19]\n\t"
            "v_fma_f64 v[0:1], v[0:1], v[16:17], v[18:19]\n\t"
            "v_fma_f64 v[0:1], v[0:1], v[16:17], v[18:19]\n\t"
            "v_fma_f64 v[0:1], v[0:1], v[16:17], v[18:19]\n\t"
            "v_fma_f64 v[0:1], v[0:1], v[16:17], v[18:19]\n\t"
            "v_fma_f64 v[0:1], v[0:1], v[16:17], v[18:19]\n\t" ::: "v0", "v1");
      } else if constexpr (KIND == 9) {   // 8 dependent DPP FMAs (chain through the DPP source), s_nop 1 each
        asm volatile(
            "s_nop 1\n\tv_fmac_f64_dpp v[0:1], v[0:1], v[18:19] row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
            "s_nop 1\n\tv_fmac_f64_dpp v[0:1], v[0:1], v[18:19] row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
            "s_nop 1\n\tv_fmac_f64_dpp v[0:1], v[0:1], v[18:19] row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
            "s_nop 1\n\tv_fmac_f64_dpp v[0:1], v[0:1], v[18:19] row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
            "s_nop 1\n\tv_fmac_f64_dpp v[0:1], v[0:1], v[18:19] row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
            "s_nop 1\n\tv_fmac_f64_dpp v[0:1], v[0:1], v[18:19] row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
            "s_nop 1\n\tv_fmac_f64_dpp v[0:1], v[0:1], v[18:19] row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
            "s_nop 1\n\tv_fmac_f64_dpp v[0:1], v[0:1], v[18:19] row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t" ::
                : "v0", "v1");
      }
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  }
  if (threadIdx.x == 0) out[0] = t1 - t0;
}

template <int KIND>
double run(unsigned long long* d, int ninst) {
  hipLaunchKernelGGL(k<KIND>, dim3(1), dim3(64), 0, 0, d);
  unsigned long long h = 0;
  (void)hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
  return static_cast<double>(h) / (static_cast<double>(ITERS) * ninst);
}

int main() {
  unsigned long long* d;
  (void)hipMalloc(&d, 8);
  printf("{\"fma_indep_8\": %.2f, ", run<0>(d, 8));
  printf("\"fma+s_mov_16\": %.2f, ", run<1>(d, 16));
  printf("\"fma+s_nop0_16\": %.2f, ", run<2>(d, 16));
  printf("\"fma+cndmask_16\": %.2f, ", run<3>(d, 16));
  printf("\"fmac_dpp_indep_8\": %.2f, ", run<4>(d, 8));
  printf("\"fma8+cndmask_e64_4 (per 12)\": %.2f, ", run<5>(d, 12));
  printf("\"s_nop0_8\": %.2f, ", run<6>(d, 8));
  printf("\"s_mov_8\": %.2f, ", run<7>(d, 8));
  printf("\"fma_dep_8\": %.2f, ", run<8>(d, 8));
  printf("\"fmac_dpp_dep_nop1 (per dpp)\": %.2f}\n", run<9>(d, 8));
  return 0;
}
