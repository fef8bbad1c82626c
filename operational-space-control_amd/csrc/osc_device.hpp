// osc_device.hpp -- shared device-side building blocks of the batched OSC solver (gfx950):
// per-model constants (DevParams), the compile-time problem dimensions and workspace / LDS layouts
// (Dims), lane primitives (row-replicated SGPR masks, 64-bit DPP row broadcasts fused into FMAs,
// 16-lane DPP reductions), staging helpers, and the host-side model table (KernelId, workspace
// sizes).  Included by every kernel translation unit (DESIGN.md §5 lists the units):
//   osc_setup.hip       kernel 1  osc_setup_kernel       (reduced QP per env)
//   osc_ipm_*.hip       kernel 2  osc_ipm_kernel & co.   (interior point + refinement), one unit
//                                                         per robot model
//   osc_dual.hip        kernel 3  osc_dual_kernel        (dual solution, optional)
//   osc_gi.hip          kernel 4  osc_gi_kernel          (wheel-row active-set fallback)
//   osc_multi.hip       the two-model grids of osc_batch_solve_multi
//   osc_api.hip         the C-ABI (include/osc_batch.h): models, tuning, launch sequencing
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <new>
#include <type_traits>

#include "osc_batch.h"

namespace osc {

constexpr int kWave = 64;
constexpr int kRow = 16;                 // lanes per environment in the IPM kernel (DPP row)
constexpr int kEnvPerWave = kWave / kRow;

// Per-model constants, device-resident (uniform loads -> scalar cache).
struct DevParams {
  double w_row[6 * OSC_MAX_SITES];   // task-row weights, [w_p per site x3 ..., w_r per site x3]
  double u_lb[OSC_MAX_NU];
  double u_ub[OSC_MAX_NU];
  double z_lb[3];
  double z_ub[3];
  double mu;
  double w_torque;
  double w_reg;
  double eps_mu;
  double inf_thresh;
  double warm_delta;                 // warm start: slacks / multipliers floored at this value
  double warm_center;                // warm start: no pair s_i lambda_i below this x their mean
  int32_t warm_restart;              // warm start: re-centre an env still far off at this iteration
  int32_t restart_iter;              // cold start: the same, later
  int32_t max_iter;
  int32_t refine_steps;              // full-space refinement steps after the interior point
  double refine_penalty;             // active-row penalty, x max diag(Hr)
  double w_sqrt[6 * OSC_MAX_SITES];  // (unused slot: keeps the layout of the fields above)
  // wheel no-slip rows (models built with them only; walter_sr_wheels/autogen/autogen.py:128-240)
  int32_t wheel_dof[OSC_MAX_SITES];  // dof of wheel i's joint, -1 = no rolling term
  double wheel_radius[OSC_MAX_SITES];
  double wheel_tol;                  // interior point: |row residual| <= wheel_tol to stop
  double refine_max_move;            // a refinement moving y by more (relative) is rejected
#ifdef OSC_STAMPS
  unsigned long long* stamps;        // diagnostic builds: [kStampBlocks][kStampSlots], IPM phases
  unsigned long long* setup_stamps;  // ... and the assembly's (one buffer for every kernel unit)
#endif
};

// Full-space refinement: at most kRefineRounds active-set rounds of at most kRefineMaxSteps
// steps each (osc_ipm.hpp; the host clamps osc_model_tuning.refine_steps to the latter).
constexpr int kRefineRounds = 8, kRefineMaxSteps = 8;

constexpr int cmax(int a, int b) { return a > b ? a : b; }
constexpr int even(int a) { return (a + 1) & ~1; }   // keep LDS/workspace regions 16-B aligned

// Reduced coordinates y = (u, z): dv = X [y; 1] = M^-1 (B u + Jc z - C) over all nv rows, so the
// torque bounds are plain bounds on y (diagonal in the Newton matrix).  The dense assembly
// products run on the FP64 matrix cores where that saves LDS round trips (FP64 MFMA has the FP64
// VALU's peak on gfx950, tools/mb_mfma64.hip: ~70 clocks per 16x16x4): T1 = H_dv X and
// [Hr | g] = X'T1 always (T1 stays in registers), Ha = 2 [J e]'W[J e] where [J e] fits one
// 16-column tile (WaLTER, NA = 15); Go2's 19 columns would pad to 32 and stay on exact 2x2 VALU
// tiles (Go2 4,096: phase B 7.7k vs 3.5k clocks per wave).  X, H_dv, f_dv and [Hr | g] are stored
// to the workspace where they are formed (no copy-out phase).
// WH_: the model carries the wheel no-slip equality rows (two per contact wheel).
template <int NV_, int NU_, int NC_, int NS_, bool WH_ = false>
struct Dims {
  static constexpr int NV = NV_, NU = NU_, NC = NC_, NS = NS_;
  static constexpr bool WH = WH_;
  static constexpr int NW = WH ? 2 * NC : 0;  // wheel no-slip rows
  static constexpr int NB = NV - NU;          // unactuated (floating-base) dofs
  static constexpr int NZ = 3 * NC;
  static constexpr int NY = NU + NZ;          // reduced variables (u, z)
  static constexpr int NY1 = NY + 1;          // + affine column
  static constexpr int NY1P = even(NY1);      // padded row stride of X
  static constexpr int S = 6 * NS;            // task rows
  static constexpr int MI = 2 * NU + 6 * NC;  // inequality rows (u box, pyramid, fz box)
  static constexpr int NX = NV + NU + NZ;     // design vector
  static constexpr int NA = NV + 1;           // [J | e] Gram size
  static constexpr int NPA = NA * (NA + 1) / 2;
  static constexpr int NPH = NY1 * (NY1 + 1) / 2 - 1;   // reduced Hessian pairs (no corner)
  static constexpr int NRL = (MI + kRow - 1) / kRow;    // inequality rows per lane (IPM)
  static_assert(NY1 <= kWave && NX <= 3 * kRow, "setup / output lane mapping");
  static_assert(NY > kRow && NY <= 2 * kRow, "IPM: two column slots per lane");
  static_assert(NU <= kRow && NB <= kRow, "IPM: one torque / base row per lane");
  static_assert(NB >= 1 && NB <= 8, "floating-base block");

  // ---- workspace per env (doubles): [g | Hr | X | H_dv | f_dv | W_SOL] ----
  // Hr (symmetric, exactly) is stored COMPACT without wheel rows (round 6):
  // [A = its rows 16 .. NY-1, all NY columns, row-major | T = the upper triangle of its leading
  // 16 x 16 block, packed row-major] -- (NY - 16) NY + 136 doubles instead of NY^2 (Go2 328 vs
  // 576, WaLTER 648 vs 1,024): what the interior point streams each iteration (the second column
  // slot = rows 16.. by symmetry) stays whole rows; hr_off() maps (i, j) into it.  Wheel models
  // keep the full row-major Hr (their rotated Newton systems read it by columns).
  static constexpr bool HRC = !WH;
  static constexpr int HRA = NY - kRow;                 // rows in A
  static constexpr int HR_T = HRA * NY;                 // T's offset in the block
  static constexpr int HR_SIZE = HRC ? HR_T + kRow * (kRow + 1) / 2 : NY * NY;
  static constexpr int W_G = 0;
  static constexpr int W_HR = even(NY);
  static constexpr int W_X = W_HR + even(HR_SIZE);
  // H_dv = 2 J'WJ + 2 w_reg I and f_dv = 2 J'W (b - t), for the full-space refinement after the
  // interior point (its gradient never goes through Hr)
  static constexpr int W_HD = W_X + NV * NY1P;
  static constexpr int W_GD = W_HD + NV * NV;
  // interior-point result handed to the refinement kernel (and, with duals requested, to the
  // dual kernel): [y | q (lambda on rows with lambda > s, else 0; row slots) | status]
  static constexpr int W_SOL = W_GD + even(NV);
  // wheel rows: the multipliers w = L'nu_Q handed to the dual kernel; the rows in
  // reduced coordinates [Q | q1] (orthonormal, NW x NY1P; Q y + q1 = 0 <=> E dv = e); the
  // dv-space basis V = R E of E's row space, R, and the y-space transform L (Q = L V X)
  static constexpr int W_NU = W_SOL + even(NY) + NRL * 16 + 2;
  static constexpr int W_AW = W_NU + even(NW);
  static constexpr int W_WV = W_AW + NW * NY1P;
  static constexpr int W_WR = W_WV + NW * NV;
  static constexpr int W_WL = W_WR + NW * NW;
  // the rotation: T (NY x NY, T[i][k] at i * NY + k) and per column k the Q row it carries (-1:
  // a free direction)
  static constexpr int W_T = W_WL + NW * NW;
  static constexpr int W_PIN = W_T + NY * NY;
  // the raw rows the active-set fallback (osc_gi_kernel) rebuilds the full QP from, copied here by
  // the setup kernel so every entry point -- the split osc_batch_solve_assembled too -- can run it:
  // M (NV x NV), C, the contact translational rows of J (3 NC x NV) and of b, the wheel directions
  static constexpr int W_RM = W_PIN + even(NY);
  static constexpr int W_RC = W_RM + NV * NV;
  static constexpr int W_RJ = W_RC + even(NV);
  static constexpr int W_RB = W_RJ + 3 * NC * NV;
  static constexpr int W_RD = W_RB + even(3 * NC);
  static constexpr int WS = WH ? W_RD + even(6 * NC) : W_NU;
  // ---- warm state per env (doubles): [valid flag, pad | y (NY, padded) | lambda (row slots)] ----
  static constexpr int WW_Y = 2;
  static constexpr int WW_L = WW_Y + even(NY);
  static constexpr int WW_M = WW_L + NRL * 16;     // contact mask the state was solved with
  static constexpr int WW = WW_M + even(NC);

  // ---- setup-kernel LDS (doubles).  Every matrix that the 2x2-tiled products read by column
  // pairs (A = [J | e | 0]) has an even row stride, so a column pair is one 16-byte LDS read. ----
  static constexpr int NAP = even(NA);                   // [J | e (| 0)] row stride
  static constexpr int NA2 = NAP / 2;                    // column pairs
  static constexpr int NBA = NA2 * (NA2 + 1) / 2;        // Ha tiles (upper triangle)
  // Ha on MFMA where [J e] fits one 16-column tile (WaLTER, NA = 15).  J is then not staged:
  // Ha's MFMA fragments come straight from global memory and LDS holds only the contact rows
  // phase C reads (WaLTER: 102 x 16 -> 24 x 16 doubles): setup LDS 20.4 -> 10.4 KB.
  static constexpr bool JG = NA <= 16;
  static constexpr int JROWS = JG ? 3 * NC : S;                         // rows of A in LDS
  static constexpr int R1 = JROWS * NAP + (JG ? 2 * even(S) : 0);      // A = [J | e | 0] (| e | w)
  static constexpr int O_E = JROWS * NAP, O_W = O_E + even(S);          // JG: e = b - t, row weights
  static constexpr int R2 = even(NV * NV) + even(NV);                   // M | C
  static constexpr int O_A = 0;
  static constexpr int O_M = R1, O_C = R1 + even(NV * NV);
  static constexpr int O_HA = R1 + R2;
  static constexpr int O_X = O_HA + even(NA * NA);
  static constexpr int O_MASK = O_X + NV * NY1P;
  // WH: Gram-Schmidt row sets, one lane per column: [E | e | I] (dv space) and [V X | V x0 - vs
  // | I] (y space); the identity columns accumulate the transforms R and L
  static constexpr int WEST = even(NV + 1 + NW);
  static constexpr int WAST = NY1P + NW;
  static constexpr int O_WE = O_MASK + even(NC);
  static constexpr int O_WA = O_WE + NW * WEST;
  // WH: Gram-Schmidt of [Q; I_NY] (NW + NY rows of NY) -> the basis T of the y space whose first
  // columns are Q's rows (compacted in place: row k = column k of T)
  static constexpr int O_WT = O_WA + NW * WAST;
  static constexpr int WTST = NY + 1;   // the basis rows' LDS stride (odd: no bank conflicts)
  static constexpr int SMEM = O_WT + (WH ? (NW + NY) * WTST : 0);
  // Lean assembly (Go2, round 6): Ha is kept as H_dv alone (row stride NV; f_dv, phase D's only
  // other use of it, comes back from the workspace), and X, whose columns phase C computes in
  // registers before storing any, overlays A (dead once they are computed): 14.2 -> 10.2 KB for
  // Go2, from 11 to 16 waves per CU (its 100 VGPRs' limit)
  static constexpr int O_X_L = 0;
  static constexpr int O_HD_L = R1 + R2;
  static constexpr int O_MASK_L = O_HD_L + even(NV * NV);
  static constexpr int SMEM_L = O_MASK_L + even(NC);
  static_assert(NV * NY1P <= R1 + R2, "lean assembly: X over A and M");
  static_assert(NW <= kRow, "IPM: one wheel row per lane of the env's row");
  static_assert(NV % 2 == 0, "setup: J rows are staged in 16-byte chunks");
  static_assert(SMEM * 8 <= 64 * 1024, "setup LDS budget per env");

};

// Offset of Hr[i][j] in the workspace's Hr block (Dims::HRC: the compact layout above).
template <class D>
__host__ __device__ constexpr int hr_off(int i, int j) {
  if constexpr (!D::HRC) {
    return i * D::NY + j;
  } else {
    if (i >= kRow) return (i - kRow) * D::NY + j;
    if (j >= kRow) return (j - kRow) * D::NY + i;
    const int a = i < j ? i : j, b = i < j ? j : i;
    return D::HR_T + a * kRow - a * (a - 1) / 2 + (b - a);
  }
}

// ---- IPM-kernel LDS per env (doubles): workspace prefix [g (| Hr)] + vectors.
// Large batches (two waves per SIMD): Hr is NOT in LDS -- each lane streams its two Hr columns
// from the L2-resident workspace into the Newton-matrix registers once per iteration, which
// keeps the footprint small enough for two waves per SIMD.  Small batches (every wavefront
// resident at once, one per SIMD): Hr joins the LDS copy when four waves' worth fits in a CU's
// 160 KB, taking the L2 round trip off every iteration's critical path. ----
template <class D, bool HRL>
struct IpmLayout {
  static constexpr int NY = D::NY, NU = D::NU, NC = D::NC, NB = D::NB;
  static constexpr int I_G = D::W_G;
  static constexpr int I_HR = D::W_HR;                 // valid when HRL: full NY x NY, row-major
  // workspace prefix copied to LDS as it stands: [g | Hr] where the workspace's Hr is full,
  // [g] alone where it is compact (HRL then expands Hr into its full LDS layout, osc_ipm.hpp)
  static constexpr int STAGE = (HRL && !D::HRC) ? D::W_X : D::W_HR;
  static constexpr int I_VY = HRL ? D::W_HR + even(NY * NY) : D::W_HR;   // y (current iterate)
  static constexpr int I_VY2 = I_VY + even(NY);        // search direction
  static constexpr int I_UV = I_VY2 + even(NY);        // (unused slot: keeps the layout fixed)
  static constexpr int I_VR = I_UV + even(NU);         // a row-space vector
  static constexpr int I_DR = I_VR + D::NRL * kRow;    // lambda / s
  static constexpr int I_MASK = I_DR + D::NRL * kRow;
  static constexpr int I_TAU = I_MASK + even(NC);
  static constexpr int I_XB = I_TAU + even(NU);
  static constexpr int I_DINV = I_XB + even(D::NV);       // 1/D of the factorization (32)
  static constexpr int IL = I_DINV + 2 * kRow;
};
template <class D>
constexpr bool hr_fits_lds() {   // four one-wave workgroups per CU, 160 KB of LDS
  return IpmLayout<D, true>::IL * 8 * kEnvPerWave * 4 <= 160 * 1024;
}

// ---- Lockstep compaction (batches past one resident wavefront per SIMD).
// The four envs of a wavefront iterate in lockstep, so a wave costs its slowest env's iteration
// count.  The park pass (CP = 1) stops every wave at the top of iteration park_it: an env not
// converged by then is PARKED -- its interior-point state (y, s, lambda, carried rp) written to
// a slot of the park area, its env index to the slot list -- and the wave finishes the rest
// (refinement, outputs) without it.  The resume pass (CP = 2) packs the parked envs four to a
// wavefront (slot order) and continues them from iteration park_it.  Every row of a wave
// evolves independently (only wave-uniform gates couple them), so each env takes exactly the
// steps it takes in one pass: results are bitwise those of the single pass.
struct ParkArgs {
  int32_t* list;    // [nenv]  env of each parked slot
  int32_t* count;   // parked envs (zeroed before the park pass)
  double* park;     // [nenv][park_doubles<D>()]  y (32) | s | lambda | rp (NRL x 16 each) | rd (32)
  int park_it;      // iteration at whose top the park pass parks
};
constexpr int kCpNone = 0, kCpPark = 1, kCpResume = 2;
template <class D>
constexpr int park_doubles() { return 4 * kRow + 3 * D::NRL * kRow; }

// Upper-triangle pair tables (i <= j), built at compile time.
template <int N, bool SKIP_CORNER>
struct Pairs {
  static constexpr int P = N * (N + 1) / 2 - (SKIP_CORNER ? 1 : 0);
  unsigned char a[P > 0 ? P : 1];
  unsigned char b[P > 0 ? P : 1];
  constexpr Pairs() : a{}, b{} {
    int p = 0;
    for (int i = 0; i < N; ++i)
      for (int j = i; j < N; ++j) {
        if (SKIP_CORNER && i == N - 1 && j == N - 1) continue;
        a[p] = static_cast<unsigned char>(i);
        b[p] = static_cast<unsigned char>(j);
        ++p;
      }
  }
};

template <int N, bool SKIP>
__device__ constexpr Pairs<N, SKIP> kPairs{};

template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

// ---- lane primitives ----------------------------------------------------------------------
// Compile-time lane masks.  A 16-bit pattern over the lanes of one row, replicated to all four
// rows of the wave, is a 64-bit SGPR constant; selecting with it needs no per-lane compare.
constexpr unsigned long long rows_mask(unsigned pattern16) {
  return static_cast<unsigned long long>(pattern16 & 0xFFFFu) * 0x0001000100010001ull;
}
constexpr unsigned lanes_from(int lo, int hi) {   // lanes lo..hi of a row (empty if hi < lo)
  unsigned m = 0;
  for (int i = lo < 0 ? 0 : lo; i <= hi && i < 16; ++i) m |= 1u << i;
  return m;
}
// The mask is materialized (s_mov) right at its use: left to itself hipcc hoists every
// distinct mask of the unrolled loops into its own SGPR pair and spills them to VGPR lanes.
template <unsigned long long MASK>
__device__ __forceinline__ unsigned long long mask_here() {
  static_assert((MASK >> 32) == (MASK & 0xFFFFFFFFull), "row-replicated masks only");
  unsigned lo, hi;
  asm volatile("s_mov_b32 %0, %2\n\ts_mov_b32 %1, %2" : "=s"(lo), "=s"(hi)
               : "i"(static_cast<unsigned>(MASK & 0xFFFFFFFFull)));
  return (static_cast<unsigned long long>(hi) << 32) | lo;
}
// MASK lanes take `set`, the others `clear` (v_cndmask_b32 x2 on an SGPR-pair mask).
template <unsigned long long MASK>
__device__ __forceinline__ double select_lanes(double set, double clear) {
  if constexpr (MASK == 0ull) {
    return clear;
  } else if constexpr (MASK == ~0ull) {
    return set;
  } else {
    int lo, hi;
    asm("v_cndmask_b32_e64 %0, %2, %3, %6\n\tv_cndmask_b32_e64 %1, %4, %5, %6"
        : "=&v"(lo), "=v"(hi)
        : "v"(__double2loint(clear)), "v"(__double2loint(set)), "v"(__double2hiint(clear)),
          "v"(__double2hiint(set)), "s"(mask_here<MASK>()));
    return __hiloint2double(hi, lo);
  }
}
// MASK lanes keep v, the others get +0.0.
template <unsigned long long MASK>
__device__ __forceinline__ double keep_lanes(double v) {
  if constexpr (MASK == 0ull) {
    return 0.0;
  } else if constexpr (MASK == ~0ull) {
    return v;
  } else {
    int lo, hi;
    asm("v_cndmask_b32_e64 %0, 0, %2, %4\n\tv_cndmask_b32_e64 %1, 0, %3, %4"
        : "=&v"(lo), "=v"(hi)
        : "v"(__double2loint(v)), "v"(__double2hiint(v)), "s"(mask_here<MASK>()));
    return __hiloint2double(hi, lo);
  }
}

// keep_lanes on a mask already in an SGPR pair (one mask_here for several selects)
__device__ __forceinline__ double keep_m(unsigned long long m, double v) {
  int lo, hi;
  asm("v_cndmask_b32_e64 %0, 0, %2, %4\n\tv_cndmask_b32_e64 %1, 0, %3, %4"
      : "=&v"(lo), "=v"(hi)
      : "v"(__double2loint(v)), "v"(__double2hiint(v)), "s"(m));
  return __hiloint2double(hi, lo);
}

// The same selects on a lane mask formed by a VALU compare of the lane's index in its row (l)
// against K straight into VCC: three issue slots (v_cmp, two v_cndmask) where the SGPR-literal
// mask takes five or six (two s_mov, an s_nop the SALU -> VALU mask read needs on gfx950, two
// v_cndmask).  A wavefront alone on its SIMD pays ~4.5 clocks for EVERY instruction it issues,
// scalar ones and s_nop included (tools/mb/mb_issue.hip, profiles/r06/issue/), which is the
// interior point's situation at 4,096 envs.  Volatile: the triangular solves place them between
// the DPP FMAs on purpose -- their three VALU instructions are the two wait states the next DPP
// read of a just-written value needs, so those FMAs carry no s_nop of their own.
// sel_eq: `set` on the lane l == K of each row, `clear` elsewhere.
// (the compare is an asm statement of its own: hipcc pads any inline asm that reads a register
// the previous inline asm wrote with an s_nop -- gfx950's conservative forwarding-hazard rule for
// asm producers -- so the compare, which reads only l, goes between the DPP FMA that wrote `set`
// and the selects that read it)
template <int K>
__device__ __forceinline__ unsigned long long lane_eq(int l) {
  unsigned long long m;
  asm volatile("v_cmp_eq_u32_e64 %0, %1, %2" : "=s"(m) : "n"(K), "v"(l));
  return m;
}
template <int K>
__device__ __forceinline__ unsigned long long lane_gt(int l) {
  unsigned long long m;
  asm volatile("v_cmp_lt_u32_e64 %0, %1, %2" : "=s"(m) : "n"(K), "v"(l));
  return m;
}
__device__ __forceinline__ double sel_mask(unsigned long long m, double set, double clear) {
  int lo, hi;
  asm volatile("v_cndmask_b32_e64 %0, %2, %3, %6\n\t"
               "v_cndmask_b32_e64 %1, %4, %5, %6"
               : "=&v"(lo), "=v"(hi)
               : "v"(__double2loint(clear)), "v"(__double2loint(set)), "v"(__double2hiint(clear)),
                 "v"(__double2hiint(set)), "s"(m));
  return __hiloint2double(hi, lo);
}
template <int K>
__device__ __forceinline__ double sel_eq(int l, double set, double clear) {
  return sel_mask(lane_eq<K>(l), set, clear);
}
// keep_gt: v on the lanes l > K of each row, +0.0 elsewhere.
template <int K>
__device__ __forceinline__ double keep_gt(int l, double v) {
  const unsigned long long m = lane_gt<K>(l);
  int lo, hi;
  asm volatile("v_cndmask_b32_e64 %0, 0, %2, %4\n\t"
               "v_cndmask_b32_e64 %1, 0, %3, %4"
               : "=&v"(lo), "=v"(hi)
               : "v"(__double2loint(v)), "v"(__double2hiint(v)), "s"(m));
  return __hiloint2double(hi, lo);
}

// Broadcast lane K of each 16-lane row to the whole row: v_mov_b64_dpp row_newbcast:K.
template <int K>
__device__ __forceinline__ double rowb(double v) {
  const long long x = __double_as_longlong(v);
  return __longlong_as_double(__builtin_amdgcn_mov_dpp(x, 0x150 + K, 0xf, 0xf, false));
}

template <int CTRL>
__device__ __forceinline__ double dpp32x2(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xf, 0xf, false);
  return __hiloint2double(hi, lo);
}
// 16-lane row reductions: quad_perm xor1 / xor2, row_half_mirror, row_mirror.  Every lane of
// the row ends with the bitwise-identical result (each combine is commutative).
__device__ __forceinline__ double row_sum(double v) {
  v += dpp32x2<0xB1>(v);
  v += dpp32x2<0x4E>(v);
  v += dpp32x2<0x141>(v);
  v += dpp32x2<0x140>(v);
  return v;
}
__device__ __forceinline__ double row_min(double v) {
  v = fmin(v, dpp32x2<0xB1>(v));
  v = fmin(v, dpp32x2<0x4E>(v));
  v = fmin(v, dpp32x2<0x141>(v));
  v = fmin(v, dpp32x2<0x140>(v));
  return v;
}
__device__ __forceinline__ double row_max(double v) {
  v = fmax(v, dpp32x2<0xB1>(v));
  v = fmax(v, dpp32x2<0x4E>(v));
  v = fmax(v, dpp32x2<0x141>(v));
  v = fmax(v, dpp32x2<0x140>(v));
  return v;
}

// ---- diagnostic stamps (OSC_STAMPS builds only; the product build compiles them out) ----
// Per wave, cycles (s_memtime) accumulated per IPM phase into DevParams::stamps (one buffer for
// every kernel unit: static __device__ arrays were per unit); read back by osc_debug_stamps.
#ifdef OSC_STAMPS
constexpr int kStampSlots = 12;
constexpr int kStampBlocks = 1 << 15;
#define STAMP_DECL unsigned long long st_acc[kStampSlots] = {}; unsigned long long st_t0 = 0;
#define STAMP_BEGIN()                                                        \
  do {                                                                       \
    __builtin_amdgcn_sched_barrier(0);                                       \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_t0)::"memory"); \
    __builtin_amdgcn_sched_barrier(0);                                       \
  } while (0)
#define STAMP_END(slot)                                                      \
  do {                                                                       \
    unsigned long long st_t1;                                                \
    __builtin_amdgcn_sched_barrier(0);                                       \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_t1)::"memory"); \
    __builtin_amdgcn_sched_barrier(0);                                       \
    st_acc[slot] += st_t1 - st_t0;                                           \
  } while (0)
#define STAMP_STORE()                                                        \
  do {                                                                       \
    if (threadIdx.x == 0 && blockIdx.x < kStampBlocks)                       \
      for (int q_ = 0; q_ < kStampSlots; ++q_)                               \
        P->stamps[blockIdx.x * kStampSlots + q_] = st_acc[q_];               \
  } while (0)
#define STAMP_STORE_SETUP()                                                  \
  do {                                                                       \
    if (threadIdx.x == 0 && blockIdx.x < kStampBlocks)                       \
      for (int q_ = 0; q_ < kStampSlots; ++q_)                               \
        P->setup_stamps[blockIdx.x * kStampSlots + q_] = st_acc[q_];         \
  } while (0)
#elif defined(OSC_PHASE_MARKS)   // static analysis builds: phase labels in the listing (tools/)
#define STAMP_DECL
#define STAMP_BEGIN() asm volatile(";@@BEGIN")
#define STAMP_END(slot) asm volatile(";@@END " #slot)
#define STAMP_STORE() do {} while (0)
#define STAMP_STORE_SETUP() do {} while (0)
#else
#define STAMP_DECL
#define STAMP_BEGIN() do {} while (0)
#define STAMP_END(slot) do {} while (0)
#define STAMP_STORE() do {} while (0)
#define STAMP_STORE_SETUP() do {} while (0)
#endif

// a wave-uniform lane's double (v_readlane_b32 x2: no LDS round trip)
__device__ __forceinline__ double readlane_d(double v, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}

// Both kernels run ONE wavefront per workgroup.  LDS instructions of a wavefront execute in
// program order, so ordering an LDS write before another lane's later read only needs the
// compiler not to move memory operations across this point.  Unlike __syncthreads() (whose
// workgroup release fence emits s_waitcnt vmcnt(0)), it leaves in-flight global loads alone:
// the Hr prefetch of the IPM kernel stays in flight across it.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

// 1/d with one Newton step (v_rcp_f64 is good to ~2^-26; one step gives ~2^-52 in exact
// arithmetic, a few ulp in practice) -- enough for pivots and barrier terms.
__device__ __forceinline__ double recip1(double d) {
  const double r = __builtin_amdgcn_rcp(d);
  return fma(r, fma(-d, r, 1.0), r);
}
// 1/d to full double precision: v_rcp_f64 + two Newton steps.
__device__ __forceinline__ double recip(double d) {
  double r = __builtin_amdgcn_rcp(d);
  double e = fma(-d, r, 1.0);
  r = fma(r, e, r);
  e = fma(-d, r, 1.0);
  return fma(r, e, r);
}

// Copy n doubles (n even, both pointers 16-byte aligned) global -> LDS, 16 B per lane.
// N2 16-byte elements copied global -> LDS by STRIDE lanes, in two halves so that every load is
// in flight before the first store (a rolled copy loop waits one memory latency per trip: the
// IPM kernel's 28-trip staging of [g | U | Hr] used to cost ~28 L2/HBM round trips).
template <int N2, int STRIDE>
struct Batch2 {
  static constexpr int T = (N2 + STRIDE - 1) / STRIDE;
  static constexpr bool kFull = N2 % STRIDE == 0;
  double2 v[T];
  __device__ __forceinline__ void load(const double* __restrict__ src, int lane) {
    const double2* s2 = reinterpret_cast<const double2*>(src);
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const int i = lane + t * STRIDE;
      v[t] = s2[(kFull || t < T - 1 || i < N2) ? i : N2 - 1];   // clamped: no branch per load
    }
  }
  // dst index of element i given by map(i) (identity for a plain copy).  Lanes past the end
  // rewrite element N2-1 with the value they loaded for it (clamped above): no branch, so the
  // compiler cannot sink the last trip's load into a conditional block behind earlier waits.
  template <class Map>
  __device__ __forceinline__ void store(double* dst, int lane, Map map) const {
    double2* d2 = reinterpret_cast<double2*>(dst);
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const int i = lane + t * STRIDE;
      d2[map((kFull || t < T - 1 || i < N2) ? i : N2 - 1)] = v[t];
    }
  }
  __device__ __forceinline__ void store(double* dst, int lane) const {
    store(dst, lane, [](int i) { return i; });
  }
};

// p-th pair (i <= j) of the row-major upper triangle of an N x N grid -- the order of
// Pairs<N, false> -- in closed form (no table load: a per-lane indexed constant-table read is a
// memory round trip at the top of a phase).  i from the quadratic, then one integer correction
// each way for the rounding of the f32 square root.
template <int N>
__device__ __forceinline__ void upper_pair(int p, int& i, int& j) {
  constexpr int B = 2 * N + 1;
  auto start = [](int r) { return r * (2 * N - r + 1) / 2; };
  int r = static_cast<int>((B - __builtin_sqrtf(static_cast<float>(B * B - 8 * p))) * 0.5f);
  r = (r + 1 < N && start(r + 1) <= p) ? r + 1 : r;
  r = (r > 0 && start(r) > p) ? r - 1 : r;
  i = r;
  j = p - start(r) + r;
}

// c += bcast_K(src) * m  in ONE instruction: v_fmac_f64_dpp with row_newbcast:K (the DPP
// operand is read from lane K of each 16-lane row).  hipcc never forms this (64-bit DPP is
// only legal with row_newbcast), hence inline asm.  The compiler's hazard recognizer cannot see
// through inline asm, so every DPP read here carries its own guard: NOP = true prefixes
// s_nop 1 (gfx9: a VALU write of the DPP source needs 2 wait states before the DPP read) for a
// source just computed by the caller; NOP = false only where the source was written by one of
// these asm statements several dependent instructions earlier.
template <int K, bool NOP = false>
__device__ __forceinline__ void fmac_bcast(double& c, double src, double m) {
  if constexpr (NOP)
    asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
                 : "+v"(c) : "v"(src), "v"(m), "n"(K));
  else
    asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
                 : "+v"(c) : "v"(src), "v"(m), "n"(K));
}
template <int K, bool NOP = false>
__device__ __forceinline__ void fmac_bcast_self(double& c, double m) {
  if constexpr (NOP)
    asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf"
                 : "+v"(c) : "v"(m), "n"(K));
  else
    asm volatile("v_fmac_f64_dpp %0, %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf"
                 : "+v"(c) : "v"(m), "n"(K));
}
// Broadcast of lane K's v within each 16-lane row, guarded (v may have been written by asm).
template <int K>
__device__ __forceinline__ double bcast_guarded(double v) {
  double r;
  asm volatile("s_nop 1\n\tv_mov_b64_dpp %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf"
               : "=v"(r) : "v"(v), "n"(K));
  return r;
}

// One model's arguments to a two-model launch.
struct PairArgs {
  const DevParams* P;
  int nenv;
  const double *M, *C, *J, *b, *T, *mask;
  double* ws;
  double *tau, *x;
  int32_t *status, *iters;
};

using Go2 = Dims<18, 12, 4, 5>;   // unitree_go2: nv 18, nu 12, 4 feet, 5 sites
using Walter = Dims<14, 8, 8, 17>;   // walter_sr(_wheels): nv 14, nu 8, 8 wheels, 17 sites
using WalterW = Dims<14, 8, 8, 17, true>;   // + the wheel no-slip rows (opt-in)

enum KernelId { K_NONE = 0, K_GO2 = 1, K_WALTER = 2, K_WALTER_WHEELS = 3 };

inline KernelId select_kernel(const osc_model_desc& d) {
  const bool wheels = d.wheel_rows != 0;
  if (d.nv == Go2::NV && d.nu == Go2::NU && d.nc == Go2::NC && d.ns == Go2::NS)
    return wheels ? K_NONE : K_GO2;
  if (d.nv == Walter::NV && d.nu == Walter::NU && d.nc == Walter::NC && d.ns == Walter::NS)
    return wheels ? K_WALTER_WHEELS : K_WALTER;
  return K_NONE;
}

inline int ww_doubles(KernelId k) {
  switch (k) {
    case K_GO2: return Go2::WW;
    case K_WALTER: return Walter::WW;
    case K_WALTER_WHEELS: return WalterW::WW;
    default: return 0;
  }
}

inline int ws_doubles(KernelId k) {
  switch (k) {
    case K_GO2: return Go2::WS;
    case K_WALTER: return Walter::WS;
    case K_WALTER_WHEELS: return WalterW::WS;
    default: return 0;
  }
}

// Park iteration per model (0: compaction off).  Measured (tools/park_sweep.py,
// profiles/r03_park_sweep.txt): WaLTER (one wavefront per SIMD at every batch size) gains from
// it; Go2's two-wave kernel loses -- its parked envs run their last iterations as a serial tail
// after the park pass instead of hidden behind other wavefronts.
inline int park_iter_default(KernelId k) { return k == K_WALTER ? 16 : 0; }
constexpr int kParkMinRounds = 4;   // batches of at least this many resident-wave rounds

inline int park_doubles_of(KernelId k) {
  switch (k) {
    case K_GO2: return park_doubles<Go2>();
    case K_WALTER: return park_doubles<Walter>();
    default: return 0;   // (no compaction with wheel rows)
  }
}

// Byte offsets of the workspace blocks (all 16-byte aligned).
struct WsLayout {
  size_t status, park, list, count, total;
};
inline WsLayout ws_layout(KernelId k, int32_t nenv) {
  const size_t n = static_cast<size_t>(nenv);
  auto pad = [](size_t b) { return (b + 15) & ~static_cast<size_t>(15); };
  WsLayout w;
  w.status = sizeof(double) * static_cast<size_t>(ws_doubles(k)) * n;
  w.park = w.status + pad(sizeof(int32_t) * n);
  w.list = w.park + sizeof(double) * static_cast<size_t>(park_doubles_of(k)) * n;
  w.count = w.list + pad(sizeof(int32_t) * n);
  w.total = w.count + (park_doubles_of(k) ? 16 : 0);
  return w;
}

inline int dual_rows(KernelId k) {
  switch (k) {
    case K_GO2: return Go2::NV + 4 * Go2::NC + Go2::NX;
    case K_WALTER: return Walter::NV + 4 * Walter::NC + Walter::NX;
    case K_WALTER_WHEELS: return WalterW::NV + WalterW::NW + 4 * WalterW::NC + WalterW::NX;
    default: return 0;
  }
}

}  // namespace osc
