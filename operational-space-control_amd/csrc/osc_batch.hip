// osc_batch.hip -- batched OSC QP assembly + solve for gfx950 (MI355X).
//
// Replaces, per environment, the reference's per-tick hot path (paths relative to the
// reference's operational-space-control/ directory):
//   * CasADi-generated H, f, Aeq, beq, Aineq, bineq  (unitree_go2/autogen/autogen.py:58-319,
//     evaluated at unitree_go2/operational_space_controller.h:457-481)
//   * OSQP stacking / update / solve                  (operational_space_controller.h:483-536)
//   * torque slice                                    (operational_space_controller.h:573)
//
// The QP (unique optimum: strictly convex, always feasible):
//   min_x  sum_r w_r (J dv + b - t)_r^2 + w_tau |u|^2 + w_reg |x|^2,   x = (dv, u, z)
//   s.t.   M dv + C - B u - Jc z = 0            B = [0; I_nu],  Jc = Jp[last 3nc rows]^T
//          (+-fx +-fy - mu fz) <= 0 per contact, fz in [z_lb, z_ub] * mask, u in [u_lb, u_ub]
//
// Method:
//   1. The dynamics rows are eliminated exactly in torque coordinates y = (u, z) (24 Go2 /
//      32 WaLTER unknowns): dv = X [y; 1] = M^-1 (B u + Jc z - C) by block elimination on the
//      base block M_bb and the Schur complement of the actuated block, so the torque bounds are
//      plain bounds on y.  y carries a dense reduced Hessian Hr = X'H_dv X + diag and gradient g.
//   2. Mehrotra predictor-corrector interior point on  min 1/2 y'Hr y + g'y  s.t. G y <= h,
//      G = [+-e_q (torque bounds); pyramid + fz bound rows (sparse)].  Newton matrix
//      K = Hr + G' diag(lambda/s) G, LDL^T with "Cholesky-infinity" pivots.
//   3. A full-space refinement on the converged active set removes the error of the explicitly
//      formed fp64 Hr (its residual never goes through Hr).
//
// Two kernels, one workspace (per env [g | Hr | X | H_dv | f_dv], fp64):
//   osc_setup_kernel  one 64-lane wavefront per environment.  Inputs are staged HBM -> LDS
//                     with 16-byte loads; the dense products (J'WJ, the reduced Hessian) run on
//                     the FP64 matrix cores or as 2x2 VALU tiles.
//   osc_ipm_kernel    FOUR environments per wavefront, one 16-lane DPP row each.  The Newton
//                     matrix lives in registers, lane l holding columns l and l+16.  The
//                     right-looking LDL^T broadcasts the pivot column inside each row with
//                     v_mov_b64_dpp row_newbcast -- a VALU operation, no LDS traffic -- and the
//                     triangular solves use lane-local data (the symmetric trailing update
//                     leaves row j of L in lane j's upper registers) plus one row broadcast per
//                     step.  Inequality rows map three/four per lane; reductions (ratio test,
//                     complementarity) are 16-lane DPP butterflies.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <new>
#include <type_traits>

#include "osc_batch.h"

namespace {

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
};

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
  static constexpr int W_G = 0;
  static constexpr int W_HR = even(NY);
  static constexpr int W_X = W_HR + even(NY * NY);
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
  static constexpr int WS = WH ? W_PIN + even(NY) : W_NU;
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
  static constexpr int SMEM = O_WT + (WH ? (NW + NY) * NY : 0);
  static_assert(NW <= kRow, "IPM: one wheel row per lane of the env's row");
  static_assert(NV % 2 == 0, "setup: J rows are staged in 16-byte chunks");
  static_assert(SMEM * 8 <= 64 * 1024, "setup LDS budget per env");

};

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
  static constexpr int I_HR = D::W_HR;                 // valid when HRL
  static constexpr int STAGE = HRL ? D::W_X : D::W_HR; // workspace prefix copied to LDS
  static constexpr int I_VY = STAGE;                   // y (current iterate)
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
  double* park;     // [nenv][park_doubles<D>()]  y (32) | s | lambda | rp (NRL x 16 each)
  int park_it;      // iteration at whose top the park pass parks
};
constexpr int kCpNone = 0, kCpPark = 1, kCpResume = 2;
template <class D>
constexpr int park_doubles() { return 2 * kRow + 3 * D::NRL * kRow; }

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
// Per wave, cycles (s_memtime) accumulated per IPM phase; read back by osc_debug_stamps.
#ifdef OSC_STAMPS
constexpr int kStampSlots = 12;
constexpr int kStampBlocks = 1 << 15;
__device__ unsigned long long g_stamps[kStampBlocks * kStampSlots];
__device__ unsigned long long g_setup_stamps[kStampBlocks * kStampSlots];
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
        g_stamps[blockIdx.x * kStampSlots + q_] = st_acc[q_];                \
  } while (0)
#define STAMP_STORE_SETUP()                                                  \
  do {                                                                       \
    if (threadIdx.x == 0 && blockIdx.x < kStampBlocks)                       \
      for (int q_ = 0; q_ < kStampSlots; ++q_)                               \
        g_setup_stamps[blockIdx.x * kStampSlots + q_] = st_acc[q_];          \
  } while (0)
#else
#define STAMP_DECL
#define STAMP_BEGIN() do {} while (0)
#define STAMP_END(slot) do {} while (0)
#define STAMP_STORE() do {} while (0)
#define STAMP_STORE_SETUP() do {} while (0)
#endif

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

// ============================ kernel 1: reduced QP per env ==================================
// Dense products of the assembly (H_dv X, X'(H_dv X), and 2 A'WA where it fits one tile) on the
// FP64 matrix cores (v_mfma_f64_16x16x4f64).
typedef double d4 __attribute__((ext_vector_type(4)));

// Sum over the 64 lanes, the same value on every lane (lane 0's butterfly result broadcast).
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, kWave);
  return __shfl(v, 0, kWave);
}

// Modified Gram-Schmidt over the NR rows of an LDS row set (row stride `stride`, `ncol` columns,
// one lane per column): the first NDOT columns are made orthonormal, the other columns follow the
// same row operations (a right-hand side, identity columns accumulating the transform).  A row
// whose residual is not above `drop` x its original norm is dependent on the earlier ones and
// becomes zero (with its transform row).  Every decision is wave-uniform.
template <int NR, int NDOT>
__device__ __forceinline__ void wave_mgs(double* rows, int stride, int ncol, int lane,
                                         double drop) {
  double a[NR];
  const bool cv = lane < ncol;
#pragma unroll
  for (int w = 0; w < NR; ++w) a[w] = cv ? rows[w * stride + lane] : 0.0;
  const bool dv = lane < NDOT;
#pragma unroll
  for (int w = 0; w < NR; ++w) {
    const double n0 = sqrt(wave_sum(dv ? a[w] * a[w] : 0.0));
#pragma unroll
    for (int v = 0; v < w; ++v) {
      const double cf = wave_sum(dv ? a[v] * a[w] : 0.0);
      a[w] = fma(-cf, a[v], a[w]);
    }
    const double nn = sqrt(wave_sum(dv ? a[w] * a[w] : 0.0));
    const double sc = (nn > drop * n0 && nn > 0.0) ? 1.0 / nn : 0.0;
    a[w] *= sc;
  }
  if (cv) {
#pragma unroll
    for (int w = 0; w < NR; ++w) rows[w * stride + lane] = a[w];
  }
}

// Gram-Schmidt over the `nrows` rows of an LDS row set (row stride `stride`, `ncol` columns, one
// lane per column): the first `ndot` columns are made orthonormal, the other columns follow the
// same row operations (a right-hand side, identity columns accumulating the transform).  A row
// whose residual is not above `drop` x its original norm is dependent on the earlier ones and
// becomes zero (with its transform row).  Every decision is wave-uniform.
// Classical Gram-Schmidt applied twice (CGS2), not modified: the projections of row w on all
// earlier rows come from one pass with lane v forming row v's dot product (no 64-lane reduction
// per pair -- modified Gram-Schmidt's 1,128 dependent reductions for the 48-row basis completion
// were most of the wheel model's setup: 975 -> 564 us for 2,048 envs), then lane c subtracts them
// from column c; the second pass restores orthogonality to working precision.  (For the 16-row
// sets the register-resident wave_mgs above stays: this LDS form measured 2.3x slower there,
// profiles/r04za/.)  `scf`: nrows doubles of LDS scratch.
__device__ __noinline__ void wave_mgs_lds(double* rows, int nrows, int stride, int ncol, int ndot,
                                          int lane, double drop, double* scf) {
  const bool cv = lane < ncol, dv = lane < ndot;
  for (int w = 0; w < nrows; ++w) {
    double aw = cv ? rows[w * stride + lane] : 0.0;
    const double n0 = sqrt(wave_sum(dv ? aw * aw : 0.0));
    for (int pass = 0; pass < 2 && w > 0; ++pass) {
      double cf = 0.0;
      if (lane < w) {
        for (int c = 0; c < ndot; ++c) cf = fma(rows[lane * stride + c], rows[w * stride + c], cf);
      }
      if (lane < w) scf[lane] = cf;
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
      if (cv) {
        for (int v = 0; v < w; ++v) aw = fma(-scf[v], rows[v * stride + lane], aw);
        rows[w * stride + lane] = aw;
      }
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
    }
    const double nn = sqrt(wave_sum(dv ? aw * aw : 0.0));
    const double sc = (nn > drop * n0 && nn > 0.0) ? 1.0 / nn : 0.0;
    if (cv) rows[w * stride + lane] = aw * sc;
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
  }
}

// The body of one setup wavefront (env = its block index); `sm` is the block's D::SMEM doubles
// of LDS.  Wrapped by osc_setup_kernel (one model) and osc_setup_pair_kernel (two models, one
// grid: BASELINE configs[4]).
template <class D>
__device__ __forceinline__ void setup_env(
    const DevParams* __restrict__ P, int env, int nenv, const double* __restrict__ gM,
    const double* __restrict__ gC, const double* __restrict__ gJ, const double* __restrict__ gb,
    const double* __restrict__ gT, const double* __restrict__ gmask, double* __restrict__ ws,
    double* __restrict__ sm, const double* __restrict__ gwd) {
  constexpr int NV = D::NV, NU = D::NU, NC = D::NC, NS = D::NS, NB = D::NB, NY = D::NY,
                NY1 = D::NY1, NY1P = D::NY1P, S = D::S, NA = D::NA;
  const int lane = threadIdx.x;
  if (env >= nenv) return;

  constexpr int NAP = D::NAP;
  double* sA = sm + D::O_A;
  double* sM = sm + D::O_M;
  double* sC = sm + D::O_C;
  double* sHa = sm + D::O_HA;
  double* sX = sm + D::O_X;
  double* sU = sm + D::O_X + NB * NY1P;   // U parked in X's last rows until X replaces it
  double* sMask = sm + D::O_MASK;

  STAMP_DECL
  STAMP_BEGIN();
  // ---------------- Phase A: stage this env's inputs HBM -> LDS ----------------
  // every load first (one memory latency), then the LDS stores
  static_assert(NV % 2 == 0 && NC % 2 == 0, "16-byte staging needs even nv and nc");
  constexpr int JC0 = 3 * (NS - NC);   // first contact translational row of J
  constexpr int JR0 = D::JG ? JC0 : 0; // first row of J staged (JG: the contact rows only)
  Batch2<D::JROWS * NV / 2, kWave> bJ;
  Batch2<NV * NV / 2, kWave> bM;
  Batch2<NV / 2, kWave> bC;
  Batch2<NC / 2, kWave> bK;
  bJ.load(gJ + static_cast<size_t>(env) * S * NV + JR0 * NV, lane);
  bM.load(gM + static_cast<size_t>(env) * NV * NV, lane);
  bC.load(gC + static_cast<size_t>(env) * NV, lane);
  bK.load(gmask + static_cast<size_t>(env) * NC, lane);
  // JG: phase B's MFMA fragments of J (row 4q + (lane >> 4), column lane & 15) loaded now, in the
  // same memory latency as the staging loads; e and the row weights go to LDS
  constexpr int KSJ = D::JG ? (S + 3) / 4 : 0;
  double jf[KSJ > 0 ? KSJ : 1];
  {
    const int lc = lane & 15, lg = lane >> 4;
#pragma unroll
    for (int q = 0; q < KSJ; ++q) {
      const int r = 4 * q + lg;
      jf[q] = gJ[static_cast<size_t>(env) * S * NV + (r < S ? r : S - 1) * NV + (lc < NV ? lc : 0)];
    }
  }
  constexpr int TEJ = D::JG ? (S + kWave - 1) / kWave : 0;
  double ebj[TEJ > 0 ? TEJ : 1], etj[TEJ > 0 ? TEJ : 1], wj[TEJ > 0 ? TEJ : 1];
#pragma unroll
  for (int q = 0; q < TEJ; ++q) {
    const int r = (lane + q * kWave < S) ? lane + q * kWave : S - 1;
    const int half = r / (3 * NS), rr = r % (3 * NS);
    ebj[q] = gb[static_cast<size_t>(env) * S + r];
    etj[q] = gT[static_cast<size_t>(env) * NS * 6 + (rr / 3) * 6 + half * 3 + rr % 3];
    wj[q] = P->w_row[r];
  }
  // A column NV: e = b - t,  t = [T[:,0:3] row-wise ; T[:,3:6] row-wise]  (autogen.py:163-168)
  constexpr int TE = D::JG ? 0 : (S + kWave - 1) / kWave;   // (JG: e enters phase B's fragments)
  double eb[TE > 0 ? TE : 1], et[TE > 0 ? TE : 1];
#pragma unroll
  for (int q = 0; q < TE; ++q) {
    const int r = (lane + q * kWave < S) ? lane + q * kWave : S - 1;
    const int half = r / (3 * NS), rr = r % (3 * NS);
    eb[q] = gb[static_cast<size_t>(env) * S + r];
    et[q] = gT[static_cast<size_t>(env) * NS * 6 + (rr / 3) * 6 + half * 3 + rr % 3];
  }
  bJ.store(sA, lane, [](int c) { return (c / (NV / 2)) * (NAP / 2) + c % (NV / 2); });   // J rows -> A rows
#pragma unroll
  for (int q = 0; q < TEJ; ++q) {
    const int r = (lane + q * kWave < S) ? lane + q * kWave : S - 1;
    sA[D::O_E + r] = ebj[q] - etj[q];
    sA[D::O_W + r] = wj[q];
  }
  bM.store(sM, lane);
  bC.store(sC, lane);
  bK.store(sMask, lane);
#pragma unroll
  for (int q = 0; q < TE; ++q) {   // lanes past S rewrite row S-1 with its own value (no branch)
    const int r = (lane + q * kWave < S) ? lane + q * kWave : S - 1;
    sA[r * NAP + NV] = eb[q] - et[q];
    if (NAP > NA) sA[r * NAP + NA] = 0.0;
  }
  wave_sync();

  STAMP_END(0);
  STAMP_BEGIN();
  // ---------------- Phase B: Ha = 2 [J e]' W [J e]  (H_dv block and f_dv column) -------------
  // H_dv = 2 J'WJ + 2 w_reg I,  f_dv = 2 J'W (b - t)   (autogen.py:131-238, 304-319)
  // One 2x2 tile of the upper triangle per lane (column pairs read as one 16-byte LDS load);
  // each entry (i <= j) accumulates fma(w_r A_ri, A_rj) over r in order.
  // (H_dv and f_dv also go to the workspace from here, no write phase)
  double* const wha = ws + static_cast<size_t>(env) * D::WS;
  auto put_ha = [&](int i, int j, double v) {
    if (i >= NA || j >= NA) return;
    v *= 2.0;
    if (i == j && i < NV) v += 2.0 * P->w_reg;
    sHa[i * NA + j] = v;
    sHa[j * NA + i] = v;
    if (j < NV) {                          // H_dv (i <= j < NV), both triangles
      wha[D::W_HD + i * NV + j] = v;
      wha[D::W_HD + j * NV + i] = v;
    } else if (j == NV && i < NV) {        // f_dv = the [J e] Gram's last column
      wha[D::W_GD + i] = v;
    }
  };
  if constexpr (D::JG) {
    // FP64 MFMA (v_mfma_f64_16x16x4f64): 16x16 tiles of the upper block triangle, K = task rows
    // in steps of 4.  Lane l feeds row/column (l & 15) of a block at k-row 4q + (l >> 4) and
    // gets back C[(l >> 4) + 4 r][l & 15] (tools/mb_mfma64.hip checks this layout on the GPU).
    // Only entries i <= j are stored (then mirrored): H_dv is exactly symmetric.
    constexpr int NBK = (NA + 15) / 16, KS = (S + 3) / 4;
    const int lc = lane & 15, lg = lane >> 4;
    d4 acc[NBK * (NBK + 1) / 2];
#pragma unroll
    for (int t = 0; t < NBK * (NBK + 1) / 2; ++t) acc[t] = d4{0.0, 0.0, 0.0, 0.0};
    // fragments of CH k-steps loaded together (row weights included), then their MFMAs: one
    // memory latency per chunk instead of one per k-step
    constexpr int CH = 8;
#pragma unroll   // (compile-time k-steps: JG indexes the register fragments jf by them)
    for (int q0 = 0; q0 < KS; q0 += CH) {
      double v[CH][NBK], wv[CH];
#pragma unroll
      for (int u = 0; u < CH; ++u) {
        const int r = 4 * (q0 + u) + lg;
        const bool rv = r < S;
        wv[u] = rv ? sA[D::O_W + r] : 0.0;
#pragma unroll
        for (int b = 0; b < NBK; ++b) {
          const int col = 16 * b + lc;
          // [J | e | 0] row r: J from the fragments loaded in phase A, e from LDS
          const double ev = sA[D::O_E + (rv ? r : 0)];
          v[u][b] = !rv ? 0.0 : (col < NV ? jf[q0 + u < KSJ ? q0 + u : 0] : (col == NV ? ev : 0.0));
        }
      }
#pragma unroll
      for (int u = 0; u < CH; ++u) {
        if (q0 + u >= KS) break;
        int t = 0;
#pragma unroll
        for (int bi = 0; bi < NBK; ++bi)
#pragma unroll
          for (int bj = bi; bj < NBK; ++bj, ++t)
            acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(wv[u] * v[u][bi], v[u][bj], acc[t], 0, 0, 0);
      }
    }
    int t = 0;
#pragma unroll
    for (int bi = 0; bi < NBK; ++bi)
#pragma unroll
      for (int bj = bi; bj < NBK; ++bj, ++t)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int i = 16 * bi + lg + 4 * rr, j = 16 * bj + lc;
          if (i <= j) put_ha(i, j, acc[t][rr]);
        }
  } else
  for (int p = lane; p < D::NBA; p += kWave) {
    int i0, j0;
    upper_pair<D::NA2>(p, i0, j0);
    i0 *= 2;
    j0 *= 2;
    double a00 = 0.0, a01 = 0.0, a10 = 0.0, a11 = 0.0;
    // (fully unrolled: unrolled 4 or 8 deep it needs 100 VGPRs instead of 256 and the CU takes 11
    // setup waves instead of 8, but the kernel is issue-bound and gets slower, 31.6 -> 34.5 us;
    // profiles/r04y/)
    for (int r = 0; r < S; ++r) {
      const double2 x = *reinterpret_cast<const double2*>(sA + r * NAP + i0);
      const double2 y = *reinterpret_cast<const double2*>(sA + r * NAP + j0);
      const double w = P->w_row[r];
      const double wx0 = w * x.x, wx1 = w * x.y;
      a00 = fma(wx0, y.x, a00);
      a01 = fma(wx0, y.y, a01);
      a10 = fma(wx1, y.x, a10);
      a11 = fma(wx1, y.y, a11);
    }
    put_ha(i0, j0, a00);
    put_ha(i0, j0 + 1, a01);
    if (i0 != j0) put_ha(i0 + 1, j0, a10);   // diagonal tile: (i0+1, i0) mirrors a01
    put_ha(i0 + 1, j0 + 1, a11);
  }

  STAMP_END(1);
  STAMP_BEGIN();
  // ---------------- Phase C: base-block elimination  X = M_bb^-1 [-M_ba | Jc_b | -C_b] -------
  // and the torque map U = M_a Pm + [M_aa | -Jc_a | C_a]  so that  u = U [y; 1].
  // (dynamics rows: autogen.py:58-89; Jc = Jp[last 3nc rows]^T: osc.h:439-445)
  // One lane per column c of [y; 1]; when two copies of the 32-lane column set fit the wave,
  // both halves solve for X (redundantly) and split the NU rows of U between them.
  constexpr bool kSplitU = 2 * NY1P <= kWave;
  constexpr int kUStep = kSplitU ? (NU + 1) / 2 : NU;
  const int c = kSplitU ? (lane & 31) : lane;
  const int a_lo = kSplitU ? (lane >> 5) * kUStep : 0;
  if (c < NY1) {
    const bool pinned = (c >= NU && c < NY) && (sMask[(c - NU) / 3] == 0.0);
    // right-hand side and U's constant term are strided LDS vectors chosen per lane (no
    // divergent branches around the reads):
    //   c < NU : -M[0:NB, NB+c],  U0 = M[NB+a, NB+c]
    //   c < NY : Jc_b column,     U0 = -Jc_a column        (row JC0 + c - NU of A)
    //   c = NY : -C_b,            U0 = C_a
    const bool cu = c < NU, cz = !cu && c < NY;
    const double* xp = cu ? sM + NB + c : (cz ? sA + (JC0 - JR0 + c - NU) * NAP : sC);
    const int xs = cu ? NV : 1;
    const double xsg = cz ? 1.0 : -1.0;
    const double* up =
        cu ? sM + NB * NV + NB + c : (cz ? sA + (JC0 - JR0 + c - NU) * NAP + NB : sC + NB);
    const double usg = cz ? -1.0 : 1.0;
    double x[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) x[i] = pinned ? 0.0 : xsg * xp[i * xs];
    // LDL^T of the NB x NB base block (redundantly per lane; NB^3/6 flops)
    double L[NB][NB];
    double dinv[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i)
#pragma unroll
      for (int j = 0; j <= i; ++j) L[i][j] = sM[i * NV + j];
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      dinv[k] = recip1(L[k][k]);
#pragma unroll
      for (int i = k + 1; i < NB; ++i) {          // trailing update with the unscaled column
        const double lik = L[i][k] * dinv[k];
#pragma unroll
        for (int j = k + 1; j <= i; ++j) L[i][j] = fma(-lik, L[j][k], L[i][j]);
      }
#pragma unroll
      for (int i = k + 1; i < NB; ++i) L[i][k] *= dinv[k];   // then scale it to unit-lower
    }
#pragma unroll
    for (int k = 0; k < NB; ++k)
#pragma unroll
      for (int i = k + 1; i < NB; ++i) x[i] = fma(-L[i][k], x[k], x[i]);
#pragma unroll
    for (int k = 0; k < NB; ++k) x[k] *= dinv[k];
#pragma unroll
    for (int k = NB - 1; k >= 0; --k)
#pragma unroll
      for (int i = 0; i < k; ++i) x[i] = fma(-L[k][i], x[k], x[i]);
    if (a_lo == 0) {
#pragma unroll
      for (int i = 0; i < NB; ++i) sX[i * NY1P + c] = x[i];
    }
#pragma unroll
    for (int t = 0; t < kUStep; ++t) {
      const int a = a_lo + t;
      if (a < NU) {
        double acc = pinned ? 0.0 : usg * up[a * xs];
#pragma unroll
        for (int i = 0; i < NB; ++i) acc = fma(sM[(NB + a) * NV + i], x[i], acc);
        sU[a * NY1P + c] = acc;
      }
    }
  } else if (c < NY1P) {   // padding column of X and U: read by the 2x2 tiles, must be 0
    if (a_lo == 0) {
#pragma unroll
      for (int i = 0; i < NB; ++i) sX[i * NY1P + c] = 0.0;
    }
#pragma unroll
    for (int t = 0; t < kUStep; ++t)
      if (a_lo + t < NU) sU[(a_lo + t) * NY1P + c] = 0.0;
  }
  wave_sync();
  {
    // y = (u, z): X = M^-1 [B | Jc | -C] over all NV rows by block elimination on the base block.
    // The code above left X_b = M_bb^-1 [-M_ba | Jc_b | -C_b] in rows 0..NB-1 and
    // U = M_ab X_b + [M_aa | -Jc_a | C_a] in rows NB.. of sX; U's first NU columns are the Schur
    // complement S = M_aa - M_ab M_bb^-1 M_ba.  Per column c:
    //   S x_a = r_a' with r_a' = e_c (u columns) or -U[:, c] (contact / affine columns)
    //   x_b = X_b[:, :NU] x_a (+ X_b[:, c] for c >= NU)
    // S = L D L' is factored once per 16-lane row (lane j holds column j; the four rows of the
    // wave repeat it): pivot k's column is broadcast inside the row with v_fmac_f64_dpp
    // row_newbcast, one instruction per trailing entry.  The solves then read L the same way --
    // lane c of any row solves column c and takes L's entries from the row's lane k by DPP --
    // so the factor never goes through LDS.  Every lane runs every step (a DPP read needs its
    // source lane active); lanes past the last column compute garbage and write zeros.
    static_assert(NU <= kRow, "S fits one 16-lane row");
    STAMP_END(2);
    STAMP_BEGIN();
    const int lj = lane & (kRow - 1);
    double col[NU];
#pragma unroll
    for (int i = 0; i < NU; ++i) col[i] = sU[i * NY1P + (lj < NU ? lj : 0)];
    double dj = 1.0;
    static_for<0, NU>([&](auto K) {
      constexpr int k = decltype(K)::value;
      const double rk = recip1(bcast_guarded<k>(col[k]));       // 1 / S_k[k][k]
      if (lj == k) dj = rk;
      const double m = (lj > k) ? -col[k] * rk : 0.0;          // -S_k[k][j] / d_k, lanes j > k
      static_for<k + 1, NU>([&](auto I) {
        constexpr int i = decltype(I)::value;
        fmac_bcast_self<k, true>(col[i], m);                    // S[i][j] -= S[i][k] S[k][j] / d_k
      });
    });
    // lane j: col[i > j] = L[i][j] d_j (unscaled column), dj = 1 / d_j
    double dinv[NU];
    static_for<0, NU>([&](auto K) {
      constexpr int k = decltype(K)::value;
      dinv[k] = bcast_guarded<k>(dj);
    });
    STAMP_END(6);
    STAMP_BEGIN();
    const int c = lane;
    const bool cu = c < NU, live = c < NY1;
    const int cc = (cu || !live) ? NU : c;   // a valid column to read for lanes that do not use it
    double xa[NU], xb[NB], xbc[NB];
#pragma unroll
    for (int i = 0; i < NU; ++i) {
      const double u = sU[i * NY1P + cc];
      xa[i] = cu ? ((i == c) ? 1.0 : 0.0) : -u;
    }
#pragma unroll
    for (int r = 0; r < NB; ++r) {
      xb[r] = sX[r * NY1P + cc];                              // X_b[:, c] (contact / affine)
      xbc[r] = sX[r * NY1P + (lj < NU ? lj : 0)];             // X_b[:, j]: the DPP source of lane j
    }
    // L z = r:  z[i] -= (L[i][k] d_k) (z[k] / d_k)
    static_for<0, NU>([&](auto K) {
      constexpr int k = decltype(K)::value;
      const double t = -xa[k] * dinv[k];
      static_for<k + 1, NU>([&](auto I) {
        constexpr int i = decltype(I)::value;
        fmac_bcast<k>(xa[i], col[i], t);
      });
    });
#pragma unroll
    for (int k = 0; k < NU; ++k) xa[k] *= dinv[k];
    // L' x = y:  x[i] = y[i] - (1 / d_i) sum_{k > i} (L[k][i] d_i) x[k]
    static_for<0, NU - 1>([&](auto J) {
      constexpr int i = NU - 2 - decltype(J)::value;
      double acc = 0.0;
      static_for<i + 1, NU>([&](auto K) {
        constexpr int k = decltype(K)::value;
        fmac_bcast<i>(acc, col[k], xa[k]);
      });
      xa[i] = fma(-dinv[i], acc, xa[i]);
    });
    STAMP_END(7);
    STAMP_BEGIN();
    // x_b = X_b[:, :NU] x_a (+ X_b[:, c] for contact / affine columns)
#pragma unroll
    for (int r = 0; r < NB; ++r) xb[r] = cu ? 0.0 : xb[r];
    static_for<0, NU>([&](auto Q) {
      constexpr int q = decltype(Q)::value;
#pragma unroll
      for (int r = 0; r < NB; ++r) fmac_bcast<q>(xb[r], xbc[r], xa[q]);
    });
    wave_sync();   // every lane has read X_b and U before any column is overwritten
    if (c < NY1P) {
      double* const wx = ws + static_cast<size_t>(env) * D::WS + D::W_X;   // X: also to the workspace
#pragma unroll
      for (int r = 0; r < NB; ++r) {
        const double v = live ? xb[r] : 0.0;
        sX[r * NY1P + c] = v;
        wx[r * NY1P + c] = v;
      }
#pragma unroll
      for (int i = 0; i < NU; ++i) {
        const double v = live ? xa[i] : 0.0;
        sX[(NB + i) * NY1P + c] = v;
        wx[(NB + i) * NY1P + c] = v;
      }
    }
    wave_sync();
    STAMP_END(8);
    STAMP_BEGIN();
  }
  if constexpr (D::WH) {
    // ---- wheel no-slip rows (walter_sr_wheels/autogen/autogen.py:128-240) ----
    // E dv = e with, for contact wheel i (mask m_i), rows 2i (longitudinal) and 2i + 1 (lateral):
    //   m_i (d_roll' J_p,i - r_i e_k') dv = -m_i d_roll' b_i,   m_i d_lat' J_p,i dv = -m_i d_lat' b_i
    // (J_p,i, b_i: the contact site's translational rows of J and b).  Seven or eight grounded
    // wheels give 14-16 rows on nv = 14 accelerations: dependent, and in y = (u, z) coordinates
    // (dv = X [y; 1]) badly scaled.  So:
    //   1. V = R E: an orthonormal basis of E's row space (Gram-Schmidt, dependent rows dropped);
    //      V dv = vs (vs = R e) is the same constraint set.
    //   2. X <- (I - V'V) X + V'[0 | vs]: the accelerations' components along the constrained
    //      directions are replaced by their constrained values.  On the feasible set this is the
    //      same dv, so the QP's optimum is unchanged, but Hr = X'H_dv X loses the large curvature
    //      (and the gradient its large terms) in exactly the directions the rows fix -- with all
    //      rows independent of rank nv, X's y columns are exactly zero.
    //   3. [Q | q1] = L [V X | V x0 - vs]: the rows in y coordinates, orthonormalised.  The
    //      interior point and the refinement carry them as exact equality rows.
    static_assert(D::JG && D::NW <= kRow, "wheel rows: contact rows of J staged in LDS");
    constexpr int NW = D::NW, WEST = D::WEST, WAST = D::WAST;
    double* sWE = sm + D::O_WE;
    double* sWA = sm + D::O_WA;
    const double* wd = gwd + static_cast<size_t>(env) * NC * 6;
    for (int p = lane; p < NW * WEST; p += kWave) {
      const int w = p / WEST, c = p % WEST;
      const int i = w >> 1, side = w & 1;
      double acc = 0.0;
      if (c <= NV) {
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          const double dc = wd[i * 6 + side * 3 + q];
          const double v = (c == NV) ? gb[static_cast<size_t>(env) * S + JC0 + 3 * i + q]
                                     : sA[(3 * i + q) * NAP + c];   // contact row 3 i + q of J
          acc = fma(dc, v, acc);
        }
        if (c < NV && side == 0 && c == P->wheel_dof[i]) acc -= P->wheel_radius[i];
        acc *= (c == NV) ? -sMask[i] : sMask[i];
      } else {
        acc = (c - NV - 1 == w) ? 1.0 : 0.0;   // R accumulates here
      }
      sWE[p] = acc;
    }
    wave_sync();
    wave_mgs<NW, NV>(sWE, WEST, NV + 1 + NW, lane, 1e-9);   // rows [V | vs | R]
    wave_sync();
    int rank = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) rank += (sWE[w * WEST + w + NV + 1] != 0.0) ? 1 : 0;
    // P = V X - [0 | vs] and the identity columns of L
    for (int p = lane; p < NW * WAST; p += kWave) {
      const int w = p / WAST, c = p % WAST;
      double acc;
      if (c < NY1P) {
        acc = (c == NY) ? -sWE[w * WEST + NV] : 0.0;
#pragma unroll
        for (int j = 0; j < NV; ++j) acc = fma(sWE[w * WEST + j], sX[j * NY1P + c], acc);
      } else {
        acc = (c - NY1P == w) ? 1.0 : 0.0;
      }
      sWA[p] = acc;
    }
    wave_sync();
    // X <- X - V'P (rank nv: the y columns are the constrained accelerations' -- exactly zero)
    double* const wx = ws + static_cast<size_t>(env) * D::WS + D::W_X;
    for (int p = lane; p < NV * NY1P; p += kWave) {
      const int j = p / NY1P, c = p % NY1P;
      double v = sX[p];
#pragma unroll
      for (int w = 0; w < NW; ++w) v = fma(-sWE[w * WEST + j], sWA[w * WAST + c], v);
      v = (rank == NV && c < NY) ? 0.0 : v;
      sX[p] = v;
      wx[p] = v;
    }
    wave_sync();
    wave_mgs<NW, NY>(sWA, WAST, WAST, lane, 1e-9);   // rows [Q | q1 | 0 | L]
    wave_sync();
    double* const wsw = ws + static_cast<size_t>(env) * D::WS;
    for (int p = lane; p < NW * NY1P; p += kWave)
      wsw[D::W_AW + p] = sWA[(p / NY1P) * WAST + p % NY1P];
    for (int p = lane; p < NW * NV; p += kWave) wsw[D::W_WV + p] = sWE[(p / NV) * WEST + p % NV];
    for (int p = lane; p < NW * NW; p += kWave) {
      const int w = p / NW, c = p % NW;
      wsw[D::W_WR + p] = sWE[w * WEST + NV + 1 + c];
      wsw[D::W_WL + p] = sWA[w * WAST + NY1P + c];
    }
    // 4. T: an orthonormal basis of the y space whose first r' columns are Q's (nonzero) rows and
    //    the rest span their null space (Gram-Schmidt of [Q; I]).  The interior point and the
    //    refinement solve their Newton systems in y^ = T'y with the rows' coordinates pinned:
    //    the rows hold exactly, and nothing of the Hessian's curvature along them enters the
    //    factorisation.  X^ = X'T replaces X, so [Hr | g] below come out in these
    //    coordinates.
    double* sWT = sm + D::O_WT;
    for (int p = lane; p < (NW + NY) * NY; p += kWave) {
      const int w = p / NY, c = p % NY;
      sWT[p] = (w < NW) ? sWA[w * WAST + c] : ((c == w - NW) ? 1.0 : 0.0);
    }
    wave_sync();
    wave_mgs_lds(sWT, NW + NY, NY, NY, NY, lane, 1e-9, sWE);   // (sWE: copied out above, free)
    wave_sync();
    int kept = 0;
    for (int w = 0; w < NW + NY; ++w) {
      const double a = lane < NY ? sWT[w * NY + lane] : 0.0;
      if (wave_sum(a * a) > 0.0) {   // wave-uniform
        if (kept < NY) {
          if (lane < NY) sWT[kept * NY + lane] = a;   // in place: kept <= w
          if (lane == 0) wsw[D::W_PIN + kept] = (w < NW) ? static_cast<double>(w) : -1.0;
        }
        ++kept;
      }
      wave_sync();
    }
    for (int k = kept; k < NY; ++k) {   // (never in practice: a column short -> pinned at zero)
      if (lane < NY) sWT[k * NY + lane] = 0.0;
      if (lane == 0) wsw[D::W_PIN + k] = -2.0;
    }
    wave_sync();
    for (int p = lane; p < NY * NY; p += kWave) {
      const int i = p / NY, k = p % NY;
      wsw[D::W_T + p] = sWT[k * NY + i];   // T[i][k]
    }
    // X^ = X'T (y columns; the affine column stays), staged in sWE (free now)
    for (int p = lane; p < NV * NY; p += kWave) {
      const int j = p / NY, k = p % NY;
      double v = 0.0;
#pragma unroll 8
      for (int i = 0; i < NY; ++i) v = fma(sX[j * NY1P + i], sWT[k * NY + i], v);
      sWE[p] = v;
    }
    wave_sync();
    for (int p = lane; p < NV * NY; p += kWave) {
      const int j = p / NY, k = p % NY;
      sX[j * NY1P + k] = sWE[p];
      wx[j * NY1P + k] = sWE[p];
    }
    wave_sync();
  }
  // J, M, C dead from here on (R1, R2 get reused)

  STAMP_END(2);
  STAMP_BEGIN();
  // ---------------- Phase D: reduced Hessian / gradient ----------------------------------
  // Hr = X' T1 + 2 (w_tau + w_reg) I_u + 2 w_reg I_z,  g = last column,  T1 = H_dv X (+ f_dv in
  // the affine column).
  {
    // FP64 MFMA: T1 = H_dv X (+ f_dv in the affine column) as 16x16 tiles
    // kept in registers, then [Hr | g] = X' T1 with T1's registers as the B operand -- register
    // r of a T1 tile holds rows (l >> 4) + 4 r, exactly the k-rows of one 4-step -- so T1 never
    // goes through LDS.  X's fragments serve both products (B of the first, A of the second).
    constexpr int RB = (NV + 15) / 16, CB = (NY1P + 15) / 16, KS = (NV + 3) / 4;
    const int lc = lane & 15, lg = lane >> 4;
    double xf[KS][CB];   // X[4q + lg][16 cb + lc]
    double hf[RB][KS];   // H_dv[16 rb + lc][4q + lg]
#pragma unroll
    for (int q = 0; q < KS; ++q) {
      const int k = 4 * q + lg;
      const bool kv = k < NV;
#pragma unroll
      for (int cb = 0; cb < CB; ++cb) {
        const int col = 16 * cb + lc;
        const double x = sX[(kv ? k : 0) * NY1P + (col < NY1P ? col : 0)];
        xf[q][cb] = (kv && col < NY1P) ? x : 0.0;
      }
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) {
        const int row = 16 * rb + lc;
        const double h = sHa[(row < NV ? row : 0) * NA + (kv ? k : 0)];
        hf[rb][q] = (kv && row < NV) ? h : 0.0;
      }
    }
    d4 t1[RB][CB];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int cb = 0; cb < CB; ++cb)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int row = 16 * rb + lg + 4 * rr, col = 16 * cb + lc;
          const double f = sHa[(row < NV ? row : 0) * NA + NV];
          t1[rb][cb][rr] = (row < NV && col == NY) ? f : 0.0;
        }
#pragma unroll
    for (int q = 0; q < KS; ++q)
#pragma unroll
      for (int rb = 0; rb < RB; ++rb)
#pragma unroll
        for (int cb = 0; cb < CB; ++cb)
          t1[rb][cb] = __builtin_amdgcn_mfma_f64_16x16x4f64(hf[rb][q], xf[q][cb], t1[rb][cb], 0, 0, 0);
    const double wu2 = 2.0 * (P->w_torque + P->w_reg);
    const double wr2 = 2.0 * P->w_reg;
    double* wsv = ws + static_cast<size_t>(env) * D::WS;   // [Hr | g] out from registers
    constexpr int NT = CB * (CB + 1) / 2;   // upper block triangle, tiles interleaved per k-step
    d4 hacc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) hacc[t] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int q = 0; q < KS; ++q) {
      int t = 0;
#pragma unroll
      for (int ab = 0; ab < CB; ++ab)
#pragma unroll
        for (int bb = ab; bb < CB; ++bb, ++t)
          hacc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(xf[q][ab], t1[q / 4][bb][q % 4], hacc[t],
                                                         0, 0, 0);
    }
    int tt = 0;
#pragma unroll
    for (int ab = 0; ab < CB; ++ab)
#pragma unroll
      for (int bb = ab; bb < CB; ++bb, ++tt) {
        const d4 h = hacc[tt];
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int a = 16 * ab + lg + 4 * rr, b = 16 * bb + lc;
          const int kz = (a >= NU) ? (a - NU) / 3 : 0;
          const double mk = sMask[kz < NC ? kz : NC - 1];
          double v = h[rr];
          if (a <= b && b < NY1 && !(a == NY && b == NY)) {
            if (b < NY && D::WH) {
              // rotated coordinates: + T'WT, W = 2 (w_tau + w_reg) on u, 2 w_reg on z, 1 on a
              // masked contact's (pinned) z -- whose coordinate T keeps as a unit vector
              const double* sT = sm + D::O_WT;
              double wab = 0.0;
#pragma unroll 8
              for (int i = 0; i < NY; ++i) {
                const int ki = (i >= NU) ? (i - NU) / 3 : 0;
                const double wi = (i < NU) ? wu2 : (sMask[ki] == 0.0 ? 1.0 : wr2);
                wab = fma(wi * sT[a * NY + i], sT[b * NY + i], wab);
              }
              v += wab;
              wsv[D::W_HR + a * NY + b] = v;
              wsv[D::W_HR + b * NY + a] = v;
            } else if (b < NY) {
              if (a == b && a < NU) v += wu2;
              if (a == b && a >= NU) v = (mk == 0.0) ? 1.0 : v + wr2;   // pinned z: identity row
              wsv[D::W_HR + a * NY + b] = v;
              wsv[D::W_HR + b * NY + a] = v;
            } else {
              wsv[D::W_G + a] = v;
            }
          }
        }
      }
    wave_sync();
  }

  STAMP_END(4);
  STAMP_BEGIN();
  // (X, H_dv, f_dv and [Hr | g] were stored to the workspace where they were formed)
  STAMP_END(5);
  STAMP_STORE_SETUP();
}

// The assembly grid maps block b to env b: an XCD-aware order that put each env's assembly on
// the XCD of its interior-point block measured no change (Go2 4,096 0.1819 vs 0.1815 ms).
template <class D>
__global__ __launch_bounds__(kWave, 2) void osc_setup_kernel(
    const DevParams* __restrict__ P, int nenv, const double* __restrict__ gM,
    const double* __restrict__ gC, const double* __restrict__ gJ, const double* __restrict__ gb,
    const double* __restrict__ gT, const double* __restrict__ gmask, double* __restrict__ ws,
    const double* __restrict__ gwd) {
  __shared__ __attribute__((aligned(16))) double sm[D::SMEM];
  setup_env<D>(P, static_cast<int>(blockIdx.x), nenv, gM, gC, gJ, gb, gT, gmask, ws, sm, gwd);
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

// Two models' setup in one grid (BASELINE configs[4]: Go2 + WaLTER on one GPU): blocks
// [0, A.nenv) are model A's envs, the rest model B's.  One launch, so the second model's
// wavefronts fill the SIMDs the first model's leave, instead of two grids contending.
template <class DA, class DB>
__global__ __launch_bounds__(kWave, 2) void osc_setup_pair_kernel(PairArgs A, PairArgs B) {
  __shared__ __attribute__((aligned(16))) double sm[cmax(DA::SMEM, DB::SMEM)];
  const int blk = static_cast<int>(blockIdx.x);
  if (blk < A.nenv)
    setup_env<DA>(A.P, blk, A.nenv, A.M, A.C, A.J, A.b, A.T, A.mask, A.ws, sm, nullptr);
  else
    setup_env<DB>(B.P, blk - A.nenv, B.nenv, B.M, B.C, B.J, B.b, B.T, B.mask, B.ws, sm, nullptr);
}

// ============================ kernel 2: interior point, 4 env / wave ========================

// a += bcast_K(src) * ma;  b += bcast_K(src) * mb  (one broadcast source, two slots).
// NOP = true guards a source that a VALU instruction may have written just before.
template <int K, bool NOP>
__device__ __forceinline__ void fmac_bcast2(double& a, double& b, double src, double ma, double mb) {
  if constexpr (NOP)
    asm volatile("s_nop 1\n\t"
                 "v_fmac_f64_dpp %0, %2, %3 row_newbcast:%5 row_mask:0xf bank_mask:0xf\n\t"
                 "v_fmac_f64_dpp %1, %2, %4 row_newbcast:%5 row_mask:0xf bank_mask:0xf"
                 : "+v"(a), "+v"(b) : "v"(src), "v"(ma), "v"(mb), "n"(K));
  else
    asm volatile("v_fmac_f64_dpp %0, %2, %3 row_newbcast:%5 row_mask:0xf bank_mask:0xf\n\t"
                 "v_fmac_f64_dpp %1, %2, %4 row_newbcast:%5 row_mask:0xf bank_mask:0xf"
                 : "+v"(a), "+v"(b) : "v"(src), "v"(ma), "v"(mb), "n"(K));
}

template <int N>
__device__ __forceinline__ void dot_rows(double& a, double& b, double x0, double x1,
                                         const double (&ma)[N], const double (&mb)[N]) {
  double a2 = 0.0, b2 = 0.0;                // two chains: no back-to-back dependent f64 ops
  static_for<0, N>([&](auto ic) {
    constexpr int i = decltype(ic)::value;
    if constexpr (i % 2 == 0)
      fmac_bcast2<i % kRow, i % kRow == 0>(a, b, i < kRow ? x0 : x1, ma[i], mb[i]);
    else
      fmac_bcast2<i % kRow, false>(a2, b2, i < kRow ? x0 : x1, ma[i], mb[i]);
  });
  a += a2;
  b += b2;
}

// LDL^T of an N x N symmetric matrix held one column per lane in two slots: lane l of a row
// holds column l in c0 and column l+16 in c1.  Right-looking; at step k every lane j > k
// applies  c_j[i] -= L[i][k] L[j][k] D_k  for i > k with the pivot column entry c_k[i]
// broadcast by DPP straight into the FMA.  On exit (for slot column j):
//   c[i], i > j : -L[i][j] D[j] / D[i]  (column j of L, unscaled, times -1/D_i: backward solve)
//   c[i], i < j : -L[j][i]              (row j of L: forward solve)
//   c[j]        : -1
//   dinv0, dinv1: 1 / D[j]
// thr0, thr1: 1e-13 x the original diagonal (Cholesky-infinity test: a pivot not above it
// becomes 1e128).  sdinv: 2 x 16 doubles of LDS for this row: every lane writes 1/D_k at step k
// (one ds_write instead of a lane select), each lane reads its own two back at the end.
// Slot-1 lanes past N (N < 32) hold a copy of column N-1 (the caller loads jj1 = N-1 there);
// they are left unmasked while column N-1 is still active, so they stay an exact mirror of it --
// finite, and never a broadcast source.
// Look-ahead: pivot k+1's test, broadcast, reciprocal and scaling are issued right after step k's
// first trailing FMA pair (which finalises column k+1's entry), so their dependent chain overlaps
// the rest of step k's FMAs instead of stalling between the steps (bitwise the same factor;
// profiles/r04f_ab_ldl_lookahead.jsonl: Go2 4,096 0.1737 -> 0.1721 ms per solve, 65,536 1.782 ->
// 1.762, WaLTER 4,096 0.2804 -> 0.2758).
// (Fusing pass 0's forward elimination into the factorisation -- the right-hand side formed
// first, its step k riding along the factor's -- measured within noise: Go2 4,096 0.1739 vs
// 0.1718 ms per solve, 65,536 1.760 vs 1.748, WaLTER 4,096 0.2754 vs 0.2768, and not bitwise;
// profiles/r04k/ab_fwd_fused.jsonl.)
template <int N>
__device__ __forceinline__ void ldl_rows(double (&c0)[N], double (&c1)[N], double* sdinv, int l,
                                         double& dinv0, double& dinv1, double thr0, double thr1) {
  // pivot k's preparation: -> (t0, t1) = -L[lane][k] for the lanes still to be eliminated
  auto prep = [&](auto kc, double& t0, double& t1) {
    constexpr int k = decltype(kc)::value;
    constexpr int s = k / kRow, kl = k % kRow;
    const double own = (s == 0) ? c0[k] : c1[k];
    const double dk = bcast_guarded<kl>(own > ((s == 0) ? thr0 : thr1) ? own : 1e128);
    const double inv = recip1(dk);
    sdinv[k] = inv;
    c0[k] = -c0[k] * inv;
    c1[k] = -c1[k] * inv;
    t0 = keep_lanes<rows_mask(lanes_from(k + 1, 15))>(c0[k]);
    constexpr unsigned kT1 = (k < kRow) ? 0xFFFFu : lanes_from(k + 1 - kRow, N - 1 - kRow);
    t1 = keep_lanes<rows_mask(kT1)>(c1[k]);
  };
  // one trailing FMA pair of step k, row i (NOP: the DPP source was written just before)
  auto upd = [&](auto kc, auto ic, double t0, double t1) {
    constexpr int k = decltype(kc)::value, i = decltype(ic)::value;
    constexpr int s = k / kRow, kl = k % kRow;
    constexpr bool nop = (i == k + 1) && (k >= 1) && (i == N - 1);
    if constexpr (s == 0) {
      fmac_bcast<kl, nop>(c1[i], c0[i], t1);
      if constexpr (k < kRow - 1) fmac_bcast_self<kl>(c0[i], t0);
    } else {
      fmac_bcast_self<kl, nop>(c1[i], t1);
    }
  };
  double ta0, ta1;
  prep(std::integral_constant<int, 0>{}, ta0, ta1);
  static_for<0, N>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    double tb0 = 0.0, tb1 = 0.0;
    if constexpr (k + 1 < N) {
      upd(kc, std::integral_constant<int, k + 1>{}, ta0, ta1);
      prep(std::integral_constant<int, k + 1>{}, tb0, tb1);
    }
    static_for<k + 2, N>([&](auto ic) { upd(kc, ic, ta0, ta1); });
    ta0 = tb0;
    ta1 = tb1;
  });
  wave_sync();
  dinv0 = sdinv[l];
  dinv1 = sdinv[(l + kRow < N) ? l + kRow : N - 1];
}

// Solve K x = r with the factor above; r0 (var l), r1 (var l+16) in, x out.  Every lane of
// the row is updated at every step (no lane masks): a lane whose value is already final saves
// it at its own pivot step and may take garbage afterwards.  The factor's row k is pre-scaled
// by -1/D_k (ldl_rows), so each step is the pivot's broadcast straight into the FMAs -- no
// multiply in the dependency chain (Go2 4,096: 0.183 -> 0.178 ms per solve;
// profiles/r03_ab_ldl_prescale.txt):
//   forward   z = L^-1 r             a_j += a_k * (-L[j][k])
//   backward  in D-scaled form       a_j += a_k * (-L[k][j] D_j / D_k),  x_j = a_j / D_j
// The other slot's FMA goes first: the own slot's FMA rewrites the pivot lane (c[k] = -1 there).
// (Masking each FMA to the lanes it may change through EXEC instead of saving was measured
// slower: 0.186 ms -- the EXEC writes cost more than the two v_cndmask they replace.)
// (ldl_fwd_rows / ldl_bwd_rows: the two halves, for callers that act on z in between.)
template <int N>
__device__ __forceinline__ void ldl_fwd_rows(const double (&c0)[N], const double (&c1)[N],
                                             double dinv0, double dinv1,
                                             double& a0, double& a1, int l) {
  double z0 = 0.0, z1 = 0.0;                // z_j, saved at step j
  static_for<0, N>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    constexpr int s = k / kRow, kl = k % kRow;
    constexpr unsigned long long kPiv = rows_mask(1u << kl);
    if constexpr (s == 0) {
      z0 = select_lanes<kPiv>(a0, z0);
      const double p = a0;
      fmac_bcast<kl, true>(a1, p, c1[k]);
      if constexpr (k < kRow - 1) fmac_bcast<kl>(a0, p, c0[k]);
    } else {
      z1 = select_lanes<kPiv>(a1, z1);
      const double p = a1;
      fmac_bcast<kl, true>(a1, p, c1[k]);
    }
  });
  a0 = z0;
  a1 = z1;
}
template <int N>
__device__ __forceinline__ void ldl_bwd_rows(const double (&c0)[N], const double (&c1)[N],
                                             double dinv0, double dinv1,
                                             double& a0, double& a1, int l) {
  double x0 = 0.0, x1 = 0.0;                // D-scaled x_j, saved at step j
  static_for<0, N>([&](auto kc) {
    constexpr int k = N - 1 - decltype(kc)::value;
    constexpr int s = k / kRow, kl = k % kRow;
    constexpr unsigned long long kPiv = rows_mask(1u << kl);
    if constexpr (s == 0) {
      x0 = select_lanes<kPiv>(a0, x0);
      const double p = a0;
      if constexpr (k >= 1) fmac_bcast<kl, true>(a0, p, c0[k]);
    } else {
      x1 = select_lanes<kPiv>(a1, x1);
      const double p = a1;
      fmac_bcast<kl, true>(a0, p, c0[k]);
      if constexpr (k > kRow) fmac_bcast<kl>(a1, p, c1[k]);
    }
  });
  a0 = x0 * dinv0;
  a1 = x1 * dinv1;
}
template <int N>
__device__ __forceinline__ void ldl_solve_rows(const double (&c0)[N], const double (&c1)[N],
                                               double dinv0, double dinv1,
                                               double& a0, double& a1, int l) {
  ldl_fwd_rows<N>(c0, c1, dinv0, dinv1, a0, a1, l);
  ldl_bwd_rows<N>(c0, c1, dinv0, dinv1, a0, a1, l);
}

// WARM = false compiles none of the warm-start / fix-up logic (the cold solve's register budget
// is unchanged by it: the two-wave Go2 variant would otherwise spill more).
// LDS doubles of one IPM wavefront.  The one-wave variant must run ONE wavefront per SIMD: when
// its registers would allow two, the LDS request (> 160 KB / 5 per workgroup) is what keeps the
// dispatcher from stacking a fifth and sixth workgroup on some CUs while others idle (Go2 in
// torque coordinates: 26 KB of LDS, 255 VGPRs -> IPM 144 -> 158 us at 4,096 envs until padded).
// The refinement pass (REFINE) streams Hr from L2 and keeps instead each env's [X | H_dv | f_dv]
// block of the workspace in LDS (RefineLds).
template <class D>
struct RefineLds {
  static constexpr int X = 0;
  static constexpr int HD = D::NV * D::NY1P;
  static constexpr int GD = HD + D::NV * D::NV;
  static constexpr int SIZE = GD + even(D::NV);   // = W_SOL - W_X in the workspace
};
// Refinement modes of the IPM body: none (the interior point alone, handing its result to
// osc_refine_kernel through W_SOL: warm-started solves past one wave per SIMD, whose fused kernel
// spills, and models created with osc_model_tuning.refine_steps = 0), the refinement pass alone
// (osc_refine_kernel), or both in one wavefront (every cold solve and the one-wave warm solve:
// no hand-off, no second launch).
constexpr int kRfNone = 0, kRfOnly = 1, kRfFused = 2;
// Full-space refinement without wheel rows: rounds of active-set changes, and
// steps per round at most (each env stops at its own convergence, at least refine_steps)
constexpr int kRefineRounds = 8, kRefineMaxSteps = 8;
template <class D, bool SMALL, int RF>
constexpr bool ipm_hrl() {   // Hr kept in LDS across the interior point's iterations
  return SMALL && RF != kRfOnly && hr_fits_lds<D>();
}
// LDS doubles per env beyond the interior point's layout: the refinement's [X | H_dv | f_dv]
// block, except that a fused pass with Hr in LDS moves X into Hr's region once the first K_A is
// assembled (registers hold it from then on) and only keeps [H_dv | f_dv] apart.
// WH: the wheel rows' LDS block of an env: the rotation T (T[i][k] at i * TST + k; odd stride:
// lanes reading a row of T or a column hit distinct banks), the Q row each column of T carries
// (-1: free), q1 per Q row, a staging vector for the rotations, and the rows' multipliers.
template <class D>
struct WheelLds {
  static constexpr int NW = D::NW, NY = D::NY, TST = NY + 1;
  static constexpr int T = 0;
  static constexpr int PIN = even(NY * TST);
  static constexpr int Q1 = PIN + even(NY);
  static constexpr int ROT = Q1 + even(NW);
  static constexpr int NUV = ROT + even(NY);
  static constexpr int SIZE = NUV + even(NW);
};
template <class D, bool SMALL, int RF>
constexpr int refine_lds_extra() {
  if constexpr (D::WH && RF == kRfFused) return WheelLds<D>::SIZE;   // (reads [X | ..] from L2)
  else if constexpr (RF == kRfNone) return 0;
  else if constexpr (RF == kRfFused && !SMALL) return 0;   // reads [X | H_dv | f_dv] from L2
  else if constexpr (RF == kRfFused && ipm_hrl<D, SMALL, RF>())   // (DMA: whole 1 KB rows)
    return (((RefineLds<D>::SIZE - RefineLds<D>::HD) / 2 + kWave - 1) / kWave) * kWave * 2;
  else return RefineLds<D>::SIZE;
}
// Two-wave variant, measured and not adopted: capping the waves resident per CU so
// each XCD's Hr working set fits its L2 (slower: the eighth wave per CU hides issue latency), and
// Hr's upper triangle packed in LDS (2.5 % slower: at full occupancy the Hr loads' latency is
// already hidden, and the packed addressing costs issue slots).
template <class D, bool SMALL, int RF = kRfNone>
constexpr int ipm_lds_doubles() {
  constexpr int il = IpmLayout<D, ipm_hrl<D, SMALL, RF>()>::IL + refine_lds_extra<D, SMALL, RF>();
  return SMALL ? cmax(kEnvPerWave * il, 160 * 1024 / 5 / 8 + 2) : kEnvPerWave * il;
}

// The body of one IPM wavefront (envs 4 blk .. 4 blk + 3); `sm` is its ipm_lds_doubles<D, SMALL>
// doubles of LDS.  Wrapped by osc_ipm_kernel (one model) and osc_ipm_pair_kernel (two models).
// WARM = false compiles none of the warm-start / fix-up logic (the cold solve's register budget
// is unchanged by it: the two-wave Go2 variant would otherwise spill more).
template <class D, bool SMALL, bool WARM, int RF_ = kRfNone, int CP = kCpNone>
__device__ __forceinline__ void ipm_block(
    const DevParams* __restrict__ P, int blk, int nenv, const double* __restrict__ gmask,
    const double* __restrict__ ws, double* __restrict__ gtau, double* __restrict__ gx,
    int32_t* __restrict__ gstatus, int32_t* __restrict__ giters, double* __restrict__ gwarm,
    int flags, double* __restrict__ sm, ParkArgs PA = ParkArgs{}) {
  static_assert(CP == kCpNone || (!WARM && RF_ == kRfFused && !D::WH),
                "compaction: cold solves with the fused refinement only");
  constexpr int NV = D::NV, NU = D::NU, NC = D::NC, NY = D::NY, NY1P = D::NY1P, MI = D::MI,
                NRL = D::NRL;
  // flags: bit 0 = the cold fix-up pass after a warm-started solve, bit 1 = hand the multipliers
  // to the dual kernel (W_SOL q, W_NU)
  const bool fixup = (flags & 1) != 0;
  const bool want_dual = (flags & 2) != 0;
  constexpr int RF = RF_;
  constexpr bool REFINE = RF == kRfOnly;      // the refinement pass alone (no interior point)
  constexpr bool HRL = ipm_hrl<D, SMALL, RF>();
  using LY = IpmLayout<D, HRL>;
  const int lane = threadIdx.x;
  const int grp = lane / kRow, l = lane % kRow;
  // resume pass: the wave's rows are parked slots (env_raw), their envs from the slot list
  const int cnt = CP == kCpResume ? *PA.count : nenv;
  if (CP == kCpResume && blk * kEnvPerWave >= cnt) return;
  const int env_raw = blk * kEnvPerWave + grp;
  const bool valid = env_raw < cnt;
  const int env = CP == kCpResume ? PA.list[valid ? env_raw : cnt - 1]
                                  : (valid ? env_raw : nenv - 1);   // spare rows replay the last
                                                                     // env, write nothing
  // Fix-up pass after a warm-started solve: only wavefronts holding an env that did not converge
  // run (cold, from the same workspace); only those envs' outputs are rewritten.
  bool write_out = valid;
  if constexpr (WARM) {
    // (an env whose refinement found no KKT point, OSC_SOLVE_UNREFINED, too: the warm start can
    // leave the interior point's early stop with an active set the refinement cannot repair,
    // ~1 env in 4,096 x 10 joint-state ticks; the cold fix-up solve runs to mu <= 1e-12)
    const bool redo = valid && fixup && gstatus[env] != OSC_SOLVE_OK;
    if (fixup && __ballot(redo) == 0) return;
    write_out = valid && (!fixup || redo);
  }

  constexpr int kEnvLds = LY::IL + refine_lds_extra<D, SMALL, RF>();
  double* B = sm + grp * kEnvLds;
  // refinement: [X | H_dv | f_dv] of this env; a fused pass with Hr in LDS keeps X in Hr's region
  constexpr bool kXinHr = RF == kRfFused && HRL;
  double* sRX = kXinHr ? B + LY::I_HR : B + LY::IL + RefineLds<D>::X;
  double* sRH = kXinHr ? B + LY::IL : B + LY::IL + RefineLds<D>::HD;
  double* sRG = sRH + (RefineLds<D>::GD - RefineLds<D>::HD);
  // Two-wave variant with the refinement fused: no LDS for [X | H_dv | f_dv] (two waves per SIMD
  // need <= 20 KB per wave), the refinement reads them from the workspace (L2 / Infinity Cache)
  // (the pointers are formed after the interior-point loop: nothing extra lives across it)
  // (so does a model with wheel rows: its LDS block holds the rows A~ instead)
  constexpr bool kRefG = RF == kRfFused && (!SMALL || D::WH);
  constexpr bool WHR = D::WH && RF == kRfFused;   // the wheel rows' rotated Newton systems
  using WL = WheelLds<D>;
  double* sWT = B + LY::IL + WL::T;
  double* sWPin = B + LY::IL + WL::PIN;
  double* sWQ1 = B + LY::IL + WL::Q1;
  double* sWRot = B + LY::IL + WL::ROT;
  double* sWNu = B + LY::IL + WL::NUV;
  // Hr columns are addressed as wave-uniform base (SGPR pair) + 32-bit lane offset + immediate:
  // 64-bit per-lane address registers for 48 loads do not fit, and their spill reloads
  // (scratch loads share vmcnt) used to serialise the whole prefetch.
  // (resume pass: the rows' envs are anywhere in the batch -- the base is the workspace itself
  // and the lane offset the env's whole one; launch_t keeps nenv x WS below 2^32 doubles)
  const double* __restrict__ wsw =
      ws + (CP == kCpResume ? size_t{0} : static_cast<size_t>(blk) * kEnvPerWave * D::WS) +
      D::W_HR;   // L2-resident
  const unsigned lane_off =
      static_cast<unsigned>(CP == kCpResume ? env : env - blk * kEnvPerWave) *
      static_cast<unsigned>(D::WS);
  double* sG = B + LY::I_G;
  double* sVy = B + LY::I_VY;
  double* sVy2 = B + LY::I_VY2;
  double* sVr = B + LY::I_VR;
  double* sDr = B + LY::I_DR;
  double* sMask = B + LY::I_MASK;
  double* sTau = B + LY::I_TAU;
  double* sXb = B + LY::I_XB;

  STAMP_DECL
  STAMP_BEGIN();
  // stage [g (| Hr)] (the workspace prefix has the LDS layout) and the mask: all loads in
  // flight before the first LDS store
  static_assert(LY::STAGE % 2 == 0 && NC <= kRow, "staging layout");
  {
    Batch2<LY::STAGE / 2, kRow> bs;
    bs.load(ws + static_cast<size_t>(env) * D::WS, l);
    const double mk = gmask[static_cast<size_t>(env) * NC + (l < NC ? l : 0)];
    if constexpr (RF == kRfFused && !kRefG && !kXinHr) {
      // the refinement's own LDS block is free all along: its [X | H_dv | f_dv] is staged now,
      // in the same memory latency (with Hr in LDS, [H_dv | f_dv] and X come by DMA later instead)
      static_assert(RefineLds<D>::SIZE % 2 == 0 && D::W_X % 2 == 0, "16-byte staging");
      Batch2<RefineLds<D>::SIZE / 2, kRow> bx;
      bx.load(ws + static_cast<size_t>(env) * D::WS + D::W_X, l);
      bx.store(sRX, l);
    }
    if constexpr (WHR) {   // T, the pin map, q1
      const double* we = ws + static_cast<size_t>(env) * D::WS;
#pragma unroll 8
      for (int p = l; p < NY * NY; p += kRow) sWT[(p / NY) * WL::TST + p % NY] = we[D::W_T + p];
      for (int p = l; p < NY; p += kRow) sWPin[p] = we[D::W_PIN + p];
      if (l < D::NW) {
        sWQ1[l] = we[D::W_AW + l * NY1P + NY];
        sWNu[l] = 0.0;
      }
    }
    bs.store(B, l);
    if (l < NC) sMask[l] = mk;
  }
  const double* sHr = B + LY::I_HR;
  wave_sync();

  // ---- inequality rows of this lane: r = l + 16 t.  Only (active, h) are kept; the row's
  // kind (torque bound q / sign, or contact k / pyramid side) is recomputed from r. ----
  bool act[NRL];
  double h[NRL];
#pragma unroll
  for (int t = 0; t < NRL; ++t) {
    const int r = l + kRow * t;
    act[t] = false;
    h[t] = 0.0;
    if (r < 2 * NU) {
      const int q = r >> 1;
      const double sg = (r & 1) ? -1.0 : 1.0;
      const double bnd = (r & 1) ? P->u_lb[q] : P->u_ub[q];
      act[t] = fabs(bnd) < P->inf_thresh;
      h[t] = sg * bnd;                                     // the row is +-y_q
    } else if (r < MI) {
      const int k = (r - 2 * NU) / 6, rt = (r - 2 * NU) % 6;
      const double m = sMask[k];
      if (m != 0.0) {
        if (rt < 4) {
          act[t] = true;                                   // friction pyramid, bineq = 0
        } else if (rt == 4) {
          const double lb = P->z_lb[2] * m;                // -fz <= -lb
          act[t] = fabs(lb) < P->inf_thresh;
          h[t] = -lb;
        } else {
          const double ub = P->z_ub[2] * m;                // fz <= ub
          act[t] = fabs(ub) < P->inf_thresh;
          h[t] = ub;
        }
      }
    }
  }
  const double mu_f = P->mu;
  // Rows of the initial least-squares fit (Hr + G'G) y0 = -g + G'h: every active row except
  // fz <= big_number, which would drag fz to ~big_number/2 together with fz >= 0 and start
  // the torque rows far outside their box (tools/ipm_model.py "y0_nofz": Go2 lockstep
  // iterations 14.9 -> 12.6, worst case 22 -> 18).
  auto init_ls = [&](int t) -> bool {
    const int r = l + kRow * t;
    return act[t] && !(r >= 2 * NU && (r - 2 * NU) % 6 == 5);
  };
  STAMP_END(0);

  // (G v)_r for all row slots at once, branch-free, every read issued first (one-wave variant):
  // torque rows read y_q, contact rows read their contact's three force entries.
  auto Gv_all = [&](const double* v, double (&out)[NRL]) {
    double uq[NRL], f0[NRL], f1[NRL], f2[NRL];
#pragma unroll
    for (int t = 0; t < NRL; ++t) {
      const int r = l + kRow * t;
      const int q = (r < 2 * NU) ? (r >> 1) : 0;
      const int k = (r >= 2 * NU && r < MI) ? (r - 2 * NU) / 6 : 0;
      uq[t] = v[q];
      f0[t] = v[NU + 3 * k];
      f1[t] = v[NU + 3 * k + 1];
      f2[t] = v[NU + 3 * k + 2];
    }
#pragma unroll
    for (int t = 0; t < NRL; ++t) {
      const int r = l + kRow * t;
      const int rt = (r - 2 * NU) % 6;
      const double sx = (rt & 1) ? -1.0 : 1.0, sy = (rt >= 2) ? -1.0 : 1.0;
      const double pyr = sx * f0[t] + sy * f1[t] - mu_f * f2[t];
      const double crow = (rt < 4) ? pyr : ((rt == 4) ? -f2[t] : f2[t]);
      const double trow = (r & 1) ? -uq[t] : uq[t];
      out[t] = !act[t] ? 0.0 : ((r < 2 * NU) ? trow : crow);
    }
  };
  // (G v)_r for row slot t
  auto Gv = [&](const double* v, int t) -> double {
    if (!act[t]) return 0.0;
    const int r = l + kRow * t;
    if (r < 2 * NU) {
      const double uq = v[r >> 1];
      return (r & 1) ? -uq : uq;
    }
    const int k = (r - 2 * NU) / 6, rt = (r - 2 * NU) % 6;
    const int z0 = NU + 3 * k;
    if (rt < 4) {
      const double sx = (rt & 1) ? -1.0 : 1.0, sy = (rt >= 2) ? -1.0 : 1.0;
      return sx * v[z0] + sy * v[z0 + 1] - mu_f * v[z0 + 2];
    }
    return (rt == 4) ? -v[z0 + 2] : v[z0 + 2];
  };
  // variable slots of this lane: j = l + 16 s
  const int j0 = l, j1 = l + kRow;
  const bool v1 = j1 < NY;
  const int jj1 = v1 ? j1 : NY - 1;
  const int jk0 = (j0 >= NU) ? (j0 - NU) / 3 : -1, jc0 = (j0 >= NU) ? (j0 - NU) % 3 : 0;
  const int jk1 = (v1 && j1 >= NU) ? (j1 - NU) / 3 : -1, jc1 = (j1 >= NU) ? (j1 - NU) % 3 : 0;
  // (G' w)_j for row-space w staged in LDS (inactive rows hold 0)
  // (G' w)_j for both variable slots of this lane, w row-space in LDS (inactive rows hold 0).
  // All reads are issued before the arithmetic (one wait, not one per torque row); the contact
  // part is branch-free: each lane reads its contact's six rows (16-byte pairs) and keeps the
  // combination of its component jc.
  auto contact_term = [&](const double* w, int jk, int jc) -> double {
    const double* wk = w + 2 * NU + 6 * (jk >= 0 ? jk : 0);
    const double2 a = *reinterpret_cast<const double2*>(wk);
    const double2 b = *reinterpret_cast<const double2*>(wk + 2);
    const double2 c = *reinterpret_cast<const double2*>(wk + 4);
    const double v0 = a.x - a.y + b.x - b.y;
    const double v1 = a.x + a.y - b.x - b.y;
    const double v2 = -mu_f * (a.x + a.y + b.x + b.y) - c.x + c.y;
    const double v = (jc == 0) ? v0 : ((jc == 1) ? v1 : v2);
    return jk >= 0 ? v : 0.0;
  };
  auto GTw2 = [&](const double* w, double& r0, double& r1) {
    // torque rows +-e_q: lane j0 < NU picks up w[2 j0] - w[2 j0 + 1]; slot j1 >= 16 > NU is a
    // contact variable
    const double2 p = *reinterpret_cast<const double2*>(w + 2 * (j0 < NU ? j0 : 0));
    const double k0 = contact_term(w, jk0, jc0), k1 = contact_term(w, jk1, jc1);
    r0 = (j0 < NU ? p.x - p.y : 0.0) + k0;
    r1 = k1;
  };
  // contact block column (B[0..2][jc]) of var slot in contact jk, from D = lambda/s
  auto contact_col = [&](int jk, int jc, double& v0, double& v1_, double& v2) {
    const double* dk = sDr + 2 * NU + 6 * jk;
    const double s4 = dk[0] + dk[1] + dk[2] + dk[3];
    const double sxy = dk[0] - dk[1] - dk[2] + dk[3];
    const double sx = dk[0] - dk[1] + dk[2] - dk[3];
    const double sy = dk[0] + dk[1] - dk[2] - dk[3];
    const double b00 = s4, b11 = s4, b01 = sxy, b02 = -mu_f * sx, b12 = -mu_f * sy,
                 b22 = mu_f * mu_f * s4 + dk[4] + dk[5];
    v0 = (jc == 0) ? b00 : (jc == 1) ? b01 : b02;
    v1_ = (jc == 0) ? b01 : (jc == 1) ? b11 : b12;
    v2 = (jc == 0) ? b02 : (jc == 1) ? b12 : b22;
  };

  // Wheel no-slip rows (WH): Q [y; 1] = 0, orthonormal rows (setup_env).  The Newton systems of
  // the interior point and the refinement are solved in y^ = T'y, T = [rows of Q | null-space
  // basis] (setup_env): K^ = H^ + sum_r D_r (T'g_r)(T'g_r)' assembled from the rows g_r of G one
  // original coordinate at a time (no cancellation of large entries), the coordinates along Q's
  // rows pinned (identity rows, step = -(Q y + q1): the rows hold after every step).  The
  // iterate itself stays in y coordinates.  (An earlier Schur-complement treatment of the rows on
  // K's factor lost the Newton steps' accuracy next to nearly dependent active rows: DESIGN.md §3.)
  constexpr int NW = D::NW;
  // this lane's slots: pinned?  (the Q row's q1 for the residual)
  bool pin0 = false, pin1 = false;
  double q10 = 0.0, q11 = 0.0;
  auto rot_load_pins = [&]() {
    if constexpr (WHR) {
      const double p0v = sWPin[j0], p1v = sWPin[jj1];
      pin0 = p0v != -1.0;
      pin1 = v1 && p1v != -1.0;
      q10 = p0v >= 0.0 ? sWQ1[static_cast<int>(p0v)] : 0.0;
      q11 = (v1 && p1v >= 0.0) ? sWQ1[static_cast<int>(p1v)] : 0.0;
    }
  };
  // T'v and T v for a y-space vector held in the lane slots (staged through sWRot)
  auto rot_in = [&](double v0, double v1v, double& o0, double& o1) {
    wave_sync();
    sWRot[j0] = v0;
    if (v1) sWRot[j1] = v1v;
    wave_sync();
    double a0 = 0.0, a1 = 0.0;
#pragma unroll
    for (int i = 0; i < NY; ++i) {
      const double r = sWRot[i];
      a0 = fma(sWT[i * WL::TST + j0], r, a0);
      a1 = fma(sWT[i * WL::TST + jj1], r, a1);
    }
    o0 = a0;
    o1 = a1;
    wave_sync();
  };
  auto rot_out = [&](double v0, double v1v, double& o0, double& o1) {
    wave_sync();
    sWRot[j0] = v0;
    if (v1) sWRot[j1] = v1v;
    wave_sync();
    double a0 = 0.0, a1 = 0.0;
#pragma unroll
    for (int k = 0; k < NY; ++k) {
      const double r = sWRot[k];
      a0 = fma(sWT[j0 * WL::TST + k], r, a0);
      a1 = fma(sWT[jj1 * WL::TST + k], r, a1);
    }
    o0 = a0;
    o1 = a1;
    wave_sync();
  };
  // rq: the rows' residual at the current y, on the pinned slots (q1 at the start, y = 0)
  double rq0 = 0.0, rq1 = 0.0, rwmax = 0.0;
  rot_load_pins();
  rq0 = pin0 ? q10 : 0.0;
  rq1 = pin1 ? q11 : 0.0;

  double c0[NY], c1[NY];
  double dinv0, dinv1;
  // WH: c0 / c1 hold H^'s columns j0, jj1; add T'(G'DG)T from sDr (D per row slot) one original
  // coordinate i at a time -- column j gains coef_i(j) T[i][:], coef_i(j) = (G'DG)[i][:] T[:][j]
  // (torque rows: diagonal; a contact's rows: its 3 x 3 block) -- then pin Q's coordinates.
  // Returns the assembled diagonal entries (the pivot threshold's reference).
  auto assemble_rot = [&](double& dg0r, double& dg1r) {
    if constexpr (WHR) {
#pragma unroll
      for (int i = 0; i < NY; ++i) {
        double a0, a1;
        if (i < NU) {
          const double d = sDr[2 * i] + sDr[2 * i + 1];
          a0 = d * sWT[i * WL::TST + j0];
          a1 = d * sWT[i * WL::TST + jj1];
        } else {
          const int k = (i - NU) / 3, ci = (i - NU) % 3, zb = NU + 3 * k;
          double b0, b1, b2;   // row ci of contact k's block (symmetric: its column ci)
          contact_col(k, ci, b0, b1, b2);
          a0 = b0 * sWT[zb * WL::TST + j0] + b1 * sWT[(zb + 1) * WL::TST + j0] +
               b2 * sWT[(zb + 2) * WL::TST + j0];
          a1 = b0 * sWT[zb * WL::TST + jj1] + b1 * sWT[(zb + 1) * WL::TST + jj1] +
               b2 * sWT[(zb + 2) * WL::TST + jj1];
        }
#pragma unroll
        for (int m = 0; m < NY; ++m) {
          const double t = sWT[i * WL::TST + m];
          c0[m] = fma(a0, t, c0[m]);
          c1[m] = fma(a1, t, c1[m]);
        }
      }
      double d0 = 0.0, d1 = 0.0;
#pragma unroll
      for (int m = 0; m < NY; ++m) {
        const bool pm = sWPin[m] != -1.0;
        c0[m] = pin0 ? ((m == j0) ? 1.0 : 0.0) : (pm ? 0.0 : c0[m]);
        c1[m] = pin1 ? ((m == jj1) ? 1.0 : 0.0) : (pm ? 0.0 : c1[m]);
        d0 = (m == j0) ? c0[m] : d0;
        d1 = (m == jj1) ? c1[m] : d1;
      }
      dg0r = d0;
      dg1r = d1;
    }
  };
  // One-wave variant whose Hr does not fit the LDS (WaLTER: 32 x 32 x 4 envs): the lane's two Hr
  // columns are loaded once and kept in registers across the iterations (the one-wave kernel has
  // 512 of them, AGPRs included) instead of being re-read from L2 every iteration.
  // (not with wheel rows: their per-iteration products need the registers; Hr comes from L2)
  constexpr bool kHrReg = SMALL && !HRL && !D::WH;
  double hr0[kHrReg ? NY : 1], hr1[kHrReg ? NY : 1];
  if constexpr (kHrReg) {
#pragma unroll
    for (int i = 0; i < NY; ++i) {
      hr0[i] = wsw[lane_off + static_cast<unsigned>(i * NY + j0)];
      hr1[i] = wsw[lane_off + static_cast<unsigned>(i * NY + jj1)];
    }
  }
  // Hr columns j0, j1 (and their diagonal entries) -> registers; re-issued at the end of every
  // iteration so the loads fly while the step is applied and the next residuals are formed.
  auto load_hr = [&]() {
    // column bases formed here, every time (hidden from loop-invariant hoisting): kept live
    // across the loop they get spilled, and spill reloads wait on vmcnt(0)
    if constexpr (HRL) {
#pragma unroll
      for (int i = 0; i < NY; ++i) {
        c0[i] = sHr[i * NY + j0];
        c1[i] = sHr[i * NY + jj1];
      }
    } else if constexpr (kHrReg) {
#pragma unroll
      for (int i = 0; i < NY; ++i) {
        c0[i] = hr0[i];
        c1[i] = hr1[i];
      }
    } else {
      unsigned off = lane_off;
      asm volatile("" : "+v"(off));
      const double* p0 = wsw + off + j0;
      const double* p1 = wsw + off + jj1;
#pragma unroll
      for (int i = 0; i < NY; ++i) {
        c0[i] = p0[i * NY];
        c1[i] = p1[i * NY];
      }
    }
  };
  const double hdg0 = HRL ? sHr[j0 * NY + j0] : wsw[lane_off + static_cast<unsigned>(j0 * NY + j0)];
  const double hdg1 =
      HRL ? sHr[jj1 * NY + jj1] : wsw[lane_off + static_cast<unsigned>(jj1 * NY + jj1)];
  load_hr();
  const double g0 = sG[j0], g1 = sG[jj1];
  double y0 = 0.0, y1 = 0.0;
  double s[NRL], lam[NRL];
#pragma unroll
  for (int t = 0; t < NRL; ++t) {
    s[t] = 1.0;
    lam[t] = 0.0;
  }
  double nact = 0.0;
#pragma unroll
  for (int t = 0; t < NRL; ++t) nact += act[t] ? 1.0 : 0.0;
  const double m_act = row_sum(nact);
  bool done = !valid;
  int32_t st = OSC_SOLVE_MAX_ITER;
  int it_done = 0;
  bool stalled = false;   // WH: stopped by the late-stall exit, not at mu <= eps_mu

  // One loop body for everything, so factorisation and solve code exist once (I-cache).
  // it == -1 builds the initial point (Mehrotra-style):
  //   (Hr + G'G) y0 = -g + G'h,  s = h - G y0,  lambda = G y0 - h,  both shifted positive.
  // The four environments of the wave iterate in lockstep; a converged one stops moving
  // (step 0) until the slowest has converged.
  // Primal residual rp = G y + s - h.  Every step takes ds = -rp - G dy exactly, so the new
  // residual is (1 - alpha) rp up to rounding, whatever the accuracy of the linear solve: it is
  // carried while mu > 1e-6 and formed from scratch after the initial point and once mu is
  // small, where the ~1e-12 rounding the carried value ignores is as large as the active
  // slacks (tools/ipm_model.py "rpcarry1e-6": same iterations as recomputing every time).
  // rd, which does depend on the solve's accuracy, is recomputed every iteration.
  double rp[NRL];
#pragma unroll
  for (int t = 0; t < NRL; ++t) rp[t] = 0.0;
  // Warm start (the reference's OsqpSolver::SetWarmStart, operational_space_controller.h:525):
  // an env whose warm state is valid starts from the previous tick's y and lambda, with the
  // slacks s = max(h - G y, delta) and lambda = max(lambda_prev, delta) (rows active now but not
  // before start at delta).  A wave whose four envs are all warm skips the least-squares initial
  // point; otherwise it runs it and the warm rows override it at iteration 0.  An env without
  // active rows always starts cold (its initial point is then the exact optimum).
  // (nothing warm-related stays live across the loop but one lane mask: the 2-wave variant has
  // no registers to spare)
  // A contact-mode switch (mask differs from the state's) changes the QP's rows: start cold.
  bool warm = false;
  if (WARM && !fixup) {
    const double* w0 = gwarm + static_cast<size_t>(env) * D::WW;
    const double same = (l >= NC || w0[D::WW_M + l] == sMask[l]) ? 1.0 : 0.0;
    warm = row_min(same) == 1.0 && w0[0] == 1.0 && m_act > 0.0;
  }
  bool any_warm = false, all_warm = false;
  if constexpr (WARM) {
    any_warm = __ballot(warm) != 0;
    all_warm = __ballot(!warm) == 0;
  }
  // Compaction (ParkArgs): the park slot's state, exactly as the park pass left it at the top of
  // iteration park_it (the y slots of every lane, v1 or not; s, lambda, rp of every row slot).
  const int pslot = env_raw < cnt ? env_raw : cnt - 1;
  auto park_at = [&](int slot) {
    return PA.park + static_cast<size_t>(slot) * park_doubles<D>();
  };
  auto resume_state = [&]() -> int {
    if constexpr (CP == kCpResume) {
      const double* pk = park_at(pslot);
      y0 = pk[l];
      y1 = pk[kRow + l];
#pragma unroll
      for (int t = 0; t < NRL; ++t) {
        s[t] = pk[2 * kRow + l + kRow * t];
        lam[t] = pk[2 * kRow + NRL * kRow + l + kRow * t];
        rp[t] = pk[2 * kRow + 2 * NRL * kRow + l + kRow * t];
      }
      sVy[j0] = y0;
      if (v1) sVy[j1] = y1;
      wave_sync();
    }
    return PA.park_it;
  };
  bool parked = false;   // park pass: this row's env went to the park area (no outputs here)
  bool refined = false;
  // WH with the duals requested: the wheel rows' multipliers for the dual kernel (W_NU; the
  // refinement's where it is kept, else the interior point's centre).  The dual kernel recovers
  // every other multiplier from the design vector itself.
  // (w = L' nu: the multipliers of the rows [V X | V x0 - vs] before their orthonormalisation,
  // which the dual kernel maps back to E's rows; every lane of the env's row takes part)
  auto put_wheel_duals = [&](double nu) {
    if constexpr (D::WH) {
      if (want_dual) {
        const double* Lw = ws + static_cast<size_t>(env) * D::WS + D::W_WL;
        const int lc = l < NW ? l : 0;
        double acc = 0.0;
        static_for<0, NW>([&](auto W) {
          constexpr int w = decltype(W)::value;
          acc = fma(Lw[w * NW + lc], bcast_guarded<w>(nu), acc);
        });
        if (write_out && l < NW)
          const_cast<double*>(ws)[static_cast<size_t>(env) * D::WS + D::W_NU + l] = acc;
      }
    }
  };
  // interior-point stop (the warm fix-up pass is a rescue: its cold solve runs to mu <= 1e-12)
  const double eps_run = (WARM && fixup) ? fmin(P->eps_mu, 1e-12) : P->eps_mu;
  if constexpr (REFINE) {
    // the interior point's result for this env (osc_ipm_kernel, W_SOL): y, and the active rows
    // as lambda > s with lambda = q > 0
    static_assert(D::W_SOL - D::W_X == RefineLds<D>::SIZE && D::W_X % 2 == 0 &&
                  RefineLds<D>::SIZE % 2 == 0, "refinement LDS block = workspace [X | H_dv | f_dv]");
    {
      Batch2<RefineLds<D>::SIZE / 2, kRow> bx;
      bx.load(ws + static_cast<size_t>(env) * D::WS + D::W_X, l);
      bx.store(sRX, l);
    }
    const double* sol = ws + static_cast<size_t>(env) * D::WS + D::W_SOL;
    y0 = sol[j0];
    y1 = v1 ? sol[j1] : 0.0;
#pragma unroll
    for (int t = 0; t < NRL; ++t) {
      const double q = sol[even(NY) + l + kRow * t];
      lam[t] = q;
      s[t] = q > 0.0 ? 0.0 : 1.0;
    }
    st = static_cast<int32_t>(sol[even(NY) + NRL * kRow]);
    sVy[j0] = y0;
    if (v1) sVy[j1] = y1;
    wave_sync();
  } else
  for (int it = CP == kCpResume ? resume_state() : (all_warm ? 0 : -1);; ++it) {
    STAMP_BEGIN();
    const bool init = it < 0;
    double mu = 0.0;
    if (WARM && it == 0 && any_warm) {
      const double* wst = gwarm + static_cast<size_t>(env) * D::WW;
      if (warm) {
        y0 = wst[D::WW_Y + j0];
        y1 = v1 ? wst[D::WW_Y + j1] : 0.0;
        sVy[j0] = y0;
        if (v1) sVy[j1] = y1;
      }
      wave_sync();
      wave_sync();
      if (warm) {
        const double dlt = P->warm_delta;
#pragma unroll
        for (int t = 0; t < NRL; ++t) {
          const double gy = Gv(sVy, t);
          const double wl = wst[D::WW_L + l + kRow * t];
          s[t] = act[t] ? fmax(h[t] - gy, dlt) : 1.0;
          lam[t] = act[t] ? fmax(wl, dlt) : 0.0;
        }
      }
      // centre the warm pairs: no s_i lambda_i below warm_center x their mean (numpy model, 1 %
      // random walk, 0.1: WaLTER mean 9.2 -> 6.5 iterations, lockstep 11.3 -> 7.8; Go2 6.6 ->
      // 5.8; most warm stalls vanish)
      double c0s = 0.0;
#pragma unroll
      for (int t = 0; t < NRL; ++t) c0s += act[t] ? s[t] * lam[t] : 0.0;
      const double mu0 = P->warm_center * row_sum(c0s) / fmax(m_act, 1.0);
      if (warm) {
#pragma unroll
        for (int t = 0; t < NRL; ++t) {
          if (act[t]) {
            lam[t] = fmax(lam[t], mu0 * recip(s[t]));
            s[t] = fmax(s[t], mu0 * recip(lam[t]));
          }
        }
      }
      if constexpr (WHR) {
        // the wheel rows' residual at the warm y (this tick's rows: directions and mask are new
        // every tick; the first Newton step's pinned coordinates step onto them exactly)
        double yh0, yh1;
        rot_in(y0, y1, yh0, yh1);
        rq0 = pin0 ? yh0 + q10 : 0.0;
        rq1 = pin1 ? yh1 + q11 : 0.0;
        rwmax = row_max(fmax(fabs(rq0), fabs(rq1)));
      }
    }
    // An env still far from converged (mu > 1e-6) at iteration `restart_iter` (warm-started:
    // `warm_restart`) is re-centred in place -- slacks h - G y + 1, multipliers 1: the cold
    // start's shape, no factorisation.  The rare solves that fall into a two-iteration limit
    // cycle of the step rule (mu oscillating near 1e-4; random-walk inputs, ~3e-6 of env-ticks,
    // round-3 warm-stall study) then finish ~10 iterations later instead of at max_iter.  No env of
    // the fresh-batch sweeps is still that far off at iteration 20 (tools/ipm_model.py
    // "recenter20": identical iteration counts).
    bool restart = false;
    if (it == P->restart_iter || (WARM && any_warm && it == P->warm_restart)) {
      double cr = 0.0;
#pragma unroll
      for (int t = 0; t < NRL; ++t) cr += act[t] ? s[t] * lam[t] : 0.0;
      const bool far = row_sum(cr) / fmax(m_act, 1.0) > 1e-6;
      const bool mine = far && !done && it == (warm ? P->warm_restart : P->restart_iter);
      restart = __ballot(mine) != 0;
      if (restart) wave_sync();
      if (mine) {
#pragma unroll
        for (int t = 0; t < NRL; ++t) {
          const double slack = h[t] - Gv(sVy, t);
          s[t] = act[t] ? fmax(slack, 0.0) + 1.0 : 1.0;
          lam[t] = act[t] ? 1.0 : 0.0;
        }
      }
    }
    if (!init) {
      double cs = 0.0;
#pragma unroll
      for (int t = 0; t < NRL; ++t) cs += act[t] ? s[t] * lam[t] : 0.0;
      mu = row_sum(cs) / fmax(m_act, 1.0);
      const bool fresh = it == 0 || mu <= 1e-6 || restart;
      if (__ballot(fresh) != 0) {   // wave-uniform
        wave_sync();
#pragma unroll
        for (int t = 0; t < NRL; ++t) {
          const double r = act[t] ? Gv(sVy, t) + s[t] - h[t] : 0.0;
          rp[t] = fresh ? r : rp[t];
        }
      }
      if (!done && mu <= eps_run && (!D::WH || rwmax <= P->wheel_tol)) {
        done = true;
        st = OSC_SOLVE_OK;
        it_done = it;
      }
      if constexpr (CP == kCpPark) {
        if (it == PA.park_it && __ballot(!done) != 0) {
          // one slot per unconverged row (lane 0 of the row takes it), its state written by
          // every lane of the row; the row then counts as done in this wave
          int slot = 0;
          if (!done && l == 0) slot = atomicAdd(PA.count, 1);
          slot = __shfl(slot, grp * kRow, kWave);
          if (!done) {
            double* pk = park_at(slot);
            pk[l] = y0;
            pk[kRow + l] = y1;
#pragma unroll
            for (int t = 0; t < NRL; ++t) {
              pk[2 * kRow + l + kRow * t] = s[t];
              pk[2 * kRow + NRL * kRow + l + kRow * t] = lam[t];
              pk[2 * kRow + 2 * NRL * kRow + l + kRow * t] = rp[t];
            }
            if (l == 0) PA.list[slot] = env;
            parked = true;
            done = true;
          }
        }
      }
      if (__ballot(!done) == 0 || it >= P->max_iter) {
        if (!done) it_done = it;
        break;
      }
    }
    double inv_s[NRL];                   // 1/s on active rows, 0 elsewhere (s = 1 at init)
#pragma unroll
    for (int t = 0; t < NRL; ++t) {
      const int r = l + kRow * t;
      inv_s[t] = act[t] ? (init ? 1.0 : recip(s[t])) : 0.0;
      sVr[r] = init ? 0.0 : (act[t] ? lam[t] : 0.0);
      sDr[r] = init ? (init_ls(t) ? 1.0 : 0.0) : lam[t] * inv_s[t];
    }
    wave_sync();

    STAMP_END(1);
    STAMP_BEGIN();
    // ---- Newton matrix K = Hr + G' D G (columns j0, j1 in registers) and rd = Hr y + g + G'lam
    double rd0, rd1;
    GTw2(sVr, rd0, rd1);
    if constexpr (WHR) rot_in(rd0, rd1, rd0, rd1);   // T'G'lam
    rd0 += g0;
    rd1 += g1;
    double dg0 = hdg0, dg1 = hdg1;
    if constexpr (WHR) {   // rd^ += H^ y^
      if (!init) {
        double yh0, yh1;
        rot_in(y0, y1, yh0, yh1);
        dot_rows<NY>(rd0, rd1, yh0, yh1, c0, c1);
      }
    } else {
      if (!init) dot_rows<NY>(rd0, rd1, y0, y1, c0, c1);    // rd += Hr y (y broadcast by DPP)
    }
    STAMP_END(8);
    STAMP_BEGIN();
    // G_u' D G_u is diagonal, d_q = D[2q] + D[2q+1] on (q, q): lane q's column j0 = q
    if constexpr (WHR) {
      assemble_rot(dg0, dg1);
    } else {
      static_assert(D::NU <= kRow, "torque variables in the first column slot");
      const double2 dd = *reinterpret_cast<const double2*>(sDr + 2 * (j0 < NU ? j0 : 0));
      const double du = (j0 < NU) ? dd.x + dd.y : 0.0;
      dg0 += du;
      static_for<0, NU>([&](auto I) {
        constexpr int i = decltype(I)::value;
        c0[i] += keep_lanes<rows_mask(1u << i)>(du);
      });
    }
    STAMP_END(9);
    STAMP_BEGIN();
    if (!WHR && jk0 >= 0) {
      double a, b, cc;
      contact_col(jk0, jc0, a, b, cc);
      dg0 += (jc0 == 0) ? a : (jc0 == 1) ? b : cc;
#pragma unroll
      for (int i = NU; i < NY; ++i) {
        const int ki = (i - NU) / 3, ci = (i - NU) % 3;
        c0[i] += (ki == jk0) ? ((ci == 0) ? a : (ci == 1) ? b : cc) : 0.0;
      }
    }
    if (!WHR && jk1 >= 0) {
      double a, b, cc;
      contact_col(jk1, jc1, a, b, cc);
      dg1 += (jc1 == 0) ? a : (jc1 == 1) ? b : cc;
#pragma unroll
      for (int i = NU; i < NY; ++i) {
        const int ki = (i - NU) / 3, ci = (i - NU) % 3;
        c1[i] += (ki == jk1) ? ((ci == 0) ? a : (ci == 1) ? b : cc) : 0.0;
      }
    }
    wave_sync();
    STAMP_END(2);
    STAMP_BEGIN();
    ldl_rows<NY>(c0, c1, B + LY::I_DINV, l, dinv0, dinv1, 1e-13 * dg0, 1e-13 * dg1);
    wave_sync();
    STAMP_END(3);

    // pass 0: affine (predictor) direction, rc = s lambda
    // pass 1: corrector, rc = s lambda + ds_aff dl_aff - sigma mu
    double ds[NRL], dl[NRL], dsdl[NRL];
#pragma unroll
    for (int t = 0; t < NRL; ++t) ds[t] = dl[t] = dsdl[t] = 0.0;
    double dy0 = 0.0, dy1 = 0.0, sig_mu = 0.0, step = 1.0, a_aff = 1.0;
    const int npass = init ? 1 : 2;
    for (int pass = 0; pass < npass; ++pass) {
      STAMP_BEGIN();
#pragma unroll
      for (int t = 0; t < NRL; ++t) {
        const double rc = fma(s[t], lam[t], dsdl[t]) - sig_mu;   // dsdl = sig_mu = 0 in pass 0
        sVr[l + kRow * t] = init ? (init_ls(t) ? h[t] : 0.0) : (rc - lam[t] * rp[t]) * inv_s[t];
      }
      wave_sync();
      GTw2(sVr, dy0, dy1);
      if constexpr (WHR) {   // in y^: T'(G'w) - rd^, the pinned slots step to the rows
        rot_in(dy0, dy1, dy0, dy1);
        dy0 = pin0 ? -rq0 : dy0 - rd0;
        dy1 = pin1 ? -rq1 : dy1 - rd1;
      } else {
        dy0 -= rd0;
        dy1 -= rd1;
      }
      STAMP_END(4);
      STAMP_BEGIN();
      ldl_solve_rows<NY>(c0, c1, dinv0, dinv1, dy0, dy1, l);
      if constexpr (WHR) rot_out(dy0, dy1, dy0, dy1);
      sVy2[j0] = dy0;
      if (v1) sVy2[j1] = dy1;
      wave_sync();
      STAMP_END(5);
      STAMP_BEGIN();
      wave_sync();
      // step to the boundary, division-free: 1 / max(1, max_r(-ds/s), max_r(-dl/lambda))
      double rmax = 1.0;
      double gdy_all[NRL];
      if constexpr (SMALL) Gv_all(sVy2, gdy_all);
#pragma unroll
      for (int t = 0; t < NRL; ++t) {
        const double rc = fma(s[t], lam[t], dsdl[t]) - sig_mu;
        const double gdy = SMALL ? gdy_all[t] : Gv(sVy2, t);
        ds[t] = act[t] ? -rp[t] - gdy : 0.0;
        dl[t] = -(rc + lam[t] * ds[t]) * inv_s[t];
        const double inv_l = (act[t] && !init) ? recip1(lam[t]) : 0.0;
        rmax = fmax(rmax, fmax(-ds[t] * inv_s[t], -dl[t] * inv_l));
      }
      step = recip(row_max(rmax));
      if (pass == 0 && !init) {
        double ca = 0.0;
#pragma unroll
        for (int t = 0; t < NRL; ++t)
          ca += act[t] ? (s[t] + step * ds[t]) * (lam[t] + step * dl[t]) : 0.0;
        a_aff = step;
        const double mu_aff = row_sum(ca) / fmax(m_act, 1.0);
        const double q = mu_aff / fmax(mu, 1e-300);
        sig_mu = q * q * mu;   // sigma = (mu_aff/mu)^2: the cube jams on rare envs (tools/ipm_hard.py)
#pragma unroll
        for (int t = 0; t < NRL; ++t) dsdl[t] = ds[t] * dl[t];
        if constexpr (WHR) {
          // late stall: once the active rows' barrier terms pass ~1e10 their dense rank-one terms
          // in the rotated Newton matrix swamp its small curvature and the affine step collapses
          // (round-3 wheel traces).  The iterate is as good as it gets there: stop on it
          // (no step) and let the refinement finish the solve.
          if (!done && mu <= 1e-8 && step < 0.1 && rwmax <= P->wheel_tol) {
            done = true;
            st = OSC_SOLVE_OK;
            it_done = it;
            stalled = true;
          }
        }
      }
      wave_sync();
      STAMP_END(6);
    }
    STAMP_BEGIN();
    if (init) {
      // here rp = 0, so ds = -G y0 and  G y0 - h = -ds - h
      y0 = dy0;
      y1 = dy1;
      double zmax = -1e300, nzmax = -1e300;
#pragma unroll
      for (int t = 0; t < NRL; ++t) {
        const double zr = -ds[t] - h[t];
        if (act[t]) {
          zmax = fmax(zmax, zr);
          nzmax = fmax(nzmax, -zr);
        }
      }
      const double ap = row_max(zmax);    // = max(-s)
      const double ad = row_max(nzmax);   // = max(-lambda)
#pragma unroll
      for (int t = 0; t < NRL; ++t) {
        const double zr = -ds[t] - h[t];
        s[t] = act[t] ? ((ap >= 0.0) ? -zr + 1.0 + ap : -zr) : 1.0;
        lam[t] = act[t] ? ((ad >= 0.0) ? zr + 1.0 + ad : zr) : 0.0;
      }
      if (m_act == 0.0 && !done) {        // unconstrained: y0 = -Hr^-1 g is the optimum
        done = true;
        st = OSC_SOLVE_OK;
        it_done = 0;
      }
    } else {
      // fraction to the boundary: 0.99 early, closer to 1 as mu -> 0 or when the affine step was
      // nearly full, never above 1 - 1e-5 (tools/ipm_model.py + tools/etatest.sh: -15% lockstep
      // iterations vs a fixed 0.99; uncapped, a few envs stall at the boundary)
      const double eta =
          fmin(1.0 - 1e-5, fmax(0.99, fmax(1.0 - mu, 1.0 - 0.1 * (1.0 - a_aff))));
      const double alpha = done ? 0.0 : fmin(1.0, eta * step);
      y0 = fma(alpha, dy0, y0);
      y1 = fma(alpha, dy1, y1);
#pragma unroll
      for (int t = 0; t < NRL; ++t) {
        s[t] = act[t] ? fma(alpha, ds[t], s[t]) : 1.0;
        lam[t] = act[t] ? fma(alpha, dl[t], lam[t]) : 0.0;
        rp[t] *= 1.0 - alpha;
      }
    }
    sVy[j0] = y0;
    if (v1) sVy[j1] = y1;
    load_hr();   // next iteration's Hr columns (the factor in c0/c1 is dead now)
    wave_sync();
    if constexpr (WHR) {   // the rows' residual at the new iterate (next step, stop test)
      double yh0, yh1;
      rot_in(y0, y1, yh0, yh1);
      rq0 = pin0 ? yh0 + q10 : 0.0;
      rq1 = pin1 ? yh1 + q11 : 0.0;
      rwmax = row_max(fmax(fabs(rq0), fabs(rq1)));
    }
    STAMP_END(7);
  }
#ifdef OSC_STAMPS
  if constexpr (RF != kRfFused) STAMP_STORE();   // the fused pass stores after its refinement
#endif
  if constexpr (RF == kRfNone) {   // hand the result to the refinement kernel
    if (write_out) {
      // (the W_SOL block is written here and read by nothing else in this kernel)
      double* sol = const_cast<double*>(ws) + static_cast<size_t>(env) * D::WS + D::W_SOL;
      sol[j0] = y0;
      if (v1) sol[j1] = y1;
#pragma unroll
      for (int t = 0; t < NRL; ++t)
        sol[even(NY) + l + kRow * t] = (act[t] && lam[t] > s[t]) ? lam[t] : 0.0;
      if (l == 0) sol[even(NY) + NRL * kRow] = static_cast<double>(st);
    }
  }

  // ---------------- full-space refinement (torque coordinates) ---------------
  // Hr is an explicitly formed fp64 product X'H_dv X whose condition number reaches ~1e10, so the
  // interior point's optimum of the reduced QP sits up to ~1e-5 (normwise) off the optimum of
  // the QP the reference defines.  Iterative refinement on the active set of the converged
  // iterate (rows with lambda > s) removes that: the residual is formed in factored form,
  //   r = X_y' (H_dv (X [y;1]) + f_dv) + 2 (w_tau + w_reg) u + 2 w_reg z + G_A' mu,
  // which never goes through Hr, and the correction comes from one LDL^T of
  // K_A = Hr + D G_A'G_A (active rows by penalty D = refine_penalty x max diag Hr; dependent rows
  // of a contact at the pyramid apex are harmless there):
  //   K_A dy = -r - D G_A'(G_A y - h_A),   mu += D (G_A (y + dy) - h_A),   y += dy.
  // Two steps take the worst envs of 32,768-env batches from 7e-6 to ~1e-13 of the exact optimum
  // (tools/ipm_model.py + the refinement study in DESIGN.md).  Envs that did not converge keep
  // their iterate; a refinement that moves y by more than 1e-3 (relative) or is not finite is
  // discarded.
  // (wheel rows: a fixed step count, the same whether or not the duals are asked for, so x and tau
  // do not depend on want_dual -- the rows' multipliers converge more slowly than y, hence 12)
  if constexpr (CP == kCpPark) write_out = write_out && !parked;   // the resume pass writes them
  const int refine_steps = P->refine_steps;
  if constexpr (RF != kRfNone) {
    // WH: an env the interior point left at max_iter is refined too (its rotated Newton systems
    // can stall short of eps_mu with the active set already right): a kept refinement -- no row
    // violated, no multiplier of the wrong sign, its last step converged -- is a KKT point of the
    // strictly convex QP, i.e. its optimum, and the env reports OK
    const bool mine = valid && (st == OSC_SOLVE_OK || (WHR && st == OSC_SOLVE_MAX_ITER));
    if (P->refine_steps > 0 && __ballot(mine) != 0) {
      const double dpen = P->refine_penalty * row_max(fmax(fabs(hdg0), fabs(hdg1)));
      const double ytol = 1e-9 * (1.0 + row_max(fmax(fabs(y0), v1 ? fabs(y1) : 0.0)));
      // the wheel rows keep round 3's fixed steps and move-bound acceptance (their refinement runs
      // refine_steps steps; the generic KKT acceptance measured no different on them)
      constexpr bool kOldWh = WHR;
      double Dr[NRL], mur[NRL];
      // WH: a row whose slack is within 1e-6 of the bound is active too -- next to the rows'
      // Schur solves the interior point's multipliers of a weakly active row can be off by orders
      // of magnitude while y is right (numpy model: 11 of 512 tumbling refinements rejected -> 0)
      const double stol =
          D::WH ? 1e-6 * (1.0 + row_max(fmax(fabs(y0), v1 ? fabs(y1) : 0.0))) : -1.0;
#pragma unroll
      for (int t = 0; t < NRL; ++t) {
        const bool a = act[t] && (lam[t] > s[t] || s[t] <= stol);
        Dr[t] = a ? dpen : 0.0;
        mur[t] = a ? lam[t] : 0.0;
      }
      const double wu = 2.0 * (P->w_torque + P->w_reg), wz = 2.0 * P->w_reg;
      double ya0 = y0, ya1 = y1;
      bool viol_env = false;
      const double* wenv = ws + static_cast<size_t>(env) * D::WS;
      const double* rX = kRefG ? wenv + D::W_X : sRX;
      const double* rH = kRefG ? wenv + D::W_HD : sRH;
      const double* rG = kRefG ? wenv + D::W_GD : sRG;
      constexpr int kUr = kRefG ? 2 : 32;   // workspace reads: few in flight (registers)
      double dlast = 0.0;   // the last refinement step's size (its convergence test)
      bool settled = false;                          // this env's final round is done
      const double yscale = row_max(fmax(fabs(y0), v1 ? fabs(y1) : 0.0));
      double yk0 = 0.0, yk1 = 0.0, dk = 0.0, nuk = 0.0;   // its result (WH: step, multiplier)
      // (no wheel rows) steps run until the env's own step has converged -- at least
      // refine_steps, at most kRefineMaxSteps per round -- and then the env is frozen (its later
      // lockstep steps are zero), so its result does not depend on its wave-mates' step counts
      bool conv = false;
      // rounds: a row the refined point violates was active at the optimum with a vanishing
      // multiplier (lambda and s both ~1e-6 when the interior point stops): it joins the active
      // set, a row whose multiplier came out negative leaves it, and the round repeats from the
      // interior point's iterate with the multipliers carried over (numpy model of the kernel on
      // joint-state batches, tools/kkt_study.py: <= 3 rounds, <= 9 steps)
      for (int round = 0; round < (WHR ? 5 : kRefineRounds); ++round) {
        STAMP_BEGIN();
#ifdef OSC_STAMPS
        st_acc[10] += 1ull << 40;   // rounds, in the top bits of the assembly+LDL slot
#endif
        if (round > 0) {   // c0 / c1 hold the last round's factor
          if constexpr (kXinHr) {
            // Hr's LDS region holds X now: Hr columns from the (L2-resident) workspace
#pragma unroll
            for (int i = 0; i < NY; ++i) {
              c0[i] = wsw[lane_off + static_cast<unsigned>(i * NY + j0)];
              c1[i] = wsw[lane_off + static_cast<unsigned>(i * NY + jj1)];
            }
          } else {
            load_hr();
          }
        }
#pragma unroll
        for (int t = 0; t < NRL; ++t) sDr[l + kRow * t] = Dr[t];
        ya0 = y0;
        ya1 = y1;
        sVy[j0] = y0;
        if (v1) sVy[j1] = y1;
        wave_sync();
        // K_A in c0 / c1 (they hold Hr's columns)
        double dg0 = hdg0, dg1 = hdg1;
        if constexpr (WHR) {
          wave_sync();
          assemble_rot(dg0, dg1);
        } else {
          const double2 dd = *reinterpret_cast<const double2*>(sDr + 2 * (j0 < NU ? j0 : 0));
          const double du = (j0 < NU) ? dd.x + dd.y : 0.0;
          dg0 += du;
          static_for<0, NU>([&](auto I) {
            constexpr int i = decltype(I)::value;
            c0[i] += keep_lanes<rows_mask(1u << i)>(du);
          });
        }
        if (!WHR && jk0 >= 0) {
          double a, b, cc;
          contact_col(jk0, jc0, a, b, cc);
          dg0 += (jc0 == 0) ? a : (jc0 == 1) ? b : cc;
#pragma unroll
          for (int i = NU; i < NY; ++i) {
            const int ki = (i - NU) / 3, ci = (i - NU) % 3;
            c0[i] += (ki == jk0) ? ((ci == 0) ? a : (ci == 1) ? b : cc) : 0.0;
          }
        }
        if (!WHR && jk1 >= 0) {
          double a, b, cc;
          contact_col(jk1, jc1, a, b, cc);
          dg1 += (jc1 == 0) ? a : (jc1 == 1) ? b : cc;
#pragma unroll
          for (int i = NU; i < NY; ++i) {
            const int ki = (i - NU) / 3, ci = (i - NU) % 3;
            c1[i] += (ki == jk1) ? ((ci == 0) ? a : (ci == 1) ? b : cc) : 0.0;
          }
        }
        // HRL: X is copied global -> LDS by DMA (no registers) into Hr's region -- free now, K_A
        // is in registers -- issued before the factorisation, waited for after it, so its latency
        // hides behind the LDL^T.  A DMA wave-instruction writes 16 B per lane to a wave-uniform
        // base + 16 B x lane, so each one fills 1 KB of ONE env's block with all 64 lanes (every
        // lane loads that env's chunk): compile-time bases, no per-env branches.
        if constexpr (kXinHr) {
          constexpr int NCH = D::NV * D::NY1P / 2;               // 16-byte chunks of X
          constexpr int NT = (NCH + kWave - 1) / kWave;
          static_assert(D::NV * D::NY1P <= even(NY * NY) && D::W_X % 2 == 0 &&
                        NT * kWave * 2 <= even(NY * NY), "X (whole DMA rows) in Hr's region");
          if (round == 0) {
            // the loop's last Hr column reads of this region (load_hr) have returned before the DMA
            // overwrites it (K_A's assembly consumed only some of them)
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            static_for<0, kEnvPerWave>([&](auto G) {
              constexpr int g = decltype(G)::value;
              const int eg = CP == kCpResume ? __builtin_amdgcn_readlane(env, g * kRow)
                             : (blk * kEnvPerWave + g < nenv ? blk * kEnvPerWave + g : nenv - 1);
              const double2* src =
                  reinterpret_cast<const double2*>(ws + static_cast<size_t>(eg) * D::WS + D::W_X);
              static_for<0, NT>([&](auto T) {
                constexpr int t = decltype(T)::value;
                const int c = lane + kWave * t < NCH ? lane + kWave * t : NCH - 1;
#if defined(__HIP_DEVICE_COMPILE__)   // (a device builtin: the host pass never runs this body)
                __builtin_amdgcn_global_load_lds(src + c, sm + g * kEnvLds + LY::I_HR + 2 * kWave * t,
                                                 16, 0, 0);
#else
                (void)src;
                (void)c;
#endif
              });
              {
                // [H_dv | f_dv] the same way, into the block's refinement region (not staged with
                // the prologue's loads: 11 of the 27 MB every wave requests at once at 4,096 envs)
                constexpr int NCH2 = (RefineLds<D>::SIZE - RefineLds<D>::HD) / 2;
                constexpr int NT2 = (NCH2 + kWave - 1) / kWave;
                static_assert(NT2 * kWave * 2 == refine_lds_extra<D, SMALL, RF>() &&
                              D::W_HD == D::W_X + RefineLds<D>::HD && D::W_HD % 2 == 0,
                              "[H_dv | f_dv] (whole DMA rows) in the refinement region");
                const double2* src2 =
                    reinterpret_cast<const double2*>(ws + static_cast<size_t>(eg) * D::WS + D::W_HD);
                static_for<0, NT2>([&](auto T) {
                  constexpr int t = decltype(T)::value;
                  const int c = lane + kWave * t < NCH2 ? lane + kWave * t : NCH2 - 1;
#if defined(__HIP_DEVICE_COMPILE__)
                  __builtin_amdgcn_global_load_lds(src2 + c, sm + g * kEnvLds + LY::IL + 2 * kWave * t,
                                                   16, 0, 0);
#else
                  (void)src2;
                  (void)c;
#endif
                });
              }
            });
          }
        }
        wave_sync();
        ldl_rows<NY>(c0, c1, B + LY::I_DINV, l, dinv0, dinv1, 1e-13 * dg0, 1e-13 * dg1);
        if constexpr (kXinHr) {
          if (round == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // X has landed
        }
        wave_sync();
        STAMP_END(8);   // (the loop's slot 8 doubles as the refinement's LDL)
        STAMP_BEGIN();
        conv = false;
        for (int k = 0; k < (kOldWh ? refine_steps : kRefineMaxSteps); ++k) {
          // WH: X holds X^ = X'T, so dv = X^ [y^; 1] (y^ = T'y staged in sVy2, free until the step)
          // and the rows' residual at y comes with y^
          const double* yv = sVy;
          if constexpr (WHR) {
            double yh0, yh1;
            rot_in(ya0, ya1, yh0, yh1);
            rq0 = pin0 ? yh0 + q10 : 0.0;
            rq1 = pin1 ? yh1 + q11 : 0.0;
            sVy2[j0] = yh0;
            if (v1) sVy2[j1] = yh1;
            wave_sync();
            yv = sVy2;
          }
          // dv = X [y; 1] (rows l, l + 16) -> sXb
#pragma unroll
          for (int t = 0; t < (NV + kRow - 1) / kRow; ++t) {
            const int rr = l + kRow * t;
            if (rr < NV) {
              const double* xr = rX + rr * NY1P;
              double a = xr[NY];
#pragma unroll kUr
              for (int i = 0; i < NY; ++i) a = fma(xr[i], yv[i], a);
              sXb[rr] = a;
            }
          }
          wave_sync();
          // gx = H_dv dv + f_dv (rows l, l + 16) -> sDr[0 .. NV)
          double gxr[(NV + kRow - 1) / kRow];
#pragma unroll
          for (int t = 0; t < (NV + kRow - 1) / kRow; ++t) {
            const int rr = l + kRow * t;
            gxr[t] = 0.0;
            if (rr < NV) {
              const double* hr = rH + rr * NV;
              double a = rG[rr];
#pragma unroll kUr
              for (int i = 0; i < NV; ++i) a = fma(hr[i], sXb[i], a);
              gxr[t] = a;
            }
          }
          wave_sync();
#pragma unroll
          for (int t = 0; t < (NV + kRow - 1) / kRow; ++t)
            if (l + kRow * t < NV) sDr[l + kRow * t] = gxr[t];
#pragma unroll
          for (int t = 0; t < NRL; ++t) sVr[l + kRow * t] = mur[t];
          wave_sync();
          if constexpr (D::WH && RF == kRfFused) {
            // gx <- (I - V'V) gx: X's columns are orthogonal to V (setup_env), so this changes
            // nothing in exact arithmetic, but it drops gx's large components along the rows'
            // constrained directions before X' multiplies them (numpy model: 5e-9 -> 1.5e-9 worst)
            const double* Vw = wenv + D::W_WV;
            double vg = 0.0;
            if (l < NW) {
#pragma unroll
              for (int j = 0; j < NV; ++j) vg = fma(Vw[l * NV + j], sDr[j], vg);
            }
            double corr[(NV + kRow - 1) / kRow];
#pragma unroll
            for (int t = 0; t < (NV + kRow - 1) / kRow; ++t) corr[t] = 0.0;
            static_for<0, NW>([&](auto W) {
              constexpr int w = decltype(W)::value;
              const double bw = bcast_guarded<w>(vg);
#pragma unroll
              for (int t = 0; t < (NV + kRow - 1) / kRow; ++t) {
                const int rr = l + kRow * t;
                corr[t] = fma(Vw[w * NV + (rr < NV ? rr : 0)], bw, corr[t]);
              }
            });
            wave_sync();
#pragma unroll
            for (int t = 0; t < (NV + kRow - 1) / kRow; ++t)
              if (l + kRow * t < NV) sDr[l + kRow * t] -= corr[t];
            wave_sync();
          }
          // r_j = X[:, j]' gx + diag_j y_j + (G_A' mu)_j for the lane's two variables
          // (WH, in y^: X^'gx + T'(W y + G_A' mu))
          double r0 = (j0 < NU ? wu : wz) * ya0, r1 = (jj1 < NU ? wu : wz) * ya1;
          double gm0, gm1;
          if constexpr (WHR) {
            GTw2(sVr, gm0, gm1);
            r0 += gm0;
            r1 += gm1;
            rot_in(r0, r1, r0, r1);
          }
#pragma unroll kUr
          for (int i = 0; i < NV; ++i) {
            r0 = fma(rX[i * NY1P + j0], sDr[i], r0);
            r1 = fma(rX[i * NY1P + jj1], sDr[i], r1);
          }
          if constexpr (!WHR) {   // (this order: the feature-off results stay bitwise)
            GTw2(sVr, gm0, gm1);
            r0 += gm0;
            r1 += gm1;
          }
          if constexpr (WHR) {
            // the pinned coordinates of r^ are Q (grad f + G_A' mu): their negatives are the rows'
            // multipliers (least squares; the last step's stand)
            const double p0v = sWPin[j0], p1v = sWPin[jj1];
            if (p0v >= 0.0) sWNu[static_cast<int>(p0v)] = -r0;
            if (v1 && p1v >= 0.0) sWNu[static_cast<int>(p1v)] = -r1;
          }
          wave_sync();
          double R3[NRL];
#pragma unroll
          for (int t = 0; t < NRL; ++t) {
            R3[t] = (Dr[t] != 0.0) ? Gv(sVy, t) - h[t] : 0.0;
            sVr[l + kRow * t] = Dr[t] * R3[t];
          }
          wave_sync();
          double b0, b1;
          GTw2(sVr, b0, b1);
          if constexpr (WHR) rot_in(b0, b1, b0, b1);
          double d0 = -r0 - b0, d1 = -r1 - b1;
          if constexpr (WHR) {
            d0 = pin0 ? -rq0 : d0;
            d1 = pin1 ? -rq1 : d1;
          }
          ldl_solve_rows<NY>(c0, c1, dinv0, dinv1, d0, d1, l);
          if constexpr (WHR) {
            rot_out(d0, d1, d0, d1);
            dlast = row_max(fmax(fabs(d0), v1 ? fabs(d1) : 0.0));
          }
          const bool frz = !kOldWh && conv;   // converged at an earlier step: no further move
          if (frz) {
            d0 = 0.0;
            d1 = 0.0;
          }
          sVy2[j0] = d0;
          if (v1) sVy2[j1] = d1;
          wave_sync();
#pragma unroll
          for (int t = 0; t < NRL; ++t) mur[t] += frz ? 0.0 : Dr[t] * (Gv(sVy2, t) + R3[t]);
          ya0 += d0;
          ya1 += d1;
          wave_sync();
          sVy[j0] = ya0;
          if (v1) sVy[j1] = ya1;
          wave_sync();
          if constexpr (!kOldWh) {
            // converged: the step fell below 1e-10 of the env's |y| (a row-wide scale: a lane
            // holding only near-zero variables must not hold the env to 1e-10 absolute)
            const double dn = row_max(fmax(fabs(d0), v1 ? fabs(d1) : 0.0));
            if (!frz) dlast = dn;
            conv = conv || (k + 1 >= refine_steps && dn <= 1e-10 * (1.0 + yscale));
            if (k + 1 >= refine_steps && __ballot(mine && !conv) == 0) break;
          }
        }
        // rows the refined point violates join the active set
        double nviol = 0.0;
#pragma unroll
        for (int t = 0; t < NRL; ++t) {
          const bool v = act[t] && Dr[t] == 0.0 && Gv(sVy, t) - h[t] > ytol;
          Dr[t] = v ? dpen : Dr[t];
          nviol += v ? 1.0 : 0.0;
        }
        {
          // ... and rows whose multiplier came out negative leave it (WH: its slack-based active
          // set can include a row the optimum leaves; otherwise a row the interior point's
          // lambda > s test took with a vanishing multiplier)
          double mmax = 0.0;
#pragma unroll
          for (int t = 0; t < NRL; ++t) mmax = fmax(mmax, Dr[t] != 0.0 ? fabs(mur[t]) : 0.0);
          const double mtol = 1e-9 * (1.0 + row_max(mmax));
#pragma unroll
          for (int t = 0; t < NRL; ++t) {
            const bool leave = Dr[t] != 0.0 && mur[t] < -mtol;
            Dr[t] = leave ? 0.0 : Dr[t];
            // (its multiplier leaves with it: the residual sums G'mu over every row slot, and a
            // stale negative multiplier there would move the next round's fixed point off the
            // optimum while no test looks at that row any more)
            mur[t] = leave ? 0.0 : mur[t];
            nviol += leave ? 1.0 : 0.0;
          }
        }
        viol_env = mine && row_max(nviol) > 0.0;
        // a round whose steps have not converged asks for another one as well (it restarts
        // from the interior point's iterate with the multipliers carried over)
        const bool more =
            viol_env || (mine && (kOldWh ? dlast > 1e-10 * (1.0 + yscale) : !conv));
        // an env whose round ended without a violation is final: a further round that a wave-mate
        // asks for must not move it (its multipliers carry over between rounds), so each env's
        // result is independent of the envs sharing its wavefront -- and of the compaction's
        // packing (ParkArgs)
        if (mine && !more && !settled) {
          settled = true;
          yk0 = ya0;
          yk1 = ya1;
          if constexpr (WHR) {
            dk = dlast;
            nuk = l < NW ? sWNu[l] : 0.0;
          }
        }
        STAMP_END(11);
        if (__ballot(more && !settled) == 0) break;
      }
      if (settled) {   // (its own last round had no violation, whatever later rounds found)
        ya0 = yk0;
        ya1 = yk1;
        viol_env = false;
        if constexpr (WHR) dlast = dk;
      }
      // Keep the refined iterate when it is a KKT point of the QP: its last round added no row
      // (primal feasible to ytol), dropped no row (no multiplier of the wrong sign) and its steps
      // converged, and it is finite.  The QP is strictly convex, so that point is its optimum,
      // however far the interior point's iterate was from it: with the internal-force curvature
      // 2 w_reg = 2e-4, the barrier of a nearly active row pushes the iterate at mu = 1e-9 up to
      // ~2e-2 off along such directions (joint-state batches, tools/kkt_study.py) -- the move
      // bound 1e-3 per lane that stood here rejected those envs (OSC_SOLVE_UNREFINED).
      // refine_max_move (default: none) remains as a tuning knob that forces rejections.
      const double mv = fmax(fabs(ya0 - y0), v1 ? fabs(ya1 - y1) : 0.0);
      const double myr = row_max(fmax(fabs(y0), v1 ? fabs(y1) : 0.0));
      // (WH: the rotated Newton systems; kept when converged -- its last step below 1e-10 of the
      // env's |y| scale, a row-wide maximum -- within 0.1 of y)
      const double ok =
          (isfinite(ya0) && isfinite(ya1) &&
           (kOldWh ? (mv <= 0.1 * (1.0 + myr) && dlast <= 1e-10 * (1.0 + myr))
                : (settled && mv <= P->refine_max_move * (1.0 + myr)))) ? 1.0 : 0.0;
      // (WH: and the wheel rows hold at the refined point)
      double wres = 0.0;
      if constexpr (WHR) {
        double yh0, yh1;
        rot_in(ya0, ya1, yh0, yh1);
        wres = row_max(fmax(pin0 ? fabs(yh0 + q10) : 0.0, pin1 ? fabs(yh1 + q11) : 0.0));
      }
      const bool keep = !viol_env && row_min(ok) == 1.0 && wres <= ytol;
      if (mine && keep) {
        y0 = ya0;
        y1 = ya1;
        refined = true;
        st = OSC_SOLVE_OK;
      }
      // a converged env whose refinement is rejected keeps the interior point's iterate, and says
      // so: it is only as accurate as the interior point's stop.  (Wheel rows: the interior point
      // runs to mu <= 1e-12 and its pinned coordinates hold the rows to rounding; where they hold
      // to ytol its iterate stands as the solution -- census, profiles/r04g_census_*: every such
      // env within 4e-12 of the exact optimum, while the refinement, started from it, ended with
      // rows violated after its rounds; the exported duals come from stationarity, not from the
      // refinement, osc_dual_kernel) -- but not an iterate the late-stall exit left at mu > eps_mu:
      // with 4 refinement steps per round one such env stood 3e-4 off (profiles/r04zd/); it is
      // UNREFINED, and the fused entries' active-set fallback solves it)
      if (mine && !keep && st == OSC_SOLVE_OK && !(WHR && rwmax <= ytol && !stalled))
        st = OSC_SOLVE_UNREFINED;
#ifdef OSC_REFINE_DIAG   // diagnostic builds only: why the refinement was rejected
      if (mine && !keep)
        st = OSC_SOLVE_UNREFINED + 16 * (viol_env ? 1 : 0) + 32 * (row_min(ok) == 1.0 ? 0 : 1) +
             64 * (wres <= ytol ? 0 : 1) + 128 * (row_min(dlast <= 1e-10 * (1.0 + myr) ? 1.0 : 0.0) == 1.0 ? 0 : 1) +
             256 * (row_min(mv <= 0.1 * (1.0 + myr) ? 1.0 : 0.0) == 1.0 ? 0 : 1);
#endif
      put_wheel_duals((mine && keep && l < NW) ? (settled ? nuk : sWNu[l]) : 0.0);
      wave_sync();
      sVy[j0] = y0;
      if (v1) sVy[j1] = y1;
      wave_sync();
    }
  }

#ifdef OSC_STAMPS
  if constexpr (RF == kRfFused) STAMP_STORE();
#endif
  if (!refined) put_wheel_duals(0.0);
  // ---------------- outputs: tau = y_u;  x = (dv, u, z) with dv = X [y; 1] -----------------
  if (REFINE && !refined) {   // the interior point kernel's outputs stand
    if (write_out && l == 0 && gstatus && st == OSC_SOLVE_UNREFINED) gstatus[env] = st;
    write_out = false;
  }
  if (l < NU) {
    const double tq = sVy[l];
    sTau[l] = tq;
    if (write_out) gtau[static_cast<size_t>(env) * NU + l] = tq;
  }
  if (gx != nullptr) {   // dv = X [y; 1], two rows per lane
    const double* yv = sVy;
    if constexpr (WHR) {   // X^ = X'T: dv = X^ [T'y; 1]
      double yh0, yh1;
      rot_in(y0, y1, yh0, yh1);
      sVy2[j0] = yh0;
      if (v1) sVy2[j1] = yh1;
      wave_sync();
      yv = sVy2;
    }
#pragma unroll
    for (int t = 0; t < (NV + kRow - 1) / kRow; ++t) {
      const int rr = l + kRow * t;
      if (rr < NV) {
        const double* xr = ws + static_cast<size_t>(env) * D::WS + D::W_X + rr * NY1P;
        double xb = xr[NY];
#pragma unroll
        for (int i = 0; i < NY; ++i) xb = fma(xr[i], yv[i], xb);
        sXb[rr] = xb;
      }
    }
  }
  wave_sync();
  const double fin = (isfinite(y0) && (!v1 || isfinite(y1))) ? 1.0 : 0.0;
  if (row_min(fin) == 0.0) st = OSC_SOLVE_NUMERICAL;
  if (write_out) {
    if (gx != nullptr) {
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        const int idx = l + kRow * t;
        if (idx < D::NX) {
          double v;
          if (idx < NV) v = sXb[idx];
          else if (idx < NV + NU) v = sTau[idx - NV];
          else v = sVy[NU + idx - NV - NU];
          gx[static_cast<size_t>(env) * D::NX + idx] = v;
        }
      }
    }
    if (l == 0 && !REFINE) {
      if (gstatus) gstatus[env] = st;
      if (giters) giters[env] = (WARM && fixup) ? P->max_iter + it_done : it_done;   // both passes
    }
    if (WARM && !REFINE) {   // this tick's y and lambda for the next one (NaN: next tick cold)
      double* wo = gwarm + static_cast<size_t>(env) * D::WW;
      wo[D::WW_Y + j0] = y0;
      if (v1) wo[D::WW_Y + j1] = y1;
#pragma unroll
      for (int t = 0; t < NRL; ++t) wo[D::WW_L + l + kRow * t] = lam[t];
      if (l < NC) wo[D::WW_M + l] = sMask[l];
      if (l == 0) wo[0] = (st == OSC_SOLVE_NUMERICAL) ? 0.0 : 1.0;
    }
  }
}

template <class D, bool SMALL, bool WARM, int RF = kRfNone>
__global__ __launch_bounds__(kWave, SMALL ? 1 : 2) void osc_ipm_kernel(
    const DevParams* __restrict__ P, int nenv, const double* __restrict__ gmask,
    const double* __restrict__ ws, double* __restrict__ gtau, double* __restrict__ gx,
    int32_t* __restrict__ gstatus, int32_t* __restrict__ giters, double* __restrict__ gwarm,
    int flags) {
  // one-wave variant: four workgroups per CU (160 KB of LDS), never five.  (The opt-in wheel
  // rows' Schur blocks take it to 53 KB per wave: three per CU)
  static_assert(!SMALL || ipm_lds_doubles<D, SMALL, RF>() * 8 <= 160 * 1024 / (D::WH ? 3 : 4),
                "IPM LDS");
  static_assert(ipm_lds_doubles<D, SMALL, RF>() * 8 <= 64 * 1024, "IPM LDS per workgroup");
  __shared__ __attribute__((aligned(16))) double sm[ipm_lds_doubles<D, SMALL, RF>()];
  ipm_block<D, SMALL, WARM, RF>(P, static_cast<int>(blockIdx.x), nenv, gmask, ws, gtau, gx,
                                    gstatus, giters, gwarm, flags, sm);
}

// The cold fused solve split in two passes for lockstep compaction (ParkArgs): CP = kCpPark
// over every env's wavefront, then CP = kCpResume over the parked envs, packed.
template <class D, bool SMALL, int CP>
__global__ __launch_bounds__(kWave, SMALL ? 1 : 2) void osc_ipm_compact_kernel(
    const DevParams* __restrict__ P, int nenv, const double* __restrict__ gmask,
    const double* __restrict__ ws, double* __restrict__ gtau, double* __restrict__ gx,
    int32_t* __restrict__ gstatus, int32_t* __restrict__ giters, int flags, ParkArgs PA) {
  __shared__ __attribute__((aligned(16))) double sm[ipm_lds_doubles<D, SMALL, kRfFused>()];
  ipm_block<D, SMALL, false, kRfFused, CP>(P, static_cast<int>(blockIdx.x), nenv, gmask, ws, gtau,
                                           gx, gstatus, giters, nullptr, flags, sm, PA);
}

// The full-space refinement pass (torque coordinates): the same body with the interior-point
// loop compiled out, started from the result the interior point left in W_SOL, so its extra
// state never weighs on the interior point's register allocation.
template <class D, bool SMALL>
__global__ __launch_bounds__(kWave, SMALL ? 1 : 2) void osc_refine_kernel(
    const DevParams* __restrict__ P, int nenv, const double* __restrict__ gmask,
    const double* __restrict__ ws, double* __restrict__ gtau, double* __restrict__ gx,
    int32_t* __restrict__ gstatus) {
  __shared__ __attribute__((aligned(16))) double sm[ipm_lds_doubles<D, SMALL, kRfOnly>()];
  ipm_block<D, SMALL, false, kRfOnly>(P, static_cast<int>(blockIdx.x), nenv, gmask, ws, gtau, gx,
                                   gstatus, nullptr, nullptr, 0, sm);
}

// Two models' interior point in one grid, one wavefront per SIMD (the one-wave variant of both):
// blocks [0, nbA) are model A's wavefronts, the rest model B's.  The dispatcher hands out blocks
// in order, so with the slower model first the faster model's wavefronts fill the SIMDs that
// the first model's early finishers free (its iteration-count tail) -- two grids on two streams
// instead split the SIMDs between the models and each pays its own tail.
template <class DA, class DB, int RF = kRfNone>
__global__ __launch_bounds__(kWave, 1) void osc_ipm_pair_kernel(PairArgs A, PairArgs B) {
  __shared__ __attribute__((aligned(16))) double
      sm[cmax(ipm_lds_doubles<DA, true, RF>(), ipm_lds_doubles<DB, true, RF>())];
  const int nbA = (A.nenv + kEnvPerWave - 1) / kEnvPerWave;
  const int blk = static_cast<int>(blockIdx.x);
  if (blk < nbA)
    ipm_block<DA, true, false, RF>(A.P, blk, A.nenv, A.mask, A.ws, A.tau, A.x, A.status,
                                       A.iters, nullptr, 0, sm);
  else
    ipm_block<DB, true, false, RF>(B.P, blk - nbA, B.nenv, B.mask, B.ws, B.tau, B.x,
                                       B.status, B.iters, nullptr, 0, sm);
}

// ============================ kernel 3: dual solution (optional output) ======================
// The reference's OsqpSolver::dual_solution (operational_space_controller.h:534-535) over its rows
// A = [Aeq; Aineq; I_n] (osc.h:483-497; with wheel rows Aeq = [dynamics; wheel rows]) in OSQP's
// sign convention (H x + f + A'y = 0, y >= 0 on an active upper bound, <= 0 on a lower one),
// recovered from the returned design vector x = (dv, u, z) by stationarity:
//   dynamics rows  nu = -M^-1 (H_dv dv + f_dv + E'nu_w)             (the dv block)
//   wheel rows     nu_w = R'(w - V g0) from the refinement's multipliers w (W_NU)
//   u box rows     nu_a - 2 (w_tau + w_reg) u                        (the u block)
//   contact k      r_k = 2 w_reg z_k - Jc_k'nu must be balanced by its active rows: the pyramid
//                  rows, fz >= 0, fz <= big_number (a tiny non-negative least squares over the
//                  active rows, every subset of at most three -- Caratheodory -- tried: the apex,
//                  where five rows are active on three forces, has non-unique multipliers);
//                  fx, fy have no bounds (y = 0); a contact off the ground (l = u = 0) takes -r_k.
// A design vector that is not optimal shows up as a residual of the z block, a u-box multiplier of
// the wrong sign or one on an inactive bound -- the KKT certificate of tests/test_gpu_wheels.py.
// One 64-lane wavefront per env; M is factored in LDS (left-looking Cholesky, lane = row).
template <class D>
__global__ __launch_bounds__(kWave) void osc_dual_kernel(
    const DevParams* __restrict__ P, int nenv, const double* __restrict__ gM,
    const double* __restrict__ gJ, const double* __restrict__ gmask,
    const double* __restrict__ gwd, const double* __restrict__ ws, const double* __restrict__ gx,
    double* __restrict__ gy) {
  constexpr int NV = D::NV, NU = D::NU, NC = D::NC, NS = D::NS, NW = D::NW, NX = D::NX,
                S = D::S, NB = D::NB;
  constexpr int NROW = NV + NW + 4 * NC + NX, JC0 = 3 * (NS - NC);
  static_assert(NC <= kWave, "one lane per contact");
  __shared__ double sL[NV * NV];
  __shared__ double sg[NV];
  __shared__ double snu[NW > 0 ? NW : 1];
  __shared__ double sq[NC * 6];   // per contact: 4 pyramid rows, fz >= 0, fz <= ub (>= 0 each)
  __shared__ double sr[NC * 3];   // per contact: r_k
  const int env = static_cast<int>(blockIdx.x), lane = static_cast<int>(threadIdx.x);
  if (env >= nenv) return;
  const double* w = ws + static_cast<size_t>(env) * D::WS;
  const double* x = gx + static_cast<size_t>(env) * NX;
  const double* J = gJ + static_cast<size_t>(env) * S * NV;
  const double* mask = gmask + static_cast<size_t>(env) * NC;
  for (int p = lane; p < NV * NV; p += kWave) sL[p] = gM[static_cast<size_t>(env) * NV * NV + p];
  if (lane < NV) {   // g0 = H_dv dv + f_dv
    double a = w[D::W_GD + lane];
    for (int j = 0; j < NV; ++j) a = fma(w[D::W_HD + lane * NV + j], x[j], a);
    sg[lane] = a;
  }
  __syncthreads();
  for (int k = 0; k < NV; ++k) {   // M = L L' (lower triangle of sL), column k
    double t = 0.0;
    if (lane >= k && lane < NV) {
      t = sL[lane * NV + k];
      for (int p = 0; p < k; ++p) t = fma(-sL[lane * NV + p], sL[k * NV + p], t);
      sL[lane * NV + k] = t;
    }
    __syncthreads();
    const double dk = sqrt(sL[k * NV + k]);
    __syncthreads();
    if (lane >= k && lane < NV) sL[lane * NV + k] = (lane == k) ? dk : t / dk;
    __syncthreads();
  }
  // L L' v = b in place (one lane, serial)
  auto chol_solve = [&](double* v) {
    for (int i = 0; i < NV; ++i) {
      double a = v[i];
      for (int p = 0; p < i; ++p) a = fma(-sL[i * NV + p], v[p], a);
      v[i] = a / sL[i * NV + i];
    }
    for (int i = NV - 1; i >= 0; --i) {
      double a = v[i];
      for (int p = i + 1; p < NV; ++p) a = fma(-sL[p * NV + i], v[p], a);
      v[i] = a / sL[i * NV + i];
    }
  };
  if constexpr (D::WH) {
    // The wheel rows' multipliers nu_w from stationarity itself (round 4; was: the refinement's
    // last residual, W_NU, which exists only where the refinement was kept and is not unique
    // where the rows are dependent).  With E the rows (mask-scaled), W = M^-1 E' and
    // nu0 = -M^-1 g0, the dynamics multipliers are nu = nu0 - W nu_w, and nu_w must make
    //   every torque off its bounds:   nu[NB + q] = 2 (w_tau + w_reg) u_q       (its box y = 0)
    //   every contact in touch:        r_k = 2 w_reg z_k - Jc_k' nu  in the span of its active
    //                                  rows' normals (component orthogonal to them = 0)
    // -- a small linear least-squares problem in nu_w (<= nu + 3 nc rows, 2 nc unknowns).  The
    // contact multipliers then follow by the NNLS below.
    __shared__ double sE[NW > 0 ? NW * NV : 1];      // E, then W' (row w = column w of W)
    __shared__ double sv0[NV];                       // nu0
    __shared__ double sA[(NU + 3 * NC) * (NW > 0 ? NW : 1)];
    __shared__ double sb[NU + 3 * NC];
    __shared__ int snrow;
    __shared__ int spiv[NW > 0 ? NW : 1];
    const double* wd = gwd + static_cast<size_t>(env) * NC * 6;
    if (lane < NW) {
      const int i = lane / 2, side = lane % 2;
      for (int j = 0; j < NV; ++j) {
        double e = 0.0;
        for (int c = 0; c < 3; ++c) e = fma(wd[6 * i + 3 * side + c], J[(JC0 + 3 * i + c) * NV + j], e);
        if (side == 0 && j == P->wheel_dof[i]) e -= P->wheel_radius[i];
        sE[lane * NV + j] = mask[i] * e;
      }
    }
    if (lane < NV) sv0[lane] = -sg[lane];
    __syncthreads();
    if (lane < NW) chol_solve(sE + lane * NV);        // row w <- (M^-1 E')[:, w]
    if (lane == NW) chol_solve(sv0);                  // nu0 = -M^-1 g0
    __syncthreads();
    // the contact rows of J against W's columns and nu0 (Jc_k' W, Jc_k' nu0), all lanes: the
    // least-squares rows below are combinations of them (lane 0 formed each one serially)
    __shared__ double sJW[3 * NC * (NW > 0 ? NW : 1)];
    __shared__ double sJN0[3 * NC];
    for (int p = lane; p < 3 * NC * NW + 3 * NC; p += kWave) {
      const int kc = p < 3 * NC * NW ? p / NW : p - 3 * NC * NW;
      const double* jr = J + (JC0 + kc) * NV;
      const double* v = p < 3 * NC * NW ? sE + (p % NW) * NV : sv0;
      double a = 0.0;
      for (int i = 0; i < NV; ++i) a = fma(jr[i], v[i], a);
      if (p < 3 * NC * NW) sJW[p] = a;
      else sJN0[kc] = a;
    }
    __syncthreads();
    if (lane == 0) {
      const double wu = 2.0 * (P->w_torque + P->w_reg), wz = 2.0 * P->w_reg, mu = P->mu;
      int n = 0;
      for (int q = 0; q < NU; ++q) {   // torques off their bounds
        const double u = x[NV + q];
        const double tol = 1e-9 * (1.0 + fabs(u));
        const bool hi = fabs(P->u_ub[q]) < P->inf_thresh && u >= P->u_ub[q] - tol;
        const bool lo = fabs(P->u_lb[q]) < P->inf_thresh && u <= P->u_lb[q] + tol;
        if (hi || lo) continue;
        for (int w = 0; w < NW; ++w) sA[n * NW + w] = -sE[w * NV + NB + q];
        sb[n++] = wu * u - sv0[NB + q];
      }
      for (int k = 0; k < NC; ++k) {   // contacts in touch: r_k orthogonal to no active normal
        if (mask[k] == 0.0) continue;
        const double f0 = x[NV + NU + 3 * k], f1 = x[NV + NU + 3 * k + 1], f2 = x[NV + NU + 3 * k + 2];
        const double tol = 1e-9 * (1.0 + fmax(fabs(f0), fmax(fabs(f1), fabs(f2))));
        double q[3][3];   // orthonormal basis of the active normals' span (Gram-Schmidt)
        int rk = 0;
        const double ub = P->z_ub[2] * mask[k], lb = P->z_lb[2] * mask[k];
        for (int i = 0; i < 6; ++i) {
          double g[3];
          double gap;
          if (i < 4) {
            g[0] = (i & 1) ? -1.0 : 1.0; g[1] = (i >= 2) ? -1.0 : 1.0; g[2] = -mu;
            gap = -(g[0] * f0 + g[1] * f1 + g[2] * f2);
          } else if (i == 4) {
            if (!(fabs(lb) < P->inf_thresh)) continue;
            g[0] = g[1] = 0.0; g[2] = -1.0; gap = f2 - lb;
          } else {
            if (!(fabs(ub) < P->inf_thresh)) continue;
            g[0] = g[1] = 0.0; g[2] = 1.0; gap = ub - f2;
          }
          if (gap > tol || rk == 3) continue;
          for (int a = 0; a < rk; ++a) {
            const double d = g[0] * q[a][0] + g[1] * q[a][1] + g[2] * q[a][2];
            for (int c = 0; c < 3; ++c) g[c] -= d * q[a][c];
          }
          const double nn = sqrt(g[0] * g[0] + g[1] * g[1] + g[2] * g[2]);
          if (nn > 1e-6) {
            for (int c = 0; c < 3; ++c) q[rk][c] = g[c] / nn;
            ++rk;
          }
        }
        // complement: e_c orthogonalised against the span and the complement vectors so far
        int nc = 0;
        double pc[3][3];
        for (int c = 0; c < 3 && rk + nc < 3; ++c) {
          double v[3] = {c == 0 ? 1.0 : 0.0, c == 1 ? 1.0 : 0.0, c == 2 ? 1.0 : 0.0};
          for (int a = 0; a < rk; ++a) {
            const double d = v[0] * q[a][0] + v[1] * q[a][1] + v[2] * q[a][2];
            for (int e = 0; e < 3; ++e) v[e] -= d * q[a][e];
          }
          for (int a = 0; a < nc; ++a) {
            const double d = v[0] * pc[a][0] + v[1] * pc[a][1] + v[2] * pc[a][2];
            for (int e = 0; e < 3; ++e) v[e] -= d * pc[a][e];
          }
          const double nn = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
          if (nn < 0.5) continue;
          for (int e = 0; e < 3; ++e) pc[nc][e] = v[e] / nn;
          // p' r_k = 0 with r_k = wz f - Jc_k' (nu0 - W nu_w)
          double rhs = 0.0;
          double* row = sA + n * NW;   // (built in place)
          for (int w = 0; w < NW; ++w) row[w] = 0.0;
          for (int cc = 0; cc < 3; ++cc) {
            const double jn0 = sJN0[3 * k + cc];
            const double fc = cc == 0 ? f0 : (cc == 1 ? f1 : f2);
            rhs = fma(pc[nc][cc], wz * fc - jn0, rhs);
            for (int w = 0; w < NW; ++w) row[w] = fma(pc[nc][cc], sJW[(3 * k + cc) * NW + w], row[w]);
          }
          sb[n++] = -rhs;   // row . nu_w = -rhs
          ++nc;
        }
      }
      snrow = n;
    }
    __syncthreads();
    // the basic least-squares solution by Householder QR with column pivoting (rank: |R_jj| >
    // 1e-10 |R_00|; the dependent rows' multipliers are zero).  (Normal equations do not do: the
    // rows that fix dv need multipliers up to ~1e6 along directions whose singular values are
    // ~1e-9 of the largest -- squared, they drown in rounding.)  Lane c owns column c (lane NW:
    // the right-hand side b): norms, reflections and updates run per column in parallel, each in
    // the serial order.
    const int n = snrow;
    double* A = sA;
    double* bb = sb;
    if (lane < NW) spiv[lane] = lane;
    double nmax0 = 0.0;
    int rank = 0;
    for (int j = 0; j < NW && j < n; ++j) {
      double v = -1.0;
      int p = lane;
      if (lane >= j && lane < NW) {
        v = 0.0;
        for (int t = j; t < n; ++t) v = fma(A[t * NW + lane], A[t * NW + lane], v);
      }
      for (int o = kWave / 2; o > 0; o >>= 1) {   // the largest, the lowest column among ties
        const double ov = __shfl_xor(v, o, kWave);
        const int op = __shfl_xor(p, o, kWave);
        if (ov > v || (ov == v && op < p)) {
          v = ov;
          p = op;
        }
      }
      const double cn = sqrt(v);
      if (j == 0) nmax0 = cn;
      if (!(cn > 1e-10 * nmax0) || cn == 0.0) break;
      __syncthreads();
      if (p != j) {   // lanes j and p swap their columns (row t: both read, then both write)
        if (lane == j || lane == p) {
          const int o = lane == j ? p : j;
          for (int t = 0; t < n; ++t) {
            const double a = A[t * NW + o];
            A[t * NW + lane] = a;
          }
        }
        if (lane == 0) {
          const int ti = spiv[j];
          spiv[j] = spiv[p];
          spiv[p] = ti;
        }
        __syncthreads();
      }
      const double ajj = A[j * NW + j];
      const double alpha = ajj > 0.0 ? -cn : cn;
      // v = A[j:, j] - alpha e_1;  H = I - 2 v v' / (v'v)
      const double v0 = ajj - alpha;
      const double vn2 = 2.0 * cn * (cn + fabs(ajj));   // = v'v, cancellation-free
      if (vn2 > 0.0 && lane > j && lane <= NW) {
        double* col = lane < NW ? A + lane : bb;
        const int cs = lane < NW ? NW : 1;
        double sd = v0 * col[j * cs];
        for (int t = j + 1; t < n; ++t) sd = fma(A[t * NW + j], col[t * cs], sd);
        const double f = 2.0 * sd / vn2;
        col[j * cs] -= f * v0;
        for (int t = j + 1; t < n; ++t) col[t * cs] = fma(-f, A[t * NW + j], col[t * cs]);
      }
      __syncthreads();
      if (lane == j) A[j * NW + j] = alpha;
      rank = j + 1;
      __syncthreads();
    }
    if (lane == 0) {
      for (int a = 0; a < NW; ++a) snu[a] = 0.0;
      for (int a = rank - 1; a >= 0; --a) {   // R z = Q'b, z -> nu_w[piv]
        double v = bb[a];
        for (int e = a + 1; e < rank; ++e) v = fma(-A[a * NW + e], snu[spiv[e]], v);
        snu[spiv[a]] = v / A[a * NW + a];
      }
    }
  }
  __syncthreads();
  if (lane < NV) {   // g_x = g0 (+ E' nu_w)
    double a = sg[lane];
    if constexpr (D::WH) {
      const double* wd = gwd + static_cast<size_t>(env) * NC * 6;
      for (int i = 0; i < NC; ++i) {
        double er = 0.0, el = 0.0;
        for (int c = 0; c < 3; ++c) {
          const double jv = J[(JC0 + 3 * i + c) * NV + lane];
          er = fma(wd[6 * i + c], jv, er);
          el = fma(wd[6 * i + 3 + c], jv, el);
        }
        if (lane == P->wheel_dof[i]) er -= P->wheel_radius[i];
        a = fma(mask[i] * er, snu[2 * i], a);
        a = fma(mask[i] * el, snu[2 * i + 1], a);
      }
    }
    sg[lane] = -a;
  }
  __syncthreads();
  if (lane == 0) {   // L L' nu = -g_x
    for (int i = 0; i < NV; ++i) {
      double a = sg[i];
      for (int p = 0; p < i; ++p) a = fma(-sL[i * NV + p], sg[p], a);
      sg[i] = a / sL[i * NV + i];
    }
    for (int i = NV - 1; i >= 0; --i) {
      double a = sg[i];
      for (int p = i + 1; p < NV; ++p) a = fma(-sL[p * NV + i], sg[p], a);
      sg[i] = a / sL[i * NV + i];
    }
  }
  __syncthreads();
  if (lane < NC) {   // contact `lane`: r_k, then its rows' multipliers
    const int k = lane;
    const double wz = 2.0 * P->w_reg, mu = P->mu;
    double r[3], f[3];
    for (int c = 0; c < 3; ++c) {
      f[c] = x[NV + NU + 3 * k + c];
      double a = wz * f[c];
      for (int i = 0; i < NV; ++i) a = fma(-J[(JC0 + 3 * k + c) * NV + i], sg[i], a);
      r[c] = a;
      sr[3 * k + c] = a;
    }
    double q[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    if (mask[k] != 0.0) {
      // rows g_i' f <= h_i: pyramid (sx, sy, -mu) <= 0, -fz <= -lb, fz <= ub
      const double ub = P->z_ub[2] * mask[k], lb = P->z_lb[2] * mask[k];
      double g[6][3], h[6];
      for (int i = 0; i < 4; ++i) {
        g[i][0] = (i & 1) ? -1.0 : 1.0;
        g[i][1] = (i >= 2) ? -1.0 : 1.0;
        g[i][2] = -mu;
        h[i] = 0.0;
      }
      g[4][0] = g[4][1] = 0.0; g[4][2] = -1.0; h[4] = -lb;
      g[5][0] = g[5][1] = 0.0; g[5][2] = 1.0;  h[5] = ub;
      const double tol = 1e-8 * (1.0 + fmax(fabs(f[0]), fmax(fabs(f[1]), fabs(f[2]))));
      int act = 0;
      for (int i = 0; i < 6; ++i) {
        const double gi = g[i][0] * f[0] + g[i][1] * f[1] + g[i][2] * f[2] - h[i];
        const bool finite = (i < 4) || fabs(h[i]) < P->inf_thresh;
        if (finite && gi >= -tol) act |= 1 << i;
      }
      // min |r + G_S' m| over m >= 0, S a subset of the active rows with |S| <= 3
      double best = r[0] * r[0] + r[1] * r[1] + r[2] * r[2];
      int bestS = 0;
      double bm[3] = {0.0, 0.0, 0.0};
      for (int S = 1; S < 64; ++S) {
        if ((S & act) != S || __builtin_popcount(S) > 3) continue;
        int id[3], n = 0;
        for (int i = 0; i < 6; ++i)
          if (S >> i & 1) id[n++] = i;
        double A[3][3], bb[3];   // (G_S G_S') m = -G_S r
        for (int a = 0; a < n; ++a) {
          bb[a] = -(g[id[a]][0] * r[0] + g[id[a]][1] * r[1] + g[id[a]][2] * r[2]);
          for (int c = 0; c < n; ++c)
            A[a][c] = g[id[a]][0] * g[id[c]][0] + g[id[a]][1] * g[id[c]][1] + g[id[a]][2] * g[id[c]][2];
        }
        bool ok = true;   // Gaussian elimination with partial pivoting, n <= 3
        for (int c = 0; c < n && ok; ++c) {
          int p = c;
          for (int a = c + 1; a < n; ++a)
            if (fabs(A[a][c]) > fabs(A[p][c])) p = a;
          if (fabs(A[p][c]) < 1e-12) { ok = false; break; }
          if (p != c) {
            for (int e = 0; e < n; ++e) { const double t = A[c][e]; A[c][e] = A[p][e]; A[p][e] = t; }
            const double t = bb[c]; bb[c] = bb[p]; bb[p] = t;
          }
          for (int a = c + 1; a < n; ++a) {
            const double fct = A[a][c] / A[c][c];
            for (int e = c; e < n; ++e) A[a][e] -= fct * A[c][e];
            bb[a] -= fct * bb[c];
          }
        }
        if (!ok) continue;
        double m[3];
        for (int a = n - 1; a >= 0; --a) {
          double t = bb[a];
          for (int e = a + 1; e < n; ++e) t -= A[a][e] * m[e];
          m[a] = t / A[a][a];
        }
        bool nonneg = true;
        for (int a = 0; a < n; ++a) nonneg = nonneg && m[a] >= 0.0;
        if (!nonneg) continue;
        double res = 0.0;
        for (int c = 0; c < 3; ++c) {
          double t = r[c];
          for (int a = 0; a < n; ++a) t += m[a] * g[id[a]][c];
          res += t * t;
        }
        if (res < best * (1.0 - 1e-12)) {
          best = res;
          bestS = S;
          for (int a = 0; a < 3; ++a) bm[a] = a < n ? m[a] : 0.0;
        }
      }
      for (int i = 0, a = 0; i < 6; ++i)
        if (bestS >> i & 1) q[i] = bm[a++];
    }
    for (int i = 0; i < 6; ++i) sq[6 * k + i] = q[i];
  }
  __syncthreads();
  double* y = gy + static_cast<size_t>(env) * NROW;
  const double wu = 2.0 * (P->w_torque + P->w_reg);
  for (int r = lane; r < NROW; r += kWave) {
    double v = 0.0;
    if (r < NV) {
      v = sg[r];
    } else if (r < NV + NW) {
      v = snu[r - NV];
    } else if (r < NV + NW + 4 * NC) {
      const int k = (r - NV - NW) / 4, rr = (r - NV - NW) % 4;
      v = sq[6 * k + rr];
    } else {
      const int c = r - NV - NW - 4 * NC;   // design variable of the box row
      if (c >= NV && c < NV + NU) {
        v = sg[NB + c - NV] - wu * x[c];
      } else if (c >= NV + NU) {
        const int zc = c - NV - NU, k = zc / 3;
        if (mask[k] == 0.0) v = -sr[zc];
        else if (zc % 3 == 2) v = sq[6 * k + 5] - sq[6 * k + 4];
      }
    }
    y[r] = v;
  }
}

// a wave-uniform lane's double (v_readlane_b32 x2: no LDS round trip)
__device__ __forceinline__ double readlane_d(double v, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}

// ==================== kernel 4: wheel-row fallback (Goldfarb-Idnani, optional) ==================
// An env the wheel-row interior point leaves at max_iter (~0.5 % of tumbling envs: QPs whose
// multipliers reach 1e7-3e8 -- the rows nearly inconsistent with the torque limits, DESIGN.md
// §3.1) is solved again by Goldfarb & Idnani's dual active-set method (Math. Programming 27,
// 1983; quadprog's algorithm, oracle/qp_exact.py::_dual_active_set) on the FULL reference QP of the
// env (x = (dv, u, z); rows as c'x >= b): start at the unconstrained minimiser, add the equality
// rows (dynamics, wheel rows, the forces of contacts off the ground), then repeatedly the most
// violated one-sided row, dropping working rows whose multiplier would turn negative.  Every
// iterate is dual feasible, so it terminates; J = L^-T Q and R are kept by Givens rotations.
// tools/gi_fallback_model.py is the numpy restatement of exactly this sequence (its torques are
// within 1e-11 of the exact oracle on every MAX_ITER env of three 2,048-env censuses).  An env the
// method certifies (rows held to 1e-8, one-sided rows feasible) reports OK with its x and tau;
// otherwise it keeps the interior point's result and status.
// One 64-lane wavefront per env, early exit for envs already OK.  Lanes own J's rows (row i of
// J = lane i), the working set's multipliers and row ids (lane j = position j), and the
// one-sided rows (lane p = row p) for the violation scan.
template <class D>
__global__ __launch_bounds__(kWave) void osc_gi_kernel(
    const DevParams* __restrict__ P, int nenv, const double* __restrict__ gM,
    const double* __restrict__ gC, const double* __restrict__ gJ, const double* __restrict__ gb,
    const double* __restrict__ gmask, const double* __restrict__ gwd,
    const double* __restrict__ ws, double* __restrict__ gtau, double* __restrict__ gx,
    int32_t* __restrict__ gstatus) {
  constexpr int NV = D::NV, NU = D::NU, NC = D::NC, NS = D::NS, NW = D::NW, NX = D::NX,
                NB = D::NB, NZ = D::NZ;
  constexpr int NXP = NX | 1;                 // odd row stride (LDS banks)
  constexpr int NEQ = NV + NW + NZ;           // dynamics, wheel rows, forces of masked contacts
  constexpr int NIN = 2 * NU + 6 * NC;        // one-sided rows: u box, pyramid, fz box
  constexpr int JC0 = 3 * (NS - NC);          // first contact translational row of J
  constexpr int kIneq = 1 << 12;              // row ids: equality k, one-sided kIneq + p
  constexpr int kMaxSteps = 400;
  static_assert(NX <= kWave && NIN <= kWave && NEQ <= kWave, "one lane per variable / row");
  const int env = static_cast<int>(blockIdx.x), lane = static_cast<int>(threadIdx.x);
  if (env >= nenv) return;
  if (gstatus[env] == OSC_SOLVE_OK) return;   // (block-uniform)
  __shared__ double sE[NEQ * NXP];            // equality rows, dense
  __shared__ double sEb[NEQ];
  __shared__ double sJ[NX * NXP];             // J (row i at i * NXP); first the Cholesky factor
  __shared__ double sR[NX * NXP];             // R, upper triangular (row i at i * NXP)
  __shared__ double sx[NX], sc[NX], sd[NX], sgc[NX], sgs[NX], sRi[NX];   // sRi: 1 / R[j][j]
  const double* wenv = ws + static_cast<size_t>(env) * D::WS;
  const double* M = gM + static_cast<size_t>(env) * NV * NV;
  const double* C = gC + static_cast<size_t>(env) * NV;
  const double* J = gJ + static_cast<size_t>(env) * D::S * NV;
  const double* bb = gb + static_cast<size_t>(env) * D::S;
  const double* mask = gmask + static_cast<size_t>(env) * NC;
  const double* wd = gwd + static_cast<size_t>(env) * NC * 6;
  const double hu = 2.0 * (P->w_torque + P->w_reg), hz = 2.0 * P->w_reg;

  auto wsum = [](double v) {
    for (int o = kWave / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
    return v;
  };
  auto wmax = [](double v) {
    for (int o = kWave / 2; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, kWave));
    return v;
  };
  // (value, index) minimum, the lowest index among ties
  auto wargmin = [](double& v, int& idx) {
    for (int o = kWave / 2; o > 0; o >>= 1) {
      const double ov = __shfl_xor(v, o, kWave);
      const int oi = __shfl_xor(idx, o, kWave);
      if (ov < v || (ov == v && oi < idx)) {
        v = ov;
        idx = oi;
      }
    }
  };
  // one-sided row p (c'x >= b): its coefficient on variable i, right-hand side, max |c|, and
  // whether it exists (finite bound; the fz box only on contacts in touch)
  auto in_coef = [&](int p, int i) -> double {
    if (p < 2 * NU) return (i == NV + p / 2) ? ((p & 1) ? 1.0 : -1.0) : 0.0;
    const int k = (p - 2 * NU) / 6, r = (p - 2 * NU) % 6, c0 = NV + NU + 3 * k;
    if (i < c0 || i >= c0 + 3) return 0.0;
    if (r < 4) {   // (sx, sy, -mu) z <= 0 (autogen.py:112-117 order)
      const double sx = (r & 1) ? -1.0 : 1.0, sy = (r >= 2) ? -1.0 : 1.0;
      return i == c0 ? -sx : (i == c0 + 1 ? -sy : P->mu);
    }
    return i == c0 + 2 ? (r == 4 ? 1.0 : -1.0) : 0.0;
  };
  auto in_rhs = [&](int p) -> double {
    if (p < 2 * NU) return (p & 1) ? P->u_lb[p / 2] : -P->u_ub[p / 2];
    const int k = (p - 2 * NU) / 6, r = (p - 2 * NU) % 6;
    return r < 4 ? 0.0 : (r == 4 ? P->z_lb[2] * mask[k] : -P->z_ub[2] * mask[k]);
  };
  auto in_valid = [&](int p) -> bool {
    if (p >= NIN) return false;
    if (p < 2 * NU) return fabs((p & 1) ? P->u_lb[p / 2] : P->u_ub[p / 2]) < P->inf_thresh;
    const int k = (p - 2 * NU) / 6, r = (p - 2 * NU) % 6;
    if (r < 4) return true;
    return mask[k] != 0.0 && fabs(r == 4 ? P->z_lb[2] : P->z_ub[2]) < P->inf_thresh;
  };
  // c_p'x - b_p from the current x in sx (the row's <= 3 nonzeros)
  auto in_slack = [&](int p) -> double {
    double v = -in_rhs(p);
    if (p < 2 * NU) return fma(in_coef(p, NV + p / 2), sx[NV + p / 2], v);
    const int c0 = NV + NU + 3 * ((p - 2 * NU) / 6);
    for (int i = c0; i < c0 + 3; ++i) v = fma(in_coef(p, i), sx[i], v);
    return v;
  };
  auto in_scale = [&](int p) -> double {
    return (p >= 2 * NU && (p - 2 * NU) % 6 < 4) ? fmax(1.0, fabs(P->mu)) : 1.0;
  };

  // ---- the equality rows (the reference's Aeq = [M, -B, -Jc], beq = -C; its wheel rows; z = 0
  // on contacts off the ground) ----
  int neq = 0;
  for (int i = 0; i < NV; ++i) {
    if (lane < NX) {
      double v;
      if (lane < NV) v = M[i * NV + lane];
      else if (lane < NV + NU) v = (i == NB + lane - NV) ? -1.0 : 0.0;
      else v = -J[(JC0 + lane - NV - NU) * NV + i];
      sE[neq * NXP + lane] = v;
    }
    if (lane == 0) sEb[neq] = -C[i];
    ++neq;
  }
  for (int w = 0; w < NW; ++w) {   // osc_qp.wheel_rows (walter_sr_wheels/autogen.py:151-205)
    const int i = w / 2, side = w % 2;
    if (lane < NX) {
      double v = 0.0;
      if (lane < NV) {
        for (int c = 0; c < 3; ++c) v = fma(wd[6 * i + 3 * side + c], J[(JC0 + 3 * i + c) * NV + lane], v);
        if (side == 0 && lane == P->wheel_dof[i]) v -= P->wheel_radius[i];
        v *= mask[i];
      }
      sE[neq * NXP + lane] = v;
    }
    if (lane == 0) {
      double e = 0.0;
      for (int c = 0; c < 3; ++c) e = fma(wd[6 * i + 3 * side + c], bb[JC0 + 3 * i + c], e);
      sEb[neq] = -mask[i] * e;
    }
    ++neq;
  }
  for (int k = 0; k < NC; ++k) {
    if (mask[k] != 0.0) continue;
    for (int c = 0; c < 3; ++c) {
      if (lane < NX) sE[neq * NXP + lane] = (lane == NV + NU + 3 * k + c) ? 1.0 : 0.0;
      if (lane == 0) sEb[neq] = 0.0;
      ++neq;
    }
  }

  // ---- H = blockdiag(H_dv, hu I, hz I) = L L';  J = L^-T;  x = -H^-1 f ----
  for (int p = lane; p < NV * NV; p += kWave) sR[(p / NV) * NXP + p % NV] = wenv[D::W_HD + p];
  __syncthreads();
  for (int k = 0; k < NV; ++k) {   // left-looking Cholesky of H_dv in sR, lane = row
    double t = 0.0;
    if (lane >= k && lane < NV) {
      t = sR[lane * NXP + k];
      for (int p = 0; p < k; ++p) t = fma(-sR[lane * NXP + p], sR[k * NXP + p], t);
      sR[lane * NXP + k] = t;
    }
    __syncthreads();
    const double dk = sqrt(sR[k * NXP + k]);
    __syncthreads();
    if (lane >= k && lane < NV) sR[lane * NXP + k] = (lane == k) ? dk : t / dk;
    __syncthreads();
  }
  if (lane < NX) {
    // lane j: column j of L^-1 (forward substitution of e_j) = row j of J = L^-T
    for (int c = 0; c < NX; ++c) sJ[lane * NXP + c] = 0.0;
    if (lane < NV) {
      double y[NV];
#pragma unroll
      for (int r = 0; r < NV; ++r) {
        double a = (r == lane) ? 1.0 : 0.0;
#pragma unroll
        for (int k = 0; k < r; ++k) a = fma(-sR[r * NXP + k], y[k], a);
        y[r] = a / sR[r * NXP + r];
      }
#pragma unroll
      for (int r = 0; r < NV; ++r) sJ[lane * NXP + r] = y[r];
    } else {
      sJ[lane * NXP + lane] = 1.0 / sqrt(lane < NV + NU ? hu : hz);
    }
  }
  __syncthreads();
  for (int p = lane; p < NX * NXP; p += kWave) sR[p] = 0.0;
  // x_dv = -J_dv J_dv' f_dv; u = z = 0
  if (lane < NX) sc[lane] = lane < NV ? wenv[D::W_GD + lane] : 0.0;
  __syncthreads();
  if (lane < NX) {
    double t = 0.0;
    for (int i = 0; i < NX; ++i) t = fma(sJ[i * NXP + lane], sc[i], t);
    sd[lane] = t;
  }
  __syncthreads();
  double xi = 0.0;   // lane i: x_i
  if (lane < NX) {
    for (int j = 0; j < NX; ++j) xi = fma(-sJ[lane * NXP + j], sd[j], xi);
    sx[lane] = xi;
  }
  // the dependence test's scale: J's largest row norm (invariant under J <- J Q)
  double rn = 0.0;
  if (lane < NX)
    for (int c = 0; c < NX; ++c) rn = fma(sJ[lane * NXP + c], sJ[lane * NXP + c], rn);
  const double jscale = sqrt(wmax(rn));
  __syncthreads();

  int q = 0;            // working rows
  int act = -1;         // lane j < q: row id of working row j
  double up = 0.0;      // lane j <= q: multipliers (j = q: the candidate's)
  double zi = 0.0;      // lane i: the primal step direction z
  double rj = 0.0;      // lane j < q: R^-1 d[:q]
  // d = J'c (lane j -> sd), z = J[:, q:] d[q:] (lane i), r = R^-1 d[:q] (lane j).  c: a dense
  // equality row in sc, or one-sided row p (<= 3 nonzeros: only those rows of J are read)
  auto directions = [&](int p) {
    if (lane < NX) {
      double t = 0.0;
      if (p < 0) {
        double t1 = 0.0, t2 = 0.0, t3 = 0.0;
        int i = 0;
        for (; i + 3 < NX; i += 4) {
          t = fma(sJ[i * NXP + lane], sc[i], t);
          t1 = fma(sJ[(i + 1) * NXP + lane], sc[i + 1], t1);
          t2 = fma(sJ[(i + 2) * NXP + lane], sc[i + 2], t2);
          t3 = fma(sJ[(i + 3) * NXP + lane], sc[i + 3], t3);
        }
        for (; i < NX; ++i) t = fma(sJ[i * NXP + lane], sc[i], t);
        t = (t + t1) + (t2 + t3);
      } else if (p < 2 * NU) {
        t = in_coef(p, NV + p / 2) * sJ[(NV + p / 2) * NXP + lane];
      } else {
        const int c0 = NV + NU + 3 * ((p - 2 * NU) / 6);
        for (int i = c0; i < c0 + 3; ++i) t = fma(in_coef(p, i), sJ[i * NXP + lane], t);
      }
      sd[lane] = t;
    }
    __syncthreads();
    zi = 0.0;
    if (lane < NX) {
      double z1 = 0.0;
      int j = q;
      for (; j + 1 < NX; j += 2) {
        zi = fma(sJ[lane * NXP + j], sd[j], zi);
        z1 = fma(sJ[lane * NXP + j + 1], sd[j + 1], z1);
      }
      if (j < NX) zi = fma(sJ[lane * NXP + j], sd[j], zi);
      zi += z1;
    }
    double dv = lane < q ? sd[lane] : 0.0;
    rj = 0.0;
    for (int jj = q - 1; jj >= 0; --jj) {   // back substitution, column-oriented
      const double v = readlane_d(dv, jj) * sRi[jj];
      if (lane == jj) rj = v;
      if (lane < jj) dv = fma(-sR[lane * NXP + jj], v, dv);
    }
  };
  // c joins the working set at position q: the rotations (j-1, j), j = NX-1 .. q+1, that fold
  // d[q+1:] into d[q] (J's columns follow); rotation j meets (d[j-1], ||d[j:]||) -- d[NX-1] itself,
  // signed, for the first -- so every (c, s) follows from d's suffix sums of squares, one wave
  // scan instead of a chain of NX - q dependent rotations.  R's column q = d[:q+1].
  auto add_row = [&]() {
    const double dl = lane < NX ? sd[lane] : 0.0;
    double ssq = (lane >= q && lane < NX) ? dl * dl : 0.0;
    for (int o = 1; o < kWave; o <<= 1) {   // suffix sums S_j = sum_{k >= j} d_k^2
      const double v = __shfl_down(ssq, o, kWave);
      if (lane + o < kWave) ssq += v;
    }
    const double sn = __shfl_down(ssq, 1, kWave);            // S_{j+1} on lane j
    const double dnext = __shfl_down(dl, 1, kWave);          // d_{j+1} on lane j
    if (lane >= q && lane < NX - 1) {   // lane j - 1 holds rotation j's (c, s)
      const double rr = sqrt(ssq);
      double c = 1.0, sv = 0.0;
      if (rr > 0.0) {
        c = dl / rr;
        sv = (lane + 1 == NX - 1 ? dnext : sqrt(sn)) / rr;
      }
      sgc[lane + 1] = c;
      sgs[lane + 1] = sv;
    }
    const double dq = __shfl(q < NX - 1 ? sqrt(ssq) : dl, q, kWave);
    __syncthreads();
    if (lane < NX) {
      double row[NX];
#pragma unroll
      for (int c = 0; c < NX; ++c) row[c] = sJ[lane * NXP + c];
#pragma unroll
      for (int j = NX - 1; j >= 1; --j) {
        if (j > q) {
          const double c = sgc[j], sv = sgs[j];
          const double a = row[j - 1], b = row[j];
          row[j - 1] = c * a + sv * b;
          row[j] = -sv * a + c * b;
        }
      }
#pragma unroll
      for (int c = 0; c < NX; ++c) sJ[lane * NXP + c] = row[c];
    }
    if (lane < q) sR[lane * NXP + q] = dl;
    if (lane == q) {
      sR[q * NXP + q] = dq;
      sRi[q] = 1.0 / dq;
    }
    __syncthreads();
  };
  // working row k leaves: R's columns k+1.. shift left and are re-triangularised by rotations of
  // rows (j, j+1), J's columns (j, j+1) follow; the lanes' ids / multipliers shift down
  auto drop_row = [&](int k) {
    if (lane < q)
      for (int c = k; c < q - 1; ++c) sR[lane * NXP + c] = sR[lane * NXP + c + 1];
    if (lane < NX) sR[lane * NXP + q - 1] = 0.0;
    __syncthreads();
    for (int j = k; j < q - 1; ++j) {
      const double a = sR[j * NXP + j], b = sR[(j + 1) * NXP + j];
      double c = 1.0, s = 0.0;
      if (b != 0.0) {
        const double r = hypot(a, b);
        c = a / r;
        s = b / r;
      }
      __syncthreads();
      if (lane >= j && lane < q - 1) {
        const double ra = sR[j * NXP + lane], rb = sR[(j + 1) * NXP + lane];
        sR[j * NXP + lane] = c * ra + s * rb;
        sR[(j + 1) * NXP + lane] = -s * ra + c * rb;
      }
      if (lane == 0) {
        sgc[j] = c;
        sgs[j] = s;
      }
      __syncthreads();
    }
    if (lane < NX) sR[(q - 1) * NXP + lane] = 0.0;
    if (lane >= k && lane < q - 1) sRi[lane] = 1.0 / sR[lane * NXP + lane];
    if (lane < NX) {
      for (int j = k; j < q - 1; ++j) {
        const double c = sgc[j], s = sgs[j];
        const double a = sJ[lane * NXP + j], b = sJ[lane * NXP + j + 1];
        sJ[lane * NXP + j] = c * a + s * b;
        sJ[lane * NXP + j + 1] = -s * a + c * b;
      }
    }
    const int na = __shfl_down(act, 1, kWave);
    const double nu_ = __shfl_down(up, 1, kWave);
    if (lane >= k && lane < q) {
      act = na;
      up = nu_;
    }
    if (lane == q) up = 0.0;
    __syncthreads();
  };

  bool ok = true;
  int steps = 0;
#ifdef OSC_GI_PROFILE
  unsigned long long tp[6] = {0, 0, 0, 0, 0, 0}, t0 = 0, t1_ = 0;
  int ndrop = 0, nadd = 0;
#define GI_T0() asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory")
#define GI_T1(k) do { asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1_)::"memory"); tp[k] += t1_ - t0; } while (0)
#else
#define GI_T0() do {} while (0)
#define GI_T1(k) do {} while (0)
#endif
  // ---- equality rows: always in, never dropped; a row dependent on those already in skipped ----
  for (int k = 0; k < neq && ok; ++k) {
    const double ck = lane < NX ? sE[k * NXP + lane] : 0.0;
    if (lane < NX) sc[lane] = ck;
    __syncthreads();
    GI_T0();
    directions(-1);
    GI_T1(0);
    const double zmax = wmax(fabs(zi)), cmax = wmax(fabs(ck));
    if (zmax <= 1e-13 * cmax * (1.0 + jscale)) continue;
    const double cx = wsum(ck * xi), zc = wsum(zi * ck);
    const double t = (sEb[k] - cx) / zc;
    if (!isfinite(t)) { ok = false; break; }
    xi = fma(t, zi, xi);
    if (lane < q) up = fma(-t, rj, up);
    if (lane == q) { up = t; act = k; }
    GI_T0();
    add_row();
    GI_T1(1);
    ++q;
  }
  if (lane < NX) sx[lane] = xi;
  __syncthreads();
  // ---- one-sided rows ----
  while (ok) {
    if (++steps > kMaxSteps) { ok = false; break; }
    GI_T0();
    // working one-sided rows as a bit set over p
    unsigned long long in_set = (lane < q && act >= kIneq) ? (1ull << (act - kIneq)) : 0ull;
    for (int o = kWave / 2; o > 0; o >>= 1) {
      const unsigned lo = __shfl_xor(static_cast<unsigned>(in_set), o, kWave);
      const unsigned hi = __shfl_xor(static_cast<unsigned>(in_set >> 32), o, kWave);
      in_set |= (static_cast<unsigned long long>(hi) << 32) | lo;
    }
    const double xs = wmax(lane < NX ? fabs(xi) : 0.0);
    double viol = INFINITY;
    int p = lane;
    if (in_valid(lane) && !((in_set >> lane) & 1ull))
      viol = in_slack(lane) / (1.0 + in_scale(lane) * xs + fabs(in_rhs(lane)));
    wargmin(viol, p);
    GI_T1(2);
    if (!(viol < -1e-14)) break;   // every one-sided row holds: optimal
    const double cp = lane < NX ? in_coef(p, lane) : 0.0;
    const double bp = in_rhs(p), scp = in_scale(p);
    if (lane < NX) sc[lane] = cp;
    __syncthreads();
    if (lane == q) up = 0.0;
    while (true) {
      if (++steps > kMaxSteps) { ok = false; break; }
      GI_T0();
      directions(p);
      GI_T1(3);
      // partial step: the working one-sided row whose multiplier reaches 0 first
      const double rmax = 1.0 + wmax(lane < q ? fabs(rj) : 0.0);
      double t1 = INFINITY;
      int kd = lane;
      if (lane < q && act >= kIneq && rj > 1e-14 * rmax) t1 = up / rj;
      wargmin(t1, kd);
      const double zmax = wmax(fabs(zi));
      const bool dependent = zmax <= 1e-13 * scp * (1.0 + jscale);
      const double cx = wsum(cp * xi), zc = wsum(zi * cp);
      const double t2 = dependent ? INFINITY : -(cx - bp) / zc;
      const double t = fmin(t1, t2);
      if (!isfinite(t)) { ok = false; break; }
      if (!dependent) xi = fma(t, zi, xi);
      if (lane < q) up = fma(-t, rj, up);
      if (lane == q) up += t;
      if (lane < NX) sx[lane] = xi;
      __syncthreads();
      if (t2 <= t1) {   // full step: p joins
        if (lane == q) act = kIneq + p;
        GI_T0();
        add_row();
        GI_T1(4);
#ifdef OSC_GI_PROFILE
        ++nadd;
#endif
        ++q;
        break;
      }
      GI_T0();
      drop_row(kd);
      GI_T1(5);
#ifdef OSC_GI_PROFILE
      ++ndrop;
#endif
      --q;
    }
  }
#ifdef OSC_GI_PROFILE
  if (lane == 0)
    printf("gi env %d ok %d steps %d neq %d q %d adds %d drops %d cyc eqdir %llu eqadd %llu scan %llu dir %llu add %llu drop %llu\n",
           env, ok ? 1 : 0, steps, neq, q, nadd, ndrop, tp[0], tp[1], tp[2], tp[3], tp[4], tp[5]);
#endif
  if (!ok) return;
  // ---- certify: every equality row held, every one-sided row feasible ----
  const double xs = wmax(lane < NX ? fabs(xi) : 0.0);
  double bad = 0.0;
  if (lane < neq) {
    double s = -sEb[lane], cm = 0.0;
    for (int i = 0; i < NX; ++i) {
      s = fma(sE[lane * NXP + i], sx[i], s);
      cm = fmax(cm, fabs(sE[lane * NXP + i]));
    }
    bad = fabs(s) / (1.0 + cm * xs + fabs(sEb[lane])) <= 1e-8 ? 0.0 : 1.0;   // (NaN: bad)
  }
  if (lane < NX && !isfinite(xi)) bad = 1.0;
  if (in_valid(lane) &&
      !(in_slack(lane) / (1.0 + in_scale(lane) * xs + fabs(in_rhs(lane))) >= -1e-9))
    bad = 1.0;
  if (!(wmax(bad) == 0.0) || !isfinite(xs)) return;
  if (gx != nullptr && lane < NX) gx[static_cast<size_t>(env) * NX + lane] = xi;
  if (lane >= NV && lane < NV + NU) gtau[static_cast<size_t>(env) * NU + lane - NV] = xi;
  if (lane == 0) gstatus[env] = OSC_SOLVE_OK;
}

using Go2 = Dims<18, 12, 4, 5>;   // unitree_go2: nv 18, nu 12, 4 feet, 5 sites
using Walter = Dims<14, 8, 8, 17>;   // walter_sr(_wheels): nv 14, nu 8, 8 wheels, 17 sites
using WalterW = Dims<14, 8, 8, 17, true>;   // + the wheel no-slip rows (opt-in)

enum KernelId { K_NONE = 0, K_GO2 = 1, K_WALTER = 2, K_WALTER_WHEELS = 3 };

KernelId select_kernel(const osc_model_desc& d) {
  const bool wheels = d.wheel_rows != 0;
  if (d.nv == Go2::NV && d.nu == Go2::NU && d.nc == Go2::NC && d.ns == Go2::NS)
    return wheels ? K_NONE : K_GO2;
  if (d.nv == Walter::NV && d.nu == Walter::NU && d.nc == Walter::NC && d.ns == Walter::NS)
    return wheels ? K_WALTER_WHEELS : K_WALTER;
  return K_NONE;
}

int ww_doubles(KernelId k) {
  switch (k) {
    case K_GO2: return Go2::WW;
    case K_WALTER: return Walter::WW;
    case K_WALTER_WHEELS: return WalterW::WW;
    default: return 0;
  }
}

int ws_doubles(KernelId k) {
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
int park_iter_default(KernelId k) { return k == K_WALTER ? 16 : 0; }
constexpr int kParkMinRounds = 4;   // batches of at least this many resident-wave rounds

int park_doubles_of(KernelId k) {
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
WsLayout ws_layout(KernelId k, int32_t nenv) {
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

int dual_rows(KernelId k) {
  switch (k) {
    case K_GO2: return Go2::NV + 4 * Go2::NC + Go2::NX;
    case K_WALTER: return Walter::NV + 4 * Walter::NC + Walter::NX;
    case K_WALTER_WHEELS: return WalterW::NV + WalterW::NW + 4 * WalterW::NC + WalterW::NX;
    default: return 0;
  }
}

}  // namespace

struct osc_model {
  osc_model_desc desc;
  KernelId kid;
  DevParams* dparams;
  int device;
  int small_batch_max;   // envs that fit one wavefront per SIMD (4 per wave x 4 SIMDs x CUs)
  bool refine;           // torque-coordinate model with refinement steps > 0
  int resident_envs;     // envs of one wavefront per SIMD over the whole device
  int park_it;           // compaction's park iteration (0: off; ParkArgs)
};

namespace {
// Model defaults of the knobs in osc_model_tuning.
void tuning_defaults(const osc_model_desc& d, osc_model_tuning& t) {
  std::memset(&t, 0, sizeof(t));
  // full-space refinement: at least two steps per round with one factorisation,
  // each env until its own step converges (numpy model: <= 3e-12 normwise on Go2 / WaLTER
  // batches, from up to 2e-2 without it); wheel rows: twelve, run to convergence (the rows'
  // multipliers, exported as duals, converge more slowly than y)
  t.refine_steps = d.wheel_rows ? 12 : 2;
  t.refine_max_move = 1e300;
  t.eps_mu = d.eps_mu;
  // warm start (round 3, profiles/r03_warm_settings.txt: delta 0.1 -> 1 and
  // centring 0.3 -> 1 cut the slowest warm envs' tail -- Go2 4,096 24.1 -> 27.2 M, WaLTER 4,096
  // 14.0 -> 20.0 M, WaLTER tumbling 8,192 20.0 -> 22.5 M solves/s -- for +0.8 / +1.1 mean
  // iterations: Go2 65,536 52.4 -> 51.6 M)
  t.warm_delta = 1.0;
  t.warm_center = 1.0;
  t.warm_restart = 22;
  t.restart_iter = 28;
  // wheel no-slip rows: pinned coordinates of the interior point's Newton
  // systems, so every step leaves them holding to rounding; the stop test asks 1e-6
  t.wheel_tol = 1e-6;
  t.small_batch_max = -1;
  t.park_it = -1;
}

#ifdef OSC_TUNING_ENV
// Diagnostic builds only (tools/*.sh sweeps): the OSC_* variables override the tuning block.  A
// release library reads no environment variable.
void tuning_from_env(osc_model_tuning& t) {
  if (const char* e = std::getenv("OSC_REFINE_STEPS")) t.refine_steps = std::atoi(e);
  if (const char* e = std::getenv("OSC_EPS_MU")) t.eps_mu = std::atof(e);
  if (const char* e = std::getenv("OSC_RESTART_ITER")) t.restart_iter = std::atoi(e);
  if (const char* e = std::getenv("OSC_WARM_RESTART")) t.warm_restart = std::atoi(e);
  if (const char* e = std::getenv("OSC_WARM_DELTA")) t.warm_delta = std::atof(e);
  if (const char* e = std::getenv("OSC_WARM_CENTER")) t.warm_center = std::atof(e);
  if (const char* e = std::getenv("OSC_REFINE_MAX_MOVE")) t.refine_max_move = std::atof(e);
  if (const char* e = std::getenv("OSC_WHEEL_TOL")) t.wheel_tol = std::atof(e);
  if (const char* e = std::getenv("OSC_SMALL_BATCH_MAX")) t.small_batch_max = std::atoi(e);
  if (const char* e = std::getenv("OSC_PARK_IT")) t.park_it = std::atoi(e);
}
#endif
}  // namespace

extern "C" int osc_model_tuning_defaults(const osc_model_desc* desc, osc_model_tuning* tuning) {
  if (!desc || !tuning) return OSC_ERR_INVALID_ARGUMENT;
  tuning_defaults(*desc, *tuning);
  return OSC_OK;
}

extern "C" int osc_model_create(const osc_model_desc* desc, osc_model** out) {
  return osc_model_create_tuned(desc, nullptr, out);
}

extern "C" int osc_model_create_tuned(const osc_model_desc* desc, const osc_model_tuning* tuning,
                                      osc_model** out) {
  if (!desc || !out) return OSC_ERR_INVALID_ARGUMENT;
  *out = nullptr;
  const osc_model_desc& d = *desc;
  if (d.nv <= 0 || d.nu <= 0 || d.nu > OSC_MAX_NU || d.nu >= d.nv || d.nc < 0 || d.ns <= 0 ||
      d.ns > OSC_MAX_SITES || d.nc > d.ns || d.max_iter < 0 || !(d.infinity > 0.0))
    return OSC_ERR_INVALID_ARGUMENT;
  const double thresh = d.infinity * 1e-10;
  // fx, fy carry no finite bounds in the reference (osc.h:297-308); the kernel has no rows
  // for them.
  for (int c = 0; c < 2; ++c)
    if (std::fabs(d.z_lb[c]) < thresh || std::fabs(d.z_ub[c]) < thresh)
      return OSC_ERR_INVALID_ARGUMENT;
  for (int i = 0; i < d.nu; ++i)
    if (!(d.u_lb[i] <= d.u_ub[i])) return OSC_ERR_INVALID_ARGUMENT;
  if (d.wheel_rows != 0 && d.wheel_rows != 1) return OSC_ERR_INVALID_ARGUMENT;
  for (int i = 0; d.wheel_rows && i < d.nc; ++i)
    if (d.wheel_dof[i] < -1 || d.wheel_dof[i] >= d.nv || !std::isfinite(d.wheel_radius[i]))
      return OSC_ERR_INVALID_ARGUMENT;
  const KernelId kid = select_kernel(d);
  if (kid == K_NONE) return OSC_ERR_UNSUPPORTED_DIMS;

  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return OSC_ERR_NO_DEVICE;
  DevParams hp;
  std::memset(&hp, 0, sizeof(hp));
  for (int i = 0; i < d.ns; ++i) {
    for (int t = 0; t < 3; ++t) {
      hp.w_row[3 * i + t] = d.w_pos[i];
      hp.w_row[3 * d.ns + 3 * i + t] = d.w_rot[i];
    }
  }
  for (int r = 0; r < 6 * d.ns; ++r) hp.w_sqrt[r] = std::sqrt(hp.w_row[r]);
  for (int i = 0; i < d.nu; ++i) {
    hp.u_lb[i] = d.u_lb[i];
    hp.u_ub[i] = d.u_ub[i];
  }
  for (int c = 0; c < 3; ++c) {
    hp.z_lb[c] = d.z_lb[c];
    hp.z_ub[c] = d.z_ub[c];
  }
  hp.mu = d.mu;
  hp.w_torque = d.w_torque;
  hp.w_reg = d.w_reg;
  osc_model_tuning t;
  if (tuning) {
    t = *tuning;
  } else {
    tuning_defaults(d, t);
#ifdef OSC_TUNING_ENV
    tuning_from_env(t);
#endif
  }
  if (t.refine_steps < 0 || t.restart_iter < 0 || t.warm_restart < 0 || !(t.eps_mu > 0.0) ||
      !(t.refine_max_move >= 0.0) || !(t.wheel_tol > 0.0) || !(t.warm_delta > 0.0) ||
      !(t.warm_center >= 0.0) || t.park_it < -1 || t.small_batch_max < -1)
    return OSC_ERR_INVALID_ARGUMENT;
  hp.eps_mu = t.eps_mu;
  hp.inf_thresh = thresh;
  hp.max_iter = d.max_iter;
  hp.warm_delta = t.warm_delta;
  hp.warm_center = t.warm_center;
  hp.warm_restart = t.warm_restart;
  hp.restart_iter = t.restart_iter;
  hp.refine_steps = t.refine_steps;
  hp.refine_penalty = 1e2;   // active-row penalty of the refinement, x max diag(Hr)
  hp.refine_max_move = t.refine_max_move;
  // The early stops (Go2 1e-6, WaLTER 1e-8: osc_desc_from_yaml) presume the refinement finishes
  // the solve; without it the interior point runs to 1e-12 itself.
  if (hp.refine_steps <= 0) hp.eps_mu = std::fmin(hp.eps_mu, 1e-12);
  for (int i = 0; i < OSC_MAX_SITES; ++i) hp.wheel_dof[i] = -1;
  for (int i = 0; d.wheel_rows && i < d.nc; ++i) {
    hp.wheel_dof[i] = d.wheel_dof[i];
    hp.wheel_radius[i] = d.wheel_radius[i];
  }
  hp.wheel_tol = t.wheel_tol;

  osc_model* m = new (std::nothrow) osc_model;
  if (!m) return OSC_ERR_DEVICE;
  m->desc = d;
  m->kid = kid;
  m->dparams = nullptr;
  m->refine = hp.refine_steps > 0;
  (void)hipGetDevice(&m->device);
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, m->device) != hipSuccess)
    cus = 0;
  // One-wave-per-SIMD variant up to the batch that fills every SIMD once; beyond it the
  // two-waves variant, except for the 32-column WaLTER system, whose Newton matrix does not fit
  // two waves' register budget (scratch spills): it always runs one wave per SIMD with AGPR
  // spill space (MI355X, 32,768 envs: 2.61 vs 2.95 ms; round-2 variant sweep).
  m->small_batch_max = (kid == K_GO2) ? kEnvPerWave * 4 * cus : INT32_MAX;
  if (t.small_batch_max >= 0) m->small_batch_max = t.small_batch_max;
  if (kid == K_WALTER_WHEELS) m->small_batch_max = INT32_MAX;   // (one-wave kernel only)
  // Lockstep compaction past one resident wavefront per SIMD (ParkArgs; 0 = off)
  m->resident_envs = kEnvPerWave * 4 * cus;
  m->park_it = t.park_it >= 0 ? t.park_it : park_iter_default(kid);
  if (kid == K_WALTER_WHEELS || m->park_it >= hp.restart_iter) m->park_it = 0;
  if (hipMalloc(&m->dparams, sizeof(DevParams)) != hipSuccess ||
      hipMemcpy(m->dparams, &hp, sizeof(DevParams), hipMemcpyHostToDevice) != hipSuccess) {
    if (m->dparams) (void)hipFree(m->dparams);
    delete m;
    return OSC_ERR_DEVICE;
  }
  *out = m;
  return OSC_OK;
}

extern "C" int osc_model_create_from_yaml(const char* robot, const char* yaml_path, osc_model** out) {
  osc_model_desc d;
  int rc = osc_desc_from_yaml(robot, yaml_path, &d);
  if (rc != OSC_OK) return rc;
  return osc_model_create(&d, out);
}

extern "C" int osc_model_destroy(osc_model* model) {
  if (!model) return OSC_ERR_INVALID_ARGUMENT;
  if (model->dparams) (void)hipFree(model->dparams);
  delete model;
  return OSC_OK;
}

extern "C" int osc_model_get_desc(const osc_model* model, osc_model_desc* desc) {
  if (!model || !desc) return OSC_ERR_INVALID_ARGUMENT;
  *desc = model->desc;
  return OSC_OK;
}

extern "C" int osc_workspace_bytes(const osc_model* model, int32_t nenv, size_t* bytes) {
  if (!model || !bytes || nenv < 0) return OSC_ERR_INVALID_ARGUMENT;
  // per-env reduced QPs, then int32 solve-status scratch for the warm fix-up pass (16-B padded),
  // then the compaction's park area, slot list and counter (ParkArgs)
  *bytes = ws_layout(model->kid, nenv).total;
  return OSC_OK;
}

extern "C" int osc_workspace_env_bytes(const osc_model* model, size_t* bytes) {
  if (!model || !bytes) return OSC_ERR_INVALID_ARGUMENT;
  *bytes = sizeof(double) * static_cast<size_t>(ws_doubles(model->kid));
  return OSC_OK;
}

namespace {

enum Stage : unsigned { kAssemble = 1u, kInteriorPoint = 2u, kBoth = 3u };

template <class D>
void launch_t(const osc_model* model, int32_t nenv, const double* M, const double* C,
              const double* J, const double* b, const double* T, const double* mask, double* tau,
              double* x, int32_t* status, int32_t* iters, double* ws, double* warm, hipStream_t s,
              unsigned stages, const double* wdir, double* y) {
  if (stages & kAssemble) {
    // one env per 64-lane wavefront (four envs per wavefront measured no faster: Go2 4,096
    // 35.3 vs 33.7 us)
    hipLaunchKernelGGL(osc_setup_kernel<D>, dim3(static_cast<unsigned>(nenv)), dim3(kWave), 0, s,
                       model->dparams, nenv, M, C, J, b, T, mask, ws, wdir);
  }
  if (!(stages & kInteriorPoint)) return;
  // All wavefronts resident at once (<= one per SIMD): the latency-optimised variant (one wave
  // per SIMD, Hr in LDS where it fits); otherwise the two-waves-per-SIMD variant.
  const unsigned nb = static_cast<unsigned>((nenv + kEnvPerWave - 1) / kEnvPerWave);
  const int flags = y != nullptr ? 2 : 0;   // hand the multipliers to the dual kernel
  if constexpr (D::WH) {
    // wheel rows: the one-wave solve with the refinement fused (launch() checked the rest); warm-
    // started: the warm pass, then the cold fix-up pass over the wavefronts holding an env the
    // warm start left unconverged (the per-env status: the caller's array, else scratch)
    // The fused entries (raw inputs at hand) then run the active-set fallback over the envs the
    // interior point left unconverged (osc_gi_kernel); it needs the per-env status too.
    const bool fallback = M && C && J && b && wdir;
    if (status == nullptr && (warm != nullptr || fallback))
      status = reinterpret_cast<int32_t*>(ws + static_cast<size_t>(D::WS) * nenv);
    if (warm == nullptr) {
      hipLaunchKernelGGL((osc_ipm_kernel<D, true, false, kRfFused>), dim3(nb), dim3(kWave), 0, s,
                         model->dparams, nenv, mask, ws, tau, x, status, iters, nullptr, flags);
    } else {
      for (int pass = 0; pass < 2; ++pass)
        hipLaunchKernelGGL((osc_ipm_kernel<D, true, true, kRfFused>), dim3(nb), dim3(kWave), 0, s,
                           model->dparams, nenv, mask, ws, tau, x, status, iters, warm,
                           flags | pass);
    }
    if (fallback)
      hipLaunchKernelGGL(osc_gi_kernel<D>, dim3(static_cast<unsigned>(nenv)), dim3(kWave), 0, s,
                         model->dparams, nenv, M, C, J, b, mask, wdir, ws, tau, x, status);
  } else {
    // A warm-started solve is followed by a cold fix-up pass over the wavefronts that hold an
    // env the warm start did not bring to convergence (it needs the per-env status: the
    // caller's array, else scratch at the end of the workspace).
    if (warm != nullptr && status == nullptr)
      status = reinterpret_cast<int32_t*>(ws + static_cast<size_t>(D::WS) * nenv);
    const bool small = nenv <= model->small_batch_max;
    // Every cold solve runs the refinement in the same wavefront (kRfFused), and so does the
    // one-wave warm solve; warm past one wave per SIMD the fused two-wave kernel spills (Go2
    // 65,536 warm 50.0 -> 44.5 M solves/s), so that case keeps the separate refinement pass.
    const bool fused = warm == nullptr && model->refine;
    const bool fused_warm = small && warm != nullptr && model->refine;
    // Lockstep compaction: more wavefronts than SIMDs, so the SIMD time the lockstep tail costs
    // is time other wavefronts could use (ParkArgs; bitwise the single pass's results)
    // (from four rounds of wavefronts per SIMD: at two, WaLTER configs[3] -- 8,192 tumbling envs,
    // masks redrawn -- is 4 % slower with it, 17.0 vs 17.7 M solves/s; at eight, 32,768, 3 %
    // faster: profiles/r03ze_*)
    const bool compact = fused && !D::WH && model->park_it > 0 &&
                         nenv >= kParkMinRounds * model->resident_envs &&
                         static_cast<size_t>(nenv) * D::WS < (size_t{1} << 32);
    if (warm == nullptr && compact) {
      const WsLayout wl = ws_layout(model->kid, nenv);
      char* base = reinterpret_cast<char*>(ws);
      ParkArgs pa;
      pa.park = reinterpret_cast<double*>(base + wl.park);
      pa.list = reinterpret_cast<int32_t*>(base + wl.list);
      pa.count = reinterpret_cast<int32_t*>(base + wl.count);
      pa.park_it = model->park_it;
      (void)hipMemsetAsync(pa.count, 0, sizeof(int32_t), s);
      if (small) {
        hipLaunchKernelGGL((osc_ipm_compact_kernel<D, true, kCpPark>), dim3(nb), dim3(kWave), 0, s,
                           model->dparams, nenv, mask, ws, tau, x, status, iters, flags, pa);
        hipLaunchKernelGGL((osc_ipm_compact_kernel<D, true, kCpResume>), dim3(nb), dim3(kWave), 0,
                           s, model->dparams, nenv, mask, ws, tau, x, status, iters, flags, pa);
      } else {
        hipLaunchKernelGGL((osc_ipm_compact_kernel<D, false, kCpPark>), dim3(nb), dim3(kWave), 0, s,
                           model->dparams, nenv, mask, ws, tau, x, status, iters, flags, pa);
        hipLaunchKernelGGL((osc_ipm_compact_kernel<D, false, kCpResume>), dim3(nb), dim3(kWave), 0,
                           s, model->dparams, nenv, mask, ws, tau, x, status, iters, flags, pa);
      }
    } else if (warm == nullptr) {
      if (fused && small)
        hipLaunchKernelGGL((osc_ipm_kernel<D, true, false, kRfFused>), dim3(nb), dim3(kWave), 0, s,
                           model->dparams, nenv, mask, ws, tau, x, status, iters, nullptr, flags);
      else if (fused)
        hipLaunchKernelGGL((osc_ipm_kernel<D, false, false, kRfFused>), dim3(nb), dim3(kWave), 0, s,
                           model->dparams, nenv, mask, ws, tau, x, status, iters, nullptr, flags);
      else if (small)
        hipLaunchKernelGGL((osc_ipm_kernel<D, true, false>), dim3(nb), dim3(kWave), 0, s,
                           model->dparams, nenv, mask, ws, tau, x, status, iters, nullptr, flags);
      else
        hipLaunchKernelGGL((osc_ipm_kernel<D, false, false>), dim3(nb), dim3(kWave), 0, s,
                           model->dparams, nenv, mask, ws, tau, x, status, iters, nullptr, flags);
    } else if (fused_warm) {
      // warm-started: the refinement runs in the same wavefront too, in pass 0 for the envs the
      // warm start converged and in the cold fix-up pass for the ones it redoes
      for (int pass = 0; pass < 2; ++pass) {
        hipLaunchKernelGGL((osc_ipm_kernel<D, true, true, kRfFused>), dim3(nb), dim3(kWave), 0, s,
                           model->dparams, nenv, mask, ws, tau, x, status, iters, warm, pass);
      }
    } else {
      for (int pass = 0; pass < 2; ++pass) {
        if (small)
          hipLaunchKernelGGL((osc_ipm_kernel<D, true, true>), dim3(nb), dim3(kWave), 0, s,
                             model->dparams, nenv, mask, ws, tau, x, status, iters, warm, pass);
        else
          hipLaunchKernelGGL((osc_ipm_kernel<D, false, true>), dim3(nb), dim3(kWave), 0, s,
                             model->dparams, nenv, mask, ws, tau, x, status, iters, warm, pass);
      }
    }
    if (model->refine && !fused && !fused_warm)   // (warm, past one wave per SIMD)
      hipLaunchKernelGGL((osc_refine_kernel<D, false>), dim3(nb), dim3(kWave), 0, s,
                         model->dparams, nenv, mask, ws, tau, x, status);
  }
  if (y != nullptr)
    hipLaunchKernelGGL(osc_dual_kernel<D>, dim3(static_cast<unsigned>(nenv)), dim3(kWave), 0, s,
                       model->dparams, nenv, M, J, mask, wdir, ws, x, y);
}

bool misaligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) != 0; }

// A model's kernels read its parameters from the device it was created on: launches go there.
bool on_model_device(const osc_model* model) {
  int cur = -1;
  return hipGetDevice(&cur) == hipSuccess && cur == model->device;
}

int launch(const osc_model* model, int32_t nenv, const double* M, const double* C, const double* J,
           const double* b, const double* T, const double* contact_mask, double* tau, double* x,
           int32_t* status, int32_t* iters, void* workspace, size_t workspace_bytes,
           void* stream, unsigned stages, double* warm = nullptr, const double* wdir = nullptr,
           double* y = nullptr) {
  if (!model || nenv < 0) return OSC_ERR_INVALID_ARGUMENT;
  if (nenv == 0) return OSC_OK;
  if (!on_model_device(model)) return OSC_ERR_INVALID_ARGUMENT;
  if (!contact_mask || misaligned16(contact_mask)) return OSC_ERR_INVALID_ARGUMENT;
  if ((stages & kAssemble) && (!M || !C || !J || !b || !T || misaligned16(M) ||
                               misaligned16(C) || misaligned16(J) || misaligned16(b) ||
                               misaligned16(T)))
    return OSC_ERR_INVALID_ARGUMENT;   // 16-byte alignment: vectorised staging loads
  if ((stages & kInteriorPoint) && !tau) return OSC_ERR_INVALID_ARGUMENT;
  const bool wheels = model->kid == K_WALTER_WHEELS;
  if (wheels && (stages & kAssemble) && wdir == nullptr) return OSC_ERR_INVALID_ARGUMENT;
  if (y != nullptr && (x == nullptr || (stages & kBoth) != kBoth)) return OSC_ERR_INVALID_ARGUMENT;
  if (y != nullptr && !model->refine) return OSC_ERR_INVALID_ARGUMENT;   // (fused path only)
  // A split call hands the reduced QP over in the caller's workspace; only the fused call may
  // take scratch of its own.
  if (stages != kBoth && !workspace) return OSC_ERR_INVALID_ARGUMENT;
  if (misaligned16(workspace)) return OSC_ERR_INVALID_ARGUMENT;
  size_t need = 0;
  osc_workspace_bytes(model, nenv, &need);
  hipStream_t s = static_cast<hipStream_t>(stream);
  double* ws = static_cast<double*>(workspace);
  bool owned = false;
  if (ws == nullptr) {   // convenience path: stream-ordered scratch
    if (hipMallocAsync(reinterpret_cast<void**>(&ws), need, s) != hipSuccess) return OSC_ERR_DEVICE;
    owned = true;
  } else if (workspace_bytes < need) {
    return OSC_ERR_INVALID_ARGUMENT;
  }
  int rc = OSC_OK;
  switch (model->kid) {
    case K_GO2:
      launch_t<Go2>(model, nenv, M, C, J, b, T, contact_mask, tau, x, status, iters, ws, warm, s,
                    stages, nullptr, y);
      break;
    case K_WALTER:
      launch_t<Walter>(model, nenv, M, C, J, b, T, contact_mask, tau, x, status, iters, ws, warm, s,
                       stages, nullptr, y);
      break;
    case K_WALTER_WHEELS:
      launch_t<WalterW>(model, nenv, M, C, J, b, T, contact_mask, tau, x, status, iters, ws, warm,
                        s, stages, wdir, y);
      break;
    default:
      rc = OSC_ERR_UNSUPPORTED_DIMS;
  }
  if (rc == OSC_OK && hipGetLastError() != hipSuccess) rc = OSC_ERR_DEVICE;
  if (owned) (void)hipFreeAsync(ws, s);
  return rc;
}

}  // namespace

extern "C" int osc_batch_solve(const osc_model* model, int32_t nenv, const double* M,
                               const double* C, const double* J, const double* b, const double* T,
                               const double* contact_mask, double* tau, double* x,
                               int32_t* status, int32_t* iters, void* workspace,
                               size_t workspace_bytes, void* stream) {
  return launch(model, nenv, M, C, J, b, T, contact_mask, tau, x, status, iters, workspace,
                workspace_bytes, stream, kBoth);
}

extern "C" int osc_dual_rows(const osc_model* model, int32_t* rows) {
  if (!model || !rows) return OSC_ERR_INVALID_ARGUMENT;
  *rows = dual_rows(model->kid);
  return OSC_OK;
}

extern "C" int osc_batch_solve_ex(const osc_model* model, int32_t nenv, const double* M,
                                  const double* C, const double* J, const double* b,
                                  const double* T, const double* contact_mask,
                                  const osc_solve_extras* extras, double* tau, double* x,
                                  int32_t* status, int32_t* iters, void* workspace,
                                  size_t workspace_bytes, void* stream) {
  const double* wdir = extras ? extras->wheel_dir : nullptr;
  if (wdir && misaligned16(wdir)) return OSC_ERR_INVALID_ARGUMENT;
  return launch(model, nenv, M, C, J, b, T, contact_mask, tau, x, status, iters, workspace,
                workspace_bytes, stream, kBoth, nullptr, wdir, extras ? extras->y : nullptr);
}

extern "C" int osc_batch_assemble_ex(const osc_model* model, int32_t nenv, const double* M,
                                     const double* C, const double* J, const double* b,
                                     const double* T, const double* contact_mask,
                                     const double* wheel_dir, void* workspace,
                                     size_t workspace_bytes, void* stream) {
  return launch(model, nenv, M, C, J, b, T, contact_mask, nullptr, nullptr, nullptr, nullptr,
                workspace, workspace_bytes, stream, kAssemble, nullptr, wheel_dir);
}

extern "C" int osc_batch_assemble(const osc_model* model, int32_t nenv, const double* M,
                                  const double* C, const double* J, const double* b,
                                  const double* T, const double* contact_mask, void* workspace,
                                  size_t workspace_bytes, void* stream) {
  return launch(model, nenv, M, C, J, b, T, contact_mask, nullptr, nullptr, nullptr, nullptr,
                workspace, workspace_bytes, stream, kAssemble);
}

namespace {

template <class DA, class DB>
void launch_pair(const osc_batch_job& a, const osc_batch_job& b, hipStream_t s) {
  auto args = [](const osc_batch_job& j) {
    PairArgs p;
    p.P = j.model->dparams;
    p.nenv = j.nenv;
    p.M = j.M; p.C = j.C; p.J = j.J; p.b = j.b; p.T = j.T; p.mask = j.contact_mask;
    p.ws = static_cast<double*>(j.workspace);
    p.tau = j.tau; p.x = j.x; p.status = j.status; p.iters = j.iters;
    return p;
  };
  const PairArgs A = args(a), B = args(b);
  hipLaunchKernelGGL((osc_setup_pair_kernel<DA, DB>),
                     dim3(static_cast<unsigned>(a.nenv + b.nenv)), dim3(kWave), 0, s, A, B);
  const unsigned nb = static_cast<unsigned>((a.nenv + kEnvPerWave - 1) / kEnvPerWave +
                                            (b.nenv + kEnvPerWave - 1) / kEnvPerWave);
  // one-wave interior point of both models with the refinement in the same wavefront
  if (a.model->refine || b.model->refine)
    hipLaunchKernelGGL((osc_ipm_pair_kernel<DA, DB, kRfFused>), dim3(nb), dim3(kWave), 0, s, A, B);
  else
    hipLaunchKernelGGL((osc_ipm_pair_kernel<DA, DB>), dim3(nb), dim3(kWave), 0, s, A, B);
}

}  // namespace

extern "C" int osc_batch_solve_multi(const osc_batch_job* jobs, int32_t njobs, void* stream) {
  if (njobs < 0 || (njobs > 0 && !jobs)) return OSC_ERR_INVALID_ARGUMENT;
  for (int i = 0; i < njobs; ++i) {   // every job checked before anything is launched
    const osc_batch_job& j = jobs[i];
    if (!j.model || j.nenv < 0) return OSC_ERR_INVALID_ARGUMENT;
    if (j.nenv == 0) continue;
    if (!j.workspace || !j.contact_mask || !j.tau) return OSC_ERR_INVALID_ARGUMENT;
    size_t need = 0;
    osc_workspace_bytes(j.model, j.nenv, &need);
    if (j.workspace_bytes < need || misaligned16(j.workspace) || misaligned16(j.contact_mask) ||
        !j.M || !j.C || !j.J || !j.b || !j.T || misaligned16(j.M) || misaligned16(j.C) ||
        misaligned16(j.J) || misaligned16(j.b) || misaligned16(j.T))
      return OSC_ERR_INVALID_ARGUMENT;
    if (j.model->kid == K_NONE || j.model->kid == K_WALTER_WHEELS) return OSC_ERR_UNSUPPORTED_DIMS;
    if (!on_model_device(j.model)) return OSC_ERR_INVALID_ARGUMENT;   // one device per call
  }
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (njobs == 2 && jobs[0].nenv > 0 && jobs[1].nenv > 0 && jobs[0].model->kid != jobs[1].model->kid &&
      jobs[0].nenv <= jobs[0].model->small_batch_max && jobs[1].nenv <= jobs[1].model->small_batch_max) {
    const bool a_walter = jobs[0].model->kid == K_WALTER;
    const osc_batch_job& w = a_walter ? jobs[0] : jobs[1];   // slower per wavefront: first
    const osc_batch_job& g = a_walter ? jobs[1] : jobs[0];
    launch_pair<Walter, Go2>(w, g, s);
    return hipGetLastError() == hipSuccess ? OSC_OK : OSC_ERR_DEVICE;
  }
  for (int i = 0; i < njobs; ++i) {
    const osc_batch_job& j = jobs[i];
    const int rc = launch(j.model, j.nenv, j.M, j.C, j.J, j.b, j.T, j.contact_mask, j.tau, j.x,
                          j.status, j.iters, j.workspace, j.workspace_bytes, stream, kBoth);
    if (rc != OSC_OK) return rc;
  }
  return OSC_OK;
}

extern "C" int osc_warm_state_bytes(const osc_model* model, int32_t nenv, size_t* bytes) {
  if (!model || !bytes || nenv < 0) return OSC_ERR_INVALID_ARGUMENT;
  *bytes = sizeof(double) * static_cast<size_t>(ww_doubles(model->kid)) * static_cast<size_t>(nenv);
  return OSC_OK;
}

namespace {
// true when the warm-state buffer is usable: non-null and at least osc_warm_state_bytes
bool warm_small(const osc_model* model, int32_t nenv, const double* warm, size_t bytes) {
  size_t need = 0;
  if (!model || !warm || osc_warm_state_bytes(model, nenv < 0 ? 0 : nenv, &need) != OSC_OK)
    return false;
  return bytes >= need;
}
}  // namespace

extern "C" int osc_batch_solve_warm(const osc_model* model, int32_t nenv, const double* M,
                                    const double* C, const double* J, const double* b,
                                    const double* T, const double* contact_mask, double* tau,
                                    double* x, int32_t* status, int32_t* iters, double* warm_state,
                                    size_t warm_state_bytes, void* workspace,
                                    size_t workspace_bytes, void* stream) {
  if (!warm_small(model, nenv, warm_state, warm_state_bytes)) return OSC_ERR_INVALID_ARGUMENT;
  return launch(model, nenv, M, C, J, b, T, contact_mask, tau, x, status, iters, workspace,
                workspace_bytes, stream, kBoth, warm_state);
}

extern "C" int osc_batch_solve_warm_ex(const osc_model* model, int32_t nenv, const double* M,
                                       const double* C, const double* J, const double* b,
                                       const double* T, const double* contact_mask,
                                       const osc_solve_extras* extras, double* tau, double* x,
                                       int32_t* status, int32_t* iters, double* warm_state,
                                       size_t warm_state_bytes, void* workspace,
                                       size_t workspace_bytes, void* stream) {
  if (!warm_small(model, nenv, warm_state, warm_state_bytes)) return OSC_ERR_INVALID_ARGUMENT;
  const double* wdir = extras ? extras->wheel_dir : nullptr;
  if (wdir && misaligned16(wdir)) return OSC_ERR_INVALID_ARGUMENT;
  return launch(model, nenv, M, C, J, b, T, contact_mask, tau, x, status, iters, workspace,
                workspace_bytes, stream, kBoth, warm_state, wdir, extras ? extras->y : nullptr);
}

extern "C" int osc_batch_solve_assembled_warm(const osc_model* model, int32_t nenv,
                                              const double* contact_mask, double* tau, double* x,
                                              int32_t* status, int32_t* iters, double* warm_state,
                                              size_t warm_state_bytes, void* workspace,
                                              size_t workspace_bytes, void* stream) {
  if (!warm_small(model, nenv, warm_state, warm_state_bytes)) return OSC_ERR_INVALID_ARGUMENT;
  return launch(model, nenv, nullptr, nullptr, nullptr, nullptr, nullptr, contact_mask, tau, x,
                status, iters, workspace, workspace_bytes, stream,
                kInteriorPoint, warm_state);
}

extern "C" int osc_batch_solve_assembled(const osc_model* model, int32_t nenv,
                                         const double* contact_mask, double* tau, double* x,
                                         int32_t* status, int32_t* iters, void* workspace,
                                         size_t workspace_bytes, void* stream) {
  return launch(model, nenv, nullptr, nullptr, nullptr, nullptr, nullptr, contact_mask, tau, x,
                status, iters, workspace, workspace_bytes, stream,
                kInteriorPoint);
}

#ifdef OSC_STAMPS
// Diagnostic build only: per-block IPM phase cycles [nblocks][8] (see STAMP_* above).
extern "C" int osc_debug_stamps(unsigned long long* host, int nblocks) {
  if (nblocks > kStampBlocks) nblocks = kStampBlocks;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * kStampSlots *
                             nblocks) == hipSuccess ? OSC_OK : OSC_ERR_DEVICE;
}
// Same for the setup kernel (one block per env): [nblocks][kStampSlots], slots 0-5 used.
extern "C" int osc_debug_setup_stamps(unsigned long long* host, int nblocks) {
  if (nblocks > kStampBlocks) nblocks = kStampBlocks;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_setup_stamps), sizeof(unsigned long long) *
                             kStampSlots * nblocks) == hipSuccess ? OSC_OK : OSC_ERR_DEVICE;
}
#endif
