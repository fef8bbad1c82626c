// osc_batch.hip -- batched OSC QP assembly + solve for gfx950 (MI355X), one wavefront per env.
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
// Method (see DESIGN.md §3 for the derivation and the accuracy study):
//   1. u is eliminated exactly from the actuated dynamics rows, and the base accelerations
//      dv_b from the 6 unactuated rows through the 6x6 base block M_bb only:
//         dv_b = M_bb^-1 (-M_ba dv_a + Jc_b z - C_b),   u = M_a dv + C_a - Jc_a z.
//      The remaining variables y = (dv_a, z) (nu + 3nc = 24 Go2 / 32 WaLTER) carry a dense
//      reduced Hessian Hr and gradient g.  Inverting only M_bb (never the full M) keeps the
//      regularisation-only curvature (2 w_reg = 2e-4, internal contact forces) resolvable in
//      fp64: torque error vs the exact optimum drops ~10x against the full-M^-1 reduction.
//   2. Mehrotra predictor-corrector interior point on  min 1/2 y'Hr y + g'y  s.t. G y <= h,
//      with G = [+-U (torque bounds, dense rows); pyramid + fz bound rows (sparse)].
//      Newton matrix K = Hr + G' diag(lambda/s) G factorised by LDL^T with "Cholesky-infinity"
//      pivots (a pivot below 1e-13 of its original diagonal is replaced by 1e128).
//
// Mapping onto CDNA4: one 64-lane wavefront = one environment = one workgroup.  Inputs are
// staged HBM -> LDS with 16-byte loads.  Dense products (J'WJ, the reduced Hessian) give every
// lane several output entries.  The Newton matrix lives in REGISTERS, one column per lane
// (lane j holds K[:, j]); the right-looking LDL^T broadcasts pivot column k with
// v_readlane, and both triangular solves run on lane-local data plus one broadcast per step
// (the symmetric trailing-matrix trick keeps row j of L in lane j's upper registers).
// Inequality rows map one per lane (48 Go2 / 64 WaLTER), so all interior-point vector work
// (residuals, ratio tests, complementarity) is lane-parallel with wavefront reductions.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstring>
#include <new>

#include "osc_batch.h"

namespace {

constexpr int kWave = 64;

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
  int32_t max_iter;
};

constexpr int cmax(int a, int b) { return a > b ? a : b; }
constexpr int even(int a) { return (a + 1) & ~1; }   // keep LDS regions 16-byte aligned

template <int NV_, int NU_, int NC_, int NS_>
struct Dims {
  static constexpr int NV = NV_, NU = NU_, NC = NC_, NS = NS_;
  static constexpr int NB = NV - NU;          // unactuated (floating-base) dofs
  static constexpr int NZ = 3 * NC;
  static constexpr int NY = NU + NZ;          // reduced variables (dv_a, z)
  static constexpr int NY1 = NY + 1;          // + affine column
  static constexpr int S = 6 * NS;            // task rows
  static constexpr int MI = 2 * NU + 6 * NC;  // inequality rows (u box, pyramid, fz box)
  static constexpr int NX = NV + NU + NZ;     // design vector
  static constexpr int NA = NV + 1;           // [J | e] Gram size
  static constexpr int NPA = NA * (NA + 1) / 2;
  static constexpr int NPH = NY1 * (NY1 + 1) / 2 - 1;   // reduced Hessian pairs (no corner)
  static_assert(NY1 <= kWave && MI <= kWave && NX <= kWave, "one row/column per lane");
  static_assert(NB >= 1 && NB <= 8, "floating-base block");

  // ---- LDS layout (doubles).  R1/R2 are reused between phases. ----
  static constexpr int R1_A = even(S * NV) + even(S) + even(NS * 6);   // J | e | T
  static constexpr int R1_D = even(NV * NY1) + even(NY * NY);           // T1 | Hr
  static constexpr int R1 = cmax(R1_A, R1_D);
  static constexpr int R2_A = even(NV * NV) + even(NV);                 // M | C
  static constexpr int R2_E = 4 * even(NY) + 3 * kWave + even(NU);      // IPM vectors
  static constexpr int R2 = cmax(R2_A, R2_E);
  static constexpr int O_J = 0, O_E = even(S * NV), O_T = O_E + even(S);
  static constexpr int O_T1 = 0, O_HR = even(NV * NY1);
  static constexpr int O_R2 = R1;
  static constexpr int O_M = O_R2, O_C = O_R2 + even(NV * NV);
  static constexpr int O_VY = O_R2, O_VY2 = O_VY + even(NY), O_DG = O_VY2 + even(NY),
                       O_G = O_DG + even(NY), O_VR = O_G + even(NY), O_DR = O_VR + kWave,
                       O_VR2 = O_DR + kWave, O_TAU = O_VR2 + kWave;   // row vectors: one per lane
  static constexpr int O_HA = O_R2 + R2;
  static constexpr int O_X = O_HA + even(NA * NA);
  static constexpr int O_U = O_X + even(NB * NY1);
  static constexpr int O_MASK = O_U + even(NU * NY1);
  static constexpr int SMEM = O_MASK + even(NC);
  static constexpr int DBG = NY * NY + NY + NU * NY1 + NB * NY1;   // debug dump per env
  static_assert(SMEM * 8 <= 64 * 1024, "LDS budget per env");
};

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

// ---- wavefront primitives -------------------------------------------------------------------
// An empty asm that "modifies" x: comparisons against the lane id made right after it cannot
// be hoisted out of loops (hipcc otherwise precomputes one 64-bit lane mask per unrolled step,
// hundreds of SGPRs, and spills them).
__device__ __forceinline__ int opaque(int x) {
  asm volatile("" : "+v"(x));
  return x;
}

__device__ __forceinline__ double bcast(double v, int k) {
  int lo = __builtin_amdgcn_readlane(__double2loint(v), k);
  int hi = __builtin_amdgcn_readlane(__double2hiint(v), k);
  return __hiloint2double(hi, lo);
}

// xor-butterfly inside each 32-lane half with ds_swizzle (bitmask mode), halves combined with
// two readlanes: the result is wave-uniform and bitwise identical on every lane.
template <int XOR>
__device__ __forceinline__ double swz_xor(double v) {
  constexpr int pat = (XOR << 10) | 0x1f;
  const int lo = __builtin_amdgcn_ds_swizzle(__double2loint(v), pat);
  const int hi = __builtin_amdgcn_ds_swizzle(__double2hiint(v), pat);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double wave_sum(double v) {
  v += swz_xor<1>(v);
  v += swz_xor<2>(v);
  v += swz_xor<4>(v);
  v += swz_xor<8>(v);
  v += swz_xor<16>(v);
  return bcast(v, 0) + bcast(v, 32);
}
__device__ __forceinline__ double wave_min(double v) {
  v = fmin(v, swz_xor<1>(v));
  v = fmin(v, swz_xor<2>(v));
  v = fmin(v, swz_xor<4>(v));
  v = fmin(v, swz_xor<8>(v));
  v = fmin(v, swz_xor<16>(v));
  return fmin(bcast(v, 0), bcast(v, 32));
}
__device__ __forceinline__ double wave_max(double v) {
  v = fmax(v, swz_xor<1>(v));
  v = fmax(v, swz_xor<2>(v));
  v = fmax(v, swz_xor<4>(v));
  v = fmax(v, swz_xor<8>(v));
  v = fmax(v, swz_xor<16>(v));
  return fmax(bcast(v, 0), bcast(v, 32));
}

// Copy n doubles (n even, both pointers 16-byte aligned) global -> LDS, 16 B per lane.
__device__ __forceinline__ void stage(double* dst, const double* __restrict__ src, int n, int lane) {
  const double2* s2 = reinterpret_cast<const double2*>(src);
  double2* d2 = reinterpret_cast<double2*>(dst);
  for (int i = lane; i < n / 2; i += kWave) d2[i] = s2[i];
}

// ---- register-resident LDL^T, one column per lane ------------------------------------------
// On entry lane j < N holds c[i] = K[i][j] (K symmetric).  On exit:
//   c[i], i > j : L[i][j]            (unit lower factor, column j)
//   c[i], i < j : L[j][i] * D[i]     (row j of L, scaled -- left by the symmetric update)
//   dinv        : 1 / D[j]
// `sdg` (LDS) holds the original diagonal (for the Cholesky-infinity test); `sdinv` (LDS)
// receives 1/D for the solves.
template <int N>
__device__ __forceinline__ void ldl_columns(double (&c)[N], double& dinv, const double* sdg,
                                            double* sdinv, int lane) {
  dinv = 0.0;
#pragma unroll
  for (int k = 0; k < N; ++k) {
    double dk = bcast(c[k], k);
    const double dg = sdg[k];
    if (!(dk > 1e-13 * dg)) dk = 1e128;   // Cholesky-infinity (Wright; PCx)
    const double inv = 1.0 / dk;
    const int ln = opaque(lane);
    if (ln == k) dinv = inv;
    const double t = (ln > k && ln < N) ? c[k] * inv : 0.0;   // L[lane][k]
#pragma unroll
    for (int i = k + 1; i < N; ++i) c[i] = fma(-bcast(c[i], k), t, c[i]);
  }
  // scale the column part (i > lane) into unit-lower L
#pragma unroll
  for (int i = 0; i < N; ++i) c[i] = (i > opaque(lane)) ? c[i] * dinv : c[i];
  if (lane < N) sdinv[lane] = dinv;
  __syncthreads();
}

// Solve K x = r with the factor above.  Lane j holds r_j on entry, x_j on exit.
template <int N>
__device__ __forceinline__ double ldl_solve(const double (&c)[N], double dinv, const double* sdinv,
                                            double r, int lane) {
  double acc = r;
#pragma unroll
  for (int k = 0; k < N; ++k) {          // forward: L z = r
    const double zs = bcast(acc, k) * sdinv[k];
    acc = (opaque(lane) > k) ? fma(-c[k], zs, acc) : acc;
  }
  acc *= dinv;                           // D w = z
#pragma unroll
  for (int k = N - 1; k >= 0; --k) {     // backward: L^T x = w
    const double xk = bcast(acc, k);
    acc = (opaque(lane) < k) ? fma(-c[k], xk, acc) : acc;
  }
  return acc;
}

// ---- the kernel ----------------------------------------------------------------------------
template <class D>
__global__ __launch_bounds__(kWave) void osc_solve_kernel(
    const DevParams* __restrict__ P, int nenv, const double* __restrict__ gM,
    const double* __restrict__ gC, const double* __restrict__ gJ, const double* __restrict__ gb,
    const double* __restrict__ gT, const double* __restrict__ gmask, double* __restrict__ gtau,
    double* __restrict__ gx, int32_t* __restrict__ gstatus, int32_t* __restrict__ giters,
    double* __restrict__ gdbg) {
  constexpr int NV = D::NV, NU = D::NU, NC = D::NC, NS = D::NS, NB = D::NB, NY = D::NY,
                NY1 = D::NY1, S = D::S, MI = D::MI, NA = D::NA;
  __shared__ __attribute__((aligned(16))) double sm[D::SMEM];
  const int env = blockIdx.x;
  const int lane = threadIdx.x;
  if (env >= nenv) return;

  double* sJ = sm + D::O_J;
  double* sE = sm + D::O_E;
  double* sT = sm + D::O_T;
  double* sM = sm + D::O_M;
  double* sC = sm + D::O_C;
  double* sHa = sm + D::O_HA;
  double* sX = sm + D::O_X;
  double* sU = sm + D::O_U;
  double* sMask = sm + D::O_MASK;
  double* sT1 = sm + D::O_T1;
  double* sHr = sm + D::O_HR;

  // ---------------- Phase A: stage this env's inputs HBM -> LDS ----------------
  stage(sJ, gJ + static_cast<size_t>(env) * S * NV, S * NV, lane);
  stage(sM, gM + static_cast<size_t>(env) * NV * NV, NV * NV, lane);
  stage(sC, gC + static_cast<size_t>(env) * NV, NV, lane);
  stage(sE, gb + static_cast<size_t>(env) * S, S, lane);
  stage(sT, gT + static_cast<size_t>(env) * NS * 6, NS * 6, lane);
  stage(sMask, gmask + static_cast<size_t>(env) * NC, NC, lane);
  __syncthreads();
  // e = b - t,  t = [T[:,0:3] row-wise ; T[:,3:6] row-wise]   (autogen.py:163-168)
  for (int r = lane; r < S; r += kWave) {
    const int half = r / (3 * NS), rr = r % (3 * NS);
    sE[r] -= sT[(rr / 3) * 6 + half * 3 + rr % 3];
  }
  __syncthreads();

  // ---------------- Phase B: Ha = 2 [J e]' W [J e]  (H_dv block and f_dv column) -------------
  // H_dv = 2 J'WJ + 2 w_reg I,  f_dv = 2 J'W (b - t)   (autogen.py:131-238, 304-319)
  for (int p = lane; p < D::NPA; p += kWave) {
    const int i = kPairs<NA, false>.a[p], j = kPairs<NA, false>.b[p];
    double acc = 0.0;
    for (int r = 0; r < S; ++r) {
      const double ai = (i < NV) ? sJ[r * NV + i] : sE[r];
      const double aj = (j < NV) ? sJ[r * NV + j] : sE[r];
      acc = fma(P->w_row[r] * ai, aj, acc);
    }
    acc *= 2.0;
    if (i == j && i < NV) acc += 2.0 * P->w_reg;
    sHa[i * NA + j] = acc;
    sHa[j * NA + i] = acc;
  }

  // ---------------- Phase C: base-block elimination  X = M_bb^-1 [-M_ba | Jc_b | -C_b] -------
  // and the torque map U = M_a P + [M_aa | -Jc_a | C_a]  so that  u = U [y; 1].
  // (dynamics rows: autogen.py:58-89; Jc = Jp[last 3nc rows]^T: osc.h:439-445)
  constexpr int JC0 = 3 * (NS - NC);   // first contact translational row of J
  if (lane < NY1) {
    const int c = lane;
    const bool pinned = (c >= NU && c < NY) && (sMask[(c - NU) / 3] == 0.0);
    double x[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      double r;
      if (c < NU) r = -sM[i * NV + NB + c];
      else if (c < NY) r = sJ[(JC0 + c - NU) * NV + i];
      else r = -sC[i];
      x[i] = pinned ? 0.0 : r;
    }
    // LDL^T of the NB x NB base block (redundantly per lane; NB^3/6 flops)
    double L[NB][NB];
    double dinv[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i)
#pragma unroll
      for (int j = 0; j <= i; ++j) L[i][j] = sM[i * NV + j];
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      dinv[k] = 1.0 / L[k][k];
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
#pragma unroll
    for (int i = 0; i < NB; ++i) sX[i * NY1 + c] = x[i];
    for (int a = 0; a < NU; ++a) {
      double acc;
      if (c < NU) acc = sM[(NB + a) * NV + NB + c];
      else if (c < NY) acc = -sJ[(JC0 + c - NU) * NV + NB + a];
      else acc = sC[NB + a];
      if (pinned) acc = 0.0;
#pragma unroll
      for (int i = 0; i < NB; ++i) acc = fma(sM[(NB + a) * NV + i], x[i], acc);
      sU[a * NY1 + c] = acc;
    }
  }
  __syncthreads();   // J, M, C dead from here on (R1, R2 get reused)

  // ---------------- Phase D: reduced Hessian / gradient ----------------------------------
  // dv = Pm [y;1] with Pm = [X ; (I_nu 0 0)],  T1 = H_dv Pm (+ f_dv in the affine column),
  // Hr = Pm' T1 + 2 (w_tau + w_reg) U'U + 2 w_reg I_z,   g = last column.
  for (int idx = lane; idx < NV * NY1; idx += kWave) {
    const int r = idx / NY1, c = idx % NY1;
    double acc = (c < NU) ? sHa[r * NA + NB + c] : ((c == NY) ? sHa[r * NA + NV] : 0.0);
#pragma unroll
    for (int i = 0; i < NB; ++i) acc = fma(sHa[r * NA + i], sX[i * NY1 + c], acc);
    sT1[r * NY1 + c] = acc;
  }
  __syncthreads();
  double* sG = sm + D::O_G;
  {
    const double wu2 = 2.0 * (P->w_torque + P->w_reg);
    const double wr2 = 2.0 * P->w_reg;
    for (int p = lane; p < D::NPH; p += kWave) {
      const int a = kPairs<NY1, true>.a[p], b = kPairs<NY1, true>.b[p];
      double acc = (a < NU) ? sT1[(NB + a) * NY1 + b] : 0.0;
#pragma unroll
      for (int r = 0; r < NB; ++r) acc = fma(sX[r * NY1 + a], sT1[r * NY1 + b], acc);
      double uu = 0.0;
#pragma unroll
      for (int q = 0; q < NU; ++q) uu = fma(sU[q * NY1 + a], sU[q * NY1 + b], uu);
      acc = fma(wu2, uu, acc);
      if (b < NY) {
        if (a == b && a >= NU) {
          acc += wr2;
          if (sMask[(a - NU) / 3] == 0.0) acc = 1.0;   // pinned z: identity row
        }
        sHr[a * NY + b] = acc;
        sHr[b * NY + a] = acc;
      } else {
        sG[a] = acc;
      }
    }
  }
  __syncthreads();

  if (gdbg != nullptr) {   // test hook (osc_debug_reduced_qp): dump the reduced QP
    double* o = gdbg + static_cast<size_t>(env) * D::DBG;
    for (int i = lane; i < NY * NY; i += kWave) o[i] = sHr[i];
    for (int i = lane; i < NY; i += kWave) o[NY * NY + i] = sG[i];
    for (int i = lane; i < NU * NY1; i += kWave) o[NY * NY + NY + i] = sU[i];
    for (int i = lane; i < NB * NY1; i += kWave) o[NY * NY + NY + NU * NY1 + i] = sX[i];
  }

  // ---------------- Phase E: Mehrotra predictor-corrector interior point ------------------
  double* sVy = sm + D::O_VY;     // broadcast copy of a y-space vector
  double* sVy2 = sm + D::O_VY2;
  double* sDg = sm + D::O_DG;     // original diagonal of K
  double* sVr = sm + D::O_VR;     // broadcast copy of a row-space vector
  double* sDr = sm + D::O_DR;     // lambda / s
  double* sDinv = sm + D::O_VR2;  // 1 / D of the LDL^T factor (NY <= MI entries)
  double* sTau = sm + D::O_TAU;

  // Row description for this lane (row r = lane).
  const int r = lane;
  bool act = false;
  double h = 0.0;
  int rq = 0, rk = 0, rt = 0;        // u-row index / contact / row type
  double rsg = 0.0;
  if (r < 2 * NU) {
    rq = r >> 1;
    rsg = (r & 1) ? -1.0 : 1.0;
    const double bnd = (r & 1) ? P->u_lb[rq] : P->u_ub[rq];
    act = fabs(bnd) < P->inf_thresh;
    h = rsg * (bnd - sU[rq * NY1 + NY]);
  } else if (r < MI) {
    rk = (r - 2 * NU) / 6;
    rt = (r - 2 * NU) % 6;
    const double m = sMask[rk];
    if (m != 0.0) {
      if (rt < 4) {
        act = true;                                   // friction pyramid, bineq = 0
        h = 0.0;
      } else if (rt == 4) {
        const double lb = P->z_lb[2] * m;             // -fz <= -lb
        act = fabs(lb) < P->inf_thresh;
        h = -lb;
      } else {
        const double ub = P->z_ub[2] * m;             // fz <= ub
        act = fabs(ub) < P->inf_thresh;
        h = ub;
      }
    }
  }
  const double mu_f = P->mu;
  const double psx = (rt & 1) ? -1.0 : 1.0;   // pyramid row signs: (1,1),(-1,1),(1,-1),(-1,-1)
  const double psy = (rt >= 2) ? -1.0 : 1.0;
  const int zc0 = NU + 3 * rk;

  // (G v)_r for v staged in LDS
  auto Gv = [&](const double* v) -> double {
    double acc = 0.0;
    if (!act) return 0.0;
    if (r < 2 * NU) {
#pragma unroll
      for (int i = 0; i < NY; ++i) acc = fma(sU[rq * NY1 + i], v[i], acc);
      return rsg * acc;
    }
    if (rt < 4) return psx * v[zc0] + psy * v[zc0 + 1] - mu_f * v[zc0 + 2];
    return (rt == 4) ? -v[zc0 + 2] : v[zc0 + 2];
  };
  // Column role for lane j (var j)
  const int j = lane;
  const int jk = (j >= NU && j < NY) ? (j - NU) / 3 : -1;
  const int jc = (j >= NU && j < NY) ? (j - NU) % 3 : 0;
  // (G' w)_j for w staged in LDS (inactive rows hold 0)
  auto GTw = [&](const double* w) -> double {
    double acc = 0.0;
    if (j >= NY) return 0.0;
#pragma unroll
    for (int q = 0; q < NU; ++q) acc = fma(sU[q * NY1 + j], w[2 * q] - w[2 * q + 1], acc);
    if (jk >= 0) {
      const double* wk = w + 2 * NU + 6 * jk;
      if (jc == 0) acc += wk[0] - wk[1] + wk[2] - wk[3];
      else if (jc == 1) acc += wk[0] + wk[1] - wk[2] - wk[3];
      else acc += -mu_f * (wk[0] + wk[1] + wk[2] + wk[3]) - wk[4] + wk[5];
    }
    return acc;
  };
  // K = Hr + G' diag(Dr) G, column j in registers; also records the diagonal in sDg.
  auto assemble = [&](double (&c)[NY]) {
    const int jj = (j < NY) ? j : 0;
#pragma unroll
    for (int i = 0; i < NY; ++i) c[i] = sHr[i * NY + jj];
    double dg = sHr[jj * NY + jj];
#pragma unroll 1
    for (int q = 0; q < NU; ++q) {   // rolled: bounds the number of U loads in flight
      const double du = sDr[2 * q] + sDr[2 * q + 1];
      const double uj = sU[q * NY1 + jj];
      const double t = du * uj;
      dg = fma(t, uj, dg);
#pragma unroll
      for (int i = 0; i < NY; ++i) c[i] = fma(t, sU[q * NY1 + i], c[i]);
    }
    if (jk >= 0) {
      const double* dk = sDr + 2 * NU + 6 * jk;
      const double s4 = dk[0] + dk[1] + dk[2] + dk[3];
      const double sxy = dk[0] - dk[1] - dk[2] + dk[3];
      const double sx = dk[0] - dk[1] + dk[2] - dk[3];
      const double sy = dk[0] + dk[1] - dk[2] - dk[3];
      const double b00 = s4, b11 = s4, b01 = sxy, b02 = -mu_f * sx, b12 = -mu_f * sy,
                   b22 = mu_f * mu_f * s4 + dk[4] + dk[5];
      const double v0 = (jc == 0) ? b00 : (jc == 1) ? b01 : b02;
      const double v1 = (jc == 0) ? b01 : (jc == 1) ? b11 : b12;
      const double v2 = (jc == 0) ? b02 : (jc == 1) ? b12 : b22;
      dg += (jc == 0) ? v0 : (jc == 1) ? v1 : v2;
#pragma unroll
      for (int i = NU; i < NY; ++i) {
        const int ki = (i - NU) / 3, ci = (i - NU) % 3;
        const double add = (ci == 0) ? v0 : (ci == 1) ? v1 : v2;
        c[i] += (ki == jk) ? add : 0.0;
      }
    }
    if (j < NY) sDg[j] = dg;
    __syncthreads();
  };

  double c[NY];
  double dinv;
  const double gj = (j < NY) ? sG[j] : 0.0;
  int32_t st = OSC_SOLVE_MAX_ITER;
  int it;
  const double m_act = wave_sum(act ? 1.0 : 0.0);   // active rows (wave-uniform)
  double yj = 0.0, s = 1.0, lam = 0.0;

  // One loop body for everything, so the factorisation and solve code exist once in the
  // binary (I-cache).  it == -1 builds the initial point (Mehrotra-style):
  //   (Hr + G'G) y0 = -g + G'h,   s = h - G y0,  lambda = G y0 - h,  both shifted positive.
  for (it = -1;; ++it) {
    const bool init = it < 0;
    double rp = 0.0, rd = gj, mu = 0.0;
    if (init) {
      sDr[r] = act ? 1.0 : 0.0;
    } else {
      const double gy = Gv(sVy);
      rp = act ? gy + s - h : 0.0;
      mu = wave_sum(act ? s * lam : 0.0) / m_act;
      if (mu <= P->eps_mu) {
        st = OSC_SOLVE_OK;
        break;
      }
      if (it >= P->max_iter) break;
      // dual residual rd = Hr y + g + G' lambda ;  D = lambda / s
      sVr[r] = act ? lam : 0.0;
      sDr[r] = act ? lam / s : 0.0;
      __syncthreads();
      rd += GTw(sVr);
      if (j < NY) {
#pragma unroll
        for (int i = 0; i < NY; ++i) rd = fma(sHr[i * NY + j], sVy[i], rd);
      }
    }
    __syncthreads();
    assemble(c);
    ldl_columns<NY>(c, dinv, sDg, sDinv, lane);

    // pass 0: affine (predictor) direction, rc = s lambda
    // pass 1: corrector, rc = s lambda + ds_aff dl_aff - sigma mu
    double ds = 0.0, dl = 0.0, dyj = 0.0, gdy = 0.0, ds_a = 0.0, dl_a = 0.0, sig_mu = 0.0,
           step = 1.0;
    const int npass = init ? 1 : 2;
    for (int pass = 0; pass < npass; ++pass) {
      const double rcv = (pass == 0) ? s * lam : fma(ds_a, dl_a, s * lam) - sig_mu;
      sVr[r] = init ? (act ? h : 0.0) : (act ? (rcv - lam * rp) / s : 0.0);
      __syncthreads();
      dyj = ldl_solve<NY>(c, dinv, sDinv, -rd + GTw(sVr), lane);
      if (j < NY) sVy2[j] = dyj;
      __syncthreads();
      gdy = Gv(sVy2);
      ds = act ? -rp - gdy : 0.0;
      dl = act ? -(rcv + lam * ds) / s : 0.0;
      double ratio = 1.0;
      if (act) {
        if (ds < 0.0) ratio = fmin(ratio, -s / ds);
        if (dl < 0.0) ratio = fmin(ratio, -lam / dl);
      }
      step = wave_min(ratio);
      if (pass == 0 && !init) {
        const double mu_aff = wave_sum(act ? (s + step * ds) * (lam + step * dl) : 0.0) / m_act;
        const double q = mu_aff / mu;
        sig_mu = q * q * q * mu;
        ds_a = ds;
        dl_a = dl;
      }
      __syncthreads();
    }
    if (init) {
      yj = dyj;
      const double zr = gdy - h;
      const double ap = wave_max(act ? zr : -1e300);    // = max(-s)
      const double ad = wave_max(act ? -zr : -1e300);   // = max(-lambda)
      s = act ? ((ap >= 0.0) ? -zr + 1.0 + ap : -zr) : 1.0;
      lam = act ? ((ad >= 0.0) ? zr + 1.0 + ad : zr) : 0.0;
    } else {
      const double alpha = fmin(1.0, 0.99 * step);
      yj = fma(alpha, dyj, yj);
      s = act ? fma(alpha, ds, s) : 1.0;
      lam = act ? fma(alpha, dl, lam) : 0.0;
    }
    if (j < NY) sVy[j] = yj;
    __syncthreads();
    if (init && m_act == 0.0) {   // unconstrained: y0 = -Hr^-1 g is the optimum
      st = OSC_SOLVE_OK;
      it = 0;
      break;
    }
  }

  // ---------------- outputs: tau = U [y;1];  x = (dv_b, dv_a, u, z) ----------------------
  double tq = 0.0;
  if (lane < NU) {
    tq = sU[lane * NY1 + NY];
#pragma unroll
    for (int i = 0; i < NY; ++i) tq = fma(sU[lane * NY1 + i], sVy[i], tq);
    sTau[lane] = tq;
  }
  double xb = 0.0;
  if (lane < NB) {
    xb = sX[lane * NY1 + NY];
#pragma unroll
    for (int i = 0; i < NY; ++i) xb = fma(sX[lane * NY1 + i], sVy[i], xb);
  }
  __syncthreads();
  const bool finite = wave_min((lane < NY) ? (isfinite(yj) ? 1.0 : 0.0) : 1.0) > 0.0;
  if (!finite) st = OSC_SOLVE_NUMERICAL;
  if (lane < NU) gtau[static_cast<size_t>(env) * NU + lane] = tq;
  if (gx != nullptr && lane < D::NX) {
    double v;
    if (lane < NB) v = xb;
    else if (lane < NV) v = sVy[lane - NB];
    else if (lane < NV + NU) v = sTau[lane - NV];
    else v = sVy[NU + lane - NV - NU];
    gx[static_cast<size_t>(env) * D::NX + lane] = v;
  }
  if (lane == 0) {
    if (gstatus) gstatus[env] = st;
    if (giters) giters[env] = it;
  }
}

using Go2 = Dims<18, 12, 4, 5>;       // unitree_go2: nv 18, nu 12, 4 feet, 5 sites
using Walter = Dims<14, 8, 8, 17>;    // walter_sr(_wheels): nv 14, nu 8, 8 wheels, 17 sites

enum KernelId { K_NONE = 0, K_GO2 = 1, K_WALTER = 2 };

KernelId select_kernel(const osc_model_desc& d) {
  if (d.nv == Go2::NV && d.nu == Go2::NU && d.nc == Go2::NC && d.ns == Go2::NS) return K_GO2;
  if (d.nv == Walter::NV && d.nu == Walter::NU && d.nc == Walter::NC && d.ns == Walter::NS)
    return K_WALTER;
  return K_NONE;
}

}  // namespace

struct osc_model {
  osc_model_desc desc;
  KernelId kid;
  DevParams* dparams;
  int device;
};

extern "C" int osc_model_create(const osc_model_desc* desc, osc_model** out) {
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
  hp.eps_mu = d.eps_mu;
  hp.inf_thresh = thresh;
  hp.max_iter = d.max_iter;

  osc_model* m = new (std::nothrow) osc_model;
  if (!m) return OSC_ERR_DEVICE;
  m->desc = d;
  m->kid = kid;
  m->dparams = nullptr;
  (void)hipGetDevice(&m->device);
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

namespace {
int launch(const osc_model* model, int32_t nenv, const double* M, const double* C, const double* J,
           const double* b, const double* T, const double* contact_mask, double* tau, double* x,
           int32_t* status, int32_t* iters, void* stream, double* dbg) {
  if (!model || nenv < 0) return OSC_ERR_INVALID_ARGUMENT;
  if (nenv == 0) return OSC_OK;
  if (!M || !C || !J || !b || !T || !contact_mask || !tau) return OSC_ERR_INVALID_ARGUMENT;
  // 16-byte alignment is required by the vectorised staging loads.
  const uintptr_t align = reinterpret_cast<uintptr_t>(M) | reinterpret_cast<uintptr_t>(C) |
                          reinterpret_cast<uintptr_t>(J) | reinterpret_cast<uintptr_t>(b) |
                          reinterpret_cast<uintptr_t>(T) |
                          reinterpret_cast<uintptr_t>(contact_mask);
  if (align & 15u) return OSC_ERR_INVALID_ARGUMENT;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const dim3 grid(static_cast<unsigned>(nenv)), block(kWave);
  switch (model->kid) {
    case K_GO2:
      hipLaunchKernelGGL(osc_solve_kernel<Go2>, grid, block, 0, s, model->dparams, nenv, M, C, J,
                         b, T, contact_mask, tau, x, status, iters, dbg);
      break;
    case K_WALTER:
      hipLaunchKernelGGL(osc_solve_kernel<Walter>, grid, block, 0, s, model->dparams, nenv, M, C,
                         J, b, T, contact_mask, tau, x, status, iters, dbg);
      break;
    default:
      return OSC_ERR_UNSUPPORTED_DIMS;
  }
  return hipGetLastError() == hipSuccess ? OSC_OK : OSC_ERR_DEVICE;
}
}  // namespace

extern "C" int osc_batch_solve(const osc_model* model, int32_t nenv, const double* M,
                               const double* C, const double* J, const double* b, const double* T,
                               const double* contact_mask, double* tau, double* x,
                               int32_t* status, int32_t* iters, void* stream) {
  return launch(model, nenv, M, C, J, b, T, contact_mask, tau, x, status, iters, stream, nullptr);
}

// Test hook, not part of include/osc_batch.h: same solve, plus a per-env dump of the reduced QP
// [Hr (NY x NY) | g (NY) | U (NU x (NY+1)) | X (NB x (NY+1))] into `dbg` (device pointer,
// osc_debug_dump_size() doubles per env).  Used by tests/test_gpu_stages.py.
extern "C" int osc_debug_dump_size(const osc_model* model) {
  if (!model) return -1;
  switch (model->kid) {
    case K_GO2: return Go2::DBG;
    case K_WALTER: return Walter::DBG;
    default: return -1;
  }
}

extern "C" int osc_debug_reduced_qp(const osc_model* model, int32_t nenv, const double* M,
                                    const double* C, const double* J, const double* b,
                                    const double* T, const double* contact_mask, double* tau,
                                    double* dbg, void* stream) {
  if (!dbg) return OSC_ERR_INVALID_ARGUMENT;
  return launch(model, nenv, M, C, J, b, T, contact_mask, tau, nullptr, nullptr, nullptr, stream,
                dbg);
}
