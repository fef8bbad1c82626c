// osc_dual.hip -- kernel 3, the dual solution of the reference's QP (optional output,
// osc_solve_extras.y): OsqpSolver::dual_solution, unitree_go2/operational_space_controller.h:
// 534-535.
#include "osc_internal.hpp"
#include "osc_wave_sum.hpp"

namespace osc {

// ============================ kernel 3: dual solution (optional output) ======================
// The reference's OsqpSolver::dual_solution (operational_space_controller.h:534-535) over its rows
// A = [Aeq; Aineq; I_n] (osc.h:483-497; with wheel rows Aeq = [dynamics; wheel rows]) in OSQP's
// sign convention (H x + f + A'y = 0, y >= 0 on an active upper bound, <= 0 on a lower one),
// recovered from the returned design vector x = (dv, u, z) by stationarity:
//   dynamics rows  nu = -M^-1 (H_dv dv + f_dv + E'nu_w)             (the dv block)
//   wheel rows     nu_w by least squares on stationarity itself (below; the interior point's W_NU
//                  is not read: it exists only where the refinement was kept, and the active-set
//                  fallback's envs have none -- ADVICE r5)
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
// (two waves per SIMD at least: with the serial solves' loops rolled the wheel model's kernel
// needs 124 VGPRs, four waves per SIMD -- it ran one per SIMD at 256 + 28 fully unrolled,
// 2,048 envs in two rounds of waves: 206 -> 155 us, the inner loops unrolled by four 149 us,
// bitwise, profiles/r05/dual/r05du{4,5}_*)
__global__ __launch_bounds__(kWave, 2) void osc_dual_kernel(
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
#ifdef OSC_DUAL_PROFILE   // per-phase clocks of one wave (diagnostic build, printf per env)
  unsigned long long dp[8] = {0, 0, 0, 0, 0, 0, 0, 0}, dt0 = 0, dt1 = 0;
#define DU_T(k) do { asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(dt1)::"memory"); dp[k] += dt1 - dt0; dt0 = dt1; } while (0)
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(dt0)::"memory");
#else
#define DU_T(k) do {} while (0)
#endif
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
  DU_T(0);
  // L L' v = b in place (one lane, serial)
  auto chol_solve = [&](double* v) {
    #pragma unroll 1
    for (int i = 0; i < NV; ++i) {
      double a = v[i];
      #pragma unroll 4
      for (int p = 0; p < i; ++p) a = fma(-sL[i * NV + p], v[p], a);
      v[i] = a / sL[i * NV + i];
    }
    #pragma unroll 1
    for (int i = NV - 1; i >= 0; --i) {
      double a = v[i];
      #pragma unroll 4
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
    DU_T(1);
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
        // orthonormal basis of the active normals' span (Gram-Schmidt), then its complement; the
        // slot loops run over compile-time slots with the runtime count as a predicate (runtime-
        // indexed arrays would live in scratch)
        double q[3][3] = {{0.0, 0.0, 0.0}, {0.0, 0.0, 0.0}, {0.0, 0.0, 0.0}};
        int rk = 0;
        const double ub = P->z_ub[2] * mask[k], lb = P->z_lb[2] * mask[k];
#pragma unroll
        for (int i = 0; i < 6; ++i) {
          double g[3];
          double gap;
          bool have = true;
          if (i < 4) {
            g[0] = (i & 1) ? -1.0 : 1.0; g[1] = (i >= 2) ? -1.0 : 1.0; g[2] = -mu;
            gap = -(g[0] * f0 + g[1] * f1 + g[2] * f2);
          } else if (i == 4) {
            have = fabs(lb) < P->inf_thresh;
            g[0] = g[1] = 0.0; g[2] = -1.0; gap = f2 - lb;
          } else {
            have = fabs(ub) < P->inf_thresh;
            g[0] = g[1] = 0.0; g[2] = 1.0; gap = ub - f2;
          }
          if (!have || gap > tol || rk == 3) continue;
#pragma unroll
          for (int a = 0; a < 3; ++a) {
            if (a < rk) {
              const double d = g[0] * q[a][0] + g[1] * q[a][1] + g[2] * q[a][2];
              for (int c = 0; c < 3; ++c) g[c] -= d * q[a][c];
            }
          }
          const double nn = sqrt(g[0] * g[0] + g[1] * g[1] + g[2] * g[2]);
          if (nn > 1e-6) {
#pragma unroll
            for (int a = 0; a < 3; ++a)
              if (a == rk)
                for (int c = 0; c < 3; ++c) q[a][c] = g[c] / nn;
            ++rk;
          }
        }
        // complement: e_c orthogonalised against the span and the complement vectors so far
        int nc = 0;
        double pc[3][3] = {{0.0, 0.0, 0.0}, {0.0, 0.0, 0.0}, {0.0, 0.0, 0.0}};
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          if (rk + nc >= 3) break;
          double v[3] = {c == 0 ? 1.0 : 0.0, c == 1 ? 1.0 : 0.0, c == 2 ? 1.0 : 0.0};
#pragma unroll
          for (int a = 0; a < 3; ++a) {
            if (a < rk) {
              const double d = v[0] * q[a][0] + v[1] * q[a][1] + v[2] * q[a][2];
              for (int e = 0; e < 3; ++e) v[e] -= d * q[a][e];
            }
          }
#pragma unroll
          for (int a = 0; a < 3; ++a) {
            if (a < nc) {
              const double d = v[0] * pc[a][0] + v[1] * pc[a][1] + v[2] * pc[a][2];
              for (int e = 0; e < 3; ++e) v[e] -= d * pc[a][e];
            }
          }
          const double nn = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
          if (nn < 0.5) continue;
          double pn[3];
          for (int e = 0; e < 3; ++e) pn[e] = v[e] / nn;
#pragma unroll
          for (int a = 0; a < 3; ++a)
            if (a == nc)
              for (int e = 0; e < 3; ++e) pc[a][e] = pn[e];
          // p' r_k = 0 with r_k = wz f - Jc_k' (nu0 - W nu_w)
          double rhs = 0.0;
          double* row = sA + n * NW;   // (built in place)
          for (int w = 0; w < NW; ++w) row[w] = 0.0;
          for (int cc = 0; cc < 3; ++cc) {
            const double jn0 = sJN0[3 * k + cc];
            const double fc = cc == 0 ? f0 : (cc == 1 ? f1 : f2);
            rhs = fma(pn[cc], wz * fc - jn0, rhs);
            for (int w = 0; w < NW; ++w) row[w] = fma(pn[cc], sJW[(3 * k + cc) * NW + w], row[w]);
          }
          sb[n++] = -rhs;   // row . nu_w = -rhs
          ++nc;
        }
      }
      snrow = n;
    }
    __syncthreads();
    DU_T(2);
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
      wave_argmax_fast(v, p);   // the largest, the lowest column among ties (same butterfly order)
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
  DU_T(3);
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
    #pragma unroll 1
    for (int i = 0; i < NV; ++i) {
      double a = sg[i];
      #pragma unroll 4
      for (int p = 0; p < i; ++p) a = fma(-sL[i * NV + p], sg[p], a);
      sg[i] = a / sL[i * NV + i];
    }
    #pragma unroll 1
    for (int i = NV - 1; i >= 0; --i) {
      double a = sg[i];
      #pragma unroll 4
      for (int p = i + 1; p < NV; ++p) a = fma(-sL[p * NV + i], sg[p], a);
      sg[i] = a / sL[i * NV + i];
    }
  }
  __syncthreads();
  DU_T(4);
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
      // rows g_i' f <= h_i: pyramid (sx, sy, -mu) <= 0, -fz <= -lb, fz <= ub; the normals as
      // closed forms of the row index (no row arrays: a runtime-indexed array lives in scratch,
      // and the subset loop below indexes by the subset's rows)
      const double ub = P->z_ub[2] * mask[k], lb = P->z_lb[2] * mask[k];
      auto gco = [&](int i, int c) -> double {
        if (i < 4) return c == 0 ? ((i & 1) ? -1.0 : 1.0) : (c == 1 ? ((i >= 2) ? -1.0 : 1.0) : -mu);
        return c == 2 ? (i == 4 ? -1.0 : 1.0) : 0.0;
      };
      const double tol = 1e-8 * (1.0 + fmax(fabs(f[0]), fmax(fabs(f[1]), fabs(f[2]))));
      int act = 0;
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        const double h = i < 4 ? 0.0 : (i == 4 ? -lb : ub);
        const double gi = gco(i, 0) * f[0] + gco(i, 1) * f[1] + gco(i, 2) * f[2] - h;
        const bool finite = (i < 4) || fabs(h) < P->inf_thresh;
        if (finite && gi >= -tol) act |= 1 << i;
      }
      // min |r + G_S' m| over m >= 0, S a subset of the active rows with |S| <= 3 (Caratheodory):
      // per subset the 3 x 3 Gram system (G_S G_S') m = -G_S r by LDL^T (symmetric positive
      // semi-definite; a pivot under 1e-12 marks a dependent subset, skipped), unused slots as
      // identity rows -- all in registers
      double best = r[0] * r[0] + r[1] * r[1] + r[2] * r[2];
      int bestS = 0;
      double bm0 = 0.0, bm1 = 0.0, bm2 = 0.0;
#pragma unroll 1
      for (int S = 1; S < 64; ++S) {
        const int n = __builtin_popcount(S);
        if ((S & act) != S || n > 3) continue;
        const int S1 = S & (S - 1), S2 = S1 & (S1 - 1);
        const int i0 = __builtin_ctz(S), i1 = S1 ? __builtin_ctz(S1) : 0, i2 = S2 ? __builtin_ctz(S2) : 0;
        const double a0 = gco(i0, 0), a1 = gco(i0, 1), a2 = gco(i0, 2);
        const double b0 = n > 1 ? gco(i1, 0) : 0.0, b1 = n > 1 ? gco(i1, 1) : 0.0,
                     b2 = n > 1 ? gco(i1, 2) : 0.0;
        const double c0 = n > 2 ? gco(i2, 0) : 0.0, c1 = n > 2 ? gco(i2, 1) : 0.0,
                     c2 = n > 2 ? gco(i2, 2) : 0.0;
        const double A00 = a0 * a0 + a1 * a1 + a2 * a2, A01 = a0 * b0 + a1 * b1 + a2 * b2,
                     A02 = a0 * c0 + a1 * c1 + a2 * c2;
        const double A11 = n > 1 ? b0 * b0 + b1 * b1 + b2 * b2 : 1.0,
                     A12 = b0 * c0 + b1 * c1 + b2 * c2;
        const double A22 = n > 2 ? c0 * c0 + c1 * c1 + c2 * c2 : 1.0;
        const double r0 = -(a0 * r[0] + a1 * r[1] + a2 * r[2]);
        const double r1 = -(b0 * r[0] + b1 * r[1] + b2 * r[2]);
        const double r2 = -(c0 * r[0] + c1 * r[1] + c2 * r[2]);
        const double d0 = A00;
        if (!(d0 >= 1e-12)) continue;
        const double l10 = A01 / d0, l20 = A02 / d0;
        const double d1 = A11 - l10 * A01;
        if (!(d1 >= 1e-12)) continue;
        const double l21 = (A12 - l20 * A01) / d1;
        const double d2 = A22 - l20 * A02 - l21 * l21 * d1;
        if (!(d2 >= 1e-12)) continue;
        const double y0 = r0, y1 = r1 - l10 * y0, y2 = r2 - l20 * y0 - l21 * y1;
        const double m2 = y2 / d2, m1 = y1 / d1 - l21 * m2, m0 = y0 / d0 - l10 * m1 - l20 * m2;
        if (!(m0 >= 0.0 && m1 >= 0.0 && m2 >= 0.0)) continue;
        double res = 0.0;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const double t = r[c] + m0 * (c == 0 ? a0 : c == 1 ? a1 : a2) +
                           m1 * (c == 0 ? b0 : c == 1 ? b1 : b2) + m2 * (c == 0 ? c0 : c == 1 ? c1 : c2);
          res += t * t;
        }
        if (res < best * (1.0 - 1e-12)) {
          best = res;
          bestS = S;
          bm0 = m0;
          bm1 = m1;
          bm2 = m2;
        }
      }
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        const int a = __builtin_popcount(bestS & ((1 << i) - 1));
        if (bestS >> i & 1) q[i] = a == 0 ? bm0 : (a == 1 ? bm1 : bm2);
      }
    }
    for (int i = 0; i < 6; ++i) sq[6 * k + i] = q[i];
  }
  __syncthreads();
  DU_T(5);
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
#ifdef OSC_DUAL_PROFILE
  DU_T(6);
  if (lane == 0 && env % 256 == 0)
    printf("dual env %d cyc chol %llu wrows %llu lsrows %llu qr %llu nu %llu nnls %llu out %llu\n", env,
           dp[0], dp[1], dp[2], dp[3], dp[4], dp[5], dp[6]);
#endif
}

template <class D>
void launch_dual(const LaunchArgs& a) {
  hipLaunchKernelGGL(osc_dual_kernel<D>, dim3(static_cast<unsigned>(a.nenv)), dim3(kWave), 0, a.s,
                     a.model->dparams, a.nenv, a.M, a.J, a.mask, a.wdir, a.ws, a.x, a.y);
}

template void launch_dual<Go2>(const LaunchArgs&);
template void launch_dual<Walter>(const LaunchArgs&);
template void launch_dual<WalterW>(const LaunchArgs&);

}  // namespace osc
