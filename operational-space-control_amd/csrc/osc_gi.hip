// osc_gi.hip -- kernel 4, the wheel-row models' active-set fallback (osc_gi_kernel): Goldfarb &
// Idnani's dual method on the full QP of an env the interior point left unconverged (DESIGN.md
// §3.1; the opt-in rows of walter_sr_wheels/autogen/autogen.py:128-240).
#include "osc_internal.hpp"
#include "osc_wave_sum.hpp"

namespace osc {

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
    const DevParams* __restrict__ P, int nenv, const double* __restrict__ gmask,
    const double* __restrict__ ws, double* __restrict__ gtau, double* __restrict__ gx,
    int32_t* __restrict__ gstatus, int32_t* __restrict__ giters, double* __restrict__ gwarm) {
  constexpr int NV = D::NV, NU = D::NU, NC = D::NC, NW = D::NW, NX = D::NX,
                NB = D::NB, NZ = D::NZ;
  constexpr int NXP = NX | 1;                 // odd row stride (LDS banks)
  constexpr int NEQ = NV + NW + NZ;           // dynamics, wheel rows, forces of masked contacts
  constexpr int NIN = 2 * NU + 6 * NC;        // one-sided rows: u box, pyramid, fz box
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
  __shared__ double2 sCS[NX];                 // add_row's rotations (c, s)
  const double* wenv = ws + static_cast<size_t>(env) * D::WS;
  // the raw rows, as the setup kernel copied them into this env's workspace block: M, C, the
  // contact rows of J (Jc, 3 NC x NV) and of b (bc), the wheel directions
  const double* M = wenv + D::W_RM;
  const double* C = wenv + D::W_RC;
  const double* Jc = wenv + D::W_RJ;
  const double* bc = wenv + D::W_RB;
  const double* mask = gmask + static_cast<size_t>(env) * NC;
  const double* wd = wenv + D::W_RD;
  const double hu = 2.0 * (P->w_torque + P->w_reg), hz = 2.0 * P->w_reg;

  // the 64-lane butterflies (sum, max, (value, index) minimum with the lowest index among ties),
  // their partners by lane-crossing VALU ops (osc_wave_sum.hpp; the shuffle form's order and bits)
  auto wsum = [](double v) { return wave_sum_fast(v); };
  auto wmax = [](double v) { return wave_max_fast(v); };
  auto wargmin = [](double& v, int& idx) { wave_argmin_fast(v, idx); };
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
      else v = -Jc[(lane - NV - NU) * NV + i];
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
        for (int c = 0; c < 3; ++c) v = fma(wd[6 * i + 3 * side + c], Jc[(3 * i + c) * NV + lane], v);
        if (side == 0 && lane == P->wheel_dof[i]) v -= P->wheel_radius[i];
        v *= mask[i];
      }
      sE[neq * NXP + lane] = v;
    }
    if (lane == 0) {
      double e = 0.0;
      for (int c = 0; c < 3; ++c) e = fma(wd[6 * i + 3 * side + c], bc[3 * i + c], e);
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

#ifdef OSC_GI_PROFILE
  unsigned long long tp[11] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, t0 = 0, t1_ = 0, ta = 0, tb = 0;
  int ndrop = 0, nadd = 0;
#define GI_T0() asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory")
#define GI_T1(k) do { asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1_)::"memory"); tp[k] += t1_ - t0; } while (0)
#define GI_TA(v) asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory")
#else
#define GI_TA(v) do {} while (0)
#define GI_T0() do {} while (0)
#define GI_T1(k) do {} while (0)
#endif
  int q = 0;            // working rows
  int act = -1;         // lane j < q: row id of working row j
  double up = 0.0;      // lane j <= q: multipliers (j = q: the candidate's)
  double zi = 0.0;      // lane i: the primal step direction z
  double rj = 0.0;      // lane j in [qe, q): R^-1 d[:q]
  int qe = kWave;       // working equality rows (positions [0, qe), never dropped), once all are in
  // d = J'c (lane j -> sd), z = J[:, q:] d[q:] (lane i), r = R^-1 d[:q] (lane j).  c: a dense
  // equality row in sc, or one-sided row p (<= 3 nonzeros: only those rows of J are read).
  // r is only back-substituted down to position qe: the equality rows' multipliers are never read
  // (no sign test, no drop, not returned), and R's triangle puts them after the one-sided rows'
  // entries in the back substitution -- so the equality phase skips it, and the one-sided steps
  // run q - qe of its serial steps instead of q (x, tau and the working set unchanged, bitwise)
  auto directions = [&](int p) {
#ifdef OSC_GI_PROFILE
    GI_TA(ta);
#endif
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
#ifdef OSC_GI_PROFILE
    GI_TA(tb);
    tp[8] += tb - ta;
    GI_TA(ta);
#endif
    zi = 0.0;
    if (lane < NX) {
      double z1 = 0.0;
      int j = q;
#pragma unroll 4
      for (; j + 1 < NX; j += 2) {
        zi = fma(sJ[lane * NXP + j], sd[j], zi);
        z1 = fma(sJ[lane * NXP + j + 1], sd[j + 1], z1);
      }
      if (j < NX) zi = fma(sJ[lane * NXP + j], sd[j], zi);
      zi += z1;
    }
#ifdef OSC_GI_PROFILE
    GI_TA(tb);
    tp[9] += tb - ta;
    GI_TA(ta);
#endif
    double dv = lane < q ? sd[lane] : 0.0;
    rj = 0.0;
    for (int jj = q - 1; jj >= qe; --jj) {   // back substitution, column-oriented
      const double v = readlane_d(dv, jj) * sRi[jj];
      if (lane == jj) rj = v;
      if (lane < jj) dv = fma(-sR[lane * NXP + jj], v, dv);
    }
#ifdef OSC_GI_PROFILE
    GI_TA(tb);
    tp[10] += tb - ta;
#endif
  };
  // c joins the working set at position q: the rotations (j-1, j), j = NX-1 .. q+1, that fold
  // d[q+1:] into d[q] (J's columns follow); rotation j meets (d[j-1], ||d[j:]||) -- d[NX-1] itself,
  // signed, for the first -- so every (c, s) follows from d's suffix sums of squares, one wave
  // scan instead of a chain of NX - q dependent rotations.  R's column q = d[:q+1].
  auto add_row = [&]() {
#ifdef OSC_GI_PROFILE
    GI_TA(ta);
#endif
    const double dl = lane < NX ? sd[lane] : 0.0;
    double ssq = (lane >= q && lane < NX) ? dl * dl : 0.0;
    for (int o = 1; o < kWave; o <<= 1) {   // suffix sums S_j = sum_{k >= j} d_k^2
      const double v = __shfl_down(ssq, o, kWave);
      if (lane + o < kWave) ssq += v;
    }
    const double sn = __shfl_down(ssq, 1, kWave);            // S_{j+1} on lane j
    const double dnext = __shfl_down(dl, 1, kWave);          // d_{j+1} on lane j
    if (lane < NX - 1) {   // lane j - 1 holds rotation j's (c, s); rotations j <= q: identity
      const double rr = sqrt(ssq);
      double c = 1.0, sv = 0.0;
      if (lane >= q && rr > 0.0) {
        c = dl / rr;
        sv = (lane + 1 == NX - 1 ? dnext : sqrt(sn)) / rr;
      }
      sCS[lane + 1] = make_double2(c, sv);
    }
    const double dq = __shfl(q < NX - 1 ? sqrt(ssq) : dl, q, kWave);
    __syncthreads();
#ifdef OSC_GI_PROFILE
    GI_TA(tb);
    tp[7] += tb - ta;
    GI_TA(ta);
#endif
    if (lane < NX) {
      double row[NX];
#pragma unroll
      for (int c = 0; c < NX; ++c) row[c] = sJ[lane * NXP + c];
      // (every rotation applied, the identity ones too: no branch per rotation, so the (c, s)
      // reads issue ahead of the chain; c * a + s * b with (1, 0) returns a, bitwise)
#pragma unroll
      for (int j = NX - 1; j >= 1; --j) {
        const double2 cs = sCS[j];
        const double c = cs.x, sv = cs.y;
        const double a = row[j - 1], b = row[j];
        row[j - 1] = c * a + sv * b;
        row[j] = -sv * a + c * b;
      }
#pragma unroll
      for (int c = 0; c < NX; ++c) sJ[lane * NXP + c] = row[c];
    }
#ifdef OSC_GI_PROFILE
    GI_TA(tb);
    tp[6] += tb - ta;
#endif
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
    if (lane == q) { up = t; act = k; }   // (the other equality rows' multipliers: not kept)
    GI_T0();
    add_row();
    GI_T1(1);
    ++q;
  }
  qe = q;
  if (lane < NX) sx[lane] = xi;
  __syncthreads();
  // ---- one-sided rows ----
  // the working one-sided rows as a bit set over p, wave-uniform, kept as rows join and leave
  // (was: rebuilt from the lanes' ids by a 64-lane OR butterfly every step; the same set)
  unsigned long long in_set = 0ull;
  while (ok) {
    if (++steps > kMaxSteps) { ok = false; break; }
    GI_T0();
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
      // (rmax: over the one-sided working rows -- the equality rows' rj are not computed)
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
        in_set |= 1ull << p;
        GI_T0();
        add_row();
        GI_T1(4);
#ifdef OSC_GI_PROFILE
        ++nadd;
#endif
        ++q;
        break;
      }
      {   // (kd: a one-sided row -- t1 only comes from those)
        const int kdu = __builtin_amdgcn_readfirstlane(kd);
        in_set &= ~(1ull << (__builtin_amdgcn_readlane(act, kdu) - kIneq));
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
    printf("gi env %d ok %d steps %d neq %d q %d adds %d drops %d cyc eqdir %llu eqadd %llu scan %llu dir %llu add %llu drop %llu rot %llu scan_cs %llu jc %llu z %llu bs %llu\n",
           env, ok ? 1 : 0, steps, neq, q, nadd, ndrop, tp[0], tp[1], tp[2], tp[3], tp[4], tp[5], tp[6], tp[7], tp[8], tp[9], tp[10]);
#endif
  if (!ok) return;
  // ---- certify: every equality row held, every one-sided row feasible, and every
  // working one-sided row's multiplier non-negative -- dual feasible in exact arithmetic, but
  // these envs carry multipliers of 1e7-3e8 and rows are dropped by absolute thresholds ----
  const double xs = wmax(lane < NX ? fabs(xi) : 0.0);
  const double umax = wmax((lane < q && act >= kIneq) ? fabs(up) : 0.0);
  double bad = 0.0;
  if (lane < q && act >= kIneq && !(up >= -1e-9 * (1.0 + umax))) bad = 1.0;
  if (lane < neq) {
    double s = -sEb[lane], cm = 0.0;
    for (int i = 0; i < NX; ++i) {
      s = fma(sE[lane * NXP + i], sx[i], s);
      cm = fmax(cm, fabs(sE[lane * NXP + i]));
    }
    // combined with the sign test above, never assigned over it: working one-sided rows sit at
    // lanes below neq whenever a dependent equality row was skipped
    if (!(fabs(s) / (1.0 + cm * xs + fabs(sEb[lane])) <= 1e-8)) bad = 1.0;   // (NaN: bad)
  }
  if (lane < NX && !isfinite(xi)) bad = 1.0;
  if (in_valid(lane) &&
      !(in_slack(lane) / (1.0 + in_scale(lane) * xs + fabs(in_rhs(lane))) >= -1e-9))
    bad = 1.0;
  if (!(wmax(bad) == 0.0) || !isfinite(xs)) return;
  if (gx != nullptr && lane < NX) gx[static_cast<size_t>(env) * NX + lane] = xi;
  if (lane >= NV && lane < NV + NU) gtau[static_cast<size_t>(env) * NU + lane - NV] = xi;
  if (lane == 0) {
    gstatus[env] = OSC_SOLVE_OK;
    // iters: -(the fallback's steps) marks an env this method solved (include/osc_batch.h)
    if (giters != nullptr) giters[env] = -steps;
    // the interior point's warm state of this env is the stalled iterate: the next tick starts
    // cold instead of paying the warm pass, the fix-up and the fallback again
    if (gwarm != nullptr) gwarm[static_cast<size_t>(env) * D::WW] = 0.0;
  }
}

template <class D>
void launch_gi(const LaunchArgs& a) {
  hipLaunchKernelGGL(osc_gi_kernel<D>, dim3(static_cast<unsigned>(a.nenv)), dim3(kWave), 0, a.s,
                     a.model->dparams, a.nenv, a.mask, a.ws, a.tau, a.x, a.status, a.iters,
                     a.warm);
}

template void launch_gi<WalterW>(const LaunchArgs&);

}  // namespace osc
