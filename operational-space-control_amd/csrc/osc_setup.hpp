// osc_setup.hpp -- kernel 1, the reduced QP per environment (osc_setup_kernel): the closed-form
// CasADi outputs H, f, Aeq, beq, Aineq, bineq of the reference (unitree_go2/autogen/autogen.py:
// 58-319, evaluated at unitree_go2/operational_space_controller.h:457-481) and the exact
// elimination of the dynamics rows onto y = (u, z).  Device code; included by
// osc_setup.hip and osc_multi.hip.
#pragma once
#include "osc_device.hpp"
#include "osc_kin_device.hpp"
#include "osc_wave_sum.hpp"

namespace osc {

// ============================ kernel 1: reduced QP per env ==================================
// Dense products of the assembly (H_dv X, X'(H_dv X), and 2 A'WA where it fits one tile) on the
// FP64 matrix cores (v_mfma_f64_16x16x4f64).
typedef double d4 __attribute__((ext_vector_type(4)));

// Sum over the 64 lanes, the same value on every lane (the shuffle butterfly's order, its
// partners by lane-crossing VALU ops: osc_wave_sum.hpp).
__device__ __forceinline__ double wave_sum(double v) { return wave_sum_fast(v); }

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
// profiles/r04za/.)  `scf`: nrows doubles of LDS scratch.  The shape is compile-time so the dot
// products' and the subtraction's LDS reads are issued ahead of their FMA chains (round 5: the
// runtime-bounded loops waited on every read, ~3.9k clocks per row pass, 58 % of the wheel
// model's assembly; the FMA order -- and so every result -- is unchanged).
template <int NROWS, int STRIDE, int NCOL, int NDOT>
__device__ __noinline__ void wave_mgs_lds(double* rows, int lane, double drop, double* scf) {
  const bool cv = lane < NCOL, dv = lane < NDOT;
  for (int w = 0; w < NROWS; ++w) {
    double aw = cv ? rows[w * STRIDE + lane] : 0.0;
    const double n0 = sqrt(wave_sum(dv ? aw * aw : 0.0));
    for (int pass = 0; pass < 2 && w > 0; ++pass) {
      double cf = 0.0;
      if (lane < w) {
        const double* rl = rows + lane * STRIDE;
        const double* rw = rows + w * STRIDE;
#pragma unroll
        for (int c = 0; c < NDOT; ++c) cf = fma(rl[c], rw[c], cf);
      }
      if (lane < w) scf[lane] = cf;
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
      if (cv) {
#pragma unroll 8
        for (int v = 0; v < w; ++v) aw = fma(-scf[v], rows[v * STRIDE + lane], aw);
        rows[w * STRIDE + lane] = aw;
      }
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
    }
    const double nn = sqrt(wave_sum(dv ? aw * aw : 0.0));
    const double sc = (nn > drop * n0 && nn > 0.0) ? 1.0 / nn : 0.0;
    if (cv) rows[w * STRIDE + lane] = aw * sc;
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
  }
}

// The body of one setup wavefront (env = its block index); `sm` is the block's D::SMEM doubles
// of LDS.  Wrapped by osc_setup_kernel (one model) and osc_setup_pair_kernel (two models, one
// grid: BASELINE configs[4]).
// KIN = true: the fused joint-state tick -- Phase A is the kinematics front end
// (osc_kin_device.hpp: the same arithmetic as osc_kinematics_kernel) for this env on all 64 lanes,
// from its qpos / qvel straight into the LDS layout Phase A would have staged M, C, J, b - t into
// (and, WaLTER, Phase B's J fragments into registers): M, C, J, b never go through HBM.  The
// kinematics' model tables and per-env state live in the region phases B-D use later (from
// D::O_HA), so the fused kernel needs kin_lds_doubles<D>() of LDS.
// LEAN = true (Go2's launches, osc_setup.hip): phase B's 2x2-tile loop unrolled 4 deep instead of
// fully -- 100 VGPRs instead of 256 -- and (kHaG below) only H_dv kept of Ha and X laid over A:
// 10.2 instead of 14.2 KB of LDS, so 16 waves fit a CU.  Round 5 adopted the unroll for batches
// past one round of interior-point waves only (4,096: 0.1646 vs 0.1620 ms, when LDS still capped
// a CU at 11 waves; profiles/r05/ab_setup_unroll4.jsonl); with the LDS cut it wins at every size
// (profiles/r06/lean_lds/).
template <class D, bool KIN = false, bool LEAN = false>
__device__ __forceinline__ void setup_env(
    const DevParams* __restrict__ P, int env, int nenv, const double* __restrict__ gM,
    const double* __restrict__ gC, const double* __restrict__ gJ, const double* __restrict__ gb,
    const double* __restrict__ gT, const double* __restrict__ gmask, double* __restrict__ ws,
    double* __restrict__ sm, const double* __restrict__ gwd,
    const osc_kin::KinDev* __restrict__ Kg = nullptr, const double* __restrict__ gqpos = nullptr,
    const double* __restrict__ gqvel = nullptr) {
  constexpr int NV = D::NV, NU = D::NU, NC = D::NC, NS = D::NS, NB = D::NB, NY = D::NY,
                NY1 = D::NY1, NY1P = D::NY1P, S = D::S, NA = D::NA;
  const int lane = threadIdx.x;
  if (env >= nenv) return;

  constexpr int NAP = D::NAP;
  double* sA = sm + D::O_A;
  double* sM = sm + D::O_M;
  double* sC = sm + D::O_C;
  // lean assembly without wheel rows: X over A, H_dv alone in LDS (osc_device.hpp Dims::SMEM_L)
  constexpr bool kHaG = LEAN && !D::WH && !KIN;
  double* sHa = sm + (kHaG ? D::O_HD_L : D::O_HA);
  double* sX = sm + (kHaG ? D::O_X_L : D::O_X);
  double* sU = sX + NB * NY1P;   // U parked in X's last rows until X replaces it
  double* sMask = sm + (kHaG ? D::O_MASK_L : D::O_MASK);

  STAMP_DECL
  STAMP_BEGIN();
  // ---------------- Phase A: stage this env's inputs HBM -> LDS ----------------
  // every load first (one memory latency), then the LDS stores
  static_assert(NV % 2 == 0 && NC % 2 == 0, "16-byte staging needs even nv and nc");
  constexpr int JC0 = 3 * (NS - NC);   // first contact translational row of J
  constexpr int JR0 = D::JG ? JC0 : 0; // first row of J staged (JG: the contact rows only)
  // JG: phase B's MFMA fragments of J (row 4q + (lane >> 4), column lane & 15)
  constexpr int KSJ = D::JG ? (S + 3) / 4 : 0;
  double jf[KSJ > 0 ? KSJ : 1];
  Batch2<NC / 2, kWave> bK;
  bK.load(gmask + static_cast<size_t>(env) * NC, lane);
  if constexpr (!KIN) {
    Batch2<D::JROWS * NV / 2, kWave> bJ;
    Batch2<NV * NV / 2, kWave> bM;
    Batch2<NV / 2, kWave> bC;
    bJ.load(gJ + static_cast<size_t>(env) * S * NV + JR0 * NV, lane);
    bM.load(gM + static_cast<size_t>(env) * NV * NV, lane);
    bC.load(gC + static_cast<size_t>(env) * NV, lane);
    // JG: phase B's MFMA fragments of J loaded now, in the same memory latency as the staging
    // loads; e and the row weights go to LDS
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
    if constexpr (D::WH) {
      // the fallback's raw rows (D::W_RM..W_RD): M, C, J's contact rows from the staged registers,
      // b's contact rows and the wheel directions straight from global
      double* wr = ws + static_cast<size_t>(env) * D::WS;
      bM.store(wr + D::W_RM, lane);
      bC.store(wr + D::W_RC, lane);
      bJ.store(wr + D::W_RJ, lane);   // (JG: bJ holds exactly the 3 NC contact rows)
      static_assert(D::JG && D::JROWS == 3 * NC, "wheel rows: the contact rows are the staged ones");
      for (int q = lane; q < 3 * NC; q += kWave) wr[D::W_RB + q] = gb[static_cast<size_t>(env) * S + JC0 + q];
      for (int q = lane; q < 6 * NC; q += kWave) wr[D::W_RD + q] = gwd[static_cast<size_t>(env) * NC * 6 + q];
    }
#pragma unroll
    for (int q = 0; q < TE; ++q) {   // lanes past S rewrite row S-1 with its own value (no branch)
      const int r = (lane + q * kWave < S) ? lane + q * kWave : S - 1;
      sA[r * NAP + NV] = eb[q] - et[q];
      if (NAP > NA) sA[r * NAP + NA] = 0.0;
    }
    wave_sync();
  } else {
    // the model tables, then this env's state, in the region phases B-D use later (the mask's
    // LDS slot lies inside it: stored once the kinematics is done)
    osc_kin::KinDev* sK = reinterpret_cast<osc_kin::KinDev*>(sm + D::O_HA);
    {
      static_assert(sizeof(osc_kin::KinDev) % 16 == 0 && D::O_HA % 2 == 0, "16-byte staging");
      const uint4* src = reinterpret_cast<const uint4*>(Kg);
      uint4* dst = reinterpret_cast<uint4*>(sK);
      for (int i = lane; i < static_cast<int>(sizeof(osc_kin::KinDev) / 16); i += kWave)
        dst[i] = src[i];
    }
    wave_sync();
    const osc_kin::KinDev* K = sK;
    const int nq = K->nq;
    const osc_kin::EnvLayout lay(nq, NV, K->nbody, NS);
    double* E = sm + D::O_HA + sizeof(osc_kin::KinDev) / 8;
    for (int i = lane; i < nq; i += kWave) E[lay.q + i] = gqpos[static_cast<size_t>(env) * nq + i];
    for (int i = lane; i < NV; i += kWave) E[lay.q + nq + i] = gqvel[static_cast<size_t>(env) * NV + i];
    wave_sync();
    osc_kin::kin_forward(K, E, lay, lane);    // (lane = body; the tree's levels)
    osc_kin::kin_backward(K, E, lay, lane);
    for (int d = lane; d < NV; d += kWave) sC[d] = osc_kin::kin_dof(K, E, lay, d);
    // sites: position, J-dot qvel -> A's column NV = b - t (JG: the e vector), the row weights
    double* wr = ws + static_cast<size_t>(env) * D::WS;
    for (int k = lane; k < NS; k += kWave) {
      double bp[3], br[3];
      osc_kin::kin_site(K, E, lay, k, bp, br);
      const double* Tk = gT + static_cast<size_t>(env) * NS * 6 + k * 6;
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const int rp = 3 * k + i, rr = 3 * NS + 3 * k + i;
        if constexpr (D::JG) {
          sA[D::O_E + rp] = bp[i] - Tk[i];
          sA[D::O_E + rr] = br[i] - Tk[3 + i];
        } else {
          sA[rp * NAP + NV] = bp[i] - Tk[i];
          sA[rr * NAP + NV] = br[i] - Tk[3 + i];
          if (NAP > NA) {
            sA[rp * NAP + NA] = 0.0;
            sA[rr * NAP + NA] = 0.0;
          }
        }
        if constexpr (D::WH) {   // the fallback's raw b rows (contact sites)
          if (k >= NS - NC) wr[D::W_RB + 3 * (k - (NS - NC)) + i] = bp[i];
        }
      }
    }
    if constexpr (D::JG) {
      for (int r = lane; r < S; r += kWave) sA[D::O_W + r] = P->w_row[r];
    }
    wave_sync();
    // M (lane = column j, rows of one parity per half-wave) and J (lane = column c, sites of one
    // parity per half-wave) from the dofs' S, F
    {
      const int j = lane & 31, par = lane >> 5;
      const bool vj = j < NV;
      const double* Dj = E + lay.dof + osc_kin::kDofStride * (vj ? j : 0);
      double Sj[6], Fj[6];
#pragma unroll
      for (int t = 0; t < 6; ++t) {
        Sj[t] = Dj[t];
        Fj[t] = Dj[6 + t];
      }
      for (int i = par; i < NV; i += 2) {
        const double* Di = E + lay.dof + osc_kin::kDofStride * i;
        double Si[6], Fi[6];
#pragma unroll
        for (int t = 0; t < 6; ++t) {
          Si[t] = Di[t];
          Fi[t] = Di[6 + t];
        }
        const double m = osc_kin::kin_m_entry(K->dof_relmask[i], K->dof_arm[i], i, j, Si, Fi, Sj, Fj);
        if (vj) sM[i * NV + j] = m;
      }
      // J rows in A (JG: only the contact sites' translational rows, which phase C reads)
      for (int k = (D::JG ? NS - NC : 0) + par; k < NS; k += 2) {
        const double* xs = E + lay.site + 3 * k;
        const double xk[3] = {xs[0], xs[1], xs[2]};
        double jp[3], jr[3];
        osc_kin::kin_j_col(vj && ((K->site_dofmask[k] >> j) & 1u), Sj, xk, jp, jr);
        if (vj) {
#pragma unroll
          for (int t = 0; t < 3; ++t) {
            sA[(3 * k + t - JR0) * NAP + j] = jp[t];
            if (!D::JG) sA[(3 * NS + 3 * k + t) * NAP + j] = jr[t];
          }
        }
      }
      if constexpr (D::JG) {
        // phase B's fragments: J[4q + (lane >> 4)][lane & 15] (rows past S: row S-1; columns past
        // NV: column 0 -- as the staged loads read them)
        const int lc = lane & 15, lg = lane >> 4;
        const int c = lc < NV ? lc : 0;
        const double* Dc = E + lay.dof + osc_kin::kDofStride * c;
        double Sc[6];
#pragma unroll
        for (int t = 0; t < 6; ++t) Sc[t] = Dc[t];
#pragma unroll
        for (int q = 0; q < KSJ; ++q) {
          const int r0 = 4 * q + lg, r = r0 < S ? r0 : S - 1;
          const int half = r / (3 * NS), rr = r % (3 * NS), k = rr / 3, t = rr % 3;
          const double* xs = E + lay.site + 3 * k;
          const double xk[3] = {xs[0], xs[1], xs[2]};
          double jp[3], jr[3];
          osc_kin::kin_j_col((K->site_dofmask[k] >> c) & 1u, Sc, xk, jp, jr);
          jf[q] = half ? jr[t] : jp[t];
        }
      }
    }
    wave_sync();
    bK.store(sMask, lane);
    wave_sync();
    if constexpr (D::WH) {
      // the fallback's raw rows (D::W_RM..): M, C, J's contact rows from LDS, the directions
      for (int q = lane; q < NV * NV; q += kWave) wr[D::W_RM + q] = sM[q];
      for (int q = lane; q < NV; q += kWave) wr[D::W_RC + q] = sC[q];
      for (int q = lane; q < 3 * NC * NV; q += kWave)
        wr[D::W_RJ + q] = sA[(q / NV) * NAP + q % NV];   // (JG: A holds exactly the contact rows)
      for (int q = lane; q < 6 * NC; q += kWave) wr[D::W_RD + q] = gwd[static_cast<size_t>(env) * NC * 6 + q];
    }
  }

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
    if constexpr (kHaG) {   // H_dv alone, row stride NV
      if (j < NV) {
        sHa[i * NV + j] = v;
        sHa[j * NV + i] = v;
      }
    } else {
      sHa[i * NA + j] = v;
      sHa[j * NA + i] = v;
    }
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
    auto ha_row = [&](int r) {
      const double2 x = *reinterpret_cast<const double2*>(sA + r * NAP + i0);
      const double2 y = *reinterpret_cast<const double2*>(sA + r * NAP + j0);
      const double w = P->w_row[r];
      const double wx0 = w * x.x, wx1 = w * x.y;
      a00 = fma(wx0, y.x, a00);
      a01 = fma(wx0, y.y, a01);
      a10 = fma(wx1, y.x, a10);
      a11 = fma(wx1, y.y, a11);
    };
    if constexpr (LEAN) {
#pragma unroll 4
      for (int r = 0; r < S; ++r) ha_row(r);
    } else {
      for (int r = 0; r < S; ++r) ha_row(r);   // (fully unrolled by the compiler)
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
  // kHaG: every lane computes its column in registers first and stores it after one barrier -- the
  // lean assembly's X region overlays A, whose contact rows the columns read.  (The other variants
  // store as they go: computing first measured 1.6 % slower for WaLTER at 65,536.)
  double x[NB];
  double uacc[kUStep];
#pragma unroll
  for (int i = 0; i < NB; ++i) x[i] = 0.0;
#pragma unroll
  for (int t = 0; t < kUStep; ++t) uacc[t] = 0.0;
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
      // a pivot <= 0: M is not positive definite (no mass matrix is) -- NaN poisons X, so the
      // env comes back OSC_SOLVE_NUMERICAL instead of an interior point on a meaningless reduction
      dinv[k] = L[k][k] > 0.0 ? recip1(L[k][k]) : __builtin_nan("");
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
    if (!kHaG && a_lo == 0) {
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
        if constexpr (kHaG) uacc[t] = acc;
        else sU[a * NY1P + c] = acc;
      }
    }
  }
  if constexpr (kHaG) wave_sync();   // A's contact rows are read: X may overwrite them now
  // (kHaG: every column; otherwise the padding columns of X and U -- read by the 2x2 tiles -- get
  // their zeros)
  if (kHaG ? c < NY1P : (c >= NY1 && c < NY1P)) {
    if (a_lo == 0) {
#pragma unroll
      for (int i = 0; i < NB; ++i) sX[i * NY1P + c] = x[i];
    }
#pragma unroll
    for (int t = 0; t < kUStep; ++t)
      if (a_lo + t < NU) sU[(a_lo + t) * NY1P + c] = uacc[t];
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
      const double pk = bcast_guarded<k>(col[k]);
      const double rk = pk > 0.0 ? recip1(pk) : __builtin_nan("");   // 1 / S_k[k][k] (M SPD)
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
    STAMP_END(9);
    STAMP_BEGIN();
    // 4. T: an orthonormal basis of the y space whose first r' columns are Q's (nonzero) rows and
    //    the rest span their null space (Gram-Schmidt of [Q; I]).  The interior point and the
    //    refinement solve their Newton systems in y^ = T'y with the rows' coordinates pinned:
    //    the rows hold exactly, and nothing of the Hessian's curvature along them enters the
    //    factorisation.  X^ = X'T replaces X, so [Hr | g] below come out in these
    //    coordinates.
    // (rows at an odd stride: the Gram-Schmidt's dot products read one row per lane, and at a stride
    // of 32 doubles every lane's read hit the same LDS bank -- 58 % of the wheel assembly's time)
    constexpr int TS = D::WTST;
    double* sWT = sm + D::O_WT;
    for (int p = lane; p < (NW + NY) * NY; p += kWave) {
      const int w = p / NY, c = p % NY;
      sWT[w * TS + c] = (w < NW) ? sWA[w * WAST + c] : ((c == w - NW) ? 1.0 : 0.0);
    }
    wave_sync();
    wave_mgs_lds<NW + NY, TS, NY, NY>(sWT, lane, 1e-9, sWE);   // (sWE: copied out above, free)
    wave_sync();
    int kept = 0;
    for (int w = 0; w < NW + NY; ++w) {
      const double a = lane < NY ? sWT[w * TS + lane] : 0.0;
      if (wave_sum(a * a) > 0.0) {   // wave-uniform
        if (kept < NY) {
          if (lane < NY) sWT[kept * TS + lane] = a;   // in place: kept <= w
          if (lane == 0) wsw[D::W_PIN + kept] = (w < NW) ? static_cast<double>(w) : -1.0;
        }
        ++kept;
      }
      wave_sync();
    }
    for (int k = kept; k < NY; ++k) {   // (never in practice: a column short -> pinned at zero)
      if (lane < NY) sWT[k * TS + lane] = 0.0;
      if (lane == 0) wsw[D::W_PIN + k] = -2.0;
    }
    wave_sync();
    for (int p = lane; p < NY * NY; p += kWave) {
      const int i = p / NY, k = p % NY;
      wsw[D::W_T + p] = sWT[k * TS + i];   // T[i][k]
    }
    STAMP_END(10);
    STAMP_BEGIN();
    // X^ = X'T (y columns; the affine column stays), staged in sWE (free now)
    for (int p = lane; p < NV * NY; p += kWave) {
      const int j = p / NY, k = p % NY;
      double v = 0.0;
#pragma unroll 8
      for (int i = 0; i < NY; ++i) v = fma(sX[j * NY1P + i], sWT[k * TS + i], v);
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
  // (kHaG: f_dv comes back from the workspace -- this wavefront's own stores of phase B, complete
  // and visible to its loads after a workgroup-scope fence)
  if constexpr (kHaG) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
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
        const int hr = row < NV ? row : 0, hk = kv ? k : 0;
        const double h = sHa[hr * (kHaG ? NV : NA) + hk];
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
          const double f = kHaG ? wha[D::W_GD + (row < NV ? row : 0)]
                                : sHa[(row < NV ? row : 0) * NA + NV];
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
    // Hr[a][b] = Hr[b][a] = v (a <= b) in the workspace's Hr layout (hr_off: compact without wheel
    // rows -- rows 16.. whole, the leading 16 x 16 block as a packed triangle)
    auto store_hr = [&](int a, int b, double v) {
      if constexpr (!D::HRC) {
        wsv[D::W_HR + a * NY + b] = v;
        wsv[D::W_HR + b * NY + a] = v;
      } else if (b >= kRow) {
        wsv[D::W_HR + hr_off<D>(b, a)] = v;                       // row b of A
        if (a >= kRow && a != b) wsv[D::W_HR + hr_off<D>(a, b)] = v;   // row a of A
      } else {
        wsv[D::W_HR + hr_off<D>(a, b)] = v;                       // the triangle
      }
    };
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
                wab = fma(wi * sT[a * D::WTST + i], sT[b * D::WTST + i], wab);
              }
              v += wab;
              store_hr(a, b, v);
            } else if (b < NY) {
              if (a == b && a < NU) v += wu2;
              if (a == b && a >= NU) v = (mk == 0.0) ? 1.0 : v + wr2;   // pinned z: identity row
              store_hr(a, b, v);
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
// (waves per SIMD of the launch bound; -DOSC_SETUP_WPS=3 for A/B builds: 168 VGPRs + 436 B of
// spills, Go2 4,096 0.166 -> 0.226 ms per solve, profiles/r05/r05wps_*)
#ifndef OSC_SETUP_WPS
#define OSC_SETUP_WPS 2
#endif
#ifndef OSC_SETUP_LEAN_WPS
#define OSC_SETUP_LEAN_WPS 4
#endif
template <class D, bool LEAN = false>
__global__ __launch_bounds__(kWave, LEAN ? OSC_SETUP_LEAN_WPS : OSC_SETUP_WPS) void osc_setup_kernel(
    const DevParams* __restrict__ P, int nenv, const double* __restrict__ gM,
    const double* __restrict__ gC, const double* __restrict__ gJ, const double* __restrict__ gb,
    const double* __restrict__ gT, const double* __restrict__ gmask, double* __restrict__ ws,
    const double* __restrict__ gwd) {
  __shared__ __attribute__((aligned(16))) double sm[(LEAN && !D::WH) ? D::SMEM_L : D::SMEM];
  setup_env<D, false, LEAN>(P, static_cast<int>(blockIdx.x), nenv, gM, gC, gJ, gb, gT, gmask, ws,
                            sm, gwd);
}

// The fused joint-state tick's assembly (setup_env<D, true>): kinematics from qpos / qvel in the
// prologue.  LDS: kin_lds_doubles(...) doubles, dynamic (the kinematics' per-env state depends on
// the tree).
extern __shared__ __attribute__((aligned(16))) double osc_setup_qpos_sm[];
template <class D>
__global__ __launch_bounds__(kWave, 2) void osc_setup_qpos_kernel(
    const DevParams* __restrict__ P, int nenv, const osc_kin::KinDev* __restrict__ Kg,
    const double* __restrict__ gqpos, const double* __restrict__ gqvel,
    const double* __restrict__ gT, const double* __restrict__ gmask, double* __restrict__ ws,
    const double* __restrict__ gwd) {
  setup_env<D, true>(P, static_cast<int>(blockIdx.x), nenv, nullptr, nullptr, nullptr, nullptr, gT,
                     gmask, ws, osc_setup_qpos_sm, gwd, Kg, gqpos, gqvel);
}
template <class D>
inline int kin_lds_doubles(int nq, int nbody) {
  const int kin = D::O_HA + static_cast<int>(sizeof(osc_kin::KinDev) / 8) +
                  osc_kin::EnvLayout(nq, D::NV, nbody, D::NS).size;
  return kin > D::SMEM ? kin : D::SMEM;
}

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

}  // namespace osc
