// osc_ipm.hpp -- kernel 2, the batched interior point + full-space refinement (osc_ipm_kernel,
// osc_ipm_compact_kernel, osc_refine_kernel, osc_ipm_pair_kernel): the reference's OSQP solve
// (unitree_go2/operational_space_controller.h:483-536) on the reduced QP, four environments per
// wavefront, and launch_ipm, the pass sequence of one call.  Device code +
// the launcher template; instantiated once per robot model (osc_ipm_go2.hip, osc_ipm_walter.hip,
// osc_ipm_wheels.hip) so the three compile in parallel.
#pragma once
#include "osc_internal.hpp"
#include "osc_ipm_asm.hpp"

namespace osc {

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
  if constexpr (N == 24 || N == 32) {       // one asm statement (osc_ipm_asm.hpp): no s_nop per pair
    dot_rows_asm<N>(a, b, a2, b2, x0, x1, ma, mb);
    a += a2;
    b += b2;
    return;
  }
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
// ASM: the scheduled one-statement form (osc_ipm_asm.hpp) -- it claims 12 VGPRs of its own, which
// the one-wave kernels (512 registers with the AGPRs) have to spare and the two-wave ones do not
// (their spills grow 12 -> 52 bytes per lane), so those keep the per-pivot form.
// du: the torque rows' diagonal terms of G'DG (lane q's column q < NU, 0 on the other lanes),
// added to each pivot where it is taken (round 6: the diagonal of K enters the factorisation only
// as its pivots, so the same K as adding du to c0[l] up front -- which took a lane select per torque
// column every iteration -- up to the rounding of the pivots' sums)
// An empty asm that "rewrites" columns I.. of both slots (ldl_rows: orders their last VALU writes)
template <int I, int N>
__device__ __forceinline__ void touch_cols(double (&c0)[N], double (&c1)[N]) {
  asm volatile("" : "+v"(c0[I]), "+v"(c1[I]));
  if constexpr (I + 1 < N) touch_cols<I + 1, N>(c0, c1);
}
template <int N, bool ASM = true>
__device__ __forceinline__ void ldl_rows(double (&c0)[N], double (&c1)[N], double* sdinv, int l,
                                         double& dinv0, double& dinv1, double thr0, double thr1,
                                         double du) {
  // pivot k's preparation: -> (t0, t1) = -L[lane][k] for the lanes still to be eliminated
  auto prep = [&](auto kc, double& t0, double& t1) {
    constexpr int k = decltype(kc)::value;
    constexpr int s = k / kRow, kl = k % kRow;
    const double own = (s == 0) ? c0[k] + du : c1[k];
    const double dk = bcast_guarded<kl>(own > ((s == 0) ? thr0 : thr1) ? own : 1e128);
    const double inv = recip1(dk);
    sdinv[k] = inv;
    c0[k] = -c0[k] * inv;
    c1[k] = -c1[k] * inv;
    // (lanes l > k by a compare on the lane index, osc_device.hpp keep_gt; in slot 1 the mirror
    // lanes past N keep their multipliers too and so stay exact copies of column N - 1)
    t0 = keep_gt<k>(l, c0[k]);
    if constexpr (k < kRow) t1 = c1[k];
    else t1 = keep_gt<k - kRow>(l, c1[k]);
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
  if constexpr (ASM && (N == 24 || N == 32)) {
    // one scheduled asm statement (tools/gen_ipm_asm.py -> osc_ipm_asm.hpp): the same
    // instructions on the same values, pivot k+1's preparation interleaved with pivot k's FMAs
    // so that the FMAs are the wait states (no s_nop, no asm-boundary padding)
    const unsigned addr = static_cast<unsigned>(
        reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) double*)sdinv));
    ldl_asm<N>(c0, c1, thr0, thr1, l, addr, du);
    wave_sync();
    dinv0 = sdinv[l];
    dinv1 = sdinv[(l + kRow < N) ? l + kRow : N - 1];
    return;
  }
  // Step 0's DPP reads take columns the caller's C++ just wrote (K = Hr + G'DG): every column goes
  // through an empty asm first and then one s_nop 1, so no schedule can put a column's VALU write
  // within the DPP read's two wait states (tests/test_asm_hazards.py; LLVM's ILP scheduler did).
  touch_cols<0, N>(c0, c1);
  asm volatile("s_nop 1");
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
  if constexpr (N == 24 || N == 32) {       // one asm statement (osc_ipm_asm.hpp), bitwise the same
    ldl_fwd_asm<N>(c0, c1, a0, a1, z0, z1, l);
    a0 = z0;
    a1 = z1;
    return;
  }
  static_for<0, N>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    constexpr int s = k / kRow, kl = k % kRow;
    if constexpr (s == 0) {
      z0 = sel_eq<kl>(l, a0, z0);   // (its three VALU instructions: the DPP read's wait states)
      const double p = a0;
      fmac_bcast<kl>(a1, p, c1[k]);
      if constexpr (k < kRow - 1) fmac_bcast<kl>(a0, p, c0[k]);
    } else {
      z1 = sel_eq<kl>(l, a1, z1);
      const double p = a1;
      fmac_bcast<kl>(a1, p, c1[k]);
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
  if constexpr (N == 24 || N == 32) {
    ldl_bwd_asm<N>(c0, c1, a0, a1, x0, x1, l);
    a0 = x0 * dinv0;
    a1 = x1 * dinv1;
    return;
  }
  static_for<0, N>([&](auto kc) {
    constexpr int k = N - 1 - decltype(kc)::value;
    constexpr int s = k / kRow, kl = k % kRow;
    if constexpr (s == 0) {
      x0 = sel_eq<kl>(l, a0, x0);
      const double p = a0;
      if constexpr (k >= 1) fmac_bcast<kl>(a0, p, c0[k]);
    } else {
      x1 = sel_eq<kl>(l, a1, x1);
      const double p = a1;
      fmac_bcast<kl>(a0, p, c0[k]);
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
// (kRefineRounds, kRefineMaxSteps: osc_device.hpp -- the host clamps refine_steps to the latter)
template <class D, bool SMALL, int RF>
constexpr bool ipm_hrl() {   // Hr kept in LDS across the interior point's iterations
  return SMALL && RF != kRfOnly && hr_fits_lds<D>();
}
// Two-wave variant (round 6): Hr's first column slot -- columns 0..15, every row
// (NY x 16 doubles per env) -- is staged into LDS once per solve, and only the second slot's
// columns are read from the workspace each iteration, as ROWS 16..NY-1 of Hr (Hr is stored exactly
// symmetric, so row j = column j bitwise): per-lane contiguous 16-byte loads over a contiguous
// (NY - 16) x NY block.  At 8,192 Go2 envs every Hr re-read used to miss L2 (37.7 MB of Hr against
// 8 x 4 MB of L2: 7x the algorithmic bytes); the streamed part is now 1.5 KB per env (12 MB).
// LDS: 246 + 384 doubles per env, 20.2 KB per wave -- eight waves per CU in 160 KB.
template <class D, bool SMALL, int RF>
constexpr bool ipm_hrh() {
  return !SMALL && !D::WH && RF != kRfOnly && D::NY > kRow &&
         (IpmLayout<D, false>::IL + D::NY * kRow) * 8 * kEnvPerWave * 8 <= 160 * 1024;
}
template <class D, bool SMALL, int RF>
constexpr int hrh_lds_extra() { return ipm_hrh<D, SMALL, RF>() ? D::NY * kRow : 0; }
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
  constexpr int il = IpmLayout<D, ipm_hrl<D, SMALL, RF>()>::IL + refine_lds_extra<D, SMALL, RF>() +
                     hrh_lds_extra<D, SMALL, RF>();
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
  // the refinement fused: a cold solve is followed by its own fix-up pass too (osc_ipm_kernel)
  constexpr bool kFix = WARM || RF_ == kRfFused;
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
  if constexpr (kFix) {
    // (an env whose refinement found no KKT point, OSC_SOLVE_UNREFINED, too: the warm start can
    // leave the interior point's early stop with an active set the refinement cannot repair,
    // ~1 env in 4,096 x 10 joint-state ticks; the cold fix-up solve runs to mu <= 1e-12)
    const bool redo = valid && fixup && gstatus[env] != OSC_SOLVE_OK;
    if (fixup && __ballot(redo) == 0) return;
    write_out = valid && (!fixup || redo);
  }

  constexpr bool HRH = ipm_hrh<D, SMALL, RF>();
  constexpr int kEnvLds = LY::IL + refine_lds_extra<D, SMALL, RF>() + hrh_lds_extra<D, SMALL, RF>();
  double* B = sm + grp * kEnvLds;
  double* sHh = B + LY::IL + refine_lds_extra<D, SMALL, RF>();   // HRH: Hr[i][0..15] at i * 16
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
  if constexpr (HRL && D::HRC) {   // the workspace's compact Hr -> its full LDS layout, once
    const int ca = l, cb = l + kRow < NY ? l + kRow : NY - 1;   // this lane's two columns
    // fused refinement: the compact block is copied whole (16-byte loads) into the refinement's
    // LDS region -- free until the [H_dv | f_dv] DMA of the refinement -- and expanded from there
    // (per-lane addresses into LDS, not into L2); otherwise read from the workspace directly
    const double* src = wsw + lane_off;
    if constexpr (kXinHr) {
      static_assert(D::HR_SIZE % 2 == 0 && D::HR_SIZE <= refine_lds_extra<D, SMALL, RF>() &&
                    D::W_HR % 2 == 0, "compact Hr staged in the refinement region");
      Batch2<D::HR_SIZE / 2, kRow> bh;
      bh.load(ws + static_cast<size_t>(env) * D::WS + D::W_HR, l);
      bh.store(B + LY::IL, l);
      wave_sync();
      src = B + LY::IL;
    }
#pragma unroll
    for (int i0 = 0; i0 < NY; i0 += 8) {
      double hv0[8], hv1[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        hv0[i] = i0 + i < NY ? src[hr_off<D>(i0 + i, ca)] : 0.0;
        hv1[i] = i0 + i < NY ? src[hr_off<D>(i0 + i, cb)] : 0.0;
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if (i0 + i < NY) {
          const_cast<double*>(sHr)[(i0 + i) * NY + ca] = hv0[i];
          if (l + kRow < NY) const_cast<double*>(sHr)[(i0 + i) * NY + cb] = hv1[i];
        }
      }
    }
  }
  if constexpr (HRH) {   // Hr's first column slot, once per solve
    static_assert(NY % 2 == 0 && D::WS % 2 == 0 && D::W_HR % 2 == 0, "16-byte Hr row loads");
#pragma unroll
    for (int i0 = 0; i0 < NY; i0 += 8) {   // (eight loads in flight: few registers live here)
      double hv[8];
#pragma unroll
      for (int i = 0; i < 8; ++i)
        hv[i] = i0 + i < NY ? wsw[lane_off + static_cast<unsigned>(hr_off<D>(i0 + i, l))] : 0.0;
#pragma unroll
      for (int i = 0; i < 8; ++i)
        if (i0 + i < NY) sHh[(i0 + i) * kRow + l] = hv[i];
    }
  }
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
  // G'DG's contact blocks into K's columns (c0 / c1), row by row (round 6): the rows of contact k
  // are NU + 3k .. NU + 3k + 2, and the lanes whose column lies in contact k form a compile-time lane
  // range of each slot -- so each row takes its entry (a, b or cc by the row's component) masked
  // to that range, and rows no lane of a slot reaches are not touched.  (It was a select per row
  // of all 12 contact rows against the lane's runtime contact index, behind a branch per slot.)
  auto add_contact_blocks = [&](double& dg0, double& dg1) __attribute__((always_inline)) {
    double a0, b0, e0, a1, b1, e1;
    contact_col(jk0 >= 0 ? jk0 : 0, jc0, a0, b0, e0);
    contact_col(jk1 >= 0 ? jk1 : 0, jc1, a1, b1, e1);
    dg0 += jk0 >= 0 ? ((jc0 == 0) ? a0 : (jc0 == 1) ? b0 : e0) : 0.0;
    dg1 += jk1 >= 0 ? ((jc1 == 0) ? a1 : (jc1 == 1) ? b1 : e1) : 0.0;
    static_for<0, NC>([&](auto Kc) __attribute__((always_inline)) {
      constexpr int k = decltype(Kc)::value, r0 = NU + 3 * k;
      constexpr unsigned m0 = r0 <= kRow - 1 ? lanes_from(r0, r0 + 2) : 0u;   // slot 0: lane = row
      constexpr unsigned m1 = lanes_from(r0 - kRow, r0 + 2 - kRow);           // slot 1: row - 16
      if constexpr (m0 != 0u) {
        const unsigned long long m = mask_here<rows_mask(m0)>();
        c0[r0] += keep_m(m, a0);
        c0[r0 + 1] += keep_m(m, b0);
        c0[r0 + 2] += keep_m(m, e0);
      }
      if constexpr (m1 != 0u) {
        const unsigned long long m = mask_here<rows_mask(m1)>();
        c1[r0] += keep_m(m, a1);
        c1[r0 + 1] += keep_m(m, b1);
        c1[r0 + 2] += keep_m(m, e1);
      }
    });
  };
  // WH: c0 / c1 hold H^'s columns j0, jj1; add T'(G'DG)T from sDr (D per row slot) one original
  // coordinate i at a time -- column j gains coef_i(j) T[i][:], coef_i(j) = (G'DG)[i][:] T[:][j]
  // (torque rows: diagonal; a contact's rows: its 3 x 3 block) -- then pin Q's coordinates.
  // Returns the assembled diagonal entries (the pivot threshold's reference).
  auto assemble_rot = [&](double& dg0r, double& dg1r) __attribute__((always_inline)) {
    if constexpr (WHR) {
      // K^ columns j0, jj1 += T' (B T)[:, j] with B = G'DG (diagonal on u, a 3 x 3 block per
      // contact), one row i of T at a time: a = (B T)[i, j] from the lane's own entries of T, then
      // c[m] += a T[i][m] with T[i][m] broadcast from the lane that owns column m
      // (v_fmac_f64_dpp row_newbcast) -- each lane reads its own two entries of row i instead of
      // the whole row from LDS (the per-iteration product of the wheel rows: NY^3 per env)
      auto rank1 = [&](double a0, double a1, double t0, double t1) __attribute__((always_inline)) {
        static_for<0, kRow>([&](auto K) __attribute__((always_inline)) {
          constexpr int k = decltype(K)::value;
          if constexpr (k < NY) {
            fmac_bcast<k, k == 0>(c0[k], t0, a0);
            fmac_bcast<k>(c1[k], t0, a1);
          }
          if constexpr (k + kRow < NY) {
            fmac_bcast<k, k == 0>(c0[k + kRow], t1, a0);
            fmac_bcast<k>(c1[k + kRow], t1, a1);
          }
        });
      };
#pragma unroll
      for (int i = 0; i < NU; ++i) {
        const double d = sDr[2 * i] + sDr[2 * i + 1];
        const double t0 = sWT[i * WL::TST + j0], t1 = sWT[i * WL::TST + jj1];
        rank1(d * t0, d * t1, t0, t1);
      }
      static_for<0, NC>([&](auto Kc) __attribute__((always_inline)) {
        constexpr int k = decltype(Kc)::value, zb = NU + 3 * k;
        double t0r[3], t1r[3];
#pragma unroll
        for (int r = 0; r < 3; ++r) {
          t0r[r] = sWT[(zb + r) * WL::TST + j0];
          t1r[r] = sWT[(zb + r) * WL::TST + jj1];
        }
        static_for<0, 3>([&](auto Ci) __attribute__((always_inline)) {
          constexpr int ci = decltype(Ci)::value;
          double b0, b1, b2;   // row ci of contact k's block (symmetric: its column ci)
          contact_col(k, ci, b0, b1, b2);
          const double a0 = b0 * t0r[0] + b1 * t0r[1] + b2 * t0r[2];
          const double a1 = b0 * t1r[0] + b1 * t1r[1] + b2 * t1r[2];
          rank1(a0, a1, t0r[ci], t1r[ci]);
        });
      });
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
      hr0[i] = wsw[lane_off + static_cast<unsigned>(hr_off<D>(i, j0))];
      hr1[i] = wsw[lane_off + static_cast<unsigned>(hr_off<D>(i, jj1))];
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
    } else if constexpr (HRH) {
      unsigned off = lane_off;
      asm volatile("" : "+v"(off));
      // column jj1 = row jj1: this lane's contiguous NY doubles, two per 16-byte load
      const double* p1 = wsw + off + hr_off<D>(jj1, 0);   // (row jj1 of A when compact)
#pragma unroll
      for (int i = 0; i < NY; ++i) c1[i] = p1[i];
#pragma unroll
      for (int i = 0; i < NY; ++i) c0[i] = sHh[i * kRow + l];
    } else {
      unsigned off = lane_off;
      asm volatile("" : "+v"(off));
      const double* p = wsw + off;
#pragma unroll
      for (int i = 0; i < NY; ++i) {
        c0[i] = p[hr_off<D>(i, j0)];
        c1[i] = p[hr_off<D>(i, jj1)];
      }
    }
  };
  const double hdg0 =
      HRL ? sHr[j0 * NY + j0] : wsw[lane_off + static_cast<unsigned>(hr_off<D>(j0, j0))];
  const double hdg1 =
      HRL ? sHr[jj1 * NY + jj1] : wsw[lane_off + static_cast<unsigned>(hr_off<D>(jj1, jj1))];
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
  // The dual residual rd = Hr y + g + G'lam is carried the same way (round 6): with the Newton
  // system K dy = G'w - rd solved, Hr dy + G'dlam = G'w - rd - G'DG dy + G'(-w + DG dy) = -rd,
  // so the step leaves (1 - alpha) rd -- up to the solve's rounding, which is why it is formed
  // from scratch (Hr y by DPP broadcasts, G'lam from LDS: 8 % of an iteration) whenever rp is:
  // at iteration 0, after a re-centring and once mu <= 1e-6.  Per env (an env's rd never depends
  // on its wave-mates'); a wave forms it only when one of its running envs needs it.  (Not with
  // wheel rows: their rd lives in rotated coordinates.)
  constexpr bool kRdCarry = !D::WH;
  double rdc0 = 0.0, rdc1 = 0.0;
  bool rd_fresh = true, rd_have = false;   // (rd_have: a compaction's resume pass starts mid-solve)
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
      rdc0 = pk[2 * kRow + 3 * NRL * kRow + l];
      rdc1 = pk[3 * kRow + 3 * NRL * kRow + l];
      rd_have = true;
      sVy[j0] = y0;
      if (v1) sVy[j1] = y1;
      wave_sync();
    }
    return PA.park_it;
  };
  bool parked = false;   // park pass: this row's env went to the park area (no outputs here)
  bool refined = false;
  // WH with the duals requested: the wheel rows' multipliers (W_NU; the refinement's where it is
  // kept, else the interior point's centre) -- a diagnostic of the workspace since round 4: the
  // dual kernel recovers every multiplier, the wheel rows' included, from the design vector.
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
  const double eps_run = (kFix && fixup) ? fmin(P->eps_mu, 1e-12) : P->eps_mu;
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
      rd_fresh = fresh || !rd_have;
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
            pk[2 * kRow + 3 * NRL * kRow + l] = rdc0;
            pk[3 * kRow + 3 * NRL * kRow + l] = rdc1;
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
    double rd0 = rdc0, rd1 = rdc1;
    if (!kRdCarry || init || __ballot(rd_fresh && !done) != 0) {   // (wave-uniform)
      double rn0, rn1;
      GTw2(sVr, rn0, rn1);
      if constexpr (WHR) rot_in(rn0, rn1, rn0, rn1);   // T'G'lam
      rn0 += g0;
      rn1 += g1;
      if constexpr (WHR) {   // rd^ += H^ y^
        if (!init) {
          double yh0, yh1;
          rot_in(y0, y1, yh0, yh1);
          dot_rows<NY>(rn0, rn1, yh0, yh1, c0, c1);
        }
      } else {
        if (!init) dot_rows<NY>(rn0, rn1, y0, y1, c0, c1);    // rd += Hr y (y broadcast by DPP)
      }
      rd0 = (!kRdCarry || rd_fresh) ? rn0 : rd0;
      rd1 = (!kRdCarry || rd_fresh) ? rn1 : rd1;
    }
    rd_have = true;
    double dg0 = hdg0, dg1 = hdg1, du = 0.0;
    STAMP_END(8);
    STAMP_BEGIN();
    // G_u' D G_u is diagonal, d_q = D[2q] + D[2q+1] on (q, q): lane q's column j0 = q
    if constexpr (WHR) {
      assemble_rot(dg0, dg1);
    } else {
      static_assert(D::NU <= kRow, "torque variables in the first column slot");
      const double2 dd = *reinterpret_cast<const double2*>(sDr + 2 * (j0 < NU ? j0 : 0));
      du = (j0 < NU) ? dd.x + dd.y : 0.0;   // (added to the pivots by ldl_rows)
      dg0 += du;
    }
    STAMP_END(9);
    STAMP_BEGIN();
    if constexpr (!WHR) add_contact_blocks(dg0, dg1);
    wave_sync();
    STAMP_END(2);
    STAMP_BEGIN();
    ldl_rows<NY, SMALL>(c0, c1, B + LY::I_DINV, l, dinv0, dinv1, 1e-13 * dg0, 1e-13 * dg1, du);
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
      // iterations vs a fixed 0.99; uncapped, a few envs stall at the boundary).  The fix-up
      // pass (an env the first pass left not OK) keeps 0.99: the envs of round 5's census that
      // stalled at max_iter with the adaptive rule (~1 in 600,000 joint-state envs) converge in
      // 15-20 iterations with it (numpy model of the kernel, tools/ipm_model.py)
      const double eta =
          fixup ? 0.99
                : fmin(1.0 - 1e-5, fmax(0.99, fmax(1.0 - mu, 1.0 - 0.1 * (1.0 - a_aff))));
      const double alpha = done ? 0.0 : fmin(1.0, eta * step);
      y0 = fma(alpha, dy0, y0);
      y1 = fma(alpha, dy1, y1);
#pragma unroll
      for (int t = 0; t < NRL; ++t) {
        s[t] = act[t] ? fma(alpha, ds[t], s[t]) : 1.0;
        lam[t] = act[t] ? fma(alpha, dl[t], lam[t]) : 0.0;
        rp[t] *= 1.0 - alpha;
      }
      if constexpr (kRdCarry) {
        rdc0 = (1.0 - alpha) * rd0;
        rdc1 = (1.0 - alpha) * rd1;
      }
    }
    sVy[j0] = y0;
    if (v1) sVy[j1] = y1;
    // next iteration's Hr columns (the factor in c0/c1 is dead now).  (Round 6: issuing them right
    // after the last pass's solve instead, so the L2 loads of the two-wave kernel fly during the
    // ratio tests, measured no gain -- Go2 8,192 0.2534 vs 0.2531 ms, 65,536 1.593 vs 1.600.)
    load_hr();
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
              c0[i] = wsw[lane_off + static_cast<unsigned>(hr_off<D>(i, j0))];
              c1[i] = wsw[lane_off + static_cast<unsigned>(hr_off<D>(i, jj1))];
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
        double dg0 = hdg0, dg1 = hdg1, du = 0.0;
        if constexpr (WHR) {
          wave_sync();
          assemble_rot(dg0, dg1);
        } else {
          const double2 dd = *reinterpret_cast<const double2*>(sDr + 2 * (j0 < NU ? j0 : 0));
          du = (j0 < NU) ? dd.x + dd.y : 0.0;
          dg0 += du;
        }
        if constexpr (!WHR) add_contact_blocks(dg0, dg1);
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
        ldl_rows<NY, SMALL>(c0, c1, B + LY::I_DINV, l, dinv0, dinv1, 1e-13 * dg0, 1e-13 * dg1, du);
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
        // rows the refined point violates join the active set -- (no wheel rows) only the most
        // violated one, and then no row leaves this round: adding every violated row while dropping
        // every negative multiplier at once cycles on the joint-state envs whose interior point
        // missed one weakly active pyramid row (a period-3 cycle through 8 rounds, ~1e-4 of the
        // envs at joint_range 1.0, tests/golden/go2_unrefined_joint_states.npz; tools/kkt_study.py
        // one_change: every such env settles in <= 4 rounds on its exact optimum)
        double nviol = 0.0, vl = 0.0, gv[NRL];
#pragma unroll
        for (int t = 0; t < NRL; ++t) {
          gv[t] = Gv(sVy, t) - h[t];
          vl = fmax(vl, (act[t] && Dr[t] == 0.0 && gv[t] > ytol) ? gv[t] : 0.0);
        }
        const double vbest = WHR ? 0.0 : row_max(vl);
#pragma unroll
        for (int t = 0; t < NRL; ++t) {
          const bool v = act[t] && Dr[t] == 0.0 && gv[t] > ytol && (WHR || gv[t] == vbest);
          Dr[t] = v ? dpen : Dr[t];
          nviol += v ? 1.0 : 0.0;
        }
        {
          // ... and rows whose multiplier came out negative leave it (WH: its slack-based active
          // set can include a row the optimum leaves; otherwise a row the interior point's
          // lambda > s test took with a vanishing multiplier) -- (no wheel rows) in a round that
          // added none, and only the most negative one
          const bool drops = WHR || vbest == 0.0;   // (uniform over the env's row of lanes)
          double mmax = 0.0, mlo = 0.0;
#pragma unroll
          for (int t = 0; t < NRL; ++t) {
            mmax = fmax(mmax, Dr[t] != 0.0 ? fabs(mur[t]) : 0.0);
            mlo = fmin(mlo, Dr[t] != 0.0 ? mur[t] : 0.0);
          }
          const double mtol = 1e-9 * (1.0 + row_max(mmax));
          const double mworst = WHR ? 0.0 : row_min(mlo);
#pragma unroll
          for (int t = 0; t < NRL; ++t) {
            const bool leave = drops && Dr[t] != 0.0 && mur[t] < -mtol && (WHR || mur[t] == mworst);
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
      if (giters) giters[env] = (kFix && fixup) ? P->max_iter + it_done : it_done;   // both passes
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
#ifndef OSC_LARGE_WAVES
#define OSC_LARGE_WAVES 2
#endif
__global__ __launch_bounds__(kWave, SMALL ? 1 : OSC_LARGE_WAVES) void osc_ipm_kernel(
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
  // flags bit 2 (warm-started, refinement fused): the cold fix-up pass runs in the same launch,
  // each wavefront right after its own warm pass (its statuses are its own global stores: the
  // fence makes them visible to its lanes) -- the separate fix-up launch, 1,024 wavefronts that
  // mostly exit at once, cost 4.2 us of a 139 us Go2 4,096 warm tick
  ipm_block<D, SMALL, WARM, RF>(P, static_cast<int>(blockIdx.x), nenv, gmask, ws, gtau, gx,
                                gstatus, giters, gwarm, flags & 3, sm);
  if constexpr (WARM || RF == kRfFused) {
    if (flags & 4) {   // (a second inlined body: a loop over both passes spilled 180 B per lane)
      // the statuses it reads are this wavefront's own stores: a workgroup-scope fence (their
      // completion) is enough -- a device-scope __threadfence() wrote the L2 back in every
      // wavefront, +15-18 % at 8,192 / 65,536 envs where two waves share each SIMD
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
      ipm_block<D, SMALL, WARM, RF>(P, static_cast<int>(blockIdx.x), nenv, gmask, ws, gtau, gx,
                                    gstatus, giters, gwarm, (flags & 2) | 1, sm);
    }
  }
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
__global__ __launch_bounds__(kWave, 1) void osc_ipm_pair_kernel(PairArgs A, PairArgs B, int flags) {
  __shared__ __attribute__((aligned(16))) double
      sm[cmax(ipm_lds_doubles<DA, true, RF>(), ipm_lds_doubles<DB, true, RF>())];
  const int nbA = (A.nenv + kEnvPerWave - 1) / kEnvPerWave;
  const int blk = static_cast<int>(blockIdx.x);
  // (flags bit 0: the cold fix-up pass over the envs left not OK, launched after the solve when
  // refinement is fused -- a second launch: a second inlined body per model spills, launch_pair)
  if (blk < nbA)
    ipm_block<DA, true, false, RF>(A.P, blk, A.nenv, A.mask, A.ws, A.tau, A.x, A.status,
                                   A.iters, nullptr, flags & 1, sm);
  else
    ipm_block<DB, true, false, RF>(B.P, blk - nbA, B.nenv, B.mask, B.ws, B.tau, B.x,
                                   B.status, B.iters, nullptr, flags & 1, sm);
}

// ---- launch_ipm: the interior-point passes of one call (after the assembly) ----
// All wavefronts resident at once (<= one per SIMD): the latency-optimised variant (one wave per
// SIMD, Hr in LDS where it fits); otherwise the two-waves-per-SIMD variant.
template <class D>
void launch_ipm(const LaunchArgs& a) {
  const osc_model* model = a.model;
  const int32_t nenv = a.nenv;
  const double* mask = a.mask;
  double* ws = a.ws;
  double *tau = a.tau, *x = a.x, *warm = a.warm;
  int32_t *status = a.status, *iters = a.iters;
  const hipStream_t s = a.s;
  const unsigned nb = static_cast<unsigned>((nenv + kEnvPerWave - 1) / kEnvPerWave);
  const int flags = a.y != nullptr ? 2 : 0;   // hand the multipliers to the dual kernel
  if constexpr (D::WH) {
    // wheel rows: the one-wave solve with the refinement fused; warm-started: the warm pass, then
    // (same launch) the cold fix-up pass in the wavefronts holding an env the warm start left
    // unconverged (the per-env status: the caller's array, else scratch -- launch_t).  The fused entries then run
    // the active-set fallback over the envs the interior point left unconverged (launch_gi).
    if (warm == nullptr) {
      hipLaunchKernelGGL((osc_ipm_kernel<D, true, false, kRfFused>), dim3(nb), dim3(kWave), 0, s,
                         model->dparams, nenv, mask, ws, tau, x, status, iters, nullptr, flags);
    } else {
      hipLaunchKernelGGL((osc_ipm_kernel<D, true, true, kRfFused>), dim3(nb), dim3(kWave), 0, s,
                         model->dparams, nenv, mask, ws, tau, x, status, iters, warm, flags | 4);
    }
  } else {
    // A warm-started solve is followed by a cold fix-up pass over the wavefronts that hold an
    // env the warm start did not bring to convergence (per-env status: launch_t).
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
    const bool compact = fused && model->park_it > 0 &&
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
      // the cold fix-up pass the one-launch solves run in their own launch (an env left not OK
      // re-solved cold to mu <= 1e-12): here a third launch, whose wavefronts without such an
      // env exit at once (round 5 census: 3 WaLTER envs in 1.6 M stalled at max_iter here)
      if (small)
        hipLaunchKernelGGL((osc_ipm_kernel<D, true, false, kRfFused>), dim3(nb), dim3(kWave), 0, s,
                           model->dparams, nenv, mask, ws, tau, x, status, iters, nullptr,
                           (flags & 2) | 1);
      else
        hipLaunchKernelGGL((osc_ipm_kernel<D, false, false, kRfFused>), dim3(nb), dim3(kWave), 0, s,
                           model->dparams, nenv, mask, ws, tau, x, status, iters, nullptr,
                           (flags & 2) | 1);
    } else if (warm == nullptr) {
      // every env the interior point or the refinement leaves not OK (MAX_ITER, UNREFINED,
      // non-finite) is re-solved cold to mu <= 1e-12 by its own wavefront in the same launch, as
      // the warm entries do (round 5's census: ~1 such env per 600,000 joint-state envs; only
      // the wavefronts holding one run the second pass)
      const int fl = flags | 4;
      if (fused && small)
        hipLaunchKernelGGL((osc_ipm_kernel<D, true, false, kRfFused>), dim3(nb), dim3(kWave), 0, s,
                           model->dparams, nenv, mask, ws, tau, x, status, iters, nullptr, fl);
      else if (fused)
        hipLaunchKernelGGL((osc_ipm_kernel<D, false, false, kRfFused>), dim3(nb), dim3(kWave), 0, s,
                           model->dparams, nenv, mask, ws, tau, x, status, iters, nullptr, fl);
      else if (small)
        hipLaunchKernelGGL((osc_ipm_kernel<D, true, false>), dim3(nb), dim3(kWave), 0, s,
                           model->dparams, nenv, mask, ws, tau, x, status, iters, nullptr, flags);
      else
        hipLaunchKernelGGL((osc_ipm_kernel<D, false, false>), dim3(nb), dim3(kWave), 0, s,
                           model->dparams, nenv, mask, ws, tau, x, status, iters, nullptr, flags);
    } else if (fused_warm) {
      // warm-started: the refinement runs in the same wavefront too, in the warm pass for the
      // envs the warm start converged and in the cold fix-up pass (same launch) for the ones it
      // redoes
      hipLaunchKernelGGL((osc_ipm_kernel<D, true, true, kRfFused>), dim3(nb), dim3(kWave), 0, s,
                         model->dparams, nenv, mask, ws, tau, x, status, iters, warm, 4);
    } else {
      // warm past one wave per SIMD (or without the refinement): the warm pass, the separate
      // refinement pass, then the cold fix-up pass over every env not OK by then -- MAX_ITER,
      // non-finite, and an env whose refinement found no KKT point, UNREFINED.  The
      // fix-up pass runs the refinement in its own wavefront (the fused two-wave warm kernel: it
      // spills, but only the wavefronts holding such an env execute it).
      if (small)
        hipLaunchKernelGGL((osc_ipm_kernel<D, true, true>), dim3(nb), dim3(kWave), 0, s,
                           model->dparams, nenv, mask, ws, tau, x, status, iters, warm, 0);
      else
        hipLaunchKernelGGL((osc_ipm_kernel<D, false, true>), dim3(nb), dim3(kWave), 0, s,
                           model->dparams, nenv, mask, ws, tau, x, status, iters, warm, 0);
      if (model->refine) {
        hipLaunchKernelGGL((osc_refine_kernel<D, false>), dim3(nb), dim3(kWave), 0, s,
                           model->dparams, nenv, mask, ws, tau, x, status);
        hipLaunchKernelGGL((osc_ipm_kernel<D, false, true, kRfFused>), dim3(nb), dim3(kWave), 0,
                           s, model->dparams, nenv, mask, ws, tau, x, status, iters, warm, 1);
      } else if (small) {
        hipLaunchKernelGGL((osc_ipm_kernel<D, true, true>), dim3(nb), dim3(kWave), 0, s,
                           model->dparams, nenv, mask, ws, tau, x, status, iters, warm, 1);
      } else {
        hipLaunchKernelGGL((osc_ipm_kernel<D, false, true>), dim3(nb), dim3(kWave), 0, s,
                           model->dparams, nenv, mask, ws, tau, x, status, iters, warm, 1);
      }
    }
  }
}

}  // namespace osc
