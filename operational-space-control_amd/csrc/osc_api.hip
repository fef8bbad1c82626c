// osc_api.hip -- the C-ABI of the batched OSC QP assembly + solve for gfx950 (MI355X):
// include/osc_batch.h.  Model creation, tuning, workspace layout and the pass sequence of every
// entry point; the kernels live in osc_setup / osc_ipm_* / osc_dual / osc_gi / osc_multi.hip.
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
#include "osc_internal.hpp"

using namespace osc;

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

#ifdef OSC_STAMPS
// Diagnostic builds only: the phase-cycle buffers every kernel unit's STAMP_STORE writes through
// DevParams (allocated with the first model), and their readers (tools/stamps.py,
// tools/setup_stamps.py): [nblocks][kStampSlots] of the last launch.
namespace {
unsigned long long* g_stamp_buf[2] = {nullptr, nullptr};
int stamps_read(int which, unsigned long long* host, int nblocks) {
  if (!g_stamp_buf[which]) return OSC_ERR_INVALID_ARGUMENT;
  if (nblocks > kStampBlocks) nblocks = kStampBlocks;
  return hipMemcpy(host, g_stamp_buf[which], sizeof(unsigned long long) * kStampSlots * nblocks,
                   hipMemcpyDeviceToHost) == hipSuccess ? OSC_OK : OSC_ERR_DEVICE;
}
}  // namespace
extern "C" int osc_debug_stamps(unsigned long long* host, int nblocks) {
  return stamps_read(0, host, nblocks);
}
extern "C" int osc_debug_setup_stamps(unsigned long long* host, int nblocks) {
  return stamps_read(1, host, nblocks);
}
#endif

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
  // Without wheel rows a round runs at most kRefineMaxSteps steps and an env counts as converged
  // only from its refine_steps-th step on: a larger minimum would leave every env UNREFINED.  It
  // is clamped to the round's length (the wheel kernels run exactly refine_steps).
  hp.refine_steps = d.wheel_rows ? t.refine_steps : std::min(t.refine_steps, kRefineMaxSteps);
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
#ifdef OSC_STAMPS
  for (auto*& b : g_stamp_buf)
    if (!b && hipMalloc(&b, sizeof(unsigned long long) * kStampSlots * kStampBlocks) != hipSuccess)
      return OSC_ERR_DEVICE;
  hp.stamps = g_stamp_buf[0];
  hp.setup_stamps = g_stamp_buf[1];
#endif

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

// One call's passes: assembly (launch_setup), interior point (launch_ipm), then the wheel-row
// fallback and the duals where asked for.
template <class D>
void launch_t(LaunchArgs a, unsigned stages, const QposArgs* q) {
  if (stages & kAssemble) {
#ifdef OSC_FUSED_TICK
    if constexpr (!D::WH) {
      if (q != nullptr) {   // the fused joint-state tick (A/B builds)
        launch_setup_qpos<D>(a, *q);
        q = nullptr;
      }
    }
#endif
    if (q == nullptr) launch_setup<D>(a);
  }
  if (!(stages & kInteriorPoint)) return;
  // Wheel-row models run the active-set fallback over the envs the interior point left
  // unconverged (osc_gi_kernel; every entry point: the setup kernel left the raw rows it needs in
  // the workspace); it needs the per-env status, and so does a warm-started solve's cold fix-up
  // pass: the caller's array, else scratch at the end of the workspace.
  const bool fallback = D::WH;
  // (and so does the cold solve's fix-up pass in the interior-point launch, refinement fused)
  if (a.status == nullptr && (a.warm != nullptr || fallback || a.model->refine))
    a.status = reinterpret_cast<int32_t*>(a.ws + static_cast<size_t>(D::WS) * a.nenv);
  launch_ipm<D>(a);
  if constexpr (D::WH) {
    if (fallback) launch_gi<D>(a);
  }
  if (a.y != nullptr) launch_dual<D>(a);
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
           double* y = nullptr, const QposArgs* q = nullptr) {
  if (!model || nenv < 0) return OSC_ERR_INVALID_ARGUMENT;
  if (nenv == 0) return OSC_OK;
  if (!on_model_device(model)) return OSC_ERR_INVALID_ARGUMENT;
  if (!contact_mask || misaligned16(contact_mask)) return OSC_ERR_INVALID_ARGUMENT;
  if (q != nullptr) {   // joint states: the kinematics runs in the assembly kernel
    if (!q->kin || !q->qpos || !q->qvel || !T || misaligned16(T) || stages != kBoth)
      return OSC_ERR_INVALID_ARGUMENT;
  } else if ((stages & kAssemble) && (!M || !C || !J || !b || !T || misaligned16(M) ||
                                      misaligned16(C) || misaligned16(J) || misaligned16(b) ||
                                      misaligned16(T))) {
    return OSC_ERR_INVALID_ARGUMENT;   // 16-byte alignment: vectorised staging loads
  }
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
  LaunchArgs a{model, nenv, M, C, J, b, T, contact_mask, tau, x, status, iters, ws, warm, s,
               wdir, y};
  switch (model->kid) {
    case K_GO2:
      launch_t<Go2>(a, stages, q);
      break;
    case K_WALTER:
      launch_t<Walter>(a, stages, q);
      break;
    case K_WALTER_WHEELS:
      launch_t<WalterW>(a, stages, q);
      break;
    default:
      rc = OSC_ERR_UNSUPPORTED_DIMS;
  }
  if (rc == OSC_OK && hipGetLastError() != hipSuccess) rc = OSC_ERR_DEVICE;
  if (owned) (void)hipFreeAsync(ws, s);
  return rc;
}

}  // namespace

#ifdef OSC_FUSED_TICK
namespace osc {
int solve_qpos_fused(const osc_model* model, const QposArgs& q, int32_t nenv, const double* T,
                     const double* contact_mask, double* tau, double* x, int32_t* status,
                     int32_t* iters, double* warm, size_t warm_bytes, void* workspace,
                     size_t workspace_bytes, void* stream) {
  if (model && model->kid == K_WALTER_WHEELS) return OSC_ERR_INVALID_ARGUMENT;   // (no directions)
  if (warm != nullptr) {
    size_t need = 0;
    if (!model || osc_warm_state_bytes(model, nenv < 0 ? 0 : nenv, &need) != OSC_OK ||
        warm_bytes < need)
      return OSC_ERR_INVALID_ARGUMENT;
  }
  return launch(model, nenv, nullptr, nullptr, nullptr, nullptr, T, contact_mask, tau, x, status,
                iters, workspace, workspace_bytes, stream, kBoth, warm, nullptr, nullptr, &q);
}
}  // namespace osc
#endif

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
    if (j.model->kid == K_NONE) return OSC_ERR_UNSUPPORTED_DIMS;
    if (j.model->kid == K_WALTER_WHEELS && (!j.wheel_dir || misaligned16(j.wheel_dir)))
      return OSC_ERR_INVALID_ARGUMENT;
    // wheel_dir must be NULL without wheel rows: a non-NULL one there is the mark of a caller
    // built against the ABI-3 job layout
    if (j.model->kid != K_WALTER_WHEELS && j.wheel_dir != nullptr) return OSC_ERR_INVALID_ARGUMENT;
    if (!on_model_device(j.model)) return OSC_ERR_INVALID_ARGUMENT;   // one device per call
  }
  hipStream_t s = static_cast<hipStream_t>(stream);
  // The two-model grid exists for exactly {walter_sr, unitree_go2} (a wheel-row model
  // next to either must not take it -- its kernels, strides and fallback differ).
  const auto kid_pair = [&](KernelId p, KernelId q) {
    return jobs[0].model->kid == p && jobs[1].model->kid == q;
  };
  if (njobs == 2 && jobs[0].nenv > 0 && jobs[1].nenv > 0 &&
      (kid_pair(K_WALTER, K_GO2) || kid_pair(K_GO2, K_WALTER)) &&
      jobs[0].nenv <= jobs[0].model->small_batch_max && jobs[1].nenv <= jobs[1].model->small_batch_max) {
    const bool a_walter = jobs[0].model->kid == K_WALTER;
    const osc_batch_job& w = a_walter ? jobs[0] : jobs[1];   // slower per wavefront: first
    const osc_batch_job& g = a_walter ? jobs[1] : jobs[0];
    launch_pair_walter_go2(w, g, s);
    return hipGetLastError() == hipSuccess ? OSC_OK : OSC_ERR_DEVICE;
  }
  for (int i = 0; i < njobs; ++i) {
    const osc_batch_job& j = jobs[i];
    const double* wdir = j.model->kid == K_WALTER_WHEELS ? j.wheel_dir : nullptr;
    const int rc = launch(j.model, j.nenv, j.M, j.C, j.J, j.b, j.T, j.contact_mask, j.tau, j.x,
                          j.status, j.iters, j.workspace, j.workspace_bytes, stream, kBoth,
                          nullptr, wdir);
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
