/*
 * osc_batch.h -- C-ABI of the MI355X-native batched operational-space-control (OSC) solver.
 *
 * One call solves, for every environment of a batch, the per-tick OSC quadratic program of
 * vannem95/operational-space-control and returns the joint torques.  The entry points replace
 * the reference's per-tick inner operator boundary (paths relative to the reference's
 * operational-space-control/ directory):
 *
 *   osc_desc_from_yaml / osc_model_create
 *       replace the build-time CasADi generation of the six QP functions and the constexpr
 *       sizes: unitree_go2/autogen/autogen.py:19-56 (YAML + sizes), :240-411 (codegen), and the
 *       hard-coded bound vectors unitree_go2/operational_space_controller.h:276-309
 *       (walter_sr/operational_space_controller.h:309-353).
 *   osc_batch_solve
 *       replaces, per environment, the six CasADi evaluations
 *       (unitree_go2/operational_space_controller.h:457-481 via unitree_go2/utilities.h:43-77:
 *        int F(const double** arg, double** res, casadi_int* iw, double* w, int mem) for
 *        F in {beq, Aeq, bineq, Aineq, H, f}), the OSQP stacking/update
 *       (operational_space_controller.h:483-529: UpdateObjectiveAndConstraintMatrices,
 *        SetObjectiveVector, SetBounds, Init, SetWarmStart), the solve
 *       (operational_space_controller.h:531-536: OsqpSolver::Solve, primal_solution,
 *        dual_solution) and the torque slice (operational_space_controller.h:573).
 *   osc_model_destroy
 *       replaces the teardown of the OSQP workspace / CasADi memory pools.
 *
 * Inputs are what update_osc_data (operational_space_controller.h:376-455) produces, batched
 * env-major, row-major per environment, IEEE fp64:
 *   M    [nenv][nv][nv]      mass matrix (mj_fullM)
 *   C    [nenv][nv]          bias forces (qfrc_bias)
 *   J    [nenv][6*ns][nv]    task Jacobian [Jp_0..Jp_{ns-1}; Jr_0..Jr_{ns-1}]
 *   b    [nenv][6*ns]        task bias acceleration  Jdot * qd
 *   T    [nenv][ns][6]       task-space acceleration targets (TaskspaceTargets, row-major)
 *   mask [nenv][nc]          contact mask (State::contact_mask)
 * The contact Jacobian is NOT an input: as in the reference it is the last 3*nc translational
 * rows of J, transposed (operational_space_controller.h:439-445).
 *
 * Outputs:
 *   tau    [nenv][nu]             torque command = x[nv : nv+nu]
 *   x      [nenv][nv+nu+3nc]      (nullable) full design vector (dv, u, z) = get_solution()
 *   status [nenv]                 (nullable) OSC_SOLVE_* code per environment
 *   iters  [nenv]                 (nullable) interior-point iterations used; max_iter + k when
 *                                 a cold fix-up pass re-solved the env (k its iterations: every
 *                                 env the first pass leaves not OK, warm or cold entry -- see
 *                                 OSC_SOLVE_UNREFINED); -k when the wheel rows' active-set
 *                                 fallback solved it in k steps (osc_batch_solve_ex / _warm_ex)
 *
 * All batch pointers passed to osc_batch_solve are DEVICE pointers (HBM-resident); `stream` is
 * a hipStream_t (NULL = default stream).  The call is asynchronous with respect to the host.
 * Every function returns an osc_status (0 = OK).  Handles are re-entrant: a model may be used
 * from several streams concurrently; there is no global state.
 */
#ifndef OSC_BATCH_H_
#define OSC_BATCH_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OSC_ABI_VERSION 4
#define OSC_MAX_SITES 32
#define OSC_MAX_NU 16

/* Return codes (map onto the reference's absl::Status use: InternalError for load failures,
 * FailedPreconditionError for lifecycle misuse -- operational_space_controller.h:112-218). */
typedef enum {
  OSC_OK = 0,
  OSC_ERR_INVALID_ARGUMENT = 1,   /* null pointer, nenv < 0, inconsistent descriptor        */
  OSC_ERR_UNSUPPORTED_DIMS = 2,   /* (nv, nu, nc, ns) has no compiled gfx950 kernel          */
  OSC_ERR_IO = 3,                 /* YAML file missing / unreadable / malformed               */
  OSC_ERR_DEVICE = 4,             /* HIP runtime error (allocation, launch)                   */
  OSC_ERR_NO_DEVICE = 5           /* no HIP device visible                                    */
} osc_status;

/* Per-environment solve status written to status[] */
typedef enum {
  OSC_SOLVE_OK = 0,               /* converged: complementarity <= eps_mu                     */
  OSC_SOLVE_MAX_ITER = 1,         /* iteration cap reached; best iterate returned             */
  OSC_SOLVE_NUMERICAL = 2,        /* non-finite values encountered (e.g. NaN inputs), or an M
                                     that is not positive definite (a pivot <= 0 in the
                                     elimination of dv; every mass matrix is SPD)              */
  OSC_SOLVE_UNREFINED = 3         /* converged (complementarity <= eps_mu) but the full-space
                                     refinement found no KKT point within its rounds (or was
                                     forced off by osc_model_tuning.refine_max_move): the
                                     interior point's iterate is returned, accurate only to its
                                     stop (up to ~2e-2 normwise at eps_mu 1e-6
                                     along the internal-force directions).  Every entry
                                     re-solves such an env (and a MAX_ITER or non-finite one)
                                     cold to mu <= 1e-12 in a fix-up pass before returning
                                     (round 5: cold solves too -- same launch, a third one
                                     after the lockstep compaction, a second one after the
                                     two-model kernel of osc_batch_solve_multi), and then it is
                                     within ~1e-5
                                     even if this status remains.  Measured: none on the
                                     synthetic and joint-state test batches; 6 of 3.1 M
                                     joint-state envs not OK before that fix-up (2 UNREFINED,
                                     4 MAX_ITER), none after (round 5 census, 48 x 65,536)     */
} osc_solve_status;

/* Everything that defines the QP of one robot -- what autogen.py bakes into generated C
 * (sizes, weights, friction) plus the bound vectors hard-coded in the controller header. */
typedef struct {
  int32_t nv;                     /* generalized velocities (mjModel::nv)                    */
  int32_t nu;                     /* actuators; B = [0_{(nv-nu) x nu}; I_nu]                  */
  int32_t nc;                     /* contact sites (last nc of the ns sites)                  */
  int32_t ns;                     /* task sites (noncontact + contact)                        */
  double mu;                      /* friction_coefficient                                     */
  double w_pos[OSC_MAX_SITES];    /* <site>_translational_tracking, site order                */
  double w_rot[OSC_MAX_SITES];    /* <site>_rotational_tracking                               */
  double w_torque;                /* weights_config.torque                                    */
  double w_reg;                   /* weights_config.regularization                            */
  double u_lb[OSC_MAX_NU];        /* torque bounds (osc.h:285-296)                            */
  double u_ub[OSC_MAX_NU];
  double z_lb[3];                 /* per-contact force bounds before the mask multiply        */
  double z_ub[3];                 /*   (osc.h:297-308): {-inf,-inf,0} / {inf,inf,big_number}  */
  double infinity;                /* OSQP_INFTY (1e30); |bound| >= infinity/1e10 = no bound   */
  double eps_mu;                  /* interior-point stop: mean complementarity <= eps_mu;
                                     models without the refinement stop at min(eps_mu, 1e-12) */
  int32_t max_iter;               /* interior-point iteration cap                             */
  /* Wheel no-slip equality rows (ABI 2) -- the design walter_sr_wheels/autogen/autogen.py:128-240
   * leaves commented out, opt-in here.  wheel_rows = 1 adds, for every contact site i (a wheel),
   *   d_roll_i . (J_p,i dv + b_i) - wheel_radius[i] * dv[wheel_dof[i]] = 0      (longitudinal)
   *   d_lat_i  . (J_p,i dv + b_i)                                     = 0      (lateral)
   * with J_p,i / b_i the contact site's translational rows of J / b (the Jacobian-dot bias
   * J_dot_p,i qd of the design) and the directions d_roll, d_lat per env (osc_solve_extras).
   * wheel_dof[i] = -1: no rolling term (a model without that wheel joint).  Each wheel's two rows
   * are multiplied by its contact mask, as the contact-force bounds are (osc.h:492-495). */
  int32_t wheel_rows;             /* 0 = off (the reference's QP), 1 = on                    */
  int32_t wheel_dof[OSC_MAX_SITES];
  double wheel_radius[OSC_MAX_SITES];
} osc_model_desc;

typedef struct osc_model osc_model;   /* opaque: descriptor + device-resident parameters */

/* Host-only: fill `desc` for `robot` ("unitree_go2", "walter_sr", "walter_sr_wheels") from a
 * YAML file in the reference's config schema (config/<robot>/<robot>_config.yaml).  Needs no
 * GPU.  `yaml_path` NULL = the robot's default config next to the library. */
int osc_desc_from_yaml(const char* robot, const char* yaml_path, osc_model_desc* desc);

/* Validate `desc`, pick the compiled kernel for its dimensions and upload its parameters to
 * the current HIP device. */
int osc_model_create(const osc_model_desc* desc, osc_model** out);

/* Solver policy knobs (ABI 3).  A release library reads no environment variable: what used to be
 * OSC_* variables is this explicit block, filled with the model's defaults by
 * osc_model_tuning_defaults and passed to osc_model_create_tuned.  None of them changes the QP;
 * they change how the interior point and the refinement get to its optimum (and so the last
 * bits of the result), or which kernel variant runs.  For experiments and tests. */
typedef struct {
  int32_t refine_steps;           /* full-space refinement: minimum steps per round (each env
                                     stops at its own convergence, at most 8 -- a larger value is
                                     clamped to 8); 0 = no refinement, the interior point then
                                     runs to eps_mu <= 1e-12.  Default 2 (wheel rows: 12, fixed,
                                     not clamped)                                                */
  double refine_max_move;         /* reject a refinement that moves y by more than this x
                                     (1 + |y|) (OSC_SOLVE_UNREFINED).  Default 1e300 (none: a
                                     kept refinement is a KKT point, i.e. the optimum)           */
  double eps_mu;                  /* interior-point stop; default the descriptor's eps_mu        */
  int32_t restart_iter;           /* cold: an env still far off (mu > 1e-6) is re-centred at this
                                     iteration.  Default 28                                      */
  int32_t warm_restart;           /* warm-started: the same.  Default 22                         */
  double warm_delta;              /* warm start: slacks / multipliers floored here.  Default 1   */
  double warm_center;             /* warm start: no pair below this x their mean.  Default 1     */
  double wheel_tol;               /* wheel rows: residual needed to stop.  Default 1e-6          */
  int32_t small_batch_max;        /* the one-wave interior-point kernel up to this batch, the
                                     two-wave one above; -1 = the device's resident batch (4 envs
                                     per wave x 4 SIMDs x CUs) for Go2, always one-wave WaLTER   */
  int32_t park_it;                /* lockstep compaction's park iteration; 0 = off; -1 = model
                                     default (WaLTER 16, Go2 off)                                */
} osc_model_tuning;

/* Fill `tuning` with the defaults of the model `desc` describes (host-only). */
int osc_model_tuning_defaults(const osc_model_desc* desc, osc_model_tuning* tuning);

/* osc_model_create with explicit tuning (NULL = the defaults). */
int osc_model_create_tuned(const osc_model_desc* desc, const osc_model_tuning* tuning,
                           osc_model** out);

/* Convenience: osc_desc_from_yaml + osc_model_create. */
int osc_model_create_from_yaml(const char* robot, const char* yaml_path, osc_model** out);

int osc_model_destroy(osc_model* model);

/* Copy of the descriptor a model was created from. */
int osc_model_get_desc(const osc_model* model, osc_model_desc* desc);

/* Device scratch the solve needs for `nenv` environments: the per-env reduced QP handed from
 * the assembly kernel to the interior-point kernel (osc_workspace_env_bytes per env, env-major
 * from the start of the buffer), then solver scratch the interior point writes: 4 B per env of
 * solve-status scratch for the warm-start fix-up pass, and the lockstep compaction's park area
 * (the interior-point state of envs parked mid-solve, 1.4 KB Go2 / 1.9 KB WaLTER per env), slot
 * list and counter. */
int osc_workspace_bytes(const osc_model* model, int32_t nenv, size_t* bytes);
/* Bytes of one environment's reduced-QP block at the start of the workspace (its stride). */
int osc_workspace_env_bytes(const osc_model* model, size_t* bytes);

/* Batched solve; see the header comment for layouts.  Device pointers, async on `stream`.
 * `workspace` (16-byte aligned, >= osc_workspace_bytes) may be NULL: the library then takes
 * stream-ordered scratch (hipMallocAsync / hipFreeAsync) on `stream` for this call. */
int osc_batch_solve(const osc_model* model, int32_t nenv,
                    const double* M, const double* C, const double* J, const double* b,
                    const double* T, const double* contact_mask,
                    double* tau, double* x, int32_t* status, int32_t* iters,
                    void* workspace, size_t workspace_bytes, void* stream);

/* The two halves of osc_batch_solve, for callers that time, overlap or reuse them.
 * osc_batch_assemble builds every environment's reduced QP (the six CasADi evaluations +
 * OSQP stacking of operational_space_controller.h:457-529, condensed onto NY = nu + 3nc reduced
 * variables y = (u, z)) into `workspace`; osc_batch_solve_assembled runs the interior-point solve
 * on it and writes the outputs exactly as osc_batch_solve does (contact_mask must be the one
 * assembled with).  Here `workspace` is required (>= osc_workspace_bytes, 16-byte aligned).  Its
 * layout per environment, in doubles: [g (NY, padded even) | Hr (padded even) | X
 * (nv x (NY+1), row stride padded even) | H_dv (nv x nv) | f_dv (nv, padded even) | solver
 * hand-off], stride osc_workspace_env_bytes, with dv = X [y; 1] = M^-1 (B u + Jc z - C),
 * H_dv = 2 J'WJ + 2 w_reg I and f_dv = 2 J'W (b - t) (wheel rows: further blocks).
 * Hr (symmetric) is stored compact (round 6) -- its rows 16 .. NY-1 whole (row-major, NY columns
 * each), then the upper triangle of its leading 16 x 16 block packed row by row: (NY-16) NY + 136
 * doubles -- except for models with wheel rows, which keep the full NY x NY row-major Hr.
 * The solve WRITES to the workspace: its per-env hand-off blocks and, past the reduced QPs, the
 * solve-status scratch, the lockstep compaction's park area, slot list and counter
 * -- one workspace serves one solve at a time; concurrent solves on several streams need a
 * workspace each (the reduced-QP blocks themselves are only read, so the same assembled QPs may
 * be copied and solved again). */
int osc_batch_assemble(const osc_model* model, int32_t nenv,
                       const double* M, const double* C, const double* J, const double* b,
                       const double* T, const double* contact_mask,
                       void* workspace, size_t workspace_bytes, void* stream);
int osc_batch_solve_assembled(const osc_model* model, int32_t nenv, const double* contact_mask,
                              double* tau, double* x, int32_t* status, int32_t* iters,
                              void* workspace, size_t workspace_bytes, void* stream);

/* Warm start across control ticks -- the reference's OsqpSolver::SetWarmStart with the previous
 * tick's primal/dual solution (operational_space_controller.h:519-526).  `warm_state` is a
 * caller-owned DEVICE buffer of osc_warm_state_bytes(model, nenv) bytes (per env: [valid flag |
 * y | lambda | contact mask] of the interior point), zero-filled before the first tick.  An env
 * starts cold when its state is not valid (zero-filled, or the last solve hit NaN), when its
 * contact mask differs from the state's (a contact-mode switch changes the QP's rows), or when
 * it has no inequality rows.  Each call reads the state and writes this tick's solution back.
 * Results agree with the cold solve to the solve's tolerance; the iteration count drops when
 * consecutive ticks are close.  A warm env that stalls is re-centred in place,
 * and any env the warm pass leaves not OK (OSC_SOLVE_MAX_ITER / _NUMERICAL / _UNREFINED) is
 * re-solved cold, to mu <= 1e-12, by the wavefront holding it right after its warm pass (the
 * same launch; past one wave per SIMD without wheel rows: a second launch that only the
 * wavefronts holding such an env execute). */
int osc_warm_state_bytes(const osc_model* model, int32_t nenv, size_t* bytes);
int osc_batch_solve_warm(const osc_model* model, int32_t nenv,
                         const double* M, const double* C, const double* J, const double* b,
                         const double* T, const double* contact_mask,
                         double* tau, double* x, int32_t* status, int32_t* iters,
                         double* warm_state, size_t warm_state_bytes,
                         void* workspace, size_t workspace_bytes, void* stream);
int osc_batch_solve_assembled_warm(const osc_model* model, int32_t nenv,
                                   const double* contact_mask, double* tau, double* x,
                                   int32_t* status, int32_t* iters,
                                   double* warm_state, size_t warm_state_bytes,
                                   void* workspace, size_t workspace_bytes, void* stream);

/* One model's batch inside a multi-model call: the arguments of osc_batch_solve for that model
 * (device pointers; `workspace` required, >= osc_workspace_bytes(model, nenv), 16-B aligned). */
typedef struct {
  const osc_model* model;
  int32_t nenv;
  const double *M, *C, *J, *b, *T, *contact_mask;
  double* tau;
  double* x;                      /* nullable */
  int32_t* status;                /* nullable */
  int32_t* iters;                 /* nullable */
  void* workspace;
  size_t workspace_bytes;
  const double* wheel_dir;        /* (ABI 4) [nenv][nc][6] DEVICE; required iff the model has wheel
                                     rows (osc_solve_extras.wheel_dir); MUST be NULL otherwise
                                     (a non-NULL one is refused: OSC_ERR_INVALID_ARGUMENT, the
                                     mark of a job built against the ABI-3 layout)              */
} osc_batch_job;

/* Several robots' batches on one GPU in one call (BASELINE configs[4]: Go2 + WaLTER Sr shards
 * per GPU).  Results are bitwise those of one osc_batch_solve (wheel rows: osc_batch_solve_ex)
 * per job.  Two jobs of different kernels (unitree_go2 + walter_sr) whose batches each fit one
 * wavefront per SIMD run as ONE assembly grid and ONE interior-point grid, the slower model's
 * wavefronts first, so the other model's wavefronts fill the SIMDs freed by the first one's
 * iteration-count tail; anything else (a wheel-row model among them) runs the jobs one after
 * another on `stream`. */
int osc_batch_solve_multi(const osc_batch_job* jobs, int32_t njobs, void* stream);

/* Per-call extras of osc_batch_solve_ex. */
typedef struct {
  /* [nenv][nc][6] DEVICE: (d_roll, d_lat) of every wheel; required iff the model has wheel rows */
  const double* wheel_dir;
  /* [nenv][osc_dual_rows] DEVICE, nullable: the dual solution in OSQP's convention
   * (H x + f + A'y = 0, y > 0 on an active upper bound, < 0 on an active lower bound) over the
   * reference's rows A = [Aeq (dynamics; wheel rows); Aineq; I_n] (operational_space_controller.h:
   * 483-497) -- the reference's OsqpSolver::dual_solution (osc.h:534-535).  Requires x != NULL. */
  double* y;
} osc_solve_extras;

/* Rows of the dual solution: nv (+ 2 nc wheel rows) + 4 nc + (nv + nu + 3 nc). */
int osc_dual_rows(const osc_model* model, int32_t* rows);

/* osc_batch_solve with the per-call extras (NULL extras = osc_batch_solve).  A model with wheel
 * rows is solved through this entry, osc_batch_solve_warm_ex, osc_batch_solve_multi (its
 * wheel_dir), or osc_batch_assemble_ex followed by osc_batch_solve_assembled(_warm).  With wheel
 * rows every one of them re-solves each env the interior point did not leave OK by a dual
 * active-set method on the full QP (iters = -steps, and a warm state of such an
 * env is invalidated, so its next tick starts cold): the assembly leaves the raw rows it needs in
 * the workspace, so the split entries run it too. */
int osc_batch_solve_ex(const osc_model* model, int32_t nenv,
                       const double* M, const double* C, const double* J, const double* b,
                       const double* T, const double* contact_mask, const osc_solve_extras* extras,
                       double* tau, double* x, int32_t* status, int32_t* iters,
                       void* workspace, size_t workspace_bytes, void* stream);
/* osc_batch_solve_warm with the per-call extras (wheel directions, duals): the warm-started tick
 * of a wheel-row model (the reference's walter_sr_wheels controller warm-starts every tick,
 * walter_sr_wheels/operational_space_controller.h:583, 591-600). */
int osc_batch_solve_warm_ex(const osc_model* model, int32_t nenv,
                            const double* M, const double* C, const double* J, const double* b,
                            const double* T, const double* contact_mask,
                            const osc_solve_extras* extras, double* tau, double* x,
                            int32_t* status, int32_t* iters, double* warm_state,
                            size_t warm_state_bytes, void* workspace, size_t workspace_bytes,
                            void* stream);
int osc_batch_assemble_ex(const osc_model* model, int32_t nenv,
                          const double* M, const double* C, const double* J, const double* b,
                          const double* T, const double* contact_mask, const double* wheel_dir,
                          void* workspace, size_t workspace_bytes, void* stream);

/* Human-readable name of an osc_status. */
const char* osc_status_string(int status);

/* Library ABI version (OSC_ABI_VERSION). */
int osc_abi_version(void);

#ifdef __cplusplus
}
#endif

#endif /* OSC_BATCH_H_ */
