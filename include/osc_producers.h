/*
 * osc_producers.h -- batched device producers of the solve's per-tick inputs (SURVEY.md §8(f)
 * row 3), so a whole control step can stay on the GPU.  Part of libosc_batch.so; same return
 * codes as osc_batch.h.  All array pointers are DEVICE pointers, env-major; `stream` is a
 * hipStream_t (NULL = default).  Paths are relative to the reference repository root.
 */
#ifndef OSC_PRODUCERS_H_
#define OSC_PRODUCERS_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Task-space PD targets of the example drivers (examples/standing.cc:143-155,
 * examples/walter_sr_standing.cc): for each environment, TaskspaceTargets row 0 =
 *   [ kp_lin (p_ref - p) + kd_lin (0 - v) ,  kp_ang vec(q_ref * conj(q)) + kd_ang (0 - w) ]
 * and rows 1..ns-1 = 0 (TaskspaceTargets::Zero()).  Quaternions are (w, x, y, z) as Eigen's.
 *   base_pos [nenv][3]  base_quat [nenv][4]  lin_vel [nenv][3]  ang_vel [nenv][3]
 *   pos_ref  [nenv][3] if pos_ref_per_env else [3] (shared);  quat_ref likewise [4]
 *   gains    host pointer to {kp_lin, kd_lin, kp_ang, kd_ang} (the examples: 150, 25, 50, 10)
 *   targets  [nenv][ns][6]  -> the T input of osc_batch_solve */
int osc_pd_base_targets(int32_t nenv, int32_t ns, const double* base_pos, const double* base_quat,
                        const double* lin_vel, const double* ang_vel, const double* pos_ref,
                        int32_t pos_ref_per_env, const double* quat_ref, int32_t quat_ref_per_env,
                        const double* gains, double* targets, void* stream);

/* Contact mask from a simulator's contact list (examples/walter_sr_true_tumbling_mjjoint.cc:
 * 473-558): contact_mask[e][k] = 1 iff one of the first ncon[e] contacts of environment e has a
 * geom (either side of the pair) g with geom_to_site[g] == k, else 0.
 *   ncon [nenv]  geom_pairs [nenv][max_con][2] (mjContact.geom)
 *   geom_to_site [ngeom]: contact-site index k of geom g, -1 for none -- built once from the
 *   model by osc_contact_geom_table below, which reproduces the example's rule exactly
 *   contact_mask [nenv][nc] -> the mask input of osc_batch_solve */
int osc_contact_mask_from_contacts(int32_t nenv, int32_t nc, int32_t max_con, const int32_t* ncon,
                                   const int32_t* geom_pairs, int32_t ngeom,
                                   const int32_t* geom_to_site, double* contact_mask,
                                   void* stream);

/* Host-only: the geom -> contact-site table of the example's contact test, from the model's
 * geom_bodyid / site_bodyid.  The example (walter_sr_true_tumbling_mjjoint.cc:436, 523-558) uses
 * ONE id list `wheel_sites_mujoco` = {3, 4, 7, 8, 11, 12, 15, 16} in two roles:
 *   (1) a contact counts when its GEOM id is in the list (contains(list, contact.geom[i]));
 *   (2) it marks the first site on that geom's body (getSiteIdsOnSameBodyAsGeom(..)[0], the
 *       lowest site id with site_bodyid == geom_bodyid), and the mask is the indicator of the
 *       list's entries read as SITE ids among the marked sites (getBinaryRepresentation).
 * So geom_to_site[g] = k iff g is in `ids` and the lowest site on g's body is ids[k]; else -1.
 *   geom_bodyid [ngeom], site_bodyid [nsite], ids [nc] (host pointers); geom_to_site [ngeom]
 *   (host) -> the table osc_contact_mask_from_contacts takes (copy it to the device). */
int osc_contact_geom_table(int32_t ngeom, const int32_t* geom_bodyid, int32_t nsite,
                           const int32_t* site_bodyid, int32_t nc, const int32_t* ids,
                           int32_t* geom_to_site);

/* Per-site task-space targets of the tumbling driver (examples/walter_sr_true_tumbling_mjjoint.cc:
 * 622-1019, WaLTER Sr site order torso | 4 shins | 4 thighs | 8 wheels), for every environment:
 *   shins  (rows 1-4): [0, 0, 0, 0, kp_s (th0 + w_s t - th) + kv_s (w_s - (th - th0)/(t - t0)), 0]
 *                      th = qpos[shin_qadr[i]] (mj_data->qpos[jnt_qposadr[2, 4, 6, 8]], :698-701)
 *   thighs (rows 5-8): [0, 0, kp_h ((z0 + dz) - z) + kv_h (v_h - (z - z0)/(t - t0)), 0, 0, 0]
 *                      z = site_xpos z of the thigh site, z0 its initial value (:873-946)
 *   torso  (row 0):    [kp_l (x0 + v_b t - x) + kv_l (v_b - vx), 0, 0,
 *                       kp_a vec(conj(q)) + kv_a (0 - w)]   (:981-1019; the example's gains are 0)
 *   wheels (rows 9-16) and all other entries: 0.
 * The example computes these finite-difference velocities against the INITIAL positions and time
 * for every tick: its `last_*` updates inside the loop declare new loop-local variables that
 * shadow the outer ones (:684-687, 767-770, 926-931), so the outer values never change.  This
 * producer reproduces that: init_* and t0 are the values captured before the loop (:363-433),
 * and t == t0 gives non-finite velocities exactly as the example's first pass does.
 *   qpos [nenv][nq], qvel [nenv][nv] (linear / angular body velocity = qvel[0:3], [3:6]),
 *   site_xpos [nenv][ns][3] (site_ids order, osc_batch_kinematics' site_xpos output),
 *   t [nenv], t0 [nenv], init_qpos [nenv][nq], init_site_xpos [nenv][ns][3]
 *   params: host pointer (osc_tumbling_params_default fills the example's values)
 *   targets [nenv][ns][6] -> the T input of osc_batch_solve.   ns must be 17, nv >= 6. */
typedef struct {
  double shin_rot_vel;                  /* 0.1 * 8 * 5 rad/s                 (:695)       */
  double shin_kp, shin_kv;              /* 800 * 3, 800 * 3                  (:756-757)   */
  double thigh_lin_vel;                 /* 0                                 (:866)       */
  double thigh_lin_kp, thigh_lin_kv;    /* 4000 * 0.5, 600 * 0.5             (:873-874)   */
  double thigh_height_offset;           /* -0.025                            (:897)       */
  double torso_lin_vel;                 /* 0.2 (x)                           (:982-985)   */
  double torso_lin_kp, torso_lin_kv;    /* 0, 0                              (:1001-1002) */
  double torso_ang_kp, torso_ang_kv;    /* 0, 0                              (:1013-1014) */
  int32_t shin_qadr[4];                 /* jnt_qposadr[2, 4, 6, 8]; 8, 10, 12, 14 for the
                                           torso / (thigh, shin) x 4 joint order           */
} osc_tumbling_params;

void osc_tumbling_params_default(osc_tumbling_params* params);

int osc_tumbling_targets(int32_t nenv, int32_t ns, int32_t nq, int32_t nv, const double* qpos,
                         const double* qvel, const double* site_xpos, const double* t,
                         const double* t0, const double* init_qpos, const double* init_site_xpos,
                         const osc_tumbling_params* params, double* targets, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* OSC_PRODUCERS_H_ */
