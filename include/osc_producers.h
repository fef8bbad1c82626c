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
 * geom (either side of the pair) that belongs to contact site k, else 0.
 *   ncon [nenv]  geom_pairs [nenv][max_con][2] (mjContact.geom)
 *   geom_to_site [ngeom]: contact-site index of each geom's body, -1 for none (built once from
 *   the model, the examples' getSiteIdsOnSameBodyAsGeom)
 *   contact_mask [nenv][nc] -> the mask input of osc_batch_solve */
int osc_contact_mask_from_contacts(int32_t nenv, int32_t nc, int32_t max_con, const int32_t* ncon,
                                   const int32_t* geom_pairs, int32_t ngeom,
                                   const int32_t* geom_to_site, double* contact_mask,
                                   void* stream);

#ifdef __cplusplus
}
#endif

#endif /* OSC_PRODUCERS_H_ */
