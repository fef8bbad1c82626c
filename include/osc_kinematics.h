/*
 * osc_kinematics.h -- batched rigid-body kinematics front end of the OSC solve (SURVEY.md §8(f)
 * row 1): per environment qpos/qvel -> the four quantities update_osc_data hands to the QP
 * (M, C, J, b), so a control step consumes coalesced joint states instead of 7.6 KB (Go2) of
 * MuJoCo output per environment.  Part of libosc_batch.so; same return codes as osc_batch.h.
 *
 * Replaces, per environment (paths relative to the reference's operational-space-control/):
 *   update_mj_data   unitree_go2/operational_space_controller.h:350-374
 *                    (qpos = [0,0,0, quat, q_m], qvel = [v, w, qd_m]; mj_fwdPosition,
 *                     mj_fwdVelocity; site_xpos)            -> osc_state_to_qpos + the kernel
 *   update_osc_data  unitree_go2/operational_space_controller.h:376-455
 *                    (mj_fullM, qfrc_bias, mj_jac / mj_jacDot per site, J = [Jp; Jr],
 *                     b = [Jpd; Jrd] qvel)                    -> osc_batch_kinematics
 *   (walter_sr/operational_space_controller.h:394-500 likewise; its site_ids re-indexing,
 *    :417, is the site list of the descriptor.)
 * MuJoCo 3.2.7 semantics (MODULE.bazel.lock:242-247), restated -- MuJoCo is not linked:
 *   free joint: qpos = (position, unit quaternion w x y z), qvel = (world-frame linear velocity
 *   of the body origin, BODY-frame angular velocity); hinge: rotation about the body-frame axis
 *   through the body-frame anchor; slide: translation along the body-frame axis; ball: rotation
 *   about the body-frame anchor, body-frame angular velocity; mj_fullM includes dof armature; qfrc_bias = inverse dynamics
 *   at zero joint acceleration (Coriolis, centrifugal, gravity); mj_jac / mj_jacDot of a point
 *   fixed to a body, world frame, rows in the reference's stacking order.
 *
 * The descriptor mirrors mjModel's fields (body_parentid, body_pos, body_quat, jnt_type,
 * jnt_axis, jnt_pos, dof_armature, body_mass, body_ipos, body_iquat, body_inertia, site_bodyid,
 * site_pos, opt.gravity), restricted to at most one joint per body, so a caller with MuJoCo
 * fills it straight from its mjModel; a MuJoCo body with several joints is
 * a chain of bodies here, one joint each, the leading ones massless at zero offset (which is how
 * mj_kinematics composes a body's joints, in order; osc_kin_desc_from_mjcf does this split).  Bodies are numbered parents first
 * (MuJoCo's order) WITHOUT the world body: parent -1 = world.  Dofs follow body order.
 */
#ifndef OSC_KINEMATICS_H_
#define OSC_KINEMATICS_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OSC_KIN_MAX_BODIES 16
#define OSC_KIN_MAX_DOFS 32
#define OSC_KIN_MAX_SITES 32

/* Joint types: MuJoCo's mjtJoint values (mjJNT_FREE = 0, mjJNT_BALL = 1, mjJNT_SLIDE = 2,
 * mjJNT_HINGE = 3); -1 = welded body.
 *   ball:  qpos = unit quaternion (w x y z) of the body relative to its parent frame, rotating
 *          about the anchor jnt_pos; qvel = body-frame angular velocity (3 dofs);
 *   slide: qpos = displacement along the body-frame axis; qvel = its rate (1 dof). */
#define OSC_KIN_JOINT_NONE (-1)
#define OSC_KIN_JOINT_FREE 0
#define OSC_KIN_JOINT_BALL 1
#define OSC_KIN_JOINT_SLIDE 2
#define OSC_KIN_JOINT_HINGE 3

typedef struct {
  int32_t nbody;                                   /* bodies, world excluded                  */
  int32_t nsite;                                   /* task sites, in the reference's order     */
  double gravity[3];                               /* mjOption::gravity                        */
  int32_t parent[OSC_KIN_MAX_BODIES];              /* body_parentid - 1 (-1 = world)           */
  int32_t jnt_type[OSC_KIN_MAX_BODIES];            /* OSC_KIN_JOINT_*                          */
  double pos[OSC_KIN_MAX_BODIES][3];               /* body_pos  (parent frame)                 */
  double quat[OSC_KIN_MAX_BODIES][4];              /* body_quat (w, x, y, z)                   */
  double axis[OSC_KIN_MAX_BODIES][3];              /* jnt_axis  (body frame; hinge, slide)     */
  double jnt_pos[OSC_KIN_MAX_BODIES][3];           /* jnt_pos   (body frame; hinge/ball anchor)*/
  double armature[OSC_KIN_MAX_BODIES];             /* dof_armature of every dof of the joint   */
  double mass[OSC_KIN_MAX_BODIES];                 /* body_mass                                */
  double ipos[OSC_KIN_MAX_BODIES][3];              /* body_ipos (COM, body frame)              */
  double iquat[OSC_KIN_MAX_BODIES][4];             /* body_iquat (principal axes)              */
  double inertia[OSC_KIN_MAX_BODIES][3];           /* body_inertia (principal moments)         */
  int32_t site_body[OSC_KIN_MAX_SITES];            /* site_bodyid - 1: body carrying the point */
  double site_pos[OSC_KIN_MAX_SITES][3];           /* site_pos (body frame)                    */
  /* Jacobian body of each task site: mj_jac / mj_jacDot take (point = site_xpos, body =
   * body_ids[i]) (operational_space_controller.h:409-412), and body_ids comes from the config's
   * body_list, not from the site.  With has_jac_body = 0 (zero-initialised descriptors) the
   * Jacobian body is site_body; otherwise site_jac_body[k] (the point stays site k's, moving
   * with that body at the current instant -- exactly mj_jac's semantics).  This is how the Go2
   * controller's model-order site rows (osc.h:373) are reproduced: see osc_kin_desc_from_mjcf. */
  int32_t has_jac_body;
  int32_t site_jac_body[OSC_KIN_MAX_SITES];
} osc_kin_desc;

typedef struct osc_kin_model osc_kin_model;        /* opaque: descriptor + device tables */

/* Host-only: fill `desc` from the JSON tree description (operational-space-control_amd/config/
 * <robot>_kinematics.json schema).  `json_path` NULL = <robot>_kinematics.json next to the
 * library's config directory.  OSC_ERR_IO on a missing/malformed file. */
int osc_kin_desc_from_json(const char* robot, const char* json_path, osc_kin_desc* desc);

/* Host-only: fill `desc` from a MuJoCo MJCF file -- the reference's xml_path, which its
 * controller loads with mj_loadXML (operational_space_controller.h:114-152).  The subset of
 * MJCF that update_osc_data's quantities depend on is read: <compiler angle eulerseq
 * inertiafromgeom inertiagrouprange>, <option gravity>, nested <default> classes (childclass /
 * class), <include file> (anywhere, relative to the main file, nested), <body pos + quat | euler |
 * axisangle | xyaxes | zaxis>, <inertial pos, orientation, mass, diaginertia | fullinertia>,
 * inertia from primitive geoms (sphere, capsule, cylinder, box, ellipsoid; mass | density; pos +
 * orientation | fromto) under inertiafromgeom auto (default: bodies without <inertial>) / true,
 * <joint type="free" | "ball" | "slide" | "hinge" axis pos armature> -- several per body, applied
 * in order (the body becomes a chain of one-joint bodies) -- <freejoint>, <site pos | fromto>.
 * Actuators, sensors, contacts, visual/asset sections are skipped (they do not enter M, C, J, b).
 * Bodies are numbered in MuJoCo's depth-first order; sites likewise.
 * Errors (OSC_ERR_IO): unreadable or malformed XML (or included file), mesh / sdf / hfield geoms
 * that would give a body its inertia, a plane geom in a moving body, a non-zero joint ref,
 * compiler settotalmass / boundmass / boundinertia, a ball joint followed by a rotating joint on
 * the same body, a free joint not alone on a top-level body, <frame> / <replicate> /
 * <composite>, unknown names.
 * Task sites: task site k = (point, Jacobian body) with Jacobian body = body_names[k] and
 *   site_order OSC_MJCF_SITES_BY_NAME:     point = the site named site_names[k]
 *                                          (walter_sr: site_xpos(site_ids), W/osc.h:417);
 *   site_order OSC_MJCF_SITES_MODEL_ORDER: point = the k-th site of the model
 *                                          (unitree_go2: Map<Matrix<ns,3>>(site_xpos), G/osc.h:373:
 *                                          rows 0..ns-1 in model order, names not consulted).
 * body_names and site_names are the config's body_list and noncontact_site_list +
 * contact_site_list (G/autogen.py:32-35); each name must exist in the model. */
#define OSC_MJCF_SITES_BY_NAME 0
#define OSC_MJCF_SITES_MODEL_ORDER 1
int osc_kin_desc_from_mjcf(const char* xml_path, const char* const* body_names,
                           const char* const* site_names, int32_t nsite, int32_t site_order,
                           osc_kin_desc* desc);
/* Same with the lists taken from the robot's YAML config (osc_desc_from_yaml's file; NULL = the
 * default one) and the robot's own convention: "unitree_go2" model order, "walter_sr" /
 * "walter_sr_wheels" by name. */
int osc_kin_desc_from_mjcf_robot(const char* robot, const char* yaml_path, const char* xml_path,
                                 osc_kin_desc* desc);

/* Validate (tree order, joint types, sizes, positive masses / inertias, unit-normalisable
 * quaternions and axes), derive the kernel tables and upload them to the current HIP device. */
int osc_kin_model_create(const osc_kin_desc* desc, osc_kin_model** out);
int osc_kin_model_create_from_json(const char* robot, const char* json_path, osc_kin_model** out);
int osc_kin_model_destroy(osc_kin_model* model);

/* nq (generalized coordinates), nv (dofs), nsite of a model. */
int osc_kin_model_dims(const osc_kin_model* model, int32_t* nq, int32_t* nv, int32_t* nsite);

/* Batched kinematics.  Device pointers, env-major, fp64, async on `stream`:
 *   qpos [nenv][nq]  qvel [nenv][nv]                                       (inputs)
 *   M [nenv][nv][nv] (mj_fullM, row-major)  C [nenv][nv] (qfrc_bias)
 *   J [nenv][6 ns][nv] ([Jp_0..Jp_{ns-1}; Jr_0..Jr_{ns-1}])  b [nenv][6 ns] (J-dot qvel)
 *   site_xpos [nenv][ns][3] (nullable)                                     (outputs)
 * M, C, J, b are exactly the inputs osc_batch_solve takes. */
int osc_batch_kinematics(const osc_kin_model* model, int32_t nenv, const double* qpos,
                         const double* qvel, double* M, double* C, double* J, double* b,
                         double* site_xpos, void* stream);

/* update_mj_data's packing (operational_space_controller.h:357-361) for a batch of State
 * structs (containers.h:32-42) held as SoA device arrays:
 *   qpos = [0, 0, 0, body_rotation (w,x,y,z), motor_position],
 *   qvel = [linear_body_velocity, angular_body_velocity, motor_velocity].
 * body_rotation [nenv][4], linear/angular_body_velocity [nenv][3], motor_* [nenv][nu];
 * qpos [nenv][7 + nu], qvel [nenv][6 + nu]. */
int osc_state_to_qpos(int32_t nenv, int32_t nu, const double* body_rotation,
                      const double* linear_body_velocity, const double* angular_body_velocity,
                      const double* motor_position, const double* motor_velocity, double* qpos,
                      double* qvel, void* stream);

/* The whole per-tick path from joint states: osc_batch_kinematics + osc_batch_solve (the
 * reference's update_mj_data .. solve_optimization + torque slice, operational_space_controller.h:
 * 350-573, for every environment).  `kin` must describe the same robot as `model` (kin nv ==
 * model nv, kin nsite == model ns; the contact sites are the model's last nc sites).  Pointers
 * as in osc_batch_solve; `workspace` (16-byte aligned, >= osc_qpos_workspace_bytes) holds the
 * per-env M, C, J, b and the reduced QP; NULL = stream-ordered scratch for this call. */
int osc_qpos_workspace_bytes(const osc_model* model, const osc_kin_model* kin, int32_t nenv,
                             size_t* bytes);
int osc_batch_solve_qpos(const osc_model* model, const osc_kin_model* kin, int32_t nenv,
                         const double* qpos, const double* qvel, const double* T,
                         const double* contact_mask, double* tau, double* x, int32_t* status,
                         int32_t* iters, void* workspace, size_t workspace_bytes, void* stream);
/* Same, warm-started from / updating `warm_state` (osc_batch.h, osc_batch_solve_warm). */
int osc_batch_solve_qpos_warm(const osc_model* model, const osc_kin_model* kin, int32_t nenv,
                              const double* qpos, const double* qvel, const double* T,
                              const double* contact_mask, double* tau, double* x,
                              int32_t* status, int32_t* iters,
                              double* warm_state, size_t warm_state_bytes,
                              void* workspace, size_t workspace_bytes, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* OSC_KINEMATICS_H_ */
