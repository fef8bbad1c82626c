// osc_producers.hip -- batched producers of the solve's per-tick inputs:
// the example drivers' task-space PD targets and contact-mask logic, moved next to the solve so
// a whole control step stays on the device.  Paths relative to the reference repository root.
//
//   osc_pd_base_targets      examples/standing.cc:143-155 (also walter_sr_standing.cc): row 0 of
//                            TaskspaceTargets = [kp_l (p_ref - p) + kd_l (0 - v);
//                                               kp_a vec(q_ref q*) + kd_a (0 - w)], rows 1.. = 0
//   osc_contact_mask_from_contacts
//                            examples/walter_sr_true_tumbling_mjjoint.cc:473-558: a contact site's
//                            mask is 1 iff some active contact of the env involves a geom the
//                            table maps to it (osc_contact_geom_table: the example's rule)
//   osc_tumbling_targets     examples/walter_sr_true_tumbling_mjjoint.cc:622-1019: per-site PD
//                            targets (shin angle, thigh height, torso) with the example's
//                            finite differences against the initial snapshot
//
// Both are HBM-bound elementwise kernels: one thread per environment (PD) / per (env, contact)
// (mask), grid-stride, 256-thread blocks.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "osc_batch.h"
#include "osc_producers.h"

namespace {

constexpr int kBlock = 256;

__global__ __launch_bounds__(kBlock) void pd_base_targets_kernel(
    int nenv, int ns, const double* __restrict__ pos, const double* __restrict__ quat,
    const double* __restrict__ lin_vel, const double* __restrict__ ang_vel,
    const double* __restrict__ pos_ref, int pos_ref_stride, const double* __restrict__ quat_ref,
    int quat_ref_stride, double kp_lin, double kd_lin, double kp_ang, double kd_ang,
    double* __restrict__ T) {
  for (int e = blockIdx.x * kBlock + threadIdx.x; e < nenv; e += gridDim.x * kBlock) {
    const double* p = pos + 3 * static_cast<size_t>(e);
    const double* q = quat + 4 * static_cast<size_t>(e);
    const double* v = lin_vel + 3 * static_cast<size_t>(e);
    const double* w = ang_vel + 3 * static_cast<size_t>(e);
    const double* pr = pos_ref + static_cast<size_t>(pos_ref_stride) * e;
    const double* qr = quat_ref + static_cast<size_t>(quat_ref_stride) * e;
    double* t = T + static_cast<size_t>(e) * ns * 6;
    // rotation error = vec(q_ref * conj(q))  (Eigen: quaternions (w, x, y, z))
    const double aw = qr[0], ax = qr[1], ay = qr[2], az = qr[3];
    const double bw = q[0], bx = -q[1], by = -q[2], bz = -q[3];
    const double rx = aw * bx + ax * bw + ay * bz - az * by;
    const double ry = aw * by - ax * bz + ay * bw + az * bx;
    const double rz = aw * bz + ax * by - ay * bx + az * bw;
    t[0] = kp_lin * (pr[0] - p[0]) + kd_lin * (0.0 - v[0]);
    t[1] = kp_lin * (pr[1] - p[1]) + kd_lin * (0.0 - v[1]);
    t[2] = kp_lin * (pr[2] - p[2]) + kd_lin * (0.0 - v[2]);
    t[3] = kp_ang * rx + kd_ang * (0.0 - w[0]);
    t[4] = kp_ang * ry + kd_ang * (0.0 - w[1]);
    t[5] = kp_ang * rz + kd_ang * (0.0 - w[2]);
    for (int i = 6; i < 6 * ns; ++i) t[i] = 0.0;   // TaskspaceTargets::Zero() for other sites
  }
}

__global__ __launch_bounds__(kBlock) void contact_mask_kernel(
    int nenv, int nc, int max_con, const int32_t* __restrict__ ncon,
    const int32_t* __restrict__ geom_pairs, int ngeom, const int32_t* __restrict__ geom_to_site,
    double* __restrict__ mask) {
  const long long total = static_cast<long long>(nenv) * nc;
  for (long long idx = static_cast<long long>(blockIdx.x) * kBlock + threadIdx.x; idx < total;
       idx += static_cast<long long>(gridDim.x) * kBlock) {
    const int e = static_cast<int>(idx / nc), k = static_cast<int>(idx % nc);
    int n = ncon[e];
    n = n < 0 ? 0 : (n > max_con ? max_con : n);
    const int32_t* g = geom_pairs + static_cast<size_t>(e) * max_con * 2;
    double m = 0.0;
    for (int c = 0; c < n; ++c) {
      const int g0 = g[2 * c], g1 = g[2 * c + 1];
      const bool hit0 = g0 >= 0 && g0 < ngeom && geom_to_site[g0] == k;
      const bool hit1 = g1 >= 0 && g1 < ngeom && geom_to_site[g1] == k;
      if (hit0 || hit1) m = 1.0;
    }
    mask[idx] = m;
  }
}

// Tumbling driver's per-site targets (walter_sr_true_tumbling_mjjoint.cc:622-1019), one thread
// per environment.  Site rows: 0 torso, 1-4 shins, 5-8 thighs, 9-16 wheels (site_ids order).
__global__ __launch_bounds__(kBlock) void tumbling_targets_kernel(
    int nenv, int ns, int nq, int nv, const double* __restrict__ qpos,
    const double* __restrict__ qvel, const double* __restrict__ site_xpos,
    const double* __restrict__ tnow, const double* __restrict__ tstart,
    const double* __restrict__ init_qpos, const double* __restrict__ init_site_xpos,
    osc_tumbling_params P, double* __restrict__ T) {
  for (int e = blockIdx.x * kBlock + threadIdx.x; e < nenv; e += gridDim.x * kBlock) {
    const double* q = qpos + static_cast<size_t>(e) * nq;
    const double* q0 = init_qpos + static_cast<size_t>(e) * nq;
    const double* v = qvel + static_cast<size_t>(e) * nv;
    const double* x = site_xpos + static_cast<size_t>(e) * ns * 3;
    const double* x0 = init_site_xpos + static_cast<size_t>(e) * ns * 3;
    const double t = tnow[e], dt = t - tstart[e];
    double* o = T + static_cast<size_t>(e) * ns * 6;
    for (int i = 0; i < 6 * ns; ++i) o[i] = 0.0;
    // shins (:694-802): angular-y command from the shin joint angle
    for (int i = 0; i < 4; ++i) {
      const double th = q[P.shin_qadr[i]], th0 = q0[P.shin_qadr[i]];
      const double w = (th - th0) / dt;
      const double target = th0 + P.shin_rot_vel * t;
      o[6 * (1 + i) + 4] = P.shin_kp * (target - th) + P.shin_kv * (P.shin_rot_vel - w);
    }
    // thighs (:866-973): linear-z command from the thigh site height
    for (int i = 0; i < 4; ++i) {
      const int r = 5 + i;
      const double z = x[3 * r + 2], z0 = x0[3 * r + 2];
      const double vz = (z - z0) / dt;
      const double err = (z0 - 0.0 + P.thigh_height_offset) - z;
      o[6 * r + 2] = P.thigh_lin_kp * err + P.thigh_lin_kv * (P.thigh_lin_vel - vz);
    }
    // torso (:981-1019): [lin_x, 0, 0, ang_x, ang_y, ang_z]
    {
      const double pe = (q0[0] + P.torso_lin_vel * t) - q[0];
      const double ve = P.torso_lin_vel - v[0];
      // rotation_error = vec(identity * conj(body_rotation)) = -(x, y, z) of (w, x, y, z)
      const double re[3] = {-q[4], -q[5], -q[6]};
      o[0] = P.torso_lin_kp * pe + P.torso_lin_kv * ve;
      for (int k = 0; k < 3; ++k)
        o[3 + k] = P.torso_ang_kp * re[k] + P.torso_ang_kv * (0.0 - v[3 + k]);
    }
  }
}

unsigned grid_for(long long n) {
  long long b = (n + kBlock - 1) / kBlock;
  if (b > 65535LL * 8) b = 65535LL * 8;
  return static_cast<unsigned>(b < 1 ? 1 : b);
}

}  // namespace

extern "C" int osc_pd_base_targets(int32_t nenv, int32_t ns, const double* base_pos,
                                   const double* base_quat, const double* lin_vel,
                                   const double* ang_vel, const double* pos_ref,
                                   int32_t pos_ref_per_env, const double* quat_ref,
                                   int32_t quat_ref_per_env, const double* gains,
                                   double* targets, void* stream) {
  if (nenv < 0 || ns < 1 || !gains) return OSC_ERR_INVALID_ARGUMENT;
  if (nenv == 0) return OSC_OK;
  if (!base_pos || !base_quat || !lin_vel || !ang_vel || !pos_ref || !quat_ref || !targets)
    return OSC_ERR_INVALID_ARGUMENT;
  hipLaunchKernelGGL(pd_base_targets_kernel, dim3(grid_for(nenv)), dim3(kBlock), 0,
                     static_cast<hipStream_t>(stream), nenv, ns, base_pos, base_quat, lin_vel,
                     ang_vel, pos_ref, pos_ref_per_env ? 3 : 0, quat_ref, quat_ref_per_env ? 4 : 0,
                     gains[0], gains[1], gains[2], gains[3], targets);
  return hipGetLastError() == hipSuccess ? OSC_OK : OSC_ERR_DEVICE;
}

extern "C" int osc_contact_mask_from_contacts(int32_t nenv, int32_t nc, int32_t max_con,
                                              const int32_t* ncon, const int32_t* geom_pairs,
                                              int32_t ngeom, const int32_t* geom_to_site,
                                              double* contact_mask, void* stream) {
  if (nenv < 0 || nc < 0 || max_con < 0 || ngeom < 0) return OSC_ERR_INVALID_ARGUMENT;
  if (nenv == 0 || nc == 0) return OSC_OK;
  if (!ncon || (max_con > 0 && !geom_pairs) || (ngeom > 0 && !geom_to_site) || !contact_mask)
    return OSC_ERR_INVALID_ARGUMENT;
  hipLaunchKernelGGL(contact_mask_kernel, dim3(grid_for(static_cast<long long>(nenv) * nc)),
                     dim3(kBlock), 0, static_cast<hipStream_t>(stream), nenv, nc, max_con, ncon,
                     geom_pairs, ngeom, geom_to_site, contact_mask);
  return hipGetLastError() == hipSuccess ? OSC_OK : OSC_ERR_DEVICE;
}

extern "C" int osc_contact_geom_table(int32_t ngeom, const int32_t* geom_bodyid, int32_t nsite,
                                      const int32_t* site_bodyid, int32_t nc, const int32_t* ids,
                                      int32_t* geom_to_site) {
  if (ngeom < 0 || nsite < 0 || nc < 0) return OSC_ERR_INVALID_ARGUMENT;
  if (ngeom > 0 && (!geom_bodyid || !geom_to_site)) return OSC_ERR_INVALID_ARGUMENT;
  if ((nsite > 0 && !site_bodyid) || (nc > 0 && !ids)) return OSC_ERR_INVALID_ARGUMENT;
  for (int g = 0; g < ngeom; ++g) {
    geom_to_site[g] = -1;
    bool listed = false;   // role (1): the GEOM id is in the list (:526, :538)
    for (int k = 0; k < nc; ++k) listed = listed || ids[k] == g;
    if (!listed) continue;
    int first = -1;        // getSiteIdsOnSameBodyAsGeom(g)[0] (:106-149, :529, :541)
    for (int s = 0; s < nsite && first < 0; ++s)
      if (site_bodyid[s] == geom_bodyid[g]) first = s;
    if (first < 0) continue;
    for (int k = 0; k < nc; ++k)   // role (2): the SITE id's position in the list (:152-163)
      if (ids[k] == first) {
        geom_to_site[g] = k;
        break;
      }
  }
  return OSC_OK;
}

extern "C" void osc_tumbling_params_default(osc_tumbling_params* p) {
  if (!p) return;
  p->shin_rot_vel = 0.1 * 8.0 * 5.0;
  p->shin_kp = 800.0 * 3.0;
  p->shin_kv = 800.0 * 3.0;
  p->thigh_lin_vel = 0.0;
  p->thigh_lin_kp = 4000.0 * 0.5;
  p->thigh_lin_kv = 600.0 * 0.5;
  p->thigh_height_offset = -0.025;
  p->torso_lin_vel = 0.2;
  p->torso_lin_kp = 0.0;
  p->torso_lin_kv = 0.0;
  p->torso_ang_kp = 0.0;
  p->torso_ang_kv = 0.0;
  const int32_t adr[4] = {8, 10, 12, 14};
  for (int i = 0; i < 4; ++i) p->shin_qadr[i] = adr[i];
}

extern "C" int osc_tumbling_targets(int32_t nenv, int32_t ns, int32_t nq, int32_t nv,
                                    const double* qpos, const double* qvel, const double* site_xpos,
                                    const double* t, const double* t0, const double* init_qpos,
                                    const double* init_site_xpos, const osc_tumbling_params* params,
                                    double* targets, void* stream) {
  if (nenv < 0 || ns != 17 || nq < 7 || nv < 6 || !params) return OSC_ERR_INVALID_ARGUMENT;
  for (int i = 0; i < 4; ++i)
    if (params->shin_qadr[i] < 7 || params->shin_qadr[i] >= nq) return OSC_ERR_INVALID_ARGUMENT;
  if (nenv == 0) return OSC_OK;
  if (!qpos || !qvel || !site_xpos || !t || !t0 || !init_qpos || !init_site_xpos || !targets)
    return OSC_ERR_INVALID_ARGUMENT;
  hipLaunchKernelGGL(tumbling_targets_kernel, dim3(grid_for(nenv)), dim3(kBlock), 0,
                     static_cast<hipStream_t>(stream), nenv, ns, nq, nv, qpos, qvel, site_xpos, t,
                     t0, init_qpos, init_site_xpos, *params, targets);
  return hipGetLastError() == hipSuccess ? OSC_OK : OSC_ERR_DEVICE;
}
