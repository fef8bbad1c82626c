// osc_producers.hip -- batched producers of the solve's per-tick inputs:
// the example drivers' task-space PD targets and contact-mask logic, moved next to the solve so
// a whole control step stays on the device.  Paths relative to the reference repository root.
//
//   osc_pd_base_targets      examples/standing.cc:143-155 (also walter_sr_standing.cc): row 0 of
//                            TaskspaceTargets = [kp_l (p_ref - p) + kd_l (0 - v);
//                                               kp_a vec(q_ref q*) + kd_a (0 - w)], rows 1.. = 0
//   osc_contact_mask_from_contacts
//                            examples/walter_sr_true_tumbling_mjjoint.cc:473-558: a contact site's
//                            mask is 1 iff some active contact of the env involves a geom that
//                            belongs to that contact site's body (either side of the pair)
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
