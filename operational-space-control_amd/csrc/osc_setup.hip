// osc_setup.hip -- kernel 1 (osc_setup.hpp) instantiated for every model: launch_setup builds
// each environment's reduced QP into the workspace (one 64-lane wavefront per environment).
#include "osc_internal.hpp"
#include "osc_setup.hpp"

namespace osc {

// one env per 64-lane wavefront (four envs per wavefront measured no faster: Go2 4,096
// 35.3 vs 33.7 us)
// (the models without MFMA assembly -- Go2 -- take the lean variant, osc_setup.hpp setup_env's
// LEAN, at every batch size: 100 VGPRs and 10.2 KB of LDS fit all of 4,096 envs' waves at once;
// against the full variant 4,096 / 2,048 -1.8 / -0.1 %, profiles/r06/lean_lds/)
template <class D>
void launch_setup(const LaunchArgs& a) {
  const dim3 grid(static_cast<unsigned>(a.nenv));
  hipLaunchKernelGGL((osc_setup_kernel<D, !D::JG>), grid, dim3(kWave), 0, a.s, a.model->dparams,
                     a.nenv, a.M, a.C, a.J, a.b, a.T, a.mask, a.ws, a.wdir);
}

template void launch_setup<Go2>(const LaunchArgs&);
template void launch_setup<Walter>(const LaunchArgs&);
template void launch_setup<WalterW>(const LaunchArgs&);

#ifdef OSC_FUSED_TICK
// the fused joint-state tick: the same assembly with the kinematics in its prologue (A/B builds
// only: measured slower than the two-kernel tick, osc_kinematics.hip solve_qpos)
template <class D>
void launch_setup_qpos(const LaunchArgs& a, const QposArgs& q) {
  const size_t lds = sizeof(double) * static_cast<size_t>(kin_lds_doubles<D>(q.nq, q.nbody));
  hipLaunchKernelGGL(osc_setup_qpos_kernel<D>, dim3(static_cast<unsigned>(a.nenv)), dim3(kWave),
                     lds, a.s, a.model->dparams, a.nenv, q.kin, q.qpos, q.qvel, a.T, a.mask, a.ws,
                     a.wdir);
}

template void launch_setup_qpos<Go2>(const LaunchArgs&, const QposArgs&);
template void launch_setup_qpos<Walter>(const LaunchArgs&, const QposArgs&);
#endif

}  // namespace osc
