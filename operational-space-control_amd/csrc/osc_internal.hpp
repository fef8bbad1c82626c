// osc_internal.hpp -- host-side internals shared by the C-ABI unit (osc_api.hip) and the kernel
// units: the model handle, the arguments of one batched call, and each kernel unit's launcher.
// The launchers are explicitly instantiated in their own units (a HIP kernel can only be launched
// from the translation unit that holds its device code: no relocatable device code here).
#pragma once
#include "osc_device.hpp"
#include "osc_qpos.hpp"

struct osc_model {
  osc_model_desc desc;
  osc::KernelId kid;
  osc::DevParams* dparams;
  int device;
  int small_batch_max;   // envs that fit one wavefront per SIMD (4 per wave x 4 SIMDs x CUs)
  bool refine;           // torque-coordinate model with refinement steps > 0
  int resident_envs;     // envs of one wavefront per SIMD over the whole device
  int park_it;           // compaction's park iteration (0: off; ParkArgs)
};

namespace osc {

// One batched call (device pointers; nullable as in include/osc_batch.h).  `status` is the
// caller's array or, where a later pass needs per-env statuses, scratch in the workspace.
struct LaunchArgs {
  const osc_model* model;
  int32_t nenv;
  const double *M, *C, *J, *b, *T, *mask;
  double* tau;
  double* x;
  int32_t* status;
  int32_t* iters;
  double* ws;
  double* warm;          // warm state, nullable (cold solve)
  hipStream_t s;
  const double* wdir;    // wheel directions (wheel-row models)
  double* y;             // duals, nullable
};

template <class D> void launch_setup(const LaunchArgs& a);   // osc_setup.hip
template <class D> void launch_setup_qpos(const LaunchArgs& a, const QposArgs& q);   // (fused tick;
                                                        // no wheel-row model: no directions)
template <class D> void launch_ipm(const LaunchArgs& a);     // osc_ipm_<model>.hip
template <class D> void launch_dual(const LaunchArgs& a);    // osc_dual.hip
template <class D> void launch_gi(const LaunchArgs& a);      // osc_gi.hip
// osc_multi.hip: WaLTER's job and Go2's job in one assembly grid and one interior-point grid
void launch_pair_walter_go2(const osc_batch_job& w, const osc_batch_job& g, hipStream_t s);

extern template void launch_setup<Go2>(const LaunchArgs&);
extern template void launch_setup<Walter>(const LaunchArgs&);
extern template void launch_setup<WalterW>(const LaunchArgs&);
#ifdef OSC_FUSED_TICK
extern template void launch_setup_qpos<Go2>(const LaunchArgs&, const QposArgs&);
extern template void launch_setup_qpos<Walter>(const LaunchArgs&, const QposArgs&);
#endif
extern template void launch_ipm<Go2>(const LaunchArgs&);
extern template void launch_ipm<Walter>(const LaunchArgs&);
extern template void launch_ipm<WalterW>(const LaunchArgs&);
extern template void launch_dual<Go2>(const LaunchArgs&);
extern template void launch_dual<Walter>(const LaunchArgs&);
extern template void launch_dual<WalterW>(const LaunchArgs&);
extern template void launch_gi<WalterW>(const LaunchArgs&);

}  // namespace osc
