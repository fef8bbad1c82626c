// osc_setup.hip -- kernel 1 (osc_setup.hpp) instantiated for every model: launch_setup builds
// each environment's reduced QP into the workspace (one 64-lane wavefront per environment).
#include "osc_internal.hpp"
#include "osc_setup.hpp"

namespace osc {

// one env per 64-lane wavefront (four envs per wavefront measured no faster: Go2 4,096
// 35.3 vs 33.7 us)
template <class D>
void launch_setup(const LaunchArgs& a) {
  hipLaunchKernelGGL(osc_setup_kernel<D>, dim3(static_cast<unsigned>(a.nenv)), dim3(kWave), 0, a.s,
                     a.model->dparams, a.nenv, a.M, a.C, a.J, a.b, a.T, a.mask, a.ws, a.wdir);
}

template void launch_setup<Go2>(const LaunchArgs&);
template void launch_setup<Walter>(const LaunchArgs&);
template void launch_setup<WalterW>(const LaunchArgs&);

}  // namespace osc

#ifdef OSC_STAMPS
// Diagnostic build only: per-block setup phase cycles [nblocks][kStampSlots], slots 0-5 used.
extern "C" int osc_debug_setup_stamps(unsigned long long* host, int nblocks) {
  using namespace osc;
  if (nblocks > kStampBlocks) nblocks = kStampBlocks;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_setup_stamps), sizeof(unsigned long long) *
                             kStampSlots * nblocks) == hipSuccess ? OSC_OK : OSC_ERR_DEVICE;
}
#endif
