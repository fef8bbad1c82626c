// osc_ipm_go2.hip -- kernel 2 (osc_ipm.hpp) instantiated for the Go2 model: every interior-point
// variant launch_ipm<Go2> can pick.  One unit per model so the three compile in parallel.
#include "osc_ipm.hpp"

namespace osc {
template void launch_ipm<Go2>(const LaunchArgs&);
}  // namespace osc

#ifdef OSC_STAMPS
// Diagnostic build only: per-block IPM phase cycles [nblocks][kStampSlots] of the last Go2
// interior-point launch (STAMP_* in osc_device.hpp; each kernel unit has its own stamp buffer).
extern "C" int osc_debug_stamps(unsigned long long* host, int nblocks) {
  using namespace osc;
  if (nblocks > kStampBlocks) nblocks = kStampBlocks;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * kStampSlots *
                             nblocks) == hipSuccess ? OSC_OK : OSC_ERR_DEVICE;
}
#endif
