// osc_ipm_wheels.hip -- kernel 2 (osc_ipm.hpp) instantiated for the WalterW model: every interior-point
// variant launch_ipm<WalterW> can pick.  One unit per model so the three compile in parallel.
#include "osc_ipm.hpp"

namespace osc {
template void launch_ipm<WalterW>(const LaunchArgs&);
}  // namespace osc
