// osc_ipm_go2.hip -- kernel 2 (osc_ipm.hpp) instantiated for the Go2 model: every interior-point
// variant launch_ipm<Go2> can pick.  One unit per model so the three compile in parallel.
#include "osc_ipm.hpp"

namespace osc {
template void launch_ipm<Go2>(const LaunchArgs&);
}  // namespace osc
