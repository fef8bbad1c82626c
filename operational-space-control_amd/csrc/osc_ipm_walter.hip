// osc_ipm_walter.hip -- kernel 2 (osc_ipm.hpp) instantiated for the Walter model: every interior-point
// variant launch_ipm<Walter> can pick.  One unit per model so the three compile in parallel.
#include "osc_ipm.hpp"

namespace osc {
template void launch_ipm<Walter>(const LaunchArgs&);
}  // namespace osc
