// osc_multi.hip -- the two-model grids of osc_batch_solve_multi (BASELINE configs[4]: a Go2 shard
// and a WaLTER Sr shard on one GPU): ONE assembly grid (osc_setup_pair_kernel) and ONE
// interior-point grid (osc_ipm_pair_kernel) over both models, the slower model's wavefronts first.
#include "osc_ipm.hpp"
#include "osc_setup.hpp"

namespace osc {

namespace {
template <class DA, class DB>
void launch_pair(const osc_batch_job& a, const osc_batch_job& b, hipStream_t s) {
  auto args = [](const osc_batch_job& j) {
    PairArgs p;
    p.P = j.model->dparams;
    p.nenv = j.nenv;
    p.M = j.M; p.C = j.C; p.J = j.J; p.b = j.b; p.T = j.T; p.mask = j.contact_mask;
    p.ws = static_cast<double*>(j.workspace);
    p.tau = j.tau; p.x = j.x; p.status = j.status; p.iters = j.iters;
    return p;
  };
  const PairArgs A = args(a), B = args(b);
  hipLaunchKernelGGL((osc_setup_pair_kernel<DA, DB>),
                     dim3(static_cast<unsigned>(a.nenv + b.nenv)), dim3(kWave), 0, s, A, B);
  const unsigned nb = static_cast<unsigned>((a.nenv + kEnvPerWave - 1) / kEnvPerWave +
                                            (b.nenv + kEnvPerWave - 1) / kEnvPerWave);
  // one-wave interior point of both models with the refinement in the same wavefront
  if (a.model->refine || b.model->refine)
    hipLaunchKernelGGL((osc_ipm_pair_kernel<DA, DB, kRfFused>), dim3(nb), dim3(kWave), 0, s, A, B);
  else
    hipLaunchKernelGGL((osc_ipm_pair_kernel<DA, DB>), dim3(nb), dim3(kWave), 0, s, A, B);
}
}  // namespace

void launch_pair_walter_go2(const osc_batch_job& w, const osc_batch_job& g, hipStream_t s) {
  launch_pair<Walter, Go2>(w, g, s);
}

}  // namespace osc
