// osc_multi.hip -- the two-model grids of osc_batch_solve_multi (BASELINE configs[4]: a Go2 shard
// and a WaLTER Sr shard on one GPU): ONE assembly grid (osc_setup_pair_kernel) and ONE
// interior-point grid (osc_ipm_pair_kernel) over both models, the slower model's wavefronts first.
#include "osc_ipm.hpp"
#include "osc_setup.hpp"

namespace osc {

namespace {
template <class DA, class DB>
void launch_pair(const osc_batch_job& a, const osc_batch_job& b, hipStream_t s) {
  // (the fix-up pass reads each env's status: the caller's array, else the workspace's scratch
  // after the per-env blocks, as launch_t places it)
  auto args = [](const osc_batch_job& j, int ws_doubles) {
    PairArgs p;
    p.P = j.model->dparams;
    p.nenv = j.nenv;
    p.M = j.M; p.C = j.C; p.J = j.J; p.b = j.b; p.T = j.T; p.mask = j.contact_mask;
    p.ws = static_cast<double*>(j.workspace);
    p.tau = j.tau; p.x = j.x; p.iters = j.iters;
    p.status = j.status ? j.status
                        : reinterpret_cast<int32_t*>(p.ws + static_cast<size_t>(ws_doubles) * j.nenv);
    return p;
  };
  const PairArgs A = args(a, DA::WS), B = args(b, DB::WS);
  hipLaunchKernelGGL((osc_setup_pair_kernel<DA, DB>),
                     dim3(static_cast<unsigned>(a.nenv + b.nenv)), dim3(kWave), 0, s, A, B);
  const unsigned nb = static_cast<unsigned>((a.nenv + kEnvPerWave - 1) / kEnvPerWave +
                                            (b.nenv + kEnvPerWave - 1) / kEnvPerWave);
  // one-wave interior point of both models with the refinement in the same wavefront
  // (then the cold fix-up pass over the envs the solve left not OK, as launch_ipm's entries do)
  if (a.model->refine || b.model->refine) {
    hipLaunchKernelGGL((osc_ipm_pair_kernel<DA, DB, kRfFused>), dim3(nb), dim3(kWave), 0, s, A, B,
                       0);
    hipLaunchKernelGGL((osc_ipm_pair_kernel<DA, DB, kRfFused>), dim3(nb), dim3(kWave), 0, s, A, B,
                       1);
  } else {
    hipLaunchKernelGGL((osc_ipm_pair_kernel<DA, DB>), dim3(nb), dim3(kWave), 0, s, A, B, 0);
  }
}
}  // namespace

void launch_pair_walter_go2(const osc_batch_job& w, const osc_batch_job& g, hipStream_t s) {
  launch_pair<Walter, Go2>(w, g, s);
}

}  // namespace osc
