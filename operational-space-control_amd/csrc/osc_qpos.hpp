// osc_qpos.hpp -- the fused joint-state tick's internal entry (osc_api.hip; -DOSC_FUSED_TICK
// builds only): osc_batch_solve_qpos(_warm) with the kinematics in the assembly kernel's prologue
// (osc_setup.hpp, setup_env<D, true>), then the interior point as for osc_batch_solve(_warm).
// Bitwise the two-kernel tick's results, measured slower (osc_kinematics.hip solve_qpos).
#pragma once
#include <cstddef>
#include <cstdint>

#include "osc_batch.h"

namespace osc_kin {
struct KinDev;
}

namespace osc {

struct QposArgs {
  const osc_kin::KinDev* kin;   // device tables of the kinematics model (osc_kin_model)
  int32_t nq, nbody;            // its sizes (the per-env LDS state of the prologue)
  const double* qpos;           // [nenv][nq] DEVICE
  const double* qvel;           // [nenv][nv] DEVICE
};

// osc_batch_solve (warm == nullptr) or osc_batch_solve_warm with M, C, J, b computed in the
// assembly kernel from qpos / qvel; `workspace` as osc_batch_solve's (required).
int solve_qpos_fused(const osc_model* model, const QposArgs& q, int32_t nenv, const double* T,
                     const double* contact_mask, double* tau, double* x, int32_t* status,
                     int32_t* iters, double* warm, size_t warm_bytes, void* workspace,
                     size_t workspace_bytes, void* stream);

}  // namespace osc
