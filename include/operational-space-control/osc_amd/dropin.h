/*
 * dropin.h -- shared implementation of the drop-in controller headers
 *   operational-space-control/{unitree_go2,walter_sr,walter_sr_wheels}/
 *       {aliases,containers,constants,operational_space_controller}.h
 * which give the examples/ programs the reference's public controller API (SURVEY.md §8(b);
 * unitree_go2/operational_space_controller.h:106-238) on top of the MI355X library:
 * libosc_controller.so (include/osc_controller.h) -> libosc_batch.so (include/osc_batch.h).
 *
 * Types are the reference's: Eigen row-major matrices / column vectors sized by the robot's
 * constexpr constants, absl::Status for the lifecycle calls.  The Eigen and absl headers are the
 * caller's own (the reference's build already provides them); only Matrix<...>::data(), size()
 * and Zero(), and absl::OkStatus / InternalError / FailedPreconditionError /
 * InvalidArgumentError are used here.
 *
 * What happens underneath: the xml_path given to the constructor is read by initialize() with the
 * library's MJCF reader (osc_kin_desc_from_mjcf_robot: bodies, joints, inertias, task sites by
 * the robot's config lists), the QP weights come from the robot's YAML config next to the
 * library (osc_desc_from_yaml), and every control tick is State -> qpos/qvel (update_mj_data's
 * packing) -> GPU kinematics -> reduced QP -> interior point -> torque on a private HIP stream,
 * warm-started from the previous tick (the reference's SetWarmStart).  OsqpSettings is accepted
 * for signature compatibility; the interior point returns the QP's optimum to 1e-12
 * complementarity, which is tighter than any OSQP eps.
 */
#pragma once

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <filesystem>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "Eigen/Dense"
#include "absl/status/status.h"

#include "osc_controller.h"

#ifndef OSC_AMD_HAVE_OSQP_SETTINGS
#define OSC_AMD_HAVE_OSQP_SETTINGS
namespace osqp {
/* Field names and defaults of osqp-cpp's OsqpSettings (osqp 0.6.3 defaults).  Define
 * OSC_AMD_HAVE_OSQP_SETTINGS before including a controller header to use osqp++.h's own. */
struct OsqpSettings {
  double rho = 0.1;
  double sigma = 1e-6;
  int scaling = 10;
  bool adaptive_rho = true;
  int adaptive_rho_interval = 0;
  double adaptive_rho_tolerance = 5.0;
  double adaptive_rho_fraction = 0.4;
  int max_iter = 4000;
  double eps_abs = 1e-3;
  double eps_rel = 1e-3;
  double eps_prim_inf = 1e-4;
  double eps_dual_inf = 1e-4;
  double alpha = 1.6;
  double delta = 1e-6;
  bool polish = false;
  int polish_refine_iter = 3;
  bool verbose = true;
  bool scaled_termination = false;
  int check_termination = 25;
  bool warm_start = true;
  double time_limit = 0.0;
};
}  // namespace osqp
#endif
using osqp::OsqpSettings;   // the reference's header brings it in with `using namespace osqp`

namespace osc_amd::dropin {

inline absl::Status to_absl(const osc_amd::Status& s) {
  switch (s.code()) {
    case osc_amd::Status::kOk: return absl::OkStatus();
    case osc_amd::Status::kFailedPrecondition: return absl::FailedPreconditionError(s.message());
    case osc_amd::Status::kInvalidArgument: return absl::InvalidArgumentError(s.message());
    default: return absl::InternalError(s.message());
  }
}

template <class M>
std::vector<double> flat(const M& m) {   // row-major for the RowMajor aliases (aliases.h)
  return std::vector<double>(m.data(), m.data() + m.size());
}

// The library's vector for an Eigen type: empty before the first solve (the reference's Zero()
// then), else exactly the type's size -- a mismatch means the header and libosc_controller.so
// disagree on the robot's dimensions, which must not surface as plausible zero torques.
template <class M>
M unflat(const std::vector<double>& v) {
  M m = M::Zero();
  if (v.empty()) return m;
  if (static_cast<std::ptrdiff_t>(v.size()) != static_cast<std::ptrdiff_t>(m.size())) {
    std::fprintf(stderr, "osc_amd::dropin: library returned %zu values for a %td-element type\n",
                 v.size(), static_cast<std::ptrdiff_t>(m.size()));
    std::abort();
  }
  std::copy(v.begin(), v.end(), m.data());
  return m;
}

/* The controller behind every robot's OperationalSpaceController: one robot's State /
 * TaskspaceTargets / torque / solution types, the reference's method set. */
template <class State, class Targets, class Torque, class Solution>
class Controller {
 public:
  Controller(const char* robot, const std::filesystem::path& xml_path, int control_rate_us)
      : impl_(std::make_unique<osc_amd::OperationalSpaceController>(
            robot, std::string(), control_rate_us, xml_path.string())) {}

  absl::Status initialize(State initial_state) { return to_absl(impl_->initialize(convert(initial_state))); }
  absl::Status initialize_optimization() { return to_absl(impl_->initialize_optimization()); }
  absl::Status initialize_thread() { return to_absl(impl_->initialize_thread()); }
  absl::Status stop_thread() { return to_absl(impl_->stop_thread()); }
  absl::Status clean_up() { return to_absl(impl_->clean_up()); }
  bool is_initialized() { return impl_->is_initialized(); }
  bool is_optimization_initialized() { return impl_->is_optimization_initialized(); }
  bool is_thread_initialized() { return impl_->is_thread_initialized(); }

  void update_state(const State& new_state) { impl_->update_state(convert(new_state)); }
  void update_taskspace_targets(const Targets& targets) { impl_->update_taskspace_targets(flat(targets)); }
  Torque get_torque_command() { return unflat<Torque>(impl_->get_torque_command()); }
  Solution get_solution() { return unflat<Solution>(impl_->get_solution()); }

 private:
  static osc_amd::State convert(const State& s) {
    osc_amd::State o;
    o.motor_position = flat(s.motor_position);
    o.motor_velocity = flat(s.motor_velocity);
    o.motor_acceleration = flat(s.motor_acceleration);
    o.torque_estimate = flat(s.torque_estimate);
    o.body_rotation = flat(s.body_rotation);
    o.linear_body_velocity = flat(s.linear_body_velocity);
    o.angular_body_velocity = flat(s.angular_body_velocity);
    o.linear_body_acceleration = flat(s.linear_body_acceleration);
    o.contact_mask = flat(s.contact_mask);
    return o;
  }

  std::unique_ptr<osc_amd::OperationalSpaceController> impl_;
};

}  // namespace osc_amd::dropin
