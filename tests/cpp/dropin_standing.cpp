// Drop-in check of the controller API: the controller calls of the reference's
// examples/standing.cc:86-164 (Go2) and examples/walter_sr_standing.cc:88-163 (WaLTER), written
// out with the same includes, namespaces, types and call sequence, compiled against
// include/operational-space-control/<robot>/ and linked with -losc_controller -losc_batch.
// MuJoCo is not in this image: mj_data->qpos / qvel / qfrc_actuator come from files instead of
// a simulation, and the simulated time advances by the control period per loop pass.  Eigen and
// absl are the test stubs under tests/cpp/stubs/ (the image has neither); the headers use only
// Eigen / absl API that exists in both.
//
//   dropin_standing lifecycle <xml>              preconditions, no device needed
//   dropin_standing run <xml> <qpos> <qvel>      the example's loop for a few ticks; prints the
//                                                last targets and torque command as JSON
// Built with -DOSC_DROPIN_ROBOT=0 (unitree_go2), 1 (walter_sr) or 2 (walter_sr_wheels).
#include <chrono>
#include <cstdio>
#include <filesystem>
#include <fstream>
#include <string>
#include <thread>
#include <vector>

#include "absl/status/status.h"
#include "absl/log/absl_check.h"

#include "Eigen/Dense"

#if OSC_DROPIN_ROBOT == 0
#include "operational-space-control/unitree_go2/aliases.h"
#include "operational-space-control/unitree_go2/containers.h"
#include "operational-space-control/unitree_go2/constants.h"
#include "operational-space-control/unitree_go2/operational_space_controller.h"
#elif OSC_DROPIN_ROBOT == 1
#include "operational-space-control/walter_sr/aliases.h"
#include "operational-space-control/walter_sr/containers.h"
#include "operational-space-control/walter_sr/constants.h"
#include "operational-space-control/walter_sr/operational_space_controller.h"
#else
#include "operational-space-control/walter_sr_wheels/aliases.h"
#include "operational-space-control/walter_sr_wheels/containers.h"
#include "operational-space-control/walter_sr_wheels/constants.h"
#include "operational-space-control/walter_sr_wheels/operational_space_controller.h"
#endif

using namespace operational_space_controller::aliases;
using namespace operational_space_controller::containers;
using namespace operational_space_controller::constants;

namespace {

std::vector<double> read_doubles(const char* path) {
  std::ifstream in(path);
  std::vector<double> v;
  double x;
  while (in >> x) v.push_back(x);
  return v;
}

int code(const absl::Status& s) { return static_cast<int>(s.code()); }

int lifecycle(const char* xml) {
  State initial_state;
  initial_state.motor_position = Vector<model::nu_size>::Zero();
  initial_state.motor_velocity = Vector<model::nu_size>::Zero();
  initial_state.body_rotation = Vector<4>{1.0, 0.0, 0.0, 0.0};
  initial_state.linear_body_velocity = Vector<3>::Zero();
  initial_state.angular_body_velocity = Vector<3>::Zero();
  initial_state.contact_mask = Vector<model::contact_site_ids_size>::Constant(1.0);

  OperationalSpaceController missing(std::filesystem::path("/nonexistent/robot.xml"));
  const int load = code(missing.initialize(initial_state));                       // osc.h:114-117
  OperationalSpaceController controller(std::filesystem::path{xml});
  const int pre_opt = code(controller.initialize_optimization());                 // :164-165
  const int pre_thread = code(controller.initialize_thread());                    // :180-182
  const int pre_stop = code(controller.stop_thread());                            // :190-191
  const int pre_clean = code(controller.clean_up());                              // :211-212
  const int init = code(controller.initialize(initial_state));
  Vector<model::nu_size> torque_command = controller.get_torque_command();        // Zero (:244)
  double tnorm = 0.0;
  for (int i = 0; i < model::nu_size; ++i) tnorm += torque_command(i) * torque_command(i);
  std::printf("{\"load\": %d, \"pre_opt\": %d, \"pre_thread\": %d, \"pre_stop\": %d, "
              "\"pre_clean\": %d, \"init\": %d, \"initialized\": %d, \"torque0_norm\": %g, "
              "\"nu\": %d, \"ns\": %d, \"n\": %d}\n",
              load, pre_opt, pre_thread, pre_stop, pre_clean, init,
              controller.is_initialized() ? 1 : 0, tnorm, model::nu_size, model::site_ids_size,
              optimization::design_vector_size);
  return 0;
}

int run(const char* xml, const char* qpos_path, const char* qvel_path) {
  std::vector<double> qpos_file = read_doubles(qpos_path);   // mutable, as mj_data->qpos
  std::vector<double> qvel_file = read_doubles(qvel_path);
  if (static_cast<int>(qpos_file.size()) != model::nq_size ||
      static_cast<int>(qvel_file.size()) != model::nv_size) {
    std::fprintf(stderr, "state files: %zu / %zu values\n", qpos_file.size(), qvel_file.size());
    return 2;
  }
  std::vector<double> qfrc(model::nv_size, 0.0);
  std::filesystem::path osc_model_path = xml;

  // ---- examples/standing.cc:86-117 ----
  OperationalSpaceController controller(
      osc_model_path
  );

  Vector<model::nq_size> qpos = Eigen::Map<Vector<model::nq_size>>(qpos_file.data());
  Vector<model::nv_size> qvel = Eigen::Map<Vector<model::nv_size>>(qvel_file.data());
  Vector<model::nv_size> qfrc_actuator = Eigen::Map<Vector<model::nv_size>>(qfrc.data());
  Vector<3> initial_position = qpos(Eigen::seqN(0, 3));

  State initial_state;
  initial_state.motor_position = qpos(Eigen::seqN(7, model::nu_size));
  initial_state.motor_velocity = qvel(Eigen::seqN(6, model::nu_size));
  initial_state.torque_estimate = qfrc_actuator(Eigen::seqN(6, model::nu_size));
  initial_state.body_rotation = qpos(Eigen::seqN(3, 4));
  initial_state.linear_body_velocity = qvel(Eigen::seqN(0, 3));
  initial_state.angular_body_velocity = qvel(Eigen::seqN(3, 3));
  initial_state.contact_mask = Vector<model::contact_site_ids_size>::Constant(1.0);

  TaskspaceTargets taskspace_targets = Matrix<model::site_ids_size, 6>::Zero();

  absl::Status result;
  result.Update(controller.initialize(initial_state));
  result.Update(controller.initialize_optimization());
  ABSL_CHECK(result.ok()) << result.message();

  controller.update_taskspace_targets(taskspace_targets);
  result.Update(controller.initialize_thread());
  ABSL_CHECK(result.ok()) << result.message();

  // ---- examples/standing.cc:119-164: the control loop (20 passes of 2 ms) ----
  TaskspaceTargets last_targets = TaskspaceTargets::Zero();
  Vector<model::nu_size> torque_command = Vector<model::nu_size>::Zero();
  for (int pass = 0; pass < 20; ++pass) {
    Vector<model::nq_size> qpos = Eigen::Map<Vector<model::nq_size>>(qpos_file.data());
    Vector<model::nv_size> qvel = Eigen::Map<Vector<model::nv_size>>(qvel_file.data());
    Vector<model::nv_size> qfrc_actuator = Eigen::Map<Vector<model::nv_size>>(qfrc.data());

    State state;
    state.motor_position = qpos(Eigen::seqN(7, model::nu_size));
    state.motor_velocity = qvel(Eigen::seqN(6, model::nu_size));
    state.torque_estimate = qfrc_actuator(Eigen::seqN(6, model::nu_size));
    state.body_rotation = qpos(Eigen::seqN(3, 4));
    state.linear_body_velocity = qvel(Eigen::seqN(0, 3));
    state.angular_body_velocity = qvel(Eigen::seqN(3, 3));
    state.contact_mask = Vector<model::contact_site_ids_size>::Constant(1.0);

    controller.update_state(state);

    TaskspaceTargets taskspace_targets = TaskspaceTargets::Zero();
#if OSC_DROPIN_ROBOT == 0
    // Position and Velocity (standing.cc:145-157; commented out in walter_sr_standing.cc)
    Eigen::Quaternion<double> body_rotation = Eigen::Quaternion<double>(state.body_rotation(0), state.body_rotation(1), state.body_rotation(2), state.body_rotation(3));
    Vector<3> body_position = qpos(Eigen::seqN(0, 3));
    Vector<3> position_error = initial_position - body_position;
    Vector<3> velocity_error = Vector<3>::Zero() - state.linear_body_velocity;
    Vector<3> rotation_error = (Eigen::Quaternion<double>(1, 0, 0, 0) * body_rotation.conjugate()).vec();
    Vector<3> angular_velocity_error = Vector<3>::Zero() - state.angular_body_velocity;
    Vector<3> linear_control = 150.0 * (position_error) + 25.0 * (velocity_error);
    Vector<3> angular_control = 50.0 * (rotation_error) + 10.0 * (angular_velocity_error);
    Eigen::Vector<double, 6> cmd {linear_control(0), linear_control(1), linear_control(2), angular_control(0), angular_control(1), angular_control(2)};
    taskspace_targets.row(0) = cmd;
#else
    (void)initial_position;   // walter_sr_standing.cc keeps it too, its PD block commented out
#endif

    controller.update_taskspace_targets(taskspace_targets);

    torque_command = controller.get_torque_command();
    last_targets = taskspace_targets;
    std::this_thread::sleep_for(std::chrono::milliseconds(2));   // mj_step's period
  }
  std::this_thread::sleep_for(std::chrono::milliseconds(30));     // >= 10 ticks on the last inputs
  torque_command = controller.get_torque_command();
  Vector<optimization::design_vector_size> solution = controller.get_solution();

  result.Update(controller.stop_thread());
  ABSL_CHECK(result.ok()) << result.message();

  std::printf("{\"targets\": [");
  for (int i = 0; i < model::site_ids_size * 6; ++i)
    std::printf("%s%.17g", i ? ", " : "", last_targets.data()[i]);
  std::printf("], \"torque\": [");
  for (int i = 0; i < model::nu_size; ++i) std::printf("%s%.17g", i ? ", " : "", torque_command(i));
  std::printf("], \"solution\": [");
  for (int i = 0; i < optimization::design_vector_size; ++i)
    std::printf("%s%.17g", i ? ", " : "", solution(i));
  std::printf("]}\n");
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc >= 3 && std::string(argv[1]) == "lifecycle") return lifecycle(argv[2]);
  if (argc >= 5 && std::string(argv[1]) == "run") return run(argv[2], argv[3], argv[4]);
  std::fprintf(stderr, "usage: dropin_standing lifecycle <xml> | run <xml> <qpos> <qvel>\n");
  return 2;
}
