// Test driver for include/osc_controller.h (run by tests/test_controller_shim.py).
//   osc_controller_test lifecycle <robot>
//       precondition / argument errors of the reference's lifecycle (operational_space_
//       controller.h:112-218); initialize_optimization's result is printed (no GPU -> Internal)
//   osc_controller_test solve <robot> <fixture.bin>
//       fixture = raw fp64: M | C | J | b | T | mask | tau_ref  for one environment; the
//       kinematics provider returns the fixture's M, C, J, b.  One synchronous tick, then the
//       control thread at 2000 us for ~60 ms.  Prints one JSON line.
//   osc_controller_test qpos <robot> <fixture.bin>
//       the GPU-kinematics controller (no KinematicsFn): fixture = raw fp64
//       qpos | qvel | T | mask | tau_ref; the State is unpacked from qpos/qvel as update_mj_data
//       packs it (osc.h:357-361).  One tick + ~60 ms of the control thread.
//   osc_controller_test gpu_lifecycle <robot>
//       argument errors of the GPU-kinematics controller (State sizes, missing tree).
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <string>
#include <thread>
#include <vector>

#include "osc_controller.h"

using osc_amd::OSCData;

static bool g_tick_graph = false;   // set_tick_graph (main's optional 4th argument)
using osc_amd::OperationalSpaceController;
using osc_amd::State;
using osc_amd::Status;

static State make_state(int nu, int nc, double mask) {
  State s;
  s.motor_position.assign(nu, 0.0);
  s.motor_velocity.assign(nu, 0.0);
  s.motor_acceleration.assign(nu, 0.0);
  s.torque_estimate.assign(nu, 0.0);
  s.body_rotation = {1.0, 0.0, 0.0, 0.0};
  s.linear_body_velocity.assign(3, 0.0);
  s.angular_body_velocity.assign(3, 0.0);
  s.linear_body_acceleration.assign(3, 0.0);
  s.contact_mask.assign(nc, mask);
  return s;
}

static int lifecycle(const std::string& robot) {
  osc_model_desc d;
  if (osc_desc_from_yaml(robot.c_str(), nullptr, &d) != OSC_OK) return 2;
  auto kin = [](const State&, OSCData*) { return Status::Ok(); };
  OperationalSpaceController c(robot, "", kin);
  const int pre_opt = c.initialize_optimization().code();
  const int pre_thread = c.initialize_thread().code();
  const int pre_stop = c.stop_thread().code();
  const int pre_clean = c.clean_up().code();
  const int bad_mask = c.initialize(make_state(d.nu, d.nc + 1, 1.0)).code();
  const int init = c.initialize(make_state(d.nu, d.nc, 1.0)).code();
  const int thread_before_opt = c.initialize_thread().code();
  const int step_before_opt = c.step().code();
  const Status opt = c.initialize_optimization();
  OperationalSpaceController bad("no_such_robot", "", kin);
  const int bad_robot = bad.initialize(make_state(d.nu, d.nc, 1.0)).code();
  std::printf("{\"pre_opt\": %d, \"pre_thread\": %d, \"pre_stop\": %d, \"pre_clean\": %d, "
              "\"bad_mask\": %d, \"init\": %d, \"thread_before_opt\": %d, "
              "\"step_before_opt\": %d, \"opt\": %d, \"bad_robot\": %d, \"torque0\": %zu, "
              "\"initialized\": %d, \"opt_initialized\": %d}\n",
              pre_opt, pre_thread, pre_stop, pre_clean, bad_mask, init, thread_before_opt,
              step_before_opt, opt.code(), bad_robot, c.get_torque_command().size(),
              c.is_initialized() ? 1 : 0, c.is_optimization_initialized() ? 1 : 0);
  return 0;
}

static int solve(const std::string& robot, const std::string& path) {
  osc_model_desc d;
  if (osc_desc_from_yaml(robot.c_str(), nullptr, &d) != OSC_OK) return 2;
  const size_t nv = d.nv, nu = d.nu, nc = d.nc, s = 6 * size_t(d.ns);
  const size_t sizes[7] = {nv * nv, nv, s * nv, s, size_t(d.ns) * 6, nc, nu};
  std::vector<std::vector<double>> f(7);
  std::ifstream in(path, std::ios::binary);
  for (int k = 0; k < 7; ++k) {
    f[k].resize(sizes[k]);
    in.read(reinterpret_cast<char*>(f[k].data()), sizes[k] * sizeof(double));
  }
  if (!in) return 3;
  std::atomic<int> calls{0};
  auto kin = [&](const State&, OSCData* o) {
    ++calls;
    o->mass_matrix = f[0];
    o->coriolis_matrix = f[1];
    o->taskspace_jacobian = f[2];
    o->taskspace_bias = f[3];
    return Status::Ok();
  };
  OperationalSpaceController c(robot, "", kin, 2000);
  c.set_tick_graph(g_tick_graph);
  State st = make_state(d.nu, d.nc, 1.0);
  st.contact_mask = f[5];
  Status r = c.initialize(st);
  if (!r.ok()) { std::printf("{\"error\": \"%s\"}\n", r.message().c_str()); return 4; }
  r = c.initialize_optimization();
  if (!r.ok()) { std::printf("{\"error\": \"%s\"}\n", r.message().c_str()); return 5; }
  c.update_taskspace_targets(f[4]);
  r = c.step();
  if (!r.ok()) { std::printf("{\"error\": \"%s\"}\n", r.message().c_str()); return 6; }
  auto err = [&](const std::vector<double>& tau) {
    double e = 0, nrm = 1.0;
    for (size_t i = 0; i < nu; ++i) nrm = std::fmax(nrm, std::fabs(f[6][i]));
    for (size_t i = 0; i < nu; ++i) e = std::fmax(e, std::fabs(tau[i] - f[6][i]));
    return e / nrm;
  };
  const double e_step = err(c.get_torque_command());
  const std::vector<double> x = c.get_solution();
  double e_slice = 0;   // torque_command == solution[nv : nv+nu]
  for (size_t i = 0; i < nu; ++i) e_slice = std::fmax(e_slice, std::fabs(x[nv + i] - c.get_torque_command()[i]));
  const int calls_before = calls;
  r = c.initialize_thread();
  std::this_thread::sleep_for(std::chrono::milliseconds(60));
  const int mid_calls = calls;
  c.update_state(st);                       // shared-state writers from another thread
  c.update_taskspace_targets(f[4]);
  std::this_thread::sleep_for(std::chrono::milliseconds(20));
  const Status stop = c.stop_thread();
  const double e_thread = err(c.get_torque_command());
  const Status clean = c.clean_up();
  std::printf("{\"err_step\": %.3e, \"err_thread\": %.3e, \"slice\": %.1e, \"status\": %d, "
              "\"iters\": %d, \"thread\": %d, \"stop\": %d, \"clean\": %d, \"ticks\": %d, "
              "\"ticks_60ms\": %d, \"n\": %zu}\n",
              e_step, e_thread, e_slice, c.last_solve_status(), c.last_iterations(), r.code(),
              stop.code(), clean.code(), int(calls) - calls_before, mid_calls - calls_before,
              x.size());
  return 0;
}

static int qpos_solve(const std::string& robot, const std::string& path) {
  osc_model_desc d;
  if (osc_desc_from_yaml(robot.c_str(), nullptr, &d) != OSC_OK) return 2;
  const size_t nv = d.nv, nu = d.nu, nc = d.nc, nq = 7 + nu;
  const size_t sizes[5] = {nq, nv, size_t(d.ns) * 6, nc, nu};
  std::vector<std::vector<double>> f(5);
  std::ifstream in(path, std::ios::binary);
  for (int k = 0; k < 5; ++k) {
    f[k].resize(sizes[k]);
    in.read(reinterpret_cast<char*>(f[k].data()), sizes[k] * sizeof(double));
  }
  if (!in) return 3;
  State st = make_state(d.nu, d.nc, 1.0);
  st.body_rotation.assign(f[0].begin() + 3, f[0].begin() + 7);
  st.motor_position.assign(f[0].begin() + 7, f[0].end());
  st.linear_body_velocity.assign(f[1].begin(), f[1].begin() + 3);
  st.angular_body_velocity.assign(f[1].begin() + 3, f[1].begin() + 6);
  st.motor_velocity.assign(f[1].begin() + 6, f[1].end());
  st.contact_mask = f[3];
  OperationalSpaceController c(robot);
  c.set_tick_graph(g_tick_graph);
  Status r = c.initialize(st);
  if (!r.ok()) { std::printf("{\"error\": \"%s\"}\n", r.message().c_str()); return 4; }
  r = c.initialize_optimization();
  if (!r.ok()) { std::printf("{\"error\": \"%s\"}\n", r.message().c_str()); return 5; }
  c.update_taskspace_targets(f[2]);
  r = c.step();
  if (!r.ok()) { std::printf("{\"error\": \"%s\"}\n", r.message().c_str()); return 6; }
  auto err = [&](const std::vector<double>& tau) {
    double e = 0, nrm = 1.0;
    for (size_t i = 0; i < nu; ++i) nrm = std::fmax(nrm, std::fabs(f[4][i]));
    for (size_t i = 0; i < nu; ++i) e = std::fmax(e, std::fabs(tau[i] - f[4][i]));
    return e / nrm;
  };
  const double e_step = err(c.get_torque_command());
  const int status = c.last_solve_status();
  r = c.initialize_thread();
  std::this_thread::sleep_for(std::chrono::milliseconds(60));
  c.update_state(st);
  std::this_thread::sleep_for(std::chrono::milliseconds(20));
  const Status stop = c.stop_thread();
  const double e_thread = err(c.get_torque_command());
  const Status clean = c.clean_up();
  std::printf("{\"err_step\": %.3e, \"err_thread\": %.3e, \"status\": %d, \"thread\": %d, "
              "\"stop\": %d, \"clean\": %d}\n",
              e_step, e_thread, status, r.code(), stop.code(), clean.code());
  return 0;
}

static int gpu_lifecycle(const std::string& robot) {
  osc_model_desc d;
  if (osc_desc_from_yaml(robot.c_str(), nullptr, &d) != OSC_OK) return 2;
  OperationalSpaceController c(robot);
  State bad = make_state(d.nu + 1, d.nc, 1.0);
  const int bad_state = c.initialize(bad).code();
  const int init = c.initialize(make_state(d.nu, d.nc, 1.0)).code();
  OperationalSpaceController nt(robot, "", 2000, "/nonexistent/tree.json");
  const int init_nt = nt.initialize(make_state(d.nu, d.nc, 1.0)).code();
  const int opt_nt = nt.initialize_optimization().code();
  std::printf("{\"bad_state\": %d, \"init\": %d, \"init_nt\": %d, \"opt_nt\": %d}\n",
              bad_state, init, init_nt, opt_nt);
  return 0;
}

int main(int argc, char** argv) {
  // solve / qpos <robot> <fixture> [graph]: "1" replays the tick as a captured hipGraph
  g_tick_graph = argc >= 5 && std::strcmp(argv[4], "1") == 0;
  if (argc >= 4 && std::strcmp(argv[1], "qpos") == 0) return qpos_solve(argv[2], argv[3]);
  if (argc >= 3 && std::strcmp(argv[1], "gpu_lifecycle") == 0) return gpu_lifecycle(argv[2]);
  if (argc >= 3 && std::strcmp(argv[1], "lifecycle") == 0) return lifecycle(argv[2]);
  if (argc >= 4 && std::strcmp(argv[1], "solve") == 0) return solve(argv[2], argv[3]);
  std::fprintf(stderr, "usage: %s lifecycle <robot> | solve <robot> <fixture.bin>\n", argv[0]);
  return 1;
}
