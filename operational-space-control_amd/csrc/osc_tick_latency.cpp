// osc_tick_latency -- single-environment control-tick latency through the controller
// (include/osc_controller.h), BASELINE configs[0]: one robot, nenv = 1, the reference's per-tick
// path (unitree_go2/operational_space_controller.h:546-589 control_loop body: update_mj_data,
// update_osc_data, update_optimization, solve, torque) against its 2,000 us control period
// (:108).
//
//   osc_tick_latency <robot> <xml|json|""> <ticks> [warmup]
//
// Each tick is OperationalSpaceController::step(): State -> qpos/qvel packing on the host, one
// host->device copy, GPU kinematics + reduced QP + interior point (warm-started from the previous
// tick, as the reference's SetWarmStart), one device->host copy of tau / x / status.  The joint
// state walks by +-0.01 rad per tick so consecutive ticks differ like a control loop's.  Prints
// one JSON line: median / p90 / p99 / max / mean tick wall time in microseconds, the share of
// ticks within the 2,000 us period, and the mean interior-point iterations.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

#include "osc_controller.h"

int main(int argc, char** argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: osc_tick_latency <robot> <tree path or \"\"> <ticks> [warmup]"
                         " [warm_delta warm_center]\n");
    return 2;
  }
  const std::string robot = argv[1];
  const int ticks = std::atoi(argv[3]);
  const int warmup = argc > 4 ? std::atoi(argv[4]) : 50;
  osc_model_desc d;
  if (osc_desc_from_yaml(robot.c_str(), nullptr, &d) != OSC_OK) return 3;

  osc_amd::OperationalSpaceController c(robot, "", 2000, argv[2]);
  // optional 5th / 6th arguments: the warm start's floors (A/B of set_warm_start_floors)
  if (argc > 6) c.set_warm_start_floors(std::atof(argv[5]), std::atof(argv[6]));
  osc_amd::State s;
  s.motor_position.assign(d.nu, 0.0);
  s.motor_velocity.assign(d.nu, 0.0);
  s.motor_acceleration.assign(d.nu, 0.0);
  s.torque_estimate.assign(d.nu, 0.0);
  s.body_rotation = {1.0, 0.0, 0.0, 0.0};
  s.linear_body_velocity.assign(3, 0.0);
  s.angular_body_velocity.assign(3, 0.0);
  s.linear_body_acceleration.assign(3, 0.0);
  s.contact_mask.assign(d.nc, 1.0);
  std::mt19937_64 rng(20251015);
  std::normal_distribution<double> n01(0.0, 1.0);
  for (int i = 0; i < d.nu; ++i) s.motor_position[i] = 0.3 * n01(rng);
  osc_amd::Status st = c.initialize(s);
  if (st.ok()) st = c.initialize_optimization();
  if (!st.ok()) {
    std::fprintf(stderr, "osc_tick_latency: %s\n", st.message().c_str());
    return 4;
  }
  std::vector<double> targets(static_cast<size_t>(d.ns) * 6, 0.0);
  for (int i = 0; i < 6; ++i) targets[i] = 10.0 * n01(rng);   // a base PD command (standing.cc)
  c.update_taskspace_targets(targets);

  std::vector<double> us;
  us.reserve(ticks);
  long long iters = 0;
  int bad = 0;
  for (int k = 0; k < warmup + ticks; ++k) {
    for (int i = 0; i < d.nu; ++i) {
      s.motor_position[i] += 0.01 * n01(rng);
      s.motor_velocity[i] = 0.5 * n01(rng);
    }
    c.update_state(s);
    const auto t0 = std::chrono::steady_clock::now();
    st = c.step();
    const auto t1 = std::chrono::steady_clock::now();
    if (!st.ok()) {
      std::fprintf(stderr, "osc_tick_latency: tick %d: %s\n", k, st.message().c_str());
      return 5;
    }
    if (k < warmup) continue;
    us.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
    iters += c.last_iterations();
    bad += c.last_solve_status() != OSC_SOLVE_OK;
  }
  std::vector<double> srt = us;
  std::sort(srt.begin(), srt.end());
  auto pct = [&](double p) {
    return srt[std::min(srt.size() - 1, static_cast<size_t>(p * (srt.size() - 1) + 0.5))];
  };
  double mean = 0.0;
  int within = 0;
  for (double v : us) {
    mean += v;
    within += v <= 2000.0;
  }
  mean /= us.size();
  std::printf("{\"robot\": \"%s\", \"ticks\": %zu, \"median_us\": %.2f, \"p90_us\": %.2f, "
              "\"p99_us\": %.2f, \"max_us\": %.2f, \"mean_us\": %.2f, "
              "\"within_2000us_frac\": %.6f, \"mean_ipm_iters\": %.3f, \"unconverged\": %d}\n",
              robot.c_str(), us.size(), pct(0.5), pct(0.9), pct(0.99), srt.back(), mean,
              static_cast<double>(within) / us.size(), static_cast<double>(iters) / us.size(), bad);
  return 0;
}
