// osc_controller.cpp -- OperationalSpaceController over the batched C-ABI (include/osc_controller.h).
//
// Mirrors unitree_go2/operational_space_controller.h (paths relative to the reference's
// operational-space-control/ directory): lifecycle and preconditions :112-218, shared-state
// accessors under one mutex :220-238, control_loop :546-589.  The QP tick itself is
// osc_batch_solve with nenv = 1 on a private HIP stream.
#include "osc_controller.h"

#include <hip/hip_runtime_api.h>

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <utility>

namespace osc_amd {
namespace {

Status from_osc(int rc, const char* what) {
  if (rc == OSC_OK) return Status::Ok();
  std::string m = std::string(what) + ": " + osc_status_string(rc);
  if (rc == OSC_ERR_INVALID_ARGUMENT || rc == OSC_ERR_UNSUPPORTED_DIMS)
    return InvalidArgumentError(m);
  return InternalError(m);   // IO, DEVICE, NO_DEVICE (osc.h:117 uses InternalError for loads)
}

constexpr size_t even(size_t n) { return (n + 1) & ~size_t(1); }

}  // namespace

OperationalSpaceController::OperationalSpaceController(std::string robot, std::string yaml_path,
                                                       KinematicsFn kinematics,
                                                       int control_rate_us)
    : robot_(std::move(robot)),
      yaml_path_(std::move(yaml_path)),
      kinematics_(std::move(kinematics)),
      control_rate_us_(control_rate_us) {}

OperationalSpaceController::OperationalSpaceController(std::string robot, std::string yaml_path,
                                                       int control_rate_us,
                                                       std::string kin_json_path)
    : robot_(std::move(robot)),
      yaml_path_(std::move(yaml_path)),
      kin_json_path_(std::move(kin_json_path)),
      control_rate_us_(control_rate_us) {
  gpu_kinematics_ = true;
}

OperationalSpaceController::~OperationalSpaceController() {
  if (thread_initialized_ && thread_.joinable()) {
    running_ = false;
    thread_.join();
  }
  release_device();
}

Status OperationalSpaceController::initialize(State initial_state) {
  // The reference loads the MuJoCo XML and resolves site/body ids here (:112-160); the QP's
  // static data comes from the YAML the reference's autogen.py reads at build time.
  const int rc = osc_desc_from_yaml(robot_.c_str(), yaml_path_.empty() ? nullptr : yaml_path_.c_str(),
                                    &desc_);
  if (rc != OSC_OK) return InternalError(std::string("Failed to load OSC config: ") + osc_status_string(rc));
  nv_ = desc_.nv;
  nu_ = desc_.nu;
  nc_ = desc_.nc;
  ns_ = desc_.ns;
  n_ = nv_ + nu_ + 3 * nc_;
  if (initial_state.contact_mask.size() != static_cast<size_t>(nc_))
    return InvalidArgumentError("State.contact_mask must have one entry per contact site");
  if (!kinematics_ && !gpu_kinematics_) return InvalidArgumentError("no kinematics provider");
  if (gpu_kinematics_) {
    // the reference loads the robot's MJCF here and resolves its sites / bodies (:114-152)
    const std::string& p = kin_json_path_;
    const bool mjcf = p.size() >= 4 && p.compare(p.size() - 4, 4, ".xml") == 0;
    // the wheel-weight config drives the same robot as walter_sr
    const std::string tree = robot_ == "walter_sr_wheels" ? "walter_sr" : robot_;
    const int krc = mjcf ? osc_kin_desc_from_mjcf_robot(robot_.c_str(),
                                                        yaml_path_.empty() ? nullptr : yaml_path_.c_str(),
                                                        p.c_str(), &kin_desc_)
                         : osc_kin_desc_from_json(tree.c_str(), p.empty() ? nullptr : p.c_str(),
                                                  &kin_desc_);
    if (krc != OSC_OK) return InternalError("Failed to load Mujoco Model");
  }
  if (gpu_kinematics_ &&
      (initial_state.motor_position.size() != static_cast<size_t>(nu_) ||
       initial_state.motor_velocity.size() != static_cast<size_t>(nu_) ||
       initial_state.body_rotation.size() != 4 || initial_state.linear_body_velocity.size() != 3 ||
       initial_state.angular_body_velocity.size() != 3))
    return InvalidArgumentError("State sizes do not match the robot (nu motors, 4 + 3 + 3 base)");
  std::lock_guard<std::mutex> lock(mutex_);
  state_ = std::move(initial_state);
  targets_.assign(static_cast<size_t>(ns_) * 6, 0.0);   // TaskspaceTargets::Zero()  (:243)
  torque_.assign(nu_, 0.0);                               // torque_command Zero      (:244)
  solution_.assign(n_, 0.0);
  initialized_ = true;
  return Status::Ok();
}

Status OperationalSpaceController::initialize_optimization() {
  if (!initialized_) return FailedPreconditionError("Operational Space Controller not initialized.");
  if (optimization_initialized_) return Status::Ok();
  // One env per tick: tighter warm-start floors than the batch defaults (1, 1), which cut the
  // slowest warm envs' tail of a 4,096-env wave set -- a tail a lone env does not have -- at +0.8
  // mean iterations.  Measured over 2,000 Go2 ticks (profiles/r04g_tick_*.json, median / p99 us):
  // (1, 1) 93.1 / 117.6, (0.1, 0.3) 85.0 / 133.1, (0.3, 0.3) 90.6 / 122.0
  osc_model_tuning tune;
  Status st = from_osc(osc_model_tuning_defaults(&desc_, &tune), "osc_model_tuning_defaults");
  if (!st.ok()) return st;
  tune.warm_delta = single_env_warm_delta_;
  tune.warm_center = single_env_warm_center_;
  st = from_osc(osc_model_create_tuned(&desc_, &tune, &model_), "osc_model_create_tuned");
  if (!st.ok()) return st;
  const size_t s = 6 * static_cast<size_t>(ns_);
  size_t in_doubles = even(nv_ * nv_) + even(nv_) + even(s * nv_) + even(s) +
                      even(ns_ * 6) + even(nc_);
  if (gpu_kinematics_) {
    st = from_osc(osc_kin_model_create(&kin_desc_, &kin_), "osc_kin_model_create");
    if (!st.ok()) {
      release_device();
      return st;
    }
    int32_t nq = 0, nv = 0, nsite = 0;
    osc_kin_model_dims(kin_, &nq, &nv, &nsite);
    if (nv != nv_ || nsite != ns_ || nq != 7 + nu_) {   // floating base + one dof per motor
      release_device();
      return InvalidArgumentError("kinematic tree does not match the OSC model");
    }
    nq_ = nq;
    in_doubles = even(nq_) + even(nv_) + even(ns_ * 6) + even(nc_);
    if (osc_qpos_workspace_bytes(model_, kin_, 1, &ws_bytes_) != OSC_OK) {
      release_device();
      return InternalError("workspace size");
    }
  } else if (osc_workspace_bytes(model_, 1, &ws_bytes_) != OSC_OK) {
    return InternalError("workspace size");
  }
  hipStream_t stream = nullptr;
  if (hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess ||
      hipMalloc(reinterpret_cast<void**>(&d_in_), in_doubles * sizeof(double)) != hipSuccess ||
      hipMalloc(reinterpret_cast<void**>(&d_out_), (even(nu_) + even(n_) + 1) * sizeof(double)) != hipSuccess ||
      hipMalloc(&d_ws_, ws_bytes_) != hipSuccess ||
      osc_warm_state_bytes(model_, 1, &warm_bytes_) != OSC_OK ||
      hipMalloc(reinterpret_cast<void**>(&d_warm_), warm_bytes_) != hipSuccess ||
      hipMemset(d_warm_, 0, warm_bytes_) != hipSuccess) {
    stream_ = stream;
    release_device();
    return InternalError("device allocation failed");
  }
  stream_ = stream;
  // tau | x | (status, iters) in one device block, so the tick's results come back in one copy
  out_doubles_ = even(nu_) + even(n_);
  d_info_ = reinterpret_cast<int32_t*>(d_out_ + out_doubles_);
  if (hipHostMalloc(reinterpret_cast<void**>(&h_in_), in_doubles * sizeof(double),
                    hipHostMallocDefault) != hipSuccess ||
      hipHostMalloc(reinterpret_cast<void**>(&h_out_), (out_doubles_ + 1) * sizeof(double),
                    hipHostMallocDefault) != hipSuccess) {
    release_device();
    return InternalError("pinned host allocation failed");
  }
  std::memset(h_in_, 0, in_doubles * sizeof(double));
  optimization_initialized_ = true;
  return Status::Ok();
}

Status OperationalSpaceController::initialize_thread() {
  if (!initialized_ || !optimization_initialized_)
    return FailedPreconditionError(
        "Initialization precoditions not met. Initialize controller and optimization before "
        "starting control thread.");
  running_ = true;
  thread_ = std::thread(&OperationalSpaceController::control_loop, this);
  thread_initialized_ = true;
  return Status::Ok();
}

Status OperationalSpaceController::stop_thread() {
  if (!thread_initialized_) return FailedPreconditionError("Operation Space Control Thread not initialized");
  running_ = false;
  if (thread_.joinable()) thread_.join();
  return Status::Ok();
}

Status OperationalSpaceController::clean_up() {
  if (!initialized_)
    return FailedPreconditionError("Operational Space Controller not initialized. Nothing to clean up");
  if (thread_initialized_ && thread_.joinable()) {
    running_ = false;
    thread_.join();
  }
  release_device();
  optimization_initialized_ = false;
  return Status::Ok();
}

void OperationalSpaceController::update_state(const State& new_state) {
  std::lock_guard<std::mutex> lock(mutex_);
  state_ = new_state;
}

void OperationalSpaceController::update_taskspace_targets(const std::vector<double>& targets) {
  std::lock_guard<std::mutex> lock(mutex_);
  targets_ = targets;
}

std::vector<double> OperationalSpaceController::get_torque_command() {
  std::lock_guard<std::mutex> lock(mutex_);
  return torque_;
}

std::vector<double> OperationalSpaceController::get_solution() {
  std::lock_guard<std::mutex> lock(mutex_);
  return solution_;
}

int OperationalSpaceController::last_solve_status() {
  std::lock_guard<std::mutex> lock(mutex_);
  return status_;
}

int OperationalSpaceController::last_iterations() {
  std::lock_guard<std::mutex> lock(mutex_);
  return iters_;
}

Status OperationalSpaceController::step() {
  if (!optimization_initialized_) return FailedPreconditionError("Optimization not initialized.");
  std::lock_guard<std::mutex> lock(mutex_);
  return tick_locked();
}

// (a) GPU kinematics: update_mj_data's packing (:357-361) on the host, then one copy and the
// whole tick on the device (osc_batch_solve_qpos).  Caller holds the mutex.
Status OperationalSpaceController::tick_gpu_kinematics_locked() {
  if (targets_.size() != static_cast<size_t>(ns_) * 6 ||
      state_.contact_mask.size() != static_cast<size_t>(nc_) ||
      state_.motor_position.size() != static_cast<size_t>(nu_) ||
      state_.motor_velocity.size() != static_cast<size_t>(nu_) || state_.body_rotation.size() != 4 ||
      state_.linear_body_velocity.size() != 3 || state_.angular_body_velocity.size() != 3)
    return InvalidArgumentError("State / targets size mismatch");
  double* h = h_in_;
  double* qpos = h;
  double* qvel = h + even(nq_);
  double* T = qvel + even(nv_);
  double* mask = T + even(ns_ * 6);
  qpos[0] = qpos[1] = qpos[2] = 0.0;                     // base position forced to 0 (:358-359)
  std::memcpy(qpos + 3, state_.body_rotation.data(), 4 * sizeof(double));
  std::memcpy(qpos + 7, state_.motor_position.data(), nu_ * sizeof(double));
  std::memcpy(qvel, state_.linear_body_velocity.data(), 3 * sizeof(double));
  std::memcpy(qvel + 3, state_.angular_body_velocity.data(), 3 * sizeof(double));
  std::memcpy(qvel + 6, state_.motor_velocity.data(), nu_ * sizeof(double));
  std::memcpy(T, targets_.data(), targets_.size() * sizeof(double));
  std::memcpy(mask, state_.contact_mask.data(), nc_ * sizeof(double));
  const size_t off = static_cast<size_t>(mask - h) + even(nc_);
  return launch_tick_locked(1, off * sizeof(double));
}

// One tick's stream work: H2D of the staged inputs, the batched entry point with nenv = 1
// (warm-started from the previous tick, as the reference's SetWarmStart :519-526), D2H of
// tau | x | status | iters into pinned memory.  Every pointer is fixed at initialization, so
// the sequence is the same every tick.
Status OperationalSpaceController::enqueue_tick_locked(int kind, size_t in_bytes) {
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  if (hipMemcpyAsync(d_in_, h_in_, in_bytes, hipMemcpyHostToDevice, stream) != hipSuccess)
    return InternalError("host to device copy failed");
  Status st;
  if (kind == 1) {
    const size_t q = even(nq_), v = q + even(nv_), t = v + even(ns_ * 6);
    st = from_osc(osc_batch_solve_qpos_warm(model_, kin_, 1, d_in_, d_in_ + q, d_in_ + v,
                                            d_in_ + t, d_out_, d_out_ + even(nu_), d_info_,
                                            d_info_ + 1, d_warm_, warm_bytes_, d_ws_, ws_bytes_,
                                            stream_),
                  "osc_batch_solve_qpos_warm");
  } else {
    const size_t nv = nv_, s = 6 * static_cast<size_t>(ns_);
    const size_t sizes[6] = {nv * nv, nv, s * nv, s, static_cast<size_t>(ns_) * 6,
                             static_cast<size_t>(nc_)};
    double* dptr[6];
    size_t off = 0;
    for (int k = 0; k < 6; ++k) {
      dptr[k] = d_in_ + off;
      off += even(sizes[k]);
    }
    st = from_osc(osc_batch_solve_warm(model_, 1, dptr[0], dptr[1], dptr[2], dptr[3], dptr[4],
                                       dptr[5], d_out_, d_out_ + even(nu_), d_info_, d_info_ + 1,
                                       d_warm_, warm_bytes_, d_ws_, ws_bytes_, stream_),
                  "osc_batch_solve_warm");
  }
  if (!st.ok()) return st;
  if (hipMemcpyAsync(h_out_, d_out_, (out_doubles_ + 1) * sizeof(double), hipMemcpyDeviceToHost,
                     stream) != hipSuccess)
    return InternalError("device to host copy failed");
  return Status::Ok();
}

// The tick as one hipGraph (set_tick_graph(true)): captured on the first tick of a kind and replayed
// afterwards (one submission instead of two copies, three or four kernel launches and two
// copies).  A capture the runtime refuses falls back to launching the same work directly.  Off by
// default: on MI355X / ROCm 7 the replay is slower than the direct launches from pinned staging
// (Go2 tick median 98 vs 92 us, WaLTER 109 vs 103 us; profiles/r02_tick_graph_ab.txt).
Status OperationalSpaceController::launch_tick_locked(int kind, size_t in_bytes) {
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  if (graph_exec_ && graph_kind_ == kind && graph_in_bytes_ == in_bytes) {
    if (hipGraphLaunch(static_cast<hipGraphExec_t>(graph_exec_), stream) != hipSuccess)
      return InternalError("tick graph launch failed");
    return Status::Ok();
  }
  drop_graph();
  if (use_graph_ && hipStreamBeginCapture(stream, hipStreamCaptureModeRelaxed) == hipSuccess) {
    Status st = enqueue_tick_locked(kind, in_bytes);
    hipGraph_t g = nullptr;
    const hipError_t ec = hipStreamEndCapture(stream, &g);
    hipGraphExec_t exec = nullptr;
    if (st.ok() && ec == hipSuccess && g &&
        hipGraphInstantiate(&exec, g, nullptr, nullptr, 0) == hipSuccess) {
      (void)hipGraphDestroy(g);
      graph_exec_ = exec;
      graph_kind_ = kind;
      graph_in_bytes_ = in_bytes;
      if (hipGraphLaunch(exec, stream) != hipSuccess)
        return InternalError("tick graph launch failed");
      return Status::Ok();
    }
    if (g) (void)hipGraphDestroy(g);
    (void)hipGetLastError();
    if (!st.ok()) return st;   // argument errors are reported as the direct path reports them
    use_graph_ = false;        // capture unsupported here: direct launches from now on
  }
  return enqueue_tick_locked(kind, in_bytes);
}

void OperationalSpaceController::drop_graph() {
  if (graph_exec_) (void)hipGraphExecDestroy(static_cast<hipGraphExec_t>(graph_exec_));
  graph_exec_ = nullptr;
  graph_kind_ = -1;
  graph_in_bytes_ = 0;
}

// The body of the reference's control_loop (:556-574), caller holds the mutex.
Status OperationalSpaceController::tick_locked() {
  Status st;
  if (gpu_kinematics_) {
    st = tick_gpu_kinematics_locked();
    if (!st.ok()) return st;
    return fetch_outputs_locked();
  }
  st = kinematics_(state_, &osc_data_);                  // update_mj_data + update_osc_data
  if (!st.ok()) return st;
  const size_t nv = nv_, s = 6 * static_cast<size_t>(ns_);
  if (osc_data_.mass_matrix.size() != nv * nv || osc_data_.coriolis_matrix.size() != nv ||
      osc_data_.taskspace_jacobian.size() != s * nv || osc_data_.taskspace_bias.size() != s ||
      targets_.size() != static_cast<size_t>(ns_) * 6 ||
      state_.contact_mask.size() != static_cast<size_t>(nc_))
    return InvalidArgumentError("OSCData / targets / contact_mask size mismatch");
  // pack M | C | J | b | T | mask (row-major per block, each block padded to 16 B)
  double* h = h_in_;
  const double* blocks[6] = {osc_data_.mass_matrix.data(), osc_data_.coriolis_matrix.data(),
                             osc_data_.taskspace_jacobian.data(), osc_data_.taskspace_bias.data(),
                             targets_.data(), state_.contact_mask.data()};
  const size_t sizes[6] = {nv * nv, nv, s * nv, s, static_cast<size_t>(ns_) * 6,
                           static_cast<size_t>(nc_)};
  size_t off = 0;
  for (int k = 0; k < 6; ++k) {
    std::memcpy(h + off, blocks[k], sizes[k] * sizeof(double));
    off += even(sizes[k]);
  }
  st = launch_tick_locked(0, off * sizeof(double));
  if (!st.ok()) return st;
  return fetch_outputs_locked();
}

// Copy tau | x | status | iters back and publish them (torque_command = x[nv : nv+nu], :573).
Status OperationalSpaceController::fetch_outputs_locked() {
  // (the tick's D2H copies into h_out_ were enqueued with it)
  if (hipStreamSynchronize(static_cast<hipStream_t>(stream_)) != hipSuccess)
    return InternalError("device to host copy failed");
  int32_t info[2];
  std::memcpy(info, h_out_ + out_doubles_, sizeof(info));
  torque_.assign(h_out_, h_out_ + nu_);                      // = solution[nv : nv+nu] (:573)
  solution_.assign(h_out_ + even(nu_), h_out_ + even(nu_) + n_);
  // The reference publishes OSQP's solution whatever its exit code (solve_optimization, :531-536,
  // never reads exit_code); so does this tick -- but a solve that is not OK is reported on stderr
  // when the status changes, and stays readable through last_solve_status().
  if (info[0] != OSC_SOLVE_OK && info[0] != status_)
    std::cerr << "OperationalSpaceController: solve status " << info[0]
              << (info[0] == OSC_SOLVE_MAX_ITER     ? " (max_iter)"
                  : info[0] == OSC_SOLVE_NUMERICAL  ? " (non-finite input or M not SPD)"
                  : info[0] == OSC_SOLVE_UNREFINED  ? " (unrefined)"
                                                    : "")
              << " after " << info[1] << " iterations; torques published as returned\n";
  status_ = info[0];
  iters_ = info[1];
  return Status::Ok();
}

// control_loop (:546-589): fixed-rate ticks, overrun logged and the schedule reset.
void OperationalSpaceController::control_loop() {
  using Clock = std::chrono::steady_clock;
  auto next_time = Clock::now();
  while (running_) {
    next_time += std::chrono::microseconds(control_rate_us_);
    {
      std::lock_guard<std::mutex> lock(mutex_);
      (void)tick_locked();   // the reference ignores per-tick errors (:567)
    }
    const auto now = Clock::now();
    if (now < next_time) {
      std::this_thread::sleep_until(next_time);
    } else {
      const auto overrun = std::chrono::duration_cast<std::chrono::microseconds>(now - next_time);
      std::cout << "Operational Space Control Loop Execution Time Exceeded Control Rate: "
                << overrun.count() << "us" << std::endl;
      next_time = now;
    }
  }
}

void OperationalSpaceController::release_device() {
  if (stream_) (void)hipStreamSynchronize(static_cast<hipStream_t>(stream_));
  drop_graph();
  if (h_in_) (void)hipHostFree(h_in_);
  if (h_out_) (void)hipHostFree(h_out_);
  h_in_ = h_out_ = nullptr;
  if (d_in_) (void)hipFree(d_in_);
  if (d_out_) (void)hipFree(d_out_);
  if (d_ws_) (void)hipFree(d_ws_);
  if (d_warm_) (void)hipFree(d_warm_);
  d_warm_ = nullptr;
  if (stream_) (void)hipStreamDestroy(static_cast<hipStream_t>(stream_));
  if (model_) (void)osc_model_destroy(model_);
  if (kin_) (void)osc_kin_model_destroy(kin_);
  kin_ = nullptr;
  d_in_ = d_out_ = nullptr;
  d_info_ = nullptr;
  d_ws_ = nullptr;
  stream_ = nullptr;
  model_ = nullptr;
}

}  // namespace osc_amd
