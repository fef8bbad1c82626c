/*
 * osc_controller.h -- drop-in counterpart of the reference's OperationalSpaceController
 * (SURVEY.md §8(f) row 2), backed by the batched C-ABI of osc_batch.h.
 *
 * Same lifecycle, method names, error convention, control thread and mutex semantics as
 * unitree_go2/operational_space_controller.h:106-238, 546-589 (walter_sr/... identical), with
 * three deliberate differences, each forced by what this build can and cannot link:
 *
 *  1. Kinematics.  The reference owns an mjModel/mjData and runs update_mj_data +
 *     update_osc_data (operational_space_controller.h:350-455) each tick.  MuJoCo is not part
 *     of this library, so the controller either
 *       (a) runs the GPU kinematics front end (include/osc_kinematics.h) on the robot's
 *           kinematic tree (<robot>_kinematics.json or any osc_kin_desc-schema JSON): the State
 *           is packed exactly as update_mj_data packs qpos/qvel (:357-361) and the whole tick is
 *           osc_batch_solve_qpos -- the constructor without a KinematicsFn; or
 *       (b) takes a caller's KinematicsFn computing what update_osc_data stores in OSCData
 *           (M = mj_fullM, C = qfrc_bias, J = [Jp; Jr], b = [Jpd; Jrd] qvel), e.g. from the
 *           caller's own mjData.
 *  2. Sizes are runtime values from the YAML config (osc_desc_from_yaml) instead of the
 *     autogen_defines.h constants, so one class serves Go2 and WaLTER.  Vectors are
 *     std::vector<double>, matrices row-major (the reference's Eigen layout, aliases.h:12-13).
 *  3. Status stands in for absl::Status (same codes the reference uses: OK,
 *     FailedPrecondition, Internal, InvalidArgument).
 *
 * Per tick (the reference's control_loop body, :556-574), under the mutex:
 *   (a) pack qpos/qvel -> one host->device copy -> osc_batch_solve_qpos(nenv = 1), or
 *   (b) kinematics(state) -> host->device copy -> osc_batch_solve(nenv = 1),
 * then torque_command = x[nv : nv+nu].  Every tick is warm-started from the previous one (the
 * reference's OsqpSolver::SetWarmStart, :519-526; osc_batch_solve_warm).
 * step() runs one such tick synchronously (for callers without the thread, and tests).
 */
#ifndef OSC_CONTROLLER_H_
#define OSC_CONTROLLER_H_

#include <atomic>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "osc_batch.h"
#include "osc_kinematics.h"

namespace osc_amd {

/* absl::Status stand-in (the codes operational_space_controller.h returns). */
class Status {
 public:
  enum Code { kOk = 0, kInvalidArgument = 3, kFailedPrecondition = 9, kInternal = 13 };
  Status() = default;
  Status(Code code, std::string message) : code_(code), message_(std::move(message)) {}
  static Status Ok() { return Status(); }
  bool ok() const { return code_ == kOk; }
  Code code() const { return code_; }
  const std::string& message() const { return message_; }

 private:
  Code code_ = kOk;
  std::string message_;
};
inline Status FailedPreconditionError(std::string m) { return Status(Status::kFailedPrecondition, std::move(m)); }
inline Status InternalError(std::string m) { return Status(Status::kInternal, std::move(m)); }
inline Status InvalidArgumentError(std::string m) { return Status(Status::kInvalidArgument, std::move(m)); }

/* containers.h:32-42 (fields sized nu, nu, nu, nu, 4, 3, 3, 3, nc). */
struct State {
  std::vector<double> motor_position;
  std::vector<double> motor_velocity;
  std::vector<double> motor_acceleration;
  std::vector<double> torque_estimate;
  std::vector<double> body_rotation;            // (w, x, y, z)
  std::vector<double> linear_body_velocity;
  std::vector<double> angular_body_velocity;
  std::vector<double> linear_body_acceleration;
  std::vector<double> contact_mask;             // nc
};

/* containers.h:13-21 -- the fields the QP reads (contact_jacobian is sliced from J). */
struct OSCData {
  std::vector<double> mass_matrix;          // nv x nv, row-major (mj_fullM)
  std::vector<double> coriolis_matrix;      // nv (qfrc_bias)
  std::vector<double> taskspace_jacobian;   // 6ns x nv, row-major: [Jp_0..Jp_ns-1; Jr_0..]
  std::vector<double> taskspace_bias;       // 6ns: [Jpd; Jrd] qvel
};

/* update_mj_data + update_osc_data (operational_space_controller.h:350-455). */
using KinematicsFn = std::function<Status(const State&, OSCData*)>;

class OperationalSpaceController {
 public:
  /* robot: "unitree_go2" | "walter_sr" | "walter_sr_wheels"; yaml_path as osc_desc_from_yaml
   * (empty = the robot's default config); control_rate_us as the reference (default 2000). */
  OperationalSpaceController(std::string robot, std::string yaml_path, KinematicsFn kinematics,
                             int control_rate_us = 2000);
  /* GPU kinematics front end: kin_json_path = the kinematic tree -- an MJCF file (*.xml, read by
   * osc_kin_desc_from_mjcf_robot with the robot's config lists, as the reference loads its
   * xml_path, operational_space_controller.h:114-152) or a tree JSON (empty = the robot's
   * default <robot>_kinematics.json next to the library's config directory).  The file is read
   * by initialize(); a load failure is InternalError("Failed to load Mujoco Model") (:117). */
  explicit OperationalSpaceController(std::string robot, std::string yaml_path = "",
                                      int control_rate_us = 2000, std::string kin_json_path = "");
  ~OperationalSpaceController();
  OperationalSpaceController(const OperationalSpaceController&) = delete;
  OperationalSpaceController& operator=(const OperationalSpaceController&) = delete;

  Status initialize(State initial_state);          // :112-160 (reads the YAML, not an XML)
  Status initialize_optimization();                // :162-176 (device model + buffers)
  Status initialize_thread();                      // :178-186
  Status stop_thread();                            // :188-195
  Status clean_up();                               // :210-218
  bool is_initialized() const { return initialized_; }                          // :198
  bool is_optimization_initialized() const { return optimization_initialized_; } // :202
  bool is_thread_initialized() const { return thread_initialized_; }           // :206

  void update_state(const State& new_state);                        // :220-223
  /* ns x 6, row-major (TaskspaceTargets). */
  void update_taskspace_targets(const std::vector<double>& targets);  // :225-228
  std::vector<double> get_torque_command();                         // :230-233 (nu)
  std::vector<double> get_solution();                               // :235-238 (nv+nu+3nc)

  /* One control tick, synchronously, under the mutex (the body of control_loop). */
  Status step();
  /* Solve status / interior-point iterations of the last tick (osc_solve_status). */
  int last_solve_status();
  int last_iterations();
  const osc_model_desc& desc() const { return desc_; }
  /* Replay the tick as one captured hipGraph instead of direct launches (default off: measured
   * slower on ROCm 7, Go2 tick median 98 vs 92 us; profiles/r02_tick_graph_ab.txt).  Call before
   * initialize_thread. */
  void set_tick_graph(bool on) { use_graph_ = on; }
  /* The warm start's floors for the controller's one-env ticks (osc_model_tuning warm_delta /
   * warm_center; default 0.3 / 0.3).  Call before initialize_optimization. */
  void set_warm_start_floors(double delta, double center) {
    single_env_warm_delta_ = delta;
    single_env_warm_center_ = center;
  }

 private:
  Status tick_locked();
  void control_loop();
  void release_device();

  Status tick_gpu_kinematics_locked();
  Status fetch_outputs_locked();
  // H2D, the tick's kernels and D2H on the private stream: captured once into a hipGraph and
  // replayed every tick (kind 0 = host kinematics inputs, 1 = joint-state inputs)
  Status launch_tick_locked(int kind, size_t in_bytes);
  Status enqueue_tick_locked(int kind, size_t in_bytes);
  void drop_graph();

  std::string robot_, yaml_path_, kin_json_path_;
  KinematicsFn kinematics_;
  bool gpu_kinematics_ = false;
  osc_kin_model* kin_ = nullptr;
  osc_kin_desc kin_desc_{};          // read by initialize(), uploaded by initialize_optimization()
  int nq_ = 0;
  int control_rate_us_;
  osc_model_desc desc_{};
  int nv_ = 0, nu_ = 0, nc_ = 0, ns_ = 0, n_ = 0;

  std::mutex mutex_;
  State state_;
  std::vector<double> targets_, torque_, solution_;
  int status_ = 0, iters_ = 0;
  OSCData osc_data_;

  bool initialized_ = false, optimization_initialized_ = false, thread_initialized_ = false;
  std::atomic<bool> running_{false};
  std::thread thread_;

  osc_model* model_ = nullptr;
  void* stream_ = nullptr;
  double* d_in_ = nullptr;          // M | C | J | b | T | mask, or qpos | qvel | T | mask
                                    // (one allocation, blocks 16-B aligned)
  double* d_out_ = nullptr;         // tau | x | status, iters (one block, one D2H per tick)
  int32_t* d_info_ = nullptr;       // status | iters: the last slot of d_out_
  void* d_ws_ = nullptr;
  size_t ws_bytes_ = 0;
  double* d_warm_ = nullptr;        // interior-point warm state carried between ticks
  size_t warm_bytes_ = 0;
  double* h_in_ = nullptr;          // pinned staging of d_in_
  double* h_out_ = nullptr;         // pinned tau | x | status, iters (int32 pair, one slot)
  size_t out_doubles_ = 0;          // tau | x doubles copied back
  void* graph_exec_ = nullptr;      // hipGraphExec_t of the captured tick
  int graph_kind_ = -1;
  size_t graph_in_bytes_ = 0;
  bool use_graph_ = false;          // set_tick_graph: replay the tick as a hipGraph
  double single_env_warm_delta_ = 0.3;    // set_warm_start_floors
  double single_env_warm_center_ = 0.3;
};

}  // namespace osc_amd

#endif  // OSC_CONTROLLER_H_
