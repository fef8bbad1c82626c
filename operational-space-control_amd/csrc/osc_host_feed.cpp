// osc_host_feed.cpp -- the host-fed batched control tick (include/osc_host_feed.h, SURVEY.md
// §8(e)): pinned host slots -> one H2D copy per tick -> the batched solve -> D2H of the torques,
// pipelined over `depth` slots on three HIP streams.  Host code over the public C-ABI only
// (osc_batch_kinematics, osc_batch_solve(_warm)); the reference it replaces is the
// per-tick hand-off of unitree_go2/operational_space_controller.h:546-573 (State and targets in
// host memory under the mutex, the solve, the torque copy back).
#include "osc_host_feed.h"

#include <hip/hip_runtime.h>

#include <cstring>
#include <new>

namespace {

constexpr size_t kAlign = 256;   // every array of a slot starts on a 256-B boundary
size_t align_up(size_t v) { return (v + kAlign - 1) / kAlign * kAlign; }

enum Ev { kH2dBeg, kH2dEnd, kKinEnd, kSolveBeg, kSolveEnd, kD2hBeg, kD2hEnd, kNumEv };

struct Slot {
  char* h_in = nullptr;        // pinned
  char* d_in = nullptr;        // HBM
  char* h_out = nullptr;       // pinned
  char* d_out = nullptr;       // HBM
  char* d_kin = nullptr;       // HBM: joint-state form, the kinematics' M, C, J, b of this slot
  hipEvent_t ev[kNumEv] = {};
  int32_t tick = -1;           // last tick submitted into this slot
};

}  // namespace

struct osc_host_feed {
  const osc_model* model = nullptr;
  const osc_kin_model* kin = nullptr;
  int32_t nenv = 0, form = 0, depth = 0, device = 0;
  uint32_t flags = 0;
  int32_t nv = 0, nu = 0, nc = 0, ns = 0, nq = 0;
  // byte offsets of the arrays inside a slot's input block: M C J b | qpos qvel, then T mask
  size_t off_M = 0, off_C = 0, off_J = 0, off_b = 0, off_qpos = 0, off_qvel = 0, off_T = 0,
         off_mask = 0, in_bytes = 0;
  size_t off_tau = 0, off_status = 0, off_iters = 0, out_bytes = 0;
  size_t kin_M = 0, kin_C = 0, kin_J = 0, kin_b = 0, kin_bytes = 0;   // joint-state form
  Slot slot[OSC_FEED_MAX_DEPTH];
  hipStream_t s_h2d = nullptr, s_solve = nullptr, s_d2h = nullptr;
  void* ws = nullptr;
  size_t ws_bytes = 0;
  double* warm = nullptr;
  size_t warm_bytes = 0;
  int32_t next = 0;            // next tick to submit
  bool failed = false;         // a submit failed part-way: the pipeline state is undefined
};

namespace {

void release(osc_host_feed* f) {
  for (auto& s : f->slot) {
    for (auto& e : s.ev)
      if (e) (void)hipEventDestroy(e);
    if (s.h_in) (void)hipHostFree(s.h_in);
    if (s.h_out) (void)hipHostFree(s.h_out);
    if (s.d_in) (void)hipFree(s.d_in);
    if (s.d_out) (void)hipFree(s.d_out);
    if (s.d_kin) (void)hipFree(s.d_kin);
  }
  for (hipStream_t st : {f->s_h2d, f->s_solve, f->s_d2h})
    if (st) (void)hipStreamDestroy(st);
  if (f->ws) (void)hipFree(f->ws);
  if (f->warm) (void)hipFree(f->warm);
  delete f;
}

bool ok(hipError_t e) { return e == hipSuccess; }

}  // namespace

extern "C" int osc_host_feed_create(const osc_model* model, const osc_kin_model* kin,
                                    int32_t nenv, int32_t form, uint32_t flags, int32_t depth,
                                    osc_host_feed** out) {
  if (!out) return OSC_ERR_INVALID_ARGUMENT;
  *out = nullptr;
  if (!model || nenv <= 0 || depth < 1 || depth > OSC_FEED_MAX_DEPTH ||
      (flags & ~OSC_FEED_WARM) != 0)
    return OSC_ERR_INVALID_ARGUMENT;
  if (form == OSC_FEED_QP ? kin != nullptr : (form != OSC_FEED_JOINT_STATES || kin == nullptr))
    return OSC_ERR_INVALID_ARGUMENT;
  osc_model_desc d;
  if (osc_model_get_desc(model, &d) != OSC_OK) return OSC_ERR_INVALID_ARGUMENT;
  if (d.wheel_rows) return OSC_ERR_INVALID_ARGUMENT;   // (per-env wheel directions: no form has them)
  osc_host_feed* f = new (std::nothrow) osc_host_feed;
  if (!f) return OSC_ERR_DEVICE;
  f->model = model;
  f->kin = kin;
  f->nenv = nenv;
  f->form = form;
  f->flags = flags;
  f->depth = depth;
  f->nv = d.nv;
  f->nu = d.nu;
  f->nc = d.nc;
  f->ns = d.ns;
  (void)hipGetDevice(&f->device);
  const size_t n = static_cast<size_t>(nenv), e8 = sizeof(double);
  size_t o = 0;
  auto take = [&](size_t bytes) {
    const size_t at = o;
    o = align_up(o + bytes);
    return at;
  };
  if (form == OSC_FEED_QP) {
    f->off_M = take(n * d.nv * d.nv * e8);
    f->off_C = take(n * d.nv * e8);
    f->off_J = take(n * 6 * d.ns * d.nv * e8);
    f->off_b = take(n * 6 * d.ns * e8);
  } else {
    int32_t knv = 0, kns = 0;
    if (osc_kin_model_dims(kin, &f->nq, &knv, &kns) != OSC_OK || knv != d.nv || kns != d.ns) {
      release(f);
      return OSC_ERR_INVALID_ARGUMENT;
    }
    f->off_qpos = take(n * f->nq * e8);
    f->off_qvel = take(n * d.nv * e8);
  }
  f->off_T = take(n * d.ns * 6 * e8);
  f->off_mask = take(n * d.nc * e8);
  f->in_bytes = o;
  o = 0;
  f->off_tau = take(n * d.nu * e8);
  f->off_status = take(n * sizeof(int32_t));
  f->off_iters = take(n * sizeof(int32_t));
  f->out_bytes = o;
  if (form == OSC_FEED_JOINT_STATES) {
    o = 0;
    f->kin_M = take(n * d.nv * d.nv * e8);
    f->kin_C = take(n * d.nv * e8);
    f->kin_J = take(n * 6 * d.ns * d.nv * e8);
    f->kin_b = take(n * 6 * d.ns * e8);
    f->kin_bytes = o;
  }

  int rc = OSC_ERR_DEVICE;
  bool good =
      ok(hipStreamCreateWithFlags(&f->s_h2d, hipStreamNonBlocking)) &&
      ok(hipStreamCreateWithFlags(&f->s_solve, hipStreamNonBlocking)) &&
      ok(hipStreamCreateWithFlags(&f->s_d2h, hipStreamNonBlocking));
  for (int i = 0; good && i < depth; ++i) {
    Slot& s = f->slot[i];
    good = ok(hipHostMalloc(reinterpret_cast<void**>(&s.h_in), f->in_bytes, hipHostMallocDefault)) &&
           ok(hipHostMalloc(reinterpret_cast<void**>(&s.h_out), f->out_bytes, hipHostMallocDefault)) &&
           ok(hipMalloc(reinterpret_cast<void**>(&s.d_in), f->in_bytes)) &&
           ok(hipMalloc(reinterpret_cast<void**>(&s.d_out), f->out_bytes)) &&
           (f->kin_bytes == 0 || ok(hipMalloc(reinterpret_cast<void**>(&s.d_kin), f->kin_bytes)));
    for (int e = 0; good && e < kNumEv; ++e) good = ok(hipEventCreate(&s.ev[e]));
    if (good) {   // zero host inputs: a tick submitted without being written solves a defined QP
      std::memset(s.h_in, 0, f->in_bytes);
      std::memset(s.h_out, 0, f->out_bytes);
    }
  }
  if (good) {
    // (the joint-state form runs the kinematics itself, into the slot's d_kin: the solve's
    // workspace is osc_batch_solve's)
    good = osc_workspace_bytes(model, nenv, &f->ws_bytes) == OSC_OK;
    good = good && ok(hipMalloc(&f->ws, f->ws_bytes));
  }
  if (good && (flags & OSC_FEED_WARM)) {
    good = osc_warm_state_bytes(model, nenv, &f->warm_bytes) == OSC_OK &&
           ok(hipMalloc(reinterpret_cast<void**>(&f->warm), f->warm_bytes)) &&
           ok(hipMemset(f->warm, 0, f->warm_bytes));   // every env cold on its first tick
  }
  if (!good) {
    release(f);
    return rc;
  }
  *out = f;
  return OSC_OK;
}

extern "C" int osc_host_feed_destroy(osc_host_feed* f) {
  if (!f) return OSC_ERR_INVALID_ARGUMENT;
  // drain every stream before freeing what they use
  for (hipStream_t st : {f->s_h2d, f->s_solve, f->s_d2h})
    if (st) (void)hipStreamSynchronize(st);
  release(f);
  return OSC_OK;
}

extern "C" int osc_host_feed_inputs(osc_host_feed* f, int32_t tick, osc_feed_inputs* in) {
  if (!f || !in || tick != f->next) return OSC_ERR_INVALID_ARGUMENT;
  if (f->failed) return OSC_ERR_DEVICE;
  Slot& s = f->slot[tick % f->depth];
  // the slot's pinned inputs are free once its previous H2D copy has completed
  if (s.tick >= 0 && !ok(hipEventSynchronize(s.ev[kH2dEnd]))) return OSC_ERR_DEVICE;
  std::memset(in, 0, sizeof(*in));
  auto at = [&](size_t off) { return reinterpret_cast<double*>(s.h_in + off); };
  if (f->form == OSC_FEED_QP) {
    in->M = at(f->off_M);
    in->C = at(f->off_C);
    in->J = at(f->off_J);
    in->b = at(f->off_b);
  } else {
    in->qpos = at(f->off_qpos);
    in->qvel = at(f->off_qvel);
  }
  in->T = at(f->off_T);
  in->contact_mask = at(f->off_mask);
  in->bytes = f->in_bytes;
  return OSC_OK;
}

namespace {
int submit_tick(osc_host_feed* f, int32_t tick);
}  // namespace

extern "C" int osc_host_feed_submit(osc_host_feed* f, int32_t tick) {
  if (!f || tick != f->next) return OSC_ERR_INVALID_ARGUMENT;
  if (f->failed) return OSC_ERR_DEVICE;
  int cur = -1;
  if (!ok(hipGetDevice(&cur)) || cur != f->device) return OSC_ERR_INVALID_ARGUMENT;
  // anything failing past this point leaves part of the tick enqueued: the feed refuses every
  // further tick (sticky OSC_ERR_DEVICE) and is only good for osc_host_feed_destroy
  const int rc = submit_tick(f, tick);
  if (rc != OSC_OK) f->failed = true;
  return rc;
}

namespace {
int submit_tick(osc_host_feed* f, int32_t tick) {
  Slot& s = f->slot[tick % f->depth];
  const bool reuse = s.tick >= 0;
  // H2D: the device inputs of this slot are free once the solve of tick - depth has read them
  if (reuse && !ok(hipStreamWaitEvent(f->s_h2d, s.ev[kSolveEnd], 0))) return OSC_ERR_DEVICE;
  if (!ok(hipEventRecord(s.ev[kH2dBeg], f->s_h2d)) ||
      !ok(hipMemcpyAsync(s.d_in, s.h_in, f->in_bytes, hipMemcpyHostToDevice, f->s_h2d)) ||
      !ok(hipEventRecord(s.ev[kH2dEnd], f->s_h2d)))
    return OSC_ERR_DEVICE;
  auto in = [&](size_t off) { return reinterpret_cast<const double*>(s.d_in + off); };
  auto kb = [&](size_t off) { return reinterpret_cast<double*>(s.d_kin + off); };
  if (f->form == OSC_FEED_JOINT_STATES) {
    // joint states: the kinematics runs on the copy stream right behind its H2D (round 6), so it
    // overlaps the previous tick's solve -- the interior point's straggler tail leaves most SIMDs
    // idle -- instead of heading this tick's solve (osc_batch_solve_qpos = osc_batch_kinematics +
    // osc_batch_solve: bitwise the same).  The slot's d_kin was last read by the solve of tick -
    // depth, which the copy stream has waited for above.
    const int krc = osc_batch_kinematics(f->kin, f->nenv, in(f->off_qpos), in(f->off_qvel),
                                         kb(f->kin_M), kb(f->kin_C), kb(f->kin_J), kb(f->kin_b),
                                         nullptr, f->s_h2d);
    if (krc != OSC_OK) return krc;
  }
  if (!ok(hipEventRecord(s.ev[kKinEnd], f->s_h2d))) return OSC_ERR_DEVICE;
  // solve: after this tick's H2D (and kinematics), and after the D2H of tick - depth has read the
  // slot's outputs
  if (!ok(hipStreamWaitEvent(f->s_solve, s.ev[kKinEnd], 0)) ||
      (reuse && !ok(hipStreamWaitEvent(f->s_solve, s.ev[kD2hEnd], 0))) ||
      !ok(hipEventRecord(s.ev[kSolveBeg], f->s_solve)))
    return OSC_ERR_DEVICE;
  double* tau = reinterpret_cast<double*>(s.d_out + f->off_tau);
  int32_t* status = reinterpret_cast<int32_t*>(s.d_out + f->off_status);
  int32_t* iters = reinterpret_cast<int32_t*>(s.d_out + f->off_iters);
  int rc;
  if (f->form == OSC_FEED_QP) {
    rc = f->warm ? osc_batch_solve_warm(f->model, f->nenv, in(f->off_M), in(f->off_C),
                                        in(f->off_J), in(f->off_b), in(f->off_T),
                                        in(f->off_mask), tau, nullptr, status, iters, f->warm,
                                        f->warm_bytes, f->ws, f->ws_bytes, f->s_solve)
                 : osc_batch_solve(f->model, f->nenv, in(f->off_M), in(f->off_C), in(f->off_J),
                                   in(f->off_b), in(f->off_T), in(f->off_mask), tau, nullptr,
                                   status, iters, f->ws, f->ws_bytes, f->s_solve);
  } else {
    const double *M = kb(f->kin_M), *C = kb(f->kin_C), *J = kb(f->kin_J), *b = kb(f->kin_b);
    rc = f->warm ? osc_batch_solve_warm(f->model, f->nenv, M, C, J, b, in(f->off_T),
                                        in(f->off_mask), tau, nullptr, status, iters, f->warm,
                                        f->warm_bytes, f->ws, f->ws_bytes, f->s_solve)
                 : osc_batch_solve(f->model, f->nenv, M, C, J, b, in(f->off_T), in(f->off_mask),
                                   tau, nullptr, status, iters, f->ws, f->ws_bytes, f->s_solve);
  }
  if (rc != OSC_OK) return rc;
  if (!ok(hipEventRecord(s.ev[kSolveEnd], f->s_solve))) return OSC_ERR_DEVICE;
  // D2H of the outputs
  if (!ok(hipStreamWaitEvent(f->s_d2h, s.ev[kSolveEnd], 0)) ||
      !ok(hipEventRecord(s.ev[kD2hBeg], f->s_d2h)) ||
      !ok(hipMemcpyAsync(s.h_out, s.d_out, f->out_bytes, hipMemcpyDeviceToHost, f->s_d2h)) ||
      !ok(hipEventRecord(s.ev[kD2hEnd], f->s_d2h)))
    return OSC_ERR_DEVICE;
  s.tick = tick;
  ++f->next;
  return OSC_OK;
}
}  // namespace

extern "C" int osc_host_feed_wait(osc_host_feed* f, int32_t tick, osc_feed_outputs* out) {
  if (!f || !out || tick < 0 || tick >= f->next || tick < f->next - f->depth)
    return OSC_ERR_INVALID_ARGUMENT;
  Slot& s = f->slot[tick % f->depth];
  if (s.tick != tick) return OSC_ERR_INVALID_ARGUMENT;
  if (!ok(hipEventSynchronize(s.ev[kD2hEnd]))) return OSC_ERR_DEVICE;
  out->tau = reinterpret_cast<const double*>(s.h_out + f->off_tau);
  out->status = reinterpret_cast<const int32_t*>(s.h_out + f->off_status);
  out->iters = reinterpret_cast<const int32_t*>(s.h_out + f->off_iters);
  out->bytes = f->out_bytes;
  return OSC_OK;
}

extern "C" int osc_host_feed_timing(osc_host_feed* f, int32_t tick, osc_feed_timing* t) {
  if (!f || !t || tick < 0 || tick >= f->next || tick < f->next - f->depth)
    return OSC_ERR_INVALID_ARGUMENT;
  Slot& s = f->slot[tick % f->depth];
  if (s.tick != tick || hipEventQuery(s.ev[kD2hEnd]) != hipSuccess) return OSC_ERR_INVALID_ARGUMENT;
  if (!ok(hipEventElapsedTime(&t->h2d_ms, s.ev[kH2dBeg], s.ev[kH2dEnd])) ||
      !ok(hipEventElapsedTime(&t->solve_ms, s.ev[kSolveBeg], s.ev[kSolveEnd])) ||
      !ok(hipEventElapsedTime(&t->d2h_ms, s.ev[kD2hBeg], s.ev[kD2hEnd])) ||
      !ok(hipEventElapsedTime(&t->kin_ms, s.ev[kH2dEnd], s.ev[kKinEnd])) ||
      !ok(hipEventElapsedTime(&t->h2d_start_to_d2h_end_ms, s.ev[kH2dBeg], s.ev[kD2hEnd])))
    return OSC_ERR_DEVICE;
  return OSC_OK;
}
