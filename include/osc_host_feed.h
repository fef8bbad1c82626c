/*
 * osc_host_feed.h -- the host-fed batched control tick: a batch's inputs start
 * in HOST memory every tick, as the reference's do (its control loop reads the State and the task
 * targets the simulation thread wrote, unitree_go2/operational_space_controller.h:546-573, under
 * the mutex of :220-238), cross PCIe to the GPU, are solved there, and the torques come back.
 * Part of libosc_batch.so; same return codes as osc_batch.h.
 *
 * The feed owns, per pipeline slot (`depth` slots, 2 = double buffering):
 *   pinned host input block   -- the caller (a simulator, one rank's host thread) writes tick k's
 *                                inputs here through the pointers osc_host_feed_inputs returns;
 *   device input block        -- the same layout in HBM, one hipMemcpyAsync per tick;
 *   device + pinned outputs   -- tau, status, iters.
 * and three HIP streams: H2D copies, solves, D2H copies.  Tick k's H2D overlaps tick k-1's solve
 * and tick k-2's D2H; the solves run in tick order on one stream, so a warm-started feed carries
 * its warm state (osc_batch_solve_warm: the reference's SetWarmStart, osc.h:519-526) from each
 * tick to the next.  Nothing crosses xGMI: one feed per GPU, each rank its own (§8(e)).
 *
 * Two input forms:
 *   OSC_FEED_QP            M, C, J, b, T, mask: what update_osc_data hands the QP (osc.h:376-455),
 *                          7,664 B per Go2 env; solved by osc_batch_solve(_warm).
 *   OSC_FEED_JOINT_STATES  qpos, qvel, T, mask: what update_mj_data packs (osc.h:350-374), 568 B
 *                          per Go2 env; the kinematics (osc_batch_kinematics) runs on the copy
 *                          stream right behind its H2D -- overlapping the previous tick's solve --
 *                          then osc_batch_solve(_warm): bitwise osc_batch_solve_qpos(_warm).
 * Layouts per array are those of osc_batch.h / osc_kinematics.h (env-major, row-major per env).
 *
 * Use (one host thread per feed):
 *   for (k = 0; ; ++k) {
 *     osc_host_feed_inputs(feed, k, &in);      // waits until slot k % depth is free
 *     ... write tick k's inputs into in.M / in.qpos / ... ...
 *     osc_host_feed_submit(feed, k);           // H2D, solve, D2H enqueued; returns at once
 *     if (k >= depth - 1) osc_host_feed_wait(feed, k - depth + 1, &out);   // torques of k-d+1
 *   }
 * Tick numbers start at 0 and are submitted in order.  The outputs of tick k stay valid until
 * tick k + depth is submitted.  depth 1 = no overlap (each tick's copies and solve in series).
 */
#ifndef OSC_HOST_FEED_H_
#define OSC_HOST_FEED_H_

#include <stddef.h>
#include <stdint.h>

#include "osc_batch.h"
#include "osc_kinematics.h"

#ifdef __cplusplus
extern "C" {
#endif

#define OSC_FEED_QP 0
#define OSC_FEED_JOINT_STATES 1

#define OSC_FEED_WARM 1u          /* flags: warm-start every tick from the previous one's solution */

#define OSC_FEED_MAX_DEPTH 8

typedef struct osc_host_feed osc_host_feed;

/* Pinned HOST pointers of one slot's inputs (the fields of the other form are NULL). */
typedef struct {
  double* M;                      /* [nenv][nv][nv]       (OSC_FEED_QP)                        */
  double* C;                      /* [nenv][nv]                                                */
  double* J;                      /* [nenv][6 ns][nv]                                          */
  double* b;                      /* [nenv][6 ns]                                              */
  double* qpos;                   /* [nenv][nq]           (OSC_FEED_JOINT_STATES)              */
  double* qvel;                   /* [nenv][nv]                                                */
  double* T;                      /* [nenv][ns][6]        (both)                               */
  double* contact_mask;           /* [nenv][nc]                                                */
  size_t bytes;                   /* the slot's whole input block (one H2D copy per tick)      */
} osc_feed_inputs;

/* Pinned HOST pointers of one tick's outputs. */
typedef struct {
  const double* tau;              /* [nenv][nu]                                                */
  const int32_t* status;          /* [nenv]  OSC_SOLVE_*                                       */
  const int32_t* iters;           /* [nenv]                                                    */
  size_t bytes;                   /* D2H bytes per tick                                        */
} osc_feed_outputs;

/* Per-stage durations of one tick, by HIP events on the stage's own stream (ms). */
typedef struct {
  float h2d_ms;
  float solve_ms;
  float d2h_ms;
  float h2d_start_to_d2h_end_ms;  /* the tick's latency on the device side                     */
  float kin_ms;                   /* OSC_FEED_JOINT_STATES: the kinematics kernel (run on the copy
                                     stream behind the H2D, overlapping the previous tick's
                                     solve); ~0 for OSC_FEED_QP                                */
} osc_feed_timing;

/* Create a feed on the current HIP device (that of `model`).  `kin` is required for
 * OSC_FEED_JOINT_STATES (the same robot: osc_batch_solve_qpos's rules) and must be NULL for
 * OSC_FEED_QP.  1 <= depth <= OSC_FEED_MAX_DEPTH.  Models with wheel rows are refused
 * (OSC_ERR_INVALID_ARGUMENT: their per-env directions are not part of either form). */
int osc_host_feed_create(const osc_model* model, const osc_kin_model* kin, int32_t nenv,
                         int32_t form, uint32_t flags, int32_t depth, osc_host_feed** out);
int osc_host_feed_destroy(osc_host_feed* feed);

/* Tick `tick`'s pinned input pointers (slot tick % depth).  Blocks until that slot's previous
 * H2D copy (tick - depth) has completed, so the caller may overwrite it.  `tick` must be the next
 * tick to submit. */
int osc_host_feed_inputs(osc_host_feed* feed, int32_t tick, osc_feed_inputs* in);

/* Enqueue tick `tick` (the next one in order): its H2D copy on the copy stream, the solve on the
 * solve stream after it, the D2H of tau / status / iters on the return stream after that.
 * Returns without waiting.  A solve error (osc_batch_solve's argument checks) is returned here; an
 * error past the argument checks leaves the tick half enqueued, so the feed then refuses every
 * further tick (OSC_ERR_DEVICE) and can only be destroyed. */
int osc_host_feed_submit(osc_host_feed* feed, int32_t tick);

/* Block until tick `tick`'s outputs are in pinned host memory and return pointers to them.
 * `tick` must be submitted and not older than the last `depth` submitted ticks. */
int osc_host_feed_wait(osc_host_feed* feed, int32_t tick, osc_feed_outputs* out);

/* Stage durations of a completed tick (osc_host_feed_wait returned for it). */
int osc_host_feed_timing(osc_host_feed* feed, int32_t tick, osc_feed_timing* timing);

#ifdef __cplusplus
}
#endif

#endif /* OSC_HOST_FEED_H_ */
