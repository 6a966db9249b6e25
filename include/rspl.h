/*
 * rspl.h -- C ABI of the MI355X-native SuperPoint -> SuperGlue -> local-BA hot path.
 *
 * Drop-in boundary for the reference's C++ API (llliuqingyu/RSPL-SLAM):
 *   SuperPoint      include/super_point.h:20-66     -> rspl_sp_*
 *   SuperGlue       include/super_glue.h:20-71      -> rspl_sg_*
 *   PointMatching   include/point_matching.h:7-18   -> rspl_pm_*
 *   LocalmapOptimization
 *                   include/g2o_optimization/g2o_optimization.h:15-19 -> rspl_ba_*
 *   FrameOptimization
 *                   include/g2o_optimization/g2o_optimization.h:20-22 -> rspl_frame_*
 *   SolvePnPWithCV  include/g2o_optimization/g2o_optimization.h:24    -> rspl_pnp_*
 * Plain pointers and sizes only; no Eigen / OpenCV / torch types.  Every call
 * returns RSPL_OK (0) or a negative RSPL_E_* code (rspl_last_error() has the
 * text).  Handles are NOT thread-safe: callers serialise, exactly as the
 * reference's MapBuilder::_gpu_mutex does (src/map_builder.cc:276-278).
 * Device memory is owned by the handle and allocated once at create time
 * (no per-call allocation, unlike Thirdparty/TensorRTBuffer buffers.h:209-233).
 *
 * Feature layout (SuperPoint output / SuperGlue input) is the reference's
 * Eigen::Matrix<double,259,Dynamic> column-major storage
 * (SuperPoint::process_output, src/super_point.cpp:285-319; resized at :298): feature i occupies doubles [259*i, 259*i+259):
 *   [0] score, [1] x, [2] y, [3..258] L2-normalised descriptor.
 */
#ifndef RSPL_H_
#define RSPL_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RSPL_OK 0
#define RSPL_E_ARG (-1)      /* bad argument / shape */
#define RSPL_E_WEIGHTS (-2)  /* weight blob missing or malformed */
#define RSPL_E_DEVICE (-3)   /* HIP runtime error */
#define RSPL_E_CAPACITY (-4) /* output or arena capacity exceeded */
#define RSPL_E_SOLVER (-5)   /* linear solve failed */

#define RSPL_FEATURE_ROWS 259

/* RSPL_PREC_FP16: fp16 MFMA operands, fp32 accumulation (the reference's TensorRT kFP16 engines,
 * src/super_point.cpp:97-99, src/super_glue.cpp:132).  RSPL_PREC_FP16X3 (SuperPoint only): split fp16 --
 * every activation and weight carried as hi + lo fp16, three fp16 MFMA products per step, fp32-grade
 * results (keypoint sets of the fp32 path) at the fp16 MFMA rate. */
enum { RSPL_PREC_FP32 = 0, RSPL_PREC_FP16 = 1, RSPL_PREC_FP16X3 = 2 };

const char* rspl_last_error(void);
const char* rspl_version(void);
/* ABI revision of the structs in this header; a consumer checks rspl_abi_version() ==
 * RSPL_ABI_VERSION at startup (the library writes caller-allocated structs such as
 * rspl_map_report at the size of ITS header).  2: rspl_map_report gained the stage times. */
#define RSPL_ABI_VERSION 2
int rspl_abi_version(void);

/* ------------------------------------------------------------------------ */
/* Runtime helpers (system ROCm HIP runtime).  Callers that share a process  */
/* with another HIP runtime (e.g. PyTorch's bundled one) use these instead,  */
/* so only one runtime ever touches the device.                              */
/* ------------------------------------------------------------------------ */
int rspl_device_count(int* count);
int rspl_set_device(int device);
int rspl_malloc(void** ptr, size_t bytes);
int rspl_free(void* ptr);
int rspl_memcpy_h2d(void* dst, const void* src, size_t bytes, void* stream);
int rspl_memcpy_d2h(void* dst, const void* src, size_t bytes, void* stream);
int rspl_memset(void* dst, int value, size_t bytes, void* stream);
int rspl_memcpy_d2d(void* dst, const void* src, size_t bytes, void* stream);
int rspl_stream_create(void** stream);
/* high != 0: the device's highest stream priority (latency-critical chains) */
int rspl_stream_create_priority(void** stream, int high);
/* A stream whose kernels stay off reserve_cus CUs spread over the chip (HIP CU mask): the
 * throughput streams (SuperPoint / SuperGlue) leave those CUs free, so the latency-bound BA
 * chain never waits behind them for a CU slot. */
int rspl_stream_create_reserving(void** stream, int reserve_cus);
int rspl_stream_destroy(void* stream);
int rspl_stream_synchronize(void* stream);
int rspl_device_synchronize(void);
/* Cross-stream ordering without host synchronisation (pipelining SuperPoint of the
 * next frame beside SuperGlue of this one): record an event on one stream, make
 * another stream wait for it. */
int rspl_event_create(void** event);
int rspl_event_record(void* event, void* stream);
int rspl_stream_wait_event(void* stream, void* event);
int rspl_event_destroy(void* event);
/* HIP-event timer on a stream: rspl_timer_record(t, 0|1, stream) marks
 * start / stop; rspl_timer_elapsed_ms waits for stop and returns ms. */
typedef struct rspl_timer rspl_timer;
int rspl_timer_create(rspl_timer** t);
int rspl_timer_record(rspl_timer* t, int which, void* stream);
int rspl_timer_elapsed_ms(rspl_timer* t, float* ms);
void rspl_timer_destroy(rspl_timer* t);

/* ------------------------------------------------------------------------ */
/* SuperPoint: SuperPointConfig (include/read_configs.h:9-18) minus TRT-only */
/* fields; max_height/max_width size the device arena like the TRT profile   */
/* kMAX does (src/super_point.cpp:46-53).                                 */
/* ------------------------------------------------------------------------ */
typedef struct {
  int max_keypoints;         /* top-k; -1 keeps all (top_k_keypoints, src/super_point.cpp:192-204) */
  double keypoint_threshold; /* scores > threshold (src/super_point.cpp:154-165) */
  int remove_borders;        /* border in pixels (src/super_point.cpp:168-183) */
  int max_height;            /* arena sizing; H, W must be multiples of 8 */
  int max_width;
  int max_batch;             /* images per batched device call (>= 1) */
  int precision;             /* RSPL_PREC_FP32 (parity), RSPL_PREC_FP16 or RSPL_PREC_FP16X3 */
  int device;                /* HIP device ordinal */
} rspl_sp_config;

typedef struct rspl_sp rspl_sp;

/* SuperPoint::SuperPoint + build() (src/super_point.cpp:13-86).
 * weights_path: RSPLWT01 blob holding the reference state_dict
 * (convert2onnx/superpoint.py:86-105). */
int rspl_sp_create(const rspl_sp_config* cfg, const char* weights_path, rspl_sp** out);

/* SuperPoint::infer (src/super_point.cpp:104-135): rectified u8 image
 * (row stride in bytes) -> features[259 * capacity]; *n_out = keypoints. */
int rspl_sp_infer(rspl_sp* sp, const uint8_t* image, int height, int width, int stride,
                  double* features, int capacity, int* n_out);

/* Device-resident batched form: B images in device memory
 * (d_images + b*image_pitch), features to d_features + b*259*capacity,
 * counts to d_counts[b] (device int32).  stream may be NULL (handle stream). */
int rspl_sp_infer_device(rspl_sp* sp, const uint8_t* d_images, int batch, int height, int width,
                         int stride, size_t image_pitch, double* d_features, int capacity,
                         int32_t* d_counts, void* stream);

/* Intermediate maps of the last device call for image b (for tests):
 * scores [H*W] f32 after NMS, desc [256*(H/8)*(W/8)] f32 channel-major. */
int rspl_sp_debug_maps(rspl_sp* sp, int b, float* scores, float* desc);

/* Test hook: the device simple_nms (convert2onnx/superpoint.py:6-33, radius 4) of a host
 * score map [H][W] (any H, W within the arena) -> out [H][W]. */
int rspl_sp_debug_nms(rspl_sp* sp, const float* scores, int height, int width, float* out);

/* Per-stage device time (HIP events on the launch stream) summed over the calls
 * made since rspl_sp_profile(sp, 1).  Stages: 0 conv1a+conv1b+pool (fused),
 * 1 conv2a..conv4b, 2 convPa|convDa, 3 1x1 heads (softmax/d2s, L2 norm),
 * 4 NMS + candidates, 5 top-k, 6 descriptor sampling. */
#define RSPL_SP_STAGES 7
int rspl_sp_profile(rspl_sp* sp, int enable);
int rspl_sp_stage_times(rspl_sp* sp, float* ms, int* calls);

void rspl_sp_destroy(rspl_sp* sp);

/* ------------------------------------------------------------------------ */
/* SuperGlue: SuperGlueConfig (include/read_configs.h:20-28).               */
/* ------------------------------------------------------------------------ */
typedef struct {
  int image_width;   /* used by PointMatching::NormalizeKeypoints */
  int image_height;
  int max_keypoints; /* per image; arena sizing (the TRT profile allows 1024, src/super_glue.cpp:54-75) */
  int max_batch;     /* pairs per batched device call */
  int sinkhorn_iterations; /* 100 (convert2onnx/superglue.py:216) */
  int precision;
  int device;
} rspl_sg_config;

typedef struct rspl_sg rspl_sg;

int rspl_sg_create(const rspl_sg_config* cfg, const char* weights_path, rspl_sg** out);

/* SuperGlue::infer (src/super_glue.cpp:137-197): f0/f1 are 259 x n feature
 * matrices whose keypoints are ALREADY normalised (as PointMatching passes
 * them).  Outputs: indices0[n0], indices1[n1] (-1 = unmatched), mscores0[n0],
 * mscores1[n1]  (decode: src/super_glue.cpp:339-367). */
int rspl_sg_infer(rspl_sg* sg, const double* f0, int n0, const double* f1, int n1,
                  int32_t* indices0, int32_t* indices1, double* mscores0, double* mscores1);

/* Device-resident batched form.  Pair p reads f0 = d_feat0 + p*259*stride_feat,
 * n0 = n0[p] (DEVICE int32 counts, e.g. rspl_sp_infer_device's d_counts),
 * likewise image 1; writes d_idx0 + p*max_kp etc.
 * normalize != 0 applies PointMatching::NormalizeKeypoints on device first. */
int rspl_sg_infer_device(rspl_sg* sg, int batch, const double* d_feat0, const int* n0,
                         const double* d_feat1, const int* n1, int stride_feat, int normalize,
                         int32_t* d_idx0, int32_t* d_idx1, double* d_ms0, double* d_ms1,
                         void* stream);

/* As rspl_sg_infer_device, with the log-Sinkhorn and decode enqueued on post_stream (after
 * an event on stream): the next call's GNN on `stream` overlaps this call's Sinkhorn.
 * Results are complete when post_stream reaches this point.  The counts are snapshotted,
 * so the caller may reuse n0/n1 once `stream` has passed the call. */
int rspl_sg_infer_device2(rspl_sg* sg, int batch, const double* d_feat0, const int* n0,
                          const double* d_feat1, const int* n1, int stride_feat, int normalize,
                          int32_t* d_idx0, int32_t* d_idx1, double* d_ms0, double* d_ms1, void* stream,
                          void* post_stream);

/* Log-assignment Z [(n0+1)*(n1+1)] f32 of the last call, pair p (for tests). */
int rspl_sg_debug_scores(rspl_sg* sg, int p, float* Z);

/* Sinkhorn health of the device paths.  The persistent log-Sinkhorn exchanges u / v between
 * co-resident workgroups with bounded spins; a pair whose exchange timed out sets a sticky
 * flag (its indices / scores are then invalid).  After synchronising the stream the results
 * were produced on, rspl_sg_status returns RSPL_OK, or RSPL_E_DEVICE with *pair_flags = the
 * bitmask of the failed pairs (bit 31 = any pair >= 31), and clears the flags.  rspl_sg_infer
 * and rspl_pm_match check it themselves. */
int rspl_sg_status(rspl_sg* sg, uint32_t* pair_flags);

/* Test hooks.  rspl_sg_debug_inject(sg, 1, limit): workgroup 0 of pair 0 reports an exchange
 * timeout at iteration 0 and every spin is bounded by `limit` polls (0 = the default), to
 * prove the failure reaches the caller.  rspl_sg_debug_sinkhorn: bins (alpha) + log_optimal_transport
 * (convert2onnx/superglue.py:185-205) of a host score matrix [n0][n1] -> Z [(n0+1)][(n1+1)].
 * rspl_sg_debug_decode: the device decode (src/super_glue.cpp:258-367) of a host Z. */
int rspl_sg_debug_inject(rspl_sg* sg, int inject, unsigned spin_limit);
int rspl_sg_debug_sinkhorn(rspl_sg* sg, const float* scores, int n0, int n1, float alpha, int iters, float* Z);
int rspl_sg_debug_decode(rspl_sg* sg, const float* Z, int n0, int n1, int32_t* indices0, int32_t* indices1,
                         double* mscores0, double* mscores1);

/* Stages: 0 prep + keypoint encoder, 1 18 GNN layers, 2 final_proj + scores + bins,
 * 3 hand-over to the post stream (queueing behind the previous call's post work; no kernel),
 * 4 log-Sinkhorn (one kernel), 5 decode. */
#define RSPL_SG_STAGES 6
int rspl_sg_profile(rspl_sg* sg, int enable);
int rspl_sg_stage_times(rspl_sg* sg, float* ms, int* calls);

void rspl_sg_destroy(rspl_sg* sg);

/* ------------------------------------------------------------------------ */
/* PointMatching (src/point_matching.cc): normalise, SuperGlue, mutual check, */
/* DMatch(i, j, 1 - (ms0 + ms1)/2).  outlier_rejection (F-matrix RANSAC,     */
/* default off in the reference) is not implemented: RSPL_E_ARG if set.      */
/* ------------------------------------------------------------------------ */
typedef struct {
  int32_t query_idx;
  int32_t train_idx;
  float distance;
} rspl_dmatch;

int rspl_pm_match(rspl_sg* sg, const double* f0, int n0, const double* f1, int n1,
                  rspl_dmatch* matches, int capacity, int* n_matches, int outlier_rejection);

/* ------------------------------------------------------------------------ */
/* Local bundle adjustment: LocalmapOptimization                            */
/* (src/g2o_optimization/g2o_optimization.cc:21-252).  Vertex ids of the    */
/* reference's std::maps are remapped to dense indices by the caller.       */
/* ------------------------------------------------------------------------ */
typedef struct {
  int n_cameras;
  const double* cameras;        /* [n][5] fx, fy, cx, cy, bf (include/camera.h:25-29) */

  int n_poses;
  const double* pose_q;         /* [n][4] rotation of T_wc, Eigen coeffs order (x, y, z, w) */
  const double* pose_p;         /* [n][3] translation of T_wc */
  const uint8_t* pose_fixed;    /* [n] Pose3d::fixed */

  int n_points;
  const double* points;         /* [n][3] world position */

  int n_lines;
  const double* lines;          /* [n][6] g2o::Line3D Pluecker (w, d) */

  int n_mono;                   /* MonoPointConstraint (types.h:54-78) */
  const int32_t* mono_pose;
  const int32_t* mono_point;
  const int32_t* mono_camera;   /* may be NULL -> camera 0 */
  const double* mono_obs;       /* [n][2] */

  int n_stereo;                 /* StereoPointConstraint (types.h:81-105) */
  const int32_t* stereo_pose;
  const int32_t* stereo_point;
  const int32_t* stereo_camera;
  const double* stereo_obs;     /* [n][3] u, v, u_right */

  int n_mono_line;              /* MonoLineConstraint (types.h:124-148) */
  const int32_t* mono_line_pose;
  const int32_t* mono_line_line;
  const int32_t* mono_line_camera;
  const double* mono_line_obs;  /* [n][4] x1 y1 x2 y2 */

  int n_stereo_line;            /* StereoLineConstraint (types.h:151-174) */
  const int32_t* stereo_line_pose;
  const int32_t* stereo_line_line;
  const int32_t* stereo_line_camera;
  const double* stereo_line_obs; /* [n][8] left x1 y1 x2 y2, right x1 y1 x2 y2 */

  /* OptimizationConfig (include/read_configs.h:50-56): chi2 thresholds; the
   * Huber deltas are (float)sqrt(threshold) (g2o_optimization.cc:77-78,125-126) */
  double th_mono_point, th_stereo_point, th_mono_line, th_stereo_line;
  int iterations_first;   /* 10 (g2o_optimization.cc:173) */
  int iterations_second;  /* 5  (g2o_optimization.cc:210) */
} rspl_ba_problem;

typedef struct {
  double* pose_q;     /* [n_poses][4] optimised T_wc rotation (x, y, z, w) */
  double* pose_p;     /* [n_poses][3] */
  double* points;     /* [n_points][3] */
  double* lines;      /* [n_lines][6] */
  uint8_t* mono_inlier;
  uint8_t* stereo_inlier;
  uint8_t* mono_line_inlier;
  uint8_t* stereo_line_inlier;
  double chi2_first;  /* robust chi2 at the end of the first optimize() */
  double chi2_second; /* chi2 at the end of the second optimize() */
  int iterations_done_first;
  int iterations_done_second;
} rspl_ba_result;

typedef struct {
  int max_poses;
  int max_points;
  int max_lines;
  int max_edges;      /* per edge type */
  int device;
} rspl_ba_config;

typedef struct rspl_ba rspl_ba;

int rspl_ba_create(const rspl_ba_config* cfg, rspl_ba** out);
int rspl_ba_local(rspl_ba* ba, const rspl_ba_problem* problem, rspl_ba_result* result);
void rspl_ba_destroy(rspl_ba* ba);
/* The reference's tracking thread (map_builder.cc:48-49, 188-276): rspl_ba_submit queues one local BA
 * call for the handle's native host thread, which runs the queued calls in order (rspl_ba_local each);
 * like the reference's feature thread it blocks while two calls are already waiting
 * (_tracking_data_buffer, map_builder.cc:176).  problem, its arrays and result must stay valid until
 * the call has run.  A queued call's inputs are read (staged) by a second host thread of the handle as
 * soon as a staging slot is free -- while the previous call still runs on the device -- so do not
 * modify a problem after submitting it.  rspl_ba_join waits until every queued call has run and returns the first failure
 * since the previous join (0: none), with the number of calls, their LM iterations (first + second
 * optimize) and their summed wall time in ms (each may be NULL).  Do not call rspl_ba_local on the
 * handle while calls are queued; rspl_ba_destroy runs the queued calls before it frees the handle. */
int rspl_ba_submit(rspl_ba* ba, const rspl_ba_problem* problem, rspl_ba_result* result);
int rspl_ba_join(rspl_ba* ba, long long* calls, long long* iterations, double* ms);
/* Run this handle's kernels only on the reserve_cus CUs that rspl_stream_create_reserving
 * streams leave free (0 = all CUs, highest stream priority: the default). */
int rspl_ba_use_reserved_cus(rspl_ba* ba, int reserve_cus);
/* Kernel timing (measurement): every `every`-th rspl_ba_local call (0: off) records HIP events on the
 * BA stream around each LM trial's two launches (device LM path); rspl_ba_kernel_times returns and
 * resets the totals -- ms[0] / launches[0]: Schur chunks + fused reduced-system solve, ms[1] /
 * launches[1]: update + cost + speculative linearisation -- over the trials that did work. */
int rspl_ba_kernel_timing(rspl_ba* ba, int every);
int rspl_ba_kernel_times(rspl_ba* ba, double* ms, long long* launches);
/* Per-call host timeline (measurement): the handle keeps the host timestamps of its last 4096 calls
 * (CLOCK_MONOTONIC seconds -- the clock of Python's time.perf_counter / time.monotonic on Linux).
 * Record of RSPL_BA_TRACE_W doubles: [0] submitted (rspl_ba_submit; rspl_ba_local: entry), [1] staging
 * started, [2] staging done, [3] device part started (tracking thread), [4] upload queued, [5] optimize(10)
 * stopped (mailbox read), [6] optimize(5) stopped, [7] call done (results written back), [8] staging slot,
 * [9] flags (1 staging slot, 2 edge-pair list, 4 pose-diagonal partials, 8 timing events: a buffer grown inside
 * the call; 16 optimize(5)'s setup ran from the speculative queue behind optimize(10)'s trials, 32 optimize(10)
 * needed trials beyond its first batch), [10] LM iterations, [11] 1 for rspl_ba_local, 0 for a submitted call.
 * rspl_ba_trace copies the oldest min(cap, recorded) records and clears the ring; *n = records copied. */
/* Line edges' Jacobians (EdgeSE3ProjectLine / EdgeStereoSE3ProjectLine do not override linearizeOplus, so
 * g2o differentiates them numerically: central difference, delta 1e-9).  0 (default): that central
 * difference; 1: its analytic delta -> 0 limit (truncation ~1e-18 relative; the central difference's own
 * cancellation noise, ~1e-7 relative, is absent -- results become smooth in the inputs). */
int rspl_ba_set_line_jacobian(rspl_ba* ba, int analytic);
#define RSPL_BA_TRACE_W 12
int rspl_ba_trace(rspl_ba* ba, double* out, int cap, int* n);
/* Test hook (host only, no device): the host staging of rspl_ba_local -- the edges of rank `rank` of
 * `nranks` (1: all) in landmark-CSR order -- with the host workers from par_edges edges (0: serial).
 * n_local = {local edges E, local point edges Ep}; lm_off [n_points + n_lines + 1]; per CSR position
 * k < E: type (0..3), pose, landmark (lines offset by n_points), camera, caller edge id (over the four
 * types in order), reduced pose id (-1: fixed or without edges); eobs: 4 doubles per point edge, then
 * 8 per line edge (arrays sized for all edges). */
int rspl_ba_debug_stage(const rspl_ba_problem* problem, int par_edges, int rank, int nranks, int* n_local,
                        int* lm_off, int8_t* etype, int* epose, int* elm, int* ecam, int* gmap, int* lpose,
                        double* eobs);

/* ------------------------------------------------------------------------ */
/* Landmark-sharded local BA: nranks handles -- one per  */
/* GPU (RCCL over xGMI), or several on one device (in-process group) -- each  */
/* call rspl_ba_local with the SAME problem.  Rank r keeps only the edges of  */
/* the landmarks it owns (landmark g owned by rank g % nranks: points first,  */
/* then lines, as in rspl_ba_problem), computes its Schur contribution       */
/* S_r = sum (Hpp - Hpl Hll^-1 Hlp) / b_r, and the ranks sum-all-reduce, per  */
/* LM trial, the reduced camera system (pose-pair blocks + gradients + the    */
/* landmark-inversion flag) and the trial's {chi2, LM scale, fail}; at        */
/* lambda-init the pose-block diagonals and each rank's landmark maximum.    */
/* Every rank factors the same reduced system, so the LM decisions agree.    */
/* Results are complete on every rank (owned landmarks and edge flags are    */
/* gathered by a final all-reduce).                                          */
/* ------------------------------------------------------------------------ */
/* in-place sum all-reduce of count doubles on a HIP stream (stream-ordered); 0 = ok */
typedef int (*rspl_allreduce_fn)(void* ctx, double* d_buf, size_t count, void* stream);
int rspl_ba_set_shard(rspl_ba* ba, int rank, int nranks, rspl_allreduce_fn allreduce, void* ctx);

/* RCCL communicator (librccl is loaded at first use).  Rank 0 makes the id, the
 * caller broadcasts its RSPL_COMM_ID_BYTES to the other ranks out of band
 * (e.g. torch.distributed), every rank creates its communicator. */
#define RSPL_COMM_ID_BYTES 128
typedef struct rspl_comm rspl_comm;
int rspl_comm_unique_id(uint8_t* id /* [RSPL_COMM_ID_BYTES] */);
int rspl_comm_create(const uint8_t* id, int rank, int nranks, int device, rspl_comm** out);
int rspl_comm_allreduce_sum(void* comm, double* d_buf, size_t count, void* stream);  /* an rspl_allreduce_fn */
void rspl_comm_destroy(rspl_comm* comm);
int rspl_ba_set_comm(rspl_ba* ba, rspl_comm* comm);

/* In-process group: nranks BA handles on ONE device, each driven by its own host
 * thread (a landmark-sharded solve inside one GPU; also how the sharded math is
 * tested on a single-GPU host).  The sum is formed in rank order on the device. */
typedef struct rspl_group rspl_group;
int rspl_group_create(int nranks, rspl_group** out);
void rspl_group_destroy(rspl_group* group);
int rspl_ba_set_group(rspl_ba* ba, rspl_group* group, int rank);

/* ------------------------------------------------------------------------ */
/* Tracking pose optimisation: FrameOptimization                            */
/* (src/g2o_optimization/g2o_optimization.cc:256-398, declared at           */
/* include/g2o_optimization/g2o_optimization.h:20-22; called per frame by   */
/* MapBuilder::FramePoseOptimization, src/map_builder.cc:583).  One pose     */
/* vertex, fixed world points, unary EdgeSE3ProjectXYZOnlyPose /            */
/* EdgeStereoSE3ProjectXYZOnlyPose edges with Huber kernels; 4 rounds of    */
/* optimize(10) from the initial pose with chi2 re-classification, kernels  */
/* dropped for the last round.  A batch of independent frames (one sequence */
/* each, or many sequences per GPU) runs in ONE kernel launch, one wavefront */
/* per frame.                                                               */
/* ------------------------------------------------------------------------ */
typedef struct {
  int n_cameras;
  const double* cameras;        /* [n][5] fx, fy, cx, cy, bf */
  double pose_q[4];             /* initial T_wc rotation (x, y, z, w) */
  double pose_p[3];             /* initial T_wc translation */
  int n_points;
  const double* points;         /* [n][3] world positions (Position3d, fixed) */
  int n_mono;                   /* MonoPointConstraint: id_point, id_camera, keypoint */
  const int32_t* mono_point;
  const int32_t* mono_camera;   /* may be NULL -> camera 0 */
  const double* mono_obs;       /* [n][2] */
  const uint8_t* mono_inlier_in;   /* Constraint::inlier on entry; NULL = all true (map_builder.cc:560) */
  int n_stereo;                 /* StereoPointConstraint */
  const int32_t* stereo_point;
  const int32_t* stereo_camera;
  const double* stereo_obs;     /* [n][3] u, v, u_right */
  const uint8_t* stereo_inlier_in;
  double th_mono_point, th_stereo_point;  /* OptimizationConfig (tracking) */
} rspl_frame_problem;

typedef struct {
  double pose_q[4];             /* optimised T_wc (x, y, z, w) */
  double pose_p[3];
  uint8_t* mono_inlier;         /* [n_mono] Constraint::inlier on exit (may be NULL) */
  uint8_t* stereo_inlier;
  int n_inliers;                /* FrameOptimization's return value */
  int rounds;                   /* optimize() rounds run (4, or 1 when < 10 edges) */
  int iterations[4];            /* LM iterations done per round */
  double chi2[4];               /* final (robust) chi2 per round */
} rspl_frame_result;

typedef struct {
  int max_batch;                /* frames per call */
  int max_edges;                /* total edges (mono + stereo) over a whole batch */
  int max_points;               /* total points over a whole batch */
  int device;
} rspl_frame_config;

typedef struct rspl_frame rspl_frame;

int rspl_frame_create(const rspl_frame_config* cfg, rspl_frame** out);
/* batch independent FrameOptimization calls; results[b] receives frame b.  Batches of more than 256
 * frames sum each frame's normal equations in another order (one wave per frame instead of four):
 * results then differ from a small batch's in the last bits, within the oracle tolerances. */
int rspl_frame_optimize(rspl_frame* h, const rspl_frame_problem* problems, int batch, rspl_frame_result* results);
void rspl_frame_destroy(rspl_frame* h);

/* ------------------------------------------------------------------------ */
/* SolvePnPWithCV (src/g2o_optimization/g2o_optimization.cc:402-461; declared at */
/* include/g2o_optimization/g2o_optimization.h:24, called per frame by          */
/* MapBuilder::FramePoseOptimization, src/map_builder.cc:515): the RANSAC of    */
/* cv::solvePnPRansac (5-point EPnP hypotheses, 100 iterations, 20 px, 0.99,    */
/* SOLVEPNP_ITERATIVE refinement on the inliers), zero distortion               */
/* (camera.cc:145-147).  The correspondences are the caller's already-filtered  */
/* (map point, keypoint) pairs (:417-431); the caller maps inlier slots back to  */
/* map-point ids (:452-457).  A batch of frames is one launch, one workgroup per */
/* frame, the hypotheses of a frame solved side by side.                        */
/* ------------------------------------------------------------------------ */
typedef struct {
  double fx, fy, cx, cy;        /* Camera::GetCamerMatrix */
  int n;                        /* correspondences; < 8 -> 0 inliers (:433) */
  const double* points;         /* [n][3] map points (world), rounded to float like cv::Point3f */
  const double* keypoints;      /* [n][2] pixels, rounded to float like cv::Point2f */
  int iterations;               /* 100 (:439); at most 128 */
  double reprojection_error;    /* 20.0 px */
  double confidence;            /* 0.99 */
} rspl_pnp_problem;

typedef struct {
  double Rwc[9];                /* row-major Rwc = Rcw^T (:447-449); valid when n_inliers > 0 */
  double twc[3];                /* -Rwc tcw */
  uint8_t* inlier;              /* [n] inlier mask of the RANSAC model (may be NULL) */
  int n_inliers;                /* SolvePnPWithCV's return value (cv_inliers.rows) */
  int hypotheses;               /* RANSAC iterations evaluated (adaptive) */
} rspl_pnp_result;

typedef struct {
  int max_batch;
  int max_points;               /* correspondences over a whole batch */
  int device;
} rspl_pnp_config;

typedef struct rspl_pnp rspl_pnp;

int rspl_pnp_create(const rspl_pnp_config* cfg, rspl_pnp** out);
int rspl_pnp_solve(rspl_pnp* h, const rspl_pnp_problem* problems, int batch, rspl_pnp_result* results);
void rspl_pnp_destroy(rspl_pnp* h);
/* debug (parity tests): frame `frame` of the last rspl_pnp_solve -- every hypothesis' inlier
   count (-1: the minimal solver failed) and R (row-major) | t, up to `max` hypotheses; returns
   the frame's hypothesis count or a negative error */
int rspl_pnp_debug_hypotheses(rspl_pnp* h, int frame, int max, int32_t* counts, double* poses);

/* ------------------------------------------------------------------------ */
/* Map-side local BA: the keyframe / map-point / map-line */
/* graph of the reference's Map (include/map.h:15-52) and                   */
/* Map::LocalMapOptimization (src/map.cc:537-808) around rspl_ba_local:      */
/* window selection (SearchNeighborFrames, :471-525; one extra fixed frame,  */
/* :593-606), the constraints that enter the BA (:608-707), outlier removal  */
/* (RemoveOutliers / RemoveLineOutliers, :712-757, :818-895), the            */
/* covisibility update (UpdateFrameConnection, :897-937), write-back and     */
/* line endpoints (UppdateMapline, :121-177).  Frames, map points and map    */
/* lines are named by id (shared_ptr -> id; a frame's map-point / map-line   */
/* slot holds an id or -1).  Equal covisibility weights are ordered by frame */
/* id (the reference: by FramePtr address, i.e. allocation order).          */
/* ------------------------------------------------------------------------ */
typedef struct {
  const double* camera;          /* [5] fx fy cx cy bf (Map::_camera) */
  /* OptimizationConfig (_backend_optimization_config, configs_euroc.yaml:56-61) */
  double th_mono_point, th_stereo_point, th_mono_line, th_stereo_line;
  int iterations_first, iterations_second;
} rspl_map_config;

typedef struct {
  int frame_id;
  double timestamp;
  const double* Twc;             /* [16] row-major 4x4 pose (Frame::GetPose) */
  int n_keypoints;
  const double* keypoints;       /* [n][3] x, y (features rows 1-2), u_right (< 0: mono) */
  int n_lines;
  const double* lines_left;      /* [n_lines][4] Frame::_lines */
  const double* lines_right;     /* [n_lines][4] Frame::_lines_right (may be NULL) */
  const uint8_t* lines_right_valid; /* [n_lines] (may be NULL: none) */
  const int32_t* pol_offsets;    /* [n_lines + 1] CSR of Frame::_points_on_lines (may be NULL) */
  const int32_t* pol_points;     /*   keypoint index */
  const double* pol_dist;        /*   distance */
  int parent_id;                 /* Frame::_parent (-1: none) */
} rspl_map_keyframe;

typedef struct {
  int n_poses, n_fixed, n_points, n_lines;
  int n_mono, n_stereo, n_mono_line, n_stereo_line;
  int n_point_outliers, n_line_outliers;
  double chi2_first, chi2_second;
  int iterations_first, iterations_second;
  /* host wall time of the call's stages, microseconds: window + constraint assembly, the GPU
   * LocalmapOptimization (rspl_ba_local incl. staging), outlier removal + covisibility + write-back */
  double assembly_us, ba_us, finish_us;
} rspl_map_report;

enum { RSPL_MAP_UNTRIANGULATED = 0, RSPL_MAP_GOOD = 1, RSPL_MAP_BAD = 2 };  /* Mappoint::Type */

typedef struct rspl_map rspl_map;
int rspl_map_create(const rspl_map_config* cfg, rspl_map** out);        /* Map::Map */
void rspl_map_destroy(rspl_map* m);
/* Map::InsertKeyframe's bookkeeping (_keyframes, _keyframe_ids; map.cc:24-28) */
int rspl_map_add_keyframe(rspl_map* m, const rspl_map_keyframe* kf);
int rspl_map_add_mappoint(rspl_map* m, int id, const double* p, int type);       /* Map::InsertMappoint */
int rspl_map_add_mapline(rspl_map* m, int id, const double* line3d, int type);   /* Map::InsertMapline */
/* Mappoint::AddObverser + Frame::InsertMappoint; Mapline::AddObverser + Frame::InsertMapline */
int rspl_map_add_point_observation(rspl_map* m, int point_id, int frame_id, int keypoint_idx);
int rspl_map_add_line_observation(rspl_map* m, int line_id, int frame_id, int line_idx);
/* bulk forms: n map points (types may be NULL: Good); n observations of frame_id */
int rspl_map_add_mappoints(rspl_map* m, int n, const int32_t* ids, const double* p, const int32_t* types);
int rspl_map_add_point_observations(rspl_map* m, int frame_id, int n, const int32_t* point_ids,
                                    const int32_t* keypoints);
int rspl_map_update_connections(rspl_map* m, int frame_id);             /* Map::UpdateFrameConnection */
/* Map::LocalMapOptimization(new_frame) with the local BA on `ba` (GPU) */
int rspl_map_local_optimization(rspl_map* m, int frame_id, rspl_ba* ba, rspl_map_report* report);
/* the same window / constraint selection without the BA (no write-back, no outlier removal) */
int rspl_map_assemble(rspl_map* m, int frame_id, rspl_map_report* report);
/* the rest of LocalMapOptimization (outlier removal, covisibility update, write-back, line
 * endpoints; map.cc:712-802) applied to the last assembled problem with a supplied BA result */
int rspl_map_finish(rspl_map* m, const rspl_ba_result* result, rspl_map_report* report);
/* the last assembled problem: ids of the dense poses / points / lines (ascending, the
 * LocalmapOptimization vertex order), and per constraint type t (mono, stereo, mono line, stereo
 * line) the dense pose / landmark index and the observation (2 / 3 / 4 / 8 doubles) */
int rspl_map_last_problem(const rspl_map* m, int32_t* pose_ids, uint8_t* pose_fixed, int32_t* point_ids,
                          int32_t* line_ids, int32_t* const* c_pose, int32_t* const* c_lm, double* const* c_obs);
int rspl_map_get_keyframe(const rspl_map* m, int frame_id, double* Twc, int* n_connections);
/* Frame::GetOrderedConnections(-1): ascending (weight, frame id) */
int rspl_map_get_connections(const rspl_map* m, int frame_id, int32_t* ids, int32_t* weights, int cap, int* n);
int rspl_map_get_mappoint(const rspl_map* m, int id, double* p, int* type, int* n_observers, int32_t* frames,
                          int32_t* keypoints, int cap);
int rspl_map_get_mapline(const rspl_map* m, int id, double* line3d, int* type, int* n_observers,
                         double* endpoints, int* endpoints_valid);
int rspl_map_get_frame_slots(const rspl_map* m, int frame_id, int32_t* mappoints, int32_t* maplines);
/* Map::SaveKeyframeTrajectory (map.cc:1007-1024): TUM "t tx ty tz qx qy qz qw", %.9f */
int rspl_map_save_trajectory(const rspl_map* m, const char* path);

/* ------------------------------------------------------------------------------------------ */
/* Line front end: the detector (cv::resize + FLD, restated, parity         */
/* unpinned), then the merge passes, the point-line assignment and the line matching.  The RCF */
/* edge net is not rebuilt (no weights): its edge map is the detector's input.                */
/* ------------------------------------------------------------------------------------------ */

/* LineDetector::LineExtractor after fld->detect (src/line_processor.cc:460-490): segments
 * [n][4] float as FLD returns them on the half-size image -> lines [n_out][4] double at full
 * size; do_merge runs MergeLines(0.05, 5, 15), FilterShortLines(30), MergeLines(0.03, 3, 50),
 * FilterShortLines(60) (:492-665, 11-24).  Host code (a sequential clustering); *n_out is set
 * even when it exceeds capacity (RSPL_E_CAPACITY). */
int rspl_line_extract(const float* segments, int n, int do_merge, double* lines, int capacity, int* n_out);

typedef struct rspl_lines rspl_lines;
typedef struct rspl_lines_config {
  int max_lines;   /* lines per image, <= 1024 */
  int max_points;  /* keypoints per image, <= 4096 */
  int max_pairs;   /* point-line pairs per image (the sum of the std::map sizes) */
  int max_matches; /* point matches per MatchLines call */
  int device;
} rspl_lines_config;

int rspl_lines_create(const rspl_lines_config* cfg, rspl_lines** out);
void rspl_lines_destroy(rspl_lines* h);
/* AssignPointsToLines(lines, points, relation) (src/line_processor.cc:163-216) on the GPU.
 * lines [n_lines][4] double; features = the 259 x N column-major keypoint records (x, y = rows
 * 1, 2).  relation as CSR: line i's points are point_idx[offsets[i] .. offsets[i+1]) in
 * ascending index order (the std::map<int, double> order) with dist[] = the map values. */
int rspl_lines_assign(rspl_lines* h, const double* lines, int n_lines, const double* features, int n_points,
                      int* offsets, int* point_idx, double* dist, int capacity);
/* MatchLines(points_on_line0, points_on_line1, point_matches, point_num0, point_num1, line_matches)
 * (src/line_processor.cc:221-283) on the GPU.  The relations as rspl_lines_assign returns them
 * (the distances are not needed); matches [n_matches][2] = (queryIdx, trainIdx);
 * line_matches [n_lines0]: the matched line of image 1, or -1. */
int rspl_lines_match(rspl_lines* h, const int* offsets0, const int* idx0, int n_lines0, const int* offsets1,
                     const int* idx1, int n_lines1, const int* matches, int n_matches, int n_points0, int n_points1,
                     int* line_matches);
/* The line part of Frame::AddLeftFeatures + Frame::AddRightFeatures (src/frame.cc:124-129,
 * 150-196): the stereo matches inside the disparity window (camera_limits = {MinXDiff,
 * MaxXDiff, MaxYDiff}, frame.cc:157-167), both images' point-line assignments (one launch),
 * MatchLines -> per left line the right line and its validity (line_matches[i] > 0, as the
 * reference tests it).  *n_kept_matches = the filtered stereo matches' count. */
int rspl_lines_stereo(rspl_lines* h, const double* lines_left, int n_left, const double* features_left,
                      int n_points_left, const double* lines_right, int n_right, const double* features_right,
                      int n_points_right, const int* stereo_matches, int n_matches, const double* camera_limits,
                      double* lines_right_out, uint8_t* lines_right_valid, int* n_kept_matches);
/* Device-resident rspl_lines_stereo for a GPU pipeline: lines (device [n][4] doubles), the
 * SuperPoint device features [2][feat_cap][259] (image 0 left, 1 right) with their device counts
 * [2], SuperGlue's device match index of each left keypoint (right keypoint or -1); outputs the
 * right line and validity per left line in device memory.  Stream-ordered: no host copy, no sync.
 * A point-line overflow of max_pairs leaves every line unmatched; rspl_lines_status reports it
 * once the stream has completed. */
int rspl_lines_stereo_device(rspl_lines* h, const double* d_lines_left, int n_left, const double* d_lines_right,
                             int n_right, const double* d_features, int feat_cap, const int32_t* d_counts,
                             const int32_t* d_match_idx, const double* camera_limits, double* d_lines_right_out,
                             uint8_t* d_lines_right_valid, void* stream);
int rspl_lines_status(rspl_lines* h, int* overflow);

/* LineDetector's detector (src/line_processor.cc:455-466): cv::resize(image, 0.5, 0.5,
 * INTER_LINEAR) and cv::ximgproc::FastLineDetector(length_threshold, distance_threshold,
 * canny_th1, canny_th2, canny_aperture_size, do_merge = false)->detect on the half image, as the
 * reference runs it on the RCF edge map (map_builder.cc:286, 327).  FLD is OpenCV contrib (not
 * vendored, absent): restated (oracle/fld_ref.py), parity unpinned.  The resize, the Sobel
 * gradients and Canny's non-maximum suppression / thresholds run on the GPU; hysteresis, chaining
 * and segment fitting on the host.  segments [n][4] float (x1 y1 x2 y2) on the HALF image, as
 * fld->detect returns them (rspl_line_extract scales and merges); even image sizes; *n_out is set
 * even when it exceeds capacity (RSPL_E_CAPACITY). */
typedef struct {
  int length_threshold;          /* 10 (configs/configs_euroc.yaml:31) */
  double distance_threshold;     /* 1.414213562 */
  double canny_th1, canny_th2;   /* 200, 250 */
  int canny_aperture_size;       /* 3 (the only size supported) */
} rspl_fld_config;
int rspl_lines_detect(rspl_lines* h, const uint8_t* image, int H, int W, int stride, const rspl_fld_config* cfg,
                      float* segments, int capacity, int* n_out);
/* LineDetector::LineExtractor (src/line_processor.cc:460-490) asynchronously: rspl_lines_detect +
 * rspl_line_extract (x2 scale, the merge passes when do_merge) on a native worker thread of the handle,
 * as the reference runs its line threads beside the point thread (map_builder.cc:285-290, 325-337).
 * The image must stay valid until rspl_lines_extract_wait returns; one job in flight per handle, and
 * no other call on the handle meanwhile.  _wait blocks for the job and writes lines [n][4] (full-size
 * x1 y1 x2 y2) and, when job_us is not NULL, the job's own duration on the worker (microseconds);
 * *n_out is set even when it exceeds capacity (RSPL_E_CAPACITY). */
int rspl_lines_extract_async(rspl_lines* h, const uint8_t* image, int H, int W, int stride,
                             const rspl_fld_config* cfg, int do_merge);
int rspl_lines_extract_wait(rspl_lines* h, double* lines, int capacity, int* n_out, double* job_us);
/* the same join, the lines copied into DEVICE memory d_lines [capacity][4] in stream order (from the
 * handle's pinned result buffer; no host synchronisation with the stream) -- the feed of
 * rspl_lines_stereo_device */
int rspl_lines_extract_wait_device(rspl_lines* h, double* d_lines, int capacity, int* n_out, double* job_us,
                                   void* stream);
/* debug (parity tests): the last rspl_lines_detect's half image and Canny classes (2 strong, 0
 * candidate, 1 none) for an H x W input, [H/2][W/2] each */
int rspl_lines_debug_canny(rspl_lines* h, int H, int W, uint8_t* half, uint8_t* cls);

#ifdef __cplusplus
}
#endif
#endif /* RSPL_H_ */
