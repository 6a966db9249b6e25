/* A plain-C consumer of include/rspl.h (test infrastructure; tests/test_abi_c.py drives it).
 *
 *   abi_consumer layout                       struct sizes / field offsets as JSON, compared with the
 *                                             ctypes mirrors (rspl-slam_amd/capi.py, ba_types.py)
 *   abi_consumer run DIR SP_WEIGHTS SG_WEIGHTS  rspl_sp_infer, rspl_sg_infer, rspl_pm_match and
 *                                             rspl_ba_local on inputs in DIR/{sp,sg,ba}_in.bin,
 *                                             outputs to DIR/{sp,sg,ba}_out.bin
 *
 * Built with gcc against the header alone (no HIP headers), linked to librspl.so. */
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "rspl.h"

#define BEGIN(T) printf("%s\"%s\": {\"size\": %zu, \"fields\": {", first_t ? "" : ", ", #T, sizeof(T)), first_t = 0, first_f = 1
#define F(T, f) printf("%s\"%s\": %zu", first_f ? "" : ", ", #f, offsetof(T, f)), first_f = 0
#define END() printf("}}")

static int layout(void) {
  int first_t = 1, first_f = 1;
  printf("{");
  BEGIN(rspl_sp_config); F(rspl_sp_config, max_keypoints); F(rspl_sp_config, keypoint_threshold);
  F(rspl_sp_config, remove_borders); F(rspl_sp_config, max_height); F(rspl_sp_config, max_width);
  F(rspl_sp_config, max_batch); F(rspl_sp_config, precision); F(rspl_sp_config, device); END();
  BEGIN(rspl_sg_config); F(rspl_sg_config, image_width); F(rspl_sg_config, image_height);
  F(rspl_sg_config, max_keypoints); F(rspl_sg_config, max_batch); F(rspl_sg_config, sinkhorn_iterations);
  F(rspl_sg_config, precision); F(rspl_sg_config, device); END();
  BEGIN(rspl_dmatch); F(rspl_dmatch, query_idx); F(rspl_dmatch, train_idx); F(rspl_dmatch, distance); END();
  BEGIN(rspl_ba_config); F(rspl_ba_config, max_poses); F(rspl_ba_config, max_points); F(rspl_ba_config, max_lines);
  F(rspl_ba_config, max_edges); F(rspl_ba_config, device); END();
  BEGIN(rspl_ba_problem);
  F(rspl_ba_problem, n_cameras); F(rspl_ba_problem, cameras); F(rspl_ba_problem, n_poses); F(rspl_ba_problem, pose_q);
  F(rspl_ba_problem, pose_p); F(rspl_ba_problem, pose_fixed); F(rspl_ba_problem, n_points); F(rspl_ba_problem, points);
  F(rspl_ba_problem, n_lines); F(rspl_ba_problem, lines); F(rspl_ba_problem, n_mono); F(rspl_ba_problem, mono_pose);
  F(rspl_ba_problem, mono_point); F(rspl_ba_problem, mono_camera); F(rspl_ba_problem, mono_obs);
  F(rspl_ba_problem, n_stereo); F(rspl_ba_problem, stereo_pose); F(rspl_ba_problem, stereo_point);
  F(rspl_ba_problem, stereo_camera); F(rspl_ba_problem, stereo_obs); F(rspl_ba_problem, n_mono_line);
  F(rspl_ba_problem, mono_line_pose); F(rspl_ba_problem, mono_line_line); F(rspl_ba_problem, mono_line_camera);
  F(rspl_ba_problem, mono_line_obs); F(rspl_ba_problem, n_stereo_line); F(rspl_ba_problem, stereo_line_pose);
  F(rspl_ba_problem, stereo_line_line); F(rspl_ba_problem, stereo_line_camera); F(rspl_ba_problem, stereo_line_obs);
  F(rspl_ba_problem, th_mono_point); F(rspl_ba_problem, th_stereo_point); F(rspl_ba_problem, th_mono_line);
  F(rspl_ba_problem, th_stereo_line); F(rspl_ba_problem, iterations_first); F(rspl_ba_problem, iterations_second);
  END();
  BEGIN(rspl_ba_result); F(rspl_ba_result, pose_q); F(rspl_ba_result, pose_p); F(rspl_ba_result, points);
  F(rspl_ba_result, lines); F(rspl_ba_result, mono_inlier); F(rspl_ba_result, stereo_inlier);
  F(rspl_ba_result, mono_line_inlier); F(rspl_ba_result, stereo_line_inlier); F(rspl_ba_result, chi2_first);
  F(rspl_ba_result, chi2_second); F(rspl_ba_result, iterations_done_first); F(rspl_ba_result, iterations_done_second);
  END();
  BEGIN(rspl_frame_config); F(rspl_frame_config, max_batch); F(rspl_frame_config, max_edges);
  F(rspl_frame_config, max_points); F(rspl_frame_config, device); END();
  BEGIN(rspl_frame_problem); F(rspl_frame_problem, n_cameras); F(rspl_frame_problem, cameras);
  F(rspl_frame_problem, pose_q); F(rspl_frame_problem, pose_p); F(rspl_frame_problem, n_points);
  F(rspl_frame_problem, points); F(rspl_frame_problem, n_mono); F(rspl_frame_problem, mono_point);
  F(rspl_frame_problem, mono_camera); F(rspl_frame_problem, mono_obs); F(rspl_frame_problem, mono_inlier_in);
  F(rspl_frame_problem, n_stereo); F(rspl_frame_problem, stereo_point); F(rspl_frame_problem, stereo_camera);
  F(rspl_frame_problem, stereo_obs); F(rspl_frame_problem, stereo_inlier_in); F(rspl_frame_problem, th_mono_point);
  F(rspl_frame_problem, th_stereo_point); END();
  BEGIN(rspl_frame_result); F(rspl_frame_result, pose_q); F(rspl_frame_result, pose_p);
  F(rspl_frame_result, mono_inlier); F(rspl_frame_result, stereo_inlier); F(rspl_frame_result, n_inliers);
  F(rspl_frame_result, rounds); F(rspl_frame_result, iterations); F(rspl_frame_result, chi2); END();
  BEGIN(rspl_pnp_config); F(rspl_pnp_config, max_batch); F(rspl_pnp_config, max_points); F(rspl_pnp_config, device);
  END();
  BEGIN(rspl_pnp_problem); F(rspl_pnp_problem, fx); F(rspl_pnp_problem, fy); F(rspl_pnp_problem, cx);
  F(rspl_pnp_problem, cy); F(rspl_pnp_problem, n); F(rspl_pnp_problem, points); F(rspl_pnp_problem, keypoints);
  F(rspl_pnp_problem, iterations); F(rspl_pnp_problem, reprojection_error); F(rspl_pnp_problem, confidence); END();
  BEGIN(rspl_pnp_result); F(rspl_pnp_result, Rwc); F(rspl_pnp_result, twc); F(rspl_pnp_result, inlier);
  F(rspl_pnp_result, n_inliers); F(rspl_pnp_result, hypotheses); END();
  BEGIN(rspl_map_config); F(rspl_map_config, camera); F(rspl_map_config, th_mono_point);
  F(rspl_map_config, th_stereo_point); F(rspl_map_config, th_mono_line); F(rspl_map_config, th_stereo_line);
  F(rspl_map_config, iterations_first); F(rspl_map_config, iterations_second); END();
  BEGIN(rspl_map_keyframe); F(rspl_map_keyframe, frame_id); F(rspl_map_keyframe, timestamp); F(rspl_map_keyframe, Twc);
  F(rspl_map_keyframe, n_keypoints); F(rspl_map_keyframe, keypoints); F(rspl_map_keyframe, n_lines);
  F(rspl_map_keyframe, lines_left); F(rspl_map_keyframe, lines_right); F(rspl_map_keyframe, lines_right_valid);
  F(rspl_map_keyframe, pol_offsets); F(rspl_map_keyframe, pol_points); F(rspl_map_keyframe, pol_dist);
  F(rspl_map_keyframe, parent_id); END();
  BEGIN(rspl_map_report); F(rspl_map_report, n_poses); F(rspl_map_report, n_fixed); F(rspl_map_report, n_points);
  F(rspl_map_report, n_lines); F(rspl_map_report, n_mono); F(rspl_map_report, n_stereo); F(rspl_map_report, n_mono_line);
  F(rspl_map_report, n_stereo_line); F(rspl_map_report, n_point_outliers); F(rspl_map_report, n_line_outliers);
  F(rspl_map_report, chi2_first); F(rspl_map_report, chi2_second); F(rspl_map_report, iterations_first);
  F(rspl_map_report, iterations_second);
  F(rspl_map_report, assembly_us); F(rspl_map_report, ba_us); F(rspl_map_report, finish_us); END();
  BEGIN(rspl_lines_config); F(rspl_lines_config, max_lines); F(rspl_lines_config, max_points);
  F(rspl_lines_config, max_pairs); F(rspl_lines_config, max_matches); F(rspl_lines_config, device); END();
  printf("}\n");
  return 0;
}

/* ---- binary I/O ---- */
static FILE* open_in(const char* dir, const char* name, const char* mode) {
  char path[4096];
  snprintf(path, sizeof path, "%s/%s", dir, name);
  FILE* f = fopen(path, mode);
  if (!f) fprintf(stderr, "cannot open %s\n", path);
  return f;
}
static void* rd(FILE* f, size_t bytes) {
  void* p = malloc(bytes ? bytes : 1);
  if (bytes && fread(p, 1, bytes, f) != bytes) {
    fprintf(stderr, "short read (%zu bytes)\n", bytes);
    exit(2);
  }
  return p;
}
static void wr(FILE* f, const void* p, size_t bytes) {
  if (bytes && fwrite(p, 1, bytes, f) != bytes) exit(2);
}
#define CHECK(call)                                                              \
  do {                                                                           \
    int rc_ = (call);                                                            \
    if (rc_ != RSPL_OK) {                                                        \
      fprintf(stderr, "%s -> %d: %s\n", #call, rc_, rspl_last_error());          \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

/* SuperPoint: sp_in.bin = int32 {H, W, k, border}, double thr, u8 image[H*W] -> int32 n, double[259 n] */
static int run_sp(const char* dir, const char* weights) {
  FILE* f = open_in(dir, "sp_in.bin", "rb");
  if (!f) return 1;
  int32_t* hdr = (int32_t*)rd(f, 4 * sizeof(int32_t));
  double* thr = (double*)rd(f, sizeof(double));
  const int H = hdr[0], W = hdr[1], k = hdr[2];
  uint8_t* img = (uint8_t*)rd(f, (size_t)H * W);
  fclose(f);
  rspl_sp_config c;
  memset(&c, 0, sizeof c);
  c.max_keypoints = k; c.keypoint_threshold = *thr; c.remove_borders = hdr[3];
  c.max_height = H; c.max_width = W; c.max_batch = 1; c.precision = RSPL_PREC_FP32; c.device = 0;
  rspl_sp* sp = NULL;
  CHECK(rspl_sp_create(&c, weights, &sp));
  double* feats = (double*)malloc(sizeof(double) * 259 * (size_t)k);
  int n = 0;
  CHECK(rspl_sp_infer(sp, img, H, W, W, feats, k, &n));
  rspl_sp_destroy(sp);
  FILE* o = open_in(dir, "sp_out.bin", "wb");
  if (!o) return 1;
  wr(o, &n, sizeof n);
  wr(o, feats, sizeof(double) * 259 * (size_t)n);
  fclose(o);
  free(feats); free(img); free(thr); free(hdr);
  return 0;
}

/* SuperGlue + PointMatching: sg_in.bin = int32 {n0, n1, width, height}, double f0[259 n0], f1[259 n1]
 * (raw SuperPoint features).  rspl_sg_infer gets them normalised here exactly as
 * PointMatching::NormalizeKeypoints does (src/point_matching.cc:50-62); rspl_pm_match gets them raw.
 * -> int32 idx0[n0], idx1[n1], double ms0[n0], ms1[n1], int32 nm, rspl_dmatch[nm] */
static int run_sg(const char* dir, const char* weights) {
  FILE* f = open_in(dir, "sg_in.bin", "rb");
  if (!f) return 1;
  int32_t* hdr = (int32_t*)rd(f, 4 * sizeof(int32_t));
  const int n0 = hdr[0], n1 = hdr[1], width = hdr[2], height = hdr[3];
  double* f0 = (double*)rd(f, sizeof(double) * 259 * (size_t)n0);
  double* f1 = (double*)rd(f, sizeof(double) * 259 * (size_t)n1);
  fclose(f);
  rspl_sg_config c;
  memset(&c, 0, sizeof c);
  c.image_width = width; c.image_height = height; c.max_keypoints = n0 > n1 ? n0 : n1; c.max_batch = 1;
  c.sinkhorn_iterations = 100; c.precision = RSPL_PREC_FP32; c.device = 0;
  rspl_sg* sg = NULL;
  CHECK(rspl_sg_create(&c, weights, &sg));
  double* g0 = (double*)malloc(sizeof(double) * 259 * (size_t)n0);
  double* g1 = (double*)malloc(sizeof(double) * 259 * (size_t)n1);
  memcpy(g0, f0, sizeof(double) * 259 * (size_t)n0);
  memcpy(g1, f1, sizeof(double) * 259 * (size_t)n1);
  const double scale = (width > height ? width : height) * 0.7;
  for (int i = 0; i < n0; i++) {
    g0[259 * i + 1] = (f0[259 * i + 1] - width / 2) / scale;
    g0[259 * i + 2] = (f0[259 * i + 2] - height / 2) / scale;
  }
  for (int i = 0; i < n1; i++) {
    g1[259 * i + 1] = (f1[259 * i + 1] - width / 2) / scale;
    g1[259 * i + 2] = (f1[259 * i + 2] - height / 2) / scale;
  }
  int32_t* i0 = (int32_t*)malloc(sizeof(int32_t) * (size_t)n0);
  int32_t* i1 = (int32_t*)malloc(sizeof(int32_t) * (size_t)n1);
  double* m0 = (double*)malloc(sizeof(double) * (size_t)n0);
  double* m1 = (double*)malloc(sizeof(double) * (size_t)n1);
  CHECK(rspl_sg_infer(sg, g0, n0, g1, n1, i0, i1, m0, m1));
  const int cap = n0 < n1 ? n0 : n1;
  rspl_dmatch* mt = (rspl_dmatch*)malloc(sizeof(rspl_dmatch) * (size_t)(cap > 0 ? cap : 1));
  int nm = 0;
  CHECK(rspl_pm_match(sg, f0, n0, f1, n1, mt, cap, &nm, 0));
  rspl_sg_destroy(sg);
  FILE* o = open_in(dir, "sg_out.bin", "wb");
  if (!o) return 1;
  wr(o, i0, sizeof(int32_t) * (size_t)n0); wr(o, i1, sizeof(int32_t) * (size_t)n1);
  wr(o, m0, sizeof(double) * (size_t)n0); wr(o, m1, sizeof(double) * (size_t)n1);
  wr(o, &nm, sizeof nm); wr(o, mt, sizeof(rspl_dmatch) * (size_t)nm);
  fclose(o);
  free(mt); free(m1); free(m0); free(i1); free(i0); free(g1); free(g0); free(f1); free(f0); free(hdr);
  return 0;
}

/* LocalmapOptimization: ba_in.bin = int32 {n_cameras, n_poses, n_points, n_lines, n_mono, n_stereo,
 * n_mono_line, n_stereo_line, iterations_first, iterations_second}, double th[4], then the arrays of
 * rspl_ba_problem in declaration order.  -> double {chi2_first, chi2_second}, int32 {it1, it2},
 * pose_q, pose_p, points, lines, the four inlier arrays (u8). */
static int run_ba(const char* dir) {
  FILE* f = open_in(dir, "ba_in.bin", "rb");
  if (!f) return 1;
  int32_t* n = (int32_t*)rd(f, 10 * sizeof(int32_t));
  double* th = (double*)rd(f, 4 * sizeof(double));
  rspl_ba_problem p;
  memset(&p, 0, sizeof p);
  p.n_cameras = n[0]; p.n_poses = n[1]; p.n_points = n[2]; p.n_lines = n[3];
  p.n_mono = n[4]; p.n_stereo = n[5]; p.n_mono_line = n[6]; p.n_stereo_line = n[7];
  p.iterations_first = n[8]; p.iterations_second = n[9];
  p.th_mono_point = th[0]; p.th_stereo_point = th[1]; p.th_mono_line = th[2]; p.th_stereo_line = th[3];
  p.cameras = (const double*)rd(f, sizeof(double) * 5 * (size_t)p.n_cameras);
  p.pose_q = (const double*)rd(f, sizeof(double) * 4 * (size_t)p.n_poses);
  p.pose_p = (const double*)rd(f, sizeof(double) * 3 * (size_t)p.n_poses);
  p.pose_fixed = (const uint8_t*)rd(f, (size_t)p.n_poses);
  p.points = (const double*)rd(f, sizeof(double) * 3 * (size_t)p.n_points);
  p.lines = (const double*)rd(f, sizeof(double) * 6 * (size_t)p.n_lines);
#define EDGES(pre, cnt, lm, od)                                                   \
  p.pre##_pose = (const int32_t*)rd(f, sizeof(int32_t) * (size_t)cnt);            \
  p.pre##_##lm = (const int32_t*)rd(f, sizeof(int32_t) * (size_t)cnt);            \
  p.pre##_camera = (const int32_t*)rd(f, sizeof(int32_t) * (size_t)cnt);          \
  p.pre##_obs = (const double*)rd(f, sizeof(double) * od * (size_t)cnt);
  EDGES(mono, p.n_mono, point, 2)
  EDGES(stereo, p.n_stereo, point, 3)
  EDGES(mono_line, p.n_mono_line, line, 4)
  EDGES(stereo_line, p.n_stereo_line, line, 8)
  fclose(f);
  rspl_ba_config c;
  memset(&c, 0, sizeof c);
  c.max_poses = p.n_poses; c.max_points = p.n_points > 0 ? p.n_points : 1; c.max_lines = p.n_lines > 0 ? p.n_lines : 1;
  c.max_edges = 1;
  const int ne[4] = {p.n_mono, p.n_stereo, p.n_mono_line, p.n_stereo_line};
  for (int i = 0; i < 4; i++)
    if (ne[i] > c.max_edges) c.max_edges = ne[i];
  c.device = 0;
  rspl_ba* ba = NULL;
  CHECK(rspl_ba_create(&c, &ba));
  rspl_ba_result r;
  memset(&r, 0, sizeof r);
  r.pose_q = (double*)malloc(sizeof(double) * 4 * (size_t)p.n_poses);
  r.pose_p = (double*)malloc(sizeof(double) * 3 * (size_t)p.n_poses);
  r.points = (double*)malloc(sizeof(double) * 3 * (size_t)(p.n_points + 1));
  r.lines = (double*)malloc(sizeof(double) * 6 * (size_t)(p.n_lines + 1));
  r.mono_inlier = (uint8_t*)malloc((size_t)p.n_mono + 1);
  r.stereo_inlier = (uint8_t*)malloc((size_t)p.n_stereo + 1);
  r.mono_line_inlier = (uint8_t*)malloc((size_t)p.n_mono_line + 1);
  r.stereo_line_inlier = (uint8_t*)malloc((size_t)p.n_stereo_line + 1);
  CHECK(rspl_ba_local(ba, &p, &r));
  rspl_ba_destroy(ba);
  FILE* o = open_in(dir, "ba_out.bin", "wb");
  if (!o) return 1;
  wr(o, &r.chi2_first, sizeof(double)); wr(o, &r.chi2_second, sizeof(double));
  wr(o, &r.iterations_done_first, sizeof(int)); wr(o, &r.iterations_done_second, sizeof(int));
  wr(o, r.pose_q, sizeof(double) * 4 * (size_t)p.n_poses); wr(o, r.pose_p, sizeof(double) * 3 * (size_t)p.n_poses);
  wr(o, r.points, sizeof(double) * 3 * (size_t)p.n_points); wr(o, r.lines, sizeof(double) * 6 * (size_t)p.n_lines);
  wr(o, r.mono_inlier, (size_t)p.n_mono); wr(o, r.stereo_inlier, (size_t)p.n_stereo);
  wr(o, r.mono_line_inlier, (size_t)p.n_mono_line); wr(o, r.stereo_line_inlier, (size_t)p.n_stereo_line);
  fclose(o);
  return 0;
}

int main(int argc, char** argv) {
  if (rspl_abi_version() != RSPL_ABI_VERSION) {  /* caller-allocated structs follow this header's layout */
    fprintf(stderr, "librspl ABI %d, header ABI %d\n", rspl_abi_version(), RSPL_ABI_VERSION);
    return 3;
  }
  if (argc >= 2 && !strcmp(argv[1], "layout")) return layout();
  if (argc >= 5 && !strcmp(argv[1], "run")) {
    int rc = run_sp(argv[2], argv[3]);
    if (!rc) rc = run_sg(argv[2], argv[4]);
    if (!rc) rc = run_ba(argv[2]);
    if (!rc) printf("ok %s\n", rspl_version());
    return rc;
  }
  fprintf(stderr, "usage: %s layout | run DIR SP_WEIGHTS SG_WEIGHTS\n", argv[0]);
  return 2;
}
