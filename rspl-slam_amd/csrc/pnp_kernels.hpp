#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace rspl {
namespace pnp {

constexpr int kMaxIters = 128;  // RANSAC iterations (hypotheses) per frame
constexpr int kHypWaves = 4;   // hypotheses (one wave each) per workgroup of pnp_hyp_kernel

struct Desc {      // one frame of the batch
  int p0, n;       // correspondences [p0, p0 + n)
  int s0, iters;   // subsets [s0, s0 + iters) of 5 indices
  double K[4];     // fx fy cx cy
  double thr2;     // reprojection_error^2
  double confidence;
};

struct Out {       // per-frame result (host-mapped)
  double Rwc[9];
  double twc[3];
  int n_inliers, hyps;
};

struct Args {
  const Desc* frames;
  const double* pts;      // [P][3], float-rounded like cv::Point3f
  const double* kps;      // [P][2], float-rounded like cv::Point2f
  const int32_t* subsets; // [S][5]
  uint8_t* inl;           // [P] host-mapped
  Out* out;               // [B] host-mapped
  double* hyp;            // [B][kMaxIters][12] hypothesis R (row-major) | t
  int* hcnt;              // [B][kMaxIters] inlier count, -1: the minimal solver failed
  unsigned long long* prof;  // RSPL_PNP_PROF (null otherwise): wall_clock64 stamps of frame 0's hypothesis 0
                             // [0, 8) and of its acceptance / refinement [8, 12)
};

// max_iters: the largest RANSAC iteration count of the batch (hypothesis grid width)
hipError_t solve(const Args& a, int batch, int max_iters, hipStream_t s);

}  // namespace pnp
}  // namespace rspl
