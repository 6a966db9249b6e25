#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace rspl {
namespace lines {

constexpr int kMaxPointsLds = 4096;  // keypoints per image handled by one workgroup (LDS tables)

// AssignPointsToLines (line_processor.cc:163-216) for B images, one 1024-thread workgroup each.
// Image b: lines[b * max_lines .. ][4] doubles, n_lines[b]; keypoint j's x at
// pts[b * pt_batch + j * pt_stride + pt_xoff], y right after it (the 259-double feature records:
// stride 259, offset 1); n_points[b].  Output per image: CSR offsets[b][max_lines + 1], point
// indices ascending within a line (the std::map order) and their distances (float, as the
// reference computes them, widened to double).  status[b] = 1 when the image's pairs exceed cap.
struct AssignArgs {
  const double* lines;
  const int* n_lines;
  const double* pts;
  size_t pt_batch;
  int pt_stride, pt_xoff;
  const int* n_points;
  int* offsets;
  int* idx;
  double* dist;
  int max_lines, cap;
  int* status;
};

// MatchLines (line_processor.cc:221-283) for P problems, one 1024-thread workgroup each.
// Problem p: two assignments (CSR off/idx with max_lines + 1 / cap strides, as AssignArgs writes
// them), matches[p * max_matches ..][2] = (queryIdx, trainIdx), n_matches[p], keypoint counts
// n_points0/1[p].  Scratch: M [P][max_lines * max_lines] ints, inv [P][2][cap] ints.
// Out: line_matches[p * max_lines + i] = matched line of image 1 or -1.
struct MatchArgs {
  const int *off0, *idx0, *n_lines0, *n_points0;
  const int *off1, *idx1, *n_lines1, *n_points1;
  int set0, set1;        // problem p reads assignment sets set0 + p*step0, set1 + p*step1
  int step0, step1;
  const int* matches;
  const int* n_matches;
  int max_lines, cap, max_matches;
  int* M;
  int* inv;
  int* out;
};

hipError_t assign(const AssignArgs& a, int B, hipStream_t s);
hipError_t match(const MatchArgs& a, int P, hipStream_t s);

}  // namespace lines
}  // namespace rspl
