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
  const int* status;     // AssignArgs::status of the sets (nullable): an overflowed set matches nothing
};

// Frame::AddRightFeatures' stereo filter (frame.cc:157-167) on the device: the SuperGlue match
// index of each left keypoint (idx[q] = right keypoint or -1) -> (q, t) pairs inside the disparity
// window, compacted in any order (MatchLines only counts them) into matches, count into *n_out.
struct StereoArgs {
  const int32_t* idx;     // [n_left_points]
  const int* n_points;    // [2] left / right keypoint counts
  const double* pts;      // left record j at pts + j * stride + xoff, right at + pt_batch
  size_t pt_batch;
  int stride, xoff;
  double min_x, max_x, max_y;
  int* matches;           // [max_matches][2]
  int* n_out;             // the full count of kept matches (may exceed max_matches)
  int* status;            // 1: more than max_matches passed the filter (the first max_matches kept)
  int max_matches;
};
// right line of each left line from the line matches (frame.cc:189-196, the reference's > 0 test)
struct RightArgs {
  const int* line_matches;  // [n_left]
  const double* lines_right;  // [max_lines][4]
  const int* n_lines;       // [2]
  double* out;              // [n_left][4]
  uint8_t* valid;           // [n_left]
};

// the detector's front (LineDetector::LineExtractor, line_processor.cc:464-465): cv::resize(0.5,
// INTER_LINEAR) of the u8 image and cv::Canny's per-pixel classification of the half image
// (3x3 Sobel, replicated border, L1 magnitude, the non-maximum suppression sectors, thresholds):
// half [h][w] u8, cls [h][w] u8 (2 strong, 0 candidate, 1 none), h = H / 2, w = W / 2
struct CannyArgs {
  const uint8_t* img;
  int H, W, stride;
  uint8_t* half;
  uint8_t* cls;
  int low, high;
};
hipError_t canny_classes(const CannyArgs& a, hipStream_t s);

hipError_t assign(const AssignArgs& a, int B, hipStream_t s);
// device-side counts of a device call: n_lines = {nl0, nl1}, n_points = counts[0..1], zeroed n_matches
hipError_t set_counts(int* n_lines, int nl0, int nl1, int* n_points, const int32_t* counts, int* n_matches,
                      hipStream_t s);
hipError_t stereo_filter(const StereoArgs& a, int max_left, hipStream_t s);
hipError_t right_lines(const RightArgs& a, int max_lines, hipStream_t s);
hipError_t match(const MatchArgs& a, int P, hipStream_t s);

}  // namespace lines
}  // namespace rspl
