// Line front end after the detector: the LineDetector merge passes on the
// host, point-to-line assignment and shared-point line matching on the GPU (line_kernels.hip).
//
//   LineDetector::LineExtractor after fld->detect   src/line_processor.cc:460-490
//   LineDetector::MergeLines, MergeTwoLines,
//   FilterShortLines, PointLineDistance, AngleDiff   src/line_processor.cc:11-161, 492-665
//   AssignPointsToLines / MatchLines                 src/line_processor.cc:163-283 (kernels)
//   Frame::AddRightFeatures (line part)              src/frame.cc:150-203
//
// The merge is a sequential clustering over a few hundred segments per image (an angle sort, a
// neighbour search that breaks early in sorted order, BFS clusters, pairwise merges whose result
// depends on the order): it stays on the host, in the reference's float / double types.  FLD
// itself (cv::ximgproc) and the RCF edge net are not rebuilt: segments enter through the API.
#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <string>
#include <thread>
#include <array>
#include <cmath>
#include <cstring>
#include <numeric>
#include <set>
#include <type_traits>
#include <unordered_map>
#include <vector>

#include "common.hpp"
#include "line_kernels.hpp"

#pragma clang fp contract(off)

using namespace rspl;

namespace {

struct Seg {
  float v[4];
};

// line_processor.cc:11-24 (float lines)
void filter_short(std::vector<Seg>& ls, float thr) {
  const float t2 = thr * thr;
  size_t k = 0;
  for (const Seg& s : ls) {
    const float dx = s.v[2] - s.v[0], dy = s.v[3] - s.v[1];
    if (dx * dx + dy * dy > t2) ls[k++] = s;
  }
  ls.resize(k);
}

// line_processor.cc:41-50: float numerator; std::pow(float, int) is a double, so is the root
float point_line_distance(const Seg& l, float x0, float y0) {
  const float x1 = l.v[0], y1 = l.v[1], x2 = l.v[2], y2 = l.v[3];
  const float num = std::fabs((y2 - y1) * x0 + (x1 - x2) * y0 + ((x2 * y1) - (x1 * y2)));
  const double a = (double)(y2 - y1), b = (double)(x1 - x2);
  return (float)(num / std::sqrt(a * a + b * b));
}

// line_processor.cc:92-96
float angle_diff(float a1, float a2) {
  const float c1 = std::fabs(a2 - a1);
  const float c2 = (float)(M_PI + (double)std::min(a1, a2) - (double)std::max(a1, a2));
  return std::min(c1, c2);
}

// line_processor.cc:98-161: length-weighted centroid and angle in double; the angle of each
// segment is atan of the float slope (the float overload, atanf)
Seg merge_two(const Seg& p, const Seg& q) {
  const float ax = p.v[0], ay = p.v[1], bx = p.v[2], by = p.v[3];
  const float cx = q.v[0], cy = q.v[1], dx = q.v[2], dy = q.v[3];
  const float dlix = bx - ax, dliy = by - ay, dljx = dx - cx, dljy = dy - cy;
  const double li = std::sqrt((double)(dlix * dlix) + (double)(dliy * dliy));
  const double lj = std::sqrt((double)(dljx * dljx) + (double)(dljy * dljy));
  const double xg = (li * (double)(ax + bx) + lj * (double)(cx + dx)) / (2.0 * (li + lj));
  const double yg = (li * (double)(ay + by) + lj * (double)(cy + dy)) / (2.0 * (li + lj));
  const double thi = dlix == 0.0f ? M_PI / 2.0 : (double)atanf(dliy / dlix);
  const double thj = dljx == 0.0f ? M_PI / 2.0 : (double)atanf(dljy / dljx);
  double thr;
  if (std::fabs(thi - thj) <= M_PI / 2.0) {
    thr = (li * thi + lj * thj) / (li + lj);
  } else {
    const double tmp = thj - M_PI * (thj / std::fabs(thj));
    thr = (li * thi + lj * tmp) / (li + lj);
  }
  const double s = std::sin(thr), c = std::cos(thr);
  const double g[4] = {((double)ay - yg) * s + ((double)ax - xg) * c, ((double)by - yg) * s + ((double)bx - xg) * c,
                       ((double)cy - yg) * s + ((double)cx - xg) * c, ((double)dy - yg) * s + ((double)dx - xg) * c};
  const double lo = std::min(g[0], std::min(g[1], std::min(g[2], g[3])));
  const double hi = std::max(g[0], std::max(g[1], std::max(g[2], g[3])));
  Seg r;
  r.v[0] = (float)(lo * std::cos(thr) + xg);
  r.v[1] = (float)(lo * std::sin(thr) + yg);
  r.v[2] = (float)(hi * std::cos(thr) + xg);
  r.v[3] = (float)(hi * std::sin(thr) + yg);
  return r;
}

// line_processor.cc:492-665
std::vector<Seg> merge_lines(const std::vector<Seg>& src, float angle_thr, float dist_thr, float ep) {
  const size_t n = src.size();
  std::vector<Seg> dst;
  if (n == 0) return dst;  // the reference maps src[0] of an empty vector (undefined): empty in, empty out
  std::vector<float> ang(n), len(n);
  for (size_t i = 0; i < n; i++) {
    const float dx = src[i].v[2] - src[i].v[0], dy = src[i].v[3] - src[i].v[1];
    ang[i] = atanf(dy / dx);
    len[i] = std::sqrt(dx * dx + dy * dy);
  }
  std::vector<size_t> order(n);
  std::iota(order.begin(), order.end(), 0);
  // equal angles (axis-aligned segments, the two edges of one ridge) keep their input order: the
  // reference's std::sort leaves ties unspecified, the restatement takes them stable
  std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) { return ang[a] < ang[b]; });
  const float ep2 = ep * ep, quarter = (float)(M_PI / 4.0);
  // neighbours in the reference's push_back order: by sorted position of the other line
  std::vector<std::vector<size_t>> nbr(n);
  for (size_t i = 0; i < n; i++) {
    const size_t a = order[i];
    float x11 = src[a].v[0], y11 = src[a].v[1], x12 = src[a].v[2], y12 = src[a].v[3];
    const float a1 = ang[a];
    const bool sx = std::fabs(a1) < quarter;
    if ((sx && x12 < x11) || (!sx && y12 < y11)) {
      std::swap(x11, x12);
      std::swap(y11, y12);
    }
    for (size_t j = i + 1; j < n; j++) {
      const size_t b = order[j];
      float x21 = src[b].v[0], y21 = src[b].v[1], x22 = src[b].v[2], y22 = src[b].v[3];
      if ((sx && x22 < x21) || (!sx && y22 < y21)) {
        std::swap(x21, x22);
        std::swap(y21, y22);
      }
      if (angle_diff(a1, ang[b]) > angle_thr) {
        if (std::fabs(a1) < (M_PI_2 - (double)angle_thr)) break;  // sorted: no later line is closer
        continue;
      }
      const float m1x = 0.5f * (src[a].v[0] + src[a].v[2]), m1y = 0.5f * (src[a].v[1] + src[a].v[3]);
      const float m2x = 0.5f * (src[b].v[0] + src[b].v[2]), m2y = 0.5f * (src[b].v[1] + src[b].v[3]);
      if (point_line_distance(src[b], m1x, m1y) > dist_thr && point_line_distance(src[a], m2x, m2y) > dist_thr)
        continue;
      float cx12, cy12, cx21, cy21;
      if ((sx && x12 > x22) || (!sx && y12 > y22)) {
        cx12 = x22; cy12 = y22; cx21 = x11; cy21 = y11;
      } else {
        cx12 = x12; cy12 = y12; cx21 = x21; cy21 = y21;
      }
      bool merge = (sx && cx12 >= cx21) || (!sx && cy12 >= cy21);
      if (!merge) merge = (cx21 - cx12) * (cx21 - cx12) + (cy21 - cy12) * (cy21 - cy12) < ep2;
      if (merge) {
        nbr[a].push_back(b);
        nbr[b].push_back(a);
      }
    }
  }
  // connected components (breadth-first, each frontier in ascending line order)
  std::vector<int> code(n, -1);
  std::vector<std::vector<size_t>> clusters;
  for (size_t i = 0; i < n; i++) {
    if (code[i] >= 0) continue;
    const int c = (int)clusters.size();
    code[i] = c;
    std::vector<size_t> todo = nbr[i], cl{i};
    while (!todo.empty()) {
      std::set<size_t> next;
      for (size_t j : todo) {
        if (code[j] < 0) {
          code[j] = c;
          cl.push_back(j);
        }
        for (size_t k : nbr[j])
          if (code[k] < 0) next.insert(k);
      }
      todo.assign(next.begin(), next.end());
    }
    clusters.push_back(std::move(cl));
  }
  // sub-clusters: longest first, each unclaimed line with its direct neighbours
  std::vector<std::vector<size_t>> subs;
  for (auto& cl : clusters) {
    if (cl.size() <= 2) {
      subs.push_back(cl);
      continue;
    }
    std::stable_sort(cl.begin(), cl.end(), [&](size_t a, size_t b) { return len[a] > len[b]; });
    std::unordered_map<size_t, size_t> at;
    for (size_t k = 0; k < cl.size(); k++) at[cl[k]] = k;
    std::vector<bool> taken(cl.size(), false);
    for (size_t k = 0; k < cl.size(); k++) {
      if (taken[k]) continue;
      std::vector<size_t> sub{cl[k]};
      for (size_t m : nbr[cl[k]]) {
        taken[at[m]] = true;
        sub.push_back(m);
      }
      subs.push_back(std::move(sub));
    }
  }
  dst.reserve(subs.size());
  for (auto& sub : subs) {
    Seg l = src[sub[0]];
    for (size_t k = 1; k < sub.size(); k++) l = merge_two(l, src[sub[k]]);
    dst.push_back(l);
  }
  return dst;
}

}  // namespace

extern "C" int rspl_line_extract(const float* segments, int n, int do_merge, double* lines, int capacity, int* n_out) {
  RSPL_CHECK_ARG(n >= 0 && n_out && (n == 0 || segments) && capacity >= 0 && (capacity == 0 || lines),
                 "rspl_line_extract: bad argument");
  std::vector<Seg> src((size_t)n);
  for (int i = 0; i < n; i++)
    for (int k = 0; k < 4; k++) src[i].v[k] = segments[4 * i + k] * 2;  // detected on the half-size image
  std::vector<Seg> dst;
  if (do_merge) {
    std::vector<Seg> tmp = merge_lines(src, 0.05f, 5.f, 15.f);
    filter_short(tmp, 30.f);
    dst = merge_lines(tmp, 0.03f, 3.f, 50.f);
    filter_short(dst, 60.f);
  } else {
    dst = std::move(src);
  }
  *n_out = (int)dst.size();
  if ((int)dst.size() > capacity) {
    set_error("%zu lines exceed capacity %d", dst.size(), capacity);
    return RSPL_E_CAPACITY;
  }
  for (size_t i = 0; i < dst.size(); i++)
    for (int k = 0; k < 4; k++) lines[4 * i + k] = (double)dst[i].v[k];
  return RSPL_OK;
}

struct rspl_lines {
  rspl_lines_config cfg{};
  hipStream_t stream = nullptr;
  Arena arena;
  int cap = 0;
  double *lines, *pts, *dist;
  int *n_lines, *n_points, *offsets, *idx, *status;
  int *matches, *n_matches, *M, *inv, *out;
  // detector (rspl_lines_detect): device image / half image / classes, pinned host copies; grown on demand
  uint8_t *d_img = nullptr, *d_det = nullptr, *h_img = nullptr, *h_det = nullptr;
  size_t det_cap = 0;  // pixels of the largest full-size image so far
  int det_H = 0, det_W = 0;  // the last detection's image size (rspl_lines_debug_canny must match it)
  std::vector<uint8_t> edge;
  std::vector<int> stack;
  // asynchronous LineExtractor (rspl_lines_extract_async / _wait): a native worker thread of the handle
  // runs detect + the merge passes, so a caller's feature thread only submits and joins (the reference's
  // line threads, map_builder.cc:285-290, 325-337)
  std::thread worker;
  std::mutex mu;
  std::condition_variable cv;
  bool job = false, done = false, quit = false;
  const uint8_t* a_img = nullptr;
  int a_H = 0, a_W = 0, a_stride = 0, a_merge = 1, a_rc = 0, a_n = 0;
  double a_us = 0;  // the job's own duration on the worker
  double ph_us[4] = {0, 0, 0, 0};  // the last detection's phases (image staged, GPU classes back, FLD), us
  // rspl_lines_extract_wait_device: the worker's lines staged in pinned memory and copied to the device in
  // stream order, through a ring of kPinSlots buffers: a slot is rewritten only once its copy of
  // kPinSlots joins ago has completed (copy_ev), so a join never waits for the stream in practice
  static constexpr int kPinSlots = 4;
  double* pin_lines[kPinSlots] = {};
  int pin_cap = 0;  // lines per slot
  hipEvent_t copy_ev[kPinSlots] = {};
  bool copy_pending[kPinSlots] = {};
  int pin_next = 0;
  rspl_fld_config a_cfg{};
  std::vector<float> a_seg;
  std::vector<double> a_lines;
  std::string a_err;
};

extern "C" int rspl_lines_create(const rspl_lines_config* cfg, rspl_lines** out) {
  RSPL_CHECK_ARG(cfg && out, "rspl_lines_create: NULL argument");
  RSPL_CHECK_ARG(cfg->max_lines > 0 && cfg->max_lines <= 1024, "max_lines must be in [1, 1024]");
  RSPL_CHECK_ARG(cfg->max_points > 0 && cfg->max_points <= lines::kMaxPointsLds, "max_points must be in [1, %d]",
                 lines::kMaxPointsLds);
  RSPL_CHECK_ARG(cfg->max_pairs > 0 && cfg->max_matches >= 0, "max_pairs must be > 0, max_matches >= 0");
  *out = nullptr;
  RSPL_HIP(hipSetDevice(cfg->device));
  auto* h = new rspl_lines();
  h->cfg = *cfg;
  h->cap = cfg->max_pairs;
  const size_t L = cfg->max_lines, N = cfg->max_points, C = cfg->max_pairs, Mm = std::max(1, cfg->max_matches);
  // two assignment sets (left / right, or frame 0 / frame 1) and two matching problems
  auto carve = [&](auto& ar) {
    auto take = [&](auto*& p, size_t n) {
      using T = std::remove_pointer_t<std::remove_reference_t<decltype(p)>>;
      if constexpr (std::is_same_v<std::remove_reference_t<decltype(ar)>, Arena>) p = ar.template take<T>(n);
      else ar.template take<T>(n);
    };
    take(h->lines, 2 * L * 4); take(h->pts, 2 * N * 2); take(h->dist, 2 * C);
    take(h->n_lines, 2); take(h->n_points, 2); take(h->offsets, 2 * (L + 1)); take(h->idx, 2 * C);
    take(h->status, 3); take(h->matches, 2 * Mm * 2); take(h->n_matches, 2); take(h->M, 2 * L * L);
    take(h->inv, 2 * 2 * C); take(h->out, 2 * L);
  };
  Sizer sz;
  carve(sz);
  if (int rc = h->arena.reserve(sz.used)) {
    delete h;
    return rc;
  }
  carve(h->arena);
  if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess ||
      hipMemset(h->status, 0, sizeof(int) * 3) != hipSuccess) {
    rspl_lines_destroy(h);
    set_error("stream creation failed");
    return RSPL_E_DEVICE;
  }
  *out = h;
  return RSPL_OK;
}

extern "C" void rspl_lines_destroy(rspl_lines* h) {
  if (!h) return;
  if (h->worker.joinable()) {
    {
      std::lock_guard<std::mutex> lk(h->mu);
      h->quit = true;
    }
    h->cv.notify_all();
    h->worker.join();
  }
  for (int k = 0; k < rspl_lines::kPinSlots; k++) {
    if (h->copy_ev[k]) {
      (void)hipEventSynchronize(h->copy_ev[k]);
      (void)hipEventDestroy(h->copy_ev[k]);
    }
    if (h->pin_lines[k]) (void)hipHostFree(h->pin_lines[k]);
  }
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  if (h->d_img) (void)hipFree(h->d_img);
  if (h->d_det) (void)hipFree(h->d_det);
  if (h->h_img) (void)hipHostFree(h->h_img);
  if (h->h_det) (void)hipHostFree(h->h_det);
  h->arena.release();
  if (h->stream) (void)hipStreamDestroy(h->stream);
  delete h;
}

namespace {

// one image's lines and keypoint (x, y) into assignment set `set`
int stage_image(rspl_lines* h, int set, const double* lines, int n_lines, const double* features, int n_points) {
  RSPL_CHECK_ARG(n_lines >= 0 && n_lines <= h->cfg.max_lines, "n_lines %d outside [0, %d]", n_lines, h->cfg.max_lines);
  RSPL_CHECK_ARG(n_points >= 0 && n_points <= h->cfg.max_points, "n_points %d outside [0, %d]", n_points,
                 h->cfg.max_points);
  RSPL_CHECK_ARG((n_lines == 0 || lines) && (n_points == 0 || features), "NULL lines / features");
  const size_t L = h->cfg.max_lines, N = h->cfg.max_points;
  std::vector<double> xy((size_t)2 * n_points);
  for (int j = 0; j < n_points; j++) {  // rows 1, 2 of the 259 x N column-major features
    xy[2 * j] = features[(size_t)259 * j + 1];
    xy[2 * j + 1] = features[(size_t)259 * j + 2];
  }
  const int cnt[2] = {n_lines, n_points};
  RSPL_HIP(hipMemcpyAsync(h->lines + set * L * 4, lines, sizeof(double) * 4 * n_lines, hipMemcpyHostToDevice, h->stream));
  RSPL_HIP(hipMemcpyAsync(h->pts + set * N * 2, xy.data(), sizeof(double) * xy.size(), hipMemcpyHostToDevice, h->stream));
  RSPL_HIP(hipMemcpyAsync(h->n_lines + set, &cnt[0], sizeof(int), hipMemcpyHostToDevice, h->stream));
  RSPL_HIP(hipMemcpyAsync(h->n_points + set, &cnt[1], sizeof(int), hipMemcpyHostToDevice, h->stream));
  RSPL_HIP(hipStreamSynchronize(h->stream));  // the host vectors above go out of scope
  return RSPL_OK;
}

int run_assign(rspl_lines* h, int B) {
  lines::AssignArgs a{};
  a.lines = h->lines; a.n_lines = h->n_lines; a.pts = h->pts; a.pt_batch = (size_t)h->cfg.max_points * 2;
  a.pt_stride = 2; a.pt_xoff = 0; a.n_points = h->n_points; a.offsets = h->offsets; a.idx = h->idx;
  a.dist = h->dist; a.max_lines = h->cfg.max_lines; a.cap = h->cap; a.status = h->status;
  RSPL_HIP(lines::assign(a, B, h->stream));
  int st[2] = {0, 0};
  RSPL_HIP(hipMemcpyAsync(st, h->status, sizeof(int) * B, hipMemcpyDeviceToHost, h->stream));
  RSPL_HIP(hipStreamSynchronize(h->stream));
  for (int b = 0; b < B; b++)
    if (st[b]) {
      set_error("point-line pairs exceed max_pairs %d", h->cap);
      return RSPL_E_CAPACITY;
    }
  return RSPL_OK;
}

int read_assignment(rspl_lines* h, int set, int n_lines, int* offsets, int* point_idx, double* dist, int capacity) {
  RSPL_HIP(hipMemcpy(offsets, h->offsets + (size_t)set * (h->cfg.max_lines + 1), sizeof(int) * (n_lines + 1),
                     hipMemcpyDeviceToHost));
  const int tot = offsets[n_lines];
  if (tot > capacity) {
    set_error("%d point-line pairs exceed capacity %d", tot, capacity);
    return RSPL_E_CAPACITY;
  }
  if (tot) {
    RSPL_HIP(hipMemcpy(point_idx, h->idx + (size_t)set * h->cap, sizeof(int) * tot, hipMemcpyDeviceToHost));
    RSPL_HIP(hipMemcpy(dist, h->dist + (size_t)set * h->cap, sizeof(double) * tot, hipMemcpyDeviceToHost));
  }
  return RSPL_OK;
}

int stage_assignment(rspl_lines* h, int set, const int* offsets, const int* idx, int n_lines, int n_points) {
  RSPL_CHECK_ARG(n_lines >= 0 && n_lines <= h->cfg.max_lines && n_points >= 0 && n_points <= h->cfg.max_points,
                 "assignment sizes outside the handle's limits");
  RSPL_CHECK_ARG(offsets && offsets[0] == 0, "offsets must start at 0");
  for (int l = 0; l < n_lines; l++) RSPL_CHECK_ARG(offsets[l + 1] >= offsets[l], "offsets must be non-decreasing");
  const int tot = offsets[n_lines];
  RSPL_CHECK_ARG(tot <= h->cap, "%d point-line pairs exceed max_pairs %d", tot, h->cap);
  for (int e = 0; e < tot; e++) RSPL_CHECK_ARG(idx[e] >= 0 && idx[e] < n_points, "point index %d outside [0, %d)", idx[e], n_points);
  const int cnt[2] = {n_lines, n_points};
  RSPL_HIP(hipMemcpy(h->offsets + (size_t)set * (h->cfg.max_lines + 1), offsets, sizeof(int) * (n_lines + 1),
                     hipMemcpyHostToDevice));
  if (tot) RSPL_HIP(hipMemcpy(h->idx + (size_t)set * h->cap, idx, sizeof(int) * tot, hipMemcpyHostToDevice));
  RSPL_HIP(hipMemcpy(h->n_lines + set, &cnt[0], sizeof(int), hipMemcpyHostToDevice));
  RSPL_HIP(hipMemcpy(h->n_points + set, &cnt[1], sizeof(int), hipMemcpyHostToDevice));
  return RSPL_OK;
}

int run_match(rspl_lines* h, int problem, int set0, int set1, const int* matches, int n_matches, int n_points0,
              int n_points1) {
  RSPL_CHECK_ARG(n_matches >= 0 && n_matches <= h->cfg.max_matches, "n_matches %d outside [0, %d]", n_matches,
                 h->cfg.max_matches);
  for (int m = 0; m < n_matches; m++)
    RSPL_CHECK_ARG(matches[2 * m] >= 0 && matches[2 * m] < n_points0 && matches[2 * m + 1] >= 0 &&
                       matches[2 * m + 1] < n_points1,
                   "match %d (%d, %d) outside the keypoint ranges", m, matches[2 * m], matches[2 * m + 1]);
  const size_t Mm = std::max(1, h->cfg.max_matches);
  if (n_matches)
    RSPL_HIP(hipMemcpy(h->matches + problem * Mm * 2, matches, sizeof(int) * 2 * n_matches, hipMemcpyHostToDevice));
  RSPL_HIP(hipMemcpy(h->n_matches + problem, &n_matches, sizeof(int), hipMemcpyHostToDevice));
  lines::MatchArgs a{};
  a.off0 = a.off1 = h->offsets; a.idx0 = a.idx1 = h->idx; a.n_lines0 = a.n_lines1 = h->n_lines;
  a.n_points0 = a.n_points1 = h->n_points; a.set0 = set0; a.set1 = set1; a.step0 = a.step1 = 0;
  a.matches = h->matches + problem * Mm * 2; a.n_matches = h->n_matches + problem; a.max_lines = h->cfg.max_lines;
  a.cap = h->cap; a.max_matches = (int)Mm; a.M = h->M + (size_t)problem * h->cfg.max_lines * h->cfg.max_lines;
  a.inv = h->inv + (size_t)problem * 2 * h->cap; a.out = h->out + (size_t)problem * h->cfg.max_lines;
  a.status = nullptr;  // host calls check the assignment status themselves
  RSPL_HIP(lines::match(a, 1, h->stream));
  RSPL_HIP(hipStreamSynchronize(h->stream));
  (void)n_points0;
  (void)n_points1;
  return RSPL_OK;
}

}  // namespace

extern "C" int rspl_lines_assign(rspl_lines* h, const double* lines, int n_lines, const double* features, int n_points,
                                 int* offsets, int* point_idx, double* dist, int capacity) {
  RSPL_CHECK_ARG(h && offsets && (capacity == 0 || (point_idx && dist)), "rspl_lines_assign: NULL argument");
  if (int rc = stage_image(h, 0, lines, n_lines, features, n_points)) return rc;
  if (int rc = run_assign(h, 1)) return rc;
  return read_assignment(h, 0, n_lines, offsets, point_idx, dist, capacity);
}

extern "C" int rspl_lines_match(rspl_lines* h, const int* offsets0, const int* idx0, int n_lines0, const int* offsets1,
                                const int* idx1, int n_lines1, const int* matches, int n_matches, int n_points0,
                                int n_points1, int* line_matches) {
  RSPL_CHECK_ARG(h && offsets0 && offsets1 && (n_matches == 0 || matches) && (n_lines0 == 0 || line_matches),
                 "rspl_lines_match: NULL argument");
  if (int rc = stage_assignment(h, 0, offsets0, idx0, n_lines0, n_points0)) return rc;
  if (int rc = stage_assignment(h, 1, offsets1, idx1, n_lines1, n_points1)) return rc;
  if (int rc = run_match(h, 0, 0, 1, matches, n_matches, n_points0, n_points1)) return rc;
  if (n_lines0) RSPL_HIP(hipMemcpy(line_matches, h->out, sizeof(int) * n_lines0, hipMemcpyDeviceToHost));
  return RSPL_OK;
}

extern "C" int rspl_lines_stereo(rspl_lines* h, const double* lines_left, int n_left, const double* features_left,
                                 int n_points_left, const double* lines_right, int n_right, const double* features_right,
                                 int n_points_right, const int* stereo_matches, int n_matches, const double* camera_limits,
                                 double* lines_right_out, uint8_t* lines_right_valid, int* n_kept_matches) {
  RSPL_CHECK_ARG(h && camera_limits && n_kept_matches && (n_left == 0 || (lines_right_out && lines_right_valid)),
                 "rspl_lines_stereo: NULL argument");
  RSPL_CHECK_ARG(n_matches >= 0 && (n_matches == 0 || stereo_matches), "bad stereo matches");
  // frame.cc:157-167: keep the stereo matches inside the disparity window
  const double min_x = camera_limits[0], max_x = camera_limits[1], max_y = camera_limits[2];
  std::vector<int> kept;
  kept.reserve((size_t)2 * n_matches);
  for (int m = 0; m < n_matches; m++) {
    const int q = stereo_matches[2 * m], t = stereo_matches[2 * m + 1];
    RSPL_CHECK_ARG(q >= 0 && q < n_points_left && t >= 0 && t < n_points_right, "stereo match %d out of range", m);
    const double dx = std::fabs(features_left[(size_t)259 * q + 1] - features_right[(size_t)259 * t + 1]);
    const double dy = std::fabs(features_left[(size_t)259 * q + 2] - features_right[(size_t)259 * t + 2]);
    if (dx > min_x && dx < max_x && dy <= max_y) {
      kept.push_back(q);
      kept.push_back(t);
    }
  }
  *n_kept_matches = (int)kept.size() / 2;
  // frame.cc:128, 181: both images' assignments in one launch; :188 MatchLines
  if (int rc = stage_image(h, 0, lines_left, n_left, features_left, n_points_left)) return rc;
  if (int rc = stage_image(h, 1, lines_right, n_right, features_right, n_points_right)) return rc;
  if (int rc = run_assign(h, 2)) return rc;
  if (int rc = run_match(h, 0, 0, 1, kept.data(), (int)kept.size() / 2, n_points_left, n_points_right)) return rc;
  std::vector<int> lm((size_t)n_left);
  if (n_left) RSPL_HIP(hipMemcpy(lm.data(), h->out, sizeof(int) * n_left, hipMemcpyDeviceToHost));
  // frame.cc:189-196 (a match to right line 0 counts as invalid, as in the reference)
  for (int i = 0; i < n_left; i++) {
    const bool ok = lm[i] > 0;
    lines_right_valid[i] = ok ? 1 : 0;
    for (int k = 0; k < 4; k++) lines_right_out[4 * i + k] = ok ? lines_right[4 * lm[i] + k] : 0.0;
  }
  return RSPL_OK;
}

// Device-resident form of rspl_lines_stereo for a GPU pipeline: SuperPoint's device features and
// counts (image 0 = left, 1 = right) and SuperGlue's device match index of each left keypoint go in,
// per left line the right line and its validity come out, all stream-ordered (no host copy, no
// synchronisation).  An assignment that overflows max_pairs leaves every left line unmatched;
// rspl_lines_status reports it after the stream has completed.
extern "C" int rspl_lines_stereo_device(rspl_lines* h, const double* d_lines_left, int n_left,
                                        const double* d_lines_right, int n_right, const double* d_features,
                                        int feat_cap, const int32_t* d_counts, const int32_t* d_match_idx,
                                        const double* camera_limits, double* d_lines_right_out,
                                        uint8_t* d_lines_right_valid, void* stream) {
  RSPL_CHECK_ARG(h && d_features && d_counts && d_match_idx && camera_limits && (n_left == 0 || d_lines_left) &&
                     (n_right == 0 || d_lines_right) && (n_left == 0 || (d_lines_right_out && d_lines_right_valid)),
                 "rspl_lines_stereo_device: NULL argument");
  RSPL_CHECK_ARG(n_left >= 0 && n_left <= h->cfg.max_lines && n_right >= 0 && n_right <= h->cfg.max_lines,
                 "line counts outside [0, %d]", h->cfg.max_lines);
  RSPL_CHECK_ARG(feat_cap > 0 && feat_cap <= h->cfg.max_points, "feat_cap outside [1, %d]", h->cfg.max_points);
  hipStream_t st = stream ? (hipStream_t)stream : h->stream;
  const size_t L = h->cfg.max_lines;
  if (n_left)
    RSPL_HIP(hipMemcpyAsync(h->lines, d_lines_left, sizeof(double) * 4 * n_left, hipMemcpyDeviceToDevice, st));
  if (n_right)
    RSPL_HIP(hipMemcpyAsync(h->lines + L * 4, d_lines_right, sizeof(double) * 4 * n_right, hipMemcpyDeviceToDevice, st));
  RSPL_HIP(lines::set_counts(h->n_lines, n_left, n_right, h->n_points, d_counts, h->n_matches, st));
  lines::AssignArgs a{};
  a.lines = h->lines; a.n_lines = h->n_lines; a.pts = d_features; a.pt_batch = (size_t)feat_cap * 259;
  a.pt_stride = 259; a.pt_xoff = 1; a.n_points = h->n_points; a.offsets = h->offsets; a.idx = h->idx;
  a.dist = h->dist; a.max_lines = h->cfg.max_lines; a.cap = h->cap; a.status = h->status;
  RSPL_HIP(lines::assign(a, 2, st));
  lines::StereoArgs sa{};
  sa.idx = d_match_idx; sa.n_points = h->n_points; sa.pts = d_features; sa.pt_batch = (size_t)feat_cap * 259;
  sa.stride = 259; sa.xoff = 1; sa.min_x = camera_limits[0]; sa.max_x = camera_limits[1]; sa.max_y = camera_limits[2];
  sa.matches = h->matches; sa.n_out = h->n_matches; sa.status = h->status + 2;
  sa.max_matches = std::max(1, h->cfg.max_matches);
  RSPL_HIP(lines::stereo_filter(sa, feat_cap, st));
  lines::MatchArgs m{};
  m.off0 = m.off1 = h->offsets; m.idx0 = m.idx1 = h->idx; m.n_lines0 = m.n_lines1 = h->n_lines;
  m.n_points0 = m.n_points1 = h->n_points; m.set0 = 0; m.set1 = 1; m.step0 = m.step1 = 0;
  m.matches = h->matches; m.n_matches = h->n_matches; m.max_lines = h->cfg.max_lines; m.cap = h->cap;
  m.max_matches = std::max(1, h->cfg.max_matches); m.M = h->M; m.inv = h->inv; m.out = h->out; m.status = h->status;
  RSPL_HIP(lines::match(m, 1, st));
  lines::RightArgs r{};
  r.line_matches = h->out; r.lines_right = h->lines + L * 4; r.n_lines = h->n_lines; r.out = d_lines_right_out;
  r.valid = d_lines_right_valid;
  RSPL_HIP(lines::right_lines(r, std::max(1, n_left), st));
  return RSPL_OK;
}

extern "C" int rspl_lines_status(rspl_lines* h, int* overflow) {
  RSPL_CHECK_ARG(h && overflow, "rspl_lines_status: NULL argument");
  int st[3] = {0, 0, 0};
  RSPL_HIP(hipMemcpy(st, h->status, sizeof(st), hipMemcpyDeviceToHost));
  *overflow = st[0] | st[1] | st[2];
  return RSPL_OK;
}

// ---------------------------------------------------------------------------------------------
// LineDetector's detector: cv::resize(0.5, INTER_LINEAR) + fld->detect (line_processor.cc:455-466,
// FastLineDetector with do_merge false), restated as oracle/fld_ref.py.  The pixel-parallel front
// (resize, Sobel, Canny's non-maximum suppression and thresholds) runs on the GPU
// (line_kernels.hip canny_kernel); the order-dependent rest runs here on the host, exactly as the
// restatement orders it: 8-connected hysteresis, the corner zeroing, chains from raster-order seeds
// (getPointChain), straight runs (extractSegments, cv::fitLine DIST_L2 refits), the length and
// border filters in float, and the brighter-side-left orientation.  Double / float types and
// operation order follow the restatement (FP contraction is off in this file): bit-exact with it.
// ---------------------------------------------------------------------------------------------
namespace {

struct FSeg {
  float x1, y1, x2, y2;
};
struct HLine {
  double a, b, c;
};

HLine line_through(double px, double py, double qx, double qy) {
  const double a = py - qy, b = qx - px, c = px * qy - py * qx;
  const double n = std::sqrt(a * a + b * b);
  return {a / n, b / n, c / n};
}

HLine fit_line(const std::vector<std::pair<int, int>>& pts, size_t n) {  // the first n points
  double sx = 0, sy = 0, sxx = 0, syy = 0, sxy = 0;
  for (size_t k = 0; k < n; k++) {
    const double x = pts[k].first, y = pts[k].second;
    sx += x;
    sy += y;
    sxx += (double)((long long)pts[k].first * pts[k].first);
    syy += (double)((long long)pts[k].second * pts[k].second);
    sxy += (double)((long long)pts[k].first * pts[k].second);
  }
  const double cnt = (double)n, cx = sx / cnt, cy = sy / cnt;
  const double dxx = sxx / cnt - cx * cx, dyy = syy / cnt - cy * cy, dxy = sxy / cnt - cx * cy;
  const double t = std::atan2(2.0 * dxy, dxx - dyy) / 2.0;
  const double vx = std::cos(t), vy = std::sin(t);
  return line_through(cx, cy, cx + vx, cy + vy);
}

inline double ldist(const HLine& l, double x, double y) { return std::fabs(l.a * x + l.b * y + l.c); }

void extract_segments(const std::vector<std::pair<int, int>>& pts, int len_thr, double dist_thr,
                      std::vector<std::array<double, 4>>& out) {
  const int total = (int)pts.size();
  std::vector<std::pair<int, int>> run;
  int i = 0;
  while (i + len_thr < total) {
    const auto ps = pts[i], pe = pts[i + len_thr];
    HLine l = line_through(ps.first, ps.second, pe.first, pe.second);
    bool is_line = true;
    for (int j = 1; j < len_thr && is_line; j++) is_line = ldist(l, pts[i + j].first, pts[i + j].second) <= dist_thr;
    if (!is_line) {
      i++;
      continue;
    }
    run.assign(pts.begin() + i, pts.begin() + i + len_thr + 1);
    l = fit_line(run, run.size());
    int j = i + len_thr + 1;
    for (; j < total; j++) {
      const double x = pts[j].first, y = pts[j].second;
      if (ldist(l, x, y) > dist_thr) {
        l = fit_line(run, run.size());
        if (ldist(l, x, y) > dist_thr) break;
      }
      run.push_back(pts[j]);
    }
    l = fit_line(run, run.size());
    auto proj = [&](const std::pair<int, int>& p, double& ox, double& oy) {
      const double d = l.a * p.first + l.b * p.second + l.c;
      ox = p.first - d * l.a;
      oy = p.second - d * l.b;
    };
    std::array<double, 4> sg;
    proj(run.front(), sg[0], sg[1]);
    proj(run.back(), sg[2], sg[3]);
    out.push_back(sg);
    i = j;
  }
}

// brighter side on the left: intensity difference at +-1.5 px along the normal, one sample per pixel
FSeg orient(const uint8_t* img, int h, int w, FSeg s) {
  const double x1 = s.x1, y1 = s.y1, x2 = s.x2, y2 = s.y2;
  const double dx = x2 - x1, dy = y2 - y1;
  const double L = std::sqrt(dx * dx + dy * dy);
  const double nx = -dy / L, ny = dx / L;
  const int n = std::max(1, (int)L);
  long long acc = 0;
  for (int k = 0; k < n; k++) {
    const double t = (k + 0.5) / n;
    const double px = x1 + t * dx, py = y1 + t * dy;
    const int lx = (int)std::floor(px + 1.5 * nx + 0.5), ly = (int)std::floor(py + 1.5 * ny + 0.5);
    const int rx = (int)std::floor(px - 1.5 * nx + 0.5), ry = (int)std::floor(py - 1.5 * ny + 0.5);
    if (lx >= 0 && lx < w && ly >= 0 && ly < h && rx >= 0 && rx < w && ry >= 0 && ry < h)
      acc += (int)img[(size_t)ly * w + lx] - (int)img[(size_t)ry * w + rx];
  }
  if (acc < 0) return {s.x2, s.y2, s.x1, s.y1};
  return s;
}

// getPointChain: neighbour index order (dr, dc); step 0 takes the first edge neighbour, later
// steps the most direction-consistent one (ties to the later index) if within 2
const int kNb[8][2] = {{1, 1}, {1, 0}, {1, -1}, {0, -1}, {-1, -1}, {-1, 0}, {-1, 1}, {0, 1}};
bool chain_step(const uint8_t* e, int h, int w, int& x, int& y, int& direction, int step) {
  float best = 7.0f;
  int bx = 0, by = 0, bd = 0;
  bool found = false;
  for (int i = 0; i < 8; i++) {
    const int ci = x + kNb[i][1], ri = y + kNb[i][0];
    if (ri < 0 || ri == h || ci < 0 || ci == w || e[(size_t)ri * w + ci] == 0) continue;
    const int d = i > 4 ? i - 8 : i;
    if (step == 0) {
      x = ci;
      y = ri;
      direction = d;
      return true;
    }
    float diff = std::fabs((float)d - (float)direction);
    diff = diff > 4.0f ? 8.0f - diff : diff;
    if (diff <= best) {
      best = diff;
      bx = ci;
      by = ri;
      bd = d;
      found = true;
    }
  }
  if (found && best < 2.0f) {
    x = bx;
    y = by;
    direction = bd;
    return true;
  }
  return false;
}

// the host part of the detector from the GPU's half image and Canny classes: hysteresis, the
// corner zeroing, chains, runs, filters, orientation; returns the segment count (written up to
// capacity)
int fld_from_classes(const uint8_t* half, const uint8_t* cls, int hh, int hw, const rspl_fld_config* cfg,
                     std::vector<uint8_t>& e, std::vector<int>& stk, float* segments, int capacity) {
  const size_t hp = (size_t)hh * hw;
  // hysteresis: strong pixels through 8-connected candidates (the edge set does not depend on order)
  e.assign(hp, 0);
  stk.clear();
  for (size_t i = 0; i < hp; i++)
    if (cls[i] == 2) {
      e[i] = 255;
      stk.push_back((int)i);
    }
  while (!stk.empty()) {
    const int i = stk.back();
    stk.pop_back();
    const int r = i / hw, c = i - r * hw;
    for (int dr = -1; dr <= 1; dr++)
      for (int dc = -1; dc <= 1; dc++) {
        const int rr = r + dr, cc = c + dc;
        if (rr < 0 || rr >= hh || cc < 0 || cc >= hw) continue;
        const size_t k = (size_t)rr * hw + cc;
        if (cls[k] == 0 && e[k] == 0) {
          e[k] = 255;
          stk.push_back((int)k);
        }
      }
  }
  // the corner zeroing of OpenCV's lineDetection (top-left 6 x 6, bottom-right 5 x 5)
  for (int r = 0; r < std::min(6, hh); r++)
    for (int c = 0; c < std::min(6, hw); c++) e[(size_t)r * hw + c] = 0;
  for (int r = std::max(hh - 5, 0); r < hh; r++)
    for (int c = std::max(hw - 5, 0); c < hw; c++) e[(size_t)r * hw + c] = 0;
  const int lt = cfg->length_threshold;
  const double dt = cfg->distance_threshold;
  std::vector<std::pair<int, int>> pts;
  std::vector<std::array<double, 4>> segs;
  int n = 0;
  for (int r = 0; r < hh; r++)
    for (int c = 0; c < hw; c++) {
      if (e[(size_t)r * hw + c] == 0) continue;
      pts.clear();
      pts.emplace_back(c, r);
      e[(size_t)r * hw + c] = 0;
      int x = c, y = r, direction = 0, step = 0;
      while (chain_step(e.data(), hh, hw, x, y, direction, step)) {
        pts.emplace_back(x, y);
        step++;
        e[(size_t)y * hw + x] = 0;
      }
      if ((int)pts.size() < lt + 1) continue;
      segs.clear();
      extract_segments(pts, lt, dt, segs);
      for (const auto& sg : segs) {
        const FSeg s{(float)sg[0], (float)sg[1], (float)sg[2], (float)sg[3]};
        const float ddx = s.x1 - s.x2, ddy = s.y1 - s.y2;
        const float length = std::sqrt(ddx * ddx + ddy * ddy);
        if (length < (float)lt) continue;
        if ((s.x1 <= 5.0f && s.x2 <= 5.0f) || (s.y1 <= 5.0f && s.y2 <= 5.0f) ||
            (s.x1 >= hw - 5.0f && s.x2 >= hw - 5.0f) || (s.y1 >= hh - 5.0f && s.y2 >= hh - 5.0f))
          continue;
        const FSeg o = orient(half, hh, hw, s);
        if (n < capacity) {
          segments[4 * n + 0] = o.x1;
          segments[4 * n + 1] = o.y1;
          segments[4 * n + 2] = o.x2;
          segments[4 * n + 3] = o.y2;
        }
        n++;
      }
    }
  return n;
}

}  // namespace

extern "C" int rspl_lines_detect(rspl_lines* h, const uint8_t* image, int H, int W, int stride,
                                 const rspl_fld_config* cfg, float* segments, int capacity, int* n_out) {
  RSPL_CHECK_ARG(h && image && cfg && n_out && (segments || capacity == 0), "rspl_lines_detect: NULL argument");
  RSPL_CHECK_ARG(H >= 4 && W >= 4 && H % 2 == 0 && W % 2 == 0 && stride >= W,
                 "image %dx%d (stride %d): even sizes >= 4 required", W, H, stride);
  RSPL_CHECK_ARG(cfg->canny_aperture_size == 3, "canny_aperture_size %d: only 3 (the configs' value)",
                 cfg->canny_aperture_size);
  RSPL_CHECK_ARG(cfg->length_threshold >= 1 && cfg->distance_threshold >= 0, "bad FLD thresholds");
  *n_out = 0;
  const size_t px = (size_t)H * W, hp = px / 4;
  const int hh = H / 2, hw = W / 2;
  if (px > h->det_cap) {  // grow the detector buffers (the stream is idle between calls)
    RSPL_HIP(hipStreamSynchronize(h->stream));
    if (h->d_img) (void)hipFree(h->d_img);
    if (h->d_det) (void)hipFree(h->d_det);
    if (h->h_img) (void)hipHostFree(h->h_img);
    if (h->h_det) (void)hipHostFree(h->h_det);
    h->d_img = h->d_det = h->h_img = h->h_det = nullptr;
    h->det_cap = 0;
    RSPL_HIP(hipMalloc((void**)&h->d_img, px));
    RSPL_HIP(hipMalloc((void**)&h->d_det, 2 * (px / 4)));
    RSPL_HIP(hipHostMalloc((void**)&h->h_img, px));
    RSPL_HIP(hipHostMalloc((void**)&h->h_det, 2 * (px / 4)));
    h->det_cap = px;
  }
  const auto tp0 = std::chrono::steady_clock::now();
  for (int r = 0; r < H; r++) memcpy(h->h_img + (size_t)r * W, image + (size_t)r * stride, W);
  const auto tp1 = std::chrono::steady_clock::now();
  hipStream_t st = h->stream;
  RSPL_HIP(hipMemcpyAsync(h->d_img, h->h_img, px, hipMemcpyHostToDevice, st));
  double lo = cfg->canny_th1, hi = cfg->canny_th2;
  if (lo > hi) std::swap(lo, hi);
  lines::CannyArgs a{};
  a.img = h->d_img; a.H = H; a.W = W; a.stride = W;
  a.half = h->d_det; a.cls = h->d_det + hp;
  a.low = (int)std::floor(lo); a.high = (int)std::floor(hi);
  RSPL_HIP(lines::canny_classes(a, st));
  RSPL_HIP(hipMemcpyAsync(h->h_det, h->d_det, 2 * hp, hipMemcpyDeviceToHost, st));
  RSPL_HIP(hipStreamSynchronize(st));
  const auto tp2 = std::chrono::steady_clock::now();
  h->det_H = H;
  h->det_W = W;
  const int n = fld_from_classes(h->h_det, h->h_det + hp, hh, hw, cfg, h->edge, h->stack, segments, capacity);
  const auto tp3 = std::chrono::steady_clock::now();
  auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
  h->ph_us[0] = us(tp0, tp1);
  h->ph_us[1] = us(tp1, tp2);
  h->ph_us[2] = us(tp2, tp3);
  *n_out = n;
  if (n > capacity) {
    set_error("%d segments exceed capacity %d", n, capacity);
    return RSPL_E_CAPACITY;
  }
  return RSPL_OK;
}

extern "C" int rspl_lines_debug_canny(rspl_lines* h, int H, int W, uint8_t* half, uint8_t* cls) {
  RSPL_CHECK_ARG(h && half && cls, "rspl_lines_debug_canny: NULL argument");
  RSPL_CHECK_ARG(H == h->det_H && W == h->det_W && H > 0,
                 "rspl_lines_debug_canny: %dx%d is not the last detection's size (%dx%d)", W, H, h->det_W, h->det_H);
  const size_t hp = (size_t)H * W / 4;
  memcpy(half, h->h_det, hp);
  memcpy(cls, h->h_det + hp, hp);
  return RSPL_OK;
}


namespace {

// the worker's job: rspl_lines_detect into a growing segment buffer, then rspl_line_extract
void extract_job(rspl_lines* h) {
  const auto t0 = std::chrono::steady_clock::now();
  int n = 0, rc;
  for (;;) {
    if (h->a_seg.size() < 4096) h->a_seg.resize(4096 * 4);
    const int cap = (int)(h->a_seg.size() / 4);
    rc = rspl_lines_detect(h, h->a_img, h->a_H, h->a_W, h->a_stride, &h->a_cfg, h->a_seg.data(), cap, &n);
    if (rc != RSPL_E_CAPACITY || n <= cap) break;
    h->a_seg.resize((size_t)n * 4);
  }
  h->a_n = 0;
  if (rc == RSPL_OK) {
    h->a_lines.resize((size_t)std::max(n, 1) * 4);  // the merges never add lines
    rc = rspl_line_extract(h->a_seg.data(), n, h->a_merge, h->a_lines.data(), std::max(n, 1), &h->a_n);
  }
  h->a_rc = rc;
  h->a_err = rc == RSPL_OK ? std::string() : std::string(rspl_last_error());
  h->a_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
  static const bool timing = getenv("RSPL_LINES_TIMING") != nullptr;  // diagnostics
  if (timing)
    fprintf(stderr, "lines_job us: stage %.1f gpu %.1f fld %.1f merge+rest %.1f total %.1f segs %d lines %d\n", h->ph_us[0],
            h->ph_us[1], h->ph_us[2], h->a_us - h->ph_us[0] - h->ph_us[1] - h->ph_us[2], h->a_us, n, h->a_n);
}

}  // namespace

extern "C" int rspl_lines_extract_async(rspl_lines* h, const uint8_t* image, int H, int W, int stride,
                                        const rspl_fld_config* cfg, int do_merge) {
  RSPL_CHECK_ARG(h && image && cfg, "rspl_lines_extract_async: NULL argument");
  {
    std::lock_guard<std::mutex> lk(h->mu);
    RSPL_CHECK_ARG(!h->job, "rspl_lines_extract_async: the previous job has not been waited for");
    h->a_img = image;
    h->a_H = H;
    h->a_W = W;
    h->a_stride = stride;
    h->a_cfg = *cfg;
    h->a_merge = do_merge;
    h->job = true;
    h->done = false;
  }
  if (!h->worker.joinable()) {
    const int dev = h->cfg.device;
    h->worker = std::thread([h, dev]() {
      (void)hipSetDevice(dev);  // the HIP device is per thread
      std::unique_lock<std::mutex> lk(h->mu);
      for (;;) {
        h->cv.wait(lk, [h] { return h->quit || (h->job && !h->done); });
        if (h->quit) return;
        lk.unlock();
        extract_job(h);
        lk.lock();
        h->done = true;
        h->cv.notify_all();
      }
    });
  }
  h->cv.notify_all();
  return RSPL_OK;
}

extern "C" int rspl_lines_extract_wait(rspl_lines* h, double* lines, int capacity, int* n_out, double* job_us) {
  RSPL_CHECK_ARG(h && n_out && (capacity == 0 || lines) && capacity >= 0, "rspl_lines_extract_wait: bad argument");
  std::unique_lock<std::mutex> lk(h->mu);
  RSPL_CHECK_ARG(h->job, "rspl_lines_extract_wait: no job submitted");
  h->cv.wait(lk, [h] { return h->done; });
  h->job = false;
  *n_out = h->a_n;
  if (job_us) *job_us = h->a_us;
  if (h->a_rc != RSPL_OK) {
    set_error("%s", h->a_err.c_str());
    return h->a_rc;
  }
  if (h->a_n > capacity) {
    set_error("%d lines exceed capacity %d", h->a_n, capacity);
    return RSPL_E_CAPACITY;
  }
  if (h->a_n) memcpy(lines, h->a_lines.data(), sizeof(double) * 4 * h->a_n);
  return RSPL_OK;
}

extern "C" int rspl_lines_extract_wait_device(rspl_lines* h, double* d_lines, int capacity, int* n_out,
                                              double* job_us, void* stream) {
  RSPL_CHECK_ARG(h && n_out && (capacity == 0 || d_lines) && capacity >= 0,
                 "rspl_lines_extract_wait_device: bad argument");
  constexpr int S = rspl_lines::kPinSlots;
  if (h->pin_cap < capacity) {  // grow every slot (their pending copies drained first)
    for (int k = 0; k < S; k++) {
      if (h->copy_pending[k]) RSPL_HIP(hipEventSynchronize(h->copy_ev[k]));
      h->copy_pending[k] = false;
      if (h->pin_lines[k]) (void)hipHostFree(h->pin_lines[k]);
      h->pin_lines[k] = nullptr;
    }
    h->pin_cap = 0;
    for (int k = 0; k < S; k++)
      RSPL_HIP(hipHostMalloc((void**)&h->pin_lines[k], sizeof(double) * 4 * capacity, hipHostMallocDefault));
    h->pin_cap = capacity;
  }
  const int k = h->pin_next;
  if (!h->copy_ev[k]) RSPL_HIP(hipEventCreateWithFlags(&h->copy_ev[k], hipEventDisableTiming));
  if (h->copy_pending[k]) {  // this slot's copy S joins ago
    RSPL_HIP(hipEventSynchronize(h->copy_ev[k]));
    h->copy_pending[k] = false;
  }
  int rc = rspl_lines_extract_wait(h, h->pin_lines[k], capacity, n_out, job_us);
  if (rc != RSPL_OK) return rc;
  if (*n_out) {
    RSPL_HIP(hipMemcpyAsync(d_lines, h->pin_lines[k], sizeof(double) * 4 * *n_out, hipMemcpyHostToDevice,
                            (hipStream_t)stream));
    RSPL_HIP(hipEventRecord(h->copy_ev[k], (hipStream_t)stream));
    h->copy_pending[k] = true;
    h->pin_next = (k + 1) % S;
  }
  return RSPL_OK;
}
