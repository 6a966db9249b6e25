// SolvePnPWithCV handle: C ABI (include/rspl.h, rspl_pnp_*) over pnp_kernels.hip.
// Mirrors cv::solvePnPRansac as called at src/g2o_optimization/g2o_optimization.cc:438-439
// (100 iterations, 20 px, 0.99, SOLVEPNP_ITERATIVE, zero distortion: camera.cc:145-147).
// The host restates the hypothesis sampling -- cv::RNG seeded with (uint64)-1 as
// RANSACPointSetRegistrator::run does, 5 distinct indices per subset -- so every hypothesis
// is known up front and the GPU solves them side by side; one upload, one launch, one sync.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "common.hpp"
#include "pnp_kernels.hpp"

using namespace rspl;

struct rspl_pnp {
  rspl_pnp_config cfg{};
  hipStream_t stream = nullptr;
  char* dev = nullptr;   // upload region: descs | points | keypoints | subsets
  size_t dev_cap = 0;
  char* stage = nullptr; // pinned, host-mapped staging, same layout
  char* stage_dev = nullptr;  // its device pointer (the upload kernel reads it)
  size_t stage_cap = 0;
  pnp::Out* out = nullptr;
  pnp::Out* out_dev = nullptr;
  uint8_t* inl = nullptr;
  uint8_t* inl_dev = nullptr;
  double* hyp = nullptr;  // per-hypothesis poses and inlier counts (device)
  int* hcnt = nullptr;
  unsigned long long* prof = nullptr;  // RSPL_PNP_PROF: in-kernel phase stamps
  std::vector<int> last_iters;  // hypotheses per frame of the last solve
};

namespace {

inline size_t al256(size_t x) { return (x + 255) & ~size_t(255); }

struct Layout {
  size_t desc, pts, kps, sub, bytes;
  Layout(int B, size_t P, size_t S) {
    desc = 0;
    pts = al256(sizeof(pnp::Desc) * B);
    kps = pts + al256(sizeof(double) * 3 * P);
    sub = kps + al256(sizeof(double) * 2 * P);
    bytes = sub + al256(sizeof(int32_t) * 5 * S);
  }
};

// cv::RNG::next (multiply-with-carry) and RANSACPointSetRegistrator::getSubset
inline unsigned rng_next(uint64_t& s) {
  s = (uint64_t)(unsigned)s * 4164903690u + (unsigned)(s >> 32);
  return (unsigned)s;
}

void subsets(int count, int iters, int32_t* idx) {
  uint64_t s = (uint64_t)-1;
  for (int h = 0; h < iters; h++) {
    int32_t* o = idx + 5 * h;
    for (int i = 0; i < 5; i++) {
      int v;
      for (;;) {
        v = (int)(rng_next(s) % (unsigned)count);
        bool dup = false;
        for (int j = 0; j < i; j++) dup |= o[j] == v;
        if (!dup) break;
      }
      o[i] = v;
    }
  }
}

}  // namespace

extern "C" int rspl_pnp_create(const rspl_pnp_config* cfg, rspl_pnp** out) {
  RSPL_CHECK_ARG(cfg && out && cfg->max_batch > 0 && cfg->max_points >= 0, "rspl_pnp_create: bad arguments");
  *out = nullptr;
  RSPL_HIP(hipSetDevice(cfg->device));
  auto* h = new rspl_pnp();
  h->cfg = *cfg;
  const Layout lay(cfg->max_batch, std::max(cfg->max_points, 1), (size_t)cfg->max_batch * pnp::kMaxIters);
  h->dev_cap = h->stage_cap = lay.bytes;
  if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess ||
      hipMalloc((void**)&h->dev, lay.bytes) != hipSuccess ||
      hipHostMalloc((void**)&h->stage, lay.bytes, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
      hipHostGetDevicePointer((void**)&h->stage_dev, h->stage, 0) != hipSuccess ||
      hipHostMalloc((void**)&h->out, sizeof(pnp::Out) * cfg->max_batch, hipHostMallocMapped | hipHostMallocCoherent) !=
          hipSuccess ||
      hipHostGetDevicePointer((void**)&h->out_dev, h->out, 0) != hipSuccess ||
      hipHostMalloc((void**)&h->inl, std::max(cfg->max_points, 1), hipHostMallocMapped | hipHostMallocCoherent) !=
          hipSuccess ||
      hipHostGetDevicePointer((void**)&h->inl_dev, h->inl, 0) != hipSuccess ||
      hipMalloc((void**)&h->hyp, sizeof(double) * 12 * pnp::kMaxIters * cfg->max_batch) != hipSuccess ||
      hipMalloc((void**)&h->hcnt, sizeof(int) * pnp::kMaxIters * cfg->max_batch) != hipSuccess) {
    set_error("rspl_pnp_create: allocation failed");
    rspl_pnp_destroy(h);
    return RSPL_E_DEVICE;
  }
  *out = h;
  return RSPL_OK;
}

extern "C" void rspl_pnp_destroy(rspl_pnp* h) {
  if (!h) return;
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  if (h->dev) (void)hipFree(h->dev);
  if (h->stage) (void)hipHostFree(h->stage);
  if (h->out) (void)hipHostFree(h->out);
  if (h->inl) (void)hipHostFree(h->inl);
  if (h->hyp) (void)hipFree(h->hyp);
  if (h->hcnt) (void)hipFree(h->hcnt);
  if (h->prof) (void)hipFree(h->prof);
  if (h->stream) (void)hipStreamDestroy(h->stream);
  delete h;
}

extern "C" int rspl_pnp_solve(rspl_pnp* h, const rspl_pnp_problem* probs, int batch, rspl_pnp_result* res) {
  RSPL_CHECK_ARG(h && (batch == 0 || (probs && res)), "rspl_pnp_solve: NULL argument");
  RSPL_CHECK_ARG(batch >= 0 && batch <= h->cfg.max_batch, "batch %d exceeds max_batch %d", batch, h->cfg.max_batch);
  if (batch == 0) return RSPL_OK;
  size_t P = 0, S = 0;
  for (int b = 0; b < batch; b++) {
    const rspl_pnp_problem& p = probs[b];
    RSPL_CHECK_ARG(p.n >= 0 && (p.n == 0 || (p.points && p.keypoints)), "frame %d: bad correspondences", b);
    RSPL_CHECK_ARG(p.iterations >= 1 && p.iterations <= pnp::kMaxIters, "frame %d: iterations must be 1..%d", b,
                   pnp::kMaxIters);
    RSPL_CHECK_ARG(p.reprojection_error > 0 && p.confidence >= 0 && p.confidence <= 1, "frame %d: bad RANSAC params",
                   b);
    P += p.n;
    S += p.n >= 8 ? p.iterations : 0;
  }
  RSPL_CHECK_ARG(P <= (size_t)h->cfg.max_points, "batch holds %zu correspondences, capacity %d", P, h->cfg.max_points);
  const Layout lay(batch, std::max<size_t>(P, 1), std::max<size_t>(S, 1));
  char* sg = h->stage;
  auto* D = reinterpret_cast<pnp::Desc*>(sg + lay.desc);
  auto* pts = reinterpret_cast<double*>(sg + lay.pts);
  auto* kps = reinterpret_cast<double*>(sg + lay.kps);
  auto* sub = reinterpret_cast<int32_t*>(sg + lay.sub);
  size_t p0 = 0, s0 = 0;
  int max_iters = 0;
  h->last_iters.assign(batch, 0);
  for (int b = 0; b < batch; b++) {
    const rspl_pnp_problem& p = probs[b];
    pnp::Desc& d = D[b];
    d.p0 = (int)p0;
    d.n = p.n;
    d.s0 = (int)s0;
    d.iters = p.n >= 8 ? p.iterations : 0;  // < 8 correspondences: return 0 (:433)
    d.K[0] = p.fx; d.K[1] = p.fy; d.K[2] = p.cx; d.K[3] = p.cy;
    d.thr2 = p.reprojection_error * p.reprojection_error;
    d.confidence = p.confidence;
    for (int i = 0; i < 3 * p.n; i++) pts[3 * p0 + i] = (double)(float)p.points[i];      // cv::Point3f (:425)
    for (int i = 0; i < 2 * p.n; i++) kps[2 * p0 + i] = (double)(float)p.keypoints[i];   // cv::Point2f (:426)
    if (d.iters) subsets(p.n, d.iters, sub + 5 * s0);
    max_iters = std::max(max_iters, d.iters);
    h->last_iters[b] = d.iters;
    p0 += p.n;
    s0 += d.iters;
  }
  hipStream_t st = h->stream;
  RSPL_HIP(upload_mapped(h->dev, h->stage_dev, lay.bytes, st));
  pnp::Args a{};
  a.frames = reinterpret_cast<const pnp::Desc*>(h->dev + lay.desc);
  a.pts = reinterpret_cast<const double*>(h->dev + lay.pts);
  a.kps = reinterpret_cast<const double*>(h->dev + lay.kps);
  a.subsets = reinterpret_cast<const int32_t*>(h->dev + lay.sub);
  a.inl = h->inl_dev;
  a.out = h->out_dev;
  a.hyp = h->hyp;
  a.hcnt = h->hcnt;
  static const bool prof = getenv("RSPL_PNP_PROF") != nullptr;
  if (prof && !h->prof) {
    RSPL_HIP(hipMalloc((void**)&h->prof, sizeof(unsigned long long) * 16));
    RSPL_HIP(hipMemset(h->prof, 0, sizeof(unsigned long long) * 16));
  }
  a.prof = prof ? h->prof : nullptr;
  RSPL_HIP(pnp::solve(a, batch, max_iters, st));
  RSPL_HIP(hipStreamSynchronize(st));
  if (prof) {  // in-kernel phases of frame 0 (us): hypothesis 0's EPnP + count, then the acceptance / refinement
    unsigned long long t[16];
    RSPL_HIP(hipMemcpy(t, h->prof, sizeof(t), hipMemcpyDeviceToHost));
    auto us = [&](int i, int j) { return t[i] && t[j] ? ((double)t[j] - (double)t[i]) / 100.0 : -1.0; };
    fprintf(stderr,
            "pnp_prof us: ctrl %.1f bary+MtM %.1f jacobi12 %.1f L+betas %.1f gn %.1f Rt %.1f count %.1f | hyp->final %.1f "
            "accept+inl %.1f refine %.1f\n",
            us(0, 1), us(1, 2), us(2, 3), us(3, 4), us(4, 5), us(5, 6), us(6, 7), us(7, 8), us(8, 9), us(9, 10));
    RSPL_HIP(hipMemset(h->prof, 0, sizeof(unsigned long long) * 16));
  }
  for (int b = 0; b < batch; b++) {
    const pnp::Out& o = h->out[b];
    rspl_pnp_result& r = res[b];
    r.n_inliers = o.n_inliers;
    r.hypotheses = o.hyps;
    if (o.n_inliers > 0) {
      memcpy(r.Rwc, o.Rwc, sizeof(r.Rwc));
      memcpy(r.twc, o.twc, sizeof(r.twc));
    }
    if (r.inlier) memcpy(r.inlier, h->inl + D[b].p0, probs[b].n);
  }
  return RSPL_OK;
}

extern "C" int rspl_pnp_debug_hypotheses(rspl_pnp* h, int frame, int max, int32_t* counts, double* poses) {
  RSPL_CHECK_ARG(h && counts && poses && max >= 0, "rspl_pnp_debug_hypotheses: bad arguments");
  RSPL_CHECK_ARG(frame >= 0 && frame < (int)h->last_iters.size(), "frame %d not in the last batch", frame);
  const int n = std::min(max, h->last_iters[frame]);
  if (n == 0) return 0;
  RSPL_HIP(hipMemcpy(counts, h->hcnt + (size_t)frame * pnp::kMaxIters, sizeof(int32_t) * n, hipMemcpyDeviceToHost));
  RSPL_HIP(hipMemcpy(poses, h->hyp + (size_t)frame * pnp::kMaxIters * 12, sizeof(double) * 12 * n,
                     hipMemcpyDeviceToHost));
  return n;
}
