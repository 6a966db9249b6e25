// Tracking pose optimisation handle: C ABI (include/rspl.h, rspl_frame_*) over frame_kernels.hip.
// Mirrors FrameOptimization (src/g2o_optimization/g2o_optimization.cc:256-398).  A call packs
// a batch of frames -- each one pose, its fixed map points and unary constraints -- into one
// pinned staging buffer (points resolved into the edge records, so the device never chases
// ids), uploads it with one async copy, runs ONE kernel (a wavefront per frame) that writes
// the poses and inlier flags straight into host-mapped memory, and synchronises once.
#include <algorithm>
#include <cmath>
#include <cstring>

#include "common.hpp"
#include "frame_kernels.hpp"

using namespace rspl;

struct rspl_frame {
  rspl_frame_config cfg{};
  hipStream_t stream = nullptr;
  Arena arena;
  // device: upload region (descriptors | edges | inlier-in, laid out per call like the
  // staging buffer), error / level / inlier scratch
  char* up = nullptr;
  uint8_t *level = nullptr, *inl = nullptr;
  double* err = nullptr;
  // pinned upload staging (descs | edges | inlier-in), mirrors the device layout
  char* stage = nullptr;      // pinned, host-mapped staging of the upload region
  char* stage_dev = nullptr;  // its device pointer (the upload kernel reads it)
  // host-mapped results
  frame::Out* out = nullptr;
  frame::Out* out_dev = nullptr;
  uint8_t* inl_out = nullptr;
  uint8_t* inl_out_dev = nullptr;
};

namespace {

struct Q {  // SE3Quat (w x y z, t), host side
  double q[4], t[3];
};

void q_to_R(const double* q, double* R) {
  const double w = q[0], x = q[1], y = q[2], z = q[3];
  const double tx = 2 * x, ty = 2 * y, tz = 2 * z;
  const double twx = tx * w, twy = ty * w, twz = tz * w, txx = tx * x, txy = ty * x, txz = tz * x;
  const double tyy = ty * y, tyz = tz * y, tzz = tz * z;
  R[0] = 1 - (tyy + tzz); R[1] = txy - twz;       R[2] = txz + twy;
  R[3] = txy + twz;       R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
  R[6] = txz - twy;       R[7] = tyz + twx;       R[8] = 1 - (txx + tyy);
}

void normalize(Q& T) {  // SE3Quat::normalizeRotation
  if (T.q[0] < 0)
    for (double& v : T.q) v = -v;
  const double n = std::sqrt(T.q[0] * T.q[0] + T.q[1] * T.q[1] + T.q[2] * T.q[2] + T.q[3] * T.q[3]);
  for (double& v : T.q) v /= n;
}

Q inverse(const Q& T) {  // SE3Quat::inverse
  Q r;
  r.q[0] = T.q[0]; r.q[1] = -T.q[1]; r.q[2] = -T.q[2]; r.q[3] = -T.q[3];
  double R[9];
  q_to_R(r.q, R);
  for (int i = 0; i < 3; i++) r.t[i] = -(R[3 * i] * T.t[0] + R[3 * i + 1] * T.t[1] + R[3 * i + 2] * T.t[2]);
  normalize(r);
  return r;
}

inline size_t al256(size_t x) { return (x + 255) & ~size_t(255); }

struct Layout {  // staging == device upload region
  size_t desc, edges, inl, bytes;
  Layout(int B, int E) {
    desc = 0;
    edges = al256(sizeof(frame::Desc) * B);
    inl = edges + al256(sizeof(frame::Edge) * (size_t)E);
    bytes = inl + al256(E);
  }
};

}  // namespace

extern "C" int rspl_frame_create(const rspl_frame_config* cfg, rspl_frame** out) {
  RSPL_CHECK_ARG(cfg && out, "rspl_frame_create: NULL argument");
  RSPL_CHECK_ARG(cfg->max_batch > 0 && cfg->max_edges >= 0 && cfg->max_points >= 0, "bad capacities");
  *out = nullptr;
  RSPL_HIP(hipSetDevice(cfg->device));
  auto* h = new rspl_frame();
  h->cfg = *cfg;
  const int B = cfg->max_batch, E = std::max(cfg->max_edges, 1);
  const Layout lay(B, E);
  const size_t scratch = al256(sizeof(double) * 4 * (size_t)E) + 2 * al256(E);
  int rc = h->arena.reserve(lay.bytes + scratch + 1024);
  if (rc) {
    delete h;
    return rc;
  }
  // the upload region first (one copy lands descs, edges and inlier flags), then scratch
  h->up = h->arena.take<char>(lay.bytes);
  h->err = h->arena.take<double>(4 * (size_t)E);
  h->level = h->arena.take<uint8_t>(E);
  h->inl = h->arena.take<uint8_t>(E);
  if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess ||
      hipHostMalloc((void**)&h->stage, lay.bytes, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
      hipHostGetDevicePointer((void**)&h->stage_dev, h->stage, 0) != hipSuccess ||
      hipHostMalloc((void**)&h->out, sizeof(frame::Out) * B, hipHostMallocMapped | hipHostMallocCoherent) !=
          hipSuccess ||
      hipHostGetDevicePointer((void**)&h->out_dev, h->out, 0) != hipSuccess ||
      hipHostMalloc((void**)&h->inl_out, E, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
      hipHostGetDevicePointer((void**)&h->inl_out_dev, h->inl_out, 0) != hipSuccess) {
    set_error("rspl_frame_create: stream / pinned allocation failed");
    rspl_frame_destroy(h);
    return RSPL_E_DEVICE;
  }
  *out = h;
  return RSPL_OK;
}

extern "C" void rspl_frame_destroy(rspl_frame* h) {
  if (!h) return;
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  h->arena.release();
  if (h->stage) (void)hipHostFree(h->stage);
  if (h->out) (void)hipHostFree(h->out);
  if (h->inl_out) (void)hipHostFree(h->inl_out);
  if (h->stream) (void)hipStreamDestroy(h->stream);
  delete h;
}

extern "C" int rspl_frame_optimize(rspl_frame* h, const rspl_frame_problem* probs, int batch,
                                   rspl_frame_result* res) {
  RSPL_CHECK_ARG(h && (batch == 0 || (probs && res)), "rspl_frame_optimize: NULL argument");
  RSPL_CHECK_ARG(batch >= 0 && batch <= h->cfg.max_batch, "batch %d exceeds max_batch %d", batch, h->cfg.max_batch);
  if (batch == 0) return RSPL_OK;
  size_t E = 0, NP = 0;
  for (int b = 0; b < batch; b++) {
    const rspl_frame_problem& p = probs[b];
    RSPL_CHECK_ARG(p.n_mono >= 0 && p.n_stereo >= 0 && p.n_points >= 0, "frame %d: negative sizes", b);
    RSPL_CHECK_ARG(p.n_cameras >= 1 && p.cameras, "frame %d: at least one camera required", b);
    RSPL_CHECK_ARG((p.n_mono == 0 || (p.mono_point && p.mono_obs)) &&
                       (p.n_stereo == 0 || (p.stereo_point && p.stereo_obs)) && (p.n_points == 0 || p.points),
                   "frame %d: NULL edge / point arrays", b);
    E += (size_t)p.n_mono + p.n_stereo;
    NP += p.n_points;
  }
  RSPL_CHECK_ARG(E <= (size_t)h->cfg.max_edges && NP <= (size_t)h->cfg.max_points,
                 "batch holds %zu edges / %zu points, capacity %d / %d", E, NP, h->cfg.max_edges, h->cfg.max_points);
  const Layout lay(batch, (int)std::max<size_t>(E, 1));
  char* sg = h->stage;
  auto* D = reinterpret_cast<frame::Desc*>(sg + lay.desc);
  auto* ed = reinterpret_cast<frame::Edge*>(sg + lay.edges);
  auto* inl = reinterpret_cast<uint8_t*>(sg + lay.inl);
  size_t e = 0;
  int max_n = 0;
  for (int b = 0; b < batch; b++) {
    const rspl_frame_problem& p = probs[b];
    frame::Desc& d = D[b];
    memset(&d, 0, sizeof(d));
    d.e0 = (int)e;
    d.n = p.n_mono + p.n_stereo;
    max_n = std::max(max_n, d.n);
    // VertexSE3Expmap estimate = SE3Quat(q, p).inverse() (:265)
    Q Twc;
    Twc.q[0] = p.pose_q[3]; Twc.q[1] = p.pose_q[0]; Twc.q[2] = p.pose_q[1]; Twc.q[3] = p.pose_q[2];
    for (int k = 0; k < 3; k++) Twc.t[k] = p.pose_p[k];
    normalize(Twc);
    const Q Tcw = inverse(Twc);
    for (int k = 0; k < 4; k++) d.T0[k] = Tcw.q[k];
    for (int k = 0; k < 3; k++) d.T0[4 + k] = Tcw.t[k];
    // const float deltaMonoPoint = sqrt(cfg.mono_point) (:279-280)
    d.delta[0] = (double)(float)std::sqrt(p.th_mono_point);
    d.delta[1] = (double)(float)std::sqrt(p.th_stereo_point);
    d.th[0] = p.th_mono_point;
    d.th[1] = p.th_stereo_point;
    for (int s = 0; s < 2; s++) {
      const int n = s ? p.n_stereo : p.n_mono;
      const int32_t* pid = s ? p.stereo_point : p.mono_point;
      const int32_t* cid = s ? p.stereo_camera : p.mono_camera;
      const double* obs = s ? p.stereo_obs : p.mono_obs;
      const uint8_t* in = s ? p.stereo_inlier_in : p.mono_inlier_in;
      for (int i = 0; i < n; i++, e++) {
        const int q = pid[i], c = cid ? cid[i] : 0;
        RSPL_CHECK_ARG(q >= 0 && q < p.n_points && c >= 0 && c < p.n_cameras,
                       "frame %d: constraint %d references a missing point / camera", b, i);
        frame::Edge& E1 = ed[e];
        for (int k = 0; k < 3; k++) E1.X[k] = p.points[3 * q + k];
        E1.obs[0] = obs[(s ? 3 : 2) * i];
        E1.obs[1] = obs[(s ? 3 : 2) * i + 1];
        E1.obs[2] = s ? obs[3 * i + 2] : 0.0;
        for (int k = 0; k < 5; k++) E1.cam[k] = p.cameras[5 * c + k];
        E1.stereo = s;
        inl[e] = in ? (in[i] != 0) : 1;
      }
    }
  }
  hipStream_t st = h->stream;
  // Frames of <= kLdsEdges edges: the kernel reads its descriptor, edges and inlier flags once, into LDS,
  // so it reads them straight from the host-mapped staging over PCIe -- no upload launch in front of it
  // (the round-5 upload kernel had put one there: 0.259 -> 0.303 ms per single frame).  Larger frames
  // re-read their edges every LM pass: they are uploaded to device memory first (one copy kernel).
  const char* src = h->stage_dev;
  if (max_n > frame::kLdsEdges) {
    RSPL_HIP(upload_mapped(h->up, h->stage_dev, lay.bytes, st));
    src = h->up;
  }
  frame::Args a{};
  a.frames = reinterpret_cast<const frame::Desc*>(src + lay.desc);
  a.edges = reinterpret_cast<const frame::Edge*>(src + lay.edges);
  a.inl_in = reinterpret_cast<const uint8_t*>(src + lay.inl);
  a.err = h->err;
  a.level = h->level;
  a.inl = h->inl;
  a.inl_out = h->inl_out_dev;
  a.out = h->out_dev;
  RSPL_HIP(frame::optimize(a, batch, max_n, st));
  RSPL_HIP(hipStreamSynchronize(st));
  for (int b = 0; b < batch; b++) {
    const frame::Out& o = h->out[b];
    rspl_frame_result& r = res[b];
    Q Tcw;
    for (int k = 0; k < 4; k++) Tcw.q[k] = o.T[k];
    for (int k = 0; k < 3; k++) Tcw.t[k] = o.T[4 + k];
    const Q Twc = inverse(Tcw);  // pose = estimate().inverse() (:394-396)
    r.pose_q[0] = Twc.q[1]; r.pose_q[1] = Twc.q[2]; r.pose_q[2] = Twc.q[3]; r.pose_q[3] = Twc.q[0];
    for (int k = 0; k < 3; k++) r.pose_p[k] = Twc.t[k];
    r.n_inliers = o.n_inliers;
    r.rounds = o.rounds;
    for (int k = 0; k < 4; k++) {
      r.iterations[k] = o.iters[k];
      r.chi2[k] = o.chi2[k];
    }
    const frame::Desc& d = D[b];
    if (r.mono_inlier) memcpy(r.mono_inlier, h->inl_out + d.e0, probs[b].n_mono);
    if (r.stereo_inlier) memcpy(r.stereo_inlier, h->inl_out + d.e0 + probs[b].n_mono, probs[b].n_stereo);
  }
  return RSPL_OK;
}
