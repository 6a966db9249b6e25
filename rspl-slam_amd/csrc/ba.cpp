// Local BA handle: C ABI (include/rspl.h) over ba_kernels.hip.
// Mirrors LocalmapOptimization (src/g2o_optimization/g2o_optimization.cc:21-252):
//   optimize(10) with Huber kernels -> chi2/depth outlier levels, kernels removed ->
//   initializeOptimization(0) + optimize(5) -> inlier flags -> write back T_wc, points, lines.
// The Levenberg-Marquardt control (g2o OptimizationAlgorithmLevenberg: tau 1e-5,
// good-step factor clamp [1/3, 2/3], ni doubling, 10 trials) runs on the host; each
// trial reads back 32 bytes (chi2, scale, fail).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>
#include <numeric>
#include <vector>

#include "ba_kernels.hpp"
#include "common.hpp"

using namespace rspl;

struct rspl_ba {
  rspl_ba_config cfg{};
  hipStream_t stream = nullptr;
  Arena arena;
  int maxE = 0, maxL = 0, maxK = 0;
  // problem
  double *cams, *T, *Tb, *X, *Xb, *L, *Lb, *eobs;
  int8_t* etype;
  int *epose, *elm, *ecam;
  // linearisation
  double *err, *rho0, *Hpp_e, *bp_e, *Hll_e, *bl_e, *Hpl_e, *Y_e;
  // active structure
  int *act_edges, *pidx, *lm_off, *lm_edges, *pose_of, *ps_off, *ps_edges, *ps_lm, *pairs;
  uint8_t *lm_act, *level, *inlier;
  // system
  double *Hll, *bl, *Dinv, *Hpp, *bp, *S, *x, *partial, *out;
  int* fail;
  double* h_out = nullptr;
};

namespace {

constexpr int kMaxCams = 16;

template <typename F>
void carve(F& ar, rspl_ba* b) {
  const size_t E = b->maxE, NL = b->maxL, K = b->maxK, nq = b->cfg.max_points, nl = b->cfg.max_lines;
  auto take = [&](auto*& p, size_t n) {
    using Tp = std::remove_pointer_t<std::remove_reference_t<decltype(p)>>;
    if constexpr (std::is_same_v<F, Arena>) p = ar.template take<Tp>(n ? n : 1);
    else ar.template take<Tp>(n ? n : 1);
  };
  take(b->cams, kMaxCams * 5);
  take(b->T, K * 8); take(b->Tb, K * 8);
  take(b->X, nq * 3); take(b->Xb, nq * 3);
  take(b->L, nl * 6); take(b->Lb, nl * 6);
  take(b->eobs, E * 8); take(b->etype, E); take(b->epose, E); take(b->elm, E); take(b->ecam, E);
  take(b->err, E * 4); take(b->rho0, E); take(b->Hpp_e, E * 36); take(b->bp_e, E * 6); take(b->Hll_e, E * 16);
  take(b->bl_e, E * 4); take(b->Hpl_e, E * 24); take(b->Y_e, E * 24);
  take(b->act_edges, E); take(b->pidx, K); take(b->lm_off, NL + 1); take(b->lm_edges, E); take(b->pose_of, K);
  take(b->ps_off, K + 1); take(b->ps_edges, E); take(b->ps_lm, E); take(b->pairs, K * (K + 1));
  take(b->lm_act, NL); take(b->level, E); take(b->inlier, E);
  take(b->Hll, NL * 16); take(b->bl, NL * 4); take(b->Dinv, NL * 16); take(b->Hpp, K * 36); take(b->bp, K * 6);
  take(b->S, 36 * K * K); take(b->x, 6 * K + 4 * NL); take(b->partial, E / 256 + 2); take(b->out, 8);
  take(b->fail, 4);
}

struct Se3h {  // host SE3Quat (w x y z, t)
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

void normalize(Se3h& T) {
  if (T.q[0] < 0)
    for (double& v : T.q) v = -v;
  const double n = std::sqrt(T.q[0] * T.q[0] + T.q[1] * T.q[1] + T.q[2] * T.q[2] + T.q[3] * T.q[3]);
  for (double& v : T.q) v /= n;
}

Se3h inverse(const Se3h& T) {  // SE3Quat::inverse
  Se3h r;
  r.q[0] = T.q[0]; r.q[1] = -T.q[1]; r.q[2] = -T.q[2]; r.q[3] = -T.q[3];
  double R[9];
  q_to_R(r.q, R);
  for (int i = 0; i < 3; i++) r.t[i] = -(R[3 * i] * T.t[0] + R[3 * i + 1] * T.t[1] + R[3 * i + 2] * T.t[2]);
  normalize(r);
  return r;
}

struct Phase {
  ba::Active A{};
  int nblocks = 0;
};

int build_active(rspl_ba* b, const std::vector<int>& act, const std::vector<int>& epose, const std::vector<int>& elm,
                 const uint8_t* fixed, int np, int nL, int robust, Phase& ph) {
  std::vector<uint8_t> pact(np, 0), lact(nL, 0);
  for (int e : act) {
    pact[epose[e]] = 1;
    lact[elm[e]] = 1;
  }
  std::vector<int> pidx(np, -1), pose_of;
  for (int p = 0; p < np; p++)
    if (pact[p] && !fixed[p]) {
      pidx[p] = (int)pose_of.size();
      pose_of.push_back(p);
    }
  const int K = (int)pose_of.size();
  std::vector<int> lm_off(nL + 1, 0), lm_edges(act.size());
  for (int e : act) lm_off[elm[e] + 1]++;
  for (int g = 0; g < nL; g++) lm_off[g + 1] += lm_off[g];
  {
    std::vector<int> fill(lm_off.begin(), lm_off.end() - 1);
    for (int e : act) lm_edges[fill[elm[e]]++] = e;
  }
  std::vector<int> ps_off(K + 1, 0), ps_edges, ps_lm;
  {
    std::vector<std::vector<int>> per(K);
    for (int e : act)
      if (pidx[epose[e]] >= 0) per[pidx[epose[e]]].push_back(e);
    for (int a = 0; a < K; a++) {
      std::stable_sort(per[a].begin(), per[a].end(), [&](int x, int y) { return elm[x] < elm[y]; });
      ps_off[a + 1] = ps_off[a] + (int)per[a].size();
      for (int e : per[a]) {
        ps_edges.push_back(e);
        ps_lm.push_back(elm[e]);
      }
    }
  }
  std::vector<int> pairs;
  for (int a = 0; a < K; a++)
    for (int c = a; c < K; c++) {
      pairs.push_back(a);
      pairs.push_back(c);
    }
  auto up = [&](auto* dst, const auto& v) {
    if (!v.empty()) return hipMemcpy(dst, v.data(), v.size() * sizeof(v[0]), hipMemcpyHostToDevice) == hipSuccess;
    return true;
  };
  bool ok = up(b->act_edges, act) && up(b->pidx, pidx) && up(b->lm_off, lm_off) && up(b->lm_edges, lm_edges) &&
            up(b->pose_of, pose_of) && up(b->ps_off, ps_off) && up(b->ps_edges, ps_edges) && up(b->ps_lm, ps_lm) &&
            up(b->pairs, pairs) && up(b->lm_act, lact);
  if (!ok) {
    set_error("BA active-structure upload failed");
    return RSPL_E_DEVICE;
  }
  ba::Active& A = ph.A;
  A.edges = b->act_edges; A.Ea = (int)act.size(); A.pidx = b->pidx; A.lm_off = b->lm_off; A.lm_edges = b->lm_edges;
  A.lm_act = b->lm_act; A.pose_of = b->pose_of; A.ps_off = b->ps_off; A.ps_edges = b->ps_edges; A.ps_lm = b->ps_lm;
  A.pairs = b->pairs; A.npairs = (int)pairs.size() / 2; A.K = K; A.nL = nL; A.robust = robust;
  ph.nblocks = ba::errors_blocks(A.Ea);
  return RSPL_OK;
}

// one g2o SparseOptimizer::optimize(iters) with OptimizationAlgorithmLevenberg
int optimize(rspl_ba* b, ba::Problem& P, ba::Lin& Lr, Phase& ph, int iters, int np, int nq, int nl, double* chi2_out,
             int* done_out) {
  hipStream_t st = b->stream;
  ba::Sys S{};
  S.Hll = b->Hll; S.bl = b->bl; S.Dinv = b->Dinv; S.Hpp = b->Hpp; S.bp = b->bp; S.S = b->S; S.x = b->x;
  S.partial = b->partial; S.out = b->out; S.fail = b->fail;
  const ba::Active& A = ph.A;
  auto read_out = [&]() -> int {
    RSPL_HIP(hipMemcpyAsync(b->h_out, b->out, sizeof(double) * 4, hipMemcpyDeviceToHost, st));
    RSPL_HIP(hipStreamSynchronize(st));
    return RSPL_OK;
  };
  int rc;
  RSPL_HIP(ba::compute_errors(P, Lr, A, S, ph.nblocks, st));
  if ((rc = read_out())) return rc;
  double currentChi = b->h_out[0];
  double lambda = 0, ni = 2;
  int done = 0;
  for (int it = 0; it < iters; it++) {
    RSPL_HIP(ba::linearize(P, Lr, A, st));
    RSPL_HIP(hipMemsetAsync(b->out + 2, 0, sizeof(double), st));
    RSPL_HIP(ba::reduce_blocks(P, Lr, A, S, st));
    if (it == 0) {
      if ((rc = read_out())) return rc;
      lambda = 1e-5 * b->h_out[2];  // computeLambdaInit: tau * max diagonal
      ni = 2;
    }
    double rho = 0;
    int qmax = 0;
    do {
      RSPL_HIP(hipMemcpyAsync(b->Tb, b->T, sizeof(double) * 8 * np, hipMemcpyDeviceToDevice, st));
      RSPL_HIP(hipMemcpyAsync(b->Xb, b->X, sizeof(double) * 3 * nq, hipMemcpyDeviceToDevice, st));
      RSPL_HIP(hipMemcpyAsync(b->Lb, b->L, sizeof(double) * 6 * nl, hipMemcpyDeviceToDevice, st));
      RSPL_HIP(hipMemsetAsync(b->fail, 0, sizeof(int), st));
      RSPL_HIP(ba::schur(P, Lr, A, S, lambda, st));
      RSPL_HIP(ba::solve_update(P, Lr, A, S, lambda, st));
      if ((rc = read_out())) return rc;
      const bool ok = b->h_out[3] == 0.0;
      const double tempChi = ok ? b->h_out[0] : std::numeric_limits<double>::max();
      rho = currentChi - tempChi;
      const double scale = ok ? b->h_out[1] + 1e-3 : 1.0;
      rho /= scale;
      if (rho > 0 && std::isfinite(tempChi) && ok) {
        double alpha = 1. - std::pow(2 * rho - 1, 3);
        alpha = std::min(alpha, 2. / 3.);
        lambda *= std::max(1. / 3., alpha);
        ni = 2;
        currentChi = tempChi;
      } else {
        lambda *= ni;
        ni *= 2;
        RSPL_HIP(hipMemcpyAsync(b->T, b->Tb, sizeof(double) * 8 * np, hipMemcpyDeviceToDevice, st));
        RSPL_HIP(hipMemcpyAsync(b->X, b->Xb, sizeof(double) * 3 * nq, hipMemcpyDeviceToDevice, st));
        RSPL_HIP(hipMemcpyAsync(b->L, b->Lb, sizeof(double) * 6 * nl, hipMemcpyDeviceToDevice, st));
        if (!std::isfinite(lambda)) break;
      }
      qmax++;
    } while (rho < 0 && qmax < 10);
    done++;
    if (qmax == 10 || rho == 0 || !std::isfinite(lambda)) break;
  }
  *chi2_out = currentChi;
  *done_out = done;
  return RSPL_OK;
}

}  // namespace

extern "C" int rspl_ba_create(const rspl_ba_config* cfg, rspl_ba** out) {
  RSPL_CHECK_ARG(cfg && out, "rspl_ba_create: NULL argument");
  RSPL_CHECK_ARG(cfg->max_poses > 0 && cfg->max_poses <= 64 && cfg->max_points >= 0 && cfg->max_lines >= 0 &&
                     cfg->max_edges >= 0,
                 "capacities: 1 <= max_poses <= 64, others >= 0");
  *out = nullptr;
  RSPL_HIP(hipSetDevice(cfg->device));
  auto* b = new rspl_ba();
  b->cfg = *cfg;
  b->maxE = 4 * cfg->max_edges;
  b->maxL = cfg->max_points + cfg->max_lines;
  b->maxK = cfg->max_poses;
  Sizer sz;
  carve(sz, b);
  int rc = b->arena.reserve(sz.used);
  if (rc) { delete b; return rc; }
  carve(b->arena, b);
  if (hipStreamCreateWithFlags(&b->stream, hipStreamNonBlocking) != hipSuccess ||
      hipHostMalloc(&b->h_out, sizeof(double) * 8) != hipSuccess) {
    set_error("stream / pinned allocation failed");
    rspl_ba_destroy(b);
    return RSPL_E_DEVICE;
  }
  *out = b;
  return RSPL_OK;
}

extern "C" void rspl_ba_destroy(rspl_ba* b) {
  if (!b) return;
  if (b->stream) (void)hipStreamSynchronize(b->stream);
  b->arena.release();
  if (b->h_out) (void)hipHostFree(b->h_out);
  if (b->stream) (void)hipStreamDestroy(b->stream);
  delete b;
}

extern "C" int rspl_ba_local(rspl_ba* b, const rspl_ba_problem* pr, rspl_ba_result* res) {
  RSPL_CHECK_ARG(b && pr && res, "rspl_ba_local: NULL argument");
  const int np = pr->n_poses, nq = pr->n_points, nl = pr->n_lines;
  const int ne[4] = {pr->n_mono, pr->n_stereo, pr->n_mono_line, pr->n_stereo_line};
  RSPL_CHECK_ARG(np >= 0 && np <= b->cfg.max_poses && nq >= 0 && nq <= b->cfg.max_points && nl >= 0 &&
                     nl <= b->cfg.max_lines,
                 "problem exceeds the handle's vertex capacity");
  for (int t = 0; t < 4; t++) RSPL_CHECK_ARG(ne[t] >= 0 && ne[t] <= b->cfg.max_edges, "edge capacity exceeded");
  RSPL_CHECK_ARG(pr->n_cameras >= 1 && pr->n_cameras <= kMaxCams && pr->cameras, "1..16 cameras required");
  RSPL_CHECK_ARG(res->pose_q && res->pose_p && (res->points || !nq) && (res->lines || !nl), "NULL result arrays");
  hipStream_t st = b->stream;
  const int E = ne[0] + ne[1] + ne[2] + ne[3], nL = nq + nl;
  // ---- vertices: VertexSE3Expmap estimate = SE3Quat(q, p).inverse() (g2o_optimization.cc:42) ----
  std::vector<double> T(8 * (size_t)np);
  for (int p = 0; p < np; p++) {
    Se3h Twc;
    Twc.q[0] = pr->pose_q[4 * p + 3];
    Twc.q[1] = pr->pose_q[4 * p + 0];
    Twc.q[2] = pr->pose_q[4 * p + 1];
    Twc.q[3] = pr->pose_q[4 * p + 2];
    for (int k = 0; k < 3; k++) Twc.t[k] = pr->pose_p[3 * p + k];
    normalize(Twc);
    const Se3h Tcw = inverse(Twc);
    for (int k = 0; k < 4; k++) T[8 * p + k] = Tcw.q[k];
    for (int k = 0; k < 3; k++) T[8 * p + 4 + k] = Tcw.t[k];
    T[8 * p + 7] = 0;
  }
  // ---- edges (unified, input order) ----
  std::vector<int8_t> etype(E);
  std::vector<int> epose(E), elm(E), ecam(E);
  std::vector<double> eobs(8 * (size_t)E, 0.0);
  const int32_t* poses[4] = {pr->mono_pose, pr->stereo_pose, pr->mono_line_pose, pr->stereo_line_pose};
  const int32_t* lms[4] = {pr->mono_point, pr->stereo_point, pr->mono_line_line, pr->stereo_line_line};
  const int32_t* cams[4] = {pr->mono_camera, pr->stereo_camera, pr->mono_line_camera, pr->stereo_line_camera};
  const double* obs[4] = {pr->mono_obs, pr->stereo_obs, pr->mono_line_obs, pr->stereo_line_obs};
  const int od[4] = {2, 3, 4, 8};
  int e = 0;
  for (int t = 0; t < 4; t++)
    for (int i = 0; i < ne[t]; i++, e++) {
      RSPL_CHECK_ARG(poses[t] && lms[t] && obs[t], "NULL edge arrays");
      const int p = poses[t][i], l = lms[t][i], c = cams[t] ? cams[t][i] : 0;
      RSPL_CHECK_ARG(p >= 0 && p < np && l >= 0 && l < (t < 2 ? nq : nl) && c >= 0 && c < pr->n_cameras,
                     "edge %d of type %d references a missing vertex/camera", i, t);
      etype[e] = (int8_t)t;
      epose[e] = p;
      elm[e] = t < 2 ? l : nq + l;
      ecam[e] = c;
      for (int k = 0; k < od[t]; k++) eobs[8 * (size_t)e + k] = obs[t][(size_t)od[t] * i + k];
    }
  auto up = [&](void* dst, const void* src, size_t bytes) {
    return bytes == 0 || hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, st) == hipSuccess;
  };
  if (!(up(b->cams, pr->cameras, sizeof(double) * 5 * pr->n_cameras) && up(b->T, T.data(), sizeof(double) * T.size()) &&
        up(b->X, pr->points, sizeof(double) * 3 * nq) && up(b->L, pr->lines, sizeof(double) * 6 * nl) &&
        up(b->etype, etype.data(), E) && up(b->epose, epose.data(), 4 * (size_t)E) &&
        up(b->elm, elm.data(), 4 * (size_t)E) && up(b->ecam, ecam.data(), 4 * (size_t)E) &&
        up(b->eobs, eobs.data(), 8 * 8 * (size_t)E))) {
    set_error("BA upload failed");
    return RSPL_E_DEVICE;
  }
  RSPL_HIP(hipMemsetAsync(b->level, 0, E ? E : 1, st));
  RSPL_HIP(hipMemsetAsync(b->err, 0, sizeof(double) * 4 * (E ? E : 1), st));
  RSPL_HIP(hipStreamSynchronize(st));
  ba::Problem P{};
  P.cams = b->cams; P.T = b->T; P.X = b->X; P.L = b->L; P.np = np; P.nq = nq; P.nl = nl;
  P.etype = b->etype; P.epose = b->epose; P.elm = b->elm; P.ecam = b->ecam; P.eobs = b->eobs;
  const double th[4] = {pr->th_mono_point, pr->th_stereo_point, pr->th_mono_line, pr->th_stereo_line};
  for (int t = 0; t < 4; t++) {
    P.th[t] = th[t];
    P.delta[t] = (double)(float)std::sqrt(th[t]);  // const float thHuber = sqrt(cfg.x) (:77-78, 125-126)
  }
  ba::Lin Lr{};
  Lr.err = b->err; Lr.rho0 = b->rho0; Lr.Hpp = b->Hpp_e; Lr.bp = b->bp_e; Lr.Hll = b->Hll_e; Lr.bl = b->bl_e;
  Lr.Hpl = b->Hpl_e; Lr.Y = b->Y_e;
  int rc;
  // ---- phase 1: all edges, Huber ----
  {
    std::vector<int> act(E);
    std::iota(act.begin(), act.end(), 0);
    Phase ph;
    if ((rc = build_active(b, act, epose, elm, pr->pose_fixed, np, nL, 1, ph))) return rc;
    if ((rc = optimize(b, P, Lr, ph, pr->iterations_first, np, nq, nl, &res->chi2_first, &res->iterations_done_first)))
      return rc;
  }
  RSPL_HIP(ba::classify(P, Lr, E, b->level, nullptr, 0, st));
  std::vector<uint8_t> level(E);
  if (E) RSPL_HIP(hipMemcpyAsync(level.data(), b->level, E, hipMemcpyDeviceToHost, st));
  RSPL_HIP(hipStreamSynchronize(st));
  // ---- phase 2: level-0 edges, no kernel ----
  {
    std::vector<int> act;
    for (int i = 0; i < E; i++)
      if (!level[i]) act.push_back(i);
    Phase ph;
    if ((rc = build_active(b, act, epose, elm, pr->pose_fixed, np, nL, 0, ph))) return rc;
    if ((rc = optimize(b, P, Lr, ph, pr->iterations_second, np, nq, nl, &res->chi2_second,
                       &res->iterations_done_second)))
      return rc;
  }
  RSPL_HIP(ba::classify(P, Lr, E, nullptr, b->inlier, 1, st));
  std::vector<uint8_t> inl(E);
  if (E) RSPL_HIP(hipMemcpyAsync(inl.data(), b->inlier, E, hipMemcpyDeviceToHost, st));
  RSPL_HIP(hipMemcpyAsync(T.data(), b->T, sizeof(double) * T.size(), hipMemcpyDeviceToHost, st));
  if (nq) RSPL_HIP(hipMemcpyAsync(res->points, b->X, sizeof(double) * 3 * nq, hipMemcpyDeviceToHost, st));
  if (nl) RSPL_HIP(hipMemcpyAsync(res->lines, b->L, sizeof(double) * 6 * nl, hipMemcpyDeviceToHost, st));
  RSPL_HIP(hipStreamSynchronize(st));
  uint8_t* outs[4] = {res->mono_inlier, res->stereo_inlier, res->mono_line_inlier, res->stereo_line_inlier};
  e = 0;
  for (int t = 0; t < 4; t++)
    for (int i = 0; i < ne[t]; i++, e++)
      if (outs[t]) outs[t][i] = inl[e];
  // write back T_wc = estimate().inverse() (:235-240)
  for (int p = 0; p < np; p++) {
    Se3h Tcw;
    for (int k = 0; k < 4; k++) Tcw.q[k] = T[8 * p + k];
    for (int k = 0; k < 3; k++) Tcw.t[k] = T[8 * p + 4 + k];
    const Se3h Twc = inverse(Tcw);
    res->pose_q[4 * p + 0] = Twc.q[1];
    res->pose_q[4 * p + 1] = Twc.q[2];
    res->pose_q[4 * p + 2] = Twc.q[3];
    res->pose_q[4 * p + 3] = Twc.q[0];
    for (int k = 0; k < 3; k++) res->pose_p[3 * p + k] = Twc.t[k];
  }
  return RSPL_OK;
}
