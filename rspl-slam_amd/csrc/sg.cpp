// SuperGlue + PointMatching handle: C ABI (include/rspl.h) over sg_kernels.hip.
// Mirrors SuperGlue::build / infer / process_output (src/super_glue.cpp:21-472) and
// PointMatching::MatchingPoints (src/point_matching.cc:12-62).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "common.hpp"
#include "sg_kernels.hpp"

using namespace rspl;

namespace {
constexpr int kLayers = 18;
constexpr int kKencIn = 16;  // keypoint-encoder input (x, y, score) zero-padded to the GEMM K step
const int kKencCh[6] = {3, 32, 64, 128, 256, 256};
}  // namespace

struct rspl_sg {
  rspl_sg_config cfg{};
  hipStream_t stream = nullptr;
  Arena arena;
  int nmax = 0, B = 0, G = 0, ld = 0;
  // weights
  float* kw[5];
  float* kb[5];
  float *wqkv, *bqkv, *wm, *bm, *w1, *b1, *w2, *b2;  // [18] stacked
  // RSPL_PREC_FP16: mlp.0 with attn.merge folded into its message half (fp32 source of hw1, bias)
  float *w1m, *b1m;
  float *wf, *bf, *bin;
  // RSPL_PREC_FP16: transposed fp16 copies [N][K] of every projection / MLP weight
  _Float16* hkw[5];
  _Float16 *hwqkv, *hwm, *hw1, *hw2, *hwf;
  _Float16 *fwqkv, *fw1, *fw2;  // the same in MFMA B-fragment order (fused GNN layers)
  // activations
  float *kin, *h1, *h2, *X, *QKV, *O, *MSG, *HID, *cpl, *Z, *val0;
  // RSPL_PREC_FP16 GNN activations: fp16 shadow of X, Q | K, V^T per head, messages, hidden
  _Float16 *Xh, *QKh, *Vth, *Oh, *MSGh, *HIDh;
  _Float16 *Qf[2], *Kf[2], *Vf[2];  // fused layers: q (row-major) / k, v (MFMA fragment order), ping-pong
  int ldv = 0;  // token stride of Vth (nmax rounded up to the 32-key attention tile; zero padded)
  unsigned long long *ug, *vg;  // Sinkhorn u / v exchange granules [B][ld] (row-block: ug = [B][2][rbG][ld])
  int rbG = 0;                  // row-block Sinkhorn workgroups per pair (0: slab kernel)
  bool sink_sc = false;         // with rbG: the scaling-form kernel
  bool sink_wide = false;       // with sink_sc: the wide two-hop kernel (640 < nmax + 1 <= 2112)
  float* cplT = nullptr;        // transposed column slabs when they exceed LDS [B][ld*ld]
  bool sink_scratch = false;
  unsigned* err = nullptr;      // [B] sticky Sinkhorn timeout flags, host-mapped (rspl_sg_status)
  unsigned* d_err = nullptr;    // device alias of err
  unsigned sk_seq = 0;
  unsigned spin_limit = 1u << 22;
  int inject = 0;
  float* dbg_alpha;             // rspl_sg_debug_sinkhorn's bin score
  int *max0, *max1, *n0, *n1;
  int32_t *idx0, *idx1;
  double *ms0, *ms1, *f0, *f1;
  // host pinned staging
  double* h_f = nullptr;
  int32_t* h_idx = nullptr;
  double* h_ms = nullptr;
  int last_n0 = 0, last_n1 = 0, last_B = 0;
  // post-stream pipelining: couplings / Z / counts double-buffered by call parity
  int *cn0, *cn1;                     // [2][B] the call's counts (the caller may reuse its own at once)
  hipEvent_t ev_ready = nullptr;      // main stream: couplings of this call written
  hipEvent_t ev_sink[2] = {nullptr, nullptr};  // post stream: Sinkhorn of parity p done with cpl[p]
  hipEvent_t ev_done = nullptr;  // post stream: the last call's decode done (debug entry points wait on it)
  unsigned long long calls = 0;
  int last_parity = 0;
  StageTimer timer;
};

namespace {

// Sinkhorn exchange granules: ug = [B][ld] (slab), [B][2][rbG][ld] (row-block / scaling form) or the wide
// kernel's hop-1 buffers [B][2][G][G][cs]; vg = [B][ld] or the wide kernel's hop-2 buffers [B][2][G cs]
size_t ug_len(const rspl_sg* s) {
  if (s->sink_wide) return (size_t)s->B * sg::sinkhorn_wide_hop1_len(s->nmax);
  return (size_t)s->B * s->ld * (s->rbG ? 2 * s->rbG : 1);
}
size_t vg_len(const rspl_sg* s) {
  return s->sink_wide ? (size_t)s->B * sg::sinkhorn_wide_hop2_len(s->nmax) : (size_t)s->B * s->ld;
}

template <typename F>
void carve(F& ar, rspl_sg* s) {
  const size_t T = (size_t)s->B * 2 * s->nmax, ld = s->ld, B = s->B;
  auto take = [&](auto*& p, size_t n) {
    using Tp = std::remove_pointer_t<std::remove_reference_t<decltype(p)>>;
    if constexpr (std::is_same_v<F, Arena>) p = ar.template take<Tp>(n);
    else ar.template take<Tp>(n);
  };
  for (int i = 0; i < 5; i++) {
    const int cin = i == 0 ? kKencIn : kKencCh[i];
    take(s->kw[i], (size_t)cin * kKencCh[i + 1]);
    take(s->kb[i], kKencCh[i + 1]);
  }
  take(s->wqkv, (size_t)kLayers * 256 * 768); take(s->bqkv, (size_t)kLayers * 768);
  take(s->wm, (size_t)kLayers * 256 * 256); take(s->bm, (size_t)kLayers * 256);
  take(s->w1, (size_t)kLayers * 512 * 512); take(s->b1, (size_t)kLayers * 512);
  take(s->w1m, (size_t)kLayers * 512 * 512); take(s->b1m, (size_t)kLayers * 512);
  take(s->w2, (size_t)kLayers * 512 * 256); take(s->b2, (size_t)kLayers * 256);
  take(s->wf, 256 * 256); take(s->bf, 256); take(s->bin, 4);
  for (int i = 0; i < 5; i++) take(s->hkw[i], (size_t)(i == 0 ? kKencIn : kKencCh[i]) * kKencCh[i + 1]);
  take(s->hwqkv, (size_t)kLayers * 256 * 768); take(s->hwm, (size_t)kLayers * 256 * 256);
  take(s->hw1, (size_t)kLayers * 512 * 512); take(s->hw2, (size_t)kLayers * 512 * 256); take(s->hwf, 256 * 256);
  take(s->fwqkv, (size_t)kLayers * 256 * 768); take(s->fw1, (size_t)kLayers * 512 * 512);
  take(s->fw2, (size_t)kLayers * 512 * 256);
  take(s->kin, T * kKencIn); take(s->h1, T * 256); take(s->h2, T * 256);
  take(s->X, T * 256); take(s->QKV, T * 768); take(s->O, T * 256); take(s->MSG, T * 256); take(s->HID, T * 512);
  take(s->Xh, T * 256); take(s->QKh, T * 512); take(s->Vth, (size_t)B * 2 * 256 * s->ldv); take(s->Oh, T * 256);
  take(s->MSGh, T * 256); take(s->HIDh, T * 512);
  for (int i = 0; i < 2; i++) {
    take(s->Qf[i], T * 256); take(s->Kf[i], (size_t)B * 2 * 256 * s->ldv); take(s->Vf[i], (size_t)B * 2 * 256 * s->ldv);
  }

  take(s->cpl, 2 * B * ld * ld); take(s->Z, 2 * B * ld * ld); take(s->ug, ug_len(s)); take(s->vg, vg_len(s));
  if (s->sink_scratch) take(s->cplT, B * ld * ld);
  take(s->dbg_alpha, 4);
  take(s->cn0, 2 * B); take(s->cn1, 2 * B);
  take(s->max0, B * s->nmax); take(s->val0, B * s->nmax); take(s->max1, B * s->nmax);
  take(s->idx0, B * s->nmax); take(s->idx1, B * s->nmax); take(s->ms0, B * s->nmax); take(s->ms1, B * s->nmax);
  take(s->n0, B); take(s->n1, B);
  take(s->f0, B * s->nmax * 259); take(s->f1, B * s->nmax * 259);
}

struct Up {
  bool ok = true;
  void operator()(float* dst, const std::vector<float>& v) {
    ok &= hipMemcpy(dst, v.data(), v.size() * sizeof(float), hipMemcpyHostToDevice) == hipSuccess;
  }
};

// BatchNorm1d eval fold (eps 1e-5): returns per-channel (scale, shift) so that
// BN(conv(x)) = conv'(x) with W' = scale * W, b' = scale * (b - mean) + beta.
bool bn_fold(const std::vector<Tensor>& ts, const std::string& pre, int c, std::vector<double>& sc,
             std::vector<double>& sh) {
  const Tensor* g = find(ts, pre + ".weight", c);
  const Tensor* b = find(ts, pre + ".bias", c);
  const Tensor* m = find(ts, pre + ".running_mean", c);
  const Tensor* v = find(ts, pre + ".running_var", c);
  if (!g || !b || !m || !v) return false;
  sc.resize(c);
  sh.resize(c);
  for (int i = 0; i < c; i++) {
    sc[i] = (double)g->data[i] / std::sqrt((double)v->data[i] + 1e-5);
    sh[i] = (double)b->data[i] - (double)m->data[i] * sc[i];
  }
  return true;
}

int upload_weights(rspl_sg* s, const std::vector<Tensor>& ts) {
  Up up;
  // KeypointEncoder (superglue.py:75-85): conv1d [co][ci][1] -> W^T [ci][co], BN folded
  for (int i = 0; i < 5; i++) {
    const int li = 3 * i, ci = kKencCh[i], co = kKencCh[i + 1], cip = i == 0 ? kKencIn : ci;
    const Tensor* w = find(ts, "kenc.encoder." + std::to_string(li) + ".weight", (int64_t)co * ci);
    const Tensor* b = find(ts, "kenc.encoder." + std::to_string(li) + ".bias", co);
    if (!w || !b) return RSPL_E_WEIGHTS;
    std::vector<double> sc(co, 1.0), sh(co, 0.0);
    if (i < 4 && !bn_fold(ts, "kenc.encoder." + std::to_string(li + 1), co, sc, sh)) return RSPL_E_WEIGHTS;
    std::vector<float> wt((size_t)cip * co, 0.f), bt(co);
    for (int o = 0; o < co; o++) {
      for (int k = 0; k < ci; k++) wt[(size_t)k * co + o] = (float)(sc[o] * w->data[(size_t)o * ci + k]);
      bt[o] = (float)(sc[o] * b->data[o] + sh[o]);
    }
    up(s->kw[i], wt);
    up(s->kb[i], bt);
  }
  // GNN layers (superglue.py:126-173)
  for (int l = 0; l < kLayers; l++) {
    const std::string p = "gnn.layers." + std::to_string(l);
    std::vector<float> wqkv((size_t)256 * 768), bqkv(768);
    for (int j = 0; j < 3; j++) {
      const Tensor* w = find(ts, p + ".attn.proj." + std::to_string(j) + ".weight", 65536);
      const Tensor* b = find(ts, p + ".attn.proj." + std::to_string(j) + ".bias", 256);
      if (!w || !b) return RSPL_E_WEIGHTS;
      for (int h = 0; h < 4; h++)
        for (int d = 0; d < 64; d++) {
          const int c = d * 4 + h, o = j * 256 + h * 64 + d;  // view(b, 64, 4, N): c = d*4 + h
          bqkv[o] = b->data[c];
          for (int k = 0; k < 256; k++) wqkv[(size_t)k * 768 + o] = w->data[(size_t)c * 256 + k];
        }
    }
    up(s->wqkv + (size_t)l * 256 * 768, wqkv);
    up(s->bqkv + (size_t)l * 768, bqkv);
    const Tensor* wm = find(ts, p + ".attn.merge.weight", 65536);
    const Tensor* bm = find(ts, p + ".attn.merge.bias", 256);
    const Tensor* w0 = find(ts, p + ".mlp.0.weight", 512 * 512);
    const Tensor* b0 = find(ts, p + ".mlp.0.bias", 512);
    const Tensor* w3 = find(ts, p + ".mlp.3.weight", 256 * 512);
    const Tensor* b3 = find(ts, p + ".mlp.3.bias", 256);
    std::vector<double> sc, sh;
    if (!wm || !bm || !w0 || !b0 || !w3 || !b3 || !bn_fold(ts, p + ".mlp.1", 512, sc, sh)) return RSPL_E_WEIGHTS;
    std::vector<float> wmt((size_t)256 * 256);
    for (int o = 0; o < 256; o++)
      for (int h = 0; h < 4; h++)
        for (int d = 0; d < 64; d++) wmt[(size_t)(h * 64 + d) * 256 + o] = wm->data[(size_t)o * 256 + d * 4 + h];
    up(s->wm + (size_t)l * 65536, wmt);
    up(s->bm + (size_t)l * 256, bm->data);
    std::vector<float> w1t((size_t)512 * 512), b1t(512);
    for (int o = 0; o < 512; o++) {
      for (int k = 0; k < 512; k++) w1t[(size_t)k * 512 + o] = (float)(sc[o] * w0->data[(size_t)o * 512 + k]);
      b1t[o] = (float)(sc[o] * b0->data[o] + sh[o]);
    }
    up(s->w1 + (size_t)l * 512 * 512, w1t);
    up(s->b1 + (size_t)l * 512, b1t);
    {  // fp16 engine: attn.merge is linear and feeds only mlp.0's message half, so
       // W1 [x; Wm o + bm] + b1 = [W1x | W1m Wm] [x; o] + (b1 + W1m bm): one GEMM fewer per layer
      std::vector<double> acc((size_t)256 * 512, 0.0), bacc(512);
      for (int o = 0; o < 512; o++) {
        double sb = sc[o] * b0->data[o] + sh[o];
        for (int m = 0; m < 256; m++) sb += sc[o] * w0->data[(size_t)o * 512 + 256 + m] * bm->data[m];
        bacc[o] = sb;
      }
      std::vector<double> w1d((size_t)256 * 512);  // message half, [m][o]
      for (int o = 0; o < 512; o++)
        for (int m = 0; m < 256; m++) w1d[(size_t)m * 512 + o] = sc[o] * w0->data[(size_t)o * 512 + 256 + m];
      for (int c = 0; c < 256; c++) {
        double* ac = acc.data() + (size_t)c * 512;
        for (int m = 0; m < 256; m++) {
          const double a = wmt[(size_t)c * 256 + m];
          const double* row = w1d.data() + (size_t)m * 512;
          for (int o = 0; o < 512; o++) ac[o] += a * row[o];
        }
      }
      std::vector<float> w1f(w1t), b1f(512);
      for (size_t i = 0; i < acc.size(); i++) w1f[(size_t)256 * 512 + i] = (float)acc[i];
      for (int o = 0; o < 512; o++) b1f[o] = (float)bacc[o];
      up(s->w1m + (size_t)l * 512 * 512, w1f);
      up(s->b1m + (size_t)l * 512, b1f);
    }
    std::vector<float> w2t((size_t)512 * 256);
    for (int o = 0; o < 256; o++)
      for (int k = 0; k < 512; k++) w2t[(size_t)k * 256 + o] = w3->data[(size_t)o * 512 + k];
    up(s->w2 + (size_t)l * 512 * 256, w2t);
    up(s->b2 + (size_t)l * 256, b3->data);
  }
  const Tensor* wf = find(ts, "final_proj.weight", 65536);
  const Tensor* bf = find(ts, "final_proj.bias", 256);
  const Tensor* bin = find(ts, "bin_score", 1);
  if (!wf || !bf || !bin) return RSPL_E_WEIGHTS;
  std::vector<float> wft((size_t)256 * 256);
  for (int o = 0; o < 256; o++)
    for (int k = 0; k < 256; k++) wft[(size_t)k * 256 + o] = wf->data[(size_t)o * 256 + k];
  up(s->wf, wft);
  up(s->bf, bf->data);
  up(s->bin, std::vector<float>{bin->data[0], 0.f, 0.f, 0.f});
  if (!up.ok) {
    set_error("SuperGlue weight upload failed");
    return RSPL_E_DEVICE;
  }
  return RSPL_OK;
}

sg::GemmArgs G_(const float* A, int lda, const float* B, int ldb, const float* bias, float* C, int ldc, int M, int N,
                int K, int epi, const _Float16* hB = nullptr) {
  sg::GemmArgs g{};
  g.hB = hB;
  g.ldbh = K;
  g.A = A; g.lda = lda; g.ksplit = K; g.B = B; g.ldb = ldb; g.bias = bias; g.C = C; g.ldc = ldc;
  g.M = M; g.N = N; g.K = K; g.alpha = 1.f; g.epi = epi;
  return g;
}

}  // namespace

// log_optimal_transport (superglue.py:185-205) on the couplings of B pairs, on stream st
static hipError_t run_sinkhorn(rspl_sg* s, const float* cpl, float* Zp, const int* cn0, const int* cn1, int B,
                               int iters, hipStream_t st, hipEvent_t t0 = nullptr, hipEvent_t t1 = nullptr) {
  hipError_t e;
  sg::SinkArgs sk{};
  sk.cpl = cpl; sk.Z = Zp; sk.cplT = s->cplT; sk.ug = s->ug; sk.vg = s->vg;
  sk.seq = s->sk_seq = (s->sk_seq % 0xFFFFFu) + 1;
  sk.spin_limit = s->spin_limit; sk.inject = s->inject;
  sk.err = s->d_err; sk.n0 = cn0; sk.n1 = cn1;
  sk.nmax = s->nmax; sk.G = s->rbG ? s->rbG : s->G; sk.rb = s->rbG > 0; sk.sc = s->sink_sc; sk.iters = iters;
  sk.wide = s->sink_wide;
  sk.sleep = 1;
  return sg::sinkhorn(sk, B, st, t0, t1);
}

extern "C" int rspl_sg_create(const rspl_sg_config* cfg, const char* weights_path, rspl_sg** out) {
  RSPL_CHECK_ARG(cfg && out, "rspl_sg_create: NULL argument");
  RSPL_CHECK_ARG(cfg->max_keypoints > 0 && cfg->max_keypoints <= 4096, "max_keypoints must be in [1, 4096]");
  RSPL_CHECK_ARG(cfg->precision == RSPL_PREC_FP32 || cfg->precision == RSPL_PREC_FP16,
                 "precision must be RSPL_PREC_FP32 or RSPL_PREC_FP16");
  RSPL_CHECK_ARG(cfg->image_width > 0 && cfg->image_height > 0, "image size must be positive");
  // the Sinkhorn exchange tag is (call sequence << 12) | (iteration + 1)
  RSPL_CHECK_ARG(cfg->sinkhorn_iterations < 4096, "sinkhorn_iterations must be < 4096");
  *out = nullptr;
  std::vector<Tensor> ts;
  int rc = load_blob(weights_path, ts);
  if (rc) return rc;
  RSPL_HIP(hipSetDevice(cfg->device));
  auto* s = new rspl_sg();
  s->cfg = *cfg;
  if (s->cfg.max_batch < 1) s->cfg.max_batch = 1;
  if (s->cfg.sinkhorn_iterations <= 0) s->cfg.sinkhorn_iterations = 100;
  s->B = s->cfg.max_batch;
  s->nmax = cfg->max_keypoints;  // output stride per pair (rspl.h)
  s->ld = s->nmax + 1;
  s->ldv = (s->nmax + 31) / 32 * 32;
  {  // Sinkhorn workgroups per pair: ~kRows rows + columns each, and at least enough that both
     // slabs fit one workgroup's LDS; all B*G workgroups must be co-resident (one per CU)
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, cfg->device) != hipSuccess || ncu < 1) {
      set_error("hipDeviceGetAttribute(MultiprocessorCount) failed");
      delete s;
      return RSPL_E_DEVICE;
    }
    constexpr int kRows = 9;  // 45 workgroups per pair at N = 400 (round-2 A/B: 32 vs 48)
    int G = std::max(1, (s->ld + kRows - 1) / kRows);
    while (G < s->ld && sg::sinkhorn_lds_bytes(s->nmax, G, true) > sg::kSinkLdsMax) G++;
    if (const char* e = getenv("RSPL_SG_SINK_G"); e && getenv("RSPL_SG_SINK") &&
        std::string(getenv("RSPL_SG_SINK")) == "slab")
      G = std::max(1, atoi(e));
    G = std::min(G, std::max(1, ncu / s->B));
    s->G = G;
    s->sink_scratch = sg::sinkhorn_lds_bytes(s->nmax, G, true) > sg::kSinkLdsMax;
    // nmax + 1 <= 640: rows in registers, one exchange per iteration -- the scaling-form kernel (8 workgroups
    // per pair); RSPL_SG_SINK=slab keeps the slab kernel; RSPL_SG_SINK_G sets the workgroups per pair
    const char* sk = getenv("RSPL_SG_SINK");
    const std::string kind = sk ? sk : "sc";
    if (kind != "slab") {
      int rg = 8;
      if (const char* e = getenv("RSPL_SG_SINK_G")) rg = std::max(1, atoi(e));
      s->sink_sc = true;
      rg = std::min(rg, std::max(1, ncu / s->B));
      while (rg <= 32 && rg * s->B <= ncu && !sg::sinkhorn_rb_rpw(s->nmax, rg)) rg++;
      if (rg * s->B <= ncu && sg::sinkhorn_rb_rpw(s->nmax, rg)) s->rbG = rg;
      // 448 < nmax + 1 <= 640 (e.g. C4's 600 keypoints): the scaling-form kernel with ten column
      // sets per lane, ceil(ld / 48) workgroups of <= 48 rows per pair
      if (!s->rbG && s->sink_sc) {
        int g = (s->ld + 47) / 48;
        if (const char* e = getenv("RSPL_SG_SINK_G")) g = std::max(1, atoi(e));
        if (g * s->B <= ncu && sg::sinkhorn_sc10_ok(s->nmax, g)) s->rbG = g;
      }
      // 640 < nmax + 1 <= 2112 (C5's 2048 keypoints): the wide scaling-form kernel, 32 rows per workgroup,
      // the column exchange in two hops (reduce-scatter to the column owners, broadcast of V)
      if (!s->rbG && s->sink_sc) {
        const int g = sg::sinkhorn_wide_groups(s->nmax);
        if (g * s->B <= ncu && sg::sinkhorn_wide_ok(s->nmax, g)) {
          s->rbG = g;
          s->sink_wide = true;
        }
      }
    }
    if (s->B * s->G > ncu && !s->rbG) {
      set_error("max_batch (%d) exceeds the CU count (%d): the Sinkhorn workgroups must be co-resident", s->B, ncu);
      delete s;
      return RSPL_E_ARG;
    }
  }
  Sizer sz;
  carve(sz, s);
  if ((rc = s->arena.reserve(sz.used))) { delete s; return rc; }
  carve(s->arena, s);
  if (hipMemset(s->ug, 0, sizeof(unsigned long long) * ug_len(s)) != hipSuccess ||
      hipMemset(s->vg, 0, sizeof(unsigned long long) * vg_len(s)) != hipSuccess ||
      hipMemset(s->Vth, 0, sizeof(_Float16) * s->B * 2 * 256 * s->ldv) != hipSuccess ||
      hipMemset(s->Kf[0], 0, sizeof(_Float16) * s->B * 2 * 256 * s->ldv) != hipSuccess ||
      hipMemset(s->Kf[1], 0, sizeof(_Float16) * s->B * 2 * 256 * s->ldv) != hipSuccess ||
      hipMemset(s->Vf[0], 0, sizeof(_Float16) * s->B * 2 * 256 * s->ldv) != hipSuccess ||
      hipMemset(s->Vf[1], 0, sizeof(_Float16) * s->B * 2 * 256 * s->ldv) != hipSuccess) {
    set_error("sinkhorn exchange buffer init failed");
    rspl_sg_destroy(s);
    return RSPL_E_DEVICE;
  }
  const size_t nm = s->nmax;
  if (s->timer.init(RSPL_SG_STAGES) != RSPL_OK || hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&s->ev_ready, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&s->ev_sink[0], hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&s->ev_sink[1], hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&s->ev_done, hipEventDisableTiming) != hipSuccess ||
      hipHostMalloc(&s->h_f, sizeof(double) * nm * 259 * 2) != hipSuccess ||
      hipHostMalloc(&s->h_idx, sizeof(int32_t) * nm * 2 + 16) != hipSuccess ||
      hipHostMalloc(&s->h_ms, sizeof(double) * nm * 2) != hipSuccess ||
      hipHostMalloc(&s->err, sizeof(unsigned) * s->B, hipHostMallocMapped) != hipSuccess ||
      hipHostGetDevicePointer((void**)&s->d_err, s->err, 0) != hipSuccess) {
    set_error("stream / pinned allocation failed");
    rspl_sg_destroy(s);
    return RSPL_E_DEVICE;
  }
  memset(s->err, 0, sizeof(unsigned) * s->B);
  if ((rc = upload_weights(s, ts))) { rspl_sg_destroy(s); return rc; }
  {  // fp16 transposed copies for RSPL_PREC_FP16 (made on the device from the fp32 layout)
    bool okh = true;
    for (int i = 0; i < 5; i++)
      okh &= sg::to_half_t(s->kw[i], i == 0 ? kKencIn : kKencCh[i], kKencCh[i + 1], s->hkw[i], s->stream) == hipSuccess;
    for (int l = 0; l < kLayers; l++) {
      okh &= sg::to_half_t(s->wqkv + (size_t)l * 256 * 768, 256, 768, s->hwqkv + (size_t)l * 256 * 768, s->stream) ==
             hipSuccess;
      okh &= sg::to_half_t(s->wm + (size_t)l * 65536, 256, 256, s->hwm + (size_t)l * 65536, s->stream) == hipSuccess;
      okh &= sg::to_half_t(s->w1m + (size_t)l * 512 * 512, 512, 512, s->hw1 + (size_t)l * 512 * 512, s->stream) ==
             hipSuccess;
      okh &= sg::to_half_t(s->w2 + (size_t)l * 512 * 256, 512, 256, s->hw2 + (size_t)l * 512 * 256, s->stream) ==
             hipSuccess;
      okh &= sg::to_frag(s->hwqkv + (size_t)l * 256 * 768, 768, 256, s->fwqkv + (size_t)l * 256 * 768, s->stream) ==
             hipSuccess;
      okh &= sg::to_frag(s->hw1 + (size_t)l * 512 * 512, 512, 512, s->fw1 + (size_t)l * 512 * 512, s->stream) ==
             hipSuccess;
      okh &= sg::to_frag(s->hw2 + (size_t)l * 512 * 256, 256, 512, s->fw2 + (size_t)l * 512 * 256, s->stream) ==
             hipSuccess;
    }
    okh &= sg::to_half_t(s->wf, 256, 256, s->hwf, s->stream) == hipSuccess;
    okh &= hipStreamSynchronize(s->stream) == hipSuccess;
    if (!okh) {
      set_error("fp16 weight conversion failed");
      rspl_sg_destroy(s);
      return RSPL_E_DEVICE;
    }
  }
  *out = s;
  return RSPL_OK;
}

extern "C" void rspl_sg_destroy(rspl_sg* s) {
  if (!s) return;

  if (s->stream) (void)hipStreamSynchronize(s->stream);
  s->arena.release();
  s->timer.destroy();
  if (s->h_f) (void)hipHostFree(s->h_f);
  if (s->h_idx) (void)hipHostFree(s->h_idx);
  if (s->h_ms) (void)hipHostFree(s->h_ms);
  if (s->err) (void)hipHostFree(s->err);
  if (s->ev_ready) (void)hipEventDestroy(s->ev_ready);
  if (s->ev_done) (void)hipEventDestroy(s->ev_done);
  for (auto& e : s->ev_sink)
    if (e) (void)hipEventDestroy(e);
  if (s->stream) (void)hipStreamDestroy(s->stream);
  delete s;
}

extern "C" int rspl_sg_infer_device(rspl_sg* s, int B, const double* d_feat0, const int* d_n0, const double* d_feat1,
                                    const int* d_n1, int stride_feat, int normalize, int32_t* d_idx0, int32_t* d_idx1,
                                    double* d_ms0, double* d_ms1, void* stream_) {
  return rspl_sg_infer_device2(s, B, d_feat0, d_n0, d_feat1, d_n1, stride_feat, normalize, d_idx0, d_idx1, d_ms0, d_ms1,
                               stream_, stream_);
}

extern "C" int rspl_sg_infer_device2(rspl_sg* s, int B, const double* d_feat0, const int* d_n0,
                                     const double* d_feat1, const int* d_n1, int stride_feat, int normalize,
                                     int32_t* d_idx0, int32_t* d_idx1, double* d_ms0, double* d_ms1, void* stream_,
                                     void* post_stream_) {
  RSPL_CHECK_ARG(s && d_feat0 && d_feat1 && d_n0 && d_n1 && d_idx0 && d_idx1 && d_ms0 && d_ms1,
                 "rspl_sg_infer_device: NULL argument");
  RSPL_CHECK_ARG(B >= 1 && B <= s->B, "batch %d outside [1, %d]", B, s->B);
  RSPL_CHECK_ARG(stride_feat >= 1, "stride_feat must be >= 1");
  hipStream_t st = stream_ ? (hipStream_t)stream_ : s->stream;
  hipStream_t pst = post_stream_ ? (hipStream_t)post_stream_ : st;
  const int nm = s->nmax, T = B * 2 * nm;
  const int par = (int)(s->calls++ & 1);
  float* cpl = s->cpl + (size_t)par * s->B * s->ld * s->ld;
  float* Zp = s->Z + (size_t)par * s->B * s->ld * s->ld;
  int* cn0 = s->cn0 + par * s->B;
  int* cn1 = s->cn1 + par * s->B;
  // counts snapshot (the post stream still reads them after the caller moved on)
  RSPL_HIP(hipMemcpyAsync(cn0, d_n0, sizeof(int) * B, hipMemcpyDeviceToDevice, st));
  RSPL_HIP(hipMemcpyAsync(cn1, d_n1, sizeof(int) * B, hipMemcpyDeviceToDevice, st));
  // process_input (+ NormalizeKeypoints when called as PointMatching)
  s->timer.mark(0, st);
  sg::PrepArgs pa{};
  pa.f0 = d_feat0; pa.f1 = d_feat1; pa.n0 = d_n0; pa.n1 = d_n1; pa.stride = stride_feat;
  pa.normalize = normalize; pa.width = s->cfg.image_width; pa.height = s->cfg.image_height;
  pa.nmax = nm; pa.kin = s->kin; pa.X = s->X; pa.B = B;
  RSPL_HIP(sg::prep(pa, st));
  // KeypointEncoder: desc += kenc([x, y, score]) (superglue.py:288-289)
  const bool h16 = s->cfg.precision == RSPL_PREC_FP16;  // the reference's kFP16 engine (super_glue.cpp:132)
  const float* in = s->kin;
  int cin = kKencIn;
  float* bufs[2] = {s->h1, s->h2};
  for (int i = 0; i < 5; i++) {
    const int co = kKencCh[i + 1];
    float* outp = i == 4 ? s->X : bufs[i & 1];
    RSPL_HIP(sg::gemm(G_(in, cin, s->kw[i], co, s->kb[i], outp, co, T, co, cin, i == 4 ? 2 : 1, h16 ? s->hkw[i] : nullptr),
                      1, st));
    in = outp;
    cin = co;
  }
  s->timer.mark(1, st);
  // AttentionalGNN (superglue.py:165-173): ['self', 'cross'] * 9; both images read pre-layer descs
  if (h16) {  // fp16 activations end to end (X itself stays fp32: the residual stream)
    RSPL_HIP(sg::to_half(s->X, s->Xh, (size_t)T * 256, st));
    auto gh = [&](const _Float16* A, int lda, const _Float16* W, int N, int K, const float* bias) {
      sg::GemmHArgs g{};
      g.A = A; g.lda = lda; g.ksplit = K; g.B = W; g.ldb = K; g.bias = bias; g.M = T; g.N = N; g.K = K;
      g.nmax = nm; g.ldv = s->ldv;
      return g;
    };
    // one launch per layer on one workgroup per 32-token tile (layer_kernel).  (Four launches per layer --
    // QKV GEMM, attention, mlp.0, mlp.3 -- were slower and were removed in round 6; round 5 measured the layer on
    // four workgroups per tile -- the same bits, slower in the pipeline: profiles/r05_experiments.md.)
    auto layer = [&](sg::LayerArgs& la, int) { return sg::gnn_layer(la, B, st); };
    {  // layer 0's q / k / v (prologue launch), then one fused launch per layer
      {
        sg::LayerArgs la{};
        la.Qn = s->Qf[0]; la.Kn = s->Kf[0]; la.Vn = s->Vf[0];
        la.X = s->X; la.Xh = s->Xh;
        la.Wq = s->fwqkv; la.bq = s->bqkv;
        la.n0 = d_n0; la.n1 = d_n1; la.nmax = nm; la.nt = s->ldv / 32; la.qkv_only = 1;
        RSPL_HIP(layer(la, -1));
      }
      for (int l = 0; l < kLayers; l++) {
        sg::LayerArgs la{};
        la.Qc = s->Qf[l & 1]; la.Kc = s->Kf[l & 1]; la.Vc = s->Vf[l & 1];
        la.Qn = s->Qf[(l + 1) & 1]; la.Kn = s->Kf[(l + 1) & 1]; la.Vn = s->Vf[(l + 1) & 1];
        la.X = s->X; la.Xh = s->Xh;
        la.W1 = s->fw1 + (size_t)l * 512 * 512; la.b1 = s->b1m + (size_t)l * 512;
        la.W2 = s->fw2 + (size_t)l * 512 * 256; la.b2 = s->b2 + (size_t)l * 256;
        const int ln = std::min(l + 1, kLayers - 1);
        la.Wq = s->fwqkv + (size_t)ln * 256 * 768; la.bq = s->bqkv + (size_t)ln * 768;
        la.n0 = d_n0; la.n1 = d_n1; la.nmax = nm; la.nt = s->ldv / 32; la.cross = l & 1; la.last = l == kLayers - 1;
        RSPL_HIP(layer(la, l));
      }
    }
  }
  for (int l = 0; l < kLayers && !h16; l++) {
    RSPL_HIP(sg::gemm(G_(s->X, 256, s->wqkv + (size_t)l * 256 * 768, 768, s->bqkv + (size_t)l * 768, s->QKV, 768, T,
                         768, 256, 0, h16 ? s->hwqkv + (size_t)l * 256 * 768 : nullptr), 1, st));
    sg::AttnArgs at{};
    at.qkv = s->QKV; at.O = s->O; at.n0 = d_n0; at.n1 = d_n1; at.nmax = nm; at.cross = l & 1;
    RSPL_HIP(sg::attention(at, B, st));
    RSPL_HIP(sg::gemm(G_(s->O, 256, s->wm + (size_t)l * 65536, 256, s->bm + (size_t)l * 256, s->MSG, 256, T, 256, 256,
                         0, h16 ? s->hwm + (size_t)l * 65536 : nullptr), 1, st));
    sg::GemmArgs g1 = G_(s->X, 256, s->w1 + (size_t)l * 512 * 512, 512, s->b1 + (size_t)l * 512, s->HID, 512, T, 512,
                         512, 1, h16 ? s->hw1 + (size_t)l * 512 * 512 : nullptr);
    g1.A2 = s->MSG;  // torch.cat([x, message], dim=1)
    g1.ksplit = 256;
    RSPL_HIP(sg::gemm(g1, 1, st));
    RSPL_HIP(sg::gemm(G_(s->HID, 512, s->w2 + (size_t)l * 512 * 256, 256, s->b2 + (size_t)l * 256, s->X, 256, T, 256,
                         512, 2, h16 ? s->hw2 + (size_t)l * 512 * 256 : nullptr), 1, st));
  }
  s->timer.mark(2, st);
  // final_proj + scores / descriptor_dim**.5 (superglue.py:295-300)
  float* MD = s->MSG;
  if (h16) {
    sg::GemmHArgs g{};
    g.A = s->Xh; g.lda = 256; g.ksplit = 256; g.B = s->hwf; g.ldb = 256; g.bias = s->bf; g.M = T; g.N = 256; g.K = 256;
    g.C32 = MD; g.ldc32 = 256;
    RSPL_HIP(sg::gemm_h(g, 0, st));
  } else {
    RSPL_HIP(sg::gemm(G_(s->X, 256, s->wf, 256, s->bf, MD, 256, T, 256, 256, 0, nullptr), 1, st));
  }
  {
    if (pst != st && s->calls > 2) RSPL_HIP(hipStreamWaitEvent(st, s->ev_sink[par], 0));
    sg::GemmArgs g = G_(MD, 256, MD + (size_t)nm * 256, 256, nullptr, cpl, s->ld, nm, nm, 256, 0);
    g.b_nt = 1;
    g.alpha = 1.f / 16.f;
    g.sA = g.sB = (long long)2 * nm * 256;
    g.sC = (long long)s->ld * s->ld;
    g.mcount = d_n0; g.ncount = d_n1; g.count_stride = 1;
    RSPL_HIP(sg::gemm(g, B, st));
  }
  sg::BinsArgs bn{};
  bn.cpl = cpl; bn.n0 = d_n0; bn.n1 = d_n1; bn.alpha = s->bin; bn.nmax = nm;
  RSPL_HIP(sg::bins(bn, B, st));
  s->timer.mark(3, st);
  if (pst != st) {  // log-Sinkhorn + decode on the post stream: the next call's GNN overlaps them
    RSPL_HIP(hipEventRecord(s->ev_ready, st));
    RSPL_HIP(hipStreamWaitEvent(pst, s->ev_ready, 0));
  }
  // log_optimal_transport (superglue.py:185-205)
  // events 4 / 5 are stamped by the Sinkhorn launch itself (its own start / end): stage 3 is the
  // post stream's hand-over wait, stage 4 exactly the Sinkhorn kernel
  RSPL_HIP(run_sinkhorn(s, cpl, Zp, cn0, cn1, B, s->cfg.sinkhorn_iterations, pst, s->timer.slot(4),
                        s->timer.slot(5)));
  if (pst != st) RSPL_HIP(hipEventRecord(s->ev_sink[par], pst));
  // decode (super_glue.cpp:339-367), threshold 0.2 hard-coded as in the reference (:355)
  sg::DecodeArgs dc{};
  dc.Z = Zp; dc.n0 = cn0; dc.n1 = cn1; dc.nmax = nm; dc.max0 = s->max0; dc.val0 = s->val0; dc.max1 = s->max1;
  dc.idx0 = d_idx0; dc.idx1 = d_idx1; dc.ms0 = d_ms0; dc.ms1 = d_ms1; dc.threshold = 0.2f;
  RSPL_HIP(sg::decode(dc, B, pst));
  RSPL_HIP(hipEventRecord(s->ev_done, pst));
  s->timer.mark(6, pst);
  s->timer.end_call();
  s->last_B = B;
  s->last_parity = par;
  return RSPL_OK;
}

// read and clear the sticky Sinkhorn flags of pairs [0, npairs) only (a host call launches pair 0:
// a flag left by an unchecked device-path call of another pair is not reported as this call's)
static int sink_status(rspl_sg* s, int npairs, uint32_t* pair_flags) {
  uint32_t f = 0;
  for (int p = 0; p < npairs && p < s->B; p++) {
    volatile unsigned* e = s->err + p;
    if (*e) f |= p < 32 ? (1u << p) : 0x80000000u;
    *e = 0;
  }
  if (pair_flags) *pair_flags = f;
  if (f) {
    set_error("superglue: cross-workgroup exchange (GNN quads / Sinkhorn) timed out (pair mask 0x%x); results of "
              "those pairs are invalid", f);
    return RSPL_E_DEVICE;
  }
  return RSPL_OK;
}

// the debug entry points reuse the exchange / scratch / Z buffers of pair 0: wait for any device-path
// call still running on a caller's post stream first
static int sync_all(rspl_sg* s) {
  RSPL_HIP(hipStreamSynchronize(s->stream));
  RSPL_HIP(hipEventSynchronize(s->ev_done));
  return RSPL_OK;
}

static int sg_host_run(rspl_sg* s, const double* f0, int n0, const double* f1, int n1, int normalize) {
  RSPL_CHECK_ARG(n0 >= 0 && n1 >= 0 && n0 <= s->cfg.max_keypoints && n1 <= s->cfg.max_keypoints,
                 "keypoint counts (%d, %d) outside [0, %d]", n0, n1, s->cfg.max_keypoints);
  RSPL_CHECK_ARG((f0 || !n0) && (f1 || !n1), "NULL feature matrix");
  const size_t nm = s->nmax;
  memcpy(s->h_f, f0, sizeof(double) * 259 * n0);
  memcpy(s->h_f + nm * 259, f1, sizeof(double) * 259 * n1);
  int32_t counts[2] = {n0, n1};
  RSPL_HIP(hipMemcpyAsync(s->f0, s->h_f, sizeof(double) * 259 * n0, hipMemcpyHostToDevice, s->stream));
  RSPL_HIP(hipMemcpyAsync(s->f1, s->h_f + nm * 259, sizeof(double) * 259 * n1, hipMemcpyHostToDevice, s->stream));
  RSPL_HIP(hipMemcpyAsync(s->n0, &counts[0], sizeof(int32_t), hipMemcpyHostToDevice, s->stream));
  RSPL_HIP(hipMemcpyAsync(s->n1, &counts[1], sizeof(int32_t), hipMemcpyHostToDevice, s->stream));
  int rc = rspl_sg_infer_device(s, 1, s->f0, s->n0, s->f1, s->n1, (int)nm, normalize, s->idx0, s->idx1, s->ms0, s->ms1,
                                s->stream);
  if (rc) return rc;
  RSPL_HIP(hipMemcpyAsync(s->h_idx, s->idx0, sizeof(int32_t) * n0, hipMemcpyDeviceToHost, s->stream));
  RSPL_HIP(hipMemcpyAsync(s->h_idx + nm, s->idx1, sizeof(int32_t) * n1, hipMemcpyDeviceToHost, s->stream));
  RSPL_HIP(hipMemcpyAsync(s->h_ms, s->ms0, sizeof(double) * n0, hipMemcpyDeviceToHost, s->stream));
  RSPL_HIP(hipMemcpyAsync(s->h_ms + nm, s->ms1, sizeof(double) * n1, hipMemcpyDeviceToHost, s->stream));
  RSPL_HIP(hipStreamSynchronize(s->stream));
  unsigned flags = 0;
  if (int rc2 = sink_status(s, 1, &flags)) return rc2;
  s->last_n0 = n0;
  s->last_n1 = n1;
  if (n0 == 0 || n1 == 0) {  // no couplings: every keypoint unmatched
    for (int i = 0; i < n0; i++) { s->h_idx[i] = -1; s->h_ms[i] = 0; }
    for (int j = 0; j < n1; j++) { s->h_idx[nm + j] = -1; s->h_ms[nm + j] = 0; }
  }
  return RSPL_OK;
}

extern "C" int rspl_sg_infer(rspl_sg* s, const double* f0, int n0, const double* f1, int n1, int32_t* indices0,
                             int32_t* indices1, double* mscores0, double* mscores1) {
  RSPL_CHECK_ARG(s && (indices0 || !n0) && (indices1 || !n1) && (mscores0 || !n0) && (mscores1 || !n1),
                 "rspl_sg_infer: NULL argument");
  int rc = sg_host_run(s, f0, n0, f1, n1, 0);
  if (rc) return rc;
  const size_t nm = s->nmax;
  memcpy(indices0, s->h_idx, sizeof(int32_t) * n0);
  memcpy(indices1, s->h_idx + nm, sizeof(int32_t) * n1);
  memcpy(mscores0, s->h_ms, sizeof(double) * n0);
  memcpy(mscores1, s->h_ms + nm, sizeof(double) * n1);
  return RSPL_OK;
}

extern "C" int rspl_pm_match(rspl_sg* s, const double* f0, int n0, const double* f1, int n1, rspl_dmatch* matches,
                             int capacity, int* n_matches, int outlier_rejection) {
  RSPL_CHECK_ARG(s && n_matches && (matches || capacity == 0), "rspl_pm_match: NULL argument");
  RSPL_CHECK_ARG(!outlier_rejection, "outlier_rejection (cv::findFundamentalMat RANSAC) is not implemented");
  int rc = sg_host_run(s, f0, n0, f1, n1, 1);  // NormalizeKeypoints on device
  if (rc) return rc;
  const size_t nm = s->nmax;
  const int32_t* i0 = s->h_idx;
  const int32_t* i1 = s->h_idx + nm;
  const double* m0 = s->h_ms;
  const double* m1 = s->h_ms + nm;
  int k = 0;
  for (int i = 0; i < n0; i++) {  // src/point_matching.cc:24-31
    const int j = i0[i];
    if (j < n1 && j >= 0 && i1[j] == i) {
      if (k >= capacity) {
        set_error("more than %d matches", capacity);
        return RSPL_E_CAPACITY;
      }
      const double d = 1.0 - (m0[i] + m1[j]) / 2.0;
      matches[k].query_idx = i;
      matches[k].train_idx = j;
      matches[k].distance = (float)d;
      k++;
    }
  }
  *n_matches = k;
  return RSPL_OK;
}

extern "C" int rspl_sg_debug_scores(rspl_sg* s, int p, float* Z) {
  RSPL_CHECK_ARG(s && Z && p >= 0 && p < s->last_B, "rspl_sg_debug_scores: bad argument");
  if (int rc = sync_all(s)) return rc;
  const int R = s->last_n0 + 1, Cc = s->last_n1 + 1;
  RSPL_HIP(hipMemcpy2D(Z, sizeof(float) * Cc, s->Z + ((size_t)s->last_parity * s->B + p) * s->ld * s->ld,
                       sizeof(float) * s->ld,
                       sizeof(float) * Cc, R, hipMemcpyDeviceToHost));
  return RSPL_OK;
}

extern "C" int rspl_sg_profile(rspl_sg* s, int enable) {
  RSPL_CHECK_ARG(s, "NULL handle");
  s->timer.reset(enable != 0);
  return RSPL_OK;
}

extern "C" int rspl_sg_stage_times(rspl_sg* s, float* ms, int* calls) {
  RSPL_CHECK_ARG(s && ms, "NULL argument");
  return s->timer.query(ms, calls);
}

extern "C" int rspl_sg_status(rspl_sg* s, uint32_t* pair_flags) {
  RSPL_CHECK_ARG(s, "rspl_sg_status: NULL handle");
  return sink_status(s, s->B, pair_flags);
}

extern "C" int rspl_sg_debug_inject(rspl_sg* s, int inject, unsigned spin_limit) {
  RSPL_CHECK_ARG(s, "NULL handle");
  s->inject = inject != 0;
  s->spin_limit = spin_limit ? spin_limit : (1u << 22);
  return RSPL_OK;
}

extern "C" int rspl_sg_debug_sinkhorn(rspl_sg* s, const float* scores, int n0, int n1, float alpha, int iters,
                                      float* Z) {
  RSPL_CHECK_ARG(s && scores && Z, "rspl_sg_debug_sinkhorn: NULL argument");
  RSPL_CHECK_ARG(n0 >= 1 && n1 >= 1 && n0 <= s->nmax && n1 <= s->nmax && iters >= 0 && iters < 4096,
                 "bad shape or iteration count (< 4096)");
  const size_t ld = s->ld;
  hipStream_t st = s->stream;
  if (int rc = sync_all(s)) return rc;
  int cnt[2] = {n0, n1};
  const float al[4] = {alpha, 0.f, 0.f, 0.f};
  RSPL_HIP(hipMemcpy2DAsync(s->cpl, sizeof(float) * ld, scores, sizeof(float) * n1, sizeof(float) * n1, n0,
                            hipMemcpyHostToDevice, st));
  RSPL_HIP(hipMemcpyAsync(s->cn0, &cnt[0], sizeof(int), hipMemcpyHostToDevice, st));
  RSPL_HIP(hipMemcpyAsync(s->cn1, &cnt[1], sizeof(int), hipMemcpyHostToDevice, st));
  RSPL_HIP(hipMemcpyAsync(s->dbg_alpha, al, sizeof(al), hipMemcpyHostToDevice, st));
  sg::BinsArgs bn{};
  bn.cpl = s->cpl; bn.n0 = s->cn0; bn.n1 = s->cn1; bn.alpha = s->dbg_alpha; bn.nmax = s->nmax;
  RSPL_HIP(sg::bins(bn, 1, st));
  RSPL_HIP(run_sinkhorn(s, s->cpl, s->Z, s->cn0, s->cn1, 1, iters, st));
  RSPL_HIP(hipMemcpy2DAsync(Z, sizeof(float) * (n1 + 1), s->Z, sizeof(float) * ld, sizeof(float) * (n1 + 1), n0 + 1,
                            hipMemcpyDeviceToHost, st));
  RSPL_HIP(hipStreamSynchronize(st));
  s->last_B = 0;  // the debug call reused pair 0's buffers
  return sink_status(s, 1, nullptr);
}

extern "C" int rspl_sg_debug_decode(rspl_sg* s, const float* Z, int n0, int n1, int32_t* indices0, int32_t* indices1,
                                    double* mscores0, double* mscores1) {
  RSPL_CHECK_ARG(s && Z && indices0 && indices1 && mscores0 && mscores1, "rspl_sg_debug_decode: NULL argument");
  RSPL_CHECK_ARG(n0 >= 1 && n1 >= 1 && n0 <= s->nmax && n1 <= s->nmax, "bad shape");
  const size_t ld = s->ld;
  hipStream_t st = s->stream;
  if (int rc = sync_all(s)) return rc;
  int cnt[2] = {n0, n1};
  RSPL_HIP(hipMemcpy2DAsync(s->Z, sizeof(float) * ld, Z, sizeof(float) * (n1 + 1), sizeof(float) * (n1 + 1), n0 + 1,
                            hipMemcpyHostToDevice, st));
  RSPL_HIP(hipMemcpyAsync(s->cn0, &cnt[0], sizeof(int), hipMemcpyHostToDevice, st));
  RSPL_HIP(hipMemcpyAsync(s->cn1, &cnt[1], sizeof(int), hipMemcpyHostToDevice, st));
  sg::DecodeArgs dc{};
  dc.Z = s->Z; dc.n0 = s->cn0; dc.n1 = s->cn1; dc.nmax = s->nmax; dc.max0 = s->max0; dc.val0 = s->val0;
  dc.max1 = s->max1; dc.idx0 = s->idx0; dc.idx1 = s->idx1; dc.ms0 = s->ms0; dc.ms1 = s->ms1; dc.threshold = 0.2f;
  RSPL_HIP(sg::decode(dc, 1, st));
  RSPL_HIP(hipMemcpyAsync(indices0, s->idx0, sizeof(int32_t) * n0, hipMemcpyDeviceToHost, st));
  RSPL_HIP(hipMemcpyAsync(indices1, s->idx1, sizeof(int32_t) * n1, hipMemcpyDeviceToHost, st));
  RSPL_HIP(hipMemcpyAsync(mscores0, s->ms0, sizeof(double) * n0, hipMemcpyDeviceToHost, st));
  RSPL_HIP(hipMemcpyAsync(mscores1, s->ms1, sizeof(double) * n1, hipMemcpyDeviceToHost, st));
  RSPL_HIP(hipStreamSynchronize(st));
  s->last_B = 0;
  return RSPL_OK;
}
