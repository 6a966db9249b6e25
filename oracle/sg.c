/*
 * ORACLE (test infrastructure only) -- fp32 CPU restatement of the SuperGlue
 * network as exported by the reference (convert2onnx/superglue.py):
 *   KeypointEncoder            :75-85   (MLP [3,32,64,128,256,256], BN eval + ReLU)
 *   MultiHeadedAttention       :88-142  (channel c = d*4 + h, scores / sqrt(64))
 *   AttentionalPropagation/GNN :145-173 (18 layers, self/cross, pre-layer sources)
 *   final_proj + scores / 16   :295-300
 *   log_optimal_transport      :176-205 (100 log-domain Sinkhorn iterations)
 * Layout: channel-major [C][N] exactly as the module's Conv1d tensors.
 */
#include <math.h>
#include <float.h>

#include "oracle_common.h"

static void conv1d(const float* in, int cin, int n, const float* w, const float* b, int cout, float* out) {
#pragma omp parallel for schedule(static)
  for (int co = 0; co < cout; co++) {
    float* o = out + (size_t)co * n;
    for (int p = 0; p < n; p++) o[p] = b[co];
    for (int ci = 0; ci < cin; ci++) {
      const float wv = w[(size_t)co * cin + ci];
      const float* ip = in + (size_t)ci * n;
      for (int p = 0; p < n; p++) o[p] += wv * ip[p];
    }
  }
}

/* BatchNorm1d eval (eps 1e-5) + ReLU, in place. */
static void bn_relu(float* x, int c, int n, const float* g, const float* bta, const float* mean,
                    const float* var) {
  for (int ch = 0; ch < c; ch++) {
    const float invstd = 1.f / sqrtf(var[ch] + 1e-5f);
    const float alpha = invstd * g[ch];
    const float beta = bta[ch] - mean[ch] * alpha;
    for (int p = 0; p < n; p++) {
      const float v = x[(size_t)ch * n + p] * alpha + beta;
      x[(size_t)ch * n + p] = v > 0.f ? v : 0.f;
    }
  }
}

typedef struct {
  const orc_weights* w;
  int err;
} ctx;

static const float* G(ctx* c, const char* fmt, int l, int64_t n) {
  char name[128];
  snprintf(name, sizeof(name), fmt, l);
  const float* p = orc_get(c->w, name, n);
  if (!p) c->err = 1;
  return p;
}

/* desc [256][n] += kenc(kpts, scores) */
static void kenc(ctx* c, const float* kpts, const float* scores, int n, float* desc) {
  static const int ch[6] = {3, 32, 64, 128, 256, 256};
  float* a = (float*)malloc(sizeof(float) * 256 * (size_t)(n ? n : 1));
  float* b = (float*)malloc(sizeof(float) * 256 * (size_t)(n ? n : 1));
  for (int p = 0; p < n; p++) {
    a[0 * n + p] = kpts[2 * p];
    a[1 * n + p] = kpts[2 * p + 1];
    a[2 * n + p] = scores[p];
  }
  for (int i = 1; i < 6; i++) {
    const int li = 3 * (i - 1);
    const float* w = G(c, "kenc.encoder.%d.weight", li, (int64_t)ch[i] * ch[i - 1]);
    const float* bb = G(c, "kenc.encoder.%d.bias", li, ch[i]);
    if (c->err) break;
    conv1d(a, ch[i - 1], n, w, bb, ch[i], b);
    if (i < 5) {
      const float* g = G(c, "kenc.encoder.%d.weight", li + 1, ch[i]);
      const float* be = G(c, "kenc.encoder.%d.bias", li + 1, ch[i]);
      const float* mu = G(c, "kenc.encoder.%d.running_mean", li + 1, ch[i]);
      const float* va = G(c, "kenc.encoder.%d.running_var", li + 1, ch[i]);
      if (c->err) break;
      bn_relu(b, ch[i], n, g, be, mu, va);
    }
    float* t = a; a = b; b = t;
  }
  if (!c->err)
    for (size_t i = 0; i < (size_t)256 * n; i++) desc[i] += a[i];
  free(a);
  free(b);
}

/* delta [256][n] = AttentionalPropagation(layer l)(x [256][n], src [256][m]) */
static void attn_prop(ctx* c, int l, const float* x, int n, const float* src, int m, float* delta) {
  const int nn = n ? n : 1, mm = m ? m : 1;
  float* q = (float*)malloc(sizeof(float) * 256 * nn);
  float* k = (float*)malloc(sizeof(float) * 256 * mm);
  float* v = (float*)malloc(sizeof(float) * 256 * mm);
  float* o = (float*)malloc(sizeof(float) * 256 * nn);
  float* cat = (float*)malloc(sizeof(float) * 512 * nn);
  float* hid = (float*)malloc(sizeof(float) * 512 * nn);
  const float* wq = G(c, "gnn.layers.%d.attn.proj.0.weight", l, 65536);
  const float* bq = G(c, "gnn.layers.%d.attn.proj.0.bias", l, 256);
  const float* wk = G(c, "gnn.layers.%d.attn.proj.1.weight", l, 65536);
  const float* bk = G(c, "gnn.layers.%d.attn.proj.1.bias", l, 256);
  const float* wv = G(c, "gnn.layers.%d.attn.proj.2.weight", l, 65536);
  const float* bv = G(c, "gnn.layers.%d.attn.proj.2.bias", l, 256);
  const float* wm = G(c, "gnn.layers.%d.attn.merge.weight", l, 65536);
  const float* bm = G(c, "gnn.layers.%d.attn.merge.bias", l, 256);
  const float* w0 = G(c, "gnn.layers.%d.mlp.0.weight", l, 512 * 512);
  const float* b0 = G(c, "gnn.layers.%d.mlp.0.bias", l, 512);
  const float* g1 = G(c, "gnn.layers.%d.mlp.1.weight", l, 512);
  const float* be1 = G(c, "gnn.layers.%d.mlp.1.bias", l, 512);
  const float* mu1 = G(c, "gnn.layers.%d.mlp.1.running_mean", l, 512);
  const float* va1 = G(c, "gnn.layers.%d.mlp.1.running_var", l, 512);
  const float* w3 = G(c, "gnn.layers.%d.mlp.3.weight", l, 256 * 512);
  const float* b3 = G(c, "gnn.layers.%d.mlp.3.bias", l, 256);
  if (!c->err) {
    conv1d(x, 256, n, wq, bq, 256, q);
    conv1d(src, 256, m, wk, bk, 256, k);
    conv1d(src, 256, m, wv, bv, 256, v);
#pragma omp parallel
    {
      float* prob = (float*)malloc(sizeof(float) * mm);
#pragma omp for collapse(2) schedule(static)
      for (int h = 0; h < 4; h++)
        for (int i = 0; i < n; i++) {
          float mx = -INFINITY;
          for (int j = 0; j < m; j++) {
            float s = 0.f;
            for (int d = 0; d < 64; d++) s += q[(size_t)(d * 4 + h) * n + i] * k[(size_t)(d * 4 + h) * m + j];
            s = s / 8.0f;
            prob[j] = s;
            if (s > mx) mx = s;
          }
          float sum = 0.f;
          for (int j = 0; j < m; j++) {
            prob[j] = expf(prob[j] - mx);
            sum += prob[j];
          }
          for (int j = 0; j < m; j++) prob[j] /= sum;
          for (int d = 0; d < 64; d++) {
            float acc = 0.f;
            for (int j = 0; j < m; j++) acc += prob[j] * v[(size_t)(d * 4 + h) * m + j];
            o[(size_t)(d * 4 + h) * n + i] = acc;
          }
        }
      free(prob);
    }
    memcpy(cat, x, sizeof(float) * 256 * (size_t)n);
    conv1d(o, 256, n, wm, bm, 256, cat + (size_t)256 * n);
    conv1d(cat, 512, n, w0, b0, 512, hid);
    bn_relu(hid, 512, n, g1, be1, mu1, va1);
    conv1d(hid, 512, n, w3, b3, 256, delta);
  }
  free(q); free(k); free(v); free(o); free(cat); free(hid);
}

static float lse(const float* x, int n, int stride) {
  float m = -INFINITY;
  for (int i = 0; i < n; i++) m = fmaxf(m, x[(size_t)i * stride]);
  if (!isfinite(m)) m = 0.f;
  float s = 0.f;
  for (int i = 0; i < n; i++) s += expf(x[(size_t)i * stride] - m);
  return logf(s) + m;
}

/* log_optimal_transport (superglue.py:176-205): scores [m][n] -> Z [(m+1)][(n+1)]. */
void orc_log_optimal_transport(const float* scores, int m, int n, float alpha, int iters, float* Z) {
  const int R = m + 1, C = n + 1;
  float* cp = (float*)malloc(sizeof(float) * (size_t)R * C);
  float* u = (float*)calloc(R, sizeof(float));
  float* v = (float*)calloc(C, sizeof(float));
  float* tmp = (float*)malloc(sizeof(float) * (size_t)(R > C ? R : C));
  for (int i = 0; i < R; i++)
    for (int j = 0; j < C; j++) cp[(size_t)i * C + j] = (i < m && j < n) ? scores[(size_t)i * n + j] : alpha;
  const float norm = -logf((float)m + (float)n);
  for (int it = 0; it < iters; it++) {
    for (int i = 0; i < R; i++) {
      for (int j = 0; j < C; j++) tmp[j] = cp[(size_t)i * C + j] + v[j];
      const float lmu = (i < m) ? norm : logf((float)n) + norm;
      u[i] = lmu - lse(tmp, C, 1);
    }
    for (int j = 0; j < C; j++) {
      for (int i = 0; i < R; i++) tmp[i] = cp[(size_t)i * C + j] + u[i];
      const float lnu = (j < n) ? norm : logf((float)m) + norm;
      v[j] = lnu - lse(tmp, R, 1);
    }
  }
  for (int i = 0; i < R; i++)
    for (int j = 0; j < C; j++) Z[(size_t)i * C + j] = cp[(size_t)i * C + j] + u[i] + v[j] - norm;
  free(cp); free(u); free(v); free(tmp);
}

/* SuperGlue.forward (superglue.py:269-305).  kpts*: [n][2] normalised, scores*: [n],
 * desc*: [256][n] channel-major.  Z: [(n0+1)*(n1+1)]. */
int orc_sg_forward(const char* weights_path, const float* kpts0, const float* scores0, const float* desc0,
                   int n0, const float* kpts1, const float* scores1, const float* desc1, int n1,
                   int iters, float* Z) {
  orc_weights ws;
  if (orc_load_weights(weights_path, &ws)) return -2;
  ctx c = {&ws, 0};
  const int a0 = n0 ? n0 : 1, a1 = n1 ? n1 : 1;
  float* d0 = (float*)malloc(sizeof(float) * 256 * a0);
  float* d1 = (float*)malloc(sizeof(float) * 256 * a1);
  float* e0 = (float*)malloc(sizeof(float) * 256 * a0);
  float* e1 = (float*)malloc(sizeof(float) * 256 * a1);
  memcpy(d0, desc0, sizeof(float) * 256 * (size_t)n0);
  memcpy(d1, desc1, sizeof(float) * 256 * (size_t)n1);
  kenc(&c, kpts0, scores0, n0, d0);
  kenc(&c, kpts1, scores1, n1, d1);
  for (int l = 0; l < 18 && !c.err; l++) {
    const int cross = l & 1; /* ['self', 'cross'] * 9 */
    attn_prop(&c, l, d0, n0, cross ? d1 : d0, cross ? n1 : n0, e0);
    attn_prop(&c, l, d1, n1, cross ? d0 : d1, cross ? n0 : n1, e1);
    for (size_t i = 0; i < (size_t)256 * n0; i++) d0[i] += e0[i];
    for (size_t i = 0; i < (size_t)256 * n1; i++) d1[i] += e1[i];
  }
  const float* wf = orc_get(&ws, "final_proj.weight", 65536);
  const float* bf = orc_get(&ws, "final_proj.bias", 256);
  const float* bin = orc_get(&ws, "bin_score", 1);
  int rc = (c.err || !wf || !bf || !bin) ? -2 : 0;
  if (!rc) {
    conv1d(d0, 256, n0, wf, bf, 256, e0);
    conv1d(d1, 256, n1, wf, bf, 256, e1);
    float* S = (float*)malloc(sizeof(float) * (size_t)a0 * a1);
#pragma omp parallel for schedule(static)
    for (int i = 0; i < n0; i++)
      for (int j = 0; j < n1; j++) {
        float s = 0.f;
        for (int d = 0; d < 256; d++) s += e0[(size_t)d * n0 + i] * e1[(size_t)d * n1 + j];
        S[(size_t)i * n1 + j] = s / 16.0f;
      }
    orc_log_optimal_transport(S, n0, n1, bin[0], iters, Z);
    free(S);
  }
  free(d0); free(d1); free(e0); free(e1);
  orc_free_weights(&ws);
  return rc;
}
