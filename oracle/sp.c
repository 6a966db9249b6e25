/*
 * ORACLE (test infrastructure only) -- fp32 CPU restatement of the SuperPoint
 * network as exported by the reference:
 *   encoder / heads      convert2onnx/superpoint.py:114-161
 *   simple_nms (r = 4)   convert2onnx/superpoint.py:6-33
 * NCHW, one image, float32 accumulation (order differs from oneDNN: results
 * agree with the reference module to ~1e-6 relative, pinned by tests/golden).
 */
#include <math.h>
#include <float.h>

#include "oracle_common.h"

#define RB 4 /* output rows per task */

static void conv3x3(const float* in, int cin, int H, int W, const float* w, const float* b, int cout,
                    float* out, int relu) {
  const int nyb = (H + RB - 1) / RB;
#pragma omp parallel
  {
    float* acc = (float*)malloc(sizeof(float) * RB * (size_t)W);
#pragma omp for collapse(2) schedule(static)
    for (int yb = 0; yb < nyb; yb++) {
      for (int co = 0; co < cout; co++) {
        const int y0 = yb * RB;
        const int nr = (y0 + RB <= H) ? RB : H - y0;
        for (int r = 0; r < nr; r++)
          for (int x = 0; x < W; x++) acc[r * W + x] = b[co];
        for (int ci = 0; ci < cin; ci++) {
          const float* ip = in + (size_t)ci * H * W;
          const float* wp = w + ((size_t)co * cin + ci) * 9;
          for (int ky = 0; ky < 3; ky++) {
            for (int kx = 0; kx < 3; kx++) {
              const float wv = wp[ky * 3 + kx];
              const int dx = kx - 1;
              const int xs = dx < 0 ? 1 : 0, xe = dx > 0 ? W - 1 : W;
              for (int r = 0; r < nr; r++) {
                const int yy = y0 + r + ky - 1;
                if (yy < 0 || yy >= H) continue;
                const float* irow = ip + (size_t)yy * W + dx;
                float* arow = acc + r * W;
                for (int x = xs; x < xe; x++) arow[x] += wv * irow[x];
              }
            }
          }
        }
        for (int r = 0; r < nr; r++) {
          float* o = out + (size_t)co * H * W + (size_t)(y0 + r) * W;
          for (int x = 0; x < W; x++) {
            float v = acc[r * W + x];
            o[x] = (relu && v < 0.f) ? 0.f : v;
          }
        }
      }
    }
    free(acc);
  }
}

static void conv1x1(const float* in, int cin, int P, const float* w, const float* b, int cout, float* out) {
#pragma omp parallel for schedule(static)
  for (int co = 0; co < cout; co++) {
    float* o = out + (size_t)co * P;
    for (int p = 0; p < P; p++) o[p] = b[co];
    for (int ci = 0; ci < cin; ci++) {
      const float wv = w[(size_t)co * cin + ci];
      const float* ip = in + (size_t)ci * P;
      for (int p = 0; p < P; p++) o[p] += wv * ip[p];
    }
  }
}

static void maxpool2(const float* in, int C, int H, int W, float* out) {
  const int h = H / 2, w = W / 2;
#pragma omp parallel for schedule(static)
  for (int c = 0; c < C; c++)
    for (int y = 0; y < h; y++)
      for (int x = 0; x < w; x++) {
        const float* p = in + (size_t)c * H * W + (size_t)(2 * y) * W + 2 * x;
        float m = p[0];
        if (p[1] > m) m = p[1];
        if (p[W] > m) m = p[W];
        if (p[W + 1] > m) m = p[W + 1];
        out[(size_t)c * h * w + (size_t)y * w + x] = m;
      }
}

/* 9x9 stride-1 max pool with -inf padding (nn.MaxPool2d(9, 1, 4)), separable. */
static void maxpool9(const float* in, int H, int W, float* tmp, float* out) {
  const int r = 4;
  for (int y = 0; y < H; y++)
    for (int x = 0; x < W; x++) {
      float m = -INFINITY;
      for (int k = -r; k <= r; k++) {
        int xx = x + k;
        if (xx >= 0 && xx < W && in[y * W + xx] > m) m = in[y * W + xx];
      }
      tmp[y * W + x] = m;
    }
  for (int y = 0; y < H; y++)
    for (int x = 0; x < W; x++) {
      float m = -INFINITY;
      for (int k = -r; k <= r; k++) {
        int yy = y + k;
        if (yy >= 0 && yy < H && tmp[yy * W + x] > m) m = tmp[yy * W + x];
      }
      out[y * W + x] = m;
    }
}

/* simple_nms (convert2onnx/superpoint.py:16-33), in place on s [H*W]. */
void orc_simple_nms(float* s, int H, int W) {
  const size_t n = (size_t)H * W;
  float* mp = (float*)malloc(sizeof(float) * n);
  float* tmp = (float*)malloc(sizeof(float) * n);
  float* f = (float*)malloc(sizeof(float) * n);
  unsigned char* mask = (unsigned char*)malloc(n);
  unsigned char* supp = (unsigned char*)malloc(n);
  maxpool9(s, H, W, tmp, mp);
  for (size_t i = 0; i < n; i++) mask[i] = (s[i] == mp[i]);
  for (int it = 0; it < 2; it++) {
    for (size_t i = 0; i < n; i++) f[i] = mask[i] ? 1.f : 0.f;
    maxpool9(f, H, W, tmp, mp);
    for (size_t i = 0; i < n; i++) {
      supp[i] = mp[i] > 0.f;
      f[i] = supp[i] ? 0.f : s[i]; /* supp_scores */
    }
    maxpool9(f, H, W, tmp, mp);
    for (size_t i = 0; i < n; i++) {
      const int new_max = (f[i] == mp[i]);
      mask[i] = mask[i] | (new_max & !supp[i]);
    }
  }
  for (size_t i = 0; i < n; i++)
    if (!mask[i]) s[i] = 0.f;
  free(mp); free(tmp); free(f); free(mask); free(supp);
}

#define GET(name, n)                         \
  const float* name = orc_get(w, #name, n); \
  if (!name) return -2;

/* Full forward: in [H*W] (already u8/255), scores [H*W] (post-NMS), desc [256*(H/8)*(W/8)]. */
int orc_sp_forward(const char* weights_path, const float* img, int H, int W, float* scores, float* desc) {
  if (H % 8 || W % 8) return -1;
  orc_weights ws;
  if (orc_load_weights(weights_path, &ws)) return -2;
  const orc_weights* w = &ws;
  int rc = 0;
  const int H2 = H / 2, W2 = W / 2, H4 = H / 4, W4 = W / 4, H8 = H / 8, W8 = W / 8;
  const size_t P8 = (size_t)H8 * W8;
  float* a = (float*)malloc(sizeof(float) * 64 * (size_t)H * W);
  float* bb = (float*)malloc(sizeof(float) * 64 * (size_t)H * W);
  {
#define W_(n, k) orc_get(w, n, k)
    const float *c1aw = W_("conv1a.weight", 64 * 9), *c1ab = W_("conv1a.bias", 64);
    const float *c1bw = W_("conv1b.weight", 64 * 64 * 9), *c1bb = W_("conv1b.bias", 64);
    const float *c2aw = W_("conv2a.weight", 64 * 64 * 9), *c2ab = W_("conv2a.bias", 64);
    const float *c2bw = W_("conv2b.weight", 64 * 64 * 9), *c2bb = W_("conv2b.bias", 64);
    const float *c3aw = W_("conv3a.weight", 128 * 64 * 9), *c3ab = W_("conv3a.bias", 128);
    const float *c3bw = W_("conv3b.weight", 128 * 128 * 9), *c3bb = W_("conv3b.bias", 128);
    const float *c4aw = W_("conv4a.weight", 128 * 128 * 9), *c4ab = W_("conv4a.bias", 128);
    const float *c4bw = W_("conv4b.weight", 128 * 128 * 9), *c4bb = W_("conv4b.bias", 128);
    const float *cPaw = W_("convPa.weight", 256 * 128 * 9), *cPab = W_("convPa.bias", 256);
    const float *cPbw = W_("convPb.weight", 65 * 256), *cPbb = W_("convPb.bias", 65);
    const float *cDaw = W_("convDa.weight", 256 * 128 * 9), *cDab = W_("convDa.bias", 256);
    const float *cDbw = W_("convDb.weight", 256 * 256), *cDbb = W_("convDb.bias", 256);
#undef W_
    if (!c1aw || !c1ab || !c1bw || !c1bb || !c2aw || !c2ab || !c2bw || !c2bb || !c3aw || !c3ab || !c3bw ||
        !c3bb || !c4aw || !c4ab || !c4bw || !c4bb || !cPaw || !cPab || !cPbw || !cPbb || !cDaw || !cDab ||
        !cDbw || !cDbb) {
      rc = -2;
      goto done;
    }
    /* shared encoder (superpoint.py:117-127) */
    conv3x3(img, 1, H, W, c1aw, c1ab, 64, a, 1);
    conv3x3(a, 64, H, W, c1bw, c1bb, 64, bb, 1);
    maxpool2(bb, 64, H, W, a);
    conv3x3(a, 64, H2, W2, c2aw, c2ab, 64, bb, 1);
    conv3x3(bb, 64, H2, W2, c2bw, c2bb, 64, a, 1);
    maxpool2(a, 64, H2, W2, bb);
    conv3x3(bb, 64, H4, W4, c3aw, c3ab, 128, a, 1);
    conv3x3(a, 128, H4, W4, c3bw, c3bb, 128, bb, 1);
    maxpool2(bb, 128, H4, W4, a);
    conv3x3(a, 128, H8, W8, c4aw, c4ab, 128, bb, 1);
    conv3x3(bb, 128, H8, W8, c4bw, c4bb, 128, a, 1); /* x = a [128][P8] */
    float* cP = bb;
    float* semi = bb + 256 * P8;
    /* detector head (superpoint.py:130-135) */
    conv3x3(a, 128, H8, W8, cPaw, cPab, 256, cP, 1);
    conv1x1(cP, 256, (int)P8, cPbw, cPbb, 65, semi);
    for (size_t p = 0; p < P8; p++) {
      float m = -INFINITY;
      for (int c = 0; c < 65; c++) m = fmaxf(m, semi[c * P8 + p]);
      float sum = 0.f;
      for (int c = 0; c < 65; c++) sum += expf(semi[c * P8 + p] - m);
      const int cy = (int)(p / W8), cx = (int)(p % W8);
      for (int c = 0; c < 64; c++) {
        const float v = expf(semi[c * P8 + p] - m) / sum;
        scores[(size_t)(cy * 8 + c / 8) * W + cx * 8 + (c % 8)] = v;
      }
    }
    orc_simple_nms(scores, H, W);
    /* descriptor head (superpoint.py:159-161) */
    float* cD = bb;
    conv3x3(a, 128, H8, W8, cDaw, cDab, 256, cD, 1);
    conv1x1(cD, 256, (int)P8, cDbw, cDbb, 256, desc);
    for (size_t p = 0; p < P8; p++) {
      float ss = 0.f;
      for (int c = 0; c < 256; c++) ss += desc[c * P8 + p] * desc[c * P8 + p];
      float nrm = sqrtf(ss);
      if (nrm < 1e-12f) nrm = 1e-12f;
      for (int c = 0; c < 256; c++) desc[c * P8 + p] /= nrm;
    }
  }
done:
  free(a);
  free(bb);
  orc_free_weights(&ws);
  return rc;
}
