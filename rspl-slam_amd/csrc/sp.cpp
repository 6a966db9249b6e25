// SuperPoint handle: C ABI (include/rspl.h) over the HIP kernels in sp_kernels.hip.
// Mirrors SuperPoint::build / infer / process_output (src/super_point.cpp:19-319):
// weights are loaded and re-laid-out once at create; every buffer is carved from
// one arena sized for max_batch x max_height x max_width.
#include <algorithm>
#include <cstring>
#include <vector>

#include "common.hpp"
#include "sp_kernels.hpp"

using namespace rspl;

static constexpr int kCandCap = 16384;  // candidates sorted whole in LDS (bitonic top-k); also the keep-all and
                                        // max_keypoints limits.  More candidates (large images) are radix-selected.

struct rspl_sp {
  rspl_sp_config cfg{};
  hipStream_t stream = nullptr;
  Arena arena;
  // weights (device)
  float *lut, *w1a, *b1a, *w1b, *b1b, *w2a, *b2a, *w2b, *b2b, *w3a, *b3a, *w3b, *b3b, *w4a, *b4a, *w4b, *b4b;
  float *wPD, *bPD, *wPb, *bPb, *wDb, *bDb;
  // RSPL_PREC_FP16: the 3x3 conv weights as fp16 [9][Cout][Cin]
  _Float16 *hw1b, *hw2a, *hw2b, *hw3a, *hw3b, *hw4a, *hw4b, *hwPD;
  _Float16 *fwPb, *fwDb;  // convPb / convDb in MFMA B-fragment order (sp::HeadHArgs / TapArgs)
  // RSPL_PREC_FP16X3: the lo halves (w - (float)(half)w) of the same arrays, same layouts
  _Float16 *lw1b, *lw2a, *lw2b, *lw3a, *lw3b, *lw4a, *lw4b, *lwPD, *lfwPb, *lfwDb;
  // activations
  float *actA, *actB, *cells, *scores, *nms, *desc;
  unsigned long long* cand;
  int* cand_count;
  int cand_cap = 0;  // candidate buffer per image: NMS survivors of the largest configured image
  unsigned* sel;
  int* sel_count;
  int32_t* counts;
  double* features;  // host-path staging [B][cap][259]
  uint8_t* image;    // host-path staging
  int feat_cap = 0;
  // host pinned staging
  double* h_features = nullptr;
  int32_t* h_counts = nullptr;
  uint8_t* h_image = nullptr;
  int last_B = 0, last_H = 0, last_W = 0;
  StageTimer timer;
};

namespace {

// torch conv weight [co][ci][3][3] -> [ky][kx][ci][co_total] at column offset co_off
// fp16 layout [9][Cout][Cin] (input channels contiguous: one 16-byte MFMA operand read)
// lo = true: the lo half of the split-fp16 pair, (half)(w - (float)(half)w)
_Float16 half_part(float w, bool lo) {
  const _Float16 hi = (_Float16)w;
  return lo ? (_Float16)(w - (float)hi) : hi;
}

void relayout3x3_h(const Tensor& t, int cin, int cout, std::vector<_Float16>& dst, int co_total, int co_off,
                   bool lo = false) {
  for (int co = 0; co < cout; co++)
    for (int ci = 0; ci < cin; ci++)
      for (int k = 0; k < 9; k++)
        dst[((size_t)k * co_total + co_off + co) * cin + ci] = half_part(t.data[((size_t)co * cin + ci) * 9 + k], lo);
}

void relayout3x3(const Tensor& t, int cin, int cout, std::vector<float>& dst, int co_total, int co_off) {
  for (int co = 0; co < cout; co++)
    for (int ci = 0; ci < cin; ci++)
      for (int k = 0; k < 9; k++) dst[((size_t)k * cin + ci) * co_total + co_off + co] = t.data[((size_t)co * cin + ci) * 9 + k];
}

template <typename F>
void carve(F& ar, rspl_sp* s, int B, int H, int W, int cap) {
  const size_t HW = (size_t)H * W, P = HW / 64;
  auto take = [&](auto*& p, size_t n) {
    using T = std::remove_pointer_t<std::remove_reference_t<decltype(p)>>;
    if constexpr (std::is_same_v<F, Arena>) p = ar.template take<T>(n);
    else ar.template take<T>(n);
  };
  take(s->lut, 256);
  take(s->w1a, 64 * 9); take(s->b1a, 64);
  take(s->w1b, 9 * 64 * 64); take(s->b1b, 64);
  take(s->w2a, 9 * 64 * 64); take(s->b2a, 64);
  take(s->w2b, 9 * 64 * 64); take(s->b2b, 64);
  take(s->w3a, 9 * 64 * 128); take(s->b3a, 128);
  take(s->w3b, 9 * 128 * 128); take(s->b3b, 128);
  take(s->w4a, 9 * 128 * 128); take(s->b4a, 128);
  take(s->w4b, 9 * 128 * 128); take(s->b4b, 128);
  take(s->wPD, 9 * 128 * 512); take(s->bPD, 512);
  take(s->hw1b, 9 * 64 * 64); take(s->hw2a, 9 * 64 * 64); take(s->hw2b, 9 * 64 * 64); take(s->hw3a, 9 * 64 * 128);
  take(s->hw3b, 9 * 128 * 128); take(s->hw4a, 9 * 128 * 128); take(s->hw4b, 9 * 128 * 128);
  take(s->hwPD, 9 * 128 * 512);
  take(s->wPb, 256 * 96); take(s->bPb, 96);
  take(s->wDb, 256 * 256); take(s->bDb, 256);
  take(s->fwPb, 256 * 96); take(s->fwDb, 256 * 256);
  take(s->lw1b, 9 * 64 * 64); take(s->lw2a, 9 * 64 * 64); take(s->lw2b, 9 * 64 * 64); take(s->lw3a, 9 * 64 * 128);
  take(s->lw3b, 9 * 128 * 128); take(s->lw4a, 9 * 128 * 128); take(s->lw4b, 9 * 128 * 128);
  take(s->lwPD, 9 * 128 * 512);
  take(s->lfwPb, 256 * 96); take(s->lfwDb, 256 * 256);
  take(s->actA, B * HW * 16);
  take(s->actB, B * HW * 16);
  take(s->cells, B * P * 512);
  take(s->scores, B * HW);
  take(s->nms, B * HW);
  take(s->desc, B * P * 256);
  take(s->cand, (size_t)B * s->cand_cap);
  take(s->cand_count, B);
  take(s->sel, (size_t)B * kCandCap);
  take(s->sel_count, B);
  take(s->counts, B);
  take(s->features, (size_t)B * cap * 259);
  take(s->image, B * HW);
}

}  // namespace

extern "C" int rspl_sp_create(const rspl_sp_config* cfg, const char* weights_path, rspl_sp** out) {
  RSPL_CHECK_ARG(cfg && out, "rspl_sp_create: NULL argument");
  RSPL_CHECK_ARG(cfg->max_height > 0 && cfg->max_width > 0 && cfg->max_height % 8 == 0 && cfg->max_width % 8 == 0,
                 "max_height/max_width must be positive multiples of 8");
  RSPL_CHECK_ARG(cfg->precision == RSPL_PREC_FP32 || cfg->precision == RSPL_PREC_FP16 ||
                     cfg->precision == RSPL_PREC_FP16X3,
                 "precision must be RSPL_PREC_FP32, RSPL_PREC_FP16 or RSPL_PREC_FP16X3");
  RSPL_CHECK_ARG(cfg->remove_borders >= 0, "remove_borders must be >= 0");
  *out = nullptr;
  std::vector<Tensor> ts;
  int rc = load_blob(weights_path, ts);
  if (rc) return rc;
  RSPL_HIP(hipSetDevice(cfg->device));
  auto* s = new rspl_sp();
  s->cfg = *cfg;
  if (s->cfg.max_batch < 1) s->cfg.max_batch = 1;
  const int B = s->cfg.max_batch, H = cfg->max_height, W = cfg->max_width;
  RSPL_CHECK_ARG(cfg->max_keypoints <= kCandCap, "max_keypoints must be <= %d", kCandCap);
  s->feat_cap = cfg->max_keypoints > 0 ? cfg->max_keypoints : kCandCap;
  // one slot per pixel: the candidate buffer cannot overflow whatever survives simple_nms
  // (flat plateaus keep every tied pixel), so no device path ever truncates it
  s->cand_cap = std::max(kCandCap, H * W);
  Sizer sz;
  carve(sz, s, B, H, W, s->feat_cap);
  if ((rc = s->arena.reserve(sz.used))) { delete s; return rc; }
  carve(s->arena, s, B, H, W, s->feat_cap);
  if (s->timer.init(RSPL_SP_STAGES) != RSPL_OK || hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess ||
      hipHostMalloc(&s->h_features, sizeof(double) * s->feat_cap * 259) != hipSuccess ||
      hipHostMalloc(&s->h_counts, sizeof(int32_t) * B) != hipSuccess ||
      hipHostMalloc(&s->h_image, (size_t)H * W) != hipSuccess) {
    set_error("stream / pinned allocation failed");
    rspl_sp_destroy(s);
    return RSPL_E_DEVICE;
  }

  // ---- weights: relayout once (convert2onnx/superpoint.py:88-105) ----
  struct C3 { const char* name; int cin, cout; float *w, *b; _Float16 *hw, *lw; };
  const C3 convs[] = {{"conv1b", 64, 64, s->w1b, s->b1b, s->hw1b, s->lw1b}, {"conv2a", 64, 64, s->w2a, s->b2a, s->hw2a, s->lw2a},
                      {"conv2b", 64, 64, s->w2b, s->b2b, s->hw2b, s->lw2b}, {"conv3a", 64, 128, s->w3a, s->b3a, s->hw3a, s->lw3a},
                      {"conv3b", 128, 128, s->w3b, s->b3b, s->hw3b, s->lw3b}, {"conv4a", 128, 128, s->w4a, s->b4a, s->hw4a, s->lw4a},
                      {"conv4b", 128, 128, s->w4b, s->b4b, s->hw4b, s->lw4b}};
  auto uph = [&](_Float16* dst, const std::vector<_Float16>& src) {
    return hipMemcpy(dst, src.data(), src.size() * sizeof(_Float16), hipMemcpyHostToDevice) == hipSuccess;
  };
  auto up = [&](float* dst, const std::vector<float>& src) {
    return hipMemcpy(dst, src.data(), src.size() * sizeof(float), hipMemcpyHostToDevice) == hipSuccess;
  };
  bool ok = true;
  for (auto& c : convs) {
    const Tensor* w = find(ts, std::string(c.name) + ".weight", (int64_t)c.cout * c.cin * 9);
    const Tensor* b = find(ts, std::string(c.name) + ".bias", c.cout);
    if (!w || !b) { rspl_sp_destroy(s); return RSPL_E_WEIGHTS; }
    std::vector<float> r((size_t)9 * c.cin * c.cout);
    relayout3x3(*w, c.cin, c.cout, r, c.cout, 0);
    std::vector<_Float16> rh((size_t)9 * c.cin * c.cout), rl(rh.size());
    relayout3x3_h(*w, c.cin, c.cout, rh, c.cout, 0);
    relayout3x3_h(*w, c.cin, c.cout, rl, c.cout, 0, true);
    ok &= up(c.w, r) && up(c.b, b->data) && uph(c.hw, rh) && uph(c.lw, rl);
  }
  const Tensor *w1a = find(ts, "conv1a.weight", 64 * 9), *b1a = find(ts, "conv1a.bias", 64);
  const Tensor *wPa = find(ts, "convPa.weight", 256 * 128 * 9), *bPa = find(ts, "convPa.bias", 256);
  const Tensor *wDa = find(ts, "convDa.weight", 256 * 128 * 9), *bDa = find(ts, "convDa.bias", 256);
  const Tensor *wPb = find(ts, "convPb.weight", 65 * 256), *bPb = find(ts, "convPb.bias", 65);
  const Tensor *wDb = find(ts, "convDb.weight", 256 * 256), *bDb = find(ts, "convDb.bias", 256);
  if (!w1a || !b1a || !wPa || !bPa || !wDa || !bDa || !wPb || !bPb || !wDb || !bDb) {
    rspl_sp_destroy(s);
    return RSPL_E_WEIGHTS;
  }
  ok &= up(s->w1a, w1a->data) && up(s->b1a, b1a->data);
  {  // convPa | convDa horizontally fused: 512 output channels
    std::vector<float> r((size_t)9 * 128 * 512), b(512);
    relayout3x3(*wPa, 128, 256, r, 512, 0);
    relayout3x3(*wDa, 128, 256, r, 512, 256);
    std::vector<_Float16> rh((size_t)9 * 128 * 512), rl(rh.size());
    relayout3x3_h(*wPa, 128, 256, rh, 512, 0);
    relayout3x3_h(*wDa, 128, 256, rh, 512, 256);
    relayout3x3_h(*wPa, 128, 256, rl, 512, 0, true);
    relayout3x3_h(*wDa, 128, 256, rl, 512, 256, true);
    ok &= uph(s->hwPD, rh) && uph(s->lwPD, rl);
    for (int i = 0; i < 256; i++) { b[i] = bPa->data[i]; b[256 + i] = bDa->data[i]; }
    ok &= up(s->wPD, r) && up(s->bPD, b);
  }
  {  // convPb [65][256] -> [256][96] (zero padded), convDb [256][256] -> [ci][co]
    std::vector<float> r(256 * 96, 0.f), b(96, 0.f), d(256 * 256);
    for (int co = 0; co < 65; co++) {
      b[co] = bPb->data[co];
      for (int ci = 0; ci < 256; ci++) r[ci * 96 + co] = wPb->data[co * 256 + ci];
    }
    for (int co = 0; co < 256; co++)
      for (int ci = 0; ci < 256; ci++) d[ci * 256 + co] = wDb->data[co * 256 + ci];
    ok &= up(s->wPb, r) && up(s->bPb, b) && up(s->wDb, d) && up(s->bDb, bDb->data);
    // fp16 fragments: [N-tile][k-step][lane][8], lane (c, h) holding W[16 t + 8 h + j][32 n + c]
    auto frag = [](const std::vector<float>& wkn, int N, bool lo) {
      std::vector<_Float16> f((size_t)256 * N);
      for (int n = 0; n < N / 32; n++)
        for (int t = 0; t < 16; t++)
          for (int lane = 0; lane < 64; lane++)
            for (int j = 0; j < 8; j++)
              f[(((size_t)n * 16 + t) * 64 + lane) * 8 + j] =
                  half_part(wkn[(size_t)(16 * t + 8 * (lane >> 5) + j) * N + 32 * n + (lane & 31)], lo);
      return f;
    };
    ok &= uph(s->fwPb, frag(r, 96, false)) && uph(s->fwDb, frag(d, 256, false)) && uph(s->lfwPb, frag(r, 96, true)) &&
          uph(s->lfwDb, frag(d, 256, true));
  }
  {  // src/super_point.cpp:148: float(u8) / 255.0 computed in double, stored as float
    std::vector<float> lut(256);
    for (int u = 0; u < 256; u++) lut[u] = (float)(double(u) / 255.0);
    ok &= up(s->lut, lut);
  }
  if (!ok) {
    set_error("weight upload failed");
    rspl_sp_destroy(s);
    return RSPL_E_DEVICE;
  }
  *out = s;
  return RSPL_OK;
}

extern "C" void rspl_sp_destroy(rspl_sp* s) {
  if (!s) return;
  if (s->stream) (void)hipStreamSynchronize(s->stream);
  s->arena.release();
  s->timer.destroy();
  if (s->h_features) (void)hipHostFree(s->h_features);
  if (s->h_counts) (void)hipHostFree(s->h_counts);
  if (s->h_image) (void)hipHostFree(s->h_image);
  if (s->stream) (void)hipStreamDestroy(s->stream);
  delete s;
}

namespace {
// NMS + threshold + borders (superpoint.py:16-33, super_point.cpp:154-183), then top-k
// (super_point.cpp:185-204); stage marks 4 -> 5 -> 6 are the caller's
int nms_topk(rspl_sp* s, int B, int H, int W, int k, hipStream_t st) {
  using namespace sp;
  RSPL_HIP(hipMemsetAsync(s->cand_count, 0, sizeof(int) * B, st));
  NmsArgs n{};  // no NMS'd map: the candidates carry the scores, the samplers read the score map
  n.scores = s->scores; n.nms_out = nullptr; n.cand = s->cand; n.cand_count = s->cand_count; n.cand_cap = s->cand_cap;
  n.H = H; n.W = W; n.threshold = s->cfg.keypoint_threshold; n.border = s->cfg.remove_borders;
  RSPL_HIP(nms(n, B, st));
  s->timer.mark(5, st);
  TopkArgs t{};
  t.cand = s->cand; t.cand_count = s->cand_count; t.cand_cap = s->cand_cap; t.lds_cap = kCandCap; t.k = k;
  t.sel = s->sel; t.sel_count = s->sel_count; t.sel_cap = kCandCap;
  RSPL_HIP(topk(t, B, st));
  return RSPL_OK;
}
}  // namespace

extern "C" int rspl_sp_infer_device(rspl_sp* s, const uint8_t* d_images, int B, int H, int W, int stride,
                                    size_t image_pitch, double* d_features, int capacity, int32_t* d_counts,
                                    void* stream_) {
  RSPL_CHECK_ARG(s && d_images && d_features && d_counts, "rspl_sp_infer_device: NULL argument");
  RSPL_CHECK_ARG(B >= 1 && B <= s->cfg.max_batch, "batch %d outside [1, %d]", B, s->cfg.max_batch);
  RSPL_CHECK_ARG(H > 0 && W > 0 && H % 8 == 0 && W % 8 == 0 && H <= s->cfg.max_height && W <= s->cfg.max_width,
                 "image %dx%d: must be multiples of 8 within %dx%d", H, W, s->cfg.max_height, s->cfg.max_width);
  RSPL_CHECK_ARG(stride >= W, "stride < width");
  const int k = s->cfg.max_keypoints;
  RSPL_CHECK_ARG(capacity >= (k > 0 ? k : kCandCap), "capacity %d below max_keypoints", capacity);
  hipStream_t st = stream_ ? (hipStream_t)stream_ : s->stream;
  const int H2 = H / 2, W2 = W / 2, H4 = H / 4, W4 = W / 4, H8 = H / 8, W8 = W / 8;
  const int P = H8 * W8;
  using namespace sp;
  ConvArgs c{};
  c.img = d_images;
  c.img_stride = stride;
  c.img_pitch = image_pitch;
  c.lut = s->lut;
  c.w1a = s->w1a;
  c.b1a = s->b1a;
  // encoder (superpoint.py:117-127)
  if (s->cfg.precision == RSPL_PREC_FP16X3) {
    // split fp16: every activation a pair of fp16 planes (hi at the buffer's start, lo half a buffer on: the
    // fp32-sized arenas hold both), three MFMA products per step (sp_kernels.hip conv3x3_x3_kernel)
    const size_t act_pl = (size_t)B * H * W * 16, cell_pl = (size_t)B * P * 512;  // halves per lo-plane offset
    _Float16* hA = reinterpret_cast<_Float16*>(s->actA);
    _Float16* hB = reinterpret_cast<_Float16*>(s->actB);
    _Float16* hC = reinterpret_cast<_Float16*>(s->cells);
    auto layer = [&](const _Float16* in, const _Float16* hw, const _Float16* lw, const float* bias, _Float16* out) {
      c.hin = in; c.hin_lo = in ? in + act_pl : nullptr; c.hw = hw; c.hw_lo = lw; c.bias = bias;
      c.hout = out; c.hout_lo = out + (out == hC ? cell_pl : act_pl);
    };
    c.H = H; c.W = W; c.cout = 64;
    layer(nullptr, s->hw1b, s->lw1b, s->b1b, hA);
    RSPL_HIP(conv3x3_x3(c, 64, true, true, B, st, s->timer.slot(0), s->timer.slot(1)));  // conv1a+1b+pool
    c.H = H2; c.W = W2; c.cout = 64; layer(hA, s->hw2a, s->lw2a, s->b2a, hB);
    RSPL_HIP(conv3x3_x3(c, 64, false, false, B, st));                                   // conv2a
    layer(hB, s->hw2b, s->lw2b, s->b2b, hA);
    RSPL_HIP(conv3x3_x3(c, 64, true, false, B, st));                                    // conv2b+pool
    c.H = H4; c.W = W4; c.cout = 128; layer(hA, s->hw3a, s->lw3a, s->b3a, hB);
    RSPL_HIP(conv3x3_x3(c, 64, false, false, B, st));                                   // conv3a
    layer(hB, s->hw3b, s->lw3b, s->b3b, hA);
    RSPL_HIP(conv3x3_x3(c, 128, true, false, B, st));                                   // conv3b+pool
    c.H = H8; c.W = W8; layer(hA, s->hw4a, s->lw4a, s->b4a, hB);
    RSPL_HIP(conv3x3_x3(c, 128, false, false, B, st));                                  // conv4a
    layer(hB, s->hw4b, s->lw4b, s->b4b, hA);
    RSPL_HIP(conv3x3_x3(c, 128, false, false, B, st));                                  // conv4b
    s->timer.mark(2, st);
    c.cout = 512; layer(hA, s->hwPD, s->lwPD, s->bPD, hC);
    RSPL_HIP(conv3x3_x3(c, 128, false, false, B, st));                                  // convPa | convDa
    s->timer.mark(3, st);
    HeadHArgs h{};
    h.cells = hC; h.cells_lo = hC + cell_pl; h.wPb = s->fwPb; h.wPb_lo = s->lfwPb; h.bPb = s->bPb;
    h.scores = s->scores; h.B = B; h.P = P; h.W8 = W8;
    RSPL_HIP(det_head_h(h, true, st));
    s->timer.mark(4, st);
    if (int rc = nms_topk(s, B, H, W, k, st)) return rc;
    s->timer.mark(6, st);
    TapArgs ta{};
    ta.cells = hC; ta.cells_lo = hC + cell_pl; ta.wDb = s->fwDb; ta.wDb_lo = s->lfwDb; ta.bDb = s->bDb;
    ta.sel = s->sel; ta.sel_count = s->sel_count; ta.sel_stride = kCandCap; ta.per_image = (k > 0 ? k : kCandCap);
    ta.nms = s->scores; ta.features = d_features; ta.feat_cap = capacity; ta.counts = d_counts; ta.B = B; ta.H = H; ta.W = W;
    RSPL_HIP(sample_taps_h(ta, true, st));
    s->timer.mark(7, st);
    s->timer.end_call();
    s->last_B = B; s->last_H = H; s->last_W = W;
    return RSPL_OK;
  } else if (s->cfg.precision == RSPL_PREC_FP16) {  // the reference's TensorRT kFP16 engine (super_point.cpp:98)
    _Float16* hA = reinterpret_cast<_Float16*>(s->actA);
    _Float16* hB = reinterpret_cast<_Float16*>(s->actB);
    c.H = H; c.W = W; c.cout = 64; c.hw = s->hw1b; c.bias = s->b1b; c.hout = hA;
    // stage 0 = the fused conv1 kernel exactly (events stamped by the launch itself)
    RSPL_HIP(conv3x3_h(c, 64, true, true, false, B, st, s->timer.slot(0), s->timer.slot(1)));  // conv1a+1b+pool
    c.H = H2; c.W = W2; c.cout = 64; c.hin = hA; c.hw = s->hw2a; c.bias = s->b2a; c.hout = hB;
    RSPL_HIP(conv3x3_h(c, 64, false, false, false, B, st));                   // conv2a
    c.hin = hB; c.hw = s->hw2b; c.bias = s->b2b; c.hout = hA;
    RSPL_HIP(conv3x3_h(c, 64, true, false, false, B, st));                    // conv2b+pool
    c.H = H4; c.W = W4; c.cout = 128; c.hin = hA; c.hw = s->hw3a; c.bias = s->b3a; c.hout = hB;
    RSPL_HIP(conv3x3_h(c, 64, false, false, false, B, st));                   // conv3a
    c.hin = hB; c.hw = s->hw3b; c.bias = s->b3b; c.hout = hA;
    RSPL_HIP(conv3x3_h(c, 128, true, false, false, B, st));                   // conv3b+pool
    c.H = H8; c.W = W8; c.hin = hA; c.hw = s->hw4a; c.bias = s->b4a; c.hout = hB;
    RSPL_HIP(conv3x3_h(c, 128, false, false, false, B, st));                  // conv4a
    c.hin = hB; c.hw = s->hw4b; c.bias = s->b4b; c.hout = hA;
    RSPL_HIP(conv3x3_h(c, 128, false, false, false, B, st));                  // conv4b
    s->timer.mark(2, st);
    c.cout = 512; c.hin = hA; c.hw = s->hwPD; c.bias = s->bPD; c.hout = reinterpret_cast<_Float16*>(s->cells);
    RSPL_HIP(conv3x3_h(c, 128, false, false, false, B, st));                  // convPa | convDa (fp16 out)
    s->timer.mark(3, st);
    // detector head (superpoint.py:130-135) on fp16 MFMA
    HeadHArgs h{};
    h.cells = c.hout; h.wPb = s->fwPb; h.bPb = s->bPb; h.scores = s->scores; h.B = B; h.P = P; h.W8 = W8;
    RSPL_HIP(det_head_h(h, false, st));
    s->timer.mark(4, st);
    if (int rc = nms_topk(s, B, H, W, k, st)) return rc;
    // descriptor head at the sampled taps + sampling + packing (superpoint.py:159-161,
    // super_point.cpp:206-319)
    s->timer.mark(6, st);
    TapArgs ta{};
    ta.cells = c.hout; ta.wDb = s->fwDb; ta.bDb = s->bDb;
    ta.sel = s->sel; ta.sel_count = s->sel_count; ta.sel_stride = kCandCap; ta.per_image = (k > 0 ? k : kCandCap);
    ta.nms = s->scores; ta.features = d_features; ta.feat_cap = capacity; ta.counts = d_counts; ta.B = B; ta.H = H; ta.W = W;
    RSPL_HIP(sample_taps_h(ta, false, st));
    s->timer.mark(7, st);
    s->timer.end_call();
    s->last_B = B; s->last_H = H; s->last_W = W;
    return RSPL_OK;
  } else {
    // encoder (superpoint.py:117-127)
    c.H = H; c.W = W; c.cout = 64; c.w = s->w1b; c.bias = s->b1b; c.out = s->actA;
    RSPL_HIP(conv3x3(c, 64, true, true, B, st, s->timer.slot(0), s->timer.slot(1)));  // conv1a+1b+pool
    c.H = H2; c.W = W2; c.cout = 64; c.in = s->actA; c.w = s->w2a; c.bias = s->b2a; c.out = s->actB;
    RSPL_HIP(conv3x3(c, 64, false, false, B, st));                             // conv2a
    c.in = s->actB; c.w = s->w2b; c.bias = s->b2b; c.out = s->actA;
    RSPL_HIP(conv3x3(c, 64, true, false, B, st));                              // conv2b+pool
    c.H = H4; c.W = W4; c.cout = 128; c.in = s->actA; c.w = s->w3a; c.bias = s->b3a; c.out = s->actB;
    RSPL_HIP(conv3x3(c, 64, false, false, B, st));                             // conv3a
    c.in = s->actB; c.w = s->w3b; c.bias = s->b3b; c.out = s->actA;
    RSPL_HIP(conv3x3(c, 128, true, false, B, st));                             // conv3b+pool
    c.H = H8; c.W = W8; c.in = s->actA; c.w = s->w4a; c.bias = s->b4a; c.out = s->actB;
    RSPL_HIP(conv3x3(c, 128, false, false, B, st));                            // conv4a
    c.in = s->actB; c.w = s->w4b; c.bias = s->b4b; c.out = s->actA;
    RSPL_HIP(conv3x3(c, 128, false, false, B, st));                            // conv4b
    s->timer.mark(2, st);
    c.cout = 512; c.in = s->actA; c.w = s->wPD; c.bias = s->bPD; c.out = s->cells;
    RSPL_HIP(conv3x3(c, 128, false, false, B, st));                            // convPa | convDa
  }
  s->timer.mark(3, st);
  // heads (superpoint.py:130-135, 159-161)
  HeadArgs h{};
  h.in = s->cells; h.B = B; h.P = P; h.W8 = W8;
  h.w = s->wPb; h.bias = s->bPb; h.scores = s->scores;
  RSPL_HIP(heads(h, 0, st));
  h.w = s->wDb; h.bias = s->bDb; h.desc = s->desc;
  RSPL_HIP(heads(h, 1, st));
  s->timer.mark(4, st);
  if (int rc = nms_topk(s, B, H, W, k, st)) return rc;
  // descriptor sampling + packing (super_point.cpp:206-319)
  s->timer.mark(6, st);
  SampleArgs sa{};
  sa.sel = s->sel; sa.sel_count = s->sel_count; sa.sel_stride = kCandCap; sa.per_image = (k > 0 ? k : kCandCap);
  sa.nms = s->scores; sa.desc = s->desc; sa.features = d_features; sa.feat_cap = capacity;
  sa.counts = d_counts; sa.B = B; sa.H = H; sa.W = W;
  RSPL_HIP(sample(sa, st));
  s->timer.mark(7, st);
  s->timer.end_call();
  s->last_B = B; s->last_H = H; s->last_W = W;
  return RSPL_OK;
}

extern "C" int rspl_sp_infer(rspl_sp* s, const uint8_t* image, int H, int W, int stride, double* features,
                             int capacity, int* n_out) {
  RSPL_CHECK_ARG(s && image && features && n_out, "rspl_sp_infer: NULL argument");
  RSPL_CHECK_ARG(H > 0 && W > 0 && H % 8 == 0 && W % 8 == 0 && H <= s->cfg.max_height && W <= s->cfg.max_width,
                 "image %dx%d: must be multiples of 8 within %dx%d", H, W, s->cfg.max_height, s->cfg.max_width);
  RSPL_CHECK_ARG(stride >= W, "stride < width");
  for (int y = 0; y < H; y++) memcpy(s->h_image + (size_t)y * W, image + (size_t)y * stride, W);
  RSPL_HIP(hipMemcpyAsync(s->image, s->h_image, (size_t)H * W, hipMemcpyHostToDevice, s->stream));
  int rc = rspl_sp_infer_device(s, s->image, 1, H, W, W, (size_t)H * W, s->features, s->feat_cap, s->counts, s->stream);
  if (rc) return rc;
  RSPL_HIP(hipMemcpyAsync(s->h_counts, s->counts, sizeof(int32_t), hipMemcpyDeviceToHost, s->stream));
  RSPL_HIP(hipStreamSynchronize(s->stream));
  int cand = 0;
  RSPL_HIP(hipMemcpy(&cand, s->cand_count, sizeof(int), hipMemcpyDeviceToHost));
  if (cand > s->cand_cap) {
    set_error("%d candidates above threshold exceed the candidate buffer %d", cand, s->cand_cap);
    return RSPL_E_CAPACITY;
  }
  if (s->cfg.max_keypoints <= 0 && cand > kCandCap) {
    set_error("keep-all (max_keypoints <= 0): %d candidates exceed %d", cand, kCandCap);
    return RSPL_E_CAPACITY;
  }
  const int n = s->h_counts[0];
  if (n > capacity) {
    set_error("%d keypoints exceed capacity %d", n, capacity);
    return RSPL_E_CAPACITY;
  }
  if (n) {
    RSPL_HIP(hipMemcpyAsync(s->h_features, s->features, sizeof(double) * 259 * n, hipMemcpyDeviceToHost, s->stream));
    RSPL_HIP(hipStreamSynchronize(s->stream));
    memcpy(features, s->h_features, sizeof(double) * 259 * n);
  }
  *n_out = n;
  return RSPL_OK;
}

extern "C" int rspl_sp_debug_maps(rspl_sp* s, int b, float* scores, float* desc) {
  RSPL_CHECK_ARG(s && b >= 0 && b < s->last_B, "no such image in the last batch");
  const int H = s->last_H, W = s->last_W;
  RSPL_HIP(hipStreamSynchronize(s->stream));
  if (scores) {  // the NMS'd map of image b, re-formed from its score map (the product path writes none)
    RSPL_HIP(hipMemsetAsync(s->cand_count, 0, sizeof(int), s->stream));
    sp::NmsArgs n{};
    n.scores = s->scores + (size_t)b * H * W; n.nms_out = s->nms; n.cand = s->cand; n.cand_count = s->cand_count;
    n.cand_cap = s->cand_cap; n.H = H; n.W = W; n.threshold = s->cfg.keypoint_threshold;
    n.border = s->cfg.remove_borders;
    RSPL_HIP(sp::nms(n, 1, s->stream));
    RSPL_HIP(hipMemcpyAsync(scores, s->nms, sizeof(float) * H * W, hipMemcpyDeviceToHost, s->stream));
    RSPL_HIP(hipStreamSynchronize(s->stream));
  }
  if (desc) {
    RSPL_CHECK_ARG(s->cfg.precision == RSPL_PREC_FP32,
                   "RSPL_PREC_FP16 forms descriptors only at the sampled keypoints' taps (no dense map)");
    // device layout [P][256] -> channel-major [256][P] like the reference tensor
    const size_t P = (size_t)H * W / 64;
    std::vector<float> tmp(P * 256);
    RSPL_HIP(hipMemcpy(tmp.data(), s->desc + (size_t)b * P * 256, sizeof(float) * P * 256, hipMemcpyDeviceToHost));
    for (size_t p = 0; p < P; p++)
      for (int c = 0; c < 256; c++) desc[c * P + p] = tmp[p * 256 + c];
  }
  return RSPL_OK;
}

extern "C" int rspl_sp_profile(rspl_sp* s, int enable) {
  RSPL_CHECK_ARG(s, "NULL handle");
  s->timer.reset(enable != 0);
  return RSPL_OK;
}

extern "C" int rspl_sp_stage_times(rspl_sp* s, float* ms, int* calls) {
  RSPL_CHECK_ARG(s && ms, "NULL argument");
  return s->timer.query(ms, calls);
}

extern "C" int rspl_sp_debug_nms(rspl_sp* s, const float* scores, int H, int W, float* out) {
  RSPL_CHECK_ARG(s && scores && out, "rspl_sp_debug_nms: NULL argument");
  RSPL_CHECK_ARG(H > 0 && W > 0 && H <= s->cfg.max_height && W <= s->cfg.max_width, "map %dx%d outside %dx%d", H, W,
                 s->cfg.max_height, s->cfg.max_width);
  hipStream_t st = s->stream;
  RSPL_HIP(hipStreamSynchronize(st));
  RSPL_HIP(hipMemcpyAsync(s->scores, scores, sizeof(float) * H * W, hipMemcpyHostToDevice, st));
  RSPL_HIP(hipMemsetAsync(s->cand_count, 0, sizeof(int), st));
  sp::NmsArgs n{};
  n.scores = s->scores; n.nms_out = s->nms; n.cand = s->cand; n.cand_count = s->cand_count; n.cand_cap = s->cand_cap;
  n.H = H; n.W = W; n.threshold = s->cfg.keypoint_threshold; n.border = s->cfg.remove_borders;
  RSPL_HIP(sp::nms(n, 1, st));
  RSPL_HIP(hipMemcpyAsync(out, s->nms, sizeof(float) * H * W, hipMemcpyDeviceToHost, st));
  RSPL_HIP(hipStreamSynchronize(st));
  s->last_B = 0;
  return RSPL_OK;
}
