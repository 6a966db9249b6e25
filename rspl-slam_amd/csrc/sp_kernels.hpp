#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace rspl {
namespace sp {

struct ConvArgs {
  const float* in;       // NHWC [B][H][W][Cin] (unused when fused with conv1a)
  const float* w;        // [9][Cin][Cout]
  const float* bias;     // [Cout]
  float* out;            // NHWC [B][H(/2)][W(/2)][Cout]
  int H, W, cout;
  int B;                 // images (set by the fp16 launcher: the persistent conv1 walks B x tiles)
  // conv1a fusion (conv1b only)
  const uint8_t* img;    // u8 images, row stride img_stride, image pitch img_pitch
  int img_stride;
  size_t img_pitch;
  const float* lut;      // [256] (float)(u / 255.0)
  const float* w1a;      // [64][9]
  const float* b1a;      // [64]
  // RSPL_PREC_FP16 path (the reference's TensorRT kFP16 engines, super_point.cpp:98):
  // fp16 NHWC activations and weights, fp32 accumulation and epilogue
  const _Float16* hin;   // NHWC [B][H][W][Cin]
  const _Float16* hw;    // [9][Cout][Cin]
  _Float16* hout;        // NHWC [B][H(/2)][W(/2)][Cout] (or `out` in fp32 for the heads)
  // RSPL_PREC_FP16X3 (split fp16, conv3x3_x3): the lo planes of hin / hw / hout (v = hi + lo)
  const _Float16* hin_lo;
  const _Float16* hw_lo;
  _Float16* hout_lo;
};

struct HeadArgs {
  const float* in;       // [B*P][512] (convPa | convDa)
  const float* w;        // [256][NPAD]
  const float* bias;     // [NPAD]
  float* scores;         // mode 0: [B][H][W]
  float* desc;           // mode 1: [B*P][256]
  int B, P, W8;
};

// RSPL_PREC_FP16 heads on v_mfma_f32_32x32x16_f16, weights in B-fragment order
// ([N-tile][k-step][lane][8]: one contiguous 1 KB operand load per wave)
struct HeadHArgs {
  const _Float16* cells; // [B*P][512] (convPa | convDa, ReLU'd, fp16)
  const _Float16* wPb;   // convPb fragments: 3 N-tiles x 16 k-steps (65 real of 96 columns)
  const float* bPb;      // [96]
  float* scores;         // [B][H][W]
  int B, P, W8;
  const _Float16* cells_lo;  // RSPL_PREC_FP16X3: lo planes of cells / wPb
  const _Float16* wPb_lo;
};

struct TapArgs {         // descriptors at the sampled keypoints' bilinear taps only
  const _Float16* cells; // [B*P][512]: convDa at channels 256..511
  const _Float16* wDb;   // convDb fragments: 8 N-tiles x 16 k-steps
  const float* bDb;      // [256]
  const unsigned* sel;
  const int* sel_count;
  int sel_stride;
  int per_image;         // keypoint slots per image (>= max selected)
  const float* nms;      // [B][H][W] score map: a kept keypoint's NMS'd value is its score
  double* features;      // [B][feat_cap][259]
  int feat_cap;
  int32_t* counts;       // [B]
  int B, H, W;
  const _Float16* cells_lo;  // RSPL_PREC_FP16X3: lo planes of cells / wDb
  const _Float16* wDb_lo;
};

struct NmsArgs {
  const float* scores;   // [B][H][W]
  float* nms_out;        // [B][H][W] NMS'd map (debug entry points; null on the product path)
  unsigned long long* cand;  // [B][cand_cap]
  int* cand_count;       // [B]
  int cand_cap;
  int H, W;
  double threshold;
  int border;
  int B;                 // images (set by nms())
};

struct TopkArgs {
  const unsigned long long* cand;
  const int* cand_count;
  int cand_cap;          // candidate buffer stride per image
  int lds_cap;           // candidates sorted whole in LDS; beyond it (k > 0) radix select first
  int k;                 // -1 = keep all
  unsigned* sel;         // [B][sel_cap] flat indices
  int* sel_count;        // [B]
  int sel_cap;
};

struct SampleArgs {
  const unsigned* sel;
  const int* sel_count;
  int sel_stride;        // row stride of sel
  int per_image;         // waves launched per image (>= max selected)
  const float* nms;      // [B][H][W] score map: a kept keypoint's NMS'd value is its score
  const float* desc;     // [B][H/8][W/8][256]
  double* features;      // [B][feat_cap][259]
  int feat_cap;
  int32_t* counts;       // [B]
  int B, H, W;
};

hipError_t conv3x3(const ConvArgs& a, int cin, bool pool, bool fuse1a, int B, hipStream_t s, hipEvent_t t0 = nullptr,
                   hipEvent_t t1 = nullptr);
// fp16 MFMA (v_mfma_f32_32x32x16_f16) variant; out_f32 writes `out` (fp32) instead of `hout`
// t0 / t1 (may be null): events stamped with the fused conv1 kernel's own start / end
hipError_t conv3x3_h(const ConvArgs& a, int cin, bool pool, bool fuse1a, bool out_f32, int B, hipStream_t s,
                     hipEvent_t t0 = nullptr, hipEvent_t t1 = nullptr);
// split-fp16 (RSPL_PREC_FP16X3) variant: hi + lo planes, three MFMA products per k-step
hipError_t conv3x3_x3(const ConvArgs& a, int cin, bool pool, bool fuse1a, int B, hipStream_t s,
                      hipEvent_t t0 = nullptr, hipEvent_t t1 = nullptr);
hipError_t heads(const HeadArgs& a, int mode, hipStream_t s);
hipError_t det_head_h(const HeadHArgs& a, bool x3, hipStream_t s);
hipError_t sample_taps_h(const TapArgs& a, bool x3, hipStream_t s);
hipError_t nms(const NmsArgs& a, int B, hipStream_t s);
hipError_t topk(const TopkArgs& a, int B, hipStream_t s);
hipError_t sample(const SampleArgs& a, hipStream_t s);

}  // namespace sp
}  // namespace rspl
