// SuperPoint forward + post-processing on gfx950 (CDNA4), fp32 MFMA path.
//
// Reference semantics:
//   network  convert2onnx/superpoint.py:114-161  (encoder, detector & descriptor heads)
//   NMS      convert2onnx/superpoint.py:16-33    (simple_nms, radius 4)
//   host     src/super_point.cpp:137-319         (u8/255, threshold, borders, top-k,
//                                                 bilinear sampling in double, packing)
// Layout: activations NHWC fp32 (channels contiguous), one batch of B images.
// Convolutions are implicit GEMMs (M = pixels, N = output channels, K = 9*Cin)
// on v_mfma_f32_32x32x2_f32 (exact fp32: one rounding per product, like fmaf).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdlib>

#include <cstdint>

#include "sp_kernels.hpp"

namespace rspl {
namespace sp {

typedef float floatx16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ floatx16 mfma32(float a, float b, floatx16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// ---------------------------------------------------------------------------
// 3x3 conv, pad 1, bias + ReLU (+ 2x2 max-pool) as an implicit GEMM.
//   block  = 4 waves; tile = TH rows x 16 cols of output pixels x 64 channels
//   wave   = TH/4 rows (TH/8 M-tiles of 2 rows x 16 cols) x 2 N-tiles of 32 ch
//   K loop = Cin in chunks of CK=16, staged in LDS with the 1-pixel halo;
//            weights staged as [9][CK][64].
// FUSE1A: the input tile is conv1a(relu) computed on the fly from the u8
// image (src/super_point.cpp:146-150 normalisation via LUT), so the 64-channel
// full-resolution conv1a map never touches HBM.
// ---------------------------------------------------------------------------
constexpr int CK = 16;
constexpr int CKP = CK + 1;  // LDS pixel stride (odd: conflict-free A reads)
constexpr int TW = 16;

template <int CIN, int TH, bool POOL, bool FUSE1A>
__global__ __launch_bounds__(256) void conv3x3_kernel(ConvArgs a) {
  static_assert(CIN % CK == 0, "Cin must be a multiple of 16");
  constexpr int HX = TW + 2, HY = TH + 2;
  constexpr int MT = TH / 8;  // M-tiles per wave
  __shared__ float halo[HY * HX * CKP];
  __shared__ float wts[9 * CK * 64];
  __shared__ float patch[FUSE1A ? (TH + 4) * (TW + 4) : 1];
  __shared__ float w1a[FUSE1A ? 64 * 10 : 1];

  const int H = a.H, W = a.W, COUT = a.cout;
  const int tiles_x = (W + TW - 1) / TW, tiles_y = (H + TH - 1) / TH;
  const int per_img = tiles_x * tiles_y;
  const int bi = blockIdx.x / per_img;
  const int t = blockIdx.x % per_img;
  const int y0 = (t / tiles_x) * TH, x0 = (t % tiles_x) * TW;
  const int co0 = blockIdx.y * 64;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int ml = lane & 31, kl = lane >> 5;

  if constexpr (FUSE1A) {
    // image patch (TH+4) x (TW+4), rows y0-2.., cols x0-2.., zero outside (conv1a padding)
    const uint8_t* img = a.img + (size_t)bi * a.img_pitch;
    for (int i = tid; i < (TH + 4) * (TW + 4); i += 256) {
      const int py = i / (TW + 4), px = i % (TW + 4);
      const int y = y0 - 2 + py, x = x0 - 2 + px;
      patch[i] = (y >= 0 && y < H && x >= 0 && x < W) ? a.lut[img[(size_t)y * a.img_stride + x]] : 0.f;
    }
    for (int i = tid; i < 64 * 10; i += 256) w1a[i] = (i % 10 < 9) ? a.w1a[(i / 10) * 9 + i % 10] : a.b1a[i / 10];
  }

  floatx16 acc[MT][2];
#pragma unroll
  for (int m = 0; m < MT; m++)
#pragma unroll
    for (int n = 0; n < 2; n++)
#pragma unroll
      for (int r = 0; r < 16; r++) acc[m][n][r] = 0.f;

  for (int c0 = 0; c0 < CIN; c0 += CK) {
    __syncthreads();
    // ---- stage input halo (chunk c0..c0+CK) ----
    if constexpr (FUSE1A) {
      for (int i = tid; i < HY * HX * CK; i += 256) {
        const int c = i % CK, pix = i / CK;
        const int hy = pix / HX, hx = pix % HX;
        const int y = y0 - 1 + hy, x = x0 - 1 + hx;
        float v = 0.f;
        if (y >= 0 && y < H && x >= 0 && x < W) {
          const float* wc = &w1a[(c0 + c) * 10];
          float s = wc[9];
#pragma unroll
          for (int ky = 0; ky < 3; ky++)
#pragma unroll
            for (int kx = 0; kx < 3; kx++) s += wc[ky * 3 + kx] * patch[(hy + ky) * (TW + 4) + hx + kx];
          v = s > 0.f ? s : 0.f;
        }
        halo[pix * CKP + c] = v;
      }
    } else {
      const float* in = a.in + (size_t)bi * H * W * CIN;
      for (int i = tid; i < HY * HX * (CK / 4); i += 256) {
        const int q = i % (CK / 4), pix = i / (CK / 4);
        const int hy = pix / HX, hx = pix % HX;
        const int y = y0 - 1 + hy, x = x0 - 1 + hx;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (y >= 0 && y < H && x >= 0 && x < W)
          v = *reinterpret_cast<const float4*>(in + ((size_t)y * W + x) * CIN + c0 + 4 * q);
        float* d = &halo[pix * CKP + 4 * q];
        d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
      }
    }
    // ---- stage weights [9][CK][64] ----
    for (int i = tid; i < 9 * CK * 16; i += 256) {
      const int n4 = i % 16, r = i / 16;  // r = kk*CK + ci
      const int kk = r / CK, ci = r % CK;
      const float4 v = *reinterpret_cast<const float4*>(a.w + ((size_t)(kk * CIN + c0 + ci)) * COUT + co0 + 4 * n4);
      *reinterpret_cast<float4*>(&wts[r * 64 + 4 * n4]) = v;
    }
    __syncthreads();
    // ---- MFMA over this chunk ----
#pragma unroll
    for (int kk = 0; kk < 9; kk++) {
      const int ky = kk / 3, kx = kk % 3;
#pragma unroll
      for (int kc = 0; kc < CK; kc += 2) {
        float av[MT], bv[2];
#pragma unroll
        for (int m = 0; m < MT; m++) {
          const int ly = wv * (TH / 4) + 2 * m + (ml >> 4);
          av[m] = halo[((ly + ky) * HX + (ml & 15) + kx) * CKP + kc + kl];
        }
#pragma unroll
        for (int n = 0; n < 2; n++) bv[n] = wts[(kk * CK + kc + kl) * 64 + n * 32 + ml];
#pragma unroll
        for (int m = 0; m < MT; m++)
#pragma unroll
          for (int n = 0; n < 2; n++) acc[m][n] = mfma32(av[m], bv[n], acc[m][n]);
      }
    }
  }

  // ---- epilogue: bias + ReLU (+ pool), NHWC store ----
#pragma unroll
  for (int n = 0; n < 2; n++) {
    const int co = co0 + n * 32 + ml;
    const float bias = a.bias[co];
#pragma unroll
    for (int m = 0; m < MT; m++) {
      const int ly = wv * (TH / 4) + 2 * m;  // first of the M-tile's two rows
      if constexpr (POOL) {
        const int H2 = H / 2, W2 = W / 2;
        float* out = a.out + (size_t)bi * H2 * W2 * COUT;
#pragma unroll
        for (int g = 0; g < 4; g++) {
          const int r0 = (g & 1) * 2 + (g >> 1) * 4;
          const int pc = (r0 & 3) + 8 * ((r0 >> 2) & 1) + 4 * kl;
          float v = fmaxf(fmaxf(acc[m][n][r0], acc[m][n][r0 + 1]), fmaxf(acc[m][n][r0 + 8], acc[m][n][r0 + 9]));
          v += bias;
          v = v > 0.f ? v : 0.f;
          const int py = (y0 + ly) >> 1, px = (x0 + pc) >> 1;
          if (py < H2 && px < W2) out[((size_t)py * W2 + px) * COUT + co] = v;
        }
      } else {
        float* out = a.out + (size_t)bi * H * W * COUT;
#pragma unroll
        for (int r = 0; r < 16; r++) {
          const int mm = (r & 3) + 8 * (r >> 2) + 4 * kl;
          const int y = y0 + ly + (mm >> 4), x = x0 + (mm & 15);
          float v = acc[m][n][r] + bias;
          v = v > 0.f ? v : 0.f;
          if (y < H && x < W) out[((size_t)y * W + x) * COUT + co] = v;
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// fp16 variant of the 3x3 conv (RSPL_PREC_FP16 = the reference's TensorRT kFP16
// engines): same tiling, v_mfma_f32_32x32x16_f16 (lane (r, h) holds A[r][8h..8h+7] and
// B[8h..8h+7][r]: one 16-byte LDS read each), 32 input channels per stage, LDS rows of
// 40 halves (80 B: conflict-free ds_read_b128), fp32 accumulation, bias/ReLU/pool epilogue.
// ---------------------------------------------------------------------------
typedef _Float16 half8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ floatx16 mfma16(half8 a, half8 b, floatx16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

constexpr int HCK = 32;       // input channels per stage
constexpr int HCS = HCK + 8;  // LDS row stride in halves

template <int CIN, int TH, bool POOL, bool OUT_F32>
__global__ __launch_bounds__(256) void conv3x3_h_kernel(ConvArgs a) {
  static_assert(CIN % HCK == 0, "Cin must be a multiple of 32");
  constexpr int HX = TW + 2, HY = TH + 2;
  constexpr int MT = TH / 8;
  __shared__ __attribute__((aligned(16))) _Float16 halo[HY * HX * HCS];
  __shared__ __attribute__((aligned(16))) _Float16 wts[9 * 64 * HCS];

  const int H = a.H, W = a.W, COUT = a.cout;
  const int tiles_x = (W + TW - 1) / TW, tiles_y = (H + TH - 1) / TH;
  const int per_img = tiles_x * tiles_y;
  const int co0 = blockIdx.y * 64;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int ml = lane & 31, kl = lane >> 5;

  constexpr int HALO8 = HY * HX * (HCK / 8), HPT = (HALO8 + 255) / 256;
  half8 pw[9], ph[HPT];  // the next stage's weights / halo in flight
  const int tile = blockIdx.x;  // one tile per workgroup (grid = tiles)
  const int bi = tile / per_img;
  const int t = tile % per_img;
  const int y0 = (t / tiles_x) * TH, x0 = (t % tiles_x) * TW;
  floatx16 acc[MT][2];
#pragma unroll
  for (int m = 0; m < MT; m++)
#pragma unroll
    for (int n = 0; n < 2; n++)
#pragma unroll
      for (int r = 0; r < 16; r++) acc[m][n][r] = 0.f;

  // software pipeline over the input-channel stages: the next stage's weights and halo are fetched into
  // registers while the current stage's MFMAs run, and written to LDS after the next barrier
  auto fetch = [&](int c0) {
#pragma unroll
    for (int r = 0; r < 9; r++) {  // weights [9][64 co][32 ci]: 2304 half8, 9 per thread
      const int i = tid + 256 * r, q = i % (HCK / 8), rr = i / (HCK / 8);
      const int kk = rr / 64, co = rr % 64;
      pw[r] = *reinterpret_cast<const half8*>(a.hw + ((size_t)kk * COUT + co0 + co) * CIN + c0 + 8 * q);
    }
    {
      const _Float16* in = a.hin + (size_t)bi * H * W * CIN;
#pragma unroll
      for (int r = 0; r < HPT; r++) {
        const int i = tid + 256 * r, q = i % (HCK / 8), pix = i / (HCK / 8);
        const int hy = pix / HX, hx = pix % HX;
        const int y = y0 - 1 + hy, x = x0 - 1 + hx;
        half8 v = {};
        if (i < HALO8 && y >= 0 && y < H && x >= 0 && x < W)
          v = *reinterpret_cast<const half8*>(in + ((size_t)y * W + x) * CIN + c0 + 8 * q);
        ph[r] = v;
      }
    }
  };
  fetch(0);
  for (int c0 = 0; c0 < CIN; c0 += HCK) {
    __syncthreads();
    {
#pragma unroll
      for (int r = 0; r < HPT; r++) {
        const int i = tid + 256 * r;
        if (i < HALO8) *reinterpret_cast<half8*>(&halo[(i / (HCK / 8)) * HCS + 8 * (i % (HCK / 8))]) = ph[r];
      }
    }
#pragma unroll
    for (int r = 0; r < 9; r++) {
      const int i = tid + 256 * r;
      *reinterpret_cast<half8*>(&wts[(i / (HCK / 8)) * HCS + 8 * (i % (HCK / 8))]) = pw[r];
    }
    __syncthreads();
    if (c0 + HCK < CIN) fetch(c0 + HCK);
#pragma unroll
    for (int kk = 0; kk < 9; kk++) {
      const int ky = kk / 3, kx = kk % 3;
#pragma unroll
      for (int ks = 0; ks < HCK; ks += 16) {
        half8 av[MT], bv[2];
#pragma unroll
        for (int m = 0; m < MT; m++) {
          const int ly = wv * (TH / 4) + 2 * m + (ml >> 4);
          av[m] = *reinterpret_cast<const half8*>(&halo[((ly + ky) * HX + (ml & 15) + kx) * HCS + ks + 8 * kl]);
        }
#pragma unroll
        for (int n = 0; n < 2; n++)
          bv[n] = *reinterpret_cast<const half8*>(&wts[(kk * 64 + n * 32 + ml) * HCS + ks + 8 * kl]);
#pragma unroll
        for (int m = 0; m < MT; m++)
#pragma unroll
          for (int n = 0; n < 2; n++) acc[m][n] = mfma16(av[m], bv[n], acc[m][n]);
      }
    }
  }

  if constexpr (!POOL && !OUT_F32) {
    // full-resolution fp16 output staged through LDS (the weight buffer, free after the last
    // stage) so the global stores are 16-byte rows of 8 channels instead of 2-byte scatters
    constexpr int OS = 72;  // halves per pixel row in LDS (64 channels + pad)
    static_assert(TH * 16 * OS <= 9 * 64 * HCS, "output tile exceeds the weight buffer");
    __syncthreads();
#pragma unroll
    for (int n = 0; n < 2; n++) {
      const float bias = a.bias[co0 + n * 32 + ml];
#pragma unroll
      for (int m = 0; m < MT; m++) {
        const int ly = wv * (TH / 4) + 2 * m;
#pragma unroll
        for (int r = 0; r < 16; r++) {
          const int mm = (r & 3) + 8 * (r >> 2) + 4 * kl;
          const float v = acc[m][n][r] + bias;
          wts[((ly + (mm >> 4)) * 16 + (mm & 15)) * OS + n * 32 + ml] = (_Float16)(v > 0.f ? v : 0.f);
        }
      }
    }
    __syncthreads();
    for (int i = tid; i < TH * 16 * 8; i += 256) {
      const int px = i >> 3, q = i & 7;
      const int y = y0 + (px >> 4), x = x0 + (px & 15);
      if (y < H && x < W)
        *reinterpret_cast<half8*>(a.hout + (size_t)bi * H * W * COUT + ((size_t)y * W + x) * COUT + co0 + 8 * q) =
            *reinterpret_cast<const half8*>(&wts[px * OS + 8 * q]);
    }
    return;
  }
  if constexpr (POOL && !OUT_F32) {
    // 2x2-pooled output tile (TH/2 x 8 pixels x 64 channels) staged through LDS the same way
    constexpr int OS = 72;
    static_assert((TH / 2) * 8 * OS <= 9 * 64 * HCS, "pooled tile exceeds the weight buffer");
    __syncthreads();
#pragma unroll
    for (int n = 0; n < 2; n++) {
      const float bias = a.bias[co0 + n * 32 + ml];
#pragma unroll
      for (int m = 0; m < MT; m++) {
        const int pyl = wv * (TH / 8) + m;  // (wv * TH/4 + 2m) / 2
#pragma unroll
        for (int g = 0; g < 4; g++) {
          const int r0 = (g & 1) * 2 + (g >> 1) * 4;
          const int pc = (r0 & 3) + 8 * ((r0 >> 2) & 1) + 4 * kl;
          float v = fmaxf(fmaxf(acc[m][n][r0], acc[m][n][r0 + 1]), fmaxf(acc[m][n][r0 + 8], acc[m][n][r0 + 9]));
          v += bias;
          wts[(pyl * 8 + (pc >> 1)) * OS + n * 32 + ml] = (_Float16)(v > 0.f ? v : 0.f);
        }
      }
    }
    __syncthreads();
    const int H2 = H / 2, W2 = W / 2;
    for (int i = tid; i < (TH / 2) * 8 * 8; i += 256) {
      const int px = i >> 3, q = i & 7;
      const int py = (y0 >> 1) + (px >> 3), pxx = (x0 >> 1) + (px & 7);
      if (py < H2 && pxx < W2)
        *reinterpret_cast<half8*>(a.hout + (size_t)bi * H2 * W2 * COUT + ((size_t)py * W2 + pxx) * COUT + co0 + 8 * q) =
            *reinterpret_cast<const half8*>(&wts[px * OS + 8 * q]);
    }
    return;
  }
#pragma unroll
  for (int n = 0; n < 2; n++) {
    const int co = co0 + n * 32 + ml;
    const float bias = a.bias[co];
#pragma unroll
    for (int m = 0; m < MT; m++) {
      const int ly = wv * (TH / 4) + 2 * m;
      if constexpr (POOL) {
        const int H2 = H / 2, W2 = W / 2;
#pragma unroll
        for (int g = 0; g < 4; g++) {
          const int r0 = (g & 1) * 2 + (g >> 1) * 4;
          const int pc = (r0 & 3) + 8 * ((r0 >> 2) & 1) + 4 * kl;
          float v = fmaxf(fmaxf(acc[m][n][r0], acc[m][n][r0 + 1]), fmaxf(acc[m][n][r0 + 8], acc[m][n][r0 + 9]));
          v += bias;
          v = v > 0.f ? v : 0.f;
          const int py = (y0 + ly) >> 1, px = (x0 + pc) >> 1;
          if (py < H2 && px < W2) {
            const size_t o = (size_t)bi * H2 * W2 * COUT + ((size_t)py * W2 + px) * COUT + co;
            if constexpr (OUT_F32) a.out[o] = v;
            else a.hout[o] = (_Float16)v;
          }
        }
      } else {
#pragma unroll
        for (int r = 0; r < 16; r++) {
          const int mm = (r & 3) + 8 * (r >> 2) + 4 * kl;
          const int y = y0 + ly + (mm >> 4), x = x0 + (mm & 15);
          float v = acc[m][n][r] + bias;
          v = v > 0.f ? v : 0.f;
          if (y < H && x < W) {
            const size_t o = (size_t)bi * H * W * COUT + ((size_t)y * W + x) * COUT + co;
            if constexpr (OUT_F32) a.out[o] = v;
            else a.hout[o] = (_Float16)v;
          }
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// conv1 (conv1a 1->64 + ReLU + conv1b 64->64 + ReLU + 2x2 max-pool, superpoint.py:120-124) with the
// whole conv1b weight tensor RESIDENT in LDS: one persistent 256-thread workgroup per CU walks 16x16-pixel
// output tiles.  The round-4 per-stage kernel (removed in round 6) restaged each 32-channel half of the weights
// per tile and per stage (two workgroups per CU, 76 KB each, phases separated by barriers: 29 % MFMA-busy SIMD
// time, profiles/r05_experiments.md).  Here per tile: the image patch (prefetched during the previous tile's
// MFMAs) -> LDS; conv1a of all 64 channels on MFMA (transposed product: 8-byte LDS stores) into the halo;
// 144 v_mfma_f32_32x32x16_f16 per wave from LDS; bias + ReLU + pool through LDS to 16-byte stores.
// LDS: weights 9 x 64 x 72 halves (82.9 KB) + halo 18 x 18 x 72 halves (46.7 KB) + patch + conv1a weights.
// The same fp16 roundings of the same fp32 accumulations as that kernel (bitwise equal in round 5's A/B):
// conv1a one MFMA over the 9 taps + bias, conv1b the MFMA k-steps in the same channel order.
// ---------------------------------------------------------------------------
constexpr int C1S = 72;  // LDS row stride (halves) of the weight and halo rows: 64 channels + 8

__global__ __launch_bounds__(256) void conv1_res_kernel(ConvArgs a) {
  constexpr int TH = 16, HX = TW + 2, HY = TH + 2, MT = TH / 8, CIN = 64;
  extern __shared__ __attribute__((aligned(16))) _Float16 c1lds[];
  _Float16* wts = c1lds;                              // [9][64 co][C1S]
  _Float16* halo = wts + 9 * 64 * C1S;                // [HY][HX][C1S]; the pooled output staging afterwards
  float* patch = reinterpret_cast<float*>(halo + HY * HX * C1S);  // [TH + 4][TW + 4]
  float* w1a = patch + (TH + 4) * (TW + 4);           // [64][10] taps + bias

  const int H = a.H, W = a.W;
  const int tiles_x = (W + TW - 1) / TW, tiles_y = (H + TH - 1) / TH;
  const int per_img = tiles_x * tiles_y, ntiles = a.B * per_img;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int ml = lane & 31, kl = lane >> 5;

  constexpr int PP = ((TH + 4) * (TW + 4) + 255) / 256;
  int pv[PP];
  auto load_patch = [&](int tile_) {
    const int bi_ = tile_ / per_img, t_ = tile_ % per_img;
    const int y0_ = (t_ / tiles_x) * TH, x0_ = (t_ % tiles_x) * TW;
    const uint8_t* img = a.img + (size_t)bi_ * a.img_pitch;
#pragma unroll
    for (int r = 0; r < PP; r++) {
      const int i = tid + 256 * r, py = i / (TW + 4), px = i % (TW + 4);
      const int y = y0_ - 2 + py, x = x0_ - 2 + px;
      pv[r] = (i < (TH + 4) * (TW + 4) && tile_ < ntiles && y >= 0 && y < H && x >= 0 && x < W)
                  ? (int)img[(size_t)y * a.img_stride + x]
                  : -1;
    }
  };
  load_patch(blockIdx.x);
  // the workgroup's resident weights: conv1b [9][64 co][64 ci] (16-byte pieces) and conv1a
  for (int i = tid; i < 9 * 64 * 8; i += 256) {
    const int q = i & 7, row = i >> 3;
    *reinterpret_cast<half8*>(&wts[row * C1S + 8 * q]) = *reinterpret_cast<const half8*>(a.hw + (size_t)row * CIN + 8 * q);
  }
  for (int i = tid; i < 64 * 10; i += 256) w1a[i] = (i % 10 < 9) ? a.w1a[(i / 10) * 9 + i % 10] : a.b1a[i / 10];
  __syncthreads();
  // conv1a B operands of the two 32-channel halves (A[c][k]: lane (c, kl) holds k = 8 kl .. 8 kl + 7)
  half8 bw[2];
#pragma unroll
  for (int hf = 0; hf < 2; hf++)
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const int k = 8 * kl + j;
      bw[hf][j] = (_Float16)(k <= 9 ? w1a[(32 * hf + ml) * 10 + k] : 0.f);
    }
  float bias[2];
#pragma unroll
  for (int n = 0; n < 2; n++) bias[n] = a.bias[n * 32 + ml];

  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int bi = tile / per_img, t = tile % per_img;
    const int y0 = (t / tiles_x) * TH, x0 = (t % tiles_x) * TW;
#pragma unroll
    for (int r = 0; r < PP; r++) {  // (every reader of the previous tile's patch and staging has passed a barrier)
      const int i = tid + 256 * r;
      // src/super_point.cpp:146-150 normalisation, (float)(u / 255.0) in double (= the host LUT)
      if (i < (TH + 4) * (TW + 4)) patch[i] = pv[r] >= 0 ? (float)((double)pv[r] / 255.0) : 0.f;
    }
    __syncthreads();
    // conv1a -> ReLU -> fp16 halo, all 64 channels: D[c][px] = W1a[c][k] P[k][px] per halo row and channel half
    {
      const int hx = ml, x = x0 - 1 + hx;
      for (int hy = wv; hy < HY; hy += 4) {
        const int y = y0 - 1 + hy;
        half8 av;
#pragma unroll
        for (int j = 0; j < 8; j++) {
          const int k = 8 * kl + j;
          float v = 0.f;
          if (hx < HX) v = k < 9 ? patch[(hy + k / 3) * (TW + 4) + hx + k % 3] : (k == 9 ? 1.f : 0.f);
          av[j] = (_Float16)v;
        }
        const bool in = y >= 0 && y < H && x >= 0 && x < W;
#pragma unroll
        for (int hf = 0; hf < 2; hf++) {
          floatx16 d;
#pragma unroll
          for (int r = 0; r < 16; r++) d[r] = 0.f;
          d = mfma16(bw[hf], av, d);
          if (hx < HX) {
#pragma unroll
            for (int q = 0; q < 4; q++) {
              typedef _Float16 half4 __attribute__((ext_vector_type(4)));
              half4 h4;
#pragma unroll
              for (int e = 0; e < 4; e++) h4[e] = (_Float16)(in ? fmaxf(d[4 * q + e], 0.f) : 0.f);
              *reinterpret_cast<half4*>(&halo[(hy * HX + hx) * C1S + 32 * hf + 8 * q + 4 * kl]) = h4;
            }
          }
        }
      }
    }
    __syncthreads();
    if (tile + (int)gridDim.x < ntiles) load_patch(tile + gridDim.x);  // in flight during the MFMAs
    floatx16 acc[MT][2];
#pragma unroll
    for (int m = 0; m < MT; m++)
#pragma unroll
      for (int n = 0; n < 2; n++)
#pragma unroll
        for (int r = 0; r < 16; r++) acc[m][n][r] = 0.f;
    // the two 32-channel stages of conv3x3_h_kernel in the same order: stage, tap, k-step
#pragma unroll
    for (int c0 = 0; c0 < CIN; c0 += 32)
#pragma unroll
      for (int kk = 0; kk < 9; kk++) {
        const int ky = kk / 3, kx = kk % 3;
#pragma unroll
        for (int ks = 0; ks < 32; ks += 16) {
          half8 av[MT], bv[2];
#pragma unroll
          for (int m = 0; m < MT; m++) {
            const int ly = wv * (TH / 4) + 2 * m + (ml >> 4);
            av[m] = *reinterpret_cast<const half8*>(&halo[((ly + ky) * HX + (ml & 15) + kx) * C1S + c0 + ks + 8 * kl]);
          }
#pragma unroll
          for (int n = 0; n < 2; n++)
            bv[n] = *reinterpret_cast<const half8*>(&wts[(kk * 64 + n * 32 + ml) * C1S + c0 + ks + 8 * kl]);
#pragma unroll
          for (int m = 0; m < MT; m++)
#pragma unroll
            for (int n = 0; n < 2; n++) acc[m][n] = mfma16(av[m], bv[n], acc[m][n]);
        }
      }
    // bias + ReLU + 2x2 max-pool, the pooled (TH / 2) x 8 x 64 tile staged in LDS (the halo, now free)
    constexpr int OS = 72;
    __syncthreads();
#pragma unroll
    for (int n = 0; n < 2; n++) {
#pragma unroll
      for (int m = 0; m < MT; m++) {
        const int pyl = wv * (TH / 8) + m;
#pragma unroll
        for (int g = 0; g < 4; g++) {
          const int r0 = (g & 1) * 2 + (g >> 1) * 4;
          const int pc = (r0 & 3) + 8 * ((r0 >> 2) & 1) + 4 * kl;
          float v = fmaxf(fmaxf(acc[m][n][r0], acc[m][n][r0 + 1]), fmaxf(acc[m][n][r0 + 8], acc[m][n][r0 + 9]));
          v += bias[n];
          halo[(pyl * 8 + (pc >> 1)) * OS + n * 32 + ml] = (_Float16)(v > 0.f ? v : 0.f);
        }
      }
    }
    __syncthreads();
    const int H2 = H / 2, W2 = W / 2;
    for (int i = tid; i < (TH / 2) * 8 * 8; i += 256) {
      const int px = i >> 3, q = i & 7;
      const int py = (y0 >> 1) + (px >> 3), pxx = (x0 >> 1) + (px & 7);
      if (py < H2 && pxx < W2)
        *reinterpret_cast<half8*>(a.hout + (size_t)bi * H2 * W2 * 64 + ((size_t)py * W2 + pxx) * 64 + 8 * q) =
            *reinterpret_cast<const half8*>(&halo[px * OS + 8 * q]);
    }
  }
}

// ---------------------------------------------------------------------------
// Split-fp16 3x3 conv (RSPL_PREC_FP16X3): fp32-grade accuracy at the fp16 MFMA rate.  Every operand is
// carried as a pair of fp16 planes, v = hi + lo (hi = (half)v, lo = (half)(v - hi): 22 significant bits,
// lo unscaled -- below |v| ~ 0.125 it is subnormal, its absolute error then under 3e-8), and each k-step
// accumulates the three products hi*hi + lo*hi + hi*lo on v_mfma_f32_32x32x16_f16 into ONE fp32
// accumulator (the dropped lo*lo term is 2^-22 relative).  Against the fp32 oracle this keeps SuperPoint's
// keypoint sets identical where the fp16 path loses 1-5 of 400 keypoints per image near the top-k cut
// (tools/sp_fp16_split.py: a CPU emulation of both paths over the C1 images).  Same tiling as
// conv3x3_h_kernel with 16 input channels per stage (LDS: hi + lo halo and weights, 86 KB at TH = 16, so a
// local-BA Schur chunk wave (35 KB) still fits beside a workgroup); conv1a (FUSE1A) runs split on MFMA
// too, from the image in fp32 (u8 / 255 as src/super_point.cpp:146-150) split into hi + lo.
// Output planes: hout (hi) and hout_lo (lo), the same NHWC layout.
// ---------------------------------------------------------------------------
constexpr int XCK = 16;       // input channels per stage
constexpr int XCS = XCK + 8;  // LDS row stride in halves (48-byte rows: conflict-free ds_read_b128)

struct Half2 {
  _Float16 hi, lo;
};
__device__ __forceinline__ Half2 split16(float v) {
  const _Float16 hi = (_Float16)v;
  return {hi, (_Float16)(v - (float)hi)};
}

template <int CIN, int TH, bool POOL, bool FUSE1A>
__global__ __launch_bounds__(256) void conv3x3_x3_kernel(ConvArgs a) {
  static_assert(CIN % 32 == 0, "Cin must be a multiple of 32");
  constexpr int HX = TW + 2, HY = TH + 2, MT = TH / 8;
  constexpr int HALO = HY * HX * XCS, WTS = 9 * 64 * XCS;
  __shared__ __attribute__((aligned(16))) _Float16 halo[2 * HALO];  // [hi | lo]
  __shared__ __attribute__((aligned(16))) _Float16 wts[2 * WTS];    // [hi | lo]: [9][64 co][XCS]
  __shared__ float patch[FUSE1A ? (TH + 4) * (TW + 4) : 1];

  const int H = a.H, W = a.W, COUT = a.cout;
  const int tiles_x = (W + TW - 1) / TW, tiles_y = (H + TH - 1) / TH;
  const int per_img = tiles_x * tiles_y;
  const int bi = blockIdx.x / per_img, t = blockIdx.x % per_img;
  const int y0 = (t / tiles_x) * TH, x0 = (t % tiles_x) * TW;
  const int co0 = blockIdx.y * 64;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int ml = lane & 31, kl = lane >> 5;

  if constexpr (FUSE1A) {
    const uint8_t* img = a.img + (size_t)bi * a.img_pitch;
    for (int i = tid; i < (TH + 4) * (TW + 4); i += 256) {
      const int py = i / (TW + 4), px = i % (TW + 4);
      const int y = y0 - 2 + py, x = x0 - 2 + px;
      // src/super_point.cpp:146-150 normalisation, (float)(u / 255.0) in double (= the host LUT)
      patch[i] = (y >= 0 && y < H && x >= 0 && x < W) ? (float)((double)img[(size_t)y * a.img_stride + x] / 255.0)
                                                      : 0.f;
    }
  }
  floatx16 acc[MT][2];
#pragma unroll
  for (int m = 0; m < MT; m++)
#pragma unroll
    for (int n = 0; n < 2; n++)
#pragma unroll
      for (int r = 0; r < 16; r++) acc[m][n][r] = 0.f;

  // next stage's weights / halo (hi and lo) in registers while the current stage runs on MFMA
  constexpr int W8 = 9 * 64 * (XCK / 8);               // half8 per weight plane per stage
  constexpr int WPT = 2 * W8 / 256;                    // 9
  static_assert(2 * W8 % 256 == 0, "weight staging");
  constexpr int HALO8 = HY * HX * (XCK / 8), HPT = (2 * HALO8 + 255) / 256;
  half8 pw[WPT], ph[FUSE1A ? 1 : HPT];
  auto fetch = [&](int c0) {
#pragma unroll
    for (int r = 0; r < WPT; r++) {
      const int i = tid + 256 * r, pl = i / W8, j = i % W8, q = j % (XCK / 8), rr = j / (XCK / 8);
      const int kk = rr / 64, co = rr % 64;
      pw[r] = *reinterpret_cast<const half8*>((pl ? a.hw_lo : a.hw) + ((size_t)kk * COUT + co0 + co) * CIN + c0 + 8 * q);
    }
    if constexpr (!FUSE1A) {
#pragma unroll
      for (int r = 0; r < HPT; r++) {
        const int i = tid + 256 * r, pl = i / HALO8, j = i % HALO8, q = j % (XCK / 8), pix = j / (XCK / 8);
        const int hy = pix / HX, hx = pix % HX;
        const int y = y0 - 1 + hy, x = x0 - 1 + hx;
        half8 v = {};
        if (i < 2 * HALO8 && y >= 0 && y < H && x >= 0 && x < W)
          v = *reinterpret_cast<const half8*>((pl ? a.hin_lo : a.hin) + (size_t)bi * H * W * CIN +
                                              ((size_t)y * W + x) * CIN + c0 + 8 * q);
        ph[r] = v;
      }
    }
  };
  // conv1a operands (FUSE1A): B[k][c] = W1a[c][k] (k < 9), the bias at k = 9, split hi / lo
  half8 bwh[FUSE1A ? 2 : 1], bwl[FUSE1A ? 2 : 1];
  if constexpr (FUSE1A) {
#pragma unroll
    for (int hf = 0; hf < 2; hf++)
#pragma unroll
      for (int j = 0; j < 8; j++) {
        const int k = 8 * kl + j, c = 32 * hf + ml;
        const Half2 w = split16(k < 9 ? a.w1a[c * 9 + k] : (k == 9 ? a.b1a[c] : 0.f));
        bwh[hf][j] = w.hi;
        bwl[hf][j] = w.lo;
      }
  }
  fetch(0);
  for (int c0 = 0; c0 < CIN; c0 += XCK) {
    __syncthreads();
    if constexpr (FUSE1A) {
      // conv1a -> ReLU for channels c0 .. c0 + 15 of the halo: the transposed product D[c][px] =
      // W1a[c][k] P[k][px] of the 32-channel half holding them (lane (px, kl) gets channels 8 q + 4 kl + e;
      // this stage keeps q = 2 (c0 % 32 / 16), + 1), three products per MFMA step
      const int hf = (c0 % 64) / 32, q0 = 2 * ((c0 % 32) / 16);
      const int hx = ml, x = x0 - 1 + hx;
      for (int hy = wv; hy < HY; hy += 4) {
        const int y = y0 - 1 + hy;
        half8 ah, al;
#pragma unroll
        for (int j = 0; j < 8; j++) {
          const int k = 8 * kl + j;
          float v = 0.f;
          if (hx < HX) v = k < 9 ? patch[(hy + k / 3) * (TW + 4) + hx + k % 3] : (k == 9 ? 1.f : 0.f);
          const Half2 p = split16(v);
          ah[j] = p.hi;
          al[j] = p.lo;
        }
        floatx16 d;
#pragma unroll
        for (int r = 0; r < 16; r++) d[r] = 0.f;
        d = mfma16(bwh[hf], ah, d);
        d = mfma16(bwh[hf], al, d);
        d = mfma16(bwl[hf], ah, d);
        const bool in = y >= 0 && y < H && x >= 0 && x < W;
        if (hx < HX) {
#pragma unroll
          for (int qq = 0; qq < 2; qq++) {
            typedef _Float16 half4 __attribute__((ext_vector_type(4)));
            half4 h4, l4;
#pragma unroll
            for (int e = 0; e < 4; e++) {
              const Half2 p = split16(in ? fmaxf(d[4 * (q0 + qq) + e], 0.f) : 0.f);
              h4[e] = p.hi;
              l4[e] = p.lo;
            }
            const int o = (hy * HX + hx) * XCS + 8 * qq + 4 * kl;
            *reinterpret_cast<half4*>(&halo[o]) = h4;
            *reinterpret_cast<half4*>(&halo[HALO + o]) = l4;
          }
        }
      }
    } else {
#pragma unroll
      for (int r = 0; r < HPT; r++) {
        const int i = tid + 256 * r, pl = i / HALO8, j = i % HALO8;
        if (i < 2 * HALO8) *reinterpret_cast<half8*>(&halo[pl * HALO + (j / (XCK / 8)) * XCS + 8 * (j % (XCK / 8))]) = ph[r];
      }
    }
#pragma unroll
    for (int r = 0; r < WPT; r++) {
      const int i = tid + 256 * r, pl = i / W8, j = i % W8;
      *reinterpret_cast<half8*>(&wts[pl * WTS + (j / (XCK / 8)) * XCS + 8 * (j % (XCK / 8))]) = pw[r];
    }
    __syncthreads();
    if (c0 + XCK < CIN) fetch(c0 + XCK);
#pragma unroll
    for (int kk = 0; kk < 9; kk++) {
      const int ky = kk / 3, kx = kk % 3;
      half8 ah[MT], al[MT], bh[2], bl[2];
#pragma unroll
      for (int m = 0; m < MT; m++) {
        const int ly = wv * (TH / 4) + 2 * m + (ml >> 4);
        const int o = ((ly + ky) * HX + (ml & 15) + kx) * XCS + 8 * kl;
        ah[m] = *reinterpret_cast<const half8*>(&halo[o]);
        al[m] = *reinterpret_cast<const half8*>(&halo[HALO + o]);
      }
#pragma unroll
      for (int n = 0; n < 2; n++) {
        const int o = (kk * 64 + n * 32 + ml) * XCS + 8 * kl;
        bh[n] = *reinterpret_cast<const half8*>(&wts[o]);
        bl[n] = *reinterpret_cast<const half8*>(&wts[WTS + o]);
      }
      // the three products in three sweeps over the (m, n) accumulators: consecutive MFMAs independent
#pragma unroll
      for (int m = 0; m < MT; m++)
#pragma unroll
        for (int n = 0; n < 2; n++) acc[m][n] = mfma16(al[m], bh[n], acc[m][n]);
#pragma unroll
      for (int m = 0; m < MT; m++)
#pragma unroll
        for (int n = 0; n < 2; n++) acc[m][n] = mfma16(ah[m], bl[n], acc[m][n]);
#pragma unroll
      for (int m = 0; m < MT; m++)
#pragma unroll
        for (int n = 0; n < 2; n++) acc[m][n] = mfma16(ah[m], bh[n], acc[m][n]);
    }
  }

  // epilogue: bias + ReLU (+ 2x2 max-pool), split into hi / lo, staged through LDS (the weight buffer) so
  // the global stores are 16-byte rows of 8 channels
  constexpr int OS = 72;  // halves per pixel row in LDS (64 channels + pad)
  constexpr int OPIX = POOL ? (TH / 2) * 8 : TH * 16;
  static_assert((POOL ? 2 : 1) * OPIX * OS <= 2 * WTS, "output tile exceeds the weight buffer");
  float bias[2];
#pragma unroll
  for (int n = 0; n < 2; n++) bias[n] = a.bias[co0 + n * 32 + ml];
  const int Ho = POOL ? H / 2 : H, Wo = POOL ? W / 2 : W;
  // POOL: both planes staged at once; otherwise hi, then lo (each fills most of the buffer)
#pragma unroll
  for (int pass = 0; pass < (POOL ? 1 : 2); pass++) {
    __syncthreads();
#pragma unroll
    for (int n = 0; n < 2; n++)
#pragma unroll
      for (int m = 0; m < MT; m++) {
        if constexpr (POOL) {
          const int pyl = wv * (TH / 8) + m;
#pragma unroll
          for (int g = 0; g < 4; g++) {
            const int r0 = (g & 1) * 2 + (g >> 1) * 4;
            const int pc = (r0 & 3) + 8 * ((r0 >> 2) & 1) + 4 * kl;
            float v = fmaxf(fmaxf(acc[m][n][r0], acc[m][n][r0 + 1]), fmaxf(acc[m][n][r0 + 8], acc[m][n][r0 + 9]));
            v += bias[n];
            const Half2 p = split16(v > 0.f ? v : 0.f);
            const int o = (pyl * 8 + (pc >> 1)) * OS + n * 32 + ml;
            wts[o] = p.hi;
            wts[OPIX * OS + o] = p.lo;
          }
        } else {
          const int ly = wv * (TH / 4) + 2 * m;
#pragma unroll
          for (int r = 0; r < 16; r++) {
            const int mm = (r & 3) + 8 * (r >> 2) + 4 * kl;
            const float v = acc[m][n][r] + bias[n];
            const Half2 p = split16(v > 0.f ? v : 0.f);
            wts[((ly + (mm >> 4)) * 16 + (mm & 15)) * OS + n * 32 + ml] = pass ? p.lo : p.hi;
          }
        }
      }
    __syncthreads();
#pragma unroll
    for (int pl = 0; pl < (POOL ? 2 : 1); pl++) {
      _Float16* out = (POOL ? (pl ? a.hout_lo : a.hout) : (pass ? a.hout_lo : a.hout)) + (size_t)bi * Ho * Wo * COUT;
      for (int i = tid; i < OPIX * 8; i += 256) {
        const int px = i >> 3, q = i & 7;
        const int y = POOL ? (y0 >> 1) + (px >> 3) : y0 + (px >> 4);
        const int x = POOL ? (x0 >> 1) + (px & 7) : x0 + (px & 15);
        if (y < Ho && x < Wo)
          *reinterpret_cast<half8*>(out + ((size_t)y * Wo + x) * COUT + co0 + 8 * q) =
              *reinterpret_cast<const half8*>(&wts[pl * OPIX * OS + px * OS + 8 * q]);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// 1x1 heads on the H/8 x W/8 cell grid.  in = [P][512] (convPa | convDa, ReLU'd).
//   MODE 0: convPb 256->65, softmax over 65, drop dustbin, depth-to-space ->
//           scores [H][W]  (superpoint.py:131-135)
//   MODE 1: convDb 256->256, per-cell L2 normalise -> desc [P][256]
//           (superpoint.py:160-161)
// One wave owns 32 cells; block = 4 waves = 128 cells.  K = 256 staged in LDS
// in chunks of 32.  Weights pre-transposed to [256][NPAD] (NPAD = 96 / 256).
// ---------------------------------------------------------------------------
template <int MODE>
__global__ __launch_bounds__(256) void head_kernel(HeadArgs a) {
  constexpr int NT = MODE == 0 ? 3 : 8;  // N-tiles of 32
  constexpr int NP = NT * 32;
  constexpr int KC = 32;
  __shared__ float As[KC][128 + 1];
  __shared__ float Bs[KC][NP];
  const int P = a.P;  // cells per image
  const int cell0 = blockIdx.x * 128;  // flattened over batch
  const int total = a.B * P;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, ml = lane & 31, kl = lane >> 5;
  const int in_off = MODE == 0 ? 0 : 256;

  floatx16 acc[NT];
#pragma unroll
  for (int n = 0; n < NT; n++)
#pragma unroll
    for (int r = 0; r < 16; r++) acc[n][r] = 0.f;

  for (int k0 = 0; k0 < 256; k0 += KC) {
    __syncthreads();
    for (int i = tid; i < 128 * (KC / 4); i += 256) {
      const int q = i % (KC / 4), c = i / (KC / 4);
      const int cell = cell0 + c;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (cell < total) v = *reinterpret_cast<const float4*>(a.in + (size_t)cell * 512 + in_off + k0 + 4 * q);
      As[4 * q + 0][c] = v.x; As[4 * q + 1][c] = v.y; As[4 * q + 2][c] = v.z; As[4 * q + 3][c] = v.w;
    }
    for (int i = tid; i < KC * (NP / 4); i += 256) {
      const int q = i % (NP / 4), k = i / (NP / 4);
      *reinterpret_cast<float4*>(&Bs[k][4 * q]) = *reinterpret_cast<const float4*>(a.w + (size_t)(k0 + k) * NP + 4 * q);
    }
    __syncthreads();
#pragma unroll 4
    for (int kc = 0; kc < KC; kc += 2) {
      const float av = As[kc + kl][wv * 32 + ml];
#pragma unroll
      for (int n = 0; n < NT; n++) acc[n] = mfma32(av, Bs[kc + kl][n * 32 + ml], acc[n]);
    }
  }

  // epilogue: rows (cells) on registers, channels on lanes (col = ml within N-tile)
#pragma unroll
  for (int n = 0; n < NT; n++) {
    const float b = a.bias[n * 32 + ml];
#pragma unroll
    for (int r = 0; r < 16; r++) acc[n][r] += b;
  }
  if constexpr (MODE == 0) {
    // channels >= 65 are padding: exclude from the softmax
#pragma unroll
    for (int r = 0; r < 16; r++) {
      float m = -INFINITY;
#pragma unroll
      for (int n = 0; n < NT; n++) {
        const int c = n * 32 + ml;
        if (c < 65) m = fmaxf(m, acc[n][r]);
      }
#pragma unroll
      for (int o = 16; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 32));
      float e[NT];
      float s = 0.f;
#pragma unroll
      for (int n = 0; n < NT; n++) {
        const int c = n * 32 + ml;
        e[n] = (c < 65) ? expf(acc[n][r] - m) : 0.f;
        s += e[n];
      }
#pragma unroll
      for (int o = 16; o >= 1; o >>= 1) s += __shfl_xor(s, o, 32);
      const int cell = cell0 + wv * 32 + (r & 3) + 8 * (r >> 2) + 4 * kl;
      if (cell < total) {
        const int bi = cell / P, p = cell % P;
        const int cy = p / a.W8, cx = p % a.W8;
        float* sc = a.scores + (size_t)bi * P * 64;
        const int Wf = a.W8 * 8;
#pragma unroll
        for (int n = 0; n < 2; n++) {  // channels 0..63 live in N-tiles 0,1
          const int c = n * 32 + ml;
          sc[(size_t)(cy * 8 + (c >> 3)) * Wf + cx * 8 + (c & 7)] = e[n] / s;
        }
      }
    }
  } else {
#pragma unroll
    for (int r = 0; r < 16; r++) {
      float s = 0.f;
#pragma unroll
      for (int n = 0; n < NT; n++) s += acc[n][r] * acc[n][r];
#pragma unroll
      for (int o = 16; o >= 1; o >>= 1) s += __shfl_xor(s, o, 32);
      float nrm = sqrtf(s);
      nrm = nrm < 1e-12f ? 1e-12f : nrm;
      const int cell = cell0 + wv * 32 + (r & 3) + 8 * (r >> 2) + 4 * kl;
      if (cell < total) {
#pragma unroll
        for (int n = 0; n < NT; n++) a.desc[(size_t)cell * 256 + n * 32 + ml] = acc[n][r] / nrm;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// RSPL_PREC_FP16 heads.  The fp16 convPa | convDa map ([P][512] halves) is read straight into
// v_mfma_f32_32x32x16_f16 A operands (lane (r, h): cell r, channels 16t + 8h .. +7); the 1x1
// weights come from L2 in B-fragment order, so neither head stages anything through LDS.
//   det_head_h:    convPb 256->65, softmax over 65, dustbin dropped, depth-to-space
//                  (superpoint.py:131-135); one wave per 32 cells.
//   sample_taps_h: convDb 256->256 + per-cell L2 normalise (superpoint.py:160-161) evaluated
//                  only at the 4 bilinear taps of each selected keypoint (the dense map is never
//                  formed: the 1x1 conv and the per-cell normalise are pointwise, so this is the
//                  same function), then the double-precision bilinear sample and renormalise of
//                  src/super_point.cpp:206-319.  A workgroup takes 8 keypoints = 32 tap rows
//                  (one M-tile); wave w owns output channels 64w .. 64w+63.
// ---------------------------------------------------------------------------
// X3 (RSPL_PREC_FP16X3): cells and weights as hi + lo fp16 planes, three products per MFMA step (the split
// arithmetic of conv3x3_x3_kernel)
template <bool X3>
__global__ __launch_bounds__(256) void det_head_h_kernel(HeadHArgs a) {
  constexpr int NT = 3;  // 96 columns, 65 real
  const int total = a.B * a.P;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, ml = lane & 31, kl = lane >> 5;
  const int base = (blockIdx.x * 4 + wv) * 32;
  if (base >= total) return;  // per wave: no barriers below
  const size_t ro = (size_t)min(base + ml, total - 1) * 512 + 8 * kl;
  half8 av[16], al[X3 ? 16 : 1];
#pragma unroll
  for (int t = 0; t < 16; t++) av[t] = *reinterpret_cast<const half8*>(a.cells + ro + 16 * t);
  if constexpr (X3)
#pragma unroll
    for (int t = 0; t < 16; t++) al[t] = *reinterpret_cast<const half8*>(a.cells_lo + ro + 16 * t);
  floatx16 acc[NT];
#pragma unroll
  for (int n = 0; n < NT; n++)
#pragma unroll
    for (int r = 0; r < 16; r++) acc[n][r] = 0.f;
  const half8* wf = reinterpret_cast<const half8*>(a.wPb) + lane;
  const half8* wfl = reinterpret_cast<const half8*>(a.wPb_lo) + lane;
#pragma unroll
  for (int t = 0; t < 16; t++) {
    half8 bv[NT], bl[X3 ? NT : 1];
#pragma unroll
    for (int n = 0; n < NT; n++) bv[n] = wf[(n * 16 + t) * 64];
    if constexpr (X3)
#pragma unroll
      for (int n = 0; n < NT; n++) bl[n] = wfl[(n * 16 + t) * 64];
    if constexpr (X3) {
#pragma unroll
      for (int n = 0; n < NT; n++) acc[n] = mfma16(al[t], bv[n], acc[n]);
#pragma unroll
      for (int n = 0; n < NT; n++) acc[n] = mfma16(av[t], bl[n], acc[n]);
    }
#pragma unroll
    for (int n = 0; n < NT; n++) acc[n] = mfma16(av[t], bv[n], acc[n]);
  }
#pragma unroll
  for (int n = 0; n < NT; n++) {
    const float b = a.bPb[n * 32 + ml];
#pragma unroll
    for (int r = 0; r < 16; r++) acc[n][r] += b;
  }
  const int Wf = a.W8 * 8;
  // the wave's 32 cells x 64 scores go through LDS, then out as rows of the full-resolution map
  // (lanes = consecutive cells of one pixel row: 32-byte pieces side by side) instead of 4-byte
  // scatters into 8 rows per cell
  __shared__ __attribute__((aligned(16))) float stage[4][32][65];
  float(*sg)[65] = stage[wv];
#pragma unroll
  for (int r = 0; r < 16; r++) {
    float m = -INFINITY;
#pragma unroll
    for (int n = 0; n < NT; n++)
      if (n * 32 + ml < 65) m = fmaxf(m, acc[n][r]);
#pragma unroll
    for (int o = 16; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 32));
    float e[NT], sum = 0.f;
#pragma unroll
    for (int n = 0; n < NT; n++) {
      e[n] = (n * 32 + ml < 65) ? expf(acc[n][r] - m) : 0.f;
      sum += e[n];
    }
#pragma unroll
    for (int o = 16; o >= 1; o >>= 1) sum += __shfl_xor(sum, o, 32);
    const int cl = (r & 3) + 8 * (r >> 2) + 4 * kl;
#pragma unroll
    for (int n = 0; n < 2; n++) sg[cl][n * 32 + ml] = e[n] / sum;  // channels 0..63 (dustbin dropped)
  }
  __builtin_amdgcn_wave_barrier();  // LDS in program order within the wave
  for (int i = lane; i < 32 * 8 * 2; i += 64) {  // (pixel row pr, cell j, half h): 4 floats each
    const int pr = i >> 6, j = (i >> 1) & 31, hh = i & 1;
    const int cell = base + j;
    if (cell >= total) continue;
    const int bi = cell / a.P, p = cell % a.P;
    const int cy = p / a.W8, cx = p % a.W8;
    const float* src = &sg[j][pr * 8 + 4 * hh];
    *reinterpret_cast<float4*>(a.scores + (size_t)bi * a.P * 64 + (size_t)(cy * 8 + pr) * Wf + cx * 8 + 4 * hh) =
        make_float4(src[0], src[1], src[2], src[3]);
  }
}

template <bool X3>
__global__ __launch_bounds__(256) void sample_taps_h_kernel(TapArgs a) {
  __shared__ int tcell[32];      // tap row 4 kp + q: cell of tap q (nw, ne, sw, se) of keypoint kp
  __shared__ double twt[32];     // its bilinear weight
  __shared__ float part[4][32];  // per-wave partial sums of squares per tap row
  __shared__ double part2[4][8]; // per-wave partial sums of squares per keypoint
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, ml = lane & 31, kl = lane >> 5;
  const int bpi = (a.per_image + 7) / 8;
  const int bi = blockIdx.x / bpi, i0 = (blockIdx.x % bpi) * 8;
  if (bi >= a.B) return;
  const int n = a.sel_count[bi];
  if (tid == 0 && i0 == 0) a.counts[bi] = n;
  if (i0 >= n) return;  // uniform over the workgroup
  const int H = a.H, W = a.W, h = H / 8, w = W / 8, P = h * w;
  if (tid < 8) {
    const int i = i0 + tid;
    int c[4] = {0, 0, 0, 0};
    double wt[4] = {0, 0, 0, 0};
    if (i < n) {
      const unsigned flat = a.sel[(size_t)bi * a.sel_stride + i];
      const int y = flat / W, x = flat % W;
      // normalize_keypoints (:276-287; s/2 is integer division) and grid_sample (:294-332)
      const double gx = ((double)x - 8 / 2 + 0.5) / (w * 8 - 8 / 2 - 0.5) * 2 - 1;
      const double gy = ((double)y - 8 / 2 + 0.5) / (h * 8 - 8 / 2 - 0.5) * 2 - 1;
      const double ix = ((gx + 1) / 2) * (w - 1), iy = ((gy + 1) / 2) * (h - 1);
      auto clip = [](int v, int m) { return v < 0 ? 0 : (v < m - 1 ? v : m - 1); };
      const int ix_nw = clip((int)floor(ix), w), iy_nw = clip((int)floor(iy), h);
      const int ix_ne = clip(ix_nw + 1, w), iy_ne = clip(iy_nw, h);
      const int ix_sw = clip(ix_nw, w), iy_sw = clip(iy_nw + 1, h);
      const int ix_se = clip(ix_nw + 1, w), iy_se = clip(iy_nw + 1, h);
      wt[0] = (ix_se - ix) * (iy_se - iy);
      wt[1] = (ix - ix_sw) * (iy_sw - iy);
      wt[2] = (ix_ne - ix) * (iy - iy_ne);
      wt[3] = (ix - ix_nw) * (iy - iy_nw);
      c[0] = iy_nw * w + ix_nw;
      c[1] = iy_ne * w + ix_ne;
      c[2] = iy_sw * w + ix_sw;
      c[3] = iy_se * w + ix_se;
      double* f = a.features + ((size_t)bi * a.feat_cap + i) * 259;
      f[0] = (double)a.nms[(size_t)bi * H * W + flat];
      f[1] = (double)x;
      f[2] = (double)y;
    }
#pragma unroll
    for (int q = 0; q < 4; q++) {
      tcell[4 * tid + q] = c[q];
      twt[4 * tid + q] = wt[q];
    }
  }
  __syncthreads();
  const size_t ro = ((size_t)bi * P + tcell[ml]) * 512 + 256 + 8 * kl;
  half8 av[16], al[X3 ? 16 : 1];
#pragma unroll
  for (int t = 0; t < 16; t++) av[t] = *reinterpret_cast<const half8*>(a.cells + ro + 16 * t);
  if constexpr (X3)
#pragma unroll
    for (int t = 0; t < 16; t++) al[t] = *reinterpret_cast<const half8*>(a.cells_lo + ro + 16 * t);
  floatx16 acc[2];
#pragma unroll
  for (int j = 0; j < 2; j++)
#pragma unroll
    for (int r = 0; r < 16; r++) acc[j][r] = 0.f;
  const half8* wf = reinterpret_cast<const half8*>(a.wDb) + lane;
  const half8* wfl = reinterpret_cast<const half8*>(a.wDb_lo) + lane;
#pragma unroll
  for (int t = 0; t < 16; t++) {
    const half8 b0 = wf[((2 * wv) * 16 + t) * 64], b1 = wf[((2 * wv + 1) * 16 + t) * 64];
    if constexpr (X3) {
      const half8 l0 = wfl[((2 * wv) * 16 + t) * 64], l1 = wfl[((2 * wv + 1) * 16 + t) * 64];
      acc[0] = mfma16(al[t], b0, acc[0]);
      acc[1] = mfma16(al[t], b1, acc[1]);
      acc[0] = mfma16(av[t], l0, acc[0]);
      acc[1] = mfma16(av[t], l1, acc[1]);
    }
    acc[0] = mfma16(av[t], b0, acc[0]);
    acc[1] = mfma16(av[t], b1, acc[1]);
  }
  // bias; per tap row (register r, lane half kl: row (r & 3) + 8 (r >> 2) + 4 kl) the sum of
  // squares over this wave's 64 channels, then over the 4 waves in a fixed order
  const float bias0 = a.bDb[64 * wv + ml], bias1 = a.bDb[64 * wv + 32 + ml];
  float ss[16];
#pragma unroll
  for (int r = 0; r < 16; r++) {
    acc[0][r] += bias0;
    acc[1][r] += bias1;
    ss[r] = acc[0][r] * acc[0][r] + acc[1][r] * acc[1][r];
  }
#pragma unroll
  for (int o = 16; o >= 1; o >>= 1)
#pragma unroll
    for (int r = 0; r < 16; r++) ss[r] += __shfl_xor(ss[r], o, 32);
  if (ml == 0)
#pragma unroll
    for (int r = 0; r < 16; r++) part[wv][(r & 3) + 8 * (r >> 2) + 4 * kl] = ss[r];
  __syncthreads();
  // keypoint kp = 2 q + kl holds its taps in registers 4q .. 4q+3 (nw, ne, sw, se)
  double v[4][2], s2[4];
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const int kp = 2 * q + kl;
    double vv0 = 0, vv1 = 0;
#pragma unroll
    for (int tp = 0; tp < 4; tp++) {
      const int rw = 4 * kp + tp;
      float nrm = sqrtf(((part[0][rw] + part[1][rw]) + part[2][rw]) + part[3][rw]);
      nrm = nrm < 1e-12f ? 1e-12f : nrm;
      const double wt = twt[rw];
      vv0 += (double)(acc[0][4 * q + tp] / nrm) * wt;
      vv1 += (double)(acc[1][4 * q + tp] / nrm) * wt;
    }
    v[q][0] = vv0;
    v[q][1] = vv1;
    s2[q] = vv0 * vv0 + vv1 * vv1;
  }
#pragma unroll
  for (int o = 16; o >= 1; o >>= 1)
#pragma unroll
    for (int q = 0; q < 4; q++) s2[q] += __shfl_xor(s2[q], o, 32);
  if (ml == 0)
#pragma unroll
    for (int q = 0; q < 4; q++) part2[wv][2 * q + kl] = s2[q];
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const int kp = 2 * q + kl, i = i0 + kp;
    if (i >= n) continue;
    const double inv = 1.0 / sqrt(((part2[0][kp] + part2[1][kp]) + part2[2][kp]) + part2[3][kp]);
    double* f = a.features + ((size_t)bi * a.feat_cap + i) * 259 + 3 + 64 * wv + ml;
    f[0] = inv * v[q][0];
    f[32] = inv * v[q][1];
  }
}

// ---------------------------------------------------------------------------
// Fused simple_nms (5 x 9x9 max-pools) + threshold / border candidate extraction.  Scores are
// softmax outputs (>= 0) and every window contains its centre, so zero padding outside the image
// equals MaxPool2d's -inf padding here.  Tile 64 x 32 outputs with the 20-pixel halo the five
// dependent pools need (104 x 72 in LDS).  Each 1-D pass gives a thread 8 consecutive outputs
// from 16 register-held inputs (van Herk / Gil-Werman with block 8: suffix maxima of the first 8,
// prefix maxima of the second, out[i] = max(suffix[i], prefix[i]) = the 9-window [i, i+8]): 2 LDS
// reads per output instead of 9.  Passes run over the whole region; values near its border are
// garbage that never reaches the output tile (each pool shrinks the valid region by 4, five pools =
// the 20-pixel halo).
// LDS: 10 bytes per region pixel (74.9 KB: two workgroups per CU, every tile of a C3 step in one
// dispatch round) -- scores S and the row-pass scratch T in fp32, max_mask K and supp_mask M in
// bytes; the two mask pools run on bytes (T reused as u8), supp_scores = M ? 0 : S is formed on the
// fly by the score pools.  XCD-aware placement: tile order is row-major per image and the tiles are
// dealt to the 8 XCDs in contiguous bands (blockIdx % 8 = XCD), so the halo rows a tile shares with
// its vertical neighbours are fetched once into that XCD's L2, not once per XCD.
// ---------------------------------------------------------------------------
constexpr int NTX = 64, NTY = 32, NH = 20, RX = NTX + 2 * NH, RY = NTY + 2 * NH;  // 104 x 72
static_assert(RX % 8 == 0 && (RX - 8) % 8 == 0 && (RY - 8) % 8 == 0, "8-output chunks tile the passes");

// 9-window max of 16 register values: out[i] = max(v[i .. i+8]), i < 8
template <typename V>
__device__ __forceinline__ void window9(const V (&v)[16], V (&o)[8]) {
  V suf[8], pre[8];
  suf[7] = v[7];
#pragma unroll
  for (int i = 6; i >= 0; i--) suf[i] = v[i] > suf[i + 1] ? v[i] : suf[i + 1];
  pre[0] = v[8];
#pragma unroll
  for (int i = 1; i < 8; i++) pre[i] = v[8 + i] > pre[i - 1] ? v[8 + i] : pre[i - 1];
#pragma unroll
  for (int i = 0; i < 8; i++) o[i] = suf[i] > pre[i] ? suf[i] : pre[i];
}
__device__ __forceinline__ void window9f(const float (&v)[16], float (&o)[8]) {
  float suf[8], pre[8];
  suf[7] = v[7];
#pragma unroll
  for (int i = 6; i >= 0; i--) suf[i] = fmaxf(v[i], suf[i + 1]);
  pre[0] = v[8];
#pragma unroll
  for (int i = 1; i < 8; i++) pre[i] = fmaxf(pre[i - 1], v[8 + i]);
#pragma unroll
  for (int i = 0; i < 8; i++) o[i] = fmaxf(suf[i], pre[i]);
}
// dst[y][x] = max_{|k|<=4} src'[y][x+k] for every row, x in [4, RX-4), src' = M ? 0 : S when SUPP
template <bool SUPP>
__device__ __forceinline__ void rowpass9(const float* S, const unsigned char* M, float* dst) {
  constexpr int CPR = (RX - 8) / 8;
  for (int c = threadIdx.x; c < CPR * RY; c += blockDim.x) {
    const int y = c / CPR, x0 = 4 + 8 * (c % CPR), b = y * RX + x0 - 4;
    const float4* p = reinterpret_cast<const float4*>(S + b);
    float v[16];
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const float4 t = p[q];
      v[4 * q] = t.x; v[4 * q + 1] = t.y; v[4 * q + 2] = t.z; v[4 * q + 3] = t.w;
    }
    if (SUPP) {
      const uint2* mp = reinterpret_cast<const uint2*>(M + b);
      const uint2 m0 = mp[0], m1 = mp[1];
      const unsigned mw[4] = {m0.x, m0.y, m1.x, m1.y};
#pragma unroll
      for (int k = 0; k < 16; k++) v[k] = ((mw[k >> 2] >> (8 * (k & 3))) & 0xff) ? 0.f : v[k];
    }
    float o[8];
    window9f(v, o);
    float4* d = reinterpret_cast<float4*>(dst + y * RX + x0);
    d[0] = make_float4(o[0], o[1], o[2], o[3]);
    d[1] = make_float4(o[4], o[5], o[6], o[7]);
  }
}
// the byte (mask) row pass: dst[y][x] = max_{|k|<=4} src[y][x+k]
__device__ __forceinline__ void rowpass9_u8(const unsigned char* src, unsigned char* dst) {
  constexpr int CPR = (RX - 8) / 8;
  for (int c = threadIdx.x; c < CPR * RY; c += blockDim.x) {
    const int y = c / CPR, x0 = 4 + 8 * (c % CPR), b = y * RX + x0 - 4;
    const uint2* mp = reinterpret_cast<const uint2*>(src + b);
    const uint2 m0 = mp[0], m1 = mp[1];
    const unsigned mw[4] = {m0.x, m0.y, m1.x, m1.y};
    unsigned v[16];
#pragma unroll
    for (int k = 0; k < 16; k++) v[k] = (mw[k >> 2] >> (8 * (k & 3))) & 0xff;
    unsigned o[8];
    window9(v, o);
    uint2 w;
    w.x = o[0] | (o[1] << 8) | (o[2] << 16) | (o[3] << 24);
    w.y = o[4] | (o[5] << 8) | (o[6] << 16) | (o[7] << 24);
    *reinterpret_cast<uint2*>(dst + y * RX + x0) = w;
  }
}
// dst[y][x] = max_{|k|<=4} src[y+k][x] for every column, y in [4, RY-4); F(o, x, y0) consumes the
// 8 outputs of column x from row y0
template <typename V, typename F>
__device__ __forceinline__ void colpass9(const V* src, F&& out) {
  constexpr int CPC = (RY - 8) / 8;
  for (int c = threadIdx.x; c < CPC * RX; c += blockDim.x) {
    const int x = c % RX, y0 = 4 + 8 * (c / RX);
    V v[16];
#pragma unroll
    for (int k = 0; k < 16; k++) v[k] = src[(y0 - 4 + k) * RX + x];
    V o[8];
    window9(v, o);
    out(o, x, y0);
  }
}

__global__ __launch_bounds__(1024) void nms_kernel(NmsArgs a) {
  __shared__ __attribute__((aligned(16))) float S[RY * RX];  // scores (0 outside the image)
  __shared__ __attribute__((aligned(16))) float T[RY * RX];  // row-pass result (fp32, or bytes)
  __shared__ __attribute__((aligned(16))) unsigned char K[RY * RX];  // max_mask
  __shared__ __attribute__((aligned(16))) unsigned char M[RY * RX];  // supp_mask
  unsigned char* T8 = reinterpret_cast<unsigned char*>(T);
  const int H = a.H, W = a.W;
  const int tiles_x = (W + NTX - 1) / NTX, tiles_y = (H + NTY - 1) / NTY;
  const int per = tiles_x * tiles_y, total = a.B * per, band = (total + 7) / 8;
  const int lt = ((int)blockIdx.x & 7) * band + ((int)blockIdx.x >> 3);  // XCD band placement
  if (lt >= total) return;
  const int bi = lt / per, t = lt % per;
  const int y0 = (t / tiles_x) * NTY - NH, x0 = (t % tiles_x) * NTX - NH;
  const float* sc = a.scores + (size_t)bi * H * W;
  for (int i = threadIdx.x; i < RY * RX; i += blockDim.x) {
    const int ly = i / RX, lx = i - ly * RX;
    const int y = y0 + ly, x = x0 + lx;
    S[i] = (y >= 0 && y < H && x >= 0 && x < W) ? sc[(size_t)y * W + x] : 0.f;
  }
  __syncthreads();
  // max_mask = scores == max_pool(scores)
  rowpass9<false>(S, M, T);
  __syncthreads();
  colpass9(T, [&](const float (&o)[8], int x, int y) {
#pragma unroll
    for (int k = 0; k < 8; k++) K[(y + k) * RX + x] = S[(y + k) * RX + x] == o[k];
  });
  __syncthreads();
  for (int it = 0; it < 2; it++) {
    // supp_mask = max_pool(max_mask) > 0 (byte pools)
    rowpass9_u8(K, T8);
    __syncthreads();
    colpass9(T8, [&](const unsigned char (&o)[8], int x, int y) {
#pragma unroll
      for (int k = 0; k < 8; k++) M[(y + k) * RX + x] = o[k] > 0;
    });
    __syncthreads();
    // supp_scores = where(supp_mask, 0, scores); new_max_mask = supp_scores == max_pool(supp_scores);
    // max_mask |= new_max_mask & ~supp_mask
    rowpass9<true>(S, M, T);
    __syncthreads();
    colpass9(T, [&](const float (&o)[8], int x, int y) {
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const int i = (y + k) * RX + x;
        const bool m = M[i] != 0;
        const float f = m ? 0.f : S[i];
        K[i] = K[i] | ((f == o[k]) && !m);
      }
    });
    __syncthreads();
  }
  // output region [NH, NH+NTY) x [NH, NH+NTX): NMS'd map (debug entry points only) + candidates.
  // The workgroup reserves its candidates' slots with ONE atomic (wave ballots + a scan of the
  // wave counts): a per-candidate atomic on the image's counter serialises thousands of
  // candidates at one L2 address.  Slot order is free: top-k orders by (score, flat index).
  static_assert(NTX * NTY == 2 * 1024, "two outputs per thread");
  __shared__ int wcount[16], wbase[16], blk_base;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  unsigned long long key[2];
  bool take[2];
  int mine = 0;
#pragma unroll
  for (int q = 0; q < 2; q++) {
    const int i = threadIdx.x + q * 1024;
    const int ly = NH + i / NTX, lx = NH + i % NTX;
    const int y = y0 + ly, x = x0 + lx;
    take[q] = false;
    key[q] = 0;
    if (y < H && x < W) {
      const float v = K[ly * RX + lx] ? S[ly * RX + lx] : 0.f;
      if (a.nms_out) a.nms_out[(size_t)bi * H * W + (size_t)y * W + x] = v;
      // find_high_score_index: float score > double threshold (src/super_point.cpp:158);
      // remove_borders: border <= y < H-border, border <= x < W-border (:244-245)
      take[q] = (double)v > a.threshold && y >= a.border && y < H - a.border && x >= a.border && x < W - a.border;
      key[q] = ((unsigned long long)(0xFFFFFFFFu - __float_as_uint(v)) << 32) | (unsigned)(y * W + x);
    }
    mine += take[q];
  }
  // exclusive prefix of `mine` within the wave (lane order), then over the waves
  int pre = mine;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(pre, o);
    if (lane >= o) pre += t;
  }
  if (lane == 63) wcount[wv] = pre;
  __syncthreads();
  if (threadIdx.x == 0) {
    int run = 0;
    for (int w = 0; w < 16; w++) {
      wbase[w] = run;
      run += wcount[w];
    }
    blk_base = run ? atomicAdd(&a.cand_count[bi], run) : 0;
  }
  __syncthreads();
  int slot = blk_base + wbase[wv] + pre - mine;
#pragma unroll
  for (int q = 0; q < 2; q++)
    if (take[q]) {
      if (slot < a.cand_cap) a.cand[(size_t)bi * a.cand_cap + slot] = key[q];
      slot++;
    }
}

// ---------------------------------------------------------------------------
// Top-k selection: one workgroup per image, bitonic sort in LDS.
// Key = (~score_bits << 32) | flat_index: ascending key order = score desc,
// then flat index asc (documented tie-break for the reference's non-stable
// std::sort, src/super_point.cpp:185-190).  If n <= k the reference does not
// sort: keypoints stay in row-major scan order (flat index asc).
// ---------------------------------------------------------------------------
// Keys are (~score bits) << 32 | flat index: ascending key = descending score, ties by flat
// index.  Up to lds_cap candidates are sorted whole in LDS (bitonic).  With more (large images)
// and k > 0, an MSB-first 8-bit radix select over the 64-bit keys (LDS histograms) finds the
// exact k-th key first; the k keys at or below it are compacted into LDS and sorted there.
__global__ __launch_bounds__(1024) void topk_kernel(TopkArgs a) {
  extern __shared__ unsigned long long keys[];
  __shared__ unsigned hist[256];
  __shared__ unsigned long long sel_prefix, sel_mask;
  __shared__ unsigned sel_want, sel_n;
  const int bi = blockIdx.x;
  int n = a.cand_count[bi];
  if (n > a.cand_cap) n = a.cand_cap;
  const bool sorted_by_score = (a.k != -1 && a.k < n);
  const unsigned long long* src = a.cand + (size_t)bi * a.cand_cap;
  if (n > a.lds_cap && !sorted_by_score) {  // keep-all beyond the LDS sort: reported by the host
    if (threadIdx.x == 0) a.sel_count[bi] = 0;
    return;
  }
  // k well below the candidate count (or beyond the LDS sort): select the k-th key first, then
  // sort only the k selected keys (the same k keys in the same order as sorting all of them)
  if (sorted_by_score && (n > a.lds_cap || n > 2 * a.k)) {
    if (threadIdx.x == 0) {
      sel_prefix = 0;
      sel_mask = 0;
      sel_want = (unsigned)a.k;
      sel_n = 0;
    }
    for (int shift = 56; shift >= 0; shift -= 8) {
      for (int i = threadIdx.x; i < 256; i += blockDim.x) hist[i] = 0;
      __syncthreads();
      const unsigned long long pre = sel_prefix, msk = sel_mask;
      for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const unsigned long long key = src[i];
        if ((key & msk) == pre) atomicAdd(&hist[(key >> shift) & 255], 1u);
      }
      __syncthreads();
      if (threadIdx.x < 64) {  // the first bin whose cumulative count reaches sel_want: wave scan
        const int l = threadIdx.x;
        unsigned h[4], sum = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
          h[j] = hist[4 * l + j];
          sum += h[j];
        }
        unsigned incl = sum;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const unsigned y = __shfl_up(incl, o);
          if (l >= o) incl += y;
        }
        const unsigned want = sel_want, excl = incl - sum;
        const bool mine = excl < want && want <= incl;
        const unsigned long long any = __ballot(mine);
        if (mine || (any == 0 && l == 63)) {  // (a bin is always found: the total reaches want)
          unsigned below = excl, d = 4 * l, j = 0;
          while (j < 3 && below + h[j] < want) below += h[j++];
          d += j;
          sel_want = want - below;
          sel_prefix |= (unsigned long long)d << shift;
          sel_mask |= 0xFFull << shift;
        }
      }
      __syncthreads();
    }
    const unsigned long long kth = sel_prefix;  // keys are unique: exactly k keys are <= kth
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
      const unsigned long long key = src[i];
      if (key <= kth) keys[atomicAdd(&sel_n, 1u)] = key;
    }
    __syncthreads();
    n = a.k;
  } else {
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
      unsigned long long key = src[i];
      if (!sorted_by_score) key &= 0xFFFFFFFFull;  // flat index only
      keys[i] = key;
    }
  }
  int L = 1;
  while (L < n) L <<= 1;
  for (int i = n + threadIdx.x; i < L; i += blockDim.x) keys[i] = ~0ull;
  __syncthreads();
  for (int size = 2; size <= L; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = threadIdx.x; i < L / 2; i += blockDim.x) {
        const int lo = 2 * i - (i & (stride - 1));
        const int hi = lo + stride;
        const bool up = ((lo & size) == 0);
        const unsigned long long x = keys[lo], y = keys[hi];
        if ((x > y) == up) {
          keys[lo] = y;
          keys[hi] = x;
        }
      }
      __syncthreads();
    }
  }
  const int kout = sorted_by_score ? a.k : n;
  for (int i = threadIdx.x; i < kout; i += blockDim.x) a.sel[(size_t)bi * a.sel_cap + i] = (unsigned)(keys[i] & 0xFFFFFFFFull);
  if (threadIdx.x == 0) a.sel_count[bi] = kout;
}

// ---------------------------------------------------------------------------
// Descriptor sampling + packing (src/super_point.cpp:206-319), fp64.
// One wave per keypoint, 4 channels per lane.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void sample_kernel(SampleArgs a) {
  const int wv = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  const int bi = wv / a.per_image, i = wv % a.per_image;
  if (bi >= a.B) return;
  const int n = a.sel_count[bi];
  if (lane == 0 && i == 0) a.counts[bi] = n;
  if (i >= n) return;
  const int H = a.H, W = a.W, h = H / 8, w = W / 8;
  const unsigned flat = a.sel[(size_t)bi * a.sel_stride + i];
  const int y = flat / W, x = flat % W;
  const float score = a.nms[(size_t)bi * H * W + flat];
  // normalize_keypoints (:276-287): s/2 is integer division
  const double gx = ((double)x - 8 / 2 + 0.5) / (w * 8 - 8 / 2 - 0.5) * 2 - 1;
  const double gy = ((double)y - 8 / 2 + 0.5) / (h * 8 - 8 / 2 - 0.5) * 2 - 1;
  // grid_sample (:294-332), align_corners=True
  const double ix = ((gx + 1) / 2) * (w - 1), iy = ((gy + 1) / 2) * (h - 1);
  auto clip = [](int v, int m) { return v < 0 ? 0 : (v < m - 1 ? v : m - 1); };
  const int ix_nw = clip((int)floor(ix), w), iy_nw = clip((int)floor(iy), h);
  const int ix_ne = clip(ix_nw + 1, w), iy_ne = clip(iy_nw, h);
  const int ix_sw = clip(ix_nw, w), iy_sw = clip(iy_nw + 1, h);
  const int ix_se = clip(ix_nw + 1, w), iy_se = clip(iy_nw + 1, h);
  const double nw = (ix_se - ix) * (iy_se - iy);
  const double ne = (ix - ix_sw) * (iy_sw - iy);
  const double sw = (ix_ne - ix) * (iy - iy_ne);
  const double se = (ix - ix_nw) * (iy - iy_nw);
  const float* d = a.desc + (size_t)bi * h * w * 256;
  const float4 vnw = *reinterpret_cast<const float4*>(d + ((size_t)iy_nw * w + ix_nw) * 256 + 4 * lane);
  const float4 vne = *reinterpret_cast<const float4*>(d + ((size_t)iy_ne * w + ix_ne) * 256 + 4 * lane);
  const float4 vsw = *reinterpret_cast<const float4*>(d + ((size_t)iy_sw * w + ix_sw) * 256 + 4 * lane);
  const float4 vse = *reinterpret_cast<const float4*>(d + ((size_t)iy_se * w + ix_se) * 256 + 4 * lane);
  double v[4];
  v[0] = (double)vnw.x * nw + (double)vne.x * ne + (double)vsw.x * sw + (double)vse.x * se;
  v[1] = (double)vnw.y * nw + (double)vne.y * ne + (double)vsw.y * sw + (double)vse.y * se;
  v[2] = (double)vnw.z * nw + (double)vne.z * ne + (double)vsw.z * sw + (double)vse.z * se;
  v[3] = (double)vnw.w * nw + (double)vne.w * ne + (double)vsw.w * sw + (double)vse.w * se;
  double ss = v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3];
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) ss += __shfl_xor(ss, o, 64);
  const double inv = 1.0 / sqrt(ss);
  double* f = a.features + ((size_t)bi * a.feat_cap + i) * 259;
  if (lane == 0) {
    f[0] = (double)score;
    f[1] = (double)x;
    f[2] = (double)y;
  }
#pragma unroll
  for (int j = 0; j < 4; j++) f[3 + 4 * lane + j] = inv * v[j];
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
template <int CIN, int TH, bool POOL, bool FUSE1A>
static hipError_t launch_conv(const ConvArgs& a, int B, hipStream_t s, hipEvent_t t0 = nullptr,
                              hipEvent_t t1 = nullptr) {
  const int tiles = ((a.W + TW - 1) / TW) * ((a.H + TH - 1) / TH);
  dim3 grid(B * tiles, a.cout / 64);
  hipExtLaunchKernelGGL((conv3x3_kernel<CIN, TH, POOL, FUSE1A>), grid, dim3(256), 0, s, t0, t1, 0, a);
  return hipGetLastError();
}

hipError_t conv3x3(const ConvArgs& a, int cin, bool pool, bool fuse1a, int B, hipStream_t s, hipEvent_t t0,
                   hipEvent_t t1) {
  const bool small = (a.H * a.W) <= 128 * 192;  // more, smaller tiles for the low-res layers
  if (fuse1a) return launch_conv<64, 16, true, true>(a, B, s, t0, t1);
  if (cin == 64 && pool) return launch_conv<64, 16, true, false>(a, B, s);
  if (cin == 64 && !pool) return small ? launch_conv<64, 8, false, false>(a, B, s) : launch_conv<64, 16, false, false>(a, B, s);
  if (cin == 128 && pool) return launch_conv<128, 16, true, false>(a, B, s);
  if (cin == 128 && !pool) return small ? launch_conv<128, 8, false, false>(a, B, s) : launch_conv<128, 16, false, false>(a, B, s);
  return hipErrorInvalidValue;
}

// the device's CU count (the persistent conv1's grid)
static int device_cus() {
  static int n = 0;
  if (!n) {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                 hipSuccess || cus <= 0)
      cus = 256;
    n = cus;
  }
  return n;
}

template <int CIN, int TH, bool POOL, bool OUT_F32>
static hipError_t launch_conv_h(const ConvArgs& a, int B, hipStream_t s) {
  const int tiles = ((a.W + TW - 1) / TW) * ((a.H + TH - 1) / TH);
  dim3 grid(B * tiles, a.cout / 64);
  hipLaunchKernelGGL((conv3x3_h_kernel<CIN, TH, POOL, OUT_F32>), grid, dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t conv3x3_h(const ConvArgs& a, int cin, bool pool, bool fuse1a, bool out_f32, int B, hipStream_t s,
                     hipEvent_t t0, hipEvent_t t1) {
  const bool small = (a.H * a.W) <= 128 * 192;
  if (fuse1a) {
    constexpr size_t lds = sizeof(_Float16) * (9 * 64 * C1S + 18 * 18 * C1S) + sizeof(float) * (20 * 20 + 64 * 10);
    static bool attr = false;
    if (!attr) {
      const hipError_t e = hipFuncSetAttribute((const void*)conv1_res_kernel,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      if (e != hipSuccess) return e;
      attr = true;
    }
    ConvArgs b = a;
    b.B = B;
    const int tiles = B * ((a.W + TW - 1) / TW) * ((a.H + 15) / 16);
    // one persistent workgroup on every other CU: each holds 131 KB of a CU's LDS for the whole conv1, so on a
    // CU it occupies no local-BA Schur chunk wave (35 KB) fits -- with a workgroup on every CU the BA chain
    // stalled for the length of conv1 every step.  Measured in the C3 pipeline (r05 experiments): 256 workgroups
    // 936 frames/s, 192 951-967, 128 976-977 (conv1 0.15 -> 0.19 ms, off the critical path).
    const int wgs = std::max(1, device_cus() / 2);
    hipExtLaunchKernelGGL(conv1_res_kernel, dim3(std::min(tiles, wgs)), dim3(256), lds, s, t0, t1, 0, b);
    return hipGetLastError();
  }
  if (out_f32) return launch_conv_h<128, 8, false, true>(a, B, s);
  if (cin == 64 && pool) return launch_conv_h<64, 16, true, false>(a, B, s);
  if (cin == 64 && !pool) return small ? launch_conv_h<64, 8, false, false>(a, B, s)
                                       : launch_conv_h<64, 16, false, false>(a, B, s);
  if (cin == 128 && pool) return launch_conv_h<128, 16, true, false>(a, B, s);
  if (cin == 128 && !pool) return small ? launch_conv_h<128, 8, false, false>(a, B, s)
                                        : launch_conv_h<128, 16, false, false>(a, B, s);
  return hipErrorInvalidValue;
}

hipError_t heads(const HeadArgs& a, int mode, hipStream_t s) {
  const int blocks = (a.B * a.P + 127) / 128;
  if (mode == 0)
    hipLaunchKernelGGL(head_kernel<0>, dim3(blocks), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(head_kernel<1>, dim3(blocks), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t det_head_h(const HeadHArgs& a, bool x3, hipStream_t s) {
  const int blocks = (a.B * a.P + 127) / 128;
  if (x3) hipLaunchKernelGGL(det_head_h_kernel<true>, dim3(blocks), dim3(256), 0, s, a);
  else hipLaunchKernelGGL(det_head_h_kernel<false>, dim3(blocks), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t sample_taps_h(const TapArgs& a, bool x3, hipStream_t s) {
  const int blocks = a.B * ((a.per_image + 7) / 8);
  if (x3) hipLaunchKernelGGL(sample_taps_h_kernel<true>, dim3(blocks), dim3(256), 0, s, a);
  else hipLaunchKernelGGL(sample_taps_h_kernel<false>, dim3(blocks), dim3(256), 0, s, a);
  return hipGetLastError();
}

template <int CIN, int TH, bool POOL, bool FUSE1A>
static hipError_t launch_conv_x3(const ConvArgs& a, int B, hipStream_t s, hipEvent_t t0 = nullptr,
                                 hipEvent_t t1 = nullptr) {
  const int tiles = ((a.W + TW - 1) / TW) * ((a.H + TH - 1) / TH);
  dim3 grid(B * tiles, a.cout / 64);
  hipExtLaunchKernelGGL((conv3x3_x3_kernel<CIN, TH, POOL, FUSE1A>), grid, dim3(256), 0, s, t0, t1, 0, a);
  return hipGetLastError();
}

hipError_t conv3x3_x3(const ConvArgs& a, int cin, bool pool, bool fuse1a, int B, hipStream_t s, hipEvent_t t0,
                      hipEvent_t t1) {
  const bool small = (a.H * a.W) <= 128 * 192;
  if (fuse1a) return launch_conv_x3<64, 16, true, true>(a, B, s, t0, t1);
  if (cin == 64 && pool) return launch_conv_x3<64, 16, true, false>(a, B, s);
  if (cin == 64 && !pool) return small ? launch_conv_x3<64, 8, false, false>(a, B, s)
                                       : launch_conv_x3<64, 16, false, false>(a, B, s);
  if (cin == 128 && pool) return launch_conv_x3<128, 16, true, false>(a, B, s);
  if (cin == 128 && !pool) return small ? launch_conv_x3<128, 8, false, false>(a, B, s)
                                        : launch_conv_x3<128, 16, false, false>(a, B, s);
  return hipErrorInvalidValue;
}

hipError_t nms(const NmsArgs& a, int B, hipStream_t s) {
  const int tiles = ((a.W + NTX - 1) / NTX) * ((a.H + NTY - 1) / NTY);
  NmsArgs b = a;
  b.B = B;
  hipLaunchKernelGGL(nms_kernel, dim3(8 * ((B * tiles + 7) / 8)), dim3(1024), 0, s, b);
  return hipGetLastError();
}

hipError_t topk(const TopkArgs& a, int B, hipStream_t s) {
  int L = 1;
  while (L < a.lds_cap) L <<= 1;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)topk_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)(L * sizeof(unsigned long long)));
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  hipLaunchKernelGGL(topk_kernel, dim3(B), dim3(1024), L * sizeof(unsigned long long), s, a);
  return hipGetLastError();
}

hipError_t sample(const SampleArgs& a, hipStream_t s) {
  const int waves = a.B * a.per_image;
  hipLaunchKernelGGL(sample_kernel, dim3((waves + 3) / 4), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace sp
}  // namespace rspl
