// SuperGlue forward + log-optimal-transport + decode on gfx950 (CDNA4), fp32 MFMA.
//
// Reference semantics (convert2onnx/superglue.py; src/super_glue.cpp):
//   KeypointEncoder :75-85, attention/MHA :88-142 (channel c = d*4 + h), GNN :145-173,
//   final_proj + scores/16 :295-300, log_optimal_transport :176-205,
//   decode (argmax / mutual / exp / 0.2) super_glue.cpp:258-367,
//   process_input (double -> float packing) super_glue.cpp:199-246,
//   PointMatching::NormalizeKeypoints point_matching.cc:50-62.
// Layout: token-major.  Token t = (pair*2 + image)*nmax + i; descriptors X[t][256].
// Q/K/V channels are stored head-contiguous (h*64 + d); the weight rows are
// permuted once on the host so this equals the reference's d*4 + h interleave.
#include <cstdlib>
#include <string>
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cfloat>
#include <cstdint>

#include "sg_kernels.hpp"

namespace rspl {
namespace sg {

typedef float floatx16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ floatx16 mfma32(float a, float b, floatx16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// ---------------------------------------------------------------------------
// Generic fp32 MFMA GEMM: 64x64 tile, BK = 32, 4 waves (2x2) of 32x32 each.
// Double-buffered LDS with a register prefetch of the next K tile issued before
// the 16 MFMAs of the current one: one barrier per K step, load latency hidden.
// ---------------------------------------------------------------------------
template <int EPI, bool BNT>
__global__ __launch_bounds__(256) void gemm_kernel(GemmArgs a) {
  __shared__ float As[2][32][64 + 4];
  __shared__ float Bs[2][32][64 + 4];
  const int z = blockIdx.z;
  int M = a.M, N = a.N;
  if (a.mcount) M = a.mcount[(size_t)z * a.count_stride];
  if (a.ncount) N = a.ncount[(size_t)z * a.count_stride];
  const int m0 = blockIdx.y * 64, n0 = blockIdx.x * 64;
  if (m0 >= M || n0 >= N) return;
  const float* A = a.A + z * a.sA;
  const float* A2 = a.A2 ? a.A2 + z * a.sA : nullptr;
  const float* B = a.B + z * a.sB;
  float* C = a.C + z * a.sC;
  const int K = a.K;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, ml = lane & 31, kl = lane >> 5;
  const int wm = wv >> 1, wn = wv & 1;
  // loader coordinates: A / B^T tiles 64 x 32 (row = tid>>3 (+32), k4 = (tid&7)*4),
  // B tile 32 x 64 (k = tid>>4 (+16), n4 = (tid&15)*4)
  const int lr = tid >> 3, lk4 = (tid & 7) * 4;
  const int bk = tid >> 4, bn4 = (tid & 15) * 4;
  float4 ra[2], rb[2];
  auto load = [&](int k0) {
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const int m = m0 + lr + 32 * h, k = k0 + lk4;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (m < M && k < K) {
        const float* src = (A2 && k >= a.ksplit) ? A2 + (size_t)m * a.lda + (k - a.ksplit) : A + (size_t)m * a.lda + k;
        v = *reinterpret_cast<const float4*>(src);
      }
      ra[h] = v;
    }
#pragma unroll
    for (int h = 0; h < 2; h++) {
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if constexpr (!BNT) {
        const int k = k0 + bk + 16 * h;
        if (k < K && n0 + bn4 < N) v = *reinterpret_cast<const float4*>(B + (size_t)k * a.ldb + n0 + bn4);
      } else {
        const int n = n0 + lr + 32 * h, k = k0 + lk4;
        if (n < N && k < K) v = *reinterpret_cast<const float4*>(B + (size_t)n * a.ldb + k);
      }
      rb[h] = v;
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const int r = lr + 32 * h;
      As[buf][lk4 + 0][r] = ra[h].x; As[buf][lk4 + 1][r] = ra[h].y;
      As[buf][lk4 + 2][r] = ra[h].z; As[buf][lk4 + 3][r] = ra[h].w;
      if constexpr (!BNT) {
        *reinterpret_cast<float4*>(&Bs[buf][bk + 16 * h][bn4]) = rb[h];
      } else {
        Bs[buf][lk4 + 0][r] = rb[h].x; Bs[buf][lk4 + 1][r] = rb[h].y;
        Bs[buf][lk4 + 2][r] = rb[h].z; Bs[buf][lk4 + 3][r] = rb[h].w;
      }
    }
  };
  floatx16 acc;
#pragma unroll
  for (int r = 0; r < 16; r++) acc[r] = 0.f;
  const int nk = (K + 31) / 32;
  load(0);
  store(0);
  __syncthreads();
  for (int kt = 0; kt < nk; kt++) {
    const int buf = kt & 1;
    if (kt + 1 < nk) load((kt + 1) * 32);
#pragma unroll
    for (int kk = 0; kk < 32; kk += 2)
      acc = mfma32(As[buf][kk + kl][wm * 32 + ml], Bs[buf][kk + kl][wn * 32 + ml], acc);
    if (kt + 1 < nk) store(buf ^ 1);
    __syncthreads();
  }
  const int n = n0 + wn * 32 + ml;
  if (n >= N) return;
  const float b = a.bias ? a.bias[n] : 0.f;
#pragma unroll
  for (int r = 0; r < 16; r++) {
    const int m = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * kl;
    if (m < M) {
      float v = acc[r] * a.alpha + b;
      float* dst = C + (size_t)m * a.ldc + n;
      if constexpr (EPI == 1) v = v > 0.f ? v : 0.f;
      if constexpr (EPI == 2) v = *dst + v;
      *dst = v;
    }
  }
}

// ---------------------------------------------------------------------------
// Split-K fp32 MFMA GEMM for the token-parallel layers (M = tokens ~ 1600 is too
// short for 64x64 tiles to fill 256 CUs): one 32x32 output tile per workgroup, the
// 4 waves take interleaved quarters of K (32-wide steps), each with a register
// prefetch into a wave-private LDS slot (no block barriers in the K loop).  The 4
// partial tiles are summed in a fixed order (w0+w1+w2+w3): deterministic.
// ---------------------------------------------------------------------------
template <int EPI>
__global__ __launch_bounds__(256) void gemm_sk_kernel(GemmArgs a) {
  __shared__ float As[4][32][33];  // [wave][k][m]
  __shared__ float Bs[4][32][33];  // [wave][k][n]
  const int z = blockIdx.z;
  int M = a.M, N = a.N;
  if (a.mcount) M = a.mcount[(size_t)z * a.count_stride];
  if (a.ncount) N = a.ncount[(size_t)z * a.count_stride];
  const int m0 = blockIdx.y * 32, n0 = blockIdx.x * 32;
  if (m0 >= M || n0 >= N) return;
  const float* A = a.A + z * a.sA;
  const float* A2 = a.A2 ? a.A2 + z * a.sA : nullptr;
  const float* B = a.B + z * a.sB;
  float* C = a.C + z * a.sC;
  const int K = a.K, nsteps = (K + 31) / 32;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, ml = lane & 31, kl = lane >> 5;
  float4 ra[4], rb[4];
  auto load = [&](int k0) {
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int i = lane + 64 * u, r = i >> 3, c4 = (i & 7) * 4;
      const int m = m0 + r, ka = k0 + c4, kb = k0 + r, n = n0 + c4;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f), w = v;
      if (m < M && ka < K) {
        const float* src = (A2 && ka >= a.ksplit) ? A2 + (size_t)m * a.lda + (ka - a.ksplit) : A + (size_t)m * a.lda + ka;
        v = *reinterpret_cast<const float4*>(src);
      }
      if (kb < K && n < N) w = *reinterpret_cast<const float4*>(B + (size_t)kb * a.ldb + n);
      ra[u] = v;
      rb[u] = w;
    }
  };
  floatx16 acc;
#pragma unroll
  for (int r = 0; r < 16; r++) acc[r] = 0.f;
  int step = wv;
  if (step < nsteps) load(step * 32);
  for (; step < nsteps; step += 4) {
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int i = lane + 64 * u, r = i >> 3, c4 = (i & 7) * 4;
      As[wv][c4 + 0][r] = ra[u].x; As[wv][c4 + 1][r] = ra[u].y;
      As[wv][c4 + 2][r] = ra[u].z; As[wv][c4 + 3][r] = ra[u].w;
      Bs[wv][r][c4 + 0] = rb[u].x; Bs[wv][r][c4 + 1] = rb[u].y;
      Bs[wv][r][c4 + 2] = rb[u].z; Bs[wv][r][c4 + 3] = rb[u].w;
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
    if (step + 4 < nsteps) load((step + 4) * 32);
#pragma unroll
    for (int kk = 0; kk < 32; kk += 2) acc = mfma32(As[wv][kk + kl][ml], Bs[wv][kk + kl][ml], acc);
  }
  // fixed-order reduction of the 4 K-partials through LDS (reuses As/Bs: 4 x 1056 >= 3 x 16 x 64)
  __syncthreads();
  float* red = &As[0][0][0];
  if (wv > 0) {
#pragma unroll
    for (int r = 0; r < 16; r++) red[((wv - 1) * 16 + r) * 64 + lane] = acc[r];
  }
  __syncthreads();
  if (wv != 0) return;
  const int n = n0 + ml;
  if (n >= N) return;
  const float b = a.bias ? a.bias[n] : 0.f;
#pragma unroll
  for (int r = 0; r < 16; r++) {
    const float s = ((acc[r] + red[(0 * 16 + r) * 64 + lane]) + red[(1 * 16 + r) * 64 + lane]) +
                    red[(2 * 16 + r) * 64 + lane];
    const int m = m0 + (r & 3) + 8 * (r >> 2) + 4 * kl;
    if (m < M) {
      float v = s * a.alpha + b;
      float* dst = C + (size_t)m * a.ldc + n;
      if constexpr (EPI == 1) v = v > 0.f ? v : 0.f;
      if constexpr (EPI == 2) v = *dst + v;
      *dst = v;
    }
  }
}

// ---------------------------------------------------------------------------
// RSPL_PREC_FP16 GEMM (the reference's TensorRT kFP16 SuperGlue engine,
// super_glue.cpp:132): v_mfma_f32_32x32x16_f16, fp32 accumulation and epilogue.
// Lane (r, h) operand fragments come straight from global memory: A = 8 consecutive
// fp32 activations of row m0+r converted to fp16, B = 8 consecutive fp16 weights of
// row n0+r of the transposed weight.  Same 32x32 tile / 4-way K split / fixed-order
// LDS reduction as gemm_sk_kernel; four 16-wide K steps in flight per wave.
// ---------------------------------------------------------------------------
typedef _Float16 half8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ floatx16 mfma16(half8 a, half8 b, floatx16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

template <int EPI>
__global__ __launch_bounds__(256) void gemm_h_kernel(GemmArgs a) {
  __shared__ float red[3 * 16 * 64];
  const int z = blockIdx.z;
  int M = a.M, N = a.N;
  if (a.mcount) M = a.mcount[(size_t)z * a.count_stride];
  if (a.ncount) N = a.ncount[(size_t)z * a.count_stride];
  const int m0 = blockIdx.y * 32, n0 = blockIdx.x * 32;
  if (m0 >= M || n0 >= N) return;
  const float* A = a.A + z * a.sA;
  const float* A2 = a.A2 ? a.A2 + z * a.sA : nullptr;
  float* C = a.C + z * a.sC;
  const int K = a.K, nsteps = K / 16;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, ml = lane & 31, kl = lane >> 5;
  const int m = m0 + ml, n = n0 + ml;
  const bool mok = m < M, nok = n < N;
  const _Float16* Brow = a.hB + (size_t)(nok ? n : 0) * a.ldbh + 8 * kl;
  floatx16 acc;
#pragma unroll
  for (int r = 0; r < 16; r++) acc[r] = 0.f;
  auto afrag = [&](int k0) {
    const int k = k0 + 8 * kl;
    half8 h = {};
    if (mok) {
      const float* src = (A2 && k >= a.ksplit) ? A2 + (size_t)m * a.lda + (k - a.ksplit) : A + (size_t)m * a.lda + k;
      const float4 u = *reinterpret_cast<const float4*>(src), v = *reinterpret_cast<const float4*>(src + 4);
      h[0] = (_Float16)u.x; h[1] = (_Float16)u.y; h[2] = (_Float16)u.z; h[3] = (_Float16)u.w;
      h[4] = (_Float16)v.x; h[5] = (_Float16)v.y; h[6] = (_Float16)v.z; h[7] = (_Float16)v.w;
    }
    return h;
  };
  auto bfrag = [&](int k0) {
    half8 h = {};
    if (nok) h = *reinterpret_cast<const half8*>(Brow + k0);
    return h;
  };
  int step = wv;
  for (; step + 12 < nsteps; step += 16) {  // 4 steps per wave in flight
    half8 av[4], bv[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      av[u] = afrag((step + 4 * u) * 16);
      bv[u] = bfrag((step + 4 * u) * 16);
    }
#pragma unroll
    for (int u = 0; u < 4; u++) acc = mfma16(av[u], bv[u], acc);
  }
  for (; step < nsteps; step += 4) acc = mfma16(afrag(step * 16), bfrag(step * 16), acc);
  if (wv > 0) {
#pragma unroll
    for (int r = 0; r < 16; r++) red[((wv - 1) * 16 + r) * 64 + lane] = acc[r];
  }
  __syncthreads();
  if (wv != 0 || !nok) return;
  const float b = a.bias ? a.bias[n] : 0.f;
#pragma unroll
  for (int r = 0; r < 16; r++) {
    const float s = ((acc[r] + red[(0 * 16 + r) * 64 + lane]) + red[(1 * 16 + r) * 64 + lane]) +
                    red[(2 * 16 + r) * 64 + lane];
    const int mm = m0 + (r & 3) + 8 * (r >> 2) + 4 * kl;
    if (mm < M) {
      float v = s * a.alpha + b;
      float* dst = C + (size_t)mm * a.ldc + n;
      if constexpr (EPI == 1) v = v > 0.f ? v : 0.f;
      if constexpr (EPI == 2) v = *dst + v;
      *dst = v;
    }
  }
}

__global__ void to_half_t_kernel(const float* W, int K, int N, _Float16* Wt) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= K * N) return;
  const int n = i / K, k = i - n * K;
  Wt[i] = (_Float16)W[(size_t)k * N + n];
}

// ---------------------------------------------------------------------------
// fp16 GNN GEMM: one 64x64 tile per 256-thread workgroup (4 waves, 32x32 each on
// v_mfma_f32_32x32x16_f16).  The whole K panel of A and B (K <= 512) is staged in LDS
// (rows padded by 16 B against bank conflicts) with every global load issued before the
// first LDS write: one memory round trip per tile, then back-to-back MFMAs.
// ---------------------------------------------------------------------------
constexpr int kGhMaxK = 512;

template <int MODE>
__global__ __launch_bounds__(256) void gemm_hh_kernel(GemmHArgs a) {
  extern __shared__ _Float16 lds_h[];
  const int K = a.K, ldk = K + 8, kc = K / 8, nch = 64 * kc;
  _Float16* As = lds_h;
  _Float16* Bs = lds_h + 64 * ldk;
  const int m0 = blockIdx.y * 64, n0 = blockIdx.x * 64;
  const int tid = threadIdx.x;
  constexpr int kMaxCh = 64 * kGhMaxK / 8 / 256;  // 16-byte chunks per thread per operand
  uint4 ra[kMaxCh], rb[kMaxCh];
#pragma unroll
  for (int u = 0; u < kMaxCh; u++) {
    const int c = tid + 256 * u;
    uint4 va = make_uint4(0, 0, 0, 0), vb = va;
    if (c < nch) {
      const int row = c / kc, k8 = (c - row * kc) * 8;
      const int m = m0 + row, n = n0 + row;
      if (m < a.M) {
        const _Float16* src = (a.A2 && k8 >= a.ksplit) ? a.A2 + (size_t)m * a.lda2 + (k8 - a.ksplit)
                                                        : a.A + (size_t)m * a.lda + k8;
        va = *reinterpret_cast<const uint4*>(src);
      }
      if (n < a.N) vb = *reinterpret_cast<const uint4*>(a.B + (size_t)n * a.ldb + k8);
    }
    ra[u] = va;
    rb[u] = vb;
  }
#pragma unroll
  for (int u = 0; u < kMaxCh; u++) {
    const int c = tid + 256 * u;
    if (c < nch) {
      const int row = c / kc, k8 = (c - row * kc) * 8;
      *reinterpret_cast<uint4*>(As + row * ldk + k8) = ra[u];
      *reinterpret_cast<uint4*>(Bs + row * ldk + k8) = rb[u];
    }
  }
  __syncthreads();
  const int lane = tid & 63, wv = tid >> 6, r32 = lane & 31, kh = lane >> 5;
  const int wm = 32 * (wv >> 1), wn = 32 * (wv & 1);
  const _Float16* ap = As + (wm + r32) * ldk + 8 * kh;
  const _Float16* bp = Bs + (wn + r32) * ldk + 8 * kh;
  floatx16 acc;
#pragma unroll
  for (int r = 0; r < 16; r++) acc[r] = 0.f;
  const int ns = K / 16;
  int st = 0;
  for (; st + 4 <= ns; st += 4) {
    half8 av[4], bv[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      av[u] = *reinterpret_cast<const half8*>(ap + 16 * (st + u));
      bv[u] = *reinterpret_cast<const half8*>(bp + 16 * (st + u));
    }
#pragma unroll
    for (int u = 0; u < 4; u++) acc = mfma16(av[u], bv[u], acc);
  }
  for (; st < ns; st++)
    acc = mfma16(*reinterpret_cast<const half8*>(ap + 16 * st), *reinterpret_cast<const half8*>(bp + 16 * st), acc);
  const int n = n0 + wn + r32;
  if (n >= a.N) return;
  const float bias = a.bias ? a.bias[n] : 0.f;
#pragma unroll
  for (int r = 0; r < 16; r++) {
    const int m = m0 + wm + (r & 3) + 8 * (r >> 2) + 4 * kh;
    if (m >= a.M) continue;
    const float v = acc[r] + bias;
    if constexpr (MODE == 0) {
      a.C32[(size_t)m * a.ldc32 + n] = v;
    } else if constexpr (MODE == 1) {
      a.C16[(size_t)m * a.ldc16 + n] = (_Float16)v;
    } else if constexpr (MODE == 2) {
      a.C16[(size_t)m * a.ldc16 + n] = (_Float16)(v > 0.f ? v : 0.f);
    } else if constexpr (MODE == 3) {
      float* d = a.C32 + (size_t)m * a.ldc32 + n;
      const float x = *d + v;
      *d = x;
      a.C16[(size_t)m * a.ldc16 + n] = (_Float16)x;
    } else {
      if (n < 512) {
        a.C16[(size_t)m * a.ldc16 + n] = (_Float16)v;
      } else {
        const int c = n - 512, set = m / a.nmax, tok = m - set * a.nmax;
        a.Vt[((size_t)(set * 4 + (c >> 6)) * 64 + (c & 63)) * a.ldv + tok] = (_Float16)v;
      }
    }
  }
}

// fp16 GEMM epilogue of one output element (MODE as gemm_hh_kernel)
template <int MODE>
__device__ __forceinline__ void gemm_h_store(const GemmHArgs& a, int m, int n, float v) {
  if constexpr (MODE == 0) {
    a.C32[(size_t)m * a.ldc32 + n] = v;
  } else if constexpr (MODE == 1) {
    a.C16[(size_t)m * a.ldc16 + n] = (_Float16)v;
  } else if constexpr (MODE == 2) {
    a.C16[(size_t)m * a.ldc16 + n] = (_Float16)(v > 0.f ? v : 0.f);
  } else if constexpr (MODE == 3) {
    float* d = a.C32 + (size_t)m * a.ldc32 + n;
    const float x = *d + v;
    *d = x;
    a.C16[(size_t)m * a.ldc16 + n] = (_Float16)x;
  } else {
    if (n < 512) {
      a.C16[(size_t)m * a.ldc16 + n] = (_Float16)v;
    } else {
      const int c = n - 512, set = m / a.nmax, tok = m - set * a.nmax;
      a.Vt[((size_t)(set * 4 + (c >> 6)) * 64 + (c & 63)) * a.ldv + tok] = (_Float16)v;
    }
  }
}

// ---------------------------------------------------------------------------
// fp16 GEMM for the GNN's small-M projections (M = 2B x nmax tokens, K = 256 / 512): one
// workgroup per 32 x (32 TN) output tile, K split four ways (wave w takes the w-th quarter,
// K / 64 <= 8 MFMA steps with every load in flight at once: a single memory round trip).
// Lane (r, h) loads its fragments straight from global memory (16 bytes of row r at
// k = 16 s + 8 h, the 32x32x16 operand layout); the four partial tiles are summed in wave
// order through LDS (16 KB) and stored coalesced.  Small LDS / VGPR footprint, so the BA's
// latency-bound kernels still find room on the CUs while the GNN runs.
// ---------------------------------------------------------------------------
constexpr int kRdU = 8;  // max K steps (16 each) per wave: K <= 512
template <int MODE, int TN>
__global__ __launch_bounds__(256) void gemm_rk_kernel(GemmHArgs a, int ntn) {
  __shared__ float red[4][TN * 16][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int tm = blockIdx.x / ntn, tn = blockIdx.x - tm * ntn;
  const int m0 = 32 * tm, n0 = 32 * TN * tn;
  const int r = lane & 31, h = lane >> 5;
  const int m = m0 + r;
  const bool mok = m < a.M;
  const int nsw = a.K / 64, k0 = wv * nsw * 16;
  const _Float16* Ap = a.A + (size_t)(mok ? m : 0) * a.lda + 8 * h;
  const _Float16* A2p = a.A2 ? a.A2 + (size_t)(mok ? m : 0) * a.lda2 + 8 * h - a.ksplit : nullptr;
  const _Float16* Bp[TN];
  bool nok[TN];
#pragma unroll
  for (int t = 0; t < TN; t++) {
    const int n = n0 + 32 * t + r;
    nok[t] = n < a.N;
    Bp[t] = a.B + (size_t)(nok[t] ? n : 0) * a.ldb + 8 * h;
  }
  half8 av[kRdU], bv[kRdU][TN];
  const half8 z = {};
#pragma unroll
  for (int u = 0; u < kRdU; u++) {
    const int k = k0 + 16 * u;
    const bool in = u < nsw;
    const _Float16* src = (A2p && k >= a.ksplit) ? A2p + k : Ap + k;
    av[u] = (in && mok) ? *reinterpret_cast<const half8*>(src) : z;
#pragma unroll
    for (int t = 0; t < TN; t++) bv[u][t] = (in && nok[t]) ? *reinterpret_cast<const half8*>(Bp[t] + k) : z;
  }
  floatx16 acc[TN];
#pragma unroll
  for (int t = 0; t < TN; t++)
#pragma unroll
    for (int i = 0; i < 16; i++) acc[t][i] = 0.f;
#pragma unroll
  for (int u = 0; u < kRdU; u++)
    if (u < nsw)
#pragma unroll
      for (int t = 0; t < TN; t++) acc[t] = mfma16(av[u], bv[u][t], acc[t]);
#pragma unroll
  for (int t = 0; t < TN; t++)
#pragma unroll
    for (int i = 0; i < 16; i++) red[wv][16 * t + i][lane] = acc[t][i];
  __syncthreads();
#pragma unroll
  for (int e = threadIdx.x; e < TN * 16 * 64; e += 256) {
    const int i16 = e >> 6, ln = e & 63;
    const float v = (red[0][i16][ln] + red[1][i16][ln]) + (red[2][i16][ln] + red[3][i16][ln]);
    const int t = i16 >> 4, i = i16 & 15;
    const int n = n0 + 32 * t + (ln & 31);
    const int mm = m0 + (i & 3) + 8 * (i >> 2) + 4 * (ln >> 5);
    if (n < a.N && mm < a.M) gemm_h_store<MODE>(a, mm, n, v + (a.bias ? a.bias[n] : 0.f));
  }
}

__global__ void to_half_kernel(const float* x, _Float16* y, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = (_Float16)x[i];
}

// ---------------------------------------------------------------------------
// One AttentionalGNN layer, fused (fp16 engine; superglue.py:88-173): a 512-thread workgroup
// owns 32 tokens of one image and runs, without leaving the CU,
//   (1) multi-head attention of its 32 queries against all keys / values of the source image
//       (self or cross), flash-style (online softmax; swapped product S^T = K Q^T, keys on registers,
//       queries on lanes): wave w takes head w & 3 and every other 32-key tile; the two partial
//       softmax states per head merge through LDS;
//   (2) mlp.0 on [x | message] (merge folded into W1, BN folded) + ReLU -> HID in LDS;
//   (3) mlp.3 + the residual: x += delta (fp32 stream, fp16 shadow, and the new fp16 x in LDS);
//   (4) the NEXT layer's q / k / v projections of the same 32 tokens (v stored transposed).
// The only cross-token dependency of a layer -- attention reads every token's k / v of the
// layer -- is the kernel boundary: Q/K/V ping-pong between two buffer sets.  All operands of the
// 32x32x16 f16 MFMAs: activations from LDS (rows padded to 1040 B), weights straight from
// global (L2-resident: 1.15 MB per layer, read once per workgroup), fp32 accumulation.
// One launch per layer instead of four (QKV GEMM, attention, mlp.0, mlp.3).
// ---------------------------------------------------------------------------
constexpr int kLdA = 520;  // halves per LDS activation row (512 + 8: 16-byte aligned, bank spread)

// acc[t] += A[32 x K] (LDS rows) * W[n0 + 32 t + r][k]^T, t < NT; W in B-fragment order
// (to_frag): the operand of (n-tile, k-step) is one contiguous 1 KB read per wave
// one output tile per wave: odd k-steps go to a second accumulator set (two independent MFMA
// dependency chains per tile instead of one), summed at the end
template <int NT, bool SPLIT = (NT < 2)>
__device__ __forceinline__ void wave_mm(const _Float16* Al, const _Float16* Wf, int n0, int K, floatx16 (&acc)[NT],
                                        int lda = kLdA) {
  floatx16 acc2[NT];
#pragma unroll
  for (int t = 0; t < NT; t++)
#pragma unroll
    for (int i = 0; i < 16; i++) acc2[t][i] = 0.f;
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5, KS = K / 16;
  const _Float16* ap = Al + r * lda + 8 * h;
  const _Float16* bp[NT];
#pragma unroll
  for (int t = 0; t < NT; t++) bp[t] = Wf + ((size_t)(n0 / 32 + t) * KS * 64 + lane) * 8;
  constexpr int U = 8;  // k-steps per chunk (16 each): the next chunk's weights load during this one
  half8 bcur[U][NT], bnxt[U][NT];
#pragma unroll
  for (int u = 0; u < U; u++)
#pragma unroll
    for (int t = 0; t < NT; t++) bcur[u][t] = *reinterpret_cast<const half8*>(bp[t] + 512 * u);
  for (int k0 = 0; k0 < K; k0 += 16 * U) {
    const bool more = k0 + 16 * U < K;
    const int ks0 = k0 / 16;
    if (more) {
#pragma unroll
      for (int u = 0; u < U; u++)
#pragma unroll
        for (int t = 0; t < NT; t++) bnxt[u][t] = *reinterpret_cast<const half8*>(bp[t] + 512 * (ks0 + U + u));
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const half8 a = *reinterpret_cast<const half8*>(ap + k0 + 16 * u);
#pragma unroll
      for (int t = 0; t < NT; t++) {
        if (SPLIT && (u & 1)) acc2[t] = mfma16(a, bcur[u][t], acc2[t]);
        else acc[t] = mfma16(a, bcur[u][t], acc[t]);
      }
    }
    if (more) {
#pragma unroll
      for (int u = 0; u < U; u++)
#pragma unroll
        for (int t = 0; t < NT; t++) bcur[u][t] = bnxt[u][t];
    }
  }
  if (SPLIT)
#pragma unroll
    for (int t = 0; t < NT; t++) acc[t] += acc2[t];
}

__global__ __launch_bounds__(512) void layer_kernel(LayerArgs a) {
  extern __shared__ _Float16 lds_l[];
  _Float16* Ab = lds_l;               // [32][kLdA]: x (0..255) | message (256..511)
  _Float16* Hb = lds_l + 32 * kLdA;   // [32][kLdA]: HID; before that the attention merge buffer
  float* Om = reinterpret_cast<float*>(Hb);  // [4 heads][64 d][32 q]
  __shared__ float Ml[4][32], Ll[4][32];
  // XCD-aware placement: the tiles of one token set go to the same XCD(s) (block b runs on XCD
  // b % 8), so each XCD's L2 holds the k / v of one set instead of all of them
  int bx, set;
  if (a.xps > 0) {
    const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
    set = xcd / a.xps;
    bx = (xcd % a.xps) * a.tpx + slot;
    if (set >= a.nsets || slot >= a.tpx || bx >= (a.nmax + 31) / 32) return;  // whole workgroup
  } else {
    bx = blockIdx.x;
    set = blockIdx.y;
  }
  const int p = set >> 1, img = set & 1;
  const int simg = a.cross ? 1 - img : img;
  const int nk = simg ? a.n1[p] : a.n0[p];
  const int q0 = bx * 32;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, c = lane & 31, kh = lane >> 5;
  const size_t tok0 = (size_t)set * a.nmax + q0;   // first token of the tile
  const int kset = p * 2 + simg;
  // x tile -> LDS (rows past the set clamp to its last token; never stored back)
  for (int e = tid; e < 32 * 32; e += 512) {
    const int row = e >> 5, ch = e & 31;
    const int q = min(q0 + row, a.nmax - 1);
    *reinterpret_cast<uint4*>(Ab + row * kLdA + 8 * ch) =
        *reinterpret_cast<const uint4*>(a.Xh + ((size_t)set * a.nmax + q) * 256 + 8 * ch);
  }
  // the fp32 residual values this lane updates in (3), fetched now so the load latency hides
  // behind attention and mlp.0: X[token row(i)][32 wv + r]
  float xres[16];
  if (!a.qkv_only) {
    const int r_ = lane & 31, h_ = lane >> 5;
#pragma unroll
    for (int i = 0; i < 16; i++) {
      const int row = (i & 3) + 8 * (i >> 2) + 4 * h_;
      const int q = min(q0 + row, a.nmax - 1);
      xres[i] = a.X[((size_t)set * a.nmax + q) * 256 + 32 * wv + r_];
    }
  }
  if (a.qkv_only) __syncthreads();  // prologue: layer 0's q / k / v from the current x
  // ---- (1) attention: head h = wv & 3, key tiles part, part + 2, ... (part = wv >> 2) ----
  if (!a.qkv_only) {
    const int h = wv & 3, part = wv >> 2;
    const _Float16* Qb = a.Qc + (size_t)set * a.nmax * 256 + h * 64;
    // fragment-ordered k / v of (source set, head): 32-key tile t, k-step / (d-half, key-half) blocks
    // of 64 lanes x 16 B, every operand load one contiguous 1 KB read
    const _Float16* Kb = a.Kc + ((size_t)(kset * 4 + h) * a.nt) * 4 * 512 + 8 * lane;
    const _Float16* Vb = a.Vc + ((size_t)(kset * 4 + h) * a.nt) * 4 * 512 + 8 * lane;
    half8 qf[4];
    {
      const _Float16* qr = Qb + (size_t)min(q0 + c, a.nmax - 1) * 256 + 8 * kh;
#pragma unroll
      for (int s4 = 0; s4 < 4; s4++) qf[s4] = *reinterpret_cast<const half8*>(qr + 16 * s4);
    }
    floatx16 o0, o1;
#pragma unroll
    for (int r = 0; r < 16; r++) {
      o0[r] = 0.f;
      o1[r] = 0.f;
    }
    float m_run = -INFINITY, l_run = 0.f;
    const int ntiles = (nk + 31) / 32;
    // operands two tiles ahead: this wave's tiles are t, t + 2, t + 4, ...; A and B alternate as the
    // operand sets (the loop body is written for a pair of tiles: static register names, no indexing)
    half8 kA[4], vA[2][2], kB[4], vB[2][2];
    auto fetch = [&](int t, half8 (&kf)[4], half8 (&vf)[2][2]) {
#pragma unroll
      for (int s4 = 0; s4 < 4; s4++) kf[s4] = *reinterpret_cast<const half8*>(Kb + ((size_t)t * 4 + s4) * 512);
#pragma unroll
      for (int dt = 0; dt < 2; dt++)
#pragma unroll
        for (int j = 0; j < 2; j++)
          vf[dt][j] = *reinterpret_cast<const half8*>(Vb + ((size_t)t * 4 + 2 * dt + j) * 512);
    };
    auto tile = [&](int t, const half8 (&kc_)[4], const half8 (&vc)[2][2]) {
      floatx16 st;
#pragma unroll
      for (int r = 0; r < 16; r++) st[r] = 0.f;
#pragma unroll
      for (int s4 = 0; s4 < 4; s4++) st = mfma16(kc_[s4], qf[s4], st);
      float x[16];
      float mx = -INFINITY;
#pragma unroll
      for (int r = 0; r < 16; r++) {
        const int key = t * 32 + (r & 3) + 8 * (r >> 2) + 4 * kh;
        x[r] = key < nk ? st[r] * 0.125f : -INFINITY;  // scores / dim**.5 (superglue.py:90)
        mx = fmaxf(mx, x[r]);
      }
      mx = fmaxf(mx, __shfl_xor(mx, 32));
      const float m_new = fmaxf(m_run, mx);
      const float alpha = __expf(m_run - m_new);
      float sum = 0.f;
#pragma unroll
      for (int r = 0; r < 16; r++) {
        x[r] = __expf(x[r] - m_new);
        sum += x[r];
      }
      sum += __shfl_xor(sum, 32);
      l_run = l_run * alpha + sum;
      m_run = m_new;
#pragma unroll
      for (int r = 0; r < 16; r++) {
        o0[r] *= alpha;
        o1[r] *= alpha;
      }
#pragma unroll
      for (int j = 0; j < 2; j++) {
        half8 pf;
#pragma unroll
        for (int u = 0; u < 8; u++) pf[u] = (_Float16)x[8 * j + u];
        o0 = mfma16(vc[0][j], pf, o0);
        o1 = mfma16(vc[1][j], pf, o1);
      }
    };
    if (part < ntiles) fetch(part, kA, vA);
    if (part + 2 < ntiles) fetch(part + 2, kB, vB);
    for (int t = part; t < ntiles; t += 4) {
      tile(t, kA, vA);
      if (t + 4 < ntiles) fetch(t + 4, kA, vA);
      if (t + 2 >= ntiles) break;
      tile(t + 2, kB, vB);
      if (t + 6 < ntiles) fetch(t + 6, kB, vB);
    }
    // merge the two partial states of each head (part 1 -> LDS -> part 0), message -> Ab
    if (part == 1) {
#pragma unroll
      for (int r = 0; r < 16; r++) {
        const int d = (r & 3) + 8 * (r >> 2) + 4 * kh;
        Om[(h * 64 + d) * 32 + c] = o0[r];
        Om[(h * 64 + 32 + d) * 32 + c] = o1[r];
      }
      if (kh == 0) {
        Ml[h][c] = m_run;
        Ll[h][c] = l_run;
      }
    }
    __syncthreads();
    if (part == 0) {
      const float m1 = Ml[h][c], l1 = Ll[h][c];
      const float M = fmaxf(m_run, m1);
      const float e0 = m_run == -INFINITY ? 0.f : __expf(m_run - M);
      const float e1 = m1 == -INFINITY ? 0.f : __expf(m1 - M);
      const float L = e0 * l_run + e1 * l1;
      const float inv = L > 0.f ? 1.f / L : 0.f;
#pragma unroll
      for (int r = 0; r < 16; r++) {
        const int d = (r & 3) + 8 * (r >> 2) + 4 * kh;
        const float v0 = (e0 * o0[r] + e1 * Om[(h * 64 + d) * 32 + c]) * inv;
        const float v1 = (e0 * o1[r] + e1 * Om[(h * 64 + 32 + d) * 32 + c]) * inv;
        Ab[c * kLdA + 256 + h * 64 + d] = (_Float16)v0;
        Ab[c * kLdA + 256 + h * 64 + 32 + d] = (_Float16)v1;
      }
    }
    __syncthreads();
  }
  const int r = lane & 31, hh = lane >> 5;
  if (!a.qkv_only) {
  // ---- (2) HID = ReLU([x | message] W1^T + b1): wave wv -> columns 64 wv .. 64 wv + 63 ----
  {
    floatx16 acc[2];
#pragma unroll
    for (int t = 0; t < 2; t++)
#pragma unroll
      for (int i = 0; i < 16; i++) acc[t][i] = 0.f;
    wave_mm<2>(Ab, a.W1, 64 * wv, 512, acc);
#pragma unroll
    for (int t = 0; t < 2; t++) {
      const int n = 64 * wv + 32 * t + r;
      const float b = a.b1[n];
#pragma unroll
      for (int i = 0; i < 16; i++) {
        const int row = (i & 3) + 8 * (i >> 2) + 4 * hh;
        const float v = acc[t][i] + b;
        Hb[row * kLdA + n] = (_Float16)(v > 0.f ? v : 0.f);
      }
    }
  }
  __syncthreads();
  // ---- (3) x += HID W2^T + b2 (fp32 stream, fp16 shadow, new x into Ab): columns 32 wv .. +31 ----
  {
    floatx16 acc[1];
#pragma unroll
    for (int i = 0; i < 16; i++) acc[0][i] = 0.f;
    wave_mm<1>(Hb, a.W2, 32 * wv, 512, acc);
    const int n = 32 * wv + r;
    const float b = a.b2[n];
#pragma unroll
    for (int i = 0; i < 16; i++) {
      const int row = (i & 3) + 8 * (i >> 2) + 4 * hh;
      if (q0 + row >= a.nmax) continue;
      const float x = xres[i] + (acc[0][i] + b);
      a.X[(tok0 + row) * 256 + n] = x;
      const _Float16 xh = (_Float16)x;
      a.Xh[(tok0 + row) * 256 + n] = xh;
      Ab[row * kLdA + n] = xh;
    }
  }
  if (a.last) return;
  __syncthreads();
  }
  // ---- (4) next layer's q | k | v of these tokens: columns 96 wv .. 96 wv + 95 ----
  {
    floatx16 acc[3];
#pragma unroll
    for (int t = 0; t < 3; t++)
#pragma unroll
      for (int i = 0; i < 16; i++) acc[t][i] = 0.f;
    wave_mm<3>(Ab, a.Wq, 96 * wv, 256, acc);
    __syncthreads();  // every wave is done with Ab: the q | k | v tile is staged over Ab + Hb
    _Float16* Tq = lds_l;  // [32 tokens][776]
#pragma unroll
    for (int t = 0; t < 3; t++) {
      const int n = 96 * wv + 32 * t + r;
      const float b = a.bq[n];
#pragma unroll
      for (int i = 0; i < 16; i++) {
        const int row = (i & 3) + 8 * (i >> 2) + 4 * hh;
        Tq[row * 776 + n] = (_Float16)(acc[t][i] + b);
      }
    }
    __syncthreads();
    // q rows out (valid tokens), 16-byte stores
    for (int e = tid; e < 32 * 32; e += 512) {
      const int row = e >> 5, ch = e & 31;
      if (q0 + row < a.nmax)
        *reinterpret_cast<uint4*>(a.Qn + (tok0 + row) * 256 + 8 * ch) = *reinterpret_cast<const uint4*>(Tq + row * 776 + 8 * ch);
    }
    // k / v in fragment order: this tile is key tile q0 / 32 of the set; 16 + 16 blocks of 1 KB
    const int kt = q0 >> 5;
    for (int e = tid; e < 2 * 16 * 64; e += 512) {
      const int isv = e >> 10, blk = (e >> 6) & 15, L = e & 63, cl = L & 31, kl = L >> 5, hd = blk >> 2, q4 = blk & 3;
      _Float16* dst = (isv ? a.Vn : a.Kn) + (((size_t)(set * 4 + hd) * a.nt + kt) * 4 + q4) * 512 + 8 * L;
      if (!isv) {  // k: key cl, dims 16 q4 + 8 kl .. +7 of head hd
        *reinterpret_cast<uint4*>(dst) = *reinterpret_cast<const uint4*>(Tq + cl * 776 + 256 + 64 * hd + 16 * q4 + 8 * kl);
      } else {  // v: dim 32 dt + cl, keys 16 j + 4 kl + {0..3, 8..11} (q4 = 2 dt + j)
        const int dt = q4 >> 1, j = q4 & 1, d = 512 + 64 * hd + 32 * dt + cl, k0 = 16 * j + 4 * kl;
        half8 v;
#pragma unroll
        for (int u = 0; u < 8; u++) v[u] = Tq[(k0 + (u < 4 ? u : u + 4)) * 776 + d];
        *reinterpret_cast<half8*>(dst) = v;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// process_input + NormalizeKeypoints: one wave per token.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void prep_kernel(PrepArgs a) {
  const int w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, lane = threadIdx.x & 63;
  const int total = a.B * 2 * a.nmax;
  if (w >= total) return;
  const int i = w % a.nmax, pi = w / a.nmax, p = pi >> 1, img = pi & 1;
  const int n = img ? a.n1[p] : a.n0[p];
  float* X = a.X + (size_t)w * 256;
  float* kin = a.kin + (size_t)w * 16;
  if (i >= n) {  // padding tokens: zeros (finite everywhere downstream)
    *reinterpret_cast<float4*>(X + 4 * lane) = make_float4(0.f, 0.f, 0.f, 0.f);
    if (lane < 16) kin[lane] = 0.f;
    return;
  }
  const double* f = (img ? a.f1 : a.f0) + ((size_t)p * a.stride + i) * 259;
  if (lane < 16) {
    float v = 0.f;
    if (lane == 0 || lane == 1) {
      double c = f[1 + lane];
      if (a.normalize) {
        const int half = (lane == 0 ? a.width : a.height) / 2;  // integer division (point_matching.cc:56-59)
        c = (c - half) / ((a.width > a.height ? a.width : a.height) * 0.7);
      }
      v = (float)c;
    } else if (lane == 2) {
      v = (float)f[0];
    }
    kin[lane] = v;
  }
  float4 d;
  d.x = (float)f[3 + 4 * lane + 0];
  d.y = (float)f[3 + 4 * lane + 1];
  d.z = (float)f[3 + 4 * lane + 2];
  d.w = (float)f[3 + 4 * lane + 3];
  *reinterpret_cast<float4*>(X + 4 * lane) = d;
}

// ---------------------------------------------------------------------------
// Multi-head attention, one head and 32 queries per block; the 4 waves split
// the keys (flash split-K) and merge through LDS.  "Swapped" product
// S^T = K Q^T puts keys on registers and queries on lanes, so the softmax
// reductions are in-lane (+ one xor-32 swap) and S^T feeds O^T = V^T P^T as
// the MFMA B operand with no data movement (keys taken in register order).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void attn_kernel(AttnArgs a) {
  __shared__ float Ks[4][32][65];
  __shared__ float Vs[4][32][64];
  __shared__ float Ml[4][32], Ll[4][32];
  const int pz = blockIdx.z, p = pz >> 1, img = pz & 1;
  const int simg = a.cross ? 1 - img : img;
  const int nq = img ? a.n1[p] : a.n0[p];
  const int nk = simg ? a.n1[p] : a.n0[p];
  const int q0 = blockIdx.x * 32;
  if (q0 >= nq || nk <= 0) return;
  const int h = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, ml = lane & 31, kl = lane >> 5;
  const float* Qb = a.qkv + (size_t)(p * 2 + img) * a.nmax * 768 + h * 64;
  const float* Kb = a.qkv + (size_t)(p * 2 + simg) * a.nmax * 768 + 256 + h * 64;
  const float* Vb = a.qkv + (size_t)(p * 2 + simg) * a.nmax * 768 + 512 + h * 64;
  float qf[32];
  {
    const int q = min(q0 + ml, nq - 1);
    const float* qr = Qb + (size_t)q * 768;
#pragma unroll
    for (int s = 0; s < 32; s++) qf[s] = qr[2 * s + kl];
  }
  floatx16 o0, o1;
#pragma unroll
  for (int r = 0; r < 16; r++) { o0[r] = 0.f; o1[r] = 0.f; }
  float m_run = -INFINITY, l_run = 0.f;
  const int ntiles = (nk + 31) / 32;
  // each wave owns key tiles wv, wv+4, ... and a private LDS slot: the next tile is
  // prefetched into registers while the current one is multiplied (no block barriers)
  float4 pk[8], pv[8];
  auto fetch = [&](int t) {
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int i = lane + 64 * u, row = i >> 4, c4 = (i & 15) * 4, key = t * 32 + row;
      float4 kv = make_float4(0.f, 0.f, 0.f, 0.f), vv = kv;
      if (key < nk) {
        kv = *reinterpret_cast<const float4*>(Kb + (size_t)key * 768 + c4);
        vv = *reinterpret_cast<const float4*>(Vb + (size_t)key * 768 + c4);
      }
      pk[u] = kv;
      pv[u] = vv;
    }
  };
  if (wv < ntiles) fetch(wv);
  for (int t = wv; t < ntiles; t += 4) {
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int i = lane + 64 * u, row = i >> 4, c4 = (i & 15) * 4;
      Ks[wv][row][c4 + 0] = pk[u].x; Ks[wv][row][c4 + 1] = pk[u].y;
      Ks[wv][row][c4 + 2] = pk[u].z; Ks[wv][row][c4 + 3] = pk[u].w;
      *reinterpret_cast<float4*>(&Vs[wv][row][c4]) = pv[u];
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes landed
    __builtin_amdgcn_wave_barrier();
    if (t + 4 < ntiles) fetch(t + 4);
    floatx16 st;
#pragma unroll
    for (int r = 0; r < 16; r++) st[r] = 0.f;
#pragma unroll
    for (int s = 0; s < 32; s++) st = mfma32(Ks[wv][ml][2 * s + kl], qf[s], st);
    float x[16];
    float mx = -INFINITY;
#pragma unroll
    for (int r = 0; r < 16; r++) {
      const int key = t * 32 + (r & 3) + 8 * (r >> 2) + 4 * kl;
      x[r] = key < nk ? st[r] * 0.125f : -INFINITY;  // scores / dim**.5 (superglue.py:90)
      mx = fmaxf(mx, x[r]);
    }
    mx = fmaxf(mx, __shfl_xor(mx, 32));
    const float m_new = fmaxf(m_run, mx);
    const float alpha = __expf(m_run - m_new);
    float sum = 0.f;
#pragma unroll
    for (int r = 0; r < 16; r++) {
      x[r] = expf(x[r] - m_new);
      sum += x[r];
    }
    sum += __shfl_xor(sum, 32);
    l_run = l_run * alpha + sum;
    m_run = m_new;
#pragma unroll
    for (int r = 0; r < 16; r++) { o0[r] *= alpha; o1[r] *= alpha; }
#pragma unroll
    for (int s = 0; s < 16; s++) {
      const int key = (s & 3) + 8 * (s >> 2) + 4 * kl;
      o0 = mfma32(Vs[wv][key][ml], x[s], o0);
      o1 = mfma32(Vs[wv][key][32 + ml], x[s], o1);
    }
  }
  __syncthreads();
  float* Om = &Ks[0][0][0];  // reuse: [4][64][32]
#pragma unroll
  for (int r = 0; r < 16; r++) {
    const int d = (r & 3) + 8 * (r >> 2) + 4 * kl;
    Om[(wv * 64 + d) * 32 + ml] = o0[r];
    Om[(wv * 64 + 32 + d) * 32 + ml] = o1[r];
  }
  if (kl == 0) {
    Ml[wv][ml] = m_run;
    Ll[wv][ml] = l_run;
  }
  __syncthreads();
  float* O = a.O + (size_t)(p * 2 + img) * a.nmax * 256 + h * 64;
  for (int idx = tid; idx < 32 * 64; idx += 256) {
    const int q = idx >> 6, d = idx & 63;
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < 4; w++) M = fmaxf(M, Ml[w][q]);
    float L = 0.f, acc = 0.f;
#pragma unroll
    for (int w = 0; w < 4; w++) {
      const float e = (Ml[w][q] == -INFINITY) ? 0.f : __expf(Ml[w][q] - M);
      L += e * Ll[w][q];
      acc += e * Om[(w * 64 + d) * 32 + q];
    }
    if (q0 + q < nq) O[(size_t)(q0 + q) * 256 + d] = acc / L;
  }
}

// ---------------------------------------------------------------------------
// Dustbin couplings (superglue.py:191-196): column n, row m and the corner = bin_score.
// ---------------------------------------------------------------------------
__global__ void bins_kernel(BinsArgs a) {
  const int p = blockIdx.y;
  const int m = a.n0[p], n = a.n1[p], ld = a.nmax + 1;
  float* C = a.cpl + (size_t)p * ld * ld;
  const float al = *a.alpha;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i <= m + n; i += gridDim.x * blockDim.x) {
    if (i < m) C[(size_t)i * ld + n] = al;        // bins0
    else C[(size_t)m * ld + (i - m)] = al;         // bins1 + corner
  }
}

// ---------------------------------------------------------------------------
// Persistent log-domain Sinkhorn (superglue.py:176-205).
// G workgroups per pair (one per CU, co-resident); workgroup g owns a slab of
// rows AND a slab of columns of the couplings, both held in LDS when they fit
// (the column slab transposed, so both passes read contiguous LDS rows).
// Per iteration (u = log_mu - LSE_row(C + v); v = log_nu - LSE_col(C + u)):
//   row pass over the own rows -> publish own u as tagged granules -> all-gather u
//   column pass over the own columns -> publish own v -> all-gather v.
// Two hand-offs of (N+1) 8-byte granules {f32 bits, tag} per workgroup and
// iteration (a single write-through store each; no flags, no counters).  One
// buffer per vector suffices: a workgroup can only publish u(it+1) after every
// workgroup has published v(it), i.e. finished reading u(it).  Spins are bounded:
// a timed-out workgroup raises the pair's sticky error flag (host-mapped, read by
// rspl_sg_status) and leaves the loop, so every wave reaches the kernel end.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
// DPP all-reduce over a wave64: quad swaps + half-row/row mirrors (in-row), then the
// four row results combined through readlane (uniform).  Fixed structure: deterministic.
template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float rdlane(float v, int l) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l)); }
__device__ __forceinline__ float wave_max_dpp(float v) {
  v = fmaxf(v, dppf<0xB1>(v));   // quad_perm [1,0,3,2]
  v = fmaxf(v, dppf<0x4E>(v));   // quad_perm [2,3,0,1]
  v = fmaxf(v, dppf<0x141>(v));  // row_half_mirror
  v = fmaxf(v, dppf<0x140>(v));  // row_mirror
  return fmaxf(fmaxf(rdlane(v, 0), rdlane(v, 16)), fmaxf(rdlane(v, 32), rdlane(v, 48)));
}
__device__ __forceinline__ float wave_sum_dpp(float v) {
  v += dppf<0xB1>(v);
  v += dppf<0x4E>(v);
  v += dppf<0x141>(v);
  v += dppf<0x140>(v);
  return (rdlane(v, 0) + rdlane(v, 16)) + (rdlane(v, 32) + rdlane(v, 48));
}

__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store(reinterpret_cast<unsigned*>(p), __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_sc1(const float* p) {
  return __uint_as_float(
      __hip_atomic_load(reinterpret_cast<const unsigned*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

constexpr int kSinkThreads = 1024;  // 16 waves: one wave per slab row / column in flight

__device__ __forceinline__ unsigned long long sk_granule(float v, unsigned tag) {
  return ((unsigned long long)tag << 32) | (unsigned long long)__float_as_uint(v);
}

// LSE over len values x[k] + w[k] (x, w in LDS, or x global) of NR rows at once by one wave
// (independent chains interleaved: the DPP reductions and exps of the rows overlap); rows of
// up to 512 values stay in registers between the max and the exp pass.  Lane-uniform results.
template <int NR>
__device__ __forceinline__ void wave_lse(const float* const (&x)[NR], const float* w, int len, int lane,
                                         float (&out)[NR]) {
  float mx[NR], s[NR];
  if (len <= 512) {
    float t[NR][8];
#pragma unroll
    for (int r = 0; r < NR; r++)
#pragma unroll
      for (int q = 0; q < 8; q++) {
        const int j = lane + 64 * q;
        t[r][q] = j < len ? x[r][j] + w[j] : -INFINITY;
      }
#pragma unroll
    for (int r = 0; r < NR; r++) {
      mx[r] = t[r][0];
#pragma unroll
      for (int q = 1; q < 8; q++) mx[r] = fmaxf(mx[r], t[r][q]);
    }
#pragma unroll
    for (int r = 0; r < NR; r++) mx[r] = wave_max_dpp(mx[r]);
#pragma unroll
    for (int r = 0; r < NR; r++) {
      s[r] = 0.f;
#pragma unroll
      for (int q = 0; q < 8; q++) s[r] += (lane + 64 * q) < len ? expf(t[r][q] - mx[r]) : 0.f;
    }
  } else {
#pragma unroll
    for (int r = 0; r < NR; r++) mx[r] = -INFINITY;
    for (int j0 = 0; j0 < len; j0 += 512)
#pragma unroll
      for (int r = 0; r < NR; r++)
#pragma unroll
        for (int q = 0; q < 8; q++) {
          const int j = j0 + lane + 64 * q;
          if (j < len) mx[r] = fmaxf(mx[r], x[r][j] + w[j]);
        }
#pragma unroll
    for (int r = 0; r < NR; r++) {
      mx[r] = wave_max_dpp(mx[r]);
      s[r] = 0.f;
    }
    for (int j0 = 0; j0 < len; j0 += 512)
#pragma unroll
      for (int r = 0; r < NR; r++)
#pragma unroll
        for (int q = 0; q < 8; q++) {
          const int j = j0 + lane + 64 * q;
          if (j < len) s[r] += expf(x[r][j] + w[j] - mx[r]);
        }
  }
#pragma unroll
  for (int r = 0; r < NR; r++) s[r] = wave_sum_dpp(s[r]);
#pragma unroll
  for (int r = 0; r < NR; r++) out[r] = logf(s[r]) + mx[r];
}

// One LSE pass over the n rows of a slab (stride ld) by the workgroup's waves: wave wv takes rows
// wv and wv + NW together.  Lane 0 of the owning wave gets each row's LSE in fn(row, lse).
template <typename F>
__device__ __forceinline__ void slab_lse(const float* slab, int ld, const float* w, int len, int n, int wv, int lane,
                                         F&& fn) {
  constexpr int NW = kSinkThreads / 64;
  for (int r = wv; r < n; r += 2 * NW) {
    if (r + NW < n) {
      const float* const xs[2] = {slab + (size_t)r * ld, slab + (size_t)(r + NW) * ld};
      float o[2];
      wave_lse<2>(xs, w, len, lane, o);
      fn(r, o[0]);
      fn(r + NW, o[1]);
    } else {
      const float* const xs[1] = {slab + (size_t)r * ld};
      float o[1];
      wave_lse<1>(xs, w, len, lane, o);
      fn(r, o[0]);
    }
  }
}

// All-gather of a vector published as tagged granules: dst[j] for j in [0, len) outside the
// caller's own range [o0, o1).  Every thread polls its granules (all loads in flight, only
// the stale ones re-read), bounded by spin_limit.  Returns true on timeout.
__device__ __forceinline__ bool sk_gather(const unsigned long long* src, float* dst, int len, int o0, int o1,
                                          unsigned tag, unsigned spin_limit) {
  bool timed_out = false;
  for (int j = threadIdx.x; j < len; j += kSinkThreads) {
    if (j >= o0 && j < o1) continue;
    unsigned long long gv = __hip_atomic_load(src + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned spins = 0;
    while ((unsigned)(gv >> 32) != tag) {
      if (++spins > spin_limit) {
        timed_out = true;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      gv = __hip_atomic_load(src + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    dst[j] = __uint_as_float((unsigned)gv);
  }
  return timed_out;
}

template <bool SLAB_IN_LDS>
__global__ __launch_bounds__(kSinkThreads) void sinkhorn_kernel(SinkArgs a) {
  extern __shared__ float sm[];
  const int p = blockIdx.y, g = blockIdx.x, G = gridDim.x;
  const int m = a.n0[p], n = a.n1[p];
  if (m <= 0 || n <= 0) return;
  const int R = m + 1, Cc = n + 1, ld = a.nmax + 1, ldp = (ld + 3) & ~3;
  const int rs = (R + G - 1) / G, cs = (Cc + G - 1) / G;
  const int r0 = min(R, g * rs), nr = min(R, r0 + rs) - r0;
  const int c0 = min(Cc, g * cs), nc = min(Cc, c0 + cs) - c0;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const float* Cg = a.cpl + (size_t)p * ld * ld;
  float* u = sm;                                   // [ld] full u
  float* v = u + ldp;                              // [ld] full v
  int* flag = reinterpret_cast<int*>(v + ldp);     // [2] timeout broadcast: u exchange, v exchange
  float* Rs;                                       // [nr][ld] own rows
  float* Cs;                                       // [nc][ld] own columns, transposed
  if constexpr (SLAB_IN_LDS) {
    Rs = v + ldp + 4;
    Cs = Rs + (size_t)rs * ld;
  } else {  // slabs too large for LDS: rows read in place, columns from a transposed scratch copy
    Rs = const_cast<float*>(Cg) + (size_t)r0 * ld;
    Cs = a.cplT + (size_t)p * ld * ld + (size_t)c0 * ld;
  }
  if constexpr (SLAB_IN_LDS) {
    for (int i = tid; i < nr * Cc; i += kSinkThreads) {
      const int r = i / Cc, j = i - r * Cc;
      Rs[r * ld + j] = Cg[(size_t)(r0 + r) * ld + j];
    }
  }
  if (nc > 0)
    for (int i = tid; i < R * nc; i += kSinkThreads) {  // consecutive threads: consecutive columns of a row
      const int r = i / nc, c = i - r * nc;
      Cs[(size_t)c * ld + r] = Cg[(size_t)r * ld + c0 + c];
    }
  for (int j = tid; j < Cc; j += kSinkThreads) v[j] = 0.f;
  for (int j = tid; j < R; j += kSinkThreads) u[j] = 0.f;  // iters == 0: Z = C - norm (u = v = 0)
  // log_mu / log_nu (superglue.py:198-200), float arithmetic as the module
  const float fm = (float)m, fn = (float)n;
  const float norm = -logf(fm + fn);
  const float lmu_bin = logf(fn) + norm, lnu_bin = logf(fm) + norm;
  if (tid < 2) flag[tid] = 0;
  __syncthreads();  // also orders the transposed scratch copy (workgroup-private) before its reads
  unsigned long long* ug = a.ug + (size_t)p * ld;
  unsigned long long* vg = a.vg + (size_t)p * ld;
  // one flag slot per exchange: a slot is rewritten only after a barrier every thread passes
  // after reading it, so all threads take the same branch
  bool failed = false;
  for (int it = 0; it < a.iters; it++) {
    const unsigned tag = (a.seq << 12) | (unsigned)(it + 1);
    // u_i = log_mu_i - LSE_j(C_ij + v_j), own rows, one wave per row
    slab_lse(Rs, ld, v, Cc, nr, wv, lane, [&](int r, float lse) {
      if (lane == 0) {
        const float ui = ((r0 + r) < m ? norm : lmu_bin) - lse;
        u[r0 + r] = ui;
        __hip_atomic_store(ug + r0 + r, sk_granule(ui, tag), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    });
    bool to = sk_gather(ug, u, R, r0, r0 + nr, tag, a.spin_limit);
    if (a.inject && p == 0 && g == 0 && it == 0) to = true;  // fault injection (rspl_sg_debug_inject)
    if (to) flag[0] = 1;
    __syncthreads();
    if (flag[0]) { failed = true; break; }
    // v_j = log_nu_j - LSE_i(C_ij + u_i), own columns, one wave per column
    slab_lse(Cs, ld, u, R, nc, wv, lane, [&](int c, float lse) {
      if (lane == 0) {
        const float vj = ((c0 + c) < n ? norm : lnu_bin) - lse;
        v[c0 + c] = vj;
        __hip_atomic_store(vg + c0 + c, sk_granule(vj, tag), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    });
    if (sk_gather(vg, v, Cc, c0, c0 + nc, tag, a.spin_limit)) flag[1] = 1;
    __syncthreads();
    if (flag[1]) { failed = true; break; }
  }
  if (failed) {
    if (tid == 0) __hip_atomic_store(a.err + p, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return;
  }
  // Z = ((couplings + u) + v) - norm (superglue.py:203, :219), own rows
  float* Z = a.Z + (size_t)p * ld * ld;
  for (int i = tid; i < nr * Cc; i += kSinkThreads) {
    const int r = i / Cc, j = i - r * Cc;
    Z[(size_t)(r0 + r) * ld + j] = ((Rs[(size_t)r * ld + j] + u[r0 + r]) + v[j]) - norm;
  }
}

// ---------------------------------------------------------------------------
// Row-block layout of the register-resident Sinkhorn (superglue.py:176-205), one exchange per
// iteration.  G workgroups per pair; workgroup g holds WHOLE rows [r0, r0 + nr) of the couplings in
// registers: wave w owns rows w + 16 k (k < RPW), lane L columns L + 64 q (q < kRbQ).
// Since every wave holds full rows and a replicated v, the row pass
//   u_i = log_mu_i - LSE_j(C_ij + v_j)
// is wave-local (no barrier, no exchange).  The column pass
//   v_j = log_nu_j - LSE_i(C_ij + u_i)
// reduces each lane's columns over its wave's rows in registers, the 16 waves through LDS,
// and the G workgroups through one all-gather of per-column partials (tagged 8-byte
// granules, double-buffered by iteration parity).  Every workgroup merges the G partials
// in the same order (g = 0 .. G-1), so all hold a bit-identical v.  Parity reuse is safe:
// workgroup g publishes iteration it + 2 into slot (it & 1) only after every peer has
// published it + 1, which each peer does only after reading all of iteration it.
// (Rounds 2-4 ran these passes in the log domain, an exp per element and iteration; the
// scaling form below replaced that kernel.)
// ---------------------------------------------------------------------------
constexpr int kRbQ = 7;                 // 7 x 64 = 448 >= nmax + 1 columns per lane set
// exp for the LSE terms: FX = false -> expf; FX = true -> v_exp_f32 on the split product
// d*log2(e) = a + e (a rounded, e its fma residual) corrected to first order: 2^a (1 + e ln 2);
// arguments are <= 0 here (shifted by the max), below -150 the result is 0 as with expf
template <bool FX>
__device__ __forceinline__ float sk_exp(float d) {
  if constexpr (!FX) {
    return expf(d);
  } else {
    d = d < -150.f ? -150.f : d;  // -inf (masked rows / columns) -> exactly 0 below; NaN stays NaN
    const float a = d * 1.44269504f;
    const float e = fmaf(d, 1.44269504f, -a) + d * 1.9259630e-8f;
    const float r = __builtin_amdgcn_exp2f(a);
    return fmaf(r, e * 0.693147181f, r);
  }
}

// ---------------------------------------------------------------------------
// Scaling-form Sinkhorn (the default for nmax + 1 <= 640): the same iterations as
// log_sinkhorn_iterations (superglue.py:176-183) written on the scalings U = exp(u - a),
// V = exp(v - b) of absorbed log potentials a, b (stabilised Sinkhorn):
//   K_ij = exp(C_ij + a_i + b_j)  (registers),   U_i = mu_i / sum_j K_ij V_j,
//   V_j = nu_j / sum_i K_ij U_i,   u = a + log U,   v = b + log V,
// so an iteration is two mat-vecs of register-resident K -- no exp per element.  Iteration 0's
// row pass runs in the log domain exactly as the module (max-shifted LSE, v = 0) and seeds a = u,
// which bounds K by mu (<= 1).  A scaling that leaves [2^-60, 2^60] is absorbed into a / b and K
// is recomputed from C: rows per workgroup (a is workgroup-local), columns on every workgroup
// alike (V is bit-identical everywhere, so every workgroup decides the same).  Layout, exchange
// and determinism as the row-block layout above: G workgroups per pair hold whole rows (wave w rows
// w + 16 k, lane L columns L + 64 q), the row pass is wave-local, the column sums go through LDS
// across waves and ONE all-gather of per-column partial sums across workgroups per iteration,
// merged in the same order everywhere.  Z = ((C + u) + v) - norm from C re-read at the end.
// ---------------------------------------------------------------------------
// orders this wave's LDS writes before its later LDS reads
__device__ __forceinline__ void wave_barrier_lds() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

template <int RPW, int GM, int Q>  // Q: 64-column lane sets (7: nmax + 1 <= 448, 10: <= 640)
__global__ __launch_bounds__(kSinkThreads) void sinkhorn_sc_kernel(SinkArgs a) {
  __shared__ float ps[16][Q * 64];   // per-wave column partial sums
  __shared__ float vs[Q * 64];       // merged V
  __shared__ int flag[4];               // 0: exchange timeout, 1: column absorb, 2 + (it & 1): row absorb
  __shared__ float as[16 * RPW];        // absorbed row potentials a (row wv + 16 k), read on absorption / at the end
  __shared__ float bs[Q * 64];       // absorbed column potentials b (identical on every workgroup)
  const int p = blockIdx.y, g = blockIdx.x, G = gridDim.x;
  const int m = a.n0[p], n = a.n1[p];
  if (m <= 0 || n <= 0) return;
  const int R = m + 1, Cc = n + 1, ld = a.nmax + 1;
  const int rs = (R + G - 1) / G;
  const int r0 = min(R, g * rs), nr = min(R, r0 + rs) - r0;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const float* Cg = a.cpl + (size_t)p * ld * ld;
  const int nk = min(RPW, max(0, (nr - wv + 15) / 16));  // the wave's rows inside the slab
  float x[RPW][Q];
#pragma unroll
  for (int k = 0; k < RPW; k++) {
    const int r = wv + 16 * k;
#pragma unroll
    for (int q = 0; q < Q; q++) {
      const int j = lane + 64 * q;
      x[k][q] = (r < nr && j < Cc) ? Cg[(size_t)(r0 + r) * ld + j] : -INFINITY;
    }
  }
  // log_mu / log_nu (superglue.py:198-200), float arithmetic as the module; mu / nu = exp of them
  const float fm = (float)m, fn = (float)n;
  const float norm = -logf(fm + fn);
  const float lmu_bin = logf(fn) + norm, lnu_bin = logf(fm) + norm;
  const float mu_in = expf(norm), mu_bin = expf(lmu_bin), nu_bin = expf(lnu_bin);
  constexpr float kLo = 8.6736174e-19f, kHi = 1.1529215e18f;  // 2^-60, 2^60
  if (tid < 4) flag[tid] = 0;
  // iteration 0, row pass in the log domain (v = 0): a = u
  float ur[RPW];
  {
    float mx[RPW], sm[RPW];
#pragma unroll
    for (int k = 0; k < RPW; k++) {
      mx[k] = x[k][0];
#pragma unroll
      for (int q = 1; q < Q; q++) mx[k] = fmaxf(mx[k], x[k][q]);
    }
#pragma unroll
    for (int k = 0; k < RPW; k++) mx[k] = wave_max_dpp(mx[k]);
#pragma unroll
    for (int k = 0; k < RPW; k++) {
      sm[k] = 0.f;
      if (k < nk)
#pragma unroll
        for (int q = 0; q < Q; q++) sm[k] += sk_exp<true>(x[k][q] - mx[k]);
    }
#pragma unroll
    for (int k = 0; k < RPW; k++) sm[k] = wave_sum_dpp(sm[k]);
#pragma unroll
    for (int k = 0; k < RPW; k++) {
      const int r = wv + 16 * k;
      // (no iterations: u = v = 0, Z = C - norm as superglue.py:202-205 -- no seed)
      if (lane == 0)
        as[wv + 16 * k] = r < nr && a.iters > 0 ? ((r0 + r) < m ? norm : lmu_bin) - (logf(sm[k]) + mx[k]) : 0.f;
      ur[k] = 1.f;
    }
  }
  float vr[Q];
#pragma unroll
  for (int q = 0; q < Q; q++) {
    bs[lane + 64 * q] = 0.f;  // every wave writes the same zeros
    vr[q] = 1.f;
  }
  wave_barrier_lds();
  // K = exp(C + a + b), masked entries exactly 0
  auto build_k = [&](bool reload) {
#pragma unroll
    for (int k = 0; k < RPW; k++) {
      const int r = wv + 16 * k;
#pragma unroll
      for (int q = 0; q < Q; q++) {
        const int j = lane + 64 * q;
        const bool in = r < nr && j < Cc;
        const float c = reload ? (in ? Cg[(size_t)(r0 + r) * ld + j] : 0.f) : x[k][q];
        x[k][q] = in ? sk_exp<true>((c + as[wv + 16 * k]) + bs[j]) : 0.f;
      }
    }
  };
  build_k(false);
  __syncthreads();
  bool failed = false;
  for (int it = 0; it < a.iters; it++) {
    const unsigned tag = (a.seq << 12) | (unsigned)(it + 1);
    if (it > 0) {  // row pass: U_i = mu_i / sum_j K_ij V_j (wave-local)
      float sm[RPW];
#pragma unroll
      for (int k = 0; k < RPW; k++) {
        sm[k] = 0.f;
        if (k < nk)
#pragma unroll
          for (int q = 0; q < Q; q++) sm[k] = fmaf(x[k][q], vr[q], sm[k]);
      }
#pragma unroll
      for (int k = 0; k < RPW; k++) sm[k] = wave_sum_dpp(sm[k]);
      bool out = false;
#pragma unroll
      for (int k = 0; k < RPW; k++) {
        const int r = wv + 16 * k;
        ur[k] = r < nr ? ((r0 + r) < m ? mu_in : mu_bin) / sm[k] : 0.f;
        out |= r < nr && !(ur[k] >= kLo && ur[k] <= kHi);
      }
      if (out && lane == 0) flag[2 + (it & 1)] = 1;
    }
    // column partials over the wave's rows, then over the 16 waves
#pragma unroll
    for (int q = 0; q < Q; q++) {
      float cs = 0.f;
#pragma unroll
      for (int k = 0; k < RPW; k++)
        if (k < nk) cs = fmaf(x[k][q], ur[k], cs);
      ps[wv][lane + 64 * q] = cs;
    }
    __syncthreads();
    if (tid == 0) flag[2 + ((it + 1) & 1)] = 0;  // next iteration's row flag (its readers are past)
    unsigned long long* slot = a.ug + (size_t)(p * 2 + (it & 1)) * G * ld;
    // two adjacent lanes per column: lane `half` sums waves 8 half .. 8 half + 7 and polls the
    // peers h with (h & 1) == half; both lanes form the same total (fp addition commutes)
    // (more than 512 columns: every thread holds two column halves; both are published before
    // either is polled, so the exchange stays one round trip)
    constexpr int NP = (Q * 128 + kSinkThreads - 1) / kSinkThreads;
    float own2[NP];
#pragma unroll
    for (int u = 0; u < NP; u++) {
      const int tt = tid + u * kSinkThreads;
      own2[u] = 0.f;
      if (tt < 2 * Cc) {
        const int j = tt >> 1, half = tt & 1;
        float S = 0.f;
#pragma unroll
        for (int w = 0; w < 8; w++) S += ps[8 * half + w][j];
        own2[u] = S + __shfl_xor(S, 1);
        if (!half)
          __hip_atomic_store(slot + (size_t)g * ld + j, sk_granule(own2[u], tag), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
      }
    }
#pragma unroll
    for (int u = 0; u < NP; u++) {
      const int tt = tid + u * kSinkThreads;
      if (tt >= 2 * Cc) continue;
      const int j = tt >> 1, half = tt & 1;
      const float own = own2[u];
      constexpr int GH = GM / 2;
      float l[GH];
      unsigned long long gv[GH];
      unsigned pend = 0;
#pragma unroll
      for (int k = 0; k < GH; k++) {
        const int h = 2 * k + half;
        l[k] = 0.f;
        if (h < G) {
          if (h == g) l[k] = own;
          else pend |= 1u << k;
        }
      }
      bool to = a.inject && p == 0 && g == 0 && it == 0;  // fault injection (rspl_sg_debug_inject)
      unsigned spins = 0;
      while (pend && !to) {
#pragma unroll
        for (int k = 0; k < GH; k++)
          if (pend >> k & 1)
            gv[k] = __hip_atomic_load(slot + (size_t)(2 * k + half) * ld + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
        for (int k = 0; k < GH; k++)
          if ((pend >> k & 1) && (unsigned)(gv[k] >> 32) == tag) {
            l[k] = __uint_as_float((unsigned)gv[k]);
            pend &= ~(1u << k);
          }
        if (!pend) break;
        if (++spins > a.spin_limit) { to = true; break; }
        for (int z = 0; z < a.sleep; z++) __builtin_amdgcn_s_sleep(1);
      }
      if (to) flag[0] = 1;
      float T = 0.f;
#pragma unroll
      for (int k = 0; k < GH; k++) T += l[k];
      T = T + __shfl_xor(T, 1);
      const float V = (j < n ? mu_in : nu_bin) / T;  // nu_j = mu_in for j < n: exp(norm)
      if (!half) {
        vs[j] = V;
        if (!(V >= kLo && V <= kHi)) flag[1] = 1;
      }
    }
    __syncthreads();
    if (flag[0]) { failed = true; break; }
#pragma unroll
    for (int q = 0; q < Q; q++) {
      const int j = lane + 64 * q;
      vr[q] = j < Cc ? vs[j] : 1.f;
    }
    const bool col_abs = flag[1] != 0, row_abs = flag[2 + (it & 1)] != 0;
    if (col_abs || row_abs) {  // rare: absorb the scalings into the log potentials, rebuild K from C
      __syncthreads();  // no wave still reads as / bs of the current K
      if (row_abs) {
#pragma unroll
        for (int k = 0; k < RPW; k++) {
          if (lane == 0) as[wv + 16 * k] += logf(ur[k] > 0.f ? ur[k] : 1.f);
          ur[k] = 1.f;
        }
      }
      if (col_abs) {
        for (int j = tid; j < Q * 64; j += kSinkThreads) bs[j] += logf(vs[j] > 0.f && j < Cc ? vs[j] : 1.f);
#pragma unroll
        for (int q = 0; q < Q; q++) vr[q] = 1.f;
      }
      __syncthreads();
      build_k(true);
      __syncthreads();  // every thread has read flag[1] before it is cleared
      if (tid == 0) flag[1] = 0;
      __syncthreads();
    }
  }
  if (failed) {
    if (tid == 0) __hip_atomic_store(a.err + p, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return;
  }
  // Z = ((couplings + u) + v) - norm (superglue.py:203, :219), own rows; u = a + log U, v = b + log V
  float* Z = a.Z + (size_t)p * ld * ld;
#pragma unroll
  for (int k = 0; k < RPW; k++) {
    const int r = wv + 16 * k;
    if (r >= nr) continue;
    const float u = as[wv + 16 * k] + logf(ur[k]);
#pragma unroll
    for (int q = 0; q < Q; q++) {
      const int j = lane + 64 * q;
      if (j < Cc) Z[(size_t)(r0 + r) * ld + j] = ((Cg[(size_t)(r0 + r) * ld + j] + u) + (bs[j] + logf(vr[q]))) - norm;
    }
  }
}

// ---------------------------------------------------------------------------
// Wide scaling-form Sinkhorn (640 < nmax + 1 <= 64 Q: C5's 2048 keypoints), the same iteration as
// sinkhorn_sc_kernel (K = exp(C + a + b) register resident for whole rows, plain sums, scalings absorbed
// into the log potentials outside [2^-60, 2^60]) on G = ceil(ld / (8 RPW)) workgroups of 512 threads per
// pair: wave w owns rows w + 8 k (k < RPW), lane L columns L + 64 q.  An all-gather of per-column
// partials would move G x ld granules into every workgroup per iteration (G ~ 65), so the column pass
// exchanges in TWO hops:
//   hop 1 (reduce-scatter): every workgroup publishes its partial sum of column j to the column's owner
//     o = j / cs (cs = ceil(ld / G) <= 64 columns per owner), laid out [parity][owner][source][cs] so an
//     owner's inputs are one contiguous run; the owner sums its columns over the G sources in a fixed
//     order (source subsets g = w (mod 8) per wave, then the 8 wave sums in wave order) and forms V_j;
//   hop 2 (broadcast): the owner publishes V_j, every workgroup reads all of V into LDS.
// Every workgroup therefore holds a bit-identical V (and takes the same column absorption decisions).
// Parity reuse: a workgroup writes hop 1 of iteration it + 2 only after reading all of V(it + 1), which
// an owner publishes only after it has read every hop-1 input of it + 1 (and of it before that); the
// owner writes V(it + 2) only after every source's hop 1 of it + 2, which follows their reads of V(it).
// ---------------------------------------------------------------------------
constexpr int kWThreads = 512;  // 8 waves: two per SIMD at <= 256 VGPRs, the partial-sum table fits LDS
constexpr int kWideRPW = 4, kWideQ = 33;  // 32 rows per workgroup, 2112 columns

bool sinkhorn_wide_ok(int nmax, int G) {
  const int ld = nmax + 1;
  return ld > 640 && ld <= kWideQ * 64 && G == (ld + 8 * kWideRPW - 1) / (8 * kWideRPW) && (ld + G - 1) / G <= 64;
}
int sinkhorn_wide_groups(int nmax) { return (nmax + 1 + 8 * kWideRPW - 1) / (8 * kWideRPW); }
size_t sinkhorn_wide_hop1_len(int nmax) {  // granules per pair: [2][G][G][cs]
  const int ld = nmax + 1, G = sinkhorn_wide_groups(nmax), cs = (ld + G - 1) / G;
  return (size_t)2 * G * G * cs;
}
size_t sinkhorn_wide_hop2_len(int nmax) {  // granules per pair: [2][G * cs]
  const int ld = nmax + 1, G = sinkhorn_wide_groups(nmax), cs = (ld + G - 1) / G;
  return (size_t)2 * G * cs;
}

template <int RPW, int Q>
__global__ __launch_bounds__(kWThreads) void sinkhorn_w_kernel(SinkArgs a) {
  constexpr int NW = kWThreads / 64;
  __shared__ float ps[NW][Q * 64];  // per-wave column partial sums
  __shared__ float vs[Q * 64];      // V (identical on every workgroup)
  __shared__ float bs[Q * 64];      // absorbed column potentials b
  __shared__ float as[NW * RPW];    // absorbed row potentials a (row wv + NW k)
  __shared__ float red[NW][64];     // owner: per-wave sums over its source subset
  __shared__ int flag[4];           // 0: exchange timeout, 1: column absorb, 2 + (it & 1): row absorb
  const int p = blockIdx.y, g = blockIdx.x, G = gridDim.x;
  const int m = a.n0[p], n = a.n1[p];
  if (m <= 0 || n <= 0) return;
  const int R = m + 1, Cc = n + 1, ld = a.nmax + 1;
  const int rs = NW * RPW, cs = (ld + G - 1) / G;
  const int r0 = min(R, g * rs), nr = min(R, r0 + rs) - r0;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const float* Cg = a.cpl + (size_t)p * ld * ld;
  const int nk = min(RPW, max(0, (nr - wv + NW - 1) / NW));  // the wave's rows inside the slab
  // row r of the slab into v[q] = C[r0 + r][lane + 64 q]: unconditional loads off one row pointer (the
  // row clamped into the matrix, the last lane set's column clamped to ld - 1), masked afterwards --
  // per-element conditional loads would keep an address per element live
  auto load_row = [&](int r, float (&v)[Q]) {
    const float* rp = Cg + (size_t)min(r0 + r, ld - 1) * ld;
#pragma unroll
    for (int q = 0; q < Q - 1; q++) v[q] = rp[lane + 64 * q];
    v[Q - 1] = rp[min(lane + 64 * (Q - 1), ld - 1)];
  };
  float x[RPW][Q];
#pragma unroll
  for (int k = 0; k < RPW; k++) {
    const int r = wv + NW * k;
    load_row(r, x[k]);
#pragma unroll
    for (int q = 0; q < Q; q++) x[k][q] = (r < nr && lane + 64 * q < Cc) ? x[k][q] : -INFINITY;
  }
  // log_mu / log_nu (superglue.py:198-200), float arithmetic as the module; mu / nu = exp of them
  const float fm = (float)m, fn = (float)n;
  const float norm = -logf(fm + fn);
  const float lmu_bin = logf(fn) + norm, lnu_bin = logf(fm) + norm;
  const float mu_in = expf(norm), mu_bin = expf(lmu_bin), nu_bin = expf(lnu_bin);
  constexpr float kLo = 8.6736174e-19f, kHi = 1.1529215e18f;  // 2^-60, 2^60
  if (tid < 4) flag[tid] = 0;
  // iteration 0, row pass in the log domain (v = 0): a = u
  float ur[RPW];
  {
    float mx[RPW], sm[RPW];
#pragma unroll
    for (int k = 0; k < RPW; k++) {
      mx[k] = x[k][0];
#pragma unroll
      for (int q = 1; q < Q; q++) mx[k] = fmaxf(mx[k], x[k][q]);
    }
#pragma unroll
    for (int k = 0; k < RPW; k++) mx[k] = wave_max_dpp(mx[k]);
#pragma unroll
    for (int k = 0; k < RPW; k++) {
      sm[k] = 0.f;
      if (k < nk)
#pragma unroll
        for (int q = 0; q < Q; q++) sm[k] += sk_exp<true>(x[k][q] - mx[k]);
    }
#pragma unroll
    for (int k = 0; k < RPW; k++) sm[k] = wave_sum_dpp(sm[k]);
#pragma unroll
    for (int k = 0; k < RPW; k++) {
      const int r = wv + NW * k;
      // (no iterations: u = v = 0, Z = C - norm as superglue.py:202-205 -- no seed)
      if (lane == 0)
        as[wv + NW * k] = r < nr && a.iters > 0 ? ((r0 + r) < m ? norm : lmu_bin) - (logf(sm[k]) + mx[k]) : 0.f;
      ur[k] = 1.f;
    }
  }
  for (int j = tid; j < Q * 64; j += kWThreads) {
    bs[j] = 0.f;
    vs[j] = 1.f;
  }
  __syncthreads();
  // K = exp(C + a + b), masked entries exactly 0
  auto build_k = [&](bool reload) {
#pragma unroll
    for (int k = 0; k < RPW; k++) {
      const int r = wv + NW * k;
      if (reload) load_row(r, x[k]);
      const float ak = as[wv + NW * k];
#pragma unroll
      for (int q = 0; q < Q; q++) {
        const int j = lane + 64 * q;
        const bool in = r < nr && j < Cc;
        x[k][q] = in ? sk_exp<true>((x[k][q] + ak) + bs[j]) : 0.f;
      }
    }
  };
  build_k(false);
  unsigned long long* h1 = a.ug + (size_t)p * 2 * G * G * cs;  // [2][owner][source][cs]
  unsigned long long* h2 = a.vg + (size_t)p * 2 * G * cs;      // [2][G * cs]
  const int c0 = g * cs, nc = max(0, min(Cc, c0 + cs) - c0);   // the columns this workgroup owns
  bool failed = false;
  for (int it = 0; it < a.iters; it++) {
    const unsigned tag = (a.seq << 12) | (unsigned)(it + 1);
    const int par = it & 1;
    if (it > 0) {  // row pass: U_i = mu_i / sum_j K_ij V_j (wave-local)
      float sm[RPW];
#pragma unroll
      for (int k = 0; k < RPW; k++) sm[k] = 0.f;
#pragma unroll
      for (int q = 0; q < Q; q++) {
        const float v = vs[lane + 64 * q];
#pragma unroll
        for (int k = 0; k < RPW; k++)
          if (k < nk) sm[k] = fmaf(x[k][q], v, sm[k]);
      }
#pragma unroll
      for (int k = 0; k < RPW; k++) sm[k] = wave_sum_dpp(sm[k]);
      bool out = false;
#pragma unroll
      for (int k = 0; k < RPW; k++) {
        const int r = wv + NW * k;
        ur[k] = r < nr ? ((r0 + r) < m ? mu_in : mu_bin) / sm[k] : 0.f;
        out |= r < nr && !(ur[k] >= kLo && ur[k] <= kHi);
      }
      if (out && lane == 0) flag[2 + (it & 1)] = 1;
    }
    // column partials over the wave's rows, then over the 8 waves
#pragma unroll
    for (int q = 0; q < Q; q++) {
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < RPW; k++)
        if (k < nk) s = fmaf(x[k][q], ur[k], s);
      ps[wv][lane + 64 * q] = s;
    }
    __syncthreads();
    if (tid == 0) flag[2 + ((it + 1) & 1)] = 0;  // next iteration's row flag (its readers are past)
    // hop 1: this workgroup's partial of column j to its owner
    for (int j = tid; j < Cc; j += kWThreads) {
      float s = 0.f;
#pragma unroll
      for (int w = 0; w < NW; w++) s += ps[w][j];
      const int o = j / cs;
      __hip_atomic_store(h1 + (((size_t)par * G + o) * G + g) * cs + (j - o * cs), sk_granule(s, tag),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // owner: lane = owned column, wave wv sums the sources g' = wv, wv + 8, ... in order
    bool to = a.inject && p == 0 && g == 0 && it == 0;  // fault injection (rspl_sg_debug_inject)
    if (lane < nc) {
      constexpr int kSrc = 9;  // <= 9 sources per wave: G <= 72 (ld <= 2112 at 32 rows per workgroup)
      const unsigned long long* src = h1 + ((size_t)par * G + g) * G * cs + lane;
      float l[kSrc];
      unsigned long long gv[kSrc];
      unsigned pend = 0;
#pragma unroll
      for (int i = 0; i < kSrc; i++) {
        l[i] = 0.f;
        if (wv + NW * i < G) pend |= 1u << i;
      }
      unsigned spins = 0;
      while (pend && !to) {
#pragma unroll
        for (int i = 0; i < kSrc; i++)
          if (pend >> i & 1) gv[i] = __hip_atomic_load(src + (size_t)(wv + NW * i) * cs, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
        for (int i = 0; i < kSrc; i++)
          if ((pend >> i & 1) && (unsigned)(gv[i] >> 32) == tag) {
            l[i] = __uint_as_float((unsigned)gv[i]);
            pend &= ~(1u << i);
          }
        if (!pend) break;
        if (++spins > a.spin_limit) { to = true; break; }
        for (int z = 0; z < a.sleep; z++) __builtin_amdgcn_s_sleep(1);
      }
      float T = 0.f;
#pragma unroll
      for (int i = 0; i < kSrc; i++) T += l[i];
      red[wv][lane] = T;
    }
    if (to) flag[0] = 1;
    __syncthreads();
    if (wv == 0 && lane < nc) {
      float T = 0.f;
#pragma unroll
      for (int w = 0; w < NW; w++) T += red[w][lane];
      const int j = c0 + lane;
      const float V = (j < n ? mu_in : nu_bin) / T;  // nu_j = mu_in for j < n: exp(norm)
      __hip_atomic_store(h2 + (size_t)par * G * cs + j, sk_granule(V, tag), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
    // hop 2: every column's V from its owner
    bool to2 = false;
    for (int j = tid; j < Cc; j += kWThreads) {
      const unsigned long long* q = h2 + (size_t)par * G * cs + j;
      unsigned long long gv = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      unsigned spins = 0;
      while ((unsigned)(gv >> 32) != tag && !to2) {
        if (++spins > a.spin_limit) { to2 = true; break; }
        for (int z = 0; z < a.sleep; z++) __builtin_amdgcn_s_sleep(1);
        gv = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      const float V = __uint_as_float((unsigned)gv);
      vs[j] = V;
      if (!(V >= kLo && V <= kHi)) flag[1] = 1;
    }
    if (to2) flag[0] = 1;
    __syncthreads();
    if (flag[0]) { failed = true; break; }
    const bool col_abs = flag[1] != 0, row_abs = flag[2 + (it & 1)] != 0;
    if (col_abs || row_abs) {  // rare: absorb the scalings into the log potentials, rebuild K from C
      if (row_abs) {
#pragma unroll
        for (int k = 0; k < RPW; k++) {
          if (lane == 0) as[wv + NW * k] += logf(ur[k] > 0.f ? ur[k] : 1.f);
          ur[k] = 1.f;
        }
      }
      if (col_abs)
        for (int j = tid; j < Q * 64; j += kWThreads) {
          bs[j] += logf(vs[j] > 0.f && j < Cc ? vs[j] : 1.f);
          vs[j] = 1.f;
        }
      __syncthreads();
      build_k(true);
      __syncthreads();  // every thread has read flag[1] before it is cleared
      if (tid == 0) flag[1] = 0;
      __syncthreads();
    }
  }
  if (failed) {
    if (tid == 0) __hip_atomic_store(a.err + p, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return;
  }
  // Z = ((couplings + u) + v) - norm (superglue.py:203, :219), own rows; u = a + log U, v = b + log V
  float* Z = a.Z + (size_t)p * ld * ld;
#pragma unroll
  for (int k = 0; k < RPW; k++) {
    const int r = wv + NW * k;
    if (r >= nr) continue;
    const float u = as[wv + NW * k] + logf(ur[k]);
    float c[Q];
    load_row(r, c);
    float* zr = Z + (size_t)(r0 + r) * ld;
#pragma unroll
    for (int q = 0; q < Q; q++) {
      const int j = lane + 64 * q;
      if (j < Cc) zr[j] = ((c[q] + u) + (bs[j] + logf(vs[j]))) - norm;
    }
  }
}

// ---------------------------------------------------------------------------
// decode (super_glue.cpp:339-367).  Pass 1: row / column argmax (strict '<'
// from -FLT_MAX: first maximum wins).  Pass 2: mutual check, exp, threshold.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void argmax_kernel(DecodeArgs a) {
  const int p = blockIdx.z, ld = a.nmax + 1;
  const int m = a.n0[p], n = a.n1[p];
  const float* Z = a.Z + (size_t)p * ld * ld;
  {  // rows: one wave per row
    const int i = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, lane = threadIdx.x & 63;
    if (i >= m) return;
    float best = -FLT_MAX;
    int idx = 0;
    for (int j = lane; j < n; j += 64) {
      const float x = Z[(size_t)i * ld + j];
      if (best < x) { best = x; idx = j; }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      const float ob = __shfl_xor(best, o);
      const int oi = __shfl_xor(idx, o);
      if (ob > best || (ob == best && oi < idx)) { best = ob; idx = oi; }
    }
    if (lane == 0) {
      a.max0[(size_t)p * a.nmax + i] = idx;
      a.val0[(size_t)p * a.nmax + i] = best;
    }
  }
}

// column argmax: 64 columns x 16 row groups per block; groups combined in LDS with the
// same strict '<' scan semantics (the smallest row index among equal maxima wins)
__global__ __launch_bounds__(1024) void col_argmax_kernel(DecodeArgs a) {
  __shared__ float bv[16][64];
  __shared__ int bi[16][64];
  const int p = blockIdx.z, ld = a.nmax + 1;
  const int m = a.n0[p], n = a.n1[p];
  const float* Z = a.Z + (size_t)p * ld * ld;
  const int c = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int j = blockIdx.x * 64 + c;
  float best = -FLT_MAX;
  int idx = 0;
  if (j < n) {
    const int per = (m + 15) / 16, i0 = rg * per, i1 = min(m, i0 + per);
#pragma unroll 8
    for (int i = i0; i < i1; i++) {
      const float x = Z[(size_t)i * ld + j];
      if (best < x) { best = x; idx = i; }
    }
    if (i0 >= i1) idx = 0x7fffffff;
  }
  bv[rg][c] = best;
  bi[rg][c] = idx;
  __syncthreads();
  if (rg == 0 && j < n) {
    float b = -FLT_MAX;
    int id = 0;
    bool any = false;
    for (int g = 0; g < 16; g++) {
      if (bi[g][c] == 0x7fffffff) continue;
      if (!any || b < bv[g][c]) { b = bv[g][c]; id = bi[g][c]; any = true; }
    }
    a.max1[(size_t)p * a.nmax + j] = id;
  }
}

__device__ __forceinline__ bool mutual0_of(const DecodeArgs& a, int p, int i, int m, int n) {
  if (n <= 0 || m <= 0) return false;
  const int j = a.max0[(size_t)p * a.nmax + i];
  return a.max1[(size_t)p * a.nmax + j] == i;
}

__global__ __launch_bounds__(256) void finalize_kernel(DecodeArgs a) {
  const int p = blockIdx.z;
  const int m = a.n0[p], n = a.n1[p];
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (blockIdx.y == 0) {
    if (t >= m) return;
    const bool mu = mutual0_of(a, p, t, m, n);
    const double ms = mu ? (double)expf(a.val0[(size_t)p * a.nmax + t]) : 0.0;  // std::exp(float)
    const bool valid = mu && ms > (double)a.threshold;
    a.ms0[(size_t)p * a.nmax + t] = ms;
    a.idx0[(size_t)p * a.nmax + t] = valid ? a.max0[(size_t)p * a.nmax + t] : -1;
  } else {
    if (t >= n) return;
    bool mu1 = false;
    int i = 0;
    if (m > 0) {
      i = a.max1[(size_t)p * a.nmax + t];
      mu1 = a.max0[(size_t)p * a.nmax + i] == t;
    }
    double ms1 = 0.0;
    bool valid1 = false;
    if (mu1) {
      const bool mu0 = mutual0_of(a, p, i, m, n);
      const double ms0 = mu0 ? (double)expf(a.val0[(size_t)p * a.nmax + i]) : 0.0;
      ms1 = ms0;
      valid1 = mu0 && ms0 > (double)a.threshold;
    }
    a.ms1[(size_t)p * a.nmax + t] = ms1;
    a.idx1[(size_t)p * a.nmax + t] = valid1 ? i : -1;
  }
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
hipError_t to_half_t(const float* W, int K, int N, _Float16* Wt, hipStream_t s) {
  hipLaunchKernelGGL(to_half_t_kernel, dim3((K * N + 255) / 256), dim3(256), 0, s, W, K, N, Wt);
  return hipGetLastError();
}

hipError_t gemm(const GemmArgs& a, int batch, hipStream_t s) {
  if (a.hB && !a.b_nt) {
    dim3 grid((a.N + 31) / 32, (a.M + 31) / 32, batch);
    if (a.epi == 1) hipLaunchKernelGGL(gemm_h_kernel<1>, grid, dim3(256), 0, s, a);
    else if (a.epi == 2) hipLaunchKernelGGL(gemm_h_kernel<2>, grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL(gemm_h_kernel<0>, grid, dim3(256), 0, s, a);
    return hipGetLastError();
  }
  if (a.b_nt) {
    dim3 grid((a.N + 63) / 64, (a.M + 63) / 64, batch);
    hipLaunchKernelGGL((gemm_kernel<0, true>), grid, dim3(256), 0, s, a);
    return hipGetLastError();
  }
  dim3 grid((a.N + 31) / 32, (a.M + 31) / 32, batch);
  if (a.epi == 1) {
    hipLaunchKernelGGL(gemm_sk_kernel<1>, grid, dim3(256), 0, s, a);
  } else if (a.epi == 2) {
    hipLaunchKernelGGL(gemm_sk_kernel<2>, grid, dim3(256), 0, s, a);
  } else {
    hipLaunchKernelGGL(gemm_sk_kernel<0>, grid, dim3(256), 0, s, a);
  }
  return hipGetLastError();
}

template <int MODE>
static hipError_t gemm_h_launch(const GemmHArgs& a, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute((const void*)gemm_hh_kernel<MODE>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize,
                                             (int)(2 * 64 * (kGhMaxK + 8) * sizeof(_Float16)));
    if (e != hipSuccess) return e;
    attr = true;
  }
  dim3 grid((a.N + 63) / 64, (a.M + 63) / 64);
  hipLaunchKernelGGL(gemm_hh_kernel<MODE>, grid, dim3(256), 2 * 64 * (a.K + 8) * sizeof(_Float16), s, a);
  return hipGetLastError();
}

template <int MODE, int TN>
static hipError_t gemm_rk_launch(const GemmHArgs& a, hipStream_t s) {
  const int ntn = (a.N + 32 * TN - 1) / (32 * TN), tiles = (a.M + 31) / 32 * ntn;
  hipLaunchKernelGGL((gemm_rk_kernel<MODE, TN>), dim3(tiles), dim3(256), 0, s, a, ntn);
  return hipGetLastError();
}

// the K-split register kernel where K allows, else the LDS-staged 64x64 one
hipError_t gemm_h(const GemmHArgs& a, int mode, hipStream_t s) {
  if (a.K > kGhMaxK || a.K % 16 != 0) return hipErrorInvalidValue;
  if (a.K % 64 == 0 && a.K <= 64 * kRdU && (!a.A2 || a.ksplit % 16 == 0)) {
    switch (mode) {
      case 0: return gemm_rk_launch<0, 1>(a, s);
      case 1: return gemm_rk_launch<1, 1>(a, s);
      case 2: return gemm_rk_launch<2, 1>(a, s);
      case 3: return gemm_rk_launch<3, 1>(a, s);
      case 4: return gemm_rk_launch<4, 1>(a, s);
    }
    return hipErrorInvalidValue;
  }
  switch (mode) {
    case 0: return gemm_h_launch<0>(a, s);
    case 1: return gemm_h_launch<1>(a, s);
    case 2: return gemm_h_launch<2>(a, s);
    case 3: return gemm_h_launch<3>(a, s);
    case 4: return gemm_h_launch<4>(a, s);
  }
  return hipErrorInvalidValue;
}

hipError_t gnn_layer(const LayerArgs& a, int B, hipStream_t s) {
  constexpr size_t lds = sizeof(_Float16) * 2 * 32 * kLdA;  // x | message, HID (>= the 32 x 776 q|k|v stage)
  static_assert(2 * kLdA >= 776, "q | k | v staging tile exceeds the LDS carve");
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute((const void*)layer_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                             (int)lds);
    if (e != hipSuccess) return e;
    attr = true;
  }
  LayerArgs la = a;
  const int sets = B * 2, tiles = (a.nmax + 31) / 32;
  la.nsets = sets;
  la.xps = sets <= 8 ? 8 / sets : 0;                                // XCDs per token set
  la.tpx = la.xps ? (tiles + la.xps - 1) / la.xps : 0;            // tiles per XCD
  if (la.xps)
    hipLaunchKernelGGL(layer_kernel, dim3(8 * la.tpx), dim3(512), lds, s, la);
  else
    hipLaunchKernelGGL(layer_kernel, dim3(tiles, sets), dim3(512), lds, s, la);
  return hipGetLastError();
}

// n-major fp16 weights Wt [N][K] -> 32x32x16 MFMA B-fragment order: block (nt, ks) = the 64 lanes'
// 16-byte operands of n-tile nt, k-step ks, lane L = r + 32 h holding Wt[32 nt + r][16 ks + 8 h ..];
// a wave's operand load is then one contiguous 1 KB read
__global__ void frag_kernel(const _Float16* Wt, int N, int K, _Float16* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;  // one 8-half operand
  const int KS = K / 16;
  if (i >= (N / 32) * KS * 64) return;
  const int L = i & 63, blk = i >> 6, nt = blk / KS, ks = blk - nt * KS, r = L & 31, h = L >> 5;
  *reinterpret_cast<uint4*>(out + (size_t)i * 8) =
      *reinterpret_cast<const uint4*>(Wt + (size_t)(32 * nt + r) * K + 16 * ks + 8 * h);
}

hipError_t to_frag(const _Float16* Wt, int N, int K, _Float16* out, hipStream_t s) {
  if (N % 32 || K % 16) return hipErrorInvalidValue;
  const int n = (N / 32) * (K / 16) * 64;
  hipLaunchKernelGGL(frag_kernel, dim3((n + 255) / 256), dim3(256), 0, s, Wt, N, K, out);
  return hipGetLastError();
}

hipError_t to_half(const float* x, _Float16* y, size_t n, hipStream_t s) {
  if (n) hipLaunchKernelGGL(to_half_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x, y, n);
  return hipGetLastError();
}

hipError_t prep(const PrepArgs& a, hipStream_t s) {
  const int waves = a.B * 2 * a.nmax;
  hipLaunchKernelGGL(prep_kernel, dim3((waves + 3) / 4), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t attention(const AttnArgs& a, int B, hipStream_t s) {
  hipLaunchKernelGGL(attn_kernel, dim3((a.nmax + 31) / 32, 4, B * 2), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t bins(const BinsArgs& a, int B, hipStream_t s) {
  hipLaunchKernelGGL(bins_kernel, dim3((2 * a.nmax + 256) / 256, B), dim3(256), 0, s, a);
  return hipGetLastError();
}

size_t sinkhorn_lds_bytes(int nmax, int G, bool slabs) {
  const size_t ld = nmax + 1, ldp = (ld + 3) & ~size_t(3), per = (ld + G - 1) / G;
  return sizeof(float) * (2 * ldp + 4 + (slabs ? 2 * per * ld : 0));
}

// the scaling-form kernel at 448 < nmax + 1 <= 640 (Q = 10, three rows per wave): G <= 16 workgroups of <= 48 rows
bool sinkhorn_sc10_ok(int nmax, int G) {
  const int ld = nmax + 1;
  return ld > kRbQ * 64 && ld <= 640 && G >= 1 && G <= 16 && (ld + G - 1) / G <= 48;
}

int sinkhorn_rb_rpw(int nmax, int G) {
  const int ld = nmax + 1, rs = (ld + G - 1) / G;
  if (ld > kRbQ * 64 || G < 1) return 0;
  if (G <= 4 && rs <= 16 * 8) return 8;
  if (G <= 8 && rs <= 16 * 4) return 4;
  if (G <= 16 && rs <= 16 * 2) return 2;
  if (G <= 32 && rs <= 16) return 1;
  return 0;
}

hipError_t sinkhorn(const SinkArgs& a, int B, hipStream_t s, hipEvent_t t0, hipEvent_t t1) {
  if (a.G < 1 || a.G > 1024) return hipErrorInvalidValue;
  dim3 grid(a.G, B);
  if (a.rb && a.sc && a.wide) {  // 640 < nmax + 1 <= 2112: two-hop column exchange
    if (!sinkhorn_wide_ok(a.nmax, a.G)) return hipErrorInvalidValue;
    hipExtLaunchKernelGGL((sinkhorn_w_kernel<kWideRPW, kWideQ>), grid, dim3(kWThreads), 0, s, t0, t1, 0, a);
    return hipGetLastError();
  }
  if (a.rb && a.sc && a.nmax + 1 > kRbQ * 64) {  // 448 < nmax + 1 <= 640: ten column sets per lane
    if (!sinkhorn_sc10_ok(a.nmax, a.G)) return hipErrorInvalidValue;
    hipExtLaunchKernelGGL((sinkhorn_sc_kernel<3, 16, 10>), grid, dim3(kSinkThreads), 0, s, t0, t1, 0, a);
    return hipGetLastError();
  }
  if (a.rb && a.sc) {  // scaling-form kernel: the workgroup count must match an instantiated (RPW, GM)
    switch (sinkhorn_rb_rpw(a.nmax, a.G)) {
#define RSPL_SK_SC(R, M)                                                                                     \
  case R:                                                                                                    \
    hipExtLaunchKernelGGL((sinkhorn_sc_kernel<R, M, kRbQ>), grid, dim3(kSinkThreads), 0, s, t0, t1, 0, a);   \
    break;
      RSPL_SK_SC(8, 4)
      RSPL_SK_SC(4, 8)
      RSPL_SK_SC(2, 16)
      RSPL_SK_SC(1, 32)
#undef RSPL_SK_SC
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
  if (a.rb) return hipErrorInvalidValue;  // (the row-block layout runs the scaling form only)
  const size_t full = sinkhorn_lds_bytes(a.nmax, a.G, true);
  if (full <= kSinkLdsMax) {
    static size_t attr = 0;
    if (attr < full) {
      hipError_t e = hipFuncSetAttribute((const void*)sinkhorn_kernel<true>,
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)full);
      if (e != hipSuccess) return e;
      attr = full;
    }
    hipExtLaunchKernelGGL((sinkhorn_kernel<true>), grid, dim3(kSinkThreads), (uint32_t)full, s, t0, t1, 0, a);
  } else {
    if (!a.cplT) return hipErrorInvalidValue;
    hipExtLaunchKernelGGL((sinkhorn_kernel<false>), grid, dim3(kSinkThreads),
                          (uint32_t)sinkhorn_lds_bytes(a.nmax, a.G, false), s, t0, t1, 0, a);
  }
  return hipGetLastError();
}

hipError_t decode(const DecodeArgs& a, int B, hipStream_t s) {
  hipLaunchKernelGGL(argmax_kernel, dim3((a.nmax * 64 + 255) / 256, 1, B), dim3(256), 0, s, a);
  hipLaunchKernelGGL(col_argmax_kernel, dim3((a.nmax + 63) / 64, 1, B), dim3(1024), 0, s, a);
  hipLaunchKernelGGL(finalize_kernel, dim3((a.nmax + 255) / 256, 2, B), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace sg
}  // namespace rspl
