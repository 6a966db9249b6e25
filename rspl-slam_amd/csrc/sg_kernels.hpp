#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace rspl {
namespace sg {

// C[m][n] = epi(alpha * sum_k A[m][k] B[k][n] + bias[n]) for m < M, n < N, per batch z.
//   A columns [0, ksplit) come from A, [ksplit, K) from A2 (both row stride lda).
//   B is [K][N] (ldb) or, with b_nt, [N][K] (ldb).
//   epi: 0 = none, 1 = ReLU, 2 = residual (C += result).
//   mcount / ncount (device, may be null) override M / N per batch.
struct GemmArgs {
  const float* A;
  const float* A2;
  int lda, ksplit;
  const float* B;
  int ldb, b_nt;
  const float* bias;
  float* C;
  int ldc;
  int M, N, K;
  float alpha;
  int epi;
  long long sA, sB, sC;
  const int* mcount;
  const int* ncount;
  const _Float16* hB;  // RSPL_PREC_FP16: weights as fp16 [N][K] (k contiguous), row stride ldbh
  int ldbh;
  int count_stride;  // ints between consecutive batches in mcount/ncount
};

// fp16 GNN GEMM (RSPL_PREC_FP16): C = epi(A B^T + bias), A [M][K] fp16 (columns [ksplit, K)
// from A2), B [N][K] fp16 (the transposed weights), K <= 512 and a multiple of 16.
//   mode 0: C32 = v          1: C16 = v          2: C16 = relu(v)
//        3: C32 += v, C16 = fp16(C32)  (the residual stream and its fp16 shadow)
//        4: QKV: channels [0, 512) -> C16 (Q | K, row stride ldc16); [512, 768) (V) ->
//           Vt[set][head][dim][token] (token = m % nmax, row stride ldv), so attention can
//           feed V^T to the MFMA straight from memory
struct GemmHArgs {
  const _Float16* A;
  const _Float16* A2;
  int lda, lda2, ksplit;
  const _Float16* B;
  int ldb;
  const float* bias;
  int M, N, K;
  float* C32;
  int ldc32;
  _Float16* C16;
  int ldc16;
  _Float16* Vt;
  int nmax, ldv;
};


// One fused AttentionalGNN layer (fp16 engine): attention -> [x | message] MLP -> residual ->
// the next layer's Q / K / V^T, per 32-token tile of one image (layer_kernel).  QK / Vt of the
// running layer are read (all tokens of the source image), the next layer's are written to the
// other buffer of the ping-pong pair.
struct LayerArgs {
  const _Float16* Qc;    // [T][256] q of this layer (head-contiguous), row-major
  const _Float16* Kc;    // k of this layer, MFMA-fragment order per (set, head, 32-key tile, k-step)
  const _Float16* Vc;    // v of this layer, fragment order per (set, head, key tile, d-half, key-half)
  _Float16* Qn;          // the next layer's (written unless last)
  _Float16* Kn;
  _Float16* Vn;
  float* X;              // [T][256] fp32 residual stream
  _Float16* Xh;          // [T][256] fp16 shadow
  const _Float16* W1;    // mlp.0 (merge folded in), [512 n][512 k] in B-fragment order (to_frag)
  const float* b1;
  const _Float16* W2;    // mlp.3 [256][512], fragment order
  const float* b2;
  const _Float16* Wq;    // next layer's q | k | v [768][256] (head-contiguous rows), fragment order
  const float* bq;
  const int* n0;
  const int* n1;
  int nmax, nt;          // tokens per image set; 32-key tiles per set in Kc / Vc (ldv / 32)
  int cross, last;
  int qkv_only;          // prologue: only phase (4) from the current x (layer 0's q / k / v)
  int nsets, xps, tpx;   // set by gnn_layer: token sets, XCDs per set (0 = plain grid), tiles per XCD
};

struct PrepArgs {
  const double* f0;   // [B][stride][259]
  const double* f1;
  const int* n0;      // device counts [B]
  const int* n1;
  int stride;         // features per batch entry
  int normalize;      // apply PointMatching::NormalizeKeypoints
  int width, height;
  int nmax;
  float* kin;         // [B][2][nmax][16] keypoint-encoder input (x, y, score, 0...)
  float* X;           // [B][2][nmax][256] descriptors
  int B;
};

struct AttnArgs {
  const float* qkv;   // [B][2][nmax][768] = Q | K | V, head-contiguous channels
  float* O;           // [B][2][nmax][256]
  const int* n0;
  const int* n1;
  int nmax;
  int cross;          // 0: self (source = same image), 1: cross
};

struct BinsArgs {
  float* cpl;         // [B][(nmax+1)^2], row stride nmax+1
  const int* n0;
  const int* n1;
  const float* alpha; // bin_score (device scalar)
  int nmax;
};

struct SinkArgs {
  const float* cpl;   // couplings [B][ld*ld]
  float* Z;           // [B][ld*ld]
  float* cplT;        // [B][ld*ld] transposed column slabs (scratch; only when the slabs exceed LDS)
  unsigned long long* ug;  // [B][ld] tagged u granules {f32 bits, tag}; row-block layout: [B][2][G][ld] partial sums
  unsigned long long* vg;  // [B][ld] tagged v granules
  unsigned seq;       // per-call tag base (never 0; granules start zeroed)
  unsigned spin_limit;  // bounded polls per granule before the exchange is declared timed out
  int inject;         // debug: workgroup 0 of pair 0 reports a timeout at iteration 0
  unsigned* err;      // [B] sticky timeout flags (host-mapped)
  const int* n0;
  const int* n1;
  int nmax, G, iters;
  int rb;             // 1: row-block layout (rows in registers, one exchange per iteration; with sc)
  int sleep;          // row-block layout: s_sleep(1) units between re-polls (run_sinkhorn: 1)
  int sc;             // with rb: the scaling-form kernel (register-resident exp(C + a + b), two mat-vecs per iteration)
  int wide;           // with sc: the wide two-hop kernel (640 < nmax + 1 <= 2112; ug / vg laid out as its hop buffers)
};

struct DecodeArgs {
  const float* Z;     // [B][ld*ld]
  const int* n0;
  const int* n1;
  int nmax;
  int* max0;          // [B][nmax]
  float* val0;
  int* max1;
  int32_t* idx0;      // [B][nmax]
  int32_t* idx1;
  double* ms0;
  double* ms1;
  float threshold;
};

hipError_t gemm(const GemmArgs& a, int batch, hipStream_t s);
// Wt[n][k] = (fp16) W[k][n] for a [K][N] fp32 weight (one-time, at create)
hipError_t to_half_t(const float* W, int K, int N, _Float16* Wt, hipStream_t s);
hipError_t to_frag(const _Float16* Wt, int N, int K, _Float16* out, hipStream_t s);
hipError_t gemm_h(const GemmHArgs& a, int mode, hipStream_t s);
hipError_t gnn_layer(const LayerArgs& a, int B, hipStream_t s);
// fp32 -> fp16, n elements
hipError_t to_half(const float* x, _Float16* y, size_t n, hipStream_t s);
hipError_t prep(const PrepArgs& a, hipStream_t s);
hipError_t attention(const AttnArgs& a, int B, hipStream_t s);
hipError_t bins(const BinsArgs& a, int B, hipStream_t s);
// t0 / t1 (may be null): events stamped with the kernel's own start / end (hipExtLaunchKernelGGL)
hipError_t sinkhorn(const SinkArgs& a, int B, hipStream_t s, hipEvent_t t0 = nullptr, hipEvent_t t1 = nullptr);
hipError_t decode(const DecodeArgs& a, int B, hipStream_t s);
// LDS bytes of one Sinkhorn workgroup (with or without the row / column slabs)
size_t sinkhorn_lds_bytes(int nmax, int G, bool slabs);
// rows per wave of the row-block Sinkhorn for G workgroups per pair (0: not supported)
int sinkhorn_rb_rpw(int nmax, int G);
// the scaling-form kernel for 448 < nmax + 1 <= 640 (ten 64-column sets per lane) takes this G
bool sinkhorn_sc10_ok(int nmax, int G);
// the wide two-hop scaling-form kernel (640 < nmax + 1 <= 2112): its workgroups per pair, the check, and
// its exchange buffers in granules per pair (hop 1 -> ug, hop 2 -> vg)
int sinkhorn_wide_groups(int nmax);
bool sinkhorn_wide_ok(int nmax, int G);
size_t sinkhorn_wide_hop1_len(int nmax);
size_t sinkhorn_wide_hop2_len(int nmax);
constexpr size_t kSinkLdsMax = 150 * 1024;  // slab budget per workgroup (160 KB LDS per CU)

}  // namespace sg
}  // namespace rspl
