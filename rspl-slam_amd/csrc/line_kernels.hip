// Line front end on gfx950: point-to-line assignment and shared-point line matching.
//
// Reference semantics:
//   AssignPointsToLines  src/line_processor.cc:163-216
//   MatchLines           src/line_processor.cc:221-283
// Both are integer / index work over a few hundred lines and keypoints per image: one 1024-thread
// workgroup per image (assignment) or per image pair (matching), tables in LDS, results in a fixed
// order (ballot compaction in keypoint order; integer counts), so they are bitwise reproducible.
// The arithmetic of the on-line test is the reference's (doubles; the distance through a float),
// with contraction off so every product is rounded as the reference's non-FMA x86 build rounds it.
#include <hip/hip_runtime.h>

#include "line_kernels.hpp"

namespace rspl {
namespace lines {

namespace {

// wave-wide exclusive prefix of a per-lane count
__device__ __forceinline__ int wave_excl(int v, int lane) {
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  return x - v;
}

// exclusive scan of data[0..n) in LDS by a 1024-thread workgroup (n <= 4 * 1024 per pass, then
// carried); returns the total.  `part` is 16 ints of LDS.
__device__ int block_excl_scan(int* data, int n, int* part) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  int carry = 0;
  for (int base = 0; base < n; base += 4096) {
    int v[4], s = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int i = base + 4 * tid + q;
      v[q] = i < n ? data[i] : 0;
      s += v[q];
    }
    const int ex = wave_excl(s, lane);
    if (lane == 63) part[wv] = ex + s;
    __syncthreads();
    int wbase = carry;
    for (int w = 0; w < wv; w++) wbase += part[w];
    int run = wbase + ex;
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int i = base + 4 * tid + q;
      if (i < n) data[i] = run;
      run += v[q];
    }
    int tot = 0;
    for (int w = 0; w < 16; w++) tot += part[w];
    __syncthreads();
    carry += tot;
  }
  return carry;
}

struct LineEq {
  double x1, y1, x2, y2, A, B, C, D, lox, hix, loy, hiy;
};

__device__ __forceinline__ LineEq line_eq(const double* l) {
#pragma clang fp contract(off)
  LineEq q;
  q.x1 = l[0];
  q.y1 = l[1];
  q.x2 = l[2];
  q.y2 = l[3];
  q.A = q.y2 - q.y1;
  q.B = q.x1 - q.x2;
  q.C = q.x2 * q.y1 - q.x1 * q.y2;
  q.D = sqrt(q.A * q.A + q.B * q.B);
  q.lox = q.x1 > q.x2 ? q.x2 : q.x1;
  q.hix = q.x1 > q.x2 ? q.x1 : q.x2;
  q.loy = q.y1 > q.y2 ? q.y2 : q.y1;
  q.hiy = q.y1 > q.y2 ? q.y1 : q.y2;
  return q;
}

// line_processor.cc:201-212: inside the 3-px-padded box, <= 6 px from the infinite line, and
// within 3 px of an endpoint or projecting between the endpoints
__device__ __forceinline__ bool on_line(const LineEq& q, double px, double py, float& d) {
#pragma clang fp contract(off)
  if (px < q.lox - 3 || px > q.hix + 3 || py < q.loy - 3 || py > q.hiy + 3) return false;
  d = (float)(fabs(q.A * px + q.B * py + q.C) / q.D);
  if (d > 6) return false;
  const double s1 = (q.x1 - px) * (q.x1 - px) + (q.y1 - py) * (q.y1 - py);
  const double s2 = (q.x2 - px) * (q.x2 - px) + (q.y2 - py) * (q.y2 - py);
  const double ls = q.D * q.D;
  return s1 <= 9 || s2 <= 9 || ((s1 < ls + s2) && (s2 < ls + s1));
}

}  // namespace

__global__ __launch_bounds__(1024) void assign_kernel(AssignArgs a) {
  extern __shared__ int cnt[];  // [max_lines + 1]
  __shared__ int part[16];
  __shared__ int total;
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int nl = min(a.n_lines[b], a.max_lines), np = a.n_points[b];
  const double* L = a.lines + (size_t)b * a.max_lines * 4;
  const double* pts = a.pts + (size_t)b * a.pt_batch + a.pt_xoff;
  int* offs = a.offsets + (size_t)b * (a.max_lines + 1);
  // pass 1: pairs per line (a wave per line, 64 keypoints per step)
  for (int l = wv; l < nl; l += 16) {
    const LineEq q = line_eq(L + 4 * l);
    int c = 0;
    for (int j0 = 0; j0 < np; j0 += 64) {
      const int j = j0 + lane;
      float d;
      const bool in = j < np && on_line(q, pts[(size_t)j * a.pt_stride], pts[(size_t)j * a.pt_stride + 1], d);
      c += __popcll(__ballot(in));
    }
    if (lane == 0) cnt[l] = c;
  }
  __syncthreads();
  const int tot = block_excl_scan(cnt, nl, part);
  if (tid == 0) total = tot;
  __syncthreads();
  for (int l = tid; l < nl; l += 1024) offs[l] = cnt[l];
  if (tid == 0) {
    offs[nl] = tot;
    a.status[b] = tot > a.cap ? 1 : 0;
  }
  if (total > a.cap) return;  // uniform
  // pass 2: the same tests, written compacted in keypoint order
  int* idx = a.idx + (size_t)b * a.cap;
  double* dist = a.dist + (size_t)b * a.cap;
  const unsigned long long below = (1ull << lane) - 1;
  for (int l = wv; l < nl; l += 16) {
    const LineEq q = line_eq(L + 4 * l);
    int base = cnt[l];
    for (int j0 = 0; j0 < np; j0 += 64) {
      const int j = j0 + lane;
      float d = 0.f;
      const bool in = j < np && on_line(q, pts[(size_t)j * a.pt_stride], pts[(size_t)j * a.pt_stride + 1], d);
      const unsigned long long m = __ballot(in);
      if (in) {
        const int pos = base + __popcll(m & below);
        idx[pos] = j;
        dist[pos] = (double)d;
      }
      base += __popcll(m);
    }
  }
}

// MatchLines.  Phases (workgroup barriers between them):
//   0  line_matches = -1; empty problems stop here (:226-231)
//   1  zero the count matrix; keypoint -> line incidence counts of both images (LDS atomics)
//   2  exclusive scans -> CSR starts of the inverse incidence (keypoint -> its lines)
//   3  fill the inverse incidence (order within a keypoint is irrelevant: only counts follow)
//   4  per match (q, t): M[l0][l1] += 1 for every line l0 through q and l1 through t (:249-259)
//   5  row maxima (first maximum: Eigen maxCoeff(&index)), one wave per row (:265-267)
//   6  per column j: first maximum over rows, the mutual test, score = v^2 / min(|P(l0)|, |P(l1)|)
//      >= 0.8 -> line_matches[l0] = j (:268-279)
__global__ __launch_bounds__(1024) void match_kernel(MatchArgs a) {
  __shared__ int c0[kMaxPointsLds + 1], c1[kMaxPointsLds + 1];
  __shared__ int f0[kMaxPointsLds], f1[kMaxPointsLds];
  __shared__ int part[16];
  __shared__ int rowloc[1024];
  const int p = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int s0 = a.set0 + p * a.step0, s1 = a.set1 + p * a.step1;
  const int n0 = a.n_lines0[s0], n1 = a.n_lines1[s1];
  const int np0 = a.n_points0[s0], np1 = a.n_points1[s1];
  const int* off0 = a.off0 + (size_t)s0 * (a.max_lines + 1);
  const int* off1 = a.off1 + (size_t)s1 * (a.max_lines + 1);
  const int* idx0 = a.idx0 + (size_t)s0 * a.cap;
  const int* idx1 = a.idx1 + (size_t)s1 * a.cap;
  int* out = a.out + (size_t)p * a.max_lines;
  for (int i = tid; i < n0; i += 1024) out[i] = -1;
  if (np0 == 0 || np1 == 0 || n0 == 0 || n1 == 0) return;
  if (a.status && (a.status[s0] | a.status[s1])) return;  // an assignment overflowed its capacity
  int* M = a.M + (size_t)p * a.max_lines * a.max_lines;
  int* inv0 = a.inv + (size_t)p * 2 * a.cap;
  int* inv1 = inv0 + a.cap;
  const int e0 = off0[n0], e1 = off1[n1];
  for (int i = tid; i < n0 * n1; i += 1024) M[i] = 0;
  for (int i = tid; i < np0; i += 1024) c0[i] = f0[i] = 0;
  for (int i = tid; i < np1; i += 1024) c1[i] = f1[i] = 0;
  __syncthreads();
  for (int e = tid; e < e0; e += 1024) atomicAdd(&c0[idx0[e]], 1);
  for (int e = tid; e < e1; e += 1024) atomicAdd(&c1[idx1[e]], 1);
  __syncthreads();
  block_excl_scan(c0, np0, part);
  block_excl_scan(c1, np1, part);
  if (tid == 0) {
    c0[np0] = e0;
    c1[np1] = e1;
  }
  __syncthreads();
  for (int l = wv; l < n0; l += 16)
    for (int e = off0[l] + lane; e < off0[l + 1]; e += 64) {
      const int q = idx0[e];
      inv0[c0[q] + atomicAdd(&f0[q], 1)] = l;
    }
  for (int l = wv; l < n1; l += 16)
    for (int e = off1[l] + lane; e < off1[l + 1]; e += 64) {
      const int t = idx1[e];
      inv1[c1[t] + atomicAdd(&f1[t], 1)] = l;
    }
  __syncthreads();
  const int nm = min(a.n_matches[p], a.max_matches);
  const int* mt = a.matches + (size_t)p * a.max_matches * 2;
  for (int m = tid; m < nm; m += 1024) {
    const int q = mt[2 * m], t = mt[2 * m + 1];
    if (q < 0 || q >= np0 || t < 0 || t >= np1) continue;  // checked by the host API
    for (int u = c0[q]; u < c0[q + 1]; u++) {
      int* row = M + (size_t)inv0[u] * n1;
      for (int v = c1[t]; v < c1[t + 1]; v++) atomicAdd(&row[inv1[v]], 1);
    }
  }
  __syncthreads();
  for (int r = wv; r < n0; r += 16) {  // row r: max over columns, first index
    int best = -1, bi = 0;
    for (int j = lane; j < n1; j += 64) {
      const int v = M[(size_t)r * n1 + j];
      if (v > best) {
        best = v;
        bi = j;
      }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      const int ov = __shfl_xor(best, o), oi = __shfl_xor(bi, o);
      if (ov > best || (ov == best && oi < bi)) {
        best = ov;
        bi = oi;
      }
    }
    if (lane == 0) rowloc[r] = bi;
  }
  __syncthreads();
  for (int j = wv; j < n1; j += 16) {  // column j: max over rows, first index
    int best = -1, bi = 0;
    for (int r = lane; r < n0; r += 64) {
      const int v = M[(size_t)r * n1 + j];
      if (v > best) {
        best = v;
        bi = r;
      }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      const int ov = __shfl_xor(best, o), oi = __shfl_xor(bi, o);
      if (ov > best || (ov == best && oi < bi)) {
        best = ov;
        bi = oi;
      }
    }
    if (lane == 0) {
      if (best < 2 || rowloc[bi] != j) continue;
      const int sz0 = off0[bi + 1] - off0[bi], sz1 = off1[j + 1] - off1[j];
      const float score = (float)(best * best) / (float)(sz0 < sz1 ? sz0 : sz1);
      if (score < 0.8f) continue;
      out[bi] = j;
    }
  }
}

// frame.cc:157-167 on the device: the stereo matches inside the disparity window, compacted in
// left-keypoint order (= the reference's loop order) by one workgroup -- ballots and a prefix over
// the 16 waves, no atomics -- so the kept list (and, past max_matches, which matches are dropped)
// is the same on every run.  *n_out = the full count; status = 1 when it exceeds max_matches.
__global__ __launch_bounds__(1024) void stereo_filter_kernel(StereoArgs a) {
#pragma clang fp contract(off)
  __shared__ int wcnt[16];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int nl = a.n_points[0], nr = a.n_points[1];
  int run = 0;
  for (int base = 0; base < nl; base += 1024) {
    const int q = base + tid;
    bool keep = false;
    int t = -1;
    if (q < nl) {
      t = a.idx[q];
      if (t >= 0 && t < nr) {
        const double* l = a.pts + (size_t)q * a.stride + a.xoff;
        const double* r = a.pts + a.pt_batch + (size_t)t * a.stride + a.xoff;
        const double dx = fabs(l[0] - r[0]), dy = fabs(l[1] - r[1]);
        keep = dx > a.min_x && dx < a.max_x && dy <= a.max_y;
      }
    }
    const unsigned long long bal = __ballot(keep);
    if (lane == 0) wcnt[wv] = __popcll(bal);
    __syncthreads();
    int before = run, total = 0;
    for (int w = 0; w < 16; w++) {
      const int c = wcnt[w];
      if (w < wv) before += c;
      total += c;
    }
    if (keep) {
      const int slot = before + __popcll(bal & ((1ull << lane) - 1ull));
      if (slot < a.max_matches) {
        a.matches[2 * slot] = q;
        a.matches[2 * slot + 1] = t;
      }
    }
    run += total;
    __syncthreads();  // wcnt is rewritten by the next round
  }
  if (tid == 0) {
    *a.n_out = run;
    *a.status = run > a.max_matches ? 1 : 0;
  }
}

__global__ __launch_bounds__(256) void right_lines_kernel(RightArgs a) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= a.n_lines[0]) return;
  const int j = a.line_matches[i];
  const bool ok = j > 0;  // frame.cc:190
  a.valid[i] = ok ? 1 : 0;
  for (int k = 0; k < 4; k++) a.out[4 * i + k] = ok ? a.lines_right[4 * j + k] : 0.0;
}

__global__ void set_counts_kernel(int* n_lines, int nl0, int nl1, int* n_points, const int32_t* counts,
                                  int* n_matches) {
  if (threadIdx.x == 0) {
    n_lines[0] = nl0;
    n_lines[1] = nl1;
    n_points[0] = counts[0];
    n_points[1] = counts[1];
    n_matches[0] = 0;
  }
}

// ---------------------------------------------------------------------------
// Detector front: one 512-thread workgroup per 32 x 16 tile of the half image.  The half image
// with a 2-pixel halo (clamped = BORDER_REPLICATE; each pixel (a + b + c + d + 2) >> 2 of its 2x2
// full-size block, cv::resize's 11-bit fixed point at scale 1/2) goes to LDS, then the L1 Sobel
// magnitudes with a 1-pixel halo (0 outside the image, as Canny's zero-padded magnitude rows),
// then each pixel's class: the TG22 / TG67 fixed-point sector (canny.cpp), its strict / non-strict
// neighbour tests, low / high thresholds.  Integer work: bit-exact with oracle/fld_ref.py.
// ---------------------------------------------------------------------------
constexpr int kCTX = 32, kCTY = 16;  // half-image tile per workgroup
__global__ __launch_bounds__(512) void canny_kernel(CannyArgs a) {
  constexpr int HX = kCTX + 4, HY = kCTY + 4, MX = kCTX + 2, MY = kCTY + 2;
  __shared__ int hs[HY * HX];
  __shared__ int mg[MY * MX];
  const int h = a.H / 2, w = a.W / 2;
  const int tx0 = blockIdx.x * kCTX, ty0 = blockIdx.y * kCTY, tid = threadIdx.x;
  for (int i = tid; i < HY * HX; i += 512) {
    const int ly = i / HX, lx = i - ly * HX;
    const int y = min(max(ty0 - 2 + ly, 0), h - 1), x = min(max(tx0 - 2 + lx, 0), w - 1);
    const uint8_t* r0 = a.img + (size_t)(2 * y) * a.stride + 2 * x;
    const uint8_t* r1 = r0 + a.stride;
    hs[i] = ((int)r0[0] + r0[1] + r1[0] + r1[1] + 2) >> 2;
  }
  __syncthreads();
  auto sob = [&](int ly, int lx, int& dx, int& dy) {  // (ly, lx) in hs coordinates, interior
    const int* p = hs + ly * HX + lx;
    dx = (p[-HX + 1] - p[-HX - 1]) + 2 * (p[1] - p[-1]) + (p[HX + 1] - p[HX - 1]);
    dy = (p[HX - 1] - p[-HX - 1]) + 2 * (p[HX] - p[-HX]) + (p[HX + 1] - p[-HX + 1]);
  };
  for (int i = tid; i < MY * MX; i += 512) {
    const int ly = i / MX, lx = i - ly * MX;
    const int y = ty0 - 1 + ly, x = tx0 - 1 + lx;
    int m = 0;
    if (y >= 0 && y < h && x >= 0 && x < w) {
      int dx, dy;
      sob(ly + 1, lx + 1, dx, dy);
      m = abs(dx) + abs(dy);
    }
    mg[i] = m;
  }
  __syncthreads();
  constexpr long long TG22 = 13573;  // (int)(0.41421356... * 2^15 + 0.5)
  for (int i = tid; i < kCTX * kCTY; i += 512) {
    const int ly = i / kCTX, lx = i - ly * kCTX;
    const int y = ty0 + ly, x = tx0 + lx;
    if (y >= h || x >= w) continue;
    int dx, dy;
    sob(ly + 2, lx + 2, dx, dy);
    const int* mp = mg + (ly + 1) * MX + (lx + 1);
    const int m = mp[0];
    uint8_t c = 1;
    if (m > a.low) {
      const long long xa = abs(dx), ya = (long long)abs(dy) << 15;
      const long long tg22x = xa * TG22;
      bool ok;
      if (ya < tg22x) {
        ok = m > mp[-1] && m >= mp[1];
      } else if (ya > tg22x + (xa << 16)) {
        ok = m > mp[-MX] && m >= mp[MX];
      } else {
        const int s = (dx ^ dy) < 0 ? -1 : 1;
        ok = m > mp[-MX - s] && m > mp[MX + s];
      }
      if (ok) c = m > a.high ? 2 : 0;
    }
    a.cls[(size_t)y * w + x] = c;
    a.half[(size_t)y * w + x] = (uint8_t)hs[(ly + 2) * HX + lx + 2];
  }
}

hipError_t canny_classes(const CannyArgs& a, hipStream_t s) {
  const int h = a.H / 2, w = a.W / 2;
  hipLaunchKernelGGL(canny_kernel, dim3((w + kCTX - 1) / kCTX, (h + kCTY - 1) / kCTY), dim3(512), 0, s, a);
  return hipGetLastError();
}

hipError_t set_counts(int* n_lines, int nl0, int nl1, int* n_points, const int32_t* counts, int* n_matches,
                      hipStream_t s) {
  hipLaunchKernelGGL(set_counts_kernel, dim3(1), dim3(64), 0, s, n_lines, nl0, nl1, n_points, counts, n_matches);
  return hipGetLastError();
}

hipError_t stereo_filter(const StereoArgs& a, int max_left, hipStream_t s) {
  (void)max_left;
  hipLaunchKernelGGL(stereo_filter_kernel, dim3(1), dim3(1024), 0, s, a);
  return hipGetLastError();
}

hipError_t right_lines(const RightArgs& a, int max_lines, hipStream_t s) {
  hipLaunchKernelGGL(right_lines_kernel, dim3((max_lines + 255) / 256), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t assign(const AssignArgs& a, int B, hipStream_t s) {
  hipLaunchKernelGGL(assign_kernel, dim3(B), dim3(1024), sizeof(int) * (a.max_lines + 1), s, a);
  return hipGetLastError();
}

hipError_t match(const MatchArgs& a, int P, hipStream_t s) {
  hipLaunchKernelGGL(match_kernel, dim3(P), dim3(1024), 0, s, a);
  return hipGetLastError();
}

}  // namespace lines
}  // namespace rspl
