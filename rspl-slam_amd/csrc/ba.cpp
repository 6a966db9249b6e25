// Local BA handle: C ABI (include/rspl.h) over ba_kernels.hip.
// Mirrors LocalmapOptimization (src/g2o_optimization/g2o_optimization.cc:21-252):
//   optimize(10) with Huber kernels -> chi2/depth outlier levels, kernels removed ->
//   initializeOptimization(0) + optimize(5) -> inlier flags -> write back T_wc, points, lines.
// The Levenberg-Marquardt control (g2o OptimizationAlgorithmLevenberg: tau 1e-5,
// good-step factor clamp [1/3, 2/3], ni doubling, 10 trials) runs on the host.  Each
// trial is 3 kernels (Schur chunks; LDL^T solve + candidate poses; landmark update + cost,
// see ba_kernels.hip); the last block of the cost kernel posts {chi2, scale, fail} and a
// sequence number to a pinned host-mapped mailbox that the host spins on (no stream
// synchronisation, no D2H copy on the critical path).  Host->device traffic goes through
// one pinned staging buffer (async copies only).
#include <immintrin.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <numeric>
#include <string>
#include <type_traits>
#include <memory>
#include <vector>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <thread>

#include "ba_kernels.hpp"
#include "common.hpp"
#include "ba_stage.hpp"

using namespace rspl;

namespace rspl {
namespace ba {
struct StagedCall;  // one call's host staging (below)
}
}  // namespace rspl

struct rspl_ba {
  rspl_ba_config cfg{};
  hipStream_t stream = nullptr;
  Arena arena;
  int maxE = 0, maxL = 0, maxK = 0, maxV = 0;
  // candidate state (ping-pong partners of the call buffer's T / X / L)
  double *Tb, *Xb, *Lb;
  // per-edge linearisation records
  double *err, *Hpp_e, *bp_e, *Hll_e, *bl_e, *Hpl_e;
  // spare linearisation set (per-edge records + landmark blocks): each trial's candidate is
  // linearised speculatively into it, and becomes current by a pointer swap when accepted
  double *Hpp_s, *bp_s, *Hll_es, *bl_es, *Hpl_s, *Hll_s, *bl_s;
  uint8_t* lm_act2;
  // system
  double *Hll, *bl, *bp, *S, *x, *partial, *partial2;
  unsigned* lm_ctr;  // [max_lines] line-landmark tickets (zeroed at create, re-armed by the kernel)
  unsigned long long* prof = nullptr;  // RSPL_BA_PROF: timing trace of one trial per call
  int prof_nb[5] = {0, 0, 0, 0, 0};    // its pair_chunk / update_errors grid sizes, group blocks, nchk, K
  rspl::ba::Active prof_A{};           // the traced trial's chunk geometry (chunk_geo)
  // landmark CSR (filled on the device) and the Schur chunk / pose-pair sums
  double *chunk, *pairfin;
  unsigned* pair_ctr;  // [npairs] chunk tickets (zeroed at create, re-armed by the kernel)
  int *pp_cnt, *pp_off;  // [npairs * nchk (+1)] edge pairs per Schur chunk, segment offsets
  size_t chunk_slots = 0;  // Schur chunks the buffers hold (capacity pose pairs x landmark ranges)
  int4* pp_buf = nullptr;  // edge-pair list {e1, e2, landmark, 0}, growable
  size_t pp_cap = 0;      // capacity in pairs
  // per-call inputs (cameras, T / X / L, edges, reduced pose ids, landmark offsets, pose pairs,
  // zeroed level / fill / flags / out), laid out exactly like the staging buffer's call
  // region: one upload per call (capacity fixed at create).  One per staging slot: the tracking
  // thread uploads the next staged call into its slot's buffer behind the current call's last kernels
  // (preupload_next), so a call's upload is off its own critical path
  char* cbuf[2] = {nullptr, nullptr};
  // pinned, host-mapped staging for uploads; the final kernel writes results straight into it.
  // Two slots: the tracking thread's next queued call is staged into one while the running call
  // reads its results from the other
  char* stage[2] = {nullptr, nullptr};
  char* stage_dev[2] = {nullptr, nullptr};
  size_t stage_cap[2] = {0, 0};
  // host-mapped mailbox
  ba::Mail* mail = nullptr;
  ba::Mail* mail_dev = nullptr;
  unsigned long long seq = 0;
  ba::Stager stg;  // host staging into landmark-CSR order (scratch and host workers reused across calls)
  // landmark sharding (rspl_ba_set_shard): this rank keeps the edges of landmarks g % nranks == rank
  int rank = 0, nranks = 1;
  rspl_allreduce_fn allreduce = nullptr;
  void* ar_ctx = nullptr;
  double* red = nullptr;       // [6 maxK + kMaxRanks + 3] lambda-init / cost all-reduce buffer
  ba::LmCtrl* lmctl = nullptr;  // device-side LM control (fast path, unsharded)
  double* lm_trace = nullptr;   // RSPL_BA_LMTRACE: per-trial decisions (debug)
  double* gbuf = nullptr;      // final gather buffer (grown on demand)
  size_t gcap = 0;
  double* pdg = nullptr;       // per-block pose-diagonal partials of the first pass (grown on demand)
  size_t pdg_cap = 0;
  // kernel timing (rspl_ba_kernel_timing): HIP events around each device-LM trial's two launches on
  // the BA stream, every ktime_every-th call; totals per launch kind (0: Schur chunks + fused solve,
  // 1: update + speculative linearisation) over the trials that did work
  int ktime_every = 0;
  unsigned long long ncalls = 0;
  bool ktime_on = false;
  std::vector<hipEvent_t> kev;  // 3 per trial
  std::vector<int> kev_eval;    // event-triple indices of the trials that did work (this call)
  int kev_used = 0;
  double kt_ms[2] = {0, 0};
  long long kt_n[2] = {0, 0};
  // native tracking thread (rspl_ba_submit / rspl_ba_join): a FIFO of calls run in order by one host
  // thread of the handle, as the reference's TrackingThread drains _tracking_data_buffer
  struct Job {
    const rspl_ba_problem* pr;
    rspl_ba_result* res;
    std::shared_ptr<ba::StagedCall> sc;  // its host staging (made by the staging thread)
    int state;                            // 0 waiting, 1 being staged, 2 staged
  };
  std::thread worker;
  std::thread stager;  // stages the next queued call into the free slot while the worker runs one
  bool slot_busy[2] = {false, false};
  std::mutex qmu;
  std::condition_variable qcv;  // the worker waits for jobs; submitters for room; joiners for idle
  std::deque<Job> jobs;
  bool busy = false, quit = false;
  bool tracking_call = false;  // run_call is running on the tracking thread (preupload_next may look ahead)
  int q_err = 0;                // first failed call since the last join
  std::string q_msg;
  long long q_done = 0, q_iters = 0;
  double q_ms = 0.0;
  // per-call host timeline (rspl_ba_trace): a ring of the last kTraceCap calls, under qmu
  static constexpr int kTraceCap = 4096;
  std::vector<double> trace;  // kTraceCap x RSPL_BA_TRACE_W
  long long trace_n = 0;      // records written since the last read
  unsigned grew = 0;          // device-side buffers grown during the running call (tracking thread)
  int line_jac = 0;           // rspl_ba_set_line_jacobian: 0 g2o's central difference, 1 its analytic limit
};

namespace {

constexpr int kMaxCams = 16;
constexpr int kMaxRanks = 64;
constexpr int kParEdges = 8192;  // staging on the host workers from this many edges
constexpr int kChunkWaves = 1024; // Schur chunk waves of one dispatch round (one wave per SIMD)
constexpr int kEventTrials = 64;  // timing-event triples created by rspl_ba_kernel_timing
// the rank's sum all-reduce, stream-ordered on the BA stream
int allreduce(rspl_ba* b, double* d, size_t n) {
  const int rc = b->allreduce(b->ar_ctx, d, n, b->stream);
  if (rc) {
    set_error("BA shard all-reduce failed (rank %d of %d, %zu doubles, rc %d)", b->rank, b->nranks, n, rc);
    return RSPL_E_DEVICE;
  }
  return RSPL_OK;
}

inline size_t al256(size_t x) { return (x + 255) & ~size_t(255); }

// per-call upload layout (staging call region == device call buffer)
struct CallLayout {
  size_t cams, T, X, L, obs, type, pose, lm, cam, gmap, lm_pose, pidx, lm_off, lm_act, pairs, ltab, level, flags, out,
      bytes;
  CallLayout() = default;
  CallLayout(int ncam, int np, int nq, int nl, int E, size_t nobs) {  // nobs: observation doubles (4 / 8 per edge)
    const size_t nL = (size_t)nq + nl;
    size_t so = 0;
    auto place = [&](size_t n) {
      const size_t o = so;
      so = al256(so + n);
      return o;
    };
    cams = place(sizeof(double) * 5 * ncam); T = place(sizeof(double) * 8 * np); X = place(sizeof(double) * 3 * nq);
    L = place(sizeof(double) * 6 * nl); obs = place(sizeof(double) * nobs); type = place(E);
    pose = place(4 * (size_t)E); lm = place(4 * (size_t)E); cam = place(4 * (size_t)E); gmap = place(4 * (size_t)E);
    lm_pose = place(4 * (size_t)E);
    pidx = place(4 * (size_t)np); lm_off = place(4 * (nL + 1)); lm_act = place(nL);
    pairs = place(8 * (size_t)np * (np + 1) / 2);
    // line-workgroup table: at most one entry per line landmark plus one per kLineBlk line edges (a
    // landmark with more edges is split) -- sized tight, as the call uploads [0, bytes) in one copy
    const size_t line_edges = nobs >= 4 * (size_t)E ? (nobs - 4 * (size_t)E) / 4 : 0;
    ltab = place(16 * ((size_t)nl + line_edges / ba::kLineBlk + 2));
    level = place(E); flags = place(4 * sizeof(int)); out = place(8 * sizeof(double));  // zeros
    bytes = so;
  }
};

// result layout written by the final kernel into the mapped staging buffer
struct DownLayout {
  size_t inl, T, X, L, bytes;
  DownLayout() = default;
  DownLayout(int np, int nq, int nl, int E) {
    inl = 0; T = al256(E); X = T + al256(sizeof(double) * 8 * np); L = X + al256(sizeof(double) * 3 * nq);
    bytes = L + al256(sizeof(double) * 6 * nl);
  }
};

// RSPL_BA_TIMING=1: host stage times of a call, microseconds since the previous mark, one stderr line
struct HostMarks {
  static bool on() {
    static const bool t = getenv("RSPL_BA_TIMING") != nullptr;
    return t;
  }
  std::chrono::steady_clock::time_point t[16];
  const char* name[16];
  int n = 0;
  void mark(const char* s) {
    if (on() && n < 16) {
      name[n] = s;
      t[n++] = std::chrono::steady_clock::now();
    }
  }
  void print(const char* label) const {
    if (!on()) return;
    fprintf(stderr, "%s", label);
    for (int i = 1; i < n; i++)
      fprintf(stderr, " %s %.1f", name[i], std::chrono::duration<double, std::micro>(t[i] - t[i - 1]).count());
    fprintf(stderr, "\n");
  }
};

// CLOCK_MONOTONIC seconds (Python's time.perf_counter clock): the per-call timeline's time base
double mono_s() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

}  // namespace

// one call's host staging: its slot and what the device part needs of it
struct rspl::ba::StagedCall {
  int slot = 0;
  int rc = RSPL_OK;  // staging failed (argument errors): reported when the call's turn comes
  std::string msg;
  int E = 0, Ep = 0, K = 0, n_lblk = 0;
  size_t pair_bound = 0;
  CallLayout cl;
  DownLayout dl;
  HostMarks tm;
  double tr[RSPL_BA_TRACE_W] = {};  // its host timeline record (rspl_ba_trace)
  bool uploaded = false;  // its inputs already queued for upload into cbuf[slot] (tracking thread only)
};

namespace {

template <typename F>
void carve(F& ar, rspl_ba* b) {
  const size_t E = b->maxE, NL = b->maxL, K = b->maxK, nq = b->cfg.max_points, nl = b->cfg.max_lines;
  auto take = [&](auto*& p, size_t n) {
    using Tp = std::remove_pointer_t<std::remove_reference_t<decltype(p)>>;
    if constexpr (std::is_same_v<F, Arena>) p = ar.template take<Tp>(n ? n : 1);
    else ar.template take<Tp>(n ? n : 1);
  };
  take(b->Tb, K * 8); take(b->Xb, nq * 3); take(b->Lb, nl * 6);
  take(b->err, E * 4); take(b->Hpp_e, E * 21); take(b->bp_e, E * 6); take(b->Hll_e, E * 16);
  take(b->bl_e, E * 4); take(b->Hpl_e, E * 24);
  take(b->Hpp_s, E * 21); take(b->bp_s, E * 6); take(b->Hll_es, E * 16); take(b->bl_es, E * 4); take(b->Hpl_s, E * 24);
  take(b->Hll_s, NL * 16); take(b->bl_s, NL * 4);
  take(b->lm_act2, NL);
  take(b->Hll, NL * 16); take(b->bl, NL * 4); take(b->bp, K * 6);
  // block partials: edge-per-thread kernels (E / 256) and landmark-group kernels (NL * 8 / 256)
  const size_t nblk = std::max(E / 256, NL * 8 / 256) + 2;
  // partial also holds the setup kernel's per-block costs: the landmark groups plus the line
  // workgroups (at most one per line landmark plus one per kLineBlk line edges)
  // (+ 1024: update_errors' XCD-aligned grid rounds the landmark blocks up to whole ranges per XCD)
  take(b->S, 36 * K * K); take(b->x, 6 * K); take(b->partial, nblk + NL + E / ba::kLineBlk + 1032);
  // partial2: scale partials, and the pose-diagonal partials (K x E/256 x 6) of the lambda init
  take(b->partial2, std::max(std::max((size_t)b->maxV / 256, nblk) + 1026, K * (E / 256 + 1) * 6));
  take(b->lm_ctr, nl);
  const size_t npairs = K * (K + 1) / 2, nchk = std::max<size_t>((NL + ba::kLmChunk - 1) / ba::kLmChunk, 1);
  // pair_ctr: + the solve ticket
  take(b->chunk, npairs * nchk * 48); take(b->pairfin, npairs * 48 + 8); take(b->pair_ctr, npairs + 1);
  take(b->red, 6 * K + kMaxRanks + 8);
  take(b->lmctl, 2);
  take(b->pp_cnt, npairs * nchk); take(b->pp_off, npairs * nchk + 1);
  b->chunk_slots = npairs * nchk;
}

// Staging slots are allocated at create for the handle's capacities (stage_bytes), so in use this never
// grows; it stays for a handle created without them.  The slot being grown is not in use (a slot is
// handed out only when its previous call has finished), so the new buffer is taken before the old one
// is released and nothing waits for the stream.
int ensure_stage(rspl_ba* b, int slot, size_t bytes, bool* grew = nullptr) {
  if (bytes <= b->stage_cap[slot]) return RSPL_OK;
  const size_t cap = std::max(bytes, b->stage_cap[slot] * 2);
  char *nh = nullptr, *nd = nullptr;
  RSPL_HIP(hipHostMalloc((void**)&nh, cap, hipHostMallocMapped | hipHostMallocCoherent));
  if (hipHostGetDevicePointer((void**)&nd, nh, 0) != hipSuccess) {
    (void)hipHostFree(nh);
    set_error("BA staging slot: no device mapping");
    return RSPL_E_DEVICE;
  }
  if (b->stage[slot]) (void)hipHostFree(b->stage[slot]);
  b->stage[slot] = nh;
  b->stage_dev[slot] = nd;
  b->stage_cap[slot] = cap;
  if (grew) *grew = true;
  return RSPL_OK;
}

// Spin on the mailbox until the kernel chain tagged `seq` has posted; surface stream
// errors and bound the wait.
int wait_mail(rspl_ba* b, unsigned long long seq, double* v) {
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  for (unsigned it = 1;; it++) {
    if (__atomic_load_n(&b->mail->seq, __ATOMIC_ACQUIRE) == seq) break;
    if ((it & 4095) == 0) {
      const hipError_t q = hipStreamQuery(b->stream);
      if (q != hipSuccess && q != hipErrorNotReady) {
        set_error("BA stream failed: %s", hipGetErrorString(q));
        return RSPL_E_DEVICE;
      }
      if (q == hipSuccess) {
        if (__atomic_load_n(&b->mail->seq, __ATOMIC_ACQUIRE) == seq) break;
        set_error("BA mailbox: stream idle but sequence %llu never posted", seq);
        return RSPL_E_DEVICE;
      }
      if (clk::now() - t0 > std::chrono::seconds(60)) {
        set_error("BA mailbox: timed out waiting for sequence %llu", seq);
        return RSPL_E_DEVICE;
      }
    }
    _mm_pause();
  }
  if (v) {
    volatile const double* mv = b->mail->v;
    for (int k = 0; k < 4; k++) v[k] = mv[k];
  }
  return RSPL_OK;
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

// RSPL_BA_PROF: one traced trial per call -> one stderr line of in-kernel spans (us, from the
// device's 100 MHz wall clock): pair_chunk first..last block start, span; gap to the solve;
// solve phases (assembly, factor, back-substitution, poses); gap; update_errors span
void report_prof(rspl_ba* b) {
  std::vector<unsigned long long> h(ba::kProfLen);
  if (hipStreamSynchronize(b->stream) != hipSuccess ||
      hipMemcpy(h.data(), b->prof, sizeof(unsigned long long) * h.size(), hipMemcpyDeviceToHost) != hipSuccess)
    return;
  // per kernel: first block start, then over blocks [b0, b1) the latest stamp of each slot
  auto us = [](unsigned long long a, unsigned long long c) { return c && a ? ((double)c - (double)a) / 100.0 : -1.0; };
  auto first = [&](int off, int b0, int b1) {
    unsigned long long t = ~0ull;
    for (int i = b0; i < std::min(b1, 4096); i++)
      if (h[off + 4 * i]) t = std::min(t, h[off + 4 * i]);
    return t;
  };
  auto last = [&](int off, int b0, int b1, int slot) {
    unsigned long long t = 0;
    for (int i = b0; i < std::min(b1, 4096); i++) t = std::max(t, h[off + 4 * i + slot]);
    return t;
  };
  const int npc = b->prof_nb[0], nue = b->prof_nb[1], nbu = b->prof_nb[2];
  const unsigned long long p0 = first(ba::kProfPc, 0, npc), u0 = first(ba::kProfUe, 0, nue);
  fprintf(stderr,
          "ba_prof us: pcstarts %.1f pcloop %.1f pcticket %.1f pcend %.1f gap %.1f asm %.1f factor %.1f back %.1f"
          " poses %.1f gap %.1f uestarts %.1f loaded %.1f grpdone %.1f groupsend %.1f lineswait %.1f linescomp %.1f"
          " linesend %.1f sApanel %.1f sAtrail %.1f sBpanel %.1f sBtrail %.1f\n",
          us(p0, last(ba::kProfPc, 0, npc, 0)), us(p0, last(ba::kProfPc, 0, npc, 1)),
          us(p0, last(ba::kProfPc, 0, npc, 2)), us(p0, last(ba::kProfPc, 0, npc, 3)),
          us(last(ba::kProfPc, 0, npc, 3), h[0]), us(h[0], h[1]), us(h[1], h[2]), us(h[2], h[3]), us(h[3], h[4]),
          us(h[4], u0), us(u0, last(ba::kProfUe, 0, nue, 0)), us(u0, last(ba::kProfUe, 0, nbu, 1)),
          us(u0, last(ba::kProfUe, 0, nbu, 2)), us(u0, last(ba::kProfUe, 0, nbu, 3)),
          us(u0, last(ba::kProfUe, nbu, nue, 1)), us(u0, last(ba::kProfUe, nbu, nue, 2)),
          us(u0, last(ba::kProfUe, nbu, nue, 3)), us(h[1], h[5]), us(h[5], h[6]), us(h[6], h[7]), us(h[7], h[8]));
  fprintf(stderr,
          "ba_prof setup us: landmarks %.1f +pdiag %.1f lines %.1f +pdiag %.1f pairs %.1f | blocks done %.1f scan %.1f "
          "pose diagonals + control %.1f\n",
          us(h[9], h[ba::kProfX]), us(h[9], h[ba::kProfX + 1]), us(h[9], h[ba::kProfX + 2]),
          us(h[9], h[ba::kProfX + 3]), us(h[9], h[ba::kProfX + 4]), us(h[9], h[10]),
          us(h[10], h[11]), us(h[11], h[12]));
  {  // per chunk: start -> loop done, quantiles over the diagonal / off-diagonal pose pairs' chunks
    const int nchk = b->prof_nb[3], K = b->prof_nb[4];
    std::vector<double> dg, od;
    for (int c = 0; c < std::min(npc, 4096) && nchk > 0; c++) {
      const unsigned long long t0 = h[ba::kProfPc + 4 * c], t1 = h[ba::kProfPc + 4 * c + 1];
      if (!t0 || !t1) continue;
      int pr = ba::chunk_geo(b->prof_A, c).pr, a = 0, base = 0;
      while (pr >= base + (K - a)) base += K - a++;
      ((pr - base == 0) ? dg : od).push_back(((double)t1 - (double)t0) / 100.0);
    }
    auto q = [](std::vector<double>& v, double f) {
      if (v.empty()) return -1.0;
      std::sort(v.begin(), v.end());
      return v[std::min(v.size() - 1, (size_t)(f * v.size()))];
    };
    fprintf(stderr, "ba_chunks us: diag50 %.1f diag90 %.1f diagmax %.1f off50 %.1f off90 %.1f offmax %.1f "
            "ndiag %zu noff %zu\n", q(dg, 0.5), q(dg, 0.9), q(dg, 1.0), q(od, 0.5), q(od, 0.9), q(od, 1.0),
            dg.size(), od.size());
  }
  {  // line workgroups of update_errors: per block start -> operands (wait), -> evaluations (comp), -> end
    std::vector<double> w, c, e, tot;
    for (int i = nbu; i < std::min(nue, 4096); i++) {
      const unsigned long long* r = &h[ba::kProfUe + 4 * i];
      if (!r[0] || !r[1] || !r[2] || !r[3]) continue;
      w.push_back((r[1] - (double)r[0]) / 100.0);
      c.push_back((r[2] - (double)r[1]) / 100.0);
      e.push_back((r[3] - (double)r[2]) / 100.0);
      tot.push_back((r[3] - (double)u0) / 100.0);
    }
    auto q = [](std::vector<double> v, double f) {
      if (v.empty()) return -1.0;
      std::sort(v.begin(), v.end());
      return v[std::min(v.size() - 1, (size_t)(f * v.size()))];
    };
    fprintf(stderr, "ba_lines us (p50/p90/max): operands %.1f/%.1f/%.1f evals %.1f/%.1f/%.1f tail %.1f/%.1f/%.1f "
            "end %.1f/%.1f/%.1f n %zu\n", q(w, .5), q(w, .9), q(w, 1), q(c, .5), q(c, .9), q(c, 1), q(e, .5), q(e, .9),
            q(e, 1), q(tot, .5), q(tot, .9), q(tot, 1), w.size());
  }
  b->prof_nb[0] = 0;
  (void)hipMemset(b->prof, 0, sizeof(unsigned long long) * ba::kProfLen);
}

// an accepted candidate becomes the current state; with lin also its speculative linearisation
void accept_swap(rspl_ba* b, ba::Problem& P, ba::Lin& Lr, ba::Sys& S, bool lin) {
  std::swap(P.T, P.Tn);
  std::swap(P.X, P.Xn);
  std::swap(P.L, P.Ln);
  if (!lin) return;
  std::swap(b->Hpp_e, b->Hpp_s); std::swap(b->bp_e, b->bp_s); std::swap(b->Hll_e, b->Hll_es);
  std::swap(b->bl_e, b->bl_es); std::swap(b->Hpl_e, b->Hpl_s);
  std::swap(b->Hll, b->Hll_s); std::swap(b->bl, b->bl_s);
  Lr.Hpp = b->Hpp_e; Lr.bp = b->bp_e; Lr.Hll = b->Hll_e; Lr.bl = b->bl_e; Lr.Hpl = b->Hpl_e;
  S.Hll = b->Hll; S.bl = b->bl;
}

// the second optimize()'s setup launch queued right behind the first optimize()'s first batch of trials,
// before the host has seen them: a no-op unless that optimize() stopped within the batch (setup_dev's gate);
// then the second optimize() starts from it instead of queueing its own after the host's round trip
struct SpecSetup {
  ba::Active A2{};           // the second optimize()'s active structure (levels, landmark activity)
  uint8_t* level = nullptr;  // where its setup classifies the edges
  int iters2 = 0;
  bool queued = false;  // queued behind a batch of the first optimize()'s trials
  bool extra = false;   // a later batch was queued after it: that setup did nothing (and none followed yet)
  bool topped_up = false;  // the first optimize() needed trials beyond its first batch
};

// the call's final kernel (inlier flags, final T / X / L into the staging slot) queued right behind the
// last optimize()'s trials instead of after the host has seen that optimize() stop: it reads the control
// after the last queued trial and does nothing unless the optimize() stopped there (then the host queues
// top-up trials and another one).  q: the sequence the finish that will post carries.
struct SpecFinish {
  bool on = false;
  ba::Lin L{};
  int E = 0;
  const int* gmap = nullptr;
  uint8_t* inl = nullptr;
  double *Th = nullptr, *Xh = nullptr, *Lh = nullptr;
  unsigned long long q = 0;
};

// optimize(iters) with the LM control on the device (fast path, unsharded): the first errors, the
// first linearisation and the control's initialisation, then `iters` trials queued back to back
// with no host round trip -- each trial's last kernel takes the accept / reject decision (ba::LmCtrl)
// and the next trial's kernels read it.  The host waits once, for the trial that stops the
// optimize(); when rejected trials leave iterations undone it queues more.  At the end the host
// pointer view follows the device's current bank.
void preupload_next(rspl_ba* b);

int optimize_dev(rspl_ba* b, ba::Problem& P, ba::Lin& Lr, ba::Sys& S, const ba::Active& A, int iters,
                 double* chi2_out, int* done_out, uint8_t* cls_level, bool build_pp, SpecFinish* fin,
                 SpecSetup* nxt, bool setup_done) {
  hipStream_t st = b->stream;
  S.lm = b->lmctl;
  S.lm_slot = 0;
  static const bool trace = getenv("RSPL_BA_LMTRACE") != nullptr;
  if (trace && !b->lm_trace) {
    RSPL_HIP(hipMalloc((void**)&b->lm_trace, sizeof(double) * 8 * 64));
    RSPL_HIP(hipMemset(b->lm_trace, 0, sizeof(double) * 8 * 64));
  }
  S.lm_trace = trace ? b->lm_trace + (iters == 10 ? 0 : 8 * 32) : nullptr;
  // errors, cost and linearisation at the current state (with cls_level: the second optimize's
  // outlier levels and landmark activity first) + computeLambdaInit into the control (slot 0);
  // nothing is posted: the host waits for the trials only
  if (setup_done) {
    // (queued behind the previous optimize()'s trials: SpecSetup)
  } else {
    const size_t need = (size_t)ba::setup_pdg_len(A);
    if (need > b->pdg_cap) {  // grow (the stream may still read the old buffer)
      RSPL_HIP(hipStreamSynchronize(st));
      if (b->pdg) (void)hipFree(b->pdg);
      b->pdg = nullptr;
      b->pdg_cap = 0;
      const size_t cap = std::max(need, (size_t)1 << 14);
      RSPL_HIP(hipMalloc((void**)&b->pdg, sizeof(double) * cap));
      b->pdg_cap = cap;
      b->grew |= 4;
    }
    ba::Sys Su = S;  // RSPL_BA_PROF: the first optimize's setup phases too
    Su.prof = b->prof && !b->prof_nb[0] && !cls_level ? b->prof : nullptr;
    RSPL_HIP(ba::setup_dev(P, Lr, A, Su, cls_level, cls_level ? const_cast<uint8_t*>(A.lm_act) : nullptr, iters,
                           build_pp ? b->pp_cnt : nullptr, b->pp_off, b->pp_buf, b->pdg, st));
  }
  unsigned long long q = b->seq;
  const unsigned long long q_first = b->seq + 1;
  ba::Lin Ls = Lr;
  Ls.Hpp = b->Hpp_s; Ls.bp = b->bp_s; Ls.Hll = b->Hll_es; Ls.bl = b->bl_es; Ls.Hpl = b->Hpl_s;
  ba::Sys Ss = S;
  Ss.Hll = b->Hll_s; Ss.bl = b->bl_s;
  int queued = 0;
  const int kev0 = b->kev_used;  // this optimize's first event triple
  auto enqueue = [&](int n) -> int {
    for (int k = 0; k < n; k++, queued++) {
      q = ++b->seq;
      ba::Spec sp{Ls, Ss};
      const bool traced = b->prof && queued == 3 && !b->prof_nb[0];
      if (traced) {
        S.prof = b->prof;
        b->prof_nb[0] = ba::chunk_count(A);
        b->prof_A = A;
        b->prof_nb[1] = ba::update_errors_blocks(A) + A.n_lblk;
        b->prof_nb[2] = ba::update_errors_blocks(A);
        b->prof_nb[3] = A.nchk;
        b->prof_nb[4] = A.K;
      }
      S.lm_slot = queued & 1;
      S.lm_post = k == n - 1;
      hipEvent_t* ev = nullptr;
      if (b->ktime_on) {
        if ((size_t)3 * (b->kev_used + 1) > b->kev.size()) {  // (pre-created by rspl_ba_kernel_timing)
          for (int i = 0; i < 3; i++) {
            hipEvent_t e;
            RSPL_HIP(hipEventCreate(&e));
            b->kev.push_back(e);
          }
          b->grew |= 8;
        }
        ev = &b->kev[3 * (size_t)b->kev_used++];
      }
      const hipError_t e = ba::trial_dev(P, Lr, A, S, q, st, sp, ev);
      S.prof = nullptr;
      if (e != hipSuccess) {
        set_error("BA trial launch failed: %s", hipGetErrorString(e));
        return RSPL_E_DEVICE;
      }
    }
    return RSPL_OK;
  };
  int rc;
  unsigned long long q_last = 0;
  auto enqueue_batch = [&](int n) -> int {  // n trials (+ the speculative finish behind them)
    int r;
    if ((r = enqueue(n))) return r;
    q_last = b->seq;
    if (fin) {
      ba::Sys Sf = S;
      Sf.lm = b->lmctl;
      Sf.lm_slot = queued & 1;  // the control slot the last queued trial writes
      Sf.prof = nullptr;
      fin->q = ++b->seq;
      fin->on = true;
      RSPL_HIP(ba::finish(P, fin->L, fin->E, fin->gmap, fin->inl, fin->Th, fin->Xh, fin->Lh, Sf, fin->q, st));
    }
    return RSPL_OK;
  };
  if ((rc = enqueue_batch(iters))) return rc;
  if (fin) preupload_next(b);  // the call's last kernels are queued: the next call's upload behind them
  // the second optimize()'s setup behind each batch, gated on the control the batch's last trial writes (the
  // one behind the batch in which this optimize() stops is the one that runs)
  auto queue_spec_setup = [&]() -> int {
    if (!nxt || (size_t)ba::setup_pdg_len(nxt->A2) > b->pdg_cap) return RSPL_OK;
    ba::Sys S2 = S;
    S2.lm = b->lmctl;
    S2.lm_slot = 0;
    S2.prof = nullptr;
    S2.lm_trace = nullptr;
    RSPL_HIP(ba::setup_dev(P, Lr, nxt->A2, S2, nxt->level, const_cast<uint8_t*>(nxt->A2.lm_act), nxt->iters2,
                           nullptr, b->pp_off, b->pp_buf, b->pdg, st, queued & 1, &Ls, &Ss));
    nxt->queued = true;
    nxt->extra = false;
    return RSPL_OK;
  };
  if ((rc = queue_spec_setup())) return rc;
  double v[4];
  for (;;) {
    // wait for the stopping trial (trials queued after it post nothing) or the last queued one
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    for (unsigned spin = 1;; spin++) {
      // seqlock read: the next trial may be posting while we read; v is s1's iff vseq is still s1
      const unsigned long long s1 = __atomic_load_n(&b->mail->seq, __ATOMIC_ACQUIRE);
      if (s1 >= q_first && s1 <= q_last) {
        volatile const double* mv = b->mail->v;
        for (int k = 0; k < 4; k++) v[k] = mv[k];
        __atomic_thread_fence(__ATOMIC_ACQUIRE);
        if (__atomic_load_n(&b->mail->vseq, __ATOMIC_ACQUIRE) == s1 && (s1 == q_last || v[3] != 0.0)) break;
      } else if (fin && s1 == fin->q) {  // the speculative finish already posted over the stopping trial's
        volatile const double* mv = b->mail->v;  // seq (it posts only the seq: v / vseq stay the trial's)
        for (int k = 0; k < 4; k++) v[k] = mv[k];
        __atomic_thread_fence(__ATOMIC_ACQUIRE);
        const unsigned long long vs = __atomic_load_n(&b->mail->vseq, __ATOMIC_ACQUIRE);
        if (vs >= q_first && vs <= q_last && v[3] != 0.0) break;
      }
      if ((spin & 4095) == 0) {
        const hipError_t e = hipStreamQuery(st);
        if (e != hipSuccess && e != hipErrorNotReady) {
          set_error("BA stream failed: %s", hipGetErrorString(e));
          return RSPL_E_DEVICE;
        }
        if (e == hipSuccess && __atomic_load_n(&b->mail->seq, __ATOMIC_ACQUIRE) < q_first) {
          set_error("BA mailbox: stream idle but no trial posted");
          return RSPL_E_DEVICE;
        }
        if (clk::now() - t0 > std::chrono::seconds(60)) {
          set_error("BA mailbox: timed out waiting for the LM trials");
          return RSPL_E_DEVICE;
        }
      }
      _mm_pause();
    }
    if (v[3] != 0.0) {
      if (b->ktime_on) {  // the trials up to the stopping one did work (later ones are no-ops)
        unsigned long long s1 = __atomic_load_n(&b->mail->seq, __ATOMIC_ACQUIRE);
        for (unsigned long long t = q_first; t <= s1 && t <= q_last; t++) b->kev_eval.push_back(kev0 + (int)(t - q_first));
      }
      break;
    }
    // rejected trials left iterations to do: queue one trial per remaining iteration
    if (nxt) nxt->extra = nxt->topped_up = true;
    if ((rc = enqueue_batch(std::max(1, iters - (int)v[1])))) return rc;
    if ((rc = queue_spec_setup())) return rc;
  }
  S.lm = nullptr;
  if (v[2] != 0.0) accept_swap(b, P, Lr, S, true);  // the device's current bank is the host's spare one
  *chi2_out = v[0];
  *done_out = (int)v[1];
  return RSPL_OK;
}

bool dev_lm(const rspl_ba* b, const ba::Active& A, int iters) {
  return b->allreduce == nullptr && iters > 0 && ba::fast_path(A.K);
}

// one g2o SparseOptimizer::optimize(iters); device LM only: cls_level -- classify the edges into it
// first (the second optimize's levels), build_pp -- build the Schur chunks' edge-pair lists (see
// setup_dev); the caller does both itself otherwise
int optimize(rspl_ba* b, ba::Problem& P, ba::Lin& Lr, ba::Sys& S, const ba::Active& A, int iters,
             double* chi2_out, int* done_out, uint8_t* cls_level = nullptr, bool build_pp = false,
             SpecFinish* fin = nullptr, SpecSetup* nxt = nullptr, bool setup_done = false) {
  hipStream_t st = b->stream;
  double v[4];
  int rc;
  const bool sh = b->allreduce != nullptr;
  if (dev_lm(b, A, iters))
    return optimize_dev(b, P, Lr, S, A, iters, chi2_out, done_out, cls_level, build_pp, fin, nxt, setup_done);
  const int n6 = 6 * A.K;
  double* so = b->red + n6 + b->nranks;  // this rank's {chi2, scale, fail} (S.shard_out)
  unsigned long long q = ++b->seq;
  RSPL_HIP(ba::compute_errors(P, Lr, A, S, q, st));
  if (sh) {  // sum the ranks' costs (and, before the first iteration, the lambda-init diagonals)
    if (iters > 0) {
      RSPL_HIP(ba::linearize(P, Lr, A, S, true, st));
      RSPL_HIP(ba::shard_fold(A, S, b->red, b->rank, b->nranks, st));
      if ((rc = allreduce(b, b->red, ba::shard_red_len(A.K, b->nranks)))) return rc;
      RSPL_HIP(ba::shard_post(S, b->red, n6, b->nranks, 0, 0, q, st));
    } else {
      if ((rc = allreduce(b, so, 3))) return rc;
      RSPL_HIP(ba::shard_post(S, b->red, n6, b->nranks, 1, 0, q, st));
    }
  } else if (iters > 0) {  // the first linearisation does not depend on the cost: queue it right behind
    RSPL_HIP(ba::linearize(P, Lr, A, S, true, st));
    q = ++b->seq;
    RSPL_HIP(ba::post(S, q, st, &A));  // posts chi2 (S.out[0]) and the max diagonal (S.out[2])
  }
  if ((rc = wait_mail(b, q, v))) return rc;
  double currentChi = v[0];
  double lambda = 1e-5 * v[2], ni = 2;  // computeLambdaInit: tau * max diagonal
  int done = 0;
  for (int it = 0; it < iters; it++) {
    // iterations after the first start from an accepted candidate, whose linearisation the
    // speculative pass of that trial already produced (now current after the swap)
    double rho = 0;
    int qmax = 0;
    do {
      q = ++b->seq;
      if (sh) {  // Schur chunks -> sum of the reduced systems -> identical solve on every rank
        RSPL_HIP(ba::trial_chunks(P, Lr, A, S, lambda, st));
        if ((rc = allreduce(b, S.pairfin, (size_t)A.npairs * 48 + 1))) return rc;
        RSPL_HIP(ba::trial_solve(P, Lr, A, S, lambda, st));
        if ((rc = allreduce(b, so, 3))) return rc;
        RSPL_HIP(ba::shard_post(S, b->red, n6, b->nranks, 1, ba::fast_path(A.K) ? 1 : 0, q, st));
      }
      // speculative linearisation of the candidate into the spare set: the GPU runs it while the
      // host reads the mailbox, so the next iteration's first kernel is already queued when the
      // host decides (a rejected trial wastes it; the current set stays).  On the fast path it
      // is fused into the trial's last kernel, otherwise queued behind the trial.
      ba::Lin Ls = Lr;
      Ls.Hpp = b->Hpp_s; Ls.bp = b->bp_s; Ls.Hll = b->Hll_es; Ls.bl = b->bl_es; Ls.Hpl = b->Hpl_s;
      ba::Sys Ss = S;
      Ss.Hll = b->Hll_s; Ss.bl = b->bl_s;
      bool fused = false;
      if (!sh) {
          ba::Spec sp{Ls, Ss};
        const bool traced = b->prof && it == 3 && qmax == 0 && !b->prof_nb[0];
        if (traced) {
          S.prof = sp.Ss.prof = b->prof;
          b->prof_nb[0] = ba::chunk_count(A);
          b->prof_A = A;
        b->prof_A = A;
          b->prof_nb[1] = ba::update_errors_blocks(A) + A.n_lblk;
          b->prof_nb[2] = ba::update_errors_blocks(A);
        }
        RSPL_HIP(ba::trial(P, Lr, A, S, lambda, q, st, it + 1 < iters ? &sp : nullptr, &fused));
        S.prof = nullptr;
      }
      if (it + 1 < iters && !fused) {
        ba::Problem Pc = P;
        Pc.T = P.Tn; Pc.X = P.Xn; Pc.L = P.Ln;
        RSPL_HIP(ba::linearize(Pc, Ls, A, Ss, false, st));
      }
      if ((rc = wait_mail(b, q, v))) return rc;
      if (getenv("RSPL_BA_LMTRACE"))
        fprintf(stderr, "lmtrace-host iters=%d it %d q %d chi2 %.17g scale %.6g fail %g lambda %.6g chi0 %.17g\n", iters, it,
                qmax, v[0], v[1], v[3], lambda, currentChi);
      const bool ok = v[3] == 0.0;
      const double tempChi = ok ? v[0] : std::numeric_limits<double>::max();
      rho = currentChi - tempChi;
      const double scale = ok ? v[1] + 1e-3 : 1.0;
      rho /= scale;
      if (rho > 0 && std::isfinite(tempChi) && ok) {
        double alpha = 1. - std::pow(2 * rho - 1, 3);
        alpha = std::min(alpha, 2. / 3.);
        lambda *= std::max(1. / 3., alpha);
        ni = 2;
        currentChi = tempChi;
        // accept: the candidate becomes the current state, and its speculative linearisation
        // (when one was made) the current one
        accept_swap(b, P, Lr, S, it + 1 < iters);
      } else {
        lambda *= ni;  // reject: the current state was never modified (no restore needed)
        ni *= 2;
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
  b->maxV = cfg->max_poses + cfg->max_points + cfg->max_lines;
  Sizer sz;
  carve(sz, b);
  int rc = b->arena.reserve(sz.used);
  if (rc) { delete b; return rc; }
  carve(b->arena, b);
  // the BA is a host-driven chain of short kernels on the tracking thread's critical path:
  // give its stream the highest priority so each trial's kernels dispatch ahead of queued
  // SuperPoint/SuperGlue work instead of waiting behind it
  int prio_lo = 0, prio_hi = 0;
  (void)hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi);
  {
    const size_t cbytes = CallLayout(kMaxCams, b->maxK, cfg->max_points, cfg->max_lines, b->maxE, 8 * (size_t)b->maxE).bytes;
    const char* what = nullptr;
    hipError_t e = hipSuccess;
    auto step = [&](hipError_t r, const char* w) {
      if (e == hipSuccess && r != hipSuccess) {
        e = r;
        what = w;
      }
    };
    step(hipStreamCreateWithPriority(&b->stream, hipStreamNonBlocking, prio_hi), "hipStreamCreateWithPriority");
    if (e == hipSuccess)
      step(hipHostMalloc((void**)&b->mail, sizeof(ba::Mail), hipHostMallocMapped | hipHostMallocCoherent), "hipHostMalloc(mailbox)");
    if (e == hipSuccess) step(hipHostGetDevicePointer((void**)&b->mail_dev, b->mail, 0), "hipHostGetDevicePointer(mailbox)");
    for (int i = 0; i < 2 && e == hipSuccess; i++) step(hipMalloc((void**)&b->cbuf[i], cbytes), "hipMalloc(call buffer)");
    if (e == hipSuccess) step(hipMemset(b->lm_ctr, 0, sizeof(unsigned) * std::max(b->cfg.max_lines, 1)), "hipMemset(lm_ctr)");
    if (e == hipSuccess)
      step(hipMemset(b->pair_ctr, 0, sizeof(unsigned) * (b->maxK * (b->maxK + 1) / 2 + 1)), "hipMemset(pair_ctr)");
    if (e != hipSuccess) {
      set_error("BA stream / mailbox allocation failed: %s: %s (call buffer %zu bytes, arena %zu bytes)", what,
                hipGetErrorString(e), cbytes, b->arena.size);
      rspl_ba_destroy(b);
      return RSPL_E_DEVICE;
    }
  }
  memset(b->mail, 0, sizeof(ba::Mail));
  // everything a call can need, allocated once here for the handle's capacities (never inside a call:
  // a pinned allocation or a hipFree there stalls the device and the pipeline beside it): both staging
  // slots, the pose-diagonal partials of the first pass and the edge-pair lists (sum over landmarks of
  // k^2 edge pairs, k = edges of the landmark; sized for 8 edges per landmark on average -- beyond that
  // the list still grows on demand, flagged in the call's trace record)
  {
    const size_t sb = std::max(CallLayout(kMaxCams, b->maxK, cfg->max_points, cfg->max_lines, b->maxE,
                                          8 * (size_t)b->maxE).bytes,
                               DownLayout(b->maxK, cfg->max_points, cfg->max_lines, b->maxE).bytes);
    ba::Active Amax{};  // the largest call: every landmark, the most line workgroups
    Amax.nL = b->maxL;
    Amax.K = b->maxK;
    Amax.n_lblk = cfg->max_lines + b->maxE / ba::kLineBlk + 2;
    const size_t pdg = (size_t)ba::setup_pdg_len(Amax);
    const size_t pp = std::max<size_t>((size_t)1 << 16, 8 * (size_t)b->maxE);
    if (ensure_stage(b, 0, sb) || ensure_stage(b, 1, sb) ||
        hipMalloc((void**)&b->pdg, sizeof(double) * pdg) != hipSuccess ||
        hipMalloc((void**)&b->pp_buf, sizeof(int4) * pp) != hipSuccess) {
      set_error("BA staging / scratch allocation failed");
      rspl_ba_destroy(b);
      return RSPL_E_DEVICE;
    }
    b->pdg_cap = pdg;
    b->pp_cap = pp;
  }
  b->trace.assign((size_t)rspl_ba::kTraceCap * RSPL_BA_TRACE_W, 0.0);
  if (getenv("RSPL_BA_PROF") &&
      (hipMalloc((void**)&b->prof, sizeof(unsigned long long) * ba::kProfLen) != hipSuccess ||
       hipMemset(b->prof, 0, sizeof(unsigned long long) * ba::kProfLen) != hipSuccess)) {
    set_error("BA trace allocation failed");
    rspl_ba_destroy(b);
    return RSPL_E_DEVICE;
  }
  *out = b;
  return RSPL_OK;
}

extern "C" int rspl_ba_use_reserved_cus(rspl_ba* b, int reserve_cus) {
  RSPL_CHECK_ARG(b, "rspl_ba_use_reserved_cus: NULL handle");
  hipStream_t ns = nullptr;
  if (reserve_cus > 0) {
    std::vector<uint32_t> mask;
    int rc = cu_mask(reserve_cus, true, mask);
    if (rc) return rc;
    RSPL_HIP(hipExtStreamCreateWithCUMask(&ns, (uint32_t)mask.size(), mask.data()));
  } else {
    int lo = 0, hi = 0;
    RSPL_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
    RSPL_HIP(hipStreamCreateWithPriority(&ns, hipStreamNonBlocking, hi));
  }
  RSPL_HIP(hipStreamSynchronize(b->stream));
  RSPL_HIP(hipStreamDestroy(b->stream));
  b->stream = ns;
  return RSPL_OK;
}

namespace {
bool queue_active(rspl_ba* b);
}

extern "C" int rspl_ba_set_shard(rspl_ba* b, int rank, int nranks, rspl_allreduce_fn fn, void* ctx) {
  RSPL_CHECK_ARG(b, "rspl_ba_set_shard: NULL handle");
  RSPL_CHECK_ARG(!queue_active(b), "rspl_ba_set_shard: calls are queued on the tracking thread (rspl_ba_join first)");
  RSPL_CHECK_ARG(nranks >= 1 && nranks <= kMaxRanks && rank >= 0 && rank < nranks, "rank %d of %d (1..%d ranks)", rank,
                 nranks, kMaxRanks);
  RSPL_CHECK_ARG(nranks == 1 || fn, "an all-reduce function is required for nranks > 1");
  // with fn the sharded schedule runs even for one rank (every all-reduce an identity): the
  // collective path can be exercised on a single GPU; fn == NULL with one rank = unsharded
  b->rank = rank;
  b->nranks = nranks;
  b->allreduce = fn;
  b->ar_ctx = ctx;
  return RSPL_OK;
}

extern "C" void rspl_ba_destroy(rspl_ba* b) {
  if (!b) return;
  if (b->worker.joinable()) {  // finish the queued calls, then stop the tracking thread
    {
      std::lock_guard<std::mutex> lk(b->qmu);
      b->quit = true;
    }
    b->qcv.notify_all();
    b->worker.join();
    b->stager.join();
  }
  for (hipEvent_t e : b->kev) (void)hipEventDestroy(e);
  if (b->stream) (void)hipStreamSynchronize(b->stream);
  if (b->gbuf) (void)hipFree(b->gbuf);
  if (b->pdg) (void)hipFree(b->pdg);
  b->arena.release();
  for (char* cb : b->cbuf)
    if (cb) (void)hipFree(cb);
  if (b->pp_buf) (void)hipFree(b->pp_buf);
  if (b->prof) (void)hipFree(b->prof);
  for (char* sg : b->stage)
    if (sg) (void)hipHostFree(sg);
  if (b->mail) (void)hipHostFree(b->mail);
  if (b->stream) (void)hipStreamDestroy(b->stream);
  delete b;
}

namespace {
int ba_local_impl(rspl_ba* b, const rspl_ba_problem* pr, rspl_ba_result* res);
int stage_call(rspl_ba* b, int slot, const rspl_ba_problem* pr, rspl_ba_result* res, ba::StagedCall& c);
int run_call(rspl_ba* b, const ba::StagedCall& c, const rspl_ba_problem* pr, rspl_ba_result* res, double* tr);
void push_trace(rspl_ba* b, const double* tr);

// calls queued on / running in the native tracking thread (rspl_ba_submit) and not yet joined
bool queue_active(rspl_ba* b) {
  std::lock_guard<std::mutex> lk(b->qmu);
  return !b->jobs.empty() || b->busy;
}

void begin_call(rspl_ba* b) {
  b->ktime_on = b->ktime_every > 0 && b->ncalls++ % (unsigned long long)b->ktime_every == 0;
  b->kev_used = 0;
  b->kev_eval.clear();
}

// A device-side failure can return while the call's kernel chain is still queued or running (a
// mailbox timeout, a failed all-reduce): drain the stream before anything of the handle is reused
// (the next call restages the mapped buffers the old chain reads) and re-arm the cross-call
// tickets and release flags the chain may have left half-counted.  If the drain itself fails the
// device is gone and the handle must be recreated (the error says so).
int end_call(rspl_ba* b, int rc) {
  if (rc != RSPL_E_DEVICE) return rc;
  const std::string msg = rspl_last_error();
  if (hipStreamSynchronize(b->stream) != hipSuccess ||
      hipMemset(b->lm_ctr, 0, sizeof(unsigned) * std::max(b->cfg.max_lines, 1)) != hipSuccess ||
      hipMemset(b->pair_ctr, 0, sizeof(unsigned) * (b->maxK * (b->maxK + 1) / 2 + 1)) != hipSuccess) {
    set_error("%s; the BA stream could not be drained: recreate the handle", msg.c_str());
    return rc;
  }
  set_error("%s", msg.c_str());
  return rc;
}
}  // namespace

extern "C" int rspl_ba_kernel_timing(rspl_ba* b, int every) {
  RSPL_CHECK_ARG(b && every >= 0, "rspl_ba_kernel_timing: NULL handle or every < 0");
  RSPL_CHECK_ARG(!queue_active(b), "rspl_ba_kernel_timing: calls are queued on the tracking thread (rspl_ba_join first)");
  // the events of a call's trials, created here rather than inside a timed call (a call queues 15 trials
  // plus top-ups after rejected ones; more are created on demand, flagged in the trace record)
  for (size_t n = b->kev.size(); every > 0 && n < 3 * (size_t)kEventTrials; n++) {
    hipEvent_t e;
    RSPL_HIP(hipEventCreate(&e));
    b->kev.push_back(e);
  }
  b->ktime_every = every;
  b->ncalls = 0;
  return RSPL_OK;
}

extern "C" int rspl_ba_set_line_jacobian(rspl_ba* b, int analytic) {
  RSPL_CHECK_ARG(b && (analytic == 0 || analytic == 1), "rspl_ba_set_line_jacobian: NULL handle or mode not 0 / 1");
  RSPL_CHECK_ARG(!queue_active(b), "rspl_ba_set_line_jacobian: calls are queued on the tracking thread (rspl_ba_join first)");
  b->line_jac = analytic;
  return RSPL_OK;
}

extern "C" int rspl_ba_trace(rspl_ba* b, double* out, int cap, int* n) {
  RSPL_CHECK_ARG(b && n && cap >= 0 && (out || cap == 0), "rspl_ba_trace: NULL argument or cap < 0");
  std::lock_guard<std::mutex> lk(b->qmu);
  const long long have = std::min<long long>(b->trace_n, rspl_ba::kTraceCap);
  const long long first = b->trace_n - have;  // oldest record still in the ring
  const int m = (int)std::min<long long>(have, cap);
  for (int i = 0; i < m; i++) {
    const size_t r = (size_t)((first + i) % rspl_ba::kTraceCap);
    std::copy(b->trace.begin() + r * RSPL_BA_TRACE_W, b->trace.begin() + (r + 1) * RSPL_BA_TRACE_W,
              out + (size_t)i * RSPL_BA_TRACE_W);
  }
  *n = m;
  b->trace_n = 0;
  return RSPL_OK;
}

extern "C" int rspl_ba_kernel_times(rspl_ba* b, double* ms, long long* launches) {
  RSPL_CHECK_ARG(b && ms && launches, "rspl_ba_kernel_times: NULL argument");
  for (int i = 0; i < 2; i++) {
    ms[i] = b->kt_ms[i];
    launches[i] = b->kt_n[i];
    b->kt_ms[i] = 0;
    b->kt_n[i] = 0;
  }
  return RSPL_OK;
}

extern "C" int rspl_ba_local(rspl_ba* b, const rspl_ba_problem* pr, rspl_ba_result* res) {
  if (!b) return ba_local_impl(b, pr, res);
  // the synchronous call stages into slot 0 and runs on the BA stream: never beside queued calls
  RSPL_CHECK_ARG(!queue_active(b), "rspl_ba_local: calls are queued on the tracking thread (rspl_ba_join first)");
  begin_call(b);
  return end_call(b, ba_local_impl(b, pr, res));
}

// ---- native tracking thread ----
// Two host threads per handle: the staging thread stages each queued call (validation, landmark-CSR
// scatter, tables: host work only) into a free staging slot as soon as it is queued; the tracking
// thread runs the staged calls on the device in order.  The next call's staging therefore overlaps
// the current call's LM trials instead of preceding them on the tracking thread's critical path; the
// calls still run one at a time and in submission order, each on the inputs given at submission.
namespace {
constexpr size_t kTrackingBuffer = 2;  // map_builder.cc:176: the feature thread waits while 2 are queued

void staging_loop(rspl_ba* b) {
  (void)hipSetDevice(b->cfg.device);
  std::unique_lock<std::mutex> lk(b->qmu);
  for (;;) {
    rspl_ba::Job* j = nullptr;
    int slot = -1;
    b->qcv.wait(lk, [&] {
      j = nullptr;
      for (rspl_ba::Job& q : b->jobs)
        if (q.state == 0) {
          j = &q;
          break;
        }
      slot = !b->slot_busy[0] ? 0 : !b->slot_busy[1] ? 1 : -1;
      return (j && slot >= 0) || (b->quit && !j);
    });
    if (!j) return;  // quit with every queued call staged
    j->state = 1;    // (deque elements stay in place while others are pushed; j is popped only when staged)
    b->slot_busy[slot] = true;
    const std::shared_ptr<ba::StagedCall> sc = j->sc;
    const rspl_ba_problem* pr = j->pr;
    rspl_ba_result* res = j->res;
    lk.unlock();
    sc->slot = slot;
    sc->tr[1] = mono_s();
    sc->rc = stage_call(b, slot, pr, res, *sc);
    sc->tr[2] = mono_s();
    sc->tr[8] = slot;
    if (sc->rc) sc->msg = rspl_last_error();
    lk.lock();
    j->state = 2;
    b->qcv.notify_all();  // the tracking thread may be waiting for it
  }
}

void tracking_loop(rspl_ba* b) {
  (void)hipSetDevice(b->cfg.device);
  std::unique_lock<std::mutex> lk(b->qmu);
  for (;;) {
    b->qcv.wait(lk, [&] { return (!b->jobs.empty() && b->jobs.front().state == 2) || (b->quit && b->jobs.empty()); });
    if (b->jobs.empty()) return;  // quit with nothing left
    const rspl_ba::Job j = b->jobs.front();
    b->jobs.pop_front();
    b->busy = true;
    lk.unlock();
    b->qcv.notify_all();  // room for a submitter
    const auto t0 = std::chrono::steady_clock::now();
    j.sc->tr[3] = mono_s();
    int rc;
    if (j.sc->rc) {
      set_error("%s", j.sc->msg.c_str());
      rc = j.sc->rc;
    } else {
      begin_call(b);
      b->tracking_call = true;
      rc = end_call(b, run_call(b, *j.sc, j.pr, j.res, j.sc->tr));
      b->tracking_call = false;
    }
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    const std::string msg = rc ? std::string(rspl_last_error()) : std::string();
    lk.lock();
    b->slot_busy[j.sc->slot] = false;
    b->busy = false;
    b->q_done++;
    b->q_ms += ms;
    if (!rc) push_trace(b, j.sc->tr);
    if (!rc) b->q_iters += j.res->iterations_done_first + j.res->iterations_done_second;
    if (rc && !b->q_err) {
      b->q_err = rc;
      b->q_msg = msg;
    }
    b->qcv.notify_all();  // a joiner may be waiting for idle; the staging thread for a free slot
  }
}
}  // namespace

extern "C" int rspl_ba_submit(rspl_ba* b, const rspl_ba_problem* pr, rspl_ba_result* res) {
  RSPL_CHECK_ARG(b && pr && res, "rspl_ba_submit: NULL argument");
  std::unique_lock<std::mutex> lk(b->qmu);
  if (!b->worker.joinable()) {
    b->worker = std::thread(tracking_loop, b);
    b->stager = std::thread(staging_loop, b);
  }
  const double t_sub = mono_s();
  b->qcv.wait(lk, [&] { return b->jobs.size() < kTrackingBuffer; });
  b->jobs.push_back({pr, res, std::make_shared<ba::StagedCall>(), 0});
  b->jobs.back().sc->tr[0] = t_sub;
  lk.unlock();
  b->qcv.notify_all();
  return RSPL_OK;
}

extern "C" int rspl_ba_join(rspl_ba* b, long long* calls, long long* iterations, double* ms) {
  RSPL_CHECK_ARG(b, "rspl_ba_join: NULL handle");
  std::unique_lock<std::mutex> lk(b->qmu);
  b->qcv.wait(lk, [&] { return b->jobs.empty() && !b->busy; });
  if (calls) *calls = b->q_done;
  if (iterations) *iterations = b->q_iters;
  if (ms) *ms = b->q_ms;
  b->q_done = b->q_iters = 0;
  b->q_ms = 0.0;
  const int rc = b->q_err;
  if (rc) set_error("%s", b->q_msg.c_str());
  b->q_err = 0;
  b->q_msg.clear();
  return rc;
}

extern "C" int rspl_ba_debug_stage(const rspl_ba_problem* pr, int par_edges, int rank, int nranks, int* n_local,
                                   int* lm_off, int8_t* etype, int* epose, int* elm, int* ecam, int* gmap,
                                   int* lpose, double* eobs) {
  RSPL_CHECK_ARG(pr && n_local && lm_off && etype && epose && elm && ecam && gmap && lpose && eobs,
                 "rspl_ba_debug_stage: NULL argument");
  RSPL_CHECK_ARG(pr->n_poses >= 0 && pr->n_points >= 0 && pr->n_lines >= 0 && pr->n_mono >= 0 &&
                     pr->n_stereo >= 0 && pr->n_mono_line >= 0 && pr->n_stereo_line >= 0 &&
                     (pr->n_poses == 0 || pr->pose_fixed) && pr->n_cameras >= 1,
                 "rspl_ba_debug_stage: bad problem sizes");
  RSPL_CHECK_ARG(nranks >= 1 && rank >= 0 && rank < nranks, "rspl_ba_debug_stage: bad rank");
  ba::Stager stg;
  int rc;
  if ((rc = stg.count(pr, nranks > 1, rank, nranks, par_edges))) return rc;
  std::vector<int> pidx(pr->n_poses);
  int K = 0;
  for (int p = 0; p < pr->n_poses; p++) pidx[p] = (stg.pose_has_edge[p] && !pr->pose_fixed[p]) ? K++ : -1;
  ba::Stager::Out so{lm_off, etype, epose, elm, ecam, gmap, lpose, eobs, pidx.data()};
  stg.place(pr, so);
  n_local[0] = stg.E;
  n_local[1] = stg.Ep;
  return RSPL_OK;
}

namespace {
// Host staging of one call into stage slot `slot` (inputs only: nothing touches the device or the
// stream in steady state, so the tracking thread's next call is staged while the current one runs)
int stage_call(rspl_ba* b, int slot, const rspl_ba_problem* pr, rspl_ba_result* res, ba::StagedCall& c) {
  RSPL_CHECK_ARG(b && pr && res, "rspl_ba_local: NULL argument");
  const int np = pr->n_poses, nq = pr->n_points, nl = pr->n_lines;
  const int ne[4] = {pr->n_mono, pr->n_stereo, pr->n_mono_line, pr->n_stereo_line};
  RSPL_CHECK_ARG(np >= 0 && np <= b->cfg.max_poses && nq >= 0 && nq <= b->cfg.max_points && nl >= 0 &&
                     nl <= b->cfg.max_lines,
                 "problem exceeds the handle's vertex capacity");
  for (int t = 0; t < 4; t++) RSPL_CHECK_ARG(ne[t] >= 0 && ne[t] <= b->cfg.max_edges, "edge capacity exceeded");
  RSPL_CHECK_ARG(pr->n_cameras >= 1 && pr->n_cameras <= kMaxCams && pr->cameras, "1..16 cameras required");
  RSPL_CHECK_ARG(res->pose_q && res->pose_p && (res->points || !nq) && (res->lines || !nl), "NULL result arrays");
  RSPL_CHECK_ARG(np == 0 || pr->pose_fixed, "NULL pose_fixed");
  const int Eg = ne[0] + ne[1] + ne[2] + ne[3], nL = nq + nl;
  // landmark sharding: this rank keeps the edges of its landmarks (g % nranks == rank)
  const bool sh = b->allreduce != nullptr;
  HostMarks tm;
  tm.mark("start");
  // ---- one staging region for the whole call, mirrored by the device call buffer ----
  int rc;
  // pass 1: validate, count the local edges per landmark, mark the poses with edges (ba_stage.cpp;
  // large unsharded calls on the handle's host workers)
  if ((rc = b->stg.count(pr, sh, b->rank, b->nranks, kParEdges))) return rc;
  const int E = b->stg.E, Ep = b->stg.Ep, n_line_local = E - Ep;
  tm.mark("count");
  const CallLayout cl(pr->n_cameras, np, nq, nl, E, 4 * (size_t)Ep + 8 * (size_t)(E - Ep));
  const DownLayout dl(np, nq, nl, Eg);  // inlier flags by global edge id
  bool grew = false;
  if ((rc = ensure_stage(b, slot, std::max(cl.bytes, dl.bytes), &grew))) return rc;
  if (grew) c.tr[9] = (double)((unsigned)c.tr[9] | 1u);
  char* sg = b->stage[slot];
  // vertices: VertexSE3Expmap estimate = SE3Quat(q, p).inverse() (g2o_optimization.cc:42)
  double* T = reinterpret_cast<double*>(sg + cl.T);
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
  int* pidx = reinterpret_cast<int*>(sg + cl.pidx);
  int K = 0;
  for (int p = 0; p < np; p++) pidx[p] = (b->stg.pose_has_edge[p] && !pr->pose_fixed[p]) ? K++ : -1;
  // pass 2: lm_off, and every local edge at its CSR position with its reduced pose and its caller's
  // edge id (landmark-CSR order, input order within a landmark: the order every per-landmark
  // reduction follows)
  int* lm_off = reinterpret_cast<int*>(sg + cl.lm_off);
  tm.mark("vertices");
  {
    ba::Stager::Out so;
    so.lm_off = lm_off;
    so.etype = reinterpret_cast<int8_t*>(sg + cl.type);
    so.epose = reinterpret_cast<int*>(sg + cl.pose);
    so.elm = reinterpret_cast<int*>(sg + cl.lm);
    so.ecam = reinterpret_cast<int*>(sg + cl.cam);
    so.gmap = reinterpret_cast<int*>(sg + cl.gmap);
    so.lpose = reinterpret_cast<int*>(sg + cl.lm_pose);
    so.eobs = reinterpret_cast<double*>(sg + cl.obs);
    so.pidx = pidx;
    b->stg.place(pr, so);
  }
  tm.mark("scatter");
  uint8_t* lm_act = reinterpret_cast<uint8_t*>(sg + cl.lm_act);
  size_t pair_bound = 0;  // sum_g k_g^2 >= edge pairs of any pose pair
  for (int g = 0; g < nL; g++) {
    const size_t k = lm_off[g + 1] - lm_off[g];
    pair_bound += k * k;
    lm_act[g] = k > 0;
  }
  // line workgroups: consecutive line landmarks packed whole into <= kLineBlk edges (and <=
  // kLineBlk landmarks), so a workgroup sums their blocks itself; a landmark with more edges
  // gets workgroups of its own, flagged split (per-edge records + last-edge ticket)
  int4* ltab = reinterpret_cast<int4*>(sg + cl.ltab);
  int n_lblk = 0;
  {
    constexpr int kB = ba::kLineBlk;
    int p0 = 0, cnt = 0, gb = -1, ge = 0;
    auto flush = [&]() {
      if (gb >= 0 && cnt > 0) ltab[n_lblk++] = make_int4(p0, cnt, gb, ge);
      gb = -1;
      cnt = 0;
    };
    for (int g = nq; g < nL; g++) {
      const int k = lm_off[g + 1] - lm_off[g];
      if (k > kB) {
        flush();
        for (int o = 0; o < k; o += kB) ltab[n_lblk++] = make_int4(lm_off[g] + o, std::min(kB, k - o) | (1 << 8), g, g + 1);
        continue;
      }
      if (gb >= 0 && (cnt + k > kB || g - gb >= kB)) flush();
      if (gb < 0) {
        p0 = lm_off[g];
        gb = g;
      }
      cnt += k;
      ge = g + 1;
    }
    flush();
  }
  int* pairs = reinterpret_cast<int*>(sg + cl.pairs);
  for (int a = 0, q = 0; a < K; a++)
    for (int c = a; c < K; c++, q++) {
      pairs[2 * q] = a;
      pairs[2 * q + 1] = c;
    }
  tm.mark("tables");
  memcpy(sg + cl.cams, pr->cameras, sizeof(double) * 5 * pr->n_cameras);
  if (nq) memcpy(sg + cl.X, pr->points, sizeof(double) * 3 * nq);
  if (nl) memcpy(sg + cl.L, pr->lines, sizeof(double) * 6 * nl);
  memset(sg + cl.level, 0, cl.bytes - cl.level);  // level, flags, out start at zero
  c.slot = slot;
  c.E = E;
  c.Ep = Ep;
  c.K = K;
  c.n_lblk = n_lblk;
  c.pair_bound = pair_bound;
  c.cl = cl;
  c.dl = dl;
  c.tm = tm;
  return RSPL_OK;
}

// The device part of one staged call: upload, both optimize() calls, results
// The next queued call's inputs, uploaded into its slot's call buffer behind the current call's last
// queued kernels (optimize(5)'s trials and the gated final kernel): the upload (~40 us over PCIe at C3)
// then runs while the host notices the current call's end and queues the next one, instead of first in
// the next call's chain.  Tracking thread only; the next call must already be staged (its slot is then
// busy until it completes, and differs from the running call's).
void preupload_next(rspl_ba* b) {
  if (!b->tracking_call) return;
  std::shared_ptr<ba::StagedCall> nx;
  {
    std::lock_guard<std::mutex> lk(b->qmu);
    if (!b->jobs.empty() && b->jobs.front().state == 2 && b->jobs.front().sc->rc == RSPL_OK) nx = b->jobs.front().sc;
  }
  if (!nx || nx->uploaded) return;
  if (upload_mapped(b->cbuf[nx->slot], b->stage_dev[nx->slot], nx->cl.bytes, b->stream) == hipSuccess)
    nx->uploaded = true;
}

int run_call(rspl_ba* b, const ba::StagedCall& c, const rspl_ba_problem* pr, rspl_ba_result* res, double* tr) {
  const int np = pr->n_poses, nq = pr->n_points, nl = pr->n_lines;
  const int ne[4] = {pr->n_mono, pr->n_stereo, pr->n_mono_line, pr->n_stereo_line};
  hipStream_t st = b->stream;
  const int Eg = ne[0] + ne[1] + ne[2] + ne[3], nL = nq + nl;
  const bool sh = b->allreduce != nullptr;
  const int E = c.E, Ep = c.Ep, n_line_local = E - Ep, K = c.K, n_lblk = c.n_lblk;
  const size_t pair_bound = c.pair_bound;
  const CallLayout& cl = c.cl;
  const DownLayout& dl = c.dl;
  char* sg = b->stage[c.slot];
  HostMarks tm = c.tm;
  int rc;
  tm.mark("run");
  b->grew = 0;
  if (pair_bound > b->pp_cap) {  // grow the edge-pair lists (the stream is idle between calls)
    RSPL_HIP(hipStreamSynchronize(st));
    if (b->pp_buf) (void)hipFree(b->pp_buf);
    b->pp_buf = nullptr;
    b->pp_cap = 0;
    const size_t cap = std::max(pair_bound, (size_t)1 << 16);
    RSPL_HIP(hipMalloc((void**)&b->pp_buf, sizeof(int4) * cap));
    b->pp_cap = cap;
    b->grew |= 2;
  }
  // the call's inputs in one upload: a copy kernel reading the host-mapped staging slot over PCIe.  Not
  // hipMemcpyAsync: its H2D path stalled the first calls after the warmup by 7-10 ms each (the SDMA engine /
  // blit-kernel choice settling; profiles/r05_bench_20step_before.json), which cost the driver's 20-step bench
  // a quarter of its rate.
  char* cb = b->cbuf[c.slot];
  if (!c.uploaded)  // (else queued behind the previous call's final kernel: preupload_next)
    RSPL_HIP(upload_mapped(cb, b->stage_dev[c.slot], cl.bytes, st));
  tm.mark("upload");
  tr[4] = mono_s();
  uint8_t* level = reinterpret_cast<uint8_t*>(cb + cl.level);
  ba::Problem P{};
  P.cams = reinterpret_cast<double*>(cb + cl.cams);
  P.T = reinterpret_cast<double*>(cb + cl.T);
  P.X = reinterpret_cast<double*>(cb + cl.X);
  P.L = reinterpret_cast<double*>(cb + cl.L);
  P.np = np; P.nq = nq; P.nl = nl; P.ncam = pr->n_cameras;
  P.Tn = b->Tb; P.Xn = b->Xb; P.Ln = b->Lb;
  P.etype = reinterpret_cast<const int8_t*>(cb + cl.type);
  P.epose = reinterpret_cast<const int*>(cb + cl.pose);
  P.elm = reinterpret_cast<const int*>(cb + cl.lm);
  P.ecam = reinterpret_cast<const int*>(cb + cl.cam);
  P.eobs = reinterpret_cast<const double*>(cb + cl.obs);
  P.Ep = Ep;
  const double th[4] = {pr->th_mono_point, pr->th_stereo_point, pr->th_mono_line, pr->th_stereo_line};
  for (int t = 0; t < 4; t++) {
    P.th[t] = th[t];
    P.delta[t] = (double)(float)std::sqrt(th[t]);  // const float thHuber = sqrt(cfg.x) (:77-78, 125-126)
  }
  P.line_jac = b->line_jac;
  ba::Lin Lr{};
  Lr.err = b->err; Lr.Hpp = b->Hpp_e; Lr.bp = b->bp_e; Lr.Hll = b->Hll_e; Lr.bl = b->bl_e;
  Lr.Hpl = b->Hpl_e;
  ba::Sys S{};
  S.Hll = b->Hll; S.bl = b->bl; S.bp = b->bp; S.S = b->S; S.x = b->x; S.partial = b->partial;
  S.partial2 = b->partial2;
  S.out = reinterpret_cast<double*>(cb + cl.out);
  S.fail = reinterpret_cast<int*>(cb + cl.flags);
  S.counter = reinterpret_cast<unsigned*>(cb + cl.flags + sizeof(int));
  S.lm_ctr = b->lm_ctr;
  S.mail = b->mail_dev;
  S.chunk = b->chunk;
  S.pairfin = b->pairfin;
  S.pair_ctr = b->pair_ctr;
  S.solve_ctr = b->pair_ctr + b->maxK * (b->maxK + 1) / 2;
  S.shard_out = sh ? b->red + 6 * K + b->nranks : nullptr;
  S.pose_scale = !sh || b->rank == 0;
  // ---- phase 1: all edges, Huber ----
  ba::Active A{};
  A.Ea = E;
  A.pidx = reinterpret_cast<const int*>(cb + cl.pidx);
  A.lm_off = reinterpret_cast<const int*>(cb + cl.lm_off);
  A.lm_pose = reinterpret_cast<const int*>(cb + cl.lm_pose);
  A.lm_act = reinterpret_cast<const uint8_t*>(cb + cl.lm_act);
  A.pairs = reinterpret_cast<const int*>(cb + cl.pairs);
  A.npairs = K * (K + 1) / 2;
  // Schur chunks: ranges of kLmChunk landmarks per pose pair while the chunk waves fit one dispatch
  // round (C3: 45 pairs x 16 ranges); with many pose pairs (C5: K = 29, 435 pairs) fewer, wider
  // ranges -- each wave then walks more passes, but the chip runs them in one round instead of ~17
  {
    const int npairs = std::max(A.npairs, 1);
    A.nchk = std::max(1, std::min((nL + ba::kLmChunk - 1) / ba::kLmChunk, kChunkWaves / npairs));
    A.lmchunk = std::max(ba::kLmChunk, ((nL + A.nchk - 1) / A.nchk + 63) / 64 * 64);
    A.nchk = std::max((nL + A.lmchunk - 1) / A.lmchunk, 1);
    // wide windows (K > the single-wave solve's, fewer than 8 ranges per pair): a diagonal pose pair walks about
    // (K - 1) / (obs - 1) times an off-diagonal pair's edge pairs (C5: ~970 vs ~170 per range) and set the chunk
    // phase alone -- its ranges are cut into kDiagSub sub-chunks (the off-diagonal pairs keep theirs)
    constexpr int kDiagSub = 8;
    A.dsub = 1;
    A.lmsub = A.lmchunk;
    A.K = K;
    if (!ba::wave_path(K) && A.nchk < 8 && (size_t)A.nchk * (A.npairs + (kDiagSub - 1) * K) <= b->chunk_slots) {
      A.dsub = kDiagSub;
      A.lmsub = ((A.lmchunk + kDiagSub - 1) / kDiagSub + 63) / 64 * 64;
    }
    ba::set_update_geometry(A);
  }
  A.n_line_edges = n_line_local;
  A.ltab = reinterpret_cast<const int4*>(cb + cl.ltab);
  A.n_lblk = n_lblk;
  A.K = K;
  A.nL = nL;
  A.robust = 1;
  A.pp_off = b->pp_off;
  A.pp = b->pp_buf;
  // on the BA stream itself: a second stream would take a hardware queue of its own (streams map
  // round-robin onto GPU_MAX_HW_QUEUES) and push a pipeline stream onto the BA's queue -- measured:
  // bench 2.17 ms per step instead of 1.5 with a side stream for the pair lists
  const bool pp_fused = dev_lm(b, A, pr->iterations_first);  // else: built here, before the first optimize
  if (!pp_fused) RSPL_HIP(ba::build_pairs(A, b->pp_cnt, b->pp_off, b->pp_buf, st));
  tm.mark("pairs");
  // phase 2's setup queued behind phase 1's trials (device LM on both, unsharded)
  SpecSetup nxt;
  nxt.A2 = A;
  nxt.A2.robust = 0;
  nxt.A2.elevel = level;
  nxt.A2.lm_act = b->lm_act2;
  nxt.level = level;
  nxt.iters2 = pr->iterations_second;
  const bool spec_setup = pp_fused && !sh && !b->ktime_on && dev_lm(b, nxt.A2, pr->iterations_second);
  if ((rc = optimize(b, P, Lr, S, A, pr->iterations_first, &res->chi2_first, &res->iterations_done_first, nullptr,
                     pp_fused, nullptr, spec_setup ? &nxt : nullptr)))
    return rc;
  tm.mark("opt1");
  tr[5] = mono_s();
  uint8_t* inl_h = reinterpret_cast<uint8_t*>(b->stage_dev[c.slot] + dl.inl);
  double* T_h = reinterpret_cast<double*>(b->stage_dev[c.slot] + dl.T);
  double* X_h = reinterpret_cast<double*>(b->stage_dev[c.slot] + dl.X);
  double* L_h = reinterpret_cast<double*>(b->stage_dev[c.slot] + dl.L);
  SpecFinish fin;
  // ---- phase 2: level-0 edges, no kernel (initializeOptimization(0), :176-213) ----
  // Same active structure with the level-1 edges masked (exact-zero records, no cost, errors
  // kept as g2o keeps them), landmark activity recomputed from the levels on the device (device LM:
  // inside the optimize's first launch).
  {
    A.robust = 0;
    A.elevel = level;
    A.lm_act = b->lm_act2;
    const bool fused = dev_lm(b, A, pr->iterations_second);
    if (!fused) {
      RSPL_HIP(ba::classify(P, Lr, E, level, nullptr, 0, st));
      RSPL_HIP(ba::landmark_active(A, level, b->lm_act2, st));
    }
    // the final kernel queued behind optimize(5)'s trials (device LM, unsharded): no host round trip
    // between that optimize()'s stop and the final kernel
    const bool spec_fin = fused && !sh && !b->ktime_on;  // (kernel timing maps events to contiguous trial seqs)
    if (spec_fin) {
      fin.L = Lr;
      fin.E = E;
      fin.gmap = reinterpret_cast<const int*>(cb + cl.gmap);
      fin.inl = inl_h;
      fin.Th = T_h;
      fin.Xh = X_h;
      fin.Lh = L_h;
    }
    if ((rc = optimize(b, P, Lr, S, A, pr->iterations_second, &res->chi2_second, &res->iterations_done_second,
                       fused ? level : nullptr, false, spec_fin ? &fin : nullptr, nullptr,
                       nxt.queued && !nxt.extra)))
      return rc;
    tm.mark("opt2");
    tr[6] = mono_s();
    // trace flags: 16 optimize(5)'s setup ran from the speculative queue, 32 optimize(10) was topped up
    tr[9] = (double)((unsigned)tr[9] | (nxt.queued && !nxt.extra ? 16u : 0u) | (nxt.topped_up ? 32u : 0u));
  }
  // ---- inlier flags + final state written by the GPU into the mapped staging buffer ----
  // (the staging call region was consumed by the upload long before: the stream is in order)
  const unsigned long long q = fin.on ? fin.q : ++b->seq;
  if (fin.on) {
    // already queued (SpecFinish)
  } else if (sh) {  // owned landmarks + local edge flags gathered by one more all-reduce: complete on every rank
    const size_t glen = 3 * (size_t)nq + 6 * (size_t)nl + Eg;
    if (glen > b->gcap) {
      RSPL_HIP(hipStreamSynchronize(st));
      if (b->gbuf) (void)hipFree(b->gbuf);
      b->gbuf = nullptr;
      b->gcap = 0;
      RSPL_HIP(hipMalloc((void**)&b->gbuf, sizeof(double) * std::max<size_t>(glen, 1024)));
      b->gcap = std::max<size_t>(glen, 1024);
    }
    RSPL_HIP(hipMemsetAsync(b->gbuf, 0, sizeof(double) * glen, st));
    RSPL_HIP(ba::shard_gather(P, Lr, E, reinterpret_cast<const int*>(cb + cl.gmap), b->rank, b->nranks, b->gbuf, st));
    if (glen && (rc = allreduce(b, b->gbuf, glen))) return rc;
    RSPL_HIP(ba::shard_finish(P, Eg, b->gbuf, inl_h, T_h, X_h, L_h, S, q, st));
  } else {
    RSPL_HIP(ba::finish(P, Lr, E, reinterpret_cast<const int*>(cb + cl.gmap), inl_h, T_h, X_h, L_h, S, q, st));
  }
  if ((rc = wait_mail(b, q, nullptr))) return rc;
  if (b->ktime_on) {  // every timed trial precedes the finish kernel in the stream: its events are complete
    for (int i : b->kev_eval) {
      float a = 0.f, c = 0.f;
      if (hipEventElapsedTime(&a, b->kev[3 * (size_t)i], b->kev[3 * (size_t)i + 1]) == hipSuccess &&
          hipEventElapsedTime(&c, b->kev[3 * (size_t)i + 1], b->kev[3 * (size_t)i + 2]) == hipSuccess) {
        b->kt_ms[0] += a;
        b->kt_ms[1] += c;
        b->kt_n[0]++;
        b->kt_n[1]++;
      }
    }
  }
  if (b->prof && b->prof_nb[0]) report_prof(b);
  tr[9] = (double)((unsigned)tr[9] | b->grew);
  if (b->lm_trace) {  // RSPL_BA_LMTRACE: the device LM decisions of both optimize() calls
    std::vector<double> h(8 * 64);
    if (hipMemcpy(h.data(), b->lm_trace, sizeof(double) * h.size(), hipMemcpyDeviceToHost) == hipSuccess)
      for (int k = 0; k < 64; k++)
        if (h[8 * k] != 0.0)
          fprintf(stderr, "lmtrace phase %d trial %d chi2 %.17g scale %.6g fail %g lambda %.6g chi0 %.17g cur %g it %g q %g\n",
                  k / 32, k % 32, h[8 * k], h[8 * k + 1], h[8 * k + 2], h[8 * k + 3], h[8 * k + 4], h[8 * k + 5],
                  h[8 * k + 6], h[8 * k + 7]);
    (void)hipMemset(b->lm_trace, 0, sizeof(double) * h.size());
  }
  if (nq) memcpy(res->points, b->stage[c.slot] + dl.X, sizeof(double) * 3 * nq);
  if (nl) memcpy(res->lines, b->stage[c.slot] + dl.L, sizeof(double) * 6 * nl);
  const double* Tout = reinterpret_cast<const double*>(b->stage[c.slot] + dl.T);
  uint8_t* outs[4] = {res->mono_inlier, res->stereo_inlier, res->mono_line_inlier, res->stereo_line_inlier};
  int e = 0;
  for (int t = 0; t < 4; t++) {
    if (outs[t]) memcpy(outs[t], b->stage[c.slot] + dl.inl + e, ne[t]);
    e += ne[t];
  }
  // write back T_wc = estimate().inverse() (:235-240)
  for (int p = 0; p < np; p++) {
    Se3h Tcw;
    for (int k = 0; k < 4; k++) Tcw.q[k] = Tout[8 * p + k];
    for (int k = 0; k < 3; k++) Tcw.t[k] = Tout[8 * p + 4 + k];
    const Se3h Twc = inverse(Tcw);
    res->pose_q[4 * p + 0] = Twc.q[1];
    res->pose_q[4 * p + 1] = Twc.q[2];
    res->pose_q[4 * p + 2] = Twc.q[3];
    res->pose_q[4 * p + 3] = Twc.q[0];
    for (int k = 0; k < 3; k++) res->pose_p[3 * p + k] = Twc.t[k];
  }
  tm.mark("final");
  tm.print("rspl_ba_local us:");
  tr[7] = mono_s();
  tr[10] = res->iterations_done_first + res->iterations_done_second;
  return RSPL_OK;
}

int ba_local_impl(rspl_ba* b, const rspl_ba_problem* pr, rspl_ba_result* res) {
  RSPL_CHECK_ARG(b && pr && res, "rspl_ba_local: NULL argument");
  ba::StagedCall c;
  c.tr[0] = c.tr[1] = mono_s();
  c.tr[11] = 1;
  int rc = stage_call(b, 0, pr, res, c);
  c.tr[2] = c.tr[3] = mono_s();
  if (!rc) rc = run_call(b, c, pr, res, c.tr);
  if (!rc) {
    std::lock_guard<std::mutex> lk(b->qmu);
    push_trace(b, c.tr);
  }
  return rc;
}

// append one record to the handle's timeline ring (qmu held)
void push_trace(rspl_ba* b, const double* tr) {
  if (b->trace.empty()) return;
  const size_t i = (size_t)(b->trace_n++ % rspl_ba::kTraceCap);
  std::copy(tr, tr + RSPL_BA_TRACE_W, b->trace.begin() + i * RSPL_BA_TRACE_W);
}
}  // namespace
