#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace rspl {
namespace ba {

// Edge types (same order as rspl_ba_problem): 0 mono point, 1 stereo point,
// 2 mono line, 3 stereo line.  Unified edge arrays in LANDMARK-CSR order, laid out by the host:
// the edges of landmark g are [lm_off[g], lm_off[g+1]) (input order within a landmark), point
// landmarks first, so an edge's position is its index everywhere (records, levels, errors) and
// gmap maps it back to the caller's edge id.  Observations: point edges at eobs + 4 e (u, v, u_r),
// line edges at eobs + 4 Ep + 8 (e - Ep).
struct Problem {
  const double* cams;    // [nc][5] fx fy cx cy bf
  double* T;             // [np][8] T_cw: q (w x y z), t (x y z), pad   (current state)
  double* X;             // [nq][3]
  double* L;             // [nl][6]
  double* Tn;            // candidate state written by the update (ping-pong)
  double* Xn;
  double* Ln;
  int np, nq, nl;
  int ncam;              // cameras (<= 16)
  const int8_t* etype;   // [E]
  const int* epose;      // [E]
  const int* elm;        // [E] landmark index: point id, or nq + line id
  const int* ecam;       // [E]
  const double* eobs;    // packed observations (see above)
  int Ep;                // point edges (the first line edge's position)
  double delta[4];       // Huber deltas per type
  double th[4];          // chi2 thresholds per type
  int line_jac;          // line edges' Jacobians: 0 g2o's central difference (delta 1e-9), 1 its analytic limit
};

struct Lin {             // per-edge linearisation records (indexed by edge id)
  double* err;           // [E][4] last computed error
  double* Hpp;           // [E][21] upper triangle, row-major (pk6): line edges; a point edge's pose block is
                         //   formed again by the diagonal Schur chunk (point_pose_block), only its diagonal
                         //   is written by the first linearisation of an optimize() (computeLambdaInit)
  double* bp;            // [E][6] line edges
  double* Hll;           // [E][16]
  double* bl;            // [E][4]
  double* Hpl;           // point edge e < Ep: 6 x 3 at 18 e; line edge: 6 x 4 at 18 Ep + 24 (e - Ep) (hpl_off)
};

struct Active {          // active structure of one optimize() phase
  int Ea;                // active edges: every edge id in [0, Ea) (input order: points, then lines)
  const int* pidx;       // [np] reduced pose index or -1
  const int* lm_off;     // [nL+1] CSR of the edges by landmark (= edge positions, see Problem)
  const int* lm_pose;    // [Ea] reduced pose of edge k (or -1)
  const uint8_t* lm_act; // [nL]
  const int* pairs;      // [npairs][2] reduced pose pairs (a <= b)
  int npairs;
  int nchk;              // Schur chunks per pose pair: landmark ranges of lmchunk
  int lmchunk;           // landmarks per Schur chunk (a multiple of 64; kLmChunk unless the pose pairs
                         //   are so many that the chunk waves would need several dispatch rounds)
  int dsub;              // Schur chunks per landmark range of a DIAGONAL pose pair: 1, or more on wide windows
                         //   (C5: a diagonal pair walks ~(K - 1) / (obs - 1) times an off-diagonal pair's edge
                         //   pairs and set the chunk phase alone); see chunk_geo
  int lmsub;             // landmarks per diagonal sub-chunk (a multiple of 64; lmchunk when dsub == 1)
  int ue_bpr;            // update_errors<true> workgroups per Schur chunk range when their landmark blocks
                         //   are dealt to the XCD that ran the range's chunks (0: plain order)
  const int* pp_off;     // [npairs * nchk + 1] segment of each chunk in the edge-pair lists
  const int4* pp;        // edge pairs {e1 of pose a, e2 of pose b, their landmark, 0}, chunk-major,
                         //   landmark order within a chunk
  int n_line_edges;      // line edges are [Ea - n_line_edges, Ea)
  const int4* ltab;      // [n_lblk] line workgroups {first CSR position, edges | split << 8, first
  int n_lblk;            //   landmark, end landmark}: whole line landmarks of <= kLineBlk edges
                         //   (summed in the workgroup), or one slice of a larger landmark (split)
  const uint8_t* elevel; // [E] or null: edge level (!= 0: outside this phase -- level 1 in the
                         // second optimize): zero linearisation records, no cost, error kept
  int K, nL;
  int robust;
};

// Schur chunk geometry.  Chunks are numbered pose pair by pose pair (row-major upper triangle); a pair owns nchk
// landmark ranges of lmchunk, a diagonal pair nchk * dsub sub-ranges of lmsub (dsub == 1: every pair nchk, chunk
// c = pr * nchk + lb, as before).  g0 .. g1: the chunk's landmarks (clamped to nL), gend its nominal end (the
// points-only test), c0 .. c1 the chunks of its pose pair.
struct ChunkGeo {
  int pr, lb, g0, g1, gend, c0, c1;
};
__host__ __device__ inline int chunk_count(const Active& A) { return A.nchk * (A.npairs + (A.dsub - 1) * A.K); }
__host__ __device__ inline ChunkGeo chunk_geo(const Active& A, int c) {
  ChunkGeo q;
  if (A.dsub <= 1) {
    q.pr = c / A.nchk;
    q.lb = c - q.pr * A.nchk;
    q.g0 = q.lb * A.lmchunk;
    q.gend = q.g0 + A.lmchunk;
    q.c0 = q.pr * A.nchk;
    q.c1 = q.c0 + A.nchk;
  } else {
    // row a (pose a's pairs a..K-1): pair base a K - a (a - 1) / 2, chunk base nchk (pair base + (dsub - 1) a)
    int a = 0;
    while (a + 1 < A.K && c >= A.nchk * ((a + 1) * A.K - (a + 1) * a / 2 + (A.dsub - 1) * (a + 1))) a++;
    const int pa = a * A.K - a * (a - 1) / 2, base = A.nchk * (pa + (A.dsub - 1) * a), nd = A.nchk * A.dsub;
    const int l = c - base;
    if (l < nd) {
      q.pr = pa;
      q.lb = l / A.dsub;
      q.g0 = q.lb * A.lmchunk + (l - q.lb * A.dsub) * A.lmsub;
      q.gend = q.g0 + A.lmsub < (q.lb + 1) * A.lmchunk ? q.g0 + A.lmsub : (q.lb + 1) * A.lmchunk;
      q.c0 = base;
      q.c1 = base + nd;
    } else {
      const int m = l - nd, j = m / A.nchk;
      q.pr = pa + 1 + j;
      q.lb = m - j * A.nchk;
      q.g0 = q.lb * A.lmchunk;
      q.gend = q.g0 + A.lmchunk;
      q.c0 = base + nd + j * A.nchk;
      q.c1 = q.c0 + A.nchk;
    }
  }
  q.g1 = q.gend < A.nL ? q.gend : A.nL;
  if (q.g1 < q.g0) q.g1 = q.g0;
  return q;
}

struct Mail {            // pinned, host-mapped: the per-trial result the host spins on
  double v[4];           // chi2, scale, maxdiag, fail
  unsigned long long seq;
  unsigned long long vseq;  // written before v (seq after it): v belongs to seq iff vseq == seq
  unsigned long long pad[2];
};

// Device-resident Levenberg-Marquardt control (g2o OptimizationAlgorithmLevenberg::solve,
// restated in ba.cpp's host loop): initialised after the first linearisation, advanced by the last
// block of every trial's update_errors kernel, read by the next trial's kernels at their start.
// Two banks of state + linearisation records alternate: `cur` names the current one (the host's
// pointer view is bank 0 at the start of each optimize()).  A trial queued after `stop` is a no-op
// that only carries the control over to the next slot.
struct LmCtrl {
  double lambda, ni, chi;  // damping, its growth factor, current chi2
  int cur;                 // current bank (0: the host's current pointers, 1: its spare/candidate ones)
  int it;                  // iterations done
  int qmax;                // trials of the running iteration
  int stop;                // 1: optimize() finished
  int iters;               // iterations requested
  int trials;              // trials evaluated (diagnostics)
};

struct Sys {
  double* Hll;           // [nL][16]  (points: 3x3 at stride 3)
  double* bl;            // [nL][4]
  double* bp;            // [K][6]   pose gradient (undamped), for the LM scale
  double* S;             // [6K][6K] reduced camera system
  double* x;             // [6K]     bs on entry of the solve, xp on exit
  double* chunk;         // [npairs * nchk][48] Schur chunk partials
  double* pairfin;       // [npairs][48] per-pose-pair sums of the chunk partials
  unsigned* pair_ctr;    // [npairs] chunk tickets (re-armed to 0 by the last chunk)
  unsigned* solve_ctr;   // [1] pose-pair ticket of the fused single-wave solve (re-armed by the solver)
  double* partial;       // [>= error blocks] chi2 partials
  double* partial2;      // [>= update blocks] scale partials
  double* out;           // [8]: 0 chi2, 1 scale, 2 maxdiag, 3 fail
  int* fail;             // [1]
  unsigned* counter;     // [1] last-block ticket of the error kernel
  unsigned* lm_ctr;      // [nl] line-landmark tickets of the linearisation (re-armed to 0 by the last edge)
  Mail* mail;            // device view of the mailbox
  // landmark sharding (null / 1 when the handle is not sharded)
  double* shard_out;     // [3] this rank's {chi2, LM scale (landmark part), fail} for the all-reduce,
                         //     written instead of posting the mailbox
  int pose_scale;        // 1: this rank adds the pose part of the LM scale (rank 0 or unsharded)
  // timing trace of one trial (RSPL_BA_PROF; null otherwise): wall_clock64 stamps
  //   [0, 8) schur_solve phases, [kProfPc + 4b + i] pair_chunk block b stamps (start, loop
  //   done, ticket, end), [kProfUe + 4b + i] update_errors block b stamps (start, update /
  //   flag wait done, before ticket, end)
  unsigned long long* prof;
  LmCtrl* lm;            // device-side LM control [2] (fast path, unsharded), null: the host decides
  double* lm_trace;      // debug (RSPL_BA_LMTRACE): per trial {chi2, scale, fail, lambda, rho, cur, it, qmax}
  int lm_slot;           // trial k reads lm[k & 1] and its last block writes lm[(k + 1) & 1]: the
                         // control a trial's blocks read never changes under them
  int lm_post;           // device LM: post the verdict even when it does not stop (the last trial the
                         // host queued); otherwise only the stopping trial posts the mailbox
};
constexpr int kProfPc = 16, kProfUe = kProfPc + 4 * 4096, kProfX = kProfUe + 4 * 4096, kProfLen = kProfX + 8;
// [kProfX + i]: setup_kernel's latest landmark / landmark + pose-diagonal / line / line + pose-diagonal / pair
// block (atomic max over the blocks)

constexpr int kLmChunk = 256;  // landmarks per Schur chunk (4 per lane; 128 measured: 1440 chunk waves exceed one dispatch round)
constexpr int kLineBlk = 8;    // line edges per linearisation workgroup

// errors (+ fused final reduction and mailbox post with sequence number seq)
hipError_t compute_errors(const Problem& P, const Lin& L, const Active& A, Sys& S, unsigned long long seq,
                          hipStream_t s);
// edge Jacobians + landmark blocks S.Hll / S.bl (+ with_maxdiag: the max diagonal of pose and
// landmark blocks into S.out[2], computeLambdaInit)
hipError_t linearize(const Problem& P, const Lin& L, const Active& A, const Sys& S, bool with_maxdiag,
                     hipStream_t s);
// mailbox post; with A, after linearize(with_maxdiag) it first folds the pose-block maxima in
hipError_t post(Sys& S, unsigned long long seq, hipStream_t s, const Active* A = nullptr, int lm_iters = 0);
// the first pass of a device-LM optimize() (S.lm set, lm_iters > 0) in one launch: errors, robust
// cost and linearisation at the current state, the pose / landmark diagonal maximum and the LM control
// (computeLambdaInit) into S.lm[0].  level != null (the second optimize): the edges' outlier levels
// from their last computed errors into level[] and the landmark activity into lm_act2 first (replaces
// classify + landmark_active); A.elevel / A.lm_act are then the caller's level / lm_act2.  pp_cnt
// != null (the call's first optimize): the Schur chunks' edge-pair lists too (replaces build_pairs:
// counted in the first launch, scanned by the second's last block, filled by a third).
// pdg: setup_pdg_len(A) doubles of per-block pose-diagonal partials.
// gate >= 0 (the second optimize's setup queued behind the first one's trials before the host has seen them):
// a no-op unless the control slot `gate` shows that optimize stopped; then the current bank from that control
// (Ls / Ss: the spare records, as the trials bank them)
hipError_t setup_dev(const Problem& P, const Lin& L, const Active& A, Sys& S, uint8_t* level, uint8_t* lm_act2,
                     int lm_iters, int* pp_cnt, int* pp_off, int4* pp, double* pdg, hipStream_t s, int gate = -1,
                     const Lin* Ls = nullptr, const Sys* Ss = nullptr);
int setup_pdg_len(const Active& A);
// speculative linearisation of a trial's candidate into a spare record set, fused into the
// trial's last kernel (fast path only)
struct Spec {
  Lin Ls;            // spare edge records (err shared with the current set)
  Sys Ss;            // spare landmark blocks Hll / bl
};
// one LM trial: Schur complement, Cholesky, back-substitution + candidate state, its cost;
// with spec on the fast path also the candidate's linearisation (*fused = true)
hipError_t trial(const Problem& P, const Lin& L, const Active& A, Sys& S, double lambda, unsigned long long seq,
                 hipStream_t s, const Spec* spec, bool* fused);
// one LM trial under device control (S.lm set, fast path): lambda, the current bank and the
// accept / reject decision live in *S.lm; the trial's last kernel advances it and posts the mailbox
// {chi2, iterations done, current bank, stop} + seq.  Always fused with the speculative linearisation
// (skipped on the device when the iteration is the last one).
hipError_t trial_dev(const Problem& P, const Lin& L, const Active& A, Sys& S, unsigned long long seq, hipStream_t s,
                     const Spec& spec, hipEvent_t* ev = nullptr);  // ev: [3] recorded before / between / after
                                                                   // the trial's two launches (kernel timing)
// edge-pair lists of the pose pairs (count, offsets, fill; A.pp_* are not read)
hipError_t build_pairs(const Active& A, int* pp_cnt, int* pp_off, int4* pp, hipStream_t s);
// lm_act[g] = landmark g has an edge of level 0 (the second optimize's active landmarks)
hipError_t landmark_active(const Active& A, const uint8_t* level, uint8_t* lm_act, hipStream_t s);
hipError_t classify(const Problem& P, const Lin& L, int E, uint8_t* level, uint8_t* inlier, int final_pass,
                    hipStream_t s);
// final inlier flags + T / X / L into host-mapped memory, then the mailbox post of seq
hipError_t finish(const Problem& P, const Lin& L, int E, const int* gmap, uint8_t* inl, double* Th, double* Xh,
                  double* Lh, Sys& S, unsigned long long seq, hipStream_t s);
// ---- landmark-sharded pieces (rspl_ba_set_shard): the host interleaves the all-reduces ----
// trial, part 1: Schur chunks of this rank's edge pairs -> pairfin; the landmark-inversion flag
// is staged into pairfin[npairs * 48] so it is summed with the system
hipError_t trial_chunks(const Problem& P, const Lin& L, const Active& A, Sys& S, double lambda, hipStream_t s);
// trial, part 2 (after the pairfin all-reduce): adopt the summed flag, assemble + factor + solve
// the (now global) reduced system, candidate state and this rank's cost / scale into shard_out
hipError_t trial_solve(const Problem& P, const Lin& L, const Active& A, Sys& S, double lambda, hipStream_t s);
// lambda init: this rank's pose-diagonal sums into red[0, 6K), its landmark max into red[6K + rank]
// (other rank slots zeroed); red[6K + nranks ...] holds shard_out
hipError_t shard_fold(const Active& A, Sys& S, double* red, int rank, int nranks, hipStream_t s);
// after the all-reduce of red: mailbox post.  mode 0: lambda init (max |pose diagonal|, max rank
// slot); mode 1: cost only; add_pose_scale: S.out[4] (fast path) joins the summed scale
hipError_t shard_post(Sys& S, const double* red, int n6, int nranks, int mode, int add_pose_scale,
                      unsigned long long seq, hipStream_t s);
// final gather: G = [X of owned points | L of owned lines | inlier flag by global edge id] (G zeroed
// by the caller), summed across ranks, then written out by shard_finish
hipError_t shard_gather(const Problem& P, const Lin& L, int E, const int* gmap, int rank, int nranks, double* G,
                        hipStream_t s);
hipError_t shard_finish(const Problem& P, int E_global, const double* G, uint8_t* inl, double* Th, double* Xh,
                        double* Lh, Sys& S, unsigned long long seq, hipStream_t s);
int shard_red_len(int K, int nranks);  // 6K + nranks + 3
bool fast_path(int K);                 // the packed-LDS Schur/LDL^T path holds 6K
bool wave_path(int K);                 // the single-wave LDL^T (fused into the Schur chunks) holds 6K
int update_blocks(const Problem& P);
int errors_blocks(int Ea);
int update_errors_blocks(const Active& A);
// sets A.ue_bpr (after nchk / lmchunk): the trial's update workgroups on the XCD whose L2 the Schur chunks of
// their landmarks just filled (RSPL_BA_UEXCD=0: plain order, A/B)
void set_update_geometry(Active& A);

}  // namespace ba
}  // namespace rspl
