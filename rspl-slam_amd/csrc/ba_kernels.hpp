#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace rspl {
namespace ba {

// Edge types (same order as rspl_ba_problem): 0 mono point, 1 stereo point,
// 2 mono line, 3 stereo line.  Unified edge arrays, obs padded to 8 doubles.
struct Problem {
  const double* cams;    // [nc][5] fx fy cx cy bf
  double* T;             // [np][8] T_cw: q (w x y z), t (x y z), pad
  double* X;             // [nq][3]
  double* L;             // [nl][6]
  int np, nq, nl;
  const int8_t* etype;   // [E]
  const int* epose;      // [E]
  const int* elm;        // [E] landmark index: point id, or nq + line id
  const int* ecam;       // [E]
  const double* eobs;    // [E][8]
  double delta[4];       // Huber deltas per type
  double th[4];          // chi2 thresholds per type
};

struct Lin {             // per-edge linearisation records (indexed by edge id)
  double* err;           // [E][4] last computed error
  double* rho0;          // [E] robust chi2 (or chi2)
  double* Hpp;           // [E][36]
  double* bp;            // [E][6]
  double* Hll;           // [E][16]
  double* bl;            // [E][4]
  double* Hpl;           // [E][24]  6 x 4 (row stride 4)
  double* Y;             // [E][24]  Hpl * Dinv
};

struct Active {          // active structure of one optimize() phase
  const int* edges;      // [Ea] active edge ids
  int Ea;
  const int* pidx;       // [np] reduced pose index or -1
  const int* lm_off;     // [nL+1] CSR over active edges by landmark
  const int* lm_edges;
  const uint8_t* lm_act; // [nL]
  const int* pose_of;    // [K] pose id of reduced index
  const int* ps_off;     // [K+1] CSR by reduced pose, sorted by landmark
  const int* ps_edges;
  const int* ps_lm;      // landmark of ps_edges[i] (sorted key)
  const int* pairs;      // [npairs][2] reduced (a <= b)
  int npairs;
  int K, nL;
  int robust;
};

struct Sys {
  double* Hll;           // [nL][16]
  double* bl;            // [nL][4]
  double* Dinv;          // [nL][16]
  double* Hpp;           // [K][36]
  double* bp;            // [K][6]
  double* S;             // [6K][6K]
  double* x;             // [6K + 4 nL]  (landmark l at 6K + 4l)
  double* partial;       // [nblocks] scratch for reductions
  double* out;           // [8]: 0 chi2, 1 scale, 2 maxdiag, 3 fail flag
  int* fail;             // [1]
};

hipError_t compute_errors(const Problem& P, const Lin& L, const Active& A, Sys& S, int nblocks, hipStream_t s);
hipError_t linearize(const Problem& P, const Lin& L, const Active& A, hipStream_t s);
hipError_t reduce_blocks(const Problem& P, const Lin& L, const Active& A, Sys& S, hipStream_t s);
hipError_t schur(const Problem& P, const Lin& L, const Active& A, Sys& S, double lambda, hipStream_t s);
hipError_t solve_update(const Problem& P, const Lin& L, const Active& A, Sys& S, double lambda, hipStream_t s);
hipError_t classify(const Problem& P, const Lin& L, int E, uint8_t* level, uint8_t* inlier, int final_pass,
                    hipStream_t s);
int errors_blocks(int Ea);

}  // namespace ba
}  // namespace rspl
