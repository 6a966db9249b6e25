#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace rspl {
namespace frame {

// One unary pose-only edge (EdgeSE3ProjectXYZOnlyPose / EdgeStereoSE3ProjectXYZOnlyPose):
// the fixed world point Xw, the measurement and the camera it was taken with, 96 bytes.
struct Edge {
  double X[3];
  double obs[3];   // u, v, u_right (u_right unused for mono)
  double cam[5];   // fx fy cx cy bf
  double stereo;   // 0 mono, 1 stereo
};

struct Desc {      // one frame of the batch
  int e0, n;       // edges [e0, e0 + n)
  int pad[2];
  double T0[8];    // initial T_cw: q (w x y z), t, pad
  double delta[2]; // Huber deltas (mono, stereo) = (float)sqrt(th)
  double th[2];    // chi2 thresholds (mono, stereo)
};

struct Out {       // per-frame result, written into host-mapped memory
  double T[8];     // final T_cw
  double chi2[4];
  int iters[4];
  int n_inliers, rounds;
  int pad[2];
};

struct Args {
  const Desc* frames;
  const Edge* edges;
  const uint8_t* inl_in;  // [E] Constraint::inlier on entry
  double* err;            // [E][4] last computed error (scratch)
  uint8_t* level;         // [E] scratch: edge level (1 = outside the next optimize)
  uint8_t* inl;           // [E] scratch: Constraint::inlier during the call
  uint8_t* inl_out;       // [E] host-mapped
  Out* out;               // [B] host-mapped
};

// frames of up to kLdsEdges edges keep their edge records, errors and flags in LDS
// (122 B per edge: 62.5 KB at the cap); larger frames work from global scratch
constexpr int kLdsEdges = 512;

// one wavefront per frame; max_n = the largest frame's edge count
hipError_t optimize(const Args& a, int batch, int max_n, hipStream_t s);

}  // namespace frame
}  // namespace rspl
