// Host staging of one LocalmapOptimization call (rspl_ba_local): the caller's edge arrays (the
// reference's per-type constraint vectors, g2o_optimization.cc:81-167) validated, counted per landmark
// and placed in landmark-CSR order -- point landmarks first, each landmark's edges contiguous, input
// order within a landmark (the order every per-landmark reduction of the kernels follows).  Large
// unsharded calls run on a few persistent host workers (HostPool); the result is identical to the
// serial passes (rspl_ba_debug_stage: tests/test_ba_stage.py).
#pragma once

#include <memory>
#include <vector>

#include "common.hpp"
#include "host_pool.hpp"

namespace rspl {
namespace ba {

struct Stager {
  // pass 1: validate the edges, count the local edges per landmark, mark the poses with edges.
  // sharded: keep the edges of landmarks g % nranks == rank.  par_edges: stage on the workers from
  // this many edges (unsharded only; <= 0: never).  Sets E (local edges), Ep (local point edges) and
  // pose_has_edge; RSPL_E_ARG (message set) on invalid input.
  int count(const rspl_ba_problem* pr, bool sharded, int rank, int nranks, int par_edges);
  // pass 2: lm_off [nL + 1] and, per CSR position k < E, the edge's type, pose, landmark, camera,
  // caller id (gmap), reduced pose (pidx of its pose) and observation (points: 4 doubles each from
  // eobs; lines: 8 doubles each from eobs + 4 Ep)
  struct Out {
    int* lm_off;
    int8_t* etype;
    int* epose;
    int* elm;
    int* ecam;
    int* gmap;
    int* lpose;
    double* eobs;
    const int* pidx;
  };
  void place(const rspl_ba_problem* pr, const Out& o);

  int E = 0, Ep = 0;
  std::vector<uint8_t> pose_has_edge;  // [np]

 private:
  bool sh_ = false, par_ = false;
  int rank_ = 0, nranks_ = 1, NP_ = 1;
  std::vector<int> lm_cnt_;                  // serial: per-landmark counts (shifted by one), then cursors
  std::unique_ptr<HostPool> pool_;
  std::vector<std::vector<int2>> bkt_;       // parallel: [part][landmark range] {caller edge id, landmark}
  std::vector<std::vector<int>> pcnt_;       // parallel: [range] per-landmark counts, then CSR cursors
  std::vector<std::vector<uint8_t>> ppact_;  // parallel: [part] poses with edges
  std::vector<int> pcut_, gcut_, rstart_;    // part p: caller edges [pcut[p], pcut[p+1]); range q:
                                             //   landmarks [gcut[q], gcut[q+1]), CSR [rstart[q], rstart[q+1])
};

}  // namespace ba
}  // namespace rspl
