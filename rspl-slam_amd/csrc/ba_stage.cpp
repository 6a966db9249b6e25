// Host staging of a local BA call into landmark-CSR order (ba_stage.hpp).
#include "ba_stage.hpp"

#include <algorithm>

namespace rspl {
namespace ba {

namespace {

constexpr int kParWorkers = 3;  // + the calling thread

// f(part) for every part of the pool, part 0 on this thread
template <typename F>
void pool_run(HostPool* pool, F& f) {
  pool->run([](void* c, int q) { (*static_cast<F*>(c))(q); }, &f);
}

struct Edges {  // the caller's per-type edge arrays (types: mono point, stereo point, mono line, stereo line)
  const int32_t* pose[4];
  const int32_t* lm[4];
  const int32_t* cam[4];
  const double* obs[4];
  int ne[4], base[5];
  explicit Edges(const rspl_ba_problem* pr) {
    const int32_t* p[4] = {pr->mono_pose, pr->stereo_pose, pr->mono_line_pose, pr->stereo_line_pose};
    const int32_t* l[4] = {pr->mono_point, pr->stereo_point, pr->mono_line_line, pr->stereo_line_line};
    const int32_t* c[4] = {pr->mono_camera, pr->stereo_camera, pr->mono_line_camera, pr->stereo_line_camera};
    const double* o[4] = {pr->mono_obs, pr->stereo_obs, pr->mono_line_obs, pr->stereo_line_obs};
    const int n[4] = {pr->n_mono, pr->n_stereo, pr->n_mono_line, pr->n_stereo_line};
    base[0] = 0;
    for (int t = 0; t < 4; t++) {
      pose[t] = p[t];
      lm[t] = l[t];
      cam[t] = c[t];
      obs[t] = o[t];
      ne[t] = n[t];
      base[t + 1] = base[t] + n[t];
    }
  }
};

}  // namespace

int Stager::count(const rspl_ba_problem* pr, bool sharded, int rank, int nranks, int par_edges) {
  const Edges ed(pr);
  const int np = pr->n_poses, nq = pr->n_points, nl = pr->n_lines, nL = nq + nl, Eg = ed.base[4];
  for (int t = 0; t < 4; t++)
    RSPL_CHECK_ARG(ed.ne[t] == 0 || (ed.pose[t] && ed.lm[t] && ed.obs[t]), "NULL edge arrays");
  sh_ = sharded;
  rank_ = rank;
  nranks_ = nranks;
  pose_has_edge.assign(np, 0);
  uint8_t* pact = pose_has_edge.data();
  E = 0;
  Ep = 0;
  par_ = !sharded && par_edges > 0 && Eg >= par_edges;
  NP_ = 1;
  if (par_) {
    // (1) by caller-edge range p: validation, poses with edges, and every edge {caller id, landmark}
    //     into the bucket of its landmark range q (bucket (p, q): input order);
    // (2) by landmark range q: its landmarks' edge counts from the buckets (p = 0, 1, ...);
    // then place(), by landmark range q: its CSR offsets and positions from the buckets in bucket
    // order (= input order within a landmark) and the gather of its CSR range -- every thread writes
    // and re-reads only its own part of the staged arrays (no false sharing)
    if (!pool_) pool_.reset(new HostPool(kParWorkers));
    const int NP = NP_ = pool_->parts();
    bkt_.resize((size_t)NP * NP);
    pcnt_.resize(NP);
    ppact_.resize(NP);
    pcut_.resize(NP + 1);
    gcut_.resize(NP + 1);
    rstart_.resize(NP + 1);
    for (int q = 0; q <= NP; q++) {
      pcut_[q] = (int)((long long)Eg * q / NP);
      gcut_[q] = (int)((long long)nL * q / NP);
    }
    std::vector<char> bad(NP, 0);
    auto bucket_part = [&](int p) {
      for (int q = 0; q < NP; q++) bkt_[(size_t)p * NP + q].clear();
      std::vector<uint8_t>& pa = ppact_[p];
      pa.assign(np, 0);
      bool bd = false;
      for (int t = 0; t < 4; t++) {
        const int i0 = std::max(pcut_[p], ed.base[t]) - ed.base[t];
        const int i1 = std::min(pcut_[p + 1], ed.base[t + 1]) - ed.base[t];
        if (i0 >= i1) continue;
        const int lmax = t < 2 ? nq : nl, loff = t < 2 ? 0 : nq;
        const int32_t *pt = ed.pose[t], *lt = ed.lm[t], *ct = ed.cam[t];
        for (int i = i0; i < i1; i++) {
          const unsigned pp = (unsigned)pt[i], l = (unsigned)lt[i];
          const bool ok =
              (pp < (unsigned)np) & (l < (unsigned)lmax) & (!ct || (unsigned)ct[i] < (unsigned)pr->n_cameras);
          bd |= !ok;
          if (!ok) continue;
          pa[pp] = 1;
          const int g = loff + (int)l;
          int q = 0;
          while (g >= gcut_[q + 1]) q++;
          bkt_[(size_t)p * NP + q].push_back(make_int2(ed.base[t] + i, g));
        }
      }
      bad[p] = bd;
    };
    pool_run(pool_.get(), bucket_part);
    for (int q = 0; q < NP; q++) par_ = par_ && !bad[q];  // invalid input: the serial pass reports it
    if (par_) {
      auto count_range = [&](int q) {
        std::vector<int>& c = pcnt_[q];
        c.assign(gcut_[q + 1] - gcut_[q], 0);
        for (int p = 0; p < NP; p++)
          for (const int2& e : bkt_[(size_t)p * NP + q]) c[e.y - gcut_[q]]++;
      };
      pool_run(pool_.get(), count_range);
      rstart_[0] = 0;
      for (int q = 0; q < NP; q++) {
        int tot = 0;
        for (int c : pcnt_[q]) tot += c;
        rstart_[q + 1] = rstart_[q] + tot;
        for (int p = 0; p < np; p++) pact[p] |= ppact_[q][p];
      }
      E = Eg;
      Ep = ed.ne[0] + ed.ne[1];
      return RSPL_OK;
    }
    NP_ = 1;
  }
  lm_cnt_.assign(nL + 1, 0);
  int* cnt = lm_cnt_.data();
  for (int t = 0; t < 4; t++) {
    const int n = ed.ne[t], lmax = t < 2 ? nq : nl, loff = t < 2 ? 0 : nq;
    const int32_t *pt = ed.pose[t], *lt = ed.lm[t], *ct = ed.cam[t];
    // branch-free validation (unsigned compares), the offending edge looked up only on failure
    bool bad = false;
    for (int i = 0; i < n; i++) {
      const unsigned p = (unsigned)pt[i], l = (unsigned)lt[i];
      bad |= (p >= (unsigned)np) | (l >= (unsigned)lmax);
    }
    if (ct)
      for (int i = 0; i < n; i++) bad |= (unsigned)ct[i] >= (unsigned)pr->n_cameras;
    if (bad)
      for (int i = 0; i < n; i++) {
        const int p = pt[i], l = lt[i], c = ct ? ct[i] : 0;
        RSPL_CHECK_ARG(p >= 0 && p < np && l >= 0 && l < lmax && c >= 0 && c < pr->n_cameras,
                       "edge %d of type %d references a missing vertex/camera", i, t);
      }
    // a pose is optimised when it has an edge on ANY rank: K agrees across ranks
    for (int i = 0; i < n; i++) pact[pt[i]] = 1;
    if (!sharded) {
      for (int i = 0; i < n; i++) cnt[loff + lt[i] + 1]++;
      E += n;
      Ep += t < 2 ? n : 0;
    } else {
      for (int i = 0; i < n; i++)
        if ((loff + lt[i]) % nranks == rank) {
          cnt[loff + lt[i] + 1]++;
          E++;
          Ep += t < 2;
        }
    }
  }
  return RSPL_OK;
}

void Stager::place(const rspl_ba_problem* pr, const Out& o) {
  const Edges ed(pr);
  const int nq = pr->n_points, nL = nq + pr->n_lines;
  int* lm_off = o.lm_off;
  int* gmap = o.gmap;
  const int* pidx = o.pidx;
  const int Ep_ = Ep;
  double* lobs = o.eobs + 4 * (size_t)Ep_;
  // every staged array written sequentially in CSR order, gathered from the caller's arrays (point
  // edges: mono / stereo picked without a branch; the third observation of a mono edge is 0)
  auto gather = [&](int k0, int k1) {
    const int e1 = ed.base[1], e2 = ed.base[2], e3 = ed.base[3];
    static const double zero = 0.0;
    for (int k = k0; k < std::min(k1, Ep_); k++) {
      const int eg = gmap[k];
      const bool st = eg >= e1;
      const int i = st ? eg - e1 : eg;
      const int32_t* pt = st ? ed.pose[1] : ed.pose[0];
      const int32_t* ct = st ? ed.cam[1] : ed.cam[0];
      const int p = pt[i];
      o.etype[k] = (int8_t)st;
      o.epose[k] = p;
      o.elm[k] = (st ? ed.lm[1] : ed.lm[0])[i];
      o.ecam[k] = ct ? ct[i] : 0;
      o.lpose[k] = pidx[p];
      const double* ob = st ? ed.obs[1] + 3 * (size_t)i : ed.obs[0] + 2 * (size_t)i;
      double* ov = o.eobs + 4 * (size_t)k;
      ov[0] = ob[0];
      ov[1] = ob[1];
      ov[2] = *(st ? ob + 2 : &zero);  // no load past a mono record
    }
    for (int k = std::max(k0, Ep_); k < k1; k++) {
      const int eg = gmap[k];
      const int t = eg >= e3 ? 3 : 2;
      const int i = eg - (t == 3 ? e3 : e2);
      const int p = ed.pose[t][i];
      o.etype[k] = (int8_t)t;
      o.epose[k] = p;
      o.elm[k] = nq + ed.lm[t][i];
      o.ecam[k] = ed.cam[t] ? ed.cam[t][i] : 0;
      o.lpose[k] = pidx[p];
      const int D = t == 3 ? 8 : 4;
      const double* ob = ed.obs[t] + (size_t)D * i;
      double* ov = lobs + 8 * (size_t)(k - Ep_);
      for (int q = 0; q < D; q++) ov[q] = ob[q];
    }
  };
  if (par_) {  // by landmark range: its CSR offsets, its positions from the buckets, its gather
    const int NP = NP_;
    auto place_range = [&](int q) {
      const int g0 = gcut_[q], g1 = gcut_[q + 1];
      int* c = pcnt_[q].data();
      int run = rstart_[q];
      for (int g = g0; g < g1; g++) {  // counts -> CSR offsets -> cursors
        lm_off[g] = run;
        const int n = c[g - g0];
        c[g - g0] = run;
        run += n;
      }
      if (q == NP - 1) lm_off[nL] = run;
      for (int p = 0; p < NP; p++)
        for (const int2& e : bkt_[(size_t)p * NP + q]) gmap[c[e.y - g0]++] = e.x;
      gather(rstart_[q], rstart_[q + 1]);
    };
    pool_run(pool_.get(), place_range);
    return;
  }
  // CSR offsets (the edges of landmark g at [lm_off[g], lm_off[g+1]), point landmarks first), then the
  // CSR permutation -- each local edge's caller id at its CSR position (input order within a landmark:
  // the order every per-landmark reduction follows); one random store per edge
  lm_off[0] = 0;
  for (int g = 0; g < nL; g++) lm_off[g + 1] = lm_off[g] + lm_cnt_[g + 1];
  int* fill = lm_cnt_.data();  // reused as the per-landmark fill cursor
  for (int g = 0; g < nL; g++) fill[g] = lm_off[g];
  for (int t = 0; t < 4; t++) {
    const int n = ed.ne[t], loff = t < 2 ? 0 : nq;
    const int32_t* lt = ed.lm[t];
    if (!sh_) {
      for (int i = 0; i < n; i++) gmap[fill[loff + lt[i]]++] = ed.base[t] + i;
    } else {
      for (int i = 0; i < n; i++)
        if ((loff + lt[i]) % nranks_ == rank_) gmap[fill[loff + lt[i]]++] = ed.base[t] + i;
    }
  }
  gather(0, E);
}

}  // namespace ba
}  // namespace rspl
