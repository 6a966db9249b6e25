// Map-side local BA: the keyframe / map-point / map-line graph the reference's Map keeps, and
// Map::LocalMapOptimization around LocalmapOptimization -- which keyframes, landmarks and
// observations enter the BA, the write-back, the outlier removal and the covisibility update.
//
// Reference (restated, not translated): src/map.cc:121-177 (UppdateMapline), :471-535
// (SearchNeighborFrames, AddFrameVertex), :537-808 (LocalMapOptimization), :810-895
// (MakeFramePair, RemoveOutliers, RemoveLineOutliers), :897-937 (UpdateFrameConnection),
// :1007-1024 (SaveKeyframeTrajectory); src/frame.cc:214-219, 372-405, 448-531 (keypoint / line
// accessors, covisibility bookkeeping); src/mappoint.cc, src/mapline.cc (observers, types).
//
// Shared pointers become ids: a frame / landmark is named by its id, and a slot of a frame's
// _mappoints / _maplines vector holds a landmark id or -1 (nullptr).  The reference orders equal
// covisibility weights (std::set<std::pair<int, FramePtr>>) by shared_ptr address, i.e. by
// allocation order; here ties are ordered by frame id (the same order when keyframes are allocated
// in id order, which is how MapBuilder creates them).
#include <algorithm>
#include <chrono>
#include <array>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <map>
#include <set>
#include <unordered_map>
#include <vector>

#include "common.hpp"

using rspl::set_error;

namespace {

enum { kUnTriangulated = 0, kGood = 1, kBad = 2 };  // Mappoint::Type / Mapline::Type

// The observer maps (frame id -> index) as a sorted vector: std::map's interface and ascending-key
// iteration order, without a heap node per observation (a landmark has tens of observers; the
// local-BA assembly walks every observer of every landmark of the window)
template <typename V>
struct FlatMap {
  using Item = std::pair<int, V>;
  std::vector<Item> v;
  using iterator = typename std::vector<Item>::iterator;
  using const_iterator = typename std::vector<Item>::const_iterator;
  iterator begin() { return v.begin(); }
  iterator end() { return v.end(); }
  const_iterator begin() const { return v.begin(); }
  const_iterator end() const { return v.end(); }
  size_t size() const { return v.size(); }
  bool empty() const { return v.empty(); }
  void clear() { v.clear(); }
  iterator lower(int k) {
    return std::lower_bound(v.begin(), v.end(), k, [](const Item& a, int key) { return a.first < key; });
  }
  const_iterator lower(int k) const {
    return std::lower_bound(v.begin(), v.end(), k, [](const Item& a, int key) { return a.first < key; });
  }
  iterator find(int k) {
    auto it = lower(k);
    return it != v.end() && it->first == k ? it : v.end();
  }
  const_iterator find(int k) const {
    auto it = lower(k);
    return it != v.end() && it->first == k ? it : v.end();
  }
  size_t count(int k) const { return find(k) != v.end(); }
  V& operator[](int k) {
    auto it = lower(k);
    if (it == v.end() || it->first != k) it = v.insert(it, Item(k, V{}));
    return it->second;
  }
  size_t erase(int k) {
    auto it = find(k);
    if (it == v.end()) return 0;
    v.erase(it);
    return 1;
  }
};

// id -> element pointer: a dense table for ids in [0, kDenseIds) (frame / landmark ids are counters),
// the hash map (which owns the elements; node-based, so pointers stay valid) for any other id
constexpr int kDenseIds = 1 << 22;
template <typename T>
struct IdIndex {
  std::vector<T*> dense;
  T* get(const std::unordered_map<int, T>& store, int id) const {
    if (id >= 0 && id < (int)dense.size()) return dense[id];
    if (id >= 0 && id < kDenseIds) return nullptr;  // dense range: absent
    auto it = store.find(id);
    return it == store.end() ? nullptr : const_cast<T*>(&it->second);
  }
  void put(int id, T* p) {
    if (id < 0 || id >= kDenseIds) return;
    if (id >= (int)dense.size()) dense.resize(std::max<size_t>(id + 1, dense.size() * 2), nullptr);
    dense[id] = p;
  }
};

struct MFrame {
  int id = 0;
  double ts = 0;
  double Twc[16] = {};                        // frame pose T_wc, row-major 4 x 4 (Frame::_pose)
  std::vector<std::array<double, 3>> kp;      // features rows 1-2 (x, y) and _u_right
  std::vector<int> mpt;                       // _mappoints: map-point id per keypoint or -1
  std::vector<std::array<double, 4>> ll, lr;  // _lines, _lines_right
  std::vector<uint8_t> lr_valid;              // _lines_right_valid
  std::vector<int> mpl;                       // _maplines: map-line id per line or -1
  std::vector<std::map<int, double>> pol;     // _points_on_lines
  std::map<int, int> conn;                    // _connections: frame id -> weight
  std::set<std::pair<int, int>> oconn;        // _ordered_connections: (weight, frame id)
  int parent = -1;
  int lmo = -1, lmo_fix = -1;                 // local_map_optimization_(fix_)frame_id
  int pidx = -1;                              // pose index in the last assembled problem

  // Frame::AddConnection(frame, weight) (frame.cc:458-469)
  void add_connection(int f, int w) {
    auto it = conn.find(f);
    const bool add = it == conn.end(), change = !add && it->second != w;
    if (add || change) {
      if (change) oconn.erase({it->second, f});
      conn[f] = w;
      oconn.insert({w, f});
    }
  }
  // Frame::AddConnection(set) (frame.cc:471-477)
  void set_connections(const std::set<std::pair<int, int>>& c) {
    oconn = c;
    conn.clear();
    for (auto& kv : c) conn[kv.second] = kv.first;
  }
  // Frame::DecreaseWeight (frame.cc:513-526)
  void decrease_weight(int f, int w) {
    auto it = conn.find(f);
    if (it == conn.end()) return;
    oconn.erase({it->second, f});
    const int ow = it->second;
    const bool remove = (ow < w + 5 && conn.size() >= 2) || ow <= w;
    if (remove) {
      conn.erase(it);
    } else {
      it->second = ow - w;
      oconn.insert({it->second, f});
    }
  }
  // GetKeypointPosition (frame.cc:214-219); the reference accepts idx == cols (an out-of-range
  // read), here idx must be in range
  bool keypoint(int idx, double* k) const {
    if (idx < 0 || idx >= (int)kp.size()) return false;
    for (int i = 0; i < 3; i++) k[i] = kp[idx][i];
    return true;
  }
  bool right_line_status(int idx) const { return idx >= 0 && idx < (int)lr_valid.size() && lr_valid[idx]; }
};

struct MPoint {  // Mappoint
  int id = 0;
  double p[3] = {};
  int type = kUnTriangulated;
  FlatMap<int> obs;        // _obversers: frame id -> keypoint index
  int lmo = -1;
  int observers() const {  // ObverserNum
    int n = 0;
    for (auto& kv : obs) n += kv.second >= 0;
    return n;
  }
  int keypoint_idx(int f) const {
    auto it = obs.find(f);
    return it == obs.end() ? -1 : it->second;
  }
};

struct MLine {  // Mapline
  int id = 0;
  double L[6] = {};  // g2o::Line3D (w, d)
  int type = kUnTriangulated;
  FlatMap<int> obs;         // frame id -> line index
  FlatMap<int> incl;        // _included_endpoints
  int lmo = -1;
  double ep[6] = {};
  bool ep_valid = false, to_update = false;
  int observers() const {
    int n = 0;
    for (auto& kv : obs) n += kv.second >= 0;
    return n;
  }
  int line_idx(int f) const {
    auto it = obs.find(f);
    return it == obs.end() ? -1 : it->second;
  }
};

// Eigen: Quaterniond from a rotation matrix (quaternionbase_assign_impl) -> (x, y, z, w)
void R_to_q(const double* M, int ld, double* q) {
  auto m = [&](int r, int c) { return M[r * ld + c]; };
  double t = m(0, 0) + m(1, 1) + m(2, 2);
  if (t > 0) {
    t = std::sqrt(t + 1.0);
    q[3] = 0.5 * t;
    t = 0.5 / t;
    q[0] = (m(2, 1) - m(1, 2)) * t;
    q[1] = (m(0, 2) - m(2, 0)) * t;
    q[2] = (m(1, 0) - m(0, 1)) * t;
  } else {
    int i = 0;
    if (m(1, 1) > m(0, 0)) i = 1;
    if (m(2, 2) > m(i, i)) i = 2;
    const int j = (i + 1) % 3, k = (j + 1) % 3;
    t = std::sqrt(m(i, i) - m(j, j) - m(k, k) + 1.0);
    q[i] = 0.5 * t;
    t = 0.5 / t;
    q[3] = (m(k, j) - m(j, k)) * t;
    q[j] = (m(j, i) + m(i, j)) * t;
    q[k] = (m(k, i) + m(i, k)) * t;
  }
}

// Eigen: Quaternion::toRotationMatrix, q = (x, y, z, w), into the upper-left 3 x 3 of a row-major
// matrix with leading dimension ld
void q_to_R(const double* q, double* M, int ld) {
  const double x = q[0], y = q[1], z = q[2], w = q[3];
  const double tx = 2 * x, ty = 2 * y, tz = 2 * z;
  const double twx = tx * w, twy = ty * w, twz = tz * w, txx = tx * x, txy = ty * x, txz = tz * x;
  const double tyy = ty * y, tyz = tz * y, tzz = tz * z;
  M[0] = 1 - (tyy + tzz); M[1] = txy - twz;       M[2] = txz + twy;
  M[ld] = txy + twz;      M[ld + 1] = 1 - (txx + tzz); M[ld + 2] = tyz - twx;
  M[2 * ld] = txz - twy;  M[2 * ld + 1] = tyz + twx;   M[2 * ld + 2] = 1 - (txx + tyy);
}

// g2o::Line3D::toCartesian: unit direction and the point solving (W^T W + 1e-9 I) p = W^T w,
// W = -[d]x (the point of the line closest to the origin, damped)
void line_to_cartesian(const double* L, double* c) {
  const double* w = L;
  const double* d = L + 3;
  const double dn = std::sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
  for (int i = 0; i < 3; i++) c[3 + i] = d[i] / dn;
  const double W[9] = {0, d[2], -d[1], -d[2], 0, d[0], d[1], -d[0], 0};  // -skew(d), row-major
  double A[9], b[3];
  for (int r = 0; r < 3; r++) {
    b[r] = 0;
    for (int k = 0; k < 3; k++) b[r] += W[k * 3 + r] * w[k];
    for (int cc = 0; cc < 3; cc++) {
      double s = 0;
      for (int k = 0; k < 3; k++) s += W[k * 3 + r] * W[k * 3 + cc];
      A[r * 3 + cc] = s + (r == cc ? 1e-9 : 0.0);
    }
  }
  // symmetric positive definite 3 x 3: Cholesky solve
  const double l00 = std::sqrt(A[0]), l10 = A[3] / l00, l20 = A[6] / l00;
  const double l11 = std::sqrt(A[4] - l10 * l10), l21 = (A[7] - l20 * l10) / l11;
  const double l22 = std::sqrt(A[8] - l20 * l20 - l21 * l21);
  const double y0 = b[0] / l00, y1 = (b[1] - l10 * y0) / l11, y2 = (b[2] - l20 * y0 - l21 * y1) / l22;
  c[2] = y2 / l22;
  c[1] = (y1 - l21 * c[2]) / l11;
  c[0] = (y0 - l10 * c[1] - l20 * c[2]) / l00;
}

}  // namespace

struct rspl_map {
  double cam[5] = {};
  rspl_map_config cfg{};
  std::unordered_map<int, MFrame> kf;  // _keyframes (by id; id order where the reference iterates it)
  std::vector<int> kf_ids;      // _keyframe_ids (insertion order)
  std::vector<int> kf_sorted;   // the same ids, ascending
  // _mappoints / _maplines: looked up by id only, never iterated (node-based: element pointers stay valid)
  std::unordered_map<int, MPoint> mp;
  std::unordered_map<int, MLine> ml;
  IdIndex<MFrame> kf_ix;
  IdIndex<MPoint> mp_ix;
  IdIndex<MLine> ml_ix;
  // the last assembled problem (rspl_map_last_problem)
  std::vector<int> pose_ids, point_ids, line_ids;
  std::vector<uint8_t> pose_fixed;
  std::vector<int32_t> c_pose[4], c_lm[4];
  std::vector<double> c_obs[4];
  std::vector<uint8_t> c_inl[4];
  // assembly scratch (kept across calls for their capacity): the window's landmarks, their
  // observers flattened, the kept landmarks (id, ordinal) and the ordinal -> dense index map
  struct Obs {
    const MFrame* f;
    int kp;
  };
  std::vector<MPoint*> lm_pts, kept_ptr;
  std::vector<int> lm_beg, lm_rank;
  std::vector<Obs> lm_obs;
  std::vector<std::pair<int, int>> kept_pts;
  // per call, by keyframe id: the frame's class for the window walk and its count of observations
  // outside the window (ids past the table: frame() and a std::map)
  enum : uint8_t { kNoFrame = 0, kWin = 1, kOut = 2, kOutFix = 3 };
  std::vector<uint8_t> fcls;
  std::vector<int> fcnt;
  std::vector<uint64_t> bad;  // remove_outliers scratch: pair keys, the pair table and its used cells
  std::vector<int> pair_cnt, pair_hit;

  MFrame* frame(int id) { return kf_ix.get(kf, id); }
  MPoint* point(int id) { return id < 0 ? nullptr : mp_ix.get(mp, id); }
  MLine* line(int id) { return id < 0 ? nullptr : ml_ix.get(ml, id); }

  // Map::UpdateFrameConnection (map.cc:897-937).  Counts per keyframe id in fcnt (ids past the
  // dense keyframe table in a std::map), read back in ascending id order.
  void update_connection(MFrame& f) {
    const std::vector<MFrame*>& kfd = kf_ix.dense;
    if (fcnt.size() < kfd.size()) fcnt.resize(kfd.size(), 0);
    std::map<int, int> big;
    bool any = false;
    const int nslot = (int)f.mpt.size();
    for (int s = 0; s < nslot; s++) {
      if (s + 8 < nslot)
        if (const MPoint* q = point(f.mpt[s + 8])) __builtin_prefetch(q);
      if (s + 4 < nslot)
        if (const MPoint* q = point(f.mpt[s + 4])) __builtin_prefetch(q->obs.v.data());
      const MPoint* m = point(f.mpt[s]);
      if (!m || m->type == kBad) continue;
      for (auto& kv : m->obs) {
        const int id = kv.first;
        if (id == f.id) continue;
        if ((unsigned)id < kfd.size()) {
          if (!kfd[id]) continue;
          fcnt[id]++;
        } else {
          if (!frame(id)) continue;
          big[id]++;
        }
        any = true;
      }
    }
    if (!any) return;
    std::set<std::pair<int, int>> good;
    int best = -1, best_w = -1;
    auto visit = [&](int id, int w) {  // ascending frame id (the reference's std::map)
      MFrame* cf = frame(id);
      if (w > best_w) {
        best = id;
        best_w = w;
      }
      if (w > 15) {
        good.insert({w, id});
        cf->add_connection(f.id, w);
      }
    };
    auto bi = big.begin();
    for (; bi != big.end() && bi->first < 0; ++bi) visit(bi->first, bi->second);
    for (int id : kf_sorted) {
      if (id < 0 || id >= (int)kfd.size() || !fcnt[id]) continue;
      const int w = fcnt[id];
      fcnt[id] = 0;
      visit(id, w);
    }
    for (; bi != big.end(); ++bi) visit(bi->first, bi->second);
    if (good.empty()) {
      good.insert({best_w, best});
      frame(best)->add_connection(f.id, best_w);
    }
    f.set_connections(good);
  }

  // Map::SearchNeighborFrames (map.cc:471-525); GetOrderedConnections is ascending by weight
  void search_neighbors(MFrame& f, std::vector<MFrame*>& nb) {
    constexpr size_t target = 9;
    const int fid = f.id;
    nb.clear();
    if (kf.size() <= target) {  // every keyframe, in id order (the reference's std::map)
      for (auto& kv : kf) nb.push_back(&kv.second);
      std::sort(nb.begin(), nb.end(), [](const MFrame* a, const MFrame* b) { return a->id < b->id; });
      for (MFrame* k : nb) k->lmo = fid;
      return;
    }
    nb.push_back(&f);
    f.lmo = fid;
    const std::vector<std::pair<int, int>> cs(f.oconn.begin(), f.oconn.end());
    const size_t first = std::min(cs.size(), target - 1);
    for (size_t i = 0; i < first; i++) {
      MFrame* c = frame(cs[i].second);
      c->lmo = fid;
      nb.push_back(c);
    }
    MFrame* par = frame(f.parent);
    if (par && par->lmo != fid) {
      par->lmo = fid;
      nb.push_back(par);
    }
    while (nb.size() < target) {
      std::map<int, int> deeper;
      for (MFrame* k : nb)
        for (auto& wc : k->oconn)
          if (frame(wc.second)->lmo != fid) deeper[wc.second] += wc.first;
      if (deeper.empty()) break;
      std::set<std::pair<int, int>> ord;
      for (auto& kv : deeper) ord.insert({kv.second, kv.first});
      size_t add = std::min(target - nb.size(), ord.size());
      for (auto it = ord.rbegin(); add > 0; add--, ++it) {
        MFrame* c = frame(it->second);
        c->lmo = fid;
        nb.push_back(c);
      }
    }
  }

  // Map::RemoveOutliers (map.cc:818-863).  frame->RemoveMappoint(mpt) runs after the observer was
  // removed, so it looks up index -1 and leaves the frame's slot as it is -- kept as in the reference.
  void remove_outliers(const std::vector<std::pair<int, int>>& outl) {
    // MakeFramePair per (outlier, other observer) as one key, ascending (max, min) order when sorted
    // as unsigned.  Frame ids are offset by 2^31 so that negative ids order too.
    auto key = [](int a, int b) {
      return (uint64_t)((uint32_t)a ^ 0x80000000u) << 32 | (uint32_t)((uint32_t)b ^ 0x80000000u);
    };
    // the pairs are counted first in a (outlier frame, observer id) table -- the outlier frames are
    // the window's few poses -- and only the distinct pairs are sorted; observers past the dense
    // keyframe table go to the key list directly
    const std::vector<MFrame*>& kfd = kf_ix.dense;
    const size_t ncol = kfd.size();
    std::vector<int> rows;  // outlier frame ids, one table row each
    bad.clear();
    pair_hit.clear();
    for (auto& fm : outl) {
      MFrame* f = frame(fm.first);
      MPoint* m = point(fm.second);
      if (!f || !m || m->type == kBad) continue;
      m->obs.erase(f->id);
      const FlatMap<int>& obs = m->obs;  // read before the clear below (the reference copies it under its lock)
      const size_t r = std::find(rows.begin(), rows.end(), f->id) - rows.begin();
      if (r == rows.size()) {
        rows.push_back(f->id);
        if (pair_cnt.size() < rows.size() * ncol) pair_cnt.resize(rows.size() * ncol, 0);
      }
      int* row = pair_cnt.data() + r * ncol;
      for (auto& ob : obs) {
        const int id = ob.first;
        if ((unsigned)id < ncol) {
          if (!kfd[id]) continue;
          if (row[id]++ == 0) pair_hit.push_back((int)(r * ncol) + id);
        } else if (frame(id)) {
          bad.push_back(key(std::max(f->id, id), std::min(f->id, id)));  // MakeFramePair
        }
      }
      if (m->observers() < 2 && m->type != kBad) {
        bool del = true;
        if (m->observers() > 0) {
          MFrame* o = frame(obs.begin()->first);
          if (o) {
            const int k = m->keypoint_idx(o->id);
            if (k >= 0 && k < (int)o->kp.size() && o->kp[k][2] < 0) {  // GetRightPosition(k) < 0: mono
              const int slot = obs.begin()->second;
              if (slot >= 0 && slot < (int)o->mpt.size()) o->mpt[slot] = -1;
            } else {
              del = false;
            }
          }
        }
        if (del) {
          m->type = kBad;
          m->obs.clear();
        }
      }
      // frame->RemoveMappoint(mpt): GetKeypointIdx(frame id) is -1 by now -> no-op
    }
    // the reference's std::map<pair, int> of counts: pairs in ascending order, each with its count
    std::vector<std::pair<uint64_t, int>> cnt;
    cnt.reserve(pair_hit.size() + bad.size());
    for (int h : pair_hit) {
      const int f = rows[h / ncol], o = h % ncol;
      cnt.push_back({key(std::max(f, o), std::min(f, o)), pair_cnt[h]});
      pair_cnt[h] = 0;
    }
    for (uint64_t k : bad) cnt.push_back({k, 1});
    std::sort(cnt.begin(), cnt.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
    for (size_t i = 0; i < cnt.size();) {
      size_t j = i;
      int n = 0;
      for (; j < cnt.size() && cnt[j].first == cnt[i].first; j++) n += cnt[j].second;
      const int a = (int)((uint32_t)(cnt[i].first >> 32) ^ 0x80000000u), b = (int)((uint32_t)cnt[i].first ^ 0x80000000u);
      frame(a)->decrease_weight(b, n);
      frame(b)->decrease_weight(a, n);
      i = j;
    }
  }

  // Map::RemoveLineOutliers (map.cc:865-895); the final frame->RemoveMapline is a no-op likewise
  void remove_line_outliers(const std::vector<std::pair<int, int>>& outl) {
    for (auto& fl : outl) {
      MFrame* f = frame(fl.first);
      MLine* l = line(fl.second);
      if (!f || !l || l->type == kBad) continue;
      l->obs.erase(f->id);
      l->incl.erase(f->id);
      const FlatMap<int>& obs = l->obs;
      if (l->observers() < 2 && l->type != kBad) {
        bool del = true;
        if (l->observers() > 0) {
          MFrame* o = frame(obs.begin()->first);
          if (o) {
            if (!o->right_line_status(l->line_idx(o->id))) {
              const int slot = obs.begin()->second;
              if (slot >= 0 && slot < (int)o->mpl.size()) o->mpl[slot] = -1;
            } else {
              del = false;
            }
          }
        }
        if (del) {
          l->type = kBad;
          l->obs.clear();
        }
      }
    }
  }

  // Map::UppdateMapline (map.cc:121-177)
  bool update_mapline(MLine& l) {
    if (l.type != kGood || l.obs.empty()) return false;
    std::vector<std::array<double, 3>> pts;
    for (auto& kv : l.obs) {
      MFrame* f = frame(kv.first);
      if (!f) continue;
      if (kv.second < 0 || kv.second >= (int)f->pol.size()) continue;  // GetPointsOnLine: empty map
      for (auto& pd : f->pol[kv.second]) {
        if (pd.first < 0 || pd.first >= (int)f->mpt.size()) continue;
        const MPoint* m = point(f->mpt[pd.first]);
        if (m && m->type == kGood) pts.push_back({m->p[0], m->p[1], m->p[2]});
      }
    }
    double c[6];
    line_to_cartesian(l.L, c);
    const double* lp = c;
    const double* v = c + 3;
    int md = 0;  // main direction: first index of the largest |component| (Eigen maxCoeff)
    for (int i = 1; i < 3; i++)
      if (std::fabs(v[i]) > std::fabs(v[md])) md = i;
    double mx = DBL_MIN, mn = DBL_MAX;  // DBL_MIN (> 0) as in the reference
    bool fmax = false, fmin = false;
    for (auto& p : pts) {
      const double dp[3] = {p[0] - lp[0], p[1] - lp[1], p[2] - lp[2]};
      const double cr[3] = {v[1] * dp[2] - v[2] * dp[1], v[2] * dp[0] - v[0] * dp[2], v[0] * dp[1] - v[1] * dp[0]};
      const double dist = std::sqrt(cr[0] * cr[0] + cr[1] * cr[1] + cr[2] * cr[2]);  // EigenPointLineDistance3D
      if (dist > 0.2) continue;
      const double di = p[md];
      if (di > mx) {
        mx = di;
        fmax = true;
      }
      if (di < mn) {
        mn = di;
        fmin = true;
      }
    }
    if (!fmax || !fmin) return false;
    const double r1 = (mx - lp[md]) / v[md], r2 = (mn - lp[md]) / v[md];
    for (int i = 0; i < 3; i++) {
      l.ep[i] = lp[i] + r1 * v[i];
      l.ep[3 + i] = lp[i] + r2 * v[i];
    }
    l.ep_valid = true;  // SetEndpoints(endpoints, false)
    l.to_update = false;
    return true;
  }

  struct PoseV {
    double q[4], p[3];
    bool fixed;
  };
  // Map::AddFrameVertex (map.cc:527-535): std::map::insert keeps an existing entry
  static void add_vertex(std::map<int, PoseV>& poses, const MFrame& f, bool fixed) {
    if (poses.count(f.id)) return;
    PoseV v;
    R_to_q(f.Twc, 4, v.q);
    for (int i = 0; i < 3; i++) v.p[i] = f.Twc[4 * i + 3];
    v.fixed = fixed;
    poses.emplace(f.id, v);
  }

  // Map::LocalMapOptimization (map.cc:537-808): assembly (into the last-problem vectors), the
  // GPU LocalmapOptimization when ba != null, then outlier removal and write-back
  int local_map_optimization(int fid, rspl_ba* ba, rspl_map_report* rep) {
    MFrame* nf = frame(fid);
    if (!nf) {
      set_error("rspl_map_local_optimization: frame %d is not a keyframe", fid);
      return RSPL_E_ARG;
    }
    static const bool timing = getenv("RSPL_MAP_TIMING") != nullptr;
    using clk = std::chrono::steady_clock;
    clk::time_point tm[6];
    int ntm = 0;
    auto mark = [&]() {
      if (timing) tm[ntm++] = clk::now();
    };
    const auto t_start = clk::now();
    mark();
    update_connection(*nf);
    mark();
    std::map<int, PoseV> poses;
    std::vector<MFrame*> nb;
    search_neighbors(*nf, nb);
    size_t fixed_num = 0;
    for (MFrame* k : nb) {
      const bool fix = k->id == 0;
      fixed_num += fix;
      add_vertex(poses, *k, fix);
    }
    // frame classes: in the window (lmo), outside it, or outside it but marked lmo_fix by an earlier
    // call for this frame id (counted as outside, yet in the window for the constraints, as the
    // reference's two checks read it)
    auto classify = [&](const MFrame* o) -> uint8_t {
      return o->lmo == fid ? kWin : o->lmo_fix == fid ? kOutFix : kOut;
    };
    {
      int top = -1;
      for (int id : kf_ids)
        if (id < kDenseIds) top = std::max(top, id);
      fcls.assign((size_t)(top + 1), kNoFrame);
      if (fcnt.size() < fcls.size()) fcnt.resize(fcls.size(), 0);
      for (int id : kf_ids)
        if (id >= 0 && id <= top) fcls[id] = classify(frame(id));
    }
    std::map<int, int> big_cnt;
    bool any_fixed = false;
    // the window's landmarks in the reference's order (frame by frame, slot by slot), each with its
    // window observers (frame, keypoint index) copied into one flat array, so the constraint pass below
    // reads them sequentially instead of chasing every landmark's observer list a second time; the
    // other observers are only counted per frame (the fixed-frame choice, map.cc:588-602)
    lm_pts.clear();
    lm_beg.clear();
    lm_obs.clear();
    std::vector<int> mpls;
    for (MFrame* k : nb) {
      const int nslot = (int)k->mpt.size();
      for (int s = 0; s < nslot; s++) {
        // the landmarks are scattered heap nodes: fetch the node 8 slots ahead and its observer list 4 ahead
        if (s + 8 < nslot)
          if (const MPoint* q = point(k->mpt[s + 8])) __builtin_prefetch(q);
        if (s + 4 < nslot)
          if (const MPoint* q = point(k->mpt[s + 4])) __builtin_prefetch(q->obs.v.data());
        MPoint* m = point(k->mpt[s]);
        if (!m || m->type != kGood || m->lmo == fid) continue;
        m->lmo = fid;
        lm_pts.push_back(m);
        lm_beg.push_back((int)lm_obs.size());
        for (auto& kv : m->obs) {
          const int id = kv.first;
          uint8_t c;
          if ((unsigned)id < fcls.size()) {
            c = fcls[id];
            if (c >= kOut) fcnt[id]++;
          } else {
            const MFrame* o = frame(id);
            c = o ? classify(o) : kNoFrame;
            if (c >= kOut) big_cnt[id]++;
          }
          if (c == kNoFrame) continue;
          any_fixed |= c >= kOut;
          if (c != kOut) lm_obs.push_back({frame(id), kv.second});
        }
      }
      for (int lid : k->mpl) {
        MLine* l = line(lid);
        if (!l || l->type != kGood || l->lmo == fid) continue;
        l->lmo = fid;
        mpls.push_back(lid);
      }
    }
    lm_beg.push_back((int)lm_obs.size());
    const size_t max_fixed = 1;
    // the frame with the most observations, ties to the larger id (the reference's
    // std::set<pair<int, FramePtr>> read from rbegin; max_fixed - fixed_num is at most 1)
    int fx_id = -1, fx_w = 0;
    auto consider = [&](int id, int w) {
      if (w > fx_w || (w == fx_w && w > 0 && id > fx_id)) {
        fx_id = id;
        fx_w = w;
      }
    };
    for (int id : kf_ids)
      if (id >= 0 && id < (int)fcls.size()) {
        consider(id, fcnt[id]);
        fcnt[id] = 0;
      }
    for (auto& kv : big_cnt) consider(kv.first, kv.second);
    const MFrame* fx = nullptr;  // the fixed frame, when its observations are not in lm_obs yet
    if (any_fixed && max_fixed > fixed_num) {
      MFrame* o = frame(fx_id);
      if (o->lmo_fix != fid) fx = o;
      o->lmo_fix = fid;
      add_vertex(poses, *o, true);
    }
    // dense poses: std::map ids in ascending order (LocalmapOptimization's vertex order); every
    // frame of the window (lmo or lmo_fix == fid) is a vertex and learns its index here
    pose_ids.clear(); point_ids.clear(); line_ids.clear(); pose_fixed.clear();
    std::vector<double> pq, pp, X, Ls;
    for (auto& kv : poses) {
      frame(kv.first)->pidx = (int)pose_ids.size();
      pose_ids.push_back(kv.first);
      pose_fixed.push_back(kv.second.fixed);
      pq.insert(pq.end(), kv.second.q, kv.second.q + 4);
      pp.insert(pp.end(), kv.second.p, kv.second.p + 3);
    }
    mark();
    auto in_window = [&](const MFrame* o) { return o->lmo == fid || o->lmo_fix == fid; };
    // constraints in the reference's order: landmark by landmark, observers by frame id (the fixed
    // frame's observation, looked up in the landmark's observer map, merged into that order), written
    // straight into the dense arrays; a landmark that is dropped (no stereo and at most one mono
    // observation) has its rows taken back.  c_lm holds the kept landmark's ordinal until the
    // landmarks are numbered by id below.
    for (int t = 0; t < 4; t++) {
      c_pose[t].clear(); c_lm[t].clear(); c_obs[t].clear();
    }
    kept_pts.clear();
    kept_ptr.clear();
    for (size_t li = 0; li < lm_pts.size(); li++) {
      const size_t b0 = c_pose[0].size(), b1 = c_pose[1].size();
      const int ord_lm = (int)kept_pts.size();
      auto emit = [&](const MFrame* o, int kpi) {
        if (kpi < 0 || kpi >= (int)o->kp.size()) return;  // GetKeypointPosition
        const double* k = o->kp[kpi].data();
        const int t = k[2] > 0 ? 1 : 0;
        c_pose[t].push_back(o->pidx);
        c_lm[t].push_back(ord_lm);
        c_obs[t].insert(c_obs[t].end(), k, k + 2 + t);
      };
      int fx_kp = fx ? lm_pts[li]->keypoint_idx(fx->id) : -1;
      for (int j = lm_beg[li]; j < lm_beg[li + 1]; j++) {
        const MFrame* o = lm_obs[j].f;
        if (fx_kp >= 0 && o->id > fx->id) {
          emit(fx, fx_kp);
          fx_kp = -1;
        }
        emit(o, lm_obs[j].kp);
      }
      if (fx_kp >= 0) emit(fx, fx_kp);
      if (c_pose[1].size() > b1 || c_pose[0].size() > b0 + 1) {
        kept_pts.push_back({lm_pts[li]->id, ord_lm});
        kept_ptr.push_back(lm_pts[li]);
      } else {
        c_pose[0].resize(b0); c_lm[0].resize(b0); c_obs[0].resize(2 * b0);
        c_pose[1].resize(b1); c_lm[1].resize(b1); c_obs[1].resize(3 * b1);
      }
    }
    std::vector<std::pair<int, MLine*>> kept_lines;
    for (int lid : mpls) {
      MLine* l = line(lid);
      if (!l || l->type != kGood) continue;
      const size_t b0 = c_pose[2].size(), b1 = c_pose[3].size();
      const int ord_lm = (int)kept_lines.size();
      for (auto& kv : l->obs) {
        MFrame* o = frame(kv.first);
        if (!o || !in_window(o)) continue;
        if (kv.second < 0 || kv.second >= (int)o->ll.size()) continue;  // GetLine
        const int t = o->right_line_status(kv.second) ? 3 : 2;          // GetLineRight
        c_pose[t].push_back(o->pidx);
        c_lm[t].push_back(ord_lm);
        c_obs[t].insert(c_obs[t].end(), o->ll[kv.second].begin(), o->ll[kv.second].end());
        if (t == 3) c_obs[t].insert(c_obs[t].end(), o->lr[kv.second].begin(), o->lr[kv.second].end());
      }
      if (c_pose[3].size() > b1 || c_pose[2].size() > b0 + 1) {
        kept_lines.push_back({lid, l});
      } else {
        c_pose[2].resize(b0); c_lm[2].resize(b0); c_obs[2].resize(4 * b0);
        c_pose[3].resize(b1); c_lm[3].resize(b1); c_obs[3].resize(8 * b1);
      }
    }
    mark();
    // dense landmarks: ascending id; constraint rows renumbered from the ordinal
    std::sort(kept_pts.begin(), kept_pts.end());
    lm_rank.resize(kept_pts.size());
    X.resize(3 * kept_pts.size());
    point_ids.resize(kept_pts.size());
    for (size_t i = 0; i < kept_pts.size(); i++) {
      const MPoint* m = kept_ptr[kept_pts[i].second];
      lm_rank[kept_pts[i].second] = (int)i;
      point_ids[i] = kept_pts[i].first;
      for (int c = 0; c < 3; c++) X[3 * i + c] = m->p[c];
    }
    for (int t = 0; t < 2; t++)
      for (auto& v : c_lm[t]) v = lm_rank[v];
    std::vector<int> line_rank(kept_lines.size());
    {
      std::vector<int> o(kept_lines.size());
      for (size_t i = 0; i < o.size(); i++) o[i] = (int)i;
      std::sort(o.begin(), o.end(), [&](int a, int b) { return kept_lines[a].first < kept_lines[b].first; });
      Ls.resize(6 * o.size());
      line_ids.resize(o.size());
      for (size_t i = 0; i < o.size(); i++) {
        line_rank[o[i]] = (int)i;
        line_ids[i] = kept_lines[o[i]].first;
        std::copy(kept_lines[o[i]].second->L, kept_lines[o[i]].second->L + 6, Ls.begin() + 6 * i);
      }
    }
    for (int t = 2; t < 4; t++)
      for (auto& v : c_lm[t]) v = line_rank[v];
    for (int t = 0; t < 4; t++) c_inl[t].assign(c_pose[t].size(), 1);
    if (rep) {
      memset(rep, 0, sizeof(*rep));
      rep->n_poses = (int)pose_ids.size();
      for (uint8_t f : pose_fixed) rep->n_fixed += f;
      rep->n_points = (int)point_ids.size();
      rep->n_lines = (int)line_ids.size();
      rep->n_mono = (int)c_pose[0].size();
      rep->n_stereo = (int)c_pose[1].size();
      rep->n_mono_line = (int)c_pose[2].size();
      rep->n_stereo_line = (int)c_pose[3].size();
    }
    mark();
    if (timing && ntm == 5) {
      auto us = [&](int i) { return std::chrono::duration<double, std::micro>(tm[i + 1] - tm[i]).count(); };
      fprintf(stderr, "rspl_map assembly us: connections %.0f window %.0f constraints %.0f dense %.0f\n", us(0), us(1),
              us(2), us(3));
    }
    last_fid = fid;
    last_cons_ok = true;
    if (!ba) return RSPL_OK;  // assembly only (rspl_map_assemble)
    const int np = (int)pose_ids.size();
    std::vector<double> rq(4 * (size_t)np), rp(3 * (size_t)np), rX(X.size()), rL(Ls.size());
    rspl_ba_problem P{};
    P.n_cameras = 1;
    P.cameras = cam;
    P.n_poses = np;
    P.pose_q = pq.data();
    P.pose_p = pp.data();
    P.pose_fixed = pose_fixed.data();
    P.n_points = (int)point_ids.size();
    P.points = X.data();
    P.n_lines = (int)line_ids.size();
    P.lines = Ls.data();
    P.n_mono = (int)c_pose[0].size(); P.mono_pose = c_pose[0].data(); P.mono_point = c_lm[0].data(); P.mono_obs = c_obs[0].data();
    P.n_stereo = (int)c_pose[1].size(); P.stereo_pose = c_pose[1].data(); P.stereo_point = c_lm[1].data(); P.stereo_obs = c_obs[1].data();
    P.n_mono_line = (int)c_pose[2].size(); P.mono_line_pose = c_pose[2].data(); P.mono_line_line = c_lm[2].data();
    P.mono_line_obs = c_obs[2].data();
    P.n_stereo_line = (int)c_pose[3].size(); P.stereo_line_pose = c_pose[3].data(); P.stereo_line_line = c_lm[3].data();
    P.stereo_line_obs = c_obs[3].data();
    P.th_mono_point = cfg.th_mono_point; P.th_stereo_point = cfg.th_stereo_point;
    P.th_mono_line = cfg.th_mono_line; P.th_stereo_line = cfg.th_stereo_line;
    P.iterations_first = cfg.iterations_first;
    P.iterations_second = cfg.iterations_second;
    rspl_ba_result R{};
    R.pose_q = rq.data(); R.pose_p = rp.data(); R.points = rX.data(); R.lines = rL.data();
    R.mono_inlier = c_inl[0].data(); R.stereo_inlier = c_inl[1].data();
    R.mono_line_inlier = c_inl[2].data(); R.stereo_line_inlier = c_inl[3].data();
    const auto t_ba = clk::now();
    const int rc = rspl_ba_local(ba, &P, &R);
    if (rc) return rc;
    const auto t_fin = clk::now();
    const int rf = finish(R, rep);
    if (rep) {
      auto us = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
      rep->assembly_us = us(t_start, t_ba);
      rep->ba_us = us(t_ba, t_fin);
      rep->finish_us = us(t_fin, clk::now());
    }
    return rf;
  }

  // the part of Map::LocalMapOptimization after LocalmapOptimization returns (map.cc:712-802), on
  // the last assembled problem: outliers, covisibility, write-back
  int last_fid = -1;
  bool last_cons_ok = false;
  int finish(const rspl_ba_result& R, rspl_map_report* rep) {
    if (!last_cons_ok || !frame(last_fid)) {
      set_error("rspl_map_finish: no assembled problem");
      return RSPL_E_ARG;
    }
    last_cons_ok = false;
    MFrame* nf = frame(last_fid);
    static const bool timing = getenv("RSPL_MAP_TIMING") != nullptr;
    using clk = std::chrono::steady_clock;
    clk::time_point tm[8];
    int ntm = 0;
    auto mark = [&]() {
      if (timing) tm[ntm++] = clk::now();
    };
    mark();
    const int np = (int)pose_ids.size();
    const double* rq = R.pose_q;
    const double* rp = R.pose_p;
    const double* rX = R.points;
    const double* rL = R.lines;
    const uint8_t* inl[4] = {R.mono_inlier, R.stereo_inlier, R.mono_line_inlier, R.stereo_line_inlier};
    for (int t = 0; t < 4; t++)
      if (inl[t]) std::copy(inl[t], inl[t] + c_pose[t].size(), c_inl[t].begin());
    if (rep) {
      rep->chi2_first = R.chi2_first;
      rep->chi2_second = R.chi2_second;
      rep->iterations_first = R.iterations_done_first;
      rep->iterations_second = R.iterations_done_second;
    }
    // outliers (map.cc:712-757), in constraint order: mono then stereo points, then lines
    std::vector<std::pair<int, int>> outl, loutl;
    for (int t = 0; t < 4; t++) {
      const std::vector<int>& ids = t < 2 ? point_ids : line_ids;
      for (size_t i = 0; i < c_pose[t].size(); i++) {
        if (c_inl[t][i]) continue;
        const int f = pose_ids[c_pose[t][i]], l = ids[c_lm[t][i]];
        if (!frame(f)) continue;
        if (t < 2 && point(l)) outl.push_back({f, l});
        if (t >= 2 && line(l)) loutl.push_back({f, l});
      }
    }
    if (rep) {
      rep->n_point_outliers = (int)outl.size();
      rep->n_line_outliers = (int)loutl.size();
    }
    mark();
    remove_outliers(outl);
    remove_line_outliers(loutl);
    mark();
    update_connection(*nf);
    mark();
    // write-back (map.cc:767-802)
    for (int i = 0; i < np; i++) {
      MFrame* f = frame(pose_ids[i]);
      if (!f) continue;
      double T[16] = {};
      q_to_R(rq + 4 * (size_t)i, T, 4);
      for (int r = 0; r < 3; r++) T[4 * r + 3] = rp[3 * (size_t)i + r];
      T[15] = 1.0;
      memcpy(f->Twc, T, sizeof(T));
    }
    for (size_t i = 0; i < point_ids.size(); i++) {
      if (i + 8 < point_ids.size()) __builtin_prefetch(point(point_ids[i + 8]), 1);
      MPoint* m = point(point_ids[i]);
      if (!m) continue;
      for (int k = 0; k < 3; k++) m->p[k] = rX[3 * i + k];
      if (m->type == kUnTriangulated) m->type = kGood;
    }
    for (size_t i = 0; i < line_ids.size(); i++) {
      MLine* l = line(line_ids[i]);
      if (!l) continue;
      for (int k = 0; k < 6; k++) l->L[k] = rL[6 * i + k];
      l->to_update = true;  // SetLine3D
      if (l->type == kUnTriangulated) l->type = kGood;
      l->ep_valid = update_mapline(*l);
    }
    mark();
    if (timing && ntm == 5) {
      auto us = [&](int i) { return std::chrono::duration<double, std::micro>(tm[i + 1] - tm[i]).count(); };
      fprintf(stderr, "rspl_map finish us: outliers %.0f remove %.0f connections %.0f write-back %.0f\n", us(0), us(1),
              us(2), us(3));
    }
    return RSPL_OK;
  }
};

// ---------------------------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------------------------
extern "C" int rspl_map_create(const rspl_map_config* cfg, rspl_map** out) {
  RSPL_CHECK_ARG(cfg && out && cfg->camera, "rspl_map_create: NULL argument");
  auto* m = new rspl_map();
  m->cfg = *cfg;
  memcpy(m->cam, cfg->camera, sizeof(m->cam));
  m->cfg.camera = m->cam;
  *out = m;
  return RSPL_OK;
}

extern "C" void rspl_map_destroy(rspl_map* m) { delete m; }

extern "C" int rspl_map_add_keyframe(rspl_map* m, const rspl_map_keyframe* k) {
  RSPL_CHECK_ARG(m && k && k->Twc, "rspl_map_add_keyframe: NULL argument");
  RSPL_CHECK_ARG(k->n_keypoints >= 0 && k->n_lines >= 0, "rspl_map_add_keyframe: negative counts");
  RSPL_CHECK_ARG(!m->kf.count(k->frame_id), "rspl_map_add_keyframe: frame %d exists", k->frame_id);
  MFrame f;
  f.id = k->frame_id;
  f.ts = k->timestamp;
  memcpy(f.Twc, k->Twc, sizeof(f.Twc));
  f.kp.resize(k->n_keypoints);
  for (int i = 0; i < k->n_keypoints; i++)
    for (int c = 0; c < 3; c++) f.kp[i][c] = k->keypoints[3 * i + c];
  f.mpt.assign(k->n_keypoints, -1);
  f.ll.resize(k->n_lines);
  f.lr.resize(k->n_lines);
  f.lr_valid.assign(k->n_lines, 0);
  f.mpl.assign(k->n_lines, -1);
  f.pol.resize(k->n_lines);
  for (int i = 0; i < k->n_lines; i++) {
    for (int c = 0; c < 4; c++) {
      f.ll[i][c] = k->lines_left[4 * i + c];
      f.lr[i][c] = k->lines_right ? k->lines_right[4 * i + c] : 0.0;
    }
    f.lr_valid[i] = k->lines_right_valid ? k->lines_right_valid[i] : 0;
    if (k->pol_offsets)
      for (int j = k->pol_offsets[i]; j < k->pol_offsets[i + 1]; j++) f.pol[i][k->pol_points[j]] = k->pol_dist[j];
  }
  f.parent = k->parent_id;
  const int fid = f.id;
  MFrame* fp = &m->kf.emplace(fid, std::move(f)).first->second;
  m->kf_ix.put(fid, fp);
  m->kf_ids.push_back(k->frame_id);
  m->kf_sorted.insert(std::upper_bound(m->kf_sorted.begin(), m->kf_sorted.end(), fid), fid);
  return RSPL_OK;
}

extern "C" int rspl_map_add_mappoint(rspl_map* m, int id, const double* p, int type) {
  RSPL_CHECK_ARG(m && p && type >= 0 && type <= 2, "rspl_map_add_mappoint: bad argument");
  RSPL_CHECK_ARG(!m->mp.count(id), "rspl_map_add_mappoint: map point %d exists", id);
  MPoint q;
  q.id = id;
  q.type = type;
  for (int i = 0; i < 3; i++) q.p[i] = p[i];
  m->mp_ix.put(id, &m->mp.emplace(id, q).first->second);
  return RSPL_OK;
}

extern "C" int rspl_map_add_mapline(rspl_map* m, int id, const double* line3d, int type) {
  RSPL_CHECK_ARG(m && line3d && type >= 0 && type <= 2, "rspl_map_add_mapline: bad argument");
  RSPL_CHECK_ARG(!m->ml.count(id), "rspl_map_add_mapline: map line %d exists", id);
  MLine l;
  l.id = id;
  l.type = type;
  for (int i = 0; i < 6; i++) l.L[i] = line3d[i];
  m->ml_ix.put(id, &m->ml.emplace(id, l).first->second);
  return RSPL_OK;
}

extern "C" int rspl_map_add_point_observation(rspl_map* m, int point_id, int frame_id, int kp) {
  RSPL_CHECK_ARG(m, "rspl_map_add_point_observation: NULL map");
  MPoint* q = m->point(point_id);
  MFrame* f = m->frame(frame_id);
  RSPL_CHECK_ARG(q && f && kp >= 0 && kp < (int)f->kp.size(), "rspl_map_add_point_observation: bad ids");
  q->obs[frame_id] = kp;  // Mappoint::AddObverser
  f->mpt[kp] = point_id;  // Frame::InsertMappoint
  return RSPL_OK;
}

extern "C" int rspl_map_add_line_observation(rspl_map* m, int line_id, int frame_id, int idx) {
  RSPL_CHECK_ARG(m, "rspl_map_add_line_observation: NULL map");
  MLine* l = m->line(line_id);
  MFrame* f = m->frame(frame_id);
  RSPL_CHECK_ARG(l && f && idx >= 0 && idx < (int)f->ll.size(), "rspl_map_add_line_observation: bad ids");
  l->obs[frame_id] = idx;
  f->mpl[idx] = line_id;
  return RSPL_OK;
}

extern "C" int rspl_map_add_mappoints(rspl_map* m, int n, const int32_t* ids, const double* p, const int32_t* types) {
  RSPL_CHECK_ARG(m && (n == 0 || (ids && p)), "rspl_map_add_mappoints: NULL argument");
  for (int i = 0; i < n; i++) {
    const int rc = rspl_map_add_mappoint(m, ids[i], p + 3 * (size_t)i, types ? types[i] : kGood);
    if (rc) return rc;
  }
  return RSPL_OK;
}

extern "C" int rspl_map_add_point_observations(rspl_map* m, int frame_id, int n, const int32_t* point_ids,
                                               const int32_t* keypoints) {
  RSPL_CHECK_ARG(m && (n == 0 || (point_ids && keypoints)), "rspl_map_add_point_observations: NULL argument");
  for (int i = 0; i < n; i++) {
    const int rc = rspl_map_add_point_observation(m, point_ids[i], frame_id, keypoints[i]);
    if (rc) return rc;
  }
  return RSPL_OK;
}

extern "C" int rspl_map_update_connections(rspl_map* m, int frame_id) {
  RSPL_CHECK_ARG(m && m->frame(frame_id), "rspl_map_update_connections: unknown frame");
  m->update_connection(*m->frame(frame_id));
  return RSPL_OK;
}

extern "C" int rspl_map_local_optimization(rspl_map* m, int frame_id, rspl_ba* ba, rspl_map_report* rep) {
  RSPL_CHECK_ARG(m && ba, "rspl_map_local_optimization: NULL argument");
  return m->local_map_optimization(frame_id, ba, rep);
}

extern "C" int rspl_map_finish(rspl_map* m, const rspl_ba_result* result, rspl_map_report* rep) {
  RSPL_CHECK_ARG(m && result && result->pose_q && result->pose_p, "rspl_map_finish: NULL argument");
  RSPL_CHECK_ARG((m->point_ids.empty() || result->points) && (m->line_ids.empty() || result->lines),
                 "rspl_map_finish: NULL landmark result");
  return m->finish(*result, rep);
}

extern "C" int rspl_map_assemble(rspl_map* m, int frame_id, rspl_map_report* rep) {
  RSPL_CHECK_ARG(m, "rspl_map_assemble: NULL map");
  return m->local_map_optimization(frame_id, nullptr, rep);
}

extern "C" int rspl_map_last_problem(const rspl_map* m, int32_t* pose_ids, uint8_t* pose_fixed, int32_t* point_ids,
                                     int32_t* line_ids, int32_t* const* c_pose, int32_t* const* c_lm,
                                     double* const* c_obs) {
  RSPL_CHECK_ARG(m, "rspl_map_last_problem: NULL map");
  if (pose_ids) std::copy(m->pose_ids.begin(), m->pose_ids.end(), pose_ids);
  if (pose_fixed) std::copy(m->pose_fixed.begin(), m->pose_fixed.end(), pose_fixed);
  if (point_ids) std::copy(m->point_ids.begin(), m->point_ids.end(), point_ids);
  if (line_ids) std::copy(m->line_ids.begin(), m->line_ids.end(), line_ids);
  for (int t = 0; t < 4; t++) {
    if (c_pose && c_pose[t]) std::copy(m->c_pose[t].begin(), m->c_pose[t].end(), c_pose[t]);
    if (c_lm && c_lm[t]) std::copy(m->c_lm[t].begin(), m->c_lm[t].end(), c_lm[t]);
    if (c_obs && c_obs[t]) std::copy(m->c_obs[t].begin(), m->c_obs[t].end(), c_obs[t]);
  }
  return RSPL_OK;
}

extern "C" int rspl_map_get_keyframe(const rspl_map* m, int frame_id, double* Twc, int* n_connections) {
  RSPL_CHECK_ARG(m, "rspl_map_get_keyframe: NULL map");
  auto it = m->kf.find(frame_id);
  RSPL_CHECK_ARG(it != m->kf.end(), "rspl_map_get_keyframe: unknown frame %d", frame_id);
  if (Twc) memcpy(Twc, it->second.Twc, sizeof(double) * 16);
  if (n_connections) *n_connections = (int)it->second.oconn.size();
  return RSPL_OK;
}

extern "C" int rspl_map_get_connections(const rspl_map* m, int frame_id, int32_t* ids, int32_t* weights, int cap,
                                        int* n) {
  RSPL_CHECK_ARG(m && n, "rspl_map_get_connections: NULL argument");
  auto it = m->kf.find(frame_id);
  RSPL_CHECK_ARG(it != m->kf.end(), "rspl_map_get_connections: unknown frame %d", frame_id);
  const auto& oc = it->second.oconn;
  *n = (int)oc.size();
  RSPL_CHECK_ARG(cap >= *n || (!ids && !weights), "rspl_map_get_connections: capacity %d < %d", cap, *n);
  int i = 0;
  for (auto& wc : oc) {  // GetOrderedConnections(-1): ascending weight
    if (ids) ids[i] = wc.second;
    if (weights) weights[i] = wc.first;
    i++;
  }
  return RSPL_OK;
}

extern "C" int rspl_map_get_mappoint(const rspl_map* m, int id, double* p, int* type, int* n_observers,
                                     int32_t* frames, int32_t* kps, int cap) {
  RSPL_CHECK_ARG(m, "rspl_map_get_mappoint: NULL map");
  auto it = m->mp.find(id);
  RSPL_CHECK_ARG(it != m->mp.end(), "rspl_map_get_mappoint: unknown map point %d", id);
  const MPoint& q = it->second;
  if (p) memcpy(p, q.p, sizeof(q.p));
  if (type) *type = q.type;
  if (n_observers) *n_observers = (int)q.obs.size();
  int i = 0;
  for (auto& kv : q.obs) {
    if (i >= cap) break;
    if (frames) frames[i] = kv.first;
    if (kps) kps[i] = kv.second;
    i++;
  }
  return RSPL_OK;
}

extern "C" int rspl_map_get_mapline(const rspl_map* m, int id, double* line3d, int* type, int* n_observers,
                                    double* endpoints, int* endpoints_valid) {
  RSPL_CHECK_ARG(m, "rspl_map_get_mapline: NULL map");
  auto it = m->ml.find(id);
  RSPL_CHECK_ARG(it != m->ml.end(), "rspl_map_get_mapline: unknown map line %d", id);
  const MLine& l = it->second;
  if (line3d) memcpy(line3d, l.L, sizeof(l.L));
  if (type) *type = l.type;
  if (n_observers) *n_observers = (int)l.obs.size();
  if (endpoints) memcpy(endpoints, l.ep, sizeof(l.ep));
  if (endpoints_valid) *endpoints_valid = l.ep_valid;
  return RSPL_OK;
}

extern "C" int rspl_map_get_frame_slots(const rspl_map* m, int frame_id, int32_t* mappoints, int32_t* maplines) {
  RSPL_CHECK_ARG(m, "rspl_map_get_frame_slots: NULL map");
  auto it = m->kf.find(frame_id);
  RSPL_CHECK_ARG(it != m->kf.end(), "rspl_map_get_frame_slots: unknown frame %d", frame_id);
  if (mappoints) std::copy(it->second.mpt.begin(), it->second.mpt.end(), mappoints);
  if (maplines) std::copy(it->second.mpl.begin(), it->second.mpl.end(), maplines);
  return RSPL_OK;
}

// Map::SaveKeyframeTrajectory (map.cc:1007-1024): "timestamp tx ty tz qx qy qz qw" per keyframe in
// insertion order, std::fixed with setprecision(9)
extern "C" int rspl_map_save_trajectory(const rspl_map* m, const char* path) {
  RSPL_CHECK_ARG(m && path, "rspl_map_save_trajectory: NULL argument");
  FILE* f = fopen(path, "w");
  if (!f) {
    set_error("rspl_map_save_trajectory: cannot open %s", path);
    return RSPL_E_ARG;
  }
  for (int id : m->kf_ids) {
    const MFrame& k = m->kf.at(id);
    double q[4];
    R_to_q(k.Twc, 4, q);
    fprintf(f, "%.9f %.9f %.9f %.9f %.9f %.9f %.9f %.9f\n", k.ts, k.Twc[3], k.Twc[7], k.Twc[11], q[0], q[1], q[2], q[3]);
  }
  fclose(f);
  return RSPL_OK;
}
