// nanoflann_restated.h — TEST INFRASTRUCTURE (oracle only): the reference's kd-tree k-NN, restated.
//
// LeGO-LOAM-BOR searches its Last clouds with nanoflann_pcl.h's KdTreeFLANN<PointXYZI>
// (nanoflann_pcl.h:100-152): nanoflann 1.3.0's KDTreeSingleIndexAdaptor<SO3_Adaptor<float, Adaptor>,
// Adaptor, 3, int> (SO3_Adaptor is L2_Simple_Adaptor: squared L2 in float), default leaf_max_size 10,
// the bounding box computed by nanoflann, queried through KNNResultSet<float, int>(k) with default
// SearchParams (eps 0).  Which of several points at exactly the same distance is returned depends on
// the tree (the first one visited wins: strict < in searchLevel and KNNResultSet::addPoint), so the
// parity oracle restates the tree itself, operation for operation:
//   buildIndex / computeBoundingBox   nanoflann.hpp:1190-1202, 1316-1337
//   divideTree                        :857-907
//   middleSplit_ / computeMinMax      :909-958, 836-848
//   planeSplit                        :967-1003
//   findNeighbors / computeInitialDistances / searchLevel   :1222-1240, 1005-1022, 1346-1409
//   KNNResultSet::init / addPoint     :157-202
// Pinned against the reference's own nanoflann.hpp (oracle/_ref/nanoflann_pin, built from
// /root/reference) on tie-heavy clouds by tests/test_oracle_cpu.py::test_nanoflann_pin.
#pragma once
#include <cstdint>
#include <limits>
#include <vector>

#if defined(__GNUC__) && !defined(__clang__)
#pragma GCC diagnostic push
#pragma GCC diagnostic ignored "-Warray-bounds"  // add_point's shifts are guarded by the capacity
#endif

namespace nfr {

template <class PointT>  // any type with float x, y, z
class KdTree {
 public:
  // buildIndex (:1190-1202) over pts[0, n)
  void build(const PointT* pts, int n) {
    pts_ = pts;
    n_ = n;
    vind_.resize(n);
    for (int i = 0; i < n; ++i) vind_[i] = i;
    nodes_.clear();
    root_ = -1;
    if (n == 0) return;
    for (int d = 0; d < 3; ++d) lo_[d] = hi_[d] = get(0, d);  // computeBoundingBox (:1316-1337)
    for (int k = 1; k < n; ++k)
      for (int d = 0; d < 3; ++d) {
        if (get(k, d) < lo_[d]) lo_[d] = get(k, d);
        if (get(k, d) > hi_[d]) hi_[d] = get(k, d);
      }
    float lo[3] = {lo_[0], lo_[1], lo_[2]}, hi[3] = {hi_[0], hi_[1], hi_[2]};
    root_ = divide(0, n, lo, hi);
  }

  // nearestKSearch(q, k) (nanoflann_pcl.h:141-152): indices / squared distances nearest first, count
  // returned.  *ties (optional): for k = 1, how many other visited points had exactly the final
  // distance (diagnostic; not part of nanoflann).
  int knn(const float q[3], int k, int* idx, float* dist, int* ties = nullptr) const {
    // KNNResultSet::init (:157-163)
    cap_ = k;
    cnt_ = 0;
    idx_ = idx;
    dst_ = dist;
    dst_[k - 1] = std::numeric_limits<float>::max();
    tie_best_ = std::numeric_limits<float>::max();
    tie_n_ = 0;
    if (n_ == 0 || root_ < 0) return 0;  // findNeighbors: size 0 -> false
    float dists[3] = {0.f, 0.f, 0.f};
    float distsq = 0.f;  // computeInitialDistances (:1005-1022)
    for (int d = 0; d < 3; ++d) {
      if (q[d] < lo_[d]) {
        dists[d] = (q[d] - lo_[d]) * (q[d] - lo_[d]);
        distsq += dists[d];
      }
      if (q[d] > hi_[d]) {
        dists[d] = (q[d] - hi_[d]) * (q[d] - hi_[d]);
        distsq += dists[d];
      }
    }
    search(q, root_, distsq, dists);
    if (ties) *ties = tie_n_;
    return cnt_;
  }

  const std::vector<int>& vind() const { return vind_; }

 private:
  struct Node {
    int child1 = -1, child2 = -1;  // -1 / -1: leaf
    int left = 0, right = 0;       // leaf: vind range
    int divfeat = 0;
    float divlow = 0.f, divhigh = 0.f;
  };
  const PointT* pts_ = nullptr;
  int n_ = 0;
  std::vector<int> vind_;
  std::vector<Node> nodes_;
  int root_ = -1;
  float lo_[3], hi_[3];  // root_bbox
  static const int kLeaf = 10;  // KDTreeSingleIndexAdaptorParams default leaf_max_size (:547)
  // KNNResultSet state (mutable: a query is const in nanoflann too)
  mutable int cap_ = 1, cnt_ = 0;
  mutable int* idx_ = nullptr;
  mutable float* dst_ = nullptr;
  mutable float tie_best_;
  mutable int tie_n_;

  float get(int i, int d) const { return d == 0 ? pts_[i].x : (d == 1 ? pts_[i].y : pts_[i].z); }

  // divideTree (:857-907); lo / hi: the node's bbox, updated to the tight bbox of its points
  int divide(int left, int right, float* lo, float* hi) {
    const int me = (int)nodes_.size();
    nodes_.push_back(Node());
    if (right - left <= kLeaf) {
      nodes_[me].left = left;
      nodes_[me].right = right;
      for (int d = 0; d < 3; ++d) lo[d] = hi[d] = get(vind_[left], d);
      for (int k = left + 1; k < right; ++k)
        for (int d = 0; d < 3; ++d) {
          if (lo[d] > get(vind_[k], d)) lo[d] = get(vind_[k], d);
          if (hi[d] < get(vind_[k], d)) hi[d] = get(vind_[k], d);
        }
      return me;
    }
    int idx, cutfeat;
    float cutval;
    middle_split(&vind_[left], right - left, idx, cutfeat, cutval, lo, hi);
    nodes_[me].divfeat = cutfeat;
    float llo[3] = {lo[0], lo[1], lo[2]}, lhi[3] = {hi[0], hi[1], hi[2]};
    lhi[cutfeat] = cutval;
    const int c1 = divide(left, left + idx, llo, lhi);
    float rlo[3] = {lo[0], lo[1], lo[2]}, rhi[3] = {hi[0], hi[1], hi[2]};
    rlo[cutfeat] = cutval;
    const int c2 = divide(left + idx, right, rlo, rhi);
    nodes_[me].child1 = c1;
    nodes_[me].child2 = c2;
    nodes_[me].divlow = lhi[cutfeat];
    nodes_[me].divhigh = rlo[cutfeat];
    for (int d = 0; d < 3; ++d) {
      lo[d] = llo[d] < rlo[d] ? llo[d] : rlo[d];  // std::min(left.low, right.low)
      hi[d] = lhi[d] < rhi[d] ? rhi[d] : lhi[d];  // std::max(left.high, right.high)
    }
    return me;
  }

  void min_max(const int* ind, int count, int d, float& mn, float& mx) const {  // computeMinMax (:836-848)
    mn = get(ind[0], d);
    mx = get(ind[0], d);
    for (int i = 1; i < count; ++i) {
      const float v = get(ind[i], d);
      if (v < mn) mn = v;
      if (v > mx) mx = v;
    }
  }

  void middle_split(int* ind, int count, int& index, int& cutfeat, float& cutval, const float* lo, const float* hi) {
    const float EPS = 0.00001f;  // (:911)
    float max_span = hi[0] - lo[0];
    for (int d = 1; d < 3; ++d) {
      const float span = hi[d] - lo[d];
      if (span > max_span) max_span = span;
    }
    float max_spread = -1;
    cutfeat = 0;
    for (int d = 0; d < 3; ++d) {
      const float span = hi[d] - lo[d];
      if (span > (1 - EPS) * max_span) {
        float mn, mx;
        min_max(ind, count, d, mn, mx);
        const float spread = mx - mn;
        if (spread > max_spread) {
          cutfeat = d;
          max_spread = spread;
        }
      }
    }
    const float split_val = (lo[cutfeat] + hi[cutfeat]) / 2;
    float mn, mx;
    min_max(ind, count, cutfeat, mn, mx);
    if (split_val < mn) cutval = mn;
    else if (split_val > mx) cutval = mx;
    else cutval = split_val;
    int lim1, lim2;
    plane_split(ind, count, cutfeat, cutval, lim1, lim2);
    if (lim1 > count / 2) index = lim1;
    else if (lim2 < count / 2) index = lim2;
    else index = count / 2;
  }

  void plane_split(int* ind, int count, int cutfeat, float cutval, int& lim1, int& lim2) {  // (:967-1003)
    int left = 0, right = count - 1;
    for (;;) {
      while (left <= right && get(ind[left], cutfeat) < cutval) ++left;
      while (right && left <= right && get(ind[right], cutfeat) >= cutval) --right;
      if (left > right || !right) break;
      const int t = ind[left]; ind[left] = ind[right]; ind[right] = t;
      ++left;
      --right;
    }
    lim1 = left;
    right = count - 1;
    for (;;) {
      while (left <= right && get(ind[left], cutfeat) <= cutval) ++left;
      while (right && left <= right && get(ind[right], cutfeat) > cutval) --right;
      if (left > right || !right) break;
      const int t = ind[left]; ind[left] = ind[right]; ind[right] = t;
      ++left;
      --right;
    }
    lim2 = left;
  }

  // KNNResultSet::addPoint (:175-202), NANOFLANN_FIRST_MATCH undefined
  void add_point(float dist, int index) const {
    int i;
    for (i = cnt_; i > 0; --i) {
      if (dst_[i - 1] > dist) {
        if (i < cap_) {
          dst_[i] = dst_[i - 1];
          idx_[i] = idx_[i - 1];
        }
      } else {
        break;
      }
    }
    if (i < cap_) {
      dst_[i] = dist;
      idx_[i] = index;
    }
    if (cnt_ < cap_) cnt_++;
  }

  void search(const float* q, int node, float mindistsq, float* dists) const {  // searchLevel (:1346-1409)
    const Node& nd = nodes_[node];
    if (nd.child1 < 0 && nd.child2 < 0) {
      const float worst_dist = dst_[cap_ - 1];
      for (int i = nd.left; i < nd.right; ++i) {
        const int index = vind_[i];
        float dist = 0.f;  // L2_Simple_Adaptor::evalMetric (:432-440)
        for (int d = 0; d < 3; ++d) {
          const float diff = q[d] - get(index, d);
          dist += diff * diff;
        }
        if (dist < tie_best_) { tie_best_ = dist; tie_n_ = 0; }
        else if (dist == tie_best_) ++tie_n_;
        if (dist < worst_dist) add_point(dist, vind_[i]);
      }
      return;
    }
    const int idx = nd.divfeat;
    const float val = q[idx];
    const float diff1 = val - nd.divlow;
    const float diff2 = val - nd.divhigh;
    int best, other;
    float cut_dist;
    if ((diff1 + diff2) < 0) {
      best = nd.child1;
      other = nd.child2;
      cut_dist = (val - nd.divhigh) * (val - nd.divhigh);
    } else {
      best = nd.child2;
      other = nd.child1;
      cut_dist = (val - nd.divlow) * (val - nd.divlow);
    }
    search(q, best, mindistsq, dists);
    const float dst = dists[idx];
    mindistsq = mindistsq + cut_dist - dst;
    dists[idx] = cut_dist;
    if (mindistsq * 1.0f <= dst_[cap_ - 1]) search(q, other, mindistsq, dists);  // epsError = 1 + eps, eps 0
    dists[idx] = dst;
  }
};

}  // namespace nfr

#if defined(__GNUC__) && !defined(__clang__)
#pragma GCC diagnostic pop
#endif
