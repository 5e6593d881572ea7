// ref_nanoflann_pin.cpp — TEST INFRASTRUCTURE: pins the oracle's brute-force 1-NN against the
// reference's own vendored nanoflann 1.3.0, compiled from where it lies under /root/reference
// (oracle/Makefile target `ref`, output in oracle/_ref/, never committed, never shipped).
//
// Builds the index exactly as nanoflann_pcl.h:100-138 does (KDTreeSingleIndexAdaptor<
// SO3_Adaptor<float, Adaptor>, Adaptor, 3, int>, default leaf_max_size 10, bbox computed by
// nanoflann) and queries it as nearestKSearch(k) does (:141-152: KNNResultSet<float,int>(k), default
// SearchParams); k = argv[1], 1 if absent (FeatureAssociation's 1-NN; MapOptimization uses k = 5).
//
// stdin:  int32 n_cloud, n_cloud x float32[3], int32 n_query, n_query x float32[3]
// stdout: n_query x k x (int32 index, float32 sq_dist), nearest first
#include <cstdint>
#include <cstdio>
#include <vector>

#include "nanoflann.hpp"

struct Adaptor {
  std::vector<float> xyz;
  inline size_t kdtree_get_point_count() const { return xyz.size() / 3; }
  inline float kdtree_get_pt(const size_t idx, int dim) const { return xyz[idx * 3 + dim]; }
  template <class BBOX>
  bool kdtree_get_bbox(BBOX&) const { return false; }
};

typedef nanoflann::KDTreeSingleIndexAdaptor<nanoflann::SO3_Adaptor<float, Adaptor>, Adaptor, 3, int> Tree;

static bool rd(void* p, size_t n) { return fread(p, 1, n, stdin) == n; }

#include <cstdlib>

int main(int argc, char** argv) {
  const int k = argc > 1 ? std::atoi(argv[1]) : 1;
  if (k < 1) return 1;
  int32_t n = 0, m = 0;
  Adaptor a;
  if (!rd(&n, 4)) return 1;
  a.xyz.resize((size_t)n * 3);
  if (n && !rd(a.xyz.data(), (size_t)n * 12)) return 1;
  if (!rd(&m, 4)) return 1;
  std::vector<float> q((size_t)m * 3);
  if (m && !rd(q.data(), (size_t)m * 12)) return 1;
  Tree tree(3, a);
  tree.buildIndex();
  for (int i = 0; i < m; ++i) {
    std::vector<int> idx(k, -1);
    std::vector<float> d(k, 0.f);
    nanoflann::KNNResultSet<float, int> rs(k);
    rs.init(idx.data(), d.data());
    tree.findNeighbors(rs, &q[(size_t)i * 3], nanoflann::SearchParams());
    for (int j = 0; j < k; ++j) {
      int32_t oi = idx[j];
      fwrite(&oi, 4, 1, stdout);
      fwrite(&d[j], 4, 1, stdout);
    }
  }
  return 0;
}
