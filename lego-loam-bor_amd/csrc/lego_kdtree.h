// lego_kdtree.h — nanoflann 1.3.0's kd-tree on gfx950, for the rare searches with an exact distance tie.
//
// The 1-NN of FeatureAssociation (nanoflann_pcl.h:141-152) and the kNN-5 of MapOptimization
// (mapOptmization.cpp:1036, :1144) run as exact uniform-grid searches, which find the right distances
// and flag a query when several points share one of them.  Which of the tied points kdtree->
// nearestKSearch returns (and in what order) is nanoflann's first visited (strict < in searchLevel and
// KNNResultSet::addPoint), a function of its tree.  So when a search has tied queries, one wave builds
// the tree of the searched cloud exactly as nanoflann 1.3.0 does (buildIndex / divideTree /
// middleSplit_ / planeSplit, nanoflann.hpp:857-1003, 1190-1202, 1316-1337; leaf_max_size 10;
// oracle/nanoflann_restated.h is the host statement) and re-runs nanoflann's searchLevel (:1346-1409)
// for those queries.  planeSplit's two Hoare passes are rank pairings: the k-th left stop (from the
// left) swaps with the k-th right stop (from the right) while it lies left of it, so each pass is two
// stop lists and one parallel swap.
#pragma once
#include <float.h>

#include "lego_device.h"

namespace lgkd {

#define KD_LEAF 10

struct KdView {
  const float4* pts;  // the searched cloud, in its own order
  KdNode* node;       // [2 * cap]
  int* vind;          // [cap]
  int* tmp;           // [2 * cap]: left stops, right stops
  float* frames;      // [10 * cap]: the build's stack, then the searches' stacks
  int vh;             // cap: points the buffers hold
};

LG_DEVICE int kd_lane() { return threadIdx.x & 63; }
LG_DEVICE int kd_popc_below(unsigned long long m) { return __popcll(m & ((1ull << kd_lane()) - 1ull)); }
LG_DEVICE float kd_wmin(float v) {
  for (int o = 32; o > 0; o >>= 1) {
    const float u = __shfl_xor(v, o);
    v = u < v ? u : v;
  }
  return v;
}
LG_DEVICE float kd_wmax(float v) {
  for (int o = 32; o > 0; o >>= 1) {
    const float u = __shfl_xor(v, o);
    v = u > v ? u : v;
  }
  return v;
}

LG_DEVICE float kd_get(const float4* pts, int i, int d) {
  const float4 p = pts[i];
  return d == 0 ? p.x : (d == 1 ? p.y : p.z);
}
LG_DEVICE void kd_sync() {  // this wave's global stores before its other lanes' loads of them
  __threadfence_block();
  __builtin_amdgcn_wave_barrier();
}

// computeMinMax (:836-848) of all three dimensions over ind[0, count) (order-independent)
LG_DEVICE void kd_minmax(const float4* pts, const int* ind, int count, float* mn, float* mx) {
  // (one load in flight a lane: a rare path, kept lean in registers for the kernels that call it)
  float a0 = FLT_MAX, a1 = FLT_MAX, a2 = FLT_MAX, b0 = -FLT_MAX, b1 = -FLT_MAX, b2 = -FLT_MAX;
  for (int t = kd_lane(); t < count; t += 64) {
    const float4 p = pts[ind[t]];
    a0 = fminf(a0, p.x); a1 = fminf(a1, p.y); a2 = fminf(a2, p.z);
    b0 = fmaxf(b0, p.x); b1 = fmaxf(b1, p.y); b2 = fmaxf(b2, p.z);
  }
  mn[0] = kd_wmin(a0); mn[1] = kd_wmin(a1); mn[2] = kd_wmin(a2);
  mx[0] = kd_wmax(b0); mx[1] = kd_wmax(b1); mx[2] = kd_wmax(b2);
}

// One planeSplit pass over ind[b, count) (:967-1003): mode 0 moves the keys < cv to the front (left
// stops: !(key < cv), right stops: key < cv), mode 1 the keys <= cv.  Returns b + the number of
// moved-to-front keys (lim1 / lim2).
LG_DEVICE int kd_pass(const float4* pts, int* ind, int b, int count, int d, float cv, int mode, int* tL, int* tR) {
  const int lane = kd_lane();
  int nL = 0, nR = 0;
  // each position is a left stop (!front) or a right stop (front)
  for (int t0 = b; t0 < count; t0 += 64) {  // left stops ascending
    const int i = t0 + lane;
    const float k = kd_get(pts, ind[min(i, count - 1)], d);
    const bool front = mode == 0 ? k < cv : k <= cv;
    const bool ls = i < count && !front;
    const unsigned long long m = __ballot(ls);
    if (ls) tL[nL + kd_popc_below(m)] = i;
    nL += __popcll(m);
  }
  for (int t0 = count - 1; t0 >= b; t0 -= 64) {  // right stops descending
    const int i = t0 - lane;
    const float k = kd_get(pts, ind[max(i, b)], d);
    const bool front = mode == 0 ? k < cv : k <= cv;
    const bool rs = i >= b && front;
    const unsigned long long m = __ballot(rs);
    if (rs) tR[nR + kd_popc_below(m)] = i;
    nR += __popcll(m);
  }
  kd_sync();
  const int K = min(nL, nR);
  for (int k0 = 0; k0 < K; k0 += 64) {  // the valid pairs (L_k < R_k) are a prefix; swaps are disjoint
    const int k = k0 + lane;
    if (k < K) {
      const int l = tL[k], r = tR[k];
      if (l < r) {
        const int x = ind[l];
        ind[l] = ind[r];
        ind[r] = x;
      }
    }
  }
  kd_sync();
  return b + nR;
}

// buildIndex by one wave (DFS over an explicit stack of {node, left, right, bbox} frames); returns the
// node count (root 0) and the root bbox in box[0..5] (lo xyz, hi xyz); -1 when the stack would overflow
// the frames buffer (a tree deeper than 10 * cap / 9 levels: never for real clouds).
LG_DEVICE int kd_build(const KdView& K, int n, float* box) {
  const int lane = kd_lane();
  for (int i = lane; i < n; i += 64) K.vind[i] = i;
  kd_sync();
  if (n <= 0) return 0;
  float lo[3], hi[3];
  kd_minmax(K.pts, K.vind, n, lo, hi);  // computeBoundingBox (:1316-1337)
  if (lane < 3) { box[lane] = lo[lane]; box[3 + lane] = hi[lane]; }
  float* fr = K.frames;  // frame: node, left, right, lo[3], hi[3] (9 words, ints as bits)
  const int max_frames = (10 * K.vh) / 9;
  auto push = [&](int sp, int nd, int l, int r, const float* a, const float* z) {  // lanes 0..8, a field each
    const float w = lane == 0 ? __int_as_float(nd) : lane == 1 ? __int_as_float(l) : lane == 2 ? __int_as_float(r)
                  : lane == 3 ? a[0] : lane == 4 ? a[1] : lane == 5 ? a[2] : lane == 6 ? z[0] : lane == 7 ? z[1] : z[2];
    if (lane < 9) fr[9 * sp + lane] = w;
  };
  push(0, 0, 0, n, lo, hi);
  kd_sync();
  int sp = 1, nodes = 1;
  const float EPS = 0.00001f;
  while (sp > 0) {
    --sp;
    const int nd = __float_as_int(fr[9 * sp]), left = __float_as_int(fr[9 * sp + 1]), right = __float_as_int(fr[9 * sp + 2]);
    float blo[3] = {fr[9 * sp + 3], fr[9 * sp + 4], fr[9 * sp + 5]}, bhi[3] = {fr[9 * sp + 6], fr[9 * sp + 7], fr[9 * sp + 8]};
    KdNode node;
    node.left = left;
    node.right = right;
    node.c1 = node.c2 = -1;
    node.divfeat = 0;
    node.divlow = node.divhigh = 0.f;
    node.pad = 0;
    const int count = right - left;
    if (count > KD_LEAF) {
      if (sp + 2 > max_frames) return -1;
      int* ind = K.vind + left;
      float mn[3], mx[3];
      kd_minmax(K.pts, ind, count, mn, mx);
      // middleSplit_ (:909-958)
      float max_span = bhi[0] - blo[0];
      for (int d = 1; d < 3; ++d) {
        const float span = bhi[d] - blo[d];
        if (span > max_span) max_span = span;
      }
      float max_spread = -1;
      int cf = 0;
      for (int d = 0; d < 3; ++d) {
        const float span = bhi[d] - blo[d];
        if (span > (1 - EPS) * max_span) {
          const float spread = mx[d] - mn[d];
          if (spread > max_spread) { cf = d; max_spread = spread; }
        }
      }
      const float split_val = (blo[cf] + bhi[cf]) / 2;
      const float cv = split_val < mn[cf] ? mn[cf] : (split_val > mx[cf] ? mx[cf] : split_val);
      const int lim1 = kd_pass(K.pts, ind, 0, count, cf, cv, 0, K.tmp, K.tmp + K.vh);
      const int lim2 = kd_pass(K.pts, ind, lim1, count, cf, cv, 1, K.tmp, K.tmp + K.vh);
      const int idx = lim1 > count / 2 ? lim1 : (lim2 < count / 2 ? lim2 : count / 2);
      // the children's tight bounds along cf (divideTree's left_bbox.high / right_bbox.low, :898-899)
      float dl = -FLT_MAX, dh = FLT_MAX;
      for (int t = lane; t < count; t += 64) {
        const float k = kd_get(K.pts, ind[t], cf);
        if (t < idx) dl = fmaxf(dl, k);
        else dh = fminf(dh, k);
      }
      node.divfeat = cf;
      node.divlow = kd_wmax(dl);
      node.divhigh = kd_wmin(dh);
      node.c1 = nodes;
      node.c2 = nodes + 1;
      nodes += 2;
      float lhi[3] = {bhi[0], bhi[1], bhi[2]}, rlo[3] = {blo[0], blo[1], blo[2]};
      lhi[cf] = cv;
      rlo[cf] = cv;
      push(sp, node.c2, left + idx, right, rlo, bhi);     // child2 below child1: child1 is built first
      push(sp + 1, node.c1, left, left + idx, blo, lhi);
      sp += 2;
    }
    if (lane == 0) K.node[nd] = node;
    kd_sync();
  }
  return nodes;
}

// nanoflann's findNeighbors / searchLevel with a KNNResultSet<float, int>(KN) (one lane; explicit stack
// of {node, mindistsq, dists[3]} frames, the other child pushed when descending and tested against the
// then-current worst distance when popped, as the recursion tests it after the best child's subtree).
// idx / dst: the KN nearest, nearest first (dst[KN-1] = FLT_MAX while fewer were found); returns the
// count found.  ovf: the stack of cap frames overflowed (the result is then not nanoflann's).
template <int KN>
LG_DEVICE int kd_knn(const KdView& K, const float* box, float4 q, float* stk, int cap, int* idx, float* dst, bool& ovf) {
  const float qv[3] = {q.x, q.y, q.z};
  int cnt = 0;  // KNNResultSet::init (:157-163)
#pragma unroll
  for (int j = 0; j < KN; ++j) { dst[j] = FLT_MAX; idx[j] = -1; }
  float dists[3] = {0.f, 0.f, 0.f};
  float distsq = 0.f;  // computeInitialDistances (:1005-1022)
  for (int d = 0; d < 3; ++d) {
    if (qv[d] < box[d]) { dists[d] = (qv[d] - box[d]) * (qv[d] - box[d]); distsq += dists[d]; }
    if (qv[d] > box[3 + d]) { dists[d] = (qv[d] - box[3 + d]) * (qv[d] - box[3 + d]); distsq += dists[d]; }
  }
  int sp = 0;
  int nd = 0;
  bool popped = false;
  float mind = distsq;
  while (true) {
    if (popped) {
      if (sp == 0) break;
      --sp;
      nd = __float_as_int(stk[5 * sp]);
      mind = stk[5 * sp + 1];
      dists[0] = stk[5 * sp + 2]; dists[1] = stk[5 * sp + 3]; dists[2] = stk[5 * sp + 4];
      if (!(mind * 1.0f <= dst[KN - 1])) continue;  // epsError = 1 + eps, eps 0
    }
    popped = true;
    KdNode n = K.node[nd];
    while (n.c1 >= 0) {
      const int dv = n.divfeat;
      const float val = qv[dv];
      const float diff1 = val - n.divlow, diff2 = val - n.divhigh;
      int bestc, other;
      float cut;
      if ((diff1 + diff2) < 0) { bestc = n.c1; other = n.c2; cut = (val - n.divhigh) * (val - n.divhigh); }
      else { bestc = n.c2; other = n.c1; cut = (val - n.divlow) * (val - n.divlow); }
      if (sp < cap) {
        stk[5 * sp] = __int_as_float(other);
        stk[5 * sp + 1] = mind + cut - dists[dv];
        for (int d = 0; d < 3; ++d) stk[5 * sp + 2 + d] = d == dv ? cut : dists[d];
        ++sp;
      } else {
        ovf = true;
      }
      n = K.node[bestc];
    }
    const float worst_entry = dst[KN - 1];  // searchLevel's leaf: worstDist() once, then addPoint
    for (int i = n.left; i < n.right; ++i) {
      const int index = K.vind[i];
      const float4 p = K.pts[index];
      float dist = 0.f;  // L2_Simple_Adaptor::evalMetric (:432-440)
      float df = qv[0] - p.x;
      dist += df * df;
      df = qv[1] - p.y;
      dist += df * df;
      df = qv[2] - p.z;
      dist += df * df;
      if (dist < worst_entry) {
        // KNNResultSet::addPoint (:175-202): after the entries <= dist, the later ones shifted right
        int pos = cnt;
#pragma unroll
        for (int j = KN - 1; j >= 0; --j)
          if (j < cnt && dst[j] > dist) pos = j;
#pragma unroll
        for (int j = KN - 1; j >= 1; --j)
          if (j > pos && j <= cnt) { dst[j] = dst[j - 1]; idx[j] = idx[j - 1]; }
#pragma unroll
        for (int j = 0; j < KN; ++j)
          if (j == pos) { dst[j] = dist; idx[j] = index; }
        if (cnt < KN) ++cnt;
      }
    }
  }
  return cnt;
}

}  // namespace lgkd
