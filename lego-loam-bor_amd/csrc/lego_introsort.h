// lego_introsort.h — libstdc++ std::sort, restated for one device lane (or the host).
//
// The reference sorts with std::sort twice on the hot path, and std::sort is not stable:
//   * the per-segment smoothness sort, featureAssociation.cpp:285-286 (by_value, utility.h:58-62);
//   * PCL VoxelGrid's (voxel index, point index) sort by voxel index only, whose permutation sets
//     the float summation order of each centroid.
// Whenever keys tie, only the exact introsort permutation reproduces the reference.  This is the
// libstdc++ algorithm (bits/stl_algo.h / stl_heap.h, unchanged from GCC 5 to GCC 11):
// __introsort_loop with _S_threshold 16 and depth limit 2*floor(log2 n), median-of-3 pivot moved to
// first (__move_median_to_first(first, first+1, mid, last-1)), __unguarded_partition, heap-sort
// fallback (__partial_sort = __make_heap + __sort_heap), then __final_insertion_sort.
// tests/test_introsort.py checks the permutation against the host's std::sort on tie-heavy inputs.
#pragma once

#ifdef __HIPCC__
#define LG_HD __host__ __device__ __forceinline__
#else
#define LG_HD inline
#endif

namespace lg {

template <typename K, typename V = int>
struct SortView {
  K* key;
  V* val;
  LG_HD bool lt(int a, int b) const { return key[a] < key[b]; }
  LG_HD void swap(int a, int b) const {
    K tk = key[a]; key[a] = key[b]; key[b] = tk;
    V tv = val[a]; val[a] = val[b]; val[b] = tv;
  }
  LG_HD void move(int dst, int src) const { key[dst] = key[src]; val[dst] = val[src]; }
};

LG_HD int floor_log2(int n) {
  int r = 0;
  while (n > 1) { n >>= 1; ++r; }
  return r;
}

template <typename K, typename V>
LG_HD void adjust_heap(const SortView<K, V>& a, int first, int hole, int len, K vk, V vv) {
  const int top = hole;
  int second = hole;
  while (second < (len - 1) / 2) {
    second = 2 * (second + 1);
    if (a.lt(first + second, first + (second - 1))) second--;
    a.move(first + hole, first + second);
    hole = second;
  }
  if ((len & 1) == 0 && second == (len - 2) / 2) {
    second = 2 * (second + 1);
    a.move(first + hole, first + (second - 1));
    hole = second - 1;
  }
  // __push_heap
  int parent = (hole - 1) / 2;
  while (hole > top && a.key[first + parent] < vk) {
    a.move(first + hole, first + parent);
    hole = parent;
    parent = (hole - 1) / 2;
  }
  a.key[first + hole] = vk;
  a.val[first + hole] = vv;
}

template <typename K, typename V>
LG_HD void heap_sort(const SortView<K, V>& a, int first, int last) {  // __partial_sort(first, last, last)
  const int len = last - first;
  if (len >= 2) {  // __make_heap
    int parent = (len - 2) / 2;
    while (true) {
      K vk = a.key[first + parent];
      V vv = a.val[first + parent];
      adjust_heap(a, first, parent, len, vk, vv);
      if (parent == 0) break;
      parent--;
    }
  }
  while (last - first > 1) {  // __sort_heap / __pop_heap
    --last;
    K vk = a.key[last];
    V vv = a.val[last];
    a.move(last, first);
    adjust_heap(a, first, 0, last - first, vk, vv);
  }
}

template <typename K, typename V>
LG_HD void move_median_to_first(const SortView<K, V>& a, int result, int x, int y, int z) {
  if (a.lt(x, y)) {
    if (a.lt(y, z)) a.swap(result, y);
    else if (a.lt(x, z)) a.swap(result, z);
    else a.swap(result, x);
  } else if (a.lt(x, z)) a.swap(result, x);
  else if (a.lt(y, z)) a.swap(result, z);
  else a.swap(result, y);
}

template <typename K, typename V>
LG_HD int unguarded_partition_pivot(const SortView<K, V>& a, int first, int last) {
  const int mid = first + (last - first) / 2;
  move_median_to_first(a, first, first + 1, mid, last - 1);
  int lo = first + 1, hi = last;
  const int pivot = first;
  while (true) {
    while (a.lt(lo, pivot)) ++lo;
    --hi;
    while (a.lt(pivot, hi)) --hi;
    if (!(lo < hi)) return lo;
    a.swap(lo, hi);
    ++lo;
  }
}

template <typename K, typename V>
LG_HD void unguarded_linear_insert(const SortView<K, V>& a, int last) {
  K vk = a.key[last];
  V vv = a.val[last];
  int next = last - 1;
  while (vk < a.key[next]) {
    a.move(last, next);
    last = next;
    --next;
  }
  a.key[last] = vk;
  a.val[last] = vv;
}

template <typename K, typename V>
LG_HD void insertion_sort(const SortView<K, V>& a, int first, int last) {
  if (first == last) return;
  for (int i = first + 1; i != last; ++i) {
    if (a.lt(i, first)) {
      K vk = a.key[i];
      V vv = a.val[i];
      for (int k = i; k > first; --k) a.move(k, k - 1);  // move_backward
      a.key[first] = vk;
      a.val[first] = vv;
    } else {
      unguarded_linear_insert(a, i);
    }
  }
}

// std::sort(key, key + n) carrying val; comparator key[a] < key[b].
template <typename K, typename V = int>
LG_HD void std_sort(K* key, V* val, int n) {
  if (n <= 1) return;
  SortView<K, V> a{key, val};
  struct Frame { int first, last, depth; };
  Frame stack[64];
  int sp = 0;
  stack[sp++] = Frame{0, n, 2 * floor_log2(n)};
  while (sp > 0) {
    Frame f = stack[--sp];
    int first = f.first, last = f.last, depth = f.depth;
    while (last - first > 16) {
      if (depth == 0) {
        heap_sort(a, first, last);
        break;
      }
      --depth;
      int cut = unguarded_partition_pivot(a, first, last);
      stack[sp++] = Frame{cut, last, depth};  // disjoint ranges: order of processing is immaterial
      last = cut;
    }
  }
  if (n > 16) {  // __final_insertion_sort
    insertion_sort(a, 0, 16);
    for (int i = 16; i != n; ++i) unguarded_linear_insert(a, i);
  } else {
    insertion_sort(a, 0, n);
  }
}

}  // namespace lg
