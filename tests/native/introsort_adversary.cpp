// Inputs that drive libstdc++'s introsort into its depth limit (the __partial_sort / heap-sort
// fallback), made with McIlroy's lazy-freezing adversary ("A Killer Adversary for Quicksort",
// 1999) run against the host's own std::sort.  Coarsening the frozen ranks (rank / c) adds ties.
//
//   introsort_adversary N C        -> prints N keys (one line, space separated)
//   introsort_adversary --check    -> for several N, C: asserts the restated introsort
//                                     (lego_introsort.h) takes the fallback and matches std::sort
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "lego_introsort.h"

static std::vector<int> adversary(int n) {
  std::vector<int> val(n, n);  // n = "gas": not yet frozen
  int nsolid = 0, candidate = 0;
  auto lt = [&](int x, int y) {
    if (val[x] == n && val[y] == n) {
      if (x == candidate) val[x] = nsolid++;
      else val[y] = nsolid++;
    }
    if (val[x] == n) candidate = x;
    else if (val[y] == n) candidate = y;
    return val[x] < val[y];
  };
  std::vector<int> ptr(n);
  for (int i = 0; i < n; ++i) ptr[i] = i;
  std::sort(ptr.begin(), ptr.end(), lt);
  for (int i = 0; i < n; ++i)
    if (val[i] == n) val[i] = nsolid++;
  return val;
}

static std::vector<unsigned> keys_for(int n, int c) {
  std::vector<int> v = adversary(n);
  std::vector<unsigned> k(n);
  for (int i = 0; i < n; ++i) k[i] = (unsigned)(v[i] / c);
  return k;
}

// The introsort loop of lego_introsort.h, counting depth-limit fallbacks.
static int count_fallbacks(std::vector<unsigned> k) {
  const int n = (int)k.size();
  std::vector<int> v(n);
  lg::SortView<unsigned, int> a{k.data(), v.data()};
  struct F { int first, last, depth; };
  std::vector<F> stack{{0, n, 2 * lg::floor_log2(n)}};
  int hits = 0;
  while (!stack.empty()) {
    F f = stack.back();
    stack.pop_back();
    int first = f.first, last = f.last, depth = f.depth;
    while (last - first > 16) {
      if (depth == 0) {
        ++hits;
        lg::heap_sort(a, first, last);
        break;
      }
      --depth;
      const int cut = lg::unguarded_partition_pivot(a, first, last);
      stack.push_back(F{cut, last, depth});
      last = cut;
    }
  }
  return hits;
}

int main(int argc, char** argv) {
  if (argc == 3) {
    const std::vector<unsigned> k = keys_for(atoi(argv[1]), atoi(argv[2]));
    for (size_t i = 0; i < k.size(); ++i) printf(i ? " %u" : "%u", k[i]);
    printf("\n");
    return 0;
  }
  if (argc == 2 && !strcmp(argv[1], "--check")) {
    int bad = 0;
    for (int n : {100, 700, 2048}) {
      for (int c : {1, 2}) {
        const std::vector<unsigned> k = keys_for(n, c);
        const int hits = count_fallbacks(k);
        struct E { unsigned key; int val; };
        std::vector<E> e(n);
        std::vector<unsigned> kk = k;
        std::vector<int> vv(n);
        for (int i = 0; i < n; ++i) { e[i] = E{k[i], i}; vv[i] = i; }
        std::sort(e.begin(), e.end(), [](const E& x, const E& y) { return x.key < y.key; });
        lg::std_sort<unsigned>(kk.data(), vv.data(), n);
        bool same = true;
        for (int i = 0; i < n; ++i) same = same && e[i].val == vv[i] && e[i].key == kk[i];
        printf("n=%d c=%d fallbacks=%d same=%d\n", n, c, hits, (int)same);
        if (!same || hits == 0) ++bad;
      }
    }
    return bad ? 1 : 0;
  }
  fprintf(stderr, "usage: introsort_adversary N C | --check\n");
  return 2;
}
