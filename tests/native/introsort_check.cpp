// Checks lego_introsort.h (the device's std::sort restatement) against the host's libstdc++
// std::sort: identical permutations of (key, val) pairs sorted by key only, on tie-heavy inputs.
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#include "lego_introsort.h"

template <typename K>
struct E { K key; int val; };
template <typename K>
struct ByKey { bool operator()(const E<K>& a, const E<K>& b) const { return a.key < b.key; } };

static uint64_t st = 0x9E3779B97F4A7C15ULL;
static uint64_t rnd() { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return st; }

template <typename K>
int check(int n, int distinct, bool sorted_input) {
  std::vector<E<K>> a(n);
  std::vector<K> k(n);
  std::vector<int> v(n);
  for (int i = 0; i < n; ++i) {
    K x = (K)(rnd() % (uint64_t)distinct);
    if (sorted_input) x = (K)(i * distinct / (n ? n : 1));
    a[i] = E<K>{x, i};
    k[i] = x;
    v[i] = i;
  }
  std::sort(a.begin(), a.end(), ByKey<K>());
  lg::std_sort<K>(k.data(), v.data(), n);
  for (int i = 0; i < n; ++i)
    if (a[i].val != v[i] || a[i].key != k[i]) return 1;
  return 0;
}

int main() {
  int bad = 0, total = 0;
  const int sizes[] = {0, 1, 2, 3, 15, 16, 17, 31, 33, 64, 100, 257, 300, 511, 1000, 1800, 2048, 3000};
  const int distincts[] = {1, 2, 3, 7, 50, 1000000};
  for (int n : sizes)
    for (int d : distincts)
      for (int rep = 0; rep < 20; ++rep) {
        bad += check<float>(n, d, false);
        bad += check<unsigned>(n, d, false);
        bad += check<float>(n, d, rep == 0);
        total += 3;
      }
  printf("introsort permutations checked %d mismatches %d\n", total, bad);
  return bad != 0;
}
