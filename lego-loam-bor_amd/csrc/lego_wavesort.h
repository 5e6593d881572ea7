// lego_wavesort.h — libstdc++ std::sort's permutation on one wave (device code shared by the front end's
// VoxelGrid, lego_kernels.hip, and the map clouds' VoxelGrid, lego_s2m.hip):
//   * heap_sort_wave: __partial_sort(first, last, last) = __make_heap + __sort_heap, the introsort's
//     depth-limit fallback;
//   * lvl_sort: the whole introsort (__introsort_loop + __final_insertion_sort) level-synchronously from
//     registers, for up to 64 R unsigned keys below 2^31 - 1 with 16-bit values.
// Bit-exact against libstdc++: tests/test_gpu_parity.py (test_device_sort_matches_libstdcxx,
// test_device_level_sort_matches_libstdcxx), every voxel_tie_order 0 parity test.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lego_device.h"
#include "lego_introsort.h"

#ifndef PROF_T  // phase timers: lego_kernels.hip's profile build defines them
#define PROF_T(v) do {} while (0)
#define PROF_ADD(slot, t0) do {} while (0)
#endif

namespace lgws {

using lg::SortView;
using lg::floor_log2;

LG_DEVICE int ws_lane() { return threadIdx.x & 63; }

// libstdc++ __adjust_heap (lego_introsort.h) on one lane, each level's two children (key and value)
// loaded before the choice.  (Reading the grandchildren too, two levels per round trip, measured
// 1.4x slower in tools/sort_bench.py: the extra LDS reads cost more than the latency they hide.)
template <typename K, typename V>
LG_DEVICE void adjust_heap_pf(const SortView<K, V>& a, int first, int hole, int len, K vk, V vv) {
  K* key = a.key + first;
  V* val = a.val + first;
  const int top = hole;
  int second = hole;
  const int lim = (len - 1) / 2;  // nodes below lim have two children
  if (second < lim) {
    int c = 2 * (second + 1);
    K kr = key[c], kl = key[c - 1];
    V vr = val[c], vl = val[c - 1];
    while (true) {
      second = c;
      K ks = kr;
      V vs = vr;
      if (kr < kl) { second = c - 1; ks = kl; vs = vl; }
      key[hole] = ks;
      val[hole] = vs;
      hole = second;
      if (!(second < lim)) break;
      c = 2 * (second + 1);
      kr = key[c]; kl = key[c - 1];
      vr = val[c]; vl = val[c - 1];
    }
  }
  if ((len & 1) == 0 && second == (len - 2) / 2) {
    second = 2 * (second + 1);
    key[hole] = key[second - 1];
    val[hole] = val[second - 1];
    hole = second - 1;
  }
  int parent = (hole - 1) / 2;  // __push_heap
  while (hole > top && key[parent] < vk) {
    key[hole] = key[parent];
    val[hole] = val[parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  key[hole] = vk;
  val[hole] = vv;
}

template <typename K>
LG_DEVICE K rdlane(K v, int l) {
  return __builtin_bit_cast(K, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}
template <typename K>
LG_DEVICE K wshfl(K v, int src) {
  return __builtin_bit_cast(K, __shfl(__builtin_bit_cast(int, v), src));
}

// __sort_heap (= repeated __pop_heap + __adjust_heap from the root) with the whole wave.
// (Round 4 measured a variant with two ballots and the descent as a branch-free walk on the scalar
// unit: bit-exact but slower, 1.40 vs 1.03 ms on the heaviest recorded ring, 157-161k vs 195k scans/s
// for order 0: ~75 dependent scalar operations a window cost more than the vector chain they replace.)
// Each pop's hole descent depends on keys only.  A window is the 5-level subtree below a window
// root x: lane l holds the key and value of one of its 62 nodes (level L = 1..5 at lanes
// [2^L - 2, 2^(L+1) - 2), siblings in lanes l, l ^ 1), read with one LDS round trip.  A node is on
// the descent path iff it and all its in-window ancestors win their sibling pair (right unless
// right < left, as __adjust_heap) and its parent has two children (parent < (len - 1) / 2), or it
// is the only (left) child of parent (len - 2) / 2 of an even-length heap whose in-window
// ancestors win -- a few VALU operations per lane against a precomputed ancestor mask.
// __push_heap then stops at the deepest path node p_u with !(k_u < value) (keys do not increase
// along a heap path), so the pop is a[parent(p_d)] = old a[p_d] for d = 1..u, a[p_u] = value: each
// path lane decides its own move (!(k_d < value)); the walk ends at the first path node that stays.
template <typename K, typename V>
LG_DEVICE void sort_heap_wave(const SortView<K, V>& a, int first, int last) {
  first = __builtin_amdgcn_readfirstlane(first);  // wave-uniform: keeps the pop loop scalar
  last = __builtin_amdgcn_readfirstlane(last);
  K* key = a.key + first;
  V* val = a.val + first;
  const int lane = ws_lane();
  const int lev = lane < 2 ? 1 : lane < 6 ? 2 : lane < 14 ? 3 : lane < 30 ? 4 : 5;
  const int off = lane - ((1 << lev) - 2);
  const int cst = (1 << lev) - 1 + off;  // node = (x << lev) + cst
  const bool right = (off & 1) != 0;
  unsigned long long anc = 0ull;  // lanes of the node's in-window ancestors (excluding itself)
  for (int j = 1; j < lev; ++j) anc |= 1ull << ((1 << j) - 2 + (off >> (lev - j)));
  const unsigned long long bottom = ((1ull << 32) - 1ull) << 30;  // level-5 lanes
  int len = last - first - 1;
  if (len < 1) return;
  // The top of the heap in registers: node t (levels 0-5) in lane t + 1, so lane l's children are lanes
  // 2l, 2l + 1, siblings share a DPP pair and a node's in-register ancestors are lanes l >> 1, l >> 2, ..
  const int tl = lane;
  K tk = key[min(max(tl - 1, 0), len)];
  V tv = val[min(max(tl - 1, 0), len)];
  unsigned long long tanc = 0ull;  // in-register ancestors below the root
  for (int j = tl >> 1; j >= 2; j >>= 1) tanc |= 1ull << j;
  const int c0 = 2 * tl;  // children lanes c0, c0 + 1 (lanes < 32)
  // The sibling tests as masks: a right child (odd lane, top, window and level 6 alike) wins unless
  // right < left, a left one iff left < right -- two compares straight into scalar masks and scalar
  // logic, then one 64-bit compare a lane against its ancestors-and-self mask -- instead of per-lane
  // boolean arithmetic (with the block-stored roots: the heaviest ring's heap pops 1.46 M -> 1.30 M cycles,
  // profiles/r06_heap_masks_ab.txt).
  const unsigned long long kOdd = 0xAAAAAAAAAAAAAAAAull, kTop = ~3ull;
  const unsigned long long tself = tanc | (1ull << tl);
  if (len >= 127) {
    // Heaps of 128 or more: levels 0-5 (nodes 0-62) stay in registers while the heap is at least that
    // large, node t in lane t + 1 (so lane l's children are lanes 2l, 2l + 1 and siblings share a DPP pair);
    // only the window below the level-5 path node (levels 6-10) is read from LDS.  Per pop: the top path
    // by the same win / ancestor ballots, one LDS window, the moves as pulls from the moving child (a
    // permute) and the window's writes.  The pop's value a[len] is read one pop ahead: the pop before can
    // only change it by ending its hole there (a[len] is the last leaf), and then it is that pop's value.
    const bool wlane = lane < 62;
    const unsigned long long kWin = (1ull << 62) - 1ull;
    const unsigned long long wself = anc | (1ull << lane);
    K nvk = key[len];
    V nvv = val[len];
    // The popped roots are kept a 64-slot block at a time (slot 64 q + l in lane l) and stored one block
    // at once: no pop reads a slot above its heap, so a slot's store can wait (a whole-wave store per
    // 64 pops instead of a one-lane store a pop).
    const int top_len = len;
    K ok = nvk;
    V ov = nvv;
    for (; len >= 127; --len) {
      const K vk = nvk;  // the pop's value; the root goes to its slot
      const V vv = nvv;
      nvk = key[len - 1];
      nvv = val[len - 1];
      const K rk = rdlane(tk, 1);
      const V rv = (V)__builtin_amdgcn_readlane((int)tv, 1);
      const bool mine = lane == (len & 63);
      ok = mine ? rk : ok;
      ov = mine ? rv : ov;
      if ((len & 63) == 0 && len + lane <= top_len) {  // block [len, len + 63] complete
        key[len + lane] = ok;
        val[len + lane] = ov;
      }
      // path through levels 1..5 (right unless right < left, as __adjust_heap)
      const K ts = __builtin_bit_cast(K, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, tk), 0xb1, 0xf, 0xf, false));
      const unsigned long long TGE = __builtin_amdgcn_ballot_w64(!(tk < ts));
      const unsigned long long TLT = __builtin_amdgcn_ballot_w64(ts < tk);
      const unsigned long long TW = ((TGE & kOdd) | (TLT & ~kOdd)) & kTop;
      const unsigned long long TP = __builtin_amdgcn_ballot_w64((TW & tself) == tself);
      const unsigned long long TM = TP & __builtin_amdgcn_ballot_w64(!(tk < vk));  // moving top path nodes (a prefix)
      const int x5l = 95 - __clzll((long long)(TP >> 32));  // the level-5 path lane
      // window below node x5 (levels 6..10; every level-5 node has two children while len >= 127)
      const int lim = (len - 1) / 2;
      const int only = (len & 1) == 0 ? len - 1 : -1;
      const int node = ((x5l - 1) << lev) + cst;
      const int par = (node - 1) >> 1;
      const int nc = wlane ? min(node, len - 1) : len - 1;
      const K kk = key[nc];
      const V vl = val[nc];
      // the top: each path node takes its moving child's (old) element
      const unsigned long long cm = tl < 32 ? (TM >> c0) & 3ull : 0ull;
      const int src = cm ? c0 + (int)((cm & 1ull) ^ 1ull) : tl;
      const K pk = wshfl(tk, src);
      const V pv = (V)__shfl((int)tv, src);
      const K ks = __builtin_bit_cast(K, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, kk), 0xb1, 0xf, 0xf, false));
      // (the only child -- node len - 1, a leaf -- counts as winning: its clamped sibling read is itself)
      const unsigned long long ONLY = __builtin_amdgcn_ballot_w64(node == only);
      const unsigned long long W = ((((__builtin_amdgcn_ballot_w64(!(kk < ks)) & kOdd) |
                                      (__builtin_amdgcn_ballot_w64(ks < kk) & ~kOdd)) & kWin) | ONLY);
      const unsigned long long P = __builtin_amdgcn_ballot_w64((W & wself) == wself) &
                                   (__builtin_amdgcn_ballot_w64(par < lim) | ONLY) & kWin;  // window path nodes
      const unsigned long long M = P & __builtin_amdgcn_ballot_w64(!(kk < vk)) & (0ull - ((TM >> x5l) & 1ull));
      const bool mv = ((M >> lane) & 1ull) != 0ull;  // (below a node that stays nothing moves)
      if (mv & (lev > 1)) {  // (level 6's parent is x5, in registers)
        key[par] = kk;
        val[par] = vl;
      }
      if (cm) { tk = pk; tv = pv; }
      if (M & 3ull) {  // x5 takes its level-6 child
        const int s6 = (int)((M & 1ull) ^ 1ull);
        const K nk = rdlane(kk, s6);
        const V nv = (V)__builtin_amdgcn_readlane((int)vl, s6);
        if (tl == x5l) { tk = nk; tv = nv; }
      }
      if (M) {
        int hole = __builtin_amdgcn_readlane(node, 63 - __clzll((long long)M));
        // a window that the path leaves through its bottom with every node moved continues below
        unsigned long long Mw = M, Pw = P;
        int xw = hole;
        while (Mw == Pw && (Mw & bottom) && xw <= lim) {
          const int node2 = (xw << lev) + cst;
          const int par2 = (node2 - 1) >> 1;
          const int nc2 = wlane ? min(node2, len - 1) : len - 1;
          const K k2 = key[nc2];
          const V v2 = val[nc2];
          const K s2 = __builtin_bit_cast(K, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, k2), 0xb1, 0xf, 0xf, false));
          const bool win2 = wlane & ((right & !(k2 < s2)) | (!right & (s2 < k2)));
          const unsigned long long W2 = __builtin_amdgcn_ballot_w64(win2);
          const bool onp2 = wlane & ((W2 & anc) == anc) & ((win2 & (par2 < lim)) | (node2 == only));
          const bool mv2 = onp2 & !(k2 < vk);
          Pw = __builtin_amdgcn_ballot_w64(onp2);
          Mw = __builtin_amdgcn_ballot_w64(mv2);
          if (mv2) {
            key[par2] = k2;
            val[par2] = v2;
          }
          if (Mw) hole = __builtin_amdgcn_readlane(node2, 63 - __clzll((long long)Mw));
          xw = hole;
        }
        if (lane == 0) { key[hole] = vk; val[hole] = vv; }
        if (hole == len - 1) { nvk = vk; nvv = vv; }
      } else {  // the deepest moved top node, or the root when none moves, takes the value
        const int th = TM ? 63 - __clzll((long long)TM) : 1;
        if (tl == th) { tk = vk; tv = vv; }
      }
    }
    {  // the last, partial block: slots len + 1 .. (its end, or top_len)
      const int p = len + 1, q = p & ~63;
      if ((p & 63) != 0 && q + lane >= p && q + lane <= top_len) {
        key[q + lane] = ok;
        val[q + lane] = ov;
      }
    }
  }
  // Heaps of at most 127: the whole heap in registers, the top as above and level 6 (nodes 63..126) in a
  // second pair, node 63 + l in lane l (children of top lane l >= 32: bottom lanes 2l - 64, 2l - 63).  A
  // pop reads no LDS: the value a[len] by a lane read, the top path by the ballots (with the reference's
  // one-child node `only` and the two-children bound `lim`), level 6 below the level-5 path node, the
  // moves as pulls; only the popped root is stored (at len, its sorted position).
  K bk = key[min(63 + lane, len)];
  V bv = val[min(63 + lane, len)];
  const int bl = lane;
  for (; len >= 1; --len) {
    const K vk = len <= 62 ? rdlane(tk, len + 1) : rdlane(bk, len - 63);
    const V vv = (V)__builtin_amdgcn_readlane(len <= 62 ? (int)tv : (int)bv, len <= 62 ? len + 1 : len - 63);
    const K rk = rdlane(tk, 1);
    const V rv = (V)__builtin_amdgcn_readlane((int)tv, 1);
    if (lane == 0) { key[len] = rk; val[len] = rv; }
    const int lim = (len - 1) / 2;
    const int only = (len & 1) == 0 ? len - 1 : -1;  // the only (left) child of node lim
    const K ts = __builtin_bit_cast(K, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, tk), 0xb1, 0xf, 0xf, false));
    // (the only child, a leaf, counts as winning; its parent is node lim, the last with children)
    const unsigned long long TONLY = __builtin_amdgcn_ballot_w64(tl - 1 == only) & kTop;
    const unsigned long long TW = ((((__builtin_amdgcn_ballot_w64(!(tk < ts)) & kOdd) |
                                     (__builtin_amdgcn_ballot_w64(ts < tk) & ~kOdd)) & kTop) | TONLY);
    const unsigned long long TP = __builtin_amdgcn_ballot_w64((TW & tself) == tself) &
                                  (__builtin_amdgcn_ballot_w64((tl >> 1) - 1 < lim) | TONLY);
    const unsigned long long TM = TP & __builtin_amdgcn_ballot_w64(!(tk < vk));  // moving top path nodes
    const bool x5m = (TM >> 32) != 0ull;  // the level-5 path node moved (only then can level 6 move)
    const int x5l = x5m ? 95 - __clzll((long long)(TP >> 32)) : 32;
    // level 6: the pair below x5 (lanes 2 x5l - 64, + 1), both children when x5 < lim, else the only one
    const K bs = __builtin_bit_cast(K, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, bk), 0xb1, 0xf, 0xf, false));
    const unsigned long long BW = (__builtin_amdgcn_ballot_w64(!(bk < bs)) & kOdd) |
                                  (__builtin_amdgcn_ballot_w64(bs < bk) & ~kOdd);
    const unsigned long long BONLY = __builtin_amdgcn_ballot_w64(63 + bl == only);
    const unsigned long long BP = x5m ? (3ull << (2 * x5l - 64)) & ((x5l - 1 < lim ? BW : 0ull) | BONLY) : 0ull;
    const unsigned long long BM = BP & __builtin_amdgcn_ballot_w64(!(bk < vk));
    // pulls from the moving child (old elements): top lanes < 32 from the top, level-5 lanes from level 6
    const unsigned long long cm = tl < 32 ? (TM >> c0) & 3ull : (BM >> (c0 - 64)) & 3ull;
    const int src = (cm ? c0 + (int)((cm & 1ull) ^ 1ull) : tl) & 63;
    const K pt = wshfl(tk, src), pb = wshfl(bk, src);
    const V qt = (V)__shfl((int)tv, src), qb = (V)__shfl((int)bv, src);
    if (cm) {
      tk = tl < 32 ? pt : pb;
      tv = tl < 32 ? qt : qb;
    }
    if (BM) {  // the deepest moved node takes the value
      if (bl == 63 - __clzll((long long)BM)) { bk = vk; bv = vv; }
    } else {
      const int th = TM ? 63 - __clzll((long long)TM) : 1;
      if (tl == th) { tk = vk; tv = vv; }
    }
  }
  if (lane == 0) { key[0] = rdlane(tk, 1); val[0] = (V)__builtin_amdgcn_readlane((int)tv, 1); }
  __syncthreads();
}

// __partial_sort(first, last, last) = __make_heap + __sort_heap.  __make_heap sifts the parents
// from (len-2)/2 down to 0; parents on one heap level have disjoint subtrees (and __push_heap stops
// at `top`), so each level runs in parallel, deepest level first.  __sort_heap's pops are a chain
// (one lane; tools/sort_bench.py measured whole-wave and register-resident variants slower).
template <typename K, typename V>
LG_DEVICE void heap_sort_wave(const SortView<K, V>& a, int first, int last) {
  const int lane = ws_lane();
  const int len = last - first;
  if (len >= 2) {
    const int plast = (len - 2) / 2;
    for (int lev = floor_log2(plast + 1); lev >= 0; --lev) {
      const int lo = (1 << lev) - 1, hi = min((2 << lev) - 2, plast);
      for (int p = hi - lane; p >= lo; p -= 64) adjust_heap_pf(a, first, p, len, a.key[first + p], a.val[first + p]);
      __syncthreads();
    }
  }
  PROF_T(t_pop0);
  // The pops are one dependent chain, usually the longest of the launch: let this wave win
  // instruction arbitration against the other waves of its SIMD while it runs them.
#ifndef LG_AB_NOPRIO
  __builtin_amdgcn_s_setprio(3);
#endif
  sort_heap_wave(a, first, last);
#ifndef LG_AB_NOPRIO
  __builtin_amdgcn_s_setprio(0);
#endif
  PROF_ADD(36, t_pop0);
}


// ============================================================================================
// Level-synchronous libstdc++ introsort (voxel_tie_order 0), one wave, n <= 64 R keys < 2^31 - 1.
//
// __introsort_loop's result does not depend on the order in which it visits its disjoint ranges,
// and every range at recursion level t has depth limit d0 - t.  So all ranges of a level are
// partitioned together, from registers: lane l holds positions [l R, l R + R) (key, value).
// __unguarded_partition on [f, l) with the median-of-3 pivot at f, per position p in (f, l):
//   left stop  lf(p) = !(key < pivot),  right stop rf(p) = !(pivot < key),
//   A(p) = #lf in (f, p),  B(p) = #rf in (p, l),  D(p) = A(p) - B(p)  (non-decreasing in p).
// Hoare's loop swaps the k-th left stop from the left with the k-th right stop from the right while
// the left one is below the right one: left stop p (rank A) is swapped iff D(p) < 0, right stop q
// (rank B) iff D(q) > 0, and the pair of rank k exchanges through two scratch slots (f + k and
// l - 1 - k; 2K < l - f).  The returned cut min(L_K, R_{K-1}) is the first position p > f with
// (lf(p) && D(p) >= 0) || (rf(p) && D(p) > 0).  Ranges still longer than 16 at depth 0 take the
// heap sort (heap_sort_wave, as the stack emulation).  __final_insertion_sort is then the stable
// order by key inside each final range (no element crosses a cut): each position's rank among the
// <= 15 neighbours of its range on either side.  Range starts are one bit per position (S, R bits a
// lane); the counts of the lanes below / above come from ballots of the per-lane totals' bits and
// one shuffle from the lane holding the range's start (or end).
// Bit-exact against libstdc++: test_device_sort_matches_libstdcxx (is_float 3), every voxel_tie_order
// 0 parity test.
// ============================================================================================
#define LV_BUF(R) (64 * (R) + 64)
// One position's work per scheduling region in the unrolled passes: left free, the scheduler
// interleaves all R positions and runs out of registers.
#define LV_SCHED() __builtin_amdgcn_sched_barrier(0)
// An opaque copy of a per-lane mask for each pass: the per-position bits ((S >> r) & 1 ...) a pass
// derives from it are then not shared with the other passes (which kept R of them live across all).
LG_DEVICE unsigned lv_opaque(unsigned v) {
  asm volatile("" : "+v"(v));
  return v;
}  // padded u64 slots: position p at p + p / R (conflict-free lanes)

template <int R>
struct VoxLvlLds {  // k_voxel<4> (R = 16, rings of <= 1,024 points): 9.2 KB per wave; <5> (R = 32): 17.4 KB
  union {
    struct { unsigned key[64 * R]; uint16_t val[64 * R]; } nat;  // natural order (in / out)
    unsigned long long buf[LV_BUF(R) + 64];                      // the sort's exchange buffer (+ dump slots)
  } u;
};

// Exclusive prefix over lanes of a per-lane count < 64, and the wave total.
LG_DEVICE void lv_lane_prefix(int c, int& ex, int& tot) {
  const unsigned long long below = (1ull << ws_lane()) - 1ull;
  ex = 0;
  tot = 0;
#pragma unroll
  for (int b = 0; b < 6; ++b) {
    const unsigned long long m = __ballot((c >> b) & 1);
    ex += __popcll(m & below) << b;
    tot += __popcll(m) << b;
  }
}

// The lanes holding the start of the range that runs into this lane (jb) and the end of the range
// that runs out of it (ja, -1: none), the first position of the former (cf) and the end of the
// latter (cl).
template <int R>
LG_DEVICE void lv_carry(unsigned S, int p0, int& jb, int& ja, int& cf, int& cl) {
  const int lane = ws_lane();
  const unsigned long long Ms = __ballot(S != 0u);
  const unsigned long long mb = Ms & ((1ull << lane) - 1ull);
  const unsigned long long ma = Ms & ~((2ull << lane) - 1ull);  // lane 63: none
  jb = mb ? 63 - __clzll((long long)mb) : 0;
  ja = ma ? __ffsll((long long)ma) - 1 : -1;
  const int lastS = S ? p0 + 31 - __clz(S) : -1;
  const int firstS = S ? p0 + __ffs(S) - 1 : 64 * R;
  cf = __shfl(lastS, jb);
  const int c1 = __shfl(firstS, ja < 0 ? lane : ja);
  cl = ja < 0 ? 64 * R : c1;
}

template <int R>
LG_DEVICE void lvl_sort(unsigned* nkey, uint16_t* nval, unsigned long long* buf, int n, int depth = -1) {
  static_assert(R >= 8 && R <= 32, "final ranks reach two lanes either side; masks are 32 bits");
  const int lane = ws_lane();
  const int p0 = lane * R;
  if (n <= 1) return;
  auto pad = [](int p) { return p + (int)((unsigned)p / R); };
  uint2* eb = reinterpret_cast<uint2*>(buf);  // (value | scratch << 16, key) pairs
  uint2* own = eb + lane * (R + 1);           // this lane's positions, padded
  const int dump = LV_BUF(R) + lane;          // exchange slot of positions that do not swap
  // e[r]: position p0 + r.  x: value (low 16 bits) | per-level scratch (high 16), y: key.  The
  // element is the whole register state: range bounds and counts are rebuilt from the start bits.
  uint2 e[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int p = p0 + r;
    const int pc = p < n ? p : n - 1;
    const unsigned kk = nkey[pc], vv = nval[pc];
    e[r] = make_uint2(vv, p < n ? kk : 0x7fffffffu);
  }
  __syncthreads();  // buf aliases nkey / nval
  // range starts: 0, and the padding range [n, 64 R) that never partitions
  unsigned S = (lane == 0 ? 1u : 0u) | ((n >= p0 && n < p0 + R) ? (1u << (n - p0)) : 0u);
  const int d0 = depth >= 0 ? depth : 2 * floor_log2(n);  // the range's depth limit (a sub-range: its own)
  const unsigned long long below = (1ull << lane) - 1ull;
  // first of the range holding position p0 + r (its start at or below it, else the carried one)
  // (positions relative to p0 inside the passes: in-lane positions are then immediates)
  auto first_of = [](unsigned Sx, int r, int cfr) {
    const unsigned sm = Sx & ((2u << r) - 1u);
    return sm ? 31 - __clz(sm) : cfr;
  };
  PROF_T(t_part0);
  for (int t = 0;; ++t) {
    int jb, ja, cf, cl;
    lv_carry<R>(S, p0, jb, ja, cf, cl);
    const int cfr = cf - p0, clr = cl - p0, nr = n - p0;
    unsigned AM = 0;  // positions in ranges that still partition (> 16 positions, not padding)
    {
      const unsigned Sx = lv_opaque(S);
      int l = clr;
#pragma unroll
      for (int r = R - 1; r >= 0; --r) {
        const int f = first_of(Sx, r, cfr);
        AM = (AM << 1) | ((l - f > 16 && f < nr) ? 1u : 0u);  // bit r after the remaining shifts
        l = ((Sx >> r) & 1u) ? r : l;
        LV_SCHED();
      }
    }
    if (__ballot(AM != 0u) == 0ull) break;
    if (t == d0) {  // depth limit: __partial_sort (heap sort) of every range still longer than 16
      PROF_T(t_hs0);
      unsigned* nk = nkey + p0;  // (base + immediate offsets: no per-position address registers)
      uint16_t* nv = nval + p0;
#pragma unroll
      for (int r = 0; r < R; ++r) { nk[r] = e[r].y; nv[r] = (uint16_t)e[r].x; }  // < RING_MAX
      __syncthreads();
      unsigned H = S & AM;
      unsigned long long HB;
      while ((HB = __ballot(H != 0u)) != 0ull) {
        const int src = __ffsll((long long)HB) - 1;
        int f = 0, l = 0;
        if (H) {
          const int r = __ffs(H) - 1;
          const unsigned hi = S & ~((2u << r) - 1u);
          f = p0 + r;
          l = hi ? p0 + __ffs(hi) - 1 : cl;
        }
        f = __builtin_amdgcn_readlane(f, src);
        l = __builtin_amdgcn_readlane(l, src);
        if (lane == src) H &= H - 1u;
        heap_sort_wave(SortView<unsigned, uint16_t>{nkey, nval}, f, l);
      }
#pragma unroll
      for (int r = 0; r < R; ++r) e[r] = make_uint2(nv[r], nk[r]);
      __syncthreads();
      PROF_ADD(7, t_hs0);
      break;
    }
    // __move_median_to_first(f, f + 1, mid, l - 1) for every partitioning range, through LDS
#pragma unroll
    for (int r = 0; r < R; ++r) own[r] = e[r];
    __syncthreads();
    {
      unsigned H = S & AM;
      while (H) {
        const int r = __ffs(H) - 1;
        H &= H - 1u;
        const unsigned hi = S & ~((2u << r) - 1u);
        const int f = p0 + r, l = hi ? p0 + __ffs(hi) - 1 : cl;
        const int x = f + 1, y = f + (l - f) / 2, z = l - 1;
        const uint2 ef = eb[pad(f)], ex = eb[pad(x)], ey = eb[pad(y)], ez = eb[pad(z)];
        int s;
        uint2 es;
        if (ex.y < ey.y) {
          if (ey.y < ez.y) { s = y; es = ey; }
          else if (ex.y < ez.y) { s = z; es = ez; }
          else { s = x; es = ex; }
        } else if (ex.y < ez.y) { s = x; es = ex; }
        else if (ey.y < ez.y) { s = z; es = ez; }
        else { s = y; es = ey; }
        eb[pad(f)] = es;
        eb[pad(s)] = ef;
      }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < R; ++r) e[r] = own[r];
    // the stop flags against each range's pivot (the key now at its start)
    unsigned lastKey = 0u;
    {
      const unsigned Sx = lv_opaque(S);
#pragma unroll
      for (int r = 0; r < R; ++r) lastKey = ((Sx >> r) & 1u) ? e[r].y : lastKey;
    }
    unsigned LF = 0u, RF = 0u;  // built top-down: bit r enters at bit 31 and moves down
    {
      const unsigned Sx = lv_opaque(S), Ax = lv_opaque(AM & ~S);
      unsigned pv = (unsigned)__shfl((int)lastKey, jb);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        pv = ((Sx >> r) & 1u) ? e[r].y : pv;
        const bool in = (Ax >> r) & 1u;  // partitioning, not the range's start
        LF = (LF >> 1) | ((in && e[r].y >= pv) ? 0x80000000u : 0u);
        RF = (RF >> 1) | ((in && e[r].y <= pv) ? 0x80000000u : 0u);
        LV_SCHED();
      }
      LF >>= 32 - R;
      RF >>= 32 - R;
    }
    // A(p) = #lf in (f, p), B(p) = #rf in (p, l): in-lane running counts, the lanes between from
    // per-lane totals
    const int tL = __popc(LF), tR = __popc(RF);
    int PL, PR, TL, TR;
    lv_lane_prefix(tL, PL, TL);
    lv_lane_prefix(tR, PR, TR);
    const int lastS = S ? p0 + 31 - __clz(S) : -1;
    const int firstS = S ? p0 + __ffs(S) - 1 : 0;
    const int tailL = S ? __popc(LF & ~((1u << (lastS - p0)) - 1u)) : tL;  // lf after the last start
    const int headR = S ? __popc(RF & ((1u << (firstS - p0)) - 1u)) : tR;  // rf before the first start
    int runA = __shfl(tailL - PL - tL, jb) + PL;                              // lf in (f, p0)
    const int yb = __shfl(PR + headR, ja < 0 ? lane : ja);
    int runB = (ja < 0 ? TR : yb) - PR - tR;                                  // rf in [p0 + R, l)
    {
      const unsigned Sx = lv_opaque(S), Lx = lv_opaque(LF);
#pragma unroll
      for (int r = 0; r < R; ++r) {  // scratch: A
        runA = ((Sx >> r) & 1u) ? 0 : runA;
        e[r].x = __builtin_amdgcn_perm((unsigned)runA, e[r].x, 0x05040100u);  // x.lo | A << 16
        runA += (int)((Lx >> r) & 1u);
      }
    }
    // swaps: each swapped position writes itself to its pair's slot (buf is scratch now: every
    // position is held in registers) and keeps the slot it reads back as scratch.  Branch-free:
    // bitwise flags, both slots computed, one select each.
    unsigned CM = 0u;  // cut candidates
    {
      const unsigned Sx = lv_opaque(S), Lx = lv_opaque(LF), Rx = lv_opaque(RF);
      int l = clr;
#pragma unroll
      for (int r = R - 1; r >= 0; --r) {
        const int f = first_of(Sx, r, cfr), A = (int)(e[r].x >> 16), B = runB;
        runB += (int)((Rx >> r) & 1u);
        runB = ((Sx >> r) & 1u) ? 0 : runB;
        const int D = A - B;
        const unsigned lf = (Lx >> r) & 1u, rf = (Rx >> r) & 1u;
        const unsigned dneg = (unsigned)D >> 31, dpos = (unsigned)(-D) >> 31;  // D < 0, D > 0
        const unsigned sw_l = lf & dneg, sw_r = rf & dpos;
        CM = (CM << 1) | (lf & (dneg ^ 1u)) | sw_r;  // bit r after the remaining shifts
        const int wl = p0 + (sw_l ? l - 1 - A : f + B), rl = p0 + (sw_l ? f + A : l - 1 - B);
        const int w = (sw_l | sw_r) ? pad(wl) : dump;
        const int rd = (sw_l | sw_r) ? pad(rl) : dump;
        eb[w] = e[r];
        e[r].x = __builtin_amdgcn_perm((unsigned)rd, e[r].x, 0x05040100u);  // x.lo | rd << 16
        l = ((Sx >> r) & 1u) ? r : l;
        LV_SCHED();
      }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const unsigned rd = e[r].x >> 16;
      const uint2 x = eb[rd];
      e[r] = rd != (unsigned)dump ? x : e[r];
    }
    __syncthreads();
    // the cut of each range: its first candidate
    const unsigned ctail = S ? (CM & ~((1u << (lastS - p0)) - 1u)) : CM;
    const unsigned long long CT = __ballot(ctail != 0u);
    unsigned seen = (CT & below & ~((1ull << jb) - 1ull)) != 0ull ? 1u : 0u;
    unsigned cuts = 0u;
    const unsigned Sx = lv_opaque(S);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      seen &= ~(Sx >> r) & 1u;
      const unsigned c = (CM >> r) & 1u;
      cuts = (cuts >> 1) | ((c & (seen ^ 1u)) << 31);
      seen |= c;
    }
    S |= cuts >> (32 - R);
  }
  PROF_ADD(6, t_part0);
  // __final_insertion_sort: the stable order by key inside each final range.  Ranges are ordered
  // (every key of a range <= every key of the next), so the keys of other ranges within +-15 never
  // count, and a range of > 16 positions (heap-sorted) is sorted already.  Keys are < 2^31 - 1 (the
  // padding's 2^31 - 1 sorts last), so bit 31 of a - b is (a < b), without compare masks.
  PROF_T(t_fin0);
  int kp[15], kn[15];  // the keys of positions p0 - 15 .. p0 - 1 and p0 + R .. p0 + R + 14 (lanes within 2)
#pragma unroll
  for (int i = 0; i < 15; ++i) {
    const int qb = i - 15, qa = R + i;             // offsets from p0
    const int db = (qb - (R - 1)) / R;             // floor(qb / R) (qb < 0): -1 or -2 lanes
    const int da = qa / R;                         // +1 or +2 lanes
    const int rb = qb - db * R, ra = qa - da * R;  // the register in that lane
    const int a = __shfl_up((int)e[rb].y, -db);
    const int b = __shfl_down((int)e[ra].y, da);
    kp[i] = lane < -db ? 0 : a;
    kn[i] = lane > 63 - da ? 0x7fffffff : b;
  }
  __syncthreads();  // buf reads are done: nkey / nval take the output
  // an opaque copy of p0: p0 + r here must not be shared with the loads before the loop (which
  // would keep R positions live through it)
  int p0o;
  asm volatile("v_mov_b32 %0, %1" : "=v"(p0o) : "v"(p0));
  unsigned* nk = nkey + p0o;
  uint16_t* nv = nval + p0o;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int kr = (int)e[r].y;
    int pos = r;
#pragma unroll
    for (int d = 1; d <= 15; ++d) {
      const int q = r - d, u = r + d;
      const int kq = q >= 0 ? (int)e[q >= 0 ? q : 0].y : kp[q + 15 >= 0 ? q + 15 : 0];
      const int ku = u < R ? (int)e[u < R ? u : 0].y : kn[u - R < 15 ? u - R : 0];
      pos += (int)(((unsigned)ku - (unsigned)kr) >> 31) - (int)(((unsigned)kr - (unsigned)kq) >> 31);
    }
    LV_SCHED();
    nk[pos] = (unsigned)kr;  // positions >= n keep their place (< 64 R <= RING_MAX)
    nv[pos] = (uint16_t)e[r].x;
  }
  __syncthreads();
  PROF_ADD(11, t_fin0);
}

}  // namespace lgws
