// lego_s2m.hip — scan-to-map LM on gfx950: MapOptimization::scan2MapOptimization
// (LeGO-LOAM/src/mapOptmization.cpp:1315-1332) and what it calls, behind include/lego_s2m.h.
//
// One workgroup per problem (one mapping sequence's current scan against its surrounding map):
//   1. hash grids over the two map clouds (replacing kdtreeCornerFromMap / kdtreeSurfFromMap,
//      :1317-1318): cells of 1.01 m, so the 1 m ball the reference's kNN-5 gate admits (:1036, :1144)
//      lies in the 27 cells around the query's; buckets hold points by a hash of the cell, each point
//      tagged with its packed cell so the search skips colliding cells;
//   2. up to 10 iterations (:1320-1328), each one pass over all queries (corner then surf, one lane a
//      query): pointAssociateToMap, exact kNN-5 of the 1 m ball by (distance, index), the line fit
//      (3x3 symmetric eigen solver, :1037-1131) or the plane fit (5x3 QR, :1145-1194), and the
//      query's row of the normal equations accumulated in double; a block reduction; thread 0 solves
//      the 6x6 system (QR, :1260), decides degeneracy at iteration 0 (:1262-1286) and convergence
//      (:1294-1311).
// Numerics follow oracle/s2m_oracle.cpp operation for operation (-ffp-contract=off; the Eigen pieces
// are the same restatements), except the normal equations' double sums, whose order differs.
#include <float.h>
#include <string.h>  // (before rocprim, whose texture iterator uses memset)
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <new>

#include <algorithm>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_segmented_radix_sort.hpp>

#include "../../include/lego_s2m.h"
#include "lego_device.h"
#include "lego_kdtree.h"
#include "lego_wavesort.h"  // lvl_sort / heap_sort_wave: the map clouds' std::sort order

using namespace lg;

namespace {

constexpr int S2M_THREADS = 1024;
constexpr int S2M_NB_MAX = 65536;  // hash buckets per map cloud (power of two)
constexpr float S2M_CELL = 1.01f;  // cell edge: >= the 1 m kNN gate plus rounding
constexpr int S2M_DIM = 1024;
constexpr int S2M_KD_STACK = 64 * 5 * 48;  // floats: 48 search frames a lane beyond 10 per map point
constexpr int S2M_LATENCY_MAX = 16;  // lego_s2m_run: up to this many problems take the latency layout
constexpr size_t S2M_WIDE_MAX = (size_t)8 << 20;  // few-clouds VoxelGrid layout: n * max_map_points <= this      // cells per axis a packed cell can hold (10 bits)

LG_DEVICE int lane_id() { return threadIdx.x & 63; }
LG_DEVICE int wave_id() { return threadIdx.x >> 6; }

struct S2mScratch {  // per problem, per map cloud
  int* start;        // [S2M_NB_MAX + 1] bucket ends after the build
  float4* pts;       // [max_map_points] x, y, z, packed cell
  int* idx;          // [max_map_points] index in the caller's cloud
  float4* rows;      // [max_map_points][2] (corner scratch only) the queries' LM rows of an iteration
  // nanoflann's tree of the map cloud, built only when a kNN-5 has an exact distance tie (lego_kdtree.h)
  KdNode* kd_node;   // [2 * max_map_points]
  int* kd_vind;      // [max_map_points]
  // shared by the problem's two clouds (the same pointers in both entries)
  int* kd_tmp;       // [2 * max_map_points] planeSplit's stop lists
  float* kd_frames;  // [10 * max_map_points + S2M_KD_STACK] the builds' stack, then the searches' stacks
  int* tieq;         // [max_map_points] an iteration's tied queries
};

// ---- restated Eigen pieces (oracle/s2m_oracle.cpp) ------------------------------------------------
LG_DEVICE float hypot_e(float x, float y) {
  const float ax = fabsf(x), ay = fabsf(y);
  float p, qp;
  if (ax > ay) { p = ax; qp = ay / p; }
  else { p = ay; qp = ax / p; }
  if (p == 0.f) return 0.f;
  return p * sqrtf(1.f + qp * qp);
}

LG_DEVICE void givens(float p, float q, float& c, float& s) {
  if (q == 0.f) {
    c = p < 0.f ? -1.f : 1.f;
    s = 0.f;
  } else if (p == 0.f) {
    c = 0.f;
    s = q < 0.f ? 1.f : -1.f;
  } else if (fabsf(p) > fabsf(q)) {
    const float t = q / p;
    float u = sqrtf(1.f + t * t);
    if (p < 0.f) u = -u;
    c = 1.f / u;
    s = -t * c;
  } else {
    const float t = p / q;
    float u = sqrtf(1.f + t * t);
    if (q < 0.f) u = -u;
    s = -1.f / u;
    c = -t * s;
  }
}

// SelfAdjointEigenSolver<Matrix3f> (Eigen 3.3.4): ascending eigenvalues, V column j = eigenvector j.
// (Every array index is a compile-time constant after unrolling, so the state stays in registers.)
LG_DEVICE void eig3(const float A[9], float ev[3], float V[9]) {
  float m[9] = {A[0], 0.f, 0.f, A[3], A[4], 0.f, A[6], A[7], A[8]};
  float scale = 0.f;
#pragma unroll
  for (int k = 0; k < 9; ++k) scale = fmaxf(scale, fabsf(m[k]));
  if (scale == 0.f) scale = 1.f;
  m[0] /= scale; m[3] /= scale; m[4] /= scale; m[6] /= scale; m[7] /= scale; m[8] /= scale;
  float d[3], e[3];
  e[2] = 0.f;
  d[0] = m[0];
  const float v1norm2 = m[6] * m[6];
  if (v1norm2 <= FLT_MIN) {
    d[1] = m[4]; d[2] = m[8]; e[0] = m[3]; e[1] = m[7];
    V[0] = 1.f; V[1] = 0.f; V[2] = 0.f; V[3] = 0.f; V[4] = 1.f; V[5] = 0.f; V[6] = 0.f; V[7] = 0.f; V[8] = 1.f;
  } else {
    const float beta = sqrtf(m[3] * m[3] + v1norm2);
    const float invBeta = 1.f / beta;
    const float m01 = m[3] * invBeta, m02 = m[6] * invBeta;
    const float q = 2.f * m01 * m[7] + m02 * (m[8] - m[4]);
    d[1] = m[4] + m02 * q;
    d[2] = m[8] - m02 * q;
    e[0] = beta;
    e[1] = m[7] - m01 * q;
    V[0] = 1.f; V[1] = 0.f; V[2] = 0.f; V[3] = 0.f; V[4] = m01; V[5] = m02; V[6] = 0.f; V[7] = m02; V[8] = -m01;
  }
  // computeFromTridiagonal_impl (maxIterations 30, n = 3): end, start in {0, 1, 2}
  int end = 2, start = 0, iter = 0;
  const float precision = 2.f * FLT_EPSILON;
  bool ok = true;
  while (end > 0) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
      if (i >= start && i < end &&
          (fabsf(e[i]) <= (fabsf(d[i]) + fabsf(d[i + 1])) * precision || fabsf(e[i]) <= FLT_MIN))
        e[i] = 0.f;
    if (end == 2 && e[1] == 0.f) end = 1;
    if (end == 1 && e[0] == 0.f) end = 0;
    if (end <= 0) break;
    iter++;
    if (iter > 90) { ok = false; break; }
    start = end - 1;
    if (start == 1 && e[0] != 0.f) start = 0;
    // tridiagonal_qr_step: Wilkinson shift
    const float dE = end == 2 ? d[2] : d[1], dE1 = end == 2 ? d[1] : d[0], ee = end == 2 ? e[1] : e[0];
    const float td = (dE1 - dE) * 0.5f;
    float mu = dE;
    if (td == 0.f) {
      mu -= fabsf(ee);
    } else {
      const float e2 = ee * ee;
      const float h = hypot_e(td, ee);
      if (e2 == 0.f) mu -= (ee / (td + (td > 0.f ? 1.f : -1.f))) * (ee / h);
      else mu -= e2 / (td + (td > 0.f ? h : -h));
    }
    float x = (start == 0 ? d[0] : d[1]) - mu, z = start == 0 ? e[0] : e[1];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      if (k < start || k >= end) continue;
      float c, s;
      givens(x, z, c, s);
      const float sdk = s * d[k] + c * e[k];
      const float dkp1 = s * e[k] + c * d[k + 1];
      d[k] = c * (c * d[k] - s * e[k]) - s * (c * e[k] - s * d[k + 1]);
      d[k + 1] = s * sdk + c * dkp1;
      e[k] = c * sdk - s * dkp1;
      if (k > start) e[k - 1 >= 0 ? k - 1 : 0] = c * e[k - 1 >= 0 ? k - 1 : 0] - s * z;
      x = e[k];
      if (k < end - 1) {
        z = -s * e[k + 1];
        e[k + 1] = c * e[k + 1];
      }
      if (!(c == 1.f && s == 0.f))
#pragma unroll
        for (int r = 0; r < 3; ++r) {
          const float xi = V[r * 3 + k], yi = V[r * 3 + k + 1];
          V[r * 3 + k] = c * xi - s * yi;
          V[r * 3 + k + 1] = s * xi + c * yi;
        }
    }
  }
  if (ok) {  // ascending: the first minimum of d[i..2] to position i, columns swapped with it
    int k = 0;
    float best = d[0];
    if (d[1] < best) { best = d[1]; k = 1; }
    if (d[2] < best) { best = d[2]; k = 2; }
    if (k == 1) {
      const float t = d[0]; d[0] = d[1]; d[1] = t;
#pragma unroll
      for (int r = 0; r < 3; ++r) { const float v = V[r * 3]; V[r * 3] = V[r * 3 + 1]; V[r * 3 + 1] = v; }
    } else if (k == 2) {
      const float t = d[0]; d[0] = d[2]; d[2] = t;
#pragma unroll
      for (int r = 0; r < 3; ++r) { const float v = V[r * 3]; V[r * 3] = V[r * 3 + 2]; V[r * 3 + 2] = v; }
    }
    if (d[2] < d[1]) {
      const float t = d[1]; d[1] = d[2]; d[2] = t;
#pragma unroll
      for (int r = 0; r < 3; ++r) { const float v = V[r * 3 + 1]; V[r * 3 + 1] = V[r * 3 + 2]; V[r * 3 + 2] = v; }
    }
  }
  ev[0] = d[0] * scale; ev[1] = d[1] * scale; ev[2] = d[2] * scale;
}

// ColPivHouseholderQR<Matrix<float, M, N>>::solve (M >= N), fully unrolled
template <int M, int N>
LG_DEVICE void qr_solve(const float* A_in, const float* b_in, float* x) {
  float A[M * N];
#pragma unroll
  for (int k = 0; k < M * N; ++k) A[k] = A_in[k];
  const float eps = FLT_EPSILON;
  float nu[N], nd[N], hc[N];
  int perm[N];
#pragma unroll
  for (int k = 0; k < N; ++k) {
    float s = 0.f;
#pragma unroll
    for (int r = 0; r < M; ++r) s += A[r * N + k] * A[r * N + k];
    nu[k] = nd[k] = sqrtf(s);
    perm[k] = k;
  }
  float maxn = 0.f;
#pragma unroll
  for (int k = 0; k < N; ++k) maxn = fmaxf(maxn, nu[k]);
  const float th_help = (maxn * eps) * (maxn * eps) / (float)M;
  const float ndt = sqrtf(eps);
  int nzp = N;
#pragma unroll
  for (int k = 0; k < N; ++k) {
    int bc = k;
    float bv = nu[k];
#pragma unroll
    for (int j = k + 1; j < N; ++j)
      if (nu[j] > bv) { bv = nu[j]; bc = j; }
    const float bsq = bv * bv;
    if (nzp == N && bsq < th_help * (float)(M - k)) nzp = k;
#pragma unroll
    for (int j = k + 1; j < N; ++j)
      if (j == bc) {
#pragma unroll
        for (int r = 0; r < M; ++r) { const float t = A[r * N + k]; A[r * N + k] = A[r * N + j]; A[r * N + j] = t; }
        float t = nu[k]; nu[k] = nu[j]; nu[j] = t;
        t = nd[k]; nd[k] = nd[j]; nd[j] = t;
        const int p = perm[k]; perm[k] = perm[j]; perm[j] = p;
      }
    float tail = 0.f;
#pragma unroll
    for (int r = k + 1; r < M; ++r) tail += A[r * N + k] * A[r * N + k];
    const float c0 = A[k * N + k];
    float tau, beta;
    if (tail <= FLT_MIN) {
      tau = 0.f;
      beta = c0;
#pragma unroll
      for (int r = k + 1; r < M; ++r) A[r * N + k] = 0.f;
    } else {
      beta = sqrtf(c0 * c0 + tail);
      if (c0 >= 0.f) beta = -beta;
#pragma unroll
      for (int r = k + 1; r < M; ++r) A[r * N + k] = A[r * N + k] / (c0 - beta);
      tau = (beta - c0) / beta;
    }
    hc[k] = tau;
    A[k * N + k] = beta;
    if (tau != 0.f)
#pragma unroll
      for (int j = k + 1; j < N; ++j) {
        float t = A[k * N + j];
#pragma unroll
        for (int r = k + 1; r < M; ++r) t += A[r * N + k] * A[r * N + j];
        A[k * N + j] -= tau * t;
#pragma unroll
        for (int r = k + 1; r < M; ++r) A[r * N + j] -= tau * A[r * N + k] * t;
      }
#pragma unroll
    for (int j = k + 1; j < N; ++j) {
      if (nu[j] != 0.f) {
        float t = fabsf(A[k * N + j]) / nu[j];
        t = (1.f + t) * (1.f - t);
        if (t < 0.f) t = 0.f;
        const float q = nu[j] / nd[j];
        const float t2 = t * q * q;
        if (t2 <= ndt) {
          float s = 0.f;
#pragma unroll
          for (int r = k + 1; r < M; ++r) s += A[r * N + j] * A[r * N + j];
          nd[j] = sqrtf(s);
          nu[j] = nd[j];
        } else {
          nu[j] *= sqrtf(t);
        }
      }
    }
  }
  float c[M];
#pragma unroll
  for (int k = 0; k < M; ++k) c[k] = b_in[k];
#pragma unroll
  for (int k = 0; k < N; ++k) {
    if (k >= nzp || hc[k] == 0.f) continue;
    float t = c[k];
#pragma unroll
    for (int r = k + 1; r < M; ++r) t += A[r * N + k] * c[r];
    c[k] -= hc[k] * t;
#pragma unroll
    for (int r = k + 1; r < M; ++r) c[r] -= hc[k] * A[r * N + k] * t;
  }
  float y[N];
#pragma unroll
  for (int i = N - 1; i >= 0; --i) {
    y[i] = 0.f;
    if (i >= nzp) continue;
    float t = c[i];
#pragma unroll
    for (int j = i + 1; j < N; ++j)
      if (j < nzp) t -= A[i * N + j] * y[j];
    y[i] = t / A[i * N + i];
  }
#pragma unroll
  for (int o = 0; o < N; ++o) {
    float v = 0.f;
#pragma unroll
    for (int i = 0; i < N; ++i)
      if (perm[i] == o) v = y[i];
    x[o] = v;
  }
}

// largest eigenvalue of a symmetric 6x6 < 100 (:1267-1285); Rayleigh / Gershgorin bounds first
__device__ __attribute__((noinline)) bool lmax6_below(const float* A, double thr) {
  double dmax = -1e300, gmax = -1e300;
  for (int i = 0; i < 6; ++i) {
    double g = 0.0;
    for (int j = 0; j < 6; ++j) g += fabs((double)A[i * 6 + j]);
    dmax = fmax(dmax, (double)A[i * 6 + i]);
    gmax = fmax(gmax, g);
  }
  if (dmax >= thr) return false;  // lambda_max >= max a_ii
  if (gmax < thr) return true;    // lambda_max <= max row sum
  double a[36];
  for (int k = 0; k < 36; ++k) a[k] = A[k];
  for (int sweep = 0; sweep < 50; ++sweep) {
    double off = 0.0;
    for (int p = 0; p < 6; ++p)
      for (int q = p + 1; q < 6; ++q) off += a[p * 6 + q] * a[p * 6 + q];
    if (off < 1e-30) break;
    for (int p = 0; p < 6; ++p)
      for (int q = p + 1; q < 6; ++q) {
        const double apq = a[p * 6 + q];
        if (apq == 0.0) continue;
        const double th = (a[q * 6 + q] - a[p * 6 + p]) / (2.0 * apq);
        const double t = (th >= 0 ? 1.0 : -1.0) / (fabs(th) + sqrt(th * th + 1.0));
        const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
        for (int k = 0; k < 6; ++k) {
          const double akp = a[k * 6 + p], akq = a[k * 6 + q];
          a[k * 6 + p] = c * akp - s * akq;
          a[k * 6 + q] = s * akp + c * akq;
        }
        for (int k = 0; k < 6; ++k) {
          const double apk = a[p * 6 + k], aqk = a[q * 6 + k];
          a[p * 6 + k] = c * apk - s * aqk;
          a[q * 6 + k] = s * apk + c * aqk;
        }
      }
  }
  double m = a[0];
  for (int k = 1; k < 6; ++k) m = fmax(m, a[k * 6 + k]);
  return m < thr;
}

// ---- hash grid -------------------------------------------------------------------------------------
LG_DEVICE int cell_of(float v, float mn) { return (int)floorf((v - mn) / S2M_CELL); }
LG_DEVICE int pack_cell(int cx, int cy, int cz) { return (cz << 20) | (cy << 10) | cx; }
LG_DEVICE int bucket_of(int packed, int lg_nb) { return (int)(((unsigned)packed * 2654435761u) >> (32 - lg_nb)); }

struct GridInfo {
  float mn[3];
  int lg_nb;
  int ok;  // every cell fits the packing
};

LG_DEVICE float block_min(float v, float* red) {
  for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o));
  __syncthreads();
  if (lane_id() == 0) red[wave_id()] = v;
  __syncthreads();
  float r = red[0];
  for (int w = 1; w < S2M_THREADS / 64; ++w) r = fminf(r, red[w]);
  return r;
}

// Build one map cloud's grid (whole workgroup).  Afterwards start[b] = end of bucket b.
LG_DEVICE void build_grid(const float4* __restrict__ cloud, int n, const S2mScratch& G, GridInfo& gi, float* red,
                          int* flag, int max_lg) {
  const int tid = threadIdx.x;
  float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
  for (int j = tid; j < n; j += S2M_THREADS) {
    const float4 p = cloud[j];
    mn[0] = fminf(mn[0], p.x); mn[1] = fminf(mn[1], p.y); mn[2] = fminf(mn[2], p.z);
    mx[0] = fmaxf(mx[0], p.x); mx[1] = fmaxf(mx[1], p.y); mx[2] = fmaxf(mx[2], p.z);
  }
  float lo[3], hi[3];
  for (int a = 0; a < 3; ++a) {
    lo[a] = block_min(mn[a], red);
    hi[a] = -block_min(-mx[a], red);
  }
  int lg = 8;
  while (lg < max_lg && (1 << lg) < n) ++lg;
  const int nb = 1 << lg;
  bool fits = true;
  for (int a = 0; a < 3; ++a) fits = fits && (n == 0 || cell_of(hi[a], lo[a]) < S2M_DIM);
  if (tid == 0) {
    for (int a = 0; a < 3; ++a) gi.mn[a] = lo[a];
    gi.lg_nb = lg;
    gi.ok = fits ? 1 : 0;
  }
  for (int b = tid; b <= nb; b += S2M_THREADS) G.start[b] = 0;
  __syncthreads();
  if (!gi.ok) return;
  for (int j = tid; j < n; j += S2M_THREADS) {
    const float4 p = cloud[j];
    const int pk = pack_cell(cell_of(p.x, lo[0]), cell_of(p.y, lo[1]), cell_of(p.z, lo[2]));
    atomicAdd(&G.start[bucket_of(pk, lg)], 1);
  }
  __syncthreads();
  // exclusive scan of the counts: a chunk per thread, then the chunk sums in thread 0 (nb <= 65536)
  const int per = (nb + S2M_THREADS - 1) / S2M_THREADS;
  const int b0 = min(tid * per, nb), b1 = min(b0 + per, nb);
  int local = 0;
  for (int b = b0; b < b1; ++b) local += G.start[b];
  flag[tid] = local;
  __syncthreads();
  if (tid == 0) {
    int run = 0;
    for (int t = 0; t < S2M_THREADS; ++t) { const int v = flag[t]; flag[t] = run; run += v; }
  }
  __syncthreads();
  int run = flag[tid];
  for (int b = b0; b < b1; ++b) { const int c = G.start[b]; G.start[b] = run; run += c; }
  __syncthreads();
  for (int j = tid; j < n; j += S2M_THREADS) {
    const float4 p = cloud[j];
    const int pk = pack_cell(cell_of(p.x, lo[0]), cell_of(p.y, lo[1]), cell_of(p.z, lo[2]));
    const int slot = atomicAdd(&G.start[bucket_of(pk, lg)], 1);
    G.pts[slot] = make_float4(p.x, p.y, p.z, __int_as_float(pk));
    G.idx[slot] = j;
  }
  __syncthreads();
}

// kNN-5 of q inside the 1 m ball by (distance, index): true when 5 points are closer than 1 (the
// reference's pointSearchSqDis[4] < 1.0); slot[] index the grid's points; tie = equal distances
// among the 6 nearest
LG_DEVICE bool knn5(const S2mScratch& G, const GridInfo& gi, float4 q, int slot[5], bool& tie) {
  float d[6];
  int ix[6], sl[6];
#pragma unroll
  for (int k = 0; k < 6; ++k) { d[k] = 1.0f; ix[k] = -1; sl[k] = -1; }
  const int qx = cell_of(q.x, gi.mn[0]), qy = cell_of(q.y, gi.mn[1]), qz = cell_of(q.z, gi.mn[2]);
  const float qv[3] = {q.x, q.y, q.z};
  const int qc[3] = {qx, qy, qz};
  // candidates ordered by (distance, index in the caller's cloud); the index is loaded only to break
  // an exact distance tie (ix = -1: not loaded yet), so the common path has no dependent load
  auto idx_of = [&](int k) {
    if (ix[k] < 0) ix[k] = G.idx[sl[k]];
    return ix[k];
  };
  auto consider = [&](const float4 p, int j, int pk) {
    if (__float_as_int(p.w) != pk) return;  // another cell in the bucket
    const float ex = q.x - p.x, ey = q.y - p.y, ez = q.z - p.z;
    const float dd = ex * ex + ey * ey + ez * ez;  // nanoflann L2_Simple_Adaptor order
    if (!(dd <= d[5]) || !(dd < 1.0f)) return;
    int id = -1;
    if (dd == d[5]) {
      id = G.idx[j];
      if (!(sl[5] < 0 || id < idx_of(5))) return;
    }
    d[5] = dd; ix[5] = id; sl[5] = j;
#pragma unroll
    for (int k = 5; k > 0; --k) {
      bool sw = d[k] < d[k - 1];
      if (d[k] == d[k - 1] && sl[k - 1] >= 0) sw = idx_of(k) < idx_of(k - 1);
      if (sw) {
        float td = d[k]; d[k] = d[k - 1]; d[k - 1] = td;
        int t = ix[k]; ix[k] = ix[k - 1]; ix[k - 1] = t;
        t = sl[k]; sl[k] = sl[k - 1]; sl[k - 1] = t;
      }
    }
  };
  // the query's cell, then its faces, edges and corners; a neighbour whose box (shrunk by 1 mm
  // against the cell assignment's rounding) lies farther than the current 6th distance holds no
  // point that could enter the 6 nearest or tie them
  for (int ring = 0; ring <= 3; ++ring)
    for (int dz = -1; dz <= 1; ++dz)
      for (int dy = -1; dy <= 1; ++dy)
        for (int dx = -1; dx <= 1; ++dx) {
          if (abs(dx) + abs(dy) + abs(dz) != ring) continue;
          const int cc[3] = {qx + dx, qy + dy, qz + dz};
          if (cc[0] < 0 || cc[0] >= S2M_DIM || cc[1] < 0 || cc[1] >= S2M_DIM || cc[2] < 0 || cc[2] >= S2M_DIM) continue;
          if (ring > 0) {
            float lb = 0.f;
#pragma unroll
            for (int a = 0; a < 3; ++a) {
              if (cc[a] == qc[a]) continue;
              const float lo = gi.mn[a] + (float)cc[a] * S2M_CELL, hi = lo + S2M_CELL;
              float e = fmaxf(fmaxf(lo - qv[a], qv[a] - hi), 0.f);
              e = fmaxf(e - 1e-3f, 0.f);
              lb += e * e;
            }
            if (lb > d[5]) continue;
          }
          const int pk = pack_cell(cc[0], cc[1], cc[2]);
          const int b = bucket_of(pk, gi.lg_nb);
          const int e = G.start[b];
          int j = b == 0 ? 0 : G.start[b - 1];
          for (; j + 3 < e; j += 4) {  // 4 loads in flight
            float4 p4[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) p4[u] = G.pts[j + u];
#pragma unroll
            for (int u = 0; u < 4; ++u) consider(p4[u], j + u, pk);
          }
          for (; j < e; ++j) consider(G.pts[j], j, pk);
        }
  tie = false;
  if (!(sl[4] >= 0)) return false;
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    slot[k] = sl[k];
    if (sl[k + 1] >= 0 && d[k] == d[k + 1]) tie = true;
  }
  return true;
}

struct Trig { float cRoll, sRoll, cPitch, sPitch, cYaw, sYaw, tX, tY, tZ; };

// pointAssociateToMap (:412-426)
LG_DEVICE float4 associate(const Trig& T, float4 pi) {
  const float x1 = T.cYaw * pi.x - T.sYaw * pi.y;
  const float y1 = T.sYaw * pi.x + T.cYaw * pi.y;
  const float z1 = pi.z;
  const float x2 = x1;
  const float y2 = T.cRoll * y1 - T.sRoll * z1;
  const float z2 = T.sRoll * y1 + T.cRoll * z1;
  return make_float4(T.cPitch * x2 + T.sPitch * z2 + T.tX, y2 + T.tY, -T.sPitch * x2 + T.cPitch * z2 + T.tZ, pi.w);
}

// cornerOptimization's per-point body (:1037-1131)
LG_DEVICE bool corner_coeff(const float4* nb, float4 sel, float4& coeff) {
  float cx = 0, cy = 0, cz = 0;
  for (int j = 0; j < 5; j++) { cx += nb[j].x; cy += nb[j].y; cz += nb[j].z; }
  cx /= 5; cy /= 5; cz /= 5;
  float a11 = 0, a12 = 0, a13 = 0, a22 = 0, a23 = 0, a33 = 0;
  for (int j = 0; j < 5; j++) {
    const float ax = nb[j].x - cx, ay = nb[j].y - cy, az = nb[j].z - cz;
    a11 += ax * ax; a12 += ax * ay; a13 += ax * az;
    a22 += ay * ay; a23 += ay * az; a33 += az * az;
  }
  a11 /= 5; a12 /= 5; a13 /= 5; a22 /= 5; a23 /= 5; a33 /= 5;
  const float A1[9] = {a11, a12, a13, a12, a22, a23, a13, a23, a33};
  float D[3], V[9];
  eig3(A1, D, V);
  if (!(D[2] > 3 * D[1])) return false;
  const float x0 = sel.x, y0 = sel.y, z0 = sel.z;
  const float x1 = (float)((double)cx + 0.1 * (double)V[0]), y1 = (float)((double)cy + 0.1 * (double)V[1]),
              z1 = (float)((double)cz + 0.1 * (double)V[2]);
  const float x2 = (float)((double)cx - 0.1 * (double)V[0]), y2 = (float)((double)cy - 0.1 * (double)V[1]),
              z2 = (float)((double)cz - 0.1 * (double)V[2]);
  const float m1 = (x0 - x1) * (y0 - y2) - (x0 - x2) * (y0 - y1);
  const float m2 = (x0 - x1) * (z0 - z2) - (x0 - x2) * (z0 - z1);
  const float m3 = (y0 - y1) * (z0 - z2) - (y0 - y2) * (z0 - z1);
  const float a012 = sqrtf(m1 * m1 + m2 * m2 + m3 * m3);
  const float l12 = sqrtf((x1 - x2) * (x1 - x2) + (y1 - y2) * (y1 - y2) + (z1 - z2) * (z1 - z2));
  const float la = ((y1 - y2) * m1 + (z1 - z2) * m2) / a012 / l12;
  const float lb = -((x1 - x2) * m1 - (z1 - z2) * m3) / a012 / l12;
  const float lc = -((x1 - x2) * m2 + (y1 - y2) * m3) / a012 / l12;
  const float ld2 = a012 / l12;
  const float s = (float)(1.0 - 0.9 * (double)fabsf(ld2));
  coeff = make_float4(s * la, s * lb, s * lc, s * ld2);
  return (double)s > 0.1;
}

// surfOptimization's per-point body (:1145-1194)
LG_DEVICE bool surf_coeff(const float4* nb, float4 sel, float4& coeff) {
  float A0[15], B0[5], X0[3];
  for (int j = 0; j < 5; j++) {
    A0[j * 3 + 0] = nb[j].x; A0[j * 3 + 1] = nb[j].y; A0[j * 3 + 2] = nb[j].z;
    B0[j] = -1.f;
  }
  qr_solve<5, 3>(A0, B0, X0);
  float pa = X0[0], pb = X0[1], pc = X0[2], pd = 1;
  const float ps = sqrtf(pa * pa + pb * pb + pc * pc);
  pa /= ps; pb /= ps; pc /= ps; pd /= ps;
  for (int j = 0; j < 5; j++)
    if ((double)fabsf(pa * nb[j].x + pb * nb[j].y + pc * nb[j].z + pd) > 0.2) return false;
  const float pd2 = pa * sel.x + pb * sel.y + pc * sel.z + pd;
  const float s = (float)(1.0 - 0.9 * (double)fabsf(pd2) / (double)sqrtf(sqrtf(sel.x * sel.x + sel.y * sel.y + sel.z * sel.z)));
  coeff = make_float4(s * pa, s * pb, s * pc, s * pd2);
  return (double)s > 0.1;
}

// One query of cornerOptimization / surfOptimization (:1030-1133, :1138-1196) and its
// LMOptimization row (:1219-1256): r0 = (arx, ary, arz, coeff.x), r1 = (coeff.y, coeff.z,
// -coeff.intensity, 1), or r1.w = 0 when the point is not selected.
struct QueryRow {
  float4 r0, r1;
  int st;
};
constexpr int S2M_ST_DEFER = 0x100;  // internal: a tied query whose row the tree search computes

LG_DEVICE QueryRow row_from_nb(bool is_corner, float4 ori, float4 sel, Trig T, const float4* nb, QueryRow out);

// defer: a query with tied distances returns S2M_ST_DEFER and no row (resolved by s2m_resolve_ties);
// otherwise the grid's (distance, index) order decides the tie
__device__ __attribute__((noinline)) QueryRow query_row(bool is_corner, float4 ori, Trig T, S2mScratch G,
                                                        GridInfo gi, bool defer = true) {
  QueryRow out;
  out.r0 = make_float4(0.f, 0.f, 0.f, 0.f);
  out.r1 = make_float4(0.f, 0.f, 0.f, 0.f);
  out.st = 0;
  const float4 sel = associate(T, ori);
  int sl[5];
  bool tie = false;
  if (!knn5(G, gi, sel, sl, tie)) return out;

  if (tie) {
    out.st |= LEGO_S2M_ST_KNN_TIE;
    if (defer) {
      out.st |= S2M_ST_DEFER;
      return out;
    }
  }
  float4 nb[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) nb[j] = G.pts[sl[j]];
  return row_from_nb(is_corner, ori, sel, T, nb, out);
}

// the query's fit and LM row from its 5 neighbours (x, y, z used)
LG_DEVICE QueryRow row_from_nb(bool is_corner, float4 ori, float4 sel, Trig T, const float4* nb, QueryRow out) {
  float4 c;
  if (!(is_corner ? corner_coeff(nb, sel, c) : surf_coeff(nb, sel, c))) return out;
  const float srx = T.sRoll, crx = T.cRoll, sry = T.sPitch, cry = T.cPitch, srz = T.sYaw, crz = T.cYaw;
  const float arx = (crx * sry * srz * ori.x + crx * crz * sry * ori.y - srx * sry * ori.z) * c.x +
                    (-srx * srz * ori.x - crz * srx * ori.y - crx * ori.z) * c.y +
                    (crx * cry * srz * ori.x + crx * cry * crz * ori.y - cry * srx * ori.z) * c.z;
  const float ary = ((cry * srx * srz - crz * sry) * ori.x + (sry * srz + cry * crz * srx) * ori.y + crx * cry * ori.z) * c.x +
                    ((-cry * crz - srx * sry * srz) * ori.x + (cry * srz - crz * srx * sry) * ori.y - crx * sry * ori.z) * c.z;
  const float arz = ((crz * srx * sry - cry * srz) * ori.x + (-cry * crz - srx * sry * srz) * ori.y) * c.x +
                    (crx * crz * ori.x - crx * srz * ori.y) * c.y +
                    ((sry * srz + cry * crz * srx) * ori.x + (crz * sry - cry * srx * srz) * ori.y) * c.z;
  out.r0 = make_float4(arx, ary, arz, c.x);
  out.r1 = make_float4(c.y, c.z, -c.w, 1.f);
  return out;
}


// Re-resolve an iteration's tied queries Gc.tieq[0, ntie) (S2M_ST_DEFER) with nanoflann's tree of their map
// cloud (kdtreeCornerFromMap / kdtreeSurfFromMap, :1317-1318; built on first use for the problem, built[c]
// 1, or -1 after a build-stack overflow), its searchLevel with a KNNResultSet(5) and the reference's
// pointSearchSqDis[4] < 1.0 gate (:1036, :1144).  A search-stack overflow keeps the grid's order.  Wave 0
// only; box: [2][6].
__device__ __attribute__((noinline)) void s2m_resolve_ties(const S2mScratch& Gc, const S2mScratch& Gs, GridInfo gc, GridInfo gs,
                                const float4* cmap, int ncm, const float4* smap, int nsm, const float4* corner,
                                const float4* surf, int nc, int ntie, const Trig& T, int* built, float* box,
                                int max_map, int* status) {
  const int lane = lane_id();
  bool need0 = false, need1 = false;
  for (int k = lane; k < ntie; k += 64) {
    if (Gc.tieq[k] < nc) need0 = true;
    else need1 = true;
  }
  const bool need[2] = {__ballot(need0) != 0ull, __ballot(need1) != 0ull};
  int bs[2];
  for (int c = 0; c < 2; ++c) {
    bs[c] = built[c];
    if (need[c] && bs[c] == 0) {
      const S2mScratch& G = c == 0 ? Gc : Gs;
      const lgkd::KdView K = {c == 0 ? cmap : smap, G.kd_node, G.kd_vind, Gc.kd_tmp, Gc.kd_frames, max_map};
      bs[c] = lgkd::kd_build(K, c == 0 ? ncm : nsm, box + 6 * c) < 0 ? -1 : 1;
      if (lane == 0) built[c] = bs[c];
      lgkd::kd_sync();
    }
  }
  const int cap = (10 * max_map + S2M_KD_STACK) / (5 * 64);  // search frames per lane (>= 48)
  for (int k0 = 0; k0 < ntie; k0 += 64) {
    const int k = k0 + lane;
    if (k >= ntie) continue;
    const int q = Gc.tieq[k];
    const bool is_corner = q < nc;
    const int c = is_corner ? 0 : 1;
    const float4 ori = is_corner ? corner[q] : surf[q - nc];
    QueryRow r;
    bool done = false;
    if (bs[c] == 1) {
      const S2mScratch& G = is_corner ? Gc : Gs;
      const float4* map = is_corner ? cmap : smap;
      const lgkd::KdView K = {map, G.kd_node, G.kd_vind, Gc.kd_tmp, Gc.kd_frames, max_map};
      const float4 sel = associate(T, ori);
      int idx[5];
      float dst[5];
      bool ovf = false;
      const int cnt = lgkd::kd_knn<5>(K, box + 6 * c, sel, Gc.kd_frames + (size_t)lane * cap * 5, cap, idx, dst, ovf);
      if (!ovf) {
        r.r0 = make_float4(0.f, 0.f, 0.f, 0.f);
        r.r1 = make_float4(0.f, 0.f, 0.f, 0.f);
        r.st = 0;
        if (cnt == 5 && dst[4] < 1.0f) {
          float4 nb[5];
#pragma unroll
          for (int j = 0; j < 5; ++j) nb[j] = map[idx[j]];
          r = row_from_nb(is_corner, ori, sel, T, nb, r);
        }
        done = true;
      }
    }
    if (!done) {  // the grid's order stands: not nanoflann's choice
      r = query_row(is_corner, ori, T, is_corner ? Gc : Gs, is_corner ? gc : gs, false);
      atomicOr(status, LEGO_S2M_ST_TIE_UNRESOLVED);
    }
    Gc.rows[2 * q] = r.r0;
    Gc.rows[2 * q + 1] = r.r1;
  }
}

constexpr int S2M_LG_SURF = 14, S2M_LG_CORNER = 13;  // bucket tables held in LDS: 64 KB + 32 KB

struct S2mLds {
  int tab_s[(1 << S2M_LG_SURF) + 1];    // the surf map's bucket ends (the grid's only dependent lookup)
  int tab_c[(1 << S2M_LG_CORNER) + 1];  // the corner map's
  float red[S2M_THREADS / 64];
  int scan[S2M_THREADS];
  double acc[S2M_THREADS / 64][28];
  GridInfo gc, gs;
  float t[6];
  Trig T;
  int flag, status, iters, nsel, degenerate;
  int ntie, kd_built[2];
  float kd_box[2][6];
};

// The normal equations (AtA upper triangle, AtB, count) over the rows of nq queries in two passes of 14
// double sums (register budget): lane tid sums rows q = tid, tid + 1024, ... in increasing q, loading R
// rows at a time (all in flight together; the second pass finds them in cache); each pass is reduced over
// the wave by xor butterflies and then per wave into L.acc (lm_solve adds the 16 wave sums in order).
// The oracle's normal_equations restates this order.
__device__ __attribute__((noinline)) void normal_equations(S2mLds& L, const float4* rows, int nq) {
  const int tid = threadIdx.x;
  constexpr int R = 4;
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    double acc[14];
#pragma unroll
    for (int k = 0; k < 14; ++k) acc[k] = 0.0;
    for (int base = 0; base < nq; base += R * S2M_THREADS) {
      float4 r0[R], r1[R];
#pragma unroll
      for (int u = 0; u < R; ++u) {
        const int q = base + u * S2M_THREADS + tid;
        const int qq = q < nq ? q : 0;
        r0[u] = rows[2 * qq];
        r1[u] = rows[2 * qq + 1];
      }
#pragma unroll
      for (int u = 0; u < R; ++u) {
        if (base + u * S2M_THREADS + tid >= nq || r1[u].w == 0.f) continue;
        const float a[6] = {r0[u].x, r0[u].y, r0[u].z, r0[u].w, r1[u].x, r1[u].y};
        const float b = r1[u].z;
        int k = 0;
#pragma unroll
        for (int r = 0; r < 6; ++r) {
#pragma unroll
          for (int j = r; j < 6; ++j) {
            if (k >= 14 * half && k < 14 * half + 14) acc[k - 14 * half] += (double)(a[r] * a[j]);
            ++k;
          }
        }
#pragma unroll
        for (int r = 0; r < 6; ++r)
          if (21 + r >= 14 * half && 21 + r < 14 * half + 14) acc[21 + r - 14 * half] += (double)(a[r] * b);
        if (half == 1) acc[13] += 1.0;
      }
    }
#pragma unroll
    for (int k = 0; k < 14; ++k)
      for (int o = 32; o > 0; o >>= 1) acc[k] += __shfl_xor(acc[k], o);
    if (lane_id() == 0)
      for (int k = 0; k < 14; ++k) L.acc[wave_id()][14 * half + k] = acc[k];
  }
}

// LMOptimization's solve (:1257-1311) on the reduced normal equations (thread 0)
__device__ __attribute__((noinline)) void lm_solve(S2mLds& L, int iterCount) {
  double s[28];
  for (int k = 0; k < 28; ++k) {
    s[k] = 0.0;
    for (int w = 0; w < S2M_THREADS / 64; ++w) s[k] += L.acc[w][k];
  }
  const int nsel = (int)s[27];
  L.iters = iterCount + 1;
  L.nsel = nsel;
  bool conv = false;
  if (nsel < 50) {
    L.status |= LEGO_S2M_ST_FEW;
  } else {
    float A[36], Bv[6], X[6];
    int k = 0;
    for (int r = 0; r < 6; ++r)
      for (int j = r; j < 6; ++j) { A[r * 6 + j] = A[j * 6 + r] = (float)s[k]; ++k; }
    for (int r = 0; r < 6; ++r) Bv[r] = (float)s[21 + r];
    qr_solve<6, 6>(A, Bv, X);
    if (iterCount == 0) {
      L.degenerate = lmax6_below(A, 100.0) ? 1 : 0;
      if (L.degenerate) L.status |= LEGO_S2M_ST_DEGENERATE;
    }
    if (L.degenerate)
      for (int j = 0; j < 6; ++j) X[j] = 0.f;  // matP = 0 (see oracle/s2m_oracle.cpp)
    for (int j = 0; j < 6; ++j) L.t[j] += X[j];
    const double r0 = (double)(X[0] * 57.29578f), r1 = (double)(X[1] * 57.29578f), r2 = (double)(X[2] * 57.29578f);
    const double t0 = (double)(X[3] * 100), t1 = (double)(X[4] * 100), t2 = (double)(X[5] * 100);
    const float deltaR = (float)sqrt(r0 * r0 + r1 * r1 + r2 * r2);
    const float deltaT = (float)sqrt(t0 * t0 + t1 * t1 + t2 * t2);
    conv = (double)deltaR < 0.05 && (double)deltaT < 0.05;
    if (conv) L.status |= LEGO_S2M_ST_CONVERGED;
  }
  L.flag = conv ? 1 : 0;
}

__global__ __launch_bounds__(S2M_THREADS) void k_s2m(lego_s2m_io io, S2mScratch* scratch, int max_map,
                                                     int max_iters) {
  __shared__ S2mLds L;
  const int p = blockIdx.x, tid = threadIdx.x;
  const float4* corner = (const float4*)io.corner + io.corner_off[p];
  const float4* surf = (const float4*)io.surf + io.surf_off[p];
  const float4* cmap = (const float4*)io.corner_map + io.corner_map_off[p];
  const float4* smap = (const float4*)io.surf_map + io.surf_map_off[p];
  const int nc = io.corner_n[p], ns = io.surf_n[p], ncm = io.corner_map_n[p], nsm = io.surf_map_n[p];
  int* info = io.info + 4 * p;
  if (!(ncm > 10 && nsm > 100)) {  // :1316
    if (tid == 0) { info[0] = 0; info[1] = 0; info[2] = 0; info[3] = LEGO_S2M_ST_SKIPPED; }
    return;
  }
  if (ncm > max_map || nsm > max_map || nc < 0 || ns < 0 || nc + ns > max_map) {
    if (tid == 0) { info[0] = -1; info[1] = 0; info[2] = 0; info[3] = LEGO_S2M_ST_SKIPPED; }
    return;
  }
  S2mScratch Gc = scratch[2 * p], Gs = scratch[2 * p + 1];
  Gc.start = L.tab_c;  // bucket tables in LDS, points in HBM
  Gs.start = L.tab_s;
  build_grid(cmap, ncm, Gc, L.gc, L.red, L.scan, S2M_LG_CORNER);
  build_grid(smap, nsm, Gs, L.gs, L.red, L.scan, S2M_LG_SURF);
  if (tid == 0) {
    for (int k = 0; k < 6; ++k) L.t[k] = io.transform[6 * p + k];
    L.degenerate = io.degenerate[p];
    L.status = 0;
    L.iters = 0;
    L.nsel = 0;
    L.flag = 0;
    L.kd_built[0] = L.kd_built[1] = 0;
  }
  __syncthreads();
  if (!L.gc.ok || !L.gs.ok) {  // a map wider than 1024 cells (1 km) on an axis
    if (tid == 0) { info[0] = -1; info[1] = 0; info[2] = 0; info[3] = LEGO_S2M_ST_SKIPPED; }
    return;
  }
  const GridInfo gc = L.gc, gs = L.gs;
  for (int iterCount = 0; iterCount < max_iters; iterCount++) {
    if (tid == 0) {  // updatePointAssociateToMapSinCos (:397-410); LMOptimization's trig is the same
      const float* t = L.t;
      L.T = Trig{cosf_g(t[0]), sinf_g(t[0]), cosf_g(t[1]), sinf_g(t[1]), cosf_g(t[2]), sinf_g(t[2]), t[3], t[4], t[5]};
      L.ntie = 0;
    }
    __syncthreads();
    const Trig T = L.T;
    // queries: each lane writes its query's LM row (or a zero flag) to the rows scratch
    for (int q = tid; q < nc + ns; q += S2M_THREADS) {
      const bool is_corner = q < nc;
      const float4 ori = is_corner ? corner[q] : surf[q - nc];
      const QueryRow r = query_row(is_corner, ori, T, is_corner ? Gc : Gs, is_corner ? gc : gs);
      if (r.st & S2M_ST_DEFER) Gc.tieq[atomicAdd(&L.ntie, 1)] = q;
      Gc.rows[2 * q] = r.r0;
      Gc.rows[2 * q + 1] = r.r1;
      if (r.st) atomicOr(&L.status, r.st & ~S2M_ST_DEFER);
    }
    __syncthreads();
    if (L.ntie > 0) {  // (uniform)
      if (wave_id() == 0)
        s2m_resolve_ties(Gc, Gs, gc, gs, cmap, ncm, smap, nsm, corner, surf, nc, L.ntie, T, L.kd_built, &L.kd_box[0][0],
                         max_map, &L.status);
      __syncthreads();
    }
    normal_equations(L, Gc.rows, nc + ns);
    __syncthreads();
    if (tid == 0) lm_solve(L, iterCount);
    __syncthreads();
    if (L.flag) break;
  }
  if (tid == 0) {
    for (int k = 0; k < 6; ++k) io.transform[6 * p + k] = L.t[k];
    io.degenerate[p] = L.degenerate;
    info[0] = 1;
    info[1] = L.iters;
    info[2] = L.nsel;
    info[3] = L.status;
  }
}


// ---- latency layout (few problems): the same computation over many workgroups a problem -----------
// k_s2m runs a problem in one workgroup, which suits hundreds of problems; a single mapping sequence
// would leave all but one CU idle.  Here a problem's grids are built by two workgroups (k_s2m_grid), each
// LM iteration's queries are spread over gridDim.x workgroups (k_s2m_rows) and one workgroup sums the
// normal equations in k_s2m's order and solves (k_s2m_solve, the same lm_solve).  The LM state lives in
// HBM between launches; a converged problem's later launches return at once.  Bit-identical to k_s2m.
struct S2mState {
  float t[6];
  int degenerate, status, iters, nsel, done;
  GridInfo gc, gs;
  int ntie, kd_built[2];  // tied queries of the iteration (k_s2m_rows -> k_s2m_solve); the trees' states
  float kd_box[2][6];
};

LG_DEVICE bool s2m_gates(const lego_s2m_io& io, int p, int max_map, int* info) {  // k_s2m's entry checks
  const int nc = io.corner_n[p], ns = io.surf_n[p], ncm = io.corner_map_n[p], nsm = io.surf_map_n[p];
  if (!(ncm > 10 && nsm > 100)) {  // :1316
    if (info) { info[0] = 0; info[1] = 0; info[2] = 0; info[3] = LEGO_S2M_ST_SKIPPED; }
    return false;
  }
  if (ncm > max_map || nsm > max_map || nc < 0 || ns < 0 || nc + ns > max_map) {
    if (info) { info[0] = -1; info[1] = 0; info[2] = 0; info[3] = LEGO_S2M_ST_SKIPPED; }
    return false;
  }
  return true;
}

// grid (2, n): x = 0 the corner map's grid, 1 the surf map's; bucket table copied to HBM
__global__ __launch_bounds__(S2M_THREADS) void k_s2m_grid(lego_s2m_io io, S2mScratch* scratch, S2mState* st,
                                                          int max_map) {
  __shared__ S2mLds L;
  const int which = blockIdx.x, p = blockIdx.y, tid = threadIdx.x;
  if (!s2m_gates(io, p, max_map, (which == 0 && tid == 0) ? io.info + 4 * p : nullptr)) {
    if (which == 0 && tid == 0) st[p].done = 1;
    return;
  }
  S2mScratch G = scratch[2 * p + which];
  int* tab = which == 0 ? L.tab_c : L.tab_s;
  G.start = tab;
  GridInfo& gi = which == 0 ? L.gc : L.gs;
  if (which == 0)
    build_grid((const float4*)io.corner_map + io.corner_map_off[p], io.corner_map_n[p], G, gi, L.red, L.scan,
               S2M_LG_CORNER);
  else
    build_grid((const float4*)io.surf_map + io.surf_map_off[p], io.surf_map_n[p], G, gi, L.red, L.scan, S2M_LG_SURF);
  const int nb = 1 << gi.lg_nb;
  int* dst = scratch[2 * p + which].start;
  for (int b = tid; b <= nb; b += S2M_THREADS) dst[b] = tab[b];
  if (tid == 0) {
    if (which == 0) {
      st[p].gc = gi;
      for (int k = 0; k < 6; ++k) st[p].t[k] = io.transform[6 * p + k];
      st[p].degenerate = io.degenerate[p];
      st[p].status = 0;
      st[p].iters = 0;
      st[p].nsel = 0;
      st[p].done = 0;
      st[p].ntie = 0;
      st[p].kd_built[0] = st[p].kd_built[1] = 0;
    } else {
      st[p].gs = gi;
    }
  }
}

// grid (G, n): one iteration's LM rows, queries q = blockIdx.x * 1024 + tid, strided by G * 1024
__global__ __launch_bounds__(S2M_THREADS) void k_s2m_rows(lego_s2m_io io, S2mScratch* scratch, S2mState* st) {
  __shared__ S2mLds L;
  const int p = blockIdx.y, tid = threadIdx.x;
  const S2mState* S = st + p;
  const int nc = io.corner_n[p], ns = io.surf_n[p];
  if (S->done || !S->gc.ok || !S->gs.ok || (int)blockIdx.x * S2M_THREADS >= nc + ns) return;
  const GridInfo gc = S->gc, gs = S->gs;
  S2mScratch Gc = scratch[2 * p], Gs = scratch[2 * p + 1];
  for (int b = tid; b <= (1 << gc.lg_nb); b += S2M_THREADS) L.tab_c[b] = Gc.start[b];
  for (int b = tid; b <= (1 << gs.lg_nb); b += S2M_THREADS) L.tab_s[b] = Gs.start[b];
  if (tid == 0) {
    const float* t = S->t;
    L.T = Trig{cosf_g(t[0]), sinf_g(t[0]), cosf_g(t[1]), sinf_g(t[1]), cosf_g(t[2]), sinf_g(t[2]), t[3], t[4], t[5]};
    L.status = 0;
  }
  __syncthreads();
  Gc.start = L.tab_c;
  Gs.start = L.tab_s;
  const Trig T = L.T;
  const float4* corner = (const float4*)io.corner + io.corner_off[p];
  const float4* surf = (const float4*)io.surf + io.surf_off[p];
  for (int q = blockIdx.x * S2M_THREADS + tid; q < nc + ns; q += gridDim.x * S2M_THREADS) {
    const bool is_corner = q < nc;
    const float4 ori = is_corner ? corner[q] : surf[q - nc];
    const QueryRow r = query_row(is_corner, ori, T, is_corner ? Gc : Gs, is_corner ? gc : gs);
    if (r.st & S2M_ST_DEFER) Gc.tieq[atomicAdd(&st[p].ntie, 1)] = q;
    Gc.rows[2 * q] = r.r0;
    Gc.rows[2 * q + 1] = r.r1;
    if (r.st) atomicOr(&L.status, r.st & ~S2M_ST_DEFER);
  }
  __syncthreads();
  if (tid == 0 && L.status) atomicOr(&st[p].status, L.status);
}

// grid (n): one iteration's normal equations and solve; the outputs are written after every iteration
__global__ __launch_bounds__(S2M_THREADS) void k_s2m_solve(lego_s2m_io io, S2mScratch* scratch, S2mState* st,
                                                           int iterCount, int max_iters, int max_map) {
  __shared__ S2mLds L;
  const int p = blockIdx.x, tid = threadIdx.x;
  S2mState* S = st + p;
  if (S->done) return;
  int* info = io.info + 4 * p;
  if (!S->gc.ok || !S->gs.ok) {  // a map wider than 1024 cells (1 km) on an axis
    __syncthreads();
    if (tid == 0) { info[0] = -1; info[1] = 0; info[2] = 0; info[3] = LEGO_S2M_ST_SKIPPED; S->done = 1; }
    return;
  }
  const int ntie = S->ntie;
  if (ntie > 0) {  // the iteration's tied queries (k_s2m_rows deferred them)
    if (wave_id() == 0) {
      const float* t = S->t;
      const Trig T = {cosf_g(t[0]), sinf_g(t[0]), cosf_g(t[1]), sinf_g(t[1]), cosf_g(t[2]), sinf_g(t[2]), t[3], t[4], t[5]};
      S2mScratch Gc = scratch[2 * p], Gs = scratch[2 * p + 1];
      s2m_resolve_ties(Gc, Gs, S->gc, S->gs, (const float4*)io.corner_map + io.corner_map_off[p], io.corner_map_n[p],
                       (const float4*)io.surf_map + io.surf_map_off[p], io.surf_map_n[p],
                       (const float4*)io.corner + io.corner_off[p], (const float4*)io.surf + io.surf_off[p],
                       io.corner_n[p], ntie, T, S->kd_built, &S->kd_box[0][0], max_map, &S->status);
    }
    __syncthreads();
    if (tid == 0) S->ntie = 0;
  }
  normal_equations(L, scratch[2 * p].rows, io.corner_n[p] + io.surf_n[p]);
  __syncthreads();
  if (tid == 0) {
    for (int k = 0; k < 6; ++k) L.t[k] = S->t[k];
    L.degenerate = S->degenerate;
    L.status = S->status;
    lm_solve(L, iterCount);
    for (int k = 0; k < 6; ++k) S->t[k] = L.t[k];
    S->degenerate = L.degenerate;
    S->status = L.status;
    S->done = (L.flag || iterCount + 1 >= max_iters) ? 1 : 0;
    for (int k = 0; k < 6; ++k) io.transform[6 * p + k] = L.t[k];
    io.degenerate[p] = L.degenerate;
    info[0] = 1;
    info[1] = L.iters;
    info[2] = L.nsel;
    info[3] = L.status;
  }
}

// ---- map-side cloud preparation -------------------------------------------------------------------
// transformPointCloud (:443-473) of part p (blockIdx.y) by its key pose
__global__ __launch_bounds__(256) void k_map_transform(lego_map_transform_io io) {
  const int p = blockIdx.y;
  __shared__ float tr[9];
  if (threadIdx.x == 0) {  // updateTransformPointCloudSinCos (:428-441): float cos / sin
    const float* q = io.pose + 6 * p;
    tr[0] = cosf_g(q[0]); tr[1] = sinf_g(q[0]); tr[2] = cosf_g(q[1]); tr[3] = sinf_g(q[1]);
    tr[4] = cosf_g(q[2]); tr[5] = sinf_g(q[2]); tr[6] = q[3]; tr[7] = q[4]; tr[8] = q[5];
  }
  __syncthreads();
  const float ctRoll = tr[0], stRoll = tr[1], ctPitch = tr[2], stPitch = tr[3], ctYaw = tr[4], stYaw = tr[5];
  const float4* in = (const float4*)io.in + io.in_off[p];
  float4* out = (float4*)io.out + io.out_off[p];
  const int n = io.in_n[p];
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const float4 f = in[i];
    const float x1 = ctYaw * f.x - stYaw * f.y;
    const float y1 = stYaw * f.x + ctYaw * f.y;
    const float z1 = f.z;
    const float x2 = x1;
    const float y2 = ctRoll * y1 - stRoll * z1;
    const float z2 = stRoll * y1 + ctRoll * z1;
    out[i] = make_float4(ctPitch * x2 + stPitch * z2 + tr[6], y2 + tr[7], -stPitch * x2 + ctPitch * z2 + tr[8], f.w);
  }
}

LG_DEVICE int block_excl_scan(int v, int* red, int& total) {
  const int lane = lane_id(), w = wave_id();
  int x = v;
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  __syncthreads();
  if (lane == 63) red[w] = x;
  __syncthreads();
  int off = 0, tot = 0;
  for (int k = 0; k < S2M_THREADS / 64; ++k) {
    if (k < w) off += red[k];
    tot += red[k];
  }
  total = tot;
  return off + x - v;
}

// VoxelGrid, part 1 (PCL applyFilter up to the sort): bounds, leaf indices, the cloud's sort segment
__global__ __launch_bounds__(S2M_THREADS) void k_vox_keys(lego_map_voxel_io io, unsigned* keys, unsigned* vals,
                                                          int* seg_b, int* seg_e, int* ovf, int cap) {
  __shared__ float red[S2M_THREADS / 64];
  __shared__ int sh[8];
  const int c = blockIdx.x, tid = threadIdx.x;
  const int n = io.in_n[c];
  const float4* in = (const float4*)io.in + io.in_off[c];
  if (n > cap || n < 0) {
    if (tid == 0) { seg_b[c] = seg_e[c] = c * cap; ovf[c] = -1; }
    return;
  }
  const float inv = 1.0f / io.leaf[c];  // inverse_leaf_size_
  float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
  for (int i = tid; i < n; i += S2M_THREADS) {  // getMinMax3D
    const float4 p = in[i];
    mn[0] = fminf(mn[0], p.x); mn[1] = fminf(mn[1], p.y); mn[2] = fminf(mn[2], p.z);
    mx[0] = fmaxf(mx[0], p.x); mx[1] = fmaxf(mx[1], p.y); mx[2] = fmaxf(mx[2], p.z);
  }
  float lo[3], hi[3];
  for (int a = 0; a < 3; ++a) {
    lo[a] = block_min(mn[a], red);
    hi[a] = -block_min(-mx[a], red);
  }
  if (tid == 0) {
    const long long dx = (long long)((hi[0] - lo[0]) * inv) + 1, dy = (long long)((hi[1] - lo[1]) * inv) + 1,
                    dz = (long long)((hi[2] - lo[2]) * inv) + 1;
    const int bad = n > 0 && dx * dy * dz > 2147483647LL;
    int min_b[3], div_b[3];
    for (int a = 0; a < 3; ++a) {
      min_b[a] = (int)floorf(lo[a] * inv);
      div_b[a] = (int)floorf(hi[a] * inv) - min_b[a] + 1;
    }
    sh[0] = min_b[0]; sh[1] = min_b[1]; sh[2] = min_b[2];
    sh[3] = div_b[0]; sh[4] = div_b[0] * div_b[1];
    sh[5] = bad;
    seg_b[c] = c * cap;
    seg_e[c] = c * cap + (bad ? 0 : n);
    ovf[c] = bad;
  }
  __syncthreads();
  if (sh[5]) return;
  const float mb0 = (float)sh[0], mb1 = (float)sh[1], mb2 = (float)sh[2];
  const int m1 = sh[3], m2 = sh[4];
  unsigned* k = keys + (size_t)c * cap;
  unsigned* v = vals + (size_t)c * cap;
  for (int i = tid; i < n; i += S2M_THREADS) {
    const float4 p = in[i];
    const int i0 = (int)(floorf(p.x * inv) - mb0), i1 = (int)(floorf(p.y * inv) - mb1), i2 = (int)(floorf(p.z * inv) - mb2);
    k[i] = (unsigned)(i0 + i1 * m1 + i2 * m2);
    v[i] = (unsigned)i;
  }
}

// VoxelGrid, part 2: one centroid per run of equal leaf index in the (stably) sorted keys
__global__ __launch_bounds__(S2M_THREADS) void k_vox_reduce(lego_map_voxel_io io, const unsigned* keys,
                                                            const unsigned* vals, const int* ovf, int cap) {
  __shared__ int red[S2M_THREADS / 64];
  const int c = blockIdx.x, tid = threadIdx.x;
  const int n = io.in_n[c];
  const float4* in = (const float4*)io.in + io.in_off[c];
  float4* out = (float4*)io.out + io.out_off[c];
  if (ovf[c] < 0) {
    if (tid == 0) { io.out_n[c] = -1; io.status[c] = 0; }
    return;
  }
  if (ovf[c]) {  // PCL: "Leaf size is too small ... Integer indices would overflow": output = input
    for (int i = tid; i < n; i += S2M_THREADS) out[i] = in[i];
    if (tid == 0) { io.out_n[c] = n; io.status[c] = LEGO_ST_VOXEL_OVERFLOW; }
    return;
  }
  const unsigned* k = keys + (size_t)c * cap;
  const unsigned* v = vals + (size_t)c * cap;
  __shared__ float4 tp[S2M_THREADS];   // the tile's points in sorted order (gathered together)
  __shared__ unsigned tk[S2M_THREADS + 1];
  int base = 0;
  for (int t0 = 0; t0 < n; t0 += S2M_THREADS) {
    const int i = t0 + tid;
    const int m = min(S2M_THREADS, n - t0);
    if (i < n) {
      tk[tid] = k[i];
      tp[tid] = in[v[i]];
    }
    if (tid == 0) tk[S2M_THREADS] = t0 > 0 ? k[t0 - 1] : 0u;
    __syncthreads();
    const bool head = i < n && (i == 0 || tk[tid] != (tid == 0 ? tk[S2M_THREADS] : tk[tid - 1]));
    int total;
    const int slot = base + block_excl_scan(head ? 1 : 0, red, total);
    if (head) {  // CentroidPoint: float sums in sorted order, / count
      float sx = 0.f, sy = 0.f, sz = 0.f, si = 0.f;
      const unsigned key = tk[tid];
      int j = tid;
      for (; j < m && tk[j] == key; ++j) {
        const float4 p = tp[j];
        sx += p.x; sy += p.y; sz += p.z; si += p.w;
      }
      int g = t0 + j;  // a run that continues past the tile
      if (j == m)
        for (; g < n && k[g] == key; ++g) {
          const float4 p = in[v[g]];
          sx += p.x; sy += p.y; sz += p.z; si += p.w;
        }
      const float cnt = (float)(g - i);
      out[slot] = make_float4(sx / cnt, sy / cnt, sz / cnt, si / cnt);
    }
    base += total;
    __syncthreads();  // the tile's LDS is reused
  }
  if (tid == 0) { io.out_n[c] = base; io.status[c] = 0; }
}

// ---- VoxelGrid for a few large clouds (the mapping thread's five) ----------------------------------
// One workgroup a cloud (k_vox_keys / segmented sort / k_vox_reduce) leaves most CUs idle when there are
// five clouds.  Here every stage runs over 1024-point tiles of every cloud: bounds by atomics, 64-bit
// keys (cloud << 32 | leaf index) at the clouds' compact offsets, one device-wide stable radix sort, head
// counts per tile, then the centroids, each tile's output slot from the counts of the tiles before it.
// Same output, bit for bit, as the per-cloud kernels.
LG_DEVICE int vxf_slots(const lego_map_voxel_io& io, int c, int cap) {  // a cloud's slots in the key arrays
  const int n = io.in_n[c];
  return (n < 0 || n > cap) ? 0 : n;
}
LG_DEVICE int ord_f(float f) {  // float -> int with the same order
  const int i = __float_as_int(f);
  return i >= 0 ? i : i ^ 0x7fffffff;
}
LG_DEVICE float unord_f(int i) { return __int_as_float(i >= 0 ? i : i ^ 0x7fffffff); }

// grid (tiles, n): bounds[6c..6c+5] = min of ord(x, y, z), min of ~ord(x, y, z) (i.e. the max); 0x7fffffff
// before the launch
__global__ __launch_bounds__(S2M_THREADS) void k_vxf_bounds(lego_map_voxel_io io, int* bounds, int cap) {
  __shared__ float red[S2M_THREADS / 64];
  const int t = blockIdx.x, c = blockIdx.y, tid = threadIdx.x;
  const int n = vxf_slots(io, c, cap);
  if (t * S2M_THREADS >= n) return;
  const float4* in = (const float4*)io.in + io.in_off[c];
  const int i = t * S2M_THREADS + tid;
  const float4 p = in[i < n ? i : t * S2M_THREADS];
  float lo[3], hi[3];
  for (int a = 0; a < 3; ++a) {
    const float x = a == 0 ? p.x : (a == 1 ? p.y : p.z);
    lo[a] = block_min(x, red);
    hi[a] = -block_min(-x, red);
  }
  if (tid == 0)
    for (int a = 0; a < 3; ++a) {
      atomicMin(&bounds[6 * c + a], ord_f(lo[a]));
      atomicMin(&bounds[6 * c + 3 + a], ~ord_f(hi[a]));
    }
}

// grid (tiles, n): leaf indices of tile t of cloud c at the cloud's compact offset; segments / overflow
// flags as k_vox_keys (seg_b = compact start, seg_e = seg_b + sorted entries)
__global__ __launch_bounds__(S2M_THREADS) void k_vxf_keys(lego_map_voxel_io io, const int* bounds,
                                                          unsigned long long* k64, unsigned* vals, int* seg_b,
                                                          int* seg_e, int* ovf, int cap, int n_clouds) {
  const int t = blockIdx.x, c = blockIdx.y, tid = threadIdx.x;
  const int n = io.in_n[c];
  const int ns = vxf_slots(io, c, cap);
  int base = 0;
  for (int q = 0; q < c; ++q) base += vxf_slots(io, q, cap);
  if (n > cap || n < 0) {
    if (t == 0 && tid == 0) { seg_b[c] = seg_e[c] = base; ovf[c] = -1; }
    return;
  }
  const float inv = 1.0f / io.leaf[c];
  float lo[3], hi[3];
  for (int a = 0; a < 3; ++a) {
    lo[a] = unord_f(bounds[6 * c + a]);
    hi[a] = unord_f(~bounds[6 * c + 3 + a]);
  }
  const long long dx = (long long)((hi[0] - lo[0]) * inv) + 1, dy = (long long)((hi[1] - lo[1]) * inv) + 1,
                  dz = (long long)((hi[2] - lo[2]) * inv) + 1;
  const bool bad = n > 0 && dx * dy * dz > 2147483647LL;
  int min_b[3], div_b[3];
  for (int a = 0; a < 3; ++a) {
    min_b[a] = (int)floorf(lo[a] * inv);
    div_b[a] = (int)floorf(hi[a] * inv) - min_b[a] + 1;
  }
  if (t == 0 && tid == 0) {
    seg_b[c] = base;
    seg_e[c] = base + (bad ? 0 : n);
    ovf[c] = bad ? 1 : 0;
  }
  const int i = t * S2M_THREADS + tid;
  if (i >= ns) return;
  const size_t slot = (size_t)base + i;
  if (bad) {  // sorts inside cloud c's own range (every later cloud keeps its compact offset); never read
    k64[slot] = (unsigned long long)c << 32;
    vals[slot] = 0u;
    return;
  }
  const float4 p = ((const float4*)io.in + io.in_off[c])[i];
  const float mb0 = (float)min_b[0], mb1 = (float)min_b[1], mb2 = (float)min_b[2];
  const int i0 = (int)(floorf(p.x * inv) - mb0), i1 = (int)(floorf(p.y * inv) - mb1), i2 = (int)(floorf(p.z * inv) - mb2);
  k64[slot] = ((unsigned long long)c << 32) | (unsigned)(i0 + i1 * div_b[0] + i2 * (div_b[0] * div_b[1]));
  vals[slot] = (unsigned)i;
}

// sorted entry i of cloud c (start = seg_b[c] in the sorted arrays): its leaf index (the low word)
LG_DEVICE unsigned vxf_key(const unsigned long long* k, size_t i) { return (unsigned)k[i]; }

// grid (tiles, n): heads (first entry of each leaf's run) per tile of the cloud's sorted entries
__global__ __launch_bounds__(S2M_THREADS) void k_vxf_heads(const unsigned long long* k, const int* seg_b,
                                                           const int* seg_e, int* tcount, int tiles) {
  __shared__ int red[S2M_THREADS / 64];
  const int t = blockIdx.x, c = blockIdx.y, tid = threadIdx.x;
  const int m = seg_e[c] - seg_b[c];
  if (t * S2M_THREADS >= m) return;
  const size_t b0 = (size_t)seg_b[c];
  const int i = t * S2M_THREADS + tid;
  const bool head = i < m && (i == 0 || vxf_key(k, b0 + i) != vxf_key(k, b0 + i - 1));
  int total;
  block_excl_scan(head ? 1 : 0, red, total);
  if (tid == 0) tcount[c * tiles + t] = total;
}

// grid (tiles, n): the centroids (CentroidPoint: float sums in sorted order, / count)
__global__ __launch_bounds__(S2M_THREADS) void k_vxf_emit(lego_map_voxel_io io, const unsigned long long* k,
                                                          const unsigned* vals, const int* seg_b, const int* seg_e,
                                                          const int* ovf, const int* tcount, int tiles) {
  __shared__ int red[S2M_THREADS / 64];
  const int t = blockIdx.x, c = blockIdx.y, tid = threadIdx.x;
  const int n = io.in_n[c];
  const float4* in = (const float4*)io.in + io.in_off[c];
  float4* out = (float4*)io.out + io.out_off[c];
  if (ovf[c] < 0) {
    if (t == 0 && tid == 0) { io.out_n[c] = -1; io.status[c] = 0; }
    return;
  }
  if (ovf[c]) {  // PCL: "Leaf size is too small ... Integer indices would overflow": output = input
    const int i = t * S2M_THREADS + tid;
    if (i < n) out[i] = in[i];
    if (t == 0 && tid == 0) { io.out_n[c] = n; io.status[c] = LEGO_ST_VOXEL_OVERFLOW; }
    return;
  }
  const int m = seg_e[c] - seg_b[c];
  if (t == 0 && tid == 0) {
    int tot = 0;
    for (int q = 0; q * S2M_THREADS < m; ++q) tot += tcount[c * tiles + q];
    io.out_n[c] = tot;
    io.status[c] = 0;
  }
  if (t * S2M_THREADS >= m) return;
  int base = 0;
  for (int q = 0; q < t; ++q) base += tcount[c * tiles + q];
  const size_t b0 = (size_t)seg_b[c];
  const int i = t * S2M_THREADS + tid;
  const unsigned key = i < m ? vxf_key(k, b0 + i) : 0u;
  const bool head = i < m && (i == 0 || key != vxf_key(k, b0 + i - 1));
  int total;
  const int slot = base + block_excl_scan(head ? 1 : 0, red, total);
  if (!head) return;
  float sx = 0.f, sy = 0.f, sz = 0.f, si = 0.f;
  int g = i;
  for (; g < m && vxf_key(k, b0 + g) == key; ++g) {
    const float4 p = in[vals[b0 + g]];
    sx += p.x; sy += p.y; sz += p.z; si += p.w;
  }
  const float cnt = (float)(g - i);
  out[slot] = make_float4(sx / cnt, sy / cnt, sz / cnt, si / cnt);
}

// ---- VoxelGrid with PCL's std::sort tie order (voxel_tie_order 0) for map clouds -----------------------
// libstdc++'s introsort over every cloud's (leaf index, point index) pairs, as the front end's VoxelGrid
// (lego_wavesort.h: lvl_sort) but device-wide while ranges are large: all ranges of a recursion level
// longer than VXS_SMALL are partitioned together, a range in chunks of VXS_CH positions (k_vxs_*), each
// Hoare stop's rank from per-chunk counts; ranges of at most VXS_SMALL positions then finish on one wave
// each with lvl_sort from their own depth limit (k_vxs_small), ranges still longer than VXS_SMALL at depth
// 0 take the heap sort (k_vxs_heap).  The pairs are sorted in place in m->d_keys / d_vals.
constexpr int VXS_SMALL = 2048;       // ranges finished by one wave (lvl_sort<32>)
constexpr int VXS_TPB = 256;          // threads per chunk block
constexpr int VXS_EPT = 16;           // positions per thread
constexpr int VXS_CH = VXS_TPB * VXS_EPT;

struct VxsSeg {  // a range [f, l) of the key arrays at depth limit d
  int f, l, d;
};

// grid (big ranges): __move_median_to_first(f, f + 1, mid, l - 1); the pivot key; the cut reset to l
__global__ __launch_bounds__(64) void k_vxs_median(const VxsSeg* segs, const int* nseg, unsigned* keys,
                                                    unsigned* vals, unsigned* pivot, int* cut) {
  const int s = blockIdx.x * 64 + threadIdx.x;
  if (s >= *nseg) return;
  const VxsSeg g = segs[s];
  const int x = g.f + 1, y = g.f + (g.l - g.f) / 2, z = g.l - 1;
  const unsigned kx = keys[x], ky = keys[y], kz = keys[z];
  int sel;
  if (kx < ky) sel = ky < kz ? y : (kx < kz ? z : x);
  else sel = kx < kz ? x : (ky < kz ? z : y);
  const unsigned kf = keys[g.f], vf = vals[g.f], ks = keys[sel], vs = vals[sel];
  keys[g.f] = ks; vals[g.f] = vs;
  keys[sel] = kf; vals[sel] = vf;
  pivot[s] = ks;
  cut[s] = g.l;
}

// Block-wide exclusive scan of a packed (lf | rf << 16) count per thread (VXS_TPB threads).
LG_DEVICE int vxs_block_scan(int v, int* sh, int& total) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int x = v;
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) sh[w] = x;
  __syncthreads();
  int off = 0, tot = 0;
  for (int k = 0; k < VXS_TPB / 64; ++k) {
    if (k < w) off += sh[k];
    tot += sh[k];
  }
  __syncthreads();
  total = tot;
  return off + x - v;
}

// the stop flags of position p of range g (p > f) against pivot pv: lf | rf << 16
LG_DEVICE int vxs_flags(unsigned k, unsigned pv) { return (k >= pv ? 1 : 0) | ((k <= pv ? 1 : 0) << 16); }

// grid (big ranges x maxch chunks, one dimension: block b is chunk b % maxch of range b / maxch): per
// chunk the counts of left / right stops (packed lf | rf << 16)
__global__ __launch_bounds__(VXS_TPB) void k_vxs_count(const VxsSeg* segs, const int* nseg, const unsigned* keys,
                                                       const unsigned* pivot, int* cnt, int maxch) {
  __shared__ int sh[VXS_TPB / 64];
  const int s = blockIdx.x / maxch, c = blockIdx.x % maxch;
  if (s >= *nseg) return;
  const VxsSeg g = segs[s];
  const int c0 = g.f + c * VXS_CH;
  if (c0 >= g.l) return;
  const unsigned pv = pivot[s];
  int v = 0;
  const int p0 = c0 + threadIdx.x * VXS_EPT;
#pragma unroll
  for (int e = 0; e < VXS_EPT; ++e) {
    const int p = p0 + e;
    if (p > g.f && p < g.l) v += vxs_flags(keys[p], pv);
  }
  int total;
  vxs_block_scan(v, sh, total);
  if (threadIdx.x == 0) cnt[(size_t)s * maxch + c] = total;
}

// grid (as k_vxs_count): each stop's rank, Hoare's swaps through the scratch slots (f + k for the
// k-th right stop, l - 1 - k for the k-th left stop), the read-back slot of every swapped position and
// the cut (the first left stop with D >= 0 or right stop with D > 0)
__global__ __launch_bounds__(VXS_TPB) void k_vxs_exchange(const VxsSeg* segs, const int* nseg, const unsigned* keys,
                                                          const unsigned* vals, const unsigned* pivot, const int* cnt,
                                                          int maxch, unsigned* xk, unsigned* xv, int* rds, int* cut) {
  __shared__ int sh[VXS_TPB / 64];
  const int s = blockIdx.x / maxch, c = blockIdx.x % maxch;
  if (s >= *nseg) return;
  const VxsSeg g = segs[s];
  const int c0 = g.f + c * VXS_CH;
  if (c0 >= g.l) return;
  const unsigned pv = pivot[s];
  const int nch = (g.l - g.f + VXS_CH - 1) / VXS_CH;
  // left / right stops of the chunks before this one, right stops of the whole range (a chunk's packed
  // counts fit 16 bits each; a range's do not)
  int beforeL = 0, beforeR = 0, totR = 0;
  for (int q = 0; q < nch; ++q) {
    const int t = cnt[(size_t)s * maxch + q];
    if (q < c) { beforeL += t & 0xffff; beforeR += t >> 16; }
    totR += t >> 16;
  }
  const int p0 = c0 + threadIdx.x * VXS_EPT;
  unsigned k[VXS_EPT];
  int v = 0;
#pragma unroll
  for (int e = 0; e < VXS_EPT; ++e) {
    const int p = p0 + e;
    k[e] = (p > g.f && p < g.l) ? keys[p] : 0u;
    if (p > g.f && p < g.l) v += vxs_flags(k[e], pv);
  }
  int total;
  const int pre = vxs_block_scan(v, sh, total);  // lf | rf << 16 before this thread's positions, in the block
  int runL = (pre & 0xffff) + beforeL, runR = (pre >> 16) + beforeR;  // lf / rf in (f, p)
  int best = 0x7fffffff;
#pragma unroll
  for (int e = 0; e < VXS_EPT; ++e) {
    const int p = p0 + e;
    if (!(p > g.f && p < g.l)) continue;
    const int fl = vxs_flags(k[e], pv);
    const int A = runL;                            // left stops in (f, p)
    const int B = totR - runR - (fl >> 16);        // right stops in (p, l)
    runL += fl & 0xffff;
    runR += fl >> 16;
    const bool lf = fl & 1, rf = fl >> 16;
    const int D = A - B;
    int rd = -1;
    if (lf && D < 0) {
      xk[g.l - 1 - A] = k[e]; xv[g.l - 1 - A] = vals[p];
      rd = g.f + A;
    } else if (rf && D > 0) {
      xk[g.f + B] = k[e]; xv[g.f + B] = vals[p];
      rd = g.l - 1 - B;
    }
    rds[p] = rd;
    if ((lf && D >= 0) || (rf && D > 0)) best = min(best, p);
  }
  for (int o = 32; o > 0; o >>= 1) best = min(best, __shfl_xor(best, o));
  if ((threadIdx.x & 63) == 0 && best != 0x7fffffff) atomicMin(&cut[s], best);
}

// grid (as k_vxs_count): swapped positions take their pair's element
__global__ __launch_bounds__(VXS_TPB) void k_vxs_readback(const VxsSeg* segs, const int* nseg, unsigned* keys,
                                                          unsigned* vals, const unsigned* xk, const unsigned* xv,
                                                          const int* rds, int maxch) {
  const int s = blockIdx.x / maxch, c = blockIdx.x % maxch;
  if (s >= *nseg) return;
  const VxsSeg g = segs[s];
  const int c0 = g.f + c * VXS_CH;
  if (c0 >= g.l) return;
  const int p0 = c0 + threadIdx.x * VXS_EPT;
#pragma unroll
  for (int e = 0; e < VXS_EPT; ++e) {
    const int p = p0 + e;
    if (p > g.f && p < g.l) {
      const int rd = rds[p];
      if (rd >= 0) { keys[p] = xk[rd]; vals[p] = xv[rd]; }
    }
  }
}

// grid (big ranges): the two sub-ranges [f, cut) and [cut, l) at depth d - 1: longer than VXS_SMALL into
// the next level's list (or, at depth 0, the heap-sort list), the others into the small list
__global__ __launch_bounds__(64) void k_vxs_split(const VxsSeg* segs, const int* nseg, const int* cut, VxsSeg* next,
                                                  int* nnext, VxsSeg* small, int* nsmall, VxsSeg* heap, int* nheap) {
  const int s = blockIdx.x * 64 + threadIdx.x;
  if (s >= *nseg) return;
  const VxsSeg g = segs[s];
  const int m = cut[s];
  const VxsSeg h[2] = {{g.f, m, g.d - 1}, {m, g.l, g.d - 1}};
  for (int i = 0; i < 2; ++i) {
    const int len = h[i].l - h[i].f;
    if (len <= VXS_SMALL) small[atomicAdd(nsmall, 1)] = h[i];
    else if (h[i].d == 0) heap[atomicAdd(nheap, 1)] = h[i];
    else next[atomicAdd(nnext, 1)] = h[i];
  }
}

// grid (clouds): every cloud's whole range, into the big (> VXS_SMALL) or small list at depth
// 2 floor(log2 n) (nothing for n <= 1 or an overflowed cloud)
__global__ __launch_bounds__(64) void k_vxs_init(const int* seg_b, const int* seg_e, int n_clouds, VxsSeg* big,
                                                 int* nbig, VxsSeg* small, int* nsmall) {
  const int c = blockIdx.x * 64 + threadIdx.x;
  if (c >= n_clouds) return;
  const int f = seg_b[c], l = seg_e[c], n = l - f;
  if (n <= 1) return;
  const VxsSeg g = {f, l, 2 * lg::floor_log2(n)};
  if (n <= VXS_SMALL) small[atomicAdd(nsmall, 1)] = g;
  else big[atomicAdd(nbig, 1)] = g;
}

// grid (small ranges): one wave each, the level-synchronous emulation from the range's depth limit in LDS
// (R = 16 for ranges of at most 1,024 positions, else 32: two kernels, each with its register budget)
// The point indices may exceed lvl_sort's 16-bit values: the sort carries range positions, and the
// indices follow through the scratch copy xv of the range.
// lvl_sort takes keys below 2^31 - 1.  k_vox_keys' leaf indices can reach that: PCL's overflow gate
// multiplies the truncated extents (hi - lo) / leaf + 1, the index uses floor(hi / leaf) - floor(lo / leaf)
// + 1 per axis, which can be one larger.  A range holding such a key sorts the number of its keys below
// each key instead (order- and tie-preserving, < 2,048), and the keys come back through the scratch xk.
template <int R>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(R == 32 ? 2 : 3)))
void k_vxs_small(const VxsSeg* segs, const int* nseg, unsigned* keys, unsigned* vals, unsigned* xk, unsigned* xv) {
  __shared__ lgws::VoxLvlLds<R> L;
  const int s = blockIdx.x;
  if (s >= *nseg) return;
  const VxsSeg g = segs[s];
  const int n = g.l - g.f;
  if ((n > 1024) != (R == 32) || n <= 1) return;
  unsigned big = 0u;
  for (int i = threadIdx.x; i < n; i += 64) {
    const unsigned k = keys[g.f + i];
    big |= k >= 0x7fffffffu ? 1u : 0u;
    L.u.nat.key[i] = k;
    L.u.nat.val[i] = (uint16_t)i;
    xv[g.f + i] = vals[g.f + i];
  }
  __syncthreads();
  const bool ranked = __ballot(big != 0u) != 0ull;
  if (ranked) {  // (pathological extents only) keys -> count of smaller keys, O(n^2 / 64) a lane
    for (int i = threadIdx.x; i < n; i += 64) xk[g.f + i] = L.u.nat.key[i];
    __syncthreads();
    for (int i0 = 0; i0 < n; i0 += 64) {
      const int i = i0 + (int)threadIdx.x;
      const unsigned k = i < n ? xk[g.f + i] : 0u;
      unsigned r = 0u;
      for (int j = 0; j < n; ++j) r += xk[g.f + j] < k ? 1u : 0u;
      if (i < n) L.u.nat.key[i] = r;
    }
    __syncthreads();
  }
  lgws::lvl_sort<R>(L.u.nat.key, L.u.nat.val, L.u.buf, n, g.d);
  for (int i = threadIdx.x; i < n; i += 64) {
    const int from = L.u.nat.val[i];
    keys[g.f + i] = ranked ? xk[g.f + from] : L.u.nat.key[i];
    vals[g.f + i] = xv[g.f + from];
  }
}

// grid (heap ranges): __partial_sort of a range longer than VXS_SMALL at depth 0, one wave, in HBM
__global__ __launch_bounds__(64) void k_vxs_heap(const VxsSeg* segs, const int* nseg, unsigned* keys,
                                                 unsigned* vals) {
  const int s = blockIdx.x;
  if (s >= *nseg) return;
  const VxsSeg g = segs[s];
  lgws::heap_sort_wave(lg::SortView<unsigned, unsigned>{keys, vals}, g.f, g.l);
}

}  // namespace

struct lego_s2m {
  int device = 0;
  int max_problems = 0, max_map = 0;
  int max_iters = 10;  // :1320; lego_test_s2m_debug lowers it
  int layout = -1;     // lego_s2m_set_layout: -1 automatic, 0 a workgroup a problem, 1 latency
  S2mState* d_state = nullptr;
  S2mScratch* d_scratch = nullptr;
  void* d_mem = nullptr;
  void* d_kd = nullptr;  // the problems' nanoflann trees (S2mScratch.kd_*)
  // host-call staging
  lego_point* d_clouds = nullptr;
  size_t cloud_cap = 0;
  int64_t* d_meta = nullptr;  // 4 offsets + 4 counts (int32 after the offsets) + transform/degenerate/info
  // VoxelGrid scratch, for vox_clouds clouds of up to max_map points: keys / values in and sorted, the
  // clouds' sort segments and overflow flags, rocprim's temporary storage
  int vox_clouds = 0;
  unsigned *d_keys = nullptr, *d_vals = nullptr, *d_keys2 = nullptr, *d_vals2 = nullptr;
  int *d_seg = nullptr, *d_ovf = nullptr;
  void* d_sort_tmp = nullptr;
  size_t sort_tmp_bytes = 0;
  // few-clouds layout (n * max_map <= S2M_WIDE_MAX): 64-bit keys in / sorted, values in / sorted
  unsigned long long *d_k64 = nullptr, *d_k64b = nullptr;
  unsigned *d_wv = nullptr, *d_wv2 = nullptr;
  int *d_wseg = nullptr, *d_wovf = nullptr, *d_wbounds = nullptr, *d_wtcount = nullptr;
  void* d_wide_tmp = nullptr;
  size_t wide_tmp_bytes = 0;
  int wide_clouds = 0;
  // voxel_tie_order 0 (PCL's std::sort order, the reference): the level-synchronous emulation's scratch
  // for vxs_clouds clouds: exchange slots, read-back slots, range lists and their counters
  int voxel_tie_order = 0;
  int vxs_clouds = 0;
  unsigned *d_xk = nullptr, *d_xv = nullptr, *d_pivot = nullptr;
  int *d_rds = nullptr, *d_cut = nullptr, *d_cnt = nullptr, *d_ctr = nullptr, *h_ctr = nullptr;
  VxsSeg *d_big = nullptr, *d_next = nullptr, *d_small = nullptr, *d_heap = nullptr;
  int cap_big = 0, cap_small = 0, vxs_maxch = 0;
};

// The LM's per-problem scratch (bucket tables, bucketed points, rows, nanoflann trees: ~200 B a map
// point) is allocated on the first lego_s2m_run, so an engine used only for lego_map_transform /
// lego_map_voxel (the mapper's VoxelGrid engine) never holds it.
static int s2m_alloc_lm(lego_s2m* m) {
  if (m->d_scratch) return LEGO_OK;
  const int max_problems = m->max_problems, max_map_points = m->max_map;
  // per problem and map cloud: bucket table, points, indices
  const size_t tab = (size_t)(S2M_NB_MAX + 1) * 4, pts = (size_t)max_map_points * 16, idx = (size_t)max_map_points * 4;
  const size_t rows = (size_t)max_map_points * 32;
  const size_t per = ((tab + 255) & ~(size_t)255) + pts + ((idx + 255) & ~(size_t)255) + rows;
  // per problem: each cloud's tree nodes and index permutation, then the shared stop lists, stacks and
  // tied-query list (every size a multiple of 256 bytes)
  const size_t mp = ((size_t)max_map_points + 63) & ~(size_t)63;
  const size_t kd_node = 2 * mp * sizeof(KdNode), kd_vind = mp * 4, kd_tmp = 2 * mp * 4, kd_frames = (10 * mp + S2M_KD_STACK) * 4,
               tieq = mp * 4;
  const size_t kd_per = 2 * (kd_node + kd_vind) + kd_tmp + kd_frames + tieq;
  // into locals: m keeps nothing of a partial failure (the next call allocates again from scratch)
  S2mScratch* d_scratch = nullptr;
  void *d_mem = nullptr, *d_kd = nullptr;
  auto fail = [&](int rc) {
    if (d_scratch) hipFree(d_scratch);
    if (d_kd) hipFree(d_kd);
    if (d_mem) hipFree(d_mem);
    return rc;
  };
  if (hipMalloc(&d_mem, per * 2 * max_problems) != hipSuccess || hipMalloc(&d_kd, kd_per * max_problems) != hipSuccess ||
      hipMalloc((void**)&d_scratch, sizeof(S2mScratch) * 2 * max_problems) != hipSuccess)
    return fail(LEGO_ENOMEM);
  S2mScratch* h = new (std::nothrow) S2mScratch[2 * max_problems];
  if (!h) return fail(LEGO_ENOMEM);
  char* base = (char*)d_mem;
  for (int k = 0; k < 2 * max_problems; ++k) {
    char* b = base + per * k;
    h[k].start = (int*)b;
    h[k].pts = (float4*)(b + ((tab + 255) & ~(size_t)255));
    h[k].idx = (int*)(b + ((tab + 255) & ~(size_t)255) + pts);
    h[k].rows = (float4*)(b + ((tab + 255) & ~(size_t)255) + pts + ((idx + 255) & ~(size_t)255));
    char* kb = (char*)d_kd + kd_per * (k / 2);
    h[k].kd_node = (KdNode*)(kb + (k % 2) * (kd_node + kd_vind));
    h[k].kd_vind = (int*)(kb + (k % 2) * (kd_node + kd_vind) + kd_node);
    h[k].kd_tmp = (int*)(kb + 2 * (kd_node + kd_vind));
    h[k].kd_frames = (float*)(kb + 2 * (kd_node + kd_vind) + kd_tmp);
    h[k].tieq = (int*)(kb + 2 * (kd_node + kd_vind) + kd_tmp + kd_frames);
  }
  const bool ok = hipMemcpy(d_scratch, h, sizeof(S2mScratch) * 2 * max_problems, hipMemcpyHostToDevice) == hipSuccess;
  delete[] h;
  if (!ok) return fail(LEGO_EDEVICE);
  m->d_mem = d_mem;
  m->d_kd = d_kd;
  m->d_scratch = d_scratch;
  return LEGO_OK;
}

extern "C" int lego_s2m_create(int32_t device, int32_t max_problems, int32_t max_map_points, lego_s2m** out) {
  if (!out) return LEGO_EINVAL;
  *out = nullptr;
  if (max_problems < 1 || max_map_points < 1 || max_map_points > LEGO_MAX_POINTS) return LEGO_EINVAL;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return LEGO_EDEVICE;
  if (hipSetDevice(device) != hipSuccess) return LEGO_EDEVICE;
  lego_s2m* m = new (std::nothrow) lego_s2m();
  if (!m) return LEGO_ENOMEM;
  m->device = device;
  m->max_problems = max_problems;
  m->max_map = max_map_points;
  if (hipMalloc((void**)&m->d_meta, 256) != hipSuccess ||
      hipMalloc((void**)&m->d_state, sizeof(S2mState) * max_problems) != hipSuccess) {
    lego_s2m_destroy(m);
    return LEGO_ENOMEM;
  }
  *out = m;
  return LEGO_OK;
}

extern "C" void lego_s2m_destroy(lego_s2m* m) {
  if (!m) return;
  hipSetDevice(m->device);
  hipDeviceSynchronize();
  if (m->d_mem) hipFree(m->d_mem);
  if (m->d_kd) hipFree(m->d_kd);
  if (m->d_scratch) hipFree(m->d_scratch);
  if (m->d_clouds) hipFree(m->d_clouds);
  if (m->d_meta) hipFree(m->d_meta);
  if (m->d_state) hipFree(m->d_state);
  for (void* p : {(void*)m->d_keys, (void*)m->d_vals, (void*)m->d_keys2, (void*)m->d_vals2, (void*)m->d_seg,
                  (void*)m->d_ovf, m->d_sort_tmp, (void*)m->d_k64, (void*)m->d_k64b, (void*)m->d_wv, (void*)m->d_wv2,
                  (void*)m->d_wseg, (void*)m->d_wovf, (void*)m->d_wbounds, (void*)m->d_wtcount, m->d_wide_tmp,
                  (void*)m->d_xk, (void*)m->d_xv, (void*)m->d_pivot, (void*)m->d_rds, (void*)m->d_cut, (void*)m->d_cnt,
                  (void*)m->d_ctr, (void*)m->d_big, (void*)m->d_next, (void*)m->d_small, (void*)m->d_heap})
    if (p) hipFree(p);
  if (m->h_ctr) hipHostFree(m->h_ctr);
  delete m;
}

extern "C" int lego_s2m_run(lego_s2m* m, int32_t n, const lego_s2m_io* io, void* hip_stream) {
  if (!m || !io || n < 1 || n > m->max_problems) return LEGO_EINVAL;
  if (!io->corner || !io->corner_off || !io->corner_n || !io->surf || !io->surf_off || !io->surf_n ||
      !io->corner_map || !io->corner_map_off || !io->corner_map_n || !io->surf_map || !io->surf_map_off ||
      !io->surf_map_n || !io->transform || !io->degenerate || !io->info)
    return LEGO_EINVAL;
  if (hipSetDevice(m->device) != hipSuccess) return LEGO_EDEVICE;
  if (const int rc = s2m_alloc_lm(m)) return rc;
  hipStream_t st = (hipStream_t)hip_stream;
  const bool lat = m->layout == 1 || (m->layout < 0 && n <= S2M_LATENCY_MAX);
  if (!lat) {
    hipLaunchKernelGGL(k_s2m, dim3(n), dim3(S2M_THREADS), 0, st, *io, m->d_scratch, m->max_map, m->max_iters);
    return hipGetLastError() == hipSuccess ? LEGO_OK : LEGO_EDEVICE;
  }
  // latency layout: enough row workgroups for one query a lane at the largest query count allowed
  const int g = std::max(1, std::min((m->max_map + S2M_THREADS - 1) / S2M_THREADS, std::max(1, 256 / n)));
  hipLaunchKernelGGL(k_s2m_grid, dim3(2, n), dim3(S2M_THREADS), 0, st, *io, m->d_scratch, m->d_state, m->max_map);
  for (int it = 0; it < m->max_iters; ++it) {
    hipLaunchKernelGGL(k_s2m_rows, dim3(g, n), dim3(S2M_THREADS), 0, st, *io, m->d_scratch, m->d_state);
    hipLaunchKernelGGL(k_s2m_solve, dim3(n), dim3(S2M_THREADS), 0, st, *io, m->d_scratch, m->d_state, it, m->max_iters,
                       m->max_map);
  }
  return hipGetLastError() == hipSuccess ? LEGO_OK : LEGO_EDEVICE;
}

extern "C" int lego_s2m_run_host(lego_s2m* m, const lego_point* corner, int32_t n_corner, const lego_point* surf,
                                 int32_t n_surf, const lego_point* corner_map, int32_t n_corner_map,
                                 const lego_point* surf_map, int32_t n_surf_map, float* transform, int32_t* degenerate,
                                 int32_t* info) {
  if (!m || !transform || !degenerate || !info || n_corner < 0 || n_surf < 0 || n_corner_map < 0 || n_surf_map < 0 ||
      (n_corner && !corner) || (n_surf && !surf) || (n_corner_map && !corner_map) || (n_surf_map && !surf_map))
    return LEGO_EINVAL;
  if (hipSetDevice(m->device) != hipSuccess) return LEGO_EDEVICE;
  const size_t total = (size_t)n_corner + n_surf + n_corner_map + n_surf_map;
  if (total > m->cloud_cap) {
    if (m->d_clouds) hipFree(m->d_clouds);
    m->d_clouds = nullptr;
    m->cloud_cap = 0;
    if (hipMalloc((void**)&m->d_clouds, (total ? total : 1) * sizeof(lego_point)) != hipSuccess) return LEGO_ENOMEM;
    m->cloud_cap = total;
  }
  const lego_point* src[4] = {corner, surf, corner_map, surf_map};
  const int32_t cnt[4] = {n_corner, n_surf, n_corner_map, n_surf_map};
  // meta: off[4] (int64), cnt[4] (int32), transform[6] (float), degenerate (int32), info[4] (int32)
  struct Meta { int64_t off[4]; int32_t n[4]; float t[6]; int32_t dg; int32_t info[4]; } h;
  int64_t o = 0;
  for (int k = 0; k < 4; ++k) {
    h.off[k] = o;
    h.n[k] = cnt[k];
    if (cnt[k] && hipMemcpy(m->d_clouds + o, src[k], (size_t)cnt[k] * sizeof(lego_point), hipMemcpyHostToDevice) != hipSuccess)
      return LEGO_EDEVICE;
    o += cnt[k];
  }
  for (int k = 0; k < 6; ++k) h.t[k] = transform[k];
  h.dg = *degenerate;
  for (int k = 0; k < 4; ++k) h.info[k] = 0;
  if (hipMemcpy(m->d_meta, &h, sizeof(h), hipMemcpyHostToDevice) != hipSuccess) return LEGO_EDEVICE;
  Meta* dm = (Meta*)m->d_meta;
  lego_s2m_io io;
  io.corner = m->d_clouds; io.corner_off = &dm->off[0]; io.corner_n = &dm->n[0];
  io.surf = m->d_clouds; io.surf_off = &dm->off[1]; io.surf_n = &dm->n[1];
  io.corner_map = m->d_clouds; io.corner_map_off = &dm->off[2]; io.corner_map_n = &dm->n[2];
  io.surf_map = m->d_clouds; io.surf_map_off = &dm->off[3]; io.surf_map_n = &dm->n[3];
  io.transform = dm->t;
  io.degenerate = &dm->dg;
  io.info = dm->info;
  int rc = lego_s2m_run(m, 1, &io, nullptr);
  if (rc) return rc;
  if (hipMemcpy(&h, m->d_meta, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return LEGO_EDEVICE;
  for (int k = 0; k < 6; ++k) transform[k] = h.t[k];
  *degenerate = h.dg;
  for (int k = 0; k < 4; ++k) info[k] = h.info[k];
  return LEGO_OK;
}

extern "C" int lego_map_transform(lego_s2m* m, int32_t n, const lego_map_transform_io* io, void* hip_stream) {
  if (!m || !io || n < 1 || !io->in || !io->in_off || !io->in_n || !io->pose || !io->out || !io->out_off)
    return LEGO_EINVAL;
  if (hipSetDevice(m->device) != hipSuccess) return LEGO_EDEVICE;
  hipLaunchKernelGGL(k_map_transform, dim3(16, n), dim3(256), 0, (hipStream_t)hip_stream, *io);
  return hipGetLastError() == hipSuccess ? LEGO_OK : LEGO_EDEVICE;
}

static int ensure_vox_scratch(lego_s2m* m, int n);
static int map_voxel_std_order(lego_s2m* m, int n, const lego_map_voxel_io* io, hipStream_t st);

extern "C" int lego_s2m_set_voxel_tie_order(lego_s2m* m, int32_t order) {
  if (!m || order < 0 || order > 1) return LEGO_EINVAL;
  m->voxel_tie_order = order;
  return LEGO_OK;
}

extern "C" int lego_map_voxel(lego_s2m* m, int32_t n, const lego_map_voxel_io* io, void* hip_stream) {
  if (!m || !io || n < 1 || !io->in || !io->in_off || !io->in_n || !io->leaf ||
      !io->out || !io->out_off || !io->out_n || !io->status)
    return LEGO_EINVAL;
  if (hipSetDevice(m->device) != hipSuccess) return LEGO_EDEVICE;
  const int cap = m->max_map;
  hipStream_t st = (hipStream_t)hip_stream;
  if (m->voxel_tie_order == 0) return map_voxel_std_order(m, n, io, st);
  if ((size_t)n * cap <= S2M_WIDE_MAX && n < 64) {
    // few clouds (the mapping thread's five): the tiled kernels and one device-wide stable radix sort
    // over the clouds' points (their counts read back first: this path synchronizes the stream)
    const int tiles_max = (cap + S2M_THREADS - 1) / S2M_THREADS;
    if (n > m->wide_clouds) {
      const size_t e = (size_t)n * cap;
      size_t tmp = 0;
      if (rocprim::radix_sort_pairs((void*)nullptr, tmp, (unsigned long long*)nullptr, (unsigned long long*)nullptr,
                                    (unsigned*)nullptr, (unsigned*)nullptr, e, 0, 38) != hipSuccess)
        return LEGO_EDEVICE;
      hipDeviceSynchronize();
      for (void* p : {(void*)m->d_k64, (void*)m->d_k64b, (void*)m->d_wv, (void*)m->d_wv2, (void*)m->d_wseg,
                      (void*)m->d_wovf, (void*)m->d_wbounds, (void*)m->d_wtcount, m->d_wide_tmp})
        if (p) hipFree(p);
      m->d_k64 = m->d_k64b = nullptr;
      m->d_wv = m->d_wv2 = nullptr;
      m->d_wseg = m->d_wovf = m->d_wbounds = m->d_wtcount = nullptr;
      m->d_wide_tmp = nullptr;
      m->wide_clouds = 0;
      if (hipMalloc((void**)&m->d_k64, e * 8) != hipSuccess || hipMalloc((void**)&m->d_k64b, e * 8) != hipSuccess ||
          hipMalloc((void**)&m->d_wv, e * 4) != hipSuccess || hipMalloc((void**)&m->d_wv2, e * 4) != hipSuccess ||
          hipMalloc((void**)&m->d_wseg, (size_t)n * 2 * 4) != hipSuccess ||
          hipMalloc((void**)&m->d_wovf, (size_t)n * 4) != hipSuccess ||
          hipMalloc((void**)&m->d_wbounds, (size_t)n * 6 * 4) != hipSuccess ||
          hipMalloc((void**)&m->d_wtcount, (size_t)n * tiles_max * 4) != hipSuccess ||
          hipMalloc(&m->d_wide_tmp, tmp) != hipSuccess)
        return LEGO_ENOMEM;
      m->wide_tmp_bytes = tmp;
      m->wide_clouds = n;
    }
    int32_t hn[64];
    if (hipMemcpyAsync(hn, io->in_n, (size_t)n * 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
      return LEGO_EDEVICE;
    size_t total = 0;
    int tiles = 1;
    for (int c = 0; c < n; ++c) {
      const int k = (hn[c] < 0 || hn[c] > cap) ? 0 : hn[c];
      total += (size_t)k;
      tiles = std::max(tiles, (k + S2M_THREADS - 1) / S2M_THREADS);
    }
    int* wb = m->d_wseg;
    int* we = m->d_wseg + m->wide_clouds;
    if (hipMemsetD32Async((hipDeviceptr_t)m->d_wbounds, 0x7fffffff, (size_t)n * 6, st) != hipSuccess)
      return LEGO_EDEVICE;
    hipLaunchKernelGGL(k_vxf_bounds, dim3(tiles, n), dim3(S2M_THREADS), 0, st, *io, m->d_wbounds, cap);
    hipLaunchKernelGGL(k_vxf_keys, dim3(tiles, n), dim3(S2M_THREADS), 0, st, *io, (const int*)m->d_wbounds, m->d_k64,
                       m->d_wv, wb, we, m->d_wovf, cap, n);
    if (hipGetLastError() != hipSuccess) return LEGO_EDEVICE;
    int bits = 32;
    while ((1 << (bits - 32)) <= n) ++bits;  // the cloud index and the overflowed clouds' n
    if (total > 0) {
      size_t tmp = m->wide_tmp_bytes;
      if (rocprim::radix_sort_pairs(m->d_wide_tmp, tmp, m->d_k64, m->d_k64b, m->d_wv, m->d_wv2, total, 0, bits, st) !=
          hipSuccess)
        return LEGO_EDEVICE;
    }
    hipLaunchKernelGGL(k_vxf_heads, dim3(tiles, n), dim3(S2M_THREADS), 0, st, (const unsigned long long*)m->d_k64b,
                       (const int*)wb, (const int*)we, m->d_wtcount, tiles);
    hipLaunchKernelGGL(k_vxf_emit, dim3(tiles, n), dim3(S2M_THREADS), 0, st, *io, (const unsigned long long*)m->d_k64b,
                       (const unsigned*)m->d_wv2, (const int*)wb, (const int*)we, (const int*)m->d_wovf,
                       (const int*)m->d_wtcount, tiles);
    return hipGetLastError() == hipSuccess ? LEGO_OK : LEGO_EDEVICE;
  }
  const int rc = ensure_vox_scratch(m, n);
  if (rc) return rc;
  int* seg_b = m->d_seg;
  int* seg_e = m->d_seg + m->vox_clouds;
  hipLaunchKernelGGL(k_vox_keys, dim3(n), dim3(S2M_THREADS), 0, st, *io, m->d_keys, m->d_vals, seg_b, seg_e, m->d_ovf,
                     cap);
  if (hipGetLastError() != hipSuccess) return LEGO_EDEVICE;
  // stable LSD radix sort of every cloud's (leaf index, point index) pairs: std::stable_sort's order
  size_t tmp = m->sort_tmp_bytes;
  if (rocprim::segmented_radix_sort_pairs(m->d_sort_tmp, tmp, m->d_keys, m->d_keys2, m->d_vals, m->d_vals2,
                                          (unsigned)((size_t)n * cap), (unsigned)n, seg_b, seg_e, 0, 32, st) !=
      hipSuccess)
    return LEGO_EDEVICE;
  hipLaunchKernelGGL(k_vox_reduce, dim3(n), dim3(S2M_THREADS), 0, st, *io, m->d_keys2, m->d_vals2, m->d_ovf, cap);
  return hipGetLastError() == hipSuccess ? LEGO_OK : LEGO_EDEVICE;
}

// scratch for n clouds of up to max_map_points: keys / values in and sorted, segments, overflow flags,
// rocPRIM's temporary storage (grows, never shrinks)
static int ensure_vox_scratch(lego_s2m* m, int n) {
  const int cap = m->max_map;
  if (n > m->vox_clouds) {
    const int nc = n;
    const size_t e = (size_t)nc * cap;
    if (e >= (1ull << 32)) return LEGO_EINVAL;
    size_t tmp = 0;
    if (rocprim::segmented_radix_sort_pairs((void*)nullptr, tmp, (unsigned*)nullptr, (unsigned*)nullptr,
                                            (unsigned*)nullptr, (unsigned*)nullptr, (unsigned)e, (unsigned)nc,
                                            (int*)nullptr, (int*)nullptr, 0, 32) != hipSuccess)
      return LEGO_EDEVICE;
    hipDeviceSynchronize();  // earlier calls may still use the old scratch
    for (void* p : {(void*)m->d_keys, (void*)m->d_vals, (void*)m->d_keys2, (void*)m->d_vals2, (void*)m->d_seg,
                    (void*)m->d_ovf, m->d_sort_tmp})
      if (p) hipFree(p);
    m->d_keys = m->d_vals = m->d_keys2 = m->d_vals2 = nullptr;
    m->d_seg = m->d_ovf = nullptr;
    m->d_sort_tmp = nullptr;
    m->vox_clouds = 0;
    if (hipMalloc((void**)&m->d_keys, e * 4) != hipSuccess || hipMalloc((void**)&m->d_vals, e * 4) != hipSuccess ||
        hipMalloc((void**)&m->d_keys2, e * 4) != hipSuccess || hipMalloc((void**)&m->d_vals2, e * 4) != hipSuccess ||
        hipMalloc((void**)&m->d_seg, (size_t)nc * 2 * 4) != hipSuccess ||
        hipMalloc((void**)&m->d_ovf, (size_t)nc * 4) != hipSuccess || hipMalloc(&m->d_sort_tmp, tmp) != hipSuccess)
      return LEGO_ENOMEM;
    m->sort_tmp_bytes = tmp;
    m->vox_clouds = nc;
  }
  return LEGO_OK;
}

// PCL's std::sort order (voxel_tie_order 0): k_vox_keys, the level-synchronous introsort emulation in place
// (device-wide levels while ranges exceed VXS_SMALL, then one wave a range), k_vox_reduce.  Synchronizes
// the stream once per device-wide level (the count of ranges still longer than VXS_SMALL).
static int map_voxel_std_order(lego_s2m* m, int n, const lego_map_voxel_io* io, hipStream_t st) {
  int rc = ensure_vox_scratch(m, n);
  if (rc) return rc;
  const int cap = m->max_map;
  const size_t e = (size_t)n * cap;
  if (n > m->vxs_clouds) {
    hipDeviceSynchronize();  // earlier calls may still use the old scratch
    for (void* p : {(void*)m->d_xk, (void*)m->d_xv, (void*)m->d_pivot, (void*)m->d_rds, (void*)m->d_cut,
                    (void*)m->d_cnt, (void*)m->d_ctr, (void*)m->d_big, (void*)m->d_next, (void*)m->d_small,
                    (void*)m->d_heap})
      if (p) hipFree(p);
    m->d_xk = m->d_xv = m->d_pivot = nullptr;
    m->d_rds = m->d_cut = m->d_cnt = m->d_ctr = nullptr;
    m->d_big = m->d_next = m->d_small = m->d_heap = nullptr;
    m->vxs_clouds = 0;
    m->cap_big = (int)(e / VXS_SMALL) + n + 16;    // ranges longer than VXS_SMALL at one level
    m->cap_small = (int)(e / 16) + 2 * n + 16;     // every finished range (> 16 positions but the last ones)
    m->vxs_maxch = (cap + VXS_CH - 1) / VXS_CH;
    if (hipMalloc((void**)&m->d_xk, e * 4) != hipSuccess || hipMalloc((void**)&m->d_xv, e * 4) != hipSuccess ||
        hipMalloc((void**)&m->d_rds, e * 4) != hipSuccess ||
        hipMalloc((void**)&m->d_pivot, (size_t)m->cap_big * 4) != hipSuccess ||
        hipMalloc((void**)&m->d_cut, (size_t)m->cap_big * 4) != hipSuccess ||
        hipMalloc((void**)&m->d_cnt, (size_t)m->cap_big * m->vxs_maxch * 4) != hipSuccess ||
        hipMalloc((void**)&m->d_ctr, 64) != hipSuccess ||
        hipMalloc((void**)&m->d_big, (size_t)m->cap_big * sizeof(VxsSeg)) != hipSuccess ||
        hipMalloc((void**)&m->d_next, (size_t)m->cap_big * sizeof(VxsSeg)) != hipSuccess ||
        hipMalloc((void**)&m->d_heap, (size_t)m->cap_big * sizeof(VxsSeg)) != hipSuccess ||
        hipMalloc((void**)&m->d_small, (size_t)m->cap_small * sizeof(VxsSeg)) != hipSuccess)
      return LEGO_ENOMEM;
    if (!m->h_ctr && hipHostMalloc((void**)&m->h_ctr, 64) != hipSuccess) return LEGO_ENOMEM;
    m->vxs_clouds = n;
  }
  int* seg_b = m->d_seg;
  int* seg_e = m->d_seg + m->vox_clouds;
  int* ctr = m->d_ctr;  // [0] big ranges, [1] next level's, [2] small, [3] heap-sort
  if (hipMemsetAsync(ctr, 0, 16, st) != hipSuccess) return LEGO_EDEVICE;
  hipLaunchKernelGGL(k_vox_keys, dim3(n), dim3(S2M_THREADS), 0, st, *io, m->d_keys, m->d_vals, seg_b, seg_e, m->d_ovf,
                     cap);
  hipLaunchKernelGGL(k_vxs_init, dim3((n + 63) / 64), dim3(64), 0, st, (const int*)seg_b, (const int*)seg_e, n,
                     m->d_big, ctr, m->d_small, ctr + 2);
  if (hipGetLastError() != hipSuccess) return LEGO_EDEVICE;
  VxsSeg *cur = m->d_big, *nxt = m->d_next;
  for (int level = 0;; ++level) {
    if (hipMemcpyAsync(m->h_ctr, ctr, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
      return LEGO_EDEVICE;
    const int nbig = m->h_ctr[0];
    if (nbig == 0) break;
    if (nbig > m->cap_big || level > 64) return LEGO_EDEVICE;  // (bounded by construction)
    const int g64 = (nbig + 63) / 64;
    // one chunk block per (range, chunk of the longest possible range): vxs_maxch comes from the largest
    // cloud, so the grid grows with nbig * max_map; HIP needs gridDim.x * blockDim.x < 2^32
    const size_t nblk = (size_t)m->vxs_maxch * (size_t)nbig;
    if (nblk * VXS_TPB >= (1ull << 32)) return LEGO_EINVAL;
    const dim3 gch((unsigned)nblk);
    if (hipMemsetAsync(ctr + 1, 0, 4, st) != hipSuccess) return LEGO_EDEVICE;
    hipLaunchKernelGGL(k_vxs_median, dim3(g64), dim3(64), 0, st, (const VxsSeg*)cur, (const int*)ctr, m->d_keys,
                       m->d_vals, m->d_pivot, m->d_cut);
    hipLaunchKernelGGL(k_vxs_count, gch, dim3(VXS_TPB), 0, st, (const VxsSeg*)cur, (const int*)ctr,
                       (const unsigned*)m->d_keys, (const unsigned*)m->d_pivot, m->d_cnt, m->vxs_maxch);
    hipLaunchKernelGGL(k_vxs_exchange, gch, dim3(VXS_TPB), 0, st, (const VxsSeg*)cur, (const int*)ctr,
                       (const unsigned*)m->d_keys, (const unsigned*)m->d_vals, (const unsigned*)m->d_pivot,
                       (const int*)m->d_cnt, m->vxs_maxch, m->d_xk, m->d_xv, m->d_rds, m->d_cut);
    hipLaunchKernelGGL(k_vxs_readback, gch, dim3(VXS_TPB), 0, st, (const VxsSeg*)cur, (const int*)ctr, m->d_keys,
                       m->d_vals, (const unsigned*)m->d_xk, (const unsigned*)m->d_xv, (const int*)m->d_rds,
                       m->vxs_maxch);
    hipLaunchKernelGGL(k_vxs_split, dim3(g64), dim3(64), 0, st, (const VxsSeg*)cur, (const int*)ctr,
                       (const int*)m->d_cut, nxt, ctr + 1, m->d_small, ctr + 2, m->d_heap, ctr + 3);
    if (hipGetLastError() != hipSuccess) return LEGO_EDEVICE;
    std::swap(cur, nxt);
    if (hipMemcpyAsync(ctr, ctr + 1, 4, hipMemcpyDeviceToDevice, st) != hipSuccess) return LEGO_EDEVICE;
  }
  if (hipMemcpyAsync(m->h_ctr, ctr, 16, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return LEGO_EDEVICE;
  const int nsmall = m->h_ctr[2], nheap = m->h_ctr[3];
  if (nsmall > m->cap_small || nheap > m->cap_big) return LEGO_EDEVICE;
  if (nsmall > 0) {
    hipLaunchKernelGGL(k_vxs_small<16>, dim3(nsmall), dim3(64), 0, st, (const VxsSeg*)m->d_small, (const int*)(ctr + 2),
                       m->d_keys, m->d_vals, m->d_xk, m->d_xv);
    hipLaunchKernelGGL(k_vxs_small<32>, dim3(nsmall), dim3(64), 0, st, (const VxsSeg*)m->d_small, (const int*)(ctr + 2),
                       m->d_keys, m->d_vals, m->d_xk, m->d_xv);
  }
  if (nheap > 0)
    hipLaunchKernelGGL(k_vxs_heap, dim3(nheap), dim3(64), 0, st, (const VxsSeg*)m->d_heap, (const int*)(ctr + 3),
                       m->d_keys, m->d_vals);
  hipLaunchKernelGGL(k_vox_reduce, dim3(n), dim3(S2M_THREADS), 0, st, *io, (const unsigned*)m->d_keys,
                     (const unsigned*)m->d_vals, m->d_ovf, cap);
  return hipGetLastError() == hipSuccess ? LEGO_OK : LEGO_EDEVICE;
}

// test hook: the LM iteration cap (10 in the product), and the LM rows of problem p's last iteration
// (per query: arx, ary, arz, coeff.x, coeff.y, coeff.z, -coeff.intensity, selected) into out[8 * nq]
extern "C" int lego_test_s2m_debug(lego_s2m* m, int32_t max_iters, int32_t p, int32_t nq, float* out) {
  if (!m || max_iters < 1 || max_iters > 10 || p < 0 || p >= m->max_problems || nq < 0 || nq > m->max_map ||
      (nq && !out))
    return LEGO_EINVAL;
  m->max_iters = max_iters;
  if (!nq) return LEGO_OK;
  if (hipSetDevice(m->device) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return LEGO_EDEVICE;
  if (!m->d_scratch) return LEGO_EINVAL;  // no lego_s2m_run yet: no rows
  S2mScratch g;
  if (hipMemcpy(&g, m->d_scratch + 2 * p, sizeof(g), hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(out, g.rows, (size_t)nq * 32, hipMemcpyDeviceToHost) != hipSuccess)
    return LEGO_EDEVICE;
  return LEGO_OK;
}

extern "C" int lego_s2m_set_layout(lego_s2m* m, int32_t layout) {
  if (!m || layout < -1 || layout > 1) return LEGO_EINVAL;
  m->layout = layout;
  return LEGO_OK;
}

