// s2m_oracle.cpp — CPU restatement of MapOptimization::scan2MapOptimization (the scan-to-map LM).
//
// TEST INFRASTRUCTURE ONLY.  Parity oracle for the MI355X product path (lego-loam-bor_amd/csrc/
// lego_s2m.hip): loaded by tests/ and tools/bench_s2m.py (as the checker / the CPU baseline), never
// by the product.
//
// Restates /root/reference/LeGO-LOAM/src/mapOptmization.cpp:1028-1332 (citations are file:line into
// that file) with the reference's expression types: float members, double literals (0.1, 0.9, 1.0,
// 0.05), unqualified libm calls on floats resolving to the float overloads (fp_mode 0, SURVEY App.
// A.1).  Built -O3 -ffp-contract=off without -march, as the reference (LeGO-LOAM/CMakeLists.txt:4).
//
// PARITY STATUS:
//   * kNN-5 (nanoflann nearestKSearch(k = 5), :1033, :1141): the 5 nearest by (distance, index) from an
//     exact search of the 1 m ball (only the 5th distance < 1.0 is ever used, :1036, :1144); when any
//     of the 6 nearest distances are equal, nanoflann's own answer from its restated tree
//     (nanoflann_restated.h, built on the first such query of a map).  oracle/_ref/nanoflann_pin (the
//     reference's vendored nanoflann 1.3.0) pins both: test_knn5_pin_nanoflann, test_nanoflann_pin.
//   * Eigen (absent here, unpinned; ROS Melodic's Eigen 3.3.4 restated):
//       SelfAdjointEigenSolver<Matrix3f> (:1077): scaling, the 3x3 Householder tridiagonalisation,
//         implicit symmetric QR with Wilkinson shifts, ascending sort with column swaps.  The
//         eigenvector signs matter: the reference reads matV1(0, j) (:1086-1091), the first
//         component of each eigenvector;
//       ColPivHouseholderQR<Matrix<float,5,3>> / <Matrix<float,6,6>> (:1153, :1260): restated in
//         float with sequential sums;
//       matAt * matA (:1258): float products summed in double, rounded to float (the FA LM's model),
//         in the product's fixed summation order (see lm_step);
//       SelfAdjointEigenSolver<Matrix<float,6,6>> (:1267): only "largest eigenvalue < 100" is used
//         (the ascending order makes :1275-1284 zero every row exactly then), by cyclic Jacobi in
//         double.
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <unordered_map>
#include <vector>

#include "../include/lego_s2m.h"
#include "nanoflann_restated.h"

extern int g_float_ne;  // lego_oracle.cpp (oracle_set_float_normal_equations)

namespace s2m {

struct Pt { float x, y, z, i; };

// ---- Eigen 3.3.4 SelfAdjointEigenSolver<Matrix3f>::compute, restated ------------------------------
// A: symmetric 3x3 (row-major, only the lower triangle is read).  evals ascending; V column j is the
// eigenvector of evals[j] (V[r * 3 + j]).
static float hypot_e(float x, float y) {  // Eigen's positive_real_hypot
  const float ax = std::fabs(x), ay = std::fabs(y);
  float p, qp;
  if (ax > ay) { p = ax; qp = ay / p; }
  else { p = ay; qp = ax / p; }
  if (p == 0.f) return 0.f;
  return p * std::sqrt(1.f + qp * qp);
}

static void givens(float p, float q, float& c, float& s) {  // JacobiRotation::makeGivens (real)
  if (q == 0.f) {
    c = p < 0.f ? -1.f : 1.f;
    s = 0.f;
  } else if (p == 0.f) {
    c = 0.f;
    s = q < 0.f ? 1.f : -1.f;
  } else if (std::fabs(p) > std::fabs(q)) {
    const float t = q / p;
    float u = std::sqrt(1.f + t * t);
    if (p < 0.f) u = -u;
    c = 1.f / u;
    s = -t * c;
  } else {
    const float t = p / q;
    float u = std::sqrt(1.f + t * t);
    if (q < 0.f) u = -u;
    s = -1.f / u;
    c = -t * s;
  }
}

void eig3(const float A[9], float evals[3], float V[9]) {
  float m[9] = {A[0], 0.f, 0.f, A[3], A[4], 0.f, A[6], A[7], A[8]};  // triangularView<Lower>
  float scale = 0.f;
  for (int k = 0; k < 9; ++k) scale = std::max(scale, std::fabs(m[k]));
  if (scale == 0.f) scale = 1.f;
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c <= r; ++c) m[r * 3 + c] /= scale;
  // tridiagonalization_inplace_selector<MatrixType, 3, false>::run
  float d[3], e[2];
  d[0] = m[0];
  const float v1norm2 = m[6] * m[6];
  if (v1norm2 <= FLT_MIN) {
    d[1] = m[4];
    d[2] = m[8];
    e[0] = m[3];
    e[1] = m[7];
    const float I[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    std::memcpy(V, I, sizeof(I));
  } else {
    const float beta = std::sqrt(m[3] * m[3] + v1norm2);
    const float invBeta = 1.f / beta;
    const float m01 = m[3] * invBeta;
    const float m02 = m[6] * invBeta;
    const float q = 2.f * m01 * m[7] + m02 * (m[8] - m[4]);
    d[1] = m[4] + m02 * q;
    d[2] = m[8] - m02 * q;
    e[0] = beta;
    e[1] = m[7] - m01 * q;
    const float Q[9] = {1, 0, 0, 0, m01, m02, 0, m02, -m01};
    std::memcpy(V, Q, sizeof(Q));
  }
  // computeFromTridiagonal_impl (maxIterations 30)
  const int n = 3;
  int end = n - 1, start = 0, iter = 0;
  const float precision = 2.f * FLT_EPSILON;
  bool ok = true;
  while (end > 0) {
    for (int i = start; i < end; ++i)
      if (std::fabs(e[i]) <= (std::fabs(d[i]) + std::fabs(d[i + 1])) * precision || std::fabs(e[i]) <= FLT_MIN)
        e[i] = 0.f;
    while (end > 0 && e[end - 1] == 0.f) end--;
    if (end <= 0) break;
    iter++;
    if (iter > 30 * n) { ok = false; break; }
    start = end - 1;
    while (start > 0 && e[start - 1] != 0.f) start--;
    // tridiagonal_qr_step: Wilkinson shift
    const float td = (d[end - 1] - d[end]) * 0.5f;
    const float ee = e[end - 1];
    float mu = d[end];
    if (td == 0.f) {
      mu -= std::fabs(ee);
    } else {
      const float e2 = ee * ee;
      const float h = hypot_e(td, ee);
      if (e2 == 0.f) mu -= (ee / (td + (td > 0.f ? 1.f : -1.f))) * (ee / h);
      else mu -= e2 / (td + (td > 0.f ? h : -h));
    }
    float x = d[start] - mu, z = e[start];
    for (int k = start; k < end; ++k) {
      float c, s;
      givens(x, z, c, s);
      const float sdk = s * d[k] + c * e[k];
      const float dkp1 = s * e[k] + c * d[k + 1];
      d[k] = c * (c * d[k] - s * e[k]) - s * (c * e[k] - s * d[k + 1]);
      d[k + 1] = s * sdk + c * dkp1;
      e[k] = c * sdk - s * dkp1;
      if (k > start) e[k - 1] = c * e[k - 1] - s * z;
      x = e[k];
      if (k < end - 1) {
        z = -s * e[k + 1];
        e[k + 1] = c * e[k + 1];
      }
      // Q = Q * G: columns k, k+1 (applyOnTheRight with the transposed rotation)
      if (!(c == 1.f && s == 0.f))
        for (int r = 0; r < 3; ++r) {
          const float xi = V[r * 3 + k], yi = V[r * 3 + k + 1];
          V[r * 3 + k] = c * xi - s * yi;
          V[r * 3 + k + 1] = s * xi + c * yi;
        }
    }
  }
  if (ok)
    for (int i = 0; i < n - 1; ++i) {  // ascending, first minimum, column swaps
      int k = i;
      for (int j = i + 1; j < n; ++j)
        if (d[j] < d[k]) k = j;
      if (k != i) {
        std::swap(d[i], d[k]);
        for (int r = 0; r < 3; ++r) std::swap(V[r * 3 + i], V[r * 3 + k]);
      }
    }
  for (int i = 0; i < 3; ++i) evals[i] = d[i] * scale;
}

// ---- ColPivHouseholderQR<Matrix<float, M, N>>::solve, restated (M >= N) ----------------------------
template <int M, int N>
void qr_solve(const float A_in[M * N], const float b_in[M], float x[N]) {
  float A[M * N];
  std::memcpy(A, A_in, sizeof(A));
  const float eps = FLT_EPSILON;
  float nu[N], nd[N], hc[N];
  int perm[N];
  for (int k = 0; k < N; ++k) {
    float s = 0.f;
    for (int r = 0; r < M; ++r) s += A[r * N + k] * A[r * N + k];
    nu[k] = nd[k] = std::sqrt(s);
    perm[k] = k;
  }
  float maxn = 0.f;
  for (int k = 0; k < N; ++k) maxn = std::max(maxn, nu[k]);
  const float th_help = (maxn * eps) * (maxn * eps) / (float)M;
  const float ndt = std::sqrt(eps);
  int nzp = N;
  for (int k = 0; k < N; ++k) {
    int bc = k;
    for (int j = k + 1; j < N; ++j)
      if (nu[j] > nu[bc]) bc = j;
    const float bsq = nu[bc] * nu[bc];
    if (nzp == N && bsq < th_help * (float)(M - k)) nzp = k;
    if (bc != k) {
      for (int r = 0; r < M; ++r) std::swap(A[r * N + k], A[r * N + bc]);
      std::swap(nu[k], nu[bc]);
      std::swap(nd[k], nd[bc]);
      std::swap(perm[k], perm[bc]);
    }
    float tail = 0.f;
    for (int r = k + 1; r < M; ++r) tail += A[r * N + k] * A[r * N + k];
    const float c0 = A[k * N + k];
    float tau, beta;
    if (tail <= FLT_MIN) {
      tau = 0.f;
      beta = c0;
      for (int r = k + 1; r < M; ++r) A[r * N + k] = 0.f;
    } else {
      beta = std::sqrt(c0 * c0 + tail);
      if (c0 >= 0.f) beta = -beta;
      for (int r = k + 1; r < M; ++r) A[r * N + k] = A[r * N + k] / (c0 - beta);
      tau = (beta - c0) / beta;
    }
    hc[k] = tau;
    A[k * N + k] = beta;
    if (tau != 0.f)
      for (int j = k + 1; j < N; ++j) {
        float t = A[k * N + j];
        for (int r = k + 1; r < M; ++r) t += A[r * N + k] * A[r * N + j];
        A[k * N + j] -= tau * t;
        for (int r = k + 1; r < M; ++r) A[r * N + j] -= tau * A[r * N + k] * t;
      }
    for (int j = k + 1; j < N; ++j) {
      if (nu[j] != 0.f) {
        float t = std::fabs(A[k * N + j]) / nu[j];
        t = (1.f + t) * (1.f - t);
        if (t < 0.f) t = 0.f;
        const float q = nu[j] / nd[j];
        const float t2 = t * q * q;
        if (t2 <= ndt) {
          float s = 0.f;
          for (int r = k + 1; r < M; ++r) s += A[r * N + j] * A[r * N + j];
          nd[j] = std::sqrt(s);
          nu[j] = nd[j];
        } else {
          nu[j] *= std::sqrt(t);
        }
      }
    }
  }
  float c[M];
  std::memcpy(c, b_in, sizeof(c));
  for (int k = 0; k < nzp; ++k) {
    if (hc[k] == 0.f) continue;
    float t = c[k];
    for (int r = k + 1; r < M; ++r) t += A[r * N + k] * c[r];
    c[k] -= hc[k] * t;
    for (int r = k + 1; r < M; ++r) c[r] -= hc[k] * A[r * N + k] * t;
  }
  float y[N];
  for (int i = 0; i < N; ++i) y[i] = 0.f;
  for (int i = nzp - 1; i >= 0; --i) {
    float t = c[i];
    for (int j = i + 1; j < nzp; ++j) t -= A[i * N + j] * y[j];
    y[i] = t / A[i * N + i];
  }
  for (int i = 0; i < N; ++i) x[perm[i]] = (i < nzp) ? y[i] : 0.f;
}

// largest eigenvalue of a symmetric 6x6 (float entries) by cyclic Jacobi in double
static double lmax6(const float A[36]) {
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
        const double t = (th >= 0 ? 1.0 : -1.0) / (std::fabs(th) + std::sqrt(th * th + 1.0));
        const double c = 1.0 / std::sqrt(t * t + 1.0), s = t * c;
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
  for (int k = 1; k < 6; ++k) m = std::max(m, a[k * 6 + k]);
  return m;
}

// ---- exact kNN-5 inside the 1 m ball (nanoflann nearestKSearch(k = 5) where it matters) ------------
struct Grid {
  float mn[3] = {0, 0, 0};
  float cs = 1.01f;
  std::unordered_map<long long, std::vector<int>> cells;
  const Pt* pts = nullptr;
  int n = 0;
  mutable nfr::KdTree<Pt> tree;  // nanoflann's tree of the map, for tied queries (built on first use)
  mutable bool tree_built = false;
  static long long key(long long x, long long y, long long z) { return (x * 73856093LL) ^ (y * 19349663LL) ^ (z * 83492791LL); }
  void build(const Pt* p, int np) {
    pts = p;
    n = np;
    cells.clear();
    for (int a = 0; a < 3; ++a) mn[a] = FLT_MAX;
    for (int j = 0; j < np; ++j) {
      mn[0] = std::min(mn[0], p[j].x); mn[1] = std::min(mn[1], p[j].y); mn[2] = std::min(mn[2], p[j].z);
    }
    for (int j = 0; j < np; ++j) cells[key(cell(p[j].x, 0), cell(p[j].y, 1), cell(p[j].z, 2))].push_back(j);
    tree_built = false;
  }
  long long cell(float v, int a) const { return (long long)std::floor((double)(v - mn[a]) / cs); }
  // the 5 nearest as (d, index) pairs, true if the 5th is closer than 1.0 (d^2); tie flags the 6th
  bool knn5(const Pt& q, int out[5], float dist[5], bool& tie) const {
    std::vector<std::pair<float, int>> cand;
    const long long cx = cell(q.x, 0), cy = cell(q.y, 1), cz = cell(q.z, 2);
    for (long long dz = -1; dz <= 1; ++dz)
      for (long long dy = -1; dy <= 1; ++dy)
        for (long long dx = -1; dx <= 1; ++dx) {
          auto it = cells.find(key(cx + dx, cy + dy, cz + dz));
          if (it == cells.end()) continue;
          for (int j : it->second) {
            const Pt& p = pts[j];
            if (cell(p.x, 0) != cx + dx || cell(p.y, 1) != cy + dy || cell(p.z, 2) != cz + dz) continue;  // hash collision
            const float ex = q.x - p.x, ey = q.y - p.y, ez = q.z - p.z;
            const float d = ex * ex + ey * ey + ez * ez;  // nanoflann L2_Simple_Adaptor order
            if (d < 1.0f) cand.push_back({d, j});
          }
        }
    tie = false;
    if (cand.size() < 5) return false;
    std::sort(cand.begin(), cand.end());
    for (int k = 0; k < 5; ++k) { out[k] = cand[k].second; dist[k] = cand[k].first; }
    for (int k = 0; k + 1 < (int)cand.size() && k < 5; ++k)
      if (cand[k].first == cand[k + 1].first) tie = true;
    if (tie) {  // equal distances among the 6 nearest: nanoflann's order (first visited wins)
      if (!tree_built) {
        tree.build(pts, n);
        tree_built = true;
      }
      const float qv[3] = {q.x, q.y, q.z};
      tree.knn(qv, 5, out, dist);
      return dist[4] < 1.0f;
    }
    return true;
  }
};

struct Trig { float cRoll, sRoll, cPitch, sPitch, cYaw, sYaw, tX, tY, tZ; };

// updatePointAssociateToMapSinCos (:397-410) + pointAssociateToMap (:412-426)
static Trig trig_of(const float t[6]) {
  return {std::cos(t[0]), std::sin(t[0]), std::cos(t[1]), std::sin(t[1]), std::cos(t[2]), std::sin(t[2]),
          t[3], t[4], t[5]};
}
static Pt associate(const Trig& T, const Pt& pi) {
  const float x1 = T.cYaw * pi.x - T.sYaw * pi.y;
  const float y1 = T.sYaw * pi.x + T.cYaw * pi.y;
  const float z1 = pi.z;
  const float x2 = x1;
  const float y2 = T.cRoll * y1 - T.sRoll * z1;
  const float z2 = T.sRoll * y1 + T.cRoll * z1;
  return {T.cPitch * x2 + T.sPitch * z2 + T.tX, y2 + T.tY, -T.sPitch * x2 + T.cPitch * z2 + T.tZ, pi.i};
}

// cornerOptimization's per-point body (:1031-1131): true + coeff when the point is selected
bool corner_coeff(const Pt* map, const int ind[5], const Pt& sel, Pt& coeff) {
  float cx = 0, cy = 0, cz = 0;
  for (int j = 0; j < 5; j++) { cx += map[ind[j]].x; cy += map[ind[j]].y; cz += map[ind[j]].z; }
  cx /= 5; cy /= 5; cz /= 5;
  float a11 = 0, a12 = 0, a13 = 0, a22 = 0, a23 = 0, a33 = 0;
  for (int j = 0; j < 5; j++) {
    const float ax = map[ind[j]].x - cx, ay = map[ind[j]].y - cy, az = map[ind[j]].z - cz;
    a11 += ax * ax; a12 += ax * ay; a13 += ax * az;
    a22 += ay * ay; a23 += ay * az; a33 += az * az;
  }
  a11 /= 5; a12 /= 5; a13 /= 5; a22 /= 5; a23 /= 5; a33 /= 5;
  const float A1[9] = {a11, a12, a13, a12, a22, a23, a13, a23, a33};
  float D[3], V[9];
  eig3(A1, D, V);
  if (!(D[2] > 3 * D[1])) return false;
  const float x0 = sel.x, y0 = sel.y, z0 = sel.z;
  // matV1(0, j): the first component of eigenvector j (:1086-1091)
  const float x1 = (float)(cx + 0.1 * V[0]), y1 = (float)(cy + 0.1 * V[1]), z1 = (float)(cz + 0.1 * V[2]);
  const float x2 = (float)(cx - 0.1 * V[0]), y2 = (float)(cy - 0.1 * V[1]), z2 = (float)(cz - 0.1 * V[2]);
  const float a012 = std::sqrt(((x0 - x1) * (y0 - y2) - (x0 - x2) * (y0 - y1)) * ((x0 - x1) * (y0 - y2) - (x0 - x2) * (y0 - y1)) +
                               ((x0 - x1) * (z0 - z2) - (x0 - x2) * (z0 - z1)) * ((x0 - x1) * (z0 - z2) - (x0 - x2) * (z0 - z1)) +
                               ((y0 - y1) * (z0 - z2) - (y0 - y2) * (z0 - z1)) * ((y0 - y1) * (z0 - z2) - (y0 - y2) * (z0 - z1)));
  const float l12 = std::sqrt((x1 - x2) * (x1 - x2) + (y1 - y2) * (y1 - y2) + (z1 - z2) * (z1 - z2));
  const float la = ((y1 - y2) * ((x0 - x1) * (y0 - y2) - (x0 - x2) * (y0 - y1)) +
                    (z1 - z2) * ((x0 - x1) * (z0 - z2) - (x0 - x2) * (z0 - z1))) / a012 / l12;
  const float lb = -((x1 - x2) * ((x0 - x1) * (y0 - y2) - (x0 - x2) * (y0 - y1)) -
                     (z1 - z2) * ((y0 - y1) * (z0 - z2) - (y0 - y2) * (z0 - z1))) / a012 / l12;
  const float lc = -((x1 - x2) * ((x0 - x1) * (z0 - z2) - (x0 - x2) * (z0 - z1)) +
                     (y1 - y2) * ((y0 - y1) * (z0 - z2) - (y0 - y2) * (z0 - z1))) / a012 / l12;
  const float ld2 = a012 / l12;
  const float s = (float)(1 - 0.9 * std::fabs(ld2));
  coeff = {s * la, s * lb, s * lc, s * ld2};
  return s > 0.1;
}

// surfOptimization's per-point body (:1139-1194)
bool surf_coeff(const Pt* map, const int ind[5], const Pt& sel, Pt& coeff) {
  float A0[15], B0[5], X0[3];
  for (int j = 0; j < 5; j++) {
    A0[j * 3 + 0] = map[ind[j]].x;
    A0[j * 3 + 1] = map[ind[j]].y;
    A0[j * 3 + 2] = map[ind[j]].z;
    B0[j] = -1.f;  // matB0.fill(-1) (:215)
  }
  qr_solve<5, 3>(A0, B0, X0);
  float pa = X0[0], pb = X0[1], pc = X0[2], pd = 1;
  const float ps = std::sqrt(pa * pa + pb * pb + pc * pc);
  pa /= ps; pb /= ps; pc /= ps; pd /= ps;
  for (int j = 0; j < 5; j++)
    if (std::fabs(pa * map[ind[j]].x + pb * map[ind[j]].y + pc * map[ind[j]].z + pd) > 0.2) return false;
  const float pd2 = pa * sel.x + pb * sel.y + pc * sel.z + pd;
  const float s = (float)(1 - 0.9 * std::fabs(pd2) / std::sqrt(std::sqrt(sel.x * sel.x + sel.y * sel.y + sel.z * sel.z)));
  coeff = {s * pa, s * pb, s * pc, s * pd2};
  return s > 0.1;
}

struct State {
  float t[6];
  bool degenerate;
};

// one LM row (:1219-1256): matA = (arx, ary, arz, coeff x, y, z), matB = -coeff intensity
static void lm_row(const Trig& T, const Pt& p, const Pt& c, float out[7]) {
  const float srx = T.sRoll, crx = T.cRoll, sry = T.sPitch, cry = T.cPitch, srz = T.sYaw, crz = T.cYaw;
  const float arx = (crx * sry * srz * p.x + crx * crz * sry * p.y - srx * sry * p.z) * c.x +
                    (-srx * srz * p.x - crz * srx * p.y - crx * p.z) * c.y +
                    (crx * cry * srz * p.x + crx * cry * crz * p.y - cry * srx * p.z) * c.z;
  const float ary = ((cry * srx * srz - crz * sry) * p.x + (sry * srz + cry * crz * srx) * p.y + crx * cry * p.z) * c.x +
                    ((-cry * crz - srx * sry * srz) * p.x + (cry * srz - crz * srx * sry) * p.y - crx * sry * p.z) * c.z;
  const float arz = ((crz * srx * sry - cry * srz) * p.x + (-cry * crz - srx * sry * srz) * p.y) * c.x +
                    (crx * crz * p.x - crx * srz * p.y) * c.y +
                    ((sry * srz + cry * crz * srx) * p.x + (crz * sry - cry * srx * srz) * p.y) * c.z;
  const float row[7] = {arx, ary, arz, c.x, c.y, c.z, -c.i};  // matA row, matB entry (:1246-1256)
  std::memcpy(out, row, sizeof(row));
}

// matAt * matA and matAt * matB (:1258-1259) in a fixed order: row q (its query index: corners first,
// then surfs) adds its float products, widened to double, into lane q % 1024's partial sums in
// increasing q; each 64-lane group reduces by xor butterflies (offsets 32, 16, .., 1) and the 16 group
// sums add in group order.  This is the order of the product's k_s2m (one lane per query, wave
// shuffles, a per-wave table); Eigen's float GEMM order cannot be restated without Eigen, and any
// fixed order is the reference's sum up to rounding.  out: 21 upper-triangle AtA entries, then 6 AtB.
static void normal_equations(const std::vector<float>& rows, const std::vector<int>& qidx, double out[27]) {
  if (g_float_ne) {  // diagnostic model: float accumulators in row order (:1258-1259 as plain loops)
    float f[27] = {0};
    for (size_t i = 0; i < qidx.size(); ++i) {
      const float* a = &rows[7 * i];
      int k = 0;
      for (int r = 0; r < 6; ++r)
        for (int j = r; j < 6; ++j) f[k++] += a[r] * a[j];
      for (int r = 0; r < 6; ++r) f[21 + r] += a[r] * a[6];
    }
    for (int k = 0; k < 27; ++k) out[k] = f[k];
    return;
  }
  constexpr int LANES = 1024, W = 64;
  std::vector<double> part((size_t)LANES * 27, 0.0);
  for (size_t i = 0; i < qidx.size(); ++i) {
    const float* a = &rows[7 * i];
    const float b = a[6];
    double* p = &part[(size_t)(qidx[i] % LANES) * 27];
    int k = 0;
    for (int r = 0; r < 6; ++r)
      for (int j = r; j < 6; ++j) p[k++] += (double)(a[r] * a[j]);
    for (int r = 0; r < 6; ++r) p[21 + r] += (double)(a[r] * b);
  }
  for (int k = 0; k < 27; ++k) {
    double s = 0.0;
    for (int w = 0; w < LANES / W; ++w) {
      double v[W], t[W];
      for (int l = 0; l < W; ++l) v[l] = part[(size_t)(w * W + l) * 27 + k];
      for (int o = W / 2; o > 0; o >>= 1) {
        for (int l = 0; l < W; ++l) t[l] = v[l] + v[l ^ o];
        std::memcpy(v, t, sizeof(v));
      }
      s += v[0];
    }
    out[k] = s;
  }
}

// LMOptimization (:1199-1312); true = converged.  qidx: each selected row's query index.
static bool lm_step(State& S, const std::vector<Pt>& ori, const std::vector<Pt>& coeffs, const std::vector<int>& qidx,
                    int iterCount) {
  const int n = (int)ori.size();
  if (n < 50) return false;
  std::vector<float> rows((size_t)7 * n);
  const Trig T = trig_of(S.t);
  for (int i = 0; i < n; i++) lm_row(T, ori[i], coeffs[i], &rows[(size_t)7 * i]);
  double ne[27];
  normal_equations(rows, qidx, ne);
  float A[36], B[6], X[6];
  int k = 0;
  for (int r = 0; r < 6; ++r)
    for (int j = r; j < 6; ++j, ++k) A[r * 6 + j] = A[j * 6 + r] = (float)ne[k];
  for (int r = 0; r < 6; ++r) B[r] = (float)ne[21 + r];
  qr_solve<6, 6>(A, B, X);
  if (iterCount == 0) S.degenerate = lmax6(A) < 100.0;  // :1262-1286 (see header)
  if (S.degenerate)
    for (int k = 0; k < 6; ++k) X[k] = 0.f;  // matX = matP * matX with matP = 0
  for (int k = 0; k < 6; ++k) S.t[k] += X[k];
  const float deltaR = (float)std::sqrt(std::pow(X[0] * 57.29578f, 2) + std::pow(X[1] * 57.29578f, 2) +
                                        std::pow(X[2] * 57.29578f, 2));
  const float deltaT = (float)std::sqrt(std::pow(X[3] * 100, 2) + std::pow(X[4] * 100, 2) + std::pow(X[5] * 100, 2));
  return deltaR < 0.05 && deltaT < 0.05;
}

}  // namespace s2m

static int scan2map(const float* corner, int n_corner, const float* surf, int n_surf, const float* corner_map,
                    int n_corner_map, const float* surf_map, int n_surf_map, float* transform, int32_t* degenerate,
                    int32_t* info, int max_iters, float* rows_out) {
  using namespace s2m;
  info[0] = 0; info[1] = 0; info[2] = 0; info[3] = 0;
  if (!(n_corner_map > 10 && n_surf_map > 100)) {  // :1316
    info[3] = LEGO_S2M_ST_SKIPPED;
    return 0;
  }
  const Pt* cs = (const Pt*)corner;
  const Pt* ss = (const Pt*)surf;
  const Pt* cm = (const Pt*)corner_map;
  const Pt* sm = (const Pt*)surf_map;
  Grid gc, gs;  // kdtreeCornerFromMap / kdtreeSurfFromMap.setInputCloud (:1317-1318)
  gc.build(cm, n_corner_map);
  gs.build(sm, n_surf_map);
  State S;
  for (int k = 0; k < 6; ++k) S.t[k] = transform[k];
  S.degenerate = *degenerate != 0;
  int status = 0, iters = 0, nsel = 0;
  std::vector<Pt> ori, coeffs;
  std::vector<int> qidx;
  for (int iterCount = 0; iterCount < max_iters; iterCount++) {
    ori.clear();
    coeffs.clear();
    qidx.clear();
    const Trig T = trig_of(S.t);
    for (int i = 0; i < n_corner; i++) {  // cornerOptimization (:1028-1134)
      const Pt sel = associate(T, cs[i]);
      int ind[5];
      float d[5];
      bool tie = false;
      if (!gc.knn5(sel, ind, d, tie)) continue;
      if (tie) status |= LEGO_S2M_ST_KNN_TIE;
      Pt c;
      if (corner_coeff(cm, ind, sel, c)) { ori.push_back(cs[i]); coeffs.push_back(c); qidx.push_back(i); }
    }
    for (int i = 0; i < n_surf; i++) {  // surfOptimization (:1136-1197)
      const Pt sel = associate(T, ss[i]);
      int ind[5];
      float d[5];
      bool tie = false;
      if (!gs.knn5(sel, ind, d, tie)) continue;
      if (tie) status |= LEGO_S2M_ST_KNN_TIE;
      Pt c;
      if (surf_coeff(sm, ind, sel, c)) { ori.push_back(ss[i]); coeffs.push_back(c); qidx.push_back(n_corner + i); }
    }
    iters = iterCount + 1;
    nsel = (int)ori.size();
    if (nsel < 50) status |= LEGO_S2M_ST_FEW;
    if (rows_out) {  // the debug view: this iteration's rows in the product's layout
      std::memset(rows_out, 0, sizeof(float) * 8 * (size_t)(n_corner + n_surf));
      const Trig T0 = trig_of(S.t);
      for (size_t i = 0; i < ori.size(); ++i) {
        float r[7];
        lm_row(T0, ori[i], coeffs[i], r);
        float* o = rows_out + 8 * (size_t)qidx[i];
        std::memcpy(o, r, sizeof(r));
        o[7] = 1.f;
      }
    }
    const bool conv = lm_step(S, ori, coeffs, qidx, iterCount);
    if (iterCount == 0 && S.degenerate && nsel >= 50) status |= LEGO_S2M_ST_DEGENERATE;
    if (conv) {
      status |= LEGO_S2M_ST_CONVERGED;
      break;
    }
  }
  for (int k = 0; k < 6; ++k) transform[k] = S.t[k];
  *degenerate = S.degenerate ? 1 : 0;
  info[0] = 1;
  info[1] = iters;
  info[2] = nsel;
  info[3] = status;
  return 0;
}

extern "C" int oracle_scan2map(const float* corner, int n_corner, const float* surf, int n_surf, const float* corner_map,
                               int n_corner_map, const float* surf_map, int n_surf_map, float* transform,
                               int32_t* degenerate, int32_t* info) {
  return scan2map(corner, n_corner, surf, n_surf, corner_map, n_corner_map, surf_map, n_surf_map, transform, degenerate,
                  info, 10, nullptr);
}

// debug view: at most max_iters LM iterations, the last iteration's rows as lego_test_s2m_debug's
extern "C" int oracle_scan2map_debug(const float* corner, int n_corner, const float* surf, int n_surf,
                                     const float* corner_map, int n_corner_map, const float* surf_map, int n_surf_map,
                                     float* transform, int32_t* degenerate, int32_t* info, int max_iters,
                                     float* rows_out) {
  return scan2map(corner, n_corner, surf, n_surf, corner_map, n_corner_map, surf_map, n_surf_map, transform, degenerate,
                  info, max_iters, rows_out);
}

// test hooks: the restated Eigen pieces and the kNN on their own
extern "C" void oracle_eig3(const float* A, float* evals, float* V) { s2m::eig3(A, evals, V); }
extern "C" void oracle_qr53(const float* A, const float* b, float* x) { s2m::qr_solve<5, 3>(A, b, x); }
extern "C" void oracle_qr66(const float* A, const float* b, float* x) { s2m::qr_solve<6, 6>(A, b, x); }
extern "C" int oracle_knn5(const float* map, int n_map, const float* q, int n_q, int32_t* ind, float* dist,
                           int32_t* flags) {
  s2m::Grid g;
  g.build((const s2m::Pt*)map, n_map);
  for (int i = 0; i < n_q; ++i) {
    bool tie = false;
    const bool ok = g.knn5(((const s2m::Pt*)q)[i], ind + 5 * i, dist + 5 * i, tie);
    flags[i] = (ok ? 1 : 0) | (tie ? 2 : 0);
  }
  return 0;
}

// MapOptimization::transformPointCloud (:428-473) with the key pose (roll, pitch, yaw, x, y, z)
extern "C" void oracle_transform_cloud(const float* in, int n, const float* pose, float* out) {
  const float ctRoll = std::cos(pose[0]), stRoll = std::sin(pose[0]);
  const float ctPitch = std::cos(pose[1]), stPitch = std::sin(pose[1]);
  const float ctYaw = std::cos(pose[2]), stYaw = std::sin(pose[2]);
  const float tInX = pose[3], tInY = pose[4], tInZ = pose[5];
  for (int i = 0; i < n; ++i) {
    const float* f = in + 4 * i;
    const float x1 = ctYaw * f[0] - stYaw * f[1];
    const float y1 = stYaw * f[0] + ctYaw * f[1];
    const float z1 = f[2];
    const float x2 = x1;
    const float y2 = ctRoll * y1 - stRoll * z1;
    const float z2 = stRoll * y1 + ctRoll * z1;
    float* t = out + 4 * i;
    t[0] = ctPitch * x2 + stPitch * z2 + tInX;
    t[1] = y2 + tInY;
    t[2] = -stPitch * x2 + ctPitch * z2 + tInZ;
    t[3] = f[3];
  }
}

// MapOptimization::transformAssociateToMap (mapOptmization.cpp:264-387): transformSum S, transformBefMapped
// B, transformAftMapped A -> transformTobeMapped T.  float throughout, the float libm overloads.
extern "C" void oracle_associate_to_map(const float* S, const float* B, const float* A, float* T) {
  using std::cos;
  using std::sin;
  float inc[6] = {0, 0, 0, 0, 0, 0};
  {
    const float x1 = cos(S[1]) * (B[3] - S[3]) - sin(S[1]) * (B[5] - S[5]);
    const float y1 = B[4] - S[4];
    const float z1 = sin(S[1]) * (B[3] - S[3]) + cos(S[1]) * (B[5] - S[5]);
    const float y2 = cos(S[0]) * y1 + sin(S[0]) * z1;
    const float z2 = -sin(S[0]) * y1 + cos(S[0]) * z1;
    inc[3] = cos(S[2]) * x1 + sin(S[2]) * y2;
    inc[4] = -sin(S[2]) * x1 + cos(S[2]) * y2;
    inc[5] = z2;
  }
  const float sbcx = sin(S[0]), cbcx = cos(S[0]), sbcy = sin(S[1]), cbcy = cos(S[1]), sbcz = sin(S[2]), cbcz = cos(S[2]);
  const float sblx = sin(B[0]), cblx = cos(B[0]), sbly = sin(B[1]), cbly = cos(B[1]), sblz = sin(B[2]), cblz = cos(B[2]);
  const float salx = sin(A[0]), calx = cos(A[0]), saly = sin(A[1]), caly = cos(A[1]), salz = sin(A[2]), calz = cos(A[2]);
  // products shared by the three angle expressions
  const float p1 = salx * sblx + calx * cblx * salz * sblz + calx * calz * cblx * cblz;
  const float p2 = calx * calz * (cbly * sblz - cblz * sblx * sbly) - calx * salz * (cbly * cblz + sblx * sbly * sblz) +
                   cblx * salx * sbly;
  const float p3 = calx * salz * (cblz * sbly - cbly * sblx * sblz) - calx * calz * (sbly * sblz + cbly * cblz * sblx) +
                   cblx * cbly * salx;
  const float srx = -sbcx * p1 - cbcx * sbcy * p2 - cbcx * cbcy * p3;
  T[0] = -std::asin(srx);
  const float q1 = caly * calz + salx * saly * salz, q2 = caly * salz - calz * salx * saly;
  const float q3 = saly * salz + caly * calz * salx, q4 = calz * saly - caly * salx * salz;
  const float srycrx = sbcx * (cblx * cblz * q2 - cblx * sblz * q1 + calx * saly * sblx) -
                       cbcx * cbcy * (q1 * (cblz * sbly - cbly * sblx * sblz) + q2 * (sbly * sblz + cbly * cblz * sblx) -
                                      calx * cblx * cbly * saly) +
                       cbcx * sbcy * (q1 * (cbly * cblz + sblx * sbly * sblz) + q2 * (cbly * sblz - cblz * sblx * sbly) +
                                      calx * cblx * saly * sbly);
  const float crycrx = sbcx * (cblx * sblz * q4 - cblx * cblz * q3 + calx * caly * sblx) +
                       cbcx * cbcy * (q3 * (sbly * sblz + cbly * cblz * sblx) + q4 * (cblz * sbly - cbly * sblx * sblz) +
                                      calx * caly * cblx * cbly) -
                       cbcx * sbcy * (q3 * (cbly * sblz - cblz * sblx * sbly) + q4 * (cbly * cblz + sblx * sbly * sblz) -
                                      calx * caly * cblx * sbly);
  T[1] = std::atan2(srycrx / cos(T[0]), crycrx / cos(T[0]));
  const float srzcrx = (cbcz * sbcy - cbcy * sbcx * sbcz) * p3 - (cbcy * cbcz + sbcx * sbcy * sbcz) * p2 + cbcx * sbcz * p1;
  const float crzcrx = (cbcy * sbcz - cbcz * sbcx * sbcy) * p2 - (sbcy * sbcz + cbcy * cbcz * sbcx) * p3 + cbcx * cbcz * p1;
  T[2] = std::atan2(srzcrx / cos(T[0]), crzcrx / cos(T[0]));
  const float x1 = cos(T[2]) * inc[3] - sin(T[2]) * inc[4];
  const float y1 = sin(T[2]) * inc[3] + cos(T[2]) * inc[4];
  const float z1 = inc[5];
  const float y2 = cos(T[0]) * y1 - sin(T[0]) * z1;
  const float z2 = sin(T[0]) * y1 + cos(T[0]) * z1;
  T[3] = A[3] - (cos(T[1]) * x1 + sin(T[1]) * z2);
  T[4] = A[4] - y2;
  T[5] = A[5] - (-sin(T[1]) * x1 + cos(T[1]) * z2);
}

// OdometryToTransform (utility.h:96-110): the mapping thread's transformSum from the odometry message,
// through tf::Matrix3x3(tf::Quaternion(q.z, -q.x, -q.y, q.w)).getRPY (tf/LinearMath/Matrix3x3.h:
// setRotation, getEulerYPR with solution 1) in double, then transform = (-pitch, -yaw, roll, position).
extern "C" void oracle_odometry_to_transform(const double* orientation, const double* position, float* transform) {
  using std::asin;
  using std::atan2;
  using std::cos;
  using std::fabs;
  const double qx = orientation[2], qy = -orientation[0], qz = -orientation[1], qw = orientation[3];
  const double d = qx * qx + qy * qy + qz * qz + qw * qw;  // Quaternion::length2
  const double s = 2.0 / d;
  const double xs = qx * s, ys = qy * s, zs = qz * s;
  const double wx = qw * xs, wy = qw * ys, wz = qw * zs;
  const double xx = qx * xs, xy = qx * ys, xz = qx * zs;
  const double yy = qy * ys, yz = qy * zs, zz = qz * zs;
  const double m00 = 1.0 - (yy + zz), m10 = xy + wz;
  const double m20 = xz - wy, m21 = yz + wx, m22 = 1.0 - (xx + yy);
  double roll, pitch, yaw;
  if (fabs(m20) >= 1) {  // gimbal lock
    yaw = 0;
    const double delta = atan2(m21, m22);
    pitch = m20 < 0 ? 3.1415926535897932384626433832795029 / 2.0 : -3.1415926535897932384626433832795029 / 2.0;
    roll = delta;
  } else {
    double a = m20;  // tfAsin clamps to [-1, 1]
    if (a < -1) a = -1;
    if (a > 1) a = 1;
    pitch = -asin(a);
    roll = atan2(m21 / cos(pitch), m22 / cos(pitch));
    yaw = atan2(m10 / cos(pitch), m00 / cos(pitch));
  }
  transform[0] = (float)-pitch;
  transform[1] = (float)-yaw;
  transform[2] = (float)roll;
  transform[3] = (float)position[0];
  transform[4] = (float)position[1];
  transform[5] = (float)position[2];
}
