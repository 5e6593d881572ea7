// lego_oracle.cpp — CPU restatement of LeGO-LOAM-BOR's per-scan hot path.
//
// TEST INFRASTRUCTURE ONLY.  This file is the parity oracle for the MI355X product path
// (lego-loam-bor_amd/csrc).  Only tests/, __graft_entry__.smoke() and bench.py's
// cpu_baseline leg may load it, and only as the checker / the CPU timing baseline.
// Nothing in the product links or calls it.
//
// It restates, function by function, /root/reference/LeGO-LOAM/src/imageProjection.cpp and
// featureAssociation.cpp (citations below are file:line into the reference), keeping the
// reference's float/double expression types, evaluation order, loop bounds and the
// cross-scan state of FeatureAssociation's work arrays.  Build: -O3, no -march, and
// -ffp-contract=off (x86-64 without -march has no FMA, as in LeGO-LOAM/CMakeLists.txt:4).
//
// PARITY STATUS:
//   * The reference cannot be built here (ROS/PCL/Eigen/Boost absent), has no
//     tests and no golden vectors.  This restatement is therefore "parity unpinned" against the
//     reference itself, except for two pinned boundaries:
//       - libm: unqualified float sin/cos/atan2/asin resolve to glibc's float functions
//         (fp_mode 0).  The oracle calls glibc directly.
//       - kd-tree 1-NN: nanoflann 1.3.0's tree and search restated (nanoflann_restated.h), exact
//         distance ties resolved as nanoflann resolves them (first visited); oracle/_ref builds the
//         reference's vendored nanoflann and checks the restatement against it.
//   * Restated third-party boundaries (unpinned): PCL VoxelGrid::applyFilter (PCL 1.7/1.8 algorithm,
//     restated below), Eigen AtA/QR/eigen (modelled: float products summed in double, column-pivoting
//     Householder QR in float, symmetric eigenvalues in double).
//   * Reference UB is given defined behaviour and flagged (LEGO_ST_* bits in include/lego_frontend.h).
#ifndef _GNU_SOURCE
#define _GNU_SOURCE  // sincos
#endif
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <functional>
#include <cstdlib>
#include <cstdio>
#include <limits>
#include <vector>

#include "../include/lego_frontend.h"
#include "nanoflann_restated.h"

// Diagnostic: both LMs' normal equations summed in float in row order (see solve_normal); 0 = the model
// the product follows.  Shared with s2m_oracle.cpp.
int g_float_ne = 0;
extern "C" void oracle_set_float_normal_equations(int on) { g_float_ne = on ? 1 : 0; }

namespace {

const double DEG_TO_RAD = M_PI / 180.0;          // utility.h:50
const float RAD2DEG = 180.0 / M_PI;              // featureAssociation.cpp:39

typedef lego_point Pt;

// The two libm overload models, selected by lego_params.fp_mode:
//   Lm<float>  fp_mode 0: unqualified sin(float) etc. resolve to the float overloads (libstdc++ >= 6's
//              <math.h> wrapper) -> glibc's sinf / cosf / atan2f / asinf / sqrtf;
//   Lm<double> fp_mode 1: they resolve to ::sin(double) etc. (pre-GCC-6 libstdc++, the ROS Indigo /
//              Kinetic toolchains of README.md:40): the expression is evaluated in double and rounded
//              where the reference stores it to float.
// T is the type the reference's expression is evaluated in.  Explicitly std::-qualified calls
// (imageProjection.cpp:190,198,237,240) are float in both models.
//
// sin and cos of the same argument: every unqualified sin(x) of the path has a cos(x) of the same x in
// the same function (TransformToStart/End, AccumulateRotation, calculateTransformation*,
// integrateTransformation, labelComponents), and GCC at -O1 and above merges such pairs into one
// sincos(x) call (its cse_sincos pass; the reference builds with -O3, CMakeLists.txt:4).  glibc 2.35's
// double sincos is not bit-identical to its sin / cos (6e-5 of float arguments in [-4, 4] differ in
// the last bit; sincosf equals sinf / cosf), so the oracle calls sincos explicitly for sn / cs, as the
// reference binary does, and plain cos for the one unpaired call, cos(ox) in AccumulateRotation
// (:489, cs1).  Without this the oracle's own results depended on how GCC inlined it.
template <class T>
struct Lm;
template <>
struct Lm<float> {
  static float sn(float x) { return sinf(x); }
  static float cs(float x) { return cosf(x); }
  static float cs1(float x) { return cosf(x); }
  static float at2(float y, float x) { return atan2f(y, x); }
  static float as(float x) { return asinf(x); }
  static float sq(float x) { return sqrtf(x); }
};
template <>
struct Lm<double> {
  static double sn(double x) { double s, c; sincos(x, &s, &c); return s; }
  static double cs(double x) { double s, c; sincos(x, &s, &c); return c; }
  static double cs1(double x) { return cos(x); }
  static double at2(double y, double x) { return atan2(y, x); }
  static double as(double x) { return asin(x); }
  static double sq(double x) { return sqrt(x); }
};

Pt nan_point() {  // imageProjection.cpp:109-112 (PCL default ctor: intensity 0)
  Pt p;
  p.x = p.y = p.z = std::numeric_limits<float>::quiet_NaN();
  p.intensity = 0.f;
  return p;
}

struct smoothness_t {  // utility.h:53-56
  float value;
  size_t ind;
};
struct by_value {  // utility.h:58-62
  bool operator()(smoothness_t const& l, smoothness_t const& r) { return l.value < r.value; }
};

// ======================================================================================
// ImageProjection (imageProjection.cpp)
// ======================================================================================
struct ImageProjection {
  int V, H, G, seg_valid_pt, seg_valid_line;
  float ang_res_x, ang_res_y, ang_bottom, segment_theta, mount;
  // per-call derived constants of labelComponents (imageProjection.cpp:414,463): float overloads
  // (fp_mode 0) or double (fp_mode 1)
  bool fp1;
  float theta_thr, sinX, cosX, sinY, cosY;
  double sinXd, cosXd, sinYd, cosYd;

  std::vector<Pt> cloud_in, full_cloud;
  std::vector<float> range_mat;
  std::vector<int8_t> ground_mat;
  std::vector<int32_t> label_mat;
  int label_count;
  // outputs (ProjectionOut)
  std::vector<Pt> segmented, outlier, scan_msg;
  std::vector<int32_t> start_ring, end_ring;
  std::vector<uint8_t> seg_ground;
  std::vector<uint32_t> seg_col;
  std::vector<float> seg_range;
  float start_ori, end_ori, ori_diff;
  // BFS scratch
  std::vector<int> q_r, q_c, ap_r, ap_c;

  explicit ImageProjection(const lego_params& p) {
    // ctor, imageProjection.cpp:57-84
    V = p.num_vertical_scans;
    H = p.num_horizontal_scans;
    float _ang_bottom = p.vertical_angle_bottom;
    float vertical_angle_top = p.vertical_angle_top;
    ang_res_x = (M_PI * 2) / (H);                                             // :64
    ang_res_y = DEG_TO_RAD * (vertical_angle_top - _ang_bottom) / float(V - 1);  // :65
    ang_bottom = -(_ang_bottom - 0.1) * DEG_TO_RAD;                           // :66
    segment_theta = p.segment_theta;
    segment_theta *= DEG_TO_RAD;                                              // :71
    seg_valid_pt = p.segment_valid_point_num;
    seg_valid_line = p.segment_valid_line_num;
    G = p.ground_scan_index;
    mount = p.sensor_mount_angle;
    mount *= DEG_TO_RAD;                                                      // :84
    fp1 = p.fp_mode == 1;
    theta_thr = fp1 ? (float)tan((double)segment_theta) : tanf(segment_theta);  // :414
    sinX = sinf(ang_res_x); cosX = cosf(ang_res_x);                           // :463 alpha=_ang_resolution_X
    sinY = sinf(ang_res_y); cosY = cosf(ang_res_y);                           // :463 alpha=_ang_resolution_Y
    sincos((double)ang_res_x, &sinXd, &cosXd);  // fp_mode 1: sin / cos(alpha) in double (one sincos, see Lm)
    sincos((double)ang_res_y, &sinYd, &cosYd);
    full_cloud.resize((size_t)V * H);
  }

  void resetParameters() {  // :107-150
    const size_t n = (size_t)V * H;
    range_mat.assign(n, FLT_MAX);
    ground_mat.assign(n, 0);
    label_mat.assign(n, 0);
    label_count = 1;
    std::fill(full_cloud.begin(), full_cloud.end(), nan_point());
    segmented.clear(); outlier.clear(); scan_msg.clear();
    start_ring.assign(V, 0); end_ring.assign(V, 0);
    seg_ground.assign(n, 0); seg_col.assign(n, 0); seg_range.assign(n, 0.f);
  }

  void findStartEndAngle() {  // :234-249
    Pt point = cloud_in.front();
    start_ori = -std::atan2(point.y, point.x);
    point = cloud_in.back();
    end_ori = -std::atan2(point.y, point.x) + 2 * M_PI;
    if (end_ori - start_ori > 3 * M_PI) {
      end_ori -= 2 * M_PI;
    } else if (end_ori - start_ori < M_PI) {
      end_ori += 2 * M_PI;
    }
    ori_diff = end_ori - start_ori;
  }

  void projectPointCloud() {  // :178-224
    const size_t cloudSize = cloud_in.size();
    for (size_t i = 0; i < cloudSize; ++i) {
      Pt thisPoint = cloud_in[i];
      float range = sqrtf(thisPoint.x * thisPoint.x + thisPoint.y * thisPoint.y + thisPoint.z * thisPoint.z);
      float verticalAngle = std::asin(thisPoint.z / range);
      int rowIdn = (verticalAngle + ang_bottom) / ang_res_y;
      if (rowIdn < 0 || rowIdn >= V) continue;
      float horizonAngle = std::atan2(thisPoint.x, thisPoint.y);
      int columnIdn = -round((horizonAngle - M_PI_2) / ang_res_x) + H * 0.5;
      if (columnIdn >= H) columnIdn -= H;
      if (columnIdn < 0 || columnIdn >= H) continue;
      if (range < 0.1) continue;
      range_mat[(size_t)rowIdn * H + columnIdn] = range;
      thisPoint.intensity = (float)rowIdn + (float)columnIdn / 10000.0;
      size_t index = columnIdn + rowIdn * H;
      full_cloud[index] = thisPoint;
    }
  }

  void groundRemoval() {  // :254-346
    for (int j = 0; j < H; ++j) {
      for (int i = 0; i < G; ++i) {
        size_t lowerInd = j + (i)*H;
        size_t upperInd = j + (i + 1) * H;
        // :264-269 intensity == -1 branch is dead (invalid cells carry intensity 0).
        float dX = full_cloud[upperInd].x - full_cloud[lowerInd].x;
        float dY = full_cloud[upperInd].y - full_cloud[lowerInd].y;
        float dZ = full_cloud[upperInd].z - full_cloud[lowerInd].z;
        // std::atan2(float, sqrt(...)): float overloads (fp_mode 0); with ::sqrt(double) the qualified
        // std::atan2(float, double) promotes to double (fp_mode 1)
        float vertical_angle = fp1 ? (float)std::atan2((double)dZ, sqrt((double)(dX * dX + dY * dY + dZ * dZ)))
                                   : std::atan2(dZ, sqrtf(dX * dX + dY * dY + dZ * dZ));
        if ((vertical_angle - mount) <= 10 * DEG_TO_RAD) {
          ground_mat[(size_t)i * H + j] = 1;
          ground_mat[(size_t)(i + 1) * H + j] = 1;
        }
      }
    }
    for (int i = 0; i < V; ++i)
      for (int j = 0; j < H; ++j)
        if (ground_mat[(size_t)i * H + j] == 1 || range_mat[(size_t)i * H + j] == FLT_MAX)
          label_mat[(size_t)i * H + j] = -1;
    // ground cloud (:303-308) is visualisation only: not restated.
    for (int j = 0; j < H; ++j) {  // 2-D scan, :312-330
      float min_range = 1000;
      size_t id_min = 0;
      for (int i = 0; i < V; ++i) {
        size_t Ind = j + (i)*H;
        float Z = full_cloud[Ind].z;
        if ((ground_mat[Ind] != 1) && (Z > 0.4) && (Z < 1.2) && (range_mat[Ind] < 40)) {
          if (range_mat[Ind] < min_range) {
            min_range = range_mat[Ind];
            id_min = Ind;
          }
        }
      }
      if (min_range < 1000) scan_msg.push_back(full_cloud[id_min]);
    }
  }

  void labelComponents(int row, int col) {  // :412-496
    std::vector<bool> lineCountFlag(V, false);
    q_r.clear(); q_c.clear(); ap_r.clear(); ap_c.clear();
    size_t qh = 0;
    q_r.push_back(row); q_c.push_back(col);
    ap_r.push_back(row); ap_c.push_back(col);
    static const int nb[4][2] = {{0, -1}, {-1, 0}, {1, 0}, {0, 1}};
    while (qh < q_r.size()) {
      int fx = q_r[qh], fy = q_c[qh];
      ++qh;
      label_mat[(size_t)fx * H + fy] = label_count;
      for (int k = 0; k < 4; ++k) {
        int thisIndX = fx + nb[k][0];
        int thisIndY = fy + nb[k][1];
        if (thisIndX < 0 || thisIndX >= V) continue;
        if (thisIndY < 0) thisIndY = H - 1;
        if (thisIndY >= H) thisIndY = 0;
        if (label_mat[(size_t)thisIndX * H + thisIndY] != 0) continue;
        float rf = range_mat[(size_t)fx * H + fy], rt = range_mat[(size_t)thisIndX * H + thisIndY];
        float d1 = std::max(rf, rt);
        float d2 = std::min(rf, rt);
        // alpha = (iter.x() == 0) ? resX : resY; sin/cos(alpha) hoisted (float overloads).
        float tang;
        if (fp1) {  // (d2 * sin(alpha) / (d1 - d2 * cos(alpha))) in double
          double sA = (nb[k][0] == 0) ? sinXd : sinYd;
          double cA = (nb[k][0] == 0) ? cosXd : cosYd;
          tang = (float)((double)d2 * sA / ((double)d1 - (double)d2 * cA));
        } else {
          float sA = (nb[k][0] == 0) ? sinX : sinY;
          float cA = (nb[k][0] == 0) ? cosX : cosY;
          tang = (d2 * sA / (d1 - d2 * cA));
        }
        if (tang > theta_thr) {
          q_r.push_back(thisIndX); q_c.push_back(thisIndY);
          label_mat[(size_t)thisIndX * H + thisIndY] = label_count;
          lineCountFlag[thisIndX] = true;
          ap_r.push_back(thisIndX); ap_c.push_back(thisIndY);
        }
      }
    }
    bool feasibleSegment = false;
    if (ap_r.size() >= 30) {
      feasibleSegment = true;
    } else if (ap_r.size() >= (size_t)seg_valid_pt) {
      int lineCount = 0;
      for (int i = 0; i < V; ++i)
        if (lineCountFlag[i] == true) ++lineCount;
      if (lineCount >= seg_valid_line) feasibleSegment = true;
    }
    if (feasibleSegment == true) {
      ++label_count;
    } else {
      for (size_t i = 0; i < ap_r.size(); ++i) label_mat[(size_t)ap_r[i] * H + ap_c[i]] = 999999;
    }
  }

  void cloudSegmentation() {  // :352-409
    for (int i = 0; i < V; ++i)
      for (int j = 0; j < H; ++j)
        if (label_mat[(size_t)i * H + j] == 0) labelComponents(i, j);
    int sizeOfSegCloud = 0;
    for (int i = 0; i < V; ++i) {
      start_ring[i] = sizeOfSegCloud - 1 + 5;
      for (int j = 0; j < H; ++j) {
        size_t c = (size_t)i * H + j;
        if (label_mat[c] > 0 || ground_mat[c] == 1) {
          if (label_mat[c] == 999999) {
            if (i > G && j % 5 == 0) {
              outlier.push_back(full_cloud[c]);
              continue;
            } else {
              continue;
            }
          }
          if (ground_mat[c] == 1) {
            if (j % 5 != 0 && j > 5 && j < H - 5) continue;
          }
          seg_ground[sizeOfSegCloud] = (ground_mat[c] == 1);
          seg_col[sizeOfSegCloud] = j;
          seg_range[sizeOfSegCloud] = range_mat[c];
          segmented.push_back(full_cloud[c]);
          ++sizeOfSegCloud;
        }
      }
      end_ring[i] = sizeOfSegCloud - 1 - 5;
    }
    // segmented_cloud_pure (:399-408) is visualisation only: not restated.
  }

  int cloudHandler(const void* pts, int n, int step, int ox, int oy, int oz) {  // :153-174
    resetParameters();
    cloud_in.clear();
    const char* base = (const char*)pts;
    for (int i = 0; i < n; ++i) {  // fromROSMsg + removeNaNFromPointCloud (:159-161)
      Pt p;
      std::memcpy(&p.x, base + (size_t)i * step + ox, 4);
      std::memcpy(&p.y, base + (size_t)i * step + oy, 4);
      std::memcpy(&p.z, base + (size_t)i * step + oz, 4);
      p.intensity = 0.f;
      if (!std::isfinite(p.x) || !std::isfinite(p.y) || !std::isfinite(p.z)) continue;
      cloud_in.push_back(p);
    }
    if (cloud_in.empty()) return LEGO_EEMPTY;
    findStartEndAngle();
    projectPointCloud();
    groundRemoval();
    cloudSegmentation();
    return LEGO_OK;
  }
};

// ======================================================================================
// PCL VoxelGrid<PointXYZI>::applyFilter restatement (PCL 1.7/1.8 voxel_grid.hpp; called from
// featureAssociation.cpp:377-379 with leaf 0.2, :101).  downsample_all_data_ = true.
// ======================================================================================
struct cloud_point_index_idx {
  unsigned int idx;
  unsigned int cloud_point_index;
  bool operator<(const cloud_point_index_idx& p) const { return (idx < p.idx); }
};

int voxel_grid(const std::vector<Pt>& in, float leaf, std::vector<Pt>& out, bool stable) {
  out.clear();
  const float inv = 1.0f / leaf;  // inverse_leaf_size_ = Array4f::Ones() / leaf_size_
  // getMinMax3D (dense path): min/max of x,y,z
  float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
  for (size_t i = 0; i < in.size(); ++i) {
    const float v[3] = {in[i].x, in[i].y, in[i].z};
    for (int d = 0; d < 3; ++d) {
      mn[d] = std::min(mn[d], v[d]);
      mx[d] = std::max(mx[d], v[d]);
    }
  }
  if (in.empty()) return 0;
  int64_t dx = static_cast<int64_t>((mx[0] - mn[0]) * inv) + 1;
  int64_t dy = static_cast<int64_t>((mx[1] - mn[1]) * inv) + 1;
  int64_t dz = static_cast<int64_t>((mx[2] - mn[2]) * inv) + 1;
  if ((dx * dy * dz) > static_cast<int64_t>(std::numeric_limits<int32_t>::max())) {
    out = in;  // "Leaf size is too small ... Integer indices would overflow": output = input
    return LEGO_ST_VOXEL_OVERFLOW;
  }
  int min_b[3], max_b[3], div_b[3], divb_mul[3];
  for (int d = 0; d < 3; ++d) {
    min_b[d] = static_cast<int>(std::floor(mn[d] * inv));
    max_b[d] = static_cast<int>(std::floor(mx[d] * inv));
    div_b[d] = max_b[d] - min_b[d] + 1;
  }
  divb_mul[0] = 1; divb_mul[1] = div_b[0]; divb_mul[2] = div_b[0] * div_b[1];
  std::vector<cloud_point_index_idx> iv;
  iv.reserve(in.size());
  for (size_t i = 0; i < in.size(); ++i) {
    int ijk0 = static_cast<int>(std::floor(in[i].x * inv) - static_cast<float>(min_b[0]));
    int ijk1 = static_cast<int>(std::floor(in[i].y * inv) - static_cast<float>(min_b[1]));
    int ijk2 = static_cast<int>(std::floor(in[i].z * inv) - static_cast<float>(min_b[2]));
    // PCL computes this in int and stores it as unsigned int; past 2^31 - 1 (extents its overflow gate,
    // which multiplies the truncated (max - min) / leaf + 1, lets through) the int wraps: the same bits
    // as this unsigned arithmetic, without the signed-overflow UB in the oracle itself
    const unsigned idx = (unsigned)ijk0 * (unsigned)divb_mul[0] + (unsigned)ijk1 * (unsigned)divb_mul[1] +
                         (unsigned)ijk2 * (unsigned)divb_mul[2];
    cloud_point_index_idx e;
    e.idx = idx;
    e.cloud_point_index = (unsigned int)i;
    iv.push_back(e);
  }
  if (const char* dump = std::getenv("LEGO_ORACLE_DUMP_VOXEL_KEYS")) {  // diagnostics: raw keys per call
    if (FILE* f = std::fopen(dump, "ab")) {
      const uint32_t n = (uint32_t)iv.size();
      std::fwrite(&n, 4, 1, f);
      for (const auto& e : iv) std::fwrite(&e.idx, 4, 1, f);
      std::fclose(f);
    }
  }
  if (stable)  // lego_params.voxel_tie_order == 1
    std::stable_sort(iv.begin(), iv.end(), std::less<cloud_point_index_idx>());
  else
    std::sort(iv.begin(), iv.end(), std::less<cloud_point_index_idx>());
  unsigned int index = 0;
  while (index < iv.size()) {
    unsigned int i = index + 1;
    while (i < iv.size() && iv[i].idx == iv[index].idx) ++i;
    // CentroidPoint<PointXYZI>: float sums in sorted order, / n
    float sx = 0.f, sy = 0.f, sz = 0.f, si = 0.f;
    for (unsigned int li = index; li < i; ++li) {
      const Pt& p = in[iv[li].cloud_point_index];
      sx += p.x; sy += p.y; sz += p.z; si += p.intensity;
    }
    const float n = static_cast<float>(i - index);
    Pt c;
    c.x = sx / n; c.y = sy / n; c.z = sz / n; c.intensity = si / n;
    out.push_back(c);
    index = i;
  }
  return 0;
}

// ======================================================================================
// Eigen boundary model (unpinned): AtA/AtB summed in double from float products, rounded to
// float; ColPivHouseholderQR<Matrix3f>::solve restated in float; largest eigenvalue of the
// symmetric 3x3 AtA by cyclic Jacobi in double.
// ======================================================================================
void qr_solve3(const float A_in[9], const float b_in[3], float x[3]) {
  float A[9];
  for (int i = 0; i < 9; ++i) A[i] = A_in[i];
  const float eps = FLT_EPSILON;
  float nu[3], nd[3], hc[3];
  int perm[3] = {0, 1, 2};
  for (int k = 0; k < 3; ++k) {
    float s = 0.f;
    for (int r = 0; r < 3; ++r) s += A[r * 3 + k] * A[r * 3 + k];
    nu[k] = nd[k] = sqrtf(s);
  }
  float maxn = std::max(nu[0], std::max(nu[1], nu[2]));
  float th_help = (maxn * eps) * (maxn * eps) / 3.0f;
  float ndt = sqrtf(eps);
  int nzp = 3;
  for (int k = 0; k < 3; ++k) {
    int bc = k;
    for (int j = k + 1; j < 3; ++j)
      if (nu[j] > nu[bc]) bc = j;
    float bsq = nu[bc] * nu[bc];
    if (nzp == 3 && bsq < th_help * float(3 - k)) nzp = k;
    if (bc != k) {
      for (int r = 0; r < 3; ++r) std::swap(A[r * 3 + k], A[r * 3 + bc]);
      std::swap(nu[k], nu[bc]); std::swap(nd[k], nd[bc]); std::swap(perm[k], perm[bc]);
    }
    // makeHouseholderInPlace on A[k..2][k]
    float tail = 0.f;
    for (int r = k + 1; r < 3; ++r) tail += A[r * 3 + k] * A[r * 3 + k];
    float c0 = A[k * 3 + k], tau, beta;
    if (tail <= FLT_MIN) {
      tau = 0.f; beta = c0;
      for (int r = k + 1; r < 3; ++r) A[r * 3 + k] = 0.f;
    } else {
      beta = sqrtf(c0 * c0 + tail);
      if (c0 >= 0.f) beta = -beta;
      for (int r = k + 1; r < 3; ++r) A[r * 3 + k] = A[r * 3 + k] / (c0 - beta);
      tau = (beta - c0) / beta;
    }
    hc[k] = tau;
    A[k * 3 + k] = beta;
    // apply H = I - tau v v^T (v = [1, essential]) to the remaining columns
    if (tau != 0.f) {
      for (int j = k + 1; j < 3; ++j) {
        float t = A[k * 3 + j];
        for (int r = k + 1; r < 3; ++r) t += A[r * 3 + k] * A[r * 3 + j];
        A[k * 3 + j] -= tau * t;
        for (int r = k + 1; r < 3; ++r) A[r * 3 + j] -= tau * A[r * 3 + k] * t;
      }
    }
    for (int j = k + 1; j < 3; ++j) {
      if (nu[j] != 0.f) {
        float t = std::fabs(A[k * 3 + j]) / nu[j];
        t = (1.f + t) * (1.f - t);
        if (t < 0.f) t = 0.f;
        float q = nu[j] / nd[j];
        float t2 = t * q * q;
        if (t2 <= ndt) {
          float s = 0.f;
          for (int r = k + 1; r < 3; ++r) s += A[r * 3 + j] * A[r * 3 + j];
          nd[j] = sqrtf(s);
          nu[j] = nd[j];
        } else {
          nu[j] *= sqrtf(t);
        }
      }
    }
  }
  float c[3] = {b_in[0], b_in[1], b_in[2]};
  for (int k = 0; k < nzp; ++k) {  // apply H_k^T (= H_k) in order
    if (hc[k] == 0.f) continue;
    float t = c[k];
    for (int r = k + 1; r < 3; ++r) t += A[r * 3 + k] * c[r];
    c[k] -= hc[k] * t;
    for (int r = k + 1; r < 3; ++r) c[r] -= hc[k] * A[r * 3 + k] * t;
  }
  float y[3] = {0.f, 0.f, 0.f};
  for (int i = nzp - 1; i >= 0; --i) {
    float t = c[i];
    for (int j = i + 1; j < nzp; ++j) t -= A[i * 3 + j] * y[j];
    y[i] = t / A[i * 3 + i];
  }
  for (int i = 0; i < 3; ++i) x[perm[i]] = y[i];
}

double eig_max_sym3(const float Af[9]) {
  double a[3][3];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) a[i][j] = Af[i * 3 + j];
  for (int sweep = 0; sweep < 32; ++sweep) {
    double off = a[0][1] * a[0][1] + a[0][2] * a[0][2] + a[1][2] * a[1][2];
    if (off == 0.0) break;
    for (int p = 0; p < 2; ++p)
      for (int q = p + 1; q < 3; ++q) {
        if (a[p][q] == 0.0) continue;
        double theta = (a[q][q] - a[p][p]) / (2.0 * a[p][q]);
        double t = (theta >= 0 ? 1.0 : -1.0) / (std::fabs(theta) + std::sqrt(theta * theta + 1.0));
        double c = 1.0 / std::sqrt(t * t + 1.0), s = t * c;
        for (int k = 0; k < 3; ++k) {  // A = J^T A J
          double akp = a[k][p], akq = a[k][q];
          a[k][p] = c * akp - s * akq;
          a[k][q] = s * akp + c * akq;
        }
        for (int k = 0; k < 3; ++k) {
          double apk = a[p][k], aqk = a[q][k];
          a[p][k] = c * apk - s * aqk;
          a[q][k] = s * apk + c * aqk;
        }
      }
  }
  return std::max(a[0][0], std::max(a[1][1], a[2][2]));
}

// ======================================================================================
// FeatureAssociation (featureAssociation.cpp)
// ======================================================================================
struct FeatureAssociation {
  int V, H;
  float scan_period, edge_thr, surf_thr, nn_dist_sqr;
  int map_div;
  // persistent work arrays, sized V*H once (fa.cpp:96-118), never cleared outside [5, M-6)
  std::vector<smoothness_t> cloudSmoothness;
  std::vector<float> cloudCurvature;
  std::vector<int> cloudNeighborPicked;
  std::vector<int> cloudLabel;
  std::vector<float> pointSearchCornerInd1, pointSearchCornerInd2;
  std::vector<float> pointSearchSurfInd1, pointSearchSurfInd2, pointSearchSurfInd3;
  // current scan
  std::vector<Pt> segmented, outlier;
  int32_t M;
  std::vector<int32_t> start_ring, end_ring;
  float start_ori, end_ori, ori_diff;
  std::vector<uint8_t> seg_ground;   // sized V*H, tail false (resetParameters :137)
  std::vector<uint32_t> seg_col;     // sized V*H, tail 0
  std::vector<float> seg_range;      // sized V*H, tail 0
  std::vector<Pt> sharp, less_sharp, flat, less_flat, less_flat_scan, less_flat_scan_ds;
  std::vector<int32_t> sharp_ind, less_sharp_ind, flat_ind;
  std::vector<Pt> corner_last, surf_last;
  std::vector<Pt> laserCloudOri, coeffSel;
  int laserCloudCornerLastNum = 0, laserCloudSurfLastNum = 0;
  bool tree_stale = false;
  float transformCur[6], transformSum[6];
  bool systemInitedLM = false;
  bool isDegenerate = false;
  size_t cycle_count = 0;
  int status = 0;
  int iters_surf = 0, iters_corner = 0;
  double quat[4] = {0, 0, 0, 1}, pos[3] = {0, 0, 0};

  bool voxel_stable = false;  // lego_params.voxel_tie_order == 1 (std::stable_sort in VoxelGrid)
  bool fp1 = false;           // lego_params.fp_mode == 1 (double libm overloads)

  explicit FeatureAssociation(const lego_params& p) {  // ctor :69-84 + initializationValue :96-157
    V = p.num_vertical_scans;
    H = p.num_horizontal_scans;
    scan_period = p.scan_period;
    edge_thr = p.edge_threshold;
    surf_thr = p.surf_threshold;
    map_div = p.mapping_frequency_divider;
    voxel_stable = p.voxel_tie_order == 1;
    fp1 = p.fp_mode == 1;
    float nearest_dist = p.nearest_feature_search_distance;
    nn_dist_sqr = nearest_dist * nearest_dist;
    const size_t n = (size_t)V * H;
    cloudSmoothness.resize(n);  // value-initialised {0, 0}
    cloudCurvature.resize(n);
    cloudNeighborPicked.resize(n);
    cloudLabel.resize(n);
    pointSearchCornerInd1.resize(n); pointSearchCornerInd2.resize(n);
    pointSearchSurfInd1.resize(n); pointSearchSurfInd2.resize(n); pointSearchSurfInd3.resize(n);
    for (int i = 0; i < 6; ++i) transformCur[i] = transformSum[i] = 0;
  }

  void adjustDistortion() {  // :161-197
    bool halfPassed = false;
    int cloudSize = (int)segmented.size();
    Pt point;
    for (int i = 0; i < cloudSize; i++) {
      point.x = segmented[i].y;
      point.y = segmented[i].z;
      point.z = segmented[i].x;
      float ori = fp1 ? (float)(-atan2((double)point.x, (double)point.z)) : -atan2f(point.x, point.z);
      if (!halfPassed) {
        if (ori < start_ori - M_PI / 2)
          ori += 2 * M_PI;
        else if (ori > start_ori + M_PI * 3 / 2)
          ori -= 2 * M_PI;
        if (ori - start_ori > M_PI) halfPassed = true;
      } else {
        ori += 2 * M_PI;
        if (ori < end_ori - M_PI * 3 / 2)
          ori += 2 * M_PI;
        else if (ori > end_ori + M_PI / 2)
          ori -= 2 * M_PI;
      }
      float relTime = (ori - start_ori) / ori_diff;
      point.intensity = int(segmented[i].intensity) + scan_period * relTime;
      segmented[i] = point;
    }
  }

  void calculateSmoothness() {  // :200-223
    int cloudSize = (int)segmented.size();
    const float* r = seg_range.data();
    for (int i = 5; i < cloudSize - 5; i++) {
      float diffRange = r[i - 5] + r[i - 4] + r[i - 3] + r[i - 2] + r[i - 1] - r[i] * 10 + r[i + 1] +
                        r[i + 2] + r[i + 3] + r[i + 4] + r[i + 5];
      cloudCurvature[i] = diffRange * diffRange;
      cloudNeighborPicked[i] = 0;
      cloudLabel[i] = 0;
      cloudSmoothness[i].value = cloudCurvature[i];
      cloudSmoothness[i].ind = i;
    }
  }

  void markOccludedPoints() {  // :226-262
    int cloudSize = (int)segmented.size();
    const float* r = seg_range.data();
    for (int i = 5; i < cloudSize - 6; ++i) {
      float depth1 = r[i];
      float depth2 = r[i + 1];
      int columnDiff = std::abs(int(seg_col[i + 1] - seg_col[i]));
      if (columnDiff < 10) {
        if (depth1 - depth2 > 0.3) {
          for (int k = 5; k >= 0; --k) cloudNeighborPicked[i - k] = 1;
        } else if (depth2 - depth1 > 0.3) {
          for (int k = 1; k <= 6; ++k) cloudNeighborPicked[i + k] = 1;
        }
      }
      float diff1 = std::abs(r[i - 1] - r[i]);
      float diff2 = std::abs(r[i + 1] - r[i]);
      if (diff1 > 0.02 * r[i] && diff2 > 0.02 * r[i]) cloudNeighborPicked[i] = 1;
    }
  }

  Pt seg_point(int ind) {  // segmentedCloud->points[ind]; ind >= M is reference UB
    if (ind >= 0 && ind < (int)segmented.size()) return segmented[ind];
    status |= LEGO_ST_STALE_IND_OOB;
    Pt z = {0.f, 0.f, 0.f, 0.f};
    return z;
  }

  void suppress(int ind) {  // :306-326 / :344-366
    const size_t colSize = (size_t)V * H;  // segmentedCloudColInd.size()
    cloudNeighborPicked[ind] = 1;
    for (int l = 1; l <= 5; l++) {
      if ((size_t)(ind + l) >= colSize) continue;
      int columnDiff = std::abs(int(seg_col[ind + l] - seg_col[ind + l - 1]));
      if (columnDiff > 10) break;
      cloudNeighborPicked[ind + l] = 1;
    }
    for (int l = -1; l >= -5; l--) {
      if (ind + l < 0) continue;
      int columnDiff = std::abs(int(seg_col[ind + l] - seg_col[ind + l + 1]));
      if (columnDiff > 10) break;
      cloudNeighborPicked[ind + l] = 1;
    }
  }

  void extractFeatures() {  // :265-383
    sharp.clear(); less_sharp.clear(); flat.clear(); less_flat.clear();
    sharp_ind.clear(); less_sharp_ind.clear(); flat_ind.clear();
    for (int i = 0; i < V; i++) {
      less_flat_scan.clear();
      for (int j = 0; j < 6; j++) {
        int sp = (start_ring[i] * (6 - j) + end_ring[i] * j) / 6;
        int ep = (start_ring[i] * (5 - j) + end_ring[i] * (j + 1)) / 6 - 1;
        if (sp >= ep) continue;
        std::sort(cloudSmoothness.begin() + sp, cloudSmoothness.begin() + ep, by_value());
        int largestPickedNum = 0;
        for (int k = ep; k >= sp; k--) {
          int ind = cloudSmoothness[k].ind;
          if (cloudNeighborPicked[ind] == 0 && cloudCurvature[ind] > edge_thr && seg_ground[ind] == false) {
            largestPickedNum++;
            if (largestPickedNum <= 2) {
              cloudLabel[ind] = 2;
              sharp.push_back(seg_point(ind)); sharp_ind.push_back(ind);
              less_sharp.push_back(seg_point(ind)); less_sharp_ind.push_back(ind);
            } else if (largestPickedNum <= 20) {
              cloudLabel[ind] = 1;
              less_sharp.push_back(seg_point(ind)); less_sharp_ind.push_back(ind);
            } else {
              break;
            }
            suppress(ind);
          }
        }
        int smallestPickedNum = 0;
        for (int k = sp; k <= ep; k++) {
          int ind = cloudSmoothness[k].ind;
          if (cloudNeighborPicked[ind] == 0 && cloudCurvature[ind] < surf_thr && seg_ground[ind] == true) {
            cloudLabel[ind] = -1;
            flat.push_back(seg_point(ind)); flat_ind.push_back(ind);
            smallestPickedNum++;
            if (smallestPickedNum >= 4) break;
            suppress(ind);
          }
        }
        for (int k = sp; k <= ep; k++)
          if (cloudLabel[k] <= 0) less_flat_scan.push_back(seg_point(k));
      }
      status |= voxel_grid(less_flat_scan, 0.2f, less_flat_scan_ds, voxel_stable);
      less_flat.insert(less_flat.end(), less_flat_scan_ds.begin(), less_flat_scan_ds.end());
    }
  }

  // TransformToStart / TransformToEnd / AccumulateRotation / integrateTransformation: unqualified
  // sin / cos / asin / atan2 on floats, evaluated in T (Lm<T>, fp_mode) and rounded where stored to float.
  void TransformToStart(const Pt* pi, Pt* po) {
    if (fp1) TransformToStartT<double>(pi, po); else TransformToStartT<float>(pi, po);
  }
  void TransformToEnd(const Pt* pi, Pt* po) {
    if (fp1) TransformToEndT<double>(pi, po); else TransformToEndT<float>(pi, po);
  }

  template <class T>
  void TransformToStartT(const Pt* pi, Pt* po) {  // :388-418
    typedef Lm<T> F;
    float s = 10 * (pi->intensity - int(pi->intensity));
    float ry = s * transformCur[1];
    float rx = s * transformCur[0];
    float rz = s * transformCur[2];
    float tx = s * transformCur[3];
    float ty = s * transformCur[4];
    float tz = s * transformCur[5];
    float x1 = F::cs(rz) * (T)(pi->x - tx) + F::sn(rz) * (T)(pi->y - ty);
    float y1 = -F::sn(rz) * (T)(pi->x - tx) + F::cs(rz) * (T)(pi->y - ty);
    float z1 = (pi->z - tz);
    float x2 = x1;
    float y2 = F::cs(rx) * (T)y1 + F::sn(rx) * (T)z1;
    float z2 = -F::sn(rx) * (T)y1 + F::cs(rx) * (T)z1;
    po->x = F::cs(ry) * (T)x2 - F::sn(ry) * (T)z2;
    po->y = y2;
    po->z = F::sn(ry) * (T)x2 + F::cs(ry) * (T)z2;
    po->intensity = pi->intensity;
  }

  template <class T>
  void TransformToEndT(const Pt* pi, Pt* po) {  // :422-471
    typedef Lm<T> F;
    float s = 10 * (pi->intensity - int(pi->intensity));
    float rx = s * transformCur[0];
    float ry = s * transformCur[1];
    float rz = s * transformCur[2];
    float tx = s * transformCur[3];
    float ty = s * transformCur[4];
    float tz = s * transformCur[5];
    float x1 = F::cs(rz) * (T)(pi->x - tx) + F::sn(rz) * (T)(pi->y - ty);
    float y1 = -F::sn(rz) * (T)(pi->x - tx) + F::cs(rz) * (T)(pi->y - ty);
    float z1 = (pi->z - tz);
    float x2 = x1;
    float y2 = F::cs(rx) * (T)y1 + F::sn(rx) * (T)z1;
    float z2 = -F::sn(rx) * (T)y1 + F::cs(rx) * (T)z1;
    float x3 = F::cs(ry) * (T)x2 - F::sn(ry) * (T)z2;
    float y3 = y2;
    float z3 = F::sn(ry) * (T)x2 + F::cs(ry) * (T)z2;
    rx = transformCur[0];
    ry = transformCur[1];
    rz = transformCur[2];
    tx = transformCur[3];
    ty = transformCur[4];
    tz = transformCur[5];
    float x4 = F::cs(ry) * (T)x3 + F::sn(ry) * (T)z3;
    float y4 = y3;
    float z4 = -F::sn(ry) * (T)x3 + F::cs(ry) * (T)z3;
    float x5 = x4;
    float y5 = F::cs(rx) * (T)y4 - F::sn(rx) * (T)z4;
    float z5 = F::sn(rx) * (T)y4 + F::cs(rx) * (T)z4;
    float x6 = F::cs(rz) * (T)x5 - F::sn(rz) * (T)y5 + (T)tx;
    float y6 = F::sn(rz) * (T)x5 + F::cs(rz) * (T)y5 + (T)ty;
    float z6 = z5 + tz;
    po->x = x6;
    po->y = y6;
    po->z = z6;
    po->intensity = int(pi->intensity);
  }

  template <class T>
  static void AccumulateRotation(float cx, float cy, float cz, float lx, float ly, float lz, float& ox,
                                 float& oy, float& oz) {  // :474-500
    typedef Lm<T> F;
    float srx = F::cs(lx) * F::cs(cx) * F::sn(ly) * F::sn(cz) - F::cs(cx) * F::cs(cz) * F::sn(lx) -
                F::cs(lx) * F::cs(ly) * F::sn(cx);
    ox = -F::as(srx);
    float srycrx = F::sn(lx) * (F::cs(cy) * F::sn(cz) - F::cs(cz) * F::sn(cx) * F::sn(cy)) +
                   F::cs(lx) * F::sn(ly) * (F::cs(cy) * F::cs(cz) + F::sn(cx) * F::sn(cy) * F::sn(cz)) +
                   F::cs(lx) * F::cs(ly) * F::cs(cx) * F::sn(cy);
    float crycrx = F::cs(lx) * F::cs(ly) * F::cs(cx) * F::cs(cy) -
                   F::cs(lx) * F::sn(ly) * (F::cs(cz) * F::sn(cy) - F::cs(cy) * F::sn(cx) * F::sn(cz)) -
                   F::sn(lx) * (F::sn(cy) * F::sn(cz) + F::cs(cy) * F::cs(cz) * F::sn(cx));
    oy = F::at2((T)srycrx / F::cs1(ox), (T)crycrx / F::cs1(ox));
    float srzcrx = F::sn(cx) * (F::cs(lz) * F::sn(ly) - F::cs(ly) * F::sn(lx) * F::sn(lz)) +
                   F::cs(cx) * F::sn(cz) * (F::cs(ly) * F::cs(lz) + F::sn(lx) * F::sn(ly) * F::sn(lz)) +
                   F::cs(lx) * F::cs(cx) * F::cs(cz) * F::sn(lz);
    float crzcrx = F::cs(lx) * F::cs(lz) * F::cs(cx) * F::cs(cz) -
                   F::cs(cx) * F::sn(cz) * (F::cs(ly) * F::sn(lz) - F::cs(lz) * F::sn(lx) * F::sn(ly)) -
                   F::sn(cx) * (F::sn(ly) * F::sn(lz) + F::cs(ly) * F::cs(lz) * F::sn(lx));
    oz = F::at2((T)srzcrx / F::cs1(ox), (T)crzcrx / F::cs1(ox));
  }

  // kdtreeCornerLast / kdtreeSurfLast->nearestKSearch(pointSel, 1, ...) (fa.cpp:512, 650;
  // nanoflann_pcl.h:141-152): nanoflann's kd-tree over the Last cloud (nanoflann_restated.h), built
  // when the LM starts (a pure function of the cloud: the reference builds it in publishCloudsLast /
  // checkSystemInitialization).  Exact distance ties go to the first point the search visits, as in
  // nanoflann; LEGO_ST_NN_TIE reports that one happened (and mattered: the point was accepted).
  nfr::KdTree<Pt> tree_corner, tree_surf;
  int nearest(const nfr::KdTree<Pt>& tree, const Pt& q, float* d_out) {
    const float qv[3] = {q.x, q.y, q.z};
    int best = -1, ties = 0;
    float bd = std::numeric_limits<float>::max();
    if (tree.knn(qv, 1, &best, &bd, &ties) == 0) best = -1;
    if (ties && bd < nn_dist_sqr) status |= LEGO_ST_NN_TIE;
    *d_out = bd;
    return best;
  }

  void findCorrespondingCornerFeatures(int iterCount) {  // :503-637
    int cornerPointsSharpNum = (int)sharp.size();
    for (int i = 0; i < cornerPointsSharpNum; i++) {
      Pt pointSel;
      TransformToStart(&sharp[i], &pointSel);
      if (iterCount % 5 == 0) {
        float sqd;
        int nn = nearest(tree_corner, pointSel, &sqd);
        int closestPointInd = -1, minPointInd2 = -1;
        if (sqd < nn_dist_sqr) {
          closestPointInd = nn;
          int closestPointScan = int(corner_last[closestPointInd].intensity);
          float pointSqDis, minPointSqDis2 = nn_dist_sqr;
          int bound = cornerPointsSharpNum;  // reference bug (:522): bounded by the CURRENT sharp count
          if (bound > laserCloudCornerLastNum) {
            if (closestPointInd + 1 < bound) status |= LEGO_ST_FWD_OOB;
            bound = laserCloudCornerLastNum;  // defined behaviour: never read past |Last|
          }
          for (int j = closestPointInd + 1; j < bound; j++) {
            if (int(corner_last[j].intensity) > closestPointScan + 2.5) break;
            pointSqDis = (corner_last[j].x - pointSel.x) * (corner_last[j].x - pointSel.x) +
                         (corner_last[j].y - pointSel.y) * (corner_last[j].y - pointSel.y) +
                         (corner_last[j].z - pointSel.z) * (corner_last[j].z - pointSel.z);
            if (int(corner_last[j].intensity) > closestPointScan) {
              if (pointSqDis < minPointSqDis2) { minPointSqDis2 = pointSqDis; minPointInd2 = j; }
            }
          }
          for (int j = closestPointInd - 1; j >= 0; j--) {
            if (int(corner_last[j].intensity) < closestPointScan - 2.5) break;
            pointSqDis = (corner_last[j].x - pointSel.x) * (corner_last[j].x - pointSel.x) +
                         (corner_last[j].y - pointSel.y) * (corner_last[j].y - pointSel.y) +
                         (corner_last[j].z - pointSel.z) * (corner_last[j].z - pointSel.z);
            if (int(corner_last[j].intensity) < closestPointScan) {
              if (pointSqDis < minPointSqDis2) { minPointSqDis2 = pointSqDis; minPointInd2 = j; }
            }
          }
        }
        pointSearchCornerInd1[i] = closestPointInd;
        pointSearchCornerInd2[i] = minPointInd2;
      }
      if (pointSearchCornerInd2[i] >= 0) {
        Pt tripod1 = corner_last[(int)pointSearchCornerInd1[i]];
        Pt tripod2 = corner_last[(int)pointSearchCornerInd2[i]];
        float x0 = pointSel.x, y0 = pointSel.y, z0 = pointSel.z;
        float x1 = tripod1.x, y1 = tripod1.y, z1 = tripod1.z;
        float x2 = tripod2.x, y2 = tripod2.y, z2 = tripod2.z;
        float m11 = ((x0 - x1) * (y0 - y2) - (x0 - x2) * (y0 - y1));
        float m22 = ((x0 - x1) * (z0 - z2) - (x0 - x2) * (z0 - z1));
        float m33 = ((y0 - y1) * (z0 - z2) - (y0 - y2) * (z0 - z1));
        float a012 = sqrtf(m11 * m11 + m22 * m22 + m33 * m33);
        float l12 = sqrtf((x1 - x2) * (x1 - x2) + (y1 - y2) * (y1 - y2) + (z1 - z2) * (z1 - z2));
        float la = ((y1 - y2) * m11 + (z1 - z2) * m22) / a012 / l12;
        float lb = -((x1 - x2) * m11 - (z1 - z2) * m33) / a012 / l12;
        float lc = -((x1 - x2) * m22 + (y1 - y2) * m33) / a012 / l12;
        float ld2 = a012 / l12;
        float s = 1;
        if (iterCount >= 5) s = 1 - 1.8 * fabsf(ld2);
        if (s > 0.1 && ld2 != 0) {
          Pt coeff;
          coeff.x = s * la; coeff.y = s * lb; coeff.z = s * lc; coeff.intensity = s * ld2;
          laserCloudOri.push_back(sharp[i]);
          coeffSel.push_back(coeff);
        }
      }
    }
  }

  void findCorrespondingSurfFeatures(int iterCount) {  // :640-779
    int surfPointsFlatNum = (int)flat.size();
    for (int i = 0; i < surfPointsFlatNum; i++) {
      Pt pointSel;
      TransformToStart(&flat[i], &pointSel);
      if (iterCount % 5 == 0) {
        float sqd;
        int nn = nearest(tree_surf, pointSel, &sqd);
        int closestPointInd = -1, minPointInd2 = -1, minPointInd3 = -1;
        if (sqd < nn_dist_sqr) {
          closestPointInd = nn;
          int closestPointScan = int(surf_last[closestPointInd].intensity);
          float pointSqDis, minPointSqDis2 = nn_dist_sqr, minPointSqDis3 = nn_dist_sqr;
          int bound = surfPointsFlatNum;  // reference bug (:661)
          if (bound > laserCloudSurfLastNum) {
            if (closestPointInd + 1 < bound) status |= LEGO_ST_FWD_OOB;
            bound = laserCloudSurfLastNum;
          }
          for (int j = closestPointInd + 1; j < bound; j++) {
            if (int(surf_last[j].intensity) > closestPointScan + 2.5) break;
            pointSqDis = (surf_last[j].x - pointSel.x) * (surf_last[j].x - pointSel.x) +
                         (surf_last[j].y - pointSel.y) * (surf_last[j].y - pointSel.y) +
                         (surf_last[j].z - pointSel.z) * (surf_last[j].z - pointSel.z);
            if (int(surf_last[j].intensity) <= closestPointScan) {
              if (pointSqDis < minPointSqDis2) { minPointSqDis2 = pointSqDis; minPointInd2 = j; }
            } else {
              if (pointSqDis < minPointSqDis3) { minPointSqDis3 = pointSqDis; minPointInd3 = j; }
            }
          }
          for (int j = closestPointInd - 1; j >= 0; j--) {
            if (int(surf_last[j].intensity) < closestPointScan - 2.5) break;
            pointSqDis = (surf_last[j].x - pointSel.x) * (surf_last[j].x - pointSel.x) +
                         (surf_last[j].y - pointSel.y) * (surf_last[j].y - pointSel.y) +
                         (surf_last[j].z - pointSel.z) * (surf_last[j].z - pointSel.z);
            if (int(surf_last[j].intensity) >= closestPointScan) {
              if (pointSqDis < minPointSqDis2) { minPointSqDis2 = pointSqDis; minPointInd2 = j; }
            } else {
              if (pointSqDis < minPointSqDis3) { minPointSqDis3 = pointSqDis; minPointInd3 = j; }
            }
          }
        }
        pointSearchSurfInd1[i] = closestPointInd;
        pointSearchSurfInd2[i] = minPointInd2;
        pointSearchSurfInd3[i] = minPointInd3;
      }
      if (pointSearchSurfInd2[i] >= 0 && pointSearchSurfInd3[i] >= 0) {
        Pt tripod1 = surf_last[(int)pointSearchSurfInd1[i]];
        Pt tripod2 = surf_last[(int)pointSearchSurfInd2[i]];
        Pt tripod3 = surf_last[(int)pointSearchSurfInd3[i]];
        float pa = (tripod2.y - tripod1.y) * (tripod3.z - tripod1.z) - (tripod3.y - tripod1.y) * (tripod2.z - tripod1.z);
        float pb = (tripod2.z - tripod1.z) * (tripod3.x - tripod1.x) - (tripod3.z - tripod1.z) * (tripod2.x - tripod1.x);
        float pc = (tripod2.x - tripod1.x) * (tripod3.y - tripod1.y) - (tripod3.x - tripod1.x) * (tripod2.y - tripod1.y);
        float pd = -(pa * tripod1.x + pb * tripod1.y + pc * tripod1.z);
        float ps = sqrtf(pa * pa + pb * pb + pc * pc);
        pa /= ps; pb /= ps; pc /= ps; pd /= ps;
        float pd2 = pa * pointSel.x + pb * pointSel.y + pc * pointSel.z + pd;
        float s = 1;
        if (iterCount >= 5)
          s = fp1 ? 1 - 1.8 * fabsf(pd2) /
                            sqrt(sqrt((double)(pointSel.x * pointSel.x + pointSel.y * pointSel.y + pointSel.z * pointSel.z)))
                  : 1 - 1.8 * fabsf(pd2) /
                            sqrtf(sqrtf(pointSel.x * pointSel.x + pointSel.y * pointSel.y + pointSel.z * pointSel.z));
        if (s > 0.1 && pd2 != 0) {
          Pt coeff;
          coeff.x = s * pa; coeff.y = s * pb; coeff.z = s * pc; coeff.intensity = s * pd2;
          laserCloudOri.push_back(flat[i]);
          coeffSel.push_back(coeff);
        }
      }
    }
  }

  // float srx = sin(transformCur[0]) (:797-802, :939-944) in either libm model
  float lm_sin(float x) const { return fp1 ? (float)Lm<double>::sn(x) : sinf(x); }
  float lm_cos(float x) const { return fp1 ? (float)Lm<double>::cs(x) : cosf(x); }

  // AtA / AtB (Eigen GEMM, modelled) + solve + degeneracy; returns x[3].  g_float_ne (diagnostic,
  // oracle_set_float_normal_equations): float accumulators in row order instead, a second model of
  // Eigen's float GEMM whose distance from the first measures how much the unpinned order can matter.
  void solve_normal(const std::vector<float>& A, const std::vector<float>& B, int iterCount, float x[3]) {
    const int n = (int)B.size();
    double ata[9] = {0}, atb[3] = {0};
    float ataf[9] = {0}, atbf[3] = {0};
    for (int i = 0; i < n; ++i) {
      const float* a = &A[3 * i];
      for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c) {
          ata[r * 3 + c] += (double)(a[r] * a[c]);
          ataf[r * 3 + c] += a[r] * a[c];
        }
        atb[r] += (double)(a[r] * B[i]);
        atbf[r] += a[r] * B[i];
      }
    }
    float AtA[9], AtB[3];
    for (int k = 0; k < 9; ++k) AtA[k] = g_float_ne ? ataf[k] : (float)ata[k];
    for (int k = 0; k < 3; ++k) AtB[k] = g_float_ne ? atbf[k] : (float)atb[k];
    qr_solve3(AtA, AtB, x);
    if (iterCount == 0) {
      // SelfAdjointEigenSolver + :879-891: degenerate iff the largest eigenvalue < 10, and then every
      // row of matV2 is zeroed, so matP = V^-1 * 0 = 0.
      isDegenerate = eig_max_sym3(AtA) < 10.0;
    } else if (isDegenerate) {
      status |= LEGO_ST_DEGEN_UB;  // matP uninitialised local at iter != 0: member semantics (matP = 0)
    }
    if (isDegenerate) {
      status |= LEGO_ST_DEGENERATE;
      x[0] = x[1] = x[2] = 0.f;
    }
  }

  bool calculateTransformationSurf(int iterCount) {  // :785-921
    int pointSelNum = (int)laserCloudOri.size();
    float srx = lm_sin(transformCur[0]);
    float crx = lm_cos(transformCur[0]);
    float sry = lm_sin(transformCur[1]);
    float cry = lm_cos(transformCur[1]);
    float srz = lm_sin(transformCur[2]);
    float crz = lm_cos(transformCur[2]);
    float tx = transformCur[3];
    float ty = transformCur[4];
    float tz = transformCur[5];
    float a1 = crx * sry * srz;
    float a2 = crx * crz * sry;
    float a3 = srx * sry;
    float a4 = tx * a1 - ty * a2 - tz * a3;
    float a5 = srx * srz;
    float a6 = crz * srx;
    float a7 = ty * a6 - tz * crx - tx * a5;
    float a8 = crx * cry * srz;
    float a9 = crx * cry * crz;
    float a10 = cry * srx;
    float a11 = tz * a10 + ty * a9 - tx * a8;
    float b1 = -crz * sry - cry * srx * srz;
    float b2 = cry * crz * srx - sry * srz;
    float b5 = cry * crz - srx * sry * srz;
    float b6 = cry * srz + crz * srx * sry;
    float c1 = -b6;
    float c2 = b5;
    float c3 = tx * b6 - ty * b5;
    float c4 = -crx * crz;
    float c5 = crx * srz;
    float c6 = ty * c5 + tx * -c4;
    float c7 = b2;
    float c8 = -b1;
    float c9 = tx * -b2 - ty * -b1;
    std::vector<float> A(3 * pointSelNum), B(pointSelNum);
    for (int i = 0; i < pointSelNum; i++) {
      Pt pointOri = laserCloudOri[i];
      Pt coeff = coeffSel[i];
      float arx = (-a1 * pointOri.x + a2 * pointOri.y + a3 * pointOri.z + a4) * coeff.x +
                  (a5 * pointOri.x - a6 * pointOri.y + crx * pointOri.z + a7) * coeff.y +
                  (a8 * pointOri.x - a9 * pointOri.y - a10 * pointOri.z + a11) * coeff.z;
      float arz = (c1 * pointOri.x + c2 * pointOri.y + c3) * coeff.x +
                  (c4 * pointOri.x - c5 * pointOri.y + c6) * coeff.y +
                  (c7 * pointOri.x + c8 * pointOri.y + c9) * coeff.z;
      float aty = -b6 * coeff.x + c4 * coeff.y + b2 * coeff.z;
      float d2 = coeff.intensity;
      A[3 * i + 0] = arx; A[3 * i + 1] = arz; A[3 * i + 2] = aty;
      B[i] = -0.05 * d2;
    }
    float x[3];
    solve_normal(A, B, iterCount, x);
    transformCur[0] += x[0];
    transformCur[2] += x[1];
    transformCur[4] += x[2];
    for (int i = 0; i < 6; i++)
      if (std::isnan(transformCur[i])) transformCur[i] = 0;
    float deltaR = sqrt(pow(RAD2DEG * (x[0]), 2) + pow(RAD2DEG * (x[1]), 2));
    float deltaT = sqrt(pow(x[2] * 100, 2));
    if (deltaR < 0.1 && deltaT < 0.1) return false;
    return true;
  }

  bool calculateTransformationCorner(int iterCount) {  // :928-1032
    int pointSelNum = (int)laserCloudOri.size();
    float srx = lm_sin(transformCur[0]);
    float crx = lm_cos(transformCur[0]);
    float sry = lm_sin(transformCur[1]);
    float cry = lm_cos(transformCur[1]);
    float srz = lm_sin(transformCur[2]);
    float crz = lm_cos(transformCur[2]);
    float tx = transformCur[3];
    float ty = transformCur[4];
    float tz = transformCur[5];
    float b1 = -crz * sry - cry * srx * srz;
    float b2 = cry * crz * srx - sry * srz;
    float b3 = crx * cry;
    float b4 = tx * -b1 + ty * -b2 + tz * b3;
    float b5 = cry * crz - srx * sry * srz;
    float b6 = cry * srz + crz * srx * sry;
    float b7 = crx * sry;
    float b8 = tz * b7 - ty * b6 - tx * b5;
    float c5 = crx * srz;
    std::vector<float> A(3 * pointSelNum), B(pointSelNum);
    for (int i = 0; i < pointSelNum; i++) {
      Pt pointOri = laserCloudOri[i];
      Pt coeff = coeffSel[i];
      float ary = (b1 * pointOri.x + b2 * pointOri.y - b3 * pointOri.z + b4) * coeff.x +
                  (b5 * pointOri.x + b6 * pointOri.y - b7 * pointOri.z + b8) * coeff.z;
      float atx = -b5 * coeff.x + c5 * coeff.y + b1 * coeff.z;
      float atz = b7 * coeff.x - srx * coeff.y - b3 * coeff.z;
      float d2 = coeff.intensity;
      A[3 * i + 0] = ary; A[3 * i + 1] = atx; A[3 * i + 2] = atz;
      B[i] = -0.05 * d2;
    }
    float x[3];
    solve_normal(A, B, iterCount, x);
    transformCur[1] += x[0];
    transformCur[3] += x[1];
    transformCur[5] += x[2];
    for (int i = 0; i < 6; i++)
      if (std::isnan(transformCur[i])) transformCur[i] = 0;
    float deltaR = sqrt(pow(RAD2DEG * (x[0]), 2));
    float deltaT = sqrt(pow(x[1] * 100, 2) + pow(x[2] * 100, 2));
    if (deltaR < 0.1 && deltaT < 0.1) return false;
    return true;
  }

  void checkSystemInitialization() {  // :1181-1209
    corner_last = less_sharp;
    surf_last = less_flat;
    laserCloudCornerLastNum = (int)corner_last.size();
    laserCloudSurfLastNum = (int)surf_last.size();
    tree_stale = false;  // trees built unconditionally (:1190-1191)
    systemInitedLM = true;
  }

  void updateTransformation() {  // :1213-1235
    if (laserCloudCornerLastNum < 10 || laserCloudSurfLastNum < 100) {
      status |= LEGO_ST_LM_SKIPPED;
      return;
    }
    if (tree_stale) status |= LEGO_ST_STALE_TREE;  // defined behaviour: search the Last cloud anyway
    tree_corner.build(corner_last.data(), laserCloudCornerLastNum);
    tree_surf.build(surf_last.data(), laserCloudSurfLastNum);
    for (int iterCount1 = 0; iterCount1 < 25; iterCount1++) {
      laserCloudOri.clear();
      coeffSel.clear();
      findCorrespondingSurfFeatures(iterCount1);
      iters_surf = iterCount1 + 1;
      if (laserCloudOri.size() < 10) continue;
      if (calculateTransformationSurf(iterCount1) == false) break;
    }
    for (int iterCount2 = 0; iterCount2 < 25; iterCount2++) {
      laserCloudOri.clear();
      coeffSel.clear();
      findCorrespondingCornerFeatures(iterCount2);
      iters_corner = iterCount2 + 1;
      if (laserCloudOri.size() < 10) continue;
      if (calculateTransformationCorner(iterCount2) == false) break;
    }
  }

  void integrateTransformation() {
    if (fp1) integrateTransformationT<double>(); else integrateTransformationT<float>();
  }
  template <class T>
  void integrateTransformationT() {  // :1241-1270
    typedef Lm<T> F;
    float rx, ry, rz, tx, ty, tz;
    AccumulateRotation<T>(transformSum[0], transformSum[1], transformSum[2], -transformCur[0], -transformCur[1],
                          -transformCur[2], rx, ry, rz);
    float x1 = F::cs(rz) * (T)(transformCur[3]) - F::sn(rz) * (T)(transformCur[4]);
    float y1 = F::sn(rz) * (T)(transformCur[3]) + F::cs(rz) * (T)(transformCur[4]);
    float z1 = transformCur[5];
    float x2 = x1;
    float y2 = F::cs(rx) * (T)y1 - F::sn(rx) * (T)z1;
    float z2 = F::sn(rx) * (T)y1 + F::cs(rx) * (T)z1;
    tx = (T)transformSum[3] - (F::cs(ry) * (T)x2 + F::sn(ry) * (T)z2);
    ty = transformSum[4] - y2;
    tz = (T)transformSum[5] - (-F::sn(ry) * (T)x2 + F::cs(ry) * (T)z2);
    transformSum[0] = rx; transformSum[1] = ry; transformSum[2] = rz;
    transformSum[3] = tx; transformSum[4] = ty; transformSum[5] = tz;
  }

  void publishOdometry() {  // :1286-1298, tf::createQuaternionMsgFromRollPitchYaw (double)
    double roll = transformSum[2], pitch = -transformSum[0], yaw = -transformSum[1];
    double hy = yaw * 0.5, hp = pitch * 0.5, hr = roll * 0.5;
    double cy = cos(hy), sy = sin(hy), cp = cos(hp), sp = sin(hp), cr = cos(hr), sr = sin(hr);
    double qx = sr * cp * cy - cr * sp * sy;
    double qy = cr * sp * cy + sr * cp * sy;
    double qz = cr * cp * sy - sr * sp * cy;
    double qw = cr * cp * cy + sr * sp * sy;
    quat[0] = -qy; quat[1] = -qz; quat[2] = qx; quat[3] = qw;
    pos[0] = transformSum[3]; pos[1] = transformSum[4]; pos[2] = transformSum[5];
  }

  void publishCloudsLast() {  // :1329-1383
    // TransformToEnd in place on lessSharp/lessFlat, then swap into *Last.  Restated out of place so
    // the pre-transform feature clouds stay readable (TransformToEnd reads all of pi before writing).
    corner_last.resize(less_sharp.size());
    for (size_t i = 0; i < less_sharp.size(); i++) TransformToEnd(&less_sharp[i], &corner_last[i]);
    surf_last.resize(less_flat.size());
    for (size_t i = 0; i < less_flat.size(); i++) TransformToEnd(&less_flat[i], &surf_last[i]);
    laserCloudCornerLastNum = (int)corner_last.size();
    laserCloudSurfLastNum = (int)surf_last.size();
    tree_stale = !(laserCloudCornerLastNum > 10 && laserCloudSurfLastNum > 100);
    for (size_t i = 0; i < outlier.size(); ++i) {  // adjustOutlierCloud :1273-1283
      Pt p = outlier[i], q;
      q.x = p.y; q.y = p.z; q.z = p.x; q.intensity = p.intensity;
      outlier[i] = q;
    }
  }

  int run() {  // one runFeatureAssociation iteration :1394-1448
    status = 0;
    iters_surf = iters_corner = 0;
    adjustDistortion();
    calculateSmoothness();
    markOccludedPoints();
    extractFeatures();
    if (!systemInitedLM) {
      checkSystemInitialization();
      status |= LEGO_ST_INIT;
      return LEGO_OK;
    }
    updateTransformation();
    integrateTransformation();
    publishOdometry();
    publishCloudsLast();
    cycle_count++;
    if ((int)cycle_count == map_div) {
      cycle_count = 0;
      status |= LEGO_ST_EMITTED;
    }
    return LEGO_OK;
  }

  void load_projection(const lego_projection_out* in) {  // _input_channel.receive (:1389-1397)
    const size_t n = (size_t)V * H;
    M = in->n_segmented;
    segmented.assign(in->segmented_cloud, in->segmented_cloud + M);
    outlier.assign(in->outlier_cloud, in->outlier_cloud + in->n_outlier);
    start_ring.assign(in->start_ring_index, in->start_ring_index + V);
    end_ring.assign(in->end_ring_index, in->end_ring_index + V);
    start_ori = in->start_orientation; end_ori = in->end_orientation; ori_diff = in->orientation_diff;
    seg_ground.assign(n, 0); seg_col.assign(n, 0); seg_range.assign(n, 0.f);
    std::copy(in->segmented_cloud_ground_flag, in->segmented_cloud_ground_flag + M, seg_ground.begin());
    std::copy(in->segmented_cloud_col_ind, in->segmented_cloud_col_ind + M, seg_col.begin());
    std::copy(in->segmented_cloud_range, in->segmented_cloud_range + M, seg_range.begin());
  }
};

}  // namespace

struct oracle_ctx {
  lego_params p;
  ImageProjection ip;
  FeatureAssociation fa;
  explicit oracle_ctx(const lego_params& q) : p(q), ip(q), fa(q) {}
};

extern "C" {

oracle_ctx* oracle_create(const lego_params* p) {
  if (!p || p->num_vertical_scans < 2 || p->num_horizontal_scans < 16) return nullptr;
  return new oracle_ctx(*p);
}

void oracle_destroy(oracle_ctx* c) { delete c; }

int oracle_cloud_handler(oracle_ctx* c, const void* pts, int n, int step, int ox, int oy, int oz,
                         lego_projection_out* out) {
  int rc = c->ip.cloudHandler(pts, n, step, ox, oy, oz);
  if (rc != LEGO_OK) return rc;
  ImageProjection& ip = c->ip;
  out->n_segmented = (int)ip.segmented.size();
  out->n_outlier = (int)ip.outlier.size();
  out->n_scan = (int)ip.scan_msg.size();
  out->segmented_cloud = ip.segmented.data();
  out->outlier_cloud = ip.outlier.data();
  out->scan_msg = ip.scan_msg.data();
  out->start_ring_index = ip.start_ring.data();
  out->end_ring_index = ip.end_ring.data();
  out->start_orientation = ip.start_ori;
  out->end_orientation = ip.end_ori;
  out->orientation_diff = ip.ori_diff;
  out->segmented_cloud_ground_flag = ip.seg_ground.data();
  out->segmented_cloud_col_ind = ip.seg_col.data();
  out->segmented_cloud_range = ip.seg_range.data();
  out->label_mat = ip.label_mat.data();
  out->ground_mat = ip.ground_mat.data();
  out->range_mat = ip.range_mat.data();
  return LEGO_OK;
}

static void fill_assoc(FeatureAssociation& fa, lego_association_out* out) {
  out->status = fa.status;
  out->n_sharp = (int)fa.sharp.size();
  out->n_less_sharp = (int)fa.less_sharp.size();
  out->n_flat = (int)fa.flat.size();
  out->n_less_flat = (int)fa.less_flat.size();
  out->corner_points_sharp = fa.sharp.data();
  out->corner_points_less_sharp = fa.less_sharp.data();  // before TransformToEnd
  out->surf_points_flat = fa.flat.data();
  out->surf_points_less_flat = fa.less_flat.data();      // before TransformToEnd
  out->sharp_ind = fa.sharp_ind.data();
  out->less_sharp_ind = fa.less_sharp_ind.data();
  out->flat_ind = fa.flat_ind.data();
  for (int i = 0; i < 6; ++i) {
    out->transform_cur[i] = fa.transformCur[i];
    out->transform_sum[i] = fa.transformSum[i];
  }
  for (int i = 0; i < 4; ++i) out->odom_orientation[i] = fa.quat[i];
  for (int i = 0; i < 3; ++i) out->odom_position[i] = fa.pos[i];
  out->lm_iter_surf = fa.iters_surf;
  out->lm_iter_corner = fa.iters_corner;
  out->n_corner_last = (int)fa.corner_last.size();
  out->n_surf_last = (int)fa.surf_last.size();
  out->n_outlier_last = (int)fa.outlier.size();
  out->cloud_corner_last = fa.corner_last.data();
  out->cloud_surf_last = fa.surf_last.data();
  out->cloud_outlier_last = fa.outlier.data();
}

int oracle_feature_association_from(oracle_ctx* c, const lego_projection_out* in, lego_association_out* out) {
  c->fa.load_projection(in);
  int rc = c->fa.run();
  if (rc != LEGO_OK) return rc;
  fill_assoc(c->fa, out);
  return LEGO_OK;
}

int oracle_feature_association(oracle_ctx* c, lego_association_out* out) {
  lego_projection_out p;
  ImageProjection& ip = c->ip;
  p.n_segmented = (int)ip.segmented.size();
  p.n_outlier = (int)ip.outlier.size();
  p.n_scan = (int)ip.scan_msg.size();
  p.segmented_cloud = ip.segmented.data();
  p.outlier_cloud = ip.outlier.data();
  p.scan_msg = ip.scan_msg.data();
  p.start_ring_index = ip.start_ring.data();
  p.end_ring_index = ip.end_ring.data();
  p.start_orientation = ip.start_ori;
  p.end_orientation = ip.end_ori;
  p.orientation_diff = ip.ori_diff;
  p.segmented_cloud_ground_flag = ip.seg_ground.data();
  p.segmented_cloud_col_ind = ip.seg_col.data();
  p.segmented_cloud_range = ip.seg_range.data();
  return oracle_feature_association_from(c, &p, out);
}

// Test hook: the FA persistent smoothness array (value, ind) for the stale-state tests.
int oracle_smoothness(oracle_ctx* c, int k, float* value, int64_t* ind) {
  if (k < 0 || (size_t)k >= c->fa.cloudSmoothness.size()) return LEGO_EINVAL;
  *value = c->fa.cloudSmoothness[k].value;
  *ind = (int64_t)c->fa.cloudSmoothness[k].ind;
  return LEGO_OK;
}

// Test hook: overwrite the LM state the next association starts from (lego_test_set_lm_state's
// counterpart): transformCur / transformSum, isDegenerate, the Last clouds and the trees' staleness.
int oracle_set_lm_state(oracle_ctx* c, const float* cur, const float* sum, int32_t degenerate, const float* corner,
                        int32_t n_corner, const float* surf, int32_t n_surf, int32_t tree_stale) {
  FeatureAssociation& f = c->fa;
  if (!f.systemInitedLM) return LEGO_EINVAL;
  for (int k = 0; k < 6; ++k) { f.transformCur[k] = cur[k]; f.transformSum[k] = sum[k]; }
  f.isDegenerate = degenerate != 0;
  f.corner_last.assign((const Pt*)corner, (const Pt*)corner + n_corner);
  f.surf_last.assign((const Pt*)surf, (const Pt*)surf + n_surf);
  f.laserCloudCornerLastNum = n_corner;
  f.laserCloudSurfLastNum = n_surf;
  f.tree_stale = tree_stale != 0;
  return LEGO_OK;
}

// Test hook: the LM members that are not in the AssociationOut (featureAssociation.h:115, the kd-tree
// rebuild flag of :1356): isDegenerate and "trees stale" after the last call.
int oracle_lm_flags(oracle_ctx* c, int32_t* degenerate, int32_t* tree_stale) {
  *degenerate = c->fa.isDegenerate ? 1 : 0;
  *tree_stale = c->fa.tree_stale ? 1 : 0;
  return LEGO_OK;
}

// Test hook: libstdc++ std::sort of (key, val) pairs by key only (the reference's sort semantics).
int oracle_std_sort(uint32_t* keys, int32_t* vals, int n, int is_float) {
  if (is_float) {
    std::vector<smoothness_t> v(n);
    for (int i = 0; i < n; ++i) { std::memcpy(&v[i].value, &keys[i], 4); v[i].ind = (size_t)vals[i]; }
    std::sort(v.begin(), v.end(), by_value());
    for (int i = 0; i < n; ++i) { std::memcpy(&keys[i], &v[i].value, 4); vals[i] = (int32_t)v[i].ind; }
  } else {
    std::vector<cloud_point_index_idx> v(n);
    for (int i = 0; i < n; ++i) { v[i].idx = keys[i]; v[i].cloud_point_index = (unsigned)vals[i]; }
    std::sort(v.begin(), v.end(), std::less<cloud_point_index_idx>());
    for (int i = 0; i < n; ++i) { keys[i] = v[i].idx; vals[i] = (int32_t)v[i].cloud_point_index; }
  }
  return 0;
}

// Test hook: nanoflann k-NN (the restated tree) of m queries against a cloud of n points (x, y, z, w
// float32 each): idx / dist [m][k], nearest first; returns 0.
int oracle_knn_tree(const float* cloud, int n, const float* q, int m, int k, int32_t* idx, float* dist) {
  nfr::KdTree<Pt> t;
  t.build((const Pt*)cloud, n);
  for (int i = 0; i < m; ++i) {
    for (int j = 0; j < k; ++j) { idx[(size_t)i * k + j] = -1; dist[(size_t)i * k + j] = 0.f; }
    t.knn(q + (size_t)4 * i, k, idx + (size_t)i * k, dist + (size_t)i * k);
  }
  return 0;
}

// Test hooks for the libm restatement: glibc's float functions as the reference calls them.
float oracle_atan2f(float y, float x) { return atan2f(y, x); }
float oracle_asinf(float x) { return asinf(x); }

// pcl::VoxelGrid<PointXYZI>::filter (the restatement above) of one cloud: out needs room for n points.
// stable: std::stable_sort's tie order (voxel_tie_order 1) instead of std::sort's.  Returns the status
// bits (LEGO_ST_VOXEL_OVERFLOW) and the output size in *n_out.
int oracle_voxel_grid(const float* in, int n, float leaf, int stable, float* out, int* n_out) {
  std::vector<Pt> v((size_t)n), o;
  if (n > 0) std::memcpy(v.data(), in, (size_t)n * sizeof(Pt));
  const int st = voxel_grid(v, leaf, o, stable != 0);
  if (!o.empty()) std::memcpy(out, o.data(), o.size() * sizeof(Pt));
  *n_out = (int)o.size();
  return st;
}

}  // extern "C"
