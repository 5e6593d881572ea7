// lego_mapper.hip — MapOptimization's loop body (mapOptmization.cpp:1521-1570, loop closure off) behind
// include/lego_s2m.h's lego_mapper_*: the host logic of the reference's mapping thread around the
// device operations of lego_s2m.hip (lego_map_transform, lego_map_voxel, lego_s2m_run), with the key
// frames' downsampled clouds kept in device memory.
//
// Host parts restated here (float, the reference's float libm overloads):
//   transformAssociateToMap  :264-387
//   extractSurroundingKeyFrames, loop closure off  :915-995 (radiusSearch sorted by distance, the 1 m
//     VoxelGrid of key poses whose intensity is the key index, the existing-list erase / append order)
//   transformUpdate  :389-395;  saveKeyFramesAndFactor without GTSAM  :1335-1478
// lego_amd.mapping.MapSequence is the same loop in Python (tests compare them).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <new>
#include <numeric>
#include <vector>

#include "../../include/lego_s2m.h"

namespace {

struct KeyFrame {
  int64_t off[3];  // corner DS, surf DS, outlier DS in the device key store
  int32_t n[3];
  float pose[6];   // roll, pitch, yaw, x, y, z
};

// transformAssociateToMap (:264-387)
void associate_to_map(const float* S, const float* B, const float* A, float* T) {
  float incre[6] = {0, 0, 0, 0, 0, 0};
  float x1 = cosf(S[1]) * (B[3] - S[3]) - sinf(S[1]) * (B[5] - S[5]);
  float y1 = B[4] - S[4];
  float z1 = sinf(S[1]) * (B[3] - S[3]) + cosf(S[1]) * (B[5] - S[5]);
  float x2 = x1;
  float y2 = cosf(S[0]) * y1 + sinf(S[0]) * z1;
  float z2 = -sinf(S[0]) * y1 + cosf(S[0]) * z1;
  incre[3] = cosf(S[2]) * x2 + sinf(S[2]) * y2;
  incre[4] = -sinf(S[2]) * x2 + cosf(S[2]) * y2;
  incre[5] = z2;
  const float sbcx = sinf(S[0]), cbcx = cosf(S[0]), sbcy = sinf(S[1]), cbcy = cosf(S[1]), sbcz = sinf(S[2]),
              cbcz = cosf(S[2]);
  const float sblx = sinf(B[0]), cblx = cosf(B[0]), sbly = sinf(B[1]), cbly = cosf(B[1]), sblz = sinf(B[2]),
              cblz = cosf(B[2]);
  const float salx = sinf(A[0]), calx = cosf(A[0]), saly = sinf(A[1]), caly = cosf(A[1]), salz = sinf(A[2]),
              calz = cosf(A[2]);
  const float srx = -sbcx * (salx * sblx + calx * cblx * salz * sblz + calx * calz * cblx * cblz) -
                    cbcx * sbcy * (calx * calz * (cbly * sblz - cblz * sblx * sbly) - calx * salz * (cbly * cblz + sblx * sbly * sblz) +
                                   cblx * salx * sbly) -
                    cbcx * cbcy * (calx * salz * (cblz * sbly - cbly * sblx * sblz) - calx * calz * (sbly * sblz + cbly * cblz * sblx) +
                                   cblx * cbly * salx);
  T[0] = -asinf(srx);
  const float srycrx = sbcx * (cblx * cblz * (caly * salz - calz * salx * saly) - cblx * sblz * (caly * calz + salx * saly * salz) +
                               calx * saly * sblx) -
                       cbcx * cbcy * ((caly * calz + salx * saly * salz) * (cblz * sbly - cbly * sblx * sblz) +
                                      (caly * salz - calz * salx * saly) * (sbly * sblz + cbly * cblz * sblx) - calx * cblx * cbly * saly) +
                       cbcx * sbcy * ((caly * calz + salx * saly * salz) * (cbly * cblz + sblx * sbly * sblz) +
                                      (caly * salz - calz * salx * saly) * (cbly * sblz - cblz * sblx * sbly) + calx * cblx * saly * sbly);
  const float crycrx = sbcx * (cblx * sblz * (calz * saly - caly * salx * salz) - cblx * cblz * (saly * salz + caly * calz * salx) +
                               calx * caly * sblx) +
                       cbcx * cbcy * ((saly * salz + caly * calz * salx) * (sbly * sblz + cbly * cblz * sblx) +
                                      (calz * saly - caly * salx * salz) * (cblz * sbly - cbly * sblx * sblz) + calx * caly * cblx * cbly) -
                       cbcx * sbcy * ((saly * salz + caly * calz * salx) * (cbly * sblz - cblz * sblx * sbly) +
                                      (calz * saly - caly * salx * salz) * (cbly * cblz + sblx * sbly * sblz) - calx * caly * cblx * sbly);
  T[1] = atan2f(srycrx / cosf(T[0]), crycrx / cosf(T[0]));
  const float srzcrx = (cbcz * sbcy - cbcy * sbcx * sbcz) * (calx * salz * (cblz * sbly - cbly * sblx * sblz) -
                                                             calx * calz * (sbly * sblz + cbly * cblz * sblx) + cblx * cbly * salx) -
                       (cbcy * cbcz + sbcx * sbcy * sbcz) * (calx * calz * (cbly * sblz - cblz * sblx * sbly) -
                                                             calx * salz * (cbly * cblz + sblx * sbly * sblz) + cblx * salx * sbly) +
                       cbcx * sbcz * (salx * sblx + calx * cblx * salz * sblz + calx * calz * cblx * cblz);
  const float crzcrx = (cbcy * sbcz - cbcz * sbcx * sbcy) * (calx * calz * (cbly * sblz - cblz * sblx * sbly) -
                                                             calx * salz * (cbly * cblz + sblx * sbly * sblz) + cblx * salx * sbly) -
                       (sbcy * sbcz + cbcy * cbcz * sbcx) * (calx * salz * (cblz * sbly - cbly * sblx * sblz) -
                                                             calx * calz * (sbly * sblz + cbly * cblz * sblx) + cblx * cbly * salx) +
                       cbcx * cbcz * (salx * sblx + calx * cblx * salz * sblz + calx * calz * cblx * cblz);
  T[2] = atan2f(srzcrx / cosf(T[0]), crzcrx / cosf(T[0]));
  x1 = cosf(T[2]) * incre[3] - sinf(T[2]) * incre[4];
  y1 = sinf(T[2]) * incre[3] + cosf(T[2]) * incre[4];
  z1 = incre[5];
  x2 = x1;
  y2 = cosf(T[0]) * y1 - sinf(T[0]) * z1;
  z2 = sinf(T[0]) * y1 + cosf(T[0]) * z1;
  T[3] = A[3] - (cosf(T[1]) * x2 + sinf(T[1]) * z2);
  T[4] = A[4] - y2;
  T[5] = A[5] - (-sinf(T[1]) * x2 + cosf(T[1]) * z2);
}

// pcl::VoxelGrid::applyFilter on a few points (the 1 m key-pose filter, :78, :930-931): stable tie order
std::vector<lego_point> voxel_small(const std::vector<lego_point>& p, float leaf) {
  std::vector<lego_point> out;
  if (p.empty()) return out;
  const float inv = 1.0f / leaf;
  float mn[3] = {p[0].x, p[0].y, p[0].z}, mx[3] = {p[0].x, p[0].y, p[0].z};
  for (const auto& q : p) {
    mn[0] = std::min(mn[0], q.x); mn[1] = std::min(mn[1], q.y); mn[2] = std::min(mn[2], q.z);
    mx[0] = std::max(mx[0], q.x); mx[1] = std::max(mx[1], q.y); mx[2] = std::max(mx[2], q.z);
  }
  int64_t min_b[3], div_b[3];
  for (int a = 0; a < 3; ++a) {
    min_b[a] = (int64_t)floorf(mn[a] * inv);
    div_b[a] = (int64_t)floorf(mx[a] * inv) - min_b[a] + 1;
  }
  std::vector<int64_t> key(p.size());
  for (size_t i = 0; i < p.size(); ++i) {
    const int64_t i0 = (int64_t)(floorf(p[i].x * inv) - (float)min_b[0]);
    const int64_t i1 = (int64_t)(floorf(p[i].y * inv) - (float)min_b[1]);
    const int64_t i2 = (int64_t)(floorf(p[i].z * inv) - (float)min_b[2]);
    key[i] = i0 + i1 * div_b[0] + i2 * div_b[0] * div_b[1];
  }
  std::vector<size_t> idx(p.size());
  std::iota(idx.begin(), idx.end(), 0);
  std::stable_sort(idx.begin(), idx.end(), [&](size_t a, size_t b) { return key[a] < key[b]; });
  for (size_t i = 0; i < idx.size();) {
    size_t j = i;
    float s[4] = {0, 0, 0, 0};
    for (; j < idx.size() && key[idx[j]] == key[idx[i]]; ++j) {
      const lego_point& q = p[idx[j]];
      s[0] += q.x; s[1] += q.y; s[2] += q.z; s[3] += q.intensity;
    }
    const float n = (float)(j - i);
    out.push_back(lego_point{s[0] / n, s[1] / n, s[2] / n, s[3] / n});
    i = j;
  }
  return out;
}

template <typename T>
bool dmalloc(T** p, size_t n) {
  return hipMalloc((void**)p, (n ? n : 1) * sizeof(T)) == hipSuccess;
}

// Grow a device array to hold `need` elements (at least doubling), keeping its first `keep` elements.
// The mapper's calls are synchronous (null stream), so nothing still reads the old array.
template <typename T>
int grow(T** p, size_t need, size_t* cap, size_t keep) {
  if (need <= *cap) return LEGO_OK;
  const size_t nc = std::max(need, *cap * 2);
  T* q = nullptr;
  if (!dmalloc(&q, nc)) return LEGO_ENOMEM;
  if (keep && *p && hipMemcpy(q, *p, keep * sizeof(T), hipMemcpyDeviceToDevice) != hipSuccess) {
    hipFree(q);
    return LEGO_EDEVICE;
  }
  if (*p) hipFree(*p);
  *p = q;
  *cap = nc;
  return LEGO_OK;
}

}  // namespace

// The reference's mapping thread has no size limits: the key-frame store, the raw surrounding map (the
// key frames' parts concatenated before the VoxelGrid), the part lists and the scan-to-map LM's clouds
// all grow on demand here; max_map_points / max_key_points are only the initial capacities.
struct lego_mapper {
  int device = 0;
  int max_map = 0;
  lego_s2m* s2m = nullptr;       // scan-to-map LM (clouds up to lm_cap points)
  int lm_cap = 0;
  lego_s2m* vox = nullptr;       // VoxelGrid engine (clouds up to vox_cap points)
  int vox_cap = 0;
  lego_point* d_keys = nullptr;  // key-frame store
  size_t keys_cap = 0;
  int64_t key_used = 0;
  lego_point* d_raw = nullptr;   // [corner map raw | surf map raw | scan corner | scan surf | scan outlier]
  lego_point* d_vox = nullptr;   // their VoxelGrids, at the same offsets
  size_t raw_cap = 0, vox_buf_cap = 0;
  lego_point* d_tot = nullptr;   // surf total: raw, then its VoxelGrid right after it
  size_t tot_cap = 0;
  size_t parts_cap = 0, off_cap = 0, n_cap = 0, off2_cap = 0, pose_cap = 0;
  int64_t* d_off = nullptr;      // part / cloud offsets
  int32_t* d_n = nullptr;
  int64_t* d_off2 = nullptr;
  float* d_pose = nullptr;
  float* d_leaf = nullptr;
  int32_t* d_out_n = nullptr;
  int32_t* d_status = nullptr;
  int64_t* d_s2m_off = nullptr;  // [4] + counts [4] + transform [6] + degenerate + info [4]
  int32_t* d_s2m_n = nullptr;
  float* d_t = nullptr;
  int32_t* d_dg = nullptr;
  int32_t* d_info = nullptr;
  std::vector<KeyFrame> kf;
  std::vector<int> existing;
  float t_sum[6] = {0}, t_tobe[6] = {0}, t_bef[6] = {0}, t_aft[6] = {0};
  float prev_pos[3] = {0, 0, 0};
  int degenerate = 0;
  int voxel_tie_order = 0;  // the VoxelGrids' tie order (lego_mapper_set_voxel_tie_order)
};

extern "C" void lego_mapper_destroy(lego_mapper* m) {
  if (!m) return;
  hipSetDevice(m->device);
  hipDeviceSynchronize();
  for (void* p : {(void*)m->d_keys, (void*)m->d_raw, (void*)m->d_vox, (void*)m->d_tot, (void*)m->d_off, (void*)m->d_n,
                  (void*)m->d_off2, (void*)m->d_pose, (void*)m->d_leaf, (void*)m->d_out_n, (void*)m->d_status,
                  (void*)m->d_s2m_off, (void*)m->d_s2m_n, (void*)m->d_t, (void*)m->d_dg, (void*)m->d_info})
    if (p) hipFree(p);
  if (m->s2m) lego_s2m_destroy(m->s2m);
  if (m->vox) lego_s2m_destroy(m->vox);
  delete m;
}

namespace {
// an s2m engine (LM or VoxelGrid) for clouds of at least `need` points: recreated larger when needed
int ensure_engine(int device, lego_s2m** e, int* cap, int64_t need, int voxel_tie_order = 0) {
  if (need <= *cap && *e) return lego_s2m_set_voxel_tie_order(*e, voxel_tie_order);
  if (need > LEGO_MAX_POINTS) return LEGO_EINVAL;
  const int64_t nc = std::min<int64_t>(LEGO_MAX_POINTS, std::max<int64_t>(need, 2 * (int64_t)*cap));
  if (*e) {
    hipDeviceSynchronize();
    lego_s2m_destroy(*e);
    *e = nullptr;
    *cap = 0;
  }
  const int rc = lego_s2m_create(device, 1, (int32_t)nc, e);
  if (rc != LEGO_OK) return rc;
  *cap = (int)nc;
  return lego_s2m_set_voxel_tie_order(*e, voxel_tie_order);
}
int ensure_parts(lego_mapper* m, size_t np) {  // part lists of np parts (and >= 8 VoxelGrid clouds)
  np = std::max<size_t>(np, 8);
  if (np <= m->parts_cap) return LEGO_OK;
  int rc;
  if ((rc = grow(&m->d_off, np, &m->off_cap, 0)) || (rc = grow(&m->d_n, np, &m->n_cap, 0)) ||
      (rc = grow(&m->d_off2, np, &m->off2_cap, 0)) || (rc = grow(&m->d_pose, 6 * np, &m->pose_cap, 0)))
    return rc;
  m->parts_cap = np;
  return LEGO_OK;
}
}  // namespace

extern "C" int lego_mapper_create(int32_t device, int32_t max_map_points, int64_t max_key_points, lego_mapper** out) {
  if (!out) return LEGO_EINVAL;
  *out = nullptr;
  if (max_map_points < 1 || max_map_points > LEGO_MAX_POINTS || max_key_points < 1) return LEGO_EINVAL;
  lego_mapper* m = new (std::nothrow) lego_mapper();
  if (!m) return LEGO_ENOMEM;
  m->device = device;
  m->max_map = max_map_points;
  if (hipSetDevice(device) != hipSuccess) {
    delete m;
    return LEGO_EDEVICE;
  }
  int rc = ensure_engine(device, &m->s2m, &m->lm_cap, max_map_points);
  if (rc == LEGO_OK) rc = ensure_engine(device, &m->vox, &m->vox_cap, 2 * (int64_t)max_map_points, m->voxel_tie_order);
  if (rc != LEGO_OK) {
    lego_mapper_destroy(m);
    return rc;
  }
  const size_t R = (size_t)5 * max_map_points;
  if (grow(&m->d_keys, (size_t)max_key_points, &m->keys_cap, 0) || grow(&m->d_raw, R, &m->raw_cap, 0) ||
      grow(&m->d_vox, R, &m->vox_buf_cap, 0) || grow(&m->d_tot, (size_t)4 * max_map_points, &m->tot_cap, 0) ||
      ensure_parts(m, 4096) || !dmalloc(&m->d_leaf, 8) || !dmalloc(&m->d_out_n, 8) || !dmalloc(&m->d_status, 8) ||
      !dmalloc(&m->d_s2m_off, 4) || !dmalloc(&m->d_s2m_n, 4) || !dmalloc(&m->d_t, 6) || !dmalloc(&m->d_dg, 1) ||
      !dmalloc(&m->d_info, 4)) {
    lego_mapper_destroy(m);
    return LEGO_ENOMEM;
  }
  *out = m;
  return LEGO_OK;
}

// OdometryToTransform (utility.h:96-110): the mapping thread's transformSum from the odometry message,
// through tf::Matrix3x3(tf::Quaternion(q.z, -q.x, -q.y, q.w)).getRPY (tf/LinearMath/Matrix3x3.h:
// setRotation, getEulerYPR with solution 1) in double, then transform = (-pitch, -yaw, roll, position).
extern "C" int lego_mapper_set_voxel_tie_order(lego_mapper* m, int32_t order) {
  if (!m || order < 0 || order > 1) return LEGO_EINVAL;
  m->voxel_tie_order = order;
  return m->vox ? lego_s2m_set_voxel_tie_order(m->vox, order) : LEGO_OK;
}

extern "C" int lego_map_odometry_to_transform(const double* orientation, const double* position, float* transform) {
  if (!orientation || !position || !transform) return LEGO_EINVAL;
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
  return LEGO_OK;
}

extern "C" int lego_map_associate(const float* transform_sum, const float* transform_bef_mapped,
                                  const float* transform_aft_mapped, float* transform_tobe_mapped) {
  if (!transform_sum || !transform_bef_mapped || !transform_aft_mapped || !transform_tobe_mapped) return LEGO_EINVAL;
  associate_to_map(transform_sum, transform_bef_mapped, transform_aft_mapped, transform_tobe_mapped);
  return LEGO_OK;
}

extern "C" int lego_mapper_key_poses(const lego_mapper* m, float* out, int32_t cap, int32_t* n) {
  if (!m || !n || (cap > 0 && !out)) return LEGO_EINVAL;
  *n = (int32_t)m->kf.size();
  for (int32_t i = 0; i < *n && i < cap; ++i) memcpy(out + 6 * i, m->kf[i].pose, 6 * sizeof(float));
  return LEGO_OK;
}

#define MCHECK(x) \
  do {                               \
    if ((x) != hipSuccess) return LEGO_EDEVICE; \
  } while (0)

extern "C" int lego_mapper_step(lego_mapper* m, const lego_point* corner_last, int32_t n_corner,
                                const lego_point* surf_last, int32_t n_surf, const lego_point* outlier_last,
                                int32_t n_outlier, const float* transform_sum, float* transform_aft_mapped,
                                int32_t* info) {
  if (!m || !transform_sum || !transform_aft_mapped || !info || n_corner < 0 || n_surf < 0 || n_outlier < 0 ||
      (n_corner && !corner_last) || (n_surf && !surf_last) || (n_outlier && !outlier_last))
    return LEGO_EINVAL;
  MCHECK(hipSetDevice(m->device));
  // Nothing of the mapper's state is committed before every capacity is in place: a failure leaves the
  // mapper as it was before the call (the caller may retry the same scan).
  float t_tobe[6];
  std::vector<int> existing = m->existing;
  // OdometryToTransform (:1540) + transformAssociateToMap (:1542)
  associate_to_map(transform_sum, m->t_bef, m->t_aft, t_tobe);
  // extractSurroundingKeyFrames, loop closure off (:915-995)
  if (!m->kf.empty()) {
    const float* c = m->t_aft + 3;  // currentRobotPosPoint, set by the last saveKeyFramesAndFactor
    std::vector<std::pair<float, int>> sel;  // radiusSearch (50 m), sorted by distance
    for (int i = 0; i < (int)m->kf.size(); ++i) {
      const float* q = m->kf[i].pose + 3;
      const float d = ((q[0] - c[0]) * (q[0] - c[0]) + (q[1] - c[1]) * (q[1] - c[1])) + (q[2] - c[2]) * (q[2] - c[2]);
      if (d < 50.0f * 50.0f) sel.push_back({d, i});
    }
    std::stable_sort(sel.begin(), sel.end(), [](const std::pair<float, int>& x, const std::pair<float, int>& y) {
      return x.first < y.first;
    });
    std::vector<lego_point> kp;
    for (const auto& e : sel) {
      const float* q = m->kf[e.second].pose + 3;
      kp.push_back(lego_point{q[0], q[1], q[2], (float)e.second});
    }
    const std::vector<lego_point> ds = voxel_small(kp, 1.0f);  // downSizeFilterSurroundingKeyPoses (:78)
    std::vector<int> ids;
    for (const auto& q : ds) ids.push_back((int)q.intensity);
    std::vector<int> keep;
    for (int id : existing)
      if (std::find(ids.begin(), ids.end(), id) != ids.end()) keep.push_back(id);
    existing = keep;
    for (int id : ids)
      if (std::find(existing.begin(), existing.end(), id) == existing.end()) existing.push_back(id);
  }
  // the map's parts: corner clouds of the existing key frames, then their surf and outlier clouds, frame
  // by frame (:982-986), transformed by their key poses into [corner raw | surf raw]
  const int np = 3 * (int)existing.size();
  int rc = ensure_parts(m, (size_t)np);
  if (rc) return rc;
  std::vector<int64_t> in_off, out_off;
  std::vector<int32_t> in_n;
  std::vector<float> pose;
  int64_t ncm = 0, nsm = 0;
  for (int id : existing) {
    const KeyFrame& k = m->kf[id];
    in_off.push_back(k.off[0]); in_n.push_back(k.n[0]); out_off.push_back(ncm); ncm += k.n[0];
    pose.insert(pose.end(), k.pose, k.pose + 6);
  }
  for (int id : existing) {
    const KeyFrame& k = m->kf[id];
    for (int j = 1; j < 3; ++j) {
      in_off.push_back(k.off[j]); in_n.push_back(k.n[j]); out_off.push_back(ncm + nsm); nsm += k.n[j];
      pose.insert(pose.end(), k.pose, k.pose + 6);
    }
  }
  // capacities for this cycle's clouds: the raw map, the scan's clouds, their VoxelGrids
  const int64_t base_sc = ncm + nsm;
  const int64_t n_raw = base_sc + n_corner + n_surf + n_outlier;
  const int64_t big = std::max<int64_t>(std::max<int64_t>(ncm, nsm), (int64_t)n_corner + n_surf + n_outlier);
  if ((rc = grow(&m->d_raw, (size_t)n_raw, &m->raw_cap, 0)) || (rc = grow(&m->d_vox, (size_t)n_raw, &m->vox_buf_cap, 0)) ||
      (rc = grow(&m->d_tot, (size_t)2 * (n_surf + n_outlier), &m->tot_cap, 0)) ||
      (rc = ensure_engine(m->device, &m->vox, &m->vox_cap, big, m->voxel_tie_order)))
    return rc;
  // the scan's clouds after the map's
  if (n_corner) MCHECK(hipMemcpy(m->d_raw + base_sc, corner_last, (size_t)n_corner * sizeof(lego_point), hipMemcpyHostToDevice));
  if (n_surf) MCHECK(hipMemcpy(m->d_raw + base_sc + n_corner, surf_last, (size_t)n_surf * sizeof(lego_point), hipMemcpyHostToDevice));
  if (n_outlier)
    MCHECK(hipMemcpy(m->d_raw + base_sc + n_corner + n_surf, outlier_last, (size_t)n_outlier * sizeof(lego_point),
                     hipMemcpyHostToDevice));
  if (np > 0) {
    MCHECK(hipMemcpy(m->d_off, in_off.data(), np * sizeof(int64_t), hipMemcpyHostToDevice));
    MCHECK(hipMemcpy(m->d_n, in_n.data(), np * sizeof(int32_t), hipMemcpyHostToDevice));
    MCHECK(hipMemcpy(m->d_off2, out_off.data(), np * sizeof(int64_t), hipMemcpyHostToDevice));
    MCHECK(hipMemcpy(m->d_pose, pose.data(), pose.size() * sizeof(float), hipMemcpyHostToDevice));
    lego_map_transform_io tio{m->d_keys, m->d_off, m->d_n, m->d_pose, m->d_raw, m->d_off2};
    int rc = lego_map_transform(m->s2m, np, &tio, nullptr);
    if (rc) return rc;
  }
  // VoxelGrids: corner map 0.2, surf map 0.4, scan corner 0.2, surf 0.4, outlier 0.4 (:71-73, :988-1017)
  const int64_t voff[5] = {0, ncm, base_sc, base_sc + n_corner, base_sc + n_corner + n_surf};
  const int32_t vn[5] = {(int32_t)ncm, (int32_t)nsm, n_corner, n_surf, n_outlier};
  const float leaf[5] = {0.2f, 0.4f, 0.2f, 0.4f, 0.4f};
  MCHECK(hipMemcpy(m->d_off, voff, sizeof(voff), hipMemcpyHostToDevice));
  MCHECK(hipMemcpy(m->d_n, vn, sizeof(vn), hipMemcpyHostToDevice));
  MCHECK(hipMemcpy(m->d_leaf, leaf, sizeof(leaf), hipMemcpyHostToDevice));
  lego_map_voxel_io vio{m->d_raw, m->d_off, m->d_n, m->d_leaf, m->d_vox, m->d_off, m->d_out_n, m->d_status};
  rc = lego_map_voxel(m->vox, 5, &vio, nullptr);
  if (rc) return rc;
  int32_t on[5];
  MCHECK(hipMemcpy(on, m->d_out_n, sizeof(on), hipMemcpyDeviceToHost));
  for (int k = 0; k < 5; ++k)
    if (on[k] < 0) return LEGO_EINVAL;
  // laserCloudSurfTotalLastDS = VoxelGrid(surf DS ++ outlier DS) (:1019-1025)
  const int32_t ntot = on[3] + on[4];
  if (on[3]) MCHECK(hipMemcpy(m->d_tot, m->d_vox + voff[3], (size_t)on[3] * sizeof(lego_point), hipMemcpyDeviceToDevice));
  if (on[4])
    MCHECK(hipMemcpy(m->d_tot + on[3], m->d_vox + voff[4], (size_t)on[4] * sizeof(lego_point), hipMemcpyDeviceToDevice));
  const int64_t toff[2] = {0, (int64_t)ntot};  // the VoxelGrid's output right after its input
  MCHECK(hipMemcpy(m->d_off2, toff, sizeof(toff), hipMemcpyHostToDevice));
  MCHECK(hipMemcpy(m->d_n + 5, &ntot, sizeof(ntot), hipMemcpyHostToDevice));
  lego_map_voxel_io vio2{m->d_tot, m->d_off2, m->d_n + 5, m->d_leaf + 1, m->d_tot, m->d_off2 + 1, m->d_out_n + 5,
                         m->d_status + 5};
  rc = lego_map_voxel(m->vox, 1, &vio2, nullptr);
  if (rc) return rc;
  // scan2MapOptimization (:1548)
  const int64_t s_off[4] = {voff[2], (int64_t)ntot, voff[0], voff[1]};
  MCHECK(hipMemcpy(m->d_s2m_off, s_off, sizeof(s_off), hipMemcpyHostToDevice));
  const int32_t s_n[3] = {on[2], on[0], on[1]};  // corner DS; surf total from the second VoxelGrid
  int32_t ntot_ds = -1;
  MCHECK(hipMemcpy(&ntot_ds, m->d_out_n + 5, sizeof(int32_t), hipMemcpyDeviceToHost));
  if (ntot_ds < 0) return LEGO_EINVAL;
  const int32_t s_cnt[4] = {s_n[0], ntot_ds, s_n[1], s_n[2]};
  // the LM engine's clouds (its gate: each map <= its capacity, the scan's corner + surf <= it)
  if ((rc = ensure_engine(m->device, &m->s2m, &m->lm_cap,
                          std::max<int64_t>(std::max(s_n[1], s_n[2]), (int64_t)s_n[0] + ntot_ds))))
    return rc;
  // the key frame this cycle may store (saveKeyFramesAndFactor), before any state changes
  if ((rc = grow(&m->d_keys, (size_t)(m->key_used + on[2] + on[3] + on[4]), &m->keys_cap, (size_t)m->key_used)))
    return rc;
  MCHECK(hipMemcpy(m->d_s2m_n, s_cnt, sizeof(s_cnt), hipMemcpyHostToDevice));
  MCHECK(hipMemcpy(m->d_t, t_tobe, sizeof(t_tobe), hipMemcpyHostToDevice));
  MCHECK(hipMemcpy(m->d_dg, &m->degenerate, sizeof(int32_t), hipMemcpyHostToDevice));
  lego_s2m_io sio;
  sio.corner = m->d_vox; sio.corner_off = m->d_s2m_off; sio.corner_n = m->d_s2m_n;
  sio.surf = m->d_tot; sio.surf_off = m->d_s2m_off + 1; sio.surf_n = m->d_s2m_n + 1;
  sio.corner_map = m->d_vox; sio.corner_map_off = m->d_s2m_off + 2; sio.corner_map_n = m->d_s2m_n + 2;
  sio.surf_map = m->d_vox; sio.surf_map_off = m->d_s2m_off + 3; sio.surf_map_n = m->d_s2m_n + 3;
  sio.transform = m->d_t; sio.degenerate = m->d_dg; sio.info = m->d_info;
  rc = lego_s2m_run(m->s2m, 1, &sio, nullptr);
  if (rc) return rc;
  int32_t degenerate = 0, inf[4];
  MCHECK(hipMemcpy(t_tobe, m->d_t, sizeof(t_tobe), hipMemcpyDeviceToHost));
  MCHECK(hipMemcpy(&degenerate, m->d_dg, sizeof(int32_t), hipMemcpyDeviceToHost));
  MCHECK(hipMemcpy(inf, m->d_info, 4 * sizeof(int32_t), hipMemcpyDeviceToHost));
  if (inf[0] < 0) return LEGO_EDEVICE;  // cannot happen: the LM engine was sized for these clouds
  // commit: every fallible step is behind us
  memcpy(info, inf, sizeof(inf));
  memcpy(m->t_sum, transform_sum, sizeof(m->t_sum));
  memcpy(m->t_tobe, t_tobe, sizeof(t_tobe));
  m->degenerate = degenerate;
  m->existing.swap(existing);
  if (info[0] == 1) {  // transformUpdate (:389-395)
    memcpy(m->t_bef, m->t_sum, sizeof(m->t_sum));
    memcpy(m->t_aft, m->t_tobe, sizeof(m->t_tobe));
  }
  // saveKeyFramesAndFactor (:1335-1478) without GTSAM
  const float* cur = m->t_aft + 3;
  const float dx = m->prev_pos[0] - cur[0], dy = m->prev_pos[1] - cur[1], dz = m->prev_pos[2] - cur[2];
  const bool moved = !(sqrtf(dx * dx + dy * dy + dz * dz) < 0.3);
  if (moved || m->kf.empty()) {
    memcpy(m->prev_pos, cur, sizeof(m->prev_pos));
    KeyFrame k;
    memcpy(k.pose, m->kf.empty() ? m->t_tobe : m->t_aft, sizeof(k.pose));
    const int32_t kn[3] = {on[2], on[3], on[4]};  // room reserved above
    for (int j = 0; j < 3; ++j) {
      k.off[j] = m->key_used;
      k.n[j] = kn[j];
      if (kn[j])
        MCHECK(hipMemcpy(m->d_keys + m->key_used, m->d_vox + voff[2 + j], (size_t)kn[j] * sizeof(lego_point),
                         hipMemcpyDeviceToDevice));
      m->key_used += kn[j];
    }
    m->kf.push_back(k);
    if (m->kf.size() > 1) memcpy(m->t_tobe, m->t_aft, sizeof(m->t_tobe));  // :1447-1459
  }
  memcpy(transform_aft_mapped, m->t_aft, sizeof(m->t_aft));
  return LEGO_OK;
}
