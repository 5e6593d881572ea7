/*
 * lego_s2m.h — C-ABI of the MI355X-native scan-to-map LM (MapOptimization's scan2MapOptimization).
 *
 * Drop-in boundary for the optimisation core of the reference's mapping thread:
 *   MapOptimization::scan2MapOptimization  (LeGO-LOAM/src/mapOptmization.cpp:1315-1332)
 *   MapOptimization::cornerOptimization    (:1028-1134)  kNN-5 line fit, point-to-line residuals
 *   MapOptimization::surfOptimization      (:1136-1197)  kNN-5 plane fit (5x3 QR), point-to-plane
 *   MapOptimization::LMOptimization        (:1199-1312)  6x6 normal equations, QR solve, degeneracy
 * with the members they read and write (mapOptimization.h:200-226): transformTobeMapped[6] and
 * isDegenerate (persisting from call to call, as the member does).  The caller keeps the rest of the
 * mapping thread (transformAssociateToMap, key-frame selection, map assembly and VoxelGrid, GTSAM):
 * it hands over, per problem, the four clouds scan2MapOptimization works on:
 *   corner      laserCloudCornerLastDS      (the scan's corner features, downsampled, lidar frame)
 *   surf        laserCloudSurfTotalLastDS   (surf + outlier features, downsampled, lidar frame)
 *   corner_map  laserCloudCornerFromMapDS   (the surrounding map's corner cloud, map frame)
 *   surf_map    laserCloudSurfFromMapDS     (the surrounding map's surf cloud, map frame)
 * Points are lego_point (pcl::PointXYZI, 16 B; lego_frontend.h).  The kd-trees the reference builds
 * over the two map clouds (:1317-1318) are replaced by per-problem hash grids built on the device.
 *
 * Many independent problems (one per mapping sequence) run in one launch, one workgroup each.  Plain
 * C, plain pointers and sizes; every entry point returns LEGO_OK (0) or a negative LEGO_E* code
 * (lego_frontend.h) and never throws.  A lego_s2m object (its scratch) serves one call at a time:
 * calls on different streams must be ordered by the caller, as the reference's single mapping
 * thread orders them.  There is no CPU fallback: without a usable HIP device
 * lego_s2m_create returns LEGO_EDEVICE.
 *
 * libm model: the mapping half implements lego_params.fp_mode 0 only (GCC >= 6 builds of the reference:
 * mapOptmization.cpp's unqualified sin / cos / sqrt on floats resolve to the float overloads).  k_s2m's
 * pointAssociateToMap / LMOptimization trig and sqrt(sqrt(.)) weights, transformPointCloud
 * (lego_map_transform) and transformAssociateToMap (lego_map_associate, lego_mapper_step) run the float
 * libm (glibc's sinf / cosf / asinf / atan2f restated); none of these entry points takes an fp_mode.  A
 * front end configured with fp_mode 1 (the GCC 4.8 / 5 double-overload model) feeding this mapping half
 * is therefore a mixed model: its scan-to-map results stay within the scan-to-map bar of a GCC >= 6
 * reference, not bit-identical to a GCC 4.8 / 5 one.  tests/test_s2m_cpu.py
 * (test_mapping_half_is_fp_mode_0) pins this.
 */
#ifndef LEGO_S2M_H
#define LEGO_S2M_H

#include <stdint.h>

#include "lego_frontend.h"

#ifdef __cplusplus
extern "C" {
#endif

/* info[4] of a problem: [0] 1 if the optimisation ran (:1316: corner map > 10 and surf map > 100
 * points), [1] LM iterations run (<= 10), [2] correspondences of the last iteration
 * (laserCloudOri size), [3] status bits below. */
#define LEGO_S2M_ST_KNN_TIE     0x01  /* equal distances among a query's 6 nearest: resolved by nanoflann's tree, as the reference */
#define LEGO_S2M_ST_DEGENERATE  0x02  /* iteration 0: largest eigenvalue of AtA < 100 (:1267-1285)        */
#define LEGO_S2M_ST_FEW         0x04  /* an iteration had < 50 correspondences (:1208: no update)           */
#define LEGO_S2M_ST_CONVERGED   0x08  /* LMOptimization returned true (:1308) before the 10th iteration     */
#define LEGO_S2M_ST_SKIPPED     0x10  /* the map gate of :1316 failed: transform and state untouched        */
#define LEGO_S2M_ST_TIE_UNRESOLVED 0x20  /* a tied query kept the grid's order: the device kd-tree's build or
                                          * search stack overflowed (not nanoflann's choice)                 */

/* Device-side batch: array i of problem p is base_i[off_i[p] .. off_i[p] + n_i[p]).  All pointers are
 * DEVICE pointers (offsets int64, counts int32, one entry per problem). */
typedef struct lego_s2m_io {
  const lego_point* corner;      const int64_t* corner_off;     const int32_t* corner_n;
  const lego_point* surf;        const int64_t* surf_off;       const int32_t* surf_n;
  const lego_point* corner_map;  const int64_t* corner_map_off; const int32_t* corner_map_n;
  const lego_point* surf_map;    const int64_t* surf_map_off;   const int32_t* surf_map_n;
  float*   transform;   /* [n][6] transformTobeMapped: initial guess in, optimised pose out     */
  int32_t* degenerate;  /* [n]    isDegenerate, in and out (mapOptimization.h:210)              */
  int32_t* info;        /* [n][4] out, see above                                                */
} lego_s2m_io;

typedef struct lego_s2m lego_s2m;

/* Scratch for up to max_problems problems whose map clouds hold up to max_map_points points each. */
int  lego_s2m_create(int32_t device, int32_t max_problems, int32_t max_map_points, lego_s2m** out);
void lego_s2m_destroy(lego_s2m* m);
/* scan2MapOptimization of n problems, asynchronous on hip_stream (NULL = default).  LEGO_EINVAL when
 * n is outside [1, max_problems]; a problem whose map cloud exceeds max_map_points gets status
 * LEGO_S2M_ST_SKIPPED and info[0] = -1. */
int  lego_s2m_run(lego_s2m* m, int32_t n, const lego_s2m_io* io, void* hip_stream);
/* One problem from host clouds (blocking): the reference's per-scan call.  transform[6] and
 * *degenerate are read and written; info[4] is written. */
int  lego_s2m_run_host(lego_s2m* m, const lego_point* corner, int32_t n_corner, const lego_point* surf,
                       int32_t n_surf, const lego_point* corner_map, int32_t n_corner_map,
                       const lego_point* surf_map, int32_t n_surf_map, float* transform, int32_t* degenerate,
                       int32_t* info);

/* ---- map-side cloud preparation ------------------------------------------------
 * The clouds scan2MapOptimization consumes are built by extractSurroundingKeyFrames (:857-996) and
 * downsampleCurrentScan (:999-1026) from two operations, batched here over n clouds (device arrays,
 * asynchronous on hip_stream):
 *   lego_map_transform  transformPointCloud (:443-473): part p of the input rotated / translated by
 *                       pose[p] = (roll, pitch, yaw, x, y, z) of its key frame (PointTypePose), written
 *                       at out + out_off[p] (parts written next to each other concatenate: the `+=`
 *                       of :909-913 / :982-986);
 *   lego_map_voxel      pcl::VoxelGrid<PointXYZI>::filter (PCL 1.7/1.8 applyFilter; leaves :71-78) of
 *                       cloud c with leaf[c]: one centroid per occupied leaf in ascending leaf order,
 *                       each the float sum of its points in the order of PCL's std::sort of the (leaf
 *                       index, point index) pairs (voxel_tie_order 0, the default: libstdc++'s introsort
 *                       permutation, bit-identical to the reference) or, after
 *                       lego_s2m_set_voxel_tie_order(m, 1), in input order (std::stable_sort's) divided
 *                       by their count.  status[c] =
 *                       LEGO_ST_VOXEL_OVERFLOW when the leaf indices would overflow int32 (PCL's warning
 *                       path: the cloud is copied unfiltered).  Clouds hold at most max_map_points
 *                       points (larger: out_n = -1). */
typedef struct lego_map_transform_io {
  const lego_point* in;  const int64_t* in_off;  const int32_t* in_n;
  const float* pose;     /* [n][6] roll, pitch, yaw, x, y, z */
  lego_point* out;       const int64_t* out_off;
} lego_map_transform_io;
typedef struct lego_map_voxel_io {
  const lego_point* in;  const int64_t* in_off;  const int32_t* in_n;
  const float* leaf;     /* [n] */
  lego_point* out;       const int64_t* out_off; /* room for in_n[c] points */
  int32_t* out_n;        /* [n] */
  int32_t* status;       /* [n] */
} lego_map_voxel_io;
int  lego_map_transform(lego_s2m* m, int32_t n, const lego_map_transform_io* io, void* hip_stream);
/* scratch for the call's n clouds of max_map_points each is allocated on first use (and regrown for a
 * larger n, after a device synchronize) */
int  lego_map_voxel(lego_s2m* m, int32_t n, const lego_map_voxel_io* io, void* hip_stream);
/* lego_map_voxel's tie order, as lego_params.voxel_tie_order: 0 (default) libstdc++ std::sort's
 * permutation (PCL's applyFilter, the reference: a level-synchronous introsort emulation, which
 * synchronizes hip_stream once per level of ranges longer than 2,048 points), 1 std::stable_sort's
 * (rocPRIM radix sort, asynchronous). */
int  lego_s2m_set_voxel_tie_order(lego_s2m* m, int32_t order);

/* ---- MapOptimization's loop body (loop closure off: loam_config.yaml:24) --------------------------------
 * One mapping sequence: MapOptimization::run (mapOptmization.cpp:1521-1570) per AssociationOut, with the
 * key frames kept in device memory:
 *   transformAssociateToMap (:264-387) from transform_sum (OdometryToTransform of the odometry, :1540),
 *   extractSurroundingKeyFrames (:915-995: key poses within 50 m by distance, their 1 m VoxelGrid, the
 *     existing key-frame list erased / extended in the reference's order; lego_map_transform + _voxel),
 *   downsampleCurrentScan (:999-1026), scan2MapOptimization (:1315-1332), transformUpdate (:389-395),
 *   saveKeyFramesAndFactor (:1335-1478) without GTSAM: with no loop closure the factor graph is a chain
 *     whose optimum is the pose just inserted (the first key frame at transformTobeMapped, later ones at
 *     transformAftMapped), so the key poses are those.
 * lego_mapper_step returns transformAftMapped after the cycle (publishTF's pose, :510-538) and info[4] as
 * lego_s2m_run's.  A mapper serves one call at a time.  max_map_points / max_key_points are initial
 * capacities only (the reference has no limits): the raw surrounding map, the scan's clouds, the key-frame
 * store and the LM's clouds grow on demand.  A failing call (LEGO_ENOMEM / LEGO_EDEVICE) leaves the mapper
 * as it was before it. */
typedef struct lego_mapper lego_mapper;
int  lego_mapper_create(int32_t device, int32_t max_map_points, int64_t max_key_points, lego_mapper** out);
void lego_mapper_destroy(lego_mapper* m);
int  lego_mapper_step(lego_mapper* m, const lego_point* corner_last, int32_t n_corner, const lego_point* surf_last,
                      int32_t n_surf, const lego_point* outlier_last, int32_t n_outlier, const float* transform_sum,
                      float* transform_aft_mapped, int32_t* info);
/* key poses so far, (roll, pitch, yaw, x, y, z) each (cloudKeyPoses6D); *n = their count */
int  lego_mapper_key_poses(const lego_mapper* m, float* out, int32_t cap, int32_t* n);
/* the tie order of the mapper's VoxelGrids (lego_s2m_set_voxel_tie_order): 0 (default) the reference's */
int  lego_mapper_set_voxel_tie_order(lego_mapper* m, int32_t order);
/* Launch layout of lego_s2m_run: 0 = one 1024-thread workgroup a problem (throughput: hundreds of
 * problems), 1 = latency (a problem's grids built by two workgroups, each LM iteration's queries spread
 * over up to 256 / n workgroups, normal equations and solve in one; 21 launches), -1 (default) = latency
 * for n <= 16.  Results are identical. */
int  lego_s2m_set_layout(lego_s2m* m, int32_t layout);
/* test hook (not for the mapping path): cap the LM iterations of later runs at max_iters (the product's 10
 * restored by passing 10) and copy problem p's LM rows of its last iteration, 8 floats a query (arx, ary,
 * arz, coeff x, y, z, -coeff intensity, 1 if selected else 0), into out[8 * nq] */
int  lego_test_s2m_debug(lego_s2m* m, int32_t max_iters, int32_t p, int32_t nq, float* out);
/* OdometryToTransform (utility.h:96-110) on the host: the mapping thread's transformSum from the
 * /laser_odom_to_init message (orientation x, y, z, w; position x, y, z), through tf's getRPY in double
 * (lego_association_out.odom_orientation / odom_position are that message). */
int  lego_map_odometry_to_transform(const double* orientation, const double* position, float* transform);
/* transformAssociateToMap (mapOptmization.cpp:264-387) on the host, float with the float libm (no device
 * needed): transformTobeMapped from transformSum / transformBefMapped / transformAftMapped. */
int  lego_map_associate(const float* transform_sum, const float* transform_bef_mapped, const float* transform_aft_mapped,
                        float* transform_tobe_mapped);

#ifdef __cplusplus
}
#endif
#endif /* LEGO_S2M_H */
