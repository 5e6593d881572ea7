/*
 * lego_frontend.h — C-ABI of the MI355X-native LeGO-LOAM-BOR front end.
 *
 * Drop-in boundary for the reference's per-scan hot path:
 *   ImageProjection::cloudHandler            (LeGO-LOAM/src/imageProjection.h:16, .cpp:153-174)
 *   FeatureAssociation::runFeatureAssociation (LeGO-LOAM/src/featureAssociation.h:19, .cpp:1386-1450)
 * and the two value types that cross the reference's thread boundary:
 *   ProjectionOut + cloud_msgs::cloud_info   (LeGO-LOAM/include/lego_loam/utility.h:64-70, cloud_msgs/msg/cloud_info.msg:1-13)
 *   AssociationOut                           (utility.h:73-80)
 *
 * Plain C, plain pointers and sizes; no torch / ROS / PCL types.  Every entry point
 * returns an int status (LEGO_OK = 0, < 0 = error) and never throws.  Output arrays
 * referenced by the *_out structs are owned by the context / batch and stay valid until
 * the next call on the same object.  A context or batch is single-threaded (the
 * reference's one-writer/one-reader Channel contract, channel.h:8-10).
 *
 * The product path is the HIP path on a gfx950 device.  There is no CPU fallback:
 * creating a context without a usable device returns LEGO_EDEVICE.
 */
#ifndef LEGO_FRONTEND_H
#define LEGO_FRONTEND_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LEGO_ABI_VERSION 1

/* ---- status codes ------------------------------------------------------------ */
#define LEGO_OK          0
#define LEGO_EINVAL     -1   /* bad parameter / shape                                   */
#define LEGO_ENOMEM     -2   /* host or device allocation failed                         */
#define LEGO_EDEVICE    -3   /* no HIP device / kernel launch or runtime failure          */
#define LEGO_ENOTSUP    -4   /* configuration / build does not support the request         */
#define LEGO_EEMPTY     -5   /* empty input cloud (reference: UB in findStartEndAngle)    */

#define LEGO_MAX_POINTS ((1 << 28) - 1)  /* points of one input cloud (larger: LEGO_EINVAL) */

/* ---- per-scan status bits reported by the association stage ------------------- */
#define LEGO_ST_INIT            0x001  /* first scan: checkSystemInitialization (fa.cpp:1181-1209)   */
#define LEGO_ST_LM_SKIPPED      0x002  /* Last clouds too small, LM skipped (fa.cpp:1214)            */
#define LEGO_ST_DEGENERATE      0x004  /* eigenvalue degeneracy hit in a solve (fa.cpp:869-898)      */
#define LEGO_ST_STALE_TREE      0x008  /* ref UB: kd-tree not rebuilt but LM ran (fa.cpp:1214,1356)   */
#define LEGO_ST_FWD_OOB         0x010  /* ref UB: forward scan bound > |Last| (fa.cpp:522,661)        */
#define LEGO_ST_NN_TIE          0x020  /* exact 1-NN distance tie, resolved as nanoflann (first visited) */
#define LEGO_ST_STALE_IND_OOB   0x040  /* ref UB: stale smoothness entry indexes past the cloud       */
#define LEGO_ST_EMITTED         0x080  /* AssociationOut sent to mapping this cycle (fa.cpp:1432)     */
#define LEGO_ST_VOXEL_OVERFLOW  0x100  /* PCL VoxelGrid index overflow: cloud copied unfiltered       */
#define LEGO_ST_DEGEN_UB        0x200  /* ref UB: degenerate at iter>0 uses uninit matP (fa.cpp:894)  */
#define LEGO_ST_TIE_UNRESOLVED  0x400  /* an exact 1-NN tie kept the grid's lowest index: the device kd-tree's
                                        * build or search stack overflowed (not nanoflann's choice)  */

/* ---- parameters: the reference's loam_config.yaml keys ------------------------- */
typedef struct lego_params {
  int32_t num_vertical_scans;              /* V   laser/num_vertical_scans       loam_config.yaml:5  */
  int32_t num_horizontal_scans;            /* H   laser/num_horizontal_scans     :6                 */
  int32_t ground_scan_index;               /* G   laser/ground_scan_index        :7                 */
  float   vertical_angle_bottom;           /* deg laser/vertical_angle_bottom    :8                 */
  float   vertical_angle_top;              /* deg laser/vertical_angle_top       :9                 */
  float   sensor_mount_angle;              /* deg laser/sensor_mount_angle       :10                */
  float   scan_period;                     /* s   laser/scan_period              :11                */
  int32_t segment_valid_point_num;         /*     imageProjection/...            :14                */
  int32_t segment_valid_line_num;          /*                                    :15                */
  float   segment_theta;                   /* deg                                :16                */
  float   edge_threshold;                  /*     featureAssociation/...         :19                */
  float   surf_threshold;                  /*                                    :20                */
  float   nearest_feature_search_distance; /* m                                  :21                */
  int32_t mapping_frequency_divider;       /*     mapping/...                    :25                */
  int32_t fp_mode;                         /* libm overload model of the reference's unqualified
                                              sin/cos/tan/atan2/asin/sqrt calls on floats (SURVEY
                                              App. A.1): 0 = float overloads (libstdc++ >= 6's
                                              <math.h>: Melodic and later), 1 = ::sin(double) etc.,
                                              rounded where stored to float (GCC 4.8 / 5: the
                                              Indigo / Kinetic toolchains of README.md:40)          */
  int32_t voxel_tie_order;                 /* order in which PCL VoxelGrid sums the points of one
                                              voxel (featureAssociation.cpp:377-379): PCL sorts
                                              (voxel, point) pairs with std::sort by voxel only, so
                                              the order is the C++ library's.  0 = libstdc++'s
                                              introsort, emulated exactly (the reference as built
                                              with GCC); 1 = ascending point order (std::stable_sort;
                                              faster: no introsort emulation).  Centroids can differ
                                              in the last bits; voxel set, count and order do not. */
} lego_params;

/* pcl::PointXYZI payload (utility.h:46); 16 B, the device layout of every cloud. */
typedef struct lego_point { float x, y, z, intensity; } lego_point;

/* ProjectionOut (utility.h:64-70) + cloud_msgs::cloud_info (cloud_info.msg:1-13). */
typedef struct lego_projection_out {
  int32_t n_segmented;                       /* |segmented_cloud|  (M)                      */
  int32_t n_outlier;                         /* |outlier_cloud|                             */
  int32_t n_scan;                            /* |scan_msg| (2-D scan, imageProjection.cpp:312-330) */
  const lego_point* segmented_cloud;         /* [M]                                         */
  const lego_point* outlier_cloud;           /* [n_outlier]                                 */
  const lego_point* scan_msg;                /* [n_scan]                                    */
  const int32_t* start_ring_index;           /* cloud_info.startRingIndex [V]               */
  const int32_t* end_ring_index;             /* cloud_info.endRingIndex   [V]               */
  float start_orientation;                   /* cloud_info.startOrientation                 */
  float end_orientation;                     /* cloud_info.endOrientation                   */
  float orientation_diff;                    /* cloud_info.orientationDiff                  */
  const uint8_t*  segmented_cloud_ground_flag; /* [M]  (ROS bool[] = uint8)                 */
  const uint32_t* segmented_cloud_col_ind;     /* [M]                                       */
  const float*    segmented_cloud_range;       /* [M]                                       */
  /* diagnostics (the reference's _label_mat/_ground_mat/_range_mat), row-major V x H */
  const int32_t* label_mat;
  const int8_t*  ground_mat;
  const float*   range_mat;
} lego_projection_out;

/* One FeatureAssociation loop body: odometry + feature clouds + AssociationOut. */
typedef struct lego_association_out {
  int32_t status;                            /* LEGO_ST_* bits                              */
  int32_t n_sharp, n_less_sharp, n_flat, n_less_flat;
  const lego_point* corner_points_sharp;     /* fa.cpp:297  (after adjustDistortion frame)  */
  const lego_point* corner_points_less_sharp;/* fa.cpp:298,301                              */
  const lego_point* surf_points_flat;        /* fa.cpp:337                                  */
  const lego_point* surf_points_less_flat;   /* fa.cpp:381 (VoxelGrid per ring)             */
  const int32_t* sharp_ind;                  /* indices into the segmented cloud            */
  const int32_t* less_sharp_ind;
  const int32_t* flat_ind;
  float transform_cur[6];                    /* featureAssociation.h:96                     */
  float transform_sum[6];                    /* featureAssociation.h:97                     */
  double odom_orientation[4];                /* /laser_odom_to_init quaternion x,y,z,w (fa.cpp:1287-1294) */
  double odom_position[3];
  int32_t lm_iter_surf, lm_iter_corner;      /* iterations run (<=25 each)                  */
  int32_t n_corner_last, n_surf_last, n_outlier_last;
  const lego_point* cloud_corner_last;       /* AssociationOut::cloud_corner_last           */
  const lego_point* cloud_surf_last;         /* AssociationOut::cloud_surf_last             */
  const lego_point* cloud_outlier_last;      /* AssociationOut::cloud_outlier_last (axis-swapped, fa.cpp:1273-1283) */
} lego_association_out;

typedef struct lego_ctx   lego_ctx;    /* one sequence: ImageProjection + FeatureAssociation state */
typedef struct lego_batch lego_batch;  /* S independent sequences advanced one scan per step      */

/* ---- parameters ---------------------------------------------------------------- */
int32_t lego_abi_version(void);
/* The reference's loam_config.yaml (VLP-16). */
void lego_params_vlp16(lego_params* p);
/* HDL-64E-like synthetic config: V=64 evenly spaced -24.8..+2.0 deg, H=2048, G=55. */
void lego_params_hdl64(lego_params* p);
int  lego_params_validate(const lego_params* p);
/* lego_params from the reference's LeGO-LOAM/config/loam_config.yaml (the rosparam keys read by
 * imageProjection.cpp:57-84 and featureAssociation.cpp:69-81; block-style YAML): keys the file does not
 * set keep lego_params_vlp16's values; lego_loam/lego_amd/fp_mode and .../voxel_tie_order are this
 * build's own.  LEGO_EINVAL for an unreadable file, a malformed line or value, or parameters that
 * lego_params_validate rejects (*p is then unchanged).  Host only: needs no device. */
int  lego_params_load_yaml(const char* path, lego_params* p);
/* Number of visible HIP devices (0 when none). */
int32_t lego_device_count(void);

/* ---- single-sequence drop-in (replaces ImageProjection + FeatureAssociation) ----- */
/* ImageProjection ctor + FeatureAssociation ctor (imageProjection.cpp:32-104, featureAssociation.cpp:41-88). */
int  lego_ctx_create(const lego_params* p, int32_t device, lego_ctx** out);
void lego_ctx_destroy(lego_ctx* ctx);
/* ImageProjection::cloudHandler minus ROS (imageProjection.cpp:153-174).  Points are read zero-copy
 * from a strided host buffer (PointCloud2 data: x,y,z float32 at the given byte offsets).  Non-finite
 * points are dropped (removeNaNFromPointCloud, :160-161).  Returns the ProjectionOut (:538-547). */
int  lego_cloud_handler(lego_ctx* ctx, const void* points, int32_t n_points, int32_t point_step,
                        int32_t off_x, int32_t off_y, int32_t off_z, lego_projection_out* out);
/* One runFeatureAssociation iteration (featureAssociation.cpp:1389-1448) on the projection the last
 * lego_cloud_handler call produced (device-resident; the reference's Channel<ProjectionOut> hop). */
int  lego_feature_association(lego_ctx* ctx, lego_association_out* out);
/* Same, on a ProjectionOut supplied by the caller (host arrays), e.g. from another producer.
 * LEGO_EINVAL for a cloud_info imageProjection cannot produce (:358-396): a column index >= H, or a
 * ring whose [start, end] leaves [0, n_segmented) or spans more than H - 10 positions. */
int  lego_feature_association_from(lego_ctx* ctx, const lego_projection_out* in, lego_association_out* out);

/* ---- batched multi-sequence engine (throughput path) ------------------------------ */
int  lego_batch_create(const lego_params* p, int32_t device, int32_t n_streams, int32_t max_points,
                       lego_batch** out);
void lego_batch_destroy(lego_batch* b);
/* Advance every stream by one scan.  d_points: DEVICE array of lego_point (x,y,z,intensity);
 * stream s's scan is d_points[d_offsets[s] .. d_offsets[s] + d_counts[s]).  d_offsets / d_counts are
 * DEVICE arrays (int64 / int32) of length n_streams.  Asynchronous on hip_stream (NULL = default).
 * The step's VoxelGrid runs on an internal stream, overlapping other work.  With lag 1 (the default,
 * lego_batch_set_lag) the step runs its scan's front end and the PREVIOUS scan's LM, so the VoxelGrid
 * has two steps to finish; with lag 0 it runs its own scan's LM.  Whatever is left (the last scan's
 * LM and the lessFlat half of publishCloudsLast) is issued by the next step or by lego_batch_flush /
 * lego_batch_sync / lego_batch_read*, which all see completed scans.  Consecutive calls may use
 * different hip_streams: a call on a new stream first waits for all work enqueued on the previous
 * one. */
int  lego_batch_step(lego_batch* b, const lego_point* d_points, const int64_t* d_offsets,
                     const int32_t* d_counts, void* hip_stream);
/* Enqueue the pending work (the last scan's LM / publish) on the last step's stream (asynchronous);
 * then a synchronize of that stream sees every output of the last step. */
int  lego_batch_flush(lego_batch* b);
int  lego_batch_sync(lego_batch* b);
/* Copy one stream's last projection / association outputs to host (blocking). */
int  lego_batch_read(lego_batch* b, int32_t s, lego_projection_out* proj, lego_association_out* assoc);
/* Poses of all streams: out[s*12 + 0..5] = transformCur, [6..11] = transformSum; status[s]. */
int  lego_batch_read_poses(lego_batch* b, float* out, int32_t* status);
/* Per-scan odometry of every stream (publishOdometry runs every scan, featureAssociation.cpp:1286-1298):
 * while set, each association of stream s writes d_traj[(s * max_scans + k) * 12 + 0..5] = transformCur
 * and [6..11] = transformSum after it, k = the stream's association count since lego_batch_reset (0:
 * the initialising scan); associations past max_scans are not recorded.  d_traj is a DEVICE array of
 * n_streams * max_scans * 12 floats, written asynchronously by the LM kernel (read it after
 * lego_batch_sync).  d_traj NULL / max_scans 0 stops recording. */
int  lego_batch_set_trajectory(lego_batch* b, float* d_traj, int32_t max_scans);
/* Sizes of the last step per stream: out[s*7 + 0..6] = segmented, outlier, scan_msg, sharp,
 * less sharp, flat, less flat point counts. */
int  lego_batch_read_counts(lego_batch* b, int32_t* out);
/* Reset every stream to the freshly constructed state (systemInitedLM = false, transforms 0). */
int  lego_batch_reset(lego_batch* b);
/* Checkpoint / resume of stream s (shard warm-start, restart after a failure): the FeatureAssociation state one
 * scan leaves for the next (featureAssociation.h:70-115: transformCur / transformSum, systemInitedLM,
 * isDegenerate, the cycle count, the Last clouds and the kd-trees' staleness, the odometry) plus the
 * persistent curvature / picked / label / smoothness vectors whose stale entries the next scan reads, in
 * lego_batch_state_size bytes of host memory.  Save flushes the pending publish / LM first; load requires the
 * same sensor layout (V, H, cap_lsharp; else LEGO_EINVAL) and may target another stream or batch.  A stream
 * loaded from a checkpoint continues exactly as the saved stream would. */
int  lego_batch_state_size(const lego_batch* b, size_t* bytes);
int  lego_batch_save_state(lego_batch* b, int32_t s, void* host, size_t bytes);
int  lego_batch_load_state(lego_batch* b, int32_t s, const void* host, size_t bytes);
int  lego_ctx_state_size(const lego_ctx* ctx, size_t* bytes);
int  lego_ctx_save_state(lego_ctx* ctx, void* host, size_t bytes);
int  lego_ctx_load_state(lego_ctx* ctx, const void* host, size_t bytes);
/* Kernel timing of the last step (ms, hipEvents on the step's stream, the pipelined path itself):
 * [0] project, [1] segment + distortion, [2] smoothness + occlusion, [3] feature extraction,
 * [4] concat + the pending lessFlat publish, [5] LM (of the previous scan with lag 1; the VoxelGrid
 * overlaps it on an internal stream). */
int  lego_batch_stage_times(lego_batch* b, float* ms6);
/* Measurement: the projection and smoothness stages (the HBM-bound pair) launched `reps` times back
 * to back on the inputs of the batch's last step (the same device arrays), between two events on
 * hip_stream; *ms_pair = mean milliseconds of one pair.  d_offsets_alt / d_counts_alt (nullable):
 * another input set in d_points; the projections alternate between the two sets, the last launch on
 * the step's own.  Idempotent: the batch's results are unchanged.  Synchronises the device first.  bench.py's roofline. */
int  lego_batch_time_hbm_stages(lego_batch* b, int32_t reps, const lego_point* d_points, const int64_t* d_offsets,
                                const int32_t* d_counts, const int64_t* d_offsets_alt, const int32_t* d_counts_alt,
                                void* hip_stream, float* ms_pair);
/* Measurement: the VoxelGrid stage (PCL VoxelGrid of every ring's lessFlat cloud, featureAssociation.cpp:
 * 377-379) of the batch's last step launched `reps` times back to back on hip_stream, alone on the device
 * (it synchronises first); *ms = mean milliseconds a launch.  Idempotent (same staged input, same output).
 * LEGO_EINVAL before the batch's first step (nothing staged).  bench.py's stages_ms.voxel_alone. */
int  lego_batch_time_voxel(lego_batch* b, int32_t reps, void* hip_stream, float* ms);
/* While timing is enabled, steps run as one slice on the caller's stream (plus the VoxelGrid stream). */
int  lego_batch_set_timing(lego_batch* b, int32_t enabled);
/* Measurement: while the probe is on, every overlap-schedule step records events around its projection
 * (k_project / the wide projection) and around its smoothness stage (k_fa_prep4) on the step's stream;
 * lego_batch_probe_times returns their mean durations inside the pipeline (ms2[0] projection, ms2[1]
 * smoothness, over *steps steps; the concurrent LM of the previous scan included) and clears them.
 * bench.py's in-pipeline roofline. */
int  lego_batch_set_probe(lego_batch* b, int32_t enabled);
int  lego_batch_probe_times(lego_batch* b, float* ms2, int32_t* steps);
/* Split the streams into `groups` (1..LEGO_MAX_GROUPS) slices, each launched on its own internal HIP
 * stream (forked from and joined back into the step's stream), so one slice's long-tail kernels
 * overlap the others'.  Results do not depend on the grouping. */
#define LEGO_MAX_GROUPS 4
int  lego_batch_set_groups(lego_batch* b, int32_t groups);
/* Pipeline depth of lego_batch_step: 0 = a step runs its own scan's LM, 1 = the previous scan's, 2 = the
 * one before (the VoxelGrid of a scan gets two steps before its publish; one stream group and timing
 * off, else run as 1; see lego_batch_step), -1 (default) = automatic: 2 with voxel_tie_order 0 and at
 * most half as many streams as compute units, else 1.  Results do not depend on it. */
int  lego_batch_set_lag(lego_batch* b, int32_t lag);
/* The pipeline depth lego_batch_step runs (0, 1 or 2: a requested 2 reads 1 while the streams are sliced
 * into groups > 1 or timing is on), or LEGO_EINVAL. */
int  lego_batch_lag(const lego_batch* b);
/* Kernel layout of the projection and segmentation: 1 = wide (a scan's work over many workgroups,
 * per-scan images in HBM), 0 = one workgroup a scan with its images in LDS (only where they fit:
 * V <= 16, V*H < 32768; else LEGO_EINVAL), 2 = the one-workgroup projection with the wide
 * segmentation (where the projection's image fits LDS), -1 (default) = automatic: wide where the images
 * do not fit LDS or where at most (compute units / 8) streams are in flight; else 0.  Results do not
 * depend on it. */
int  lego_batch_set_wide(lego_batch* b, int32_t mode);
/* The layout in effect (0, 1 or 2 as lego_batch_set_wide), or LEGO_EINVAL. */
int  lego_batch_wide(const lego_batch* b);

/* ---- test hooks ------------------------------------------------------------------ */
/* Evaluate the device libm restatement on host arrays: which = 0 asinf(a), 1 atan2f(a, b),
 * 2 atanf(a), 3 sqrtf(a), 4 a / b.  Lets tests compare gfx950 results with the host's glibc.
 * which = 5 / 6: groundRemoval's pair test atan2f(dZ = a, r = b) <= 10 deg (mount 0) as k_project
 * decides it (polynomial with a margin, glibc-faithful fallback) / by the glibc-faithful path only.
 * which = 7 / 8: sinf(a) / cosf(a) (the LM trig).  which = 9 / 10: the pair test in fp_mode 1 (va =
 * (float)atan2(double(dZ), sqrt(double(s2)))), fast + exact / exact only; 11: fp_mode 0 exact only.
 * (5, 6, 9, 10, 11 take s2 = b * b.) */
int  lego_test_libm(const float* a, const float* b, float* out, int32_t n, int32_t which);
/* The device's double libm of fp_mode 1 (lego_libm.h, fdlibm): which = 0 sin(a), 1 cos(a), 2 atan2(a, b),
 * 3 asin(a), 4 sqrt(a), 5 a / b. */
int  lego_test_libm_d(const double* a, const double* b, double* out, int32_t n, int32_t which);
/* Sort (key, val) pairs by key with the device's wave-parallel std::sort emulation (n <= 2048);
 * keys are uint32 (is_float 0) or float bit patterns (1); is_float 2 runs k_extract's segment
 * sort (float keys, n <= 512: register sort when keys are distinct, else the emulation); is_float 3
 * runs k_voxel's level-synchronous emulation (uint32 keys, values < 2^16). */
int  lego_test_sort(uint32_t* keys, int32_t* vals, int32_t n, int32_t is_float);
/* Projection cell (row * H + col, or -1 = rejected) of n points (x, y, z, w float32) by the fast path
 * of k_project (-2 = too close to a decision boundary, decided by the exact path) and by the exact
 * glibc-faithful path (imageProjection.cpp:186-207). */
int  lego_test_project_cells(const lego_params* p, const float* xyzw, int32_t n, int32_t* fast, int32_t* exact);
/* Overwrite the LM state the next lego_feature_association* call starts from: transformCur (the warm
 * start), transformSum, isDegenerate, the Last clouds (TransformToEnd'ed, as AssociationOut returns them)
 * and the kd-trees' staleness (fa.cpp:1356).  LEGO_EINVAL before the first association.  For per-pair LM
 * parity with a reference's state injected. */
int  lego_test_set_lm_state(lego_ctx* ctx, const float* transform_cur, const float* transform_sum,
                            int32_t degenerate, const lego_point* corner_last, int32_t n_corner,
                            const lego_point* surf_last, int32_t n_surf, int32_t tree_stale);
/* nanoflann's kNN as the device resolves exact distance ties (the tree built as nanoflann 1.3.0 builds
 * it, its searchLevel with a KNNResultSet(k)): k = 1 the LM's 1-NN, k = 5 scan-to-map's kNN-5; m queries
 * against a cloud of n points (x, y, z, w float32 each); out idx[m][k] nearest first (-1 past the count
 * found, -2: search stack overflow) and squared distances. */
int  lego_test_kd_knn(const float* cloud, int32_t n, const float* queries, int32_t m, int32_t k, int32_t* idx,
                      float* dist);
#ifdef __cplusplus
}
#endif
#endif /* LEGO_FRONTEND_H */
