// lego_device.h — device-side types and libm restatement for the gfx950 kernels.
//
// Numerics contract: every kernel is compiled with -ffp-contract=off
// (x86-64 reference has no FMA), float division/sqrt correctly rounded (HIP default), and the
// reference's float/double promotions written out explicitly.
//
// libm: the reference calls glibc's float asinf / atan2f (std::asin/std::atan2 on float, and the
// unqualified float overloads, fp_mode 0).  glibc 2.35's implementations of these are the fdlibm
// algorithms (flt-32/e_asinf.c, s_atanf.c, e_atan2f.c): restated below operation for operation.
// Verified bit-identical against the container's glibc on all 2^31 asinf inputs in [-1,1], every
// 3rd float for atanf and 3e8 random atan2f pairs (tests/test_libm.py keeps a sampled check).
// sinf/cosf (used only inside the LM, which is checked within tolerance) are evaluated in double
// and rounded once.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define LG_DEVICE __device__ __forceinline__

#include "lego_libm.h"

// Streaming (non-temporal) vector stores for outputs that no later instruction of the same kernel
// reads: they do not displace lines the kernel still reads back through L2 (k_project's column pass
// re-gathers the winning input points).
LG_DEVICE void st_nt(float* p, float v) { __builtin_nontemporal_store(v, p); }
LG_DEVICE void st_nt(int* p, int v) { __builtin_nontemporal_store(v, p); }
LG_DEVICE void st_nt(int8_t* p, int8_t v) { __builtin_nontemporal_store(v, p); }
LG_DEVICE void st_nt(uint8_t* p, uint8_t v) { __builtin_nontemporal_store(v, p); }
LG_DEVICE void st_nt(float4* p, float4 v) {
  typedef float f4v __attribute__((ext_vector_type(4)));
  const f4v w = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(w, (f4v*)p);
}
LG_DEVICE void st_nt(int2* p, int2 v) {
  typedef int i2v __attribute__((ext_vector_type(2)));
  const i2v w = {v.x, v.y};
  __builtin_nontemporal_store(w, (i2v*)p);
}


// ---- shared POD types (host + device) ---------------------------------------------------------
struct LgParams {  // ImageProjection / FeatureAssociation ctor constants (host-derived)
  int V, H, G, VH;
  float ang_res_x, ang_res_y, ang_bottom, mount;
  float sinX, cosX, sinY, cosY, theta_thr;
  int seg_valid_pt, seg_valid_line;
  float scan_period, edge_thr, surf_thr, nn_dist_sqr;
  int map_div;
  int cap_sharp, cap_lsharp, cap_flat;  // per-ring caps: 12, 120, 24
  int s0;                               // first stream of the launch (stream groups; 0 otherwise)
  int ncu;                              // compute units of the device (k_extract's ring rotation)
  int voxel_stable;                     // lego_params.voxel_tie_order == 1
  int epoch;                            // per-launch token for k_extract's first-pass flags
  float inv_res_x, inv_res_y;           // (float)(1 / ang_res_*) for the fast projection path
  int fast_proj;                        // the fast path's margins hold for these resolutions
  int par;                              // staging slot of the launch's scan (scan index mod LG_SLOTS):
                                        // its features, lessFlat and VoxelGrid output
  int S;                                // streams of the batch (staging stride)
  int wide;                             // 1: k_pw_* / k_sw_* (many workgroups a scan); 2: k_project, k_sw_*
  unsigned wtag;                        // wide mode: launch tag in the winner image entries' top 4 bits
  int max_points;                       // input capacity per scan (wide scatter grid)
  int fp1;                              // lego_params.fp_mode == 1: unqualified libm calls in double
  int traj_cap;                         // scans a stream's trajectory record holds (0: none; LgBufs.traj)
  double sinXd, cosXd, sinYd, cosYd;    // fp_mode 1: sin / cos(double(alpha)) of labelComponents (:463)
};

struct LgState {  // FeatureAssociation members that persist across scans (featureAssociation.h)
  float cur[6];
  float sum[6];
  int initialized;       // systemInitedLM
  int is_degenerate;     // isDegenerate
  int cycle;             // _cycle_count
  int last_buf;          // which half of the Last double buffer holds *Last
  int n_corner_last, n_surf_last;
  int tree_stale;        // kd-trees were not rebuilt at the last publishCloudsLast
  int status;            // LEGO_ST_* of the last association
  int iters_surf, iters_corner;
  int pub_copy;          // k_publish stores the lessFlat cloud untransformed (checkSystemInitialization)
  int n_assoc;           // associations run on this stream since the reset (the trajectory record's index)
  int pad_;
  double quat[4];  // (unused: the odometry quaternion is computed on the host at readback, odom_quat)
  double pos[3];
};

// counts[] slots per stream
enum {
  CNT_M = 0, CNT_OUTLIER = 1, CNT_SCAN = 2, CNT_SHARP = 3, CNT_LSHARP = 4, CNT_FLAT = 5, CNT_LFLAT = 6,
  CNT_STATUS = 7, CNT_N = 8
};

// nanoflann kd-tree node (exact-tie resolution of the LM's 1-NN): children (-1: leaf), vind range,
// split dimension and the children's facing bounds (nanoflann.hpp node_type.sub / .lr)
struct KdNode {
  int c1, c2, left, right;
  int divfeat;
  float divlow, divhigh;
  int pad;
};

// Staging slots of the front end -> VoxelGrid -> LM pipeline: scan k uses slot k mod LG_SLOTS, whose
// previous user (scan k - LG_SLOTS) has published before scan k's k_concat refills it.
#define LG_SLOTS 3

struct LgBufs {  // device buffers, all indexed [stream][...]
  // ImageProjection
  float* range;          // [S][VH]
  float4* cloud;         // [S][VH]  _full_cloud
  int8_t* ground;        // [S][VH]
  int32_t* label;        // [S][VH]
  int32_t* winner;       // [S][VH]  wide mode: "later point wins" image (tagged entries, column-major)
  int32_t* proj_mm;      // [S][2]   wide mode: first / last finite input point
  int32_t* colcnt;       // [S][H]   wide mode: k_pw_slice's touches a column (k_pw_fix reads and clears it)
  int32_t* cc_parent;    // [S][VH]  wide mode: union-find parent (or -1: not eligible)
  int32_t* cc_cnt;       // [S][VH]  component size of a root, then its label
  unsigned long long* cc_mask;  // [S][VH]  rows of a root's non-seed members
  int4* seg_tiles;       // [S][tiles] wide mode: per tile feasible roots, segmented cells, outliers
  int32_t* scan_cand;    // [S][H]
  float* orient;         // [S][4]
  float4* seg_pts;       // [S][VH]
  float* seg_range;      // [S][VH]
  uint32_t* seg_col;     // [S][VH]
  uint8_t* seg_ground;   // [S][VH]
  int32_t* ring_start;   // [S][V]
  int32_t* ring_end;     // [S][V]
  float4* outlier;       // [S][VH]
  float4* scan_msg;      // [S][H]
  int32_t* counts;       // [S][CNT_N]
  // FeatureAssociation persistent work arrays
  float* curv;           // [S][VH]
  uint8_t* picked;       // [S][VH]
  int8_t* flabel;        // [S][VH]
  int2* smooth;          // [S][VH]  {float bits of value, ind}
  uint16_t* xinfo;       // [S][VH]  k_extract's per-position greedy state, built by k_sortseg
  int32_t* fp_sync;      // [S][2]   stale ind of smoothness slot 4, first-pass done epoch
  float4* seg_fa;        // [S][VH]  segmentedCloud after adjustDistortion
  float4* outlier_fa;    // [S][VH]  adjustOutlierCloud
  // per-ring staging
  float4* r_sharp; int32_t* r_sharp_ind;    // [S][V][cap_sharp]
  float4* r_lsharp; int32_t* r_lsharp_ind;  // [S][V][cap_lsharp]
  float4* r_flat; int32_t* r_flat_ind;      // [S][V][cap_flat]
  int32_t* r_counts;                        // [S][V][4]   sharp, lessSharp, flat (k_extract), unused
  int32_t* r_status;                        // [S][V]      k_extract status bits
  // [LG_SLOTS][...]: slots by scan (LgParams.par = scan index mod LG_SLOTS), so scan k's VoxelGrid /
  // publish / LM may run while scans k+1 and k+2 fill the other slots (pipeline lag up to 2)
  float4* lf_stage;                         // [LG_SLOTS][S][V][H] surfPointsLessFlatScan per ring (k_concat)
  int32_t* lf_count;                        // [LG_SLOTS][S][V]
  float4* r_lflat;                          // [LG_SLOTS][S][V][H] VoxelGrid output per ring (k_voxel)
  int32_t* r_vcount;                        // [LG_SLOTS][S][V]    its point count
  int32_t* r_vstatus;                       // [LG_SLOTS][S][V]    k_voxel status bits
  // concatenated features
  float4* f_sharp; int32_t* f_sharp_ind;    // [LG_SLOTS][S][V*cap_sharp]
  float4* f_lsharp; int32_t* f_lsharp_ind;  // [LG_SLOTS][S][V*cap_lsharp]
  float4* f_flat; int32_t* f_flat_ind;      // [LG_SLOTS][S][V*cap_flat]
  int32_t* fcnt;                            // [LG_SLOTS][S][4]  sharp, lessSharp, flat counts, status (k_lm)
  float4* f_lflat;                          // [S][VH]
  // Last clouds, double-buffered
  float4* corner_last;   // [S][2][V*cap_lsharp]
  float4* surf_last;     // [S][2][VH]
  float4* grid_pts;      // [S][VH]  LM scratch: Last cloud bucketed by grid cell (xyz, index bits)
  LgState* state;        // [S]      written by k_lm / k_publish only (k_lm stores it whole)
  float* traj;           // [S][traj_cap][12]  optional (lego_batch_set_trajectory): transformCur and
                         //          transformSum after each association of the stream, by k_lm
  // nanoflann tree of a Last cloud, built by k_lm only when a 1-NN has an exact distance tie
  KdNode* kd_node;       // [S][2*VH]
  int32_t* kd_vind;      // [S][VH]
  int32_t* kd_tmp;       // [S][2*VH]  stop positions of planeSplit's passes
  float* kd_frames;      // [S][10*VH] build stack, then the searches' stacks
  int32_t* fe_state;     // [S][2]   written by the front end only: [0] 0 or LEGO_EEMPTY for the last
                         // projection; [1] scans whose features k_concat has assembled, > 0 at a scan's
                         // front end iff its FeatureAssociation pass is not the initialising one
                         // (adjustOutlierCloud runs in publishCloudsLast, :1273-1283, which the first
                         // pass skips), however far the LM lags behind
};
