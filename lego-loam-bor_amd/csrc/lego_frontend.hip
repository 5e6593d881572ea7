// lego_frontend.hip — host engine + C-ABI (include/lego_frontend.h).
//
// A lego_batch owns S independent sequences ("streams") laid out stream-major in HBM and advances
// all of them by one scan per step with one launch per stage (lego_kernels.hip).  A lego_ctx is a
// batch of one plus host staging: the drop-in for one ImageProjection + FeatureAssociation pair.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <cfloat>
#include <cstdlib>
#include <new>
#include <utility>
#include <vector>

#include "../../include/lego_frontend.h"
#include "lego_device.h"

int lg_launch_project(const LgParams& P, const LgBufs& B, int S, const float4* pts, const int64_t* offs,
                      const int32_t* cnts, hipStream_t st);
int lg_launch_segment(const LgParams& P, const LgBufs& B, int S, hipStream_t st);
int lg_launch_fa_prep(const LgParams& P, const LgBufs& B, int S, hipStream_t st, bool distort);
int lg_launch_extract(const LgParams& P, const LgBufs& B, int S, hipStream_t st);
int lg_launch_concat(const LgParams& P, const LgBufs& B, int S, hipStream_t st);
int lg_launch_lm(const LgParams& P, const LgBufs& B, int S, hipStream_t st);
int lg_launch_voxel(const LgParams& P, const LgBufs& B, int S, hipStream_t st);
int lg_launch_publish(const LgParams& P, const LgBufs& B, int S, hipStream_t st);

namespace {

const double DEG_TO_RAD = M_PI / 180.0;  // utility.h:50

// ImageProjection / FeatureAssociation ctor arithmetic with the reference's types
// (imageProjection.cpp:57-84, featureAssociation.cpp:69-81); glibc trig for the labelComponents
// constants (:414, :463), as the reference evaluates them per call: the float overloads (fp_mode 0)
// or ::tan / ::sin / ::cos in double (fp_mode 1).
LgParams derive(const lego_params& p) {
  LgParams P;
  memset(&P, 0, sizeof(P));
  P.V = p.num_vertical_scans;
  P.H = p.num_horizontal_scans;
  P.G = p.ground_scan_index;
  P.VH = P.V * P.H;
  float ang_bottom = p.vertical_angle_bottom;
  float top = p.vertical_angle_top;
  P.ang_res_x = (M_PI * 2) / (P.H);
  P.ang_res_y = DEG_TO_RAD * (top - ang_bottom) / float(P.V - 1);
  P.ang_bottom = -(ang_bottom - 0.1) * DEG_TO_RAD;
  float theta = p.segment_theta;
  theta *= DEG_TO_RAD;
  float mount = p.sensor_mount_angle;
  mount *= DEG_TO_RAD;
  P.mount = mount;
  P.fp1 = p.fp_mode == 1;
  P.theta_thr = P.fp1 ? (float)tan((double)theta) : tanf(theta);
  // the reference's sin(alpha) / cos(alpha) pair, merged into one sincos by GCC (see oracle Lm<double>)
  sincos((double)P.ang_res_x, &P.sinXd, &P.cosXd);
  sincos((double)P.ang_res_y, &P.sinYd, &P.cosYd);
  P.sinX = sinf(P.ang_res_x);
  P.cosX = cosf(P.ang_res_x);
  P.sinY = sinf(P.ang_res_y);
  P.cosY = cosf(P.ang_res_y);
  P.seg_valid_pt = p.segment_valid_point_num;
  P.seg_valid_line = p.segment_valid_line_num;
  P.scan_period = p.scan_period;
  P.edge_thr = p.edge_threshold;
  P.surf_thr = p.surf_threshold;
  float nd = p.nearest_feature_search_distance;
  P.nn_dist_sqr = nd * nd;
  P.map_div = p.mapping_frequency_divider;
  P.voxel_stable = p.voxel_tie_order == 1;
  P.cap_sharp = 12;   // 2 per segment x 6 (fa.cpp:295)
  P.cap_lsharp = 120; // 20 per segment x 6 (fa.cpp:299)
  P.cap_flat = 24;    // 4 per segment x 6 (fa.cpp:340)
  // fast projection path (lego_kernels.hip proj_cell_fast): margins hold for resolutions >= 0.1 deg
  P.inv_res_x = (float)(1.0 / (double)P.ang_res_x);
  P.inv_res_y = (float)(1.0 / (double)P.ang_res_y);
  P.fast_proj = (double)P.ang_res_x >= 0.1 * DEG_TO_RAD && (double)P.ang_res_y >= 0.1 * DEG_TO_RAD;
  return P;
}

template <typename T>
int dalloc(T** p, size_t n, std::vector<void*>& owned) {
  if (n == 0) n = 1;
  if (hipMalloc((void**)p, n * sizeof(T)) != hipSuccess) return LEGO_ENOMEM;
  owned.push_back((void*)*p);
  return LEGO_OK;
}

// Pinned (page-locked) host buffer, grown on demand: device-to-host copies into it are truly
// asynchronous, so a read issues all its copies on one stream and waits once.
struct Pinned {
  void* p = nullptr;
  size_t cap = 0;
  template <typename T>
  T* get(size_t n) {
    const size_t bytes = (n > 0 ? n : 1) * sizeof(T);
    if (bytes > cap) {
      if (p) hipHostFree(p);
      p = nullptr;
      cap = 0;
      if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) return nullptr;
      cap = bytes;
    }
    return (T*)p;
  }
  ~Pinned() {
    if (p) hipHostFree(p);
  }
};

// async copy of n elements into pinned h; *out = host pointer (valid until the next read)
template <typename T>
int d2h(Pinned& h, const T* d, size_t n, hipStream_t st, T** out) {
  T* hp = h.get<T>(n);
  if (!hp) return LEGO_ENOMEM;
  *out = hp;
  if (n == 0) return LEGO_OK;
  return hipMemcpyAsync(hp, d, n * sizeof(T), hipMemcpyDeviceToHost, st) == hipSuccess ? LEGO_OK : LEGO_EDEVICE;
}

}  // namespace

int lg_derive_params(const lego_params& p, LgParams* out) {  // test hooks (lego_kernels.hip)
  const int rc = lego_params_validate(&p);
  if (rc != LEGO_OK) return rc;
  *out = derive(p);
  return LEGO_OK;
}

bool lg_lds_projection(const LgParams& P);  // lego_kernels.hip
bool lg_lds_segment(const LgParams& P);

// Wide mode (k_pw_* / k_sw_*: a scan's projection and segmentation over many workgroups) where one
// workgroup a scan cannot hold the images in LDS, and where too few scans are in flight to fill
// the device with one workgroup each.
// The wide layout (many small workgroups a scan) where the one-workgroup-a-scan kernels cannot hold the
// scan in LDS, for few scans, and for the reference's VoxelGrid order with at most one scan a CU.  With
// that order a scan's VoxelGrid launch (one wave a ring) runs ~0.85 ms, set by its few heap-sort-bound
// rings; once it no longer waits behind the previous launch it overlaps the next scan's front end, and
// one VoxelGrid wave on a SIMD already keeps the whole-CU k_project (4 x 110 VGPRs a SIMD) and
// k_segment_lds (4 x 128) off that CU, while the wide kernels' small workgroups fill the room left
// (round 5, same box: 235.1-237.8k vs 212.2-216.7k scans/s).
static int lg_wide_auto(const LgParams& P, int S) {
  return (!lg_lds_projection(P) || !lg_lds_segment(P) || S * 8 <= P.ncu || (!P.voxel_stable && S <= P.ncu)) ? 1 : 0;
}

#define LG_PROBE_MAX 64  // probe events kept: the last LG_PROBE_MAX steps (lego_batch_probe_times)

// Automatic pipeline depth: lag 2 for the reference's VoxelGrid order with at most half as many scans as
// compute units (its slowest ring, a heap-sort fallback of ~1 ms, then needs more than one short step:
// C5's 80 sequences 156k vs 104k scans/s), else lag 1 (C3's 256: 230-236k vs 214-216k).
static int lg_lag_auto(const LgParams& P, int S) { return (!P.voxel_stable && 2 * S <= P.ncu) ? 2 : 1; }

struct lego_batch {
  lego_params params;
  LgParams P;
  int wide_req = -1;  // lego_batch_set_wide: -1 auto, 0 / 1 forced
  LgBufs B;
  int S = 0;
  int max_points = 0;
  int device = 0;
  std::vector<void*> owned;
  hipEvent_t ev[8];
  bool timing = false;
  bool events = false;
  int epoch = 0;  // k_extract first-pass token (LgParams.epoch), never 0 after the first launch
  int wepoch = 0;  // wide projection's launch counter 1..15 (LgParams.wtag), 0: image zeroed
  // stream groups: the S sequences split into `groups` slices, each launched on its own HIP stream
  // so one slice's long-tail kernels overlap the next slice's (fork/join on the caller's stream)
  int groups = 1;
  hipStream_t gs[LEGO_MAX_GROUPS] = {};
  hipEvent_t fork = nullptr, join[LEGO_MAX_GROUPS] = {};
  // The stream of the last call that enqueued work; a step on another stream first waits for
  // everything enqueued there (ev_chain), so the pending kernels it issues are ordered after it.
  hipStream_t last_stream = nullptr;
  bool has_last = false;
  hipEvent_t ev_chain = nullptr;
  // Pipeline (per scan k of every stream): front end(k) -> k_concat(k) -> k_voxel(k) on the side
  // stream vs -> k_publish(k) after k_lm(k) and k_voxel(k), before k_lm(k+1).  Each scan uses the
  // staging half of its parity, so the next scan's front end never waits for it.
  //   lag 0: step k runs k_publish(k-1), then k_lm(k);  k_publish(k) stays pending.
  //   lag 1: step k runs k_publish(k-2), then k_lm(k-1); k_publish(k-1) and k_lm(k) stay pending,
  //          so k_voxel(k) has two steps of other work to hide behind.
  //   lag 2 (overlap schedule only; the others run it as lag 1): step k runs k_publish(k-3), then
  //          k_lm(k-2); k_voxel(k) starts a whole step before k_lm(k) and is due only at k_publish(k),
  //          and consecutive VoxelGrid launches alternate between two streams, so one launch's
  //          slowest ring no longer holds the next one back.
  // lego_batch_flush (and every read) issues what is pending.
  int lag = 1;
  int lag_req = -1;  // lego_batch_set_lag: -1 automatic (lg_lag_auto)
  hipStream_t vs[LEGO_MAX_GROUPS] = {};
  hipEvent_t ev_cat[LEGO_MAX_GROUPS] = {}, ev_vox[LEGO_MAX_GROUPS][LG_SLOTS] = {};
  hipEvent_t ev_cats[LG_SLOTS] = {};  // overlap schedule: k_concat of the scan in each slot
  bool fe_ran = false;       // a front-end step has staged input since create / reset (lego_batch_time_voxel)
  int vox_alt = 0;           // lag 2: the stream of the next VoxelGrid launch (vs[0] / gs[0])
  int par = 0;               // staging slot of the next front-end scan
  int last_par = 0;          // slot of the last front-end scan (reads)
  bool pend_pub = false;     // k_publish of a scan whose k_lm has run (slot pub_par)
  int pub_par = 0;
  bool pend_lm = false;      // k_lm of the last front-end scan (lag >= 1; slot lm_par)
  int lm_par = 0;
  bool pend_lm_old = false;  // lag 2: k_lm of the scan before it (slot lm_par_old)
  int lm_par_old = 0;
  int pend_groups = 1;       // slicing of the pending work
  // Overlap schedule (one slice, lag 1, timing off): k_publish(k-2) and k_lm(k-1) go to the internal
  // LM stream ls at the start of step k, ordered after k_concat(k-1) (ev_cat) and k_voxel(k-2)
  // (ev_vox), so a CU whose scan's LM has finished takes the next front end's workgroups instead of
  // idling until the slowest LM of the launch ends.  k_concat(k) waits for k_publish(k-2) (ev_pub),
  // which follows k_lm(k-2) on ls: the feature / staging halves of parity k are free then.
  bool pend_ovl = false;     // the pending work belongs to the overlap schedule
  hipStream_t ls = nullptr;
  hipEvent_t ev_pub = nullptr, ev_ls = nullptr, ev_fe = nullptr;

  // Probe (lego_batch_set_probe): events around k_project and around k_fa_prep in the overlap
  // schedule, four per step, so the HBM-bound pair's durations inside the pipeline can be read
  // (lego_batch_probe_times) beside the back-to-back figure of lego_batch_time_hbm_stages.  A ring of
  // LG_PROBE_MAX steps: a probe left on reuses the oldest events instead of growing the list.
  bool probe = false;
  std::vector<hipEvent_t> pev;
  int probe_n = 0;
  hipEvent_t* probe_cur = nullptr;  // this step's four events while it is being enqueued
  // pinned host mirrors for lego_batch_read / the single-context outputs
  Pinned h_seg, h_out, h_scan, h_sharp, h_lsharp, h_flat, h_lflat, h_clast, h_slast, h_olast;
  Pinned h_rs, h_re, h_label, h_sharp_ind, h_lsharp_ind, h_flat_ind, h_gflag, h_col, h_range_seg, h_range, h_ground;
  Pinned h_hdr;  // counts, orientation and state of the stream being read
  ~lego_batch() {
    hipSetDevice(device);
    hipDeviceSynchronize();  // nothing of this batch may still run on its buffers or streams
    for (void* p : owned) hipFree(p);
    if (events)
      for (int i = 0; i < 8; ++i) hipEventDestroy(ev[i]);
    for (hipEvent_t e : pev) hipEventDestroy(e);
    for (int g = 0; g < LEGO_MAX_GROUPS; ++g) {
      if (gs[g]) hipStreamDestroy(gs[g]);
      if (join[g]) hipEventDestroy(join[g]);
      if (vs[g]) hipStreamDestroy(vs[g]);
      if (ev_cat[g]) hipEventDestroy(ev_cat[g]);
      for (int h = 0; h < LG_SLOTS; ++h)
        if (ev_vox[g][h]) hipEventDestroy(ev_vox[g][h]);
    }
    for (int h = 0; h < LG_SLOTS; ++h)
      if (ev_cats[h]) hipEventDestroy(ev_cats[h]);
    if (fork) hipEventDestroy(fork);
    if (ev_chain) hipEventDestroy(ev_chain);
    if (ls) hipStreamDestroy(ls);
    if (ev_pub) hipEventDestroy(ev_pub);
    if (ev_ls) hipEventDestroy(ev_ls);
    if (ev_fe) hipEventDestroy(ev_fe);
  }
};

// Mapped, coherent pinned host memory that kernels write directly (the single-context readback)
struct Mapped {
  char* p = nullptr;   // host pointer
  char* dp = nullptr;  // device pointer to the same memory
  size_t cap = 0;
  int alloc(size_t bytes) {
    if (hipHostMalloc((void**)&p, bytes, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
      p = nullptr;
      return LEGO_ENOMEM;
    }
    if (hipHostGetDevicePointer((void**)&dp, p, 0) != hipSuccess) return LEGO_EDEVICE;
    cap = bytes;
    return LEGO_OK;
  }
  ~Mapped() {
    if (p) hipHostFree(p);
  }
};

struct lego_ctx {
  lego_batch* b = nullptr;
  float4* d_in = nullptr;  // [0]: the point count (int32), [1, cap]: the points
  int64_t* d_off = nullptr;
  int cap = 0;
  Pinned h_in;       // fromROSMsg gather target, count first (pinned: one asynchronous upload)
  Mapped pk_proj;    // ProjectionOut arrays, written by k_pack (layout: proj_layout)
  Mapped pk_assoc;   // AssociationOut arrays (assoc_layout)
  ~lego_ctx() {
    if (b) {
      hipSetDevice(b->device);
      hipDeviceSynchronize();
      if (d_in) hipFree(d_in);
      if (d_off) hipFree(d_off);
      delete b;
    }
  }
};

extern "C" {

int32_t lego_abi_version(void) { return LEGO_ABI_VERSION; }

void lego_params_vlp16(lego_params* p) {  // LeGO-LOAM/config/loam_config.yaml
  p->num_vertical_scans = 16;
  p->num_horizontal_scans = 1800;
  p->ground_scan_index = 7;
  p->vertical_angle_bottom = -15.f;
  p->vertical_angle_top = 15.f;
  p->sensor_mount_angle = 0.f;
  p->scan_period = 0.1f;
  p->segment_valid_point_num = 5;
  p->segment_valid_line_num = 3;
  p->segment_theta = 60.f;
  p->edge_threshold = 0.1f;
  p->surf_threshold = 0.1f;
  p->nearest_feature_search_distance = 5.f;
  p->mapping_frequency_divider = 5;
  p->fp_mode = 0;
  p->voxel_tie_order = 0;
}

void lego_params_hdl64(lego_params* p) {
  lego_params_vlp16(p);
  p->num_vertical_scans = 64;
  p->num_horizontal_scans = 2048;
  p->ground_scan_index = 55;
  p->vertical_angle_bottom = -24.8f;
  p->vertical_angle_top = 2.0f;
}

int lego_params_validate(const lego_params* p) {
  if (!p) return LEGO_EINVAL;
  if (p->fp_mode != 0 && p->fp_mode != 1) return LEGO_EINVAL;
  if (p->voxel_tie_order != 0 && p->voxel_tie_order != 1) return LEGO_EINVAL;
  if (p->num_vertical_scans < 2 || p->num_vertical_scans > 64) return LEGO_EINVAL;
  if (p->num_horizontal_scans < 16 || p->num_horizontal_scans > 2048) return LEGO_EINVAL;
  if (p->ground_scan_index < 0 || p->ground_scan_index >= p->num_vertical_scans) return LEGO_EINVAL;
  if (p->mapping_frequency_divider < 1) return LEGO_EINVAL;
  if (!(p->vertical_angle_top > p->vertical_angle_bottom)) return LEGO_EINVAL;
  return LEGO_OK;
}

int32_t lego_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int lego_batch_create(const lego_params* p, int32_t device, int32_t n_streams, int32_t max_points,
                      lego_batch** out) {
  if (!out) return LEGO_EINVAL;
  *out = nullptr;
  int rc = lego_params_validate(p);
  if (rc != LEGO_OK) return rc;
  if (n_streams < 1 || max_points < 1 || max_points > LEGO_MAX_POINTS) return LEGO_EINVAL;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return LEGO_EDEVICE;
  if (hipSetDevice(device) != hipSuccess) return LEGO_EDEVICE;
  lego_batch* b = new (std::nothrow) lego_batch();
  if (!b) return LEGO_ENOMEM;
  b->params = *p;
  b->P = derive(*p);
  int ncu = 0;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || ncu <= 0) ncu = 256;
  b->P.ncu = ncu;
  b->P.S = n_streams;
  b->S = n_streams;
  b->max_points = max_points;
  b->device = device;
  const LgParams& P = b->P;
  LgBufs& B = b->B;
  memset(&B, 0, sizeof(B));
  const size_t S = n_streams, VH = P.VH, V = P.V, H = P.H;
  std::vector<void*>& o = b->owned;
  b->P.max_points = max_points;
  b->wide_req = -1;
  b->P.wide = lg_wide_auto(P, n_streams);
  b->lag = lg_lag_auto(P, n_streams);
  const size_t tiles = (VH + 1023) / 1024;  // SW_TILE
  rc = LEGO_OK;
#define A(ptr, n) if (rc == LEGO_OK) rc = dalloc(&B.ptr, (n), o)
  A(range, S * VH); A(cloud, S * VH); A(ground, S * VH); A(label, S * VH);
  A(winner, S * VH); A(proj_mm, S * 2); A(colcnt, S * H); A(seg_tiles, S * tiles);
  A(cc_parent, S * VH); A(cc_cnt, S * VH); A(cc_mask, S * VH);
  A(scan_cand, S * H); A(orient, S * 4);
  A(seg_pts, S * VH); A(seg_range, S * VH); A(seg_col, S * VH); A(seg_ground, S * VH);
  A(ring_start, S * V); A(ring_end, S * V); A(outlier, S * VH); A(scan_msg, S * H); A(counts, S * CNT_N);
  A(curv, S * VH); A(picked, S * VH); A(flabel, S * VH); A(smooth, S * VH); A(xinfo, S * VH); A(fp_sync, S * 2); A(seg_fa, S * VH); A(outlier_fa, S * VH);
  A(r_sharp, S * V * P.cap_sharp); A(r_sharp_ind, S * V * P.cap_sharp);
  A(r_lsharp, S * V * P.cap_lsharp); A(r_lsharp_ind, S * V * P.cap_lsharp);
  A(r_flat, S * V * P.cap_flat); A(r_flat_ind, S * V * P.cap_flat);
  A(r_counts, S * V * 4); A(r_status, S * V);
  A(lf_stage, LG_SLOTS * S * V * H); A(lf_count, LG_SLOTS * S * V);
  A(r_lflat, LG_SLOTS * S * V * H); A(r_vcount, LG_SLOTS * S * V); A(r_vstatus, LG_SLOTS * S * V);
  A(f_sharp, LG_SLOTS * S * V * P.cap_sharp); A(f_sharp_ind, LG_SLOTS * S * V * P.cap_sharp);
  A(f_lsharp, LG_SLOTS * S * V * P.cap_lsharp); A(f_lsharp_ind, LG_SLOTS * S * V * P.cap_lsharp);
  A(f_flat, LG_SLOTS * S * V * P.cap_flat); A(f_flat_ind, LG_SLOTS * S * V * P.cap_flat); A(fcnt, LG_SLOTS * S * 4);
  A(f_lflat, S * VH);
  A(corner_last, S * 2 * V * P.cap_lsharp); A(surf_last, S * 2 * VH); A(grid_pts, S * VH);
  A(state, S); A(fe_state, S * 2);
  A(kd_node, S * 2 * VH); A(kd_vind, S * VH); A(kd_tmp, S * 2 * VH); A(kd_frames, S * 10 * VH);
#undef A
  if (rc != LEGO_OK) {
    delete b;
    return rc;
  }
  rc = lego_batch_reset(b);
  if (rc != LEGO_OK) {
    delete b;
    return rc;
  }
  *out = b;
  return LEGO_OK;
}

void lego_batch_destroy(lego_batch* b) { delete b; }

int lego_batch_reset(lego_batch* b) {
  if (!b) return LEGO_EINVAL;
  hipSetDevice(b->device);
  // no kernel of an unsynchronised step may still write the state cleared below (the memsets go on
  // the null stream, which is not ordered against non-blocking streams); pending work is dropped
  if (hipDeviceSynchronize() != hipSuccess) return LEGO_EDEVICE;
  const size_t S = b->S, VH = b->P.VH;
  LgBufs& B = b->B;
  // FeatureAssociation's vectors are value-initialised (fa.cpp:96-128); transforms zero (:135-138)
  if (hipMemset(B.curv, 0, S * VH * sizeof(float)) != hipSuccess) return LEGO_EDEVICE;
  if (hipMemset(B.picked, 0, S * VH) != hipSuccess) return LEGO_EDEVICE;
  if (hipMemset(B.flabel, 0, S * VH) != hipSuccess) return LEGO_EDEVICE;
  if (hipMemset(B.smooth, 0, S * VH * sizeof(int2)) != hipSuccess) return LEGO_EDEVICE;
  if (hipMemset(B.fp_sync, 0, S * 2 * sizeof(int32_t)) != hipSuccess) return LEGO_EDEVICE;
  b->epoch = 0;
  b->pend_pub = b->pend_lm = b->pend_lm_old = b->pend_ovl = false;
  b->par = b->last_par = 0;
  b->fe_ran = false;
  // the VoxelGrid's staged ring sizes and outputs: empty until a step stages them
  if (hipMemset(B.lf_count, 0, LG_SLOTS * S * b->P.V * sizeof(int32_t)) != hipSuccess) return LEGO_EDEVICE;
  if (hipMemset(B.r_vcount, 0, LG_SLOTS * S * b->P.V * sizeof(int32_t)) != hipSuccess) return LEGO_EDEVICE;
  if (hipMemset(B.state, 0, S * sizeof(LgState)) != hipSuccess) return LEGO_EDEVICE;
  if (hipMemset(B.fe_state, 0, S * 2 * sizeof(int32_t)) != hipSuccess) return LEGO_EDEVICE;
  if (hipMemset(B.counts, 0, S * CNT_N * sizeof(int32_t)) != hipSuccess) return LEGO_EDEVICE;
  // wide mode's per-scan scratch: winner image zeroed (no launch tag: every cell empty); first point
  // INT_MAX and last point -1 (every launch leaves them so)
  b->wepoch = 0;
  if (hipMemset(B.winner, 0, S * VH * sizeof(int32_t)) != hipSuccess) return LEGO_EDEVICE;
  if (hipMemset(B.colcnt, 0, S * b->P.H * sizeof(int32_t)) != hipSuccess) return LEGO_EDEVICE;
  {
    std::vector<int32_t> mm(2 * S);
    for (size_t s = 0; s < S; ++s) { mm[2 * s] = 0x7fffffff; mm[2 * s + 1] = -1; }
    if (hipMemcpy(B.proj_mm, mm.data(), mm.size() * sizeof(int32_t), hipMemcpyHostToDevice) != hipSuccess)
      return LEGO_EDEVICE;
  }
  if (hipDeviceSynchronize() != hipSuccess) return LEGO_EDEVICE;
  return LEGO_OK;
}

int lego_batch_set_timing(lego_batch* b, int32_t enabled) {
  if (!b) return LEGO_EINVAL;
  hipSetDevice(b->device);
  if (enabled && !b->events) {
    for (int i = 0; i < 8; ++i)
      if (hipEventCreate(&b->ev[i]) != hipSuccess) return LEGO_EDEVICE;
    b->events = true;
  }
  b->timing = enabled != 0;
  return LEGO_OK;
}

// The next wide projection launch's tag (LgParams.wtag, k_pw_scatter): a counter 1..15 in the top 4
// bits of the winner image's entries.  At the wrap the image is zeroed on `st`, before the launches
// that follow there (every earlier launch is ordered before them on `st`: chain_stream / joins).
static int next_wtag(lego_batch* b, hipStream_t st) {
  if (b->P.wide != 1) return LEGO_OK;
  if (++b->wepoch > 15) {
    b->wepoch = 1;
    if (hipMemsetAsync(b->B.winner, 0, (size_t)b->S * b->P.VH * sizeof(int32_t), st) != hipSuccess)
      return LEGO_EDEVICE;
  }
  b->P.wtag = (unsigned)b->wepoch << 28;
  return LEGO_OK;
}

// Streams [s0, s0 + n) of the batch.  Stage events are recorded only for the whole batch (timing).
static int run_projection(lego_batch* b, const float4* pts, const int64_t* offs, const int32_t* cnts, hipStream_t st,
                          int s0, int n) {
  LgParams P = b->P;
  P.s0 = s0;
  if (b->probe_cur) hipEventRecord(b->probe_cur[0], st);
  int rc = lg_launch_project(P, b->B, n, pts, offs, cnts, st);
  if (rc) return rc;
  if (b->probe_cur) hipEventRecord(b->probe_cur[1], st);
  if (b->timing) hipEventRecord(b->ev[1], st);
  rc = lg_launch_segment(P, b->B, n, st);
  if (rc) return rc;
  if (b->timing) hipEventRecord(b->ev[2], st);
  return LEGO_OK;
}

// k_publish of the slice [s0, s0 + n) for its scan of parity `par`, after that scan's k_voxel.
static int issue_publish(lego_batch* b, hipStream_t st, int g, int s0, int n, int par) {
  LgParams P = b->P;
  P.s0 = s0;
  P.par = par;
  if (hipStreamWaitEvent(st, b->ev_vox[g][par], 0) != hipSuccess) return LEGO_EDEVICE;
  return lg_launch_publish(P, b->B, n, st);
}

static int issue_lm(lego_batch* b, hipStream_t st, int s0, int n, int par) {
  LgParams P = b->P;
  P.s0 = s0;
  P.par = par;
  return lg_launch_lm(P, b->B, n, st);
}

// One slice [s0, s0 + n) of the streams through FeatureAssociation (slice g, on st), for the scan of
// parity b->par whose projection has run.  distort: the ProjectionOut came from the host
// (adjustDistortion / adjustOutlierCloud run in k_fa_prep instead of k_segment).  lag: as
// lego_batch::lag; the pending flags are read here and advanced by the caller (advance_pipeline).
static int run_association(lego_batch* b, hipStream_t st, int s0, int n, bool distort, int g, bool lag) {
  LgParams P = b->P;
  P.s0 = s0;
  P.epoch = b->epoch;
  P.par = b->par;
  int rc = lg_launch_fa_prep(P, b->B, n, st, distort);
  if (rc) return rc;
  if (b->timing) hipEventRecord(b->ev[3], st);
  rc = lg_launch_extract(P, b->B, n, st);
  if (rc) return rc;
  if (b->timing) hipEventRecord(b->ev[4], st);
  // a pending publish frees the staging half this scan's k_concat / k_voxel are about to fill
  if (b->pend_pub && (rc = issue_publish(b, st, g, s0, n, b->pub_par))) return rc;
  rc = lg_launch_concat(P, b->B, n, st);
  if (rc) return rc;
  if (hipEventRecord(b->ev_cat[g], st) != hipSuccess) return LEGO_EDEVICE;
  if (hipStreamWaitEvent(b->vs[g], b->ev_cat[g], 0) != hipSuccess) return LEGO_EDEVICE;
  rc = lg_launch_voxel(P, b->B, n, b->vs[g]);
  if (rc) return rc;
  if (hipEventRecord(b->ev_vox[g][P.par], b->vs[g]) != hipSuccess) return LEGO_EDEVICE;
  if (b->timing) hipEventRecord(b->ev[5], st);
  if (!lag) rc = issue_lm(b, st, s0, n, P.par);
  else if (b->pend_lm) rc = issue_lm(b, st, s0, n, b->lm_par);
  if (b->timing) hipEventRecord(b->ev[6], st);
  return rc;
}

// After every slice of a step ran run_association(lag): what is pending now.
static void advance_pipeline(lego_batch* b, bool lag, int groups) {
  if (lag) {
    b->pend_pub = b->pend_lm;  // the LM that ran leaves its publish
    b->pub_par = b->lm_par;
    b->pend_lm = true;
    b->lm_par = b->par;
  } else {
    b->pend_pub = true;
    b->pub_par = b->par;
    b->pend_lm = false;
  }
  b->pend_groups = groups;
  b->last_par = b->par;
  b->par = (b->par + 1) % LG_SLOTS;
}

// Internal side streams: non-blocking, default priority, every CU (lower priorities and CU masks for the
// VoxelGrid streams were measured and not kept).
static hipError_t make_side_stream(hipStream_t* st) { return hipStreamCreateWithFlags(st, hipStreamNonBlocking); }

static int ensure_streams(lego_batch* b, int groups) {
  if (!b->fork && hipEventCreateWithFlags(&b->fork, hipEventDisableTiming) != hipSuccess) return LEGO_EDEVICE;
  if (!b->ev_chain && hipEventCreateWithFlags(&b->ev_chain, hipEventDisableTiming) != hipSuccess) return LEGO_EDEVICE;
  for (int g = 0; g < groups; ++g) {
    if (!b->gs[g] && make_side_stream(&b->gs[g]) != hipSuccess) return LEGO_EDEVICE;
    if (!b->join[g] && hipEventCreateWithFlags(&b->join[g], hipEventDisableTiming) != hipSuccess) return LEGO_EDEVICE;
    if (!b->vs[g] && make_side_stream(&b->vs[g]) != hipSuccess) return LEGO_EDEVICE;
    if (!b->ev_cat[g] && hipEventCreateWithFlags(&b->ev_cat[g], hipEventDisableTiming) != hipSuccess)
      return LEGO_EDEVICE;
    for (int h = 0; h < LG_SLOTS; ++h)
      if (!b->ev_vox[g][h] && hipEventCreateWithFlags(&b->ev_vox[g][h], hipEventDisableTiming) != hipSuccess)
        return LEGO_EDEVICE;
  }
  return LEGO_OK;
}

// Work is about to be enqueued on st: if the last call enqueued on another stream, st first waits
// for all of it (the pending kernels issued on st read what those launches write).
static int chain_stream(lego_batch* b, hipStream_t st) {
  if (b->has_last && b->last_stream != st) {
    if (!b->ev_chain && hipEventCreateWithFlags(&b->ev_chain, hipEventDisableTiming) != hipSuccess)
      return LEGO_EDEVICE;
    if (hipEventRecord(b->ev_chain, b->last_stream) != hipSuccess) return LEGO_EDEVICE;
    if (hipStreamWaitEvent(st, b->ev_chain, 0) != hipSuccess) return LEGO_EDEVICE;
  }
  b->last_stream = st;
  b->has_last = true;
  return LEGO_OK;
}

static int ensure_ls(lego_batch* b) {
  if (!b->ls && make_side_stream(&b->ls) != hipSuccess) return LEGO_EDEVICE;
  if (!b->ev_pub && hipEventCreateWithFlags(&b->ev_pub, hipEventDisableTiming) != hipSuccess) return LEGO_EDEVICE;
  if (!b->ev_ls && hipEventCreateWithFlags(&b->ev_ls, hipEventDisableTiming) != hipSuccess) return LEGO_EDEVICE;
  if (!b->ev_fe && hipEventCreateWithFlags(&b->ev_fe, hipEventDisableTiming) != hipSuccess) return LEGO_EDEVICE;
  for (int h = 0; h < LG_SLOTS; ++h)
    if (!b->ev_cats[h] && hipEventCreateWithFlags(&b->ev_cats[h], hipEventDisableTiming) != hipSuccess)
      return LEGO_EDEVICE;
  return ensure_streams(b, 1);
}

// k_voxel of the scan in slot par on the VoxelGrid stream (alternating with gs[0] when alt), after that
// scan's k_concat and, when given, the event `after`.
static int launch_vox(lego_batch* b, int par, bool alt, hipEvent_t after) {
  LgParams P = b->P;
  P.s0 = 0;
  P.par = par;
  hipStream_t vst = (alt && b->vox_alt) ? b->gs[0] : b->vs[0];
  b->vox_alt ^= 1;
  if (hipStreamWaitEvent(vst, b->ev_cats[par], 0) != hipSuccess) return LEGO_EDEVICE;
  if (after && hipStreamWaitEvent(vst, after, 0) != hipSuccess) return LEGO_EDEVICE;
  int rc = lg_launch_voxel(P, b->B, b->S, vst);
  if (rc) return rc;
  if (hipEventRecord(b->ev_vox[0][par], vst) != hipSuccess) return LEGO_EDEVICE;
  return LEGO_OK;
}

// The front end of the overlap schedule after the projection: smoothness, extraction, then (after
// publish(k-2) on ls when one was issued) k_concat and the side stream's k_voxel.
static int run_association_ovl(lego_batch* b, hipStream_t st, bool wait_pub) {
  LgParams P = b->P;
  P.s0 = 0;
  P.epoch = b->epoch;
  P.par = b->par;
  if (b->probe_cur) hipEventRecord(b->probe_cur[2], st);
  int rc = lg_launch_fa_prep(P, b->B, b->S, st, false);
  if (b->probe_cur) hipEventRecord(b->probe_cur[3], st);
  if (!rc) rc = lg_launch_extract(P, b->B, b->S, st);
  if (rc) return rc;
  if (wait_pub && hipStreamWaitEvent(st, b->ev_pub, 0) != hipSuccess) return LEGO_EDEVICE;
  rc = lg_launch_concat(P, b->B, b->S, st);
  if (rc) return rc;
  if (hipEventRecord(b->ev_cats[P.par], st) != hipSuccess) return LEGO_EDEVICE;
  // Lag 2: every other scan's VoxelGrid on gs[0] (idle in this schedule), so k_voxel(k) may still run
  // while k_voxel(k + 1) starts; a stream of its own measured slower for both orders (212k vs 268k
  // scans/s with the stable order): one more stream than the 4 hardware queues.
  return launch_vox(b, P.par, b->lag >= 2, nullptr);
}

// Issue the pending k_publish / k_lm (each publish joined with its k_voxel) on the stream of the
// call that left them, in the pending work's slicing.
static int flush_pending(lego_batch* b) {
  if (!b->pend_pub && !b->pend_lm) return LEGO_OK;
  if (b->pend_ovl) {  // on ls: publish(k-1), [k_lm(k-1), publish(k-1),] k_lm(k), publish(k); then the
                      // last step's stream waits for ls
    int rc = LEGO_OK;
    if (b->pend_pub) rc = issue_publish(b, b->ls, 0, 0, b->S, b->pub_par);
    for (int q = 0; q < 2 && !rc; ++q) {
      const bool has = q == 0 ? b->pend_lm_old : b->pend_lm;
      const int lp = q == 0 ? b->lm_par_old : b->lm_par;
      if (!has) continue;
      if (hipStreamWaitEvent(b->ls, b->ev_cats[lp], 0) != hipSuccess) return LEGO_EDEVICE;
      rc = issue_lm(b, b->ls, 0, b->S, lp);
      if (!rc) rc = issue_publish(b, b->ls, 0, 0, b->S, lp);
    }
    if (rc) return rc;
    if (hipEventRecord(b->ev_ls, b->ls) != hipSuccess) return LEGO_EDEVICE;
    if (hipStreamWaitEvent(b->last_stream, b->ev_ls, 0) != hipSuccess) return LEGO_EDEVICE;
    b->pend_pub = b->pend_lm = b->pend_lm_old = b->pend_ovl = false;
    return LEGO_OK;
  }
  const int G = b->pend_groups;
  hipStream_t st = b->last_stream;
  for (int g = 0; g < G; ++g) {
    const int s0 = (int)((long long)b->S * g / G), s1 = (int)((long long)b->S * (g + 1) / G);
    int rc = LEGO_OK;
    if (b->pend_pub) rc = issue_publish(b, st, g, s0, s1 - s0, b->pub_par);
    if (!rc && b->pend_lm) rc = issue_lm(b, st, s0, s1 - s0, b->lm_par);
    if (!rc && b->pend_lm) rc = issue_publish(b, st, g, s0, s1 - s0, b->lm_par);
    if (rc) return rc;
  }
  b->pend_pub = b->pend_lm = false;
  return LEGO_OK;
}

// ---- checkpoint / resume of one stream's FeatureAssociation state (featureAssociation.h:70-115) ----------
// What one scan leaves for the next: LgState (transformCur / transformSum, systemInitedLM, isDegenerate, the
// cycle count, the Last clouds' half and sizes, the kd-trees' staleness, the odometry), the initialisation
// count of the front end (fe_state[1], adjustOutlierCloud's switch), both halves of the Last clouds, and the
// persistent curvature / picked / label / smoothness vectors whose stale entries the next scan reads (SURVEY
// App. B).  Everything else a step writes is rewritten by the next step.  k_extract's first-pass flag
// (fp_sync) is reset by a load: it is compared with the loading batch's own launch epochs.
struct LgCkptHdr {
  uint32_t magic, version;
  int32_t V, H, cap_lsharp, state_bytes;
};
static const uint32_t kCkptMagic = 0x4b43474cu;  // "LGCK"
static size_t ckpt_bytes(const LgParams& P) {
  const size_t VH = P.VH, cl = (size_t)P.V * P.cap_lsharp;
  return sizeof(LgCkptHdr) + sizeof(LgState) + sizeof(int32_t) + 2 * cl * sizeof(float4) + 2 * VH * sizeof(float4) +
         VH * (sizeof(float) + 1 + 1 + sizeof(int2));
}

int lego_batch_state_size(const lego_batch* b, size_t* bytes) {
  if (!b || !bytes) return LEGO_EINVAL;
  *bytes = ckpt_bytes(b->P);
  return LEGO_OK;
}

// The stream's pieces in checkpoint order: (device pointer, bytes).
static void ckpt_pieces(lego_batch* b, int s, std::vector<std::pair<void*, size_t>>& out) {
  const LgParams& P = b->P;
  const LgBufs& B = b->B;
  const size_t VH = P.VH, cl = (size_t)P.V * P.cap_lsharp;
  out.clear();
  out.push_back({B.state + s, sizeof(LgState)});
  out.push_back({B.fe_state + 2 * (size_t)s + 1, sizeof(int32_t)});
  out.push_back({B.corner_last + (size_t)s * 2 * cl, 2 * cl * sizeof(float4)});
  out.push_back({B.surf_last + (size_t)s * 2 * VH, 2 * VH * sizeof(float4)});
  out.push_back({B.curv + (size_t)s * VH, VH * sizeof(float)});
  out.push_back({B.picked + (size_t)s * VH, VH});
  out.push_back({B.flabel + (size_t)s * VH, VH});
  out.push_back({B.smooth + (size_t)s * VH, VH * sizeof(int2)});
}

int lego_batch_save_state(lego_batch* b, int32_t s, void* host, size_t bytes) {
  if (!b || !host || s < 0 || s >= b->S || bytes < ckpt_bytes(b->P)) return LEGO_EINVAL;
  if (hipSetDevice(b->device) != hipSuccess) return LEGO_EDEVICE;
  int rc = flush_pending(b);  // the stream's last scan published (its Last clouds, LgState)
  if (rc) return rc;
  if (hipDeviceSynchronize() != hipSuccess) return LEGO_EDEVICE;
  LgCkptHdr h{kCkptMagic, 1u, b->P.V, b->P.H, b->P.cap_lsharp, (int32_t)sizeof(LgState)};
  char* o = (char*)host;
  memcpy(o, &h, sizeof(h));
  o += sizeof(h);
  std::vector<std::pair<void*, size_t>> pc;
  ckpt_pieces(b, s, pc);
  for (auto& q : pc) {
    if (hipMemcpy(o, q.first, q.second, hipMemcpyDeviceToHost) != hipSuccess) return LEGO_EDEVICE;
    o += q.second;
  }
  return LEGO_OK;
}

int lego_batch_load_state(lego_batch* b, int32_t s, const void* host, size_t bytes) {
  if (!b || !host || s < 0 || s >= b->S || bytes < ckpt_bytes(b->P)) return LEGO_EINVAL;
  LgCkptHdr h;
  memcpy(&h, host, sizeof(h));
  if (h.magic != kCkptMagic || h.version != 1u || h.V != b->P.V || h.H != b->P.H || h.cap_lsharp != b->P.cap_lsharp ||
      h.state_bytes != (int32_t)sizeof(LgState))
    return LEGO_EINVAL;  // another sensor layout or library version
  if (hipSetDevice(b->device) != hipSuccess) return LEGO_EDEVICE;
  int rc = flush_pending(b);  // no kernel of this batch may still write the stream
  if (rc) return rc;
  if (hipDeviceSynchronize() != hipSuccess) return LEGO_EDEVICE;
  const char* o = (const char*)host + sizeof(h);
  std::vector<std::pair<void*, size_t>> pc;
  ckpt_pieces(b, s, pc);
  for (auto& q : pc) {
    if (hipMemcpy(q.first, o, q.second, hipMemcpyHostToDevice) != hipSuccess) return LEGO_EDEVICE;
    o += q.second;
  }
  if (hipMemset(b->B.fp_sync + 2 * (size_t)s, 0, 2 * sizeof(int32_t)) != hipSuccess) return LEGO_EDEVICE;
  if (hipDeviceSynchronize() != hipSuccess) return LEGO_EDEVICE;
  return LEGO_OK;
}

int lego_ctx_state_size(const lego_ctx* c, size_t* bytes) { return c ? lego_batch_state_size(c->b, bytes) : LEGO_EINVAL; }
int lego_ctx_save_state(lego_ctx* c, void* host, size_t bytes) {
  return c ? lego_batch_save_state(c->b, 0, host, bytes) : LEGO_EINVAL;
}
int lego_ctx_load_state(lego_ctx* c, const void* host, size_t bytes) {
  return c ? lego_batch_load_state(c->b, 0, host, bytes) : LEGO_EINVAL;
}

int lego_batch_set_groups(lego_batch* b, int32_t groups) {
  if (!b || groups < 1 || groups > LEGO_MAX_GROUPS) return LEGO_EINVAL;
  if (hipSetDevice(b->device) != hipSuccess) return LEGO_EDEVICE;
  groups = groups > b->S ? b->S : groups;
  int rc = flush_pending(b);  // the pending work belongs to the old slicing
  if (rc) return rc;
  rc = ensure_streams(b, groups);
  if (rc) return rc;
  b->groups = groups;
  return LEGO_OK;
}

int lego_batch_set_lag(lego_batch* b, int32_t lag) {
  if (!b || lag < -1 || lag > 2) return LEGO_EINVAL;
  if (hipSetDevice(b->device) != hipSuccess) return LEGO_EDEVICE;
  int rc = flush_pending(b);  // the pending work belongs to the old schedule
  if (rc) return rc;
  b->lag_req = lag;
  b->lag = lag < 0 ? lg_lag_auto(b->P, b->S) : lag;
  return LEGO_OK;
}

// The depth lego_batch_step runs: lag 2 runs as 1 when the streams are sliced (groups > 1) or timing is on.
int lego_batch_lag(const lego_batch* b) {
  if (!b) return LEGO_EINVAL;
  return (b->lag >= 2 && (b->groups > 1 || b->timing)) ? 1 : b->lag;
}

int lego_batch_set_wide(lego_batch* b, int32_t mode) {
  if (!b || mode < -1 || mode > 2) return LEGO_EINVAL;
  if (mode == 0 && (!lg_lds_projection(b->P) || !lg_lds_segment(b->P))) return LEGO_EINVAL;
  if (mode == 2 && !lg_lds_projection(b->P)) return LEGO_EINVAL;
  // both layouts keep the persistent state alike and leave their scratch reset: switchable at any step
  b->wide_req = mode;
  b->P.wide = mode < 0 ? lg_wide_auto(b->P, b->S) : mode;
  return LEGO_OK;
}

int lego_batch_wide(const lego_batch* b) { return b ? b->P.wide : LEGO_EINVAL; }

int lego_batch_step(lego_batch* b, const lego_point* d_points, const int64_t* d_offsets, const int32_t* d_counts,
                    void* hip_stream) {
  if (!b || !d_points || !d_offsets || !d_counts) return LEGO_EINVAL;
  if (hipSetDevice(b->device) != hipSuccess) return LEGO_EDEVICE;
  hipStream_t st = (hipStream_t)hip_stream;
  b->probe_cur = nullptr;  // set again below for an overlap-schedule step while the probe is on
  b->epoch = b->epoch == 0x7fffffff ? 1 : b->epoch + 1;
  const bool lag = b->lag != 0;
  // timing: per-stage events on the caller's stream, one slice (the pipelined path itself)
  const int G = b->timing ? 1 : b->groups;
  int rc = ensure_streams(b, G);
  if (rc) return rc;
  if ((b->pend_pub || b->pend_lm) && b->pend_groups != G) {
    rc = flush_pending(b);
    if (rc) return rc;
  }
  rc = chain_stream(b, st);
  if (!rc) rc = next_wtag(b, st);
  if (rc) return rc;
  const bool ovl = G <= 1 && lag && !b->timing;
  if (ovl != b->pend_ovl && (b->pend_pub || b->pend_lm)) {  // the pending work belongs to the other schedule
    rc = flush_pending(b);
    if (rc) return rc;
  }
  if (ovl) {
    rc = ensure_ls(b);
    if (rc) return rc;
    if (b->probe) {  // four events of this step (lego_batch_probe_times), a ring of LG_PROBE_MAX steps
      const int slot = b->probe_n % LG_PROBE_MAX;
      while ((int)b->pev.size() < 4 * (slot + 1)) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return LEGO_EDEVICE;
        b->pev.push_back(e);
      }
      b->probe_cur = &b->pev[4 * slot];
      ++b->probe_n;
    }
    const bool pub_now = b->pend_pub;
    // With the stable VoxelGrid order, k_lm(k-1) starts after this scan's projection and segmentation:
    // those whole-CU kernels (k_project 124 KB, k_segment_lds 115 KB of LDS) then get the CUs first
    // instead of waiting for each CU's k_lm workgroup to retire, and k_lm overlaps the rest of the front
    // end (small workgroups) and the VoxelGrid.  k_publish(k-2) stays at the top of the step.  C3:
    // 248-250k -> 265k scans/s.  With the reference's introsort order the heavier k_voxel(k) then
    // meets k_lm(k-1) head-on (193k -> 167-177k scans/s), so that order keeps k_lm at the top too
    // (where the measured variants are listed).
    // With more scans than CUs the reference order takes it too (S = 1024: 239k vs 226k scans/s; at S = 256
    // 188k vs 195k with lag 1, so not there), and so does lag 2 (k_lm(k-2)'s inputs are ready long before:
    // 214.6k vs 210.8k; round 4, profiles/r04_schedule_ab.txt).
    const bool lm_after_fe = b->P.voxel_stable || b->S > b->P.ncu || b->lag >= 2;
    if (b->pend_pub) {  // publish(k-2) on ls, after its k_voxel (issue_publish waits for ev_vox)
      rc = issue_publish(b, b->ls, 0, 0, b->S, b->pub_par);
      if (!rc && hipEventRecord(b->ev_pub, b->ls) != hipSuccess) rc = LEGO_EDEVICE;
      if (rc) return rc;
    }
    if (lm_after_fe) {
      rc = run_projection(b, (const float4*)d_points, d_offsets, d_counts, st, 0, b->S);
      if (!rc && hipEventRecord(b->ev_fe, st) != hipSuccess) rc = LEGO_EDEVICE;
      if (!rc && hipStreamWaitEvent(b->ls, b->ev_fe, 0) != hipSuccess) rc = LEGO_EDEVICE;
      if (rc) return rc;
    }
    // the LM issued now: lag 1, k_lm(k-1) (the newest pending); lag 2, k_lm(k-2) (the older one)
    const bool deep = b->lag >= 2;
    const bool lm_now = deep ? b->pend_lm_old : b->pend_lm;
    const int lm_slot = deep ? b->lm_par_old : b->lm_par;
    if (lm_now) {  // on ls, after that scan's k_concat
      if (hipStreamWaitEvent(b->ls, b->ev_cats[lm_slot], 0) != hipSuccess) rc = LEGO_EDEVICE;
      if (!rc) rc = issue_lm(b, b->ls, 0, b->S, lm_slot);
    }
    if (!rc && !lm_after_fe) rc = run_projection(b, (const float4*)d_points, d_offsets, d_counts, st, 0, b->S);
    if (!rc) rc = run_association_ovl(b, st, pub_now);
    b->probe_cur = nullptr;
    if (rc) return rc;
    // pending now: the publish of the LM just issued, then (lag 2) k_lm(k-1), and k_lm(k)
    b->pend_pub = lm_now;
    b->pub_par = lm_slot;
    if (deep) {
      b->pend_lm_old = b->pend_lm;
      b->lm_par_old = b->lm_par;
    }
    b->pend_lm = true;
    b->lm_par = b->par;
    b->pend_groups = 1;
    b->pend_ovl = true;
    b->last_par = b->par;
    b->par = (b->par + 1) % LG_SLOTS;
    b->fe_ran = true;
    return LEGO_OK;
  }
  if (G <= 1) {
    if (b->timing) hipEventRecord(b->ev[0], st);
    rc = run_projection(b, (const float4*)d_points, d_offsets, d_counts, st, 0, b->S);
    if (!rc) rc = run_association(b, st, 0, b->S, false, 0, lag);
  } else {
    if (hipEventRecord(b->fork, st) != hipSuccess) return LEGO_EDEVICE;
    for (int g = 0; g < G && !rc; ++g) {
      const int s0 = (int)((long long)b->S * g / G), s1 = (int)((long long)b->S * (g + 1) / G);
      if (hipStreamWaitEvent(b->gs[g], b->fork, 0) != hipSuccess) return LEGO_EDEVICE;
      rc = run_projection(b, (const float4*)d_points, d_offsets, d_counts, b->gs[g], s0, s1 - s0);
      if (!rc) rc = run_association(b, b->gs[g], s0, s1 - s0, false, g, lag);
      if (rc) break;
      if (hipEventRecord(b->join[g], b->gs[g]) != hipSuccess) return LEGO_EDEVICE;
      if (hipStreamWaitEvent(st, b->join[g], 0) != hipSuccess) return LEGO_EDEVICE;
    }
  }
  if (rc) return rc;
  advance_pipeline(b, lag, G);
  b->fe_ran = true;
  return LEGO_OK;
}

int lego_batch_set_trajectory(lego_batch* b, float* d_traj, int32_t max_scans) {
  if (!b || max_scans < 0 || (max_scans > 0 && !d_traj)) return LEGO_EINVAL;
  if (hipSetDevice(b->device) != hipSuccess) return LEGO_EDEVICE;
  int rc = flush_pending(b);  // pending LMs record where the caller asked when it issued them
  if (rc) return rc;
  b->B.traj = max_scans > 0 ? d_traj : nullptr;
  b->P.traj_cap = max_scans > 0 ? max_scans : 0;
  return LEGO_OK;
}

int lego_batch_set_probe(lego_batch* b, int32_t enabled) {
  if (!b) return LEGO_EINVAL;
  b->probe = enabled != 0;
  b->probe_n = 0;
  return LEGO_OK;
}

int lego_batch_probe_times(lego_batch* b, float* ms2, int32_t* steps) {
  if (!b || !ms2 || !steps) return LEGO_EINVAL;
  hipSetDevice(b->device);
  double a = 0.0, f = 0.0;
  const int n = b->probe_n < LG_PROBE_MAX ? b->probe_n : LG_PROBE_MAX;  // the ring's last n steps
  for (int k = 0; k < n; ++k) {
    hipEvent_t* e = &b->pev[4 * k];
    float x = 0.f, y = 0.f;
    if (hipEventSynchronize(e[3]) != hipSuccess || hipEventElapsedTime(&x, e[0], e[1]) != hipSuccess ||
        hipEventElapsedTime(&y, e[2], e[3]) != hipSuccess)
      return LEGO_EDEVICE;
    a += x;
    f += y;
  }
  *steps = n;
  ms2[0] = n ? (float)(a / n) : 0.f;
  ms2[1] = n ? (float)(f / n) : 0.f;
  b->probe_n = 0;
  return LEGO_OK;
}

int lego_batch_flush(lego_batch* b) {
  if (!b) return LEGO_EINVAL;
  if (hipSetDevice(b->device) != hipSuccess) return LEGO_EDEVICE;
  return flush_pending(b);
}

int lego_batch_sync(lego_batch* b) {
  if (!b) return LEGO_EINVAL;
  hipSetDevice(b->device);
  int rc = flush_pending(b);
  if (rc) return rc;
  return hipDeviceSynchronize() == hipSuccess ? LEGO_OK : LEGO_EDEVICE;
}

int lego_batch_stage_times(lego_batch* b, float* ms6) {
  if (!b || !ms6 || !b->timing) return LEGO_EINVAL;
  hipSetDevice(b->device);
  if (hipEventSynchronize(b->ev[6]) != hipSuccess) return LEGO_EDEVICE;
  for (int i = 0; i < 6; ++i) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, b->ev[i], b->ev[i + 1]) != hipSuccess) return LEGO_EDEVICE;
    ms6[i] = ms;
  }
  return LEGO_OK;
}

// The HBM-bound pair of stages (projection, then calculateSmoothness / markOccludedPoints) launched
// `reps` times back to back on the caller's stream between two events, on the inputs of the batch's
// last step: the mean duration of one pair without the per-stage event gaps.  With a second input
// set (another step's offsets / counts into the same point array) the projections alternate between
// the two, ending on the step's own, so no launch re-reads the input its predecessor just read.  Both stages are
// idempotent on those inputs (k_project rewrites the same images from the same points; k_fa_prep
// reads only k_segment's output), so the batch's results are unchanged.
int lego_batch_time_hbm_stages(lego_batch* b, int32_t reps, const lego_point* d_points, const int64_t* d_offsets,
                               const int32_t* d_counts, const int64_t* d_offsets_alt, const int32_t* d_counts_alt,
                               void* hip_stream, float* ms_pair) {
  if (!b || reps < 1 || !d_points || !d_offsets || !d_counts || !ms_pair) return LEGO_EINVAL;
  if (hipSetDevice(b->device) != hipSuccess) return LEGO_EDEVICE;
  hipStream_t st = (hipStream_t)hip_stream;
  int rc = flush_pending(b);
  if (rc) return rc;
  if (hipDeviceSynchronize() != hipSuccess) return LEGO_EDEVICE;  // nothing else on the device
  hipEvent_t e0, e1;
  if (hipEventCreate(&e0) != hipSuccess) return LEGO_EDEVICE;
  if (hipEventCreate(&e1) != hipSuccess) {
    hipEventDestroy(e0);
    return LEGO_EDEVICE;
  }
  LgParams P = b->P;
  P.s0 = 0;
  P.epoch = b->epoch;
  P.par = b->par;
  if (hipEventRecord(e0, st) != hipSuccess) rc = LEGO_EDEVICE;
  for (int r = 0; r < reps && !rc; ++r) {
    const bool alt = d_offsets_alt && d_counts_alt && ((reps - 1 - r) & 1);  // the last launch: the step's own
    rc = next_wtag(b, st);
    if (rc) break;
    P.wtag = b->P.wtag;
    rc = lg_launch_project(P, b->B, b->S, (const float4*)d_points, alt ? d_offsets_alt : d_offsets,
                           alt ? d_counts_alt : d_counts, st);
    if (!rc) rc = lg_launch_fa_prep(P, b->B, b->S, st, false);
  }
  if (!rc && hipEventRecord(e1, st) != hipSuccess) rc = LEGO_EDEVICE;
  float ms = 0.f;
  if (!rc && hipEventSynchronize(e1) != hipSuccess) rc = LEGO_EDEVICE;
  if (!rc && hipEventElapsedTime(&ms, e0, e1) != hipSuccess) rc = LEGO_EDEVICE;
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  if (!rc) *ms_pair = ms / reps;
  return rc;
}

int lego_batch_time_voxel(lego_batch* b, int32_t reps, void* hip_stream, float* ms) {
  if (!b || reps < 1 || !ms || !b->fe_ran) return LEGO_EINVAL;  // no step has staged the VoxelGrid's input
  if (hipSetDevice(b->device) != hipSuccess) return LEGO_EDEVICE;
  hipStream_t st = (hipStream_t)hip_stream;
  int rc = flush_pending(b);
  if (rc) return rc;
  if (hipDeviceSynchronize() != hipSuccess) return LEGO_EDEVICE;  // nothing else on the device
  hipEvent_t e0, e1;
  if (hipEventCreate(&e0) != hipSuccess) return LEGO_EDEVICE;
  if (hipEventCreate(&e1) != hipSuccess) {
    hipEventDestroy(e0);
    return LEGO_EDEVICE;
  }
  LgParams P = b->P;
  P.s0 = 0;
  P.par = b->last_par;  // the last step's staged lessFlat clouds and VoxelGrid output
  if (hipEventRecord(e0, st) != hipSuccess) rc = LEGO_EDEVICE;
  for (int r = 0; r < reps && !rc; ++r) rc = lg_launch_voxel(P, b->B, b->S, st);
  if (!rc && hipEventRecord(e1, st) != hipSuccess) rc = LEGO_EDEVICE;
  float t = 0.f;
  if (!rc && hipEventSynchronize(e1) != hipSuccess) rc = LEGO_EDEVICE;
  if (!rc && hipEventElapsedTime(&t, e0, e1) != hipSuccess) rc = LEGO_EDEVICE;
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  if (!rc) *ms = t / reps;
  return rc;
}

// publishOdometry's orientation (featureAssociation.cpp:1287-1294): tf::createQuaternionMsgFromRollPitchYaw(
// transformSum[2], -transformSum[0], -transformSum[1]) in double, then (-y, -z, x, w).  Computed here, on the
// host with glibc's sin / cos (the reference's own), when the odometry is read back.
static void odom_quat(const float* sum, double* q4) {
  const double roll = sum[2], pitch = -(double)sum[0], yaw = -(double)sum[1];
  const double hy = yaw * 0.5, hp = pitch * 0.5, hr = roll * 0.5;
  const double cyw = cos(hy), syw = sin(hy), cp = cos(hp), sp = sin(hp), cr = cos(hr), sr = sin(hr);
  const double qx = sr * cp * cyw - cr * sp * syw;
  const double qy = cr * sp * cyw + sr * cp * syw;
  const double qz = cr * cp * syw - sr * sp * cyw;
  const double qw = cr * cp * cyw + sr * sp * syw;
  q4[0] = -qy; q4[1] = -qz; q4[2] = qx; q4[3] = qw;
}

// Header of stream s (counts, orientation, state) into pinned memory, on st, then wait for it.
struct ReadHdr {
  int32_t cnt[CNT_N];
  float ori[4];
  int32_t fe[2];  // proj_status, front-end scans
  LgState S;
};
static int read_hdr(lego_batch* b, int s, hipStream_t st, ReadHdr** out) {
  const LgBufs& B = b->B;
  ReadHdr* h = b->h_hdr.get<ReadHdr>(1);
  if (!h) return LEGO_ENOMEM;
  if (hipMemcpyAsync(h->cnt, B.counts + (size_t)s * CNT_N, sizeof(h->cnt), hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipMemcpyAsync(h->ori, B.orient + (size_t)s * 4, sizeof(h->ori), hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipMemcpyAsync(&h->S, B.state + s, sizeof(h->S), hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipMemcpyAsync(h->fe, B.fe_state + (size_t)s * 2, sizeof(h->fe), hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return LEGO_EDEVICE;
  *out = h;
  return LEGO_OK;
}

// ProjectionOut of stream s: every array copy issued on st, one wait (h = read_hdr's header)
static int read_proj(lego_batch* b, int s, const ReadHdr* h, hipStream_t st, lego_projection_out* o) {
  const LgParams& P = b->P;
  const LgBufs& B = b->B;
  const size_t VH = P.VH;
  const int M = h->cnt[CNT_M];
  int rc = LEGO_OK;
  lego_point *seg, *outl, *scan;
  int32_t *rs, *re, *label;
  uint8_t* gflag;
  uint32_t* col;
  float *range_seg, *range;
  int8_t* ground;
  rc |= d2h(b->h_seg, (const lego_point*)(B.seg_pts + s * VH), M, st, &seg);
  rc |= d2h(b->h_out, (const lego_point*)(B.outlier + s * VH), h->cnt[CNT_OUTLIER], st, &outl);
  rc |= d2h(b->h_scan, (const lego_point*)(B.scan_msg + (size_t)s * P.H), h->cnt[CNT_SCAN], st, &scan);
  rc |= d2h(b->h_rs, B.ring_start + (size_t)s * P.V, P.V, st, &rs);
  rc |= d2h(b->h_re, B.ring_end + (size_t)s * P.V, P.V, st, &re);
  rc |= d2h(b->h_gflag, B.seg_ground + s * VH, M, st, &gflag);
  rc |= d2h(b->h_col, B.seg_col + s * VH, M, st, &col);
  rc |= d2h(b->h_range_seg, B.seg_range + s * VH, M, st, &range_seg);
  rc |= d2h(b->h_label, B.label + s * VH, VH, st, &label);
  rc |= d2h(b->h_ground, B.ground + s * VH, VH, st, &ground);
  rc |= d2h(b->h_range, B.range + s * VH, VH, st, &range);
  if (rc) return LEGO_EDEVICE;
  if (hipStreamSynchronize(st) != hipSuccess) return LEGO_EDEVICE;
  o->n_segmented = M;
  o->n_outlier = h->cnt[CNT_OUTLIER];
  o->n_scan = h->cnt[CNT_SCAN];
  o->segmented_cloud = seg;
  o->outlier_cloud = outl;
  o->scan_msg = scan;
  o->start_ring_index = rs;
  o->end_ring_index = re;
  o->start_orientation = h->ori[0];
  o->end_orientation = h->ori[1];
  o->orientation_diff = h->ori[2];
  o->segmented_cloud_ground_flag = gflag;
  o->segmented_cloud_col_ind = col;
  o->segmented_cloud_range = range_seg;
  o->label_mat = label;
  o->ground_mat = ground;
  o->range_mat = range;
  return LEGO_OK;
}

// AssociationOut of stream s (as read_proj)
static int read_assoc(lego_batch* b, int s, const ReadHdr* h, hipStream_t st, lego_association_out* o) {
  const LgParams& P = b->P;
  const LgBufs& B = b->B;
  const size_t VH = P.VH, V = P.V;
  const int32_t* cnt = h->cnt;
  const LgState& S = h->S;
  int rc = LEGO_OK;
  lego_point *sharp, *lsharp, *flat, *lflat, *clast, *slast, *olast;
  int32_t *sharp_ind, *lsharp_ind, *flat_ind;
  const size_t hs = (size_t)b->last_par * b->S + s;  // the feature half of the last scan
  rc |= d2h(b->h_sharp, (const lego_point*)(B.f_sharp + hs * V * P.cap_sharp), cnt[CNT_SHARP], st, &sharp);
  rc |= d2h(b->h_sharp_ind, B.f_sharp_ind + hs * V * P.cap_sharp, cnt[CNT_SHARP], st, &sharp_ind);
  rc |= d2h(b->h_lsharp, (const lego_point*)(B.f_lsharp + hs * V * P.cap_lsharp), cnt[CNT_LSHARP], st, &lsharp);
  rc |= d2h(b->h_lsharp_ind, B.f_lsharp_ind + hs * V * P.cap_lsharp, cnt[CNT_LSHARP], st, &lsharp_ind);
  rc |= d2h(b->h_flat, (const lego_point*)(B.f_flat + hs * V * P.cap_flat), cnt[CNT_FLAT], st, &flat);
  rc |= d2h(b->h_flat_ind, B.f_flat_ind + hs * V * P.cap_flat, cnt[CNT_FLAT], st, &flat_ind);
  rc |= d2h(b->h_lflat, (const lego_point*)(B.f_lflat + s * VH), cnt[CNT_LFLAT], st, &lflat);
  const size_t cls = V * P.cap_lsharp;
  rc |= d2h(b->h_clast, (const lego_point*)(B.corner_last + (size_t)s * 2 * cls + (size_t)S.last_buf * cls),
            S.n_corner_last, st, &clast);
  rc |= d2h(b->h_slast, (const lego_point*)(B.surf_last + (size_t)s * 2 * VH + (size_t)S.last_buf * VH),
            S.n_surf_last, st, &slast);
  rc |= d2h(b->h_olast, (const lego_point*)(B.outlier_fa + s * VH), cnt[CNT_OUTLIER], st, &olast);
  if (rc) return LEGO_EDEVICE;
  if (hipStreamSynchronize(st) != hipSuccess) return LEGO_EDEVICE;
  o->status = S.status;
  o->n_sharp = cnt[CNT_SHARP];
  o->n_less_sharp = cnt[CNT_LSHARP];
  o->n_flat = cnt[CNT_FLAT];
  o->n_less_flat = cnt[CNT_LFLAT];
  o->corner_points_sharp = sharp;
  o->corner_points_less_sharp = lsharp;
  o->surf_points_flat = flat;
  o->surf_points_less_flat = lflat;
  o->sharp_ind = sharp_ind;
  o->less_sharp_ind = lsharp_ind;
  o->flat_ind = flat_ind;
  for (int i = 0; i < 6; ++i) {
    o->transform_cur[i] = S.cur[i];
    o->transform_sum[i] = S.sum[i];
  }
  odom_quat(S.sum, o->odom_orientation);
  for (int i = 0; i < 3; ++i) o->odom_position[i] = S.pos[i];
  o->lm_iter_surf = S.iters_surf;
  o->lm_iter_corner = S.iters_corner;
  o->n_corner_last = S.n_corner_last;
  o->n_surf_last = S.n_surf_last;
  o->n_outlier_last = cnt[CNT_OUTLIER];
  o->cloud_corner_last = clast;
  o->cloud_surf_last = slast;
  o->cloud_outlier_last = olast;
  return LEGO_OK;
}

int lego_batch_read(lego_batch* b, int32_t s, lego_projection_out* proj, lego_association_out* assoc) {
  if (!b || s < 0 || s >= b->S) return LEGO_EINVAL;
  hipSetDevice(b->device);
  if (flush_pending(b) != LEGO_OK) return LEGO_EDEVICE;
  if (hipDeviceSynchronize() != hipSuccess) return LEGO_EDEVICE;
  ReadHdr* h = nullptr;
  int rc = read_hdr(b, s, nullptr, &h);
  if (!rc && proj) rc = read_proj(b, s, h, nullptr, proj);
  if (!rc && assoc) rc = read_assoc(b, s, h, nullptr, assoc);
  return rc;
}

int lego_batch_read_poses(lego_batch* b, float* out, int32_t* status) {
  if (!b) return LEGO_EINVAL;
  hipSetDevice(b->device);
  if (flush_pending(b) != LEGO_OK) return LEGO_EDEVICE;
  if (hipDeviceSynchronize() != hipSuccess) return LEGO_EDEVICE;
  std::vector<LgState> S(b->S);
  if (hipMemcpy(S.data(), b->B.state, S.size() * sizeof(LgState), hipMemcpyDeviceToHost) != hipSuccess)
    return LEGO_EDEVICE;
  for (int s = 0; s < b->S; ++s) {
    if (out)
      for (int k = 0; k < 6; ++k) {
        out[s * 12 + k] = S[s].cur[k];
        out[s * 12 + 6 + k] = S[s].sum[k];
      }
    if (status) status[s] = S[s].status;
  }
  return LEGO_OK;
}

int lego_batch_read_counts(lego_batch* b, int32_t* out) {
  if (!b || !out) return LEGO_EINVAL;
  hipSetDevice(b->device);
  if (flush_pending(b) != LEGO_OK) return LEGO_EDEVICE;
  if (hipDeviceSynchronize() != hipSuccess) return LEGO_EDEVICE;
  std::vector<int32_t> c((size_t)b->S * CNT_N);
  if (hipMemcpy(c.data(), b->B.counts, c.size() * sizeof(int32_t), hipMemcpyDeviceToHost) != hipSuccess)
    return LEGO_EDEVICE;
  for (int s = 0; s < b->S; ++s) {
    const int32_t* k = &c[(size_t)s * CNT_N];
    int32_t* o = out + (size_t)s * 7;
    o[0] = k[CNT_M]; o[1] = k[CNT_OUTLIER]; o[2] = k[CNT_SCAN]; o[3] = k[CNT_SHARP];
    o[4] = k[CNT_LSHARP]; o[5] = k[CNT_FLAT]; o[6] = k[CNT_LFLAT];
  }
  return LEGO_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------------------------
// single-context readback: one kernel copies every output array of the call (sizes read on the
// device) straight into mapped pinned host memory, then one wait.  It replaces a header read (four
// copies and a wait) and a copy per array (each a runtime blit launch, ~5-20 us apart on the
// timeline of one scan).
// ---------------------------------------------------------------------------------------------
namespace {
struct PackDesc {
  const char* src;       // device array
  const int32_t* sel;    // nullable: src += *sel * sel_stride (the Last double buffer)
  long long sel_stride;
  char* dst;             // device view of the mapped host region
  const int32_t* cnt;    // nullable: element count read on the device, capped at `fixed`
  int32_t fixed;         // element count (or the cap of *cnt)
  int32_t elem;          // bytes per element
};
#define PACK_MAX 16
struct PackArgs {
  PackDesc d[PACK_MAX];
};

__global__ __launch_bounds__(256) void k_pack(PackArgs a) {
  const PackDesc& d = a.d[blockIdx.y];
  const long long n = d.cnt ? min(max(*d.cnt, 0), d.fixed) : d.fixed;
  const char* src = d.src + (d.sel ? (long long)*d.sel * d.sel_stride : 0ll);
  const size_t bytes = (size_t)n * d.elem;
  const size_t stride = (size_t)gridDim.x * blockDim.x, t0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool vec = ((((uintptr_t)src) | ((uintptr_t)d.dst)) & 15) == 0;
  const size_t nv = vec ? bytes / 16 : 0;
  for (size_t i = t0; i < nv; i += stride) ((uint4*)d.dst)[i] = ((const uint4*)src)[i];
  for (size_t i = nv * 16 + t0; i < bytes; i += stride) d.dst[i] = src[i];
}

// Region offsets of a pack buffer (each region 256-byte aligned; sizes at capacity)
struct PackLayout {
  size_t off[PACK_MAX];
  size_t total;
};
PackLayout make_layout(const size_t* bytes, int n) {
  PackLayout L{};
  size_t o = 0;
  for (int i = 0; i < n; ++i) {
    L.off[i] = o;
    o += (bytes[i] + 255) & ~(size_t)255;
  }
  L.total = o;
  return L;
}
// proj: 0 header, 1 segmented, 2 outlier, 3 scan, 4 ring start, 5 ring end, 6 ground flag, 7 col,
// 8 range (segmented), 9 label, 10 ground, 11 range image
constexpr int PJ_N = 12;
PackLayout proj_layout(const LgParams& P) {
  const size_t VH = P.VH;
  const size_t b[PJ_N] = {sizeof(ReadHdr), VH * 16, VH * 16, (size_t)P.H * 16, (size_t)P.V * 4, (size_t)P.V * 4,
                          VH, VH * 4, VH * 4, VH * 4, VH, VH * 4};
  return make_layout(b, PJ_N);
}
// assoc: 0 header, 1 sharp, 2 sharp ind, 3 less sharp, 4 less sharp ind, 5 flat, 6 flat ind,
// 7 less flat, 8 corner Last, 9 surf Last, 10 outlier Last
constexpr int AS_N = 11;
PackLayout assoc_layout(const LgParams& P) {
  const size_t VH = P.VH, V = P.V;
  const size_t b[AS_N] = {sizeof(ReadHdr), V * P.cap_sharp * 16, V * P.cap_sharp * 4, V * P.cap_lsharp * 16,
                          V * P.cap_lsharp * 4, V * P.cap_flat * 16, V * P.cap_flat * 4, VH * 16,
                          V * P.cap_lsharp * 16, VH * 16, VH * 16};
  return make_layout(b, AS_N);
}

// the header's four parts (counts, orientation, front-end state, LgState) of stream s
int hdr_descs(const lego_batch* b, int s, char* dst, PackDesc* d) {
  const LgBufs& B = b->B;
  d[0] = {(const char*)(B.counts + (size_t)s * CNT_N), nullptr, 0, dst + offsetof(ReadHdr, cnt), nullptr,
          (int32_t)sizeof(int32_t) * CNT_N, 1};
  d[1] = {(const char*)(B.orient + (size_t)s * 4), nullptr, 0, dst + offsetof(ReadHdr, ori), nullptr, 16, 1};
  d[2] = {(const char*)(B.fe_state + (size_t)s * 2), nullptr, 0, dst + offsetof(ReadHdr, fe), nullptr, 8, 1};
  d[3] = {(const char*)(B.state + s), nullptr, 0, dst + offsetof(ReadHdr, S), nullptr, (int32_t)sizeof(LgState), 1};
  return 4;
}

int launch_pack(const PackDesc* d, int n, hipStream_t st) {
  PackArgs a{};
  for (int i = 0; i < n; ++i) a.d[i] = d[i];
  hipLaunchKernelGGL(k_pack, dim3(16, n), dim3(256), 0, st, a);
  return hipGetLastError() == hipSuccess ? LEGO_OK : LEGO_EDEVICE;
}

// ProjectionOut of stream 0 into c->pk_proj, then one wait; out's arrays point into it
int pack_proj(lego_ctx* c, lego_projection_out* o, int* fe_status) {
  lego_batch* b = c->b;
  const LgParams& P = b->P;
  const LgBufs& B = b->B;
  const PackLayout L = proj_layout(P);
  char* dp = c->pk_proj.dp;
  const int32_t* cnt = B.counts;
  const int VH = P.VH;
  PackDesc d[PACK_MAX];
  int n = hdr_descs(b, 0, dp + L.off[0], d);
  d[n++] = {(const char*)B.seg_pts, nullptr, 0, dp + L.off[1], cnt + CNT_M, VH, 16};
  d[n++] = {(const char*)B.outlier, nullptr, 0, dp + L.off[2], cnt + CNT_OUTLIER, VH, 16};
  d[n++] = {(const char*)B.scan_msg, nullptr, 0, dp + L.off[3], cnt + CNT_SCAN, P.H, 16};
  d[n++] = {(const char*)B.ring_start, nullptr, 0, dp + L.off[4], nullptr, P.V, 4};
  d[n++] = {(const char*)B.ring_end, nullptr, 0, dp + L.off[5], nullptr, P.V, 4};
  d[n++] = {(const char*)B.seg_ground, nullptr, 0, dp + L.off[6], cnt + CNT_M, VH, 1};
  d[n++] = {(const char*)B.seg_col, nullptr, 0, dp + L.off[7], cnt + CNT_M, VH, 4};
  d[n++] = {(const char*)B.seg_range, nullptr, 0, dp + L.off[8], cnt + CNT_M, VH, 4};
  d[n++] = {(const char*)B.label, nullptr, 0, dp + L.off[9], nullptr, VH, 4};
  d[n++] = {(const char*)B.ground, nullptr, 0, dp + L.off[10], nullptr, VH, 1};
  d[n++] = {(const char*)B.range, nullptr, 0, dp + L.off[11], nullptr, VH, 4};
  if (launch_pack(d, n, nullptr) != LEGO_OK || hipStreamSynchronize(nullptr) != hipSuccess) return LEGO_EDEVICE;
  char* hp = c->pk_proj.p;
  const ReadHdr* h = (const ReadHdr*)(hp + L.off[0]);
  *fe_status = h->fe[0];
  if (!o) return LEGO_OK;
  o->n_segmented = h->cnt[CNT_M];
  o->n_outlier = h->cnt[CNT_OUTLIER];
  o->n_scan = h->cnt[CNT_SCAN];
  o->segmented_cloud = (lego_point*)(hp + L.off[1]);
  o->outlier_cloud = (lego_point*)(hp + L.off[2]);
  o->scan_msg = (lego_point*)(hp + L.off[3]);
  o->start_ring_index = (int32_t*)(hp + L.off[4]);
  o->end_ring_index = (int32_t*)(hp + L.off[5]);
  o->start_orientation = h->ori[0];
  o->end_orientation = h->ori[1];
  o->orientation_diff = h->ori[2];
  o->segmented_cloud_ground_flag = (uint8_t*)(hp + L.off[6]);
  o->segmented_cloud_col_ind = (uint32_t*)(hp + L.off[7]);
  o->segmented_cloud_range = (float*)(hp + L.off[8]);
  o->label_mat = (int32_t*)(hp + L.off[9]);
  o->ground_mat = (int8_t*)(hp + L.off[10]);
  o->range_mat = (float*)(hp + L.off[11]);
  return LEGO_OK;
}

// AssociationOut of stream 0 into c->pk_assoc, then one wait
int pack_assoc(lego_ctx* c, lego_association_out* o) {
  lego_batch* b = c->b;
  const LgParams& P = b->P;
  const LgBufs& B = b->B;
  const PackLayout L = assoc_layout(P);
  char* dp = c->pk_assoc.dp;
  const int32_t* cnt = B.counts;
  const size_t VH = P.VH, V = P.V;
  const size_t hs = (size_t)b->last_par;  // the feature half of the last scan (S = 1)
  const size_t cls = V * P.cap_lsharp;
  const int32_t* last_buf = (const int32_t*)((const char*)B.state + offsetof(LgState, last_buf));
  const int32_t* n_cl = (const int32_t*)((const char*)B.state + offsetof(LgState, n_corner_last));
  const int32_t* n_sl = (const int32_t*)((const char*)B.state + offsetof(LgState, n_surf_last));
  PackDesc d[PACK_MAX];
  int n = hdr_descs(b, 0, dp + L.off[0], d);
  d[n++] = {(const char*)(B.f_sharp + hs * V * P.cap_sharp), nullptr, 0, dp + L.off[1], cnt + CNT_SHARP,
            (int32_t)(V * P.cap_sharp), 16};
  d[n++] = {(const char*)(B.f_sharp_ind + hs * V * P.cap_sharp), nullptr, 0, dp + L.off[2], cnt + CNT_SHARP,
            (int32_t)(V * P.cap_sharp), 4};
  d[n++] = {(const char*)(B.f_lsharp + hs * V * P.cap_lsharp), nullptr, 0, dp + L.off[3], cnt + CNT_LSHARP,
            (int32_t)cls, 16};
  d[n++] = {(const char*)(B.f_lsharp_ind + hs * V * P.cap_lsharp), nullptr, 0, dp + L.off[4], cnt + CNT_LSHARP,
            (int32_t)cls, 4};
  d[n++] = {(const char*)(B.f_flat + hs * V * P.cap_flat), nullptr, 0, dp + L.off[5], cnt + CNT_FLAT,
            (int32_t)(V * P.cap_flat), 16};
  d[n++] = {(const char*)(B.f_flat_ind + hs * V * P.cap_flat), nullptr, 0, dp + L.off[6], cnt + CNT_FLAT,
            (int32_t)(V * P.cap_flat), 4};
  d[n++] = {(const char*)B.f_lflat, nullptr, 0, dp + L.off[7], cnt + CNT_LFLAT, (int32_t)VH, 16};
  d[n++] = {(const char*)B.corner_last, last_buf, (long long)(cls * 16), dp + L.off[8], n_cl, (int32_t)cls, 16};
  d[n++] = {(const char*)B.surf_last, last_buf, (long long)(VH * 16), dp + L.off[9], n_sl, (int32_t)VH, 16};
  d[n++] = {(const char*)B.outlier_fa, nullptr, 0, dp + L.off[10], cnt + CNT_OUTLIER, (int32_t)VH, 16};
  if (launch_pack(d, n, nullptr) != LEGO_OK || hipStreamSynchronize(nullptr) != hipSuccess) return LEGO_EDEVICE;
  char* hp = c->pk_assoc.p;
  const ReadHdr* h = (const ReadHdr*)(hp + L.off[0]);
  if (!o) return LEGO_OK;
  const int32_t* k = h->cnt;
  const LgState& S = h->S;
  o->status = S.status;
  o->n_sharp = k[CNT_SHARP];
  o->n_less_sharp = k[CNT_LSHARP];
  o->n_flat = k[CNT_FLAT];
  o->n_less_flat = k[CNT_LFLAT];
  o->corner_points_sharp = (lego_point*)(hp + L.off[1]);
  o->sharp_ind = (int32_t*)(hp + L.off[2]);
  o->corner_points_less_sharp = (lego_point*)(hp + L.off[3]);
  o->less_sharp_ind = (int32_t*)(hp + L.off[4]);
  o->surf_points_flat = (lego_point*)(hp + L.off[5]);
  o->flat_ind = (int32_t*)(hp + L.off[6]);
  o->surf_points_less_flat = (lego_point*)(hp + L.off[7]);
  for (int i = 0; i < 6; ++i) {
    o->transform_cur[i] = S.cur[i];
    o->transform_sum[i] = S.sum[i];
  }
  odom_quat(S.sum, o->odom_orientation);
  for (int i = 0; i < 3; ++i) o->odom_position[i] = S.pos[i];
  o->lm_iter_surf = S.iters_surf;
  o->lm_iter_corner = S.iters_corner;
  o->n_corner_last = S.n_corner_last;
  o->n_surf_last = S.n_surf_last;
  o->n_outlier_last = k[CNT_OUTLIER];
  o->cloud_corner_last = (lego_point*)(hp + L.off[8]);
  o->cloud_surf_last = (lego_point*)(hp + L.off[9]);
  o->cloud_outlier_last = (lego_point*)(hp + L.off[10]);
  return LEGO_OK;
}
}  // namespace

extern "C" {

// ---------------------------------------------------------------------------------------------
// single-sequence drop-in
// ---------------------------------------------------------------------------------------------
int lego_ctx_create(const lego_params* p, int32_t device, lego_ctx** out) {
  if (!out) return LEGO_EINVAL;
  *out = nullptr;
  if (!p) return LEGO_EINVAL;
  lego_ctx* c = new (std::nothrow) lego_ctx();
  if (!c) return LEGO_ENOMEM;
  const int cap = p->num_vertical_scans > 0 && p->num_horizontal_scans > 0
                      ? 4 * p->num_vertical_scans * p->num_horizontal_scans : 1;
  int rc = lego_batch_create(p, device, 1, cap, &c->b);
  if (rc != LEGO_OK) {
    delete c;
    return rc;
  }
  c->cap = 0;
  if (hipMalloc((void**)&c->d_off, sizeof(int64_t)) != hipSuccess ||
      hipMalloc((void**)&c->d_in, sizeof(float4)) != hipSuccess) {
    delete c;
    return LEGO_ENOMEM;
  }
  if ((rc = c->pk_proj.alloc(proj_layout(c->b->P).total)) != LEGO_OK ||
      (rc = c->pk_assoc.alloc(assoc_layout(c->b->P).total)) != LEGO_OK) {
    delete c;
    return rc;
  }
  int64_t zero = 0;
  hipMemcpy(c->d_off, &zero, sizeof(zero), hipMemcpyHostToDevice);
  *out = c;
  return LEGO_OK;
}

void lego_ctx_destroy(lego_ctx* ctx) { delete ctx; }

int lego_cloud_handler(lego_ctx* c, const void* points, int32_t n, int32_t step, int32_t ox, int32_t oy, int32_t oz,
                       lego_projection_out* out) {
  if (!c || (!points && n > 0) || n < 0 || n > LEGO_MAX_POINTS || step < 12 || ox < 0 || oy < 0 || oz < 0 || ox + 4 > step ||
      oy + 4 > step || oz + 4 > step)
    return LEGO_EINVAL;
  lego_batch* b = c->b;
  hipSetDevice(b->device);
  // fromROSMsg: gather x,y,z from the strided PointCloud2 payload (intensity is not used by the path),
  // behind the point count: one pinned buffer, one upload
  float4* hin = c->h_in.get<float4>((size_t)n + 1);
  if (!hin) return LEGO_ENOMEM;
  *(int32_t*)hin = n;
  float4* hp = hin + 1;
  const char* base = (const char*)points;
  if (ox == 0 && oy == 4 && oz == 8 && step == 16) {  // x, y, z, intensity records: the payload as it is
    if (n > 0) memcpy(hp, base, (size_t)n * 16);       // (the 4th word is never read by the kernels)
  } else if (ox == 0 && oy == 4 && oz == 8) {  // padded records (PointXYZIR's 32 bytes): 16 bytes each
    for (int i = 0; i < n; ++i) memcpy(&hp[i], base + (size_t)i * step, 16);
  } else {
    for (int i = 0; i < n; ++i) {
      float4 q;
      memcpy(&q.x, base + (size_t)i * step + ox, 4);
      memcpy(&q.y, base + (size_t)i * step + oy, 4);
      memcpy(&q.z, base + (size_t)i * step + oz, 4);
      q.w = 0.f;
      hp[i] = q;
    }
  }
  if (n > c->cap) {
    hipStreamSynchronize(nullptr);  // the previous call's kernels may still read d_in (they do not: every
                                    // call ends with a wait; kept for safety)
    if (c->d_in) hipFree(c->d_in);
    c->d_in = nullptr;
    if (hipMalloc((void**)&c->d_in, ((size_t)n + 1) * sizeof(float4)) != hipSuccess) return LEGO_ENOMEM;
    c->cap = n;
  }
  // everything in order on the null stream: upload, kernels, the pack into mapped host memory, one wait
  if (hipMemcpyAsync(c->d_in, hin, ((size_t)n + 1) * sizeof(float4), hipMemcpyHostToDevice, nullptr) != hipSuccess)
    return LEGO_EDEVICE;
  int rc = chain_stream(b, nullptr);
  if (!rc) rc = next_wtag(b, nullptr);
  if (rc) return rc;
  rc = run_projection(b, c->d_in + 1, c->d_off, (const int32_t*)c->d_in, nullptr, 0, 1);
  if (rc) return rc;
  int fe = LEGO_OK;
  rc = pack_proj(c, out, &fe);
  if (rc) return rc;
  return fe;
}

static int feature_association(lego_ctx* c, lego_association_out* out, bool distort) {
  lego_batch* b = c->b;
  hipSetDevice(b->device);
  b->epoch = b->epoch == 0x7fffffff ? 1 : b->epoch + 1;
  // lag 0, then flushed: VoxelGrid on the side stream while k_lm runs, then k_publish (joined with
  // it) before the reads
  int rc = ensure_streams(b, 1);
  if (!rc) rc = chain_stream(b, nullptr);
  if (!rc) rc = run_association(b, nullptr, 0, 1, distort, 0, false);
  if (rc) return rc;
  advance_pipeline(b, false, 1);
  rc = flush_pending(b);
  if (rc) return rc;
  return pack_assoc(c, out);  // also the wait for the kernels
}

int lego_feature_association(lego_ctx* c, lego_association_out* out) {
  if (!c) return LEGO_EINVAL;
  return feature_association(c, out, false);
}

// Test hook: overwrite the LM state the next association starts from (per pair, the
// reference's transformCur_in and Last clouds injected).  After the first association only.
int lego_test_set_lm_state(lego_ctx* c, const float* cur6, const float* sum6, int32_t degenerate,
                           const lego_point* corner_last, int32_t n_corner, const lego_point* surf_last,
                           int32_t n_surf, int32_t tree_stale) {
  if (!c || !cur6 || !sum6 || n_corner < 0 || n_surf < 0 || (n_corner && !corner_last) || (n_surf && !surf_last))
    return LEGO_EINVAL;
  lego_batch* b = c->b;
  const LgParams& P = b->P;
  const LgBufs& B = b->B;
  // the corner Last cloud's kd-tree / grid scratch is sized by V*H (kd_vind, kd_tmp, kd_node, grid_pts):
  // with H < cap_lsharp an injected cloud of V*cap_lsharp points would not fit it
  if (n_corner > std::min(P.V * P.cap_lsharp, P.VH) || n_surf > P.VH) return LEGO_EINVAL;
  hipSetDevice(b->device);
  if (flush_pending(b) != LEGO_OK || hipDeviceSynchronize() != hipSuccess) return LEGO_EDEVICE;
  LgState S;
  if (hipMemcpy(&S, B.state, sizeof(S), hipMemcpyDeviceToHost) != hipSuccess) return LEGO_EDEVICE;
  if (!S.initialized) return LEGO_EINVAL;
  for (int k = 0; k < 6; ++k) {
    S.cur[k] = cur6[k];
    S.sum[k] = sum6[k];
  }
  S.is_degenerate = degenerate ? 1 : 0;
  S.n_corner_last = n_corner;
  S.n_surf_last = n_surf;
  S.tree_stale = tree_stale ? 1 : 0;
  const size_t cls = (size_t)P.V * P.cap_lsharp;
  if ((n_corner && hipMemcpy(B.corner_last + (size_t)S.last_buf * cls, corner_last, (size_t)n_corner * 16,
                             hipMemcpyHostToDevice) != hipSuccess) ||
      (n_surf && hipMemcpy(B.surf_last + (size_t)S.last_buf * P.VH, surf_last, (size_t)n_surf * 16,
                           hipMemcpyHostToDevice) != hipSuccess) ||
      hipMemcpy(B.state, &S, sizeof(S), hipMemcpyHostToDevice) != hipSuccess)
    return LEGO_EDEVICE;
  return LEGO_OK;
}

int lego_feature_association_from(lego_ctx* c, const lego_projection_out* in, lego_association_out* out) {
  if (!c || !in) return LEGO_EINVAL;
  lego_batch* b = c->b;
  const LgParams& P = b->P;
  const LgBufs& B = b->B;
  const int M = in->n_segmented;
  if (M < 0 || M > P.VH || in->n_outlier < 0 || in->n_outlier > P.VH) return LEGO_EINVAL;
  // cloud_info as imageProjection builds it (:358-396): column indices < H, and each ring's
  // [start, end] inside the cloud and at most one point per column wide (k_extract stages a ring's
  // window of H + 11 positions)
  for (int i = 0; i < M; ++i)
    if (in->segmented_cloud_col_ind[i] >= (uint32_t)P.H) return LEGO_EINVAL;
  for (int r = 0; r < P.V; ++r) {
    const int st = in->start_ring_index[r], en = in->end_ring_index[r];
    if (st < 0 || st > M + 4 || en < -6 || en >= M || en - st > P.H - 10) return LEGO_EINVAL;
  }
  hipSetDevice(b->device);
  // the reference's Channel<ProjectionOut>::receive (fa.cpp:1389-1397): upload the message
  bool ok = true;
  auto up = [&](void* d, const void* h, size_t bytes) {
    if (bytes && hipMemcpy(d, h, bytes, hipMemcpyHostToDevice) != hipSuccess) ok = false;
  };
  up(B.seg_pts, in->segmented_cloud, (size_t)M * sizeof(float4));
  up(B.seg_range, in->segmented_cloud_range, (size_t)M * sizeof(float));
  up(B.seg_col, in->segmented_cloud_col_ind, (size_t)M * sizeof(uint32_t));
  up(B.seg_ground, in->segmented_cloud_ground_flag, (size_t)M);
  up(B.ring_start, in->start_ring_index, (size_t)P.V * sizeof(int32_t));
  up(B.ring_end, in->end_ring_index, (size_t)P.V * sizeof(int32_t));
  up(B.outlier, in->outlier_cloud, (size_t)in->n_outlier * sizeof(float4));
  float ori[4] = {in->start_orientation, in->end_orientation, in->orientation_diff, 1.f};
  up(B.orient, ori, sizeof(ori));
  int32_t cnt[CNT_N] = {M, in->n_outlier, 0, 0, 0, 0, 0, 0};
  up(B.counts, cnt, sizeof(cnt));
  if (!ok) return LEGO_EDEVICE;
  return feature_association(c, out, true);
}

}  // extern "C"
