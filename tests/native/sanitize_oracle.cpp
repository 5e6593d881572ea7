// Host-code sanitizer driver: the CPU oracle (oracle/lego_oracle.cpp, oracle/s2m_oracle.cpp)
// and the synthetic-sweep generator, compiled with -fsanitize=address,undefined by
// tests/test_sanitizers_cpu.py, run over VLP-16 / HDL-64E sequences, edge clouds (tiny, all-NaN,
// colliding, out of range), the VoxelGrid on overflowing / empty / duplicate clouds and scan-to-map
// problems.  Any sanitizer report aborts with a non-zero status.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../include/lego_frontend.h"

extern "C" {
typedef struct lego_synth_cfg {
  int32_t V, H;
  float elev_bottom_deg, elev_top_deg, sensor_height;
  int32_t base_seed;
  float dropout, range_noise, az_jitter_deg, max_range, speed, yaw_rate_deg, roll_pitch_noise_deg, scan_period;
} lego_synth_cfg;
void lego_synth_vlp16(lego_synth_cfg* c);
void lego_synth_hdl64(lego_synth_cfg* c);
int lego_synth_scan(const lego_synth_cfg* c, int seq, int scan, float* out, int cap);

struct oracle_ctx;
oracle_ctx* oracle_create(const lego_params* p);
void oracle_destroy(oracle_ctx* c);
int oracle_cloud_handler(oracle_ctx* c, const void* pts, int n, int step, int ox, int oy, int oz, lego_projection_out* out);
int oracle_feature_association(oracle_ctx* c, lego_association_out* out);
int oracle_voxel_grid(const float* in, int n, float leaf, int stable, float* out, int* n_out);
int oracle_scan2map(const float* corner, int n_corner, const float* surf, int n_surf, const float* corner_map,
                    int n_corner_map, const float* surf_map, int n_surf_map, float* transform, int32_t* degenerate,
                    int32_t* info);
}

// the parameters the C-ABI library would give (lego_params_vlp16 / _hdl64; restated: no GPU library here)
static lego_params params(bool hdl, int fp_mode, int order) {
  lego_params p;
  std::memset(&p, 0, sizeof(p));
  p.num_vertical_scans = hdl ? 64 : 16;
  p.num_horizontal_scans = hdl ? 2048 : 1800;
  p.ground_scan_index = hdl ? 55 : 7;
  p.vertical_angle_bottom = hdl ? -24.8f : -15.f;
  p.vertical_angle_top = hdl ? 2.0f : 15.f;
  p.scan_period = 0.1f;
  p.segment_valid_point_num = 5;
  p.segment_valid_line_num = 3;
  p.segment_theta = 60.f;
  p.edge_threshold = 0.1f;
  p.surf_threshold = 0.1f;
  p.nearest_feature_search_distance = 5.f;
  p.mapping_frequency_divider = 5;
  p.fp_mode = fp_mode;
  p.voxel_tie_order = order;
  return p;
}

static int run_sequence(bool hdl, int fp_mode, int order, int seq, int scans, std::vector<std::vector<float>>* keep) {
  lego_synth_cfg cfg;
  if (hdl) lego_synth_hdl64(&cfg); else lego_synth_vlp16(&cfg);
  const lego_params p = params(hdl, fp_mode, order);
  oracle_ctx* c = oracle_create(&p);
  if (!c) return 1;
  const int cap = 4 * cfg.V * cfg.H;
  std::vector<float> pts((size_t)cap * 4);
  for (int k = 0; k < scans; ++k) {
    const int n = lego_synth_scan(&cfg, seq, k, pts.data(), cap);
    if (n < 0) return 1;
    std::vector<float> cloud(pts.begin(), pts.begin() + (size_t)4 * n);
    if (k == scans - 1 && keep) keep->push_back(cloud);
    // edge variants on some scans: a NaN every 37th point, every 101st point duplicated later
    if (k % 3 == 1)
      for (int i = 0; i < n; i += 37) cloud[(size_t)4 * i] = NAN;
    if (k % 3 == 2)
      for (int i = 0; i < n; i += 101) cloud.insert(cloud.end(), cloud.begin() + 4 * i, cloud.begin() + 4 * i + 4);
    lego_projection_out po;
    lego_association_out ao;
    if (oracle_cloud_handler(c, cloud.data(), (int)(cloud.size() / 4), 16, 0, 4, 8, &po) != LEGO_OK) return 1;
    if (oracle_feature_association(c, &ao) != LEGO_OK) return 1;
  }
  oracle_destroy(c);
  return 0;
}

int main() {
  int bad = 0;
  std::vector<std::vector<float>> last;
  for (int fp = 0; fp < 2; ++fp)
    for (int order = 0; order < 2; ++order) bad |= run_sequence(false, fp, order, 3 + fp + 2 * order, 7, &last);
  bad |= run_sequence(true, 0, 0, 1, 3, nullptr);
  // tiny / empty / all-NaN / out-of-range clouds
  {
    const lego_params p = params(false, 0, 0);
    oracle_ctx* c = oracle_create(&p);
    lego_projection_out po;
    lego_association_out ao;
    std::vector<float> nanc(64 * 4, NAN), far(64 * 4, 500.f), tiny(last[0].begin(), last[0].begin() + 40 * 4);
    if (oracle_cloud_handler(c, nanc.data(), 64, 16, 0, 4, 8, &po) != LEGO_EEMPTY) bad = 1;
    if (oracle_cloud_handler(c, nanc.data(), 0, 16, 0, 4, 8, &po) != LEGO_EEMPTY) bad = 1;
    for (int r = 0; r < 3; ++r) {
      for (const auto* cl : {&far, &tiny, &last[0]}) {
        if (oracle_cloud_handler(c, cl->data(), (int)(cl->size() / 4), 16, 0, 4, 8, &po) != LEGO_OK) bad = 1;
        if (oracle_feature_association(c, &ao) != LEGO_OK) bad = 1;
      }
    }
    oracle_destroy(c);
  }
  // VoxelGrid: overflowing leaf indices, empty, one point, duplicates
  {
    std::vector<float> out(last[0].size() + 64);
    int n_out = 0;
    oracle_voxel_grid(last[0].data(), (int)(last[0].size() / 4), 1e-4f, 0, out.data(), &n_out);
    oracle_voxel_grid(last[0].data(), 0, 0.2f, 1, out.data(), &n_out);
    oracle_voxel_grid(last[0].data(), 1, 0.2f, 0, out.data(), &n_out);
    std::vector<float> dup;
    for (int r = 0; r < 16; ++r) dup.insert(dup.end(), last[0].begin(), last[0].begin() + 4 * 200);
    std::vector<float> out2(dup.size());
    oracle_voxel_grid(dup.data(), (int)(dup.size() / 4), 0.2f, 0, out2.data(), &n_out);
  }
  // scan-to-map on a scan against the union of the last scans (and degenerate / empty inputs)
  {
    std::vector<float> map;
    for (const auto& l : last) map.insert(map.end(), l.begin(), l.end());
    float t[6] = {0.001f, 0.002f, 0.f, 0.05f, 0.f, 0.1f};
    int32_t dg = 0, info[4];
    const int nm = (int)(map.size() / 4), ns = (int)(last[1].size() / 4);
    oracle_scan2map(last[1].data(), ns / 10, last[1].data(), ns, map.data(), nm / 10, map.data(), nm, t, &dg, info);
    oracle_scan2map(last[1].data(), 0, last[1].data(), 0, map.data(), 0, map.data(), 0, t, &dg, info);
  }
  printf("sanitized oracle run: %s\n", bad ? "FAILED" : "ok");
  return bad;
}
