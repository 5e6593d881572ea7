// lego_config.cpp — lego_params from the reference's config/loam_config.yaml (include/lego_frontend.h).
//
// The reference reads its parameters with ros::NodeHandle::getParam("/lego_loam/<section>/<key>")
// (imageProjection.cpp:57-84, featureAssociation.cpp:69-81) from the rosparam server, which roslaunch
// fills from LeGO-LOAM/config/loam_config.yaml (keys :4-25).  Without ROS this loader reads that file:
// the block-style YAML subset the file uses (nested maps by indentation, "key: scalar" lines, # comments,
// no flow collections or anchors).  Keys are matched by their full path below lego_loam; other keys
// (loop closure, the mapping radii) are ignored, and keys the file does not set keep
// lego_params_vlp16's values.  lego_amd/fp_mode and lego_amd/voxel_tie_order (this build's own
// parameters) may also be set there.
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/lego_frontend.h"

namespace {

std::string trim(const std::string& s) {
  size_t a = 0, b = s.size();
  while (a < b && (s[a] == ' ' || s[a] == '\t' || s[a] == '\r' || s[a] == '\n')) ++a;
  while (b > a && (s[b - 1] == ' ' || s[b - 1] == '\t' || s[b - 1] == '\r' || s[b - 1] == '\n')) --b;
  return s.substr(a, b - a);
}

// the value without a trailing comment (a '#' preceded by whitespace) and without quotes
std::string scalar(const std::string& v) {
  std::string r = v;
  for (size_t i = 0; i < r.size(); ++i)
    if (r[i] == '#' && (i == 0 || r[i - 1] == ' ' || r[i - 1] == '\t')) {
      r = r.substr(0, i);
      break;
    }
  r = trim(r);
  if (r.size() >= 2 && ((r.front() == '"' && r.back() == '"') || (r.front() == '\'' && r.back() == '\'')))
    r = r.substr(1, r.size() - 2);
  return r;
}

bool parse_int(const std::string& s, int32_t* out) {
  if (s.empty()) return false;
  char* end = nullptr;
  errno = 0;
  const long v = strtol(s.c_str(), &end, 10);
  if (errno || *end != '\0' || v < -2147483647L - 1 || v > 2147483647L) return false;
  *out = (int32_t)v;
  return true;
}

bool parse_float(const std::string& s, float* out) {  // rosparam's YAML floats (ints accepted, as getParam)
  if (s.empty()) return false;
  char* end = nullptr;
  errno = 0;
  const double v = strtod(s.c_str(), &end);
  if (errno || *end != '\0' || !std::isfinite(v)) return false;
  *out = (float)v;
  return true;
}

}  // namespace

extern "C" int lego_params_load_yaml(const char* path, lego_params* p) {
  if (!path || !p) return LEGO_EINVAL;
  FILE* f = fopen(path, "r");
  if (!f) return LEGO_EINVAL;
  lego_params q;
  lego_params_vlp16(&q);
  std::vector<std::pair<int, std::string>> stack;  // (indent, key) of the open maps
  char buf[4096];
  int rc = LEGO_OK;
  while (rc == LEGO_OK && fgets(buf, sizeof(buf), f)) {
    const std::string line(buf);
    if (line.size() + 1 >= sizeof(buf) && line.back() != '\n') { rc = LEGO_EINVAL; break; }  // over-long line
    size_t ind = 0;
    while (ind < line.size() && line[ind] == ' ') ++ind;
    const std::string body = trim(line.substr(ind));
    if (body.empty() || body[0] == '#' || body == "---" || body == "...") continue;
    if (line[ind] == '\t') { rc = LEGO_EINVAL; break; }  // YAML forbids tab indentation
    const size_t colon = body.find(':');
    if (colon == std::string::npos || colon == 0 || (colon + 1 < body.size() && body[colon + 1] != ' ')) {
      rc = LEGO_EINVAL;  // not a "key:" / "key: value" line (sequences and flow styles are not used by the file)
      break;
    }
    const std::string key = trim(body.substr(0, colon));
    const std::string val = scalar(body.substr(colon + 1));
    while (!stack.empty() && stack.back().first >= (int)ind) stack.pop_back();
    if (val.empty()) {  // a map opens
      stack.push_back({(int)ind, key});
      continue;
    }
    std::string path_;
    for (const auto& e : stack) path_ += e.second + "/";
    path_ += key;
    bool ok = true;
    if (path_ == "lego_loam/laser/num_vertical_scans") ok = parse_int(val, &q.num_vertical_scans);
    else if (path_ == "lego_loam/laser/num_horizontal_scans") ok = parse_int(val, &q.num_horizontal_scans);
    else if (path_ == "lego_loam/laser/ground_scan_index") ok = parse_int(val, &q.ground_scan_index);
    else if (path_ == "lego_loam/laser/vertical_angle_bottom") ok = parse_float(val, &q.vertical_angle_bottom);
    else if (path_ == "lego_loam/laser/vertical_angle_top") ok = parse_float(val, &q.vertical_angle_top);
    else if (path_ == "lego_loam/laser/sensor_mount_angle") ok = parse_float(val, &q.sensor_mount_angle);
    else if (path_ == "lego_loam/laser/scan_period") ok = parse_float(val, &q.scan_period);
    else if (path_ == "lego_loam/imageProjection/segment_valid_point_num") ok = parse_int(val, &q.segment_valid_point_num);
    else if (path_ == "lego_loam/imageProjection/segment_valid_line_num") ok = parse_int(val, &q.segment_valid_line_num);
    else if (path_ == "lego_loam/imageProjection/segment_theta") ok = parse_float(val, &q.segment_theta);
    else if (path_ == "lego_loam/featureAssociation/edge_threshold") ok = parse_float(val, &q.edge_threshold);
    else if (path_ == "lego_loam/featureAssociation/surf_threshold") ok = parse_float(val, &q.surf_threshold);
    else if (path_ == "lego_loam/featureAssociation/nearest_feature_search_distance")
      ok = parse_float(val, &q.nearest_feature_search_distance);
    else if (path_ == "lego_loam/mapping/mapping_frequency_divider") ok = parse_int(val, &q.mapping_frequency_divider);
    else if (path_ == "lego_loam/lego_amd/fp_mode") ok = parse_int(val, &q.fp_mode);
    else if (path_ == "lego_loam/lego_amd/voxel_tie_order") ok = parse_int(val, &q.voxel_tie_order);
    if (!ok) rc = LEGO_EINVAL;  // a known key with a malformed value
  }
  if (ferror(f)) rc = LEGO_EINVAL;
  fclose(f);
  if (rc != LEGO_OK) return rc;
  rc = lego_params_validate(&q);
  if (rc != LEGO_OK) return rc;
  *p = q;
  return LEGO_OK;
}
