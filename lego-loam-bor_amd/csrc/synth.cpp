// synth.cpp — deterministic synthetic lidar sweeps.
//
// Ray-casts a VLP-16 / HDL-64E-like sensor through a per-sequence scene (ground plane, yawed boxes,
// vertical cylinders) while the sensor moves along a planar arc.  Points are emitted in Velodyne
// firing order (azimuth-major, clockwise sweep; within a column the interleaved laser order
// 0,V/2,1,V/2+1,...) and expressed in the sensor frame at their own firing time, so per-scan motion
// distortion is present as in real data.  All randomness is splitmix64 seeded by
// (base_seed, sequence, scan): the same call always yields the same float32 bytes.
//
// This is input generation for tests and the benchmark, not part of the reference's hot path.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#ifdef _OPENMP
#include <omp.h>
#endif

extern "C" {
typedef struct lego_synth_cfg {
  int32_t V, H;
  float elev_bottom_deg, elev_top_deg;  // evenly spaced rings
  float sensor_height;                  // ground plane at z = -sensor_height
  int32_t base_seed;
  float dropout;                        // probability a return is lost
  float range_noise;                    // sigma (m)
  float az_jitter_deg;                  // uniform +- jitter of each column's azimuth
  float max_range;                      // returns beyond are dropped
  float speed;                          // m per scan
  float yaw_rate_deg;                   // deg per scan
  float roll_pitch_noise_deg;           // per-scan sigma
  float scan_period;                    // s (only for time bookkeeping)
} lego_synth_cfg;
}

namespace {

struct Rng {
  uint64_t s;
  explicit Rng(uint64_t seed) : s(seed) {}
  uint64_t next() {
    uint64_t z = (s += 0x9E3779B97F4A7C15ULL);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
  }
  double uni() { return (next() >> 11) * (1.0 / 9007199254740992.0); }
  double uni(double a, double b) { return a + (b - a) * uni(); }
  double gauss() {
    double u1 = uni(), u2 = uni();
    if (u1 < 1e-300) u1 = 1e-300;
    return std::sqrt(-2.0 * std::log(u1)) * std::cos(2.0 * M_PI * u2);
  }
};

uint64_t mix(uint64_t a, uint64_t b, uint64_t c) {
  Rng r(a * 0x9E3779B97F4A7C15ULL ^ (b + 0x632BE59BD9B4E019ULL) * 0xD6E8FEB86659FD93ULL ^
        (c + 0x1234567ULL) * 0xA0761D6478BD642FULL);
  r.next();
  return r.next();
}

struct Box { double cx, cy, hx, hy, z0, z1, cyaw, syaw; };
struct Cyl { double cx, cy, r, z0, z1; };
struct Scene { std::vector<Box> boxes; std::vector<Cyl> cyls; double ground_z; };

void pose_at(const lego_synth_cfg& c, double u, double& px, double& py, double& yaw) {
  const double w = c.yaw_rate_deg * M_PI / 180.0;  // rad per scan
  yaw = w * u;
  if (std::fabs(w) < 1e-12) {
    px = c.speed * u; py = 0.0;
  } else {
    px = c.speed / w * std::sin(w * u);
    py = c.speed / w * (1.0 - std::cos(w * u));
  }
}

Scene make_scene(const lego_synth_cfg& c, int seq) {
  Scene sc;
  sc.ground_z = -c.sensor_height;
  Rng r(mix((uint64_t)c.base_seed, (uint64_t)seq, 0xFFFFFFFFULL));
  // path samples for corridor rejection (first 300 scans)
  std::vector<double> pxs, pys;
  for (int k = 0; k <= 300; k += 2) {
    double x, y, yaw;
    pose_at(c, k, x, y, yaw);
    pxs.push_back(x); pys.push_back(y);
  }
  auto clear_of_path = [&](double x, double y, double rad) {
    for (size_t i = 0; i < pxs.size(); ++i) {
      double dx = x - pxs[i], dy = y - pys[i];
      if (dx * dx + dy * dy < (rad + 2.5) * (rad + 2.5)) return false;
    }
    return true;
  };
  // enclosure: tall building facades around the trajectory's circle (campus-like), so the upper
  // rings return as they do in the Stevens VLP-16 data
  {
    const double w = c.yaw_rate_deg * M_PI / 180.0;
    const double ccx = 0.0, ccy = (std::fabs(w) < 1e-12) ? 0.0 : c.speed / w;
    const int nw = 12 + (int)(r.next() % 5);
    for (int k = 0; k < nw; ++k) {
      double a = 2.0 * M_PI * (k + r.uni(-0.15, 0.15)) / nw;
      double rad = r.uni(28.0, 55.0);
      Box b;
      b.cx = ccx + rad * std::cos(a);
      b.cy = ccy + rad * std::sin(a);
      b.hx = rad * M_PI / nw * r.uni(0.75, 1.1);  // half chord: small gaps between facades
      b.hy = r.uni(0.5, 2.0);
      b.z0 = sc.ground_z;
      b.z1 = sc.ground_z + r.uni(10.0, 28.0);
      double yw = a + M_PI / 2;  // tangential
      b.cyaw = std::cos(yw); b.syaw = std::sin(yw);
      sc.boxes.push_back(b);
    }
  }
  int nb = sc.boxes.size() + 6 + (int)(r.next() % 7);
  for (int tries = 0; (int)sc.boxes.size() < nb && tries < 2000; ++tries) {
    double d = r.uni(6.0, 60.0), a = r.uni(-M_PI, M_PI);
    Box b;
    b.cx = d * std::cos(a) + r.uni(0.0, 15.0);
    b.cy = d * std::sin(a);
    b.hx = r.uni(1.0, 10.0);
    b.hy = r.uni(0.5, 3.0);
    b.z0 = sc.ground_z;
    b.z1 = sc.ground_z + r.uni(1.0, 8.0);
    double yw = r.uni(-M_PI, M_PI);
    b.cyaw = std::cos(yw); b.syaw = std::sin(yw);
    if (!clear_of_path(b.cx, b.cy, std::sqrt(b.hx * b.hx + b.hy * b.hy))) continue;
    sc.boxes.push_back(b);
  }
  int ncy = 10 + (int)(r.next() % 21);
  for (int tries = 0; (int)sc.cyls.size() < ncy && tries < 4000; ++tries) {
    double d = r.uni(3.0, 50.0), a = r.uni(-M_PI, M_PI);
    Cyl y;
    y.cx = d * std::cos(a) + r.uni(0.0, 15.0);
    y.cy = d * std::sin(a);
    y.r = r.uni(0.1, 0.5);
    y.z0 = sc.ground_z;
    y.z1 = sc.ground_z + r.uni(2.0, 6.0);
    if (!clear_of_path(y.cx, y.cy, y.r)) continue;
    sc.cyls.push_back(y);
  }
  return sc;
}

// nearest hit distance along (o + t d), t > 0; returns 1e30 if none
double cast(const Scene& sc, const double o[3], const double d[3]) {
  double best = 1e30;
  if (d[2] < -1e-9) {
    double t = (sc.ground_z - o[2]) / d[2];
    if (t > 0 && t < best) best = t;
  }
  for (const Box& b : sc.boxes) {
    // box frame: rotate by -yaw around (cx, cy)
    double ox = o[0] - b.cx, oy = o[1] - b.cy;
    double lox = b.cyaw * ox + b.syaw * oy, loy = -b.syaw * ox + b.cyaw * oy;
    double ldx = b.cyaw * d[0] + b.syaw * d[1], ldy = -b.syaw * d[0] + b.cyaw * d[1];
    double lo[3] = {lox, loy, o[2]}, ld[3] = {ldx, ldy, d[2]};
    double lo_b[3] = {-b.hx, -b.hy, b.z0}, hi_b[3] = {b.hx, b.hy, b.z1};
    double tmin = 0.0, tmax = best;
    bool hit = true;
    for (int k = 0; k < 3 && hit; ++k) {
      if (std::fabs(ld[k]) < 1e-12) {
        if (lo[k] < lo_b[k] || lo[k] > hi_b[k]) hit = false;
      } else {
        double t1 = (lo_b[k] - lo[k]) / ld[k], t2 = (hi_b[k] - lo[k]) / ld[k];
        if (t1 > t2) { double tt = t1; t1 = t2; t2 = tt; }
        if (t1 > tmin) tmin = t1;
        if (t2 < tmax) tmax = t2;
        if (tmin > tmax) hit = false;
      }
    }
    if (hit && tmin > 1e-6 && tmin < best) best = tmin;
  }
  for (const Cyl& y : sc.cyls) {
    double ox = o[0] - y.cx, oy = o[1] - y.cy;
    double a = d[0] * d[0] + d[1] * d[1];
    if (a < 1e-12) continue;
    double bq = 2.0 * (ox * d[0] + oy * d[1]);
    double cq = ox * ox + oy * oy - y.r * y.r;
    double disc = bq * bq - 4.0 * a * cq;
    if (disc < 0) continue;
    double t = (-bq - std::sqrt(disc)) / (2.0 * a);
    if (t <= 1e-6 || t >= best) continue;
    double z = o[2] + t * d[2];
    if (z < y.z0 || z > y.z1) continue;
    best = t;
  }
  return best;
}

int gen_scan(const lego_synth_cfg& c, const Scene& sc, int seq, int scan, float* out, int cap) {
  Rng r(mix((uint64_t)c.base_seed, (uint64_t)seq, (uint64_t)scan));
  const double deg = M_PI / 180.0;
  double roll = c.roll_pitch_noise_deg * deg * r.gauss();
  double pitch = c.roll_pitch_noise_deg * deg * r.gauss();
  double cr = std::cos(roll), sr = std::sin(roll), cp = std::cos(pitch), spp = std::sin(pitch);
  const double theta0 = M_PI - 1e-3;  // sweep starts behind the sensor, clockwise
  int n = 0;
  for (int col = 0; col < c.H; ++col) {
    double u = scan + (double)col / c.H;
    double px, py, yaw;
    pose_at(c, u, px, py, yaw);
    double cy = std::cos(yaw), sy = std::sin(yaw);
    double theta = theta0 - 2.0 * M_PI * col / c.H + c.az_jitter_deg * deg * r.uni(-1.0, 1.0);
    double ct = std::cos(theta), st = std::sin(theta);
    for (int k = 0; k < c.V; ++k) {
      int ring = (k % 2 == 0) ? k / 2 : c.V / 2 + k / 2;
      double phi = (c.elev_bottom_deg + ring * (c.elev_top_deg - c.elev_bottom_deg) / (c.V - 1)) * deg;
      double ds[3] = {std::cos(phi) * ct, std::cos(phi) * st, std::sin(phi)};
      // R = Rz(yaw) * Ry(pitch) * Rx(roll)
      double x1 = ds[0], y1 = cr * ds[1] - sr * ds[2], z1 = sr * ds[1] + cr * ds[2];
      double x2 = cp * x1 + spp * z1, y2 = y1, z2 = -spp * x1 + cp * z1;
      double dw[3] = {cy * x2 - sy * y2, sy * x2 + cy * y2, z2};
      double o[3] = {px, py, 0.0};
      double t = cast(sc, o, dw);
      double drop = r.uni();
      double noise = c.range_noise * r.gauss();
      if (t > c.max_range || drop < c.dropout) continue;
      double rr = t + noise;
      if (n >= cap) return -1;
      out[4 * n + 0] = (float)(rr * ds[0]);
      out[4 * n + 1] = (float)(rr * ds[1]);
      out[4 * n + 2] = (float)(rr * ds[2]);
      out[4 * n + 3] = (float)ring;
      ++n;
    }
  }
  return n;
}

}  // namespace

extern "C" {

void lego_synth_vlp16(lego_synth_cfg* c) {
  c->V = 16; c->H = 1800;
  c->elev_bottom_deg = -15.f; c->elev_top_deg = 15.f;
  c->sensor_height = 0.7f;
  c->base_seed = 42;
  c->dropout = 0.03f;
  c->range_noise = 0.01f;
  c->az_jitter_deg = 0.04f;
  c->max_range = 100.f;
  c->speed = 0.1f;
  c->yaw_rate_deg = 0.5f;
  c->roll_pitch_noise_deg = 0.1f;
  c->scan_period = 0.1f;
}

void lego_synth_hdl64(lego_synth_cfg* c) {
  lego_synth_vlp16(c);
  c->V = 64; c->H = 2048;
  c->elev_bottom_deg = -24.8f; c->elev_top_deg = 2.0f;
  c->sensor_height = 1.73f;
}

// One scan of sequence `seq`.  out: capacity cap points of 4 floats.  Returns the point count,
// or -1 if cap is too small.
int lego_synth_scan(const lego_synth_cfg* c, int seq, int scan, float* out, int cap) {
  Scene sc = make_scene(*c, seq);
  return gen_scan(*c, sc, seq, scan, out, cap);
}

// Many scans in parallel: scan i = (seqs[i], scans[i]) written at out + offsets[i]*4 (points),
// counts[i] = point count (or -1).
int lego_synth_batch(const lego_synth_cfg* c, int n, const int* seqs, const int* scans, float* out,
                     const int64_t* offsets, int cap, int* counts, int nthreads) {
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
  for (int i = 0; i < n; ++i) {
    Scene sc = make_scene(*c, seqs[i]);
    counts[i] = gen_scan(*c, sc, seqs[i], scans[i], out + 4 * offsets[i], cap);
  }
  for (int i = 0; i < n; ++i)
    if (counts[i] < 0) return -1;
  return 0;
}

}  // extern "C"
