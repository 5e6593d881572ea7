// lego_rosbag.hpp — ROS bag v2.0 reading and writing without ROS, for the front end's input side.
//
// The reference replays bags through rosbag::View (LeGO-LOAM/src/main.cpp:62-76) and hands every
// sensor_msgs/PointCloud2 to ImageProjection::cloudHandler, which decodes it with pcl::fromROSMsg
// (imageProjection.cpp:159-161).  Here:
//   * BagReader walks a bag file (format 2.0: records of {header fields, data}; chunks with
//     compression "none", "bz2" or "lz4") and calls back once per message of the wanted topic, in
//     file order (rosbag record writes chunks in time order);
//   * decode_pointcloud2 turns a serialized PointCloud2 into the zero-copy PointCloud2View that
//     lego_cloud_handler / ImageProjection::cloudHandler take (float32 x, y, z at field offsets);
//   * BagWriter writes a valid bag (bag header, chunks, connection / index / chunk-info records),
//     used to package synthetic or converted sweeps.
// bz2 / lz4 chunks are inflated with the system's libbz2.so.1 / liblz4.so.1, loaded at run time.
// Header-only C++14.  Errors throw lego_amd::BagError.
#pragma once

#include <dlfcn.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <functional>
#include <initializer_list>
#include <map>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "lego_loam_amd.hpp"

namespace lego_amd {

struct BagError : std::runtime_error {
  explicit BagError(const std::string& w) : std::runtime_error("rosbag: " + w) {}
};

// One decoded message's stamp and topic, plus its serialized bytes (valid during the callback).
struct BagMessage {
  std::string topic, type;
  uint32_t sec = 0, nsec = 0;
  const uint8_t* data = nullptr;
  size_t size = 0;
  double stamp() const { return sec + 1e-9 * nsec; }
};

namespace bagdetail {

inline uint32_t u32(const uint8_t* p) {
  uint32_t v;
  std::memcpy(&v, p, 4);
  return v;
}
inline uint64_t u64(const uint8_t* p) {
  uint64_t v;
  std::memcpy(&v, p, 8);
  return v;
}

// "name=value" fields of a record header (or of a connection header)
inline std::map<std::string, std::string> fields(const uint8_t* p, size_t n) {
  std::map<std::string, std::string> f;
  size_t i = 0;
  while (i + 4 <= n) {
    const uint32_t len = u32(p + i);
    i += 4;
    if (len > n - i) throw BagError("truncated header field");
    const char* s = (const char*)(p + i);
    const void* eq = std::memchr(s, '=', len);
    if (!eq) throw BagError("header field without '='");
    const size_t k = (const char*)eq - s;
    f[std::string(s, k)] = std::string(s + k + 1, len - k - 1);
    i += len;
  }
  return f;
}

inline uint32_t f32(const std::map<std::string, std::string>& f, const char* k) {
  auto it = f.find(k);
  if (it == f.end() || it->second.size() != 4) throw BagError(std::string("missing field ") + k);
  return u32((const uint8_t*)it->second.data());
}

// bz2 / lz4-frame inflation through the system libraries (no development headers needed)
inline void inflate(const std::string& how, const uint8_t* src, size_t n, std::vector<uint8_t>& dst, size_t out_size) {
  // a garbled size must not turn into a huge allocation (rosbag chunks are ~768 KB by default)
  if (how == "none" ? n != out_size : out_size > ((size_t)1 << 30)) throw BagError("implausible chunk size");
  dst.resize(out_size);
  if (how == "none") {
    std::memcpy(dst.data(), src, n);
    return;
  }
  if (how == "bz2") {
    static void* h = dlopen("libbz2.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) throw BagError("bz2 chunk but libbz2.so.1 is not available");
    typedef int (*fn_t)(char*, unsigned*, char*, unsigned, int, int);
    fn_t fn = (fn_t)dlsym(h, "BZ2_bzBuffToBuffDecompress");
    if (!fn) throw BagError("libbz2 without BZ2_bzBuffToBuffDecompress");
    unsigned out = (unsigned)out_size;
    if (fn((char*)dst.data(), &out, (char*)src, (unsigned)n, 0, 0) != 0 || out != out_size)
      throw BagError("bz2 inflate failed");
    return;
  }
  if (how == "lz4") {  // roslz4 writes the LZ4 frame format
    static void* h = dlopen("liblz4.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) throw BagError("lz4 chunk but liblz4.so.1 is not available");
    typedef size_t (*create_t)(void**, unsigned);
    typedef size_t (*free_t)(void*);
    typedef size_t (*dec_t)(void*, void*, size_t*, const void*, size_t*, const void*);
    typedef unsigned (*iserr_t)(size_t);
    create_t create = (create_t)dlsym(h, "LZ4F_createDecompressionContext");
    free_t destroy = (free_t)dlsym(h, "LZ4F_freeDecompressionContext");
    dec_t dec = (dec_t)dlsym(h, "LZ4F_decompress");
    iserr_t iserr = (iserr_t)dlsym(h, "LZ4F_isError");
    if (!create || !destroy || !dec || !iserr) throw BagError("liblz4 without the LZ4F frame API");
    void* ctx = nullptr;
    if (iserr(create(&ctx, 100 /* LZ4F_VERSION */))) throw BagError("lz4 context");
    size_t in_off = 0, out_off = 0;
    while (in_off < n && out_off < out_size) {
      size_t src_len = n - in_off, dst_len = out_size - out_off;
      const size_t r = dec(ctx, dst.data() + out_off, &dst_len, src + in_off, &src_len, nullptr);
      if (iserr(r)) {
        destroy(ctx);
        throw BagError("lz4 inflate failed");
      }
      in_off += src_len;
      out_off += dst_len;
      if (r == 0) break;
    }
    destroy(ctx);
    if (out_off != out_size) throw BagError("lz4 chunk size mismatch");
    return;
  }
  throw BagError("unsupported chunk compression '" + how + "'");
}

}  // namespace bagdetail

class BagReader {
 public:
  explicit BagReader(const std::string& path) {
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) throw BagError("cannot open " + path);
    std::fseek(f, 0, SEEK_END);
    const long n = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    buf_.resize(n > 0 ? (size_t)n : 0);
    const size_t got = n > 0 ? std::fread(buf_.data(), 1, buf_.size(), f) : 0;
    std::fclose(f);
    static const char magic[] = "#ROSBAG V2.0\n";
    if (got != buf_.size() || buf_.size() < 13 || std::memcmp(buf_.data(), magic, 13) != 0)
      throw BagError(path + " is not a ROS bag v2.0");
  }

  // Calls fn for every message on `topic` (all topics if empty), in file order.
  void for_each(const std::string& topic, const std::function<void(const BagMessage&)>& fn) {
    conns_.clear();
    walk(buf_.data() + 13, buf_.size() - 13, topic, fn, 0);
  }

  // topic -> message type, for every connection in the bag
  std::map<std::string, std::string> topics() {
    std::map<std::string, std::string> t;
    for_each("\x01", [](const BagMessage&) {});  // no topic has this name: connections only
    for (const auto& c : conns_) t[c.second.first] = c.second.second;
    return t;
  }

 private:
  std::vector<uint8_t> buf_;
  std::map<uint32_t, std::pair<std::string, std::string>> conns_;  // conn -> (topic, type)

  void walk(const uint8_t* p, size_t n, const std::string& topic, const std::function<void(const BagMessage&)>& fn,
            int depth) {
    using namespace bagdetail;
    size_t i = 0;
    while (i + 4 <= n) {
      const uint32_t hl = u32(p + i);
      if (hl > n - i - 4) throw BagError("truncated record header");
      const uint8_t* h = p + i + 4;
      const size_t di = i + 4 + hl;
      if (di + 4 > n) throw BagError("truncated record");
      const uint32_t dl = u32(p + di);
      if (dl > n - di - 4) throw BagError("truncated record data");
      const uint8_t* d = p + di + 4;
      const auto f = fields(h, hl);
      auto op = f.find("op");
      if (op == f.end() || op->second.size() != 1) throw BagError("record without op");
      switch ((uint8_t)op->second[0]) {
        case 0x05: {  // chunk
          if (depth > 0) throw BagError("nested chunk");
          auto c = f.find("compression");
          std::vector<uint8_t> raw;
          inflate(c == f.end() ? "none" : c->second, d, dl, raw, f32(f, "size"));
          walk(raw.data(), raw.size(), topic, fn, depth + 1);
          break;
        }
        case 0x07: {  // connection: topic in the record header, type in the connection header
          const uint32_t id = f32(f, "conn");
          const auto ch = fields(d, dl);
          auto t = f.find("topic");
          auto ty = ch.find("type");
          conns_[id] = std::make_pair(t == f.end() ? std::string() : t->second,
                                      ty == ch.end() ? std::string() : ty->second);
          break;
        }
        case 0x02: {  // message data
          const uint32_t id = f32(f, "conn");
          auto it = conns_.find(id);
          if (it == conns_.end()) throw BagError("message before its connection record");
          if (topic.empty() || topic == it->second.first) {
            auto tm = f.find("time");
            if (tm == f.end() || tm->second.size() != 8) throw BagError("message without time");
            BagMessage m;
            m.topic = it->second.first;
            m.type = it->second.second;
            m.sec = u32((const uint8_t*)tm->second.data());
            m.nsec = u32((const uint8_t*)tm->second.data() + 4);
            m.data = d;
            m.size = dl;
            fn(m);
          }
          break;
        }
        default:  // bag header (0x03), index data (0x04), chunk info (0x06): not needed to replay
          break;
      }
      i = di + 4 + dl;
    }
  }
};

// sensor_msgs/PointCloud2 (ROS1 serialization) -> the strided view of lego_cloud_handler.
// Requires float32 x, y, z fields (datatype 7, count 1) in a little-endian cloud.  The view points
// into `msg`'s bytes.  Throws BagError on anything else.
inline PointCloud2View decode_pointcloud2(const BagMessage& msg) {
  using namespace bagdetail;
  const uint8_t* p = msg.data;
  const size_t n = msg.size;
  size_t i = 0;
  auto need = [&](size_t k) {
    if (k > n - i) throw BagError("truncated PointCloud2");
  };
  auto rd32 = [&]() { need(4); uint32_t v = u32(p + i); i += 4; return v; };
  auto rdstr = [&]() { const uint32_t l = rd32(); need(l); std::string s((const char*)p + i, l); i += l; return s; };
  PointCloud2View v;
  rd32();  // header.seq
  const uint32_t sec = rd32(), nsec = rd32();
  rdstr();  // header.frame_id
  v.stamp = sec + 1e-9 * nsec;
  const uint32_t height = rd32(), width = rd32();
  const uint32_t nf = rd32();
  int ox = -1, oy = -1, oz = -1;
  for (uint32_t k = 0; k < nf; ++k) {
    const std::string name = rdstr();
    const uint32_t off = rd32();
    need(1);
    const uint8_t type = p[i++];
    const uint32_t count = rd32();
    const bool f32ok = type == 7 && count == 1;  // sensor_msgs/PointField FLOAT32
    if (name == "x" && f32ok) ox = (int)off;
    if (name == "y" && f32ok) oy = (int)off;
    if (name == "z" && f32ok) oz = (int)off;
  }
  need(1);
  if (p[i++] != 0) throw BagError("big-endian PointCloud2 not supported");
  const uint32_t point_step = rd32();
  rd32();  // row_step
  const uint32_t dl = rd32();
  need(dl);
  if (ox < 0 || oy < 0 || oz < 0) throw BagError("PointCloud2 without float32 x, y, z");
  for (const int o : {ox, oy, oz})  // every field inside the point (found by the sanitizer build's fuzz corpus)
    if ((uint64_t)(uint32_t)o + 4u > point_step) throw BagError("PointCloud2 field outside its point_step");
  const uint64_t npts = (uint64_t)height * width;
  if (npts * point_step > dl || npts > 0x7fffffffull) throw BagError("PointCloud2 data shorter than its points");
  v.data = p + i;
  v.width = (int32_t)npts;
  v.point_step = (int32_t)point_step;
  v.off_x = ox;
  v.off_y = oy;
  v.off_z = oz;
  return v;
}

// Writes a bag with one PointCloud2 topic (x, y, z, intensity float32, 16-byte points), chunked
// (compression "none"), with the index, connection and chunk-info records rosbag expects.
class BagWriter {
 public:
  BagWriter(const std::string& path, const std::string& topic, const std::string& frame_id = "velodyne",
            size_t chunk_threshold = 768 * 1024)
      : topic_(topic), frame_(frame_id), threshold_(chunk_threshold) {
    f_ = std::fopen(path.c_str(), "wb");
    if (!f_) throw BagError("cannot create " + path);
    std::fwrite("#ROSBAG V2.0\n", 1, 13, f_);
    header_pos_ = std::ftell(f_);
    write_bag_header(0, 0, 0);
  }
  ~BagWriter() {
    if (f_) close();
  }
  BagWriter(const BagWriter&) = delete;
  BagWriter& operator=(const BagWriter&) = delete;

  // one sweep: n points of (x, y, z, intensity)
  void write(double stamp, const float* xyzi, int32_t n) {
    const uint32_t sec = (uint32_t)stamp, nsec = (uint32_t)((stamp - sec) * 1e9 + 0.5);
    std::string m;
    put32(m, seq_++);
    put32(m, sec);
    put32(m, nsec);
    putstr(m, frame_);
    put32(m, 1);             // height
    put32(m, (uint32_t)n);   // width
    put32(m, 4);             // fields
    const char* names[4] = {"x", "y", "z", "intensity"};
    for (int k = 0; k < 4; ++k) {
      putstr(m, names[k]);
      put32(m, 4u * k);
      m.push_back((char)7);  // FLOAT32
      put32(m, 1);
    }
    m.push_back((char)0);    // is_bigendian
    put32(m, 16);            // point_step
    put32(m, 16u * (uint32_t)n);
    put32(m, 16u * (uint32_t)n);
    m.append((const char*)xyzi, (size_t)n * 16);
    m.push_back((char)1);    // is_dense
    if (chunk_.empty()) {
      chunk_start_ = ((uint64_t)nsec << 32) | sec;
      chunk_.append(conn_record());
    }
    const uint64_t t = ((uint64_t)nsec << 32) | sec;
    index_.push_back(std::make_pair(t, (uint32_t)chunk_.size()));
    std::string h;
    field(h, "op", std::string(1, '\x02'));
    field(h, "conn", u32s(0));
    field(h, "time", std::string((const char*)&t, 8));
    record(chunk_, h, m);
    chunk_end_ = t;
    if (chunk_.size() >= threshold_) flush_chunk();
  }

  void close() {
    flush_chunk();
    const uint64_t index_pos = (uint64_t)std::ftell(f_);
    std::string out = conn_record();
    for (const auto& ci : chunk_infos_) out += ci;
    std::fwrite(out.data(), 1, out.size(), f_);
    std::fseek(f_, header_pos_, SEEK_SET);
    write_bag_header(index_pos, 1, (uint32_t)chunk_infos_.size());
    std::fclose(f_);
    f_ = nullptr;
  }

 private:
  FILE* f_ = nullptr;
  std::string topic_, frame_, chunk_;
  size_t threshold_;
  long header_pos_ = 0;
  uint32_t seq_ = 0;
  uint64_t chunk_start_ = 0, chunk_end_ = 0;
  std::vector<std::pair<uint64_t, uint32_t>> index_;
  std::vector<std::string> chunk_infos_;

  static void put32(std::string& s, uint32_t v) { s.append((const char*)&v, 4); }
  static void putstr(std::string& s, const std::string& v) { put32(s, (uint32_t)v.size()); s += v; }
  static std::string u32s(uint32_t v) { return std::string((const char*)&v, 4); }
  static std::string u64s(uint64_t v) { return std::string((const char*)&v, 8); }
  static void field(std::string& h, const std::string& k, const std::string& v) {
    put32(h, (uint32_t)(k.size() + 1 + v.size()));
    h += k;
    h += '=';
    h += v;
  }
  static void record(std::string& out, const std::string& h, const std::string& d) {
    put32(out, (uint32_t)h.size());
    out += h;
    put32(out, (uint32_t)d.size());
    out += d;
  }
  std::string conn_record() const {
    std::string h, d, r;
    field(h, "op", std::string(1, '\x07'));
    field(h, "conn", u32s(0));
    field(h, "topic", topic_);
    field(d, "topic", topic_);
    field(d, "type", "sensor_msgs/PointCloud2");
    field(d, "md5sum", "1158d486dd51d683ce2f1be655c3c181");
    field(d, "message_definition", "");
    record(r, h, d);
    return r;
  }
  void write_bag_header(uint64_t index_pos, uint32_t conns, uint32_t chunks) {
    std::string h, r;
    field(h, "op", std::string(1, '\x03'));
    field(h, "index_pos", u64s(index_pos));
    field(h, "conn_count", u32s(conns));
    field(h, "chunk_count", u32s(chunks));
    const size_t pad = 4096 - 4 - h.size() - 4;  // the bag header record is padded to 4 KiB
    record(r, h, std::string(pad, ' '));
    std::fwrite(r.data(), 1, r.size(), f_);
  }
  void flush_chunk() {
    if (chunk_.empty()) return;
    const uint64_t chunk_pos = (uint64_t)std::ftell(f_);
    std::string h, out;
    field(h, "op", std::string(1, '\x05'));
    field(h, "compression", "none");
    field(h, "size", u32s((uint32_t)chunk_.size()));
    record(out, h, chunk_);
    std::string ih, id;  // index data for the chunk's one connection
    field(ih, "op", std::string(1, '\x04'));
    field(ih, "ver", u32s(1));
    field(ih, "conn", u32s(0));
    field(ih, "count", u32s((uint32_t)index_.size()));
    for (const auto& e : index_) {
      id += u64s(e.first);
      id += u32s(e.second);
    }
    record(out, ih, id);
    std::fwrite(out.data(), 1, out.size(), f_);
    std::string ch, cd, ci;
    field(ch, "op", std::string(1, '\x06'));
    field(ch, "ver", u32s(1));
    field(ch, "chunk_pos", u64s(chunk_pos));
    field(ch, "start_time", u64s(chunk_start_));
    field(ch, "end_time", u64s(chunk_end_));
    field(ch, "count", u32s(1));
    cd += u32s(0);
    cd += u32s((uint32_t)index_.size());
    record(ci, ch, cd);
    chunk_infos_.push_back(ci);
    chunk_.clear();
    index_.clear();
  }
};

}  // namespace lego_amd
