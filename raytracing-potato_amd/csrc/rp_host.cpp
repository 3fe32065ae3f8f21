// rp_host.cpp -- librp_host.so: host-side loaders and helpers (include/rp_host.h).
#include "../../include/rp_host.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "rp_bvh.h"
#include "rp_kernel.h"

namespace {

thread_local std::string g_err;

int fail(const std::string& m) {
  g_err = m;
  return RP_EINVAL;
}

// ---- OBJ (mesh.rs:39-183) ------------------------------------------------------------------------

struct Cursor {
  const char* p;
};

bool space1(Cursor& c) {  // nom space1: one or more ' ' / '\t'
  if (*c.p != ' ' && *c.p != '\t') return false;
  while (*c.p == ' ' || *c.p == '\t') c.p++;
  return true;
}

// nom 7 number::complete::double: sign, digits, '.', digits, exponent; or inf/infinity/nan.
bool number(Cursor& c, double& out) {
  const char* s = c.p;
  const char* q = s;
  if (*q == '+' || *q == '-') q++;
  for (const char* w : {"infinity", "inf", "nan"}) {
    size_t n = std::strlen(w);
    if (strncasecmp(q, w, n) == 0) {
      std::string tok(s, (size_t)(q - s) + n);
      out = std::strtod(tok.c_str(), nullptr);
      c.p = q + n;
      return true;
    }
  }
  int digits = 0;
  while (*q >= '0' && *q <= '9') q++, digits++;
  if (*q == '.') {
    q++;
    while (*q >= '0' && *q <= '9') q++, digits++;
  }
  if (!digits) return false;
  if (*q == 'e' || *q == 'E') {
    const char* e = q + 1;
    if (*e == '+' || *e == '-') e++;
    if (*e >= '0' && *e <= '9') {
      while (*e >= '0' && *e <= '9') e++;
      q = e;
    }
  }
  std::string tok(s, (size_t)(q - s));
  out = std::strtod(tok.c_str(), nullptr);  // correctly rounded, as Rust's str::parse::<f64>
  c.p = q;
  return true;
}

struct ObjIndex {
  uint32_t p;
  int64_t n, t;  // -1 = None
  bool operator==(const ObjIndex& o) const { return p == o.p && n == o.n && t == o.t; }
};
struct ObjIndexHash {
  size_t operator()(const ObjIndex& k) const {
    uint64_t h = (uint64_t)k.p * 0x9E3779B97F4A7C15ull;
    h ^= (uint64_t)(k.n + 1) * 0xBF58476D1CE4E5B9ull + (h << 6) + (h >> 2);
    h ^= (uint64_t)(k.t + 1) * 0x94D049BB133111EBull + (h << 6) + (h >> 2);
    return (size_t)h;
  }
};

// parse_index (mesh.rs:59-71): separated_list1(tag("/"), opt(integer)).
// Returns 1 ok, 0 "position index not provided" (the face parser stops), -1 fatal (index 0 underflow).
int parse_index(Cursor& c, ObjIndex& out) {
  std::vector<int64_t> vals;
  const char* q = c.p;
  for (;;) {
    uint64_t v = 0;
    int nd = 0;
    bool ovf = false;
    while (*q >= '0' && *q <= '9') {
      v = v * 10 + (uint64_t)(*q - '0');
      if (v > 0xffffffffull) ovf = true;
      q++, nd++;
    }
    vals.push_back(nd && !ovf ? (int64_t)v : -1);
    if (*q == '/') {
      q++;
      continue;
    }
    break;
  }
  if (vals[0] < 0) return 0;
  auto conv = [](int64_t v, int64_t& o) -> bool {
    if (v < 0) { o = -1; return true; }
    if (v == 0) return false;  // `x - 1` on u32 0: the reference panics
    o = v - 1;
    return true;
  };
  int64_t p;
  if (!conv(vals[0], p)) return -1;
  out.p = (uint32_t)p;
  out.t = -1;
  out.n = -1;
  if (vals.size() > 1 && !conv(vals[1], out.t)) return -1;
  if (vals.size() > 2 && !conv(vals[2], out.n)) return -1;
  c.p = q;
  return 1;
}

// ---- sky panorama --------------------------------------------------------------------------------

double hash01(int64_t x, int64_t y, int64_t seed) {
  // randomness.rs noise::integer restated, mapped to [0, 1)
  uint64_t h = 0x369E6D3B899E43CFull * (uint64_t)x + 0x53F89E7FFDA3B07Dull * (uint64_t)y +
               0x577C2C6E4019D645ull * (uint64_t)seed;
  h = (uint64_t)((int64_t)h >> 13) ^ h;
  h = h * (h * h * 60493ull + 19990303ull) + 1376312589ull;
  return (double)(h >> 11) * (1.0 / 9007199254740992.0);
}

double smooth(double t) { return t * t * (3.0 - 2.0 * t); }

// Value noise on a lattice that wraps horizontally every `period` cells (seamless at u = 0 / 1).
double value_noise(double x, double y, int64_t period, int64_t seed) {
  double fx = std::floor(x), fy = std::floor(y);
  int64_t ix = (int64_t)fx, iy = (int64_t)fy;
  double tx = smooth(x - fx), ty = smooth(y - fy);
  auto w = [&](int64_t a) { return ((a % period) + period) % period; };
  double a = hash01(w(ix), iy, seed), b = hash01(w(ix + 1), iy, seed);
  double c = hash01(w(ix), iy + 1, seed), d = hash01(w(ix + 1), iy + 1, seed);
  double ab = a + (b - a) * tx, cd = c + (d - c) * tx;
  return ab + (cd - ab) * ty;
}

uint8_t quant(double x) {
  if (!(x > 0.0)) return 0;
  if (x >= 1.0) return 255;
  return (uint8_t)(x * 255.0 + 0.5);
}

}  // namespace

extern "C" {

const char* rph_last_error(void) { return g_err.c_str(); }

void rph_free(void* p) { std::free(p); }

void rph_mesh_free(rph_mesh* m) {
  if (!m) return;
  std::free(m->positions);
  std::free(m->normals);
  std::free(m->uvs);
  std::free(m->indices);
  std::memset(m, 0, sizeof *m);
}

int rph_obj_load(const char* path, rph_mesh* out) {
  if (!out || !path) return fail("NULL argument");
  std::memset(out, 0, sizeof *out);
  std::ifstream f(path, std::ios::binary);
  if (!f) return fail(std::string("cannot open ") + path);
  std::vector<double> P, N, T;
  std::vector<ObjIndex> verts;
  std::vector<std::pair<uint32_t, uint32_t>> faces;  // first vertex, count
  std::string line;
  while (std::getline(f, line)) {
    while (!line.empty() && (line.back() == '\r' || line.back() == '\n')) line.pop_back();
    Cursor c{line.c_str()};
    double v[3];
    // alt((v, vn, vt, f)) (mesh.rs:88-95); a line none of them parses is skipped (mesh.rs:117-120)
    if (c.p[0] == 'v' && (c.p[1] == ' ' || c.p[1] == '\t')) {
      c.p += 1;
      if (space1(c) && number(c, v[0]) && space1(c) && number(c, v[1]) && space1(c) && number(c, v[2]))
        P.insert(P.end(), v, v + 3);
    } else if (c.p[0] == 'v' && c.p[1] == 'n') {
      c.p += 2;
      if (space1(c) && number(c, v[0]) && space1(c) && number(c, v[1]) && space1(c) && number(c, v[2]))
        N.insert(N.end(), v, v + 3);
    } else if (c.p[0] == 'v' && c.p[1] == 't') {
      c.p += 2;
      if (space1(c) && number(c, v[0]) && space1(c) && number(c, v[1])) T.insert(T.end(), v, v + 2);
    } else if (c.p[0] == 'f') {
      c.p += 1;
      if (!space1(c)) continue;
      ObjIndex idx;
      int r = parse_index(c, idx);
      if (r < 0) return fail("face index 0 (1-based indices underflow)");
      if (r == 0) continue;
      uint32_t first = (uint32_t)verts.size(), cnt = 0;
      for (;;) {
        verts.push_back(idx);
        cnt++;
        Cursor save = c;
        if (!space1(c)) break;
        r = parse_index(c, idx);
        if (r < 0) return fail("face index 0 (1-based indices underflow)");
        if (r == 0) {
          c = save;
          break;
        }
      }
      faces.emplace_back(first, cnt);
    }
  }
  // mesh.rs:151-166: unique (p, n, t) tuples in first-use order
  std::unordered_map<ObjIndex, uint32_t, ObjIndexHash> uniq;
  uniq.reserve(verts.size() * 2 + 1);
  std::vector<uint32_t> remap(verts.size());
  std::vector<double> pos, nrm, uv;
  for (size_t k = 0; k < verts.size(); k++) {
    const ObjIndex& key = verts[k];
    auto it = uniq.find(key);
    if (it == uniq.end()) {
      if ((size_t)key.p * 3 >= P.size() || (key.n >= 0 && (size_t)key.n * 3 >= N.size()) ||
          (key.t >= 0 && (size_t)key.t * 2 >= T.size()))
        return fail("face references a missing v/vn/vt (index out of bounds)");
      uint32_t id = (uint32_t)(pos.size() / 3);
      uniq.emplace(key, id);
      pos.insert(pos.end(), &P[3 * (size_t)key.p], &P[3 * (size_t)key.p] + 3);
      if (key.n >= 0) nrm.insert(nrm.end(), &N[3 * (size_t)key.n], &N[3 * (size_t)key.n] + 3);
      else nrm.insert(nrm.end(), {0.0, 0.0, 0.0});
      if (key.t >= 0) uv.insert(uv.end(), &T[2 * (size_t)key.t], &T[2 * (size_t)key.t] + 2);
      else uv.insert(uv.end(), {0.0, 0.0});
      remap[k] = id;
    } else {
      remap[k] = it->second;
    }
  }
  std::vector<uint32_t> indices;
  indices.reserve(faces.size() * 3);
  for (auto& fc : faces) {
    if (fc.second != 3) return fail("Non-triangular face are not supported");  // mesh.rs:170-172
    for (uint32_t q = 0; q < 3; q++) indices.push_back(remap[fc.first + q]);
  }
  uint32_t nv = (uint32_t)(pos.size() / 3);
  out->n_vertices = nv;
  out->n_indices = (uint32_t)indices.size();
  out->positions = (double*)std::malloc(sizeof(double) * (pos.size() + 1));
  out->normals = (double*)std::malloc(sizeof(double) * (nrm.size() + 1));
  out->uvs = (double*)std::malloc(sizeof(double) * (uv.size() + 1));
  out->indices = (uint32_t*)std::malloc(sizeof(uint32_t) * (indices.size() + 1));
  if (!out->positions || !out->normals || !out->uvs || !out->indices) {
    rph_mesh_free(out);
    return fail("out of memory");
  }
  if (!pos.empty()) std::memcpy(out->positions, pos.data(), sizeof(double) * pos.size());
  if (!nrm.empty()) std::memcpy(out->normals, nrm.data(), sizeof(double) * nrm.size());
  if (!uv.empty()) std::memcpy(out->uvs, uv.data(), sizeof(double) * uv.size());
  if (!indices.empty()) std::memcpy(out->indices, indices.data(), sizeof(uint32_t) * indices.size());
  return RP_OK;
}

int rph_tga_load(const char* path, uint32_t* width, uint32_t* height, uint8_t** rgba) {
  if (!path || !width || !height || !rgba) return fail("NULL argument");
  std::ifstream f(path, std::ios::binary);
  if (!f) return fail(std::string("cannot open ") + path);
  uint8_t hd[18];
  if (!f.read(reinterpret_cast<char*>(hd), 18)) return fail("truncated TGA header");
  const uint32_t w = hd[12] | (hd[13] << 8), h = hd[14] | (hd[15] << 8);
  const uint8_t bpp = hd[16], desc = hd[17];
  // image.rs:81-88
  if (hd[0] != 0 || hd[1] != 0 || hd[2] != 2 || (bpp != 24 && bpp != 32))
    return fail("This tga header is not supported");
  const size_t bytes = (size_t)w * h * (bpp / 8);
  std::vector<uint8_t> raw(bytes);
  if (bytes && !f.read(reinterpret_cast<char*>(raw.data()), (std::streamsize)bytes)) return fail("truncated TGA data");
  uint8_t* img = (uint8_t*)std::malloc((size_t)w * h * 4 + 1);
  if (!img) return fail("out of memory");
  const size_t step = bpp / 8;
  for (uint32_t y0 = 0; y0 < h; y0++) {
    const uint32_t y = (desc & (1 << 5)) ? h - 1 - y0 : y0;  // image.rs:95-99 (top-left origin -> flip)
    for (uint32_t x = 0; x < w; x++) {
      const uint8_t* s = &raw[((size_t)y0 * w + x) * step];
      uint8_t* o = img + 4 * ((size_t)x + (size_t)y * w);
      o[0] = s[2];
      o[1] = s[1];
      o[2] = s[0];
      o[3] = bpp == 32 ? s[3] : 0xff;
    }
  }
  *width = w;
  *height = h;
  *rgba = img;
  return RP_OK;
}

int rph_tga_save(const char* path, uint32_t width, uint32_t height, const uint8_t* rgba) {
  if (!path || (!rgba && (uint64_t)width * height != 0)) return fail("NULL argument");
  if (width > 65535 || height > 65535) return fail("image too large for a TGA header (u16 try_into)");
  std::ofstream f(path, std::ios::binary);
  if (!f) return fail(std::string("cannot create ") + path);
  uint8_t hd[18] = {0};
  hd[2] = 2;
  hd[16] = 32;
  hd[12] = (uint8_t)width;
  hd[13] = (uint8_t)(width >> 8);
  hd[14] = (uint8_t)height;
  hd[15] = (uint8_t)(height >> 8);
  f.write(reinterpret_cast<const char*>(hd), 18);
  std::vector<uint8_t> row((size_t)width * 4);
  for (uint32_t y = 0; y < height; y++) {
    for (uint32_t x = 0; x < width; x++) {
      const uint8_t* p = rgba + 4 * ((size_t)x + (size_t)y * width);
      row[4 * x] = p[2];
      row[4 * x + 1] = p[1];
      row[4 * x + 2] = p[0];
      row[4 * x + 3] = p[3];
    }
    f.write(reinterpret_cast<const char*>(row.data()), (std::streamsize)row.size());
  }
  return f ? RP_OK : fail("write failed");
}

void rph_to_srgb_u8(const double* rgb, uint64_t n, uint8_t* rgba) {
  for (uint64_t i = 0; i < n; i++) {
    for (int c = 0; c < 3; c++) {
      double x = rgb[3 * i + c];
      if (x < 0.0) x = 0.0;  // f64::clamp keeps NaN; powf(NaN) = NaN; `as u8` maps NaN to 0
      if (x > 1.0) x = 1.0;
      double y = 255.0 * std::pow(x, 1.0 / 2.2);
      rgba[4 * i + c] = !(y > 0.0) ? 0 : (y >= 255.0 ? 255 : (uint8_t)y);
    }
    rgba[4 * i + 3] = 0xff;
  }
}

void rph_lookat(const double position[3], const double target[3], const double up[3], double orientation[9]) {
  double z[3] = {position[0] - target[0], position[1] - target[1], position[2] - target[2]};
  const double n = std::sqrt((z[0] * z[0] + z[1] * z[1]) + z[2] * z[2]);
  for (double& c : z) c = c / n;
  const double x[3] = {up[1] * z[2] - up[2] * z[1], up[2] * z[0] - up[0] * z[2], up[0] * z[1] - up[1] * z[0]};
  const double y[3] = {z[1] * x[2] - z[2] * x[1], z[2] * x[0] - z[0] * x[2], z[0] * x[1] - z[1] * x[0]};
  for (int k = 0; k < 3; k++) {
    orientation[k] = x[k];
    orientation[3 + k] = y[k];
    orientation[6 + k] = z[k];
  }
}

int rph_sky_panorama(uint32_t width, uint32_t height, uint8_t* rgba) {
  if (!rgba || width == 0 || height == 0) return fail("bad arguments");
  const double sun_u = 0.30, sun_v = 0.78;  // azimuth / elevation of the sun in texture space
  for (uint32_t j = 0; j < height; j++) {
    const double v = ((double)j + 0.5) / (double)height;  // 0 = nadir, 1 = zenith
    for (uint32_t i = 0; i < width; i++) {
      const double u = ((double)i + 0.5) / (double)width;
      double r, g, b;
      if (v >= 0.5) {
        const double t = (v - 0.5) * 2.0;  // horizon -> zenith
        const double s = std::sqrt(t);
        r = 0.92 + (0.22 - 0.92) * s;
        g = 0.95 + (0.42 - 0.95) * s;
        b = 1.00 + (0.85 - 1.00) * s;
        // clouds: two octaves of horizontally seamless value noise, thinning towards the zenith
        const double x = u * 24.0, y = v * 12.0;
        double c = 0.65 * value_noise(x, y, 24, 7) + 0.35 * value_noise(2.0 * x, 2.0 * y, 48, 11);
        c = (c - 0.55) * 4.0;
        if (c < 0.0) c = 0.0;
        if (c > 1.0) c = 1.0;
        c = c * (1.0 - t * 0.6);
        r = r + (1.0 - r) * c;
        g = g + (1.0 - g) * c;
        b = b + (1.0 - b) * c;
      } else {
        const double t = (0.5 - v) * 2.0;  // horizon -> nadir
        r = 0.42 - 0.22 * t;
        g = 0.38 - 0.20 * t;
        b = 0.33 - 0.18 * t;
        const double gr = value_noise(u * 96.0, v * 48.0, 96, 3);
        r = r * (0.85 + 0.3 * gr);
        g = g * (0.85 + 0.3 * gr);
        b = b * (0.85 + 0.3 * gr);
      }
      // sun disc + halo (u spans 2*pi, v spans pi: weight du by 2)
      double du = u - sun_u;
      if (du > 0.5) du -= 1.0;
      if (du < -0.5) du += 1.0;
      const double dist2 = (2.0 * du) * (2.0 * du) + (v - sun_v) * (v - sun_v);
      if (dist2 < 0.0004) {
        r = 1.0; g = 0.97; b = 0.88;
      } else {
        const double halo = 0.0012 / (dist2 + 0.0012);
        r = r + (1.0 - r) * halo * 0.8;
        g = g + (0.95 - g) * halo * 0.8;
        b = b + (0.8 - b) * halo * 0.8;
      }
      uint8_t* o = rgba + 4 * ((size_t)j * width + i);
      o[0] = quant(r);
      o[1] = quant(g);
      o[2] = quant(b);
      o[3] = 0xff;
    }
  }
  return RP_OK;
}

int rph_bvh_traversal_stats(const rp_scene_desc* desc, const double* rays, uint64_t n, uint32_t node_format,
                            uint64_t* per_ray) {
  return rph_bvh_traversal_stats_ex(desc, rays, n, node_format, RP_COLLAPSE_AUTO, per_ray);
}

int rph_bvh_traversal_stats_ex(const rp_scene_desc* desc, const double* rays, uint64_t n, uint32_t node_format,
                               uint32_t collapse, uint64_t* per_ray) {
  // CPU model of rp_device.h's traversal over the same packed 4-wide tree: child boxes tested in f32 with
  // per-axis outward bounds (t = fma(P, inv, nb|fb), quantized: fma(q, s inv, fma(o, inv, nb|fb))), rcp
  // emulated by a correctly rounded 1/x, the min/max slab form instead of the device's octant selection
  // (the same values), near-first order, exact f64
  // primitive tests.  per_ray: n x 3 {wide nodes visited, primitive tests, closest hittable id or
  // 2^64-1}.  tests/test_bvh.py checks the closest hits against brute force.
  std::string err;
  int rc = rpb::validate(desc, err);
  if (rc != RP_OK) return fail(err);
  rpb::PackedScene ps;
  rpb::BuildOptions bo;
  bo.node_format = node_format;
  bo.collapse = collapse == RP_COLLAPSE_GREEDY ? rpb::COLLAPSE_GREEDY : rpb::COLLAPSE_SAH;
  rc = rpb::build(desc, bo, ps, err);
  if (rc != RP_OK) return fail(err);
  const bool q8 = ps.node_format != rpl::NODES_F32;  // Node4Q or Node8Q: the frame term
  const bool w8 = ps.node_format == rpl::NODES_W8;
  auto down = [](double x) { float f = (float)x; if ((double)f > x) f = std::nextafter(f, -INFINITY); return f; };
  auto up = [](double x) { float f = (float)x; if ((double)f < x) f = std::nextafter(f, INFINITY); return f; };
  for (uint64_t r = 0; r < n; r++) {
    const double* q = rays + 8 * r;
    const double o[3] = {q[0], q[1], q[2]}, d[3] = {q[3], q[4], q[5]};
    const double tmin = q[6];
    float inv[3], nb[3], fb[3];  // per axis: slope, near- and far-plane addends (rp_device.h setup_ray32)
    for (int k = 0; k < 3; k++) {
      const float o32 = (float)o[k];
      inv[k] = std::fmin(std::fmax(1.0f / (float)d[k], -0x1p64f), 0x1p64f);
      const float oinv = o32 * inv[k];
      const double e = std::fabs(o[k] - (double)o32);
      const double Dk = ((e == 0.0 ? 0.0 : e * std::fabs((double)inv[k]) * (1.0 + 0x1p-20)) + std::fabs((double)oinv) * 0x1p-23 +
                         ((!q8 || (std::fabs(inv[k]) == 0x1p64f && o32 == 0.0f))
                              ? 0.0
                              : std::fabs((double)inv[k]) * (2.0 * ps.qbound + std::fabs((double)o32)) * 0x1p-23 * (1.0 + 0x1p-20))) *
                        (1.0 + 0x1p-20);
      nb[k] = down(-(double)oinv - Dk);
      fb[k] = up(-(double)oinv + Dk);
    }
    const float tmin32 = down(tmin);
    double best = q[7];
    float best32 = up(best);
    int64_t bestp = -1;
    uint64_t visits = 0, tests = 0;
    auto test = [&](uint32_t k) {
      tests++;
      const rpl::Prim& p = ps.prims[k];
      if (p.kind == rpl::PRIM_TRIANGLE) {
        const double* g = p.g;
        const double pa[3] = {g[0] - o[0], g[1] - o[1], g[2] - o[2]};
        const double ba[3] = {g[3], g[4], g[5]}, ca[3] = {g[6], g[7], g[8]};
        double det = ba[0] * ca[1] * d[2] + ba[1] * ca[2] * d[0] + ba[2] * ca[0] * d[1] - ba[0] * ca[2] * d[1] -
                     ba[1] * ca[0] * d[2] - ba[2] * ca[1] * d[0];
        if (std::fabs(det) < 1e-7) return;
        double inv_det = 1.0 / det;
        double t = (pa[0] * (ba[1] * ca[2] - ba[2] * ca[1]) + pa[1] * (ba[2] * ca[0] - ba[0] * ca[2]) +
                    pa[2] * (ba[0] * ca[1] - ba[1] * ca[0])) * inv_det;
        double u = (pa[0] * (ca[1] * d[2] - ca[2] * d[1]) + pa[1] * (ca[2] * d[0] - ca[0] * d[2]) +
                    pa[2] * (ca[0] * d[1] - ca[1] * d[0])) * inv_det;
        double v = (pa[0] * (ba[2] * d[1] - ba[1] * d[2]) + pa[1] * (ba[0] * d[2] - ba[2] * d[0]) +
                    pa[2] * (ba[1] * d[0] - ba[0] * d[1])) * inv_det;
        double w = 1.0 - u - v;
        if (t < tmin || t > best || u < 0.0 || v < 0.0 || w < 0.0) return;
        best = t;
        bestp = ps.prim_refs[k].src;
      } else {
        const double tc[3] = {o[0] - p.g[0], o[1] - p.g[1], o[2] - p.g[2]};
        double a = (d[0] * d[0] + d[1] * d[1]) + d[2] * d[2];
        double hb = (d[0] * tc[0] + d[1] * tc[1]) + d[2] * tc[2];
        double cq = ((tc[0] * tc[0] + tc[1] * tc[1]) + tc[2] * tc[2]) - p.g[3] * p.g[3];
        double delta = hb * hb - a * cq;
        if (delta <= 0.0) return;
        double sq = std::sqrt(delta);
        double t = (-hb - sq) / a;
        if (t < tmin || t > best) {
          t = (-hb + sq) / a;
          if (t < tmin || t > best) return;
        }
        best = t;
        bestp = ps.prim_refs[k].src;
      }
      best32 = up(best);
    };
    // the always-tested primitives first (rp_bvh.h BuildOptions::always_max), as the kernel does
    for (uint32_t k = ps.always_first; k < ps.always_first + ps.n_always; k++) test(k);
    if (w8) {
      // 8-wide: children in rank order slot ^ octant; a stack of groups {family index | imask, rank bits}; the
      // leaf children's primitives are tested when their node is visited (the kernel parks them, same hits)
      const uint32_t oct = (d[0] < 0.0 ? 1u : 0u) | (d[1] < 0.0 ? 2u : 0u) | (d[2] < 0.0 ? 4u : 0u);
      std::vector<std::pair<uint32_t, uint32_t>> groups;  // {inner word, remaining rank bits}
      auto visit = [&](uint32_t node) {
        visits++;
        const rpl::Node8Q& nd = ps.wnodes[node];
        float A[3], Bn[3], Bf[3];
        for (int k = 0; k < 3; k++) {
          A[k] = nd.s[k] * inv[k];
          Bn[k] = std::fma(nd.o[k], inv[k], nb[k]);
          Bf[k] = std::fma(nd.o[k], inv[k], fb[k]);
        }
        const uint8_t* L[3] = {nd.lo_x, nd.lo_y, nd.lo_z};
        const uint8_t* H[3] = {nd.hi_x, nd.hi_y, nd.hi_z};
        uint32_t hits = 0;
        for (int c = 0; c < 8; c++) {
          float tnear = tmin32, tfar = best32;
          for (int k = 0; k < 3; k++) {
            const float a = std::fma((float)L[k][c], A[k], Bn[k]), b = std::fma((float)H[k][c], A[k], Bn[k]);
            const float a2 = std::fma((float)L[k][c], A[k], Bf[k]), b2 = std::fma((float)H[k][c], A[k], Bf[k]);
            tnear = std::fmax(tnear, std::fmin(a, b));
            tfar = std::fmin(tfar, std::fmax(a2, b2));
          }
          if (std::fma(tnear, 1.0f - 0x1p-19f, -0x1p-100f) <= tfar) hits |= 1u << c;
        }
        uint32_t pm = 0;
        for (int c = 0; c < 8; c++)
          if (hits >> c & 1u) pm |= nd.pmask[c];
        for (; pm; pm &= pm - 1u) test(nd.prim + (uint32_t)__builtin_ctz(pm));
        const uint32_t ih = hits & (nd.inner >> 24);
        uint32_t ranks = 0;
        for (int c = 0; c < 8; c++)
          if (ih >> c & 1u) ranks |= 1u << (c ^ oct);
        if (ranks) groups.push_back({nd.inner, ranks});
      };
      visit(ps.root);
      while (!groups.empty()) {
        auto& g = groups.back();
        const uint32_t rk = (uint32_t)__builtin_ctz(g.second), slot = rk ^ oct, word = g.first;
        g.second &= g.second - 1u;
        if (!g.second) groups.pop_back();
        visit((word & rpl::W8_INDEX) + (uint32_t)__builtin_popcount((word >> 24) & ((1u << slot) - 1u)));
      }
      per_ray[3 * r] = visits;
      per_ray[3 * r + 1] = tests;
      per_ray[3 * r + 2] = bestp < 0 ? ~0ull : (uint64_t)bestp;
      continue;
    }
    std::vector<uint32_t> stack;
    uint32_t cur = ps.root;
    for (;;) {
      while (!(cur & rpl::ENTRY_LEAF)) {
        visits++;
        const uint32_t* child;
        float near4[4][3], far4[4][3];  // per child and axis: both planes with the near / far addend
        if (q8) {
          const rpl::Node4Q& nd = ps.qnodes[cur];
          float A[3], Bn[3], Bf[3];
          for (int k = 0; k < 3; k++) {
            A[k] = nd.s[k] * inv[k];
            Bn[k] = std::fma(nd.o[k], inv[k], nb[k]);
            Bf[k] = std::fma(nd.o[k], inv[k], fb[k]);
          }
          const uint8_t* L[3] = {nd.lo_x, nd.lo_y, nd.lo_z};
          const uint8_t* H[3] = {nd.hi_x, nd.hi_y, nd.hi_z};
          // plane t values directly: t = fma(q, A, B) (the device's dequantized form)
          for (int c = 0; c < 4; c++)
            for (int k = 0; k < 3; k++) {
              const float a = std::fma((float)L[k][c], A[k], Bn[k]), b = std::fma((float)H[k][c], A[k], Bn[k]);
              const float a2 = std::fma((float)L[k][c], A[k], Bf[k]), b2 = std::fma((float)H[k][c], A[k], Bf[k]);
              near4[c][k] = std::fmin(a, b);
              far4[c][k] = std::fmax(a2, b2);
            }
          child = nd.child;
        } else {
          const rpl::Node4& nd = ps.nodes[cur];
          const float* lo[3] = {nd.lo_x, nd.lo_y, nd.lo_z};
          const float* hi[3] = {nd.hi_x, nd.hi_y, nd.hi_z};
          for (int c = 0; c < 4; c++)
            for (int k = 0; k < 3; k++) {
              const float a = std::fma(lo[k][c], inv[k], nb[k]), b = std::fma(hi[k][c], inv[k], nb[k]);
              const float a2 = std::fma(lo[k][c], inv[k], fb[k]), b2 = std::fma(hi[k][c], inv[k], fb[k]);
              near4[c][k] = std::fmin(a, b);
              far4[c][k] = std::fmax(a2, b2);
            }
          child = nd.child;
        }
        float tn[4];
        uint32_t cc[4];
        for (int c = 0; c < 4; c++) {
          float tnear = tmin32, tfar = best32;
          for (int k = 0; k < 3; k++) {
            tnear = std::fmax(tnear, near4[c][k]);
            tfar = std::fmin(tfar, far4[c][k]);
          }
          const bool hit = std::fma(tnear, 1.0f - 0x1p-19f, -0x1p-100f) <= tfar && child[c] != rpl::ENTRY_EMPTY;
          tn[c] = hit ? tnear : INFINITY;
          cc[c] = child[c];
        }
        for (int a = 0; a < 4; a++)  // stable sort by tn (matches the device network for distinct keys)
          for (int b = a + 1; b < 4; b++)
            if (tn[b] < tn[a]) { std::swap(tn[a], tn[b]); std::swap(cc[a], cc[b]); }
        for (int c = 3; c >= 1; c--)
          if (tn[c] != INFINITY) stack.push_back(cc[c]);
        if (tn[0] != INFINITY) cur = cc[0];
        else if (stack.empty()) cur = rpl::ENTRY_EMPTY;
        else { cur = stack.back(); stack.pop_back(); }
      }
      if (cur == rpl::ENTRY_EMPTY) break;
      const uint32_t first = cur & rpl::LEAF_FIRST_MASK, cnt = ((cur >> rpl::LEAF_SHIFT) & 7u) + 1u;
      for (uint32_t k = first; k < first + cnt; k++) test(k);
      if (stack.empty()) cur = rpl::ENTRY_EMPTY;
      else { cur = stack.back(); stack.pop_back(); }
    }
    per_ray[3 * r] = visits;
    per_ray[3 * r + 1] = tests;
    per_ray[3 * r + 2] = bestp < 0 ? ~0ull : (uint64_t)bestp;
  }
  return RP_OK;
}

int rph_bvh_selfcheck(const rp_scene_desc* desc, uint32_t node_format, uint64_t* stats) {
  return rph_bvh_selfcheck_ex(desc, node_format, RP_COLLAPSE_AUTO, stats);
}

int rph_bvh_selfcheck_ex(const rp_scene_desc* desc, uint32_t node_format, uint32_t collapse, uint64_t* stats) {
  std::string err;
  int rc = rpb::validate(desc, err);
  if (rc != RP_OK) return fail(err);
  rpb::PackedScene ps;
  rpb::BuildOptions bo;
  bo.node_format = node_format;
  bo.collapse = collapse == RP_COLLAPSE_GREEDY ? rpb::COLLAPSE_GREEDY : rpb::COLLAPSE_SAH;
  rc = rpb::build(desc, bo, ps, err);
  if (rc != RP_OK) return fail(err);
  rc = rpb::check(ps, err);
  if (rc != RP_OK) {
    g_err = err;
    return rc;
  }
  if (stats) {
    stats[0] = ps.n_nodes();
    stats[1] = ps.n_leaves;
    stats[2] = ps.max_depth;
    stats[3] = desc->n_hittables;
  }
  return RP_OK;
}

int rph_bvh_tree_hash(const rp_scene_desc* desc, uint32_t node_format, uint32_t threads, uint64_t* hash) {
  std::string err;
  int rc = rpb::validate(desc, err);
  if (rc != RP_OK) return fail(err);
  rpb::PackedScene ps;
  rpb::BuildOptions bo;
  bo.node_format = node_format;
  bo.threads = threads;
  rc = rpb::build(desc, bo, ps, err);
  if (rc != RP_OK) return fail(err);
  uint64_t h = 0xcbf29ce484222325ull;  // FNV-1a over the packed records
  auto mix = [&](const void* p, size_t n) {
    const uint8_t* b = static_cast<const uint8_t*>(p);
    for (size_t i = 0; i < n; i++) h = (h ^ b[i]) * 0x100000001b3ull;
  };
  if (ps.node_format == rpl::NODES_W8) mix(ps.wnodes.data(), ps.wnodes.size() * sizeof(rpl::Node8Q));
  else if (ps.node_format == rpl::NODES_Q8) mix(ps.qnodes.data(), ps.qnodes.size() * sizeof(rpl::Node4Q));
  else mix(ps.nodes.data(), ps.nodes.size() * sizeof(rpl::Node4));
  mix(ps.prim_refs.data(), ps.prim_refs.size() * sizeof(rpl::PrimRef));
  *hash = h;
  return RP_OK;
}

namespace {
inline uint32_t rotl32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }
// ChaCha12 block `ctr` of `key` (randomness.rs:5 StdRng = rand_chacha 0.3 ChaCha12Rng).
void chacha12_block(const uint32_t key[8], uint64_t ctr, uint32_t out[16]) {
  uint32_t x[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, key[0], key[1], key[2], key[3],
                    key[4],      key[5],      key[6],      key[7],      (uint32_t)ctr, (uint32_t)(ctr >> 32), 0u, 0u};
  uint32_t s[16];
  std::memcpy(s, x, sizeof s);
  auto qr = [&](int a, int b, int c, int d) {
    x[a] += x[b]; x[d] ^= x[a]; x[d] = rotl32(x[d], 16);
    x[c] += x[d]; x[b] ^= x[c]; x[b] = rotl32(x[b], 12);
    x[a] += x[b]; x[d] ^= x[a]; x[d] = rotl32(x[d], 8);
    x[c] += x[d]; x[b] ^= x[c]; x[b] = rotl32(x[b], 7);
  };
  for (int r = 0; r < 6; r++) {
    qr(0, 4, 8, 12); qr(1, 5, 9, 13); qr(2, 6, 10, 14); qr(3, 7, 11, 15);
    qr(0, 5, 10, 15); qr(1, 6, 11, 12); qr(2, 7, 8, 13); qr(3, 4, 9, 14);
  }
  for (int i = 0; i < 16; i++) out[i] = x[i] + s[i];
}
}  // namespace

int rph_stdrng_u64(const uint8_t seed[32], uint64_t first, uint64_t n, uint64_t* out) {
  if (!seed || (n && !out)) return fail("NULL argument");
  uint32_t key[8];
  for (int i = 0; i < 8; i++)
    key[i] = (uint32_t)seed[4 * i] | (uint32_t)seed[4 * i + 1] << 8 | (uint32_t)seed[4 * i + 2] << 16 |
             (uint32_t)seed[4 * i + 3] << 24;
  // draw k = words 2k, 2k+1 of the keystream = block k / 8, u64 k % 8 of it
  auto work = [&](uint64_t a, uint64_t b) {
    uint32_t w[16];
    uint64_t blk = ~0ull;
    for (uint64_t k = a; k < b; k++) {
      const uint64_t d = first + k;
      if (d / 8 != blk) {
        blk = d / 8;
        chacha12_block(key, blk, w);
      }
      const uint32_t q = (uint32_t)(d % 8);
      out[k] = (uint64_t)w[2 * q] | (uint64_t)w[2 * q + 1] << 32;
    }
  };
  const unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  const unsigned nt = n < (1u << 20) ? 1u : hw;
  std::vector<std::thread> th;
  const uint64_t per = (n + nt - 1) / nt;
  for (unsigned t = 1; t < nt; t++) {
    const uint64_t a = std::min<uint64_t>(n, t * per), b = std::min<uint64_t>(n, a + per);
    if (a < b) th.emplace_back(work, a, b);
  }
  work(0, std::min<uint64_t>(n, per));
  for (auto& t : th) t.join();
  return RP_OK;
}

int rph_make_div32(uint32_t d, uint32_t* m, uint32_t* s) {
  if (d == 0 || !m || !s) return fail("rph_make_div32: d must be >= 1 and m, s non-NULL");
  const rpk::Div32 v = rpk::make_div32(d);
  *m = v.m;
  *s = v.s;
  return RP_OK;
}

}  // extern "C"
