// san_driver.cpp -- native driver of the host code for the sanitizer builds ("Host ASan/UBSan build of the
// C++ oracle").  Built by `make -C raytracing-potato_amd sanitize` with -fsanitize=thread (TSan) and with
// -fsanitize=address,undefined, linked with the host library's sources (rp_host.cpp, rp_bvh.cpp) and the oracle
// (oracle/rp_oracle.c) directly -- no Python and no LD_PRELOAD between the sanitizer and the code.  It exercises:
//   - the multi-threaded binned-SAH builder and its SAH-optimal / greedy 4-wide collapse at 1, 3, 8 and 16 threads
//     (rph_bvh_tree_hash: the tree must not depend on the thread count) and the structural self-check, on a random
//     triangle soup, a mesh with shared vertices and degenerate (zero-area, duplicated) triangles, and spheres;
//   - the CPU traversal model (rph_bvh_traversal_stats_ex) over random rays;
//   - the OBJ and TGA readers (mesh.rs:145-183, image.rs:73-114) on files this driver writes, including truncated and
//     malformed ones (they must fail cleanly), and the TGA writer;
//   - the bulk StdRng (rph_stdrng_u64, threaded) against the oracle's sequential stream;
//   - the oracle's threaded renderer (or_render, the reference driver's tile queue) at 1 and 8 threads: same image.
// Exit status 0 = every check passed and the sanitizer reported nothing (a report aborts with a non-zero status).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../include/rp_host.h"
#include "../oracle/rp_oracle.h"

static int g_fail = 0;
#define CHECK(c)                                                      \
  do {                                                                \
    if (!(c)) {                                                       \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      g_fail = 1;                                                     \
    }                                                                 \
  } while (0)

struct MeshScene {
  std::vector<double> pos, nrm, uv;
  std::vector<uint32_t> idx;
  std::vector<rp_hittable> hit;
  rp_mesh mesh{};
  rp_material mat[2]{};
  rp_scene_desc desc{};
  void finish(uint32_t n_spheres, std::mt19937_64& rng) {
    mesh.n_vertices = (uint32_t)(pos.size() / 3);
    mesh.n_indices = (uint32_t)idx.size();
    mesh.positions = pos.data();
    mesh.normals = nrm.data();
    mesh.uvs = uv.data();
    mesh.indices = idx.data();
    mesh.material = 0;
    for (uint32_t t = 0; t < mesh.n_indices / 3; t++) {
      rp_hittable h{};
      h.kind = RP_HITTABLE_TRIANGLE;
      h.mesh = 0;
      h.triangle = 3 * t;
      hit.push_back(h);
    }
    std::uniform_real_distribution<double> u(-1.0, 1.0);
    for (uint32_t k = 0; k < n_spheres; k++) {
      rp_hittable h{};
      h.kind = RP_HITTABLE_SPHERE;
      h.material = 1;
      h.center[0] = u(rng);
      h.center[1] = u(rng);
      h.center[2] = u(rng);
      h.radius = k == 0 ? 1000.0 : 0.05 + 0.1 * (u(rng) + 1.0);  // one huge sphere: an always-tested primitive
      if (k == 0) h.center[1] = -1001.0;
      hit.push_back(h);
    }
    mat[0].scatter.kind = RP_SCATTER_LAMBERT;
    mat[0].absorb.kind = RP_ABSORB_ALBEDO;
    mat[0].absorb.color[0] = mat[0].absorb.color[1] = mat[0].absorb.color[2] = 0.6;
    mat[1].scatter.kind = RP_SCATTER_METAL;
    mat[1].scatter.param = 0.2;
    mat[1].absorb.kind = RP_ABSORB_WHITE_BODY;
    desc.root_kind = RP_ROOT_BVH;
    desc.n_hittables = (uint32_t)hit.size();
    desc.hittables = hit.data();
    desc.n_meshes = 1;
    desc.meshes = &mesh;
    desc.n_materials = 2;
    desc.materials = mat;
    desc.n_textures = 0;
    desc.textures = nullptr;
    desc.background.kind = RP_EMIT_SKY_GRADIENT;
  }
};

static void add_vertex(MeshScene& s, double x, double y, double z) {
  s.pos.insert(s.pos.end(), {x, y, z});
  const double n = std::sqrt(x * x + y * y + z * z) + 1e-9;
  s.nrm.insert(s.nrm.end(), {x / n, y / n, z / n});
  s.uv.insert(s.uv.end(), {0.5 * (x + 1.0), 0.5 * (y + 1.0)});
}

static MeshScene soup(uint32_t n, uint64_t seed) {  // random small triangles in [-1, 1]^3 (config C5's construction)
  MeshScene s;
  std::mt19937_64 rng(seed);
  std::uniform_real_distribution<double> u(-1.0, 1.0);
  for (uint32_t t = 0; t < n; t++) {
    const double cx = u(rng), cy = u(rng), cz = u(rng);
    for (int v = 0; v < 3; v++) {
      add_vertex(s, cx + 0.02 * u(rng), cy + 0.02 * u(rng), cz + 0.02 * u(rng));
      s.idx.push_back(3 * t + v);
    }
  }
  s.finish(8, rng);
  return s;
}

static MeshScene grid_with_degenerates(uint32_t side, uint64_t seed) {  // shared vertices, zero-area + duplicates
  MeshScene s;
  std::mt19937_64 rng(seed);
  for (uint32_t j = 0; j <= side; j++)
    for (uint32_t i = 0; i <= side; i++) add_vertex(s, (double)i / side - 0.5, 0.0, (double)j / side - 0.5);
  for (uint32_t j = 0; j < side; j++)
    for (uint32_t i = 0; i < side; i++) {
      const uint32_t a = j * (side + 1) + i, b = a + 1, c = a + side + 1, d = c + 1;
      s.idx.insert(s.idx.end(), {a, b, c, b, d, c});
      if ((i + j) % 7 == 0) s.idx.insert(s.idx.end(), {a, a, b});  // zero-area triangle
      if ((i + j) % 11 == 0) s.idx.insert(s.idx.end(), {a, b, c});  // duplicate triangle (exact-t ties)
    }
  s.finish(3, rng);
  return s;
}

static void check_tree(const char* name, const rp_scene_desc& d) {
  for (uint32_t fmt : {1u, 2u, 3u}) {    // RP_NODES_F32, Q8, W8
    for (uint32_t col : {1u, 2u}) {      // RP_COLLAPSE_GREEDY, SAH
      uint64_t st[16] = {0};
      const int rc = rph_bvh_selfcheck_ex(&d, fmt, col, st);
      if (rc != RP_OK) std::fprintf(stderr, "%s fmt %u collapse %u: %s\n", name, fmt, col, rph_last_error());
      CHECK(rc == RP_OK);
    }
    uint64_t h0 = 0;
    for (uint32_t threads : {1u, 3u, 8u, 16u}) {
      uint64_t h = 0;
      CHECK(rph_bvh_tree_hash(&d, fmt, threads, &h) == RP_OK);
      if (threads == 1) h0 = h;
      CHECK(h == h0);
    }
  }
  std::mt19937_64 rng(5);
  std::uniform_real_distribution<double> u(-1.5, 1.5);
  const uint32_t n = 4096;
  std::vector<double> rays(8 * n);
  for (uint32_t r = 0; r < n; r++) {
    double* q = &rays[8 * r];
    q[0] = u(rng); q[1] = u(rng); q[2] = 3.0;
    q[3] = 0.1 * u(rng); q[4] = 0.1 * u(rng); q[5] = -1.0;
    if (r % 17 == 0) q[3] = 0.0;  // axis-parallel components
    q[6] = 1e-3;
    q[7] = (r % 5 == 0) ? 2.5 : INFINITY;
  }
  std::vector<uint64_t> per(4 * n);
  for (uint32_t fmt : {1u, 2u, 3u}) CHECK(rph_bvh_traversal_stats_ex(&d, rays.data(), n, fmt, 2u, per.data()) == RP_OK);
  std::printf("%s: %u hittables, trees deterministic at 1/3/8/16 threads, self-checks pass\n", name, d.n_hittables);
}

static void write_file(const std::string& path, const std::string& bytes) {
  FILE* f = std::fopen(path.c_str(), "wb");
  std::fwrite(bytes.data(), 1, bytes.size(), f);
  std::fclose(f);
}

static void check_io(const std::string& dir) {
  const std::string obj = dir + "/t.obj";
  write_file(obj, "# test\nv 0 0 0\nv 1 0 0\nv 0 1 0\nv 1 1 0\nvn 0 0 1\nvt 0 0\nvt 1 0\nvt 0 1\nvt 1 1\n"
                  "f 1/1/1 2/2/1 3/3/1\nf 2/2/1 4/4/1 3/3/1\n");
  rph_mesh m{};
  CHECK(rph_obj_load(obj.c_str(), &m) == RP_OK);
  CHECK(m.n_indices == 6);
  rph_mesh_free(&m);
  or_mesh_data om{};
  CHECK(or_obj_load(obj.c_str(), &om) == 0);
  or_mesh_free(&om);
  // malformed: an index past the vertices, a truncated face, garbage numbers, an empty file
  const char* bad[] = {"v 0 0 0\nvn 0 0 1\nvt 0 0\nf 1/1/1 2/1/1 3/1/1\n", "v 0 0 0\nf 1/1/1 1/1\n",
                       "v x y z\nf a b c\n", ""};
  for (const char* b : bad) {
    write_file(dir + "/bad.obj", b);
    rph_mesh mb{};
    if (rph_obj_load((dir + "/bad.obj").c_str(), &mb) == RP_OK) rph_mesh_free(&mb);
    or_mesh_data ob{};
    if (or_obj_load((dir + "/bad.obj").c_str(), &ob) == 0) or_mesh_free(&ob);
  }
  CHECK(rph_obj_load((dir + "/missing.obj").c_str(), &m) != RP_OK);
  // TGA: write, read back, and truncated / unsupported headers
  const uint32_t w = 37, h = 11;
  std::vector<uint8_t> img(4 * w * h);
  for (size_t i = 0; i < img.size(); i++) img[i] = (uint8_t)(i * 31 + 7);
  for (size_t i = 3; i < img.size(); i += 4) img[i] = 255;
  const std::string tga = dir + "/t.tga";
  CHECK(rph_tga_save(tga.c_str(), w, h, img.data()) == RP_OK);
  uint32_t rw = 0, rh = 0;
  uint8_t* back = nullptr;
  CHECK(rph_tga_load(tga.c_str(), &rw, &rh, &back) == RP_OK);
  CHECK(rw == w && rh == h && back && std::memcmp(back, img.data(), img.size()) == 0);
  rph_free(back);
  uint8_t* ob2 = nullptr;
  CHECK(or_tga_load(tga.c_str(), &rw, &rh, &ob2) == 0);
  or_free(ob2);
  FILE* f = std::fopen(tga.c_str(), "rb");
  std::string all;
  char buf[4096];
  size_t k;
  while ((k = std::fread(buf, 1, sizeof buf, f)) > 0) all.append(buf, k);
  std::fclose(f);
  for (size_t cut : {size_t(0), size_t(5), size_t(17), size_t(18), all.size() / 2, all.size() - 1}) {
    write_file(dir + "/cut.tga", all.substr(0, cut));
    uint8_t* p = nullptr;
    if (rph_tga_load((dir + "/cut.tga").c_str(), &rw, &rh, &p) == RP_OK) rph_free(p);
    p = nullptr;
    if (or_tga_load((dir + "/cut.tga").c_str(), &rw, &rh, &p) == 0) or_free(p);
  }
  std::string rle = all;
  rle[2] = 10;  // RLE: unsupported
  write_file(dir + "/rle.tga", rle);
  uint8_t* p = nullptr;
  CHECK(rph_tga_load((dir + "/rle.tga").c_str(), &rw, &rh, &p) != RP_OK);
  std::printf("OBJ/TGA readers and writer: round trip exact, malformed inputs refused\n");
}

static void check_rng() {
  uint8_t seed[32];
  for (int i = 0; i < 32; i++) seed[i] = (uint8_t)(i * 13 + 1);
  const uint64_t n = 3u << 20;
  std::vector<uint64_t> bulk(n), seq(n);
  CHECK(rph_stdrng_u64(seed, 0, n, bulk.data()) == RP_OK);
  or_rng r;
  or_rng_from_seed(&r, seed, 12);
  for (uint64_t i = 0; i < n; i++) seq[i] = or_rng_next_u64(&r);
  CHECK(bulk == seq);
  std::printf("threaded bulk StdRng == the oracle's sequential stream (%llu draws)\n", (unsigned long long)n);
}

static void check_oracle_render(const MeshScene& s) {
  or_scene* os = or_scene_create(&s.desc);
  CHECK(os != nullptr);
  if (!os) return;
  rp_camera cam{};
  cam.aspect_ratio = 1.0;
  cam.fov = 1.2;
  cam.focal_dist = 1.0;
  const double p[3] = {0.0, 0.5, 3.0}, t[3] = {0.0, 0.0, 0.0}, up[3] = {0.0, 1.0, 0.0};
  or_lookat(p, t, up, cam.orientation);
  std::memcpy(cam.position, p, sizeof p);
  rp_render_params rp{};
  rp.width = 48;
  rp.height = 32;
  rp.spp = 4;
  rp.max_bounce = 8;
  rp.seed = 7;
  rp.tile_w = rp.tile_h = 8;
  std::vector<double> a(3 * 48 * 32), b(3 * 48 * 32);
  uint64_t ca[OR_C_N] = {0}, cb[OR_C_N] = {0};
  CHECK(or_render(os, &cam, &rp, a.data(), nullptr, ca, 1) == 0);
  CHECK(or_render(os, &cam, &rp, b.data(), nullptr, cb, 8) == 0);
  CHECK(std::memcmp(a.data(), b.data(), a.size() * sizeof(double)) == 0);
  CHECK(ca[OR_C_RAYS] == cb[OR_C_RAYS]);
  const double secs = or_render_baseline(os, &cam, 32, 32, 2, 8, 16, 8, 11, nullptr, ca);
  CHECK(secs >= 0.0);
  or_scene_destroy(os);
  std::printf("oracle render at 1 and 8 threads: identical frames; threaded baseline driver ran\n");
}

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : "/tmp";
  MeshScene a = soup(200000, 11);  // >= 2^16 primitives: the parallel build form (rp_bvh.cpp ParallelBuild) runs
  check_tree("soup", a.desc);
  MeshScene b = grid_with_degenerates(40, 3);
  check_tree("grid+degenerates", b.desc);
  check_io(dir);
  check_rng();
  check_oracle_render(b);
  std::printf(g_fail ? "FAILED\n" : "ALL CHECKS PASSED\n");
  return g_fail;
}
