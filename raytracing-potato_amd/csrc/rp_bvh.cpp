// rp_bvh.cpp -- scene validation, binned-SAH BVH2 build, packing into rp_layout.h records.
#include "rp_bvh.h"

#include <algorithm>
#include <functional>
#include <cmath>
#include <cstring>
#include <limits>

namespace rpb {

namespace {

struct Box {
  double lo[3], hi[3];
  void reset() {
    for (int k = 0; k < 3; k++) {
      lo[k] = std::numeric_limits<double>::infinity();
      hi[k] = -std::numeric_limits<double>::infinity();
    }
  }
  // AABB::union (utility.rs:130-135): exact min/max, so parents contain children bit-exactly.
  void grow(const Box& b) {
    for (int k = 0; k < 3; k++) {
      lo[k] = std::fmin(lo[k], b.lo[k]);
      hi[k] = std::fmax(hi[k], b.hi[k]);
    }
  }
  double area() const {
    double dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
    if (!(dx >= 0) || !(dy >= 0) || !(dz >= 0)) return 0.0;
    return 2.0 * (dx * dy + dy * dz + dz * dx);
  }
};

struct Ref {
  Box box;
  double c[3];
  uint32_t id;
};

// Binary SAH tree (intermediate): built top-down with binned SAH, then collapsed into 4-wide nodes.
struct BinNode {
  Box box;
  int32_t left = -1, right = -1;  // inner: children indices
  uint32_t first = 0, count = 0;  // leaf: primitives [first, first + count) of `order`
  bool leaf() const { return count > 0; }
};

struct Builder {
  const BuildOptions& opt;
  std::vector<Ref>& refs;
  std::vector<BinNode>& bin;
  std::vector<uint32_t>& order;  // leaf-ordered hittable ids
  uint64_t n_leaves = 0;

  // Returns the split position m in (b, e) or b when the range should be a leaf.
  uint32_t split(uint32_t b, uint32_t e, const Box& box) {
    uint32_t n = e - b;
    Box cb;
    cb.reset();
    for (uint32_t i = b; i < e; i++)
      for (int k = 0; k < 3; k++) {
        cb.lo[k] = std::fmin(cb.lo[k], refs[i].c[k]);
        cb.hi[k] = std::fmax(cb.hi[k], refs[i].c[k]);
      }
    const uint32_t NB = std::max(2u, std::min(opt.bins, n));
    double best_cost = std::numeric_limits<double>::infinity();
    int best_axis = -1;
    uint32_t best_bin = 0;
    std::vector<Box> bb(NB);
    std::vector<uint32_t> bn(NB);
    std::vector<double> right_area(NB);
    std::vector<uint32_t> right_n(NB);
    for (int ax = 0; ax < 3; ax++) {
      double ext = cb.hi[ax] - cb.lo[ax];
      if (!(ext > 0.0)) continue;
      double scale = (double)NB / ext;
      for (uint32_t k = 0; k < NB; k++) { bb[k].reset(); bn[k] = 0; }
      for (uint32_t i = b; i < e; i++) {
        int k = (int)((refs[i].c[ax] - cb.lo[ax]) * scale);
        k = std::min<int>(std::max(k, 0), (int)NB - 1);
        bb[k].grow(refs[i].box);
        bn[k]++;
      }
      Box acc;
      acc.reset();
      uint32_t cnt = 0;
      for (int k = (int)NB - 1; k >= 1; k--) {
        acc.grow(bb[k]);
        cnt += bn[k];
        right_area[k] = acc.area();
        right_n[k] = cnt;
      }
      acc.reset();
      cnt = 0;
      for (uint32_t k = 0; k + 1 < NB; k++) {
        acc.grow(bb[k]);
        cnt += bn[k];
        if (cnt == 0 || right_n[k + 1] == 0) continue;
        double cost = acc.area() * cnt + right_area[k + 1] * right_n[k + 1];
        if (cost < best_cost) { best_cost = cost; best_axis = ax; best_bin = k; }
      }
    }
    double parent_area = box.area();
    double leaf_cost = opt.cost_intersect * n;
    if (best_axis >= 0) {
      double split_cost = opt.cost_traverse +
                          (parent_area > 0.0 ? opt.cost_intersect * best_cost / parent_area : opt.cost_intersect * n);
      if (n <= opt.max_leaf && leaf_cost <= split_cost) return b;
      double ext = cb.hi[best_axis] - cb.lo[best_axis];
      double scale = (double)NB / ext;
      auto mid = std::partition(refs.begin() + b, refs.begin() + e, [&](const Ref& r) {
        int k = (int)((r.c[best_axis] - cb.lo[best_axis]) * scale);
        k = std::min<int>(std::max(k, 0), (int)NB - 1);
        return (uint32_t)k <= best_bin;
      });
      uint32_t m = (uint32_t)(mid - refs.begin());
      if (m > b && m < e) return m;
    }
    if (n <= opt.max_leaf) return b;
    // Degenerate centroids (or a failed partition): object median on the longest centroid axis.
    int ax = 0;
    for (int k = 1; k < 3; k++)
      if (cb.hi[k] - cb.lo[k] > cb.hi[ax] - cb.lo[ax]) ax = k;
    uint32_t m = b + n / 2;
    std::nth_element(refs.begin() + b, refs.begin() + m, refs.begin() + e, [ax](const Ref& x, const Ref& y) {
      if (x.c[ax] != y.c[ax]) return x.c[ax] < y.c[ax];
      return x.id < y.id;
    });
    return m;
  }

  // Builds range [b, e) whose box is `box` into bin[]; returns its index.
  int32_t build(uint32_t b, uint32_t e, const Box& box) {
    const int32_t self = (int32_t)bin.size();
    bin.emplace_back();
    bin[self].box = box;
    const uint32_t m = split(b, e, box);
    if (m == b) {
      bin[self].first = (uint32_t)order.size();
      bin[self].count = e - b;
      for (uint32_t i = b; i < e; i++) order.push_back(refs[i].id);
      n_leaves++;
      return self;
    }
    Box lb, rb;
    lb.reset();
    rb.reset();
    for (uint32_t i = b; i < m; i++) lb.grow(refs[i].box);
    for (uint32_t i = m; i < e; i++) rb.grow(refs[i].box);
    const int32_t l = build(b, m, lb);
    const int32_t r = build(m, e, rb);
    bin[self].left = l;
    bin[self].right = r;
    return self;
  }
};

// The quantization frame of a wide node from its exact box (rp_layout.h qframe); an axis without a finite
// extent (NaN geometry only) gets the frame at 0.
void node_frame(const Box& b, rpl::Node4& n) {
  for (int a = 0; a < 3; a++) {
    const bool ok = std::isfinite(b.lo[a]) && std::isfinite(b.hi[a]) && b.lo[a] <= b.hi[a];
    rpl::qframe(ok ? b.lo[a] : 0.0, ok ? b.hi[a] : 0.0, n.o[a], n.s[a]);
  }
}

// Collapse the binary tree into 4-wide nodes: each wide node takes its binary node's two children and
// repeatedly opens the inner child of largest surface area until it has 4 children (Wald et al.).
struct Collapser {
  const std::vector<BinNode>& bin;
  std::vector<rpl::Node4>& out;
  uint32_t max_depth = 0;

  uint32_t emit(int32_t bi, uint32_t depth) {
    if (depth > max_depth) max_depth = depth;
    const uint32_t self = (uint32_t)out.size();
    out.emplace_back();
    std::vector<int32_t> kids;
    if (bin[bi].leaf()) {
      kids.push_back(bi);  // root that is a single leaf
    } else {
      kids = {bin[bi].left, bin[bi].right};
      while (kids.size() < 4) {
        int best = -1;
        double area = -1.0;
        for (size_t k = 0; k < kids.size(); k++)
          if (!bin[kids[k]].leaf() && bin[kids[k]].box.area() > area) { area = bin[kids[k]].box.area(); best = (int)k; }
        if (best < 0) break;
        const int32_t open = kids[best];
        kids[best] = bin[open].left;
        kids.push_back(bin[open].right);
      }
    }
    uint32_t entries[4];
    {
      rpl::Node4& n = out[self];
      Box nb;
      nb.reset();
      for (int32_t k : kids) nb.grow(bin[k].box);
      node_frame(nb, n);
      for (int c = 0; c < 4; c++) {
        if ((size_t)c >= kids.size()) {
          rpl::empty_child(n, c);
          entries[c] = rpl::ENTRY_EMPTY;
          continue;
        }
        const BinNode& k = bin[kids[c]];
        rpl::quantize_child(n, c, k.box.lo, k.box.hi);
        entries[c] = k.leaf() ? rpl::ENTRY_LEAF | ((k.count - 1) << rpl::LEAF_SHIFT) | k.first : 0u;
      }
    }
    for (int c = 0; c < 4; c++)
      if ((size_t)c < kids.size() && !bin[kids[c]].leaf()) entries[c] = emit(kids[c], depth + 1);
    for (int c = 0; c < 4; c++) out[self].child[c] = entries[c];
    return self;
  }
};

Box hittable_box(const rp_scene_desc* d, const rp_hittable& h) {
  Box b;
  if (h.kind == RP_HITTABLE_SPHERE) {
    // hittable.rs:124-129
    for (int k = 0; k < 3; k++) {
      b.lo[k] = h.center[k] - h.radius;
      b.hi[k] = h.center[k] + h.radius;
    }
  } else {
    // hittable.rs:131-140
    const rp_mesh& m = d->meshes[h.mesh];
    const double* a = m.positions + 3 * (size_t)m.indices[h.triangle];
    const double* bb = m.positions + 3 * (size_t)m.indices[h.triangle + 1];
    const double* c = m.positions + 3 * (size_t)m.indices[h.triangle + 2];
    for (int k = 0; k < 3; k++) {
      b.lo[k] = std::fmin(std::fmin(a[k], bb[k]), c[k]);
      b.hi[k] = std::fmax(std::fmax(a[k], bb[k]), c[k]);
    }
  }
  return b;
}

}  // namespace

int validate(const rp_scene_desc* d, std::string& err) {
  auto fail = [&](const std::string& m) { err = m; return (int)RP_EINVAL; };
  if (!d) return fail("scene description is NULL");
  if (d->root_kind != RP_ROOT_BVH && d->root_kind != RP_ROOT_LIST) return fail("unknown root_kind");
  if (d->root_kind == RP_ROOT_BVH && d->n_hittables == 0)
    return fail("Bvh::new over zero hittables (bvh.rs:40 unreachable!())");
  if (d->n_hittables && !d->hittables) return fail("hittables is NULL");
  if (d->n_meshes && !d->meshes) return fail("meshes is NULL");
  if (d->n_materials && !d->materials) return fail("materials is NULL");
  if (d->n_textures && !d->textures) return fail("textures is NULL");
  auto check_tex = [&](uint32_t t, const char* what) -> bool {
    if (t >= d->n_textures) { err = std::string(what) + ": TextureId out of range"; return false; }
    return true;
  };
  for (uint32_t i = 0; i < d->n_textures; i++) {
    const rp_texture& t = d->textures[i];
    if (t.kind > RP_TEXTURE_PERLIN) return fail("texture " + std::to_string(i) + ": unknown kind");
    if (t.kind == RP_TEXTURE_IMAGE && (!t.rgba || t.width == 0 || t.height == 0))
      return fail("texture " + std::to_string(i) + ": empty image");
    if (t.kind == RP_TEXTURE_CHECKER) {
      if (!check_tex(t.odd, "checker odd") || !check_tex(t.even, "checker even")) return RP_EINVAL;
    }
  }
  // Checker chains must terminate (the reference would recurse forever).
  for (uint32_t i = 0; i < d->n_textures; i++) {
    std::vector<uint32_t> stack{i};
    std::vector<uint8_t> seen(d->n_textures, 0);
    uint64_t steps = 0;
    while (!stack.empty()) {
      uint32_t t = stack.back();
      stack.pop_back();
      if (++steps > 64ull * d->n_textures + 64) return fail("checker textures form a cycle");
      if (d->textures[t].kind == RP_TEXTURE_CHECKER) {
        if (seen[t]) return fail("checker textures form a cycle");
        seen[t] = 1;
        stack.push_back(d->textures[t].odd);
        stack.push_back(d->textures[t].even);
      }
    }
  }
  for (uint32_t i = 0; i < d->n_materials; i++) {
    const rp_material& m = d->materials[i];
    if (m.scatter.kind > RP_SCATTER_DIELECTRIC) return fail("material " + std::to_string(i) + ": bad scatter");
    if (m.absorb.kind > RP_ABSORB_ALBEDO_MAP) return fail("material " + std::to_string(i) + ": bad absorb");
    if (m.emit.kind > RP_EMIT_SKY_SPHERE) return fail("material " + std::to_string(i) + ": bad emit");
    if (m.absorb.kind == RP_ABSORB_ALBEDO_MAP && !check_tex(m.absorb.texture, "AlbedoMap")) return RP_EINVAL;
    if (m.emit.kind == RP_EMIT_SKY_SPHERE && !check_tex(m.emit.texture, "SkySphere")) return RP_EINVAL;
  }
  if (d->background.kind > RP_EMIT_SKY_SPHERE) return fail("background: bad emit kind");
  if (d->background.kind == RP_EMIT_SKY_SPHERE && !check_tex(d->background.texture, "background SkySphere"))
    return RP_EINVAL;
  for (uint32_t i = 0; i < d->n_meshes; i++) {
    const rp_mesh& m = d->meshes[i];
    if (m.n_vertices && (!m.positions || !m.normals || !m.uvs)) return fail("mesh " + std::to_string(i) + ": NULL arrays");
    if (m.n_indices && !m.indices) return fail("mesh " + std::to_string(i) + ": NULL indices");
    if (m.material >= d->n_materials) return fail("mesh " + std::to_string(i) + ": MaterialId out of range");
    for (uint32_t k = 0; k < m.n_indices; k++)
      if (m.indices[k] >= m.n_vertices) return fail("mesh " + std::to_string(i) + ": vertex index out of range");
  }
  for (uint32_t i = 0; i < d->n_hittables; i++) {
    const rp_hittable& h = d->hittables[i];
    if (h.kind == RP_HITTABLE_SPHERE) {
      if (h.material >= d->n_materials) return fail("sphere " + std::to_string(i) + ": MaterialId out of range");
    } else if (h.kind == RP_HITTABLE_TRIANGLE) {
      if (h.mesh >= d->n_meshes) return fail("triangle " + std::to_string(i) + ": MeshId out of range");
      if ((uint64_t)h.triangle + 2 >= d->meshes[h.mesh].n_indices)
        return fail("triangle " + std::to_string(i) + ": TriangleId out of range");
    } else {
      return fail("hittable " + std::to_string(i) + ": unknown kind");
    }
  }
  return RP_OK;
}

// Does sampling texture t read hit.uv?  (DebugUVs and Image do; Checker if either branch does;
// Solid/Noise/Perlin/Missing do not -- texture.rs:21-118).  validate() guarantees termination.
static bool texture_reads_uv(const rp_scene_desc* d, uint32_t t, int depth = 0) {
  if (t >= d->n_textures || depth > 64) return true;
  const rp_texture& x = d->textures[t];
  if (x.kind == RP_TEXTURE_DEBUG_UVS || x.kind == RP_TEXTURE_IMAGE) return true;
  if (x.kind == RP_TEXTURE_CHECKER)
    return texture_reads_uv(d, x.odd, depth + 1) || texture_reads_uv(d, x.even, depth + 1);
  return false;
}

int build(const rp_scene_desc* d, const BuildOptions& opt, PackedScene& out, std::string& err) {
  out = PackedScene();
  // ---- shading tables
  std::vector<uint64_t> vbase(d->n_meshes + 1, 0);
  for (uint32_t i = 0; i < d->n_meshes; i++) vbase[i + 1] = vbase[i] + d->meshes[i].n_vertices;
  if (vbase[d->n_meshes] > 0xffffffffull) { err = "too many vertices"; return RP_EINVAL; }
  out.vnrm.resize(3 * vbase[d->n_meshes] + 3);
  out.vuv.resize(2 * vbase[d->n_meshes] + 2);
  for (uint32_t i = 0; i < d->n_meshes; i++) {
    const rp_mesh& m = d->meshes[i];
    if (m.n_vertices) {
      std::memcpy(&out.vnrm[3 * vbase[i]], m.normals, sizeof(double) * 3 * m.n_vertices);
      std::memcpy(&out.vuv[2 * vbase[i]], m.uvs, sizeof(double) * 2 * m.n_vertices);
    }
  }
  for (uint32_t i = 0; i < d->n_materials; i++) {
    const rp_material& s = d->materials[i];
    rpl::Material m{};
    m.scatter_kind = s.scatter.kind;
    m.scatter_param = s.scatter.param;
    m.absorb_kind = s.absorb.kind;
    m.absorb_tex = s.absorb.texture;
    m.emit_kind = s.emit.kind;
    m.emit_tex = s.emit.texture;
    // uv is only computed on the device when something will read it (the value is the reference's)
    m.needs_uv = (s.absorb.kind == RP_ABSORB_ALBEDO_MAP && texture_reads_uv(d, s.absorb.texture)) ||
                 (s.emit.kind == RP_EMIT_SKY_SPHERE && texture_reads_uv(d, s.emit.texture));
    for (int k = 0; k < 3; k++) {
      m.absorb_color[k] = s.absorb.color[k];
      m.emit_color[k] = s.emit.color[k];
    }
    out.materials.push_back(m);
  }
  if (out.materials.empty()) out.materials.push_back(rpl::Material{});
  for (uint32_t i = 0; i < d->n_textures; i++) {
    const rp_texture& s = d->textures[i];
    rpl::Texture t{};
    t.kind = s.kind;
    t.odd = s.odd;
    t.even = s.even;
    t.width = s.width;
    t.height = s.height;
    t.seed = s.seed;
    for (int k = 0; k < 3; k++) t.color[k] = s.color[k];
    t.texel_offset = out.texels.size();
    if (s.kind == RP_TEXTURE_IMAGE) {
      size_t n = (size_t)s.width * s.height;
      size_t off = out.texels.size();
      out.texels.resize(off + n);
      std::memcpy(&out.texels[off], s.rgba, n * 4);
    }
    out.textures.push_back(t);
  }
  if (out.textures.empty()) out.textures.push_back(rpl::Texture{});
  if (out.texels.empty()) out.texels.push_back(0);
  out.background.kind = d->background.kind;
  out.background.tex = d->background.texture;
  out.background.needs_uv = d->background.kind == RP_EMIT_SKY_SPHERE && texture_reads_uv(d, d->background.texture);
  if (d->background.kind == RP_EMIT_SKY_SPHERE && d->textures[d->background.texture].kind == RP_TEXTURE_IMAGE) {
    const rpl::Texture& t = out.textures[d->background.texture];
    out.background.img_w = t.width;
    out.background.img_h = t.height;
    out.background.img_off = (uint32_t)t.texel_offset;
  }
  for (int k = 0; k < 3; k++) out.background.color[k] = d->background.color[k];

  if (opt.tables_only) return RP_OK;

  // ---- BVH over all hittables (a List root is served by the same tree: closest hit is
  //      independent of visit order except exact-t ties)
  uint32_t n = d->n_hittables;
  if (n > rpl::MAX_PRIMS) { err = "too many hittables for the node encoding"; return RP_EINVAL; }
  // the kernels address primitives and wide nodes by 32-bit byte offsets (<= n nodes of 128 B)
  if ((uint64_t)n * sizeof(rpl::Prim) > 0xFFFFFFFFull) { err = "too many hittables for 32-bit device offsets"; return RP_EINVAL; }
  if (opt.max_leaf < 1 || opt.max_leaf > rpl::LEAF_MAX) { err = "max_leaf out of range"; return RP_EINVAL; }
  std::vector<Ref> refs(n);
  for (uint32_t i = 0; i < n; i++) {
    refs[i].box = hittable_box(d, d->hittables[i]);
    for (int k = 0; k < 3; k++) refs[i].c[k] = 0.5 * (refs[i].box.lo[k] + refs[i].box.hi[k]);
    refs[i].id = i;
  }
  // always-tested primitives (BuildOptions::always_max): out of the tree, appended after its leaves
  std::vector<uint32_t> always;
  if (opt.always_max > 0 && n > 1) {
    const uint32_t m = std::min<uint32_t>(opt.always_max, n - 1);
    std::vector<uint32_t> idx(n);
    for (uint32_t i = 0; i < n; i++) idx[i] = i;
    std::partial_sort(idx.begin(), idx.begin() + m, idx.end(),
                      [&](uint32_t a, uint32_t b) { return refs[a].box.area() > refs[b].box.area(); });
    Box rest;
    rest.reset();
    for (uint32_t i = m; i < n; i++) rest.grow(refs[idx[i]].box);
    const double ra = rest.area();
    for (uint32_t j = 0; j < m; j++)
      if (std::isfinite(refs[idx[j]].box.area()) && refs[idx[j]].box.area() > 0.0 &&
          refs[idx[j]].box.area() >= opt.always_ratio * ra)
        always.push_back(idx[j]);
    std::sort(always.begin(), always.end());
    if (!always.empty()) {
      std::vector<Ref> tree_refs;
      tree_refs.reserve(n - always.size());
      for (uint32_t i = 0, a = 0; i < n; i++) {
        if (a < always.size() && always[a] == i) { a++; continue; }
        tree_refs.push_back(refs[i]);
      }
      refs.swap(tree_refs);
    }
  }
  const uint32_t n_tree = (uint32_t)refs.size();
  double amax = 0.0;
  for (const Ref& r : refs)
    for (int k = 0; k < 3; k++) amax = std::fmax(amax, std::fmax(std::fabs(r.box.lo[k]), std::fabs(r.box.hi[k])));
  if (!(amax <= rpl::COORD_MAX)) {
    err = "primitive coordinates beyond +-2^54 (or infinite) are not supported by the quantized tree";
    return RP_EINVAL;
  }
  out.qbound = rpl::qbound(amax);
  std::vector<uint32_t> order;
  order.reserve(n);
  std::vector<BinNode> bin;
  bin.reserve(n_tree ? 2 * (size_t)n_tree : 1);
  Builder B{opt, refs, bin, order};
  if (n_tree == 0) {
    rpl::Node4 root{};
    for (int a = 0; a < 3; a++) rpl::qframe(0.0, 0.0, root.o[a], root.s[a]);
    for (int c = 0; c < 4; c++) {
      rpl::empty_child(root, c);
      root.child[c] = rpl::ENTRY_EMPTY;
    }
    out.nodes.push_back(root);
    out.max_depth = 0;
  } else {
    Box all;
    all.reset();
    for (auto& r : refs) all.grow(r.box);
    B.build(0, n_tree, all);
    out.nodes.reserve(bin.size() / 2 + 1);
    Collapser C{bin, out.nodes};
    C.emit(0, 0);
    out.max_depth = C.max_depth;
  }
  out.root = 0;
  out.n_leaves = B.n_leaves;
  out.always_first = (uint32_t)order.size();
  out.n_always = (uint32_t)always.size();
  for (uint32_t a : always) order.push_back(a);

  // ---- primitives in leaf order
  out.prims.resize(order.size() ? order.size() : 1);
  std::memset(out.prims.data(), 0, sizeof(rpl::Prim) * out.prims.size());
  out.prim_refs.resize(out.prims.size());
  std::memset(out.prim_refs.data(), 0, sizeof(rpl::PrimRef) * out.prim_refs.size());
  for (size_t k = 0; k < order.size(); k++) {
    const rp_hittable& h = d->hittables[order[k]];
    rpl::Prim& p = out.prims[k];
    rpl::PrimRef& pr = out.prim_refs[k];
    pr.src = order[k];
    if (h.kind == RP_HITTABLE_SPHERE) {
      p.kind = rpl::PRIM_SPHERE;
      p.material = h.material;
      for (int c = 0; c < 3; c++) p.g[c] = h.center[c];
      p.g[3] = h.radius;
    } else {
      const rp_mesh& m = d->meshes[h.mesh];
      uint32_t i0 = m.indices[h.triangle], i1 = m.indices[h.triangle + 1], i2 = m.indices[h.triangle + 2];
      const double* a = m.positions + 3 * (size_t)i0;
      const double* b = m.positions + 3 * (size_t)i1;
      const double* c = m.positions + 3 * (size_t)i2;
      p.kind = rpl::PRIM_TRIANGLE;
      p.material = m.material;
      for (int k2 = 0; k2 < 3; k2++) {
        p.g[k2] = a[k2];
        p.g[3 + k2] = a[k2] - b[k2];  // ba, hittable.rs:71 (same IEEE subtraction as on the device)
        p.g[6 + k2] = a[k2] - c[k2];  // ca, hittable.rs:72
      }
      pr.v[0] = (uint32_t)(vbase[h.mesh] + i0);
      pr.v[1] = (uint32_t)(vbase[h.mesh] + i1);
      pr.v[2] = (uint32_t)(vbase[h.mesh] + i2);
    }
  }
  return RP_OK;
}

// One primitive record + reference (the packing of build(), in hittable order).
static void pack_prim(const rp_scene_desc* d, const std::vector<uint64_t>& vbase, uint32_t id, rpl::Prim& p,
                      rpl::PrimRef& pr) {
  const rp_hittable& h = d->hittables[id];
  std::memset(&p, 0, sizeof p);
  std::memset(&pr, 0, sizeof pr);
  pr.src = id;
  if (h.kind == RP_HITTABLE_SPHERE) {
    p.kind = rpl::PRIM_SPHERE;
    p.material = h.material;
    for (int c = 0; c < 3; c++) p.g[c] = h.center[c];
    p.g[3] = h.radius;
  } else {
    const rp_mesh& m = d->meshes[h.mesh];
    uint32_t i0 = m.indices[h.triangle], i1 = m.indices[h.triangle + 1], i2 = m.indices[h.triangle + 2];
    const double* a = m.positions + 3 * (size_t)i0;
    const double* b = m.positions + 3 * (size_t)i1;
    const double* c = m.positions + 3 * (size_t)i2;
    p.kind = rpl::PRIM_TRIANGLE;
    p.material = m.material;
    for (int k2 = 0; k2 < 3; k2++) {
      p.g[k2] = a[k2];
      p.g[3 + k2] = a[k2] - b[k2];  // ba, hittable.rs:71
      p.g[6 + k2] = a[k2] - c[k2];  // ca, hittable.rs:72
    }
    pr.v[0] = (uint32_t)(vbase[h.mesh] + i0);
    pr.v[1] = (uint32_t)(vbase[h.mesh] + i1);
    pr.v[2] = (uint32_t)(vbase[h.mesh] + i2);
  }
}

int prim_input(const rp_scene_desc* d, PrimInput& out, std::string& err) {
  const uint32_t n = d->n_hittables;
  if (n > rpl::MAX_PRIMS) { err = "too many hittables for the node encoding"; return RP_EINVAL; }
  if ((uint64_t)n * sizeof(rpl::Prim) > 0xFFFFFFFFull) { err = "too many hittables for 32-bit device offsets"; return RP_EINVAL; }
  std::vector<uint64_t> vbase(d->n_meshes + 1, 0);
  for (uint32_t i = 0; i < d->n_meshes; i++) vbase[i + 1] = vbase[i] + d->meshes[i].n_vertices;
  out.prims.resize(n);
  out.refs.resize(n);
  out.boxes.resize(6 * (size_t)n);
  for (int k = 0; k < 3; k++) {
    out.cmin[k] = std::numeric_limits<double>::infinity();
    out.cmax[k] = -std::numeric_limits<double>::infinity();
  }
  out.amax = 0.0;
  for (uint32_t i = 0; i < n; i++) {
    pack_prim(d, vbase, i, out.prims[i], out.refs[i]);
    const Box b = hittable_box(d, d->hittables[i]);
    for (int k = 0; k < 3; k++) {
      out.boxes[6 * (size_t)i + k] = b.lo[k];
      out.boxes[6 * (size_t)i + 3 + k] = b.hi[k];
      out.amax = std::fmax(out.amax, std::fmax(std::fabs(b.lo[k]), std::fabs(b.hi[k])));
      const double c = 0.5 * (b.lo[k] + b.hi[k]);
      out.cmin[k] = std::fmin(out.cmin[k], c);
      out.cmax[k] = std::fmax(out.cmax[k], c);
    }
  }
  if (!(out.amax <= rpl::COORD_MAX)) {
    err = "primitive coordinates beyond +-2^54 (or infinite) are not supported by the quantized tree";
    return RP_EINVAL;
  }
  return RP_OK;
}

int check(const PackedScene& s, std::string& err) {
  // Every primitive referenced exactly once; every node frame exact and inside qbound (rp_layout.h); every
  // quantized child box contains its subtree's exact f64 primitive boxes; acyclic, no deeper than max_depth.
  std::vector<uint8_t> used(s.prims.size(), 0);
  std::vector<uint8_t> visited(s.nodes.size(), 0);
  size_t np = 0;
  auto prim_box = [&](const rpl::Prim& p, Box& b) {
    if (p.kind == rpl::PRIM_SPHERE) {
      for (int q = 0; q < 3; q++) { b.lo[q] = p.g[q] - p.g[3]; b.hi[q] = p.g[q] + p.g[3]; }
    } else {
      for (int q = 0; q < 3; q++) {
        // b = a - (a - b) up to one rounding: shrink by an ulp-scale slack for the check only
        double a = p.g[q], bq = a - p.g[3 + q], c = a - p.g[6 + q];
        double slack = 4.0 * std::numeric_limits<double>::epsilon() * (std::fabs(a) + std::fabs(p.g[3 + q]) + std::fabs(p.g[6 + q]));
        b.lo[q] = std::fmin(std::fmin(a, bq), c) + slack;
        b.hi[q] = std::fmax(std::fmax(a, bq), c) - slack;
      }
    }
  };
  if (!(s.qbound > 0.0)) { err = "qbound not set"; return RP_EINTERNAL; }
  // subtree box of `entry` into `out`; false (err set) on the first violation
  std::function<bool(uint32_t, uint32_t, Box&)> walk = [&](uint32_t entry, uint32_t depth, Box& out) -> bool {
    out.reset();
    if (entry & rpl::ENTRY_LEAF) {
      uint32_t first = entry & rpl::LEAF_FIRST_MASK, cnt = ((entry >> rpl::LEAF_SHIFT) & 7u) + 1;
      for (uint32_t k = first; k < first + cnt; k++) {
        if (k >= s.prims.size() || used[k]) { err = "primitive referenced twice or out of range"; return false; }
        used[k] = 1;
        np++;
        Box b;
        prim_box(s.prims[k], b);
        out.grow(b);
      }
      return true;
    }
    if (entry >= s.nodes.size()) { err = "node index out of range"; return false; }
    if (visited[entry]) { err = "node visited twice"; return false; }
    visited[entry] = 1;
    if (depth > s.max_depth) { err = "depth exceeds max_depth"; return false; }
    const rpl::Node4& n = s.nodes[entry];
    for (int a = 0; a < 3; a++) {
      if (!(n.s[a] >= 0x1p-60f) || !std::isfinite(n.o[a]) || !(std::fabs((double)n.o[a]) <= s.qbound) ||
          !(255.0 * (double)n.s[a] <= s.qbound)) {
        err = "node frame outside qbound";
        return false;
      }
    }
    const uint8_t* L[3] = {n.lo_x, n.lo_y, n.lo_z};
    const uint8_t* H[3] = {n.hi_x, n.hi_y, n.hi_z};
    for (int c = 0; c < 4; c++) {
      if (n.child[c] == rpl::ENTRY_EMPTY) continue;
      Box sub;
      if (!walk(n.child[c], depth + 1, sub)) return false;
      for (int a = 0; a < 3; a++) {
        if (!(sub.lo[a] <= sub.hi[a])) continue;  // nothing finite below on this axis
        if (!(rpl::plane_q(n.o[a], n.s[a], L[a][c]) <= sub.lo[a]) || !(rpl::plane_q(n.o[a], n.s[a], H[a][c]) >= sub.hi[a])) {
          err = "quantized child box does not contain its subtree";
          return false;
        }
      }
      out.grow(sub);
    }
    return true;
  };
  Box all;
  if (!walk(s.root, 0, all)) return RP_EINTERNAL;
  size_t expect = s.prims.size() - s.n_always;  // the always-tested tail is outside the tree
  if (np != expect && !(np == 0 && s.prims.size() == 1)) {
    err = "primitive count mismatch";
    return RP_EINTERNAL;
  }
  return RP_OK;
}

}  // namespace rpb
