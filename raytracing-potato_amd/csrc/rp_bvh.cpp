// rp_bvh.cpp -- scene validation, binned-SAH BVH2 build, packing into rp_layout.h records.
#include "rp_bvh.h"

#include <algorithm>
#include <atomic>
#include <memory>
#include <thread>
#include <functional>
#include <cmath>
#include <cstring>
#include <limits>

namespace rpb {

namespace {

// Running min / max of an accumulator that is never NaN (it starts at +-inf): a NaN operand leaves it
// unchanged, as fmin / fmax would.  Branch-free (minsd / maxsd): the libm calls gcc emits for std::fmin
// without -ffinite-math-only, and then a branchy inline form, were most of the host SAH build time.
inline double min_(double acc, double v) { return v < acc ? v : acc; }
inline double max_(double acc, double v) { return v > acc ? v : acc; }

// Threads of the host build: the machine's, at most 16 (a GPU box's share of its host).
unsigned build_threads() {
  const unsigned h = std::thread::hardware_concurrency();
  return h == 0 ? 1u : std::min(h, 16u);
}

// f(begin, end) over [0, n) in `threads` contiguous chunks (inline below min_items items).
template <class F>
void parallel_for(size_t n, unsigned threads, F f, size_t min_items = 1u << 16) {
  if (threads <= 1 || n < min_items) { f((size_t)0, n); return; }
  std::vector<std::thread> th;
  const size_t chunk = (n + threads - 1) / threads;
  for (unsigned t = 0; t < threads; t++) {
    const size_t b = t * chunk, e = std::min(n, b + chunk);
    if (b < e) th.emplace_back([=] { f(b, e); });
  }
  for (auto& x : th) x.join();
}

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
      lo[k] = min_(lo[k], b.lo[k]);
      hi[k] = max_(hi[k], b.hi[k]);
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
  unsigned par = 1;  // threads for the centroid-bounds and binning passes of large ranges (ParallelBuild::top)

  // Returns the split position m in (b, e) or b when the range should be a leaf; for a split, lb / rb are
  // the exact boxes of [b, m) and [m, e).  One binning pass over the range for all three axes (then the
  // partition); the child boxes are unions of the chosen side's bins (exact min/max: the same values as a
  // pass over the children).
  uint32_t split(uint32_t b, uint32_t e, const Box& box, Box& lb, Box& rb) {
    uint32_t n = e - b;
    // large ranges: both passes split over `par` threads, partial bounds and bins merged (min / max / sums
    // are order-independent, so the merged values are the serial pass's)
    const unsigned P = (par > 1 && n >= (1u << 18)) ? par : 1u;
    const size_t chunk = (n + P - 1) / P;
    auto run = [&](auto&& f) {
      if (P == 1) { f(0u, b, e); return; }
      std::vector<std::thread> th;
      for (unsigned t = 0; t < P; t++) {
        const uint32_t cb_ = b + (uint32_t)std::min<size_t>(n, t * chunk), ce = b + (uint32_t)std::min<size_t>(n, (t + 1) * chunk);
        th.emplace_back([&f, t, cb_, ce] { f(t, cb_, ce); });
      }
      for (auto& x : th) x.join();
    };
    std::vector<Box> cbp(P);
    run([&](unsigned t, uint32_t lo, uint32_t hi) {
      Box c;
      c.reset();
      for (uint32_t i = lo; i < hi; i++)
        for (int k = 0; k < 3; k++) {
          c.lo[k] = min_(c.lo[k], refs[i].c[k]);
          c.hi[k] = max_(c.hi[k], refs[i].c[k]);
        }
      cbp[t] = c;
    });
    Box cb;
    cb.reset();
    for (const Box& c : cbp) cb.grow(c);
    const uint32_t NB = std::max(2u, std::min(opt.bins, n));
    double scale[3];
    bool live[3];
    for (int ax = 0; ax < 3; ax++) {
      const double ext = cb.hi[ax] - cb.lo[ax];
      live[ax] = ext > 0.0;
      scale[ax] = live[ax] ? (double)NB / ext : 0.0;
    }
    bb_.resize(3 * (size_t)NB);
    bn_.resize(3 * (size_t)NB);
    right_area_.resize(NB);
    right_n_.resize(NB);
    for (uint32_t k = 0; k < 3 * NB; k++) { bb_[k].reset(); bn_[k] = 0; }
    auto bin_of = [&](const Ref& r, int ax) {
      int k = (int)((r.c[ax] - cb.lo[ax]) * scale[ax]);
      return std::min<int>(std::max(k, 0), (int)NB - 1);
    };
    if ((live[0] || live[1] || live[2]) && P == 1) {
      for (uint32_t i = b; i < e; i++)
        for (int ax = 0; ax < 3; ax++) {
          if (!live[ax]) continue;
          const int k = ax * (int)NB + bin_of(refs[i], ax);
          bb_[k].grow(refs[i].box);
          bn_[k]++;
        }
    } else if (live[0] || live[1] || live[2]) {
      std::vector<std::vector<Box>> pb(P, std::vector<Box>(3 * (size_t)NB));
      std::vector<std::vector<uint32_t>> pn(P, std::vector<uint32_t>(3 * (size_t)NB, 0u));
      run([&](unsigned t, uint32_t lo, uint32_t hi) {
        for (Box& x : pb[t]) x.reset();
        for (uint32_t i = lo; i < hi; i++)
          for (int ax = 0; ax < 3; ax++) {
            if (!live[ax]) continue;
            const int k = ax * (int)NB + bin_of(refs[i], ax);
            pb[t][k].grow(refs[i].box);
            pn[t][k]++;
          }
      });
      for (unsigned t = 0; t < P; t++)
        for (uint32_t k = 0; k < 3 * NB; k++) {
          bb_[k].grow(pb[t][k]);
          bn_[k] += pn[t][k];
        }
    }
    double best_cost = std::numeric_limits<double>::infinity();
    int best_axis = -1;
    uint32_t best_bin = 0;
    for (int ax = 0; ax < 3; ax++) {
      if (!live[ax]) continue;
      const Box* bb = &bb_[ax * NB];
      const uint32_t* bn = &bn_[ax * NB];
      Box acc;
      acc.reset();
      uint32_t cnt = 0;
      for (int k = (int)NB - 1; k >= 1; k--) {
        acc.grow(bb[k]);
        cnt += bn[k];
        right_area_[k] = acc.area();
        right_n_[k] = cnt;
      }
      acc.reset();
      cnt = 0;
      for (uint32_t k = 0; k + 1 < NB; k++) {
        acc.grow(bb[k]);
        cnt += bn[k];
        if (cnt == 0 || right_n_[k + 1] == 0) continue;
        double cost = acc.area() * cnt + right_area_[k + 1] * right_n_[k + 1];
        if (cost < best_cost) { best_cost = cost; best_axis = ax; best_bin = k; }
      }
    }
    double parent_area = box.area();
    double leaf_cost = opt.cost_intersect * n;
    if (best_axis >= 0) {
      double split_cost = opt.cost_traverse +
                          (parent_area > 0.0 ? opt.cost_intersect * best_cost / parent_area : opt.cost_intersect * n);
      if (n <= opt.max_leaf && leaf_cost <= split_cost) return b;
      auto mid = std::partition(refs.begin() + b, refs.begin() + e,
                                [&](const Ref& r) { return (uint32_t)bin_of(r, best_axis) <= best_bin; });
      uint32_t m = (uint32_t)(mid - refs.begin());
      if (m > b && m < e) {
        lb.reset();
        rb.reset();
        for (uint32_t k = 0; k < NB; k++) (k <= best_bin ? lb : rb).grow(bb_[best_axis * NB + k]);
        return m;
      }
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
    lb.reset();
    rb.reset();
    for (uint32_t i = b; i < m; i++) lb.grow(refs[i].box);
    for (uint32_t i = m; i < e; i++) rb.grow(refs[i].box);
    return m;
  }

  // Builds range [b, e) whose box is `box` into bin[]; returns its index.
  int32_t build(uint32_t b, uint32_t e, const Box& box) {
    const int32_t self = (int32_t)bin.size();
    bin.emplace_back();
    bin[self].box = box;
    Box lb, rb;
    const uint32_t m = split(b, e, box, lb, rb);
    if (m == b) {
      bin[self].first = (uint32_t)order.size();
      bin[self].count = e - b;
      for (uint32_t i = b; i < e; i++) order.push_back(refs[i].id);
      n_leaves++;
      return self;
    }
    const int32_t l = build(b, m, lb);
    const int32_t r = build(m, e, rb);
    bin[self].left = l;
    bin[self].right = r;
    return self;
  }

  std::vector<Box> bb_;  // split() scratch: NB bins per axis
  std::vector<uint32_t> bn_, right_n_;
  std::vector<double> right_area_;
};

// Parallel form of Builder::build with the identical result.  The top of the tree is split serially-in-
// parallel (the two halves of a large range on two threads) down to ranges of at most `task` primitives;
// those subtrees are built by independent Builders on a thread pool; the pieces are then spliced in the
// serial builder's depth-first order (self, left, right), so node numbers, leaf order and the tree are
// exactly Builder::build's (the split of a range depends only on the range's contents).
struct TopNode {
  Box box;
  uint32_t b = 0, e = 0;
  int kind = 0;  // 0 inner, 1 leaf (a range split() kept whole), 2 task (built by a Builder later)
  std::unique_ptr<TopNode> left, right;
  size_t task = 0;
};

struct ParallelBuild {
  const BuildOptions& opt;
  std::vector<Ref>& refs;
  uint32_t task_max;
  unsigned threads;

  struct Task {
    uint32_t b, e;
    Box box;
    std::vector<BinNode> bin;
    std::vector<uint32_t> order;
    uint64_t n_leaves = 0;
  };
  std::vector<Task> tasks;

  void top(TopNode& t, uint32_t b, uint32_t e, const Box& box, unsigned par) {
    t.box = box;
    t.b = b;
    t.e = e;
    if (e - b <= task_max) { t.kind = 2; return; }
    std::vector<BinNode> scratch_bin;
    std::vector<uint32_t> scratch_order;
    Builder B{opt, refs, scratch_bin, scratch_order};
    B.par = par;
    Box lb, rb;
    const uint32_t m = B.split(b, e, box, lb, rb);
    if (m == b) { t.kind = 1; return; }
    t.left.reset(new TopNode());
    t.right.reset(new TopNode());
    if (par > 1) {
      std::thread th([&] { top(*t.left, b, m, lb, par / 2); });
      top(*t.right, m, e, rb, par - par / 2);
      th.join();
    } else {
      top(*t.left, b, m, lb, 1);
      top(*t.right, m, e, rb, 1);
    }
  }

  void collect(TopNode& t) {
    if (t.kind == 2) {
      t.task = tasks.size();
      tasks.push_back(Task{t.b, t.e, t.box, {}, {}, 0});
    } else if (t.kind == 0) {
      collect(*t.left);
      collect(*t.right);
    }
  }

  // Depth-first numbering of the spliced tree: top nodes are written here, each task's block of nodes and
  // leaf-order entries is reserved at its offsets (copied afterwards, in parallel).
  struct Place { size_t task; int32_t node; uint32_t order, refb; };
  int32_t splice(const TopNode& t, std::vector<BinNode>& bin, uint32_t& n_order, uint64_t& n_leaves,
                 std::vector<Place>& places) {
    const int32_t self = (int32_t)bin.size();
    if (t.kind == 2) {
      const Task& k = tasks[t.task];
      places.push_back(Place{t.task, self, n_order, 0});
      bin.resize(bin.size() + k.bin.size());
      n_order += (uint32_t)k.order.size();
      n_leaves += k.n_leaves;
      return self;
    }
    bin.emplace_back();
    bin[self].box = t.box;
    if (t.kind == 1) {
      bin[self].first = n_order;
      bin[self].count = t.e - t.b;
      n_order += t.e - t.b;
      n_leaves++;
      places.push_back(Place{~(size_t)0, self, bin[self].first, t.b});  // leaf kept whole: ids of refs[b, e)
      return self;
    }
    const int32_t l = splice(*t.left, bin, n_order, n_leaves, places);
    const int32_t r = splice(*t.right, bin, n_order, n_leaves, places);
    bin[self].left = l;
    bin[self].right = r;
    return self;
  }

  uint64_t run(uint32_t n, const Box& all, std::vector<BinNode>& bin, std::vector<uint32_t>& order) {
    TopNode root;
    top(root, 0, n, all, threads);
    collect(root);
    std::atomic<size_t> next{0};
    auto worker = [&] {
      for (size_t i; (i = next.fetch_add(1)) < tasks.size();) {
        Task& k = tasks[i];
        k.bin.reserve(2 * (size_t)(k.e - k.b));
        Builder B{opt, refs, k.bin, k.order};
        B.build(k.b, k.e, k.box);
        k.n_leaves = B.n_leaves;
      }
    };
    std::vector<std::thread> pool;
    for (unsigned t = 1; t < threads; t++) pool.emplace_back(worker);
    worker();
    for (auto& th : pool) th.join();
    uint64_t n_leaves = 0;
    uint32_t n_order = 0;
    std::vector<Place> places;
    splice(root, bin, n_order, n_leaves, places);
    order.resize(n_order);
    parallel_for(places.size(), std::min<unsigned>(threads, (unsigned)places.size()), [&](size_t b, size_t e) {
      for (size_t i = b; i < e; i++) {
        const Place& p = places[i];
        if (p.task == ~(size_t)0) {
          const BinNode& leaf = bin[p.node];
          for (uint32_t k = 0; k < leaf.count; k++) order[p.order + k] = refs[p.refb + k].id;
          continue;
        }
        const Task& k = tasks[p.task];
        for (size_t j = 0; j < k.bin.size(); j++) {
          BinNode n = k.bin[j];
          if (n.leaf()) n.first += p.order;
          else { n.left += p.node; n.right += p.node; }
          bin[p.node + j] = n;
        }
        std::copy(k.order.begin(), k.order.end(), order.begin() + p.order);
      }
    }, 2);
    return n_leaves;
  }
};

// The quantization frame of a wide node from its exact box (rp_layout.h qframe); an axis without a finite
// extent (NaN geometry only) gets the frame at 0.
template <class N>
void node_frame(const Box& b, N& n) {
  for (int a = 0; a < 3; a++) {
    const bool ok = std::isfinite(b.lo[a]) && std::isfinite(b.hi[a]) && b.lo[a] <= b.hi[a];
    rpl::qframe(ok ? b.lo[a] : 0.0, ok ? b.hi[a] : 0.0, n.o[a], n.s[a]);
  }
}

// SAH-optimal choice of a wide node's children (BuildOptions::collapse = COLLAPSE_SAH): the cut through the
// binary subtree under a wide node that minimises the SAH cost of the 4-wide tree (the dynamic program of
// Ylitie et al. 2017 §3, restricted to the binary tree's own leaves).  For a binary node n:
//   E(n)    = its cost as ONE child entry: leaf  A(n) * count * c_prim;  inner  A(n) * c_node + G(n)
//   G(n)    = min_{i=1..3} F(l, i) + F(r, 4 - i)        (the wide node of n: its 4 slots over l and r)
//   F(n, j) = min( min_{i=1..j-1} F(l, i) + F(r, j - i),  E(n) )   (n covered by at most j entries)
// A is the surface area (the parent-relative hit probability up to a constant), c_node / c_prim the builder's
// cost_traverse / cost_intersect.  The greedy rule below (open the largest-area child) fills every slot but
// may spend a slot where a deeper level saves more.  Ties go to the split (a shallower tree), then to the
// smaller i, so the plan is a function of the binary tree alone (any thread count builds the same tree).
struct CollapsePlan {
  // per binary node: choice[j - 1] for j = 1..4 slots: 0 = one entry (n itself), i = i slots to l, j - i to r
  std::vector<uint8_t> choice;
  void build(const std::vector<BinNode>& bin, double c_node, double c_prim) {
    const size_t n = bin.size();
    std::vector<double> F(4 * n);
    choice.assign(4 * n, 0);
    // both binary builders number a node before its children (Builder::build, ParallelBuild::splice: pre-order),
    // so descending ids visit children before parents -- no post-order list (8 B per node) is needed
    for (size_t q = n; q-- > 0;) {
      const int32_t v = (int32_t)q;
      const BinNode& b = bin[v];
      double* f = &F[4 * (size_t)v];
      uint8_t* c = &choice[4 * (size_t)v];
      const double a = b.box.area();
      if (b.leaf()) {
        for (int j = 0; j < 4; j++) { f[j] = a * (double)b.count * c_prim; c[j] = 0; }
        continue;
      }
      const double* fl = &F[4 * (size_t)b.left];
      const double* fr = &F[4 * (size_t)b.right];
      double g = std::numeric_limits<double>::infinity();
      uint8_t gi = 1;
      for (int i = 1; i <= 3; i++)
        if (fl[i - 1] + fr[3 - i] < g) { g = fl[i - 1] + fr[3 - i]; gi = (uint8_t)i; }
      const double e = a * c_node + g;
      f[0] = e;
      c[0] = gi << 4;  // j = 1: n is one entry; the high nibble keeps G's split (n's own wide node)
      for (int j = 2; j <= 4; j++) {
        double best = std::numeric_limits<double>::infinity();
        uint8_t bi = 1;
        for (int i = 1; i < j; i++)
          if (fl[i - 1] + fr[j - i - 1] < best) { best = fl[i - 1] + fr[j - i - 1]; bi = (uint8_t)i; }
        if (e < best) { best = e; bi = 0; }
        f[j - 1] = best;
        c[j - 1] = bi;
      }
    }
  }
  // the wide node of inner binary node bi: its children (binary node ids) in left-to-right order
  int kids(const std::vector<BinNode>& bin, int32_t bi, int32_t out[4]) const {
    int nk = 0;
    const int g = choice[4 * (size_t)bi] >> 4;
    expand(bin, bin[bi].left, g, out, nk);
    expand(bin, bin[bi].right, 4 - g, out, nk);
    return nk;
  }
  void expand(const std::vector<BinNode>& bin, int32_t v, int j, int32_t out[4], int& nk) const {
    const int i = bin[v].leaf() ? 0 : (choice[4 * (size_t)v + (size_t)(j - 1)] & 15);
    if (i == 0) { out[nk++] = v; return; }
    expand(bin, bin[v].left, i, out, nk);
    expand(bin, bin[v].right, j - i, out, nk);
  }
};

// Collapse the binary tree into 4-wide nodes: each wide node takes its binary node's two children and
// repeatedly opens the inner child of largest surface area until it has 4 children (Wald et al.), or
// (COLLAPSE_SAH) takes the SAH-optimal cut of CollapsePlan.
// The wide nodes are written in the scene's node format (child boxes from the exact f64 boxes).
// Numbering: the inner children of a node are consecutive records (a family), and families are laid out
// depth-first -- a ray that enters several children of a node reads neighbouring records (the same or
// the next cache line) instead of records a whole subtree apart.  With par > 1 the inner children's
// subtrees are collapsed on threads into local arrays (local root at 0) whose roots are copied into the
// family's slots and whose descendants are appended in child order: the serial numbering and records.
struct Collapser {
  const std::vector<BinNode>& bin;
  uint32_t fmt;
  unsigned par = 1;
  std::vector<rpl::Node4> nodes;
  std::vector<rpl::Node4Q> qnodes;
  uint32_t max_depth = 0;
  const CollapsePlan* plan = nullptr;  // COLLAPSE_SAH (else the greedy largest-area rule)

  uint32_t size() const { return (uint32_t)(fmt == rpl::NODES_Q8 ? qnodes.size() : nodes.size()); }
  uint32_t* child(uint32_t i) { return fmt == rpl::NODES_Q8 ? qnodes[i].child : nodes[i].child; }
  uint32_t add(uint32_t n = 1) {
    const uint32_t first = size();
    if (fmt == rpl::NODES_Q8) qnodes.resize(qnodes.size() + n);
    else nodes.resize(nodes.size() + n);
    return first;
  }
  // record i of another collapse into slot `dst`, its inner entries shifted by `shift`
  void put(uint32_t dst, Collapser& o, uint32_t i, uint32_t shift) {
    if (fmt == rpl::NODES_Q8) qnodes[dst] = o.qnodes[i];
    else nodes[dst] = o.nodes[i];
    for (int c = 0; c < 4; c++)
      if (!(child(dst)[c] & rpl::ENTRY_LEAF)) child(dst)[c] += shift;
  }

  uint32_t emit_root(int32_t bi) {
    const uint32_t root = add();
    fill(root, bi, 0);
    return root;
  }

  // writes record `self` for binary node bi and, recursively, its descendants
  void fill(uint32_t self, int32_t bi, uint32_t depth) {
    if (depth > max_depth) max_depth = depth;
    int32_t kids[4];
    int nk = 0;
    if (bin[bi].leaf()) {
      kids[nk++] = bi;  // root that is a single leaf
    } else if (plan) {
      nk = plan->kids(bin, bi, kids);
    } else {
      kids[nk++] = bin[bi].left;
      kids[nk++] = bin[bi].right;
      while (nk < 4) {
        int best = -1;
        double area = -1.0;
        for (int k = 0; k < nk; k++)
          if (!bin[kids[k]].leaf() && bin[kids[k]].box.area() > area) { area = bin[kids[k]].box.area(); best = k; }
        if (best < 0) break;
        const int32_t open = kids[best];
        kids[best] = bin[open].left;
        kids[nk++] = bin[open].right;
      }
    }
    if (fmt == rpl::NODES_Q8) {
      rpl::Node4Q& n = qnodes[self];
      Box nb;
      nb.reset();
      for (int k = 0; k < nk; k++) nb.grow(bin[kids[k]].box);
      node_frame(nb, n);
      for (int c = 0; c < 4; c++) {
        if (c < nk) rpl::quantize_child(n, c, bin[kids[c]].box.lo, bin[kids[c]].box.hi);
        else rpl::empty_child(n, c);
      }
    } else {
      rpl::Node4& n = nodes[self];
      for (int c = 0; c < 4; c++) {
        if (c < nk) rpl::f32_child(n, c, bin[kids[c]].box.lo, bin[kids[c]].box.hi);
        else rpl::f32_empty(n, c);
      }
    }
    uint32_t entries[4];
    int inner = 0;
    for (int c = 0; c < 4; c++) {
      if (c >= nk) { entries[c] = rpl::ENTRY_EMPTY; continue; }
      const BinNode& k = bin[kids[c]];
      entries[c] = k.leaf() ? rpl::ENTRY_LEAF | ((k.count - 1) << rpl::LEAF_SHIFT) | k.first : 0u;
      inner += !k.leaf();
    }
    // the family: the inner children's records, consecutive
    const uint32_t fam = inner ? add((uint32_t)inner) : 0u;
    for (int c = 0, j = 0; c < nk; c++)
      if (!bin[kids[c]].leaf()) entries[c] = fam + (uint32_t)j++;
    for (int c = 0; c < 4; c++) child(self)[c] = entries[c];
    if (par > 1 && inner >= 2) {
      std::vector<std::unique_ptr<Collapser>> sub;
      std::vector<std::thread> th;
      for (int c = 0; c < nk; c++) {
        if (bin[kids[c]].leaf()) continue;
        sub.emplace_back(new Collapser{bin, fmt, std::max(1u, par / (unsigned)inner), {}, {}, 0, plan});
        Collapser* sc = sub.back().get();
        const int32_t kb = kids[c];
        th.emplace_back([sc, kb] { sc->emit_root(kb); });
      }
      for (auto& t : th) t.join();
      for (int j = 0; j < inner; j++) {
        // local record 0 -> family slot; local records 1.. -> appended at `base` (local i -> base + i - 1)
        Collapser& sc = *sub[j];
        const uint32_t base = size();
        const uint32_t n = sc.size();
        put(fam + (uint32_t)j, sc, 0, base - 1u);
        add(n - 1u);
        for (uint32_t i = 1; i < n; i++) put(base + i - 1u, sc, i, base - 1u);
        max_depth = std::max(max_depth, depth + 1 + sc.max_depth);
      }
    } else {
      for (int c = 0, j = 0; c < nk; c++)
        if (!bin[kids[c]].leaf()) fill(fam + (uint32_t)j++, kids[c], depth + 1);
    }
  }
};

// Collapse the binary tree into 8-wide quantized nodes (rp_layout.h Node8Q): the same opening rule as Collapser
// up to 8 children; each child goes to the slot of the octant its box centre lies in relative to the node's
// centre (greedy assignment by the largest alignment of centre offset and slot direction, Ylitie et al. 2017), so
// that a ray's rank order slot ^ octant approximates near-first.  Records are numbered in families as in
// Collapser (inner children consecutive, in slot order); the leaf children's primitives are re-laid out as one
// run per node in slot order (`prims`: positions in the binary tree's leaf order), depth-first.  With par > 1 the
// inner children's subtrees are collapsed on threads and spliced: the serial numbering, records and run order.
struct Collapser8 {
  const std::vector<BinNode>& bin;
  const std::vector<uint32_t>& leaf_order;  // binary leaf order: BinNode first/count index it
  unsigned par = 1;
  std::vector<rpl::Node8Q> nodes;
  std::vector<uint32_t> prims;  // hittable ids in the new leaf order
  uint32_t max_depth = 0;

  uint32_t emit_root(int32_t bi) {
    nodes.emplace_back();
    fill(0, bi, 0);
    return 0;
  }
  // record i of another collapse into slot `dst`, its family index shifted by `ns` and its run by `ps`
  void put(uint32_t dst, const Collapser8& o, uint32_t i, uint32_t ns, uint32_t ps) {
    rpl::Node8Q n = o.nodes[i];
    if (n.inner >> 24) n.inner = (n.inner & ~rpl::W8_INDEX) | (((n.inner & rpl::W8_INDEX) + ns) & rpl::W8_INDEX);
    n.prim += ps;
    nodes[dst] = n;
  }

  void fill(uint32_t self, int32_t bi, uint32_t depth) {
    if (depth > max_depth) max_depth = depth;
    int32_t kids[8];
    int nk = 0;
    if (bin[bi].leaf()) {
      kids[nk++] = bi;
    } else {
      kids[nk++] = bin[bi].left;
      kids[nk++] = bin[bi].right;
      while (nk < 8) {
        int best = -1;
        double area = -1.0;
        for (int k = 0; k < nk; k++)
          if (!bin[kids[k]].leaf() && bin[kids[k]].box.area() > area) { area = bin[kids[k]].box.area(); best = k; }
        if (best < 0) break;
        const int32_t open = kids[best];
        kids[best] = bin[open].left;
        kids[nk++] = bin[open].right;
      }
    }
    Box nb;
    nb.reset();
    for (int k = 0; k < nk; k++) nb.grow(bin[kids[k]].box);
    // slot assignment: greedy on score(k, s) = sum over axes of +-(centre_k - centre_node)
    int32_t at[8];
    for (int s = 0; s < 8; s++) at[s] = -1;
    {
      double sc[8][8];
      for (int k = 0; k < nk; k++) {
        double v[3];
        for (int a = 0; a < 3; a++) v[a] = 0.5 * (bin[kids[k]].box.lo[a] + bin[kids[k]].box.hi[a]) - 0.5 * (nb.lo[a] + nb.hi[a]);
        for (int s = 0; s < 8; s++) {
          double t = 0.0;
          for (int a = 0; a < 3; a++) t += (s >> a & 1) ? v[a] : -v[a];
          sc[k][s] = t == t ? t : 0.0;  // NaN geometry: no preference
        }
      }
      bool used_k[8] = {false, false, false, false, false, false, false, false};
      for (int round = 0; round < nk; round++) {
        int bk = -1, bs = -1;
        double bv = -HUGE_VAL;
        for (int k = 0; k < nk; k++) {
          if (used_k[k]) continue;
          for (int s = 0; s < 8; s++)
            if (at[s] < 0 && (bk < 0 || sc[k][s] > bv)) { bv = sc[k][s]; bk = k; bs = s; }
        }
        used_k[bk] = true;
        at[bs] = bk;
      }
    }
    rpl::Node8Q& n = nodes[self];
    node_frame(nb, n);
    n.prim = (uint32_t)prims.size();
    uint32_t imask = 0, off = 0;
    for (int s = 0; s < 8; s++) {
      n.pmask[s] = 0;
      if (at[s] < 0) { rpl::empty_child(n, s); continue; }
      const BinNode& k = bin[kids[at[s]]];
      rpl::quantize_child(n, s, k.box.lo, k.box.hi);
      if (k.leaf()) {
        n.pmask[s] = (uint32_t)(((1ull << k.count) - 1ull) << off);
        for (uint32_t q = 0; q < k.count; q++) prims.push_back(leaf_order[k.first + q]);
        off += k.count;
      } else {
        imask |= 1u << s;
      }
    }
    for (int q = 0; q < 4; q++) n.pad[q] = 0;
    const uint32_t inner = (uint32_t)__builtin_popcount(imask);
    const uint32_t fam = inner ? (uint32_t)nodes.size() : 0u;
    if (inner) nodes.resize(nodes.size() + inner);
    nodes[self].inner = (fam & rpl::W8_INDEX) | imask << 24;  // (nodes may have moved)
    if (par > 1 && inner >= 2) {
      std::vector<std::unique_ptr<Collapser8>> sub;
      std::vector<std::thread> th;
      for (int s = 0; s < 8; s++) {
        if (!(imask >> s & 1u)) continue;
        sub.emplace_back(new Collapser8{bin, leaf_order, std::max(1u, par / inner), {}, {}, 0});
        Collapser8* sc = sub.back().get();
        const int32_t kb = kids[at[s]];
        th.emplace_back([sc, kb] { sc->emit_root(kb); });
      }
      for (auto& t : th) t.join();
      for (uint32_t j = 0; j < inner; j++) {
        Collapser8& sc = *sub[j];
        const uint32_t base = (uint32_t)nodes.size();
        const uint32_t pbase = (uint32_t)prims.size();
        const uint32_t m = (uint32_t)sc.nodes.size();
        nodes.resize(nodes.size() + m - 1u);
        put(fam + j, sc, 0, base - 1u, pbase);
        for (uint32_t i = 1; i < m; i++) put(base + i - 1u, sc, i, base - 1u, pbase);
        prims.insert(prims.end(), sc.prims.begin(), sc.prims.end());
        max_depth = std::max(max_depth, depth + 1 + sc.max_depth);
      }
    } else {
      for (int s = 0, j = 0; s < 8; s++)
        if (imask >> s & 1u) fill(fam + (uint32_t)j++, kids[at[s]], depth + 1);
    }
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
  // the kernel carries a hit's material in 31 bits beside its primitive kind (rp_device.h HitRec::km)
  if (d->n_materials >= 0x7FFFFFFFu) return fail("too many materials (>= 2^31 - 1)");
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

static void pack_prim(const rp_scene_desc* d, const std::vector<uint64_t>& vbase, uint32_t id, rpl::Prim& p,
                      rpl::PrimRef& pr);

int build(const rp_scene_desc* d, const BuildOptions& opt, PackedScene& out, std::string& err) {
  out = PackedScene();
  const unsigned threads = opt.threads ? opt.threads : build_threads();
  // ---- shading tables
  std::vector<uint64_t> vbase(d->n_meshes + 1, 0);
  for (uint32_t i = 0; i < d->n_meshes; i++) vbase[i + 1] = vbase[i] + d->meshes[i].n_vertices;
  if (vbase[d->n_meshes] > 0xffffffffull) { err = "too many vertices"; return RP_EINVAL; }
  if (opt.vertex_tables) {
    out.vnrm.resize(3 * vbase[d->n_meshes] + 3);
    out.vuv.resize(2 * vbase[d->n_meshes] + 2);
  }
  for (uint32_t i = 0; i < d->n_meshes && opt.vertex_tables; i++) {
    const rp_mesh& m = d->meshes[i];
    // vertex runs in parallel chunks (C5: 30 M vertices, 1.2 GB)
    parallel_for(m.n_vertices, threads, [&](size_t b, size_t e) {
      std::memcpy(&out.vnrm[3 * (vbase[i] + b)], m.normals + 3 * b, sizeof(double) * 3 * (e - b));
      std::memcpy(&out.vuv[2 * (vbase[i] + b)], m.uvs + 2 * b, sizeof(double) * 2 * (e - b));
    });
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
  if (opt.node_format > rpl::NODES_W8) { err = "unknown node format"; return RP_EINVAL; }

  // ---- BVH over all hittables (a List root is served by the same tree: closest hit is
  //      independent of visit order except exact-t ties)
  uint32_t n = d->n_hittables;
  if (n > rpl::MAX_PRIMS) { err = "too many hittables for the node encoding"; return RP_EINVAL; }
  // the kernels address primitives and wide nodes by 32-bit byte offsets (<= n nodes of 128 B)
  if ((uint64_t)n * sizeof(rpl::Prim) > 0xFFFFFFFFull) { err = "too many hittables for 32-bit device offsets"; return RP_EINVAL; }
  if (opt.max_leaf < 1 || opt.max_leaf > rpl::LEAF_MAX) { err = "max_leaf out of range"; return RP_EINVAL; }
  std::vector<Ref> refs(n);
  parallel_for(n, threads, [&](size_t b, size_t e) {
    for (size_t i = b; i < e; i++) {
      refs[i].box = hittable_box(d, d->hittables[i]);
      for (int k = 0; k < 3; k++) refs[i].c[k] = 0.5 * (refs[i].box.lo[k] + refs[i].box.hi[k]);
      refs[i].id = (uint32_t)i;
    }
  });
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
    for (int k = 0; k < 3; k++) amax = max_(max_(amax, std::fabs(r.box.lo[k])), std::fabs(r.box.hi[k]));
  out.node_format = opt.node_format ? opt.node_format : auto_node_format(d->n_hittables, amax);
  if (out.node_format == rpl::NODES_W8 && opt.max_leaf > rpl::W8_MAX_LEAF) {
    err = "the 8-wide nodes hold leaves of at most 4 primitives (max_leaf <= 4)";
    return RP_EINVAL;
  }
  if (out.node_format != rpl::NODES_F32 && !(amax <= rpl::COORD_MAX)) {
    err = "primitive coordinates beyond +-2^54 (or infinite) are not supported by the quantized nodes";
    return RP_EINVAL;
  }
  out.qbound = rpl::qbound(amax);
  std::vector<uint32_t> order;
  order.reserve(n);
  std::vector<BinNode> bin;
  bin.reserve(n_tree ? 2 * (size_t)n_tree : 1);
  Builder B{opt, refs, bin, order};
  if (n_tree == 0) {
    if (out.node_format == rpl::NODES_W8) {
      rpl::Node8Q root{};
      for (int a = 0; a < 3; a++) rpl::qframe(0.0, 0.0, root.o[a], root.s[a]);
      for (int c = 0; c < 8; c++) rpl::empty_child(root, c);
      out.wnodes.push_back(root);
    } else if (out.node_format == rpl::NODES_Q8) {
      rpl::Node4Q root{};
      for (int a = 0; a < 3; a++) rpl::qframe(0.0, 0.0, root.o[a], root.s[a]);
      for (int c = 0; c < 4; c++) {
        rpl::empty_child(root, c);
        root.child[c] = rpl::ENTRY_EMPTY;
      }
      out.qnodes.push_back(root);
    } else {
      rpl::Node4 root{};
      for (int c = 0; c < 4; c++) {
        rpl::f32_empty(root, c);
        root.child[c] = rpl::ENTRY_EMPTY;
      }
      out.nodes.push_back(root);
    }
    out.max_depth = 0;
  } else {
    Box all;
    all.reset();
    for (auto& r : refs) all.grow(r.box);
    // large trees: the parallel form (identical tree); tasks of ~n/256 primitives, at least 16 k
    if (n_tree >= (1u << 16) && threads > 1) {
      ParallelBuild P{opt, refs, std::max<uint32_t>(n_tree / 256, 1u << 14), threads, {}};
      B.n_leaves = P.run(n_tree, all, bin, order);
    } else {
      B.build(0, n_tree, all);
    }
    if (out.node_format == rpl::NODES_W8) {
      Collapser8 C{bin, order, threads, {}, {}, 0};
      C.nodes.reserve(bin.size() / 6 + 1);
      C.prims.reserve(order.size());
      C.emit_root(0);
      if (C.nodes.size() > rpl::W8_MAX_NODES) { err = "too many 8-wide nodes (> 2^24)"; return RP_EINVAL; }
      out.wnodes.swap(C.nodes);
      order.swap(C.prims);  // the tree's primitives in the 8-wide leaf order
      out.max_depth = C.max_depth;
    } else {
      CollapsePlan plan;
      if (opt.collapse == COLLAPSE_SAH) plan.build(bin, opt.cost_traverse, opt.cost_intersect);
      Collapser C{bin, out.node_format, threads, {}, {}, 0, opt.collapse == COLLAPSE_SAH ? &plan : nullptr};
      if (out.node_format == rpl::NODES_Q8) C.qnodes.reserve(bin.size() / 2 + 1);
      else C.nodes.reserve(bin.size() / 2 + 1);
      C.emit_root(0);
      out.nodes.swap(C.nodes);
      out.qnodes.swap(C.qnodes);
      out.max_depth = C.max_depth;
    }
  }
  out.root = 0;
  out.n_leaves = B.n_leaves;
  out.always_first = (uint32_t)order.size();
  out.n_always = (uint32_t)always.size();
  for (uint32_t a : always) order.push_back(a);

  // ---- primitives in leaf order (value-initialised: a scene without primitives keeps one zero record)
  out.prims.resize(order.size() ? order.size() : 1);
  out.prim_refs.resize(out.prims.size());
  parallel_for(order.size(), threads, [&](size_t b, size_t e) {
    for (size_t k = b; k < e; k++) pack_prim(d, vbase, order[k], out.prims[k], out.prim_refs[k]);
  });
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
  // chunks on up to 16 threads (the per-chunk bounds merge by min / max: the same values as one pass)
  const unsigned T = n >= (1u << 16) ? std::max(1u, std::min(16u, std::thread::hardware_concurrency())) : 1u;
  std::vector<double> part(7 * (size_t)T);
  auto run = [&](unsigned t) {
    const uint32_t lo = (uint32_t)((uint64_t)n * t / T), hi = (uint32_t)((uint64_t)n * (t + 1) / T);
    double cmn[3] = {INFINITY, INFINITY, INFINITY}, cmx[3] = {-INFINITY, -INFINITY, -INFINITY}, am = 0.0;
    for (uint32_t i = lo; i < hi; i++) {
      pack_prim(d, vbase, i, out.prims[i], out.refs[i]);
      const Box b = hittable_box(d, d->hittables[i]);
      for (int k = 0; k < 3; k++) {
        out.boxes[6 * (size_t)i + k] = b.lo[k];
        out.boxes[6 * (size_t)i + 3 + k] = b.hi[k];
        am = std::fmax(am, std::fmax(std::fabs(b.lo[k]), std::fabs(b.hi[k])));
        const double c = 0.5 * (b.lo[k] + b.hi[k]);
        cmn[k] = std::fmin(cmn[k], c);
        cmx[k] = std::fmax(cmx[k], c);
      }
    }
    double* q = &part[7 * (size_t)t];
    for (int k = 0; k < 3; k++) { q[k] = cmn[k]; q[3 + k] = cmx[k]; }
    q[6] = am;
  };
  if (T == 1) {
    run(0);
  } else {
    std::vector<std::thread> th;
    for (unsigned t = 0; t < T; t++) th.emplace_back(run, t);
    for (auto& x : th) x.join();
  }
  for (unsigned t = 0; t < T; t++) {
    const double* q = &part[7 * (size_t)t];
    for (int k = 0; k < 3; k++) {
      out.cmin[k] = std::fmin(out.cmin[k], q[k]);
      out.cmax[k] = std::fmax(out.cmax[k], q[3 + k]);
    }
    out.amax = std::fmax(out.amax, q[6]);
  }
  return RP_OK;
}

int check(const PackedScene& s, std::string& err) {
  // Every primitive referenced exactly once; every stored child box (f32, or quantized in a frame inside
  // qbound, rp_layout.h) contains its subtree's exact f64 primitive boxes; acyclic, no deeper than max_depth.
  std::vector<uint8_t> used(s.prims.size(), 0);
  std::vector<uint8_t> visited(s.n_nodes(), 0);
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
  if (s.node_format != rpl::NODES_F32 && !(s.qbound > 0.0)) { err = "qbound not set"; return RP_EINTERNAL; }
  auto frame_ok = [&](const float* o, const float* sc) {
    for (int a = 0; a < 3; a++)
      if (!(sc[a] >= 0x1p-60f) || !std::isfinite(o[a]) || !(std::fabs((double)o[a]) <= s.qbound) ||
          !(255.0 * (double)sc[a] <= s.qbound))
        return false;
    return true;
  };
  // 8-wide tree: inner children at inner + rank in imask, leaf children's primitives as pmask bits of the run
  std::function<bool(uint32_t, uint32_t, Box&)> walk8 = [&](uint32_t node, uint32_t depth, Box& out) -> bool {
    out.reset();
    if (node >= s.wnodes.size()) { err = "node index out of range"; return false; }
    if (visited[node]) { err = "node visited twice"; return false; }
    visited[node] = 1;
    if (depth > s.max_depth) { err = "depth exceeds max_depth"; return false; }
    const rpl::Node8Q& n = s.wnodes[node];
    if (!frame_ok(n.o, n.s)) { err = "node frame outside qbound"; return false; }
    const uint32_t imask = n.inner >> 24;
    const uint8_t* L[3] = {n.lo_x, n.lo_y, n.lo_z};
    const uint8_t* H[3] = {n.hi_x, n.hi_y, n.hi_z};
    uint32_t seen = 0;
    for (int c = 0; c < 8; c++) {
      const bool inner = imask >> c & 1u;
      if (inner && n.pmask[c]) { err = "slot both inner and leaf"; return false; }
      if (n.pmask[c] & seen) { err = "overlapping leaf runs"; return false; }
      seen |= n.pmask[c];
      if (!inner && !n.pmask[c]) continue;
      Box sub;
      if (inner) {
        const uint32_t ch = (n.inner & rpl::W8_INDEX) + (uint32_t)__builtin_popcount(imask & ((1u << c) - 1u));
        if (!walk8(ch, depth + 1, sub)) return false;
      } else {
        sub.reset();
        if (__builtin_popcount(n.pmask[c]) > (int)rpl::W8_MAX_LEAF) { err = "leaf too large"; return false; }
        for (uint32_t m = n.pmask[c]; m; m &= m - 1u) {
          const uint64_t k = (uint64_t)n.prim + (uint32_t)__builtin_ctz(m);
          if (k >= s.prims.size() || used[k]) { err = "primitive referenced twice or out of range"; return false; }
          used[k] = 1;
          np++;
          Box b;
          prim_box(s.prims[k], b);
          sub.grow(b);
        }
      }
      for (int a = 0; a < 3; a++) {
        if (!(sub.lo[a] <= sub.hi[a])) continue;
        if (!(rpl::plane_q(n.o[a], n.s[a], L[a][c]) <= sub.lo[a]) || !(rpl::plane_q(n.o[a], n.s[a], H[a][c]) >= sub.hi[a])) {
          err = "child box does not contain its subtree";
          return false;
        }
      }
      out.grow(sub);
    }
    return true;
  };
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
    if (entry >= s.n_nodes()) { err = "node index out of range"; return false; }
    if (visited[entry]) { err = "node visited twice"; return false; }
    visited[entry] = 1;
    if (depth > s.max_depth) { err = "depth exceeds max_depth"; return false; }
    const uint32_t* child;
    double plo[4][3], phi[4][3];  // the stored child box planes, exact in f64
    if (s.node_format == rpl::NODES_Q8) {
      const rpl::Node4Q& n = s.qnodes[entry];
      if (!frame_ok(n.o, n.s)) { err = "node frame outside qbound"; return false; }
      const uint8_t* L[3] = {n.lo_x, n.lo_y, n.lo_z};
      const uint8_t* H[3] = {n.hi_x, n.hi_y, n.hi_z};
      for (int c = 0; c < 4; c++)
        for (int a = 0; a < 3; a++) {
          plo[c][a] = rpl::plane_q(n.o[a], n.s[a], L[a][c]);
          phi[c][a] = rpl::plane_q(n.o[a], n.s[a], H[a][c]);
        }
      child = n.child;
    } else {
      const rpl::Node4& n = s.nodes[entry];
      for (int c = 0; c < 4; c++) {
        plo[c][0] = n.lo_x[c]; plo[c][1] = n.lo_y[c]; plo[c][2] = n.lo_z[c];
        phi[c][0] = n.hi_x[c]; phi[c][1] = n.hi_y[c]; phi[c][2] = n.hi_z[c];
      }
      child = n.child;
    }
    for (int c = 0; c < 4; c++) {
      if (child[c] == rpl::ENTRY_EMPTY) continue;
      Box sub;
      if (!walk(child[c], depth + 1, sub)) return false;
      for (int a = 0; a < 3; a++) {
        if (!(sub.lo[a] <= sub.hi[a])) continue;  // nothing finite below on this axis
        if (!(plo[c][a] <= sub.lo[a]) || !(phi[c][a] >= sub.hi[a])) {
          err = "child box does not contain its subtree";
          return false;
        }
      }
      out.grow(sub);
    }
    return true;
  };
  Box all;
  if (!(s.node_format == rpl::NODES_W8 ? walk8(s.root, 0, all) : walk(s.root, 0, all))) return RP_EINTERNAL;
  size_t expect = s.prims.size() - s.n_always;  // the always-tested tail is outside the tree
  if (np != expect && !(np == 0 && s.prims.size() == 1)) {
    err = "primitive count mismatch";
    return RP_EINTERNAL;
  }
  return RP_OK;
}

}  // namespace rpb
