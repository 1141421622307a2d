// rt_bvh.cpp — host-side world-BVH rebuild (binned SAH) for the device traversal.
//
// The reference's makeBVH (src/Lib.hs:941-961) splits at the median of a random axis after a
// stable sort by box minimum, so boxes become long strips and a huge primitive (the r = 1000
// ground sphere of the book-one scenes) sits on one spine at every level. For a world tree with
// no ConstantMedium in it, the closest hit over the tree (hit, src/Lib.hs:970-1109) does not
// depend on the tree's shape except for exact ties (two primitives at bit-identical t): every
// leaf's own hit test is unchanged, and boxes only cull. So the device may traverse a better
// tree over the SAME leaves (spheres, rects, cuboids, instance sub-DAGs, moving spheres, each
// bounded exactly as boundingBox bounds it). Media are leaves too: their tier-B draws are keyed per
// occurrence (unfold_media) and their candidate hit does not depend on the walk's bound (DESIGN.md
// §3.2). The lights tree is never touched (its BVH sizes weight htblPdfValue / htblRandom,
// src/Lib.hs:694-723).
#include <algorithm>
#include <array>
#include <cstdlib>
#include <string>
#include <cmath>
#include <functional>
#include <vector>

#include "rt.h"
#include "rt_internal.h"
#include "rt_wide.h"

namespace rt {

namespace {

constexpr double kEps = 0.0001;
constexpr int kMaxStackNeed = 30;  // RT_STACK - 2 (rt_device.h): the upload validator's bound
inline double gmax(double x, double y) { return x <= y ? y : x; }
inline double gmin(double x, double y) { return x <= y ? x : y; }

struct Builder {
  std::vector<rt_node>& nodes;
  int bins = 64;  // SAH centroid bins per axis (C5: 96.3 wide-node visits per sample vs 99.8 at 16)
  std::vector<Box> boxes;  // per leaf
  std::vector<int> leaf_ids;
  std::vector<double> cx[3];

  int emit_bvh(int l, int r, const Box& b, int axis) {
    rt_node n{};
    for (int i = 0; i < 3; ++i) {
      n.f[i] = b.mn[i];
      n.f[3 + i] = b.mx[i];
    }
    n.type = RT_NODE_BVH;
    n.a = l;
    n.b = r;
    n.c = RT_BVH_ORDERED | axis;  // world-only node: `c` carries the split axis, not htblSize
    nodes.push_back(n);
    return (int)nodes.size() - 1;
  }

  static Box merge(const Box& a, const Box& b) {
    Box o;
    for (int i = 0; i < 3; ++i) {
      o.mn[i] = std::min(a.mn[i], b.mn[i]);
      o.mx[i] = std::max(a.mx[i], b.mx[i]);
    }
    return o;
  }
  static double area(const Box& b) {
    const double dx = b.mx[0] - b.mn[0], dy = b.mx[1] - b.mn[1], dz = b.mx[2] - b.mn[2];
    return 2.0 * (dx * dy + dy * dz + dz * dx);
  }

  // Build over items[lo, hi); returns the node id and its box.
  int build(std::vector<int>& items, int lo, int hi, Box& out) {
    const int n = hi - lo;
    if (n == 1) {
      out = boxes[items[lo]];
      return leaf_ids[items[lo]];
    }
    Box bb = boxes[items[lo]], cb;
    for (int a = 0; a < 3; ++a) cb.mn[a] = cb.mx[a] = cx[a][items[lo]];
    for (int i = lo + 1; i < hi; ++i) {
      bb = merge(bb, boxes[items[i]]);
      for (int a = 0; a < 3; ++a) {
        cb.mn[a] = std::min(cb.mn[a], cx[a][items[i]]);
        cb.mx[a] = std::max(cb.mx[a], cx[a][items[i]]);
      }
    }
    int mid = lo + n / 2;
    int split_axis = 0;
    {
      double best_ext = -1;
      for (int a = 0; a < 3; ++a)
        if (cb.mx[a] - cb.mn[a] > best_ext) { best_ext = cb.mx[a] - cb.mn[a]; split_axis = a; }
    }
    if (n > 2 && bins == 0) {  // full sweep: every split between centroid-sorted items, each axis
      double best = INFINITY;
      int best_axis = -1, best_k = 0;
      std::vector<int> ord(items.begin() + lo, items.begin() + hi);
      std::vector<double> right(n);
      for (int a = 0; a < 3; ++a) {
        std::stable_sort(ord.begin(), ord.end(), [&](int x, int y) { return cx[a][x] < cx[a][y]; });
        Box acc = boxes[ord[n - 1]];
        for (int k = n - 1; k > 0; --k) {  // right[k] = area of items k..n-1
          acc = merge(acc, boxes[ord[k]]);
          right[k] = area(acc);
        }
        acc = boxes[ord[0]];
        for (int k = 1; k < n; ++k) {  // left = items 0..k-1
          if (k > 1) acc = merge(acc, boxes[ord[k - 1]]);
          const double cost = area(acc) * k + right[k] * (n - k);
          if (cost < best) {
            best = cost;
            best_axis = a;
            best_k = k;
          }
        }
      }
      if (best_axis >= 0) {
        const int a = best_axis;
        split_axis = a;
        std::stable_sort(items.begin() + lo, items.begin() + hi,
                         [&](int x, int y) { return cx[a][x] < cx[a][y]; });
        mid = lo + best_k;
      }
    } else if (n > 2) {
      const int kBins = bins;
      double best = INFINITY;
      int best_axis = -1, best_bin = 0;
      for (int a = 0; a < 3; ++a) {
        const double ext = cb.mx[a] - cb.mn[a];
        if (!(ext > 0)) continue;
        std::vector<Box> bin_box(kBins);
        std::vector<int> bin_cnt(kBins, 0);
        for (int i = lo; i < hi; ++i) {
          int k = (int)((cx[a][items[i]] - cb.mn[a]) / ext * kBins);
          k = std::min(kBins - 1, std::max(0, k));
          bin_box[k] = bin_cnt[k] ? merge(bin_box[k], boxes[items[i]]) : boxes[items[i]];
          ++bin_cnt[k];
        }
        // sweep: cost(split after bin k) = A_left * N_left + A_right * N_right
        std::vector<double> right_area(kBins);
        std::vector<int> right_cnt(kBins);
        Box acc;
        int cnt = 0;
        for (int k = kBins - 1; k > 0; --k) {
          if (bin_cnt[k]) {
            acc = cnt ? merge(acc, bin_box[k]) : bin_box[k];
            cnt += bin_cnt[k];
          }
          right_area[k] = cnt ? area(acc) : 0.0;
          right_cnt[k] = cnt;
        }
        cnt = 0;
        for (int k = 0; k < kBins - 1; ++k) {
          if (bin_cnt[k]) {
            acc = cnt ? merge(acc, bin_box[k]) : bin_box[k];
            cnt += bin_cnt[k];
          }
          if (!cnt || !right_cnt[k + 1]) continue;
          const double cost = area(acc) * cnt + right_area[k + 1] * right_cnt[k + 1];
          if (cost < best) {
            best = cost;
            best_axis = a;
            best_bin = k;
          }
        }
      }
      if (best_axis >= 0) {
        const int a = best_axis;
        split_axis = a;
        const double ext = cb.mx[a] - cb.mn[a];
        auto it = std::stable_partition(items.begin() + lo, items.begin() + hi, [&](int i) {
          int k = (int)((cx[a][i] - cb.mn[a]) / ext * kBins);
          k = std::min(kBins - 1, std::max(0, k));
          return k <= best_bin;
        });
        mid = (int)(it - items.begin());
        if (mid == lo || mid == hi) mid = lo + n / 2;
      }
    }
    Box bl, br;
    const int l = build(items, lo, mid, bl);
    const int r = build(items, mid, hi, br);
    out = merge(bl, br);
    if (n == 2) {  // two leaves: order them along the axis their centroids differ most
      double best_d = -1;
      for (int a = 0; a < 3; ++a) {
        const double dd = std::fabs(cx[a][items[lo]] - cx[a][items[lo + 1]]);
        if (dd > best_d) { best_d = dd; split_axis = a; }
      }
      if (cx[split_axis][items[lo]] > cx[split_axis][items[lo + 1]]) {
        return emit_bvh(r, l, out, split_axis);
      }
    }
    return emit_bvh(l, r, out, split_axis);
  }
};

}  // namespace

// boundingBox (src/Lib.hs:905-927) over the flat node array (Rotate's box re-derived with its
// 3x3x3 corner fold, exactly as `rotate` computes it at construction).
bool flat_box(const std::vector<rt_node>& nodes, int id, Box* out) {
  const rt_node& n = nodes[id];
  switch (n.type) {
    case RT_NODE_SPHERE:
      for (int i = 0; i < 3; ++i) { out->mn[i] = n.f[i] - n.f[3]; out->mx[i] = n.f[i] + n.f[3]; }
      return true;
    case RT_NODE_MOVING_SPHERE: {
      const double r = nodes[id + 1].f[3];
      for (int i = 0; i < 3; ++i) {
        out->mn[i] = gmin(n.f[i] - r, n.f[3 + i] - r);
        out->mx[i] = gmax(n.f[i] + r, n.f[3 + i] + r);
      }
      return true;
    }
    case RT_NODE_RECT_XY:
      out->mn[0] = n.f[0]; out->mn[1] = n.f[2]; out->mn[2] = n.f[4] - kEps;
      out->mx[0] = n.f[1]; out->mx[1] = n.f[3]; out->mx[2] = n.f[4] + kEps;
      return true;
    case RT_NODE_RECT_XZ:
      out->mn[0] = n.f[0]; out->mn[1] = n.f[4] - kEps; out->mn[2] = n.f[2];
      out->mx[0] = n.f[1]; out->mx[1] = n.f[4] + kEps; out->mx[2] = n.f[3];
      return true;
    case RT_NODE_RECT_YZ:
      out->mn[0] = n.f[4] - kEps; out->mn[1] = n.f[0]; out->mn[2] = n.f[2];
      out->mx[0] = n.f[4] + kEps; out->mx[1] = n.f[1]; out->mx[2] = n.f[3];
      return true;
    case RT_NODE_BVH:
    case RT_NODE_CUBOID:
      for (int i = 0; i < 3; ++i) { out->mn[i] = n.f[i]; out->mx[i] = n.f[3 + i]; }
      return true;
    case RT_NODE_TRANSLATE: {
      Box c;
      if (!flat_box(nodes, n.a, &c)) return false;
      for (int i = 0; i < 3; ++i) { out->mn[i] = c.mn[i] + n.f[i]; out->mx[i] = c.mx[i] + n.f[i]; }
      return true;
    }
    case RT_NODE_ROTATE: {
      Box hb;
      if (!flat_box(nodes, n.a, &hb)) return false;
      const double s = n.f[0], c = n.f[1];
      double mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
      // The reference's `rotate` bounds the rotated child over the points i, j, k in {0, 1, 2}
      // (src/Lib.hs:732-761): the corners and points extrapolated a whole box extent beyond them, a box
      // 3x as wide per axis. The re-bounded trees' boxes only cull (ties are redone on the caller's tree,
      // which keeps the reference's boxes), so they bound the child by its 8 corners (rotation is
      // linear), widened by 2^-30 of the magnitudes against rounding (round 6: the 1000-sphere frame of
      // next_week_final was opened by every ray through its 27-times-larger box). RTAMD_TIGHT_ROTATE=0
      // keeps the reference's box.
      static const bool tight = !(std::getenv("RTAMD_TIGHT_ROTATE") && std::getenv("RTAMD_TIGHT_ROTATE")[0] == '0');
      for (int idx = 26; idx >= 0; --idx) {
        const double i = idx / 9, j = (idx / 3) % 3, k = idx % 3;
        if (tight && (i > 1 || j > 1 || k > 1)) continue;
        const double p0 = i * hb.mx[0] + (1 - i) * hb.mn[0], p1 = j * hb.mx[1] + (1 - j) * hb.mn[1],
                     p2 = k * hb.mx[2] + (1 - k) * hb.mn[2];
        double q[3];
        if (n.b == 0) { q[0] = p0; q[1] = c * p1 - s * p2; q[2] = s * p1 + c * p2; }
        else if (n.b == 1) { q[0] = c * p0 + s * p2; q[1] = p1; q[2] = -s * p0 + c * p2; }
        else { q[0] = c * p0 - s * p1; q[1] = s * p0 + c * p1; q[2] = p2; }
        for (int a = 0; a < 3; ++a) { mn[a] = gmin(q[a], mn[a]); mx[a] = gmax(q[a], mx[a]); }
      }
      for (int a = 0; a < 3; ++a) {
        const double pad = tight ? 0x1p-30 * (std::fabs(mn[a]) + std::fabs(mx[a]) + 1.0) : 0.0;
        out->mn[a] = mn[a] - pad;
        out->mx[a] = mx[a] + pad;
      }
      return true;
    }
    case RT_NODE_CONSTANT_MEDIUM:
      return flat_box(nodes, n.a, out);
    default:
      return false;
  }
}

// Per-node traversal-stack needs (entries) over a flat node array whose children precede their
// parents: the recurrence rt_upload_scene's validator applies (bvh_stack_need for BVH nodes, one
// entry per open instance frame, 0 for primitives and Translate/Rotate chains over one). False
// when a child does not precede its parent.
bool stack_needs(const std::vector<rt_node>& nodes, std::vector<int>& need) {
  const int n = (int)nodes.size();
  need.assign(n, 0);
  std::vector<char> chain(n, 0);
  for (int i = 0; i < n; ++i) {
    const rt_node& x = nodes[i];
    switch (x.type) {
      case RT_NODE_BVH:
        if (x.a < 0 || x.a >= i || x.b < 0 || x.b >= i) return false;
        need[i] = bvh_stack_need(x, need[x.a], need[x.b]);
        break;
      case RT_NODE_TRANSLATE:
      case RT_NODE_ROTATE:
        if (x.a < 0 || x.a >= i) return false;
        if (chain[x.a]) chain[i] = 1;
        else need[i] = 1 + need[x.a];
        break;
      case RT_NODE_SPHERE:
      case RT_NODE_MOVING_SPHERE:
      case RT_NODE_RECT_XY:
      case RT_NODE_RECT_XZ:
      case RT_NODE_RECT_YZ:
      case RT_NODE_CUBOID:
        chain[i] = 1;
        break;
      default:
        break;
    }
  }
  return true;
}

// Rebuild the world tree rooted at `root` over its leaves; appends nodes, returns the new root
// (or `root` unchanged when the tree is not eligible). Eligible: no ConstantMedium anywhere
// under the root, every leaf boundable, finite boxes.
namespace {

bool has_media(const std::vector<rt_node>& nodes, int k) {
  const rt_node& m = nodes[k];
  if (m.type == RT_NODE_CONSTANT_MEDIUM) return true;
  if (m.type == RT_NODE_BVH) return has_media(nodes, m.a) || has_media(nodes, m.b);
  if (m.type == RT_NODE_TRANSLATE || m.type == RT_NODE_ROTATE) return has_media(nodes, m.a);
  return false;
}

// Binned-SAH tree over the given leaves (appended to `nodes`, every node RT_BVH_ORDERED); -1 when a
// leaf is not boundable or the tree would need a deeper stack than the LDS walk has (a degenerate
// split sequence, e.g. exponentially spaced centroids, can give such a spine).
int sah_over_leaves(std::vector<rt_node>& nodes, const std::vector<int>& leaves) {
  Builder b{nodes};
  // RTAMD_SAH_BINS: centroid bins per axis (0 = a full sweep over the sorted centroids)
  if (const char* e = std::getenv("RTAMD_SAH_BINS")) b.bins = std::max(0, std::min(4096, std::atoi(e)));
  const int n = (int)leaves.size();
  b.boxes.resize(n);
  b.leaf_ids = leaves;
  for (int a = 0; a < 3; ++a) b.cx[a].resize(n);
  for (int i = 0; i < n; ++i) {
    if (!flat_box(nodes, leaves[i], &b.boxes[i])) return -1;
    for (int a = 0; a < 3; ++a) {
      if (!std::isfinite(b.boxes[i].mn[a]) || !std::isfinite(b.boxes[i].mx[a])) return -1;
      b.cx[a][i] = 0.5 * (b.boxes[i].mn[a] + b.boxes[i].mx[a]);
    }
  }
  std::vector<int> items(n);
  for (int i = 0; i < n; ++i) items[i] = i;
  Box rb;
  const size_t n_before = nodes.size();
  const int new_root = b.build(items, 0, n, rb);
  std::vector<int> need;
  if (!stack_needs(nodes, need) || need[new_root] > kMaxStackNeed) {
    nodes.resize(n_before);
    return -1;
  }
  return new_root;
}

// The leaves under a BVH subtree: its maximal non-BVH nodes, each once (BVHNode h h, src/Lib.hs:948:
// a repeated leaf cannot change the closest hit).
void collect_leaves(const std::vector<rt_node>& nodes, int id, std::vector<int>& out, std::vector<char>& seen) {
  const rt_node& n = nodes[id];
  if (n.type == RT_NODE_BVH) {
    collect_leaves(nodes, n.a, out, seen);
    collect_leaves(nodes, n.b, out, seen);
  } else if (!seen[id]) {
    seen[id] = 1;
    out.push_back(id);
  }
}

}  // namespace

// Rebuild the world tree rooted at `root` over its leaves; appends nodes, returns the new root
// (or `root` unchanged when the tree is not eligible). Eligible: no ConstantMedium anywhere
// under the root, no Unhittable leaf, every leaf boundable, finite boxes.
int rebuild_world_bvh(std::vector<rt_node>& nodes, int root) {
  if (nodes[root].type != RT_NODE_BVH || has_media(nodes, root)) return root;
  std::vector<int> leaves;
  std::vector<char> seen(nodes.size(), 0);
  collect_leaves(nodes, root, leaves, seen);
  for (int id : leaves)
    if (nodes[id].type == RT_NODE_UNHITTABLE || nodes[id].type == RT_NODE_EXT) return root;
  // Small trees (e.g. the 8-object Cornell box) keep the reference tree: nothing to gain, and its
  // visiting order was measured faster there.
  if (leaves.size() < 16) return root;
  const int r = sah_over_leaves(nodes, leaves);
  return r < 0 ? root : r;
}

namespace {

bool kMediaSkeleton = false;  // (RTAMD_MEDIA_SKELETON=1, read by rebuild_media_skeleton)
bool kMediaFirst = true;      // (RTAMD_MEDIA_FIRST=0 leaves the world's media in its SAH tree)

// rebuild_media_skeleton's recursion: the id that replaces node `id` (itself when unchanged).
int skeleton(std::vector<rt_node>& nodes, int id, int depth) {
  if (depth > 512) return id;
  const rt_node n = nodes[id];  // (a copy: `nodes` grows)
  if (n.type == RT_NODE_BVH) {
    // (round 5: media are leaves too, keyed per occurrence by unfold_media: no skeleton is kept above
    // them; RTAMD_MEDIA_SKELETON=1 keeps it, for A/B runs — same images, since the draws are keyed)
    if (!kMediaSkeleton || !has_media(nodes, id)) {
      // a subtree: its leaves, instance frames first rebuilt inside, re-bounded by SAH
      std::vector<int> leaves;
      std::vector<char> seen(nodes.size(), 0);
      collect_leaves(nodes, id, leaves, seen);
      // The world's own media (outside instance frames) are hoisted out of the SAH tree: a chain of
      // RT_BVH_MEDIA_FIRST nodes above it, one per medium, entered left (the medium) first. A medium's
      // tier-B candidate does not depend on the walk's bound or order (keyed draw, unbounded candidate), so
      // testing it first changes no result, and its candidate (the fog of next_week_final is hit by
      // nearly every ray) bounds the walk of the rest from the start; the rest's tree is no longer
      // inflated by a medium's box (the fog's boundary is a radius-5000 sphere around the whole scene).
      std::vector<int> media;
      if (depth == 0 && kMediaFirst) {
        std::vector<int> rest;
        for (int leaf : leaves) (nodes[leaf].type == RT_NODE_CONSTANT_MEDIUM ? media : rest).push_back(leaf);
        if (!rest.empty() && !media.empty()) leaves.swap(rest);
        else media.clear();
      }
      bool changed = false;
      for (int& leaf : leaves) {
        if (nodes[leaf].type == RT_NODE_UNHITTABLE || nodes[leaf].type == RT_NODE_EXT) return id;
        const int nl = skeleton(nodes, leaf, depth + 1);
        changed |= nl != leaf;
        leaf = nl;
      }
      // (small worlds keep the caller's tree, media where they are)
      if (leaves.size() + media.size() < 16 && !changed) return id;
      int r = leaves.size() == 1 ? leaves[0] : sah_over_leaves(nodes, leaves);
      if (r < 0) return id;
      for (size_t k = media.size(); k-- > 0;) {
        Box mb, rb;
        if (!flat_box(nodes, media[k], &mb) || !flat_box(nodes, r, &rb)) return id;
        rt_node h{};
        for (int i = 0; i < 3; ++i) {
          h.f[i] = std::min(mb.mn[i], rb.mn[i]);
          h.f[3 + i] = std::max(mb.mx[i], rb.mx[i]);
        }
        h.type = RT_NODE_BVH;
        h.a = media[k];
        h.b = r;
        h.c = RT_BVH_ORDERED | RT_BVH_MEDIA_FIRST;
        nodes.push_back(h);
        r = (int)nodes.size() - 1;
      }
      return r;
    }
    const int a = skeleton(nodes, n.a, depth + 1), b = skeleton(nodes, n.b, depth + 1);
    if (a == n.a && b == n.b) return id;
    rt_node m = n;  // the skeleton node itself keeps its place, box and left-first order
    m.a = a;
    m.b = b;
    nodes.push_back(m);
    return (int)nodes.size() - 1;
  }
  if (n.type == RT_NODE_TRANSLATE || n.type == RT_NODE_ROTATE) {  // a frame: rebuild inside
    const int a = skeleton(nodes, n.a, depth + 1);
    if (a == n.a) return id;
    rt_node m = n;
    m.a = a;
    nodes.push_back(m);
    return (int)nodes.size() - 1;
  }
  return id;  // primitives, chains, media (their boundary is a primitive chain)
}

}  // namespace

// Worlds the walk must take in the reference's own order (ConstantMedium draws, instance frames):
// the skeleton of BVH nodes above media stays as it is (left first, the caller's boxes), while every
// media-free subtree below it — and every tree inside an instance frame — is re-bounded by SAH over
// the same leaves. A media-free subtree's closest hit (and so the bound the walk carries on with)
// does not depend on its shape except for exact ties, which the walk detects (rt_trace.h). Returns
// the new root (== root when nothing changed).
int rebuild_media_skeleton(std::vector<rt_node>& nodes, int root) {
  const char* ms = std::getenv("RTAMD_MEDIA_SKELETON");
  kMediaSkeleton = ms && ms[0] == '1';
  const char* mf = std::getenv("RTAMD_MEDIA_FIRST");
  kMediaFirst = !(mf && mf[0] == '0');
  const size_t n0 = nodes.size();
  const int r = skeleton(nodes, root, 0);
  std::vector<int> need;
  if (r != root && (!stack_needs(nodes, need) || need[r] > kMaxStackNeed)) {
    nodes.resize(n0);
    return root;
  }
  return r;
}

namespace {

// Nearest float below / above a double (the fp32 box contains the fp64 one).
float f32_down(double x) {
  float f = (float)x;
  if ((double)f > x) f = std::nextafter(f, -INFINITY);
  return f;
}
float f32_up(double x) {
  float f = (float)x;
  if ((double)f < x) f = std::nextafter(f, INFINITY);
  return f;
}

struct WideBuilder {
  const std::vector<rt_node>& nodes;
  std::vector<rt_wnode>& out;
  bool ok = true;

  bool box_of(int id, Box& b) const { return flat_box(nodes, id, &b); }
  static double area(const Box& b) {
    const double dx = b.mx[0] - b.mn[0], dy = b.mx[1] - b.mn[1], dz = b.mx[2] - b.mn[2];
    return 2.0 * (dx * dy + dy * dz + dz * dx);
  }

  // SAH-optimal collapse (Ylitie, Karras & Laine 2017, "Efficient incoherent ray traversal on GPUs
  // through compressed wide BVHs", sec. 3): cost[i][j] = the least SAH cost of the binary subtree at
  // i spread over at most j child slots of its parent; one slot holds a leaf (a primitive test,
  // c_prim * area) or a wide node (c_node * area + the best spread of i's children over 4 slots).
  // pick[i][j] = how many of those slots the left child takes (0: j - 1 slots were as good).
  bool sah = false;
  int K = RT_WIDE;  // child slots per wide node: 4, or 8 (a pair of 4-wide records, build_wide8_bvh)
  double c_node = 1.0, c_prim = 1.0;
  std::vector<std::array<double, 2 * RT_WIDE + 1>> cost;
  std::vector<std::array<int, 2 * RT_WIDE + 1>> pick;
  std::vector<char> done;

  double spread(int i, int j) {  // best split of internal node i's two children over j >= 2 slots
    const rt_node& n = nodes[i];
    double best = INFINITY;
    for (int k = 1; k < j; ++k) {
      const double c = solve(n.a, k) + solve(n.b, j - k);
      if (c < best) { best = c; pick[i][j] = k; }
    }
    return best;
  }
  double solve(int i, int j) {
    if (!done[i]) {
      done[i] = 1;
      Box b;
      if (!box_of(i, b)) { ok = false; return 0; }
      const double a = area(b);
      if (nodes[i].type != RT_NODE_BVH) {
        for (int k = 1; k <= K; ++k) cost[i][k] = c_prim * a;
      } else {
        cost[i][1] = c_node * a + spread(i, K);
        pick[i][1] = pick[i][K];  // (the wide node's own slots, see kids_sah)
        for (int k = 2; k <= K; ++k) {
          const double c = spread(i, k);
          if (cost[i][k - 1] <= c) { cost[i][k] = cost[i][k - 1]; pick[i][k] = 0; }
          else cost[i][k] = c;
        }
      }
    }
    return cost[i][j];
  }
  // the slots node i's subtree occupies when given j of them
  void slots(int i, int j, std::vector<int>& out) {
    if (j == 1 || nodes[i].type != RT_NODE_BVH) { out.push_back(i); return; }
    const int k = pick[i][j];
    if (k == 0) { slots(i, j - 1, out); return; }
    slots(nodes[i].a, k, out);
    slots(nodes[i].b, j - k, out);
  }
  std::vector<int> kids_sah(int id) {
    solve(id, 1);
    std::vector<int> kids;
    const int k = pick[id][1];  // the split that cost[id][1] (a wide node at id) was priced with
    slots(nodes[id].a, k, kids);
    slots(nodes[id].b, K - k, kids);
    return kids;
  }

  // Collapse the binary node `id` into one wide node: SAH-optimal child slots (sah), or open the
  // largest-area interior child until four children are reached or none is interior. Returns the
  // wide id; *need = stack entries.
  int build(int id, int depth, int* need) {
    if (depth > 256) { ok = false; return 0; }
    std::vector<int> kids{nodes[id].a, nodes[id].b};
    if (sah) {
      kids = kids_sah(id);
      if (!ok) return 0;
    }
    for (;;) {
      if (sah || (int)kids.size() >= K) break;
      int best = -1;
      double best_area = -1;
      for (int k = 0; k < (int)kids.size(); ++k) {
        const rt_node& n = nodes[kids[k]];
        if (n.type != RT_NODE_BVH) continue;
        Box b;
        if (!box_of(kids[k], b)) { ok = false; return 0; }
        const double a = area(b);
        if (a > best_area) { best_area = a; best = k; }
      }
      if (best < 0) break;
      const rt_node& n = nodes[kids[best]];
      kids[best] = n.a;
      kids.insert(kids.begin() + best + 1, n.b);
    }
    // K = 8: the node is the record pair (2 me, 2 me + 1), its children ordered by box centre along the
    // axis of the node's largest extent, the lower four in the first record; pad[0] of the first record
    // holds that axis, so that a walk can take the half farther along the ray first (rt_trace.h wide_node8)
    int order_axis = -1;
    if (K == 2 * RT_WIDE) {
      Box nb;
      if (!box_of(id, nb)) { ok = false; return 0; }
      order_axis = 0;
      for (int a = 1; a < 3; ++a)
        if (nb.mx[a] - nb.mn[a] > nb.mx[order_axis] - nb.mn[order_axis]) order_axis = a;
      std::vector<std::pair<double, int>> keyed;
      for (int kid : kids) {
        Box b;
        if (!box_of(kid, b)) { ok = false; return 0; }
        keyed.push_back({b.mn[order_axis] + b.mx[order_axis], kid});
      }
      std::stable_sort(keyed.begin(), keyed.end(), [](const std::pair<double, int>& x, const std::pair<double, int>& y) {
        return x.first < y.first;
      });
      // the lower half first: ceil(n / 2) children in the first record, the rest in the second
      const int n = (int)keyed.size(), lo_n = (n + 1) / 2;
      std::vector<int> sorted(2 * RT_WIDE, -1);
      for (int k = 0; k < n; ++k) sorted[k < lo_n ? k : RT_WIDE + (k - lo_n)] = keyed[k].second;
      kids = sorted;  // (-1: an unused slot)
    }
    const int recs = K / RT_WIDE;
    const int me = (int)out.size() / recs;
    for (int r = 0; r < recs; ++r) out.push_back(rt_wnode{});
    int child_need = 0, used = 0;
    for (int r = 0; r < recs; ++r) {
    rt_wnode w{};
    if (recs == 2) w.pad[0] = r == 0 ? order_axis : -1;
    // (a pair's half: its first real child, for an unused slot's harmless leaf)
    int first = -1;
    for (int k = 0; k < RT_WIDE; ++k)
      if (first < 0 && r * RT_WIDE + k < (int)kids.size() && kids[r * RT_WIDE + k] >= 0) first = kids[r * RT_WIDE + k];
    if (first < 0)
      for (int kid : kids)
        if (kid >= 0) { first = kid; break; }
    for (int kk = 0; kk < RT_WIDE; ++kk) {
      const int k = r * RT_WIDE + kk;
      if (k >= (int)kids.size() || kids[k] < 0) {
        // unused slot: an empty box (never accepted by a finite test) over a harmless leaf — the
        // first leaf below this node, re-testing which cannot change the closest hit — so that
        // rays accepting every child (fp32 slack = inf) need no slot check
        for (int a = 0; a < 3; ++a) { w.lo[a][kk] = INFINITY; w.hi[a][kk] = -INFINITY; }
        int leaf = first;
        while (nodes[leaf].type == RT_NODE_BVH) leaf = nodes[leaf].a;
        w.child[kk] = ~leaf;
        continue;
      }
      ++used;
      Box b;
      if (!box_of(kids[k], b)) { ok = false; return 0; }
      for (int a = 0; a < 3; ++a) { w.lo[a][kk] = f32_down(b.mn[a]); w.hi[a][kk] = f32_up(b.mx[a]); }
      if (nodes[kids[k]].type == RT_NODE_BVH) {
        int cn = 0;
        w.child[kk] = build(kids[k], depth + 1, &cn);
        if (!ok) return 0;
        child_need = std::max(child_need, cn);
      } else {
        w.child[kk] = ~kids[k];
      }
    }
    out[recs * me + r] = w;
    }
    // the nearest hit child is entered, the others (<= K - 1) wait on the stack meanwhile
    *need = used - 1 + child_need;
    return me;
  }
};

}  // namespace

// 4-wide collapse of the binary world tree at `root` (rebuilt or the reference's own). Returns
// false when the root is not a BVH node or a box is not finite.
bool build_wide_bvh(const std::vector<rt_node>& nodes, int root, std::vector<rt_wnode>& out, int* stack_need) {
  out.clear();
  *stack_need = 0;
  if (root < 0 || root >= (int)nodes.size() || nodes[root].type != RT_NODE_BVH) return false;
  WideBuilder b{nodes, out};
  // RTAMD_WIDE_BUILD=greedy: the largest-area opening; default: the SAH-optimal collapse
  const char* wb = std::getenv("RTAMD_WIDE_BUILD");
  b.sah = !(wb && std::string(wb) == "greedy");
  if (const char* cp = std::getenv("RTAMD_SAH_CPRIM")) b.c_prim = std::atof(cp);
  if (b.sah) {
    b.cost.assign(nodes.size(), {});
    b.pick.assign(nodes.size(), {});
    b.done.assign(nodes.size(), 0);
  }
  b.build(root, 0, stack_need);
  if (!b.ok) {
    out.clear();
    return false;
  }
  return true;
}

// The 8-wide collapse of the same tree (round 6, A/B: RTAMD_W8=1 at upload, spheres-only worlds): node p is
// the record pair (2p, 2p + 1) of `out`, child ids >= 0 are pair indices. Same SAH-optimal programme with 8
// child slots.
bool build_wide8_bvh(const std::vector<rt_node>& nodes, int root, std::vector<rt_wnode>& out, int* stack_need) {
  out.clear();
  *stack_need = 0;
  if (root < 0 || root >= (int)nodes.size() || nodes[root].type != RT_NODE_BVH) return false;
  WideBuilder b{nodes, out};
  b.sah = true;
  b.K = 2 * RT_WIDE;
  b.cost.assign(nodes.size(), {});
  b.pick.assign(nodes.size(), {});
  b.done.assign(nodes.size(), 0);
  b.build(root, 0, stack_need);
  if (!b.ok) {
    out.clear();
    return false;
  }
  return true;
}

// Tier-B medium draws are keyed by the medium's occurrence (include/rt.h): the preorder
// rank of the occurrence among the medium occurrences of the caller's tree walked from the world root
// (BVH left child before right, into Translate/Rotate children; a medium's boundary holds none). A DAG
// can reach one ConstantMedium record along several paths (BVHNode h h, src/Lib.hs:948; shared
// sub-trees), and each occurrence draws with its own key. So every record on a path to a medium is
// copied once per path (appended, children before parents) and each medium copy carries key + 1 in
// f[1]; media-free sub-trees stay shared. A medium already keyed (f[1] >= 1: an unfolded array uploaded
// again) keeps its key — only when every occurrence is keyed, each by a distinct integer key below 2^31
// (a keyed record reached along two paths, or a caller's key equal to an unkeyed occurrence's
// rank, would make two occurrences draw the same numbers). Returns the unfolded root (`root` itself when
// no medium lies below it); -1 when the unfolded tree would be too large (more than 2^22 records) or is
// not a DAG with children first; -2 when the keys break that rule.
int unfold_media(std::vector<rt_node>& nodes, int root) {
  const int n0 = (int)nodes.size();
  if (root < 0 || root >= n0) return -1;
  std::vector<signed char> memo(n0, -1);
  bool ok = true;
  std::function<bool(int, int)> has = [&](int id, int depth) -> bool {
    if (id < 0 || id >= n0 || depth > 4096) {
      ok = false;
      return false;
    }
    if (memo[id] >= 0) return memo[id] != 0;
    const rt_node& x = nodes[id];
    bool m = false;
    if (x.type == RT_NODE_CONSTANT_MEDIUM) m = true;
    else if (x.type == RT_NODE_BVH) m = (x.a < id && x.b < id) ? (has(x.a, depth + 1) | has(x.b, depth + 1)) : (ok = false);
    else if (x.type == RT_NODE_TRANSLATE || x.type == RT_NODE_ROTATE) m = x.a < id ? has(x.a, depth + 1) : (ok = false);
    memo[id] = m ? 1 : 0;
    return m;
  };
  if (!has(root, 0)) return ok ? root : -1;
  uint32_t rank = 0, keyed = 0;
  bool keys_ok = true;
  std::vector<double> keys;  // (the caller's keys, f[1] = key + 1)
  std::function<int(int)> copy = [&](int id) -> int {
    if (!ok || !has(id, 0)) return id;
    if ((int)nodes.size() >= (1 << 22)) {
      ok = false;
      return id;
    }
    rt_node x = nodes[id];  // (a copy: `nodes` grows)
    if (x.type == RT_NODE_CONSTANT_MEDIUM) {
      if (x.f[1] >= 1.0) {
        ++keyed;
        keys_ok &= x.f[1] <= 0x1p31 && x.f[1] == std::floor(x.f[1]);
        keys.push_back(x.f[1]);
      } else {
        x.f[1] = (double)rank + 1.0;
      }
      ++rank;
    } else if (x.type == RT_NODE_BVH) {
      const int a = copy(x.a);
      const int b = copy(x.b);
      x.a = a;
      x.b = b;
    } else {  // Translate / Rotate
      x.a = copy(x.a);
    }
    nodes.push_back(x);
    return (int)nodes.size() - 1;
  };
  const int r = copy(root);
  if (ok && keyed) {  // keyed occurrences: all of them, with distinct keys
    std::sort(keys.begin(), keys.end());
    keys_ok &= keyed == rank && std::adjacent_find(keys.begin(), keys.end()) == keys.end();
  }
  if (!ok || !keys_ok) {
    nodes.resize(n0);
    return ok ? -2 : -1;
  }
  return r;
}

// The world tree the device walks, as rt_upload_scene builds it (after unfold_media): worlds with
// instance frames (Translate/Rotate over a BVH) or media are re-bounded by SAH over their leaves —
// media are leaves like any other, their tier-B draws being keyed by occurrence and their candidate hit
// computed without the walk's bound (order-independent) — with every tree inside a frame
// re-bounded in the frame's coordinates (rebuild_media_skeleton; RTAMD_SKELETON=0: the caller's tree
// as is); the others are rebuilt whole (rebuild_world_bvh).
int rebuild_for_device(std::vector<rt_node>& nodes, int root) {
  bool media = false, frames = false;
  std::vector<char> seen(nodes.size(), 0);
  std::function<void(int)> scan = [&](int id) {
    if (seen[id]) return;
    seen[id] = 1;
    const rt_node& n = nodes[id];
    if (n.type == RT_NODE_CONSTANT_MEDIUM) media = true;
    if (n.type == RT_NODE_BVH) {
      scan(n.a);
      scan(n.b);
    } else if (n.type == RT_NODE_TRANSLATE || n.type == RT_NODE_ROTATE) {
      int k = n.a;
      while (nodes[k].type == RT_NODE_TRANSLATE || nodes[k].type == RT_NODE_ROTATE) k = nodes[k].a;
      frames |= nodes[k].type == RT_NODE_BVH || nodes[k].type == RT_NODE_CONSTANT_MEDIUM;
      scan(n.a);
    }
  };
  scan(root);
  if (!media && !frames) return rebuild_world_bvh(nodes, root);
  const char* e = std::getenv("RTAMD_SKELETON");
  if (e && e[0] == '0') return root;
  return rebuild_media_skeleton(nodes, root);
}

// rt_qnode (rt_wide.h) from rt_wnode: per node and axis a power-of-two grid step s and an origin on the
// grid (k s, |k| < 2^23) below every child's lower plane, with the node's planes within 255 steps; each
// child's fp32 box is rounded outward to the grid. False when a node's planes do not fit an fp32 grid.
bool quantize_wide(const std::vector<rt_wnode>& in, std::vector<rt_qnode>& out) {
  out.assign(in.size(), rt_qnode{});
  for (size_t i = 0; i < in.size(); ++i) {
    const rt_wnode& w = in[i];
    rt_qnode& q = out[i];
    for (int k = 0; k < RT_WIDE; ++k) q.child[k] = w.child[k];
    for (int a = 0; a < 3; ++a) {
      double L = INFINITY, H = -INFINITY;
      for (int k = 0; k < RT_WIDE; ++k)
        if (w.lo[a][k] <= w.hi[a][k]) {  // (an unused slot has lo = +inf, hi = -inf)
          L = std::min(L, (double)w.lo[a][k]);
          H = std::max(H, (double)w.hi[a][k]);
        }
      uint32_t qlo = 0, qhi = 0;
      if (!(L <= H)) {  // no child box on this axis (every slot unused)
        q.origin[a] = 0.0f;
        q.scale[a] = 1.0f;
        for (int k = 0; k < RT_WIDE; ++k) qlo |= 255u << (8 * k);
        q.qlo[a] = qlo;
        q.qhi[a] = 0;
        continue;
      }
      if (!std::isfinite(L) || !std::isfinite(H)) return false;
      int e = -126;
      {
        const double span = (H - L) / 254.0, mag = std::max(std::fabs(L), std::fabs(H)) / 8388352.0;
        const double need = std::max(span, mag);
        if (need > 0) e = std::max(e, (int)std::ceil(std::log2(need)));
      }
      double s = 0, org = 0;
      for (;; ++e) {
        if (e > 127) return false;
        s = std::ldexp(1.0, e);
        const double kk = std::floor(L / s);
        org = kk * s;
        // (every plane the node can decode, org + q s for q <= 255, stays a finite fp32 value)
        if (std::fabs(kk) + 256.0 < 8388608.0 && std::ceil((H - org) / s) <= 255.0 &&
            org + 255.0 * s <= 3.4028234663852886e38)
          break;
      }
      q.origin[a] = (float)org;  // (exact: |kk| < 2^23, s a normal power of two)
      q.scale[a] = (float)s;
      for (int k = 0; k < RT_WIDE; ++k) {
        uint32_t lo = 255, hi = 0;
        if (w.lo[a][k] <= w.hi[a][k]) {
          lo = (uint32_t)std::floor(((double)w.lo[a][k] - org) / s);
          hi = (uint32_t)std::ceil(((double)w.hi[a][k] - org) / s);
        } else {
          // an unused slot: empty on every axis
          lo = 255;
          hi = 0;
        }
        qlo |= lo << (8 * k);
        qhi |= hi << (8 * k);
      }
      q.qlo[a] = qlo;
      q.qhi[a] = qhi;
    }
    // an unused slot stays empty on every axis even where this axis saw no box at all
    for (int k = 0; k < RT_WIDE; ++k) {
      bool used = true;
      for (int a = 0; a < 3; ++a) used &= w.lo[a][k] <= w.hi[a][k];
      if (!used)
        for (int a = 0; a < 3; ++a) {
          q.qlo[a] = (q.qlo[a] & ~(255u << (8 * k))) | (255u << (8 * k));
          q.qhi[a] &= ~(255u << (8 * k));
        }
    }
  }
  return true;
}

}  // namespace rt

extern "C" int rt_quantize_wide(const void* wnodes, int n, void* out) {
  if (!wnodes || !out || n < 0) {
    rt::set_error("rt_quantize_wide: bad argument");
    return RT_E_INVALID;
  }
  const rt_wnode* w = static_cast<const rt_wnode*>(wnodes);
  std::vector<rt_qnode> q;
  if (!rt::quantize_wide(std::vector<rt_wnode>(w, w + n), q)) {
    rt::set_error("rt_quantize_wide: a node's boxes do not fit an fp32 grid");
    return RT_E_UNSUPPORTED;
  }
  std::copy(q.begin(), q.end(), static_cast<rt_qnode*>(out));
  return RT_OK;
}

extern "C" int rt_rebuild_bvh(const rt_scene_desc* in, rt_node* out_nodes, int capacity, int* out_n, int* out_root) {
  if (!in || !out_n || !out_root || !in->nodes || in->n_nodes <= 0 || in->world_root < 0 ||
      in->world_root >= in->n_nodes) {
    rt::set_error("rt_rebuild_bvh: bad argument");
    return RT_E_INVALID;
  }
  std::vector<rt_node> nodes(in->nodes, in->nodes + in->n_nodes);
  const int unfolded = rt::unfold_media(nodes, in->world_root);
  if (unfolded < 0) {
    rt::set_error(unfolded == -2 ? "rt_rebuild_bvh: medium keys (f[1]) set on some occurrences only, or repeated"
                                 : "rt_rebuild_bvh: the world tree is not a DAG with children first, or unfolds too large");
    return RT_E_INVALID;
  }
  const int root = rt::rebuild_for_device(nodes, unfolded);
  *out_n = (int)nodes.size();
  *out_root = root;
  if (out_nodes) {
    if (capacity < (int)nodes.size()) {
      rt::set_error("rt_rebuild_bvh: capacity too small");
      return RT_E_INVALID;
    }
    std::copy(nodes.begin(), nodes.end(), out_nodes);
  }
  return RT_OK;
}

extern "C" int rt_tree_stack_need(const rt_node* nodes, int n_nodes, int root, int* out_need) {
  if (!nodes || n_nodes <= 0 || root < 0 || root >= n_nodes || !out_need) {
    rt::set_error("rt_tree_stack_need: bad argument");
    return RT_E_INVALID;
  }
  std::vector<int> need;
  if (!rt::stack_needs(std::vector<rt_node>(nodes, nodes + n_nodes), need)) {
    rt::set_error("rt_tree_stack_need: a child must precede its parent");
    return RT_E_INVALID;
  }
  *out_need = need[root];
  return RT_OK;
}

extern "C" int rt_wide_bvh(const rt_node* nodes, int n_nodes, int root, void* out, int capacity, int* out_n,
                           int* out_stack_need) {
  if (!nodes || n_nodes <= 0 || root < 0 || root >= n_nodes || !out_n || !out_stack_need) {
    rt::set_error("rt_wide_bvh: bad argument");
    return RT_E_INVALID;
  }
  std::vector<rt_node> v(nodes, nodes + n_nodes);
  std::vector<rt_wnode> w;
  int need = 0;
  if (!rt::build_wide_bvh(v, root, w, &need)) {
    rt::set_error("rt_wide_bvh: the root is not a BVH node (or a box is not boundable)");
    return RT_E_UNSUPPORTED;
  }
  *out_n = (int)w.size();
  *out_stack_need = need;
  if (out) {
    if (capacity < (int)w.size()) {
      rt::set_error("rt_wide_bvh: capacity too small");
      return RT_E_INVALID;
    }
    std::copy(w.begin(), w.end(), static_cast<rt_wnode*>(out));
  }
  return RT_OK;
}
