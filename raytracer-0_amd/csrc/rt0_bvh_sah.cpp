// rt0_bvh_sah.cpp -- binned-SAH BVH of the triangle models (host build).
//
// The reference has no acceleration structure (intersection() loops over every
// mesh, raytracer.glsl:1006-1036; its iTriangle, 864-892, is commented out).
// rt0_bvh.hip builds a Morton-code LBVH on the device in well under a
// millisecond, but a Morton split is a spatial-median split: it ignores where
// the triangles' surface area lies, so its boxes overlap and rays visit more
// nodes than they need.  This builder gives the same node format the quality
// of a surface-area-heuristic tree (HLBVH's top levels, all the way down):
//   * top-down, one triangle per leaf (the walk in rt0_integrator.h is
//     unchanged: n-1 inner nodes, leaf links ~i);
//   * per node the split plane minimising A(L)*N(L) + A(R)*N(R), from 32
//     centroid bins per axis, or, below 64 triangles, from an exact sweep
//     over the centroids sorted on each axis;
//   * depth-first (pre-order) node layout: a left child is stored right after
//     its parent, so the near-first walk mostly reads the next 64 B, and the
//     triangles are stored in leaf order (the walk's TriDev reads follow the
//     same order);
//   * subtrees of >= 16k triangles are built on their own threads: every
//     subtree's node and leaf ranges are known from its triangle count
//     (a subtree of m triangles holds m-1 inner nodes), so the threads write
//     disjoint parts of the output and the result does not depend on timing.
// The scene changes rarely (index.html:1167-1196 recompiles on change), so the
// build runs on the host at the first render after a change (~30 ms for the
// 81,920-triangle C5 model) and is uploaded with the scene.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <thread>
#include <vector>

#include "rt0_device.h"
#include "rt0_internal.h"

namespace {

struct Aabb {
  float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  void grow(const Aabb &b) {
    for (int a = 0; a < 3; a++) {
      lo[a] = std::min(lo[a], b.lo[a]);
      hi[a] = std::max(hi[a], b.hi[a]);
    }
  }
  void grow(const float p[3]) {
    for (int a = 0; a < 3; a++) {
      lo[a] = std::min(lo[a], p[a]);
      hi[a] = std::max(hi[a], p[a]);
    }
  }
  float half_area() const {
    const float x = hi[0] - lo[0], y = hi[1] - lo[1], z = hi[2] - lo[2];
    return (x < 0.f || y < 0.f || z < 0.f) ? 0.f : x * y + y * z + z * x;
  }
};

struct Builder {
  const std::vector<Aabb> &box;    // per triangle
  const std::vector<float> &cen;   // per triangle centroid (3 floats)
  std::vector<uint32_t> &idx;      // triangle order; leaves in this order at the end
  std::vector<BvhNode> &nodes;

  static constexpr int kBins = 32, kSweep = 64, kThreadMin = 16384;

  // Split [b, e) (e - b >= 2) into [b, m) and [m, e); both non-empty.
  int split(int b, int e) {
    const int n = e - b;
    Aabb cb;
    for (int i = b; i < e; i++) cb.grow(&cen[3 * (size_t)idx[i]]);
    float best = INFINITY;
    int best_axis = -1;
    int best_k = 0;  // sweep: left count; binned: first bin of the right side
    if (n <= kSweep) {
      std::vector<uint32_t> tmp(idx.begin() + b, idx.begin() + e);
      std::vector<float> rarea(n);
      for (int a = 0; a < 3; a++) {
        if (!(cb.hi[a] > cb.lo[a])) continue;
        std::sort(tmp.begin(), tmp.end(), [&](uint32_t x, uint32_t y) {
          const float cx = cen[3 * (size_t)x + a], cy = cen[3 * (size_t)y + a];
          return cx < cy || (cx == cy && x < y);
        });
        Aabb r;
        for (int i = n - 1; i > 0; i--) {
          r.grow(box[tmp[i]]);
          rarea[i] = r.half_area();
        }
        Aabb l;
        for (int i = 0; i < n - 1; i++) {
          l.grow(box[tmp[i]]);
          const float c = l.half_area() * (float)(i + 1) + rarea[i + 1] * (float)(n - 1 - i);
          if (c < best) {
            best = c;
            best_axis = a;
            best_k = i + 1;
          }
        }
      }
      if (best_axis < 0) return b + n / 2;  // every centroid equal: halve the range
      std::sort(idx.begin() + b, idx.begin() + e, [&](uint32_t x, uint32_t y) {
        const float cx = cen[3 * (size_t)x + best_axis], cy = cen[3 * (size_t)y + best_axis];
        return cx < cy || (cx == cy && x < y);
      });
      return b + best_k;
    }
    for (int a = 0; a < 3; a++) {
      const float ext = cb.hi[a] - cb.lo[a];
      if (!(ext > 0.f)) continue;
      const float scale = (float)kBins / ext;
      Aabb bb[kBins];
      int cnt[kBins] = {};
      for (int i = b; i < e; i++) {
        const uint32_t t = idx[i];
        const int k = std::min(kBins - 1, (int)((cen[3 * (size_t)t + a] - cb.lo[a]) * scale));
        cnt[k]++;
        bb[k].grow(box[t]);
      }
      float rarea[kBins];
      int rcnt[kBins];
      Aabb r;
      int rc = 0;
      for (int k = kBins - 1; k > 0; k--) {
        r.grow(bb[k]);
        rc += cnt[k];
        rarea[k] = r.half_area();
        rcnt[k] = rc;
      }
      Aabb l;
      int lc = 0;
      for (int k = 0; k < kBins - 1; k++) {
        l.grow(bb[k]);
        lc += cnt[k];
        if (lc == 0 || rcnt[k + 1] == 0) continue;
        const float c = l.half_area() * (float)lc + rarea[k + 1] * (float)rcnt[k + 1];
        if (c < best) {
          best = c;
          best_axis = a;
          best_k = k + 1;
        }
      }
    }
    if (best_axis < 0) return b + n / 2;
    // the same bin assignment as above decides the side (no float re-derivation)
    const float ext = cb.hi[best_axis] - cb.lo[best_axis], scale = (float)kBins / ext;
    auto left = [&](uint32_t t) {
      return std::min(kBins - 1, (int)((cen[3 * (size_t)t + best_axis] - cb.lo[best_axis]) * scale)) < best_k;
    };
    const int m = (int)(std::stable_partition(idx.begin() + b, idx.begin() + e, left) - idx.begin());
    return (m == b || m == e) ? b + n / 2 : m;
  }

  // Build the subtree of triangles [b, e) whose root is inner node `node`
  // (e - b >= 2); its inner nodes are [node, node + e - b - 1) in pre-order.
  // Returns the boxes of the root's two children; *depth = edges to the
  // deepest leaf.
  void build(int node, int b, int e, Aabb &out, int &depth) {
    const int m = split(b, e);
    Aabb cb[2];
    int d[2] = {0, 0};
    int link[2];
    const int lo[2] = {b, m}, hi[2] = {m, e};
    const int child_node[2] = {node + 1, node + (m - b)};  // left subtree holds m-b-1 inner nodes
    std::thread th;
    for (int s = 0; s < 2; s++) {
      if (hi[s] - lo[s] == 1) {
        cb[s] = box[idx[lo[s]]];
        link[s] = ~lo[s];
        continue;
      }
      link[s] = child_node[s];
      if (s == 0 && e - b >= 2 * kThreadMin && m - b >= kThreadMin && e - m >= kThreadMin) {
        th = std::thread([&, s] { build(child_node[s], lo[s], hi[s], cb[s], d[s]); });
      } else {
        build(child_node[s], lo[s], hi[s], cb[s], d[s]);
      }
    }
    if (th.joinable()) th.join();
    BvhNode &nd = nodes[node];
    nd.lx0 = cb[0].lo[0];
    nd.ly0 = cb[0].lo[1];
    nd.lz0 = cb[0].lo[2];
    nd.lx1 = cb[0].hi[0];
    nd.ly1 = cb[0].hi[1];
    nd.lz1 = cb[0].hi[2];
    nd.rx0 = cb[1].lo[0];
    nd.ry0 = cb[1].lo[1];
    nd.rz0 = cb[1].lo[2];
    nd.rx1 = cb[1].hi[0];
    nd.ry1 = cb[1].hi[1];
    nd.rz1 = cb[1].hi[2];
    nd.left = link[0];
    nd.right = link[1];
    nd.pad0 = nd.pad1 = 0;
    out = cb[0];
    out.grow(cb[1]);
    depth = 1 + std::max(d[0], d[1]);
  }
};

}  // namespace

namespace rt0h {

int bvh_build_sah(int n, const float *v, const int32_t *model, std::vector<BvhNode> &nodes, std::vector<TriDev> &tris) {
  if (n <= 0) return -1;
  std::vector<Aabb> box((size_t)n);
  std::vector<float> cen(3 * (size_t)n);
  for (int i = 0; i < n; i++) {
    const float *t = v + 9 * (size_t)i;
    for (int k = 0; k < 3; k++) box[i].grow(t + 3 * k);
    for (int a = 0; a < 3; a++) cen[3 * (size_t)i + a] = (t[a] + t[3 + a] + t[6 + a]) * (1.0f / 3.0f);
  }
  std::vector<uint32_t> idx((size_t)n);
  for (int i = 0; i < n; i++) idx[i] = (uint32_t)i;
  nodes.assign((size_t)std::max(1, n - 1), BvhNode{});
  int depth = 0;
  if (n == 1) {  // a one-triangle tree: the root holds the leaf twice (as rt0_bvh.hip)
    const Aabb &b = box[0];
    nodes[0] = BvhNode{b.lo[0], b.lo[1], b.lo[2], b.lo[0], b.hi[0], b.hi[1], b.hi[2], b.lo[1],
                       b.lo[2], b.hi[0], b.hi[1], b.hi[2], ~0, ~0, 0, 0};
  } else {
    Builder B{box, cen, idx, nodes};
    Aabb root;
    B.build(0, 0, n, root, depth);
  }
  tris.resize((size_t)n);
  for (int i = 0; i < n; i++) {
    const uint32_t src = idx[i];
    const float *t = v + 9 * (size_t)src;
    TriDev &d = tris[i];
    d.v0x = t[0];
    d.v0y = t[1];
    d.v0z = t[2];
    d.model = model[src] & ~RT0_TRI_CULL_BIT;
    d.e0x = t[3] - t[0];
    d.e0y = t[4] - t[1];
    d.e0z = t[5] - t[2];
    d.cull = (model[src] & RT0_TRI_CULL_BIT) ? 1 : 0;
    d.e1x = t[6] - t[0];
    d.e1y = t[7] - t[1];
    d.e1z = t[8] - t[2];
    d.eps = 0.001f * std::sqrt(d.e0x * d.e0x + d.e0y * d.e0y + d.e0z * d.e0z) *
            std::sqrt(d.e1x * d.e1x + d.e1y * d.e1y + d.e1z * d.e1z);
  }
  return depth;
}

// The LDS treelet (rt0_integrator.h bvh_fetch): whole top levels of the tree,
// breadth-first, as nodes [0, T); every other node keeps its pre-order place
// after them.  Only the numbering changes (links follow): the same tree, the
// same walks.
int bvh_treelet_order(std::vector<BvhNode> &nodes, int max_nodes) {
  const int n = (int)nodes.size();
  if (n == 0 || max_nodes < 1) return 0;
  std::vector<int> top{0};
  for (size_t lo = 0;;) {  // top[lo..) is the deepest level taken
    std::vector<int> next;
    for (size_t i = lo; i < top.size(); i++)
      for (int ch : {nodes[(size_t)top[i]].left, nodes[(size_t)top[i]].right})
        if (ch >= 0) next.push_back(ch);
    if (next.empty() || top.size() + next.size() > (size_t)max_nodes) break;
    lo = top.size();
    top.insert(top.end(), next.begin(), next.end());
  }
  std::vector<int> id(n, -1);
  int k = 0;
  for (int t : top) id[(size_t)t] = k++;
  for (int i = 0; i < n; i++)
    if (id[(size_t)i] < 0) id[(size_t)i] = k++;
  std::vector<BvhNode> out((size_t)n);
  for (int i = 0; i < n; i++) {
    BvhNode b = nodes[(size_t)i];
    if (b.left >= 0) b.left = id[(size_t)b.left];
    if (b.right >= 0) b.right = id[(size_t)b.right];
    out[(size_t)id[(size_t)i]] = b;
  }
  nodes.swap(out);
  return (int)top.size();
}

}  // namespace rt0h
