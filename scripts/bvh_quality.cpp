// bvh_quality.cpp -- offline BVH quality probe (CPU; no GPU needed).
//
// Builds the device LBVH's tree shape on the CPU (Morton codes + Karras split,
// the algorithm of raytracer-0_amd/csrc/rt0_bvh.hip) and the binned-SAH tree
// of rt0_bvh_sah.cpp for the same world-space triangles, then walks sets of
// C5-like rays through both with the integrator's exact traversal order
// (rt0_integrator.h bvh_closest: near child first, one-triangle leaves tested
// in place) and prints the nodes visited per ray.  The GPU's counting instance
// (bench.py events_per_sample.bvh_node) is the measurement that counts; this
// only ranks builder variants before a GPU run.
//
//   python3 scripts/bvh_quality.py        (writes the C5 model, builds, runs)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <functional>
#include <random>
#include <cstdlib>
#include <vector>

#include "../raytracer-0_amd/csrc/rt0_device.h"
#include "../raytracer-0_amd/csrc/rt0_internal.h"

struct V3 {
  float x, y, z;
};
static V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
static V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
static V3 operator*(V3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
static float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static V3 cross(V3 a, V3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
static V3 nrm(V3 a) { return a * (1.0f / std::sqrt(dot(a, a))); }

// ---- CPU replica of the device LBVH (rt0_bvh.hip)
static uint32_t spread10(uint32_t v) {
  v = (v * 0x00010001u) & 0xFF0000FFu;
  v = (v * 0x00000101u) & 0x0F00F00Fu;
  v = (v * 0x00000011u) & 0xC30C30C3u;
  v = (v * 0x00000005u) & 0x49249249u;
  return v;
}
static int delta(const std::vector<uint32_t> &c, int n, int i, int j) {
  if (j < 0 || j >= n) return -1;
  return c[i] != c[j] ? __builtin_clz(c[i] ^ c[j]) : 32 + __builtin_clz((uint32_t)(i ^ j));
}
static void lbvh(int n, const float *v, std::vector<BvhNode> &nodes, std::vector<int> &order) {
  float lo[3] = {1e30f, 1e30f, 1e30f}, hi[3] = {-1e30f, -1e30f, -1e30f};
  for (long i = 0; i < 9L * n; i++) {
    lo[i % 3] = std::min(lo[i % 3], v[i]);
    hi[i % 3] = std::max(hi[i % 3], v[i]);
  }
  std::vector<std::pair<uint32_t, int>> kc(n);
  for (int i = 0; i < n; i++) {
    const float *t = v + 9L * i;
    uint32_t q[3];
    for (int a = 0; a < 3; a++) {
      const float c = (t[a] + t[3 + a] + t[6 + a]) * (1.0f / 3.0f);
      const float inv = hi[a] > lo[a] ? 1.0f / (hi[a] - lo[a]) : 0.f;
      q[a] = (uint32_t)std::min(std::max((c - lo[a]) * inv * 1024.0f, 0.0f), 1023.0f);
    }
    kc[i] = {(spread10(q[0]) << 2) | (spread10(q[1]) << 1) | spread10(q[2]), i};
  }
  std::stable_sort(kc.begin(), kc.end(), [](auto &a, auto &b) { return a.first < b.first; });
  std::vector<uint32_t> c(n);
  order.resize(n);
  for (int i = 0; i < n; i++) c[i] = kc[i].first, order[i] = kc[i].second;
  std::vector<std::pair<int, int>> child(n - 1);
  for (int i = 0; i < n - 1; i++) {
    const int d = delta(c, n, i, i + 1) - delta(c, n, i, i - 1) >= 0 ? 1 : -1;
    const int dmin = delta(c, n, i, i - d);
    int lmax = 2;
    while (delta(c, n, i, i + lmax * d) > dmin) lmax *= 2;
    int l = 0;
    for (int t = lmax / 2; t >= 1; t /= 2)
      if (delta(c, n, i, i + (l + t) * d) > dmin) l += t;
    const int j = i + l * d, dn = delta(c, n, i, j);
    int s = 0;
    for (int div = 2;; div *= 2) {
      const int t = (l + div - 1) / div;
      if (delta(c, n, i, i + (s + t) * d) > dn) s += t;
      if (t <= 1) break;
    }
    const int g = i + s * d + std::min(d, 0);
    child[i] = {std::min(i, j) == g ? ~g : g, std::max(i, j) == g + 1 ? ~(g + 1) : g + 1};
  }
  // boxes bottom-up (recursive)
  nodes.assign(n - 1, BvhNode{});
  struct B {
    float lo[3], hi[3];
  };
  std::function<B(int)> box = [&](int link) -> B {
    B b;
    if (link < 0) {
      const float *t = v + 9L * order[~link];
      for (int a = 0; a < 3; a++) {
        b.lo[a] = std::min(t[a], std::min(t[3 + a], t[6 + a]));
        b.hi[a] = std::max(t[a], std::max(t[3 + a], t[6 + a]));
      }
      return b;
    }
    B l = box(child[link].first), r = box(child[link].second);
    BvhNode &nd = nodes[link];
    nd = BvhNode{l.lo[0], l.lo[1], l.lo[2], r.lo[0], l.hi[0], l.hi[1], l.hi[2], r.lo[1],
                 r.lo[2], r.hi[0], r.hi[1], r.hi[2], child[link].first, child[link].second, 0, 0};
    for (int a = 0; a < 3; a++) b.lo[a] = std::min(l.lo[a], r.lo[a]), b.hi[a] = std::max(l.hi[a], r.hi[a]);
    return b;
  };
  box(0);
}

// ---- the integrator's walk (rt0_integrator.h bvh_closest), counting nodes
struct Tri {
  V3 v0, e0, e1;
};
static bool tri_test(const Tri &T, V3 o, V3 d, float tmin, float &t) {
  const V3 h = cross(d, T.e1);
  const float a = dot(T.e0, h);
  const float eps = 0.001f * std::sqrt(dot(T.e0, T.e0)) * std::sqrt(dot(T.e1, T.e1));
  if (a > -eps && a < eps) return false;
  const float f = 1.0f / a;
  const V3 s = o - T.v0;
  const float u = f * dot(s, h);
  if (u < 0.f || u > 1.f) return false;
  const V3 q = cross(s, T.e0);
  const float w = f * dot(d, q);
  if (w < 0.f || u + w > 1.f) return false;
  t = f * dot(T.e1, q);
  return t > 0.001f && t < tmin;
}
static float enter(const float *b, V3 o, V3 inv, float tmin) {
  const float tx0 = (b[0] - o.x) * inv.x, tx1 = (b[3] - o.x) * inv.x;
  const float ty0 = (b[1] - o.y) * inv.y, ty1 = (b[4] - o.y) * inv.y;
  const float tz0 = (b[2] - o.z) * inv.z, tz1 = (b[5] - o.z) * inv.z;
  const float tn = std::max(std::max(std::min(tx0, tx1), std::min(ty0, ty1)), std::max(std::min(tz0, tz1), 0.0f));
  const float tf = std::min(std::min(std::max(tx0, tx1), std::max(ty0, ty1)), std::max(tz0, tz1));
  return (tn <= tf && tn < tmin) ? tn : INFINITY;
}
static int g_order = 0;  // 0: entry distance (tl <= tr); 1: ties by direction along the centre axis; 2: direction only
static int walk(const std::vector<BvhNode> &N, const std::vector<Tri> &T, V3 o, V3 d, float &tmin, bool any,
                long &visits) {
  const V3 inv{1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
  int stk[64], sp = 0, node = 0, best = -1;
  for (;;) {
    const BvhNode &n = N[node];
    const float lb[6] = {n.lx0, n.ly0, n.lz0, n.lx1, n.ly1, n.lz1}, rb[6] = {n.rx0, n.ry0, n.rz0, n.rx1, n.ry1, n.rz1};
    float tl = enter(lb, o, inv, tmin), tr = enter(rb, o, inv, tmin);
    ++visits;
    for (int s = 0; s < 2; s++) {
      const int c = s ? n.right : n.left;
      float &tc = s ? tr : tl;
      if (tc != INFINITY && c < 0) {
        float t;
        if (tri_test(T[~c], o, d, tmin, t)) tmin = t, best = ~c;
        tc = INFINITY;
      }
    }
    if (any && best >= 0) break;
    if (tl != INFINITY && tr != INFINITY) {
      bool lf = tl <= tr;
      if (g_order) {
        const float cx = (n.rx0 + n.rx1) - (n.lx0 + n.lx1), cy = (n.ry0 + n.ry1) - (n.ly0 + n.ly1),
                    cz = (n.rz0 + n.rz1) - (n.lz0 + n.lz1);
        const float ax = std::fabs(cx), ay = std::fabs(cy), az = std::fabs(cz);
        const float dd = (ax >= ay && ax >= az) ? d.x * cx : (ay >= az ? d.y * cy : d.z * cz);
        const bool dir_left = dd >= 0.f;  // moving toward the right child's side: left first
        if (g_order == 2 || tl == tr) lf = dir_left;
      }
      stk[sp++] = lf ? n.right : n.left;
      node = lf ? n.left : n.right;
    } else if (tl != INFINITY) {
      node = n.left;
    } else if (tr != INFINITY) {
      node = n.right;
    } else {
      if (sp == 0) break;
      node = stk[--sp];
    }
  }
  return best;
}

static float sah_cost(const std::vector<BvhNode> &N) {  // sum over inner nodes of child areas / root area
  auto ha = [](float x0, float y0, float z0, float x1, float y1, float z1) {
    const float x = x1 - x0, y = y1 - y0, z = z1 - z0;
    return x * y + y * z + z * x;
  };
  double s = 0;
  for (const BvhNode &n : N) s += ha(n.lx0, n.ly0, n.lz0, n.lx1, n.ly1, n.lz1) + ha(n.rx0, n.ry0, n.rz0, n.rx1, n.ry1, n.rz1);
  const BvhNode &r = N[0];
  const double root = ha(std::min(r.lx0, r.rx0), std::min(r.ly0, r.ry0), std::min(r.lz0, r.rz0), std::max(r.lx1, r.rx1),
                         std::max(r.ly1, r.ry1), std::max(r.lz1, r.rz1));
  return (float)(s / root);
}

int main(int argc, char **argv) {
  if (argc < 2) return 2;
  FILE *f = fopen(argv[1], "rb");
  std::vector<float> v;
  float buf[9];
  while (fread(buf, sizeof(float), 9, f) == 9) v.insert(v.end(), buf, buf + 9);
  fclose(f);
  const int n = (int)(v.size() / 9);
  std::vector<int32_t> owner(n, 0);
  std::vector<BvhNode> Ns;
  std::vector<TriDev> Ts;
  const int depth = rt0h::bvh_build_sah(n, v.data(), owner.data(), Ns, Ts);
  std::vector<Tri> Tsah(n);
  for (int i = 0; i < n; i++)
    Tsah[i] = Tri{{Ts[i].v0x, Ts[i].v0y, Ts[i].v0z}, {Ts[i].e0x, Ts[i].e0y, Ts[i].e0z}, {Ts[i].e1x, Ts[i].e1y, Ts[i].e1z}};
  std::vector<BvhNode> Nl;
  std::vector<int> order;
  lbvh(n, v.data(), Nl, order);
  std::vector<Tri> Tl(n);
  for (int i = 0; i < n; i++) {
    const float *t = v.data() + 9L * order[i];
    Tl[i] = Tri{{t[0], t[1], t[2]}, {t[3] - t[0], t[4] - t[1], t[5] - t[2]}, {t[6] - t[0], t[7] - t[1], t[8] - t[2]}};
  }
  printf("triangles %d  sah depth %d  SAH cost: lbvh %.1f  sah %.1f\n", n, depth, sah_cost(Nl), sah_cost(Ns));
  // C5 camera (workloads.json) and lights
  const V3 cam{0.f, 0.4f, 1.5f}, w = nrm({0.f, -0.3f, -1.f});
  const V3 u = nrm(cross(w, {0.f, 1.f, 0.f})), vv = cross(u, w);
  const float tv = std::tan(55.f * 0.01745329f * 0.5f);
  const V3 lights[10] = {{2.2f, 1.6f, -2.5f},   {1.78f, 1.9f, -1.207f}, {0.68f, 1.6f, -0.408f}, {-0.68f, 1.9f, -0.408f},
                         {-1.78f, 1.6f, -1.207f}, {-2.2f, 1.9f, -2.5f},  {-1.78f, 1.6f, -3.793f}, {-0.68f, 1.9f, -4.592f},
                         {0.68f, 1.6f, -4.592f}, {1.78f, 1.9f, -3.793f}};
  std::mt19937 rng(7);
  std::uniform_real_distribution<float> U(0.f, 1.f);
  const char *names[4] = {"camera (closest)", "sphere-surface scatter (closest)", "ground->light (any)",
                          "surface->light (any)"};
  long vis[2][4] = {}, cnt[4] = {}, hit_agree = 0, hit_total = 0;
  const int R = 256;
  if (getenv("ORDER")) g_order = atoi(getenv("ORDER"));
  for (int py = 0; py < R; py++)
    for (int px = 0; px < R; px++) {
      const float sx = 2.f * (px + 0.5f) / R - 1.f, sy = 2.f * (py + 0.5f) / R - 1.f;
      const V3 d = nrm(u * (sx * tv) + vv * (sy * tv) + w);
      float tq = 1e4f;
      const float tp = (-1.0f - cam.y) / d.y;  // ground plane y = -1
      if (d.y < 0.f) tq = tp;
      float ts = tq, tl = tq;
      long a = 0, b = 0;
      const int hs = walk(Ns, Tsah, cam, d, ts, false, a), hl = walk(Nl, Tl, cam, d, tl, false, b);
      vis[0][0] += a, vis[1][0] += b, cnt[0]++;
      hit_total++;
      hit_agree += (hs >= 0) == (hl >= 0) && ts == tl;
      V3 p;
      if (hs >= 0) {
        p = cam + d * ts;
        // scattered rays from the surface hit: one outward, one inward (refraction-like)
        const V3 nn = nrm(p - V3{0.f, 0.f, -2.5f});
        for (int s = 0; s < 2; s++) {
          V3 r = nrm(V3{U(rng) - 0.5f, U(rng) - 0.5f, U(rng) - 0.5f});
          if ((dot(r, nn) > 0.f) != (s == 0)) r = r * -1.f;
          const V3 o = p + r * 0.002f;
          float t1 = 1e4f, t2 = 1e4f;
          long c1 = 0, c2 = 0;
          walk(Ns, Tsah, o, r, t1, false, c1);
          walk(Nl, Tl, o, r, t2, false, c2);
          vis[0][1] += c1, vis[1][1] += c2, cnt[1]++;
        }
        for (int k = 0; k < 10; k += 3) {  // shadow rays to some lights
          const V3 o = p + nn * 0.001f, L = lights[k] - o;
          const float dist = std::sqrt(dot(L, L));
          const V3 r = L * (1.f / dist);
          float t1 = dist, t2 = dist;
          long c1 = 0, c2 = 0;
          walk(Ns, Tsah, o, r, t1, true, c1);
          walk(Nl, Tl, o, r, t2, true, c2);
          vis[0][3] += c1, vis[1][3] += c2, cnt[3]++;
        }
      } else if (d.y < 0.f) {
        p = cam + d * tq;
        for (int k = 0; k < 10; k += 3) {
          const V3 o = p + V3{0.f, 0.001f, 0.f}, L = lights[k] - o;
          const float dist = std::sqrt(dot(L, L));
          const V3 r = L * (1.f / dist);
          float t1 = dist, t2 = dist;
          long c1 = 0, c2 = 0;
          walk(Ns, Tsah, o, r, t1, true, c1);
          walk(Nl, Tl, o, r, t2, true, c2);
          vis[0][2] += c1, vis[1][2] += c2, cnt[2]++;
        }
      }
    }
  printf("closest-hit agreement on camera rays: %.5f\n", (double)hit_agree / hit_total);
  printf("%-36s %10s %8s %8s %7s\n", "ray set", "rays", "lbvh", "sah", "ratio");
  long tot[2] = {};
  for (int s = 0; s < 4; s++) {
    tot[0] += vis[0][s], tot[1] += vis[1][s];
    printf("%-36s %10ld %8.2f %8.2f %7.3f\n", names[s], cnt[s], (double)vis[1][s] / cnt[s], (double)vis[0][s] / cnt[s],
           (double)vis[0][s] / std::max(1L, vis[1][s]));
  }
  printf("%-36s %10s %8s %8s %7.3f\n", "all", "", "", "", (double)tot[0] / tot[1]);
  return 0;
}
