// rt0_bvh.hip -- LBVH build on gfx950 for the triangle models.
//
// The reference has no acceleration structure: intersection() loops over
// every mesh (raytracer.glsl:1006-1036), and its triangle path (iTriangle,
// 864-892, and the bvh.js/mesh.js of .gitignore) was never shipped.  For the
// ~100k-triangle model of BASELINE config 5 a per-ray loop is hopeless, so
// the triangles get a linear BVH built on the device (Karras 2012, the
// Morton-code radix tree behind HLBVH):
//   1. k_morton   30-bit Morton code of each triangle centroid (scene box);
//   2. rocPRIM/hipCUB radix sort of (code, triangle) pairs;
//   3. k_karras   one thread per internal node finds its key range and split
//                 (ties broken by index, so duplicate codes still form a tree);
//   4. k_refit    bottom-up boxes, one thread per leaf, the second thread to
//                 reach a node (atomic counter) merges its children;
//   5. k_pack     64-B BvhNodes (both child boxes in the parent: one fetch per
//                 visited node tests two boxes) and 48-B TriDevs in leaf order;
//   6. k_depth    the deepest leaf, checked against the traversal stack.
// All kernels are one pass over n elements: the build is HBM/latency bound and
// takes well under a millisecond for 100k triangles.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstdint>
#include <vector>

#include "rt0_device.h"

namespace {

__device__ __forceinline__ uint32_t spread10(uint32_t v) {  // 10 bits -> every third bit
  v = (v * 0x00010001u) & 0xFF0000FFu;
  v = (v * 0x00000101u) & 0x0F00F00Fu;
  v = (v * 0x00000011u) & 0xC30C30C3u;
  v = (v * 0x00000005u) & 0x49249249u;
  return v;
}

__global__ void k_morton(int n, const float *__restrict__ v, float3 lo, float3 inv_ext, uint32_t *__restrict__ code,
                         uint32_t *__restrict__ idx) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float *t = v + 9 * (size_t)i;
  const float cx = (t[0] + t[3] + t[6]) * (1.0f / 3.0f), cy = (t[1] + t[4] + t[7]) * (1.0f / 3.0f),
              cz = (t[2] + t[5] + t[8]) * (1.0f / 3.0f);
  auto q = [](float x) { return (uint32_t)fminf(fmaxf(x * 1024.0f, 0.0f), 1023.0f); };
  const uint32_t x = q((cx - lo.x) * inv_ext.x), y = q((cy - lo.y) * inv_ext.y), z = q((cz - lo.z) * inv_ext.z);
  code[i] = (spread10(x) << 2) | (spread10(y) << 1) | spread10(z);
  idx[i] = (uint32_t)i;
}

__device__ __forceinline__ int delta(const uint32_t *__restrict__ c, int n, int i, int j) {
  if (j < 0 || j >= n) return -1;
  const uint32_t a = c[i], b = c[j];
  return a != b ? __clz(a ^ b) : 32 + __clz((uint32_t)(i ^ j));
}

// internal node i of [0, n-2]; combined index space: internal k -> k, leaf k -> n-1+k
__global__ void k_karras(int n, const uint32_t *__restrict__ c, int2 *__restrict__ child, int *__restrict__ parent) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n - 1) return;
  const int d = delta(c, n, i, i + 1) - delta(c, n, i, i - 1) >= 0 ? 1 : -1;
  const int dmin = delta(c, n, i, i - d);
  int lmax = 2;
  while (delta(c, n, i, i + lmax * d) > dmin) lmax *= 2;
  int l = 0;
  for (int t = lmax / 2; t >= 1; t /= 2)
    if (delta(c, n, i, i + (l + t) * d) > dmin) l += t;
  const int j = i + l * d;
  const int dnode = delta(c, n, i, j);
  int s = 0;
  for (int div = 2;; div *= 2) {
    const int t = (l + div - 1) / div;
    if (delta(c, n, i, i + (s + t) * d) > dnode) s += t;
    if (t <= 1) break;
  }
  const int g = i + s * d + min(d, 0);
  const int left = min(i, j) == g ? (n - 1) + g : g;
  const int right = max(i, j) == g + 1 ? (n - 1) + g + 1 : g + 1;
  child[i] = make_int2(left, right);
  parent[left] = i;
  parent[right] = i;
}

struct Box {
  float x0, y0, z0, x1, y1, z1;
};

__global__ void k_refit(int n, const float *__restrict__ v, const uint32_t *__restrict__ idx,
                        const int2 *__restrict__ child, const int *__restrict__ parent, Box *__restrict__ box,
                        int *__restrict__ flag) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float *t = v + 9 * (size_t)idx[i];
  Box b;
  b.x0 = fminf(t[0], fminf(t[3], t[6]));
  b.y0 = fminf(t[1], fminf(t[4], t[7]));
  b.z0 = fminf(t[2], fminf(t[5], t[8]));
  b.x1 = fmaxf(t[0], fmaxf(t[3], t[6]));
  b.y1 = fmaxf(t[1], fmaxf(t[4], t[7]));
  b.z1 = fmaxf(t[2], fmaxf(t[5], t[8]));
  int node = (n - 1) + i;
  box[node] = b;
  if (n == 1) return;
  __threadfence();
  node = parent[node];
  for (int guard = 0; guard < 256; ++guard) {  // depth < RT0_BVH_STACK (checked): the guard never binds
    // the first child to arrive leaves; the second merges both boxes
    if (atomicAdd(&flag[node], 1) == 0) return;
    __threadfence();
    const int2 ch = child[node];
    // the sibling box was written by another CU in this kernel: read around
    // the (non-coherent) L1
    const volatile Box *vb = box;
    const Box a{vb[ch.x].x0, vb[ch.x].y0, vb[ch.x].z0, vb[ch.x].x1, vb[ch.x].y1, vb[ch.x].z1};
    const Box c{vb[ch.y].x0, vb[ch.y].y0, vb[ch.y].z0, vb[ch.y].x1, vb[ch.y].y1, vb[ch.y].z1};
    Box m;
    m.x0 = fminf(a.x0, c.x0);
    m.y0 = fminf(a.y0, c.y0);
    m.z0 = fminf(a.z0, c.z0);
    m.x1 = fmaxf(a.x1, c.x1);
    m.y1 = fmaxf(a.y1, c.y1);
    m.z1 = fmaxf(a.z1, c.z1);
    box[node] = m;
    __threadfence();
    if (node == 0) return;
    node = parent[node];
  }
}

__global__ void k_pack(int n, const float *__restrict__ v, const int32_t *__restrict__ model,
                       const uint32_t *__restrict__ idx, const int2 *__restrict__ child, const Box *__restrict__ box,
                       BvhNode *__restrict__ nodes, TriDev *__restrict__ tris) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  {  // triangle i in leaf order
    const uint32_t src = idx[i];
    const float *t = v + 9 * (size_t)src;
    TriDev d;
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
    d.eps = 0.001f * sqrtf(d.e0x * d.e0x + d.e0y * d.e0y + d.e0z * d.e0z) *
            sqrtf(d.e1x * d.e1x + d.e1y * d.e1y + d.e1z * d.e1z);
    tris[i] = d;
  }
  if (n == 1 && i == 0) {  // a one-triangle tree: the root holds the leaf twice
    const Box b = box[0];
    nodes[0] = BvhNode{b.x0, b.y0, b.z0, b.x0, b.x1, b.y1, b.z1, b.y0, b.z0, b.x1, b.y1, b.z1, ~0, ~0, 0, 0};
    return;
  }
  if (i >= n - 1) return;
  const int2 ch = child[i];
  const Box l = box[ch.x], r = box[ch.y];
  BvhNode nd;
  nd.lx0 = l.x0;
  nd.ly0 = l.y0;
  nd.lz0 = l.z0;
  nd.lx1 = l.x1;
  nd.ly1 = l.y1;
  nd.lz1 = l.z1;
  nd.rx0 = r.x0;
  nd.ry0 = r.y0;
  nd.rz0 = r.z0;
  nd.rx1 = r.x1;
  nd.ry1 = r.y1;
  nd.rz1 = r.z1;
  nd.left = ch.x >= n - 1 ? ~(ch.x - (n - 1)) : ch.x;
  nd.right = ch.y >= n - 1 ? ~(ch.y - (n - 1)) : ch.y;
  nd.pad0 = nd.pad1 = 0;
  nodes[i] = nd;
}

__global__ void k_depth(int n, const int *__restrict__ parent, int *__restrict__ depth) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || n == 1) return;
  int node = (n - 1) + i, d = 0;
  while (node != 0 && d < 1024) {  // a corrupt tree reports depth 1024 instead of hanging
    node = parent[node];
    ++d;
  }
  atomicMax(depth, d);
}

}  // namespace

// Build the LBVH of n world-space triangles (v: 9 floats each, model: owner
// index) into caller-allocated nodes[max(1, n-1)] and tris[n].  Returns the
// tree depth (edges root -> deepest leaf) in *depth_out.
extern "C" hipError_t rt0_bvh_build(int n, const float *d_v, const int32_t *d_model, float3 lo, float3 hi,
                                    BvhNode *d_nodes, TriDev *d_tris, int *depth_out,
                                    hipStream_t s) {
  if (n <= 0) return hipErrorInvalidValue;
  const float3 ext = make_float3(hi.x - lo.x, hi.y - lo.y, hi.z - lo.z);
  const float3 inv = make_float3(ext.x > 0.f ? 1.0f / ext.x : 0.f, ext.y > 0.f ? 1.0f / ext.y : 0.f,
                                 ext.z > 0.f ? 1.0f / ext.z : 0.f);
  uint32_t *code = nullptr, *code2 = nullptr, *idx = nullptr, *idx2 = nullptr;
  int2 *child = nullptr;
  int *parent = nullptr, *flag = nullptr, *depth = nullptr;
  Box *box = nullptr;
  void *tmp = nullptr;
  size_t tmp_bytes = 0;
  hipError_t e = hipSuccess;
  const int B = 256, G = (n + B - 1) / B;
#define TRY(x)                 \
  do {                         \
    e = (x);                   \
    if (e != hipSuccess) goto out; \
  } while (0)
  TRY(hipMallocAsync((void **)&code, n * 4, s));
  TRY(hipMallocAsync((void **)&code2, n * 4, s));
  TRY(hipMallocAsync((void **)&idx, n * 4, s));
  TRY(hipMallocAsync((void **)&idx2, n * 4, s));
  TRY(hipMallocAsync((void **)&child, (size_t)(n > 1 ? n - 1 : 1) * sizeof(int2), s));
  TRY(hipMallocAsync((void **)&parent, (size_t)(2 * n) * 4, s));
  TRY(hipMallocAsync((void **)&flag, (size_t)n * 4, s));
  TRY(hipMallocAsync((void **)&depth, 4, s));
  TRY(hipMallocAsync((void **)&box, (size_t)(2 * n) * sizeof(Box), s));
  TRY(hipMemsetAsync(flag, 0, (size_t)n * 4, s));
  TRY(hipMemsetAsync(depth, 0, 4, s));
  hipLaunchKernelGGL(k_morton, dim3(G), dim3(B), 0, s, n, d_v, lo, inv, code, idx);
  TRY(hipGetLastError());
  TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, code, code2, idx, idx2, n, 0, 30, s));
  TRY(hipMallocAsync(&tmp, tmp_bytes, s));
  TRY(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, code, code2, idx, idx2, n, 0, 30, s));
  if (n > 1) {
    hipLaunchKernelGGL(k_karras, dim3((n - 1 + B - 1) / B), dim3(B), 0, s, n, code2, child, parent);
    TRY(hipGetLastError());
  }
  hipLaunchKernelGGL(k_refit, dim3(G), dim3(B), 0, s, n, d_v, idx2, child, parent, box, flag);
  TRY(hipGetLastError());
  // (n == 1: leaf 0 and the root share combined index 0, so box[0] is the leaf box)
  hipLaunchKernelGGL(k_pack, dim3(G), dim3(B), 0, s, n, d_v, d_model, idx2, child, box, d_nodes, d_tris);
  TRY(hipGetLastError());
  hipLaunchKernelGGL(k_depth, dim3(G), dim3(B), 0, s, n, parent, depth);
  TRY(hipGetLastError());
  TRY(hipMemcpyAsync(depth_out, depth, 4, hipMemcpyDeviceToHost, s));
  TRY(hipStreamSynchronize(s));
out:
  for (void *p : {(void *)code, (void *)code2, (void *)idx, (void *)idx2, (void *)child, (void *)parent, (void *)flag,
                  (void *)depth, (void *)box, tmp})
    if (p) (void)hipFreeAsync(p, s);
  (void)hipStreamSynchronize(s);
  return e;
#undef TRY
}
