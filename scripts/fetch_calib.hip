// fetch_calib.hip -- calibrate rocprofv3's FETCH_SIZE on gfx950 for the access
// shapes of the rt0 kernels (VERDICT r02 "Next" item 1).
//
// MI355X_MICROARCH.md (HBM): FETCH_SIZE reports half the bytes of a 16-B/lane
// streaming read; other widths are uncalibrated.  The C3/C5 traffic ratios in
// profiles/ were derived with that x2 factor, but their reads are 64-B BVH
// node gathers (four float4 per lane, random nodes) and bilinear reservoir taps
// (2 x 2 float4 texels per lane: 32 contiguous bytes in each of two rows).
// Each kernel below reads a 1 GiB table (4x the Infinity Cache) EXACTLY ONCE
// in one of those shapes, in random order, so the true HBM bytes are known:
//   k_stream  16 B per lane, consecutive lanes consecutive (the guide's case)
//   k_node64  64 B per lane (4 x float4), lanes at random 64-B records
//   k_bilin   2 x 2 float4 texels per lane (x, x+1) x (y, y+1) of a 4096-wide
//             plane, lanes at random 2x2 blocks
// Run under `rocprofv3 --pmc FETCH_SIZE --kernel-trace` and divide
// FETCH_SIZE x 1024 by the printed byte counts (scripts/fetch_calib.py).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                    \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

__global__ void k_stream(const float4 *__restrict__ a, size_t n, float *__restrict__ out) {
  float s = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const float4 v = a[i];
    s += v.x + v.y + v.z + v.w;
  }
  if (s == 1234.5f) out[0] = s;  // never true for the zero table: keeps the loads live
}

// i -> (i * A + C) mod 2^k: a bijection on [0, 2^k) (A odd) that sends
// neighbouring lanes to records ~A apart, so no two lanes of a wave share a
// line and every record is read exactly once, with no permutation table to read
__device__ __forceinline__ uint32_t scatter(uint32_t i, uint32_t mask) { return (i * 2654435761u + 40503u) & mask; }

__global__ void k_node64(const float4 *__restrict__ a, size_t n_rec, float *__restrict__ out) {
  float s = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n_rec; i += (size_t)gridDim.x * blockDim.x) {
    const float4 *r = a + 4 * (size_t)scatter((uint32_t)i, (uint32_t)n_rec - 1u);
    const float4 p = r[0], q = r[1], u = r[2], v = r[3];
    s += p.x + q.y + u.z + v.w;
  }
  if (s == 1234.5f) out[0] = s;
}

__global__ void k_bilin(const float4 *__restrict__ a, size_t n_blk, int width, float *__restrict__ out) {
  const int bw = width / 2;
  float s = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n_blk; i += (size_t)gridDim.x * blockDim.x) {
    const uint32_t b = scatter((uint32_t)i, (uint32_t)n_blk - 1u);
    const size_t x = 2 * (size_t)(b % bw), y = 2 * (size_t)(b / bw);
    const float4 t00 = a[y * width + x], t10 = a[y * width + x + 1];
    const float4 t01 = a[(y + 1) * width + x], t11 = a[(y + 1) * width + x + 1];
    s += t00.x + t10.y + t01.z + t11.w;
  }
  if (s == 1234.5f) out[0] = s;
}

int main() {
  const size_t bytes = 1ull << 30;  // 1 GiB: past the 256 MiB Infinity Cache
  const size_t n4 = bytes / 16;
  float4 *a = nullptr;
  float *out = nullptr;
  CK(hipMalloc(&a, bytes));
  CK(hipMemset(a, 0, bytes));
  CK(hipMalloc(&out, 4));
  const size_t n_rec = bytes / 64;  // 2^24 records of 64 B
  const dim3 G(256 * 8 * 8), B(256);
  // bilinear blocks: a 4096-wide plane of float4 (64 KiB per row, 16384 rows),
  // 2^24 blocks of 2 x 2 texels
  const int width = 4096;
  const size_t n_blk = (n4 / width / 2) * (width / 2);
  for (int rep = 0; rep < 2; rep++) {
    hipLaunchKernelGGL(k_stream, G, B, 0, 0, a, n4, out);
    hipLaunchKernelGGL(k_node64, G, B, 0, 0, a, n_rec, out);
    hipLaunchKernelGGL(k_bilin, G, B, 0, 0, a, n_blk, width, out);
  }
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  printf("{\"k_stream\": %zu, \"k_node64\": %zu, \"k_bilin\": %zu}\n", n4 * 16, n_rec * 64, n_blk * 64);
  return 0;
}
