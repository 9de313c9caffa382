// valu_peak.hip -- measured FP32 vector peaks of MI355X (gfx950) for the
// roofline of the rt0 integrator (a branchy scalar-FP32 VALU kernel).
//
// MI355X_MICROARCH.md quotes 157.3 TFLOP/s FP32 vector (spec): 256 CUs x
// 4 SIMD32 x 2.4 GHz x 64 FLOP/clk, which needs every FMA to be a PACKED
// v_pk_fma_f32 (two lanes' worth per 32-wide pass).  Scalar v_fma_f32 code --
// the compiler's output for the integrator, -fno-slp-vectorize -- can reach at
// most half of it.  Each kernel runs 16 independent FMA chains per lane over
// a long loop at full occupancy (8 waves/SIMD, 8192 workgroups):
//   k_fma     v_fma_f32          (2 FLOP per lane-instruction)
//   k_pk_fma  v_pk_fma_f32       (4 FLOP per lane-instruction)
// Timed with hipEvents over several launches; FLOP/s = 2 x FMAs / s.
#include <hip/hip_runtime.h>

#include <cstdio>

// build: hipcc -O3 -fno-slp-vectorize --offload-arch=gfx950 valu_peak.hip -o valu_peak
// (without -fno-slp-vectorize the compiler packs k_fma's chains into v_pk_fma_f32 too)

typedef float f2 __attribute__((ext_vector_type(2)));

#define ITERS 4096

__global__ __launch_bounds__(256) void k_fma(float *out, float a, float b) {
  float x[16];
#pragma unroll
  for (int k = 0; k < 16; k++) x[k] = threadIdx.x * 1e-7f + k;
  for (int i = 0; i < ITERS; i++) {
#pragma unroll
    for (int k = 0; k < 16; k++) x[k] = __builtin_fmaf(x[k], a, b);
  }
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < 16; k++) s += x[k];
  if (s == 12345.0f) out[0] = s;
}

__global__ __launch_bounds__(256) void k_pk_fma(float *out, float a, float b) {
  f2 x[8];
#pragma unroll
  for (int k = 0; k < 8; k++) x[k] = f2{threadIdx.x * 1e-7f + k, threadIdx.x * 2e-7f + k};
  const f2 va = f2{a, a}, vb = f2{b, b};
  for (int i = 0; i < ITERS; i++) {
#pragma unroll
    for (int k = 0; k < 8; k++) x[k] = __builtin_elementwise_fma(x[k], va, vb);
  }
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < 8; k++) s += x[k].x + x[k].y;
  if (s == 12345.0f) out[0] = s;
}

int main() {
  float *out;
  (void)hipMalloc(&out, 4);
  const dim3 G(8192), B(256);
  const double fmas = (double)G.x * B.x * ITERS * 16;  // both kernels: 16 FMA per lane per iteration
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const char *names[2] = {"v_fma_f32", "v_pk_fma_f32"};
  for (int k = 0; k < 2; k++) {
    for (int w = 0; w < 2; w++) {  // warm-up (clock ramp), then timed
      const int reps = w ? 10 : 3;
      (void)hipEventRecord(e0);
      for (int r = 0; r < reps; r++) {
        if (k == 0) hipLaunchKernelGGL(k_fma, G, B, 0, 0, out, 0.999f, 1e-3f);
        else hipLaunchKernelGGL(k_pk_fma, G, B, 0, 0, out, 0.999f, 1e-3f);
      }
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms = 0.f;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (w) printf("{\"kernel\": \"%s\", \"tflops\": %.2f, \"ms_per_launch\": %.4f}\n", names[k],
                    2.0 * fmas * reps / (ms * 1e-3) / 1e12, ms / reps);
    }
  }
  if (hipGetLastError() != hipSuccess) return 1;
  return 0;
}
