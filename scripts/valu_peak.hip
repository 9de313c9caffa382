// valu_peak.hip -- measured VALU issue rates of MI355X (gfx950) for the
// roofline of the rt0 integrator (a branchy scalar-FP32 VALU kernel).
//
// MI355X_MICROARCH.md quotes 157.3 TFLOP/s FP32 vector (spec): 256 CUs x
// 4 SIMDs x 2.4 GHz x 64 FLOP/clk.  Which instructions reach that rate is
// measured here rather than assumed: each kernel runs 16 independent chains
// of ONE instruction per lane (inline asm, so the compiler can neither fuse,
// pack nor fold them) over a long loop at full occupancy (8192 workgroups of
// 256), timed with hipEvents over several launches after a warm-up.
//   v_fma_f32 / v_pk_fma_f32   -> FP32 TFLOP/s (2 / 4 FLOP per lane-op)
//   every kernel               -> wave64 instructions per SIMD per ns, and
//                                 SIMD cycles per instruction at the clock
//                                 the fma kernel implies (spec: 2 cycles)
// plus pairs interleaved 1:1 (fma+add_u32, fma+exp, fma+cndmask) to see
// whether two instruction classes share one issue port.  Covers the classes
// the integrator issues: FP32 add/mul/fma, moves, integer add/shift/multiply
// (the RNG hash, raytracer.glsl:302-306), conversions, floor (hash2), the
// transcendentals (exp, sqrt, rcp, sin), compares and selects.
#include <hip/hip_runtime.h>

#include <cstdio>

// build: hipcc -O3 -fno-slp-vectorize --offload-arch=gfx950 valu_peak.hip -o valu_peak

#define ITERS 2048

#define CHAINS(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)

// one kernel per instruction; `body` is the asm statement applied to chain k
#define VKERNEL(name, decl, init, body, fold)                                  \
  __global__ __launch_bounds__(256) void name(float *out, float a, float b) { \
    decl;                                                                      \
    init;                                                                      \
    for (int i = 0; i < ITERS; i++) {                                          \
      CHAINS(body)                                                             \
    }                                                                          \
    float s = 0.f;                                                             \
    fold;                                                                      \
    if (s == 12345.0f) out[0] = s;                                             \
  }

#define DECL_F float x[16]
#define INIT_F                                           \
  _Pragma("unroll") for (int k = 0; k < 16; k++) x[k] = threadIdx.x * 1e-7f + k
#define FOLD_F _Pragma("unroll") for (int k = 0; k < 16; k++) s += x[k]

#define B_FMA(k) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x[k]) : "v"(a), "v"(b));
#define B_ADD(k) asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[k]) : "v"(b));
#define B_MUL(k) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(x[k]) : "v"(a));
#define B_MOV(k) asm volatile("v_mov_b32 %0, %0" : "+v"(x[k]));
#define B_IADD(k) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[k]) : "v"(b));
#define B_EXP(k) asm volatile("v_exp_f32 %0, %0" : "+v"(x[k]));
#define B_IMUL(k) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x[k]) : "v"(b));
#define B_CVT(k) asm volatile("v_cvt_f32_i32 %0, %0" : "+v"(x[k]));
#define B_FLOOR(k) asm volatile("v_floor_f32 %0, %0" : "+v"(x[k]));
#define B_SQRT(k) asm volatile("v_sqrt_f32 %0, %0" : "+v"(x[k]));
#define B_RCP(k) asm volatile("v_rcp_f32 %0, %0" : "+v"(x[k]));
#define B_SIN(k) asm volatile("v_sin_f32 %0, %0" : "+v"(x[k]));
#define B_LSHR(k) asm volatile("v_lshrrev_b32 %0, %1, %0" : "+v"(x[k]) : "v"(b));
#define B_CND(k) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(x[k]) : "v"(b), "s"(m));
#define B_CMP(k) asm volatile("v_cmp_gt_f32_e64 %0, %1, %2" : "=s"(mk[k & 3]) : "v"(x[k]), "v"(a));
#define B_FMA_IADD(k) \
  asm volatile("v_fma_f32 %0, %0, %2, %3\n\tv_add_u32 %1, %1, %3" : "+v"(x[k]), "+v"(y[k]) : "v"(a), "v"(b));
#define B_FMA_EXP(k) \
  asm volatile("v_fma_f32 %0, %0, %2, %3\n\tv_exp_f32 %1, %1" : "+v"(x[k]), "+v"(y[k]) : "v"(a), "v"(b));
#define B_FMA_CND(k) \
  asm volatile("v_fma_f32 %0, %0, %2, %3\n\tv_cndmask_b32_e64 %1, %1, %3, %4" : "+v"(x[k]), "+v"(y[k]) : "v"(a), "v"(b), "s"(m));

typedef float f2 __attribute__((ext_vector_type(2)));
#define B_PK(k) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(p[k]) : "v"(va), "v"(vb));

VKERNEL(k_fma, DECL_F, INIT_F, B_FMA, FOLD_F)
VKERNEL(k_add, DECL_F, INIT_F, B_ADD, FOLD_F)
VKERNEL(k_mul, DECL_F, INIT_F, B_MUL, FOLD_F)
VKERNEL(k_mov, DECL_F, INIT_F, B_MOV, FOLD_F)
VKERNEL(k_iadd, DECL_F, INIT_F, B_IADD, FOLD_F)
VKERNEL(k_exp, DECL_F, INIT_F, B_EXP, FOLD_F)
VKERNEL(k_imul, DECL_F, INIT_F, B_IMUL, FOLD_F)
VKERNEL(k_cvt, DECL_F, INIT_F, B_CVT, FOLD_F)
VKERNEL(k_floor, DECL_F, INIT_F, B_FLOOR, FOLD_F)
VKERNEL(k_sqrt, DECL_F, INIT_F, B_SQRT, FOLD_F)
VKERNEL(k_rcp, DECL_F, INIT_F, B_RCP, FOLD_F)
VKERNEL(k_sin, DECL_F, INIT_F, B_SIN, FOLD_F)
VKERNEL(k_lshr, DECL_F, INIT_F, B_LSHR, FOLD_F)
VKERNEL(k_cnd, DECL_F; unsigned long long m = __ballot(threadIdx.x & 1), INIT_F, B_CND, FOLD_F)
VKERNEL(k_cmp, DECL_F; unsigned long long mk[4]; mk[0] = mk[1] = mk[2] = mk[3] = 0, INIT_F, B_CMP,
        FOLD_F; s += (float)(mk[0] ^ mk[1] ^ mk[2] ^ mk[3]))
__global__ __launch_bounds__(256) void k_pk_fma(float *out, float a, float b) {
  f2 p[16];
  f2 va, vb;
  va.x = va.y = a;
  vb.x = vb.y = b;
#pragma unroll
  for (int k = 0; k < 16; k++) {
    p[k].x = threadIdx.x * 1e-7f + k;
    p[k].y = threadIdx.x * 2e-7f + k;
  }
  for (int i = 0; i < ITERS; i++) {
    CHAINS(B_PK)
  }
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < 16; k++) s += p[k].x + p[k].y;
  if (s == 12345.0f) out[0] = s;
}
VKERNEL(k_fma_iadd, DECL_F; float y[16], INIT_F; _Pragma("unroll") for (int k = 0; k < 16; k++) y[k] = x[k],
        B_FMA_IADD, FOLD_F; _Pragma("unroll") for (int k = 0; k < 16; k++) s += y[k])
VKERNEL(k_fma_exp, DECL_F; float y[16], INIT_F; _Pragma("unroll") for (int k = 0; k < 16; k++) y[k] = x[k],
        B_FMA_EXP, FOLD_F; _Pragma("unroll") for (int k = 0; k < 16; k++) s += y[k])
VKERNEL(k_fma_cnd, DECL_F; float y[16]; unsigned long long m = __ballot(threadIdx.x & 1),
        INIT_F; _Pragma("unroll") for (int k = 0; k < 16; k++) y[k] = x[k], B_FMA_CND,
        FOLD_F; _Pragma("unroll") for (int k = 0; k < 16; k++) s += y[k])

// exactness of the hardware reciprocal square root at powers of four (the
// integrator normalises unit axis vectors: is v_rsq_f32(1) exactly 1?)
__global__ void k_rsq_exact(const float *in, float *out) {
  const int i = threadIdx.x;
  out[i] = __builtin_amdgcn_rsqf(in[i]);
}

struct K {
  const char *name;
  void (*fn)(float *, float, float);
  int instr_per_chain_iter;  // wave instructions per chain per iteration
  double flop_per_lane_instr;  // FP32 FLOP per lane per instruction (0: not an FP32 arithmetic op)
};

int main() {
  float *out;
  (void)hipMalloc(&out, 4);
  const dim3 G(8192), B(256);
  const K ks[] = {{"v_fma_f32", k_fma, 1, 2.0},       {"v_pk_fma_f32", k_pk_fma, 1, 4.0},
                  {"v_add_f32", k_add, 1, 1.0},       {"v_mul_f32", k_mul, 1, 1.0},
                  {"v_mov_b32", k_mov, 1, 0.0},       {"v_add_u32", k_iadd, 1, 0.0},
                  {"v_exp_f32", k_exp, 1, 0.0},       {"v_cndmask_b32", k_cnd, 1, 0.0},
                  {"v_cmp_gt_f32", k_cmp, 1, 0.0},    {"v_mul_lo_u32", k_imul, 1, 0.0},
                  {"v_cvt_f32_i32", k_cvt, 1, 0.0},   {"v_floor_f32", k_floor, 1, 0.0},
                  {"v_sqrt_f32", k_sqrt, 1, 0.0},     {"v_rcp_f32", k_rcp, 1, 0.0},
                  {"v_sin_f32", k_sin, 1, 0.0},       {"v_lshrrev_b32", k_lshr, 1, 0.0},
                  {"fma+add_u32", k_fma_iadd, 2, 1.0},
                  {"fma+exp", k_fma_exp, 2, 1.0},     {"fma+cndmask", k_fma_cnd, 2, 1.0}};
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const double waves = (double)G.x * B.x / 64.0;
  double fma_ns_per_instr = 0.0;  // per SIMD
  for (const K &k : ks) {
    float ms = 0.f;
    for (int w = 0; w < 2; w++) {  // warm-up (clock ramp), then timed
      const int reps = w ? 10 : 3;
      (void)hipEventRecord(e0);
      for (int r = 0; r < reps; r++) hipLaunchKernelGGL(k.fn, G, B, 0, 0, out, 0.999f, 1e-3f);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      (void)hipEventElapsedTime(&ms, e0, e1);
      ms /= reps;
    }
    const double instr = waves * ITERS * 16.0 * k.instr_per_chain_iter;  // wave instructions per launch
    const double per_simd_per_ns = instr / 1024.0 / (ms * 1e6);
    if (fma_ns_per_instr == 0.0) fma_ns_per_instr = 1.0 / per_simd_per_ns;
    const double tflops = instr * 64.0 * k.flop_per_lane_instr / (ms * 1e-3) / 1e12;
    printf("{\"kernel\": \"%s\", \"tflops\": %.2f, \"wave_instr_per_simd_per_ns\": %.4f, "
           "\"relative_to_fma\": %.3f, \"ms_per_launch\": %.4f}\n",
           k.name, tflops, per_simd_per_ns, per_simd_per_ns * fma_ns_per_instr, ms);
  }
  {
    const float h_in[4] = {1.0f, 4.0f, 0.25f, 16.0f};
    float *d_in, *d_out, h_out[4];
    (void)hipMalloc(&d_in, sizeof h_in);
    (void)hipMalloc(&d_out, sizeof h_out);
    (void)hipMemcpy(d_in, h_in, sizeof h_in, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_rsq_exact, dim3(1), dim3(4), 0, 0, d_in, d_out);
    (void)hipMemcpy(h_out, d_out, sizeof h_out, hipMemcpyDeviceToHost);
    printf("{\"kernel\": \"v_rsq_f32 exactness\", \"in\": [1, 4, 0.25, 16], \"out\": [%.9g, %.9g, %.9g, %.9g], "
           "\"exact\": %s}\n",
           h_out[0], h_out[1], h_out[2], h_out[3],
           (h_out[0] == 1.0f && h_out[1] == 0.5f && h_out[2] == 2.0f && h_out[3] == 0.25f) ? "true" : "false");
  }
  if (hipGetLastError() != hipSuccess) return 1;
  return 0;
}
