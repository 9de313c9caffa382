// rt0_pass_inst.hip -- one ahead-of-time instance of the pass kernel, selected
// by RT0_VARIANT (the Makefile builds this file five times, in parallel):
//   0 Cornell-class  1 +SDF  2 +volumetrics/spectral  3 +ReSTIR  4 counting.
// The instances read the scene from HBM (DynScene) and the flags/constants
// from kernel arguments (DynCfg); rt0_kernels.hip dispatches between them.
#include "rt0_integrator.h"

using namespace rt0;

#ifndef RT0_VARIANT
#error "RT0_VARIANT (0..4) selects the instance"
#endif
#if RT0_VARIANT == 0
#define RT0_INST false, false, false, false, false
#elif RT0_VARIANT == 1
#define RT0_INST false, false, true, false, false
#elif RT0_VARIANT == 2
#define RT0_INST false, true, true, true, false
#elif RT0_VARIANT == 3
#define RT0_INST true, true, true, true, false
#else
#define RT0_INST true, true, true, true, true
#endif
#define RT0_CAT2(a, b) a##b
#define RT0_CAT(a, b) RT0_CAT2(a, b)

template <bool RESTIR, bool VOL, bool SDF, bool SPECTRAL, bool COUNT>
__global__ __launch_bounds__(256) void rt0_pass_kernel(const LaunchParams P) {
  pass_body<DynScene, DynCfg, RESTIR, VOL, SDF, SPECTRAL, COUNT>(P, DynScene{P.scene}, DynCfg(P));
}

extern "C" hipError_t RT0_CAT(rt0_launch_pass_v, RT0_VARIANT)(const LaunchParams *p, dim3 grid, hipStream_t stream) {
  hipLaunchKernelGGL((rt0_pass_kernel<RT0_INST>), grid, dim3(256), 0, stream, *p);
  return hipGetLastError();
}
