// rt0_jit.h -- scene-specialising run-time compilation (see rt0_jit.cpp).
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/rt0.h"

#include "rt0_device.h"

namespace rt0h {

// Everything the generated kernel bakes in besides the scene itself.
struct JitKey {
  uint32_t flags;
  int max_bounces, max_diff, max_spec, max_trans, max_scatter, marching_steps, restir_samples;
  float fudge;
  bool restir, vol, sdf, spectral;
  int bvh_stack = 0;  // LDS traversal stack entries (push bound + 1) when the scene has models
  int halo_check = 1;  // RT0_HALO_CHECK: sharded launches count reservoir fetches outside the halo
  int defer = 0;       // RT0_DEFER_NEE: ReSTIR light sampling in its own kernel (rt0_jit_nee + rt0_jit_resolve)
  int nee_regions = 2;  // RT0_NEE_REGIONS: pass-wave record regions per light-sampling wave
  int walk = 0;         // RT0_NEE_WALK: the light-sampling calls' triangle occlusion queries in rt0_jit_walk
  int fused = 0;        // RT0_FUSED_RESOLVE: rt0_jit_nee completes the samples (deferred keys without walk)
  int stack16 = 0;      // RT0_BVH_STACK16: every BVH node index fits 16 + 64 / RT0_BVH_STACK bits
  int wf = 0;           // RT0_WAVEFRONT: passes as wavefront rounds (rt0_jit_wf_shade + rt0_jit_wf_march / _walk)
};

// The kernels of one compiled module: the pass kernel and, for a deferred
// ReSTIR key, the light-sampling and resolve kernels (hipFunction_t each).
struct JitFns {
  void *pass = nullptr, *nee = nullptr, *resolve = nullptr;
  void *walk = nullptr;  // RT0_NEE_WALK keys
  // RT0_WAVEFRONT keys (no pass kernel then); wf_march is the round's
  // traversal kernel: the SDF march, or for ReSTIR keys the closest-hit walk
  void *wf_shade = nullptr, *wf_march = nullptr, *wf_plan = nullptr;
  int wf_march_blocks = 0;  // workgroups of the march kernel the device holds at once
};

std::string jit_source(const SceneDev &s, const JitKey &k);
int jit_stack_entries(const JitKey &k);  // RT0_BVH_STACK of the module (bvh_stack rounded up to 8)
int jit_compile(const std::string &src, std::vector<char> &code, std::string &err);
// runtime feature flags (F_*) of a config, and the JIT key of (config, scene)
uint32_t flags_from_config(const rt0_config &c);
JitKey make_jit_key(const rt0_config &c, int n_sdfs);
// flatten validated mesh records into the device scene layout
SceneDev make_scene_dev(const rt0_mesh *m, int ne, int ns, int nm, const int32_t *li, int nl);
// Compile (or fetch from the process cache) the kernel for this scene/config on
// `device`.
int jit_get(const SceneDev &s, const JitKey &k, int device, JitFns *fns, std::string &err);
int jit_launch(void *fn, const LaunchParams *p, unsigned gx, unsigned gy, unsigned gz, void *stream,
               unsigned block = 256);

}  // namespace rt0h
