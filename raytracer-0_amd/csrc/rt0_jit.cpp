// rt0_jit.cpp -- scene-specialising run-time compilation (hipRTC, gfx950).
//
// The reference compiles its integrator per scene: the scene and the flags are
// spliced into the shader text (tools.js:22-61) and the program is rebuilt on
// every change (index.html:1167-1196).  This is the MI355X counterpart: the
// integrator source (rt0_device.h + rt0_integrator.h, embedded into librt0.so
// at build time) is compiled with hipRTC together with a generated scene
// struct whose geometry, materials and light list are compile-time constants
// and a config struct whose defines/constants are constexpr.  The mesh loops
// then unroll with constant indices, every type dispatch and feature test
// folds, and the scene never costs a memory load.  Camera and frame stay
// kernel arguments (they are per-pass uniforms in the reference).
//
// Compiled modules are cached per (source hash, device) for the process.
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <sstream>
#include <string>
#include <vector>

#include <dlfcn.h>
#include <link.h>
#include <unistd.h>

extern char **environ;

#include "../../include/rt0.h"
#include "rt0_device.h"
#include "rt0_jit.h"

extern "C" const char rt0_jit_source_text[];  // generated: rt0_device.h + rt0_integrator.h

namespace rt0h {

static std::string fl(float v) {
  char b[64];
  snprintf(b, sizeof b, "%.9ef", v);
  return b;
}

static std::string strip_includes(const char *src) {
  std::istringstream is(src);
  std::string line, out;
  while (std::getline(is, line)) {
    size_t p = line.find_first_not_of(" \t");
    if (p != std::string::npos && line.compare(p, 8, "#include") == 0) continue;
    if (p != std::string::npos && line.compare(p, 12, "#pragma once") == 0) continue;
    out += line;
    out += '\n';
  }
  return out;
}

int jit_stack_entries(const JitKey &k) { return ((k.bvh_stack + 7) / 8) * 8; }

std::string jit_source(const SceneDev &s, const JitKey &k) {
  std::ostringstream o;
  if (const char *x = getenv("RT0_JIT_EXTRA")) o << "// options: " << x << "\n";  // part of the cache key
  o << "#define RT0_JIT 1\n";
  // the LDS traversal stack sized to this tree (depth + 1 entries, rounded up to
  // 8) instead of the ahead-of-time kernels' 48: 48 x 256 lanes x 4 B = 48 KiB
  // per workgroup would cap a CU at three workgroups
  if (k.bvh_stack > 0) o << "#define RT0_BVH_STACK " << jit_stack_entries(k) << "\n";
  o << "#define RT0_HALO_CHECK " << k.halo_check << "\n";
  if (k.defer) o << "#define RT0_DEFER_NEE 1\n#define RT0_NEE_REGIONS " << k.nee_regions << "\n";
  if (k.defer && k.walk) o << "#define RT0_NEE_WALK 1\n";
  if (k.defer && !k.walk && k.fused) o << "#define RT0_FUSED_RESOLVE 1\n";
  if (k.bvh_stack > 0 && k.stack16) o << "#define RT0_BVH_STACK16 1\n";
  // the tree's top levels in LDS (rt0_integrator.h bvh_fetch; rt0_host.cpp kTreeletNodes)
  if (k.bvh_stack > 0) o << "#ifndef RT0_TREELET\n#define RT0_TREELET 64\n#endif\n";
  if (k.wf) o << "#define RT0_WAVEFRONT 1\n";
  // ReSTIR light sampling fetches its reservoir taps two at a time
  // (rt0_integrator.h RT0_TAP_BATCH; C3 0.600 vs 0.652 ms per pass at the
  // occupancy target below) unless the kernel also walks the BVH, where the
  // extra registers cost more than the halved round trips save (C5 22.95 vs
  // 18.39 ms, inline light sampling); with the walks in their own kernel C5's
  // light-sampling kernel takes the batch at 3 waves per SIMD (2 150-2 158 vs
  // 2 136-2 141 Msamples/s, profiles/r06/c5_tap_batch)
  if (k.restir && (s.n_models == 0 || k.walk)) o << "#ifndef RT0_TAP_BATCH\n#define RT0_TAP_BATCH 2\n#endif\n";
  o << "using __hip_internal::int32_t; using __hip_internal::uint16_t; using __hip_internal::uint32_t; using __hip_internal::uint64_t;\n";
  // the embedded device source only: profiling probes build their own
  // library from a patched copy (scripts/probes.sh), none is read at run time
  o << strip_includes(rt0_jit_source_text);
  const int nt = s.n_total;
  o << "namespace rt0 {\n";
  o << "__constant__ const GeomRec kJitGeom[" << (nt > 0 ? nt : 1) << "] = {";
  for (int i = 0; i < nt; i++) {
    const GeomRec &g = s.geom[i];
    o << "{" << fl(g.px) << "," << fl(g.py) << "," << fl(g.pz) << "," << fl(g.j0) << "," << g.type << "," << fl(g.d0)
      << "," << fl(g.j1) << "," << fl(g.j2) << "},";
  }
  o << "};\n__constant__ const MatRec kJitMat[" << (nt > 0 ? nt : 1) << "] = {";
  for (int i = 0; i < nt; i++) {
    const MatRec &m = s.mat[i];
    o << "{" << fl(m.cr) << "," << fl(m.cg) << "," << fl(m.cb) << "," << m.type << "," << fl(m.er) << "," << fl(m.eg)
      << "," << fl(m.eb) << "," << fl(m.nt) << "},";
  }
  // the same records with max(c, 0.001) and max(e, 0.001) applied
  // (raytracer.glsl:2071, 2077): what the bounce step reads when no mesh has
  // a texture, so the clamps cost no instructions per hit (JitScene::mat_shade)
  o << "};\n__constant__ const MatRec kJitMatS[" << (nt > 0 ? nt : 1) << "] = {";
  for (int i = 0; i < nt; i++) {
    const MatRec &m = s.mat[i];
    auto c = [](float v) { return fl(std::max(v, 0.001f)); };
    o << "{" << c(m.cr) << "," << c(m.cg) << "," << c(m.cb) << "," << m.type << "," << c(m.er) << "," << c(m.eg)
      << "," << c(m.eb) << "," << fl(m.nt) << "},";
  }
  o << "};\n__constant__ const TexRec kJitTex[" << (nt > 0 ? nt : 1) << "] = {";
  for (int i = 0; i < nt; i++) {
    const TexRec &t = s.tex[i];
    o << "{" << fl(t.cmr) << "," << fl(t.cmg) << "," << fl(t.cmb) << "," << t.type << "," << fl(t.emr) << ","
      << fl(t.emg) << "," << fl(t.emb) << "," << t.opts << "u," << fl(t.p0) << "," << fl(t.p1) << "," << fl(t.p2)
      << "," << fl(t.p3) << "},";
  }
  o << "};\n__constant__ const float kJitJ3[" << (nt > 0 ? nt : 1) << "] = {";
  for (int i = 0; i < nt; i++) o << fl(s.j3[i]) << ",";
  o << "};\n__constant__ const int kJitSdfKind[" << (nt > 0 ? nt : 1) << "] = {";
  for (int i = 0; i < nt; i++) o << s.sdf_kind[i] << ",";
  o << "};\n__constant__ const int kJitLights[" << (s.n_lights > 0 ? s.n_lights : 1) << "] = {";
  for (int i = 0; i < s.n_lights; i++) o << s.light_index[i] << ",";
  if (s.n_lights == 0) o << "-1";
  o << "};\n";
  o << "struct JitScene {\n"
       "  static constexpr bool kStatic = true;\n"
       "  static constexpr int kMeshes = "
    << s.n_meshes << ", kSdfs = " << s.n_sdfs << ", kLights = " << s.n_lights << ", kModels = " << s.n_models
    << ";\n"
       "  static constexpr bool kMayHaveModels = kModels > 0;\n"
       "  __device__ static constexpr int n_meshes() { return kMeshes; }\n"
       "  __device__ static constexpr int n_sdfs() { return kSdfs; }\n"
       "  __device__ static constexpr int n_models() { return kModels; }\n"
       "  __device__ static constexpr int n_lights() { return kLights; }\n"
       "  __device__ static GeomRec geom(int i) { return kJitGeom[i]; }\n"
       "  __device__ static MatRec mat(int i) { return kJitMat[i]; }\n"
       "  __device__ static MatRec mat_shade(int i) { return kJitMatS[i]; }\n"
       "  __device__ static float j3(int i) { return kJitJ3[i]; }\n"
       "  __device__ static int sdf_kind(int i) { return kJitSdfKind[i]; }\n"
       "  __device__ static int light(int i) { return kJitLights[i]; }\n"
    << "  __device__ static TexRec tex(int i) { return kJitTex[i]; }\n"
       "  __device__ static constexpr bool any_tex() { return "
    << (s.any_tex ? "true" : "false") << "; }\n"
       "};\n";
  o << "struct JitCfg {\n"
       "  __device__ static constexpr uint32_t flags() { return "
    << k.flags << "u; }\n  __device__ static constexpr int max_bounces() { return " << k.max_bounces
    << "; }\n  __device__ static constexpr int max_diff() { return " << k.max_diff
    << "; }\n  __device__ static constexpr int max_spec() { return " << k.max_spec
    << "; }\n  __device__ static constexpr int max_trans() { return " << k.max_trans
    << "; }\n  __device__ static constexpr int max_scatter() { return " << k.max_scatter
    << "; }\n  __device__ static constexpr int marching_steps() { return " << k.marching_steps
    << "; }\n  __device__ static constexpr int restir_samples() { return " << k.restir_samples
    << "; }\n  __device__ static constexpr float fudge() { return " << fl(k.fudge) << "; }\n};\n";
  o << "}  // namespace rt0\n";
  const char *rt = k.restir ? "true" : "false", *vol = k.vol ? "true" : "false", *sdf = k.sdf ? "true" : "false",
             *spc = k.spectral ? "true" : "false";
  o << "extern \"C\" __global__ __launch_bounds__(256) ";
  // occupancy targets measured per kernel family (scripts/ab_configs.sh, ab_c5.sh,
  // gpu_ab_taps.sh): BVH traversal is load-latency bound -- C5 4096^2 129.9 ms
  // (3 waves/SIMD: 131 VGPRs and a 48-entry LDS stack) -> 78.3 ms at 6; the
  // ReSTIR kernel with batched taps at 4 (128 VGPRs; at 5 it spills: C3 0.85
  // ms per pass, at 3 0.65, at 4 0.60); the quadric/SDF kernels already sit at
  // <= 64 VGPRs (8 waves) and are left alone.  A deferred ReSTIR pass kernel
  // holds no reservoir code and is left to the compiler unless it walks a BVH;
  // its light-sampling kernel takes the ReSTIR targets.
  // (occupancy targets re-measured in rounds 4 and 5: DESIGN 4.13)
  if (k.wf && k.restir)  // (the wavefront ReSTIR shade kernel walks no BVH: left to the compiler)
    ;
  else if (s.n_models > 0)  // with 16-bit stack entries the LDS allows 8: C5 9.14 vs 9.38 ms per pass at 6
    o << "\n#ifndef RT0_BVH_WAVES\n#define RT0_BVH_WAVES " << (k.stack16 && k.bvh_stack > 0 ? 8 : 6)
      << "\n#endif\n__attribute__((amdgpu_waves_per_eu(RT0_BVH_WAVES))) ";
  else if (k.restir && !k.defer)
    o << "__attribute__((amdgpu_waves_per_eu(4))) ";
  if (k.wf) {
    // wavefront rounds, no pass kernel: SDF scenes (rt0_integrator.h
    // wf_shade_body + wf_march_body) or ReSTIR scenes with triangle models
    // (wf_restir_shade_body + wf_walk_body, then the deferred-pass kernels below)
    // (the SDF shade kernel's occupancy: RT0_WF_SHADE_WAVES through RT0_JIT_EXTRA, an A/B handle)
    if (!k.restir)
      o << "\n#ifdef RT0_WF_SHADE_WAVES\n__attribute__((amdgpu_waves_per_eu(RT0_WF_SHADE_WAVES)))\n#endif\n";
    o << "void rt0_jit_wf_shade(const LaunchParams P) {\n"
      << (k.restir ? "  rt0::wf_restir_shade_body<rt0::JitScene, rt0::JitCfg, " : "  rt0::wf_shade_body<rt0::JitScene, rt0::JitCfg, ")
      << vol << ", " << spc << ">(P, rt0::JitScene{}, rt0::JitCfg{});\n}\n";
    o << "extern \"C\" __global__ __launch_bounds__(256) void rt0_jit_wf_plan(const LaunchParams P) { "
         "rt0::wf_plan_body(P); }\n";
    o << "extern \"C\" __global__ __launch_bounds__(256) ";
    if (k.restir)
      o << "void rt0_jit_wf_walk(const LaunchParams P) { rt0::wf_walk_body(P); }\n";
    else
      o << "void rt0_jit_wf_march(const LaunchParams P) {\n"
           "  rt0::wf_march_body<rt0::JitScene, rt0::JitCfg>(P, rt0::JitScene{}, rt0::JitCfg{});\n}\n";
    if (!k.restir) return o.str();
  } else {
    o << "void rt0_jit_pass(const LaunchParams P) {\n"
         "  rt0::pass_body<rt0::JitScene, rt0::JitCfg, "
      << rt << ", " << vol << ", " << sdf << ", " << spc << ", false>(P, rt0::JitScene{}, rt0::JitCfg{});\n}\n";
  }
  if (k.defer) {
    o << "extern \"C\" __global__ __launch_bounds__(256) ";
    // (RT0_NEE_WAVES through RT0_JIT_EXTRA: an A/B handle)
    // 6: it walks the BVH itself; 3: batched taps beside the walk kernel's scenes' larger light loops
    o << "\n#ifndef RT0_NEE_WAVES\n#define RT0_NEE_WAVES " << (s.n_models > 0 ? (k.walk ? 3 : 6) : 4)
      << "\n#endif\n__attribute__((amdgpu_waves_per_eu(RT0_NEE_WAVES))) ";
    o << "void rt0_jit_nee(const LaunchParams P) {\n"
         "  rt0::nee_body<rt0::JitScene, rt0::JitCfg, "
      << vol << ", " << sdf << ", " << spc << ">(P, rt0::JitScene{}, rt0::JitCfg{});\n}\n";
    if (k.walk || !k.fused)
      o << "extern \"C\" __global__ __launch_bounds__(256) void rt0_jit_resolve(const LaunchParams P) {\n"
           "  rt0::resolve_body<rt0::JitScene, rt0::JitCfg, "
        << spc << ">(P, rt0::JitScene{}, rt0::JitCfg{});\n}\n";
    if (k.walk)
      o << "extern \"C\" __global__ __launch_bounds__(256) void rt0_jit_walk(const LaunchParams P) { rt0::walk_body(P); }\n";
  }
  return o.str();
}

struct CacheEntry {
  hipModule_t mod = nullptr;
  JitFns fns;
};
static std::mutex g_mu;
static std::map<std::pair<uint64_t, int>, CacheEntry> g_cache;

static uint64_t fnv1a(const std::string &s) {
  uint64_t h = 1469598103934665603ull;
  for (unsigned char c : s) h = (h ^ c) * 1099511628211ull;
  return h;
}

// Debugging aid: RT0_JIT_DUMP=<prefix> keeps every generated source and code
// object as <prefix>_<source hash>_<pid><ext>.
static void dump_artifact(const std::string &src, const char *ext, const void *data, size_t n) {
  const char *dump = getenv("RT0_JIT_DUMP");
  if (!dump) return;
  char name[512];
  snprintf(name, sizeof name, "%s_%016llx_%d%s", dump, (unsigned long long)fnv1a(src), (int)getpid(), ext);
  if (FILE *f = fopen(name, "wb")) {
    fwrite(data, 1, n, f);
    fclose(f);
  }
}

// The compiler is pinned: hipRTC is loaded from the ROCm install librt0 was
// built against ($ROCM_PATH or /opt/rocm; RT0_HIPRTC overrides the path) into
// a private link namespace (dlmopen).  A process that imported PyTorch first
// already has torch's bundled, older libhiprtc.so.7 under the same soname;
// binding to that one would make the generated code -- and so the last bits of
// every pixel -- depend on import order.  The private namespace keeps one
// compiler (and one answer) for every host: Python with or without torch, node.
struct Rtc {
  decltype(&hiprtcCreateProgram) create = nullptr;
  decltype(&hiprtcCompileProgram) compile = nullptr;
  decltype(&hiprtcGetProgramLogSize) log_size = nullptr;
  decltype(&hiprtcGetProgramLog) log = nullptr;
  decltype(&hiprtcGetCodeSize) code_size = nullptr;
  decltype(&hiprtcGetCode) get_code = nullptr;
  decltype(&hiprtcDestroyProgram) destroy = nullptr;
  // `environ` of the private namespace's own libc copy: it was set from the
  // process environment when the namespace was created, and a later
  // setenv()/putenv() in the process (Python's os.environ, node's
  // process.env) may free that array -- hipRTC's getenv() calls then read
  // freed memory (the crash of the round-3 test run, in hiprtcCreateProgram).
  // jit_compile points it at the process's current environment first.
  char ***ns_environ = nullptr;
  std::string path, error;
};

static const Rtc &rtc() {
  static Rtc r;
  static std::once_flag once;
  std::call_once(once, [] {
    if (const char *p = getenv("RT0_HIPRTC")) r.path = p;
    else r.path = std::string(getenv("ROCM_PATH") ? getenv("ROCM_PATH") : "/opt/rocm") + "/lib/libhiprtc.so.7";
    void *h = dlmopen(LM_ID_NEWLM, r.path.c_str(), RTLD_NOW | RTLD_LOCAL);
    if (!h) {
      const char *e = dlerror();
      r.error = "cannot load hipRTC from " + r.path + ": " + (e ? e : "?");
      return;
    }
    r.create = (decltype(r.create))dlsym(h, "hiprtcCreateProgram");
    r.compile = (decltype(r.compile))dlsym(h, "hiprtcCompileProgram");
    r.log_size = (decltype(r.log_size))dlsym(h, "hiprtcGetProgramLogSize");
    r.log = (decltype(r.log))dlsym(h, "hiprtcGetProgramLog");
    r.code_size = (decltype(r.code_size))dlsym(h, "hiprtcGetCodeSize");
    r.get_code = (decltype(r.get_code))dlsym(h, "hiprtcGetCode");
    r.destroy = (decltype(r.destroy))dlsym(h, "hiprtcDestroyProgram");
    r.ns_environ = (char ***)dlsym(h, "environ");  // found in the namespace's libc (a dependency of hipRTC)
    if (!r.create || !r.compile || !r.log_size || !r.log || !r.code_size || !r.get_code || !r.destroy)
      r.error = "hipRTC at " + r.path + " lacks an entry point";
  });
  return r;
}

int jit_compile(const std::string &src, std::vector<char> &code, std::string &err) {
  const Rtc &R = rtc();
  if (!R.error.empty()) {
    err = R.error;
    return RT0_E_HIP;
  }
  dump_artifact(src, ".hip", src.data(), src.size());
  if (R.ns_environ && *R.ns_environ != environ) *R.ns_environ = environ;  // (Rtc::ns_environ)
  hiprtcProgram prog;
  if (R.create(&prog, src.c_str(), "rt0_jit.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS) {
    err = "hiprtcCreateProgram failed";
    return RT0_E_HIP;
  }
  // -fno-slp-vectorize: SLP-packed v_pk_*_f32 pairs cost more issue cycles on
  // gfx950 than the scalar ops they replace (measured: +19% samples/s without)
  std::vector<std::string> ov = {"--offload-arch=gfx950", "-O3", "-ffp-contract=fast-honor-pragmas", "-fno-slp-vectorize",
                                 "-std=c++17"};
  if (const char *x = getenv("RT0_JIT_EXTRA")) {  // tuning knob: extra compiler options, ' ' or ',' separated
    std::string e(x);
    for (char &ch : e)
      if (ch == ',') ch = ' ';
    std::istringstream is(e);
    for (std::string w; is >> w;) ov.push_back(w);
  }
  std::vector<const char *> opts;
  for (auto &s : ov) opts.push_back(s.c_str());
  hiprtcResult r = R.compile(prog, (int)opts.size(), opts.data());
  if (r != HIPRTC_SUCCESS) {
    size_t ls = 0;
    R.log_size(prog, &ls);
    std::string log(ls, '\0');
    if (ls) R.log(prog, &log[0]);
    R.destroy(&prog);
    err = "JIT compile failed: " + log.substr(0, 2000);
    return RT0_E_HIP;
  }
  size_t cs = 0;
  R.code_size(prog, &cs);
  code.resize(cs);
  R.get_code(prog, code.data());
  R.destroy(&prog);
  dump_artifact(src, ".co", code.data(), code.size());
  return RT0_OK;
}

int jit_get(const SceneDev &s, const JitKey &k, int device, JitFns *fns, std::string &err) {
  std::string src = jit_source(s, k);
  uint64_t h = fnv1a(src);
  std::lock_guard<std::mutex> lock(g_mu);
  auto it = g_cache.find({h, device});
  if (it != g_cache.end()) {
    *fns = it->second.fns;
    return RT0_OK;
  }
  std::vector<char> code;
  int rc = jit_compile(src, code, err);
  if (rc != RT0_OK) return rc;
  CacheEntry e;
  hipFunction_t f[4] = {};
  bool ok = hipModuleLoadData(&e.mod, code.data()) == hipSuccess;
  if (ok && k.wf) {
    hipFunction_t s = nullptr, m = nullptr, pl = nullptr;
    int per_cu = 0, cus = 0;
    // (the round's traversal kernel: the SDF march, or the ReSTIR scenes' closest-hit walk)
    ok = hipModuleGetFunction(&s, e.mod, "rt0_jit_wf_shade") == hipSuccess &&
         hipModuleGetFunction(&m, e.mod, k.restir ? "rt0_jit_wf_walk" : "rt0_jit_wf_march") == hipSuccess &&
         hipModuleGetFunction(&pl, e.mod, "rt0_jit_wf_plan") == hipSuccess &&
         hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, m, 256, 0) == hipSuccess &&
         hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess;
    e.fns.wf_shade = (void *)s;
    e.fns.wf_march = (void *)m;
    e.fns.wf_plan = (void *)pl;
    e.fns.wf_march_blocks = std::max(1, per_cu) * std::max(1, cus);
  } else if (ok) {
    ok = hipModuleGetFunction(&f[0], e.mod, "rt0_jit_pass") == hipSuccess;
  }
  if (ok && k.defer)
    ok = hipModuleGetFunction(&f[1], e.mod, "rt0_jit_nee") == hipSuccess &&
         (k.fused && !k.walk ? true : hipModuleGetFunction(&f[2], e.mod, "rt0_jit_resolve") == hipSuccess);
  if (ok && k.defer && k.walk)
    ok = hipModuleGetFunction(&f[3], e.mod, "rt0_jit_walk") == hipSuccess;
  if (!ok) {
    err = "hipModuleLoadData/GetFunction failed for the JIT module";
    return RT0_E_HIP;
  }
  e.fns.pass = (void *)f[0];  // (null for a wavefront key)
  e.fns.nee = (void *)f[1];
  e.fns.resolve = (void *)f[2];
  e.fns.walk = (void *)f[3];
  g_cache[{h, device}] = e;
  *fns = e.fns;
  return RT0_OK;
}

int jit_launch(void *fn, const LaunchParams *p, unsigned gx, unsigned gy, unsigned gz, void *stream, unsigned block) {
  void *args[] = {(void *)p};
  hipError_t e = hipModuleLaunchKernel((hipFunction_t)fn, gx, gy, gz, block, 1, 1, 0, (hipStream_t)stream, args, nullptr);
  return e == hipSuccess ? RT0_OK : RT0_E_HIP;
}

}  // namespace rt0h

namespace rt0h {

uint32_t flags_from_config(const rt0_config &g) {
  uint32_t f = 0;
  if (g.defines & RT0_USE_PROCEDURAL_SKY) f |= F_SKY;
  if (g.defines & RT0_USE_BIASED_SAMPLING) f |= F_BIASED;
  if (g.sample_lights) f |= F_SAMPLE_LIGHTS;
  if (g.use_mis) f |= F_MIS;
  if (g.use_restir) f |= F_RESTIR;
  if (g.defines & RT0_USE_RESTIR) f |= F_RESTIR_DEF;
  if (g.defines & RT0_USE_SPECTRAL) f |= F_SPECTRAL;
  if (g.defines & RT0_USE_VOLUMETRICS) f |= F_VOL;
  if (g.defines & RT0_USE_CUBEMAP) f |= F_CUBEMAP;
  if (g.render_mode == 1) f |= F_ANIM;
  return f;
}

JitKey make_jit_key(const rt0_config &g, int n_sdfs) {
  JitKey k;
  k.flags = flags_from_config(g);
  k.max_bounces = g.max_bounces;
  k.max_diff = g.max_diff_bounces;
  k.max_spec = g.max_spec_bounces;
  k.max_trans = g.max_trans_bounces;
  k.max_scatter = g.max_scattering_events;
  k.marching_steps = g.marching_steps;
  k.restir_samples = g.restir_samples;
  k.fudge = g.fudge_factor;
  k.restir = (g.defines & RT0_USE_RESTIR) != 0;
  k.vol = (g.defines & RT0_USE_VOLUMETRICS) != 0;
  k.sdf = n_sdfs > 0;
  k.spectral = (g.defines & RT0_USE_SPECTRAL) != 0;
  return k;
}

SceneDev make_scene_dev(const rt0_mesh *m, int ne, int ns, int nm, const int32_t *li, int nl) {
  SceneDev s;
  memset(&s, 0, sizeof s);
  s.n_meshes = ne;
  s.n_sdfs = ns;
  s.n_models = nm;
  s.n_lights = nl;
  s.n_total = ne + ns + nm;
  for (int i = 0; i < s.n_total; i++) {
    GeomRec &g = s.geom[i];
    g.px = m[i].pos[0];
    g.py = m[i].pos[1];
    g.pz = m[i].pos[2];
    g.j0 = m[i].joker[0];
    g.j1 = m[i].joker[1];
    g.j2 = m[i].joker[2];
    g.type = m[i].type;
    // exact rewrites of the per-test arithmetic (rt0_device.h)
    g.d0 = m[i].type == 0 ? m[i].joker[0] * m[i].joker[0] : m[i].type == 1 ? -m[i].joker[0] : m[i].joker[0] * 0.5f;
    s.j3[i] = m[i].joker[3];
    s.sdf_kind[i] = m[i].sdf_kind;
    MatRec &r = s.mat[i];
    r.cr = m[i].c[0];
    r.cg = m[i].c[1];
    r.cb = m[i].c[2];
    r.er = m[i].e[0];
    r.eg = m[i].e[1];
    r.eb = m[i].e[2];
    r.nt = m[i].nt;
    r.type = m[i].mat_type;
    TexRec &t = s.tex[i];
    t.type = m[i].tex_type;
    t.cmr = m[i].tex_c_mask[0];
    t.cmg = m[i].tex_c_mask[1];
    t.cmb = m[i].tex_c_mask[2];
    t.emr = m[i].tex_e_mask[0];
    t.emg = m[i].tex_e_mask[1];
    t.emb = m[i].tex_e_mask[2];
    t.opts = m[i].mat_opts;
    t.p0 = m[i].tex_params[0];
    t.p1 = m[i].tex_params[1];
    t.p2 = m[i].tex_params[2];
    t.p3 = m[i].tex_params[3];
    if (m[i].tex_type != -1) s.any_tex = 1;
  }
  for (int i = 0; i < nl; i++) s.light_index[i] = li[i];
  return s;
}

}  // namespace rt0h

#include "rt0_internal.h"

extern "C" int rt0_jit_compile(const char *scene_text, const char *const *sdf_meshes, int n_sdf, const rt0_config *cfg,
                               size_t *code_size, char *err, size_t err_len) {
  if (!scene_text || !cfg) return RT0_E_ARG;
  std::vector<rt0_mesh> m;
  std::vector<int32_t> l;
  int ne = 0, ns = 0, nm = 0;
  std::string e;
  int rc = rt0h::parse_scene_glsl(scene_text, sdf_meshes, n_sdf, m, ne, ns, nm, l, e);
  if (rc == RT0_OK) {
    if (ne + ns + nm > RT0_MAX_MESH || (int)l.size() > RT0_MAX_LIGHTS) {
      rc = RT0_E_UNSUPPORTED;
      e = "scene too large";
    }
  }
  std::vector<char> code;
  if (rc == RT0_OK) {
    SceneDev s = rt0h::make_scene_dev(m.data(), ne, ns, nm, l.data(), (int)l.size());
    rt0h::JitKey key = rt0h::make_jit_key(*cfg, ns);
    // the kernels rt0_render launches: deferred light sampling for ReSTIR (rt0_host.cpp)
    const char *d = getenv("RT0_DEFER_NEE");
    key.defer = key.restir && key.max_bounces > 0 && key.max_bounces <= RT0_NEE_MAX_BOUNCES && (!d || atoi(d) != 0);
    // (the host also needs a built BVH; here the scene's TRIANGLE entries decide)
    key.walk = key.defer && nm > 0 && ns == 0 && !s.any_tex && !(key.flags & F_ANIM) ? 1 : 0;
    {  // (rt0_host.cpp fused_resolve)
      const char *fr = getenv("RT0_FUSED_RESOLVE");
      key.fused = key.defer && !key.walk && (!fr || atoi(fr) != 0) ? 1 : 0;
    }
    // (the tree's depth and size are unknown here: RT0_BVH_STACK16=1 and
    // RT0_JIT_STACK=<entries> select what rt0_render would for such a tree)
    // the wavefront rounds rt0_render uses for such a scene (rt0_host.cpp wf_eligible)
    const char *wfe = getenv("RT0_WAVEFRONT");
    const int wf_mode = wfe ? atoi(wfe) : 1;
    bool wf = wf_mode > 0 && key.max_bounces >= 1 && key.max_bounces <= 127;
    if (key.restir) {
      wf = wf && wf_mode >= 2 && key.walk && cfg->render_mode == 0;
    } else {
      wf = wf && ns > 0 && nm == 0 && s.n_lights <= 32;
      for (int i = ne; i < ne + ns; i++) wf = wf && s.mat[i].type != 0;
      for (int i = 0; i < s.n_lights; i++) wf = wf && s.light_index[i] < ne;
    }
    key.wf = wf ? 1 : 0;
    const char *w16 = getenv("RT0_BVH_STACK16"), *st = getenv("RT0_JIT_STACK");
    key.stack16 = w16 && atoi(w16) != 0 ? 1 : 0;
    if (st && nm > 0) key.bvh_stack = atoi(st);
    rc = rt0h::jit_compile(rt0h::jit_source(s, key), code, e);
  }
  if (code_size) *code_size = code.size();
  if (err && err_len) {
    snprintf(err, err_len, "%s", e.c_str());
  }
  return rc;
}
