#!/usr/bin/env python3
"""mask_kat.py -- known-answer shaders that pin how the oracle's executor
(SwiftShader 4.1, run by oracle/gen/glrun.c) masks side effects after `break`.

TEST INFRASTRUCTURE ONLY (build container; needs the kaleido SwiftShader
bundle).  None of these shaders is reference text: they are minimal GLSL ES
3.00 programs with the reference's control-flow shape -- a bounded loop
(radiance(), raytracer.glsl:1994) whose lanes `break` at different iterations,
followed in the same iteration by a call (brdf(), 2094) into a function that
writes a GLOBAL (sampleLightsReSTIR's `g_final_reservoir = final_reservoir`,
1757, read by main() after the loop, 2173-2174).

GLSL ES 3.00 (spec 6.4, "Jumps"): a fragment that executed `break` executes
nothing more of the loop.  What the executor does instead (every case below;
tests/test_oracle_golden.py::test_mask_kat_model re-derives each output from
these rules):
  1. in the iteration in which a lane breaks, the calls after the `break`
     still run for it, and writes to globals inside the callee are not masked
     (break_then_call, global_in_callee_if, nested_break, nested_call);
     writes in the loop body itself are (global_in_loop);
  2. the callee sees its parameters as the lane's PREVIOUS call left them:
     `in` copies and `inout` values after that call (arg_before_break,
     struct_arg, inout_arg); the caller's argument copies are masked;
  3. with no previous call the parameter registers hold another fragment's
     values (the lane of the quad processed before): undefined;
  4. only that one iteration: later iterations are masked (uniform_stop:
     also when every lane of the quad breaks together);
  5. loops inside the callee run for the lane only when the compiler unrolls
     them -- constant trip count <= 4 with no break/continue (callee_loops);
  6. `continue` does not produce the effect (after_continue);
  7. a local array indexed by a loop variable inside a function (map()'s
     `sdf_meshes[i]`, raytracer.glsl:701-709) is read at the index held by
     the FIRST lane of the 2x2 quad (x, y both even): once that lane has
     left the caller's loop, the other three read a stale index -- here
     element 0 (local_array_index).  This is why two-SDF scenes render
     differently with their SDF statements swapped.
The summary (per-pixel outputs of every case) is tests/golden/mask_kat.json.

DEPARTURES (json key "departures"; run with SwiftShader ThreadCount=1, the
executor being thread-count dependent): shaders whose GLSL ES
3.00 result is known in closed form, recorded with it:
  8. a `continue` in a loop whose body has a `break` AFTER it (the reference's
     volumetric bounce loop: continue at raytracer.glsl:2050, breaks at 2057,
     2065, 2089, 2101) retires the lane: continue_then_break renders 1 where
     GLSL semantics give 31, on every pixel; the same loop without the later
     break (continue_no_break) or with the break before the continue
     (break_then_continue) is executed correctly.  How many lanes of the
     reference's own loop the executor retires depends on the generated code
     (in reference-shaped loops it varied with a compile-time constant), so
     the restatement does not model it: volumetric scenes deeper than one
     bounce are darker in the reference than under GLSL semantics
     (c4_mandelbulb_deep: -9% mean radiance; the medium-free
     c4_mandelbulb_deep_novol agrees to 0.1%);
  9. the two-light in-scatter construct (raytracer.glsl:2011-2044 as
     make_shader.js rewrites it, a light loop over the const light_index array
     calling an intersection() with a mesh loop, inside radiance()'s loop with
     lanes breaking at different iterations) is executed correctly
     (inscatter_two_lights): the two-light departure is brdf's light loop
     (rule 11 below), not this one.

QUAD CONTINUE (json key "quad_continue"; 2x2 images, ThreadCount=1): the
reference's bounce loop reduced to its control flow (radiance(),
raytracer.glsl:1994-2102 with intersection(), brdf() and the light loop cut
away -- each cut kept the effect on the reference shader's own quads):
depth-indexed `continue`s from the scatter block (2050, after its
SCATTERING_EVENTS cap `break`, 2049), then a bounce update and the caps
`break` (2100-2101).  Each lane has its own set of iterations that take the
`continue`; the executor's loop-exit histories per lane:
 10. a lane that takes the `continue` in the loop's FIRST iteration is retired
     there unless it is the quad's first lane (x, y even); with that lane not
     covered (a scissor / primitive edge) every lane goes on.  Continues in
     later iterations are honoured.  About a third of these quads never
     finish (HANG, a 30 s limit; which ones depends on the code around the
     loop: the same masks finished in a copy without the KAT header's
     helpers).  (continue_then_break above, a different body, retires lane 0
     too: the rule depends on the code shape, so this case follows the
     reference's.)
QUAD LIGHTS (json key "quad_lights"; 8x8, ThreadCount=1): brdf's light loop
(raytracer.glsl:1955-1974: `for i < light_index.length()` over the const
light index array) called from a bounce loop whose lanes break at different
iterations and skip the call in others (a specular bounce's `continue`);
each lane records, per iteration, 1 + light_index[0] + 4 light_index[1] as
read (10 when both reads are right):
 11. the loop-indexed read uses the index register of the quad's FIRST lane:
     both reads are right exactly when that lane runs the loop in the same
     iteration, live or as the ghost call of the iteration it breaks in
     (rule 1); otherwise both read one stale index.  The stale index depends
     on the code shape: the end of the loop (out of bounds, reads 0: value 1)
     in a loop without `continue` before its break (quad_lights_plain), 0
     (value 6) with a never-taken `continue` there (quad_lights_shape), either
     with a taken one (quad_lights_scatter, the medium's scatter `continue`).
Measured on the reference shader itself (make_golden.py instrument_paths):
this rule is one of several departures in its volumetric loop -- others make
a lane repeat depth 0, and about a third of 2x2 quads never finish -- so the
fixture keeps executor path records and marks the lanes that run as GLSL says.

usage: python3 oracle/gen/mask_kat.py [--only quad_lights]
"""
import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
GEN = os.path.join(REPO, "oracle", "_gen", "mask_kat")
GLRUN = os.path.join(REPO, "oracle", "_ref", "glrun")
W = H = 8

HEAD = """#version 300 es
precision highp float;
precision highp int;
uniform vec2 u_resolution;
uniform uint u_frame;
layout(location = 0) out vec4 FragColor;
layout(location = 1) out vec4 ReSTIRData;
layout(location = 2) out vec4 ReSTIRAux;
// lane l of the 2x2 quad q stops at iteration stopOf()
int stopOf(ivec2 p) {
  int lane = (p.x & 1) + 2 * (p.y & 1);
  int quad = ((p.x >> 1) + (p.y >> 1)) & 3;
  return (lane * 3 + quad) % 5;
}
float g0; float g1; float g2; float g3;
"""

# Each body sets g0..g3 (and o0..o3, written to ReSTIRData) and leaves `stop`
# and the loop-local `loc` in scope for the epilogue.
EPILOGUE = """
  FragColor = vec4(g0, g1, g2, g3);
  ReSTIRData = vec4(o0, o1, o2, o3);
  ReSTIRAux = vec4(float(stop), 0.0, 0.0, 0.0);
}
"""

CASES = {
    # 1: global written by a callee after the break test; loop-body counter
    "break_then_call": """
void touch(float v) { g0 = v; g1 += 1.0; }
void main() {
  g0 = -1.0; g1 = 0.0; g2 = 0.0; g3 = 0.0;
  int stop = stopOf(ivec2(gl_FragCoord.xy));
  float loc = 0.0;
  for (int i = 0; i < 6; ++i) {
    if (i == stop) break;
    touch(float(i));
    loc += 1.0;
  }
  float o0 = loc, o1 = 0.0, o2 = 0.0, o3 = 0.0;
""",
    # 1: the same writes in the loop body (no call): masked
    "global_in_loop": """
void main() {
  g0 = -1.0; g1 = 0.0; g2 = 0.0; g3 = 0.0;
  int stop = stopOf(ivec2(gl_FragCoord.xy));
  float loc = 0.0;
  for (int i = 0; i < 6; ++i) {
    if (i == stop) break;
    g0 = float(i); g1 += 1.0;
    loc += 1.0;
  }
  float o0 = loc, o1 = 0.0, o2 = 0.0, o3 = 0.0;
""",
    # 1: the callee's write inside an `if` of the callee (brdf's if-chain)
    "global_in_callee_if": """
void touch(float v, bool on) { if (on) { g0 = v; g1 += 1.0; } }
void main() {
  g0 = -1.0; g1 = 0.0; g2 = 0.0; g3 = 0.0;
  int stop = stopOf(ivec2(gl_FragCoord.xy));
  float loc = 0.0;
  for (int i = 0; i < 6; ++i) {
    if (i == stop) break;
    touch(float(i), gl_FragCoord.x > -1.0);
    loc += 1.0;
  }
  float o0 = loc, o1 = 0.0, o2 = 0.0, o3 = 0.0;
""",
    # 1: break nested one `if` deeper (radiance's break sites sit in ifs)
    "nested_break": """
void touch(float v) { g0 = v; g1 += 1.0; }
void main() {
  g0 = -1.0; g1 = 0.0; g2 = 0.0; g3 = 0.0;
  int stop = stopOf(ivec2(gl_FragCoord.xy));
  float loc = 0.0;
  for (int i = 0; i < 6; ++i) {
    if (i >= stop) {
      if (gl_FragCoord.y > -1.0) break;
    }
    touch(float(i));
    loc += 1.0;
  }
  float o0 = loc, o1 = 0.0, o2 = 0.0, o3 = 0.0;
""",
    # 1+2: a call inside the callee (brdf -> sampleLightsReSTIR)
    "nested_call": """
void inner(float v) { g0 = v; g1 += 1.0; }
void outer(float v, bool b) { float q = v * 2.0; if (b) inner(q); }
void main() {
  g0 = -1.0; g1 = 0.0; g2 = 0.0; g3 = 0.0;
  int stop = stopOf(ivec2(gl_FragCoord.xy));
  float loc = 0.0;
  for (int i = 0; i < 6; ++i) {
    loc = float(i) * 10.0 + 5.0;
    if (i == stop) break;
    outer(loc, true);
  }
  float o0 = loc, o1 = 0.0, o2 = 0.0, o3 = 0.0;
""",
    # 2: the argument is updated BEFORE the break: the callee still sees the
    # previous call's copy
    "arg_before_break": """
void touch(float v) { g0 = v; g1 += 1.0; }
void main() {
  g0 = -1.0; g1 = 0.0; g2 = 0.0; g3 = 0.0;
  int stop = stopOf(ivec2(gl_FragCoord.xy));
  float loc = 0.0;
  for (int i = 0; i < 6; ++i) {
    loc = float(i) * 10.0 + 5.0;
    if (i == stop) break;
    touch(loc);
  }
  float o0 = loc, o1 = 0.0, o2 = 0.0, o3 = 0.0;
""",
    # 2: a struct argument (brdf's `in Hit hit`)
    "struct_arg": """
struct S { vec3 p; int k; };
void touch(S s) { g0 = s.p.x + float(s.k); g1 += 1.0; }
void main() {
  g0 = -1.0; g1 = 0.0; g2 = 0.0; g3 = 0.0;
  int stop = stopOf(ivec2(gl_FragCoord.xy));
  S s = S(vec3(0.0), 0);
  float loc = 0.0;
  for (int i = 0; i < 6; ++i) {
    s.p = vec3(float(i) * 10.0 + 5.0); s.k = 100 * i;
    if (i == stop) break;
    touch(s);
  }
  loc = s.p.x;
  float o0 = loc, o1 = 0.0, o2 = 0.0, o3 = 0.0;
""",
    # 2: an `inout` argument (brdf's r/mask/acc/bounceIsSpecular) and an `in`
    "inout_arg": """
void touch(inout float v, float w) { g0 = v + 1000.0 * w; g1 += 1.0; v += 0.5; }
void main() {
  g0 = -1.0; g1 = 0.0; g2 = 0.0; g3 = 0.0;
  int stop = stopOf(ivec2(gl_FragCoord.xy));
  float loc = 0.0; float w = 0.0;
  for (int i = 0; i < 6; ++i) {
    loc = float(i) * 10.0 + 5.0;
    if (i == stop) break;
    w = float(i);
    touch(loc, w);
  }
  float o0 = loc, o1 = 0.0, o2 = 0.0, o3 = 0.0;
""",
    # 4: all four lanes of a quad break in the same iteration
    "uniform_stop": """
void touch(float v) { g0 = v; g1 += 1.0; }
void main() {
  g0 = -1.0; g1 = 0.0; g2 = 0.0; g3 = 0.0;
  int stop = 2 + ((int(gl_FragCoord.x) >> 2) & 1);
  float loc = 0.0;
  for (int i = 0; i < 6; ++i) {
    loc = float(i) * 10.0 + 5.0;
    if (i == stop) break;
    touch(loc);
  }
  float o0 = loc, o1 = 0.0, o2 = 0.0, o3 = 0.0;
""",
    # 5: loops inside the callee: trip counts 2, 3, 4, 5, 9, 16 and 2 with
    # continue / break; a loop bounded by a local (sampleLightsReSTIR's
    # candidate and spatial loops)
    "callee_loops": """
const int NC = 9;
float o0; float o1; float o2; float o3;
void work(float v) {
  for (int i = 0; i < 2; ++i) g0 += 1.0;
  for (int i = 0; i < 3; ++i) g1 += 1.0;
  for (int i = 0; i < 4; ++i) g2 += 1.0;
  for (int i = 0; i < 5; ++i) g3 += 1.0;
  for (int i = 0; i < NC; ++i) o0 += 1.0;
  for (int i = 0; i < 2; ++i) { if (v < -100.0) continue; o1 += 1.0; }
  for (int i = 0; i < 2; ++i) { if (v < -100.0) break; o2 += 1.0; }
  int n = int(v) + 3;
  for (int i = 0; i < n; ++i) o3 += 1.0;
}
void main() {
  g0 = 0.0; g1 = 0.0; g2 = 0.0; g3 = 0.0; o0 = 0.0; o1 = 0.0; o2 = 0.0; o3 = 0.0;
  int stop = stopOf(ivec2(gl_FragCoord.xy));
  float loc = 0.0;
  for (int i = 0; i < 6; ++i) {
    loc = 0.0;
    if (i == stop) break;
    work(loc);
  }
""",
    # 7: a callee's local array indexed by its loop variable (map()'s
    # sdf_meshes[i] min-combine) while quad-mates have left the caller's loop;
    # per-iteration results in g0..g3, o0..o1
    "local_array_index": """
float f(float v) {
  float arr[2];
  arr[0] = v;
  arr[1] = 0.5 * v;
  float r = arr[0];
  for (int i = 1; i < 2; ++i) r = mix(arr[i], r, float(r < arr[i]));
  return r;
}
void main() {
  int stop = stopOf(ivec2(gl_FragCoord.xy));
  float acc[6];
  for (int k = 0; k < 6; ++k) acc[k] = -1.0;
  for (int i = 0; i < 6; ++i) {
    acc[i] = f(float(i + 1) * 10.0 + gl_FragCoord.x);
    if (i == stop) break;
  }
  g0 = acc[0]; g1 = acc[1]; g2 = acc[2]; g3 = acc[3];
  float o0 = acc[4], o1 = acc[5], o2 = 0.0, o3 = 0.0;
""",
    # 6: continue instead of break
    "after_continue": """
void touch(float v) { g0 = v; g1 += 1.0; }
void main() {
  g0 = -1.0; g1 = 0.0; g2 = 0.0; g3 = 0.0;
  int stop = stopOf(ivec2(gl_FragCoord.xy));
  float loc = 0.0;
  for (int i = 0; i < 6; ++i) {
    if (i == stop) continue;
    touch(float(i));
    loc += 1.0;
  }
  float o0 = loc, o1 = 0.0, o2 = 0.0, o3 = 0.0;
""",
}


# rule 8/9 cases: name -> (body, GLSL ES 3.00 value of o0 per pixel (x, y))
LOOP_FN = """
float f() {
  float acc = 0.0;
  for (int d = 0; d < 5; ++d) {
    int code = d == 0 ? 0 : ((d == 4) ? 3 : 1);
    %s
  }
  return acc;
}
void main() {
  g0 = 0.0; g1 = 0.0; g2 = 0.0; g3 = 0.0;
  int stop = 0;
  float loc = f();
  float o0 = loc, o1 = 0.0, o2 = 0.0, o3 = 0.0;
"""
INSCATTER = """
struct Hit2 { int index; float t; };
struct M { vec3 pos; float r; int t; };
M meshes[3];
const lowp int LIDX[2] = int[](1, 2);
float isect(vec3 o, vec3 d, out Hit2 h) {
  h.index = 0; float tmin = 1e4;
  for (int i = 0; i < 3; i++) {
    vec3 oc = o - meshes[i].pos; float b = dot(oc, d); float c = dot(oc, oc) - meshes[i].r * meshes[i].r;
    float disc = b * b - c;
    if (disc < 0.0) continue;
    float t = -b - sqrt(disc);
    if (t > 0.001 && t < tmin) { tmin = t; h.index = i; }
  }
  return tmin;
}
float radiance(vec3 p, int stop) {
  float loc = 0.0;
  for (int d = 0; d < 6; ++d) {
    if (d == stop) break;
    int num = int(LIDX.length());
    for (int li = 0; li < num; ++li) {
      int light_idx = int(LIDX[li]);
      if (!(light_idx < 0)) {
        M lm = meshes[light_idx];
        if (!(lm.t != 0)) {
          vec3 dir = normalize(lm.pos - p);
          Hit2 sh;
          float ts = isect(p, dir, sh);
          if (!(sh.index != light_idx)) { loc += float(light_idx) * (float(d) * 10.0 + 1.0); }
        }
      }
    }
  }
  return loc;
}
void main() {
  meshes[0] = M(vec3(0.0, 0.0, 0.0), 1.0, 1);
  meshes[1] = M(vec3(-3.0, 3.0, 0.0), 0.5, 0);
  meshes[2] = M(vec3(3.0, 3.0, 0.0), 0.5, 0);
  g0 = 0.0; g1 = 0.0; g2 = 0.0; g3 = 0.0;
  int stop = stopOf(ivec2(gl_FragCoord.xy));
  vec3 p = vec3(floor(gl_FragCoord.x) - 3.5, -2.0, floor(gl_FragCoord.y) - 3.5);
  float loc = radiance(p, stop);
  float o0 = loc, o1 = 0.0, o2 = 0.0, o3 = 0.0;
"""


def _inscatter_glsl(x, y):
    """GLSL value of INSCATTER's o0 (float64 geometry: the visibility decisions are far from grazing)."""
    ms = [(np.array([0.0, 0, 0]), 1.0), (np.array([-3.0, 3, 0]), 0.5), (np.array([3.0, 3, 0]), 0.5)]
    p = np.array([x - 3.5, -2.0, y - 3.5])
    lane, quad = (x & 1) + 2 * (y & 1), ((x >> 1) + (y >> 1)) & 3
    stop = (lane * 3 + quad) % 5
    per = 0
    for L in (1, 2):
        d = ms[L][0] - p
        d /= np.linalg.norm(d)
        tmin, idx = 1e4, 0
        for i, (c, r) in enumerate(ms):
            oc = p - c
            b, cc = oc @ d, oc @ oc - r * r
            if b * b - cc < 0:
                continue
            t = -b - np.sqrt(b * b - cc)
            if 0.001 < t < tmin:
                tmin, idx = t, i
        per += L if idx == L else 0
    return float(sum(per * (d * 10 + 1) for d in range(stop)))


DEPARTURES = {
    # rule 8: continue at d = 0, a break later in the body (taken at d = 4): GLSL 1 + 10 + 10 + 10 = 31
    "continue_then_break": (LOOP_FN % "if (code == 0) { acc += 1.0; continue; }\n    if (code == 3) break;\n    acc += 10.0;",
                            lambda x, y: 31.0),
    # controls: no later break (41), the break before the continue (41)
    "continue_no_break": (LOOP_FN % "if (code == 0) { acc += 1.0; continue; }\n    acc += 10.0;", lambda x, y: 41.0),
    "break_then_continue": (LOOP_FN % "if (code == 0) { acc += 1.0; if (acc > 100.0) break; continue; }\n    acc += 10.0;",
                            lambda x, y: 41.0),
    # rule 9: the two-light in-scatter construct
    "inscatter_two_lights": (INSCATTER, _inscatter_glsl),
}


QUAD_LOOP = """
struct Ray { vec3 o; vec3 d; };
struct Hit { vec3 pos; vec3 n; };
lowp int SCATTERING_EVENTS = 0;
lowp int DIFF_BOUNCES = 0;
const lowp int MAX_BOUNCES = 12;
const lowp int MAX_SCATTERING_EVENTS = 12;
float g_it = 0.0; float g_h = 0.0; float g_ev = 0.0;
vec3 radiance(Ray r, float seed) {
  vec3 acc = vec3(0.);
  int lane = (int(gl_FragCoord.x) & 1) + 2 * (int(gl_FragCoord.y) & 1);
  int cm = lane == 0 ? %d : lane == 1 ? %d : lane == 2 ? %d : %d;
  for (int depth = 0; depth < MAX_BOUNCES; ++depth) {
    g_it += 1.0; g_h = g_h * 16.0 + float(depth);
    Hit hit;
    float t = 2.0; hit.pos = r.o + t * r.d; hit.n = vec3(0.0, 1.0, 0.0);
    {
      float scatter_d = ((cm >> depth) & 1) != 0 ? 0.0 : 100.0;
      if (scatter_d < t) {
        r = Ray(r.o + scatter_d * r.d, normalize(r.d + vec3(0.1, 0.2, 0.3)));
        ++SCATTERING_EVENTS;
        if (SCATTERING_EVENTS >= MAX_SCATTERING_EVENTS) { g_ev = g_ev * 8.0 + 6.0; break; }
        g_ev = g_ev * 8.0 + 1.0;
        continue;
      }
    }
    r.o = hit.pos + hit.n * 0.001; r.d = reflect(r.d, hit.n); ++DIFF_BOUNCES;
    if (depth >= 5) { g_ev = g_ev * 8.0 + 5.0; break; }
    g_ev = g_ev * 8.0 + 7.0;
  }
  return acc;
}
void main() {
  vec3 a = radiance(Ray(vec3(0.0), vec3(0.0, 0.0, -1.0)), 0.5);
  FragColor = vec4(a, 0.0);
  ReSTIRData = vec4(g_it, g_ev, float(SCATTERING_EVENTS), float(DIFF_BOUNCES));
  ReSTIRAux = vec4(0.0);
}
"""
QUAD_EV = {1: "S", 5: "T", 6: "X", 7: "."}
# (continue masks of lanes 0..3 over depth, covered lanes as a scissor x y w h or None)
QUAD_CASES = [((cm0, cm1, cm2, cm3), cov)
              for cov in (None, (0, 0, 2, 1), (1, 0, 1, 2), (0, 1, 2, 1))
              for (cm0, cm1, cm2, cm3) in ((1, 1, 1, 1), (3, 1, 0, 0), (1, 3, 2, 0), (0, 1, 1, 1), (2, 2, 6, 5),
                                           (0, 0, 0, 0), (5, 1, 9, 3))]


def quad_glsl(cm):
    """GLSL ES 3.00 exit history of QUAD_LOOP for a lane with continue mask cm."""
    ev = ""
    for d in range(12):
        if (cm >> d) & 1:
            ev += "S"
            continue
        if d >= 5:
            return ev + "T"
        ev += "."
    return ev


def run_quad(cms, cov, cwd):
    frag = os.path.join(GEN, "quad_%s_%s.frag" % ("_".join(map(str, cms)), "all" if cov is None else "_".join(map(str, cov))))
    with open(frag, "w") as f:
        f.write(HEAD + QUAD_LOOP % tuple(cms))
    prefix = frag[:-5]
    cmd = [GLRUN, "--frag", frag, "--w", "2", "--h", "2", "--frames", "1", "--single", "--restir-out", "--out", prefix]
    if cov is not None:
        cmd += ["--scissor"] + [str(v) for v in cov]
    try:
        subprocess.run(cmd, check=True, capture_output=True, text=True, cwd=cwd, timeout=30)
    except subprocess.TimeoutExpired:  # the executor did not finish the quad
        return [{"lane": lane, "covered": None, "exec": "HANG", "glsl": quad_glsl(cms[lane])} for lane in range(4)]
    c = np.fromfile("%s_f1_r.bin" % prefix, dtype=np.float32).reshape(2, 2, 4)[..., 1:]
    out = []
    for lane in range(4):
        x, y = lane & 1, lane >> 1
        covered = cov is None or (cov[0] <= x < cov[0] + cov[2] and cov[1] <= y < cov[1] + cov[3])
        v, ev = int(round(float(c[y, x, 0]))) if covered else 0, ""
        while v:
            ev = QUAD_EV.get(v % 8, "?") + ev
            v //= 8
        out.append({"lane": lane, "covered": covered, "exec": ev if covered else None, "glsl": quad_glsl(cms[lane])})
    return out


QL_TPL = """
const lowp int LIDX[2] = int[](1, 2);
int specOf(ivec2 p) {
  int lane = (p.x & 1) + 2 * (p.y & 1);
  int quad = ((p.x >> 1) + (p.y >> 1)) & 3;
  return (lane * 5 + quad * 3) %% 7;
}
int scatOf(ivec2 p) {
  int lane = (p.x & 1) + 2 * (p.y & 1);
  int quad = ((p.x >> 1) + (p.y >> 1)) & 3;
  return %s;
}
void nee(int d, inout float rec[4]) {
  float v = 1.0;
  for (int i = 0; i < int(LIDX.length()); ++i) {
    int idx = int(LIDX[i]);
    if (idx >= 0) v += float(idx) * (i == 0 ? 1.0 : 4.0);
  }
  rec[d] = v;
}
void main() {
  g0 = 0.0; g1 = 0.0; g2 = 0.0; g3 = 0.0;
  ivec2 p = ivec2(gl_FragCoord.xy);
  int stop = stopOf(p);
  int sm = specOf(p);
  int sc = scatOf(p);
  float rec[4];
  for (int k = 0; k < 4; ++k) rec[k] = 0.0;
  for (int d = 0; d < 4; ++d) {
    %s
    if (d == stop) break;
    if (((sm >> d) & 1) != 0) continue;
    nee(d, rec);
  }
  float o0 = rec[0], o1 = rec[1], o2 = rec[2], o3 = float(sm);
  g0 = rec[3]; g1 = float(sc);
"""
# name -> (scatOf body, the statement before the break)
QL_CASES = {
    "quad_lights_plain": ("0", ""),
    "quad_lights_shape": ("0", "if (u_frame > 1000u) continue;"),
    "quad_lights_scatter": ("((lane * 3 + quad * 5) % 4) << 1", "if (((sc >> d) & 1) != 0) continue;"),
}


def run_case(name, body, cwd=None):
    frag = os.path.join(GEN, name + ".frag")
    with open(frag, "w") as f:
        f.write(HEAD + body + EPILOGUE)
    prefix = os.path.join(GEN, name)
    subprocess.run([GLRUN, "--frag", frag, "--w", str(W), "--h", str(H), "--frames", "1", "--single",
                    "--restir-out", "--out", prefix], check=True, capture_output=True, text=True, cwd=cwd)

    def load(tag):
        return np.fromfile("%s_f1_%s.bin" % (prefix, tag), dtype=np.float32).reshape(H, W, 4)

    g, o, a = load("c"), load("r"), load("a")
    return [{"x": x, "y": y, "stop": int(a[y, x, 0]), "g": [float(v) for v in g[y, x]],
             "o": [float(v) for v in o[y, x]]} for y in range(H) for x in range(W)]


def threads1_dir():
    t1 = os.path.join(GEN, "threads1")
    os.makedirs(t1, exist_ok=True)
    with open(os.path.join(t1, "SwiftShader.ini"), "w") as f:
        f.write("[Processor]\nThreadCount=1\n")
    return t1


def quad_lights(t1):
    out = {}
    for name, (scat, pre) in QL_CASES.items():
        rows = run_case(name, QL_TPL % (scat, pre), cwd=t1)
        out[name] = [{"x": r["x"], "y": r["y"], "stop": r["stop"], "spec": int(r["o"][3]), "scat": int(r["g"][1]),
                      "rec": r["o"][:3] + [r["g"][0]]} for r in rows]
        print(name, [r["rec"] for r in out[name][:4]])
    return out


def main():
    os.makedirs(GEN, exist_ok=True)
    path = os.path.join(REPO, "tests", "golden", "mask_kat.json")
    if sys.argv[1:] == ["--only", "quad_lights"]:  # refresh that section alone (the others take minutes)
        with open(path) as f:
            out = json.load(f)
        out["quad_lights"] = quad_lights(threads1_dir())
        with open(path, "w") as f:
            json.dump(out, f, separators=(",", ":"))
        return
    out = {"_doc": "per-pixel outputs of the known-answer shaders of oracle/gen/mask_kat.py run by the oracle's "
                   "executor (SwiftShader 4.1); g = FragColor (g0..g3), o = ReSTIRData (o0..o3)",
           "width": W, "height": H, "cases": {}}
    for name, body in CASES.items():
        rows = run_case(name, body)
        out["cases"][name] = rows
        print(name)
        for r in rows[:4]:
            print("   x=%d y=%d stop=%d g=%s o=%s" % (r["x"], r["y"], r["stop"], r["g"], r["o"]))
    # departures from GLSL semantics, one executor thread (deterministic)
    t1 = threads1_dir()
    out["departures"] = {}
    for name, (body, glsl) in DEPARTURES.items():
        rows = run_case(name, body, cwd=t1)
        out["departures"][name] = [{"x": r["x"], "y": r["y"], "exec": r["o"][0], "glsl": glsl(r["x"], r["y"])}
                                   for r in rows]
        bad = sum(1 for r in out["departures"][name] if r["exec"] != r["glsl"])
        print("%s: %d of %d pixels depart from GLSL semantics" % (name, bad, len(rows)))
    out["quad_continue"] = []
    for cms, cov in QUAD_CASES:
        rows = run_quad(cms, cov, t1)
        out["quad_continue"].append({"cms": list(cms), "cov": list(cov) if cov else None, "lanes": rows})
        print("quad_continue cms %s cov %s: %s" % (cms, cov, [r["exec"] for r in rows]))
    out["quad_lights"] = quad_lights(t1)
    with open(path, "w") as f:
        json.dump(out, f, separators=(",", ":"))


if __name__ == "__main__":
    main()
