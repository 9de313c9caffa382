/*
 * glrun.c -- headless runner that executes the REFERENCE fragment shader
 * (raytracer-0 shaders/pathtracing/raytracer.glsl, expanded by the
 * reference's own parseShader, tools.js:22-61) on SwiftShader's
 * OpenGL ES 3.0 implementation, on the CPU of THIS container.
 *
 * TEST INFRASTRUCTURE ONLY.  This program is the golden-vector generator for
 * tests/golden/; it never runs on the GPU box and nothing in the product links
 * it.  SwiftShader (libEGL/libGLESv2) is the copy bundled with the `kaleido`
 * Python package in this image; it is dlopen()ed at run time.
 *
 * It replays what GlslViewport.render() does per pass (index.js:986-1105):
 *   - u_frame = ++passes (1-based), u_time, u_resolution, camera uniforms
 *     (index.js:419-423, 1010-1015);
 *   - texture units 0..12 as in index.js:149-163;
 *   - MRT: attachment0 = accumulator, 1/2 = ReSTIR reservoirs (index.js:1041-1044);
 *   - the ReSTIR 4-deep swap chain swapReSTIRBuffers() (index.js:795-820) and
 *     the front/back accumulator swap (index.js:1100-1104).
 * All float textures are RGBA32F, LINEAR, CLAMP_TO_EDGE (index.js:660-664).
 *
 * Modes:
 *   --single : unit 0 is bound to an all-zero texture every pass, so attachment0
 *              holds exactly that pass's sample (raytracer.glsl:2168 with prev=0).
 *   default  : true progressive accumulation through the back buffer.
 * Output per pass k (1-based): <prefix>_f<k>_c.bin (W*H*4 f32, row 0 = bottom row
 * as glReadPixels returns it) and, with --restir-out, _r.bin / _a.bin.
 */
#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef void *EGLDisplay, *EGLConfig, *EGLSurface, *EGLContext;
typedef int32_t EGLint;
typedef unsigned int EGLBoolean;
typedef unsigned int GLenum, GLuint, GLbitfield;
typedef int GLint, GLsizei;
typedef float GLfloat;
typedef char GLchar;
typedef unsigned char GLboolean;
typedef intptr_t GLsizeiptr;

#define EGL_SURFACE_TYPE 0x3033
#define EGL_PBUFFER_BIT 0x0001
#define EGL_RENDERABLE_TYPE 0x3040
#define EGL_OPENGL_ES3_BIT 0x0040
#define EGL_NONE 0x3038
#define EGL_WIDTH 0x3057
#define EGL_HEIGHT 0x3056
#define EGL_CONTEXT_CLIENT_VERSION 0x3098
#define EGL_RED_SIZE 0x3024
#define EGL_GREEN_SIZE 0x3023
#define EGL_BLUE_SIZE 0x3022
#define EGL_ALPHA_SIZE 0x3021

#define GL_FRAGMENT_SHADER 0x8B30
#define GL_VERTEX_SHADER 0x8B31
#define GL_COMPILE_STATUS 0x8B81
#define GL_LINK_STATUS 0x8B82
#define GL_TEXTURE_2D 0x0DE1
#define GL_TEXTURE0 0x84C0
#define GL_TEXTURE_MAG_FILTER 0x2800
#define GL_TEXTURE_MIN_FILTER 0x2801
#define GL_TEXTURE_WRAP_S 0x2802
#define GL_TEXTURE_WRAP_T 0x2803
#define GL_LINEAR 0x2601
#define GL_CLAMP_TO_EDGE 0x812F
#define GL_RGBA 0x1908
#define GL_RGBA32F 0x8814
#define GL_FLOAT 0x1406
#define GL_RGBA8 0x8058
#define GL_RGB 0x1907
#define GL_RGB8 0x8051
#define GL_UNSIGNED_BYTE 0x1401
#define GL_REPEAT 0x2901
#define GL_TEXTURE_CUBE_MAP 0x8513
#define GL_TEXTURE_CUBE_MAP_POSITIVE_X 0x8515
#define GL_UNPACK_ALIGNMENT 0x0CF5
#define GL_FRAMEBUFFER 0x8D40
#define GL_COLOR_ATTACHMENT0 0x8CE0
#define GL_FRAMEBUFFER_COMPLETE 0x8CD5
#define GL_ARRAY_BUFFER 0x8892
#define GL_STATIC_DRAW 0x88E4
#define GL_TRIANGLES 0x0004
#define GL_READ_FRAMEBUFFER 0x8CA8
#define GL_SCISSOR_TEST 0x0C11

#define F(ret, name, args) static ret(*p_##name) args;
F(EGLDisplay, eglGetDisplay, (void *))
F(EGLBoolean, eglInitialize, (EGLDisplay, EGLint *, EGLint *))
F(EGLBoolean, eglChooseConfig, (EGLDisplay, const EGLint *, EGLConfig *, EGLint, EGLint *))
F(EGLSurface, eglCreatePbufferSurface, (EGLDisplay, EGLConfig, const EGLint *))
F(EGLContext, eglCreateContext, (EGLDisplay, EGLConfig, EGLContext, const EGLint *))
F(EGLBoolean, eglMakeCurrent, (EGLDisplay, EGLSurface, EGLSurface, EGLContext))
F(EGLint, eglGetError, (void))
F(GLuint, glCreateShader, (GLenum))
F(void, glShaderSource, (GLuint, GLsizei, const GLchar *const *, const GLint *))
F(void, glCompileShader, (GLuint))
F(void, glGetShaderiv, (GLuint, GLenum, GLint *))
F(void, glGetShaderInfoLog, (GLuint, GLsizei, GLsizei *, GLchar *))
F(GLuint, glCreateProgram, (void))
F(void, glAttachShader, (GLuint, GLuint))
F(void, glBindAttribLocation, (GLuint, GLuint, const GLchar *))
F(void, glLinkProgram, (GLuint))
F(void, glGetProgramiv, (GLuint, GLenum, GLint *))
F(void, glGetProgramInfoLog, (GLuint, GLsizei, GLsizei *, GLchar *))
F(void, glUseProgram, (GLuint))
F(GLint, glGetUniformLocation, (GLuint, const GLchar *))
F(void, glUniform1i, (GLint, GLint))
F(void, glUniform1ui, (GLint, GLuint))
F(void, glUniform1f, (GLint, GLfloat))
F(void, glUniform2f, (GLint, GLfloat, GLfloat))
F(void, glUniform3f, (GLint, GLfloat, GLfloat, GLfloat))
F(void, glGenTextures, (GLsizei, GLuint *))
F(void, glBindTexture, (GLenum, GLuint))
F(void, glActiveTexture, (GLenum))
F(void, glTexParameteri, (GLenum, GLenum, GLint))
F(void, glTexImage2D, (GLenum, GLint, GLint, GLsizei, GLsizei, GLint, GLenum, GLenum, const void *))
F(void, glPixelStorei, (GLenum, GLint))
F(void, glGenFramebuffers, (GLsizei, GLuint *))
F(void, glBindFramebuffer, (GLenum, GLuint))
F(void, glFramebufferTexture2D, (GLenum, GLenum, GLenum, GLuint, GLint))
F(GLenum, glCheckFramebufferStatus, (GLenum))
F(void, glDrawBuffers, (GLsizei, const GLenum *))
F(void, glReadBuffer, (GLenum))
F(void, glGenBuffers, (GLsizei, GLuint *))
F(void, glBindBuffer, (GLenum, GLuint))
F(void, glBufferData, (GLenum, GLsizeiptr, const void *, GLenum))
F(void, glEnableVertexAttribArray, (GLuint))
F(void, glVertexAttribPointer, (GLuint, GLint, GLenum, GLboolean, GLsizei, const void *))
F(void, glViewport, (GLint, GLint, GLsizei, GLsizei))
F(void, glScissor, (GLint, GLint, GLsizei, GLsizei))
F(void, glEnable, (GLenum))
F(void, glDrawArrays, (GLenum, GLint, GLsizei))
F(void, glReadPixels, (GLint, GLint, GLsizei, GLsizei, GLenum, GLenum, void *))
F(void, glFinish, (void))
F(GLenum, glGetError, (void))
#undef F

static const char *SS_DIR =
    "/usr/local/lib/python3.10/dist-packages/kaleido/executable/bin/swiftshader";

static double now_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

static void die(const char *m) {
  fprintf(stderr, "glrun: %s\n", m);
  exit(2);
}

static void load(void) {
  char path[1024];
  const char *dir = getenv("SWIFTSHADER_DIR");
  if (!dir) dir = SS_DIR;
  snprintf(path, sizeof path, "%s/libGLESv2.so", dir);
  void *gles = dlopen(path, RTLD_NOW | RTLD_GLOBAL);
  snprintf(path, sizeof path, "%s/libEGL.so", dir);
  void *egl = dlopen(path, RTLD_NOW | RTLD_GLOBAL);
  if (!gles || !egl) die(dlerror());
#define L(lib, name)                                   \
  p_##name = (__typeof__(p_##name))dlsym(lib, #name); \
  if (!p_##name) die("missing symbol " #name);
  L(egl, eglGetDisplay) L(egl, eglInitialize) L(egl, eglChooseConfig)
  L(egl, eglCreatePbufferSurface) L(egl, eglCreateContext) L(egl, eglMakeCurrent)
  L(egl, eglGetError)
  L(gles, glCreateShader) L(gles, glShaderSource) L(gles, glCompileShader)
  L(gles, glGetShaderiv) L(gles, glGetShaderInfoLog) L(gles, glCreateProgram)
  L(gles, glAttachShader) L(gles, glBindAttribLocation) L(gles, glLinkProgram)
  L(gles, glGetProgramiv) L(gles, glGetProgramInfoLog) L(gles, glUseProgram)
  L(gles, glGetUniformLocation) L(gles, glUniform1i) L(gles, glUniform1ui)
  L(gles, glUniform1f) L(gles, glUniform2f) L(gles, glUniform3f)
  L(gles, glGenTextures) L(gles, glBindTexture) L(gles, glActiveTexture)
  L(gles, glTexParameteri) L(gles, glTexImage2D) L(gles, glGenFramebuffers)
  L(gles, glBindFramebuffer) L(gles, glFramebufferTexture2D)
  L(gles, glCheckFramebufferStatus) L(gles, glDrawBuffers) L(gles, glReadBuffer)
  L(gles, glGenBuffers) L(gles, glBindBuffer) L(gles, glBufferData)
  L(gles, glEnableVertexAttribArray) L(gles, glVertexAttribPointer)
  L(gles, glViewport) L(gles, glScissor) L(gles, glEnable) L(gles, glDrawArrays) L(gles, glReadPixels)
  L(gles, glFinish) L(gles, glGetError) L(gles, glPixelStorei)
#undef L
}

static char *slurp(const char *fn) {
  FILE *f = fopen(fn, "rb");
  if (!f) die("cannot open shader file");
  fseek(f, 0, SEEK_END);
  long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  char *s = (char *)malloc(n + 1);
  if (fread(s, 1, n, f) != (size_t)n) die("short read");
  s[n] = 0;
  fclose(f);
  return s;
}

static GLuint compile(GLenum kind, const char *src) {
  GLuint s = p_glCreateShader(kind);
  p_glShaderSource(s, 1, &src, NULL);
  p_glCompileShader(s);
  GLint ok = 0;
  p_glGetShaderiv(s, GL_COMPILE_STATUS, &ok);
  if (!ok) {
    static char log[1 << 16];
    p_glGetShaderInfoLog(s, sizeof log, NULL, log);
    fprintf(stderr, "shader compile error:\n%s\n", log);
    exit(3);
  }
  return s;
}

static GLuint mktex(int w, int h, const float *data) {
  GLuint t;
  p_glGenTextures(1, &t);
  p_glBindTexture(GL_TEXTURE_2D, t);
  p_glTexParameteri(GL_TEXTURE_2D, GL_TEXTURE_WRAP_S, GL_CLAMP_TO_EDGE);
  p_glTexParameteri(GL_TEXTURE_2D, GL_TEXTURE_WRAP_T, GL_CLAMP_TO_EDGE);
  p_glTexParameteri(GL_TEXTURE_2D, GL_TEXTURE_MAG_FILTER, GL_LINEAR);
  p_glTexParameteri(GL_TEXTURE_2D, GL_TEXTURE_MIN_FILTER, GL_LINEAR);
  p_glTexImage2D(GL_TEXTURE_2D, 0, GL_RGBA32F, w, h, 0, GL_RGBA, GL_FLOAT, data);
  return t;
}

/* An RGBA8 asset texture as GlslViewport.loadTexture creates it (index.js:
 * 703-727): REPEAT, LINEAR mag/min filtering; file = raw w*h*4 bytes, first row
 * = the image's first (top) row, which WebGL uploads to t = 0. */
static unsigned char *slurp_bytes(const char *fn, size_t n) {
  FILE *f = fopen(fn, "rb");
  if (!f) die("cannot open texture file");
  unsigned char *b = (unsigned char *)malloc(n);
  if (fread(b, 1, n, f) != n) die("short texture file");
  fclose(f);
  return b;
}
static GLuint mktex8(int w, int h, const char *fn) {
  unsigned char *b = slurp_bytes(fn, (size_t)w * h * 4);
  GLuint t;
  p_glGenTextures(1, &t);
  p_glBindTexture(GL_TEXTURE_2D, t);
  p_glTexParameteri(GL_TEXTURE_2D, GL_TEXTURE_WRAP_S, GL_REPEAT);
  p_glTexParameteri(GL_TEXTURE_2D, GL_TEXTURE_WRAP_T, GL_REPEAT);
  p_glTexParameteri(GL_TEXTURE_2D, GL_TEXTURE_MAG_FILTER, GL_LINEAR);
  p_glTexParameteri(GL_TEXTURE_2D, GL_TEXTURE_MIN_FILTER, GL_LINEAR);
  p_glTexImage2D(GL_TEXTURE_2D, 0, GL_RGBA8, w, h, 0, GL_RGBA, GL_UNSIGNED_BYTE, b);
  free(b);
  return t;
}
/* The cubemap of index.js:300-331: six RGB8 faces in the reference's target
 * order (-X, -Y, -Z, +X, +Y, +Z), MIN_FILTER LINEAR, default wrap/mag.
 * file = 6 consecutive size*size*3 faces. */
static GLuint mkcube(int size, const char *fn) {
  size_t face = (size_t)size * size * 3;
  unsigned char *b = slurp_bytes(fn, face * 6);
  static const int target_of[6] = {1, 3, 5, 0, 2, 4}; /* -X -Y -Z +X +Y +Z -> GL enum offsets */
  GLuint t;
  p_glGenTextures(1, &t);
  p_glBindTexture(GL_TEXTURE_CUBE_MAP, t);
  p_glPixelStorei(GL_UNPACK_ALIGNMENT, 1);
  for (int i = 0; i < 6; i++)
    p_glTexImage2D(GL_TEXTURE_CUBE_MAP_POSITIVE_X + target_of[i], 0, GL_RGB8, size, size, 0, GL_RGB, GL_UNSIGNED_BYTE,
                   b + face * i);
  p_glTexParameteri(GL_TEXTURE_CUBE_MAP, GL_TEXTURE_MIN_FILTER, GL_LINEAR);
  free(b);
  return t;
}

static void dump(const char *prefix, int frame, const char *tag, int w, int h,
                 GLuint fb, int attachment) {
  size_t n = (size_t)w * h * 4;
  float *px = (float *)malloc(n * sizeof(float));
  p_glBindFramebuffer(GL_READ_FRAMEBUFFER, fb);
  p_glReadBuffer(GL_COLOR_ATTACHMENT0 + attachment);
  p_glReadPixels(0, 0, w, h, GL_RGBA, GL_FLOAT, px);
  char fn[1024];
  snprintf(fn, sizeof fn, "%s_f%d_%s.bin", prefix, frame, tag);
  FILE *f = fopen(fn, "wb");
  if (!f) die("cannot write output");
  fwrite(px, sizeof(float), n, f);
  fclose(f);
  free(px);
}

int main(int argc, char **argv) {
  const char *frag = NULL, *prefix = "out";
  int w = 64, h = 64, frames = 4, frame0 = 1, single = 0, restir_out = 0;
  float cam[9] = {0, 0, 2.8f, 0, 0, -1, 50, 0, 3.5f};
  float time_ms = 0.0f;
  float dtime_ms = 0.0f;
  const char *tex_file[6] = {0};
  int tex_w[6] = {0}, tex_h[6] = {0};
  const char *cube_file = NULL;
  int cube_size = 0;
  int temporal_frames = 5; /* index.js:258 default temporalFrames */
  int sc[4] = {0, 0, 0, 0}; /* --scissor x y w h: only these fragments run (w = 0: all) */
  for (int i = 1; i < argc; i++) {
    if (!strcmp(argv[i], "--frag")) frag = argv[++i];
    else if (!strcmp(argv[i], "--out")) prefix = argv[++i];
    else if (!strcmp(argv[i], "--w")) w = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--h")) h = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--frames")) frames = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--frame0")) frame0 = atoi(argv[++i]); /* u_frame of the first pass */
    else if (!strcmp(argv[i], "--single")) single = 1;
    else if (!strcmp(argv[i], "--restir-out")) restir_out = 1;
    else if (!strcmp(argv[i], "--time")) time_ms = (float)atof(argv[++i]);
    else if (!strcmp(argv[i], "--dtime")) dtime_ms = (float)atof(argv[++i]); /* u_time step per pass */
    else if (!strcmp(argv[i], "--tex")) { /* --tex UNIT(1..5) W H file.rgba8 */
      int u = atoi(argv[++i]);
      if (u < 1 || u > 5) die("--tex unit must be 1..5 (u_tex0..3, u_rnd_tex)");
      tex_w[u] = atoi(argv[++i]);
      tex_h[u] = atoi(argv[++i]);
      tex_file[u] = argv[++i];
    } else if (!strcmp(argv[i], "--cube")) { /* --cube SIZE file.rgb8 */
      cube_size = atoi(argv[++i]);
      cube_file = argv[++i];
    }
    else if (!strcmp(argv[i], "--scissor")) {
      for (int k = 0; k < 4; k++) sc[k] = atoi(argv[++i]);
    }
    else if (!strcmp(argv[i], "--cam")) {
      for (int k = 0; k < 9; k++) cam[k] = (float)atof(argv[++i]);
    } else die("unknown argument");
  }
  if (!frag) die("--frag required");
  load();

  EGLDisplay dpy = p_eglGetDisplay(NULL);
  EGLint maj, min;
  if (!p_eglInitialize(dpy, &maj, &min)) die("eglInitialize failed");
  EGLint cfg_attr[] = {EGL_SURFACE_TYPE, EGL_PBUFFER_BIT, EGL_RENDERABLE_TYPE,
                       EGL_OPENGL_ES3_BIT, EGL_RED_SIZE, 8, EGL_GREEN_SIZE, 8,
                       EGL_BLUE_SIZE, 8, EGL_ALPHA_SIZE, 8, EGL_NONE};
  EGLConfig cfg;
  EGLint ncfg = 0;
  if (!p_eglChooseConfig(dpy, cfg_attr, &cfg, 1, &ncfg) || ncfg < 1) die("eglChooseConfig");
  EGLint pb_attr[] = {EGL_WIDTH, 16, EGL_HEIGHT, 16, EGL_NONE};
  EGLSurface surf = p_eglCreatePbufferSurface(dpy, cfg, pb_attr);
  EGLint ctx_attr[] = {EGL_CONTEXT_CLIENT_VERSION, 3, EGL_NONE};
  EGLContext ctx = p_eglCreateContext(dpy, cfg, NULL, ctx_attr);
  if (!ctx || !p_eglMakeCurrent(dpy, surf, surf, ctx)) die("context creation failed");

  /* full-screen quad, same vertices as index.js:237-240 */
  static const char *vs =
      "#version 300 es\nprecision highp float;\n"
      "layout(location = 0) in vec2 a_position;\n"
      "void main(void){ gl_Position = vec4(a_position, 0.0, 1.0); }\n";
  char *fs = slurp(frag);
  GLuint prog = p_glCreateProgram();
  p_glAttachShader(prog, compile(GL_VERTEX_SHADER, vs));
  p_glAttachShader(prog, compile(GL_FRAGMENT_SHADER, fs));
  p_glLinkProgram(prog);
  GLint ok = 0;
  p_glGetProgramiv(prog, GL_LINK_STATUS, &ok);
  if (!ok) {
    static char log[1 << 16];
    p_glGetProgramInfoLog(prog, sizeof log, NULL, log);
    fprintf(stderr, "link error:\n%s\n", log);
    return 3;
  }
  p_glUseProgram(prog);
  double t0 = now_s();
  fprintf(stderr, "glrun: linked\n");

  GLuint vb;
  static const float quad[12] = {-1, -1, 1, -1, -1, 1, -1, 1, 1, -1, 1, 1};
  p_glGenBuffers(1, &vb);
  p_glBindBuffer(GL_ARRAY_BUFFER, vb);
  p_glBufferData(GL_ARRAY_BUFFER, sizeof quad, quad, GL_STATIC_DRAW);
  p_glEnableVertexAttribArray(0);
  p_glVertexAttribPointer(0, 2, GL_FLOAT, 0, 0, 0);

  float *zeros = (float *)calloc((size_t)w * h * 4, sizeof(float));
  /* textures, named as in index.js */
  GLuint front = mktex(w, h, zeros), back = mktex(w, h, zeros), zero = mktex(w, h, zeros);
  GLuint rbuf = mktex(w, h, zeros), raux = mktex(w, h, zeros);
  GLuint rbuf_back = mktex(w, h, zeros), raux_back = mktex(w, h, zeros);
  GLuint h1 = mktex(w, h, zeros), h1a = mktex(w, h, zeros);
  GLuint h2 = mktex(w, h, zeros), h2a = mktex(w, h, zeros);

  GLuint asset[6] = {0};
  for (int u = 1; u <= 5; u++)
    if (tex_file[u]) asset[u] = mktex8(tex_w[u], tex_h[u], tex_file[u]);
  GLuint cube = cube_file ? mkcube(cube_size, cube_file) : 0;

  GLuint fb;
  p_glGenFramebuffers(1, &fb);
  p_glBindFramebuffer(GL_FRAMEBUFFER, fb);
  GLenum bufs[3] = {GL_COLOR_ATTACHMENT0, GL_COLOR_ATTACHMENT0 + 1, GL_COLOR_ATTACHMENT0 + 2};
  p_glDrawBuffers(3, bufs);

  /* uniforms (index.js:384-440) */
  p_glUniform2f(p_glGetUniformLocation(prog, "u_resolution"), (float)w, (float)h);
  p_glUniform3f(p_glGetUniformLocation(prog, "u_camPos"), cam[0], cam[1], cam[2]);
  p_glUniform3f(p_glGetUniformLocation(prog, "u_camLookAt"), cam[3], cam[4], cam[5]);
  p_glUniform3f(p_glGetUniformLocation(prog, "u_camParams"), cam[6], cam[7], cam[8]);
  static const char *units[13] = {"u_bufferA", "u_tex0", "u_tex1", "u_tex2", "u_tex3",
                                  "u_rnd_tex", "u_cubemap", "u_restir_buffer",
                                  "u_restir_aux", "u_restir_history1",
                                  "u_restir_history1_aux", "u_restir_history2",
                                  "u_restir_history2_aux"};
  for (int u = 0; u < 13; u++) {
    GLint loc = p_glGetUniformLocation(prog, units[u]);
    if (loc >= 0) p_glUniform1i(loc, u);
  }
  GLint frame_loc = p_glGetUniformLocation(prog, "u_frame");
  GLint time_loc = p_glGetUniformLocation(prog, "u_time");
  GLint tf_loc = p_glGetUniformLocation(prog, "u_temporalFrames");
  p_glViewport(0, 0, w, h);
  /* A scissored tile: the same uniforms and fragment coordinates as the full
   * image, only the tile's fragments are shaded (the executor does not finish
   * some fragments of the volumetric shaders: one glrun per tile isolates them) */
  if (sc[2] > 0 && sc[3] > 0) {
    p_glEnable(GL_SCISSOR_TEST);
    p_glScissor(sc[0], sc[1], sc[2], sc[3]);
  }

  for (int pass = 1; pass <= frames; pass++) {
    p_glUseProgram(prog);
    if (frame_loc >= 0) p_glUniform1ui(frame_loc, (GLuint)(frame0 + pass - 1));
    if (time_loc >= 0) p_glUniform1f(time_loc, time_ms + (float)(pass - 1) * dtime_ms);
    if (tf_loc >= 0) p_glUniform1i(tf_loc, temporal_frames);
    p_glActiveTexture(GL_TEXTURE0 + 0);
    p_glBindTexture(GL_TEXTURE_2D, single ? zero : back);
    for (int u = 1; u <= 5; u++) {
      p_glActiveTexture(GL_TEXTURE0 + u);
      p_glBindTexture(GL_TEXTURE_2D, asset[u]);
    }
    p_glActiveTexture(GL_TEXTURE0 + 6);
    p_glBindTexture(GL_TEXTURE_CUBE_MAP, cube);
    p_glActiveTexture(GL_TEXTURE0 + 7);  p_glBindTexture(GL_TEXTURE_2D, rbuf_back);
    p_glActiveTexture(GL_TEXTURE0 + 8);  p_glBindTexture(GL_TEXTURE_2D, raux_back);
    p_glActiveTexture(GL_TEXTURE0 + 9);  p_glBindTexture(GL_TEXTURE_2D, h1);
    p_glActiveTexture(GL_TEXTURE0 + 10); p_glBindTexture(GL_TEXTURE_2D, h1a);
    p_glActiveTexture(GL_TEXTURE0 + 11); p_glBindTexture(GL_TEXTURE_2D, h2);
    p_glActiveTexture(GL_TEXTURE0 + 12); p_glBindTexture(GL_TEXTURE_2D, h2a);

    p_glBindFramebuffer(GL_FRAMEBUFFER, fb);
    p_glFramebufferTexture2D(GL_FRAMEBUFFER, GL_COLOR_ATTACHMENT0, GL_TEXTURE_2D, front, 0);
    p_glFramebufferTexture2D(GL_FRAMEBUFFER, GL_COLOR_ATTACHMENT0 + 1, GL_TEXTURE_2D, rbuf, 0);
    p_glFramebufferTexture2D(GL_FRAMEBUFFER, GL_COLOR_ATTACHMENT0 + 2, GL_TEXTURE_2D, raux, 0);
    if (p_glCheckFramebufferStatus(GL_FRAMEBUFFER) != GL_FRAMEBUFFER_COMPLETE) die("fbo incomplete");
    p_glDrawArrays(GL_TRIANGLES, 0, 6);
    p_glFinish();
    if (p_glGetError() != 0) die("GL error after draw");
    fprintf(stderr, "glrun: pass %d done at %.1f s after link\n", pass, now_s() - t0);

    dump(prefix, frame0 + pass - 1, "c", w, h, fb, 0);
    if (restir_out) {
      dump(prefix, frame0 + pass - 1, "r", w, h, fb, 1);
      dump(prefix, frame0 + pass - 1, "a", w, h, fb, 2);
    }

    /* swapReSTIRBuffers (index.js:795-820) */
    GLuint o2 = h2, o2a = h2a;
    h2 = h1; h2a = h1a;
    h1 = rbuf_back; h1a = raux_back;
    rbuf_back = o2; raux_back = o2a;
    GLuint tr = rbuf, ta = raux;
    rbuf = rbuf_back; raux = raux_back;
    rbuf_back = tr; raux_back = ta;
    /* front/back swap (index.js:1102-1104) */
    GLuint t = back; back = front; front = t;
  }
  fprintf(stderr, "glrun: %d pass(es) %dx%d done (EGL %d.%d)\n", frames, w, h, maj, min);
  return 0;
}
