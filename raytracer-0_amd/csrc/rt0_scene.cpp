// rt0_scene.cpp -- host-side front-end: parses the reference's compile-time
// strings into flat records.
//
// The reference never parses anything: parseShader (tools.js:22-61) splices
// GlslViewport.defines/.constants at `#constants`, .scene at `#scene` and
// .sdf_meshes at `#sdf_meshes`, and the GLSL compiler does the rest.  This file
// accepts exactly those strings (the grammar produced by index.js:11-85 and
// index.html:610-717) and produces rt0_config / rt0_mesh records.
#include <algorithm>
#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rt0.h"
#include "rt0_internal.h"

namespace rt0h {

// Texture table, raytracer.glsl:112-141: the textures the material table
// references, keyed by their type (each type has one definition there).
struct TexDef {
  int type;
  float cm[3], em[3], params[4];
};
static const TexDef kTextures[] = {
    {-1, {1, 1, 1}, {1, 1, 1}, {0, 0, 0, 0}},        // NULL_TEX (131)
    {0, {1, 1, 1}, {1, 1, 1}, {0, 0, 0, 1}},         // TEX_0 (134)
    {1, {1, 1, 1}, {1, 1, 1}, {0, 0, 0, 1}},         // TEX_1
    {2, {1, 1, 1}, {1, 1, 1}, {0, 0, 0, 1}},         // TEX_2
    {3, {1, 1, 1}, {1, 1, 1}, {0, 0, 0, 1}},         // TEX_3
    {6, {1, 1, 1}, {1, 1, 1}, {16, 16, 16, 16}},     // TEX_VALUE_NOISE (139)
    {7, {1, 1, 1}, {0, 0, 0}, {5, 5, 2, 0}},         // TEX_CHECK (140)
    {9, {0.7f, 0.25f, 0.055f}, {0.6f, 0.2f, 0.6f}, {16, 10, 16, 0}},  // TEX_METAL (141)
};

// Material table, raytracer.glsl:165-224; opts = Material.opts bits (1 colour
// texture, 2 emission texture).
struct MatDef {
  const char *name;
  float c[3], e[3], nt;
  int type, tex;
  unsigned opts;
};
static const float IOR_GLASS = 1.53f, IOR_SAPPHIRE = 1.77f, IOR_WATER = 1.33f, IOR_COAT = 1.4f;
static const MatDef kMaterials[] = {
    {"NULL_MAT", {0, 0, 0}, {0, 0, 0}, 0.f, -1, -1, 0u},
    {"MAT_REFR_CLEAR", {1.f, 0.5f, 0.f}, {0, 0, 0}, IOR_GLASS, 4, -1, 0u},
    {"MAT_REFR_CLEAR_2", {1, 1, 1}, {0, 0, 0}, IOR_GLASS, 5, -1, 0u},
    {"MAT_REFR_SAPPHIRE", {1, 1, 1}, {0, 0, 0}, IOR_SAPPHIRE, 4, -1, 0u},
    {"MAT_REFR_WATER", {0.25f, 0.64f, 0.88f}, {0, 0, 0}, IOR_WATER, 4, -1, 0u},
    {"MAT_REFR_TEST", {1, 1, 1}, {0, 0, 0}, IOR_GLASS, 4, 1, 1u},
    {"MAT_LIGHT_4", {1, 1, 1}, {4, 4, 4}, 0.f, 0, -1, 0u},
    {"MAT_LIGHT_CANDLE_4", {1.0f, 0.57647058823f, 0.16078431372f}, {4, 4, 4}, 0.f, 0, -1, 0u},
    {"MAT_LIGHT_HALOGEN_4", {1.0f, 0.94509803921f, 0.87843137254f}, {4, 4, 4}, 0.f, 0, -1, 0u},
    {"MAT_LIGHT_DEMO", {1, 1, 1}, {10, 10, 10}, 0.f, 0, -1, 0u},
    {"MAT_LIGHT_4_TEX", {1, 1, 1}, {1, 1, 1}, 0.f, 0, 1, 1u},
    {"MAT_CLEAR_SKY", {0.25098039215f, 0.61176470588f, 1.0f}, {1, 1, 1}, 0.f, 1, -1, 0u},
    {"MAT_OVERCAST_SKY", {0.78823529411f, 0.8862745098f, 1.0f}, {1, 1, 1}, 0.f, 1, -1, 0u},
    {"MAT_DIRECT_SUNLIGHT", {1, 1, 1}, {1, 1, 1}, 0.f, 1, -1, 0u},
    {"MAT_MIRROR", {1, 1, 1}, {0, 0, 0}, 0.f, 3, -1, 0u},
    {"MAT_METAL", {0.6f, 0.6f, 0.6f}, {0, 0, 0}, 0.f, 3, 9, 2u},
    {"MAT_BLACK", {0, 0, 0}, {0, 0, 0}, 0.f, 2, -1, 0u},
    {"MAT_WHITE", {1, 1, 1}, {0, 0, 0}, 0.f, 2, -1, 0u},
    {"MAT_RED", {1, 0, 0}, {0, 0, 0}, 0.f, 2, -1, 0u},
    {"MAT_GREEN", {0, 1, 0}, {0, 0, 0}, 0.f, 2, -1, 0u},
    {"MAT_BLUE", {0, 0, 1}, {0, 0, 0}, 0.f, 2, -1, 0u},
    {"MAT_CORNELL_WHITE", {1, 1, 1}, {0, 0, 0}, 0.f, 2, -1, 0u},
    {"MAT_CORNELL_RED", {0.7f, 0.12f, 0.05f}, {0, 0, 0}, 0.f, 2, -1, 0u},
    {"MAT_CORNELL_GREEN", {0.2f, 0.4f, 0.36f}, {0, 0, 0}, 0.f, 2, -1, 0u},
    {"MAT_YELLOW", {1, 1, 0}, {0, 0, 0}, 0.f, 2, -1, 0u},
    {"MAT_PURPLE", {0.50196078431f, 0, 0.50196078431f}, {0, 0, 0}, 0.f, 2, -1, 0u},
    {"MAT_CHECK_WHITE", {0, 0, 0}, {0, 0, 0}, 0.f, 2, 7, 1u},
    {"MAT_COAT_NAVY", {0, 0, 0.50196078431f}, {1, 1, 1}, IOR_COAT, 6, -1, 0u},
    {"MAT_COAT_PURPLE", {0.50196078431f, 0, 0.50196078431f}, {0, 0, 0}, IOR_COAT, 6, -1, 0u},
    {"MAT_COAT_WAX", {0.9333f, 0.6666f, 0.6f}, {0.005f, 0.005f, 0.005f}, IOR_COAT, 6, -1, 0u},
    {"MAT_TEST", {1, 1, 1}, {0, 0, 0}, 0.f, 2, 1, 1u},
    {"MAT_SPECTRAL_FLINT", {1, 1, 1}, {0, 0, 0}, -1.7167f, 4, -1, 0u},
    {"MAT_SPECTRAL_DIAMOND", {1, 1, 1}, {0, 0, 0}, -2.3991f, 4, -1, 0u},
};

static std::string strip_comments(const char *s) {
  std::string out;
  for (size_t i = 0; s[i];) {
    if (s[i] == '/' && s[i + 1] == '/') {
      while (s[i] && s[i] != '\n') i++;
    } else if (s[i] == '/' && s[i + 1] == '*') {
      i += 2;
      while (s[i] && !(s[i] == '*' && s[i + 1] == '/')) i++;
      if (s[i]) i += 2;
    } else {
      out.push_back(s[i++]);
    }
  }
  return out;
}

static void skip_ws(const char *&p) {
  while (*p && isspace((unsigned char)*p)) p++;
}
static bool ident(const char *&p, std::string &out) {
  skip_ws(p);
  if (!(isalpha((unsigned char)*p) || *p == '_')) return false;
  out.clear();
  while (isalnum((unsigned char)*p) || *p == '_') out.push_back(*p++);
  return true;
}
static bool expect(const char *&p, char c) {
  skip_ws(p);
  if (*p != c) return false;
  p++;
  return true;
}
// vecN(a, b, ...) with GLSL scalar broadcast; numeric literals only
static bool parse_vec(const char *&p, int n, float *out) {
  std::string id;
  if (!ident(p, id)) return false;
  if (id != (n == 3 ? "vec3" : "vec4")) return false;
  if (!expect(p, '(')) return false;
  float v[4] = {0, 0, 0, 0};
  int k = 0;
  for (;;) {
    skip_ws(p);
    char *end;
    float x = strtof(p, &end);
    if (end == p) return false;
    if (k < 4) v[k] = x;
    k++;
    p = end;
    skip_ws(p);
    if (*p == ',') {
      p++;
      continue;
    }
    if (*p == ')') {
      p++;
      break;
    }
    return false;
  }
  if (k != 1 && k != n) return false;
  for (int i = 0; i < n; i++) out[i] = (k == 1) ? v[0] : v[i];
  return true;
}

int lookup_material(const std::string &name, rt0_mesh &m) {
  for (const MatDef &d : kMaterials) {
    if (name == d.name) {
      for (int i = 0; i < 3; i++) {
        m.c[i] = d.c[i];
        m.e[i] = d.e[i];
      }
      m.nt = d.nt;
      m.mat_type = d.type;
      m.tex_type = d.tex;
      m.mat_opts = d.opts;
      for (const TexDef &t : kTextures) {
        if (t.type != d.tex) continue;
        for (int i = 0; i < 3; i++) {
          m.tex_c_mask[i] = t.cm[i];
          m.tex_e_mask[i] = t.em[i];
        }
        for (int i = 0; i < 4; i++) m.tex_params[i] = t.params[i];
      }
      return 0;
    }
  }
  return -1;
}

int parse_scene_glsl(const char *text, const char *const *sdf, int n_sdf, std::vector<rt0_mesh> &meshes,
                     int &n_euclid, int &n_sdfs, int &n_models, std::vector<int32_t> &lights, std::string &err) {
  if (!text) {
    err = "scene text is NULL";
    return RT0_E_ARG;
  }
  std::string s = strip_comments(text);
  meshes.clear();
  lights.clear();
  // Mesh(MAT, TYPE, vec3(...), vec4(...)) entries in order
  const char *p = s.c_str();
  while ((p = strstr(p, "Mesh"))) {
    const char *q = p + 4;
    bool word_start = (p == s.c_str()) || !(isalnum((unsigned char)p[-1]) || p[-1] == '_');
    p = q;
    if (!word_start || isalnum((unsigned char)*q) || *q == '_') continue;
    skip_ws(q);
    if (*q != '(') continue;  // `Mesh meshes[...]`, `Mesh[](`
    q++;
    rt0_mesh m;
    memset(&m, 0, sizeof m);
    std::string mat, type;
    if (!ident(q, mat) || !expect(q, ',') || !ident(q, type) || !expect(q, ',') || !parse_vec(q, 3, m.pos) ||
        !expect(q, ',') || !parse_vec(q, 4, m.joker) || !expect(q, ')')) {
      err = "cannot parse Mesh entry near: " + std::string(p - 4, strnlen(p - 4, 60));
      return RT0_E_ARG;
    }
    if (lookup_material(mat, m)) {
      err = "unknown material " + mat;
      return RT0_E_ARG;
    }
    if (type == "SPHERE") m.type = 0;
    else if (type == "PLANE") m.type = 1;
    else if (type == "BOX") m.type = 2;
    else if (type == "SDF") m.type = 3;
    else if (type == "TRIANGLE") m.type = 5;  // a triangle model (rt0_set_model), index.html:648-649
    else if (type == "GRID_SDF") {
      err = "mesh type " + type + " has no implementation in the reference integrator";
      return RT0_E_UNSUPPORTED;
    } else {
      err = "There's no such thing as " + type;  // index.html:651
      return RT0_E_ARG;
    }
    m.sdf_kind = -1;
    meshes.push_back(m);
    p = q;
  }
  // light_index[N] = int[](a, b, ...)
  const char *l = strstr(s.c_str(), "light_index");
  if (!l) {
    err = "scene has no light_index[] array";
    return RT0_E_ARG;
  }
  const char *a = strstr(l, "int[]");
  const char *b = a ? strchr(a, '(') : nullptr;
  if (!b) {
    err = "cannot parse light_index[]";
    return RT0_E_ARG;
  }
  b++;
  for (;;) {
    skip_ws(b);
    if (*b == ')') break;
    char *end;
    long v = strtol(b, &end, 10);
    if (end == b) {
      err = "cannot parse light_index[] value";
      return RT0_E_ARG;
    }
    lights.push_back((int32_t)v);
    b = end;
    skip_ws(b);
    if (*b == ',') b++;
  }
  // meshes[0..NUM_MESHES) Euclidean, then SDFs (index.html:702-717 addresses
  // meshes[NUM_MESHES + i]), then the models (meshes[NUM_MESHES + NUM_SDFS +
  // NUM_MODELS], index.html:669)
  n_euclid = 0;
  n_sdfs = 0;
  n_models = 0;
  for (const rt0_mesh &m : meshes) {
    if (m.type == 5) {
      n_models++;
    } else if (m.type == 3) {
      if (n_models) {
        err = "TRIANGLE models must follow the SDF meshes";
        return RT0_E_ARG;
      }
      n_sdfs++;
    } else {
      if (n_sdfs || n_models) {
        err = "SDF meshes and TRIANGLE models must follow the Euclidean meshes";
        return RT0_E_ARG;
      }
      n_euclid++;
    }
  }
  // sdf_meshes statements: sdf_meshes[i] = vec2(<prim>(p-meshes[NUM_MESHES + i].pos, ...), i);
  static const char *prims[] = {"sdBox", "udRoundBox", "sdSphere", "sdTriPrism", "sdCone", "MengerSponge", "Mandelbulb"};
  std::vector<int> kind(n_sdfs, -1);
  for (int k = 0; k < n_sdf; k++) {
    std::string st = strip_comments(sdf[k] ? sdf[k] : "");
    const char *q = strstr(st.c_str(), "sdf_meshes");
    if (!q) continue;
    q = strchr(q, '[');
    if (!q) {
      err = "cannot parse sdf_meshes statement";
      return RT0_E_ARG;
    }
    int idx = atoi(q + 1);
    const char *v = strstr(q, "vec2");
    v = v ? strchr(v, '(') : nullptr;
    if (!v) {
      err = "cannot parse sdf_meshes statement";
      return RT0_E_ARG;
    }
    v++;
    std::string fn;
    if (!ident(v, fn)) {
      err = "cannot parse sdf_meshes statement";
      return RT0_E_ARG;
    }
    int found = -1;
    for (int j = 0; j < 7; j++)
      if (fn == prims[j]) found = j;
    if (found < 0) {
      err = "unsupported SDF primitive " + fn;
      return RT0_E_UNSUPPORTED;
    }
    if (idx < 0 || idx >= n_sdfs) {
      err = "sdf_meshes index out of range";
      return RT0_E_ARG;
    }
    kind[idx] = found;
  }
  for (int i = 0; i < n_sdfs; i++) {
    if (kind[i] < 0) {
      err = "SDF mesh " + std::to_string(i) + " has no sdf_meshes statement";
      return RT0_E_ARG;
    }
    meshes[n_euclid + i].sdf_kind = kind[i];
  }
  return RT0_OK;
}

static const char *kDefineNames[7] = {"USE_CUBEMAP",  "USE_PROCEDURAL_SKY", "USE_BIASED_SAMPLING", "USE_BIDIRECTIONAL",
                                      "USE_RESTIR",   "USE_SPECTRAL",       "USE_VOLUMETRICS"};

void default_config(rt0_config &c) {
  // index.js:11-35
  c.defines = RT0_USE_PROCEDURAL_SKY | RT0_USE_BIASED_SAMPLING;
  c.max_bounces = 12;
  c.max_diff_bounces = 4;
  c.max_spec_bounces = 4;
  c.max_trans_bounces = 12;
  c.max_scattering_events = 12;
  c.marching_steps = 128;
  c.fudge_factor = 0.9f;
  c.sample_lights = 1;
  c.use_mis = 0;
  c.use_restir = 0;
  c.light_path_length = 2;
  c.restir_samples = 16;
  c.render_mode = 0;
}

int parse_config(const char *const *defines, int nd, const char *const *constants, int nc, rt0_config &c,
                 std::string &err) {
  default_config(c);
  c.defines = 0;
  for (int i = 0; i < nd; i++) {
    std::string d = defines[i] ? defines[i] : "";
    size_t at = d.find("#define");
    if (at == std::string::npos) {
      err = "cannot parse define: " + d;
      return RT0_E_ARG;
    }
    bool commented = d.find("//") != std::string::npos && d.find("//") < at;
    const char *q = d.c_str() + at + 7;
    std::string name;
    if (!ident(q, name)) {
      err = "cannot parse define: " + d;
      return RT0_E_ARG;
    }
    int bit = -1;
    for (int k = 0; k < 7; k++)
      if (name == kDefineNames[k]) bit = k;
    if (bit < 0) {
      err = "unknown define " + name;
      return RT0_E_ARG;
    }
    if (!commented) c.defines |= 1u << bit;
  }
  for (int i = 0; i < nc; i++) {
    std::string s = constants[i] ? constants[i] : "";
    size_t eq = s.find('=');
    if (eq == std::string::npos) {
      err = "cannot parse constant: " + s;
      return RT0_E_ARG;
    }
    std::string lhs = s.substr(0, eq);
    size_t e = lhs.find_last_not_of(" \t");
    size_t b = lhs.find_last_of(" \t", e);
    std::string name = lhs.substr(b == std::string::npos ? 0 : b + 1, e - (b == std::string::npos ? 0 : b + 1) + 1);
    std::string rhs = s.substr(eq + 1);
    size_t semi = rhs.find(';');
    if (semi != std::string::npos) rhs = rhs.substr(0, semi);
    const char *r = rhs.c_str();
    skip_ws(r);
    double v;
    if (!strncmp(r, "true", 4)) v = 1;
    else if (!strncmp(r, "false", 5)) v = 0;
    else {
      char *end;
      v = strtod(r, &end);
      if (end == r) {
        err = "cannot parse constant value: " + s;
        return RT0_E_ARG;
      }
    }
    int iv = (int)v;
    if (name == "MAX_BOUNCES") c.max_bounces = iv;
    else if (name == "MAX_DIFF_BOUNCES") c.max_diff_bounces = iv;
    else if (name == "MAX_SPEC_BOUNCES") c.max_spec_bounces = iv;
    else if (name == "MAX_TRANS_BOUNCES") c.max_trans_bounces = iv;
    else if (name == "MAX_SCATTERING_EVENTS") c.max_scattering_events = iv;
    else if (name == "MARCHING_STEPS") c.marching_steps = iv;
    else if (name == "FUDGE_FACTOR") c.fudge_factor = (float)v;
    else if (name == "sample_lights") c.sample_lights = iv;
    else if (name == "use_mis") c.use_mis = iv;
    else if (name == "use_restir") c.use_restir = iv;
    else if (name == "LIGHT_PATH_LENGTH") c.light_path_length = iv;
    else if (name == "RESTIR_SAMPLES") c.restir_samples = iv;
    else if (name == "RENDER_MODE") c.render_mode = iv;
    else {
      err = "unknown constant " + name;
      return RT0_E_ARG;
    }
  }
  return RT0_OK;
}

}  // namespace rt0h

// ---------------------------------------------------------------- OBJ models
// The reference's triangle path loaded a Wavefront OBJ (models/Stanford/Happy
// Buddha.obj, .gitignore) through its unshipped mesh.js.  Vertices (`v x y z`)
// and faces (`f a b c ...`, each a `v`, `v/vt`, `v//vn` or `v/vt/vn` token,
// 1-based or negative = relative); polygons are fan-triangulated; other
// records are ignored.
namespace rt0h {
int parse_obj(const char *text, size_t len, std::vector<float> &pos, std::vector<int32_t> &tris, std::string &err) {
  pos.clear();
  tris.clear();
  const char *p = text, *end = text + len;
  long line = 0;
  while (p < end) {
    const char *eol = (const char *)memchr(p, '\n', (size_t)(end - p));
    if (!eol) eol = end;
    ++line;
    std::string ln(p, (size_t)(eol - p));
    p = eol + 1;
    const char *q = ln.c_str();
    while (*q == ' ' || *q == '\t') ++q;
    if (q[0] == 'v' && (q[1] == ' ' || q[1] == '\t')) {
      char *e;
      float xyz[3];
      const char *r = q + 2;
      for (int k = 0; k < 3; ++k) {
        xyz[k] = strtof(r, &e);
        if (e == r) {
          err = "OBJ line " + std::to_string(line) + ": bad vertex";
          return RT0_E_ARG;
        }
        r = e;
      }
      pos.insert(pos.end(), xyz, xyz + 3);
    } else if (q[0] == 'f' && (q[1] == ' ' || q[1] == '\t')) {
      std::vector<int32_t> f;
      const char *r = q + 2;
      const long nv = (long)(pos.size() / 3);
      for (;;) {
        while (*r == ' ' || *r == '\t' || *r == '\r') ++r;
        if (!*r) break;
        char *e;
        long v = strtol(r, &e, 10);
        if (e == r) {
          err = "OBJ line " + std::to_string(line) + ": bad face";
          return RT0_E_ARG;
        }
        v = v < 0 ? nv + v : v - 1;
        if (v < 0 || v >= nv) {
          err = "OBJ line " + std::to_string(line) + ": face index out of range";
          return RT0_E_ARG;
        }
        f.push_back((int32_t)v);
        r = e;
        while (*r && *r != ' ' && *r != '\t') ++r;  // skip /vt/vn
      }
      for (size_t k = 2; k < f.size(); ++k) {
        tris.push_back(f[0]);
        tris.push_back(f[k - 1]);
        tris.push_back(f[k]);
      }
    }
  }
  return RT0_OK;
}
}  // namespace rt0h

extern "C" int rt0_obj_read(const char *path, float **positions, int *n_vertices, int32_t **indices,
                            int *n_triangles) {
  if (!path || !positions || !n_vertices || !indices || !n_triangles) return RT0_E_ARG;
  FILE *f = fopen(path, "rb");
  if (!f) return RT0_E_ARG;
  std::string text;
  char buf[1 << 16];
  size_t k;
  while ((k = fread(buf, 1, sizeof buf, f)) > 0) text.append(buf, k);
  fclose(f);
  std::vector<float> pos;
  std::vector<int32_t> tri;
  std::string err;
  int rc = rt0h::parse_obj(text.data(), text.size(), pos, tri, err);
  if (rc != RT0_OK) return rc;
  *positions = (float *)malloc(std::max<size_t>(1, pos.size()) * sizeof(float));
  *indices = (int32_t *)malloc(std::max<size_t>(1, tri.size()) * sizeof(int32_t));
  if (!*positions || !*indices) return RT0_E_ARG;
  memcpy(*positions, pos.data(), pos.size() * sizeof(float));
  memcpy(*indices, tri.data(), tri.size() * sizeof(int32_t));
  *n_vertices = (int)(pos.size() / 3);
  *n_triangles = (int)(tri.size() / 3);
  return RT0_OK;
}
