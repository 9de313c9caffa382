// rt0_jpeg.cpp -- baseline JPEG decoder for the reference's cubemap faces.
//
// The reference loads its environment as six JPEG files through the browser
// (`new Image()` + texImage2D(gl.RGB), index.js:298-331; cubemaps/Tropical
// Beach/*.jpg are baseline, 8-bit, 3-component JFIF).  This decodes that
// subset: SOF0 baseline Huffman, 1 or 3 components, sampling factors 1..2,
// restart intervals, JFIF YCbCr -> RGB.  Chroma is upsampled with the
// triangle ("fancy") filter libjpeg applies by default; the IDCT is the exact
// separable float transform.  Progressive / arithmetic / 12-bit files are
// rejected with RT0_E_UNSUPPORTED.  Host code, no device work.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/rt0.h"

namespace {

const int kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
                         41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
                         30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

struct Huff {
  // canonical code tables: for each length, first code and index of the first symbol
  int mincode[17], maxcode[18], valptr[17];
  uint8_t vals[256];
  bool present = false;
};

struct Comp {
  int id, h, v, tq, td, ta;
  int bw, bh;               // blocks per line / column (padded to the MCU grid)
  std::vector<uint8_t> pix;  // decoded samples, bw*8 x bh*8
  int dc = 0;
};

struct Decoder {
  const uint8_t *p, *end;
  uint16_t qt[4][64];
  Huff hd[4], ha[4];
  std::vector<Comp> comps;
  int width = 0, height = 0, hmax = 1, vmax = 1, restart = 0;
  uint32_t bitbuf = 0;
  int bitcnt = 0;
  bool marker_hit = false;
  const char *err = nullptr;

  int u16(const uint8_t *q) const { return q[0] << 8 | q[1]; }

  int fill_byte() {
    if (marker_hit || p >= end) return 0;  // pad with zeros past a marker
    uint8_t b = *p;
    if (b == 0xFF) {
      uint8_t n = p + 1 < end ? p[1] : 0;
      if (n == 0x00) {
        p += 2;
        return 0xFF;
      }
      marker_hit = true;  // RSTn / EOI: stop consuming
      return 0;
    }
    ++p;
    return b;
  }
  int bits(int n) {
    while (bitcnt < n) {
      bitbuf = (bitbuf << 8) | (uint32_t)fill_byte();
      bitcnt += 8;
    }
    int v = (int)((bitbuf >> (bitcnt - n)) & ((1u << n) - 1));
    bitcnt -= n;
    return v;
  }
  int decode_huff(const Huff &h) {
    int code = 0;
    for (int l = 1; l <= 16; ++l) {
      code = (code << 1) | bits(1);
      if (h.maxcode[l] >= 0 && code <= h.maxcode[l] && code >= h.mincode[l]) return h.vals[h.valptr[l] + code - h.mincode[l]];
    }
    err = "corrupt Huffman code";
    return 0;
  }
  static int extend(int v, int n) { return n == 0 ? 0 : (v < (1 << (n - 1)) ? v - (1 << n) + 1 : v); }

  bool read_dht(const uint8_t *q, int len) {
    const uint8_t *e = q + len;
    while (q < e) {
      int tc = q[0] >> 4, th = q[0] & 15;
      if (th > 3 || tc > 1) return false;
      Huff &h = tc ? ha[th] : hd[th];
      int count[17] = {0}, total = 0;
      for (int l = 1; l <= 16; ++l) total += count[l] = q[l];
      if (total > 256 || q + 17 + total > e) return false;
      memcpy(h.vals, q + 17, total);
      int code = 0, k = 0;
      for (int l = 1; l <= 16; ++l) {
        h.valptr[l] = k;
        h.mincode[l] = code;
        code += count[l];
        k += count[l];
        h.maxcode[l] = count[l] ? code - 1 : -1;
        code <<= 1;
      }
      h.present = true;
      q += 17 + total;
    }
    return true;
  }
  bool read_dqt(const uint8_t *q, int len) {
    const uint8_t *e = q + len;
    while (q < e) {
      int pq = q[0] >> 4, tq = q[0] & 15;
      if (tq > 3) return false;
      for (int i = 0; i < 64; ++i) qt[tq][kZigzag[i]] = pq ? (uint16_t)u16(q + 1 + 2 * i) : q[1 + i];
      q += 1 + (pq ? 128 : 64);
    }
    return true;
  }

  // exact separable IDCT of one block, level shift and clamp
  static void idct(const float in[64], uint8_t *out, int stride) {
    static float c[8][8];
    static bool init = false;
    if (!init) {
      for (int x = 0; x < 8; ++x)
        for (int u = 0; u < 8; ++u)
          c[x][u] = (u == 0 ? (float)M_SQRT1_2 : 1.0f) * cosf((2 * x + 1) * u * (float)M_PI / 16.0f);
      init = true;
    }
    float tmp[64];
    for (int y = 0; y < 8; ++y)
      for (int u = 0; u < 8; ++u) {
        float s = 0.f;
        for (int v = 0; v < 8; ++v) s += c[y][v] * in[v * 8 + u];
        tmp[y * 8 + u] = s;
      }
    for (int y = 0; y < 8; ++y)
      for (int x = 0; x < 8; ++x) {
        float s = 0.f;
        for (int u = 0; u < 8; ++u) s += c[x][u] * tmp[y * 8 + u];
        int v = (int)lrintf(s * 0.25f + 128.0f);
        out[y * stride + x] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
      }
  }

  bool decode_block(Comp &c, uint8_t *out, int stride) {
    float blk[64] = {0};
    int t = decode_huff(hd[c.td]);
    if (t > 11) return false;
    c.dc += extend(bits(t), t);
    blk[0] = (float)(c.dc * qt[c.tq][0]);
    for (int k = 1; k < 64;) {
      int rs = decode_huff(ha[c.ta]);
      int r = rs >> 4, s = rs & 15;
      if (s == 0) {
        if (r != 15) break;  // EOB
        k += 16;
        continue;
      }
      k += r;
      if (k > 63) return false;
      blk[kZigzag[k]] = (float)(extend(bits(s), s) * qt[c.tq][kZigzag[k]]);
      ++k;
    }
    idct(blk, out, stride);
    return err == nullptr;
  }

  bool restart_marker() {
    bitcnt = 0;
    bitbuf = 0;
    marker_hit = false;
    if (p + 1 < end && p[0] == 0xFF && p[1] >= 0xD0 && p[1] <= 0xD7) p += 2;
    for (Comp &c : comps) c.dc = 0;
    return true;
  }

  bool scan(const uint8_t *q) {
    int ns = q[0];
    std::vector<Comp *> sc;
    for (int i = 0; i < ns; ++i) {
      int id = q[1 + 2 * i], tab = q[2 + 2 * i];
      Comp *c = nullptr;
      for (Comp &x : comps)
        if (x.id == id) c = &x;
      if (!c) return false;
      c->td = tab >> 4;
      c->ta = tab & 15;
      if (c->td > 3 || c->ta > 3 || !hd[c->td].present || !ha[c->ta].present) return false;
      sc.push_back(c);
    }
    if (ns != (int)comps.size()) return false;  // baseline files here are interleaved
    const int mcux = (width + 8 * hmax - 1) / (8 * hmax), mcuy = (height + 8 * vmax - 1) / (8 * vmax);
    int todo = restart;
    for (int my = 0; my < mcuy; ++my)
      for (int mx = 0; mx < mcux; ++mx) {
        if (restart && todo == 0) {
          restart_marker();
          todo = restart;
        }
        for (Comp *c : sc)
          for (int by = 0; by < c->v; ++by)
            for (int bx = 0; bx < c->h; ++bx) {
              int X = (mx * c->h + bx) * 8, Y = (my * c->v + by) * 8;
              if (!decode_block(*c, c->pix.data() + (size_t)Y * c->bw * 8 + X, c->bw * 8)) return false;
            }
        if (restart) --todo;
      }
    return true;
  }

  // chroma sample of component c at luma-grid pixel (x, y): the triangle
  // filter of libjpeg's fancy upsampling (3/4 nearer, 1/4 farther sample)
  float sample(const Comp &c, int x, int y) const {
    const int sx = hmax / c.h, sy = vmax / c.v, W = c.bw * 8;
    const int cw = (width * c.h + hmax - 1) / hmax, ch = (height * c.v + vmax - 1) / vmax;
    auto at = [&](int i, int j) {
      i = i < 0 ? 0 : (i >= cw ? cw - 1 : i);
      j = j < 0 ? 0 : (j >= ch ? ch - 1 : j);
      return (float)c.pix[(size_t)j * W + i];
    };
    float fx = sx == 1 ? (float)x : (x + 0.5f) / sx - 0.5f, fy = sy == 1 ? (float)y : (y + 0.5f) / sy - 0.5f;
    int x0 = (int)floorf(fx), y0 = (int)floorf(fy);
    float a = fx - x0, b = fy - y0;
    return (1 - b) * ((1 - a) * at(x0, y0) + a * at(x0 + 1, y0)) + b * ((1 - a) * at(x0, y0 + 1) + a * at(x0 + 1, y0 + 1));
  }

  int run(uint8_t **rgba_out) {
    if (end - p < 4 || p[0] != 0xFF || p[1] != 0xD8) return RT0_E_ARG;
    p += 2;
    bool frame = false;
    while (p + 4 <= end) {
      if (p[0] != 0xFF) return RT0_E_ARG;
      int m = p[1];
      if (m == 0xFF) {
        ++p;
        continue;
      }
      if (m == 0xD9) break;
      int len = u16(p + 2);
      const uint8_t *q = p + 4;
      if (q + len - 2 > end) return RT0_E_ARG;
      if (m == 0xC4) {
        if (!read_dht(q, len - 2)) return RT0_E_ARG;
      } else if (m == 0xDB) {
        if (!read_dqt(q, len - 2)) return RT0_E_ARG;
      } else if (m == 0xDD) {
        restart = u16(q);
      } else if (m == 0xC0) {
        if (q[0] != 8) return RT0_E_UNSUPPORTED;
        height = u16(q + 1);
        width = u16(q + 3);
        int nc = q[5];
        if (width <= 0 || height <= 0 || (nc != 1 && nc != 3)) return RT0_E_UNSUPPORTED;
        comps.resize(nc);
        for (int i = 0; i < nc; ++i) {
          Comp &c = comps[i];
          c.id = q[6 + 3 * i];
          c.h = q[7 + 3 * i] >> 4;
          c.v = q[7 + 3 * i] & 15;
          c.tq = q[8 + 3 * i];
          if (c.h < 1 || c.h > 2 || c.v < 1 || c.v > 2 || c.tq > 3) return RT0_E_UNSUPPORTED;
          hmax = c.h > hmax ? c.h : hmax;
          vmax = c.v > vmax ? c.v : vmax;
        }
        const int mcux = (width + 8 * hmax - 1) / (8 * hmax), mcuy = (height + 8 * vmax - 1) / (8 * vmax);
        for (Comp &c : comps) {
          c.bw = mcux * c.h;
          c.bh = mcuy * c.v;
          c.pix.assign((size_t)c.bw * 8 * c.bh * 8, 0);
        }
        frame = true;
      } else if (m >= 0xC1 && m <= 0xCF && m != 0xC4 && m != 0xC8 && m != 0xCC) {
        return RT0_E_UNSUPPORTED;  // progressive / lossless / arithmetic
      } else if (m == 0xDA) {
        if (!frame) return RT0_E_ARG;
        p = q + len - 2;
        if (!scan(q) || err) return RT0_E_ARG;
        // skip to the next marker (EOI)
        while (p + 1 < end && !(p[0] == 0xFF && p[1] != 0x00 && !(p[1] >= 0xD0 && p[1] <= 0xD7))) ++p;
        continue;
      }
      p = q + len - 2;
    }
    if (!frame) return RT0_E_ARG;
    uint8_t *out = (uint8_t *)malloc((size_t)width * height * 4);
    if (!out) return RT0_E_ARG;
    for (int y = 0; y < height; ++y)
      for (int x = 0; x < width; ++x) {
        uint8_t *o = out + ((size_t)y * width + x) * 4;
        const Comp &Yc = comps[0];
        float Y = (Yc.h == hmax && Yc.v == vmax) ? (float)Yc.pix[(size_t)y * Yc.bw * 8 + x] : sample(Yc, x, y);
        if (comps.size() == 1) {
          o[0] = o[1] = o[2] = (uint8_t)Y;
        } else {
          float cb = sample(comps[1], x, y) - 128.f, cr = sample(comps[2], x, y) - 128.f;
          float rgb[3] = {Y + 1.402f * cr, Y - 0.344136f * cb - 0.714136f * cr, Y + 1.772f * cb};
          for (int k = 0; k < 3; ++k) {
            int v = (int)lrintf(rgb[k]);
            o[k] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
          }
        }
        o[3] = 255;
      }
    *rgba_out = out;
    return RT0_OK;
  }
};

bool read_all(const char *path, std::vector<uint8_t> &out) {
  FILE *f = fopen(path, "rb");
  if (!f) return false;
  fseek(f, 0, SEEK_END);
  long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  if (n < 0) {
    fclose(f);
    return false;
  }
  out.resize((size_t)n);
  bool ok = fread(out.data(), 1, out.size(), f) == out.size();
  fclose(f);
  return ok;
}

}  // namespace

extern "C" {

int rt0_jpeg_decode(const uint8_t *data, size_t size, int *w, int *h, uint8_t **rgba_out) {
  if (!data || !w || !h || !rgba_out) return RT0_E_ARG;
  *rgba_out = nullptr;
  Decoder d;
  d.p = data;
  d.end = data + size;
  int rc = d.run(rgba_out);
  if (rc != RT0_OK) return rc;
  *w = d.width;
  *h = d.height;
  return RT0_OK;
}

int rt0_jpeg_read(const char *path, int *w, int *h, uint8_t **rgba_out) {
  std::vector<uint8_t> buf;
  if (!path || !read_all(path, buf)) return RT0_E_ARG;
  return rt0_jpeg_decode(buf.data(), buf.size(), w, h, rgba_out);
}

}  // extern "C"
