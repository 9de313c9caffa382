// rt0_image.cpp -- image assets either side of the integrator:
// PNG decode for the texture units the reference loads with
// `new Image()` + texImage2D (index.js:257-300, 699-728), PNG encode of the
// tonemapped canvas (tonemapper.glsl -> RGBA8), and PFM for the HDR
// accumulator.  zlib does the deflate; the PNG container, filters and CRCs are
// here.  Host code, no device work.
#include <zlib.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rt0.h"

namespace {

uint32_t be32(const uint8_t *p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }
void put32(std::vector<uint8_t> &v, uint32_t x) {
  v.push_back((uint8_t)(x >> 24));
  v.push_back((uint8_t)(x >> 16));
  v.push_back((uint8_t)(x >> 8));
  v.push_back((uint8_t)x);
}

bool read_file(const char *path, std::vector<uint8_t> &out) {
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

int paeth(int a, int b, int c) {
  int p = a + b - c, pa = abs(p - a), pb = abs(p - b), pc = abs(p - c);
  return (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c);
}

}  // namespace

extern "C" {

void rt0_free(void *p) { free(p); }

int rt0_png_decode(const uint8_t *data, size_t size, int *w_out, int *h_out, uint8_t **rgba_out) {
  if (!data || !w_out || !h_out || !rgba_out) return RT0_E_ARG;
  static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', 13, 10, 26, 10};
  if (size < 8 || memcmp(data, sig, 8)) return RT0_E_ARG;
  size_t pos = 8;
  uint32_t w = 0, h = 0;
  int depth = 0, ctype = -1, interlace = 0;
  std::vector<uint8_t> idat, plte, trns;
  bool end = false;
  while (!end && pos + 12 <= size) {
    uint32_t len = be32(data + pos);
    const uint8_t *type = data + pos + 4, *body = data + pos + 8;
    if (pos + 12 + (size_t)len > size) return RT0_E_ARG;
    if (crc32(crc32(0L, Z_NULL, 0), type, len + 4) != be32(body + len)) return RT0_E_ARG;
    if (!memcmp(type, "IHDR", 4) && len >= 13) {
      w = be32(body);
      h = be32(body + 4);
      depth = body[8];
      ctype = body[9];
      interlace = body[12];
    } else if (!memcmp(type, "PLTE", 4)) {
      plte.assign(body, body + len);
    } else if (!memcmp(type, "tRNS", 4)) {
      trns.assign(body, body + len);
    } else if (!memcmp(type, "IDAT", 4)) {
      idat.insert(idat.end(), body, body + len);
    } else if (!memcmp(type, "IEND", 4)) {
      end = true;
    }
    pos += 12 + len;
  }
  if (!w || !h || w > 32768 || h > 32768) return RT0_E_ARG;
  // 8-bit, non-interlaced: gray, RGB, palette, gray+alpha, RGBA
  static const int chans[7] = {1, 0, 3, 1, 2, 0, 4};
  if (depth != 8 || interlace || ctype < 0 || ctype > 6 || !chans[ctype]) return RT0_E_UNSUPPORTED;
  const int bpp = chans[ctype];
  const size_t stride = (size_t)w * bpp;
  std::vector<uint8_t> raw((stride + 1) * h);
  uLongf rawlen = (uLongf)raw.size();
  if (uncompress(raw.data(), &rawlen, idat.data(), (uLong)idat.size()) != Z_OK || rawlen != raw.size()) return RT0_E_ARG;
  std::vector<uint8_t> px(stride * h);
  for (uint32_t y = 0; y < h; y++) {
    const uint8_t ft = raw[y * (stride + 1)];
    const uint8_t *src = &raw[y * (stride + 1) + 1];
    uint8_t *dst = &px[y * stride];
    const uint8_t *up = y ? &px[(y - 1) * stride] : nullptr;
    for (size_t i = 0; i < stride; i++) {
      int a = i >= (size_t)bpp ? dst[i - bpp] : 0, b = up ? up[i] : 0, c = (up && i >= (size_t)bpp) ? up[i - bpp] : 0;
      int pred = ft == 0 ? 0 : ft == 1 ? a : ft == 2 ? b : ft == 3 ? (a + b) / 2 : ft == 4 ? paeth(a, b, c) : -1;
      if (pred < 0) return RT0_E_ARG;
      dst[i] = (uint8_t)(src[i] + pred);
    }
  }
  uint8_t *out = (uint8_t *)malloc((size_t)w * h * 4);
  if (!out) return RT0_E_ARG;
  for (size_t i = 0; i < (size_t)w * h; i++) {
    const uint8_t *s = &px[i * bpp];
    uint8_t *d = out + i * 4;
    switch (ctype) {
      case 0: d[0] = d[1] = d[2] = s[0]; d[3] = 255; break;
      case 2: d[0] = s[0]; d[1] = s[1]; d[2] = s[2]; d[3] = 255; break;
      case 3:
        if ((size_t)s[0] * 3 + 2 >= plte.size()) {
          free(out);
          return RT0_E_ARG;
        }
        d[0] = plte[s[0] * 3]; d[1] = plte[s[0] * 3 + 1]; d[2] = plte[s[0] * 3 + 2];
        d[3] = s[0] < trns.size() ? trns[s[0]] : 255;
        break;
      case 4: d[0] = d[1] = d[2] = s[0]; d[3] = s[1]; break;
      default: memcpy(d, s, 4); break;
    }
  }
  *w_out = (int)w;
  *h_out = (int)h;
  *rgba_out = out;
  return RT0_OK;
}

int rt0_png_read(const char *path, int *w, int *h, uint8_t **rgba) {
  if (!path) return RT0_E_ARG;
  std::vector<uint8_t> buf;
  if (!read_file(path, buf)) return RT0_E_ARG;
  return rt0_png_decode(buf.data(), buf.size(), w, h, rgba);
}

int rt0_png_write(const char *path, int w, int h, const uint8_t *rgba, int flip_y) {
  if (!path || !rgba || w <= 0 || h <= 0) return RT0_E_ARG;
  const size_t stride = (size_t)w * 4;
  std::vector<uint8_t> raw((stride + 1) * h);
  for (int y = 0; y < h; y++) {
    raw[y * (stride + 1)] = 0;  // filter: none
    const int sy = flip_y ? h - 1 - y : y;
    memcpy(&raw[y * (stride + 1) + 1], rgba + (size_t)sy * stride, stride);
  }
  uLongf zlen = compressBound((uLong)raw.size());
  std::vector<uint8_t> z(zlen);
  if (compress2(z.data(), &zlen, raw.data(), (uLong)raw.size(), 6) != Z_OK) return RT0_E_ARG;
  z.resize(zlen);
  std::vector<uint8_t> png = {0x89, 'P', 'N', 'G', 13, 10, 26, 10};
  auto chunk = [&](const char *type, const std::vector<uint8_t> &body) {
    put32(png, (uint32_t)body.size());
    size_t start = png.size();
    png.insert(png.end(), type, type + 4);
    png.insert(png.end(), body.begin(), body.end());
    put32(png, (uint32_t)crc32(crc32(0L, Z_NULL, 0), &png[start], (uInt)(body.size() + 4)));
  };
  std::vector<uint8_t> ihdr;
  put32(ihdr, (uint32_t)w);
  put32(ihdr, (uint32_t)h);
  ihdr.insert(ihdr.end(), {8, 6, 0, 0, 0});  // 8-bit RGBA, deflate, no filter method, no interlace
  chunk("IHDR", ihdr);
  chunk("IDAT", z);
  chunk("IEND", {});
  FILE *f = fopen(path, "wb");
  if (!f) return RT0_E_ARG;
  bool ok = fwrite(png.data(), 1, png.size(), f) == png.size();
  ok = (fclose(f) == 0) && ok;
  return ok ? RT0_OK : RT0_E_ARG;
}

int rt0_pfm_write(const char *path, int w, int h, const float *rgba, float scale) {
  if (!path || !rgba || w <= 0 || h <= 0) return RT0_E_ARG;
  FILE *f = fopen(path, "wb");
  if (!f) return RT0_E_ARG;
  fprintf(f, "PF\n%d %d\n-1.0\n", w, h);  // little-endian; rows bottom to top, as the accumulator
  std::vector<float> row((size_t)w * 3);
  bool ok = true;
  for (int y = 0; y < h && ok; y++) {
    for (int x = 0; x < w; x++)
      for (int c = 0; c < 3; c++) row[(size_t)x * 3 + c] = rgba[((size_t)y * w + x) * 4 + c] * scale;
    ok = fwrite(row.data(), sizeof(float), row.size(), f) == row.size();
  }
  ok = (fclose(f) == 0) && ok;
  return ok ? RT0_OK : RT0_E_ARG;
}

}  // extern "C"
