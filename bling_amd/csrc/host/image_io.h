// image_io.h -- the texture-image readers behind the `.bling` loader's `image { file ... }` textures
// and `l { file ... }` environment maps.  The reference decodes these with JuicyPixels
// (IO/Bitmap.hs:13-29 readTexture -> JP.readImage, Texture.hs:110-126 decodeImage); JuicyPixels is
// a Hackage dependency absent from /root/reference, so this is a restatement of the two published
// formats the reference accepts on those paths:
//   * PNG (ISO/IEC 15948): 8-bit greyscale (Y8), RGB (RGB8), RGBA (RGBA8) and palette images (to
//     RGB8), with or without Adam7 interlacing; zlib inflates the IDAT stream.  16-bit and grey+alpha
//     images decode to JuicyPixels types the reference rejects ("unsupported image type"), so they
//     are refused here too.  JPEG (ImageYCbCr8) is not read: the loader names it and stops.
//   * Radiance RGBE (.hdr): "#?RADIANCE" / "#?RGBE" header, FORMAT=32-bit_rle_rgbe, a "-Y h +X w"
//     resolution line, flat or new-style run-length scanlines; a pixel (r, g, b, e) reads as
//     c * 2^(e - 136), e = 0 -> 0 (Ward's RGBE).  The e = 0 convention is JuicyPixels' documented
//     one; the fixtures hold no pixel where the conventions could differ (parity unpinned there).
// Host code: plain C++ and zlib, no device types.
#pragma once
#include <zlib.h>

#include <cmath>
#include <cstdint>
#include <cstring>
#include <fstream>
#include <iterator>
#include <stdexcept>
#include <string>
#include <vector>

namespace bimg {

struct Decoded {
  int width = 0, height = 0;
  int channels = 0;            // 1 = Y8, 3 = RGB8 / RGBF, 4 = RGBA8
  bool is_float = false;       // RGBE -> RGBF
  std::vector<uint8_t> bytes;  // 8-bit images, row-major from the top row
  std::vector<float> rgbf;     // RGBF images
};

inline std::vector<uint8_t> read_file(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("cannot open " + path);
  return std::vector<uint8_t>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

// ---------------------------------------------------------------- PNG
inline uint32_t be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

inline uint8_t paeth(int a, int b, int c) {
  const int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
  return (uint8_t)((pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c));
}

// undo the per-row filters of one (sub)image of w x h pixels, bpp bytes each; in holds h rows of
// 1 + w * bpp bytes, out receives h rows of w * bpp bytes
inline void unfilter(const uint8_t* in, uint8_t* out, int w, int h, int bpp) {
  const size_t stride = (size_t)w * bpp;
  for (int y = 0; y < h; ++y) {
    const uint8_t ft = in[y * (stride + 1)];
    const uint8_t* src = in + y * (stride + 1) + 1;
    uint8_t* dst = out + y * stride;
    const uint8_t* up = y ? dst - stride : nullptr;
    for (size_t i = 0; i < stride; ++i) {
      const int a = i >= (size_t)bpp ? dst[i - bpp] : 0, b = up ? up[i] : 0, c = (up && i >= (size_t)bpp) ? up[i - bpp] : 0;
      int v = src[i];
      switch (ft) {
        case 0: break;
        case 1: v += a; break;
        case 2: v += b; break;
        case 3: v += (a + b) >> 1; break;
        case 4: v += paeth(a, b, c); break;
        default: throw std::runtime_error("png: bad filter type " + std::to_string(ft));
      }
      dst[i] = (uint8_t)v;
    }
  }
}

inline Decoded decode_png(const std::vector<uint8_t>& f, const std::string& name) {
  static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', 0x0d, 0x0a, 0x1a, 0x0a};
  if (f.size() < 8 || std::memcmp(f.data(), sig, 8) != 0) throw std::runtime_error(name + ": not a PNG file");
  int w = 0, h = 0, depth = 0, ctype = -1, interlace = 0;
  std::vector<uint8_t> idat, plte;
  size_t p = 8;
  bool end = false;
  while (!end) {
    if (p + 12 > f.size()) throw std::runtime_error(name + ": truncated PNG");
    const uint32_t len = be32(&f[p]);
    const char* type = (const char*)&f[p + 4];
    if (p + 12 + (size_t)len > f.size()) throw std::runtime_error(name + ": truncated PNG chunk");
    const uint8_t* d = &f[p + 8];
    // chunk CRC over the type and data (PNG spec 5.3): a corrupt chunk is rejected, not decoded
    if ((uint32_t)crc32(crc32(0L, Z_NULL, 0), (const Bytef*)type, (uInt)(4 + len)) != be32(&f[p + 8 + len]))
      throw std::runtime_error(name + ": PNG chunk CRC mismatch");
    if (!std::memcmp(type, "IHDR", 4)) {
      if (len < 13) throw std::runtime_error(name + ": bad IHDR");
      w = (int)be32(d); h = (int)be32(d + 4); depth = d[8]; ctype = d[9]; interlace = d[12];
      if (d[10] != 0 || d[11] != 0) throw std::runtime_error(name + ": unknown PNG compression / filter method");
      if (interlace > 1) throw std::runtime_error(name + ": unknown PNG interlace method");
    } else if (!std::memcmp(type, "PLTE", 4)) {
      plte.assign(d, d + len);
    } else if (!std::memcmp(type, "IDAT", 4)) {
      idat.insert(idat.end(), d, d + len);
    } else if (!std::memcmp(type, "IEND", 4)) {
      end = true;
    }
    p += 12 + (size_t)len;
  }
  if (w <= 0 || h <= 0 || w > (1 << 15) || h > (1 << 15)) throw std::runtime_error(name + ": bad PNG size");
  if (depth != 8) throw std::runtime_error(name + ": unsupported image type (PNG bit depth " + std::to_string(depth) + ")");
  int spp;                                                    // samples per stored pixel
  switch (ctype) {
    case 0: spp = 1; break;
    case 2: spp = 3; break;
    case 3: spp = 1; if (plte.size() < 3) throw std::runtime_error(name + ": palette PNG without PLTE"); break;
    case 6: spp = 4; break;
    default: throw std::runtime_error(name + ": unsupported image type (PNG colour type " + std::to_string(ctype) + ")");
  }
  // inflate: the exact size follows from the header (one filter byte per row of each pass)
  static const int ax0[7] = {0, 4, 0, 2, 0, 1, 0}, ay0[7] = {0, 0, 4, 0, 2, 0, 1};
  static const int adx[7] = {8, 8, 4, 4, 2, 2, 1}, ady[7] = {8, 8, 8, 4, 4, 2, 2};
  auto pass_w = [&](int k) { return interlace ? (w - ax0[k] + adx[k] - 1) / adx[k] : w; };
  auto pass_h = [&](int k) { return interlace ? (h - ay0[k] + ady[k] - 1) / ady[k] : h; };
  const int npass = interlace ? 7 : 1;
  size_t raw_n = 0;
  for (int k = 0; k < npass; ++k) {
    const int pw = w > ax0[k] ? pass_w(k) : 0, ph = h > ay0[k] ? pass_h(k) : 0;
    if (pw > 0 && ph > 0) raw_n += (size_t)ph * (1 + (size_t)pw * spp);
  }
  std::vector<uint8_t> raw(raw_n);
  uLongf out_n = (uLongf)raw_n;
  if (uncompress(raw.data(), &out_n, idat.data(), (uLong)idat.size()) != Z_OK || out_n != raw_n)
    throw std::runtime_error(name + ": corrupt PNG image data");
  std::vector<uint8_t> px((size_t)w * h * spp);
  size_t off = 0;
  for (int k = 0; k < npass; ++k) {
    const int pw = w > ax0[k] ? pass_w(k) : 0, ph = h > ay0[k] ? pass_h(k) : 0;
    if (pw <= 0 || ph <= 0) continue;
    std::vector<uint8_t> sub((size_t)pw * ph * spp);
    unfilter(raw.data() + off, sub.data(), pw, ph, spp);
    off += (size_t)ph * (1 + (size_t)pw * spp);
    for (int y = 0; y < ph; ++y)
      for (int x = 0; x < pw; ++x) {
        const int X = interlace ? ax0[k] + x * adx[k] : x, Y = interlace ? ay0[k] + y * ady[k] : y;
        std::memcpy(&px[((size_t)Y * w + X) * spp], &sub[((size_t)y * pw + x) * spp], spp);
      }
  }
  Decoded r;
  r.width = w; r.height = h;
  if (ctype == 3) {                                           // palette -> RGB8
    r.channels = 3;
    r.bytes.resize((size_t)w * h * 3);
    for (size_t i = 0; i < (size_t)w * h; ++i) {
      const size_t e = (size_t)px[i] * 3;
      if (e + 2 >= plte.size()) throw std::runtime_error(name + ": palette index out of range");
      std::memcpy(&r.bytes[i * 3], &plte[e], 3);
    }
  } else {
    r.channels = spp;
    r.bytes = std::move(px);
  }
  return r;
}

// ---------------------------------------------------------------- Radiance RGBE
inline Decoded decode_hdr(const std::vector<uint8_t>& f, const std::string& name) {
  size_t p = 0;
  auto line = [&]() {
    std::string s;
    while (p < f.size() && f[p] != '\n') s += (char)f[p++];
    if (p >= f.size()) throw std::runtime_error(name + ": truncated Radiance header");
    ++p;
    return s;
  };
  const std::string magic = line();
  if (magic.rfind("#?RADIANCE", 0) != 0 && magic.rfind("#?RGBE", 0) != 0)
    throw std::runtime_error(name + ": not a Radiance HDR file");
  for (;;) {
    const std::string s = line();
    if (s.empty()) break;
    if (s.rfind("FORMAT=", 0) == 0 && s != "FORMAT=32-bit_rle_rgbe")
      throw std::runtime_error(name + ": unsupported Radiance format " + s.substr(7));
  }
  const std::string res = line();
  int w = 0, h = 0;
  char ys[3] = {0}, xs[3] = {0};
  if (std::sscanf(res.c_str(), "%2s %d %2s %d", ys, &h, xs, &w) != 4 || std::string(ys) != "-Y" || std::string(xs) != "+X")
    throw std::runtime_error(name + ": unsupported Radiance orientation '" + res + "' (only -Y h +X w)");
  if (w <= 0 || h <= 0 || w > (1 << 15) || h > (1 << 15)) throw std::runtime_error(name + ": bad HDR size");
  std::vector<uint8_t> rgbe((size_t)w * h * 4);
  std::vector<uint8_t> row((size_t)w * 4);
  for (int y = 0; y < h; ++y) {
    uint8_t* out = &rgbe[(size_t)y * w * 4];
    const bool rle = w >= 8 && w < 32768 && p + 4 <= f.size() && f[p] == 2 && f[p + 1] == 2 && ((f[p + 2] << 8) | f[p + 3]) == w;
    if (!rle) {                                               // flat scanline
      if (p + (size_t)w * 4 > f.size()) throw std::runtime_error(name + ": truncated HDR data");
      for (int x = 0; x < w; ++x) {
        if (f[p] == 1 && f[p + 1] == 1 && f[p + 2] == 1) throw std::runtime_error(name + ": old-style RLE HDR is not supported");
        std::memcpy(out + 4 * x, &f[p], 4);
        p += 4;
      }
      continue;
    }
    p += 4;
    for (int c = 0; c < 4; ++c) {                             // four planes, each run-length coded
      int x = 0;
      while (x < w) {
        if (p >= f.size()) throw std::runtime_error(name + ": truncated HDR data");
        int n = f[p++];
        if (n > 128) {
          n -= 128;
          if (x + n > w || p >= f.size()) throw std::runtime_error(name + ": bad HDR run");
          const uint8_t v = f[p++];
          for (int k = 0; k < n; ++k) row[(size_t)(x++) * 4 + c] = v;
        } else {
          if (n == 0 || x + n > w || p + n > f.size()) throw std::runtime_error(name + ": bad HDR run");
          for (int k = 0; k < n; ++k) row[(size_t)(x++) * 4 + c] = f[p++];
        }
      }
    }
    std::memcpy(out, row.data(), row.size());
  }
  Decoded r;
  r.width = w; r.height = h; r.channels = 3; r.is_float = true;
  r.rgbf.resize((size_t)w * h * 3);
  for (size_t i = 0; i < (size_t)w * h; ++i) {
    const int e = rgbe[i * 4 + 3];
    const float s = e == 0 ? 0.f : std::ldexp(1.f, e - 136);   // exact power of two
    for (int c = 0; c < 3; ++c) r.rgbf[i * 3 + c] = (float)rgbe[i * 4 + c] * s;
  }
  return r;
}

// JP.readImage: the format from the file's magic bytes
inline Decoded read_image(const std::string& path) {
  const std::vector<uint8_t> f = read_file(path);
  if (f.size() >= 8 && f[0] == 0x89 && f[1] == 'P' && f[2] == 'N' && f[3] == 'G') return decode_png(f, path);
  if (f.size() >= 2 && f[0] == '#' && f[1] == '?') return decode_hdr(f, path);
  if (f.size() >= 2 && f[0] == 0xff && f[1] == 0xd8) throw std::runtime_error(path + ": JPEG images are not supported");
  throw std::runtime_error(path + ": unknown image format");
}

}  // namespace bimg
