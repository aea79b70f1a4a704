// loader.cpp -- `.bling` scene loader: a C++ restatement of the reference's Parsec grammar
// (src/lib/Graphics/Bling/IO/*.hs) for the constructs the benchmark scenes use, producing the
// flattened bling_scene_desc of include/bling_scene.h.  The parser is host code and unchanged in
// the reference design; it is restated here only because GHC is not available in this image.
//
// Parse-state mirrors PState (IO/ParserCore.hs:45-58).  Spectra are converted to the 16-band
// representation at parse time exactly like the reference (fromSpd / rgbToSpectrum).
#include "../common/scene_features.h"
#include "../common/perlin.h"
#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../../include/bling_host.h"
#include "../common/spectral_data.h"
#include "../common/sky_model.h"
#include "../common/cr_math.h"
#include "hmath.h"
#include "image_io.h"

using namespace bh;

namespace {

thread_local std::string g_err;

struct ParseError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

typedef std::vector<float> Spec;  // always 16 bands

Spec sconst(float v) { return Spec(16, v); }

// ---------------------------------------------------------------- spectra (Spectrum.hs)
// avgSpd for an IrregularSpd (Spectrum.hs:307-314) and fromSpd (Spectrum.hs:329-335).
float lerpf(float t, float a, float b) { return (1.f - t) * a + t * b; }            // Math.hs:108-110

Spec from_irregular(std::vector<std::pair<float, float>> pts) {
  // mkSpd sorts by lambda with a stable sort (Spectrum.hs:199-207)
  std::stable_sort(pts.begin(), pts.end(),
                   [](const std::pair<float, float>& a, const std::pair<float, float>& b) { return a.first < b.first; });
  Spec s(16);
  int n = (int)pts.size();
  for (int i = 0; i < 16; ++i) {
    float l0 = lerpf((float)i / 16.f, 400.f, 700.f);
    float l1 = lerpf((float)(i + 1) / 16.f, 400.f, 700.f);
    if (l1 <= pts.front().first) { s[i] = pts.front().second; continue; }
    if (l0 >= pts.back().first) { s[i] = pts.back().second; continue; }
    int i0 = 0, i1 = n - 1;
    for (int k = 0; k < n; ++k) if (pts[k].first >= l0) { i0 = k; break; }
    for (int k = 0; k < n; ++k) if (pts[k].first >= l1) { i1 = k; break; }
    float acc = 0.f;
    int cnt = i1 - i0 + 1;
    for (int k = i0; k <= i1; ++k) acc = acc + pts[k].second;
    s[i] = acc / (float)cnt;
  }
  return s;
}

Spec band_scale(const float* b, float f) { Spec r(16); for (int i = 0; i < 16; ++i) r[i] = b[i] * f; return r; }
Spec sadd(const Spec& a, const Spec& b) { Spec r(16); for (int i = 0; i < 16; ++i) r[i] = a[i] + b[i]; return r; }

// rgbToSpectrum (Spectrum.hs:146-159); bases order r,g,b,c,m,y,w.  The third branch's `r <= b`
// test is kept as written.
Spec rgb_to_spectrum(const float (*B)[16], float r, float g, float b) {
  const float *rb = B[0], *gb = B[1], *bb = B[2], *cb = B[3], *mb = B[4], *yb = B[5], *wb = B[6];
  if (r <= g && r <= b)
    return sadd(band_scale(wb, r), g <= b ? sadd(band_scale(cb, g - r), band_scale(bb, b - g))
                                          : sadd(band_scale(cb, b - r), band_scale(gb, g - b)));
  if (g <= r && g <= b)
    return sadd(band_scale(wb, g), r <= b ? sadd(band_scale(mb, r - g), band_scale(bb, b - r))
                                          : sadd(band_scale(mb, b - g), band_scale(rb, r - b)));
  return sadd(band_scale(wb, b), r <= b ? sadd(band_scale(yb, r - b), band_scale(gb, g - r))
                                        : sadd(band_scale(yb, g - b), band_scale(rb, r - g)));
}

// sBlackBody (Spectrum.hs:480-493): fromSpd of an SpdFunc = per band (f l0 + f l1) * 0.5
Spec black_body(float temp) {
  auto planck = [&](float w) {
    float wp = w * 1e-9f;
    float p5 = 1.f / (wp * wp * wp * wp * wp);
    return (0.4e-9f * (3.74183e-16f * p5)) / (std::exp(1.4388e-2f / (wp * temp)) - 1.f);
  };
  Spec s(16);
  for (int i = 0; i < 16; ++i) {
    float l0 = lerpf((float)i / 16.f, 400.f, 700.f);
    float l1 = lerpf((float)(i + 1) / 16.f, 400.f, 700.f);
    s[i] = (planck(l0) + planck(l1)) * 0.5f;
  }
  return s;
}

// ---------------------------------------------------------------- noise (Texture.hs:341-414)
using bperlin::perlin3d;
using bperlin::fbm;
// ScalarMap2d (MaterialParser.hs:232-245): fbm z {octaves, omega} | scale f <map>
struct ScalarMap2d {
  int kind = 0;                 // 0 = fbm (texMap3dTo2d (fbm o w) z), 1 = scale f m
  float z = 0.f, omega = 0.f, f = 1.f;
  int octaves = 0;
  std::unique_ptr<ScalarMap2d> child;
  float eval(float x, float y) const {
    if (kind == 1) return f * child->eval(x, y);
    return fbm(octaves, omega, x, y, z);
  }
};

// ---------------------------------------------------------------- filters (Filter.hs)
float eval_filter(int kind, const float* p, float x, float y) {
  switch (kind) {
    case BLING_FILTER_BOX: return (std::fabs(x) < 0.5f && std::fabs(y) < 0.5f) ? 1.f : 0.f;
    case BLING_FILTER_GAUSS: {  // p: w h alpha expX expY
      auto g = [&](float d, float ev) { return hmax(0.f, std::exp(-p[2] * d * d) - ev); };
      return g(x, p[3]) * g(y, p[4]);
    }
    case BLING_FILTER_SINC: {  // p: w h tau
      auto s1 = [&](float v) {
        if (std::fabs(v) > 1.f) return 0.f;
        if (std::fabs(v) < 1e-5f) return 1.f;
        float xp = std::fabs(v) * kPi;
        float lz = std::sin(xp * p[2]) / (xp * p[2]);
        float sc = std::sin(xp) / xp;
        return sc * lz;
      };
      return s1(x * (1.f / p[0])) * s1(y * (1.f / p[1]));
    }
    case BLING_FILTER_MITCHELL: {  // Filter.hs:75-85, p: w h b c
      float b = p[2], c = p[3];
      auto m1d = [&](float xp) {
        float xx = std::fabs(2.f * xp);
        if (xx > 1.f)
          return ((((-b) - 6.f * c) * xx * xx * xx + (6.f * b + 30.f * c) * xx * xx +
                   ((-12.f) * b - 48.f * c) * xx + (8.f * b + 24.f * c)) * (1.f / 6.f));
        return (((12.f - 9.f * b - 6.f * c) * xx * xx * xx + ((-18.f) + 12.f * b + 6.f * c) * xx * xx +
                 (6.f - 2.f * b)) * (1.f / 6.f));
      };
      float iw = 1.f / p[0], ih = 1.f / p[1];
      return m1d(x * iw) * m1d(y * ih);
    }
    case BLING_FILTER_TRIANGLE: {  // Filter.hs:95-96
      float v = hmax(0.f, p[0] - std::fabs(x * 2.f)) * hmax(0.f, p[1] - std::fabs(y * 2.f));
      return v / (p[0] * p[1]);
    }
  }
  return 0.f;
}

void build_filter(bling_filter& f, int kind, const float* p) {
  f.kind = kind;
  if (kind == BLING_FILTER_BOX) { f.width = 0.5f; f.height = 0.5f; }
  else { f.width = p[0]; f.height = p[1]; }
  // mkTableFilter (Image.hs:48-61)
  for (int y = 0; y < 16; ++y) {
    float fy = ((float)y + 0.5f) * f.height / 16.f;
    for (int x = 0; x < 16; ++x) {
      float fx = ((float)x + 0.5f) * f.width / 16.f;
      f.table[y * 16 + x] = eval_filter(kind, p, fx, fy);
    }
  }
}

// ---------------------------------------------------------------- tokenizer
class Lexer {
 public:
  explicit Lexer(std::string s) : s_(std::move(s)) {}
  // ws (IO/ParserCore.hs:103-111): whitespace and '#' comments
  void skip() {
    for (;;) {
      while (p_ < s_.size() && std::isspace((unsigned char)s_[p_])) ++p_;
      if (p_ < s_.size() && s_[p_] == '#') { while (p_ < s_.size() && s_[p_] != '\n') ++p_; continue; }
      break;
    }
  }
  bool eof() { skip(); return p_ >= s_.size(); }
  char peekc() { skip(); return p_ < s_.size() ? s_[p_] : '\0'; }
  bool accept(char c) { if (peekc() == c) { ++p_; return true; } return false; }
  void expect(char c) {
    if (!accept(c)) fail(std::string("expected '") + c + "'");
  }
  // pString: many1 alphaNum
  std::string word() {
    skip();
    size_t b = p_;
    while (p_ < s_.size() && std::isalnum((unsigned char)s_[p_])) ++p_;
    if (b == p_) fail("expected identifier");
    return s_.substr(b, p_ - b);
  }
  std::string peek_word() { size_t save = p_; std::string w; try { w = word(); } catch (...) { w.clear(); } p_ = save; return w; }
  bool is_word(const char* w) { return peek_word() == w; }
  void expect_word(const char* w) { std::string x = word(); if (x != w) fail(std::string("expected ") + w + ", got " + x); }
  // flt' (IO/ParserCore.hs:114-122): [+-] digits [. digits]; correctly rounded like `read`
  float flt() {
    skip();
    size_t b = p_;
    std::string t;
    if (p_ < s_.size() && (s_[p_] == '+' || s_[p_] == '-')) t += s_[p_++];
    size_t d0 = p_;
    while (p_ < s_.size() && std::isdigit((unsigned char)s_[p_])) t += s_[p_++];
    if (p_ == d0) { p_ = b; fail("expected number"); }
    if (p_ < s_.size() && s_[p_] == '.') {
      t += s_[p_++];
      while (p_ < s_.size() && std::isdigit((unsigned char)s_[p_])) t += s_[p_++];
    }
    return std::strtof(t.c_str(), nullptr);
  }
  bool peek_number() {
    char c = peekc();
    if (std::isdigit((unsigned char)c)) return true;
    if ((c == '-' || c == '+') && p_ + 1 < s_.size() && std::isdigit((unsigned char)s_[p_ + 1])) return true;
    return false;
  }
  int integ() {
    skip();
    size_t b = p_;
    while (p_ < s_.size() && std::isdigit((unsigned char)s_[p_])) ++p_;
    if (b == p_) fail("expected integer");
    return std::atoi(s_.substr(b, p_ - b).c_str());
  }
  std::string qstring() {
    skip();
    if (p_ >= s_.size() || s_[p_] != '"') fail("expected quoted string");
    ++p_;
    std::string r;
    while (p_ < s_.size() && s_[p_] != '"') {
      if (s_[p_] == '\\' && p_ + 1 < s_.size()) { r += s_[p_]; r += s_[p_ + 1]; p_ += 2; continue; }
      r += s_[p_++];
    }
    if (p_ >= s_.size()) fail("unterminated string");
    ++p_;
    return r;
  }
  int hexpair() {
    skip();
    if (p_ + 1 >= s_.size()) fail("expected hex digit");
    std::string h = s_.substr(p_, 2);
    p_ += 2;
    return (int)std::strtol(h.c_str(), nullptr, 16);
  }
  [[noreturn]] void fail(const std::string& m) {
    int line = 1;
    for (size_t i = 0; i < p_ && i < s_.size(); ++i) line += s_[i] == '\n';
    throw ParseError("line " + std::to_string(line) + ": " + m);
  }

 private:
  std::string s_;
  size_t p_ = 0;
};

// ---------------------------------------------------------------- scene under construction
struct Overrides {
  bool image = false; int w = 0, h = 0;
  bool strat = false; int nu = 0, nv = 0;
  bool random = false; int spp = 0;
  bool path = false; int md = 0, sd = 0;
  bool direct = false; int dmd = 0;
  bool force_path = false;
  bool filter = false; int fkind = 0; float fp[5] = {0, 0, 0, 0, 0};
  bool sppm = false; int sp_photons = 0, sp_md = 0; float sp_radius = 0.f, sp_alpha = 0.8f;
  int sppm_threads = 0;
};

struct Mat { bling_material m; };

struct PrimBlock {       // one `prim` statement: several primitives in order
  std::vector<std::pair<int, int>> prims;   // (kind, index)
};

struct LightRec { bling_light l; std::vector<float> func, cdf, fint, mfunc, mcdf, texels; };

struct Builder {
  // PState
  int resX = 640, resY = 480;
  bling_render_config cfg{};
  bling_filter filter{};
  bling_camera camera{};
  Xf xf = identityX();
  int material = 0;
  bool has_emit = false;
  Spec emit;
  int currId = 0;
  std::string base;
  Overrides ov;

  std::vector<float> verts;
  std::vector<uint32_t> tris;
  std::vector<int32_t> tri_mat;
  std::vector<float> tri_uv;
  std::vector<float> tri_n;
  std::vector<uint8_t> tri_hasn;
  std::vector<bling_shape> shapes;
  bling_fractal fractal{};
  std::vector<bling_material> materials;
  std::vector<bling_texture> textures;
  std::vector<bling_scalar_texture> scalar_textures;
  std::vector<PrimBlock> blocks;
  std::vector<std::unique_ptr<LightRec>> parsed_lights;  // in parse order
  std::vector<int> shape_light_shape;                    // shapes that carry emission
  std::vector<Spec> shape_light_rad;

  // final flattened arrays
  std::vector<int32_t> prim_kind, prim_index;
  std::vector<bling_light> lights;
  bling_scene_desc desc{};
  std::string summary;

  // texture images (bling_image): texel tables folded at parse time
  std::vector<std::vector<float>> image_data;
  std::vector<bling_image> images;
  std::map<std::pair<std::string, int>, int> image_index;   // (resolved path, channels) -> image

  std::string resolve(const std::string& fname) const {     // resolveFile (IO/ParserCore.hs:203-206)
    return (base.empty() || (!fname.empty() && fname[0] == '/')) ? fname : base + "/" + fname;
  }
  // readImageTextureMap / readImageScalarMap (Texture.hs:110-126): an RGB8 / RGBA8 / palette PNG as
  // pixelSpectrum texels (rgbToSpectrumRefl . unGamma of c / 255, Texture.hs:87-89; RGBA drops the
  // alpha: dropTransparency), a Y8 PNG as c / 255 scalars (getPixelScalar, :103-108)
  int add_image(const std::string& path, bool scalar) {
    const auto key = std::make_pair(path, scalar ? 1 : 16);
    auto it = image_index.find(key);
    if (it != image_index.end()) return it->second;
    const bimg::Decoded im = bimg::read_image(path);
    const size_t n = (size_t)im.width * im.height;
    std::vector<float> tx;
    if (scalar) {
      if (im.is_float || im.channels != 1) throw ParseError(path + ": unsupported image type (a scalar image texture needs a greyscale PNG)");
      tx.resize(n);
      for (size_t i = 0; i < n; ++i) tx[i] = (float)im.bytes[i] / 255.f;
    } else {
      if (im.is_float || (im.channels != 3 && im.channels != 4))
        throw ParseError(path + ": unsupported image type (an image texture needs an RGB / RGBA / palette PNG)");
      float lut[256];                                        // unGamma: (c / 255) ** 2.2
      for (int c = 0; c < 256; ++c) lut[c] = bcr::powf((float)c / 255.f, 2.2f);
      tx.resize(n * 16);
      for (size_t i = 0; i < n; ++i) {
        const uint8_t* px = &im.bytes[i * im.channels];
        const Spec sp = rgb_to_spectrum(BLING_RGB_REFL_BANDS, lut[px[0]], lut[px[1]], lut[px[2]]);
        std::copy(sp.begin(), sp.end(), tx.begin() + i * 16);
      }
    }
    bling_image bi{};
    bi.width = im.width; bi.height = im.height; bi.channels = scalar ? 1 : 16;
    image_data.push_back(std::move(tx));
    images.push_back(bi);
    image_index[key] = (int)images.size() - 1;
    return (int)images.size() - 1;
  }

  int add_texture_const(const Spec& s) {
    bling_texture t{};
    t.kind = BLING_TEX_CONST; t.tex1 = t.tex2 = -1;
    for (int i = 0; i < 16; ++i) t.value[i] = s[i];
    textures.push_back(t);
    return (int)textures.size() - 1;
  }

  Builder() {
    // startState (IO/RenderJob.hs:20-29): 640x480, default renderer, box filter, default camera
    cfg.renderer = BLING_RENDERER_SAMPLER_PATH;
    cfg.sampler = BLING_SAMPLER_STRATIFIED; cfg.nu = 2; cfg.nv = 2; cfg.spp = 4;   // RendererParser.hs:20-21
    cfg.max_depth = 7; cfg.sample_depth = 3;                                       // IntegratorParser.hs:13-14
    float none[5] = {0, 0, 0, 0, 0};
    build_filter(filter, BLING_FILTER_BOX, none);
    make_camera(translateX(v3(0, 0, -5)), 0.f, 1.f, 90.f, 640.f, 480.f);           // CameraParser.hs:14-17
    // defaultMaterial (MaterialParser.hs:21-22)
    bling_material m{};
    m.kind = BLING_MAT_MATTE;
    m.tex[0] = add_texture_const(rgb_to_spectrum(BLING_RGB_REFL_BANDS, 0.9f, 0.9f, 0.9f));
    m.tex[1] = m.tex[2] = m.tex[3] = -1;
    m.stex[0] = m.stex[1] = m.stex[2] = m.stex[3] = -1;
    m.scalar[0] = 0.f;
    materials.push_back(m);
    material = 0;
  }

  // mkPerspectiveCamera / mkProjective (Camera.hs:108-147)
  void make_camera(const Xf& c2w, float lr, float fd, float fov, float sx, float sy) {
    Xf p = perspectiveX(fov, 1e-2f, 1000.f);
    float aspect = sx / sy;
    float s0, s1, s2, s3;
    if (aspect > 1.f) { s0 = -aspect; s1 = aspect; s2 = -1.f; s3 = 1.f; }
    else { s0 = -1.f; s1 = 1.f; s2 = -1.f / aspect; s3 = 1.f / aspect; }
    Xf st1 = scaleX(v3(sx, sy, 1.f));
    Xf st2 = scaleX(v3(1.f / (s1 - s0), 1.f / (s2 - s3), 1.f));
    Xf t = translateX(v3(-s0, -s3, 0.f));
    Xf s2r = cat(t, cat(st2, st1));       // t <> st2 <> st1 (infixr)
    Xf r2s = inverseX(s2r);
    Xf r2c = cat(r2s, inverseX(p));
    camera.kind = BLING_CAM_PERSPECTIVE;
    std::memcpy(camera.c2w, c2w.m.m, 64); std::memcpy(camera.c2w_inv, c2w.inv.m, 64);
    std::memcpy(camera.r2c, r2c.m.m, 64); std::memcpy(camera.r2c_inv, r2c.inv.m, 64);
    camera.lens_radius = lr; camera.focal_distance = fd;
    camera.xres = sx; camera.yres = sy;
  }
};

// ---------------------------------------------------------------- grammar
struct Parser {
  Lexer& L;
  Builder& B;

  template <class F> void block(F f) { L.expect('{'); f(); L.expect('}'); }      // pBlock
  template <class F> void named_block(const char* n, F f) { L.expect_word(n); block(f); }

  Spec spectrum() {                                     // pSpectrum (IO/ParserCore.hs:139-147)
    std::string t = L.word();
    if (t == "rgbR" || t == "rgbI") {
      float r, g, b;
      if (L.accept('%')) { r = L.hexpair() / 255.f; g = L.hexpair() / 255.f; b = L.hexpair() / 255.f; }
      else { r = L.flt(); g = L.flt(); b = L.flt(); }
      return rgb_to_spectrum(t == "rgbR" ? BLING_RGB_REFL_BANDS : BLING_RGB_ILLUM_BANDS, r, g, b);
    }
    if (t == "spd") {                                   // pSpectrumSpd: sepBy1 (l v) ','
      std::vector<std::pair<float, float>> pts;
      block([&] {
        do { float l = L.flt(); float v = L.flt(); pts.emplace_back(l, v); } while (L.accept(','));
      });
      return from_irregular(pts);
    }
    if (t == "temp") return black_body(L.flt());
    L.fail("unknown spectrum type " + t);
  }

  Xf transform_block() {                                // pTransform (IO/TransformParser.hs:21-26)
    std::vector<Xf> ts;
    block([&] {
      while (L.peekc() != '}') ts.push_back(any_transform());
    });
    Xf acc = identityX();                               // mconcat = foldr (<>) mempty
    for (int i = (int)ts.size() - 1; i >= 0; --i) acc = cat(ts[i], acc);
    return acc;
  }
  V3 vec() { float x = L.flt(); float y = L.flt(); float z = L.flt(); return v3(x, y, z); }
  V3 named_vec(const char* n) { L.expect_word(n); return vec(); }
  float named_float(const char* n) { L.expect_word(n); return L.flt(); }
  int named_int(const char* n) { L.expect_word(n); return L.integ(); }

  Xf any_transform() {
    std::string w = L.word();
    if (w == "rotateX") return rotateXX(L.flt());
    if (w == "rotateY") return rotateYX(L.flt());
    if (w == "rotateZ") return rotateZX(L.flt());
    if (w == "scale") return scaleX(vec());
    if (w == "translate") return translateX(vec());
    if (w == "identity") return identityX();
    if (w == "lookAt") {
      Xf r;
      block([&] { V3 p = named_vec("pos"); V3 l = named_vec("look"); V3 u = named_vec("up"); r = lookAtX(p, l, u); });
      return r;
    }
    if (w == "matrix") {
      M4 m;
      block([&] {
        for (int r = 0; r < 4; ++r) { L.expect_word("m"); for (int c = 0; c < 4; ++c) m.m[r * 4 + c] = L.flt(); }
      });
      return fromMatrixX(m);
    }
    L.fail("unknown transform " + w);
  }

  // pTextureMapping2d (MaterialParser.hs:160-178): only uv is needed by the benchmark scenes
  void uv_mapping(bling_texture& t) {
    named_block("map", [&] {
      std::string n = L.word();
      if (n != "uv") L.fail("unsupported 2d mapping " + n);
      t.uv_map[0] = L.flt(); t.uv_map[1] = L.flt(); t.uv_map[2] = L.flt(); t.uv_map[3] = L.flt();
    });
  }

  // pTextureMapping2d "map" (MaterialParser.hs:160-178): uv su sv ou ov -> p[0..3]; planar vu vv ou ov
  // -> p[0..7] (vu xyz, vv xyz, ou, ov); returns the bling_map2d kind
  int mapping2d(float* p) {
    int kind = BLING_MAP_UV;
    named_block("map", [&] {
      const std::string n = L.word();
      if (n == "planar") {
        kind = BLING_MAP_PLANAR;
        const V3 vu = vec(), vv = vec();
        p[0] = vu.x; p[1] = vu.y; p[2] = vu.z; p[3] = vv.x; p[4] = vv.y; p[5] = vv.z;
        p[6] = L.flt(); p[7] = L.flt();
      } else if (n == "uv") {
        for (int k = 0; k < 4; ++k) p[k] = L.flt();
      } else {
        L.fail("unknown 2d mapping " + n);
      }
    });
    return kind;
  }
  // pImageTexture / pImageScalar (MaterialParser.hs:106-113, 189-196): file "<name>" map { ... };
  // the image is read when its name is parsed (readFileBS' of resolveFile)
  int image_file(bool scalar) {
    L.expect_word("file");
    const std::string fn = L.qstring();
    try {
      return B.add_image(B.resolve(fn), scalar);
    } catch (const std::exception& e) {
      L.fail(e.what());
    }
  }

  int spectrum_texture(const char* name) {              // pSpectrumTexture (MaterialParser.hs:198-226)
    int idx = -1;
    named_block(name, [&] {
      std::string tp = L.word();
      if (tp == "constant") { idx = B.add_texture_const(spectrum()); return; }
      if (tp == "image") {                               // pBlock pImageTexture
        bling_texture t{};
        t.kind = BLING_TEX_IMAGE;
        block([&] {
          t.tex1 = image_file(false);
          float mp[8] = {0, 0, 0, 0, 0, 0, 0, 0};
          t.tex2 = mapping2d(mp);
          if (t.tex2 == BLING_MAP_UV) for (int k = 0; k < 4; ++k) t.uv_map[k] = mp[k];
          else for (int k = 0; k < 8; ++k) t.value[k] = mp[k];
        });
        B.textures.push_back(t);
        idx = (int)B.textures.size() - 1;
        return;
      }
      if (tp == "graphPaper") {
        bling_texture t{};
        t.kind = BLING_TEX_GRAPHPAPER;
        t.line_width = L.flt();
        uv_mapping(t);                                   // mandatory `map` (trap T3)
        t.tex1 = simple_child(spectrum_texture("tex1"));
        t.tex2 = simple_child(spectrum_texture("tex2"));
        B.textures.push_back(t);
        idx = (int)B.textures.size() - 1;
        return;
      }
      if (tp == "blend") {                               // spectrumBlend <$> tex1 <*> tex2 <*> f
        bling_texture t{};
        t.kind = BLING_TEX_BLEND;
        t.tex1 = simple_child(spectrum_texture("tex1"));
        t.tex2 = simple_child(spectrum_texture("tex2"));
        t.stex = scalar_texture_index("f");
        B.textures.push_back(t);
        idx = (int)B.textures.size() - 1;
        return;
      }
      if (tp == "checker") {                             // checkerBoard <$> pVec <*> tex1 <*> tex2
        bling_texture t{};
        t.kind = BLING_TEX_CHECKER;
        const V3 s = vec();
        t.uv_map[0] = s.x; t.uv_map[1] = s.y; t.uv_map[2] = s.z;
        t.tex1 = simple_child(spectrum_texture("tex1"));
        t.tex2 = simple_child(spectrum_texture("tex2"));
        B.textures.push_back(t);
        idx = (int)B.textures.size() - 1;
        return;
      }
      if (tp == "gradient") {                            // gradient (mkGradient steps) f (MaterialParser.hs:211-218)
        const int f = scalar_texture_index("f");
        std::vector<std::pair<float, Spec>> steps;       // sepBy (pos, pSpectrum) ','
        named_block("steps", [&] {
          if (L.peekc() == '}') return;
          do { const float pos = L.flt(); steps.emplace_back(pos, spectrum()); } while (L.accept(','));
        });
        if (steps.empty()) L.fail("empty list given to mkGradient");
        std::stable_sort(steps.begin(), steps.end(),     // sortBy (compare `on` fst): stable
                         [](const auto& a, const auto& b) { return a.first < b.first; });
        bling_texture t{};
        t.kind = BLING_TEX_GRADIENT;
        t.stex = f;
        t.tex1 = (int)B.textures.size() + 1;             // the steps follow the gradient record
        t.tex2 = (int)steps.size();
        B.textures.push_back(t);
        idx = (int)B.textures.size() - 1;
        for (const auto& s : steps) {
          const int k = B.add_texture_const(s.second);
          B.textures[k].line_width = s.first;
        }
        return;
      }
      L.fail("unsupported spectrum texture " + tp);
    });
    return idx;
  }

  // children of graphPaper / blend / checker: the device resolves them to a stored spectrum
  // (constant, or a graphPaper chain of constants); a computed texture below another is refused
  int simple_child(int ti) {
    if (B.textures[ti].kind >= BLING_TEX_BLEND)
      L.fail("blend / gradient / checker / image textures are supported at the top of a material's texture only");
    return ti;
  }
  // a scalar texture as a bling_scalar_texture index (a constant becomes a CONST record)
  int scalar_texture_index(const char* name) {
    float cv = 0.f;
    int c = scalar_texture_any(name, &cv);
    if (c < 0) { bling_scalar_texture k{}; k.kind = BLING_STEX_CONST; k.value = cv; B.scalar_textures.push_back(k); c = (int)B.scalar_textures.size() - 1; }
    return c;
  }

  float scalar_texture(const char* name) {              // pScalarTexture where a material folds a constant
    float v = 0;
    if (scalar_texture_any(name, &v) >= 0) L.fail(std::string(name) + ": only constant scalar textures are supported here");
    return v;
  }

  // pScalarTexture (MaterialParser.hs:115-156): returns -1 and the value for `constant`, else the
  // index of a bling_scalar_texture evaluated at the hit (scale / fbm / perlin)
  int scalar_texture_any(const char* name, float* cval) {
    int idx = -1;
    named_block(name, [&] { idx = scalar_texture_body(cval); });
    return idx;
  }
  int stex_scale_depth = 0;     // nesting of `scale` scalar textures (BLING_STEX_MAX_SCALE)
  int scalar_texture_body(float* cval) {
    std::string tp = L.word();
    bling_scalar_texture t{};
    if (tp == "constant") { *cval = L.flt(); return -1; }
    if (tp == "image") {                                  // pBlock pImageScalar
      t.kind = BLING_STEX_IMAGE;
      block([&] {
        t.child = image_file(true);
        t.octaves = mapping2d(t.w2t);
      });
      B.scalar_textures.push_back(t);
      return (int)B.scalar_textures.size() - 1;
    }
    if (tp == "scale") {                                  // scaleTexture a s (tex)
      t.kind = BLING_STEX_SCALE; t.a = L.flt(); t.s = L.flt();
      if (++stex_scale_depth > BLING_STEX_MAX_SCALE)
        L.fail("scalar texture: more than " + std::to_string(BLING_STEX_MAX_SCALE) + " nested `scale` textures");
      float cv = 0.f;
      int c = scalar_texture_any("tex", &cv);
      --stex_scale_depth;
      if (c < 0) { bling_scalar_texture k{}; k.kind = BLING_STEX_CONST; k.value = cv; B.scalar_textures.push_back(k); c = (int)B.scalar_textures.size() - 1; }
      t.child = c;
    } else if (tp == "crystal") {                        // quasiCrystal o (pTextureMapping2d "map")
      t.kind = BLING_STEX_CRYSTAL;
      t.octaves = named_int("octaves");
      if (t.octaves < 1 || t.octaves > 64) L.fail("crystal: octaves must lie in [1, 64]");
      named_block("map", [&] {
        const std::string n = L.word();
        if (n != "planar") L.fail("crystal: only the planar 2d mapping is supported, got " + n);
        const V3 vu = vec(), vv = vec();                  // planarMapping (vu, vv) (ou, ov)
        t.w2t[0] = vu.x; t.w2t[1] = vu.y; t.w2t[2] = vu.z;
        t.w2t[3] = vv.x; t.w2t[4] = vv.y; t.w2t[5] = vv.z;
        t.w2t[6] = L.flt(); t.w2t[7] = L.flt();
      });
      // angles o = take o $ enumFromThen 0 (pi / fromIntegral o): GHC's numericEnumFromThen n m =
      // n : numericEnumFromThen m (m + m - n); each wave's (cos th, sin th) as libm's binary32
      const float step = 3.14159265358979323846f / (float)t.octaves;
      float a0 = 0.f, a1 = step;
      t.child = (int)B.scalar_textures.size() + 1;        // the angle records follow this one
      B.scalar_textures.push_back(t);
      const int self = (int)B.scalar_textures.size() - 1;
      for (int k = 0; k < t.octaves; ++k) {
        bling_scalar_texture w{};
        w.kind = BLING_STEX_CONST;
        w.a = std::cos(a0); w.s = std::sin(a0);
        B.scalar_textures.push_back(w);
        const float a2 = (a1 + a1) - a0;
        a0 = a1; a1 = a2;
      }
      return self;
    } else if (tp == "fbm" || tp == "perlin" || tp == "cellNoise") {
      if (tp == "fbm") { t.kind = BLING_STEX_FBM; t.octaves = named_int("octaves"); t.omega = named_float("omega"); }   // pFbmMap
      else if (tp == "perlin") t.kind = BLING_STEX_PERLIN;
      else {                                              // cellNoise <distance> (MaterialParser.hs:124-133)
        t.kind = BLING_STEX_CELLNOISE;
        const std::string dn = L.word();
        if (dn == "euclidian") t.octaves = BLING_CELL_EUCLIDIAN;
        else if (dn == "euclidian2") t.octaves = BLING_CELL_EUCLIDIAN2;
        else if (dn == "manhattan") t.octaves = BLING_CELL_MANHATTAN;
        else if (dn == "chebyshev") t.octaves = BLING_CELL_CHEBYSHEV;
        else L.fail("unknown distance function " + dn);
      }
      named_block("map", [&] {                            // pTextureMapping3d: identity <transform>
        L.expect_word("identity");
        Xf x = transform_block();
        std::memcpy(t.w2t, x.m.m, 64);                    // identityMapping3d w2t: transPoint w2t p
      });
    } else {
      L.fail("unsupported scalar texture " + tp);
    }
    B.scalar_textures.push_back(t);
    return (int)B.scalar_textures.size() - 1;
  }

  // value of a constant spectrum texture; materials whose BxDF spectra are folded on the host
  // (transMatte, shinyMetal) accept constant textures only
  Spec const_texture(int ti, const char* what) {
    const bling_texture& tx = B.textures[ti];
    if (tx.kind != BLING_TEX_CONST) L.fail(std::string(what) + ": only constant textures are supported");
    Spec s(16);
    for (int i = 0; i < 16; ++i) s[i] = tx.value[i];
    return s;
  }
  static Spec sclamp(Spec s, float lo, float hi) {     // sClamp (Spectrum.hs:453-456): max lo (min hi x)
    for (int i = 0; i < 16; ++i) { float x = s[i] <= hi ? s[i] : hi; s[i] = lo <= x ? x : lo; }
    return s;
  }
  static Spec fr_approx_eta(const Spec& r) {           // frApproxEta (Fresnel.hs:72-74)
    Spec c = sclamp(r, 0.f, 0.999f), o(16);
    for (int i = 0; i < 16; ++i) { float q = std::sqrt(c[i]); o[i] = (1.f + q) / (1.f - q); }
    return o;
  }
  static Spec fr_approx_k(const Spec& r) {             // frApproxK (Fresnel.hs:76-78)
    Spec c = sclamp(r, 0.f, 0.999f), o(16);
    for (int i = 0; i < 16; ++i) o[i] = std::sqrt(c[i] / (1.f - c[i])) * 2.f;
    return o;
  }

  int material_body() {                                 // pMaterial' (MaterialParser.hs:30-42)
    std::string t = L.word();
    bling_material m{};
    m.tex[0] = m.tex[1] = m.tex[2] = m.tex[3] = -1;
    m.stex[0] = m.stex[1] = m.stex[2] = m.stex[3] = -1;
    if (t == "matte") { m.kind = BLING_MAT_MATTE; m.tex[0] = spectrum_texture("kd"); m.scalar[0] = scalar_texture("sigma"); }
    else if (t == "plastic") { m.kind = BLING_MAT_PLASTIC; m.tex[0] = spectrum_texture("kd"); m.tex[1] = spectrum_texture("ks"); m.scalar[0] = scalar_texture("rough"); }
    else if (t == "glass") { m.kind = BLING_MAT_GLASS; m.scalar[0] = scalar_texture("ior"); m.tex[0] = spectrum_texture("kr"); m.tex[1] = spectrum_texture("kt"); }
    else if (t == "metal") { m.kind = BLING_MAT_METAL; m.tex[0] = spectrum_texture("eta"); m.tex[1] = spectrum_texture("k"); m.scalar[0] = scalar_texture("rough"); }
    else if (t == "mirror") { m.kind = BLING_MAT_MIRROR; m.tex[0] = spectrum_texture("kr"); }
    else if (t == "blackbody") { m.kind = BLING_MAT_BLACKBODY; }
    else if (t == "transMatte") {                          // pMatteTranslucent / translucentMatte
      int kr = spectrum_texture("kr"), kt = spectrum_texture("kt");
      m.scalar[0] = scalar_texture("ks");
      Spec r = sclamp(const_texture(kr, "transMatte kr"), 0.f, 1.f);      // sClamp 0 1 (kr dgs)
      Spec tt = sclamp(const_texture(kt, "transMatte kt"), 0.f, 1.f);
      Spec tr(16);
      for (int i = 0; i < 16; ++i) tr[i] = tt[i] * (1.f - r[i]);          // sClamp 0 1 kt * (white - r)
      m.kind = BLING_MAT_TRANSMATTE;
      m.tex[0] = B.add_texture_const(r);
      m.tex[1] = B.add_texture_const(tr);
    } else if (t == "shinyMetal") {                        // pShinyMetal / mkShinyMetal
      int kr = spectrum_texture("kr"), ks = spectrum_texture("ks");
      m.scalar[0] = scalar_texture("rough");
      Spec r = const_texture(kr, "shinyMetal kr"), s = const_texture(ks, "shinyMetal ks");
      m.kind = BLING_MAT_SHINYMETAL;
      m.tex[0] = B.add_texture_const(fr_approx_eta(s)); m.tex[1] = B.add_texture_const(fr_approx_k(s));
      m.tex[2] = B.add_texture_const(fr_approx_eta(r)); m.tex[3] = B.add_texture_const(fr_approx_k(r));
    }
    else if (t == "substrate") {                          // pSubstrateMaterial / mkSubstrate (Material.hs:111-128)
      int kd = spectrum_texture("kd"), ks = spectrum_texture("ks"), ka = spectrum_texture("ka");
      float ur = 0.f, vr = 0.f, depth = 0.f;
      m.stex[0] = scalar_texture_any("urough", &ur);
      m.stex[1] = scalar_texture_any("vrough", &vr);
      m.stex[2] = scalar_texture_any("depth", &depth);
      auto fix_exponent = [](float e) { return (e > 10000.f || std::isnan(e)) ? 10000.f : e; };   // Microfacet.hs:128-130
      auto max0 = [](float x) { return 0.f <= x ? x : 0.f; };                                  // max 0 (GHC max)
      m.kind = BLING_MAT_SUBSTRATE;
      m.tex[0] = B.add_texture_const(sclamp(const_texture(kd, "substrate kd"), 0.f, 1.f));
      m.tex[1] = B.add_texture_const(sclamp(const_texture(ks, "substrate ks"), 0.f, 1.f));
      m.tex[2] = B.add_texture_const(sclamp(const_texture(ka, "substrate ka"), 0.f, 1.f));
      m.scalar[0] = fix_exponent(1.f / max0(ur));          // mkAnisotropic (1 / u) (1 / v)
      m.scalar[1] = fix_exponent(1.f / max0(vr));
      m.scalar[2] = depth;
    }
    else if (t == "bumpMap") {                            // pBumpMap / bumpMapped (Reflection.hs:344-345)
      float cv = 0.f;
      int d = scalar_texture_any("bump", &cv);
      if (d < 0) { bling_scalar_texture k{}; k.kind = BLING_STEX_CONST; k.value = cv; B.scalar_textures.push_back(k); d = (int)B.scalar_textures.size() - 1; }
      int inner = material_body();
      if (B.materials[inner].stex[3] >= 0) L.fail("bumpMap of a bumpMap is not supported");
      B.materials[inner].stex[3] = d;
      return inner;
    }
    else L.fail("unsupported material " + t);
    B.materials.push_back(m);
    return (int)B.materials.size() - 1;
  }

  void shape_prim(PrimBlock& pb) {                      // "shape" -> mkGeom (PrimitiveParser.hs:63-67)
    bling_shape s{};
    block([&] {
      std::string t = L.word();
      auto radians = [](float deg) { return deg / 180.f * 3.14159265358979f; };      // Math.hs:62-66
      auto clampd = [](float v) { return v < 0.f ? 0.f : (v > 360.f ? 360.f : v); };
      if (t == "quad") { s.kind = BLING_SHAPE_QUAD; s.params[0] = L.flt(); s.params[1] = L.flt(); }
      else if (t == "sphere") { s.kind = BLING_SHAPE_SPHERE; s.params[0] = named_float("radius"); }
      else if (t == "box") {                                     // mkBox (Shape.hs:41-44)
        V3 a = named_vec("pmin"), b = named_vec("pmax");
        s.kind = BLING_SHAPE_BOX;
        s.params[0] = std::min(a.x, b.x); s.params[1] = std::min(a.y, b.y); s.params[2] = std::min(a.z, b.z);
        s.params[3] = std::max(a.x, b.x); s.params[4] = std::max(a.y, b.y); s.params[5] = std::max(a.z, b.z);
      } else if (t == "cylinder") {                              // mkCylinder (Shape.hs:47-56)
        float r = named_float("radius"), z0 = named_float("zmin"), z1 = named_float("zmax"), pm = named_float("phiMax");
        s.kind = BLING_SHAPE_CYLINDER;
        s.params[0] = r; s.params[1] = std::min(z0, z1); s.params[2] = std::max(z0, z1); s.params[3] = radians(clampd(pm));
      } else if (t == "disk") {                                  // mkDisk (Shape.hs:59-68)
        float h = named_float("height"), r0 = named_float("radius"), r1 = named_float("innerRadius"), pm = named_float("phiMax");
        s.kind = BLING_SHAPE_DISK;
        s.params[0] = h; s.params[1] = std::max(r0, r1); s.params[2] = std::min(r0, r1); s.params[3] = radians(clampd(pm));
      }
      else L.fail("unsupported shape " + t);
    });
    s.material = B.material;
    s.shape_id = B.currId++;                            // nextId
    std::memcpy(s.o2w, B.xf.m.m, 64);
    std::memcpy(s.w2o, B.xf.inv.m, 64);
    s.light = -1;
    int si = (int)B.shapes.size();
    if (B.has_emit) { B.shape_light_shape.push_back(si); B.shape_light_rad.push_back(B.emit); s.light = -2; }
    B.shapes.push_back(s);
    pb.prims.emplace_back(1, si);
  }

  void add_triangle(const V3* p, int mat, const float* uv, const V3* n) {
    uint32_t base = (uint32_t)(B.verts.size() / 3);
    for (int k = 0; k < 3; ++k) { B.verts.push_back(p[k].x); B.verts.push_back(p[k].y); B.verts.push_back(p[k].z); }
    B.tris.push_back(base); B.tris.push_back(base + 1); B.tris.push_back(base + 2);
    B.tri_mat.push_back(mat);
    for (int k = 0; k < 6; ++k) B.tri_uv.push_back(uv[k]);
    for (int k = 0; k < 3; ++k) {
      B.tri_n.push_back(n ? n[k].x : 0.f); B.tri_n.push_back(n ? n[k].y : 0.f); B.tri_n.push_back(n ? n[k].z : 0.f);
    }
    B.tri_hasn.push_back(n ? 1 : 0);
  }

  void mesh_prim(PrimBlock& pb) {                       // pMesh (PrimitiveParser.hs:130-138)
    int vc = named_int("vertexCount");
    int fc = named_int("faceCount");
    std::vector<V3> vs;
    for (int i = 0; i < vc; ++i) { L.expect_word("v"); vs.push_back(vec()); }
    std::vector<int> idx;
    for (int f = 0; f < fc; ++f) {
      L.expect_word("f");
      std::vector<int> face;
      while (std::isdigit((unsigned char)L.peekc())) face.push_back(L.integ());
      // triangulate (TriangleMesh.hs:23-29): fan (f0, f1, f2), (f0, f2, f3), ...
      for (size_t k = 1; k + 1 < face.size(); ++k) { idx.push_back(face[0]); idx.push_back(face[k]); idx.push_back(face[k + 1]); }
    }
    for (int i : idx) if (i < 0 || i >= vc) L.fail("mesh index out of bounds");
    static const float defuv[6] = {0, 0, 1, 0, 1, 1};   // triangleDefaultUVs (TriangleMesh.hs:119-120)
    for (size_t t = 0; t < idx.size() / 3; ++t) {
      V3 p[3];
      for (int k = 0; k < 3; ++k) p[k] = xpoint(B.xf.m, vs[idx[3 * t + k]]);   // p' = transPoint o2w
      add_triangle(p, B.material, defuv, nullptr);
      pb.prims.emplace_back(0, (int)B.tri_mat.size() - 1);
    }
  }

  void wavefront_prim(PrimBlock& pb) {                  // "waveFront" (PrimitiveParser.hs:69-72)
    std::string fname = L.qstring();
    std::map<std::string, int> mmap;                    // pNamedMaterialMap
    named_block("materials", [&] {
      while (L.peekc() == '"') {
        std::string n = L.qstring();
        int m = -1;
        block([&] { m = material_body(); });
        mmap[n] = m;
      }
    });
    int defmat = B.material;
    auto lookup = [&](const std::string& n) { auto it = mmap.find(n); return it == mmap.end() ? defmat : it->second; };
    std::string path = B.base.empty() ? fname : B.base + "/" + fname;
    std::ifstream in(path);
    if (!in) L.fail("cannot read " + path);
    // waveFrontParser (IO/WaveFront.hs:118-211)
    std::vector<V3> ps, ns;
    std::vector<std::pair<float, float>> uvs;
    std::vector<int> fv, fuv, fn;                       // per face-VERTEX entry
    std::vector<std::pair<std::string, int>> mtls;      // (name, #face-vertex entries so far)
    std::string line;
    while (std::getline(in, line)) {
      if (line.rfind("vn", 0) == 0) {
        std::istringstream ss(line.substr(2)); float x, y, z; ss >> x >> y >> z;
        ns.push_back(normalize(v3(x, y, z)));
      } else if (line.rfind("vt", 0) == 0) {
        std::istringstream ss(line.substr(2)); float u = 0, v = 1; ss >> u; if (!(ss >> v)) v = 1;
        uvs.emplace_back(u, v);
      } else if (line.rfind("v ", 0) == 0) {
        std::istringstream ss(line.substr(1)); float x, y, z; ss >> x >> y >> z;
        ps.push_back(v3(x, y, z));
      } else if (line.rfind("f ", 0) == 0) {
        std::istringstream ss(line.substr(1));
        std::string tok;
        std::vector<int> a, b, c;
        while (ss >> tok) {
          int vi = 0, ti = 0, ni = 0;
          size_t s1 = tok.find('/');
          vi = std::atoi(tok.substr(0, s1).c_str());
          if (s1 != std::string::npos) {
            size_t s2 = tok.find('/', s1 + 1);
            std::string ts = tok.substr(s1 + 1, s2 == std::string::npos ? std::string::npos : s2 - s1 - 1);
            ti = ts.empty() ? 0 : std::atoi(ts.c_str());
            if (s2 != std::string::npos) ni = std::atoi(tok.substr(s2 + 1).c_str());
          }
          a.push_back(vi - 1); b.push_back(ti - 1); c.push_back(ni - 1);   // pred
        }
        for (size_t k = 1; k + 1 < a.size(); ++k) {
          size_t o[3] = {0, k, k + 1};
          for (int q = 0; q < 3; ++q) { fv.push_back(a[o[q]]); fuv.push_back(b[o[q]]); fn.push_back(c[o[q]]); }
        }
      } else if (line.rfind("usemtl", 0) == 0) {
        mtls.emplace_back(line.size() > 7 ? line.substr(7) : std::string(), (int)fv.size());
      }
    }
    std::vector<V3> pst;
    for (auto& p : ps) pst.push_back(xpoint(B.xf.m, p));   // pst = transPoint trans (normals untouched)
    // matIntervals (IO/WaveFront.hs:93-97): starts are in face-VERTEX entries but the final end is
    // the TRIANGLE count, so the last material run is dropped (trap T15, kept on purpose).
    int cnt = (int)fv.size() / 3;
    std::vector<std::pair<std::string, int>> starts = {{"default", 0}};
    for (auto& m : mtls) starts.push_back(m);
    std::vector<int> ends;
    for (auto& m : mtls) ends.push_back(m.second);
    ends.push_back(cnt);
    for (size_t k = 0; k < starts.size(); ++k) {
      int s = starts[k].second, l = ends[k] - s;
      if (l <= 0) continue;
      int mat = lookup(starts[k].first);
      for (int i = s; i <= s + l - 1; i += 3) {
        V3 p[3] = {pst[fv[i]], pst[fv[i + 1]], pst[fv[i + 2]]};
        // wfTriUVs: the THIRD uv index repeats entry i+1 (trap T9)
        int i1 = fuv[i], i2 = fuv[i + 1], i3 = fuv[i + 1];
        float uv[6];
        if (i1 >= 0 && i2 >= 0 && i3 >= 0) {
          uv[0] = uvs[i1].first; uv[1] = uvs[i1].second; uv[2] = uvs[i2].first; uv[3] = uvs[i2].second;
          uv[4] = uvs[i3].first; uv[5] = uvs[i3].second;
        } else { const float d[6] = {0, 0, 1, 0, 1, 1}; std::memcpy(uv, d, sizeof uv); }
        int n1 = fn[i], n2 = fn[i + 1], n3 = fn[i + 1];
        if (n1 < 0 && n2 < 0 && n3 < 0) add_triangle(p, mat, uv, nullptr);
        else {
          if (n1 < 0 || n2 < 0 || (size_t)n1 >= ns.size() || (size_t)n2 >= ns.size()) L.fail("bad normal index");
          V3 nn[3] = {ns[n1], ns[n2], ns[n3]};
          add_triangle(p, mat, uv, nn);
        }
        pb.prims.emplace_back(0, (int)B.tri_mat.size() - 1);
      }
    }
  }

  std::unique_ptr<ScalarMap2d> scalar_map2d() {        // pScalarMap2d (MaterialParser.hs:232-245)
    auto m = std::make_unique<ScalarMap2d>();
    block([&] {
      std::string t = L.word();
      if (t == "fbm") {
        m->kind = 0; m->z = L.flt();
        m->octaves = named_int("octaves"); m->omega = named_float("omega");         // pFbmMap
      } else if (t == "scale") {
        m->kind = 1; m->f = L.flt(); m->child = scalar_map2d();
      } else L.fail("unknown scalar map type" + t);
    });
    return m;
  }

  // heightMap (Primitive/Heightmap.hs:15-50) as a triangle mesh (mkTriangleMesh, TriangleMesh.hs:38-57)
  void heightmap_prim(PrimBlock& pb) {
    int ns = L.integ(), nt = L.integ();
    std::unique_ptr<ScalarMap2d> elev = scalar_map2d();
    Xf tr = transform_block();                           // the heightMap's own o2w, not the state's
    if (ns < 2 || nt < 2) L.fail("heightMap needs at least 2 x 2 samples");
    const float fns = (float)ns, fnt = (float)nt;
    const float ex = 1.f / fns, ez = 1.f / fnt;
    std::vector<V3> ps, nrm;
    std::vector<float> uv;
    for (int zi = 0; zi < nt; ++zi)
      for (int xi = 0; xi < ns; ++xi) {
        float x = (float)xi / (fns - 1.f), z = (float)zi / (fnt - 1.f);
        ps.push_back(xpoint(tr.m, v3(x, elev->eval(x, z), z)));
        float dx = elev->eval(x - ex, z) - elev->eval(x + ex, z);
        float dz = elev->eval(x, z - ez) - elev->eval(x, z + ez);
        V3 n = normalize(v3(dx, ex + ez, dz));
        nrm.push_back(xnormal(tr.inv, v3(-n.x, -n.y, -n.z)));   // transNormal o2w (- normalize v)
        uv.push_back(x / (fns - 1.f)); uv.push_back(z / (fns - 1.f));   // z / (fns - 1): as written
      }
    auto vert = [&](int x, int y) { return x + y * ns; };
    auto tri = [&](int a, int b, int c) {
      V3 p[3] = {ps[a], ps[b], ps[c]}, n[3] = {nrm[a], nrm[b], nrm[c]};
      float t[6] = {uv[2 * a], uv[2 * a + 1], uv[2 * b], uv[2 * b + 1], uv[2 * c], uv[2 * c + 1]};
      add_triangle(p, B.material, t, n);
      pb.prims.emplace_back(0, (int)B.tri_mat.size() - 1);
    };
    for (int y = 0; y <= nt - 2; ++y)
      for (int x = 0; x <= ns - 2; ++x) {
        tri(vert(x, y), vert(x + 1, y), vert(x + 1, y + 1));
        tri(vert(x, y), vert(x + 1, y + 1), vert(x, y + 1));
      }
  }

  // bezier (PrimitiveParser.hs:32-37, 121-128): bicubic patches of 48 floats tessellated into one
  // triangle mesh with shading normals dpdu x dpdv and uvs (tesselateBezier, Primitive/Bezier.hs:75-105).
  // Every sum and product keeps GHC's left-to-right order (sum = foldl (+) 0).
  static float bern(float u, int x) {                   // bernstein (Bezier.hs:27-35)
    float i = 1.f - u;
    switch (x) {
      case 0: return 1.f * i * i * i;
      case 1: return 3.f * u * i * i;
      case 2: return 3.f * u * u * i;
      default: return 1.f * u * u * u;
    }
  }
  static float bern_d(float u, int x) {                 // bernsteinDeriv (Bezier.hs:39-47)
    float i = 1.f - u;
    switch (x) {
      case 0: return 3.f * -(i * i);
      case 1: return 3.f * (i * i - 2.f * u * i);
      case 2: return 3.f * (2.f * u * i - u * u);
      default: return 3.f * (u * u);
    }
  }
  void bezier_prim(PrimBlock& pb) {
    int subs = named_int("subdivs");
    std::vector<std::vector<float>> patches;
    while (L.is_word("p")) {
      std::vector<float> c;
      named_block("p", [&] {
        if (L.peek_number()) {
          c.push_back(L.flt());
          while (L.accept(',')) c.push_back(L.flt());
        }
      });
      if (c.size() != 48) L.fail("error parsing bezier patch: must give 48 values per patch");   // mkPatch
      patches.push_back(std::move(c));
    }
    if (patches.empty()) L.fail("bezier needs at least one patch");
    if (subs < 1) L.fail("bezier subdivs must be positive");
    const float step = 1.f / (float)subs;
    const int vstride = subs + 1;
    for (const auto& c : patches) {                     // onePatch (Bezier.hs:60-73)
      std::vector<V3> ps, ns;
      std::vector<float> uv;
      for (int i = 0; i <= subs; ++i)
        for (int j = 0; j <= subs; ++j) {
          float u = (float)i * step, v = (float)j * step;
          float bu[4], bdu[4], bv[4], bdv[4];
          for (int k = 0; k < 4; ++k) { bu[k] = bern(u, k); bdu[k] = bern_d(u, k); bv[k] = bern(v, k); bdv[k] = bern_d(v, k); }
          auto ev = [&](const float* bj, const float* bi) {    // evalPatch's ev (Bezier.hs:50-58)
            float r[3];
            for (int o = 0; o < 3; ++o) {
              float acc = 0.f;
              for (int ii = 0; ii < 4; ++ii)
                for (int jj = 0; jj < 4; ++jj) acc = acc + c[ii * 12 + jj * 3 + o] * bj[jj] * bi[ii];
              r[o] = acc;
            }
            return v3(r[0], r[1], r[2]);
          };
          V3 p = ev(bu, bv), dpdu = ev(bdu, bv), dpdv = ev(bu, bdv);
          ps.push_back(xpoint(B.xf.m, p));                        // transPoint o2w
          ns.push_back(xnormal(B.xf.inv, cross(dpdu, dpdv)));     // transNormal o2w (dpdu `cross` dpdv)
          uv.push_back((float)i * step); uv.push_back((float)j * step);
        }
      auto tri = [&](int a, int b, int d) {
        V3 p[3] = {ps[a], ps[b], ps[d]}, n[3] = {ns[a], ns[b], ns[d]};
        float t[6] = {uv[2 * a], uv[2 * a + 1], uv[2 * b], uv[2 * b + 1], uv[2 * d], uv[2 * d + 1]};
        add_triangle(p, B.material, t, n);
        pb.prims.emplace_back(0, (int)B.tri_mat.size() - 1);
      };
      for (int i = 0; i < subs; ++i)
        for (int j = 0; j < subs; ++j) {
          int v00 = i * vstride + j, v10 = (i + 1) * vstride + j, v01 = i * vstride + j + 1, v11 = (i + 1) * vstride + j + 1;
          tri(v00, v10, v01);
          tri(v10, v11, v01);
        }
    }
  }

  void primitive() {                                    // pPrimitive (PrimitiveParser.hs:28-76)
    PrimBlock pb;
    block([&] {
      std::string t = L.word();
      if (t == "heightMap") heightmap_prim(pb);
      else if (t == "bezier") bezier_prim(pb);
      else if (t == "julia") {                          // mkJuliaQuat (PrimitiveParser.hs:47-52)
        if (B.fractal.present) L.fail("only one fractal primitive supported");
        B.fractal.present = 1;
        B.fractal.kind = BLING_FRACTAL_JULIA;
        L.expect_word("c");                             // pNamedQuat "c": flt, pVec
        for (int k = 0; k < 4; ++k) B.fractal.julia_c[k] = L.flt();
        B.fractal.epsilon = named_float("epsilon");
        B.fractal.iterations = named_int("iterations");
        B.fractal.order = 0;
        B.fractal.material = B.material;
        pb.prims.emplace_back(2, 0);
      }
      else if (t == "mesh") mesh_prim(pb);
      else if (t == "shape") shape_prim(pb);
      else if (t == "waveFront") wavefront_prim(pb);
      else if (t == "mandelbulb") {
        if (B.fractal.present) L.fail("only one fractal primitive supported");
        B.fractal.present = 1;
        B.fractal.kind = BLING_FRACTAL_MANDELBULB;
        B.fractal.order = named_int("order");
        B.fractal.epsilon = named_float("epsilon");
        B.fractal.iterations = named_int("iterations");
        B.fractal.material = B.material;
        pb.prims.emplace_back(2, 0);
      } else L.fail("unsupported primitive " + t);
    });
    B.blocks.push_back(std::move(pb));
  }

  void light() {                                        // pLight (LightParser.hs:17-27)
    block([&] {
      std::string t = L.word();
      auto lr = std::make_unique<LightRec>();
      std::memset(&lr->l, 0, sizeof lr->l);
      if (t == "point" || t == "directional") {         // pPointLight / pDirectionalLight (LightParser.hs:38-51)
        lr->l.kind = t == "point" ? BLING_LIGHT_POINT : BLING_LIGHT_DIRECTIONAL;
        L.expect_word("intensity");
        Spec sp = spectrum();
        for (int i = 0; i < 16; ++i) lr->l.radiance[i] = sp[i];
        V3 v = named_vec(t == "point" ? "position" : "normal");
        if (t == "directional") v = normalize(v);       // mkDirectional s n = Directional s (normalize n)
        lr->l.delta_vec[0] = v.x; lr->l.delta_vec[1] = v.y; lr->l.delta_vec[2] = v.z;
        B.parsed_lights.push_back(std::move(lr));
        return;
      }
      if (t != "infinite") L.fail("unknown light type " + t);
      lr->l.kind = BLING_LIGHT_INFINITE;
      Xf xf = transform_block();                        // pInfiniteArea: t, then `l`
      std::memcpy(lr->l.w2l, xf.m.m, 64);
      std::memcpy(lr->l.l2w, xf.inv.m, 64);
      L.expect_word("l");
      block([&] {                                       // pDiscSpectrumMap2d
        std::string tp = L.word();
        if (tp == "constant") {
          lr->l.env_kind = BLING_ENV_CONSTANT;
          Spec s = spectrum();
          for (int i = 0; i < 16; ++i) lr->l.env_const[i] = s[i];
        } else if (tp == "sunSky") {
          lr->l.env_kind = BLING_ENV_SUNSKY;
          V3 east = named_vec("east");
          V3 sdir = named_vec("sunDir");
          float turb = named_float("turbidity");
          bling_sky_init(&lr->l, east.x, east.y, east.z, sdir.x, sdir.y, sdir.z, turb);
        } else if (tp == "file") {                      // readTexture (IO/Bitmap.hs:13-29)
          const std::string fn = B.resolve(L.qstring());
          bimg::Decoded im;
          try { im = bimg::read_image(fn); } catch (const std::exception& e) { L.fail(e.what()); }
          if (!im.is_float) L.fail(fn + ": can't convert image format to texture");
          lr->l.env_kind = BLING_ENV_IMAGE;
          lr->l.env_w = im.width; lr->l.env_h = im.height;
          const size_t n = (size_t)im.width * im.height;
          lr->texels.resize(n * 16);                    // rgbToSpectrumIllum per pixel (rgbfToTexMap)
          for (size_t i = 0; i < n; ++i) {
            const Spec sp = rgb_to_spectrum(BLING_RGB_ILLUM_BANDS, im.rgbf[i * 3], im.rgbf[i * 3 + 1], im.rgbf[i * 3 + 2]);
            std::copy(sp.begin(), sp.end(), lr->texels.begin() + i * 16);
          }
          lr->l.env_texels = lr->texels.data();
        } else L.fail("unknown map type " + tp);
      });
      B.parsed_lights.push_back(std::move(lr));
    });
  }

  void renderer() {                                     // pRenderer (RendererParser.hs:23-54)
    block([&] {
      std::string t = L.word();
      if (t == "sampler") {
        named_block("sampled", [&] {
          named_block("sampler", [&] {
            std::string st = L.word();
            if (st == "stratified") { B.cfg.sampler = BLING_SAMPLER_STRATIFIED; B.cfg.nu = L.integ(); B.cfg.nv = L.integ(); B.cfg.spp = B.cfg.nu * B.cfg.nv; }
            else if (st == "random") { B.cfg.sampler = BLING_SAMPLER_RANDOM; B.cfg.spp = L.integ(); }
            else L.fail("unknown sampler " + st);
          });
          named_block("integrator", [&] {
            std::string it = L.word();
            if (it == "path") {
              B.cfg.max_depth = named_int("maxDepth"); B.cfg.sample_depth = named_int("sampleDepth");
              B.cfg.renderer = BLING_RENDERER_SAMPLER_PATH; B.cfg.integrator = BLING_INTEGRATOR_PATH;
            } else if (it == "directLighting") {                              // IntegratorParser.hs:37-39
              B.cfg.max_depth = named_int("maxDepth"); B.cfg.sample_depth = 0;
              B.cfg.renderer = BLING_RENDERER_SAMPLER_PATH; B.cfg.integrator = BLING_INTEGRATOR_DIRECT;
            }
            else { B.cfg.renderer = BLING_RENDERER_OTHER; while (L.peekc() != '}') { if (L.peek_number()) L.flt(); else L.word(); } }
          });
        });
      } else if (t == "sppm") {                       // RendererParser.hs:40-45
        B.cfg.sppm_photons = named_int("photonCount");
        B.cfg.max_depth = named_int("maxDepth");
        B.cfg.sppm_radius = named_float("radius");
        B.cfg.sppm_alpha = L.is_word("alpha") ? named_float("alpha") : 0.8f;   // option 0.8
        B.cfg.renderer = BLING_RENDERER_SPPM;
      } else {
        // metropolis / light: not served (trap T1); skip its arguments
        B.cfg.renderer = BLING_RENDERER_OTHER;
        while (L.peekc() != '}') { if (L.peek_number()) L.flt(); else L.word(); }
      }
    });
  }

  void filter() {                                       // pFilter (IO/RenderJob.hs:75-103)
    std::string t = L.word();
    float p[5] = {0, 0, 0, 0, 0};
    int kind;
    if (t == "box") kind = BLING_FILTER_BOX;
    else if (t == "gauss") { kind = BLING_FILTER_GAUSS; p[0] = L.flt(); p[1] = L.flt(); p[2] = L.flt(); p[3] = std::exp(-p[2] * p[0] * p[0]); p[4] = std::exp(-p[2] * p[1] * p[1]); }
    else if (t == "sinc") { kind = BLING_FILTER_SINC; p[0] = L.flt(); p[1] = L.flt(); p[2] = L.flt(); }
    else if (t == "triangle") { kind = BLING_FILTER_TRIANGLE; p[0] = L.flt(); p[1] = L.flt(); }
    else if (t == "mitchell") { kind = BLING_FILTER_MITCHELL; p[0] = L.flt(); p[1] = L.flt(); p[2] = L.flt(); p[3] = L.flt(); }
    else L.fail("unknown pixel filter " + t);
    build_filter(B.filter, kind, p);
  }

  void camera() {                                       // pCamera (CameraParser.hs:18-38)
    block([&] {
      std::string t = L.word();
      if (t == "perspective") {
        float fov = named_float("fov"), lr = named_float("lensRadius"), fd = named_float("focalDistance");
        B.make_camera(B.xf, lr, fd, fov, (float)B.resX, (float)B.resY);   // reads resX/resY NOW (T2)
      } else if (t == "environment") {
        B.camera.kind = BLING_CAM_ENVIRONMENT;
        std::memcpy(B.camera.c2w, B.xf.m.m, 64); std::memcpy(B.camera.c2w_inv, B.xf.inv.m, 64);
        B.camera.xres = (float)B.resX; B.camera.yres = (float)B.resY;
      } else L.fail("unknown camera " + t);
    });
  }

  void object() {                                       // object (IO/RenderJob.hs:44-64)
    std::string n = L.word();
    if (n == "filter") filter();
    else if (n == "prim") primitive();
    else if (n == "imageSize") {
      int sx = L.integ(), sy = L.integ();
      if (B.ov.image) { sx = B.ov.w; sy = B.ov.h; }      // override in place (T2)
      B.resX = sx; B.resY = sy;
    }
    else if (n == "renderer") renderer();
    else if (n == "transform") { Xf t = transform_block(); B.xf = cat(t, B.xf); }           // pGlobalTrans
    else if (n == "newTransform") { B.xf = identityX(); Xf t = transform_block(); B.xf = cat(t, B.xf); }
    else if (n == "camera") camera();
    else if (n == "light") light();
    else if (n == "material") { block([&] { B.material = material_body(); }); }
    else if (n == "emission") {
      block([&] {
        if (L.is_word("none")) { L.word(); B.has_emit = false; }
        else { B.emit = spectrum(); B.has_emit = true; }
      });
    }
    else L.fail("unknown object type " + n);
  }

  void job() { while (!L.eof()) object(); }
};

Overrides parse_overrides(const char* s) {
  Overrides o;
  if (!s) return o;
  std::string str(s);
  std::stringstream ss(str);
  std::string kv;
  while (std::getline(ss, kv, ';')) {
    if (kv.empty()) continue;
    size_t eq = kv.find('=');
    std::string k = kv.substr(0, eq), v = eq == std::string::npos ? "" : kv.substr(eq + 1);
    std::vector<std::string> parts;
    std::stringstream vs(v);
    std::string p;
    while (std::getline(vs, p, ',')) parts.push_back(p);
    auto I = [&](size_t i) { if (i >= parts.size()) throw ParseError("bad override " + kv); return std::atoi(parts[i].c_str()); };
    auto Fv = [&](size_t i) { if (i >= parts.size()) throw ParseError("bad override " + kv); return std::strtof(parts[i].c_str(), nullptr); };
    if (k == "image") { o.image = true; o.w = I(0); o.h = I(1); }
    else if (k == "stratified") { o.strat = true; o.nu = I(0); o.nv = I(1); }
    else if (k == "random") { o.random = true; o.spp = I(0); }
    else if (k == "path") { o.path = true; o.md = I(0); o.sd = I(1); }
    else if (k == "direct") { o.direct = true; o.dmd = I(0); }
    else if (k == "force_path") { o.force_path = I(0) != 0; }
    else if (k == "sppm") {                             // sppm=photonCount,maxDepth,radius[,alpha]
      o.sppm = true; o.sp_photons = I(0); o.sp_md = I(1); o.sp_radius = Fv(2);
      o.sp_alpha = parts.size() > 3 ? Fv(3) : 0.8f;
    }
    else if (k == "sppm_threads") { o.sppm_threads = I(0); if (o.sppm_threads < 1) throw ParseError("bad override " + kv); }
    else if (k == "filter") {
      o.filter = true;
      if (parts.empty()) throw ParseError("bad filter override");
      const std::string& t = parts[0];
      if (t == "box") o.fkind = BLING_FILTER_BOX;
      else if (t == "triangle") { o.fkind = BLING_FILTER_TRIANGLE; o.fp[0] = Fv(1); o.fp[1] = Fv(2); }
      else if (t == "mitchell") { o.fkind = BLING_FILTER_MITCHELL; for (int i = 0; i < 4; ++i) o.fp[i] = Fv(1 + i); }
      else throw ParseError("bad filter override " + t);
    }
    else throw ParseError("unknown override " + k);
  }
  return o;
}

}  // namespace

struct bling_host_scene {
  Builder b;
};

extern "C" {

int bling_host_load(const char* path, const char* overrides, bling_host_scene** out) {
  if (!path || !out) { g_err = "null argument"; return -1; }
  *out = nullptr;
  try {
    std::ifstream in(path);
    if (!in) { g_err = std::string("cannot open ") + path; return -1; }
    std::stringstream buf;
    buf << in.rdbuf();
    auto s = std::make_unique<bling_host_scene>();
    Builder& B = s->b;
    B.ov = parse_overrides(overrides);
    std::string p(path);
    size_t sl = p.find_last_of('/');
    B.base = sl == std::string::npos ? "." : p.substr(0, sl);
    Lexer L(buf.str());
    Parser P{L, B};
    P.job();
    // renderer overrides (trap T1: the last `renderer` block wins; the harness forces path)
    // force_path selects the sampler renderer and keeps a parsed surface integrator; path= / direct=
    // also replace the integrator
    if (B.ov.force_path || B.ov.path || B.ov.direct || B.ov.strat || B.ov.random) {
      if (B.ov.force_path || B.ov.path || B.ov.direct) B.cfg.renderer = BLING_RENDERER_SAMPLER_PATH;
      if (B.ov.path) { B.cfg.max_depth = B.ov.md; B.cfg.sample_depth = B.ov.sd; B.cfg.integrator = BLING_INTEGRATOR_PATH; }
      if (B.ov.direct) { B.cfg.max_depth = B.ov.dmd; B.cfg.sample_depth = 0; B.cfg.integrator = BLING_INTEGRATOR_DIRECT; }
      if (B.ov.strat) { B.cfg.sampler = BLING_SAMPLER_STRATIFIED; B.cfg.nu = B.ov.nu; B.cfg.nv = B.ov.nv; B.cfg.spp = B.ov.nu * B.ov.nv; }
      if (B.ov.random) { B.cfg.sampler = BLING_SAMPLER_RANDOM; B.cfg.spp = B.ov.spp; }
    }
    if (B.ov.sppm) {
      B.cfg.renderer = BLING_RENDERER_SPPM; B.cfg.sppm_photons = B.ov.sp_photons; B.cfg.max_depth = B.ov.sp_md;
      B.cfg.sppm_radius = B.ov.sp_radius; B.cfg.sppm_alpha = B.ov.sp_alpha;
    }
    // numCapabilities of the modelled reference run (SPPM.hs:449, 474): photons per pass are
    // threads * sn^2; 8 = this build machine's core count unless overridden
    B.cfg.sppm_threads = B.ov.sppm_threads > 0 ? B.ov.sppm_threads : 8;
    if (B.ov.filter) build_filter(B.filter, B.ov.fkind, B.ov.fp);
    B.cfg.width = B.resX;
    B.cfg.height = B.resY;
    if (B.cfg.sampler == BLING_SAMPLER_STRATIFIED) B.cfg.spp = B.cfg.nu * B.cfg.nv;

    // prims = p ++ prims: later blocks first (IO/RenderJob.hs:52)
    for (int k = (int)B.blocks.size() - 1; k >= 0; --k)
      for (auto& pr : B.blocks[k].prims) { B.prim_kind.push_back(pr.first); B.prim_index.push_back(pr.second); }
    // lights = parsed lights (prepended => reverse parse order) ++ geometric lights in prim order
    for (int k = (int)B.parsed_lights.size() - 1; k >= 0; --k) B.lights.push_back(B.parsed_lights[k]->l);
    for (size_t i = 0; i < B.prim_kind.size(); ++i) {
      if (B.prim_kind[i] != 1) continue;
      int si = B.prim_index[i];
      for (size_t q = 0; q < B.shape_light_shape.size(); ++q)
        if (B.shape_light_shape[q] == si) {
          bling_light l;
          std::memset(&l, 0, sizeof l);
          l.kind = BLING_LIGHT_AREA;
          l.shape = si;
          for (int b = 0; b < 16; ++b) l.radiance[b] = B.shape_light_rad[q][b];
          B.shapes[si].light = (int)B.lights.size();
          B.lights.push_back(l);
        }
    }
    bling_scene_desc& d = B.desc;
    std::memset(&d, 0, sizeof d);
    d.num_vertices = (uint32_t)(B.verts.size() / 3);
    d.vertices = B.verts.data();
    d.num_triangles = (uint32_t)B.tri_mat.size();
    d.tri_indices = B.tris.data();
    d.tri_material = B.tri_mat.data();
    d.tri_uvs = B.tri_uv.data();
    bool anyn = std::any_of(B.tri_hasn.begin(), B.tri_hasn.end(), [](uint8_t x) { return x != 0; });
    d.tri_normals = anyn ? B.tri_n.data() : nullptr;
    d.tri_has_normals = anyn ? B.tri_hasn.data() : nullptr;
    d.num_shapes = (uint32_t)B.shapes.size();
    d.shapes = B.shapes.data();
    d.fractal = B.fractal;
    d.num_prims = (uint32_t)B.prim_kind.size();
    d.prim_kind = B.prim_kind.data();
    d.prim_index = B.prim_index.data();
    d.num_materials = (uint32_t)B.materials.size();
    d.materials = B.materials.data();
    d.num_textures = (uint32_t)B.textures.size();
    d.textures = B.textures.data();
    d.num_scalar_textures = (uint32_t)B.scalar_textures.size();
    d.scalar_textures = B.scalar_textures.data();
    d.num_lights = (uint32_t)B.lights.size();
    d.lights = B.lights.data();
    d.camera = B.camera;
    d.filter = B.filter;
    d.config = B.cfg;
    for (size_t k = 0; k < B.images.size(); ++k) B.images[k].texels = B.image_data[k].data();
    d.num_images = (uint32_t)B.images.size();
    d.images = B.images.data();
    // the infinite lights' Dist2D arrays live in the parsed LightRec objects
    for (size_t k = 0; k < B.lights.size(); ++k) {
      if (B.lights[k].kind != BLING_LIGHT_INFINITE) continue;
      LightRec* lr = B.parsed_lights[B.parsed_lights.size() - 1 - k].get();
      bling_sky_build_dist(&B.lights[k], lr->func, lr->cdf, lr->fint, lr->mfunc, lr->mcdf);
    }
    std::ostringstream sm;
    sm << "image " << B.resX << "x" << B.resY << ", prims " << d.num_prims << " (triangles "
       << d.num_triangles << ", shapes " << d.num_shapes << ", fractal " << d.fractal.present << "), lights "
       << d.num_lights << ", materials " << d.num_materials << ", renderer "
       << (B.cfg.renderer != BLING_RENDERER_SAMPLER_PATH ? "other" : B.cfg.integrator == BLING_INTEGRATOR_DIRECT ? "direct" : "path")
       << " md=" << B.cfg.max_depth
       << " sd=" << B.cfg.sample_depth << " sampler "
       << (B.cfg.sampler == BLING_SAMPLER_STRATIFIED ? "stratified " : "random ") << B.cfg.nu << "x"
       << B.cfg.nv << " spp=" << B.cfg.spp << ", filter " << B.filter.kind << " " << B.filter.width << "x"
       << B.filter.height;
    B.summary = sm.str();
    *out = s.release();
    return 0;
  } catch (const std::exception& e) {
    g_err = std::string(path) + ": " + e.what();
    return -1;
  }
}

const bling_scene_desc* bling_host_desc(const bling_host_scene* s) { return s ? &s->b.desc : nullptr; }
void bling_host_config(const bling_host_scene* s, bling_render_config* out) { *out = s->b.desc.config; }
void bling_host_filter_size(const bling_host_scene* s, float* wh) { wh[0] = s->b.desc.filter.width; wh[1] = s->b.desc.filter.height; }
void bling_host_filter_table(const bling_host_scene* s, float* out256) {
  std::memcpy(out256, s->b.desc.filter.table, sizeof s->b.desc.filter.table);
}
void bling_host_counts(const bling_host_scene* s, uint32_t* out6) {
  const bling_scene_desc& d = s->b.desc;
  out6[0] = d.num_triangles; out6[1] = d.num_shapes; out6[2] = d.fractal.present ? 1u : 0u;
  out6[3] = d.num_prims; out6[4] = d.num_lights; out6[5] = bfeat::scene_features(&d);
}
const char* bling_host_summary(const bling_host_scene* s) { return s ? s->b.summary.c_str() : ""; }
void bling_host_free(bling_host_scene* s) { delete s; }
const char* bling_host_last_error(void) { return g_err.c_str(); }

void bling_host_film_to_rgb(const float* film, int w, int h, float* rgb) {
  // getPixel with splat weight 0 (Image.hs:302-315) then xyzToRgb (Spectrum.hs:162-168)
  for (int i = 0; i < w * h; ++i) {
    float W = film[4 * i], X = film[4 * i + 1], Y = film[4 * i + 2], Z = film[4 * i + 3];
    float x = 0, y = 0, z = 0;
    if (W != 0.f) { float iw = 1.f / W; x = 0.f * 0.f + X * iw; y = 0.f * 0.f + Y * iw; z = 0.f * 0.f + Z * iw; }
    rgb[3 * i + 0] = 3.240479f * x - 1.537150f * y - 0.498535f * z;
    rgb[3 * i + 1] = (-0.969256f) * x + 1.875991f * y + 0.041556f * z;
    rgb[3 * i + 2] = 0.055648f * x - 0.204043f * y + 1.057311f * z;
  }
}

void bling_host_film_splat_to_rgb(const float* film, const float* splat, float sw, int w, int h, float* rgb) {
  // getPixel (Image.hs:301-314) with the splat buffer and weight, then xyzToRgb
  for (int i = 0; i < w * h; ++i) {
    float W = film[4 * i], X = film[4 * i + 1], Y = film[4 * i + 2], Z = film[4 * i + 3];
    float sr = splat ? splat[3 * i] : 0.f, sg = splat ? splat[3 * i + 1] : 0.f, sb = splat ? splat[3 * i + 2] : 0.f;
    float x, y, z;
    if (W == 0.f) { x = sw * sr; y = sw * sg; z = sw * sb; }
    else { float iw = 1.f / W; x = sw * sr + X * iw; y = sw * sg + Y * iw; z = sw * sb + Z * iw; }
    rgb[3 * i + 0] = 3.240479f * x - 1.537150f * y - 0.498535f * z;
    rgb[3 * i + 1] = (-0.969256f) * x + 1.875991f * y + 0.041556f * z;
    rgb[3 * i + 2] = 0.055648f * x - 0.204043f * y + 1.057311f * z;
  }
}

void bling_host_rgb_pixels_splat(const float* film, const float* splat, float sw, int w, int h, unsigned char* out) {
  const float xg = 1.f / 2.2f;                                    // gamma x = let x' = 1 / x
  auto hmax = [](float a, float b) { return a <= b ? b : a; };    // GHC Ord Float max / min
  auto hmin = [](float a, float b) { return a <= b ? a : b; };
  std::vector<float> rgb((size_t)3 * w * h);
  bling_host_film_splat_to_rgb(film, splat, sw, w, h, rgb.data());
  for (size_t i = 0; i < rgb.size(); ++i) {
    float g = std::pow(rgb[i], xg);                               // r ** x' (powf)
    float c = hmin(1.f, hmax(0.f, g)) * 255.f;
    out[i] = (unsigned char)(int)std::nearbyint(c);               // round: half to even
  }
}

void bling_host_rgb_pixels(const float* film, int w, int h, unsigned char* out) {
  const float xg = 1.f / 2.2f;                                    // gamma x = let x' = 1 / x
  auto hmax = [](float a, float b) { return a <= b ? b : a; };    // GHC Ord Float max / min
  auto hmin = [](float a, float b) { return a <= b ? a : b; };
  std::vector<float> rgb((size_t)3 * w * h);
  bling_host_film_to_rgb(film, w, h, rgb.data());
  for (size_t i = 0; i < rgb.size(); ++i) {
    float g = std::pow(rgb[i], xg);                               // r ** x' (powf)
    float c = hmin(1.f, hmax(0.f, g)) * 255.f;
    out[i] = (unsigned char)(int)std::nearbyint(c);               // round: half to even
  }
}

namespace {
uint32_t crc32_png(const unsigned char* p, size_t n, uint32_t c = 0xFFFFFFFFu) {
  static uint32_t tab[256];
  static bool init = false;
  if (!init) {
    for (uint32_t k = 0; k < 256; ++k) {
      uint32_t v = k;
      for (int j = 0; j < 8; ++j) v = (v & 1u) ? 0xEDB88320u ^ (v >> 1) : v >> 1;
      tab[k] = v;
    }
    init = true;
  }
  for (size_t i = 0; i < n; ++i) c = tab[(c ^ p[i]) & 0xFFu] ^ (c >> 8);
  return c;
}
void put_be32(std::vector<unsigned char>& v, uint32_t x) {
  v.push_back((unsigned char)(x >> 24)); v.push_back((unsigned char)(x >> 16));
  v.push_back((unsigned char)(x >> 8)); v.push_back((unsigned char)x);
}
void png_chunk(std::vector<unsigned char>& out, const char* type, const std::vector<unsigned char>& data) {
  put_be32(out, (uint32_t)data.size());
  size_t start = out.size();
  out.insert(out.end(), type, type + 4);
  out.insert(out.end(), data.begin(), data.end());
  put_be32(out, crc32_png(out.data() + start, out.size() - start) ^ 0xFFFFFFFFu);
}
}  // namespace

int bling_host_write_png(const char* path, const float* film, int w, int h) {
  return bling_host_write_png_splat(path, film, nullptr, 0.f, w, h);
}

int bling_host_write_png_splat(const char* path, const float* film, const float* splat, float sw, int w, int h) {
  if (w <= 0 || h <= 0) { g_err = "empty image"; return -1; }
  std::vector<unsigned char> px((size_t)3 * w * h);
  if (splat) bling_host_rgb_pixels_splat(film, splat, sw, w, h, px.data());
  else bling_host_rgb_pixels(film, w, h, px.data());
  // raw scanlines, filter type 0
  std::vector<unsigned char> raw;
  raw.reserve((size_t)h * (3 * w + 1));
  for (int y = 0; y < h; ++y) {
    raw.push_back(0);
    raw.insert(raw.end(), px.begin() + (size_t)3 * w * y, px.begin() + (size_t)3 * w * (y + 1));
  }
  // zlib stream of stored deflate blocks (<= 65535 bytes each) + Adler-32
  std::vector<unsigned char> z = {0x78, 0x01};
  size_t off = 0;
  do {
    size_t n = std::min<size_t>(65535, raw.size() - off);
    bool last = off + n == raw.size();
    z.push_back(last ? 1 : 0);
    z.push_back((unsigned char)(n & 0xFF)); z.push_back((unsigned char)(n >> 8));
    z.push_back((unsigned char)(~n & 0xFF)); z.push_back((unsigned char)((~n >> 8) & 0xFF));
    z.insert(z.end(), raw.begin() + off, raw.begin() + off + n);
    off += n;
  } while (off < raw.size());
  uint32_t a = 1, b = 0;
  for (unsigned char c : raw) { a = (a + c) % 65521u; b = (b + a) % 65521u; }
  put_be32(z, (b << 16) | a);
  std::vector<unsigned char> out = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1A, '\n'};
  std::vector<unsigned char> ihdr;
  put_be32(ihdr, (uint32_t)w); put_be32(ihdr, (uint32_t)h);
  ihdr.push_back(8); ihdr.push_back(2); ihdr.push_back(0); ihdr.push_back(0); ihdr.push_back(0);   // 8-bit RGB
  png_chunk(out, "IHDR", ihdr);
  png_chunk(out, "IDAT", z);
  png_chunk(out, "IEND", {});
  FILE* f = std::fopen(path, "wb");
  if (!f) { g_err = std::string("cannot write ") + path; return -1; }
  std::fwrite(out.data(), 1, out.size(), f);
  std::fclose(f);
  return 0;
}

int bling_host_write_hdr(const char* path, const float* rgb, int w, int h) {
  FILE* f = std::fopen(path, "wb");
  if (!f) { g_err = std::string("cannot write ") + path; return -1; }
  std::fprintf(f, "#?RADIANCE\nFORMAT=32-bit_rle_rgbe\n\n-Y %d +X %d\n", h, w);
  for (int i = 0; i < w * h; ++i) {
    float r = std::max(0.f, rgb[3 * i]), g = std::max(0.f, rgb[3 * i + 1]), b = std::max(0.f, rgb[3 * i + 2]);
    float m = std::max(r, std::max(g, b));
    unsigned char e[4] = {0, 0, 0, 0};
    if (m >= 1e-32f) {
      int ex;
      float sc = std::frexp(m, &ex) * 256.f / m;
      e[0] = (unsigned char)(r * sc); e[1] = (unsigned char)(g * sc); e[2] = (unsigned char)(b * sc);
      e[3] = (unsigned char)(ex + 128);
    }
    std::fwrite(e, 1, 4, f);
  }
  std::fclose(f);
  return 0;
}

}  // extern "C"
