/*
 * bling_host.h -- host side of the boundary: the `.bling` scene loader and film output.
 *
 * In the reference this is Haskell and stays unchanged (north_star: "unchanged: parser,
 * Material/Texture, Film/tonemap"): parseJob (IO/RenderJob.hs:31-34) and the PState parsers in
 * IO/ *.hs, plus getPixel/xyzToRgb (Image.hs:302-315) and the HDR writer (IO/Bitmap.hs:36-41).
 * GHC is absent from this image, so this C++ library restates them for the config subset and
 * produces the flattened bling_scene_desc that bling_scene_upload() (bling.h) consumes.
 */
#ifndef BLING_HOST_H
#define BLING_HOST_H

#include "bling_scene.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct bling_host_scene bling_host_scene;

/* Parse a .bling file (parseJob, IO/RenderJob.hs:31-65).
 * overrides: NULL or "key=value;..." applied at parse time, e.g.
 *   "image=1024,1024;stratified=8,8;path=15,3"   (imageSize is patched IN PLACE, trap T2)
 *   "random=512"  "filter=triangle,2,2"  "force_path=1" (trap T1: the last renderer wins)
 * Returns 0 or a negative error (message via bling_host_last_error). */
int bling_host_load(const char* path, const char* overrides, bling_host_scene** out);

const bling_scene_desc* bling_host_desc(const bling_host_scene* s);

/* Renderer configuration and filter extent of the parsed job (for drivers). */
void bling_host_config(const bling_host_scene* s, bling_render_config* out);
void bling_host_filter_size(const bling_host_scene* s, float* wh);
/* The 16x16 filter table (mkTableFilter, Image.hs:48-61) and the scene's prim/shape/light counts
 * (out[0..5] = triangles, shapes, fractal present, prims, lights, feature bits) for tests/tools. */
void bling_host_filter_table(const bling_host_scene* s, float* out256);
void bling_host_counts(const bling_host_scene* s, uint32_t* out6);

/* Human-readable summary of the parsed scene (prettyPrint Scene, Scene.hs:28-35). */
const char* bling_host_summary(const bling_host_scene* s);

void bling_host_free(bling_host_scene* s);

const char* bling_host_last_error(void);

/* Film -> RGB (getPixel: XYZ/W + splat, then xyzToRgb; Image.hs:302-315, Spectrum.hs:162-168).
 * film: w*h*4 (W,X,Y,Z); rgb_out: w*h*3. */
void bling_host_film_to_rgb(const float* film, int w, int h, float* rgb_out);

/* Radiance HDR (.hdr, RGBE) writer for the RGB image (writeRgbe, IO/Bitmap.hs:36-41). */
int bling_host_write_hdr(const char* path, const float* rgb, int w, int h);

/* rgbPixels (Image.hs:317-331) of the whole film: getPixel with splat weight 1 and an empty splat
 * buffer, gamma 2.2 (Float `**` = powf of 1/2.2), clamp to [0,1] with Haskell min/max NaN rules,
 * * 255 and Haskell `round` (half to even).  out_rgb8: w*h*3 bytes, row-major from the top. */
void bling_host_rgb_pixels(const float* film, int w, int h, unsigned char* out_rgb8);

/* 8-bit RGB PNG of rgbPixels (writePng, IO/Bitmap.hs:40-41 / Progress.hs:29).  The reference's
 * own float -> 8-bit step lives in JuicyPixels (absent here), so the pixels are the
 * reference's rgbPixels mapping; the zlib stream uses stored (uncompressed) deflate blocks. */
int bling_host_write_png(const char* path, const float* film, int w, int h);

/* getPixel with a splat buffer (w*h*3 XYZ, may be NULL) and splat weight sw (Image.hs:301-314):
 * XYZ = sw * splat (+ film XYZ / W when W != 0), then xyzToRgb.  SPPM's pass-k image uses
 * sw = 1 / (threads * k * sn^2) (Renderer/SPPM.hs:460). */
void bling_host_film_splat_to_rgb(const float* film, const float* splat, float sw, int w, int h, float* rgb_out);
void bling_host_rgb_pixels_splat(const float* film, const float* splat, float sw, int w, int h,
                                 unsigned char* out_rgb8);
int bling_host_write_png_splat(const char* path, const float* film, const float* splat, float sw, int w, int h);

#ifdef __cplusplus
}
#endif
#endif
