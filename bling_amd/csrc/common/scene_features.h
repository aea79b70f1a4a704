// scene_features.h -- which material / light / shape kinds a flattened scene uses (the FT_* bits of
// core/dev_scene.h).  Shared by the device core (kernel profile selection) and the host loader
// (reported to tools and tests).
#pragma once
#include <stdint.h>
#include "../../../include/bling_scene.h"

namespace bfeat {

enum : uint32_t {
  MATTE = 1u << 0, PLASTIC = 1u << 1, GLASS = 1u << 2, METAL = 1u << 3, MIRROR = 1u << 4,
  GRAPHPAPER = 1u << 5, AREA = 1u << 6, ENV_CONST = 1u << 7, ENV_SKY = 1u << 8,
  SPHERE = 1u << 9, TRI_NORMALS = 1u << 10, FRACTAL = 1u << 11, TRIS = 1u << 12,
  SHAPES2 = 1u << 13, TRANSMATTE = 1u << 14, SHINYMETAL = 1u << 15, SUBSTRATE = 1u << 16, BUMP = 1u << 17,
  PROCTEX = 1u << 18,                // per-hit computed spectra (blend / gradient / checker), cellNoise, crystal
  DELTA = 1u << 19,                   // point / directional lights (delta distributions)
  ENV_IMG = 1u << 20,                 // infinite lights with an image map
  MULTI_LIGHT = 1u << 21              // more than one light (the one-light profile's kernels read light 0)
};

inline uint32_t scene_features(const bling_scene_desc* d) {
  uint32_t f = 0;
  for (uint32_t i = 0; i < d->num_materials; ++i) {
    switch (d->materials[i].kind) {
      case BLING_MAT_MATTE: f |= MATTE; break;
      case BLING_MAT_PLASTIC: f |= PLASTIC; break;
      case BLING_MAT_GLASS: f |= GLASS; break;
      case BLING_MAT_METAL: f |= METAL; break;
      case BLING_MAT_MIRROR: f |= MIRROR; break;
      case BLING_MAT_TRANSMATTE: f |= TRANSMATTE; break;
      case BLING_MAT_SHINYMETAL: f |= SHINYMETAL; break;
      case BLING_MAT_SUBSTRATE: f |= SUBSTRATE; break;
      default: break;
    }
    if (d->materials[i].stex[3] >= 0) f |= BUMP;
  }
  for (uint32_t i = 0; i < d->num_textures; ++i) {
    if (d->textures[i].kind == BLING_TEX_GRAPHPAPER) f |= GRAPHPAPER;
    if (d->textures[i].kind >= BLING_TEX_BLEND) f |= PROCTEX;
  }
  for (uint32_t i = 0; i < d->num_scalar_textures; ++i)
    if (d->scalar_textures[i].kind >= BLING_STEX_CELLNOISE) f |= PROCTEX;
  for (uint32_t i = 0; i < d->num_lights; ++i) {
    const bling_light& l = d->lights[i];
    if (l.kind == BLING_LIGHT_AREA) f |= AREA;
    else if (l.kind == BLING_LIGHT_POINT || l.kind == BLING_LIGHT_DIRECTIONAL) f |= DELTA;
    else f |= (l.env_kind == BLING_ENV_SUNSKY) ? ENV_SKY : (l.env_kind == BLING_ENV_IMAGE) ? ENV_IMG : ENV_CONST;
  }
  for (uint32_t i = 0; i < d->num_shapes; ++i)
    if (d->shapes[i].kind == BLING_SHAPE_SPHERE) f |= SPHERE;
    else if (d->shapes[i].kind != BLING_SHAPE_QUAD) f |= SHAPES2;
  if (d->num_triangles) f |= TRIS;
  if (d->tri_normals && d->tri_has_normals)
    for (uint32_t i = 0; i < d->num_triangles; ++i)
      if (d->tri_has_normals[i]) { f |= TRI_NORMALS; break; }
  if (d->fractal.present) f |= FRACTAL;
  if (d->num_lights > 1) f |= MULTI_LIGHT;
  return f;
}

}  // namespace bfeat
