/*
 * bling_scene.h -- flattened, plain-C scene description handed across the drop-in boundary.
 *
 * The reference keeps its scene as opaque Haskell closures (Primitive, Material, Texture, Light:
 * Primitive.hs:21-27, Reflection.hs:42, Texture.hs:59, Light.hs:31-45), so a device core cannot be
 * fed from a built `Scene`.  The host captures the same information at PARSE time
 * (IO/PrimitiveParser.hs:28-76, IO/MaterialParser.hs:30-42, IO/LightParser.hs:17-27,
 * IO/CameraParser.hs:18-28) into the SoA arrays below.  Everything is world space unless noted;
 * matrices are row-major 4x4 with their stored inverse (Transform.hs:124-127).
 *
 * All arrays are caller-owned; bling_scene_upload() copies what it needs.
 */
#ifndef BLING_SCENE_H
#define BLING_SCENE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BLING_NBANDS 16

/* ---- spectrum textures (Texture.hs:134-250; pSpectrumTexture, IO/MaterialParser.hs:198-226) ---- */
enum bling_tex_kind {
    BLING_TEX_CONST = 0,       /* constant spectrum (Texture.hs:159-162)                    */
    BLING_TEX_GRAPHPAPER = 1,  /* graphPaper lw (uv su sv ou ov) tex1 tex2 (Texture.hs:191-207) */
    /* computed per hit (feature bit FT_PROCTEX); only at the top of a material's texture slot,
     * their children are constant or graphPaper textures (the loader enforces it) */
    BLING_TEX_BLEND = 2,       /* spectrumBlend tex1 tex2 f (Texture.hs:135-145): f = stex      */
    BLING_TEX_GRADIENT = 3,    /* gradient f steps (Texture.hs:225-250): steps = records tex1 ..
                                  tex1 + tex2 - 1, constant, sorted by position (in line_width) */
    BLING_TEX_CHECKER = 4,     /* checkerBoard (sx sy sz) tex1 tex2 (Texture.hs:209-219); the
                                  scale vector in uv_map[0..2]                                 */
    BLING_TEX_IMAGE = 5        /* imageTexture (Texture.hs:128-129) of an RGB8 / RGBA8 / palette
                                  PNG (readImageTextureMap, :110-118): tex1 = the bling_image,
                                  tex2 = bling_map2d kind; uv: uv_map = (su, sv, ou, ov); planar:
                                  value[0..7] = vu xyz, vv xyz, ou, ov (pTextureMapping2d,
                                  MaterialParser.hs:160-178).  Texels hold pixelSpectrum
                                  (rgbToSpectrumRefl . unGamma, Texture.hs:87-89), folded on the host */
};
/* pTextureMapping2d kinds (MaterialParser.hs:160-178; Texture.hs:166-179) */
enum bling_map2d_kind { BLING_MAP_UV = 0, BLING_MAP_PLANAR = 1 };

typedef struct bling_texture {
    int32_t kind;
    int32_t tex1, tex2;        /* graphPaper / blend / checker: children; gradient: first step,
                                  number of steps                                              */
    float   line_width;        /* graphPaper lw; gradient step: its position                 */
    float   uv_map[4];         /* uvMapping (su, sv, ou, ov) (Texture.hs:166-170)           */
    float   value[BLING_NBANDS];
    int32_t stex;              /* blend / gradient: the scalar texture f (bling_scalar_texture) */
} bling_texture;

/* ---- scalar textures evaluated at a hit (pScalarTexture, IO/MaterialParser.hs:115-156;
 * Texture.hs:152-188, 340-420); used where a material takes a non-constant scalar ---- */
enum bling_stex_kind {
    BLING_STEX_CONST = 0,      /* constant v                                                 */
    BLING_STEX_SCALE = 1,      /* scale a s tex: a + s * child (scaleTexture, Texture.hs:185)  */
    BLING_STEX_FBM = 2,        /* fbm octaves omega map { identity <transform> }               */
    BLING_STEX_PERLIN = 3,     /* perlin map { identity <transform> } (noiseTexture)          */
    BLING_STEX_CELLNOISE = 4,  /* cellNoise <dist> map { identity <transform> } (Worley,
                                  Texture.hs:256-315): octaves = the distance function          */
    BLING_STEX_CRYSTAL = 5,    /* crystal octaves o map { planar vu vv ou ov } (quasiCrystal,
                                  Texture.hs:317-338): w2t[0..2] = vu, w2t[3..5] = vv, w2t[6..7]
                                  = (ou, ov); child = the first of o CONST records holding
                                  a = cos th, s = sin th of each wave's angle (host libm)        */
    BLING_STEX_IMAGE = 6       /* image { file "x.png" map {...} } of a Y8 PNG (pImageScalar,
                                  MaterialParser.hs:106-113; getPixelScalar, Texture.hs:103-108):
                                  child = the bling_image (one channel, byte / 255), octaves =
                                  bling_map2d kind, w2t[0..3] = uv (su, sv, ou, ov) or w2t[0..7] =
                                  planar (vu xyz, vv xyz, ou, ov)                                */
};
enum bling_cell_dist {         /* pScalarTexture's distance names (MaterialParser.hs:124-133)  */
    BLING_CELL_EUCLIDIAN = 0,  /* len (a - b)                                                 */
    BLING_CELL_EUCLIDIAN2 = 1, /* sqLen (a - b)                                               */
    BLING_CELL_MANHATTAN = 2,
    BLING_CELL_CHEBYSHEV = 3
};
/* deepest chain of nested `scale` scalar textures the device unwinds (eval_stex); the loader
 * rejects deeper chains, so device and oracle never disagree on one */
#define BLING_STEX_MAX_SCALE 8

typedef struct bling_scalar_texture {
    int32_t kind;
    int32_t child;             /* scale: index of the scaled texture                          */
    int32_t octaves;           /* fbm                                                         */
    float   value;             /* constant                                                    */
    float   a, s;              /* scale                                                       */
    float   omega;             /* fbm                                                         */
    float   w2t[16];           /* identityMapping3d: the parsed transform, applied with
                                  transPoint to the shading point (Texture.hs:152-156)          */
} bling_scalar_texture;

/* ---- decoded texture images (IO/Bitmap.hs, Texture.hs:87-126), row-major from the top row ---- */
typedef struct bling_image {
    int32_t width, height;
    int32_t channels;          /* 16: per-texel spectra (BLING_TEX_IMAGE), 1: scalar (BLING_STEX_IMAGE) */
    int32_t reserved;
    const float* texels;       /* width * height * channels                                   */
} bling_image;

/* ---- materials (Material.hs:32-96) ---- */
enum bling_mat_kind {
    BLING_MAT_BLACKBODY = 0,   /* blackBodyMaterial: no BxDFs (Reflection.hs:337-338)        */
    BLING_MAT_MATTE = 1,       /* tex[0]=kd, scalar[0]=sigma  -> Lambertian / OrenNayar       */
    BLING_MAT_PLASTIC = 2,     /* tex[0]=kd, tex[1]=ks, scalar[0]=rough                       */
    BLING_MAT_GLASS = 3,       /* tex[0]=kr, tex[1]=kt, scalar[0]=ior                         */
    BLING_MAT_METAL = 4,       /* tex[0]=eta, tex[1]=k, scalar[0]=rough                       */
    BLING_MAT_MIRROR = 5,      /* tex[0]=kr                                                   */
    BLING_MAT_TRANSMATTE = 6,  /* translucentMatte (Material.hs:43-53): tex[0] = sClamp 0 1 kr,
                                  tex[1] = sClamp 0 1 kt * (white - r) (both folded on the host,
                                  constant textures only), scalar[0] = ks (sigma)              */
    BLING_MAT_SHINYMETAL = 7,  /* mkShinyMetal (Material.hs:98-109): conductor spectra folded on
                                  the host (constant kr / ks only): tex[0] = frApproxEta ks,
                                  tex[1] = frApproxK ks (glossy lobe), tex[2] = frApproxEta kr,
                                  tex[3] = frApproxK kr (specular lobe), scalar[0] = rough     */
    BLING_MAT_SUBSTRATE = 8    /* mkSubstrate (Material.hs:111-128): one FresnelBlend lobe with an
                                  anisotropic distribution (Microfacet.hs:56-105); constant
                                  textures folded on the host: tex[0..2] = sClamp 0 1 of kd, ks, ka;
                                  scalar[0] = fixExponent (1 / max 0 urough), scalar[1] = the same
                                  of vrough, scalar[2] = depth; a non-constant urough / vrough /
                                  depth sets stex[0..2] and is evaluated (and folded) per hit    */
};

typedef struct bling_material {
    int32_t kind;
    int32_t tex[4];            /* spectrum texture indices, -1 if unused                     */
    float   scalar[4];         /* constant scalar textures                                    */
    int32_t stex[4];           /* stex[0..2]: scalar texture replacing scalar[k] at a hit;
                                  stex[3]: bumpMap displacement (Reflection.hs:344-377); -1 = none */
} bling_material;

/* ---- analytic shapes wrapped by mkGeom (Geometry.hs:14-37, Shape.hs) ---- */
enum bling_shape_kind {
    BLING_SHAPE_QUAD = 1,      /* params: sx, sy            (Shape.hs:157-171)               */
    BLING_SHAPE_SPHERE = 2,    /* params: radius            (Shape.hs:173-229)               */
    BLING_SHAPE_DISK = 3,      /* params: height, radius, inner radius, phiMax [rad] (:142-155) */
    BLING_SHAPE_CYLINDER = 4,  /* params: radius, zmin, zmax, phiMax [rad]          (:113-140) */
    BLING_SHAPE_BOX = 5        /* params: pmin xyz, pmax xyz                         (:86-111)  */
};

typedef struct bling_shape {
    int32_t kind;
    int32_t material;
    int32_t light;             /* index into lights[] (area light), -1 if not emissive       */
    int32_t shape_id;          /* nextId at parse time; AreaLight equality (Light.hs:48-50)  */
    float   params[8];
    float   o2w[16], w2o[16];  /* object-to-world matrix and its stored inverse              */
} bling_shape;

/* ---- the distance-estimated fractal primitive: Mandelbulb (Fractal.hs:23-35) or quaternion
 * Julia set (Fractal.hs:148-160); at most one per scene ---- */
enum bling_fractal_kind { BLING_FRACTAL_MANDELBULB = 0, BLING_FRACTAL_JULIA = 1 };

typedef struct bling_fractal {
    int32_t present;
    int32_t material;
    int32_t order;             /* Mandelbulb order                                            */
    int32_t iterations;
    float   epsilon;
    int32_t kind;              /* bling_fractal_kind                                          */
    float   julia_c[4];        /* Julia c = Quaternion real (i, j, k)                         */
} bling_fractal;

/* ---- lights (Light.hs:31-45) ---- */
enum bling_light_kind {
    BLING_LIGHT_AREA = 1,
    BLING_LIGHT_INFINITE = 2,
    BLING_LIGHT_POINT = 3,         /* mkPointLight intensity position (Light.hs:57-61, 147-150)    */
    BLING_LIGHT_DIRECTIONAL = 4    /* mkDirectional intensity normal (Light.hs:52-54, 143-145)     */
};
enum bling_envmap_kind {
    BLING_ENV_CONSTANT = 0,    /* constSpectrumMap2d (Texture.hs:131-132), size 1x1          */
    BLING_ENV_SUNSKY = 1,      /* mkSunSkyLight (SunSky.hs:12-24), size 640x480              */
    BLING_ENV_IMAGE = 2        /* l { file "x.hdr" } (MaterialParser.hs:258-264): a Radiance RGBE
                                  image read as RGBF (IO/Bitmap.hs:13-29), size w x h; texels =
                                  rgbToSpectrumIllum per pixel, folded on the host               */
};

typedef struct bling_light {
    int32_t kind;
    /* area */
    int32_t shape;             /* index into shapes[]                                        */
    float   radiance[BLING_NBANDS];
    /* infinite: w2l is the parsed transform used as world->light (T14, Light.hs:76) */
    float   w2l[16], l2w[16];
    int32_t env_kind;
    float   env_const[BLING_NBANDS];
    /* sun/sky state (SunSky.hs:45-65, 96-125), precomputed on the host */
    float   sky_basis[9];      /* coordinateSystem' rows s,t,n                               */
    float   sun_dir_local[3];  /* normalize (worldToLocal basis sunDir)                       */
    float   sun_theta;
    float   perez_x[5], perez_y[5], perez_Y[5];
    float   zenith_x, zenith_y, zenith_Y;
    float   sun_radiance[BLING_NBANDS];
    /* Dist2D over the env map (Montecarlo.hs:80-104): nu x nv conditionals + marginal */
    int32_t dist_nu, dist_nv;
    const float* dist_func;    /* nv * nu  (row v: conditional func)                         */
    const float* dist_cdf;     /* nv * (nu + 1)                                              */
    const float* dist_func_int;/* nv     (funcInt of each conditional)                       */
    const float* marg_func;    /* nv                                                          */
    const float* marg_cdf;     /* nv + 1                                                      */
    float   marg_func_int;
    /* point: the position; directional: the normalised direction.  Their intensity is radiance[] */
    float   delta_vec[3];
    /* BLING_ENV_IMAGE: the map's size and its w * h * 16 texel spectra (row-major from the top) */
    int32_t env_w, env_h;
    const float* env_texels;
} bling_light;

/* ---- camera (Camera.hs:24-33, 108-147) ---- */
enum bling_camera_kind { BLING_CAM_PERSPECTIVE = 0, BLING_CAM_ENVIRONMENT = 1 };

typedef struct bling_camera {
    int32_t kind;
    float   c2w[16], c2w_inv[16];
    float   r2c[16], r2c_inv[16];
    float   lens_radius, focal_distance;
    float   xres, yres;        /* environment camera                                          */
} bling_camera;

/* ---- pixel filter as the 16x16 table of Image.hs:40-61 ---- */
enum bling_filter_kind {
    BLING_FILTER_BOX = 0, BLING_FILTER_GAUSS = 1, BLING_FILTER_SINC = 2,
    BLING_FILTER_MITCHELL = 3, BLING_FILTER_TRIANGLE = 4
};

typedef struct bling_filter {
    int32_t kind;
    float   width, height;     /* filterSize (Filter.hs:61-66)                              */
    float   table[256];        /* mkTableFilter (Image.hs:48-61)                              */
} bling_filter;

/* ---- renderer configuration (IO/RendererParser.hs, IO/IntegratorParser.hs) ---- */
enum bling_sampler_kind { BLING_SAMPLER_STRATIFIED = 0, BLING_SAMPLER_RANDOM = 1 };
enum bling_renderer_kind {
    BLING_RENDERER_SAMPLER_PATH = 0,   /* sampler renderer (Rendering.hs:77-78) + surface integrator      */
    BLING_RENDERER_OTHER = 1,          /* metropolis / light tracer: not served                            */
    BLING_RENDERER_SPPM = 2            /* sppm photonCount maxDepth radius [alpha] (RendererParser.hs:40-45) */
};
/* the sampler renderer's surface integrator (IO/IntegratorParser.hs:15-47) */
enum bling_integrator_kind {
    BLING_INTEGRATOR_PATH = 0,     /* path maxDepth sampleDepth        (Integrator/Path.hs)           */
    BLING_INTEGRATOR_DIRECT = 1    /* directLighting maxDepth          (Integrator/DirectLighting.hs) */
};

typedef struct bling_render_config {
    int32_t renderer;          /* which renderer block won (T1)                               */
    int32_t sampler;
    int32_t nu, nv;            /* stratified                                                  */
    int32_t spp;               /* random                                                      */
    int32_t max_depth, sample_depth;
    int32_t width, height;     /* imageSize (resX, resY)                                      */
    int32_t integrator;        /* bling_integrator_kind (sample_depth unused for DIRECT)       */
    /* SPPM (Renderer/SPPM.hs:40-54, 466-480); max_depth is its eye-path depth */
    int32_t sppm_photons;      /* photonCount: photons per pass before rounding (n)            */
    float   sppm_radius;       /* initial search radius r (r2 starts at r * r)                 */
    float   sppm_alpha;        /* radius shrink alpha, default 0.8                             */
    int32_t sppm_threads;      /* numCapabilities of the reference run: photons per pass are
                                  threads * sn^2, sn = max 1 (ceiling (sqrt (n / threads)))    */
} bling_render_config;

typedef struct bling_scene_desc {
    /* triangles (TriangleMesh.hs:39-60; vertices already transformed to world space) */
    uint32_t      num_vertices;
    const float*  vertices;    /* 3 * num_vertices                                            */
    uint32_t      num_triangles;
    const uint32_t* tri_indices;  /* 3 * num_triangles                                         */
    const int32_t*  tri_material; /* num_triangles                                             */
    const float*  tri_uvs;     /* 6 * num_triangles: (u0,v0,u1,v1,u2,v2) (TriangleMesh.hs:119-120) */
    const float*  tri_normals; /* 9 * num_triangles world-space shading normals, or NULL      */
    const uint8_t* tri_has_normals; /* num_triangles, or NULL                                  */

    uint32_t            num_shapes;
    const bling_shape*  shapes;
    bling_fractal       fractal;

    /* the reference primitive list order (mkScene input, IO/RenderJob.hs:41):
       prim_kind 0 = triangle (index into triangles), 1 = shape, 2 = fractal */
    uint32_t        num_prims;
    const int32_t*  prim_kind;
    const int32_t*  prim_index;

    uint32_t              num_materials;
    const bling_material* materials;
    uint32_t              num_textures;
    const bling_texture*  textures;
    uint32_t                     num_scalar_textures;
    const bling_scalar_texture*  scalar_textures;

    /* scene lights in Scene.hs:42 order: parsed lights, then geometric (area) lights */
    uint32_t           num_lights;
    const bling_light* lights;

    bling_camera        camera;
    bling_filter        filter;
    bling_render_config config;

    /* texture images (BLING_TEX_IMAGE / BLING_STEX_IMAGE) */
    uint32_t           num_images;
    const bling_image* images;
} bling_scene_desc;

#ifdef __cplusplus
}
#endif
#endif /* BLING_SCENE_H */
