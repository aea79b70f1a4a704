"""ctypes mirror of include/bling_scene.h (test infrastructure): read-only views of the flattened
scene description a parsed Job hands to bling_scene_upload, so known-answer tests can compare the
loader's precomputed values (camera matrices, band spectra, sun / sky state) with independent
restatements of the reference formulas.  Layout: natural alignment, no packing (the C header)."""
import ctypes as C

import numpy as np

NB = 16
f32p = C.POINTER(C.c_float)


class Texture(C.Structure):
    _fields_ = [("kind", C.c_int32), ("tex1", C.c_int32), ("tex2", C.c_int32), ("line_width", C.c_float),
                ("uv_map", C.c_float * 4), ("value", C.c_float * NB), ("stex", C.c_int32)]


class ScalarTexture(C.Structure):
    _fields_ = [("kind", C.c_int32), ("child", C.c_int32), ("octaves", C.c_int32), ("value", C.c_float),
                ("a", C.c_float), ("s", C.c_float), ("omega", C.c_float), ("w2t", C.c_float * 16)]


class Material(C.Structure):
    _fields_ = [("kind", C.c_int32), ("tex", C.c_int32 * 4), ("scalar", C.c_float * 4), ("stex", C.c_int32 * 4)]


class Shape(C.Structure):
    _fields_ = [("kind", C.c_int32), ("material", C.c_int32), ("light", C.c_int32), ("shape_id", C.c_int32),
                ("params", C.c_float * 8), ("o2w", C.c_float * 16), ("w2o", C.c_float * 16)]


class Fractal(C.Structure):
    _fields_ = [("present", C.c_int32), ("material", C.c_int32), ("order", C.c_int32), ("iterations", C.c_int32),
                ("epsilon", C.c_float), ("kind", C.c_int32), ("julia_c", C.c_float * 4)]


class Light(C.Structure):
    _fields_ = [("kind", C.c_int32), ("shape", C.c_int32), ("radiance", C.c_float * NB),
                ("w2l", C.c_float * 16), ("l2w", C.c_float * 16), ("env_kind", C.c_int32),
                ("env_const", C.c_float * NB), ("sky_basis", C.c_float * 9), ("sun_dir_local", C.c_float * 3),
                ("sun_theta", C.c_float), ("perez_x", C.c_float * 5), ("perez_y", C.c_float * 5),
                ("perez_Y", C.c_float * 5), ("zenith_x", C.c_float), ("zenith_y", C.c_float), ("zenith_Y", C.c_float),
                ("sun_radiance", C.c_float * NB), ("dist_nu", C.c_int32), ("dist_nv", C.c_int32),
                ("dist_func", f32p), ("dist_cdf", f32p), ("dist_func_int", f32p), ("marg_func", f32p),
                ("marg_cdf", f32p), ("marg_func_int", C.c_float), ("delta_vec", C.c_float * 3),
                ("env_w", C.c_int32), ("env_h", C.c_int32), ("env_texels", f32p)]


class Image(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("channels", C.c_int32), ("reserved", C.c_int32),
                ("texels", f32p)]


class Camera(C.Structure):
    _fields_ = [("kind", C.c_int32), ("c2w", C.c_float * 16), ("c2w_inv", C.c_float * 16), ("r2c", C.c_float * 16),
                ("r2c_inv", C.c_float * 16), ("lens_radius", C.c_float), ("focal_distance", C.c_float),
                ("xres", C.c_float), ("yres", C.c_float)]


class Filter(C.Structure):
    _fields_ = [("kind", C.c_int32), ("width", C.c_float), ("height", C.c_float), ("table", C.c_float * 256)]


class RenderConfig(C.Structure):
    _fields_ = [("renderer", C.c_int32), ("sampler", C.c_int32), ("nu", C.c_int32), ("nv", C.c_int32),
                ("spp", C.c_int32), ("max_depth", C.c_int32), ("sample_depth", C.c_int32),
                ("width", C.c_int32), ("height", C.c_int32), ("integrator", C.c_int32),
                ("sppm_photons", C.c_int32), ("sppm_radius", C.c_float), ("sppm_alpha", C.c_float),
                ("sppm_threads", C.c_int32)]


class SceneDesc(C.Structure):
    _fields_ = [("num_vertices", C.c_uint32), ("vertices", f32p), ("num_triangles", C.c_uint32),
                ("tri_indices", C.POINTER(C.c_uint32)), ("tri_material", C.POINTER(C.c_int32)),
                ("tri_uvs", f32p), ("tri_normals", f32p), ("tri_has_normals", C.POINTER(C.c_uint8)),
                ("num_shapes", C.c_uint32), ("shapes", C.POINTER(Shape)), ("fractal", Fractal),
                ("num_prims", C.c_uint32), ("prim_kind", C.POINTER(C.c_int32)), ("prim_index", C.POINTER(C.c_int32)),
                ("num_materials", C.c_uint32), ("materials", C.POINTER(Material)),
                ("num_textures", C.c_uint32), ("textures", C.POINTER(Texture)),
                ("num_scalar_textures", C.c_uint32), ("scalar_textures", C.POINTER(ScalarTexture)),
                ("num_lights", C.c_uint32), ("lights", C.POINTER(Light)),
                ("camera", Camera), ("filter", Filter), ("config", RenderConfig),
                ("num_images", C.c_uint32), ("images", C.POINTER(Image))]


def desc(job) -> SceneDesc:
    """The Job's bling_scene_desc (valid while the Job lives)."""
    return SceneDesc.from_address(job.desc)


def arr(x, shape=None) -> np.ndarray:
    a = np.array(x, dtype=np.float32)
    return a.reshape(shape) if shape else a
