// bling_main.cpp -- command-line front end: the reference's "render one .bling once" harness
// (commented out in src/cmdline/Main.hs:15-42: parseJob >>= render renderer job prog, writing
// pass-NNNNN.png and .hdr at PassDone) over the host loader and the MI355X core.
//
//   bling <scene.bling> [--overrides "image=W,H;..."] [--passes N] [--out prefix] [--device D]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "bling.h"
#include "bling_host.h"

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s scene.bling [--overrides S] [--passes N] [--out prefix] [--device D]\n", argv[0]);
    return 2;
  }
  const char* scene = argv[1];
  const char* ov = nullptr;
  const char* out = "pass";
  int passes = 1, device = 0;
  for (int i = 2; i + 1 < argc; i += 2) {
    if (!std::strcmp(argv[i], "--overrides")) ov = argv[i + 1];
    else if (!std::strcmp(argv[i], "--passes")) passes = std::atoi(argv[i + 1]);
    else if (!std::strcmp(argv[i], "--out")) out = argv[i + 1];
    else if (!std::strcmp(argv[i], "--device")) device = std::atoi(argv[i + 1]);
  }
  bling_host_scene* hs = nullptr;
  if (bling_host_load(scene, ov, &hs) != 0) { std::fprintf(stderr, "%s\n", bling_host_last_error()); return 1; }
  std::printf("Job Stats\n   %s\n", bling_host_summary(hs));
  const bling_scene_desc* d = bling_host_desc(hs);
  bling_ctx* ctx = nullptr;
  if (bling_create(&device, 1, &ctx) != 0 || bling_scene_upload(ctx, d) != 0) {
    std::fprintf(stderr, "%s\n", bling_last_error());
    return 1;
  }
  int w = d->config.width, h = d->config.height;
  std::vector<float> film((size_t)w * h * 4, 0.f), rgb((size_t)w * h * 3);
  for (int p = 1; p <= passes; ++p) {
    bling_pass_params pp{0x0B11A6u, (uint32_t)p, 0, 1, 1, 0};
    bling_stats st;
    if (bling_render_pass(ctx, &pp, film.data(), &st) != 0) { std::fprintf(stderr, "%s\n", bling_last_error()); return 1; }
    uint64_t rays = st.rays_camera + st.rays_continuation + st.rays_mis + st.rays_shadow;
    std::printf("pass %d: %.1f ms, %llu samples, %.1f Mrays/s\n", p, st.ms_total, (unsigned long long)st.camera_samples,
                rays / (st.ms_total * 1e3));
    // progressWriter (IO/Progress.hs:23-36): <out>-NNNNN.png and .hdr after every pass
    char name[512];
    std::snprintf(name, sizeof name, "%s-%05d", out, p);
    std::printf("Writing %s...\n", name);
    bling_host_film_to_rgb(film.data(), w, h, rgb.data());
    if (bling_host_write_png((std::string(name) + ".png").c_str(), film.data(), w, h) != 0 ||
        bling_host_write_hdr((std::string(name) + ".hdr").c_str(), rgb.data(), w, h) != 0) {
      std::fprintf(stderr, "%s\n", bling_host_last_error());
      return 1;
    }
  }
  bling_destroy(ctx);
  bling_host_free(hs);
  return 0;
}
