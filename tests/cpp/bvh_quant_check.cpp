// Checks bvh::quantize4 (bling_amd/csrc/core/bvh_build.cpp) on random scenes: every used child's
// decoded box contains its float box, each plane lies within one quantization step of it, links are
// unchanged.  Built and run by tests/test_bvh_quant.py (CPU only).
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "../../bling_amd/csrc/core/bvh_build.h"

static int check(const std::vector<bvh::Box>& boxes, const char* name) {
  std::vector<uint32_t> refs(boxes.size());
  for (size_t i = 0; i < refs.size(); ++i) refs[i] = (uint32_t)i;
  const bvh::Result R = bvh::build(boxes, refs, 2);
  const bvh::Result4 Q = bvh::collapse4(R);
  const std::vector<uint32_t> qn = bvh::quantize4(Q);
  const size_t n = Q.nodes.size() / 28;
  if (qn.size() != 16 * n) { std::printf("FAIL %s: size\n", name); return 1; }
  size_t planes = 0, bad = 0;
  double slack = 0.0;
  for (size_t q = 0; q < n; ++q) {
    const float* nd = &Q.nodes[28 * q];
    const uint32_t* w = &qn[16 * q];
    for (int k = 0; k < 4; ++k) {
      int32_t l0, l1;
      std::memcpy(&l0, &nd[24 + k], 4);
      std::memcpy(&l1, &w[12 + k], 4);
      if (l0 != l1) { std::printf("FAIL %s: link node %zu slot %d\n", name, q, k); return 1; }
      if (l0 == bvh::EMPTY4) continue;
      for (int a = 0; a < 3; ++a) {
        float o, s;
        std::memcpy(&o, &w[a], 4);
        std::memcpy(&s, &w[3 + a], 4);
        const uint32_t ql = (w[6 + a] >> (8 * k)) & 0xFFu, qh = (w[9 + a] >> (8 * k)) & 0xFFu;
        const float lo = bvh::dequant(ql, s, o), hi = bvh::dequant(qh, s, o);
        const float flo = nd[4 * a + k], fhi = nd[4 * (3 + a) + k];
        planes += 2;
        if (!(lo <= flo) || !(hi >= fhi)) {
          std::printf("FAIL %s: node %zu slot %d axis %d: [%.9g, %.9g] does not contain [%.9g, %.9g]\n", name, q, k, a,
                      lo, hi, flo, fhi);
          return 1;
        }
        // within one step (plus the sum's rounding) of the float plane
        const double tol = (double)s * 1.0001 + 1e-6 * std::fabs((double)o);
        if ((double)flo - lo > tol || (double)hi - fhi > tol) ++bad;
        slack += ((double)flo - lo + (double)hi - fhi) / (double)s;
      }
    }
  }
  std::printf("%s: %zu nodes, %zu planes, %zu loose, mean slack %.3f steps\n", name, n, planes, bad, slack / planes);
  return bad ? 1 : 0;
}

int main() {
  std::mt19937 rng(1234);
  std::uniform_real_distribution<float> U(0.f, 1.f);
  int fails = 0;
  // triangles' boxes in a unit cube, a large offset scene (1e5), flat (zero-extent) boxes, mixed scales
  const struct { const char* name; float off, size, ext; bool flat; } cases[] = {
      {"unit", 0.f, 1.f, 0.05f, false},      {"offset", 1.0e5f, 50.f, 2.f, false}, {"flat", -3.f, 10.f, 0.5f, true},
      {"wide", -2.0e3f, 4.0e3f, 400.f, false}, {"tiny", 1.f, 1e-3f, 1e-5f, false}};
  for (const auto& c : cases) {
    std::vector<bvh::Box> boxes(20000);
    for (auto& b : boxes) {
      for (int a = 0; a < 3; ++a) {
        const float p = c.off + c.size * U(rng), e = c.ext * U(rng) * U(rng);
        b.lo[a] = p;
        b.hi[a] = (c.flat && a == 1) ? p : p + e;
      }
    }
    fails += check(boxes, c.name);
  }
  return fails ? 1 : 0;
}
