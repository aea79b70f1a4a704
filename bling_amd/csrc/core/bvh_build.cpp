// bvh_build.cpp -- binned SAH BVH2 (16 bins per axis over primitive centroids), padded child boxes
// for conservative float culling, depth capped so the LDS traversal stack (32 entries) can never
// overflow.  Runs once per scene upload; build time is excluded from Mrays/s.
#include "bvh_build.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>
#include <stdexcept>

namespace bvh {
namespace {

constexpr int NBINS = 16;
constexpr float INF = std::numeric_limits<float>::infinity();

struct Item { Box b; float c[3]; uint32_t ref; };

Box empty() { Box b; for (int k = 0; k < 3; ++k) { b.lo[k] = INF; b.hi[k] = -INF; } return b; }
void grow(Box& a, const Box& b) {
  for (int k = 0; k < 3; ++k) { a.lo[k] = std::min(a.lo[k], b.lo[k]); a.hi[k] = std::max(a.hi[k], b.hi[k]); }
}
float area(const Box& b) {
  float d[3];
  for (int k = 0; k < 3; ++k) d[k] = std::max(0.f, b.hi[k] - b.lo[k]);
  return 2.f * (d[0] * d[1] + d[0] * d[2] + d[1] * d[2]);
}
// widen by a few ulps of the box magnitude so rounding in the slab test never culls a true hit
Box padded(Box b) {
  float m = 0.f;
  for (int k = 0; k < 3; ++k) m = std::max(m, std::max(std::fabs(b.lo[k]), std::fabs(b.hi[k])));
  float e = m * 2e-6f + 1e-30f;
  for (int k = 0; k < 3; ++k) { b.lo[k] -= e; b.hi[k] += e; }
  return b;
}

struct Builder {
  std::vector<Item>& it;
  Result& R;
  int max_leaf, max_depth;

  int32_t leaf(int b, int e) {
    int n = e - b;
    if (n > 255) throw std::runtime_error("BVH leaf with more than 255 primitives at the depth cap");
    uint32_t first = (uint32_t)R.refs.size();
    for (int i = b; i < e; ++i) R.refs.push_back(it[i].ref);
    R.leaves++;
    R.max_leaf = std::max(R.max_leaf, n);
    return (int32_t)~((first << 8) | (uint32_t)n);
  }

  Box bounds(int b, int e) { Box x = empty(); for (int i = b; i < e; ++i) grow(x, it[i].b); return x; }

  // best SAH split of [b, e): returns mid (b < mid < e) or -1 if a leaf is cheaper
  int split(int b, int e, int depth) {
    int n = e - b;
    if (depth >= max_depth) return -1;
    Box cb = empty();
    for (int i = b; i < e; ++i)
      for (int k = 0; k < 3; ++k) { cb.lo[k] = std::min(cb.lo[k], it[i].c[k]); cb.hi[k] = std::max(cb.hi[k], it[i].c[k]); }
    float pa = area(bounds(b, e));
    float best = INF; int bax = -1, bbin = -1;
    for (int ax = 0; ax < 3; ++ax) {
      float ext = cb.hi[ax] - cb.lo[ax];
      if (!(ext > 0.f)) continue;
      Box bb[NBINS]; int cnt[NBINS] = {0};
      for (int k = 0; k < NBINS; ++k) bb[k] = empty();
      float sc = NBINS / ext;
      for (int i = b; i < e; ++i) {
        int k = std::min(NBINS - 1, (int)((it[i].c[ax] - cb.lo[ax]) * sc));
        cnt[k]++; grow(bb[k], it[i].b);
      }
      float ra[NBINS]; int rc[NBINS];
      Box acc = empty(); int ac = 0;
      for (int k = NBINS - 1; k > 0; --k) { grow(acc, bb[k]); ac += cnt[k]; ra[k] = area(acc); rc[k] = ac; }
      acc = empty(); ac = 0;
      for (int k = 0; k < NBINS - 1; ++k) {
        grow(acc, bb[k]); ac += cnt[k];
        if (ac == 0 || rc[k + 1] == 0) continue;
        float c = 1.f + (area(acc) * ac + ra[k + 1] * rc[k + 1]) / pa;
        if (c < best) { best = c; bax = ax; bbin = k; }
      }
    }
    if (bax < 0) {                       // all centroids coincide: split by index if too large
      if (n <= max_leaf) return -1;
      return b + n / 2;
    }
    if (n <= max_leaf && best >= (float)n) return -1;
    float ext = cb.hi[bax] - cb.lo[bax], sc = NBINS / ext, lo = cb.lo[bax];
    auto mid = std::partition(it.begin() + b, it.begin() + e, [&](const Item& x) {
      return std::min(NBINS - 1, (int)((x.c[bax] - lo) * sc)) <= bbin;
    });
    int m = (int)(mid - it.begin());
    if (m == b || m == e) m = b + n / 2;
    return m;
  }

  // emits the node for range [b, e) split at m, returns its index
  int32_t node(int b, int m, int e, int depth) {
    int32_t idx = (int32_t)(R.nodes.size() / 16);
    R.nodes.resize(R.nodes.size() + 16, 0.f);
    R.depth = std::max(R.depth, depth + 1);
    int32_t links[2];
    Box boxes[2];
    int rb[2] = {b, m}, re[2] = {m, e};
    for (int c = 0; c < 2; ++c) {
      if (re[c] == rb[c]) { boxes[c] = empty(); links[c] = (int32_t)~0u; continue; }   // empty leaf
      boxes[c] = padded(bounds(rb[c], re[c]));
      int s = split(rb[c], re[c], depth + 1);
      links[c] = s < 0 ? leaf(rb[c], re[c]) : node(rb[c], s, re[c], depth + 1);
    }
    float* n = &R.nodes[16 * idx];
    n[0] = boxes[0].lo[0]; n[1] = boxes[0].lo[1]; n[2] = boxes[0].lo[2]; n[3] = boxes[0].hi[0];
    n[4] = boxes[0].hi[1]; n[5] = boxes[0].hi[2]; n[6] = boxes[1].lo[0]; n[7] = boxes[1].lo[1];
    n[8] = boxes[1].lo[2]; n[9] = boxes[1].hi[0]; n[10] = boxes[1].hi[1]; n[11] = boxes[1].hi[2];
    std::memcpy(&n[12], &links[0], 4);
    std::memcpy(&n[13], &links[1], 4);
    return idx;
  }
};

}  // namespace

Result build(const std::vector<Box>& boxes, const std::vector<uint32_t>& refs_in, int max_leaf, int max_depth) {
  Result R;
  std::vector<Item> it(boxes.size());
  for (size_t i = 0; i < boxes.size(); ++i) {
    it[i].b = boxes[i];
    for (int k = 0; k < 3; ++k) it[i].c[k] = 0.5f * (boxes[i].lo[k] + boxes[i].hi[k]);
    it[i].ref = refs_in[i];
  }
  Builder B{it, R, max_leaf, max_depth};
  int n = (int)it.size();
  if (n <= 1) B.node(0, n, n, 0);                      // child 0 = leaf with everything, child 1 empty
  else {
    int m = B.split(0, n, 0);
    if (m < 0) m = n / 2;
    B.node(0, m, n, 0);
  }
  // Breadth-first node order: the top levels form a prefix of the array, which the traversal
  // kernels keep in LDS (dev_trace.h).
  const size_t nn = R.nodes.size() / 16;
  std::vector<int32_t> order, newidx(nn, -1);
  order.reserve(nn);
  order.push_back(0);
  newidx[0] = 0;
  for (size_t q = 0; q < order.size(); ++q) {
    const float* nd = &R.nodes[16 * (size_t)order[q]];
    for (int c = 0; c < 2; ++c) {
      int32_t link;
      std::memcpy(&link, &nd[12 + c], 4);
      if (link >= 0) { newidx[link] = (int32_t)order.size(); order.push_back(link); }
    }
  }
  std::vector<float> bfs(R.nodes.size());
  for (size_t k = 0; k < nn; ++k) {
    std::memcpy(&bfs[16 * k], &R.nodes[16 * (size_t)order[k]], 16 * sizeof(float));
    for (int c = 0; c < 2; ++c) {
      int32_t link;
      std::memcpy(&link, &bfs[16 * k + 12 + c], 4);
      if (link >= 0) { link = newidx[link]; std::memcpy(&bfs[16 * k + 12 + c], &link, 4); }
    }
  }
  R.nodes.swap(bfs);
  return R;
}

namespace {
void thread_node(const Result& R, int32_t node, std::vector<float>& out) {
  const float* n = &R.nodes[16 * (size_t)node];
  for (int c = 0; c < 2; ++c) {
    int32_t link;
    std::memcpy(&link, &n[12 + c], 4);
    if (link == (int32_t)~0u) continue;                  // empty child
    const size_t e = out.size();
    out.resize(e + 8);
    for (int k = 0; k < 6; ++k) out[e + k] = n[6 * c + k];
    const int32_t code = link < 0 ? link : -1;
    std::memcpy(&out[e + 6], &code, 4);
    if (link >= 0) thread_node(R, link, out);
    const int32_t skip = (int32_t)(out.size() / 8);
    std::memcpy(&out[e + 7], &skip, 4);
  }
}
}  // namespace

std::vector<float> threaded(const Result& R) {
  std::vector<float> out;
  if (!R.nodes.empty()) thread_node(R, 0, out);
  return out;
}

namespace {
struct Slot { Box b; int32_t link; };   // one child of a BVH4 node: padded box + BVH2 link

Slot child2(const Result& R, int32_t node, int c) {
  const float* n = &R.nodes[16 * (size_t)node];
  Slot s;
  for (int k = 0; k < 3; ++k) { s.b.lo[k] = n[6 * c + k]; s.b.hi[k] = n[6 * c + 3 + k]; }
  std::memcpy(&s.link, &n[12 + c], 4);
  return s;
}

struct Collapser {
  const Result& R;
  std::vector<std::vector<Slot>> kids;   // per BVH4 node (build order), its children (links are BVH2)

  // children of BVH2 node `node` opened up to four: the inner child of largest area is replaced by
  // its own two children while there is room (empty BVH2 children are dropped)
  std::vector<Slot> open(int32_t node) {
    std::vector<Slot> v;
    for (int c = 0; c < 2; ++c) { Slot s = child2(R, node, c); if (s.link != (int32_t)~0u) v.push_back(s); }
    for (;;) {
      int best = -1; float ba = -1.f;
      for (size_t k = 0; k < v.size(); ++k) {
        if (v[k].link < 0) continue;
        int grand = 0;
        for (int c = 0; c < 2; ++c) if (child2(R, v[k].link, c).link != (int32_t)~0u) ++grand;
        if (v.size() - 1 + grand > 4) continue;
        const float a = area(v[k].b);
        if (a > ba) { ba = a; best = (int)k; }
      }
      if (best < 0) break;
      const int32_t in = v[best].link;
      v.erase(v.begin() + best);
      for (int c = 0; c < 2; ++c) { Slot s = child2(R, in, c); if (s.link != (int32_t)~0u) v.insert(v.begin() + best + c, s); }
    }
    return v;
  }
};
}  // namespace

Result4 collapse4(const Result& R) {
  Result4 Q;
  if (R.nodes.empty()) return Q;
  Collapser C{R, {}};
  // breadth-first: BVH4 node q is opened from BVH2 node src[q]; its inner children get the next ids
  std::vector<int32_t> src{0}, lvl{0}, stk{0};
  for (size_t q = 0; q < src.size(); ++q) {
    std::vector<Slot> v = C.open(src[q]);
    const int pushes = (int)v.size() - 1 > 0 ? (int)v.size() - 1 : 0;
    float* nd;
    Q.nodes.resize(Q.nodes.size() + 28, 0.f);
    nd = &Q.nodes[28 * q];
    Q.depth = std::max(Q.depth, lvl[q] + 1);
    Q.stack_need = std::max(Q.stack_need, stk[q] + pushes);
    for (int k = 0; k < 4; ++k) {
      int32_t link = EMPTY4;
      if (k < (int)v.size()) {
        for (int a = 0; a < 3; ++a) { nd[4 * a + k] = v[k].b.lo[a]; nd[4 * (3 + a) + k] = v[k].b.hi[a]; }
        if (v[k].link >= 0) {
          link = (int32_t)src.size();
          src.push_back(v[k].link); lvl.push_back(lvl[q] + 1); stk.push_back(stk[q] + pushes);
        } else {
          link = v[k].link;
        }
      } else {
        for (int a = 0; a < 3; ++a) { nd[4 * a + k] = INF; nd[4 * (3 + a) + k] = -INF; }
      }
      std::memcpy(&nd[24 + k], &link, 4);
    }
  }
  return Q;
}

namespace {
// One axis of one node: the scale exponent e and the bytes of the (up to) four children.  e starts
// where 255 steps cover the extent and grows until every hi byte fits.
void quant_axis(const float* lo, const float* hi, const bool* used, float o, float* scale, uint32_t* wlo,
                uint32_t* whi) {
  double ext = 0.0;
  for (int k = 0; k < 4; ++k) if (used[k]) ext = std::max(ext, (double)hi[k] - (double)o);
  int e = -126;
  if (ext > 0.0) { std::frexp(ext / 255.0, &e); e = std::max(e - 1, -126); }
  for (;; ++e) {
    if (e > 119) throw std::runtime_error("BVH4 child box too large to quantize");
    const float s = std::ldexp(1.f, e);
    uint32_t bl = 0u, bh = 0u;
    bool ok = true;
    for (int k = 0; k < 4 && ok; ++k) {
      if (!used[k]) { bl |= 255u << (8 * k); continue; }
      double ql = std::floor(((double)lo[k] - (double)o) / s), qh = std::ceil(((double)hi[k] - (double)o) / s);
      int64_t a = (int64_t)std::max(0.0, std::min(ql, 255.0)), b = (int64_t)std::max(0.0, std::min(qh, 256.0));
      while (a > 0 && dequant((uint32_t)a, s, o) > lo[k]) --a;
      while (b <= 255 && dequant((uint32_t)b, s, o) < hi[k]) ++b;
      if (b > 255 || dequant((uint32_t)a, s, o) > lo[k]) { ok = false; break; }
      bl |= (uint32_t)a << (8 * k);
      bh |= (uint32_t)b << (8 * k);
    }
    if (ok) { *scale = s; *wlo = bl; *whi = bh; return; }
  }
}
}  // namespace

std::vector<uint32_t> quantize4(const Result4& Q) {
  const size_t n = Q.nodes.size() / 28;
  std::vector<uint32_t> out(16 * n, 0u);
  for (size_t q = 0; q < n; ++q) {
    const float* nd = &Q.nodes[28 * q];
    uint32_t* w = &out[16 * q];
    bool used[4];
    for (int k = 0; k < 4; ++k) {
      int32_t link;
      std::memcpy(&link, &nd[24 + k], 4);
      used[k] = link != EMPTY4;
      std::memcpy(&w[12 + k], &link, 4);
    }
    for (int a = 0; a < 3; ++a) {
      float o = INF;
      for (int k = 0; k < 4; ++k) {
        if (!used[k]) continue;
        if (!std::isfinite(nd[4 * a + k]) || !std::isfinite(nd[4 * (3 + a) + k]))
          throw std::runtime_error("BVH4 child box with non-finite bounds");
        o = std::min(o, nd[4 * a + k]);
      }
      if (o == INF) o = 0.f;                      // a node without children (empty scene root)
      float s;
      quant_axis(&nd[4 * a], &nd[4 * (3 + a)], used, o, &s, &w[6 + a], &w[9 + a]);
      std::memcpy(&w[a], &o, 4);
      std::memcpy(&w[3 + a], &s, 4);
    }
  }
  return out;
}

}  // namespace bvh
