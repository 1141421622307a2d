// rt_internal.h — host-side helpers shared by the C-ABI translation units (not installed).
#pragma once
#include <cstdint>
#include <map>
#include <string>
#include <vector>

#include "rt.h"

namespace rt {

// splitmix-0.1 (System.Random.SplitMix): mix64 is the MurmurHash3 finaliser, mixGamma uses
// Stafford's variant 13 (the reverse of Java's SplittableRandom).
inline uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 33)) * 0xff51afd7ed558ccdULL;
  z = (z ^ (z >> 33)) * 0xc4ceb9fe1a85ec53ULL;
  return z ^ (z >> 33);
}
inline uint64_t mix64v13(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
inline uint64_t mix_gamma(uint64_t z) {
  z = mix64v13(z) | 1ULL;
  const int n = __builtin_popcountll(z ^ (z >> 1));
  return n >= 24 ? z : (z ^ 0xaaaaaaaaaaaaaaaaULL);
}
// mkStdGen n = StdGen (mkSMGen (fromIntegral n))  (random-1.2.0; src/Random.hs:20-21)
inline void mk_smgen(uint64_t s, uint64_t out[2]) {
  out[0] = mix64(s);
  out[1] = mix_gamma(s + 0x9e3779b97f4a7c15ULL);
}
// nextWord64
inline uint64_t sm_next(uint64_t& seed, uint64_t gamma) {
  seed += gamma;
  return mix64(seed);
}
// random-1.2.0 `random :: Double` = 1 - word64 / 2^64 (src/Random.hs:23-25)
inline double word_to_draw(uint64_t w) { return 1.0 - (double)w / 18446744073709551616.0; }

void set_error(const std::string& s);
const char* last_error();

struct Box {
  double mn[3], mx[3];
};

// Traversal-stack entries a BVH node needs (rt_trace.h traverse / walk_step), given its
// children's needs. Caller's (makeBVH) nodes are walked left first, with b waiting on the stack
// while a is walked (hit BVHNode, src/Lib.hs:971-988). A rebuilt node (RT_BVH_ORDERED) enters the
// child on the ray's side of the split first, so either child can be walked above the other.
inline int bvh_stack_need(const rt_node& x, int need_a, int need_b) {
  // (either child first; an RT_BVH_MEDIA_FIRST node enters its left child first, like a reference node)
  if ((x.c & RT_BVH_ORDERED) && !(x.c & RT_BVH_MEDIA_FIRST)) return 1 + (need_a > need_b ? need_a : need_b);
  return (1 + need_a > need_b) ? 1 + need_a : need_b;
}

}  // namespace rt

struct rt_builder {
  uint64_t seed, gamma;  // RandGen (SMGen)
  std::vector<rt_node> nodes;
  std::vector<rt_material> materials;
  std::vector<rt_texture> textures;
  std::vector<rt_perlin> perlins;
  std::vector<rt_image> images;
  std::vector<uint8_t> pool;
  std::map<int, rt::Box> rotate_boxes;  // Rotate's stored box (src/Lib.hs:733)
  bool failed = false;

  // randomDoubleM (src/Lib.hs:1119-1125) over random-1.2.0 / splitmix-0.1
  double draw() { return rt::word_to_draw(rt::sm_next(seed, gamma)); }
  double draw_r(double mn, double mx) { double rd = draw(); return mn + (mx - mn) * rd; }
};
