// rt_k_spheres_global.hip — the spheres-only variant's 4-wide kernel that reads the tree from global memory
// (worlds whose tree does not fit the LDS: config 5), in a unit of its own so that it can be built with the
// rare-fallback branches marked unlikely (RT_COLD_BRANCHES, rt_device.h): C5 -1.2 % (same images); the
// LDS-staged kernel of the same variant (C2) is 0.4 % slower with them and stays in rt_k_spheres.hip. The
// kernels live in an anonymous namespace, so each unit's instantiations are its own.
#define RT_COLD_BRANCHES 1
#include "rt_kernels.h"

namespace rt {
const void* philox_kernel_spheres_global(int w) {
  constexpr unsigned V = kVarSpheres | F_WIDE;
  if (w == 2) return (const void*)render_philox2<V, 2>;
  if (w == 4) return (const void*)render_philox2<V, 4>;
  if (w == 1) return (const void*)render_philox2<V, 1>;
  return (const void*)render_philox2<V, 3>;
}
}  // namespace rt
