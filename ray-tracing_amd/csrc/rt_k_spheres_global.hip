// rt_k_spheres_global.hip — the spheres-only variant's 4-wide kernel that reads the tree from global memory
// (worlds whose tree does not fit the LDS: config 5), in a unit of its own so that it is built without the
// opaque Philox key that the spheres unit sets (RT_PHILOX_OPAQUE_KEY, rt_device.h: C5 +0.5 % with it). The
// kernels live in an anonymous namespace, so each unit's instantiations are its own.
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
