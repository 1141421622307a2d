// rt_prepare.h — the host half of rt_upload_scene (rt_prepare.cpp): a validated, tagged device copy of
// a scene descriptor, ready to be copied to HBM. No HIP.
#pragma once
#include <vector>

#include "rt.h"
#include "rt_internal.h"
#include "rt_layout.h"
#include "rt_wide.h"

namespace rt {

struct PreparedScene {
  std::vector<rt_node> nodes;     // device node array: the caller's nodes + the rebuilt tree, type flags
                                  // (RT_CHAIN_PRIM), RT_ISBOX child tags, RT_WROOT marks (mixed walks)
  std::vector<rtd::DMat> mats;    // device materials
  std::vector<rt_wnode> wnodes;   // 4-wide trees: the world's (media-free worlds) or the re-bounded subtrees'
  std::vector<rt_node> leaves;    // their leaf table (c = flat node id)
  // spheres-only worlds with a 4-wide world tree: the same tree quantised (rt_qnode, 64 B) and the leaf
  // table's spheres as (center, radius) quadruples, for the kernels that read them from global memory
  std::vector<rt_qnode> qnodes;
  std::vector<double> sleaves;
  int world = 0, world_ref = 0;   // walk roots (with RT_ISBOX): the device tree's and the caller's
  int world_root = 0;             // the device tree's root id (untagged)
  int lights = -1;
  unsigned features = 0;          // rtd::F_* bits of the scene (+ F_FRAMES)
  int stack_need = 0;             // binary / mixed walk stack bound (entries)
  int frame_depth = 0;            // deepest nesting of instance frames (the device tree's or the caller's)
  int wide_stack_need = 0;        // 4-wide walk stack bound
  bool rebuilt_bvh = false, mixed_wide = false, replace_ok = false, ref_walk = false;
  bool w8 = false;                // wnodes hold the 8-wide tree as record pairs (RTAMD_W8=1, A/B; F_W8)
};

// Validates `desc` and prepares its device copy (RT_OK, or an error code with rt_last_error set).
int prepare_scene(const rt_scene_desc* desc, uint32_t flags, PreparedScene& out);

}  // namespace rt
