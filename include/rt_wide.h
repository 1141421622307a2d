// rt_wide.h — the device's 4-wide BVH record (internal; shared by the host builder in rt_bvh.cpp
// and the traversal in rt_trace.h). Not part of the C ABI: rt_upload_scene derives it from the
// flattened world tree when the world holds no ConstantMedium and no instance frames.
//
// One record is 128 bytes = one LDS/L2 line pair: four child boxes as single-precision rows
// (lo[axis][child], hi[axis][child]), rounded OUTWARD from the fp64 boxes so that each box
// contains the double-precision one, then four child references. The fp32 test over these boxes
// only culls (it accepts every ray the fp64 slab test over the same boxes accepts, see
// wide_keys2 in rt_trace.h); every leaf is still hit-tested in fp64 exactly as the reference.
#pragma once
#include <stdint.h>

#define RT_WIDE 4

typedef struct rt_wnode {
  float lo[3][RT_WIDE];
  float hi[3][RT_WIDE];
  int32_t child[RT_WIDE];  // >= 0: wide node id; < 0: leaf, ~child = flat rt_node id (an unused
                           // slot: empty box lo = +inf, hi = -inf over a leaf of this node)
  int32_t pad[RT_WIDE];
} rt_wnode;

// The same node with its child boxes quantised to 8 bits per plane against a per-node grid (64 bytes:
// half an L2 line; the kernels that read the tree from global memory, where the 100k-sphere world's
// nodes and leaves do not fit an XCD's L2). Per axis a, plane q of child k is origin[a] + q * scale[a]
// exactly in fp32: scale is a power of two and origin an integer multiple of it below 2^23 * scale, so
// the decoded boxes are fp32 planes containing the node's fp32 boxes (lo rounded down, hi up to the grid)
// and the fp32 test over them culls conservatively, as over rt_wnode's. qlo[a] / qhi[a] hold child k's
// lower / upper plane in byte k. An unused slot has qlo 255 and qhi 0 on every axis (an empty box) and
// refers to a leaf of this node, as in rt_wnode.
typedef struct rt_qnode {
  float origin[3];
  float scale[3];
  uint32_t qlo[3];
  uint32_t qhi[3];
  int32_t child[RT_WIDE];
} rt_qnode;

#ifdef __cplusplus
static_assert(sizeof(rt_wnode) == 128, "rt_wnode is 128 bytes");
static_assert(sizeof(rt_qnode) == 64, "rt_qnode is 64 bytes");
#endif
