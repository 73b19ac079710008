// sphere_bvh.h — host-built bounding-volume hierarchy over the scene spheres.
//
// The reference tests every sphere for every ray (check_spheres,
// compute_shader.wgsl:355-404). The kernel instead walks this BVH and tests
// only the spheres in boxes the ray can reach, with boxes inflated by a per-ray
// margin that provably covers the f32 rounding of the reference's formula
// (DESIGN.md §5.2), so the closest sphere — and with the (t, index)
// lexicographic minimum, the tie winner — is exactly the one the brute-force
// sweep finds.
#pragma once
#include <stdint.h>

#include <vector>

#include "rt_abi.h"

// 32-byte node, depth-first order. Internal: left child = this + 1, right child
// follows the left subtree. `skip` = first node after this subtree.
struct SphereBvhNode {
    float bmin[3];
    uint32_t skip;
    float bmax[3];
    uint32_t leaf;  // kSphereBvhInternal, or first_slot | (count << 24)
};
static_assert(sizeof(SphereBvhNode) == 32, "node layout");

constexpr uint32_t kSphereBvhInternal = 0xffffffffu;
constexpr uint32_t kSphereBvhLeafMax = 4;
// The kernel tests spheres in aligned groups of 4 slots (one leaf = one group);
// unused slots hold a NaN sphere that no ray hits, and this original index.
constexpr uint32_t kSphereGroup = 4;
constexpr uint32_t kSphereDummyOrig = 0xffffffffu;

struct SphereSlots {
    // Spheres in kernel order: the brute-force ("always") set first, in
    // original index order (n_always slots, swept in groups of 4 and then one by
    // one), padding to a group boundary, then the BVH leaves' spheres in leaf
    // order, each leaf one padded group of kSphereGroup slots (at most
    // 4 * count + 4 slots in all).
    uint32_t n_always = 0;            // brute-force slots (not padded)
    std::vector<float> slot_sph;        // 4 per slot: centre.xyz, radius*radius
    std::vector<uint32_t> slot_orig;    // original sphere index of each slot
    std::vector<SphereBvhNode> nodes;   // empty when every sphere is brute-forced
    float extent = 0.0f;                // max over BVH spheres of |centre| + radius (rounded up)
    float r_min = 0.0f, r_max = 0.0f;   // radius range over BVH spheres (rounded down / up)
};

// Build the slot layout for the first `count` spheres. With `use_bvh` false (or
// too few spheres to pay off) every sphere is in the brute-force set.
void build_sphere_slots(const rt_scene_sphere* spheres, uint32_t count, bool use_bvh, SphereSlots* out,
                        uint32_t leaf_max = kSphereBvhLeafMax);

// Direction-ordered copies of a depth-first BVH (same boxes and leaves): layout
// k (k = octant of the ray direction: bit 0 set if d.x < 0, bit 1 d.y, bit 2 d.z)
// lists, at every internal node, first the child that a ray of that octant
// reaches first along the axis that separates the two children's centres
// most, so the stackless skip walk visits near children first and its
// distance pruning starts early. The 8 layouts are concatenated (node indices
// and skips absolute); a skip that leaves a layout is 8 * nodes.size(), so
// "node >= total" ends every walk. Visiting order does not change the result
// (the lexicographic minimum, conservative pruning).
// With swap_boxes, layout k also stores every box as (near corner, far corner)
// for its octant (bmin/bmax swapped on the axes of k's set bits), for the
// min/max-free slab test (rt_bvh_slab.h: slab_hit_ordered); layout 0 is
// unchanged either way. Only valid when box_layout_orderable(in).
// src (optional) receives, per output node, the index of its node in `in` (the
// device re-derives the layouts from `in` after a refit: rt_derive_tri_octants).
void order_bvh_by_octant(const std::vector<SphereBvhNode>& in, std::vector<SphereBvhNode>* out,
                         bool swap_boxes = false, std::vector<uint32_t>* src = nullptr);

// Every box is valid (bmin <= bmax) with finite coordinates of magnitude
// <= 1e8, so that no plane * (1/d, capped at 1e30) overflows: the premise of
// slab_hit_ordered's equivalence with slab_hit.
bool box_layout_orderable(const std::vector<SphereBvhNode>& nodes);

// Generic builder: binned-SAH BVH over axis-aligned boxes (lo/hi, 3 floats each
// per primitive), leaves of at most `leaf_max` primitives. Returns depth-first
// nodes (same layout as SphereBvhNode; leaf = first | count << 24 indexing
// `leaf_order`) and the primitive order of the leaves.
// Subtrees that would reach below `max_depth` levels are split at the median
// instead (balanced: a subtree of n primitives is then ceil(log2 n) levels deep).
void build_box_bvh(const std::vector<float>& lo, const std::vector<float>& hi, uint32_t leaf_max,
                   std::vector<SphereBvhNode>* nodes, std::vector<uint32_t>* leaf_order,
                   uint32_t max_depth = 0xffffffffu);

// Triangle side (check_triangles, compute_shader.wgsl:422-517). One primitive
// per (object, sub-object) pair the reference's sweep visits, in sweep order.
struct SubObjectPrim {
    uint32_t object;    // object index (ray_in_bounds on its box, :431)
    uint32_t sub;       // sub-object index (ray_in_bounds on its box, :441)
    uint32_t seq_base;  // position of the sub-object's first triangle in the reference's sweep order
    uint32_t range;     // first_triangle_index | triangle_count << 27 (kPrimRangeNone: read the sub-object)
};
constexpr uint32_t kPrimRangeNone = 0xffffffffu;
// The sub-object's triangle range packed into its leaf record when it fits (first < 2^27, count < 32),
// so a leaf test can start its triangle loads without the sub-object record (pathtrace.hip tri_leaf).
inline uint32_t prim_range(uint32_t first, uint32_t count) {
    return (first < (1u << 27) && count < 32u) ? (first | (count << 27)) : kPrimRangeNone;
}
static_assert(sizeof(SubObjectPrim) == 16, "prim layout");

struct TriangleAccel {
    std::vector<SubObjectPrim> prims;  // in BVH leaf order (one prim per leaf)
    std::vector<SphereBvhNode> nodes;
    float extent = 0.0f;  // max |coordinate| over sub-object boxes (rounded up)
};

// Build over the first `object_count` objects. Sub-objects with no triangles
// are left out (they can never produce a hit); non-finite boxes are kept with
// an all-enclosing box.
void build_triangle_accel(const rt_object_info* objects, uint32_t object_count, const rt_sub_object_info* subs,
                          uint32_t sub_count, TriangleAccel* out);

