// arx_bvh.hpp -- host-side SAH BVH builder (replaces optixAccelBuild/optixAccelCompact,
// R/prebuild/obj_raytracer/AudioRenderer.cpp:179-208).
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

#include "arx_layout.hpp"

namespace arx {

struct ChildRef {
    float lo[3], hi[3];  // padded box
    int32_t ref;         // inner: node index; leaf: first triangle
    int32_t count;       // 0 = inner node
};

struct BvhBuild {
    std::vector<BvhNode> nodes;  // indices local to this build
    std::vector<TriRec> tris;    // leaf order, indices local to this build
    ChildRef root;
    int depth = 0;
};

// SAH build parameters (process-wide; the defaults are the production setting, design tools
// such as tools/bvh_stats.cpp vary them).
// The defaults below were picked on the C3 trace (profiles/r02/ab_sah.log): 128
// object and 128 spatial bins, leaves of at most 2 triangles and spatial splits tried down to an
// overlap of 1e-5 of the root area run ≈7 % faster than 32 / 32 / leaves <= 4 / 1e-3 (node step
// priced at one triangle test: 1.1 % faster than 0.8 over three paired runs at these settings).  Design experiments (build.py --exp TAG -D ARX_SAH_TRAV=...) vary them; the
// product build takes none of these macros.
#ifndef ARX_SAH_TRAV
#define ARX_SAH_TRAV 1.0f
#endif
#ifndef ARX_BVH_ROTATIONS
#define ARX_BVH_ROTATIONS 8
#endif
#ifndef ARX_SAH_LEAF_MAX
#define ARX_SAH_LEAF_MAX 2
#endif
#ifndef ARX_SAH_BINS
#define ARX_SAH_BINS 128
#endif
#ifndef ARX_SAH_SPATIAL_BINS
#define ARX_SAH_SPATIAL_BINS 128
#endif
#ifndef ARX_SAH_SPATIAL_ALPHA
#define ARX_SAH_SPATIAL_ALPHA 1e-5f
#endif
#ifndef ARX_SAH_SPATIAL_BUDGET
#define ARX_SAH_SPATIAL_BUDGET 3.0f
#endif
struct BuildParams {
    int bins = ARX_SAH_BINS;           // centroid bins per axis (<= 256)
    int leaf_max = ARX_SAH_LEAF_MAX;  // SAH may stop at <= leaf_max triangles (always splits above)
    float trav_cost = ARX_SAH_TRAV;   // SAH cost of a node step relative to ...
    float isect_cost = 1.0f; // ... one triangle test
    // Spatial splits (SBVH, Stich, Friedrich & Dietrich 2009): a triangle may be referenced by
    // several leaves, each bounding only its clipped part.  Tried at nodes whose best object
    // split leaves children overlapping by more than spatial_alpha of the root's area, while
    // the references stay below (1 + spatial_budget) x the triangle count.
    bool spatial = true;
    int spatial_bins = ARX_SAH_SPATIAL_BINS;  // split planes per axis (<= 256)
    float spatial_alpha = ARX_SAH_SPATIAL_ALPHA;
    float spatial_budget = ARX_SAH_SPATIAL_BUDGET;
    int spatial_max_depth = 64;  // spatial splits only above this depth
    // Depth cap of the spatial builder: once depth + log2(refs / leaf_max) reaches it, nodes are
    // split at the object median of their widest centroid axis, so every leaf sits at depth <=
    // max_depth (the kernel's 28-entry LDS stack then needs no spill path).
    int max_depth = kLdsStack - 2;
    int threads = 8;  // top-level subtrees built concurrently (spatial builder)
    // Tree rotations after the spatial build (Kensler 2008): passes over the tree, top down, each
    // node swapping its smaller-area side's child with a grandchild when that shrinks the inner
    // node between them, never deepening the tree past its built depth.  On the C3 scene: inner-
    // node SAH -2.7 %, node visits per query -3.7 % (tools/bvh_stats.cpp).
    int rotation_passes = ARX_BVH_ROTATIONS;
};
// Process-wide parameters: production defaults, never read from the environment; design tools
// (tools/bvh_stats.cpp, tools/bvh_check.cpp) edit the struct before building.
BuildParams& build_params();

// tri_v: n*9 floats, tri_abs: n floats (may be nullptr -> absorption_fill).
void build_bvh(const float* tri_v, const float* tri_abs, float absorption_fill, int64_t n, int32_t id_base,
               BvhBuild& out);
// Shift all node / triangle references by the given offsets (placing the build inside a
// bigger array).  The root reference is shifted too.
void relocate_bvh(BvhBuild& b, int32_t node_offset, int32_t tri_offset);
// Tree rotations on a finished build (BuildParams::rotation_passes; the spatial builder runs them).
void rotate_tree(BvhBuild& b, int passes);
// Renumber the nodes so the first k inner nodes in breadth-first order from the root take
// indices 0..k-1 (the rest keep their order, so parents still precede their children): the
// top levels of the scene tree share cache lines.
void bfs_prefix_order(BvhBuild& b, size_t k);
BvhNode make_node(const ChildRef& c0, const ChildRef& c1);
ChildRef empty_child();
// Structural check of a device-ready node array (acyclic, references in range).
bool validate_bvh(const BvhNode* nodes, size_t n_nodes, size_t n_tris, const char** why);
// Same check for nodes [first, first + n_nodes) of an array of total_nodes (`nodes` points at node
// `first`), so a listener move re-validates only the receiver sub-tree and the top node.
bool validate_bvh_range(const BvhNode* nodes, size_t first, size_t n_nodes, size_t total_nodes, size_t n_tris,
                        const char** why);
// Coded copy of validated nodes for the coded node step: d = (code0, code1, 0, 0) with
// code = inner node index (>= 0), ~(first*16 + count) for a leaf (< 0; the traversal-stack
// entry format), or kEmptyChildCode for an empty child: a leaf of 0 triangles, i.e. a no-op if
// its inverted box ever passes the slab test (-1 is kept free: it means "no entry").  Boxes are
// unchanged.
void code_nodes(const BvhNode* in, size_t n, BvhNode* out);
// Grid for QNode2 trees covering the box [lo, hi] (scene, receiver and emitter) with a margin
// of margin_frac of the largest extent on every side, so listener moves inside the room keep
// the grid.
QGrid make_qgrid(const float lo[3], const float hi[3], double margin_frac = 0.1);
// True if the box [lo, hi] lies inside the grid with room for the outward rounding.
bool qgrid_contains(const QGrid& g, const float lo[3], const float hi[3]);
// Quantized copy of coded nodes: every child box is rounded outward to the grid with a margin of
// 0.1 step (for the kernel's f32 slab arithmetic, see arx_trace.hip node_step7);
// empty children become a one-step box at the grid corner.  False if a box leaves the grid.
bool quantize_nodes16(const BvhNode* coded, size_t n, const QGrid& g, QNode2* out);
}  // namespace arx
