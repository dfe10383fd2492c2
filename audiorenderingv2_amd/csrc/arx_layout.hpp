// arx_layout.hpp -- HBM data layout shared by the host builder and the HIP kernels.
//
// Scene (replaces the OptiX GAS + SBT, AudioRenderer.cpp:95-218, 413-464):
//   tris  : TriRec[n_scene + n_receiver], 48 B each, in BVH leaf order so a leaf is a
//           contiguous range (3 x 16-B loads per triangle, no index indirection).
//           v0.w = absorption (SBT mat_absorption), v1.w = global triangle id (tie-break).
//   nodes : BvhNode[], 64 B each (4 x 16-B loads).  Node 0 is a fixed top node whose two
//           children are the static-scene root and the receiver root, so a listener move
//           rewrites only the receiver sub-tree and node 0.
// A child reference is (ref, count): count > 0 -> leaf of triangles [ref, ref+count);
// count == 0 -> inner node index ref.  Empty children carry an inverted box.
#pragma once
#include <cstdint>

namespace arx {

struct alignas(16) TriRec {
    float v0[3];
    float absorption;
    float v1[3];
    int32_t id;
    float v2[3];
    int32_t pad;
};
static_assert(sizeof(TriRec) == 48, "TriRec must be 48 B");

// Aila-Laine style node: both children's boxes side by side.
//   a = (c0.lo.x, c0.hi.x, c0.lo.y, c0.hi.y)
//   b = (c1.lo.x, c1.hi.x, c1.lo.y, c1.hi.y)
//   c = (c0.lo.z, c0.hi.z, c1.lo.z, c1.hi.z)
//   d = (c0.ref, c1.ref, c0.count, c1.count)
struct alignas(16) BvhNode {
    float a[4];
    float b[4];
    float c[4];
    int32_t d[4];
};
static_assert(sizeof(BvhNode) == 64, "BvhNode must be 64 B");

// Wide node (W = 4: 128 B = one L2 line; W = 8: 256 B), collapsed from the binary SAH tree.
// Boxes are stored per axis and bound (SoA) so one 16-B load brings the same plane of four
// children; ref/cnt as in BvhNode (cnt 0 inner, > 0 leaf, -1 empty slot).
template <int W>
struct alignas(16) WideNode {
    float lox[W], hix[W], loy[W], hiy[W], loz[W], hiz[W];
    int32_t ref[W];
    int32_t cnt[W];
};
static_assert(sizeof(WideNode<4>) == 128, "WideNode<4> must be 128 B");
static_assert(sizeof(WideNode<8>) == 256, "WideNode<8> must be 256 B");

// Quantized 4-wide node, 64 B (4 x 16-B loads), child boxes on an 8-bit grid per axis:
// plane = origin + q * 2^e (exact in real arithmetic), rounded outward when built so every
// child box contains its padded exact box (conservative; Ylitie et al. 2017 style).
//   dword 0-2 origin xyz (f32), dword 3 biased exponents ex | ey << 8 | ez << 16
//   dword 4-9 qlo.x, qhi.x, qlo.y, qhi.y, qlo.z, qhi.z: byte c = child c
//   dword 10 counts: byte c = 0 inner, 1..15 leaf, 0xFF empty;  dword 11 unused
//   dword 12-15 ref[4]: inner node index / first triangle
struct alignas(16) QNode4 {
    float origin[3];
    uint32_t exps;
    uint32_t q[6];
    uint32_t counts;
    uint32_t pad;
    int32_t ref[4];
};
static_assert(sizeof(QNode4) == 64, "QNode4 must be 64 B");
// Node-format code of QNode4 trees where a "width" is passed (2, 4, 8 are BvhNode / WideNode<W>).
constexpr int kWideQ4 = 5;

// 16-bit quantized binary node, 32 B (2 x 16-B loads instead of 3.5 for the f32 node): the
// coded node (code_nodes) with both child boxes on one scene-wide 16-bit grid per axis,
// plane = grid.origin + q * grid.scale (real arithmetic), rounded outward with a 0.1-step margin so
// the kernel's f32 slab arithmetic stays conservative (quantize_nodes16, arx_bvh.cpp).
// Each 16-B half is one child: q[0..2] = x, y, z as (lo | hi << 16), code as in code_nodes, so
// a lane pair can fetch a node with one 16-B load each (node_step8p).
struct QChild {
    uint32_t q[3];
    int32_t code;
};
struct alignas(16) QNode2 {
    QChild c[2];
};
static_assert(sizeof(QNode2) == 32, "QNode2 must be 32 B");

// 4-wide quantized node (variants 1000+): four QChild slots, child codes as in code_nodes (an
// inner code is a wide-node index).
struct alignas(16) QWide4 {
    QChild c[4];
};
static_assert(sizeof(QWide4) == 64, "QWide4 must be 64 B");

// The scene-wide grid of QNode2 trees.
struct QGrid {
    float origin[3];
    float scale[3];
};

// LDS traversal stack depth per lane; the builder caps tree depth below it.
constexpr int kStackDepth = 40;      // v1/v2 (A/B variants): trees up to depth 39
constexpr int kMaxStackDepth = 64;   // deepest stack variant of the default kernel
constexpr int kMaxBuildDepth = kMaxStackDepth - 2;
constexpr int kSpeedOfSound = 343;  // devicePrograms.cu:13

// Trace kernel arguments (passed by value; lives in kernarg/SGPRs).
struct TraceArgs {
    const BvhNode* nodes;
    const TriRec* tris;
    unsigned long long* hist;       // [2*ir_len] int64 fixed point, L then R
    unsigned long long* counters;   // [0] queries [1] receiver hits [2] misses [3] error flag
    uint64_t seed;
    uint64_t ray_begin;
    uint64_t ray_end;
    float emitter[3];
    float center[3];
    float e0;
    float energy_thres;
    float hrtf;
    float dist_limit;
    double inv_unit;
    uint32_t max_bounces;
    int32_t sample_rate;
    int32_t ir_len;
    int32_t delay;
    int32_t is_mono;
    int32_t max_visits;  // traversal guard: > number of inner nodes (each is visited at most once)
    int32_t bvh_depth;   // inner levels on the longest root path (top node included) = max stack use
    // wide-tree kernels (trace_width() > 2)
    const void* wnodes;  // WideNode<W>[], node 0 = top (scene root, receiver root)
    int32_t* spill;      // traversal-stack overflow beyond the LDS part: [depth][spill_lanes]
    uint64_t spill_lanes;
    int32_t stack_need;  // worst-case stack entries for this tree: (W-1) * wide depth + 2
    int32_t spill_depth; // set by the launcher: stack_need - LDS entries (>= 0)
    // phased launches (tail compaction): ray states parked between launches, 48 B each:
    // float4(pos, e), float4(dir, dist), int4(depth, 0, 0, 0)
    void* stash[2];
    unsigned long long* stash_count;  // [2] device counters
    uint64_t stash_cap;               // records per stash buffer
    // set by the launcher per phase: source pool (-1 = fresh ray ids) and drain threshold
    int32_t pool_from;   // -1 or 0/1: read states from stash[pool_from]
    int32_t drain_low;   // 0: never drain; else drain a wave once exhausted with < drain_low active lanes
    // refill options (kernel variants 700+): precomputed directions of rays [ray_begin, ray_end)
    // as float4(dir, 0), and static per-wave ray ranges instead of the global cursor
    const void* dirs;
    int32_t static_ranges;
    void* dirs_buf;      // capacity for the launcher's direction pre-pass (dirs_cap rays)
    uint64_t dirs_cap;
    // coded copy of `nodes` (code_nodes, arx_bvh.hpp): d = (code0, code1, 0, 0)
    const BvhNode* cnodes;
    // 16-bit quantized copy of cnodes (QNode2, same indices) and its grid; kernel variants
    // with quantized nodes fall back to cnodes when qnodes is null (see launch_v3)
    const QNode2* qnodes;
    QGrid qgrid;
    // octant copies (octant_nodes16): copy o of node i at qnodes[o * qostride + i], o = 0 plain
    uint32_t qostride;
    // quantized copy of the 4-wide tree (wnodes, variants 1000+), same grid; null: unusable
    const QWide4* qwnodes;
    uint32_t qcount;  // nodes in cnodes / qnodes (top + scene + receiver)
};

}  // namespace arx
