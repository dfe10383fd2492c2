// arx_layout.hpp -- HBM data layout shared by the host builder and the HIP kernels.
//
// Scene (replaces the OptiX GAS + SBT, AudioRenderer.cpp:95-218, 413-464):
//   tris  : TriRec[n_scene + n_receiver], 48 B each, in BVH leaf order so a leaf is a
//           contiguous range (3 x 16-B loads per triangle, no index indirection).
//           v0.w = absorption (SBT mat_absorption), v1.w = global triangle id (tie-break).
//   nodes : BvhNode[] (host build, 64 B) -> coded copy (f32 fallback) and QNode2[] (32 B, the
//           default).  Node 0 is a fixed top node whose two children are the static-scene root
//           and the receiver root, so a listener move rewrites only the receiver sub-tree and
//           node 0.
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

// 16-bit quantized binary node, 32 B (2 x 16-B loads instead of 3.5 for the f32 node): the
// coded node (code_nodes) with both child boxes on one scene-wide 16-bit grid per axis,
// plane = grid.origin + q * grid.scale (real arithmetic), rounded outward with a kQ16Margin-step
// margin so the kernel's f32 slab arithmetic stays conservative (quantize_nodes16, arx_bvh.cpp).
// Each 16-B half is one child: q[0..2] = x, y, z as (lo | hi << 16), code as in code_nodes.
struct QChild {
    uint32_t q[3];
    int32_t code;
};
struct alignas(16) QNode2 {
    QChild c[2];
};
static_assert(sizeof(QNode2) == 32, "QNode2 must be 32 B");

// ---- 4-wide compressed tree (CW4) ------------------------------------------------------------
// The BVH2 collapsed to 4 children per node (arx_wide.cpp).  Nodes and leaf triangles live in one
// buffer of 16-B units (wbuf): node N's children form one block at N.base -- its inner children's
// nodes (2 units each) first, then its leaves' triangle records (3 units each, TriRec), so one
// 32-bit base addresses both.  A node is 32 B = two 16-B loads (QNode2 needs two as well, for two
// children instead of four):
//   w0 = ox | oy << 14 | ex << 28          frame origin (units of 4 grid quanta) and exponents:
//   w1 = oz | ey << 14 | ez << 18 | meta << 22   axis k spans 4*o_k + [0, 63 * 2^e_k] grid quanta
//   w2..w6: 24 six-bit planes, five per word at bits 0, 6, 12, 18, 24; child c's planes are
//           slots 6c .. 6c+5 = x lo, x hi, y lo, y hi, z lo, z hi (plane = 4*o + q * 2^e)
//   w7 = base (16-B units)
// meta: 2 bits per child slot: 0 empty, 1 inner, 2 leaf of 1 triangle, 3 leaf of 2; inner slots
// come first, then leaves, then empties.  Planes round the padded f32 boxes outward onto the
// 16-bit grid with the 0.1-step margin of QNode2, then outward again onto the node's 6-bit frame,
// so culling stays conservative.
constexpr int kW4Units = 2;  // 16-B units per node
constexpr int kTriUnits = 3;  // 16-B units per TriRec
struct alignas(16) QNode4C {
    uint32_t w[8];
};
static_assert(sizeof(QNode4C) == 32, "QNode4C must be 32 B");

// The grid-independent f32 form of a CW4 node, kept on the device so that a new grid re-quantizes
// every node there (launch_requant_w4): four padded child boxes, the meta bits, the block base and
// the node's own unit.
struct alignas(16) W4NodeF {
    float lo[4][3];
    float hi[4][3];
    uint32_t meta;
    uint32_t base;
    uint32_t self;
    uint32_t pad;
};
static_assert(sizeof(W4NodeF) == 112, "W4NodeF must be 112 B");

// Stack-entry / child code of an empty child in the coded and quantized nodes (code_nodes,
// arx_bvh.hpp): a leaf of 0 triangles (-1 is kept free: it means "no entry").
constexpr int32_t kEmptyChildCode = ~16;

// Outward rounding margin of QNode2 planes, in grid steps (quantize_nodes16 and its device twins in
// arx_receiver.hip).  The trace kernel forms a plane as the float 2^23 + q straight from its bits and
// computes t = fma(2^23 + q, ix, -C) with C = 2^23 * ix + (o - origin) * inv rounded once: that
// rounding is at most half an ulp of C <= 0.504 step, plus < 0.02 step for the other roundings
// (|t| <= 2^16 steps), so 0.75 step keeps every slab conservative.  A step is 1/65000 of the grid.
constexpr double kQ16Margin = 0.75;

// The scene-wide grid of QNode2 trees.
struct QGrid {
    float origin[3];
    float scale[3];
};

// LDS traversal stack rows per lane of the trace kernel; trees with bvh_depth >= kLdsStack take
// the global-memory stack instance of the same kernel.  The SBVH builder caps its depth at 26
// (BuildParams::max_depth), so the production scenes always fit the LDS stack.
#ifndef ARX_LDS_STACK
#define ARX_LDS_STACK 28  // design experiments only (build.py --exp); BuildParams::max_depth follows it
#endif
constexpr int kLdsStack = ARX_LDS_STACK;
constexpr int kMaxBuildDepth = 62;
constexpr int kSpeedOfSound = 343;  // devicePrograms.cu:13

// Trace kernel arguments (passed by value; lives in kernarg/SGPRs).
struct TraceArgs {
    const BvhNode* cnodes;          // coded nodes (code_nodes): f32 boxes, d = (code0, code1, 0, 0)
    const QNode2* qnodes;           // 16-bit quantized copy (same indices); null: use cnodes
    QGrid qgrid;
    const TriRec* tris;
    unsigned long long* hist;       // [2*ir_len] int64 fixed point, L then R
    unsigned long long* counters;   // [0] queries [1] receiver hits [2] misses [3] error flag
    const void* dirs;               // float4 per-ray directions of [ray_begin, ray_end) (direction pre-pass)
    int32_t* gstack;                // global traversal stack [rows][gstack_lanes] (deep trees only)
    uint64_t gstack_lanes;
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
    int32_t bvh_depth;   // inner levels on the longest root path (top node included) = max stack use
    unsigned long long* prof;  // per-wave records of a profiling build (ARX_TRACE_PROF); null otherwise
    const void* wbuf;          // CW4 buffer (nodes + leaf triangles, 16-B units); null: a BVH2 path
    unsigned long long* cursor;  // the launch's ray-pool cursor (reset by the direction pre-pass)
    uint32_t dyn_share;          // rays in the pool: n * dyn_share / 256 (set by launch_trace)
    uint32_t dyn_chunk;          // rays per pool atomic
    uint64_t clear_bins;         // > 0: the direction pre-pass also zeroes hist[0, clear_bins) ...
    int32_t clear_counters;      // ... and counters[0, clear_counters) (render(): no separate clear launch)
};
// Node formats of the trace kernel (arx_stats::trace_format)
constexpr int kFmtF32 = 0, kFmtQ16 = 1, kFmtW4 = 2;
// Per-wave record of a profiling build (ARX_TRACE_PROF=1, arx_debug_trace_profile): u64 words
constexpr int kProfWords = 16;

}  // namespace arx
