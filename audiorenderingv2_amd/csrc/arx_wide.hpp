// arx_wide.hpp -- the 4-wide compressed tree (CW4, arx_layout.hpp): host collapse of the BVH2 and
// the quantization shared by the host and the device kernels (arx_receiver.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "arx_bvh.hpp"
#include "arx_layout.hpp"

namespace arx {

// One CW4 node from its f32 form for grid g: child boxes onto the 16-bit grid (quantize_nodes16's
// outward arithmetic and 0.1-step margin), then onto the node's own 6-bit frame (outward again).
// False if a box leaves the grid (its planes then span the whole frame: still conservative).
__host__ __device__ inline bool quantize_w4(const W4NodeF& n, const QGrid& g, QNode4C& out) {
    int32_t glo[4][3], ghi[4][3];
    int32_t flo[3] = {1 << 30, 1 << 30, 1 << 30}, fhi[3] = {0, 0, 0};
    bool ok = true, any = false;
    for (int c = 0; c < 4; ++c) {
        const bool used = ((n.meta >> (2 * c)) & 3u) != 0u;
        for (int k = 0; k < 3; ++k) {
            int32_t l = 0, h = 0;
            if (used) {
                const double dl = floor(((double)n.lo[c][k] - (double)g.origin[k]) / (double)g.scale[k] - 0.1);
                const double dh = ceil(((double)n.hi[c][k] - (double)g.origin[k]) / (double)g.scale[k] + 0.1);
                if (!(n.lo[c][k] <= n.hi[c][k]) || !(dl >= 0.0) || !(dh <= 65535.0)) {
                    ok = false;
                    l = 0;
                    h = 65535;
                } else {
                    l = (int32_t)dl;
                    h = (int32_t)dh;
                }
                flo[k] = flo[k] < l ? flo[k] : l;
                fhi[k] = fhi[k] > h ? fhi[k] : h;
            }
            glo[c][k] = l;
            ghi[c][k] = h;
        }
        any = any || used;
    }
    uint32_t o[3], e[3];
    for (int k = 0; k < 3; ++k) {
        if (!any) flo[k] = fhi[k] = 0;
        o[k] = (uint32_t)flo[k] >> 2;
        const int32_t ext = fhi[k] - 4 * (int32_t)o[k];
        uint32_t ek = 2;
        while ((63 << ek) < ext) ++ek;  // ext <= 65538 -> ek <= 11
        e[k] = ek;
    }
    for (int i = 0; i < 8; ++i) out.w[i] = 0u;
    out.w[0] = o[0] | (o[1] << 14) | (e[0] << 28);
    out.w[1] = o[2] | (e[1] << 14) | (e[2] << 18) | ((n.meta & 0xFFu) << 22);
    for (int c = 0; c < 4; ++c) {
        if (((n.meta >> (2 * c)) & 3u) == 0u) continue;
        for (int k = 0; k < 3; ++k) {
            const int32_t b = 4 * (int32_t)o[k];
            const uint32_t ql = (uint32_t)(glo[c][k] - b) >> e[k];
            const uint32_t qh = (uint32_t)(ghi[c][k] - b + (1 << e[k]) - 1) >> e[k];
            const int s0 = 6 * c + 2 * k, s1 = s0 + 1;
            out.w[2 + s0 / 5] |= ql << (6 * (s0 % 5));
            out.w[2 + s1 / 5] |= qh << (6 * (s1 % 5));
        }
    }
    out.w[7] = n.base;
    return ok;
}

// A CW4 tree laid out in the 16-B-unit buffer (one part of wbuf: the scene's, or the receiver's).
struct W4Build {
    std::vector<W4NodeF> nodes;   // nodes[0] = the part's root (at unit root_unit)
    std::vector<int32_t> src;     // per node, 8 ints: the BVH2 (ref, count) of each child slot
    std::vector<std::pair<uint32_t, int32_t>> leaf_tris;  // (unit, index into the BVH2 build's tris)
    uint32_t unit_end = 0;        // first unit after this part
    int depth = 0;                // CW4 levels on the longest root path
};

// Collapse a BVH2 build (node refs global: nodes[ref - node_base]; leaf refs index b.tris minus
// tri_base) under `root` into CW4 nodes: each node takes its BVH2 children and opens the largest
// (surface area) inner child or leaf of more than 2 triangles until it holds 4; remaining inner
// children become CW4 nodes, leaves of <= 2 triangles become leaf slots.  The root node is placed
// at root_unit, blocks are allocated breadth first from first_unit.
void collapse_w4(const BvhBuild& b, int32_t node_base, int32_t tri_base, const ChildRef& root, uint32_t root_unit,
                 uint32_t first_unit, W4Build& out);

}  // namespace arx
