// arx_b16.hpp -- the compact binary tree (B16, arx_layout.hpp): one 16-B unit per BVH2 node.
//
// The 16-bit BVH2 (QNode2, 32 B) spends two 16-B loads per node step.  B16 keeps the same tree --
// the same nodes, children and child order, so the traversal visits what the BVH2 visits up to the
// looser boxes -- and stores each node in one unit: both children's boxes as 8-bit planes on a
// frame shared by the nodes of an aligned block of 2^kB16BlockBits units, and the children as one
// block base plus a 4-bit kind per child.  The 8-bit planes are the 16-bit planes rounded outward
// again, so culling stays conservative and every closest hit is the BVH2's.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "arx_layout.hpp"

namespace arx {

// Frame of one block, from the 16-bit child planes of the nodes that live in it: per axis the
// lowest plane `o` and the smallest e with every plane in o + [0, 255 * 2^e].
struct B16FrameAcc {
    uint32_t lo[3] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
    uint32_t hi[3] = {0u, 0u, 0u};
    __host__ __device__ void add(const QNode2& q, uint32_t w3) {
        for (int c = 0; c < 2; ++c) {
            if (((w3 >> (4 * c)) & 15u) == 0u) continue;  // empty child
            for (int k = 0; k < 3; ++k) {
                const uint32_t l = q.c[c].q[k] & 0xFFFFu, h = q.c[c].q[k] >> 16;
                lo[k] = l < lo[k] ? l : lo[k];
                hi[k] = h > hi[k] ? h : hi[k];
            }
        }
    }
    __host__ __device__ uint2 frame() const {
        uint32_t o[3], e[3];
        for (int k = 0; k < 3; ++k) {
            o[k] = lo[k] <= hi[k] ? lo[k] : 0u;
            const uint32_t ext = lo[k] <= hi[k] ? hi[k] - lo[k] : 0u;
            uint32_t ek = 0;
            while ((255u << ek) < ext) ++ek;  // ext <= 65535 -> ek <= 9
            e[k] = ek;
        }
        return make_uint2(o[0] | (o[1] << 16), o[2] | (e[0] << 16) | (e[1] << 20) | (e[2] << 24));
    }
};

// The unit of a B16 node: its QNode2's 16-bit planes onto the block frame f (outward), w3 as laid out.
__host__ __device__ inline uint4 b16_node(const QNode2& q, uint32_t w3, uint2 f) {
    const uint32_t o[3] = {f.x & 0xFFFFu, f.x >> 16, f.y & 0xFFFFu};
    const uint32_t e[3] = {(f.y >> 16) & 15u, (f.y >> 20) & 15u, (f.y >> 24) & 15u};
    uint32_t w[3];
    for (int k = 0; k < 3; ++k) {
        uint32_t word = 0u;
        for (int c = 0; c < 2; ++c) {
            uint32_t ql = 1u, qh = 0u;  // empty child: near > far on either ray direction
            if (((w3 >> (4 * c)) & 15u) != 0u) {
                const uint32_t l = q.c[c].q[k] & 0xFFFFu, h = q.c[c].q[k] >> 16;
                ql = (l - o[k]) >> e[k];
                qh = (h - o[k] + (1u << e[k]) - 1u) >> e[k];
            }
            word |= (ql | (qh << 8)) << (16 * c);
        }
        w[k] = word;
    }
    return make_uint4(w[0], w[1], w[2], w3);
}

// Layout of one part of the B16 buffer (the scene's, or the receiver's): which QNode2 each node
// unit holds and its w3, and the triangle records' units.  Nodes are placed breadth first; a
// node's children chunk goes into the node's own block while it has room, else it opens a new
// block (a chunk of leaves only may go into the current overflow block).
struct B16Build {
    std::vector<uint32_t> node_units;  // units of this part's nodes
    std::vector<int32_t> node_src;     // per node: its QNode2 index
    std::vector<uint32_t> node_w3;     // per node: kinds | base << 8
    std::vector<std::pair<uint32_t, int32_t>> tri_units;  // (first unit, TriRec index)
    std::vector<uint32_t> blocks;      // blocks this part owns (frames to compute)
    uint32_t unit_end = 0;             // first unit after this part's last block
};

// Lay out the tree under root_node (coded[i] is QNode2 index node_base + i; children codes in d[0..1]
// as code_nodes writes them) with the root at root_unit.  The root's chunk goes into the root's
// block from unit `fill` on if fill is not 0, else into a new block; new blocks start at first_block.
// False (why set) if a leaf holds more triangles than a kind can say or the buffer outgrows the
// 24-bit base.
bool layout_b16(const BvhNode* coded, int32_t node_base, int32_t root_node, uint32_t root_unit, uint32_t fill,
               uint32_t first_block, B16Build& out, const char** why, int block_bits = kB16BlockBits);

}  // namespace arx
