// arx_b16.cpp -- layout of the compact binary tree (B16, arx_b16.hpp) and a host simulation of its
// traversal beside the 16-bit BVH2's (arx_debug_b16_stats).
#include "arx_b16.hpp"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <deque>
#include <random>
#include <unordered_map>

#include "arx_bvh.hpp"
#include "arx_internal.hpp"

namespace arx {

bool layout_b16(const BvhNode* coded, int32_t node_base, int32_t root_node, uint32_t root_unit, uint32_t fill,
               uint32_t first_block, B16Build& out, const char** why, int block_bits) {
    out = B16Build();
    const uint32_t bsize = 1u << block_bits;
    std::unordered_map<uint32_t, uint32_t> fill_of;  // block -> next free unit
    if (fill != 0u) fill_of[root_unit >> block_bits] = fill;
    uint32_t next_block = first_block;
    uint32_t leaf_block = 0xFFFFFFFFu;  // current block for chunks of leaves only
    auto open_block = [&]() {
        const uint32_t b = next_block++;
        fill_of[b] = b << block_bits;
        out.blocks.push_back(b);
        return b;
    };
    std::deque<std::pair<int32_t, uint32_t>> queue;  // (QNode2 index, unit)
    queue.emplace_back(root_node, root_unit);
    while (!queue.empty()) {
        const auto [node, unit] = queue.front();
        queue.pop_front();
        const BvhNode& bn = coded[node - node_base];
        uint32_t kind[2];
        int32_t first[2] = {0, 0};
        uint32_t n_inner = 0, n_tri_units = 0;
        for (int c = 0; c < 2; ++c) {
            const int32_t code = bn.d[c];
            kind[c] = 0u;
            if (code >= 0) {
                kind[c] = kB16Inner;
                ++n_inner;
            } else if (code != kEmptyChildCode) {
                const int32_t v = ~code;
                const uint32_t cnt = (uint32_t)(v & 15);
                if (cnt >= kB16Inner) {
                    *why = "leaf of more than 14 triangles";
                    return false;
                }
                kind[c] = cnt;
                first[c] = v >> 4;
                n_tri_units += (uint32_t)kTriUnits * cnt;
            }
        }
        const uint32_t size = n_inner + n_tri_units;
        if (size > bsize) {
            *why = "children chunk larger than a block";
            return false;
        }
        uint32_t base = 0u;
        if (size > 0u) {
            const uint32_t blk = unit >> block_bits;
            auto it = fill_of.find(blk);
            if (it != fill_of.end() && it->second + size <= ((blk + 1u) << block_bits)) {
                base = it->second;
                it->second += size;
            } else if (n_inner == 0u) {  // leaves only: no frame needed, any block with room
                if (leaf_block == 0xFFFFFFFFu || fill_of[leaf_block] + size > ((leaf_block + 1u) << block_bits))
                    leaf_block = open_block();
                base = fill_of[leaf_block];
                fill_of[leaf_block] += size;
            } else {
                const uint32_t b = open_block();
                base = b << block_bits;
                fill_of[b] += size;
            }
        }
        if (base >= (1u << 24) || next_block >= ((1u << 24) >> block_bits)) {
            *why = "B16 buffer beyond the 24-bit base";
            return false;
        }
        out.node_units.push_back(unit);
        out.node_src.push_back(node);
        out.node_w3.push_back(kind[0] | (kind[1] << 4) | (base << 8));
        uint32_t k = 0, t_units = 0;
        for (int c = 0; c < 2; ++c)
            if (kind[c] == kB16Inner) queue.emplace_back(bn.d[c], base + k++);
        for (int c = 0; c < 2; ++c)
            if (kind[c] != kB16Inner && kind[c] != 0u)
                for (uint32_t t = 0; t < kind[c]; ++t) {
                    out.tri_units.emplace_back(base + n_inner + t_units, first[c] + (int32_t)t);
                    t_units += (uint32_t)kTriUnits;
                }
    }
    out.unit_end = next_block << block_bits;
    return true;
}

}  // namespace arx

// ---- host simulation (arx_debug_b16_stats) ------------------------------------------------------
namespace arx {
namespace {

struct SRay {
    double o[3], d[3], inv[3];
};

double box_entry(const SRay& r, const double lo[3], const double hi[3], double tmax) {
    double tn = 0.0, tf = tmax;
    for (int k = 0; k < 3; ++k) {
        double a = (lo[k] - r.o[k]) * r.inv[k], b = (hi[k] - r.o[k]) * r.inv[k];
        if (a > b) std::swap(a, b);
        tn = std::max(tn, a);
        tf = std::min(tf, b);
    }
    return tn <= tf ? tn : HUGE_VAL;
}

bool tri_hit(const SRay& r, const TriRec& t, double* tout) {
    const double e1[3] = {(double)t.v1[0] - t.v0[0], (double)t.v1[1] - t.v0[1], (double)t.v1[2] - t.v0[2]};
    const double e2[3] = {(double)t.v2[0] - t.v0[0], (double)t.v2[1] - t.v0[1], (double)t.v2[2] - t.v0[2]};
    const double p[3] = {r.d[1] * e2[2] - r.d[2] * e2[1], r.d[2] * e2[0] - r.d[0] * e2[2], r.d[0] * e2[1] - r.d[1] * e2[0]};
    const double det = e1[0] * p[0] + e1[1] * p[1] + e1[2] * p[2];
    if (det == 0.0) return false;
    const double id = 1.0 / det;
    const double s[3] = {r.o[0] - t.v0[0], r.o[1] - t.v0[1], r.o[2] - t.v0[2]};
    const double u = (s[0] * p[0] + s[1] * p[1] + s[2] * p[2]) * id;
    if (u < 0.0 || u > 1.0) return false;
    const double q[3] = {s[1] * e1[2] - s[2] * e1[1], s[2] * e1[0] - s[0] * e1[2], s[0] * e1[1] - s[1] * e1[0]};
    const double v = (r.d[0] * q[0] + r.d[1] * q[1] + r.d[2] * q[2]) * id;
    if (v < 0.0 || u + v > 1.0) return false;
    const double tt = (e2[0] * q[0] + e2[1] * q[1] + e2[2] * q[2]) * id;
    if (!(tt >= 0.0)) return false;
    *tout = tt;
    return true;
}

struct Hit {
    double t = HUGE_VAL;
    int32_t id = 0x7fffffff;
    int32_t tri = -1;
    void take(double t2, int32_t id2, int32_t tri2) {
        if (t2 < t || (t2 == t && id2 < id)) {
            t = t2;
            id = id2;
            tri = tri2;
        }
    }
};

// The kernel's traversal order (node_step / leaf_step): both children tested, the nearer hit one
// taken (inner node or leaf), the farther pushed; a leaf is tested, then the stack popped.
// Node(entry, lo, hi, code) decodes a node entry's two children; Leaf(code, hit) tests a leaf.
template <typename Node, typename Leaf>
void traverse(const SRay& r, int32_t root, Hit& h, uint64_t& steps, Node node_fn, Leaf leaf_fn) {
    int32_t stk[128];
    int sp = 0;
    int32_t cur = root;
    while (cur != -1) {
        if (cur >= 0) {
            ++steps;
            double lo[2][3], hi[2][3];
            int32_t code[2];
            node_fn(cur, lo, hi, code);
            double tn[2];
            for (int c = 0; c < 2; ++c) tn[c] = box_entry(r, lo[c], hi[c], h.t);
            const bool h0 = tn[0] != HUGE_VAL, h1 = tn[1] != HUGE_VAL;
            const bool near1 = h1 && (!h0 || tn[1] < tn[0]);
            if (h0 && h1) stk[sp++] = near1 ? code[0] : code[1];
            if (h0 || h1) cur = near1 ? code[1] : code[0];
            else cur = sp > 0 ? stk[--sp] : -1;
        } else {
            leaf_fn(cur, h);
            cur = sp > 0 ? stk[--sp] : -1;
        }
    }
}

}  // namespace
}  // namespace arx

using namespace arx;

/* out: [0] queries [1] / [2] BVH2 node steps / triangle tests per query [3] / [4] the same for B16
 * [5] B16 frame switches per query (node steps into another block than the lane's last) [6] queries
 * whose closest hits differ [7] B16 units [8] B16 blocks [9] BVH2 nodes [10] B16 layout ok. */
extern "C" arx_status arx_debug_b16_stats(const float* tri_v, const float* tri_abs, int64_t n, const float* emitter,
                                         int64_t n_rays, int32_t bounces, uint64_t seed, int32_t block_bits,
                                         double* out, size_t n_out) {
    if (!emitter || !out || n_out < 11 || n_rays < 0 || bounces < 1 || block_bits < 3 || block_bits > 12)
        return fail(ARX_ERR_INVALID_ARGUMENT, "bad arguments");
    arx_status st = check_scene_input(tri_v, tri_abs, n);
    if (st != ARX_OK) return st;
    SceneRef img = build_scene_image(tri_v, tri_abs, n);
    const BvhBuild& b = img->bvh;
    std::memset(out, 0, n_out * sizeof(double));
    if (b.root.count != 0) return ARX_OK;  // a scene of one leaf: nothing to compare
    float lo[3], hi[3];
    for (int k = 0; k < 3; ++k) {
        lo[k] = std::min(b.root.lo[k], emitter[k]);
        hi[k] = std::max(b.root.hi[k], emitter[k]);
    }
    const QGrid g = make_qgrid(lo, hi, 0.1);
    // QNode2 index i = scene node i (coded[i - 1]); index 0 unused here (no top node)
    std::vector<QNode2> q2(img->coded.size() + 1);
    if (!quantize_nodes16(img->coded.data(), img->coded.size(), g, q2.data() + 1))
        return fail(ARX_ERR_INTERNAL, "grid");
    B16Build L;
    const char* why = "";
    if (!layout_b16(img->coded.data(), 1, 1, kB16SceneRoot, 3, 1, L, &why, block_bits)) {
        out[10] = 0.0;
        return ARX_OK;
    }
    const uint32_t n_blocks = L.unit_end >> block_bits;
    std::vector<B16FrameAcc> acc(n_blocks);
    for (size_t i = 0; i < L.node_units.size(); ++i)
        acc[L.node_units[i] >> block_bits].add(q2[(size_t)L.node_src[i]], L.node_w3[i]);
    std::vector<uint2> frames(n_blocks);
    for (uint32_t k = 0; k < n_blocks; ++k) frames[k] = acc[k].frame();
    std::vector<uint4> units(L.unit_end, make_uint4(0u, 0u, 0u, 0u));
    for (size_t i = 0; i < L.node_units.size(); ++i)
        units[L.node_units[i]] =
            b16_node(q2[(size_t)L.node_src[i]], L.node_w3[i], frames[L.node_units[i] >> block_bits]);
    std::vector<int32_t> unit_tri(L.unit_end, -1);
    for (const auto& ut : L.tri_units) unit_tri[ut.first] = ut.second;

    auto q16_box = [&](uint32_t word, int k, double& l, double& h) {
        l = (double)g.origin[k] + (double)(word & 0xFFFFu) * (double)g.scale[k];
        h = (double)g.origin[k] + (double)(word >> 16) * (double)g.scale[k];
    };
    std::mt19937_64 rng(seed);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    uint64_t queries = 0, s2 = 0, t2 = 0, sc = 0, tc = 0, switches = 0, mism = 0;
    uint32_t cur_block = 0xFFFFFFFFu;
    for (int64_t ray = 0; ray < n_rays; ++ray) {
        const double cz = 2.0 * U(rng) - 1.0, ph = 2.0 * M_PI * U(rng), sz = std::sqrt(std::max(0.0, 1.0 - cz * cz));
        double o[3] = {emitter[0], emitter[1], emitter[2]}, d[3] = {sz * std::cos(ph), sz * std::sin(ph), cz};
        for (int bnc = 0; bnc < bounces; ++bnc) {
            SRay r;
            for (int k = 0; k < 3; ++k) {
                r.o[k] = o[k];
                r.d[k] = d[k];
                r.inv[k] = d[k] != 0.0 ? 1.0 / d[k] : (std::signbit(d[k]) ? -1e300 : 1e300);
            }
            ++queries;
            Hit h2, hc;
            traverse(
                r, 1, h2, s2,
                [&](int32_t nd, double lo2[2][3], double hi2[2][3], int32_t code[2]) {
                    const QNode2& q = q2[(size_t)nd];
                    for (int c = 0; c < 2; ++c) {
                        for (int k = 0; k < 3; ++k) q16_box(q.c[c].q[k], k, lo2[c][k], hi2[c][k]);
                        code[c] = q.c[c].code;
                    }
                },
                [&](int32_t code, Hit& h) {
                    const int32_t v = ~code;
                    for (int t = 0; t < (v & 15); ++t) {
                        ++t2;
                        double tt;
                        const TriRec& tr = b.tris[(size_t)((v >> 4) + t)];
                        if (tri_hit(r, tr, &tt)) h.take(tt, tr.id, (v >> 4) + t);
                    }
                });
            traverse(
                r, (int32_t)kB16SceneRoot, hc, sc,
                [&](int32_t u, double lo2[2][3], double hi2[2][3], int32_t code[2]) {
                    const uint32_t blk = (uint32_t)u >> block_bits;
                    if (blk != cur_block) {
                        ++switches;
                        cur_block = blk;
                    }
                    const uint4 w = units[(size_t)u];
                    const uint2 f = frames[blk];
                    const uint32_t of[3] = {f.x & 0xFFFFu, f.x >> 16, f.y & 0xFFFFu};
                    const uint32_t e[3] = {(f.y >> 16) & 15u, (f.y >> 20) & 15u, (f.y >> 24) & 15u};
                    const uint32_t ws[3] = {w.x, w.y, w.z};
                    for (int c = 0; c < 2; ++c)
                        for (int k = 0; k < 3; ++k) {
                            const uint32_t ql = (ws[k] >> (16 * c)) & 0xFFu, qh = (ws[k] >> (16 * c + 8)) & 0xFFu;
                            lo2[c][k] = (double)g.origin[k] + (double)(of[k] + (ql << e[k])) * (double)g.scale[k];
                            hi2[c][k] = (double)g.origin[k] + (double)(of[k] + (qh << e[k])) * (double)g.scale[k];
                        }
                    const uint32_t k0 = w.w & 15u, k1 = (w.w >> 4) & 15u, base = w.w >> 8;
                    const uint32_t i0 = k0 == kB16Inner, i1 = k1 == kB16Inner, n_in = i0 + i1;
                    code[0] = i0 ? (int32_t)base : ~(int32_t)((base + n_in) * 16u + k0);
                    code[1] = i1 ? (int32_t)(base + i0) : ~(int32_t)((base + n_in + 3u * (i0 ? 0u : k0)) * 16u + k1);
                },
                [&](int32_t code, Hit& h) {
                    const int32_t v = ~code;
                    for (int t = 0; t < (v & 15); ++t) {
                        ++tc;
                        double tt;
                        const int32_t ti = unit_tri[(size_t)((v >> 4) + 3 * t)];
                        const TriRec& tr = b.tris[(size_t)ti];
                        if (tri_hit(r, tr, &tt)) h.take(tt, tr.id, ti);
                    }
                });
            if (h2.id != hc.id || h2.t != hc.t) ++mism;
            if (h2.tri < 0) break;
            const TriRec& tr = b.tris[(size_t)h2.tri];
            const double e1[3] = {(double)tr.v1[0] - tr.v0[0], (double)tr.v1[1] - tr.v0[1], (double)tr.v1[2] - tr.v0[2]};
            const double e2[3] = {(double)tr.v2[0] - tr.v0[0], (double)tr.v2[1] - tr.v0[1], (double)tr.v2[2] - tr.v0[2]};
            const double nn[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2],
                                  e1[0] * e2[1] - e1[1] * e2[0]};
            const double nl = std::sqrt(nn[0] * nn[0] + nn[1] * nn[1] + nn[2] * nn[2]);
            if (!(nl > 0.0)) break;
            const double dn = (d[0] * nn[0] + d[1] * nn[1] + d[2] * nn[2]) / (nl * nl);
            for (int k = 0; k < 3; ++k) {
                const double p = o[k] + h2.t * d[k];
                d[k] = d[k] - 2.0 * dn * nn[k];
                o[k] = p + 1e-3 * d[k];
            }
        }
    }
    const double q = (double)std::max<uint64_t>(queries, 1);
    out[0] = (double)queries;
    out[1] = (double)s2 / q;
    out[2] = (double)t2 / q;
    out[3] = (double)sc / q;
    out[4] = (double)tc / q;
    out[5] = (double)switches / q;
    out[6] = (double)mism;
    out[7] = (double)L.unit_end;
    out[8] = (double)n_blocks;
    out[9] = (double)img->coded.size();
    out[10] = 1.0;
    return ARX_OK;
}
