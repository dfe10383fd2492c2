// arx_wide.cpp -- host collapse of the BVH2 into the 4-wide compressed tree (CW4, arx_layout.hpp).
//
// The BVH2 (arx_bvh.cpp, the SBVH that replaces optixAccelBuild, AudioRenderer.cpp:179-208) is
// kept as built; the CW4 copy only regroups its nodes: every CW4 child is a BVH2 node or a BVH2
// leaf (leaves of more than 2 triangles are split into pieces of <= 2 under the leaf's box), so a
// child's box is exactly the BVH2 box it came from and the closest hit cannot change.
#include "arx_wide.hpp"

#include <algorithm>
#include <functional>
#include <cmath>
#include <cstring>
#include <deque>

namespace arx {
namespace {

// A BVH2 child reference as the collapse sees it: an inner node (count 0), a leaf range of count
// triangles starting at ref, or nothing (count < 0).
struct Item {
    ChildRef c;
};

float area(const ChildRef& c) {
    const float dx = c.hi[0] - c.lo[0], dy = c.hi[1] - c.lo[1], dz = c.hi[2] - c.lo[2];
    return dx * dy + dy * dz + dz * dx;
}

bool openable(const ChildRef& c) { return c.count == 0 || c.count > 2; }

// The (up to two) pieces an openable item splits into.
int open_item(const BvhBuild& b, int32_t node_base, const ChildRef& c, ChildRef out[2]) {
    if (c.count == 0) {
        const BvhNode& n = b.nodes[(size_t)(c.ref - node_base)];
        int k = 0;
        for (int s = 0; s < 2; ++s) {
            ChildRef r;
            const float* xy = s == 0 ? n.a : n.b;
            r.lo[0] = xy[0];
            r.hi[0] = xy[1];
            r.lo[1] = xy[2];
            r.hi[1] = xy[3];
            r.lo[2] = n.c[2 * s];
            r.hi[2] = n.c[2 * s + 1];
            r.ref = n.d[s];
            r.count = n.d[2 + s];
            if (r.count >= 0) out[k++] = r;
        }
        return k;
    }
    // a leaf of > 2 triangles: two halves under the leaf's box
    const int32_t h = c.count / 2;
    out[0] = c;
    out[0].count = h;
    out[1] = c;
    out[1].ref = c.ref + h;
    out[1].count = c.count - h;
    return 2;
}

// Up to 4 children for a node whose BVH2 children are `start`: open the largest openable child
// while there is room.
std::vector<ChildRef> gather(const BvhBuild& b, int32_t node_base, std::vector<ChildRef> set) {
    while (set.size() < 4) {
        int best = -1;
        float best_a = -1.0f;
        for (size_t i = 0; i < set.size(); ++i)
            if (openable(set[i]) && area(set[i]) > best_a) {
                best_a = area(set[i]);
                best = (int)i;
            }
        if (best < 0) break;
        ChildRef pieces[2];
        const int k = open_item(b, node_base, set[(size_t)best], pieces);
        if (set.size() - 1 + (size_t)k > 4) break;
        set.erase(set.begin() + best);
        for (int i = 0; i < k; ++i) set.push_back(pieces[i]);
    }
    return set;
}

}  // namespace

void collapse_w4(const BvhBuild& b, int32_t node_base, int32_t tri_base, const ChildRef& root, uint32_t root_unit,
                 uint32_t first_unit, W4Build& out) {
    out.nodes.clear();
    out.src.clear();
    out.leaf_tris.clear();
    out.depth = 0;
    struct Pending {
        std::vector<ChildRef> items;  // the BVH2 children this CW4 node starts from
        uint32_t self;
        int depth;
    };
    std::deque<Pending> queue;
    {
        std::vector<ChildRef> start;
        if (root.count >= 0) {
            if (openable(root)) {
                ChildRef pieces[2];
                const int k = open_item(b, node_base, root, pieces);
                start.assign(pieces, pieces + k);
            } else {
                start.push_back(root);
            }
        }
        queue.push_back({start, root_unit, 1});
    }
    uint32_t cursor = first_unit;
    while (!queue.empty()) {
        Pending p = queue.front();
        queue.pop_front();
        std::vector<ChildRef> set = gather(b, node_base, p.items);
        // slot order: inner children (CW4 nodes) first, then leaves
        std::stable_partition(set.begin(), set.end(), [](const ChildRef& c) { return openable(c); });
        W4NodeF n;
        std::memset(&n, 0, sizeof(n));
        int n_inner = 0, n_leaf_tris = 0;
        for (const ChildRef& c : set) {
            if (openable(c)) ++n_inner;
            else n_leaf_tris += c.count;
        }
        n.base = cursor;
        n.self = p.self;
        cursor += (uint32_t)(kW4Units * n_inner + kTriUnits * n_leaf_tris);
        std::vector<int32_t> src(8, 0);
        int inner_k = 0, leaf_t = 0;
        for (size_t s = 0; s < set.size(); ++s) {
            const ChildRef& c = set[s];
            for (int k = 0; k < 3; ++k) {
                n.lo[s][k] = c.lo[k];
                n.hi[s][k] = c.hi[k];
            }
            src[2 * s] = c.ref;
            src[2 * s + 1] = c.count;
            if (openable(c)) {
                n.meta |= 1u << (2 * s);
                std::vector<ChildRef> items;
                ChildRef pieces[2];
                const int k = open_item(b, node_base, c, pieces);
                items.assign(pieces, pieces + k);
                queue.push_back({items, n.base + (uint32_t)(kW4Units * inner_k), p.depth + 1});
                ++inner_k;
            } else {
                n.meta |= (uint32_t)(1 + c.count) << (2 * s);
                for (int t = 0; t < c.count; ++t)
                    out.leaf_tris.emplace_back(n.base + (uint32_t)(kW4Units * n_inner + kTriUnits * (leaf_t + t)),
                                               c.ref + t - tri_base);
                leaf_t += c.count;
            }
        }
        for (size_t s = set.size(); s < 4; ++s) {
            src[2 * s] = 0;
            src[2 * s + 1] = -1;
        }
        out.nodes.push_back(n);
        out.src.insert(out.src.end(), src.begin(), src.end());
        out.depth = std::max(out.depth, p.depth);
    }
    out.unit_end = cursor;
}

}  // namespace arx

// ---- host simulation of both traversals (arx_debug_wide_stats) -------------------------------
#include <random>

#include "arx_internal.hpp"

namespace arx {
namespace {

struct SimRay {
    double o[3], d[3], inv[3];
};

void sim_setup(SimRay& r, const double o[3], const double d[3]) {
    for (int k = 0; k < 3; ++k) {
        r.o[k] = o[k];
        r.d[k] = d[k];
        r.inv[k] = d[k] != 0.0 ? 1.0 / d[k] : (std::signbit(d[k]) ? -1e300 : 1e300);
    }
}

// slab test of a world box; returns entry t or +inf on a miss
double sim_box(const SimRay& r, const double lo[3], const double hi[3], double tmax) {
    double tn = 0.0, tf = tmax;
    for (int k = 0; k < 3; ++k) {
        double a = (lo[k] - r.o[k]) * r.inv[k], b = (hi[k] - r.o[k]) * r.inv[k];
        if (a > b) std::swap(a, b);
        tn = std::max(tn, a);
        tf = std::min(tf, b);
    }
    return tn <= tf ? tn : HUGE_VAL;
}

// Moller-Trumbore in f64, both faces, t >= 0
bool sim_tri(const SimRay& r, const TriRec& t, double* tout) {
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

struct SimHit {
    double t = HUGE_VAL;
    int32_t id = 0x7fffffff;
    int32_t rec = -1;
    void take(double t2, int32_t id2, int32_t rec2) {
        if (t2 < t || (t2 == t && id2 < id)) {
            t = t2;
            id = id2;
            rec = rec2;
        }
    }
};

void grid_box(const QGrid& g, const uint32_t q[3], double lo[3], double hi[3]) {
    for (int k = 0; k < 3; ++k) {
        lo[k] = (double)g.origin[k] + (double)(q[k] & 0xffffu) * (double)g.scale[k];
        hi[k] = (double)g.origin[k] + (double)(q[k] >> 16) * (double)g.scale[k];
    }
}

}  // namespace
}  // namespace arx

using namespace arx;

extern "C" arx_status arx_debug_wide_stats(const float* tri_v, const float* tri_abs, int64_t n, const float* emitter,
                                           int64_t n_rays, int32_t bounces, uint64_t seed, double* out,
                                           size_t n_out) {
    if (!emitter || !out || n_out < 16 || n_rays < 0 || bounces < 1)
        return fail(ARX_ERR_INVALID_ARGUMENT, "bad arguments");
    arx_status st = check_scene_input(tri_v, tri_abs, n);
    if (st != ARX_OK) return st;
    SceneRef img = build_scene_image(tri_v, tri_abs, n);
    const BvhBuild& b = img->bvh;
    float lo[3], hi[3];
    for (int k = 0; k < 3; ++k) {
        lo[k] = std::min(b.root.lo[k], emitter[k]);
        hi[k] = std::max(b.root.hi[k], emitter[k]);
    }
    const QGrid g = make_qgrid(lo, hi, 0.1);
    // BVH2 quantized copy (node i + 1 = coded[i])
    std::vector<QNode2> q2(img->coded.size());
    const bool q2_ok = quantize_nodes16(img->coded.data(), img->coded.size(), g, q2.data());
    // CW4 copy: the scene root at unit 2, blocks from unit 4
    W4Build w;
    collapse_w4(b, 1, 0, b.root, 2, 4, w);
    std::vector<QNode4C> wn(w.unit_end / 2 + 2);
    std::vector<int32_t> unit_node(w.unit_end + 4, -1);  // unit -> CW4 node (sim lookup)
    std::vector<int32_t> unit_tri(w.unit_end + 4, -1);   // unit -> TriRec index
    int64_t q4_fail = 0;
    for (size_t i = 0; i < w.nodes.size(); ++i) {
        QNode4C qn;
        if (!quantize_w4(w.nodes[i], g, qn)) ++q4_fail;
        wn[i] = qn;
        unit_node[w.nodes[i].self] = (int32_t)i;
    }
    for (const auto& lt : w.leaf_tris) unit_tri[lt.first] = lt.second;
    std::mt19937_64 rng(seed);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    uint64_t queries = 0, q2_steps = 0, q2_tris = 0, q4_steps = 0, q4_tris = 0, mism = 0, misses = 0;
    int max_stack = 0;
    std::vector<uint64_t> stack_hist(64, 0);
    std::vector<uint64_t> visits(q2.size() + 2, 0);  // BVH2 node steps per node
    for (int64_t ray = 0; ray < n_rays; ++ray) {
        const double cz = 2.0 * U(rng) - 1.0, ph = 2.0 * M_PI * U(rng), sz = std::sqrt(std::max(0.0, 1.0 - cz * cz));
        double o[3] = {emitter[0], emitter[1], emitter[2]}, d[3] = {sz * std::cos(ph), sz * std::sin(ph), cz};
        for (int bnc = 0; bnc < bounces; ++bnc) {
            SimRay r;
            sim_setup(r, o, d);
            ++queries;
            // BVH2 over the quantized nodes, nearest first (node i = q2[i - 1]; node 1 = scene root)
            SimHit h2;
            {
                int stk[128];
                int sp = 0;
                int node = b.root.count == 0 ? b.root.ref : -1;
                if (b.root.count > 0)
                    for (int t = 0; t < b.root.count; ++t) {
                        double tt;
                        ++q2_tris;
                        if (sim_tri(r, b.tris[(size_t)(b.root.ref + t)], &tt)) h2.take(tt, b.tris[(size_t)(b.root.ref + t)].id, b.root.ref + t);
                    }
                while (node >= 0) {
                    ++q2_steps;
                    ++visits[(size_t)node];
                    const QNode2& qn = q2[(size_t)node - 1];
                    double tn[2];
                    int code[2];
                    for (int c = 0; c < 2; ++c) {
                        double l[3], hh[3];
                        grid_box(g, qn.c[c].q, l, hh);
                        code[c] = qn.c[c].code;
                        tn[c] = code[c] == kEmptyChildCode ? HUGE_VAL : sim_box(r, l, hh, h2.t);
                    }
                    int order[2] = {0, 1};
                    if (tn[1] < tn[0]) std::swap(order[0], order[1]);
                    int next = -1;
                    for (int j = 1; j >= 0; --j) {
                        const int c = order[j];
                        if (tn[c] == HUGE_VAL) continue;
                        if (code[c] < 0) {  // leaf: processed right away (the kernel's leaf batch keeps this order)
                            if (j == 0 && next < 0) {
                                const int v = ~code[c];
                                for (int t = 0; t < (v & 15); ++t) {
                                    ++q2_tris;
                                    double tt;
                                    const int32_t ti = (v >> 4) + t;
                                    if (sim_tri(r, b.tris[(size_t)ti], &tt)) h2.take(tt, b.tris[(size_t)ti].id, ti);
                                }
                            } else {
                                stk[sp++] = code[c];
                            }
                        } else if (j == 0) {
                            next = code[c];
                        } else {
                            stk[sp++] = code[c];
                        }
                    }
                    // pop until an inner node (leaves popped are tested)
                    while (next < 0 && sp > 0) {
                        const int e = stk[--sp];
                        if (e >= 0) {
                            next = e;
                        } else {
                            const int v = ~e;
                            for (int t = 0; t < (v & 15); ++t) {
                                ++q2_tris;
                                double tt;
                                const int32_t ti = (v >> 4) + t;
                                if (sim_tri(r, b.tris[(size_t)ti], &tt)) h2.take(tt, b.tris[(size_t)ti].id, ti);
                            }
                        }
                    }
                    node = next;
                }
            }
            // CW4, nearest first
            SimHit h4;
            {
                int64_t stk[256];
                int sp = 0;
                int64_t entry = 2;  // unit of the root node
                while (true) {
                    if (entry >= 0) {
                        ++q4_steps;
                        const int32_t ni = unit_node[(size_t)entry];
                        const QNode4C& qn = wn[(size_t)ni];
                        const uint32_t meta = (qn.w[1] >> 22) & 0xFFu;
                        const uint32_t oo[3] = {qn.w[0] & 0x3FFFu, (qn.w[0] >> 14) & 0x3FFFu, qn.w[1] & 0x3FFFu};
                        const uint32_t ee[3] = {qn.w[0] >> 28, (qn.w[1] >> 14) & 0xFu, (qn.w[1] >> 18) & 0xFu};
                        double tn[4];
                        int64_t code[4];
                        int n_inner = 0;
                        for (int c = 0; c < 4; ++c) n_inner += ((meta >> (2 * c)) & 3u) == 1u;
                        int leaf_t = 0;
                        for (int c = 0; c < 4; ++c) {
                            const uint32_t m = (meta >> (2 * c)) & 3u;
                            tn[c] = HUGE_VAL;
                            code[c] = 0;
                            if (!m) continue;
                            double l[3], hh[3];
                            for (int k = 0; k < 3; ++k) {
                                const int s0 = 6 * c + 2 * k, s1 = s0 + 1;
                                const uint32_t ql = (qn.w[2 + s0 / 5] >> (6 * (s0 % 5))) & 63u;
                                const uint32_t qh = (qn.w[2 + s1 / 5] >> (6 * (s1 % 5))) & 63u;
                                l[k] = (double)g.origin[k] + (double)(4 * oo[k] + (ql << ee[k])) * (double)g.scale[k];
                                hh[k] = (double)g.origin[k] + (double)(4 * oo[k] + (qh << ee[k])) * (double)g.scale[k];
                            }
                            tn[c] = sim_box(r, l, hh, h4.t);
                            if (m == 1u) {
                                code[c] = (int64_t)qn.w[7] + 2 * c;  // inner slots come first
                            } else {
                                const int cnt = (int)m - 1;
                                code[c] = ~(((int64_t)qn.w[7] + 2 * n_inner + 3 * leaf_t) * 4 + cnt);
                                leaf_t += cnt;
                            }
                        }
                        int ord[4] = {0, 1, 2, 3};
                        std::sort(ord, ord + 4, [&](int a, int bb) { return tn[a] < tn[bb]; });
                        int hits = 0;
                        while (hits < 4 && tn[ord[hits]] != HUGE_VAL) ++hits;
                        for (int j = hits - 1; j >= 1; --j) stk[sp++] = code[ord[j]];
                        max_stack = std::max(max_stack, sp);
                        stack_hist[(size_t)std::min(sp, 63)]++;
                        if (hits > 0) {
                            entry = code[ord[0]];
                            continue;
                        }
                    } else {
                        const int64_t v = ~entry;
                        const int cnt = (int)(v & 3);
                        const int64_t u = v >> 2;
                        for (int t = 0; t < cnt; ++t) {
                            ++q4_tris;
                            const int32_t ti = unit_tri[(size_t)(u + 3 * t)];
                            double tt;
                            if (ti >= 0 && sim_tri(r, b.tris[(size_t)ti], &tt)) h4.take(tt, b.tris[(size_t)ti].id, ti);
                        }
                    }
                    if (sp == 0) break;
                    entry = stk[--sp];
                }
            }
            if (h2.id != h4.id || h2.t != h4.t) ++mism;
            if (h2.rec < 0) {
                ++misses;
                break;
            }
            const TriRec& tr = b.tris[(size_t)h2.rec];
            const double e1[3] = {(double)tr.v1[0] - tr.v0[0], (double)tr.v1[1] - tr.v0[1], (double)tr.v1[2] - tr.v0[2]};
            const double e2[3] = {(double)tr.v2[0] - tr.v0[0], (double)tr.v2[1] - tr.v0[1], (double)tr.v2[2] - tr.v0[2]};
            double nn[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
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
    std::memset(out, 0, n_out * sizeof(double));
    const double q = (double)std::max<uint64_t>(queries, 1);
    out[0] = (double)queries;
    out[1] = (double)q2_steps / q;
    out[2] = (double)q2_tris / q;
    out[3] = (double)q4_steps / q;
    out[4] = (double)q4_tris / q;
    out[5] = (double)max_stack;
    out[6] = (double)mism;
    out[7] = (double)w.nodes.size();
    out[8] = (double)w.depth;
    out[9] = (double)b.nodes.size();
    out[10] = (double)b.depth;
    out[11] = (double)(q2_ok ? 0 : 1) + (double)q4_fail;
    out[12] = (double)misses;
    uint64_t tot = 0, acc = 0;
    for (uint64_t v : stack_hist) tot += v;
    for (size_t i = 0; i < stack_hist.size(); ++i) {  // 99.9th percentile of the stack depth after a push
        acc += stack_hist[i];
        if (acc >= tot - tot / 1000) {
            out[13] = (double)i;
            break;
        }
    }
    out[14] = (double)w.unit_end;
    if (n_out >= 32) {  // share of BVH2 node steps on K = 32 .. 4096 nodes: the K most visited
        // ([16..23]) and the K with the largest box surface area ([24..31], ray-independent)
        std::vector<uint64_t> sorted(visits);
        std::sort(sorted.begin(), sorted.end(), std::greater<uint64_t>());
        std::vector<std::pair<double, int32_t>> area;
        for (size_t i = 0; i < q2.size(); ++i)
            for (int c = 0; c < 2; ++c) {
                const int32_t code = q2[i].c[c].code;
                if (code <= 0) continue;
                double l[3], hh[3];
                grid_box(g, q2[i].c[c].q, l, hh);
                const double e0 = hh[0] - l[0], e1 = hh[1] - l[1], e2 = hh[2] - l[2];
                area.push_back({-(e0 * e1 + e1 * e2 + e2 * e0), code});
            }
        area.push_back({-HUGE_VAL, 1});
        std::sort(area.begin(), area.end());
        const double steps = (double)std::max<uint64_t>(q2_steps, 1);
        for (int j = 0; j < 8; ++j) {
            const size_t k = (size_t)32 << j;
            uint64_t in_top = 0, in_area = 0;
            for (size_t i = 0; i < std::min(k, sorted.size()); ++i) in_top += sorted[i];
            for (size_t i = 0; i < std::min(k, area.size()); ++i) in_area += visits[(size_t)area[i].second];
            out[16 + j] = (double)in_top / steps;
            out[24 + j] = (double)in_area / steps;
        }
    }
    return ARX_OK;
}
