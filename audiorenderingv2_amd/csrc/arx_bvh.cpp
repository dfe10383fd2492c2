// arx_bvh.cpp -- binned-SAH BVH2 builder for the trace kernel's 64-B node layout.
//
// The reference builds an OptiX GAS over per-material meshes (AudioRenderer.cpp:95-218);
// here the static scene is built once and the receiver halves get their own small
// sub-tree (rebuilt per listener move in milliseconds).  The default builder uses spatial
// splits (SBVH): a triangle may appear in several leaves (duplicate TriRecs with the same
// global id, so the closest hit and its tie-break are unchanged).  Boxes are padded by
// 1e-5 * max|coordinate| so that box rejection is conservative w.r.t. the watertight
// triangle test: the BVH closest hit is exactly the brute-force closest hit.
#include "arx_bvh.hpp"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <future>
#include <limits>

namespace arx {
namespace {

constexpr int kMaxBins = 256;
// Spatial splits only for builds of at least this many triangles: the receiver halves (about
// a thousand small, evenly sized triangles, rebuilt on every listener move) gain nothing.
constexpr int64_t kSpatialMinTris = 4096;

struct Prim {
    float lo[3], hi[3], c[3];
    int32_t idx;
};

struct Box {
    float lo[3] = {std::numeric_limits<float>::max(), std::numeric_limits<float>::max(),
                   std::numeric_limits<float>::max()};
    float hi[3] = {-std::numeric_limits<float>::max(), -std::numeric_limits<float>::max(),
                   -std::numeric_limits<float>::max()};
    void grow(const float* l, const float* h) {
        for (int k = 0; k < 3; ++k) {
            lo[k] = std::min(lo[k], l[k]);
            hi[k] = std::max(hi[k], h[k]);
        }
    }
    void grow_pt(const float* p) { grow(p, p); }
    bool empty() const { return lo[0] > hi[0]; }
    float area() const {
        if (empty()) return 0.0f;
        float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
        return 2.0f * (dx * dy + dy * dz + dz * dx);
    }
};

struct Builder {
    BuildParams prm = build_params();
    std::vector<Prim> prims;
    BvhBuild* out;
    const float* tri_v;
    const float* tri_abs;
    float abs_fill;
    int32_t id_base;
    float pad;

    ChildRef make_ref(const Box& b, int32_t ref, int32_t count) const {
        ChildRef c;
        for (int k = 0; k < 3; ++k) {
            c.lo[k] = b.lo[k] - pad;
            c.hi[k] = b.hi[k] + pad;
        }
        c.ref = ref;
        c.count = count;
        return c;
    }

    ChildRef leaf(int64_t begin, int64_t end, const Box& b) {
        int32_t first = (int32_t)out->tris.size();
        for (int64_t i = begin; i < end; ++i) {
            int32_t src = prims[i].idx;
            TriRec t;
            std::memset(&t, 0, sizeof(t));
            const float* v = tri_v + 9 * (int64_t)src;
            for (int k = 0; k < 3; ++k) {
                t.v0[k] = v[k];
                t.v1[k] = v[3 + k];
                t.v2[k] = v[6 + k];
            }
            t.absorption = tri_abs ? tri_abs[src] : abs_fill;
            t.id = id_base + src;
            out->tris.push_back(t);
        }
        return make_ref(b, first, (int32_t)(end - begin));
    }

    ChildRef build(int64_t begin, int64_t end, int depth) {
        Box bounds, cbounds;
        for (int64_t i = begin; i < end; ++i) {
            bounds.grow(prims[i].lo, prims[i].hi);
            cbounds.grow_pt(prims[i].c);
        }
        const int64_t n = end - begin;
        out->depth = std::max(out->depth, depth);
        if (n <= 1 || depth >= kMaxBuildDepth) return leaf(begin, end, bounds);

        // binned SAH over centroids
        int best_axis = -1, best_split = -1;
        float best_cost = std::numeric_limits<float>::max();
        for (int axis = 0; axis < 3; ++axis) {
            float cmin = cbounds.lo[axis], cmax = cbounds.hi[axis];
            if (!(cmax > cmin)) continue;
            const int kBins = prm.bins;
            float scale = kBins / (cmax - cmin);
            Box bb[kMaxBins];
            int64_t cnt[kMaxBins] = {0};
            for (int64_t i = begin; i < end; ++i) {
                int b = std::min(kBins - 1, (int)((prims[i].c[axis] - cmin) * scale));
                cnt[b]++;
                bb[b].grow(prims[i].lo, prims[i].hi);
            }
            float right_area[kMaxBins];
            int64_t right_cnt[kMaxBins];
            Box acc;
            int64_t ac = 0;
            for (int b = kBins - 1; b > 0; --b) {
                acc.grow(bb[b].lo, bb[b].hi);
                ac += cnt[b];
                right_area[b] = acc.area();
                right_cnt[b] = ac;
            }
            Box lacc;
            int64_t lc = 0;
            for (int b = 0; b < kBins - 1; ++b) {
                lacc.grow(bb[b].lo, bb[b].hi);
                lc += cnt[b];
                if (lc == 0 || right_cnt[b + 1] == 0) continue;
                float cost = lacc.area() * (float)lc + right_area[b + 1] * (float)right_cnt[b + 1];
                if (cost < best_cost) {
                    best_cost = cost;
                    best_axis = axis;
                    best_split = b;
                }
            }
        }
        float parent_area = bounds.area();
        float sah = prm.trav_cost + (parent_area > 0 ? prm.isect_cost * best_cost / parent_area : 0.0f);
        if (n <= prm.leaf_max && (best_axis < 0 || sah >= prm.isect_cost * (float)n)) return leaf(begin, end, bounds);

        int64_t mid;
        if (best_axis >= 0) {
            float cmin = cbounds.lo[best_axis], cmax = cbounds.hi[best_axis];
            const int kBins = prm.bins;
            float scale = kBins / (cmax - cmin);
            auto it = std::stable_partition(prims.begin() + begin, prims.begin() + end, [&](const Prim& p) {
                int b = std::min(kBins - 1, (int)((p.c[best_axis] - cmin) * scale));
                return b <= best_split;
            });
            mid = it - prims.begin();
        } else {
            mid = begin + n / 2;  // all centroids coincide: split by position in the list
        }
        if (mid == begin || mid == end) mid = begin + n / 2;

        int32_t me = (int32_t)out->nodes.size();
        out->nodes.emplace_back();
        ChildRef l = build(begin, mid, depth + 1);
        ChildRef r = build(mid, end, depth + 1);
        out->nodes[me] = make_node(l, r);
        ChildRef self = make_ref(bounds, me, 0);
        return self;
    }
};


// ---- spatial-split builder (BuildParams::spatial) ----
struct Ref {
    Box b;
    int32_t idx;
};

inline float center(const Box& b, int k) { return 0.5f * (b.lo[k] + b.hi[k]); }

inline Box intersect(const Box& a, const Box& b) {
    Box r;
    for (int k = 0; k < 3; ++k) {
        r.lo[k] = std::max(a.lo[k], b.lo[k]);
        r.hi[k] = std::min(a.hi[k], b.hi[k]);
    }
    return r;
}

inline float overlap_area(const Box& a, const Box& b) {
    Box r = intersect(a, b);
    for (int k = 0; k < 3; ++k)
        if (!(r.lo[k] <= r.hi[k])) return 0.0f;
    return r.area();
}

struct SpatialBuilder {
    BuildParams prm = build_params();
    BvhBuild* out;
    const float* tri_v;
    const float* tri_abs;
    float abs_fill;
    int32_t id_base;
    float pad;
    float min_overlap;     // alpha * root area
    int64_t refs_left;     // extra references still allowed

    ChildRef make_ref(const Box& b, int32_t ref, int32_t count) const {
        ChildRef c;
        for (int k = 0; k < 3; ++k) {
            c.lo[k] = b.lo[k] - pad;
            c.hi[k] = b.hi[k] + pad;
        }
        c.ref = ref;
        c.count = count;
        return c;
    }

    ChildRef leaf(const std::vector<Ref>& refs, const Box& b) {
        const int32_t first = (int32_t)out->tris.size();
        for (const Ref& r : refs) {
            TriRec t;
            std::memset(&t, 0, sizeof(t));
            const float* v = tri_v + 9 * (int64_t)r.idx;
            for (int k = 0; k < 3; ++k) {
                t.v0[k] = v[k];
                t.v1[k] = v[3 + k];
                t.v2[k] = v[6 + k];
            }
            t.absorption = tri_abs ? tri_abs[r.idx] : abs_fill;
            t.id = id_base + r.idx;
            out->tris.push_back(t);
        }
        return make_ref(b, first, (int32_t)refs.size());
    }

    // Boxes of the parts of triangle r.idx on either side of the plane x[axis] = pos, each
    // intersected with the reference's own box (which already bounds the referenced part).
    // The crossing points are computed in double; the node padding covers the f32 rounding.
    void split_ref(const Ref& r, int axis, float pos, Box& lb, Box& rb) const {
        const float* v = tri_v + 9 * (int64_t)r.idx;
        lb = Box();
        rb = Box();
        for (int e = 0; e < 3; ++e) {
            const float* a = v + 3 * e;
            const float* b = v + 3 * ((e + 1) % 3);
            if (a[axis] <= pos) lb.grow_pt(a);
            if (a[axis] >= pos) rb.grow_pt(a);
            if ((a[axis] < pos && pos < b[axis]) || (b[axis] < pos && pos < a[axis])) {
                const double t = ((double)pos - a[axis]) / ((double)b[axis] - a[axis]);
                float p[3];
                for (int k = 0; k < 3; ++k) p[k] = (float)((double)a[k] + t * ((double)b[k] - a[k]));
                p[axis] = pos;
                lb.grow_pt(p);
                rb.grow_pt(p);
            }
        }
        lb = intersect(lb, r.b);
        rb = intersect(rb, r.b);
        lb.hi[axis] = std::min(lb.hi[axis], pos);
        rb.lo[axis] = std::max(rb.lo[axis], pos);
    }

    static bool valid(const Box& b) { return b.lo[0] <= b.hi[0] && b.lo[1] <= b.hi[1] && b.lo[2] <= b.hi[2]; }

    struct ObjectSplit {
        int axis = -1, bin = -1;
        float cost = std::numeric_limits<float>::max();
        Box left, right;
    };

    ObjectSplit object_split(const std::vector<Ref>& refs, const Box& cb) const {
        ObjectSplit best;
        const int nb = prm.bins;
        for (int axis = 0; axis < 3; ++axis) {
            const float cmin = cb.lo[axis], cmax = cb.hi[axis];
            if (!(cmax > cmin)) continue;
            const float scale = nb / (cmax - cmin);
            Box bb[kMaxBins];
            int64_t cnt[kMaxBins] = {0};
            for (const Ref& r : refs) {
                const int b = std::min(nb - 1, (int)((center(r.b, axis) - cmin) * scale));
                cnt[b]++;
                bb[b].grow(r.b.lo, r.b.hi);
            }
            Box racc[kMaxBins];
            int64_t rcnt[kMaxBins];
            Box acc;
            int64_t ac = 0;
            for (int b = nb - 1; b > 0; --b) {
                acc.grow(bb[b].lo, bb[b].hi);
                ac += cnt[b];
                racc[b] = acc;
                rcnt[b] = ac;
            }
            Box lacc;
            int64_t lc = 0;
            for (int b = 0; b < nb - 1; ++b) {
                lacc.grow(bb[b].lo, bb[b].hi);
                lc += cnt[b];
                if (lc == 0 || rcnt[b + 1] == 0) continue;
                const float cost = lacc.area() * (float)lc + racc[b + 1].area() * (float)rcnt[b + 1];
                if (cost < best.cost) {
                    best.cost = cost;
                    best.axis = axis;
                    best.bin = b;
                    best.left = lacc;
                    best.right = racc[b + 1];
                }
            }
        }
        return best;
    }

    struct SpatialSplit {
        int axis = -1;
        float pos = 0.0f;
        float cost = std::numeric_limits<float>::max();
    };

    SpatialSplit spatial_split(const std::vector<Ref>& refs, const Box& bounds) const {
        SpatialSplit best;
        // no more planes than references (at least 16): the same trees on the GPU, ~30 % less
        // host build time at spatial_alpha 1e-5 (profiles/r02/ab_sah.log batch 8)
        const int nb = std::min(prm.spatial_bins, (int)std::max<size_t>(16, std::min<size_t>(refs.size(), 1 << 20)));
        for (int axis = 0; axis < 3; ++axis) {
            const float lo = bounds.lo[axis], hi = bounds.hi[axis];
            if (!(hi > lo)) continue;
            const float w = (hi - lo) / nb;
            const float scale = nb / (hi - lo);
            Box bb[kMaxBins];
            int64_t enter[kMaxBins] = {0}, exit_[kMaxBins] = {0};
            auto bin_of = [&](float x) { return std::min(nb - 1, std::max(0, (int)((x - lo) * scale))); };
            for (const Ref& r : refs) {
                const int b0 = bin_of(r.b.lo[axis]), b1 = bin_of(r.b.hi[axis]);
                enter[b0]++;
                exit_[b1]++;
                Ref cur = r;
                for (int b = b0; b < b1; ++b) {
                    Box lb, rb;
                    split_ref(cur, axis, lo + w * (float)(b + 1), lb, rb);
                    if (valid(lb)) bb[b].grow(lb.lo, lb.hi);
                    cur.b = rb;
                    if (!valid(rb)) break;
                }
                if (valid(cur.b)) bb[b1].grow(cur.b.lo, cur.b.hi);
            }
            Box racc[kMaxBins];
            int64_t rcnt[kMaxBins];
            Box acc;
            int64_t ac = 0;
            for (int b = nb - 1; b > 0; --b) {
                acc.grow(bb[b].lo, bb[b].hi);
                ac += exit_[b];
                racc[b] = acc;
                rcnt[b] = ac;
            }
            Box lacc;
            int64_t lc = 0;
            for (int b = 0; b < nb - 1; ++b) {
                lacc.grow(bb[b].lo, bb[b].hi);
                lc += enter[b];
                if (lc == 0 || rcnt[b + 1] == 0) continue;
                const float cost = lacc.area() * (float)lc + racc[b + 1].area() * (float)rcnt[b + 1];
                if (cost < best.cost) {
                    best.cost = cost;
                    best.axis = axis;
                    best.pos = lo + w * (float)(b + 1);
                }
            }
        }
        return best;
    }

    // Partition by a spatial plane; straddling references are split, or kept whole on one side
    // when that is cheaper ("reference unsplitting", Stich et al. 2009 section 4.3).
    void partition_spatial(std::vector<Ref>& refs, int axis, float pos, std::vector<Ref>& L, std::vector<Ref>& R) {
        Box lb, rb;
        std::vector<Ref> straddle;
        for (const Ref& r : refs) {
            if (r.b.hi[axis] <= pos) {
                L.push_back(r);
                lb.grow(r.b.lo, r.b.hi);
            } else if (r.b.lo[axis] >= pos) {
                R.push_back(r);
                rb.grow(r.b.lo, r.b.hi);
            } else {
                straddle.push_back(r);
            }
        }
        for (const Ref& r : straddle) {
            Box pl, pr;
            split_ref(r, axis, pos, pl, pr);
            const bool okl = valid(pl), okr = valid(pr);
            if (!okr || (okl && refs_left <= 0)) {  // all on the left (or no budget: keep whole)
                if (!okr || !okl) {
                    L.push_back(r);
                    lb.grow(r.b.lo, r.b.hi);
                    continue;
                }
            }
            if (!okl) {
                R.push_back(r);
                rb.grow(r.b.lo, r.b.hi);
                continue;
            }
            const float nl = (float)L.size(), nr = (float)R.size();
            Box lu = lb, ru = rb, ls = lb, rs = rb;
            lu.grow(r.b.lo, r.b.hi);
            ru.grow(r.b.lo, r.b.hi);
            ls.grow(pl.lo, pl.hi);
            rs.grow(pr.lo, pr.hi);
            const float c_split = ls.area() * (nl + 1) + rs.area() * (nr + 1);
            const float c_left = lu.area() * (nl + 1) + rb.area() * nr;
            const float c_right = lb.area() * nl + ru.area() * (nr + 1);
            if (refs_left > 0 && c_split < c_left && c_split < c_right) {
                L.push_back(Ref{pl, r.idx});
                R.push_back(Ref{pr, r.idx});
                lb = ls;
                rb = rs;
                --refs_left;
            } else if (c_left <= c_right) {
                L.push_back(r);
                lb = lu;
            } else {
                R.push_back(r);
                rb = ru;
            }
        }
    }

    ChildRef build(std::vector<Ref>& refs, int depth) {
        Box bounds, cb;
        for (const Ref& r : refs) {
            bounds.grow(r.b.lo, r.b.hi);
            const float c[3] = {center(r.b, 0), center(r.b, 1), center(r.b, 2)};
            cb.grow_pt(c);
        }
        const int64_t n = (int64_t)refs.size();
        out->depth = std::max(out->depth, depth);
        if (n <= 1 || depth >= kMaxBuildDepth) {
            if (n > 15) std::abort();  // cannot happen below the depth cap for real scenes
            return leaf(refs, bounds);
        }
        // depth cap: median splits from here on (each halves the references)
        int need = 0;
        while (((int64_t)prm.leaf_max << need) < n) ++need;
        if (depth + need >= prm.max_depth) return median_split(refs, bounds, cb, depth);
        ObjectSplit os = object_split(refs, cb);
        SpatialSplit ss;
        if (os.axis >= 0 && refs_left > 0 && depth < prm.spatial_max_depth && overlap_area(os.left, os.right) > min_overlap) ss = spatial_split(refs, bounds);
        const float best_cost = std::min(os.cost, ss.cost);
        const float parent_area = bounds.area();
        const float sah = prm.trav_cost + (parent_area > 0 ? prm.isect_cost * best_cost / parent_area : 0.0f);
        const bool have = os.axis >= 0 || ss.axis >= 0;
        if (n <= prm.leaf_max && (!have || sah >= prm.isect_cost * (float)n)) return leaf(refs, bounds);

        std::vector<Ref> L, R;
        if (ss.axis >= 0 && ss.cost < os.cost) {
            partition_spatial(refs, ss.axis, ss.pos, L, R);
            if (L.empty() || R.empty() || ((int64_t)L.size() == n && (int64_t)R.size() == n)) {
                L.clear();
                R.clear();
                ss.axis = -1;
            }
        }
        if (L.empty() && R.empty()) {
            if (os.axis >= 0) {
                const float cmin = cb.lo[os.axis], cmax = cb.hi[os.axis];
                const float scale = prm.bins / (cmax - cmin);
                for (const Ref& r : refs) {
                    const int b = std::min(prm.bins - 1, (int)((center(r.b, os.axis) - cmin) * scale));
                    (b <= os.bin ? L : R).push_back(r);
                }
            }
            if (L.empty() || R.empty()) {  // all centroids coincide: split by position in the list
                L.assign(refs.begin(), refs.begin() + n / 2);
                R.assign(refs.begin() + n / 2, refs.end());
            }
        }
        std::vector<Ref>().swap(refs);
        return inner(L, R, bounds, depth);
    }

    ChildRef median_split(std::vector<Ref>& refs, const Box& bounds, const Box& cb, int depth) {
        const int64_t n = (int64_t)refs.size();
        if (n <= prm.leaf_max || n <= 1) return leaf(refs, bounds);
        int axis = 0;
        for (int k = 1; k < 3; ++k)
            if (cb.hi[k] - cb.lo[k] > cb.hi[axis] - cb.lo[axis]) axis = k;
        std::vector<Ref> L(refs.begin(), refs.end());
        std::nth_element(L.begin(), L.begin() + n / 2, L.end(), [axis](const Ref& a, const Ref& b) {
            const float ca = center(a.b, axis), cb_ = center(b.b, axis);
            return ca < cb_ || (ca == cb_ && a.idx < b.idx);
        });
        std::vector<Ref> R(L.begin() + n / 2, L.end());
        L.resize((size_t)(n / 2));
        std::vector<Ref>().swap(refs);
        return inner(L, R, bounds, depth);
    }

    // Inner node over L and R.  Near the root the two subtrees are built concurrently into
    // builds of their own and appended in depth-first order (the same layout as serially).
    ChildRef inner(std::vector<Ref>& L, std::vector<Ref>& R, const Box& bounds, int depth) {
        const int32_t me = (int32_t)out->nodes.size();
        out->nodes.emplace_back();
        ChildRef l, r;
        if ((1 << depth) <= prm.threads && L.size() + R.size() > 4096) {
            BvhBuild bl, br;
            SpatialBuilder sl = *this, sr = *this;
            sl.out = &bl;
            sr.out = &br;
            const double share = (double)L.size() / (double)(L.size() + R.size());
            sl.refs_left = (int64_t)((double)refs_left * share);
            sr.refs_left = refs_left - sl.refs_left;
            auto fut = std::async(std::launch::async, [&] { return sl.build(L, depth + 1); });
            r = sr.build(R, depth + 1);
            l = fut.get();
            refs_left = sl.refs_left + sr.refs_left;
            const int32_t nb = (int32_t)out->nodes.size(), tb = (int32_t)out->tris.size();
            bl.root = l;
            br.root = r;
            relocate_bvh(bl, nb, tb);
            relocate_bvh(br, nb + (int32_t)bl.nodes.size(), tb + (int32_t)bl.tris.size());
            out->nodes.insert(out->nodes.end(), bl.nodes.begin(), bl.nodes.end());
            out->nodes.insert(out->nodes.end(), br.nodes.begin(), br.nodes.end());
            out->tris.insert(out->tris.end(), bl.tris.begin(), bl.tris.end());
            out->tris.insert(out->tris.end(), br.tris.begin(), br.tris.end());
            out->depth = std::max(out->depth, std::max(bl.depth, br.depth));
            l = bl.root;
            r = br.root;
        } else {
            l = build(L, depth + 1);
            r = build(R, depth + 1);
        }
        out->nodes[me] = make_node(l, r);
        return make_ref(bounds, me, 0);
    }
};

}  // namespace

BuildParams& build_params() {
    static BuildParams p;  // production defaults; design tools (tools/bvh_*.cpp) edit it before building
    return p;
}

ChildRef empty_child() {
    ChildRef c;
    for (int k = 0; k < 3; ++k) {
        c.lo[k] = 1e30f;
        c.hi[k] = -1e30f;
    }
    c.ref = 0;
    c.count = -1;  // empty: the kernel skips count < 0 (a min/max slab test would accept an inverted box)
    return c;
}

BvhNode make_node(const ChildRef& c0, const ChildRef& c1) {
    BvhNode n;
    n.a[0] = c0.lo[0]; n.a[1] = c0.hi[0]; n.a[2] = c0.lo[1]; n.a[3] = c0.hi[1];
    n.b[0] = c1.lo[0]; n.b[1] = c1.hi[0]; n.b[2] = c1.lo[1]; n.b[3] = c1.hi[1];
    n.c[0] = c0.lo[2]; n.c[1] = c0.hi[2]; n.c[2] = c1.lo[2]; n.c[3] = c1.hi[2];
    n.d[0] = c0.ref; n.d[1] = c1.ref; n.d[2] = c0.count; n.d[3] = c1.count;
    return n;
}


// ---- tree rotations (BuildParams::rotation_passes) ----
namespace {
float half_area(const ChildRef& c) {
    const float dx = c.hi[0] - c.lo[0], dy = c.hi[1] - c.lo[1], dz = c.hi[2] - c.lo[2];
    return dx * dy + dy * dz + dz * dx;
}
ChildRef node_child(const BvhNode& n, int s) {
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
    return r;
}
void set_node_child(BvhNode& n, int s, const ChildRef& r) {
    float* xy = s == 0 ? n.a : n.b;
    xy[0] = r.lo[0];
    xy[1] = r.hi[0];
    xy[2] = r.lo[1];
    xy[3] = r.hi[1];
    n.c[2 * s] = r.lo[2];
    n.c[2 * s + 1] = r.hi[2];
    n.d[s] = r.ref;
    n.d[2 + s] = r.count;
}
bool is_inner(const ChildRef& c) { return c.count == 0 && c.ref >= 0; }
ChildRef unite(const ChildRef& a, const ChildRef& b, int32_t ref) {
    ChildRef r;
    for (int k = 0; k < 3; ++k) {
        r.lo[k] = std::min(a.lo[k], b.lo[k]);
        r.hi[k] = std::max(a.hi[k], b.hi[k]);
    }
    r.ref = ref;
    r.count = 0;
    return r;
}

// Heights (1 + the children's, leaves 0) by a post-order walk from the root; returns the root's.
int subtree_heights(const BvhBuild& b, std::vector<int>& h) {
    h.assign(b.nodes.size(), 0);
    if (!is_inner(b.root)) return 0;
    std::vector<int32_t> order, st{b.root.ref};
    while (!st.empty()) {
        const int32_t v = st.back();
        st.pop_back();
        order.push_back(v);
        for (int s = 0; s < 2; ++s) {
            const ChildRef c = node_child(b.nodes[(size_t)v], s);
            if (is_inner(c)) st.push_back(c.ref);
        }
    }
    for (size_t k = order.size(); k-- > 0;) {
        const int32_t v = order[k];
        int m = 0;
        for (int s = 0; s < 2; ++s) {
            const ChildRef c = node_child(b.nodes[(size_t)v], s);
            if (is_inner(c)) m = std::max(m, h[(size_t)c.ref]);
        }
        h[(size_t)v] = 1 + m;
    }
    return h[(size_t)b.root.ref];
}

// One top-down pass: at node N with children (L, R), L inner with children (L0, L1), swap R with
// the Lx whose exchange gives the smallest new L' = (R, Ly), if that is smaller than L (only L's
// box changes, so the sum of inner-node areas -- the SAH's traversal term -- drops by exactly the
// difference).  R moves one level down: allowed only while R's deepest inner node stays within
// the cap.  Boxes are unions of the stored (padded) child boxes, so every box stays conservative
// and the leaves are untouched.  Returns the number of rotations.  (Kensler's grandchild <->
// grandchild swaps as well: the same node visits per query on the C3 scene, not kept.)
int64_t rotation_pass(BvhBuild& b, int cap) {
    std::vector<int> h;
    subtree_heights(b, h);
    int64_t n_rot = 0;
    std::vector<std::pair<int32_t, int>> q;  // (node, depth below the tree's root + 1)
    if (is_inner(b.root)) q.push_back({b.root.ref, 1});
    for (size_t qi = 0; qi < q.size(); ++qi) {
        const int32_t N = q[qi].first;
        const int dN = q[qi].second;
        for (int side = 0; side < 2; ++side) {
            const ChildRef L = node_child(b.nodes[(size_t)N], side), R = node_child(b.nodes[(size_t)N], 1 - side);
            if (!is_inner(L) || (is_inner(R) && dN + 1 + h[(size_t)R.ref] > cap)) continue;
            const float aL = half_area(L);
            int best = -1;
            float best_a = aL;
            for (int x = 0; x < 2; ++x) {
                const float a = half_area(unite(R, node_child(b.nodes[(size_t)L.ref], 1 - x), L.ref));
                if (a < best_a) {
                    best_a = a;
                    best = x;
                }
            }
            if (best < 0) continue;
            const ChildRef Lx = node_child(b.nodes[(size_t)L.ref], best), Ly = node_child(b.nodes[(size_t)L.ref], 1 - best);
            set_node_child(b.nodes[(size_t)L.ref], best, R);
            set_node_child(b.nodes[(size_t)N], side, unite(R, Ly, L.ref));
            set_node_child(b.nodes[(size_t)N], 1 - side, Lx);
            h[(size_t)L.ref] = 1 + std::max(is_inner(R) ? h[(size_t)R.ref] : 0, is_inner(Ly) ? h[(size_t)Ly.ref] : 0);
            ++n_rot;
            break;  // one rotation per node and pass
        }
        for (int s = 0; s < 2; ++s) {
            const ChildRef c = node_child(b.nodes[(size_t)N], s);
            if (is_inner(c)) q.push_back({c.ref, dN + 1});
        }
    }
    return n_rot;
}
}  // namespace

void rotate_tree(BvhBuild& b, int passes) {
    if (passes <= 0 || !is_inner(b.root)) return;
    std::vector<int> h;
    const int cap = subtree_heights(b, h);  // the deepest inner node stays where it was built
    int64_t total = 0;
    for (int p = 0; p < passes; ++p) {
        const int64_t n = rotation_pass(b, cap);
        total += n;
        if (n == 0) break;
    }
    if (total == 0) return;
    // Rotations move subtrees under other parents: renumber the nodes in depth-first pre-order
    // (child 0 first, as the builder allocates them), so every parent precedes its children again
    // (validate_bvh, bfs_prefix_order and the receiver refit's level schedule rely on it).
    std::vector<int32_t> order, st{b.root.ref};
    order.reserve(b.nodes.size());
    while (!st.empty()) {
        const int32_t v = st.back();
        st.pop_back();
        order.push_back(v);
        for (int s = 1; s >= 0; --s) {
            const ChildRef c = node_child(b.nodes[(size_t)v], s);
            if (is_inner(c)) st.push_back(c.ref);
        }
    }
    std::vector<int32_t> remap(b.nodes.size(), -1);
    for (size_t k = 0; k < order.size(); ++k) remap[(size_t)order[k]] = (int32_t)k;
    std::vector<BvhNode> out(order.size());
    for (size_t k = 0; k < order.size(); ++k) {
        BvhNode nd = b.nodes[(size_t)order[k]];
        for (int s = 0; s < 2; ++s)
            if (nd.d[2 + s] == 0 && nd.d[s] >= 0) nd.d[s] = remap[(size_t)nd.d[s]];
        out[k] = nd;
    }
    b.nodes.swap(out);
    b.root.ref = remap[(size_t)b.root.ref];
}

void build_bvh(const float* tri_v, const float* tri_abs, float absorption_fill, int64_t n, int32_t id_base,
               BvhBuild& out) {
    out.nodes.clear();
    out.tris.clear();
    out.depth = 0;
    if (n <= 0) {
        out.root = empty_child();
        return;
    }
    if (build_params().spatial && n >= kSpatialMinTris) {
        SpatialBuilder sb;
        sb.out = &out;
        sb.tri_v = tri_v;
        sb.tri_abs = tri_abs;
        sb.abs_fill = absorption_fill;
        sb.id_base = id_base;
        float mx = 0.0f;
        std::vector<Ref> refs((size_t)n);
        Box root;
        for (int64_t i = 0; i < n; ++i) {
            const float* v = tri_v + 9 * i;
            Box& b = refs[(size_t)i].b;
            for (int k = 0; k < 3; ++k) {
                b.lo[k] = std::min(v[k], std::min(v[3 + k], v[6 + k]));
                b.hi[k] = std::max(v[k], std::max(v[3 + k], v[6 + k]));
                mx = std::max(mx, std::max(std::fabs(b.lo[k]), std::fabs(b.hi[k])));
            }
            refs[(size_t)i].idx = (int32_t)i;
            root.grow(b.lo, b.hi);
        }
        sb.pad = std::max(1e-5f * mx, 1e-6f);
        sb.min_overlap = sb.prm.spatial_alpha * root.area();
        sb.refs_left = (int64_t)((double)sb.prm.spatial_budget * (double)n);
        out.tris.reserve((size_t)n + (size_t)sb.refs_left);
        out.root = sb.build(refs, 1);
        rotate_tree(out, sb.prm.rotation_passes);
        return;
    }
    Builder b;
    b.out = &out;
    b.tri_v = tri_v;
    b.tri_abs = tri_abs;
    b.abs_fill = absorption_fill;
    b.id_base = id_base;
    float mx = 0.0f;
    b.prims.resize((size_t)n);
    for (int64_t i = 0; i < n; ++i) {
        Prim& p = b.prims[i];
        const float* v = tri_v + 9 * i;
        for (int k = 0; k < 3; ++k) {
            p.lo[k] = std::min(v[k], std::min(v[3 + k], v[6 + k]));
            p.hi[k] = std::max(v[k], std::max(v[3 + k], v[6 + k]));
            p.c[k] = 0.5f * (p.lo[k] + p.hi[k]);
            mx = std::max(mx, std::max(std::fabs(p.lo[k]), std::fabs(p.hi[k])));
        }
        p.idx = (int32_t)i;
    }
    b.pad = std::max(1e-5f * mx, 1e-6f);
    out.nodes.reserve((size_t)(2 * n / std::max(1, b.prm.leaf_max) + 16));
    out.tris.reserve((size_t)n);
    out.root = b.build(0, n, 1);
}

void relocate_bvh(BvhBuild& b, int32_t node_offset, int32_t tri_offset) {
    auto fix = [&](int32_t& ref, int32_t count) {
        if (count >= 0) ref += (count > 0) ? tri_offset : node_offset;
    };
    for (BvhNode& n : b.nodes) {
        fix(n.d[0], n.d[2]);
        fix(n.d[1], n.d[3]);
    }
    fix(b.root.ref, b.root.count);
}

void bfs_prefix_order(BvhBuild& b, size_t k) {
    const size_t n = b.nodes.size();
    if (n == 0 || b.root.count != 0) return;
    k = std::min(k, n);
    std::vector<int32_t> order;  // the first k inner nodes in breadth-first order
    order.reserve(k);
    order.push_back(b.root.ref);
    for (size_t h = 0; h < order.size() && order.size() < k; ++h) {
        const BvhNode& nd = b.nodes[(size_t)order[h]];
        for (int c = 0; c < 2 && order.size() < k; ++c)
            if (nd.d[2 + c] == 0) order.push_back(nd.d[c]);
    }
    std::vector<int32_t> map(n, -1);
    int32_t next = 0;
    for (int32_t i : order) map[(size_t)i] = next++;
    for (size_t i = 0; i < n; ++i)  // the rest keep their relative order (parents before children)
        if (map[i] < 0) map[i] = next++;
    std::vector<BvhNode> out(n);
    for (size_t i = 0; i < n; ++i) {
        BvhNode nd = b.nodes[i];
        for (int c = 0; c < 2; ++c)
            if (nd.d[2 + c] == 0) nd.d[c] = map[(size_t)nd.d[c]];
        out[(size_t)map[i]] = nd;
    }
    b.nodes.swap(out);
    b.root.ref = map[(size_t)b.root.ref];
}

bool validate_bvh(const BvhNode* nodes, size_t n_nodes, size_t n_tris, const char** why) {
    return validate_bvh_range(nodes, 0, n_nodes, n_nodes, n_tris, why);
}

bool validate_bvh_range(const BvhNode* nodes, size_t first, size_t n_nodes, size_t total_nodes, size_t n_tris,
                        const char** why) {
    // Every inner child must have a larger index than its parent (the builder emits nodes in
    // pre-order): that makes the graph acyclic, so traversal always terminates.
    for (size_t k = 0; k < n_nodes; ++k) {
        const size_t i = first + k;
        for (int c = 0; c < 2; ++c) {
            const int32_t ref = nodes[k].d[c], count = nodes[k].d[2 + c];
            if (count < 0) continue;
            if (count > 0) {
                if (ref < 0 || (size_t)ref + (size_t)count > n_tris) {
                    *why = "leaf range out of bounds";
                    return false;
                }
                if (count > 15 || ref >= (1 << 27)) {  // stack leaf tag: -(first*16 + count) - 1
                    *why = "leaf larger than 15 triangles or beyond 2^27 (degenerate scene)";
                    return false;
                }
            } else if (ref <= (int64_t)i || (size_t)ref >= total_nodes) {
                *why = "inner child index not after its parent";
                return false;
            }
        }
    }
    return true;
}

void code_nodes(const BvhNode* in, size_t n, BvhNode* out) {
    for (size_t i = 0; i < n; ++i) {
        BvhNode o = in[i];
        for (int c = 0; c < 2; ++c) {
            const int32_t ref = in[i].d[c], count = in[i].d[2 + c];
            o.d[c] = count < 0 ? kEmptyChildCode : count == 0 ? ref : ~(ref * 16 + count);
        }
        o.d[2] = 0;
        o.d[3] = 0;
        out[i] = o;
    }
}

QGrid make_qgrid(const float lo[3], const float hi[3], double margin_frac) {
    double ext = 0.0;
    for (int k = 0; k < 3; ++k) ext = std::max(ext, (double)hi[k] - (double)lo[k]);
    const double margin = std::max(margin_frac * ext, 1e-2);
    QGrid g;
    for (int k = 0; k < 3; ++k) {
        const double o = (double)lo[k] - margin;
        const double e = ((double)hi[k] + margin) - o;
        g.origin[k] = (float)o;
        // plane q = 65535 lies past hi + margin/2 even after the f32 rounding of origin and scale
        g.scale[k] = (float)(e / 65000.0);
    }
    return g;
}

namespace {
// Outward rounding margin in grid steps: kQ16Margin (arx_layout.hpp, with the kernel's error bound).
constexpr double kQMargin = kQ16Margin;
// Outward grid index of a plane (lo: floor, hi: ceil) with the margin above; < 0 / > 65535
// when it falls outside the grid.
int64_t q_lo(const QGrid& g, int k, float v) {
    return (int64_t)std::floor(((double)v - (double)g.origin[k]) / (double)g.scale[k] - kQMargin);
}
int64_t q_hi(const QGrid& g, int k, float v) {
    return (int64_t)std::ceil(((double)v - (double)g.origin[k]) / (double)g.scale[k] + kQMargin);
}
}  // namespace

bool qgrid_contains(const QGrid& g, const float lo[3], const float hi[3]) {
    for (int k = 0; k < 3; ++k) {
        if (!(g.scale[k] > 0.0f) || !std::isfinite(lo[k]) || !std::isfinite(hi[k])) return false;
        if (q_lo(g, k, lo[k]) < 0 || q_hi(g, k, hi[k]) > 65535) return false;
    }
    return true;
}

bool quantize_nodes16(const BvhNode* coded, size_t n, const QGrid& g, QNode2* out) {
    for (size_t i = 0; i < n; ++i) {
        const BvhNode& b = coded[i];
        // child c: x = (a|b)[0..1], y = (a|b)[2..3], z = c[2c .. 2c+1]
        for (int c = 0; c < 2; ++c) {
            const float* xy = c == 0 ? b.a : b.b;
            const float lo[3] = {xy[0], xy[2], b.c[2 * c]};
            const float hi[3] = {xy[1], xy[3], b.c[2 * c + 1]};
            const bool empty = b.d[c] == kEmptyChildCode;
            for (int k = 0; k < 3; ++k) {
                uint32_t ql = 1, qh = 0;  // empty: the slab between planes 0 and 1 (grid corner)
                if (!empty) {
                    if (!(lo[k] <= hi[k])) return false;
                    const int64_t l = q_lo(g, k, lo[k]), h = q_hi(g, k, hi[k]);
                    if (l < 0 || h > 65535) return false;
                    ql = (uint32_t)l;
                    qh = (uint32_t)h;
                }
                out[i].c[c].q[k] = ql | (qh << 16);
            }
            out[i].c[c].code = b.d[c];
        }
    }
    return true;
}

}  // namespace arx
