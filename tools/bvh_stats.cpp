// bvh_stats -- host-side traversal statistics of the trace kernel's trees (design tool).
//
// Builds the production binary SAH tree (arx_bvh.cpp), then replays closest-hit queries of
// bouncing rays (specular reflection, same scene) and counts per query: node visits, triangle
// tests and bytes fetched.  (The 4-/8-wide collapses it compared in round 1 are in the git
// history at commit 62a5de6.)
//
//   g++ -O2 -std=c++17 -I audiorenderingv2_amd/csrc tools/bvh_stats.cpp \
//       audiorenderingv2_amd/csrc/arx_bvh.cpp oracle/liboracle.so -o /tmp/bvh_stats
//   /tmp/bvh_stats scene.f32 n_tris ex ey ez n_rays bounces
// (The insertion-based optimisation tried in round 4 -- REINSERT / RESEG -- is at commit 198ae4a.)
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "arx_bvh.hpp"
extern "C" void orc_ray_direction(uint64_t seed, uint64_t ray_id, float dir[3]);  // oracle/arx_oracle.c (CHAINS=1)

using namespace arx;

struct Q {
    float o[3], d[3], inv[3];
};

static bool tri_hit(const TriRec& t, const Q& q, float& tt) {
    // Moller-Trumbore (statistics only; the product uses the watertight test)
    const float e1[3] = {t.v1[0] - t.v0[0], t.v1[1] - t.v0[1], t.v1[2] - t.v0[2]};
    const float e2[3] = {t.v2[0] - t.v0[0], t.v2[1] - t.v0[1], t.v2[2] - t.v0[2]};
    const float p[3] = {q.d[1] * e2[2] - q.d[2] * e2[1], q.d[2] * e2[0] - q.d[0] * e2[2], q.d[0] * e2[1] - q.d[1] * e2[0]};
    const float det = e1[0] * p[0] + e1[1] * p[1] + e1[2] * p[2];
    if (std::fabs(det) < 1e-12f) return false;
    const float inv = 1.0f / det;
    const float s[3] = {q.o[0] - t.v0[0], q.o[1] - t.v0[1], q.o[2] - t.v0[2]};
    const float u = (s[0] * p[0] + s[1] * p[1] + s[2] * p[2]) * inv;
    if (u < 0 || u > 1) return false;
    const float qq[3] = {s[1] * e1[2] - s[2] * e1[1], s[2] * e1[0] - s[0] * e1[2], s[0] * e1[1] - s[1] * e1[0]};
    const float v = (q.d[0] * qq[0] + q.d[1] * qq[1] + q.d[2] * qq[2]) * inv;
    if (v < 0 || u + v > 1) return false;
    tt = (e2[0] * qq[0] + e2[1] * qq[1] + e2[2] * qq[2]) * inv;
    return tt >= 0;
}

static bool slab(const float lo[3], const float hi[3], const Q& q, float tmax, float& tn) {
    float a = 0.0f, b = tmax;
    for (int k = 0; k < 3; ++k) {
        float t0 = (lo[k] - q.o[k]) * q.inv[k], t1 = (hi[k] - q.o[k]) * q.inv[k];
        if (t0 > t1) std::swap(t0, t1);
        a = std::max(a, t0);
        b = std::min(b, t1);
    }
    tn = a;
    return a <= b;
}

struct Stats {
    double visits = 0, tests = 0, leaves = 0, maxstack = 0, skips2 = 0;
    double shallow[8] = {};  // visits to nodes at depth <= 2 + k below the top node
    double nhit[9] = {};     // visits by number of children hit
};

struct Tree {
    int W;
    std::vector<ChildRef> kids;  // W per node
    size_t n = 0;
    std::vector<int> depth;  // node depth below the top node (0)
    std::vector<int> parent, owner;  // parent node of each node; the node holding each triangle record's leaf
    void set_links(size_t n_recs) {
        parent.assign(n, -1);
        owner.assign(n_recs, -1);
        for (size_t i = 0; i < n; ++i)
            for (int s = 0; s < W; ++s) {
                const ChildRef& c = kids[(size_t)W * i + s];
                if (c.count == 0 && c.ref >= 0 && (size_t)c.ref < n) parent[c.ref] = (int)i;
                if (c.count > 0)
                    for (int k = 0; k < c.count; ++k) owner[(size_t)c.ref + k] = (int)i;
            }
    }
    static int code_of(const ChildRef& c) { return c.count > 0 ? -(c.ref * 16 + c.count) - 1 : c.ref; }
    // ENTRY=k: start a bounce's query at the ancestor (depth <= k) of the node holding the record it
    // left from, with the siblings of that ancestor's path pushed untested (deepest on top)
    void entry_stack(int rec, int k, std::vector<int>& out) const {
        out.clear();
        int e = owner[(size_t)rec];
        while (depth[(size_t)e] > k) e = parent[(size_t)e];
        std::vector<int> sib;
        for (int x = e; parent[(size_t)x] >= 0; x = parent[(size_t)x]) {
            const int p = parent[(size_t)x];
            for (int s = 0; s < W; ++s) {
                const ChildRef& c = kids[(size_t)W * p + s];
                if (c.count < 0) continue;
                if (c.count == 0 && c.ref == x) continue;
                sib.push_back(code_of(c));
            }
        }
        for (auto it = sib.rbegin(); it != sib.rend(); ++it) out.push_back(*it);
        out.push_back(e);
    }
    // ENTRYT=k: as ENTRY, but each sibling's box (the 16-B half of its parent that holds it) is tested
    // against the query first and pushed only when hit; returns the boxes tested
    int entry_stack_tested(int rec, int k, const Q& q, std::vector<int>& out) const {
        out.clear();
        int e = owner[(size_t)rec];
        while (depth[(size_t)e] > k) e = parent[(size_t)e];
        std::vector<int> sib;
        int tested = 0;
        for (int x = e; parent[(size_t)x] >= 0; x = parent[(size_t)x]) {
            const int p = parent[(size_t)x];
            for (int s = 0; s < W; ++s) {
                const ChildRef& c = kids[(size_t)W * p + s];
                if (c.count < 0) continue;
                if (c.count == 0 && c.ref == x) continue;
                ++tested;
                float tn;
                if (slab(c.lo, c.hi, q, 1e30f, tn)) sib.push_back(code_of(c));
            }
        }
        for (auto it = sib.rbegin(); it != sib.rend(); ++it) out.push_back(*it);
        out.push_back(e);
        return tested;
    }
    void set_depths() {
        depth.assign(n, 1 << 20);
        depth[0] = 0;
        for (size_t i = 0; i < n; ++i)  // parents come before their children
            for (int s = 0; s < W; ++s) {
                const ChildRef& c = kids[(size_t)W * i + s];
                if (c.count == 0 && c.ref >= 0 && (size_t)c.ref < n) depth[c.ref] = std::min(depth[c.ref], depth[i] + 1);
            }
    }
};

static Tree from_binary(const std::vector<BvhNode>& nodes, const BvhNode& top) {
    Tree t;
    t.W = 2;
    t.n = nodes.size() + 1;
    t.kids.resize(2 * t.n);
    auto put = [&](size_t i, const BvhNode& n) {
        for (int c = 0; c < 2; ++c) {
            ChildRef& r = t.kids[2 * i + c];
            const float* ab = c == 0 ? n.a : n.b;
            r.lo[0] = ab[0]; r.hi[0] = ab[1]; r.lo[1] = ab[2]; r.hi[1] = ab[3];
            r.lo[2] = n.c[2 * c]; r.hi[2] = n.c[2 * c + 1];
            r.ref = n.d[c];
            r.count = n.d[2 + c];
        }
    };
    put(0, top);
    for (size_t i = 0; i < nodes.size(); ++i) put(i + 1, nodes[i]);
    return t;
}


// closest hit with near-first order; returns hit tri index or -1
static int trace(const Tree& t, const std::vector<TriRec>& tris, const Q& q, Stats& st, float& best,
                 const std::vector<int>* start = nullptr) {
    best = 1e30f;
    int hit = -1;
    std::vector<std::pair<float, int>> stack;  // (tn, code) ; code >= 0 node, < 0 leaf
    if (start && !start->empty())  // ENTRY: the untested siblings of the entry node's path, then the entry node
        for (int c : *start) stack.push_back({0.0f, c});
    else
        stack.push_back({0.0f, 0});
    size_t maxs = 0;
    bool after_leaf = false, continue_culling = false;
    while (!stack.empty()) {
        auto [tn0, code] = stack.back();  // (copies: DEPTH2 may replace them)
        stack.pop_back();
        static const bool nocull = std::getenv("NOCULL") != nullptr;  // the GPU stack keeps no distances
        // QCULL=k: the kernel's packed stack word (round 5) -- the entry distance kept as a 7-bit
        // lower bound floor(tn * 2^k) (saturating at 127), a pop culled when that bound exceeds the
        // best hit; DEPTH2=1: only the two topmost entries are looked at per pop (a culled top is
        // replaced by the one below it, which is taken unchecked)
        static const int qcull = std::getenv("QCULL") ? std::atoi(std::getenv("QCULL")) : -1;
        static const bool depth2 = std::getenv("DEPTH2") != nullptr;
        // LEAFCULL=1: pops are checked only right after a leaf (where the best hit changes), and
        // there as many as are culled; a node step's own pop is taken unchecked
        static const bool leafcull = std::getenv("LEAFCULL") != nullptr;
        const bool check = !leafcull || after_leaf;
        after_leaf = false;
        if (qcull >= 0 && leafcull) {
            auto key = [&](float tn) { return std::min(255.0f, std::floor(tn * std::ldexp(1.0f, qcull))); };
            auto culled = [&](float tn) { return key(tn) > std::floor(best * std::ldexp(1.0f, qcull)); };
            if (check && culled(tn0)) continue_culling = true;
            if (continue_culling) {
                if (culled(tn0)) continue;
                continue_culling = false;
            }
        } else if (qcull >= 0) {
            auto key = [&](float tn) { return std::min(127.0f, std::floor(tn * std::ldexp(1.0f, qcull))); };
            auto culled = [&](float tn) { return key(tn) > std::floor(best * std::ldexp(1.0f, qcull)); };
            if (culled(tn0)) {
                if (!depth2) continue;
                if (stack.empty()) break;
                auto nx = stack.back();
                stack.pop_back();
                tn0 = nx.first;
                code = nx.second;
                st.skips2 += 1;
            }
        } else if (tn0 > best && !nocull) {
            continue;
        }
        if (code < 0) {
            const int v = -code - 1, first = v >> 4, cnt = v & 15;
            st.leaves += 1;
            after_leaf = true;
            for (int k = 0; k < cnt; ++k) {
                st.tests += 1;
                float tt;
                if (tri_hit(tris[first + k], q, tt) && tt < best) {
                    best = tt;
                    hit = first + k;
                }
            }
            continue;
        }
        st.visits += 1;
        if (!t.depth.empty())
            for (int k = 0; k < 8; ++k) st.shallow[k] += t.depth[code] <= 2 + k ? 1 : 0;
        std::vector<std::pair<float, int>> hits;
        for (int s = 0; s < t.W; ++s) {
            const ChildRef& c = t.kids[(size_t)t.W * code + s];
            if (c.count < 0) continue;
            float tn;
            if (!slab(c.lo, c.hi, q, best, tn)) continue;
            hits.push_back({tn, c.count > 0 ? -(c.ref * 16 + c.count) - 1 : c.ref});
        }
        st.nhit[std::min<size_t>(hits.size(), 8)] += 1;
        std::sort(hits.begin(), hits.end(), [](auto& a, auto& b) { return a.first > b.first; });
        for (auto& h : hits) stack.push_back(h);
        maxs = std::max(maxs, stack.size());
    }
    st.maxstack = std::max(st.maxstack, (double)maxs);
    return hit;
}

int main(int argc, char** argv) {
    if (argc < 8) {
        std::fprintf(stderr, "usage: bvh_stats scene.f32 n_tris ex ey ez n_rays bounces\n");
        return 1;
    }
    const long n = std::atol(argv[2]);
    std::vector<float> tv(9 * n);
    FILE* f = std::fopen(argv[1], "rb");
    if (!f || std::fread(tv.data(), 4, tv.size(), f) != tv.size()) return 2;
    std::fclose(f);
    const float em[3] = {(float)std::atof(argv[3]), (float)std::atof(argv[4]), (float)std::atof(argv[5])};
    const int nr = std::atoi(argv[6]), nb = std::atoi(argv[7]);
    BuildParams& bp = build_params();
    if (const char* e = std::getenv("BINS")) bp.bins = std::atoi(e);
    if (const char* e = std::getenv("LEAF")) bp.leaf_max = std::atoi(e);
    if (const char* e = std::getenv("TRAV")) bp.trav_cost = (float)std::atof(e);
    if (const char* e = std::getenv("ISECT")) bp.isect_cost = (float)std::atof(e);
    if (const char* e = std::getenv("SPATIAL")) bp.spatial = std::atoi(e) != 0;
    if (const char* e = std::getenv("ALPHA")) bp.spatial_alpha = (float)std::atof(e);
    if (const char* e = std::getenv("SDEPTH")) bp.spatial_max_depth = std::atoi(e);
    if (const char* e = std::getenv("BUDGET")) bp.spatial_budget = (float)std::atof(e);
    if (const char* e = std::getenv("ROT")) bp.rotation_passes = std::atoi(e);
    std::printf("params: bins %d leaf_max %d trav %.2f isect %.2f rotation passes %d\n", bp.bins, bp.leaf_max, bp.trav_cost,
                bp.isect_cost, bp.rotation_passes);
    BvhBuild b;
    std::vector<float> ab(n, 0.5f);
    const auto t_build = std::chrono::steady_clock::now();
    build_bvh(tv.data(), ab.data(), 0.5f, n, 0, b);
    std::printf("build %.2f s\n", std::chrono::duration<double>(std::chrono::steady_clock::now() - t_build).count());
    relocate_bvh(b, 1, 0);
    BvhNode top = make_node(b.root, empty_child());
    Tree t2 = from_binary(b.nodes, top);
    std::printf("spatial %d alpha %g budget %g: refs %zu\n", (int)bp.spatial, bp.spatial_alpha, bp.spatial_budget, b.tris.size());
    std::printf("tris %ld  binary nodes %zu depth %d\n", n, b.nodes.size(), b.depth);
    t2.set_depths();
    t2.set_links(b.tris.size());
    const int entry_k = std::getenv("ENTRY") ? std::atoi(std::getenv("ENTRY")) : -1;
    const int entry_t = std::getenv("ENTRYT") ? std::atoi(std::getenv("ENTRYT")) : -1;
    double sib_tests = 0;
    {
        int md = 0;
        for (size_t i = 0; i < t2.n; ++i)
            if (t2.depth[i] < (1 << 20)) md = std::max(md, t2.depth[i]);
        std::printf("max inner-node depth below the top node: %d\n", md);
    }
    {
        long cnt[40] = {};
        for (size_t i = 0; i < t2.n; ++i) if (t2.depth[i] < 40) ++cnt[t2.depth[i]];
        long cum = 0;
        std::printf("binary nodes by depth (cumulative):");
        for (int d = 0; d < 12; ++d) std::printf(" %d:%ld", d, cum += cnt[d]);
        std::printf("\n");
    }
    Tree* trees[1] = {&t2};
    const double node_bytes[1] = {32};  // QNode2
    std::uniform_real_distribution<float> U(0.0f, 1.0f);
    for (int k = 0; k < 1; ++k) {
        Stats st;
        long queries = 0;
        std::mt19937 r2(7);
        // per-ray node visits (CHAINS=1: the launch's rays in order, directions from the oracle's
        // Philox stream, seed 1): the lane chains of the small-launch trace (one ray per lane)
        static const bool chains = std::getenv("CHAINS") != nullptr;
        std::vector<double> ray_visits;
        for (int i = 0; i < nr; ++i) {
            const float z = 2 * U(r2) - 1, ph = 6.2831853f * U(r2), s = std::sqrt(1 - z * z);
            Q q;
            float o[3] = {em[0], em[1], em[2]}, d[3] = {s * std::cos(ph), s * std::sin(ph), z};
            if (chains) orc_ray_direction(1, (uint64_t)i, d);
            const double v_before = st.visits + st.leaves;
            std::vector<int> start;
            for (int bn = 0; bn < nb; ++bn) {
                for (int a = 0; a < 3; ++a) {
                    q.o[a] = o[a];
                    q.d[a] = d[a];
                    q.inv[a] = 1.0f / (std::fabs(d[a]) < 1e-20f ? 1e-20f : d[a]);
                }
                float tt;
                const int h = trace(*trees[k], b.tris, q, st, tt, &start);
                ++queries;
                if (h < 0) break;
                if (entry_k >= 0) trees[k]->entry_stack(h, entry_k, start);
                const int hit_rec = h;
                const TriRec& tr = b.tris[h];
                const float e1[3] = {tr.v1[0] - tr.v0[0], tr.v1[1] - tr.v0[1], tr.v1[2] - tr.v0[2]};
                const float e2[3] = {tr.v2[0] - tr.v0[0], tr.v2[1] - tr.v0[1], tr.v2[2] - tr.v0[2]};
                float ng[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
                const float l = std::sqrt(ng[0] * ng[0] + ng[1] * ng[1] + ng[2] * ng[2]);
                for (float& c : ng) c /= l;
                const float dn = 2 * (d[0] * ng[0] + d[1] * ng[1] + d[2] * ng[2]);
                for (int a = 0; a < 3; ++a) {
                    o[a] = o[a] + tt * d[a];
                    d[a] -= dn * ng[a];
                    o[a] += 1e-3f * d[a];
                }
                if (entry_t >= 0) {
                    Q qn;
                    for (int a = 0; a < 3; ++a) {
                        qn.o[a] = o[a];
                        qn.d[a] = d[a];
                        qn.inv[a] = 1.0f / (std::fabs(d[a]) < 1e-20f ? 1e-20f : d[a]);
                    }
                    sib_tests += trees[k]->entry_stack_tested(hit_rec, entry_t, qn, start);
                }
            }
            if (chains) ray_visits.push_back(st.visits + st.leaves - v_before);
        }
        if (chains && !ray_visits.empty()) {
            // waves of 64 consecutive rays (the small launch's static ranges): a wave's lanes step
            // in lockstep, so its chain is at least its longest lane's
            std::vector<double> wave_max;
            for (size_t w = 0; w < ray_visits.size(); w += 64)
                wave_max.push_back(*std::max_element(ray_visits.begin() + w,
                                                     ray_visits.begin() + std::min(ray_visits.size(), w + 64)));
            std::vector<double> sv = ray_visits;
            std::sort(sv.begin(), sv.end());
            std::sort(wave_max.begin(), wave_max.end());
            double mean = 0;
            for (double v : sv) mean += v;
            mean /= sv.size();
            std::printf("per-ray node steps + leaf visits: mean %.1f p50 %.0f p99 %.0f p99.9 %.0f max %.0f\n", mean,
                        sv[sv.size() / 2], sv[sv.size() * 99 / 100], sv[sv.size() * 999 / 1000], sv.back());
            std::printf("per-wave (64 rays) longest lane: mean %.1f p50 %.0f max %.0f\n",
                        [&] { double m = 0; for (double v : wave_max) m += v; return m / wave_max.size(); }(),
                        wave_max[wave_max.size() / 2], wave_max.back());
        }
        const double v = st.visits / queries, te = st.tests / queries, lv = st.leaves / queries;
        if (entry_t >= 0) std::printf("ENTRYT=%d: sibling box tests per query %.2f\n", entry_t, sib_tests / queries);
        std::printf("W=%d: %ld queries  visits %.1f  leaves %.1f  tri tests %.1f  node bytes %.0f  tri bytes %.0f  "
                    "max stack %.0f\n",
                    trees[k]->W, queries, v, lv, te, v * node_bytes[k], te * 48.0, st.maxstack);
        std::printf("   visits by children hit: 0: %.3f 1: %.3f 2: %.3f 3+: %.3f\n", st.nhit[0] / st.visits,
                    st.nhit[1] / st.visits, st.nhit[2] / st.visits,
                    (st.visits - st.nhit[0] - st.nhit[1] - st.nhit[2]) / st.visits);
        if (k == 0) {
            std::printf("   share of visits at depth <=");
            for (int d = 0; d < 8; ++d) std::printf(" %d: %.3f", 2 + d, st.shallow[d] / st.visits);
            std::printf("\n");
        }
    }
    return 0;
}
