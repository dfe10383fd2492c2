// layout_stats -- cache-line behaviour of BVH node orders for the trace kernel (design tool).
//
// Builds the production tree (arx_bvh.cpp, SBVH by default), replays bouncing closest-hit
// queries (nearest-first, like node_step8) and reports, per node layout, how many 128-B lines
// a query's node fetches touch and how often a fetch hits the line of the ray's previous
// fetch, for 32-B (QNode2) nodes.  Layouts: the builder's depth-first order, and treelets
// (a node with its inner children, optionally one grandchild, packed into one 128-B line).
//
//   g++ -O2 -std=c++17 -pthread -I audiorenderingv2_amd/csrc tools/layout_stats.cpp \
//       audiorenderingv2_amd/csrc/arx_bvh.cpp -o /tmp/layout_stats
//   /tmp/layout_stats scene.f32 n_tris ex ey ez n_rays bounces
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <unordered_set>
#include <vector>

#include "arx_bvh.hpp"

using namespace arx;

struct Q {
    float o[3], d[3], inv[3];
};

static bool tri_hit(const TriRec& t, const Q& q, float& tt) {
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

static bool slab(const BvhNode& n, int c, const Q& q, float tmax, float& tn) {
    const float* ab = c == 0 ? n.a : n.b;
    const float lo[3] = {ab[0], ab[2], n.c[2 * c]}, hi[3] = {ab[1], ab[3], n.c[2 * c + 1]};
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

// fetched node indices of one closest-hit query (nearest-first, far child pushed)
static int trace(const std::vector<BvhNode>& nodes, const std::vector<TriRec>& tris, const Q& q,
                 std::vector<int>& fetched, float& best) {
    best = 1e30f;
    int hit = -1;
    std::vector<int> stack;
    int node = 0;
    fetched.clear();
    while (true) {
        if (node >= 0) {
            fetched.push_back(node);
            const BvhNode& n = nodes[node];
            float tn0, tn1;
            const bool h0 = n.d[2] >= 0 && slab(n, 0, q, best, tn0);
            const bool h1 = n.d[3] >= 0 && slab(n, 1, q, best, tn1);
            auto code = [&](int c) { return n.d[2 + c] > 0 ? -(n.d[c] * 16 + n.d[2 + c]) - 1 : n.d[c]; };
            if (h0 && h1) {
                const bool near1 = tn1 < tn0;
                stack.push_back(code(near1 ? 0 : 1));
                node = code(near1 ? 1 : 0);
            } else if (h0 || h1) {
                node = code(h0 ? 0 : 1);
            } else {
                if (stack.empty()) break;
                node = stack.back();
                stack.pop_back();
            }
            continue;
        }
        const int v = -node - 1, first = v >> 4, cnt = v & 15;
        for (int k = 0; k < cnt; ++k) {
            float tt;
            if (tri_hit(tris[first + k], q, tt) && tt < best) {
                best = tt;
                hit = first + k;
            }
        }
        if (stack.empty()) break;
        node = stack.back();
        stack.pop_back();
    }
    return hit;
}

// treelet layout: slot (128 B = 4 nodes) per treelet root, holding the root, its inner
// children and (grand > 0) the first inner grandchild.  Returns position (in nodes) per node.
static std::vector<int64_t> treelets(const std::vector<BvhNode>& nodes, bool grand, int64_t& used) {
    std::vector<int64_t> pos(nodes.size(), -1);
    std::vector<int> roots{0};
    int64_t next = 0;
    auto inner = [&](int n, int c) { return nodes[n].d[2 + c] == 0 ? nodes[n].d[c] : -1; };
    while (!roots.empty()) {
        const int r = roots.back();
        roots.pop_back();
        next = (next + 3) & ~int64_t(3);
        int slot[4] = {r, -1, -1, -1};
        int k = 1;
        for (int c = 0; c < 2; ++c)
            if (inner(r, c) >= 0) slot[k++] = inner(r, c);
        std::vector<int> later;
        if (grand && k < 4) {
            for (int j = 1; j < k && k < 4; ++j)
                for (int c = 0; c < 2 && k < 4; ++c)
                    if (inner(slot[j], c) >= 0) slot[k++] = inner(slot[j], c);
        }
        std::vector<char> placed(4, 0);
        for (int j = 0; j < k; ++j) pos[slot[j]] = next + j;
        // children of the slot's nodes that are not in the slot become treelet roots
        for (int j = k - 1; j >= 0; --j)
            for (int c = 1; c >= 0; --c) {
                const int ch = inner(slot[j], c);
                if (ch < 0) continue;
                bool in = false;
                for (int m = 0; m < k; ++m) in |= slot[m] == ch;
                if (!in) roots.push_back(ch);
            }
        next += k;
    }
    used = next;
    return pos;
}

int main(int argc, char** argv) {
    if (argc < 8) {
        std::fprintf(stderr, "usage: layout_stats scene.f32 n_tris ex ey ez n_rays bounces\n");
        return 1;
    }
    const long n = std::atol(argv[2]);
    std::vector<float> tv(9 * n);
    FILE* f = std::fopen(argv[1], "rb");
    if (!f || std::fread(tv.data(), 4, tv.size(), f) != tv.size()) return 2;
    std::fclose(f);
    const float em[3] = {(float)std::atof(argv[3]), (float)std::atof(argv[4]), (float)std::atof(argv[5])};
    const int nr = std::atoi(argv[6]), nb = std::atoi(argv[7]);
    BvhBuild b;
    build_bvh(tv.data(), nullptr, 0.5f, n, 0, b);
    std::printf("nodes %zu refs %zu depth %d\n", b.nodes.size(), b.tris.size(), b.depth);
    int64_t used_t = 0, used_g = 0;
    std::vector<int64_t> dfs(b.nodes.size());
    for (size_t i = 0; i < dfs.size(); ++i) dfs[i] = (int64_t)i;
    const std::vector<int64_t> t3 = treelets(b.nodes, false, used_t);
    const std::vector<int64_t> t4 = treelets(b.nodes, true, used_g);
    struct L {
        const char* name;
        const std::vector<int64_t>* pos;
        int64_t size;
        double same = 0, lines = 0, fetch = 0;
    } layouts[] = {{"depth-first", &dfs, (int64_t)dfs.size()}, {"treelet(node+children)", &t3, used_t},
                   {"treelet(+grandchild)", &t4, used_g}};
    std::uniform_real_distribution<float> U(0.0f, 1.0f);
    std::mt19937 rng(7);
    std::vector<int> fetched;
    long queries = 0;
    for (int i = 0; i < nr; ++i) {
        const float z = 2 * U(rng) - 1, ph = 6.2831853f * U(rng), s = std::sqrt(1 - z * z);
        float o[3] = {em[0], em[1], em[2]}, d[3] = {s * std::cos(ph), s * std::sin(ph), z};
        for (int bn = 0; bn < nb; ++bn) {
            Q q;
            for (int a = 0; a < 3; ++a) {
                q.o[a] = o[a];
                q.d[a] = d[a];
                q.inv[a] = 1.0f / (std::fabs(d[a]) < 1e-20f ? 1e-20f : d[a]);
            }
            float tt;
            const int h = trace(b.nodes, b.tris, q, fetched, tt);
            ++queries;
            for (L& l : layouts) {
                std::unordered_set<int64_t> lines;
                int64_t prev = -1;
                for (int nd : fetched) {
                    const int64_t line = (*l.pos)[nd] / 4;  // 4 x 32-B nodes per 128-B line
                    l.same += line == prev;
                    prev = line;
                    lines.insert(line);
                }
                l.lines += (double)lines.size();
                l.fetch += (double)fetched.size();
            }
            if (h < 0) break;
            const TriRec& tr = b.tris[h];
            const float e1[3] = {tr.v1[0] - tr.v0[0], tr.v1[1] - tr.v0[1], tr.v1[2] - tr.v0[2]};
            const float e2[3] = {tr.v2[0] - tr.v0[0], tr.v2[1] - tr.v0[1], tr.v2[2] - tr.v0[2]};
            float ng[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
            const float ln = std::sqrt(ng[0] * ng[0] + ng[1] * ng[1] + ng[2] * ng[2]);
            for (float& c : ng) c /= ln;
            const float dn = 2 * (d[0] * ng[0] + d[1] * ng[1] + d[2] * ng[2]);
            for (int a = 0; a < 3; ++a) {
                o[a] = o[a] + tt * d[a];
                d[a] -= dn * ng[a];
                o[a] += 1e-3f * d[a];
            }
        }
    }
    for (const L& l : layouts)
        std::printf("%-24s size %.1f MB  fetches/query %.1f  distinct lines/query %.1f  same line as previous %.3f\n",
                    l.name, (double)l.size * 32 / 1e6, l.fetch / queries, l.lines / queries, l.same / l.fetch);
    return 0;
}
