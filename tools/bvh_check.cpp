// bvh_check -- host-side correctness checks of the production BVH builder (tests/test_bvh_host.py).
//
// For a triangle soup (raw f32, 9 per triangle) it builds the default tree (arx_bvh.cpp: SBVH
// with spatial splits), its coded copy and the 16-bit quantized copy, and checks:
//   1. structure (validate_bvh) and that every triangle is referenced by some leaf, after the
//      breadth-first renumbering of the top nodes (bfs_prefix_order, as arx_set_scene);
//   2. every quantized child box contains its f32 box (outward rounding), in exact arithmetic;
//   3. closest hits of random rays through the f32 tree and through the dequantized tree equal
//      the brute-force closest hit (same triangle id, same t) -- i.e. the spatial splits never
//      drop the part of a triangle a ray hits.
// Exit status 0 and "ok ..." on success.
//
//   g++ -O2 -std=c++17 -pthread -I audiorenderingv2_amd/csrc tools/bvh_check.cpp \
//       audiorenderingv2_amd/csrc/arx_bvh.cpp -o /tmp/bvh_check && /tmp/bvh_check scene.f32 n_tris n_rays
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "arx_bvh.hpp"

using namespace arx;

namespace {

struct Ray {
    double o[3], d[3];
};

// double-precision Moller-Trumbore with a tiny tolerance: the same test for brute force and
// for the trees, so the comparison checks traversal coverage only
bool hit_tri(const float* v, const Ray& r, double& t) {
    double e1[3], e2[3], p[3], s[3], q[3];
    for (int k = 0; k < 3; ++k) {
        e1[k] = (double)v[3 + k] - v[k];
        e2[k] = (double)v[6 + k] - v[k];
        s[k] = r.o[k] - v[k];
    }
    p[0] = r.d[1] * e2[2] - r.d[2] * e2[1];
    p[1] = r.d[2] * e2[0] - r.d[0] * e2[2];
    p[2] = r.d[0] * e2[1] - r.d[1] * e2[0];
    const double det = e1[0] * p[0] + e1[1] * p[1] + e1[2] * p[2];
    if (std::fabs(det) < 1e-18) return false;
    const double inv = 1.0 / det;
    const double u = (s[0] * p[0] + s[1] * p[1] + s[2] * p[2]) * inv;
    if (u < 0.0 || u > 1.0) return false;
    q[0] = s[1] * e1[2] - s[2] * e1[1];
    q[1] = s[2] * e1[0] - s[0] * e1[2];
    q[2] = s[0] * e1[1] - s[1] * e1[0];
    const double w = (r.d[0] * q[0] + r.d[1] * q[1] + r.d[2] * q[2]) * inv;
    if (w < 0.0 || u + w > 1.0) return false;
    t = (e2[0] * q[0] + e2[1] * q[1] + e2[2] * q[2]) * inv;
    return t >= 0.0;
}

struct Box {
    double lo[3], hi[3];
};

bool slab(const Box& b, const Ray& r, double tmax) {
    double a = 0.0, z = tmax;
    for (int k = 0; k < 3; ++k) {
        if (r.d[k] == 0.0) {
            if (r.o[k] < b.lo[k] || r.o[k] > b.hi[k]) return false;
            continue;
        }
        double t0 = (b.lo[k] - r.o[k]) / r.d[k], t1 = (b.hi[k] - r.o[k]) / r.d[k];
        if (t0 > t1) std::swap(t0, t1);
        a = std::max(a, t0);
        z = std::min(z, t1);
    }
    return a <= z;
}

Box child_box(const BvhNode& n, int c) {
    const float* ab = c == 0 ? n.a : n.b;
    return Box{{ab[0], ab[2], n.c[2 * c]}, {ab[1], ab[3], n.c[2 * c + 1]}};
}

Box qbox(const QNode2& q, int c, const QGrid& g) {
    Box b;
    for (int k = 0; k < 3; ++k) {
        const uint32_t w = q.c[c].q[k];
        b.lo[k] = (double)g.origin[k] + (double)(w & 0xffffu) * (double)g.scale[k];
        b.hi[k] = (double)g.origin[k] + (double)(w >> 16) * (double)g.scale[k];
    }
    return b;
}

// closest hit through the tree (boxes from `box(node, child)`), tie -> lowest triangle id
template <typename BoxFn>
int closest(const std::vector<BvhNode>& nodes, const std::vector<TriRec>& tris, const Ray& r, BoxFn box,
            double& best) {
    best = 1e300;
    int best_id = -1;
    std::vector<int> stack{0};
    while (!stack.empty()) {
        const int i = stack.back();
        stack.pop_back();
        for (int c = 0; c < 2; ++c) {
            const int ref = nodes[i].d[c], cnt = nodes[i].d[2 + c];
            if (cnt < 0 || !slab(box(i, c), r, best)) continue;
            if (cnt == 0) {
                stack.push_back(ref);
                continue;
            }
            for (int k = 0; k < cnt; ++k) {
                const TriRec& t = tris[ref + k];
                const float v[9] = {t.v0[0], t.v0[1], t.v0[2], t.v1[0], t.v1[1], t.v1[2], t.v2[0], t.v2[1], t.v2[2]};
                double tt;
                if (hit_tri(v, r, tt) && (tt < best || (tt == best && t.id < best_id))) {
                    best = tt;
                    best_id = t.id;
                }
            }
        }
    }
    return best_id;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 4) {
        std::fprintf(stderr, "usage: bvh_check scene.f32 n_tris n_rays\n");
        return 2;
    }
    const long n = std::atol(argv[2]);
    const int n_rays = std::atoi(argv[3]);
    std::vector<float> tv(9 * (size_t)n);
    FILE* f = std::fopen(argv[1], "rb");
    if (!f || std::fread(tv.data(), 4, tv.size(), f) != tv.size()) return 2;
    std::fclose(f);
    // ARX_SBVH=0: the object-split builder (the product never reads the environment; this
    // checker sets the process-wide build parameters itself)
    if (const char* e = std::getenv("ARX_SBVH")) build_params().spatial = std::atof(e) > 0.0;
    BvhBuild b;
    build_bvh(tv.data(), nullptr, 0.5f, n, 0, b);
    // renumbered as arx_set_scene does: the first k inner nodes in breadth-first order
    const size_t k_bfs = std::getenv("BFS_K") ? (size_t)std::atol(std::getenv("BFS_K")) : 1023;
    bfs_prefix_order(b, k_bfs);
    if (b.root.count == 0) {
        std::vector<int32_t> order{b.root.ref};
        for (size_t h = 0; h < order.size() && order.size() < k_bfs; ++h)
            for (int c = 0; c < 2 && order.size() < k_bfs; ++c)
                if (b.nodes[(size_t)order[h]].d[2 + c] == 0) order.push_back(b.nodes[(size_t)order[h]].d[c]);
        for (size_t i = 0; i < order.size(); ++i)
            if (order[i] != (int32_t)i) {
                std::printf("FAIL breadth-first prefix: position %zu holds node %d\n", i, order[i]);
                return 1;
            }
    }
    // the kernel's two-level layout: node 0 = top (scene root, empty receiver)
    relocate_bvh(b, 1, 0);
    std::vector<BvhNode> nodes{make_node(b.root, empty_child())};
    nodes.insert(nodes.end(), b.nodes.begin(), b.nodes.end());
    const char* why = "";
    if (!validate_bvh(nodes.data(), nodes.size(), b.tris.size(), &why)) {
        std::printf("FAIL structure: %s\n", why);
        return 1;
    }
    std::vector<char> seen((size_t)n, 0);
    for (const TriRec& t : b.tris) seen[(size_t)t.id] = 1;
    for (long i = 0; i < n; ++i)
        if (!seen[(size_t)i]) {
            std::printf("FAIL triangle %ld in no leaf\n", i);
            return 1;
        }
    std::vector<BvhNode> coded(nodes.size());
    code_nodes(nodes.data(), nodes.size(), coded.data());
    float lo[3], hi[3];
    for (int k = 0; k < 3; ++k) {
        lo[k] = b.root.lo[k];
        hi[k] = b.root.hi[k];
    }
    const QGrid g = make_qgrid(lo, hi);
    std::vector<QNode2> q(nodes.size());
    if (!quantize_nodes16(coded.data(), coded.size(), g, q.data())) {
        std::printf("FAIL quantization\n");
        return 1;
    }
    for (size_t i = 0; i < nodes.size(); ++i)
        for (int c = 0; c < 2; ++c) {
            if (nodes[i].d[2 + c] < 0) continue;
            const Box fb = child_box(nodes[i], c), qb = qbox(q[i], c, g);
            for (int k = 0; k < 3; ++k)
                if (!(qb.lo[k] <= fb.lo[k] && qb.hi[k] >= fb.hi[k])) {
                    std::printf("FAIL quantized box %zu/%d axis %d\n", i, c, k);
                    return 1;
                }
            if (q[i].c[c].code != coded[i].d[c]) {
                std::printf("FAIL quantized code %zu/%d\n", i, c);
                return 1;
            }
        }
    std::mt19937 rng(12345);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    int hits = 0;
    for (int i = 0; i < n_rays; ++i) {
        Ray r;
        for (int k = 0; k < 3; ++k) r.o[k] = lo[k] + (hi[k] - lo[k]) * U(rng);
        const double z = 2 * U(rng) - 1, ph = 6.283185307179586 * U(rng), s = std::sqrt(1 - z * z);
        r.d[0] = s * std::cos(ph);
        r.d[1] = s * std::sin(ph);
        r.d[2] = z;
        double bt = 1e300;
        int bid = -1;
        for (long j = 0; j < n; ++j) {
            double tt;
            if (hit_tri(&tv[9 * (size_t)j], r, tt) && (tt < bt || (tt == bt && j < bid))) {
                bt = tt;
                bid = (int)j;
            }
        }
        double t1, t2;
        const int h1 = closest(nodes, b.tris, r, [&](int nd, int c) { return child_box(nodes[nd], c); }, t1);
        const int h2 = closest(nodes, b.tris, r, [&](int nd, int c) { return qbox(q[nd], c, g); }, t2);
        if (h1 != bid || h2 != bid || (bid >= 0 && (t1 != bt || t2 != bt))) {
            std::printf("FAIL ray %d: brute %d (%.9g) f32 tree %d quantized tree %d\n", i, bid, bt, h1, h2);
            return 1;
        }
        hits += bid >= 0;
    }
    std::printf("ok: %ld triangles, %zu references, %zu nodes, depth %d, %d/%d rays hit\n", n, b.tris.size(),
                nodes.size(), b.depth, hits, n_rays);
    return 0;
}
