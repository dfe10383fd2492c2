// tree_hash -- FNV-1a hash of the production SAH build (arx_bvh.cpp) of a triangle soup, built
// twice in one process (tests/test_bvh_host.py: the threaded builder must give one tree).
//   tree_hash scene.f32 n_tris
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "arx_bvh.hpp"

using namespace arx;

static unsigned long long tree_hash(const BvhBuild& b) {
    unsigned long long h = 1469598103934665603ull;
    auto mix = [&](const void* p, size_t len) {
        const unsigned char* c = static_cast<const unsigned char*>(p);
        for (size_t i = 0; i < len; ++i) {
            h ^= c[i];
            h *= 1099511628211ull;
        }
    };
    mix(b.nodes.data(), b.nodes.size() * sizeof(BvhNode));
    mix(b.tris.data(), b.tris.size() * sizeof(TriRec));
    mix(&b.root, sizeof(b.root));
    return h;
}

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    const long n = std::atol(argv[2]);
    std::vector<float> tv((size_t)n * 9);
    FILE* f = std::fopen(argv[1], "rb");
    if (!f || std::fread(tv.data(), 4, tv.size(), f) != tv.size()) return 2;
    std::fclose(f);
    std::vector<float> ab((size_t)n, 0.5f);
    unsigned long long h[2];
    size_t nodes = 0;
    for (int k = 0; k < 2; ++k) {
        BvhBuild b;
        build_bvh(tv.data(), ab.data(), 0.5f, n, 0, b);
        h[k] = tree_hash(b);
        nodes = b.nodes.size();
    }
    std::printf("%016llx %016llx %zu\n", h[0], h[1], nodes);
    return 0;
}
