// arx_receiver.hip -- moving-listener update on the device, and the
// device re-quantization of the node tree (a new scene, or the grid grown for a listener that
// walked off it: no host work inside a frame).
//
// The reference re-places the receiver half-spheres on the host (place_receiver_half,
// OptixModel.cpp:159-257) and then rebuilds the whole GAS, pipeline and SBT (reload,
// AudioRenderer.cpp:466-486) for every listener move.  Here the receiver sub-tree is built ONCE in
// the receiver's local frame (arx_capi.cpp, when the receiver model or the scene changes); a move
// is one kernel launch on the renderer's stream, with no host work beyond its arguments:
//   1. every receiver triangle is transformed to world space with place_receiver_half's exact
//      operation order (the vertex transform of OptixModel.cpp:178-193, glm::rotate about +Y by
//      -yaw, then + listener position) and written to its TriRec slot;
//   2. the sub-tree's boxes are refit bottom-up, level by level (fixed topology), padded, and
//      written as the coded f32 node (the fallback format) and the 16-bit quantized node;
//   3. the top node's receiver child is rewritten from the refit root box.
// The closest hit does not depend on the tree (any conservative tree gives the same hit and
// tie-break), so the result stays bit-exact with the oracle, which builds its own tree.
#include <hip/hip_runtime.h>

#include "arx_kernels.hpp"
#include "arx_layout.hpp"
#include "arx_wide.hpp"

namespace arx {
namespace {

constexpr int kRefitThreads = 256;

__device__ __forceinline__ int32_t child_code(int32_t ref, int32_t count) {
    return count < 0 ? kEmptyChildCode : count == 0 ? ref : ~(ref * 16 + count);  // code_nodes (arx_bvh.cpp)
}

// Outward 16-bit grid index of a plane with the kQ16Margin margin: quantize_nodes16's arithmetic
// (arx_bvh.cpp) bit for bit (IEEE f64 division), like the device re-quantization below.
__device__ __forceinline__ bool quantize_axis(const QGrid& g, const double* /*inv*/, int k, float lo, float hi,
                                              uint32_t& word) {
    const double l = floor(((double)lo - (double)g.origin[k]) / (double)g.scale[k] - kQ16Margin);
    const double h = ceil(((double)hi - (double)g.origin[k]) / (double)g.scale[k] + kQ16Margin);
    if (!(l >= 0.0) || !(h <= 65535.0)) return false;
    word = (uint32_t)l | ((uint32_t)h << 16);
    return true;
}

// Box (lo, hi) of child c, unpadded, into the node's coded f32 form (padded) and its quantized half.
__device__ void write_child(const RefitArgs& a, const double* inv, int32_t node, int c, const float* lo,
                            const float* hi, int32_t code, bool empty) {
    BvhNode* n = a.cnodes + node;
    float* ab = c == 0 ? n->a : n->b;
    if (empty) {  // the inverted box of empty_child(): never passes the slab test
        ab[0] = 1e30f; ab[1] = -1e30f; ab[2] = 1e30f; ab[3] = -1e30f;
        n->c[2 * c] = 1e30f;
        n->c[2 * c + 1] = -1e30f;
    } else {
        ab[0] = lo[0] - a.pad; ab[1] = hi[0] + a.pad; ab[2] = lo[1] - a.pad; ab[3] = hi[1] + a.pad;
        n->c[2 * c] = lo[2] - a.pad;
        n->c[2 * c + 1] = hi[2] + a.pad;
    }
    n->d[c] = code;
    if (!a.qnodes) return;
    QChild& q = a.qnodes[node].c[c];
    for (int k = 0; k < 3; ++k) {
        uint32_t w = 1u;  // empty: the slab between planes 0 and 1 (quantize_nodes16)
        if (!empty && !quantize_axis(a.grid, inv, k, lo[k] - a.pad, hi[k] + a.pad, w)) {
            atomicMax(a.flag, a.flag_value);  // off the grid: the host's bound should have prevented it
            w = 0u | (65535u << 16);
        }
        q.q[k] = w;
    }
    q.code = code;
}

constexpr int kRefitBatch = 4;  // global loads each thread keeps in flight

__device__ __forceinline__ size_t refit_nd_offset(int32_t n_tris, int32_t n_nodes) {  // in floats, 16-B aligned
    return ((size_t)9 * n_tris + (size_t)6 * n_nodes + 3) & ~(size_t)3;
}

__global__ __launch_bounds__(kRefitThreads) void receiver_refit_kernel(RefitArgs a) {
    extern __shared__ float lds[];
    float* wv = lds;                   // world vertices, 9 per receiver triangle
    float* nb = lds + 9 * a.n_tris;    // node boxes (lo xyz, hi xyz), unpadded
    int4* nd = reinterpret_cast<int4*>(lds + refit_nd_offset(a.n_tris, a.n_nodes));  // child (ref, count) pairs
    const double inv[3] = {1.0 / (double)a.grid.scale[0], 1.0 / (double)a.grid.scale[1], 1.0 / (double)a.grid.scale[2]};
    int32_t* lnodes = reinterpret_cast<int32_t*>(nd + a.n_nodes);                     // the level schedule
    int32_t* lstart = lnodes + a.n_nodes;
    // 0. the nodes' child records and the level schedule into LDS, so the level loop below makes no
    //    global round trips
    for (int i = threadIdx.x; i <= a.n_levels; i += kRefitThreads) lstart[i] = a.level_start[i];
    for (int i0 = threadIdx.x; i0 < a.n_nodes; i0 += kRefitBatch * kRefitThreads) {
        int32_t l[kRefitBatch];
#pragma unroll
        for (int k = 0; k < kRefitBatch; ++k) {
            const int i = i0 + k * kRefitThreads;
            l[k] = i < a.n_nodes ? a.level_nodes[i] : 0;
        }
#pragma unroll
        for (int k = 0; k < kRefitBatch; ++k) {
            const int i = i0 + k * kRefitThreads;
            if (i < a.n_nodes) lnodes[i] = l[k];
        }
    }
    for (int i0 = threadIdx.x; i0 < a.n_nodes; i0 += kRefitBatch * kRefitThreads) {
        int4 v[kRefitBatch];
#pragma unroll
        for (int k = 0; k < kRefitBatch; ++k) {
            const int i = i0 + k * kRefitThreads;
            v[k] = i < a.n_nodes ? *reinterpret_cast<const int4*>(a.local_nodes[i].d) : make_int4(0, 0, 0, 0);
        }
#pragma unroll
        for (int k = 0; k < kRefitBatch; ++k) {
            const int i = i0 + k * kRefitThreads;
            if (i < a.n_nodes) nd[i] = v[k];
        }
    }
    // 1. transform (OptixModel.cpp:178-193 with glm's operation order, as arx_place_receiver_vertices)
    for (int i0 = threadIdx.x; i0 < a.n_tris; i0 += kRefitBatch * kRefitThreads) {
      TriRec pre[kRefitBatch];
#pragma unroll
      for (int k = 0; k < kRefitBatch; ++k) {
          const int i = i0 + k * kRefitThreads;
          if (i < a.n_tris) pre[k] = a.local_tris[i];
      }
#pragma unroll
      for (int k = 0; k < kRefitBatch; ++k) {
        const int i = i0 + k * kRefitThreads;
        if (i >= a.n_tris) break;
        const TriRec src = pre[k];
        TriRec dst = src;
        const float* v[3] = {src.v0, src.v1, src.v2};
        float* o[3] = {dst.v0, dst.v1, dst.v2};
        for (int j = 0; j < 3; ++j) {
            const float vx = v[j][0], vy = v[j][1], vz = v[j][2];
            const float ox = (a.m[0] * vx + a.m[1] * vy) + (a.m[2] * vz + 0.0f);
            const float oy = (a.m[3] * vx + a.m[4] * vy) + (a.m[5] * vz + 0.0f);
            const float oz = (a.m[6] * vx + a.m[7] * vy) + (a.m[8] * vz + 0.0f);
            o[j][0] = a.t[0] + ox;
            o[j][1] = a.t[1] + oy;
            o[j][2] = a.t[2] + oz;
            wv[9 * i + 3 * j + 0] = o[j][0];
            wv[9 * i + 3 * j + 1] = o[j][1];
            wv[9 * i + 3 * j + 2] = o[j][2];
        }
        a.tris[a.tri_base + i] = dst;
      }
    }
    __syncthreads();
    // box of a child reference (global refs): a leaf's triangles or an already refit node
    auto child_box = [&](int32_t ref, int32_t count, float* lo, float* hi) {
        for (int k = 0; k < 3; ++k) {
            lo[k] = __builtin_huge_valf();
            hi[k] = -__builtin_huge_valf();
        }
        if (count > 0) {
            for (int32_t t = ref - a.tri_base; t < ref - a.tri_base + count; ++t)
                for (int j = 0; j < 3; ++j)
                    for (int k = 0; k < 3; ++k) {
                        lo[k] = fminf(lo[k], wv[9 * t + 3 * j + k]);
                        hi[k] = fmaxf(hi[k], wv[9 * t + 3 * j + k]);
                    }
        } else if (count == 0) {
            const float* b = nb + 6 * (ref - a.node_base);
            for (int k = 0; k < 3; ++k) {
                lo[k] = b[k];
                hi[k] = b[3 + k];
            }
        }
    };
    // 2. bottom-up refit, deepest level first (fixed topology)
    for (int L = 0; L < a.n_levels; ++L) {
        for (int i = lstart[L] + threadIdx.x; i < lstart[L + 1]; i += kRefitThreads) {
            const int32_t ln = lnodes[i];
            const int4 d4 = nd[ln];
            const int32_t sd[4] = {d4.x, d4.y, d4.z, d4.w};
            float blo[3] = {__builtin_huge_valf(), __builtin_huge_valf(), __builtin_huge_valf()};
            float bhi[3] = {-__builtin_huge_valf(), -__builtin_huge_valf(), -__builtin_huge_valf()};
            for (int c = 0; c < 2; ++c) {
                const int32_t ref = sd[c], count = sd[2 + c];
                float lo[3], hi[3];
                child_box(ref, count, lo, hi);
                write_child(a, inv, a.node_base + ln, c, lo, hi, child_code(ref, count), count < 0);
                for (int k = 0; k < 3; ++k) {
                    blo[k] = fminf(blo[k], lo[k]);
                    bhi[k] = fmaxf(bhi[k], hi[k]);
                }
            }
            for (int k = 0; k < 3; ++k) {
                nb[6 * ln + k] = blo[k];
                nb[6 * ln + 3 + k] = bhi[k];
            }
        }
        __syncthreads();
    }
    // 3. the top node's receiver child (child 1) from the root
    if (threadIdx.x == 0) {
        float lo[3], hi[3];
        child_box(a.root_ref, a.root_count, lo, hi);
        write_child(a, inv, 0, 1, lo, hi, child_code(a.root_ref, a.root_count), a.root_count < 0);
    }
    if (!a.wbuf) return;
    // 4. the CW4 copy: every receiver CW4 node from the refit boxes of its BVH2 children (padded as
    //    the coded nodes), its leaf triangles, and the top node
    for (int i = threadIdx.x; i < a.n_w4; i += kRefitThreads) {
        const int32_t* sd = a.w4_nodes + 11 * i;
        W4NodeF n;
        n.meta = (uint32_t)sd[8];
        n.base = (uint32_t)sd[9];
        n.self = (uint32_t)sd[10];
        n.pad = 0u;
        for (int c = 0; c < 4; ++c) {
            float lo[3], hi[3];
            child_box(sd[2 * c], sd[2 * c + 1], lo, hi);
            for (int k = 0; k < 3; ++k) {
                n.lo[c][k] = lo[k] - a.pad;
                n.hi[c][k] = hi[k] + a.pad;
            }
        }
        QNode4C q;
        if (!quantize_w4(n, a.grid, q)) atomicMax(a.flag, a.flag_value);
        a.wbuf[n.self] = make_uint4(q.w[0], q.w[1], q.w[2], q.w[3]);
        a.wbuf[n.self + 1] = make_uint4(q.w[4], q.w[5], q.w[6], q.w[7]);
    }
    for (int i = threadIdx.x; i < a.n_w4_tris; i += kRefitThreads) {
        const uint32_t unit = (uint32_t)a.w4_tris[2 * i];
        const int32_t t = a.w4_tris[2 * i + 1];
        const TriRec src = a.local_tris[t];
        const float* v = wv + 9 * t;
        a.wbuf[unit] = make_uint4(__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]),
                                  __float_as_uint(src.absorption));
        a.wbuf[unit + 1] = make_uint4(__float_as_uint(v[3]), __float_as_uint(v[4]), __float_as_uint(v[5]), (uint32_t)src.id);
        a.wbuf[unit + 2] = make_uint4(__float_as_uint(v[6]), __float_as_uint(v[7]), __float_as_uint(v[8]), (uint32_t)src.pad);
    }
    if (threadIdx.x == 0) {
        W4NodeF n;
        n.meta = (a.scene_nonempty ? 1u : 0u) | (a.root_count >= 0 ? 1u << 2 : 0u);
        n.base = 2u;
        n.self = 0u;
        n.pad = 0u;
        float lo[3], hi[3];
        child_box(a.root_ref, a.root_count, lo, hi);
        for (int k = 0; k < 3; ++k) {
            n.lo[0][k] = a.scene_lo[k];
            n.hi[0][k] = a.scene_hi[k];
            n.lo[1][k] = lo[k] - a.pad;
            n.hi[1][k] = hi[k] + a.pad;
            n.lo[2][k] = n.lo[3][k] = 0.0f;
            n.hi[2][k] = n.hi[3][k] = 0.0f;
        }
        QNode4C q;
        if (!quantize_w4(n, a.grid, q)) atomicMax(a.flag, a.flag_value);
        a.wbuf[0] = make_uint4(q.w[0], q.w[1], q.w[2], q.w[3]);
        a.wbuf[1] = make_uint4(q.w[4], q.w[5], q.w[6], q.w[7]);
    }
}

__global__ __launch_bounds__(256) void requant_w4_kernel(const W4NodeF* __restrict__ nodes, uint64_t n, QGrid g,
                                                          uint4* __restrict__ wbuf, unsigned int* flag,
                                                          unsigned int flag_value) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const W4NodeF nd = nodes[i];
    QNode4C q;
    if (!quantize_w4(nd, g, q)) atomicMax(flag, flag_value);
    wbuf[nd.self] = make_uint4(q.w[0], q.w[1], q.w[2], q.w[3]);
    wbuf[nd.self + 1] = make_uint4(q.w[4], q.w[5], q.w[6], q.w[7]);
}

// One quantized child: quantize_nodes16 (arx_bvh.cpp) on the device.  The f64 division is IEEE
// correctly rounded on gfx950 as on the host, so q is the host's q bit for bit.
__device__ __forceinline__ bool requant_child(const QGrid& g, const float* xy, const float* z, int32_t code,
                                              QChild& out) {
    const float lo[3] = {xy[0], xy[2], z[0]};
    const float hi[3] = {xy[1], xy[3], z[1]};
    const bool empty = code == kEmptyChildCode;
    bool ok = true;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        uint32_t ql = 1u, qh = 0u;  // empty: the slab between planes 0 and 1 (grid corner)
        if (!empty) {
            const double l = floor(((double)lo[k] - (double)g.origin[k]) / (double)g.scale[k] - kQ16Margin);
            const double h = ceil(((double)hi[k] - (double)g.origin[k]) / (double)g.scale[k] + kQ16Margin);
            if (!(lo[k] <= hi[k]) || !(l >= 0.0) || !(h <= 65535.0)) {
                ok = false;
                ql = 0u;
                qh = 65535u;  // the whole axis: still conservative
            } else {
                ql = (uint32_t)l;
                qh = (uint32_t)h;
            }
        }
        out.q[k] = ql | (qh << 16);
    }
    out.code = code;
    return ok;
}

__global__ __launch_bounds__(256) void requant16_kernel(const BvhNode* __restrict__ coded, uint64_t n, QGrid g,
                                                         QNode2* __restrict__ out, unsigned int* flag,
                                                         unsigned int flag_value) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const BvhNode b = coded[i];
    QNode2 q;
    const bool ok0 = requant_child(g, b.a, b.c, b.d[0], q.c[0]);
    const bool ok1 = requant_child(g, b.b, b.c + 2, b.d[1], q.c[1]);
    out[i] = q;
    if (!(ok0 && ok1)) atomicMax(flag, flag_value);
}

}  // namespace

hipError_t launch_requant_w4(const W4NodeF* nodes, uint64_t n, const QGrid& g, uint4* wbuf, unsigned int* flag,
                             unsigned int flag_value, hipStream_t s) {
    (void)hipGetLastError();
    if (n == 0) return hipSuccess;
    if (!nodes || !wbuf || !flag) return hipErrorInvalidValue;
    hipLaunchKernelGGL(requant_w4_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, nodes, n, g, wbuf, flag,
                       flag_value);
    return hipGetLastError();
}

hipError_t launch_requant16(const BvhNode* coded, uint64_t n, const QGrid& g, QNode2* out, unsigned int* flag,
                            unsigned int flag_value, hipStream_t s) {
    (void)hipGetLastError();
    if (n == 0) return hipSuccess;
    if (!coded || !out || !flag) return hipErrorInvalidValue;
    hipLaunchKernelGGL(requant16_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, coded, n, g, out, flag,
                       flag_value);
    return hipGetLastError();
}

size_t receiver_refit_lds(int32_t n_tris, int32_t n_nodes, int32_t n_levels) {
    return ((((size_t)9 * n_tris + (size_t)6 * n_nodes + 3) & ~(size_t)3) + (size_t)5 * n_nodes + (size_t)n_levels + 1) *
           4;
}

hipError_t launch_receiver_refit(const RefitArgs& a, hipStream_t s) {
    (void)hipGetLastError();
    hipLaunchKernelGGL(receiver_refit_kernel, dim3(1), dim3(kRefitThreads), receiver_refit_lds(a.n_tris, a.n_nodes, a.n_levels),
                       s,
                       a);
    return hipGetLastError();
}

}  // namespace arx
