// arx_trace.hip -- fused acoustic ray-trace kernel for gfx950 (MI355X).
//
// One lane owns one ray for its whole life (raygen -> bounce loop -> histogram),
// replacing the OptiX pipeline of R/prebuild/obj_raytracer/devicePrograms.cu:
//   __raygen__renderFrame   :192-254  -> trace_ray() prologue + bounce loop
//   optixTrace / RT cores   :240-251  -> closest_hit(): software BVH2 traversal,
//                                        per-lane LDS stack, watertight triangle test
//   __closesthit__radiance  :62-180   -> trace_ray() hit block
//   __miss__radiance        :186-190  -> trace_ray() miss branch
// Work distribution: grid-stride over global ray ids.  The IR histogram is int64 fixed
// point (unit e0*2^-frac_bits) accumulated with 64-bit atomics: order-independent,
// bitwise reproducible and exactly summable across GPUs.
//
// Arithmetic is IEEE f32 with no contraction (built -ffp-contract=off) so that every
// ray follows bit-for-bit the path computed by the CPU oracle (oracle/arx_oracle.c).
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "arx_kernels.hpp"
#include "arx_layout.hpp"

namespace arx {
namespace {

constexpr int kBlock = 128;

// ------------------------------------------------------------------- RNG ---
__device__ __forceinline__ void philox4x32_10(uint32_t& c0, uint32_t& c1, uint32_t& c2, uint32_t& c3, uint32_t k0,
                                              uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r > 0) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        const uint32_t hi0 = __umulhi(0xD2511F53u, c0);
        const uint32_t lo0 = 0xD2511F53u * c0;
        const uint32_t hi1 = __umulhi(0xCD9E8D57u, c2);
        const uint32_t lo1 = 0xCD9E8D57u * c2;
        const uint32_t n0 = hi1 ^ c1 ^ k0;
        const uint32_t n2 = hi0 ^ c3 ^ k1;
        c0 = n0;
        c1 = lo1;
        c2 = n2;
        c3 = lo0;
    }
}

__device__ __forceinline__ float u01(uint32_t x) { return (float)((x >> 8) + 1u) * (1.0f / 16777216.0f); }

// cos/sin(2*pi*u), u in (0,1]: exact quadrant reduction in turns + fma Horner (same
// coefficients and order as the oracle, so the result is bitwise identical).
__device__ __forceinline__ void sincos_turns(double u, double& s_out, double& c_out) {
    const double a = 4.0 * u;
    const double q = floor(a);
    const double f = a - q;
    const int iq = ((int)q) & 3;
    const double r = f * 1.5707963267948966;
    const double r2 = r * r;
    double ps = -1.0 / 121645100408832000.0;
    ps = __fma_rn(ps, r2, 1.0 / 355687428096000.0);
    ps = __fma_rn(ps, r2, -1.0 / 1307674368000.0);
    ps = __fma_rn(ps, r2, 1.0 / 6227020800.0);
    ps = __fma_rn(ps, r2, -1.0 / 39916800.0);
    ps = __fma_rn(ps, r2, 1.0 / 362880.0);
    ps = __fma_rn(ps, r2, -1.0 / 5040.0);
    ps = __fma_rn(ps, r2, 1.0 / 120.0);
    ps = __fma_rn(ps, r2, -1.0 / 6.0);
    const double sr = __fma_rn(r * r2, ps, r);
    double pc = 1.0 / 2432902008176640000.0;
    pc = __fma_rn(pc, r2, -1.0 / 6402373705728000.0);
    pc = __fma_rn(pc, r2, 1.0 / 20922789888000.0);
    pc = __fma_rn(pc, r2, -1.0 / 87178291200.0);
    pc = __fma_rn(pc, r2, 1.0 / 479001600.0);
    pc = __fma_rn(pc, r2, -1.0 / 3628800.0);
    pc = __fma_rn(pc, r2, 1.0 / 40320.0);
    pc = __fma_rn(pc, r2, -1.0 / 720.0);
    pc = __fma_rn(pc, r2, 1.0 / 24.0);
    pc = __fma_rn(pc, r2, -1.0 / 2.0);
    const double cr = __fma_rn(r2, pc, 1.0);
    double c, s;
    if (iq == 0) {
        c = cr;
        s = sr;
    } else if (iq == 1) {
        c = -sr;
        s = cr;
    } else if (iq == 2) {
        c = -cr;
        s = -sr;
    } else {
        c = sr;
        s = -cr;
    }
    s_out = s;
    c_out = c;
}

// devicePrograms.cu:216-224 with Philox(seed, ray id) instead of curand(clock64(), tid).
__device__ __forceinline__ float3 ray_direction(uint64_t seed, uint64_t rid) {
    uint32_t c0 = (uint32_t)rid, c1 = (uint32_t)(rid >> 32), c2 = 0u, c3 = 0u;
    philox4x32_10(c0, c1, c2, c3, (uint32_t)seed, (uint32_t)(seed >> 32));
    const float u1 = u01(c0);
    const float u2 = u01(c1);
    const double cz = 2.0 * (double)u2 - 1.0;
    const double sz = __dsqrt_rn(1.0 - cz * cz);
    double st, ct;
    sincos_turns((double)u1, st, ct);
    return make_float3((float)(sz * ct), (float)(sz * st), (float)cz);
}

// ------------------------------------------------------------ geometry ---
struct Ray {
    float o[3];      // origin
    float op[3];     // origin permuted (kx, ky, kz)
    float inv[3];    // safe reciprocal direction (box test only)
    float sx, sy, sz;
    int kx, ky, kz;
};

__device__ __forceinline__ float sel3(float x, float y, float z, int k) { return k == 0 ? x : (k == 1 ? y : z); }

__device__ __forceinline__ void setup_ray(Ray& r, float3 o, float3 d) {
    r.o[0] = o.x;
    r.o[1] = o.y;
    r.o[2] = o.z;
    const float ax = fabsf(d.x), ay = fabsf(d.y), az = fabsf(d.z);
    const int kz = (ax > ay) ? ((ax > az) ? 0 : 2) : ((ay > az) ? 1 : 2);
    int kx = kz + 1;
    if (kx == 3) kx = 0;
    int ky = kx + 1;
    if (ky == 3) ky = 0;
    const float dkz = sel3(d.x, d.y, d.z, kz);
    if (dkz < 0.0f) {
        const int t = kx;
        kx = ky;
        ky = t;
    }
    r.kx = kx;
    r.ky = ky;
    r.kz = kz;
    r.sx = sel3(d.x, d.y, d.z, kx) / dkz;
    r.sy = sel3(d.x, d.y, d.z, ky) / dkz;
    r.sz = 1.0f / dkz;
    r.op[0] = sel3(o.x, o.y, o.z, kx);
    r.op[1] = sel3(o.x, o.y, o.z, ky);
    r.op[2] = sel3(o.x, o.y, o.z, kz);
    // Box-test reciprocals: v_rcp_f32 (1 ulp) instead of a correctly rounded division -- the
    // slab test only has to be conservative, and a 1e-7 relative error in t is far inside the
    // 1e-5 * max|coordinate| box padding; the closest hit comes from the exact triangle test.
    const float dd[3] = {d.x, d.y, d.z};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        float v = dd[k];
        if (fabsf(v) < 1e-20f) v = (v < 0.0f) ? -1e-20f : 1e-20f;
        r.inv[k] = __builtin_amdgcn_rcpf(v);
    }
}

// Watertight ray/triangle test (Woop, Benthin, Wald 2013); t >= 0 (optixTrace tmin 0).
// Vertex components are selected by (kx,ky,kz) then differenced against the permuted
// origin: the same values as A[k] = v[k] - o[k] indexed afterwards (oracle order).
struct Hit {
    float U, V, W, det, t;
};

__device__ __forceinline__ bool tri_test(const Ray& r, float4 p0, float4 p1, float4 p2, Hit& h) {
    const float Ax = sel3(p0.x, p0.y, p0.z, r.kx) - r.op[0];
    const float Ay = sel3(p0.x, p0.y, p0.z, r.ky) - r.op[1];
    const float Az = sel3(p0.x, p0.y, p0.z, r.kz) - r.op[2];
    const float Bx = sel3(p1.x, p1.y, p1.z, r.kx) - r.op[0];
    const float By = sel3(p1.x, p1.y, p1.z, r.ky) - r.op[1];
    const float Bz = sel3(p1.x, p1.y, p1.z, r.kz) - r.op[2];
    const float Cx = sel3(p2.x, p2.y, p2.z, r.kx) - r.op[0];
    const float Cy = sel3(p2.x, p2.y, p2.z, r.ky) - r.op[1];
    const float Cz = sel3(p2.x, p2.y, p2.z, r.kz) - r.op[2];
    const float ax = Ax - r.sx * Az;
    const float ay = Ay - r.sy * Az;
    const float bx = Bx - r.sx * Bz;
    const float by = By - r.sy * Bz;
    const float cx = Cx - r.sx * Cz;
    const float cy = Cy - r.sy * Cz;
    const float U = cx * by - cy * bx;
    const float V = ax * cy - ay * cx;
    const float W = bx * ay - by * ax;
    if ((U < 0.0f || V < 0.0f || W < 0.0f) && (U > 0.0f || V > 0.0f || W > 0.0f)) return false;
    const float det = U + V + W;
    if (det == 0.0f) return false;
    const float az = r.sz * Az;
    const float bz = r.sz * Bz;
    const float cz = r.sz * Cz;
    const float T = U * az + V * bz + W * cz;
    const float t = T / det;
    if (!(t >= 0.0f)) return false;
    h.U = U;
    h.V = V;
    h.W = W;
    h.det = det;
    h.t = t;
    return true;
}

__device__ __forceinline__ void leaf_hits(const TriRec* __restrict__ tris, const Ray& r, int first, int count,
                                          float& best_t, int& best_id, int& best) {
    for (int k = 0; k < count; ++k) {
        const float4* tp = reinterpret_cast<const float4*>(tris + first + k);
        const float4 p0 = tp[0], p1 = tp[1], p2 = tp[2];
        Hit h;
        if (tri_test(r, p0, p1, p2, h)) {
            const int id = __float_as_int(p1.w);
            if (h.t < best_t || (h.t == best_t && id < best_id)) {
                best_t = h.t;
                best_id = id;
                best = first + k;
            }
        }
    }
}

// Leaf test with the loads of V triangles in flight together.  Slots past the leaf's end are
// clamped to its last triangle: re-testing a triangle cannot change the (t, id) minimum.
template <int V>
__device__ __forceinline__ void leaf_hits_vec(const TriRec* __restrict__ tris, const Ray& r, int first, int count,
                                              float& best_t, int& best_id, int& best) {
    if constexpr (V == 1) {
        leaf_hits(tris, r, first, count, best_t, best_id, best);
    } else {
        for (int k = 0; k < count; k += V) {
            float4 p[V][3];
            int idx[V];
#pragma unroll
            for (int j = 0; j < V; ++j) {
                idx[j] = first + min(k + j, count - 1);
                const float4* tp = reinterpret_cast<const float4*>(tris + idx[j]);
                p[j][0] = tp[0];
                p[j][1] = tp[1];
                p[j][2] = tp[2];
            }
#pragma unroll
            for (int j = 0; j < V; ++j) {
                Hit h;
                if (tri_test(r, p[j][0], p[j][1], p[j][2], h)) {
                    const int id = __float_as_int(p[j][1].w);
                    if (h.t < best_t || (h.t == best_t && id < best_id)) {
                        best_t = h.t;
                        best_id = id;
                        best = idx[j];
                    }
                }
            }
        }
    }
}

// Branch-free watertight test: same arithmetic and result as tri_test, decided by selects.
__device__ __forceinline__ bool tri_test_nb(const Ray& r, float4 p0, float4 p1, float4 p2, float& t_out) {
    const float Ax = sel3(p0.x, p0.y, p0.z, r.kx) - r.op[0];
    const float Ay = sel3(p0.x, p0.y, p0.z, r.ky) - r.op[1];
    const float Az = sel3(p0.x, p0.y, p0.z, r.kz) - r.op[2];
    const float Bx = sel3(p1.x, p1.y, p1.z, r.kx) - r.op[0];
    const float By = sel3(p1.x, p1.y, p1.z, r.ky) - r.op[1];
    const float Bz = sel3(p1.x, p1.y, p1.z, r.kz) - r.op[2];
    const float Cx = sel3(p2.x, p2.y, p2.z, r.kx) - r.op[0];
    const float Cy = sel3(p2.x, p2.y, p2.z, r.ky) - r.op[1];
    const float Cz = sel3(p2.x, p2.y, p2.z, r.kz) - r.op[2];
    const float ax = Ax - r.sx * Az;
    const float ay = Ay - r.sy * Az;
    const float bx = Bx - r.sx * Bz;
    const float by = By - r.sy * Bz;
    const float cx = Cx - r.sx * Cz;
    const float cy = Cy - r.sy * Cz;
    const float U = cx * by - cy * bx;
    const float V = ax * cy - ay * cx;
    const float W = bx * ay - by * ax;
    const bool mixed = (U < 0.0f || V < 0.0f || W < 0.0f) && (U > 0.0f || V > 0.0f || W > 0.0f);
    const float det = U + V + W;
    const float az = r.sz * Az;
    const float bz = r.sz * Bz;
    const float cz = r.sz * Cz;
    const float T = U * az + V * bz + W * cz;
    const float t = T / det;
    t_out = t;
    return !mixed && det != 0.0f && t >= 0.0f;
}

// Leaf step without divergent control flow: the trip count is the wave's largest pending
// leaf (uniform), lanes with shorter or no leaves re-test a clamped slot (cannot change the
// (t, id) minimum) or a dummy triangle whose result is discarded.
template <int V>
__device__ __forceinline__ void leaf_hits_u(const TriRec* __restrict__ tris, const Ray& r, int first, int count,
                                            float& best_t, int& best_id, int& best) {
    for (int k = 0; __ballot(k < count) != 0ull; k += V) {
        float4 p[V][3];
        int idx[V];
#pragma unroll
        for (int j = 0; j < V; ++j) {
            idx[j] = count > 0 ? first + min(k + j, count - 1) : 0;
            const float4* tp = reinterpret_cast<const float4*>(tris + idx[j]);
            p[j][0] = tp[0];
            p[j][1] = tp[1];
            p[j][2] = tp[2];
        }
#pragma unroll
        for (int j = 0; j < V; ++j) {
            float th;
            const bool hit = tri_test_nb(r, p[j][0], p[j][1], p[j][2], th) && count > 0;
            const int id = __float_as_int(p[j][1].w);
            const bool better = hit && (th < best_t || (th == best_t && id < best_id));
            best_t = better ? th : best_t;
            best_id = better ? id : best_id;
            best = better ? idx[j] : best;
        }
    }
}

// Per-lane traversal state of one closest-hit query over the two-level BVH (node 0 = top).
struct Trav {
    float best_t;
    int best_id;
    int best;    // TriRec index of the closest hit so far, -1 = none
    int node;    // inner node to visit next
    int sp;      // LDS stack depth
    int visits;
};

__device__ __forceinline__ void trav_init(Trav& t) {
    t.best_t = __builtin_huge_valf();
    t.best_id = 0x7fffffff;
    t.best = -1;
    t.node = 0;
    t.sp = 0;
    t.visits = 0;
}

// One traversal step: visit t.node (test both children, intersect leaf children in place,
// descend near-first / pop).  Returns false when the query is finished.
template <int BLOCK, int STACK>
__device__ __forceinline__ bool trav_step(const TraceArgs& a, const Ray& r, Trav& t, int* __restrict__ stk, int lane,
                                          bool& overflow) {
    if (++t.visits > a.max_visits) {  // malformed tree guard: never spin forever
        overflow = true;
        return false;
    }
    const float4* np = reinterpret_cast<const float4*>(a.nodes + t.node);
    const float4 na = np[0];
    const float4 nb = np[1];
    const float4 nc = np[2];
    const int4 nd = *reinterpret_cast<const int4*>(np + 3);
    const float ox = r.o[0], oy = r.o[1], oz = r.o[2];
    const float ix = r.inv[0], iy = r.inv[1], iz = r.inv[2];
    // child 0
    const float x00 = (na.x - ox) * ix, x01 = (na.y - ox) * ix;
    const float y00 = (na.z - oy) * iy, y01 = (na.w - oy) * iy;
    const float z00 = (nc.x - oz) * iz, z01 = (nc.y - oz) * iz;
    const float tn0 = fmaxf(fmaxf(fminf(x00, x01), fminf(y00, y01)), fmaxf(fminf(z00, z01), 0.0f));
    const float tf0 = fminf(fminf(fmaxf(x00, x01), fmaxf(y00, y01)), fminf(fmaxf(z00, z01), t.best_t));
    // child 1
    const float x10 = (nb.x - ox) * ix, x11 = (nb.y - ox) * ix;
    const float y10 = (nb.z - oy) * iy, y11 = (nb.w - oy) * iy;
    const float z10 = (nc.z - oz) * iz, z11 = (nc.w - oz) * iz;
    const float tn1 = fmaxf(fmaxf(fminf(x10, x11), fminf(y10, y11)), fmaxf(fminf(z10, z11), 0.0f));
    const float tf1 = fminf(fminf(fmaxf(x10, x11), fmaxf(y10, y11)), fminf(fmaxf(z10, z11), t.best_t));
    bool h0 = tn0 <= tf0 && nd.z >= 0;  // count < 0: empty child
    bool h1 = tn1 <= tf1 && nd.w >= 0;
    if (h0 && nd.z > 0) {
        leaf_hits(a.tris, r, nd.x, nd.z, t.best_t, t.best_id, t.best);
        h0 = false;
    }
    if (h1 && nd.w > 0) {
        leaf_hits(a.tris, r, nd.y, nd.w, t.best_t, t.best_id, t.best);
        h1 = false;
    }
    if (h0 && h1) {
        const bool swap = tn1 < tn0;
        const int near_n = swap ? nd.y : nd.x;
        const int far_n = swap ? nd.x : nd.y;
        if (t.sp < STACK) {
            stk[t.sp * BLOCK + lane] = far_n;
            ++t.sp;
        } else {
            overflow = true;
        }
        t.node = near_n;
    } else if (h0) {
        t.node = nd.x;
    } else if (h1) {
        t.node = nd.y;
    } else {
        if (t.sp == 0) return false;
        --t.sp;
        t.node = stk[t.sp * BLOCK + lane];
    }
    return true;
}

// glm-style helpers (glm::dot is x*x + y*y + z*z left to right)
__device__ __forceinline__ float dot3(float3 a, float3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ float3 sub3(float3 a, float3 b) { return make_float3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ float3 add3(float3 a, float3 b) { return make_float3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ float3 scale3(float s, float3 a) { return make_float3(s * a.x, s * a.y, s * a.z); }

__device__ __forceinline__ void hist_add(unsigned long long* h, int k, float e, double inv_unit) {
    const long long q = __double2ll_rn((double)e * inv_unit);
    if (q != 0) atomicAdd(h + k, (unsigned long long)q);
}

// Per-lane ray state (PRD, PRD.h:5-14, minus the pointer plumbing).
struct RayState {
    float3 pos, dir;
    float e, dist;
    int depth;
};

// Loop guard of __raygen__renderFrame (devicePrograms.cu:233-236).
__device__ __forceinline__ bool wants_query(const TraceArgs& a, const RayState& s) {
    return s.dist < a.dist_limit && s.e > a.energy_thres && s.depth >= 0 && (uint32_t)s.depth < a.max_bounces;
}

__device__ __forceinline__ void ray_init(const TraceArgs& a, RayState& s, uint64_t rid) {
    if (a.dirs) {  // precomputed by dirs_kernel (same function, launcher pre-pass)
        const float4 d = reinterpret_cast<const float4*>(a.dirs)[rid - a.ray_begin];
        s.dir = make_float3(d.x, d.y, d.z);
    } else {
        s.dir = ray_direction(a.seed, rid);
    }
    s.pos = make_float3(a.emitter[0], a.emitter[1], a.emitter[2]);
    s.e = a.e0;
    s.dist = 0.0f;
    s.depth = 0;
    if (!(s.dir.x != 0.0f || s.dir.y != 0.0f || s.dir.z != 0.0f)) s.depth = -1;  // :230, no trace
}

// __closesthit__radiance (devicePrograms.cu:62-180) for TriRec `hit`, or __miss__radiance
// (:186-190) when hit < 0.  r is the ray the query was traced with.
__device__ __forceinline__ void shade(const TraceArgs& a, RayState& s, const Ray& r, int hit, uint32_t& n_rx,
                                      uint32_t& n_miss) {
    if (hit < 0) {
        ++n_miss;
        s.depth = -1;
        return;
    }
    const float4* tp = reinterpret_cast<const float4*>(a.tris + hit);
    const float4 p0 = tp[0], p1 = tp[1], p2 = tp[2];
    const float3 P1 = make_float3(p0.x, p0.y, p0.z);
    const float3 P2 = make_float3(p1.x, p1.y, p1.z);
    const float3 P3 = make_float3(p2.x, p2.y, p2.z);
    const float ab = p0.w;
    // Ng = normalize(cross(P2-P1, P3-P1))  (:75-77)
    const float3 U = sub3(P2, P1), V = sub3(P3, P1);
    const float3 cr = make_float3(U.y * V.z - V.y * U.z, U.z * V.x - V.z * U.x, U.x * V.y - V.x * U.y);
    const float3 Ng = scale3(1.0f / sqrtf(dot3(cr, cr)), cr);
    Hit h;
    tri_test(r, p0, p1, p2, h);
    const float bu = h.V / h.det;
    const float bv = h.W / h.det;
    const float w0 = (1.0f - bu) - bv;
    const float3 P = add3(add3(scale3(w0, P1), scale3(bu, P2)), scale3(bv, P3));  // :81
    const float3 seg = sub3(P, s.pos);
    s.dist += sqrtf(dot3(seg, seg));  // :83
    float e = s.e;
    if (ab < 0.0f) {  // receiver chord weighting, r = 1 (:91-122)
        const float3 center = make_float3(a.center[0], a.center[1], a.center[2]);
        const float3 nd = scale3(1.0f / sqrtf(dot3(s.dir, s.dir)), s.dir);
        const float3 oc = sub3(P, center);
        const float qa = dot3(nd, nd);
        const float qb = 2.0f * dot3(oc, nd);
        const float qc = dot3(oc, oc) - 1.0f;
        const float disc = qb * qb - (4.0f * qa) * qc;
        if (disc <= 0.0f) {
            e = 0.0f;
        } else {
            const float sq = sqrtf(disc);
            const float t1 = (-qb - sq) / (2.0f * qa);
            const float t2 = (-qb + sq) / (2.0f * qa);
            const float3 i1 = add3(P, scale3(t1, nd));
            const float3 i2 = add3(P, scale3(t2, nd));
            const float3 di = sub3(i1, i2);
            e = e * sqrtf(dot3(di, di));
        }
    }
    if (ab == -1.0f || ab == -2.0f) {  // receiver halves (:128-170)
        ++n_rx;
        const int k = (int)roundf((s.dist / (float)kSpeedOfSound) * (float)a.sample_rate);
        if (k < a.ir_len) {
            unsigned long long* hl = a.hist;
            unsigned long long* hr = a.hist + a.ir_len;
            unsigned long long* own = (ab == -1.0f) ? hl : hr;
            unsigned long long* other = (ab == -1.0f) ? hr : hl;
            hist_add(own, k, e, a.inv_unit);
            if (!a.is_mono) {
                const int kk = (k + a.delay < a.ir_len) ? k + a.delay : k;
                hist_add(other, kk, e * (1.0f - a.hrtf), a.inv_unit);
            }
        }
        s.depth = -1;
    } else {  // specular reflection + absorption (:173-175)
        const float s2 = 2.0f * dot3(s.dir, Ng);
        s.dir = sub3(s.dir, scale3(s2, Ng));
        e = e * (1.0f - ab);
        ++s.depth;
    }
    s.e = e;
    s.pos = add3(P, scale3(1e-3f, s.dir));  // :179
}

__device__ __forceinline__ void flush_counters(const TraceArgs& a, uint32_t n_q, uint32_t n_rx, uint32_t n_miss,
                                               bool overflow, int lane) {
    unsigned int vq = n_q, vr = n_rx, vm = n_miss, vo = overflow ? 1u : 0u;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        vq += __shfl_xor(vq, off, 64);
        vr += __shfl_xor(vr, off, 64);
        vm += __shfl_xor(vm, off, 64);
        vo |= __shfl_xor(vo, off, 64);
    }
    if ((lane & 63) == 0) {
        if (vq) atomicAdd(a.counters + 0, (unsigned long long)vq);
        if (vr) atomicAdd(a.counters + 1, (unsigned long long)vr);
        if (vm) atomicAdd(a.counters + 2, (unsigned long long)vm);
        if (vo) atomicOr(a.counters + 3, 1ull);
    }
}

// v1: grid-stride, one ray per lane start to finish; the wave waits for its slowest ray.
template <int BLOCK, int STACK>
__global__ __launch_bounds__(BLOCK) void trace_kernel_v1(TraceArgs a) {
    __shared__ int stk[STACK * BLOCK];
    const int lane = threadIdx.x;
    const uint64_t n = a.ray_end - a.ray_begin;
    uint32_t n_q = 0, n_rx = 0, n_miss = 0;
    bool overflow = false;
    for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + lane; i < n; i += (uint64_t)gridDim.x * BLOCK) {
        RayState s;
        ray_init(a, s, a.ray_begin + i);
        while (wants_query(a, s)) {
            ++n_q;
            Ray r;
            setup_ray(r, s.pos, s.dir);
            Trav t;
            trav_init(t);
            while (trav_step<BLOCK, STACK>(a, r, t, stk, lane, overflow)) {
            }
            shade(a, s, r, t.best, n_rx, n_miss);
        }
    }
    flush_counters(a, n_q, n_rx, n_miss, overflow, lane);
}

// v2: persistent waves over a global ray cursor.  Lanes whose query is finished wait
// (masked) until THRESH lanes of the wave are waiting, then the wave shades them, refills
// finished rays from the cursor (one atomic per wave) and starts their next queries, so a
// wave never idles behind its slowest ray.  Results are identical to v1: the histogram is
// order-independent and every ray follows the same arithmetic.
template <int BLOCK, int STACK, int THRESH>
__global__ __launch_bounds__(BLOCK) void trace_kernel_v2(TraceArgs a) {
    __shared__ int stk[STACK * BLOCK];
    const int lane = threadIdx.x;
    const uint64_t n = a.ray_end - a.ray_begin;
    unsigned long long* const cursor = a.counters + 4;
    uint32_t n_q = 0, n_rx = 0, n_miss = 0;
    bool overflow = false;
    bool active = false;    // lane holds a ray
    bool trav = false;      // lane is inside a closest-hit query
    bool exhausted = false; // wave-uniform: the cursor passed n
    RayState s;
    Ray r;
    Trav t;
    trav_init(t);
    s.depth = -1;
    while (true) {
        // (1) shade lanes whose query finished; a ray that will not query again retires
        if (active && !trav) {
            shade(a, s, r, t.best, n_rx, n_miss);
            if (!wants_query(a, s)) active = false;
        }
        // (2) refill retired lanes from the global cursor, one atomic per wave
        const unsigned long long need = __ballot(!active);
        if (need != 0ull && !exhausted) {
            const int cnt = __popcll(need);
            const int leader = __ffsll((unsigned long long)need) - 1;
            unsigned long long base = 0;
            if ((lane & 63) == leader) base = atomicAdd(cursor, (unsigned long long)cnt);
            const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)base, leader);
            const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(base >> 32), leader);
            base = ((unsigned long long)hi << 32) | lo;
            if (!active) {
                const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(need >> 32),
                                                                __builtin_amdgcn_mbcnt_lo((uint32_t)need, 0u));
                const uint64_t i = base + rank;
                if (i < n) {
                    ray_init(a, s, a.ray_begin + i);
                    active = wants_query(a, s);
                }
            }
            if (base + (unsigned long long)cnt >= n) exhausted = true;
        }
        // (3) start the next query of every active lane that is not traversing
        if (active && !trav) {
            ++n_q;
            setup_ray(r, s.pos, s.dir);
            trav_init(t);
            trav = true;
        }
        if (__ballot(active) == 0ull) {
            if (exhausted) break;
            continue;  // every fetched ray retired without a query: fetch again
        }
        // (4) traverse until THRESH lanes are waiting to be shaded (or all are)
        while (true) {
            const unsigned long long tmask = __ballot(trav);
            if (tmask == 0ull) break;
            if (__popcll(__ballot(active && !trav)) >= THRESH) break;
            if (trav) trav = trav_step<BLOCK, STACK>(a, r, t, stk, lane, overflow);
        }
    }
    flush_counters(a, n_q, n_rx, n_miss, overflow, lane);
}

// ---- v3: v2's persistent refill loop + postponed leaves ("while-while", Aila & Laine 2009).
// A lane that hits a leaf parks it (one pending slot; further leaves go on the stack as
// tagged entries) and idles until enough lanes of the wave hold a leaf; then the whole
// wave runs the triangle tests together.  Box tests use the fma form t = lo*inv - o*inv
// (only their conservativeness matters; boxes are padded), so node steps are cheaper.
// Stack entry: >= 0 inner node; < 0 leaf, -(first*16 + count) - 1 (count <= 15).
struct Trav3 {
    float best_t;
    int best_id;
    int best;
    int node;   // inner node to visit, -1 = pop next
    int sp;
    int pf, pc; // pending leaf (first, count); pc == 0: none
    int visits;
};

__device__ __forceinline__ int leaf_code(int first, int count) { return -(first * 16 + count) - 1; }

template <int BLOCK, int STACK>
__device__ __forceinline__ void push3(Trav3& t, int* __restrict__ stk, int lane, int v, bool& overflow) {
    if (t.sp < STACK) {
        stk[t.sp * BLOCK + lane] = v;
        ++t.sp;
    } else {
        overflow = true;
    }
}

typedef float f2v __attribute__((ext_vector_type(2)));

// One node step for a lane with no pending leaf and work left (node >= 0 or sp > 0).
// PK: the 12 slab FMAs as 6 v_pk_fma_f32 (same IEEE result per element).
template <int BLOCK, int STACK, bool PK = false>
__device__ __forceinline__ void node_step3(const TraceArgs& a, const Ray& r, float oix, float oiy, float oiz, Trav3& t,
                                           int* __restrict__ stk, int lane, bool& overflow) {
    if (t.node < 0) {  // pop
        --t.sp;
        const int e = stk[t.sp * BLOCK + lane];
        if (e >= 0) {
            t.node = e;
        } else {
            const int v = -e - 1;
            t.pf = v >> 4;
            t.pc = v & 15;
            return;
        }
    }
    const float4* np = reinterpret_cast<const float4*>(a.nodes + t.node);
    const float4 na = np[0];
    const float4 nb = np[1];
    const float4 nc = np[2];
    const int4 nd = *reinterpret_cast<const int4*>(np + 3);
    const float ix = r.inv[0], iy = r.inv[1], iz = r.inv[2];
    float x00, x01, y00, y01, z00, z01, x10, x11, y10, y11, z10, z11;
    if constexpr (PK) {
        const f2v ix2 = {ix, ix}, iy2 = {iy, iy}, iz2 = {iz, iz};
        const f2v ox2 = {-oix, -oix}, oy2 = {-oiy, -oiy}, oz2 = {-oiz, -oiz};
        const f2v X0 = __builtin_elementwise_fma((f2v){na.x, na.y}, ix2, ox2);
        const f2v Y0 = __builtin_elementwise_fma((f2v){na.z, na.w}, iy2, oy2);
        const f2v Z0 = __builtin_elementwise_fma((f2v){nc.x, nc.y}, iz2, oz2);
        const f2v X1 = __builtin_elementwise_fma((f2v){nb.x, nb.y}, ix2, ox2);
        const f2v Y1 = __builtin_elementwise_fma((f2v){nb.z, nb.w}, iy2, oy2);
        const f2v Z1 = __builtin_elementwise_fma((f2v){nc.z, nc.w}, iz2, oz2);
        x00 = X0.x; x01 = X0.y; y00 = Y0.x; y01 = Y0.y; z00 = Z0.x; z01 = Z0.y;
        x10 = X1.x; x11 = X1.y; y10 = Y1.x; y11 = Y1.y; z10 = Z1.x; z11 = Z1.y;
    } else {
        x00 = __builtin_fmaf(na.x, ix, -oix); x01 = __builtin_fmaf(na.y, ix, -oix);
        y00 = __builtin_fmaf(na.z, iy, -oiy); y01 = __builtin_fmaf(na.w, iy, -oiy);
        z00 = __builtin_fmaf(nc.x, iz, -oiz); z01 = __builtin_fmaf(nc.y, iz, -oiz);
        x10 = __builtin_fmaf(nb.x, ix, -oix); x11 = __builtin_fmaf(nb.y, ix, -oix);
        y10 = __builtin_fmaf(nb.z, iy, -oiy); y11 = __builtin_fmaf(nb.w, iy, -oiy);
        z10 = __builtin_fmaf(nc.z, iz, -oiz); z11 = __builtin_fmaf(nc.w, iz, -oiz);
    }
    const float tn0 = fmaxf(fmaxf(fminf(x00, x01), fminf(y00, y01)), fmaxf(fminf(z00, z01), 0.0f));
    const float tf0 = fminf(fminf(fmaxf(x00, x01), fmaxf(y00, y01)), fminf(fmaxf(z00, z01), t.best_t));
    const float tn1 = fmaxf(fmaxf(fminf(x10, x11), fminf(y10, y11)), fmaxf(fminf(z10, z11), 0.0f));
    const float tf1 = fminf(fminf(fmaxf(x10, x11), fmaxf(y10, y11)), fminf(fmaxf(z10, z11), t.best_t));
    const bool h0 = tn0 <= tf0 && nd.z >= 0;
    const bool h1 = tn1 <= tf1 && nd.w >= 0;
    const bool l0 = h0 && nd.z > 0, l1 = h1 && nd.w > 0;  // leaf children hit
    const bool i0 = h0 && nd.z == 0, i1 = h1 && nd.w == 0;  // inner children hit
    // leaves: nearer one parked, the other pushed
    if (l0 && l1) {
        const bool swap = tn1 < tn0;
        t.pf = swap ? nd.y : nd.x;
        t.pc = swap ? nd.w : nd.z;
        push3<BLOCK, STACK>(t, stk, lane, swap ? leaf_code(nd.x, nd.z) : leaf_code(nd.y, nd.w), overflow);
    } else if (l0) {
        t.pf = nd.x;
        t.pc = nd.z;
    } else if (l1) {
        t.pf = nd.y;
        t.pc = nd.w;
    }
    if (i0 && i1) {
        const bool swap = tn1 < tn0;
        push3<BLOCK, STACK>(t, stk, lane, swap ? nd.x : nd.y, overflow);
        t.node = swap ? nd.y : nd.x;
    } else if (i0) {
        t.node = nd.x;
    } else if (i1) {
        t.node = nd.y;
    } else {
        t.node = -1;
    }
}

// Traversal stack of S entries per lane in LDS; deeper entries spill to a per-lane global
// column (a.spill[(sp - S) * a.spill_lanes + gid], sized on the host for the tree).
template <int BLOCK, int S>
__device__ __forceinline__ void pushw(const TraceArgs& a, Trav3& t, int* __restrict__ stk, int lane, uint32_t gid, int v,
                                      bool& overflow) {
    if (t.sp < S) {
        stk[t.sp * BLOCK + lane] = v;
    } else if (t.sp - S < a.spill_depth) {
        a.spill[(uint64_t)(t.sp - S) * a.spill_lanes + gid] = v;
    } else {
        overflow = true;
        return;
    }
    ++t.sp;
}

template <int BLOCK, int S>
__device__ __forceinline__ int popw(const TraceArgs& a, Trav3& t, const int* __restrict__ stk, int lane, uint32_t gid) {
    --t.sp;
    if (t.sp < S) return stk[t.sp * BLOCK + lane];
    return a.spill[(uint64_t)(t.sp - S) * a.spill_lanes + gid];
}

// Coded node step (nodes from TraceArgs::cnodes, code_nodes in arx_bvh.hpp): a child word is
// already a stack entry (inner >= 0, leaf < 0, empty = kEmptyChildCode = a 0-triangle leaf), so the step
// is "hit or not" per child and one nearest-first choice: the nearer hit child is next (a
// leaf becomes the pending leaf), the farther one is pushed.  (A v_med3 clamp of the z slab
// looks cheaper but accepts every box behind the ray / beyond the hit that is entered through
// a z face with tn == tf: 4x the leaf tests.)  Requires t.pc == 0.
// BUF: fetch through a buffer resource (32-bit offsets, no 64-bit address VALU), and only the
// 56 bytes the step uses (the compiler widens a plain 8-byte tail load to 16 bytes).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t node_rsrc(const BvhNode* nodes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<BvhNode*>(nodes), (short)0, 0x7fffffff, 0x00020000);
}

// SPILL: STACK LDS entries + the global spill column (pushw / popw).
// Q16: 32-B QNode2 nodes (two 16-B loads; rs over TraceArgs::qnodes).  A slab plane is
// grid.origin + q * grid.scale, so t = (origin + q*scale - o) * inv = q * (scale*inv) +
// (origin - o)*inv: the caller passes ix = scale*inv and oix = (o - origin)*inv per axis, and the
// step is the same fma per plane after one u16 -> f32 conversion.  Conservative: the f32 error
// of that form is below 5 * 2^-24 * (grid extent) * |inv| for origins on the grid, far below the
// 0.1-step outward margin of every quantized plane (quantize_nodes16; the emitter is checked per launch).
template <int BLOCK, int STACK, bool BUF = false, bool SPILL = false, bool Q16 = false>
__device__ __forceinline__ void node_step7(const TraceArgs& a, const Ray& r, float oix, float oiy, float oiz, Trav3& t,
                                           int* __restrict__ stk, int lane, bool& overflow,
                                           __amdgpu_buffer_rsrc_t rs, uint32_t gid = 0) {
    if (t.node < 0) {  // pop
        int e;
        if constexpr (SPILL) {
            e = popw<BLOCK, STACK>(a, t, stk, lane, gid);
        } else {
            --t.sp;
            e = stk[t.sp * BLOCK + lane];
        }
        if (e < 0) {
            const int v = ~e;
            t.pf = v >> 4;
            t.pc = v & 15;
            return;
        }
        t.node = e;
    }
    float4 na, nb, nc;
    int2 nd;
    if constexpr (Q16) {
        const int off = t.node * (int)sizeof(QNode2);
        const uint4 A = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
        const uint4 B = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off + 16, 0, 0));
        // same register roles as the f32 node: na = (x0 lo, x0 hi, y0 lo, y0 hi), nb = child 1,
        // nc = (z0 lo, z0 hi, z1 lo, z1 hi)
        na = make_float4((float)(A.x & 0xffffu), (float)(A.x >> 16), (float)(A.y & 0xffffu), (float)(A.y >> 16));
        nb = make_float4((float)(B.x & 0xffffu), (float)(B.x >> 16), (float)(B.y & 0xffffu), (float)(B.y >> 16));
        nc = make_float4((float)(A.z & 0xffffu), (float)(A.z >> 16), (float)(B.z & 0xffffu), (float)(B.z >> 16));
        nd = make_int2((int)A.w, (int)B.w);
    } else if constexpr (BUF) {
        const int off = t.node * (int)sizeof(BvhNode);
        na = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
        nb = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, off + 16, 0, 0));
        nc = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, off + 32, 0, 0));
        nd = __builtin_bit_cast(int2, __builtin_amdgcn_raw_buffer_load_b64(rs, off + 48, 0, 0));
    } else {
        const float4* np = reinterpret_cast<const float4*>(a.cnodes + t.node);
        na = np[0];
        nb = np[1];
        nc = np[2];
        nd = *reinterpret_cast<const int2*>(np + 3);
    }
    const float ix = r.inv[0], iy = r.inv[1], iz = r.inv[2];
    const float x00 = __builtin_fmaf(na.x, ix, -oix), x01 = __builtin_fmaf(na.y, ix, -oix);
    const float y00 = __builtin_fmaf(na.z, iy, -oiy), y01 = __builtin_fmaf(na.w, iy, -oiy);
    const float z00 = __builtin_fmaf(nc.x, iz, -oiz), z01 = __builtin_fmaf(nc.y, iz, -oiz);
    const float x10 = __builtin_fmaf(nb.x, ix, -oix), x11 = __builtin_fmaf(nb.y, ix, -oix);
    const float y10 = __builtin_fmaf(nb.z, iy, -oiy), y11 = __builtin_fmaf(nb.w, iy, -oiy);
    const float z10 = __builtin_fmaf(nc.z, iz, -oiz), z11 = __builtin_fmaf(nc.w, iz, -oiz);
    const float tn0 = fmaxf(fmaxf(fminf(x00, x01), fminf(y00, y01)), fmaxf(fminf(z00, z01), 0.0f));
    const float tf0 = fminf(fminf(fmaxf(x00, x01), fmaxf(y00, y01)), fminf(fmaxf(z00, z01), t.best_t));
    const float tn1 = fmaxf(fmaxf(fminf(x10, x11), fminf(y10, y11)), fmaxf(fminf(z10, z11), 0.0f));
    const float tf1 = fminf(fminf(fmaxf(x10, x11), fmaxf(y10, y11)), fminf(fmaxf(z10, z11), t.best_t));
    const bool h0 = tn0 <= tf0, h1 = tn1 <= tf1;
    const bool near1 = h1 && (!h0 || tn1 < tn0);
    const int next = (h0 || h1) ? (near1 ? nd.y : nd.x) : -1;
    if (h0 && h1) {
        if constexpr (SPILL)
            pushw<BLOCK, STACK>(a, t, stk, lane, gid, near1 ? nd.x : nd.y, overflow);
        else
            push3<BLOCK, STACK>(t, stk, lane, near1 ? nd.x : nd.y, overflow);
    }
    // next >= 0: visit it; next < 0: a leaf (or -1: nothing) becomes the pending leaf, pop after
    const int v = ~next;
    t.node = next < 0 ? -1 : next;
    t.pf = v >> 4;                 // don't care while pc == 0
    t.pc = next < 0 ? (v & 15) : 0;
}

// Quad-cooperative node fetch through LDS (gfx950 buffer_load_dwordx4 ... lds).  Load k makes
// lane 4q+i fetch 16-B chunk i of quad-member k's node, so each wave-instruction touches 16
// distinct 64-B lines instead of 64 (the vector-memory address path is charged per line);
// the data lands in the wave's LDS stage as [k][lane] 16-B slots, i.e. the node of lane 4q+k
// is the 64 contiguous bytes at k*1024 + q*64.  Wave-wide: every lane passes a node (lanes
// without one pass 0 and ignore the result).
typedef __attribute__((address_space(3))) void* lds_ptr_t;

__device__ __forceinline__ void coop_fetch_lds(__amdgpu_buffer_rsrc_t rs, int node, int wl, int* stage) {
    const int c = (wl & 3) * 16;
    const int s0 = __builtin_amdgcn_mov_dpp(node, 0x00, 0xF, 0xF, false);
    const int s1 = __builtin_amdgcn_mov_dpp(node, 0x55, 0xF, 0xF, false);
    const int s2 = __builtin_amdgcn_mov_dpp(node, 0xAA, 0xF, 0xF, false);
    const int s3 = __builtin_amdgcn_mov_dpp(node, 0xFF, 0xF, 0xF, false);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)(stage), 16, s0 * 64 + c, 0, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)(stage + 256), 16, s1 * 64 + c, 0, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)(stage + 512), 16, s2 * 64 + c, 0, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)(stage + 768), 16, s3 * 64 + c, 0, 0, 0);
}

// node_step7 (coded nodes, spill stack) with the cooperative fetch.  Called by all lanes of
// the wave; `go` marks the lanes that take a step (t.pc == 0 and work left).
// CHECK 1: count lanes present at the fetch + compare with a direct load; 2: compare only.
// FIX (read-after-DMA experiments): 1 explicit vmcnt(0) + s_nop delay, 2 explicit vmcnt(0),
// 3 dword LDS reads.
template <int BLOCK, int STACK, int CHECK = 0, int FIX = 0>
__device__ __forceinline__ void node_step9(const TraceArgs& a, const Ray& r, float oix, float oiy, float oiz, Trav3& t,
                                           int* __restrict__ stk, int lane, bool& overflow,
                                           __amdgpu_buffer_rsrc_t rs, uint32_t gid, int* stage, bool go) {
    if constexpr (CHECK == 1) {  // lanes present at the wave-wide fetch
        const int present = __popcll(__ballot(true));
        if ((lane & 63) == 0) atomicAdd(a.counters + 12, (unsigned long long)present);
        if ((lane & 63) == 0) atomicAdd(a.counters + 13, 1ull);
    }
    bool fetch = go;
    if (go && t.node < 0) {  // pop
        const int e = popw<BLOCK, STACK>(a, t, stk, lane, gid);
        if (e < 0) {
            const int v = ~e;
            t.pf = v >> 4;
            t.pc = v & 15;
            fetch = false;
        } else {
            t.node = e;
        }
    }
    const int wl = lane & 63;
    coop_fetch_lds(rs, fetch ? t.node : 0, wl, stage);
    if constexpr (FIX == 1) asm volatile("s_waitcnt vmcnt(0)\n\ts_nop 7\n\ts_nop 7" ::: "memory");
    if constexpr (FIX == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (!fetch) return;
    float4 na, nb, nc;
    int2 nd;
    if constexpr (FIX == 3) {
        const volatile int* sv = stage + (wl & 3) * 256 + (wl >> 2) * 16;
        na = make_float4(__int_as_float(sv[0]), __int_as_float(sv[1]), __int_as_float(sv[2]), __int_as_float(sv[3]));
        nb = make_float4(__int_as_float(sv[4]), __int_as_float(sv[5]), __int_as_float(sv[6]), __int_as_float(sv[7]));
        nc = make_float4(__int_as_float(sv[8]), __int_as_float(sv[9]), __int_as_float(sv[10]), __int_as_float(sv[11]));
        nd = make_int2(sv[12], sv[13]);
    } else {
        const int4* sp = reinterpret_cast<const int4*>(stage + (wl & 3) * 256 + (wl >> 2) * 16);
        na = __builtin_bit_cast(float4, sp[0]);
        nb = __builtin_bit_cast(float4, sp[1]);
        nc = __builtin_bit_cast(float4, sp[2]);
        nd = *reinterpret_cast<const int2*>(sp + 3);
    }
    if constexpr (CHECK > 0) {
        const float4* np = reinterpret_cast<const float4*>(a.cnodes + t.node);
        const float4 ra = np[0], rb = np[1], rc = np[2];
        const int2 rd = *reinterpret_cast<const int2*>(np + 3);
        const bool same = ra.x == na.x && ra.y == na.y && ra.z == na.z && ra.w == na.w && rb.x == nb.x &&
                          rb.y == nb.y && rb.z == nb.z && rb.w == nb.w && rc.x == nc.x && rc.y == nc.y &&
                          rc.z == nc.z && rc.w == nc.w && rd.x == nd.x && rd.y == nd.y;
        if (!same) atomicAdd(a.counters + 14, 1ull);
        atomicAdd(a.counters + 15, 1ull);
    }
    const float ix = r.inv[0], iy = r.inv[1], iz = r.inv[2];
    const float x00 = __builtin_fmaf(na.x, ix, -oix), x01 = __builtin_fmaf(na.y, ix, -oix);
    const float y00 = __builtin_fmaf(na.z, iy, -oiy), y01 = __builtin_fmaf(na.w, iy, -oiy);
    const float z00 = __builtin_fmaf(nc.x, iz, -oiz), z01 = __builtin_fmaf(nc.y, iz, -oiz);
    const float x10 = __builtin_fmaf(nb.x, ix, -oix), x11 = __builtin_fmaf(nb.y, ix, -oix);
    const float y10 = __builtin_fmaf(nb.z, iy, -oiy), y11 = __builtin_fmaf(nb.w, iy, -oiy);
    const float z10 = __builtin_fmaf(nc.z, iz, -oiz), z11 = __builtin_fmaf(nc.w, iz, -oiz);
    const float tn0 = fmaxf(fmaxf(fminf(x00, x01), fminf(y00, y01)), fmaxf(fminf(z00, z01), 0.0f));
    const float tf0 = fminf(fminf(fmaxf(x00, x01), fmaxf(y00, y01)), fminf(fmaxf(z00, z01), t.best_t));
    const float tn1 = fmaxf(fmaxf(fminf(x10, x11), fminf(y10, y11)), fmaxf(fminf(z10, z11), 0.0f));
    const float tf1 = fminf(fminf(fmaxf(x10, x11), fmaxf(y10, y11)), fminf(fmaxf(z10, z11), t.best_t));
    const bool h0 = tn0 <= tf0, h1 = tn1 <= tf1;
    const bool near1 = h1 && (!h0 || tn1 < tn0);
    const int next = (h0 || h1) ? (near1 ? nd.y : nd.x) : -1;
    if (h0 && h1) pushw<BLOCK, STACK>(a, t, stk, lane, gid, near1 ? nd.x : nd.y, overflow);
    const int v = ~next;
    t.node = next < 0 ? -1 : next;
    t.pf = v >> 4;
    t.pc = next < 0 ? (v & 15) : 0;
}

// DBG: wave-level utilisation counters in counters[8..15] (variant 98): outer iterations,
// node-step iterations, lanes in node steps, leaf-step iterations, lanes in leaf steps,
// lanes shading, lanes idle (active, query done) at node/leaf iterations.
// Parked ray state (phased launches): float4(pos, e), float4(dir, dist), int4(depth, 0, 0, 0).
__device__ __forceinline__ void park_ray(const TraceArgs& a, int to, uint64_t slot, const RayState& s) {
    float4* rec = reinterpret_cast<float4*>(a.stash[to]) + 3 * slot;
    rec[0] = make_float4(s.pos.x, s.pos.y, s.pos.z, s.e);
    rec[1] = make_float4(s.dir.x, s.dir.y, s.dir.z, s.dist);
    rec[2] = make_float4(__int_as_float(s.depth), 0.0f, 0.0f, 0.0f);
}

__device__ __forceinline__ void unpark_ray(const TraceArgs& a, uint64_t slot, RayState& s) {
    const float4* rec = reinterpret_cast<const float4*>(a.stash[a.pool_from]) + 3 * slot;
    const float4 r0 = rec[0], r1 = rec[1], r2 = rec[2];
    s.pos = make_float3(r0.x, r0.y, r0.z);
    s.e = r0.w;
    s.dir = make_float3(r1.x, r1.y, r1.z);
    s.dist = r1.w;
    s.depth = __float_as_int(r2.x);
}

// Phase drain (wave-uniform): once the pool is exhausted and fewer than drain_low lanes still
// hold rays, the wave parks every ray that sits at a query boundary into the next phase's
// stash; the wave ends when its last in-flight query has been parked.
__device__ __forceinline__ void drain_wave(const TraceArgs& a, bool exhausted, bool trav, bool& active,
                                           bool& draining, const RayState& s, int lane, bool& overflow) {
    if (a.drain_low <= 0 || !exhausted) return;
    if (!draining && __popcll(__ballot(active)) < a.drain_low) draining = true;
    if (!draining) return;
    const unsigned long long park = __ballot(active && !trav);
    if (park == 0ull) return;
    const int to = a.pool_from < 0 ? 0 : 1 - a.pool_from;
    const int leader = __ffsll((unsigned long long)park) - 1;
    unsigned long long base = 0;
    if ((lane & 63) == leader) base = atomicAdd(a.stash_count + to, (unsigned long long)__popcll(park));
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)base, leader);
    const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(base >> 32), leader);
    base = ((unsigned long long)hi << 32) | lo;
    if (active && !trav) {
        const uint32_t rank =
            __builtin_amdgcn_mbcnt_hi((uint32_t)(park >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)park, 0u));
        if (base + rank < a.stash_cap) {
            park_ray(a, to, base + rank, s);
            active = false;
        } else {
            overflow = true;  // cannot happen with stash_cap >= lanes of the grid; keep the ray
        }
    }
}

// Branch-free node step (same traversal order as node_step3).  Divergent `if`s cost scalar
// exec-mask bookkeeping that one scalar unit per CU executes for all 20 waves -- the node
// loop was bound by it -- so every decision here is a v_cndmask and the stack is written
// unconditionally (to a dummy row STACK when nothing is pushed).  Requires stk[(STACK+1)*BLOCK].
template <int BLOCK, int STACK>
__device__ __forceinline__ void node_step5(const TraceArgs& a, const Ray& r, float oix, float oiy, float oiz, Trav3& t,
                                           int* __restrict__ stk, int lane, bool& overflow) {
    // pop (lanes whose next node is on the stack); a popped leaf becomes the pending leaf
    const bool do_pop = t.node < 0;
    const int sp_pop = t.sp - 1;
    const int e = stk[(do_pop ? sp_pop : STACK) * BLOCK + lane];
    t.sp = do_pop ? sp_pop : t.sp;
    const bool got_leaf = do_pop && e < 0;
    const int ne = ~e;  // -(first*16 + count) - 1 -> first*16 + count
    t.pf = got_leaf ? (ne >> 4) : t.pf;
    t.pc = got_leaf ? (ne & 15) : t.pc;
    const int node = do_pop ? (got_leaf ? 0 : e) : t.node;  // got_leaf: harmless visit of node 0, discarded
    const float4* np = reinterpret_cast<const float4*>(a.nodes + node);
    const float4 na = np[0];
    const float4 nb = np[1];
    const float4 nc = np[2];
    const int4 nd = *reinterpret_cast<const int4*>(np + 3);
    const float ix = r.inv[0], iy = r.inv[1], iz = r.inv[2];
    const float x00 = __builtin_fmaf(na.x, ix, -oix), x01 = __builtin_fmaf(na.y, ix, -oix);
    const float y00 = __builtin_fmaf(na.z, iy, -oiy), y01 = __builtin_fmaf(na.w, iy, -oiy);
    const float z00 = __builtin_fmaf(nc.x, iz, -oiz), z01 = __builtin_fmaf(nc.y, iz, -oiz);
    const float tn0 = fmaxf(fmaxf(fminf(x00, x01), fminf(y00, y01)), fmaxf(fminf(z00, z01), 0.0f));
    const float tf0 = fminf(fminf(fmaxf(x00, x01), fmaxf(y00, y01)), fminf(fmaxf(z00, z01), t.best_t));
    const float x10 = __builtin_fmaf(nb.x, ix, -oix), x11 = __builtin_fmaf(nb.y, ix, -oix);
    const float y10 = __builtin_fmaf(nb.z, iy, -oiy), y11 = __builtin_fmaf(nb.w, iy, -oiy);
    const float z10 = __builtin_fmaf(nc.z, iz, -oiz), z11 = __builtin_fmaf(nc.w, iz, -oiz);
    const float tn1 = fmaxf(fmaxf(fminf(x10, x11), fminf(y10, y11)), fmaxf(fminf(z10, z11), 0.0f));
    const float tf1 = fminf(fminf(fmaxf(x10, x11), fmaxf(y10, y11)), fminf(fmaxf(z10, z11), t.best_t));
    const bool h0 = !got_leaf && tn0 <= tf0 && nd.z >= 0;
    const bool h1 = !got_leaf && tn1 <= tf1 && nd.w >= 0;
    const bool l0 = h0 && nd.z > 0, l1 = h1 && nd.w > 0;
    const bool i0 = h0 && nd.z == 0, i1 = h1 && nd.w == 0;
    const bool swap = tn1 < tn0;
    // leaves: the nearer hit leaf is parked, a second one pushed
    const bool two_l = l0 && l1;
    const bool near_is1 = two_l ? swap : l1;
    const bool any_l = l0 || l1;
    t.pf = any_l ? (near_is1 ? nd.y : nd.x) : t.pf;
    t.pc = any_l ? (near_is1 ? nd.w : nd.z) : t.pc;
    {
        const int code = swap ? leaf_code(nd.x, nd.z) : leaf_code(nd.y, nd.w);
        const bool fits = t.sp < STACK;
        overflow = overflow || (two_l && !fits);
        const bool push = two_l && fits;
        stk[(push ? t.sp : STACK) * BLOCK + lane] = code;
        t.sp += push ? 1 : 0;
    }
    // inner children: visit the nearer, push the other
    const bool two_i = i0 && i1;
    {
        const int far_n = swap ? nd.x : nd.y;
        const bool fits = t.sp < STACK;
        overflow = overflow || (two_i && !fits);
        const bool push = two_i && fits;
        stk[(push ? t.sp : STACK) * BLOCK + lane] = far_n;
        t.sp += push ? 1 : 0;
    }
    const int next = two_i ? (swap ? nd.y : nd.x) : (i0 ? nd.x : (i1 ? nd.y : -1));
    t.node = got_leaf ? -1 : next;
}

// ---- quad-cooperative node fetch -------------------------------------------------------
// The vector-memory return path charges per distinct 64-B block per wave-instruction
// (tools/td_microbench.hip: a divergent dwordx4 with 64 distinct blocks costs ~4x one whose
// quads share blocks).  Fetching a 64-B node as 4 per-lane dwordx4 loads therefore pays for
// the node's block 4 times.  Here load k makes the 4 lanes of a quad read the 4 chunks of
// quad-member k's node (one block per quad), and a 2-round DPP transpose (xor 1, xor 2
// within the quad) hands every lane its own node.  Must run with all 64 lanes active;
// lanes without a node pass node 0 and discard the result.
__device__ __forceinline__ int dpp_bcast(int v, int k) {
    switch (k) {  // quad_perm [k,k,k,k]
        case 0: return __builtin_amdgcn_mov_dpp(v, 0x00, 0xF, 0xF, false);
        case 1: return __builtin_amdgcn_mov_dpp(v, 0x55, 0xF, 0xF, false);
        case 2: return __builtin_amdgcn_mov_dpp(v, 0xAA, 0xF, 0xF, false);
        default: return __builtin_amdgcn_mov_dpp(v, 0xFF, 0xF, 0xF, false);
    }
}

template <int XOR>
__device__ __forceinline__ int dpp_xor(int v) {  // quad_perm [1,0,3,2] / [2,3,0,1]
    return __builtin_amdgcn_mov_dpp(v, XOR == 1 ? 0xB1 : 0x4E, 0xF, 0xF, false);
}

struct Chunk {
    int v[4];
};

__device__ __forceinline__ void coop_fetch_node(const BvhNode* __restrict__ nodes, int node, int lane, float4& na,
                                                float4& nb, float4& nc, int4& nd) {
    const int q = lane & 3;
    Chunk R[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int src = dpp_bcast(node, k);
        const int4 x = reinterpret_cast<const int4*>(nodes + src)[q];
        R[k].v[0] = x.x;
        R[k].v[1] = x.y;
        R[k].v[2] = x.z;
        R[k].v[3] = x.w;
    }
    // lane q holds row q of M[chunk][owner]; transpose so that it holds column q
    Chunk S[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const bool take = ((k ^ q) & 1) != 0;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int o = dpp_xor<1>(R[k ^ 1].v[c]);
            S[k].v[c] = take ? o : R[k].v[c];
        }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const bool take = ((k ^ q) & 2) != 0;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int o = dpp_xor<2>(S[k ^ 2].v[c]);
            R[k].v[c] = take ? o : S[k].v[c];
        }
    }
    na = make_float4(__int_as_float(R[0].v[0]), __int_as_float(R[0].v[1]), __int_as_float(R[0].v[2]),
                     __int_as_float(R[0].v[3]));
    nb = make_float4(__int_as_float(R[1].v[0]), __int_as_float(R[1].v[1]), __int_as_float(R[1].v[2]),
                     __int_as_float(R[1].v[3]));
    nc = make_float4(__int_as_float(R[2].v[0]), __int_as_float(R[2].v[1]), __int_as_float(R[2].v[2]),
                     __int_as_float(R[2].v[3]));
    nd = make_int4(R[3].v[0], R[3].v[1], R[3].v[2], R[3].v[3]);
}

// node_step3 with the quad-cooperative fetch: the pop is per lane, the fetch is wave-wide,
// the box tests and stack updates are per lane again.
template <int BLOCK, int STACK>
__device__ __forceinline__ void node_step6(const TraceArgs& a, const Ray& r, float oix, float oiy, float oiz, Trav3& t,
                                           int* __restrict__ stk, int lane, bool& overflow, bool can_node) {
    int node = -1;
    if (can_node) {
        if (t.node < 0) {  // pop
            --t.sp;
            const int e = stk[t.sp * BLOCK + lane];
            if (e >= 0) {
                t.node = e;
            } else {
                const int v = -e - 1;
                t.pf = v >> 4;
                t.pc = v & 15;
            }
        }
        node = t.node;
    }
    float4 na, nb, nc;
    int4 nd;
    coop_fetch_node(a.nodes, node >= 0 ? node : 0, lane, na, nb, nc, nd);
    if (node < 0) return;
    const float ix = r.inv[0], iy = r.inv[1], iz = r.inv[2];
    const float x00 = __builtin_fmaf(na.x, ix, -oix), x01 = __builtin_fmaf(na.y, ix, -oix);
    const float y00 = __builtin_fmaf(na.z, iy, -oiy), y01 = __builtin_fmaf(na.w, iy, -oiy);
    const float z00 = __builtin_fmaf(nc.x, iz, -oiz), z01 = __builtin_fmaf(nc.y, iz, -oiz);
    const float tn0 = fmaxf(fmaxf(fminf(x00, x01), fminf(y00, y01)), fmaxf(fminf(z00, z01), 0.0f));
    const float tf0 = fminf(fminf(fmaxf(x00, x01), fmaxf(y00, y01)), fminf(fmaxf(z00, z01), t.best_t));
    const float x10 = __builtin_fmaf(nb.x, ix, -oix), x11 = __builtin_fmaf(nb.y, ix, -oix);
    const float y10 = __builtin_fmaf(nb.z, iy, -oiy), y11 = __builtin_fmaf(nb.w, iy, -oiy);
    const float z10 = __builtin_fmaf(nc.z, iz, -oiz), z11 = __builtin_fmaf(nc.w, iz, -oiz);
    const float tn1 = fmaxf(fmaxf(fminf(x10, x11), fminf(y10, y11)), fmaxf(fminf(z10, z11), 0.0f));
    const float tf1 = fminf(fminf(fmaxf(x10, x11), fmaxf(y10, y11)), fminf(fmaxf(z10, z11), t.best_t));
    const bool h0 = tn0 <= tf0 && nd.z >= 0;
    const bool h1 = tn1 <= tf1 && nd.w >= 0;
    const bool l0 = h0 && nd.z > 0, l1 = h1 && nd.w > 0;
    const bool i0 = h0 && nd.z == 0, i1 = h1 && nd.w == 0;
    if (l0 && l1) {
        const bool swap = tn1 < tn0;
        t.pf = swap ? nd.y : nd.x;
        t.pc = swap ? nd.w : nd.z;
        push3<BLOCK, STACK>(t, stk, lane, swap ? leaf_code(nd.x, nd.z) : leaf_code(nd.y, nd.w), overflow);
    } else if (l0) {
        t.pf = nd.x;
        t.pc = nd.z;
    } else if (l1) {
        t.pf = nd.y;
        t.pc = nd.w;
    }
    if (i0 && i1) {
        const bool swap = tn1 < tn0;
        push3<BLOCK, STACK>(t, stk, lane, swap ? nd.x : nd.y, overflow);
        t.node = swap ? nd.y : nd.x;
    } else if (i0) {
        t.node = nd.x;
    } else if (i1) {
        t.node = nd.y;
    } else {
        t.node = -1;
    }
}

template <int BLOCK, int STACK, int THRESH, int LEAF_THRESH, int MINW, bool DBG = false, int LV = 1, int NS = 3,
          int MIG = 0>
__global__ __launch_bounds__(BLOCK, MINW) void trace_kernel_v3(TraceArgs a) {
    uint64_t d_outer = 0, d_nit = 0, d_nl = 0, d_lit = 0, d_ll = 0, d_sh = 0, d_idle = 0, d_pend = 0, d_inact = 0;
    uint64_t c_outer = 0, c_node = 0, c_leaf = 0, c_mark = 0;  // DBG: s_memtime cycles per phase
    if constexpr (DBG) c_mark = __builtin_amdgcn_s_memtime();
    __shared__ int stk[(STACK + 1) * BLOCK];  // row STACK: dummy target of branch-free pushes
    // NS >= 200: the NS - 200 step scheme over 16-bit quantized QNode2 nodes (NS - 200 >= 40)
    constexpr bool QN = NS >= 200;
    constexpr int NSB = QN ? NS - 200 : NS;
    static_assert(!QN || (NSB >= 40 && NSB < 80), "quantized nodes: buffer-load coded steps only");
    constexpr bool COOP = NSB >= 80;  // cooperative LDS fetch (node_step9)
    constexpr int kCheck9 = (NSB >= 100 && NSB < 120) ? 1 : (NSB >= 120 && NSB < 140) ? 2 : 0;
    constexpr int kFix9 = NSB >= 180 ? 3 : NSB >= 160 ? 2 : NSB >= 140 ? 1 : 0;
    __shared__ __attribute__((aligned(16))) int stage_all[COOP ? BLOCK * 16 : 4];
    int* const stage = stage_all + (COOP ? (threadIdx.x >> 6) * 1024 : 0);
    const __amdgpu_buffer_rsrc_t nrs =  // coded nodes (NS >= 40) or their quantized copy
        QN ? __builtin_amdgcn_make_buffer_rsrc(const_cast<QNode2*>(a.qnodes), (short)0, 0x7fffffff, 0x00020000)
           : node_rsrc(a.cnodes);
    const uint32_t gid = blockIdx.x * BLOCK + threadIdx.x;     // spill column (NS >= 60)
    // MIG > 0: block-level ray migration (see migrate comment below); LDS queue of parked rays
    constexpr int MQ = MIG > 0 ? 64 : 1;
    __shared__ float4 mq_a[MQ], mq_b[MQ];
    __shared__ int mq_d[MQ];
    __shared__ int mq_lock, mq_count, mq_live;
    if constexpr (MIG > 0) {
        if (threadIdx.x == 0) {
            mq_lock = 0;
            mq_count = 0;
            mq_live = BLOCK / 64;
        }
        __syncthreads();
    }
    const int lane = threadIdx.x;
    const uint64_t n = a.pool_from < 0 ? a.ray_end - a.ray_begin : a.stash_count[a.pool_from];
    // static per-wave ranges (a.static_ranges): wave w owns pool entries [w_next, w_end).
    // 1: n / n_waves each; 2: whole 64-ray chunks spread evenly (a wave's last round is full,
    // not a few lanes); 3: whole chunks, the surplus chunks on the first waves.
    const uint32_t wave_id = __builtin_amdgcn_readfirstlane((blockIdx.x * BLOCK + threadIdx.x) >> 6);
    const uint32_t n_waves = gridDim.x * (BLOCK / 64);
    uint64_t w_next, w_end;
    if (a.static_ranges >= 2) {
        const uint64_t chunks = (n + 63) / 64;
        uint64_t c0, c1;
        if (a.static_ranges == 2) {
            c0 = chunks * wave_id / n_waves;
            c1 = chunks * (wave_id + 1) / n_waves;
        } else {
            const uint64_t q = chunks / n_waves, rem = chunks % n_waves;
            c0 = q * wave_id + min((uint64_t)wave_id, rem);
            c1 = c0 + q + (wave_id < rem ? 1 : 0);
        }
        w_next = min(n, 64 * c0);
        w_end = min(n, 64 * c1);
    } else {
        w_next = n * wave_id / n_waves;
        w_end = n * (wave_id + 1) / n_waves;
    }
    bool draining = false;
    unsigned long long* const cursor = a.counters + 4;
    uint32_t n_q = 0, n_rx = 0, n_miss = 0;
    bool overflow = false;
    bool active = false;
    bool trav = false;
    bool exhausted = false;
    RayState s;
    Ray r;
    Trav3 t;
    float oix = 0.f, oiy = 0.f, oiz = 0.f;
    s.depth = -1;
    // every field defined: lanes that never receive a ray must not see a stale pending leaf
    t.best_t = __builtin_huge_valf();
    t.best_id = 0x7fffffff;
    t.best = -1;
    t.node = -1;
    t.sp = 0;
    t.pf = 0;
    t.pc = 0;
    t.visits = 0;
    while (true) {
        if constexpr (DBG) {
            ++d_outer;
            d_sh += __popcll(__ballot(active && !trav));
        }
        if (active && !trav) {
            shade(a, s, r, t.best, n_rx, n_miss);
            if (!wants_query(a, s)) active = false;
        }
        drain_wave(a, exhausted, trav, active, draining, s, lane, overflow);
        const unsigned long long need = __ballot(!active);
        if (need != 0ull && !exhausted) {
            const int cnt = __popcll(need);
            unsigned long long base = 0;
            uint64_t lim = n;
            if (a.static_ranges) {  // wave-uniform, no atomic on the critical path
                base = w_next;
                lim = w_end;
                w_next += (uint64_t)cnt;
            } else {
                const int leader = __ffsll((unsigned long long)need) - 1;
                if ((lane & 63) == leader) base = atomicAdd(cursor, (unsigned long long)cnt);
                const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)base, leader);
                const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(base >> 32), leader);
                base = ((unsigned long long)hi << 32) | lo;
            }
            if (!active) {
                const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(need >> 32),
                                                                __builtin_amdgcn_mbcnt_lo((uint32_t)need, 0u));
                const uint64_t i = base + rank;
                if (i < lim) {
                    if (a.pool_from < 0)
                        ray_init(a, s, a.ray_begin + i);
                    else
                        unpark_ray(a, i, s);
                    active = wants_query(a, s);
                }
            }
            if (base + (unsigned long long)cnt >= lim) exhausted = true;
        }
        if constexpr (MIG > 0) {
            // Block-level migration once this wave's range is exhausted.  Under an LDS lock:
            //  * a sparse wave (<= MIG rays, all at a query boundary) parks its rays in the block
            //    queue and exits -- unless it is the last live wave of the block;
            //  * a wave with empty lanes pulls parked rays;
            //  * a wave with no rays exits only when the queue is empty.
            // The last live wave never parks, so parked rays are always picked up; no wave ever
            // waits for another (the lock is held for a few LDS operations only).
            const unsigned long long act = __ballot(active);
            const unsigned long long bnd = __ballot(active && !trav);
            const int n_act = __popcll(act);
            const int peek = __builtin_amdgcn_readfirstlane(
                __hip_atomic_load(&mq_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
            // the lock is only worth taking to park (sparse wave at a boundary), to pull (queue
            // non-empty) or to leave (no rays); the decision is re-checked under the lock
            const bool want = (n_act > 0 && act == bnd && n_act <= MIG) || (n_act < 64 && peek > 0) || n_act == 0;
            if (exhausted && want) {
                const int wl = lane & 63;
                if (wl == 0) {
                    while (atomicCAS(&mq_lock, 0, 1) != 0) __builtin_amdgcn_s_sleep(1);
                }
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                const int qcnt = __builtin_amdgcn_readfirstlane(__hip_atomic_load(&mq_count, __ATOMIC_RELAXED,
                                                                                  __HIP_MEMORY_SCOPE_WORKGROUP));
                const int live = __builtin_amdgcn_readfirstlane(__hip_atomic_load(&mq_live, __ATOMIC_RELAXED,
                                                                                  __HIP_MEMORY_SCOPE_WORKGROUP));
                bool leave = false;
                int new_cnt = qcnt, new_live = live;
                if (n_act > 0 && act == bnd && n_act <= MIG && live > 1 && qcnt + n_act <= MQ) {
                    if (active) {
                        const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(act >> 32),
                                                                        __builtin_amdgcn_mbcnt_lo((uint32_t)act, 0u));
                        const int slot = qcnt + (int)rank;
                        mq_a[slot] = make_float4(s.pos.x, s.pos.y, s.pos.z, s.e);
                        mq_b[slot] = make_float4(s.dir.x, s.dir.y, s.dir.z, s.dist);
                        mq_d[slot] = s.depth;
                        active = false;
                    }
                    new_cnt = qcnt + n_act;
                    new_live = live - 1;
                    leave = true;
                } else if (n_act < 64 && qcnt > 0) {
                    const int take = min(qcnt, 64 - n_act);
                    if (!active) {
                        const unsigned long long idle = ~act;
                        const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(idle >> 32),
                                                                        __builtin_amdgcn_mbcnt_lo((uint32_t)idle, 0u));
                        if ((int)rank < take) {
                            const int slot = qcnt - 1 - (int)rank;
                            const float4 qa = mq_a[slot], qb = mq_b[slot];
                            s.pos = make_float3(qa.x, qa.y, qa.z);
                            s.e = qa.w;
                            s.dir = make_float3(qb.x, qb.y, qb.z);
                            s.dist = qb.w;
                            s.depth = mq_d[slot];
                            active = true;  // parked at a query boundary that wanted a query
                        }
                    }
                    new_cnt = qcnt - take;
                } else if (n_act == 0 && qcnt == 0) {
                    new_live = live - 1;
                    leave = true;
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                if (wl == 0) {
                    __hip_atomic_store(&mq_count, new_cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    __hip_atomic_store(&mq_live, new_live, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                    atomicExch(&mq_lock, 0);
                }
                if (leave) break;
            }
        }
        if (active && !trav) {
            ++n_q;
            setup_ray(r, s.pos, s.dir);
            if constexpr (QN) {  // grid form of the slab planes (node_step7 Q16)
                oix = (r.o[0] - a.qgrid.origin[0]) * r.inv[0];
                oiy = (r.o[1] - a.qgrid.origin[1]) * r.inv[1];
                oiz = (r.o[2] - a.qgrid.origin[2]) * r.inv[2];
                r.inv[0] *= a.qgrid.scale[0];
                r.inv[1] *= a.qgrid.scale[1];
                r.inv[2] *= a.qgrid.scale[2];
            } else {
                oix = r.o[0] * r.inv[0];
                oiy = r.o[1] * r.inv[1];
                oiz = r.o[2] * r.inv[2];
            }
            t.best_t = __builtin_huge_valf();
            t.best_id = 0x7fffffff;
            t.best = -1;
            t.node = 0;
            t.sp = 0;
            t.pc = 0;
            t.pf = 0;
            t.visits = 0;
            trav = true;
        }
        if (__ballot(active) == 0ull) {
            if (exhausted) break;
            continue;
        }
        if constexpr (DBG) {
            const uint64_t now = __builtin_amdgcn_s_memtime();
            c_outer += now - c_mark;
            c_mark = now;
        }
        while (true) {
            if (trav && t.pc == 0 && t.node < 0 && t.sp == 0) trav = false;  // query finished
            const bool can_node = trav && t.pc == 0;
            const unsigned long long m_node = __ballot(can_node);
            const unsigned long long m_leaf = __ballot(trav && t.pc > 0);
            if ((m_node | m_leaf) == 0ull) break;
            const int n_idle = __popcll(__ballot(active && !trav));
            if (n_idle >= THRESH) break;
            if constexpr (DBG) d_idle += n_idle;
            if (m_node != 0ull && __popcll(m_leaf) < LEAF_THRESH) {
                if constexpr (DBG) {
                    ++d_nit;
                    d_nl += __popcll(m_node);
                    d_pend += __popcll(m_leaf);
                    d_inact += __popcll(__ballot(!active));
                }
                if constexpr (COOP) {  // wave-wide steps: 1 + NSB % 20
                    node_step9<BLOCK, STACK, kCheck9, kFix9>(a, r, oix, oiy, oiz, t, stk, lane, overflow, nrs, gid, stage,
                                                          can_node);
#pragma unroll
                    for (int k = 0; k < NSB % 20; ++k) {
                        const bool go = can_node && t.pc == 0 && (t.node >= 0 || t.sp > 0);
                        if (__ballot(go) == 0ull) break;
                        node_step9<BLOCK, STACK, kCheck9, kFix9>(a, r, oix, oiy, oiz, t, stk, lane, overflow, nrs, gid,
                                                              stage, go);
                    }
                } else if constexpr (NSB == 6) {
                    node_step6<BLOCK, STACK>(a, r, oix, oiy, oiz, t, stk, lane, overflow, can_node);  // all lanes
                } else if (can_node) {
                    if constexpr (NSB >= 60)
                        node_step7<BLOCK, STACK, true, true, QN>(a, r, oix, oiy, oiz, t, stk, lane, overflow, nrs, gid);
                    else if constexpr (NSB >= 40)
                        node_step7<BLOCK, STACK, true, false, QN>(a, r, oix, oiy, oiz, t, stk, lane, overflow, nrs);
                    else if constexpr (NSB >= 20)
                        node_step7<BLOCK, STACK>(a, r, oix, oiy, oiz, t, stk, lane, overflow, nrs);
                    else if constexpr (NSB == 5)
                        node_step5<BLOCK, STACK>(a, r, oix, oiy, oiz, t, stk, lane, overflow);
                    else if constexpr (NSB == 7)
                        node_step3<BLOCK, STACK, true>(a, r, oix, oiy, oiz, t, stk, lane, overflow);
                    else
                        node_step3<BLOCK, STACK>(a, r, oix, oiy, oiz, t, stk, lane, overflow);
                }
                if constexpr (COOP) {
                } else if constexpr (NSB >= 20) {  // coded node step + NSB % 20 extra steps (NSB >= 40: buffer loads)
#pragma unroll
                    for (int k = 0; k < NSB % 20; ++k) {
                        if (can_node && t.pc == 0 && (t.node >= 0 || t.sp > 0))
                            node_step7<BLOCK, STACK, (NSB >= 40), (NSB >= 60), QN>(a, r, oix, oiy, oiz, t, stk, lane, overflow,
                                                                             nrs, gid);
                    }
                } else if constexpr (NSB >= 8) {
                    // Extra node steps for lanes that can go on, without the loop control above:
                    // NS 8/9/10 = 1/2/3 extra steps; NS 11/12 = up to 3 while >= 24/16 lanes can;
                    // NS 13/14 = 5/7 extra; NS 15/16 = up to 7 while >= 24/32; NS 17 = up to 15 while >= 24.
                    constexpr int kExtra = NSB <= 10 ? NSB - 7 : NSB <= 12 ? 3 : NSB == 13 ? 5 : NSB <= 16 ? 7 : 15;
                    constexpr int kMinLanes = (NSB == 11 || NSB == 15 || NSB == 17) ? 24 : NSB == 12 ? 16 : NSB == 16 ? 32 : 0;
#pragma unroll
                    for (int k = 0; k < kExtra; ++k) {
                        const bool go = can_node && t.pc == 0 && (t.node >= 0 || t.sp > 0);
                        if constexpr (kMinLanes > 0) {
                            if (k > 0 && __popcll(__ballot(go)) < kMinLanes) break;
                        }
                        if (go) node_step3<BLOCK, STACK>(a, r, oix, oiy, oiz, t, stk, lane, overflow);
                    }
                }
                if constexpr (DBG) {
                    const uint64_t now = __builtin_amdgcn_s_memtime();
                    c_node += now - c_mark;
                    c_mark = now;
                }
            } else {
                if constexpr (DBG) {
                    ++d_lit;
                    d_ll += __popcll(m_leaf);
                }
                if constexpr (NSB == 5) {
                    const bool mine = trav && t.pc > 0;
                    leaf_hits_u<LV>(a.tris, r, t.pf, mine ? t.pc : 0, t.best_t, t.best_id, t.best);
                    t.pc = mine ? 0 : t.pc;
                } else if (trav && t.pc > 0) {
                    leaf_hits_vec<LV>(a.tris, r, t.pf, t.pc, t.best_t, t.best_id, t.best);
                    t.pc = 0;
                }
                if constexpr (DBG) {
                    const uint64_t now = __builtin_amdgcn_s_memtime();
                    c_leaf += now - c_mark;
                    c_mark = now;
                }
            }
        }
    }
    flush_counters(a, n_q, n_rx, n_miss, overflow, lane);
    if constexpr (DBG) {
        if ((lane & 63) == 0) {
            atomicAdd(a.counters + 8, (unsigned long long)d_outer);
            atomicAdd(a.counters + 9, (unsigned long long)d_nit);
            atomicAdd(a.counters + 10, (unsigned long long)d_nl);
            atomicAdd(a.counters + 11, (unsigned long long)d_lit);
            atomicAdd(a.counters + 12, (unsigned long long)d_ll);
            atomicAdd(a.counters + 13, (unsigned long long)d_sh);
            atomicAdd(a.counters + 14, (unsigned long long)d_idle);
            atomicAdd(a.counters + 5, (unsigned long long)c_node);
            atomicAdd(a.counters + 15, (unsigned long long)c_leaf);
            atomicAdd(a.counters + 7, (unsigned long long)c_outer);
            atomicAdd(a.counters + 6, (unsigned long long)(d_pend << 32 | (d_inact & 0xffffffffull)));
        }
    }
}

// ---- v5: branch-minimal coded traversal ---------------------------------------------------
// t.node holds the lane's next stack entry: >= 0 an inner node (take a node step), <= -2 a
// leaf ~(first*16 + count) (pending until the wave's leaf phase), -1 = the query is done.
// Entries are popped at the END of a node step (and of a leaf test), so a lane at -1 has an
// empty stack and the step guard is just `t.node >= 0`.  Inside the step every decision is a
// select and the far child is written unconditionally (to the slot above the top of the
// stack, or to the spare row STACK), so the only exec-mask work per step is that guard: the
// branchy steps spent ~52 scalar instructions per step on exec masks, and the CU's one scalar
// unit serves all 20 waves.
// NF: node format.  0 coded BvhNode (56 B), 1 QNode2 (32 B), 2 QNode2 octant copy of this ray's
// direction signs (obase = byte offset of that copy): each axis word is (near | far << 16), so
// the slab test takes max / min of the near / far planes without the per-axis min/max.
template <int BLOCK, int STACK, int NF>
__device__ __forceinline__ void node_step8(const Ray& r, float oix, float oiy, float oiz, Trav3& t,
                                           int* __restrict__ stk, int lane, __amdgpu_buffer_rsrc_t rs,
                                           int obase = 0) {
    constexpr int FMT = NF & 15;  // NF >> 4: cache-policy bits of the QNode2 loads (design experiments)
    constexpr int CP = NF >> 4;
    // the pop candidate is read first, so its LDS latency hides under the node fetch (the
    // slot sp - 1 is not touched by this step's write to slot sp)
    const int sp = t.sp;
    const int sp_pop = max(sp - 1, 0);
    int top = stk[sp_pop * BLOCK + lane];
    const float ix = r.inv[0], iy = r.inv[1], iz = r.inv[2];
    float tn0, tf0, tn1, tf1;
    int c0, c1;
    if constexpr (FMT == 2) {
        const int off = obase + t.node * (int)sizeof(QNode2);
        const uint4 A = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
        const uint4 B = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off + 16, 0, 0));
        // child 0: A.x, A.y, A.z; child 1: B.x, B.y, B.z (x, y, z words)
        const float nx0 = __builtin_fmaf((float)(A.x & 0xffffu), ix, -oix), fx0 = __builtin_fmaf((float)(A.x >> 16), ix, -oix);
        const float ny0 = __builtin_fmaf((float)(A.y & 0xffffu), iy, -oiy), fy0 = __builtin_fmaf((float)(A.y >> 16), iy, -oiy);
        const float nz0 = __builtin_fmaf((float)(A.z & 0xffffu), iz, -oiz), fz0 = __builtin_fmaf((float)(A.z >> 16), iz, -oiz);
        const float nx1 = __builtin_fmaf((float)(B.x & 0xffffu), ix, -oix), fx1 = __builtin_fmaf((float)(B.x >> 16), ix, -oix);
        const float ny1 = __builtin_fmaf((float)(B.y & 0xffffu), iy, -oiy), fy1 = __builtin_fmaf((float)(B.y >> 16), iy, -oiy);
        const float nz1 = __builtin_fmaf((float)(B.z & 0xffffu), iz, -oiz), fz1 = __builtin_fmaf((float)(B.z >> 16), iz, -oiz);
        tn0 = fmaxf(fmaxf(nx0, ny0), fmaxf(nz0, 0.0f));
        tf0 = fminf(fminf(fx0, fy0), fminf(fz0, t.best_t));
        tn1 = fmaxf(fmaxf(nx1, ny1), fmaxf(nz1, 0.0f));
        tf1 = fminf(fminf(fx1, fy1), fminf(fz1, t.best_t));
        c0 = (int)A.w;
        c1 = (int)B.w;
    } else {
    float4 na, nb, nc;
    if constexpr (FMT == 1) {  // QNode2 (node_step7 Q16)
        const int off = t.node * (int)sizeof(QNode2);
        const uint4 A = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, CP));
        const uint4 B = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off + 16, 0, CP));
        na = make_float4((float)(A.x & 0xffffu), (float)(A.x >> 16), (float)(A.y & 0xffffu), (float)(A.y >> 16));
        nb = make_float4((float)(B.x & 0xffffu), (float)(B.x >> 16), (float)(B.y & 0xffffu), (float)(B.y >> 16));
        nc = make_float4((float)(A.z & 0xffffu), (float)(A.z >> 16), (float)(B.z & 0xffffu), (float)(B.z >> 16));
        c0 = (int)A.w;
        c1 = (int)B.w;
    } else {  // coded BvhNode, 56 B
        const int off = t.node * (int)sizeof(BvhNode);
        na = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
        nb = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, off + 16, 0, 0));
        nc = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, off + 32, 0, 0));
        const int2 d = __builtin_bit_cast(int2, __builtin_amdgcn_raw_buffer_load_b64(rs, off + 48, 0, 0));
        c0 = d.x;
        c1 = d.y;
    }
    const float x00 = __builtin_fmaf(na.x, ix, -oix), x01 = __builtin_fmaf(na.y, ix, -oix);
    const float y00 = __builtin_fmaf(na.z, iy, -oiy), y01 = __builtin_fmaf(na.w, iy, -oiy);
    const float z00 = __builtin_fmaf(nc.x, iz, -oiz), z01 = __builtin_fmaf(nc.y, iz, -oiz);
    const float x10 = __builtin_fmaf(nb.x, ix, -oix), x11 = __builtin_fmaf(nb.y, ix, -oix);
    const float y10 = __builtin_fmaf(nb.z, iy, -oiy), y11 = __builtin_fmaf(nb.w, iy, -oiy);
    const float z10 = __builtin_fmaf(nc.z, iz, -oiz), z11 = __builtin_fmaf(nc.w, iz, -oiz);
    tn0 = fmaxf(fmaxf(fminf(x00, x01), fminf(y00, y01)), fmaxf(fminf(z00, z01), 0.0f));
    tf0 = fminf(fminf(fmaxf(x00, x01), fmaxf(y00, y01)), fminf(fmaxf(z00, z01), t.best_t));
    tn1 = fmaxf(fmaxf(fminf(x10, x11), fminf(y10, y11)), fmaxf(fminf(z10, z11), 0.0f));
    tf1 = fminf(fminf(fmaxf(x10, x11), fmaxf(y10, y11)), fminf(fmaxf(z10, z11), t.best_t));
    }
    // bitwise ops on the bools: && / || would become exec-mask branches again
    const bool h0 = tn0 <= tf0, h1 = tn1 <= tf1;
    const bool near1 = h1 & (!h0 | (tn1 < tn0));
    const int c_near = near1 ? c1 : c0;
    const int c_far = near1 ? c0 : c1;
    // The stack never overflows: it holds at most one entry per tree level and the launcher
    // requires STACK > bvh_depth.  The clamp only keeps the write inside the array.
    stk[min(sp, STACK - 1) * BLOCK + lane] = c_far;  // above the top of the stack unless pushed
    asm volatile("" : "+v"(top));  // the pop read stays unconditional (no branch around it)
    const bool any = h0 | h1;
    const int popped = sp > 0 ? top : -1;
    t.node = any ? c_near : popped;
    t.sp = any ? sp + (int)(h0 & h1) : sp_pop;
}

// NF 6: node_step8 over QNode2 with the top LC nodes (the top node and the scene tree's
// breadth-first prefix, bfs_prefix_order) held in LDS: those lanes read the node from LDS, the
// others from memory, so the vector-memory data path (TD, ~90 % busy) carries only the deeper
// steps.  The two reads are exec-masked (one branch pair per step).
template <int BLOCK, int STACK, int LC>
__device__ __forceinline__ void node_step8c(const Ray& r, float oix, float oiy, float oiz, Trav3& t,
                                            int* __restrict__ stk, int lane, __amdgpu_buffer_rsrc_t rs,
                                            const uint4* __restrict__ lcache) {
    const int sp = t.sp;
    const int sp_pop = max(sp - 1, 0);
    int top = stk[sp_pop * BLOCK + lane];
    const float ix = r.inv[0], iy = r.inv[1], iz = r.inv[2];
    uint4 A, B;
    if (t.node < LC) {
        A = lcache[2 * t.node];
        B = lcache[2 * t.node + 1];
    } else {
        const int off = t.node * (int)sizeof(QNode2);
        A = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
        B = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off + 16, 0, 0));
    }
    const float4 na = make_float4((float)(A.x & 0xffffu), (float)(A.x >> 16), (float)(A.y & 0xffffu), (float)(A.y >> 16));
    const float4 nb = make_float4((float)(B.x & 0xffffu), (float)(B.x >> 16), (float)(B.y & 0xffffu), (float)(B.y >> 16));
    const float4 nc = make_float4((float)(A.z & 0xffffu), (float)(A.z >> 16), (float)(B.z & 0xffffu), (float)(B.z >> 16));
    const int c0 = (int)A.w, c1 = (int)B.w;
    const float x00 = __builtin_fmaf(na.x, ix, -oix), x01 = __builtin_fmaf(na.y, ix, -oix);
    const float y00 = __builtin_fmaf(na.z, iy, -oiy), y01 = __builtin_fmaf(na.w, iy, -oiy);
    const float z00 = __builtin_fmaf(nc.x, iz, -oiz), z01 = __builtin_fmaf(nc.y, iz, -oiz);
    const float x10 = __builtin_fmaf(nb.x, ix, -oix), x11 = __builtin_fmaf(nb.y, ix, -oix);
    const float y10 = __builtin_fmaf(nb.z, iy, -oiy), y11 = __builtin_fmaf(nb.w, iy, -oiy);
    const float z10 = __builtin_fmaf(nc.z, iz, -oiz), z11 = __builtin_fmaf(nc.w, iz, -oiz);
    const float tn0 = fmaxf(fmaxf(fminf(x00, x01), fminf(y00, y01)), fmaxf(fminf(z00, z01), 0.0f));
    const float tf0 = fminf(fminf(fmaxf(x00, x01), fmaxf(y00, y01)), fminf(fmaxf(z00, z01), t.best_t));
    const float tn1 = fmaxf(fmaxf(fminf(x10, x11), fminf(y10, y11)), fmaxf(fminf(z10, z11), 0.0f));
    const float tf1 = fminf(fminf(fmaxf(x10, x11), fmaxf(y10, y11)), fminf(fmaxf(z10, z11), t.best_t));
    const bool h0 = tn0 <= tf0, h1 = tn1 <= tf1;
    const bool near1 = h1 & (!h0 | (tn1 < tn0));
    const int c_near = near1 ? c1 : c0;
    const int c_far = near1 ? c0 : c1;
    stk[min(sp, STACK - 1) * BLOCK + lane] = c_far;
    asm volatile("" : "+v"(top));
    const bool any = h0 | h1;
    const int popped = sp > 0 ? top : -1;
    t.node = any ? c_near : popped;
    t.sp = any ? sp + (int)(h0 & h1) : sp_pop;
}

// NF 3: pair-cooperative fetch of QNode2 nodes.  The vector-memory data path is charged per
// distinct 64-B block per wave-instruction (td_microbench), and two per-lane 16-B loads of a
// 32-B node touch 2 x 64 blocks per step.  Here lane pair (2p, 2p+1) fetches its two nodes
// together: load 0 brings each lane its own node's child (lane & 1), load 1 the partner node's
// child (lane & 1) -- the half the partner is missing -- and one DPP swap hands it over, so
// each load touches 32 blocks.  The two children are then tested symmetrically ("mine" = the
// child this lane loaded, "other" = the swapped one; their codes travel with them), so the
// order of a tie between equally near children depends on the lane's parity: the closest hit,
// a minimum over every triangle not culled, does not.  Runs with the whole wave active (the
// partner may need this lane's load); lanes without a step (go false) fetch node 0 and keep
// their state.
__device__ __forceinline__ int swap_pair(int v) { return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false); }

template <int BLOCK, int STACK>
__device__ __forceinline__ void node_step8p(const Ray& r, float oix, float oiy, float oiz, Trav3& t,
                                            int* __restrict__ stk, int lane, __amdgpu_buffer_rsrc_t rs, bool go,
                                            int half) {
    const int sp = t.sp;
    const int sp_pop = max(sp - 1, 0);
    int top = stk[sp_pop * BLOCK + lane];  // pop candidate first (see node_step8)
    const int me = max(t.node, 0);
    const int pn = swap_pair(me);
    const uint4 D0 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, me * (int)sizeof(QNode2) + half, 0, 0));
    const uint4 D1 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, pn * (int)sizeof(QNode2) + half, 0, 0));
    uint4 Y;
    Y.x = (uint32_t)swap_pair((int)D1.x);
    Y.y = (uint32_t)swap_pair((int)D1.y);
    Y.z = (uint32_t)swap_pair((int)D1.z);
    Y.w = (uint32_t)swap_pair((int)D1.w);
    const float ix = r.inv[0], iy = r.inv[1], iz = r.inv[2];
    const float xa0 = __builtin_fmaf((float)(D0.x & 0xffffu), ix, -oix), xa1 = __builtin_fmaf((float)(D0.x >> 16), ix, -oix);
    const float ya0 = __builtin_fmaf((float)(D0.y & 0xffffu), iy, -oiy), ya1 = __builtin_fmaf((float)(D0.y >> 16), iy, -oiy);
    const float za0 = __builtin_fmaf((float)(D0.z & 0xffffu), iz, -oiz), za1 = __builtin_fmaf((float)(D0.z >> 16), iz, -oiz);
    const float xb0 = __builtin_fmaf((float)(Y.x & 0xffffu), ix, -oix), xb1 = __builtin_fmaf((float)(Y.x >> 16), ix, -oix);
    const float yb0 = __builtin_fmaf((float)(Y.y & 0xffffu), iy, -oiy), yb1 = __builtin_fmaf((float)(Y.y >> 16), iy, -oiy);
    const float zb0 = __builtin_fmaf((float)(Y.z & 0xffffu), iz, -oiz), zb1 = __builtin_fmaf((float)(Y.z >> 16), iz, -oiz);
    const float tna = fmaxf(fmaxf(fminf(xa0, xa1), fminf(ya0, ya1)), fmaxf(fminf(za0, za1), 0.0f));
    const float tfa = fminf(fminf(fmaxf(xa0, xa1), fmaxf(ya0, ya1)), fminf(fmaxf(za0, za1), t.best_t));
    const float tnb = fmaxf(fmaxf(fminf(xb0, xb1), fminf(yb0, yb1)), fmaxf(fminf(zb0, zb1), 0.0f));
    const float tfb = fminf(fminf(fmaxf(xb0, xb1), fmaxf(yb0, yb1)), fminf(fmaxf(zb0, zb1), t.best_t));
    const int ca = (int)D0.w, cb = (int)Y.w;
    const bool ha = go & (tna <= tfa), hb = go & (tnb <= tfb);
    const bool nearb = hb & (!ha | (tnb < tna));
    const int c_near = nearb ? cb : ca;
    const int c_far = nearb ? ca : cb;
    stk[min(sp, STACK - 1) * BLOCK + lane] = c_far;  // above the top of the stack unless pushed
    asm volatile("" : "+v"(top));
    const bool any = ha | hb;
    const int popped = sp > 0 ? top : -1;
    const int nn = any ? c_near : popped;
    const int ns = any ? sp + (int)(ha & hb) : sp_pop;
    t.node = go ? nn : t.node;
    t.sp = go ? ns : t.sp;
}

// Leaf phase of v5: test the pending leaf, then pop the next entry.
template <int BLOCK, int LV>
__device__ __forceinline__ void leaf_step8(const TraceArgs& a, const Ray& r, Trav3& t, const int* __restrict__ stk,
                                           int lane) {
    const int v = ~t.node;
    if constexpr (LV == 0) {  // buffer loads: 32-bit offsets off a scalar base (no 64-bit address math)
        const __amdgpu_buffer_rsrc_t trs =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<TriRec*>(a.tris), (short)0, 0x7fffffff, 0x00020000);
        const int first = v >> 4, count = v & 15;
        for (int k = 0; k < count; ++k) {
            const int off = (first + k) * (int)sizeof(TriRec);
            const float4 p0 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(trs, off, 0, 0));
            const float4 p1 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(trs, off + 16, 0, 0));
            const float4 p2 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(trs, off + 32, 0, 0));
            Hit h;
            if (tri_test(r, p0, p1, p2, h)) {
                const int id = __float_as_int(p1.w);
                if (h.t < t.best_t || (h.t == t.best_t && id < t.best_id)) {
                    t.best_t = h.t;
                    t.best_id = id;
                    t.best = first + k;
                }
            }
        }
    } else {
        leaf_hits_vec<LV>(a.tris, r, v >> 4, v & 15, t.best_t, t.best_id, t.best);
    }
    const int sp = t.sp;
    const int sp_pop = max(sp - 1, 0);
    int top = stk[sp_pop * BLOCK + lane];
    asm volatile("" : "+v"(top));
    t.node = sp > 0 ? top : -1;
    t.sp = sp_pop;
}

// Persistent waves as v3 (static per-wave ray ranges, direction pre-pass, refill at THRESH
// idle lanes, postponed leaves) over node_step8: NSTEPS guarded steps per inner iteration.
// POOL > 0: the last POOL percent of the rays form a shared pool that waves done with their
// static range take from in refill-sized pieces (one atomic per refill, only near the end), so
// waves whose rays ran long do not hold the launch open while others idle.
// TAIL > 0: once the wave's rays are all handed out, the shading threshold drops from THRESH to
// (live rays) / TAIL (at least 1), so finished queries of the last rays are shaded and
// re-issued promptly instead of waiting for THRESH idle lanes that will never come.
// DIET = 2: only the counters below.  DIET = 1: fewer VGPRs held across the traversal loop, for 6 waves per SIMD: the ray state
// (position, direction, energy, distance, depth) is kept in a per-lane 48-B record of a.stash[0]
// from the query's setup to its shading instead of in registers, and the query / receiver /
// miss counters are wave-level (scalar) sums of ballots.
template <int BLOCK, int STACK, int THRESH, int LEAF_THRESH, int MINW, int NSTEPS, int NF, int LV = 1, int POOL = 0,
          int TAIL = 0, int LC = 0, int DIET = 0>
__global__ __launch_bounds__(BLOCK, MINW) void trace_kernel_v5(TraceArgs a) {
    constexpr int FMT = NF & 15;
    constexpr bool Q16 = FMT >= 1;
    // STACK rows: sp <= bvh_depth < STACK (launch_v5), so the unconditional write to slot sp
    // stays in the array
    // NF 6: LC cached nodes (8 ints each) after the stack rows
    __shared__ int stk[STACK * BLOCK + (FMT == 6 ? 8 * LC : 0)];
    const __amdgpu_buffer_rsrc_t nrs =
        FMT == 5 ? __builtin_amdgcn_make_buffer_rsrc(const_cast<QWide4*>(a.qwnodes), (short)0, 0x7fffffff, 0x00020000)
        : Q16    ? __builtin_amdgcn_make_buffer_rsrc(const_cast<QNode2*>(a.qnodes), (short)0, 0x7fffffff, 0x00020000)
                 : node_rsrc(a.cnodes);
    const int lane = threadIdx.x;
    const uint64_t n = a.ray_end - a.ray_begin;
    const uint64_t n_static = POOL > 0 ? n - n * (uint64_t)POOL / 100 : n;  // [n_static, n): the pool
    const uint32_t wave_id = __builtin_amdgcn_readfirstlane((blockIdx.x * BLOCK + threadIdx.x) >> 6);
    const uint32_t n_waves = gridDim.x * (BLOCK / 64);
    uint64_t w_next = n_static * wave_id / n_waves;
    uint64_t w_end = n_static * (wave_id + 1) / n_waves;
    bool pool = false;  // this wave has moved on to the shared pool
    unsigned long long* const cursor = a.counters + 4;
    uint32_t n_q = 0, n_rx = 0, n_miss = 0;
    bool overflow = false;  // impossible by construction for node_step8; NF 5 checks it
    bool active = false, trav = false, exhausted = POOL > 0 ? false : w_next >= w_end;
    RayState s;
    s.depth = -1;
    Ray r;
    Trav3 t;
    t.best_t = __builtin_huge_valf();
    t.best_id = 0x7fffffff;
    t.best = -1;
    t.node = -1;
    t.sp = 0;
    t.pf = 0;
    t.pc = 0;
    t.visits = 0;
    float oix = 0.f, oiy = 0.f, oiz = 0.f;
    int obase = 0;  // NF 2: byte offset of the ray's octant copy
    uint4* const lcache = reinterpret_cast<uint4*>(stk + STACK * BLOCK);
    uint32_t wq = 0, wrx = 0, wms = 0;  // DIET: wave-level counters
    float4* const srec = reinterpret_cast<float4*>(a.stash[0]) + (size_t)3 * (blockIdx.x * BLOCK + threadIdx.x);
    if constexpr (FMT == 6) {  // the top LC nodes (a.qcount valid ones) into LDS
        for (int i = lane; i < 2 * LC; i += BLOCK) {
            uint4 v = make_uint4(0u, 0u, 0u, 0u);
            if ((uint32_t)(i >> 1) < a.qcount)
                v = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(nrs, i * 16, 0, 0));
            lcache[i] = v;
        }
        __syncthreads();
    }
    while (true) {
        if constexpr (DIET == 2) {  // scalar counters only
            uint32_t rx = 0, ms = 0;
            if (active && !trav) {
                shade(a, s, r, t.best, rx, ms);
                if (!wants_query(a, s)) active = false;
            }
            wrx += (uint32_t)__popcll(__ballot(rx != 0));
            wms += (uint32_t)__popcll(__ballot(ms != 0));
        } else if constexpr (DIET == 1) {  // the ray state of every lane back from its record (stored at setup)
            const float4 A = srec[0], B = srec[1], C = srec[2];
            s.pos = make_float3(A.x, A.y, A.z);
            s.e = A.w;
            s.dir = make_float3(B.x, B.y, B.z);
            s.dist = B.w;
            s.depth = __float_as_int(C.x);
            uint32_t rx = 0, ms = 0;
            if (active && !trav) {
                shade(a, s, r, t.best, rx, ms);
                if (!wants_query(a, s)) active = false;
            }
            wrx += (uint32_t)__popcll(__ballot(rx != 0));
            wms += (uint32_t)__popcll(__ballot(ms != 0));
        } else if (active && !trav) {
            shade(a, s, r, t.best, n_rx, n_miss);
            if (!wants_query(a, s)) active = false;
        }
        const unsigned long long need = __ballot(!active);
        if (need != 0ull && !exhausted) {
            const int cnt = __popcll(need);
            if (POOL > 0 && !pool && w_next >= w_end) pool = true;
            uint64_t base = w_next;
            if (POOL > 0 && pool) {  // one atomic per refill, wave-uniform result
                const int leader = __ffsll((unsigned long long)need) - 1;
                unsigned long long got = 0;
                if ((lane & 63) == leader) got = atomicAdd(cursor, (unsigned long long)cnt);
                const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)got, leader);
                const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(got >> 32), leader);
                base = n_static + (((uint64_t)hi << 32) | lo);
                w_end = n;
            } else {
                w_next += (uint64_t)cnt;
            }
            if (!active) {
                const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(need >> 32),
                                                                __builtin_amdgcn_mbcnt_lo((uint32_t)need, 0u));
                const uint64_t i = base + rank;
                if (i < w_end) {
                    ray_init(a, s, a.ray_begin + i);
                    active = wants_query(a, s);
                }
            }
            if (base + (uint64_t)cnt >= w_end && (POOL == 0 || pool)) exhausted = true;
        }
        if constexpr (DIET) wq += (uint32_t)__popcll(__ballot(active && !trav));
        if (active && !trav) {
            if constexpr (!DIET) ++n_q;
            setup_ray(r, s.pos, s.dir);
            if constexpr (DIET == 1) {
                srec[0] = make_float4(s.pos.x, s.pos.y, s.pos.z, s.e);
                srec[1] = make_float4(s.dir.x, s.dir.y, s.dir.z, s.dist);
                srec[2] = make_float4(__int_as_float(s.depth), 0.0f, 0.0f, 0.0f);
            }
            if constexpr (Q16) {  // grid form of the slab planes (node_step7 Q16)
                oix = (r.o[0] - a.qgrid.origin[0]) * r.inv[0];
                oiy = (r.o[1] - a.qgrid.origin[1]) * r.inv[1];
                oiz = (r.o[2] - a.qgrid.origin[2]) * r.inv[2];
                r.inv[0] *= a.qgrid.scale[0];
                r.inv[1] *= a.qgrid.scale[1];
                r.inv[2] *= a.qgrid.scale[2];
                if constexpr (FMT == 2) {
                    const int oct = (r.inv[0] < 0.0f ? 1 : 0) | (r.inv[1] < 0.0f ? 2 : 0) | (r.inv[2] < 0.0f ? 4 : 0);
                    obase = oct * (int)a.qostride * (int)sizeof(QNode2);
                }
            } else {
                oix = r.o[0] * r.inv[0];
                oiy = r.o[1] * r.inv[1];
                oiz = r.o[2] * r.inv[2];
            }
            t.best_t = __builtin_huge_valf();
            t.best_id = 0x7fffffff;
            t.best = -1;
            t.node = 0;
            t.sp = 0;
            trav = true;
        }
        if (__ballot(active) == 0ull) {
            if (exhausted) break;
            continue;
        }
        while (true) {
            if (trav && t.node == -1) trav = false;  // query done (its stack is empty)
            const unsigned long long m_node = __ballot(t.node >= 0);
            const unsigned long long m_leaf = __ballot(t.node <= -2);
            if ((m_node | m_leaf) == 0ull) break;
            int thr = THRESH;
            if constexpr (TAIL > 0) {
                if (exhausted) thr = min(THRESH, max(1, (int)__popcll(__ballot(active)) / TAIL));
            }
            if (__popcll(__ballot(active && !trav)) >= thr) break;
            if (m_node != 0ull && __popcll(m_leaf) < LEAF_THRESH) {
                if constexpr (FMT == 3) {  // whole-wave steps (pair-cooperative fetch)
                    const int half = (lane & 1) * (int)sizeof(QChild);
#pragma unroll
                    for (int k = 0; k < NSTEPS; ++k) {
                        const bool go = t.node >= 0;
                        if (__ballot(go) == 0ull) break;
                        node_step8p<BLOCK, STACK>(r, oix, oiy, oiz, t, stk, lane, nrs, go, half);
                    }
                } else if constexpr (FMT == 6) {
#pragma unroll
                    for (int k = 0; k < NSTEPS; ++k)
                        if (t.node >= 0) node_step8c<BLOCK, STACK, LC>(r, oix, oiy, oiz, t, stk, lane, nrs, lcache);
                } else if constexpr (FMT == 5) {
#pragma unroll
                    for (int k = 0; k < NSTEPS; ++k)
                        if (t.node >= 0) node_step8w<BLOCK, STACK, NF>(r, oix, oiy, oiz, t, stk, lane, nrs, overflow);
                } else {
#pragma unroll
                    for (int k = 0; k < NSTEPS; ++k)
                        if (t.node >= 0) node_step8<BLOCK, STACK, NF>(r, oix, oiy, oiz, t, stk, lane, nrs, obase);
                }
            } else if (t.node <= -2) {
                leaf_step8<BLOCK, LV>(a, r, t, stk, lane);
            }
        }
    }
    if constexpr (DIET) {
        const bool l0 = (lane & 63) == 0;
        flush_counters(a, l0 ? wq : 0u, l0 ? wrx : 0u, l0 ? wms : 0u, overflow, lane);
    } else {
        flush_counters(a, n_q, n_rx, n_miss, overflow, lane);
    }
}

// ---------------------------------------------------------------- wide tree (v4) ---
// Same persistent-wave scheme as v3 over W-wide nodes (W = 4: one 128-B line per node):
// the dependent node-fetch chain per query is about half (W=4) or a third (W=8) of BVH2's.
// Per node step all W child boxes are tested (their planes arrive as SoA float4s), the hit
// children are sorted by entry distance with a sorting network, the nearest inner child is
// visited next, the nearest leaf is parked as the pending leaf, and the rest are pushed far
// to near.  The stack keeps S entries per lane in LDS and spills deeper entries to a
// per-lane global region sized on the host for the tree's worst case.
__device__ __forceinline__ void cswap(float& ka, int& va, float& kb, int& vb) {
    const bool sw = kb < ka;
    const float k = sw ? kb : ka;
    const int v = sw ? vb : va;
    kb = sw ? ka : kb;
    vb = sw ? va : vb;
    ka = k;
    va = v;
}

template <int W>
__device__ __forceinline__ void sort_children(float* k, int* v) {
    if constexpr (W == 4) {
        cswap(k[0], v[0], k[1], v[1]);
        cswap(k[2], v[2], k[3], v[3]);
        cswap(k[0], v[0], k[2], v[2]);
        cswap(k[1], v[1], k[3], v[3]);
        cswap(k[1], v[1], k[2], v[2]);
    } else {  // Batcher's 8-input network, 19 comparators
        cswap(k[0], v[0], k[1], v[1]); cswap(k[2], v[2], k[3], v[3]);
        cswap(k[4], v[4], k[5], v[5]); cswap(k[6], v[6], k[7], v[7]);
        cswap(k[0], v[0], k[2], v[2]); cswap(k[1], v[1], k[3], v[3]);
        cswap(k[4], v[4], k[6], v[6]); cswap(k[5], v[5], k[7], v[7]);
        cswap(k[1], v[1], k[2], v[2]); cswap(k[5], v[5], k[6], v[6]);
        cswap(k[0], v[0], k[4], v[4]); cswap(k[1], v[1], k[5], v[5]);
        cswap(k[2], v[2], k[6], v[6]); cswap(k[3], v[3], k[7], v[7]);
        cswap(k[2], v[2], k[4], v[4]); cswap(k[3], v[3], k[5], v[5]);
        cswap(k[1], v[1], k[2], v[2]); cswap(k[3], v[3], k[4], v[4]);
        cswap(k[5], v[5], k[6], v[6]);
    }
}

// NF 5: branch-free step over 4-wide quantized nodes (QWide4, 64 B = four 16-B child records):
// about half the dependent node fetches of the binary tree per query.  All four child slabs are
// tested, the hit children sorted by entry distance (misses keyed +inf), the nearest becomes the
// next entry and the other hits are written far to near above the top of the stack.  The three
// slot writes are unconditional and issued from the highest slot down, so a write clamped to
// row STACK - 1 is overwritten by the valid one.  The stack holds up to three entries per wide
// level, more than STACK for the deepest trees: *ovf is set if a push would leave the array
// (the host then reports the overflow).
__device__ __forceinline__ void qchild_slab(uint4 c, float ix, float iy, float iz, float oix, float oiy, float oiz,
                                            float best_t, float& key, int& code, int& hit) {
    const float x0 = __builtin_fmaf((float)(c.x & 0xffffu), ix, -oix), x1 = __builtin_fmaf((float)(c.x >> 16), ix, -oix);
    const float y0 = __builtin_fmaf((float)(c.y & 0xffffu), iy, -oiy), y1 = __builtin_fmaf((float)(c.y >> 16), iy, -oiy);
    const float z0 = __builtin_fmaf((float)(c.z & 0xffffu), iz, -oiz), z1 = __builtin_fmaf((float)(c.z >> 16), iz, -oiz);
    const float tn = fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fmaxf(fminf(z0, z1), 0.0f));
    const float tf = fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fminf(fmaxf(z0, z1), best_t));
    const bool h = tn <= tf;
    key = h ? tn : __builtin_huge_valf();
    code = (int)c.w;
    hit = (int)h;
}

template <int BLOCK, int STACK, int NF>
__device__ __forceinline__ void node_step8w(const Ray& r, float oix, float oiy, float oiz, Trav3& t,
                                            int* __restrict__ stk, int lane, __amdgpu_buffer_rsrc_t rs, bool& ovf) {
    constexpr int CP = NF >> 4;
    const int sp = t.sp;
    const int sp_pop = max(sp - 1, 0);
    int top = stk[sp_pop * BLOCK + lane];
    const int off = t.node * (int)sizeof(QWide4);
    const uint4 A = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, CP));
    const uint4 B = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off + 16, 0, CP));
    const uint4 C = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off + 32, 0, CP));
    const uint4 D = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off + 48, 0, CP));
    const float ix = r.inv[0], iy = r.inv[1], iz = r.inv[2];
    float k[4];
    int v[4], h[4];
    qchild_slab(A, ix, iy, iz, oix, oiy, oiz, t.best_t, k[0], v[0], h[0]);
    qchild_slab(B, ix, iy, iz, oix, oiy, oiz, t.best_t, k[1], v[1], h[1]);
    qchild_slab(C, ix, iy, iz, oix, oiy, oiz, t.best_t, k[2], v[2], h[2]);
    qchild_slab(D, ix, iy, iz, oix, oiy, oiz, t.best_t, k[3], v[3], h[3]);
    const int nh = h[0] + h[1] + h[2] + h[3];
    sort_children<4>(k, v);
    const int s0 = nh == 4 ? v[3] : (nh == 3 ? v[2] : v[1]);
    const int s1 = nh == 4 ? v[2] : v[1];
    stk[min(sp + 2, STACK - 1) * BLOCK + lane] = v[1];
    stk[min(sp + 1, STACK - 1) * BLOCK + lane] = s1;
    stk[min(sp, STACK - 1) * BLOCK + lane] = s0;
    asm volatile("" : "+v"(top));
    const bool any = nh > 0;
    const int popped = sp > 0 ? top : -1;
    const int ns = sp + nh - 1;
    ovf = ovf | (ns > STACK);
    t.node = any ? v[0] : popped;
    t.sp = any ? ns : sp_pop;
}

template <int W, int BLOCK, int S>
__device__ __forceinline__ void node_step_w(const TraceArgs& a, const Ray& r, float oix, float oiy, float oiz, Trav3& t,
                                            int* __restrict__ stk, int lane, uint32_t gid, bool& overflow) {
    if (t.node < 0) {  // pop
        const int e = popw<BLOCK, S>(a, t, stk, lane, gid);
        if (e >= 0) {
            t.node = e;
        } else {
            const int v = -e - 1;
            t.pf = v >> 4;
            t.pc = v & 15;
            return;
        }
    }
    if (++t.visits > a.max_visits) {  // malformed tree guard: end the query, flag the launch
        overflow = true;
        t.node = -1;
        t.sp = 0;
        return;
    }
    const float4* np = reinterpret_cast<const float4*>(reinterpret_cast<const WideNode<W>*>(a.wnodes) + t.node);
    constexpr int Q = W / 4;  // float4s per plane array
    float lx[W], hx[W], ly[W], hy[W], lz[W], hz[W];
    int ref[W], cnt[W];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const float4 v0 = np[0 * Q + q], v1 = np[1 * Q + q], v2 = np[2 * Q + q];
        const float4 v3 = np[3 * Q + q], v4 = np[4 * Q + q], v5 = np[5 * Q + q];
        const int4 v6 = *reinterpret_cast<const int4*>(np + 6 * Q + q);
        const int4 v7 = *reinterpret_cast<const int4*>(np + 7 * Q + q);
        lx[4 * q + 0] = v0.x; lx[4 * q + 1] = v0.y; lx[4 * q + 2] = v0.z; lx[4 * q + 3] = v0.w;
        hx[4 * q + 0] = v1.x; hx[4 * q + 1] = v1.y; hx[4 * q + 2] = v1.z; hx[4 * q + 3] = v1.w;
        ly[4 * q + 0] = v2.x; ly[4 * q + 1] = v2.y; ly[4 * q + 2] = v2.z; ly[4 * q + 3] = v2.w;
        hy[4 * q + 0] = v3.x; hy[4 * q + 1] = v3.y; hy[4 * q + 2] = v3.z; hy[4 * q + 3] = v3.w;
        lz[4 * q + 0] = v4.x; lz[4 * q + 1] = v4.y; lz[4 * q + 2] = v4.z; lz[4 * q + 3] = v4.w;
        hz[4 * q + 0] = v5.x; hz[4 * q + 1] = v5.y; hz[4 * q + 2] = v5.z; hz[4 * q + 3] = v5.w;
        ref[4 * q + 0] = v6.x; ref[4 * q + 1] = v6.y; ref[4 * q + 2] = v6.z; ref[4 * q + 3] = v6.w;
        cnt[4 * q + 0] = v7.x; cnt[4 * q + 1] = v7.y; cnt[4 * q + 2] = v7.z; cnt[4 * q + 3] = v7.w;
    }
    const float ix = r.inv[0], iy = r.inv[1], iz = r.inv[2];
    const float inf = __builtin_huge_valf();
    float key[W];
    int code[W];
#pragma unroll
    for (int c = 0; c < W; ++c) {
        const float x0 = __builtin_fmaf(lx[c], ix, -oix), x1 = __builtin_fmaf(hx[c], ix, -oix);
        const float y0 = __builtin_fmaf(ly[c], iy, -oiy), y1 = __builtin_fmaf(hy[c], iy, -oiy);
        const float z0 = __builtin_fmaf(lz[c], iz, -oiz), z1 = __builtin_fmaf(hz[c], iz, -oiz);
        const float tn = fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fmaxf(fminf(z0, z1), 0.0f));
        const float tf = fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fminf(fmaxf(z0, z1), t.best_t));
        const bool hit = tn <= tf && cnt[c] >= 0;
        key[c] = hit ? tn : inf;
        code[c] = cnt[c] > 0 ? leaf_code(ref[c], cnt[c]) : ref[c];
    }
    sort_children<W>(key, code);
    // nearest inner child -> next node, nearest leaf -> pending; the rest pushed far to near
    int next = -1, leaf = 0;
    bool got_inner = false, got_leaf = false;
    bool skip[W];
#pragma unroll
    for (int j = 0; j < W; ++j) {
        const bool h = key[j] < inf;
        const bool take_inner = h && code[j] >= 0 && !got_inner;
        const bool take_leaf = h && code[j] < 0 && !got_leaf;
        next = take_inner ? code[j] : next;
        leaf = take_leaf ? code[j] : leaf;
        got_inner = got_inner || take_inner;
        got_leaf = got_leaf || take_leaf;
        skip[j] = !h || take_inner || take_leaf;
    }
#pragma unroll
    for (int j = W - 1; j >= 0; --j)
        if (!skip[j]) pushw<BLOCK, S>(a, t, stk, lane, gid, code[j], overflow);
    t.node = next;
    if (got_leaf) {
        const int v = -leaf - 1;
        t.pf = v >> 4;
        t.pc = v & 15;
    }
}

__device__ __forceinline__ float ubyte(uint32_t w, int c) { return (float)((w >> (8 * c)) & 0xFFu); }

// QNode4 step: plane t = fma(q, 2^e * inv, fma(origin, inv, -o*inv)), i.e. the same slab
// arithmetic as the f32 trees with the grid step folded into the reciprocal (2^e * inv is
// exact); quantized boxes enclose the padded boxes, so culling stays conservative.
template <int BLOCK, int S>
__device__ __forceinline__ void node_step_q4(const TraceArgs& a, const Ray& r, float oix, float oiy, float oiz,
                                             Trav3& t, int* __restrict__ stk, int lane, uint32_t gid, bool& overflow) {
    if (t.node < 0) {  // pop
        const int e = popw<BLOCK, S>(a, t, stk, lane, gid);
        if (e >= 0) {
            t.node = e;
        } else {
            const int v = -e - 1;
            t.pf = v >> 4;
            t.pc = v & 15;
            return;
        }
    }
    if (++t.visits > a.max_visits) {
        overflow = true;
        t.node = -1;
        t.sp = 0;
        return;
    }
    const uint4* np = reinterpret_cast<const uint4*>(reinterpret_cast<const QNode4*>(a.wnodes) + t.node);
    const uint4 h0 = np[0], h1 = np[1], h2 = np[2];
    const int4 rf = *reinterpret_cast<const int4*>(np + 3);
    const float ix = r.inv[0], iy = r.inv[1], iz = r.inv[2];
    const float sx = __uint_as_float((h0.w & 0xFFu) << 23) * ix;
    const float sy = __uint_as_float(((h0.w >> 8) & 0xFFu) << 23) * iy;
    const float sz = __uint_as_float(((h0.w >> 16) & 0xFFu) << 23) * iz;
    const float bx = __builtin_fmaf(__uint_as_float(h0.x), ix, -oix);
    const float by = __builtin_fmaf(__uint_as_float(h0.y), iy, -oiy);
    const float bz = __builtin_fmaf(__uint_as_float(h0.z), iz, -oiz);
    const float inf = __builtin_huge_valf();
    const int ref[4] = {rf.x, rf.y, rf.z, rf.w};
    float key[4];
    int code[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const float x0 = __builtin_fmaf(ubyte(h1.x, c), sx, bx), x1 = __builtin_fmaf(ubyte(h1.y, c), sx, bx);
        const float y0 = __builtin_fmaf(ubyte(h1.z, c), sy, by), y1 = __builtin_fmaf(ubyte(h1.w, c), sy, by);
        const float z0 = __builtin_fmaf(ubyte(h2.x, c), sz, bz), z1 = __builtin_fmaf(ubyte(h2.y, c), sz, bz);
        const float tn = fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fmaxf(fminf(z0, z1), 0.0f));
        const float tf = fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fminf(fmaxf(z0, z1), t.best_t));
        const int cnt = (int)((h2.z >> (8 * c)) & 0xFFu);
        const bool hit = tn <= tf && cnt != 0xFF;
        key[c] = hit ? tn : inf;
        code[c] = cnt > 0 ? leaf_code(ref[c], cnt) : ref[c];
    }
    sort_children<4>(key, code);
    int next = -1, leaf = 0;
    bool got_inner = false, got_leaf = false;
    bool skip[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const bool h = key[j] < inf;
        const bool take_inner = h && code[j] >= 0 && !got_inner;
        const bool take_leaf = h && code[j] < 0 && !got_leaf;
        next = take_inner ? code[j] : next;
        leaf = take_leaf ? code[j] : leaf;
        got_inner = got_inner || take_inner;
        got_leaf = got_leaf || take_leaf;
        skip[j] = !h || take_inner || take_leaf;
    }
#pragma unroll
    for (int j = 3; j >= 0; --j)
        if (!skip[j]) pushw<BLOCK, S>(a, t, stk, lane, gid, code[j], overflow);
    t.node = next;
    if (got_leaf) {
        const int v = -leaf - 1;
        t.pf = v >> 4;
        t.pc = v & 15;
    }
}

// W == kWideQ4 selects QNode4 trees
template <int W, int BLOCK, int S, int THRESH, int LEAF_THRESH, int MINW>
__global__ __launch_bounds__(BLOCK, MINW) void trace_kernel_w(TraceArgs a) {
    __shared__ int stk[S * BLOCK];
    const int lane = threadIdx.x;
    const uint32_t gid = blockIdx.x * BLOCK + threadIdx.x;
    const uint64_t n = a.ray_end - a.ray_begin;
    const uint32_t wave_id = __builtin_amdgcn_readfirstlane((blockIdx.x * BLOCK + threadIdx.x) >> 6);
    const uint32_t n_waves = gridDim.x * (BLOCK / 64);
    uint64_t w_next = n * wave_id / n_waves;
    const uint64_t w_end = n * (wave_id + 1) / n_waves;
    unsigned long long* const cursor = a.counters + 4;
    uint32_t n_q = 0, n_rx = 0, n_miss = 0;
    bool overflow = false;
    bool active = false;
    bool trav = false;
    bool exhausted = false;
    RayState s;
    Ray r;
    Trav3 t;
    float oix = 0.f, oiy = 0.f, oiz = 0.f;
    s.depth = -1;
    t.best_t = __builtin_huge_valf();
    t.best_id = 0x7fffffff;
    t.best = -1;
    t.node = -1;
    t.sp = 0;
    t.pf = 0;
    t.pc = 0;
    t.visits = 0;
    while (true) {
        if (active && !trav) {
            shade(a, s, r, t.best, n_rx, n_miss);
            if (!wants_query(a, s)) active = false;
        }
        const unsigned long long need = __ballot(!active);
        if (need != 0ull && !exhausted) {
            const int cnt = __popcll(need);
            unsigned long long base = 0;
            uint64_t lim = n;
            if (a.static_ranges) {
                base = w_next;
                lim = w_end;
                w_next += (uint64_t)cnt;
            } else {
                const int leader = __ffsll((unsigned long long)need) - 1;
                if ((lane & 63) == leader) base = atomicAdd(cursor, (unsigned long long)cnt);
                const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)base, leader);
                const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(base >> 32), leader);
                base = ((unsigned long long)hi << 32) | lo;
            }
            if (!active) {
                const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(need >> 32),
                                                                __builtin_amdgcn_mbcnt_lo((uint32_t)need, 0u));
                const uint64_t i = base + rank;
                if (i < lim) {
                    ray_init(a, s, a.ray_begin + i);
                    active = wants_query(a, s);
                }
            }
            if (base + (unsigned long long)cnt >= lim) exhausted = true;
        }
        if (active && !trav) {
            ++n_q;
            setup_ray(r, s.pos, s.dir);
            oix = r.o[0] * r.inv[0];
            oiy = r.o[1] * r.inv[1];
            oiz = r.o[2] * r.inv[2];
            t.best_t = __builtin_huge_valf();
            t.best_id = 0x7fffffff;
            t.best = -1;
            t.node = 0;
            t.sp = 0;
            t.pc = 0;
            t.pf = 0;
            t.visits = 0;
            trav = true;
        }
        if (__ballot(active) == 0ull) {
            if (exhausted) break;
            continue;
        }
        while (true) {
            if (trav && t.pc == 0 && t.node < 0 && t.sp == 0) trav = false;  // query finished
            const bool can_node = trav && t.pc == 0;
            const unsigned long long m_node = __ballot(can_node);
            const unsigned long long m_leaf = __ballot(trav && t.pc > 0);
            if ((m_node | m_leaf) == 0ull) break;
            if (__popcll(__ballot(active && !trav)) >= THRESH) break;
            if (m_node != 0ull && __popcll(m_leaf) < LEAF_THRESH) {
                if (can_node) {
                    if constexpr (W == kWideQ4)
                        node_step_q4<BLOCK, S>(a, r, oix, oiy, oiz, t, stk, lane, gid, overflow);
                    else
                        node_step_w<W, BLOCK, S>(a, r, oix, oiy, oiz, t, stk, lane, gid, overflow);
                }
            } else if (trav && t.pc > 0) {
                leaf_hits(a.tris, r, t.pf, t.pc, t.best_t, t.best_id, t.best);
                t.pc = 0;
            }
        }
    }
    flush_counters(a, n_q, n_rx, n_miss, overflow, lane);
}

__global__ void finalize_ir_kernel(const long long* __restrict__ hist, float* __restrict__ L, float* __restrict__ R,
                                   int32_t ir_len, double unit, int32_t mono) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= ir_len) return;
    float l = (float)((double)hist[k] * unit);
    float r = (float)((double)hist[ir_len + k] * unit);
    if (mono) {  // addIRs (kernels.cu:519-527)
        const float s = l + r;
        l = s;
        r = s;
    }
    L[k] = l;
    R[k] = r;
}

// Direction pre-pass of the refill variants: float4(dir, 0) for rays [first, first + count).
__global__ void dirs_kernel(uint64_t seed, uint64_t first, uint64_t count, float4* out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const float3 d = ray_direction(seed, first + i);
    out[i] = make_float4(d.x, d.y, d.z, 0.0f);
}

__global__ void ray_dir_kernel(uint64_t seed, uint64_t first, uint64_t count, float* out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const float3 d = ray_direction(seed, first + i);
    out[3 * i + 0] = d.x;
    out[3 * i + 1] = d.y;
    out[3 * i + 2] = d.z;
}

}  // namespace

int trace_block_size() { return kBlock; }

namespace {
// Kernel variants for A/B measurement (ARX_TRACE_KERNEL, read per launch); all are
// bit-identical in results.  Default = the fastest measured on MI355X.
constexpr int kDefaultVariant = 0;  // 0 = variant 921 (see launch_trace's default)

template <typename K>
int persistent_grid(K kernel, int block, uint64_t n_rays, int cus) {
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, block, 0) != hipSuccess || per_cu <= 0) per_cu = 4;
    uint64_t want = (n_rays + block - 1) / block;
    uint64_t cap = (uint64_t)per_cu * (uint64_t)(cus > 0 ? cus : 256);
    if (const char* f = getenv("ARX_GRID_PCT")) {  // design experiments: a smaller persistent grid,
        const int pct = atoi(f);                   // or (> 100) fewer rays per lane in small launches
        if (pct > 0 && pct < 100) {
            cap = std::max<uint64_t>(1, cap * (uint64_t)pct / 100);
            want = std::max<uint64_t>(1, want * (uint64_t)pct / 100);
        }
        if (pct > 100) want = want * (uint64_t)pct / 100;
    }
    return (int)(want < cap ? (want > 0 ? want : 1) : cap);
}

template <int BLOCK, int THRESH>
hipError_t launch_v2(const TraceArgs& a, int cus, hipStream_t s) {
    hipError_t e = hipMemsetAsync(a.counters + 4, 0, sizeof(unsigned long long), s);  // ray cursor
    if (e != hipSuccess) return e;
    auto k = trace_kernel_v2<BLOCK, kStackDepth, THRESH>;
    const int grid = persistent_grid(k, BLOCK, a.ray_end - a.ray_begin, cus);
    hipLaunchKernelGGL(k, dim3(grid), dim3(BLOCK), 0, s, a);
    return hipGetLastError();
}
int env_int(const char* name, int def) {
    const char* v = getenv(name);
    return (v && v[0]) ? atoi(v) : def;
}

// Tail compaction: phase 0 traces fresh ray ids; once a wave runs dry it parks its in-flight
// rays (at query boundaries) into a stash and exits, and the next phase refills full waves from
// that stash.  The last phase runs to completion.  Counts live on the device, so the phases
// are enqueued back to back without host synchronisation; empty phases exit immediately.
template <int BLOCK, int THRESH, int LEAF_THRESH, int STACK = kStackDepth, int MINW = 1, bool DBG = false, int LV = 1,
          int NS = 3, int REFILL = 0, int MIG = 0>
hipError_t launch_v3(const TraceArgs& args, int cus, hipStream_t s) {
    TraceArgs a = args;
    // REFILL bit 0: directions from a pre-pass; bit 1: static per-wave ranges, bit 2 / 3 in
    // whole 64-ray chunks, spread / surplus first (see trace_kernel_v3)
    a.dirs = nullptr;
    a.static_ranges = (REFILL & 2) ? ((REFILL & 4) ? 2 : (REFILL & 8) ? 3 : 1) : 0;
    const uint64_t n_rays = a.ray_end - a.ray_begin;
    if ((REFILL & 1) && a.dirs_buf && n_rays <= a.dirs_cap && n_rays > 0) {
        const uint64_t g = (n_rays + 255) / 256;
        hipLaunchKernelGGL(dirs_kernel, dim3((unsigned)g), dim3(256), 0, s, a.seed, a.ray_begin, n_rays,
                           reinterpret_cast<float4*>(a.dirs_buf));
        a.dirs = a.dirs_buf;
    }
    if constexpr (NS >= 200) {  // quantized nodes unavailable (emitter off the grid): the f32 coded nodes
        if (!a.qnodes) return launch_v3<BLOCK, THRESH, LEAF_THRESH, STACK, MINW, DBG, LV, NS - 200, REFILL, MIG>(args, cus, s);
    }
    auto k = trace_kernel_v3<BLOCK, STACK, THRESH, LEAF_THRESH, MINW, DBG, LV, NS, MIG>;
    int grid = persistent_grid(k, BLOCK, a.ray_end - a.ray_begin, cus);
    if constexpr (NS % 200 >= 60) {  // STACK LDS entries, the rest of the worst case (bvh_depth) spills (NS >= 80 too)
        a.spill_depth = a.bvh_depth + 1 > STACK ? a.bvh_depth + 1 - STACK : 0;
        if (a.spill_depth > 0) {
            if (!a.spill) return hipErrorInvalidValue;
            const uint64_t max_grid = a.spill_lanes / BLOCK;  // every lane owns a spill column
            if ((uint64_t)grid > max_grid) grid = (int)max_grid;
            if (grid <= 0) return hipErrorInvalidValue;
        }
    }
    const int phases = (a.stash[0] && a.stash[1] && a.stash_count) ? std::max(1, env_int("ARX_PHASES", 1)) : 1;
    const int low = env_int("ARX_DRAIN_LOW", 32);
    if ((uint64_t)grid * BLOCK > a.stash_cap && phases > 1) return hipErrorInvalidValue;
    for (int p = 0; p < phases; ++p) {
        a.pool_from = p == 0 ? -1 : (p - 1) % 2;
        a.drain_low = (p + 1 < phases) ? low : 0;
        hipError_t e = hipMemsetAsync(a.counters + 4, 0, sizeof(unsigned long long), s);  // ray cursor
        if (e != hipSuccess) return e;
        if (a.drain_low > 0) {
            const int to = a.pool_from < 0 ? 0 : 1 - a.pool_from;
            e = hipMemsetAsync(a.stash_count + to, 0, sizeof(unsigned long long), s);
            if (e != hipSuccess) return e;
        }
        hipLaunchKernelGGL(k, dim3(grid), dim3(BLOCK), 0, s, a);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}
template <int W, int BLOCK, int S, int THRESH, int LEAF_THRESH, int MINW, int REFILL = 0>
hipError_t launch_w(TraceArgs a, int cus, hipStream_t s) {
    if (!a.wnodes) return hipErrorInvalidValue;
    a.dirs = nullptr;
    a.static_ranges = (REFILL & 2) ? 1 : 0;
    const uint64_t n_rays = a.ray_end - a.ray_begin;
    if ((REFILL & 1) && a.dirs_buf && n_rays <= a.dirs_cap && n_rays > 0) {
        const uint64_t g = (n_rays + 255) / 256;
        hipLaunchKernelGGL(dirs_kernel, dim3((unsigned)g), dim3(256), 0, s, a.seed, a.ray_begin, n_rays,
                           reinterpret_cast<float4*>(a.dirs_buf));
        a.dirs = a.dirs_buf;
    }
    hipError_t e = hipMemsetAsync(a.counters + 4, 0, sizeof(unsigned long long), s);  // ray cursor
    if (e != hipSuccess) return e;
    auto k = trace_kernel_w<W, BLOCK, S, THRESH, LEAF_THRESH, MINW>;
    int grid = persistent_grid(k, BLOCK, a.ray_end - a.ray_begin, cus);
    a.spill_depth = a.stack_need > S ? a.stack_need - S : 0;
    if (a.spill_depth > 0) {
        if (!a.spill) return hipErrorInvalidValue;
        const uint64_t max_grid = a.spill_lanes / BLOCK;  // every lane owns a spill column
        if ((uint64_t)grid > max_grid) grid = (int)max_grid;
        if (grid <= 0) return hipErrorInvalidValue;
    }
    hipLaunchKernelGGL(k, dim3(grid), dim3(BLOCK), 0, s, a);
    return hipGetLastError();
}
// v5 launcher: direction pre-pass + static per-wave ranges; trees deeper than the LDS stack
// take the spill-stack v3 kernel, quantized variants without a usable grid the f32 nodes.
template <int BLOCK, int STACK, int THRESH, int LEAF_THRESH, int MINW, int NSTEPS, int NF, int LV = 1, int POOL = 0,
          int TAIL = 0, int LC = 0, int DIET = 0>
hipError_t launch_v5(const TraceArgs& args, int cus, hipStream_t s) {
    if constexpr ((NF & 15) == 5) {  // 4-wide quantized: without its grid copy, the binary steps
        if (!args.qwnodes) return launch_v5<BLOCK, STACK, THRESH, LEAF_THRESH, MINW, 12, 1, LV, POOL, TAIL>(args, cus, s);
    } else if constexpr (NF >= 1) {
        if (!args.qnodes) return launch_v5<BLOCK, STACK, THRESH, LEAF_THRESH, MINW, NSTEPS, 0, LV, POOL, TAIL>(args, cus, s);
    }
    if ((NF & 15) != 5 && args.bvh_depth + 1 > STACK) return launch_v3<128, 12, 12, 28, 5, false, 1, 71, 3>(args, cus, s);
    TraceArgs a = args;
    a.static_ranges = 1;
    a.dirs = nullptr;
    const uint64_t n_rays = a.ray_end - a.ray_begin;
    if (a.dirs_buf && n_rays <= a.dirs_cap && n_rays > 0) {
        const uint64_t g = (n_rays + 255) / 256;
        hipLaunchKernelGGL(dirs_kernel, dim3((unsigned)g), dim3(256), 0, s, a.seed, a.ray_begin, n_rays,
                           reinterpret_cast<float4*>(a.dirs_buf));
        a.dirs = a.dirs_buf;
    }
    if constexpr (POOL > 0) {
        const hipError_t e = hipMemsetAsync(a.counters + 4, 0, sizeof(unsigned long long), s);  // pool cursor
        if (e != hipSuccess) return e;
    }
    auto k = trace_kernel_v5<BLOCK, STACK, THRESH, LEAF_THRESH, MINW, NSTEPS, NF, LV, POOL, TAIL, LC, DIET>;
    const int grid = persistent_grid(k, BLOCK, n_rays, cus);
    if (DIET == 1 && (!a.stash[0] || (uint64_t)grid * BLOCK > a.stash_cap))  // one ray-state record per lane
        return launch_v5<128, 28, 12, 12, 5, 12, 1>(args, cus, s);
    hipLaunchKernelGGL(k, dim3(grid), dim3(BLOCK), 0, s, a);
    return hipGetLastError();
}
}  // namespace

int trace_width() {
    const int v = trace_variant();
    if (v >= 300 && v < 310) return 4;
    if (v >= 310 && v < 320) return 8;
    if ((v >= 320 && v < 340) || (v >= 720 && v < 730)) return kWideQ4;
    if (v >= 1000 && v < 1020) return 4;  // QWide4 copy of the 4-wide tree (trace_kernel_v5 NF 5)
    return 2;
}

bool trace_octant_nodes() {
    const int v = trace_variant();
    return v >= 932 && v <= 937;
}

int trace_variant() {
    const char* v = getenv("ARX_TRACE_KERNEL");
    return (v && v[0]) ? atoi(v) : kDefaultVariant;
}

int trace_grid_size(uint64_t n_rays, int device_cus) {
    const uint64_t blocks = (n_rays + kBlock - 1) / kBlock;
    const uint64_t cap = (uint64_t)(device_cus > 0 ? device_cus : 256) * 16;
    return (int)(blocks < cap ? (blocks > 0 ? blocks : 1) : cap);
}

hipError_t launch_trace(const TraceArgs& a, int cus, hipStream_t s) {
    switch (trace_variant()) {
        case 1: {
            const int grid = trace_grid_size(a.ray_end - a.ray_begin, cus);
            hipLaunchKernelGGL((trace_kernel_v1<kBlock, kStackDepth>), dim3(grid), dim3(kBlock), 0, s, a);
            return hipGetLastError();
        }
        case 3: return launch_v2<128, 8>(a, cus, s);
        case 4: return launch_v2<128, 32>(a, cus, s);
        case 5: return launch_v2<64, 16>(a, cus, s);
        case 6: return launch_v2<256, 16>(a, cus, s);
        case 7: return launch_v2<64, 32>(a, cus, s);
        case 10: return launch_v3<128, 16, 32>(a, cus, s);
        case 11: return launch_v3<128, 16, 16>(a, cus, s);
        case 12: return launch_v3<128, 16, 48>(a, cus, s);
        case 13: return launch_v3<128, 8, 32>(a, cus, s);
        case 14: return launch_v3<64, 16, 32>(a, cus, s);
        case 15: return launch_v3<128, 32, 32>(a, cus, s);
        case 16: return launch_v3<128, 16, 8>(a, cus, s);
        case 17: return launch_v3<128, 16, 4>(a, cus, s);
        case 18: return launch_v3<128, 24, 12>(a, cus, s);
        case 19: return launch_v3<128, 16, 12, 32>(a, cus, s);
        case 20: return launch_v3<128, 16, 12, 32, 5>(a, cus, s);
        case 21: return launch_v3<64, 16, 12, 32, 5>(a, cus, s);
        case 22: return launch_v3<128, 16, 12, 32, 6>(a, cus, s);
        // sweep: 1TL = THRESH T*8, LEAF_THRESH L*4
        case 138: return launch_v3<128, 24, 8>(a, cus, s);
        case 144: return launch_v3<128, 32, 16>(a, cus, s);
        case 143: return launch_v3<128, 32, 12>(a, cus, s);
        case 142: return launch_v3<128, 32, 8>(a, cus, s);
        case 153: return launch_v3<128, 40, 12>(a, cus, s);
        case 152: return launch_v3<128, 40, 8>(a, cus, s);
        case 163: return launch_v3<128, 48, 12>(a, cus, s);
        case 162: return launch_v3<128, 48, 8>(a, cus, s);
        case 173: return launch_v3<128, 56, 12>(a, cus, s);
        case 201: return launch_v3<128, 32, 12, 32, 5>(a, cus, s);
        case 202: return launch_v3<64, 32, 12, 32, 5>(a, cus, s);
        case 203: return launch_v3<256, 32, 12, 32, 5>(a, cus, s);
        case 204: return launch_v3<64, 32, 12>(a, cus, s);
        case 205: return launch_v3<256, 32, 12>(a, cus, s);
        case 206: return launch_v3<128, 28, 12, 32, 5>(a, cus, s);
        case 207: return launch_v3<128, 32, 12, 28, 5>(a, cus, s);
        case 2: return launch_v2<128, 16>(a, cus, s);
        case 98: return launch_v3<128, 32, 12, 28, 5, true>(a, cus, s);  // utilisation counters
        // triangle loads of 2 / 4 leaf triangles in flight together
        case 400: return launch_v3<128, 32, 12, 28, 5, false, 2>(a, cus, s);
        case 401: return launch_v3<128, 32, 12, 28, 5, false, 4>(a, cus, s);
        case 402: return launch_v3<128, 32, 8, 28, 5, false, 2>(a, cus, s);
        case 403: return launch_v3<128, 32, 16, 28, 5, false, 2>(a, cus, s);
        case 404: return launch_v3<128, 24, 12, 28, 5, false, 2>(a, cus, s);
        case 405: return launch_v3<128, 32, 12, 28, 4, false, 2>(a, cus, s);
        // branch-free node step + uniform leaf loop (NS = 5)
        case 500: return launch_v3<128, 32, 12, 28, 5, false, 1, 5>(a, cus, s);
        case 501: return launch_v3<128, 32, 12, 28, 5, false, 2, 5>(a, cus, s);
        case 502: return launch_v3<128, 32, 8, 28, 5, false, 1, 5>(a, cus, s);
        case 503: return launch_v3<128, 32, 16, 28, 5, false, 1, 5>(a, cus, s);
        case 504: return launch_v3<128, 32, 24, 28, 5, false, 1, 5>(a, cus, s);
        case 505: return launch_v3<128, 32, 12, 28, 4, false, 1, 5>(a, cus, s);
        case 506: return launch_v3<128, 32, 12, 28, 6, false, 1, 5>(a, cus, s);
        case 507: return launch_v3<128, 24, 12, 28, 5, false, 1, 5>(a, cus, s);
        case 508: return launch_v3<128, 40, 12, 28, 5, false, 1, 5>(a, cus, s);
        case 509: return launch_v3<64, 32, 12, 28, 5, false, 1, 5>(a, cus, s);
        case 598: return launch_v3<128, 32, 12, 28, 5, true, 1, 5>(a, cus, s);  // instrumented
        // quad-cooperative node fetch (NS = 6)
        case 600: return launch_v3<128, 32, 12, 28, 5, false, 1, 6>(a, cus, s);
        case 601: return launch_v3<128, 32, 12, 28, 5, false, 2, 6>(a, cus, s);
        case 602: return launch_v3<128, 32, 8, 28, 5, false, 1, 6>(a, cus, s);
        case 603: return launch_v3<128, 32, 16, 28, 5, false, 1, 6>(a, cus, s);
        case 604: return launch_v3<128, 24, 12, 28, 5, false, 1, 6>(a, cus, s);
        case 605: return launch_v3<128, 40, 12, 28, 5, false, 1, 6>(a, cus, s);
        case 606: return launch_v3<128, 32, 12, 28, 4, false, 1, 6>(a, cus, s);
        case 607: return launch_v3<128, 32, 12, 28, 6, false, 1, 6>(a, cus, s);
        case 608: return launch_v3<64, 32, 12, 28, 5, false, 1, 6>(a, cus, s);
        case 698: return launch_v3<128, 32, 12, 28, 5, true, 1, 6>(a, cus, s);  // instrumented
        // refill: 701 pre-pass directions, 702 static ranges, 703 both; then THRESH retunes
        case 701: return launch_v3<128, 32, 12, 28, 5, false, 1, 3, 1>(a, cus, s);
        case 702: return launch_v3<128, 32, 12, 28, 5, false, 1, 3, 2>(a, cus, s);
        case 703: return launch_v3<128, 32, 12, 28, 5, false, 1, 3, 3>(a, cus, s);
        case 704: return launch_v3<128, 24, 12, 28, 5, false, 1, 3, 3>(a, cus, s);
        case 705: return launch_v3<128, 16, 12, 28, 5, false, 1, 3, 3>(a, cus, s);
        case 706: return launch_v3<128, 12, 12, 28, 5, false, 1, 3, 3>(a, cus, s);
        case 707: return launch_v3<128, 8, 12, 28, 5, false, 1, 3, 3>(a, cus, s);
        case 708: return launch_v3<128, 40, 12, 28, 5, false, 1, 3, 3>(a, cus, s);
        case 709: return launch_v3<128, 24, 8, 28, 5, false, 1, 3, 3>(a, cus, s);
        case 798: return launch_v3<128, 32, 12, 28, 5, true, 1, 3, 3>(a, cus, s);  // instrumented
        case 710: return launch_v3<128, 12, 8, 28, 5, false, 1, 3, 3>(a, cus, s);
        case 711: return launch_v3<128, 12, 16, 28, 5, false, 1, 3, 3>(a, cus, s);
        case 712: return launch_v3<128, 10, 12, 28, 5, false, 1, 3, 3>(a, cus, s);
        case 713: return launch_v3<128, 14, 12, 28, 5, false, 1, 3, 3>(a, cus, s);
        case 714: return launch_v3<128, 12, 12, 28, 5, false, 2, 3, 3>(a, cus, s);
        case 715: return launch_v3<128, 12, 6, 28, 5, false, 1, 3, 3>(a, cus, s);
        case 716: return launch_v3<64, 12, 12, 28, 5, false, 1, 3, 3>(a, cus, s);
        case 717: return launch_v3<128, 12, 12, 28, 5, false, 1, 3, 1>(a, cus, s);
        // quantized 4-wide + refill
        case 720: return launch_w<kWideQ4, 128, 24, 12, 12, 5, 3>(a, cus, s);
        case 721: return launch_w<kWideQ4, 128, 24, 16, 12, 5, 3>(a, cus, s);
        case 722: return launch_w<kWideQ4, 128, 24, 8, 12, 5, 3>(a, cus, s);
        case 723: return launch_w<kWideQ4, 128, 28, 12, 12, 5, 3>(a, cus, s);
        case 724: return launch_w<kWideQ4, 128, 24, 12, 8, 5, 3>(a, cus, s);
        case 725: return launch_w<kWideQ4, 128, 24, 12, 16, 5, 3>(a, cus, s);
        // packed slab FMAs (NS = 7) on the 706 configuration
        case 730: return launch_v3<128, 12, 12, 28, 5, false, 1, 7, 3>(a, cus, s);
        case 731: return launch_v3<128, 14, 12, 28, 5, false, 1, 7, 3>(a, cus, s);
        case 732: return launch_v3<128, 12, 12, 28, 5, false, 2, 7, 3>(a, cus, s);
        case 733: return launch_v3<128, 32, 12, 28, 5, false, 1, 7, 0>(a, cus, s);
        case 739: return launch_v3<128, 12, 12, 28, 5, true, 1, 7, 3>(a, cus, s);  // instrumented
        case 799: return launch_v3<128, 12, 12, 28, 5, true, 1, 3, 3>(a, cus, s);  // instrumented 706
        // block-level ray migration (MIG = park threshold), larger blocks
        case 800: return launch_v3<256, 12, 12, 28, 5, false, 1, 3, 3, 24>(a, cus, s);
        case 801: return launch_v3<512, 12, 12, 28, 5, false, 1, 3, 3, 24>(a, cus, s);
        case 802: return launch_v3<640, 12, 12, 28, 5, false, 1, 3, 3, 24>(a, cus, s);
        case 803: return launch_v3<512, 12, 12, 28, 5, false, 1, 3, 3, 32>(a, cus, s);
        case 804: return launch_v3<512, 12, 12, 28, 5, false, 1, 3, 3, 16>(a, cus, s);
        case 805: return launch_v3<640, 12, 12, 28, 5, false, 1, 3, 3, 40>(a, cus, s);
        case 806: return launch_v3<128, 12, 12, 28, 5, false, 1, 3, 3, 24>(a, cus, s);
        case 807: return launch_v3<512, 12, 12, 28, 5, false, 1, 3, 3, 0>(a, cus, s);
        case 808: return launch_v3<640, 12, 12, 28, 5, false, 1, 3, 3, 0>(a, cus, s);
        case 810: return launch_v3<320, 12, 12, 28, 5, false, 1, 3, 3, 24>(a, cus, s);
        case 811: return launch_v3<320, 12, 12, 28, 5, false, 1, 3, 3, 0>(a, cus, s);
        case 812: return launch_v3<384, 12, 12, 28, 5, false, 1, 3, 3, 24>(a, cus, s);
        case 813: return launch_v3<384, 12, 12, 28, 5, false, 1, 3, 3, 0>(a, cus, s);
        case 814: return launch_v3<256, 12, 12, 28, 5, false, 1, 3, 3, 0>(a, cus, s);
        case 815: return launch_v3<320, 12, 12, 28, 5, false, 1, 3, 3, 32>(a, cus, s);
        case 816: return launch_v3<320, 12, 12, 28, 5, false, 1, 3, 3, 16>(a, cus, s);
        case 817: return launch_v3<320, 16, 12, 28, 5, false, 1, 3, 3, 24>(a, cus, s);
        case 898: return launch_v3<320, 12, 12, 28, 5, true, 1, 3, 3, 24>(a, cus, s);  // instrumented
        // two node steps per inner iteration (NS = 8)
        case 740: return launch_v3<128, 12, 12, 28, 5, false, 1, 8, 3>(a, cus, s);
        case 741: return launch_v3<128, 16, 12, 28, 5, false, 1, 8, 3>(a, cus, s);
        case 742: return launch_v3<128, 12, 16, 28, 5, false, 1, 8, 3>(a, cus, s);
        case 743: return launch_v3<128, 12, 8, 28, 5, false, 1, 8, 3>(a, cus, s);
        case 744: return launch_v3<128, 12, 12, 28, 5, false, 1, 9, 3>(a, cus, s);
        case 745: return launch_v3<128, 12, 12, 28, 5, false, 1, 10, 3>(a, cus, s);
        case 746: return launch_v3<128, 12, 12, 28, 5, false, 1, 11, 3>(a, cus, s);
        case 747: return launch_v3<128, 12, 12, 28, 5, false, 1, 12, 3>(a, cus, s);
        case 748: return launch_v3<128, 16, 16, 28, 5, false, 1, 9, 3>(a, cus, s);
        case 750: return launch_v3<128, 12, 12, 28, 5, false, 1, 13, 3>(a, cus, s);
        case 751: return launch_v3<128, 12, 12, 28, 5, false, 1, 14, 3>(a, cus, s);
        case 752: return launch_v3<128, 12, 12, 28, 5, false, 1, 15, 3>(a, cus, s);
        case 753: return launch_v3<128, 12, 12, 28, 5, false, 1, 16, 3>(a, cus, s);
        case 754: return launch_v3<128, 12, 12, 28, 5, false, 1, 17, 3>(a, cus, s);
        case 755: return launch_v3<128, 12, 16, 28, 5, false, 1, 10, 3>(a, cus, s);
        case 756: return launch_v3<128, 12, 8, 28, 5, false, 1, 10, 3>(a, cus, s);
        case 757: return launch_v3<128, 8, 12, 28, 5, false, 1, 10, 3>(a, cus, s);
        case 758: return launch_v3<128, 16, 12, 28, 5, false, 1, 10, 3>(a, cus, s);
        case 759: return launch_v3<128, 12, 12, 28, 5, true, 1, 10, 3>(a, cus, s);  // instrumented
        // coded nodes (node_step7) + extra steps
        case 760: return launch_v3<128, 12, 12, 28, 5, false, 1, 20, 3>(a, cus, s);
        case 761: return launch_v3<128, 12, 12, 28, 5, false, 1, 21, 3>(a, cus, s);
        case 763: return launch_v3<128, 12, 12, 28, 5, false, 1, 23, 3>(a, cus, s);
        case 765: return launch_v3<128, 12, 12, 28, 5, false, 1, 25, 3>(a, cus, s);
        case 767: return launch_v3<128, 12, 12, 28, 5, false, 1, 27, 3>(a, cus, s);
        case 768: return launch_v3<128, 12, 16, 28, 5, false, 1, 27, 3>(a, cus, s);
        case 769: return launch_v3<128, 12, 12, 28, 5, true, 1, 27, 3>(a, cus, s);  // instrumented
        // coded nodes fetched through a buffer resource (56 B per node)
        case 770: return launch_v3<128, 12, 12, 28, 5, false, 1, 47, 3>(a, cus, s);
        case 771: return launch_v3<128, 12, 12, 28, 5, false, 1, 43, 3>(a, cus, s);
        case 772: return launch_v3<128, 12, 12, 28, 5, false, 1, 51, 3>(a, cus, s);
        case 773: return launch_v3<128, 12, 12, 28, 5, false, 1, 55, 3>(a, cus, s);
        case 774: return launch_v3<128, 12, 16, 28, 5, false, 1, 47, 3>(a, cus, s);
        case 775: return launch_v3<128, 16, 12, 28, 5, false, 1, 47, 3>(a, cus, s);
        case 776: return launch_v3<128, 12, 12, 28, 5, false, 1, 31, 3>(a, cus, s);
        case 779: return launch_v3<128, 12, 12, 28, 5, true, 1, 47, 3>(a, cus, s);  // instrumented
        // whole-chunk static ranges
        case 780: return launch_v3<128, 12, 12, 28, 5, false, 1, 51, 7>(a, cus, s);
        case 781: return launch_v3<128, 12, 12, 28, 5, false, 1, 51, 11>(a, cus, s);
        case 782: return launch_v3<128, 12, 12, 28, 5, false, 1, 47, 7>(a, cus, s);
        case 783: return launch_v3<128, 16, 12, 28, 5, false, 1, 51, 7>(a, cus, s);
        case 784: return launch_v3<128, 8, 12, 28, 5, false, 1, 51, 7>(a, cus, s);
        case 789: return launch_v3<128, 12, 12, 28, 5, true, 1, 51, 7>(a, cus, s);  // instrumented
        // short LDS stack + global spill column (NS >= 60) at higher occupancy targets
        case 792: return launch_v3<128, 12, 12, 16, 5, false, 1, 71, 3>(a, cus, s);
        case 793: return launch_v3<128, 12, 12, 16, 6, false, 1, 71, 3>(a, cus, s);
        case 794: return launch_v3<128, 12, 12, 16, 8, false, 1, 71, 3>(a, cus, s);
        case 795: return launch_v3<128, 12, 12, 20, 6, false, 1, 71, 3>(a, cus, s);
        case 796: return launch_v3<128, 12, 12, 12, 8, false, 1, 71, 3>(a, cus, s);
        case 797: return launch_v3<128, 12, 12, 16, 7, false, 1, 71, 3>(a, cus, s);
        // cooperative LDS node fetch (NS >= 80) + spill stack
        case 850: return launch_v3<128, 12, 12, 12, 5, false, 1, 91, 3>(a, cus, s);
        case 851: return launch_v3<128, 12, 12, 16, 5, false, 1, 91, 3>(a, cus, s);
        case 852: return launch_v3<128, 12, 12, 12, 5, false, 1, 87, 3>(a, cus, s);
        case 853: return launch_v3<128, 12, 12, 12, 5, false, 1, 83, 3>(a, cus, s);
        case 854: return launch_v3<128, 12, 12, 8, 5, false, 1, 91, 3>(a, cus, s);
        case 855: return launch_v3<128, 12, 12, 12, 6, false, 1, 91, 3>(a, cus, s);
        case 856: return launch_v3<128, 12, 12, 12, 4, false, 1, 91, 3>(a, cus, s);
        case 858: return launch_v3<128, 12, 12, 12, 5, false, 1, 111, 3>(a, cus, s);  // fetch self-check
        case 857: return launch_v3<128, 12, 12, 12, 5, false, 1, 131, 3>(a, cus, s);  // compare-only self-check
        case 860: return launch_v3<128, 12, 12, 12, 5, false, 1, 151, 3>(a, cus, s);  // FIX 1
        case 861: return launch_v3<128, 12, 12, 12, 5, false, 1, 171, 3>(a, cus, s);  // FIX 2
        case 862: return launch_v3<128, 12, 12, 12, 5, false, 1, 191, 3>(a, cus, s);  // FIX 3
        case 859: return launch_v3<128, 12, 12, 12, 5, true, 1, 91, 3>(a, cus, s);  // instrumented
        case 863: return launch_v3<128, 12, 12, 28, 5, false, 1, 71, 3>(a, cus, s);  // default for deep trees
        case 749: return launch_v3<128, 12, 12, 28, 5, true, 1, 8, 3>(a, cus, s);  // instrumented
        // 16-bit quantized 32-B nodes (NS = 200 + the f32 scheme)
        case 900: return launch_v3<128, 12, 12, 28, 5, false, 1, 251, 3>(a, cus, s);
        case 901: return launch_v3<128, 12, 12, 28, 5, false, 1, 271, 3>(a, cus, s);
        case 902: return launch_v3<128, 12, 12, 28, 5, false, 1, 247, 3>(a, cus, s);
        case 903: return launch_v3<128, 12, 12, 28, 5, false, 1, 255, 3>(a, cus, s);
        case 904: return launch_v3<128, 16, 12, 28, 5, false, 1, 251, 3>(a, cus, s);
        case 905: return launch_v3<128, 12, 12, 28, 6, false, 1, 251, 3>(a, cus, s);
        case 906: return launch_v3<128, 12, 16, 28, 5, false, 1, 251, 3>(a, cus, s);
        case 907: return launch_v3<128, 12, 12, 24, 6, false, 1, 271, 3>(a, cus, s);
        case 908: return launch_v3<128, 12, 12, 20, 6, false, 1, 271, 3>(a, cus, s);
        case 909: return launch_v3<128, 12, 12, 28, 5, true, 1, 251, 3>(a, cus, s);  // instrumented
        // branch-minimal coded steps, pop at the end of a step (trace_kernel_v5)
        case 920: return launch_v5<128, 28, 12, 12, 5, 12, 0>(a, cus, s);
        case 921: return launch_v5<128, 28, 12, 12, 5, 12, 1>(a, cus, s);
        case 922: return launch_v5<128, 28, 12, 12, 5, 8, 0>(a, cus, s);
        case 923: return launch_v5<128, 28, 12, 12, 5, 16, 0>(a, cus, s);
        case 924: return launch_v5<128, 28, 16, 12, 5, 12, 0>(a, cus, s);
        case 925: return launch_v5<128, 28, 12, 8, 5, 12, 0>(a, cus, s);
        case 926: return launch_v5<128, 28, 12, 16, 5, 12, 0>(a, cus, s);
        case 927: return launch_v5<128, 28, 8, 12, 5, 12, 0>(a, cus, s);
        case 928: return launch_v5<128, 28, 12, 12, 5, 6, 0>(a, cus, s);
        case 929: return launch_v5<128, 28, 12, 12, 5, 16, 1>(a, cus, s);
        case 930: return launch_v5<128, 25, 12, 12, 6, 12, 0>(a, cus, s);  // 6 waves/SIMD (trees <= 24 deep)
        case 931: return launch_v5<128, 25, 12, 12, 6, 12, 1>(a, cus, s);
        // 6 waves per SIMD: 26-entry stack (13.3 KB per block; trees up to 25 levels)
        case 970: return launch_v5<128, 26, 12, 12, 6, 12, 1>(a, cus, s);
        case 971: return launch_v5<128, 26, 12, 12, 6, 8, 1>(a, cus, s);
        // static ranges + a shared pool of the last POOL % of the rays
        case 960: return launch_v5<128, 28, 12, 12, 5, 12, 1, 1, 5>(a, cus, s);
        case 961: return launch_v5<128, 28, 12, 12, 5, 12, 1, 1, 10>(a, cus, s);
        case 962: return launch_v5<128, 28, 12, 12, 5, 12, 1, 1, 25>(a, cus, s);
        case 963: return launch_v5<128, 28, 12, 12, 5, 12, 1, 1, 50>(a, cus, s);
        case 964: return launch_v5<128, 28, 12, 12, 5, 12, 1, 1, 100>(a, cus, s);
        // tail shading threshold (TAIL)
        case 990: return launch_v5<128, 28, 12, 12, 5, 12, 1, 1, 0, 1>(a, cus, s);
        case 991: return launch_v5<128, 28, 12, 12, 5, 12, 1, 1, 0, 2>(a, cus, s);
        case 992: return launch_v5<128, 28, 12, 12, 5, 12, 1, 1, 0, 4>(a, cus, s);
        case 993: return launch_v5<128, 28, 12, 12, 5, 12, 1, 1, 0, 8>(a, cus, s);
        case 994: return launch_v5<128, 28, 12, 12, 5, 12, 1, 1, 0, 64>(a, cus, s);
        // cache-policy bits on the node loads (aux = NF >> 4)
        case 980: return launch_v5<128, 28, 12, 12, 5, 12, 17>(a, cus, s);
        case 981: return launch_v5<128, 28, 12, 12, 5, 12, 33>(a, cus, s);
        case 982: return launch_v5<128, 28, 12, 12, 5, 12, 49>(a, cus, s);
        case 983: return launch_v5<128, 28, 12, 12, 5, 12, 65>(a, cus, s);
        // 4-wide quantized branch-free steps (node_step8w)
        case 1000: return launch_v5<128, 28, 12, 12, 5, 8, 5>(a, cus, s);
        case 1001: return launch_v5<128, 28, 12, 12, 4, 8, 5>(a, cus, s);
        case 1002: return launch_v5<128, 28, 12, 12, 5, 6, 5>(a, cus, s);
        case 1003: return launch_v5<128, 28, 12, 8, 5, 8, 5>(a, cus, s);
        case 1004: return launch_v5<128, 28, 12, 12, 5, 4, 5>(a, cus, s);
        case 1005: return launch_v5<128, 28, 12, 12, 5, 5, 5>(a, cus, s);
        case 1006: return launch_v5<128, 28, 12, 16, 5, 6, 5>(a, cus, s);
        case 1007: return launch_v5<128, 28, 16, 12, 5, 6, 5>(a, cus, s);
        case 1008: return launch_v5<128, 28, 12, 12, 5, 3, 5>(a, cus, s);
        case 1009: return launch_v5<128, 28, 12, 12, 5, 6, 5, 1, 0, 8>(a, cus, s);
        case 1010: return launch_v5<128, 28, 12, 12, 5, 6, 5, 1, 0, 64>(a, cus, s);
        // top of the tree in LDS (node_step8c): 64 / 32 nodes per 128-lane block, 128 per 256,
        // 320 per 640 (10 waves, 2 blocks per CU)
        // leaf triangles through buffer loads (leaf_step8 LV = 0)
        case 1200: return launch_v5<128, 28, 12, 12, 5, 12, 1, 0>(a, cus, s);
        // ray state in memory + scalar counters (DIET): 6 waves per SIMD with a 26-entry stack
        // (trees deeper than 25 take the spill-stack kernel), or 5 with the default stack
        case 1300: return launch_v5<128, 26, 12, 12, 6, 12, 1, 1, 0, 0, 0, 1>(a, cus, s);
        case 1301: return launch_v5<128, 28, 12, 12, 5, 12, 1, 1, 0, 0, 0, 1>(a, cus, s);
        case 1302: return launch_v5<128, 26, 12, 12, 6, 8, 1, 1, 0, 0, 0, 1>(a, cus, s);
        case 1303: return launch_v5<128, 28, 12, 12, 5, 12, 1, 1, 0, 0, 0, 2>(a, cus, s);  // scalar counters only
        case 1100: return launch_v5<128, 28, 12, 12, 5, 12, 6, 1, 0, 0, 64>(a, cus, s);
        case 1101: return launch_v5<128, 28, 12, 12, 5, 12, 6, 1, 0, 0, 32>(a, cus, s);
        case 1102: return launch_v5<256, 28, 12, 12, 5, 12, 6, 1, 0, 0, 128>(a, cus, s);
        case 1103: return launch_v5<640, 28, 12, 12, 5, 12, 6, 1, 0, 0, 320>(a, cus, s);
        case 1104: return launch_v5<256, 28, 12, 12, 5, 12, 1>(a, cus, s);
        case 1105: return launch_v5<640, 28, 12, 12, 5, 12, 1>(a, cus, s);
        // tunings of the default (921)
        case 950: return launch_v5<128, 28, 8, 12, 5, 12, 1>(a, cus, s);
        case 951: return launch_v5<128, 28, 16, 12, 5, 12, 1>(a, cus, s);
        case 952: return launch_v5<128, 28, 12, 8, 5, 12, 1>(a, cus, s);
        case 953: return launch_v5<128, 28, 12, 16, 5, 12, 1>(a, cus, s);
        case 954: return launch_v5<128, 28, 12, 12, 5, 12, 1, 2>(a, cus, s);
        case 955: return launch_v5<128, 28, 12, 12, 5, 10, 1>(a, cus, s);
        case 956: return launch_v5<128, 28, 12, 12, 5, 14, 1>(a, cus, s);
        case 957: return launch_v5<64, 28, 12, 12, 5, 12, 1>(a, cus, s);
        case 958: return launch_v5<128, 28, 10, 10, 5, 12, 1>(a, cus, s);
        case 959: return launch_v5<128, 28, 14, 14, 5, 12, 1>(a, cus, s);
        case 940: return launch_v5<128, 28, 12, 12, 5, 12, 3>(a, cus, s);  // pair-cooperative fetch
        case 941: return launch_v5<128, 28, 12, 12, 5, 16, 3>(a, cus, s);
        case 942: return launch_v5<128, 28, 12, 12, 5, 8, 3>(a, cus, s);
        case 943: return launch_v5<128, 28, 16, 12, 5, 12, 3>(a, cus, s);
        case 944: return launch_v5<128, 28, 12, 16, 5, 12, 3>(a, cus, s);
        case 945: return launch_v5<128, 28, 12, 8, 5, 12, 3>(a, cus, s);
        case 932: return launch_v5<128, 28, 12, 12, 5, 12, 2>(a, cus, s);  // octant copies of the quantized nodes
        case 933: return launch_v5<128, 28, 12, 12, 5, 16, 2>(a, cus, s);
        case 934: return launch_v5<128, 28, 16, 12, 5, 12, 2>(a, cus, s);
        case 935: return launch_v5<128, 28, 12, 16, 5, 12, 2>(a, cus, s);
        case 936: return launch_v5<128, 28, 12, 8, 5, 12, 2>(a, cus, s);
        case 937: return launch_v5<128, 28, 8, 12, 5, 12, 2>(a, cus, s);
        // 31-entry LDS stack (16 KB per 128-lane block: 10 blocks fill the 160 KB of LDS)
        case 910: return launch_v3<128, 12, 12, 31, 5, false, 1, 251, 3>(a, cus, s);
        case 911: return launch_v3<128, 12, 12, 31, 5, false, 1, 51, 3>(a, cus, s);
        case 912: return launch_v3<128, 12, 12, 31, 5, false, 1, 271, 3>(a, cus, s);
        // wide trees (trace_width(): 300-309 -> 4-wide, 310-319 -> 8-wide)
        case 300: return launch_w<4, 128, 24, 32, 12, 5>(a, cus, s);
        case 301: return launch_w<4, 128, 32, 32, 12, 5>(a, cus, s);
        case 302: return launch_w<4, 128, 16, 32, 12, 6>(a, cus, s);
        case 303: return launch_w<4, 64, 24, 16, 12, 5>(a, cus, s);
        case 304: return launch_w<4, 128, 24, 16, 12, 5>(a, cus, s);
        case 305: return launch_w<4, 128, 24, 48, 12, 5>(a, cus, s);
        case 306: return launch_w<4, 128, 24, 32, 24, 5>(a, cus, s);
        case 307: return launch_w<4, 128, 20, 32, 12, 4>(a, cus, s);
        case 310: return launch_w<8, 128, 24, 32, 12, 4>(a, cus, s);
        case 311: return launch_w<8, 128, 32, 32, 12, 4>(a, cus, s);
        case 312: return launch_w<8, 128, 16, 32, 12, 5>(a, cus, s);
        case 313: return launch_w<8, 64, 24, 16, 12, 4>(a, cus, s);
        // quantized 4-wide (QNode4, 64 B)
        case 320: return launch_w<kWideQ4, 128, 24, 32, 12, 5>(a, cus, s);
        case 321: return launch_w<kWideQ4, 128, 32, 32, 12, 5>(a, cus, s);
        case 322: return launch_w<kWideQ4, 128, 16, 32, 12, 6>(a, cus, s);
        case 323: return launch_w<kWideQ4, 128, 20, 32, 12, 4>(a, cus, s);
        case 324: return launch_w<kWideQ4, 64, 24, 16, 12, 5>(a, cus, s);
        case 325: return launch_w<kWideQ4, 128, 24, 16, 12, 5>(a, cus, s);
        case 326: return launch_w<kWideQ4, 128, 24, 48, 12, 5>(a, cus, s);
        case 327: return launch_w<kWideQ4, 128, 24, 32, 24, 5>(a, cus, s);
        case 328: return launch_w<kWideQ4, 256, 24, 64, 12, 5>(a, cus, s);
        case 329: return launch_w<kWideQ4, 128, 28, 32, 12, 5>(a, cus, s);
        default:  // = 921: static per-wave ray ranges, direction pre-pass, refill at 12 idle lanes,
                  // branch-free steps (trace_kernel_v5) over the 32-B quantized nodes, 12 per inner
                  // iteration; launch_v5 takes the f32 coded nodes when the emitter is off the
                  // quantization grid and the spill-stack v3 kernel (863) for trees deeper than
                  // the 28-entry LDS stack
            return launch_v5<128, 28, 12, 12, 5, 12, 1>(a, cus, s);
        case 778:  // the round-1e default: 772, or 863 for trees deeper than its LDS stack
            if (a.bvh_depth < 28) return launch_v3<128, 12, 12, 28, 5, false, 1, 51, 3>(a, cus, s);
            return launch_v3<128, 12, 12, 28, 5, false, 1, 71, 3>(a, cus, s);
    }
}

hipError_t launch_finalize_ir(const long long* hist, float* ir_left, float* ir_right, int32_t ir_len, double unit,
                              int32_t is_mono, hipStream_t s) {
    const int b = 256;
    const int g = (ir_len + b - 1) / b;
    if (g > 0) hipLaunchKernelGGL(finalize_ir_kernel, dim3(g), dim3(b), 0, s, hist, ir_left, ir_right, ir_len, unit, is_mono);
    return hipGetLastError();
}

hipError_t launch_ray_directions(uint64_t seed, uint64_t first, uint64_t count, float* d_out, hipStream_t s) {
    const int b = 256;
    const uint64_t g = (count + b - 1) / b;
    if (g > 0) hipLaunchKernelGGL(ray_dir_kernel, dim3((unsigned)g), dim3(b), 0, s, seed, first, count, d_out);
    return hipGetLastError();
}

}  // namespace arx
