// arx_trace.hip -- fused acoustic ray-trace kernel for gfx950 (MI355X).
//
// One lane carries one ray through all of its bounces (raygen -> closest hit -> shading ->
// histogram), replacing the OptiX pipeline of R/prebuild/obj_raytracer/devicePrograms.cu:
//   __raygen__renderFrame   :192-254  -> ray_init() + the refill loop of trace_kernel
//   optixTrace / RT cores   :240-251  -> node_step() / leaf_step(): software traversal of the
//                                        two-level BVH2 (16-bit quantized nodes), per-lane
//                                        stack, watertight triangle test
//   __closesthit__radiance  :62-180   -> shade()
//   __miss__radiance        :186-190  -> shade() with hit < 0
// Work distribution: persistent waves, each owning a static range of ray ids; a wave leaves
// its traversal loop when THRESH lanes wait for shading, shades them and refills retired lanes
// from its range.  The IR histogram is int64 fixed point (unit e0*2^-frac_bits) accumulated
// with 64-bit atomics: order-independent, bitwise reproducible and exactly summable across GPUs.
//
// Arithmetic is IEEE f32 with no contraction (built -ffp-contract=off) so that every ray follows
// bit for bit the path computed by the CPU oracle (oracle/arx_oracle.c).
//
// This file holds only the production kernel (one template, four instances: quantized or f32
// nodes x LDS or global stack).  The round-1 design experiments (wide trees, octant copies,
// cooperative fetch, LDS node caches, ray pools, phased launches) are in
// the git history at commit 62a5de6 (audiorenderingv2_amd/csrc/arx_trace.hip).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>

#include "arx_kernels.hpp"
#include "arx_layout.hpp"

#ifndef ARX_TRACE_BITFLOAT
#define ARX_TRACE_BITFLOAT 1  // 16-bit planes as the float 2^23 + q built by v_perm (0: u16 -> f32 conversions)
#endif
#ifndef ARX_TRACE_SIGNSEL
#define ARX_TRACE_SIGNSEL 1  // per-ray near/far plane selection in the 16-bit node step (0: min / max per slab)
#endif

namespace arx {
namespace {

#ifndef ARX_TRACE_BLOCK
#define ARX_TRACE_BLOCK 128
#endif
#ifndef ARX_TRACE_NCACHE
#define ARX_TRACE_NCACHE 0
#endif
constexpr int kBlock = ARX_TRACE_BLOCK;
// Top-of-tree node cache: the 16-bit path copies quantized nodes [0, kNodeCache) (the top node, then
// the scene tree's breadth-first prefix, bfs_prefix_order) into LDS at launch and reads them from
// there.  Those nodes take a large share of the node steps (arx_debug_wide_stats [16..31]) and
// would otherwise be L1 hits that still cost the TD its per-lane cycles.  The node buffer always
// holds >= 1025 nodes (ensure_device_scene allocates n_nodes + 1024), so the copy stays in bounds.
constexpr int kNodeCache = ARX_TRACE_NCACHE;
static_assert(kNodeCache >= 0 && kNodeCache <= 1024, "node cache: at most the buffer's 1024 spare nodes");

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
    uint32_t nsel[3];  // v_perm selectors per axis: the near plane (ARX_TRACE_SIGNSEL, node_step)
#if ARX_TRACE_BITFLOAT
    uint32_t fsel[3];  // ... and the far plane
#endif
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
#if ARX_TRACE_BITFLOAT
        // a (lo | hi << 16) plane word: near = lo for a positive reciprocal, hi for a negative one;
        // bytes 4-5 (lo) or 6-7 (hi) of {word, 2^23} under 2^23's upper bytes 2-3
        r.nsel[k] = r.inv[k] >= 0.0f ? 0x03020504u : 0x03020706u;
        r.fsel[k] = r.inv[k] >= 0.0f ? 0x03020706u : 0x03020504u;
#else
        // a (lo | hi << 16) plane word: keep for a positive reciprocal (lo is the near plane), swap
        // the halves for a negative one
        r.nsel[k] = r.inv[k] >= 0.0f ? 0x03020100u : 0x01000302u;
#endif
    }
}

// The closest hit so far of one query: t, triangle id (tie-break), the TriRec's unit (-1 none) and
// the test's V, W and det, so shade() needs no second triangle test.
struct Best {
    float t;
    int id;
    int unit;
    float v, w, det;
};

// Watertight ray/triangle test (Woop, Benthin, Wald 2013), t >= 0 (optixTrace tmin 0), and the
// closest-hit update (ties to the lowest id) for a lane where `valid`.  Vertex components are selected
// by (kx,ky,kz) then differenced against the permuted origin: the same values as A[k] = v[k] - o[k]
// indexed afterwards (oracle order).  Branch-free: the early exits of the textbook form and an
// if-based update left the compiler shuffling the Best fields between registers at every join
// (DESIGN.md section 6.3).
__device__ __forceinline__ void take_hit(const Ray& r, float4 p0, float4 p1, float4 p2, int unit, Best& b,
                                         bool valid) {
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
    const bool edge = !(((U < 0.0f) | (V < 0.0f) | (W < 0.0f)) & ((U > 0.0f) | (V > 0.0f) | (W > 0.0f)));
    const float det = U + V + W;
    const float az = r.sz * Az;
    const float bz = r.sz * Bz;
    const float cz = r.sz * Cz;
    const float T = U * az + V * bz + W * cz;
    const float t = T / det;
    const int id = __float_as_int(p1.w);
    const bool take = valid & edge & (det != 0.0f) & (t >= 0.0f) & ((t < b.t) | ((t == b.t) & (id < b.id)));
    b.t = take ? t : b.t;
    b.id = take ? id : b.id;
    b.unit = take ? unit : b.unit;
    b.v = take ? V : b.v;
    b.w = take ? W : b.w;
    b.det = take ? det : b.det;
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
    // ray_direction(a.seed, rid), precomputed by the launcher's pre-pass (dirs_kernel)
    const float4 d = reinterpret_cast<const float4*>(a.dirs)[rid - a.ray_begin];
    s.dir = make_float3(d.x, d.y, d.z);
    s.pos = make_float3(a.emitter[0], a.emitter[1], a.emitter[2]);
    s.e = a.e0;
    s.dist = 0.0f;
    s.depth = 0;
    if (!(s.dir.x != 0.0f || s.dir.y != 0.0f || s.dir.z != 0.0f)) s.depth = -1;  // :230, no trace
}

// __closesthit__radiance (devicePrograms.cu:62-180) for TriRec `hit`, or __miss__radiance
// (:186-190) when hit < 0.  r is the ray the query was traced with.
__device__ __forceinline__ void shade(const TraceArgs& a, const float4* __restrict__ tbase, RayState& s, const Ray& r,
                                      const Best& best, uint32_t& n_rx, uint32_t& n_miss) {
    const int hit = best.unit;
    if (hit < 0) {
        ++n_miss;
        s.depth = -1;
        return;
    }
    const float4* tp = tbase + hit;  // hit = the triangle's 16-B unit (leaf_step)
    const float4 p0 = tp[0], p1 = tp[1], p2 = tp[2];
    const float3 P1 = make_float3(p0.x, p0.y, p0.z);
    const float3 P2 = make_float3(p1.x, p1.y, p1.z);
    const float3 P3 = make_float3(p2.x, p2.y, p2.z);
    const float ab = p0.w;
    // Ng = normalize(cross(P2-P1, P3-P1))  (:75-77)
    const float3 U = sub3(P2, P1), V = sub3(P3, P1);
    const float3 cr = make_float3(U.y * V.z - V.y * U.z, U.z * V.x - V.z * U.x, U.x * V.y - V.x * U.y);
    const float hv = best.v, hw = best.w, hdet = best.det;
    const float bu = hv / hdet;
    const float bv = hw / hdet;
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
        // reflection about the unnormalised normal, dir - (2 (dir . cr) / (cr . cr)) cr: the same
        // mirror as with normalize(cr) (:75-77, :173) for one division, no square root
        const float s2 = (2.0f * dot3(s.dir, cr)) / dot3(cr, cr);
        s.dir = sub3(s.dir, scale3(s2, cr));
        e = e * (1.0f - ab);
        ++s.depth;
    }
    s.e = e;
    s.pos = add3(P, scale3(1e-3f, s.dir));  // :179
}

__device__ __forceinline__ void flush_counters(const TraceArgs& a, uint32_t n_q, uint32_t n_rx, uint32_t n_miss,
                                               int lane) {
    unsigned int vq = n_q, vr = n_rx, vm = n_miss;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        vq += __shfl_xor(vq, off, 64);
        vr += __shfl_xor(vr, off, 64);
        vm += __shfl_xor(vm, off, 64);
    }
    if ((lane & 63) == 0) {
        if (vq) atomicAdd(a.counters + 0, (unsigned long long)vq);
        if (vr) atomicAdd(a.counters + 1, (unsigned long long)vr);
        if (vm) atomicAdd(a.counters + 2, (unsigned long long)vm);
    }
}
// ------------------------------------------------------------ traversal ---
// Per-lane state of one closest-hit query over the two-level BVH (node 0 = top node).
// node: the lane's next stack entry -- >= 0 an inner node, <= -2 a pending leaf
// ~(first*16 + count), -1 done.  Empty children carry a 0-triangle leaf code (kEmptyChildCode).
struct Trav {
    Best best;  // closest hit so far
    int node;
    int sp;    // stack depth
};

// Traversal stack of one lane.  LDS: ROWS entries at stk[slot * BLOCK + lane].  Global (trees
// deeper than the LDS rows): a column of bvh_depth + 1 entries at gstack[slot * lanes + gid],
// coalesced across the wave like the LDS rows.  A stack holds at most one entry per tree level,
// so rows > bvh_depth never overflows.
// Both give the step two accessors: below(sp) reads the entry a pop would take (slot sp - 1; any
// value when sp == 0) and put(sp, v) writes slot sp, the one above the top.
//   LdsStack: slot s lives in row s + 1 and row 0 is a dummy, so below(sp) is row sp and put(sp) is
//   row sp + 1: one address for both (the write's +1 row is the instruction's offset), no clamps --
//   the launcher takes this stack only for trees with bvh_depth + 1 <= ROWS, and a stack holds at
//   most one entry per level.
//   kSentinel: below(0) is -1 (LdsStack's dummy row, written once per launch), so a pop needs no
//   empty-stack test.
template <int BLOCK, int ROWS>
struct LdsStack {
    static constexpr bool kSentinel = true;
    int* base;  // &stk[lane]
    __device__ __forceinline__ int below(int sp) const { return base[sp * BLOCK]; }
    __device__ __forceinline__ void put(int sp, int v) const { base[(sp + 1) * BLOCK] = v; }
};
struct GlobalStack {
    static constexpr bool kSentinel = false;
    int* base;  // &gstack[gid]
    uint64_t stride;
    int nrows;
    __device__ __forceinline__ int below(int sp) const { return base[(uint64_t)max(sp - 1, 0) * stride]; }
    __device__ __forceinline__ void put(int sp, int v) const { base[(uint64_t)min(sp, nrows - 1) * stride] = v; }
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t buffer_rsrc(const void* p, short stride = 0) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), stride, 0x7fffffff, 0x00020000);
}

// lanes in a wave mask, as a 32-bit scalar (two s_bcnt1_i32_b32): compares against it stay on the SALU
__device__ __forceinline__ uint32_t lanes32(unsigned long long m) {
    return (uint32_t)__builtin_popcount((uint32_t)m) + (uint32_t)__builtin_popcount((uint32_t)(m >> 32));
}
#ifndef ARX_TRACE_IDXEN
#define ARX_TRACE_IDXEN 1  // QNode2 loads indexed by node (idxen, a 32-B stride resource): no address VALU (C3 -1.6 %, profiles/r05/ab_idxen.txt); 0: byte offsets
#endif
typedef int arx_i32x4 __attribute__((ext_vector_type(4)));
// buffer_load_dwordx4 ... idxen: address = base + vindex * stride + voffset + inst offset (the
// hardware's structured-buffer addressing; clang has no builtin for it, the LLVM intrinsic is bound
// by name as composable_kernel's amd_buffer_addressing.hpp does for the raw forms)
__device__ arx_i32x4 arx_struct_buffer_load_b128(__amdgpu_buffer_rsrc_t rsrc, int vindex, int voffset, int soffset,
                                                 int aux) __asm("llvm.amdgcn.struct.ptr.buffer.load.v4i32");
#ifndef ARX_TRACE_SFETCH
#define ARX_TRACE_SFETCH 0  // design experiment: the wave leader's node by one scalar load (see node_step)
#endif
typedef int arx_i32x8 __attribute__((ext_vector_type(8)));
// s_buffer_load_dwordx8 (a scalar LOAD through the scalar data cache; the descriptor as 4 SGPRs)
__device__ arx_i32x8 arx_s_buffer_load_b256(arx_i32x4 rsrc, int offset, int aux) __asm("llvm.amdgcn.s.buffer.load.v8i32");
__device__ __forceinline__ uint4 node_half(__amdgpu_buffer_rsrc_t rs, int node, int half) {
#if ARX_TRACE_IDXEN
    const arx_i32x4 v = arx_struct_buffer_load_b128(rs, node, half * 16, 0, 0);
    return make_uint4((uint32_t)v.x, (uint32_t)v.y, (uint32_t)v.z, (uint32_t)v.w);
#else
    return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, node * (int)sizeof(QNode2) + half * 16, 0, 0));
#endif
}

// One branch-free node step: test both children of t.node, continue with the nearer hit child,
// push the farther one, or pop when neither is hit.  Entries are popped at the end of a step,
// so the only guard is t.node >= 0; everything inside is a select (bitwise & / | on the bools:
// && / || compile back to exec-mask branches).
//   Q16: 32-B QNode2 (two 16-B buffer loads).  A slab plane is grid.origin + q * grid.scale, so
//        t = q * (scale*inv) + (origin - o)*inv: the caller passes ix = scale*inv and
//        oix = (o - origin)*inv per axis, and each plane is one u16 -> f32 conversion and one fma.
//        Conservative: the f32 error of that form is below 5 * 2^-24 * (grid extent) * |inv| for
//        origins on the grid, far below the 0.1-step outward margin of every quantized plane
//        (quantize_nodes16; the launcher checks the emitter is on the grid).
//   f32: the coded BvhNode (56 of its 64 B), ix = inv, oix = o*inv.
template <int FMT, typename Stack, bool PIN = true>
__device__ __forceinline__ void node_step(const Ray& r, float oix, float oiy, float oiz, Trav& t, const Stack& stk,
                                          __amdgpu_buffer_rsrc_t rs, const uint4* __restrict__ ncache,
                                          arx_i32x4 qrs) {
    constexpr bool Q16 = FMT == kFmtQ16;
    // the pop candidate is read first, so its latency hides under the node fetch (slot sp - 1 is
    // not touched by this step's write to slot sp)
    const int sp = t.sp;
    const int sp_pop = max(sp - 1, 0);
    int top = stk.below(sp);
    const float ix = r.inv[0], iy = r.inv[1], iz = r.inv[2];
    float4 na, nb, nc;
    int c0, c1;
    uint4 A = make_uint4(0u, 0u, 0u, 0u), B = A;
    if constexpr (Q16) {
        if constexpr (kNodeCache > 0) {
            // every lane reads the LDS copy (clamped index; a few cycles per wave) and only the
            // lanes below the cached prefix skip the global fetch: separate registers for the two,
            // so the LDS reads never wait behind the buffer loads
            const bool cached = t.node < kNodeCache;
            uint4 Ag = make_uint4(0u, 0u, 0u, 0u), Bg = Ag;
            if (!cached) {
                const int off = t.node * (int)sizeof(QNode2);
                Ag = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
                Bg = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off + 16, 0, 0));
            }
            const int ci = 2 * min(t.node, kNodeCache - 1);
            const uint4 Al = ncache[ci], Bl = ncache[ci + 1];
            A = make_uint4(cached ? Al.x : Ag.x, cached ? Al.y : Ag.y, cached ? Al.z : Ag.z, cached ? Al.w : Ag.w);
            B = make_uint4(cached ? Bl.x : Bg.x, cached ? Bl.y : Bg.y, cached ? Bl.z : Bg.z, cached ? Bl.w : Bg.w);
        } else {
#if ARX_TRACE_SFETCH
            // the wave leader's node (the first lane stepping) by one scalar load, no vector-memory
            // (TD) work; only the lanes at another node issue the two 16-B vector loads
            const int lead = __builtin_amdgcn_readfirstlane(t.node);
            const arx_i32x8 sn = arx_s_buffer_load_b256(qrs, lead * (int)sizeof(QNode2), 0);
            if (t.node != lead) {
                A = node_half(rs, t.node, 0);
                B = node_half(rs, t.node, 1);
            } else {
                A = make_uint4((uint32_t)sn.s0, (uint32_t)sn.s1, (uint32_t)sn.s2, (uint32_t)sn.s3);
                B = make_uint4((uint32_t)sn.s4, (uint32_t)sn.s5, (uint32_t)sn.s6, (uint32_t)sn.s7);
            }
#else
            A = node_half(rs, t.node, 0);
            B = node_half(rs, t.node, 1);
#endif
        }
        na = make_float4((float)(A.x & 0xffffu), (float)(A.x >> 16), (float)(A.y & 0xffffu), (float)(A.y >> 16));
        nb = make_float4((float)(B.x & 0xffffu), (float)(B.x >> 16), (float)(B.y & 0xffffu), (float)(B.y >> 16));
        nc = make_float4((float)(A.z & 0xffffu), (float)(A.z >> 16), (float)(B.z & 0xffffu), (float)(B.z >> 16));
        c0 = (int)A.w;
        c1 = (int)B.w;
    } else {
        const int off = t.node * (int)sizeof(BvhNode);
        na = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
        nb = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, off + 16, 0, 0));
        nc = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, off + 32, 0, 0));
        const int2 d = __builtin_bit_cast(int2, __builtin_amdgcn_raw_buffer_load_b64(rs, off + 48, 0, 0));
        c0 = d.x;
        c1 = d.y;
    }
    float tn0, tf0, tn1, tf1;
    if constexpr (Q16 && ARX_TRACE_SIGNSEL) {
        // near / far planes picked per ray (the reciprocal's sign) by a byte permute of each plane
        // word: no min / max per slab.  The fma is monotone in q, so the near plane's t is the
        // min of the two and the result is the min / max form's, bit for bit; an empty child's
        // (1, 0) planes come out near > far on either sign.
#if ARX_TRACE_BITFLOAT
        // Each plane straight from its bits: v_perm puts the near (far) 16-bit half under the
        // exponent byte of 2^23, giving the float 2^23 + q exactly, and oix here is
        // C = fma(2^23, ix, (o - origin) * inv) (trace_kernel): t = fma(2^23 + q, ix, -C) is
        // q * ix - (o - origin) * inv up to C's rounding, <= 0.504 step, which the kQ16Margin
        // outward rounding of every plane covers (arx_layout.hpp).  No int -> float conversions.
        auto pl = [](uint32_t w, uint32_t sel) { return __uint_as_float(__builtin_amdgcn_perm(w, 0x4B000000u, sel)); };
        const float nx0 = __builtin_fmaf(pl(A.x, r.nsel[0]), ix, -oix), fx0 = __builtin_fmaf(pl(A.x, r.fsel[0]), ix, -oix);
        const float ny0 = __builtin_fmaf(pl(A.y, r.nsel[1]), iy, -oiy), fy0 = __builtin_fmaf(pl(A.y, r.fsel[1]), iy, -oiy);
        const float nz0 = __builtin_fmaf(pl(A.z, r.nsel[2]), iz, -oiz), fz0 = __builtin_fmaf(pl(A.z, r.fsel[2]), iz, -oiz);
        const float nx1 = __builtin_fmaf(pl(B.x, r.nsel[0]), ix, -oix), fx1 = __builtin_fmaf(pl(B.x, r.fsel[0]), ix, -oix);
        const float ny1 = __builtin_fmaf(pl(B.y, r.nsel[1]), iy, -oiy), fy1 = __builtin_fmaf(pl(B.y, r.fsel[1]), iy, -oiy);
        const float nz1 = __builtin_fmaf(pl(B.z, r.nsel[2]), iz, -oiz), fz1 = __builtin_fmaf(pl(B.z, r.fsel[2]), iz, -oiz);
#else
        const uint32_t ax = __builtin_amdgcn_perm(A.x, A.x, r.nsel[0]), ay = __builtin_amdgcn_perm(A.y, A.y, r.nsel[1]);
        const uint32_t az = __builtin_amdgcn_perm(A.z, A.z, r.nsel[2]), bxw = __builtin_amdgcn_perm(B.x, B.x, r.nsel[0]);
        const uint32_t byw = __builtin_amdgcn_perm(B.y, B.y, r.nsel[1]), bzw = __builtin_amdgcn_perm(B.z, B.z, r.nsel[2]);
        const float nx0 = __builtin_fmaf((float)(ax & 0xffffu), ix, -oix), fx0 = __builtin_fmaf((float)(ax >> 16), ix, -oix);
        const float ny0 = __builtin_fmaf((float)(ay & 0xffffu), iy, -oiy), fy0 = __builtin_fmaf((float)(ay >> 16), iy, -oiy);
        const float nz0 = __builtin_fmaf((float)(az & 0xffffu), iz, -oiz), fz0 = __builtin_fmaf((float)(az >> 16), iz, -oiz);
        const float nx1 = __builtin_fmaf((float)(bxw & 0xffffu), ix, -oix), fx1 = __builtin_fmaf((float)(bxw >> 16), ix, -oix);
        const float ny1 = __builtin_fmaf((float)(byw & 0xffffu), iy, -oiy), fy1 = __builtin_fmaf((float)(byw >> 16), iy, -oiy);
        const float nz1 = __builtin_fmaf((float)(bzw & 0xffffu), iz, -oiz), fz1 = __builtin_fmaf((float)(bzw >> 16), iz, -oiz);
#endif
        tn0 = fmaxf(fmaxf(fmaxf(nx0, ny0), nz0), 0.0f);
        tf0 = fminf(fminf(fminf(fx0, fy0), fz0), t.best.t);
        tn1 = fmaxf(fmaxf(fmaxf(nx1, ny1), nz1), 0.0f);
        tf1 = fminf(fminf(fminf(fx1, fy1), fz1), t.best.t);
    } else {
        const float x00 = __builtin_fmaf(na.x, ix, -oix), x01 = __builtin_fmaf(na.y, ix, -oix);
        const float y00 = __builtin_fmaf(na.z, iy, -oiy), y01 = __builtin_fmaf(na.w, iy, -oiy);
        const float z00 = __builtin_fmaf(nc.x, iz, -oiz), z01 = __builtin_fmaf(nc.y, iz, -oiz);
        const float x10 = __builtin_fmaf(nb.x, ix, -oix), x11 = __builtin_fmaf(nb.y, ix, -oix);
        const float y10 = __builtin_fmaf(nb.z, iy, -oiy), y11 = __builtin_fmaf(nb.w, iy, -oiy);
        const float z10 = __builtin_fmaf(nc.z, iz, -oiz), z11 = __builtin_fmaf(nc.w, iz, -oiz);
        tn0 = fmaxf(fmaxf(fminf(x00, x01), fminf(y00, y01)), fmaxf(fminf(z00, z01), 0.0f));
        tf0 = fminf(fminf(fmaxf(x00, x01), fmaxf(y00, y01)), fminf(fmaxf(z00, z01), t.best.t));
        tn1 = fmaxf(fmaxf(fminf(x10, x11), fminf(y10, y11)), fmaxf(fminf(z10, z11), 0.0f));
        tf1 = fminf(fminf(fmaxf(x10, x11), fmaxf(y10, y11)), fminf(fmaxf(z10, z11), t.best.t));
    }
    const bool h0 = tn0 <= tf0, h1 = tn1 <= tf1;
    const bool near1 = h1 & (!h0 | (tn1 < tn0));
    const int c_near = near1 ? c1 : c0;
    const int c_far = near1 ? c0 : c1;
    stk.put(sp, c_far);  // above the top of the stack unless pushed
    // PIN: an empty asm keeps the pop read unconditional (no branch around it); the small-launch
    // instance leaves it to the compiler, which keeps it unconditional too, without the asm's s_nop
    if constexpr (PIN) asm volatile("" : "+v"(top));
    const bool any = h0 | h1, both = h0 & h1;
    if constexpr (Stack::kSentinel) {  // row 0 holds -1: a pop of the empty stack ends the query
        // near1 -> c1; else h0 -> c0; else neither child was hit (near1 is false only with !h1 or h0)
        t.node = near1 ? c1 : (h0 ? c0 : top);
        t.sp = sp + (h0 ? 0 : -1) + (int)h1;  // push, continue or pop; -1 only once the query is done
    } else {
        t.node = any ? c_near : (sp > 0 ? top : -1);
        t.sp = any ? (both ? sp + 1 : sp) : sp_pop;
    }
}

// CW4 step (arx_layout.hpp): one 32-B node = two 16-B loads for four children.  Plane q of axis k
// is 4*o_k + q*2^e_k grid quanta, so t = fma(q, ix*2^e, fma(o, 4*ix, -oix)) (ix*2^e exact): the
// Q16 slab arithmetic with the frame folded in.  The hit children are sorted by entry distance
// (a 5-exchange network), the nearest is taken and the others are pushed farthest first.  Up to
// three pushes per step: the stack rows above ROWS live in the global overflow column (deep
// trees; the hot path never touches it while every lane's stack stays below ROWS - 3).
__device__ __forceinline__ void cas(float& ka, int& va, float& kb, int& vb) {
    const bool sw = kb < ka;
    const float k0 = sw ? kb : ka, k1 = sw ? ka : kb;
    const int v0 = sw ? vb : va, v1 = sw ? va : vb;
    ka = k0;
    kb = k1;
    va = v0;
    vb = v1;
}

template <int S>
__device__ __forceinline__ float w4_plane(const uint32_t (&w)[5]) {
    return (float)((w[S / 5] >> (6 * (S % 5))) & 63u);
}

template <int C>
__device__ __forceinline__ float w4_child(const uint32_t (&w)[5], float sx, float bx, float sy, float by, float sz,
                                          float bz, float best_t, float& tf_out) {
    const float x0 = __builtin_fmaf(w4_plane<6 * C + 0>(w), sx, bx), x1 = __builtin_fmaf(w4_plane<6 * C + 1>(w), sx, bx);
    const float y0 = __builtin_fmaf(w4_plane<6 * C + 2>(w), sy, by), y1 = __builtin_fmaf(w4_plane<6 * C + 3>(w), sy, by);
    const float z0 = __builtin_fmaf(w4_plane<6 * C + 4>(w), sz, bz), z1 = __builtin_fmaf(w4_plane<6 * C + 5>(w), sz, bz);
    tf_out = fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fminf(fmaxf(z0, z1), best_t));
    return fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fmaxf(fminf(z0, z1), 0.0f));
}

template <int BLOCK, int ROWS>
struct W4Stack {
    static constexpr bool kSentinel = false;
    int* lds;        // &stk[lane]
    int* glob;       // &gstack[gid]: rows ROWS.. (overflow)
    uint64_t stride;
    __device__ __forceinline__ int read(int slot) const {
        return slot < ROWS ? lds[slot * BLOCK] : glob[(uint64_t)(slot - ROWS) * stride];
    }
    __device__ __forceinline__ void write(int slot, int v) const {
        if (slot < ROWS) lds[slot * BLOCK] = v;
        else glob[(uint64_t)(slot - ROWS) * stride] = v;
    }
    __device__ __forceinline__ int below(int sp) const { return read(max(sp - 1, 0)); }
};

template <typename Stack>
__device__ __forceinline__ void node_step_w4(const Ray& r, float oix, float oiy, float oiz, Trav& t, const Stack& stk,
                                             __amdgpu_buffer_rsrc_t rs) {
    const int sp = t.sp;
    const int sp_pop = max(sp - 1, 0);
    int top = stk.read(sp_pop);
    const int off = t.node * 16;
    const uint4 A = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
    const uint4 B = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off + 16, 0, 0));
    const float ix = r.inv[0], iy = r.inv[1], iz = r.inv[2];
    const float sx = __builtin_ldexpf(ix, (int)(A.x >> 28));
    const float sy = __builtin_ldexpf(iy, (int)((A.y >> 14) & 15u));
    const float sz = __builtin_ldexpf(iz, (int)((A.y >> 18) & 15u));
    const float bx = __builtin_fmaf((float)(A.x & 0x3FFFu), 4.0f * ix, -oix);
    const float by = __builtin_fmaf((float)((A.x >> 14) & 0x3FFFu), 4.0f * iy, -oiy);
    const float bz = __builtin_fmaf((float)(A.y & 0x3FFFu), 4.0f * iz, -oiz);
    const uint32_t meta = A.y >> 22;  // bits 30..31 are zero
    const uint32_t w[5] = {A.z, A.w, B.x, B.y, B.z};
    const int base = (int)B.w;
    const float inf = __builtin_huge_valf();
    float tf0, tf1, tf2, tf3;
    const float tn0 = w4_child<0>(w, sx, bx, sy, by, sz, bz, t.best.t, tf0);
    const float tn1 = w4_child<1>(w, sx, bx, sy, by, sz, bz, t.best.t, tf1);
    const float tn2 = w4_child<2>(w, sx, bx, sy, by, sz, bz, t.best.t, tf2);
    const float tn3 = w4_child<3>(w, sx, bx, sy, by, sz, bz, t.best.t, tf3);
    const uint32_t m0 = meta & 3u, m1 = (meta >> 2) & 3u, m2 = (meta >> 4) & 3u, m3 = (meta >> 6) & 3u;
    float k0 = ((tn0 <= tf0) & (m0 != 0u)) ? tn0 : inf;
    float k1 = ((tn1 <= tf1) & (m1 != 0u)) ? tn1 : inf;
    float k2 = ((tn2 <= tf2) & (m2 != 0u)) ? tn2 : inf;
    float k3 = ((tn3 <= tf3) & (m3 != 0u)) ? tn3 : inf;
    // child codes: inner slots come first (node at base + 2c), then the leaves' triangles
    const int i1 = m1 == 1u, i2 = m2 == 1u, i3 = m3 == 1u;
    const int n_inner = (int)(m0 == 1u) + i1 + i2 + i3;
    const int l0 = m0 >= 2u ? (int)m0 - 1 : 0, l1 = m1 >= 2u ? (int)m1 - 1 : 0, l2 = m2 >= 2u ? (int)m2 - 1 : 0;
    const int lb = base + 2 * n_inner;
    int c0 = m0 == 1u ? base : ~(lb * 4 + l0);
    int c1 = i1 ? base + 2 : ~((lb + 3 * l0) * 4 + l1);
    int c2 = i2 ? base + 4 : ~((lb + 3 * (l0 + l1)) * 4 + l2);
    int c3 = i3 ? base + 6 : ~((lb + 3 * (l0 + l1 + l2)) * 4 + (m3 >= 2u ? (int)m3 - 1 : 0));
    cas(k0, c0, k1, c1);
    cas(k2, c2, k3, c3);
    cas(k0, c0, k2, c2);
    cas(k1, c1, k3, c3);
    cas(k1, c1, k2, c2);
    const int hits = (int)(k0 < inf) + (int)(k1 < inf) + (int)(k2 < inf) + (int)(k3 < inf);
    // pushes above the top (the farthest deepest): hits 4 -> c3 c2 c1, 3 -> c2 c1, 2 -> c1
    stk.write(sp, hits == 4 ? c3 : (hits == 3 ? c2 : c1));
    stk.write(sp + 1, hits == 4 ? c2 : c1);
    stk.write(sp + 2, c1);
    asm volatile("" : "+v"(top));
    const int popped = sp > 0 ? top : -1;
    t.node = hits > 0 ? c0 : popped;
    t.sp = hits > 0 ? sp + hits - 1 : sp_pop;
}

// Leaf step, run by every lane of a leaf phase with no divergent branch: lanes
// without a pending leaf, and the second record of a one-triangle leaf, load through a buffer
// offset past the resource's range, which returns zeros without a memory access, and their tests
// are masked off.  Straight-line code lets the closest-hit state stay in its registers (the
// divergent form made the compiler copy it in and out at every join).
__device__ __forceinline__ float4 tri_unit(__amdgpu_buffer_rsrc_t rs, uint32_t off) {
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
}
template <int FMT, typename Stack>
__device__ __forceinline__ void leaf_step(__amdgpu_buffer_rsrc_t trs, const Ray& r, Trav& t, const Stack& stk) {
    const bool lf = t.node <= -2;
    const int v = ~t.node;
    const int unit = FMT == kFmtW4 ? (v >> 2) : 3 * (v >> 4);
    const int count = lf ? (FMT == kFmtW4 ? (v & 3) : (v & 15)) : 0;
    constexpr uint32_t kNoLoad = 0x80000000u;  // > num_records (0x7fffffff): zeros, no access
    const uint32_t o0 = count > 0 ? (uint32_t)unit * 16u : kNoLoad;
    const uint32_t o1 = count > 1 ? (uint32_t)(unit + 3) * 16u : kNoLoad;
    const float4 p0 = tri_unit(trs, o0), p1 = tri_unit(trs, o0 + 16u), p2 = tri_unit(trs, o0 + 32u);
    const float4 q0 = tri_unit(trs, o1), q1 = tri_unit(trs, o1 + 16u), q2 = tri_unit(trs, o1 + 32u);
    take_hit(r, p0, p1, p2, unit, t.best, count > 0);
    take_hit(r, q0, q1, q2, unit + 3, t.best, count > 1);
    // A leaf of more than 2 triangles (only below the builder's depth cap) continues as the same leaf
    // two triangles on, instead of a loop here: the step stays loop-free (a divergent loop in it
    // made the compiler move the closest-hit state into other registers and back at every join).
    const bool more = count > 2;
    const int rest = FMT == kFmtW4 ? ~((unit + 6) * 4 + (count - 2)) : ~(((unit / 3) + 2) * 16 + (count - 2));
    const int sp = t.sp;
    int top = stk.below(sp);
    asm volatile("" : "+v"(top));
    if constexpr (Stack::kSentinel) {
        t.node = lf ? (more ? rest : top) : t.node;
        t.sp = (lf & !more) ? sp - 1 : sp;
    } else {
        t.node = lf ? (more ? rest : (sp > 0 ? top : -1)) : t.node;
        t.sp = (lf & !more) ? max(sp - 1, 0) : sp;
    }
}

// Highest VGPR the trace kernel claims, so that its allocation (granule 8) admits exactly
// ARX_TRACE_WAVES waves per SIMD: 5 -> 88 VGPRs (512/88 = 5.8), 4 -> 104, 6 -> 80.  Every wave of
// a persistent launch owns an equal share of the rays, so a SIMD holding one wave more than the
// others sets the launch time; with 74 VGPRs the SIMDs of a CU took 6/6/4/4 of its 20 waves
// (+12 % on C3 against the same code at 88 VGPRs, tools/gpu_ab.sh, r02 log).
#ifndef ARX_TRACE_WAVES
#define ARX_TRACE_WAVES 5
#endif
#ifndef ARX_TRACE_COUNT
#define ARX_TRACE_COUNT 0  // 1: count node steps / leaf triangle tests into counters[4..5]
#endif
// Dynamic tail (launch_trace): launches with at least kDynMinRaysPerWave rays per wave put
// kDynShare/256 of their rays into the chunk pool of trace_kernel, kDynChunk rays per pool atomic.
// Small launches (about a ray per lane: C2, one 8-GPU rank's C5 shard) keep static ranges: there a
// chunk is a whole wave's work and the pool only lengthens the longest chains.
#ifndef ARX_TRACE_DYN_SHARE
#define ARX_TRACE_DYN_SHARE 128
#endif
#ifndef ARX_TRACE_DYN_CHUNK
#define ARX_TRACE_DYN_CHUNK 8
#endif
#ifndef ARX_TRACE_DYN_MIN
#define ARX_TRACE_DYN_MIN 96
#endif
constexpr int kDynShare = ARX_TRACE_DYN_SHARE, kDynChunk = ARX_TRACE_DYN_CHUNK, kDynMinRaysPerWave = ARX_TRACE_DYN_MIN;
#ifndef ARX_TRACE_PROF
#define ARX_TRACE_PROF 0  // 1: per-wave timing and lane-occupancy records into TraceArgs::prof
#endif
#if ARX_TRACE_WAVES == 5
#define ARX_TRACE_VGPR_FENCE "v87"
#elif ARX_TRACE_WAVES == 4
#define ARX_TRACE_VGPR_FENCE "v103"
#elif ARX_TRACE_WAVES == 6
#define ARX_TRACE_VGPR_FENCE "v79"
#else
#error "ARX_TRACE_WAVES must be 4, 5 or 6"
#endif

// The persistent trace kernel.  Each wave owns the static ray range [w_next, w_end) of its
// launch.  Outer loop: shade the lanes whose query finished, refill retired lanes with new rays
// (directions from the pre-pass), set up the next query of every lane that needs one.  Inner
// loop: NSTEPS guarded node steps per iteration; leaves are postponed and intersected wave-wide
// once LEAF_THRESH lanes hold one (or no lane can step); the loop is left when THRESH lanes wait
// for shading.
// LEAN (the small-launch instance): no per-lane "traversing" flag -- a lane's query is done when its
// node is -1 -- so the inner loop counts the lanes waiting for shading from wave masks on the SALU
// (C2 0.366 -> 0.350 ms; the pool instance measured +1 % with it, profiles/r05/ab_loop.txt).
template <int BLOCK, int THRESH, int LEAF_THRESH, int MINW, int NSTEPS, int FMT, bool GSTACK, bool LEAN = false>
__global__ __launch_bounds__(BLOCK, MINW) void trace_kernel(TraceArgs a) {
    constexpr bool Q16 = FMT == kFmtQ16;
    constexpr bool W4 = FMT == kFmtW4;
    __shared__ int stk_lds[GSTACK ? 1 : (kLdsStack + 1) * BLOCK];  // + LdsStack's dummy row
    __shared__ uint4 ncache[(Q16 && kNodeCache > 0) ? 2 * kNodeCache : 1];
    if constexpr (Q16 && kNodeCache > 0) {
        const uint4* q = reinterpret_cast<const uint4*>(a.qnodes);
        for (int i = threadIdx.x; i < 2 * kNodeCache; i += BLOCK) ncache[i] = q[i];
        __syncthreads();
    }
    // Hold the VGPR allocation at the count that fits exactly MINW waves per SIMD (see
    // ARX_TRACE_VGPR_FENCE): the kernel needs ~74, which would let the dispatcher put 6 waves on
    // some SIMDs and 4 on others.
    asm volatile("" ::: ARX_TRACE_VGPR_FENCE);
    const int lane = threadIdx.x;
    const uint32_t gid = blockIdx.x * BLOCK + threadIdx.x;
    using Stack = typename std::conditional<
        W4, W4Stack<BLOCK, kLdsStack>,
        typename std::conditional<GSTACK, GlobalStack, LdsStack<BLOCK, kLdsStack>>::type>::type;
    Stack stk;
    if constexpr (W4) {  // LDS rows, then the global overflow column
        stk.lds = stk_lds + lane;
        stk.glob = a.gstack + gid;
        stk.stride = a.gstack_lanes;
    } else if constexpr (GSTACK) {
        stk.base = a.gstack + gid;
        stk.stride = a.gstack_lanes;
        stk.nrows = a.bvh_depth + 1;
    } else {
        stk.base = stk_lds + lane;
        stk_lds[lane] = -1;  // the dummy row under the stack (LdsStack::kSentinel)
    }
    const __amdgpu_buffer_rsrc_t nrs = W4 ? buffer_rsrc(a.wbuf)
                                          : (Q16 ? buffer_rsrc(a.qnodes, ARX_TRACE_IDXEN ? (short)sizeof(QNode2) : (short)0)
                                                 : buffer_rsrc(a.cnodes));
    // the quantized nodes' descriptor as four scalars (the scalar-load experiment, ARX_TRACE_SFETCH)
    arx_i32x4 qrs;
    {
        const unsigned long long qa = (unsigned long long)a.qnodes;
        qrs.x = (int)(uint32_t)qa;
        qrs.y = (int)((qa >> 32) & 0xffffu);
        qrs.z = 0x7fffffff;
        qrs.w = 0x00020000;
    }
    const float4* tbase = W4 ? reinterpret_cast<const float4*>(a.wbuf) : reinterpret_cast<const float4*>(a.tris);
    const __amdgpu_buffer_rsrc_t trs = buffer_rsrc(tbase);
    const uint64_t n = a.ray_end - a.ray_begin;
    const uint32_t wave_id = __builtin_amdgcn_readfirstlane(gid >> 6);
    const uint32_t n_waves = gridDim.x * (BLOCK / 64);
    // Rays [0, n_static) are dealt out statically (one contiguous range per wave); the rest form a
    // pool handed out in chunks of kDynChunk rays, one atomic per chunk, to waves whose static range
    // has run out -- equal work per wave still leaves waves finishing at different times (their
    // SIMD, CU and XCD neighbours differ), and the pool lets the fast ones finish the launch.
    const uint64_t n_dyn = (n * (uint64_t)a.dyn_share) >> 8;
    const uint32_t dyn_chunk = a.dyn_chunk;
    const uint64_t n_static = n - n_dyn;
    uint64_t w_next = n_static * wave_id / n_waves;
    uint64_t w_end = n_static * (wave_id + 1) / n_waves;
    uint32_t n_q = 0, n_rx = 0, n_miss = 0;
#if ARX_TRACE_COUNT  // measurement builds only (build.py --exp ... -D ARX_TRACE_COUNT=1)
    uint32_t n_steps = 0, n_tris = 0;
    // the scalar-fetch probe: node lane-steps whose node is the wave leader's (the first lane with a
    // node to step), and node-step slots the wave ran -- a scalar load of the leader's node could
    // serve the former without vector-memory (TD) work
    uint32_t n_leader = 0, n_slots = 0;
#endif
#if ARX_TRACE_PROF  // measurement builds only: wave-uniform tallies (popcounts of ballots)
    // [0] start [1] end [2] rays [3] queries [4] node-step slots run [5] node lane-steps [6] leaf
    // phases [7] leaf lanes [8] shade phases [9] shade lanes [10] outer iterations [11] inner
    // iterations [12] time the wave's ray range ran out [13] wave id [14] refill phases [15] -
    uint64_t pf[kProfWords] = {};
    pf[0] = __builtin_readcyclecounter();
    pf[13] = wave_id;
    // HW_REG_HW_ID (wave / SIMD / CU / SE of this wave) | HW_REG_XCC_ID << 32: s_memtime counts per
    // XCD, so start skews compare waves of one XCD only
    pf[15] = (uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 4) |
             ((uint64_t)__builtin_amdgcn_s_getreg((15 << 11) | 20) << 32);
#endif
    bool active = false, trav = false, exhausted = w_next >= w_end && n_dyn == 0;
    RayState s;
    s.depth = -1;
    Ray r;
    Trav t;
    t.best.t = __builtin_huge_valf();
    t.best.id = 0x7fffffff;
    t.best.unit = -1;
    t.node = -1;
    t.sp = 0;
    float oix = 0.f, oiy = 0.f, oiz = 0.f;
    while (true) {
#if ARX_TRACE_PROF
        ++pf[10];
        {
            const unsigned long long sh = __ballot(active && (LEAN ? t.node == -1 : !trav));
            if (sh) {
                ++pf[8];
                pf[9] += __popcll(sh);
            }
        }
#endif
        if (active && (LEAN ? t.node == -1 : !trav)) {  // the query is done: shade it
            shade(a, tbase, s, r, t.best, n_rx, n_miss);
            if (!wants_query(a, s)) active = false;
        }
        const unsigned long long need = __ballot(!active);
#if ARX_TRACE_PROF
        if (need != 0ull && !exhausted) {
            ++pf[14];
            pf[2] += std::min<uint64_t>(__popcll(need), w_end - w_next);
            if (w_next + __popcll(need) >= w_end) pf[12] = __builtin_readcyclecounter();
        }
#endif
        if (need != 0ull && !exhausted && w_next >= w_end) {  // the static range ran out: a pool chunk
            unsigned long long c = 0ull;
            if ((lane & 63) == 0) c = atomicAdd(a.cursor, (unsigned long long)dyn_chunk);
            const uint64_t start = n_static + __builtin_amdgcn_readfirstlane((uint32_t)c) +
                                   ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(c >> 32)) << 32);
            w_next = start;
            w_end = start + dyn_chunk < n ? start + dyn_chunk : n;
            if (start >= n) exhausted = true;
        }
        if (need != 0ull && !exhausted) {
            const int cnt = __popcll(need);
            const uint64_t base = w_next;
            w_next += (uint64_t)cnt;
            if (!active) {
                const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(need >> 32),
                                                                __builtin_amdgcn_mbcnt_lo((uint32_t)need, 0u));
                const uint64_t i = base + rank;
                if (i < w_end) {
                    ray_init(a, s, a.ray_begin + i);
                    active = wants_query(a, s);
                }
            }
            if (w_next >= w_end && n_dyn == 0) exhausted = true;
        }
        if (active && (LEAN ? t.node == -1 : !trav)) {
            ++n_q;
            setup_ray(r, s.pos, s.dir);
            if constexpr (Q16 || W4) {  // grid form of the slab planes (node_step, node_step_w4)
                oix = (r.o[0] - a.qgrid.origin[0]) * r.inv[0];
                oiy = (r.o[1] - a.qgrid.origin[1]) * r.inv[1];
                oiz = (r.o[2] - a.qgrid.origin[2]) * r.inv[2];
                r.inv[0] *= a.qgrid.scale[0];
                r.inv[1] *= a.qgrid.scale[1];
                r.inv[2] *= a.qgrid.scale[2];
#if ARX_TRACE_SIGNSEL && ARX_TRACE_BITFLOAT
                if constexpr (Q16) {  // node_step's C = 2^23 * ix + (o - origin) * inv, one rounding
                    oix = __builtin_fmaf(8388608.0f, r.inv[0], oix);
                    oiy = __builtin_fmaf(8388608.0f, r.inv[1], oiy);
                    oiz = __builtin_fmaf(8388608.0f, r.inv[2], oiz);
                }
#endif
            } else {
                oix = r.o[0] * r.inv[0];
                oiy = r.o[1] * r.inv[1];
                oiz = r.o[2] * r.inv[2];
            }
            t.best.t = __builtin_huge_valf();
            t.best.id = 0x7fffffff;
            t.best.unit = -1;
            t.node = 0;  // the top node (node 0; unit 0 of the CW4 buffer)
            t.sp = 0;
            trav = true;
        }
        if (__ballot(active) == 0ull) {
            if (exhausted) break;
            continue;
        }
        const unsigned long long m_active = LEAN ? __ballot(active) : 0ull;  // fixed inside the traversal loop
        while (true) {
            if (!LEAN && trav && t.node == -1) trav = false;  // query done (its stack is empty)
            const unsigned long long m_node = __ballot(t.node >= 0);
            const unsigned long long m_leaf = __ballot(t.node <= -2);
            if ((m_node | m_leaf) == 0ull) break;
            if constexpr (LEAN) {  // active lanes whose query is done (node -1) wait to be shaded
                if (lanes32(m_active & ~(m_node | m_leaf)) >= (uint32_t)THRESH) break;
            } else {
                if (__popcll(__ballot(active && !trav)) >= THRESH) break;
            }
#if ARX_TRACE_PROF
            ++pf[11];
#endif
            if (m_node != 0ull && (LEAN ? lanes32(m_leaf) < (uint32_t)LEAF_THRESH : __popcll(m_leaf) < LEAF_THRESH)) {
#pragma unroll
                for (int k = 0; k < NSTEPS; ++k) {
#if ARX_TRACE_PROF
                    const unsigned long long mk = __ballot(t.node >= 0);
                    if (mk) {
                        ++pf[4];
                        pf[5] += __popcll(mk);
                    }
#endif
#if ARX_TRACE_COUNT
                    {
                        const unsigned long long ml = __ballot(t.node >= 0);
                        if (ml) {
                            const int lead = __shfl(t.node, (int)__builtin_ctzll(ml), 64);
                            n_leader += (t.node >= 0 && t.node == lead) ? 1u : 0u;
                            n_slots += (lane & 63) == 0 ? 1u : 0u;
                        }
                    }
#endif
                    if (t.node >= 0) {
#if ARX_TRACE_COUNT
                        ++n_steps;
#endif
                        if constexpr (W4) node_step_w4(r, oix, oiy, oiz, t, stk, nrs);
                        else node_step<FMT, Stack, !LEAN>(r, oix, oiy, oiz, t, stk, nrs, ncache, qrs);
                    }
                }
            } else {
#if ARX_TRACE_PROF
                ++pf[6];
                pf[7] += __popcll(m_leaf);
#endif
#if ARX_TRACE_COUNT
                if (t.node <= -2) n_tris += (uint32_t)((~t.node) & (W4 ? 3 : 15));
#endif
                leaf_step<FMT>(trs, r, t, stk);
            }
        }
    }
#if ARX_TRACE_PROF
    {
        unsigned int vq = n_q;
        for (int off = 32; off > 0; off >>= 1) vq += __shfl_xor(vq, off, 64);
        pf[3] = vq;
        pf[1] = __builtin_readcyclecounter();
        // one word per lane (a vector store with per-lane addresses)
        const int l = lane & 63;
        uint64_t v = 0;
#pragma unroll
        for (int k = 0; k < kProfWords; ++k) v = (l == k) ? pf[k] : v;
        if (a.prof && l < kProfWords) a.prof[(uint64_t)wave_id * kProfWords + l] = v;
    }
#endif
    flush_counters(a, n_q, n_rx, n_miss, lane);
#if ARX_TRACE_COUNT  // [4] node steps, [5] leaf triangle tests (lane level), [6] leader-node lane-steps, [7] step slots
    atomicAdd(a.counters + 4, (unsigned long long)n_steps);
    atomicAdd(a.counters + 5, (unsigned long long)n_tris);
    atomicAdd(a.counters + 6, (unsigned long long)n_leader);
    atomicAdd(a.counters + 7, (unsigned long long)n_slots);
#endif
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

// dst += src over n int64 bins (a group's shards summed on one device, arx_group.cpp).
__global__ void hist_add_kernel(long long* __restrict__ dst, const long long* __restrict__ src, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] += src[i];
}

// Histogram and counters zeroed in one launch (arx_clear_histogram; two memsets were two
// launches of a few microseconds each, one of them for a few dozen bytes).
__global__ void clear_kernel(unsigned long long* __restrict__ hist, uint64_t n, unsigned long long* __restrict__ counters,
                             int n_counters) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) hist[i] = 0ull;
    if (i < (uint64_t)n_counters) counters[i] = 0ull;
}

// Direction pre-pass: float4(dir, 0) for rays [first, first + count); with clear_bins > 0 it also
// zeroes the histogram and the counters the trace accumulates into (render(): one launch fewer per
// frame, and the kernel boundary it cost).
__global__ void dirs_kernel(uint64_t seed, uint64_t first, uint64_t count, float4* out, unsigned long long* cursor,
                            unsigned long long* __restrict__ hist, uint64_t clear_bins,
                            unsigned long long* __restrict__ counters, int clear_counters) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) *cursor = 0ull;  // the trace launch's chunk pool (trace_kernel) starts empty-handed
    if (i < clear_bins) hist[i] = 0ull;
    if (i < (uint64_t)clear_counters) counters[i] = 0ull;
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

// Production tuning: 128-lane blocks, exactly kWaves waves per SIMD, shade at
// 12 idle lanes, leaves at 12 pending, 12 node steps per inner iteration.  The ARX_TRACE_* macros
// exist only for design experiments (build.py --exp builds a separate library under
// tools/experiments/); the product build never defines them.
#ifndef ARX_TRACE_THRESH
#define ARX_TRACE_THRESH 12
#endif
#ifndef ARX_TRACE_STEPS
#define ARX_TRACE_STEPS 12
#endif
#ifndef ARX_TRACE_LEAF_THRESH
#define ARX_TRACE_LEAF_THRESH 12
#endif
#ifndef ARX_TRACE_SMALL_BLOCK
#define ARX_TRACE_SMALL_BLOCK 256  // block size of launches without the ray pool (0: kBlock)
#endif
constexpr int kSmallBlock = ARX_TRACE_SMALL_BLOCK;
// ... and their node steps per inner iteration / pending leaves before a leaf batch: shorter
// iterations suit a launch whose time is its longest lane chain (C2 0.419 -> 0.403 ms with 10
// steps, 0.408 with 8 leaves; C3 unchanged within noise, profiles/r03/ab_tune.txt)
#ifndef ARX_TRACE_SMALL_STEPS
#define ARX_TRACE_SMALL_STEPS 10
#endif
#ifndef ARX_TRACE_SMALL_LEAF
#define ARX_TRACE_SMALL_LEAF 8
#endif
constexpr int kSmallSteps = ARX_TRACE_SMALL_STEPS, kSmallLeaf = ARX_TRACE_SMALL_LEAF;
// waves per SIMD the small-launch instance is compiled for
constexpr int kSmallWaves = ARX_TRACE_WAVES;
constexpr int kThresh = ARX_TRACE_THRESH, kLeafThresh = ARX_TRACE_LEAF_THRESH, kWaves = ARX_TRACE_WAVES, kSteps = ARX_TRACE_STEPS;
constexpr int kSimdsPerCu = 4;

// Persistent grid of BLOCK-lane blocks: exactly kWaves waves per SIMD on every CU, fewer blocks
// for small launches (one ray per lane).
template <int BLOCK, bool GSTACK, int FMT>
int trace_grid(const TraceArgs& args, int cus, uint64_t n_rays) {
    constexpr int per_cu = kSimdsPerCu * kWaves * 64 / BLOCK;
    static_assert(per_cu * BLOCK == kSimdsPerCu * kWaves * 64, "blocks must fill the CU's wave slots exactly");
    const uint64_t want = (n_rays + BLOCK - 1) / BLOCK;
    uint64_t cap = (uint64_t)per_cu * (uint64_t)(cus > 0 ? cus : 256);
    if (GSTACK || FMT == kFmtW4) cap = std::min<uint64_t>(cap, args.gstack_lanes / BLOCK);  // one stack column per lane
    return (int)std::max<uint64_t>(1, std::min(want, cap));
}

// The ray pool (and the kBlock instance) for launches with at least kDynMinRaysPerWave rays per wave
// of the full grid; smaller launches take the kSmallBlock instance with static ranges.
template <int FMT, bool GSTACK>
bool uses_pool(const TraceArgs& args, int cus) {
    const uint64_t n_rays = args.ray_end - args.ray_begin;
    const int grid = trace_grid<kBlock, GSTACK, FMT>(args, cus, n_rays);
    return n_rays >= (uint64_t)kDynMinRaysPerWave * (uint64_t)grid * (kBlock / 64);
}

template <int FMT, bool GSTACK>
hipError_t launch(const TraceArgs& args, int cus, hipStream_t s) {
    const uint64_t n_rays = args.ray_end - args.ray_begin;
#ifdef ARX_TRACE_DYN_LDS
    static const size_t dyn_lds = ARX_TRACE_DYN_LDS;  // design experiments only
#else
    static const size_t dyn_lds = 0;
#endif
    const int grid = trace_grid<kBlock, GSTACK, FMT>(args, cus, n_rays);
    TraceArgs a2 = args;
    const bool dyn = uses_pool<FMT, GSTACK>(args, cus);
    a2.dyn_share = dyn ? (uint32_t)kDynShare : 0u;
    a2.dyn_chunk = (uint32_t)kDynChunk;
    const uint64_t pre = std::max<uint64_t>(n_rays, args.clear_bins);
    hipLaunchKernelGGL(dirs_kernel, dim3((unsigned)((pre + 255) / 256)), dim3(256), 0, s, args.seed, args.ray_begin,
                       n_rays, reinterpret_cast<float4*>(const_cast<void*>(args.dirs)), args.cursor, args.hist,
                       args.clear_bins, args.counters, args.clear_counters);
    if (kSmallBlock > 0 && !dyn) {
        // Small launches (about a ray per lane: C2, one 8-GPU rank's C5 shard) in 4-wave blocks,
        // one wave per SIMD each: 0.465 -> 0.44 ms at C2
        constexpr int SB = kSmallBlock > 0 ? kSmallBlock : kBlock;
        const int g2 = trace_grid<SB, GSTACK, FMT>(args, cus, n_rays);
        hipLaunchKernelGGL((trace_kernel<SB, kThresh, kSmallLeaf, kSmallWaves, kSmallSteps, FMT, GSTACK, true>), dim3(g2), dim3(SB),
                           dyn_lds, s, a2);
    } else {
        hipLaunchKernelGGL((trace_kernel<kBlock, kThresh, kLeafThresh, kWaves, kSteps, FMT, GSTACK>), dim3(grid),
                           dim3(kBlock), dyn_lds, s, a2);
    }
    return hipGetLastError();
}

}  // namespace

hipError_t launch_trace(const TraceArgs& a, int cus, hipStream_t s, bool force_global_stack) {
    if (a.ray_end <= a.ray_begin) return hipSuccess;
    (void)hipGetLastError();  // report this launch's error, not a stale one of an earlier runtime call
    if (!a.dirs || !a.cnodes || !a.tris || !a.hist || !a.counters || !a.cursor) return hipErrorInvalidValue;
    if (a.wbuf) {  // CW4: LDS rows + a global overflow column per lane (W4Stack)
        if (!a.gstack || a.gstack_lanes < (uint64_t)kBlock) return hipErrorInvalidValue;
        return launch<kFmtW4, false>(a, cus, s);
    }
    const bool gstack = force_global_stack || a.bvh_depth + 1 > kLdsStack;
    if (gstack && (!a.gstack || a.gstack_lanes < (uint64_t)kBlock)) return hipErrorInvalidValue;
    if (a.qnodes) return gstack ? launch<kFmtQ16, true>(a, cus, s) : launch<kFmtQ16, false>(a, cus, s);
    return gstack ? launch<kFmtF32, true>(a, cus, s) : launch<kFmtF32, false>(a, cus, s);
}

#ifndef ARX_TRACE_SRC_ID
#define ARX_TRACE_SRC_ID 0ull  // set by build.py: hash of this kernel's sources and experiment macros
#endif
uint64_t trace_kernel_source_id() { return ARX_TRACE_SRC_ID; }

bool trace_uses_small_block(const TraceArgs& a, int cus, bool force_global_stack) {
    if (kSmallBlock <= 0 || a.ray_end <= a.ray_begin) return false;
    if (a.wbuf) return !uses_pool<kFmtW4, false>(a, cus);
    const bool gstack = force_global_stack || a.bvh_depth + 1 > kLdsStack;
    if (a.qnodes) return gstack ? !uses_pool<kFmtQ16, true>(a, cus) : !uses_pool<kFmtQ16, false>(a, cus);
    return gstack ? !uses_pool<kFmtF32, true>(a, cus) : !uses_pool<kFmtF32, false>(a, cus);
}

namespace {
template <int B, int L, int S, bool LEAN>
const void* lds_stack_instance(int fmt) {
    constexpr int W = LEAN ? kSmallWaves : kWaves;
    return fmt == kFmtW4    ? reinterpret_cast<const void*>(trace_kernel<B, kThresh, L, W, S, kFmtW4, false, LEAN>)
           : fmt == kFmtQ16 ? reinterpret_cast<const void*>(trace_kernel<B, kThresh, L, W, S, kFmtQ16, false, LEAN>)
                            : reinterpret_cast<const void*>(trace_kernel<B, kThresh, L, W, S, kFmtF32, false, LEAN>);
}
}  // namespace

hipError_t trace_kernel_occupancy(int fmt, bool small, int* vgprs, int* waves_admitted, int* waves_target) {
    hipFuncAttributes fa;
    constexpr int SB = kSmallBlock > 0 ? kSmallBlock : kBlock;
    const void* k = small ? lds_stack_instance<SB, kSmallLeaf, kSmallSteps, true>(fmt)
                          : lds_stack_instance<kBlock, kLeafThresh, kSteps, false>(fmt);
    const hipError_t e = hipFuncGetAttributes(&fa, k);
    if (e != hipSuccess) return e;
    // gfx950: 512 VGPRs per SIMD lane slot, allocated in granules of 8
    const int alloc = (fa.numRegs + 7) / 8 * 8;
    *vgprs = fa.numRegs;
    *waves_admitted = alloc > 0 ? std::min(8, 512 / alloc) : 8;
    *waves_target = small ? kSmallWaves : kWaves;
    return hipSuccess;
}

hipError_t launch_finalize_ir(const long long* hist, float* ir_left, float* ir_right, int32_t ir_len, double unit,
                              int32_t is_mono, hipStream_t s) {
    (void)hipGetLastError();
    const int b = 256;
    const int g = (ir_len + b - 1) / b;
    if (g > 0) hipLaunchKernelGGL(finalize_ir_kernel, dim3(g), dim3(b), 0, s, hist, ir_left, ir_right, ir_len, unit, is_mono);
    return hipGetLastError();
}

hipError_t launch_hist_add(long long* dst, const long long* src, uint64_t n, hipStream_t s) {
    (void)hipGetLastError();
    const uint64_t g = (n + 255) / 256;
    if (g > 0) hipLaunchKernelGGL(hist_add_kernel, dim3((unsigned)g), dim3(256), 0, s, dst, src, n);
    return hipGetLastError();
}

hipError_t launch_clear(unsigned long long* hist, uint64_t n, unsigned long long* counters, int n_counters,
                        hipStream_t s) {
    (void)hipGetLastError();
    const uint64_t m = n > (uint64_t)n_counters ? n : (uint64_t)n_counters;
    const uint64_t g = (m + 255) / 256;
    if (g > 0) hipLaunchKernelGGL(clear_kernel, dim3((unsigned)g), dim3(256), 0, s, hist, n, counters, n_counters);
    return hipGetLastError();
}

hipError_t launch_ray_directions(uint64_t seed, uint64_t first, uint64_t count, float* d_out, hipStream_t s) {
    (void)hipGetLastError();
    const int b = 256;
    const uint64_t g = (count + b - 1) / b;
    if (g > 0) hipLaunchKernelGGL(ray_dir_kernel, dim3((unsigned)g), dim3(b), 0, s, seed, first, count, d_out);
    return hipGetLastError();
}

}  // namespace arx
