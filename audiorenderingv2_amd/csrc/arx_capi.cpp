// arx_capi.cpp -- C ABI of libarx.so (include/arx.h): renderer state, scene upload,
// listener placement and the render / convolution entry points.
//
// Host-side counterpart of R/prebuild/obj_raytracer/AudioRenderer.cpp (OptiX setup,
// buildAccel, buildSBT, reload, render, convoluteAudioFile), re-designed for HIP:
// one stream per renderer, persistent device buffers (the reference cudaMallocs and
// frees inside every call, AudioRenderer.cpp:593-750), status codes instead of
// throw/exit, and no full rebuild when the listener moves.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iterator>
#include <map>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "arx_internal.hpp"

using namespace arx;

#ifndef ARX_TRACE_PROF
#define ARX_TRACE_PROF 0  // measurement builds only (build.py --exp TAG -D ARX_TRACE_PROF=1)
#endif

namespace {
thread_local std::string g_last_error;
}  // namespace

arx_status arx::fail(arx_status s, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return s;
}

// shared with arx_io.cpp so the loaders report through arx_last_error()
void arx_set_last_error(const std::string& m) { g_last_error = m; }

namespace {

float initial_energy(const arx_config& c) {
    // devicePrograms.cu:208 -- (x*y*z) is an int product in the reference
    const int32_t n = c.rays_x * c.rays_y * c.rays_z;
    return (float)((double)c.base_power / ((double)n * 4.18879020478));
}

arx_status check_config(const arx_config* c) {
    if (!c) return fail(ARX_ERR_INVALID_ARGUMENT, "config is NULL");
    if (c->rays_x <= 0 || c->rays_y <= 0 || c->rays_z <= 0)
        return fail(ARX_ERR_INVALID_ARGUMENT, "rays dims must be positive");
    if ((uint64_t)c->rays_x * (uint64_t)c->rays_y * (uint64_t)c->rays_z > 0x7fffffffull)
        return fail(ARX_ERR_INVALID_ARGUMENT, "x*y*z must fit int32 (devicePrograms.cu:208 int product)");
    if (c->sample_rate <= 0) return fail(ARX_ERR_INVALID_ARGUMENT, "sample_rate must be positive");
    if (!(c->hrtf_absorption_rate >= 0.0f && c->hrtf_absorption_rate <= 1.0f))
        return fail(ARX_ERR_INVALID_ARGUMENT, "hrtf_absorption_rate must be in [0, 1]");
    if (c->ir_length_in_seconds == 0) return fail(ARX_ERR_INVALID_ARGUMENT, "ir_length_in_seconds must be >= 1");
    const uint64_t L = (uint64_t)c->ir_length_in_seconds * (uint64_t)c->sample_rate;
    if (L > 0x7fffffffull) return fail(ARX_ERR_INVALID_ARGUMENT, "ir length too large");
    return ARX_OK;
}

// OptixModel.cpp:178-193 (glm::rotate(mat4(1), -radians(yaw), +Y) * v, then + camera),
// restated with glm's exact operation order (matrix_transform.inl rotate, type_mat4x4.inl
// operator*): x' = (c*x + R10*y) + (s*z + 0), y' = (0*x + R11*y) + (0*z + 0),
// z' = (-s*x + 0*y) + (c*z + 0) with c = cos(-a), s = sin(-a), R11 = c + (1 - c).
void place_vertices(const float* local, int64_t n_vertices, float x, float y, float z, float yaw_deg, float* out) {
    const float ang = yaw_deg * static_cast<float>(0.01745329251994329576923690768489);  // glm::radians
    const float a = -ang;
    const float c = std::cos(a);
    const float s = std::sin(a);
    const float t1 = 1.0f - c;   // temp = (1 - c) * axis, axis = (0, 1, 0)
    const float r00 = c + 0.0f * 0.0f;
    const float r10 = t1 * 0.0f - s * 0.0f;
    const float r20 = 0.0f * 0.0f + s * 1.0f;
    const float r01 = 0.0f * 1.0f + s * 0.0f;
    const float r11 = c + t1 * 1.0f;
    const float r21 = 0.0f * 1.0f - s * 0.0f;
    const float r02 = 0.0f * 0.0f - s * 1.0f;
    const float r12 = t1 * 0.0f + s * 0.0f;
    const float r22 = c + 0.0f * 0.0f;
    for (int64_t i = 0; i < n_vertices; ++i) {
        const float vx = local[3 * i + 0], vy = local[3 * i + 1], vz = local[3 * i + 2];
        const float ox = (r00 * vx + r10 * vy) + (r20 * vz + 0.0f * 1.0f);
        const float oy = (r01 * vx + r11 * vy) + (r21 * vz + 0.0f * 1.0f);
        const float oz = (r02 * vx + r12 * vy) + (r22 * vz + 0.0f * 1.0f);
        out[3 * i + 0] = x + ox;
        out[3 * i + 1] = y + oy;
        out[3 * i + 2] = z + oz;
    }
}

// Rotation of place_vertices (row-major r00 r10 r20 / r01 r11 r21 / r02 r12 r22), exactly its floats.
void receiver_rotation(float yaw_deg, float m[9]) {
    const float ang = yaw_deg * static_cast<float>(0.01745329251994329576923690768489);
    const float a = -ang, c = std::cos(a), s = std::sin(a), t1 = 1.0f - c;
    m[0] = c + 0.0f * 0.0f; m[1] = t1 * 0.0f - s * 0.0f; m[2] = 0.0f * 0.0f + s * 1.0f;
    m[3] = 0.0f * 1.0f + s * 0.0f; m[4] = c + t1 * 1.0f; m[5] = 0.0f * 1.0f - s * 0.0f;
    m[6] = 0.0f * 0.0f - s * 1.0f; m[7] = t1 * 0.0f + s * 0.0f; m[8] = c + 0.0f * 0.0f;
}

// The receiver sub-tree, built once in the receiver's local frame whenever the receiver model or
// the scene changes (its triangle ids and offsets follow the scene); listener moves refit it on
// the device (arx_receiver.hip).  Larger receivers than the refit kernel's LDS holds are rebuilt on
// the host per move instead (recv_refit = false).
arx_status prepare_receiver_model(arx_renderer* r) {
    std::vector<float> tv, ab;
    float radius = 0.0f;
    for (int side = 0; side < 2; ++side) {
        const std::vector<float>& loc = r->recv_local[side];
        tv.insert(tv.end(), loc.begin(), loc.end());
        ab.insert(ab.end(), loc.size() / 9, side == 0 ? -1.0f : -2.0f);
        for (size_t i = 0; i + 2 < loc.size(); i += 3)
            radius = std::max(radius, std::sqrt(loc[i] * loc[i] + loc[i + 1] * loc[i + 1] + loc[i + 2] * loc[i + 2]));
    }
    const int64_t n = (int64_t)ab.size();
    r->recv_refit = n <= kRefitMaxTris;
    r->recv_radius = radius * 1.0001f + 1e-6f;  // |R v| = |v|: the rotated halves stay in this ball
    if (!r->recv_refit) return ARX_OK;
    const BvhBuild& sc = r->scene_img->bvh;
    build_bvh(tv.data(), ab.data(), 0.0f, n, (int32_t)r->scene_img->n_input, r->recv);
    relocate_bvh(r->recv, 1 + (int32_t)sc.nodes.size(), (int32_t)sc.tris.size());
    const char* why = "";
    const size_t total_nodes = 1 + sc.nodes.size() + r->recv.nodes.size();
    const size_t total_tris = sc.tris.size() + r->recv.tris.size();
    if (!validate_bvh_range(r->recv.nodes.data(), 1 + sc.nodes.size(), r->recv.nodes.size(), total_nodes,
                            total_tris, &why))
        return fail(ARX_ERR_INTERNAL, "BVH validation failed (receiver): %s", why);
    // refit schedule: inner nodes by depth, deepest level first
    const int32_t base = 1 + (int32_t)sc.nodes.size();
    std::vector<int32_t> depth(r->recv.nodes.size(), 0);
    int32_t max_d = 0;
    for (size_t i = 0; i < r->recv.nodes.size(); ++i)  // parents precede children (pre-order)
        for (int c = 0; c < 2; ++c)
            if (r->recv.nodes[i].d[2 + c] == 0) {
                const int32_t ch = r->recv.nodes[i].d[c] - base;
                depth[(size_t)ch] = depth[i] + 1;
                max_d = std::max(max_d, depth[(size_t)ch]);
            }
    std::vector<int32_t> order, start;
    for (int32_t d = max_d; d >= 0 && !r->recv.nodes.empty(); --d) {
        start.push_back((int32_t)order.size());
        for (size_t i = 0; i < r->recv.nodes.size(); ++i)
            if (depth[i] == d) order.push_back((int32_t)i);
    }
    start.push_back((int32_t)order.size());
    r->recv_levels = r->recv.nodes.empty() ? 0 : (int32_t)start.size() - 1;
    if (receiver_refit_lds((int32_t)r->recv.tris.size(), (int32_t)r->recv.nodes.size(), r->recv_levels) > 160 * 1024) {
        r->recv_refit = false;  // beyond one workgroup's LDS: rebuilt on the host per move instead
        return ARX_OK;
    }
    hipFree(r->d_recv_local);
    hipFree(r->d_recv_nodes);
    hipFree(r->d_recv_levels);
    r->d_recv_local = nullptr;
    r->d_recv_nodes = nullptr;
    r->d_recv_levels = nullptr;
    ARX_HIP(hipMalloc(&r->d_recv_local, std::max<size_t>(1, r->recv.tris.size()) * sizeof(TriRec)));
    ARX_HIP(hipMalloc(&r->d_recv_nodes, std::max<size_t>(1, r->recv.nodes.size()) * sizeof(BvhNode)));
    ARX_HIP(hipMalloc(&r->d_recv_levels, (order.size() + start.size()) * sizeof(int32_t)));
    if (!r->recv.tris.empty())
        ARX_HIP(hipMemcpyAsync(r->d_recv_local, r->recv.tris.data(), r->recv.tris.size() * sizeof(TriRec),
                               hipMemcpyHostToDevice, r->stream));
    if (!r->recv.nodes.empty())
        ARX_HIP(hipMemcpyAsync(r->d_recv_nodes, r->recv.nodes.data(), r->recv.nodes.size() * sizeof(BvhNode),
                               hipMemcpyHostToDevice, r->stream));
    std::vector<int32_t> lv(order);
    lv.insert(lv.end(), start.begin(), start.end());
    ARX_HIP(hipMemcpyAsync(r->d_recv_levels, lv.data(), lv.size() * sizeof(int32_t), hipMemcpyHostToDevice, r->stream));
    ARX_HIP(hipStreamSynchronize(r->stream));  // pageable sources
    r->recv_level_count = (int32_t)order.size();
    if (!r->use_w4) return ARX_OK;
    // opt-in CW4 path only: the receiver's CW4 layout (root at unit kW4RecvRoot, blocks after the
    // scene's) for the refit
    collapse_w4(r->recv, base, (int32_t)sc.tris.size(), r->recv.root, kW4RecvRoot, r->scene_img->wide().w4.unit_end,
                r->recv4);
    std::vector<int32_t> w4n(11 * r->recv4.nodes.size()), w4t(2 * r->recv4.leaf_tris.size());
    for (size_t i = 0; i < r->recv4.nodes.size(); ++i) {
        std::copy(r->recv4.src.begin() + 8 * i, r->recv4.src.begin() + 8 * i + 8, w4n.begin() + 11 * i);
        w4n[11 * i + 8] = (int32_t)r->recv4.nodes[i].meta;
        w4n[11 * i + 9] = (int32_t)r->recv4.nodes[i].base;
        w4n[11 * i + 10] = (int32_t)r->recv4.nodes[i].self;
    }
    for (size_t i = 0; i < r->recv4.leaf_tris.size(); ++i) {
        w4t[2 * i] = (int32_t)r->recv4.leaf_tris[i].first;
        w4t[2 * i + 1] = r->recv4.leaf_tris[i].second;
    }
    hipFree(r->d_recv_w4);
    hipFree(r->d_recv_w4_tris);
    r->d_recv_w4 = nullptr;
    r->d_recv_w4_tris = nullptr;
    ARX_HIP(hipMalloc(&r->d_recv_w4, std::max<size_t>(1, w4n.size()) * sizeof(int32_t)));
    ARX_HIP(hipMalloc(&r->d_recv_w4_tris, std::max<size_t>(1, w4t.size()) * sizeof(int32_t)));
    if (!w4n.empty())
        ARX_HIP(hipMemcpyAsync(r->d_recv_w4, w4n.data(), w4n.size() * sizeof(int32_t), hipMemcpyHostToDevice, r->stream));
    if (!w4t.empty())
        ARX_HIP(hipMemcpyAsync(r->d_recv_w4_tris, w4t.data(), w4t.size() * sizeof(int32_t), hipMemcpyHostToDevice,
                               r->stream));
    ARX_HIP(hipStreamSynchronize(r->stream));  // pageable sources
    return ARX_OK;
}

// Box padding of the refit kernel (RefitArgs::pad): at least the builder's 1e-5 * max|coordinate|
// for any vertex of the placed receiver (|v| <= |center| + radius).
float refit_pad(const arx_renderer* r) {
    float mx = 0.0f;
    for (int k = 0; k < 3; ++k) mx = std::max(mx, std::fabs(r->center[k]));
    return std::max(1e-5f * (mx + r->recv_radius) * 1.001f, 1e-6f);
}

// World-space bound of the placed receiver (for the quantization grid): the refit path's ball
// widened by the refit kernel's box padding (the padded boxes it quantizes must stay on the grid),
// or the host-built sub-tree's root box.
void receiver_bound(const arx_renderer* r, float lo[3], float hi[3], bool* empty) {
    *empty = (r->recv_local[0].size() + r->recv_local[1].size()) == 0;
    const float pad = r->recv_refit ? refit_pad(r) : 0.0f;
    for (int k = 0; k < 3; ++k) {
        if (r->recv_refit) {
            lo[k] = r->center[k] - r->recv_radius - 2.0f * pad;
            hi[k] = r->center[k] + r->recv_radius + 2.0f * pad;
        } else {
            lo[k] = r->recv.root.lo[k];
            hi[k] = r->recv.root.hi[k];
        }
    }
}

// The trace kernel addresses nodes and triangle records through buffer resources with 32-bit byte
// offsets and num_records 0x7fffffff (arx_trace.hip buffer_rsrc; a load past it returns zeros, which
// the leaf step uses for idle lanes): every record must end below 2^31 bytes, or a triangle would read
// back as zeros (det 0, a silently dropped hit).  44.7 M triangle records / 33.5 M coded nodes.

// Frames in flight (no-ops with one): the current set's stream waits for every other set's last
// trace / for the set that did the last step of a chain (convolutions, all-reduces, scene writes),
// and records its own.
using FifEvents = hipEvent_t[arx_renderer::kMaxFrames];
arx_status fif_wait_all(arx_renderer* r, FifEvents& ev) {
    if (r->fif > 1)
        for (int s = 0; s < r->fif; ++s)
            if (s != r->slot) ARX_HIP(hipStreamWaitEvent(r->stream, ev[s], 0));
    return ARX_OK;
}
arx_status fif_done_one(arx_renderer* r, FifEvents& ev) {
    if (r->fif > 1) ARX_HIP(hipEventRecord(ev[r->slot], r->stream));
    return ARX_OK;
}
arx_status fif_wait_last(arx_renderer* r, FifEvents& ev, int32_t last) {
    if (r->fif > 1 && last >= 0 && last != r->slot) ARX_HIP(hipStreamWaitEvent(r->stream, ev[last], 0));
    return ARX_OK;
}
arx_status fif_done_last(arx_renderer* r, FifEvents& ev, int32_t& last) {
    if (r->fif > 1) {
        ARX_HIP(hipEventRecord(ev[r->slot], r->stream));
        last = r->slot;
    }
    return ARX_OK;
}

arx_status ensure_device_scene(arx_renderer* r) {
    if (!r->scene_img) return fail(ARX_ERR_NOT_READY, "arx_set_scene has not been called");
    const bool writes = r->scene_dirty || r->recv_model_dirty || r->recv_pose_dirty || !r->qgrid_set;
    if (writes) {
        // the uploads, re-quantization and receiver refit below write the tree the other frame in
        // flight may still be tracing
        const arx_status st = fif_wait_traced(r);
        if (st != ARX_OK) return st;
        ++r->tree_gen;  // this write's off-grid flag value (arx_renderer::d_tree_flag)
    }
    const SceneImage& img = *r->scene_img;
    const BvhBuild& sc = img.bvh;
    const bool model_changed = r->recv_model_dirty || r->scene_dirty;
    if (model_changed) {
        arx_status st = prepare_receiver_model(r);
        if (st != ARX_OK) return st;
    }
    const bool pose_changed = model_changed || r->recv_pose_dirty;
    if (!r->recv_refit && pose_changed) {
        // host path (receivers beyond the refit kernel's capacity): receiver halves placed in world
        // space, left then right (placeReceiver OptixModel.cpp:153-157), sub-tree rebuilt
        std::vector<float> tv;
        std::vector<float> ab;
        for (int side = 0; side < 2; ++side) {
            const std::vector<float>& loc = r->recv_local[side];
            const int64_t nt = (int64_t)loc.size() / 9;
            size_t base = tv.size();
            tv.resize(base + loc.size());
            place_vertices(loc.data(), 3 * nt, r->center[0], r->center[1], r->center[2], r->yaw, tv.data() + base);
            ab.insert(ab.end(), (size_t)nt, side == 0 ? -1.0f : -2.0f);
        }
        build_bvh(tv.data(), ab.data(), 0.0f, (int64_t)ab.size(), (int32_t)img.n_input, r->recv);
        relocate_bvh(r->recv, 1 + (int32_t)sc.nodes.size(), (int32_t)sc.tris.size());
        if (r->use_w4)
            collapse_w4(r->recv, 1 + (int32_t)sc.nodes.size(), (int32_t)sc.tris.size(), r->recv.root, kW4RecvRoot,
                        img.wide().w4.unit_end, r->recv4);
    }
    const size_t n_nodes = 1 + sc.nodes.size() + r->recv.nodes.size();
    const size_t n_tris = sc.tris.size() + r->recv.tris.size();
    arx_status fit = check_buffer_offsets(n_nodes, n_tris);
    if (fit != ARX_OK) return fit;
    bool full = r->scene_dirty;
    if (n_nodes > r->nodes_cap) {
        if (r->d_cnodes) ARX_HIP(hipFree(r->d_cnodes));
        if (r->d_qnodes) ARX_HIP(hipFree(r->d_qnodes));
        r->d_cnodes = nullptr;
        r->d_qnodes = nullptr;
        size_t cap = n_nodes + 1024;
        ARX_HIP(hipMalloc(&r->d_cnodes, cap * sizeof(BvhNode)));
        ARX_HIP(hipMalloc(&r->d_qnodes, cap * sizeof(QNode2)));
        r->nodes_cap = cap;
        full = true;
    }
    if (n_tris > r->tris_cap || r->d_tris == nullptr) {
        if (r->d_tris) ARX_HIP(hipFree(r->d_tris));
        r->d_tris = nullptr;
        size_t cap = std::max<size_t>(n_tris + 4096, 1);
        ARX_HIP(hipMalloc(&r->d_tris, cap * sizeof(TriRec)));
        r->tris_cap = cap;
        full = true;
    }
    // CW4 (opt-in, use_w4 only): the buffer holds the scene's units, then the receiver's; the f32
    // records are the top node, the scene's nodes and (host-built receivers) the receiver's
    static const SceneImage::Wide kNoWide;
    const SceneImage::Wide& wide = r->use_w4 ? img.wide() : kNoWide;
    const size_t w_units = r->use_w4 ? std::max<size_t>(r->recv4.unit_end, wide.w4.unit_end) : 0;
    const size_t host_recv_w4 = (r->recv_refit || !r->use_w4) ? 0 : r->recv4.nodes.size();
    const size_t n_w4f = r->use_w4 ? 1 + wide.w4.nodes.size() + host_recv_w4 : 0;
    if (w_units > r->wbuf_cap) {
        if (r->d_wbuf) ARX_HIP(hipFree(r->d_wbuf));
        r->d_wbuf = nullptr;
        const size_t cap = w_units + 4096;
        ARX_HIP(hipMalloc(&r->d_wbuf, cap * 16));
        r->wbuf_cap = cap;
        full = true;
    }
    if (n_w4f > r->w4f_cap) {
        if (r->d_w4f) ARX_HIP(hipFree(r->d_w4f));
        r->d_w4f = nullptr;
        const size_t cap = n_w4f + 1024;
        ARX_HIP(hipMalloc(&r->d_w4f, cap * sizeof(W4NodeF)));
        r->w4f_cap = cap;
        full = true;
    }
    r->n_w4f = n_w4f;
    // The quantization grid: made when the scene changes, grown when the receiver leaves it (a
    // listener walking out of the room): the new grid spans the old one, the scene, the receiver
    // and the emitter with half the extent as margin, so such a walk re-grids once or twice, not
    // per frame.  Either way the quantized copy is re-made on the device from the coded nodes
    // (launch_requant16): no host quantization, no upload, no synchronisation inside a frame.  An
    // emitter off the grid (checked per launch, arx_trace_rays) makes that launch take the f32 nodes.
    float rlo[3], rhi[3];
    bool recv_empty = false;
    receiver_bound(r, rlo, rhi, &recv_empty);
    const bool grow = !full && r->qgrid_set && pose_changed && !recv_empty && !qgrid_contains(r->qgrid, rlo, rhi);
    const bool regrid = full || !r->qgrid_set || grow;
    if (regrid) {
        float lo[3], hi[3];
        for (int k = 0; k < 3; ++k) {
            lo[k] = hi[k] = r->emitter[k];
            if (sc.root.count >= 0) {
                lo[k] = std::min(lo[k], sc.root.lo[k]);
                hi[k] = std::max(hi[k], sc.root.hi[k]);
            }
            if (!recv_empty) {
                lo[k] = std::min(lo[k], rlo[k]);
                hi[k] = std::max(hi[k], rhi[k]);
            }
            if (grow) {
                lo[k] = std::min(lo[k], r->qgrid.origin[k]);
                hi[k] = std::max(hi[k], r->qgrid.origin[k] + 65000.0f * r->qgrid.scale[k]);
            }
        }
        r->qgrid = make_qgrid(lo, hi, grow ? 0.5 : 0.1);
        r->qgrid_set = true;
    }
    const bool host_recv = !r->recv_refit;
    const bool top_changed = full || model_changed || (host_recv && pose_changed);
    if (full || top_changed) {
        // host uploads, only when the scene or the receiver model changed, or on the host-receiver
        // path: the top node (its receiver child comes from the refit kernel on the refit path),
        // the scene's coded nodes and triangles, the receiver part on the host path
        BvhNode top = make_node(sc.root, host_recv ? r->recv.root : empty_child());
        const char* why = "";
        if ((host_recv && !validate_bvh_range(r->recv.nodes.data(), 1 + sc.nodes.size(), r->recv.nodes.size(), n_nodes,
                                              n_tris, &why)) ||
            !validate_bvh_range(&top, 0, 1, n_nodes, n_tris, &why))
            return fail(ARX_ERR_INTERNAL, "BVH validation failed: %s", why);
        BvhNode ctop;  // pageable sources below live until the synchronisation at the end of this block
        code_nodes(&top, 1, &ctop);
        std::vector<BvhNode> crecv(host_recv ? r->recv.nodes.size() : 0);
        if (host_recv) code_nodes(r->recv.nodes.data(), r->recv.nodes.size(), crecv.data());
        ARX_HIP(hipMemcpyAsync(r->d_cnodes, &ctop, sizeof(BvhNode), hipMemcpyHostToDevice, r->stream));
        if (full && !img.coded.empty())
            ARX_HIP(hipMemcpyAsync(r->d_cnodes + 1, img.coded.data(), img.coded.size() * sizeof(BvhNode),
                                   hipMemcpyHostToDevice, r->stream));
        if (full && !sc.tris.empty())
            ARX_HIP(hipMemcpyAsync(r->d_tris, sc.tris.data(), sc.tris.size() * sizeof(TriRec), hipMemcpyHostToDevice,
                                   r->stream));
        if (host_recv && !crecv.empty())
            ARX_HIP(hipMemcpyAsync(r->d_cnodes + 1 + sc.nodes.size(), crecv.data(), crecv.size() * sizeof(BvhNode),
                                   hipMemcpyHostToDevice, r->stream));
        if (host_recv && !r->recv.tris.empty())
            ARX_HIP(hipMemcpyAsync(r->d_tris + sc.tris.size(), r->recv.tris.data(), r->recv.tris.size() * sizeof(TriRec),
                                   hipMemcpyHostToDevice, r->stream));
        // CW4 (opt-in): the scene's buffer image and node records once per scene; the top node's
        // record (child 0 the scene root, child 1 the host-built receiver's root or, on the refit
        // path, a placeholder the refit kernel replaces); a host-built receiver's records and triangles
        std::vector<uint32_t> rimage;
        if (r->use_w4) {
            W4NodeF wtop;
            std::memset(&wtop, 0, sizeof(wtop));
            wtop.base = kW4SceneRoot;
            wtop.self = 0;
            if (sc.root.count >= 0) {
                wtop.meta |= 1u;
                for (int k = 0; k < 3; ++k) {
                    wtop.lo[0][k] = sc.root.lo[k];
                    wtop.hi[0][k] = sc.root.hi[k];
                }
            }
            if (host_recv && r->recv.root.count >= 0) {
                wtop.meta |= 1u << 2;
                for (int k = 0; k < 3; ++k) {
                    wtop.lo[1][k] = r->recv.root.lo[k];
                    wtop.hi[1][k] = r->recv.root.hi[k];
                }
            }
            ARX_HIP(hipMemcpyAsync(r->d_w4f, &wtop, sizeof(W4NodeF), hipMemcpyHostToDevice, r->stream));
            if (full && !wide.wimage.empty())
                ARX_HIP(hipMemcpyAsync(r->d_wbuf, wide.wimage.data(), wide.wimage.size() * sizeof(uint32_t),
                                       hipMemcpyHostToDevice, r->stream));
            if (full && !wide.w4.nodes.empty())
                ARX_HIP(hipMemcpyAsync(r->d_w4f + 1, wide.w4.nodes.data(), wide.w4.nodes.size() * sizeof(W4NodeF),
                                       hipMemcpyHostToDevice, r->stream));
            if (host_recv) {
                if (!r->recv4.nodes.empty())
                    ARX_HIP(hipMemcpyAsync(r->d_w4f + 1 + wide.w4.nodes.size(), r->recv4.nodes.data(),
                                           r->recv4.nodes.size() * sizeof(W4NodeF), hipMemcpyHostToDevice, r->stream));
                const size_t u0 = wide.w4.unit_end;
                rimage.assign((r->recv4.unit_end - u0) * 4, 0u);
                for (const auto& lt : r->recv4.leaf_tris)
                    std::memcpy(rimage.data() + (size_t)(lt.first - u0) * 4, &r->recv.tris[(size_t)lt.second], sizeof(TriRec));
                if (!rimage.empty())
                    ARX_HIP(hipMemcpyAsync(r->d_wbuf + u0, rimage.data(), rimage.size() * sizeof(uint32_t),
                                           hipMemcpyHostToDevice, r->stream));
            }
        }
        ARX_HIP(hipStreamSynchronize(r->stream));
    }
    if (regrid || top_changed) {
        // the quantized copy of the top node and the scene (and the host-built receiver) from the
        // coded nodes on the device; on the refit path the refit below writes the receiver's
        // quantized nodes itself (its coded ones may not exist yet)
        const size_t nq = host_recv ? n_nodes : 1 + sc.nodes.size();
        ARX_HIP(launch_requant16(r->d_cnodes, nq, r->qgrid, r->d_qnodes, r->d_tree_flag, r->tree_gen, r->stream));
        if (r->use_w4)
            ARX_HIP(launch_requant_w4(r->d_w4f, r->n_w4f, r->qgrid, r->d_wbuf, r->d_tree_flag, r->tree_gen, r->stream));
        ++r->requants;
    }
    r->q_valid = recv_empty || qgrid_contains(r->qgrid, rlo, rhi);
    if (r->recv_refit && (pose_changed || full || regrid)) {
        // the listener move itself: one kernel, no host copies, no synchronisation
        RefitArgs a;
        std::memset(&a, 0, sizeof(a));
        a.local_tris = r->d_recv_local;
        a.n_tris = (int32_t)r->recv.tris.size();
        a.tri_base = (int32_t)sc.tris.size();
        a.local_nodes = r->d_recv_nodes;
        a.n_nodes = (int32_t)r->recv.nodes.size();
        a.node_base = 1 + (int32_t)sc.nodes.size();
        a.level_nodes = r->d_recv_levels;
        a.level_start = r->d_recv_levels + r->recv_level_count;
        a.n_levels = r->recv_levels;
        a.root_ref = r->recv.root.ref;
        a.root_count = r->recv.root.count;
        receiver_rotation(r->yaw, a.m);
        for (int k = 0; k < 3; ++k) a.t[k] = r->center[k];
        // >= the builder's pad; receiver_bound covers it (a debug pad does not: the off-grid test)
        a.pad = r->debug_refit_pad > 0.0f ? r->debug_refit_pad : refit_pad(r);
        a.grid = r->qgrid;
        a.tris = r->d_tris;
        a.cnodes = r->d_cnodes;
        a.qnodes = r->q_valid ? r->d_qnodes : nullptr;
        a.flag = r->d_tree_flag;
        a.flag_value = r->tree_gen;
        if (r->q_valid && r->use_w4) {  // the opt-in CW4 copy follows the quantized one (same grid)
            a.wbuf = r->d_wbuf;
            a.w4_nodes = r->d_recv_w4;
            a.n_w4 = (int32_t)r->recv4.nodes.size();
            a.w4_tris = r->d_recv_w4_tris;
            a.n_w4_tris = (int32_t)r->recv4.leaf_tris.size();
            a.scene_nonempty = sc.root.count >= 0 ? 1 : 0;
            for (int k = 0; k < 3; ++k) {
                a.scene_lo[k] = sc.root.lo[k];
                a.scene_hi[k] = sc.root.hi[k];
            }
        }
        if (a.n_tris > 0) ARX_HIP(launch_receiver_refit(a, r->stream));
    }
    r->scene_dirty = false;
    r->recv_model_dirty = false;
    r->recv_pose_dirty = false;
    if (writes) {  // the other frame set's next trace waits for these writes
        const arx_status st = fif_done_last(r, r->ev_scene, r->last_scene);
        if (st != ARX_OK) return st;
    }
    r->stats.n_scene_tris = img.n_input;
    r->stats.n_receiver_tris = (int64_t)r->recv.tris.size();
    r->stats.n_nodes = (int64_t)n_nodes;
    r->stats.bvh_depth = 1 + std::max(sc.depth, r->recv.depth);
    r->stats.tree_hash = img.hash;
    r->depth4 = r->use_w4 ? 1 + std::max(wide.w4.depth, r->recv4.depth) : 0;
    return ARX_OK;
}

}  // namespace

// A streaming convolution (arx_stream_*).  It belongs to its renderer: arx_destroy releases the
// device side of every stream still attached (r = NULL afterwards), so a stream outliving its
// renderer fails cleanly instead of touching freed memory.
struct arx_stream {
    arx_renderer* r = nullptr;
    int device = 0;
    StreamPlan* plan = nullptr;
    uint64_t ir_generation = ~0ull;  // the IR the partition spectra were made from
    double* d_in = nullptr;          // host-API staging: block frames in, 2 * block out
    double* d_out = nullptr;
};

namespace {
void release_stream(arx_stream* s) {
    hipSetDevice(s->device);
    if (s->r) sync_renderer(s->r);
    if (s->plan) stream_plan_destroy(s->plan);
    hipFree(s->d_in);
    hipFree(s->d_out);
    s->plan = nullptr;
    s->d_in = s->d_out = nullptr;
    s->r = nullptr;
}

arx_status live_stream(const arx_stream* s) {
    if (!s) return fail(ARX_ERR_INVALID_ARGUMENT, "stream is NULL");
    if (!s->r) return fail(ARX_ERR_NOT_READY, "the stream's renderer was destroyed");
    return ARX_OK;
}
}  // namespace

namespace {
std::atomic<uint64_t> g_scene_builds{0};

// 64-bit content hash (word-wise multiply / xor-shift mix; not cryptographic): identifies a built
// tree in stored profiles (arx_stats::tree_hash).
uint64_t hash_words(const void* p, size_t bytes, uint64_t h) {
    const uint8_t* b = static_cast<const uint8_t*>(p);
    size_t i = 0;
    for (; i + 8 <= bytes; i += 8) {
        uint64_t w;
        std::memcpy(&w, b + i, 8);
        h ^= w * 0x9E3779B97F4A7C15ull;
        h = (h << 27 | h >> 37) * 0xC2B2AE3D27D4EB4Full;
    }
    for (; i < bytes; ++i) h = (h ^ b[i]) * 0x100000001B3ull;
    h ^= h >> 33;
    h *= 0xFF51AFD7ED558CCDull;
    h ^= h >> 33;
    return h;
}

uint64_t scene_hash(const BvhBuild& b) {
    uint64_t h = hash_words(b.nodes.data(), b.nodes.size() * sizeof(BvhNode), 0x243F6A8885A308D3ull);
    return hash_words(b.tris.data(), b.tris.size() * sizeof(TriRec), h);
}

// serialized scene: header, nodes, triangle records
struct SceneHeader {
    uint64_t magic;
    uint64_t n_nodes, n_tris;
    int64_t n_input;
    uint64_t hash;
    ChildRef root;
    int32_t depth;
    int32_t pad;
};
constexpr uint64_t kSceneMagic = 0x3145435341585241ull;  // "ARXSCE1"
}  // namespace

arx_status arx::check_scene_input(const float* tri_v, const float* tri_abs, int64_t n) {
    if (n < 0 || (n > 0 && (!tri_v || !tri_abs))) return fail(ARX_ERR_INVALID_ARGUMENT, "bad scene arrays");
    if (n > (int64_t)0x3fffffff) return fail(ARX_ERR_INVALID_ARGUMENT, "too many triangles");
    for (int64_t i = 0; i < 9 * n; ++i)
        if (!std::isfinite(tri_v[i])) return fail(ARX_ERR_INVALID_ARGUMENT, "non-finite vertex at %lld", (long long)i / 9);
    // absorption in [0, 1], or the receiver marks -1 / -2 (getMaterialAbsorption): the int64
    // fixed-point histogram's headroom (arx_frac_bits) assumes a ray's energy never grows
    for (int64_t i = 0; i < n; ++i) {
        const float ab = tri_abs[i];
        if (!(ab >= 0.0f && ab <= 1.0f) && ab != -1.0f && ab != -2.0f)
            return fail(ARX_ERR_INVALID_ARGUMENT, "absorption %g of triangle %lld: must be in [0, 1] (or -1 / -2 receiver)",
                        (double)ab, (long long)i);
    }
    return ARX_OK;
}

namespace {
// The part of a scene image derived from its BVH2: the coded copy.
void finish_scene_image(SceneImage& img) {
    img.coded.resize(img.bvh.nodes.size());
    code_nodes(img.bvh.nodes.data(), img.bvh.nodes.size(), img.coded.data());
}
}  // namespace

// The opt-in CW4 collapse and its buffer's triangle image, made once, on first request.
const SceneImage::Wide& SceneImage::wide() const {
    std::call_once(wide_once_, [this] {
        collapse_w4(bvh, 1, 0, bvh.root, kW4SceneRoot, kW4SceneUnit, wide_.w4);
        wide_.wimage.assign((size_t)wide_.w4.unit_end * 4, 0u);
        for (const auto& lt : wide_.w4.leaf_tris)
            std::memcpy(wide_.wimage.data() + (size_t)lt.first * 4, &bvh.tris[(size_t)lt.second], sizeof(TriRec));
    });
    return wide_;
}

namespace {
// Process-wide cache of built scenes, keyed by a 128-bit hash of the input arrays: renderers and
// groups given the same geometry (a second group for frames in flight, a C++ shim beside a Python
// renderer) share one build.  Weak references: a scene no renderer holds any more is rebuilt.
std::mutex g_scene_cache_mu;
std::map<std::pair<uint64_t, uint64_t>, std::weak_ptr<const SceneImage>> g_scene_cache;
}  // namespace

// The builder settings a tree depends on (build_params(): leaf size from arx_debug_set_leaf_max,
// the tools' edits), hashed field by field so the scene cache never hands out a tree built with
// other settings.  `threads` only changes the build's speed, not its result.
uint64_t build_params_hash() {
    const BuildParams& b = build_params();
    const int32_t iv[] = {b.bins, b.leaf_max, b.spatial ? 1 : 0, b.spatial_bins, b.spatial_max_depth, b.max_depth,
                          b.rotation_passes};
    const float fv[] = {b.trav_cost, b.isect_cost, b.spatial_alpha, b.spatial_budget};
    return hash_words(fv, sizeof(fv), hash_words(iv, sizeof(iv), 0xB7E151628AED2A6Bull));
}

SceneRef arx::build_scene_image(const float* tri_v, const float* tri_abs, int64_t n) {
    const size_t bytes = (size_t)(n > 0 ? n : 0);
    const uint64_t prm = build_params_hash();
    const std::pair<uint64_t, uint64_t> key{
        hash_words(tri_abs, bytes * sizeof(float), hash_words(tri_v, 9 * bytes * sizeof(float), 0x9E3779B97F4A7C15ull)) ^ prm,
        hash_words(tri_v, 9 * bytes * sizeof(float), hash_words(tri_abs, bytes * sizeof(float), 0x6A09E667F3BCC909ull) ^
                                                         (uint64_t)n)};
    {
        std::lock_guard<std::mutex> lock(g_scene_cache_mu);
        auto it = g_scene_cache.find(key);
        if (it != g_scene_cache.end()) {
            if (SceneRef hit = it->second.lock()) return hit;
            g_scene_cache.erase(it);
        }
    }
    auto img = std::make_shared<SceneImage>();
    build_bvh(tri_v, tri_abs, 0.5f, n, 0, img->bvh);
    bfs_prefix_order(img->bvh, 1023);  // the top levels of the scene tree breadth-first (node locality)
    relocate_bvh(img->bvh, 1, 0);
    finish_scene_image(*img);
    img->n_input = n;
    img->hash = scene_hash(img->bvh);
    g_scene_builds.fetch_add(1);
    std::lock_guard<std::mutex> lock(g_scene_cache_mu);
    for (auto it = g_scene_cache.begin(); it != g_scene_cache.end();)  // drop scenes nobody holds any more
        it = it->second.expired() ? g_scene_cache.erase(it) : std::next(it);
    g_scene_cache[key] = img;
    return img;
}

std::vector<uint8_t> arx::serialize_scene(const SceneImage& s) {
    SceneHeader h;
    std::memset(&h, 0, sizeof(h));
    h.magic = kSceneMagic;
    h.n_nodes = s.bvh.nodes.size();
    h.n_tris = s.bvh.tris.size();
    h.n_input = s.n_input;
    h.hash = s.hash;
    h.root = s.bvh.root;
    h.depth = s.bvh.depth;
    const size_t nb = h.n_nodes * sizeof(BvhNode), tb = h.n_tris * sizeof(TriRec);
    std::vector<uint8_t> out(sizeof(h) + nb + tb);
    std::memcpy(out.data(), &h, sizeof(h));
    if (nb) std::memcpy(out.data() + sizeof(h), s.bvh.nodes.data(), nb);
    if (tb) std::memcpy(out.data() + sizeof(h) + nb, s.bvh.tris.data(), tb);
    return out;
}

SceneRef arx::deserialize_scene(const uint8_t* p, size_t n, const char** why) {
    SceneHeader h;
    if (!p || n < sizeof(h)) {
        *why = "short scene image";
        return nullptr;
    }
    std::memcpy(&h, p, sizeof(h));
    if (h.magic != kSceneMagic || h.n_nodes > (1ull << 31) || h.n_tris > (1ull << 31) ||
        n != sizeof(h) + h.n_nodes * sizeof(BvhNode) + h.n_tris * sizeof(TriRec)) {
        *why = "malformed scene image";
        return nullptr;
    }
    auto img = std::make_shared<SceneImage>();
    img->bvh.nodes.resize(h.n_nodes);
    img->bvh.tris.resize(h.n_tris);
    if (h.n_nodes) std::memcpy(img->bvh.nodes.data(), p + sizeof(h), h.n_nodes * sizeof(BvhNode));
    if (h.n_tris)
        std::memcpy(img->bvh.tris.data(), p + sizeof(h) + h.n_nodes * sizeof(BvhNode), h.n_tris * sizeof(TriRec));
    img->bvh.root = h.root;
    img->bvh.depth = h.depth;
    img->n_input = h.n_input;
    img->hash = scene_hash(img->bvh);
    if (img->hash != h.hash) {
        *why = "scene image hash mismatch";
        return nullptr;
    }
    if (!validate_bvh_range(img->bvh.nodes.data(), 1, img->bvh.nodes.size(), 1 + img->bvh.nodes.size(),
                            img->bvh.tris.size(), why))
        return nullptr;
    finish_scene_image(*img);
    return img;
}

arx_status arx::set_scene_image(arx_renderer* r, SceneRef img) {
    const char* why = "";
    const BvhBuild& b = img->bvh;
    const arx_status fit = check_buffer_offsets(1 + b.nodes.size(), b.tris.size());
    if (fit != ARX_OK) return fit;
    if (!validate_bvh_range(b.nodes.data(), 1, b.nodes.size(), 1 + b.nodes.size(), b.tris.size(), &why))
        return fail(ARX_ERR_INTERNAL, "BVH validation failed (scene): %s", why);
    r->scene_img = std::move(img);
    r->scene_dirty = true;
    r->recv_model_dirty = true;  // receiver ids and offsets follow the scene
    return ARX_OK;
}

arx_status arx::last_trace_ms(arx_renderer* r, bool wait, double* ms) {
    if (r->trace_launches == 0) return fail(ARX_ERR_NOT_READY, "no trace launch yet");
    const int slot = (int)((r->trace_launches - 1) % arx_renderer::kTraceRing);
    if (wait) ARX_HIP(hipEventSynchronize(r->tev1[slot]));
    float f = 0.f;
    ARX_HIP(hipEventElapsedTime(&f, r->tev0[slot], r->tev1[slot]));
    *ms = f;
    return ARX_OK;
}

extern "C" {

}  // extern "C"

namespace {
// Device times of the last min(n, ring) launches recorded in one of the renderer's event rings.
arx_status ring_times(arx_renderer* r, const hipEvent_t* ev0, const hipEvent_t* ev1, uint64_t launches, double* ms,
                      size_t n, size_t* n_out) {
    if (!r || (n > 0 && !ms)) return fail(ARX_ERR_INVALID_ARGUMENT, "bad arguments");
    ARX_HIP(hipSetDevice(r->cfg.device));
    const uint64_t have = std::min<uint64_t>(launches, (uint64_t)arx_renderer::kTraceRing);
    const uint64_t k = std::min<uint64_t>(have, (uint64_t)n);
    for (uint64_t i = 0; i < k; ++i) {  // oldest of the last k first
        const int slot = (int)((launches - k + i) % arx_renderer::kTraceRing);
        ARX_HIP(hipEventSynchronize(ev1[slot]));
        float f = 0.f;
        ARX_HIP(hipEventElapsedTime(&f, ev0[slot], ev1[slot]));
        ms[i] = f;
    }
    if (n_out) *n_out = (size_t)k;
    return ARX_OK;
}
}  // namespace

extern "C" {

arx_status arx_trace_times(arx_renderer* r, double* ms, size_t n, size_t* n_out) {
    return r ? ring_times(r, r->tev0, r->tev1, r->trace_launches, ms, n, n_out)
             : fail(ARX_ERR_INVALID_ARGUMENT, "renderer is NULL");
}

arx_status arx_conv_times(arx_renderer* r, double* ms, size_t n, size_t* n_out) {
    return r ? ring_times(r, r->cev0, r->cev1, r->conv_launches, ms, n, n_out)
             : fail(ARX_ERR_INVALID_ARGUMENT, "renderer is NULL");
}

arx_status arx_live_times(arx_renderer* r, double* ms, size_t n, size_t* n_out) {
    return r ? ring_times(r, r->lev0, r->lev1, r->live_launches, ms, n, n_out)
             : fail(ARX_ERR_INVALID_ARGUMENT, "renderer is NULL");
}

int32_t arx_timing_ring(void) { return arx_renderer::kTraceRing; }
uint64_t arx_trace_kernel_id(void) { return trace_kernel_source_id(); }
uint64_t arx_conv_kernel_id(void) { return conv_kernel_source_id(); }

arx_status arx_debug_set_leaf_max(int32_t leaf_max) {
    if (leaf_max < 1 || leaf_max > 15) return fail(ARX_ERR_INVALID_ARGUMENT, "leaf_max %d outside [1, 15]", leaf_max);
    build_params().leaf_max = leaf_max;
    return ARX_OK;
}

int32_t arx_device_count(void) {
    int n = 0;
    return hipGetDeviceCount(&n) == hipSuccess ? (int32_t)n : -1;
}

arx_status arx_device_alloc(int32_t device, size_t bytes, void** out) {
    if (!out) return fail(ARX_ERR_INVALID_ARGUMENT, "out is NULL");
    *out = nullptr;
    ARX_HIP(hipSetDevice(device));
    ARX_HIP(hipMalloc(out, std::max<size_t>(bytes, 1)));
    return ARX_OK;
}

void arx_device_free(int32_t device, void* p) {
    if (!p) return;
    hipSetDevice(device);
    hipFree(p);
}

arx_status arx_memcpy(int32_t device, void* dst, const void* src, size_t bytes) {
    if (bytes > 0 && (!dst || !src)) return fail(ARX_ERR_INVALID_ARGUMENT, "NULL buffer");
    ARX_HIP(hipSetDevice(device));
    if (bytes > 0) ARX_HIP(hipMemcpy(dst, src, bytes, hipMemcpyDefault));
    return ARX_OK;
}

uint64_t arx_scene_build_count(void) { return g_scene_builds.load(); }

arx_status arx_debug_scene_roundtrip(const float* tri_v, const float* tri_abs, int64_t n, uint64_t* hash,
                                     uint64_t* bytes) {
    arx_status st = check_scene_input(tri_v, tri_abs, n);
    if (st != ARX_OK) return st;
    SceneRef a = build_scene_image(tri_v, tri_abs, n);
    const std::vector<uint8_t> img = serialize_scene(*a);
    const char* why = "";
    SceneRef b = deserialize_scene(img.data(), img.size(), &why);
    if (!b) return fail(ARX_ERR_INTERNAL, "scene image: %s", why);
    const bool same = a->hash == b->hash && a->n_input == b->n_input && a->bvh.depth == b->bvh.depth &&
                      a->bvh.nodes.size() == b->bvh.nodes.size() && a->bvh.tris.size() == b->bvh.tris.size() &&
                      std::memcmp(a->bvh.nodes.data(), b->bvh.nodes.data(), a->bvh.nodes.size() * sizeof(BvhNode)) == 0 &&
                      std::memcmp(a->bvh.tris.data(), b->bvh.tris.data(), a->bvh.tris.size() * sizeof(TriRec)) == 0 &&
                      std::memcmp(a->coded.data(), b->coded.data(), a->coded.size() * sizeof(BvhNode)) == 0 &&
                      a->wide().wimage == b->wide().wimage && a->wide().w4.nodes.size() == b->wide().w4.nodes.size() &&
                      std::memcmp(a->wide().w4.nodes.data(), b->wide().w4.nodes.data(),
                                  a->wide().w4.nodes.size() * sizeof(W4NodeF)) == 0 &&
                      std::memcmp(&a->bvh.root, &b->bvh.root, sizeof(ChildRef)) == 0;
    if (!same) return fail(ARX_ERR_INTERNAL, "scene image round trip changed the tree");
    if (hash) *hash = a->hash;
    if (bytes) *bytes = img.size();
    return ARX_OK;
}

const char* arx_status_string(arx_status s) {
    switch (s) {
        case ARX_OK: return "ok";
        case ARX_ERR_INVALID_ARGUMENT: return "invalid argument";
        case ARX_ERR_HIP: return "HIP error";
        case ARX_ERR_OUT_OF_MEMORY: return "out of memory";
        case ARX_ERR_NOT_READY: return "not ready";
        case ARX_ERR_IO: return "I/O error";
        case ARX_ERR_INTERNAL: return "internal error";
    }
    return "unknown status";
}

const char* arx_last_error(void) { return g_last_error.c_str(); }

int arx_abi_version(void) { return ARX_ABI_VERSION; }

int arx_frac_bits(uint64_t n) {
    int lg = 0;
    while (((uint64_t)1 << lg) < n && lg < 63) ++lg;
    int fb = 59 - lg;
    return std::min(52, std::max(8, fb));
}

void arx_default_config(arx_config* c) {
    if (!c) return;
    std::memset(c, 0, sizeof(*c));
    c->rays_x = c->rays_y = c->rays_z = 100;  // Context.cpp:114
    c->ir_length_in_seconds = 2;              // :21
    c->sample_rate = 44100;                   // live-mode default (:221)
    c->base_power = 100.0f;                   // :113
    c->energy_thres = 0.0f;                   // :115
    c->max_bounces = 10;                      // :116
    c->hrtf_absorption_rate = 1.0f;           // round(0.9) (:117, :145)
    c->is_mono = 0;
    c->seed = 1;
    c->device = 0;
}

float arx_material_absorption(const char* name, const char* const* names, const float* absorption, size_t n) {
    if (!name) return 0.5f;
    if (std::strcmp(name, "receiver_left") == 0) return -1.0f;
    if (std::strcmp(name, "receiver_right") == 0) return -2.0f;
    for (size_t i = 0; i < n; ++i)
        if (names && names[i] && std::strcmp(names[i], name) == 0) return absorption[i];
    return 0.5f;
}

}  // extern "C"

namespace {
void free_frame_set(arx_renderer::FrameSet& f) {
    if (f.stream) hipStreamDestroy(f.stream);
    hipFree(f.d_hist);
    hipFree(f.d_ir);
    hipFree(f.d_counters);
    hipFree(f.d_dirs);
    if (f.h_counters) hipHostFree(f.h_counters);
    f = arx_renderer::FrameSet{};
}
}  // namespace

arx_status arx::fif_wait_traced(arx_renderer* r) { return fif_wait_all(r, r->ev_traced); }
arx_status arx::fif_wait_conv(arx_renderer* r) { return fif_wait_last(r, r->ev_conv, r->last_conv); }
arx_status arx::fif_wait_reduced(arx_renderer* r) { return fif_wait_last(r, r->ev_reduced, r->last_reduced); }
arx_status arx::fif_done_reduced(arx_renderer* r) { return fif_done_last(r, r->ev_reduced, r->last_reduced); }
arx_status arx::sync_renderer(arx_renderer* r) {
    ARX_HIP(hipSetDevice(r->cfg.device));
    if (r->stream) ARX_HIP(hipStreamSynchronize(r->stream));
    for (const auto& f : r->alt)
        if (f.stream) ARX_HIP(hipStreamSynchronize(f.stream));
    return ARX_OK;
}
namespace {
arx_status fif_done_conv(arx_renderer* r) { return fif_done_last(r, r->ev_conv, r->last_conv); }
}  // namespace

extern "C" {

// The per-launch timing events only time: no system-scope fence when they are recorded (with one,
// each marker wrote back and invalidated the caches, a few microseconds of stream time per event).
constexpr unsigned kTimingEvent = hipEventDisableSystemFence;

arx_status arx_create(const arx_config* cfg, arx_renderer** out) {
    if (!out) return fail(ARX_ERR_INVALID_ARGUMENT, "out is NULL");
    *out = nullptr;
    arx_status st = check_config(cfg);
    if (st != ARX_OK) return st;
    int ndev = 0;
    ARX_HIP(hipGetDeviceCount(&ndev));
    if (cfg->device < 0 || cfg->device >= ndev)
        return fail(ARX_ERR_INVALID_ARGUMENT, "device %d out of range (%d devices)", cfg->device, ndev);
    ARX_HIP(hipSetDevice(cfg->device));
    arx_renderer* r = new (std::nothrow) arx_renderer();
    if (!r) return fail(ARX_ERR_OUT_OF_MEMORY, "host allocation failed");
    std::memset(&r->stats, 0, sizeof(r->stats));
    r->cfg = *cfg;
    r->ir_len = (int32_t)(cfg->ir_length_in_seconds * (uint32_t)cfg->sample_rate);
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, cfg->device) == hipSuccess) r->cus = prop.multiProcessorCount;
    auto cleanup = [&](arx_status s) {
        arx_destroy(r);
        return s;
    };
    hipError_t e;
    if ((e = hipStreamCreateWithFlags(&r->own_stream, hipStreamNonBlocking)) != hipSuccess ||
        (e = hipMalloc(&r->d_hist, 2 * (size_t)r->ir_len * sizeof(unsigned long long))) != hipSuccess ||
        (e = hipMalloc(&r->d_ir, 2 * (size_t)r->ir_len * sizeof(float))) != hipSuccess ||
        (e = hipMalloc(&r->d_counters, (kCursor + 1) * sizeof(unsigned long long))) != hipSuccess ||
        (e = hipHostMalloc(&r->h_counters, kCounters * sizeof(unsigned long long), hipHostMallocDefault)) != hipSuccess ||
        (e = hipMalloc(&r->d_tree_flag, sizeof(unsigned int))) != hipSuccess ||
        (e = hipHostMalloc(&r->h_tree_flag, sizeof(unsigned int), hipHostMallocDefault)) != hipSuccess)
        return cleanup(fail(ARX_ERR_HIP, "arx_create: %s", hipGetErrorString(e)));
    r->stream = r->own_stream;
    for (int i = 0; i < arx_renderer::kTraceRing; ++i)
        if ((e = hipEventCreateWithFlags(&r->tev0[i], kTimingEvent)) != hipSuccess ||
            (e = hipEventCreateWithFlags(&r->tev1[i], kTimingEvent)) != hipSuccess ||
            (e = hipEventCreateWithFlags(&r->cev0[i], kTimingEvent)) != hipSuccess ||
            (e = hipEventCreateWithFlags(&r->cev1[i], kTimingEvent)) != hipSuccess ||
            (e = hipEventCreateWithFlags(&r->lev0[i], kTimingEvent)) != hipSuccess ||
            (e = hipEventCreateWithFlags(&r->lev1[i], kTimingEvent)) != hipSuccess)
            return cleanup(fail(ARX_ERR_HIP, "arx_create: %s", hipGetErrorString(e)));
    // the production trace kernels' register allocation, as the runtime sees it (arx_stats)
    for (int f = 0; f < 3; ++f)
        for (int small = 0; small < 2; ++small)
            if ((e = trace_kernel_occupancy(f, small != 0, &r->occ[f][small][0], &r->occ[f][small][1],
                                            &r->occ[f][small][2])) != hipSuccess)
                return cleanup(fail(ARX_ERR_HIP, "arx_create: trace kernel attributes: %s", hipGetErrorString(e)));
    r->stats.trace_vgprs = r->occ[kFmtQ16][0][0];
    r->stats.trace_waves_per_simd = r->occ[kFmtQ16][0][1];
    r->stats.trace_waves_target = r->occ[kFmtQ16][0][2];
    r->stats.trace_format = kFmtQ16;
    r->stats.trace_grid_cus = r->cus;
    if ((e = hipMemsetAsync(r->d_hist, 0, 2 * (size_t)r->ir_len * sizeof(unsigned long long), r->stream)) != hipSuccess ||
        (e = hipMemsetAsync(r->d_ir, 0, 2 * (size_t)r->ir_len * sizeof(float), r->stream)) != hipSuccess ||
        (e = hipMemsetAsync(r->d_counters, 0, kCounters * sizeof(unsigned long long), r->stream)) != hipSuccess ||
        (e = hipMemsetAsync(r->d_tree_flag, 0, sizeof(unsigned int), r->stream)) != hipSuccess ||
        (e = hipStreamSynchronize(r->stream)) != hipSuccess)
        return cleanup(fail(ARX_ERR_HIP, "arx_create: %s", hipGetErrorString(e)));
    *out = r;
    return ARX_OK;
}

void arx_destroy(arx_renderer* r) {
    if (!r) return;
    hipSetDevice(r->cfg.device);
    if (r->stream) hipStreamSynchronize(r->stream);
    for (auto& f : r->alt) {
        if (f.stream) hipStreamSynchronize(f.stream);
        free_frame_set(f);
    }
    for (int k = 0; k < arx_renderer::kMaxFrames; ++k)
        for (hipEvent_t e : {r->ev_traced[k], r->ev_conv[k], r->ev_reduced[k], r->ev_scene[k]})
            if (e) hipEventDestroy(e);
    for (arx_stream* s : r->streams) release_stream(s);  // the handles stay valid but detached
    r->streams.clear();
    if (r->conv) conv_plan_destroy(r->conv);
    if (r->conv_live) conv_plan_destroy(r->conv_live);
    hipFree(r->d_live_in);
    hipFree(r->d_live_out);
    hipFree(r->d_cnodes);
    hipFree(r->d_qnodes);
    hipFree(r->d_tris);
    hipFree(r->d_gstack);
    hipFree(r->d_dirs);
    hipFree(r->d_prof);
    hipFree(r->d_recv_local);
    hipFree(r->d_recv_nodes);
    hipFree(r->d_recv_levels);
    hipFree(r->d_recv_w4);
    hipFree(r->d_recv_w4_tris);
    hipFree(r->d_wbuf);
    hipFree(r->d_w4f);
    hipFree(r->d_hist);
    hipFree(r->d_ir);
    hipFree(r->d_counters);
    hipFree(r->d_tree_flag);
    if (r->h_tree_flag) hipHostFree(r->h_tree_flag);
    hipFree(r->d_conv_in);
    hipFree(r->d_conv_out);
    if (r->h_counters) hipHostFree(r->h_counters);
    for (int i = 0; i < arx_renderer::kTraceRing; ++i) {
        if (r->tev0[i]) hipEventDestroy(r->tev0[i]);
        if (r->tev1[i]) hipEventDestroy(r->tev1[i]);
        if (r->cev0[i]) hipEventDestroy(r->cev0[i]);
        if (r->cev1[i]) hipEventDestroy(r->cev1[i]);
        if (r->lev0[i]) hipEventDestroy(r->lev0[i]);
        if (r->lev1[i]) hipEventDestroy(r->lev1[i]);
    }
    if (r->own_stream) hipStreamDestroy(r->own_stream);
    delete r;
}

arx_status arx_get_config(const arx_renderer* r, arx_config* out) {
    if (!r || !out) return fail(ARX_ERR_INVALID_ARGUMENT, "NULL argument");
    *out = r->cfg;
    return ARX_OK;
}

arx_status arx_set_stream(arx_renderer* r, void* s) {
    if (!r) return fail(ARX_ERR_INVALID_ARGUMENT, "renderer is NULL");
    if (r->fif != 1) return fail(ARX_ERR_INVALID_ARGUMENT, "a caller's stream needs one frame in flight (arx_set_frames_in_flight)");
    r->stream = (hipStream_t)s;
    return ARX_OK;
}

void* arx_get_stream(const arx_renderer* r) { return r ? (void*)r->stream : nullptr; }

arx_status arx_set_scene(arx_renderer* r, const float* tri_v, const float* tri_abs, int64_t n) {
    if (!r) return fail(ARX_ERR_INVALID_ARGUMENT, "renderer is NULL");
    const arx_status st = check_scene_input(tri_v, tri_abs, n);
    if (st != ARX_OK) return st;
    SceneRef img = build_scene_image(tri_v, tri_abs, n);
    if (!img) return fail(ARX_ERR_OUT_OF_MEMORY, "scene build failed");
    return set_scene_image(r, std::move(img));
}

arx_status arx_set_receiver_model(arx_renderer* r, int side, const float* tri_v, int64_t n) {
    if (!r || side < 0 || side > 1 || n < 0 || (n > 0 && !tri_v))
        return fail(ARX_ERR_INVALID_ARGUMENT, "bad receiver model arguments");
    r->recv_local[side].assign(tri_v, tri_v + 9 * n);
    r->recv_model_dirty = true;
    return ARX_OK;
}

arx_status arx_place_receiver_vertices(const float* local_xyz, int64_t n_vertices, float x, float y, float z,
                                       float yaw_deg, float* out_xyz) {
    if (n_vertices < 0 || (n_vertices > 0 && (!local_xyz || !out_xyz)))
        return fail(ARX_ERR_INVALID_ARGUMENT, "bad arguments");
    place_vertices(local_xyz, n_vertices, x, y, z, yaw_deg, out_xyz);
    return ARX_OK;
}

arx_status arx_set_emitter(arx_renderer* r, float x, float y, float z) {
    if (!r) return fail(ARX_ERR_INVALID_ARGUMENT, "renderer is NULL");
    r->emitter[0] = x;
    r->emitter[1] = y;
    r->emitter[2] = z;
    return ARX_OK;
}

arx_status arx_set_listener(arx_renderer* r, float x, float y, float z, float yaw_deg) {
    if (!r) return fail(ARX_ERR_INVALID_ARGUMENT, "renderer is NULL");
    r->center[0] = x;
    r->center[1] = y;
    r->center[2] = z;
    r->yaw = yaw_deg;
    r->recv_pose_dirty = true;
    return ARX_OK;
}

arx_status arx_set_thresholds(arx_renderer* r, float energy, uint32_t max_bounces) {
    if (!r) return fail(ARX_ERR_INVALID_ARGUMENT, "renderer is NULL");
    r->cfg.energy_thres = energy;
    r->cfg.max_bounces = max_bounces;
    return ARX_OK;
}

arx_status arx_set_hrtf_absorption_rate(arx_renderer* r, float v) {
    if (!r) return fail(ARX_ERR_INVALID_ARGUMENT, "renderer is NULL");
    if (!(v >= 0.0f && v <= 1.0f))  // the cross-ear factor (1 - hrtf) stays in [0, 1] (histogram headroom)
        return fail(ARX_ERR_INVALID_ARGUMENT, "hrtf_absorption_rate %g must be in [0, 1]", (double)v);
    r->cfg.hrtf_absorption_rate = v;
    return ARX_OK;
}

arx_status arx_set_base_power(arx_renderer* r, float v) {
    if (!r) return fail(ARX_ERR_INVALID_ARGUMENT, "renderer is NULL");
    r->cfg.base_power = v;
    return ARX_OK;
}

arx_status arx_set_mono_output(arx_renderer* r, int mono) {
    if (!r) return fail(ARX_ERR_INVALID_ARGUMENT, "renderer is NULL");
    r->cfg.is_mono = mono ? 1 : 0;
    return ARX_OK;
}

arx_status arx_set_seed(arx_renderer* r, uint64_t seed) {
    if (!r) return fail(ARX_ERR_INVALID_ARGUMENT, "renderer is NULL");
    r->cfg.seed = seed;
    return ARX_OK;
}

arx_status arx_clear_histogram(arx_renderer* r) {
    if (!r) return fail(ARX_ERR_INVALID_ARGUMENT, "renderer is NULL");
    const arx_status st = arx::begin_frame(r);
    if (st != ARX_OK) return st;
    ARX_HIP(launch_clear(r->hist(), 2 * (uint64_t)r->ir_len, r->d_counters, (int)kCounters, r->stream));
    return ARX_OK;
}

}  // extern "C"

arx_status arx::begin_frame(arx_renderer* r) {
    ARX_HIP(hipSetDevice(r->cfg.device));
    if (r->fif > 1) {  // a frame starts: it takes the next set's stream, histogram, IR, counters and directions
        arx_renderer::FrameSet cur{r->own_stream, r->d_hist, r->d_ir, r->d_counters, r->h_counters, r->d_dirs, r->dirs_cap};
        const arx_renderer::FrameSet& nx = r->alt[0];
        r->own_stream = nx.stream;
        r->stream = r->own_stream;
        r->d_hist = nx.d_hist;
        r->d_ir = nx.d_ir;
        r->d_counters = nx.d_counters;
        r->h_counters = nx.h_counters;
        r->d_dirs = nx.d_dirs;
        r->dirs_cap = nx.dirs_cap;
        for (int i = 0; i + 1 < r->fif - 1; ++i) r->alt[i] = r->alt[i + 1];
        r->alt[r->fif - 2] = cur;
        r->slot = (r->slot + 1) % r->fif;
    }
    return ARX_OK;
}

extern "C" {

arx_status arx_trace_rays(arx_renderer* r, uint64_t ray_begin, uint64_t ray_end) {
    return r ? arx::trace_rays(r, ray_begin, ray_end, r->timing) : fail(ARX_ERR_INVALID_ARGUMENT, "renderer is NULL");
}

arx_status arx_set_timing(arx_renderer* r, int32_t on) {
    if (!r) return fail(ARX_ERR_INVALID_ARGUMENT, "renderer is NULL");
    r->timing = on != 0;
    return ARX_OK;
}

}  // extern "C"

arx_status arx::trace_rays(arx_renderer* r, uint64_t ray_begin, uint64_t ray_end, bool timed, bool clear) {
    if (!r) return fail(ARX_ERR_INVALID_ARGUMENT, "renderer is NULL");
    if (ray_end < ray_begin) return fail(ARX_ERR_INVALID_ARGUMENT, "ray_end < ray_begin");
    // global ray ids index the launch of N = x*y*z rays: energies are normalised by N and the
    // int64 fixed point's headroom (arx_frac_bits) assumes at most N rays per histogram
    if (ray_end > n_rays(r->cfg))
        return fail(ARX_ERR_INVALID_ARGUMENT, "ray_end %llu exceeds the launch's %llu rays", (unsigned long long)ray_end,
                    (unsigned long long)n_rays(r->cfg));
    ARX_HIP(hipSetDevice(r->cfg.device));
    arx_status st = ensure_device_scene(r);
    if (st != ARX_OK) return st;
    const arx_config& c = r->cfg;
    TraceArgs a;
    std::memset(&a, 0, sizeof(a));
    a.cnodes = r->d_cnodes;
    // quantized nodes only while the emitter (the one ray origin off the geometry) is on the
    // grid: the slab arithmetic's error bound assumes origins within the grid's extent
    const float* em = r->emitter;
    a.qnodes = (r->q_valid && !r->force_f32_nodes && qgrid_contains(r->qgrid, em, em)) ? r->d_qnodes : nullptr;
    // the CW4 tree on the same condition when asked for (arx_debug_set_trace_path bit 3; measured
    // 1.9x slower than the BVH2 on C3: DESIGN.md section 6.3)
    a.wbuf = (a.qnodes && r->use_w4 && !r->force_global_stack) ? r->d_wbuf : nullptr;
    a.qgrid = r->qgrid;
    a.tris = r->d_tris;
    a.hist = r->hist();
    a.counters = r->d_counters;
    a.cursor = r->d_counters + kCursor;
    a.seed = c.seed;
    a.ray_begin = ray_begin;
    a.ray_end = ray_end;
    for (int k = 0; k < 3; ++k) {
        a.emitter[k] = r->emitter[k];
        a.center[k] = r->center[k];
    }
    a.e0 = initial_energy(c);
    a.inv_unit = (a.e0 != 0.0f) ? std::ldexp(1.0, arx_frac_bits(n_rays(c))) / (double)a.e0 : 0.0;
    a.energy_thres = c.energy_thres;
    a.hrtf = c.hrtf_absorption_rate;
    int32_t secs = r->ir_len / c.sample_rate;  // devicePrograms.cu:227-228
    secs = std::max(1, std::min(secs, 999));
    a.dist_limit = (float)(secs * kSpeedOfSound + 1);
    a.max_bounces = c.max_bounces;
    a.sample_rate = c.sample_rate;
    a.ir_len = r->ir_len;
    a.delay = (int32_t)((double)c.sample_rate * 0.00044);  // devicePrograms.cu:125
    a.is_mono = c.is_mono;
    a.bvh_depth = r->stats.bvh_depth;
    if (clear) {
        a.clear_bins = 2 * (uint64_t)r->ir_len;
        a.clear_counters = kCounters;
    }
    if (ray_end == ray_begin) {  // nothing to trace: the clear alone
        if (clear) ARX_HIP(launch_clear(r->hist(), 2 * (uint64_t)r->ir_len, r->d_counters, (int)kCounters, r->stream));
        return ARX_OK;
    }
    if (ray_end - ray_begin > r->dirs_cap) {  // direction pre-pass buffer
        if (r->d_dirs) ARX_HIP(hipFree(r->d_dirs));
        r->d_dirs = nullptr;
        r->dirs_cap = 0;
        ARX_HIP(hipMalloc(&r->d_dirs, (ray_end - ray_begin) * 16));
        r->dirs_cap = ray_end - ray_begin;
    }
    a.dirs = r->d_dirs;
    const bool gstack = r->force_global_stack || a.bvh_depth + 1 > kLdsStack;
    // CW4: up to three pushes per level; the rows beyond the LDS rows overflow into a global column
    const size_t w4_rows = (size_t)std::max(1, 3 * r->depth4 + 3 - kLdsStack);
    if (gstack || a.wbuf) {  // trees deeper than the LDS stack: one global column of bvh_depth + 1 entries per lane
        const size_t lanes = trace_max_lanes(r->cus);
        const size_t need = (a.wbuf ? w4_rows : (size_t)(a.bvh_depth + 1)) * lanes;
        if (need > r->gstack_cap) {
            if (r->d_gstack) ARX_HIP(hipFree(r->d_gstack));
            r->d_gstack = nullptr;
            r->gstack_cap = 0;
            ARX_HIP(hipMalloc(&r->d_gstack, need * sizeof(int32_t)));
            r->gstack_cap = need;
        }
        a.gstack = r->d_gstack;
        a.gstack_lanes = lanes;
        // one global stack per renderer: with frames in flight, after the other frames' traces
        if (const arx_status w = fif_wait_all(r, r->ev_traced); w != ARX_OK) return w;
    }
#if ARX_TRACE_PROF  // measurement builds only: per-wave records (arx_debug_trace_profile)
    {
        const size_t words = (size_t)r->cus * 64 * kProfWords;  // >= waves of any trace grid
        if (!r->d_prof) {
            ARX_HIP(hipMalloc(&r->d_prof, words * sizeof(unsigned long long)));
            r->prof_words = words;
        }
        ARX_HIP(hipMemsetAsync(r->d_prof, 0, words * sizeof(unsigned long long), r->stream));
        a.prof = r->d_prof;
    }
#endif
    // frames in flight: after the other frame set's last writes to the tree (its refit, re-gridding
    // or upload), which this launch reads
    if (const arx_status w = fif_wait_last(r, r->ev_scene, r->last_scene); w != ARX_OK) return w;
    const int slot = (int)(r->trace_launches % arx_renderer::kTraceRing);
    const int fmt = a.wbuf ? kFmtW4 : (a.qnodes ? kFmtQ16 : kFmtF32);
    // the instance launch_trace takes (ray pool or small launch): the profile guard reads these
    const int small = trace_uses_small_block(a, r->cus, r->force_global_stack) ? 1 : 0;
    r->stats.trace_format = fmt;
    r->stats.trace_vgprs = r->occ[fmt][small][0];
    r->stats.trace_waves_per_simd = r->occ[fmt][small][1];
    r->stats.trace_waves_target = r->occ[fmt][small][2];
    if (timed) ARX_HIP(hipEventRecord(r->tev0[slot], r->stream));
    // Frames in flight: a ray-pool launch is sized for half the CUs' wave slots, so the next frame's
    // launch runs beside it for its whole length instead of only in its tail.  A launch of 1M rays
    // gives each lane about three rays; the last of them leave the lanes idle one by one, and a wave
    // holds its slot until its last lane is done (C3 on the full grid: 5.87e9 queries/s at 1M rays
    // against 7.23e9 at 10M).  Two half grids side by side: C3 2.60 -> 2.44 ms per frame (DESIGN.md
    // section 6.3, profiles/r06/grid_ab_*.txt); more than half each makes a launch's last blocks wait
    // for the other's (55 %: 2.9 ms).  One frame in flight keeps the full grid, and so do the traces
    // on the renderer's one global stack (deep trees, CW4): they wait for every other frame's trace
    // above, so they never run beside one.
#ifndef ARX_SHARED_GRID_PCT
#define ARX_SHARED_GRID_PCT 50  // design experiments only (build.py --exp): other shares
#endif
    const bool shared_grid = r->fif >= 2 && !small && !gstack && !a.wbuf;
    const int grid_cus = shared_grid ? std::max(1, r->cus * ARX_SHARED_GRID_PCT / 100) : r->cus;
    r->stats.trace_grid_cus = grid_cus;
    ARX_HIP(launch_trace(a, grid_cus, r->stream, r->force_global_stack));
    if (timed) {
        ARX_HIP(hipEventRecord(r->tev1[slot], r->stream));
        ++r->trace_launches;
    }
    return fif_done_one(r, r->ev_traced);
}

extern "C" {

arx_status arx_finalize_ir(arx_renderer* r) {
    if (!r) return fail(ARX_ERR_INVALID_ARGUMENT, "renderer is NULL");
    ARX_HIP(hipSetDevice(r->cfg.device));
    const float e0 = initial_energy(r->cfg);
    const double unit = std::ldexp((double)e0, -arx_frac_bits(n_rays(r->cfg)));
    ARX_HIP(launch_finalize_ir((const long long*)r->hist(), r->d_ir, r->d_ir + r->ir_len, r->ir_len, unit,
                               r->cfg.is_mono, r->stream));
    r->conv_ir_dirty = true;
    r->conv_live_ir_dirty = true;
    ++r->ir_generation;
    return ARX_OK;
}

arx_status arx_render(arx_renderer* r, double* render_ms) {
    if (!r) return fail(ARX_ERR_INVALID_ARGUMENT, "renderer is NULL");
#ifdef ARX_EXP_SEPARATE_CLEAR  // design experiments only: the clear as a launch of its own (round-5 A/B)
    arx_status st = arx_clear_histogram(r);
    if (st != ARX_OK) return st;
    st = arx::trace_rays(r, 0, n_rays(r->cfg), r->timing || render_ms != nullptr, false);
#else
    arx_status st = arx::begin_frame(r);  // the clear rides on the direction pre-pass
    if (st != ARX_OK) return st;
    st = arx::trace_rays(r, 0, n_rays(r->cfg), r->timing || render_ms != nullptr, true);
#endif
    if (st != ARX_OK) return st;
    st = arx_finalize_ir(r);
    if (st != ARX_OK) return st;
    if (render_ms) return last_trace_ms(r, true, render_ms);
    return ARX_OK;
}

arx_status arx_set_frames_in_flight(arx_renderer* r, int32_t n) {
    if (!r) return fail(ARX_ERR_INVALID_ARGUMENT, "renderer is NULL");
    if (n < 1 || n > arx_renderer::kMaxFrames)
        return fail(ARX_ERR_INVALID_ARGUMENT, "frames in flight: 1 to %d, not %d", arx_renderer::kMaxFrames, n);
    if (n == r->fif) return ARX_OK;
    ARX_HIP(hipSetDevice(r->cfg.device));
    if (n > 1 && r->stream != r->own_stream)
        return fail(ARX_ERR_INVALID_ARGUMENT, "frames in flight need the renderer's own streams (arx_set_stream)");
    if (n > 1 && r->d_hist_ext) return fail(ARX_ERR_INVALID_ARGUMENT, "frames in flight need the renderer's own histograms");
    // nothing of the old arrangement stays in flight: the sets' order and the event slots start over
    const arx_status st = sync_renderer(r);
    if (st != ARX_OK) return st;
    for (int k = n - 1; k < arx_renderer::kMaxFrames - 1; ++k) free_frame_set(r->alt[k]);  // the current set stays
    for (int k = 0; k < n; ++k)
        for (hipEvent_t* e : {&r->ev_traced[k], &r->ev_conv[k], &r->ev_reduced[k], &r->ev_scene[k]})
            if (!*e) ARX_HIP(hipEventCreateWithFlags(e, hipEventDisableTiming));
    const size_t bins = 2 * (size_t)r->ir_len;
    for (int k = 0; k < n - 1; ++k) {
        if (r->alt[k].stream) continue;
        arx_renderer::FrameSet f;
        hipError_t e;
        if ((e = hipStreamCreateWithFlags(&f.stream, hipStreamNonBlocking)) != hipSuccess ||
            (e = hipMalloc(&f.d_hist, bins * sizeof(unsigned long long))) != hipSuccess ||
            (e = hipMalloc(&f.d_ir, bins * sizeof(float))) != hipSuccess ||
            (e = hipMalloc(&f.d_counters, (kCursor + 1) * sizeof(unsigned long long))) != hipSuccess ||
            (e = hipHostMalloc(&f.h_counters, kCounters * sizeof(unsigned long long), hipHostMallocDefault)) != hipSuccess ||
            (e = hipMemsetAsync(f.d_hist, 0, bins * sizeof(unsigned long long), f.stream)) != hipSuccess ||
            (e = hipMemsetAsync(f.d_ir, 0, bins * sizeof(float), f.stream)) != hipSuccess ||
            (e = hipMemsetAsync(f.d_counters, 0, (kCursor + 1) * sizeof(unsigned long long), f.stream)) != hipSuccess ||
            (e = hipStreamSynchronize(f.stream)) != hipSuccess) {
            free_frame_set(f);
            for (int q = 0; q < arx_renderer::kMaxFrames - 1; ++q) free_frame_set(r->alt[q]);
            r->fif = 1;
            r->slot = 0;
            return fail(ARX_ERR_HIP, "arx_set_frames_in_flight: %s", hipGetErrorString(e));
        }
        r->alt[k] = f;
    }
    r->fif = n;
    r->slot = 0;
    r->last_conv = r->last_reduced = r->last_scene = -1;
    return ARX_OK;
}

arx_status arx_histogram_device(arx_renderer* r, int64_t** d_hist, size_t* n) {
    if (!r || !d_hist) return fail(ARX_ERR_INVALID_ARGUMENT, "NULL argument");
    *d_hist = (int64_t*)r->hist();
    if (n) *n = 2 * (size_t)r->ir_len;
    return ARX_OK;
}

arx_status arx_attach_histogram(arx_renderer* r, int64_t* d_hist, size_t n) {
    if (!r) return fail(ARX_ERR_INVALID_ARGUMENT, "renderer is NULL");
    if (d_hist && n != 2 * (size_t)r->ir_len)
        return fail(ARX_ERR_INVALID_ARGUMENT, "histogram needs 2*ir_len = %zu elements, got %zu", 2 * (size_t)r->ir_len, n);
    if (d_hist && r->fif != 1)
        return fail(ARX_ERR_INVALID_ARGUMENT, "an attached histogram needs one frame in flight (arx_set_frames_in_flight)");
    r->d_hist_ext = (unsigned long long*)d_hist;
    return ARX_OK;
}

arx_status arx_ir_device(arx_renderer* r, float** d_left, float** d_right, size_t* ir_len) {
    if (!r) return fail(ARX_ERR_INVALID_ARGUMENT, "renderer is NULL");
    if (d_left) *d_left = r->d_ir;
    if (d_right) *d_right = r->d_ir + r->ir_len;
    if (ir_len) *ir_len = (size_t)r->ir_len;
    return ARX_OK;
}

arx_status arx_copy_ir(arx_renderer* r, float* h_left, float* h_right, size_t ir_len) {
    if (!r) return fail(ARX_ERR_INVALID_ARGUMENT, "renderer is NULL");
    if (ir_len != (size_t)r->ir_len) return fail(ARX_ERR_INVALID_ARGUMENT, "ir_len %zu != %d", ir_len, r->ir_len);
    ARX_HIP(hipSetDevice(r->cfg.device));
    if (h_left) ARX_HIP(hipMemcpyAsync(h_left, r->d_ir, ir_len * sizeof(float), hipMemcpyDeviceToHost, r->stream));
    if (h_right)
        ARX_HIP(hipMemcpyAsync(h_right, r->d_ir + r->ir_len, ir_len * sizeof(float), hipMemcpyDeviceToHost, r->stream));
    ARX_HIP(hipStreamSynchronize(r->stream));
    return ARX_OK;
}

arx_status arx_get_stats(arx_renderer* r, arx_stats* out) {
    if (!r || !out) return fail(ARX_ERR_INVALID_ARGUMENT, "NULL argument");
    ARX_HIP(hipSetDevice(r->cfg.device));
    ARX_HIP(hipMemcpyAsync(r->h_counters, r->d_counters, kCounters * sizeof(unsigned long long), hipMemcpyDeviceToHost,
                           r->stream));
    ARX_HIP(hipMemcpyAsync(r->h_tree_flag, r->d_tree_flag, sizeof(unsigned int), hipMemcpyDeviceToHost, r->stream));
    ARX_HIP(hipStreamSynchronize(r->stream));
    r->stats.queries = r->h_counters[0];
    r->stats.receiver_hits = r->h_counters[1];
    r->stats.misses = r->h_counters[2];
    double tms = 0.0;
    if (last_trace_ms(r, false, &tms) == ARX_OK) r->stats.trace_ms = tms;
    float cms = 0.f;
    const int cslot = (int)((r->conv_launches + arx_renderer::kTraceRing - 1) % arx_renderer::kTraceRing);
    if (r->conv_launches > 0 && hipEventElapsedTime(&cms, r->cev0[cslot], r->cev1[cslot]) == hipSuccess)
        r->stats.conv_ms = cms;
    *out = r->stats;
    // the tree as last written (generation tree_gen) has a box off the quantization grid
    if (r->tree_gen != 0 && *r->h_tree_flag == r->tree_gen)
        return fail(ARX_ERR_INTERNAL, "receiver refit / re-quantization: a box left the quantization grid");
    return ARX_OK;
}

arx_status arx_debug_trace_counters(arx_renderer* r, uint64_t* out, size_t n) {
    if (!r || !out || n > (size_t)kCounters) return fail(ARX_ERR_INVALID_ARGUMENT, "bad arguments");
    ARX_HIP(hipSetDevice(r->cfg.device));
    ARX_HIP(hipMemcpyAsync(r->h_counters, r->d_counters, kCounters * sizeof(unsigned long long), hipMemcpyDeviceToHost,
                           r->stream));
    ARX_HIP(hipStreamSynchronize(r->stream));
    for (size_t i = 0; i < n; ++i) out[i] = r->h_counters[i];
    return ARX_OK;
}

arx_status arx_set_ir(arx_renderer* r, const float* h_left, const float* h_right, size_t ir_len) {
    if (!r || !h_left || !h_right) return fail(ARX_ERR_INVALID_ARGUMENT, "NULL argument");
    if (ir_len != (size_t)r->ir_len) return fail(ARX_ERR_INVALID_ARGUMENT, "ir_len %zu != %d", ir_len, r->ir_len);
    ARX_HIP(hipSetDevice(r->cfg.device));
    ARX_HIP(hipMemcpyAsync(r->d_ir, h_left, ir_len * sizeof(float), hipMemcpyHostToDevice, r->stream));
    ARX_HIP(hipMemcpyAsync(r->d_ir + r->ir_len, h_right, ir_len * sizeof(float), hipMemcpyHostToDevice, r->stream));
    ARX_HIP(hipStreamSynchronize(r->stream));
    r->conv_ir_dirty = true;
    r->conv_live_ir_dirty = true;
    ++r->ir_generation;
    return ARX_OK;
}

arx_status arx_set_ir_device(arx_renderer* r, const float* d_left, const float* d_right, size_t ir_len) {
    if (!r || !d_left || !d_right) return fail(ARX_ERR_INVALID_ARGUMENT, "NULL argument");
    if (ir_len != (size_t)r->ir_len) return fail(ARX_ERR_INVALID_ARGUMENT, "ir_len %zu != %d", ir_len, r->ir_len);
    ARX_HIP(hipSetDevice(r->cfg.device));
    ARX_HIP(hipMemcpyAsync(r->d_ir, d_left, ir_len * sizeof(float), hipMemcpyDeviceToDevice, r->stream));
    ARX_HIP(hipMemcpyAsync(r->d_ir + r->ir_len, d_right, ir_len * sizeof(float), hipMemcpyDeviceToDevice, r->stream));
    r->conv_ir_dirty = true;
    r->conv_live_ir_dirty = true;
    ++r->ir_generation;
    return ARX_OK;
}

// spectra = false: leave a changed IR's spectra to the next conv_run (which folds them into its
// own first pass)
static arx_status ensure_conv(arx_renderer* r, bool spectra = true) {
    if (!r->conv) {
        char err[256] = {0};
        r->conv = conv_plan_create(r->ir_len, r->cfg.sample_rate, r->cfg.device, err, sizeof(err));
        if (!r->conv) return fail(ARX_ERR_INTERNAL, "convolution plan: %s", err);
        r->conv_ir_dirty = true;
    }
    if (spectra && r->conv_ir_dirty) {
        ARX_HIP(conv_set_ir(r->conv, r->d_ir, r->d_ir + r->ir_len, r->stream));
        r->conv_ir_dirty = false;
    }
    return ARX_OK;
}

static arx_status ensure_conv_live(arx_renderer* r, int32_t block) {
    if (!r->conv_live || conv_plan_block(r->conv_live) < block) {
        if (r->conv_live) conv_plan_destroy(r->conv_live);
        char err[256] = {0};
        // plan block = the longest block seen, rounded up to 4096 frames (main.cpp:37)
        const int32_t b = std::min<int32_t>(r->ir_len, std::max<int32_t>(4096, block));
        r->conv_live = conv_plan_create(r->ir_len, b, r->cfg.device, err, sizeof(err));
        if (!r->conv_live) return fail(ARX_ERR_INTERNAL, "live convolution plan: %s", err);
        r->conv_live_ir_dirty = true;
    }
    if (r->conv_live_ir_dirty) {
        ARX_HIP(conv_set_ir(r->conv_live, r->d_ir, r->d_ir + r->ir_len, r->stream));
        r->conv_live_ir_dirty = false;
    }
    return ARX_OK;
}

arx_status arx_prepare_ir_spectra(arx_renderer* r, int which) {
    if (!r) return fail(ARX_ERR_INVALID_ARGUMENT, "renderer is NULL");
    ARX_HIP(hipSetDevice(r->cfg.device));
    arx_status st = fif_wait_conv(r);
    if (st == ARX_OK && (which & 1)) st = ensure_conv(r);
    if (st == ARX_OK && (which & 2)) st = ensure_conv_live(r, 1);
    return st == ARX_OK ? fif_done_conv(r) : st;
}

arx_status arx_conv_describe(arx_renderer* r, int which, char* buf, size_t len) {
    if (!r || !buf || len == 0) return fail(ARX_ERR_INVALID_ARGUMENT, "NULL renderer or buffer");
    if (which != 1 && which != 2) return fail(ARX_ERR_INVALID_ARGUMENT, "which must be 1 (file) or 2 (live)");
    ARX_HIP(hipSetDevice(r->cfg.device));
    arx_status st = fif_wait_conv(r);
    if (st == ARX_OK) st = which == 1 ? ensure_conv(r) : ensure_conv_live(r, 1);
    if (st != ARX_OK) return st;
    std::snprintf(buf, len, "%s", conv_plan_describe(which == 1 ? r->conv : r->conv_live));
    return fif_done_conv(r);
}

arx_status arx_convolute_device(arx_renderer* r, const float* d_in, size_t n_frames, float* d_out_left,
                                float* d_out_right) {
    return arx::convolute_pairs(r, d_in, n_frames, d_out_left, d_out_right, 0, INT64_MAX);
}

}  // extern "C"

arx_status arx::convolute_pairs(arx_renderer* r, const float* d_in, size_t n_frames, float* d_out_left,
                                float* d_out_right, int64_t pair_begin, int64_t pair_end) {
    if (!r) return fail(ARX_ERR_INVALID_ARGUMENT, "renderer is NULL");
    if (n_frames > 0 && (!d_in || !d_out_left || !d_out_right)) return fail(ARX_ERR_INVALID_ARGUMENT, "NULL buffer");
    ARX_HIP(hipSetDevice(r->cfg.device));
    // the plan's spectra and scratch, and the caller's outputs, are shared with the other frame in flight
    arx_status st = fif_wait_conv(r);
    if (st == ARX_OK) st = ensure_conv(r, false);
    if (st != ARX_OK) return st;
    const bool ir_new = r->conv_ir_dirty;
    const int slot = (int)(r->conv_launches % arx_renderer::kTraceRing);
    if (r->timing) ARX_HIP(hipEventRecord(r->cev0[slot], r->stream));
    ARX_HIP(conv_run_pairs(r->conv, d_in, (int64_t)n_frames, d_out_left, d_out_right, ir_new ? r->d_ir : nullptr,
                           ir_new ? r->d_ir + r->ir_len : nullptr, pair_begin, pair_end, r->stream));
    r->conv_ir_dirty = false;
    if (r->timing) {
        ARX_HIP(hipEventRecord(r->cev1[slot], r->stream));
        ++r->conv_launches;
    }
    return fif_done_conv(r);
}

bool arx::conv_shards(arx_renderer* r) {
    return ensure_conv(r, false) == ARX_OK && conv_plan_shards(r->conv);
}

extern "C" {

arx_status arx_convolute_prepare_input(arx_renderer* r, const float* d_in, size_t n_frames) {
    if (!r) return fail(ARX_ERR_INVALID_ARGUMENT, "renderer is NULL");
    if (n_frames > 0 && !d_in) return fail(ARX_ERR_INVALID_ARGUMENT, "NULL buffer");
    ARX_HIP(hipSetDevice(r->cfg.device));
    arx_status st = fif_wait_conv(r);  // the plan's scratch is shared with the other frame in flight
    if (st == ARX_OK) st = ensure_conv(r, false);
    if (st != ARX_OK) return st;
    ARX_HIP(conv_prepare_input(r->conv, d_in, (int64_t)n_frames, r->stream));
    return fif_done_conv(r);
}

arx_status arx_convolute_prepared(arx_renderer* r, float* d_out_left, float* d_out_right, size_t* n_frames) {
    if (!r) return fail(ARX_ERR_INVALID_ARGUMENT, "renderer is NULL");
    if (!r->conv || !conv_has_prepared(r->conv))
        return fail(ARX_ERR_NOT_READY, "no prepared input (arx_convolute_prepare_input; another file convolution on "
                                       "this renderer discards it)");
    const int64_t n = conv_prepared_frames(r->conv);
    if (n > 0 && (!d_out_left || !d_out_right)) return fail(ARX_ERR_INVALID_ARGUMENT, "NULL buffer");
    ARX_HIP(hipSetDevice(r->cfg.device));
    arx_status st = fif_wait_conv(r);
    if (st != ARX_OK) return st;
    const bool ir_new = r->conv_ir_dirty;
    const int slot = (int)(r->conv_launches % arx_renderer::kTraceRing);
    if (r->timing) ARX_HIP(hipEventRecord(r->cev0[slot], r->stream));
    ARX_HIP(conv_run_prepared(r->conv, d_out_left, d_out_right, ir_new ? r->d_ir : nullptr,
                              ir_new ? r->d_ir + r->ir_len : nullptr, r->stream));
    r->conv_ir_dirty = false;
    if (r->timing) {
        ARX_HIP(hipEventRecord(r->cev1[slot], r->stream));
        ++r->conv_launches;
    }
    if (n_frames) *n_frames = (size_t)n;
    return fif_done_conv(r);
}

arx_status arx_convolute_audio_file(arx_renderer* r, const float* h_in, size_t in_bytes, float* h_out_left,
                                    float* h_out_right, double* conv_ms, double* proc_ms) {
    if (!r) return fail(ARX_ERR_INVALID_ARGUMENT, "renderer is NULL");
    const size_t n = in_bytes / sizeof(float);  // AudioRenderer.cpp:689: bytes / sizeof(float)
    if (n > 0 && (!h_in || !h_out_left || !h_out_right)) return fail(ARX_ERR_INVALID_ARGUMENT, "NULL buffer");
    ARX_HIP(hipSetDevice(r->cfg.device));
    if (const arx_status w = fif_wait_conv(r); w != ARX_OK) return w;  // the staging buffers below
    struct Events {  // destroyed on every return below
        hipEvent_t e[2] = {nullptr, nullptr};
        ~Events() {
            for (hipEvent_t x : e)
                if (x) hipEventDestroy(x);
        }
    } ev;
    ARX_HIP(hipEventCreate(&ev.e[0]));
    ARX_HIP(hipEventCreate(&ev.e[1]));
    hipEvent_t p0 = ev.e[0], p1 = ev.e[1];
    ARX_HIP(hipEventRecord(p0, r->stream));
    if (n > r->conv_cap) {
        hipFree(r->d_conv_in);
        hipFree(r->d_conv_out);
        r->d_conv_in = r->d_conv_out = nullptr;
        r->conv_cap = 0;
        ARX_HIP(hipMalloc(&r->d_conv_in, n * sizeof(float)));
        ARX_HIP(hipMalloc(&r->d_conv_out, 2 * n * sizeof(float)));
        r->conv_cap = n;
    }
    if (n > 0) ARX_HIP(hipMemcpyAsync(r->d_conv_in, h_in, n * sizeof(float), hipMemcpyHostToDevice, r->stream));
    const bool timing = r->timing;
    r->timing = timing || conv_ms != nullptr;  // the convolution's own window when asked for
    arx_status st = arx_convolute_device(r, r->d_conv_in, n, r->d_conv_out, r->d_conv_out + n);
    r->timing = timing;
    if (st != ARX_OK) return st;
    if (n > 0) {
        ARX_HIP(hipMemcpyAsync(h_out_left, r->d_conv_out, n * sizeof(float), hipMemcpyDeviceToHost, r->stream));
        ARX_HIP(hipMemcpyAsync(h_out_right, r->d_conv_out + n, n * sizeof(float), hipMemcpyDeviceToHost, r->stream));
    }
    ARX_HIP(hipEventRecord(p1, r->stream));
    ARX_HIP(hipEventSynchronize(p1));
    float ms = 0.f;
    if (conv_ms) {
        const int slot = (int)((r->conv_launches - 1) % arx_renderer::kTraceRing);
        ARX_HIP(hipEventElapsedTime(&ms, r->cev0[slot], r->cev1[slot]));
        *conv_ms = ms;
    }
    if (proc_ms) {
        ARX_HIP(hipEventElapsedTime(&ms, p0, p1));
        *proc_ms = ms;
    }
    return ARX_OK;
}

arx_status arx_convolute_live_device(arx_renderer* r, const double* d_in, size_t n_in, double* d_out) {
    if (!r) return fail(ARX_ERR_INVALID_ARGUMENT, "renderer is NULL");
    if (n_in > (size_t)r->ir_len)  // the reference copies the block into an ir_len buffer (AudioRenderer.cpp:600-603)
        return fail(ARX_ERR_INVALID_ARGUMENT, "live block of %zu samples exceeds ir_len %d", n_in, r->ir_len);
    if ((n_in > 0 && !d_in) || !d_out) return fail(ARX_ERR_INVALID_ARGUMENT, "NULL buffer");
    ARX_HIP(hipSetDevice(r->cfg.device));
    arx_status st = fif_wait_conv(r);
    if (st == ARX_OK) st = ensure_conv_live(r, (int32_t)std::max<size_t>(n_in, 1));
    if (st != ARX_OK) return st;
    const int slot = (int)(r->live_launches % arx_renderer::kTraceRing);
    ARX_HIP(hipEventRecord(r->lev0[slot], r->stream));
    ARX_HIP(conv_run_live(r->conv_live, d_in, (int64_t)n_in, d_out, r->stream));
    ARX_HIP(hipEventRecord(r->lev1[slot], r->stream));
    ++r->live_launches;
    return fif_done_conv(r);
}

arx_status arx_convolute_live_block(arx_renderer* r, const double* h_in, size_t in_bytes, double* h_out,
                                    size_t out_len) {
    if (!r) return fail(ARX_ERR_INVALID_ARGUMENT, "renderer is NULL");
    const size_t n_in = in_bytes / sizeof(double);
    if (out_len != 2 * (size_t)r->ir_len)
        return fail(ARX_ERR_INVALID_ARGUMENT, "output must hold 2*ir_len = %zu doubles", 2 * (size_t)r->ir_len);
    if ((n_in > 0 && !h_in) || !h_out) return fail(ARX_ERR_INVALID_ARGUMENT, "NULL buffer");
    if (n_in > (size_t)r->ir_len)
        return fail(ARX_ERR_INVALID_ARGUMENT, "live block of %zu samples exceeds ir_len %d", n_in, r->ir_len);
    ARX_HIP(hipSetDevice(r->cfg.device));
    if (const arx_status w = fif_wait_conv(r); w != ARX_OK) return w;  // the staging buffers below
    if (!r->d_live_in) {
        ARX_HIP(hipMalloc(&r->d_live_in, (size_t)r->ir_len * sizeof(double)));
        ARX_HIP(hipMalloc(&r->d_live_out, 2 * (size_t)r->ir_len * sizeof(double)));
    }
    if (n_in > 0) ARX_HIP(hipMemcpyAsync(r->d_live_in, h_in, n_in * sizeof(double), hipMemcpyHostToDevice, r->stream));
    arx_status st = arx_convolute_live_device(r, r->d_live_in, n_in, r->d_live_out);
    if (st != ARX_OK) return st;
    ARX_HIP(hipMemcpyAsync(h_out, r->d_live_out, out_len * sizeof(double), hipMemcpyDeviceToHost, r->stream));
    ARX_HIP(hipStreamSynchronize(r->stream));
    return ARX_OK;
}

arx_status arx_debug_node_images(arx_renderer* r, void* cnodes, void* qnodes, size_t n_nodes, float* grid,
                                 uint64_t* requants) {
    if (!r) return fail(ARX_ERR_INVALID_ARGUMENT, "renderer is NULL");
    if (n_nodes > (size_t)r->stats.n_nodes) return fail(ARX_ERR_INVALID_ARGUMENT, "only %lld nodes", (long long)r->stats.n_nodes);
    ARX_HIP(hipSetDevice(r->cfg.device));
    ARX_HIP(hipStreamSynchronize(r->stream));
    if (cnodes && n_nodes) ARX_HIP(hipMemcpy(cnodes, r->d_cnodes, n_nodes * sizeof(BvhNode), hipMemcpyDeviceToHost));
    if (qnodes && n_nodes) ARX_HIP(hipMemcpy(qnodes, r->d_qnodes, n_nodes * sizeof(QNode2), hipMemcpyDeviceToHost));
    if (grid)
        for (int k = 0; k < 3; ++k) {
            grid[k] = r->qgrid.origin[k];
            grid[3 + k] = r->qgrid.scale[k];
        }
    if (requants) *requants = r->requants;
    return ARX_OK;
}

arx_status arx_debug_trace_profile(arx_renderer* r, uint64_t* out, size_t n_words, size_t* n_out) {
    if (!r || (n_words > 0 && !out)) return fail(ARX_ERR_INVALID_ARGUMENT, "bad arguments");
    if (!r->d_prof) return fail(ARX_ERR_NOT_READY, "not a profiling build (ARX_TRACE_PROF) or no trace yet");
    ARX_HIP(hipSetDevice(r->cfg.device));
    ARX_HIP(hipStreamSynchronize(r->stream));
    const size_t k = std::min(n_words, r->prof_words);
    ARX_HIP(hipMemcpy(out, r->d_prof, k * sizeof(uint64_t), hipMemcpyDeviceToHost));
    if (n_out) *n_out = k;
    return ARX_OK;
}

arx_status arx_debug_check_tree_limits(uint64_t n_nodes, uint64_t n_tris) {
    return check_buffer_offsets((size_t)n_nodes, (size_t)n_tris);
}

arx_status arx_debug_set_refit_pad(arx_renderer* r, float pad) {
    if (!r || !(pad >= 0.0f) || !std::isfinite(pad)) return fail(ARX_ERR_INVALID_ARGUMENT, "bad arguments");
    r->debug_refit_pad = pad;
    r->recv_pose_dirty = true;  // the next trace refits with it
    return ARX_OK;
}

arx_status arx_debug_set_trace_path(arx_renderer* r, int path) {
    if (!r || path < 0 || path > 15 || (path & 4)) return fail(ARX_ERR_INVALID_ARGUMENT, "bad arguments");
    r->force_f32_nodes = (path & 1) != 0;
    r->force_global_stack = (path & 2) != 0;
    const bool w4 = (path & 8) != 0;
    if (w4 && !r->use_w4) {  // the opt-in CW4 copy is made and uploaded at the next trace
        r->scene_dirty = true;
        r->recv_model_dirty = true;
    }
    r->use_w4 = w4;
    return ARX_OK;
}

arx_status arx_debug_ray_directions(uint64_t seed, uint64_t first, uint64_t count, float* h_out, int device) {
    if (count > 0 && !h_out) return fail(ARX_ERR_INVALID_ARGUMENT, "NULL output");
    if (count == 0) return ARX_OK;
    ARX_HIP(hipSetDevice(device));
    float* d = nullptr;
    ARX_HIP(hipMalloc(&d, 3 * count * sizeof(float)));
    hipError_t e = launch_ray_directions(seed, first, count, d, nullptr);
    if (e == hipSuccess) e = hipMemcpy(h_out, d, 3 * count * sizeof(float), hipMemcpyDeviceToHost);
    hipFree(d);
    if (e != hipSuccess) return fail(ARX_ERR_HIP, "ray directions: %s", hipGetErrorString(e));
    return ARX_OK;
}

// ---- streaming convolution (UPOLS, arx_conv.hip) --------------------------------------------------
}  // extern "C"

extern "C" {

arx_status arx_stream_create(arx_renderer* r, int32_t block_frames, arx_stream** out) {
    if (!r || !out) return fail(ARX_ERR_INVALID_ARGUMENT, "NULL argument");
    *out = nullptr;
    if (block_frames <= 0 || block_frames > 4096 || block_frames > r->ir_len)
        return fail(ARX_ERR_INVALID_ARGUMENT, "stream block of %d frames: must be in [1, min(4096, ir_len)]", block_frames);
    ARX_HIP(hipSetDevice(r->cfg.device));
    arx_stream* s = new (std::nothrow) arx_stream();
    if (!s) return fail(ARX_ERR_OUT_OF_MEMORY, "host allocation failed");
    s->r = r;
    s->device = r->cfg.device;
    char err[256] = {0};
    s->plan = stream_plan_create(r->ir_len, block_frames, r->cfg.device, err, sizeof(err));
    if (!s->plan) {
        delete s;
        return fail(ARX_ERR_INTERNAL, "stream plan: %s", err);
    }
    if (hipMalloc(&s->d_in, (size_t)block_frames * sizeof(double)) != hipSuccess ||
        hipMalloc(&s->d_out, 2 * (size_t)block_frames * sizeof(double)) != hipSuccess) {
        release_stream(s);
        delete s;
        return fail(ARX_ERR_OUT_OF_MEMORY, "stream buffers");
    }
    r->streams.push_back(s);
    *out = s;
    return ARX_OK;
}

void arx_stream_destroy(arx_stream* s) {
    if (!s) return;
    if (s->r) {
        std::vector<arx_stream*>& v = s->r->streams;
        v.erase(std::remove(v.begin(), v.end(), s), v.end());
        release_stream(s);
    }
    delete s;
}

arx_status arx_stream_reset(arx_stream* s) {
    arx_status st = live_stream(s);
    if (st != ARX_OK) return st;
    ARX_HIP(hipSetDevice(s->r->cfg.device));
    if (const arx_status w = fif_wait_conv(s->r); w != ARX_OK) return w;
    ARX_HIP(stream_reset(s->plan, s->r->stream));
    return fif_done_conv(s->r);
}

arx_status arx_stream_info(const arx_stream* s, int32_t* block, int32_t* partitions, int32_t* fft_size) {
    const arx_status st = live_stream(s);
    if (st != ARX_OK) return st;
    if (block) *block = stream_plan_block(s->plan);
    if (partitions) *partitions = stream_plan_partitions(s->plan);
    if (fft_size) *fft_size = stream_plan_fft(s->plan);
    return ARX_OK;
}

arx_status arx_stream_process_device(arx_stream* s, const double* d_in, size_t n_frames, double* d_out) {
    if (const arx_status st0 = live_stream(s); st0 != ARX_OK) return st0;
    const int32_t B = stream_plan_block(s->plan);
    if (n_frames > (size_t)B) return fail(ARX_ERR_INVALID_ARGUMENT, "%zu frames exceed the stream block %d", n_frames, B);
    if ((n_frames > 0 && !d_in) || !d_out) return fail(ARX_ERR_INVALID_ARGUMENT, "NULL buffer");
    arx_renderer* r = s->r;
    ARX_HIP(hipSetDevice(r->cfg.device));
    if (const arx_status w = fif_wait_conv(r); w != ARX_OK) return w;  // the stream's delay line and spectra
    if (s->ir_generation != r->ir_generation) {  // the IR changed: new partition spectra
        ARX_HIP(stream_set_ir(s->plan, r->d_ir, r->d_ir + r->ir_len, r->stream));
        s->ir_generation = r->ir_generation;
    }
    const int slot = (int)(r->live_launches % arx_renderer::kTraceRing);
    ARX_HIP(hipEventRecord(r->lev0[slot], r->stream));
    ARX_HIP(stream_run(s->plan, d_in, (int64_t)n_frames, d_out, r->stream));
    ARX_HIP(hipEventRecord(r->lev1[slot], r->stream));
    ++r->live_launches;
    return fif_done_conv(r);
}

arx_status arx_stream_process(arx_stream* s, const double* h_in, size_t n_frames, double* h_out, size_t out_len) {
    if (const arx_status st0 = live_stream(s); st0 != ARX_OK) return st0;
    const int32_t B = stream_plan_block(s->plan);
    if (out_len != 2 * (size_t)B) return fail(ARX_ERR_INVALID_ARGUMENT, "output must hold 2*block = %d doubles", 2 * B);
    if (n_frames > (size_t)B) return fail(ARX_ERR_INVALID_ARGUMENT, "%zu frames exceed the stream block %d", n_frames, B);
    if ((n_frames > 0 && !h_in) || !h_out) return fail(ARX_ERR_INVALID_ARGUMENT, "NULL buffer");
    arx_renderer* r = s->r;
    ARX_HIP(hipSetDevice(r->cfg.device));
    if (const arx_status w = fif_wait_conv(r); w != ARX_OK) return w;  // the staging buffers below
    if (n_frames > 0)
        ARX_HIP(hipMemcpyAsync(s->d_in, h_in, n_frames * sizeof(double), hipMemcpyHostToDevice, r->stream));
    const arx_status st = arx_stream_process_device(s, s->d_in, n_frames, s->d_out);
    if (st != ARX_OK) return st;
    ARX_HIP(hipMemcpyAsync(h_out, s->d_out, out_len * sizeof(double), hipMemcpyDeviceToHost, r->stream));
    ARX_HIP(hipStreamSynchronize(r->stream));
    return ARX_OK;
}

}  // extern "C"

// (declared in arx_internal.hpp: arx_group.cpp checks a rank-0 build before broadcasting it)
arx_status arx::check_buffer_offsets(size_t n_nodes, size_t n_tris) {
    constexpr uint64_t kMax = 0x7fffffffull;
    if ((uint64_t)n_tris * sizeof(TriRec) > kMax)
        return fail(ARX_ERR_INVALID_ARGUMENT, "scene too large: %llu triangle records x %zu B exceed the trace kernel's "
                    "31-bit buffer offsets", (unsigned long long)n_tris, sizeof(TriRec));
    if ((uint64_t)n_nodes * sizeof(BvhNode) > kMax)
        return fail(ARX_ERR_INVALID_ARGUMENT, "scene too large: %llu BVH nodes x %zu B exceed the trace kernel's "
                    "31-bit buffer offsets", (unsigned long long)n_nodes, sizeof(BvhNode));
    return ARX_OK;
}
