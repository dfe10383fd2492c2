// arx_internal.hpp -- libarx.so internals shared by the C ABI translation units
// (arx_capi.cpp: one renderer; arx_group.cpp: ray-sharded multi-GPU groups).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/arx.h"
#include "arx_bvh.hpp"
#include "arx_kernels.hpp"
#include "arx_layout.hpp"
#include "arx_wide.hpp"

namespace arx {

// Records the message for arx_last_error() (thread-local) and returns s.
arx_status fail(arx_status s, const char* fmt, ...) __attribute__((format(printf, 2, 3)));

#define ARX_HIP(call)                                                                                      \
    do {                                                                                                   \
        hipError_t e_ = (call);                                                                            \
        if (e_ != hipSuccess)                                                                              \
            return ::arx::fail(e_ == hipErrorOutOfMemory ? ARX_ERR_OUT_OF_MEMORY : ARX_ERR_HIP,             \
                               "%s failed: %s (%s:%d)", #call, hipGetErrorString(e_), __FILE__, __LINE__);   \
    } while (0)

// device counters (per frame set, cleared by each frame): [0] queries [1] receiver hits [2] misses
// [3] error flag [4..7] counting builds (node steps, triangle tests, leader-node steps, step slots); the trace launch's ray-pool cursor lives after
// them (kCursor, reset by each launch itself).  The tree's off-grid flag is NOT among them: it is
// written by the tree updates that run before a frame's clear (arx_renderer::d_tree_flag).
constexpr int kCounters = 8;
constexpr int kCursor = 8;
// receivers up to this many triangles (and whose refit fits one workgroup's LDS: 9 floats per
// triangle, 11 words per node) are moved by the device refit; larger ones are rebuilt on the host
// per move
constexpr int64_t kRefitMaxTris = 3000;

inline uint64_t n_rays(const arx_config& c) {
    return (uint64_t)(int64_t)c.rays_x * (uint64_t)(int64_t)c.rays_y * (uint64_t)(int64_t)c.rays_z;
}

// The static scene as the host builds it once (buildAccel, AudioRenderer.cpp:95-218): the SBVH
// relocated into the device layout (scene nodes from index 1, node 0 being the top node; scene
// triangle records from 0) and its coded copy (code_nodes).  Immutable once built, shared by every
// renderer of a group (each uploads it to its own device).
struct SceneImage {
    BvhBuild bvh;
    std::vector<BvhNode> coded;
    int64_t n_input = 0;  // triangles given to arx_set_scene (global ids 0 .. n_input-1)
    uint64_t hash = 0;    // content hash of nodes and triangle records (profile guards)
    // The opt-in 4-wide compressed copy (CW4, arx_debug_set_trace_path bit 3; measured 1.9x slower
    // than the BVH2): made on first request only, never by the product path.
    struct Wide {
        W4Build w4;                    // scene root at unit 2, blocks from unit kW4SceneUnit
        std::vector<uint32_t> wimage;  // CW4 buffer units [0, w4.unit_end) x 4 words: leaf triangles
                                       // filled, node slots zero (quantized on the device)
    };
    const Wide& wide() const;
  private:
    mutable std::once_flag wide_once_;
    mutable Wide wide_;
};
// CW4 buffer: top node at unit 0, its block (scene root node, receiver root node) at units 2..5
constexpr uint32_t kW4SceneRoot = 2, kW4RecvRoot = 4, kW4SceneUnit = 6;
using SceneRef = std::shared_ptr<const SceneImage>;

// Input checks of arx_set_scene (finite vertices, absorption in [0, 1] or the receiver marks).
arx_status check_scene_input(const float* tri_v, const float* tri_abs, int64_t n);
// The trace kernel's 31-bit buffer offsets: a tree of n_nodes coded nodes and n_tris triangle records
// must fit them (ARX_ERR_INVALID_ARGUMENT otherwise).
arx_status check_buffer_offsets(size_t n_nodes, size_t n_tris);
// One host build (counted by arx_scene_build_count).
SceneRef build_scene_image(const float* tri_v, const float* tri_abs, int64_t n);
// Byte image of a build for the rank path's RCCL broadcast, and its inverse (NULL + why on a
// malformed image).
std::vector<uint8_t> serialize_scene(const SceneImage& s);
SceneRef deserialize_scene(const uint8_t* p, size_t n, const char** why);

}  // namespace arx

struct arx_renderer;
struct arx_stream;
namespace arx {
// Device time (ms) of the renderer's last trace launch; wait = synchronise on it first.
arx_status last_trace_ms(arx_renderer* r, bool wait, double* ms);
// arx_trace_rays with the per-launch events recorded or not (arx_set_timing, or a caller asking for the
// time); clear: the direction pre-pass zeroes the histogram and counters first (render() after
// begin_frame, instead of arx_clear_histogram's launch)
arx_status trace_rays(arx_renderer* r, uint64_t ray_begin, uint64_t ray_end, bool timed, bool clear = false);
// arx_clear_histogram without its launch: with frames in flight, the next frame takes the next set
arx_status begin_frame(arx_renderer* r);
// Install a built scene (arx_set_scene's second half): uploaded at the next trace.
arx_status set_scene_image(arx_renderer* r, SceneRef img);
// Frames in flight (arx_set_frames_in_flight): the current set's stream waits for the other set's
// last trace / convolution / all-reduce (no-ops with one frame in flight); `done_*` record the
// current set's.
arx_status fif_wait_traced(arx_renderer* r);
arx_status fif_wait_conv(arx_renderer* r);
arx_status fif_wait_reduced(arx_renderer* r);
arx_status fif_done_reduced(arx_renderer* r);
// Both frame sets' streams synchronised.
arx_status sync_renderer(arx_renderer* r);
// arx_convolute_device restricted to the file's one-second block pairs [pair_begin, pair_end)
// (conv_run_pairs; the group's time-block shards).
arx_status convolute_pairs(arx_renderer* r, const float* d_in, size_t n_frames, float* d_out_left, float* d_out_right,
                           int64_t pair_begin, int64_t pair_end);
// Whether the renderer's file convolution plan convolves a shard on its own (conv_plan_shards).
bool conv_shards(arx_renderer* r);
}  // namespace arx

// One renderer = one device (AudioRenderer, AudioRenderer.h:16-152).
struct arx_renderer {
    arx_config cfg;
    int32_t ir_len = 0;
    int cus = 256;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    // timing events: rings of (start, end) pairs around the last kTraceRing trace launches
    // (arx_trace_times), file convolutions (arx_conv_times) and live / streaming convolutions
    // (arx_live_times)
    static constexpr int kTraceRing = 256;
    hipEvent_t tev0[kTraceRing] = {}, tev1[kTraceRing] = {};
    uint64_t trace_launches = 0;  // timed trace launches (the ring's index)
    bool timing = true;           // arx_set_timing: record the per-launch events
    hipEvent_t cev0[kTraceRing] = {}, cev1[kTraceRing] = {};
    uint64_t conv_launches = 0;
    hipEvent_t lev0[kTraceRing] = {}, lev1[kTraceRing] = {};
    uint64_t live_launches = 0;

    float emitter[3] = {0.f, 0.f, 0.f};
    float center[3] = {0.f, 0.f, 0.f};
    float yaw = 0.f;

    // host scene (shared with the other members of a group)
    arx::SceneRef scene_img;
    std::vector<float> recv_local[2];
    arx::BvhBuild recv;
    bool scene_dirty = true;
    bool recv_model_dirty = true;  // receiver halves or scene changed: rebuild the local sub-tree
    bool recv_pose_dirty = true;   // listener moved: refit on the device
    bool scene_set = false;
    // receiver sub-tree in its local frame (refit path) and its device images
    bool recv_refit = true;
    float recv_radius = 0.0f;
    arx::TriRec* d_recv_local = nullptr;
    arx::BvhNode* d_recv_nodes = nullptr;
    int32_t* d_recv_levels = nullptr;  // level-ordered node indices, then level starts
    int32_t recv_levels = 0, recv_level_count = 0;

    // device
    arx::BvhNode* d_cnodes = nullptr;  // coded copy of the tree (code_nodes): the f32 fallback
    arx::QNode2* d_qnodes = nullptr;   // 16-bit quantized copy of d_cnodes (same indices): the default
    // CW4 copy: buffer, f32 node records (top node, scene, host-built receiver) for the device
    // re-quantization, the receiver's CW4 layout (refit path) and its device tables
    uint4* d_wbuf = nullptr;
    size_t wbuf_cap = 0;           // units
    arx::W4NodeF* d_w4f = nullptr;
    size_t w4f_cap = 0;
    size_t n_w4f = 0;              // records in use
    arx::W4Build recv4;
    int32_t* d_recv_w4 = nullptr;  // 11 ints per receiver CW4 node
    int32_t* d_recv_w4_tris = nullptr;
    bool use_w4 = false;           // arx_debug_set_trace_path bit 3: the CW4 tree
    int32_t depth4 = 0;            // CW4 levels (top node included): bounds the stack (3 per level)
    int32_t occ[3][2][3] = {};     // per node format and instance (0 pool, 1 small launches): VGPRs, waves admitted, waves targeted
    arx::QGrid qgrid{};
    bool qgrid_set = false;
    bool q_valid = false;         // d_qnodes matches the tree (re-quantized on the device, arx_receiver.hip)
    uint64_t requants = 0;        // device re-quantizations issued (new scene or grid)
    size_t nodes_cap = 0;
    arx::TriRec* d_tris = nullptr;
    size_t tris_cap = 0;
    int32_t* d_gstack = nullptr;  // global traversal stack for trees deeper than the LDS stack
    size_t gstack_cap = 0;        // int32 entries
    void* d_dirs = nullptr;       // direction pre-pass (float4 per ray of the largest trace call)
    uint64_t dirs_cap = 0;
    bool force_global_stack = false;  // arx_debug_set_trace_path
    bool force_f32_nodes = false;
    unsigned long long* d_hist = nullptr;  // 2*ir_len (own)
    unsigned long long* d_hist_ext = nullptr;  // caller-attached (arx_attach_histogram)
    unsigned long long* hist() const { return d_hist_ext ? d_hist_ext : d_hist; }
    float* d_ir = nullptr;                 // 2*ir_len: L then R
    unsigned long long* d_counters = nullptr;
    unsigned long long* h_counters = nullptr;  // pinned
    // The tree's off-grid flag (a receiver refit or re-quantization put a box outside the quantization
    // grid; its quantized copy then falls back to whole-axis boxes): one word per renderer, outside the
    // per-frame counters the direction pre-pass clears.  Each tree write (ensure_device_scene) runs with
    // a new generation tree_gen and raises the word to it (atomic max) on failure, so the flag reports
    // the tree as last written -- no clear launch, and a later clean write retires an old failure.
    unsigned int* d_tree_flag = nullptr;
    unsigned int* h_tree_flag = nullptr;  // pinned
    uint32_t tree_gen = 0;
    float debug_refit_pad = 0.0f;  // arx_debug_set_refit_pad: the refit kernel's box padding (0 = automatic)

    uint64_t ir_generation = 0;  // bumped whenever the IR changes (finalize_ir, set_ir): streams re-transform
    arx::ConvPlan* conv_live = nullptr;  // mic path plan (block = live block length)
    bool conv_live_ir_dirty = true;
    double* d_live_in = nullptr;
    double* d_live_out = nullptr;

    arx::ConvPlan* conv = nullptr;
    bool conv_ir_dirty = true;
    float* d_conv_in = nullptr;
    float* d_conv_out = nullptr;
    size_t conv_cap = 0;

    std::vector<arx_stream*> streams;  // live streaming convolutions of this renderer (arx_stream_create)

    // Frames in flight (arx_set_frames_in_flight, up to kMaxFrames): a frame's start
    // (arx_clear_histogram) rotates the stream, histogram, IR, counters and direction buffer above
    // with the sets in `alt`, so frame k + 1 traces on its own stream while frame k's trace finishes
    // and its IR is convolved.  The frames wait for each other only where they share state: writes to
    // the shared scene / receiver buffers (and traces on the one global stack) for every other set's
    // last trace (ev_traced); each trace for the last scene writes (ev_scene), each use of the shared
    // convolution plans and of the caller's output buffers for the last convolution (ev_conv), a
    // group's all-reduce for the last all-reduce on the same communicator (ev_reduced).  `slot` names
    // the set in the fields above; last_* the set that did the last such step (-1: none yet).
    static constexpr int kMaxFrames = 3;
    struct FrameSet {
        hipStream_t stream = nullptr;
        unsigned long long* d_hist = nullptr;
        float* d_ir = nullptr;
        unsigned long long* d_counters = nullptr;
        unsigned long long* h_counters = nullptr;
        void* d_dirs = nullptr;
        uint64_t dirs_cap = 0;
    };
    int32_t fif = 1;
    int32_t slot = 0;
    FrameSet alt[kMaxFrames - 1];
    hipEvent_t ev_traced[kMaxFrames] = {}, ev_conv[kMaxFrames] = {}, ev_reduced[kMaxFrames] = {},
               ev_scene[kMaxFrames] = {};
    int32_t last_conv = -1, last_reduced = -1, last_scene = -1;

    unsigned long long* d_prof = nullptr;  // per-wave records (profiling builds, ARX_TRACE_PROF)
    size_t prof_words = 0;
    int32_t last_format = 0;  // node format of the last trace launch (arx_stats::trace_format)
    arx_stats stats;
};

