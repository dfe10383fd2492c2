// arx_group.cpp -- ray-sharded multi-GPU rendering behind the C ABI (include/arx.h, arx_group_*).
//
// The reference renders on one GPU (deviceID 0 hard-coded, AudioRenderer.cpp:252) and has no
// collective anywhere.  Here a group holds one renderer per GPU; rank g of G
// traces the global ray ids [g*N/G, (g+1)*N/G) of the same N-ray launch (the Philox key is the
// global id, so the union of shards is exactly the single-GPU launch), and ONE RCCL all-reduce
// (int64 SUM) of the 2*ir_len fixed-point histogram over xGMI leaves the full IR on every rank:
// exact, so the IR is bitwise independent of G.
//
// Two ways to form a group:
//   arx_group_create       one process drives several GPUs (ncclCommInitAll);
//   arx_group_create_rank  one GPU per process (torchrun-style), joined through an RCCL unique
//                          id that rank 0 shares out of band (ncclCommInitRank).
// A device listed more than once in arx_group_create (oversubscribing one GPU, e.g. to test the
// sharding on a single-GPU box) cannot join an RCCL communicator twice; such a group sums its
// histograms on that device instead (hist_add kernel) -- the same exact int64 sum.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdio>
#include <cmath>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "arx_internal.hpp"
#include "arx_scene_share.hpp"

using namespace arx;

struct arx_group {
    std::vector<arx_renderer*> members;  // local members, member i = global rank rank0 + i
    std::vector<ncclComm_t> comms;       // one per member (empty: single rank or on-device sum)
    int32_t n_ranks = 1;
    int32_t rank0 = 0;
    bool device_sum = false;             // all members on one device: sum there, no RCCL
    std::vector<hipEvent_t> traced;      // per member: its shard's trace is done
    hipEvent_t summed = nullptr;         // member 0: the on-device sum is done
    // arx_debug_group_force_collectives: every collective issued at one rank too (a one-GPU box runs
    // the RCCL call paths, stream order and frames-in-flight event chain the multi-GPU job takes);
    // out_of_place: the histogram all-reduce into a receive buffer pre-filled with 0xFF, then copied
    // back, so a one-rank collective must move the data for the IR to come out right
    bool force_collectives = false;
    bool out_of_place = false;
    std::vector<unsigned long long*> d_recv;  // per member: the out-of-place receive buffer (2*ir_len)
    // collectives the group issued (arx_debug_group_collectives): [0] histogram all-reduces, [1] f64
    // all-reduces, [2] scene broadcasts (rank path)
    uint64_t n_coll[3] = {0, 0, 0};
    // per member: HIP events around its histogram all-reduce (recorded when the member's timing is on
    // or render_ms is asked for), a ring like the renderer's trace ring (arx_group_allreduce_times)
    static constexpr int kRing = 256;
    struct ArEvents {
        hipEvent_t e0[kRing] = {}, e1[kRing] = {};
        uint64_t n = 0;
    };
    std::vector<ArEvents> ar;
};

namespace {

#define ARX_NCCL(call)                                                                            \
    do {                                                                                          \
        ncclResult_t e_ = (call);                                                                 \
        if (e_ != ncclSuccess)                                                                    \
            return fail(ARX_ERR_HIP, "%s failed: %s (%s:%d)", #call, ncclGetErrorString(e_), __FILE__, __LINE__); \
    } while (0)

void destroy_members(arx_group* g) {
    for (size_t i = 0; i < g->d_recv.size(); ++i) {
        hipSetDevice(g->members[i]->cfg.device);
        hipFree(g->d_recv[i]);
    }
    g->d_recv.clear();
    for (ncclComm_t c : g->comms)
        if (c) ncclCommDestroy(c);
    g->comms.clear();
    for (size_t i = 0; i < g->traced.size(); ++i) {
        hipSetDevice(g->members[i]->cfg.device);
        if (g->traced[i]) hipEventDestroy(g->traced[i]);
    }
    for (size_t i = 0; i < g->ar.size(); ++i) {
        hipSetDevice(g->members[i]->cfg.device);
        for (int k = 0; k < arx_group::kRing; ++k) {
            if (g->ar[i].e0[k]) hipEventDestroy(g->ar[i].e0[k]);
            if (g->ar[i].e1[k]) hipEventDestroy(g->ar[i].e1[k]);
        }
    }
    g->ar.clear();
    if (g->summed) {
        hipSetDevice(g->members[0]->cfg.device);
        hipEventDestroy(g->summed);
    }
    for (arx_renderer* r : g->members) arx_destroy(r);
    g->members.clear();
}

arx_status make_members(arx_group* g, const arx_config* cfg, const int32_t* devices, int32_t n) {
    for (int32_t i = 0; i < n; ++i) {
        arx_config c = *cfg;
        c.device = devices[i];
        arx_renderer* r = nullptr;
        arx_status st = arx_create(&c, &r);
        if (st != ARX_OK) return st;
        g->members.push_back(r);
        hipEvent_t ev = nullptr;
        ARX_HIP(hipSetDevice(c.device));
        ARX_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        g->traced.push_back(ev);
    }
    return ARX_OK;
}

template <typename F>
arx_status for_all(arx_group* g, F f) {
    if (!g) return fail(ARX_ERR_INVALID_ARGUMENT, "group is NULL");
    for (arx_renderer* r : g->members) {
        const arx_status st = f(r);
        if (st != ARX_OK) return st;
    }
    return ARX_OK;
}

}  // namespace

extern "C" {

arx_status arx_group_create(const arx_config* cfg, const int32_t* devices, int32_t n_devices, arx_group** out) {
    if (!out || !cfg || n_devices <= 0) return fail(ARX_ERR_INVALID_ARGUMENT, "bad group arguments");
    *out = nullptr;
    std::vector<int32_t> devs(n_devices);
    for (int32_t i = 0; i < n_devices; ++i) devs[i] = devices ? devices[i] : i;
    std::vector<int32_t> sorted = devs;
    std::sort(sorted.begin(), sorted.end());
    const bool distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
    const bool one_device = sorted.front() == sorted.back();
    if (!distinct && !one_device)
        return fail(ARX_ERR_INVALID_ARGUMENT, "a group lists distinct GPUs (RCCL) or one GPU several times, not a mix");
    arx_group* g = new (std::nothrow) arx_group();
    if (!g) return fail(ARX_ERR_OUT_OF_MEMORY, "host allocation failed");
    g->n_ranks = n_devices;
    g->rank0 = 0;
    g->device_sum = n_devices > 1 && !distinct;
    arx_status st = make_members(g, cfg, devs.data(), n_devices);
    if (st == ARX_OK && g->device_sum) {
        if (hipSetDevice(devs[0]) != hipSuccess || hipEventCreateWithFlags(&g->summed, hipEventDisableTiming) != hipSuccess)
            st = fail(ARX_ERR_HIP, "arx_group_create: event creation failed");
    }
    if (st == ARX_OK && distinct) {  // RCCL even for one GPU: the group collectives work at every size
        g->comms.assign(n_devices, nullptr);
        const ncclResult_t e = ncclCommInitAll(g->comms.data(), n_devices, devs.data());
        if (e != ncclSuccess) {
            g->comms.clear();
            st = fail(ARX_ERR_HIP, "ncclCommInitAll(%d devices) failed: %s", n_devices, ncclGetErrorString(e));
        }
    }
    if (st != ARX_OK) {
        destroy_members(g);
        delete g;
        return st;
    }
    *out = g;
    return ARX_OK;
}

arx_status arx_group_unique_id(uint8_t* id, size_t n) {
    if (!id || n != NCCL_UNIQUE_ID_BYTES) return fail(ARX_ERR_INVALID_ARGUMENT, "the RCCL unique id is %d bytes", NCCL_UNIQUE_ID_BYTES);
    ncclUniqueId u;
    ARX_NCCL(ncclGetUniqueId(&u));
    std::memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
    return ARX_OK;
}

arx_status arx_group_create_rank(const arx_config* cfg, int32_t n_ranks, int32_t rank, const uint8_t* id, size_t n,
                                 arx_group** out) {
    if (!out || !cfg || n_ranks <= 0 || rank < 0 || rank >= n_ranks || (id && n != NCCL_UNIQUE_ID_BYTES) ||
        (n_ranks > 1 && !id))
        return fail(ARX_ERR_INVALID_ARGUMENT, "bad group rank arguments");
    *out = nullptr;
    arx_group* g = new (std::nothrow) arx_group();
    if (!g) return fail(ARX_ERR_OUT_OF_MEMORY, "host allocation failed");
    g->n_ranks = n_ranks;
    g->rank0 = rank;
    const int32_t dev = cfg->device;
    arx_status st = make_members(g, cfg, &dev, 1);
    ncclUniqueId u;
    if (st == ARX_OK) {
        if (id) {
            std::memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
        } else if (ncclGetUniqueId(&u) != ncclSuccess) {  // a one-rank group needs no shared id
            st = fail(ARX_ERR_HIP, "ncclGetUniqueId failed");
        }
    }
    if (st == ARX_OK) {
        g->comms.assign(1, nullptr);
        hipSetDevice(dev);
        const ncclResult_t e = ncclCommInitRank(&g->comms[0], n_ranks, u, rank);
        if (e != ncclSuccess) {
            g->comms.clear();
            st = fail(ARX_ERR_HIP, "ncclCommInitRank(rank %d of %d) failed: %s", rank, n_ranks, ncclGetErrorString(e));
        }
    }
    if (st != ARX_OK) {
        destroy_members(g);
        delete g;
        return st;
    }
    *out = g;
    return ARX_OK;
}

void arx_group_destroy(arx_group* g) {
    if (!g) return;
    for (arx_renderer* r : g->members) sync_renderer(r);
    destroy_members(g);
    delete g;
}

int32_t arx_group_members(const arx_group* g) { return g ? (int32_t)g->members.size() : 0; }

int32_t arx_group_ranks(const arx_group* g) { return g ? g->n_ranks : 0; }

arx_renderer* arx_group_member(arx_group* g, int32_t i) {
    if (!g || i < 0 || i >= (int32_t)g->members.size()) return nullptr;
    return g->members[i];
}

// The scene tree is built once per group (buildAccel, AudioRenderer.cpp:95-218, runs once per scene
// in the reference too) and shared by the members; each uploads it to its own device at its next
// trace.  In a one-GPU-per-process group, rank 0 builds and the tree's byte image goes to the other
// ranks with RCCL broadcasts (share_from_rank0, arx_scene_share.hpp: every rank enters every
// collective, a failure on any rank fails the call on all of them).
}  // extern "C"

namespace {
// share_from_rank0's transport over the group's communicator, staged through device memory on the
// member's stream.
struct RcclChannel {
    ncclComm_t comm;
    hipStream_t stream;
    bool root;
    uint64_t* d_word = nullptr;
    uint8_t* d_buf = nullptr;
    std::string err;

    ~RcclChannel() {
        hipStreamSynchronize(stream);
        hipFree(d_word);
        hipFree(d_buf);
    }
    bool hip(hipError_t e, const char* what) {
        if (e != hipSuccess && err.empty()) err = std::string(what) + ": " + hipGetErrorString(e);
        return e == hipSuccess;
    }
    bool nccl(ncclResult_t e, const char* what) {
        if (e != ncclSuccess && err.empty()) err = std::string(what) + ": " + ncclGetErrorString(e);
        return e == ncclSuccess;
    }
    bool word(uint64_t* v, bool bcast) {
        if (!d_word && !hip(hipMalloc(&d_word, sizeof(uint64_t)), "hipMalloc")) return false;
        return hip(hipMemcpyAsync(d_word, v, sizeof(uint64_t), hipMemcpyHostToDevice, stream), "upload") &&
               nccl(bcast ? ncclBroadcast(d_word, d_word, 1, ncclUint64, 0, comm, stream)
                          : ncclAllReduce(d_word, d_word, 1, ncclUint64, ncclMax, comm, stream),
                    bcast ? "ncclBroadcast(size)" : "ncclAllReduce(flag)") &&
               hip(hipMemcpyAsync(v, d_word, sizeof(uint64_t), hipMemcpyDeviceToHost, stream), "download") &&
               hip(hipStreamSynchronize(stream), "sync");
    }
    bool bcast_u64(uint64_t* v) { return word(v, true); }
    bool max_u64(uint64_t* v) { return word(v, false); }
    bool stage(uint64_t bytes) { return hip(hipMalloc(&d_buf, std::max<uint64_t>(bytes, 1)), "hipMalloc(image)"); }
    bool bcast_bytes(uint8_t* host, uint64_t bytes) {
        return (!root || hip(hipMemcpyAsync(d_buf, host, bytes, hipMemcpyHostToDevice, stream), "upload")) &&
               nccl(ncclBroadcast(d_buf, d_buf, bytes, ncclUint8, 0, comm, stream), "ncclBroadcast(tree)") &&
               (root || hip(hipMemcpyAsync(host, d_buf, bytes, hipMemcpyDeviceToHost, stream), "download")) &&
               hip(hipStreamSynchronize(stream), "sync");
    }
};

// share_from_rank0's transport through caller callbacks (arx_debug_share_scene).
struct CallbackChannel {
    arx_share_u64_fn word;
    arx_share_bytes_fn bytes_fn;
    void* ctx;
    std::string err;
    bool bcast_u64(uint64_t* v) { return word(ctx, v, 0) == 0 || (err = "word broadcast failed", false); }
    bool max_u64(uint64_t* v) { return word(ctx, v, 1) == 0 || (err = "word all-reduce failed", false); }
    bool stage(uint64_t) { return true; }
    bool bcast_bytes(uint8_t* host, uint64_t n) { return bytes_fn(ctx, host, n) == 0 || (err = "byte broadcast failed", false); }
};

// arx_group_set_scene's rank path over any transport: rank 0 checks and builds the scene, every other
// rank reads the broadcast image; every rank returns the same status class.
template <class Chan>
arx_status share_scene(Chan& ch, int32_t rank, const float* tri_v, const float* tri_abs, int64_t n, SceneRef* out) {
    SceneRef img;
    arx_status root_st = ARX_OK;
    std::string root_err, consume_err;
    const ShareResult res = share_from_rank0(
        ch, rank,
        [&](std::vector<uint8_t>& bytes) {
            root_st = check_scene_input(tri_v, tri_abs, n);
            if (root_st == ARX_OK) {
                img = build_scene_image(tri_v, tri_abs, n);
                if (!img) root_st = fail(ARX_ERR_OUT_OF_MEMORY, "scene build failed");
            }
            // a tree beyond the trace kernel's buffer offsets fails here, on every rank, before its
            // image is staged and broadcast (every rank's set_scene_image would reject it anyway)
            if (root_st == ARX_OK) root_st = check_buffer_offsets(1 + img->bvh.nodes.size(), img->bvh.tris.size());
            if (root_st != ARX_OK) {
                root_err = arx_last_error();
                return false;
            }
            bytes = serialize_scene(*img);
            return true;
        },
        [&](const std::vector<uint8_t>& bytes) {
            const char* why = "";
            img = deserialize_scene(bytes.data(), bytes.size(), &why);
            if (!img) consume_err = why;
            return (bool)img;
        });
    switch (res) {
        case ShareResult::ok:
            *out = img;
            return ARX_OK;
        case ShareResult::root_failed:
            return rank == 0 ? fail(root_st, "%s", root_err.c_str())
                             : fail(ARX_ERR_INVALID_ARGUMENT, "scene broadcast: rank 0 could not build the scene");
        case ShareResult::staging_failed:
            return fail(ARX_ERR_OUT_OF_MEMORY, "scene broadcast (rank %d): a rank could not stage the image%s%s", rank,
                        ch.err.empty() ? "" : ": ", ch.err.c_str());
        case ShareResult::consume_failed:
            return fail(ARX_ERR_INTERNAL, "scene broadcast (rank %d): a rank could not read the image%s%s", rank,
                        consume_err.empty() ? "" : ": ", consume_err.c_str());
        case ShareResult::transport_failed:
            break;
    }
    return fail(ARX_ERR_HIP, "scene broadcast (rank %d): %s", rank, ch.err.c_str());
}

// Rank r of G traces the global ray ids [r*N/G, (r+1)*N/G) of the N-ray launch.
void shard_of(uint64_t n, int32_t rank, int32_t n_ranks, uint64_t* b, uint64_t* e) {
    const unsigned __int128 nn = n;
    *b = (uint64_t)(nn * (uint64_t)rank / (uint64_t)n_ranks);
    *e = (uint64_t)(nn * (uint64_t)(rank + 1) / (uint64_t)n_ranks);
}

// Rank r of G convolves the block pairs [r*P/G, (r+1)*P/G) of a file's P = ceil(floor(n/sr) / 2) pairs
// of one-second blocks (convoluteFromAudioBuffer's blocks, kernels.cu:404-430, two per FFT pair).
void conv_pairs_of(int32_t sample_rate, uint64_t n_frames, int32_t rank, int32_t n_ranks, uint64_t* b, uint64_t* e) {
    const uint64_t sr = sample_rate > 0 ? (uint64_t)sample_rate : 1;
    const uint64_t S = n_frames / sr;
    if (S == 0) {  // no block: rank 0 writes the (zero) output, the others nothing (conv_run_pairs)
        *b = rank == 0 ? 0 : 1;
        *e = 1;
        return;
    }
    shard_of((S + 1) / 2, rank, n_ranks, b, e);
}
}  // namespace

extern "C" {

arx_status arx_group_set_scene(arx_group* g, const float* tri_v, const float* tri_abs, int64_t n) {
    if (!g || g->members.empty()) return fail(ARX_ERR_INVALID_ARGUMENT, "group is NULL or empty");
    const bool rank_path = (g->n_ranks > 1 || g->force_collectives) && g->members.size() == 1 && g->comms.size() == 1;
    SceneRef img;
    if (!rank_path) {
        const arx_status st = check_scene_input(tri_v, tri_abs, n);
        if (st != ARX_OK) return st;
        img = build_scene_image(tri_v, tri_abs, n);
        if (!img) return fail(ARX_ERR_OUT_OF_MEMORY, "scene build failed");
    } else {
        arx_renderer* r = g->members[0];
        ARX_HIP(hipSetDevice(r->cfg.device));
        RcclChannel ch{g->comms[0], r->stream, g->rank0 == 0};
        const arx_status st = share_scene(ch, g->rank0, tri_v, tri_abs, n, &img);
        if (st != ARX_OK) return st;
        ++g->n_coll[2];
    }
    return for_all(g, [&](arx_renderer* m) { return set_scene_image(m, img); });
}

void arx_group_shard(uint64_t n_rays, int32_t rank, int32_t n_ranks, uint64_t* begin, uint64_t* end) {
    shard_of(n_rays, rank, n_ranks, begin, end);
}

// The rank path's scene hand-over over a caller's transport (tests: two processes over gloo).
arx_status arx_debug_share_scene(int32_t rank, const float* tri_v, const float* tri_abs, int64_t n,
                                 arx_share_u64_fn word, arx_share_bytes_fn bytes, void* ctx, uint64_t* tree_hash) {
    if (rank < 0 || !word || !bytes) return fail(ARX_ERR_INVALID_ARGUMENT, "bad arguments");
    CallbackChannel ch{word, bytes, ctx};
    SceneRef img;
    const arx_status st = share_scene(ch, rank, tri_v, tri_abs, n, &img);
    if (st == ARX_OK && tree_hash) *tree_hash = img->hash;
    return st;
}

arx_status arx_group_set_receiver_model(arx_group* g, int side, const float* tri_v, int64_t n) {
    return for_all(g, [&](arx_renderer* r) { return arx_set_receiver_model(r, side, tri_v, n); });
}
arx_status arx_group_set_emitter(arx_group* g, float x, float y, float z) {
    return for_all(g, [&](arx_renderer* r) { return arx_set_emitter(r, x, y, z); });
}
arx_status arx_group_set_listener(arx_group* g, float x, float y, float z, float yaw_deg) {
    return for_all(g, [&](arx_renderer* r) { return arx_set_listener(r, x, y, z, yaw_deg); });
}
arx_status arx_group_set_thresholds(arx_group* g, float energy, uint32_t max_bounces) {
    return for_all(g, [&](arx_renderer* r) { return arx_set_thresholds(r, energy, max_bounces); });
}
arx_status arx_group_set_hrtf_absorption_rate(arx_group* g, float rate) {
    return for_all(g, [&](arx_renderer* r) { return arx_set_hrtf_absorption_rate(r, rate); });
}
arx_status arx_group_set_base_power(arx_group* g, float p) {
    return for_all(g, [&](arx_renderer* r) { return arx_set_base_power(r, p); });
}
arx_status arx_group_set_mono_output(arx_group* g, int mono) {
    return for_all(g, [&](arx_renderer* r) { return arx_set_mono_output(r, mono); });
}
arx_status arx_group_set_seed(arx_group* g, uint64_t seed) {
    return for_all(g, [&](arx_renderer* r) { return arx_set_seed(r, seed); });
}

arx_status arx_group_render(arx_group* g, double* render_ms) {
    if (!g || g->members.empty()) return fail(ARX_ERR_INVALID_ARGUMENT, "group is NULL or empty");
    const uint64_t n = n_rays(g->members[0]->cfg);
    const size_t bins = 2 * (size_t)g->members[0]->ir_len;
    // 1. every local member traces its shard (async on its own stream)
    for (size_t i = 0; i < g->members.size(); ++i) {
        arx_renderer* r = g->members[i];
        uint64_t b = 0, e = 0;
        shard_of(n, g->rank0 + (int32_t)i, g->n_ranks, &b, &e);
        arx_status st = begin_frame(r);  // the clear rides on the direction pre-pass
        if (st == ARX_OK) st = trace_rays(r, b, e, r->timing || render_ms != nullptr, true);
        if (st != ARX_OK) return st;
    }
    // 2. the exchange step: int64 SUM of the histograms (a group of one rank has nothing to sum:
    //    its communicator is kept for the group's other collectives, the render skips the no-op
    //    unless arx_debug_group_force_collectives asks for it)
    if (!g->comms.empty() && (g->n_ranks > 1 || g->force_collectives)) {
        // with frames in flight, each member's all-reduce after its previous one (the collectives on
        // a communicator keep their order whichever stream they run on)
        for (arx_renderer* r : g->members) {
            const arx_status st = fif_wait_reduced(r);
            if (st != ARX_OK) return st;
        }
        if (g->out_of_place) {  // the receive buffers hold 0xFF until the collective writes them
            if (g->d_recv.size() != g->members.size()) g->d_recv.assign(g->members.size(), nullptr);
            for (size_t i = 0; i < g->members.size(); ++i) {
                arx_renderer* r = g->members[i];
                ARX_HIP(hipSetDevice(r->cfg.device));
                if (!g->d_recv[i]) ARX_HIP(hipMalloc(&g->d_recv[i], bins * sizeof(long long)));
                ARX_HIP(hipMemsetAsync(g->d_recv[i], 0xFF, bins * sizeof(long long), r->stream));
            }
        }
        // the all-reduce's own window on every member's stream (arx_group_allreduce_times)
        const bool timed = render_ms != nullptr || g->members[0]->timing;
        if (timed) {
            if (g->ar.size() != g->members.size()) g->ar.resize(g->members.size());
            for (size_t i = 0; i < g->members.size(); ++i) {
                arx_renderer* r = g->members[i];
                arx_group::ArEvents& ev = g->ar[i];
                const int k = (int)(ev.n % arx_group::kRing);
                ARX_HIP(hipSetDevice(r->cfg.device));
                if (!ev.e0[k]) ARX_HIP(hipEventCreateWithFlags(&ev.e0[k], hipEventDisableSystemFence));
                if (!ev.e1[k]) ARX_HIP(hipEventCreateWithFlags(&ev.e1[k], hipEventDisableSystemFence));
                ARX_HIP(hipEventRecord(ev.e0[k], r->stream));
            }
        }
        ARX_NCCL(ncclGroupStart());
        for (size_t i = 0; i < g->members.size(); ++i) {
            arx_renderer* r = g->members[i];
            void* recv = g->out_of_place ? (void*)g->d_recv[i] : (void*)r->hist();
            const ncclResult_t e = ncclAllReduce(r->hist(), recv, bins, ncclInt64, ncclSum, g->comms[i], r->stream);
            if (e != ncclSuccess) {
                ncclGroupEnd();
                return fail(ARX_ERR_HIP, "ncclAllReduce failed: %s", ncclGetErrorString(e));
            }
        }
        ARX_NCCL(ncclGroupEnd());
        ++g->n_coll[0];
        if (timed)
            for (size_t i = 0; i < g->members.size(); ++i) {
                arx_renderer* r = g->members[i];
                arx_group::ArEvents& ev = g->ar[i];
                ARX_HIP(hipSetDevice(r->cfg.device));
                ARX_HIP(hipEventRecord(ev.e1[(int)(ev.n % arx_group::kRing)], r->stream));
                ++ev.n;
            }
        if (g->out_of_place)  // the sum back into the histogram the finalise reads, before the next frame's
            for (size_t i = 0; i < g->members.size(); ++i) {  // all-reduce may write the receive buffer
                arx_renderer* r = g->members[i];
                ARX_HIP(hipSetDevice(r->cfg.device));
                ARX_HIP(hipMemcpyAsync(r->hist(), g->d_recv[i], bins * sizeof(long long), hipMemcpyDeviceToDevice,
                                       r->stream));
            }
        for (arx_renderer* r : g->members) {
            const arx_status st = fif_done_reduced(r);
            if (st != ARX_OK) return st;
        }
    } else if (g->device_sum) {
        // Member 0's stream does all of it -- sum the shards into member 0's histogram, then copy the
        // total back into every other member's -- and the others wait for that before finalising.
        // Every access to member 0's histogram is thus ordered on member 0's own stream, so its next
        // clear cannot overtake a copy still reading it, and member i's next clear (after its
        // finalise, after `summed`) cannot overtake the copy writing its histogram.
        arx_renderer* r0 = g->members[0];
        ARX_HIP(hipSetDevice(r0->cfg.device));
        for (size_t i = 1; i < g->members.size(); ++i) {
            arx_renderer* r = g->members[i];
            ARX_HIP(hipEventRecord(g->traced[i], r->stream));
            ARX_HIP(hipStreamWaitEvent(r0->stream, g->traced[i], 0));
            ARX_HIP(launch_hist_add((long long*)r0->hist(), (const long long*)r->hist(), bins, r0->stream));
        }
        for (size_t i = 1; i < g->members.size(); ++i)
            ARX_HIP(hipMemcpyAsync(g->members[i]->hist(), r0->hist(), bins * sizeof(long long), hipMemcpyDeviceToDevice,
                                   r0->stream));
        ARX_HIP(hipEventRecord(g->summed, r0->stream));
        for (size_t i = 1; i < g->members.size(); ++i) ARX_HIP(hipStreamWaitEvent(g->members[i]->stream, g->summed, 0));
    }
    // 3. every member finalises the full IR
    for (arx_renderer* r : g->members) {
        const arx_status st = arx_finalize_ir(r);
        if (st != ARX_OK) return st;
    }
    if (render_ms) {  // the reference's window (AudioRenderer.cpp:495-518): the longest shard trace
        double worst = 0.0;
        for (arx_renderer* r : g->members) {
            ARX_HIP(hipSetDevice(r->cfg.device));
            double ms = 0.0;
            const arx_status st = last_trace_ms(r, true, &ms);
            if (st != ARX_OK) return st;
            worst = std::max(worst, ms);
        }
        *render_ms = worst;
    }
    return ARX_OK;
}

arx_status arx_group_allreduce_times(arx_group* g, int32_t member, double* ms, size_t n, size_t* n_out) {
    if (!g || member < 0 || member >= (int32_t)g->members.size() || (n > 0 && !ms))
        return fail(ARX_ERR_INVALID_ARGUMENT, "bad arguments");
    if (n_out) *n_out = 0;
    if ((size_t)member >= g->ar.size()) return ARX_OK;  // no timed all-reduce yet
    const arx_group::ArEvents& ev = g->ar[(size_t)member];
    ARX_HIP(hipSetDevice(g->members[(size_t)member]->cfg.device));
    const uint64_t k = std::min<uint64_t>(std::min<uint64_t>(ev.n, (uint64_t)arx_group::kRing), (uint64_t)n);
    for (uint64_t i = 0; i < k; ++i) {  // oldest of the last k first
        const int slot = (int)((ev.n - k + i) % arx_group::kRing);
        ARX_HIP(hipEventSynchronize(ev.e1[slot]));
        float f = 0.f;
        ARX_HIP(hipEventElapsedTime(&f, ev.e0[slot], ev.e1[slot]));
        ms[i] = f;
    }
    if (n_out) *n_out = (size_t)k;
    return ARX_OK;
}

void arx_group_conv_shard(int32_t sample_rate, uint64_t n_frames, int32_t rank, int32_t n_ranks, uint64_t* begin,
                          uint64_t* end) {
    uint64_t pb = 0, pe = 0;
    conv_pairs_of(sample_rate, n_frames, rank, n_ranks, &pb, &pe);
    const uint64_t sr = sample_rate > 0 ? (uint64_t)sample_rate : 1;
    const uint64_t S = n_frames / sr, P = (S + 1) / 2;
    if (P == 0) {  // nothing convolved: rank 0 owns the (zero) output
        *begin = rank == 0 ? 0 : n_frames;
        *end = n_frames;
        return;
    }
    *begin = pb == 0 ? 0 : std::min<uint64_t>(2 * pb * sr, n_frames);
    *end = pe == P ? n_frames : std::min<uint64_t>(2 * pe * sr, n_frames);
    if (pe == pb) *begin = *end;
}

arx_status arx_group_convolute_device(arx_group* g, const float* const* d_in, size_t n_frames,
                                      float* const* d_out_left, float* const* d_out_right) {
    if (!g || g->members.empty() || !d_in || !d_out_left || !d_out_right)
        return fail(ARX_ERR_INVALID_ARGUMENT, "bad arguments");
    for (size_t i = 0; i < g->members.size(); ++i) {
        arx_renderer* r = g->members[i];
        uint64_t pb = 0, pe = 0;
        conv_pairs_of(r->cfg.sample_rate, n_frames, g->rank0 + (int32_t)i, g->n_ranks, &pb, &pe);
        const arx_status st = convolute_pairs(r, d_in[i], n_frames, d_out_left[i], d_out_right[i], (int64_t)pb,
                                              (int64_t)pe);
        if (st != ARX_OK) return st;
    }
    return ARX_OK;
}

arx_status arx_group_convolute_audio_file(arx_group* g, const float* h_in, size_t in_bytes, float* h_out_left,
                                          float* h_out_right, double* convolute_ms, double* process_ms) {
    if (!g || g->members.empty()) return fail(ARX_ERR_INVALID_ARGUMENT, "group is NULL or empty");
    const size_t n = in_bytes / sizeof(float);  // AudioRenderer.cpp:689: bytes / sizeof(float)
    if (n > 0 && (!h_in || !h_out_left || !h_out_right)) return fail(ARX_ERR_INVALID_ARGUMENT, "NULL buffer");
    arx_renderer* r0 = g->members[0];
    // one rank, or a plan that does not shard: the whole file on this process's first member
    if (g->n_ranks == 1 || !conv_shards(r0))
        return arx_convolute_audio_file(r0, h_in, in_bytes, h_out_left, h_out_right, convolute_ms, process_ms);
    struct Events {  // per member: the call's window on its stream; destroyed on every return below
        std::vector<std::pair<int32_t, hipEvent_t>> e;
        ~Events() {
            for (auto& d : e) {
                hipSetDevice(d.first);
                hipEventDestroy(d.second);
            }
        }
    } ev;
    const int32_t sr = r0->cfg.sample_rate;
    std::vector<uint64_t> conv_slot(g->members.size(), 0);
    for (size_t i = 0; i < g->members.size(); ++i) {
        arx_renderer* r = g->members[i];
        const int32_t rank = g->rank0 + (int32_t)i;
        ARX_HIP(hipSetDevice(r->cfg.device));
        if (const arx_status w = fif_wait_conv(r); w != ARX_OK) return w;  // the staging buffers below
        hipEvent_t p0 = nullptr, p1 = nullptr;
        ARX_HIP(hipEventCreate(&p0));
        ev.e.emplace_back(r->cfg.device, p0);
        ARX_HIP(hipEventCreate(&p1));
        ev.e.emplace_back(r->cfg.device, p1);
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
        uint64_t pb = 0, pe = 0, b = 0, e = 0;
        conv_pairs_of(sr, n, rank, g->n_ranks, &pb, &pe);
        arx_group_conv_shard(sr, n, rank, g->n_ranks, &b, &e);
        // only the input this shard reads: its block pairs and the seam pair before them
        const uint64_t S = n / (uint64_t)sr;
        const uint64_t in_lo = std::min<uint64_t>(pb > 0 ? 2 * (pb - 1) * (uint64_t)sr : 0, n);
        const uint64_t in_hi = (pe > pb && S > 0) ? std::min<uint64_t>(2 * pe * (uint64_t)sr, n) : in_lo;
        if (in_hi > in_lo)
            ARX_HIP(hipMemcpyAsync(r->d_conv_in + in_lo, h_in + in_lo, (in_hi - in_lo) * sizeof(float),
                                   hipMemcpyHostToDevice, r->stream));
        const bool timing = r->timing;
        r->timing = timing || convolute_ms != nullptr;  // the convolution's own window when asked for
        arx_status st = convolute_pairs(r, r->d_conv_in, n, r->d_conv_out, r->d_conv_out + n, (int64_t)pb, (int64_t)pe);
        conv_slot[i] = r->conv_launches;
        r->timing = timing;
        if (st != ARX_OK) return st;
        if (e > b) {  // this rank's output frames back into the caller's buffers
            ARX_HIP(hipMemcpyAsync(h_out_left + b, r->d_conv_out + b, (e - b) * sizeof(float), hipMemcpyDeviceToHost,
                                   r->stream));
            ARX_HIP(hipMemcpyAsync(h_out_right + b, r->d_conv_out + n + b, (e - b) * sizeof(float),
                                   hipMemcpyDeviceToHost, r->stream));
        }
        ARX_HIP(hipEventRecord(p1, r->stream));
    }
    double conv = 0.0, proc = 0.0;
    for (size_t i = 0; i < g->members.size(); ++i) {
        arx_renderer* r = g->members[i];
        ARX_HIP(hipSetDevice(r->cfg.device));
        hipEvent_t p0 = ev.e[2 * i].second, p1 = ev.e[2 * i + 1].second;
        ARX_HIP(hipEventSynchronize(p1));
        float ms = 0.f;
        ARX_HIP(hipEventElapsedTime(&ms, p0, p1));
        proc = std::max(proc, (double)ms);
        if (convolute_ms && conv_slot[i] > 0) {
            const int slot = (int)((conv_slot[i] - 1) % arx_renderer::kTraceRing);
            ARX_HIP(hipEventElapsedTime(&ms, r->cev0[slot], r->cev1[slot]));
            conv = std::max(conv, (double)ms);
        }
    }
    if (convolute_ms) *convolute_ms = conv;
    if (process_ms) *process_ms = proc;
    return ARX_OK;
}

int32_t arx_group_conv_sharded(arx_group* g) {
    if (!g || g->members.empty()) return -1;
    return conv_shards(g->members[0]) ? 1 : 0;
}

arx_status arx_group_synchronize(arx_group* g) {
    return for_all(g, [&](arx_renderer* r) { return sync_renderer(r); });
}

arx_status arx_group_set_frames_in_flight(arx_group* g, int32_t n) {
    return for_all(g, [&](arx_renderer* r) { return arx_set_frames_in_flight(r, n); });
}

arx_status arx_group_set_timing(arx_group* g, int32_t on) {
    return for_all(g, [&](arx_renderer* r) { return arx_set_timing(r, on); });
}

arx_status arx_group_copy_ir(arx_group* g, float* h_left, float* h_right, size_t ir_len) {
    if (!g || g->members.empty()) return fail(ARX_ERR_INVALID_ARGUMENT, "group is NULL or empty");
    return arx_copy_ir(g->members[0], h_left, h_right, ir_len);
}

arx_status arx_group_allreduce_f64(arx_group* g, double* values, size_t n, int op) {
    if (!g || g->members.empty() || (n > 0 && !values) || (op != 0 && op != 1))
        return fail(ARX_ERR_INVALID_ARGUMENT, "bad arguments");
    if (g->comms.empty() || n == 0 || ((int32_t)g->members.size() == g->n_ranks && !g->force_collectives))
        return ARX_OK;  // one process (unless arx_debug_group_force_collectives)
    for (arx_renderer* r : g->members) {  // nothing of a frame in flight left ahead of this collective
        const arx_status st0 = sync_renderer(r);
        if (st0 != ARX_OK) return st0;
    }
    // this process's values enter through member 0; the other local members add the identity.  Out
    // of place (arx_debug_group_force_collectives): into receive buffers pre-filled with NaN.
    const bool oop = g->out_of_place;
    std::vector<double*> bufs(g->members.size(), nullptr), outs(g->members.size(), nullptr);
    std::vector<double> ident(n, op == 0 ? 0.0 : -HUGE_VAL);
    arx_status st = ARX_OK;
    for (size_t i = 0; i < g->members.size() && st == ARX_OK; ++i) {
        arx_renderer* r = g->members[i];
        if (hipSetDevice(r->cfg.device) != hipSuccess || hipMalloc(&bufs[i], n * sizeof(double)) != hipSuccess ||
            hipMemcpyAsync(bufs[i], i == 0 ? values : ident.data(), n * sizeof(double), hipMemcpyHostToDevice,
                           r->stream) != hipSuccess)
            st = fail(ARX_ERR_HIP, "arx_group_allreduce_f64: staging failed");
        else if (oop && (hipMalloc(&outs[i], n * sizeof(double)) != hipSuccess ||
                         hipMemsetAsync(outs[i], 0xFF, n * sizeof(double), r->stream) != hipSuccess))
            st = fail(ARX_ERR_HIP, "arx_group_allreduce_f64: staging failed");
        if (!oop) outs[i] = bufs[i];
    }
    if (st == ARX_OK) {
        ncclGroupStart();
        ncclResult_t e = ncclSuccess;
        for (size_t i = 0; i < g->members.size() && e == ncclSuccess; ++i)
            e = ncclAllReduce(bufs[i], outs[i], n, ncclFloat64, op == 0 ? ncclSum : ncclMax, g->comms[i],
                              g->members[i]->stream);
        const ncclResult_t e2 = ncclGroupEnd();
        if (e != ncclSuccess || e2 != ncclSuccess)
            st = fail(ARX_ERR_HIP, "ncclAllReduce(f64) failed: %s", ncclGetErrorString(e != ncclSuccess ? e : e2));
        else
            ++g->n_coll[1];
    }
    if (st == ARX_OK) {
        arx_renderer* r0 = g->members[0];
        if (hipSetDevice(r0->cfg.device) != hipSuccess ||
            hipMemcpyAsync(values, outs[0], n * sizeof(double), hipMemcpyDeviceToHost, r0->stream) != hipSuccess)
            st = fail(ARX_ERR_HIP, "arx_group_allreduce_f64: download failed");
    }
    for (size_t i = 0; i < g->members.size(); ++i) {
        hipSetDevice(g->members[i]->cfg.device);
        hipStreamSynchronize(g->members[i]->stream);
        hipFree(bufs[i]);
        if (oop) hipFree(outs[i]);
    }
    return st;
}

arx_status arx_debug_group_force_collectives(arx_group* g, int32_t on, int32_t out_of_place) {
    if (!g || g->members.empty()) return fail(ARX_ERR_INVALID_ARGUMENT, "group is NULL or empty");
    if (on && g->comms.empty())
        return fail(ARX_ERR_INVALID_ARGUMENT, "an oversubscribed group (one GPU listed several times) has no communicator");
    for (arx_renderer* r : g->members) {  // nothing of a frame in flight left behind the switch
        const arx_status st = sync_renderer(r);
        if (st != ARX_OK) return st;
    }
    g->force_collectives = on != 0;
    g->out_of_place = on != 0 && out_of_place != 0;
    return ARX_OK;
}

arx_status arx_debug_group_collectives(const arx_group* g, uint64_t* out3) {
    if (!g || !out3) return fail(ARX_ERR_INVALID_ARGUMENT, "NULL argument");
    for (int k = 0; k < 3; ++k) out3[k] = g->n_coll[k];
    return ARX_OK;
}

arx_status arx_runtime_info(char* buf, size_t len) {
    if (!buf || len == 0) return fail(ARX_ERR_INVALID_ARGUMENT, "NULL buffer");
    Dl_info hip_dl, nccl_dl;
    const char* hip_path = dladdr(reinterpret_cast<void*>(&hipGetDeviceCount), &hip_dl) && hip_dl.dli_fname
                               ? hip_dl.dli_fname : "?";
    const char* nccl_path = dladdr(reinterpret_cast<void*>(&ncclGetVersion), &nccl_dl) && nccl_dl.dli_fname
                                ? nccl_dl.dli_fname : "?";
    int hv = 0, nv = 0;
    hipRuntimeGetVersion(&hv);
    ncclGetVersion(&nv);
    std::snprintf(buf, len, "hip=%s (runtime %d) rccl=%s (version %d)", hip_path, hv, nccl_path, nv);
    return ARX_OK;
}

arx_status arx_group_get_stats(arx_group* g, arx_stats* out) {
    if (!g || g->members.empty() || !out) return fail(ARX_ERR_INVALID_ARGUMENT, "NULL argument");
    arx_stats sum;
    std::memset(&sum, 0, sizeof(sum));
    for (arx_renderer* r : g->members) {
        arx_stats s;
        const arx_status st = arx_get_stats(r, &s);
        if (st != ARX_OK) return st;
        sum.queries += s.queries;
        sum.receiver_hits += s.receiver_hits;
        sum.misses += s.misses;
        sum.trace_ms = std::max(sum.trace_ms, s.trace_ms);
        sum.conv_ms = std::max(sum.conv_ms, s.conv_ms);
        sum.n_scene_tris = s.n_scene_tris;
        sum.n_receiver_tris = s.n_receiver_tris;
        sum.n_nodes = s.n_nodes;
        sum.bvh_depth = s.bvh_depth;
        sum.tree_hash = s.tree_hash;
        sum.trace_vgprs = s.trace_vgprs;
        sum.trace_waves_per_simd = s.trace_waves_per_simd;
        sum.trace_waves_target = s.trace_waves_target;
        sum.trace_format = s.trace_format;
        sum.trace_grid_cus = s.trace_grid_cus;
    }
    *out = sum;
    return ARX_OK;
}

}  // extern "C"
