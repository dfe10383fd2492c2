/*
 * arx.h -- C ABI of the MI355X acoustic impulse-response engine (libarx.so).
 *
 * Drop-in boundary for the GPU path of sgrazi/AudioRenderingV2's obj_raytracer.
 * The reference exposes that path as the C++ class AudioRenderer
 * (R/prebuild/obj_raytracer/AudioRenderer.h:16-152) over free CUDA/cuFFT
 * functions (R/prebuild/obj_raytracer/kernels.cuh:17-28).  Every entry point
 * below names the reference member/function it replaces.  Plain pointers and
 * sizes only; no C++ or torch types.  Every call returns an arx_status
 * (the reference throws or exit()s: optix7.h:8-45, kernels.cu:7-68); the
 * message of the last failure on the calling thread is arx_last_error().
 *
 * Threading: one renderer is driven by one host thread at a time (the
 * reference's AudioRenderer is not thread-safe either, AudioRenderer.h; the
 * app serialises it with output_buffer_mutex, main.cpp:38-63).  All GPU work
 * is issued on the renderer's HIP stream (arx_set_stream), never the null
 * stream; calls that return host data synchronise that stream.
 */
#ifndef ARX_H
#define ARX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ARX_ABI_VERSION 2

typedef enum arx_status {
    ARX_OK = 0,
    ARX_ERR_INVALID_ARGUMENT = 1,
    ARX_ERR_HIP = 2,          /* HIP runtime / kernel failure (reference: CUDA_CHECK throw) */
    ARX_ERR_OUT_OF_MEMORY = 3,
    ARX_ERR_NOT_READY = 4,    /* e.g. render before a scene was set */
    ARX_ERR_IO = 5,
    ARX_ERR_INTERNAL = 6      /* device-side invariant violated (e.g. BVH stack overflow) */
} arx_status;

typedef struct arx_renderer arx_renderer;

/* Construction parameters: Context::loadContext (R/prebuild/obj_raytracer/Context.cpp:15-236)
 * feeding AudioRenderer(model, ir_length_in_seconds, sample_rate, materials, rays)
 * (AudioRenderer.h:24) and the setters called before render (main.cpp:548-553). */
typedef struct arx_config {
    int32_t rays_x, rays_y, rays_z;     /* rays.{x,y,z}; N = x*y*z (Context.cpp:125-133) */
    uint32_t ir_length_in_seconds;      /* renderer_parameters.ir_length_in_seconds (rounded) */
    int32_t sample_rate;                /* audio file rate, 44100 in live mode (Context.cpp:197-224) */
    float base_power;                   /* pathtracer_parameters.base_power */
    float energy_thres;                 /* ray_energy_threshold */
    uint32_t max_bounces;               /* ray_max_bounces (rounded) */
    float hrtf_absorption_rate;         /* round()ed by the reference config reader (Context.cpp:145) */
    int32_t is_mono;                    /* scene_parameters.mono */
    uint64_t seed;                      /* Philox key; replaces curand_init(clock64(), tid) (devicePrograms.cu:216-217) */
    int32_t device;                     /* HIP device ordinal (reference hard-codes 0, AudioRenderer.cpp:252) */
} arx_config;

typedef struct arx_stats {
    uint64_t queries;        /* closest-hit queries issued (== optixTrace calls) */
    uint64_t receiver_hits;  /* rays terminated on a receiver half */
    uint64_t misses;         /* rays terminated by __miss__radiance */
    double trace_ms;         /* device time of the last trace kernel (HIP events) */
    double conv_ms;          /* device time of the last convolution */
    int64_t n_scene_tris, n_receiver_tris, n_nodes;
    int32_t bvh_depth;
    /* guards for stored profiles (bench.py): the scene tree's content hash (nodes + triangle
     * records of the static scene), and the production trace kernel's register allocation as the
     * runtime reports it (hipFuncGetAttributes) with the waves per SIMD it admits and the waves per
     * SIMD the persistent launch is sized for (a mismatch means the compiler changed the
     * allocation: the launch would leave SIMDs unevenly loaded) */
    uint64_t tree_hash;
    int32_t trace_vgprs;
    int32_t trace_waves_per_simd;
    int32_t trace_waves_target;
    int32_t trace_format;    /* node format of the last trace launch: 0 f32 BVH2, 1 16-bit quantized BVH2,
                              * 2 4-wide compressed (CW4) */
    int32_t trace_grid_cus;  /* CUs the last trace launch's persistent grid was sized for: the device's,
                              * or half of them for a ray-pool launch with frames in flight (its wave
                              * slots then hold two frames' launches side by side, arx_set_frames_in_flight) */
} arx_stats;

const char* arx_status_string(arx_status s);
const char* arx_last_error(void);
int arx_abi_version(void);
void arx_default_config(arx_config* cfg); /* the reference's defaults (Context.cpp:19-117) */

/* AudioRenderer::AudioRenderer (AudioRenderer.h:24; AudioRenderer.cpp:60-93):
 * allocates the IR histogram/IR buffers (ir_len = ir_length_in_seconds*sample_rate bins). */
arx_status arx_create(const arx_config* cfg, arx_renderer** out);
void arx_destroy(arx_renderer* r);
arx_status arx_get_config(const arx_renderer* r, arx_config* out);
/* Issue all work on this hipStream_t, used as given (NULL = the legacy null stream).  The
 * renderer starts on a non-blocking stream of its own; arx_get_stream returns the current one. */
arx_status arx_set_stream(arx_renderer* r, void* hip_stream);
void* arx_get_stream(const arx_renderer* r);

/* ---- Device buffers and runtime -------------------------------------------------------------
 * Small helpers so that a caller (bench.py, a C host) needs no other GPU framework for its device
 * buffers and can see which HIP / RCCL runtime libarx resolved.  No reference equivalent (its
 * CUDABuffer, CUDABuffer.h:10-68, is internal). */
int32_t arx_device_count(void); /* HIP devices visible to this process; < 0 on error */
arx_status arx_device_alloc(int32_t device, size_t bytes, void** out);
void arx_device_free(int32_t device, void* p);
/* Synchronous copy between any two of host / device memory (hipMemcpyDefault). */
arx_status arx_memcpy(int32_t device, void* dst, const void* src, size_t bytes);
/* "hip=<path of the loaded libamdhip64> (runtime version) rccl=<path of the loaded librccl>
 * (version)" into buf[len]. */
arx_status arx_runtime_info(char* buf, size_t len);
/* Scene trees built by this process so far (arx_set_scene / arx_group_set_scene): a group builds
 * its tree once and shares it between its members, and geometry identical to a scene some renderer
 * still holds reuses that build (a process-wide cache keyed by a 128-bit hash of the arrays). */
uint64_t arx_scene_build_count(void);

/* Static scene geometry: AudioRenderer::buildAccel + buildSBT (AudioRenderer.cpp:95-218, 413-464),
 * with getMaterialAbsorption (:34-56) already applied per triangle by the caller
 * (arx_material_absorption).  tri_vertices: n_tris*9 floats (P1,P2,P3 in mesh index order);
 * triangle order is the global id used to break equal-distance ties.  Builds the
 * SAH BVH on the host and uploads it (once; receivers are kept in a separate sub-tree).
 * Absorption must lie in [0, 1] (or be -1 / -2, the receiver marks): unlike the reference, which
 * takes any config value, the int64 fixed-point IR needs energies that never grow. */
arx_status arx_set_scene(arx_renderer* r, const float* tri_vertices, const float* tri_absorption,
                         int64_t n_tris);
/* The two receiver half-spheres in their local frame: HalfSphere (HalfSphere.cpp:3-31) loaded
 * from leftHalf.obj (side 0) / rightHalf.obj (side 1); n_tris*9 floats. */
arx_status arx_set_receiver_model(arx_renderer* r, int side, const float* tri_vertices_local,
                                  int64_t n_tris);
/* place_receiver_half's vertex transform alone (OptixModel.cpp:178-193): v' = (x,y,z) +
 * rotate(-radians(yaw), +Y) * v with glm's operation order; host-only, no device needed. */
arx_status arx_place_receiver_vertices(const float* local_xyz, int64_t n_vertices, float x, float y, float z,
                                       float yaw_deg, float* out_xyz);
/* getMaterialAbsorption (AudioRenderer.cpp:34-56): receiver_left -1, receiver_right -2,
 * exact name match in the config list, else 0.5. */
float arx_material_absorption(const char* name, const char* const* names, const float* absorption,
                              size_t n_materials);

/* setEmitterPosInOptix (AudioRenderer.cpp:752-756). */
arx_status arx_set_emitter(arx_renderer* r, float x, float y, float z);
/* placeReceiver + setSphereCenterInOptix (OptixModel.cpp:153-257, AudioRenderer.cpp:758-762):
 * receiver halves rotated by -yaw about +Y, translated to (x,y,z); sphere center = (x,y,z).
 * Rebuilds only the receiver sub-tree (no full rebuild, unlike reload() :466-486). */
arx_status arx_set_listener(arx_renderer* r, float x, float y, float z, float yaw_deg);
arx_status arx_set_thresholds(arx_renderer* r, float energy, uint32_t max_bounces); /* :764-768 */
arx_status arx_set_hrtf_absorption_rate(arx_renderer* r, float rate);             /* :770-773 */
arx_status arx_set_base_power(arx_renderer* r, float base_power);                 /* :775-778 */
arx_status arx_set_mono_output(arx_renderer* r, int mono);                        /* :800-803 */
arx_status arx_set_seed(arx_renderer* r, uint64_t seed);

/* AudioRenderer::render (AudioRenderer.h:27; AudioRenderer.cpp:489-523): clear, trace all
 * N rays, finalize the stereo IR (mono merge = addIRs, kernels.cu:519-527).  render_ms gets the
 * trace kernel's device time (the reference's timed window, :495-518). */
arx_status arx_render(arx_renderer* r, double* render_ms);
/* Frames in flight (n = 1 to 3; no reference equivalent -- its render() blocks, AudioRenderer.cpp:
 * 489-523).  With n > 1, consecutive render() calls rotate over n streams, histograms and IRs:
 * frame k + 1 traces while frame k's trace finishes and its IR is convolved, so a render/convolute
 * loop keeps the GPU full.  Results are those of one frame at a time, bit for bit: every getter,
 * convolution and IR copy refers to the last frame started, and the two frames meet only where they
 * share state (scene and receiver uploads wait for the other frame's trace; convolutions, IR
 * spectra and the caller's output buffers for its convolution).  A trace launch large enough for
 * the ray pool is then sized for half the CUs' wave slots (arx_stats.trace_grid_cus), so two frames'
 * launches run side by side instead of meeting only in each other's tail; a single frame
 * (arx_set_frames_in_flight(r, 1)) is therefore faster alone, a render/convolute loop faster in
 * total.  Not with arx_set_stream or arx_attach_histogram (ARX_ERR_INVALID_ARGUMENT either way
 * round). */
arx_status arx_set_frames_in_flight(arx_renderer* r, int32_t n);

/* Building blocks of render() for ray-sharded multi-GPU use (no reference equivalent; the
 * reference is single-GPU).  The histogram is 2*ir_len int64 in device memory: [L | R],
 * fixed point with unit e0*2^-frac_bits, so a sum over shards (RCCL int64 SUM) is exact. */
arx_status arx_clear_histogram(arx_renderer* r);
/* Global ray ids, ray_end <= N = x*y*z (the energy and fixed-point normalisation assume N rays). */
arx_status arx_trace_rays(arx_renderer* r, uint64_t ray_begin, uint64_t ray_end);
arx_status arx_histogram_device(arx_renderer* r, int64_t** d_hist, size_t* n_elems);
/* Accumulate into caller-owned device memory (2*ir_len int64, e.g. a torch tensor that RCCL
 * all-reduces in place); NULL restores the renderer's own buffer. */
arx_status arx_attach_histogram(arx_renderer* r, int64_t* d_hist, size_t n_elems);
arx_status arx_finalize_ir(arx_renderer* r);
arx_status arx_ir_device(arx_renderer* r, float** d_left, float** d_right, size_t* ir_len);
arx_status arx_copy_ir(arx_renderer* r, float* h_left, float* h_right, size_t ir_len);
/* Counters of the last frame (synchronises the renderer's stream).  ARX_ERR_INTERNAL (stats still
 * filled in) when the tree as last written has a box off the 16-bit quantization grid (receiver refit
 * or device re-quantization; never with the host's grid bounds). */
arx_status arx_get_stats(arx_renderer* r, arx_stats* out);
/* Device times (HIP events on the renderer's stream) of the last min(n, arx_timing_ring()) trace launches, oldest
 * first, into ms[0..*n_out); synchronises on them.  The reference's timed window (Time taken by
 * Optix, AudioRenderer.cpp:495-518), kept per launch so a benchmark can average a timed region. */
arx_status arx_trace_times(arx_renderer* r, double* ms, size_t n, size_t* n_out);
/* The same for the last min(n, 64) file convolutions (arx_convolute_device / _audio_file; the
 * reference's "Time taken just to convolute", AudioRenderer.cpp:688-696). */
arx_status arx_conv_times(arx_renderer* r, double* ms, size_t n, size_t* n_out);
/* The same for the last min(n, 64) live-path convolutions (arx_convolute_live_* and the streaming
 * convolution's blocks, arx_stream_process*). */
arx_status arx_live_times(arx_renderer* r, double* ms, size_t n, size_t* n_out);
/* Capacity of the per-launch timing rings above (launches kept). */
int32_t arx_timing_ring(void);
/* Per-launch timing on (1, the default) or off (0).  Each timed launch puts two event markers on the
 * stream, ~4.5 us of stream time apiece on MI355X (tools/step_gaps.py): off, trace and file
 * convolution launches go to the stream alone and the rings above stop growing.  A call that asks
 * for its time -- arx_render / arx_group_render with render_ms, arx_convolute_audio_file with
 * convolute_ms -- is timed either way, as the reference times render() only when render_ms is given
 * (AudioRenderer.h:27).  arx_get_stats' trace_ms / conv_ms then report the last timed launch. */
arx_status arx_set_timing(arx_renderer* r, int32_t on);

/* Identity of the trace kernel compiled into this library: a hash of its sources and experiment
 * macros (build.py trace_source_id).  Stored PMC profiles carry it with the tree hash and VGPR
 * count, and bench.py uses a stored profile only when all three match its own run.  No
 * reference counterpart (measurement plumbing). */
uint64_t arx_trace_kernel_id(void);
/* The same for the file convolution's kernels (build.py conv_source_id): the guard of the stored
 * convolution traffic profile (profiles/<round>/conv_traffic.json). */
uint64_t arx_conv_kernel_id(void);
/* Replace the renderer's IR with caller data (host, ir_len floats per ear), e.g. a stored or
 * measured IR; the next convolution uses it.  No reference equivalent (its IR only comes
 * from render()). */
arx_status arx_set_ir(arx_renderer* r, const float* h_left, const float* h_right, size_t ir_len);
/* Same from device memory on the renderer's device (e.g. another renderer's IR, arx_ir_device),
 * asynchronous on the renderer's stream: the caller orders it after the IR's producer (a HIP
 * event) and keeps the source unchanged until the copy has run. */
arx_status arx_set_ir_device(arx_renderer* r, const float* d_left, const float* d_right, size_t ir_len);
int arx_frac_bits(uint64_t n_rays_total);

/* ---- Multi-GPU ray sharding ------------------------------------------------------------------
 * No reference equivalent: the reference renders on device 0 only (AudioRenderer.cpp:252) and has
 * no collective (SURVEY.md §2, §8b "set device count", §8e).  A group holds one renderer per GPU;
 * rank g of G traces the global ray ids [g*N/G, (g+1)*N/G) of the same N = x*y*z ray launch, and
 * ONE RCCL all-reduce (int64 SUM over xGMI) of the 2*ir_len fixed-point histogram leaves the full
 * IR on every member -- exact, so the IR is bitwise independent of G.  Convolution then runs on any
 * member (arx_group_member + arx_convolute_*). */
typedef struct arx_group arx_group;
/* One process driving n_devices GPUs: devices[i] (devices NULL = 0..n_devices-1), ncclCommInitAll
 * (also for n_devices = 1).  cfg->device is ignored.  Listing ONE device several times
 * oversubscribes it (e.g. to run the sharded path on a single-GPU box): RCCL cannot take a device
 * twice, so such a group sums its shards on that device instead (the same exact int64 sum). */
arx_status arx_group_create(const arx_config* cfg, const int32_t* devices, int32_t n_devices, arx_group** out);
/* One GPU per process (torchrun-style launch): rank 0 calls arx_group_unique_id and shares the
 * ARX_GROUP_ID_BYTES bytes out of band; every rank then calls arx_group_create_rank with its rank and
 * cfg->device (ncclCommInitRank).  id may be NULL when n_ranks == 1. */
#define ARX_GROUP_ID_BYTES 128
arx_status arx_group_unique_id(uint8_t* id, size_t id_bytes);
arx_status arx_group_create_rank(const arx_config* cfg, int32_t n_ranks, int32_t rank, const uint8_t* id,
                                 size_t id_bytes, arx_group** out);
void arx_group_destroy(arx_group* g);
int32_t arx_group_members(const arx_group* g); /* renderers in this process */
int32_t arx_group_ranks(const arx_group* g);   /* G: shards of the launch */
/* Member i's renderer (owned by the group; NULL if out of range) for convolution / IR access. */
arx_renderer* arx_group_member(arx_group* g, int32_t i);
/* The scene tree is built ONCE per group on the host and shared by every member (each uploads it
 * to its own device); in a one-GPU-per-process group (arx_group_create_rank) this is collective:
 * rank 0 builds and the tree goes to the other ranks with one RCCL broadcast over xGMI, so every
 * rank must call it (their arrays are not read). */
arx_status arx_group_set_scene(arx_group* g, const float* tri_vertices, const float* tri_absorption, int64_t n_tris);
/* The shard of rank `rank` of `n_ranks` in an n-ray launch: global ray ids [begin, end) =
 * [rank*n/n_ranks, (rank+1)*n/n_ranks) (exact 128-bit products).  Host only; arx_group_render uses it. */
void arx_group_shard(uint64_t n_rays, int32_t rank, int32_t n_ranks, uint64_t* begin, uint64_t* end);
/* Tests only: arx_group_set_scene's one-GPU-per-process hand-over (rank 0 checks and builds the
 * scene, the other ranks read its broadcast byte image; a failure on any rank fails the call on all)
 * over a caller's transport instead of RCCL.  word(ctx, v, op): op 0 = broadcast *v from rank 0,
 * op 1 = all-reduce max into *v; bytes(ctx, buf, n): broadcast n bytes from rank 0's buf into every
 * rank's; both collective, 0 on success.  Host only; tree_hash = the tree every rank now holds. */
typedef int (*arx_share_u64_fn)(void* ctx, uint64_t* value, int op);
typedef int (*arx_share_bytes_fn)(void* ctx, uint8_t* buf, uint64_t n);
arx_status arx_debug_share_scene(int32_t rank, const float* tri_vertices, const float* tri_absorption, int64_t n_tris,
                                 arx_share_u64_fn word, arx_share_bytes_fn bytes, void* ctx, uint64_t* tree_hash);
/* The single-renderer setters, applied to every member. */
arx_status arx_group_set_receiver_model(arx_group* g, int side, const float* tri_vertices_local, int64_t n_tris);
arx_status arx_group_set_emitter(arx_group* g, float x, float y, float z);
arx_status arx_group_set_listener(arx_group* g, float x, float y, float z, float yaw_deg);
arx_status arx_group_set_thresholds(arx_group* g, float energy, uint32_t max_bounces);
arx_status arx_group_set_hrtf_absorption_rate(arx_group* g, float rate);
arx_status arx_group_set_base_power(arx_group* g, float base_power);
arx_status arx_group_set_mono_output(arx_group* g, int mono);
arx_status arx_group_set_seed(arx_group* g, uint64_t seed);
/* render() over the group: clear, trace every local shard, all-reduce, finalize on every member
 * (async on the members' streams).  render_ms (if not NULL; synchronises) = the longest shard's
 * trace kernel time.  After an error the members may be at different frames (and, on the rank path,
 * peers may wait in the collective this rank skipped): destroy the group, do not render on it again. */
arx_status arx_group_render(arx_group* g, double* render_ms);
/* arx_set_frames_in_flight on every member; a member's all-reduce waits for its previous one, so
 * the collectives on each communicator keep their order.  That event chain runs on one GPU with
 * every collective forced (arx_debug_group_force_collectives, tests/test_gpu_collectives.py: 1 to 3
 * frames, in and out of place, bit-identical to a plain renderer); its first multi-GPU run is the
 * 8-GPU bench, which keeps the one-GPU frames-in-flight policy at every N. */
arx_status arx_group_set_frames_in_flight(arx_group* g, int32_t n);
/* arx_set_timing on every member; with it on (or render_ms asked for), arx_group_render also puts HIP
 * events around each member's histogram all-reduce. */
arx_status arx_group_set_timing(arx_group* g, int32_t on);
/* Device times of member `member`'s last min(n, 256) timed histogram all-reduces (the RCCL collective's
 * window on that member's stream, queueing behind the member's own trace excluded), oldest first;
 * synchronises on them.  *n_out = 0 when no all-reduce was timed (a one-rank group skips its no-op
 * all-reduce unless arx_debug_group_force_collectives). */
arx_status arx_group_allreduce_times(arx_group* g, int32_t member, double* ms, size_t n, size_t* n_out);

/* Time-block sharded file convolution ("time blocks sharded ... only the n - sr overlap
 * is summed at shard seams"; the reference convolves on one GPU, kernels.cu:404-430).  The file's
 * floor(n/sr) one-second blocks form P = ceil(blocks / 2) FFT pairs; rank g of G convolves the pairs
 * [g*P/G, (g+1)*P/G) with its member's IR and writes the output frames they own,
 * arx_group_conv_shard's [begin, end), into its member's full-length buffers d_out_left[i] /
 * d_out_right[i] (n_frames floats each, on member i's device; d_in[i] there holds the whole file).
 * The seam -- the tail of the block before a shard -- is re-made by the shard itself from that block's
 * input, not received from the neighbour, so the data path has no collective; the union of the ranks'
 * frames is arx_convolute_device's output bit for bit.  Plans without the chained pass
 * (arx_group_conv_sharded == 0: ir_len != 2 sr, or an IR length without a direct mixed-radix split)
 * convolve and write the whole file on every rank.  Asynchronous on the members' streams, like
 * arx_convolute_device; arx_conv_times per member time each shard. */
arx_status arx_group_convolute_device(arx_group* g, const float* const* d_in, size_t n_frames,
                                      float* const* d_out_left, float* const* d_out_right);
/* AudioRenderer::convoluteAudioFile over the group (AudioRenderer.cpp:663-750: host buffers, sizes in
 * BYTES, reference normalisation): every member of this process convolves its time-block shard
 * (arx_group_convolute_device), copying in only the input its pairs read and copying back only the
 * frames it owns, so in a group of one process over several GPUs h_out_left / h_out_right receive
 * the whole convolved file -- bit-identical to arx_convolute_audio_file -- with the work spread over
 * the GPUs.  On the one-GPU-per-process path each process fills its own ranks' frames (the caller
 * gathers).  One rank, or a plan that does not shard: arx_convolute_audio_file on member 0.
 * convolute_ms = the longest member's convolution window, process_ms = the longest member's whole
 * call window (copies included); synchronising. */
arx_status arx_group_convolute_audio_file(arx_group* g, const float* h_in, size_t in_bytes, float* h_out_left,
                                          float* h_out_right, double* convolute_ms, double* process_ms);
/* The output frames [begin, end) rank `rank` of n_ranks owns in a sharded convolution of n_frames at
 * sample_rate (host only; ranges of the ranks tile [0, n_frames)). */
void arx_group_conv_shard(int32_t sample_rate, uint64_t n_frames, int32_t rank, int32_t n_ranks, uint64_t* begin,
                          uint64_t* end);
/* 1 if the group's convolution plan shards (see arx_group_convolute_device), 0 if every rank convolves
 * the whole file, -1 on error. */
int32_t arx_group_conv_sharded(arx_group* g);
arx_status arx_group_synchronize(arx_group* g);
arx_status arx_group_copy_ir(arx_group* g, float* h_left, float* h_right, size_t ir_len); /* member 0 */
/* Queries / receiver hits / misses summed over this process's members; times = the longest. */
arx_status arx_group_get_stats(arx_group* g, arx_stats* out);
/* values[0..n) of this process combined over all processes of the group (op 0 = sum, 1 = max)
 * with one RCCL all-reduce, in place; synchronising, so it doubles as a barrier.  A group whose
 * members all live in this process returns values unchanged. */
arx_status arx_group_allreduce_f64(arx_group* g, double* values, size_t n, int op);

/* AudioRenderer::convoluteAudioFile (AudioRenderer.h:31; AudioRenderer.cpp:663-750) over
 * convoluteFromAudioBuffer (kernels.cuh:21; kernels.cu:382-438): 1-s blocks zero padded to
 * ir_len, circular convolution with each IR, overlap-added, tail (len mod sr) unprocessed,
 * divided by (ir_len/2).  Host buffers, sizes in BYTES like the reference. */
arx_status arx_convolute_audio_file(arx_renderer* r, const float* h_in, size_t in_bytes, float* h_out_left,
                                    float* h_out_right, double* convolute_ms, double* process_ms);
/* Same on device-resident buffers (n_frames floats each); no host synchronisation. */
arx_status arx_convolute_device(arx_renderer* r, const float* d_in, size_t n_frames, float* d_out_left,
                                float* d_out_right);
/* Input reuse for the reference's re-render pattern: full_render_cycle (AudioRenderer.cpp:790-798,
 * called by main.cpp:40-67 on every listener move) convolves the SAME file with every new IR.
 * arx_convolute_prepare_input transforms the file's one-second blocks once (device input, n_frames
 * samples).  The transform is queued on the renderer's stream, not run by the call: the caller may
 * overwrite d_in only once that stream has finished it (after arx_get_stats, arx_copy_ir or a
 * synchronisation of the stream, or from work ordered after it on that stream); arx_convolute_prepared then
 * convolves them with the renderer's current IR into the caller's device outputs (n_frames each,
 * *n_frames set when non-NULL) -- bit-identical to arx_convolute_device on the same input, without
 * the input's forward transform.  The prepared input stays until the next arx_convolute_device /
 * arx_convolute_audio_file / arx_convolute_prepare_input on this renderer (ARX_ERR_NOT_READY after). */
arx_status arx_convolute_prepare_input(arx_renderer* r, const float* d_in, size_t n_frames);
arx_status arx_convolute_prepared(arx_renderer* r, float* d_out_left, float* d_out_right, size_t* n_frames);

/* AudioRenderer::convoluteLiveInput (AudioRenderer.h:29; AudioRenderer.cpp:593-661) over
 * convoluteFromLiveInput (kernels.cu:345-377) minus the CircularBuffer (which stays with the
 * caller, include/arx_circular_buffer.hpp): one mic block of in_bytes/8 f64 samples (<= ir_len),
 * zero padded to ir_len, circularly convolved with each IR in f64, divided by (ir_len/2) and
 * zipped L/R into h_out[2*ir_len] (out_len must be 2*ir_len).  IR spectra are cached between
 * callbacks (the reference re-plans and re-transforms them every callback). */
arx_status arx_convolute_live_block(arx_renderer* r, const double* h_in, size_t in_bytes, double* h_out,
                                    size_t out_len);
/* Same on device buffers (n_in f64 samples in, 2*ir_len f64 out), no host synchronisation. */
arx_status arx_convolute_live_device(arx_renderer* r, const double* d_in, size_t n_in, double* d_out);
/* Recompute the cached IR spectra now (async on the renderer's stream) instead of lazily in the
 * next convolution: which = 1 file path, 2 live path, 3 both.  Lets a moving-listener frame
 * (re-trace + reduce + new spectra) finish before audio needs it. */
arx_status arx_prepare_ir_spectra(arx_renderer* r, int which);
/* Describe the convolution plan (which = 1 file path, 2 live path; created if needed) into
 * buf[len]: "mixed-radix direct circular: n=.. sr=.. (N1xN2) f64" when ir_len factors into two
 * 7-smooth sub-lengths <= 512 (FFT length = ir_len, as the reference's cuFFT plans), else
 * "pow2 linear+fold: ..." (power-of-two length >= ir_len + block - 1, folded back). */
arx_status arx_conv_describe(arx_renderer* r, int which, char* buf, size_t len);

/* Streaming convolution for the RtAudio duplex callback (replaces the
 * per-callback full-length circular convolution of convoluteLiveInput, AudioRenderer.cpp:593-661,
 * whose 2*ir_len outputs the reference's CircularBuffer wraps onto itself, main.cpp:189-195, which
 * stays available as arx_convolute_live_block -- the compat path).  Uniformly partitioned
 * overlap-save in f64 on the renderer's device and stream: each call consumes one block of
 * n_frames <= block_frames f64 input frames (shorter blocks are zero padded) and returns
 * block_frames output frames zipped L/R (2*block_frames doubles) = the linear convolution of the
 * input stream with the renderer's current IR, scaled like the reference's live path
 * (ir_len / (ir_len/2), normalizeBuffers).  Latency: one block.  A new IR (render, set_ir) applies
 * from the next block on; the input history is kept.  block_frames in [1, min(4096, ir_len)]. */
typedef struct arx_stream arx_stream;
arx_status arx_stream_create(arx_renderer* r, int32_t block_frames, arx_stream** out);
void arx_stream_destroy(arx_stream* s);
arx_status arx_stream_reset(arx_stream* s); /* forget the input history */
arx_status arx_stream_info(const arx_stream* s, int32_t* block_frames, int32_t* partitions, int32_t* fft_size);
arx_status arx_stream_process(arx_stream* s, const double* h_in, size_t n_frames, double* h_out, size_t out_len);
/* Same on device buffers (n_frames f64 in, 2*block_frames f64 out), no host synchronisation. */
arx_status arx_stream_process_device(arx_stream* s, const double* d_in, size_t n_frames, double* d_out);

/* Tests only: issue every collective of the group even at one rank -- the histogram all-reduce of
 * arx_group_render (with frames in flight on every member's frame stream, chained by events), the
 * f64 all-reduce of arx_group_allreduce_f64 and the rank path's scene broadcast of
 * arx_group_set_scene -- so a one-GPU box runs the RCCL call paths a multi-GPU job takes.  out_of_place
 * != 0: the all-reduces write separate receive buffers pre-filled with 0xFF (the histogram's is then
 * copied back), so the result is right only if the collective moved the data.  Synchronises the
 * members first.  ARX_ERR_INVALID_ARGUMENT for a group without a communicator (one GPU listed
 * several times). */
arx_status arx_debug_group_force_collectives(arx_group* g, int32_t on, int32_t out_of_place);
/* Collectives the group has issued: out3[0] histogram all-reduces, [1] f64 all-reduces, [2] scene
 * broadcasts (rank path). */
arx_status arx_debug_group_collectives(const arx_group* g, uint64_t* out3);

/* Debug / parity hooks. */
arx_status arx_debug_ray_directions(uint64_t seed, uint64_t first_ray, uint64_t count, float* h_out_xyz,
                                    int device);
/* Host only: build the scene tree, turn it into the byte image a rank-0 build broadcasts to the
 * other ranks (arx_group_set_scene), read it back and check it is the same tree; returns the tree's
 * content hash (arx_stats::tree_hash) and the image size. */
arx_status arx_debug_scene_roundtrip(const float* tri_vertices, const float* tri_absorption, int64_t n_tris,
                                     uint64_t* tree_hash, uint64_t* image_bytes);
/* The device node arrays as the last trace used them (synchronises): n_nodes coded f32 nodes
 * (64 B each) into cnodes and their 16-bit quantized copy (32 B each, made on the device) into
 * qnodes (either may be NULL), the quantization grid (origin xyz, scale xyz) into grid[6], and the
 * device re-quantizations issued so far into *requants. */
arx_status arx_debug_node_images(arx_renderer* r, void* cnodes, void* qnodes, size_t n_nodes, float* grid,
                                 uint64_t* requants);
/* Tests only: the most triangles the SAH builder may leave in one leaf (process-wide, for the
 * builds that follow; production 2, range 1..15), so leaves of more than two triangles -- which
 * production trees hold only below the builder's depth cap -- can be traced and checked. */
arx_status arx_debug_set_leaf_max(int32_t leaf_max);
/* Host only: build the scene, its 16-bit quantized BVH2 and its 4-wide compressed copy (CW4), and
 * trace n_rays random rays from the emitter through `bounces` specular reflections on the CPU with
 * both traversals (nearest first, f64 slab and triangle tests); out[16]: [0] queries, [1] / [2]
 * BVH2 node steps / triangle tests per query, [3] / [4] the same for CW4, [5] CW4 max stack depth,
 * [6] queries whose two closest hits differ, [7] CW4 nodes, [8] CW4 depth, [9] BVH2 nodes, [10]
 * BVH2 depth, [11] quantization failures, [12] misses, [13] CW4 99.9th-percentile stack depth,
 * [14] CW4 buffer units. */
arx_status arx_debug_wide_stats(const float* tri_vertices, const float* tri_absorption, int64_t n_tris,
                                const float* emitter, int64_t n_rays, int32_t bounces, uint64_t seed, double* out,
                                size_t n_out);
/* Profiling builds only (ARX_TRACE_PROF=1, tools/trace_profile.py): the last trace launch's
 * per-wave records, 16 uint64 per wave (start / end shader clock, rays, queries, node-step slots
 * and lane-steps, leaf phases and lanes, shade phases and lanes, loop iterations, the time the
 * wave's ray range ran out, wave id); ARX_ERR_NOT_READY in the product build. */
arx_status arx_debug_trace_profile(arx_renderer* r, uint64_t* out, size_t n_words, size_t* n_out);
/* Raw device counters of the last trace (n <= 8): [0] queries [1] receiver hits [2] misses. */
arx_status arx_debug_trace_counters(arx_renderer* r, uint64_t* out, size_t n);
/* Host only: the tree-size guard every scene passes (arx_set_scene, arx_group_set_scene): the trace
 * kernel addresses nodes (64 B) and triangle records (48 B) with 31-bit buffer offsets, so n_nodes * 64
 * and n_tris * 48 must stay <= 2^31 - 1 (ARX_ERR_INVALID_ARGUMENT beyond).  The 28-bit triangle index
 * of a leaf code (~(index * 16 + count)) is wider than that limit needs. */
arx_status arx_debug_check_tree_limits(uint64_t n_nodes, uint64_t n_tris);
/* Tests only: the receiver refit kernel's box padding (0 = automatic, the builder's pad).  A pad far
 * beyond the quantization grid's margin makes the refit raise the tree's off-grid flag (its quantized
 * boxes then fall back to whole-axis, still conservative), which arx_get_stats reports as
 * ARX_ERR_INTERNAL until a later tree write (a listener move, a new scene) is clean again. */
arx_status arx_debug_set_refit_pad(arx_renderer* r, float pad);
/* Force the trace kernel's other paths (parity tests of the paths real scenes rarely take): the
 * default is the 16-bit quantized BVH2 with the LDS stack; bit 0 = the f32 coded BVH2 (taken
 * automatically while the emitter is off the quantization grid), bit 1 = the global-memory
 * traversal stack (taken automatically for trees deeper than the LDS stack), bit 3 = the 4-wide
 * compressed tree (CW4, arx_layout.hpp: half the node loads per query, twice the VALU; slower on
 * MI355X, kept as a measured alternative); 0 = automatic. */
arx_status arx_debug_set_trace_path(arx_renderer* r, int path);

/* ---- Input formats (host only, no device needed) ------------------------------------------ */

/* OBJ scene / receiver model: tinyobj v2.0.0 LoadObj with triangulation (R/prebuild/common/
 * 3rdParty/tiny_obj_loader.h:2095-2600) then one mesh per (shape, material id ascending) with
 * (v,n,t) vertex dedup -- loadOBJ (R/prebuild/obj_raytracer/OptixModel.cpp:75-151).
 * mtl_dir NULL = the OBJ's directory (loadOBJ :79).  first_shape_only + forced_name give
 * HalfSphere + place_receiver_half (HalfSphere.cpp:3-31, OptixModel.cpp:197-220): pass
 * mtl_dir = path up to (excluding) the last '/', forced_name "receiver_left"/"receiver_right".
 * Fails (ARX_ERR_IO) when the OBJ has no materials, like the reference's throw. */
typedef struct arx_model arx_model;
arx_status arx_model_load_obj(const char* path, const char* mtl_dir, int first_shape_only,
                              const char* forced_name, arx_model** out);
void arx_model_free(arx_model* m);
int64_t arx_model_mesh_count(const arx_model* m);
int64_t arx_model_material_count(const arx_model* m);
/* tinyobj's shapes.size(), materials.size(), attrib.vertices.size()/3 */
void arx_model_info(const arx_model* m, int64_t* n_shapes, int64_t* n_materials, int64_t* n_positions);
/* Mesh i: TriangleMesh {material_name, vertex, index} (OptixModel.h); pointers live until free. */
arx_status arx_model_mesh(const arx_model* m, int64_t i, const char** name, const float** vertices,
                          int64_t* n_vertices, const int32_t** indices, int64_t* n_triangles);
int64_t arx_model_triangle_count(const arx_model* m);
/* Triangle soup for arx_set_scene (9 floats per triangle, meshes in model order) with
 * getMaterialAbsorption per mesh name (AudioRenderer.cpp:34-56, :455); tri_absorption may be NULL. */
arx_status arx_model_flatten(const arx_model* m, const char* const* names, const float* absorption,
                             size_t n_materials, float* tri_vertices, float* tri_absorption);

/* WAV: AudioFile<float>::load / decodeWaveFile (R/prebuild/obj_raytracer/AudioFile.h:502-640,
 * sample conversion :1242-1269): PCM 8/16/24/32-bit and IEEE float 32.  *samples is malloc'd,
 * channel-major (channels x frames, like AudioFile::samples); release with arx_free. */
arx_status arx_wav_load(const char* path, float** samples, int32_t* channels, int64_t* frames,
                        int32_t* sample_rate, int32_t* bit_depth);
void arx_free(void* p);

/* ---- Output formats (host only) ------------------------------------------------------------ */

/* AudioFile<float>::save as export_audio uses it (main.cpp:709-716; AudioFile.h:842-955):
 * samples channel-major; 32-bit is written as IEEE float, 8/16-bit are clamped to [-1, 1]. */
arx_status arx_wav_save(const char* path, const float* samples, int32_t channels, int64_t frames,
                        int32_t sample_rate, int32_t bit_depth);
/* normalizeToRangeMinusOneToOne (main.cpp:628-651), in place; constant input -> INVALID_ARGUMENT. */
arx_status arx_normalize_min_max(float* data, size_t n);
/* One value per line, std::ostream default float format -- the output_ir_{left,right}.txt and
 * output_convolute_{left,right}.txt dumps (AudioRenderer.cpp:525-567, 720-744). */
arx_status arx_write_float_lines(const char* path, const float* data, size_t n);

/* config.json: Context::loadContext's parameters (R/prebuild/obj_raytracer/Context.cpp:15-164)
 * with its defaults and rounding (unsigned fields and both re_render thresholds and
 * hrtf_absorption_rate are round()ed), parsed with cJSON 1.7.16 semantics (case-insensitive
 * keys, first duplicate wins, trailing text ignored). */
#define ARX_PATH_MAX 1024
#define ARX_NAME_MAX 128
#define ARX_MAX_MATERIALS 256
typedef struct arx_app_config {
    float initial_volume;
    uint32_t ir_length_in_seconds, width, height;
    int32_t write_first_ir_to_file, write_first_output_to_file;
    float re_render_distance_threshold, re_render_angle_threshold;
    int32_t mono;
    char scene_file_path[ARX_PATH_MAX];
    char audio_file_path[ARX_PATH_MAX];     /* "" = live mic input, sample rate 44100 */
    char materials_file_path[ARX_PATH_MAX];
    float initial_receiver_pos[3];
    float initial_emitter_pos[3];
    float base_power;
    float rays[3];                          /* gdt::vec3f; launch dims are int(rays) (LaunchParams.h:24) */
    float ray_energy_threshold;
    uint32_t ray_max_bounces;
    float hrtf_absorption_rate;
    int32_t n_materials;
    char material_names[ARX_MAX_MATERIALS][ARX_NAME_MAX];
    float material_absorption[ARX_MAX_MATERIALS];
} arx_app_config;
void arx_default_app_config(arx_app_config* c);
arx_status arx_parse_app_config(const char* text, size_t len, arx_app_config* c);
arx_status arx_load_app_config(const char* path, arx_app_config* c);

#ifdef __cplusplus
}
#endif
#endif /* ARX_H */
