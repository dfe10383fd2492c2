// arx_kernels.hpp -- host-callable launchers for the HIP kernels (libarx.so internals).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "arx_layout.hpp"

namespace arx {

// Trace kernel (raygen + traversal + closest-hit + histogram, fused) over rays
// [a.ray_begin, a.ray_end); cus = compute units of the device (persistent grid size).
// Quantized nodes when a.qnodes is set, else the f32 coded nodes; the global-memory stack when
// the tree is deeper than the LDS stack or force_global_stack (a parity hook).
hipError_t launch_trace(const TraceArgs& a, int cus, hipStream_t s, bool force_global_stack = false);
// Lanes of the largest persistent trace grid (columns of the global traversal stack).
inline uint64_t trace_max_lanes(int cus) { return (uint64_t)(cus > 0 ? cus : 256) * 2048ull; }
// i64 histogram -> f32 IR (+ mono merge); unit = e0 * 2^-frac_bits.
hipError_t launch_finalize_ir(const long long* hist, float* ir_left, float* ir_right, int32_t ir_len,
                              double unit, int32_t is_mono, hipStream_t s);
// dst[i] += src[i], i < n (int64 histogram bins).
hipError_t launch_hist_add(long long* dst, const long long* src, uint64_t n, hipStream_t s);
hipError_t launch_clear(unsigned long long* hist, uint64_t n, unsigned long long* counters, int n_counters,
                        hipStream_t s);
hipError_t launch_ray_directions(uint64_t seed, uint64_t first, uint64_t count, float* d_out, hipStream_t s);
// Register allocation of the production trace kernel instance (hipFuncGetAttributes numRegs), the
// waves per SIMD it admits, and the waves per SIMD the persistent grid is sized for.
// Register allocation of the LDS-stack trace instance of node format fmt, the large-launch (ray pool)
// or the small-launch one (small), and which of the two launch_trace takes for these arguments.
hipError_t trace_kernel_occupancy(int fmt, bool small, int* vgprs, int* waves_admitted, int* waves_target);
bool trace_uses_small_block(const TraceArgs& a, int cus, bool force_global_stack);
// identity of the trace kernel in this build (build.py trace_source_id; arx_trace_kernel_id)
uint64_t trace_kernel_source_id();

// ---- moving listener (arx_receiver.hip): transform + fixed-topology refit of the receiver ----
struct RefitArgs {
    const TriRec* local_tris;   // receiver triangles in leaf order, local frame (ids, absorption set)
    int32_t n_tris;
    int32_t tri_base;           // global TriRec index of the first receiver triangle
    const BvhNode* local_nodes; // receiver sub-tree (relocated: global refs), boxes unused
    int32_t n_nodes;
    int32_t node_base;          // global node index of local node 0
    const int32_t* level_nodes; // local node indices, deepest level first
    const int32_t* level_start; // [n_levels + 1] offsets into level_nodes
    int32_t n_levels;
    int32_t root_ref, root_count;  // the receiver root as a child reference (global)
    float m[9];                 // rotation, row-major in place_vertices' order (r00 r10 r20, r01 r11 r21, r02 r12 r22)
    float t[3];                 // listener position
    float pad;                  // box padding (>= the builder's 1e-5 * max|coordinate|)
    QGrid grid;
    TriRec* tris;               // outputs
    BvhNode* cnodes;
    QNode2* qnodes;             // null: the quantized copy is not maintained (receiver off the grid)
    unsigned int* flag;         // raised to flag_value if a box fell off the grid (never, given the host's bound)
    unsigned int flag_value;    // the tree write's generation (arx_renderer::tree_gen)
    // CW4 copy (null wbuf: not maintained): the receiver's CW4 nodes (11 ints each: the BVH2
    // (ref, count) of the 4 slots, meta, base, self unit), its leaf triangles ((unit, local index)
    // pairs) and the top node (unit 0: child 0 = the scene root, unit 2; child 1 = the receiver
    // root, unit 4)
    uint4* wbuf;
    const int32_t* w4_nodes;
    int32_t n_w4;
    const int32_t* w4_tris;
    int32_t n_w4_tris;
    float scene_lo[3], scene_hi[3];
    int32_t scene_nonempty;
};
size_t receiver_refit_lds(int32_t n_tris, int32_t n_nodes, int32_t n_levels);  // bytes of LDS
hipError_t launch_receiver_refit(const RefitArgs& a, hipStream_t s);
// The quantized copy of nodes [0, n) re-made on the device from the coded f32 nodes for grid g
// (quantize_nodes16's arithmetic, bit for bit): a new scene or a grown grid costs one launch and
// no host work or upload.  *flag is raised to flag_value (atomic max) if a box falls off the grid.
hipError_t launch_requant16(const BvhNode* coded, uint64_t n, const QGrid& g, QNode2* out, unsigned int* flag,
                            unsigned int flag_value, hipStream_t s);
// The CW4 nodes of n f32 node records (W4NodeF: top node, scene, host-built receiver) quantized for
// grid g into the CW4 buffer at their own units (quantize_w4, arx_wide.hpp).
hipError_t launch_requant_w4(const W4NodeF* nodes, uint64_t n, const QGrid& g, uint4* wbuf, unsigned int* flag,
                             unsigned int flag_value, hipStream_t s);

// ---- convolution (arx_conv.hip) ----
struct ConvPlan;  // opaque, defined in arx_conv.hip
ConvPlan* conv_plan_create(int32_t ir_len, int32_t sample_rate, int device, char* err, size_t errlen);
void conv_plan_destroy(ConvPlan* p);
// Spectra of the two IRs (device f32, ir_len each), kept for the following conv_run calls.
hipError_t conv_set_ir(ConvPlan* p, const float* d_ir_left, const float* d_ir_right, hipStream_t s);
// Device-resident file-mode convolution (kernels.cu:382-438 + AudioRenderer.cpp:706-711).  With
// d_ir_left / d_ir_right the IR spectra are recomputed from them first (on the direct path inside
// the audio's own column pass); with NULLs the spectra of the last conv_set_ir are used.
hipError_t conv_run(ConvPlan* p, const float* d_in, int64_t n_frames, float* d_out_left, float* d_out_right,
                    const float* d_ir_left, const float* d_ir_right, hipStream_t s);
// A time-block shard of conv_run: the one-second block pairs [pair_begin, pair_end) of the file
// (clamped), writing the output frames those pairs own (arx_group_conv_shard) -- bit-identical to the
// same frames of conv_run.  Plans without the chained pass C (conv_plan_shards false) convolve and
// write the whole file.
hipError_t conv_run_pairs(ConvPlan* p, const float* d_in, int64_t n_frames, float* d_out_left, float* d_out_right,
                          const float* d_ir_left, const float* d_ir_right, int64_t pair_begin, int64_t pair_end,
                          hipStream_t s);
bool conv_plan_shards(const ConvPlan* p);
const char* conv_plan_describe(const ConvPlan* p);
// Input reuse: conv_prepare_input transforms a file's blocks once (kept in the plan until the next
// conv_run or conv_prepare_input); conv_run_prepared convolves them with the current IR (new spectra
// from d_ir_left / d_ir_right when given), bit-identical to conv_run on the same input.
hipError_t conv_prepare_input(ConvPlan* p, const float* d_in, int64_t n_frames, hipStream_t s);
hipError_t conv_run_prepared(ConvPlan* p, float* d_out_left, float* d_out_right, const float* d_ir_left,
                             const float* d_ir_right, hipStream_t s);
bool conv_has_prepared(const ConvPlan* p);
int64_t conv_prepared_frames(const ConvPlan* p);
// Live (mic) block: plans created with sample_rate = block length.  One block of n_in <= block
// f64 samples, circular length-ir_len convolution with both IR spectra, / (ir_len/2), zipped
// L/R into 2*ir_len doubles (AudioRenderer.cpp:593-651, kernels.cu:345-377, 450-487).
hipError_t conv_run_live(ConvPlan* p, const double* d_in, int64_t n_in, double* d_out_interleaved, hipStream_t s);
int32_t conv_plan_block(const ConvPlan* p);
// identity of the convolution kernels in this build (build.py conv_source_id; arx_conv_kernel_id)
uint64_t conv_kernel_source_id();

// ---- streaming convolution (arx_conv.hip): uniformly partitioned overlap-save, f64 ----
struct StreamPlan;  // opaque
// block: frames per callback (<= 4096); FFT size = the power of two >= 2*block.
StreamPlan* stream_plan_create(int32_t ir_len, int32_t block, int device, char* err, size_t errlen);
void stream_plan_destroy(StreamPlan* p);
hipError_t stream_reset(StreamPlan* p, hipStream_t s);                      // zero history + delay line
hipError_t stream_set_ir(StreamPlan* p, const float* d_ir_left, const float* d_ir_right, hipStream_t s);
// One block (n_in <= block f64 frames, zero padded) -> 2*block zipped L/R doubles.
hipError_t stream_run(StreamPlan* p, const double* d_in, int64_t n_in, double* d_out_interleaved, hipStream_t s);
int32_t stream_plan_block(const StreamPlan* p);
int32_t stream_plan_partitions(const StreamPlan* p);
int32_t stream_plan_fft(const StreamPlan* p);

}  // namespace arx
