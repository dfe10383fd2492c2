// td_microbench -- vector-memory return-path cost of divergent 16-B gathers on gfx950
// (design tool for the trace kernel; not part of libarx.so).
//
//   hipcc --offload-arch=gfx950 -O3 tools/td_microbench.hip -o /tmp/td_microbench && /tmp/td_microbench
//
// Every lane issues ITERS independent global_load_dwordx4 from a table of 16 KB ... 64 MB (L1,
// L2, Infinity Cache resident), with addresses drawn so that one wave-instruction touches a
// chosen number of distinct 64-B blocks, with a chosen fraction of active lanes.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

constexpr int ITERS = 256;

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

// mode 0: every lane its own random 64-B block (64 blocks / instruction)
// mode 1: quads share a block, lane j of the quad reads 16-B chunk j (16 blocks / instruction)
// mode 2: the whole wave reads one block (1 block / instruction)
// mode 3: every lane its own block but only `active` lanes participate
// mode 4: pairs share a block, lane reads chunk (lane&1)*2 (32 blocks / instruction)
__global__ void gather(const float4* __restrict__ table, uint32_t n_blocks, int mode, int active, float* out) {
    const int lane = threadIdx.x & 63;
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    float4 acc = make_float4(0, 0, 0, 0);
    if (mode == 3 && lane >= active) return;
    for (int it = 0; it < ITERS; ++it) {
        uint32_t key;
        int chunk;
        if (mode == 0 || mode == 3) {
            key = mix(wave * 7919u + it * 131u + lane * 1000003u);
            chunk = 0;
        } else if (mode == 1) {
            key = mix(wave * 7919u + it * 131u + (lane >> 2) * 1000003u);
            chunk = lane & 3;
        } else if (mode == 4) {
            key = mix(wave * 7919u + it * 131u + (lane >> 1) * 1000003u);
            chunk = (lane & 1) * 2;
        } else {
            key = mix(wave * 7919u + it * 131u);
            chunk = lane & 3;
        }
        const float4 v = table[(size_t)(key % n_blocks) * 4 + chunk];
        acc.x += v.x;
        acc.y += v.y;
        acc.z += v.z;
        acc.w += v.w;
    }
    if (acc.x + acc.y + acc.z + acc.w == 12345.0f) out[0] = acc.x;  // keep the loads alive
}

int main() {
    {  // device limits the trace kernel's launch geometry depends on
        int v[4] = {0, 0, 0, 0};
        hipDeviceGetAttribute(&v[0], hipDeviceAttributeMaxSharedMemoryPerBlock, 0);
        hipDeviceGetAttribute(&v[1], hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, 0);
        hipDeviceGetAttribute(&v[2], hipDeviceAttributeSharedMemPerBlockOptin, 0);
        hipDeviceGetAttribute(&v[3], hipDeviceAttributeClockRate, 0);
        std::printf("lds per block %d, per CU %d, opt-in per block %d, clock %d kHz\n", v[0], v[1], v[2], v[3]);
    }
    int cus = 256;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int waves_per_cu = 20, block = 128;
    const int grid = cus * waves_per_cu * 64 / block;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    float* out;
    hipMalloc(&out, 4);
    struct Case {
        const char* name;
        int mode, active;
    } cases[] = {{"64 distinct blocks/instr, 64 lanes", 0, 64},
                 {"32 blocks (pairs, 2 chunks)", 4, 64},
                 {"16 blocks (quads, 4 chunks)", 1, 64},
                 {"1 block (whole wave)", 2, 64},
                 {"distinct blocks, 32 lanes active", 3, 32},
                 {"distinct blocks, 16 lanes active", 3, 16},
                 {"distinct blocks, 8 lanes active", 3, 8}};
    // table sizes: L1-resident, one XCD's L2 (4 MB) and below, Infinity Cache, beyond
    const size_t sizes_kb[] = {16, 256, 2048, 16384, 65536};
    for (size_t kb : sizes_kb) {
        const size_t bytes = kb << 10;
        const uint32_t n_blocks = (uint32_t)(bytes / 64);
        float4* table;
        hipMalloc(&table, bytes);
        hipMemset(table, 0, bytes);
        std::printf("-- table %zu KB\n", kb);
        for (const Case& c : cases) {
            if (kb != 16384 && c.mode != 0 && c.mode != 2) continue;  // the sharing sweep at 16 MB only
            hipLaunchKernelGGL(gather, dim3(grid), dim3(block), 0, 0, table, n_blocks, c.mode, c.active, out);
            hipEventRecord(e0);
            const int reps = 5;
            for (int r = 0; r < reps; ++r)
                hipLaunchKernelGGL(gather, dim3(grid), dim3(block), 0, 0, table, n_blocks, c.mode, c.active, out);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            ms /= reps;
            const double instr_per_cu = (double)waves_per_cu * ITERS;
            const double cyc = ms * 1e-3 * 2.1e9;  // ~effective clock under load
            const double lane_loads = (double)grid * block * ITERS * ((c.mode == 3) ? (double)c.active / 64.0 : 1.0);
            std::printf("%-40s %.3f ms  %.1f cycles per wave-instruction per CU  %.4g 16-B lane loads/s\n", c.name, ms,
                        cyc / instr_per_cu, lane_loads / (ms * 1e-3));
        }
        hipFree(table);
    }
    return 0;
}
