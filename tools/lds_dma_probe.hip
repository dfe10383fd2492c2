// lds_dma_probe -- where does buffer_load_dwordx4 ... lds put each lane's 16 bytes on gfx950?
// (design check for the cooperative node fetch in arx_trace.hip; not part of libarx.so)
//   hipcc --offload-arch=gfx950 -O3 tools/lds_dma_probe.hip -o tools/lds_dma_probe.bin
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef __attribute__((address_space(3))) void* lds_ptr_t;

// mode 0: lane L loads 16 B at byte offset L*16 of `src`; dump the wave's 1 KB of LDS.
// mode 1: the quad-cooperative pattern of coop_fetch_lds (node = lane, chunk = lane & 3).
__global__ void probe(const int* src, int* out, int mode) {
    __shared__ __attribute__((aligned(16))) int stage[1024];
    const int lane = threadIdx.x;
    for (int i = lane; i < 1024; i += 64) stage[i] = -1;
    __syncthreads();
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, 0x7fffffff, 0x00020000);
    if (mode == 0) {
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)stage, 16, lane * 16, 0, 0, 0);
    } else {
        const int node = lane;
        const int c = (lane & 3) * 16;
        const int s0 = __builtin_amdgcn_mov_dpp(node, 0x00, 0xF, 0xF, false);
        const int s1 = __builtin_amdgcn_mov_dpp(node, 0x55, 0xF, 0xF, false);
        const int s2 = __builtin_amdgcn_mov_dpp(node, 0xAA, 0xF, 0xF, false);
        const int s3 = __builtin_amdgcn_mov_dpp(node, 0xFF, 0xF, 0xF, false);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)(stage), 16, s0 * 64 + c, 0, 0, 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)(stage + 256), 16, s1 * 64 + c, 0, 0, 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)(stage + 512), 16, s2 * 64 + c, 0, 0, 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)(stage + 768), 16, s3 * 64 + c, 0, 0, 0);
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    for (int i = lane; i < 1024; i += 64) out[i] = stage[i];
}

int main() {
    std::vector<int> h(64 * 16);
    for (int i = 0; i < 64 * 16; ++i) h[i] = i;  // dword i of the table (node n = i / 16)
    int *src, *out;
    hipMalloc(&src, h.size() * 4);
    hipMalloc(&out, 1024 * 4);
    hipMemcpy(src, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    std::vector<int> o(1024);
    for (int mode = 0; mode < 2; ++mode) {
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, src, out, mode);
        hipMemcpy(o.data(), out, 1024 * 4, hipMemcpyDeviceToHost);
        std::printf("mode %d: first 24 dwords:", mode);
        for (int i = 0; i < 24; ++i) std::printf(" %d", o[i]);
        std::printf("\n  dwords 256..271:");
        for (int i = 256; i < 272; ++i) std::printf(" %d", o[i]);
        int bad = 0;
        for (int i = 0; i < 1024; ++i) {
            int want;
            if (mode == 0) want = i < 256 ? i : -1;
            else { const int k = i / 256, q = (i % 256) / 16, d = i % 16; want = (4 * q + k) * 16 + d; }
            bad += o[i] != want;
        }
        std::printf("\n  mismatches vs assumed layout: %d\n", bad);
    }
    return 0;
}
