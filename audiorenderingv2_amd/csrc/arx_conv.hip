// arx_conv.hip -- file-mode FFT convolution for gfx950.
//
// Semantics restated from R/prebuild/obj_raytracer/kernels.cu:382-438
// (convoluteFromAudioBuffer) + AudioRenderer.cpp:706-711: the input is cut into
// S = floor(len/sr) one-second blocks (the tail len mod sr is never processed), each
// block is zero padded to n = ir_len and CIRCULARLY convolved (length n) with the IR,
// the unnormalised results (n * circconv) are overlap-added at 1-s hops clipped to len,
// and the sum is divided by (ir_len/2) (integer division).
//
// MI355X design: instead of 4 launches + 2 cuFFT calls + 3 device syncs per block, all
// blocks of both channels are convolved by four batched launches:
//   A  fwd column FFTs (length N1, in LDS) of the block PAIRS packed as re/im
//      (x = block_2p + i*block_2p+1: one complex FFT serves two real blocks, and the
//      inverse of (X * H) returns both results in re/im because h is real), times the
//      four-step twiddle W_M^(n2*k1);
//   B  per row: fwd row FFT (N2), * H_c, inverse row FFT, * W_M^(-n2*k1) -- for both
//      channels from one forward pass (spectrum kept in registers);
//   C  inverse column FFTs -> M * linear convolution of each block, to a f64 scratch;
//   D  overlap-add gather with the circular fold cc[i] = lin[i] + lin[i+n], scaled
//      n/(M*(n/2)), rounded once to f32 (deterministic, no atomics).
// FFT length: when n = N1 x N2 with both factors 7-smooth and <= 512 (every 2-s IR at the usual
// rates: 96000 = 300 x 320 at 48 kHz), M = n itself -- the reference's own circular length -- with
// mixed-radix (8/4/2/3/5/7) sub-FFTs and no fold ("direct" path, pass_*_mr).  Otherwise M is the
// power of two >= n + sr - 1 (linear convolution, folded back to length n in pass D), so every
// (ir_len, sr) pair works with radix-8/4/2 stages.  At C3 the direct path moves 2.7x fewer
// FFT points per block pair than 2^18.
// All FFT arithmetic is f64: the result matches the f64 oracle to ~1e-15 relative
// before the single f32 rounding (the "1 ULP of max|y|" bar of SURVEY.md §8c).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <vector>

#include "arx_kernels.hpp"

namespace arx {

constexpr int kMaxRadices = 12;
constexpr int kMaxSubLen = 512;  // N1, N2 <= 512: n <= 2^18 (longer IRs take the power-of-two path)

struct Factors {
    int32_t L;
    int32_t count;
    int32_t r[kMaxRadices];
};

struct ConvPlan {
    bool direct = false;  // mixed-radix FFTs of length n (no fold); else the power-of-two path
    bool r7 = false;      // direct: radix-7 stages present (selects the kernels that carry them)
    Factors f1{}, f2{};   // direct: the radices of N1 and N2
    int32_t n = 0;      // ir_len (circular length of the reference)
    int32_t sr = 0;     // hop (block length)
    int32_t M = 0;      // FFT length (power of two >= n + sr - 1, or n on the direct path)
    int32_t N1 = 0, N2 = 0, lg1 = 0, lg2 = 0;
    int32_t tc = 1;     // columns per workgroup in passes A / C
    int device = 0;
    double2* d_tw = nullptr;     // W_M^e, e in [0, M)
    double2* d_H = nullptr;      // 2 * M, transposed layout [k1][k2]
    double2* d_G = nullptr;      // direct: M, the packed IR h_L + i h_R after pass A's columns
    double2* d_S = nullptr;      // scratch spectra: pairs_cap * 3 * M (shared + 2 channels)
    double* d_Y = nullptr;       // per block, per channel M*lin (length n + sr - 1)
    int64_t pairs_cap = 0;
    // input reuse (conv_prepare_input): the prepared file's length, and where its spectra live --
    // S[pair][0] on the direct path with the chained pass C, else a copy of the input (d_prep_in)
    // that conv_run_prepared convolves in full
    bool prepared = false;
    bool prep_spectra = false;
    int64_t prep_frames = 0;
    float* d_prep_in = nullptr;
    size_t prep_cap = 0;
    char desc[160] = {0};
};

namespace {

constexpr int kThreads = 256;

__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
    return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ double2 cadd(double2 a, double2 b) { return make_double2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ double2 csub(double2 a, double2 b) { return make_double2(a.x - b.x, a.y - b.y); }
// multiply by sign*i
__device__ __forceinline__ double2 mul_si(double2 a, int sign) {
    return sign < 0 ? make_double2(a.y, -a.x) : make_double2(-a.y, a.x);
}
__device__ __forceinline__ double2 twiddle(const double2* __restrict__ tw, int32_t M, int64_t e, int sign) {
    const double2 w = tw[e & (M - 1)];
    return sign < 0 ? w : make_double2(w.x, -w.y);
}

// Twiddle sources for lds_fft: W_M^e from one table of M entries, or (TwSplit) the product of two
// small LDS tables hi[e >> lgLo] = W_M^(e & ~(2^lgLo - 1)) and lo[e & (2^lgLo - 1)] = W_M^(e mod 2^lgLo),
// for transforms whose full table would not fit in LDS beside the data.
struct TwFlat {
    const double2* tw;
    int32_t M;
    __device__ double2 operator()(int64_t e, int sign) const { return twiddle(tw, M, e, sign); }
};
struct TwSplit {
    const double2* hi;
    const double2* lo;
    int32_t lgLo, M;
    __device__ double2 operator()(int64_t e, int sign) const {
        const int64_t m = e & (M - 1);
        const double2 w = cmul(hi[m >> lgLo], lo[m & ((1 << lgLo) - 1)]);
        return sign < 0 ? w : make_double2(w.x, -w.y);
    }
};

// In-place Stockham FFT of length L = 2^lg on buf[0..L) (LDS), executed by the nt
// threads t in [0, nt) of this group; every thread of the workgroup must call it (it
// contains __syncthreads()).  Twiddle W_L^e = tw[e * (M/L)].
__device__ void lds_fft(double2* buf, int L, int lg, int sign, int t, int nt, const double2* __restrict__ tw,
                        int32_t M);
template <class TW>
__device__ void lds_fft_t(double2* buf, int L, int lg, int sign, int t, int nt, const TW& twf, int32_t M) {
    const int mstep = M >> lg;  // M / L
    int Ns = 1;
    int stages4 = lg >> 1;
    for (int s = 0; s < stages4; ++s) {
        const int quarter = L >> 2;
        double2 v[4][4];
        int jj[4];
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const int j = t + b * nt;
            jj[b] = j;
            if (j < quarter) {
                const int k = j & (Ns - 1);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    double2 x = buf[j + r * quarter];
                    if (r > 0) x = cmul(x, twf((int64_t)r * k * (L / (Ns * 4)) * mstep, sign));
                    v[b][r] = x;
                }
            }
        }
        __syncthreads();
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const int j = jj[b];
            if (j < quarter) {
                const int k = j & (Ns - 1);
                const double2 a0 = cadd(v[b][0], v[b][2]);
                const double2 a1 = csub(v[b][0], v[b][2]);
                const double2 a2 = cadd(v[b][1], v[b][3]);
                const double2 a3 = mul_si(csub(v[b][1], v[b][3]), sign);
                const int d = (j - k) * 4 + k;  // (j/Ns)*Ns*4 + j%Ns
                buf[d] = cadd(a0, a2);
                buf[d + Ns] = cadd(a1, a3);
                buf[d + 2 * Ns] = csub(a0, a2);
                buf[d + 3 * Ns] = csub(a1, a3);
            }
        }
        __syncthreads();
        Ns <<= 2;
    }
    if (lg & 1) {  // final radix-2 stage
        const int half = L >> 1;
        double2 v[8][2];
        int jj[8];
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const int j = t + b * nt;
            jj[b] = j;
            if (j < half) {
                const int k = j & (Ns - 1);
                v[b][0] = buf[j];
                v[b][1] = cmul(buf[j + half], twf((int64_t)k * (L / (Ns * 2)) * mstep, sign));
            }
        }
        __syncthreads();
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const int j = jj[b];
            if (j < half) {
                const int k = j & (Ns - 1);
                const int d = (j - k) * 2 + k;
                buf[d] = cadd(v[b][0], v[b][1]);
                buf[d + Ns] = csub(v[b][0], v[b][1]);
            }
        }
        __syncthreads();
    }
}

__device__ void lds_fft(double2* buf, int L, int lg, int sign, int t, int nt, const double2* __restrict__ tw,
                        int32_t M) {
    lds_fft_t(buf, L, lg, sign, t, nt, TwFlat{tw, M}, M);
}

// ---- 512-point FFTs (the 48 kHz plans): one wave per row / column, radix-8 in registers ----
// Stockham radix-8 over 3 stages: each lane holds 8 elements (j + 64 r), so the row is loaded
// and stored coalesced, the first stage starts from registers, the last one ends in them
// (natural order), and only 2 LDS exchanges per FFT remain -- versus 5 stages x 2 block
// barriers with half the threads idle in the generic radix-4 path.  A wave's LDS operations
// execute in order, so the exchanges inside one wave need no block barrier.
__device__ __forceinline__ double2 mul_w8(double2 a, int sign) {  // * e^(sign i pi/4)
    const double c = 0.70710678118654752440;
    return sign < 0 ? make_double2(c * (a.x + a.y), c * (a.y - a.x)) : make_double2(c * (a.x - a.y), c * (a.x + a.y));
}
__device__ __forceinline__ double2 mul_w83(double2 a, int sign) {  // * e^(sign 3 i pi/4)
    const double c = 0.70710678118654752440;
    return sign < 0 ? make_double2(c * (a.y - a.x), -c * (a.x + a.y)) : make_double2(-c * (a.x + a.y), c * (a.x - a.y));
}
// in-place 8-point DFT, y[q] = sum_r x[r] e^(sign 2 pi i r q / 8)
__device__ __forceinline__ void dft8(double2* x, int sign) {
    double2 a[4], b[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        a[r] = cadd(x[r], x[r + 4]);
        b[r] = csub(x[r], x[r + 4]);
    }
    b[1] = mul_w8(b[1], sign);
    b[2] = mul_si(b[2], sign);
    b[3] = mul_w83(b[3], sign);
    // 4-point DFTs of a (even outputs) and b (odd outputs)
    const double2 a0 = cadd(a[0], a[2]), a1 = csub(a[0], a[2]), a2 = cadd(a[1], a[3]), a3 = mul_si(csub(a[1], a[3]), sign);
    const double2 b0 = cadd(b[0], b[2]), b1 = csub(b[0], b[2]), b2 = cadd(b[1], b[3]), b3 = mul_si(csub(b[1], b[3]), sign);
    x[0] = cadd(a0, a2);
    x[4] = csub(a0, a2);
    x[2] = cadd(a1, a3);
    x[6] = csub(a1, a3);
    x[1] = cadd(b0, b2);
    x[5] = csub(b0, b2);
    x[3] = cadd(b1, b3);
    x[7] = csub(b1, b3);
}
// 512-point FFT of the row held as x[r] = element j + 64 r (lane j of the wave); result in the
// same layout.  buf: the wave's 512-element LDS scratch; twl: W_512^e in LDS.
__device__ __forceinline__ void fft512_wave(double2* x, double2* buf, const double2* twl, int j, int sign) {
    dft8(x, sign);  // stage 1 (Ns = 1): no twiddles
#pragma unroll
    for (int q = 0; q < 8; ++q) buf[8 * j + q] = x[q];
    __builtin_amdgcn_wave_barrier();
    {  // stage 2 (Ns = 8)
        const int k = j & 7;
#pragma unroll
        for (int r = 0; r < 8; ++r) x[r] = buf[j + 64 * r];
#pragma unroll
        for (int r = 1; r < 8; ++r) x[r] = cmul(x[r], twiddle(twl, 512, 8 * r * k, sign));
        dft8(x, sign);
        const int d = (j - k) * 8 + k;
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int q = 0; q < 8; ++q) buf[d + 8 * q] = x[q];
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int r = 0; r < 8; ++r) x[r] = buf[j + 64 * r];  // stage 3 (Ns = 64): k = j
#pragma unroll
    for (int r = 1; r < 8; ++r) x[r] = cmul(x[r], twiddle(twl, 512, r * j, sign));
    dft8(x, sign);
    __builtin_amdgcn_wave_barrier();
}

// ---- 256-point FFTs (the 16 kHz plans, M = 2^16 = 256 x 256): one wave per row / column,
// four radix-4 Stockham stages, each lane one butterfly per stage on elements j + 64 r (the
// lane's registers), so the first stage starts from registers, the last one ends in them in
// natural order, and 3 in-wave LDS exchanges remain.
__device__ __forceinline__ void dft4(double2* x, int sign) {
    const double2 a0 = cadd(x[0], x[2]), a1 = csub(x[0], x[2]), a2 = cadd(x[1], x[3]), a3 = mul_si(csub(x[1], x[3]), sign);
    x[0] = cadd(a0, a2);
    x[1] = cadd(a1, a3);
    x[2] = csub(a0, a2);
    x[3] = csub(a1, a3);
}
__device__ __forceinline__ void fft256_wave(double2* x, double2* buf, const double2* twl, int j, int sign) {
    dft4(x, sign);  // Ns = 1: no twiddles
#pragma unroll
    for (int q = 0; q < 4; ++q) buf[4 * j + q] = x[q];
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int Ns = 4; Ns <= 16; Ns *= 4) {
        const int k = j & (Ns - 1);
#pragma unroll
        for (int r = 0; r < 4; ++r) x[r] = buf[j + 64 * r];
#pragma unroll
        for (int r = 1; r < 4; ++r) x[r] = cmul(x[r], twiddle(twl, 256, (64 / Ns) * r * k, sign));
        dft4(x, sign);
        const int d = (j - k) * 4 + k;
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int q = 0; q < 4; ++q) buf[d + Ns * q] = x[q];
        __builtin_amdgcn_wave_barrier();
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) x[r] = buf[j + 64 * r];  // Ns = 64: k = j
#pragma unroll
    for (int r = 1; r < 4; ++r) x[r] = cmul(x[r], twiddle(twl, 256, r * j, sign));
    dft4(x, sign);
    __builtin_amdgcn_wave_barrier();
}

// L-point wave FFT of x[r] = element j + 64 r (L = 256 or 512)
template <int L>
__device__ __forceinline__ void fft_wave(double2* x, double2* buf, const double2* twl, int j, int sign) {
    if constexpr (L == 512)
        fft512_wave(x, buf, twl, j, sign);
    else
        fft256_wave(x, buf, twl, j, sign);
}

// Column FFTs of the tile in LDS (tc columns of L, then the twiddle table) by the block's
// 4 waves, tc / 4 columns each.
template <int L>
__device__ __forceinline__ void columns_wave(double2* lds, const double2* twl, int tc, int sign) {
    constexpr int R = L / 64;
    const int w = threadIdx.x >> 6, j = threadIdx.x & 63;
    const int per_wave = tc / 4;
    for (int cc = 0; cc < per_wave; ++cc) {
        double2* cl = lds + (size_t)(per_wave * w + cc) * L;
        double2 x[R];
#pragma unroll
        for (int r = 0; r < R; ++r) x[r] = cl[j + 64 * r];
        fft_wave<L>(x, cl, twl, j, sign);
#pragma unroll
        for (int r = 0; r < R; ++r) cl[j + 64 * r] = x[r];
    }
    __syncthreads();
}

struct PassArgs {
    const double2* tw;
    int32_t M, N1, N2, lg1, lg2, tc;
    int32_t n, sr;
    int64_t n_blocks;   // S
    int64_t n_pairs;
    const float* in;    // audio input (mode 0) or IR pair base (mode 1)
    const float* ir_l;
    const float* ir_r;
    double2* S;         // [pair][3][M]: 0 = forward (shared), 1/2 = per channel
    double2* H;         // [2][M]
    double2* G;         // [M]: pass_a_mr mode 0's packed IR batch
    double* Y;          // [block][2][ylen]
    int64_t ylen;       // n + sr - 1
    float* out_l;
    float* out_r;
    int64_t len;
    double scale;
    const double* in_d;  // live block input (f64)
    int64_t n_in;        // live block length (<= block length of the plan)
    double* out_d;       // live output, interleaved L/R, 2*n doubles
    // chained pass C of a time-block shard (conv_run_pairs): the first local pair whose output
    // segments are written (1 when local pair 0 is the seam pair, re-transformed only for its
    // second block's tail), and whether the segment after the last pair is this shard's (the file's
    // last shard)
    int32_t emit_from;
    int32_t tail;
};

// Pass A: forward column FFTs.  mode 0: batch = block pair p; mode 1: batch = IR channel c.
template <int MODE>
__global__ __launch_bounds__(kThreads) void pass_a(PassArgs a) {
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    const int tc = a.tc;
    const int per = kThreads / tc;
    const int col = threadIdx.x / per;  // local column
    const int t = threadIdx.x % per;
    const int64_t batch = blockIdx.y;
    const int n2_0 = blockIdx.x * tc;
    const int n2 = n2_0 + col;
    double2* buf = lds + (size_t)col * a.N1;
    // the N1 twiddles W_N1^e, staged once in LDS after the columns (a global load per
    // butterfly put an L2 round trip into every FFT stage)
    double2* twl = lds + (size_t)tc * a.N1;
    for (int i = threadIdx.x; i < a.N1; i += kThreads) twl[i] = a.tw[(size_t)i * (a.M / a.N1)];
    // load column n2: element n1 at x[N2*n1 + n2]
    for (int i = threadIdx.x; i < tc * a.N1; i += kThreads) {
        const int c = i % tc, n1 = i / tc;  // consecutive threads -> consecutive columns
        const int64_t idx = (int64_t)a.N2 * n1 + n2_0 + c;
        double2 x = make_double2(0.0, 0.0);
        if (MODE == 0) {
            if (idx < a.sr) {
                const int64_t b0 = 2 * batch, b1 = 2 * batch + 1;
                if (b0 < a.n_blocks) x.x = (double)a.in[b0 * a.sr + idx];
                if (b1 < a.n_blocks) x.y = (double)a.in[b1 * a.sr + idx];
            }
        } else if (MODE == 2) {  // live block (f64 samples), zero padded
            if (idx < a.n_in) x.x = a.in_d[idx];
        } else {
            if (idx < a.n) x.x = (double)(batch == 0 ? a.ir_l : a.ir_r)[idx];
        }
        lds[(size_t)c * a.N1 + n1] = x;
    }
    __syncthreads();
    if (a.N1 == 512 && tc == 8) {  // 4 waves x 2 columns, radix-8 in registers (fft512_wave)
        columns_wave<512>(lds, twl, tc, -1);
    } else if (a.N1 == 256 && tc == 16) {  // 4 waves x 4 columns, radix-4 in registers
        columns_wave<256>(lds, twl, tc, -1);
    } else {
        lds_fft(buf, a.N1, a.lg1, -1, t, per, twl, a.N1);
    }
    // twiddle W_M^(n2*k1) and store transposed: S[k1*N2 + n2]
    double2* dst = (MODE != 1) ? a.S + (size_t)batch * 3 * a.M : a.H + (size_t)batch * a.M;
    for (int i = threadIdx.x; i < tc * a.N1; i += kThreads) {
        const int c = i % tc, k1 = i / tc;
        const int64_t e = (int64_t)(n2_0 + c) * k1;
        const double2 x = cmul(lds[(size_t)c * a.N1 + k1], twiddle(a.tw, a.M, e, -1));
        dst[(int64_t)k1 * a.N2 + n2_0 + c] = x;
    }
}

// Pass B.  mode 0: row FFT, * H_c, inverse row FFT, * W_M^(-n2*k1) for c = 0, 1.
//          mode 1: row FFT only (IR spectrum, in place in H).
template <int MODE>
__global__ __launch_bounds__(kThreads) void pass_b(PassArgs a) {
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    const int k1 = blockIdx.x;
    const int64_t batch = blockIdx.y;
    const int N2 = a.N2;
    constexpr bool kMul = MODE == 0 || MODE == 4;  // multiply by H and invert
    double2* row = (MODE == 1) ? a.H + (size_t)batch * a.M + (int64_t)k1 * N2 : a.S + (size_t)batch * 3 * a.M + (int64_t)k1 * N2;
    double2* twl = lds + N2;  // W_N2^e staged in LDS (see pass A)
    for (int i = threadIdx.x; i < N2; i += kThreads) {
        lds[i] = row[i];
        twl[i] = a.tw[(size_t)i * (a.M / N2)];
    }
    __syncthreads();
    lds_fft(lds, N2, a.lg2, -1, threadIdx.x, kThreads, twl, N2);
    if (MODE == 1) {
        for (int i = threadIdx.x; i < N2; i += kThreads) row[i] = lds[i];
        return;
    }
    constexpr int kMaxPer = 16;  // N2 <= 4096
    double2 keep[kMaxPer];
#pragma unroll
    for (int b = 0; b < kMaxPer; ++b) {
        const int i = threadIdx.x + b * kThreads;
        if (i < N2) keep[b] = lds[i];
    }
    for (int c = 0; c < 2; ++c) {
        const double2* Hc = a.H + (size_t)c * a.M + (int64_t)k1 * N2;
#pragma unroll
        for (int b = 0; b < kMaxPer; ++b) {
            const int i = threadIdx.x + b * kThreads;
            if (i < N2) lds[i] = cmul(keep[b], Hc[i]);
        }
        __syncthreads();
        lds_fft(lds, N2, a.lg2, +1, threadIdx.x, kThreads, twl, N2);
        double2* dst = a.S + ((size_t)batch * 3 + 1 + c) * a.M + (int64_t)k1 * N2;
        for (int i = threadIdx.x; i < N2; i += kThreads)
            dst[i] = cmul(lds[i], twiddle(a.tw, a.M, (int64_t)i * k1, +1));
        __syncthreads();
    }
}

template <int MODE, int L>
__global__ __launch_bounds__(kThreads) void pass_bw(PassArgs a) {
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    constexpr int kRows = kThreads / 64;
    constexpr int R = L / 64;
    const int w = threadIdx.x >> 6, j = threadIdx.x & 63;
    const int k1 = blockIdx.x * kRows + w;
    const int64_t batch = blockIdx.y;
    double2* buf = lds + w * L;
    double2* twl = lds + kRows * L;
    for (int i = threadIdx.x; i < L; i += kThreads) twl[i] = a.tw[(size_t)i * (a.M / L)];
    double2* row = (MODE == 0) ? a.S + (size_t)batch * 3 * a.M + (int64_t)k1 * L : a.H + (size_t)batch * a.M + (int64_t)k1 * L;
    double2 x[R];
#pragma unroll
    for (int r = 0; r < R; ++r) x[r] = row[j + 64 * r];
    __syncthreads();  // twiddle table
    fft_wave<L>(x, buf, twl, j, -1);
    if (MODE == 1) {
#pragma unroll
        for (int r = 0; r < R; ++r) row[j + 64 * r] = x[r];
        return;
    }
    double2 keep[R];
#pragma unroll
    for (int r = 0; r < R; ++r) keep[r] = x[r];
    for (int c = 0; c < 2; ++c) {
        const double2* Hc = a.H + (size_t)c * a.M + (int64_t)k1 * L;
#pragma unroll
        for (int r = 0; r < R; ++r) x[r] = cmul(keep[r], Hc[j + 64 * r]);
        fft_wave<L>(x, buf, twl, j, +1);
        double2* dst = a.S + ((size_t)batch * 3 + 1 + c) * a.M + (int64_t)k1 * L;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int i = j + 64 * r;
            dst[i] = cmul(x[r], twiddle(a.tw, a.M, (int64_t)i * k1, +1));
        }
    }
}

// Pass C: inverse column FFTs of each (pair, channel) -> M * linear convolution of the
// two blocks of the pair (re / im), written to Y for indices < n + sr - 1.
__global__ __launch_bounds__(kThreads) void pass_c(PassArgs a) {
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    const int tc = a.tc;
    const int per = kThreads / tc;
    const int col = threadIdx.x / per;
    const int t = threadIdx.x % per;
    const int64_t pair = blockIdx.y >> 1;
    const int ch = blockIdx.y & 1;
    const int n2_0 = blockIdx.x * tc;
    const double2* src = a.S + ((size_t)pair * 3 + 1 + ch) * a.M;
    double2* twl = lds + (size_t)tc * a.N1;  // W_N1^e staged in LDS (see pass A)
    for (int i = threadIdx.x; i < a.N1; i += kThreads) twl[i] = a.tw[(size_t)i * (a.M / a.N1)];
    for (int i = threadIdx.x; i < tc * a.N1; i += kThreads) {
        const int c = i % tc, k1 = i / tc;
        lds[(size_t)c * a.N1 + k1] = src[(int64_t)k1 * a.N2 + n2_0 + c];
    }
    __syncthreads();
    if (a.N1 == 512 && tc == 8) {  // as in pass A
        columns_wave<512>(lds, twl, tc, +1);
    } else if (a.N1 == 256 && tc == 16) {
        columns_wave<256>(lds, twl, tc, +1);
    } else {
        lds_fft(lds + (size_t)col * a.N1, a.N1, a.lg1, +1, t, per, twl, a.N1);
    }
    const int64_t b0 = 2 * pair, b1 = 2 * pair + 1;
    double* y0 = a.Y + (b0 * 2 + ch) * a.ylen;
    double* y1 = a.Y + (b1 * 2 + ch) * a.ylen;
    for (int i = threadIdx.x; i < tc * a.N1; i += kThreads) {
        const int c = i % tc, n1 = i / tc;
        const int64_t idx = (int64_t)a.N2 * n1 + n2_0 + c;
        if (idx < a.ylen) {
            const double2 v = lds[(size_t)c * a.N1 + n1];
            if (b0 < a.n_blocks) y0[idx] = v.x;
            if (b1 < a.n_blocks) y1[idx] = v.y;
        }
    }
}

// Pass D: out_c[j] = scale * sum_s (lin_s[j - s*sr] + lin_s[j - s*sr + n]) over the
// blocks whose window [s*sr, s*sr + n) covers j (kernels.cu:425-428 clip at len).
__global__ __launch_bounds__(kThreads) void pass_d(PassArgs a) {
    const int64_t j = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (j >= a.len) return;
    const int ch = blockIdx.y;
    int64_t s_hi = j / a.sr;
    if (s_hi > a.n_blocks - 1) s_hi = a.n_blocks - 1;
    int64_t s_lo = (j - a.n + 1 <= 0) ? 0 : (j - a.n + 1 + a.sr - 1) / a.sr;
    double acc = 0.0;
    for (int64_t s = s_lo; s <= s_hi; ++s) {
        const int64_t i = j - s * a.sr;
        const double* y = a.Y + (s * 2 + ch) * a.ylen;
        double v = y[i];
        if (i + a.n < a.ylen) v += y[i + a.n];
        acc += v;
    }
    (ch == 0 ? a.out_l : a.out_r)[j] = (float)(acc * a.scale);
}

// Live pass D (convoluteLiveInput, AudioRenderer.cpp:623-644): the single block's circular
// length-n convolution (lin[i] + lin[i+n]) for i in [0, n), scaled n/(M*(n/2)) (Z2D x n then
// normalizeBuffers' /(ir_len/2)) and zipped L/R (d_zipArrays, kernels.cu:469-479), in f64.
__global__ __launch_bounds__(kThreads) void pass_d_live(PassArgs a) {
    const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (i >= a.n) return;
#pragma unroll
    for (int ch = 0; ch < 2; ++ch) {
        const double* y = a.Y + ch * a.ylen;
        double v = y[i];
        if (i + a.n < a.ylen) v += y[i + a.n];
        a.out_d[2 * i + ch] = v * a.scale;
    }
}

// ==================================================================================================
// Mixed-radix direct path: when ir_len n = N1 x N2 with both factors 7-smooth and <= 1024 (every
// 2 s IR at 16 / 32 / 44.1 / 48 / 96 kHz), the block circular convolution of length n is computed
// with FFTs of length n itself -- the reference's own transform length (cuFFT, kernels.cu:413-437)
// -- instead of the power of two >= n + sr - 1 and the fold: 96000 instead of 2^18 points per
// 48 kHz block pair, no fold terms in pass D.  Same four passes and layouts as above; the sub-FFTs
// are one wave per row / column in LDS, Stockham stages of radix 8, 4, 2, 3, 5, 7.

// y[q] = sum_r x[r] e^(sign 2 pi i r q / R) for odd prime R, with the cos / sin of 2 pi m / R
template <int R>
struct OddDft;
template <>
struct OddDft<3> {
    static constexpr double c[3] = {1.0, -0.5, -0.5};
    static constexpr double s[3] = {0.0, 0.86602540378443864676, -0.86602540378443864676};
};
template <>
struct OddDft<5> {
    static constexpr double c[5] = {1.0, 0.30901699437494742410, -0.80901699437494742410, -0.80901699437494742410,
                                    0.30901699437494742410};
    static constexpr double s[5] = {0.0, 0.95105651629515357212, 0.58778525229247312917, -0.58778525229247312917,
                                    -0.95105651629515357212};
};
template <>
struct OddDft<7> {
    static constexpr double c[7] = {1.0, 0.62348980185873353053, -0.22252093395631440429, -0.90096886790241912624,
                                    -0.90096886790241912624, -0.22252093395631440429, 0.62348980185873353053};
    static constexpr double s[7] = {0.0, 0.78183148246802980871, 0.97492791218182360702, 0.43388373911755812048,
                                    -0.43388373911755812048, -0.97492791218182360702, -0.78183148246802980871};
};

template <int R>
__device__ __forceinline__ void dft_radix(double2* x, int sign) {
    if constexpr (R == 2) {
        const double2 a = x[0], b = x[1];
        x[0] = cadd(a, b);
        x[1] = csub(a, b);
    } else if constexpr (R == 4) {
        dft4(x, sign);
    } else if constexpr (R == 8) {
        dft8(x, sign);
    } else {  // odd prime: pair r with R - r
        constexpr int H = R / 2;
        double2 a[H + 1], b[H + 1];
#pragma unroll
        for (int r = 1; r <= H; ++r) {
            a[r] = cadd(x[r], x[R - r]);
            b[r] = csub(x[r], x[R - r]);
        }
        double2 y0 = x[0];
#pragma unroll
        for (int r = 1; r <= H; ++r) y0 = cadd(y0, a[r]);
        double2 y[R];
#pragma unroll
        for (int q = 1; q <= H; ++q) {
            double2 t = x[0], u = make_double2(0.0, 0.0);
#pragma unroll
            for (int r = 1; r <= H; ++r) {
                const int m = (r * q) % R;
                t.x += OddDft<R>::c[m] * a[r].x;
                t.y += OddDft<R>::c[m] * a[r].y;
                u.x += OddDft<R>::s[m] * b[r].x;
                u.y += OddDft<R>::s[m] * b[r].y;
            }
            const double2 iu = mul_si(u, sign);  // sign * i * u
            y[q] = cadd(t, iu);
            y[R - q] = csub(t, iu);
        }
        x[0] = y0;
#pragma unroll
        for (int q = 1; q < R; ++q) x[q] = y[q];
    }
}

// LDS slot of element i of a sub-FFT buffer between its first two stages when SW: the elements'
// 8-element blocks XOR-swizzled (block k's slots permuted by k mod 8; a tail short of a whole block
// stays put).  The first stage of an even length stores with stride R in {2, 4, 8}: unswizzled, the 8
// lanes of a ds_write_b128 group land on one or two 128-B bank rows (up to 8-way conflicts); swizzled
// they cover all 8.  The second stage reads through the same map and stores in natural order.
template <bool SW>
__device__ __forceinline__ int lds_ix(int i, int L8) {
    return (SW && i < L8) ? (i ^ ((i >> 3) & 7)) : i;
}

// One Stockham stage of radix R over buf[0..L) (LDS, this wave's row / column), Ns = product of
// the earlier radices; twl = W_L^e.  Every lane first reads all its butterflies, then writes.
// SWI / SWO: the input / output is in the lds_ix swizzled order.
template <int R, int LM, bool SWI, bool SWO>
__device__ __forceinline__ void mr_stage(double2* buf, const double2* twl, int L, int Ns, int j, int sign) {
    constexpr int kMaxB = (LM / R + 63) / 64;  // butterflies per lane for L <= LM
    const int nb = L / R, step = L / (Ns * R), L8 = L & ~7;
    double2 v[kMaxB][R];
#pragma unroll
    for (int i = 0; i < kMaxB; ++i) {
        const int b = j + 64 * i;
        if (b < nb) {
            const int k = b % Ns;
#pragma unroll
            for (int q = 0; q < R; ++q) {
                double2 x = buf[lds_ix<SWI>(b + q * nb, L8)];
                if (q > 0) {
                    const double2 w = twl[q * k * step];
                    x = cmul(x, sign < 0 ? w : make_double2(w.x, -w.y));
                }
                v[i][q] = x;
            }
            dft_radix<R>(v[i], sign);
        }
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int i = 0; i < kMaxB; ++i) {
        const int b = j + 64 * i;
        if (b < nb) {
            const int k = b % Ns;
            const int d = (b - k) * R + k;
#pragma unroll
            for (int q = 0; q < R; ++q) buf[lds_ix<SWO>(d + q * Ns, L8)] = v[i][q];
        }
    }
    __builtin_amdgcn_wave_barrier();
}

template <bool R7, int LM, bool SWI, bool SWO>
__device__ __forceinline__ void mr_stage_r(int r, double2* buf, const double2* twl, int L, int Ns, int j, int sign) {
    switch (r) {
        case 8: mr_stage<8, LM, SWI, SWO>(buf, twl, L, Ns, j, sign); break;
        case 4: mr_stage<4, LM, SWI, SWO>(buf, twl, L, Ns, j, sign); break;
        case 2: mr_stage<2, LM, SWI, SWO>(buf, twl, L, Ns, j, sign); break;
        case 3: mr_stage<3, LM, SWI, SWO>(buf, twl, L, Ns, j, sign); break;
        case 5: mr_stage<5, LM, SWI, SWO>(buf, twl, L, Ns, j, sign); break;
        default:
            if constexpr (R7) mr_stage<7, LM, SWI, SWO>(buf, twl, L, Ns, j, sign);
            break;
    }
}

// In-place FFT of buf[0..f.L) by one wave (lane j), natural order in and out.  R7: the plan has
// radix-7 stages (their 7-point DFT costs ~20 VGPRs in every kernel that may run one).  An even
// length starts with its radix-2^k stages (factor7), so its first stage stores swizzled (lds_ix).
template <bool R7, int LM>
__device__ __forceinline__ void fft_mr_wave(double2* buf, const double2* twl, const Factors& f, int j, int sign) {
    const bool even = (f.L & 1) == 0;
    int Ns = 1;
    for (int s = 0; s < f.count; ++s) {
        if (even && s == 0)
            mr_stage_r<false, LM, false, true>(f.r[s], buf, twl, f.L, Ns, j, sign);
        else if (even && s == 1)
            mr_stage_r<R7, LM, true, false>(f.r[s], buf, twl, f.L, Ns, j, sign);
        else
            mr_stage_r<R7, LM, false, false>(f.r[s], buf, twl, f.L, Ns, j, sign);
        Ns *= f.r[s];
    }
}

// Compile-time plans for the sub-FFT lengths of the usual IRs (300 x 320 at 48 kHz, 160 x 200 at
// 16 kHz, 315 x 280 at 44.1 kHz, 250 x 256 at 32 kHz): the same radix order as factor7, but every
// stage's R, Ns and butterfly count are constants, so the index arithmetic (b mod Ns, twiddle
// exponents, guards) folds away -- it was most of the generic stages' VALU work.
constexpr int ct_radix(int L, int s) {
    int v = L, t = 0;
    while (v % 2 == 0) {
        v /= 2;
        ++t;
    }
    int idx = 0;
    for (; t >= 3; t -= 3, ++idx)
        if (idx == s) return 8;
    if (t == 2 && idx++ == s) return 4;
    if (t == 1 && idx++ == s) return 2;
    for (int q = 3; q <= 7; q += 2)
        while (v % q == 0) {
            v /= q;
            if (idx++ == s) return q;
        }
    return 0;  // past the last stage
}
constexpr int ct_ns(int L, int s) {
    int ns = 1;
    for (int i = 0; i < s; ++i) ns *= ct_radix(L, i);
    return ns;
}

template <int R, int NS, int L, bool SWI, bool SWO>
__device__ __forceinline__ void mr_stage_ct(double2* buf, const double2* twl, int j, int sign) {
    constexpr int nb = L / R, step = L / (NS * R), kB = (nb + 63) / 64;
    double2 v[kB][R];
#pragma unroll
    for (int i = 0; i < kB; ++i) {
        const int b = j + 64 * i;
        if (nb % 64 == 0 || i < kB - 1 || b < nb) {
            const int k = b % NS;
#pragma unroll
            for (int q = 0; q < R; ++q) {
                double2 x = buf[lds_ix<SWI>(b + q * nb, L & ~7)];
                if (q > 0 && NS > 1) {
                    const double2 w = twl[q * k * step];
                    x = cmul(x, sign < 0 ? w : make_double2(w.x, -w.y));
                }
                v[i][q] = x;
            }
            dft_radix<R>(v[i], sign);
        }
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int i = 0; i < kB; ++i) {
        const int b = j + 64 * i;
        if (nb % 64 == 0 || i < kB - 1 || b < nb) {
            const int k = b % NS;
            const int d = (b - k) * R + k;
#pragma unroll
            for (int q = 0; q < R; ++q) buf[lds_ix<SWO>(d + q * NS, L & ~7)] = v[i][q];
        }
    }
    __builtin_amdgcn_wave_barrier();
}

template <int L, int S>
__device__ __forceinline__ void fft_ct_stages(double2* buf, const double2* twl, int j, int sign) {
    if constexpr (ct_radix(L, S) != 0) {
        constexpr bool sw = L % 2 == 0;  // swizzled between the first two stages (lds_ix)
        mr_stage_ct<ct_radix(L, S), ct_ns(L, S), L, sw && S == 1, sw && S == 0>(buf, twl, j, sign);
        fft_ct_stages<L, S + 1>(buf, twl, j, sign);
    }
}

// mr_stage_ct over two independent buffers at once (pass B's two inverse row FFTs): the same
// indices and twiddles, twice the independent work between a lane's LDS round trips.
template <int R, int NS, int L, bool SWI, bool SWO>
__device__ __forceinline__ void mr_stage_ct2(double2* buf0, double2* buf1, const double2* twl, int j, int sign) {
    constexpr int nb = L / R, step = L / (NS * R), kB = (nb + 63) / 64;
    double2 v[kB][R], u[kB][R];
#pragma unroll
    for (int i = 0; i < kB; ++i) {
        const int b = j + 64 * i;
        if (nb % 64 == 0 || i < kB - 1 || b < nb) {
            const int k = b % NS;
#pragma unroll
            for (int q = 0; q < R; ++q) {
                double2 x = buf0[lds_ix<SWI>(b + q * nb, L & ~7)];
                double2 y = buf1[lds_ix<SWI>(b + q * nb, L & ~7)];
                if (q > 0 && NS > 1) {
                    const double2 w = twl[q * k * step];
                    const double2 ws = sign < 0 ? w : make_double2(w.x, -w.y);
                    x = cmul(x, ws);
                    y = cmul(y, ws);
                }
                v[i][q] = x;
                u[i][q] = y;
            }
            dft_radix<R>(v[i], sign);
            dft_radix<R>(u[i], sign);
        }
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int i = 0; i < kB; ++i) {
        const int b = j + 64 * i;
        if (nb % 64 == 0 || i < kB - 1 || b < nb) {
            const int k = b % NS;
            const int d = (b - k) * R + k;
#pragma unroll
            for (int q = 0; q < R; ++q) {
                buf0[lds_ix<SWO>(d + q * NS, L & ~7)] = v[i][q];
                buf1[lds_ix<SWO>(d + q * NS, L & ~7)] = u[i][q];
            }
        }
    }
    __builtin_amdgcn_wave_barrier();
}

template <int L, int S>
__device__ __forceinline__ void fft_ct_stages2(double2* buf0, double2* buf1, const double2* twl, int j, int sign) {
    if constexpr (ct_radix(L, S) != 0) {
        constexpr bool sw = L % 2 == 0;
        mr_stage_ct2<ct_radix(L, S), ct_ns(L, S), L, sw && S == 1, sw && S == 0>(buf0, buf1, twl, j, sign);
        fft_ct_stages2<L, S + 1>(buf0, buf1, twl, j, sign);
    }
}

// Two in-place FFTs of the same length by one wave (interleaved for a compile-time plan).
template <bool R7, int LM, int L>
__device__ __forceinline__ void fft2_wave_any(double2* buf0, double2* buf1, const double2* twl, const Factors& f, int j,
                                              int sign) {
    if constexpr (L > 0) {
        fft_ct_stages2<L, 0>(buf0, buf1, twl, j, sign);
    } else {
        fft_mr_wave<R7, LM>(buf0, twl, f, j, sign);
        fft_mr_wave<R7, LM>(buf1, twl, f, j, sign);
    }
}

// In-place FFT of one row / column by one wave: the compile-time plan when L > 0, else the
// run-time plan f (R7 / LM: see fft_mr_wave).
template <bool R7, int LM, int L>
__device__ __forceinline__ void fft_wave_any(double2* buf, const double2* twl, const Factors& f, int j, int sign) {
    if constexpr (L > 0)
        fft_ct_stages<L, 0>(buf, twl, j, sign);
    else
        fft_mr_wave<R7, LM>(buf, twl, f, j, sign);
}

// Workgroups are dealt round-robin over the 8 XCDs: give each XCD a contiguous run of tiles, so
// that the tiles sharing a 128-B line (pass A's f32 rows, pass C's f64 rows) share its L2.
__device__ __forceinline__ int xcd_tile(int bid, int nblk) {
    return (nblk & 7) ? bid : (bid & 7) * (nblk >> 3) + (bid >> 3);
}

struct MrArgs {
    PassArgs p;
    Factors f1, f2;  // the column (N1) and row (N2) sub-FFTs
    int32_t batches;  // pass B: batches in its 1-D grid
    int32_t chain;    // pass_c_chain: pairs per block
};

// Measurement builds only (build.py --exp cprof -D ARX_CONV_PROF=1, tools/conv_phases.py): per
// workgroup of passes A / B / C, the 100-MHz device real-time counter at entry, after its loads
// reached LDS, after its FFT and at its last store; kProfSlot words per workgroup, pass k's records
// from k * kProfPass.  The product build compiles none of it.
#ifndef ARX_CONV_PROF
#define ARX_CONV_PROF 0
#endif
#if ARX_CONV_PROF
constexpr int kProfSlot = 8, kProfPass = 4096 * kProfSlot;
__device__ unsigned long long g_conv_prof[3 * kProfPass];
struct ConvProf {
    unsigned long long t[4] = {0, 0, 0, 0};
    __device__ void mark(int k) { t[k] = __builtin_amdgcn_s_memrealtime(); }
    // one word per lane of wave 0 (a vector store with per-lane addresses)
    __device__ void flush(int pass) {
        const int l = (int)threadIdx.x;
        if (l >= kProfSlot) return;
        const unsigned wg = blockIdx.y * gridDim.x + blockIdx.x;
        unsigned long long v = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) v = l == k ? t[k] : v;
        v = l == 4 ? (unsigned long long)__builtin_amdgcn_s_getreg((15 << 11) | 20) : v;  // XCC id
        v = l == 5 ? (unsigned long long)wg : v;
        if (wg < 4096) g_conv_prof[pass * kProfPass + wg * kProfSlot + l] = v;
    }
};
#define CONV_PROF_DECL ConvProf prof_;
#define CONV_PROF_MARK(k) prof_.mark(k)
#define CONV_PROF_FLUSH(pass) prof_.flush(pass)
#else
#define CONV_PROF_DECL
#define CONV_PROF_MARK(k)
#define CONV_PROF_FLUSH(pass)
#endif


// dst[i] = src[i * stride], i < count <= 64 IT, by the nt >= 64 threads (all loads issued before
// the LDS stores)
template <int IT>
__device__ __forceinline__ void stage_table(double2* dst, const double2* __restrict__ src, int count, int stride,
                                            int nt) {
    double2 v[IT];
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int i = threadIdx.x + it * nt;
        v[it] = i < count ? src[(size_t)i * stride] : make_double2(0.0, 0.0);
    }
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int i = threadIdx.x + it * nt;
        if (i < count) dst[i] = v[it];
    }
}


// LDS column stride of passes A / C with tc columns per block: N1 padded to the residue that keeps
// the tile's transposing stores (a ds_write_b128 group of 8 lanes spans 8 columns for tc = 8) and
// the loads that read it back free of bank conflicts: 7 mod 16 for tc = 8, 4 mod 8 for 4, 8 mod 16
// for 2 (an enumeration over the usual N1 on the banking model of MI355X_MICROARCH.md's LDS table).
__host__ __device__ inline int mr_col_stride(int N1, int tc) {
    const int t = tc >= 8 ? 7 : (tc == 4 ? 4 : 8), m = tc == 4 ? 8 : 16;
    return N1 + ((t - N1) % m + m) % m;
}

// Pass A: forward column FFTs of length N1 (one wave per column, tc = waves per block), * W_n^(n2 k1),
// stored transposed S[k1 N2 + n2].  LDS: tile tc x sc (mr_col_stride), W_N1 (N1), W_n^r (N2).  Mode 0's
// batch past the block pairs (batch = n_pairs) is the IR, packed h_L + i h_R: its columns go to
// G (pass_b_pair), so the IR spectra's column pass rides in the same launch as the audio's.  Mode 1
// (IR spectra alone): batch c = IR channel c, to H.
template <int MODE, bool R7, int LM, int L1>
__global__ __launch_bounds__(512) void pass_a_mr(MrArgs m) {
    constexpr int IT = LM / 64;  // per-lane elements of a column, per-thread tile loads
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    const PassArgs& a = m.p;
    const int nt = blockDim.x, tc = nt >> 6, lgc = __builtin_ctz(tc), N1 = a.N1, N2 = a.N2;
    const int64_t batch = blockIdx.y;
    const bool ir = MODE == 1 || (MODE == 0 && batch >= a.n_pairs);
    const int64_t ch = MODE == 1 ? batch : batch - a.n_pairs;
    const int n2_0 = xcd_tile(blockIdx.x, gridDim.x) * tc, sc = mr_col_stride(N1, tc);
    double2* twl = lds + (size_t)tc * sc;
    double2* tr = twl + N1;
    CONV_PROF_DECL
    CONV_PROF_MARK(0);
    double2 v[IT];
#pragma unroll
    for (int it = 0; it < IT; ++it) {  // every load in flight before the first use
        const int i = threadIdx.x + it * nt;
        const int c = i & (tc - 1), n1 = i >> lgc, n2 = n2_0 + c;
        const int64_t idx = (int64_t)N2 * n1 + n2;
        double2 x = make_double2(0.0, 0.0);
        if (n1 < N1 && n2 < N2) {
            if (MODE == 0 && ir) {
                x.x = (double)a.ir_l[idx];
                x.y = (double)a.ir_r[idx];
            } else if (ir) {
                x.x = (double)(ch == 0 ? a.ir_l : a.ir_r)[idx];
            } else if (MODE == 0) {
                if (idx < a.sr) {
                    const int64_t b0 = 2 * batch, b1 = 2 * batch + 1;
                    if (b0 < a.n_blocks) x.x = (double)a.in[b0 * a.sr + idx];
                    if (b1 < a.n_blocks) x.y = (double)a.in[b1 * a.sr + idx];
                }
            } else {
                if (idx < a.n_in) x.x = a.in_d[idx];
            }
        }
        v[it] = x;
    }
    stage_table<IT>(twl, a.tw, N1, N2, nt);  // W_N1^i = W_n^(i N2)
    stage_table<IT>(tr, a.tw, N2, 1, nt);
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int i = threadIdx.x + it * nt;
        const int c = i & (tc - 1), n1 = i >> lgc;
        if (n1 < N1) lds[(size_t)c * sc + n1] = v[it];
    }
    __syncthreads();
    CONV_PROF_MARK(1);
    fft_wave_any<R7, LM, L1>(lds + (size_t)(threadIdx.x >> 6) * sc, twl, m.f1, threadIdx.x & 63, -1);
    __syncthreads();
    CONV_PROF_MARK(2);
    double2* dst = MODE == 0 && ir ? a.G : ir ? a.H + (size_t)ch * a.M : a.S + (size_t)batch * 3 * a.M;
    // W_n^(n2 k1) = W_N1^q W_n^r with n2 k1 = q N2 + r; this thread's column n2 is fixed and k1 steps
    // by 64, so (q, r) advance by (64 n2) div / mod N2 -- one division per thread, not per element
    const int c = threadIdx.x & (tc - 1), n2 = n2_0 + c;
    const int k10 = threadIdx.x >> lgc;
    const int step = 64 * n2, dq = step / N2, dr = step - dq * N2;
    int q = (n2 * k10) / N2, r = n2 * k10 - q * N2;
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int k1 = k10 + 64 * it;
        if (k1 < N1 && n2 < N2) dst[(int64_t)k1 * N2 + n2] = cmul(lds[(size_t)c * sc + k1], cmul(twl[q], tr[r]));
        q += dq;
        r += dr;
        if (r >= N2) {
            r -= N2;
            ++q;
        }
    }
    CONV_PROF_MARK(3);
    if (MODE == 0) CONV_PROF_FLUSH(0);
}

// Pass B: per row k1 (one wave; nt / 64 rows per block): forward row FFT (N2); mode 1 stores it (IR
// spectrum); mode 0 multiplies by H_c, inverse row FFT, * W_n^(-n2 k1), for both channels.  Input
// reuse (conv_prepare_input / conv_run_prepared): mode 3 stores the forward row FFT of an audio
// block pair in place (S[pair][0] becomes the pair's full spectrum X), mode 4 is mode 0 on such an
// X (no forward FFT) -- the same arithmetic as mode 0 in two launches, so the outputs are identical.
// LDS: 2 x N2 per row (the spectrum; H_0's row, then the product), W_N2 (N2) -- small enough for
// 3 blocks per CU, so one round of blocks covers the C3 grid.
template <int MODE, bool R7, int LM, int L2>
__global__ __launch_bounds__(512) void pass_b_mr(MrArgs m) {
    constexpr int IT = LM / 64;
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    const PassArgs& a = m.p;
    const int nt = blockDim.x, rows = nt >> 6, N1 = a.N1, N2 = a.N2;
    const int w = threadIdx.x >> 6, j = threadIdx.x & 63;
    // 1-D grid of (row group, batch), dealt so that every batch of a row group runs on the same XCD:
    // the H rows the batches share are fetched into that XCD's L2 once, not once per batch.
    const int batches = (int)m.batches;
    const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
    const int group = (slot / batches) * 8 + xcd;
    const int64_t batch = slot % batches;
    const int k1 = group * rows + w;
    double2* spec = lds + (size_t)w * 2 * N2;
    double2* work = spec + N2;
    double2* tw2 = lds + (size_t)rows * 2 * N2;
    const bool live = k1 < N1;
    constexpr bool kMul = MODE == 0 || MODE == 4;  // multiply by H and invert
    double2* row = (MODE == 1) ? a.H + (size_t)batch * a.M + (int64_t)k1 * N2 : a.S + (size_t)batch * 3 * a.M + (int64_t)k1 * N2;
    // every global operand of the row up front: the row, H_0 and H_1's rows and the four-step
    // twiddles, so the wave's only global round trip before its stores is this one
    // W_n^(n2 k1) = W_N1^q W_n^r with n2 k1 = q N2 + r (as in pass A): two small tables that stay in
    // L2, where the direct W_n^(n2 k1) gathered lines from all of the n-entry table
    double2 v[IT], h[IT], h1[IT], twq[IT], twr[IT];
    const int step = 64 * k1, dq = step / N2, dr = step - dq * N2;
    int q = (j * k1) / N2, r = j * k1 - q * N2;
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int i = j + 64 * it;
        const bool in = live && i < N2;
        const bool in0 = kMul && in;
        v[it] = in ? row[i] : make_double2(0.0, 0.0);
        h[it] = in0 ? a.H[(int64_t)k1 * N2 + i] : make_double2(0.0, 0.0);
        h1[it] = in0 ? a.H[(size_t)a.M + (int64_t)k1 * N2 + i] : make_double2(0.0, 0.0);
        twq[it] = in0 ? a.tw[(int64_t)q * N2] : make_double2(1.0, 0.0);
        twr[it] = in0 ? a.tw[r] : make_double2(1.0, 0.0);
        q += dq;
        r += dr;
        if (r >= N2) {
            r -= N2;
            ++q;
        }
    }
    stage_table<IT>(tw2, a.tw, N2, N1, nt);  // W_N2^i = W_n^(i N1)
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int i = j + 64 * it;
        if (live && i < N2) {
            spec[i] = v[it];
            if (kMul) work[i] = h[it];
        }
    }
    __syncthreads();
    if (!live) return;  // no block barrier below
    if (MODE != 4) fft_wave_any<R7, LM, L2>(spec, tw2, m.f2, j, -1);
    if (MODE == 1 || MODE == 3) {
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int i = j + 64 * it;
            if (i < N2) row[i] = spec[i];
        }
        return;
    }
    // both channels' products (spec x H_0 -> work, spec x H_1 -> spec), then both inverse row FFTs
    // interleaved
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int i = j + 64 * it;
        if (i < N2) {
            const double2 x = spec[i];
            work[i] = cmul(x, work[i]);
            spec[i] = cmul(x, h1[it]);
        }
    }
    __builtin_amdgcn_wave_barrier();
    fft2_wave_any<R7, LM, L2>(work, spec, tw2, m.f2, j, +1);
    double2* dst0 = a.S + ((size_t)batch * 3 + 1) * a.M + (int64_t)k1 * N2;
    double2* dst1 = dst0 + a.M;
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int i = j + 64 * it;
        if (i < N2) {
            const double2 w = cmul(twq[it], twr[it]);
            const double2 t = make_double2(w.x, -w.y);
            dst0[i] = cmul(work[i], t);
            dst1[i] = cmul(spec[i], t);
        }
    }
}

// Pass B of a file convolution with a new IR, the IR's row FFTs folded in (no separate IR pass):
// pass A transformed the columns of g = h_L + i h_R as one packed batch (G).  For real h_L, h_R,
//   H_L[k] = (G[k] + conj(G[-k])) / 2,   H_R[k] = (G[k] - conj(G[-k])) / (2i),
// and with k = k1 + N1 k2, -k lies in row k1' = N1 - k1 at column N2 - 1 - k2 (k1 != 0), or in
// row 0 at column (N2 - k2) mod N2 (k1 = 0).  A block is the two waves of mirror rows k1, k1' of
// one block pair (rows 0 and N1/2 are their own mirrors and share a block): each wave
// transforms its S row and its G row (interleaved), reads its mirror's G row from LDS, and goes on
// as pass_b_mr<0>.  Block pair 0 also stores H_L / H_R, the spectra later calls reuse.
// LDS: 2 x N2 per wave (S's spectrum; G's row, then the product), W_N2 (N2).
// XS (input reuse, conv_run_prepared): the S rows already hold the block pairs' row spectra (pass_b_mr
// mode 3), so only the G rows are transformed forward.
// HONLY (the IR spectra alone, conv_set_ir): no block pair -- the G rows are transformed and H_L / H_R
// stored, by the same arithmetic as the fused pass's, so the spectra a convolution uses are the same
// bits whichever call made them.
template <bool R7, int LM, int L2, bool XS, bool HONLY = false>
__global__ __launch_bounds__(128) void pass_b_pair(MrArgs m) {
    constexpr int IT = LM / 64;
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    const PassArgs& a = m.p;
    const int N1 = a.N1, N2 = a.N2, units = (N1 + 1) / 2;
    const int w = threadIdx.x >> 6, j = threadIdx.x & 63;
    const int batches = (int)m.batches;
    const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
    const int u = (slot / batches) * 8 + xcd;  // mirror-row unit, dealt as pass_b_mr's row groups
    const int64_t batch = slot % batches;
    if (u >= units) return;  // the whole block: no barrier is reached
    CONV_PROF_DECL
    CONV_PROF_MARK(0);
    const bool self = u == 0;  // rows 0 and N1 / 2: each its own mirror
    const int k1 = w == 0 ? u : (self ? N1 / 2 : N1 - u);
    const bool live = !(self && w == 1 && (N1 & 1));  // odd N1: row 0 has no partner row
    double2* spec = lds + (size_t)w * 2 * N2;
    double2* gbuf = spec + N2;
    double2* gmir = self ? gbuf : lds + (size_t)(w ^ 1) * 2 * N2 + N2;
    double2* tw2 = lds + (size_t)4 * N2;
    double2* row = HONLY ? nullptr : a.S + (size_t)batch * 3 * a.M + (int64_t)k1 * N2;
    double2 v[IT], g[IT], twq[IT], twr[IT];
    const int step = 64 * k1, dq = step / N2, dr = step - dq * N2;
    int q = (j * k1) / N2, r = j * k1 - q * N2;
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int i = j + 64 * it;
        const bool in = live && i < N2;
        v[it] = (in && !HONLY) ? row[i] : make_double2(0.0, 0.0);
        g[it] = in ? a.G[(int64_t)k1 * N2 + i] : make_double2(0.0, 0.0);
        twq[it] = in ? a.tw[(int64_t)q * N2] : make_double2(1.0, 0.0);
        twr[it] = in ? a.tw[r] : make_double2(1.0, 0.0);
        q += dq;
        r += dr;
        if (r >= N2) {
            r -= N2;
            ++q;
        }
    }
    stage_table<IT>(tw2, a.tw, N2, N1, 128);  // W_N2^i = W_n^(i N1)
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int i = j + 64 * it;
        if (i < N2) {
            spec[i] = v[it];
            gbuf[i] = g[it];
        }
    }
    __syncthreads();
    CONV_PROF_MARK(1);
    if constexpr (XS || HONLY)
        fft_wave_any<R7, LM, L2>(gbuf, tw2, m.f2, j, -1);
    else
        fft2_wave_any<R7, LM, L2>(spec, gbuf, tw2, m.f2, j, -1);
    __syncthreads();  // the mirror row's G spectrum is complete
    double2 h0[IT], h1[IT];
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int i = j + 64 * it;
        if (i < N2) {
            const int mi = k1 == 0 ? (i == 0 ? 0 : N2 - i) : N2 - 1 - i;
            const double2 x = gbuf[i], y = gmir[mi];
            h0[it] = make_double2(0.5 * (x.x + y.x), 0.5 * (x.y - y.y));  // (G + conj(G-)) / 2
            h1[it] = make_double2(0.5 * (x.y + y.y), -0.5 * (x.x - y.x));  // (G - conj(G-)) / 2i
        } else {
            h0[it] = h1[it] = make_double2(0.0, 0.0);
        }
    }
    if (batch == 0 && live) {
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int i = j + 64 * it;
            if (i < N2) {
                a.H[(int64_t)k1 * N2 + i] = h0[it];
                a.H[(size_t)a.M + (int64_t)k1 * N2 + i] = h1[it];
            }
        }
    }
    if constexpr (HONLY) return;  // no barrier below is reached by any wave
    __syncthreads();  // every mirror read is done before gbuf is overwritten
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int i = j + 64 * it;
        if (i < N2) {
            const double2 x = spec[i];
            gbuf[i] = cmul(x, h0[it]);
            spec[i] = cmul(x, h1[it]);
        }
    }
    __builtin_amdgcn_wave_barrier();
    fft2_wave_any<R7, LM, L2>(gbuf, spec, tw2, m.f2, j, +1);
    CONV_PROF_MARK(2);
#if ARX_CONV_PROF
    if (!live) {
        CONV_PROF_MARK(3);
        CONV_PROF_FLUSH(1);
        return;
    }
#endif
    if (!live) return;
    double2* dst0 = a.S + ((size_t)batch * 3 + 1) * a.M + (int64_t)k1 * N2;
    double2* dst1 = dst0 + a.M;
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int i = j + 64 * it;
        if (i < N2) {
            const double2 tw = cmul(twq[it], twr[it]);
            const double2 t = make_double2(tw.x, -tw.y);
            dst0[i] = cmul(gbuf[i], t);
            dst1[i] = cmul(spec[i], t);
        }
    }
    CONV_PROF_MARK(3);
    CONV_PROF_FLUSH(1);
}

// Pass C: inverse column FFTs of each (pair, channel) -> n * circular convolution of the pair's two
// blocks (re / im), to Y (length n per block and channel).  LDS: tile tc x sc, W_N1 (N1).
template <bool R7, int LM, int L1>
__global__ __launch_bounds__(512) void pass_c_mr(MrArgs m) {
    constexpr int IT = LM / 64;
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    const PassArgs& a = m.p;
    const int nt = blockDim.x, tc = nt >> 6, lgc = __builtin_ctz(tc), N1 = a.N1, N2 = a.N2;
    const int64_t pair = blockIdx.y >> 1;
    const int ch = blockIdx.y & 1;
    const int n2_0 = xcd_tile(blockIdx.x, gridDim.x) * tc, sc = mr_col_stride(N1, tc);
    const double2* src = a.S + ((size_t)pair * 3 + 1 + ch) * a.M;
    double2* twl = lds + (size_t)tc * sc;
    double2 v[IT];
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int i = threadIdx.x + it * nt;
        const int c = i & (tc - 1), k1 = i >> lgc, n2 = n2_0 + c;
        v[it] = (k1 < N1 && n2 < N2) ? src[(int64_t)k1 * N2 + n2] : make_double2(0.0, 0.0);
    }
    stage_table<IT>(twl, a.tw, N1, N2, nt);
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int i = threadIdx.x + it * nt;
        const int c = i & (tc - 1), k1 = i >> lgc;
        if (k1 < N1) lds[(size_t)c * sc + k1] = v[it];
    }
    __syncthreads();
    fft_wave_any<R7, LM, L1>(lds + (size_t)(threadIdx.x >> 6) * sc, twl, m.f1, threadIdx.x & 63, +1);
    __syncthreads();
    const int64_t b0 = 2 * pair, b1 = 2 * pair + 1;
    double* y0 = a.Y + (b0 * 2 + ch) * a.ylen;
    double* y1 = a.Y + (b1 * 2 + ch) * a.ylen;
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int i = threadIdx.x + it * nt;
        const int c = i & (tc - 1), n1 = i >> lgc, n2 = n2_0 + c;
        if (n1 < N1 && n2 < N2) {
            const int64_t idx = (int64_t)N2 * n1 + n2;
            const double2 x = lds[(size_t)c * sc + n1];
            if (b0 < a.n_blocks) y0[idx] = x.x;
            if (b1 < a.n_blocks) y1[idx] = x.y;
        }
    }
}

// Pass C for n = 2 sr and N1 even, fused with the seam sum: a block runs one column tile of one
// channel through a chain of consecutive pairs p0 .. p1-1 (m.chain per block), preceded by pair
// p0-1 again when p0 > 0.  Rows n1 < N1/2 of a pair's inverse columns hold the first half of each
// block's window (i = idx < sr), rows n1 + N1/2 the second: the pair's odd output segment 2p+1 =
// y_2p[i + sr] + y_2p+1[i] (hi.x + lo.y) lies inside the pair, and the even segment 2p =
// y_2p-1[i + sr] + y_2p[i] adds the previous pair's hi.y, which this thread computed for the same
// (column, row) one step earlier and holds in registers.  Sums in pass D's order (0 + F + E),
// rounded once; no block window goes through HBM (Y), and no seam pass runs.
template <bool R7, int LM, int L1>
__device__ __forceinline__ void pass_c_chain_body(const MrArgs& m) {
    constexpr int IT = LM / 64;
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    const PassArgs& a = m.p;
    const int nt = blockDim.x, tc = nt >> 6, lgc = __builtin_ctz(tc), N1 = a.N1, N2 = a.N2, half = N1 >> 1;
    const int ch = blockIdx.y & 1;
    const int64_t p0 = a.emit_from + (int64_t)(blockIdx.y >> 1) * m.chain;
    const int64_t p1 = p0 + m.chain < a.n_pairs ? p0 + m.chain : a.n_pairs;
    const int n2_0 = xcd_tile(blockIdx.x, gridDim.x) * tc, sc = mr_col_stride(N1, tc);
    double2* twl = lds + (size_t)tc * sc;
    const int64_t sr = a.sr;
    float* out = ch == 0 ? a.out_l : a.out_r;
    CONV_PROF_DECL
    CONV_PROF_MARK(0);
    stage_table<IT>(twl, a.tw, N1, N2, nt);
    double2 v[IT];
    double fprev[IT];  // hi.y of the previous pair at this thread's (column, row) slots
    const int64_t pstart = p0 > 0 ? p0 - 1 : 0;
    auto load = [&](int64_t pair) {
        const double2* src = a.S + ((size_t)pair * 3 + 1 + ch) * a.M;
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int i = threadIdx.x + it * nt;
            const int c = i & (tc - 1), k1 = i >> lgc, n2 = n2_0 + c;
            v[it] = (k1 < N1 && n2 < N2) ? src[(int64_t)k1 * N2 + n2] : make_double2(0.0, 0.0);
        }
    };
    load(pstart);
#pragma unroll
    for (int it = 0; it < IT; ++it) fprev[it] = 0.0;
    for (int64_t pair = pstart; pair < p1; ++pair) {
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int i = threadIdx.x + it * nt;
            const int c = i & (tc - 1), k1 = i >> lgc;
            if (k1 < N1) lds[(size_t)c * sc + k1] = v[it];
        }
        __syncthreads();
#if ARX_CONV_PROF
        if (pair == pstart) CONV_PROF_MARK(1);
#endif
        if (pair + 1 < p1) load(pair + 1);  // in flight during this pair's FFT
        fft_wave_any<R7, LM, L1>(lds + (size_t)(threadIdx.x >> 6) * sc, twl, m.f1, threadIdx.x & 63, +1);
        __syncthreads();
#if ARX_CONV_PROF
        if (pair == pstart) CONV_PROF_MARK(2);
#endif
        const int64_t b1 = 2 * pair + 1;
        const bool odd = b1 < a.n_blocks;  // the pair's second block exists
        const bool emit = pair >= p0;     // pair p0 - 1 only supplies fprev
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int i = threadIdx.x + it * nt;
            const int c = i & (tc - 1), n1 = i >> lgc, n2 = n2_0 + c;
            if (n1 < half && n2 < N2) {
                const int64_t idx = (int64_t)N2 * n1 + n2;
                const double2 lo = lds[(size_t)c * sc + n1], hi = lds[(size_t)c * sc + n1 + half];
                if (emit) {
                    const int64_t te = 2 * pair * sr + idx, to = b1 * sr + idx;
                    if (te < a.len) {
                        double acc = 0.0;
                        acc += fprev[it];  // F_p-1 (zero for p = 0)
                        acc += lo.x;       // E_p
                        out[te] = (float)(acc * a.scale);
                    }
                    if (to < a.len) {
                        double acc = 0.0;
                        acc += hi.x;
                        if (odd) acc += lo.y;
                        out[to] = (float)(acc * a.scale);
                    }
                }
                fprev[it] = odd ? hi.y : 0.0;
            }
        }
        __syncthreads();  // the tile is rewritten by the next pair
    }
    if (p1 == a.n_pairs && a.tail) {  // the segment after the last pair: F_last alone
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int i = threadIdx.x + it * nt;
            const int c = i & (tc - 1), n1 = i >> lgc, n2 = n2_0 + c;
            if (n1 < half && n2 < N2) {
                const int64_t idx = (int64_t)N2 * n1 + n2, t = 2 * p1 * sr + idx;
                if (t < a.len) {
                    double acc = 0.0;
                    acc += fprev[it];
                    out[t] = (float)(acc * a.scale);
                }
            }
        }
    }
    CONV_PROF_MARK(3);
    CONV_PROF_FLUSH(2);
}
// The compile-time plans (L1 > 0) fit in 168 VGPRs = 3 waves per SIMD without spilling; left to
// itself the compiler took 169 (2 waves), so the C3 launch's 640 four-wave blocks (2.5 waves per
// SIMD) ran in two rounds (8.5 us entry skew, tools/conv_phases.py).  The run-time plans keep the
// unconstrained allocation (168 would spill there).
template <bool R7, int LM, int L1>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(3))) void pass_c_chain3(MrArgs m) {
    pass_c_chain_body<R7, LM, L1>(m);
}
template <bool R7, int LM, int L1>
__global__ __launch_bounds__(512) void pass_c_chain(MrArgs m) {
    pass_c_chain_body<R7, LM, L1>(m);
}

int ilog2(int64_t v) {
    int l = 0;
    while (((int64_t)1 << l) < v) ++l;
    return l;
}

// L = 8^a 4^b 2^c 3^d 5^e 7^f; false if L has another prime factor
bool factor7(int32_t L, Factors& f) {
    f.L = L;
    f.count = 0;
    int32_t v = L, twos = 0;
    while (v % 2 == 0) {
        v /= 2;
        ++twos;
    }
    auto push = [&](int r) {
        if (f.count < kMaxRadices) f.r[f.count] = r;
        ++f.count;
    };
    for (; twos >= 3; twos -= 3) push(8);
    if (twos == 2) push(4);
    if (twos == 1) push(2);
    for (int q : {3, 5, 7})
        while (v % q == 0) {
            v /= q;
            push(q);
        }
    return v == 1 && f.count <= kMaxRadices;
}

// n = N1 x N2, both 7-smooth and <= kMaxSubLen; prefer N2 % 8 == 0 (full 128-B row segments in
// passes A / C), then the most balanced split.
bool direct_split(int32_t n, int32_t& N1, int32_t& N2) {
    Factors f;
    int64_t best = -1;
    for (int32_t d = 2; d <= kMaxSubLen; ++d) {
        if (n % d) continue;
        const int32_t e = n / d;
        if (e < 2 || e > kMaxSubLen || !factor7(d, f) || !factor7(e, f)) continue;
        const int64_t score = (e % 8 ? 1000000 : 0) + std::abs(d - e);
        if (best < 0 || score < best) {
            best = score;
            N1 = d;
            N2 = e;
        }
    }
    return best >= 0;
}

}  // namespace

ConvPlan* conv_plan_create(int32_t ir_len, int32_t sample_rate, int device, char* err, size_t errlen) {
    auto bad = [&](const char* m) -> ConvPlan* {
        if (err && errlen) std::snprintf(err, errlen, "%s", m);
        return nullptr;
    };
    if (ir_len <= 0 || sample_rate <= 0) return bad("ir_len and sample_rate must be positive");
    const int64_t need = (int64_t)ir_len + (int64_t)std::min(ir_len, sample_rate) - 1;
    const int lg = ilog2(std::max<int64_t>(need, 4));
    if (lg > 24) return bad("FFT length above 2^24 is not supported");
    ConvPlan* p = new ConvPlan();
    p->n = ir_len;
    p->sr = sample_rate;
    p->device = device;
    int32_t d1 = 0, d2 = 0;
    if (ir_len >= sample_rate && direct_split(ir_len, d1, d2) && factor7(d1, p->f1) && factor7(d2, p->f2)) {
        p->direct = true;
        for (int i = 0; i < p->f1.count; ++i) p->r7 |= p->f1.r[i] == 7;
        for (int i = 0; i < p->f2.count; ++i) p->r7 |= p->f2.r[i] == 7;
        p->M = ir_len;
        p->N1 = d1;
        p->N2 = d2;
        p->tc = 8;  // unused on this path (see mr_tiles)
        std::snprintf(p->desc, sizeof(p->desc), "mixed-radix direct circular: n=%d sr=%d (%dx%d) f64", p->n, p->sr,
                      p->N1, p->N2);
    } else {
        p->M = 1 << lg;
        p->lg1 = lg / 2;
        p->lg2 = lg - p->lg1;
        p->N1 = 1 << p->lg1;
        p->N2 = 1 << p->lg2;
        p->tc = std::max(1, std::min(std::min(16, p->N2), 4096 / p->N1));
        std::snprintf(p->desc, sizeof(p->desc), "pow2 linear+fold: n=%d sr=%d M=%d (%dx%d) f64", p->n, p->sr, p->M,
                      p->N1, p->N2);
    }
    hipSetDevice(device);
    std::vector<double2> tw((size_t)p->M);
    const long double two_pi = 6.283185307179586476925286766559L;
    for (int64_t e = 0; e < p->M; ++e) {
        const long double ang = two_pi * (long double)e / (long double)p->M;
        tw[(size_t)e] = make_double2((double)cosl(ang), -(double)sinl(ang));
    }
    if (hipMalloc(&p->d_tw, (size_t)p->M * sizeof(double2)) != hipSuccess ||
        hipMalloc(&p->d_H, 2 * (size_t)p->M * sizeof(double2)) != hipSuccess ||
        (p->direct && hipMalloc(&p->d_G, (size_t)p->M * sizeof(double2)) != hipSuccess) ||
        hipMemcpy(p->d_tw, tw.data(), (size_t)p->M * sizeof(double2), hipMemcpyHostToDevice) != hipSuccess) {
        conv_plan_destroy(p);
        return bad("device allocation failed");
    }
    return p;
}

void conv_plan_destroy(ConvPlan* p) {
    if (!p) return;
    hipFree(p->d_prep_in);
    hipFree(p->d_tw);
    hipFree(p->d_H);
    hipFree(p->d_G);
    hipFree(p->d_S);
    hipFree(p->d_Y);
    delete p;
}

const char* conv_plan_describe(const ConvPlan* p) { return p ? p->desc : ""; }

// Pass B: the wave-per-row pass (pass_bw) for rows of 512 or 256, else the generic radix-4 pass.
template <int MODE>
static void launch_pass_b(const ConvPlan* p, unsigned batches, const PassArgs& a, hipStream_t s) {
    if (p->N2 == 512 && p->N1 % 4 == 0)
        hipLaunchKernelGGL((pass_bw<MODE, 512>), dim3(p->N1 / 4, batches), dim3(kThreads), (4 + 1) * 512 * sizeof(double2), s, a);
    else if (p->N2 == 256 && p->N1 % 4 == 0)
        hipLaunchKernelGGL((pass_bw<MODE, 256>), dim3(p->N1 / 4, batches), dim3(kThreads), (4 + 1) * 256 * sizeof(double2), s, a);
    else
        hipLaunchKernelGGL(pass_b<MODE>, dim3(p->N1, batches), dim3(kThreads), 2 * (size_t)p->N2 * sizeof(double2), s, a);
}

// per block and channel: n (direct) or the linear length n + sr - 1 that pass D folds
static int64_t plan_ylen(const ConvPlan* p) {
    return p->direct ? (int64_t)p->n : (int64_t)p->n + std::min(p->n, p->sr) - 1;
}

static PassArgs base_args(const ConvPlan* p) {
    PassArgs a;
    std::memset(&a, 0, sizeof(a));
    a.tw = p->d_tw;
    a.M = p->M;
    a.N1 = p->N1;
    a.N2 = p->N2;
    a.lg1 = p->lg1;
    a.lg2 = p->lg2;
    a.tc = p->tc;
    a.n = p->n;
    a.sr = p->sr;
    a.H = p->d_H;
    a.G = p->d_G;
    a.ylen = plan_ylen(p);
    a.emit_from = 0;
    a.tail = 1;
    return a;
}

static MrArgs mr_args(const ConvPlan* p, const PassArgs& a) {
    MrArgs m;
    m.p = a;
    m.f1 = p->f1;
    m.f2 = p->f2;
    m.batches = 1;
    m.chain = 1;
    return m;
}
// Direct-path launch shapes: passes A / C run one wave per column, tc columns per block (8 for the
// batched block pairs, 2 for the two IR channels and the single live block, for more blocks);
// pass B one wave per row, `rows` rows per block.
static unsigned mr_tiles(const ConvPlan* p, int tc) { return (unsigned)((p->N2 + tc - 1) / tc); }
static size_t mr_lds_a(const ConvPlan* p, int tc) {
    return ((size_t)tc * mr_col_stride(p->N1, tc) + p->N1 + p->N2) * sizeof(double2);
}
static size_t mr_lds_c(const ConvPlan* p, int tc) { return ((size_t)tc * mr_col_stride(p->N1, tc) + p->N1) * sizeof(double2); }
static unsigned mr_rows(const ConvPlan* p, int rows) { return (unsigned)((p->N1 + rows - 1) / rows); }
static size_t mr_lds_b(const ConvPlan* p, int rows) { return ((size_t)rows * 2 * p->N2 + p->N2) * sizeof(double2); }
template <bool R7, int LM, int L2, bool XS = false, bool HONLY = false>
static void launch_b_pair(const ConvPlan* p, int batches, MrArgs m, hipStream_t s) {
    const unsigned units8 = (unsigned)((p->N1 + 1) / 2 + 7) / 8 * 8;  // see pass_b_pair's XCD mapping
    m.batches = batches;
    hipLaunchKernelGGL((pass_b_pair<R7, LM, L2, XS, HONLY>), dim3(units8 * (unsigned)batches), dim3(128), mr_lds_b(p, 2),
                       s, m);
}
template <int MODE, bool R7, int LM, int L2>
static void launch_b_mr(const ConvPlan* p, int rows, int batches, MrArgs m, hipStream_t s) {
    const unsigned groups8 = (mr_rows(p, rows) + 7) / 8 * 8;  // see pass_b_mr's XCD mapping
    m.batches = batches;
    hipLaunchKernelGGL((pass_b_mr<MODE, R7, LM, L2>), dim3(groups8 * (unsigned)batches), dim3(64 * rows), mr_lds_b(p, rows), s,
                       m);
}

#ifndef ARX_CONV_TCA
#define ARX_CONV_TCA 8
#endif
// IR spectra alone (arx_prepare_ir_spectra, the live path, a file shorter than one block): the packed
// IR h_L + i h_R through pass A's IR batch (to G) and pass B's mirror-row split (to H) -- the route a
// file convolution with a new IR takes, so H comes out the same bits either way
template <bool R7, int LM, int L1, int L2>
static void mr_ir(const ConvPlan* p, const PassArgs& a, hipStream_t s) {
    const MrArgs m = mr_args(p, a);
    MrArgs mi = m;
    mi.p.n_pairs = 0;  // batch 0 of this launch is the IR (pass_a_mr mode 0's batch past the pairs)
    hipLaunchKernelGGL((pass_a_mr<0, R7, LM, L1>), dim3(mr_tiles(p, ARX_CONV_TCA), 1u), dim3(64 * ARX_CONV_TCA),
                       mr_lds_a(p, ARX_CONV_TCA), s, mi);
    launch_b_pair<R7, LM, L2, false, true>(p, 1, m, s);
}

// File convolution; with_ir: the packed IR's columns ride in pass A's launch as an extra batch and
// its rows in pass B (pass_b_pair).
// Launch shapes (columns per block in A / C, rows per block in B); the ARX_CONV_* macros exist only
// for design-experiment builds (build.py --exp).
#ifndef ARX_CONV_TCA
#define ARX_CONV_TCA 8
#endif
#ifndef ARX_CONV_TCC
#define ARX_CONV_TCC 4
#endif
#ifndef ARX_CONV_ROWSB
#define ARX_CONV_ROWSB 4
#endif
#ifndef ARX_CONV_CHAIN
#define ARX_CONV_CHAIN 2
#endif
template <bool R7, int LM, int L1, int L2>
static void mr_pass_c(const ConvPlan* p, const PassArgs& a, int64_t pairs, hipStream_t s);
template <bool R7, int LM, int L1, int L2>
static void mr_file(const ConvPlan* p, const PassArgs& a, int64_t pairs, bool with_ir, hipStream_t s) {
    MrArgs m = mr_args(p, a);
    hipLaunchKernelGGL((pass_a_mr<0, R7, LM, L1>), dim3(mr_tiles(p, ARX_CONV_TCA), (unsigned)(pairs + (with_ir ? 1 : 0))),
                       dim3(64 * ARX_CONV_TCA), mr_lds_a(p, ARX_CONV_TCA), s, m);
    if (with_ir)
        launch_b_pair<R7, LM, L2>(p, (int)pairs, m, s);
    else
        launch_b_mr<0, R7, LM, L2>(p, ARX_CONV_ROWSB, (int)pairs, m, s);
    mr_pass_c<R7, LM, L1, L2>(p, a, pairs, s);
}

// Input reuse, step 1 (conv_prepare_input): the audio's columns (pass A) and forward rows (pass B
// mode 3) once; S[pair][0] keeps every block pair's spectrum.
template <bool R7, int LM, int L1, int L2>
static void mr_prepare(const ConvPlan* p, const PassArgs& a, int64_t pairs, hipStream_t s) {
    MrArgs m = mr_args(p, a);
    hipLaunchKernelGGL((pass_a_mr<0, R7, LM, L1>), dim3(mr_tiles(p, ARX_CONV_TCA), (unsigned)pairs), dim3(64 * ARX_CONV_TCA),
                       mr_lds_a(p, ARX_CONV_TCA), s, m);
    launch_b_mr<3, R7, LM, L2>(p, ARX_CONV_ROWSB, (int)pairs, m, s);
}

// Input reuse, step 2 (conv_run_prepared): a new IR's columns alone in pass A (one batch, to G), then
// pass B without the audio's forward rows (pass_b_pair<XS> with a new IR, mode 4 without), then pass C.
template <bool R7, int LM, int L1, int L2>
static void mr_prepared(const ConvPlan* p, const PassArgs& a, int64_t pairs, bool with_ir, hipStream_t s) {
    MrArgs m = mr_args(p, a);
    if (with_ir) {
        MrArgs mi = m;
        mi.p.n_pairs = 0;  // batch 0 of this launch is the IR (pass_a_mr mode 0's batch past the pairs)
        hipLaunchKernelGGL((pass_a_mr<0, R7, LM, L1>), dim3(mr_tiles(p, ARX_CONV_TCA), 1u), dim3(64 * ARX_CONV_TCA),
                           mr_lds_a(p, ARX_CONV_TCA), s, mi);
        launch_b_pair<R7, LM, L2, true>(p, (int)pairs, m, s);
    } else {
        launch_b_mr<4, R7, LM, L2>(p, ARX_CONV_ROWSB, (int)pairs, m, s);
    }
    mr_pass_c<R7, LM, L1, L2>(p, a, pairs, s);
}

template <bool R7, int LM, int L1, int L2>
static void mr_pass_c(const ConvPlan* p, const PassArgs& a, int64_t pairs, hipStream_t s) {
    MrArgs m = mr_args(p, a);
    if (p->n == 2 * p->sr && p->N1 % 2 == 0) {  // inverse columns and seams in one pass
        m.chain = ARX_CONV_CHAIN;
        const unsigned chains = (unsigned)((pairs - a.emit_from + m.chain - 1) / m.chain);
        if constexpr (L1 > 0)
            hipLaunchKernelGGL((pass_c_chain3<R7, LM, L1>), dim3(mr_tiles(p, ARX_CONV_TCC), 2 * chains),
                               dim3(64 * ARX_CONV_TCC), mr_lds_c(p, ARX_CONV_TCC), s, m);
        else
            hipLaunchKernelGGL((pass_c_chain<R7, LM, L1>), dim3(mr_tiles(p, ARX_CONV_TCC), 2 * chains),
                               dim3(64 * ARX_CONV_TCC), mr_lds_c(p, ARX_CONV_TCC), s, m);
        return;
    }
    hipLaunchKernelGGL((pass_c_mr<R7, LM, L1>), dim3(mr_tiles(p, ARX_CONV_TCC), (unsigned)(2 * pairs)),
                       dim3(64 * ARX_CONV_TCC), mr_lds_c(p, ARX_CONV_TCC), s, m);
    hipLaunchKernelGGL(pass_d, dim3((unsigned)((a.len + kThreads - 1) / kThreads), 2), dim3(kThreads), 0, s, a);
}

template <bool R7, int LM, int L1, int L2>
static void mr_live(const ConvPlan* p, const PassArgs& a, hipStream_t s) {
    const MrArgs m = mr_args(p, a);
    hipLaunchKernelGGL((pass_a_mr<2, R7, LM, L1>), dim3(mr_tiles(p, 2), 1), dim3(128), mr_lds_a(p, 2), s, m);
    launch_b_mr<0, R7, LM, L2>(p, 1, 1, m, s);
    hipLaunchKernelGGL((pass_c_mr<R7, LM, L1>), dim3(mr_tiles(p, 2), 2), dim3(128), mr_lds_c(p, 2), s, m);
}

// The kernels exist for the sub-FFT pairs with compile-time plans (fft_ct_stages) and, for any
// other split, for sub-FFT lengths <= 320 / <= 512 with and without radix-7 stages.
template <typename Fn>
static void mr_dispatch(const ConvPlan* p, Fn&& fn) {
    using std::integral_constant;
    const int N1 = p->N1, N2 = p->N2;
    if (N1 == 300 && N2 == 320)
        fn(std::false_type{}, integral_constant<int, 320>{}, integral_constant<int, 300>{}, integral_constant<int, 320>{});
    else if (N1 == 160 && N2 == 200)
        fn(std::false_type{}, integral_constant<int, 320>{}, integral_constant<int, 160>{}, integral_constant<int, 200>{});
    else if (N1 == 315 && N2 == 280)
        fn(std::true_type{}, integral_constant<int, 320>{}, integral_constant<int, 315>{}, integral_constant<int, 280>{});
    else if (N1 == 250 && N2 == 256)
        fn(std::false_type{}, integral_constant<int, 320>{}, integral_constant<int, 250>{}, integral_constant<int, 256>{});
    else if (std::max(N1, N2) <= 320) {
        if (p->r7)
            fn(std::true_type{}, integral_constant<int, 320>{}, integral_constant<int, 0>{}, integral_constant<int, 0>{});
        else
            fn(std::false_type{}, integral_constant<int, 320>{}, integral_constant<int, 0>{}, integral_constant<int, 0>{});
    } else {
        if (p->r7)
            fn(std::true_type{}, integral_constant<int, 512>{}, integral_constant<int, 0>{}, integral_constant<int, 0>{});
        else
            fn(std::false_type{}, integral_constant<int, 512>{}, integral_constant<int, 0>{}, integral_constant<int, 0>{});
    }
}

#if ARX_CONV_PROF
// Measurement builds only: read (and clear) the per-workgroup phase records (tools/conv_phases.py).
extern "C" int arx_exp_conv_profile(unsigned long long* out, size_t n_words) {
    const size_t total = 3 * (size_t)kProfPass;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_conv_prof), std::min(n_words, total) * 8, 0, hipMemcpyDeviceToHost) != hipSuccess)
        return 1;
    std::vector<unsigned long long> z(total, 0ull);
    return hipMemcpyToSymbol(HIP_SYMBOL(g_conv_prof), z.data(), total * 8, 0, hipMemcpyHostToDevice) != hipSuccess;
}
#endif

hipError_t conv_set_ir(ConvPlan* p, const float* d_ir_left, const float* d_ir_right, hipStream_t s) {
    (void)hipGetLastError();  // report this launch's error, not a stale one
    PassArgs a = base_args(p);
    a.ir_l = d_ir_left;
    a.ir_r = d_ir_right;
    const size_t lds_a = ((size_t)p->tc + 1) * p->N1 * sizeof(double2);  // + the twiddle table
    if (p->direct) {
        mr_dispatch(p, [&](auto r7, auto lm, auto l1, auto l2) {
            mr_ir<decltype(r7)::value, decltype(lm)::value, decltype(l1)::value, decltype(l2)::value>(p, a, s);
        });
        return hipGetLastError();
    }
    hipLaunchKernelGGL(pass_a<1>, dim3(p->N2 / p->tc, 2), dim3(kThreads), lds_a, s, a);
    launch_pass_b<1>(p, 2, a, s);
    return hipGetLastError();
}

// The chained pass C (inverse columns and seams in one pass, no block windows in HBM): n = 2 sr on the
// direct path with N1 even.  Only these plans convolve a time-block shard on its own.
static bool chain_plan(const ConvPlan* p) { return p->direct && p->n == 2 * p->sr && p->N1 % 2 == 0; }

bool conv_plan_shards(const ConvPlan* p) { return p && chain_plan(p); }

hipError_t conv_run(ConvPlan* p, const float* d_in, int64_t n_frames, float* d_out_left, float* d_out_right,
                    const float* d_ir_left, const float* d_ir_right, hipStream_t s) {
    return conv_run_pairs(p, d_in, n_frames, d_out_left, d_out_right, d_ir_left, d_ir_right, 0, INT64_MAX, s);
}

// conv_run restricted to the block pairs [pair_begin, pair_end) (time blocks sharded
// across GPUs).  On a chained plan the shard runs passes A and B over its pairs plus the pair before
// them (the seam: its second block's tail F, re-made here instead of received from the neighbour) and
// pass C emits exactly the output segments of its own pairs -- the same per-pair arithmetic in the
// same summation order as the whole file's chains (which re-make the previous pair at every chain
// boundary already), so the union of the shards is the whole convolution bit for bit.  Other plans
// convolve the whole file (every frame written).
hipError_t conv_run_pairs(ConvPlan* p, const float* d_in, int64_t n_frames, float* d_out_left, float* d_out_right,
                          const float* d_ir_left, const float* d_ir_right, int64_t pair_begin, int64_t pair_end,
                          hipStream_t s) {
    const bool with_ir = d_ir_left && d_ir_right;
    if (with_ir && (!p->direct || n_frames < p->sr)) {  // spectra first, then the audio
        const hipError_t e = conv_set_ir(p, d_ir_left, d_ir_right, s);
        if (e != hipSuccess) return e;
        return conv_run_pairs(p, d_in, n_frames, d_out_left, d_out_right, nullptr, nullptr, pair_begin, pair_end, s);
    }
    if (n_frames <= 0) return hipSuccess;
    p->prepared = false;  // any other file convolution discards a prepared input (pass A overwrites its spectra)
    int64_t S = n_frames / p->sr;  // kernels.cu:413
    if (S == 0) {  // nothing convolved: the reference output stays zero (a shard past pair 0 owns none of it)
        if (pair_begin > 0) return hipSuccess;
        hipError_t e = hipMemsetAsync(d_out_left, 0, (size_t)n_frames * sizeof(float), s);
        if (e == hipSuccess) e = hipMemsetAsync(d_out_right, 0, (size_t)n_frames * sizeof(float), s);
        return e;
    }
    const int64_t all_pairs = (S + 1) / 2;
    int64_t base = 0, pairs = all_pairs;  // local pair 0 = global pair `base`
    int32_t emit_from = 0, tail = 1;
    if (chain_plan(p) && (pair_begin > 0 || pair_end < all_pairs)) {
        const int64_t pb = std::max<int64_t>(0, std::min(pair_begin, all_pairs));
        const int64_t pe = std::max<int64_t>(pb, std::min(pair_end, all_pairs));
        if (pe == pb) {  // an empty shard: its IR spectra still follow the IR
            if (!with_ir) return hipSuccess;
            return conv_set_ir(p, d_ir_left, d_ir_right, s);
        }
        base = pb > 0 ? pb - 1 : 0;
        emit_from = pb > 0 ? 1 : 0;
        tail = pe == all_pairs ? 1 : 0;
        pairs = pe - base;
        const int64_t off = 2 * base * (int64_t)p->sr;
        d_in += off;
        d_out_left += off;
        d_out_right += off;
        n_frames -= off;
        S = std::min<int64_t>(S - 2 * base, 2 * pairs);
    }
    const int64_t ylen = plan_ylen(p);
    // the chained pass C (mr_file) keeps the block windows on chip: no Y
    const bool windows = !(p->direct && p->n == 2 * p->sr && p->N1 % 2 == 0);
    if (pairs > p->pairs_cap || (windows && !p->d_Y)) {
        hipFree(p->d_S);
        hipFree(p->d_Y);
        p->d_S = nullptr;
        p->d_Y = nullptr;
        p->pairs_cap = 0;
        hipError_t e = hipMalloc(&p->d_S, (size_t)pairs * 3 * p->M * sizeof(double2));
        if (e != hipSuccess) return e;
        if (windows) {
            e = hipMalloc(&p->d_Y, (size_t)pairs * 2 * 2 * ylen * sizeof(double));
            if (e != hipSuccess) return e;
        }
        p->pairs_cap = pairs;
    }
    (void)hipGetLastError();  // report this launch's error, not a stale one
    PassArgs a = base_args(p);
    a.in = d_in;
    a.S = p->d_S;
    a.Y = p->d_Y;
    a.n_blocks = S;
    a.n_pairs = pairs;
    a.len = n_frames;
    a.out_l = d_out_left;
    a.out_r = d_out_right;
    a.scale = (double)p->n / ((double)p->M * (double)(p->n / 2));  // AudioRenderer.cpp:709
    a.ir_l = d_ir_left;
    a.ir_r = d_ir_right;
    a.emit_from = emit_from;
    a.tail = tail;
    const size_t lds_a = ((size_t)p->tc + 1) * p->N1 * sizeof(double2);  // + the twiddle table
    if (p->direct) {
        mr_dispatch(p, [&](auto r7, auto lm, auto l1, auto l2) {
            mr_file<decltype(r7)::value, decltype(lm)::value, decltype(l1)::value, decltype(l2)::value>(p, a, pairs,
                                                                                                        with_ir, s);
        });
        return hipGetLastError();
    } else {
        hipLaunchKernelGGL(pass_a<0>, dim3(p->N2 / p->tc, (unsigned)pairs), dim3(kThreads), lds_a, s, a);
        launch_pass_b<0>(p, (unsigned)pairs, a, s);
        hipLaunchKernelGGL(pass_c, dim3(p->N2 / p->tc, (unsigned)(2 * pairs)), dim3(kThreads), lds_a, s, a);
    }
    hipLaunchKernelGGL(pass_d, dim3((unsigned)((n_frames + kThreads - 1) / kThreads), 2), dim3(kThreads), 0, s, a);
    return hipGetLastError();
}

// Input reuse (the reference's re-render pattern: full_render_cycle convolves the same file with
// every new IR, AudioRenderer.cpp:790-798, main.cpp:40-67).  conv_prepare_input transforms the file's
// block pairs once (pass A + forward rows, S[pair][0] keeps the spectra); conv_run_prepared then costs
// a new IR's spectra (its columns alone in pass A, its rows in pass B), the products and the inverse
// rows (pass B, no forward FFT of the audio) and pass C.  Same arithmetic as conv_run in the same
// order, so the output is bit-identical.  Plans without the chained pass C keep a copy of the input
// and convolve it in full.
static bool reuse_spectra(const ConvPlan* p) { return p->direct && p->n == 2 * p->sr && p->N1 % 2 == 0; }

static hipError_t ensure_scratch(ConvPlan* p, int64_t pairs) {
    if (pairs <= p->pairs_cap && p->d_S) return hipSuccess;
    hipFree(p->d_S);
    hipFree(p->d_Y);
    p->d_S = nullptr;
    p->d_Y = nullptr;
    p->pairs_cap = 0;
    p->prepared = false;
    const hipError_t e = hipMalloc(&p->d_S, (size_t)pairs * 3 * p->M * sizeof(double2));
    if (e == hipSuccess) p->pairs_cap = pairs;
    return e;
}

hipError_t conv_prepare_input(ConvPlan* p, const float* d_in, int64_t n_frames, hipStream_t s) {
    p->prepared = false;
    p->prep_frames = n_frames > 0 ? n_frames : 0;
    p->prep_spectra = reuse_spectra(p);
    const int64_t S = p->prep_frames / p->sr, pairs = (S + 1) / 2;
    (void)hipGetLastError();
    if (!p->prep_spectra) {  // keep the samples: conv_run_prepared convolves them in full
        if ((size_t)p->prep_frames > p->prep_cap) {
            hipFree(p->d_prep_in);
            p->d_prep_in = nullptr;
            p->prep_cap = 0;
            const hipError_t e = hipMalloc(&p->d_prep_in, (size_t)p->prep_frames * sizeof(float));
            if (e != hipSuccess) return e;
            p->prep_cap = (size_t)p->prep_frames;
        }
        if (p->prep_frames > 0) {
            const hipError_t e = hipMemcpyAsync(p->d_prep_in, d_in, (size_t)p->prep_frames * sizeof(float),
                                                hipMemcpyDeviceToDevice, s);
            if (e != hipSuccess) return e;
        }
        p->prepared = true;
        return hipSuccess;
    }
    if (S > 0) {
        hipError_t e = ensure_scratch(p, pairs);
        if (e != hipSuccess) return e;
        PassArgs a = base_args(p);
        a.in = d_in;
        a.S = p->d_S;
        a.n_blocks = S;
        a.n_pairs = pairs;
        a.len = p->prep_frames;
        mr_dispatch(p, [&](auto r7, auto lm, auto l1, auto l2) {
            mr_prepare<decltype(r7)::value, decltype(lm)::value, decltype(l1)::value, decltype(l2)::value>(p, a, pairs, s);
        });
        e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    p->prepared = true;
    return hipSuccess;
}

bool conv_has_prepared(const ConvPlan* p) { return p && p->prepared; }
int64_t conv_prepared_frames(const ConvPlan* p) { return p && p->prepared ? p->prep_frames : 0; }

hipError_t conv_run_prepared(ConvPlan* p, float* d_out_left, float* d_out_right, const float* d_ir_left,
                             const float* d_ir_right, hipStream_t s) {
    if (!p->prepared) return hipErrorInvalidValue;
    const int64_t n_frames = p->prep_frames;
    if (!p->prep_spectra) {
        const hipError_t e = conv_run(p, p->d_prep_in, n_frames, d_out_left, d_out_right, d_ir_left, d_ir_right, s);
        p->prepared = true;  // conv_run above reads the kept copy; nothing of it is overwritten
        return e;
    }
    const bool with_ir = d_ir_left && d_ir_right;
    const int64_t S = n_frames / p->sr;
    if (S == 0) {  // no block: the output stays zero (kernels.cu:413), the IR spectra still follow the IR
        if (with_ir) {
            const hipError_t e = conv_set_ir(p, d_ir_left, d_ir_right, s);
            if (e != hipSuccess) return e;
        }
        if (n_frames <= 0) return hipSuccess;
        hipError_t e = hipMemsetAsync(d_out_left, 0, (size_t)n_frames * sizeof(float), s);
        if (e == hipSuccess) e = hipMemsetAsync(d_out_right, 0, (size_t)n_frames * sizeof(float), s);
        return e;
    }
    const int64_t pairs = (S + 1) / 2;
    (void)hipGetLastError();
    PassArgs a = base_args(p);
    a.S = p->d_S;
    a.n_blocks = S;
    a.n_pairs = pairs;
    a.len = n_frames;
    a.out_l = d_out_left;
    a.out_r = d_out_right;
    a.scale = (double)p->n / ((double)p->M * (double)(p->n / 2));  // AudioRenderer.cpp:709
    a.ir_l = d_ir_left;
    a.ir_r = d_ir_right;
    mr_dispatch(p, [&](auto r7, auto lm, auto l1, auto l2) {
        mr_prepared<decltype(r7)::value, decltype(lm)::value, decltype(l1)::value, decltype(l2)::value>(p, a, pairs,
                                                                                                      with_ir, s);
    });
    return hipGetLastError();
}

int32_t conv_plan_block(const ConvPlan* p) { return p ? p->sr : 0; }

hipError_t conv_run_live(ConvPlan* p, const double* d_in, int64_t n_in, double* d_out_interleaved, hipStream_t s) {
    if (n_in < 0 || n_in > p->sr) return hipErrorInvalidValue;
    const int64_t ylen = plan_ylen(p);
    if (p->pairs_cap < 1 || !p->d_Y) {
        hipFree(p->d_S);
        hipFree(p->d_Y);
        p->d_S = nullptr;
        p->d_Y = nullptr;
        hipError_t e = hipMalloc(&p->d_S, (size_t)3 * p->M * sizeof(double2));
        if (e != hipSuccess) return e;
        e = hipMalloc(&p->d_Y, (size_t)2 * 2 * ylen * sizeof(double));
        if (e != hipSuccess) return e;
        p->pairs_cap = 1;
    }
    (void)hipGetLastError();  // report this launch's error, not a stale one
    PassArgs a = base_args(p);
    a.in_d = d_in;
    a.n_in = n_in;
    a.S = p->d_S;
    a.Y = p->d_Y;
    a.n_blocks = 1;
    a.n_pairs = 1;
    a.out_d = d_out_interleaved;
    a.scale = (double)p->n / ((double)p->M * (double)(p->n / 2));  // Z2D (x n) / (ir_len/2)
    const size_t lds_a = ((size_t)p->tc + 1) * p->N1 * sizeof(double2);  // + the twiddle table
    if (p->direct) {
        mr_dispatch(p, [&](auto r7, auto lm, auto l1, auto l2) {
            mr_live<decltype(r7)::value, decltype(lm)::value, decltype(l1)::value, decltype(l2)::value>(p, a, s);
        });
    } else {
        hipLaunchKernelGGL(pass_a<2>, dim3(p->N2 / p->tc, 1), dim3(kThreads), lds_a, s, a);
        launch_pass_b<0>(p, 1, a, s);
        hipLaunchKernelGGL(pass_c, dim3(p->N2 / p->tc, 2), dim3(kThreads), lds_a, s, a);
    }
    hipLaunchKernelGGL(pass_d_live, dim3((unsigned)((p->n + kThreads - 1) / kThreads)), dim3(kThreads), 0, s, a);
    return hipGetLastError();
}

// ==================================================================================================
// Streaming convolution for the RtAudio duplex callback: uniformly
// partitioned overlap-save (UPOLS) in f64, replacing the reference's per-callback full-length
// circular convolution (AudioRenderer.cpp:593-661, kernels.cu:345-377) whose 2*ir_len outputs the
// CircularBuffer then wraps onto itself (main.cpp:189-195).  Per block of B frames:
//   fwd  X_b = FFT_N(last N input samples)                   (one workgroup, LDS, N <= 8192)
//   mac  Z   = sum_p X_(b-p) * G_p,  G_p = FFT_N(hL_p + i hR_p), h_p = h[pB, (p+1)B) zero padded
//   inv  y_L + i y_R = IFFT_N(Z)[N-B, N)                     (one workgroup, LDS)
// N = the power of two >= 2B, P = ceil(ir_len / B).  Because h_L and h_R are real, one complex
// spectrum per partition (G_p) and one inverse FFT serve both ears.  Output: B frames zipped L/R,
// scaled like the reference's live path, ir_len / (ir_len/2) x the linear convolution
// (normalizeBuffers, kernels.cu:450-467), but without the circular wrap and the CircularBuffer
// aliasing.  The frequency-domain delay line keeps input spectra, so a new IR (a moving listener)
// takes effect at the next block without a glitch-inducing restart.
struct StreamPlan {
    int32_t B = 0, N = 0, lgN = 0, P = 0, n = 0;
    int64_t blocks = 0;           // processed since reset (slot of block b = b % P)
    double2* d_tw = nullptr;      // W_N^e
    double2* d_G = nullptr;       // P * N partition spectra
    double2* d_X = nullptr;       // P * N input spectra ring (frequency-domain delay line)
    double2* d_Z = nullptr;       // N accumulated spectrum
    double* d_hist = nullptr;     // N - B input history
    double scale = 0.0;
};

namespace {

constexpr int kStreamThreads = 1024;  // lds_fft needs >= N/16 threads

// The stream kernels' twiddles: W_N^e = hi[e >> 6] * lo[e & 63] from two small tables staged in LDS
// after the N-point buffer (a global table lookup per butterfly put an L2 round trip into every
// stage of these single-workgroup FFTs).
__device__ __forceinline__ TwSplit stream_twiddles(double2* lds, int32_t N, int32_t lgN, const double2* __restrict__ tw) {
    const int lgLo = lgN < 6 ? lgN : 6;
    double2* hi = lds + N;
    double2* lo = hi + (N >> lgLo);
    for (int i = threadIdx.x; i < (N >> lgLo); i += kStreamThreads) hi[i] = tw[(size_t)i << lgLo];
    for (int i = threadIdx.x; i < (1 << lgLo); i += kStreamThreads) lo[i] = tw[i];
    return TwSplit{hi, lo, lgLo, N};
}
static size_t stream_lds(int32_t N) { return ((size_t)N + (size_t)(N >> 4) + 64) * sizeof(double2); }

// G_p = FFT_N(hL[pB + i] + i hR[pB + i], i < B, zero padded): one workgroup per partition.
__global__ __launch_bounds__(kStreamThreads) void stream_ir_kernel(const float* __restrict__ hl,
                                                                   const float* __restrict__ hr, int32_t n,
                                                                   int32_t B, int32_t N, int32_t lgN,
                                                                   const double2* __restrict__ tw,
                                                                   double2* __restrict__ G) {
    extern __shared__ double2 buf[];
    const int p = blockIdx.x;
    for (int i = threadIdx.x; i < N; i += kStreamThreads) {
        const int64_t k = (int64_t)p * B + i;
        buf[i] = (i < B && k < n) ? make_double2((double)hl[k], (double)hr[k]) : make_double2(0.0, 0.0);
    }
    const TwSplit twf = stream_twiddles(buf, N, lgN, tw);
    __syncthreads();
    lds_fft_t(buf, N, lgN, -1, threadIdx.x, kStreamThreads, twf, N);
    for (int i = threadIdx.x; i < N; i += kStreamThreads) G[(size_t)p * N + i] = buf[i];
}

// X_b = FFT_N([history (N - B), block (B)]), history <- the window's last N - B samples.
__global__ __launch_bounds__(kStreamThreads) void stream_fwd_kernel(const double* __restrict__ in, int32_t n_in,
                                                                    double* __restrict__ hist, int32_t B, int32_t N,
                                                                    int32_t lgN, const double2* __restrict__ tw,
                                                                    double2* __restrict__ X) {
    extern __shared__ double2 buf[];
    const int H = N - B;
    for (int i = threadIdx.x; i < N; i += kStreamThreads) {
        double v;
        if (i < H) v = hist[i];
        else v = (i - H < n_in) ? in[i - H] : 0.0;
        buf[i] = make_double2(v, 0.0);
    }
    const TwSplit twf = stream_twiddles(buf, N, lgN, tw);
    __syncthreads();
    for (int i = threadIdx.x; i < H; i += kStreamThreads) hist[i] = buf[i + B].x;
    lds_fft_t(buf, N, lgN, -1, threadIdx.x, kStreamThreads, twf, N);  // (its first barrier orders the reads above)
    for (int i = threadIdx.x; i < N; i += kStreamThreads) X[i] = buf[i];
}

// Z[k] = sum_p X_((b - p) mod P)[k] * G_p[k]: one thread per bin, coalesced over k.
__global__ __launch_bounds__(256) void stream_mac_kernel(const double2* __restrict__ X, const double2* __restrict__ G,
                                                         int32_t P, int32_t N, int32_t newest,
                                                         double2* __restrict__ Z) {
    const int k = blockIdx.x * 256 + threadIdx.x;
    if (k >= N) return;
    double2 acc = make_double2(0.0, 0.0);
    int slot = newest;
    for (int p = 0; p < P; ++p) {
        const double2 x = X[(size_t)slot * N + k];
        const double2 g = G[(size_t)p * N + k];
        acc.x = fma(x.x, g.x, fma(-x.y, g.y, acc.x));
        acc.y = fma(x.x, g.y, fma(x.y, g.x, acc.y));
        slot = slot == 0 ? P - 1 : slot - 1;
    }
    Z[k] = acc;
}

// y_L + i y_R = IFFT_N(Z)[N - B, N), zipped and scaled.
__global__ __launch_bounds__(kStreamThreads) void stream_inv_kernel(const double2* __restrict__ Z, int32_t B,
                                                                    int32_t N, int32_t lgN,
                                                                    const double2* __restrict__ tw, double scale,
                                                                    double* __restrict__ out) {
    extern __shared__ double2 buf[];
    for (int i = threadIdx.x; i < N; i += kStreamThreads) buf[i] = Z[i];
    const TwSplit twf = stream_twiddles(buf, N, lgN, tw);
    __syncthreads();
    lds_fft_t(buf, N, lgN, +1, threadIdx.x, kStreamThreads, twf, N);
    for (int i = threadIdx.x; i < B; i += kStreamThreads) {
        const double2 v = buf[N - B + i];
        out[2 * i] = v.x * scale;
        out[2 * i + 1] = v.y * scale;
    }
}

}  // namespace

StreamPlan* stream_plan_create(int32_t ir_len, int32_t block, int device, char* err, size_t errlen) {
    auto bad = [&](const char* m) -> StreamPlan* {
        if (err && errlen) std::snprintf(err, errlen, "%s", m);
        return nullptr;
    };
    if (ir_len <= 0 || block <= 0 || block > 4096) return bad("stream block must be in [1, 4096] frames");
    StreamPlan* p = new StreamPlan();
    p->B = block;
    p->lgN = ilog2(2 * (int64_t)block);
    p->lgN = std::max(p->lgN, 4);
    p->N = 1 << p->lgN;
    p->P = (int32_t)(((int64_t)ir_len + block - 1) / block);
    p->n = ir_len;
    p->scale = (double)ir_len / ((double)p->N * (double)(ir_len / 2));  // unnormalised IFFT, / (ir_len/2)
    hipSetDevice(device);
    std::vector<double2> tw((size_t)p->N);
    const long double two_pi = 6.283185307179586476925286766559L;
    for (int64_t e = 0; e < p->N; ++e) {
        const long double ang = two_pi * (long double)e / (long double)p->N;
        tw[(size_t)e] = make_double2((double)cosl(ang), -(double)sinl(ang));
    }
    const size_t spec = (size_t)p->P * p->N * sizeof(double2);
    if (hipMalloc(&p->d_tw, (size_t)p->N * sizeof(double2)) != hipSuccess || hipMalloc(&p->d_G, spec) != hipSuccess ||
        hipMalloc(&p->d_X, spec) != hipSuccess || hipMalloc(&p->d_Z, (size_t)p->N * sizeof(double2)) != hipSuccess ||
        hipMalloc(&p->d_hist, (size_t)(p->N - p->B + 1) * sizeof(double)) != hipSuccess ||
        hipMemcpy(p->d_tw, tw.data(), (size_t)p->N * sizeof(double2), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemset(p->d_G, 0, spec) != hipSuccess) {
        stream_plan_destroy(p);
        return bad("device allocation failed");
    }
    if (stream_reset(p, nullptr) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
        stream_plan_destroy(p);
        return bad("stream reset failed");
    }
    return p;
}

void stream_plan_destroy(StreamPlan* p) {
    if (!p) return;
    hipFree(p->d_tw);
    hipFree(p->d_G);
    hipFree(p->d_X);
    hipFree(p->d_Z);
    hipFree(p->d_hist);
    delete p;
}

hipError_t stream_reset(StreamPlan* p, hipStream_t s) {
    p->blocks = 0;
    hipError_t e = hipMemsetAsync(p->d_X, 0, (size_t)p->P * p->N * sizeof(double2), s);
    if (e == hipSuccess) e = hipMemsetAsync(p->d_hist, 0, (size_t)(p->N - p->B + 1) * sizeof(double), s);
    return e;
}

hipError_t stream_set_ir(StreamPlan* p, const float* d_ir_left, const float* d_ir_right, hipStream_t s) {
    (void)hipGetLastError();  // report this launch's error, not a stale one
    hipLaunchKernelGGL(stream_ir_kernel, dim3(p->P), dim3(kStreamThreads), stream_lds(p->N), s, d_ir_left,
                       d_ir_right, p->n, p->B, p->N, p->lgN, p->d_tw, p->d_G);
    return hipGetLastError();
}

hipError_t stream_run(StreamPlan* p, const double* d_in, int64_t n_in, double* d_out_interleaved, hipStream_t s) {
    (void)hipGetLastError();  // report this launch's error, not a stale one
    if (n_in < 0 || n_in > p->B) return hipErrorInvalidValue;
    const int32_t slot = (int32_t)(p->blocks % p->P);
    const size_t lds = stream_lds(p->N);
    hipLaunchKernelGGL(stream_fwd_kernel, dim3(1), dim3(kStreamThreads), lds, s, d_in, (int32_t)n_in, p->d_hist, p->B,
                       p->N, p->lgN, p->d_tw, p->d_X + (size_t)slot * p->N);
    hipLaunchKernelGGL(stream_mac_kernel, dim3((unsigned)((p->N + 255) / 256)), dim3(256), 0, s, p->d_X, p->d_G, p->P,
                       p->N, slot, p->d_Z);
    hipLaunchKernelGGL(stream_inv_kernel, dim3(1), dim3(kStreamThreads), lds, s, p->d_Z, p->B, p->N, p->lgN, p->d_tw,
                       p->scale, d_out_interleaved);
    ++p->blocks;
    return hipGetLastError();
}

#ifndef ARX_CONV_SRC_ID
#define ARX_CONV_SRC_ID 0ull  // set by build.py: hash of this file's sources and experiment macros
#endif
uint64_t conv_kernel_source_id() { return ARX_CONV_SRC_ID; }

int32_t stream_plan_block(const StreamPlan* p) { return p ? p->B : 0; }
int32_t stream_plan_partitions(const StreamPlan* p) { return p ? p->P : 0; }
int32_t stream_plan_fft(const StreamPlan* p) { return p ? p->N : 0; }

}  // namespace arx
