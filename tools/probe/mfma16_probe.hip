// Microbenchmark (diagnostic only): v_mfma_f32_16x16x4_f32 with A operands streamed from a
// footprint of F bytes (4 x b128 per 16 MFMAs = twice the bytes per FLOP of the 32x32x2 stream),
// one or two waves per SIMD, plus K independent VALU per MFMA.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 bload4(__amdgpu_buffer_rsrc_t rs, int voff, int soff) {
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, 0));
}

template <int MASK, int K>
__global__ __launch_bounds__(512) void probe(const float* w, int ngroups, float* out) {
    const int lane = threadIdx.x & 63;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)w, 0, 0x7fffffff, 0x00020000);
    f32x4 acc[16];
    for (int i = 0; i < 16; ++i) acc[i] = f32x4{0};
    float ring[4][16];
    for (int s = 0; s < 4; ++s)
        for (int i = 0; i < 16; ++i) ring[s][i] = w[(s * 16 + i) * 64 + lane];
    float b = w[lane];
    float x0 = b, x1 = b * 2, x2 = b * 3, x3 = b * 4;
    for (int g0 = 0; g0 < ngroups; g0 += 4) {
#pragma unroll
        for (int gg = 0; gg < 4; ++gg) {
            __builtin_amdgcn_sched_barrier(0);
            const int g = (g0 + gg + 2 + blockIdx.x * 97 + (threadIdx.x >> 6) * 31) & MASK;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const f32x4 x = bload4(rs, lane * 16 + i * 1024, g * 4096);
                ring[(gg + 2) % 4][4 * i] = x[0], ring[(gg + 2) % 4][4 * i + 1] = x[1];
                ring[(gg + 2) % 4][4 * i + 2] = x[2], ring[(gg + 2) % 4][4 * i + 3] = x[3];
            }
#pragma unroll
            for (int rb = 15; rb >= 0; --rb) {
                acc[rb] = __builtin_amdgcn_mfma_f32_16x16x4f32(ring[gg][rb], b, acc[rb], 0, 0, 0);
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    x0 = x0 * 1.0001f + 0.5f;
                    if (k % 4 == 1) x1 = x1 * 1.0001f + 0.5f;
                    if (k % 4 == 2) x2 = x2 * 1.0001f + 0.5f;
                    if (k % 4 == 3) x3 = x3 * 1.0001f + 0.5f;
                }
            }
            if (K) {
#pragma unroll
                for (int rb = 0; rb < 16; ++rb) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x002, 2 * K, 0);
                }
            }
        }
    }
    float s = x0 + x1 + x2 + x3;
    for (int i = 0; i < 16; ++i) s += acc[i][0] + acc[i][3];
    out[blockIdx.x * 512 + threadIdx.x] = s;
}

template <int MASK, int K>
void run(const float* w, float* out, int ngroups, int threads) {
    for (int rep = 0; rep < 2; ++rep) {
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        hipEventRecord(e0, 0);
        hipLaunchKernelGGL((probe<MASK, K>), dim3(256), dim3(threads), 0, 0, w, ngroups, out);
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        if (rep == 1) {
            const double n_mfma = 256.0 * threads / 64 * ngroups * 16;
            printf("16x16x4 footprint %5.1f MB  waves/SIMD %d  VALU/MFMA %d:  %.1f TFLOP/s\n", (MASK + 1) * 4096 / 1048576.0,
                   threads / 256, K, n_mfma * 2048 / (ms * 1e-3) / 1e12);
        }
    }
}

int main() {
    float *w, *out;
    hipMalloc(&w, 4096 * 4096);
    hipMemset(w, 0, 4096 * 4096);
    hipMalloc(&out, 256 * 512 * 4);
    const int ng = 8192;
    run<63, 0>(w, out, ng, 256);
    run<63, 0>(w, out, ng, 512);
    run<2047, 0>(w, out, ng, 256);
    run<2047, 0>(w, out, ng, 512);
    run<4095, 0>(w, out, ng, 512);
    run<2047, 2>(w, out, ng, 256);
    run<2047, 2>(w, out, ng, 512);
    run<2047, 4>(w, out, ng, 256);
    run<2047, 4>(w, out, ng, 512);
    return 0;
}
