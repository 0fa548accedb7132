// Microbenchmark (diagnostic only): cost of streaming the A operands of v_mfma_f32_32x32x2_f32
// from L2 with buffer_load_dwordx4 (16 floats = 16 MFMAs per 4 loads, ring of 4 slots, prefetch
// distance 2) vs. MFMAs on register-resident operands.  One wave per SIMD, 256 workgroups.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ f32x4 bload4(__amdgpu_buffer_rsrc_t rs, int voff, int soff) {
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, 0));
}

template <int MODE>  // 0: operands resident, 1: streamed (4 b128 per 16 MFMAs) from 256 KB, 2: from 8 MB, 3: 16 MB
__global__ __launch_bounds__(256, 1) void probe(const float* w, int ngroups, float* out, unsigned long long* cyc) {
    const int lane = threadIdx.x & 63;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)w, 0, 0x7fffffff, 0x00020000);
    f32x16 acc[8];
    for (int i = 0; i < 8; ++i) acc[i] = f32x16{0};
    float ring[4][16];
    for (int s = 0; s < 4; ++s)
        for (int i = 0; i < 16; ++i) ring[s][i] = w[(s * 16 + i) * 64 + lane];
    const float b0 = w[lane], b1 = w[64 + lane];
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int g0 = 0; g0 < ngroups; g0 += 4) {
#pragma unroll
        for (int gg = 0; gg < 4; ++gg) {
            __builtin_amdgcn_sched_barrier(0);
            if (MODE >= 1) {
                const int mask = MODE == 1 ? 63 : (MODE == 2 ? 2047 : 4095);  // 4 KB groups
                const int g = (g0 + gg + 2 + (MODE >= 2 ? blockIdx.x * 97 : 0)) & mask;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const f32x4 x = bload4(rs, lane * 16 + i * 1024, g * 4096);
                    ring[(gg + 2) % 4][4 * i] = x[0], ring[(gg + 2) % 4][4 * i + 1] = x[1];
                    ring[(gg + 2) % 4][4 * i + 2] = x[2], ring[(gg + 2) % 4][4 * i + 3] = x[3];
                }
            }
#pragma unroll
            for (int t = 1; t >= 0; --t)
#pragma unroll
                for (int rb = 7; rb >= 0; --rb)
                    acc[rb] = __builtin_amdgcn_mfma_f32_32x32x2f32(ring[gg][rb * 2 + t], t ? b1 : b0, acc[rb], 0, 0, 0);
        }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0;
    for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][15];
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (threadIdx.x == 0) atomicAdd(cyc, t1 - t0);
}

template <int MODE>
void run(const float* w, float* out, unsigned long long* d, int ngroups) {
    for (int rep = 0; rep < 2; ++rep) {
        hipMemset(d, 0, 8);
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        hipEventRecord(e0, 0);
        hipLaunchKernelGGL(probe<MODE>, dim3(256), dim3(256), 0, 0, w, ngroups, out, d);
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        if (rep == 1) {
            const double n_mfma = 256.0 * 4 * ngroups * 16;
            printf("mode=%d (%s)  %.3f ms  %.1f TFLOP/s  %.1f ns per MFMA per SIMD\n", MODE,
                   MODE == 0 ? "operands resident" : (MODE == 1 ? "streamed, 256 KB footprint" : (MODE == 2 ? "streamed, 8 MB footprint" : "streamed, 16 MB footprint")), ms,
                   n_mfma * 4096 / (ms * 1e-3) / 1e12, ms * 1e6 / (ngroups * 16.0));
        }
    }
}

int main() {
    float *w, *out;
    unsigned long long* d;
    hipMalloc(&w, 4096 * 4096);
    hipMemset(w, 0, 4096 * 4096);
    hipMalloc(&out, 256 * 256 * 4);
    hipMalloc(&d, 8);
    const int ng = 16384;
    run<0>(w, out, d, ng);
    run<1>(w, out, d, ng);
    run<2>(w, out, d, ng);
    run<3>(w, out, d, ng);
    return 0;
}
