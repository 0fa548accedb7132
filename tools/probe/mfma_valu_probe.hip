// Microbenchmark (diagnostic only): cycles per v_mfma_f32_32x32x2_f32 when K independent
// VALU instructions sit between consecutive MFMAs (one wave per SIMD), and the same for
// dependent accumulation on one accumulator.  Prints one line per K.
#include <hip/hip_runtime.h>
#include <cstdio>

#ifndef ITERS
#define ITERS 4096
#endif
#define STR2(x) #x
#define STR(x) STR2(x)

template <int K, int DEP>
__global__ __launch_bounds__(512) void probe(unsigned long long* out) {
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            if (DEP)
                asm volatile("v_mfma_f32_32x32x2_f32 a[0:15], v40, v41, a[0:15]" ::: "a0", "a1", "a2", "a3", "a4", "a5", "a6", "a7", "a8", "a9", "a10", "a11", "a12", "a13", "a14", "a15");
            else if (r % 4 == 0)
                asm volatile("v_mfma_f32_32x32x2_f32 a[0:15], v40, v41, a[0:15]" ::: "a0", "a1", "a2", "a3", "a4", "a5", "a6", "a7", "a8", "a9", "a10", "a11", "a12", "a13", "a14", "a15");
            else if (r % 4 == 1)
                asm volatile("v_mfma_f32_32x32x2_f32 a[16:31], v40, v41, a[16:31]" ::: "a16", "a17", "a18", "a19", "a20", "a21", "a22", "a23", "a24", "a25", "a26", "a27", "a28", "a29", "a30", "a31");
            else if (r % 4 == 2)
                asm volatile("v_mfma_f32_32x32x2_f32 a[32:47], v40, v41, a[32:47]" ::: "a32", "a33", "a34", "a35", "a36", "a37", "a38", "a39", "a40", "a41", "a42", "a43", "a44", "a45", "a46", "a47");
            else
                asm volatile("v_mfma_f32_32x32x2_f32 a[48:63], v40, v41, a[48:63]" ::: "a48", "a49", "a50", "a51", "a52", "a53", "a54", "a55", "a56", "a57", "a58", "a59", "a60", "a61", "a62", "a63");
#pragma unroll
            for (int k = 0; k < K; ++k) asm volatile("v_add_f32 v%0, v42, v43" ::"n"(44 + (k % 16)) : "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59");
        }
    }
    asm volatile("s_nop 7\n s_nop 7" ::);
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) atomicAdd(out, t1 - t0);
}

template <int K, int DEP>
void run(unsigned long long* d, int threads = 256) {
    hipMemset(d, 0, 8);
    hipLaunchKernelGGL((probe<K, DEP>), dim3(256), dim3(threads), 0, 0, d);
    hipMemset(d, 0, 8);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, 0);
    hipLaunchKernelGGL((probe<K, DEP>), dim3(256), dim3(threads), 0, 0, d);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    unsigned long long h = 0;
    hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
    const double per_wave = (double)h / (256.0 * threads / 64);
    const double n_mfma = 256.0 * threads / 64 * ITERS * 16;
    printf("waves/SIMD=%d K=%2d dep=%d  memtime cycles/MFMA %.1f   wall %.3f ms -> %.1f TFLOP/s, %.1f ns/MFMA/SIMD\n", K, DEP,
           per_wave / (ITERS * 16.0), ms, n_mfma * 4096 / (ms * 1e-3) / 1e12, ms * 1e6 / (ITERS * 16.0));
    (void)0;
}

int main() {
    unsigned long long* d;
    hipMalloc(&d, 8);
    run<0, 0>(d); run<2, 0>(d); run<4, 0>(d); run<6, 0>(d); run<8, 0>(d); run<10, 0>(d); run<12, 0>(d);
    run<14, 0>(d); run<16, 0>(d); run<20, 0>(d);
    run<0, 1>(d); run<4, 1>(d); run<8, 1>(d);
    run<0, 0>(d, 512); run<4, 0>(d, 512); run<8, 0>(d, 512); run<12, 0>(d, 512); run<16, 0>(d, 512);
    run<20, 0>(d, 512);
    hipFree(d);
    return 0;
}
