// Microbenchmark (diagnostic only): v_mfma_f32_32x32x2_f32 stream (8 independent accumulators,
// operands resident) with K independent compiler-scheduled v_max_i32 / v_fma_f32 between
// consecutive MFMAs (sched_group_barrier interleave), one wave per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int K, int OP>
__global__ __launch_bounds__(256, 1) void probe(const float* in, float* out, int iters) {
    const int lane = threadIdx.x & 63;
    f32x16 acc[8];
    for (int i = 0; i < 8; ++i) acc[i] = f32x16{0};
    float a = in[lane], b = in[64 + lane];
    float x[16];
    for (int i = 0; i < 16; ++i) x[i] = in[128 + i * 64 + lane];
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int rb = 0; rb < 8; ++rb) {
                acc[rb] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[rb], 0, 0, 0);
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    const int i = (rb * K + k) & 15;
                    if (OP == 0)
                        x[i] = __builtin_bit_cast(float, max(__builtin_bit_cast(int, x[i]), 0) + 1);
                    else if (OP == 1)
                        x[i] = __builtin_fmaf(x[i], 1.0001f, 0.5f);
                    else if (OP == 2)
                        x[i] = x[i] + 0.5f;
                    else if (OP == 3)
                        x[i] = x[i] * 1.0001f;
                    else if (OP == 4)
                        x[i] = __builtin_bit_cast(float, max(__builtin_bit_cast(int, x[i]), 0));
                    else if (OP == 5)
                        x[i] = __builtin_amdgcn_exp2f(x[i]);
                    else if (OP == 6)
                        x[i] = __builtin_bit_cast(float, __builtin_bit_cast(int, x[i]) ^ 0x5);
                }
            }
            if (K) {
#pragma unroll
                for (int rb = 0; rb < 8; ++rb) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x002, K * (OP == 0 ? 2 : 1), 0);
                }
            }
        }
    }
    float s = 0;
    for (int i = 0; i < 16; ++i) s += x[i];
    for (int i = 0; i < 8; ++i) s += acc[i][0];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int K, int OP>
void run(const float* in, float* out) {
    const int iters = 2048;
    for (int rep = 0; rep < 2; ++rep) {
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        hipEventRecord(e0, 0);
        hipLaunchKernelGGL((probe<K, OP>), dim3(256), dim3(256), 0, 0, in, out, iters);
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        const double n = 256.0 * 4 * iters * 32;
        const char* nm[] = {"v_max_i32+v_add_u32", "v_fma_f32", "v_add_f32", "v_mul_f32", "v_max_i32", "v_exp_f32", "v_xor_b32"};
        if (rep) printf("K=%2d %-20s per MFMA: %.1f TFLOP/s  (%.2f ns per MFMA per SIMD)\n", K, nm[OP],
                        n * 4096 / (ms * 1e-3) / 1e12, ms * 1e6 / (iters * 32.0));
    }
}

int main() {
    float *in, *out;
    hipMalloc(&in, 4096 * 4);
    hipMemset(in, 0, 4096 * 4);
    hipMalloc(&out, 256 * 256 * 4);
    run<0, 1>(in, out);
    run<4, 1>(in, out);
    run<8, 1>(in, out);
    run<4, 2>(in, out);
    run<8, 2>(in, out);
    run<4, 3>(in, out);
    run<4, 4>(in, out);
    run<8, 4>(in, out);
    run<12, 4>(in, out);
    run<4, 5>(in, out);
    run<4, 6>(in, out);
    run<8, 6>(in, out);
    return 0;
}
