// Microbenchmark (diagnostic only): one bf16x6 256x256 hidden layer (mlp_layer_x6: lead groups,
// fused relu/bias, split of the next input block under the MFMAs) per iteration, one wave per SIMD,
// biases in LDS, weights streamed from a footprint of FOOT distinct layers (1: L2-hot; 7: one net's
// hidden layers; 14: two nets, more than an XCD's 4 MB L2).  Ideal: 768 MFMAs x 32 = 24,576 cycles.
#include "../../a-nerf_amd/csrc/anerf_render.hip"

constexpr int LAYER_FLOATS = 128 * 12 * 256 / 4;  // 128 groups x 3 KiB

__global__ __launch_bounds__(256, 1) void layer_probe_x6(const float* w, int nlayers, int foot, float* out,
                                                         unsigned long long* cyc) {
    __shared__ float bias[2 * 256];
    const int lane = threadIdx.x & 63;
    for (int i = threadIdx.x; i < 512; i += 256) bias[i] = 0.001f * (i % 7);
    __syncthreads();
    f32x16 acc[8], h[8];
    for (int i = 0; i < 8; ++i) acc[i] = f32x16{0.5f}, h[i] = f32x16{0};
    Ring ring;
    float sig = 0.0f;
    bool pre = false;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int L = 0; L < nlayers; ++L) {
        const float* wl = w + (size_t)(L % foot) * LAYER_FLOATS;
        const float* wn = w + (size_t)((L + 1) % foot) * LAYER_FLOATS;
        mlp_layer_x6<8, 8, true, false>(acc, acc, h, bias, wl, lane, ring, pre, wn, nullptr, sig);
        pre = true;
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0;
    for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][15];
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (lane == 0) atomicAdd(cyc, t1 - t0);  // every wave
}

int main() {
    float *w, *out;
    unsigned long long* d;
    const int maxfoot = 14;  // 384 KiB per layer
    hipMalloc(&w, (size_t)maxfoot * LAYER_FLOATS * 4);
    hipMemset(w, 0, (size_t)maxfoot * LAYER_FLOATS * 4);
    hipMalloc(&out, 256 * 256 * 4);
    hipMalloc(&d, 8);
    const int nl = 56;
    for (int foot : {1, 7, 8, 9, 10, 11, 12, 14})
        for (int rep = 0; rep < 2; ++rep) {
            hipMemset(d, 0, 8);
            hipEvent_t e0, e1;
            hipEventCreate(&e0);
            hipEventCreate(&e1);
            hipEventRecord(e0, 0);
            hipLaunchKernelGGL(layer_probe_x6, dim3(256), dim3(256), 0, 0, w, nl, foot, out, d);
            hipEventRecord(e1, 0);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            unsigned long long hcyc = 0;
            hipMemcpy(&hcyc, d, 8, hipMemcpyDeviceToHost);
            if (rep == 1)
                printf("x6 layer, footprint %2d layers: %.1f TFLOP/s (bf16 MFMA), %.0f cycles per layer per wave "
                       "(ideal 24576: %.1f %%)\n",
                       foot, 256.0 * 4 * nl * 768 * 32768 / (ms * 1e-3) / 1e12, (double)hcyc / (256 * 4) / nl,
                       100.0 * 24576 / ((double)hcyc / (256 * 4) / nl));
        }
    return 0;
}
