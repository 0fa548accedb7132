// Microbenchmark (diagnostic only): cost of one dense 256x256 layer of the render kernel
// (mlp_layer: lead groups + fused relu/bias boundary) against the same MFMA stream without the
// boundary work.  One wave per SIMD, weights L2-resident, biases in LDS.
#include "../../a-nerf_amd/csrc/anerf_render.hip"

template <int MODE>
__global__ __launch_bounds__(256, 1) void layer_probe(const float* w, int nlayers, float* out, unsigned long long* cyc) {
    __shared__ float bias[2 * 256];
    const int lane = threadIdx.x & 63;
    for (int i = threadIdx.x; i < 512; i += 256) bias[i] = 0.001f * (i % 7);
    __syncthreads();
    f32x16 acc[8], h[8];
    for (int i = 0; i < 8; ++i) acc[i] = f32x16{0}, h[i] = f32x16{0};
    Ring ring;
    ring_preload<16>(ring, w, lane);
    float sig = 0.0f;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int L = 0; L < nlayers; ++L) {
        if (MODE == 0)
            mlp_layer<8, 8, true, true, false>(acc, acc, h, bias, w, lane, ring, w, nullptr, sig);
        else
            mlp_layer<8, 8, false, false, false>(acc, h, h, nullptr, w, lane, ring, w, nullptr, sig);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0;
    for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][15];
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (threadIdx.x == 0) atomicAdd(cyc, t1 - t0);
}

int main() {
    float *w, *out;
    unsigned long long* d;
    hipMalloc(&w, 64 * 4096);
    hipMemset(w, 0, 64 * 4096);
    hipMalloc(&out, 256 * 256 * 4);
    hipMalloc(&d, 8);
    const int nl = 64;
    for (int mode = 0; mode < 2; ++mode)
        for (int rep = 0; rep < 2; ++rep) {
            hipMemset(d, 0, 8);
            hipEvent_t e0, e1;
            hipEventCreate(&e0);
            hipEventCreate(&e1);
            hipEventRecord(e0, 0);
            if (mode == 0) hipLaunchKernelGGL(layer_probe<0>, dim3(256), dim3(256), 0, 0, w, nl, out, d);
            else hipLaunchKernelGGL(layer_probe<1>, dim3(256), dim3(256), 0, 0, w, nl, out, d);
            hipEventRecord(e1, 0);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            unsigned long long h = 0;
            hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
            if (rep == 1)
                printf("%s: %.1f TFLOP/s, %.0f cycles per layer per wave (1024 MFMAs = 65536 at peak)\n",
                       mode == 0 ? "mlp_layer (lead groups + relu/bias boundary)" : "same stream, no boundary work",
                       256.0 * 4 * nl * 1024 * 4096 / (ms * 1e-3) / 1e12, (double)h / (256 * 4) / nl);
        }
    return 0;
}
