// Microbenchmark (diagnostic only, round 4): what the power-limited clock pays for in the bf16x6 hidden
// layer.  mlp_layer_x6 (256x256, one wave per SIMD, four waves per CU in step, random weights and
// activations) built three ways with ANERF_X6_PROBE (anerf_mlp.hpp):
//   0 — the product layer: weight groups streamed from a 7-layer (2.6 MiB) footprint;
//   1 — no weight loads (the ring keeps its first contents);
//   3 — loads from a 4-group footprint (L1-resident: no L2 traffic, the full L1 -> VGPR traffic).
// Reports TFLOP/s (wall), cycles per layer (s_memtime) and the clock they imply.
//   hipcc --offload-arch=gfx950 -O3 -DANERF_X6_PROBE=N tools/probe/power_probe.hip -o tools/probe/power_probe_N
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "../../include/anerf.h"
#include "../../a-nerf_amd/csrc/anerf_device.hpp"
using namespace anerf;
#include "../../a-nerf_amd/csrc/anerf_types.hpp"
#include "../../a-nerf_amd/csrc/anerf_mlp.hpp"

constexpr int LAYER_FLOATS = 128 * 12 * 256 / 4;  // 128 groups x 3 KiB

__device__ __forceinline__ float hash01(unsigned x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return (float)(x & 0xffffff) * (1.0f / 16777216.0f);
}

__global__ __launch_bounds__(256, 1) void layer_speed(const float* w, int nl, int foot, float* out,
                                                      unsigned long long* cyc) {
    __shared__ __attribute__((aligned(16))) float bias[512];
    const int lane = threadIdx.x & 63;
    for (int i = threadIdx.x; i < 512; i += 256) bias[i] = 0.05f * hash01(i * 7 + 3) - 0.02f;
    __syncthreads();
    f32x16 acc[8], h[8];
    for (int rb = 0; rb < 8; ++rb)
        for (int r = 0; r < 16; ++r) acc[rb][r] = 2.0f * hash01(blockIdx.x * 9973 + threadIdx.x * 131 + rb * 16 + r) - 0.8f;
    Ring ring;
    float sig = 0.0f;
    bool pre = false;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int L = 0; L < nl; ++L) {
        const float* wl = w + (size_t)(L % foot) * LAYER_FLOATS;
        const float* wn = w + (size_t)((L + 1) % foot) * LAYER_FLOATS;
        __builtin_amdgcn_s_barrier();
        mlp_layer_x6<8, 8, true, false>(acc, acc, h, bias, wl, lane, ring, pre, wn, nullptr, sig);
        pre = true;
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0;
    for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][15];
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (lane == 0) atomicAdd(cyc, t1 - t0);
}

int main() {
    std::mt19937 rng(7);
    std::uniform_real_distribution<float> uw(-0.0625f, 0.0625f);
    const int foot = 7;
    // random weights as bf16 planes (w0, w1, w2 of a random float, truncation split: never NaN / inf)
    std::vector<float> hw((size_t)foot * LAYER_FLOATS);
    for (size_t i = 0; i < hw.size(); i += 12)
        for (int l = 0; l < 4; ++l) {
            uint32_t p[3] = {0, 0, 0};
            for (int half = 0; half < 2; ++half) {
                float v = uw(rng);
                for (int f = 0; f < 3; ++f) {
                    uint32_t u;
                    std::memcpy(&u, &v, 4);
                    const uint32_t hi = u & 0xffff0000u;
                    float hf;
                    std::memcpy(&hf, &hi, 4);
                    p[f] |= (hi >> 16) << (16 * half);
                    v -= hf;
                }
            }
            for (int f = 0; f < 3; ++f) std::memcpy(&hw[i + 4 * f + l], &p[f], 4);  // (layout irrelevant here)
        }
    float *w, *out;
    unsigned long long* cyc;
    hipMalloc(&w, hw.size() * 4);
    hipMemcpy(w, hw.data(), hw.size() * 4, hipMemcpyHostToDevice);
    hipMalloc(&out, 256 * 256 * 4);
    hipMalloc(&cyc, 8);
    const int nl = 440, reps = 20;
    for (int rnd = 0; rnd < 3; ++rnd) {
        hipLaunchKernelGGL(layer_speed, dim3(256), dim3(256), 0, 0, w, nl, foot, out, cyc);
        hipDeviceSynchronize();
        hipMemset(cyc, 0, 8);
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        hipEventRecord(e0, 0);
        for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(layer_speed, dim3(256), dim3(256), 0, 0, w, nl, foot, out, cyc);
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        unsigned long long c = 0;
        hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
        const double cyc_wave = (double)c / (256.0 * 4 * reps), cyc_layer = cyc_wave / nl;
        printf("ANERF_X6_PROBE=%d: %.1f TFLOP/s, %.0f cyc/layer (%.1f %% of 24576), clock %.3f GHz\n", ANERF_X6_PROBE,
               256.0 * 4 * reps * nl * 768.0 * 32768.0 / (ms * 1e-3) / 1e12, cyc_layer, 100.0 * 24576 / cyc_layer,
               cyc_wave / (ms * 1e-3 / reps) / 1e9);
    }
    return 0;
}
