// Microbenchmark (diagnostic only, round 4): the fp16 hidden layer (mlp_layer_h3, NP = 3 / 4
// products) alone — 256x256, one wave per SIMD, four waves per CU in step (a barrier per layer),
// random fp16 weight planes streamed from a 7-layer footprint (1.75 MiB), random activations.
// Reports TFLOP/s (wall), cycles per layer (s_memtime) against the MFMA-only ideal (128 groups x NP
// MFMAs x 32 cycles) and the clock they imply.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DPROBE_NP=4 tools/probe/h4_probe.hip -o tools/probe/h4_probe_4
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#ifdef PROBE_STAMPS  // per-phase cycles of the layer: 0 preamble, 1 lead groups, 2 middle blocks, 3 last block
__device__ unsigned long long g_ph[4];
#define ANERF_H3_STAMPS g_ph
#endif
#include "../../include/anerf.h"
#include "../../a-nerf_amd/csrc/anerf_device.hpp"
using namespace anerf;
#include "../../a-nerf_amd/csrc/anerf_types.hpp"
#include "../../a-nerf_amd/csrc/anerf_mlp.hpp"

#ifndef PROBE_NP
#define PROBE_NP 4
#endif
constexpr int LAYER_FLOATS = 64 * 16 * 64;  // 64 ring slots x 16 floats x 64 lanes

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
    int es = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int L = 0; L < nl; ++L) {
        const float* wl = w + (size_t)(L % foot) * LAYER_FLOATS;
        const float* wn = w + (size_t)((L + 1) % foot) * LAYER_FLOATS;
        __builtin_amdgcn_s_barrier();
        es = 0;  // (keep the scale exponents bounded over hundreds of layers)
        mlp_layer_h3<8, 8, true, false, PROBE_NP>(acc, acc, h, bias, wl, lane, ring, pre, wn, nullptr, sig, es, -9, 137);
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
    std::uniform_int_distribution<int> um(0, 1023), us(0, 1);
    const int foot = 7;
    // random fp16 pairs with exponents around 2^-1 (w * 2^ew, ew = -9 below: |w| ~ 2^-10)
    std::vector<float> hw((size_t)foot * LAYER_FLOATS);
    for (auto& v : hw) {
        uint32_t lo = (uint32_t)((us(rng) << 15) | (14 << 10) | um(rng));
        uint32_t hi = (uint32_t)((us(rng) << 15) | (14 << 10) | um(rng));
        const uint32_t u = lo | (hi << 16);
        std::memcpy(&v, &u, 4);
    }
    float *w, *out;
    unsigned long long* cyc;
    hipMalloc(&w, hw.size() * 4);
    hipMemcpy(w, hw.data(), hw.size() * 4, hipMemcpyHostToDevice);
    hipMalloc(&out, 256 * 256 * 4);
    hipMalloc(&cyc, 8);
    const int nl = 440, reps = 20;
    const double ideal = 128.0 * PROBE_NP * 32.0;
#ifdef PROBE_STAMPS
    unsigned long long zero[4] = {0, 0, 0, 0};
#endif
    for (int rnd = 0; rnd < 3; ++rnd) {
        hipLaunchKernelGGL(layer_speed, dim3(256), dim3(256), 0, 0, w, nl, foot, out, cyc);
        hipDeviceSynchronize();
        hipMemset(cyc, 0, 8);
#ifdef PROBE_STAMPS
        hipMemcpyToSymbol(HIP_SYMBOL(g_ph), zero, sizeof(zero));
#endif
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
        printf("fp16 layer NP=%d: %.1f TFLOP/s (16-bit MFMA), %.0f cyc/layer (%.1f %% of ideal %.0f), clock %.3f GHz\n", PROBE_NP,
               256.0 * 4 * reps * nl * 128.0 * PROBE_NP * 32768.0 / (ms * 1e-3) / 1e12, cyc_layer, 100.0 * ideal / cyc_layer,
               ideal, cyc_wave / (ms * 1e-3 / reps) / 1e9);
#ifdef PROBE_STAMPS
        unsigned long long ph[4];
        hipMemcpyFromSymbol(ph, HIP_SYMBOL(g_ph), sizeof(ph));
        const double den = 256.0 * 4 * reps * nl;
        printf("  per layer: preamble %.0f, lead groups %.0f (16 groups), middle blocks %.0f (96), last block %.0f (16) cycles\n",
               ph[0] / den, ph[1] / den, ph[2] / den, ph[3] / den);
#endif
    }
    return 0;
}
