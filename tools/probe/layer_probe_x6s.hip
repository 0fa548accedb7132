// Microbenchmark (diagnostic only, round 4): the bf16x6 256x256 hidden layer on the two MFMA shapes.
//   x6  — the product's mlp_layer_x6: v_mfma_f32_32x32x16_bf16, lane = sample l & 31, 6 MFMAs per group;
//   x6s — the same layer on v_mfma_f32_16x16x32_bf16 (a 32-sample block = two 16-column blocks,
//         lane l holds samples l & 15 and 16 + (l & 15), rows 16 a + 4 (l >> 4) + i): 12 MFMAs of half
//         the cycles per 3 KiB weight group, the same bytes and the same MFMA cycles per layer.
// MI355X_MICROARCH.md (Matrix cores, DVFS item 7): on random operands the 16x16x32 loop holds a higher
// clock than the 32x32x16 one at equal cycles per FLOP.  This probe measures that on THIS layer, with
// random weights and activations (zeros would hold the clock up and hide it), footprint 1 (L2-hot) and
// 7 layers (one net's hidden set), and checks the x6s layout against a double-precision host product.
#include "../../a-nerf_amd/csrc/anerf_render.hip"

#include <random>

using namespace anerf;

constexpr int LAYER_FLOATS = 128 * 12 * 256 / 4;  // 128 groups x 3 KiB

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// group (ob, a) of the x6s layer: both column blocks c, six products each, small terms first
__device__ __forceinline__ void mfma_x6s(const float (&w)[16], const X6T (&T)[2], f32x16& acc, int a) {
    const bf16x8 w0 = frag_of(w, 0), w1 = frag_of(w, 1), w2 = frag_of(w, 2);
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        const int o = 8 * c + 4 * a;
        f32x4 x = f32x4{acc[o], acc[o + 1], acc[o + 2], acc[o + 3]};
        x = mfma16(w2, T[c].frag(0), x);
        x = mfma16(w1, T[c].frag(1), x);
        x = mfma16(w0, T[c].frag(2), x);
        x = mfma16(w1, T[c].frag(0), x);
        x = mfma16(w0, T[c].frag(1), x);
        x = mfma16(w0, T[c].frag(0), x);
        acc[o] = x[0], acc[o + 1] = x[1], acc[o + 2] = x[2], acc[o + 3] = x[3];
    }
}

#ifndef X6S_NV
#define X6S_NV 2
#endif
__device__ __forceinline__ void x6s_group_schedule() {
#if X6S_NV
    group_schedule<12, 3, 1, X6S_NV>();
#endif
}

// bias in LDS for x6s: [rb][g = lane >> 4][a][i] (8 floats per (rb, g))
template <int RBO, int RBI, bool OUT_SAME>
__device__ __forceinline__ void mlp_layer_x6s(f32x16 (&out)[RBO], f32x16 (&ain)[RBI], f32x16 (&h)[RBI],
                                              const float* __restrict__ bias, const float* __restrict__ wp, int lane,
                                              Ring& ring, bool preloaded, const float* __restrict__ next) {
    static_assert(RBO <= RBI, "x6s layer shape");
    constexpr int NG = 2 * RBO * RBI;
    constexpr int PD = 3;
    constexpr int NQ = 2 * RBO;
    const int g4 = lane >> 4;
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(wp);
    const __amdgpu_buffer_rsrc_t rn = make_rsrc(next ? next : wp);
    auto convert_half = [&](int rb, int half) {
#pragma unroll
        for (int i = 8 * half; i < 8 * half + 8; ++i) h[rb][i] = relu_act(ain[rb][i]);
        if (OUT_SAME && rb < RBO) {
            const f32x4* p = reinterpret_cast<const f32x4*>(bias + (rb * 4 + g4) * 8);
            const f32x4 v0 = p[0], v1 = p[1];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                out[rb][8 * half + e] = v0[e];
                out[rb][8 * half + 4 + e] = v1[e];
            }
        }
    };
    if constexpr (!OUT_SAME) {
#pragma unroll
        for (int rb = 0; rb < RBO; ++rb) out[rb] = f32x16{0};
    }
    const bool has_next = next != nullptr;
    auto prefetch = [&](int g) {
        if (g + PD < NG)
            load_group<12>(ring.v[(g + PD) % 4], rs, lane, g + PD);
        else if (NG % 4 == 0)
            load_group<12>(ring.v[(g + PD) % 4], rn, lane, has_next ? g + PD - NG : NG - 1);
    };
    auto pair_group = [](int p, int q0) { return q0 + (p * (NQ - q0 > 0 ? NQ - q0 : 1)) / 8; };
    if (!preloaded) {
#pragma unroll
        for (int g = 0; g < PD; ++g) load_group<12>(ring.v[g], rs, lane, g);
    }
    convert_half(0, 0);
    convert_half(0, 1);
    X6T T[2], Tn[2];
#pragma unroll
    for (int p = 0; p < 8; ++p) split3_block_pair(h[0], T, p);
    constexpr int QL = NQ > 2 ? 2 : NQ;
#pragma clang loop unroll(full)
    for (int g = 0; g < NQ; ++g) {
        __builtin_amdgcn_sched_barrier(0);
        prefetch(g);
        const int ob = g >> 1, a = g & 1;
        mfma_x6s(ring.v[g % 4], T, out[ob], a);
        if (ob + 1 < RBI && (ob + 1 < RBO || ob == 0)) convert_half(ob + 1, a);
        if (RBI > 1) {
#pragma unroll
            for (int p = 0; p < 8; ++p)
                if (pair_group(p, QL) == (g < QL ? -1 : g) || (g == NQ - 1 && pair_group(p, QL) > g))
                    split3_block_pair(h[1], Tn, p);
        }
        x6s_group_schedule();
    }
#pragma clang loop unroll(full)
    for (int ib = 1; ib < RBI; ++ib) {
        T[0] = Tn[0];
        T[1] = Tn[1];
        const bool conv_next = ib + 1 < RBI && ib + 1 >= (RBO > 2 ? RBO : 2);
        const int q0 = conv_next ? (NQ > 2 ? 2 : NQ) : 0;
#pragma clang loop unroll(full)
        for (int q = 0; q < NQ; ++q) {
            const int ob = q >> 1, a = q & 1;
            const int g = NQ + (ib - 1) * NQ + q;
            __builtin_amdgcn_sched_barrier(0);
            prefetch(g);
            mfma_x6s(ring.v[g % 4], T, out[ob], a);
            if (ib + 1 < RBI) {
                if (conv_next && q < 2) convert_half(ib + 1, q);
#pragma unroll
                for (int p = 0; p < 8; ++p)
                    if (pair_group(p, q0) == q || (q == NQ - 1 && pair_group(p, q0) > q))
                        split3_block_pair(h[ib + 1], Tn, p);
            }
            x6s_group_schedule();
        }
    }
}

// host packing of the x6s layer: group g -> (ob, a, ib); lane l: row 32 ob + 16 a + (l & 15), slot
// (l >> 4, j) -> input column 32 ib + 16 (j >> 2) + 4 (l >> 4) + (j & 3)
std::vector<float> pack_layer_x6s(const float* Wt, int n_out, int ld, int col_off, int n_in) {
    const int RBO = n_out / 32, RBI = n_in / 32, NQ = 2 * RBO;
    const int ng = 2 * RBO * RBI;
    return pack_groups(ng, 12, [&](int g, int sl, int l) {
        const int f = sl >> 2, e = sl & 3;
        int ob, a, ib;
        if (g < NQ) {
            ob = g >> 1, a = g & 1, ib = 0;
        } else {
            const int idx = g - NQ, q = idx % NQ;
            ib = 1 + idx / NQ, ob = q >> 1, a = q & 1;
        }
        const int row = 32 * ob + 16 * a + (l & 15), gq = l >> 4;
        uint32_t bits = 0;
        for (int jj = 0; jj < 2; ++jj) {
            const int j = 2 * e + jj;
            const int col = col_off + 32 * ib + 16 * (j >> 2) + 4 * gq + (j & 3);
            float r = Wt[(size_t)row * ld + col];
            uint16_t v = 0;
            for (int p = 0; p <= f; ++p) {
                v = bf16_rne(r);
                r -= bf16_to_f(v);
            }
            bits |= (uint32_t)v << (16 * jj);
        }
        float o;
        std::memcpy(&o, &bits, 4);
        return o;
    });
}

// ---- correctness: one wave, one layer, X [32 samples][256] -> Y [32][256] = W relu(X) + b
template <bool S>
__global__ __launch_bounds__(64, 1) void check_layer(const float* w, const float* X, const float* b, float* Y) {
    __shared__ __attribute__((aligned(16))) float bias[256];
    const int lane = threadIdx.x;
    for (int i = lane; i < 256; i += 64) {
        if (S) {  // [rb][g][a][i] -> row 32 rb + 16 a + 4 g + i
            const int rb = i / 32, g = (i / 8) % 4, a = (i / 4) % 2, k = i % 4;
            bias[i] = b[32 * rb + 16 * a + 4 * g + k];
        } else {  // (rb * 2 + hh) * 16 + r -> row 32 rb + acc_row(r, hh)
            const int rb = i / 32, hh = (i / 16) % 2, r = i % 16;
            bias[i] = b[32 * rb + acc_row(r, hh)];
        }
    }
    __syncthreads();
    f32x16 acc[8], h[8];
    for (int rb = 0; rb < 8; ++rb)
        for (int r = 0; r < 16; ++r) {
            int smp, row;
            if (S) {
                const int c = r / 8, a = (r / 4) % 2, i = r % 4;
                smp = 16 * c + (lane & 15), row = 32 * rb + 16 * a + 4 * (lane >> 4) + i;
            } else {
                smp = lane & 31, row = 32 * rb + acc_row(r, lane >> 5);
            }
            acc[rb][r] = X[smp * 256 + row];
        }
    Ring ring;
    float sig = 0.0f;
    if (S)
        mlp_layer_x6s<8, 8, true>(acc, acc, h, bias, w, lane, ring, false, nullptr);
    else
        mlp_layer_x6<8, 8, true, false>(acc, acc, h, bias, w, lane, ring, false, nullptr, nullptr, sig);
    for (int rb = 0; rb < 8; ++rb)
        for (int r = 0; r < 16; ++r) {
            int smp, row;
            if (S) {
                const int c = r / 8, a = (r / 4) % 2, i = r % 4;
                smp = 16 * c + (lane & 15), row = 32 * rb + 16 * a + 4 * (lane >> 4) + i;
            } else {
                smp = lane & 31, row = 32 * rb + acc_row(r, lane >> 5);
            }
            Y[smp * 256 + row] = acc[rb][r];
        }
}

// ---- speed: nl layers per wave over a footprint of `foot` weight sets, random activations
__device__ __forceinline__ float hash01(unsigned x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return (float)(x & 0xffffff) * (1.0f / 16777216.0f);
}

template <bool S, bool SYNC = false>
__global__ __launch_bounds__(256, 1) void layer_speed(const float* w, int nl, int foot, float* out,
                                                      unsigned long long* cyc, int copies = 1) {
    __shared__ __attribute__((aligned(16))) float bias[256];
    const int lane = threadIdx.x & 63;
    for (int i = threadIdx.x; i < 256; i += 256) bias[i] = 0.05f * hash01(i * 7 + 3) - 0.02f;
    __syncthreads();
    f32x16 acc[8], h[8];
    for (int rb = 0; rb < 8; ++rb)
        for (int r = 0; r < 16; ++r) acc[rb][r] = 2.0f * hash01(blockIdx.x * 9973 + threadIdx.x * 131 + rb * 16 + r) - 0.8f;
    Ring ring;
    float sig = 0.0f;
    bool pre = false;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int L = 0; L < nl; ++L) {
        // (copies > 1: wave w streams its own copy of the weights, so the CU's four waves share no L1 line)
        const int cw = ((int)threadIdx.x >> 6) % copies;
        const float* wl = w + (size_t)(L % foot + cw * foot) * LAYER_FLOATS;
        const float* wn = w + (size_t)((L + 1) % foot + cw * foot) * LAYER_FLOATS;
        if (SYNC) __builtin_amdgcn_s_barrier();
        if (S)
            mlp_layer_x6s<8, 8, true>(acc, acc, h, bias, wl, lane, ring, pre, wn);
        else
            mlp_layer_x6<8, 8, true, false>(acc, acc, h, bias, wl, lane, ring, pre, wn, nullptr, sig);
        pre = true;
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0;
    for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][15];
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (lane == 0) atomicAdd(cyc, t1 - t0);
}

// ---- bare MFMA loops on random register operands (4 independent accumulators)
template <bool S>
__global__ __launch_bounds__(256, 1) void bare(int iters, float* out, unsigned long long* cyc) {
    const int lane = threadIdx.x & 63;
    unsigned u[8];
    for (int i = 0; i < 8; ++i) u[i] = __builtin_bit_cast(unsigned, 0.5f + hash01(lane * 8 + i + blockIdx.x * 512));
    const bf16x8 a = __builtin_bit_cast(bf16x8, u32x4{u[0], u[1], u[2], u[3]});
    const bf16x8 b = __builtin_bit_cast(bf16x8, u32x4{u[4], u[5], u[6], u[7]});
    float s = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (S) {
        f32x4 c[8];
        for (int k = 0; k < 8; ++k) c[k] = f32x4{0};
        for (int it = 0; it < iters; ++it)
#pragma unroll
            for (int k = 0; k < 8; ++k) c[k] = mfma16(a, b, c[k]);
        for (int k = 0; k < 8; ++k) s += c[k][0];
    } else {
        f32x16 c[4];
        for (int k = 0; k < 4; ++k) c[k] = f32x16{0};
        for (int it = 0; it < iters; ++it)
#pragma unroll
            for (int k = 0; k < 4; ++k) c[k] = mfma_bf16_32x32x16(a, b, c[k]);
        for (int k = 0; k < 4; ++k) s += c[k][0];
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (lane == 0) atomicAdd(cyc, t1 - t0);
}

static float time_launches(void (*launch)(), unsigned long long* dcyc, double* cyc_out, int reps) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    launch();  // warm
    hipDeviceSynchronize();
    hipMemset(dcyc, 0, 8);
    hipEventRecord(e0, 0);
    for (int r = 0; r < reps; ++r) launch();
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    unsigned long long c = 0;
    hipMemcpy(&c, dcyc, 8, hipMemcpyDeviceToHost);
    *cyc_out = (double)c;
    return ms;
}

static float *g_w6, *g_w6s, *g_out;
static unsigned long long* g_cyc;
static int g_nl, g_foot, g_iters;
static void L6() { hipLaunchKernelGGL(layer_speed<false>, dim3(256), dim3(256), 0, 0, g_w6, g_nl, g_foot, g_out, g_cyc); }
static void L6s() { hipLaunchKernelGGL(layer_speed<true>, dim3(256), dim3(256), 0, 0, g_w6s, g_nl, g_foot, g_out, g_cyc); }
static void L6sync() { hipLaunchKernelGGL((layer_speed<false, true>), dim3(256), dim3(256), 0, 0, g_w6, g_nl, g_foot, g_out, g_cyc); }
static int g_copies = 1;
static void L6c() { hipLaunchKernelGGL((layer_speed<false, true>), dim3(256), dim3(256), 0, 0, g_w6, g_nl, g_foot, g_out, g_cyc, g_copies); }
static void B32() { hipLaunchKernelGGL(bare<false>, dim3(256), dim3(256), 0, 0, g_iters, g_out, g_cyc); }
static void B16() { hipLaunchKernelGGL(bare<true>, dim3(256), dim3(256), 0, 0, g_iters, g_out, g_cyc); }

int main() {
    std::mt19937 rng(1234);
    std::uniform_real_distribution<float> uw(-0.0625f, 0.0625f), ux(-1.0f, 1.5f);
    // ---- correctness of both layouts against a double-precision product
    {
        std::vector<float> Wt(256 * 256), X(32 * 256), b(256);
        for (auto& v : Wt) v = uw(rng);
        for (auto& v : X) v = ux(rng);
        for (auto& v : b) v = 0.1f * uw(rng);
        for (int S = 0; S < 2; ++S) {
            std::vector<float> pk = S ? pack_layer_x6s(Wt.data(), 256, 256, 0, 256) : pack_layer_x6(Wt.data(), 256, 256, 0, 256);
            float *dw, *dx, *db, *dy;
            hipMalloc(&dw, pk.size() * 4);
            hipMalloc(&dx, X.size() * 4);
            hipMalloc(&db, 256 * 4);
            hipMalloc(&dy, X.size() * 4);
            hipMemcpy(dw, pk.data(), pk.size() * 4, hipMemcpyHostToDevice);
            hipMemcpy(dx, X.data(), X.size() * 4, hipMemcpyHostToDevice);
            hipMemcpy(db, b.data(), 256 * 4, hipMemcpyHostToDevice);
            if (S)
                hipLaunchKernelGGL(check_layer<true>, dim3(1), dim3(64), 0, 0, dw, dx, db, dy);
            else
                hipLaunchKernelGGL(check_layer<false>, dim3(1), dim3(64), 0, 0, dw, dx, db, dy);
            std::vector<float> Y(X.size());
            hipMemcpy(Y.data(), dy, Y.size() * 4, hipMemcpyDeviceToHost);
            double maxerr = 0, maxref = 0;
            for (int s = 0; s < 32; ++s)
                for (int r = 0; r < 256; ++r) {
                    double acc = b[r];
                    for (int k = 0; k < 256; ++k) acc += (double)Wt[r * 256 + k] * std::max(0.0, (double)X[s * 256 + k]);
                    maxerr = std::max(maxerr, std::fabs(acc - Y[s * 256 + r]));
                    maxref = std::max(maxref, std::fabs(acc));
                }
            printf("check %s: max |err| %.3g (max |y| %.3g) %s\n", S ? "x6s (16x16x32)" : "x6  (32x32x16)", maxerr, maxref,
                   maxerr < 2e-6 * maxref ? "OK" : "FAIL");
            hipFree(dw), hipFree(dx), hipFree(db), hipFree(dy);
        }
    }
    // ---- speed
    const int maxfoot = 12;
    std::vector<float> Wt(256 * 256);
    std::vector<float> h6, h6s;
    for (int L = 0; L < maxfoot; ++L) {
        for (auto& v : Wt) v = uw(rng);
        auto a = pack_layer_x6(Wt.data(), 256, 256, 0, 256);
        auto c = pack_layer_x6s(Wt.data(), 256, 256, 0, 256);
        h6.insert(h6.end(), a.begin(), a.end());
        h6s.insert(h6s.end(), c.begin(), c.end());
    }
    hipMalloc(&g_w6, h6.size() * 4);
    hipMalloc(&g_w6s, h6s.size() * 4);
    hipMemcpy(g_w6, h6.data(), h6.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(g_w6s, h6s.data(), h6s.size() * 4, hipMemcpyHostToDevice);
    hipMalloc(&g_out, 256 * 256 * 4);
    hipMalloc(&g_cyc, 8);
    g_iters = 20000;
    for (int round = 0; round < 2; ++round) {
        for (int S = 0; S < 2; ++S) {
            double cyc;
            const int reps = 40;
            const float ms = time_launches(S ? B16 : B32, g_cyc, &cyc, reps);
            const double nmfma = 256.0 * 4 * reps * g_iters * (S ? 8 : 4);
            const double flop = nmfma * (S ? 16384.0 : 32768.0);
            const double cyc_per = cyc / (256.0 * 4 * reps) / (g_iters * (S ? 8 : 4));
            printf("bare %s: %.1f TFLOP/s, %.2f cyc/MFMA, clock %.2f GHz\n", S ? "16x16x32" : "32x32x16", flop / (ms * 1e-3) / 1e12,
                   cyc_per, cyc / (256.0 * 4 * reps) / (ms * 1e-3 / reps) / 1e9);
        }
        for (int foot : {1, 7, 9, 10, 11, 12}) {
            g_foot = foot;
            g_nl = 440;
            for (int S = 0; S < 3; ++S) {
                if (S == 1 && foot != 7) continue;
                double cyc;
                const int reps = 10;
                const float ms = time_launches(S == 1 ? L6s : (S == 2 ? L6sync : L6), g_cyc, &cyc, reps);
                const double flop = 256.0 * 4 * reps * g_nl * 768.0 * 32768.0;
                const double cyc_layer = cyc / (256.0 * 4 * reps) / g_nl;
                printf("layer %s foot %2d (%.2f MiB): %.1f TFLOP/s (bf16 MFMA), %.0f cyc/layer (ideal 24576: %.1f %%), clock %.2f GHz\n",
                       S == 1 ? "x6s    " : (S == 2 ? "x6 sync" : "x6     "), foot, foot * 0.375, flop / (ms * 1e-3) / 1e12, cyc_layer, 100.0 * 24576 / cyc_layer,
                       cyc / (256.0 * 4 * reps) / (ms * 1e-3 / reps) / 1e9);
            }
        }
    }
    // L1 sharing: the four waves of a CU on one weight stream (copies 1) or on four (copies 4), in step
    for (int rnd = 0; rnd < 2; ++rnd)
        for (int cp : {1, 4}) {
            g_foot = 2;
            g_copies = cp;
            g_nl = 440;
            double cyc;
            const int reps = 10;
            const float ms = time_launches(L6c, g_cyc, &cyc, reps);
            const double flop = 256.0 * 4 * reps * g_nl * 768.0 * 32768.0;
            const double cyc_layer = cyc / (256.0 * 4 * reps) / g_nl;
            printf("layer x6 sync, 2 layers x %d copies (%s): %.1f TFLOP/s, %.0f cyc/layer (%.1f %%), clock %.2f GHz\n", cp,
                   cp == 1 ? "L1-shared" : "no L1 sharing", flop / (ms * 1e-3) / 1e12, cyc_layer, 100.0 * 24576 / cyc_layer,
                   cyc / (256.0 * 4 * reps) / (ms * 1e-3 / reps) / 1e9);
        }
    return 0;
}
