// Numerics probe (diagnostic only): what v_mfma_f32_32x32x16_f16 / _bf16 compute for one 32x32x16
// product, D = A B + C, against the exact (double) sum, over operand magnitudes 2^k.  The error is
// reported relative to sum |a b| + |c| of each output (an fp32 pipeline stays at ~2^-24 of that).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <bool BF>
__global__ void mm(const uint16_t* A, const uint16_t* B, const float* C, float* D) {
    const int l = threadIdx.x, h = l >> 5, c = l & 31;
    uint16_t a[8], b[8];
    for (int j = 0; j < 8; ++j) {
        a[j] = A[c * 16 + 8 * h + j];  // A[row = l & 31][k]
        b[j] = B[(8 * h + j) * 32 + c];  // B[k][col = l & 31]
    }
    f32x16 acc;
    for (int r = 0; r < 16; ++r) acc[r] = C[((r & 3) + 8 * (r >> 2) + 4 * h) * 32 + c];
    if constexpr (BF)
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*reinterpret_cast<bf16x8*>(a), *reinterpret_cast<bf16x8*>(b), acc,
                                                     0, 0, 0);
    else
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(*reinterpret_cast<f16x8*>(a), *reinterpret_cast<f16x8*>(b), acc,
                                                    0, 0, 0);
    for (int r = 0; r < 16; ++r) D[((r & 3) + 8 * (r >> 2) + 4 * h) * 32 + c] = acc[r];
}

static uint16_t to_f16(float f) { _Float16 h = (_Float16)f; return *reinterpret_cast<uint16_t*>(&h); }
static float from_f16(uint16_t u) { return (float)*reinterpret_cast<_Float16*>(&u); }
static uint16_t to_bf16(float f) { uint32_t u = *reinterpret_cast<uint32_t*>(&f); return (uint16_t)((u + 0x7fff + ((u >> 16) & 1)) >> 16); }
static float from_bf16(uint16_t b) { uint32_t u = (uint32_t)b << 16; return *reinterpret_cast<float*>(&u); }

int main() {
    uint16_t *dA, *dB;
    float *dC, *dD;
    hipMalloc(&dA, 32 * 16 * 2);
    hipMalloc(&dB, 16 * 32 * 2);
    hipMalloc(&dC, 32 * 32 * 4);
    hipMalloc(&dD, 32 * 32 * 4);
    std::mt19937 g(7);
    std::uniform_real_distribution<float> u(0.5f, 1.0f);
    for (int bf = 0; bf < 2; ++bf)
        for (int mode = 0; mode < 3; ++mode)  // 0: all terms ~ 2^ka 2^kb; 1: + C ~ 2^(ka+kb+4); 2: one large term per dot
            for (int ka = 0; ka <= 15; ka += (bf ? 5 : 1)) {
                const int kb = ka;
                std::vector<uint16_t> A(512), B(512);
                std::vector<float> Af(512), Bf(512), C(1024, 0.0f), D(1024);
                for (int i = 0; i < 512; ++i) {
                    float x = std::ldexp(u(g), ka) * (g() & 1 ? -1.0f : 1.0f);
                    float y = std::ldexp(u(g), kb) * (g() & 1 ? -1.0f : 1.0f);
                    if (mode == 2 && (i % 16) != 0) { x = std::ldexp(x, -8); }
                    A[i] = bf ? to_bf16(x) : to_f16(x);
                    B[i] = bf ? to_bf16(y) : to_f16(y);
                    Af[i] = bf ? from_bf16(A[i]) : from_f16(A[i]);
                    Bf[i] = bf ? from_bf16(B[i]) : from_f16(B[i]);
                }
                if (mode == 1)
                    for (int i = 0; i < 1024; ++i) C[i] = std::ldexp(u(g), ka + kb + 4) * (g() & 1 ? -1.0f : 1.0f);
                hipMemcpy(dA, A.data(), 1024, hipMemcpyHostToDevice);
                hipMemcpy(dB, B.data(), 1024, hipMemcpyHostToDevice);
                hipMemcpy(dC, C.data(), 4096, hipMemcpyHostToDevice);
                if (bf) hipLaunchKernelGGL(mm<true>, dim3(1), dim3(64), 0, 0, dA, dB, dC, dD);
                else hipLaunchKernelGGL(mm<false>, dim3(1), dim3(64), 0, 0, dA, dB, dC, dD);
                hipMemcpy(D.data(), dD, 4096, hipMemcpyDeviceToHost);
                double worst = 0.0;
                for (int i = 0; i < 32; ++i)
                    for (int j = 0; j < 32; ++j) {
                        double s = C[i * 32 + j], sa = std::fabs(C[i * 32 + j]);
                        for (int k = 0; k < 16; ++k) {
                            const double p = (double)Af[i * 16 + k] * Bf[k * 32 + j];
                            s += p;
                            sa += std::fabs(p);
                        }
                        worst = std::max(worst, std::fabs(D[i * 32 + j] - s) / sa);
                    }
                printf("%s mode %d  |a| ~ 2^%2d |b| ~ 2^%2d: max |D - exact| / sum|terms| = %.3e  (log2 %.1f)\n",
                       bf ? "bf16" : "f16 ", mode, ka, kb, worst, worst > 0 ? std::log2(worst) : -99.0);
            }
    return 0;
}
