// Probe (diagnostic only, round 5): v_mfma_scale_f32_32x32x64_f8f6f4 with e4m3 A/B -- which lane holds
// which k (checked against a CPU product for candidate maps, exact small-integer data), the block-scale
// semantics (E8M0 scale operand), and the issue rate next to v_mfma_f32_32x32x16_f16.
//   hipcc --offload-arch=gfx950 -O3 tools/probe/mfma_f8_probe.hip -o tools/probe/mfma_f8_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

__global__ void one(const i32x8* a, const i32x8* b, f32x16* c, int sa, int sb) {
    const int l = threadIdx.x;
    f32x16 acc = c[l];  // (the caller's accumulator: zero, or large values whose low bits must survive)
    acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a[l], b[l], acc, 0, 0, 0, sa, 0, sb);
    c[l] = acc;
}

template <int MODE>  // 0: fp8 scaled 32x32x64, 1: f16 32x32x16
__global__ __launch_bounds__(256, 1) void rate(const i32x8* a, const i32x8* b, f32x16* c, int n,
                                               unsigned long long* cyc) {
    const int l = threadIdx.x & 63;
    i32x8 x = a[l], y = b[l];
    f32x16 acc[4] = {};
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if constexpr (MODE == 0)
                acc[k] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(x, y, acc[k], 0, 0, 0, 127, 0, 127);
            else
                acc[k] = __builtin_amdgcn_mfma_f32_32x32x16_f16(
                    __builtin_bit_cast(f16x8, (int __attribute__((ext_vector_type(4)))){x[0], x[1], x[2], x[3]}),
                    __builtin_bit_cast(f16x8, (int __attribute__((ext_vector_type(4)))){y[0], y[1], y[2], y[3]}),
                    acc[k], 0, 0, 0);
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    c[blockIdx.x * 256 + threadIdx.x] = acc[0] + acc[1] + acc[2] + acc[3];
    if (threadIdx.x == 0) atomicAdd(cyc, t1 - t0);
}

__global__ void cvt(unsigned* o, float s) {
    typedef short s16x2 __attribute__((ext_vector_type(2)));
    const s16x2 v = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(__builtin_bit_cast(s16x2, 0u), 1.0f, 0.0078125f, s, false);
    o[0] = __builtin_bit_cast(unsigned, v);
    o[1] = __builtin_amdgcn_cvt_pk_fp8_f32(1.0f, 0.0078125f, 0, false);
    o[2] = __builtin_amdgcn_cvt_pk_fp8_f32(1.0f, 0.0078125f, 0x12345678, true);
}

static float e4m3(unsigned char v) {
    const int s = v >> 7, e = (v >> 3) & 15, m = v & 7;
    float x = e == 0 ? std::ldexp((float)m / 8.0f, -6) : std::ldexp(1.0f + m / 8.0f, e - 7);
    return s ? -x : x;
}

int main() {
    std::mt19937 rng(3);
    std::uniform_int_distribution<int> ue(4, 10), um(0, 7), us(0, 1);
    std::vector<unsigned char> A(64 * 32), B(64 * 32);  // [lane][byte]
    for (auto& v : A) v = (unsigned char)((us(rng) << 7) | (ue(rng) << 3) | um(rng));
    for (auto& v : B) v = (unsigned char)((us(rng) << 7) | (ue(rng) << 3) | um(rng));
    i32x8 *da, *db;
    f32x16* dc;
    unsigned long long* cyc;
    hipMalloc(&da, 64 * 32);
    hipMalloc(&db, 64 * 32);
    hipMalloc(&dc, 256 * 256 * 64);
    hipMalloc(&cyc, 8);
    hipMemcpy(da, A.data(), 64 * 32, hipMemcpyHostToDevice);
    hipMemcpy(db, B.data(), 64 * 32, hipMemcpyHostToDevice);
    // candidate k maps: lane half h, byte t -> k
    auto kmap = [](int map, int h, int t) {
        if (map == 0) return 32 * h + t;                       // contiguous halves
        if (map == 1) return 16 * (t / 8) + 8 * h + (t % 8);   // 8-byte runs interleaved by half
        return 32 * (t / 16) + 16 * h + (t % 16);               // 16-byte runs interleaved by half
    };
    for (int sa : {127, 119, 100}) {
        // sa 100: products ~2^-27 of the accumulator's 1000-ish values (the x1 w1 term's place in fp16x4): is the
        // accumulator kept to fp32 (the error then ~ulp(1000) = 6e-5) or truncated to the dot product's width?
        std::vector<float> C0(64 * 16, 0.0f);
        if (sa == 100)
            for (int i = 0; i < 64 * 16; ++i) C0[i] = 1000.0f + (float)i * 0.0001220703125f;
        hipMemcpy(dc, C0.data(), 64 * 64, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(one, dim3(1), dim3(64), 0, 0, da, db, dc, sa, 127);
        std::vector<float> C(64 * 16);
        hipMemcpy(C.data(), dc, 64 * 64, hipMemcpyDeviceToHost);
        for (int map = 0; map < 3; ++map) {
            double maxerr = 0, maxref = 0;
            for (int l = 0; l < 64; ++l)
                for (int r = 0; r < 16; ++r) {
                    const int col = l & 31, row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
                    double ref = 0;
                    for (int h = 0; h < 2; ++h)
                        for (int t = 0; t < 32; ++t) {
                            (void)kmap(map, h, t);
                            // A: lane (row, h) byte t; B: lane (col, h) byte t, same k for both
                            ref += (double)e4m3(A[(row + 32 * h) * 32 + t]) * (double)e4m3(B[(col + 32 * h) * 32 + t]);
                        }
                    ref *= std::ldexp(1.0, sa - 127);
                    ref += (double)C0[l * 16 + r];
                    maxerr = std::fmax(maxerr, std::fabs(ref - C[l * 16 + r]));
                    maxref = std::fmax(maxref, std::fabs(ref));
                }
            printf("scale_a %d, same-slot pairing (map %d irrelevant when A and B share it): max |gpu - cpu| %.3e "
                   "(max |ref| %.3e)\n", sa, map, maxerr, maxref);
            break;
        }
    }
    {
        unsigned* o;
        hipMalloc(&o, 12);
        hipLaunchKernelGGL(cvt, dim3(1), dim3(1), 0, 0, o, 256.0f);
        unsigned h[3];
        hipMemcpy(h, o, 12, hipMemcpyDeviceToHost);
        printf("cvt_scalef32_pk_fp8_f32(1.0, 2^-7, scale 256) -> bytes %02x %02x = %g %g (x * 256 would be 256, 2; x / 256: "
               "2^-8, 2^-15)\n", h[0] & 255, (h[0] >> 8) & 255, e4m3(h[0] & 255), e4m3((h[0] >> 8) & 255));
        printf("cvt_pk_fp8_f32(1.0, 2^-7) -> %08x (%g %g); word_sel 1 into 0x12345678 -> %08x\n", h[1],
               e4m3(h[1] & 255), e4m3((h[1] >> 8) & 255), h[2]);
    }
    for (int mode = 0; mode < 2; ++mode) {
        const int n = 2000;
        hipMemset(cyc, 0, 8);
        if (mode == 0) hipLaunchKernelGGL(rate<0>, dim3(256), dim3(256), 0, 0, da, db, dc, n, cyc);
        else hipLaunchKernelGGL(rate<1>, dim3(256), dim3(256), 0, 0, da, db, dc, n, cyc);
        hipDeviceSynchronize();
        unsigned long long c = 0;
        hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
        printf("%s: %.1f cycles per MFMA (one wave per SIMD)\n", mode == 0 ? "v_mfma_scale_f32_32x32x64_f8f6f4 e4m3" :
               "v_mfma_f32_32x32x16_f16", (double)c / 256.0 / (4.0 * n));
    }
    return 0;
}
