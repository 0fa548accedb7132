// anerf_device.hpp — device helpers of the MI355X A-NeRF render path (gfx950 / CDNA4).
//
// Numerics follow what the reference's torch CPU ops compute (SURVEY §8a hazards), so the
// GPU path and the CPU oracle agree to float rounding:
//   * torch.linspace(0,1,n) float32: step rounded to float, values in double;
//   * torch bmm of 4x4 @ [p;1] and torch.norm are fma chains;
//   * torch.sum(float32) is a cascade with 8-wide vector accumulators (rows >= 8) or the
//     4-way scalar ILP path (short or strided rows); cumprod / cumsum accumulate in double.
// The TU is compiled with -ffp-contract=off: every other mul/add is separately rounded.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

namespace anerf {

// ------------------------------------------------------------------ MFMA
// v_mfma_f32_32x32x2_f32: D[i][j] = sum_k A[i][k] B[k][j] + C; lane l supplies A[l&31][l>>5] and
// B[l>>5][l&31]; D row = (r&3) + 8(r>>2) + 4(l>>5), col = l&31 for register r.
__device__ __forceinline__ f32x16 mfma_f32_32x32x2(float a, float b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// v_mfma_f32_32x32x16_bf16: lane l supplies A[l&31][8(l>>5) + j] and B[8(l>>5) + j][l&31], j = 0..7;
// same C/D layout as the f32 form.  Products of bf16 are exact in the f32 accumulation.
__device__ __forceinline__ f32x16 mfma_bf16_32x32x16(bf16x8 a, bf16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
// bf16x3 product: a b ~= a_hi b_hi + a_hi b_lo + a_lo b_hi (the dropped a_lo b_lo is 2^-16 smaller),
// small terms first
__device__ __forceinline__ f32x16 mfma_x3(bf16x8 ah, bf16x8 al, bf16x8 bh, bf16x8 bl, f32x16 c) {
    c = mfma_bf16_32x32x16(al, bh, c);
    c = mfma_bf16_32x32x16(ah, bl, c);
    return mfma_bf16_32x32x16(ah, bh, c);
}

// output row (within a 32-row block) held by register r of lane-half h
__host__ __device__ constexpr int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// ------------------------------------------------------------------ torch-exact scalar helpers
__device__ __forceinline__ float torch_linspace01(int i, int n) {
    if (n == 1) return 0.0f;
    float step = 1.0f / (float)(n - 1);
    return (i < n / 2) ? (float)((double)step * i) : (float)(1.0 - (double)step * (n - 1 - i));
}

// sample_from_lineseg's z at t (core/utils/ray_utils.py:223-226): near (1 - t) + far t, or with
// lindisp 1 / (1/near (1 - t) + 1/far t) — torch's float32 operations in its order (correctly rounded
// divisions; near = 0 gives inf and the IEEE results torch gives)
__host__ __device__ __forceinline__ float lineseg_z(float nr, float fr, float t, bool lindisp) {
    if (!lindisp) return nr * (1.0f - t) + fr * t;
    return 1.0f / ((1.0f / nr) * (1.0f - t) + (1.0f / fr) * t);
}

__device__ __forceinline__ float norm3(float a, float b, float c) { return sqrtf(fmaf(c, c, fmaf(b, b, a * a))); }
__device__ __forceinline__ float norm2(float a, float b) { return sqrtf(fmaf(b, b, a * a)); }
// Branch-free sin/cos (ocml's sincosf branches to a Payne-Hanek path for large arguments, which
// splits the MFMA scheduling regions the encoding is interleaved into).  Cody-Waite reduction by
// pi/2 in three fma steps (exact for |x| < 2^14 * pi/2; the encoder's arguments are distances to
// joints times 2^t, t < 10) and minimax polynomials on [-pi/4, pi/4]: within 2 ulp of sinf/cosf.
__device__ __forceinline__ void sincos_rr(float x, float& s, float& c) {
    const float k = __builtin_rintf(x * 0.636619772f);
    float r = fmaf(-k, 1.57079637e+00f, x);
    r = fmaf(-k, -4.37113883e-08f, r);
    r = fmaf(-k, -1.71512451e-15f, r);
    const float r2 = r * r;
    float ps = fmaf(r2, -1.95152959e-4f, 8.33216087e-3f);
    ps = fmaf(r2, ps, -1.66666546e-1f);
    ps = fmaf(r2 * r, ps, r);
    float pc = fmaf(r2, 2.44331571e-5f, -1.38873163e-3f);
    pc = fmaf(r2, pc, 4.16666457e-2f);
    pc = fmaf(r2 * r2, pc, fmaf(-0.5f, r2, 1.0f));
    const int q = (int)k;
    const float a = (q & 1) ? pc : ps;
    const float b = (q & 1) ? ps : pc;
    s = (q & 2) ? -a : a;
    c = ((q + 1) & 2) ? -b : b;
}

__device__ __forceinline__ float sigmoid(float x) { return 1.0f / (1.0f + expf(-x)); }
// alpha = 1 - exp(-x) of raw2outputs (nerf.py:186-187) for x = act(sigma) * delta in float32, with exp
// rounded to nearest like the CPU reference's: OCML's expf (<= 1 ulp) returned 1.0 for exp(-4.09e-8),
// whose nearest float is 1 - 2^-24, and on a near-empty ray that one quantum IS the ray's alpha and
// its disp (hazard H12, tests/golden/h12_nearempty_c5.npz).  exp in double, rounded once to float.
__device__ __forceinline__ float alpha_of(float x) { return 1.0f - (float)exp(-(double)x); }
// torch.relu keeps NaN
__device__ __forceinline__ float relu(float x) { return x < 0.0f ? 0.0f : x; }
// MLP activation relu in one VALU op: signed-integer max of the bit pattern maps every float with
// the sign bit set to +0 and keeps the rest (incl. +NaN, which is what the GPU generates and what
// the host NaN fill produces).  Differs from relu only in -0 -> +0 and -NaN -> 0.
// x if m else +0.0, as an integer AND (never turned into a branch; free beside f32 MFMAs)
__device__ __forceinline__ float mask_f(float x, bool m) {
    return __builtin_bit_cast(float, __builtin_bit_cast(int, x) & -(int)m);
}
__device__ __forceinline__ float relu_act(float x) {
    return __builtin_bit_cast(float, max(__builtin_bit_cast(int, x), 0));
}

// numpy pairwise float32 sum (np.nanmean of get_near_far_in_cylinder, ray_utils.py:332)
__device__ inline float np_leaf_sum(const float* a, int64_t n) {
    if (n < 8) {
        float res = 0.0f;
        for (int64_t i = 0; i < n; ++i) res += a[i];
        return res;
    }
    float r0 = a[0], r1 = a[1], r2 = a[2], r3 = a[3], r4 = a[4], r5 = a[5], r6 = a[6], r7 = a[7];
    int64_t i;
    for (i = 8; i < n - (n % 8); i += 8) {
        r0 += a[i + 0]; r1 += a[i + 1]; r2 += a[i + 2]; r3 += a[i + 3];
        r4 += a[i + 4]; r5 += a[i + 5]; r6 += a[i + 6]; r7 += a[i + 7];
    }
    float res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
    for (; i < n; ++i) res += a[i];
    return res;
}

__device__ inline float np_pairwise_sum(const float* a, int64_t n) {
    // post-order walk of numpy's split tree with explicit stacks
    int64_t node_off[64], node_n[64];
    int node_exp[64];
    float vals[64];
    int ns = 0, vs = 0;
    node_off[0] = 0; node_n[0] = n; node_exp[0] = 0; ns = 1;
    while (ns > 0) {
        --ns;
        int64_t off = node_off[ns], cnt = node_n[ns];
        int ex = node_exp[ns];
        if (cnt <= 128) {
            vals[vs++] = np_leaf_sum(a + off, cnt);
        } else if (!ex) {
            int64_t n2 = cnt / 2;
            n2 -= n2 % 8;
            node_off[ns] = off; node_n[ns] = cnt; node_exp[ns] = 1; ++ns;
            node_off[ns] = off + n2; node_n[ns] = cnt - n2; node_exp[ns] = 0; ++ns;
            node_off[ns] = off; node_n[ns] = n2; node_exp[ns] = 0; ++ns;
        } else {
            float r = vals[--vs];
            float l = vals[--vs];
            vals[vs++] = l + r;
        }
    }
    return vals[0];
}

// The same tree split for a workgroup: the leaves (<= 128 elements, left to right) are listed once,
// summed by many threads, then combined in the tree's order.  np_pairwise_leaves returns the leaf
// count, or -1 when there are more than `cap`.  st_off / st_n: [64] walk stacks the caller provides (LDS: a
// private array indexed at run time would live in scratch, ~1 us per access).
__device__ inline int np_pairwise_leaves(int64_t n, int* off, int* cnt, int cap, int* st_off, int* st_n) {
    int ns = 1, nl = 0;
    st_off[0] = 0; st_n[0] = (int)n;
    while (ns > 0) {
        --ns;
        const int o = st_off[ns], c = st_n[ns];
        if (c <= 128) {
            if (nl == cap) return -1;
            off[nl] = o; cnt[nl] = c; ++nl;
        } else {
            int n2 = c / 2;
            n2 -= n2 % 8;
            st_off[ns] = o + n2; st_n[ns] = c - n2; ++ns;   // right half after the left one
            st_off[ns] = o; st_n[ns] = n2; ++ns;
        }
    }
    return nl;
}

// np_pairwise_sum given the leaf sums in left-to-right order; node_n / node_exp / vals: [64] caller stacks (LDS)
__device__ inline float np_pairwise_combine(const float* leaf, int64_t n, int* node_n, int* node_exp, float* vals) {
    int ns = 1, vs = 0, k = 0;
    node_n[0] = (int)n; node_exp[0] = 0;
    while (ns > 0) {
        --ns;
        const int cnt = node_n[ns];
        if (cnt <= 128) {
            vals[vs++] = leaf[k++];
        } else if (!node_exp[ns]) {
            int n2 = cnt / 2;
            n2 -= n2 % 8;
            node_exp[ns] = 1; ++ns;
            node_n[ns] = cnt - n2; node_exp[ns] = 0; ++ns;
            node_n[ns] = n2; node_exp[ns] = 0; ++ns;
        } else {
            const float r = vals[--vs];
            const float l = vals[--vs];
            vals[vs++] = l + r;
        }
    }
    return vals[0];
}

// ---- torch CPU float32 sum (aten SumKernel cascade_sum; see oracle/anerf_oracle.c) ----
__device__ __forceinline__ int ceil_log2_i64(int64_t x) {
    int r = 0;
    while (((int64_t)1 << r) < x) ++r;
    return r;
}

// row_sum<ilp=4> over n elements of WIDTH lanes each; element e lane l at x[(e*WIDTH + l)*xs]
template <int WIDTH>
__device__ inline void torch_row_sum(const float* x, int64_t xs, int64_t n, float* out) {
    const int64_t size = n / 4;
    int lp = ceil_log2_i64(size) / 4;
    if (lp < 4) lp = 4;
    const int64_t step = (int64_t)1 << lp, mask = step - 1;
    float acc[4][4][WIDTH];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int l = 0; l < WIDTH; ++l) acc[j][k][l] = 0.0f;
    int64_t i = 0;
    while (i + step <= size) {
        for (int64_t jj = 0; jj < step; ++jj, ++i)
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int l = 0; l < WIDTH; ++l) acc[0][k][l] += x[((4 * i + k) * WIDTH + l) * xs];
#pragma unroll
        for (int j = 1; j < 4; ++j) {
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int l = 0; l < WIDTH; ++l) {
                    acc[j][k][l] += acc[j - 1][k][l];
                    acc[j - 1][k][l] = 0.0f;
                }
            if ((i & (mask << (j * lp))) != 0) break;
        }
    }
    for (; i < size; ++i)
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int l = 0; l < WIDTH; ++l) acc[0][k][l] += x[((4 * i + k) * WIDTH + l) * xs];
#pragma unroll
    for (int j = 1; j < 4; ++j)
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int l = 0; l < WIDTH; ++l) acc[0][k][l] += acc[j][k][l];
    for (int64_t e = size * 4; e < n; ++e)
#pragma unroll
        for (int l = 0; l < WIDTH; ++l) acc[0][0][l] += x[(e * WIDTH + l) * xs];
#pragma unroll
    for (int k = 1; k < 4; ++k)
#pragma unroll
        for (int l = 0; l < WIDTH; ++l) acc[0][0][l] += acc[0][k][l];
#pragma unroll
    for (int l = 0; l < WIDTH; ++l) out[l] = acc[0][0][l];
}

// torch.sum of a contiguous float32 row
__device__ inline float torch_sum(const float* x, int64_t n) {
    if (n >= 8) {
        float r[8];
        const int64_t nv = n / 8;
        torch_row_sum<8>(x, 1, nv, r);
        float fin = 0.0f;
        for (int64_t k = nv * 8; k < n; ++k) fin += x[k];
#pragma unroll
        for (int l = 0; l < 8; ++l) fin += r[l];
        return fin;
    }
    float r1[1];
    torch_row_sum<1>(x, 1, n, r1);
    return r1[0];
}

// torch.sum over a non-inner dim with stride xs (e.g. (N,S,3).sum(-2))
__device__ inline float torch_sum_strided(const float* x, int64_t xs, int64_t n) {
    float r1[1];
    torch_row_sum<1>(x, xs, n, r1);
    return r1[0];
}

// ------------------------------------------------------------------ geometry / encoding
// q = S[0:3, :] @ [p; 1] as torch's bmm computes it (fma chain, k ascending)
__device__ __forceinline__ void joint_local(const float* S, float px, float py, float pz, float& qx, float& qy,
                                            float& qz) {
    qx = fmaf(S[3], 1.0f, fmaf(S[2], pz, fmaf(S[1], py, S[0] * px)));
    qy = fmaf(S[7], 1.0f, fmaf(S[6], pz, fmaf(S[5], py, S[4] * px)));
    qz = fmaf(S[11], 1.0f, fmaf(S[10], pz, fmaf(S[9], py, S[8] * px)));
}

// rotated ray direction R_j d (transform_batch_rays, encoders.py:25-37)
__device__ __forceinline__ void joint_rot(const float* S, float dx, float dy, float dz, float& ex, float& ey,
                                          float& ez) {
    ex = fmaf(S[2], dz, fmaf(S[1], dy, S[0] * dx));
    ey = fmaf(S[6], dz, fmaf(S[5], dy, S[4] * dx));
    ez = fmaf(S[10], dz, fmaf(S[9], dy, S[8] * dx));
}

// cutoff window w = 1 - sigmoid(tau (dist - c))  (cutoff_embedder.py:139-145)
__device__ __forceinline__ float cutoff_w(float tau, float dist, float c) { return 1.0f - sigmoid(tau * (dist - c)); }

}  // namespace anerf
