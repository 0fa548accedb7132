// anerf_render.hip — MI355X (gfx950) render path of A-NeRF behind the C ABI in include/anerf.h.
//
// One fused kernel renders a group of R rays per 256-thread workgroup (4 waves, one per SIMD):
//   coarse z (linspace) -> per-sample skeleton-relative encoding generated IN REGISTERS as the
//   MFMA B operand -> 8x256 MLP on v_mfma_f32_32x32x2_f32 with activations resident in the
//   accumulator/VGPR file across layers (the transposed product out^T = W^T in^T keeps each
//   layer's accumulator layout directly usable as the next layer's B operand; weights are
//   packed on the host in that permuted k order) -> alpha / rgb heads on the VALU ->
//   compositing + sample_pdf + merge-sort per ray in LDS -> fine pass over all S+I samples.
// The view layer is factorised: its per-sample direction input dv = T_k(e_jc) * w'_j is
// split into a per-ray matrix G[j][n] (computed once per ray in LDS) and the per-sample cutoff
// weights w'_j, so the per-sample K of the view layer is W + NJ + 1 instead of W + 27 NJ.
//
// Reference behaviour restated (paths relative to danielajisafe/A-NeRF):
//   core/raycasters.py:361-474 render_rays, 476-555 encode_inputs, 557-577 run_network
//   core/encoders.py:8-37, 101-122, 172-193; core/cutoff_embedder.py:111-174
//   core/networks/nerf.py:90-205; core/utils/ray_utils.py:6-28, 157-251, 255-344
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/anerf.h"
#include "anerf_device.hpp"

using namespace anerf;

// Diagnostic build only (-DANERF_STAMPS): per-phase shader-cycle totals, summed over waves into
// RenderArgs::stamps[16]; read only by tools/stamps.py, never part of an output.
struct Stamps {
#ifdef ANERF_STAMPS
    unsigned long long last, acc[24];
#endif
};
#ifdef ANERF_STAMPS
#define STAMP_INIT(st)                                      \
    do {                                                    \
        (st).last = __builtin_amdgcn_s_memtime();           \
        for (int i_ = 0; i_ < 24; ++i_) (st).acc[i_] = 0;   \
    } while (0)
#define STAMP(st, i)                                                      \
    do {                                                                  \
        __builtin_amdgcn_sched_barrier(0);                                \
        const unsigned long long now_ = __builtin_amdgcn_s_memtime();     \
        (st).acc[i] += now_ - (st).last;                                  \
        (st).last = now_;                                                 \
        __builtin_amdgcn_sched_barrier(0);                                \
    } while (0)
#define STAMP_FLUSH(st, ptr)                                              \
    do {                                                                  \
        if ((threadIdx.x & 63) == 0 && (ptr))                             \
            for (int i_ = 0; i_ < 24; ++i_) atomicAdd((ptr) + i_, (st).acc[i_]); \
    } while (0)
#else
#define STAMP_INIT(st) do { } while (0)
#define STAMP(st, i) do { } while (0)
#define STAMP_FLUSH(st, ptr) do { } while (0)
#endif

#define MAXL 16

// ======================================================================= device model
struct NetDev {
    const float* wl[MAXL];   // packed layer weights; [0] bone-direction part of x, [i>0] activation (regs) part
    const float* wl0v;       // layer 0, per-joint windowed part of x (dist, sin, cos)
    const float* bl[MAXL];   // packed biases [RB][2][16]
    const float* wskipu;     // skip layer, bone-direction part of x, or null
    const float* wskipv;     // skip layer, per-joint windowed part of x
    const float* walpha;     // [2][RB][16]
    const float* wfeat;      // packed regs W->W
    const float* bfeat;      // packed bias
    const float* wview;      // packed regs W->W/2 (feature part of views_linears.0)
    const float* wvdir;      // [NJ][W/2][28] direction part (k*3 + c, padded), transposed
    const float* wvcode;     // [cfc][W/2] code part, transposed
    const float* bview;      // [W/2]
    const float* wrgb;       // [3][2][RBV][16]
    const float* brgb;       // [3]
    const float* codes;      // [n_codes + 1][cfc]: last row = eval-mode mean code
    float balpha;
};

struct ModelDev {
    int nj, njh2, ngh, D, skip, mr, mrv, use_cutoff, cutoff_inputs, cutoff_viewdir, cfc, n_codes, softplus;
    int sparse;  // windowed features are exactly 0 where w == 0 (use_cutoff && cutoff_inputs)
    float shift, B, tau, tau_v;
    const float* cutoff;
    const float* cutoff_v;
    NetDev net[2];
};

struct RenderArgs {
    const float* rb;
    int64_t n;
    int stride, S, I, R;
    const float* skts;
    const int32_t* ray_pose;
    const float* cams;
    const float* near;
    const float* far;
    float *rgb, *disp, *acc, *rgb0, *disp0, *acc0, *alpha, *alpha0;
    float *dbg_z0, *dbg_raw0, *dbg_w0, *dbg_z1, *dbg_raw1;
    unsigned long long* mfma_count;
    unsigned long long* stamps;
};

// ======================================================================= LDS plan
struct LdsPlan {
    int ray, sk, zc, zf, raw, g, scr, bias, cut, uf, wv;  // float offsets (uf < 0: no u-feature store)
    int total;                          // floats
    int sk_stride, z_stride, raw_stride, g_stride, scr_stride, uf_stride, wv_stride;
};

__host__ __device__ inline int pad32(int x) { return (x + 31) & ~31; }

__host__ __device__ inline LdsPlan make_plan(int R, int nj, int W, int S, int T, int mrv, int ngh, int D, int njh2,
                                             bool with_uf) {
    LdsPlan p;
    const int wh = W / 2;
    const int nk = 1 + 2 * mrv;
    p.sk_stride = nj * 12;
    p.z_stride = pad32(T > S ? T : S);
    p.raw_stride = p.z_stride * 4;
    p.g_stride = 2 * ngh * wh;
    int scr_a = 8 * p.z_stride;          // composite / importance scratch
    int scr_b = ((3 * nk + 3) & ~3) * nj + 256;  // trig table for G + per-part bias partials (256 / WH parts x WH)
    p.scr_stride = (scr_a > scr_b ? scr_a : scr_b);
    int o = 0;
    p.ray = o; o += 16 * R;
    p.sk = o; o += p.sk_stride * R;
    p.zc = o; o += p.z_stride * R;
    p.zf = o; o += p.z_stride * R;
    p.raw = o; o += p.raw_stride * R;
    p.g = o; o += p.g_stride * R;
    p.scr = o; o += p.scr_stride * R;
    o = (o + 3) & ~3;
    p.bias = o; o += (D + 2) * W;  // the current net's hidden + feature biases, accumulator order; w_alpha
    p.cut = o; o += 3 * nj;        // window: cutoff distances (points, view directions), live thresholds
    o = (o + 3) & ~3;
    p.uf_stride = 64 * 3 * njh2;   // per wave: the L0 bone directions, re-read by the skip layer
    p.uf = with_uf ? o : -1;
    if (with_uf) o += 4 * p.uf_stride;
    p.wv_stride = 64 * njh2;       // per wave: view-direction window weights w'_j of the current block
    p.wv = o; o += 4 * p.wv_stride;
    p.total = (o + 3) & ~3;
    return p;
}

// ======================================================================= MLP building blocks
// Weight streams are read with buffer loads: one SGPR descriptor per array plus a single 32-bit
// lane offset, so the unrolled K loops carry no per-load 64-bit address registers.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const float* p) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)p, 0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ f32x2 bload2(__amdgpu_buffer_rsrc_t rs, int voff, int soff) {
    return __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(rs, voff, soff, 0));
}
__device__ __forceinline__ f32x4 bload4(__amdgpu_buffer_rsrc_t rs, int voff, int soff) {
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, 0));
}

template <int RB>
__device__ __forceinline__ void load_bias(f32x16 (&acc)[RB], const float* __restrict__ bp_lds, int hh) {
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
        const f32x4* p = reinterpret_cast<const f32x4*>(bp_lds + (rb * 2 + hh) * 16);
        f32x4 v0 = p[0], v1 = p[1], v2 = p[2], v3 = p[3];
        acc[rb] = f32x16{v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3],
                         v2[0], v2[1], v2[2], v2[3], v3[0], v3[1], v3[2], v3[3]};
    }
}

// Weight streams are cut into groups of F floats per lane (one MFMA A operand each), stored
// [group][F/4][64 lanes][4] so that every b128 load reads 1 KiB contiguous.  A 4-slot register
// ring is shared by consecutive phases: group g of a layer lives in slot g % 4, the prefetch
// distance is 2 groups, and the last two groups of a layer prefetch groups 0 and 1 of the next
// phase so it starts without a load bubble.
struct Ring {
    float v[4][16];
};

template <int F>
__device__ __forceinline__ void load_group(float (&slot)[16], __amdgpu_buffer_rsrc_t rs, int lane, int g) {
#pragma unroll
    for (int i = 0; i < F / 4; ++i) {
        const f32x4 x = bload4(rs, lane * 16 + i * 1024, g * F * 256);  // (i * 1024 -> immediate offset)
        slot[4 * i] = x[0], slot[4 * i + 1] = x[1], slot[4 * i + 2] = x[2], slot[4 * i + 3] = x[3];
    }
}

template <int F>
__device__ __forceinline__ void ring_preload(Ring& ring, const float* __restrict__ wp, int lane) {
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(wp);
    load_group<F>(ring.v[0], rs, lane, 0);
    load_group<F>(ring.v[1], rs, lane, 1);
}

// One dense layer, out[RBO] (+)= W^T act(in) over 32*RBI inputs, with the layer boundary fused in:
// the previous layer's accumulators ain[rb] are turned into B operands h[rb] (relu, or used as
// they are for the feature -> view edge) and the output blocks are initialised with their bias
// *inside* the first groups, under the MFMAs.  To make that possible the first RBO groups are
// "lead" groups: group rb < RBO runs k-steps 0..15 (input block 0) of output block rb only, so
// block rb+1 is converted while block rb accumulates; the remaining groups are k-major
// (KG = 16/RBO k-steps x RBO blocks = 16 MFMAs each).  ALPHA folds the alpha head
// (sig += w_alpha . h in k-step order) into the groups as VALU filler.
template <int RBO, int RBI, bool RELU_IN, bool OUT_SAME, bool ALPHA>
__device__ __forceinline__ void mlp_layer(f32x16 (&out)[RBO], f32x16 (&ain)[RBI], f32x16 (&h)[RBI],
                                          const float* __restrict__ bias, const float* __restrict__ wp, int lane,
                                          Ring& ring, const float* __restrict__ next, const float* __restrict__ wa,
                                          float& sig) {
    constexpr int KG = 16 / RBO;
    constexpr int NQ = 16 * RBI;
    constexpr int NG = RBO + (NQ - 16) / KG;
    static_assert(RBO * KG == 16 && (NQ - 16) % KG == 0, "group shape");
    const int hh = lane >> 5;
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(wp);
    const __amdgpu_buffer_rsrc_t rn = make_rsrc(next);
    auto init_out = [&](int rb) {  // bias (OUT_SAME layers) or zero
        if constexpr (OUT_SAME) {
            const f32x4* p = reinterpret_cast<const f32x4*>(bias + (rb * 2 + hh) * 16);
            const f32x4 v0 = p[0], v1 = p[1], v2 = p[2], v3 = p[3];
            out[rb] = f32x16{v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3],
                             v2[0], v2[1], v2[2], v2[3], v3[0], v3[1], v3[2], v3[3]};
        } else {
            out[rb] = f32x16{0};
        }
    };
    auto convert = [&](int rb) {
        if constexpr (RELU_IN) {
#pragma unroll
            for (int i = 0; i < 16; ++i) h[rb][i] = relu_act(ain[rb][i]);
        }
        if constexpr (OUT_SAME) {
            if (rb < RBO) init_out(rb);
        }
    };
    auto B = [&](int q) -> float { return RELU_IN ? h[q >> 4][q & 15] : ain[q >> 4][q & 15]; };
    if constexpr (!OUT_SAME) {
#pragma unroll
        for (int rb = 0; rb < RBO; ++rb) init_out(rb);
    }
    convert(0);
#pragma unroll
    for (int g = 0; g < NG; ++g) {
        __builtin_amdgcn_sched_barrier(0);
        if (g + 2 < NG)
            load_group<16>(ring.v[(g + 2) % 4], rs, lane, g + 2);
        else if (NG % 4 == 0 && next)
            load_group<16>(ring.v[(g + 2) % 4], rn, lane, g + 2 - NG);
        if (g < RBO) {
#pragma unroll
            for (int t = 15; t >= 0; --t)  // (last-loaded float first: one vmcnt wait per group)
                out[g] = mfma_f32_32x32x2(ring.v[g % 4][t], B(t), out[g]);
            if (ALPHA && g == 0) {
                const f32x4* w4 = reinterpret_cast<const f32x4*>(wa + hh * 16 * RBI);
#pragma unroll
                for (int t = 0; t < 16; ++t) sig = fmaf(w4[t >> 2][t & 3], B(t), sig);
            }
            if (g + 1 < RBO) {
                convert(g + 1);
            } else {
#pragma unroll
                for (int rb = RBO; rb < RBI; ++rb) convert(rb);
            }
        } else {
            const int q0 = 16 + (g - RBO) * KG;
#pragma unroll
            for (int t = 0; t < KG; ++t) {
                const float b = B(q0 + t);
#pragma unroll
                for (int rb = RBO - 1; rb >= 0; --rb)
                    out[rb] = mfma_f32_32x32x2(ring.v[g % 4][rb * KG + t], b, out[rb]);
                if (ALPHA) sig = fmaf(wa[hh * 16 * RBI + q0 + t], b, sig);
            }
        }
    }
}

// The MLP input x = [v (k*NJ + j), r (NJ*NV + 3j + c)] is split into two k-streams:
//  * the bone-direction part u_j = q_j/|q_j| (never windowed): k-step 3p+c pairs joint p (lane
//    half 0) with joint p + NJH2 (half 1); this pass also ballots the cutoff window per joint;
//  * the windowed part of joint j: k-step t pairs sin_t (half 0) with cos_t (half 1), then
//    (dist, 0); executed only for joints whose window w_j is non-zero for some sample of the
//    block.  w_j rounds to exactly 0 far from a joint, making those 2*MR+1 inputs exact zeros
//    whose MFMAs add nothing: skipping them is bit-exact.
struct JointMask {
    uint64_t m0, m1;
};

__device__ __forceinline__ int mask_pop(uint64_t& a0, uint64_t& a1) {
    if (a0) {
        const int j = __builtin_ctzll(a0);
        a0 &= a0 - 1;
        return j;
    }
    if (a1) {
        const int j = 64 + __builtin_ctzll(a1);
        a1 &= a1 - 1;
        return j;
    }
    return -1;
}

// Pin a value's computation before this point: IR passes otherwise sink the software-pipelined
// encoding math out of the MFMA region it was written in (sched_barrier only binds the
// machine scheduler).
__device__ __forceinline__ void pin(float x) { asm volatile("" ::"v"(x)); }
__device__ __forceinline__ void pin(bool x) { asm volatile("" ::"v"((int)x)); }

// Compile-time interleave of one scheduling region: NM MFMAs, each followed by up to NV VALU
// instructions (one wave per SIMD: without it the scheduler issues the MFMAs back to back and
// leaves the encoding VALU exposed after them).
template <int NM, int NV>
__device__ __forceinline__ void interleave_mfma_valu() {
#pragma unroll
    for (int i = 0; i < NM; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, NV, 0);
    }
}

// u-part weight groups: 2 k-steps x RB row blocks = 2*RB floats per lane (slot float 2*rb + t)
template <int RB>
__device__ __forceinline__ void load_u_group(f32x2 (&slot)[RB], __amdgpu_buffer_rsrc_t rs, int lane, int g) {
#pragma unroll
    for (int i = 0; i < RB / 2; ++i) {
        const f32x4 x = bload4(rs, lane * 16 + i * 1024, g * 2 * RB * 256);
        slot[2 * i] = f32x2{x[0], x[1]};
        slot[2 * i + 1] = f32x2{x[2], x[3]};
    }
}
template <int RB>
__device__ __forceinline__ void ring_take(f32x2 (&slot)[RB], const float (&v)[16]) {
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) slot[rb] = f32x2{v[2 * rb], v[2 * rb + 1]};
}

// Window tables in LDS: cut[j] = c_j, cut[NJ + j] = c'_j (view directions), cut[2NJ + j] = thr2_j,
// a conservative squared-distance bound of the window's support: w_j = 1 - 1/(1 + e),
// e = expf(-tau (d - c_j)), is exactly 0 iff 1 + e rounds to 1, i.e. e <= 2^-24, i.e.
// tau (d - c_j) >= 24 ln 2 = 16.6355 (up to expf's rounding).  With a 0.05 margin on that
// argument (and 1e-5 on the square), d^2 >= thr2 implies w_j == 0 exactly; joints that are
// "live" by this test but have w_j == 0 just add exact zeros.
__device__ __forceinline__ float live_thr2(float tau, float c) {
    if (!(tau > 0.0f)) return __builtin_inff();
    const float d0 = c + 16.69f / tau;
    return d0 <= 0.0f ? -1.0f : d0 * d0 * 1.00001f;
}

__device__ __forceinline__ void stage_cut(const ModelDev& M, float* __restrict__ cut, int tid) {
    for (int j = tid; j < 3 * M.nj; j += blockDim.x) {
        const int k = j % M.nj;
        cut[j] = j < M.nj ? M.cutoff[k] : (j < 2 * M.nj ? M.cutoff_v[k] : live_thr2(M.tau, M.cutoff[k]));
    }
}

// One joint's skeleton row (3x4 of the world->joint transform) and live threshold, loaded from
// LDS into registers two MFMA groups before use, so the encoder math never waits on LDS.
struct JRow {
    f32x4 a, b, c;
    float thr2, cv;
};

__device__ __forceinline__ JRow load_row(const float* __restrict__ sk, const float* __restrict__ cut, int j, int nj) {
    const int jc = j < nj ? j : 0;
    const f32x4* p = reinterpret_cast<const f32x4*>(sk + 12 * jc);
    return JRow{p[0], p[1], p[2], cut[2 * nj + jc], cut[nj + jc]};
}

// bone direction u_j = q / max(|q|, 1e-12) of this lane's sample (q * rsq(max(|q|^2, 1e-24)),
// within 2 ulp) and whether the joint's window may be non-zero (d^2 < thr2, conservative, see
// live_thr2).  Branch-free (per-lane selects) so that it stays in the MFMA region it is
// scheduled into.
// With WV, also the joint's view-direction window w'_j = 1 - sigmoid(tau' (|q| - c'_j)) (hardware
// sqrt/exp2/rcp, a few ulp; 0 for padding joints or without cutoff_viewdir) for the view layer.
template <bool WV>
__device__ __forceinline__ void u_joint(const ModelDev& M, const JRow& r, bool valid, float px, float py, float pz,
                                        float& u0, float& u1, float& u2, bool& live, float& wv) {
#ifdef ANERF_EXP_UFAST  // timing experiment only (stamps build): encoder VALU removed
    u0 = px * r.a[0]; u1 = py; u2 = pz; live = false; wv = 0.0f; return;
#endif
    float qx = fmaf(r.a[3], 1.0f, fmaf(r.a[2], pz, fmaf(r.a[1], py, r.a[0] * px)));
    float qy = fmaf(r.b[3], 1.0f, fmaf(r.b[2], pz, fmaf(r.b[1], py, r.b[0] * px)));
    float qz = fmaf(r.c[3], 1.0f, fmaf(r.c[2], pz, fmaf(r.c[1], py, r.c[0] * px)));
    qx = valid ? qx : 0.0f;
    qy = valid ? qy : 0.0f;
    qz = valid ? qz : 0.0f;
    const float d2 = fmaf(qz, qz, fmaf(qy, qy, qx * qx));
    const float inv = __builtin_amdgcn_rsqf(fmaxf(d2, 1e-24f));
    u0 = qx * inv;
    u1 = qy * inv;
    u2 = qz * inv;
    live = valid & (!M.sparse | !(d2 >= r.thr2));  // (no short-circuit: no branch; NaN -> live)
    if constexpr (WV) {
        const float d = __builtin_amdgcn_sqrtf(d2);
        const float e = __builtin_amdgcn_exp2f(-(M.tau_v * (d - r.cv)) * 1.44269504f);
        const float w = 1.0f - __builtin_amdgcn_rcpf(1.0f + e);
        wv = (valid && M.cutoff_viewdir) ? w : 0.0f;
    }
}

// The geometry of pair-of-pairs pp+1 is computed under the MFMAs of pp (software pipeline:
// between two sched_barriers the scheduler interleaves the VALU with the async MFMAs).
template <int RB>
__device__ __forceinline__ void u_part(f32x16 (&acc)[RB], const ModelDev& M, const float* __restrict__ wp,
                                       const float* __restrict__ sk, const float* __restrict__ cut, float px,
                                       float py, float pz, int lane, JointMask* mask, float* __restrict__ uf,
                                       float* __restrict__ wvo, Ring& sh, const float* __restrict__ next,
                                       Stamps& st) {
    const int hh = lane >> 5;
    const int njh2 = M.njh2;
    const int npp = njh2 / 2;
    const int total_groups = 3 * npp;
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(wp);
    f32x2 ring[3][RB];  // groups 0 and 1 were prefetched into the shared ring by the caller
    ring_take<RB>(ring[0], sh.v[0]);
    ring_take<RB>(ring[1], sh.v[1]);
    uint64_t m0 = 0, m1 = 0;
    float f[6];
    bool lv0, lv1;
    const int nj = M.nj, j0 = hh * njh2;
    JRow ra = load_row(sk, cut, j0, nj), rb2 = load_row(sk, cut, j0 + 1, nj);
    float wv0, wv1;
    u_joint<true>(M, ra, j0 < nj, px, py, pz, f[0], f[1], f[2], lv0, wv0);
    u_joint<true>(M, rb2, j0 + 1 < nj, px, py, pz, f[3], f[4], f[5], lv1, wv1);
    if (wvo) {  // w'_j of k-step p of the view layer's direction part (joint p + h NJH2)
        wvo[lane] = wv0;
        wvo[64 + lane] = wv1;
    }
    ra = load_row(sk, cut, j0 + 2, nj);
    rb2 = load_row(sk, cut, j0 + 3, nj);
    STAMP(st, 14);
    for (int pp = 0; pp < npp; ++pp) {
        if (mask) {
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const uint64_t b = __ballot(k == 0 ? lv0 : lv1);
                const int ja = 2 * pp + k, jb = ja + njh2;
                if (b & 0xffffffffull) {
                    if (ja < 64) m0 |= 1ull << ja; else m1 |= 1ull << (ja - 64);
                }
                if (b >> 32) {
                    if (jb < 64) m0 |= 1ull << jb; else m1 |= 1ull << (jb - 64);
                }
            }
        }
        if (uf) {  // keep this block's bone directions for the skip layer: [group][lane][2]
#pragma unroll
            for (int g = 0; g < 3; ++g)
                *reinterpret_cast<f32x2*>(uf + ((pp * 3 + g) * 64 + lane) * 2) = f32x2{f[2 * g], f[2 * g + 1]};
        }
        float fn[6];
        bool ln0 = false, ln1 = false;
#pragma unroll
        for (int g = 0; g < 3; ++g) {
            __builtin_amdgcn_sched_barrier(0);
            const int gn = min(pp * 3 + g + 2, total_groups - 1);  // (a harmless reload at the end)
            load_u_group<RB>(ring[(g + 2) % 3], rs, lane, gn);
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                const float b = f[2 * g + t];
#pragma unroll
                for (int rb = 0; rb < RB; ++rb) acc[rb] = mfma_f32_32x32x2(ring[g % 3][rb][t], b, acc[rb]);
            }
            if (g == 0) {  // joint 2pp+2 from its prefetched row; then prefetch joint 2pp+4
                float wv;
                u_joint<true>(M, ra, j0 + 2 * pp + 2 < nj, px, py, pz, fn[0], fn[1], fn[2], ln0, wv);
                pin(fn[0]), pin(fn[1]), pin(fn[2]), pin(ln0);
                if (wvo && 2 * pp + 2 < njh2) wvo[(2 * pp + 2) * 64 + lane] = wv;
                ra = load_row(sk, cut, j0 + 2 * pp + 4, nj);
            }
            if (g == 1) {
                float wv;
                u_joint<true>(M, rb2, j0 + 2 * pp + 3 < nj, px, py, pz, fn[3], fn[4], fn[5], ln1, wv);
                pin(fn[3]), pin(fn[4]), pin(fn[5]), pin(ln1);
                if (wvo && 2 * pp + 3 < njh2) wvo[(2 * pp + 3) * 64 + lane] = wv;
                rb2 = load_row(sk, cut, j0 + 2 * pp + 5, nj);
            }
            interleave_mfma_valu<2 * RB, 8>();
        }
#pragma unroll
        for (int i = 0; i < 6; ++i) f[i] = fn[i];
        lv0 = ln0;
        lv1 = ln1;
    }
    if (mask) {
        mask->m0 = m0;
        mask->m1 = m1;
    }
    if (next) ring_preload<16>(sh, next, lane);
}

// The skip layer's bone-direction part from the features u_part stored in LDS: a pure MFMA
// stream (B operands read one group ahead) with the weight ring two groups ahead.
template <int RB>
__device__ __forceinline__ void u_part_lds(f32x16 (&acc)[RB], const ModelDev& M, const float* __restrict__ wp,
                                           const float* __restrict__ uf, int lane, Ring& sh,
                                           const float* __restrict__ next) {
    const int total_groups = 3 * (M.njh2 / 2);
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(wp);
    const f32x2* ub = reinterpret_cast<const f32x2*>(uf) + lane;
    f32x2 ring[3][RB];
    ring_take<RB>(ring[0], sh.v[0]);
    ring_take<RB>(ring[1], sh.v[1]);
    f32x2 bc = ub[0];
    for (int g0 = 0; g0 < total_groups; g0 += 3) {
#pragma unroll
        for (int gg = 0; gg < 3; ++gg) {
            __builtin_amdgcn_sched_barrier(0);
            const int g = g0 + gg;
            const int gn = min(g + 2, total_groups - 1);
            load_u_group<RB>(ring[(gg + 2) % 3], rs, lane, gn);
            const f32x2 bn = ub[min(g + 1, total_groups - 1) * 64];
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int rb = 0; rb < RB; ++rb) acc[rb] = mfma_f32_32x32x2(ring[gg][rb][t], bc[t], acc[rb]);
            bc = bn;
        }
    }
    if (next) ring_preload<16>(sh, next, lane);
}

template <int MR>
struct VPart {
    static constexpr int KB = ((MR + 1) + 1) & ~1;  // k-steps per joint (even)
    static constexpr int GB = KB / 2;               // float2 groups per joint
};

__device__ __forceinline__ void v_geom(const ModelDev& M, const float* __restrict__ sk, const float* __restrict__ cut,
                                       int j, float px, float py, float pz, float& dist, float& w) {
    float qx, qy, qz;
    joint_local(sk + 12 * j, px, py, pz, qx, qy, qz);
    dist = norm3(qx, qy, qz);
    const float wc = cutoff_w(M.tau, dist, cut[j]);
    w = M.use_cutoff ? wc : 1.0f;
}

template <int RB, int MR>
__device__ __forceinline__ void v_part(f32x16 (&acc)[RB], const ModelDev& M, const float* __restrict__ wp,
                                       const float* __restrict__ sk, const float* __restrict__ cut, float px,
                                       float py, float pz, int lane, JointMask mask, Stamps& st) {
    constexpr int GB = VPart<MR>::GB;
    constexpr int KB = VPart<MR>::KB;
    constexpr int PER = (MR + GB - 2) / (GB - 1);  // sin/cos terms of the next joint per group 1..GB-1
    const int hh = lane >> 5;
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(wp);
    const int voff = lane * 8;
    const bool dist_in = M.use_cutoff && M.cutoff_inputs;
    uint64_t r0 = mask.m0, r1 = mask.m1;
    int j = mask_pop(r0, r1);
    if (j < 0) return;
    int jn = mask_pop(r0, r1);
    f32x2 ring[GB][RB];
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) ring[g][rb] = bload2(rs, voff, ((j * GB + g) * RB + rb) * 512);
    float f[KB];
    {
        float dist, w;
        v_geom(M, sk, cut, j, px, py, pz, dist, w);
#pragma unroll
        for (int t = 0; t < MR; ++t) {
            float sn, cs;
            sincos_rr(dist * (float)(1 << t), sn, cs);
            f[t] = (hh ? cs : sn) * w;
        }
        f[MR] = hh ? 0.0f : (dist_in ? dist * w : dist);
#pragma unroll
        for (int t = MR + 1; t < KB; ++t) f[t] = 0.0f;
    }
    STAMP(st, 15);
    while (j >= 0) {
        float fn[KB];
        float dn = 0.0f, wn = 0.0f;
        const int jg = jn >= 0 ? jn : j;  // geometry of the next joint (harmless redo at the end)
#pragma unroll
        for (int g = 0; g < GB; ++g) {
            __builtin_amdgcn_sched_barrier(0);
            constexpr int PD = 2;
            if (g + PD < GB) {
#pragma unroll
                for (int rb = 0; rb < RB; ++rb)
                    ring[(g + PD) % GB][rb] = bload2(rs, voff, ((j * GB + g + PD) * RB + rb) * 512);
            } else {  // the next joint's first groups (this joint's again after the last: harmless)
#pragma unroll
                for (int rb = 0; rb < RB; ++rb)
                    ring[(g + PD) % GB][rb] = bload2(rs, voff, ((jg * GB + g + PD - GB) * RB + rb) * 512);
            }
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                const float b = f[2 * g + t];
#pragma unroll
                for (int rb = 0; rb < RB; ++rb) acc[rb] = mfma_f32_32x32x2(ring[g][rb][t], b, acc[rb]);
            }
            // next joint's features under these MFMAs
            if (g == 0) {
                v_geom(M, sk, cut, jg, px, py, pz, dn, wn);
                pin(dn), pin(wn);
            } else {
#pragma unroll
                for (int t = (g - 1) * PER; t < g * PER && t < MR; ++t) {
                    float sn, cs;
                    sincos_rr(dn * (float)(1 << t), sn, cs);
                    fn[t] = (hh ? cs : sn) * wn;
                    pin(fn[t]);
                }
            }
            interleave_mfma_valu<2 * RB, 8>();
        }
        fn[MR] = hh ? 0.0f : (dist_in ? dn * wn : dn);
#pragma unroll
        for (int t = MR + 1; t < KB; ++t) fn[t] = 0.0f;
#pragma unroll
        for (int t = 0; t < KB; ++t) f[t] = fn[t];
        j = jn;
        jn = mask_pop(r0, r1);
    }
}

// View layer, per-ray direction part: acc[RBV] += G^T * [w'_j, 1]  (G in LDS).  k-step p pairs
// joint p (lane half 0) with joint p + NJH2 (half 1), exactly the u part's pairing, so w'_j comes
// from the u part (wvp, stored per lane); k-step NJH2 adds the bias / framecode column NJ.  The G
// values of the next k-step are read under the current k-step's MFMAs.
template <int RBV>
__device__ __forceinline__ void view_dir_part(f32x16 (&acc)[RBV], const ModelDev& M, const float* __restrict__ G,
                                              const float* __restrict__ wvp, int lane) {
    constexpr int WH = RBV * 32;
    const int hh = lane >> 5, sl = lane & 31;
    const int njh2 = M.njh2;
    auto col = [&](int p) { return p < njh2 ? p + hh * njh2 : M.nj + hh; };
    float gv[RBV];
#pragma unroll
    for (int rb = 0; rb < RBV; ++rb) gv[rb] = G[col(0) * WH + sl + 32 * rb];
    float b = wvp[lane];
    for (int p = 0; p <= njh2; ++p) {
        __builtin_amdgcn_sched_barrier(0);
        const int pn = min(p + 1, njh2);
        float gn[RBV];
#pragma unroll
        for (int rb = 0; rb < RBV; ++rb) gn[rb] = G[col(pn) * WH + sl + 32 * rb];
        const float bn = pn < njh2 ? wvp[pn * 64 + lane] : (hh ? 0.0f : 1.0f);
#pragma unroll
        for (int rb = 0; rb < RBV; ++rb) acc[rb] = mfma_f32_32x32x2(gv[rb], b, acc[rb]);
#pragma unroll
        for (int rb = 0; rb < RBV; ++rb) gv[rb] = gn[rb];
        b = bn;
    }
}

// Encoder + density trunk of one 32-sample block: L0 (u and v parts), the hidden layers with the
// skip; acc ends as the pre-activation of the last hidden layer.  `after_last` is the weight stream
// that follows (the feature layer, or nothing for density-only queries).
template <int W, int MR>
__device__ __forceinline__ void mlp_trunk(const ModelDev& M, const NetDev& net, const float* __restrict__ sk,
                                          const float* __restrict__ cut, float px, float py, float pz, int lane,
                                          const float* __restrict__ bias, float* __restrict__ uf,
                                          float* __restrict__ wvo, f32x16 (&acc)[W / 32], f32x16 (&h)[W / 32],
                                          Ring& ring, JointMask& mask, const float* __restrict__ after_last,
                                          Stamps& st) {
    constexpr int RB = W / 32;
    const int hh = lane >> 5;
    float nosig = 0.0f;
    constexpr bool HANDOFF = (2 * RB == 16);  // u-part groups have the regs layers' group size
    ring_preload<2 * RB>(ring, net.wl[0], lane);  // the u part's first groups, early
    load_bias<RB>(acc, bias, hh);
    STAMP(st, 10);
    u_part<RB>(acc, M, net.wl[0], sk, cut, px, py, pz, lane, &mask, uf, wvo, ring, M.D > 1 ? net.wl[1] : after_last,
               st);
    STAMP(st, 8);
    v_part<RB, MR>(acc, M, net.wl0v, sk, cut, px, py, pz, lane, mask, st);
    STAMP(st, 9);
    for (int L = 1; L < M.D; ++L) {
        const float* after = L + 1 < M.D ? net.wl[L + 1] : after_last;
        const bool skl = (L == M.skip + 1);
        mlp_layer<RB, RB, true, true, false>(acc, acc, h, bias + L * W, net.wl[L], lane, ring,
                                             skl ? (HANDOFF ? net.wskipu : nullptr) : after, nullptr, nosig);
        STAMP(st, 11);
        if (skl) {  // x part after the h part
            if (!HANDOFF) ring_preload<2 * RB>(ring, net.wskipu, lane);
            if (uf)
                u_part_lds<RB>(acc, M, net.wskipu, uf, lane, ring, after);
            else
                u_part<RB>(acc, M, net.wskipu, sk, cut, px, py, pz, lane, nullptr, nullptr, nullptr, ring, after, st);
            v_part<RB, MR>(acc, M, net.wskipv, sk, cut, px, py, pz, lane, mask, st);
            STAMP(st, 12);
        }
    }
}

// One 32-sample block of one ray through a whole NeRF: raw (rgb, sigma) into LDS.
template <int W, int MR>
__device__ void mlp_block(const ModelDev& M, const NetDev& net, const float* __restrict__ ray,
                          const float* __restrict__ sk, const float* __restrict__ cut, const float* __restrict__ z,
                          int n, int s0,
                          const float* __restrict__ G, float* __restrict__ raw_out, int lane,
                          unsigned long long* mfma_count, const float* __restrict__ bias, float* __restrict__ uf,
                          float* __restrict__ wvp, Stamps& st) {
    constexpr int RB = W / 32;
    constexpr int RBV = (W / 2) / 32;
    const int sl = lane & 31, hh = lane >> 5;
    int s = s0 + sl;
    if (s >= n) s = n - 1;
    const float zs = z[s];
    // pts = rays_o + rays_d * z (raycasters.py:658), separately rounded
    const float px = ray[0] + ray[3] * zs;
    const float py = ray[1] + ray[4] * zs;
    const float pz = ray[2] + ray[5] * zs;

    f32x16 acc[RB], h[RB];
    JointMask mask;
    Ring ring;
    mlp_trunk<W, MR>(M, net, sk, cut, px, py, pz, lane, bias, uf, wvp, acc, h, ring, mask, net.wview, st);
    // views_linears.0 with feature_linear fused in (W' = Wv_f Wf, see pack_net) on relu(h_last),
    // alpha_linear folded into its groups (same relu'd B operands), + the factorised
    // direction / code / bias part from G, then relu
    float sig = 0.0f;
    f32x16 av[RBV];
    mlp_layer<RBV, RB, true, false, true>(av, acc, h, nullptr, net.wview, lane, ring, nullptr, bias + (M.D + 1) * W,
                                          sig);
    STAMP(st, 16);
    sig += __shfl_xor(sig, 32);
    sig += net.balpha;
    view_dir_part<RBV>(av, M, G, wvp, lane);
    STAMP(st, 17);
    float rgb[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const float* wr = net.wrgb + (c * 2 + hh) * RBV * 16;
        float a = 0.0f;
#pragma unroll
        for (int rb = 0; rb < RBV; ++rb)
#pragma unroll
            for (int i = 0; i < 16; ++i) a += wr[rb * 16 + i] * relu_act(av[rb][i]);
        a += __shfl_xor(a, 32);
        rgb[c] = a + net.brgb[c];
    }
    STAMP(st, 13);
    if (mfma_count && lane == 0) {  // exact MFMA work of this block (wave-uniform quantities)
        const int act = __builtin_popcountll(mask.m0) + __builtin_popcountll(mask.m1);
        const int xk = 3 * M.njh2 + act * VPart<MR>::KB;  // k-steps of one x part
        long long k = (long long)xk * RB + (long long)(M.D - 1) * (W / 2) * RB + (long long)(W / 2) * RBV +
                      (long long)(M.njh2 + 1) * RBV;
        if (M.skip + 1 < M.D) k += (long long)xk * RB;
        atomicAdd(mfma_count, (unsigned long long)k);
    }
    if (hh == 0 && s0 + sl < n) {
        float* o = raw_out + 4 * (s0 + sl);
        o[0] = rgb[0];
        o[1] = rgb[1];
        o[2] = rgb[2];
        o[3] = sig;
    }
}

// ======================================================================= per-ray stages
// Per-ray view factor G[c][n] for every ray of the group (all threads). Needs Tt scratch.
// Thread t owns output row n = t % WH and the joint columns c = t / WH (mod 256 / WH) for ALL rays
// of the group, so every weight it loads is used once per ray; the 3 * NK weights of the next
// column are loaded while the current column is reduced (double buffer).
template <int WH, int MRV>
__device__ void compute_view_factor(const ModelDev& M, const NetDev& net, float* lds, const LdsPlan& P, int nr,
                                    int tid, Stamps& st) {
    constexpr int NK = 1 + 2 * MRV;
    constexpr int KC = 3 * NK;
    constexpr int NPART = 256 / WH;
    const int nj = M.nj;
    // trig table Tt[j][k*3 + c] (27 values, padded to 28) of the normalised joint-frame ray
    // directions, one (ray, joint, coordinate) per thread
    constexpr int TP = (KC + 3) & ~3;
    for (int idx = tid; idx < nr * nj * 3; idx += blockDim.x) {
        const int r = idx / (nj * 3), j = (idx / 3) % nj, c = idx % 3;
        const float* ray = lds + P.ray + 16 * r;
        const float* S = lds + P.sk + P.sk_stride * r + 12 * j;
        float ex, ey, ez;
        joint_rot(S, ray[3], ray[4], ray[5], ex, ey, ez);
        const float en = fmaxf(norm3(ex, ey, ez), 1e-12f);
        const float e = (c == 0 ? ex : (c == 1 ? ey : ez)) / en;
        float* Tt = lds + P.scr + P.scr_stride * r + TP * j;
        Tt[c] = e;
#pragma unroll
        for (int f = 0; f < MRV; ++f) {
            float sn, cs;
            sincos_rr(e * (float)(1 << f), sn, cs);
            Tt[(1 + 2 * f) * 3 + c] = sn;
            Tt[(2 + 2 * f) * 3 + c] = cs;
        }
        if (c == 0)
            for (int k = KC; k < TP; ++k) Tt[k] = 0.0f;
    }
    __syncthreads();
    STAMP(st, 7);
    const int ncol = 2 * M.ngh;
    const int kfw = M.cutoff_inputs ? 0 : 1;             // first k term multiplied by w'
    const int kend = M.cutoff_viewdir ? kfw : NK;         // k terms the cutoff does not weight
    const int nn = tid % WH, part = tid / WH;
    // G[c][n] = sum_k Wvdir[c][k][n] T_k(e_c), 4 rays at a time (independent FMA chains), the
    // column's 27 weights in registers (next column's loaded under the current one)
    if (part < NPART) {
        const __amdgpu_buffer_rsrc_t rs = make_rsrc(net.wvdir);
        if (kend > 0)  // this thread's partial of the unweighted terms, per ray, in scratch
            for (int r = 0; r < nr; ++r) lds[P.scr + P.scr_stride * r + TP * nj + part * WH + nn] = 0.0f;
        float wc[TP], wn[TP];
        auto load_col = [&](float (&dst)[TP], int col) {
#pragma unroll
            for (int q = 0; q < TP / 4; ++q) {
                const f32x4 x = bload4(rs, (col * WH + nn) * TP * 4 + q * 16, 0);
                dst[4 * q] = x[0], dst[4 * q + 1] = x[1], dst[4 * q + 2] = x[2], dst[4 * q + 3] = x[3];
            }
        };
        int c = part;
        if (c < nj) load_col(wc, c);
        for (; c < nj; c += NPART) {
            const int cn = c + NPART;
            if (cn < nj) load_col(wn, cn);
            for (int r0 = 0; r0 < nr; r0 += 4) {
                float v[4] = {0.0f, 0.0f, 0.0f, 0.0f}, u[4] = {0.0f, 0.0f, 0.0f, 0.0f};
                if (kend == 0 && kfw == 0 && M.cutoff_viewdir) {  // every term is windowed (the usual flags)
#pragma unroll
                    for (int q = 0; q < TP / 4; ++q) {
#pragma unroll
                        for (int rr = 0; rr < 4; ++rr) {
                            const int r = min(r0 + rr, nr - 1);
                            const f32x4 t = *reinterpret_cast<const f32x4*>(lds + P.scr + P.scr_stride * r + TP * c + 4 * q);
#pragma unroll
                            for (int e = 0; e < 4; ++e)
                                if (4 * q + e < KC) v[rr] = fmaf(wc[4 * q + e], t[e], v[rr]);
                        }
                    }
                } else {
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) {
                        const int r = min(r0 + rr, nr - 1);
                        const float* tc = lds + P.scr + P.scr_stride * r + TP * c;
#pragma unroll
                        for (int k = 0; k < NK; ++k)
#pragma unroll
                            for (int cc = 0; cc < 3; ++cc) {
                                const float term = wc[k * 3 + cc] * tc[k * 3 + cc];
                                if (M.cutoff_viewdir && k >= kfw) v[rr] += term;
                                if (k < kend) u[rr] += term;
                            }
                    }
                }
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) {
                    const int r = r0 + rr;
                    if (r < nr) {
                        lds[P.g + P.g_stride * r + c * WH + nn] = v[rr];
                        if (kend > 0) lds[P.scr + P.scr_stride * r + TP * nj + part * WH + nn] += u[rr];
                    }
                }
            }
#pragma unroll
            for (int kc = 0; kc < TP; ++kc) wc[kc] = wn[kc];
        }
    }
    __syncthreads();
    for (int idx = tid; idx < nr * WH; idx += blockDim.x) {
        const int r = idx / WH, n2 = idx % WH;
        const float* ray = lds + P.ray + 16 * r;
        float* G = lds + P.g + P.g_stride * r;
        float b = net.bview[n2];
        if (M.cfc) {
            const float cam = ray[6];
            const int64_t row = cam < 0.0f ? (int64_t)M.n_codes : (int64_t)cam;
            for (int m = 0; m < M.cfc; ++m) b += net.wvcode[m * WH + n2] * net.codes[row * M.cfc + m];
        }
        if (kend > 0)
            for (int pp = 0; pp < NPART; ++pp) b += lds[P.scr + P.scr_stride * r + ((KC + 3) & ~3) * nj + pp * WH + n2];
        G[nj * WH + n2] = b;
        for (int c = nj + 1; c < ncol; ++c) G[c * WH + n2] = 0.0f;
    }
    __syncthreads();
}

__device__ __forceinline__ float density_act(const ModelDev& M, float x) {
    if (!M.softplus) return relu(x);
    const float y = x - M.shift;  // F.softplus(beta=1, threshold=20)
    return y > 20.0f ? y : log1pf(expf(y));
}

// raw2outputs (nerf.py:150-205) of ray slot r over n samples; wave-cooperative, all waves call it.
// scr layout: w[zs], wz[zs], wc[3 zs], fac[zs], al[zs]
// Results (rgb[3], disp, acc) are left in res[0..4] (LDS) for the caller to store.
// Per-ray stages run one wave per ray on the ray's own LDS scratch: a wave-level fence orders the
// LDS hand-offs between lanes (a wave's LDS operations complete in order), no workgroup barrier.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

// raw2outputs (nerf.py:150-205) for one ray: alpha, transmittance (torch's CPU cumprod: a
// sequential double product, run by lane 0 four samples per LDS access), weights (left in scr
// for importance sampling), and rgb / depth / acc as wave reductions.  Results in res[0..4].
__device__ void composite(const ModelDev& M, const float* ray, const float* z, const float* raw, int n, float* scr,
                          int zs, bool active, int lane, float* o_alpha, float* res) {
    float* w = scr;
    float* fac = scr + 5 * zs;
    float* al = scr + 6 * zs;
    if (active) {
        const float dn = ray[9];  // |d| cached in slot 9
        for (int i = lane; i < n; i += 64) {
            float dist = (i + 1 < n) ? (z[i + 1] - z[i]) : 1e10f;
            dist = dist * dn;
            const float a = 1.0f - expf(-density_act(M, raw[4 * i + 3] / M.B) * dist);
            al[i] = a;
            fac[i] = (1.0f - a) + 1e-10f;
            if (o_alpha) o_alpha[i] = a;
        }
    }
    wave_sync();
    if (active && lane == 0) {
        double T = 1.0;
        int i = 0;
        for (; i + 4 <= n; i += 4) {
            const f32x4 f = *reinterpret_cast<const f32x4*>(fac + i);
            f32x4 o;
            o[0] = (float)T; T *= (double)f[0];
            o[1] = (float)T; T *= (double)f[1];
            o[2] = (float)T; T *= (double)f[2];
            o[3] = (float)T; T *= (double)f[3];
            *reinterpret_cast<f32x4*>(w + i) = o;
        }
        for (; i < n; ++i) {
            w[i] = (float)T;
            T *= (double)fac[i];
        }
    }
    wave_sync();
    float sa = 0.0f, sd = 0.0f, sr = 0.0f, sg = 0.0f, sb = 0.0f;
    if (active) {
        for (int i = lane; i < n; i += 64) {
            const float wi = al[i] * w[i];
            w[i] = wi;
            sa += wi;
            sd += wi * z[i];
            sr += wi * (sigmoid(raw[4 * i + 0]) * 1.002f - 0.001f);
            sg += wi * (sigmoid(raw[4 * i + 1]) * 1.002f - 0.001f);
            sb += wi * (sigmoid(raw[4 * i + 2]) * 1.002f - 0.001f);
        }
    }
    sa = wave_sum(sa), sd = wave_sum(sd), sr = wave_sum(sr), sg = wave_sum(sg), sb = wave_sum(sb);
    if (active && lane == 0) {
        const float ratio = sd / (sa + 1e-10f);
        float dsp = 1.0f / fmaxf(ratio, 1e-10f);
        if (ratio != ratio) dsp = ratio;  // torch.max propagates NaN
        if (fabsf(sa) <= 1e-8f) dsp = 0.0f;
        res[0] = sr;
        res[1] = sg;
        res[2] = sb;
        res[3] = dsp;
        res[4] = sa < 1.0f ? sa : 1.0f;
    }
    wave_sync();
}

__device__ __forceinline__ bool z_less(float a, float b) { return a < b || (b != b && a == a); }
__device__ __forceinline__ bool z_eq(float a, float b) { return a == b || (a != a && b != b); }

// isample_from_lineseg + sample_pdf(det) + sort (ray_utils.py:157-201, 255-289) for ray slot r.
// weights w (S) in scr; writes sorted z_all (S+I) to zf.
__device__ void importance(const float* zc, const float* w, int S, int I, float* zf, float* scr2, bool active,
                           int lane) {
    const int nb = S - 1;  // bins = mids
    float* mids = scr2;
    float* wp = scr2 + nb;
    float* cdf = scr2 + 2 * nb;
    float* zall = scr2 + 3 * nb + 1;  // S + I unsorted
    if (active) {
        for (int i = lane; i < nb; i += 64) mids[i] = 0.5f * (zc[i + 1] + zc[i]);
        for (int i = lane; i < nb - 1; i += 64) wp[i] = w[i + 1] + 1e-5f;
    }
    wave_sync();
    if (active) {
        // pdf = wp / torch.sum(wp) (every lane computes the same cascade sum), in parallel; then
        // torch's CPU cumsum, a sequential double sum, by lane 0 four values per LDS access
        const float sum = torch_sum(wp, nb - 1);
        for (int i = lane; i < nb - 1; i += 64) wp[i] = wp[i] / sum;
    }
    wave_sync();
    if (active && lane == 0) {
        double c = 0.0;
        cdf[0] = 0.0f;
        int i = 0;
        for (; i + 4 <= nb - 1; i += 4) {
            float q[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) q[k] = wp[i + k];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                c += (double)q[k];
                cdf[i + k + 1] = (float)c;
            }
        }
        for (; i < nb - 1; ++i) {
            c += (double)wp[i];
            cdf[i + 1] = (float)c;
        }
    }
    wave_sync();
    if (active) {
        for (int k = lane; k < I; k += 64) {
            const float u = torch_linspace01(k, I);
            int lo = 0, hi = nb;  // searchsorted(right=True) over nb cdf entries
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (cdf[mid] <= u) lo = mid + 1; else hi = mid;
            }
            const int below = max(lo - 1, 0), above = min(lo, nb - 1);
            const float cb = cdf[below], ca = cdf[above];
            const float bb = mids[below], ba = mids[above];
            float denom = ca - cb;
            if (denom < 1e-5f) denom = 1.0f;
            const float t = (u - cb) / denom;
            zall[S + k] = bb + t * (ba - bb);
        }
        for (int i = lane; i < S; i += 64) zall[i] = zc[i];
    }
    wave_sync();
    const int T = S + I;
    if (active) {
        // both lists are normally sorted (z monotone in t, samples monotone in u): merge by binary
        // search; otherwise a stable O(T^2) rank sort.  Both equal torch.sort's values.
        bool ok = true;
        for (int e = lane; e < T; e += 64) {
            const float v = zall[e];
            if (v != v) ok = false;
            if (e != 0 && e != S && !(zall[e - 1] <= v)) ok = false;
        }
        if (__all(ok)) {
            const float* zs = zall + S;
            for (int e = lane; e < T; e += 64) {
                const float v = zall[e];
                int lo, hi, rank;
                if (e < S) {  // coarse sample: after fine samples strictly below it
                    lo = 0; hi = I;
                    while (lo < hi) { const int mid = (lo + hi) >> 1; if (zs[mid] < v) lo = mid + 1; else hi = mid; }
                    rank = e + lo;
                } else {      // fine sample: after coarse samples <= it
                    lo = 0; hi = S;
                    while (lo < hi) { const int mid = (lo + hi) >> 1; if (zall[mid] <= v) lo = mid + 1; else hi = mid; }
                    rank = (e - S) + lo;
                }
                zf[rank] = v;
            }
        } else {
            for (int e = lane; e < T; e += 64) {
                const float v = zall[e];
                int rank = 0;
                for (int f = 0; f < T; ++f) {
                    const float x = zall[f];
                    rank += z_less(x, v) || (z_eq(x, v) && f < e);
                }
                zf[rank] = v;
            }
        }
    }
    wave_sync();
}

// The current net's hidden biases, feature bias and alpha_linear row into LDS ([D + 2][W]): all
// global loads issued before the first LDS store (one memory latency instead of D + 2).
template <int W>
__device__ __forceinline__ void stage_bias(const ModelDev& M, const NetDev& net, float* __restrict__ dst, int tid) {
    static_assert(W <= 256, "one element per thread and row");
    if (tid >= W) return;
    float v[MAXL + 2];
#pragma unroll
    for (int L = 0; L < MAXL + 2; ++L)
        if (L < M.D + 2) v[L] = L < M.D ? net.bl[L][tid] : (L == M.D ? net.bfeat[tid] : net.walpha[tid]);
#pragma unroll
    for (int L = 0; L < MAXL + 2; ++L)
        if (L < M.D + 2) dst[L * W + tid] = v[L];
}

// ======================================================================= fused render kernel
template <int W, int MR>
__global__ __launch_bounds__(256, 1) void render_kernel(ModelDev M, RenderArgs A, LdsPlan P) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    constexpr int WH = W / 2;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int R = A.R, S = A.S, I = A.I, T = S + I;
    const int64_t ray0 = (int64_t)blockIdx.x * R;
    const int nr = (int)min((int64_t)R, A.n - ray0);

    // ---- rays, poses, skeleton transforms into LDS
    for (int r = tid; r < nr; r += blockDim.x) {
        const int64_t i = ray0 + r;
        const float* src = A.rb + i * A.stride;
        float* d = lds + P.ray + 16 * r;
        for (int c = 0; c < 6; ++c) d[c] = src[c];
        d[6] = A.cams ? A.cams[i] : -1.0f;
        d[7] = A.near[i];
        d[8] = A.far[i];
        d[9] = norm3(src[3], src[4], src[5]);
        d[10] = __int_as_float(A.ray_pose ? A.ray_pose[i] : 0);
    }
    __syncthreads();
    for (int idx = tid; idx < nr * M.nj * 12; idx += blockDim.x) {
        const int r = idx / (M.nj * 12), e = idx % (M.nj * 12);
        const int j = e / 12, c = e % 12;
        const int pose = __float_as_int(lds[P.ray + 16 * r + 10]);
        lds[P.sk + P.sk_stride * r + e] = A.skts[((int64_t)pose * M.nj + j) * 16 + c];
    }
    stage_cut(M, lds + P.cut, tid);
    // coarse samples (sample_from_lineseg, ray_utils.py:218-224)
    for (int idx = tid; idx < nr * S; idx += blockDim.x) {
        const int r = idx / S, s = idx % S;
        const float t = torch_linspace01(s, S);
        const float nearv = lds[P.ray + 16 * r + 7], farv = lds[P.ray + 16 * r + 8];
        lds[P.zc + P.z_stride * r + s] = nearv * (1.0f - t) + farv * t;
    }
    __syncthreads();

    Stamps st;
    STAMP_INIT(st);
    STAMP(st, 0);
    const int n_pass = I > 0 ? 2 : 1;
    for (int pass = 0; pass < n_pass; ++pass) {
        const NetDev& net = M.net[pass];
        const int n = pass == 0 ? S : T;
        const int zoff = pass == 0 ? P.zc : P.zf;
        stage_bias<W>(M, net, lds + P.bias, tid);  // (synced below)
        compute_view_factor<WH, 4>(M, net, lds, P, nr, tid, st);
        STAMP(st, 1);
        // ---- MLP over 32-sample blocks, round-robin over the 4 waves
        const int nb = (n + 31) / 32;
        for (int b = wave; b < nr * nb; b += 4) {
            const int r = b / nb, s0 = (b % nb) * 32;
            mlp_block<W, MR>(M, net, lds + P.ray + 16 * r, lds + P.sk + P.sk_stride * r, lds + P.cut,
                             lds + zoff + P.z_stride * r, n, s0, lds + P.g + P.g_stride * r,
                             lds + P.raw + P.raw_stride * r, lane, A.mfma_count, lds + P.bias,
                             (P.uf >= 0 && M.skip + 1 < M.D) ? lds + P.uf + wave * P.uf_stride : nullptr,
                             lds + P.wv + wave * P.wv_stride, st);
        }
        STAMP(st, 2 + 2 * pass);
        __syncthreads();
        STAMP(st, 6);
        // ---- composite (+ importance sampling after the coarse pass); one wave per ray
        for (int r0 = 0; r0 < R; r0 += 4) {
            const int r = r0 + wave;
            const bool active = r < nr;
            const int64_t i = ray0 + r;
            const float* ray = lds + P.ray + 16 * min(r, R - 1);
            const float* z = lds + zoff + P.z_stride * min(r, R - 1);
            const float* raw = lds + P.raw + P.raw_stride * min(r, R - 1);
            float* scr = lds + P.scr + P.scr_stride * min(r, R - 1);
            const bool final_pass = pass == n_pass - 1;
            float* o_rgb = final_pass ? A.rgb : A.rgb0;
            float* o_disp = final_pass ? A.disp : A.disp0;
            float* o_acc = final_pass ? A.acc : A.acc0;
            float* o_alpha = final_pass ? A.alpha : A.alpha0;
            float* pal = (active && o_alpha) ? o_alpha + i * n : nullptr;
            if (active) {
                float* dz = pass == 0 ? A.dbg_z0 : A.dbg_z1;
                float* draw = pass == 0 ? A.dbg_raw0 : A.dbg_raw1;
                for (int s = lane; s < n; s += 64) {
                    if (dz) dz[i * n + s] = z[s];
                    if (draw)
                        for (int c = 0; c < 4; ++c) draw[(i * n + s) * 4 + c] = raw[4 * s + c];
                }
            }
            float* res = scr + 7 * P.z_stride;
            composite(M, ray, z, raw, n, scr, P.z_stride, active, lane, pal, res);
            if (active && lane < 5) {
                const float v = res[lane];
                if (lane < 3) {
                    if (o_rgb) o_rgb[3 * i + lane] = v;
                } else if (lane == 3) {
                    if (o_disp) o_disp[i] = v;
                } else if (o_acc) {
                    o_acc[i] = v;
                }
            }
            if (pass == 0 && I > 0) {
                if (active && A.dbg_w0)
                    for (int s = lane; s < S; s += 64) A.dbg_w0[i * S + s] = scr[s];
                importance(z, scr, S, I, lds + P.zf + P.z_stride * min(r, R - 1), scr + P.z_stride, active, lane);
            }
        }
        __syncthreads();
        STAMP(st, 3 + 2 * pass);
    }
    STAMP_FLUSH(st, A.stamps);
}

// ======================================================================= density-only queries
// RayCaster.render_pts_density / render_mesh_density (core/raycasters.py:579-648): the trunk of
// one network and alpha_linear at arbitrary points (or at the (res+1)^3 mesh grid, generated here:
// point (a, b, c) = (t[b], t[a], t[c]) + kp0, the 'xy' meshgrid order of the reference).
struct DensityArgs {
    const float* pts;  // N x 3, or NULL for the grid
    const float* t;    // grid axis, res1 floats
    const float* kp0;  // 3
    int64_t res1;
    int64_t n;
    const float* skts;  // NJ x 16, one pose
    int net;
    float* out;  // N raw densities
};

__host__ __device__ inline LdsPlan make_density_plan(int nj, int W, int D, int njh2) {
    LdsPlan p;
    std::memset(&p, 0, sizeof(p));
    int o = 0;
    p.sk = o; o += 12 * nj;
    p.cut = o; o += 3 * nj;
    o = (o + 3) & ~3;
    p.bias = o; o += (D + 2) * W;
    p.uf_stride = 64 * 3 * njh2;
    p.uf = o; o += 4 * p.uf_stride;
    p.total = (o + 3) & ~3;
    return p;
}

template <int W, int MR>
__global__ __launch_bounds__(256, 1) void density_kernel(ModelDev M, DensityArgs A, LdsPlan P) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    constexpr int RB = W / 32;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, hh = lane >> 5;
    const NetDev& net = M.net[A.net];
    for (int idx = tid; idx < M.nj * 12; idx += blockDim.x) lds[P.sk + idx] = A.skts[(idx / 12) * 16 + idx % 12];
    stage_cut(M, lds + P.cut, tid);
    stage_bias<W>(M, net, lds + P.bias, tid);
    __syncthreads();
    Stamps st;
    float* uf = (M.skip + 1 < M.D) ? lds + P.uf + wave * P.uf_stride : nullptr;
    const float* wa = lds + P.bias + (M.D + 1) * W + hh * (W / 2);
    const int64_t nb = (A.n + 31) / 32;
    for (int64_t b = (int64_t)blockIdx.x * 4 + wave; b < nb; b += (int64_t)gridDim.x * 4) {
        const int64_t s_out = b * 32 + (lane & 31);
        const int64_t s = s_out < A.n ? s_out : A.n - 1;
        float px, py, pz;
        if (A.pts) {
            px = A.pts[3 * s], py = A.pts[3 * s + 1], pz = A.pts[3 * s + 2];
        } else {
            const int64_t a = s / (A.res1 * A.res1), r = s % (A.res1 * A.res1);
            px = A.t[r / A.res1] + A.kp0[0];
            py = A.t[a] + A.kp0[1];
            pz = A.t[r % A.res1] + A.kp0[2];
        }
        f32x16 acc[RB], h[RB];
        JointMask mask;
        Ring ring;
        mlp_trunk<W, MR>(M, net, lds + P.sk, lds + P.cut, px, py, pz, lane, lds + P.bias, uf, nullptr, acc, h, ring,
                         mask, nullptr, st);
        // alpha_linear on relu(h_last), in the k-step order of the render path's fused alpha head
        float sig = 0.0f;
#pragma unroll
        for (int q = 0; q < W / 2; ++q) sig = fmaf(wa[q], relu_act(acc[q >> 4][q & 15]), sig);
        sig += __shfl_xor(sig, 32);
        sig += net.balpha;
        if (hh == 0 && s_out < A.n) A.out[s_out] = sig;
    }
}

// ======================================================================= small kernels
__global__ void near_far_kernel(const float* __restrict__ rb, int stride, int64_t n, const float* __restrict__ cyls,
                                const int32_t* __restrict__ ray_pose, float* __restrict__ near_out,
                                float* __restrict__ far_out, uint8_t* __restrict__ qnan) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float* r = rb + i * stride;
    const float* cy = cyls + 5 * (ray_pose ? ray_pose[i] : 0);
    const float nearv = r[6], farv = r[7];
    // g_axes = [0, -1]: the x-z ground plane (ray_utils.py:292-327)
    const float rn0 = r[0] + r[3] * nearv, rn1 = r[2] + r[5] * nearv;
    const float rf0 = r[0] + r[3] * farv, rf1 = r[2] + r[5] * farv;
    const float nc0 = cy[0] - rn0, nc1 = cy[1] - rn1;
    const float nf0 = rf0 - rn0, nf1 = rf1 - rn1;
    const float nfn = norm2(nf0, nf1);
    const float scale = norm2(r[3], r[5]);
    const float cross = nc0 * nf1 - nc1 * nf0;
    const float dist = fabsf(cross) / nfn;
    const float rad = cy[2];
    const float Q = sqrtf(rad * rad - dist * dist);
    const float K = (nc0 * nf0 + nc1 * nf1) / nfn;
    const float mask = (Q < K) ? 1.0f : 0.0f;
    near_out[i] = nearv + (mask * (K - Q)) / scale;
    far_out[i] = nearv + (K + Q) / scale;
    qnan[i] = (Q != Q) ? 1 : 0;
}

// one workgroup per chunk: NaN rows <- np.nanmean of the chunk (ray_utils.py:328-342)
__global__ void nan_fill_kernel(const float* __restrict__ rb, int stride, int64_t n, int chunk,
                                float* __restrict__ near_io, float* __restrict__ far_io,
                                const uint8_t* __restrict__ qnan, float* __restrict__ scratch) {
    const int64_t c0 = (int64_t)blockIdx.x * chunk;
    const int64_t c1 = min(c0 + chunk, n);
    __shared__ int any;
    __shared__ float means[2];
    if (threadIdx.x == 0) any = 0;
    __syncthreads();
    for (int64_t i = c0 + threadIdx.x; i < c1; i += blockDim.x)
        if (near_io[i] != near_io[i]) any = 1;
    __syncthreads();
    if (!any) return;
    float* buf = scratch + c0;  // NaN -> 0 copies, one vector at a time
    for (int v = 0; v < 2; ++v) {
        const float* src = v == 0 ? near_io : far_io;
        for (int64_t i = c0 + threadIdx.x; i < c1; i += blockDim.x) buf[i - c0] = (src[i] != src[i]) ? 0.0f : src[i];
        __syncthreads();
        if (threadIdx.x == 0) {
            int64_t cnt = 0;
            for (int64_t i = c0; i < c1; ++i) cnt += (src[i] == src[i]);
            means[v] = cnt ? (float)((double)np_pairwise_sum(buf, c1 - c0) / (double)cnt) : __int_as_float(0x7fc00000);
        }
        __syncthreads();
    }
    for (int64_t i = c0 + threadIdx.x; i < c1; i += blockDim.x) {
        if (qnan[i]) {
            const float* r = rb + i * stride;
            near_io[i] = (means[0] != means[0]) ? r[6] : means[0];
            far_io[i] = (means[1] != means[1]) ? r[7] : means[1];
        }
    }
}

// A frame's traced pixels: an explicit index list, or (idx == NULL) the row-major half-open box
// [x0, x0 + bw) x [y0, ...) of kp_to_valid_rays (ray_utils.py:127-130) generated on the fly.
struct PixelSet {
    const int64_t* idx;
    int64_t x0, y0, bw;
    __device__ __forceinline__ int64_t pixel(int64_t t, int W) const {
        return idx ? idx[t] : (y0 + t / bw) * W + x0 + t % bw;
    }
};

__global__ void gen_rays_kernel(const float* __restrict__ c2w, int H, int W, float fx, float fy, float cx, float cy,
                                PixelSet px, int64_t n, float nearv, float farv, float* __restrict__ out) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const int64_t p = px.pixel(t, W);
    const float x = (float)(p % W), y = (float)(p / W);
    // dirs = ((i - cx)/fx, -(j - cy)/fy, -1); rays_d = sum(dirs * c2w[:3,:3], -1) (ray_utils.py:22-25)
    const float d0 = (x - cx) / fx;
    const float d1 = -(y - cy) / fy;
    const float d2 = -1.0f;
    float* o = out + t * 11;
    float dd[3];
    for (int r = 0; r < 3; ++r) {
        dd[r] = (d0 * c2w[4 * r + 0] + d1 * c2w[4 * r + 1]) + d2 * c2w[4 * r + 2];
        o[r] = c2w[4 * r + 3];
        o[3 + r] = dd[r];
    }
    o[6] = nearv;
    o[7] = farv;
    const float nn = norm3(dd[0], dd[1], dd[2]);  // viewdirs = d / |d| (core/trainer.py:123)
    o[8] = dd[0] / nn;
    o[9] = dd[1] / nn;
    o[10] = dd[2] / nn;
}

__global__ void compose_fill_kernel(const float* __restrict__ bg, int white, int64_t hw, float* __restrict__ out_rgb,
                                    float* __restrict__ out_disp, float* __restrict__ out_acc) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= hw) return;
    for (int c = 0; c < 3; ++c) out_rgb[3 * p + c] = bg ? bg[3 * p + c] : (white ? 1.0f : 0.0f);
    out_disp[p] = 0.0f;
    if (out_acc) out_acc[p] = 0.0f;
}

__global__ void compose_scatter_kernel(const float* __restrict__ rgb, const float* __restrict__ disp,
                                       const float* __restrict__ acc, PixelSet px, int W, int64_t n,
                                       float* __restrict__ out_rgb, float* __restrict__ out_disp,
                                       float* __restrict__ out_acc) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t p = px.pixel(i, W);
    const float a = acc[i];
    for (int c = 0; c < 3; ++c) out_rgb[3 * p + c] = rgb[3 * i + c] + (1.0f - a) * out_rgb[3 * p + c];
    const float d = disp[i];
    out_disp[p] = (d != d) ? 0.0f : d;  // disps[isnan] = 0 (run_nerf.py:140-141)
    if (out_acc) out_acc[p] = a;
}

// full torch-order feature vectors (encode_inputs + embedders), one thread per point
__global__ void encode_points_kernel(ModelDev M, const float* __restrict__ skts, const float* __restrict__ pts,
                                     const float* __restrict__ dirs, int64_t n, float* __restrict__ feat) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int nj = M.nj, nv = 1 + 2 * M.mr, nk = 1 + 2 * M.mrv;
    const int cx = nj * nv + 3 * nj;
    const int F = cx + 3 * nj * nk;
    float* f = feat + i * F;
    const float px = pts[3 * i], py = pts[3 * i + 1], pz = pts[3 * i + 2];
    const float dx = dirs[3 * i], dy = dirs[3 * i + 1], dz = dirs[3 * i + 2];
    for (int j = 0; j < nj; ++j) {
        float S[12];
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 4; ++c) S[4 * r + c] = skts[j * 16 + 4 * r + c];
        float qx, qy, qz;
        joint_local(S, px, py, pz, qx, qy, qz);
        const float dist = norm3(qx, qy, qz);
        const float dn = fmaxf(dist, 1e-12f);
        const float w = M.use_cutoff ? cutoff_w(M.tau, dist, M.cutoff[j]) : 1.0f;
        f[j] = (M.use_cutoff && M.cutoff_inputs) ? dist * w : dist;
        for (int fi = 0; fi < M.mr; ++fi) {
            float s, c;
            sincosf(dist * (float)(1 << fi), &s, &c);
            f[(1 + 2 * fi) * nj + j] = s * w;
            f[(2 + 2 * fi) * nj + j] = c * w;
        }
        f[nj * nv + 3 * j + 0] = qx / dn;
        f[nj * nv + 3 * j + 1] = qy / dn;
        f[nj * nv + 3 * j + 2] = qz / dn;
        float ex, ey, ez;
        joint_rot(S, dx, dy, dz, ex, ey, ez);
        const float en = fmaxf(norm3(ex, ey, ez), 1e-12f);
        const float e[3] = {ex / en, ey / en, ez / en};
        const float wv = M.cutoff_viewdir ? cutoff_w(M.tau_v, dist, M.cutoff_v[j]) : 1.0f;
        for (int c = 0; c < 3; ++c) {
            f[cx + 3 * j + c] = (M.cutoff_viewdir && M.cutoff_inputs) ? e[c] * wv : e[c];
            for (int fi = 0; fi < M.mrv; ++fi) {
                float s, co;
                sincosf(e[c] * (float)(1 << fi), &s, &co);
                f[cx + (1 + 2 * fi) * 3 * nj + 3 * j + c] = s * wv;
                f[cx + (2 + 2 * fi) * 3 * nj + 3 * j + c] = co * wv;
            }
        }
    }
}

// ======================================================================= host side
namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define HIP_TRY(x)                                                                              \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) return fail(ANERF_EHIP, std::string(#x ": ") + hipGetErrorString(e_)); \
    } while (0)

// ---- packing (host): k-source maps into the MFMA operand order
struct Packer {
    std::vector<float> buf;
    size_t add(const std::vector<float>& v) {
        size_t off = buf.size();
        buf.insert(buf.end(), v.begin(), v.end());
        while (buf.size() % 64) buf.push_back(0.0f);  // 256-byte alignment of every array
        return off;
    }
};

// W torch [n_out][ld]; kmap(q, h) -> input column or -1; nq k-steps (even); out [nq/2][RB][64][2]
template <class F>
std::vector<float> pack_kmajor(const float* Wt, int n_out, int ld, int nq, F kmap) {
    const int RB = n_out / 32;
    std::vector<float> out((size_t)(nq / 2) * RB * 128, 0.0f);
    for (int g = 0; g < nq / 2; ++g)
        for (int rb = 0; rb < RB; ++rb)
            for (int l = 0; l < 64; ++l)
                for (int t = 0; t < 2; ++t) {
                    const int q = 2 * g + t;
                    const int col = kmap(q, l >> 5);
                    const int row = 32 * rb + (l & 31);
                    out[(((size_t)g * RB + rb) * 64 + l) * 2 + t] = col >= 0 ? Wt[(size_t)row * ld + col] : 0.0f;
                }
    return out;
}

// ng groups of F floats per lane, stored [group][F/4][64 lanes][4] (one 1 KiB b128 load per F/4);
// fn(g, s, lane) = value of slot float s of lane `lane` in group g
template <class Fn>
std::vector<float> pack_groups(int ng, int F, Fn fn) {
    std::vector<float> out((size_t)ng * F * 64, 0.0f);
    for (int g = 0; g < ng; ++g)
        for (int i = 0; i < F / 4; ++i)
            for (int l = 0; l < 64; ++l)
                for (int e = 0; e < 4; ++e) out[(((size_t)g * (F / 4) + i) * 64 + l) * 4 + e] = fn(g, 4 * i + e, l);
    return out;
}

// dense layer for mlp_layer: RBO lead groups (block rb, k-steps 0..15) then k-major groups of
// KG = 16/RBO k-steps x RBO blocks (slot float rb*KG + t); k-step q, half h -> input column
// col_off + 32 (q >> 4) + acc_row(q & 15, h)
std::vector<float> pack_layer(const float* Wt, int n_out, int ld, int col_off, int n_in) {
    const int RBO = n_out / 32, RBI = n_in / 32, KG = 16 / RBO;
    const int ng = RBO + (16 * RBI - 16) / KG;
    return pack_groups(ng, 16, [&](int g, int sl, int l) {
        int rb, q;
        if (g < RBO) {
            rb = g, q = sl;
        } else {
            rb = sl / KG, q = 16 + (g - RBO) * KG + sl % KG;
        }
        const int col = col_off + 32 * (q >> 4) + acc_row(q & 15, l >> 5);
        return Wt[(size_t)(32 * rb + (l & 31)) * ld + col];
    });
}

// bone-direction part: k-step q = 3p + c, half h -> joint p + h*njh2, column nv*nj + 3j + c;
// groups of 2 k-steps x RB blocks (slot float 2 rb + t)
std::vector<float> pack_upart(const float* Wt, int n_out, int ld, int nj, int njh2, int mr) {
    const int nv = 1 + 2 * mr, RB = n_out / 32;
    return pack_groups(3 * njh2 / 2, 2 * RB, [&](int g, int sl, int l) {
        const int rb = sl / 2, q = 2 * g + sl % 2;
        const int p = q / 3, c = q % 3;
        const int j = p + (l >> 5) * njh2;
        return j < nj ? Wt[(size_t)(32 * rb + (l & 31)) * ld + nv * nj + 3 * j + c] : 0.0f;
    });
}

// windowed part, per joint j: k-step t < mr -> (sin_t, cos_t) = columns ((1+2t)NJ + j, (2+2t)NJ + j);
// t == mr -> (dist, pad); padded to an even count.  Layout [joint][group][RB][64][2].
std::vector<float> pack_vpart(const float* Wt, int n_out, int ld, int nj, int mr) {
    const int kb = ((mr + 1) + 1) & ~1;
    std::vector<float> out;
    for (int j = 0; j < nj; ++j) {
        std::vector<float> pj = pack_kmajor(Wt, n_out, ld, kb, [&](int t, int h) {
            if (t < mr) return (1 + 2 * t + h) * nj + j;
            if (t == mr && h == 0) return j;
            return -1;
        });
        out.insert(out.end(), pj.begin(), pj.end());
    }
    return out;
}

// per-lane-half vectors [rb][h][16] of a length-n vector in accumulator row order
std::vector<float> pack_rowvec(const float* v, int n, bool half_major) {
    const int RB = n / 32;
    std::vector<float> out((size_t)RB * 32, 0.0f);
    for (int rb = 0; rb < RB; ++rb)
        for (int h = 0; h < 2; ++h)
            for (int i = 0; i < 16; ++i) {
                const size_t idx = half_major ? ((size_t)h * RB + rb) * 16 + i : ((size_t)rb * 2 + h) * 16 + i;
                out[idx] = v[32 * rb + acc_row(i, h)];
            }
    return out;
}

}  // namespace

struct anerf_model {
    anerf_model_desc desc;
    int device;
    int njh2, ngh;
    float* dev_buf;
    size_t dev_bytes;
    ModelDev md;
};

template <int WIDTH>
static void host_row_sum(const float* x, int64_t xs, int64_t n, float* out) {
    // host twin of torch_row_sum (used for the eval-mode mean framecode)
    const int64_t size = n / 4;
    int lp = 0;
    while (((int64_t)1 << lp) < size) ++lp;
    lp /= 4;
    if (lp < 4) lp = 4;
    const int64_t step = (int64_t)1 << lp, mask = step - 1;
    float acc[4][4][WIDTH] = {};
    int64_t i = 0;
    while (i + step <= size) {
        for (int64_t jj = 0; jj < step; ++jj, ++i)
            for (int k = 0; k < 4; ++k)
                for (int l = 0; l < WIDTH; ++l) acc[0][k][l] += x[((4 * i + k) * WIDTH + l) * xs];
        for (int j = 1; j < 4; ++j) {
            for (int k = 0; k < 4; ++k)
                for (int l = 0; l < WIDTH; ++l) {
                    acc[j][k][l] += acc[j - 1][k][l];
                    acc[j - 1][k][l] = 0.0f;
                }
            if ((i & (mask << (j * lp))) != 0) break;
        }
    }
    for (; i < size; ++i)
        for (int k = 0; k < 4; ++k)
            for (int l = 0; l < WIDTH; ++l) acc[0][k][l] += x[((4 * i + k) * WIDTH + l) * xs];
    for (int j = 1; j < 4; ++j)
        for (int k = 0; k < 4; ++k)
            for (int l = 0; l < WIDTH; ++l) acc[0][k][l] += acc[j][k][l];
    for (int64_t e = size * 4; e < n; ++e)
        for (int l = 0; l < WIDTH; ++l) acc[0][0][l] += x[(e * WIDTH + l) * xs];
    for (int k = 1; k < 4; ++k)
        for (int l = 0; l < WIDTH; ++l) acc[0][0][l] += acc[0][k][l];
    for (int l = 0; l < WIDTH; ++l) out[l] = acc[0][0][l];
}

static int validate_desc(const anerf_model_desc* d) {
    if (!d) return fail(ANERF_EINVAL, "desc is NULL");
    if (d->net_width != 64 && d->net_width != 128 && d->net_width != 256)
        return fail(ANERF_EINVAL, "net_width must be 64, 128 or 256");
    if (d->net_depth < 2 || d->net_depth > MAXL) return fail(ANERF_EINVAL, "net_depth outside [2, 16]");
    if (d->multires != 7 && d->multires != 10) return fail(ANERF_EINVAL, "multires must be 7 or 10");
    if (d->multires_views != 4) return fail(ANERF_EINVAL, "multires_views must be 4 (the reference default)");
    if (d->n_joints < 1 || d->n_joints > 128) return fail(ANERF_EINVAL, "n_joints outside [1, 128]");
    if (d->skip < 0) return fail(ANERF_EINVAL, "skip must be >= 0");
    if (d->framecode_ch < 0 || d->framecode_ch > 64) return fail(ANERF_EINVAL, "framecode_ch outside [0, 64]");
    if (d->framecode_ch > 0 && d->n_framecodes <= 0) return fail(ANERF_EINVAL, "n_framecodes must be > 0");
    if (d->density_scale == 0.0f) return fail(ANERF_EINVAL, "density_scale must be non-zero");
    return ANERF_OK;
}

static int pack_net(const anerf_model_desc* d, int njh2, const anerf_net_weights* w, Packer& pk,
                    std::vector<size_t>& offs) {
    const int W = d->net_width, WH = W / 2, nj = d->n_joints, mr = d->multires, mrv = d->multires_views;
    const int cin = nj * (1 + 2 * mr) + 3 * nj;
    const int nk = 1 + 2 * mrv;
    const int cv = 3 * nj * nk, cfc = d->framecode_ch;
    const int ldv = W + cv + cfc;
    for (int i = 0; i < d->net_depth; ++i)
        if (!w->pts_w[i] || !w->pts_b[i]) return fail(ANERF_EINVAL, "missing pts_linears weight");
    if (!w->alpha_w || !w->alpha_b || !w->feature_w || !w->feature_b || !w->views_w || !w->views_b || !w->rgb_w ||
        !w->rgb_b)
        return fail(ANERF_EINVAL, "missing head weight");
    if (cfc && !w->codes) return fail(ANERF_EINVAL, "framecode weights missing");
    offs.clear();
    // [0] layer 0 u part, [1..D-1] activation parts, [D] layer 0 v part, [D+1, D+2] skip u / v parts,
    // [D+3 ..] biases
    offs.push_back(pk.add(pack_upart(w->pts_w[0], W, cin, nj, njh2, mr)));
    for (int i = 1; i < d->net_depth; ++i) {
        const bool sk = (i == d->skip + 1);
        offs.push_back(pk.add(pack_layer(w->pts_w[i], W, sk ? cin + W : W, sk ? cin : 0, W)));
    }
    offs.push_back(pk.add(pack_vpart(w->pts_w[0], W, cin, nj, mr)));
    const int skl = d->skip + 1;
    if (skl < d->net_depth) {
        offs.push_back(pk.add(pack_upart(w->pts_w[skl], W, cin + W, nj, njh2, mr)));
        offs.push_back(pk.add(pack_vpart(w->pts_w[skl], W, cin + W, nj, mr)));
    } else {
        offs.push_back((size_t)-1);
        offs.push_back((size_t)-1);
    }
    for (int i = 0; i < d->net_depth; ++i) offs.push_back(pk.add(pack_rowvec(w->pts_b[i], W, false)));
    offs.push_back(pk.add(pack_rowvec(w->alpha_w, W, true)));                         // walpha
    // feature_linear has no activation, so views_linears.0's feature block and feature_linear fuse
    // into one layer on the last hidden state (nerf.py:110-112): W' = Wv_f Wf (WH x W) and
    // b' = Wv_f bf + bv, formed in double and rounded once.  The feature layer disappears.
    std::vector<float> wfused((size_t)WH * W), bfused(WH);
    for (int n = 0; n < WH; ++n) {
        std::vector<double> row(W, 0.0);
        double bacc = (double)w->views_b[n];
        for (int m = 0; m < W; ++m) {
            const double v = (double)w->views_w[(size_t)n * ldv + m];
            const float* wf = w->feature_w + (size_t)m * W;
            for (int k = 0; k < W; ++k) row[k] += v * (double)wf[k];
            bacc += v * (double)w->feature_b[m];
        }
        for (int k = 0; k < W; ++k) wfused[(size_t)n * W + k] = (float)row[k];
        bfused[n] = (float)bacc;
    }
    offs.push_back(pk.add(std::vector<float>()));                                     // wfeat (fused away)
    offs.push_back(pk.add(pack_rowvec(w->feature_b, W, false)));                      // bfeat (unused)
    offs.push_back(pk.add(pack_layer(wfused.data(), WH, W, 0, W)));                   // wview = Wv_f Wf
    {
        const int tp = (3 * nk + 3) & ~3;
        std::vector<float> t((size_t)nj * WH * tp, 0.0f);
        for (int j = 0; j < nj; ++j)
            for (int k = 0; k < nk; ++k)
                for (int c = 0; c < 3; ++c)
                    for (int n = 0; n < WH; ++n)
                        t[((size_t)j * WH + n) * tp + k * 3 + c] = w->views_w[(size_t)n * ldv + W + k * 3 * nj + 3 * j + c];
        offs.push_back(pk.add(t));                                                    // wvdir
    }
    {
        std::vector<float> t((size_t)std::max(cfc, 1) * WH, 0.0f);
        for (int m = 0; m < cfc; ++m)
            for (int n = 0; n < WH; ++n) t[(size_t)m * WH + n] = w->views_w[(size_t)n * ldv + W + cv + m];
        offs.push_back(pk.add(t));                                                    // wvcode
    }
    offs.push_back(pk.add(bfused));                                                   // bview = Wv_f bf + bv
    {
        std::vector<float> t;
        for (int c = 0; c < 3; ++c) {
            // [c][h][rb][16]
            std::vector<float> v = pack_rowvec(w->rgb_w + (size_t)c * WH, WH, true);
            t.insert(t.end(), v.begin(), v.end());
        }
        offs.push_back(pk.add(t));                                                    // wrgb
    }
    offs.push_back(pk.add(std::vector<float>(w->rgb_b, w->rgb_b + 3)));               // brgb
    {
        std::vector<float> t((size_t)(std::max(d->n_framecodes, 0) + 1) * std::max(cfc, 1), 0.0f);
        if (cfc) {
            std::memcpy(t.data(), w->codes, sizeof(float) * (size_t)d->n_framecodes * cfc);
            for (int m = 0; m < cfc; ++m) {  // codes.weight.mean(0) = torch sum over dim 0 / n
                float s;
                host_row_sum<1>(w->codes + m, cfc, d->n_framecodes, &s);
                t[(size_t)d->n_framecodes * cfc + m] = s / (float)d->n_framecodes;
            }
        }
        offs.push_back(pk.add(t));                                                    // codes
    }
    return ANERF_OK;
}

static void bind_net(const anerf_model_desc* d, const float* base, const std::vector<size_t>& o, float balpha,
                     NetDev& nd) {
    std::memset(&nd, 0, sizeof(nd));
    const int D = d->net_depth;
    size_t k = 0;
    nd.wl[0] = base + o[k++];
    for (int i = 1; i < D; ++i) nd.wl[i] = base + o[k++];
    nd.wl0v = base + o[k++];
    nd.wskipu = o[k] == (size_t)-1 ? nullptr : base + o[k];
    ++k;
    nd.wskipv = o[k] == (size_t)-1 ? nullptr : base + o[k];
    ++k;
    for (int i = 0; i < D; ++i) nd.bl[i] = base + o[k++];
    nd.walpha = base + o[k++];
    nd.wfeat = base + o[k++];
    nd.bfeat = base + o[k++];
    nd.wview = base + o[k++];
    nd.wvdir = base + o[k++];
    nd.wvcode = base + o[k++];
    nd.bview = base + o[k++];
    nd.wrgb = base + o[k++];
    nd.brgb = base + o[k++];
    nd.codes = base + o[k++];
    nd.balpha = balpha;
}

#ifdef ANERF_STAMPS
static unsigned long long* g_stamps = nullptr;
extern "C" void anerf_diag_set_stamps(unsigned long long* p) { g_stamps = p; }  // diagnostic build only
#endif

extern "C" {

int anerf_abi_version(void) { return ANERF_ABI_VERSION; }

const char* anerf_last_error(void) { return g_err.c_str(); }

int anerf_model_create(const anerf_model_desc* desc, const anerf_net_weights* coarse, const anerf_net_weights* fine,
                       const anerf_embed_params* embed, int device, anerf_model** out) {
    if (!out) return fail(ANERF_EINVAL, "out is NULL");
    *out = nullptr;
    int rc = validate_desc(desc);
    if (rc) return rc;
    if (!coarse || !embed) return fail(ANERF_EINVAL, "coarse weights / embed params are NULL");
    if (desc->has_fine && !fine) return fail(ANERF_EINVAL, "has_fine but fine weights are NULL");
    if (!embed->cutoff_dist || !embed->cutoff_dist_v) return fail(ANERF_EINVAL, "cutoff_dist is NULL");
    const int nj = desc->n_joints;
    const int njh2 = (((nj + 1) / 2) + 1) & ~1;  // joint pairs of the u part, even
    const int ngh = std::max(2 * njh2, nj + 2) / 2;  // G columns / 2: joint p + h*NJH2 at k-step p, bias at NJ
    Packer pk;
    std::vector<size_t> oc, of;
    rc = pack_net(desc, njh2, coarse, pk, oc);
    if (rc) return rc;
    if (desc->has_fine) {
        rc = pack_net(desc, njh2, fine, pk, of);
        if (rc) return rc;
    }
    const size_t off_cut = pk.add(std::vector<float>(embed->cutoff_dist, embed->cutoff_dist + nj));
    const size_t off_cutv = pk.add(std::vector<float>(embed->cutoff_dist_v, embed->cutoff_dist_v + nj));

    int prev = 0;
    HIP_TRY(hipGetDevice(&prev));
    HIP_TRY(hipSetDevice(device));
    float* dbuf = nullptr;
    const size_t bytes = pk.buf.size() * sizeof(float);
    hipError_t e = hipMalloc(&dbuf, bytes);
    if (e == hipSuccess) e = hipMemcpy(dbuf, pk.buf.data(), bytes, hipMemcpyHostToDevice);
    hipSetDevice(prev);
    if (e != hipSuccess) {
        if (dbuf) hipFree(dbuf);
        return fail(ANERF_EHIP, std::string("weight upload: ") + hipGetErrorString(e));
    }
    anerf_model* m = new anerf_model();
    m->desc = *desc;
    m->device = device;
    m->njh2 = njh2;
    m->ngh = ngh;
    m->dev_buf = dbuf;
    m->dev_bytes = bytes;
    ModelDev& md = m->md;
    std::memset(&md, 0, sizeof(md));
    md.nj = nj;
    md.njh2 = njh2;
    md.sparse = desc->use_cutoff && desc->cutoff_inputs;
    md.ngh = ngh;
    md.D = desc->net_depth;
    md.skip = desc->skip;
    md.mr = desc->multires;
    md.mrv = desc->multires_views;
    md.use_cutoff = desc->use_cutoff;
    md.cutoff_inputs = desc->cutoff_inputs;
    md.cutoff_viewdir = desc->cutoff_viewdir;
    md.cfc = desc->framecode_ch;
    md.n_codes = desc->n_framecodes;
    md.softplus = desc->density_softplus;
    md.shift = desc->softplus_shift;
    md.B = desc->density_scale;
    md.tau = embed->tau;
    md.tau_v = embed->tau_v;
    md.cutoff = dbuf + off_cut;
    md.cutoff_v = dbuf + off_cutv;
    bind_net(desc, dbuf, oc, coarse->alpha_b[0], md.net[0]);
    if (desc->has_fine) bind_net(desc, dbuf, of, fine->alpha_b[0], md.net[1]);
    else md.net[1] = md.net[0];
    *out = m;
    return ANERF_OK;
}

int anerf_model_destroy(anerf_model* m) {
    if (!m) return ANERF_OK;
    if (m->dev_buf) hipFree(m->dev_buf);
    delete m;
    return ANERF_OK;
}

size_t anerf_model_bytes(const anerf_model* m) { return m ? m->dev_bytes : 0; }

static size_t ws_near_far_bytes(int64_t n) {
    // near, far, fill scratch (floats) + qnan flags, each 256-byte aligned
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    return 3 * al(sizeof(float) * (size_t)n) + al((size_t)n);
}

size_t anerf_workspace_size(const anerf_model* m, int64_t n_rays, int32_t n_samples, int32_t n_importance) {
    (void)m; (void)n_samples; (void)n_importance;
    return ws_near_far_bytes(n_rays > 0 ? n_rays : 1);
}

static int launch_near_far(const float* rb, int stride, int64_t n, const float* cyls, const int32_t* ray_pose,
                           int chunk, char* ws, float** near_o, float** far_o, hipStream_t st) {
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    float* nearp = reinterpret_cast<float*>(ws);
    float* farp = reinterpret_cast<float*>(ws + al(sizeof(float) * n));
    float* scratch = reinterpret_cast<float*>(ws + 2 * al(sizeof(float) * n));
    uint8_t* qnan = reinterpret_cast<uint8_t*>(ws + 3 * al(sizeof(float) * n));
    const int bs = 256;
    hipLaunchKernelGGL(near_far_kernel, dim3((unsigned)((n + bs - 1) / bs)), dim3(bs), 0, st, rb, stride, n, cyls,
                       ray_pose, nearp, farp, qnan);
    const int64_t nchunks = (n + chunk - 1) / chunk;
    hipLaunchKernelGGL(nan_fill_kernel, dim3((unsigned)nchunks), dim3(256), 0, st, rb, stride, n, chunk, nearp, farp,
                       qnan, scratch);
    HIP_TRY(hipGetLastError());
    *near_o = nearp;
    *far_o = farp;
    return ANERF_OK;
}

int anerf_near_far(const float* ray_batch, int32_t ray_stride, int64_t n_rays, const float* cyls,
                   const int32_t* ray_pose, int32_t chunk, float* near_out, float* far_out, void* workspace,
                   size_t workspace_bytes, void* stream) {
    if (n_rays <= 0) return ANERF_OK;
    if (!ray_batch || !cyls || !near_out || !far_out || ray_stride < 8 || chunk <= 0)
        return fail(ANERF_EINVAL, "anerf_near_far: bad arguments");
    if (!workspace || workspace_bytes < ws_near_far_bytes(n_rays)) return fail(ANERF_EWORKSPACE, "workspace too small");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    float *np_, *fp_;
    int rc = launch_near_far(ray_batch, ray_stride, n_rays, cyls, ray_pose, chunk, (char*)workspace, &np_, &fp_, st);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(near_out, np_, sizeof(float) * n_rays, hipMemcpyDeviceToDevice, st));
    HIP_TRY(hipMemcpyAsync(far_out, fp_, sizeof(float) * n_rays, hipMemcpyDeviceToDevice, st));
    return ANERF_OK;
}

int anerf_render_rays(const anerf_model* m, const float* ray_batch, int32_t ray_stride, int64_t n_rays,
                      const float* skts, const float* cyls, int32_t n_poses, const int32_t* ray_pose,
                      const float* cams, int32_t n_samples, int32_t n_importance, int32_t chunk, int32_t precision,
                      float* rgb, float* disp, float* acc, float* rgb0, float* disp0, float* acc0, float* alpha,
                      float* alpha0, const anerf_debug* debug, void* workspace, size_t workspace_bytes,
                      void* stream) {
    if (!m) return fail(ANERF_EINVAL, "model is NULL");
    if (n_rays < 0) return fail(ANERF_EINVAL, "n_rays < 0");
    if (n_rays == 0) return ANERF_OK;
    if (precision != ANERF_PREC_FP32) return fail(ANERF_EINVAL, "unsupported precision");
    if (!ray_batch || ray_stride < 8 || !skts || !cyls || n_poses < 1 || !rgb || !disp || !acc)
        return fail(ANERF_EINVAL, "anerf_render_rays: bad arguments");
    if (n_samples < 2 || n_samples > 1024 || n_importance < 0 || n_importance > 2048)
        return fail(ANERF_EINVAL, "n_samples must be in [2, 1024], n_importance in [0, 2048]");
    if (n_importance > 0 && !m->desc.has_fine) return fail(ANERF_EINVAL, "n_importance > 0 needs a fine network");
    if (n_importance > 0 && n_samples < 3) return fail(ANERF_EINVAL, "importance sampling needs n_samples >= 3");
    if (m->desc.framecode_ch > 0 && !cams) return fail(ANERF_EINVAL, "model uses framecodes: cams required");
    if (chunk <= 0) return fail(ANERF_EINVAL, "chunk must be > 0");
    if (!workspace || workspace_bytes < anerf_workspace_size(m, n_rays, n_samples, n_importance))
        return fail(ANERF_EWORKSPACE, "workspace too small");
    int dev = -1;
    HIP_TRY(hipGetDevice(&dev));
    if (dev != m->device) return fail(ANERF_EINVAL, "current device differs from the model's device");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);

    float *nearp, *farp;
    int rc = launch_near_far(ray_batch, ray_stride, n_rays, cyls, ray_pose, chunk, (char*)workspace, &nearp, &farp, st);
    if (rc) return rc;
    if (debug && debug->near) HIP_TRY(hipMemcpyAsync(debug->near, nearp, 4 * n_rays, hipMemcpyDeviceToDevice, st));
    if (debug && debug->far) HIP_TRY(hipMemcpyAsync(debug->far, farp, 4 * n_rays, hipMemcpyDeviceToDevice, st));

    const int S = n_samples, I = n_importance, T = S + I;
    // rays per workgroup: >= 8 coarse 32-sample blocks (2 per wave) and >= 4 rays, so the per-ray
    // stages (view factor, compositing: one wave per ray) use all 4 waves
    const int nbc = (S + 31) / 32;
    int R = std::max(4, 8 / nbc);
    R = std::min(R, 8);
    const int W = m->desc.net_width;
    const int nj = m->desc.n_joints, mrv = m->desc.multires_views, D = m->desc.net_depth;
    LdsPlan P = make_plan(R, nj, W, S, T, mrv, m->ngh, D, m->njh2, true);
    if (P.total * 4 > 160 * 1024) P = make_plan(R, nj, W, S, T, mrv, m->ngh, D, m->njh2, false);
    while (R > 1 && P.total * 4 > 160 * 1024) {
        R /= 2;
        P = make_plan(R, nj, W, S, T, mrv, m->ngh, D, m->njh2, false);
    }
    if (P.total * 4 > 160 * 1024) return fail(ANERF_EINVAL, "configuration exceeds the 160 KiB LDS budget");

    RenderArgs a;
    std::memset(&a, 0, sizeof(a));
    a.rb = ray_batch;
    a.n = n_rays;
    a.stride = ray_stride;
    a.S = S;
    a.I = I;
    a.R = R;
    a.skts = skts;
    a.ray_pose = ray_pose;
    a.cams = cams;
    a.near = nearp;
    a.far = farp;
    a.rgb = rgb;
    a.disp = disp;
    a.acc = acc;
    a.rgb0 = rgb0;
    a.disp0 = disp0;
    a.acc0 = acc0;
    a.alpha = alpha;
    a.alpha0 = alpha0;
    if (debug) {
        a.dbg_z0 = debug->z_coarse;
        a.dbg_raw0 = debug->raw_coarse;
        a.dbg_w0 = debug->weights0;
        a.dbg_z1 = debug->z_fine;
        a.dbg_raw1 = debug->raw_fine;
        a.mfma_count = debug->mfma_count;
    }
#ifdef ANERF_STAMPS
    a.stamps = g_stamps;
#endif
    const unsigned grid = (unsigned)((n_rays + R - 1) / R);
    const size_t lds_bytes = (size_t)P.total * 4;
    const int mr = m->desc.multires;
#define ANERF_LAUNCH(WW, MM)                                                                         \
    do {                                                                                            \
        auto kfn = render_kernel<WW, MM>;                                                           \
        HIP_TRY(hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize,  \
                                    (int)lds_bytes));                                               \
        hipLaunchKernelGGL(kfn, dim3(grid), dim3(256), lds_bytes, st, m->md, a, P);                \
    } while (0)
    if (W == 256 && mr == 7) ANERF_LAUNCH(256, 7);
    else if (W == 128 && mr == 7) ANERF_LAUNCH(128, 7);
    else if (W == 64 && mr == 7) ANERF_LAUNCH(64, 7);
    else if (W == 256 && mr == 10) ANERF_LAUNCH(256, 10);
    else if (W == 128 && mr == 10) ANERF_LAUNCH(128, 10);
    else if (W == 64 && mr == 10) ANERF_LAUNCH(64, 10);
    else return fail(ANERF_EINVAL, "no kernel instance for this width / multires");
#undef ANERF_LAUNCH
    HIP_TRY(hipGetLastError());
    return ANERF_OK;
}

int anerf_gen_rays(const float* c2w, int32_t H, int32_t W, float focal_x, float focal_y, float center_x,
                   float center_y, int32_t has_center, const int64_t* idx, int64_t n, float nearv, float farv,
                   float* ray_batch_out, void* stream) {
    if (n == 0) return ANERF_OK;
    if (!c2w || !idx || !ray_batch_out || H <= 0 || W <= 0 || n < 0) return fail(ANERF_EINVAL, "anerf_gen_rays: bad arguments");
    const float cx = has_center ? center_x : (float)(W * 0.5);
    const float cy = has_center ? center_y : (float)(H * 0.5);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(gen_rays_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, c2w, H, W, focal_x,
                       focal_y, cx, cy, PixelSet{idx, 0, 0, 1}, n, nearv, farv, ray_batch_out);
    HIP_TRY(hipGetLastError());
    return ANERF_OK;
}

int anerf_gen_rays_box(const float* c2w, int32_t H, int32_t W, float focal_x, float focal_y, float center_x,
                       float center_y, int32_t has_center, int32_t x0, int32_t y0, int32_t x1, int32_t y1, float nearv,
                       float farv, float* ray_batch_out, void* stream) {
    if (!c2w || !ray_batch_out || H <= 0 || W <= 0 || x0 < 0 || y0 < 0 || x1 > W || y1 > H)
        return fail(ANERF_EINVAL, "anerf_gen_rays_box: bad arguments");
    if (x1 <= x0 || y1 <= y0) return ANERF_OK;
    const int64_t n = (int64_t)(x1 - x0) * (y1 - y0);
    const float cx = has_center ? center_x : (float)(W * 0.5);
    const float cy = has_center ? center_y : (float)(H * 0.5);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(gen_rays_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, c2w, H, W, focal_x,
                       focal_y, cx, cy, PixelSet{nullptr, x0, y0, x1 - x0}, n, nearv, farv, ray_batch_out);
    HIP_TRY(hipGetLastError());
    return ANERF_OK;
}

int anerf_compose(const float* rgb, const float* disp, const float* acc, const int64_t* idx, int64_t n,
                  const float* bg, int32_t white_bkgd, int64_t hw, float* out_rgb, float* out_disp, float* out_acc,
                  void* stream) {
    if (hw <= 0 || !out_rgb || !out_disp || n < 0 || (n > 0 && (!rgb || !disp || !acc || !idx)))
        return fail(ANERF_EINVAL, "anerf_compose: bad arguments");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(compose_fill_kernel, dim3((unsigned)((hw + 255) / 256)), dim3(256), 0, st, bg, white_bkgd, hw,
                       out_rgb, out_disp, out_acc);
    if (n > 0)
        hipLaunchKernelGGL(compose_scatter_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, rgb, disp, acc,
                           PixelSet{idx, 0, 0, 1}, 1, n, out_rgb, out_disp, out_acc);
    HIP_TRY(hipGetLastError());
    return ANERF_OK;
}

int anerf_compose_box(const float* rgb, const float* disp, const float* acc, int32_t x0, int32_t y0, int32_t x1,
                      int32_t y1, const float* bg, int32_t white_bkgd, int32_t H, int32_t W, float* out_rgb,
                      float* out_disp, float* out_acc, void* stream) {
    const bool empty = x1 <= x0 || y1 <= y0;
    if (H <= 0 || W <= 0 || !out_rgb || !out_disp || x0 < 0 || y0 < 0 || x1 > W || y1 > H ||
        (!empty && (!rgb || !disp || !acc)))
        return fail(ANERF_EINVAL, "anerf_compose_box: bad arguments");
    const int64_t hw = (int64_t)H * W;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(compose_fill_kernel, dim3((unsigned)((hw + 255) / 256)), dim3(256), 0, st, bg, white_bkgd, hw,
                       out_rgb, out_disp, out_acc);
    if (!empty) {
        const int64_t n = (int64_t)(x1 - x0) * (y1 - y0);
        hipLaunchKernelGGL(compose_scatter_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, rgb, disp, acc,
                           PixelSet{nullptr, x0, y0, x1 - x0}, W, n, out_rgb, out_disp, out_acc);
    }
    HIP_TRY(hipGetLastError());
    return ANERF_OK;
}

int anerf_encode_points(const anerf_model* m, const float* skts, const float* pts, const float* dirs, int64_t n_points,
                        float* feat_out, void* stream) {
    if (!m || !skts || !pts || !dirs || !feat_out || n_points < 0) return fail(ANERF_EINVAL, "anerf_encode_points: bad arguments");
    if (n_points == 0) return ANERF_OK;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(encode_points_kernel, dim3((unsigned)((n_points + 127) / 128)), dim3(128), 0, st, m->md, skts,
                       pts, dirs, n_points, feat_out);
    HIP_TRY(hipGetLastError());
    return ANERF_OK;
}

static int launch_density(const anerf_model* m, DensityArgs a, void* stream) {
    if (a.n == 0) return ANERF_OK;
    int dev = -1;
    HIP_TRY(hipGetDevice(&dev));
    if (dev != m->device) return fail(ANERF_EINVAL, "current device differs from the model's device");
    if (a.net < 0) a.net = m->desc.has_fine ? 1 : 0;  // the reference's default network (raycasters.py:616-620)
    if (a.net > 1 || (a.net == 1 && !m->desc.has_fine)) return fail(ANERF_EINVAL, "no such network");
    const int W = m->desc.net_width, mr = m->desc.multires;
    const LdsPlan P = make_density_plan(m->desc.n_joints, W, m->desc.net_depth, m->njh2);
    if (P.total * 4 > 160 * 1024) return fail(ANERF_EINVAL, "configuration exceeds the 160 KiB LDS budget");
    const int64_t nb = (a.n + 31) / 32;
    const unsigned grid = (unsigned)std::min<int64_t>((nb + 3) / 4, 256 * 32);
    const size_t lds_bytes = (size_t)P.total * 4;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
#define ANERF_LAUNCH(WW, MM)                                                                         \
    do {                                                                                            \
        auto kfn = density_kernel<WW, MM>;                                                          \
        HIP_TRY(hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize,  \
                                    (int)lds_bytes));                                               \
        hipLaunchKernelGGL(kfn, dim3(grid), dim3(256), lds_bytes, st, m->md, a, P);                \
    } while (0)
    if (W == 256 && mr == 7) ANERF_LAUNCH(256, 7);
    else if (W == 128 && mr == 7) ANERF_LAUNCH(128, 7);
    else if (W == 64 && mr == 7) ANERF_LAUNCH(64, 7);
    else if (W == 256 && mr == 10) ANERF_LAUNCH(256, 10);
    else if (W == 128 && mr == 10) ANERF_LAUNCH(128, 10);
    else if (W == 64 && mr == 10) ANERF_LAUNCH(64, 10);
    else return fail(ANERF_EINVAL, "no kernel instance for this width / multires");
#undef ANERF_LAUNCH
    HIP_TRY(hipGetLastError());
    return ANERF_OK;
}

int anerf_density_points(const anerf_model* m, const float* pts, int64_t n_points, const float* skts, int32_t net,
                         float* raw_out, void* stream) {
    if (!m || n_points < 0) return fail(ANERF_EINVAL, "anerf_density_points: bad arguments");
    if (n_points == 0) return ANERF_OK;
    if (!pts || !skts || !raw_out) return fail(ANERF_EINVAL, "anerf_density_points: bad arguments");
    DensityArgs a;
    std::memset(&a, 0, sizeof(a));
    a.pts = pts;
    a.n = n_points;
    a.skts = skts;
    a.net = net;
    a.out = raw_out;
    return launch_density(m, a, stream);
}

int anerf_density_grid(const anerf_model* m, const float* axis, int32_t res1, const float* kp0, const float* skts,
                       int32_t net, float* raw_out, void* stream) {
    if (!m || !axis || !kp0 || !skts || !raw_out || res1 < 1) return fail(ANERF_EINVAL, "anerf_density_grid: bad arguments");
    DensityArgs a;
    std::memset(&a, 0, sizeof(a));
    a.t = axis;
    a.kp0 = kp0;
    a.res1 = res1;
    a.n = (int64_t)res1 * res1 * res1;
    a.skts = skts;
    a.net = net;
    a.out = raw_out;
    return launch_density(m, a, stream);
}

}  // extern "C"
