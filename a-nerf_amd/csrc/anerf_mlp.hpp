// anerf_mlp.hpp — MFMA building blocks of the fused MLP: weight ring, dense layer with fused boundary, encoder k-streams (bone directions, windowed joints), view-direction part, trunk and one 32-sample block.
// Part of the single translation unit anerf_render.hip (included there, in order).
#pragma once

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
// Non-temporal (nt, cache-policy bit 2 on gfx950) forms for the weight streams an XCD's L2 should not
// keep: the per-joint windowed parts (touched only for the block's live joints) and the view-direction
// rows of G (once per ray and pass).  Cached like the hidden layers' streams, these push one net's
// touched set (4.3 MB in bf16x6) past the 4 MB L2, and the cyclic hidden-layer stream then misses
// (tools/probe/layer_probe_x6: 90 % of the MFMA rate up to a 3.8 MB footprint, 84 % at 4.2 MB).
#ifndef ANERF_NT_V
#define ANERF_NT_V 0
#endif
#ifndef ANERF_NT_G
#define ANERF_NT_G 0
#endif
__device__ __forceinline__ f32x2 bload2_v(__amdgpu_buffer_rsrc_t rs, int voff, int soff) {
    return __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(rs, voff, soff, ANERF_NT_V ? 2 : 0));
}
__device__ __forceinline__ f32x4 bload4_g(__amdgpu_buffer_rsrc_t rs, int voff, int soff) {
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, ANERF_NT_G ? 2 : 0));
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

// ---- bf16x3 form of mlp_layer for the dense RBI*32 -> RBO*32 activation parts (ANERF_PREC_BF16X3).
// One v_mfma_f32_32x32x16_bf16 covers 16 k (vs 2 for the f32 form); the x = x_hi + x_lo split of an
// operand costs 3 of them per product, ~5.3x the f32 MFMA rate.  The B operands are the previous
// layer's accumulators: relu, then registers 8s..8s+7 of block rb -> fragments hi/lo of k-step s,
// kept in h[rb] as [hi s0 | lo s0 | hi s1 | lo s1] (4 registers each).  Same lead / k-major group
// schedule as mlp_layer (pack_layer_x3), 6 MFMAs per 16-float group.
__device__ __forceinline__ bf16x8 frag_of(const f32x16& v, int f) {
    return __builtin_bit_cast(bf16x8, f32x4{v[4 * f], v[4 * f + 1], v[4 * f + 2], v[4 * f + 3]});
}
__device__ __forceinline__ bf16x8 frag_of(const float (&v)[16], int f) {
    return __builtin_bit_cast(bf16x8, f32x4{v[4 * f], v[4 * f + 1], v[4 * f + 2], v[4 * f + 3]});
}
__device__ __forceinline__ f32x16 split_block(const f32x16& a) {
    f32x16 o;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        bf16x8 hi, lo;
#pragma unroll
        for (int j = 0; j < 8; ++j) hi[j] = (__bf16)relu_act(a[8 * s + j]);
#pragma unroll
        for (int j = 0; j < 8; ++j) lo[j] = (__bf16)(relu_act(a[8 * s + j]) - (float)hi[j]);
        const f32x4 h4 = __builtin_bit_cast(f32x4, hi), l4 = __builtin_bit_cast(f32x4, lo);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            o[8 * s + e] = h4[e];
            o[8 * s + 4 + e] = l4[e];
        }
    }
    return o;
}

template <int RBO, int RBI>
__device__ __forceinline__ void mlp_layer_x3(f32x16 (&out)[RBO], f32x16 (&ain)[RBI], f32x16 (&h)[RBI],
                                             const float* __restrict__ bias, const float* __restrict__ wp, int lane,
                                             Ring& ring, const float* __restrict__ next) {
    static_assert(RBO <= RBI && RBO % 2 == 0, "x3 layer shape");
    constexpr int NG = RBO + (RBI - 1) * RBO;
    const int hh = lane >> 5;
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(wp);
    const __amdgpu_buffer_rsrc_t rn = make_rsrc(next);
    auto convert = [&](int rb) {
        h[rb] = split_block(ain[rb]);
        if (rb < RBO) {
            const f32x4* p = reinterpret_cast<const f32x4*>(bias + (rb * 2 + hh) * 16);
            const f32x4 v0 = p[0], v1 = p[1], v2 = p[2], v3 = p[3];
            out[rb] = f32x16{v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3],
                             v2[0], v2[1], v2[2], v2[3], v3[0], v3[1], v3[2], v3[3]};
        }
    };
    auto prefetch = [&](int g) {
        if (g + 2 < NG)
            load_group<16>(ring.v[(g + 2) % 4], rs, lane, g + 2);
        else if (NG % 4 == 0 && next)
            load_group<16>(ring.v[(g + 2) % 4], rn, lane, g + 2 - NG);
    };
    convert(0);
#pragma clang loop unroll(full)
    for (int g = 0; g < RBO; ++g) {  // lead groups: output block g, input block 0
        __builtin_amdgcn_sched_barrier(0);
        prefetch(g);
        const float (&a)[16] = ring.v[g % 4];
#pragma clang loop unroll(full)
        for (int s = 1; s >= 0; --s)  // (last-loaded fragments first)
            out[g] = mfma_x3(frag_of(a, 2 * s), frag_of(a, 2 * s + 1), frag_of(h[0], 2 * s), frag_of(h[0], 2 * s + 1),
                             out[g]);
        if (g + 1 < RBO) {
            convert(g + 1);
        } else {
#pragma clang loop unroll(full)
            for (int rb = RBO; rb < RBI; ++rb) convert(rb);
        }
    }
#pragma clang loop unroll(full)
    for (int ib = 1; ib < RBI; ++ib) {
#pragma clang loop unroll(full)
        for (int s = 0; s < 2; ++s) {
            const bf16x8 bh = frag_of(h[ib], 2 * s), bl = frag_of(h[ib], 2 * s + 1);
#pragma clang loop unroll(full)
            for (int p = 0; p < RBO / 2; ++p) {
                const int g = RBO + (ib - 1) * RBO + s * (RBO / 2) + p;
                __builtin_amdgcn_sched_barrier(0);
                prefetch(g);
                const float (&a)[16] = ring.v[g % 4];
                out[2 * p + 1] = mfma_x3(frag_of(a, 2), frag_of(a, 3), bh, bl, out[2 * p + 1]);
                out[2 * p] = mfma_x3(frag_of(a, 0), frag_of(a, 1), bh, bl, out[2 * p]);
            }
        }
    }
}

// ---- bf16x6 form (ANERF_PREC_BF16X6): x = x0 + x1 + x2 and w = w0 + w1 + w2, product ~= the six
// x_i w_j with i + j <= 2: six v_mfma_f32_32x32x16_bf16 per 16 k.  Weights are split on the host
// (bf16 RNE of the running remainder).  Activations are split here by TRUNCATION, with integer
// masks: x0 = x & 0xffff0000, r = x - x0 (exact), x1 = r & 0xffff0000, x2 = r - x1 (exact, <= 8
// significant bits, so it is a bf16), i.e. x = x0 + x1 + x2 exactly; the dropped x1 w2 + x2 w1 +
// x2 w2 are below 2^-23 of |x w| (fp32 product rounding is 2^-24).  Packing two values per dword is
// one v_perm_b32 per component.
// The activations stay f32 (relu'd) in h[]; the split of input block ib + 1 (8 value pairs ->
// T[2] = 2 k16-steps x 3 components x 4 dwords) is spread one pair at a time over the groups of
// block ib, so the VALU work sits in the MFMA gaps (a v_mfma_f32_32x32x16_bf16 hides ~5 single-issue
// VALU instructions, MI355X_MICROARCH.md), and so are the relu / bias conversions of the lead
// groups.  Weight groups are 12 floats (fragments w0, w1, w2 of one (ob, ib, s)), prefetched 3
// groups ahead in the 4-slot ring.
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
struct X6T {
    unsigned d[3][4];
    __device__ __forceinline__ bf16x8 frag(int c) const {
        return __builtin_bit_cast(bf16x8, u32x4{d[c][0], d[c][1], d[c][2], d[c][3]});
    }
};

// values a, b -> dword q of the three components (a in the low half: element 2q of the fragment)
__device__ __forceinline__ void split3_pair(float a, float b, X6T& t, int q) {
    const unsigned ua = __builtin_bit_cast(unsigned, a), ub = __builtin_bit_cast(unsigned, b);
    const float ra = a - __builtin_bit_cast(float, ua & 0xffff0000u);
    const float rb = b - __builtin_bit_cast(float, ub & 0xffff0000u);
    const unsigned ura = __builtin_bit_cast(unsigned, ra), urb = __builtin_bit_cast(unsigned, rb);
    const float qa = ra - __builtin_bit_cast(float, ura & 0xffff0000u);
    const float qb = rb - __builtin_bit_cast(float, urb & 0xffff0000u);
    t.d[0][q] = __builtin_amdgcn_perm(ub, ua, 0x07060302u);
    t.d[1][q] = __builtin_amdgcn_perm(urb, ura, 0x07060302u);
    t.d[2][q] = __builtin_amdgcn_perm(__builtin_bit_cast(unsigned, qb), __builtin_bit_cast(unsigned, qa), 0x07060302u);
}

// value pair p (0..7) of a 16-value input block: k16-step p >> 2, dword p & 3
__device__ __forceinline__ void split3_block_pair(const f32x16& hb, X6T (&t)[2], int p) {
    const int s = p >> 2, q = p & 3;
#if ANERF_X6_PROBE == 2  // (diagnostic builds of tools/probe only: no split arithmetic)
    const float v = hb[8 * s + 2 * q];
    t[s].d[0][q] = t[s].d[1][q] = t[s].d[2][q] = __builtin_bit_cast(unsigned, v);
    return;
#endif
    split3_pair(hb[8 * s + 2 * q], hb[8 * s + 2 * q + 1], t[s], q);
}

// Issue-order pins of the split layers' groups (round 3, A/B on the box, tools/gpu_ab3.sh): the
// scheduler otherwise packs a group's split / relu work into one or two MFMA gaps.  bf16x6 +1.25 %,
// fp16x3 +0.4 % with at most three VALU per gap (two: +1.1 %); the same pin on u_part_x6: -0.1 %.
// The fp16 layers (round 4, with the fp16x4 four-MFMA groups): two VALU per gap +0.85 % fp16x4 over
// three, fp16x3 neutral; one +0.55 %, four +0.2 %, five -0.8 % (profiles/r04h3il_ab*.txt)
#ifndef ANERF_X6_IL
#define ANERF_X6_IL 3
#endif
#ifndef ANERF_H3_IL
#define ANERF_H3_IL 2
#endif
// One x6 group's issue order: each of the six MFMAs followed by at most one weight load and three
// VALU instructions (the split / relu / bias work of the group), so no MFMA gap carries more than
// the ~5 single-issue instructions an MFMA of this shape hides (MI355X_MICROARCH.md).
// (NM MFMAs; the first NLG each followed by NL vector-memory reads; then up to NV VALU instructions)
template <int NM, int NLG, int NL, int NV>
__device__ __forceinline__ void group_schedule() {
#pragma unroll
    for (int i = 0; i < NM; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        if (i < NLG) __builtin_amdgcn_sched_group_barrier(0x020, NL, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, NV, 0);
    }
}
__device__ __forceinline__ void x6_group_schedule() {
#if ANERF_X6_IL
    group_schedule<6, 3, 1, ANERF_X6_IL>();
#endif
}

__device__ __forceinline__ f32x16 mfma_x6(const float (&w)[16], const X6T& x, f32x16 c) {
    const bf16x8 w0 = frag_of(w, 0), w1 = frag_of(w, 1), w2 = frag_of(w, 2);
    c = mfma_bf16_32x32x16(w2, x.frag(0), c);  // small terms first
    c = mfma_bf16_32x32x16(w1, x.frag(1), c);
    c = mfma_bf16_32x32x16(w0, x.frag(2), c);
    c = mfma_bf16_32x32x16(w1, x.frag(0), c);
    c = mfma_bf16_32x32x16(w0, x.frag(1), c);
    return mfma_bf16_32x32x16(w0, x.frag(0), c);
}

// OUT_SAME: out aliases ain (hidden layers: out[rb] = bias once ain[rb] is consumed); otherwise out
// starts at zero (the view layer).  ALPHA folds sig += w_alpha . h in the fp32 path's k order.
// RELU_IN = false takes ain as it is (the training forward's feature -> view edge, no activation).
// side(g) runs after group g's prefetch (the training forward drains its stores there; NoSide: nothing).
struct NoSide {
    __device__ __forceinline__ void operator()(int) const {}
};
template <int RBO, int RBI, bool OUT_SAME, bool ALPHA, bool RELU_IN = true, class Side = NoSide>
__device__ __forceinline__ void mlp_layer_x6(f32x16 (&out)[RBO], f32x16 (&ain)[RBI], f32x16 (&h)[RBI],
                                             const float* __restrict__ bias, const float* __restrict__ wp, int lane,
                                             Ring& ring, bool preloaded, const float* __restrict__ next,
                                             const float* __restrict__ wa, float& sig, Side* side = nullptr) {
    static_assert(RBO <= RBI, "x6 layer shape");
    constexpr int NG = 2 * RBO * RBI;
    constexpr int PD = 3;  // prefetch distance (groups)
    constexpr int NQ = 2 * RBO;  // groups per input block
    const int hh = lane >> 5;
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(wp);
    const __amdgpu_buffer_rsrc_t rn = make_rsrc(next ? next : wp);
    auto convert_half = [&](int rb, int half) {  // relu of 8 inputs (+ their 8 bias outputs)
#pragma unroll
        for (int i = 8 * half; i < 8 * half + 8; ++i) h[rb][i] = RELU_IN ? relu_act(ain[rb][i]) : ain[rb][i];
        if (OUT_SAME && rb < RBO) {
            const f32x4* p = reinterpret_cast<const f32x4*>(bias + (rb * 2 + hh) * 16 + 8 * half);
            const f32x4 v0 = p[0], v1 = p[1];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                out[rb][8 * half + e] = v0[e];
                out[rb][8 * half + 4 + e] = v1[e];
            }
        }
    };
    auto alpha = [&](int ib, int s) {  // k = 16 ib + 8 s + j, the order of mlp_layer's fold
        if constexpr (ALPHA) {
            const f32x4* w4 = reinterpret_cast<const f32x4*>(wa + hh * 16 * RBI + 16 * ib + 8 * s);
            const f32x4 u0 = w4[0], u1 = w4[1];
#pragma unroll
            for (int j = 0; j < 8; ++j) sig = fmaf(j < 4 ? u0[j] : u1[j - 4], h[ib][8 * s + j], sig);
        }
    };
    if constexpr (!OUT_SAME) {
#pragma unroll
        for (int rb = 0; rb < RBO; ++rb) out[rb] = f32x16{0};
    }
    // group g + PD of this layer, or the next x6 phase's first groups; without a next phase the
    // last group is reloaded instead (harmless): loads issued on every path keep the compiler's
    // counted vmcnt waits exact (a conditional load makes the following waits drain to 0)
    const bool has_next = next != nullptr;
    auto prefetch = [&](int g) {
#if ANERF_X6_PROBE == 1  // (diagnostic builds of tools/probe only: no weight loads)
        return;
#elif ANERF_X6_PROBE == 3  // (diagnostic: loads from a 4-group, L1-resident footprint)
        load_group<12>(ring.v[(g + PD) % 4], rs, lane, (g + PD) % 4);
        return;
#endif
        if (g + PD < NG)
            load_group<12>(ring.v[(g + PD) % 4], rs, lane, g + PD);
        else if (NG % 4 == 0)
            load_group<12>(ring.v[(g + PD) % 4], rn, lane, has_next ? g + PD - NG : NG - 1);
    };
    // group (of the NQ - q0 groups from q0 on) that splits pair p of the next block
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
    // lead groups: output block g/2, input block 0, k16-step g&1; block ob + 1 is converted (a half
    // per group) under the MFMAs of block ob; block 1's split follows from group 2 on
    constexpr int QL = NQ > 2 ? 2 : NQ;  // first lead group that may split block 1
#pragma clang loop unroll(full)
    for (int g = 0; g < NQ; ++g) {
        __builtin_amdgcn_sched_barrier(0);
        prefetch(g);
        if constexpr (!std::is_same<Side, NoSide>::value) (*side)(g);
        const int ob = g >> 1, s = g & 1;
        out[ob] = mfma_x6(ring.v[g % 4], T[s], out[ob]);
        if (ob == 0) alpha(0, s);
        if (ob + 1 < RBI && (ob + 1 < RBO || ob == 0)) convert_half(ob + 1, s);
        if (RBI > 1) {
#pragma unroll
            for (int p = 0; p < 8; ++p)
                if (pair_group(p, QL) == (g < QL ? -1 : g) || (g == NQ - 1 && pair_group(p, QL) > g))
                    split3_block_pair(h[1], Tn, p);
        }
        x6_group_schedule();
    }
#pragma clang loop unroll(full)
    for (int ib = 1; ib < RBI; ++ib) {
        T[0] = Tn[0];
        T[1] = Tn[1];
        // blocks >= max(RBO, 2) are converted under the first two groups of the block before them
        const bool conv_next = ib + 1 < RBI && ib + 1 >= (RBO > 2 ? RBO : 2);
        const int q0 = conv_next ? (NQ > 2 ? 2 : NQ) : 0;
#pragma clang loop unroll(full)
        for (int q = 0; q < NQ; ++q) {
            const int s = q / RBO, ob = q % RBO;
            const int g = NQ + (ib - 1) * NQ + q;
            __builtin_amdgcn_sched_barrier(0);
            prefetch(g);
            if constexpr (!std::is_same<Side, NoSide>::value) (*side)(g);
            out[ob] = mfma_x6(ring.v[g % 4], T[s], out[ob]);
            if (ob == RBO - 1) alpha(ib, s);
            if (ib + 1 < RBI) {
                if (conv_next && q < 2) convert_half(ib + 1, q);
#pragma unroll
                for (int p = 0; p < 8; ++p)
                    if (pair_group(p, q0) == q || (q == NQ - 1 && pair_group(p, q0) > q))
                        split3_block_pair(h[ib + 1], Tn, p);
            }
            x6_group_schedule();
        }
    }
}

// ---- fp16x3 form (ANERF_PREC_FP16X3): per-sample power-of-two scaling, then x = x0 + x1 and
// w = w0 + w1 in fp16 (22 significant bits each), product ~= x0 w0 + x0 w1 + x1 w0: three
// v_mfma_f32_32x32x16_f16 per 16 k (half of bf16x6's six) with exact fp16 products and fp32
// accumulation; the dropped x1 w1 is ~2^-22 of |x w|.  fp16's narrow exponent range is handled by
// scaling: the weights of a layer by 2^ew on the host (max |w| in [2^10, 2^11)), the input of every
// sample (the 32-sample block's column, a lane and its partner lane l ^ 32) by t = 2^shift so its
// largest relu'd activation lies in [2^10, 2^11) — values far below the sample's maximum lose
// only what is below ~2^-34 of that maximum.  (Measured on gfx950: with both operands' maxima at
// 2^13..2^15 — products ~2^28, 16-term dot products past ~2^31 — the f16 MFMA returned wrong sums
// for some samples; at 2^12 and below it matched the fp32 path.  2^10 leaves a 2^5 margin.)
// The accumulators then hold the layer's output times 2^es (es = a per-sample integer: all scales
// are exact powers of two, so the scaling itself never rounds); the next layer rescales from
// there, the skip layer's x parts scale their B operands to it and the heads unscale.
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
struct H3T {
    unsigned d[2][4];
    __device__ __forceinline__ f16x8 frag(int c) const {
        return __builtin_bit_cast(f16x8, u32x4{d[c][0], d[c][1], d[c][2], d[c][3]});
    }
};

__device__ __forceinline__ float pow2f(int e) { return __builtin_bit_cast(float, (e + 127) << 23); }  // |e| <= 126

// values a, b (relu'd, in the input's units) times t -> dword q of the two fp16 components: the high
// part rounds x to 11 significant bits in the f32 encoding (exact in fp16), the low part is the
// exact remainder rounded to nearest even (v_cvt_pk_f16_f32), so x0 + x1 is within 2^-23 |x| of x
// (a quarter of the values are not exact: the remainder can need 12 bits)
#ifndef ANERF_SPLIT_MIX
#define ANERF_SPLIT_MIX 1
#endif
#ifdef ANERF_H3_STAMPS  // (tools/probe/h4_probe.hip -DPROBE_STAMPS only: per-phase cycles of a layer, summed
                        // into ANERF_H3_STAMPS[4] = preamble, lead groups, middle blocks, last block)
#define ANERF_H3_HOOK(b)                                                       \
    do {                                                                       \
        const unsigned long long now_ = __builtin_amdgcn_s_memtime();          \
        ph_acc[ph_cur] += now_ - ph_last;                                      \
        ph_last = now_;                                                        \
        ph_cur = (b);                                                          \
    } while (0)
#else
#define ANERF_H3_HOOK(b) do { } while (0)
#endif
__device__ __forceinline__ void split2_pair(float a, float b, float t, H3T& T, int q) {
    typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
    const float xa = a * t, xb = b * t;
#if ANERF_SPLIT_MIX
    // (round 5) the high parts as one RNE conversion of the pair, the remainders x - x0 read the fp16 high
    // part straight from the packed pair by v_fma_mix_f32 (exact: x - x0 fits 13 bits), then one RNE
    // conversion: 4 instructions per pair where the integer rounding took 6
    const unsigned hi = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2{xa, xb}), f16x2));
    float la, lb;
    asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=v"(la) : "v"(hi), "v"(xa));
    asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(lb) : "v"(hi), "v"(xb));
    T.d[0][q] = hi;
    T.d[1][q] = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2{la, lb}), f16x2));
#else
    const float ha = __builtin_bit_cast(float, (__builtin_bit_cast(unsigned, xa) + 0x1000u) & 0xffffe000u);
    const float hb = __builtin_bit_cast(float, (__builtin_bit_cast(unsigned, xb) + 0x1000u) & 0xffffe000u);
    T.d[0][q] = __builtin_bit_cast(unsigned, __builtin_amdgcn_cvt_pkrtz(ha, hb));
    T.d[1][q] = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2{xa - ha, xb - hb}), f16x2));
#endif
}

// fp16x4 with the x1 w1 product in fp8 (ANERF_F8_X1W1, round 5): the same split, and the low parts x1 also
// as e4m3 bytes of the x1 w1 MFMA's B operand (x1 scaled by 2^8 into e4m3's range; the MFMA's block scale
// 2^-8 undoes it): byte 2 (p & 1) .. +1 of dword `d` (two pairs per dword)
#ifndef ANERF_F8_X1W1
#define ANERF_F8_X1W1 0
#endif
// (round 6, experiment switch, off) the hidden layers' per-sample fp16 scale from a bound formed by the previous
// layer (mlp_layer_h3): measured -0.6 % (1.2048 vs 1.2118 M rays/s, three alternating runs on one box, outputs
// unchanged to 1e-8, profiles/r06i_ab_h3_bound.txt): the converts' maxima and 40 B/lane more scratch cost what
// the drain before the scale saved
#ifndef ANERF_H3_BOUND
#define ANERF_H3_BOUND 0
#endif
template <bool HI_WORD>
__device__ __forceinline__ void split2_pair_f8(float a, float b, float t, H3T& T, int q, unsigned& x8) {
    typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
    const float xa = a * t, xb = b * t;
    const unsigned hi = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2{xa, xb}), f16x2));
    float la, lb;
    asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=v"(la) : "v"(hi), "v"(xa));
    asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(lb) : "v"(hi), "v"(xb));
    T.d[0][q] = hi;
    T.d[1][q] = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2{la, lb}), f16x2));
    x8 = (unsigned)__builtin_amdgcn_cvt_pk_fp8_f32(la * 256.0f, lb * 256.0f, (int)x8, HI_WORD);
}

__device__ __forceinline__ void split2_block_pair_f8(const f32x16& hb, float t, H3T (&T)[2], int p,
                                                     unsigned (&X8)[8], int half) {
    const int s = p >> 2, q = p & 3;
    if (p & 1)
        split2_pair_f8<true>(hb[8 * s + 2 * q], hb[8 * s + 2 * q + 1], t, T[s], q, X8[4 * half + (p >> 1)]);
    else
        split2_pair_f8<false>(hb[8 * s + 2 * q], hb[8 * s + 2 * q + 1], t, T[s], q, X8[4 * half + (p >> 1)]);
}

__device__ __forceinline__ void split2_block_pair(const f32x16& hb, float t, H3T (&T)[2], int p) {
    const int s = p >> 2, q = p & 3;
#if ANERF_X6_PROBE == 2  // (diagnostic builds of tools/probe only: no split arithmetic)
    T[s].d[0][q] = T[s].d[1][q] = __builtin_bit_cast(unsigned, hb[8 * s + 2 * q]);
    return;
#endif
    split2_pair(hb[8 * s + 2 * q], hb[8 * s + 2 * q + 1], t, T[s], q);
}

// mlp_layer_h3's group: three MFMAs, the ring slot's four loads (even groups) after the first two
// (NP = 3: fp16x3, NP = 4: fp16x4)
#ifndef ANERF_H3_NLG  // (experiments: MFMAs followed by loads, loads after each; NLG x NL = 4)
#define ANERF_H3_NLG 2
#endif
#ifndef ANERF_H3_LEAD_IL  // VALU per MFMA gap in the lead groups (input copies + bias initialisation; round 5
                          // A/B: 4 +0.2 % over 2, 6 -0.2 %, profiles/r05e_ab.txt)
#define ANERF_H3_LEAD_IL 4
#endif
template <int NP, int NV = ANERF_H3_IL>
__device__ __forceinline__ void h3_group_schedule() {
#if ANERF_H3_IL
    group_schedule<NP, ANERF_H3_NLG, 4 / ANERF_H3_NLG, NV>();
#endif
}

__device__ __forceinline__ f32x16 mfma_f16_32x32x16(f16x8 a, f16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

// group `half` (0 / 1) of a 16-float ring slot: fragments w0 (floats 8 half .. +3), w1 (+4 .. +7).
// NP = 4 (ANERF_PREC_FP16X4) adds x1 w1: the product is then (x - r_x)(w - r_w) with |r_x| <= 2^-23 |x|
// and |r_w| <= 2^-23 |w| (the split remainders), i.e. within ~2^-22 of |x w| — the same bound as
// bf16x6's dropped x1 w2 + x2 w1 + x2 w2 + r_w terms — with four products instead of six.
template <int NP>
__device__ __forceinline__ f32x16 mfma_h3(const float (&w)[16], int half, const H3T& x, f32x16 c) {
    const int o = 8 * half;
    const f16x8 w0 = __builtin_bit_cast(f16x8, f32x4{w[o], w[o + 1], w[o + 2], w[o + 3]});
    const f16x8 w1 = __builtin_bit_cast(f16x8, f32x4{w[o + 4], w[o + 5], w[o + 6], w[o + 7]});
    if constexpr (NP == 4) c = mfma_f16_32x32x16(w1, x.frag(1), c);
    c = mfma_f16_32x32x16(w1, x.frag(0), c);  // small terms first
    c = mfma_f16_32x32x16(w0, x.frag(1), c);
    return mfma_f16_32x32x16(w0, x.frag(0), c);
}

// The input scale t = 2^shift of one sample: its largest relu'd input (signed-integer max of the
// bit patterns, 0 for all-negative / zero inputs; NaN stays large) over this lane's and the partner
// lane's values, scaled into [2^10, 2^11).  es: exponent of the units the input is in; on return the units of this layer's
// output, es + shift + ew, kept within [-100, 60] so that bias * 2^es stays finite.
// h3_scale_bits: the same from m, the bit pattern of a sample's largest relu'd input -- or of a bound on it (the
// scaled maximum then lies at or below [2^10, 2^11): never above, the fp16 MFMA's range stays safe).
__device__ __forceinline__ float h3_scale_bits(int m, int& es, int ew, int top, int cap = 60) {
    int shift = m > 0 ? top - (m >> 23) : 0;  // (m >> 23: the biased exponent; top = 127 + 10)
    // (cap: the skip layer's h part keeps its output units at most 2^cap, so that the fp16 x parts'
    // features, scaled into those units, stay in range: enc16_units)
    shift = max(shift, -100 - es - ew);
    shift = min(shift, cap - es - ew);
    shift = min(max(shift, -126), 126);
    es += shift + ew;
    return pow2f(shift);
}

template <int RBI>
__device__ __forceinline__ float h3_scale(const f32x16 (&a)[RBI], int& es, int ew, int top, int cap = 60) {
    int m = 0;
#pragma unroll
    for (int rb = 0; rb < RBI; ++rb)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            // (through a scalar: hipcc's __builtin_bit_cast of an ext-vector element lvalue reads
            // element 0 of the vector, whatever the index)
            const float v = a[rb][i];
            m = max(m, __builtin_bit_cast(int, v));
        }
    m = max(m, __shfl_xor(m, 32));
    return h3_scale_bits(m, es, ew, top, cap);
}

// mlp_layer_x6's schedule with 8-float groups (3 MFMAs each), two groups per ring slot (slot
// (g / 2) % 4, prefetched 3 slots = 6 groups ahead).  OUT_SAME layers alias out and ain; bias * 2^es
// initialises the outputs.  ALPHA folds sig += w_alpha . h with h in the INPUT's units.
// (round 6) Bound-based scale: with use_bnd the per-sample scale comes from *bnd, a bound on the sample's largest
// relu'd input (bit pattern, in the input's units) that the PREVIOUS layer formed in the middle of its MFMAs,
// instead of the maximum over all 128 inputs, which needed every MFMA of the previous layer to retire first
// (h3_scale: the drain at each layer boundary).  A hidden layer (OUT_SAME, RBO == RBI) with rsum > 0 forms the
// bound for the next: the true maximum M of its relu'd inputs (taken as its converts run, both lanes of the
// sample) through |y_i| <= sum_k |W_ik| |x_k| + |b_i| <= rsum M + bmax (rsum, bmax: host constants of this
// layer, real units), in the output's units and widened by 2^-10 for the fp32 rounding of its own arithmetic.
template <int RBO, int RBI, bool OUT_SAME, bool ALPHA, int NP = 3>
__device__ __forceinline__ void mlp_layer_h3(f32x16 (&out)[RBO], f32x16 (&ain)[RBI], f32x16 (&h)[RBI],
                                             const float* __restrict__ bias, const float* __restrict__ wp, int lane,
                                             Ring& ring, bool preloaded, const float* __restrict__ next,
                                             const float* __restrict__ wa, float& sig, int& es, int ew, int top,
                                             int cap = 60, const float* __restrict__ w8 = nullptr, bool use_bnd = false,
                                             int* bnd = nullptr, float rsum = -1.0f, float bmax = 0.0f) {
    static_assert(RBO <= RBI, "h3 layer shape");
    // F8: fp16x4 with x1 w1 as one v_mfma_scale_f32_32x32x64_f8f6f4 (e4m3) per output block and pair of
    // input blocks (64 k) instead of four f16 MFMAs: w8 holds the e4m3 w1 groups (pack_layer_f8)
    constexpr bool F8 = (NP == 4) && ANERF_F8_X1W1 && (RBI % 2 == 0);
    constexpr int NPG = F8 ? 3 : NP;  // f16 products per 16 k
#ifdef ANERF_H3_STAMPS
    unsigned long long ph_last = __builtin_amdgcn_s_memtime(), ph_acc[4] = {0, 0, 0, 0};
    int ph_cur = 0;
#endif
    constexpr int NG = 2 * RBO * RBI;
    constexpr int NS = NG / 2;  // ring slots of this layer
    constexpr int PS = 2;       // prefetch distance (slots)
    constexpr int NQ = 2 * RBO;  // groups per input block
    const int hh = lane >> 5;
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(wp);
    const __amdgpu_buffer_rsrc_t rn = make_rsrc(next ? next : wp);
#if ANERF_X6_PROBE == 4  // (diagnostic builds of tools/probe only: no per-sample scale)
    const float t = 1.0f;
#else
    const float t = use_bnd ? h3_scale_bits(*bnd, es, ew, top, cap) : h3_scale<RBI>(ain, es, ew, top, cap);
#endif
    const float S = pow2f(es);
    constexpr bool MKB = OUT_SAME && RBO == RBI;  // (hidden layers: the true input maximum for the next bound)
    int mx = 0;
    auto convert_half = [&](int rb, int half) {  // relu of 8 inputs (+ their 8 scaled bias outputs)
#pragma unroll
        for (int i = 8 * half; i < 8 * half + 8; ++i) h[rb][i] = relu_act(ain[rb][i]);
        if constexpr (MKB) {  // (integer maxima of the bit patterns, three operands each)
#pragma unroll
            for (int i = 8 * half; i < 8 * half + 8; i += 2) {
                const float a = h[rb][i], b = h[rb][i + 1];
                mx = max(mx, max(__builtin_bit_cast(int, a), __builtin_bit_cast(int, b)));
            }
        }
        if (OUT_SAME && rb < RBO) {
            const f32x4* p = reinterpret_cast<const f32x4*>(bias + (rb * 2 + hh) * 16 + 8 * half);
            const f32x4 v0 = p[0], v1 = p[1];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                out[rb][8 * half + e] = v0[e] * S;
                out[rb][8 * half + 4 + e] = v1[e] * S;
            }
        }
    };
    auto alpha = [&](int ib, int s) {  // k = 16 ib + 8 s + j, the order of mlp_layer's fold
        if constexpr (ALPHA) {
            const f32x4* w4 = reinterpret_cast<const f32x4*>(wa + hh * 16 * RBI + 16 * ib + 8 * s);
            const f32x4 u0 = w4[0], u1 = w4[1];
#pragma unroll
            for (int j = 0; j < 8; ++j) sig = fmaf(j < 4 ? u0[j] : u1[j - 4], h[ib][8 * s + j], sig);
        }
    };
    if constexpr (!OUT_SAME) {
#pragma unroll
        for (int rb = 0; rb < RBO; ++rb) out[rb] = f32x16{0};
    }
    // slot G + PS of this layer at its first group, or the next h3 phase's first slots (this layer's
    // last slot again without one: harmless; unconditional loads keep the counted vmcnt waits exact)
    const bool has_next = next != nullptr;
    auto prefetch = [&](int g) {
#if ANERF_X6_PROBE == 1  // (diagnostic builds of tools/probe only: no weight loads)
        return;
#endif
        if (g & 1) return;
        const int G = g >> 1;
        if (G + PS < NS)
            load_group<16>(ring.v[(G + PS) % 4], rs, lane, G + PS);
        else if (NS % 4 == 0)
            load_group<16>(ring.v[(G + PS) % 4], rn, lane, has_next ? G + PS - NS : NS - 1);
    };
    auto pair_group = [](int p, int q0) { return q0 + (p * (NQ - q0 > 0 ? NQ - q0 : 1)) / 8; };
    if (!preloaded) {
#pragma unroll
        for (int G = 0; G < PS && G < NS; ++G) load_group<16>(ring.v[G], rs, lane, G);
    }
    convert_half(0, 0);
    convert_half(0, 1);
    H3T T[2], Tn[2];
    // (F8) e4m3 x1 of input blocks 2c, 2c + 1 in X8[c & 1] (block b: half b & 1); w1 groups in a 2-slot ring
    unsigned X8[2][8];
    float W8[2][16];
    const __amdgpu_buffer_rsrc_t r8 = make_rsrc(w8 ? w8 : wp);
    auto split_block_pair = [&](int b, int p, H3T (&TT)[2]) {
        if constexpr (F8) split2_block_pair_f8(h[b], t, TT, p, X8[(b >> 1) & 1], b & 1);
        else split2_block_pair(h[b], t, TT, p);
    };
    auto load8 = [&](int c, int o8) {  // w1 group (c, o8): output block o8, input blocks 2c, 2c + 1
        if constexpr (F8) load_group<8>(W8[o8 & 1], r8, lane, c * RBO + o8);
    };
    auto mfma8 = [&](int c, int o8) {
        if constexpr (F8) {
            typedef int i32x8 __attribute__((ext_vector_type(8)));
            typedef float f32x8 __attribute__((ext_vector_type(8)));
            const float (&w)[16] = W8[o8 & 1];
            const unsigned (&x)[8] = X8[c & 1];
            const i32x8 a = __builtin_bit_cast(i32x8, (f32x8){w[0], w[1], w[2], w[3], w[4], w[5], w[6], w[7]});
            const i32x8 bx = i32x8{(int)x[0], (int)x[1], (int)x[2], (int)x[3], (int)x[4], (int)x[5], (int)x[6], (int)x[7]};
            // (e4m3 both; block scales 2^-8 (E8M0 119) undo the 2^8 of the packed w1 and of x1)
            out[o8] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, bx, out[o8], 0, 0, 0, 119, 0, 119);
        }
    };
#pragma unroll
    for (int p = 0; p < 8; ++p) split_block_pair(0, p, T);
    constexpr int QL = NQ > 2 ? 2 : NQ;
#pragma clang loop unroll(full)
    for (int g = 0; g < NQ; ++g) {
        __builtin_amdgcn_sched_barrier(0);
        ANERF_H3_HOOK(1);
        prefetch(g);
        if (F8 && g == NQ - 1) load8(0, 0);
        const int ob = g >> 1, s = g & 1;
        out[ob] = mfma_h3<NPG>(ring.v[(g >> 1) % 4], g & 1, T[s], out[ob]);
        if (ob == 0) alpha(0, s);
        if (ob + 1 < RBI && (ob + 1 < RBO || ob == 0)) convert_half(ob + 1, s);
        if (RBI > 1) {
#pragma unroll
            for (int p = 0; p < 8; ++p)
                if (pair_group(p, QL) == (g < QL ? -1 : g) || (g == NQ - 1 && pair_group(p, QL) > g))
                    split_block_pair(1, p, Tn);
        }
        h3_group_schedule<NPG, ANERF_H3_LEAD_IL>();
    }
    if constexpr (MKB) {  // every input converted: the next layer's bound, under this layer's MFMAs
        if (bnd) {
            mx = max(mx, __shfl_xor(mx, 32));
            const float M = __builtin_bit_cast(float, mx) * t * pow2f(ew);  // (output units; powers of two: exact)
            const float B = fmaf(rsum, M, bmax * S) * (1.0f + 0x1p-10f);
            *bnd = rsum > 0.0f ? __builtin_bit_cast(int, B) : -1;
        }
    }
#pragma clang loop unroll(full)
    for (int ib = 1; ib < RBI; ++ib) {
        T[0] = Tn[0];
        T[1] = Tn[1];
        const bool conv_next = ib + 1 < RBI && ib + 1 >= (RBO > 2 ? RBO : 2);
        const int q0 = conv_next ? (NQ > 2 ? 2 : NQ) : 0;
#pragma clang loop unroll(full)
        for (int q = 0; q < NQ; ++q) {
            const int s = q / RBO, ob = q % RBO;
            const int g = NQ + (ib - 1) * NQ + q;
            // (F8) odd input blocks: the x1 w1 MFMA of output block q >> 1 in odd groups, its successor's
            // w1 group loaded there; even blocks load the next pair's first group in their last group
            const bool f8mm = F8 && (ib & 1) && (q & 1);
            __builtin_amdgcn_sched_barrier(0);
            ANERF_H3_HOOK(ib + 1 < RBI ? 2 : 3);
            prefetch(g);
            if (F8 && !(ib & 1) && q == NQ - 1) load8(ib / 2, 0);
            out[ob] = mfma_h3<NPG>(ring.v[(g >> 1) % 4], g & 1, T[s], out[ob]);
            if (f8mm) {
                mfma8(ib / 2, q >> 1);
                if ((q >> 1) + 1 < RBO) load8(ib / 2, (q >> 1) + 1);
            }
            if (ob == RBO - 1) alpha(ib, s);
            if (ib + 1 < RBI) {
                if (conv_next && q < 2) convert_half(ib + 1, q);
#pragma unroll
                for (int p = 0; p < 8; ++p)
                    if (pair_group(p, q0) == q || (q == NQ - 1 && pair_group(p, q0) > q))
                        split_block_pair(ib + 1, p, Tn);
            }
            if (f8mm)
                h3_group_schedule<NPG + 1>();
            else
                h3_group_schedule<NPG>();
        }
    }
    __builtin_amdgcn_sched_barrier(0);
    ANERF_H3_HOOK(0);
#ifdef ANERF_H3_STAMPS
    if ((threadIdx.x & 63) == 0)
        for (int i = 0; i < 4; ++i) atomicAdd(ANERF_H3_STAMPS + i, ph_acc[i]);
#endif
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

// The mask is wave-uniform (built from ballots), but the compiler loses that through the struct and
// then keeps it -- and every joint index popped from it -- in VGPRs: each per-joint weight load's
// scalar offset became a waterfall loop (readfirstlane / compare / exec loop around every
// buffer_load).  Read it back into SGPRs once.
__device__ __forceinline__ uint64_t uniform64(uint64_t v) {
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

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
// (with --cutoff_bones) cut[3NJ + j] = c^b_j (bone directions);
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
    for (int j = tid; j < (M.bone_cut ? 4 : 3) * M.nj; j += blockDim.x) {
        const int k = j % M.nj;
        cut[j] = j < M.nj       ? M.cutoff[k]
                 : j < 2 * M.nj ? M.cutoff_v[k]
                 : j < 3 * M.nj ? live_thr2(M.tau, M.cutoff[k])
                                : M.cutoff_b[k];
    }
}

// One joint's skeleton row (3x4 of the world->joint transform) and live threshold, loaded from
// LDS into registers two MFMA groups before use, so the encoder math never waits on LDS.
struct JRow {
    f32x4 a, b, c;
    float thr2, cv, cb;
};

__device__ __forceinline__ JRow load_row(const float* __restrict__ sk, const float* __restrict__ cut, int j, int nj,
                                         bool bone_cut) {
    const int jc = j < nj ? j : 0;
    const f32x4* p = reinterpret_cast<const f32x4*>(sk + 12 * jc);
    return JRow{p[0], p[1], p[2], cut[2 * nj + jc], cut[nj + jc], bone_cut ? cut[3 * nj + jc] : 0.0f};
}

// bone direction u_j = q / max(|q|, 1e-12) of this lane's sample (q * rsq(max(|q|^2, 1e-24)),
// within 2 ulp) and whether the joint's window may be non-zero (d^2 < thr2, conservative, see
// live_thr2).  Branch-free (per-lane selects) so that it stays in the MFMA region it is
// scheduled into.
// With WV, also the joint's view-direction window w'_j = 1 - sigmoid(tau' (|q| - c'_j)) (hardware
// sqrt/exp2/rcp, a few ulp; 0 for padding joints or without cutoff_viewdir) for the view layer.
// (BC: -1 reads M.bone_cut in a uniform branch, 0 / 1 fix it at compile time, 2 selects — no branch inside
// an MFMA region)
template <bool WV, int BC = -1>
__device__ __forceinline__ void u_joint(const ModelDev& M, const JRow& r, bool valid, float px, float py, float pz,
                                        float& u0, float& u1, float& u2, bool& live, float& wv) {
#ifdef ANERF_EXP_UFAST  // timing experiment only (stamps build): encoder VALU removed
    u0 = px * r.a[0]; u1 = py; u2 = pz; live = false; wv = 0.0f; return;
#endif
    float qx = fmaf(r.a[3], 1.0f, fmaf(r.a[2], pz, fmaf(r.a[1], py, r.a[0] * px)));
    float qy = fmaf(r.b[3], 1.0f, fmaf(r.b[2], pz, fmaf(r.b[1], py, r.b[0] * px)));
    float qz = fmaf(r.c[3], 1.0f, fmaf(r.c[2], pz, fmaf(r.c[1], py, r.c[0] * px)));
    qx = mask_f(qx, valid);
    qy = mask_f(qy, valid);
    qz = mask_f(qz, valid);
    const float d2 = fmaf(qz, qz, fmaf(qy, qy, qx * qx));
    const float inv = __builtin_amdgcn_rsqf(fmaxf(d2, 1e-24f));
    u0 = qx * inv;
    u1 = qy * inv;
    u2 = qz * inv;
    if constexpr (BC == 2) {  // (the window as a select: both sides computed, no branch)
        const float wb = 1.0f - __builtin_amdgcn_rcpf(
                                    1.0f + __builtin_amdgcn_exp2f(-(M.tau_b * (__builtin_amdgcn_sqrtf(d2) - r.cb)) *
                                                                  1.44269504f));
        const float f = M.bone_cut ? wb : 1.0f;
        u0 *= f;
        u1 *= f;
        u2 *= f;
    } else if (BC > 0 || (BC < 0 && M.bone_cut)) {  // --cutoff_bones: u_j w_b (uniform branch), w_b = 1 - sigmoid(tau_b (|q| - c^b_j))
        const float wb = 1.0f - __builtin_amdgcn_rcpf(
                                    1.0f + __builtin_amdgcn_exp2f(-(M.tau_b * (__builtin_amdgcn_sqrtf(d2) - r.cb)) *
                                                                  1.44269504f));
        u0 *= wb;
        u1 *= wb;
        u2 *= wb;
    }
    live = valid & (!M.sparse | !(d2 >= r.thr2));  // (no short-circuit: no branch; NaN -> live)
    if constexpr (WV) {
        const float d = __builtin_amdgcn_sqrtf(d2);
        const float e = __builtin_amdgcn_exp2f(-(M.tau_v * (d - r.cv)) * 1.44269504f);
        const float w = 1.0f - __builtin_amdgcn_rcpf(1.0f + e);
        // select by an integer mask: a ?: on an expensive operand becomes an exec-masked branch,
        // which splits the MFMA region this math is interleaved into
        wv = mask_f(w, valid & (M.cutoff_viewdir != 0));
    }
}

// The geometry of pair-of-pairs pp+1 is computed under the MFMAs of pp (software pipeline:
// between two sched_barriers the scheduler interleaves the VALU with the async MFMAs).
template <int RB, bool WV>
__device__ __forceinline__ void u_part(f32x16 (&acc)[RB], const ModelDev& M, const float* __restrict__ wp,
                                       const float* __restrict__ sk, const float* __restrict__ cut, float px,
                                       float py, float pz, int lane, JointMask* mask, float* __restrict__ uf,
                                       float* __restrict__ wvo, Ring& sh, const float* __restrict__ next,
                                       Stamps& st, float xs = 1.0f) {
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
    JRow ra = load_row(sk, cut, j0, nj, M.bone_cut != 0), rb2 = load_row(sk, cut, j0 + 1, nj, M.bone_cut != 0);
    float wv0, wv1;
    u_joint<WV>(M, ra, j0 < nj, px, py, pz, f[0], f[1], f[2], lv0, wv0);
    u_joint<WV>(M, rb2, j0 + 1 < nj, px, py, pz, f[3], f[4], f[5], lv1, wv1);
    if constexpr (WV) {  // w'_j of k-step p of the view layer's direction part (joint p + h NJH2)
        wvo[lane] = wv0;
        wvo[64 + lane] = wv1;
    }
    ra = load_row(sk, cut, j0 + 2, nj, M.bone_cut != 0);
    rb2 = load_row(sk, cut, j0 + 3, nj, M.bone_cut != 0);
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
                const float b = f[2 * g + t] * xs;
#pragma unroll
                for (int rb = 0; rb < RB; ++rb) acc[rb] = mfma_f32_32x32x2(ring[g % 3][rb][t], b, acc[rb]);
            }
            if (g == 0) {  // joint 2pp+2 from its prefetched row; then prefetch joint 2pp+4
                float wv;
                u_joint<WV>(M, ra, j0 + 2 * pp + 2 < nj, px, py, pz, fn[0], fn[1], fn[2], ln0, wv);
                pin(fn[0]), pin(fn[1]), pin(fn[2]), pin(ln0);
                if constexpr (WV) wvo[min(2 * pp + 2, njh2) * 64 + lane] = wv;  // (row njh2: discard)
                ra = load_row(sk, cut, j0 + 2 * pp + 4, nj, M.bone_cut != 0);
            }
            if (g == 1) {
                float wv;
                u_joint<WV>(M, rb2, j0 + 2 * pp + 3 < nj, px, py, pz, fn[3], fn[4], fn[5], ln1, wv);
                pin(fn[3]), pin(fn[4]), pin(fn[5]), pin(ln1);
                if constexpr (WV) wvo[min(2 * pp + 3, njh2) * 64 + lane] = wv;
                rb2 = load_row(sk, cut, j0 + 2 * pp + 5, nj, M.bone_cut != 0);
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
                                           const float* __restrict__ next, float xs = 1.0f) {
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
                for (int rb = 0; rb < RB; ++rb) acc[rb] = mfma_f32_32x32x2(ring[gg][rb][t], bc[t] * xs, acc[rb]);
            bc = bn;
        }
    }
    if (next) ring_preload<16>(sh, next, lane);
}

// ---- bf16x6 bone-direction parts (P == 2, layer 0 and the skip layer)
#ifndef ANERF_UF_UNROLL
#define ANERF_UF_UNROLL 2
#endif
// VALU pass: the 3 NJH2 bone-direction features of this lane (sample l & 31, joints h NJH2 ..
// h NJH2 + NJH2 - 1) into the wave's LDS store as [q][64 lanes] (q = 3 p + c: conflict-free
// b32 rows), the per-joint live ballots (JointMask) and the view windows w'_j — what u_part
// computes under its f32 MFMAs.  The two x parts then read the features from LDS.
template <bool WV>
__device__ __forceinline__ void u_features_lds(const ModelDev& M, const float* __restrict__ sk,
                                               const float* __restrict__ cut, float px, float py, float pz, int lane,
                                               JointMask* mask, float* __restrict__ uf, float* __restrict__ wvo) {
    const int hh = lane >> 5, njh2 = M.njh2, nj = M.nj, j0 = hh * njh2;
    // (njh2 <= 64: joint p of half 0 is mask bit p, joint p + njh2 of half 1 bit p + njh2 < 128.  The
    // bits are set branch-free with scalar selects; two joints per iteration for instruction-level
    // parallelism in the dependent transcendental chains of u_joint)
    uint64_t m0 = 0, m1 = 0;
    auto set_bits = [&](int p, uint64_t b) {
        const uint64_t lo = (b & 0xffffffffull) ? 1ull : 0ull, hi = (b >> 32) ? 1ull : 0ull;
        const int jb = p + njh2;
        m0 |= lo << p;
        m0 |= (jb < 64 ? hi : 0ull) << (jb & 63);
        m1 |= (jb >= 64 ? hi : 0ull) << (jb & 63);
    };
    // (U joints per iteration: the chains of U joints interleave; round 5: U = 4, was 2)
    constexpr int U = ANERF_UF_UNROLL;
    JRow r[U];
#pragma unroll
    for (int k = 0; k < U; ++k) r[k] = load_row(sk, cut, j0 + min(k, njh2 - 1), nj, M.bone_cut != 0);
    for (int p = 0; p < njh2; p += U) {
        JRow n[U];
#pragma unroll
        for (int k = 0; k < U; ++k) n[k] = load_row(sk, cut, j0 + min(p + U + k, njh2 - 1), nj, M.bone_cut != 0);
        float u[U][3], wv[U];
        bool live[U];
#pragma unroll
        for (int k = 0; k < U; ++k)
            u_joint<WV>(M, r[k], (p + k < njh2) && (j0 + p + k < nj), px, py, pz, u[k][0], u[k][1], u[k][2], live[k],
                        wv[k]);
#pragma unroll
        for (int k = 0; k < U; ++k) {
            if (p + k < njh2) {  // (uniform)
                uf[(3 * (p + k) + 0) * 64 + lane] = u[k][0];
                uf[(3 * (p + k) + 1) * 64 + lane] = u[k][1];
                uf[(3 * (p + k) + 2) * 64 + lane] = u[k][2];
                if constexpr (WV) wvo[(p + k) * 64 + lane] = wv[k];
                set_bits(p + k, __ballot(live[k]));
            }
        }
#pragma unroll
        for (int k = 0; k < U; ++k) r[k] = n[k];
    }
    if (mask) {
        mask->m0 = m0;
        mask->m1 = m1;
    }
}

// Live-joint count of one 32-sample block: the union over its samples of the cutoff-window test that
// u_features_lds ballots (lane half h: joints h NJH2 + p), without the features.  The render kernel
// orders a workgroup's blocks by it (bf16x6): the four waves pass a workgroup barrier at every hidden
// layer, so a wave whose block has fewer live joints (fewer windowed MFMAs) waits there for the others.
__device__ __forceinline__ int block_live_count(const ModelDev& M, const float* __restrict__ ray,
                                                const float* __restrict__ sk, const float* __restrict__ cut,
                                                const float* __restrict__ z, int n, int s0, int lane) {
    if (!M.sparse) return M.nj;
    int s = s0 + (lane & 31);
    if (s >= n) s = n - 1;
    const float zs = z[s];
    const float px = ray[0] + ray[3] * zs, py = ray[1] + ray[4] * zs, pz = ray[2] + ray[5] * zs;
    const int hh = lane >> 5, njh2 = M.njh2, nj = M.nj, j0 = hh * njh2;
    int cnt = 0;
    for (int p0 = 0; p0 < njh2; p0 += 4) {  // (four joints' rows loaded together: one LDS latency per four)
        JRow r[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) r[k] = load_row(sk, cut, j0 + min(p0 + k, njh2 - 1), nj, false);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float qx = fmaf(r[k].a[3], 1.0f, fmaf(r[k].a[2], pz, fmaf(r[k].a[1], py, r[k].a[0] * px)));
            const float qy = fmaf(r[k].b[3], 1.0f, fmaf(r[k].b[2], pz, fmaf(r[k].b[1], py, r[k].b[0] * px)));
            const float qz = fmaf(r[k].c[3], 1.0f, fmaf(r[k].c[2], pz, fmaf(r[k].c[1], py, r[k].c[0] * px)));
            const float d2 = fmaf(qz, qz, fmaf(qy, qy, qx * qx));
            const uint64_t b = __ballot((p0 + k < njh2) & (j0 + p0 + k < nj) & !(d2 >= r[k].thr2));
            cnt += ((b & 0xffffffffull) != 0) + ((b >> 32) != 0);
        }
    }
    return cnt;
}

#ifndef ANERF_X6_BARRIERS
#define ANERF_X6_BARRIERS 3
#endif
// Precision modes whose four waves run the hidden layers in lock step (a workgroup barrier before
// each, blocks in live-joint order): the split modes bf16x6, fp16x4 and fp16x3 (+2.6 % fp16x4,
// +0.8 % fp16x3, bit-identical outputs: profiles/r04i_ab_fp16x4.txt, r04y_ab_h3lock.txt)
template <int P>
constexpr bool lockstep_mode() { return P >= 2; }

// One x part's bone-direction contraction from the LDS features as bf16x6: k16-step s takes
// features 8 s .. 8 s + 7 of each lane half (zero past 3 NJH2), split by truncation (split3_pair);
// the next step's 8 features are read from LDS in its first group and split, a pair per group,
// in groups 4..7 (the LDS latency is covered by four groups of MFMAs).  Weight groups (s, rb) of 12
// floats with the 3-group prefetch in the 4-slot ring (RB % 4 == 0 keeps every slot index static);
// `preloaded`: groups 0..2 are already in slots 0..2 (issued before the VALU feature pass, or by
// the previous layer).
template <int RB>
__device__ __forceinline__ void u_part_x6_preload(const float* __restrict__ wp, int lane, Ring& ring) {
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(wp);
#pragma unroll
    for (int g = 0; g < 3; ++g) load_group<12>(ring.v[g], rs, lane, g);
}

template <int RB>
__device__ __forceinline__ void u_part_x6(f32x16 (&acc)[RB], const ModelDev& M, const float* __restrict__ wp,
                                          const float* __restrict__ uf, int lane, Ring& ring, bool preloaded,
                                          float xs = 1.0f) {
    static_assert(RB % 4 == 0 && RB >= 4, "u_part_x6 needs RB % 4 == 0");
    constexpr int PD = 3;
    const int nq = 3 * M.njh2, ns = (nq + 7) / 8, ng = ns * RB;
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(wp);
    if (!preloaded) u_part_x6_preload<RB>(wp, lane, ring);
    // Every group issues its loads and every step its LDS reads unconditionally (clamped: the last
    // groups reload the last group, the last step reads features it does not use), so the
    // compiler's counted vmcnt / lgkmcnt waits stay exact: a conditional load makes them drain.
    // (xs: a power of two, so the scaled features split exactly as the unscaled ones)
    auto feat = [&](int q) { return mask_f(uf[min(q, nq - 1) * 64 + lane] * xs, q < nq); };
    X6T cur[1], nxt[1];
    float fn[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) split3_pair(feat(2 * e), feat(2 * e + 1), cur[0], e);
    for (int s = 0; s < ns; ++s) {
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) {
            const int g = s * RB + rb;
            __builtin_amdgcn_sched_barrier(0);
            load_group<12>(ring.v[(rb + PD) % 4], rs, lane, min(g + PD, ng - 1));
            if (rb == 0) {
#pragma unroll
                for (int j = 0; j < 8; ++j) fn[j] = feat(8 * (s + 1) + j);
            }
            acc[rb] = mfma_x6(ring.v[rb % 4], cur[0], acc[rb]);
            if (rb >= RB - 4) {
                const int e = rb - (RB - 4);
                split3_pair(fn[2 * e], fn[2 * e + 1], nxt[0], e);
            }
        }
        cur[0] = nxt[0];
    }
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
    w = M.use_cutoff ? wc : 1.0f;  // (uniform)
}

template <int RB, int MR>
__device__ __forceinline__ void v_part(f32x16 (&acc)[RB], const ModelDev& M, const float* __restrict__ wp,
                                       const float* __restrict__ sk, const float* __restrict__ cut, float px,
                                       float py, float pz, int lane, JointMask mask, Stamps& st, float xs = 1.0f) {
    constexpr int GB = VPart<MR>::GB;
    constexpr int KB = VPart<MR>::KB;
    constexpr int PER = (MR + GB - 2) / (GB - 1);  // sin/cos terms of the next joint per group 1..GB-1
    const int hh = lane >> 5;
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(wp);
    const int voff = lane * 8;
    const bool dist_in = M.use_cutoff && M.cutoff_inputs;
    uint64_t r0 = uniform64(mask.m0), r1 = uniform64(mask.m1);
    int j = mask_pop(r0, r1);
    if (j < 0) return;
    int jn = mask_pop(r0, r1);
    f32x2 ring[GB][RB];
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) ring[g][rb] = bload2_v(rs, voff, ((j * GB + g) * RB + rb) * 512);
    float f[KB];
    {
        float dist, w, u, uf;
        v_geom(M, sk, cut, j, px, py, pz, dist, w);
        w *= xs;  // (a power of two: the products equal the unscaled ones times xs exactly)
        kp_inputs(M.cut_to, M.shift_in, dist, cut[j], u, uf);  // (u = uf = dist without the flags)
#pragma unroll
        for (int t = 0; t < MR; ++t) {
            float sn, cs;
            sincos_rr(uf * (float)(1 << t), sn, cs);
            f[t] = (hh ? cs : sn) * w;
        }
        f[MR] = hh ? 0.0f : (dist_in ? u * w : u * xs);
#pragma unroll
        for (int t = MR + 1; t < KB; ++t) f[t] = 0.0f;
    }
    STAMP(st, 15);
    while (j >= 0) {
        float fn[KB];
        float dn = 0.0f, dfn = 0.0f, wn = 0.0f;  // next joint: raw input, frequency input, window
        const int jg = jn >= 0 ? jn : j;  // geometry of the next joint (harmless redo at the end)
#pragma unroll
        for (int g = 0; g < GB; ++g) {
            __builtin_amdgcn_sched_barrier(0);
            constexpr int PD = 2;
            if (g + PD < GB) {
#pragma unroll
                for (int rb = 0; rb < RB; ++rb)
                    ring[(g + PD) % GB][rb] = bload2_v(rs, voff, ((j * GB + g + PD) * RB + rb) * 512);
            } else {  // the next joint's first groups (this joint's again after the last: harmless)
#pragma unroll
                for (int rb = 0; rb < RB; ++rb)
                    ring[(g + PD) % GB][rb] = bload2_v(rs, voff, ((jg * GB + g + PD - GB) * RB + rb) * 512);
            }
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                const float b = f[2 * g + t];
#pragma unroll
                for (int rb = 0; rb < RB; ++rb) acc[rb] = mfma_f32_32x32x2(ring[g][rb][t], b, acc[rb]);
            }
            // next joint's features under these MFMAs
            if (g == 0) {
                float dd;
                v_geom(M, sk, cut, jg, px, py, pz, dd, wn);
                wn *= xs;
                kp_inputs(M.cut_to, M.shift_in, dd, cut[jg], dn, dfn);
                pin(dn), pin(dfn), pin(wn);
            } else {
#pragma unroll
                for (int t = (g - 1) * PER; t < g * PER && t < MR; ++t) {
                    float sn, cs;
                    sincos_rr(dfn * (float)(1 << t), sn, cs);
                    fn[t] = (hh ? cs : sn) * wn;
                    pin(fn[t]);
                }
            }
            interleave_mfma_valu<2 * RB, 8>();
        }
        fn[MR] = hh ? 0.0f : (dist_in ? dn * wn : dn * xs);
#pragma unroll
        for (int t = MR + 1; t < KB; ++t) fn[t] = 0.0f;
#pragma unroll
        for (int t = 0; t < KB; ++t) f[t] = fn[t];
        j = jn;
        jn = mask_pop(r0, r1);
    }
}

// The windowed part as bf16x6 (precision modes 2 and 3, RB % 4 == 0): per live joint, lane half h
// holds features 8 s + i of k16-step s — i < MR: sin_i (h = 0) / cos_i (h = 1) of the frequency
// input times the window, i == MR: the distance input (h = 0), zero otherwise: v_part's f[] — split
// by truncation (exact), against weight groups (joint, s, rb) of 12 floats (pack_vpart_x6) in the
// 4-slot ring, three groups ahead (the last three groups of a joint load the next live joint's
// first).  Six bf16 MFMAs (32 cycles) per 16 k instead of eight f32 ones (64 cycles).  The next
// live joint's geometry (group 0), sincos terms (one per group) and splits (as soon as a pair is
// complete) run under this joint's MFMAs.
template <int MR, int NG>
struct VPartX6 {
    static constexpr int KS = (MR + 1 + 7) / 8;        // k16-steps per joint
    static constexpr int NF = 8 * KS;                  // features per lane half
    static constexpr int PER = (MR + NG - 2) / (NG - 1);  // sincos terms per group 1 .. NG - 1
    // the group in which feature q of the next joint is complete (sincos t in group t / PER + 1;
    // the distance input and the zero padding in group 1)
    static constexpr int ready(int q) { return q < MR ? q / PER + 1 : 1; }
    static constexpr int pair_ready(int e) { return ready(2 * e) > ready(2 * e + 1) ? ready(2 * e) : ready(2 * e + 1); }
};

template <int RB, int MR>
__device__ __forceinline__ void v_part_x6(f32x16 (&acc)[RB], const ModelDev& M, const float* __restrict__ wp,
                                          const float* __restrict__ sk, const float* __restrict__ cut, float px,
                                          float py, float pz, int lane, JointMask mask, Ring& ring,
                                          float xs = 1.0f) {
    static_assert(RB % 4 == 0, "v_part_x6 keeps ring slots static: groups per joint % 4 == 0");
    constexpr int NG = VPartX6<MR, 1>::KS * RB, PD = 3;  // groups per joint
    using V = VPartX6<MR, NG>;
    constexpr int KS = V::KS, NF = V::NF, PER = V::PER;
    const int hh = lane >> 5;
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(wp);
    const bool dist_in = M.use_cutoff && M.cutoff_inputs;
    uint64_t r0 = uniform64(mask.m0), r1 = uniform64(mask.m1);
    int j = mask_pop(r0, r1);
    if (j < 0) return;
    int jn = mask_pop(r0, r1);
#pragma unroll
    for (int d = 0; d < PD; ++d) load_group<12>(ring.v[d], rs, lane, j * NG + d);
    X6T cur[KS];
    {
        float f[NF];
        float dist, w, u, uf;
        v_geom(M, sk, cut, j, px, py, pz, dist, w);
        w *= xs;  // (a power of two: the products equal the unscaled ones times xs exactly)
        kp_inputs(M.cut_to, M.shift_in, dist, cut[j], u, uf);
#pragma unroll
        for (int t = 0; t < MR; ++t) {
            float sn, cs;
            sincos_rr(uf * (float)(1 << t), sn, cs);
            f[t] = (hh ? cs : sn) * w;
        }
        f[MR] = hh ? 0.0f : (dist_in ? u * w : u * xs);
#pragma unroll
        for (int t = MR + 1; t < NF; ++t) f[t] = 0.0f;
#pragma unroll
        for (int e = 0; e < NF / 2; ++e) split3_pair(f[2 * e], f[2 * e + 1], cur[e / 4], e % 4);
    }
    while (j >= 0) {
        X6T nxt[KS];
        float fn[NF];
        float dn = 0.0f, dfn = 0.0f, wn = 0.0f;  // next joint: raw input, frequency input, window
        const int jg = jn >= 0 ? jn : j;          // (a harmless redo of this joint after the last)
#pragma unroll
        for (int g = 0; g < NG; ++g) {
            const int s = g / RB, rb = g % RB;
            __builtin_amdgcn_sched_barrier(0);
            const int gp = g + PD;
            load_group<12>(ring.v[gp % 4], rs, lane, gp < NG ? j * NG + gp : jg * NG + gp - NG);
            acc[rb] = mfma_x6(ring.v[g % 4], cur[s], acc[rb]);
            if (g == 0) {
                float dd;
                v_geom(M, sk, cut, jg, px, py, pz, dd, wn);
                wn *= xs;
                kp_inputs(M.cut_to, M.shift_in, dd, cut[jg], dn, dfn);
                pin(dn), pin(dfn), pin(wn);
            } else {
#pragma unroll
                for (int t = (g - 1) * PER; t < g * PER && t < MR; ++t) {
                    float sn, cs;
                    sincos_rr(dfn * (float)(1 << t), sn, cs);
                    fn[t] = (hh ? cs : sn) * wn;
                    pin(fn[t]);
                }
            }
            if (g == 1) {
                fn[MR] = hh ? 0.0f : (dist_in ? dn * wn : dn * xs);
#pragma unroll
                for (int t = MR + 1; t < NF; ++t) fn[t] = 0.0f;
            }
#pragma unroll
            for (int e = 0; e < NF / 2; ++e)
                if (V::pair_ready(e) == g) split3_pair(fn[2 * e], fn[2 * e + 1], nxt[e / 4], e % 4);
            interleave_mfma_valu<6, 6>();
        }
#pragma unroll
        for (int k = 0; k < KS; ++k) cur[k] = nxt[k];
        j = jn;
        jn = mask_pop(r0, r1);
    }
}

// ---- fp16 encoder-fed parts (fp16x4 NP = 4, fp16x3 NP = 3; ModelDev::enc16): u_part_x6 / v_part_x6 with
// the features times a power of two t (the part's units, enc16_units: layer 0 a constant, the skip layer
// per sample) split into two fp16 parts (split2_pair) against weight groups of 8 floats = fragments
// [w0, w1] (pack_upart_h / pack_vpart_h), NP products per 16 k instead of bf16x6's six.
template <int RB>
__device__ __forceinline__ void u_part_h_preload(const float* __restrict__ wp, int lane, Ring& ring) {
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(wp);
#pragma unroll
    for (int g = 0; g < 3; ++g) load_group<8>(ring.v[g], rs, lane, g);
}

template <int RB, int NP>
__device__ __forceinline__ void u_part_h(f32x16 (&acc)[RB], const ModelDev& M, const float* __restrict__ wp,
                                         const float* __restrict__ uf, int lane, Ring& ring, bool preloaded, float t) {
    static_assert(RB % 4 == 0 && RB >= 4, "u_part_h needs RB % 4 == 0");
    constexpr int PD = 3;
    const int nq = 3 * M.njh2, ns = (nq + 7) / 8, ng = ns * RB;
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(wp);
    if (!preloaded) u_part_h_preload<RB>(wp, lane, ring);
    auto feat = [&](int q) { return mask_f(uf[min(q, nq - 1) * 64 + lane], q < nq); };  // (as u_part_x6)
    H3T cur, nxt;
    float fn[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) split2_pair(feat(2 * e), feat(2 * e + 1), t, cur, e);
    for (int s = 0; s < ns; ++s) {
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) {
            const int g = s * RB + rb;
            __builtin_amdgcn_sched_barrier(0);
            load_group<8>(ring.v[(rb + PD) % 4], rs, lane, min(g + PD, ng - 1));
            if (rb == 0) {
#pragma unroll
                for (int j = 0; j < 8; ++j) fn[j] = feat(8 * (s + 1) + j);
            }
            acc[rb] = mfma_h3<NP>(ring.v[rb % 4], 0, cur, acc[rb]);
            if (rb >= RB - 4) {
                const int e = rb - (RB - 4);
                split2_pair(fn[2 * e], fn[2 * e + 1], t, nxt, e);
            }
        }
        cur = nxt;
    }
}

// (round 5, ANERF_UFUSE) layer 0's fp16 bone-direction part with u_features_lds's VALU pass under its MFMAs:
// k-step s (8 features) runs while joints 3 s + 3 .. 3 s + 5 are computed, one per two-group scheduling
// region, and the features of k-step s + 1 (joints <= 3 s + 5) are read back and split in the last two
// regions.  The features still go through the LDS store (the skip layer reads them again; LDS is in order
// within a wave).  Joints past NJH2 - 1 recompute the last one (identical stores and ballots: no branch).
// --cutoff_bones' window is a select (a uniform branch would split the MFMA regions).
#ifndef ANERF_UFUSE
#define ANERF_UFUSE 0
#endif
#ifndef ANERF_UFUSE_PF  // (the next joint's skeleton row loaded one region ahead)
#define ANERF_UFUSE_PF 1
#endif
#ifndef ANERF_UFUSE_IL
#define ANERF_UFUSE_IL 1
#endif
#ifndef ANERF_UFUSE_BC  // (2: --cutoff_bones' window as a select; 0: the caller takes the unfused path with it)
#define ANERF_UFUSE_BC 2
#endif
template <int RB, int NP, bool WV>
__device__ __forceinline__ void u_part_h_fused(f32x16 (&acc)[RB], const ModelDev& M, const float* __restrict__ wp,
                                               const float* __restrict__ sk, const float* __restrict__ cut, float px,
                                               float py, float pz, int lane, JointMask* mask, float* __restrict__ uf,
                                               float* __restrict__ wvo, Ring& ring, float t) {
    static_assert(RB == 8, "u_part_h_fused: eight groups per k-step (three joint regions + the split region)");
    constexpr int PD = 3, NV = NP == 4 ? 8 : 10;
    const int hh = lane >> 5, njh2 = M.njh2, nj = M.nj, j0 = hh * njh2;
    const int nq = 3 * njh2, ns = (nq + 7) / 8, ng = ns * RB;
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(wp);
    uint64_t m0 = 0, m1 = 0;
    const bool bc = M.bone_cut != 0;
    auto row = [&](int p) {  // (load_row with the bone window's column selected by address: no branch)
        const int j = j0 + min(p, njh2 - 1), jc = j < nj ? j : 0;
        const f32x4* q = reinterpret_cast<const f32x4*>(sk + 12 * jc);
        return JRow{q[0], q[1], q[2], cut[2 * nj + jc], cut[nj + jc], cut[(bc ? 3 : 2) * nj + jc]};
    };
    auto joint = [&](int p, const JRow& r) {
        const int pc = min(p, njh2 - 1);
        float u0, u1, u2, wv;
        bool live;
        u_joint<WV, ANERF_UFUSE_BC>(M, r, j0 + pc < nj, px, py, pz, u0, u1, u2, live, wv);
        uf[(3 * pc + 0) * 64 + lane] = u0;
        uf[(3 * pc + 1) * 64 + lane] = u1;
        uf[(3 * pc + 2) * 64 + lane] = u2;
        if constexpr (WV) wvo[pc * 64 + lane] = wv;
        const uint64_t b = __ballot(live);  // (as u_features_lds: joint pc, half 1 joint pc + njh2)
        const uint64_t lo = (b & 0xffffffffull) ? 1ull : 0ull, hi = (b >> 32) ? 1ull : 0ull;
        const int jb = pc + njh2;
        m0 |= lo << pc;
        m0 |= (jb < 64 ? hi : 0ull) << (jb & 63);
        m1 |= (jb >= 64 ? hi : 0ull) << (jb & 63);
    };
    auto feat = [&](int q) { return mask_f(uf[min(q, nq - 1) * 64 + lane], q < nq); };
    {
        const JRow r0 = row(0), r1 = row(1), r2 = row(2);
        joint(0, r0);
        joint(1, r1);
        joint(2, r2);
    }
#if ANERF_UFUSE_PF
    JRow rn = row(3);
#endif
    H3T cur, nxt;
#pragma unroll
    for (int e = 0; e < 4; ++e) split2_pair(feat(2 * e), feat(2 * e + 1), t, cur, e);
    for (int s = 0; s < ns; ++s) {
        float fn[8];
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) {
            const int g = s * RB + rb;
            if (rb % 2 == 0) __builtin_amdgcn_sched_barrier(0);
            load_group<8>(ring.v[(rb + PD) % 4], rs, lane, min(g + PD, ng - 1));
            acc[rb] = mfma_h3<NP>(ring.v[rb % 4], 0, cur, acc[rb]);
            if (rb == 0 || rb == 2 || rb == 4) {
                const int p = 3 * s + 3 + rb / 2;
#if ANERF_UFUSE_PF
                const JRow r = rn;
                rn = row(p + 1);
                joint(p, r);
#else
                joint(p, row(p));
#endif
            }
            if (rb == 5) {
#pragma unroll
                for (int j = 0; j < 8; ++j) fn[j] = feat(8 * (s + 1) + j);
            }
            if (rb >= 6) {
                const int e = 2 * (rb - 6);
                split2_pair(fn[2 * e], fn[2 * e + 1], t, nxt, e);
                split2_pair(fn[2 * e + 2], fn[2 * e + 3], t, nxt, e + 1);
            }
#if ANERF_UFUSE_IL
            if (rb % 2 == 1) interleave_mfma_valu<2 * NP, NV>();
#endif
        }
        cur = nxt;
    }
    if (mask) {
        mask->m0 = m0;
        mask->m1 = m1;
    }
}

template <int RB, int MR, int NP>
__device__ __forceinline__ void v_part_h(f32x16 (&acc)[RB], const ModelDev& M, const float* __restrict__ wp,
                                         const float* __restrict__ sk, const float* __restrict__ cut, float px,
                                         float py, float pz, int lane, JointMask mask, Ring& ring, float t) {
    static_assert(RB % 4 == 0, "v_part_h keeps ring slots static: groups per joint % 4 == 0");
    constexpr int NG = VPartX6<MR, 1>::KS * RB, PD = 3;  // groups per joint
    using V = VPartX6<MR, NG>;
    constexpr int KS = V::KS, NF = V::NF, PER = V::PER;
    const int hh = lane >> 5;
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(wp);
    const bool dist_in = M.use_cutoff && M.cutoff_inputs;
    uint64_t r0 = uniform64(mask.m0), r1 = uniform64(mask.m1);
    int j = mask_pop(r0, r1);
    if (j < 0) return;
    int jn = mask_pop(r0, r1);
#pragma unroll
    for (int d = 0; d < PD; ++d) load_group<8>(ring.v[d], rs, lane, j * NG + d);
    H3T cur[KS];
    {
        float f[NF];
        float dist, w, u, uf;
        v_geom(M, sk, cut, j, px, py, pz, dist, w);
        kp_inputs(M.cut_to, M.shift_in, dist, cut[j], u, uf);
#pragma unroll
        for (int q = 0; q < MR; ++q) {
            float sn, cs;
            sincos_rr(uf * (float)(1 << q), sn, cs);
            f[q] = (hh ? cs : sn) * w;
        }
        f[MR] = hh ? 0.0f : (dist_in ? u * w : u);
#pragma unroll
        for (int q = MR + 1; q < NF; ++q) f[q] = 0.0f;
#pragma unroll
        for (int e = 0; e < NF / 2; ++e) split2_pair(f[2 * e], f[2 * e + 1], t, cur[e / 4], e % 4);
    }
    while (j >= 0) {
        H3T nxt[KS];
        float fn[NF];
        float dn = 0.0f, dfn = 0.0f, wn = 0.0f;  // next joint: raw input, frequency input, window
        const int jg = jn >= 0 ? jn : j;          // (a harmless redo of this joint after the last)
#pragma unroll
        for (int g = 0; g < NG; ++g) {
            const int s = g / RB, rb = g % RB;
            __builtin_amdgcn_sched_barrier(0);
            const int gp = g + PD;
            load_group<8>(ring.v[gp % 4], rs, lane, gp < NG ? j * NG + gp : jg * NG + gp - NG);
            acc[rb] = mfma_h3<NP>(ring.v[g % 4], 0, cur[s], acc[rb]);
            if (g == 0) {
                float dd;
                v_geom(M, sk, cut, jg, px, py, pz, dd, wn);
                kp_inputs(M.cut_to, M.shift_in, dd, cut[jg], dn, dfn);
                pin(dn), pin(dfn), pin(wn);
            } else {
#pragma unroll
                for (int q = (g - 1) * PER; q < g * PER && q < MR; ++q) {
                    float sn, cs;
                    sincos_rr(dfn * (float)(1 << q), sn, cs);
                    fn[q] = (hh ? cs : sn) * wn;
                    pin(fn[q]);
                }
            }
            if (g == 1) {
                fn[MR] = hh ? 0.0f : (dist_in ? dn * wn : dn);
#pragma unroll
                for (int q = MR + 1; q < NF; ++q) fn[q] = 0.0f;
            }
#pragma unroll
            for (int e = 0; e < NF / 2; ++e)
                if (V::pair_ready(e) == g) split2_pair(fn[2 * e], fn[2 * e + 1], t, nxt[e / 4], e % 4);
            interleave_mfma_valu<NP, 6>();
        }
#pragma unroll
        for (int k = 0; k < KS; ++k) cur[k] = nxt[k];
        j = jn;
        jn = mask_pop(r0, r1);
    }
}

// View layer, per-ray direction part: acc[RBV] += G^T * [w'_j, 1]  (G in LDS).  k-step p pairs
// joint p (lane half 0) with joint p + NJH2 (half 1), exactly the u part's pairing, so w'_j comes
// from the u part (wvp, stored per lane); k-step NJH2 adds the bias / framecode column NJ.  The G
// values of the next k-step are read under the current k-step's MFMAs.
// k-steps whose two joints have w'_j == 0 at every sample of the ray (bits of `live`, from
// compute_view_factor) add exact zeros and are skipped; returns the k-steps run (MFMA tally).
template <int RBV>
__device__ __forceinline__ int view_dir_part(f32x16 (&acc)[RBV], const ModelDev& M, const float* __restrict__ G,
                                             const float* __restrict__ wvp, const unsigned* __restrict__ live,
                                             int lane, float bs = 1.0f) {
    constexpr int WH = RBV * 32;
    const int hh = lane >> 5, sl = lane & 31;
    const int njh2 = M.njh2;
    const uint64_t L0 = uniform64((uint64_t)live[0] | ((uint64_t)live[1] << 32));
    const uint64_t L1 = uniform64((uint64_t)live[2] | ((uint64_t)live[3] << 32));
    auto bit = [&](int j) { return ((j < 64 ? L0 >> j : L1 >> (j - 64)) & 1ull) != 0; };
    auto next_p = [&](int p) {  // the next k-step with a live joint (njh2: the bias / code step)
        while (p < njh2 && !bit(p) && !bit(p + njh2)) ++p;
        return p;
    };
    auto col = [&](int p) { return p < njh2 ? p + hh * njh2 : M.nj + hh; };
    int p = next_p(0), steps = 0;
    float gv[RBV];
#pragma unroll
    for (int rb = 0; rb < RBV; ++rb) gv[rb] = G[col(p) * WH + sl + 32 * rb];
    // (bs: the units of acc, 2^es for the fp16x3 view layer: the B operands carry it)
    float b = p < njh2 ? wvp[p * 64 + lane] * bs : (hh ? 0.0f : bs);
    while (true) {
        __builtin_amdgcn_sched_barrier(0);
        const int pn = p < njh2 ? next_p(p + 1) : njh2;
        float gn[RBV];
#pragma unroll
        for (int rb = 0; rb < RBV; ++rb) gn[rb] = G[col(pn) * WH + sl + 32 * rb];
        const float bn = pn < njh2 ? wvp[pn * 64 + lane] * bs : (hh ? 0.0f : bs);
#pragma unroll
        for (int rb = 0; rb < RBV; ++rb) acc[rb] = mfma_f32_32x32x2(gv[rb], b, acc[rb]);
        ++steps;
        if (p == njh2) break;
#pragma unroll
        for (int rb = 0; rb < RBV; ++rb) gv[rb] = gn[rb];
        b = bn;
        p = pn;
    }
    return steps;
}

// Encoder + density trunk of one 32-sample block: L0 (u and v parts), the hidden layers with the
// skip; acc ends as the pre-activation of the last hidden layer.  `after_last` is the weight stream
// that follows (the feature layer, or nothing for density-only queries).
template <int W, int MR, bool WV, int P, bool SYNC = WV>
__device__ __forceinline__ bool mlp_trunk(const ModelDev& M, const NetDev& net, const float* __restrict__ sk,
                                          const float* __restrict__ cut, float px, float py, float pz, int lane,
                                          const float* __restrict__ bias, float* __restrict__ uf,
                                          float* __restrict__ wvo, f32x16 (&acc)[W / 32], f32x16 (&h)[W / 32],
                                          Ring& ring, JointMask& mask, const float* __restrict__ after_last,
                                          Stamps& st, int& es, int* bnd = nullptr, bool* have_bnd = nullptr) {
    constexpr int RB = W / 32;
    const int hh = lane >> 5;
    float nosig = 0.0f;
    es = 0;  // (fp16x3: the exponent of the accumulators' units, see mlp_layer_h3)
    constexpr bool HANDOFF = (2 * RB == 16);  // u-part groups have the regs layers' group size
    // bf16x6 / fp16x3 with the LDS feature store: features in a VALU pass, both bone-direction parts as x6
    constexpr bool UX6 = (P >= 2) && (RB % 4 == 0);
    const bool ux6 = UX6 && M.ux6 && uf != nullptr;
    // fp16x4 / fp16x3 with bounded windowed features: the encoder-fed parts as fp16 splits (NP products),
    // in units 2^enc_e0 (layer 0) and below 2^enc_cap (the skip layer), enc16_units
    constexpr bool H16 = (P >= 3) && UX6;
    constexpr int NPH = P == 4 ? 4 : 3;
    const bool enc16 = H16 && ux6 && M.enc16;
    if (!ux6) ring_preload<2 * RB>(ring, net.wl[0], lane);  // the u part's first groups, early
    load_bias<RB>(acc, bias, hh);
    if (enc16) {  // (a power of two: exact)
        const float s0 = pow2f(net.enc_e0);
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) acc[rb] = acc[rb] * s0;
    }
    STAMP(st, 10);
    const float* const* wl = P >= 3 ? net.wlh : (P == 2 ? net.wl6 : (P ? net.wl3 : net.wl));  // hidden-layer streams
    if (enc16) {
        if constexpr (H16) u_part_h_preload<RB>(net.wuh[0], lane, ring);  // (latency under the VALU pass)
        const float t0 = pow2f(net.enc_e0 - net.ewh_u[0]);
        if (ANERF_UFUSE && RB == 8 && (ANERF_UFUSE_BC == 2 || !M.bone_cut)) {
            if constexpr (H16 && RB == 8)
                u_part_h_fused<RB, NPH, WV>(acc, M, net.wuh[0], sk, cut, px, py, pz, lane, &mask, uf, wvo, ring, t0);
        } else {
            u_features_lds<WV>(M, sk, cut, px, py, pz, lane, &mask, uf, wvo);
            STAMP(st, 14);
            if constexpr (H16) u_part_h<RB, NPH>(acc, M, net.wuh[0], uf, lane, ring, true, t0);
        }
    } else if (ux6) {
        if constexpr (UX6) u_part_x6_preload<RB>(net.wu6, lane, ring);  // (latency under the VALU pass)
        u_features_lds<WV>(M, sk, cut, px, py, pz, lane, &mask, uf, wvo);
        STAMP(st, 14);
        if constexpr (UX6) u_part_x6<RB>(acc, M, net.wu6, uf, lane, ring, true);
    } else {
        // (bf16x6 layers have 12-float groups: the phases before them do not prefetch into the ring for them)
        u_part<RB, WV>(acc, M, net.wl[0], sk, cut, px, py, pz, lane, &mask, uf, wvo, ring,
                       M.D > 1 ? (P >= 2 ? nullptr : wl[1]) : after_last, st);
    }
    STAMP(st, 8);
    // (precision modes 2 / 3: the windowed parts as bf16x6; the u part's ring groups are consumed)
    constexpr bool VX6 = (P >= 2) && (RB % 4 == 0);
    if (enc16) {
        if constexpr (H16)
            v_part_h<RB, MR, NPH>(acc, M, net.wvh[0], sk, cut, px, py, pz, lane, mask, ring,
                                  pow2f(net.enc_e0 - net.ewh_v[0]));
        es = net.enc_e0;
    } else if constexpr (VX6) {
        v_part_x6<RB, MR>(acc, M, net.wv6, sk, cut, px, py, pz, lane, mask, ring);
    } else {
        v_part<RB, MR>(acc, M, net.wl0v, sk, cut, px, py, pz, lane, mask, st);
    }
    STAMP(st, 9);
    bool pre6 = false;
    // fp16 modes (ANERF_H3_BOUND): layer L >= 2 takes its scale from the bound layer L - 1 formed, unless L - 1 is the
    // skip layer (its x parts join the output after the h part; their features have no bound here)
    bool hb = false;
    for (int L = 1; L < M.D; ++L) {
        const float* after = L + 1 < M.D ? wl[L + 1] : after_last;
        const bool skl = (L == M.skip + 1);
        // bf16x6 render: the workgroup's four waves enter every hidden layer together (s_barrier, no
        // memory fence: the ring's loads stay in flight), so each 3 KiB weight group is read from L2
        // about once per CU and the other waves hit the CU's L1 — the hidden layers stream 12 KiB per
        // CU per group otherwise, and the waves drift apart over the windowed parts' live joints.
        // +2.1 % (A/B, profiles/r03_ab_experiments.txt); the calling block loop must have the same
        // trip count on every wave (SYNC: the render and density kernels' block loops).
        // (ANERF_X6_BARRIERS, experiments: 3 before every hidden layer, 2 before layer 1 and the layer
        // after the skip layer, 1 before layer 1 only, 0 none)
        constexpr int XB = ANERF_X6_BARRIERS;
        if constexpr (SYNC && lockstep_mode<P>() && XB > 0) {
            if (XB == 3 || L == 1 || (XB == 2 && L == M.skip + 2)) {
                __builtin_amdgcn_s_barrier();
                STAMP(st, 18);  // (stamps build: the wait at this barrier)
            }
        }
        if constexpr (P >= 3) {
            // the next h3 phase (the next hidden layer or the view layer) is prefetched; not across the
            // skip layer's x parts, which load themselves and scale their B operands by 2^es (the
            // units the h part left in the accumulators)
            const float* nxth = skl ? nullptr : after;
            const bool use = ANERF_H3_BOUND && bnd && hb;
            mlp_layer_h3<RB, RB, true, false, P == 4 ? 4 : 3>(acc, acc, h, bias + L * W, wl[L], lane, ring, pre6, nxth, nullptr,
                                              nosig, es, net.ewl[L], M.h3_top, (skl && enc16) ? net.enc_cap : 60,
                                              net.wl8[L], use, ANERF_H3_BOUND ? bnd : nullptr,
                                              skl ? -1.0f : net.hrsum[L], net.hbmax[L]);
            hb = !skl;
            pre6 = nxth != nullptr;
            if (skl) {  // the f32 skip x parts take their first groups from the ring (the x6 one loads itself)
                if (!ux6) ring_preload<2 * RB>(ring, net.wskipu, lane);
                after = nullptr;
            }
        } else if constexpr (P == 2) {
            // the next x6 phase: the next layer, after_last, or the skip layer's x6 bone-direction part
            // (selected by uniform values only: uf is a per-wave LDS pointer, derived from threadIdx,
            // and a pointer selected by it becomes a VGPR whose buffer loads waterfall)
            const float* nxt6 = skl ? ((UX6 && M.ux6) ? net.wskipu6 : nullptr) : after;
            mlp_layer_x6<RB, RB, true, false>(acc, acc, h, bias + L * W, wl[L], lane, ring, pre6, nxt6, nullptr,
                                              nosig);
            pre6 = nxt6 != nullptr && !skl;  // (the skip x part consumes its preloaded groups itself)
            if (skl) {  // the skip x part preloads its own groups; the phase after it loads itself
                if (!ux6) ring_preload<2 * RB>(ring, net.wskipu, lane);
                after = nullptr;
            }
        } else {
            const float* nxt = skl ? (HANDOFF ? net.wskipu : nullptr) : after;
            if constexpr (P == 1)
                mlp_layer_x3<RB, RB>(acc, acc, h, bias + L * W, wl[L], lane, ring, nxt);
            else
                mlp_layer<RB, RB, true, true, false>(acc, acc, h, bias + L * W, wl[L], lane, ring, nxt, nullptr, nosig);
            if (skl && !HANDOFF) ring_preload<2 * RB>(ring, net.wskipu, lane);
        }
        STAMP(st, 11);
        if (skl && enc16) {  // fp16 x parts, their features scaled into the h part's per-sample units
            if constexpr (H16) {
                u_part_h<RB, NPH>(acc, M, net.wuh[1], uf, lane, ring, false, pow2f(max(es - net.ewh_u[1], -126)));
                v_part_h<RB, MR, NPH>(acc, M, net.wvh[1], sk, cut, px, py, pz, lane, mask, ring,
                                      pow2f(max(es - net.ewh_v[1], -126)));
            }
            STAMP(st, 12);
        } else if (skl) {  // x part after the h part (in the h part's units: B operands times xs)
            const float xs = P >= 3 ? pow2f(es) : 1.0f;
            if (ux6) {
                if constexpr (UX6) u_part_x6<RB>(acc, M, net.wskipu6, uf, lane, ring, P == 2, xs);
            } else if (uf)
                u_part_lds<RB>(acc, M, net.wskipu, uf, lane, ring, after, xs);
            else
                u_part<RB, false>(acc, M, net.wskipu, sk, cut, px, py, pz, lane, nullptr, nullptr, nullptr, ring, after,
                                  st, xs);
            if constexpr (VX6)
                v_part_x6<RB, MR>(acc, M, net.wskipv6, sk, cut, px, py, pz, lane, mask, ring, xs);
            else
                v_part<RB, MR>(acc, M, net.wskipv, sk, cut, px, py, pz, lane, mask, st, xs);
            STAMP(st, 12);
        }
    }
    if (have_bnd) *have_bnd = ANERF_H3_BOUND && bnd && hb && M.D > 1;
    return pre6;  // (bf16x6 / fp16x3: after_last's first groups are in the ring)
}

// One 32-sample block of one ray through a whole NeRF: raw (rgb, sigma) into LDS.
template <int W, int MR, int P>
__device__ void mlp_block(const ModelDev& M, const NetDev& net, const float* __restrict__ ray,
                          const float* __restrict__ sk, const float* __restrict__ cut, const float* __restrict__ z,
                          int n, int s0,
                          const float* __restrict__ G, float* __restrict__ raw_out, int lane,
                          unsigned long long* mfma_count, const float* __restrict__ bias, float* __restrict__ uf,
                          float* __restrict__ wvp, Stamps& st, bool store = true) {
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
    int es = 0;
    int bnd = -1;
    bool have_bnd = false;
    const bool pre = mlp_trunk<W, MR, true, P>(M, net, sk, cut, px, py, pz, lane, bias, uf, wvp, acc, h, ring, mask,
                                               P >= 3 ? net.wviewh : (P == 2 ? net.wview6 : net.wview), st, es,
                                               P >= 3 ? &bnd : nullptr, &have_bnd);
    // views_linears.0 with feature_linear fused in (W' = Wv_f Wf, see pack_net) on relu(h_last),
    // alpha_linear folded into its groups (same relu'd B operands), + the factorised
    // direction / code / bias part from G, then relu
    float sig = 0.0f;
    f32x16 av[RBV];
    if constexpr (P >= 3) {
        const int es_h = es;  // the alpha head sums the last hidden layer's activations, in its units
        mlp_layer_h3<RBV, RB, false, true, P == 4 ? 4 : 3>(av, acc, h, nullptr, net.wviewh, lane, ring, pre, nullptr,
                                           bias + (M.D + 1) * W, sig, es, net.ew_view, M.h3_top, 60, net.wview8,
                                           have_bnd, &bnd);
        sig *= pow2f(-es_h);
    } else if constexpr (P == 2)
        mlp_layer_x6<RBV, RB, false, true>(av, acc, h, nullptr, net.wview6, lane, ring, pre, nullptr,
                                           bias + (M.D + 1) * W, sig);
    else
        mlp_layer<RBV, RB, true, false, true>(av, acc, h, nullptr, net.wview, lane, ring, nullptr,
                                              bias + (M.D + 1) * W, sig);
    STAMP(st, 16);
    sig += __shfl_xor(sig, 32);
    sig += net.balpha;
    const int vsteps = view_dir_part<RBV>(av, M, G, wvp, reinterpret_cast<const unsigned*>(ray) + 12, lane,
                                          P >= 3 ? pow2f(es) : 1.0f);
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
        if constexpr (P >= 3) a *= pow2f(-es);  // (the view layer's units)
        rgb[c] = a + net.brgb[c];
    }
    STAMP(st, 13);
    if (mfma_count && lane == 0) {  // exact MFMA work of this block (wave-uniform quantities)
        const int act = __builtin_popcountll(mask.m0) + __builtin_popcountll(mask.m1);
        const bool ux6 = (P >= 2) && (RB % 4 == 0) && uf != nullptr && M.ux6;  // as in mlp_trunk
        constexpr bool vx6 = (P >= 2) && (RB % 4 == 0);
        const int npe = (P >= 3 && ux6 && M.enc16) ? (P == 4 ? 4 : 3) : 6;  // products of the encoder-fed parts
        const int xk = (ux6 ? 0 : 3 * M.njh2) + (vx6 ? 0 : act * VPart<MR>::KB);  // f32 k-steps of one x part
        long long k = (long long)xk * RB + (long long)vsteps * RBV;
        const int nx = (M.skip + 1 < M.D) ? 2 : 1;
        if (ux6) atomicAdd(mfma_count + 1, (unsigned long long)(nx * ((3 * M.njh2 + 7) / 8) * RB * npe));
        if (vx6) atomicAdd(mfma_count + 1, (unsigned long long)(nx * act * VPartX6<MR, 1>::KS * RB * npe));
        constexpr int NPR = P == 2 ? 6 : (P == 4 ? 4 : 3);  // products per k16-step
        if (P >= 2)  // view layer, bf16x6 / fp16x3 / fp16x4
            atomicAdd(mfma_count + 1, (unsigned long long)(RBV * RB * 2 * NPR));
        else
            k += (long long)(W / 2) * RBV;
        if (M.skip + 1 < M.D) k += (long long)xk * RB;
        const long long hid = (long long)(M.D - 1) * RB * RB;  // 32x32 blocks of the hidden layers
        if (P != 0) {
            atomicAdd(mfma_count + 1, (unsigned long long)(hid * 2 * NPR));  // 2 k16-steps x products
        } else {
            k += hid * 16;
        }
        atomicAdd(mfma_count, (unsigned long long)k);
    }
    if (store && hh == 0 && s0 + sl < n) {
        float* o = raw_out + 4 * (s0 + sl);
        o[0] = rgb[0];
        o[1] = rgb[1];
        o[2] = rgb[2];
        o[3] = sig;
    }
}

