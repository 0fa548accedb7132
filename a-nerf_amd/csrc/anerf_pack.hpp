// anerf_pack.hpp — host side: weight packing into the MFMA operand streams, descriptor validation, model binding.
// Part of the single translation unit anerf_render.hip (included there, in order).
#pragma once

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

// ---- bf16x3 split of the dense layers (ANERF_PREC_BF16X3): w = w_hi + w_lo, each bf16 (RNE)
uint16_t bf16_rne(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    if ((u & 0x7f800000u) == 0x7f800000u) return (uint16_t)((u >> 16) | ((u & 0xffffu) ? 0x40u : 0u));
    return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}
float bf16_to_f(uint16_t b) {
    const uint32_t u = (uint32_t)b << 16;
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}

// dense layer for mlp_layer_x3 (v_mfma_f32_32x32x16_bf16): a group is 4 fragments of 8 bf16 per
// lane (one b128 each).  Fragment (ob, ib, s) of lane l = (r, h), element j holds
// W[32 ob + r][col_off + 32 ib + 16 s + 8 (j >> 2) + 4 h + (j & 3)] (the k order of an accumulator
// tile used as B operand, registers 8s..8s+7).  Lead groups g < RBO: [hi, lo] of (g, 0, 0) and
// (g, 0, 1); then per input block ib >= 1, k-step s, output pair (2p, 2p+1): [hi, lo] of both.
std::vector<float> pack_layer_x3(const float* Wt, int n_out, int ld, int col_off, int n_in) {
    const int RBO = n_out / 32, RBI = n_in / 32;
    const int ng = RBO + (RBI - 1) * RBO;
    return pack_groups(ng, 16, [&](int g, int sl, int l) {
        const int f = sl >> 2, e = sl & 3;  // fragment, bf16 pair within it
        int ob, ib, s;
        if (g < RBO) {
            ob = g, ib = 0, s = f >> 1;
        } else {
            const int idx = g - RBO, r = idx % RBO;
            ib = 1 + idx / RBO, s = r / (RBO / 2), ob = 2 * (r % (RBO / 2)) + (f >> 1);
        }
        const bool lo = f & 1;
        const int h = l >> 5, row = 32 * ob + (l & 31);
        uint32_t bits = 0;
        for (int jj = 0; jj < 2; ++jj) {
            const int j = 2 * e + jj;
            const int col = col_off + 32 * ib + 16 * s + 8 * (j >> 2) + 4 * h + (j & 3);
            const float w = Wt[(size_t)row * ld + col];
            const uint16_t hi = bf16_rne(w);
            const uint16_t v = lo ? bf16_rne(w - bf16_to_f(hi)) : hi;
            bits |= (uint32_t)v << (16 * jj);
        }
        float out;
        std::memcpy(&out, &bits, 4);
        return out;
    });
}

// ---- bf16x6 split (ANERF_PREC_BF16X6): w = w0 + w1 + w2, each bf16 (RNE of the running remainder;
// the remainders are exact in fp32), so w0 + w1 + w2 carries >= 24 significant bits of w.
// Groups of 12 floats = fragments [w0, w1, w2] of (ob, ib, s) (element j as in pack_layer_x3).
// Order: lead groups 2 ob + s (input block 0), then per input block ib >= 1, k-step s, block ob.
std::vector<float> pack_layer_x6(const float* Wt, int n_out, int ld, int col_off, int n_in) {
    const int RBO = n_out / 32, RBI = n_in / 32;
    const int ng = 2 * RBO * RBI;
    return pack_groups(ng, 12, [&](int g, int sl, int l) {
        const int f = sl >> 2, e = sl & 3;  // fragment (split part), bf16 pair within it
        int ob, ib, s;
        if (g < 2 * RBO) {
            ob = g >> 1, ib = 0, s = g & 1;
        } else {
            const int idx = g - 2 * RBO;
            ib = 1 + idx / (2 * RBO), s = (idx / RBO) & 1, ob = idx % RBO;
        }
        const int h = l >> 5, row = 32 * ob + (l & 31);
        uint32_t bits = 0;
        for (int jj = 0; jj < 2; ++jj) {
            const int j = 2 * e + jj;
            const int col = col_off + 32 * ib + 16 * s + 8 * (j >> 2) + 4 * h + (j & 3);
            float r = Wt[(size_t)row * ld + col];
            uint16_t v = 0;
            for (int p = 0; p <= f; ++p) {
                v = bf16_rne(r);
                r -= bf16_to_f(v);
            }
            bits |= (uint32_t)v << (16 * jj);
        }
        float out;
        std::memcpy(&out, &bits, 4);
        return out;
    });
}

// ---- fp16x3 split (ANERF_PREC_FP16X3): the block is scaled by 2^ew (max |w| 2^ew in [2^10, 2^11),
// see anerf_mlp.hpp on the f16 MFMA's range), then w = w0 + w1, each fp16 (RNE of the
// running remainder), i.e. >= 22 significant bits.  Groups (ob, ib, s) in pack_layer_x6's order,
// 8 floats each (fragments w0, w1, element j as in pack_layer_x3), two consecutive groups per
// 16-float ring slot.
uint16_t f16_rne(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    const uint32_t sign = (u >> 16) & 0x8000u;
    const uint32_t a = u & 0x7fffffffu;
    if (a >= 0x7f800000u) return (uint16_t)(sign | 0x7c00u | (a > 0x7f800000u ? 0x200u : 0u));
    if (a >= 0x477ff000u) return (uint16_t)(sign | 0x7c00u);  // rounds past 65504: inf
    if (a < 0x38800000u) {  // below 2^-14: fp16 subnormal (or zero), units of 2^-24
        const double q = (double)(*reinterpret_cast<const float*>(&a)) * 16777216.0;
        return (uint16_t)(sign | (uint32_t)std::nearbyint(q));
    }
    const uint32_t e = (a >> 23) - 112, m = a & 0x7fffffu;
    uint32_t h = (e << 10) | (m >> 13);
    const uint32_t rem = m & 0x1fffu;
    if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) ++h;
    return (uint16_t)(sign | h);
}
float f16_to_f(uint16_t b) {
    const uint32_t sign = (uint32_t)(b & 0x8000u) << 16, e = (b >> 10) & 0x1fu, m = b & 0x3ffu;
    uint32_t u;
    if (e == 0) {
        const float v = (float)m * 5.9604644775390625e-08f;  // m 2^-24 (exact)
        std::memcpy(&u, &v, 4);
        u |= sign;
    } else if (e == 31) {
        u = sign | 0x7f800000u | (m << 13);
    } else {
        u = sign | ((e + 112) << 23) | (m << 13);
    }
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}

// fp16 operand range of the fp16x3 / fp16x4 layers: maxima in [2^T, 2^(T+1)), T = ANERF_H3_TARGET = 10.
// A compile-time constant (experiment builds of tools/build_ab.sh may pass -DANERF_H3_TARGET=...; the
// shipped library never reads it from the environment).  The probe of the f16 MFMA
// (tools/probe/mfma_f16_numerics.hip) returned wrong sums once both operands' maxima reached 2^13 (products
// ~2^28), and matched the fp32 path at 2^12 and below: targets above 11 (maxima up to 2^12) are rejected at
// build time, and so are targets below 6 (the low fp16 parts of ordinary values would turn subnormal).
#ifndef ANERF_H3_TARGET
#define ANERF_H3_TARGET 10
#endif
static_assert(ANERF_H3_TARGET >= 6 && ANERF_H3_TARGET <= 11,
              "ANERF_H3_TARGET outside the probed safe range [6, 11] of the f16 MFMA");
constexpr int h3_target() { return ANERF_H3_TARGET; }

// power-of-two exponent ew with max |W[:, col_off : col_off + n_in]| 2^ew in [2^T, 2^(T+1))
int h3_exponent(const float* Wt, int n_out, int ld, int col_off, int n_in) {
    float mx = 0.0f;
    for (int r = 0; r < n_out; ++r)
        for (int c = 0; c < n_in; ++c) mx = std::max(mx, std::fabs(Wt[(size_t)r * ld + col_off + c]));
    if (!(mx > 0.0f) || !std::isfinite(mx)) return 0;
    int e;
    std::frexp(mx, &e);  // mx in [2^(e-1), 2^e)
    return std::max(-100, std::min(100, h3_target() + 1 - e));
}

std::vector<float> pack_layer_h3(const float* Wt, int n_out, int ld, int col_off, int n_in, int ew) {
    const int RBO = n_out / 32, RBI = n_in / 32;
    const int ng = 2 * RBO * RBI;
    const float sc = std::ldexp(1.0f, ew);
    return pack_groups(ng / 2, 16, [&](int gg, int sl, int l) {
        const int g = 2 * gg + (sl >> 3), f = (sl >> 2) & 1, e = sl & 3;  // group, fragment, f16 pair
        int ob, ib, s;
        if (g < 2 * RBO) {
            ob = g >> 1, ib = 0, s = g & 1;
        } else {
            const int idx = g - 2 * RBO;
            ib = 1 + idx / (2 * RBO), s = (idx / RBO) & 1, ob = idx % RBO;
        }
        const int h = l >> 5, row = 32 * ob + (l & 31);
        uint32_t bits = 0;
        for (int jj = 0; jj < 2; ++jj) {
            const int j = 2 * e + jj;
            const int col = col_off + 32 * ib + 16 * s + 8 * (j >> 2) + 4 * h + (j & 3);
            const float w = Wt[(size_t)row * ld + col] * sc;  // (exact: a power of two)
            const uint16_t w0 = f16_rne(w);
            const uint16_t v = f ? f16_rne(w - f16_to_f(w0)) : w0;
            bits |= (uint32_t)v << (16 * jj);
        }
        float out;
        std::memcpy(&out, &bits, 4);
        return out;
    });
}

// ---- e4m3 (OCP fp8, the MFMA's "fp8") round to nearest even with saturation at 448: 1 sign, 4 exponent
// (bias 7), 3 mantissa bits; subnormals below 2^-6 in units of 2^-9
uint8_t f8e4m3_rne(float f) {
    if (std::isnan(f)) return 0x7f;
    const uint8_t sign = std::signbit(f) ? 0x80 : 0;
    double a = std::fabs((double)f);
    if (a >= 464.0) return sign | 0x7e;  // (448 is the largest finite; 464 would round past it)
    int e;
    std::frexp(a, &e);  // a in [2^(e-1), 2^e)
    int E = e - 1;      // a = 1.m x 2^E
    if (E < -6) {       // subnormal: units of 2^-9
        const double q = std::nearbyint(a * 512.0);
        return sign | (uint8_t)q;  // (q == 8 is 2^-6, the smallest normal: the encoding carries over)
    }
    double m = std::nearbyint((a / std::ldexp(1.0, E) - 1.0) * 8.0);
    if (m >= 8.0) { m = 0.0; ++E; }
    if (E > 8) return sign | 0x7e;
    return sign | (uint8_t)(((E + 7) << 3) | (int)m);
}

// fp16x4's x1 w1 products on v_mfma_scale_f32_32x32x64_f8f6f4 (ANERF_F8_X1W1): for output block ob and the
// input block pair (2c, 2c + 1), lane l (row 32 ob + (l & 31), half h = l >> 5) holds 32 bytes: byte t is the
// e4m3 of w1 x 2^8 -- w1 the low fp16 part of the layer's scaled weight (pack_layer_h3: w x 2^ew = w0 + w1) --
// for input block 2c + (t >> 4) and its element i = t & 15 in the order the kernel's split packs x1 (k16-step
// i >> 3, element i & 7: column 32 ib + 16 s + 8 (j >> 2) + 4 h + (j & 3)).  Groups (c, ob), 8 floats each.
std::vector<float> pack_layer_f8(const float* Wt, int n_out, int ld, int col_off, int n_in, int ew) {
    const int RBO = n_out / 32, RBI = n_in / 32;
    const float sc = std::ldexp(1.0f, ew);
    return pack_groups((RBI / 2) * RBO, 8, [&](int g, int sl, int l) {
        const int c = g / RBO, ob = g % RBO, h = l >> 5, row = 32 * ob + (l & 31);
        uint32_t bits = 0;
        for (int b = 0; b < 4; ++b) {
            const int t = 4 * sl + b, ib = 2 * c + (t >> 4), i = t & 15, s = i >> 3, j = i & 7;
            const int col = col_off + 32 * ib + 16 * s + 8 * (j >> 2) + 4 * h + (j & 3);
            const float w = Wt[(size_t)row * ld + col] * sc;
            const float w1 = f16_to_f(f16_rne(w - f16_to_f(f16_rne(w))));
            bits |= (uint32_t)f8e4m3_rne(w1 * 256.0f) << (8 * b);
        }
        float out;
        std::memcpy(&out, &bits, 4);
        return out;
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

// bone-direction part as bf16x6 groups for u_part_x6: k16-step s, lane half h, element j -> feature
// q = 8 s + j of that half (joint h njh2 + q / 3, component q % 3; zero past 3 njh2 or nj), column
// nv nj + 3 joint + comp; groups (s, rb) of 12 floats = fragments w0, w1, w2 (as pack_layer_x6).
std::vector<float> pack_upart_x6(const float* Wt, int n_out, int ld, int nj, int njh2, int mr) {
    const int nv = 1 + 2 * mr, RB = n_out / 32, nq = 3 * njh2, ns = (nq + 7) / 8;
    return pack_groups(ns * RB, 12, [&](int g, int sl, int l) {
        const int s = g / RB, rb = g % RB, f = sl >> 2, e = sl & 3;
        const int h = l >> 5, row = 32 * rb + (l & 31);
        uint32_t bits = 0;
        for (int jj = 0; jj < 2; ++jj) {
            const int q = 8 * s + 2 * e + jj, joint = q / 3 + h * njh2, c = q % 3;
            float r = (q < nq && joint < nj) ? Wt[(size_t)row * ld + nv * nj + 3 * joint + c] : 0.0f;
            uint16_t v = 0;
            for (int p = 0; p <= f; ++p) {
                v = bf16_rne(r);
                r -= bf16_to_f(v);
            }
            bits |= (uint32_t)v << (16 * jj);
        }
        float out;
        std::memcpy(&out, &bits, 4);
        return out;
    });
}

// The windowed parts are laid out for the kernel instance's frequency count mrl (layout_multires:
// 7 or 10) and filled from the model's mr <= mrl: the k-slots of frequencies mr .. mrl - 1 carry
// zero weights (their features are computed and add exact zeros), so every multires up to 10 runs on
// the two instances.
int layout_multires(int mr) { return mr <= 7 ? 7 : 10; }
int layout_multires_views(int mrv) { return mrv == 0 ? 0 : 4; }

// windowed part, per joint j: k-step t < mr -> (sin_t, cos_t) = columns ((1+2t)NJ + j, (2+2t)NJ + j);
// mr <= t < mrl -> zero; t == mrl -> (dist, pad); padded to an even count.  Layout [joint][group][RB][64][2].
std::vector<float> pack_vpart(const float* Wt, int n_out, int ld, int nj, int mr, int mrl) {
    const int kb = ((mrl + 1) + 1) & ~1;
    std::vector<float> out;
    for (int j = 0; j < nj; ++j) {
        std::vector<float> pj = pack_kmajor(Wt, n_out, ld, kb, [&](int t, int h) {
            if (t < mr) return (1 + 2 * t + h) * nj + j;
            if (t == mrl && h == 0) return j;
            return -1;
        });
        out.insert(out.end(), pj.begin(), pj.end());
    }
    return out;
}

// windowed part as bf16x6 groups for v_part_x6: joint j, k16-step s, lane half h, element i ->
// feature q = 8 s + i of that half: q < mr -> sin_q (h = 0) / cos_q (h = 1) = column
// (1 + 2q + h) nj + j, q == mrl and h == 0 -> the distance input (column j), else zero; groups
// (j, s, rb) of 12 floats = fragments w0, w1, w2 (as pack_layer_x6).
std::vector<float> pack_vpart_x6(const float* Wt, int n_out, int ld, int nj, int mr, int mrl) {
    const int RB = n_out / 32, ks = (mrl + 1 + 7) / 8;
    return pack_groups(nj * ks * RB, 12, [&](int g, int sl, int l) {
        const int j = g / (ks * RB), s = (g / RB) % ks, rb = g % RB, f = sl >> 2, e = sl & 3;
        const int h = l >> 5, row = 32 * rb + (l & 31);
        uint32_t bits = 0;
        for (int jj = 0; jj < 2; ++jj) {
            const int q = 8 * s + 2 * e + jj;
            const int col = q < mr ? (1 + 2 * q + h) * nj + j : (q == mrl && h == 0 ? j : -1);
            float r = col >= 0 ? Wt[(size_t)row * ld + col] : 0.0f;
            uint16_t v = 0;
            for (int p = 0; p <= f; ++p) {
                v = bf16_rne(r);
                r -= bf16_to_f(v);
            }
            bits |= (uint32_t)v << (16 * jj);
        }
        float out;
        std::memcpy(&out, &bits, 4);
        return out;
    });
}

// ---- fp16 split of the encoder-fed parts (fp16x4 / fp16x3 with ModelDev::enc16): the weights of a part
// scaled by 2^ew (its own h3_exponent), then w = w0 + w1 in fp16 (RNE of the running remainder), groups of
// 8 floats = fragments [w0, w1] (element j of lane half h as in pack_upart_x6 / pack_vpart_x6), one group
// per ring slot (u_part_h / v_part_h).
uint32_t f16_split_bits(float a, float b, int part) {
    const uint16_t a0 = f16_rne(a), b0 = f16_rne(b);
    const uint16_t va = part ? f16_rne(a - f16_to_f(a0)) : a0, vb = part ? f16_rne(b - f16_to_f(b0)) : b0;
    return (uint32_t)va | ((uint32_t)vb << 16);
}

std::vector<float> pack_upart_h(const float* Wt, int n_out, int ld, int nj, int njh2, int mr, int ew) {
    const int nv = 1 + 2 * mr, RB = n_out / 32, nq = 3 * njh2, ns = (nq + 7) / 8;
    const float sc = std::ldexp(1.0f, ew);
    return pack_groups(ns * RB, 8, [&](int g, int sl, int l) {
        const int s = g / RB, rb = g % RB, f = sl >> 2, e = sl & 3;
        const int h = l >> 5, row = 32 * rb + (l & 31);
        float v[2];
        for (int jj = 0; jj < 2; ++jj) {
            const int q = 8 * s + 2 * e + jj, joint = q / 3 + h * njh2, c = q % 3;
            v[jj] = (q < nq && joint < nj) ? Wt[(size_t)row * ld + nv * nj + 3 * joint + c] * sc : 0.0f;
        }
        const uint32_t bits = f16_split_bits(v[0], v[1], f);
        float out;
        std::memcpy(&out, &bits, 4);
        return out;
    });
}

std::vector<float> pack_vpart_h(const float* Wt, int n_out, int ld, int nj, int mr, int mrl, int ew) {
    const int RB = n_out / 32, ks = (mrl + 1 + 7) / 8;
    const float sc = std::ldexp(1.0f, ew);
    return pack_groups(nj * ks * RB, 8, [&](int g, int sl, int l) {
        const int j = g / (ks * RB), s = (g / RB) % ks, rb = g % RB, f = sl >> 2, e = sl & 3;
        const int h = l >> 5, row = 32 * rb + (l & 31);
        float v[2];
        for (int jj = 0; jj < 2; ++jj) {
            const int q = 8 * s + 2 * e + jj;
            const int col = q < mr ? (1 + 2 * q + h) * nj + j : (q == mrl && h == 0 ? j : -1);
            v[jj] = col >= 0 ? Wt[(size_t)row * ld + col] * sc : 0.0f;
        }
        const uint32_t bits = f16_split_bits(v[0], v[1], f);
        float out;
        std::memcpy(&out, &bits, 4);
        return out;
    });
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
    std::vector<float> cut_host;  // the kp embedder's cutoff distances (enc16_units)
};

// Units of the fp16 encoder-fed parts (fp16x4 / fp16x3).  Their features are bounded: the bone directions
// |u_j| <= 1 (times w_b <= 1), the windowed sin / cos times w_j in [-1, 1], and -- with sparse windows --
// the distance input |dist w_j| (|(c_j - dist) w_j| under --cut_to_dist) < max(|c_j|, c_j + 16.69 / tau):
// w_j is exactly 0 beyond d^2 >= thr2_j = (c_j + 16.69 / tau)^2 (1 + 1e-5) (live_thr2).  So fixed powers of
// two put them in fp16's range, like the hidden layers' per-sample scales: the bone directions times 2^T,
// the windowed features times 2^fv with 2^fv x their bound < 2^(T+1).  Layer 0's accumulators hold the
// output times 2^e0, e0 = min(ew_u + T, ew_v + fv) (ew: the part's weight exponent), so neither feature set
// passes 2^(T+1) scaled; the skip layer's h part keeps its per-sample units below 2^cap, cap = min(ew_u' + T,
// ew_v' + fv), for the same reason.  Without bounded windows (no cutoff inputs, tau <= 0) or with extreme
// weight exponents the parts stay bf16x6 (enc16 = 0).
static void enc16_units(anerf_model* m) {
    ModelDev& md = m->md;
    md.enc16 = 0;
    for (int i = 0; i < 2; ++i) md.net[i].enc_e0 = 0, md.net[i].enc_cap = 60;
    if (!md.sparse || !(md.tau > 0.0f) || !std::isfinite(md.tau)) return;
    double vb = 1.0;
    for (const float c : m->cut_host) {
        if (!std::isfinite(c)) return;
        vb = std::max(vb, std::max(std::fabs((double)c), (double)c + 16.69 / (double)md.tau) * 1.001);
    }
    if (!(vb < 1e30)) return;
    int eb;
    std::frexp(vb, &eb);  // vb < 2^eb
    const int T = h3_target(), fv = T + 1 - eb;
    for (int i = 0; i < 2; ++i) {
        NetDev& n = md.net[i];
        const bool skip = n.wuh[1] != nullptr;
        const int e0 = std::min(n.ewh_u[0] + T, n.ewh_v[0] + fv);
        const int cap = skip ? std::min(n.ewh_u[1] + T, n.ewh_v[1] + fv) : 60;
        for (int e : {n.ewh_u[0], n.ewh_v[0], n.ewh_u[1], n.ewh_v[1], e0, cap})
            if (e < -60 || e > 60) return;
        n.enc_e0 = e0;
        n.enc_cap = cap;
    }
    md.enc16 = 1;
}

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
    if (d->multires < 1 || d->multires > 10)
        return fail(ANERF_EINVAL, "multires outside [1, 10] (kernel instances: 7 and 10, smaller counts zero-padded)");
    if (d->multires_views < 0 || d->multires_views > 4)
        return fail(ANERF_EINVAL, "multires_views outside [0, 4] (kernel instances: 0 and 4, 1-3 zero-padded)");
    if (d->single_net && d->has_fine) return fail(ANERF_EINVAL, "single_net models have no separate fine network");
    if (d->n_joints < 1 || d->n_joints > 128) return fail(ANERF_EINVAL, "n_joints outside [1, 128]");
    if (d->skip < 0) return fail(ANERF_EINVAL, "skip must be >= 0");
    if (d->framecode_ch < 0 || d->framecode_ch > 64) return fail(ANERF_EINVAL, "framecode_ch outside [0, 64]");
    if (d->framecode_ch > 0 && d->n_framecodes <= 0) return fail(ANERF_EINVAL, "n_framecodes must be > 0");
    if (d->density_scale == 0.0f) return fail(ANERF_EINVAL, "density_scale must be non-zero");
    if (d->multires_bones < 0 || d->multires_bones > 10) return fail(ANERF_EINVAL, "multires_bones outside [0, 10]");
    if (d->encoder_flags & ~(ANERF_ENC_CUT_TO_DIST | ANERF_ENC_CUTOFF_SHIFT | ANERF_ENC_CUTOFF_BONES | ANERF_ENC_VIEW_RAW |
                             ANERF_ENC_KP_RELPOS | ANERF_ENC_VIEW_ANGLE | ANERF_ENC_KP_QUERYPTS | ANERF_ENC_VIEW_WINDOWS))
        return fail(ANERF_EINVAL, "unknown encoder_flags bits");
    if ((d->encoder_flags & ANERF_ENC_KP_RELPOS) && (d->encoder_flags & ANERF_ENC_KP_QUERYPTS))
        return fail(ANERF_EINVAL, "ANERF_ENC_KP_RELPOS and ANERF_ENC_KP_QUERYPTS are two kp types");
    if ((d->encoder_flags & ANERF_ENC_KP_QUERYPTS) && (d->encoder_flags & ANERF_ENC_CUTOFF_BONES) && d->use_cutoff)
        return fail(ANERF_EINVAL, "ANERF_ENC_KP_QUERYPTS with ANERF_ENC_CUTOFF_BONES: the reference's bone embedder "
                                  "fails on it (cutoff_dim 3 for 3 NJ inputs)");
    if ((d->encoder_flags & ANERF_ENC_KP_QUERYPTS) && d->n_joints < 3)
        return fail(ANERF_EINVAL, "ANERF_ENC_KP_QUERYPTS needs n_joints >= 3");
    if ((d->encoder_flags & ANERF_ENC_VIEW_RAW) && (d->encoder_flags & ANERF_ENC_VIEW_ANGLE))
        return fail(ANERF_EINVAL, "ANERF_ENC_VIEW_RAW and ANERF_ENC_VIEW_ANGLE are two view types");
    if (d->encoder_flags & ANERF_ENC_VIEW_WINDOWS) {
        if (!d->cutoff_viewdir || !d->use_cutoff || !d->cutoff_inputs)
            return fail(ANERF_EINVAL, "ANERF_ENC_VIEW_WINDOWS needs cutoff_viewdir, use_cutoff and cutoff_inputs (every "
                                      "view feature windowed)");
        if (d->multires_bones > 0 || (d->encoder_flags & (ANERF_ENC_KP_RELPOS | ANERF_ENC_VIEW_ANGLE | ANERF_ENC_KP_QUERYPTS)))
            return fail(ANERF_EINVAL, "ANERF_ENC_VIEW_WINDOWS is not for a staged encoder");
    }
    return ANERF_OK;
}

// A staged encoder (anerf.h, ABI 15): the training stages serve the model, the fused kernels do not.
static bool desc_staged(const anerf_model_desc* d) {
    return d->multires_bones > 0 || (d->encoder_flags & (ANERF_ENC_KP_RELPOS | ANERF_ENC_VIEW_ANGLE | ANERF_ENC_KP_QUERYPTS));
}

static int pack_net(const anerf_model_desc* d, int njh2, const anerf_net_weights* w, Packer& pk,
                    std::vector<size_t>& offs) {
    const int W = d->net_width, WH = W / 2, nj = d->n_joints, mr = d->multires, mrv = d->multires_views;
    const int mrl = layout_multires(mr), nkl = 1 + 2 * layout_multires_views(mrv);  // kernel layouts
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
    offs.push_back(pk.add(pack_vpart(w->pts_w[0], W, cin, nj, mr, mrl)));
    const int skl = d->skip + 1;
    if (skl < d->net_depth) {
        offs.push_back(pk.add(pack_upart(w->pts_w[skl], W, cin + W, nj, njh2, mr)));
        offs.push_back(pk.add(pack_vpart(w->pts_w[skl], W, cin + W, nj, mr, mrl)));
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
        // [joint][WH][tp] rows of the view-direction weights in the instance's trig-table layout (nkl
        // terms per component); the model's nk <= nkl terms filled, the rest zero
        const int tp = (3 * nkl + 3) & ~3;
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
    for (int i = 1; i < d->net_depth; ++i) {                                          // bf16x3 hidden layers
        const bool sk = (i == d->skip + 1);
        offs.push_back(pk.add(pack_layer_x3(w->pts_w[i], W, sk ? cin + W : W, sk ? cin : 0, W)));
    }
    for (int i = 1; i < d->net_depth; ++i) {                                          // bf16x6 hidden layers
        const bool sk = (i == d->skip + 1);
        offs.push_back(pk.add(pack_layer_x6(w->pts_w[i], W, sk ? cin + W : W, sk ? cin : 0, W)));
    }
    offs.push_back(pk.add(pack_layer_x6(wfused.data(), WH, W, 0, W)));               // wview6
    offs.push_back(pk.add(pack_upart_x6(w->pts_w[0], W, cin, nj, njh2, mr)));          // wu6 (layer 0)
    if (skl < d->net_depth)                                                           // wskipu6
        offs.push_back(pk.add(pack_upart_x6(w->pts_w[skl], W, cin + W, nj, njh2, mr)));
    else
        offs.push_back((size_t)-1);
    for (int i = 1; i < d->net_depth; ++i) {                                          // fp16x3 hidden layers
        const bool sk = (i == d->skip + 1);
        const int ld = sk ? cin + W : W, c0 = sk ? cin : 0;
        const int ew = h3_exponent(w->pts_w[i], W, ld, c0, W);
        offs.push_back((size_t)(int64_t)ew);  // (exponent, read back by bind_net)
        offs.push_back(pk.add(pack_layer_h3(w->pts_w[i], W, ld, c0, W, ew)));
    }
    {
        const int ew = h3_exponent(wfused.data(), WH, W, 0, W);
        offs.push_back((size_t)(int64_t)ew);
        offs.push_back(pk.add(pack_layer_h3(wfused.data(), WH, W, 0, W, ew)));     // wviewh
    }
    offs.push_back(pk.add(pack_vpart_x6(w->pts_w[0], W, cin, nj, mr, mrl)));               // wv6 (layer 0)
    if (skl < d->net_depth)                                                           // wskipv6
        offs.push_back(pk.add(pack_vpart_x6(w->pts_w[skl], W, cin + W, nj, mr, mrl)));
    else
        offs.push_back((size_t)-1);
    for (int i = 1; i < d->net_depth; ++i) {                                          // fp16x4 x1 w1 (e4m3)
        const bool sk = (i == d->skip + 1);
        const int ld = sk ? cin + W : W, c0 = sk ? cin : 0;
        offs.push_back(pk.add(pack_layer_f8(w->pts_w[i], W, ld, c0, W, h3_exponent(w->pts_w[i], W, ld, c0, W))));
    }
    offs.push_back(pk.add(pack_layer_f8(wfused.data(), WH, W, 0, W, h3_exponent(wfused.data(), WH, W, 0, W))));
    // fp16 encoder-fed parts (u: columns nv nj .. cin, v: columns 0 .. nv nj), each with its own exponent:
    // layer 0's, then the skip layer's (exponent 0 / no buffer without a skip layer)
    for (int part = 0; part < 2; ++part) {
        const bool has = part == 0 || skl < d->net_depth;
        const float* Wp = part == 0 ? w->pts_w[0] : (has ? w->pts_w[skl] : nullptr);
        const int ld = part == 0 ? cin : cin + W;
        const int nv = 1 + 2 * mr;
        const int ewu = has ? h3_exponent(Wp, W, ld, nv * nj, 3 * nj) : 0;
        const int ewv = has ? h3_exponent(Wp, W, ld, 0, nv * nj) : 0;
        offs.push_back((size_t)(int64_t)ewu);
        offs.push_back(has ? pk.add(pack_upart_h(Wp, W, ld, nj, njh2, mr, ewu)) : (size_t)-1);
        offs.push_back((size_t)(int64_t)ewv);
        offs.push_back(has ? pk.add(pack_vpart_h(Wp, W, ld, nj, mr, mrl, ewv)) : (size_t)-1);
    }
    // (round 6) the fp16 modes' scale bounds of each hidden layer's h part (mlp_layer_h3): max_i sum_k |W_ik| and
    // max_i |b_i|, summed in double and rounded up to float (bit patterns, read back by bind_net)
    for (int i = 1; i < d->net_depth; ++i) {
        const bool sk = (i == d->skip + 1);
        const int ld = sk ? cin + W : W, c0 = sk ? cin : 0;
        double rs = 0.0, bm = 0.0;
        for (int r = 0; r < W; ++r) {
            double s = 0.0;
            for (int c = 0; c < W; ++c) s += std::fabs((double)w->pts_w[i][(size_t)r * ld + c0 + c]);
            rs = std::max(rs, s);
            bm = std::max(bm, std::fabs((double)w->pts_b[i][r]));
        }
        float rf = (float)rs, bf = (float)bm;
        if ((double)rf < rs) rf = std::nextafter(rf, INFINITY);
        if ((double)bf < bm) bf = std::nextafter(bf, INFINITY);
        uint32_t ur, ub;
        std::memcpy(&ur, &rf, 4);
        std::memcpy(&ub, &bf, 4);
        offs.push_back((size_t)ur);
        offs.push_back((size_t)ub);
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
    for (int i = 1; i < D; ++i) nd.wl3[i] = base + o[k++];
    for (int i = 1; i < D; ++i) nd.wl6[i] = base + o[k++];
    nd.wview6 = base + o[k++];
    nd.wu6 = base + o[k++];
    nd.wskipu6 = o[k] == (size_t)-1 ? nullptr : base + o[k];
    ++k;
    for (int i = 1; i < D; ++i) {
        nd.ewl[i] = (int)(int64_t)o[k++];
        nd.wlh[i] = base + o[k++];
    }
    nd.ew_view = (int)(int64_t)o[k++];
    nd.wviewh = base + o[k++];
    nd.wv6 = base + o[k++];
    nd.wskipv6 = o[k] == (size_t)-1 ? nullptr : base + o[k];
    ++k;
    for (int i = 1; i < D; ++i) nd.wl8[i] = base + o[k++];
    nd.wview8 = base + o[k++];
    for (int part = 0; part < 2; ++part) {
        nd.ewh_u[part] = (int)(int64_t)o[k++];
        nd.wuh[part] = o[k] == (size_t)-1 ? nullptr : base + o[k];
        ++k;
        nd.ewh_v[part] = (int)(int64_t)o[k++];
        nd.wvh[part] = o[k] == (size_t)-1 ? nullptr : base + o[k];
        ++k;
    }
    for (int i = 1; i < D; ++i) {
        const uint32_t ur = (uint32_t)o[k++], ub = (uint32_t)o[k++];
        std::memcpy(&nd.hrsum[i], &ur, 4);
        std::memcpy(&nd.hbmax[i], &ub, 4);
    }
    nd.balpha = balpha;
}

