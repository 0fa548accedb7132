// anerf_types.hpp — device-side model / launch argument structs, diagnostic stamps, LDS plan.
// Part of the single translation unit anerf_render.hip (included there, in order).
#pragma once


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
#elif defined(ANERF_ASM_MARKS)  // (diagnostic: phase markers in the device assembly, tools only)
#define STAMP_INIT(st) do { } while (0)
#define STAMP(st, i) asm volatile(";@@STAMP " #i)
#define STAMP_FLUSH(st, ptr) do { } while (0)
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
    const float* wl3[MAXL];  // [i>0] activation parts as bf16x3 fragments (pack_layer_x3)
    const float* wl6[MAXL];  // [i>0] activation parts as bf16x6 fragments (pack_layer_x6)
    const float* wview6;     // wview as bf16x6 fragments
    const float* wu6;        // layer 0 bone-direction part as bf16x6 fragments (pack_upart_x6)
    const float* wskipu6;    // the skip layer's, or null
    const float* wv6;        // layer 0 windowed part as bf16x6 groups (pack_vpart_x6)
    const float* wskipv6;    // the skip layer's, or null
    const float* wlh[MAXL];  // [i>0] activation parts as fp16x3 fragments (pack_layer_h3), scaled by 2^ewl[i]
    const float* wviewh;     // wview as fp16x3 fragments, scaled by 2^ew_view
    int ewl[MAXL], ew_view;
    // (round 6) per hidden layer (h part only): max_i sum_k |W_ik| and max_i |b_i| (real units, rounded up), the
    // next layer's scale bound (mlp_layer_h3)
    float hrsum[MAXL], hbmax[MAXL];
    // fp16 encoder-fed parts (ModelDev::enc16): [0] layer 0, [1] the skip layer (null without one); the
    // bone-direction (u) and windowed (v) weights scaled by 2^ewh_u / 2^ewh_v (pack_upart_h, pack_vpart_h)
    const float* wuh[2];
    const float* wvh[2];
    int ewh_u[2], ewh_v[2];
    const float* wl8[MAXL];  // [i>0] fp16x4's x1 w1 products: the e4m3 w1 of the fp16 planes (pack_layer_f8)
    const float* wview8;     // the same for wviewh
    int enc_e0;   // exponent of layer 0's accumulator units (enc16)
    int enc_cap;  // the largest exponent of the skip layer's accumulator units its x parts' features allow
    float balpha;
};

struct ModelDev {
    int nj, njh2, ngh, D, skip, mr, mrv, use_cutoff, cutoff_inputs, cutoff_viewdir, cfc, n_codes, softplus;
    int sparse;  // windowed features are exactly 0 where w == 0 (use_cutoff && cutoff_inputs)
    int ux6;     // bf16x6: bone-direction parts as x6 from the LDS feature store (u_part_x6)
    int single_net;  // one network for both passes; the fine pass evaluates only the I new samples
    int cut_to, shift_in;  // kp encoder input transforms (ANERF_ENC_CUT_TO_DIST / _CUTOFF_SHIFT)
    int h3_top;      // fp16x3: biased exponent the largest scaled activation of a sample gets (127 + 10)
    int bone_cut;    // --cutoff_bones (+ use_cutoff, cutoff_inputs): bone directions times w_b
    int view_raw;    // --view_type world: the view input is R_j d, not normalised (ANERF_ENC_VIEW_RAW)
    // staged encoders (ABI 15, training stages only; anerf.h): bone frequencies, relpos kp inputs, ray angles;
    // bone_win: the bone embedder is a CutoffEmbedder (--cutoff_bones + use_cutoff: windows its sin / cos)
    int mrb, kp_relpos, view_angle, bone_win, staged;
    int kp_query;  // --kp_dist_type querypts: the world point as the kp input (cutoff[0..2] its 3 cutoffs)
    int view_win;  // ANERF_ENC_VIEW_WINDOWS: the training layout's view part is the NJ view windows (anerf.h)
    // fp16x4 / fp16x3: the encoder-fed parts (bone-direction and windowed x parts of layer 0 and the skip
    // layer) as fp16 splits too, when every windowed feature is bounded (sparse windows, tau > 0; host:
    // enc16_units in anerf_pack.hpp); bf16x6 parts otherwise
    int enc16;
    float shift, B, tau, tau_v, tau_b;
    const float* cutoff;
    const float* cutoff_v;
    const float* cutoff_b;
    NetDev net[2];
};

struct RenderArgs {
    const float* rb;
    int64_t n;
    int stride, S, I, R;
    int n_poses;
    const float* skts;
    const int32_t* ray_pose;
    const float* cams;
    const float* near;
    const float* far;
    float *rgb, *disp, *acc, *rgb0, *disp0, *acc0, *alpha, *alpha0;
    float *dbg_z0, *dbg_raw0, *dbg_w0, *dbg_z1, *dbg_raw1;
    unsigned long long* mfma_count;
    unsigned long long* stamps;
    int pass0, pass1;  // passes [pass0, pass1) of this launch (0 coarse, 1 fine)
    float* zf_ws;      // n x T: the fine pass's sorted z, handed from the coarse launch to the fine one
    int lindisp;       // sample_from_lineseg in inverse depth (ANERF_FLAG_LINDISP)
    unsigned* queue;   // ANERF_PERSIST: this launch's 8 band counters (workspace, zeroed before the launch)
};

// ======================================================================= LDS plan
struct LdsPlan {
    int ray, sk, zc, zf, raw, g, scr, bias, cut, uf, wv;  // float offsets (uf < 0: no u-feature store)
    int bord, bord_n;                   // block order (bf16x6): live-joint counts [bord_n], then the order
    int total;                          // floats
    int sk_stride, z_stride, raw_stride, g_stride, scr_stride, uf_stride, wv_stride;
};

__host__ __device__ inline int pad32(int x) { return (x + 31) & ~31; }

// The kp CutoffEmbedder's inputs for distance `dist` to a joint with cutoff c
// (core/cutoff_embedder.py:125-134): the raw input u = c - dist under --cut_to_dist (else dist), the
// frequencies' input u * (2 / c) - 1 under --cutoff_shift (else u); two roundings each, as torch.
__device__ __forceinline__ void kp_inputs(int cut_to, int shift_in, float dist, float c, float& u, float& uf) {
    u = cut_to ? c - dist : dist;
    uf = shift_in ? u * (2.0f / c) - 1.0f : u;
}

__host__ __device__ inline LdsPlan make_plan(int R, int nj, int W, int S, int T, int mrv, int ngh, int D, int njh2,
                                             bool with_uf, bool bone_cut) {
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
    p.cut = o; o += (bone_cut ? 4 : 3) * nj;  // windows: cutoffs (points, view directions), live thresholds
                                               // (, bone cutoffs)
    o = (o + 3) & ~3;
    p.uf_stride = 64 * 3 * njh2;   // per wave: the L0 bone directions, re-read by the skip layer
    p.uf = with_uf ? o : -1;
    if (with_uf) o += 4 * p.uf_stride;
    p.wv_stride = 64 * (njh2 + 1);  // per wave: view-direction windows w'_j of the block (+ a discard row)
    p.wv = o; o += 4 * p.wv_stride;
    p.bord_n = (R * (((T > S ? T : S) + 31) / 32) + 3) & ~3;  // 32-sample blocks of the workgroup
    p.bord = o; o += 2 * p.bord_n + 4;  // (+ the persistent launch's item slot)
    p.total = (o + 3) & ~3;
    return p;
}

