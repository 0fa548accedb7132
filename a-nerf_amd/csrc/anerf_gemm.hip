// anerf_gemm.hip — the training MLP's linear layers on the bf16 MFMA pipe.
//
// Training runs the reference's NeRF (core/networks/nerf.py:94-148) forward and backward over
// M = rays x samples rows (131 k - 164 k per step at the reference's N_rand 2048, 64 + 16 samples).
// Every product here is fp32 in, fp32 out, with both operands split into bf16 planes (round to
// nearest even of the running remainder) and v_mfma_f32_32x32x16_bf16 products accumulated in
// fp32: bf16x3 = two planes, the three products x_lo w_hi + x_hi w_lo + x_hi w_hi (~16 significant
// bits per operand); bf16x6 = three planes, the six products with i + j <= 2 (fp32-accurate).  The
// training default ("mixed", mlp.py) runs the forward in bf16x6 and the backward in bf16x3.
//
//   forward / input gradient (NT): C[m][n] = epi(sum_k A[m][k] B[n][k]); A = up to three fp32
//     column segments (the reference's cat([x, h]) / cat([feature, views, code]) never built),
//     split into LDS as it is staged; B = the layer's weight (forward) or its transpose (input
//     gradient), split once per step into bf16 planes (anerf_mlp_split_weights).  Epilogue: + bias,
//     relu (forward); relu' mask by the saved activation (> 0) and accumulate (backward); the output
//     is up to three column segments (e.g. the view layer's input gradient: feature part, the
//     encoder's view columns, the framecodes).
//   weight gradient (TN): dW[n][k] = sum_m dY[m][n] X[m][k] over M split into slabs, one partial
//     tile per (slab, tile) in a workspace, summed in a second launch in slab order (deterministic,
//     no atomics); the bias gradient sum_m dY[m][n] is summed from the staged dY in the same pass.
//
// Both kernels: 128 x 128 outputs per 256-thread workgroup, two workgroups per CU (<= 256 VGPRs,
// <= 80 KB LDS each) so one workgroup's prologue and epilogue overlap the other's MFMAs.  fp32
// operands arrive through buffer loads whose descriptors end at the tile's (slab's) last row, so
// ragged rows and columns outside an operand segment read zero with no clamp or select; they are
// split with v_cvt_pk_bf16_f32 into bf16 LDS planes (two stages, loads two steps ahead).  The
// forward reads its A fragments row-wise (ds_read_b128); the weight gradient, whose operands are
// both [m][.] activations, reads them column-wise with the hardware transpose ds_read_b64_tr_b16.
// Workgroups are mapped so tiles that re-read the same rows run on one XCD's L2.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>
#include <cstdlib>
#include <string>

#include "../../include/anerf.h"

int anerf_internal_fail(int code, const char* msg);  // anerf_render.hip: sets anerf_last_error()

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int BM = 128, BN = 128, NTHR = 256;
// k columns per step of the bf16x3 single-segment forward / input-gradient instances: 32, or 64
// (half the barriers, twice the A bytes in flight; experiment switch)
#ifndef ANERF_GEMM_SK64
#define ANERF_GEMM_SK64 0
#endif
// forward / input gradient row-tile height (experiment switch): 128 rows, two workgroups per CU; or 64
// rows, four per CU (half the accumulators, LDS and epilogue per workgroup: more tiles in flight to
// cover the per-tile load and store latency at K = 256)
#ifndef ANERF_GEMM_BM
#define ANERF_GEMM_BM 128
#endif
// B-fragment ring depth of the single-segment forward / input-gradient instances (2 or 4)
#ifndef ANERF_GEMM_BD
#define ANERF_GEMM_BD 4
#endif
// forward / input gradient column-tile width (round 5): 2 = 256 columns per workgroup where N % 256 == 0, 1 = 128
// (A/B, profiles/r05j_gemm.txt: 256 columns 108.6 -> 134-139 us forward at M = 163,840, training 203 k -> 189 k:
// one workgroup per CU instead of two exposes the staging; not kept)
#ifndef ANERF_GEMM_CB
#define ANERF_GEMM_CB 1
#endif
constexpr int MAXSEG = 3;

struct SegD {
    const float* p;
    long long ld;
    int start, cols;
    int vec;  // float4 loads allowed (ld, start, pointer 16-byte aligned)
};
struct OSegD {
    float* p;
    long long ld;
    int start, cols;
    const float* mask;
    long long ldm;
    int accum;
};

struct NTArgs {
    long long M;
    int N, K;
    SegD a[MAXSEG];
    int na;
    const unsigned short* b;  // split weights, fragment-major (split_weights_kernel)
    int ksteps;               // k16 steps of B (padded)
    const float* bias;
    int relu;
    OSegD c[MAXSEG];
    int nc;
    int tiles_n, total;
    // fp16x4 (F16 instances): per-row maxima of A (non-negative floats' bit patterns, the producing
    // layer's rout) and the weights' exponent (split buffer tail); rout: this product's row maxima
    const int* rin;
    const int* bexp;
    int* rout;
};

struct TNArgs {
    long long M;
    int N, K;  // dW is N x K
    const float* dy;
    long long lddy;
    SegD x[MAXSEG];
    int nx;
    int tiles_k, tiles, total, splits;
    long long rows_per_split;
    float* ws;   // [splits][Npad][Kpad]
    float* wsb;  // [splits][Npad] bias partials, or null
    int npad, kpad;
};

// logical tile of a workgroup: the hardware deals workgroups round-robin over the 8 XCDs; this
// bijection gives each XCD a contiguous run of logical ids (MI355X guide, "XCD swizzle")
__device__ __forceinline__ int xcd_logical(int wg, int total) {
    const int xcd = wg & 7, q = total >> 3, r = total & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (wg >> 3);
}

typedef __attribute__((address_space(1))) const f32x4 gf32x4;

__device__ __forceinline__ f32x16 mfma(const bf16x8& a, const bf16x8& b, const f32x16& c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x16 mfma16(const bf16x8& a, const bf16x8& b, const f32x16& c) {  // (f16 bits)
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}
__device__ __forceinline__ float pow2i(int e) { return __builtin_bit_cast(float, (e + 127) << 23); }  // |e| <= 126
// fp16x4 row scale: the shift that puts a row's largest |value| (bits m of a non-negative float) in
// [2^10, 2^11) (anerf_mlp.hpp h3_scale; 0 for an all-zero row)
// (clamped to pow2i's exponent range: rows of any finite magnitude from 2^-126 up scale into fp16's range)
__device__ __forceinline__ int f16_row_shift(int m) {
    int s = m > 0 ? 137 - (m >> 23) : 0;
    return min(max(s, -126), 126);
}

// ---------------------------------------------------------------- forward / input gradient
// 128 rows x 128 columns per workgroup, two workgroups per CU (4 waves; wave w computes all 128 rows
// x columns 32 w .. 32 w + 31 = 4 blocks, so the waves read disjoint B fragments).  A (activations,
// fp32 in HBM, up to three column segments) is staged 32 columns per step: buffer loads through
// per-tile segment descriptors whose range ends at the last row (rows past M and columns outside a
// segment read zero, so no clamp, no select, no zero fill), issued two steps ahead into two register
// sets, split with v_cvt_pk_bf16_f32 into NPL bf16 planes ([row][k], swizzled 64 B rows: conflict-free
// ds_read_b128 fragment reads and staging writes); two LDS stages, one barrier per step.  B (the split weights, a few
// hundred KB shared by every workgroup) is read straight from L2 as MFMA fragments, stored
// fragment-major (1 KB per 32-column block, k16 step and plane, in lane order), one k16 step ahead.
// The epilogue goes through LDS in whole 512 B output rows (bias, relu, relu' mask, accumulate,
// output segments); with two workgroups per CU one's epilogue and prologue overlap the other's MFMAs.
constexpr int BNW = 256;      // row padding of the split weights (whole 256-row tiles)
constexpr int NBN = 128;      // output columns per workgroup
// LDS planes [row][SKT k] bf16.  SKT 32: 64 B rows, the four 16 B chunks of a row XOR-swizzled by bits
// 2-3 of the row; SKT 64: 128 B rows, the eight chunks swizzled by bits 1-3.  Fragment reads
// (ds_read_b128, 16 rows x one chunk per lane group) and staging writes (ds_write_b64, whole rows per
// 16-lane group) are both conflict-free
template <int SKT>
__device__ __forceinline__ int nt_off(int row, int k) {
    if constexpr (SKT == 32) return row * 32 + ((((k >> 3) ^ (row >> 2)) & 3) << 3) + (k & 7);
    return row * 64 + ((((k >> 3) ^ (row >> 1)) & 7) << 3) + (k & 7);
}
constexpr unsigned NOOB = 0x80000000u;  // a lane offset past every descriptor's range

template <int NPL, int TBM, int SKT = 32>
struct NTGeo {
    static constexpr int RBM = TBM / 32;               // 32-row blocks per tile
    static constexpr int RPS = 1024 / SKT;             // rows per staging pass (256 threads x 4 columns)
    static constexpr int NRS = TBM / RPS;              // staging passes per step
    static constexpr int PLANE = TBM * SKT;            // bf16 elements
    static constexpr int STAGE = NPL * PLANE;
    static constexpr int STAGES_BYTES = 2 * STAGE * 2;
    static constexpr int TILE_BYTES = TBM * 132 * 4;  // epilogue tile [TBM][132] fp32
    static constexpr int TAB = STAGES_BYTES > TILE_BYTES ? STAGES_BYTES : TILE_BYTES;  // segment tables
    static constexpr int LDS_BYTES = TAB + 256 + 4 * TBM;  // (+ segment tables, fp16x4 row shifts)
};

// output segment tables in LDS: per-lane segment choices read their pointer and stride from here
// (an indexed read of the kernel-argument struct makes clang copy it to scratch)
struct SegTab {
    float* op[MAXSEG];
    long long old[MAXSEG];
    const float* mask[MAXSEG];
    long long ldm[MAXSEG];
    int accum[MAXSEG];
};

// CB: 32-column blocks per wave -- 1: a 128-column tile, two workgroups per CU; 2 (round 5): a 256-column
// tile, one workgroup per CU, so that every A row is staged once for all 256 output columns (the 128-column
// tiles staged each row twice: with K = 256 the A rows are half the vector-memory bytes of a step)
template <int NPL, int NSEG, int TBM, int SKT = 32, bool F16 = false, int CB = 1>
__global__ __launch_bounds__(NTHR, CB == 1 ? 256 / TBM : 1) void mlp_nt_kernel(NTArgs g) {
    static_assert(!F16 || (NPL == 2 && NSEG == 1), "fp16x4: two fp16 planes, one A segment");
    static_assert(!F16 || CB == 1, "fp16x4's row-max epilogue works on 128-column tiles");
    using G = NTGeo<NPL, TBM, SKT>;
    constexpr int RBM = G::RBM, NRS = G::NRS, SK = SKT, KK = SKT / 16;
    extern __shared__ __attribute__((aligned(16))) unsigned short lds[];
    const int logical = xcd_logical(blockIdx.x, g.total);
    const int mt = logical / g.tiles_n, nt = logical % g.tiles_n;
    const long long m0 = (long long)mt * TBM;
    const int n0 = nt * NBN * CB;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // (kernel-argument fields as locals: referencing `g` inside the lambdas makes clang copy the
    // whole argument struct to scratch and reload fields from there in the loop)
    const int Kd = g.K, ksteps = g.ksteps;
    const long long Md = g.M;
    const int nst = (Kd + SK - 1) / SK;  // steps
    const int nk = (Kd + 15) / 16;        // k16 steps of the B planes
    SegTab* const tab = reinterpret_cast<SegTab*>(reinterpret_cast<char*>(lds) + G::TAB);
    int* const rsh = reinterpret_cast<int*>(reinterpret_cast<char*>(lds) + G::TAB + 256);  // F16: row shifts
    if constexpr (F16) {
        if (tid < TBM) {
            const long long m = m0 + tid;
            rsh[tid] = m < Md ? f16_row_shift(g.rin[m]) : 0;
        }
    }
    if (tid < MAXSEG) {
        const int u = tid < g.nc ? tid : 0;
        tab->op[tid] = g.c[u].p;
        tab->old[tid] = g.c[u].ld;
        tab->mask[tid] = g.c[u].mask;
        tab->ldm[tid] = g.c[u].ldm;
        tab->accum[tid] = g.c[u].accum;
    }
    // staging: rows sr + RPS i (i < NRS), columns sc .. sc + 3 of the step; a wave instruction reads
    // 8 rows x 128 B (SKT 32) or 4 rows x 256 B (SKT 64)
    constexpr int RPS = G::RPS;
    const int sr = tid / (SKT / 4), sc = 4 * (tid % (SKT / 4));
    const long long rows_left = Md - m0;
    const int rows = rows_left < TBM ? (int)rows_left : TBM;
    __amdgpu_buffer_rsrc_t ars[NSEG];
    unsigned arow[NSEG], astep[NSEG];
    int ast[NSEG], alim[NSEG];
#pragma unroll
    for (int sg = 0; sg < NSEG; ++sg) {
        const long long ld = g.a[sg].ld;
#ifdef ANERF_GEMM_PROBE_A  // (timing diagnostic only, wrong results: every tile reads rows 0..127, L2-hot)
        ars[sg] = __builtin_amdgcn_make_buffer_rsrc((void*)(g.a[sg].p), 0, (int)(rows * ld * 4), 0x00020000);
#else
        ars[sg] = __builtin_amdgcn_make_buffer_rsrc((void*)(g.a[sg].p + m0 * ld), 0, (int)(rows * ld * 4), 0x00020000);
#endif
        arow[sg] = (unsigned)(sr * ld * 4);
        astep[sg] = (unsigned)(RPS * ld * 4);
        ast[sg] = g.a[sg].start;
        alim[sg] = g.a[sg].start + (g.a[sg].cols + 3) / 4 * 4;
    }
    // this wave's B fragments: column block (n0 + 32 w) / 32 (the planes are zero padded to whole
    // 256-row tiles, so no block index needs a clamp)
    const long long bstride = (long long)ksteps * NPL * 512;  // elements per 32-column block
    const unsigned short* const bl = g.b + ((n0 + 32 * CB * wave) / 32) * bstride + lane * 8;

    f32x16 acc[RBM][CB];
#pragma unroll
    for (int i = 0; i < RBM; ++i)
#pragma unroll
        for (int cb = 0; cb < CB; ++cb) acc[i][cb] = f32x16{0};
    float ts[NRS];  // F16: the row scales 2^shift of this thread's staging rows
#pragma unroll
    for (int i = 0; i < NRS; ++i) {
        ts[i] = 1.0f;
        if constexpr (F16) {
            const long long m = m0 + sr + RPS * i;
            ts[i] = m < Md ? pow2i(f16_row_shift(g.rin[m])) : 1.0f;
        }
    }

    struct BF {
        u32x4 v[NPL][CB];
    };
    auto fetch_b = [&](int kt, BF& f) {
        kt = kt < nk ? kt : nk - 1;
        const unsigned short* bk = bl + (long long)kt * NPL * 512;
#pragma unroll
        for (int cb = 0; cb < CB; ++cb)
#pragma unroll
            for (int p = 0; p < NPL; ++p) f.v[p][cb] = *reinterpret_cast<const u32x4*>(bk + cb * bstride + p * 512);
    };
    struct RA {
        f32x4 v[NRS][NSEG];
    };
    // (steps past K read nothing: every column is outside every segment)
    auto fetch_a = [&](int st, RA& R) {
        const int col = st * SK + sc;
#pragma unroll
        for (int sg = 0; sg < NSEG; ++sg) {
            const unsigned vo = col >= ast[sg] && col < alim[sg] ? arow[sg] + (unsigned)(col - ast[sg]) * 4u : NOOB;
#pragma unroll
            for (int i = 0; i < NRS; ++i)
                R.v[i][sg] = __builtin_bit_cast(
                    f32x4, __builtin_amdgcn_raw_buffer_load_b128(ars[sg], vo + (unsigned)i * astep[sg], 0, 0));
        }
    };
    auto stage_a = [&](int buf, const RA& R) {
        unsigned short* const P = lds + buf * G::STAGE + nt_off<SKT>(sr, sc);  // (row sr + RPS i: same swizzle)
#pragma unroll
        for (int i = 0; i < NRS; ++i) {
            float v[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                // (through float rvalues: clang's bit_cast of a vector-element lvalue reads element 0)
                const float x0 = R.v[i][0][e];
                unsigned b = __builtin_bit_cast(unsigned, x0);
#pragma unroll
                for (int sg = 1; sg < NSEG; ++sg) {  // (one segment is live per lane, the others read 0)
                    const float xs = R.v[i][sg][e];
                    b |= __builtin_bit_cast(unsigned, xs);
                }
                v[e] = __builtin_bit_cast(float, b);
            }
            if constexpr (F16) {  // x t = x0 + x1: fp16 round to nearest, then the exact remainder's
                typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
                unsigned w0[2], w1[2];
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    const f32x2 x = (f32x2){v[2 * q] * ts[i], v[2 * q + 1] * ts[i]};
                    const f16x2 hi = __builtin_convertvector(x, f16x2);
                    const f32x2 r = x - __builtin_convertvector(hi, f32x2);
                    w0[q] = __builtin_bit_cast(unsigned, hi);
                    w1[q] = __builtin_bit_cast(unsigned, __builtin_convertvector(r, f16x2));
                }
                *reinterpret_cast<u32x2*>(P + RPS * i * SK) = u32x2{w0[0], w0[1]};
                *reinterpret_cast<u32x2*>(P + G::PLANE + RPS * i * SK) = u32x2{w1[0], w1[1]};
                continue;
            }
#pragma unroll
            for (int p = 0; p < NPL; ++p) {
                unsigned w[2];
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    const bf16x2 h = __builtin_convertvector((f32x2){v[2 * q], v[2 * q + 1]}, bf16x2);
                    w[q] = __builtin_bit_cast(unsigned, h);
                    if (p + 1 < NPL) {
                        v[2 * q] -= (float)h[0];
                        v[2 * q + 1] -= (float)h[1];
                    }
                }
                typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
                *reinterpret_cast<u32x2*>(P + p * G::PLANE + RPS * i * SK) = u32x2{w[0], w[1]};
            }
        }
    };
    auto step = [&](int buf, int kk, const BF& f) {
        const unsigned short* A = lds + buf * G::STAGE;
        const int r = lane & 31, kh = 16 * kk + 8 * (lane >> 5);
        bf16x8 a[NPL][RBM], b[NPL][CB];
#pragma unroll
        for (int i = 0; i < RBM; ++i)
#pragma unroll
            for (int p = 0; p < NPL; ++p)
                a[p][i] = *reinterpret_cast<const bf16x8*>(A + p * G::PLANE + nt_off<SKT>(32 * i + r, kh));
#pragma unroll
        for (int p = 0; p < NPL; ++p)
#pragma unroll
            for (int cb = 0; cb < CB; ++cb) b[p][cb] = __builtin_bit_cast(bf16x8, f.v[p][cb]);
#pragma unroll
        for (int cb = 0; cb < CB; ++cb)
#pragma unroll
            for (int i = 0; i < RBM; ++i) {
                f32x16 c = acc[i][cb];
                if constexpr (F16) {  // the four products, small terms first
                    c = mfma16(a[1][i], b[1][cb], c);
                    c = mfma16(a[1][i], b[0][cb], c);
                    c = mfma16(a[0][i], b[1][cb], c);
                    acc[i][cb] = mfma16(a[0][i], b[0][cb], c);
                    continue;
                }
                if constexpr (NPL == 3) {
                    c = mfma(a[2][i], b[0][cb], c);
                    c = mfma(a[1][i], b[1][cb], c);
                    c = mfma(a[0][i], b[2][cb], c);
                }
                c = mfma(a[1][i], b[0][cb], c);
                c = mfma(a[0][i], b[1][cb], c);
                acc[i][cb] = mfma(a[0][i], b[0][cb], c);
            }
    };
    // B fragments (the split weights, L2-resident) in a ring of BD k16-steps, prefetched BD - 1 steps
    // ahead: the waves' SQ counters showed them parked at s_waitcnt 45 % of the time with the B loads
    // one k16-step (12 MFMAs) ahead of their use (profiles/r04l_pmc_waves.txt); two more register sets
    // fit the single-segment instances (ANERF_GEMM_BD; the multi-segment ones keep the 2-ring)
    constexpr int BD = (NSEG == 1 && ANERF_GEMM_BD == 4 && CB == 1) ? 4 : 2;
    RA R0, R1;
    BF f[BD];
    fetch_a(0, R0);
    fetch_a(1, R1);
#pragma unroll
    for (int j = 0; j < BD - 1; ++j) fetch_b(j, f[j]);
    __builtin_amdgcn_sched_barrier(0);
    stage_a(0, R0);
    __syncthreads();
    // (sched_barrier after every fetch: without it the scheduler sinks the loads to their first use
    // to save registers, and each then waits out its full round trip)
    // k16-step q0 + j of an iteration (j < 2 KK: buffer j / KK, half j % KK) uses f[j % BD] (BD divides
    // 2 KK) and first fetches step q0 + j + BD - 1 into the slot the previous step freed
    for (int st = 0; st < nst; st += 2) {
        const int q0 = KK * st;
        fetch_a(st + 2, R0);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int kk = 0; kk < KK; ++kk) {
            fetch_b(q0 + kk + BD - 1, f[(kk + BD - 1) % BD]);
            __builtin_amdgcn_sched_barrier(0);
            step(0, kk, f[kk % BD]);
            __builtin_amdgcn_sched_barrier(0);
        }
        if (st + 1 < nst) stage_a(1, R1);
        __syncthreads();
        if (st + 1 >= nst) break;
        fetch_a(st + 3, R1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int kk = 0; kk < KK; ++kk) {
            fetch_b(q0 + KK + kk + BD - 1, f[(KK + kk + BD - 1) % BD]);
            __builtin_amdgcn_sched_barrier(0);
            step(1, kk, f[(KK + kk) % BD]);
            __builtin_amdgcn_sched_barrier(0);
        }
        if (st + 2 < nst) stage_a(0, R0);
        __syncthreads();
    }
    // epilogue through LDS: the waves write their accumulators (lane = column (lane & 31), registers
    // = rows (r & 3) + 8 (r >> 2) + 4 (lane >> 5)) into a [128][132] fp32 tile, then every wave
    // instruction handles two whole 512 B output rows with 16 B per lane (bias, relu, relu' mask,
    // accumulate, segment split).
    constexpr int TP = 132;  // tile pitch (floats)
    float* const tile = reinterpret_cast<float*>(lds);
    // (CB 2: two passes over the [128][132] tile, 128 columns each, written by waves 2 hh and 2 hh + 1)
#pragma unroll
    for (int hh = 0; hh < CB; ++hh) {
    if (hh) __syncthreads();
    if (CB == 1 || (wave >> 1) == hh) {
#pragma unroll
        for (int cb = 0; cb < CB; ++cb)
#pragma unroll
            for (int i = 0; i < RBM; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int row = 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                    tile[row * TP + 32 * CB * wave + 32 * cb - 128 * hh + (lane & 31)] = acc[i][cb][r];
                }
    }
    __syncthreads();
    // thread t: rows 8 q + (t >> 5) (q < TBM / 8), columns 4 (t & 31) .. + 3
    const int c4 = 4 * (tid & 31), rb = tid >> 5;
    const int n = n0 + 128 * hh + c4;
    const int Nd = g.N;
    if (n < Nd) {
        const int cs1 = g.nc > 1 ? g.c[1].start : Nd, cs2 = g.nc > 2 ? g.c[2].start : Nd;
        const float* const bias = g.bias;
        const int relu = g.relu;
        const int si = n >= cs2 ? 2 : (n >= cs1 ? 1 : 0);
        float* const op = tab->op[si];
        const long long old = tab->old[si];
        const float* const mp = tab->mask[si];
        const long long ldm = tab->ldm[si];
        const bool need_acc = tab->accum[si] != 0;
        const bool pre = tab->accum[si] == 2;  // (the old value joins the pre-activation: before the relu)
        const int start = si == 2 ? cs2 : (si == 1 ? cs1 : 0);
        const int col = n - start;
        const int send = si == 2 ? Nd : (si == 1 ? cs2 : cs1);  // end of this segment
        // the whole float4 inside one segment and 16 B aligned: vector path, else per element
        const bool vec = n + 4 <= send && ((((uintptr_t)(op + col)) | (old * 4)) & 15) == 0 &&
                         (!mp || ((((uintptr_t)(mp + col)) | (ldm * 4)) & 15) == 0);
        f32x4 bv = {0.0f, 0.0f, 0.0f, 0.0f};
        if (bias) {
#pragma unroll
            for (int e = 0; e < 4; ++e) bv[e] = n + e < Nd ? bias[n + e] : 0.0f;
        }
        // mask / accumulate operands of all 16 rows first (clamped rows: no load waits on a branch)
        f32x4 mk[TBM / 8], ov[TBM / 8];
        if (vec && op && mp) {
#pragma unroll
            for (int q = 0; q < TBM / 8; ++q) {
                long long m = m0 + 8 * q + rb;
                m = m < Md ? m : Md - 1;
                mk[q] = *(gf32x4*)(mp + m * ldm + col);
            }
        }
        if (vec && op && need_acc) {
#pragma unroll
            for (int q = 0; q < TBM / 8; ++q) {
                long long m = m0 + 8 * q + rb;
                m = m < Md ? m : Md - 1;
                ov[q] = *(gf32x4*)(op + m * old + col);
            }
        }
        int* const rout = g.rout;  // (the host allows it with n % 128 == 0: every lane of a row is here)
        const float uw = F16 ? pow2i(-g.bexp[0]) : 1.0f;  // fp16x4: undo the weights' and rows' scales
        if (vec) {
#pragma unroll
            for (int q = 0; q < TBM / 8; ++q) {
                const int row = 8 * q + rb;
                const long long m = m0 + row;
                f32x4 v = *reinterpret_cast<const f32x4*>(tile + row * TP + c4);
                if constexpr (F16) {
                    const float ur = pow2i(-rsh[row]);
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] = v[e] * uw * ur;  // (exact: powers of two)
                }
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    v[e] += bv[e];
                    if (pre) v[e] += ov[q][e];
                    if (relu) v[e] = fmaxf(v[e], 0.0f);
                }
                if (rout) {  // the row's largest |output| (for the next layer's fp16x4 scale): a max over
                    // each 16-lane DPP row (quad xor 1, xor 2, half-row mirror, row mirror), one atomic per row
                    int mx = __builtin_bit_cast(
                        int, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
                    mx = max(mx, __builtin_amdgcn_update_dpp(0, mx, 0xB1, 0xF, 0xF, false));
                    mx = max(mx, __builtin_amdgcn_update_dpp(0, mx, 0x4E, 0xF, 0xF, false));
                    mx = max(mx, __builtin_amdgcn_update_dpp(0, mx, 0x141, 0xF, 0xF, false));
                    mx = max(mx, __builtin_amdgcn_update_dpp(0, mx, 0x140, 0xF, 0xF, false));
                    if ((lane & 15) == 0 && m < Md) atomicMax(rout + m, mx);
                }
                if (op && m < Md) {
                    if (mp) {
#pragma unroll
                        for (int e = 0; e < 4; ++e) v[e] = mk[q][e] > 0.0f ? v[e] : 0.0f;
                    }
                    if (need_acc && !pre) {
#pragma unroll
                        for (int e = 0; e < 4; ++e) v[e] += ov[q][e];
                    }
                    *reinterpret_cast<f32x4*>(op + m * old + col) = v;
                }
            }
        } else {  // (segment boundaries inside the float4, ragged last columns, unaligned outputs)
#pragma unroll 1
            for (int q = 0; q < TBM / 8; ++q) {
                const int row = 8 * q + rb;
                const long long m = m0 + row;
                if (m >= Md) break;
#pragma unroll 1
                for (int e = 0; e < 4; ++e) {
                    const int ne = n + e;
                    if (ne >= Nd) break;
                    const int se = ne >= cs2 ? 2 : (ne >= cs1 ? 1 : 0);
                    float* const ope = tab->op[se];
                    if (!ope) continue;
                    float x = tile[row * TP + c4 + e];
                    if constexpr (F16) x = x * uw * pow2i(-rsh[row]);
                    x += bv[e];
                    const int ce = ne - (se == 2 ? cs2 : (se == 1 ? cs1 : 0));
                    float* de = ope + m * tab->old[se] + ce;
                    if (tab->accum[se] == 2) x += *de;
                    if (relu) x = fmaxf(x, 0.0f);
                    if (rout) atomicMax(rout + m, __builtin_bit_cast(int, fabsf(x)));
                    const float* const mpe = tab->mask[se];
                    if (mpe && !(mpe[m * tab->ldm[se] + ce] > 0.0f)) x = 0.0f;
                    if (tab->accum[se] == 1) x += *de;
                    *de = x;
                }
            }
        }
    }
    }  // (hh: the tile's 128-column halves)
}

// ---------------------------------------------------------------- weight gradient
// dW tile 128 (n) x 128 (k) per workgroup over a slab of rows (4 waves, 2 x 2: 64 x 64 each).  Both
// operands are activations read along their rows: a step stages 16 rows of dY (columns n0..) and of
// X (columns k0..) (32 rows for bf16x3 with one X segment), a thread 8 consecutive columns of a row
// (a wave instruction reads four whole 512 B row pieces), split into NPL bf16 planes kept row-major
// ([row][128], swizzled 256 B rows, one ds_write_b128 per plane and row).  The MFMA fragments (8
// rows of one column) come back through the hardware transpose read ds_read_b64_tr_b16, two per
// fragment, conflict-free with the swizzle.
// Loads are buffer loads through per-step descriptors whose range ends at the slab's last row, so
// rows past the slab and columns outside the operand read zero without a clamp or a select; a
// thread's offsets are constant over the whole slab.  Two LDS stages, two register sets in flight;
// the partial tile leaves through LDS in full rows.  The bias gradient (k-tile 0) sums the staged
// dY per column in a fixed order.
constexpr int TSK = 32;                 // rows per step, at most (slabs are whole pairs of steps)
// a lane offset past every descriptor's range: a step's range is at most 32 rows x ld x 4 B < 2^29
// for ld < 2^22 (checked on the host), and TOOB plus 16 rows of offset stays below 2^31
constexpr unsigned TOOB = 0x40000000u;

// plane [row][128 bf16]: 256 B rows whose 16 B chunks are XOR-swizzled by 4 (row & 3), so the four
// rows of a transposed read's lane group (64 B each) land on disjoint banks and a staging write (8
// lanes x one chunk of a row) stays conflict-free
__device__ __forceinline__ int tn_off(int row, int chunk) { return row * 256 + ((chunk ^ (4 * (row & 3))) << 4); }

template <int NPL, int NSEG>
struct TNGeo {
    // rows per step: 32 where two register sets of them fit in 256 VGPRs (bf16x3, one X segment),
    // else 16
    static constexpr int SK = NPL == 2 && NSEG == 1 ? 32 : 16;
    static constexpr int PR = SK / 16;             // rows per staging thread
    static constexpr int PLANE = SK * 256;         // bytes
    static constexpr int STAGE = 2 * NPL * PLANE;  // dY planes, then X planes
    static constexpr int LDS_BYTES = 2 * STAGE > 128 * 132 * 4 ? 2 * STAGE : 128 * 132 * 4;
};

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

template <int SK>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rows_rsrc(const float* p, long long ld, long long mb, long long mhi) {
    long long rows = mhi - mb;
    rows = rows < 0 ? 0 : (rows > SK ? SK : rows);
    return __builtin_amdgcn_make_buffer_rsrc((void*)(p + mb * ld), 0, (int)(rows * ld * 4), 0x00020000);
}

template <int NPL, int NSEG>
__global__ __launch_bounds__(NTHR, 2) void mlp_tn_kernel(TNArgs g) {
    using G = TNGeo<NPL, NSEG>;
    constexpr int SK = G::SK, PR = G::PR;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds8[];
    const int logical = xcd_logical(blockIdx.x, g.total);
    const int split = logical / g.tiles, tile = logical % g.tiles;
    const int nt = tile / g.tiles_k, kt_ = tile % g.tiles_k;
    const int n0 = nt * BN, k0 = kt_ * BM;
    const long long mlo = (long long)split * g.rows_per_split;
    long long mhi = mlo + g.rows_per_split;
    if (mhi > g.M) mhi = g.M;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave >> 1, wc = wave & 1;
    // staging unit: rows r + 16 u (u < PR) of the step, columns c8 .. c8 + 7 of the tile
    const int r = tid >> 4, c8 = 8 * (tid & 15);
    const unsigned ystep = (unsigned)(16 * g.lddy * 4);
    const float* const dyp = g.dy;
    const long long lddy = g.lddy;
    const int nlim = (g.N + 3) / 4 * 4;
    unsigned voy[2];
#pragma unroll
    for (int f = 0; f < 2; ++f) {
        const int col = n0 + c8 + 4 * f;
        voy[f] = col < nlim ? (unsigned)(r * lddy + col) * 4u : TOOB;
    }
    const float* xp[NSEG];
    long long xld[NSEG];
    unsigned vox[2][NSEG], xstep[NSEG];
#pragma unroll
    for (int sg = 0; sg < NSEG; ++sg) {
        xp[sg] = g.x[sg].p;
        xld[sg] = g.x[sg].ld;
        xstep[sg] = (unsigned)(16 * xld[sg] * 4);
        const int st0 = g.x[sg].start, lim = st0 + (g.x[sg].cols + 3) / 4 * 4;
#pragma unroll
        for (int f = 0; f < 2; ++f) {
            const int col = k0 + c8 + 4 * f;
            vox[f][sg] = col >= st0 && col < lim ? (unsigned)(r * xld[sg] + (col - st0)) * 4u : TOOB;
        }
    }
    const bool do_bias = g.wsb != nullptr && kt_ == 0;
    float bsum[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) bsum[e] = 0.0f;

    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{0};

    struct Regs {
        f32x4 y[PR][2], x[PR][2][NSEG];
    };
    // (a TOOB lane offset plus 16 rows stays past the range: ld < 2^22)
    auto fetch = [&](long long mb, Regs& R) {
        const __amdgpu_buffer_rsrc_t ry = rows_rsrc<SK>(dyp, lddy, mb, mhi);
#pragma unroll
        for (int u = 0; u < PR; ++u)
#pragma unroll
            for (int f = 0; f < 2; ++f)
                R.y[u][f] = __builtin_bit_cast(
                    f32x4, __builtin_amdgcn_raw_buffer_load_b128(ry, voy[f] + (unsigned)u * ystep, 0, 0));
#pragma unroll
        for (int sg = 0; sg < NSEG; ++sg) {
            const __amdgpu_buffer_rsrc_t rx = rows_rsrc<SK>(xp[sg], xld[sg], mb, mhi);
#pragma unroll
            for (int u = 0; u < PR; ++u)
#pragma unroll
                for (int f = 0; f < 2; ++f)
                    R.x[u][f][sg] = __builtin_bit_cast(
                        f32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, vox[f][sg] + (unsigned)u * xstep[sg], 0, 0));
        }
    };
    // 8 values -> NPL planes of packed bf16 pairs (round to nearest even of the running remainder)
    auto split_store = [&](float (&v)[8], unsigned char* dst) {
#pragma unroll
        for (int p = 0; p < NPL; ++p) {
            u32x4 w;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const bf16x2 h = __builtin_convertvector((f32x2){v[2 * q], v[2 * q + 1]}, bf16x2);
                w[q] = __builtin_bit_cast(unsigned, h);
                if (p + 1 < NPL) {
                    v[2 * q] -= (float)h[0];
                    v[2 * q + 1] -= (float)h[1];
                }
            }
            *reinterpret_cast<u32x4*>(dst + p * G::PLANE) = w;
        }
    };
    auto stage = [&](int buf, const Regs& R) {
#pragma unroll
        for (int u = 0; u < PR; ++u) {
            // (rows r + 16 u share r's swizzle)
            unsigned char* const P = lds8 + buf * G::STAGE + tn_off(r + 16 * u, c8 >> 3);
            float y[8], x[8];
#pragma unroll
            for (int f = 0; f < 2; ++f)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    y[4 * f + e] = R.y[u][f][e];
                    // (through float rvalues: clang's bit_cast of a vector-element lvalue reads element 0)
                    const float x0 = R.x[u][f][0][e];
                    unsigned b = __builtin_bit_cast(unsigned, x0);
#pragma unroll
                    for (int sg = 1; sg < NSEG; ++sg) {  // (one segment is live per lane, the others read 0)
                        const float xs = R.x[u][f][sg][e];
                        b |= __builtin_bit_cast(unsigned, xs);
                    }
                    x[4 * f + e] = __builtin_bit_cast(float, b);
                }
            if (do_bias) {
#pragma unroll
                for (int e = 0; e < 8; ++e) bsum[e] += y[e];
            }
            split_store(y, P);
            split_store(x, P + NPL * G::PLANE);
        }
    };
    // fragment = rows 16 kk + 8h .. + 7 of columns cb .. cb + 31: lane 4q + p of each 16-lane group
    // addresses row q (+4) at column 4p of its half (8 B = half of chunk cb / 8 + 2 g1 + p / 2)
    const int h = lane >> 5, q = (lane >> 2) & 3, p4 = lane & 3, g1 = (lane >> 4) & 1;
    auto frag = [&](const unsigned char* plane, int kk, int cb) {
        const int row = 16 * kk + 8 * h + q, chunk = (cb >> 3) + 2 * g1 + (p4 >> 1);
        const unsigned char* a = plane + tn_off(row, chunk) + 8 * (p4 & 1);
        const unsigned char* a4 = plane + tn_off(row + 4, chunk) + 8 * (p4 & 1);  // (same swizzle)
        const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)a);
        const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)a4);
        return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    };
    auto step = [&](int buf) {
        const unsigned char* const P = lds8 + buf * G::STAGE;
#pragma unroll
        for (int kk = 0; kk < PR; ++kk) {
            bf16x8 a[NPL][2], b[NPL][2];
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int p = 0; p < NPL; ++p) {
                    a[p][i] = frag(P + p * G::PLANE, kk, 64 * wr + 32 * i);
                    b[p][i] = frag(P + (NPL + p) * G::PLANE, kk, 64 * wc + 32 * i);
                }
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    f32x16 c = acc[i][j];
                    if constexpr (NPL == 3) {
                        c = mfma(a[2][i], b[0][j], c);
                        c = mfma(a[1][i], b[1][j], c);
                        c = mfma(a[0][i], b[2][j], c);
                    }
                    c = mfma(a[1][i], b[0][j], c);
                    c = mfma(a[0][i], b[1][j], c);
                    acc[i][j] = mfma(a[0][i], b[0][j], c);
                }
        }
    };
    // two LDS stages, two register sets: the loads of step s + 2 fly during steps s and s + 1
    const int nsteps = mhi > mlo ? (int)((mhi - mlo + SK - 1) / SK) : 0;
    Regs R0, R1;
    if (nsteps > 0) {
        fetch(mlo, R0);
        fetch(mlo + SK, R1);
        __builtin_amdgcn_sched_barrier(0);
        stage(0, R0);
    }
    __syncthreads();
    for (int st = 0; st < nsteps; st += 2) {
        fetch(mlo + (long long)(st + 2) * SK, R0);
        __builtin_amdgcn_sched_barrier(0);  // (keep the loads ahead of the MFMAs)
        step(0);
        __builtin_amdgcn_sched_barrier(0);
        if (st + 1 < nsteps) stage(1, R1);
        __syncthreads();
        if (st + 1 >= nsteps) break;
        fetch(mlo + (long long)(st + 3) * SK, R1);
        __builtin_amdgcn_sched_barrier(0);
        step(1);
        __builtin_amdgcn_sched_barrier(0);
        if (st + 2 < nsteps) stage(0, R0);
        __syncthreads();
    }
    // partial tile through LDS ([128][132] fp32), then whole 512 B rows into the workspace
    float* const tile_f = reinterpret_cast<float*>(lds8);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = 64 * wr + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                tile_f[row * 132 + 64 * wc + 32 * j + (lane & 31)] = acc[i][j][r];
            }
    __syncthreads();
    float* const wt = g.ws + (long long)split * g.npad * g.kpad + (long long)n0 * g.kpad + k0;
#pragma unroll 8
    for (int q = 0; q < 16; ++q) {  // 256 threads = 8 rows x 32 float4 per pass
        const int row = 8 * q + (tid >> 5);
        const f32x4 v = *reinterpret_cast<const f32x4*>(tile_f + row * 132 + 4 * (tid & 31));
        *reinterpret_cast<f32x4*>(wt + (long long)row * g.kpad + 4 * (tid & 31)) = v;
    }
    if (do_bias) {  // column sums over the 16 staging rows, in a fixed order
        __syncthreads();
        float* const red = tile_f;  // [16][128]
#pragma unroll
        for (int e = 0; e < 8; ++e) red[r * 128 + c8 + e] = bsum[e];
        __syncthreads();
        if (tid < 128) {
            float t = red[tid];
#pragma unroll
            for (int w = 1; w < 16; ++w) t += red[w * 128 + tid];
            g.wsb[(long long)split * g.npad + n0 + tid] = t;
        }
    }
}

// dst[row][col] (+)= sum over the slabs of src[t][row][col]: a workgroup takes 128 columns of one row,
// 32 float4 column groups x 8 slab groups (each a contiguous run of slabs, 4 loads in flight), the 8
// partial sums then added in slab-group order through LDS (deterministic).  src rows hold a multiple
// of 128 columns (the workspace's padding).  Row `rows` (when bsrc is set) is the bias gradient:
// the same sum over bsrc[t][col] (slab stride bstride, bcols columns) into bdst, in the same launch.
__global__ __launch_bounds__(256) void mlp_reduce_kernel(const float* __restrict__ src, int splits,
                                                         long long split_stride, long long row_stride, int cols,
                                                         float* __restrict__ dst, long long ldd, int accum, int rows,
                                                         const float* __restrict__ bsrc, long long bstride,
                                                         int bcols, float* __restrict__ bdst) {
    __shared__ f32x4 part[8][32];
    const int cg = threadIdx.x & 31, sgi = threadIdx.x >> 5;
    int row = blockIdx.y;
    const int c0 = blockIdx.x * 128 + 4 * cg;
    if (row == rows) {  // (uniform per workgroup) the bias row
        src = bsrc;
        split_stride = bstride;
        row_stride = 0;
        cols = bcols;
        dst = bdst;
        ldd = 0;
        row = 0;
    }
    if (blockIdx.x * 128 >= cols) return;  // (a row narrower than the grid; uniform per workgroup)
    const int chunk = (splits + 7) / 8;
    const int t0 = sgi * chunk, t1 = t0 + chunk < splits ? t0 + chunk : splits;
    const float* p = src + row * row_stride + c0;
    f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
    int t = t0;
    for (; t + 4 <= t1; t += 4) {
        f32x4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const f32x4*>(p + (t + u) * split_stride);
#pragma unroll
        for (int u = 0; u < 4; ++u) acc += v[u];
    }
    for (; t < t1; ++t) acc += *reinterpret_cast<const f32x4*>(p + t * split_stride);
    part[sgi][cg] = acc;
    __syncthreads();
    if (sgi == 0) {
        f32x4 s = part[0][cg];
#pragma unroll
        for (int w = 1; w < 8; ++w) s += part[w][cg];
        float* o = dst + row * ldd + c0;
#pragma unroll
        for (int e = 0; e < 4; ++e)
            if (c0 + e < cols) o[e] = accum ? o[e] + s[e] : s[e];
    }
}

// weight -> NPL bf16 planes in MFMA fragment order: for 32-row block nb, k16 step ks, plane p one
// 1 KB run of 64 lanes x 8 bf16, lane l = row nb*32 + (l & 31), columns ks*16 + 8 (l >> 5) + 0..7
// (the B operand lane map of v_mfma_f32_32x32x16_bf16), zero padded.  Rows are w's rows (or, when
// transposed, w's columns).
__device__ __forceinline__ void split_weights_elem(const float* __restrict__ w, int n, int k, long long ldw,
                                                   int transpose, int nblocks, int ksteps, int npl,
                                                   unsigned short* __restrict__ out, long long idx,
                                                   const int* __restrict__ f16exp = nullptr) {
    const long long per = (long long)nblocks * ksteps * 512;
    if (idx >= per) return;
    const int e = (int)(idx & 7), l = (int)((idx >> 3) & 63);
    const long long blk = idx >> 9;  // nb * ksteps + ks
    const int ks = (int)(blk % ksteps), nb = (int)(blk / ksteps);
    const int row = nb * 32 + (l & 31), col = ks * 16 + 8 * (l >> 5) + e;
    const int rows = transpose ? k : n, cols = transpose ? n : k;
    const int wn = transpose ? col : row, wk = transpose ? row : col;
    float x = (row < rows && col < cols) ? w[(long long)wn * ldw + wk] : 0.0f;
    if (f16exp) {  // fp16x4: w 2^ew = w0 + w1, fp16 round to nearest of the running remainder
        x *= pow2i(f16exp[0]);
        const _Float16 h0 = (_Float16)x;
        const _Float16 h1 = (_Float16)(x - (float)h0);
        out[((blk * 2 + 0) << 9) + (l << 3) + e] = __builtin_bit_cast(unsigned short, h0);
        out[((blk * 2 + 1) << 9) + (l << 3) + e] = __builtin_bit_cast(unsigned short, h1);
        return;
    }
    for (int p = 0; p < npl; ++p) {
        const __bf16 xh = (__bf16)x;
        out[((blk * npl + p) << 9) + (l << 3) + e] = __builtin_bit_cast(unsigned short, xh);
        x -= (float)xh;
    }
}

__global__ void split_weights_kernel(const float* __restrict__ w, int n, int k, long long ldw, int transpose,
                                     int nblocks, int ksteps, int npl, unsigned short* __restrict__ out) {
    split_weights_elem(w, n, k, ldw, transpose, nblocks, ksteps, npl, out,
                       (long long)blockIdx.x * blockDim.x + threadIdx.x);  // one (nb, ks, lane, e)
}

constexpr int MAXJOBS = 32;
struct SplitJob {
    const float* w;
    unsigned short* out;
    int* f16exp;  // fp16x4: the weights' exponent (the split buffer's tail), else null
    long long ldw;
    int n, k, transpose, nblocks, ksteps, npl;
    int block0;  // first workgroup of this job
};
struct SplitBatch {
    SplitJob j[MAXJOBS];
    int n;
};

// every job's workgroups in one grid: a workgroup finds its job by a uniform scan of the starts
__global__ void split_weights_batch_kernel(SplitBatch b) {
    int q = 0;
    for (int t = 1; t < b.n; ++t)
        if ((int)blockIdx.x >= b.j[t].block0) q = t;
    // (fields through locals: a per-job select of the argument struct stays in scalar registers)
    const SplitJob J = b.j[q];
    split_weights_elem(J.w, J.n, J.k, J.ldw, J.transpose, J.nblocks, J.ksteps, J.npl, J.out,
                       (long long)(blockIdx.x - J.block0) * blockDim.x + threadIdx.x, J.f16exp);
}

// fp16x4 weights: the exponent ew that puts max |w| in [2^10, 2^11) (the render path's h3_exponent),
// one workgroup per job, written to the job's split-buffer tail before the split reads it
// one 1024-thread workgroup per fp16x4 job: wave w reads rows w, w + 16, ... (coalesced, 4 loads in
// flight per lane), then a wave and a workgroup max
__global__ __launch_bounds__(1024) void split_exponent_kernel(SplitBatch b) {
    const SplitJob J = b.j[blockIdx.x];
    if (!J.f16exp) return;
    __shared__ int red[16];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int m = 0;
    for (int r = wave; r < J.n; r += 16) {
        const float* const row = J.w + (long long)r * J.ldw;
#pragma unroll 4
        for (int c = lane; c < J.k; c += 64) m = max(m, __builtin_bit_cast(int, fabsf(row[c])));
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = max(m, __shfl_xor(m, o));
    if (lane == 0) red[wave] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        int mm = 0;
#pragma unroll
        for (int i = 0; i < 16; ++i) mm = max(mm, red[i]);
        J.f16exp[0] = (mm > 0 && mm < 0x7f800000) ? min(max(137 - (mm >> 23), -126), 126) : 0;
    }
}

// ---------------------------------------------------------------- hidden layer backward, fused (round 6)
// One launch per 256 x 256 hidden layer produces both products of its backward from ONE read of dY (the
// layer's pre-activation gradient) and X (its input, the previous layer's relu output):
//   dX = (dY W) * (X > 0)        the input gradient, relu' masked (what mlp_nt_kernel's backward epilogue does)
//   dW = dY^T X, db = sum_m dY    the weight and bias gradients (what mlp_tn_kernel does)
// The two-kernel schedule read dY and X twice (336 MB per layer at M = 163,840 in fp32) and ran the products on
// two streams; here a persistent workgroup per CU owns a contiguous range of rows and walks it in 32-row chunks:
// each chunk's dY and X are staged once into LDS as bf16 hi / lo planes (bf16x3, the backward's arithmetic in
// the "mixed" mode) and feed both products.
// Eight waves, two per SIMD (256 registers each).  Every wave w keeps rows 32 w .. 32 w + 31 of the workgroup's
// 256 x 256 dW partial (8 tiles of 32 x 32, 128 accumulator registers) over the whole row range; it leaves once,
// into a per-workgroup workspace slab summed in slab order by mlp_reduce_kernel (deterministic, no atomics).
// The other work is split by role, one wave of each role per SIMD:
//   * stager waves (0-3) load the next chunks' dY and X rows from HBM and split them into the LDS planes, a
//     unit (one row piece) every other slot of the current chunk's compute, a whole chunk ahead;
//   * dX waves (4-7) compute dX's columns 64 (w - 4) .. + 63 of every chunk, their B operand (the split W^T)
//     from L2 as MFMA fragments one k16 step ahead.
// The split keeps HBM loads out of the waves that wait on L2 loads: vector-memory loads of a wave complete in
// order (vmcnt), so a wave that issued a chunk's HBM loads could not wait for a later W^T fragment before them.
// LDS per chunk: dY hi, dY lo, X hi, X lo ([32][256] bf16 each, 512 B rows whose 16 B chunks are XOR-swizzled
// by ((r & 3) << 2) | ((r >> 2) & 3): conflict-free for the transposed dW fragment reads (4 rows x 64 B per
// lane group), the row-wise dX fragment reads (16 rows of one chunk per group) and the staging writes) and the
// relu' mask bytes; two stages, plus the db column sums.
constexpr int DGW_W = 256;                           // layer width (inputs = outputs)
constexpr int DGW_CH = 32;                           // rows per chunk
constexpr int DGW_THR = 512;                         // eight waves
constexpr int DGW_PLANE = DGW_CH * DGW_W * 2;        // 16 KB: one bf16 plane [32][256]
constexpr int DGW_MASKB = DGW_CH * DGW_W;            // 8 KB: relu' mask bytes [32][256]
constexpr int DGW_GA = 4 * DGW_PLANE + DGW_MASKB;     // the head pass: the chunk's 32 alpha gradients (fp32)
constexpr int DGW_STAGE = DGW_GA + DGW_CH * 4;
constexpr int DGW_BSUM = 8 * DGW_W * 4;              // 8 KB: the db column sums [8 staging rows][256]
constexpr int DGW_LDS = 2 * DGW_STAGE + DGW_BSUM;    // 152.25 KB
#ifndef ANERF_DGW_BD
#define ANERF_DGW_BD 4
#endif
constexpr int DGW_BD = ANERF_DGW_BD;                 // W^T fragment ring depth (k16 steps)
static_assert((DGW_W / 16) % DGW_BD == 0, "the W^T ring runs on across chunks: its depth divides the k16 steps");
// (ANERF_DGW_PROBE, timing diagnostics of experiment builds only, wrong results: 1 no dX MFMAs, 2 no dW MFMAs,
// 3 no W^T loads, 4 no chunk staging after the first)
#ifndef ANERF_DGW_PROBE
#define ANERF_DGW_PROBE 0
#endif

struct DGWArgs {
    long long M, rows_per_wg;
    const float* dy;
    long long lddy;
    const float* x;
    long long ldx;
    const unsigned short* wt;  // split W^T, bf16x3 planes (anerf_mlp_split_weights, transpose = 1)
    float* dx;
    long long lddx;
    float* ws;   // [workgroups][256 (+ 1)][256] dW partials
    float* wsb;  // [workgroups][256 (+ 4)] db partials
    const float* wa;  // the head pass: alpha_linear's weight row [256] (its gradient column is dy's column 256)
};

__device__ __forceinline__ int dgw_off(int row, int chunk) {
    return row * 512 + ((chunk ^ (((row & 3) << 2) | ((row >> 2) & 3))) << 4);
}

// 8 values -> bf16 hi (RNE) and lo (RNE of the exact remainder) at the same swizzled chunk of two planes
__device__ __forceinline__ void dgw_split_store(const float (&v)[8], unsigned char* hi, unsigned char* lo, int off) {
    u32x4 wh, wl;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const bf16x2 h = __builtin_convertvector((f32x2){v[2 * q], v[2 * q + 1]}, bf16x2);
        wh[q] = __builtin_bit_cast(unsigned, h);
        const bf16x2 l = __builtin_convertvector((f32x2){v[2 * q] - (float)h[0], v[2 * q + 1] - (float)h[1]}, bf16x2);
        wl[q] = __builtin_bit_cast(unsigned, l);
    }
    *reinterpret_cast<u32x4*>(hi + off) = wh;
    *reinterpret_cast<u32x4*>(lo + off) = wl;
}

// HEAD (the feature_linear + alpha_linear pass, anerf_mlp_backward_head): dY has a 257th column g_a, the gradient
// of alpha_linear's output.  dX gains its rank-1 term, (dY W + g_a w_a^T) * (X > 0), in the epilogue (g_a staged
// per chunk in LDS, w_a in two registers per dX lane); dW gains the row g_a^T X and db the entry sum g_a, summed by
// the stager waves in fp32 as they split X (slab row 256, db entry 256)
template <bool HEAD>
__global__ __launch_bounds__(DGW_THR, 1) void mlp_dgw_kernel(DGWArgs g) {
    constexpr int SROWS = HEAD ? DGW_W + 1 : DGW_W, BST = HEAD ? DGW_W + 4 : DGW_W;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds8[];
    // (the wave index as a uniform value: a buffer descriptor built from a per-lane value compiles to a
    // waterfall loop around every load, and the role branches must be uniform)
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool stager = wave < 4;
    const long long M = g.M;
    const long long mlo = (long long)blockIdx.x * g.rows_per_wg;
    const long long mhi = mlo + g.rows_per_wg < M ? mlo + g.rows_per_wg : M;
    const int nch = mhi > mlo ? (int)((mhi - mlo + DGW_CH - 1) / DGW_CH) : 0;

    // dW fragments (8 rows of one column) through the transpose read, as mlp_tn_kernel's: lane 4 q + p4 of each
    // 16-lane group addresses row q (+ 4) at columns 16 g1 + 4 p4 of the 32-column block.  `ln` is the lane index
    // re-pinned in every slot, so that no slot's address arithmetic is hoisted and kept live across the loop
    int ln = lane;
    auto tfrag = [&](const unsigned char* plane, int kk, int cb) {
        const int h = ln >> 5, q = (ln >> 2) & 3, p4 = ln & 3, g1 = (ln >> 4) & 1;
        const int row = 16 * kk + 8 * h + q, chunk = (cb >> 3) + 2 * g1 + (p4 >> 1);
        const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
            (lds_bf16x4*)(plane + dgw_off(row, chunk) + 8 * (p4 & 1)));
        const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
            (lds_bf16x4*)(plane + dgw_off(row + 4, chunk) + 8 * (p4 & 1)));
        return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    };
    // dX A fragments: row (lane & 31) of the chunk, k = 16 kt + 8 (lane >> 5) .. + 7 (one ds_read_b128)
    auto rfrag = [&](const unsigned char* plane, int kt) {
        return *reinterpret_cast<const bf16x8*>(plane + dgw_off(ln & 31, 2 * kt + (ln >> 5)));
    };
    auto pin_lane = [&]() {
        ln = lane;
        asm volatile("" : "+v"(ln));
    };

    f32x16 aw[8];  // dW rows 32 w .., columns 32 ib ..
#pragma unroll
    for (int j = 0; j < 8; ++j) aw[j] = f32x16{0};
    // the dW work of slot t (kk = t / 8, ib = t % 8), A fragments of the k16 step in `ad`
    auto dw_slot = [&](const unsigned char* S, int t, bf16x8 (&ad)[2]) {
        const int kk = t >> 3, ib = t & 7;
        if (ib == 0) {
#pragma unroll
            for (int p = 0; p < 2; ++p) ad[p] = tfrag(S + p * DGW_PLANE, kk, 32 * wave);
        }
        const bf16x8 bx0 = tfrag(S + 2 * DGW_PLANE, kk, 32 * ib), bx1 = tfrag(S + 3 * DGW_PLANE, kk, 32 * ib);
        if (ANERF_DGW_PROBE != 2) {
            f32x16 c = mfma(ad[1], bx0, aw[ib]);
            c = mfma(ad[0], bx1, c);
            aw[ib] = mfma(ad[0], bx0, c);
        }
    };

    if (stager) {
        // ------------------------------------------------------------------ stager waves
        // staging: thread t < 256 -> columns c8 .. c8 + 7 of rows sr + 8 u (u < 4) of dY and X: 8 units (u, operand)
        // of two float4 loads each (a wave instruction reads two whole rows)
        const int c8 = 8 * (tid & 31), sr = tid >> 5;
        const long long lddy = g.lddy, ldx = g.ldx;
        const float* const dyp = g.dy;
        const float* const xp = g.x;
        const unsigned voy = (unsigned)((sr * lddy + c8) * 4), vox = (unsigned)((sr * ldx + c8) * 4);
        const int ystep = (int)(8 * lddy * 4), xstep = (int)(8 * ldx * 4);
        f32x4 R[8][2];  // unit k = 2 u + operand (0: dY, 1: X)
        // (HEAD) g_a of the X unit's rows, loaded with that unit (it is consumed when the unit is staged, before the
        // next chunk's loads reuse the register); the thread's sums of g_a X over its rows and columns, and of g_a
        float Ga[4] = {0.0f, 0.0f, 0.0f, 0.0f};
        float xa[8] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
        float dba = 0.0f;
        const unsigned voa = (unsigned)(sr * lddy * 4);
        // (chunk rows past the workgroup's range read zero: the descriptors end at its last row; one lane offset per
        // operand, the row step and the 16 B piece in the uniform offset)
        auto fetch_unit = [&](int s, int k) {
            const long long r0 = mlo + (long long)s * DGW_CH;
            long long rows = mhi - r0;
            rows = rows < 0 ? 0 : (rows > DGW_CH ? DGW_CH : rows);
            const int u = k >> 1;
            const float* const base = (k & 1) ? xp + r0 * ldx : dyp + r0 * lddy;
            const long long ld = (k & 1) ? ldx : lddy;
            const __amdgpu_buffer_rsrc_t rs =
                __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, (int)(rows * ld * 4), 0x00020000);
            const unsigned vo = (k & 1) ? vox : voy;
            const int step = (k & 1) ? xstep : ystep;
#pragma unroll
            for (int f = 0; f < 2; ++f)
                R[k][f] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, vo, u * step + 16 * f, 0));
            if (HEAD && (k & 1)) {  // (the descriptor ends at the last row's column lddy - 1: rows past it read 0)
                const long long nb = rows * lddy * 4 - DGW_W * 4;
                const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
                    (void*)(dyp + r0 * lddy + DGW_W), 0, (int)(nb > 0 ? nb : 0), 0x00020000);
                Ga[u] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ra, voa, u * ystep, 0));
            }
        };
        // db: the thread's running column sums of its staging rows, in LDS (its own 32 B of [8][256])
        float* const bsum = reinterpret_cast<float*>(lds8 + 2 * DGW_STAGE) + sr * DGW_W + c8;
        *reinterpret_cast<f32x4*>(bsum) = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
        *reinterpret_cast<f32x4*>(bsum + 4) = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
        auto stage_unit = [&](int buf, int k) {
            unsigned char* const S = lds8 + buf * DGW_STAGE;
            const int r = sr + 8 * (k >> 1);
            const int off = dgw_off(r, c8 >> 3);
            float v[8];
#pragma unroll
            for (int f = 0; f < 2; ++f)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    // (through float rvalues: clang's bit_cast of a vector-element lvalue reads element 0)
                    const float t = R[k][f][e];
                    v[4 * f + e] = t;
                }
            if (k & 1) {
                if (HEAD) {
                    const float ga = Ga[k >> 1];
#pragma unroll
                    for (int e = 0; e < 8; ++e) xa[e] = fmaf(ga, v[e], xa[e]);
                    if ((tid & 31) == 0) {
                        reinterpret_cast<float*>(S + DGW_GA)[r] = ga;
                        dba += ga;
                    }
                }
                dgw_split_store(v, S + 2 * DGW_PLANE, S + 3 * DGW_PLANE, off);
                unsigned mk[2] = {0u, 0u};
#pragma unroll
                for (int e = 0; e < 8; ++e)
                    if (v[e] > 0.0f) mk[e >> 2] |= 1u << (8 * (e & 3));
                typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
                *reinterpret_cast<u32x2*>(S + 4 * DGW_PLANE + r * DGW_W + c8) = u32x2{mk[0], mk[1]};
            } else {
                f32x4 b0 = *reinterpret_cast<const f32x4*>(bsum), b1 = *reinterpret_cast<const f32x4*>(bsum + 4);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    b0[e] += v[e];
                    b1[e] += v[4 + e];
                }
                *reinterpret_cast<f32x4*>(bsum) = b0;
                *reinterpret_cast<f32x4*>(bsum + 4) = b1;
                dgw_split_store(v, S, S + DGW_PLANE, off);
            }
        };
        if (nch > 0) {
#pragma unroll
            for (int k = 0; k < 8; ++k) fetch_unit(0, k);
#pragma unroll
            for (int k = 0; k < 8; ++k) stage_unit(0, k);
        }
        if (nch > 1) {
#pragma unroll
            for (int k = 0; k < 8; ++k) fetch_unit(1, k);
        }
        __syncthreads();
        for (int s = 0; s < nch; ++s) {
            const unsigned char* const S = lds8 + (s & 1) * DGW_STAGE;
            bf16x8 ad[2];
#pragma unroll
            for (int t = 0; t < 16; ++t) {
                __builtin_amdgcn_sched_barrier(0);
                pin_lane();
                // unit t / 2 of the next chunk into the other stage (free since the barrier that ended chunk s - 1),
                // then its loads for the chunk after: a whole chunk of compute to land
                if (ANERF_DGW_PROBE != 4 && (t & 1) == 0) {
                    if (s + 1 < nch) stage_unit((s + 1) & 1, t >> 1);
                    if (s + 2 < nch) fetch_unit(s + 2, t >> 1);
                }
                dw_slot(S, t, ad);
            }
            __syncthreads();
        }
        if (HEAD) {  // (every stage read is done: the last barrier above) the thread's alpha sums into stage 0
            float* const sc = reinterpret_cast<float*>(lds8);
#pragma unroll
            for (int e = 0; e < 8; ++e) sc[sr * DGW_W + c8 + e] = xa[e];
            if ((tid & 31) == 0) sc[8 * DGW_W + sr] = dba;
        }
    } else {
        // ------------------------------------------------------------------ dX waves
        const int xw = wave - 4;  // dX columns 64 xw .. 64 xw + 63: blocks 2 xw, 2 xw + 1
        const long long lddx = g.lddx;
        // the split W^T (fragment-major: 32-column block nb, k16 step ks, plane p = 1 KB in lane order) of the
        // wave's two blocks (a buffer descriptor: the lane's 16 B in the lane offset, the step in the uniform one)
        constexpr int WBS = (DGW_W / 16) * 2 * 512;  // elements per 32-column block
        const __amdgpu_buffer_rsrc_t rwt =
            __builtin_amdgcn_make_buffer_rsrc((void*)(g.wt + (long long)(2 * xw) * WBS), 0, 2 * WBS * 2, 0x00020000);
        const unsigned vwl = (unsigned)lane * 16;
        struct WF {
            u32x4 v[2][2];  // [block][plane]
        };
        // (the fragments of k16 step kt are the same for every chunk: the ring runs on across the chunks, so the
        // first steps of chunk s + 1 are in flight before chunk s's dX stores, which count in vmcnt with them)
        auto fetch_w = [&](int kt, WF& f) {
            kt &= DGW_W / 16 - 1;
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int p = 0; p < 2; ++p) {
#if ANERF_DGW_PROBE == 3
                    f.v[j][p] = u32x4{vwl, vwl, vwl, (unsigned)kt};
#else
                    f.v[j][p] = __builtin_bit_cast(
                        u32x4, __builtin_amdgcn_raw_buffer_load_b128(rwt, vwl, j * WBS * 2 + (kt * 2 + p) * 1024, 0));
#endif
                }
        };
        WF wf[DGW_BD];
#pragma unroll
        for (int j = 0; j < DGW_BD - 1; ++j) fetch_w(j, wf[j]);
        float wa[2] = {0.0f, 0.0f};  // (HEAD) w_a at the lane's two dX columns
        if (HEAD) {
#pragma unroll
            for (int j = 0; j < 2; ++j) wa[j] = g.wa[64 * xw + 32 * j + (lane & 31)];
        }
        __syncthreads();
        for (int s = 0; s < nch; ++s) {
            const unsigned char* const S = lds8 + (s & 1) * DGW_STAGE;
            f32x16 ax[2] = {f32x16{0}, f32x16{0}};
            bf16x8 ad[2];
#pragma unroll
            for (int t = 0; t < 16; ++t) {
                __builtin_amdgcn_sched_barrier(0);
                pin_lane();
                fetch_w(t + DGW_BD - 1, wf[(t + DGW_BD - 1) % DGW_BD]);
                const bf16x8 ay0 = rfrag(S, t), ay1 = rfrag(S + DGW_PLANE, t);
                const WF& f = wf[t % DGW_BD];
                if (ANERF_DGW_PROBE != 1) {
#pragma unroll
                    for (int j = 0; j < 2; ++j) {  // small terms first
                        const bf16x8 b0 = __builtin_bit_cast(bf16x8, f.v[j][0]), b1 = __builtin_bit_cast(bf16x8, f.v[j][1]);
                        f32x16 c = mfma(ay1, b0, ax[j]);
                        c = mfma(ay0, b1, c);
                        ax[j] = mfma(ay0, b0, c);
                    }
                }
                dw_slot(S, t, ad);
            }
            // dX epilogue: relu' mask bytes from LDS, buffer stores straight from the accumulator layout (a wave
            // instruction writes two whole 128 B row pieces; the descriptor ends at the chunk's last row, so the
            // rows past the workgroup's range are dropped without a branch, and the row offsets ride in SGPRs)
            const long long r0 = mlo + (long long)s * DGW_CH;
            long long rows = mhi - r0;
            rows = rows > DGW_CH ? DGW_CH : rows;
            const __amdgpu_buffer_rsrc_t rd =
                __builtin_amdgcn_make_buffer_rsrc((void*)(g.dx + r0 * lddx), 0, (int)(rows * lddx * 4), 0x00020000);
            const unsigned char* const mk = S + 4 * DGW_PLANE;
            const float* const gal = reinterpret_cast<const float*>(S + DGW_GA);
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int col = 64 * xw + 32 * j + (lane & 31);
                const unsigned vo = (unsigned)((4 * (lane >> 5) * lddx + col) * 4);
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int rr = (r & 3) + 8 * (r >> 2);
                    const float a = HEAD ? fmaf(gal[rr + 4 * (lane >> 5)], wa[j], ax[j][r]) : ax[j][r];
                    const float v = mk[(rr + 4 * (lane >> 5)) * DGW_W + col] ? a : 0.0f;
                    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), rd, vo, (int)(rr * lddx * 4),
                                                          0);
                }
            }
            __syncthreads();
        }
    }
    // the dW partial: [256][256] floats of this workgroup, straight from the accumulators (buffer stores, the
    // per-register row and block offsets in SGPRs)
    {
        const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(g.ws + (long long)blockIdx.x * SROWS * DGW_W), 0, DGW_W * DGW_W * 4, 0x00020000);
        const unsigned vo = (unsigned)(((32 * wave + 4 * (lane >> 5)) * DGW_W + (lane & 31)) * 4);
#pragma unroll
        for (int ib = 0; ib < 8; ++ib)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int rr = (r & 3) + 8 * (r >> 2);
                const float v = aw[ib][r];
                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), rw, vo,
                                                      (rr * DGW_W + 32 * ib) * 4, 0);
            }
    }
    // db partial: the 8 staging rows' column sums, added in a fixed order
    const float* const red = reinterpret_cast<const float*>(lds8 + 2 * DGW_STAGE);  // [8][256]
    __syncthreads();
    if (tid < DGW_W) {
        float t = red[tid];
#pragma unroll
        for (int w = 1; w < 8; ++w) t += red[w * DGW_W + tid];
        g.wsb[(long long)blockIdx.x * BST + tid] = t;
        if (HEAD) {  // alpha's dW row and db entry, the 8 staging rows' sums in a fixed order
            const float* const sc = reinterpret_cast<const float*>(lds8);
            float a = sc[tid];
#pragma unroll
            for (int w = 1; w < 8; ++w) a += sc[w * DGW_W + tid];
            g.ws[(long long)blockIdx.x * SROWS * DGW_W + DGW_W * DGW_W + tid] = a;
            if (tid < 4) {
                float d = 0.0f;
                if (tid == 0) {
                    d = sc[8 * DGW_W];
#pragma unroll
                    for (int w = 1; w < 8; ++w) d += sc[8 * DGW_W + w];
                }
                g.wsb[(long long)blockIdx.x * BST + DGW_W + tid] = d;  // (entries 257-259: zero padding)
            }
        }
    }
}

// rows per workgroup: one persistent workgroup per CU over whole 32-row chunks
int dgw_plan(int64_t m, long long* rows_per_wg) {
    static int cus = 0;
    if (!cus) {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) ==
                                                    hipSuccess && n > 0)
            cus = n;
        else
            cus = 256;
    }
    long long chunks = (m + DGW_CH - 1) / DGW_CH;
    if (chunks < 1) chunks = 1;
    const long long per = (chunks + cus - 1) / cus;  // chunks per workgroup
    *rows_per_wg = per * DGW_CH;
    return (int)((chunks + per - 1) / per);
}

// ---------------------------------------------------------------- layer forward, persistent (round 6)
// y = act(x W^T + b) of one layer with 256 outputs -- the hidden layers (pts_linears[i], core/networks/nerf.py:133-139),
// layer 0 and the skip layer on [x | h] (the concatenation as two operand segments, never built) and feature_linear
// (no activation) with alpha_linear beside it (:141-145) -- with the arithmetic of mlp_nt_kernel<NPL, *> (x and W split
// into NPL bf16 planes, the same products in the same order per k16 step, k16 steps ascending from a zero
// accumulator, + bias, relu): the 256 outputs are bit-identical to anerf_mlp_gemm's.  What changes is the schedule.
// mlp_nt_kernel runs 128 x 128 tiles, two per CU, each staging its A rows, looping its k steps and storing through
// its epilogue in turn: in the training step a 256 x 256 layer ran at 2.3-2.5 TB/s of its 336 MB (M = 163,840) with
// every byte moved once, i.e. bound by the tiles' serial prologue / k-loop / epilogue latency, not by bandwidth.
// Here one persistent workgroup per CU walks a contiguous row range in 64-row chunks, each as ceil(K / 128) units of
// 128 k columns, with the work split by role (as mlp_dgw_kernel):
//   * stager waves (0-3): load a unit's x rows from HBM two units ahead, split them into the LDS planes of the other
//     stage, and copy the previous chunk's output tile from LDS to HBM in whole-row 16 B stores (head: also
//     alpha = x . w_alpha + b_alpha in fp32 from the rows they stage, written to its own column);
//   * compute waves (4-7): output columns 64 (w - 4) .. + 63 of every chunk (2 x 2 blocks of 32 x 32), the split W
//     fragments from L2 in a 4-deep ring that runs on across units and chunks, the A fragments from LDS a k16 step
//     ahead; after a chunk's last unit, bias (+ relu) into the LDS output tile.
// So the compute waves issue no HBM access at all (their in-order vmcnt holds only L2 weight loads) and the HBM
// reads, the splits and the stores overlap the MFMAs of the current unit.
// LDS: two stages of NPL planes [64][128] bf16 (256 B rows, the 16 B chunks XOR-swizzled by row & 15: the staging
// writes, 16 lanes x one row, and the fragment reads, 16 rows x one chunk, are conflict-free) + the fp32 output
// tile [64][256] (64 KB): 160 KB at bf16x6, 128 KB at bf16x3.
constexpr int FW_W = 256;     // outputs
constexpr int FW_CH = 64;     // rows per chunk
constexpr int FW_KH = 128;    // k columns per unit
constexpr int FW_THR = 512;   // eight waves
constexpr int FW_BD = 4;      // W fragment ring depth (k16 steps; divides a unit's 8)
// (ANERF_FW_PROBE, timing diagnostics of experiment builds only, wrong results: 1 no MFMAs, 2 no W loads after the
// ring's first, 3 no x loads after the first units, 4 no output stores, 5 = 3 + 4, 6 = 2 + 3 + 4, 7 = 6 + no staging
// after the first units, 8 = 6 + no A fragment reads after the first units, 9 = 6 + no epilogue, 10 = 6 + no barriers
// in the unit loop)
#ifndef ANERF_FW_PROBE
#define ANERF_FW_PROBE 0
#endif
// (experiment switch) 1: the compute waves store their outputs straight from the accumulators (no LDS tile, the
// storer waves idle)
#ifndef ANERF_FW_MAP
#define ANERF_FW_MAP 0
#endif
// (experiment switch) 1: the MFMAs of a k16 step interleaved over the four accumulators
#ifndef ANERF_FW_IL
#define ANERF_FW_IL 0
#endif
// (experiment switch) s_setprio of the compute waves (0: none)
#ifndef ANERF_FW_PRIO
#define ANERF_FW_PRIO 0
#endif
#ifndef ANERF_FW_DIRECT
#define ANERF_FW_DIRECT 0
#endif
template <int NPL>
struct FWGeo {
    static constexpr int PLANE = FW_CH * FW_KH * 2;  // 16 KB
    static constexpr int STAGE = NPL * PLANE;
    static constexpr int OUT = FW_CH * FW_W * 4;     // 64 KB
    static constexpr int LDS = 2 * STAGE + OUT;
};

struct FWArgs {
    long long M, rows_per_wg;
    const float* x0;  // operand segments: columns [0, c0) of x0 rows, then [c0, K) of x1 rows (or none)
    const float* x1;
    long long ld0, ld1;
    int c0, K, nk, nu;        // k16 steps of W (ceil(K / 16)), units per chunk (ceil(K / 128) >= 2)
    const unsigned short* w;  // split W, NPL bf16 planes (anerf_mlp_split_weights, transpose = 0)
    const float* bias;  // or null
    int relu;
    int nval;  // output columns of this launch's 256-column tile that exist (% 4 == 0)
    float* y;
    long long ldy;
    const float* wa;  // head: alpha_linear's weight [K] and bias [1], alpha out (column 0 of rows with ld lda), or null
    const float* ba;
    float* alpha;
    long long lda;
};

__device__ __forceinline__ int fw_off(int row, int chunk) { return row * 256 + ((chunk ^ (row & 15)) << 4); }

template <int NPL, int NSEG, bool HEAD>
__global__ __launch_bounds__(FW_THR, 1) void mlp_fwd_kernel(FWArgs g) {
    using G = FWGeo<NPL>;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds8[];
    float* const otile = reinterpret_cast<float*>(lds8 + 2 * G::STAGE);  // [64][256]
    // (ANERF_FW_MAP 1, experiment: the roles on the odd (compute) and even hardware waves instead of 4-7 / 0-3)
    const int hw = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const int wave = ANERF_FW_MAP ? ((hw & 1) ? 4 + (hw >> 1) : (hw >> 1)) : hw;
    const int lane = (int)threadIdx.x & 63, tid = wave * 64 + lane;
    const long long M = g.M;
    const long long mlo = (long long)blockIdx.x * g.rows_per_wg;
    const long long mhi = mlo + g.rows_per_wg < M ? mlo + g.rows_per_wg : M;
    const int nch = mhi > mlo ? (int)((mhi - mlo + FW_CH - 1) / FW_CH) : 0;
    const int nu = g.nu;
    const int nun = nu * nch;  // units
    // (kernel-argument fields as locals: a lambda referencing `g` makes clang copy the whole argument struct to
    // scratch and reload the fields from there)
    const float* const x0p = g.x0;
    const float* const x1p = g.x1;
    float* const yp = g.y;
    const float* const wap = g.wa;
    float* const alp = g.alpha;
    const long long lda = g.lda;
    auto chunk_rows = [&](int s) {  // (0 past the last chunk)
        long long rows = mhi - (mlo + (long long)s * FW_CH);
        return (int)(rows < 0 ? 0 : (rows > FW_CH ? FW_CH : rows));
    };

    if (wave < 2) {
        // ------------------------------------------------------------------ loader waves
        // thread t < 128: columns c8 .. c8 + 7 of the unit (two float4 loads) in rows r8 + 8 p (p < 8).  Their vmcnt
        // holds only these loads, issued unconditionally (past the last unit through a zero-range descriptor, which
        // reads 0 and moves nothing), so every wait the compiler places is exact: a unit's loads land while two units
        // of MFMAs run
        const int c8 = 8 * (tid & 15), r8 = tid >> 4;
        const long long ld0 = g.ld0, ld1 = g.ld1;
        const int c0 = g.c0, K = g.K;
        const unsigned vo0 = (unsigned)(r8 * ld0 * 4), vo1 = (unsigned)(r8 * ld1 * 4);
        const unsigned st0 = (unsigned)(8 * ld0 * 4), st1 = (unsigned)(8 * ld1 * 4);
        // two register sets (unit v in set v & 1, loaded two units before it is staged); one with two segments (the
        // second segment's loads need their own registers until merged: one unit ahead)
        constexpr int NS = NSEG == 2 ? 1 : 2;
        f32x4 RR[NS][8][2];
        auto fetch = [&](int u, f32x4 (&R)[8][2]) __attribute__((always_inline)) {
            if ((ANERF_FW_PROBE == 3 || ANERF_FW_PROBE >= 5) && u >= 2) return;
            const int s = u / nu, kh = u - s * nu;
            const long long r0 = mlo + (long long)s * FW_CH;
            const int rows = chunk_rows(s);
            const __amdgpu_buffer_rsrc_t rs0 =
                __builtin_amdgcn_make_buffer_rsrc((void*)(x0p + r0 * ld0), 0, (int)(rows * ld0 * 4), 0x00020000);
            // (columns outside a segment read zero through an offset past its range; a float4 never straddles
            // segments: c0 % 4 == 0.  Row steps ride in the lane offset, which the range check covers, so the rows
            // past the chunk read zero)
            unsigned o0[2], o1[2];
#pragma unroll
            for (int f = 0; f < 2; ++f) {
                const int c = FW_KH * kh + c8 + 4 * f;
                o0[f] = c < c0 ? vo0 + (unsigned)c * 4u : NOOB;
                o1[f] = c >= c0 && c < K ? vo1 + (unsigned)(c - c0) * 4u : NOOB;
            }
#pragma unroll
            for (int p = 0; p < 8; ++p)
#pragma unroll
                for (int f = 0; f < 2; ++f)
                    R[p][f] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs0, o0[f] + p * st0, 0, 0));
            if constexpr (NSEG == 2) {
                const __amdgpu_buffer_rsrc_t rs1 =
                    __builtin_amdgcn_make_buffer_rsrc((void*)(x1p + r0 * ld1), 0, (int)(rows * ld1 * 4), 0x00020000);
#pragma unroll
                for (int p = 0; p < 8; ++p)
#pragma unroll
                    for (int f = 0; f < 2; ++f) {
                        const f32x4 v = __builtin_bit_cast(
                            f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs1, o1[f] + p * st1, 0, 0));
#pragma unroll
                        for (int e = 0; e < 4; ++e) {  // (one segment is live per lane, the other reads 0)
                            const float a = R[p][f][e], b = v[e];
                            R[p][f][e] = __builtin_bit_cast(float, __builtin_bit_cast(unsigned, a) |
                                                                       __builtin_bit_cast(unsigned, b));
                        }
                    }
            }
        };
        // HEAD (k = 256: two units): alpha_linear's weights at the thread's columns of either unit, loaded once; the
        // partial sums of its eight rows over the chunk's units
        float wa0[8], wa1[8], asum[8];
        float ba = 0.0f;
        if constexpr (HEAD) {
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                wa0[e] = wap[c8 + e];
                wa1[e] = wap[FW_KH + c8 + e];
                asum[e] = 0.0f;
            }
            ba = g.ba[0];
        }
        auto stage = [&](int u, int buf, const f32x4 (&R)[8][2]) __attribute__((always_inline)) {
            if (ANERF_FW_PROBE == 7 && u >= 2) return;
            unsigned char* const S = lds8 + buf * G::STAGE;
            const int s = u / nu, kh = u - s * nu;
#pragma unroll
            for (int p = 0; p < 8; ++p) {
                float v[8];
#pragma unroll
                for (int f = 0; f < 2; ++f)
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        // (through float rvalues: clang's bit_cast of a vector-element lvalue reads element 0)
                        const float t = R[p][f][e];
                        v[4 * f + e] = t;
                    }
                if constexpr (HEAD) {
                    float a = kh ? asum[p] : 0.0f;
#pragma unroll
                    for (int e = 0; e < 8; ++e) a = fmaf(kh ? wa1[e] : wa0[e], v[e], a);
                    asum[p] = a;
                }
                const int off = fw_off(r8 + 8 * p, c8 >> 3);
                // (mlp_nt_kernel's split: round to nearest even, the exact remainder split again)
#pragma unroll
                for (int pl = 0; pl < NPL; ++pl) {
                    u32x4 w;
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const bf16x2 h = __builtin_convertvector((f32x2){v[2 * q], v[2 * q + 1]}, bf16x2);
                        w[q] = __builtin_bit_cast(unsigned, h);
                        if (pl + 1 < NPL) {
                            v[2 * q] -= (float)h[0];
                            v[2 * q + 1] -= (float)h[1];
                        }
                    }
                    *reinterpret_cast<u32x4*>(S + pl * G::PLANE + off) = w;
                }
            }
            if constexpr (HEAD) {
                if (kh == nu - 1) {  // the chunk's alpha: the 16 lanes of a row, then one store per row
                    const long long r0 = mlo + (long long)s * FW_CH;
                    const int rows = chunk_rows(s);
#pragma unroll
                    for (int p = 0; p < 8; ++p) {
                        float a = asum[p];
                        a += __shfl_xor(a, 8, 16);
                        a += __shfl_xor(a, 4, 16);
                        a += __shfl_xor(a, 2, 16);
                        a += __shfl_xor(a, 1, 16);
                        const int row = r8 + 8 * p;
                        if ((tid & 15) == 0 && row < rows) alp[(r0 + row) * lda] = a + ba;
                    }
                }
            }
        };
        fetch(0, RR[0]);
        if constexpr (NS == 2) fetch(1, RR[NS - 1]);
        if (nun > 0) stage(0, 0, RR[0]);
        fetch(NS, RR[0]);
        __syncthreads();
        // unit u (parity P = u & 1, static): stage unit u + 1 from its set into the other LDS stage (free since the
        // barrier that ended unit u - 1), then load unit u + 1 + NS into that set
        auto body = [&](int u, auto P) __attribute__((always_inline)) {
            constexpr int Q = 1 - decltype(P)::value;
            constexpr int SET = NS == 2 ? Q : 0;
            if (u + 1 < nun) stage(u + 1, Q, RR[SET]);
            fetch(u + 1 + NS, RR[SET]);
            if (ANERF_FW_PROBE != 10) __syncthreads();
        };
        for (int u = 0; u < nun; u += 2) {
            body(u, std::integral_constant<int, 0>{});
            if (u + 1 < nun) body(u + 1, std::integral_constant<int, 1>{});
        }
    } else if (wave < 4) {
        // ------------------------------------------------------------------ storer waves
        // the output tile of chunk s (written by the compute waves before the barrier ending its last unit) during
        // the next chunk's first unit (nu >= 2: before they write it again): thread t < 128 of the role, rows 2 q +
        // (t >> 6), columns 4 (t & 63) .. + 3 (a wave instruction stores one whole 1 KB row).  Stores only, never
        // waited on
        const int t = tid - 128;
        const long long ldy = g.ldy;
        const int nval = g.nval;
        auto copy_out = [&](int s) __attribute__((always_inline)) {
            if (ANERF_FW_PROBE == 4 || ANERF_FW_PROBE >= 5 || ANERF_FW_DIRECT) return;
            const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(
                (void*)(yp + (mlo + (long long)s * FW_CH) * ldy), 0, (int)(chunk_rows(s) * ldy * 4), 0x00020000);
            const int c4 = 4 * (t & 63), rq = t >> 6;
            const unsigned vo = c4 < nval ? (unsigned)((rq * ldy + c4) * 4) : NOOB;  // (columns past the tile's n)
#pragma unroll
            for (int q = 0; q < FW_CH / 2; ++q) {
                const f32x4 v = *reinterpret_cast<const f32x4*>(otile + (2 * q + rq) * FW_W + c4);
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rd, vo + (unsigned)(2 * q * ldy * 4),
                                                       0, 0);
            }
        };
        __syncthreads();
        for (int u = 0; u < nun; ++u) {
            if (u >= nu && u % nu == 0) copy_out(u / nu - 1);
            if (ANERF_FW_PROBE != 10) __syncthreads();
        }
        if (nch > 0) copy_out(nch - 1);
    } else {
        // ------------------------------------------------------------------ compute waves
        const int xw = wave - 4;  // output columns 64 xw .. 64 xw + 63: blocks 2 xw, 2 xw + 1
#if ANERF_FW_PRIO
        // (experiment) the compute waves' instruction issue ahead of the loader / storer waves' on the same SIMD
        __builtin_amdgcn_s_setprio(ANERF_FW_PRIO);
#endif
        const unsigned short* const wp = g.w;
#if ANERF_FW_DIRECT
        float* const ypc = yp;
        const long long ldyc = g.ldy;
#endif
        const int nk = g.nk, ku = 8 * nu;   // W's k16 steps; k16 steps of a chunk's units
        const int WBS = ((g.K + 15) / 16) * NPL * 512;  // elements per 32-column block of the split W
        const __amdgpu_buffer_rsrc_t rw =
            __builtin_amdgcn_make_buffer_rsrc((void*)(wp + (long long)(2 * xw) * WBS), 0, 2 * WBS * 2, 0x00020000);
        const unsigned vwl = (unsigned)lane * 16;
        struct WF {
            u32x4 v[2][NPL];  // [block][plane]
        };
        // global k16 index q = 8 u + t: the chunk's step q % ku; steps past W's (the last unit's padding, whose
        // A columns are zero) are neither loaded nor multiplied
        auto fetch_w = [&](int q, WF& f) {
            if ((ANERF_FW_PROBE == 2 || ANERF_FW_PROBE >= 6) && q >= FW_BD) return;
            int kt = q % ku;
            kt = kt < nk ? kt : nk - 1;  // (a straight-line instruction stream: the padding steps reload the last)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int p = 0; p < NPL; ++p)
                    f.v[j][p] = __builtin_bit_cast(
                        u32x4, __builtin_amdgcn_raw_buffer_load_b128(rw, vwl, (j * WBS + (kt * NPL + p) * 512) * 2, 0));
        };
        const float* const bp = g.bias;
        const int n0c = 64 * xw + (lane & 31);
        const float b0 = bp && n0c < g.nval ? bp[n0c] : 0.0f, b1 = bp && n0c + 32 < g.nval ? bp[n0c + 32] : 0.0f;
        const bool relu = g.relu != 0;
        WF wf[FW_BD];
#pragma unroll
        for (int j = 0; j < FW_BD - 1; ++j) fetch_w(j, wf[j]);
        f32x16 acc[2][2];
        __syncthreads();
        for (int u = 0; u < nun; ++u) {
            const unsigned char* const S = lds8 + (u & 1) * G::STAGE;
            const int kh = u % nu;
            if (!kh) {
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{0};
            }
            // A fragments of k16 step t (rows 32 i + (lane & 31), k chunk 2 t + (lane >> 5)), read a step ahead
            bf16x8 A[2][NPL][2];
            auto read_a = [&](int t, bf16x8 (&a)[NPL][2]) {
#pragma unroll
                for (int p = 0; p < NPL; ++p)
#pragma unroll
                    for (int i = 0; i < 2; ++i)
                        a[p][i] = *reinterpret_cast<const bf16x8*>(S + p * G::PLANE +
                                                                   fw_off(32 * i + (lane & 31), 2 * t + (lane >> 5)));
            };
            read_a(0, A[0]);
#pragma unroll
            for (int t = 0; t < FW_KH / 16; ++t) {
                __builtin_amdgcn_sched_barrier(0);
                fetch_w(8 * u + t + FW_BD - 1, wf[(t + FW_BD - 1) % FW_BD]);  // ((8 u + t) % FW_BD = t % FW_BD)
                if (t + 1 < FW_KH / 16 && (ANERF_FW_PROBE != 8 || u < 2)) read_a(t + 1, A[(t + 1) & 1]);
                __builtin_amdgcn_sched_barrier(0);
                if (8 * kh + t >= nk || ANERF_FW_PROBE == 1) continue;
                const bf16x8 (&a)[NPL][2] = A[t & 1];
                const WF& f = wf[t % FW_BD];
#if ANERF_FW_IL
                // (experiment) the four accumulators' chains interleaved product by product (each accumulator's own
                // product order unchanged: the same bits)
                constexpr int NPR = NPL == 3 ? 6 : 3;
                constexpr int PA[6] = {NPL == 3 ? 2 : 1, 1, 0, 1, 0, 0}, PB[6] = {0, 1, 2, 0, 1, 0};
                constexpr int O = NPL == 3 ? 0 : 3;
#pragma unroll
                for (int q = 0; q < NPR; ++q)
#pragma unroll
                    for (int j = 0; j < 2; ++j)
#pragma unroll
                        for (int i = 0; i < 2; ++i)
                            acc[i][j] = mfma(a[PA[O + q]][i], __builtin_bit_cast(bf16x8, f.v[j][PB[O + q]]), acc[i][j]);
#else
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    bf16x8 b[NPL];
#pragma unroll
                    for (int p = 0; p < NPL; ++p) b[p] = __builtin_bit_cast(bf16x8, f.v[j][p]);
#pragma unroll
                    for (int i = 0; i < 2; ++i) {  // (mlp_nt_kernel's product order: small terms first)
                        f32x16 c = acc[i][j];
                        if constexpr (NPL == 3) {
                            c = mfma(a[2][i], b[0], c);
                            c = mfma(a[1][i], b[1], c);
                            c = mfma(a[0][i], b[2], c);
                        }
                        c = mfma(a[1][i], b[0], c);
                        c = mfma(a[0][i], b[1], c);
                        acc[i][j] = mfma(a[0][i], b[0], c);
                    }
                }
#endif
            }
            if (kh == nu - 1) {  // the chunk's output: + bias (, relu), into the tile (its previous copy left before
                                 // the barrier that ended unit u - 1)
#if ANERF_FW_DIRECT
                // (experiment) straight from the accumulators to HBM: a wave instruction writes two 128 B row pieces;
                // the descriptor ends at the chunk's last row
                const int s = u / nu;
                const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(
                    (void*)(ypc + (mlo + (long long)s * FW_CH) * ldyc), 0, (int)(chunk_rows(s) * ldyc * 4), 0x00020000);
#endif
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j)
#pragma unroll
                        for (int r = 0; r < 16; ++r) {
                            if (ANERF_FW_PROBE == 9) continue;
                            const int row = 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                            float v = acc[i][j][r];
                            v += j ? b1 : b0;
                            if (relu) v = fmaxf(v, 0.0f);
#if ANERF_FW_DIRECT
                            __builtin_amdgcn_raw_buffer_store_b32(
                                __builtin_bit_cast(unsigned, v), rd,
                                (unsigned)((row * ldyc + 64 * xw + 32 * j + (lane & 31)) * 4), 0, 0);
#else
                            otile[row * FW_W + 64 * xw + 32 * j + (lane & 31)] = v;
#endif
                        }
            }
            if (ANERF_FW_PROBE != 10) __syncthreads();
        }
    }
}

// rows per workgroup: one persistent workgroup per CU over whole 64-row chunks
int fw_plan(int64_t m, long long* rows_per_wg) {
    static int cus = 0;
    if (!cus) {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) ==
                                                    hipSuccess && n > 0)
            cus = n;
        else
            cus = 256;
    }
    long long chunks = (m + FW_CH - 1) / FW_CH;
    if (chunks < 1) chunks = 1;
    const long long per = (chunks + cus - 1) / cus;
    *rows_per_wg = per * FW_CH;
    return (int)((chunks + per - 1) / per);
}

inline int rup(long long x, int a) { return (int)((x + a - 1) / a * a); }

int planes_of(int precision) {
    return precision == ANERF_MLP_BF16X6 ? 3 : ((precision == ANERF_MLP_BF16X3 || precision == ANERF_MLP_FP16X4) ? 2 : 0);
}
// the fp16x4 exponent sits after the planes (anerf_mlp_split_bytes adds 256 bytes for it)
size_t split_plane_bytes(int rows, int cols, int npl) { return (size_t)2 * npl * rup(rows, BNW) * rup(cols, 16); }

// the dynamic LDS (up to 67 KB) is above the default limit: raised once per kernel instance
// (set on every call: the attribute belongs to the current device, and a cached failure would stick)
template <int NPL, int NSEG, int TBM, int SKT, bool F16 = false, int CB = 1>
hipError_t nt_attr() {
    return hipFuncSetAttribute((const void*)mlp_nt_kernel<NPL, NSEG, TBM, SKT, F16, CB>,
                               hipFuncAttributeMaxDynamicSharedMemorySize, NTGeo<NPL, TBM, SKT>::LDS_BYTES);
}
template <int NPL, int NSEG>
hipError_t tn_attr() {
    return hipFuncSetAttribute((const void*)mlp_tn_kernel<NPL, NSEG>, hipFuncAttributeMaxDynamicSharedMemorySize,
                               TNGeo<NPL, NSEG>::LDS_BYTES);
}

// Operand segments: every segment but the last a multiple of 4 columns, all 16-byte aligned with
// ld % 4 == 0 (4-column groups never straddle segments; float4 loads); the last segment's row is
// read up to round_up(cols, 4) columns (ld >= that; those columns must be finite).
int set_segs(const anerf_seg* in, int n, int total, SegD* out) {
    if (n < 1 || n > MAXSEG || !in) return anerf_internal_fail(ANERF_EINVAL, "1 to 3 operand segments");
    int start = 0;
    for (int i = 0; i < n; ++i) {
        const bool last = i + 1 == n;
        if (!in[i].p || in[i].cols < 1 || in[i].ld < (last ? (in[i].cols + 3) / 4 * 4 : in[i].cols))
            return anerf_internal_fail(ANERF_EINVAL, "bad operand segment (ld < cols, rounded to 4 for the last)");
        if (in[i].ld % 4 || (uintptr_t)in[i].p % 16 || (!last && in[i].cols % 4))
            return anerf_internal_fail(ANERF_EINVAL, "operand segments need 16-byte aligned rows and, but for the "
                                                     "last, a multiple of 4 columns");
        out[i].p = in[i].p;
        out[i].ld = in[i].ld;
        out[i].start = start;
        out[i].cols = in[i].cols;
        out[i].vec = 1;
        start += in[i].cols;
    }
    if (start != total) return anerf_internal_fail(ANERF_EINVAL, "operand segments do not add up to k");
    return ANERF_OK;
}

// weight-gradient workgroups per launch (experiment switch): ~512 = two per CU; fewer slabs write and re-read fewer
// partial tiles
#ifndef ANERF_WGRAD_WG
#define ANERF_WGRAD_WG 512
#endif
int wgrad_plan(int64_t m, int32_t n, int32_t k, int* splits, long long* rows) {
    const int tiles = ((n + BN - 1) / BN) * ((k + BM - 1) / BM);
    long long s = (ANERF_WGRAD_WG + tiles - 1) / tiles;  // ~ANERF_WGRAD_WG workgroups
    const long long smax = (m + 255) / 256;         // >= 256 rows per slab
    if (s > smax) s = smax;
    if (s < 1) s = 1;
    long long r = (m + s - 1) / s;
    r = (r + 2 * TSK - 1) / (2 * TSK) * (2 * TSK);
    *rows = r;
    *splits = (int)((m + r - 1) / r);
    if (*splits < 1) *splits = 1;
    return tiles;
}

}  // namespace

extern "C" {

size_t anerf_mlp_split_bytes(int32_t rows, int32_t cols, int32_t precision) {
    return split_plane_bytes(rows, cols, planes_of(precision)) + (precision == ANERF_MLP_FP16X4 ? 256 : 0);
}

int anerf_mlp_split_weights(const float* w, int32_t n, int32_t k, int64_t ldw, int32_t transpose, int32_t precision,
                            void* out, void* stream) {
    const int npl = planes_of(precision);
    if (!w || !out || n < 1 || k < 1 || ldw < k || !npl)
        return anerf_internal_fail(ANERF_EINVAL, "anerf_mlp_split_weights: bad arguments");
    if (precision == ANERF_MLP_FP16X4) {  // (the exponent pass: through the batch path)
        anerf_split_job j = {w, n, k, ldw, transpose, precision, out};
        return anerf_mlp_split_weights_batch(&j, 1, stream);
    }
    const int rows = transpose ? k : n, cols = transpose ? n : k;
    const int nblocks = (rows + BNW - 1) / BNW * (BNW / 32), ksteps = (cols + 15) / 16;  // whole 256-row tiles
    const long long tot = (long long)nblocks * ksteps * 512;
    hipLaunchKernelGGL(split_weights_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), w, n, k, (long long)ldw, transpose, nblocks, ksteps, npl,
                       static_cast<unsigned short*>(out));
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? ANERF_OK : anerf_internal_fail(ANERF_EHIP, hipGetErrorString(e));
}

int anerf_mlp_split_weights_batch(const anerf_split_job* jobs, int32_t n_jobs, void* stream) {
    if (!jobs || n_jobs < 1 || n_jobs > MAXJOBS)
        return anerf_internal_fail(ANERF_EINVAL, "anerf_mlp_split_weights_batch: 1 to 32 jobs");
    SplitBatch b = {};
    long long blocks = 0;
    for (int i = 0; i < n_jobs; ++i) {
        const anerf_split_job& q = jobs[i];
        const int npl = planes_of(q.precision);
        if (!q.w || !q.out || q.n < 1 || q.k < 1 || q.ldw < q.k || !npl)
            return anerf_internal_fail(ANERF_EINVAL, "anerf_mlp_split_weights_batch: bad job");
        const int rows = q.transpose ? q.k : q.n, cols = q.transpose ? q.n : q.k;
        SplitJob& J = b.j[i];
        J.w = q.w;
        J.out = static_cast<unsigned short*>(q.out);
        J.ldw = q.ldw;
        J.n = q.n;
        J.k = q.k;
        J.transpose = q.transpose;
        J.nblocks = (rows + BNW - 1) / BNW * (BNW / 32);
        J.ksteps = (cols + 15) / 16;
        J.npl = npl;
        J.f16exp = q.precision == ANERF_MLP_FP16X4
                       ? reinterpret_cast<int*>(static_cast<char*>(q.out) + split_plane_bytes(rows, cols, 2))
                       : nullptr;
        J.block0 = (int)blocks;
        blocks += ((long long)J.nblocks * J.ksteps * 512 + 255) / 256;
    }
    if (blocks > 0x7fffffff) return anerf_internal_fail(ANERF_EINVAL, "anerf_mlp_split_weights_batch: too large");
    b.n = n_jobs;
    bool any16 = false;
    for (int i = 0; i < n_jobs; ++i) any16 |= b.j[i].f16exp != nullptr;
    if (any16)
        hipLaunchKernelGGL(split_exponent_kernel, dim3((unsigned)n_jobs), dim3(1024), 0,
                           reinterpret_cast<hipStream_t>(stream), b);
    hipLaunchKernelGGL(split_weights_batch_kernel, dim3((unsigned)blocks), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), b);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? ANERF_OK : anerf_internal_fail(ANERF_EHIP, hipGetErrorString(e));
}

int anerf_mlp_gemm(int64_t m, int32_t n, int32_t k, const anerf_seg* a, int32_t n_a, const void* b_split,
                   int32_t precision, const float* bias, int32_t relu, const anerf_oseg* c, int32_t n_c, void* stream) {
    return anerf_mlp_gemm_rows(m, n, k, a, n_a, b_split, precision, bias, relu, c, n_c, nullptr, nullptr, stream);
}

int anerf_mlp_gemm_rows(int64_t m, int32_t n, int32_t k, const anerf_seg* a, int32_t n_a, const void* b_split,
                        int32_t precision, const float* bias, int32_t relu, const anerf_oseg* c, int32_t n_c,
                        const int32_t* rowmax_in, int32_t* rowmax_out, void* stream) {
    const int npl = planes_of(precision);
    if (m < 0 || n < 1 || k < 1 || !b_split || !c || n_c < 1 || n_c > MAXSEG || !npl)
        return anerf_internal_fail(ANERF_EINVAL, "anerf_mlp_gemm: bad arguments");
    const bool f16 = precision == ANERF_MLP_FP16X4;
    if (f16 && (n_a != 1 || !rowmax_in))
        return anerf_internal_fail(ANERF_EINVAL, "anerf_mlp_gemm: fp16x4 takes one A segment and its row maxima");
    if (!f16 && rowmax_in) return anerf_internal_fail(ANERF_EINVAL, "anerf_mlp_gemm: row maxima are fp16x4 input");
    if (rowmax_out && n % NBN) return anerf_internal_fail(ANERF_EINVAL, "anerf_mlp_gemm: row maxima need n % 128 == 0");
    // the epilogue's row max is taken on the vector path of one aligned output segment, before any mask or
    // accumulation: outside that case it would not be the maximum of what is stored
    if (rowmax_out && (n_c != 1 || c[0].mask || c[0].accumulate || !c[0].p || (reinterpret_cast<uintptr_t>(c[0].p) & 15) ||
                       (c[0].ld & 3)))
        return anerf_internal_fail(ANERF_EINVAL, "anerf_mlp_gemm: row maxima need one 16-byte aligned output segment "
                                                 "(ld % 4 == 0) without mask or accumulation");
    if (m == 0) return ANERF_OK;
    NTArgs g = {};
    g.M = m;
    g.N = n;
    g.K = k;
    int rc = set_segs(a, n_a, k, g.a);
    if (rc) return rc;
    for (int i = 0; i < n_a; ++i)  // (a 128-row tile's byte range fits a buffer descriptor)
        if (a[i].ld >= (1 << 22)) return anerf_internal_fail(ANERF_EINVAL, "anerf_mlp_gemm: operand ld >= 2^22");
    g.na = n_a;
    g.b = static_cast<const unsigned short*>(b_split);
    g.ksteps = (k + 15) / 16;
    g.bias = bias;
    g.relu = relu != 0;
    int start = 0;
    for (int i = 0; i < n_c; ++i) {
        if (c[i].cols < 1 || (c[i].p && c[i].ld < c[i].cols))
            return anerf_internal_fail(ANERF_EINVAL, "bad output segment");
        if (c[i].accumulate < 0 || c[i].accumulate > 2)
            return anerf_internal_fail(ANERF_EINVAL, "output segment accumulate must be 0, 1 or 2");
        g.c[i] = OSegD{c[i].p, c[i].ld, start, c[i].cols, c[i].mask, c[i].ldm, c[i].accumulate};
        start += c[i].cols;
    }
    if (start != n) return anerf_internal_fail(ANERF_EINVAL, "output segments do not add up to n");
    g.nc = n_c;
    // row-tile height: 128, or (ANERF_GEMM_BM 64) 64 for the single-segment instances
    // (the fp16x4 instance is always 128 rows high)
    const int tbm = (ANERF_GEMM_BM == 64 && n_a == 1 && !f16) ? 64 : 128;
    // 256-column tiles (CB 2) where the columns are whole 256s (the trunk and view-input layers at W 256)
    const int cb = (ANERF_GEMM_CB == 2 && !f16 && tbm == 128 && n % 256 == 0) ? 2 : 1;
    g.tiles_n = (n + NBN * cb - 1) / (NBN * cb);
    const long long tiles = (long long)((m + tbm - 1) / tbm) * g.tiles_n;
    if (tiles > 0x7fffffff) return anerf_internal_fail(ANERF_EINVAL, "anerf_mlp_gemm: too many tiles");
    g.total = (int)tiles;
    g.rin = rowmax_in;
    g.rout = rowmax_out;
    g.bexp = f16 ? reinterpret_cast<const int*>(static_cast<const char*>(b_split) + split_plane_bytes(n, k, 2))
                 : nullptr;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    hipError_t e = hipSuccess;
    if (f16) {
        e = nt_attr<2, 1, 128, 32, true>();
        if (e != hipSuccess) return anerf_internal_fail(ANERF_EHIP, hipGetErrorString(e));
        constexpr int LB = NTGeo<2, 128, 32>::LDS_BYTES;
        hipLaunchKernelGGL((mlp_nt_kernel<2, 1, 128, 32, true>), dim3((unsigned)tiles), dim3(NTHR), LB, st, g);
        e = hipGetLastError();
        return e == hipSuccess ? ANERF_OK : anerf_internal_fail(ANERF_EHIP, hipGetErrorString(e));
    }
#define ANERF_NT_LAUNCH(P, S)                                                                         \
    if (npl == P && n_a == S) {                                                                       \
        constexpr int TB = (ANERF_GEMM_BM == 64 && S == 1) ? 64 : 128;                                \
        constexpr int SKT = (ANERF_GEMM_SK64 && P == 2 && S == 1) ? 64 : 32;                          \
        constexpr int LB = NTGeo<P, TB, SKT>::LDS_BYTES;                                              \
        if (TB == 128 && cb == 2) {                                                                   \
            e = nt_attr<P, S, TB, SKT, false, 2>();                                                   \
            if (e != hipSuccess) return anerf_internal_fail(ANERF_EHIP, hipGetErrorString(e));        \
            hipLaunchKernelGGL((mlp_nt_kernel<P, S, TB, SKT, false, 2>), dim3((unsigned)tiles), dim3(NTHR), LB, st, g); \
        } else {                                                                                      \
            e = nt_attr<P, S, TB, SKT>();                                                             \
            if (e != hipSuccess) return anerf_internal_fail(ANERF_EHIP, hipGetErrorString(e));        \
            hipLaunchKernelGGL((mlp_nt_kernel<P, S, TB, SKT>), dim3((unsigned)tiles), dim3(NTHR), LB, st, g); \
        }                                                                                             \
    }
    ANERF_NT_LAUNCH(3, 1)
    ANERF_NT_LAUNCH(3, 2)
    ANERF_NT_LAUNCH(3, 3)
    ANERF_NT_LAUNCH(2, 1)
    ANERF_NT_LAUNCH(2, 2)
    ANERF_NT_LAUNCH(2, 3)
#undef ANERF_NT_LAUNCH
    e = hipGetLastError();
    return e == hipSuccess ? ANERF_OK : anerf_internal_fail(ANERF_EHIP, hipGetErrorString(e));
}

}  // extern "C"

namespace {
// workspace of the hidden (head = false) or head pass: per workgroup a [256 (+ 1)][256] dW slab, then per
// workgroup 256 (+ 4) db entries
size_t dgw_workspace(int64_t m, bool head) {
    long long rows;
    const int nwg = dgw_plan(m, &rows);
    return (size_t)4 * nwg * ((head ? DGW_W + 1 : DGW_W) * DGW_W + (head ? DGW_W + 4 : DGW_W));
}

int dgw_reduce(const char* fn, bool head, int64_t m, int32_t width, const void* workspace, size_t workspace_bytes,
               float* dw, int64_t lddw, float* db, void* stream) {
    if (width != DGW_W || m < 0 || !dw || !db || lddw < width)
        return anerf_internal_fail(ANERF_EINVAL, (std::string(fn) + ": bad arguments").c_str());
    if (!workspace || workspace_bytes < dgw_workspace(m, head))
        return anerf_internal_fail(ANERF_EWORKSPACE, (std::string(fn) + ": workspace too small").c_str());
    long long rows;
    const int nwg = dgw_plan(m, &rows);
    const float* ws = static_cast<const float*>(workspace);
    const int sr = head ? DGW_W + 1 : DGW_W, bst = head ? DGW_W + 4 : DGW_W;
    // dW rows 0 .. sr - 1 and the bias row sr (sr entries), summed over the workgroups' slabs in order
    hipLaunchKernelGGL(mlp_reduce_kernel, dim3(head ? 3 : DGW_W / 128, sr + 1), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), ws, nwg, (long long)sr * DGW_W, (long long)DGW_W, DGW_W,
                       dw, (long long)lddw, 0, sr, ws + (size_t)nwg * sr * DGW_W, (long long)bst, sr, db);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? ANERF_OK : anerf_internal_fail(ANERF_EHIP, hipGetErrorString(e));
}

int dgw_launch(const char* fn, bool head, int64_t m, int32_t width, const float* dy, int64_t lddy, const float* x,
               int64_t ldx, const void* wt_split, const float* wa, int32_t precision, float* dx, int64_t lddx,
               float* dw, int64_t lddw, float* db, void* workspace, size_t workspace_bytes, void* stream) {
    const std::string f(fn);
    if (width != DGW_W || precision != ANERF_MLP_BF16X3)
        return anerf_internal_fail(ANERF_EINVAL, (f + ": width 256 and ANERF_MLP_BF16X3 only").c_str());
    if (m < 0 || !dy || !x || !wt_split || !dx || (!dw != !db) || (dw && lddw < width) || (head && !wa))
        return anerf_internal_fail(ANERF_EINVAL, (f + ": bad arguments").c_str());
    // (float4 loads of whole rows; a 32-row chunk's byte range fits a buffer descriptor; the head's dy rows also
    // hold alpha's gradient at column 256)
    if ((reinterpret_cast<uintptr_t>(dy) | reinterpret_cast<uintptr_t>(x)) & 15 || (lddy | ldx) & 3 ||
        lddy < width + (head ? 1 : 0) || ldx < width || lddx < width || lddy >= (1 << 22) || ldx >= (1 << 22) ||
        lddx >= (1 << 22))
        return anerf_internal_fail(ANERF_EINVAL, (f + ": dy / x need 16 B aligned rows, ld % 4 == 0, width <= ld "
                                                      "< 2^22 (head: dy ld > width; dx: width <= ld < 2^22)").c_str());
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (!workspace || workspace_bytes < dgw_workspace(m, head))
        return anerf_internal_fail(ANERF_EWORKSPACE, (f + ": workspace too small").c_str());
    if (m == 0) {  // (the slabs of an empty sum: one zero slab, so that a deferred reduce writes zeros)
        hipError_t e = hipMemsetAsync(workspace, 0, dgw_workspace(m, head), st);
        if (e != hipSuccess) return anerf_internal_fail(ANERF_EHIP, hipGetErrorString(e));
        return dw ? dgw_reduce(fn, head, m, width, workspace, workspace_bytes, dw, lddw, db, stream) : ANERF_OK;
    }
    DGWArgs g = {};
    const int nwg = dgw_plan(m, &g.rows_per_wg);
    g.M = m;
    g.dy = dy;
    g.lddy = lddy;
    g.x = x;
    g.ldx = ldx;
    g.wt = static_cast<const unsigned short*>(wt_split);
    g.dx = dx;
    g.lddx = lddx;
    g.ws = static_cast<float*>(workspace);
    g.wsb = g.ws + (size_t)nwg * (head ? DGW_W + 1 : DGW_W) * DGW_W;
    g.wa = wa;
    const void* kern = head ? (const void*)mlp_dgw_kernel<true> : (const void*)mlp_dgw_kernel<false>;
    hipError_t e = hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, DGW_LDS);
    if (e != hipSuccess) return anerf_internal_fail(ANERF_EHIP, hipGetErrorString(e));
    if (head)
        hipLaunchKernelGGL(mlp_dgw_kernel<true>, dim3((unsigned)nwg), dim3(DGW_THR), DGW_LDS, st, g);
    else
        hipLaunchKernelGGL(mlp_dgw_kernel<false>, dim3((unsigned)nwg), dim3(DGW_THR), DGW_LDS, st, g);
    e = hipGetLastError();
    if (e != hipSuccess) return anerf_internal_fail(ANERF_EHIP, hipGetErrorString(e));
    return dw ? dgw_reduce(fn, head, m, width, workspace, workspace_bytes, dw, lddw, db, stream) : ANERF_OK;
}
}  // namespace

extern "C" {

size_t anerf_mlp_backward_hidden_workspace(int64_t m, int32_t width) {
    return width != DGW_W || m < 0 ? 0 : dgw_workspace(m, false);
}

int anerf_mlp_backward_hidden(int64_t m, int32_t width, const float* dy, int64_t lddy, const float* x, int64_t ldx,
                              const void* wt_split, int32_t precision, float* dx, int64_t lddx, float* dw, int64_t lddw,
                              float* db, void* workspace, size_t workspace_bytes, void* stream) {
    return dgw_launch("anerf_mlp_backward_hidden", false, m, width, dy, lddy, x, ldx, wt_split, nullptr, precision, dx,
                      lddx, dw, lddw, db, workspace, workspace_bytes, stream);
}

int anerf_mlp_backward_hidden_reduce(int64_t m, int32_t width, const void* workspace, size_t workspace_bytes, float* dw,
                                     int64_t lddw, float* db, void* stream) {
    return dgw_reduce("anerf_mlp_backward_hidden_reduce", false, m, width, workspace, workspace_bytes, dw, lddw, db,
                      stream);
}

}  // extern "C"

namespace {
// y[m][0, n) = act(sum_k a[m][k] W[o][k] + b[o]) on the persistent kernel, one launch per 256 output columns
int fw_launch(const char* fn, int64_t m, int32_t n, int32_t k, const anerf_seg* a, int32_t n_a, const void* w_split,
              int32_t precision, const float* bias, int32_t relu, float* y, int64_t ldy, const float* w_alpha,
              const float* b_alpha, float* alpha, int64_t ld_alpha, void* stream) {
    const std::string f(fn);
    const int npl = precision == ANERF_MLP_BF16X6 ? 3 : (precision == ANERF_MLP_BF16X3 ? 2 : 0);
    if (!npl) return anerf_internal_fail(ANERF_EINVAL, (f + ": ANERF_MLP_BF16X6 or _BF16X3").c_str());
    if (m < 0 || n < 4 || n % 4 || !a || n_a < 1 || n_a > 2 || !w_split || !y || k <= FW_KH || k % 4)
        return anerf_internal_fail(ANERF_EINVAL, (f + ": bad arguments (n % 4 == 0, 1 or 2 segments, 128 < k, "
                                                      "k % 4 == 0)").c_str());
    if (!w_alpha != !alpha || !w_alpha != !b_alpha || (alpha && ld_alpha < 1))
        return anerf_internal_fail(ANERF_EINVAL, (f + ": w_alpha, b_alpha, alpha all or none").c_str());
    const bool head = alpha != nullptr;
    if (head && (n_a != 1 || k != FW_W || n != FW_W))
        return anerf_internal_fail(ANERF_EINVAL, (f + ": alpha with one segment, k = n = 256 only").c_str());
    // (float4 loads and stores of whole rows; a 64-row chunk's byte range fits a buffer descriptor; the loaders read
    // units ahead of the stores, so y must not overlap an operand)
    int cols = 0;
    for (int i = 0; i < n_a; ++i) {
        if (!a[i].p || a[i].cols < 4 || a[i].cols % 4 || a[i].ld < a[i].cols || a[i].ld % 4 || a[i].ld >= (1 << 22) ||
            (reinterpret_cast<uintptr_t>(a[i].p) & 15))
            return anerf_internal_fail(ANERF_EINVAL, (f + ": segments need 16 B aligned rows, cols % 4 == 0, cols <= "
                                                          "ld < 2^22, ld % 4 == 0").c_str());
        cols += a[i].cols;
    }
    if (cols != k) return anerf_internal_fail(ANERF_EINVAL, (f + ": segments do not add up to k").c_str());
    if ((reinterpret_cast<uintptr_t>(y) & 15) || (ldy & 3) || ldy < n || ldy >= (1 << 22))
        return anerf_internal_fail(ANERF_EINVAL, (f + ": y needs 16 B aligned rows, ld % 4 == 0, n <= ld < 2^22").c_str());
    if (m == 0) return ANERF_OK;
    const uintptr_t yb = reinterpret_cast<uintptr_t>(y), ye = yb + 4 * ((m - 1) * ldy + n);
    for (int i = 0; i < n_a; ++i) {
        const uintptr_t xb = reinterpret_cast<uintptr_t>(a[i].p), xe = xb + 4 * ((m - 1) * a[i].ld + a[i].cols);
        if (xb < ye && yb < xe) return anerf_internal_fail(ANERF_EINVAL, (f + ": y overlaps an operand").c_str());
    }
    FWArgs g = {};
    const int nwg = fw_plan(m, &g.rows_per_wg);
    g.M = m;
    g.x0 = a[0].p;
    g.ld0 = a[0].ld;
    g.c0 = a[0].cols;
    g.x1 = n_a > 1 ? a[1].p : nullptr;
    g.ld1 = n_a > 1 ? a[1].ld : 0;
    g.K = k;
    g.nk = (k + 15) / 16;
    g.nu = (k + FW_KH - 1) / FW_KH;
    g.relu = relu != 0;
    g.ldy = ldy;
    g.wa = w_alpha;
    g.ba = b_alpha;
    g.alpha = alpha;
    g.lda = ld_alpha;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const int lb = npl == 3 ? FWGeo<3>::LDS : FWGeo<2>::LDS;
    const long long wtile = (long long)(FW_W / 32) * g.nk * npl * 512;  // split-W elements of 256 output rows
    hipError_t e = hipSuccess;
    for (int n0 = 0; n0 < n; n0 += FW_W) {  // (the split W's rows are zero-padded to whole 256s)
        g.w = static_cast<const unsigned short*>(w_split) + (n0 / FW_W) * wtile;
        g.bias = bias ? bias + n0 : nullptr;
        g.nval = n - n0 < FW_W ? n - n0 : FW_W;
        g.y = y + n0;
#define ANERF_FW_LAUNCH(P, S, H)                                                                                   \
        if (npl == P && n_a == S && head == H) {                                                                   \
            e = hipFuncSetAttribute((const void*)mlp_fwd_kernel<P, S, H>, hipFuncAttributeMaxDynamicSharedMemorySize, lb); \
            if (e != hipSuccess) return anerf_internal_fail(ANERF_EHIP, (f + ": " + hipGetErrorString(e)).c_str()); \
            hipLaunchKernelGGL((mlp_fwd_kernel<P, S, H>), dim3((unsigned)nwg), dim3(FW_THR), lb, st, g);         \
        }
        ANERF_FW_LAUNCH(3, 1, false)
        ANERF_FW_LAUNCH(3, 2, false)
        ANERF_FW_LAUNCH(3, 1, true)
        ANERF_FW_LAUNCH(2, 1, false)
        ANERF_FW_LAUNCH(2, 2, false)
        ANERF_FW_LAUNCH(2, 1, true)
#undef ANERF_FW_LAUNCH
        e = hipGetLastError();
        if (e != hipSuccess) return anerf_internal_fail(ANERF_EHIP, (f + ": " + hipGetErrorString(e)).c_str());
    }
    return ANERF_OK;
}
}  // namespace

extern "C" {

int anerf_mlp_forward_layer(int64_t m, int32_t k, const anerf_seg* a, int32_t n_a, const void* w_split,
                            int32_t precision, const float* bias, int32_t relu, float* y, int64_t ldy,
                            const float* w_alpha, const float* b_alpha, float* alpha, int64_t ld_alpha, void* stream) {
    if (!bias) return anerf_internal_fail(ANERF_EINVAL, "anerf_mlp_forward_layer: bias required");
    return fw_launch("anerf_mlp_forward_layer", m, FW_W, k, a, n_a, w_split, precision, bias, relu, y, ldy, w_alpha,
                     b_alpha, alpha, ld_alpha, stream);
}

int anerf_mlp_gemm_persistent(int64_t m, int32_t n, int32_t k, const anerf_seg* a, int32_t n_a, const void* b_split,
                              int32_t precision, const float* bias, int32_t relu, float* c, int64_t ldc, void* stream) {
    return fw_launch("anerf_mlp_gemm_persistent", m, n, k, a, n_a, b_split, precision, bias, relu, c, ldc, nullptr,
                     nullptr, nullptr, 0, stream);
}

int anerf_mlp_forward_hidden(int64_t m, int32_t width, const float* x, int64_t ldx, const void* w_split,
                             int32_t precision, const float* bias, float* y, int64_t ldy, void* stream) {
    if (width != FW_W) return anerf_internal_fail(ANERF_EINVAL, "anerf_mlp_forward_hidden: width 256");
    const anerf_seg seg = {x, ldx, FW_W};
    return anerf_mlp_forward_layer(m, FW_W, &seg, 1, w_split, precision, bias, 1, y, ldy, nullptr, nullptr, nullptr, 0,
                                   stream);
}

size_t anerf_mlp_backward_head_workspace(int64_t m, int32_t width) {
    return width != DGW_W || m < 0 ? 0 : dgw_workspace(m, true);
}

int anerf_mlp_backward_head(int64_t m, int32_t width, const float* dy, int64_t lddy, const float* x, int64_t ldx,
                            const void* wt_split, const float* w_alpha, int32_t precision, float* dx, int64_t lddx,
                            float* dw, int64_t lddw, float* db, void* workspace, size_t workspace_bytes, void* stream) {
    return dgw_launch("anerf_mlp_backward_head", true, m, width, dy, lddy, x, ldx, wt_split, w_alpha, precision, dx,
                      lddx, dw, lddw, db, workspace, workspace_bytes, stream);
}

int anerf_mlp_backward_head_reduce(int64_t m, int32_t width, const void* workspace, size_t workspace_bytes, float* dw,
                                   int64_t lddw, float* db, void* stream) {
    return dgw_reduce("anerf_mlp_backward_head_reduce", true, m, width, workspace, workspace_bytes, dw, lddw, db,
                      stream);
}

size_t anerf_mlp_wgrad_workspace(int64_t m, int32_t n, int32_t k) {
    int splits;
    long long rows;
    wgrad_plan(m, n, k, &splits, &rows);
    return (size_t)4 * splits * rup(n, BN) * (rup(k, BM) + 1);
}

int anerf_mlp_wgrad(int64_t m, int32_t n, int32_t k, const float* dy, int64_t lddy, const anerf_seg* x, int32_t n_x,
                    int32_t precision, float* dw, int64_t lddw, float* db, int32_t accumulate, void* workspace,
                    size_t workspace_bytes, void* stream) {
    const int npl = planes_of(precision);
    if (m < 0 || n < 1 || k < 1 || !dy || lddy < n || !dw || lddw < k || !npl || precision == ANERF_MLP_FP16X4)
        return anerf_internal_fail(ANERF_EINVAL, "anerf_mlp_wgrad: bad arguments");
    // dY is read as float4 groups of whole rows: 16 B aligned, ld a multiple of 4 and >= n rounded up
    // to 4 (the padding columns only reach the discarded rows n.. of the tile)
    if (lddy >= (1 << 22)) return anerf_internal_fail(ANERF_EINVAL, "anerf_mlp_wgrad: lddy >= 2^22");
    for (int i = 0; i < n_x && x; ++i)
        if (x[i].ld >= (1 << 22)) return anerf_internal_fail(ANERF_EINVAL, "anerf_mlp_wgrad: x ld >= 2^22");
    if ((reinterpret_cast<uintptr_t>(dy) & 15) || (lddy & 3) || lddy < (n + 3) / 4 * 4)
        return anerf_internal_fail(ANERF_EINVAL, "anerf_mlp_wgrad: dy must be 16 B aligned with ld % 4 == 0 "
                                                 "and ld >= round_up(n, 4)");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    TNArgs g = {};
    int rc = set_segs(x, n_x, k, g.x);
    if (rc) return rc;
    if (m == 0) {  // empty sum
        if (!accumulate) {
            hipError_t e = hipMemset2DAsync(dw, lddw * 4, 0, (size_t)k * 4, n, st);
            if (e == hipSuccess && db) e = hipMemsetAsync(db, 0, (size_t)n * 4, st);
            if (e != hipSuccess) return anerf_internal_fail(ANERF_EHIP, hipGetErrorString(e));
        }
        return ANERF_OK;
    }
    if (!workspace || workspace_bytes < anerf_mlp_wgrad_workspace(m, n, k))
        return anerf_internal_fail(ANERF_EWORKSPACE, "anerf_mlp_wgrad: workspace too small");
    g.M = m;
    g.N = n;
    g.K = k;
    g.dy = dy;
    g.lddy = lddy;
    g.nx = n_x;
    g.tiles = wgrad_plan(m, n, k, &g.splits, &g.rows_per_split);
    g.tiles_k = (k + BM - 1) / BM;
    g.npad = rup(n, BN);
    g.kpad = rup(k, BM);
    g.total = g.tiles * g.splits;
    g.ws = static_cast<float*>(workspace);
    g.wsb = db ? g.ws + (size_t)g.splits * g.npad * g.kpad : nullptr;
    hipError_t e = hipSuccess;
#define ANERF_TN_LAUNCH(P, S)                                                                         \
    if (npl == P && n_x == S) {                                                                       \
        e = tn_attr<P, S>();                                                                          \
        if (e != hipSuccess) return anerf_internal_fail(ANERF_EHIP, hipGetErrorString(e));            \
        constexpr int lds_ = TNGeo<P, S>::LDS_BYTES;                                                  \
        hipLaunchKernelGGL((mlp_tn_kernel<P, S>), dim3((unsigned)g.total), dim3(NTHR), lds_, st, g);  \
    }
    ANERF_TN_LAUNCH(3, 1)
    ANERF_TN_LAUNCH(3, 2)
    ANERF_TN_LAUNCH(3, 3)
    ANERF_TN_LAUNCH(2, 1)
    ANERF_TN_LAUNCH(2, 2)
    ANERF_TN_LAUNCH(2, 3)
#undef ANERF_TN_LAUNCH
    // dW rows 0 .. n - 1 and (with db) the bias row n in one launch
    const int gx = (db && g.npad > g.kpad ? g.npad : g.kpad) / 128;
    hipLaunchKernelGGL(mlp_reduce_kernel, dim3((unsigned)gx, (unsigned)(n + (db ? 1 : 0))), dim3(256), 0, st, g.ws,
                       g.splits, (long long)g.npad * g.kpad, (long long)g.kpad, k, dw, (long long)lddw,
                       accumulate != 0, n, g.wsb, (long long)g.npad, n, db);
    e = hipGetLastError();
    return e == hipSuccess ? ANERF_OK : anerf_internal_fail(ANERF_EHIP, hipGetErrorString(e));
}

}  // extern "C"
