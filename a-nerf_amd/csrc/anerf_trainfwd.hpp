// anerf_trainfwd.hpp — the training MLP's forward (NeRF.forward, core/networks/nerf.py:94-148) as one
// fused kernel: SURVEY §8(f) row 2.  Part of the single translation unit anerf_render.hip.
//
// Layer by layer on the split-bf16 GEMMs (anerf_gemm.hip) every [M, 256] activation goes to HBM and
// comes back for the next layer.  Here a wave keeps a 32-sample block's activations in its
// accumulators from layer 0 to the rgb head, as the render kernel does (mlp_layer_x6: bf16x6, the
// same fp32-accurate arithmetic as the GEMMs' bf16x6 forward), and writes each layer's output once,
// for the backward, in whole rows through a per-wave LDS transpose.  The encoder features are the
// training encoder's [M, F] rows (x = columns [0, dnet), views = [dnet, dnet + nv)), read as MFMA B
// operands straight from HBM (xmem_x6), split into three bf16 planes by truncation (exact).
// Weights are packed once per optimiser step by anerf_mlp_forward_pack (one launch): the dense
// activation parts in the render kernel's pack_layer_x6 order (k = the previous layer's accumulator
// order), the memory parts as groups (k16 step, output block) in natural column order.
// Outputs: h_0 .. h_{D-1} (post-relu), hf = feature_linear (no activation), g = relu(views_linears.0),
// raw = [rgb_linear(g), alpha_linear(h_{D-1})] — the tensors mlp.py's backward saves.
#pragma once

constexpr unsigned TF_NOOB = 0x80000000u;  // a lane offset past every buffer range: the load reads 0

// ---- packing (device: the weights change every optimiser step)
struct TfPackJob {
    const float* w;  // [n_out][ld] fp32 (torch nn.Linear layout)
    float* out;      // groups of 12 floats per lane, [group][3][64][4]
    int ld, n_out, col_off, n_in;  // regs: n_in = inputs (multiple of 32); mem: n_in = K columns
    int kind;                      // 0: activation part (pack_layer_x6 order), 1: memory part
    int ngroups;
    long long dw0;  // first dword of this job in the launch's grid
};
constexpr int TF_MAXJOBS = 24;
struct TfPackBatch {
    TfPackJob j[TF_MAXJOBS];
    int n;
};

__global__ void tf_pack_kernel(TfPackBatch b) {
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    int q = 0;
    for (int i = 1; i < b.n; ++i)
        if (t >= b.j[i].dw0) q = i;
    const TfPackJob J = b.j[q];
    const long long d = t - J.dw0;
    if (d < 0 || d >= (long long)J.ngroups * 768) return;
    const int e = (int)(d & 3), l = (int)((d >> 2) & 63), f = (int)((d >> 8) % 3);
    const int g = (int)(d / 768);
    const int h = l >> 5, rowl = l & 31;
    int ob, col0;  // output block; column of element j = col0 + colj(j)
    if (J.kind == 0) {  // pack_layer_x6's group order: lead groups 2 ob + s, then (ib >= 1, s, ob)
        const int RBO = J.n_out / 32;
        int ib, s;
        if (g < 2 * RBO) {
            ob = g >> 1, ib = 0, s = g & 1;
        } else {
            const int idx = g - 2 * RBO;
            ib = 1 + idx / (2 * RBO), s = (idx / RBO) & 1, ob = idx % RBO;
        }
        col0 = 32 * ib + 16 * s;
    } else {  // groups (s, ob): k16 step s, natural column order k = 16 s + 8 h + j
        const int RBO = J.n_out / 32;
        const int s = g / RBO;
        ob = g % RBO;
        col0 = 16 * s;
    }
    const int row = 32 * ob + rowl;
    unsigned bits = 0;
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
        const int j = 2 * e + jj;
        const int k = J.kind == 0 ? col0 + 8 * (j >> 2) + 4 * h + (j & 3) : col0 + 8 * h + j;
        float r = (J.kind == 0 || k < J.n_in) ? J.w[(long long)row * J.ld + J.col_off + k] : 0.0f;
        unsigned short v = 0;
        for (int p = 0; p <= f; ++p) {  // RNE of the running remainder (exact in fp32)
            const __bf16 hb = (__bf16)r;
            v = __builtin_bit_cast(unsigned short, hb);
            r -= (float)hb;
        }
        bits |= (unsigned)v << (16 * jj);
    }
    reinterpret_cast<unsigned*>(J.out)[d] = bits;
}

// ---- forward kernel
struct TfArgs {
    int D, skip, dnet, nv, cfc;
    long long M;
    const float* feat;
    long long ldf;
    const float* codes;
    long long ldc;
    const float* wx0;    // layer 0 (memory part, K = dnet)
    const float* wl[MAXL];  // layers 1 .. D-1, activation part
    const float* wskipx;    // the skip layer's x part (memory, K = dnet) or null
    const float* wf;        // feature_linear (activation part)
    const float* wvf;       // views_linears.0, feature part (activation part, W/2 outputs)
    const float* wvv;       // views_linears.0, view part (memory, K = nv)
    const float* wvc;       // views_linears.0, framecode part (memory, K = cfc) or null
    const float* b[MAXL];
    const float* bf;
    const float* wa;
    const float* ba;  // [1]
    const float* bv;
    const float* wrgb;  // [3][W/2]
    const float* brgb;  // [3]
    float* h[MAXL];
    float* hf;
    float* g;
    float* raw;  // [M][4]
};

// out[RBO] += W_part^T x over columns [col_off, col_off + K) of the rows of `ra` (this block's rows;
// rows past M read 0), x split by truncation into three bf16 planes; weight groups (s, rb) in the
// 4-slot ring three groups ahead, x four k16 steps ahead (HBM latency); side(g) after each group's
// prefetch (the store drain).
constexpr int TF_XD = 4;  // k16 steps of x in flight (and the unroll: ring slots stay compile-time)
__host__ __device__ constexpr int tf_xsteps(int K) { return ((K + 15) / 16 + TF_XD - 1) / TF_XD * TF_XD; }

template <int RBO, class Side = NoSide>
__device__ __forceinline__ void xmem_x6(f32x16 (&out)[RBO], __amdgpu_buffer_rsrc_t ra, unsigned arow, int col_off,
                                        int K, const float* __restrict__ wp, int lane, Ring& ring,
                                        bool preloaded = false, Side* side = nullptr) {
    constexpr int PD = 3;
    const int h = lane >> 5;
    const int ns = tf_xsteps(K);
    const int ng = ns * RBO;
    const __amdgpu_buffer_rsrc_t rw = make_rsrc(wp);
    if (!preloaded)
#pragma unroll
        for (int d = 0; d < PD; ++d) load_group<12>(ring.v[d], rw, lane, d);
    auto fetch_x = [&](int s, f32x4 (&x)[2]) {
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const int k = 16 * s + 8 * h + 4 * c;
            const unsigned vo = k < K ? arow + (unsigned)(col_off + k) * 4u : TF_NOOB;  // (K % 4 == 0)
            x[c] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(ra, vo, 0, 0));
        }
    };
    f32x4 xr[TF_XD][2];
#pragma unroll
    for (int d = 0; d < TF_XD; ++d) fetch_x(d, xr[d]);
    for (int s0 = 0; s0 < ns; s0 += TF_XD) {
#pragma unroll
        for (int ss = 0; ss < TF_XD; ++ss) {
            const int s = s0 + ss;
            X6T t;
            split3_pair(xr[ss][0][0], xr[ss][0][1], t, 0);
            split3_pair(xr[ss][0][2], xr[ss][0][3], t, 1);
            split3_pair(xr[ss][1][0], xr[ss][1][1], t, 2);
            split3_pair(xr[ss][1][2], xr[ss][1][3], t, 3);
            __builtin_amdgcn_sched_barrier(0);
            fetch_x(s + TF_XD, xr[ss]);  // (past K: zero)
#pragma unroll
            for (int rb = 0; rb < RBO; ++rb) {
                // (s0 * RBO is a multiple of 4: the slots are static)
                const int slot = (ss * RBO + rb) & 3;
                const int g = s * RBO + rb;
                __builtin_amdgcn_sched_barrier(0);
                load_group<12>(ring.v[(slot + PD) & 3], rw, lane, min(g + PD, ng - 1));
                if constexpr (!std::is_same<Side, NoSide>::value) (*side)(g);
                out[rb] = mfma_x6(ring.v[slot], t, out[rb]);
            }
        }
    }
}

// The stores of one staged tile (the wave's LDS rows: a layer's output, 32 samples x 32 RBO columns)
// spread over the groups of the next MFMA phase: instruction i (RPI rows of 8 RBO lanes x 16 B) at
// every `every`-th group call (the calls of consecutive phases count on).  Issued in a burst, a layer's 32 KB of stores delay every weight load issued after
// them (the vector memory counter retires in order); one store per few groups stays under the MFMAs.
struct TfDrain {
    const float* stage;
    float* dst;
    long long ld, row0;
    int rows, lane, sp, lg, n, next, every, cnt;  // lg: log2(lanes per row)
    __device__ __forceinline__ void start(const float* st, float* d, long long ld_, long long r0, int rows_, int lane_,
                                          int sp_, int rbo, int groups) {
        stage = st, dst = d, ld = ld_, row0 = r0, rows = rows_, lane = lane_, sp = sp_;
        lg = rbo == 8 ? 6 : (rbo == 4 ? 5 : (rbo == 2 ? 4 : 3));
        n = 32 >> (6 - lg);  // 32 rows / (rows per instruction)
        next = 0, cnt = 0;
        every = groups > n ? groups / n : 1;
    }
    __device__ __forceinline__ void issue() {
        const int row = (next << (6 - lg)) + (lane >> lg), c4 = 4 * (lane & ((1 << lg) - 1));
        const f32x4 v = *reinterpret_cast<const f32x4*>(stage + row * sp + c4);
        if (row < rows) *reinterpret_cast<f32x4*>(dst + (row0 + row) * ld + c4) = v;
        ++next;
    }
    __device__ __forceinline__ void operator()(int) {
        if (++cnt >= every) {
            cnt = 0;
            if (next < n) issue();
        }
    }
    __device__ __forceinline__ void flush() {
        while (next < n) issue();
    }
};

// act(a) (block rows = samples, registers = columns) into the wave's LDS tile [32][sp] (the caller
// has drained the previous tile); TfDrain writes it out as whole rows
template <int RBO>
__device__ __forceinline__ void tf_stage(const f32x16 (&a)[RBO], bool relu, float* __restrict__ stage, int sp,
                                         int lane) {
    const int h = lane >> 5, r = lane & 31;
    wave_sync();  // (the drain's LDS reads of the previous tile are complete)
#pragma unroll
    for (int rb = 0; rb < RBO; ++rb)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            f32x4 v = {a[rb][4 * q], a[rb][4 * q + 1], a[rb][4 * q + 2], a[rb][4 * q + 3]};
            if (relu)
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = relu_act(v[e]);
            *reinterpret_cast<f32x4*>(stage + r * sp + 32 * rb + 8 * q + 4 * h) = v;
        }
    wave_sync();
}

template <int W>
__global__ __launch_bounds__(256, 1) void train_mlp_fwd_kernel(TfArgs A) {
    constexpr int RB = W / 32, RBV = RB / 2, WH = W / 2;
    constexpr int SP = W + 4;  // stage pitch (floats): rows 16 B aligned, consecutive rows 4 banks apart
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int D = A.D;
    float* const bias = lds;                                  // [D + 1][W] + [W/2], accumulator order
    float* const wal = bias + (D + 1) * W + WH;               // [2][RB][16]
    float* const wrl = wal + 2 * RB * 16;                     // [3][2][RBV][16]
    float* const stage_all = wrl + 3 * 2 * RBV * 16;          // [4][32][SP]
    const int tid = threadIdx.x;
    // biases and head weights in accumulator order: element i of lane half hh of block rb is
    // output 32 rb + acc_row(i, hh)
    for (int t = tid; t < (D + 1) * W + WH; t += blockDim.x) {
        const int L = t / W, o = t % W;
        const int rb = o >> 5, hh = (o >> 4) & 1, i = o & 15;
        const int n = 32 * rb + acc_row(i, hh);
        bias[t] = L < D ? A.b[L][n] : (L == D ? A.bf[n] : A.bv[n]);
    }
    for (int t = tid; t < 2 * RB * 16; t += blockDim.x) {
        const int hh = t / (16 * RB), ib = (t / 16) % RB, i = t % 16;
        wal[t] = A.wa[32 * ib + acc_row(i, hh)];
    }
    for (int t = tid; t < 3 * 2 * RBV * 16; t += blockDim.x) {
        const int c = t / (2 * RBV * 16), hh = (t / (RBV * 16)) & 1, rb = (t / 16) % RBV, i = t % 16;
        wrl[t] = A.wrgb[c * WH + 32 * rb + acc_row(i, hh)];
    }
    __syncthreads();
    // (the wave index through readfirstlane: a VGPR-derived block index would make every buffer
    // descriptor below a VGPR and each load a waterfall loop)
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63, hh = lane >> 5;
    float* const stage = stage_all + wave * 32 * SP;
    const long long nblk = (A.M + 31) / 32;
    const long long nw = (long long)gridDim.x * 4;
    const unsigned arowf = (unsigned)((lane & 31) * A.ldf * 4);
    const unsigned arowc = (unsigned)((lane & 31) * A.ldc * 4);
    TfDrain drain;
    drain.n = 0, drain.next = 0, drain.cnt = 0, drain.every = 1;  // (nothing pending)
    constexpr int NGH = 2 * RB * RB;  // groups of a W -> W layer
    for (long long blk = (long long)blockIdx.x * 4 + wave; blk < nblk; blk += nw) {
        const long long row0 = blk * 32;
        const int rows = (int)min((long long)32, A.M - row0);
#ifdef ANERF_TF_XL2  // (diagnostic A/B only: every wave reads feature rows 0..63, L2-resident)
        const __amdgpu_buffer_rsrc_t rf = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(A.feat + (blk & 1) * 32 * A.ldf), 0, (int)(rows * A.ldf * 4), 0x00020000);
#else
        const __amdgpu_buffer_rsrc_t rf =
            __builtin_amdgcn_make_buffer_rsrc((void*)(A.feat + row0 * A.ldf), 0, (int)(rows * A.ldf * 4), 0x00020000);
#endif
        Ring ring;
        f32x16 acc[RB], h[RB];
        float nosig = 0.0f;
        load_bias<RB>(acc, bias, hh);
        // layer 0 (the previous block's g tile drains under it)
        xmem_x6<RB, TfDrain>(acc, rf, arowf, 0, A.dnet, A.wx0, lane, ring, false, &drain);
        drain.flush();
        tf_stage<RB>(acc, true, stage, SP, lane);
        drain.start(stage, A.h[0], W, row0, rows, lane, SP, RB, NGH);
        for (int L = 1; L < D; ++L) {
            mlp_layer_x6<RB, RB, true, false, true, TfDrain>(acc, acc, h, bias + L * W, A.wl[L], lane, ring, false,
                                                             nullptr, nullptr, nosig, &drain);
            if (L == A.skip + 1) xmem_x6<RB, TfDrain>(acc, rf, arowf, 0, A.dnet, A.wskipx, lane, ring, false, &drain);
            drain.flush();
            tf_stage<RB>(acc, true, stage, SP, lane);
            drain.start(stage, A.h[L], W, row0, rows, lane, SP, RB, NGH);
        }
        // feature_linear (no activation) with alpha_linear folded into its groups
        float sig = 0.0f;
        mlp_layer_x6<RB, RB, true, true, true, TfDrain>(acc, acc, h, bias + D * W, A.wf, lane, ring, false, nullptr,
                                                        wal, sig, &drain);
        sig += __shfl_xor(sig, 32);
        drain.flush();
        tf_stage<RB>(acc, false, stage, SP, lane);
        drain.start(stage, A.hf, W, row0, rows, lane, SP, RB, 2 * RBV * RB + tf_xsteps(A.nv) * RBV);
        // views_linears.0 on [feature | views | framecode], relu
        f32x16 av[RBV];
        mlp_layer_x6<RBV, RB, false, false, false, TfDrain>(av, acc, h, nullptr, A.wvf, lane, ring, false, nullptr,
                                                            nullptr, nosig, &drain);
        xmem_x6<RBV, TfDrain>(av, rf, arowf, A.dnet, A.nv, A.wvv, lane, ring, false, &drain);
        if (A.cfc > 0) {
            const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc((void*)(A.codes + row0 * A.ldc), 0,
                                                                                (int)(rows * A.ldc * 4), 0x00020000);
            xmem_x6<RBV, TfDrain>(av, rc, arowc, 0, A.cfc, A.wvc, lane, ring, false, &drain);
        }
#pragma unroll
        for (int rb = 0; rb < RBV; ++rb)
#pragma unroll
            for (int i = 0; i < 16; ++i) av[rb][i] += bias[(D + 1) * W + (rb * 2 + hh) * 16 + i];
        drain.flush();
        tf_stage<RBV>(av, true, stage, SP, lane);
        // (drained under the next block's layer 0, or at the end)
        drain.start(stage, A.g, WH, row0, rows, lane, SP, RBV, tf_xsteps(A.dnet) * RB);
        // rgb_linear on relu(g)
        float rgb[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const float* wr = wrl + (c * 2 + hh) * RBV * 16;
            float a = 0.0f;
#pragma unroll
            for (int rb = 0; rb < RBV; ++rb)
#pragma unroll
                for (int i = 0; i < 16; ++i) a = fmaf(wr[rb * 16 + i], relu_act(av[rb][i]), a);
            a += __shfl_xor(a, 32);
            rgb[c] = a + A.brgb[c];
        }
        if (hh == 0 && (lane & 31) < rows)
            *reinterpret_cast<f32x4*>(A.raw + (row0 + (lane & 31)) * 4) = f32x4{rgb[0], rgb[1], rgb[2], sig + A.ba[0]};
    }
    drain.flush();
}
