// anerf_kernels.hpp — __global__ kernels: fused render kernel, density-only kernel, near/far + NaN fill, ray generation, composition, encoding stage.
// Part of the single translation unit anerf_render.hip (included there, in order).
#pragma once

// ======================================================================= fused render kernel
#ifndef ANERF_BLOCK_SORT
#define ANERF_BLOCK_SORT 1  // (0: blocks in ray order; tools/build_ab.sh experiments)
#endif
#ifndef ANERF_PERSIST
#define ANERF_PERSIST 1  // persistent workgroups over XCD-banded queues (+3.6 % fp16x4, bit-identical; 0: one workgroup per item)
#endif
// The rays [ray0, ray0 + R) of one workgroup: both passes (or the launch's one) end to end.
template <int W, int MR, int PREC>
__device__ __forceinline__ void render_item(const ModelDev& M, const RenderArgs& A, const LdsPlan& P,
                                            float* __restrict__ lds, int64_t ray0) {
    constexpr int WH = W / 2;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int R = A.R, S = A.S, I = A.I, T = S + I;
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
        // (an out-of-range pose index renders NaN and is never dereferenced)
        lds[P.sk + P.sk_stride * r + e] = (pose >= 0 && pose < A.n_poses) ? A.skts[((int64_t)pose * M.nj + j) * 16 + c]
                                                                           : __int_as_float(0x7fc00000);
    }
    stage_cut(M, lds + P.cut, tid);
    // coarse samples (sample_from_lineseg, ray_utils.py:218-224)
    for (int idx = tid; idx < nr * S; idx += blockDim.x) {
        const int r = idx / S, s = idx % S;
        const float t = torch_linspace01(s, S);
        const float nearv = lds[P.ray + 16 * r + 7], farv = lds[P.ray + 16 * r + 8];
        lds[P.zc + P.z_stride * r + s] = lineseg_z(nearv, farv, t, A.lindisp != 0);
    }
    if (A.pass0 == 1) {  // fine-only launch: the sorted fine z of the coarse launch
        // (16 B per lane: the item's nr x T floats are one contiguous run, rows 16-B aligned)
        if (T % 4 == 0 && (reinterpret_cast<uintptr_t>(A.zf_ws) & 15) == 0) {
            const f32x4* src = reinterpret_cast<const f32x4*>(A.zf_ws + ray0 * T);
            for (int idx = tid; idx < nr * T / 4; idx += blockDim.x) {
                const int r = (4 * idx) / T, s = (4 * idx) % T;
                *reinterpret_cast<f32x4*>(lds + P.zf + P.z_stride * r + s) = __builtin_nontemporal_load(src + idx);
            }
        } else {
            for (int idx = tid; idx < nr * T; idx += blockDim.x) {
                const int r = idx / T, s = idx % T;
                lds[P.zf + P.z_stride * r + s] = __builtin_nontemporal_load(A.zf_ws + (ray0 + r) * T + s);
            }
        }
    }
    __syncthreads();

    Stamps st;
    STAMP_INIT(st);
    STAMP(st, 0);
    const int n_pass = I > 0 ? 2 : 1;
    for (int pass = A.pass0; pass < min(A.pass1, n_pass); ++pass) {
        const NetDev& net = M.net[pass];
        const int n = pass == 0 ? S : T;
        const int zoff = pass == 0 ? P.zc : P.zf;
        // single_net fine pass (raycasters.py:462-468): the same network on the I new samples only
        // (z_is, left by importance() in the ray's scratch at 6 z_stride), raws after the coarse ones
        // (cat([raw, raw_is]) order), merged by sorted_idx below; biases and G are still in LDS
        const bool only_new = pass == 1 && M.single_net;
        if (!only_new) {
            stage_bias<W>(M, net, lds + P.bias, tid);  // (synced below)
            if (M.mrv == 0) compute_view_factor<WH, 0>(M, net, lds, P, nr, tid, st);
            else compute_view_factor<WH, 4>(M, net, lds, P, nr, tid, st);
        }
        STAMP(st, 1);
        // ---- MLP over 32-sample blocks, four at a time (one per wave)
        const int nm = only_new ? I : n;
        const int nb = (nm + 31) / 32, nbt = nr * nb;
        auto block_z = [&](int r) {
            return only_new ? lds + P.scr + P.scr_stride * r + 6 * P.z_stride : lds + zoff + P.z_stride * r;
        };
        int* const bcnt = reinterpret_cast<int*>(lds + P.bord);
        int* const bord = bcnt + P.bord_n;
        if constexpr (lockstep_mode<PREC>() && ANERF_BLOCK_SORT) {
            // bf16x6: the four waves meet at a workgroup barrier before every hidden layer (L1 sharing of
            // the weight stream), where a wave whose block has fewer live joints waits for the others
            // (5.8 % of the wave-cycles, profiles/r04c_stamps_bf16x6.txt).  The blocks of the workgroup
            // run in ascending order of their live-joint counts, so the four blocks of an iteration have
            // about equal windowed work.  (Outputs are unchanged: a block's arithmetic does not depend on
            // the wave that runs it.)
            for (int b = wave; b < nbt; b += 4) {
                const int r = b / nb;
                const int c = block_live_count(M, lds + P.ray + 16 * r, lds + P.sk + P.sk_stride * r, lds + P.cut,
                                               block_z(r), nm, (b % nb) * 32, lane);
                if (lane == 0) bcnt[b] = c;
            }
            __syncthreads();
            for (int i = tid; i < nbt; i += blockDim.x) {
                const int ci = bcnt[i];
                int rank = 0;
                for (int j = 0; j < nbt; ++j) {
                    const int cj = bcnt[j];
                    rank += (cj < ci) | ((cj == ci) & (j < i));
                }
                bord[rank] = i;
            }
            __syncthreads();
        }
        // (the same trip count on every wave: bf16x6's mlp_trunk has a workgroup barrier per hidden
        // layer; a wave past the last block redoes that block without storing or counting it)
        for (int it = 0; it < (nbt + 3) / 4; ++it) {
            const bool own = it * 4 + wave < nbt;
            if constexpr (!lockstep_mode<PREC>())  // (no workgroup barrier inside: a wave without a block is done)
                if (!own) break;
            const int bi = own ? it * 4 + wave : nbt - 1;
            const int b = (lockstep_mode<PREC>() && ANERF_BLOCK_SORT) ? bord[bi] : bi;
            const int r = b / nb, s0 = (b % nb) * 32;
            const float* zr = block_z(r);
            float* rawr = lds + P.raw + P.raw_stride * r + (only_new ? 4 * S : 0);
            mlp_block<W, MR, PREC>(M, net, lds + P.ray + 16 * r, lds + P.sk + P.sk_stride * r, lds + P.cut,
                             zr, nm, s0, lds + P.g + P.g_stride * r, rawr, lane, own ? A.mfma_count : nullptr,
                             lds + P.bias, (P.uf >= 0 && M.skip + 1 < M.D) ? lds + P.uf + wave * P.uf_stride : nullptr,
                             lds + P.wv + wave * P.wv_stride, st, own);
        }
        STAMP(st, 2 + 2 * pass);
        __syncthreads();
        STAMP(st, 6);
        // ---- composite (+ importance sampling after the coarse pass); one wave per ray
        for (int r0 = 0; r0 < R; r0 += 4) {
            // (the wave index as a scalar here: the ray index and the output pointers become wave-uniform SGPR
            // values instead of 64-bit per-lane pointers the allocator kept live, spilled, across the MLP)
            const int r = r0 + __builtin_amdgcn_readfirstlane(wave);
            const bool active = r < nr;
            const int64_t i = ray0 + r;
            const float* ray = lds + P.ray + 16 * min(r, R - 1);
            const float* z = lds + zoff + P.z_stride * min(r, R - 1);
            float* raw = lds + P.raw + P.raw_stride * min(r, R - 1);
            float* scr = lds + P.scr + P.scr_stride * min(r, R - 1);
            if (only_new) {  // raw = cat([raw, raw_is])[sorted_idx] (_merge_encodings on 'raw', :466-468)
                const int* src = reinterpret_cast<const int*>(scr + 7 * P.z_stride);
                if (active)
                    for (int k = lane; k < T; k += 64)
                        *reinterpret_cast<f32x4*>(scr + 4 * k) = *reinterpret_cast<const f32x4*>(raw + 4 * src[k]);
                wave_sync();
                if (active)
                    for (int k = lane; k < T; k += 64)
                        *reinterpret_cast<f32x4*>(raw + 4 * k) = *reinterpret_cast<const f32x4*>(scr + 4 * k);
                wave_sync();
            }
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
                importance(z, scr, S, I, lds + P.zf + P.z_stride * min(r, R - 1), scr + P.z_stride, active, lane,
                           nullptr, M.single_net != 0, M.single_net ? reinterpret_cast<int*>(scr + 7 * P.z_stride) : nullptr,
                           M.single_net ? scr + 6 * P.z_stride : nullptr);
            }
        }
        __syncthreads();
        STAMP(st, 3 + 2 * pass);
    }
    if (I > 0 && A.pass1 == 1) {  // coarse-only launch: hand the fine z over
        // (non-temporal: 0.8 KB per ray streams through L2 and would evict weight groups; 16 B per lane where
        // T % 4 == 0 -- whole 64-B lines per quarter wave instead of 4-B pieces)
        if (T % 4 == 0 && (reinterpret_cast<uintptr_t>(A.zf_ws) & 15) == 0) {
            f32x4* dst = reinterpret_cast<f32x4*>(A.zf_ws + ray0 * T);
            for (int idx = tid; idx < nr * T / 4; idx += blockDim.x) {
                const int r = (4 * idx) / T, s = (4 * idx) % T;
                __builtin_nontemporal_store(*reinterpret_cast<const f32x4*>(lds + P.zf + P.z_stride * r + s), dst + idx);
            }
        } else {
            for (int idx = tid; idx < nr * T; idx += blockDim.x) {
                const int r = idx / T, s = idx % T;
                __builtin_nontemporal_store(lds[P.zf + P.z_stride * r + s], A.zf_ws + (ray0 + r) * T + s);
            }
        }
    }
    STAMP_FLUSH(st, A.stamps);
}

// One launch of the render pass(es).  ANERF_PERSIST (default): as many workgroups as are resident at
// once (the host sizes the grid by occupancy), each taking R-ray items from eight queues, queue g = the
// g-th contiguous band of the ray list, starting with its own (blockIdx & 7: workgroups b and b + 8
// share an XCD under the round-robin dispatch — a locality choice only, correctness does not depend on
// it) and stealing from the others when it is empty, so each XCD's L2 sees the live joints of one band
// of the frame while the stealing evens out the bands' different costs (round 3's static XCD bands
// lost 5 % to exactly that imbalance); +3.6 % fp16x4, outputs bit-identical (an item's arithmetic does
// not depend on the workgroup that runs it).  ANERF_PERSIST 0: workgroup b renders rays [b R, b R + R).
template <int W, int MR, int PREC>
__global__ __launch_bounds__(256, 1) void render_kernel(ModelDev M, RenderArgs A, LdsPlan P) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    if constexpr (!ANERF_PERSIST) {
        render_item<W, MR, PREC>(M, A, P, lds, (int64_t)blockIdx.x * A.R);
    } else {
        const int64_t items = (A.n + A.R - 1) / A.R;
        int* const slot = reinterpret_cast<int*>(lds + P.bord) + 2 * P.bord_n;
        const int g0 = blockIdx.x & 7;
        for (;;) {
            if (threadIdx.x == 0) {
                int64_t item = -1;
                for (int k = 0; k < 8 && item < 0; ++k) {
                    const int g = (g0 + k) & 7;
                    const int64_t b0 = items * g / 8, b1 = items * (g + 1) / 8;
                    if (b1 <= b0) continue;
                    const unsigned t = atomicAdd(A.queue + g, 1u);
                    if ((int64_t)t < b1 - b0) item = b0 + t;
                }
                slot[0] = (int)item;
            }
            __syncthreads();
            const int item = slot[0];
            if (item < 0) break;
            render_item<W, MR, PREC>(M, A, P, lds, (int64_t)item * A.R);
            __syncthreads();
        }
    }
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

__host__ __device__ inline LdsPlan make_density_plan(int nj, int W, int D, int njh2, bool bone_cut) {
    LdsPlan p;
    std::memset(&p, 0, sizeof(p));
    int o = 0;
    p.sk = o; o += 12 * nj;
    p.cut = o; o += (bone_cut ? 4 : 3) * nj;
    o = (o + 3) & ~3;
    p.bias = o; o += (D + 2) * W;
    p.uf_stride = 64 * 3 * njh2;
    p.uf = o; o += 4 * p.uf_stride;
    p.total = (o + 3) & ~3;
    return p;
}

template <int W, int MR, int PREC>
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
    // (the same trip count on every wave: bf16x6's mlp_trunk has a workgroup barrier per hidden layer;
    // a wave past the last block redoes it without storing)
    for (int64_t base = (int64_t)blockIdx.x * 4; base < nb; base += (int64_t)gridDim.x * 4) {
        const bool own = base + wave < nb;
        if constexpr (!lockstep_mode<PREC>())
            if (!own) break;
        const int64_t b = own ? base + wave : nb - 1;
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
        int es = 0;
        mlp_trunk<W, MR, false, PREC, true>(M, net, lds + P.sk, lds + P.cut, px, py, pz, lane, lds + P.bias, uf, nullptr, acc, h, ring,
                         mask, nullptr, st, es);
        // alpha_linear on relu(h_last), in the k-step order of the render path's fused alpha head
        float sig = 0.0f;
#pragma unroll
        for (int q = 0; q < W / 2; ++q) sig = fmaf(wa[q], relu_act(acc[q >> 4][q & 15]), sig);
        if constexpr (PREC >= 3) sig *= pow2f(-es);  // (fp16x3 / fp16x4: the last layer's units)
        sig += __shfl_xor(sig, 32);
        sig += net.balpha;
        if (own && hh == 0 && s_out < A.n) A.out[s_out] = sig;
    }
}

// ======================================================================= small kernels
// ANERF_FLAG_NEAR_FAR: the caller's filled near / far (ray_batch columns 6, 7) into the workspace
__global__ void near_far_given_kernel(const float* __restrict__ rb, int stride, int64_t n, float* __restrict__ near_out,
                                      float* __restrict__ far_out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    near_out[i] = rb[i * stride + 6];
    far_out[i] = rb[i * stride + 7];
}

__global__ void near_far_kernel(const float* __restrict__ rb, int stride, int64_t n, const float* __restrict__ cyls,
                                const int32_t* __restrict__ ray_pose, int n_poses, float* __restrict__ near_out,
                                float* __restrict__ far_out, uint8_t* __restrict__ qnan) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float* r = rb + i * stride;
    const int pose = ray_pose ? ray_pose[i] : 0;
    if (pose < 0 || pose >= n_poses) {  // out-of-range pose index: a miss (filled by the chunk mean)
        near_out[i] = far_out[i] = __int_as_float(0x7fc00000);
        qnan[i] = 1;
        return;
    }
    const float* cy = cyls + 5 * pose;
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
constexpr int NF_LEAVES = 1024;  // leaves of <= 128 rays: chunks up to ~65 k rays in parallel
constexpr int NF_LDS = 8192;     // chunks up to this many rays sum from LDS

__global__ void nan_fill_kernel(const float* __restrict__ rb, int stride, int64_t n, int chunk,
                                float* __restrict__ near_io, float* __restrict__ far_io,
                                const uint8_t* __restrict__ qnan, float* __restrict__ scratch) {
    const int64_t c0 = (int64_t)blockIdx.x * chunk;
    const int64_t c1 = min(c0 + chunk, n);
    const int64_t m = c1 - c0;
    __shared__ int any, n_leaves, valid[2];
    __shared__ float means[2];
    __shared__ int leaf_off[NF_LEAVES], leaf_cnt[NF_LEAVES];
    __shared__ float leaf_sum[NF_LEAVES];
    if (threadIdx.x == 0) { any = 0; valid[0] = valid[1] = 0; }
    __syncthreads();
    for (int64_t i = c0 + threadIdx.x; i < c1; i += blockDim.x)
        if (near_io[i] != near_io[i]) any = 1;
    __syncthreads();
    if (!any) return;
    __shared__ int st_a[64], st_b[64];  // (the tree walks' stacks, thread 0)
    __shared__ float st_v[64];
    if (threadIdx.x == 0) n_leaves = np_pairwise_leaves(m, leaf_off, leaf_cnt, NF_LEAVES, st_a, st_b);
    // NaN -> 0 copies, one vector at a time: in LDS for chunks up to NF_LDS rays (the leaf sums' loads then wait
    // on LDS, not on L2: 55 -> a few us for a 2048-ray training batch), else in the scratch
    __shared__ float lbuf[NF_LDS];
    float* buf = m <= NF_LDS ? lbuf : scratch + c0;
    for (int v = 0; v < 2; ++v) {
        const float* src = v == 0 ? near_io : far_io;
        int mine = 0;
        for (int64_t i = c0 + threadIdx.x; i < c1; i += blockDim.x) {
            const float x = src[i];
            buf[i - c0] = (x != x) ? 0.0f : x;
            mine += (x == x);
        }
        atomicAdd(&valid[v], mine);
        __syncthreads();
        // numpy's pairwise sum (np.nanmean, ray_utils.py:332): leaves in parallel, then the tree
        if (n_leaves >= 0)
            for (int k = threadIdx.x; k < n_leaves; k += blockDim.x) leaf_sum[k] = np_leaf_sum(buf + leaf_off[k], leaf_cnt[k]);
        __syncthreads();
        if (threadIdx.x == 0) {
            const float sum = n_leaves >= 0 ? np_pairwise_combine(leaf_sum, m, st_a, st_b, st_v) : np_pairwise_sum(buf, m);
            means[v] = valid[v] ? (float)((double)sum / (double)valid[v]) : __int_as_float(0x7fc00000);
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

// one full torch-order feature vector (encode_inputs + embedders, core/raycasters.py:476-555 and
// cutoff_embedder.py:111-174) of point p and ray direction d under the joint transforms S (NJ x 16)
__device__ void encode_row(const ModelDev& M, const float* __restrict__ skts, float px, float py, float pz, float dx,
                           float dy, float dz, float* __restrict__ f) {
    const int nj = M.nj, nv = 1 + 2 * M.mr;
    const int cx = nj * nv + 3 * nj;
    for (int j = 0; j < nj; ++j) {
        float S[12];
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 4; ++c) S[4 * r + c] = skts[j * 16 + 4 * r + c];
        float qx, qy, qz;
        joint_local(S, px, py, pz, qx, qy, qz);
        const float dist = norm3(qx, qy, qz);
        const float dn = fmaxf(dist, 1e-12f);
        const float w = M.use_cutoff ? cutoff_w(M.tau, dist, M.cutoff[j]) : 1.0f;
        float u, uf;
        kp_inputs(M.cut_to, M.shift_in, dist, M.cutoff[j], u, uf);
        f[j] = (M.use_cutoff && M.cutoff_inputs) ? u * w : u;
        for (int fi = 0; fi < M.mr; ++fi) {
            float s, c;
            sincosf(uf * (float)(1 << fi), &s, &c);
            f[(1 + 2 * fi) * nj + j] = s * w;
            f[(2 + 2 * fi) * nj + j] = c * w;
        }
        // bone directions, times w_b under --cutoff_bones (bone CutoffEmbedder, multires_bones 0)
        const float wb = M.bone_cut ? cutoff_w(M.tau_b, dist, M.cutoff_b[j]) : 1.0f;
        f[nj * nv + 3 * j + 0] = M.bone_cut ? (qx / dn) * wb : qx / dn;
        f[nj * nv + 3 * j + 1] = M.bone_cut ? (qy / dn) * wb : qy / dn;
        f[nj * nv + 3 * j + 2] = M.bone_cut ? (qz / dn) * wb : qz / dn;
        float ex, ey, ez;
        joint_rot(S, dx, dy, dz, ex, ey, ez);
        const float en = M.view_raw ? 1.0f : fmaxf(norm3(ex, ey, ez), 1e-12f);  // (world: R_j d itself)
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

// full torch-order feature vectors, one thread per point
__global__ void encode_points_kernel(ModelDev M, const float* __restrict__ skts, const float* __restrict__ pts,
                                     const float* __restrict__ dirs, int64_t n, float* __restrict__ feat) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int F = M.nj * (1 + 2 * M.mr) + 3 * M.nj + 3 * M.nj * (1 + 2 * M.mrv);
    encode_row(M, skts, pts[3 * i], pts[3 * i + 1], pts[3 * i + 2], dirs[3 * i], dirs[3 * i + 1], dirs[3 * i + 2],
               feat + i * F);
}

