// anerf_stages.hpp — per-ray stages: view factor G, compositing (raw2outputs), importance sampling + merge, bias staging.
// Part of the single translation unit anerf_render.hip (included there, in order).
#pragma once

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
    const int kfw0 = M.cutoff_inputs ? 0 : 1;
    // Per-ray live view windows (ray slot words 12..15, a bit per joint).  w'_j = 1 - sigmoid(tau'
    // (d - c'_j)) is exactly 0 at a sample with d^2 >= live_thr2(tau', c'_j) (the margins of
    // live_thr2); the samples of a ray lie on the segment o + z d, z in [near, far], so a joint whose
    // closest approach to the segment is beyond that bound (+0.1 % for the rounding of the samples'
    // points and transforms) has w'_j == 0 at every sample: its G column and its k-step of the view
    // layer's direction part only ever add exact zeros and are skipped (bit-identical results).
    // Only when every direction term is windowed (the usual flags); otherwise every joint is live.
    const bool cull = M.cutoff_viewdir && kfw0 == 0;
    for (int i = tid; i < nr * 4; i += blockDim.x)
        reinterpret_cast<unsigned*>(lds + P.ray + 16 * (i >> 2))[12 + (i & 3)] = cull ? 0u : 0xffffffffu;
    __syncthreads();
    if (cull)
        for (int idx = tid; idx < nr * nj; idx += blockDim.x) {
            const int r = idx / nj, j = idx % nj;
            const float* ray = lds + P.ray + 16 * r;
            const float* S = lds + P.sk + P.sk_stride * r + 12 * j;
            float ax, ay, az, bx, by, bz;
            joint_local(S, ray[0], ray[1], ray[2], ax, ay, az);
            joint_rot(S, ray[3], ray[4], ray[5], bx, by, bz);
            const float nearv = ray[7], farv = ray[8];
            const float bb = fmaf(bz, bz, fmaf(by, by, bx * bx));
            float t = bb > 0.0f ? -fmaf(az, bz, fmaf(ay, by, ax * bx)) / bb : nearv;
            t = fminf(fmaxf(t, nearv), farv);
            const float qx = fmaf(t, bx, ax), qy = fmaf(t, by, ay), qz = fmaf(t, bz, az);
            const float d2 = fmaf(qz, qz, fmaf(qy, qy, qx * qx));
            const float thr = live_thr2(M.tau_v, lds[P.cut + nj + j]);
            // (NaN near / far / transforms: live)
            const bool live = !(nearv <= farv) || !(d2 >= thr * 1.001f);
            if (live) atomicOr(reinterpret_cast<unsigned*>(lds + P.ray + 16 * r) + 12 + (j >> 5), 1u << (j & 31));
        }
    __syncthreads();
    // the union over the workgroup's rays: G columns are computed (and trig rows filled) for it
    uint64_t U0 = 0, U1 = 0;
    for (int r = 0; r < nr; ++r) {
        const unsigned* w = reinterpret_cast<const unsigned*>(lds + P.ray + 16 * r) + 12;
        U0 |= (uint64_t)w[0] | ((uint64_t)w[1] << 32);
        U1 |= (uint64_t)w[2] | ((uint64_t)w[3] << 32);
    }
    U0 = uniform64(U0);
    U1 = uniform64(U1);
    auto live_col = [&](int c) { return ((c < 64 ? U0 >> c : U1 >> (c - 64)) & 1ull) != 0; };
    // trig table Tt[j][k*3 + c] (27 values, padded to 28) of the normalised joint-frame ray
    // directions, one (ray, joint, coordinate) per thread
    constexpr int TP = (KC + 3) & ~3;
    for (int idx = tid; idx < nr * nj * 3; idx += blockDim.x) {
        const int r = idx / (nj * 3), j = (idx / 3) % nj, c = idx % 3;
        if (!live_col(j)) continue;
        const float* ray = lds + P.ray + 16 * r;
        const float* S = lds + P.sk + P.sk_stride * r + 12 * j;
        float ex, ey, ez;
        joint_rot(S, ray[3], ray[4], ray[5], ex, ey, ez);
        const float en = M.view_raw ? 1.0f : fmaxf(norm3(ex, ey, ez), 1e-12f);  // (world: R_j d itself)
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
                const f32x4 x = bload4_g(rs, (col * WH + nn) * TP * 4 + q * 16, 0);
                dst[4 * q] = x[0], dst[4 * q + 1] = x[1], dst[4 * q + 2] = x[2], dst[4 * q + 3] = x[3];
            }
        };
        // this thread's columns c = part (mod NPART): dead ones (for every ray) are zeroed, live
        // ones computed, the next live column's weights loaded under the current one
        for (int cz = part; cz < nj; cz += NPART)
            if (!live_col(cz))
                for (int r = 0; r < nr; ++r) lds[P.g + P.g_stride * r + cz * WH + nn] = 0.0f;
        auto next_col = [&](int c) {
            while (c < nj && !live_col(c)) c += NPART;
            return c;
        };
        int c = next_col(part);
        if (c < nj) load_col(wc, c);
        for (; c < nj;) {
            const int cn = next_col(c + NPART);
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
            c = cn;
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
            const float a = alpha_of(density_act(M, raw[4 * i + 3] / M.B) * dist);
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
// u: the I uniform samples of this ray (training, det=False: torch.rand), or NULL for the
// deterministic linspace of eval.
// single_net (is_only, ray_utils.py:270-277): the weights are 0.5 (max(w_l, w_k) + max(w_k, w_u)) + 0.01
// instead of w_k; src (optional) receives sorted_idx (src[rank] = index into cat([z, z_is])) and
// zis (optional) the I new samples in sample order.
__device__ __forceinline__ float torch_maximum(float a, float b) { return (a != a || a > b) ? a : b; }

__device__ void importance(const float* zc, const float* w, int S, int I, float* zf, float* scr2, bool active,
                           int lane, const float* u_rand = nullptr, bool is_only = false, int* src = nullptr,
                           float* zis = nullptr) {
    const int nb = S - 1;  // bins = mids
    float* mids = scr2;
    float* wp = scr2 + nb;
    float* cdf = scr2 + 2 * nb;
    float* zall = scr2 + 3 * nb + 1;  // S + I unsorted
    if (active) {
        for (int i = lane; i < nb; i += 64) mids[i] = 0.5f * (zc[i + 1] + zc[i]);
        if (is_only) {
            for (int i = lane; i < nb - 1; i += 64) {
                const float t = torch_maximum(w[i], w[i + 1]) + torch_maximum(w[i + 1], w[i + 2]);
                wp[i] = (0.5f * t + 0.01f) + 1e-5f;
            }
        } else {
            for (int i = lane; i < nb - 1; i += 64) wp[i] = w[i + 1] + 1e-5f;
        }
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
            const float u = u_rand ? u_rand[k] : torch_linspace01(k, I);
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
            const float zk = bb + t * (ba - bb);
            zall[S + k] = zk;
            if (zis) zis[k] = zk;
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
                if (src) src[rank] = e;
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
                if (src) src[rank] = e;
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

