"""Benchmark: rays/s of the A-NeRF render path (BASELINE.json configs 3 and 5).

A "step" renders one synthetic frame (64 coarse + 128 importance samples, 24-joint skeleton,
8x256 MLP): ray generation from the frame's bounding-cylinder pixel list, the fused render
kernel, and frame composition — all on the GPU with inputs resident in HBM (the pixel list of
kp_to_valid_rays is computed on the host before the timed region).

* Plain `python bench.py` (no launcher): config 3, one 512x512 frame per step on one GPU.
* Under torch.distributed.run (any world size, 1 included; default `--shard pixels --res 1024`):
  config 5, the north star's layout — ONE 1024x1024 frame per step whose ray list is cut into whole
  4096-ray chunks across the ranks (each rank generates and renders only its range), then one RCCL
  all-gather of the 20 B/ray outputs assembles the frame on every rank (strong scaling).  A 1 -> 8
  sweep under the launcher is therefore one workload.  `--shard frames` keeps the weak-scaling
  layout (one independent frame per rank, no collective).
Rank 0 reports the job's rays / max-over-ranks time, and per-rank render / all-gather / compose ms.

Headline precision: fp16x4 (operands scaled by exact powers of two and split into two fp16 parts each,
x = x0 + x1 and W = W0 + W1 within 2^-23 of |x|, |W|; all four products, fp32 accumulation: each product
within ~2^-22 of |x W|, the bound of bf16x6's dropped terms, so fp32-accurate like bf16x6 with four
16-bit MFMAs per 16 k instead of six).  The other modes — bf16x6 (the round-3 headline), fp16x3, fp32,
bf16x3 — are timed on the same frame (`other_precisions`).

Extra JSON fields:
  roofline      dominant kernel (render_kernel, coarse + fine launch) against the peak of the MFMA
                pipe its MLP runs on: `achieved` = the reference's algorithmic FLOPs (SURVEY §8(d):
                1,723,648 per sample x 256 samples per ray) / the launches' time (HIP events on the
                launch stream), `frac` = achieved / peak; `frac_executed` prices the MFMA
                instructions the launches actually issue (kernel-side tally, agrees with PMC
                SQ_INSTS_MFMA) against the instruction-mix-weighted peak — it differs because the
                kernel skips exact-zero cutoff-window k-steps and fuses feature_linear (fewer FLOPs)
                and splits operands for fp32 accuracy (more FLOPs); the peaks assume 2.4 GHz, and
                `mfma_busy_at_profile_clock` rescales frac_executed to the effective clock of the
                committed PMC summary (GRBM_GUI_ACTIVE / kernel time; the chip is power-limited here)
  parity        every N: the oracle's outputs for an evenly spaced sample of the frame's rays (near /
                far from the whole frame's chunks) against the GPU's (at N > 1 the all-gathered frame);
                exits non-zero above 1e-4
  cpu_baseline  the C oracle (oracle/anerf_oracle.c, OpenMP on every CPU of the process's affinity
                mask) on that bounded sample, rank 0 at N = 1
"""
import argparse
import glob
import importlib
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

BASELINE = json.load(open(os.path.join(REPO, "BASELINE.json")))
FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md, FP32 matrix (1024 SIMDs x 64 FLOP/clk x 2.4 GHz)
BF16_MFMA_PEAK_TFLOPS = 2516.6  # MI355X_MICROARCH.md, BF16 dense (1024 SIMDs x 1024 FLOP/clk x 2.4 GHz)
DTYPE = {
    "fp32": "fp32 (v_mfma_f32_32x32x2_f32)",
    "bf16x6": "fp32-accurate split bf16: hidden, view and bone-direction layers with x = x0+x1+x2 exactly (24 bits), "
              "W = W0+W1+W2, the six bf16 MFMA products with i + j <= 2 (each dropped term below 2^-23 of |x W|), fp32 "
              "accumulate; encoder, windowed layer-0 part, heads, compositing fp32",
    "fp16x3": "22-bit operands: split fp16 after exact power-of-two scaling (x = x0+x1 within 2^-23 |x|, W = W0+W1), "
              "three fp16 MFMA products (x1 W1, ~2^-22 of |x W|, dropped), fp32 accumulate; the bone-direction and "
              "windowed layer-0 / skip-layer parts the same way in fixed power-of-two units of their bounded features "
              "at widths 128/256 when the windows bound them (bf16x6 otherwise, fp32 at 64); encoder, heads, "
              "compositing fp32",
    "fp16x4": "fp32-accurate split fp16: hidden and view layers after exact power-of-two scaling, x = x0+x1 and "
              "W = W0+W1 (remainders within 2^-23 of |x|, |W|), the four fp16 MFMA products x_i W_j (dropped: the "
              "remainders' ~2^-22 of |x W|, the bound of bf16x6's dropped terms), fp32 accumulate; the bone-direction "
              "and windowed layer-0 / skip-layer parts the same way in fixed power-of-two units of their bounded "
              "features at widths 128/256 (round 5; bf16x6 when the windows do not bound them); encoder, heads, "
              "compositing fp32",
    "bf16x3": "16-bit operands: split bf16 (x = hi+lo, W = hi+lo, three bf16 MFMA products), fp32 accumulate; "
              "fp32 elsewhere",
}
PRODUCTS = {"fp32": 1, "bf16x6": 6, "fp16x4": 4, "fp16x3": 3, "bf16x3": 3}
FLOP_F32_MFMA = 32 * 32 * 2 * 2     # v_mfma_f32_32x32x2_f32
FLOP_BF16_MFMA = 32 * 32 * 16 * 2   # v_mfma_f32_32x32x16_bf16
TILE = 256  # pixels mode: rays per tile of the round-robin split (distributed.tile_rows)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--res", type=int, default=None, help="frame size (default 512; 1024 in pixels mode at N > 1)")
    ap.add_argument("--tau", type=float, default=79.6, help="cutoff temperature of the synthetic checkpoint")
    ap.add_argument("--joints", type=int, default=24)
    ap.add_argument("--samples", type=int, default=64)
    ap.add_argument("--importance", type=int, default=128)
    ap.add_argument("--cpu-rays", type=int, default=20000, help="rays in the CPU-baseline sample")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline (and its parity check)")
    ap.add_argument("--no-tau20", action="store_true", help="skip the tau = 20 kernel timing")
    ap.add_argument("--no-balance", action="store_true", help="skip the 8-shard balance projection (N = 1)")
    ap.add_argument("--other-configs", default=",".join(OTHER_CONFIGS),
                    help="N = 1: the other 1-GPU configurations measured in the same run ('' = none)")
    ap.add_argument("--no-train", action="store_true",
                    help="skip the training-step leg (SURVEY §8(f) row 2: tools/train_bench.py, N = 1 only)")
    ap.add_argument("--shard", default=None, choices=["frames", "pixels"],
                    help="frames: one frame per rank (weak scaling, no collective); pixels: ONE frame per step "
                         "split into ray-balanced ranges across the ranks (near / far from the whole frame's "
                         "4096-ray chunks) + an RCCL all-gather of the ray outputs (strong scaling, BASELINE "
                         "config 5's layout; the default under torch.distributed.run)")
    ap.add_argument("--also", default="bf16x6,fp16x3,fp32,bf16x3",
                    help="other precision modes timed on the same frame afterwards (rank 0, N=1; '' = none)")
    ap.add_argument("--no-tally", action="store_true",
                    help="skip the untimed MFMA-tally calls (count_mfma) so that every render_kernel dispatch of the "
                         "run is a warmup or timed step: the PMC passes of tools/gpu_pmc.sh (frac_executed null)")
    ap.add_argument("--lib", default=None,
                    help="A/B tooling: an experiment build of libanerf_hip.so (default: the in-tree library; "
                         "ANERF_LIB_PATH is honoured by this harness, never by the package)")
    ap.add_argument("--precision", default="fp16x4", choices=["fp32", "bf16x6", "fp16x4", "fp16x3", "bf16x3"],
                    help="MLP arithmetic (include/anerf.h ANERF_PREC_*)")
    return ap.parse_args()


def traffic_from_profiles(precision):
    """(HBM bytes per render call, file, effective clock GHz) of render_kernel from the newest committed rocprofv3 --pmc
    summary of this precision mode (profiles/*pmc*.json, field "precision"; untagged files are fp32).
    Copied from that profile, not measured by this run (PMC passes need their own rocprofv3 runs)."""
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", "*pmc*.json")), reverse=True):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        if d.get("precision", "fp32") == precision and "render_kernel_hbm_bytes_per_launch" in d:
            return d["render_kernel_hbm_bytes_per_launch"], os.path.relpath(f, REPO), d.get("effective_clock_GHz")
    return None, None, None


def _config_name(H, S, I, nj):
    """BASELINE.json's config numbering; other shapes are 'custom'."""
    known = {(256, 64, 0, 24): "config2", (512, 64, 128, 24): "config3", (512, 64, 128, 65): "config4",
             (1024, 64, 128, 24): "config5"}
    return known.get((H, S, I, nj), "custom")


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def kernel_time(rc, rb, S, I, skts, cyl, reps=4):
    """Mean HIP-event time (ms) of render_rays on rb (first of reps+1 calls discarded) and the
    launches' MFMA tally (one extra counted call)."""
    n = rb.shape[0]
    ts = []
    for it in range(reps + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        rc.render_rays(rb, S, skts=skts.expand(n, -1, -1, -1), cyls=cyl.expand(n, -1), N_importance=I, chunk=4096,
                       ret_alpha=False)
        e1.record()
        torch.cuda.synchronize()
        if it:
            ts.append(e0.elapsed_time(e1))
    rc.render_rays(rb, S, skts=skts.expand(n, -1, -1, -1), cyls=cyl.expand(n, -1), N_importance=I, chunk=4096,
                   ret_alpha=False, count_mfma=True)
    torch.cuda.synchronize()
    return float(np.mean(ts)), tuple(int(v) for v in rc.last_mfma.tolist())


def shard_projection(rc, rb_nf, S, I, skts, cyl, world=8, reps=2):
    """The pixel-sharded step's balance projected on this one GPU: the frame's rays (near / far already
    filled over the whole frame) cut into `world` shards by the tiled split bench.py runs under the
    launcher (distributed.tile_rows) and by contiguous equal-ray ranges, each shard rendered alone
    (best of `reps` HIP-event timings).  An N-rank step waits for its slowest shard: max / mean."""
    dmod = importlib.import_module("a-nerf_amd.distributed")
    n = rb_nf.shape[0]
    splits = {"tiles": [dmod.tile_rows(n, world, r, TILE) for r in range(world)],
              "ranges": [torch.arange(s0, s1) for s0, s1 in dmod.ray_ranges(n, world)]}
    res = {}
    for name, parts in splits.items():
        ms = []
        for rows in parts:
            sub = rb_nf.index_select(0, rows.to(rb_nf.device))
            m = sub.shape[0]
            best = None
            for _ in range(reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                rc.render_rays(sub, S, skts=skts.expand(m, -1, -1, -1), cyls=cyl.expand(m, -1), N_importance=I,
                               chunk=4096, ret_alpha=False, near_far_given=True)
                e1.record()
                torch.cuda.synchronize()
                t = e0.elapsed_time(e1)
                best = t if best is None else min(best, t)
            ms.append(best)
        res[name] = {"shard_ms": [round(x, 3) for x in ms], "max_over_mean": round(max(ms) * len(ms) / sum(ms), 4)}
    return {"world": world, "tile": TILE, "frame_rays": n, "split_run_under_the_launcher": "tiles", **res}


# Every other 1-GPU configuration of BASELINE.json, and the reference's shipped render configuration
# (configs/mixamo/mixamo.txt:28-38,55: 8x256, 64 + 16 samples, opt_framecode), measured in the headline
# precision on its own frame: kernel rays/s, frac, frac_executed and a 2,000-ray oracle parity check.
OTHER_CONFIGS = {
    "config2": dict(res=256, S=64, I=0, joints=24, seed=13, desc="256x256, 64 coarse samples, 24-joint, 8x256"),
    "config4": dict(res=512, S=64, I=128, joints=65, seed=14,
                    desc="512x512, 64+128 samples, 65-joint synthetic skeleton (LDS-pressure case), 8x256"),
    "mixamo_shipped": dict(res=512, S=64, I=16, joints=24, seed=15, framecode=True, cam=2,
                           desc="configs/mixamo/mixamo.txt: 512x512, 64+16 samples, 24-joint, 8x256, "
                                "opt_framecode (5 codes, camera 2)"),
}


def other_config_leg(a, name, spec, dev, n_parity=2000):
    """One OTHER_CONFIGS entry: its own synthetic scene and seeded checkpoint, the whole bounding box's rays,
    render kernel time (kernel_time), the MFMA tally's executed fraction, and the C oracle on n_parity
    evenly spaced rays (near / far of the whole frame's chunks) at 1e-4 (near-empty disp: + the
    reference's measured spread, oracle.h12_spread)."""
    anerf = importlib.import_module("a-nerf_amd")
    syn = importlib.import_module("a-nerf_amd.synthetic")
    _lib = importlib.import_module("a-nerf_amd._lib")
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle
    H, S, I, nj = spec["res"], spec["S"], spec["I"], spec["joints"]
    fc = bool(spec.get("framecode"))
    cfg = anerf.RenderConfig(n_joints=nj, N_samples=S, N_importance=I, precision=a.precision, opt_framecode=fc,
                             n_framecodes=5 if fc else 0).validate()
    ck = syn.make_checkpoint(spec["seed"], n_joints=nj, D=8, W=256, fine=I > 0, tau=a.tau, use_framecode=fc,
                             n_framecodes=5 if fc else 0)
    sc = syn.make_scene(n_joints=nj, H=H, W=H, seed=spec["seed"])
    rc = anerf.RayCaster(cfg, ck, device=dev.index or 0)
    idxs, cyls, boxes = anerf.rays.valid_pixels(sc["c2ws"], H, H, sc["focal"], kps=sc["kps"], ext_scale=0.001)
    (x0, y0), (x1, y1) = (int(v) for v in boxes[0][0]), (int(v) for v in boxes[0][1])
    n = (x1 - x0) * (y1 - y0)
    c2w_np = np.ascontiguousarray(sc["c2ws"][0][:3, :4])
    c2w = torch.from_numpy(c2w_np).to(dev)
    rb = torch.empty(n, 11, device=dev)
    _lib.check(_lib.load().anerf_gen_rays_box(_lib.ptr(c2w), H, H, sc["focal"], sc["focal"], 0.0, 0.0, 0, x0, y0, x1,
                                              y1, 0.0, 1.0, _lib.ptr(rb), _lib.stream_handle(dev)), "gen_rays_box")
    skts = torch.from_numpy(sc["skts"][0:1]).to(dev)
    cyl = torch.from_numpy(cyls[0:1]).to(dev)
    cams = torch.full((n,), float(spec.get("cam", 0)), device=dev) if fc else None
    ts = []
    for it in range(4):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        out = rc.render_rays(rb, S, skts=skts.expand(n, -1, -1, -1), cyls=cyl.expand(n, -1), cams=cams,
                             N_importance=I, chunk=4096, ret_alpha=False)
        e1.record()
        torch.cuda.synchronize()
        if it:
            ts.append(e0.elapsed_time(e1))
    ms = float(np.mean(ts))
    rc.render_rays(rb, S, skts=skts.expand(n, -1, -1, -1), cyls=cyl.expand(n, -1), cams=cams, N_importance=I,
                   chunk=4096, ret_alpha=False, count_mfma=True)
    torch.cuda.synchronize()
    nf, nb = (int(v) for v in rc.last_mfma.tolist())
    ppeak, pflop = mix_peak(nf, nb)
    flop_ray = anerf.flops_per_sample(cfg) * anerf.samples_per_ray(cfg)
    # parity: the oracle on evenly spaced rays of this frame
    om = oracle.OracleModel(cfg, ck)
    rb_h = oracle.gen_rays(sc["c2ws"][0][:3, :4], H, H, sc["focal"], idxs[0])
    near_f, far_f, _, _ = om.near_far(rb_h, cyls[0:1], chunk=4096)
    sel = np.linspace(0, n - 1, min(n_parity, n)).astype(np.int64)
    ref = om.render_rays(rb_h[sel], sc["skts"][0], cyls[0:1], chunk=4096, nthreads=cpu_threads(), near=near_f[sel],
                         far=far_f[sel], cams=np.full(len(sel), float(spec.get("cam", 0)), np.float32) if fc else None)
    sel_d = torch.from_numpy(sel).to(dev)
    keys = ["rgb_map", "disp_map", "acc_map"] + (["rgb0", "disp0", "acc0"] if I > 0 else [])
    errs, ne_n, ne_err = {}, 0, 0.0
    for k in keys:
        d = np.abs(out[k].index_select(0, sel_d).cpu().numpy().astype(np.float64) - ref[k]).reshape(len(sel), -1).max(-1)
        acc_k = ref["acc0" if k.endswith("0") else "acc_map"]
        empty = ((acc_k > 0) & (acc_k < 2.0 ** -20)) if k.startswith("disp") else np.zeros(len(sel), bool)
        errs[k] = float(f"{d[~empty].max():.3e}")
        if empty.any():
            ne_n, ne_err = max(ne_n, int(empty.sum())), max(ne_err, float(d[empty].max()))
    ne_tol = 1e-4 + oracle.h12_spread()["float64"]
    ok = max(errs.values()) <= 1e-4 and ne_err <= ne_tol
    return {"workload": spec["desc"], "rays_per_frame": n, "tau": a.tau, "precision": a.precision,
            "kernel_ms": round(ms, 3), "rays_per_s_kernel": round(n / (ms * 1e-3), 1),
            "reference_flop_per_ray": flop_ray,
            "frac": round(flop_ray * n / (ms * 1e-3) / 1e12 / pipe_peak(a.precision), 4),
            "frac_executed": round(pflop / (ms * 1e-3) / 1e12 / ppeak, 4),
            "parity": {"rays": int(len(sel)), "max_abs_err": errs, "near_empty_rays": ne_n,
                       "near_empty_disp_max_abs_err": float(f"{ne_err:.3e}"), "ok": bool(ok),
                       "against": "C oracle, near/far from the whole frame's 4096-ray chunks"}}


def mix_peak(n_f32, n_bf16):
    """Instruction-mix-weighted MFMA peak (TFLOP/s) and the executed FLOPs of a tally."""
    flop = n_f32 * FLOP_F32_MFMA + n_bf16 * FLOP_BF16_MFMA
    t = n_f32 * FLOP_F32_MFMA / (FP32_MFMA_PEAK_TFLOPS * 1e12) + n_bf16 * FLOP_BF16_MFMA / (BF16_MFMA_PEAK_TFLOPS * 1e12)
    return flop / t / 1e12, flop


def pipe_peak(precision):
    """Peak of the MFMA pipe the precision mode's MLP runs on (the algorithmic roofline's peak)."""
    return FP32_MFMA_PEAK_TFLOPS if precision == "fp32" else BF16_MFMA_PEAK_TFLOPS


def cpu_threads():
    """Every CPU of this process's affinity mask (what the CPU baseline runs on)."""
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def parity_leg(a, cfg, ck, sc, cyls, idx, c2w_np, H, W, out, n, dev, want_cpu):
    """The C oracle on an evenly spaced sample of the frame's rays (rays and the whole frame's chunked
    near / far generated on the host by the oracle itself; the oracle's gen_rays is bit-exact with
    anerf_gen_rays, tests/test_gpu_parity.py) against the GPU's outputs `out` (ray order).  Returns
    (parity, cpu_baseline or None)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle
    cores = cpu_threads()
    om = oracle.OracleModel(cfg, ck)
    rb_h = oracle.gen_rays(c2w_np, H, W, sc["focal"], idx)
    near_f, far_f, _, _ = om.near_far(rb_h, cyls[0:1], chunk=4096)  # the whole frame's chunk NaN fill
    sel = np.linspace(0, n - 1, min(a.cpu_rays, n)).astype(np.int64)
    # (timed as two interleaved halves: the line reports both rates and their spread)
    halves = [np.arange(0, len(sel), 2), np.arange(1, len(sel), 2)]
    parts, dts = [], []
    for h in halves:
        t1 = time.perf_counter()
        parts.append(om.render_rays(rb_h[sel[h]], sc["skts"][0], cyls[0:1], chunk=4096, nthreads=cores,
                                    near=near_f[sel[h]], far=far_f[sel[h]]))
        dts.append(time.perf_counter() - t1)
    ref = {}
    for k in ("rgb_map", "disp_map", "acc_map"):
        v = np.empty((len(sel),) + parts[0][k].shape[1:], parts[0][k].dtype)
        for h, pr in zip(halves, parts):
            v[h] = pr[k]
        ref[k] = v
    dt = sum(dts)
    cpu = None
    if want_cpu:
        rates = [len(h) / t for h, t in zip(halves, dts)]
        cpu = {"value": round(len(sel) / dt, 2), "unit": "rays/s", "cores": cores, "kind": "port",
               "cpu_model": cpu_model(), "cpus_in_affinity_mask": cores,
               "samples_rays_per_s": [round(r, 2) for r in rates],
               "spread": round((max(rates) - min(rates)) / (len(sel) / dt), 4),
               "sample": f"{len(sel)} rays evenly spaced over the frame's {n} bbox rays, C oracle "
                         f"(oracle/anerf_oracle.c, OpenMP, {cores} threads = every CPU of the process's affinity "
                         f"mask), {dt:.1f} s wall, timed as two interleaved halves (samples_rays_per_s; the rate "
                         f"moves ~30 % between boxes of the same model, profiles r04k vs BENCH_r04)"}
    sel_d = torch.from_numpy(sel).to(dev)
    diff = {k: np.abs(out[k].index_select(0, sel_d).cpu().numpy().astype(np.float64) - ref[k].astype(np.float64))
            for k in ("rgb_map", "disp_map", "acc_map")}
    # H12: on a near-empty ray (0 < acc < 2^-20) disp = 1 / max(1e-10, depth / acc) is a ratio
    # of a few 2^-24 alpha quanta; the reference's own float32 disp on such rays sits up to 1.92e-4 from
    # its float64 value (tests/golden/h12_spread_c5.npz, oracle.h12_spread).  Such rays are counted and
    # their disp held to 1e-4 + that measured spread; every other output of every ray to 1e-4
    empty = (ref["acc_map"] > 0) & (ref["acc_map"] < 2.0 ** -20)
    errs = {k: float(v[~empty].max() if k == "disp_map" and empty.any() and (~empty).any() else v.max())
            for k, v in diff.items()}
    ne_err = float(diff["disp_map"][empty].max()) if empty.any() else 0.0
    ne_tol = 1e-4 + oracle.h12_spread()["float64"]
    ok = max(errs.values()) <= 1e-4 and ne_err <= ne_tol
    parity = {"rays": int(len(sel)), "max_abs_err": {k: float(f"{v:.3e}") for k, v in errs.items()},
              "near_empty_rays": int(empty.sum()), "near_empty_disp_max_abs_err": float(f"{ne_err:.3e}"),
              "tol": 1e-4, "near_empty_tol": {"disp": float(f"{ne_tol:.3e}"),
                                             "source": "1e-4 + the reference's own float32-vs-float64 disp spread on "
                                                       "near-empty rays (tests/golden/h12_spread_c5.npz)"},
              "ok": bool(ok),
              "against": "C oracle (pinned to the reference's golden fixtures) on the same rays, near/far "
                         "from the whole frame's 4096-ray chunks"}
    return parity, cpu


def main():
    a = parse()
    # stdout carries exactly one line, the result: everything else the process or its libraries
    # print (RCCL's version banner at communicator set-up goes to fd 1) is sent to stderr
    out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # under torch.distributed.run every world size (1 included) takes the process-group path and, by
    # default, config 5's pixel sharding, so a 1 -> 8 sweep measures one workload; a plain
    # `python bench.py` is config 3 on one GPU
    launched = "WORLD_SIZE" in os.environ and "MASTER_ADDR" in os.environ
    dist = launched or world > 1
    shard = a.shard or ("pixels" if dist else "frames")
    pixels = shard == "pixels"
    if a.res is None:
        a.res = 1024 if (pixels and dist) else 512
    backend = None
    if dist:
        import torch.distributed as tdist
        torch.cuda.set_device(local)
        tdist.init_process_group("nccl")
        backend = tdist.get_backend()
    dev = torch.device(f"cuda:{local}")
    torch.cuda.set_device(dev)

    sys.path.insert(0, os.path.join(REPO, "tools"))
    importlib.import_module("_ablib").apply(a.lib)  # (A/B builds only; the default is the in-tree library)
    anerf = importlib.import_module("a-nerf_amd")
    syn = importlib.import_module("a-nerf_amd.synthetic")
    _lib = importlib.import_module("a-nerf_amd._lib")
    dmod = importlib.import_module("a-nerf_amd.distributed")
    near_far = importlib.import_module("a-nerf_amd.raycaster").near_far
    lib = _lib.load()

    H = W = a.res
    S, I = a.samples, a.importance
    cfg = anerf.RenderConfig(n_joints=a.joints, N_samples=S, N_importance=I, precision=a.precision).validate()
    ck = syn.make_checkpoint(13, n_joints=a.joints, D=8, W=256, fine=I > 0, tau=a.tau)
    sc = syn.make_scene(n_joints=a.joints, H=H, W=W, seed=13 if pixels else 13 + rank)
    rc = anerf.RayCaster(cfg, ck, device=local)
    idxs, cyls, boxes = anerf.rays.valid_pixels(sc["c2ws"], H, W, sc["focal"], kps=sc["kps"], ext_scale=0.001)
    (x0, y0), (x1, y1) = (int(v) for v in boxes[0][0]), (int(v) for v in boxes[0][1])
    n = (x1 - x0) * (y1 - y0)
    c2w_np = np.ascontiguousarray(sc["c2ws"][0][:3, :4])
    c2w = torch.from_numpy(c2w_np).to(dev)
    skts = torch.from_numpy(sc["skts"][0:1]).to(dev)
    cyl = torch.from_numpy(cyls[0:1]).to(dev)
    img = torch.empty(H * W, 3, device=dev)
    dimg = torch.empty(H * W, device=dev)
    aimg = torch.empty(H * W, device=dev)
    st = _lib.stream_handle(dev)
    ev = []
    sharded = pixels and dist
    # this rank's rays: pixels mode = the frame's ray list cut into 256-ray tiles dealt round-robin over
    # the ranks (distributed.tile_rows: per-ray cost follows the live joints, and contiguous ranges put
    # the torso's rays on a few ranks, 1.05x max/mean vs 1.002x, tools/shard_balance.py); every rank
    # generates the whole box's rays and fills near / far (cylinder + chunk NaN fill) over the whole
    # frame's chunks (0.1 ms), so its rays render exactly as in the whole frame (ANERF_FLAG_NEAR_FAR),
    # and renders its own tiles; otherwise the whole box
    rb_all = torch.empty(n, 11, device=dev)
    if sharded:
        rank_rows = [dmod.tile_rows(n, world, r, TILE) for r in range(world)]
        rows_mine = rank_rows[rank].to(dev)
        n_mine = int(rows_mine.shape[0])
        rb = torch.empty(max(n_mine, 1), 11, device=dev)[:n_mine]
        gather = dmod.ShardGather(n, 4096, world, dev, rank_rows=rank_rows)
    else:
        n_mine, rb = n, rb_all
    idx_all = torch.from_numpy(np.ascontiguousarray(idxs[0], np.int64)).to(dev)
    last = {}

    def render(r):
        m = r.shape[0]
        return rc.render_rays(r, S, skts=skts.expand(m, -1, -1, -1), cyls=cyl.expand(m, -1), N_importance=I,
                              chunk=4096, ret_alpha=False, near_far_given=sharded)

    def event():
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        return e

    def step(record):
        _lib.check(lib.anerf_gen_rays_box(_lib.ptr(c2w), H, W, sc["focal"], sc["focal"], 0.0, 0.0, 0, x0, y0, x1,
                                          y1, 0.0, 1.0, _lib.ptr(rb_all), st), "gen_rays_box")
        if sharded and n_mine:
            near_far(rb_all, cyl, chunk=4096, out=(rb_all[:, 6], rb_all[:, 7]))
            torch.index_select(rb_all, 0, rows_mine, out=rb)
        e0 = event()
        out = render(rb) if n_mine else None
        e1 = event()
        if sharded:  # one RCCL all-gather of (rgb, disp, acc), then every rank composes the frame
            out = gather(out)
            e2 = event()
            _lib.check(lib.anerf_compose(_lib.ptr(out["rgb_map"]), _lib.ptr(out["disp_map"]), _lib.ptr(out["acc_map"]),
                                         _lib.ptr(idx_all), n, None, 0, H * W, _lib.ptr(img), _lib.ptr(dimg),
                                         _lib.ptr(aimg), st), "compose")
        else:
            e2 = e1
            _lib.check(lib.anerf_compose_box(_lib.ptr(out["rgb_map"]), _lib.ptr(out["disp_map"]),
                                             _lib.ptr(out["acc_map"]), x0, y0, x1, y1, None, 0, H, W, _lib.ptr(img),
                                             _lib.ptr(dimg), _lib.ptr(aimg), st), "compose_box")
        e3 = event()
        if record:
            ev.append((e0, e1, e2, e3))
        last["out"] = out

    for _ in range(a.warmup):
        step(False)
    torch.cuda.synchronize()
    if dist:
        tdist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step(True)
    torch.cuda.synchronize()
    if dist:
        tdist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([e0.elapsed_time(e1) for e0, e1, _, _ in ev]))
    phase = torch.tensor([kern_ms, float(np.mean([e1.elapsed_time(e2) for _, e1, e2, _ in ev])),
                          float(np.mean([e2.elapsed_time(e3) for _, _, e2, e3 in ev])), float(n_mine)],
                         device=dev, dtype=torch.float64)
    rays_job = n * a.steps / (world if sharded else 1)  # pixels: the ranks share one frame per step
    per_rank = [phase.cpu().tolist()]
    if dist:
        t = torch.tensor([elapsed, float(rays_job)], device=dev, dtype=torch.float64)
        tmax = t[:1].clone()
        tdist.all_reduce(tmax, op=tdist.ReduceOp.MAX)
        tdist.all_reduce(t[1:], op=tdist.ReduceOp.SUM)
        elapsed, rays_job = float(tmax.item()), float(t[1].item())
        allp = torch.empty(world, 4, device=dev, dtype=torch.float64)
        tdist.all_gather_into_tensor(allp, phase)
        per_rank = allp.cpu().tolist()

    # the launches' MFMA work (kernel-side tally of one extra, untimed call over this rank's rays) and
    # the work an exact fp32 implementation must do after exact-zero window skipping: the fp32 mode's
    # tally of the same rays (v_mfma_f32_32x32x2_f32, FLOP_F32_MFMA each)
    if a.no_tally:  # (PMC passes: no dispatch outside the timed steps)
        n_f32 = n_bf16 = req_f32 = None
    else:
        rc.render_rays(rb, S, skts=skts.expand(n_mine, -1, -1, -1), cyls=cyl.expand(n_mine, -1), N_importance=I,
                       chunk=4096, ret_alpha=False, count_mfma=True, near_far_given=sharded)
        torch.cuda.synchronize()
        n_f32, n_bf16 = (int(v) for v in rc.last_mfma.tolist())
    if a.no_tally:
        pass
    elif a.precision == "fp32":
        req_f32 = n_f32
    else:
        rc32 = anerf.RayCaster(anerf.RenderConfig(n_joints=a.joints, N_samples=S, N_importance=I,
                                                  precision="fp32").validate(), ck, device=local)
        rc32.render_rays(rb, S, skts=skts.expand(n_mine, -1, -1, -1), cyls=cyl.expand(n_mine, -1), N_importance=I,
                         chunk=4096, ret_alpha=False, count_mfma=True, near_far_given=sharded)
        torch.cuda.synchronize()
        req_f32 = int(rc32.last_mfma[0].item())
        del rc32
    peak_exec, flop_exec = mix_peak(n_f32, n_bf16) if n_f32 is not None else (None, None)
    flop_ray = anerf.flops_per_sample(cfg) * anerf.samples_per_ray(cfg)  # SURVEY §8(d), reference work
    achieved_alg = flop_ray * n_mine / (kern_ms * 1e-3) / 1e12
    achieved_exec = flop_exec / (kern_ms * 1e-3) / 1e12 if flop_exec is not None else None
    achieved_req = req_f32 * FLOP_F32_MFMA / (kern_ms * 1e-3) / 1e12 if req_f32 is not None else None
    r4 = lambda x: round(x, 4) if x is not None else None  # noqa: E731
    peak = pipe_peak(a.precision)
    # the committed PMC summaries are of config 3's frame; other shapes report null
    traffic, traffic_src, prof_clock = (traffic_from_profiles(a.precision)
                                        if _config_name(H, S, I, a.joints) == "config3" else (None, None, None))

    # N = 1 extras on the same frame: the other precision modes, and this mode at tau = 20 (the untrained
    # value: wider cutoff windows, more live joints per block than tau = 79.6)
    others, tau20 = {}, None
    if rank == 0 and world == 1:
        for p in [x for x in a.also.split(",") if x and x != a.precision]:
            rcp = anerf.RayCaster(anerf.RenderConfig(n_joints=a.joints, N_samples=S, N_importance=I,
                                                     precision=p).validate(), ck, device=local)
            pms, (pf, pb) = kernel_time(rcp, rb, S, I, skts, cyl)
            ppeak, pflop = mix_peak(pf, pb)
            others[p] = {"rays_per_s_kernel": round(n_mine / (pms * 1e-3), 1), "kernel_ms": round(pms, 3),
                         "frac": round(flop_ray * n_mine / (pms * 1e-3) / 1e12 / pipe_peak(p), 4),
                         "frac_executed": round(pflop / (pms * 1e-3) / 1e12 / ppeak, 4),
                         "frac_required": (round(req_f32 * FLOP_F32_MFMA / (pms * 1e-3) / 1e12 / pipe_peak(p), 4)
                                           if req_f32 is not None else None),
                         "dtype": DTYPE[p]}
            del rcp
        if a.tau != 20.0 and not a.no_tau20:
            ck20 = syn.make_checkpoint(13, n_joints=a.joints, D=8, W=256, fine=I > 0, tau=20.0)
            rc20 = anerf.RayCaster(cfg, ck20, device=local)
            tms, (tf, tb) = kernel_time(rc20, rb, S, I, skts, cyl)
            tpeak, tflop = mix_peak(tf, tb)
            tau20 = {"tau": 20.0, "rays_per_s_kernel": round(n_mine / (tms * 1e-3), 1), "kernel_ms": round(tms, 3),
                     "frac": round(flop_ray * n_mine / (tms * 1e-3) / 1e12 / peak, 4),
                     "frac_executed": round(tflop / (tms * 1e-3) / 1e12 / tpeak, 4)}
            del rc20

    # N = 1: the 8-rank pixel split's balance, projected on this GPU (each shard of this frame alone)
    balance = None
    if rank == 0 and world == 1 and not a.no_balance:
        rb_nf = rb_all.clone()
        near_far(rb_nf, cyl, chunk=4096, out=(rb_nf[:, 6], rb_nf[:, 7]))
        balance = shard_projection(rc, rb_nf, S, I, skts, cyl)
        del rb_nf

    # N = 1: every other 1-GPU BASELINE configuration and the shipped mixamo configuration, same precision
    other_cfgs = {}
    if rank == 0 and world == 1:
        for name in [x for x in a.other_configs.split(",") if x]:
            other_cfgs[name] = other_config_leg(a, name, OTHER_CONFIGS[name], dev)
            torch.cuda.empty_cache()

    # N = 1: the training step of the same path at the reference's training configuration (§8(f) row 2)
    training = None
    if rank == 0 and world == 1 and not a.no_train:
        sys.path.insert(0, os.path.join(REPO, "tools"))
        import train_bench
        training = train_bench.measure(train_bench.parser().parse_args(["--steps", "10", "--warmup", "2"]), dev=dev)
        training.pop("data", None)
        # BASELINE config 4's 65-joint skeleton in the same step: the full view columns (the
        # view-window layout needs NJ W / 2 <= 4096 and 16-byte feature segments, train.view_windows_ok)
        t65 = train_bench.measure(train_bench.parser().parse_args(["--steps", "6", "--warmup", "2", "--joints", "65"]),
                                  dev=dev)
        training["joints65"] = {k: t65[k] for k in ("value", "ms_per_step", "joints", "view_layout")}
        torch.cuda.empty_cache()

    # parity at every N (rank 0: the all-gathered frame in pixels mode, its own frame in frames mode); the
    # CPU baseline at N = 1 only
    cpu, parity = None, None
    if rank == 0 and not a.no_cpu:
        parity, cpu = parity_leg(a, cfg, ck, sc, cyls, idxs[0], c2w_np, H, W, last["out"], n, dev, world == 1)

    if rank == 0:
        value = rays_job / elapsed
        workload = (f"{_config_name(H, S, I, a.joints)}: {H}x{W} frame, {S}+{I} samples, {a.joints}-joint, 8x256 MLP, "
                    + (f"one frame per step split over {world} GPU(s) in {TILE}-ray tiles dealt round-robin (near/far from the whole frame's 4096-ray chunks) + RCCL all-gather"
                       if sharded else "one frame per GPU per step"))
        ranks = [{"rank": r, "rays": int(p[3]), "render_ms": round(p[0], 3), "all_gather_ms": round(p[1], 3),
                  "compose_ms": round(p[2], 3)} for r, p in enumerate(per_rank)]
        line = {
            "metric": BASELINE["metric"], "value": round(value, 1), "unit": "rays/s", "n_gpus": world,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(1e3 * elapsed / a.steps, 3),
            "higher_is_better": True, "scaling": "strong" if sharded else "weak", "vs_baseline": None,
            "dtype": DTYPE[a.precision], "precision": a.precision,
            "data": "synthetic (seeded SMPL-24 pose + seeded 8x256 weights; no dataset/checkpoint offline)",
            "config": {"workload": workload, "rays_per_frame": n, "tau": a.tau,
                       "parallelism": f"{'pixel-shard' if sharded else 'frame-per-rank'} x{world}",
                       "n_ranks": world, "backend": backend},
            "per_rank": ranks,
            "roofline": {"bound": "mfma", "achieved": round(achieved_alg, 2), "peak": round(peak, 1),
                         "unit": "TFLOP/s", "frac": round(achieved_alg / peak, 4),
                         "traffic": traffic, "traffic_source": traffic_src,
                         "traffic_measured_in_this_run": False,
                         "traffic_note": "2 x FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md, HBM / rocprofv3): L2 "
                                         "fabric-side bytes, which count Infinity-Cache (L3) hits. The fp16 modes' "
                                         "per-net streamed weight set (two fp16 planes, 4 B per weight: hidden layers "
                                         "1.8 MB + the view and encoder-fed parts) fits an XCD's 4 MB L2; bf16x6's "
                                         "(three bf16 planes, 6 B per weight: 2.75 MB + the rest) is just over it, so "
                                         "its weight groups are re-read from the 256 MB L3 (5-5.6 GB per frame); the "
                                         "bytes a render call must move are unique_bytes_per_step + ~8 MB of weights",
                         "unique_bytes_per_step": int(n_mine * (4 * 11 + 4 * 10) + (n_mine * (S + I) * 4 * 2 if I > 0 else 0)),
                         "kernel_ms": round(kern_ms, 3),
                         "launches_per_step": 2 if I > 0 else 1,
                         "flop": "algorithmic: the reference's MLP FLOPs (SURVEY §8(d), reference_flop_per_ray x "
                                 "this rank's rays per step) / kernel_ms; peak = the MFMA pipe of this precision "
                                 "mode (BF16 dense 2516.6 TF for the split modes, FP32 matrix 157.3 TF for fp32); "
                                 "traffic = PMC HBM bytes per render call (both launches), copied from "
                                 "traffic_source (rocprofv3 --pmc passes run separately), not measured here",
                         "timing": "HIP events on the launch stream around anerf_render_rays: the coarse and the "
                                   "fine render_kernel launch (+ near/far, 0.2 %); rocprofv3's render_kernel "
                                   "average x launches_per_step agrees (profiles/)",
                         "achieved_executed": r4(achieved_exec), "peak_executed_mix": r4(peak_exec),
                         "frac_executed": r4(achieved_exec / peak_exec) if achieved_exec is not None else None,
                         # the peaks assume 2.4 GHz; the chip runs this load power-limited below that
                         # (GRBM_GUI_ACTIVE / kernel time in the same committed PMC summary as traffic)
                         "profile_clock_GHz": prof_clock,
                         "mfma_busy_at_profile_clock": (round(achieved_exec / peak_exec * 2.4 / prof_clock, 4)
                                                        if prof_clock and achieved_exec is not None else None),
                         "achieved_required": r4(achieved_req),
                         "frac_required": r4(achieved_req / peak) if achieved_req is not None else None,
                         "required": "the FLOPs an exact fp32 implementation must do after exact-zero cutoff-window "
                                     "skipping and the feature_linear fusion (the fp32 mode's MFMA tally of the same "
                                     "rays x 4096 FLOP) / kernel_ms / peak: why fp32's algorithmic frac exceeds 1",
                         "mfma_tally": "kernel-side tally of issued MFMA instructions (agrees with PMC SQ_INSTS_MFMA); "
                                       "mfma_bf16_per_step counts the 32x32x16 16-bit MFMAs (bf16 or f16, same rate)",
                         "mfma_f32_per_step": n_f32, "mfma_bf16_per_step": n_bf16,
                         "mfma_f32_required_per_step": req_f32,
                         "reference_flop_per_ray": flop_ray},
            "parity": parity,
            "tau20": tau20,
            "shard_balance_projection": balance,
            "other_configs": other_cfgs or None,
            "cpu_baseline": cpu,
            "other_precisions": others or None,
            "training": training,
        }
        print(json.dumps(line), file=out, flush=True)
    if dist:
        tdist.destroy_process_group()
    if parity is not None and not parity["ok"]:
        sys.exit(f"parity check failed: {parity}")
    bad = {k: v["parity"] for k, v in (other_cfgs or {}).items() if not v["parity"]["ok"]} if rank == 0 else {}
    if bad:
        sys.exit(f"parity check failed on other configs: {bad}")


if __name__ == "__main__":
    main()
