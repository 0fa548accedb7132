"""Benchmark: rays/s of the A-NeRF render path at BASELINE.json config 3.

A "step" renders one synthetic 512x512 frame (64 coarse + 128 importance samples, 24-joint
skeleton, 8x256 MLP): ray generation from the frame's bounding-cylinder pixel list, the fused
render kernel, and frame composition — all on the GPU with inputs resident in HBM (the
box of kp_to_valid_rays is computed on the host before the timed region; the pixels are
enumerated on the device).

Multi-GPU (launched by torch.distributed.run): each rank renders its own frame (a different
pose) per step — frames are independent, so there is no collective in the data path and
scaling is weak; rank 0 reports total rays / max-over-ranks time.

Extra JSON fields:
  roofline      dominant kernel (render_kernel) vs the FP32 MFMA peak, per-launch duration
                from HIP events on the launch stream; `achieved` counts the MFMA FLOPs the
                launch executes (exact device counter: the kernel skips MFMAs on inputs that
                the cutoff window makes exactly zero, so it executes fewer FLOPs than the
                reference's 1,723,648 per sample x 256 samples per ray);
                `reference_equivalent_tflops` prices the same launch at the reference's FLOPs
  cpu_baseline  the C oracle (oracle/anerf_oracle.c, OpenMP) on a bounded sample of the same
                frame's rays, rank 0 at N=1 only
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
    "fp32": "fp32",
    "bf16x6": "fp32-accurate split bf16 (hidden + view layers: x = x0+x1+x2, W = W0+W1+W2, six bf16 MFMA "
              "products per term, fp32 accumulate; encoder, layer 0, compositing fp32)",
    "bf16x3": "split bf16 (hidden layers: x = hi+lo, W = hi+lo, three bf16 MFMA products, fp32 accumulate; "
              "fp32 elsewhere)",
}
FLOP_F32_MFMA = 32 * 32 * 2 * 2     # v_mfma_f32_32x32x2_f32
FLOP_BF16_MFMA = 32 * 32 * 16 * 2   # v_mfma_f32_32x32x16_bf16


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--res", type=int, default=512)
    ap.add_argument("--joints", type=int, default=24)
    ap.add_argument("--samples", type=int, default=64)
    ap.add_argument("--importance", type=int, default=128)
    ap.add_argument("--cpu-rays", type=int, default=20000, help="rays in the CPU-baseline sample")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--shard", default="frames", choices=["frames", "pixels"],
                    help="frames: one frame per rank (weak scaling, no collective); pixels: ONE frame per step "
                         "split into whole 4096-ray chunks across the ranks + an RCCL all-gather of the ray "
                         "outputs (strong scaling, BASELINE config 5's layout)")
    ap.add_argument("--also", default="fp32,bf16x3",
                    help="other precision modes timed on the same frame afterwards (rank 0, N=1; '' = none)")
    ap.add_argument("--precision", default="bf16x6", choices=["fp32", "bf16x6", "bf16x3"],
                    help="MLP arithmetic (include/anerf.h ANERF_PREC_*)")
    return ap.parse_args()


def traffic_from_profiles(precision):
    """Per-launch HBM bytes of render_kernel from the newest committed rocprofv3 --pmc summary of
    this precision mode (profiles/*pmc*.json, field "precision"; untagged files are fp32)."""
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", "*pmc*.json")), reverse=True):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        if d.get("precision", "fp32") == precision and "render_kernel_hbm_bytes_per_launch" in d:
            return d["render_kernel_hbm_bytes_per_launch"]
    return None


def _config_name(H, S, I, nj):
    """BASELINE.json's config numbering; other shapes are 'custom'."""
    known = {(256, 64, 0, 24): "config2", (512, 64, 128, 24): "config3", (512, 64, 128, 65): "config4",
             (1024, 64, 128, 24): "config5"}
    return known.get((H, S, I, nj), "custom")


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    if dist:
        import torch.distributed as tdist
        torch.cuda.set_device(local)
        tdist.init_process_group("nccl")
    dev = torch.device(f"cuda:{local}")
    torch.cuda.set_device(dev)

    anerf = importlib.import_module("a-nerf_amd")
    syn = importlib.import_module("a-nerf_amd.synthetic")
    _lib = importlib.import_module("a-nerf_amd._lib")
    lib = _lib.load()

    H = W = a.res
    S, I = a.samples, a.importance
    cfg = anerf.RenderConfig(n_joints=a.joints, N_samples=S, N_importance=I, precision=a.precision).validate()
    ck = syn.make_checkpoint(13, n_joints=a.joints, D=8, W=256, fine=I > 0, tau=79.6)
    pixels = a.shard == "pixels"
    sc = syn.make_scene(n_joints=a.joints, H=H, W=W, seed=13 if pixels else 13 + rank)
    rc = anerf.RayCaster(cfg, ck, device=local)
    idxs, cyls, boxes = anerf.rays.valid_pixels(sc["c2ws"], H, W, sc["focal"], kps=sc["kps"], ext_scale=0.001)
    (x0, y0), (x1, y1) = (int(v) for v in boxes[0][0]), (int(v) for v in boxes[0][1])
    n = (x1 - x0) * (y1 - y0)
    c2w = torch.from_numpy(np.ascontiguousarray(sc["c2ws"][0][:3, :4])).to(dev)
    skts = torch.from_numpy(sc["skts"][0:1]).to(dev)
    cyl = torch.from_numpy(cyls[0:1]).to(dev)
    rb = torch.empty(n, 11, device=dev)
    img = torch.empty(H * W, 3, device=dev)
    dimg = torch.empty(H * W, device=dev)
    aimg = torch.empty(H * W, device=dev)
    st = _lib.stream_handle(dev)
    ev = []
    dmod = importlib.import_module("a-nerf_amd.distributed")

    def step(record):
        _lib.check(lib.anerf_gen_rays_box(_lib.ptr(c2w), H, W, sc["focal"], sc["focal"], 0.0, 0.0, 0, x0, y0, x1, y1,
                                          0.0, 1.0, _lib.ptr(rb), st), "gen_rays_box")
        if record:
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record()
        if pixels:  # this rank's whole-chunk range of the frame, then one all-gather (distributed.py)
            out = dmod.render_rays_sharded(
                lambda r: rc.render_rays(r, S, skts=skts.expand(r.shape[0], -1, -1, -1),
                                         cyls=cyl.expand(r.shape[0], -1), N_importance=I, chunk=4096,
                                         ret_alpha=False), rb, 4096) if dist else \
                rc.render_rays(rb, S, skts=skts.expand(n, -1, -1, -1), cyls=cyl.expand(n, -1), N_importance=I,
                               chunk=4096, ret_alpha=False)
        else:
            out = rc.render_rays(rb, S, skts=skts.expand(n, -1, -1, -1), cyls=cyl.expand(n, -1), N_importance=I,
                                 chunk=4096, ret_alpha=False)
        if record:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            ev.append((e0, e1))
        _lib.check(lib.anerf_compose_box(_lib.ptr(out["rgb_map"]), _lib.ptr(out["disp_map"]),
                                         _lib.ptr(out["acc_map"]), x0, y0, x1, y1, None, 0, H, W, _lib.ptr(img),
                                         _lib.ptr(dimg), _lib.ptr(aimg), st), "compose_box")

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
    kern_ms = float(np.mean([e0.elapsed_time(e1) for e0, e1 in ev]))
    rays_job = n * a.steps / (world if pixels else 1)  # pixels: the ranks share one frame per step
    if dist:
        t = torch.tensor([elapsed, float(rays_job)], device=dev, dtype=torch.float64)
        tmax = t[:1].clone()
        tdist.all_reduce(tmax, op=tdist.ReduceOp.MAX)
        tdist.all_reduce(t[1:], op=tdist.ReduceOp.SUM)
        elapsed, rays_job = float(tmax.item()), float(t[1].item())

    # executed MFMA work of one launch (exact device-side counter, one extra untimed launch) over the
    # rays this rank renders per step (pixels mode: its whole-chunk share of the frame)
    s0, s1 = dmod.chunk_ranges(n, 4096, world)[rank] if (pixels and dist) else (0, n)
    n_mine = s1 - s0
    rc.render_rays(rb[s0:s1], S, skts=skts.expand(n_mine, -1, -1, -1), cyls=cyl.expand(n_mine, -1), N_importance=I,
                   chunk=4096, ret_alpha=False, count_mfma=True)
    torch.cuda.synchronize()
    n_f32, n_bf16 = (int(v) for v in rc.last_mfma.tolist())
    flop_exec = n_f32 * FLOP_F32_MFMA + n_bf16 * FLOP_BF16_MFMA
    # the launch's MFMA work at each pipe's peak rate: the time the MFMA pipes must be busy
    t_mfma = n_f32 * FLOP_F32_MFMA / (FP32_MFMA_PEAK_TFLOPS * 1e12) + n_bf16 * FLOP_BF16_MFMA / (BF16_MFMA_PEAK_TFLOPS * 1e12)
    peak_tf = flop_exec / t_mfma / 1e12  # = 157.3 for fp32; the instruction-mix-weighted peak otherwise
    flop_ray = anerf.flops_per_sample(cfg) * anerf.samples_per_ray(cfg)  # SURVEY §8(d), reference work
    achieved_tf = flop_exec / (kern_ms * 1e-3) / 1e12
    ref_equiv_tf = flop_ray * n_mine / (kern_ms * 1e-3) / 1e12
    # the committed PMC summaries are of config 3's frame; other shapes report null
    traffic = traffic_from_profiles(a.precision) if _config_name(H, S, I, a.joints) == "config3" else None

    # the other precision modes on the same frame (kernel time of render_rays, HIP events), N=1 only
    others = {}
    if rank == 0 and world == 1:
        for p in [x for x in a.also.split(",") if x and x != a.precision]:
            rcp = anerf.RayCaster(anerf.RenderConfig(n_joints=a.joints, N_samples=S, N_importance=I,
                                                     precision=p).validate(), ck, device=local)
            ts = []
            for it in range(4):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                rcp.render_rays(rb, S, skts=skts.expand(n, -1, -1, -1), cyls=cyl.expand(n, -1), N_importance=I,
                                chunk=4096, ret_alpha=False)
                e1.record()
                torch.cuda.synchronize()
                if it:
                    ts.append(e0.elapsed_time(e1))
            rcp.render_rays(rb, S, skts=skts.expand(n, -1, -1, -1), cyls=cyl.expand(n, -1), N_importance=I,
                            chunk=4096, ret_alpha=False, count_mfma=True)
            torch.cuda.synchronize()
            pf, pb = (int(v) for v in rcp.last_mfma.tolist())
            pms = float(np.mean(ts))
            pflop = pf * FLOP_F32_MFMA + pb * FLOP_BF16_MFMA
            ppeak = pflop / (pf * FLOP_F32_MFMA / (FP32_MFMA_PEAK_TFLOPS * 1e12) +
                             pb * FLOP_BF16_MFMA / (BF16_MFMA_PEAK_TFLOPS * 1e12)) / 1e12
            others[p] = {"rays_per_s_kernel": round(n / (pms * 1e-3), 1), "kernel_ms": round(pms, 3),
                         "roofline_frac": round(pflop / (pms * 1e-3) / 1e12 / ppeak, 4), "dtype": DTYPE[p]}
            del rcp

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import oracle
        cores = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
        om = oracle.OracleModel(cfg, ck)
        rb_h = rb.cpu().numpy()
        sel = np.linspace(0, n - 1, min(a.cpu_rays, n)).astype(np.int64)
        t1 = time.perf_counter()
        om.render_rays(rb_h[sel], sc["skts"][0], cyls[0:1], chunk=4096, nthreads=cores)
        dt = time.perf_counter() - t1
        cpu = {"value": round(len(sel) / dt, 2), "unit": "rays/s", "cores": cores, "kind": "port",
               "sample": f"{len(sel)} rays evenly spaced over the frame's {n} bbox rays, C oracle "
                         f"(oracle/anerf_oracle.c, OpenMP {cores} threads), {dt:.1f} s wall"}

    if rank == 0:
        value = rays_job / elapsed
        line = {
            "metric": BASELINE["metric"], "value": round(value, 1), "unit": "rays/s", "n_gpus": world,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(1e3 * elapsed / a.steps, 3),
            "higher_is_better": True, "scaling": "strong" if pixels else "weak", "vs_baseline": None,
            "dtype": DTYPE[a.precision],
            "data": "synthetic (seeded SMPL-24 pose + seeded 8x256 weights; no dataset/checkpoint offline)",
            "config": {"workload": f"{_config_name(H, S, I, a.joints)}: {H}x{W} frame, {S}+{I} samples, {a.joints}-joint, 8x256 MLP, " +
                                   (f"one frame per step split over {world} GPU(s) in whole 4096-ray chunks + RCCL "
                                    f"all-gather" if pixels else "one frame per GPU per step"),
                       "rays_per_frame": n,
                       "parallelism": f"{'pixel-shard' if pixels else 'frame-per-rank'} x{world}"},
            "roofline": {"bound": "mfma", "achieved": round(achieved_tf, 2), "peak": round(peak_tf, 1),
                         "unit": "TFLOP/s", "frac": round(achieved_tf / peak_tf, 4),
                         "traffic": traffic, "kernel_ms": round(kern_ms, 3),
                         "launches_per_step": 2 if I > 0 else 1,
                         "timing": "HIP events on the launch stream around anerf_render_rays: the coarse and the "
                                   "fine render_kernel launch (+ near/far, 0.2 %); rocprofv3's render_kernel "
                                   "average x launches_per_step agrees (profiles/)",
                         "flop": "executed MFMA FLOPs of one step's launches (device counters) / their time "
                                 "(kernel_ms), the same ratio as per launch; peak = the FP32 (157.3) and BF16 "
                                 "(2516.6 TF) MFMA peaks weighted by the step's instruction mix; traffic per step",
                         "mfma_f32_per_step": n_f32, "mfma_bf16_per_step": n_bf16,
                         "reference_flop_per_ray": flop_ray,
                         "reference_equivalent_tflops": round(ref_equiv_tf, 2)},
            "cpu_baseline": cpu,
            "other_precisions": others or None,
        }
        print(json.dumps(line), flush=True)
    if dist:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
