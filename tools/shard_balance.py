"""Multi-GPU load balance measured on ONE GPU: config 5's 1024^2 frame (the
north star's pixel-sharded layout, bf16x6) cut into the 8 shards of each split that
a-nerf_amd/distributed.py offers, every shard rendered alone with HIP events on the launch stream.
Per-ray cost is not constant (exact-zero window skipping: cost follows the live joints along the
ray), so equal ray counts need not be equal times.  Prints one JSON line per split with the per-shard
milliseconds and max / mean; the slowest shard is what an 8-rank step waits for.

  python tools/shard_balance.py [--precision bf16x6] [--world 8] [--reps 3]"""
import argparse
import importlib
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import _ablib  # noqa: E402,F401  (ANERF_LIB_PATH: an experiment build, A/B tooling only)
anerf = importlib.import_module("a-nerf_amd")
syn = importlib.import_module("a-nerf_amd.synthetic")
dmod = importlib.import_module("a-nerf_amd.distributed")
_lib = importlib.import_module("a-nerf_amd._lib")
near_far = importlib.import_module("a-nerf_amd.raycaster").near_far


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--precision", default="bf16x6")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--res", type=int, default=1024)
    a = ap.parse_args()
    H, seed, tau = a.res, 13, 79.6
    sc = syn.make_scene(n_joints=24, H=H, W=H, seed=seed)
    ck = syn.make_checkpoint(seed, n_joints=24, D=8, W=256, fine=True, tau=tau)
    idx, cyls, boxes = anerf.rays.valid_pixels(sc["c2ws"], H, H, sc["focal"], kps=sc["kps"], ext_scale=0.001)
    (x0, y0), (x1, y1) = (int(v) for v in boxes[0][0]), (int(v) for v in boxes[0][1])
    n = (x1 - x0) * (y1 - y0)
    c2w = torch.from_numpy(np.ascontiguousarray(sc["c2ws"][0][:3, :4])).cuda()
    rb = torch.empty(n, 11, device="cuda")
    _lib.check(_lib.load().anerf_gen_rays_box(_lib.ptr(c2w), H, H, sc["focal"], sc["focal"], 0.0, 0.0, 0, x0, y0, x1,
                                              y1, 0.0, 1.0, _lib.ptr(rb), _lib.stream_handle()), "gen_rays_box")
    cy = torch.from_numpy(cyls[0:1]).cuda()
    sk = torch.from_numpy(sc["skts"][0:1]).cuda()
    near_far(rb, cy, chunk=4096, out=(rb[:, 6], rb[:, 7]))  # the whole frame's chunk NaN fill (H1)
    cfg = anerf.RenderConfig(N_samples=64, N_importance=128, precision=a.precision).validate()
    rc = anerf.RayCaster(cfg, ck)

    def render(rows):
        m = rows.shape[0]
        return rc.render_rays(rb.index_select(0, rows), 64, skts=sk.expand(m, -1, -1, -1), cyls=cy.expand(m, -1),
                              N_importance=128, chunk=4096, ret_alpha=False, near_far_given=True)

    def timed(rows):
        rows_b = rb.index_select(0, rows)
        m = rows.shape[0]
        best = None
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            rc.render_rays(rows_b, 64, skts=sk.expand(m, -1, -1, -1), cyls=cy.expand(m, -1), N_importance=128,
                           chunk=4096, ret_alpha=False, near_far_given=True)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1)
            best = ms if best is None else min(best, ms)
        return best

    splits = {"ray_ranges (contiguous, equal rays)": [torch.arange(s0, s1, device="cuda")
                                                     for s0, s1 in dmod.ray_ranges(n, a.world)]}
    if hasattr(dmod, "tile_rows"):
        for tile in (256, 1024):
            splits[f"tile_rows (tiles of {tile} rays round-robin)"] = [
                dmod.tile_rows(n, a.world, r, tile).cuda() for r in range(a.world)]
    render(torch.arange(0, min(n, 65536), device="cuda"))  # warm-up
    whole = timed(torch.arange(n, device="cuda"))
    print(json.dumps({"frame": f"config 5, {H}^2, {n} rays, {a.precision}", "whole_frame_ms": round(whole, 3),
                      "whole_frame_rays_per_s": round(n / whole * 1e3)}))
    ref = render(torch.arange(n, device="cuda"))
    for name, parts in splits.items():
        ms = [timed(rows) for rows in parts]
        # the union of the shards is the frame, bit for bit
        outs = [render(rows) for rows in parts]
        ok = True
        for k in ("rgb_map", "disp_map", "acc_map"):
            full = torch.empty_like(ref[k])
            for rows, o in zip(parts, outs):
                full[rows] = o[k]
            ok &= bool(torch.equal(full, ref[k]))
        mean = sum(ms) / len(ms)
        print(json.dumps({"split": name, "world": a.world, "rays": [int(r.shape[0]) for r in parts],
                          "shard_ms": [round(x, 3) for x in ms], "max_over_mean": round(max(ms) / mean, 4),
                          "sum_ms": round(sum(ms), 3), "union_bit_identical": ok,
                          "projected_rays_per_s_at_world": round(n / max(ms) * 1e3)}))


if __name__ == "__main__":
    main()
