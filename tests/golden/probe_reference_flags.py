"""Record how the REFERENCE behaves on flag paths this build refuses, so the refusal is checked
against the reference rather than asserted (runs only where /root/reference exists; writes
reference_flags.json next to this file).

use_viewdirs=False: create_raycaster leaves embeddirs_fn = None (core/raycasters.py:66-67) and
encode_inputs calls it (:538), so RayCaster.render_rays raises TypeError before any output.
Usage: python tests/golden/probe_reference_flags.py
"""
import json
import os
import sys
import tempfile
import traceback

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402


def probe_no_viewdirs(mods, tmp):
    return probe(mods, tmp, [])


def probe(mods, tmp, flags):
    """render_rays of 16 rays under the given flags: None, or the reference's own exception."""
    run_nerf, _, raycasters, _, sk = mods
    argv = ["--N_samples", "32", "--N_importance", "16", "--netdepth", "4", "--netwidth", "128", "--use_cutoff",
            "--cutoff_inputs", "--ext_scale", "0.001", "--chunk", "4096", "--no_reload", "--basedir", tmp,
            "--expname", "x"] + flags
    args = run_nerf.config_parser().parse_args(argv)
    os.makedirs(os.path.join(tmp, "x"), exist_ok=True)
    data_attrs = {"skel_type": sk.SMPLSkeleton, "near": 0.0, "far": 1.0, "n_views": 5,
                  "joint_coords": np.zeros((24, 3, 3), np.float32)}
    _, rk, _, _, _, _ = raycasters.create_raycaster(args, data_attrs)
    rk["ray_caster"].eval()
    rc = rk["ray_caster"]
    attrs = {f"{e}.{a}": bool(getattr(getattr(rc, e), a)) for e in ("embed_fn", "embeddirs_fn")
             for a in ("normalize", "cut_to_cutoff", "shift_inputs") if hasattr(getattr(rc, e), a)}
    sc = mg.scene_for(dict(H=64, NJ=24, seed=41))
    (o, d), _, cyls, _ = mg.rays_for(mods, sc)
    sc["cyls"] = cyls
    try:
        import torch
        torch.manual_seed(0)
        mg.render_subset(mods, rk, o[:16], d[:16], sc)
        return {"raises": None, "embedder_attributes": attrs}
    except Exception as e:  # the reference's own failure, recorded
        tb = traceback.extract_tb(e.__traceback__)
        ref = [f"{os.path.relpath(f.filename, mg.REF)}:{f.lineno}" for f in tb if f.filename.startswith(mg.REF)]
        return {"raises": type(e).__name__, "message": str(e), "reference_frames": ref}


def main():
    mods = mg.import_reference()
    with tempfile.TemporaryDirectory() as tmp:
        out = {"use_viewdirs=False": probe_no_viewdirs(mods, tmp)}
        # the remaining refused embedder flags, with the view branch on as in every shipped config
        vd = ["--use_viewdirs", "--cutoff_viewdir"]
        for name, flags in (("normalize_cutoff", ["--normalize_cutoff"]), ("cut_to_dist", ["--cut_to_dist"]),
                            ("cutoff_shift", ["--cutoff_shift"]),
                            ("cutoff_bones", ["--cutoff_bones"]),
                            ("cutoff_bones+multires_bones=2", ["--cutoff_bones", "--multires_bones", "2"])):
            out[name] = probe(mods, tmp, vd + flags)
        # the non-default encoder selectors (core/raycasters.py:251-305)
        for name, flags in (("kp_dist_type=cat", ["--kp_dist_type", "cat"]),
                            ("kp_dist_type=relpos", ["--kp_dist_type", "relpos"]),
                            ("kp_dist_type=querypts", ["--kp_dist_type", "querypts"]),
                            ("view_type=rayangle", ["--view_type", "rayangle"]),
                            ("view_type=world", ["--view_type", "world"]),
                            ("bone_type=axisang", ["--bone_type", "axisang"])):
            try:
                out[name] = probe(mods, tmp, vd + flags)
            except Exception as e:  # (raised while building the caster)
                out[name] = {"raises": type(e).__name__, "message": str(e), "at": "create_raycaster"}
    path = os.path.join(HERE, "reference_flags.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
