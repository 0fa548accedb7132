"""MI355X-native A-NeRF render path: drop-in RayCaster / render / render_path over HIP kernels.

Import as ``importlib.import_module("a-nerf_amd")`` (the directory name is not a Python
identifier).  The compute lives in libanerf_hip.so (C ABI: include/anerf.h); this package is
the host-side mirror of the reference interface (core/raycasters.py, core/trainer.py,
run_nerf.py).
"""
from .config import RenderConfig, flops_per_sample, samples_per_ray
from .raycaster import RayCaster, create_raycaster, load_checkpoint
from .render import batchify_rays, render, render_path, render_frames
from . import dataset, rays, synthetic, train
from .dataset import RayImageDataset, RayImageSampler

__all__ = ["RenderConfig", "RayCaster", "create_raycaster", "load_checkpoint", "render", "render_path",
           "render_frames", "batchify_rays", "rays", "synthetic", "dataset", "RayImageDataset", "RayImageSampler", "flops_per_sample", "samples_per_ray"]
