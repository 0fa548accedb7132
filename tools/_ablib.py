"""A/B tooling only: ANERF_LIB_PATH names an experiment build of libanerf_hip.so (tools/build_ab.sh) for the
tools/*.py scripts and bench.py.  The product package itself reads no environment (_lib.LIB_PATH is the in-tree
library); this module hands the path to `_lib.use_library` before the first load."""
import importlib
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def apply(path=None):
    path = path or os.environ.get("ANERF_LIB_PATH")
    if path:
        importlib.import_module("a-nerf_amd._lib").use_library(path)
    return path


apply()
