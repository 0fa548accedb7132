"""Build libanerf_hip.so in-tree (hipcc, gfx950).  Used by __graft_entry__.build().

Rebuilds are content-addressed: a sha256 over the compiler command, every file under csrc/ and
include/anerf.h is stored next to the library (`libanerf_hip.so.stamp`).  A shipped binary whose
stamp does not match the sources is rebuilt, never reused because of its mtime.

The two translation units compile in parallel into objects cached under `.objs/` by the hash of
their own dependencies (anerf_gemm.hip reads only include/anerf.h), then link into the library:
an edit of the training GEMMs recompiles one unit, not the render kernels' instances.
"""
import hashlib
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
HEADER = os.path.join(os.path.dirname(HERE), "include", "anerf.h")
SRC = [os.path.join(CSRC, "anerf_render.hip"), os.path.join(CSRC, "anerf_gemm.hip")]
OUT = os.path.join(HERE, "libanerf_hip.so")
STAMP = OUT + ".stamp"
OBJS = os.path.join(HERE, ".objs")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-slp-vectorize", "-fPIC", "-shared",
         "-Wno-unused-result"]
CFLAGS = [f for f in FLAGS if f != "-shared"]


def _hash(files, extra=""):
    h = hashlib.sha256()
    h.update((" ".join(FLAGS) + extra).encode())
    for d in files:
        if os.path.isfile(d):
            h.update(os.path.basename(d).encode())
            with open(d, "rb") as f:
                h.update(f.read())
    return h.hexdigest()


def source_hash():
    """sha256 over the flags and the bytes of csrc/* + include/anerf.h (sorted by name)."""
    deps = sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC))
    deps.append(HEADER)
    return _hash(deps)


def unit_deps(src):
    """The files a translation unit reads: anerf_gemm.hip only the C header, anerf_render.hip every csrc header."""
    if os.path.basename(src) == "anerf_gemm.hip":
        return [src, HEADER]
    return [src] + sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hpp")) + [HEADER]


def stamp_matches():
    if not (os.path.exists(OUT) and os.path.exists(STAMP)):
        return False
    with open(STAMP) as f:
        return f.read().strip() == source_hash()


def _object(src, verbose, force=False):
    """The unit's cached object, compiled if its dependencies changed (discarded if they moved meanwhile)."""
    digest = _hash(unit_deps(src), "-c")
    name = os.path.splitext(os.path.basename(src))[0]
    obj = os.path.join(OBJS, f"{name}.{digest[:20]}.o")
    if os.path.exists(obj) and not force:
        return obj
    tmp = obj + ".tmp"
    cmd = [HIPCC] + CFLAGS + ["-c", "-o", tmp, src]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    # hipcc reads the headers once per offload pass: a source edited during the build can give the host and
    # the device passes different struct layouts (a torn object).  Keep only an object whose inputs did not move
    if _hash(unit_deps(src), "-c") != digest:
        os.remove(tmp)
        raise RuntimeError(f"sources of {name} changed during the build: the object was discarded, build again")
    for old in os.listdir(OBJS):  # (one cached object per unit)
        if old.startswith(name + ".") and old.endswith(".o"):
            os.remove(os.path.join(OBJS, old))
    os.replace(tmp, obj)
    return obj


def build(force=False, verbose=True):
    if not force and stamp_matches():
        return OUT
    digest = source_hash()
    os.makedirs(OBJS, exist_ok=True)
    with ThreadPoolExecutor(max(1, len(SRC))) as ex:
        objs = list(ex.map(lambda s: _object(s, verbose, force), SRC))
    tmp = OUT + ".tmp"
    if os.path.exists(tmp):
        os.remove(tmp)
    cmd = [HIPCC] + FLAGS + ["-o", tmp] + objs
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    if source_hash() != digest:
        if os.path.exists(tmp):
            os.remove(tmp)
        raise RuntimeError("sources changed during the build: the library was discarded, build again")
    # replace the library in one rename (a copy of the tree never sees a half-written file)
    os.replace(tmp, OUT)
    with open(STAMP, "w") as f:
        f.write(digest + "\n")
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
