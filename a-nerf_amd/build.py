"""Build libanerf_hip.so in-tree (hipcc, gfx950).  Used by __graft_entry__.build().

Rebuilds are content-addressed: a sha256 over the compiler command, every file under csrc/ and
include/anerf.h is stored next to the library (`libanerf_hip.so.stamp`).  A shipped binary whose
stamp does not match the sources is rebuilt, never reused because of its mtime.
"""
import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = [os.path.join(HERE, "csrc", "anerf_render.hip"), os.path.join(HERE, "csrc", "anerf_gemm.hip")]
OUT = os.path.join(HERE, "libanerf_hip.so")
STAMP = OUT + ".stamp"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-slp-vectorize", "-fPIC", "-shared",
         "-Wno-unused-result"]


def source_hash():
    """sha256 over the flags and the bytes of csrc/* + include/anerf.h (sorted by name)."""
    h = hashlib.sha256()
    h.update(" ".join(FLAGS).encode())
    csrc = os.path.join(HERE, "csrc")
    deps = sorted(os.path.join(csrc, f) for f in os.listdir(csrc))
    deps.append(os.path.join(os.path.dirname(HERE), "include", "anerf.h"))
    for d in deps:
        if os.path.isfile(d):
            h.update(os.path.basename(d).encode())
            with open(d, "rb") as f:
                h.update(f.read())
    return h.hexdigest()


def stamp_matches():
    if not (os.path.exists(OUT) and os.path.exists(STAMP)):
        return False
    with open(STAMP) as f:
        return f.read().strip() == source_hash()


def build(force=False, verbose=True):
    if not force and stamp_matches():
        return OUT
    digest = source_hash()
    tmp = OUT + ".tmp"
    if os.path.exists(tmp):
        os.remove(tmp)
    cmd = [HIPCC] + FLAGS + ["-o", tmp] + SRC
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    # hipcc reads the headers once per offload pass: a source edited during the build can give the host and
    # the device passes different struct layouts (a torn library).  Keep only a build whose sources did not
    # move, and replace the library in one rename (a copy of the tree never sees a half-written file).
    if source_hash() != digest:
        if os.path.exists(tmp):
            os.remove(tmp)
        raise RuntimeError("sources changed during the build: the library was discarded, build again")
    os.replace(tmp, OUT)
    with open(STAMP, "w") as f:
        f.write(digest + "\n")
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
