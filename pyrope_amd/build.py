"""Builds libpyrope_hip.so in-tree for gfx950 (hipcc; no JIT cache, no torch extension).

`python -m pyrope_amd.build` or `__graft_entry__.build()`.
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libpyrope_hip.so")
SOURCES = ["kernels.hip", "filter.hip", "filter16.hip", "filter16r.hip", "stream16.hip", "sq8.hip", "coarse.hip", "engine.cpp", "persist.cpp", "capi.cpp"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

# -ffp-contract=off: the parity contract (bit-identical scores) forbids FMA contraction.
COMMON = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-Wall", "-Wno-unused-function",
          "-I" + os.path.join(HERE, "..", "include")]


def _stale() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, f) for f in os.listdir(CSRC)] + [os.path.join(HERE, "..", "include", "pyrope_ann.h")]
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False) -> str:
    """Compile (if stale or forced) and link the library.  Safe against concurrent callers (e.g. the
    rank processes of a multi-GPU bench): an exclusive lock file serializes builds, the staleness
    check is repeated under the lock, objects carry the builder's pid and the .so is linked to a
    temporary name and renamed into place, so no process ever loads a half-written library."""
    if not force and not _stale():
        return OUT
    import fcntl
    with open(OUT + ".lock", "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        try:
            if not force and not _stale():
                return OUT  # another process built it while this one waited
            return _build_locked(verbose)
        finally:
            fcntl.flock(lk, fcntl.LOCK_UN)


def _build_locked(verbose: bool) -> str:
    objs = []
    jobs = []
    tag = f".{os.getpid()}"
    for src in SOURCES:
        obj = os.path.join(CSRC, src.rsplit(".", 1)[0] + tag + ".o")
        cmd = [HIPCC] + COMMON + ["-c", os.path.join(CSRC, src), "-o", obj]
        if src.endswith(".hip"):
            # no SLP: packed FP32 has no extra rate on gfx950 and its op_sel broadcasts double VGPRs
            cmd[1:1] = ["--offload-arch=gfx950", "-x", "hip", "-fno-slp-vectorize"]
        else:
            cmd[1:1] = ["-x", "c++", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include"]
        objs.append(obj)
        jobs.append(subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    failed = False
    for src, job in zip(SOURCES, jobs):
        out, _ = job.communicate()
        if job.returncode != 0:
            failed = True
            sys.stderr.write(f"--- {src} ---\n{out}\n")
        elif verbose and out:
            sys.stderr.write(out)
    if failed:
        raise RuntimeError("libpyrope_hip build failed")
    tmp = OUT + tag + ".tmp"
    link = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", tmp] + objs
    try:
        subprocess.run(link, check=True)
        os.replace(tmp, OUT)  # atomic: a concurrent loader sees the old or the new library
    finally:
        for o in objs + [tmp]:
            if os.path.exists(o):
                os.remove(o)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
