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
SOURCES = ["kernels.hip", "sort.hip", "filter.hip", "tiles16.hip", "sample16.hip", "scan.hip", "pq32.hip", "sq8.hip", "coarse.hip", "shard.hip", "engine.cpp", "multi.cpp", "persist.cpp", "capi.cpp"]
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
    check is repeated under the lock, objects are written to temporary names and renamed, and the .so
    is linked to a temporary name and renamed into place, so no process ever loads a half-written
    library."""
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


def _headers():
    hs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    return hs + [os.path.join(HERE, "..", "include", "pyrope_ann.h")]


def _build_locked(verbose: bool) -> str:
    """Called with the build lock held: objects live in build/ under fixed names, and a source is
    recompiled when its object is older than it or than any header (incremental rebuilds)."""
    odir = os.path.join(HERE, "build")
    os.makedirs(odir, exist_ok=True)
    hdr_t = max(os.path.getmtime(h) for h in _headers())
    objs = []
    jobs = []
    for src in SOURCES:
        sp = os.path.join(CSRC, src)
        obj = os.path.join(odir, src.rsplit(".", 1)[0] + ".o")
        objs.append(obj)
        if os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(sp), hdr_t):
            continue
        tmpo = obj + ".tmp.o"
        cmd = [HIPCC] + COMMON + ["-c", sp, "-o", tmpo]
        if src.endswith(".hip"):
            # no SLP: packed FP32 has no extra rate on gfx950 and its op_sel broadcasts double VGPRs
            cmd[1:1] = ["--offload-arch=gfx950", "-x", "hip", "-fno-slp-vectorize"]
        else:
            cmd[1:1] = ["-x", "c++", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include"]
        jobs.append((src, obj, tmpo, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                                                        text=True)))
    failed = False
    for src, obj, tmpo, job in jobs:
        out, _ = job.communicate()
        if job.returncode != 0:
            failed = True
            sys.stderr.write(f"--- {src} ---\n{out}\n")
            if os.path.exists(tmpo):
                os.remove(tmpo)
        else:
            os.replace(tmpo, obj)
            if verbose and out:
                sys.stderr.write(out)
    if failed:
        raise RuntimeError("libpyrope_hip build failed")
    tmp = OUT + f".{os.getpid()}.tmp"
    link = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", tmp] + objs + ["-ldl"]
    try:
        subprocess.run(link, check=True)
        os.replace(tmp, OUT)  # atomic: a concurrent loader sees the old or the new library
    finally:
        if os.path.exists(tmp):
            os.remove(tmp)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
