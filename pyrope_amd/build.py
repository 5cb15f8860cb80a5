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
SOURCES = ["kernels.hip", "filter.hip", "filter16.hip", "sq8.hip", "coarse.hip", "engine.cpp", "persist.cpp", "capi.cpp"]
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
    if not force and not _stale():
        return OUT
    objs = []
    jobs = []
    for src in SOURCES:
        obj = os.path.join(CSRC, src.rsplit(".", 1)[0] + ".o")
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
    link = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", OUT] + objs
    subprocess.run(link, check=True)
    for o in objs:
        os.remove(o)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
