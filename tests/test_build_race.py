"""Concurrent builds of libpyrope_hip.so: the ranks of a multi-GPU bench each
call build(); with sources newer than the shipped .so they must not compile into the same files at
once.  build.py serializes builders with a file lock and re-checks staleness under it, so exactly one
process compiles and links, the others wait and then load the finished library.

Runs on CPU with a stand-in compiler (HIPCC points to a script that writes its -o file and logs the
call), on a temporary copy of the package sources."""
import os
import shutil
import subprocess
import sys
import textwrap
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

FAKE = textwrap.dedent("""\
    #!/usr/bin/env python3
    import os, sys, time
    a = sys.argv[1:]
    out = a[a.index("-o") + 1]
    with open(os.environ["FAKE_HIPCC_LOG"], "a") as f:
        f.write(("link " if "-shared" in a else "compile ") + os.path.basename(out) + "\\n")
    time.sleep(0.3)
    with open(out, "wb") as f:
        f.write(b"x" * 64)
    """)


def _setup(tmp_path):
    pkg = tmp_path / "pyrope_amd"
    shutil.copytree(os.path.join(ROOT, "pyrope_amd", "csrc"), pkg / "csrc")
    shutil.copy(os.path.join(ROOT, "pyrope_amd", "build.py"), pkg / "build.py")
    shutil.copytree(os.path.join(ROOT, "include"), tmp_path / "include")
    fake = tmp_path / "fake_hipcc"
    fake.write_text(FAKE)
    fake.chmod(0o755)
    return pkg, fake


def _run_builders(pkg, fake, log, n):
    env = dict(os.environ, HIPCC=str(fake), FAKE_HIPCC_LOG=str(log))
    code = f"import sys; sys.path.insert(0, {str(pkg)!r}); import build; print(build.build())"
    procs = [subprocess.Popen([sys.executable, "-c", code], env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                              text=True) for _ in range(n)]
    outs = [p.communicate(timeout=120) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e
    return [o.strip() for o, _ in outs]


def test_concurrent_ranks_build_once(tmp_path):
    pkg, fake = _setup(tmp_path)
    log = tmp_path / "calls.log"
    # a stale shipped library: older than every source
    so = pkg / "libpyrope_hip.so"
    so.write_bytes(b"old")
    os.utime(so, (1, 1))
    outs = _run_builders(pkg, fake, log, 4)
    assert all(o == str(so) for o in outs)
    calls = log.read_text().split("\n")[:-1]
    import importlib.util
    spec = importlib.util.spec_from_file_location("b", str(pkg / "build.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    assert sum(c.startswith("compile") for c in calls) == len(b.SOURCES)  # one process compiled
    assert sum(c.startswith("link") for c in calls) == 1
    assert so.read_bytes() == b"x" * 64
    assert not [f for f in os.listdir(pkg) if f.endswith(".tmp")]
    # fresh now: a second round of ranks compiles nothing
    _run_builders(pkg, fake, log, 3)
    assert log.read_text().split("\n")[:-1] == calls


def test_incremental_rebuild_recompiles_only_the_touched_source(tmp_path):
    pkg, fake = _setup(tmp_path)
    log = tmp_path / "calls.log"
    _run_builders(pkg, fake, log, 1)
    n0 = len(log.read_text().split("\n")[:-1])
    src = pkg / "csrc" / "sample16.hip"
    t = os.path.getmtime(pkg / "libpyrope_hip.so") + 1
    os.utime(src, (t, t))
    time.sleep(1.2)  # the rebuilt objects and library are newer than the touched source
    _run_builders(pkg, fake, log, 2)
    new = log.read_text().split("\n")[:-1][n0:]
    assert len(new) == 2 and new[0] == "compile sample16.o.tmp.o" and new[1].startswith("link "), new
