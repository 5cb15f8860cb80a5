"""bench.py end to end at a small size (one GPU): the JSON line carries the contract's fields,
the CPU baseline's answers equal the GPU's bit for bit, and recall is a fraction."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_small_json_line():
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--n", "300000", "--nlist", "64", "--nprobe", "8",
           "--nq", "2000", "--steps", "3", "--warmup", "1", "--recall-queries", "200", "--cpu-seconds", "1",
           "--block-rows", "40000", "--add-rows", "100000"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1]
    out = json.loads(line)
    for key in ["metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"]:
        assert key in out
    assert out["n_gpus"] == 1 and out["value"] > 0
    assert 0.0 < out["recall_at_10"] <= 1.0
    cpu = out["cpu_baseline"]
    assert cpu["parity"]["ids_equal"] and cpu["parity"]["scores_bit_identical"]
    assert cpu["cores"] >= 1 and "host" in cpu
    assert 0 < out["roofline"]["frac"] < 1.5
