"""bench.py's driver contract: defaults (N=1, a window that finishes within minutes) on CPU, and
on the GPU the one JSON line -- BASELINE.json's metric, whole-job value, the roofline object of
the dominant kernel and the workload name."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_default_window():
    sys.path.insert(0, REPO)
    try:
        import bench
    finally:
        sys.path.remove(REPO)
    a = bench.parse_args([])
    assert (a.gpus, a.steps, a.warmup) == (1, 200, 100)
    a = bench.parse_args(["--gpus", "2", "--steps", "7", "--warmup", "3"])
    assert (a.gpus, a.steps, a.warmup) == (2, 7, 3)   # the driver's K / W are taken as given


@pytest.mark.gpu
def test_bench_line(gpu):
    legs = ["--no-cpu", "--no-warm", "--no-front-end", "--no-single-env", "--no-north-star",
            "--no-mixed"]
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "10",
                        "--warmup", "5", *legs], capture_output=True, text=True, timeout=240,
                       cwd=REPO)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    line = json.loads(lines[0])
    with open(os.path.join(REPO, "BASELINE.json")) as f:
        metric = json.load(f)["metric"]
    assert line["metric"] == metric
    assert (line["n_gpus"], line["steps"], line["warmup"]) == (1, 10, 5)
    assert line["unit"] == "solves/s" and line["higher_is_better"] is True
    assert line["scaling"] == "weak" and line["vs_baseline"] is None
    assert line["dtype"] == "f64"
    # whole-job throughput = envs / time per step
    nenv = line["config"]["envs_per_gpu"]
    assert line["value"] == pytest.approx(nenv / (line["ms_per_step"] * 1e-3), rel=1e-9)
    assert "workload" in line["config"] and "configs[1]" in line["config"]["workload"]
    assert line["converged_frac"] == 1.0
    rf = line["roofline"]
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and rf["peak"] == 8000.0
    assert rf["frac"] == pytest.approx(rf["achieved"] / rf["peak"], rel=1e-9)
    # achieved = algorithmic bytes per launch / the kernel's own event-timed duration
    assert rf["achieved"] == pytest.approx(
        rf["bytes_per_solve"] * nenv / (rf["kernel_ms"] * 1e-3) / 1e9, rel=1e-9)
    assert 0.0 < rf["kernel_ms"] < line["ms_per_step"]
