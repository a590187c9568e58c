"""bench.py output contract on one MI355X (the driver parses this line every round).

Runs ``bench.py`` as a child process (one extra GPU process, bounded by a timeout) for a few
steps and checks the single JSON line: metric / config named by BASELINE.json, whole-job
value consistent with ms_per_step and the global batch, vs_baseline against BASELINE.md's
part-3 number, bf16 compute, the captured hipGraph path, and a finite training loss.
"""
import json
import math
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run_bench(*extra, steps=4, warmup=3):
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--steps", str(steps), "--warmup",
           str(warmup), *extra]
    p = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_json_contract(native_ext):
    import bench
    # timed steps 10..19: the window the lr-0.1 numerics test characterises
    r = _run_bench(steps=10, warmup=10)
    for k in ["metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"]:
        assert k in r, k
    assert r["metric"].startswith("images/sec") and r["unit"] == "images/s"
    assert r["n_gpus"] == 1 and r["steps"] == 10 and r["warmup"] == 10
    # the reference protocol: global batch 256 split int(256/N) per GPU (strong scaling)
    assert r["higher_is_better"] is True and r["scaling"] == "strong"
    assert r["dtype"] == "bf16" and r["data"].startswith("synthetic")
    cfg = r["config"]
    assert cfg["model"] == "vgg11" and cfg["global_batch"] == 256 and cfg["parallelism"] == "dp1"
    assert cfg["hipgraph"] is True
    assert cfg["optimizer"].startswith("SGD(lr=0.1, momentum=0.9, wd=1e-4)")  # the reference's
    # value is the whole-job rate implied by the timed steps
    assert math.isclose(r["value"], cfg["global_batch"] / (r["ms_per_step"] / 1e3), rel_tol=1e-3)
    assert math.isclose(r["vs_baseline"], r["value"] / bench.BASELINE_IMG_S, rel_tol=1e-2)
    # lr 0.1 / momentum 0.9 from random init: the first ~10 steps spike. Over steps 10..19 of the
    # bench's synthetic batches, the fp32 family of test_gpu_model.py::
    # test_vgg11_lr01_headline_regime_tracks_fp32_family (fp32, bf16-emulated, two half-ulp
    # perturbed fp32 runs) averages 3.2-4.2. The bound is that range widened by 40 %. Six bench
    # runs gave 2.97-4.27 (profiles/r4z12_bench_loss_window.md)
    assert math.isfinite(r["train_loss_mean"]) and 2.3 <= r["train_loss_mean"] <= 5.9, \
        r["train_loss_mean"]
    assert r["replicas_consistent"] is True
    # the reference's own timing window (iterations 1..39, host sync per iteration)
    assert r["avg_ms_iter_1_39"] > 0 and r["img_s_iter_1_39"] > 0


def test_bench_protocol_batch_split(native_ext):
    """--global-batch B splits int(B/N) per GPU (strong); --per-gpu-batch fixes it (weak)."""
    r = _run_bench("--global-batch", "32", "--ref-window", "0")
    assert r["scaling"] == "strong" and r["config"]["global_batch"] == 32
    assert r["config"]["per_gpu_batch"] == 32 and r["avg_ms_iter_1_39"] is None
    r = _run_bench("--per-gpu-batch", "64", "--ref-window", "0")
    assert r["scaling"] == "weak" and r["config"]["global_batch"] == 64
