"""The reference entry points with 3 ranks on CPU (Gloo), launched the reference way.

Each rank is its own ``python partX/main.py --num-nodes 3 --rank R --master-ip 127.0.0.1
--master-port P`` process (reference README). Three workers is the case the
reference's report calls out: the per-rank batch is int(B / 3), so the global batch shrinks
(SURVEY.md §7.4, 256 -> 255). The reference validates its parts by comparing the final test
loss / accuracy across parts: here every rank of a part must report the SAME
test line (replicas stayed identical), and 2A, 2B and DDP must agree with each other.
"""
import os
import re
import subprocess
import sys

import pytest

from dist_helpers import free_port

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORLD = 3
PARTS = ["part2/part2a", "part2/part2b", "part3"]
TEST_RE = re.compile(r"Test set: Average loss: ([0-9.]+), Accuracy: (\d+)/(\d+)")


def _run_part(part):
    port = free_port()
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.pop("RANK", None)
    env.pop("WORLD_SIZE", None)
    procs = []
    for r in range(WORLD):
        cmd = [sys.executable, os.path.join(REPO, part, "main.py"), "--num-nodes", str(WORLD),
               "--rank", str(r), "--master-ip", "127.0.0.1", "--master-port", str(port),
               "--device", "cpu", "--global-batch", "13", "--train-size", "96",
               "--test-size", "24", "--max-batches", "3", "--threads", "1"]
        procs.append(subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                      text=True, env=env))
    outs = []
    try:
        for p in procs:
            o, e = p.communicate(timeout=300)
            assert p.returncode == 0, e[-3000:]
            outs.append(o)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return outs


@pytest.fixture(scope="module")
def runs():
    return {part: _run_part(part) for part in PARTS}


def _test_line(out):
    m = [TEST_RE.search(l) for l in out.splitlines()]
    m = [x for x in m if x]
    assert m, out[-2000:]
    return float(m[-1].group(1)), int(m[-1].group(2)), int(m[-1].group(3))


def test_three_ranks_report_identical_test_results(runs):
    for part, outs in runs.items():
        lines = [_test_line(o) for o in outs]
        assert all(l == lines[0] for l in lines), (part, lines)
        assert lines[0][2] == 24  # the unsharded test set, evaluated by every rank


def test_parts_agree(runs):
    loss = {part: _test_line(outs[0])[0] for part, outs in runs.items()}
    ref = loss["part2/part2a"]
    for part, v in loss.items():
        assert abs(v - ref) <= 1e-3 * max(1.0, abs(ref)), loss


def test_setup_diagnostics_lines(runs):
    # test_distributed_setup()'s four lines (reference part2/part2a/main.py:42-49); the 1-39
    # timing lines need 40 iterations and are pinned by test_cli_contract.py
    for part, outs in runs.items():
        for r, o in enumerate(outs):
            for want in ["Is initialized: True", "Backend: gloo", f"World size: {WORLD}",
                         f"Rank: {r}"]:
                assert want in o, (part, r, want, o[-1500:])
