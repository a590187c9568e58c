"""bench.py end to end on the CPU (ATen + Gloo): the multi-rank launch, the fallback ladder and
the JSON contract (utils/ladder.py; verdict round 5, "make the first multi-GPU run unable to
come back empty").

The driver's multi-GPU command is ``python -m torch.distributed.run --nnodes=1 --nproc-per-node
N --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...``; ``bench.py --gpus N`` without
a launcher spawns the ranks itself. Both must print ONE JSON line from the first attempt that
succeeds, even when the planned attempt's ranks fail (``DDP_AMD_FAULT_INJECT=<rank>:bench0:...``
fires only in attempt 0). Reference run being protected: /root/reference/part3/main.py:159-186.
"""
import json
import os
import subprocess
import sys

import pytest

from dist_helpers import free_port

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--device", "cpu", "--global-batch", "8", "--steps", "2", "--warmup", "1",
         "--train-size", "32", "--ref-window", "0"]


def _env(**extra):
    env = dict(os.environ, OMP_NUM_THREADS="1", DDP_AMD_WATCHDOG_S="10", **extra)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT",
              "DDP_AMD_LADDER_ATTEMPT", "DDP_AMD_FAULT_INJECT"):
        env.pop(k, None)
    env.update(extra)
    return env


def _run(cmd, env, timeout=240):
    p = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=timeout)
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    return p.returncode, lines, p.stderr


def _torchrun(n, extra_args=(), **env):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(REPO, "bench.py"), "--gpus", str(n), *SMALL, *extra_args]
    return _run(cmd, _env(**env))


def _self(n, extra_args=(), **env):
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(n), *SMALL, *extra_args]
    return _run(cmd, _env(**env))


def _one_json(lines, err):
    assert len(lines) == 1, (lines, err[-3000:])
    return json.loads(lines[0])


def test_single_rank_output_has_no_ladder():
    rc, lines, err = _self(1)
    assert rc == 0, err[-3000:]
    d = _one_json(lines, err)
    assert d["n_gpus"] == 1 and "attempts" not in d
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in d, k


def test_torchrun_clean_run_reports_one_successful_attempt():
    rc, lines, err = _torchrun(2)
    assert rc == 0, err[-3000:]
    d = _one_json(lines, err)
    assert d["n_gpus"] == 2 and d["launcher"] == "torchrun"
    assert d["config"]["global_batch"] == 8 and d["config"]["per_gpu_batch"] == 4
    assert d["replicas_consistent"] is True
    assert d["attempts"] == [{"name": "planned", "ok": True}]


def test_torchrun_falls_back_when_a_rank_dies_in_the_planned_attempt():
    rc, lines, err = _torchrun(2, DDP_AMD_FAULT_INJECT="1:bench0:exit")
    assert rc == 0, err[-3000:]
    d = _one_json(lines, err)
    att = d["attempts"]
    assert [a["name"] for a in att] == ["planned", "inline-ddp"]
    assert att[0]["ok"] is False and att[1]["ok"] is True
    # the injected exit (code 17) of rank 1 names the failure, not its peer's broken connection
    assert att[0]["reason"] == "exit 17" and att[0]["rank"] == 1, att[0]
    assert "fault injected" in att[0]["stderr_tail"]
    assert d["n_gpus"] == 2 and d["replicas_consistent"] is True


@pytest.mark.parametrize("mode", ["exit", "hang"])
def test_self_launch_falls_back(mode):
    rc, lines, err = _self(2, DDP_AMD_FAULT_INJECT=f"0:bench0:{mode}")
    assert rc == 0, err[-3000:]
    d = _one_json(lines, err)
    att = d["attempts"]
    assert att[0]["ok"] is False and att[-1]["ok"] is True and len(att) == 2, att
    if mode == "exit":
        assert att[0]["reason"] == "exit 17" and att[0]["rank"] == 0
    else:  # rank 0 hangs: rank 1's watchdog ends the attempt (exit 3)
        assert "watchdog" in att[0]["reason"], att[0]


def test_every_attempt_failing_exits_nonzero_without_a_json_line():
    # "bench" (no attempt index) fires in every attempt: no number, a non-zero exit, and the
    # attempt records on stderr
    rc, lines, err = _self(2, ["--strategy", "allreduce"], DDP_AMD_FAULT_INJECT="1:bench:exit")
    assert rc != 0 and not lines, (rc, lines)
    tail = [ln for ln in err.splitlines() if ln.startswith('{"error"')]
    assert tail, err[-2000:]
    rec = json.loads(tail[-1])["attempts"]
    assert [a["name"] for a in rec] == ["planned", "eager"]  # 2B's ladder
    assert [a["ok"] for a in rec] == [False, False]
