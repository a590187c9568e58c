"""Self-launcher (ddp_amd/utils/launch.py): ``bench.py --gpus N`` / ``tools/comm_bench.py --gpus
N`` spawn one process per GPU themselves — reference: one process per node started with
--num-nodes/--rank (/root/reference/README.md:8-19, part3/main.py:160-167).

CPU only: stub children record what they were given; the bench's own guards (too few devices,
WORLD_SIZE vs --gpus) must fail loudly; comm_bench runs end to end over Gloo through the
launcher and writes a bucket-sizing table."""
import json
import os
import subprocess
import sys
import time

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

STUB = r'''
import json, os, sys, time
out = sys.argv[1]
r = int(os.environ["RANK"])
rec = {k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE",
                                       "MASTER_ADDR", "MASTER_PORT", "DDP_AMD_LAUNCHER")}
rec["pid"], rec["ppid"] = os.getpid(), os.getppid()
mode = sys.argv[2] if len(sys.argv) > 2 else "ok"
with open(os.path.join(out, f"rank{r}.json"), "w") as f:
    json.dump(rec, f)
print(f"stdout-of-rank-{r}", flush=True)
if mode == "fail3" and r == 3:
    sys.exit(7)
if mode in ("fail3", "hang"):
    time.sleep(120)
'''


@pytest.fixture
def stub(tmp_path):
    p = tmp_path / "stub.py"
    p.write_text(STUB)
    return str(p)


def _clean_env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT", "TORCHELASTIC_RUN_ID"):
        env.pop(k, None)
    return env


def test_spawn_eight_ranks_one_port_no_exec(stub, tmp_path, monkeypatch):
    from ddp_amd.utils import launch
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    import torch
    rc = launch.spawn([sys.executable, stub, str(tmp_path)], 8, timeout_s=120)
    assert rc == 0
    recs = [json.loads((tmp_path / f"rank{r}.json").read_text()) for r in range(8)]
    assert [int(x["RANK"]) for x in recs] == list(range(8))
    assert [int(x["LOCAL_RANK"]) for x in recs] == list(range(8))
    assert {x["WORLD_SIZE"] for x in recs} == {"8"} and {x["LOCAL_WORLD_SIZE"] for x in recs} == {"8"}
    assert len({x["MASTER_PORT"] for x in recs}) == 1
    assert {x["MASTER_ADDR"] for x in recs} == {"127.0.0.1"}
    assert {x["DDP_AMD_LAUNCHER"] for x in recs} == {"self"}
    # spawned children of THIS process (no exec of the parent), which never touched the GPU
    assert {x["ppid"] for x in recs} == {os.getpid()}
    assert len({x["pid"] for x in recs}) == 8
    assert not torch.cuda.is_initialized()


def test_only_rank0_stdout_reaches_parent_stdout(stub, tmp_path):
    code = ("import sys; sys.path.insert(0, %r); from ddp_amd.utils import launch; "
            "sys.exit(launch.spawn([sys.executable, %r, %r], 4, timeout_s=120))"
            % (REPO, stub, str(tmp_path)))
    p = subprocess.run([sys.executable, "-c", code], env=_clean_env(), capture_output=True,
                       text=True, timeout=300)
    assert p.returncode == 0, p.stderr
    assert p.stdout.split() == ["stdout-of-rank-0"]
    for r in (1, 2, 3):
        assert f"stdout-of-rank-{r}" in p.stderr


def test_failing_rank_stops_the_others(stub, tmp_path):
    from ddp_amd.utils import launch
    t0 = time.monotonic()
    rc = launch.spawn([sys.executable, stub, str(tmp_path), "fail3"], 6, timeout_s=120,
                      grace_s=1.0, log=lambda m: None)
    assert rc == 7
    assert time.monotonic() - t0 < 60  # the sleeping peers were killed, not waited for
    pids = [json.loads((tmp_path / f"rank{r}.json").read_text())["pid"] for r in range(6)]
    time.sleep(0.5)
    for pid in pids:
        assert not os.path.exists(f"/proc/{pid}") or open(f"/proc/{pid}/stat").read().split()[2] == "Z"


def test_timeout_kills_every_rank(stub, tmp_path):
    from ddp_amd.utils import launch
    rc = launch.spawn([sys.executable, stub, str(tmp_path), "hang"], 3, timeout_s=2.0,
                      log=lambda m: None)
    assert rc == 124


def test_bench_refuses_more_ranks_than_gpus():
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "8"],
                       env=_clean_env(), capture_output=True, text=True, timeout=300)
    assert p.returncode != 0
    assert "GPU(s) visible" in p.stderr
    assert p.stdout.strip() == ""  # no JSON line


def test_bench_refuses_world_size_mismatch():
    env = _clean_env()
    env.update(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT="29999")
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "4"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode != 0
    assert "WORLD_SIZE=2" in p.stderr and p.stdout.strip() == ""


def test_comm_bench_through_launcher_writes_table(tmp_path):
    table = tmp_path / "comm_tuning.json"
    table.write_text(json.dumps({"worlds": {"2": {"source": "model", "fp32": [
        {"bytes": 65536, "us": 12.0, "algbw_GBps": 5.0, "busbw_GBps": 5.0}]}}}))
    p = subprocess.run([sys.executable, os.path.join(REPO, "tools", "comm_bench.py"),
                        "--gpus", "2", "--device", "cpu", "--iters", "2", "--min-kb", "64",
                        "--max-mb", "1", "--write-table", str(table)],
                       env=_clean_env(), capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    rows = [json.loads(line) for line in p.stdout.splitlines() if line.startswith("{")]
    assert [r["bytes"] for r in rows] == [65536, 262144, 1048576]
    assert all(r["correct"] and r["world"] == 2 for r in rows)
    t = json.loads(table.read_text())
    ent = t["worlds"]["2"]
    assert ent["source"] == "measured-gloo-cpu"  # measured rows replaced the model rows
    assert [r["bytes"] for r in ent["fp32"]] == [65536, 262144, 1048576]
    from ddp_amd.parallel.bucket_plan import choose_bucket_caps, rows_for
    rws, src = rows_for(t, 2, "fp32")
    assert src.startswith("measured-gloo-cpu table (world 2")
    cap, first, why = choose_bucket_caps(2, 40 << 20, overlap=True, table=t)
    assert cap >= 7 * 512 * 1024 and "measured-gloo-cpu" in why


def _alive(pid):
    try:
        with open(f"/proc/{pid}/stat") as f:
            return f.read().split()[2] != "Z"
    except OSError:
        return False


@pytest.mark.parametrize("sig", ["SIGTERM", "SIGHUP", "SIGKILL"])
def test_parent_signal_leaves_no_rank_behind(stub, tmp_path, sig):
    """A launcher that is terminated (scheduler timeout, closed terminal: SIGTERM / SIGHUP) or
    killed outright (SIGKILL) must not orphan its ranks: they live in their own sessions, so the
    signal never reaches them by itself (utils/launch.py _SignalGuard + PR_SET_PDEATHSIG)."""
    import signal as _signal
    code = ("import sys; sys.path.insert(0, %r); from ddp_amd.utils import launch; "
            "sys.exit(launch.spawn([sys.executable, %r, %r, 'hang'], 3, timeout_s=300))"
            % (REPO, stub, str(tmp_path)))
    parent = subprocess.Popen([sys.executable, "-c", code], env=_clean_env(),
                              stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    try:
        deadline = time.monotonic() + 120
        while time.monotonic() < deadline and not all(
                (tmp_path / f"rank{r}.json").exists() for r in range(3)):
            time.sleep(0.1)
        pids = [json.loads((tmp_path / f"rank{r}.json").read_text())["pid"] for r in range(3)]
        assert all(_alive(p) for p in pids)
        parent.send_signal(getattr(_signal, sig))
        rc = parent.wait(timeout=60)
        if sig != "SIGKILL":
            assert rc == 128 + int(getattr(_signal, sig)), rc
        deadline = time.monotonic() + 20
        while time.monotonic() < deadline and any(_alive(p) for p in pids):
            time.sleep(0.1)
        assert not any(_alive(p) for p in pids), "a rank outlived its launcher"
    finally:
        if parent.poll() is None:
            parent.kill()
