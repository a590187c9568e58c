"""Launch mapping, --graph epoch schedule and failure detection (CPU, no GPU needed).

* Reference-style one-node launch: ``python part3/main.py --num-nodes 8 --rank R`` once per GPU
  (reference README.md:8-19, part3/main.py:29,36-40) must put rank R on GPU R; torchrun's
  LOCAL_RANK wins when present.
* ``--graph`` epochs replay only the full batches and run the partial tail batch eagerly, so the
  samples seen per epoch equal the eager loader's (and the reference DataLoader's).
* Failure detection (the reference has none, part2/part2a/main.py:58): one of
  three Gloo ranks of ``part3/main.py`` dies (or hangs) mid-epoch; every surviving rank must exit
  NON-ZERO within the watchdog timeout instead of blocking forever.
"""
import os
import subprocess
import sys
import time

import pytest
import torch

from dist_helpers import free_port

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_reference_style_rank_maps_to_its_own_gpu(monkeypatch):
    from ddp_amd.utils import local_rank_of, pick_device
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 8)
    monkeypatch.setattr(torch.cuda, "set_device", lambda d: None)
    monkeypatch.delenv("LOCAL_RANK", raising=False)
    for r in range(8):
        assert pick_device("auto", local_rank=local_rank_of(r)) == torch.device("cuda", r)
    # more ranks than GPUs on the node: wrap around (several nodes' worth of ranks)
    assert pick_device("auto", local_rank=local_rank_of(11)) == torch.device("cuda", 3)
    # torchrun: LOCAL_RANK is authoritative
    monkeypatch.setenv("LOCAL_RANK", "5")
    assert pick_device("auto", local_rank=local_rank_of(0)) == torch.device("cuda", 5)


class _Stop(Exception):
    pass


@pytest.mark.parametrize("rank,ndev,expect", [(3, 8, 3), (3, 2, 1), (0, 4, 0)])
def test_apps_main_puts_reference_rank_on_its_gpu(monkeypatch, rank, ndev, expect):
    """``part3/main.py --num-nodes 4 --rank R`` (reference flags, no LOCAL_RANK) selects GPU
    R % ndev before joining the process group: run the real main() with a mocked device count
    and stop it at the rendezvous."""
    from ddp_amd.engine import apps
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(torch.cuda, "device_count", lambda: ndev)
    monkeypatch.setattr(torch.cuda, "set_device", lambda d: None)
    monkeypatch.delenv("LOCAL_RANK", raising=False)
    seen = {}

    def rendezvous(ip, port, r, world, backend="gloo"):
        seen.update(rank=r, world=world)
        raise _Stop

    chosen = []
    real_pick = apps.pick_device
    monkeypatch.setattr(apps, "pick_device", lambda *a, **k: chosen.append(real_pick(*a, **k)) or chosen[-1])
    monkeypatch.setattr(apps, "init_distributed_setup", rendezvous)
    with pytest.raises(_Stop):
        apps.main("part3", ["--num-nodes", "4", "--rank", str(rank), "--master-ip", "127.0.0.1"])
    assert seen == {"rank": rank, "world": 4}
    assert chosen == [torch.device("cuda", expect)]


@pytest.mark.parametrize("n,B,world", [(50000, 256, 1), (50000, 128, 2), (50000, 32, 8),
                                       (50000, 85, 3), (96, 32, 1)])
def test_graph_epoch_covers_exactly_the_eager_samples(n, B, world):
    """The --graph schedule (floor(L/B) replays of B samples + one eager tail of L % B) visits
    exactly the eager loader's batches: same samples, same batch sizes."""
    from ddp_amd.data.loader import shard_indices
    from ddp_amd.engine.trainer import graph_epoch_plan
    for rank in {0, world - 1}:
        idx = shard_indices(n, world, rank)
        L = len(idx)
        eager = [idx[s:s + B] for s in range(0, L, B)]
        nfull, tail = graph_epoch_plan(L, B)
        graph = [idx[i * B:(i + 1) * B] for i in range(nfull)]
        if tail:
            graph.append(idx[nfull * B:nfull * B + tail])
        assert graph == eager
        assert sum(len(b) for b in graph) == L


def _launch(world, extra_env, extra_args, timeout):
    port = free_port()
    env = dict(os.environ, OMP_NUM_THREADS="1", **extra_env)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    procs = []
    for r in range(world):
        cmd = [sys.executable, os.path.join(REPO, "part3", "main.py"), "--num-nodes", str(world),
               "--rank", str(r), "--master-ip", "127.0.0.1", "--master-port", str(port),
               "--device", "cpu", "--global-batch", "12", "--train-size", "96",
               "--test-size", "12", "--max-batches", "6", "--threads", "1", *extra_args]
        procs.append(subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                      text=True, env=env, start_new_session=True))
    t0 = time.monotonic()
    res = []
    try:
        for p in procs:
            left = max(1.0, timeout - (time.monotonic() - t0))
            o, e = p.communicate(timeout=left)
            res.append((p.returncode, o, e, time.monotonic() - t0))
    finally:
        for p in procs:
            if p.poll() is None:
                os.killpg(p.pid, 9)
                p.wait()
    return res


@pytest.mark.parametrize("mode", ["exit", "hang"])
def test_surviving_ranks_exit_nonzero_when_a_peer_fails(mode):
    res = _launch(3, {"DDP_AMD_FAULT_INJECT": f"1:2:{mode}"}, ["--watchdog-s", "8"], timeout=150)
    codes = [r[0] for r in res]
    if mode == "exit":
        assert codes[1] == 17, res[1][2][-2000:]
    for r in (0, 2):
        assert codes[r] != 0, (mode, codes, res[r][2][-2000:])
    # nobody finished the epoch's test pass
    for rc, out, err, _ in res:
        assert "Test set:" not in out
    if mode == "hang":
        # the hung rank's own watchdog ended it (exit 3); its peers were ended by their watchdogs
        # or by the broken connection, well before the 30-min collective timeout
        assert codes[1] == 3, (codes, res[1][2][-2000:])
        assert "watchdog" in res[1][2]
        assert all(r[3] < 120 for r in res)


def test_healthy_run_is_not_killed_by_the_watchdog():
    res = _launch(2, {}, ["--watchdog-s", "60"], timeout=150)
    for rc, out, err, _ in res:
        assert rc == 0, err[-2000:]
        assert "Test set:" in out


def test_rccl_uid_bootstrap_over_the_store():
    """Three ranks, three communicators each (two with the default key): every rank builds each
    communicator from the SAME uid published by rank 0, and no two communicators share one."""
    from dist_helpers import run_workers, uid_bootstrap_worker
    out = run_workers(uid_bootstrap_worker, 3)
    for r, v in out.items():
        assert "error" not in v, v.get("error")
        assert v["live"]
    u0 = out[0]["uids"]
    assert len(set(u0)) == 3
    for r in (1, 2):
        assert out[r]["uids"] == u0
