"""Sync-strategy equivalence on CPU with Gloo, world size 2.

2A (gather/mean/scatter, and the gather/mean/broadcast variant) == 2B (all-reduce/ws) == 3 (bucketed DDP) == the average of the
per-rank gradients, and every strategy leaves the replicas bit-identical.
"""
import pytest
import torch

from dist_helpers import run_workers, train_worker, local_grad_worker

WORLD = 2
STEPS = 2
B = 4


@pytest.fixture(scope="module")
def results():
    out = {}
    for strat in ["gather_scatter", "gather_broadcast", "allreduce", "ddp"]:
        out[strat] = run_workers(train_worker, WORLD, strat, STEPS, B, 4.0)
        for r, v in out[strat].items():
            assert "error" not in v, v.get("error")
    out["ddp_bf16"] = run_workers(train_worker, WORLD, "ddp_bf16", STEPS, B, 4.0)
    for r, v in out["ddp_bf16"].items():
        assert "error" not in v, v.get("error")
    out["local"] = run_workers(local_grad_worker, WORLD, B)
    return out


def test_replicas_identical_every_strategy(results):
    for strat in ["gather_scatter", "gather_broadcast", "allreduce", "ddp"]:
        r = results[strat]
        assert torch.equal(r[0]["params"], r[1]["params"]), strat
        assert torch.equal(r[0]["grads0"], r[1]["grads0"]), strat


def test_synced_grad_is_mean_of_local_grads(results):
    loc = results["local"]
    expected = (loc[0]["grads0"] + loc[1]["grads0"]) / WORLD
    for strat in ["gather_scatter", "gather_broadcast", "allreduce", "ddp"]:
        g = results[strat][0]["grads0"]
        assert torch.allclose(g, expected, rtol=1e-5, atol=1e-7), strat


def test_strategies_agree(results):
    a = results["gather_scatter"][0]["params"]
    for strat in ["gather_broadcast", "allreduce", "ddp"]:
        assert torch.allclose(results[strat][0]["params"], a, rtol=1e-5, atol=1e-6), strat


def test_ddp_buckets_cover_all_params_in_reverse(results):
    buckets = results["ddp"][0]["buckets"]
    assert len(buckets) > 1
    covered = []
    for s, e, _, _ in buckets:
        covered += list(range(s, e))
    assert sorted(covered) == list(range(34))
    assert buckets[0][1] == 34  # first bucket holds the LAST parameters (ready first)
    assert results["ddp"][0]["consistent"] is True


def test_ddp_bf16_grad_comm(results):
    """grad_comm_dtype="bf16": replicas stay bit-identical and the synced gradient is the
    mean of the local gradients up to bf16 rounding of the communicated values."""
    r = results["ddp_bf16"]
    assert torch.equal(r[0]["params"], r[1]["params"])
    assert r[0]["consistent"] is True
    loc = results["local"]
    expected = (loc[0]["grads0"] + loc[1]["grads0"]) / WORLD
    g = r[0]["grads0"]
    rel = float((g - expected).norm() / expected.norm())
    assert 0 < rel < 1e-2, rel
    # the communicated values were bf16: the result carries at most 8 significant bits + 1 add
    assert not torch.equal(g, results["ddp"][0]["grads0"])


def test_ddp_no_sync_accumulation():
    """DDP.no_sync: the first backward accumulates locally (no communication, replicas differ),
    the next one all-reduces the accumulated gradient = mean over ranks of (g1 + g2)."""
    from dist_helpers import nosync_worker
    out = run_workers(nosync_worker, WORLD, B)
    for r, v in out.items():
        assert "error" not in v, v.get("error")
    assert not torch.allclose(out[0]["after_nosync"], out[1]["after_nosync"])
    for r in range(WORLD):
        assert torch.allclose(out[r]["ddp"], out[r]["manual"], rtol=1e-4, atol=1e-6)
    assert torch.equal(out[0]["ddp"], out[1]["ddp"])


def test_ddp_broadcast_buffers_flat():
    """Buffers (BN running statistics) are broadcast from rank 0 before every forward as one
    collective per dtype, so every replica's forward starts from rank 0's running statistics
    (the forward's own momentum update then mixes in each rank's batch statistics)."""
    from dist_helpers import buffers_worker
    out = run_workers(buffers_worker, WORLD)
    for r, v in out.items():
        assert "error" not in v, v.get("error")
        assert v["flat"] is True
    b0 = {k: torch.as_tensor(v) for k, v in out[0]["bufs"].items()}
    b1 = {k: torch.as_tensor(v) for k, v in out[1]["bufs"].items()}
    # both ranks started the forward from rank 0's statistics (mean filled with 1.0, var 10.0);
    # the forward's own update then mixes in each rank's batch statistics with momentum 0.1
    for k in b0:
        if k.endswith("num_batches_tracked"):
            assert torch.equal(b0[k], b1[k])
    assert float(b1["1.running_mean"].mean()) < 1.5  # started from rank 0's 1.0, not rank 1's 2.0
    assert float(b1["4.running_var"].mean()) < 15.0  # started from 10.0, not 20.0


def test_allreduce_bandwidth_sweep():
    """parallel/commbench.py (the tools/comm_bench.py sweep) on Gloo: correct sums, positive
    timings, the same (max-over-ranks) numbers on every rank."""
    from dist_helpers import commbench_worker
    out = run_workers(commbench_worker, WORLD)
    for r, v in out.items():
        assert "error" not in v, v.get("error")
        assert [row["bytes"] for row in v["rows"]] == [1 << 12, 1 << 16]
        for row in v["rows"]:
            assert row["correct"] and row["us"] > 0 and row["busbw_GBps"] > 0
    assert out[0]["rows"] == out[1]["rows"]


def test_startup_probe_table_plans_buckets():
    """bench.py --gpus N>1 measures the all-reduce curve on its own communicator before planning
    buckets (bucket_plan.probe_table): every rank gets the SAME table (max over ranks), marked
    "measured at start-up", and DDP's 'auto' caps are planned from it."""
    from dist_helpers import probe_worker
    out = run_workers(probe_worker, WORLD)
    for r, v in out.items():
        assert "error" not in v, v.get("error")
        assert v["src"].startswith("measured at start-up table (world 2")
        assert "measured at start-up" in v["reason"]
        rows = v["table"]["worlds"]["2"]["fp32"]
        assert [row["bytes"] for row in rows] == [1 << 14, 1 << 16, 1 << 18]
        assert v["pred"] == rows[1]["us"] and v["pred_mid"] > 0
        assert v["nb"] >= 1
    assert out[0]["table"] == out[1]["table"]
