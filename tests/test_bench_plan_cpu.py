"""bench.py's per-bucket update plan of the pipelined multi-GPU step (``choose_update``), CPU only:
the multi-GPU branch the driver's scaling run takes, exercised without GPUs. Plans: "ar" =
all-reduce + replicated SGD, "s16" = reduce-scatter + shard SGD + bf16 operand all-gather
(parallel/zero.py ShardedBf16Update), priced by parallel/cut_plan.py bucket_costs on the start-up
probe's rows. Reference: DDP's bucketed all-reduce, /root/reference/part3/main.py:174."""
import argparse
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402


class _Model:
    def __init__(self):
        from ddp_amd.models import VGG11
        from ddp_amd.optim.arena import ParamArena
        self.module = VGG11()
        self.arena = ParamArena(list(self.module.parameters()), krsc=False)


def _args(update="auto", grad_comm="fp32", zero=False):
    return argparse.Namespace(update=update, grad_comm=grad_comm, zero=zero)


def _table(world, rs_scale):
    """A probe table in bench's layout: all-reduce rows of a 300 GB/s-bus ring + 10 us latency,
    reduce-scatter / all-gather columns = rs_scale x half the all-reduce time."""
    rows = []
    for k in range(18, 27, 2):
        b = 1 << k
        us = 10.0 + 2 * (world - 1) / world * b / 300e3
        alg = b / us / 1e3
        rows.append({"bytes": b, "us": us, "algbw_GBps": alg,
                     "busbw_GBps": alg * 2 * (world - 1) / world,
                     "rs_us": rs_scale * 0.5 * us, "ag16_us": rs_scale * 0.5 * (10.0 + (us - 10.0) / 2)})
    return {"worlds": {str(world): {"source": "measured at start-up", "fp32": rows}}}


def test_auto_shards_the_big_buckets_on_eight_ranks():
    m = _Model()
    plan = bench.choose_update(_args(), m, [3, 6], 8, _table(8, 1.0), None, 8)
    assert plan["update"][:2] == ["s16", "s16"], plan
    assert len(plan["bucket_costs"]) == 3 and plan["source"].startswith("priced on")


def test_auto_keeps_all_reduce_when_the_probe_says_sharding_is_slow():
    m = _Model()
    plan = bench.choose_update(_args(), m, [3, 6], 8, _table(8, 3.0), None, 8)
    assert plan["update"] == ["ar", "ar", "ar"], plan


def test_single_rank_bf16_wire_and_zero_never_shard():
    m = _Model()
    assert bench.choose_update(_args(), m, [3, 6], 1, None, None, 1)["update"] == ["ar"] * 3
    assert bench.choose_update(_args(grad_comm="bf16"), m, [3, 6], 8, _table(8, 1.0), None,
                               8)["update"] == ["ar"] * 3
    assert bench.choose_update(_args(zero=True), m, [3, 6], 8, _table(8, 1.0), None,
                               8)["update"] == ["ar"] * 3


def test_forced_and_planned_plans():
    m = _Model()
    assert bench.choose_update(_args("shard16"), m, [3, 6], 4, None, None, 4)["update"] == ["s16"] * 3
    assert bench.choose_update(_args("allreduce"), m, [3, 6], 4, None, None, 4)["update"] == ["ar"] * 3
    assert bench.choose_update(_args("s16,ar,ar"), m, [3, 6], 4, None, None, 4)["update"] == \
        ["s16", "ar", "ar"]
    with pytest.raises(SystemExit):
        bench.choose_update(_args("s16,ar"), m, [3, 6], 4, None, None, 4)
    cut_plan = {"cuts": [3, 6], "update": ["s16", "ar", "ar"]}
    got = bench.choose_update(_args(), m, [3, 6], 8, _table(8, 1.0), cut_plan, 8)
    assert got == {"update": ["s16", "ar", "ar"], "source": "cut planner"}


@pytest.mark.parametrize("world", [3, 5, 6, 7])
def test_sharding_only_where_every_bucket_divides(world):
    m = _Model()
    a = m.arena
    pidx = {id(p): i for i, p in enumerate(a.params)}
    firsts = sorted(pidx[id(m.module.first_param_of_stage(c))] for c in (3, 6))
    bounds = [a.offsets[f] for f in firsts] + [a.total]
    sizes = [bounds[0]] + [y - x for x, y in zip(bounds, bounds[1:])]
    even = all(n % world == 0 and (n // world) % 4 == 0 for n in sizes)
    plan = bench.choose_update(_args(), m, [3, 6], world, _table(world, 1.0), None, world)
    if not even:
        assert plan["update"] == ["ar"] * 3
        with pytest.raises(SystemExit):
            bench.choose_update(_args("shard16"), m, [3, 6], world, None, None, world)
    else:
        assert "s16" in plan["update"]


def test_auto_never_shards_without_measured_shard_columns():
    """--update auto may choose s16 only from THIS node's measured reduce-scatter / all-gather
    times (advisor round 5): the model table or a probe without those columns -> all-reduce."""
    m = _Model()
    t = _table(8, 1.0)
    for r in t["worlds"]["8"]["fp32"]:
        del r["rs_us"], r["ag16_us"]
    plan = bench.choose_update(_args(), m, [3, 6], 8, t, None, 8)
    assert plan["update"] == ["ar"] * 3 and "measured" in plan["source"]
    assert bench.choose_update(_args(), m, [3, 6], 8, None, None, 8)["update"] == ["ar"] * 3
    assert not bench.shard_columns_measured(None, 8)
    assert bench.shard_columns_measured(_table(8, 1.0), 8)
