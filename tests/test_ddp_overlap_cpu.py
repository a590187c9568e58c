"""Bucketed DDP scheduling on CPU (reference DDP: part3/main.py:174).

* the native C++ readiness/launch state machine (csrc/runtime/buckets.h BucketScheduler, the
  one the GPU Reducer runs) and its Python twin (parallel/ddp.py) produce identical launch
  sequences, logs and rebuilt orders for the same hook orders;
* on Gloo (2 ranks) each bucket's all-reduce is launched from the gradient hooks while the rest
  of the backward is still running (launch log: parameters marked at launch < all), and after
  iteration 0 the launch order is rebuilt from the observed gradient-ready order (torch DDP's
  bucket rebuild), identically on every rank, with replicas staying bit-identical.
"""
import random

import pytest
import torch

from dist_helpers import overlap_worker, run_workers

VGG_NUMELS = [1728, 64, 64, 64, 73728, 128, 128, 128, 294912, 256, 256, 256, 589824, 256, 256,
              256, 1179648, 512, 512, 512, 2359296, 512, 512, 512, 2359296, 512, 512, 512,
              2359296, 512, 512, 512, 5120, 10]


def _offsets(numels):
    out, off = [], 0
    for n in numels:
        out.append(off)
        off += (n + 63) // 64 * 64
    return out


@pytest.fixture(scope="module")
def native_cpu():
    from ddp_amd.ops.common import native
    return native()


def _drive(s, seq):
    launches = []
    for p in seq:
        launches += list(s.mark(p))
    launches += list(s.finish())
    return launches


@pytest.mark.parametrize("cap_mb", [1, 4, 25, 256])
def test_native_scheduler_matches_python_twin(native_cpu, cap_mb):
    from ddp_amd.parallel.ddp import BucketScheduler, plan_buckets
    offs = _offsets(VGG_NUMELS)
    plan = plan_buckets(offs, VGG_NUMELS, 4, cap_mb << 20, 1 << 20)
    assert [tuple(b) for b in native_cpu.plan_buckets(offs, VGG_NUMELS, 4, cap_mb << 20, 1 << 20)] == plan
    n = len(VGG_NUMELS)
    rng = random.Random(cap_mb)
    cpp, py = native_cpu.BucketScheduler(plan, n), BucketScheduler(plan, n)
    for it in range(6):
        if it == 0:
            seq = list(range(n - 1, -1, -1))  # the backward's natural order
        else:
            seq = list(range(n))
            rng.shuffle(seq)
        assert _drive(cpp, seq) == _drive(py, seq)
        assert list(cpp.ready_order()) == py.ready_order() == seq
        assert [tuple(x) for x in cpp.launch_log()] == py.launch_log()
        o1, o2 = list(cpp.order_from_ready(seq)), py.order_from_ready(seq)
        assert o1 == o2 and sorted(o1) == list(range(len(plan)))
        if it % 2:  # alternate between a rebuilt order and the plan order
            cpp.set_launch_order(o1)
            py.set_launch_order(o2)
        else:
            cpp.set_launch_order(list(range(len(plan))))
            py.set_launch_order(list(range(len(plan))))
    # the natural backward order launches each bucket the moment its last gradient arrives
    cpp.set_launch_order(list(range(len(plan))))
    _drive(cpp, list(range(n - 1, -1, -1)))
    marks = [m for _, m in cpp.launch_log()]
    assert marks == sorted(marks) and marks[-1] == n
    if len(plan) > 1:
        assert marks[0] < n


def test_scheduler_rejects_misuse(native_cpu):
    from ddp_amd.parallel.ddp import BucketScheduler, plan_buckets
    offs = _offsets(VGG_NUMELS)
    plan = plan_buckets(offs, VGG_NUMELS, 4, 4 << 20, 1 << 20)
    for s in (native_cpu.BucketScheduler(plan, len(VGG_NUMELS)),
              BucketScheduler(plan, len(VGG_NUMELS))):
        s.mark(33)
        with pytest.raises(RuntimeError, match="twice"):
            s.mark(33)
        with pytest.raises(RuntimeError, match="never produced"):
            s.finish()
        s.prepare()
        with pytest.raises(RuntimeError, match="permutation"):
            s.set_launch_order([0] * len(plan))
    with pytest.raises(RuntimeError):
        native_cpu.BucketScheduler([(0, 2, 0, 10)], 3)  # parameter 2 in no bucket


def test_ddp_rebuilds_launch_order_after_iteration0():
    """Parameters registered opposite to their use: iteration 0 launches the bucket that
    completed first only at the end (plan order); after the rebuild it launches first, on every
    rank; gradients stay the rank average (replicas identical)."""
    out = run_workers(overlap_worker, 2, "swapped")
    for r, v in out.items():
        assert "error" not in v, v.get("error")
    v = out[0]
    nb, np_ = v["n_buckets"], v["n_params"]
    assert nb == np_ == 4
    log0, log1 = v["logs"][0], v["logs"][1]
    # iteration 0 (plan order 0..3 = reverse parameter order): early.* grads arrive last
    assert v["orders"][0] == [0, 1, 2, 3]
    # the plan's first buckets (early.*) complete last, the late.* buckets wait behind them
    assert [m for _, m in log0][0] >= 3 and [m for _, m in log0][2:] == [4, 4]
    # rebuilt: completion order, identical on both ranks, first launch after 1 mark
    assert v["orders"][1] == out[1]["orders"][1] != [0, 1, 2, 3]
    assert sorted(v["orders"][1]) == [0, 1, 2, 3]
    assert log1[0][1] == 1 and [b for b, _ in log1] == v["orders"][1]
    assert v["consistent"] and out[1]["consistent"]
    assert torch.equal(out[0]["params"], out[1]["params"])


def test_ddp_vgg_buckets_launch_during_backward():
    """VGG-11, 4 MiB buckets (+1 MiB first) on Gloo: every bucket but the last is launched
    (async all-reduce) while later gradients are still being computed."""
    out = run_workers(overlap_worker, 2, "vgg")
    for r, v in out.items():
        assert "error" not in v, v.get("error")
    v = out[0]
    for log in v["logs"]:
        marks = [m for _, m in log]
        assert len(marks) == v["n_buckets"] > 2
        assert marks[0] < v["n_params"] and marks[-2] < v["n_params"]
    # rebuilt from the observed order (ATen's conv backward finishes the weight before the
    # bias, so a weight-only bucket can complete before the bucket in front of it)
    assert v["orders"][1] == out[1]["orders"][1]
    assert sorted(v["orders"][1]) == list(range(v["n_buckets"]))
    assert v["logs"][1][0][1] <= v["logs"][0][0][1]
    assert torch.equal(out[0]["params"], out[1]["params"])
