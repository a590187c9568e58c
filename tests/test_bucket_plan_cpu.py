"""Bucket sizing from the all-reduce bandwidth table (parallel/bucket_plan.py)
with synthetic tables: knee detection, world-size fallback, the inline single-bucket rule, the
reference fallback without a table, table merging (tools/comm_bench.py --write-table) and the
DDP wrapper's ``bucket_cap_mb="auto"``."""
import json

import pytest
import torch

from ddp_amd.parallel import bucket_plan as bp

MIB = 1 << 20


def _table(world, plateau=300.0, half=4 * MIB, source="measured"):
    # saturating curve busbw = plateau * S / (S + half): 80% of the plateau at S = 4 * half
    rows = [{"bytes": 1 << k, "busbw_GBps": plateau * (1 << k) / ((1 << k) + half)}
            for k in range(14, 29)]
    return {"worlds": {str(world): {"source": source, "fp32": rows}}}


def test_knee_is_80_percent_of_plateau():
    t = _table(8, half=2 * MIB)
    rows, src = bp.rows_for(t, 8)
    assert src == "measured table (world 8, fp32)"
    k = bp.knee_bytes(rows, 0.8)
    assert 6 * MIB <= k <= 9 * MIB  # analytic: 8 MiB (log-interpolated between table points)
    assert bp.busbw_at(rows, k) >= 0.78 * max(r["busbw_GBps"] for r in rows)
    cap, first, why = bp.choose_bucket_caps(8, 36_920_000, table=t)
    assert cap == pytest.approx(k, rel=1e-6) and first == max(MIB, cap // 4)
    assert "measured" in why


def test_floor_fallback_and_inline_rules():
    # a very flat curve: the knee is tiny, the 7-link x 512 KiB floor wins
    cap, first, _ = bp.choose_bucket_caps(8, 36_920_000, table=_table(8, half=1024))
    assert cap == 7 * 512 * 1024 and first == MIB
    # world 4 is not tabulated: the largest smaller world's rows (2) are used
    t = _table(2, half=MIB)
    cap4, _, why = bp.choose_bucket_caps(4, 36_920_000, table=t)
    assert "world 2" in why and cap4 == pytest.approx(bp.knee_bytes(bp.rows_for(t, 2)[0]))
    # inline collectives (captured step) or one rank: one bucket
    assert bp.choose_bucket_caps(8, 1234, overlap=False, table=t)[:2] == (1234, 1234)
    assert bp.choose_bucket_caps(1, 1234, table=t)[:2] == (1234, 1234)
    # no table: torch DDP's defaults (the reference, part3/main.py:174)
    assert bp.choose_bucket_caps(8, 36_920_000, table={})[:2] == (25 * MIB, MIB)


def test_merge_rows_replaces_model(tmp_path):
    p = tmp_path / "t.json"
    p.write_text(json.dumps({"worlds": {"8": {"source": "model", "fp32": [], "bf16": []}}}))
    rows = [{"bytes": 1 << 20, "us": 10.0, "algbw_GBps": 100.0, "busbw_GBps": 175.0, "correct": True},
            {"bytes": 1 << 22, "us": 1.0, "algbw_GBps": 1.0, "busbw_GBps": 1.0, "correct": False}]
    t = bp.merge_rows(str(p), 8, "fp32", rows)
    ent = json.loads(p.read_text())["worlds"]["8"]
    assert ent["source"] == "measured" and "bf16" not in ent
    assert ent["fp32"] == [{"bytes": 1 << 20, "us": 10.0, "algbw_GBps": 100.0, "busbw_GBps": 175.0}]
    assert t["worlds"]["8"] == ent


def test_checked_in_table_and_model():
    t = bp.load_table()
    for w in ("2", "4", "8"):
        assert t["worlds"][w]["fp32"]
    rows = bp.model_rows(8)
    assert rows[-1]["busbw_GBps"] > rows[0]["busbw_GBps"]
    cap, first, why = bp.choose_bucket_caps(8, 36_920_000)
    assert 7 * 512 * 1024 <= cap <= 36_920_000 and MIB <= first <= cap


def test_ddp_auto_bucket_caps(monkeypatch, tmp_path):
    """DistributedDataParallel(bucket_cap_mb="auto") sizes its buckets from the table (CPU,
    world 1 -> one bucket; a fake world-8 communicator -> several buckets of <= the cap)."""
    from ddp_amd.models import VGG11
    from ddp_amd.parallel import DistributedDataParallel

    class FakeComm:
        world, rank = 8, 0

        def all_reduce_async(self, t):
            raise AssertionError("not used")

        def broadcast(self, t, root):  # construction-time parameter broadcast: no-op here
            return t

    p = tmp_path / "t.json"
    p.write_text(json.dumps(_table(8, half=MIB)))
    monkeypatch.setenv("DDP_AMD_COMM_TUNING_FILE", str(p))
    torch.manual_seed(0)
    m = DistributedDataParallel(VGG11(), FakeComm(), bucket_cap_mb="auto", first_bucket_cap_mb="auto")
    knee = bp.knee_bytes(bp.rows_for(_table(8, half=MIB), 8)[0])
    assert "measured table (world 8" in m.bucket_plan_reason
    assert len(m.buckets) > 3
    biggest_multi = max(c * 4 for s, e, _, c in m.buckets if e - s > 1)
    assert biggest_multi <= knee + 64 * 4
