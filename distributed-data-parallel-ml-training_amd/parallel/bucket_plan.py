"""Gradient-bucket sizing from an all-reduce bandwidth table.

The reference uses torch DDP's fixed 25 MiB buckets (+1 MiB first bucket,
/root/reference/part3/main.py:174). On MI355X the right size depends on the RCCL bus-bandwidth
curve over xGMI (7 point-to-point links per GPU, a ring uses one per hop): a bucket must be big
enough that the per-collective latency is amortised (bus bandwidth near its plateau), and no
bigger, so that the first bucket starts early and the last one exposes little time.

``comm_tuning.json`` (next to this file) holds one bus-bandwidth-vs-size table per world size
(``tools/comm_bench.py --write-table`` produces measured rows; a row set whose ``source`` is
``"model"`` is a latency + bandwidth model used until a node has been measured). At start-up
``choose_bucket_caps`` picks:

* eager / overlapped reducer: the smallest size whose bus bandwidth reaches ``eff`` (default
  0.8) of the table's plateau, floored at ``floor_bytes`` (7 links x 512 KiB: every link moves
  a >= 512 KiB chunk), as the bucket cap; the first bucket a quarter of it (>= 1 MiB);
* a captured step whose collectives are inline (no overlap to buy): one bucket — a single
  collective has the least total latency.
"""
import bisect
import json
import math
import os

TABLE_FILE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "comm_tuning.json")
MIB = 1 << 20


def load_table(path=None):
    path = path or os.environ.get("DDP_AMD_COMM_TUNING_FILE", TABLE_FILE)
    if not os.path.exists(path):
        return {}
    with open(path) as f:
        return json.load(f)


def rows_for(table, world, dtype="fp32"):
    """(rows sorted by bytes, source) for the largest tabulated world size <= ``world``
    (source reads e.g. "measured table (world 8, fp32)")."""
    worlds = sorted(int(w) for w in table.get("worlds", {}))
    cands = [w for w in worlds if w <= world] or worlds
    if not cands:
        return [], None
    ent = table["worlds"][str(cands[-1])]
    key = dtype if ent.get(dtype) else "fp32"
    rows = ent.get(key) or []
    rows = sorted((r for r in rows if r.get("busbw_GBps")), key=lambda r: r["bytes"])
    return rows, f"{ent.get('source', 'measured')} table (world {cands[-1]}, {key})"


def busbw_at(rows, nbytes):
    """Bus bandwidth at ``nbytes``, interpolated linearly in log2(size)."""
    if not rows:
        raise ValueError("empty table")
    xs = [math.log2(r["bytes"]) for r in rows]
    x = math.log2(max(nbytes, 1))
    i = bisect.bisect_left(xs, x)
    if i == 0:
        return rows[0]["busbw_GBps"]
    if i >= len(xs):
        return rows[-1]["busbw_GBps"]
    t = (x - xs[i - 1]) / (xs[i] - xs[i - 1])
    return rows[i - 1]["busbw_GBps"] * (1 - t) + rows[i]["busbw_GBps"] * t


def knee_bytes(rows, eff=0.8):
    """Smallest tabulated size (log-interpolated) whose bus bandwidth is >= eff x plateau."""
    peak = max(r["busbw_GBps"] for r in rows)
    prev = None
    for r in rows:
        if r["busbw_GBps"] >= eff * peak:
            if prev is None:
                return r["bytes"]
            # interpolate in log2(size) between prev (below) and r (above)
            y0, y1 = prev["busbw_GBps"], r["busbw_GBps"]
            t = (eff * peak - y0) / max(y1 - y0, 1e-12)
            x = math.log2(prev["bytes"]) + t * (math.log2(r["bytes"]) - math.log2(prev["bytes"]))
            return int(2 ** x)
        prev = r
    return rows[-1]["bytes"]


def choose_bucket_caps(world, total_bytes, overlap=True, dtype="fp32", table=None, eff=0.8,
                       floor_bytes=7 * 512 * 1024):
    """Return (cap_bytes, first_cap_bytes, why). ``total_bytes`` = gradient bytes on the wire."""
    if not overlap or world <= 1:
        return total_bytes, total_bytes, "single bucket (collectives inline: no overlap to buy)"
    table = load_table() if table is None else table
    rows, source = rows_for(table, world, dtype)
    if not rows:
        return 25 * MIB, 1 * MIB, "no comm table: torch DDP defaults"
    knee = knee_bytes(rows, eff)
    cap = max(knee, floor_bytes)
    cap = min(cap, max(total_bytes, floor_bytes))
    first = max(1 * MIB, cap // 4)
    return int(cap), int(first), f"{source}: {eff:.0%} of plateau at {knee / MIB:.2f} MiB"


def model_rows(world, latency_us=12.0, link_GBps=153.0, links_used=1, sizes=None):
    """Latency + bandwidth model of a ring all-reduce: t = latency + 2 (n-1)/n S / (links x
    link_GBps) -> bus bandwidth rows in the comm_bench format (source "model")."""
    sizes = sizes or [1 << k for k in range(16, 28, 2)]
    rows = []
    for s in sizes:
        t_us = latency_us + 2 * (world - 1) / world * s / (links_used * link_GBps * 1e3)
        alg = s / t_us / 1e3
        rows.append({"bytes": s, "us": round(t_us, 2), "algbw_GBps": round(alg, 3),
                     "busbw_GBps": round(alg * 2 * (world - 1) / world, 3)})
    return rows


def probe_table(comm, world, dtype="fp32", device="cuda", sizes=None, iters=10, warmup=3):
    """Measure the all-reduce bus-bandwidth curve on the live communicator (every rank takes
    part; per-size time = the max over ranks, so all ranks build the same table) and return it
    in the comm_tuning.json layout with source "measured at start-up". ~50 ms on a node."""
    import torch
    from .commbench import allreduce_sweep
    sizes = sizes or [1 << k for k in range(18, 27, 2)]  # 256 KiB .. 64 MiB
    dt = torch.bfloat16 if dtype == "bf16" else torch.float32
    rows = allreduce_sweep(comm, sizes, dtype=dt, device=device, iters=iters, warmup=warmup)
    ok = all(r.get("correct", True) for r in rows)
    # decide together: a rank that raised alone would leave its peers blocked in the next
    # collective (a late watchdog failure instead of this clear error)
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        flag = torch.tensor([1 if ok else 0], dtype=torch.int64)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        ok = bool(flag.item())
    if not ok:
        raise RuntimeError("start-up all-reduce probe returned wrong sums (on at least one rank)")
    rows = [{k: r[k] for k in ("bytes", "us", "algbw_GBps", "busbw_GBps")} for r in rows]
    if dtype == "fp32" and os.environ.get("DDP_AMD_SHARD_PROBE", "1") != "0":
        # the sharded update's collectives at the same bucket sizes (parallel/cut_plan.py
        # shard16_us prices it from these columns instead of the half-all-reduce model)
        from .commbench import shard_sweep
        sh = {r["bytes"]: r for r in shard_sweep(comm, [r["bytes"] for r in rows], device=device,
                                                  iters=iters, warmup=warmup)}
        for r in rows:
            if r["bytes"] in sh:
                r["rs_us"], r["ag16_us"] = sh[r["bytes"]]["rs_us"], sh[r["bytes"]]["ag16_us"]
    return {"worlds": {str(world): {"source": "measured at start-up", dtype: rows}}}


def predict_us(rows, nbytes):
    """All-reduce time of ``nbytes`` from bus-bandwidth rows (ring: bus = alg x 2(n-1)/n is
    folded into the rows' own us where a row matches; interpolated otherwise)."""
    for r in rows:
        if r["bytes"] == nbytes:
            return r["us"]
    ref = rows[-1]
    scale = ref["busbw_GBps"] / max(ref["algbw_GBps"], 1e-12)  # 2(n-1)/n
    return nbytes * scale / (busbw_at(rows, nbytes) * 1e3)


def merge_rows(path, world, dtype, rows, source="measured"):
    """Write measured comm_bench rows for (world, dtype) into the table at ``path``."""
    table = load_table(path) if os.path.exists(path) else {}
    ent = table.setdefault("worlds", {}).setdefault(str(world), {})
    if ent.get("source") == "model":
        ent.clear()  # measured rows replace the model for this world size entirely
    ent["source"] = source
    ent[dtype] = [{k: r[k] for k in ("bytes", "us", "algbw_GBps", "busbw_GBps", "rs_us",
                                     "ag16_us") if k in r}
                  for r in rows if r.get("correct", True)]
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        json.dump(table, f, indent=1)
    os.replace(tmp, path)
    return table
