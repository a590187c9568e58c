"""Backward cut points of the pipelined multi-GPU DDP step, chosen on the node.

The pipelined step (engine/step.py SegmentedDDPStep) cuts the captured backward before some
fused stages; after each segment the comm stream all-reduces that segment's gradient bucket and
runs its share of the SGD while the earlier layers are still back-propagating. Which cuts are
best depends on two measured curves of the machine it runs on:

* how long each fused stage's backward takes at this per-GPU batch (``stage_us``, timed with
  device events on segment graphs cut at EVERY stage: engine/step.py ``profile_stage_times``),
  and
* how long an all-reduce of a bucket takes (the start-up probe's bus-bandwidth rows,
  ``bucket_plan.probe_table``, or ``comm_tuning.json``).

``plan_cuts`` replays the step's two-stream schedule for every candidate cut set and keeps the
one with the earliest finish: the main stream runs segment j, then the comm stream (in bucket
order, one stream) waits for it and runs bucket j's all-reduce + its SGD; every extra cut costs a
graph boundary plus a flag signal / wait (``seg_overhead_us``). The step ends when both the last
segment and the last bucket's update are done; "exposed" = the part of the communication that is
not hidden under the backward.

Reference: torch DDP's fixed 25 MB buckets, rebuilt after iteration 0
(/root/reference/part3/main.py:174); SURVEY.md §5.8 (bucket sizing for 7 xGMI links).
"""
import itertools

from .bucket_plan import predict_us

# Constants fitted on one MI355X (round 5, profiles/r5d_cut_sweep.md): the stand-in cut sweep
# (53 configurations: VGG-11 at 32 / 64 / 128 / 256 images per GPU, 4-7 cut sets, all-reduce,
# sharded and mixed per-bucket plans, 32-CU stand-in collectives at 171 GB/s) against the
# per-stage times of tools/stage_times.py; with these values every configuration is predicted
# within 4.5 % (tests/test_cut_plan.py).
#
# Cost of one segment boundary (graph launch gap + flag signal / wait + the cross-stage fusions
# a cut disables: the consumer conv's fused BatchNorm input, the BN-backward sums in the next
# dgrad). Grows with the per-GPU batch because the disabled fusions move more bytes:
# us = SEG_BOUNDARY_US + SEG_BOUNDARY_US_PER_IMAGE x batch (stage times measured with a cut
# before EVERY stage already contain one boundary each).
SEG_BOUNDARY_US = 14.0
SEG_BOUNDARY_US_PER_IMAGE = 0.035
SEG_OVERHEAD_US = SEG_BOUNDARY_US + SEG_BOUNDARY_US_PER_IMAGE * 32
# fused SGD + bf16 re-pack per fp32 parameter byte (sgd_pack_kernel: 42 us for VGG-11's 36.9 MB)
SGD_US_PER_BYTE = 42.4 / 36.9e6
# the comm stream's flag wait + collective launch, per bucket (fit: 4 us; the pipeline probe,
# profiles/r5c_probe_*.md, shows 2-4 us beyond the modelled collective + SGD on the big buckets)
COMM_OVERHEAD_US = 4.0
# a collective occupies CUs: the backward that runs under it is slowed by this fraction of the
# overlap. Measured with the 32-CU stand-in (tools/pipeline_probe.py: -0.03 .. +0.06 over four
# configurations) and fitted at 0. The stand-in holds its CUs in an s_sleep loop, so a live RCCL
# kernel (which moves its data through the CUs) may contend more: this is the one factor a
# one-GPU box cannot measure.
CONTENTION = 0.0


def seg_boundary_us(per_gpu_batch):
    """Segment-boundary cost at this per-GPU batch (see SEG_BOUNDARY_US)."""
    return SEG_BOUNDARY_US + SEG_BOUNDARY_US_PER_IMAGE * per_gpu_batch


# the sharded bf16-gather update issues one more collective and its shard SGD with the slot
# copies per bucket (fitted 15 us beyond the two modelled collectives + 1/w SGD; the pipeline
# probe shows 20-25 us including that SGD)
SHARD16_EXTRA_US = 15.0
# ... and the step-tail launch after the last bucket (fitted 0: it replaces the signal launch)
SHARD16_TAIL_US = 0.0
# the optimizer update on the comm stream is a memory-bound pass: the backward running beside
# it slows by this fraction of the overlap (fitted 0 on the sweep)
SGD_CONTENTION = 0.0


def shard16_us(rows, fp32_bytes, world):
    """Reduce-scatter of ``fp32_bytes`` of gradients + all-gather of the bucket's bf16 operand
    image (half the bytes). Measured columns of the start-up probe (``rs_us`` / ``ag16_us``,
    parallel/commbench.py shard_sweep) when present, else the ring model: a reduce-scatter or an
    all-gather of S input bytes moves half an all-reduce's traffic, t = 0.5 x t_allreduce(S)."""
    if not rows:
        return 0.0
    if all("rs_us" in r and "ag16_us" in r for r in rows):
        return _interp(rows, fp32_bytes, "rs_us") + _interp(rows, fp32_bytes, "ag16_us")
    return 0.5 * predict_us(rows, fp32_bytes) + 0.5 * predict_us(rows, fp32_bytes // 2)


def _interp(rows, nbytes, key):
    """Column ``key`` (us) at ``nbytes``: linear in size between rows, proportional beyond."""
    rs = sorted(rows, key=lambda r: r["bytes"])
    if nbytes <= rs[0]["bytes"]:
        return rs[0][key]
    for a, b in zip(rs, rs[1:]):
        if nbytes <= b["bytes"]:
            t = (nbytes - a["bytes"]) / (b["bytes"] - a["bytes"])
            return a[key] * (1 - t) + b[key] * t
    return rs[-1][key] * nbytes / rs[-1]["bytes"]


def bucket_costs(rows, pb, wire_scale, world, sgd):
    """(all-reduce plan, sharded plan) of one bucket of ``pb`` fp32 parameter bytes, each as
    (collective us, update us)."""
    wire = int(pb * wire_scale)
    ar = (predict_us(rows, wire) if rows else 0.0, sgd(pb))
    s16 = (shard16_us(rows, pb, world), sgd(pb) / max(world, 1) + SHARD16_EXTRA_US)
    return ar, s16


def _overlap(a, b, spans):
    return sum(max(0.0, min(b, e) - max(a, s)) for s, e in spans)


def schedule(stage_us, param_bytes, cuts, rows, wire_scale=1.0, head_bytes=0,
             seg_overhead_us=SEG_OVERHEAD_US, sgd_us=None, comm_overhead_us=COMM_OVERHEAD_US,
             contention=CONTENTION, update="allreduce", world=8,
             shard16_tail_us=None, sgd_contention=None):
    """Replay one pipelined step with cuts before the stages in ``cuts``.

    stage_us[i]: backward time of fused stage i (stage S-1's entry also carries the forward and
    the classifier head: every candidate's first segment contains it). param_bytes[i]: fp32
    bytes of stage i's parameters (head_bytes: the classifier's, in the first bucket).
    wire_scale: wire bytes per fp32 byte (0.5 for a bf16 wire). sgd_us(bytes) -> update time
    (default: SGD_US_PER_BYTE). ``update``: "allreduce" (all-reduce + replicated SGD per
    bucket), "shard16" (reduce-scatter + 1/world SGD + bf16 operand all-gather,
    parallel/zero.py ShardedBf16Update; fp32 gradients only) or "auto" (the cheaper of the two
    per bucket). Returns a dict with the step time, the per-bucket wire bytes, the predicted
    collective time per bucket, the per-bucket plan ("ar" / "s16") and the exposed
    communication time."""
    S = len(stage_us)
    cuts = sorted(set(int(c) for c in cuts))
    if any(not 0 < c < S for c in cuts):
        raise ValueError(f"cuts must lie in 1..{S - 1}")
    sgd = sgd_us or (lambda b: b * SGD_US_PER_BYTE)
    if shard16_tail_us is None:
        shard16_tail_us = SHARD16_TAIL_US
    if sgd_contention is None:
        sgd_contention = SGD_CONTENTION
    bounds = [S] + cuts[::-1] + [0]
    t_main = 0.0
    free = 0.0
    buckets, ar, busy, plan, sgd_busy = [], [], [], [], []
    free_before_last = 0.0
    forced = None
    if isinstance(update, (list, tuple)):
        forced, update = list(update), "auto"
        if len(forced) != len(bounds) - 1:
            raise ValueError("per-bucket plan does not match the cuts")
    if update not in ("allreduce", "shard16", "auto"):
        raise ValueError("update must be allreduce, shard16, auto or a per-bucket list")
    shard_ok = update != "allreduce" and wire_scale == 1.0 and world > 1
    for j in range(len(bounds) - 1):
        if j == len(bounds) - 2:
            free_before_last = free
        lo, hi = bounds[j + 1], bounds[j]
        # stage_us come from a step cut before EVERY stage (profile_stage_times), so each holds
        # one segment boundary: a segment of several stages saves the boundaries inside it
        seg = sum(stage_us[lo:hi]) - (hi - lo - 1) * seg_overhead_us
        # (one pass: the buckets launched so far slow this segment by their overlap with it)
        t_main += seg + contention * _overlap(t_main, t_main + seg, busy) + \
            sgd_contention * _overlap(t_main, t_main + seg, sgd_busy)
        pb = sum(param_bytes[lo:hi]) + (head_bytes if j == 0 else 0)
        wire = int(pb * wire_scale)
        (t_ar, u_ar), (t_s, u_s) = bucket_costs(rows, pb, wire_scale, world, sgd)
        last = j == len(bounds) - 2
        if last:  # the sharded plan's step tail (small-tensor unpack + re-pack + signal)
            u_s += shard16_tail_us
        code = "ar"
        if forced is not None:
            code = forced[j]
        elif shard_ok and (update == "shard16" or t_s + u_s < t_ar + u_ar):
            code = "s16"
        if code == "s16":
            t_ar, u_ar, wire = t_s, u_s, int(pb * 1.5)
        elif last and forced is not None and "s16" in forced:
            u_ar += shard16_tail_us
        start = max(t_main, free) + comm_overhead_us
        free = start + t_ar + u_ar
        busy.append((start, start + t_ar))
        sgd_busy.append((start + t_ar, free))
        buckets.append(wire)
        ar.append(t_ar)
        plan.append(code)
    end = max(t_main, free)
    # slack: how long before the end of the backward the earlier buckets are all done (a plan
    # that finishes them with margin tolerates a slower collective than the probe measured)
    return {"cuts": cuts, "step_us": end, "backward_us": t_main, "exposed_us": end - t_main,
            "slack_us": t_main - free_before_last, "bucket_bytes": buckets, "allreduce_us": ar,
            "update": plan}


def schedule_inline(stage_us, param_bytes, rows, wire_scale=1.0, head_bytes=0, sgd_us=None):
    """One graph, one bucket all-reduced inline after the whole backward (cuts = [])."""
    sgd = sgd_us or (lambda b: b * SGD_US_PER_BYTE)
    pb = sum(param_bytes) + head_bytes
    wire = int(pb * wire_scale)
    t_ar = predict_us(rows, wire) if rows else 0.0
    t = sum(stage_us)
    return {"cuts": [], "step_us": t + t_ar + sgd(pb), "backward_us": t,
            "exposed_us": t_ar + sgd(pb), "bucket_bytes": [wire], "allreduce_us": [t_ar]}


def plan_cuts(stage_us, param_bytes, rows, wire_scale=1.0, head_bytes=0, max_cuts=3,
              seg_overhead_us=SEG_OVERHEAD_US, sgd_us=None, comm_overhead_us=COMM_OVERHEAD_US,
              tie_us=1.0, candidates=None, contention=CONTENTION, update="allreduce", world=8):
    """Best cut set and the predicted schedules of the candidates: (best_schedule, ranked list
    of (step_us, cuts)). Among the sets within ``tie_us`` of the fastest: the fewest cuts, then
    the most slack (the earlier buckets finish furthest ahead of the end of the backward).
    ``candidates``: restrict the search to these cut sets (default: every set of 1..max_cuts)."""
    S = len(stage_us)
    if S < 2:
        raise ValueError("need at least two stages")
    if candidates is None:
        candidates = [c for k in range(1, min(max_cuts, S - 1) + 1)
                      for c in itertools.combinations(range(1, S), k)]
    cands = []
    for c in candidates:
        c = tuple(sorted(c))
        r = schedule(stage_us, param_bytes, c, rows, wire_scale, head_bytes,
                     seg_overhead_us, sgd_us, comm_overhead_us, contention, update, world)
        cands.append((r["step_us"], len(c), c, r))
    fastest = min(t for t, _, _, _ in cands)
    near = [x for x in cands if x[0] <= fastest + tie_us]
    near.sort(key=lambda x: (x[1], -x[3]["slack_us"], x[0]))
    best = near[0][3]
    ranked = sorted(((round(t, 1), list(c)) for t, _, c, _ in cands))
    return best, ranked


def stand_in_rows(world, algbw_GBps, sizes=None):
    """Bus-bandwidth rows of a fixed-algorithm-bandwidth collective (the one-GPU timed stand-in of
    profiles/r2_pipelined_ddp.md: bytes / algbw), in the comm_tuning.json row format."""
    sizes = sizes or [1 << k for k in range(12, 27)]
    f = 2 * (world - 1) / world
    return [{"bytes": s, "us": s / (algbw_GBps * 1e3), "algbw_GBps": algbw_GBps,
             "busbw_GBps": algbw_GBps * f} for s in sizes]
