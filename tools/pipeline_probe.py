"""Where does the pipelined multi-GPU step's time go? (one GPU, timed stand-in collectives)

    python tools/pipeline_probe.py --batch 32 --cuts 3,6 --update shard16 --gbps 171

Builds the bench.py configuration (VGG-11, on-device data, DDP wrapper, fused SGD) and the
pipelined step (engine/step.py SegmentedDDPStep) with 32-CU stand-in collectives lasting their
modelled time at ``--gbps`` (8-GPU all-reduce algorithm bandwidth), then measures:

* ``wall_ms``: back-to-back replayed steps (what bench.py times), and ``host_ms``: the host's
  own enqueue time per step in that loop (host-bound when it approaches wall_ms);
* a device timeline from HIP timing events recorded in the same back-to-back stream of steps:
  every segment graph on the main stream, every bucket's comm-stream work (stand-in
  collective(s) + update) — start / end relative to the step's first segment;
* the same segments with NO collective (``--gbps 0``-style run of the identical step) to
  measure how much the stand-ins slow the backward running beside them (``contention``) and
  the per-bucket comm-stream overhead beyond the modelled collective time (``comm_overhead``),
  the two constants of parallel/cut_plan.py.
Prints markdown tables and one JSON line.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def build(a, gbps, update):
    import torch
    import ddp_amd
    from ddp_amd.data import SyntheticCIFAR10, DeviceLoader
    from ddp_amd.engine import SegmentedDDPStep, CrossEntropyLoss
    from ddp_amd.models import build as build_model
    from ddp_amd.optim import FusedSGD
    from ddp_amd.parallel import DistributedDataParallel, RcclCommunicator
    torch.manual_seed(ddp_amd.SEED)
    dev = torch.device("cuda", 0)
    loader = DeviceLoader(SyntheticCIFAR10(True), a.batch, dev, 1, 0, train=True, cpad=8)
    model = DistributedDataParallel(build_model(a.model).to(dev), RcclCommunicator(0, 1, 0),
                                    bucket_cap_mb=256.0, first_bucket_cap_mb=256.0,
                                    captured=True)
    opt = FusedSGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    st = SegmentedDDPStep(model, opt, CrossEntropyLoss(), loader,
                          split=[int(v) for v in a.cuts.split(",")], emulate_gbps=gbps,
                          emulate=0, update=update, emulate_world=a.world,
                          emulate_passes=a.passes)
    st.warmup(2)
    st.capture()
    return st


def measure(st, steps, probe_steps):
    import torch
    main = torch.cuda.current_stream()
    T = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    for _ in range(10):
        st.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        st.step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    wall_ms, host_ms = (t2 - t0) * 1e3 / steps, (t1 - t0) * 1e3 / steps
    # timeline of back-to-back steps (no host sync between them)
    rows = []
    st.probe = []
    for _ in range(probe_steps):
        evs = []
        st.step(seg_events=evs)
        rows.append(evs)
    torch.cuda.synchronize()
    probe, st.probe = st.probe, None
    nb = len(st.buckets)
    out = []
    for k, evs in enumerate(rows):
        ref = evs[0]
        segs = [(ref.elapsed_time(evs[i]), ref.elapsed_time(evs[i + 1])) for i in range(len(evs) - 1)]
        comm = [(j, ref.elapsed_time(s), ref.elapsed_time(e)) for j, s, e in probe[k * nb:(k + 1) * nb]]
        out.append({"segments": segs, "comm": comm})
    _ = main
    return wall_ms, host_ms, out


def median(v):
    v = sorted(v)
    return v[len(v) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="vgg11")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--cuts", default="3,6")
    ap.add_argument("--update", default="shard16", choices=["allreduce", "shard16"])
    ap.add_argument("--gbps", type=float, default=171.0)
    ap.add_argument("--world", type=int, default=8, help="emulated world of the sharded update")
    ap.add_argument("--passes", type=int, default=1,
                    help="stand-in passes over the bucket paced over the modelled time (an "
                         "all-reduce: 2 = a ring's read + write traffic; the sharded plan's two "
                         "collectives get half each)")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--probe-steps", type=int, default=9)
    a = ap.parse_args()
    res = {}
    for tag, gbps in (("standin", a.gbps), ("nocomm", 0.0)):
        st = build(a, gbps, a.update if gbps > 0 else "allreduce")
        wall, host, tl = measure(st, a.steps, a.probe_steps)
        nb = len(st.buckets)
        seg = [(median([t["segments"][i][0] for t in tl]), median([t["segments"][i][1] for t in tl]))
               for i in range(nb)]
        com = [(median([t["comm"][j][1] for t in tl]), median([t["comm"][j][2] for t in tl]))
               for j in range(nb)]
        res[tag] = {"wall_ms": round(wall, 4), "host_ms": round(host, 4),
                    "segments_ms": [[round(x, 4), round(y, 4)] for x, y in seg],
                    "comm_ms": [[round(x, 4), round(y, 4)] for x, y in com],
                    "bucket_elems": [hi - lo for (_, (lo, hi)) in st.buckets],
                    "update": list(st.update)}
        del st
        import gc
        import torch
        gc.collect()
        torch.cuda.synchronize()
    s, n = res["standin"], res["nocomm"]
    seg_s = [y - x for x, y in s["segments_ms"]]
    seg_n = [y - x for x, y in n["segments_ms"]]
    # contention: slow-down of the segments that ran beside a collective (all but the first)
    extra = sum(seg_s[1:]) - sum(seg_n[1:])
    busy = sum(y - x for x, y in s["comm_ms"][:-1])
    contention = extra / busy if busy > 0 else 0.0
    # comm-stream time beyond the modelled collective time, per bucket
    model_us = []
    for j, ne in enumerate(s["bucket_elems"]):
        if s["update"][j] == "s16":
            model_us.append(0.5 * 4 * ne / (a.gbps * 1e3) + 0.5 * 2 * ne / (a.gbps * 1e3))
        else:
            model_us.append(4 * ne / (a.gbps * 1e3))
    comm_us = [(y - x) * 1e3 for x, y in s["comm_ms"]]
    print(f"VGG-11 b{a.batch}, cuts {a.cuts}, update {a.update}, stand-in {a.gbps} GB/s "
          f"(emulated world {a.world}, {a.passes} pass(es) over each bucket)\n")
    print("| run | wall ms/step | host enqueue ms/step |")
    print("|---|---|---|")
    for tag in ("standin", "nocomm"):
        print(f"| {tag} | {res[tag]['wall_ms']} | {res[tag]['host_ms']} |")
    print("\n| segment | no-comm us | with stand-in us | start .. end ms (stand-in run) |")
    print("|---|---|---|---|")
    for i, (x, y) in enumerate(s["segments_ms"]):
        print(f"| {i} | {seg_n[i] * 1e3:.1f} | {seg_s[i] * 1e3:.1f} | {x:.3f} .. {y:.3f} |")
    print("\n| bucket | plan | elements | comm-stream us | modelled collective us | start .. end ms |")
    print("|---|---|---|---|---|---|")
    for j, (x, y) in enumerate(s["comm_ms"]):
        print(f"| {j} | {s['update'][j]} | {s['bucket_elems'][j]} | {comm_us[j]:.1f} | "
              f"{model_us[j]:.1f} | {x:.3f} .. {y:.3f} |")
    over = [c - m for c, m in zip(comm_us, model_us)]
    print(f"\ncontention (backward slow-down per us of concurrent collective): {contention:.3f}; "
          f"comm-stream overhead beyond the modelled collective per bucket: "
          f"{', '.join(f'{v:.1f}' for v in over)} us")
    res.update(contention=round(contention, 4), comm_overhead_us=[round(v, 1) for v in over],
               batch=a.batch, cuts=a.cuts, update=a.update, gbps=a.gbps, world=a.world,
               passes=a.passes)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
