"""Multi-process (Gloo, CPU) workers for the distributed tests."""
import os
import socket
import sys

import torch
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run_workers(fn, world, *args, timeout=300):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=fn, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(world):
            r, payload = q.get(timeout=timeout)
            out[r] = {k: (torch.from_numpy(v) if hasattr(v, "dtype") and hasattr(v, "shape") else v)
                      for k, v in payload.items()}
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for p in procs:
        assert p.exitcode == 0, f"worker exit code {p.exitcode}"
    return out


def _init(rank, world, port):
    sys.path.insert(0, REPO)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)


def train_worker(rank, world, port, q, strategy, steps, per_rank_batch, bucket_mb):
    try:
        _init(rank, world, port)
        import torch.distributed as dist
        from ddp_amd.models import VGG11
        from ddp_amd.optim import FusedSGD
        from ddp_amd.parallel import (TorchCommunicator, DistributedDataParallel, STRATEGIES,
                                      check_replicas)
        from ddp_amd.engine import CrossEntropyLoss
        from ddp_amd.data import SyntheticCIFAR10, CPULoader
        torch.manual_seed(89395)
        model = VGG11()
        comm = TorchCommunicator()
        if strategy in ("ddp", "ddp_bf16"):
            model = DistributedDataParallel(model, comm, bucket_cap_mb=bucket_mb,
                                            first_bucket_cap_mb=min(bucket_mb, 1.0),
                                            grad_comm_dtype="bf16" if strategy == "ddp_bf16"
                                            else "fp32")
        opt = FusedSGD(model.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4)
        crit = CrossEntropyLoss()
        loader = CPULoader(SyntheticCIFAR10(True, n=per_rank_batch * world * steps),
                           per_rank_batch, num_replicas=world, rank=rank)
        first_grads = None
        for i, (x, y) in enumerate(loader):
            if i >= steps:
                break
            opt.zero_grad()
            loss = crit(model(x), y)
            loss.backward()
            if strategy in STRATEGIES:
                STRATEGIES[strategy](model, comm)
            if first_grads is None:
                first_grads = torch.cat([p.grad.reshape(-1).clone() for p in model.parameters()])
            opt.step()
        params = torch.cat([p.detach().reshape(-1).clone() for p in model.parameters()])
        consistent = None
        if strategy in ("ddp", "ddp_bf16"):
            consistent = check_replicas(model.arena, world)
            info = {"buckets": list(model.buckets)}
        else:
            info = {}
        dist.destroy_process_group()
        q.put((rank, {"params": params.numpy(), "grads0": first_grads.numpy(),
                      "consistent": consistent, **info}))
    except Exception as e:  # surface the error in the parent
        import traceback
        q.put((rank, {"error": traceback.format_exc()}))
        raise


def local_grad_worker(rank, world, port, q, per_rank_batch):
    """Gradients of each rank WITHOUT synchronisation (to build the expected average)."""
    _init(rank, world, port)
    import torch.distributed as dist
    from ddp_amd.models import VGG11
    from ddp_amd.engine import CrossEntropyLoss
    from ddp_amd.data import SyntheticCIFAR10, CPULoader
    torch.manual_seed(89395)
    model = VGG11()
    loader = CPULoader(SyntheticCIFAR10(True, n=per_rank_batch * world), per_rank_batch,
                       num_replicas=world, rank=rank)
    x, y = next(iter(loader))
    CrossEntropyLoss()(model(x), y).backward()
    g = torch.cat([p.grad.reshape(-1).clone() for p in model.parameters()])
    dist.destroy_process_group()
    q.put((rank, {"grads0": g.numpy()}))


def nosync_worker(rank, world, port, q, per_rank_batch):
    """DDP.no_sync gradient accumulation vs manual accumulate-then-average."""
    try:
        _init(rank, world, port)
        import torch.distributed as dist
        from ddp_amd.models import VGG11
        from ddp_amd.optim import FusedSGD
        from ddp_amd.parallel import TorchCommunicator, DistributedDataParallel
        from ddp_amd.engine import CrossEntropyLoss
        from ddp_amd.data import SyntheticCIFAR10, CPULoader
        torch.manual_seed(89395)
        plain = VGG11()
        torch.manual_seed(89395)
        ddp = DistributedDataParallel(VGG11(), TorchCommunicator(), bucket_cap_mb=4.0)
        opt_p = FusedSGD(plain.parameters(), lr=0.05)
        opt_d = FusedSGD(ddp.parameters(), lr=0.05)
        crit = CrossEntropyLoss()
        loader = CPULoader(SyntheticCIFAR10(True, n=per_rank_batch * world * 2), per_rank_batch,
                           num_replicas=world, rank=rank)
        batches = [b for _, b in zip(range(2), loader)]
        opt_p.zero_grad()
        opt_d.zero_grad()
        for x, y in batches:
            crit(plain(x), y).backward()
        with ddp.no_sync():
            crit(ddp(batches[0][0]), batches[0][1]).backward()
        local_after_nosync = torch.cat([p.grad.reshape(-1).clone() for p in ddp.parameters()])
        crit(ddp(batches[1][0]), batches[1][1]).backward()
        g_ddp = torch.cat([p.grad.reshape(-1).clone() for p in ddp.parameters()])
        g_man = torch.cat([p.grad.reshape(-1).clone() for p in plain.parameters()])
        dist.all_reduce(g_man)
        g_man /= world
        dist.destroy_process_group()
        q.put((rank, {"ddp": g_ddp.numpy(), "manual": g_man.numpy(),
                      "after_nosync": local_after_nosync.numpy()}))
    except Exception:
        import traceback
        q.put((rank, {"error": traceback.format_exc()}))
        raise


def buffers_worker(rank, world, port, q):
    """DDP broadcast_buffers with flattened buffers: after a forward every rank holds rank 0's
    running statistics, and the module's buffers are views into the flat per-dtype tensors."""
    try:
        _init(rank, world, port)
        import torch.nn as nn
        import torch.distributed as dist
        from ddp_amd.parallel import TorchCommunicator, DistributedDataParallel
        torch.manual_seed(0)
        m = nn.Sequential(nn.Conv2d(3, 8, 3, padding=1), nn.BatchNorm2d(8), nn.ReLU(),
                          nn.Conv2d(8, 8, 3, padding=1), nn.BatchNorm2d(8), nn.Flatten(),
                          nn.Linear(8 * 8 * 8, 4))
        ddp = DistributedDataParallel(m, TorchCommunicator())
        with torch.no_grad():  # diverge the replicas' running stats
            m[1].running_mean.fill_(float(rank + 1))
            m[4].running_var.fill_(float(10 * (rank + 1)))
        x = torch.randn(4, 3, 8, 8) + rank
        ddp(x).sum().backward()
        bufs = {n: b.clone() for n, b in m.named_buffers()}
        flat_views = all(b.untyped_storage().data_ptr() in
                         {f.untyped_storage().data_ptr() for f in ddp._flat_buffers}
                         for b in m.buffers())
        dist.destroy_process_group()
        q.put((rank, {"bufs": {k: v.numpy() for k, v in bufs.items()}, "flat": flat_views}))
    except Exception:
        import traceback
        q.put((rank, {"error": traceback.format_exc()}))
        raise


def commbench_worker(rank, world, port, q):
    try:
        _init(rank, world, port)
        from ddp_amd.parallel import TorchCommunicator
        from ddp_amd.parallel.commbench import allreduce_sweep
        rows = allreduce_sweep(TorchCommunicator(), [1 << 12, 1 << 16], iters=3, warmup=1)
        q.put((rank, {"rows": rows}))
    except Exception as e:  # pragma: no cover - surfaced by the parent
        import traceback
        q.put((rank, {"error": traceback.format_exc() + repr(e)}))


def probe_worker(rank, world, port, q):
    """bench.py's start-up probe (bucket_plan.probe_table) on Gloo, then DDP 'auto' bucket caps
    planned from that table (overlapped reducer)."""
    try:
        _init(rank, world, port)
        from ddp_amd.models import VGG11
        from ddp_amd.parallel import TorchCommunicator, DistributedDataParallel
        from ddp_amd.parallel import bucket_plan as bp
        comm = TorchCommunicator()
        t = bp.probe_table(comm, world, "fp32", device="cpu", sizes=[1 << 14, 1 << 16, 1 << 18],
                           iters=2, warmup=1)
        torch.manual_seed(0)
        m = DistributedDataParallel(VGG11(), comm, bucket_cap_mb="auto", first_bucket_cap_mb="auto",
                                    comm_table=t)
        rows, src = bp.rows_for(t, world)
        q.put((rank, {"table": t, "reason": m.bucket_plan_reason, "src": src,
                      "pred": bp.predict_us(rows, 1 << 16), "pred_mid": bp.predict_us(rows, 1 << 17),
                      "nb": len(m.buckets)}))
    except Exception as e:  # pragma: no cover - surfaced by the parent
        import traceback
        q.put((rank, {"error": traceback.format_exc() + repr(e)}))


class _Swapped(torch.nn.Module):
    """Parameters registered in the opposite order of their use: ``late`` is defined first but
    applied last, so its gradient is ready FIRST in backward while the reverse-parameter-order
    bucket plan puts it in the LAST bucket (what torch DDP's post-iteration-0 rebuild fixes)."""

    def __init__(self):
        super().__init__()
        self.late = torch.nn.Linear(32, 4)
        self.early = torch.nn.Linear(16, 32)

    def forward(self, x):
        return self.late(torch.relu(self.early(x)))


def overlap_worker(rank, world, port, q, model_name):
    """DDP on Gloo: per-iteration bucket launch logs (bucket, parameters marked at launch),
    launch order before/after the iteration-0 rebuild, final parameters and gradients."""
    try:
        _init(rank, world, port)
        import torch.distributed as dist
        from ddp_amd.parallel import TorchCommunicator, DistributedDataParallel, check_replicas
        from ddp_amd.optim import FusedSGD
        torch.manual_seed(7)
        if model_name == "swapped":
            model = _Swapped()
            cap, first = 0.0001, 0.0001  # one bucket per parameter tensor
            xs = [torch.randn(8, 16) + rank for _ in range(3)]
            ys = [torch.randint(0, 4, (8,)) for _ in range(3)]
        else:
            from ddp_amd.models import VGG11
            model = VGG11()
            cap, first = 4.0, 1.0
            xs = [torch.randn(4, 3, 32, 32) + rank for _ in range(2)]
            ys = [torch.randint(0, 10, (4,)) for _ in range(2)]
        ddp = DistributedDataParallel(model, TorchCommunicator(), bucket_cap_mb=cap,
                                      first_bucket_cap_mb=first)
        opt = FusedSGD(ddp.parameters(), lr=0.05, momentum=0.9)
        logs, orders = [], []
        for x, y in zip(xs, ys):
            opt.zero_grad()
            torch.nn.functional.cross_entropy(ddp(x), y).backward()
            orders.append(list(ddp.reducer.launch_order()))  # the order this backward used
            logs.append(list(ddp.reducer.launch_log()))
            opt.step()
        ok = check_replicas(ddp.arena, world)
        params = torch.cat([p.detach().reshape(-1).clone() for p in ddp.parameters()])
        nb = len(ddp.buckets)
        dist.destroy_process_group()
        q.put((rank, {"logs": logs, "orders": orders, "consistent": ok,
                      "params": params.numpy(), "n_buckets": nb,
                      "n_params": len(list(ddp.parameters()))}))
    except Exception:
        import traceback
        q.put((rank, {"error": traceback.format_exc()}))
        raise


def zero_worker(rank, world, port, q, steps):
    """Replicated DDP update (all-reduce + SGD on every parameter) vs the ZeRO-1 sharded update
    (reduce-scatter -> SGD on this rank's shard -> all-gather), same init and data."""
    try:
        _init(rank, world, port)
        import torch.distributed as dist
        from ddp_amd.models import VGG11
        from ddp_amd.optim import FusedSGD
        from ddp_amd.parallel import TorchCommunicator, DistributedDataParallel, check_replicas
        from ddp_amd.parallel.zero import ShardedUpdate, arena_buckets
        from ddp_amd.engine import CrossEntropyLoss
        from ddp_amd.data import SyntheticCIFAR10, CPULoader
        comm = TorchCommunicator()
        crit = CrossEntropyLoss()
        loader = CPULoader(SyntheticCIFAR10(True, n=4 * world * steps), 4, num_replicas=world,
                           rank=rank)
        batches = [b for _, b in zip(range(steps), loader)]
        out = {}
        for mode in ("replicated", "zero"):
            torch.manual_seed(89395)
            ddp = DistributedDataParallel(VGG11(), comm, bucket_cap_mb=4.0)
            opt = FusedSGD(ddp.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4)
            upd = None
            if mode == "zero":
                a = ddp.arena
                pidx = {id(p): i for i, p in enumerate(a.params)}
                firsts = [pidx[id(ddp.module.layers[i].weight)] for i in (11, 22)]  # stages 3, 6
                upd = ShardedUpdate(a, opt, comm, arena_buckets(a, firsts))
                assert len(upd.buckets) == 3
                shards = [upd.shard(j) for j in range(3)]
            for x, y in batches:
                opt.zero_grad()
                if upd is None:
                    crit(ddp(x), y).backward()
                    opt.step()
                else:
                    with ddp.no_sync():
                        crit(ddp(x), y).backward()
                    for j in range(len(upd.buckets)):
                        upd.step(j)
            out[mode] = torch.cat([p.detach().reshape(-1).clone() for p in ddp.parameters()])
            out[mode + "_consistent"] = check_replicas(ddp.arena, world)
            if upd is not None:
                out["grad_zero"] = bool((ddp.arena.grad == 0).all())
                out["shards"] = shards
                out["bucket_sizes"] = [hi - lo for (_, (lo, hi)) in upd.buckets]
        dist.destroy_process_group()
        q.put((rank, {"replicated": out["replicated"].numpy(), "zero": out["zero"].numpy(),
                      "rc": out["replicated_consistent"], "zc": out["zero_consistent"],
                      "grad_zero": out["grad_zero"], "shards": out["shards"],
                      "bucket_sizes": out["bucket_sizes"]}))
    except Exception:
        import traceback
        q.put((rank, {"error": traceback.format_exc()}))
        raise


def shard16_worker(rank, world, port, q, steps):
    """Replicated update with the GPU's operand semantics (fp32 all-reduce + SGD on the fp32
    master of every parameter; the forward reads bf16(master) of the conv weights) vs the
    sharded update with the bf16 operand all-gather (parallel/zero.py ShardedBf16Update): same
    init and data, cuts before stages 3 and 6 (three buckets)."""
    try:
        _init(rank, world, port)
        import torch.distributed as dist
        from ddp_amd.models import VGG11
        from ddp_amd.optim import FusedSGD
        from ddp_amd.parallel import TorchCommunicator, DistributedDataParallel, check_replicas
        from ddp_amd.parallel.comm import AVG
        from ddp_amd.parallel.zero import ShardedBf16Update, arena_buckets, operand_tensors
        from ddp_amd.engine import CrossEntropyLoss
        from ddp_amd.data import SyntheticCIFAR10, CPULoader
        comm = TorchCommunicator()
        crit = CrossEntropyLoss()
        loader = CPULoader(SyntheticCIFAR10(True, n=4 * world * steps), 4, num_replicas=world,
                           rank=rank)
        batches = [b for _, b in zip(range(steps), loader)]
        out = {}
        lr, m, wd = 0.05, 0.9, 1e-4
        for mode in ("replicated", "shard16"):
            torch.manual_seed(89395)
            ddp = DistributedDataParallel(VGG11(), comm, bucket_cap_mb=4.0)
            opt = FusedSGD(ddp.parameters(), lr=lr, momentum=m, weight_decay=wd)
            a = ddp.arena
            pidx = {id(p): i for i, p in enumerate(a.params)}
            firsts = [pidx[id(ddp.module.layers[i].weight)] for i in (11, 22)]  # stages 3, 6
            buckets = arena_buckets(a, firsts)
            op = operand_tensors(a)
            ends = list(a.offsets[1:]) + [a.total]
            upd = None
            if mode == "shard16":
                upd = ShardedBf16Update(a, opt, comm, buckets)
                out["shards"] = [upd.shard(j) for j in range(len(buckets))]
                out["n_operand"] = sum(op)
                out["wire"] = [upd.wire_bytes(j) for j in range(len(buckets))]
            else:
                master, mom = a.data.detach().clone(), torch.zeros_like(a.data)

                def materialize():
                    with torch.no_grad():
                        for (o, e), is_op in zip(zip(a.offsets, ends), op):
                            a.data[o:e] = (master[o:e].to(torch.bfloat16).float() if is_op
                                           else master[o:e])
                materialize()
            for x, y in batches:
                opt.zero_grad()
                with ddp.no_sync():
                    crit(ddp(x), y).backward()
                if upd is not None:
                    for j in range(len(buckets)):
                        upd.step(j)
                else:
                    with torch.no_grad():
                        comm.all_reduce(a.grad, AVG)
                        d = a.grad.add(master, alpha=wd)
                        mom.mul_(m).add_(d)
                        master.add_(mom, alpha=-lr)
                        a.grad.zero_()
                    materialize()
            out[mode + "_operand"] = a.data.detach().clone()
            if upd is not None:
                out["grad_zero"] = bool((a.grad == 0).all())
                out["operands_consistent"] = check_replicas(a, world)
                upd.gather_masters()
                out[mode] = upd.master.clone()
                out[mode + "_momentum"] = upd.momentum.clone()  # gathered from the owners
                out["data_is_master"] = bool(torch.equal(a.data, upd.master))
                out["masters_consistent"] = check_replicas(a, world)
            else:
                out[mode] = master.clone()
                out[mode + "_momentum"] = mom.clone()
        dist.destroy_process_group()
        q.put((rank, {"replicated": out["replicated"].numpy(), "shard16": out["shard16"].numpy(),
                      "replicated_operand": out["replicated_operand"].numpy(),
                      "shard16_operand": out["shard16_operand"].numpy(),
                      "replicated_momentum": out["replicated_momentum"].numpy(),
                      "shard16_momentum": out["shard16_momentum"].numpy(),
                      "grad_zero": out["grad_zero"], "shards": out["shards"],
                      "operands_consistent": out["operands_consistent"],
                      "masters_consistent": out["masters_consistent"],
                      "data_is_master": out["data_is_master"], "n_operand": out["n_operand"],
                      "wire": out["wire"]}))
    except Exception:
        import traceback
        q.put((rank, {"error": traceback.format_exc()}))
        raise


def uid_bootstrap_worker(rank, world, port, q):
    """RcclCommunicator's ncclUniqueId exchange over the c10d TCPStore with a stand-in native
    module (no GPU): rank 0 creates each uid, every rank constructs its communicator from it."""
    try:
        _init(rank, world, port)
        import os as _os
        import torch.distributed as dist
        from ddp_amd.ops import common
        from ddp_amd.parallel import comm as cm

        class FakeComm:
            def __init__(self, r, w, uid, dev):
                self.uid, self.live = bytes(uid), True

        class FakeNative:
            RcclComm = FakeComm

            @staticmethod
            def make_unique_id():
                return _os.urandom(128)

        common._NATIVE = FakeNative()
        a = cm.RcclCommunicator(rank, world, 0)
        b = cm.RcclCommunicator(rank, world, 0, key="ddp_amd/rccl_uid_overlap")
        c = cm.RcclCommunicator(rank, world, 0)
        out = {"uids": [x.comm.uid.hex() for x in (a, b, c)], "live": a.live and c.live}
        dist.barrier()  # rank 0 hosts the store: nobody leaves while a peer may still read it
        dist.destroy_process_group()
        q.put((rank, out))
    except Exception:
        import traceback
        q.put((rank, {"error": traceback.format_exc()}))
        raise
