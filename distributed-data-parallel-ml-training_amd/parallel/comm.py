"""Process-group bootstrap and communicators.

Reference parity:
* ``init_distributed_setup`` (part2/part2a/main.py:52-58): sets MASTER_ADDR/MASTER_PORT and
  calls ``init_process_group``; ``test_distributed_setup`` (part2/part2a/main.py:42-49) prints
  the four diagnostic lines; ``dist.destroy_process_group`` at the end (part3/main.py:186).
* The reference's data plane is Gloo over TCP.

MI355X design: one process per GPU. torch.distributed (Gloo, CPU) is the *control plane* —
rendezvous through the TCPStore at --master-ip:--master-port, barriers, timing reductions,
printing the setup. The *data plane* is our native RCCL communicator over xGMI
(csrc/runtime/comm.cpp): rank 0 creates the ncclUniqueId and publishes it through the same
TCPStore. On CPU-only runs (tests, part1 on CPU) a TorchCommunicator over Gloo implements the
same interface so every strategy can be exercised without GPUs.
"""
import datetime
import os

import torch
import torch.distributed as dist

# dtype / op codes shared with csrc/runtime/comm.cpp
_DT = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2, torch.int32: 3, torch.int64: 4,
       torch.uint8: 5}
SUM, PROD, MAX, MIN, AVG = 0, 1, 2, 3, 4
# set once a single-rank RCCL communicator exists (RcclCommunicator self_comm): graph captures
# then use the multi-GPU "thread_local" mode, exactly as on a node
SELF_COMM_ACTIVE = False
_TORCH_OP = {SUM: dist.ReduceOp.SUM, PROD: dist.ReduceOp.PRODUCT, MAX: dist.ReduceOp.MAX,
             MIN: dist.ReduceOp.MIN}


def init_distributed_setup(master_ip, master_port, rank, world_size, backend="gloo",
                           timeout_s=1800):
    """Reference-compatible bootstrap (part2/part2a/main.py:52-58).

    Under torchrun (TORCHELASTIC_USE_AGENT_STORE) the launcher's rendezvous store is the one the
    process group joins, so --master-ip/--master-port must not redirect it: a mismatch would
    make every rank wait for a store nobody hosts. The launcher's MASTER_ADDR/PORT win there."""
    if os.environ.get("TORCHELASTIC_USE_AGENT_STORE") == "True" and "MASTER_PORT" in os.environ:
        env = (os.environ.get("MASTER_ADDR"), os.environ["MASTER_PORT"])
        if (str(master_ip), str(master_port)) != env:
            print(f"[ddp_amd] launched by torchrun: using its rendezvous {env[0]}:{env[1]} "
                  f"instead of --master-ip/--master-port {master_ip}:{master_port}", flush=True)
        master_ip, master_port = env
    os.environ["MASTER_ADDR"] = str(master_ip)
    os.environ["MASTER_PORT"] = str(master_port)
    dist.init_process_group(backend, rank=rank, world_size=world_size,
                            timeout=datetime.timedelta(seconds=timeout_s))


def test_distributed_setup():
    """Reference-format diagnostics (part2/part2a/main.py:42-49)."""
    print(f'Is initialized: {dist.is_initialized()}')
    print(f'Backend: {dist.get_backend()}')
    print(f'World size: {dist.get_world_size()}')
    print(f'Rank: {dist.get_rank()}\n')


def destroy():
    if dist.is_initialized():
        dist.destroy_process_group()


def _store():
    # the default group's store is the TCPStore created by init_process_group (env://)
    return dist.distributed_c10d._get_default_store()


class TorchCommunicator:
    """torch.distributed (Gloo on CPU) implementation of the communicator interface."""

    kind = "torch"

    def __init__(self, group=None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.live = self.world > 1

    def all_reduce(self, t, op=SUM):
        if op == AVG:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
            t /= self.world
        else:
            dist.all_reduce(t, op=_TORCH_OP[op], group=self.group)

    def all_reduce_async(self, t):
        return dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group, async_op=True)

    def broadcast(self, t, src=0):
        dist.broadcast(t, src, group=self.group)

    def all_gather(self, t):
        out = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(out, t, group=self.group)
        return out

    def reduce_scatter_inplace(self, buf, op=AVG, stream=None):
        """Flat ``buf`` (numel divisible by world): this rank's shard
        ``buf[rank*n/w:(rank+1)*n/w]`` receives the reduction over ranks (ZeRO-1)."""
        n = buf.numel() // self.world
        out = torch.empty(n, dtype=buf.dtype)
        dist.reduce_scatter_tensor(out, buf.contiguous(), op=dist.ReduceOp.SUM, group=self.group)
        if op == AVG:
            out /= self.world
        buf[self.rank * n:(self.rank + 1) * n].copy_(out)

    def all_gather_inplace(self, buf, stream=None):
        """Flat ``buf``: every rank's shard is gathered into every rank's ``buf``."""
        n = buf.numel() // self.world
        mine = buf[self.rank * n:(self.rank + 1) * n].clone()
        dist.all_gather_into_tensor(buf, mine, group=self.group)

    def gather(self, t, dst=0):
        """Reference 2A gather (part2/part2a/main.py:104-107,114): returns the list on dst."""
        if self.rank == dst:
            lst = [torch.zeros_like(t) for _ in range(self.world)]
            dist.gather(t, lst, dst=dst, group=self.group)
            return lst
        dist.gather(t, dst=dst, group=self.group)
        return None

    def scatter_replicated(self, t, src=0):
        """Reference 2A scatter of [mean]*ws (part2/part2a/main.py:110,115)."""
        if self.rank == src:
            dist.scatter(t, [t] * self.world, src=src, group=self.group)
        else:
            dist.scatter(t, src=src, group=self.group)

    def barrier(self):
        dist.barrier(group=self.group)

    def synchronize(self):
        pass


_UID_SEQ = 0


class RcclCommunicator:
    """Native RCCL communicator (one GPU per process, collectives over xGMI)."""

    kind = "rccl"

    def __init__(self, rank=None, world=None, device=None, key="ddp_amd/rccl_uid", self_comm=None):
        """``self_comm`` (default: env ``DDP_AMD_RCCL_SELF=1``): at world size 1, create a real
        single-rank RCCL communicator instead of skipping every collective, so a one-GPU box runs
        the same RCCL calls (inside captured graphs, on a second communicator, ...) as a node."""
        from ..ops.common import native
        self.rank = dist.get_rank() if rank is None else rank
        self.world = dist.get_world_size() if world is None else world
        self.device = torch.cuda.current_device() if device is None else device
        if self_comm is None:
            self_comm = os.environ.get("DDP_AMD_RCCL_SELF", "0") == "1"
        n = native()
        uid = b""
        if self.world > 1:
            # every communicator gets its own store key (construction order is the same on every
            # rank), so a second communicator never reads a stale uid of an earlier one
            global _UID_SEQ
            _UID_SEQ += 1
            key = f"{key}/{_UID_SEQ}"
            store = _store()
            if self.rank == 0:
                uid = n.make_unique_id()
                store.set(key, uid)
            else:
                store.wait([key])
                uid = store.get(key)
        elif self_comm:
            global SELF_COMM_ACTIVE
            uid = n.make_unique_id()
            SELF_COMM_ACTIVE = True
        self.comm = n.RcclComm(self.rank, self.world, uid, self.device)
        self.live = bool(self.comm.live)  # collectives reach RCCL (world > 1 or self_comm)

    @staticmethod
    def _s():
        return torch.cuda.current_stream().cuda_stream

    def all_reduce(self, t, op=SUM):
        self.comm.all_reduce(t.data_ptr(), t.numel(), _DT[t.dtype], op, self._s())

    def broadcast(self, t, src=0):
        self.comm.broadcast(t.data_ptr(), t.numel(), _DT[t.dtype], src, self._s())

    def all_gather(self, t):
        out = torch.empty((self.world,) + tuple(t.shape), dtype=t.dtype, device=t.device)
        self.comm.all_gather(t.data_ptr(), out.data_ptr(), t.numel(), _DT[t.dtype], self._s())
        return list(out.unbind(0))

    def reduce_scatter_inplace(self, buf, op=AVG, stream=None):
        """In-place ncclReduceScatter of flat ``buf``: the shard at rank*n/w receives the result
        (NCCL's in-place convention recvbuff = sendbuff + rank * recvcount)."""
        n = buf.numel() // self.world
        es = buf.element_size()
        s = stream.cuda_stream if stream is not None else self._s()
        self.comm.reduce_scatter(buf.data_ptr(), buf.data_ptr() + self.rank * n * es, n,
                                 _DT[buf.dtype], op, s)

    def all_gather_inplace(self, buf, stream=None):
        """In-place ncclAllGather of flat ``buf`` (sendbuff = recvbuff + rank * sendcount)."""
        n = buf.numel() // self.world
        es = buf.element_size()
        s = stream.cuda_stream if stream is not None else self._s()
        self.comm.all_gather(buf.data_ptr() + self.rank * n * es, buf.data_ptr(), n,
                             _DT[buf.dtype], s)

    def gather_into(self, t, buf, dst=0):
        """Grouped send/recv gather of t into buf[world, numel] on dst."""
        self.comm.gather(t.data_ptr(), buf.data_ptr() if buf is not None else 0, t.numel(),
                         _DT[t.dtype], dst, self._s())

    def reserve_staging(self, nbytes):
        """Pre-size the single-rank scatter staging buffer (before any graph capture; during a
        capture this is a no-op and scatter_replicated refuses to grow the buffer)."""
        if torch.cuda.is_current_stream_capturing():
            return
        self.comm.reserve_stage(int(nbytes))

    def scatter_replicated(self, t, src=0):
        self.comm.scatter_replicated(t.data_ptr(), t.numel(), _DT[t.dtype], src, self._s())

    def barrier(self):
        if dist.is_initialized():
            dist.barrier()

    def synchronize(self):
        torch.cuda.synchronize()

    def check_health(self):
        err = self.comm.async_error()
        if err != 0:
            raise RuntimeError(f"RCCL async error {err}")

    def abort(self):
        self.comm.abort()


def is_live(comm):
    """True when ``comm``'s collectives actually run (world > 1, or a single-rank RCCL
    communicator created with ``self_comm``)."""
    return bool(getattr(comm, "live", comm.world > 1))


def make_communicator(device):
    """RCCL on GPU, torch.distributed (Gloo) on CPU."""
    if torch.device(device).type == "cuda":
        return RcclCommunicator()
    return TorchCommunicator()
