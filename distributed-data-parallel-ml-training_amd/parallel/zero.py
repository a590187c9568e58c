"""ZeRO-1-style sharded optimizer update for the bucketed DDP step (opt-in).

The reference replicates the optimizer on every rank (/root/reference/part3/main.py:176:
``optim.SGD(ddp_model.parameters(), ...)`` after an all-reduce of every gradient). Here, per
gradient bucket (a contiguous slice [lo, hi) of the flat arenas, n = hi - lo elements):

    reduce-scatter(avg) of grad[lo:hi]   -> this rank's shard s_r = [lo + r n/w, lo + (r+1) n/w)
    SGD on the shard only                 (fp32 master + momentum of 1/w of the parameters)
    all-gather of param[lo:hi]            -> every rank holds the updated fp32 master weights
    bf16 re-pack of the bucket's conv weights, grad[lo:hi] = 0

The wire bytes equal the all-reduce's (a ring all-reduce IS reduce-scatter + all-gather), the
SGD work per rank drops w-fold, and the replicas stay bit-identical (the gathered values are the
owners' results). On two ranks the reduced gradient is bit-identical to the all-reduce's (a + b
either way), so parameters match the replicated path exactly; beyond that the reduction order of
a standalone reduce-scatter may differ from the all-reduce's in the last bit.

GPU: the pipelined step (engine/step.py SegmentedDDPStep(zero=True), ``bench.py --zero``) runs
it per bucket on the comm stream. CPU (Gloo): the same sequence with torch.distributed
(tests/test_zero_cpu.py).
"""
import torch


class ShardedUpdate:
    def __init__(self, arena, optimizer, comm, buckets):
        """``buckets``: list of ((i0, i1), (lo, hi)) — parameter and element ranges.

        A bucket whose element count does not divide by the world size (arena slices are only
        64-element aligned: worlds 3, 5, 6, 7) is sharded unevenly — ranks 0..e-1 own
        ceil(n/w) elements, the rest floor(n/w) — and its collectives run on a [w, ceil(n/w)]
        zero-padded staging image (two strided copies in, two out) so every rank's
        reduce-scatter / all-gather chunk has the same size."""
        self.arena, self.opt, self.comm = arena, optimizer, comm
        self.world, self.rank = comm.world, comm.rank
        self.buckets = [tuple(map(tuple, b)) for b in buckets]
        for (_, (lo, hi)) in self.buckets:
            if hi - lo < self.world:
                raise ValueError(f"bucket of {hi - lo} elements is smaller than the world size "
                                 f"{self.world}")
        per = max(-(-(hi - lo) // self.world) for (_, (lo, hi)) in self.buckets)
        self._stage = None
        if any((hi - lo) % self.world for (_, (lo, hi)) in self.buckets):
            self._stage = torch.zeros(2, self.world * per, dtype=arena.data.dtype,
                                      device=arena.data.device)

    def _split(self, j):
        (_, (lo, hi)) = self.buckets[j]
        n = hi - lo
        base, extra = divmod(n, self.world)
        return lo, n, base, extra

    def shard(self, j):
        lo, n, base, extra = self._split(j)
        r = self.rank
        s0 = lo + r * base + min(r, extra)
        return s0, s0 + base + (1 if r < extra else 0)

    def _image(self, buf, j):
        """[w, per] view of staging row ``buf`` for bucket j (per = ceil(n/w))."""
        lo, n, base, extra = self._split(j)
        per = base + (1 if extra else 0)
        return self._stage[buf, :self.world * per].view(self.world, per)

    def _pack(self, src, img, j):
        lo, n, base, extra = self._split(j)
        k = extra * (base + 1)
        if extra:
            img[:extra, :base + 1].copy_(src[:k].view(extra, base + 1))
            img[extra:, base:].zero_()
        img[extra:, :base].copy_(src[k:].view(self.world - extra, base))

    def _unpack(self, img, dst, j):
        lo, n, base, extra = self._split(j)
        k = extra * (base + 1)
        if extra:
            dst[:k].view(extra, base + 1).copy_(img[:extra, :base + 1])
        dst[k:].view(self.world - extra, base).copy_(img[extra:, :base])

    @torch.no_grad()
    def step(self, j, stream=None, counter=None, skip=None):
        from .comm import AVG
        (i0, i1), (lo, hi) = self.buckets[j]
        a = self.arena
        cuda = a.data.is_cuda
        ctx = torch.cuda.stream(stream) if (cuda and stream is not None) else _null()
        with ctx:
            g, p = a.grad[lo:hi], a.data[lo:hi]
            s0, s1 = self.shard(j)
            if (hi - lo) % self.world == 0:
                self.comm.reduce_scatter_inplace(g, AVG, stream=stream)
                self.opt.step_elements(s0, s1, stream=stream, counter=counter, skip=skip)
                self.comm.all_gather_inplace(p, stream=stream)
            else:  # uneven shards through the padded [w, per] staging image
                gi, pi = self._image(0, j), self._image(1, j)
                self._pack(g, gi, j)
                self.comm.reduce_scatter_inplace(gi.view(-1), AVG, stream=stream)
                a.grad[s0:s1].copy_(gi[self.rank, :s1 - s0])
                self.opt.step_elements(s0, s1, stream=stream, counter=counter, skip=skip)
                self._pack(p, pi, j)
                self.comm.all_gather_inplace(pi.view(-1), stream=stream)
                self._unpack(pi, p, j)
            self.opt.repack_params(i0, i1, stream=stream)
            g.zero_()


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def arena_buckets(arena, first_params):
    """((i0, i1), (lo, hi)) ranges, last layers first, for buckets starting at the given
    parameter indices (ascending): the DDP pipelined step's layout."""
    bounds = [len(arena.params)] + sorted(first_params)[::-1] + [0]
    out = []
    for j in range(len(bounds) - 1):
        i1, i0 = bounds[j], bounds[j + 1]
        if i0 == i1:
            continue
        lo = arena.offsets[i0]
        hi = arena.offsets[i1] if i1 < len(arena.params) else arena.total
        out.append(((i0, i1), (lo, hi)))
    return out


# ------------------------------------------------------------------------------------------------
# Sharded update with a bf16 OPERAND all-gather
# ------------------------------------------------------------------------------------------------

def operand_tensors(arena):
    """Per parameter: True when the forward reads it only through a bf16 operand copy with the
    fp32 master's own element order (conv weights stored [K][R][S][C] with C == Cr, 1x1 convs,
    GEMM-run Linear weights: ops/layers.py ConvBNActSpec.wc). Those travel as bf16 in the
    sharded update; every other tensor (biases, BatchNorm gamma/beta, the channel-padded input
    conv, the fp32 classifier of VGG) keeps an fp32 all-gather. CPU arenas (no operand copies):
    4-D weights whose input channels are a multiple of 8, the GPU rule for the same model."""
    out = []
    for i, p in enumerate(arena.params):
        pack = getattr(p, "_ddp_amd_pack", None)
        if arena.data.is_cuda:
            if pack is None:  # read in fp32 by its kernel (or no operand copy yet): fp32 wire
                out.append(False)
                continue
            pp, wc, wt, K, Cr, C, R, S, krsc = pack()
            out.append(bool(wc) and not wt and C == Cr and (bool(krsc) or R * S == 1)
                       and pp == arena.data.data_ptr() + 4 * arena.offsets[i])
        else:
            out.append(p.dim() == 4 and p.shape[1] % 8 == 0)
    return out


class ShardedBf16Update:
    """Reduce-scatter fp32 gradients -> SGD on this rank's shard -> all-gather of the bf16
    OPERAND bytes the forward actually reads (plus the small fp32 tensors), per gradient bucket.

    The replicated path (/root/reference/part3/main.py:174-177: all-reduce every gradient, SGD
    on every rank) moves 2 x (w-1)/w x 4 bytes per parameter per rank and runs the whole SGD on
    every rank. ShardedUpdate (above) halves the SGD but still moves the same bytes (its
    all-gather carries fp32 masters). Here the all-gather carries what the next forward reads:
    the conv weights' bf16 MFMA operand image (ops/layers.py ConvBNActSpec.wc, re-pointed into
    one bf16 "shadow" arena at the fp32 arena's element offsets, so a bucket's operand bytes are
    one contiguous slice), and the small tensors (biases, BatchNorm gamma/beta, the
    channel-padded input conv, VGG's fp32 classifier) as fp32 through a per-bucket send slot:

        reduce-scatter(avg) fp32 grad[lo:hi]            -> shard [s0, s1) of this rank
        one launch: SGD on master[s0:s1] (+ momentum), shadow[s0:s1] = bf16(new), small
                    tensors' new values -> send slot, grad[lo:hi] = 0
        ONE RCCL group: all-gather bf16 shadow[lo:hi] + all-gather fp32 slots [w][M]
    and once per step, after the last bucket (``tail``): one launch copies every bucket's
    gathered slots into the fp32 masters of the small tensors, re-packs the operand of the
    channel-padded input conv (its master is complete only then) and signals the step's
    "every parameter updated" flag (only the next forward reads any of it).

    Wire bytes per rank: (w-1)/w x (4 + 2) per operand parameter instead of (w-1)/w x 8: 25 %
    fewer; SGD per rank: 1/w of the parameters. Gradients are reduced in fp32 (the reference's
    precision) and every rank computes with bf16(master) exactly as the replicated path does,
    so the two paths agree to the reduction order of the fp32 sums.

    Masters: a rank's fp32 master of an operand tensor is authoritative only on its own shard
    (the forward never reads the master). ``gather_masters()`` all-gathers them (fp32) for
    check_replicas / state_dict. Bucket sizes must divide by w into multiples of 4 elements
    (64-aligned buckets at w in {1, 2, 4, 8}); other worlds use ShardedUpdate / all-reduce.

    ``emulate_world`` (one-GPU studies, comm.world == 1): shard as rank 0 of that many ranks and
    stand in for the collectives with timed passes (engine/step.py SegmentedDDPStep). The other
    ranks' shards are then simply not updated (timing only).

    CPU (Gloo) twin: the arena on the CPU is the FORWARD operand (the model's conv weights hold
    bf16-rounded values, as the GPU forward reads them), and the fp32 masters live in
    ``self.master`` (tests/test_zero_cpu.py compares it with a replicated twin)."""

    def __init__(self, arena, optimizer, comm, buckets, which=None, emulate_world=None):
        self.arena, self.opt, self.comm = arena, optimizer, comm
        self.cuda = arena.data.is_cuda
        self.rank = comm.rank
        self.world = int(emulate_world or comm.world)
        self.emulated = self.world != comm.world
        if self.emulated and comm.world != 1:
            raise ValueError("emulate_world needs a single-rank communicator")
        self.buckets = [tuple(map(tuple, b)) for b in buckets]
        self.which = set(range(len(self.buckets)) if which is None else which)
        for j in self.which:
            (_, (lo, hi)) = self.buckets[j]
            n = hi - lo
            if n % self.world or (n // self.world) % 4:
                raise ValueError(f"bucket {j} ({n} elements) does not shard evenly over "
                                 f"{self.world} ranks")
        self.op = operand_tensors(arena)
        dev = arena.data.device
        # tensor ranges [offset_i, offset_{i+1}) incl. padding (padding stays 0 under SGD)
        ends = list(arena.offsets[1:]) + [arena.total]
        self._tensors = list(zip(arena.offsets, ends, self.op))
        self.data16 = torch.zeros(arena.total, dtype=torch.bfloat16, device=dev)
        self._plan = {}
        slot_total = 0
        for j in sorted(self.which):
            plan = self._plan_bucket(j, slot_total)
            slot_total += self.world * plan["M"]
            self._plan[j] = plan
        self.slots = torch.zeros(max(slot_total, 4), dtype=torch.float32, device=dev)
        if self.cuda:
            self._bind_operands()
            self._tables = {j: self._device_tables(j) for j in self.which}
            self._tail_table()
        else:
            self.master = arena.data.detach().clone()
            self.momentum = torch.zeros_like(self.master)
            self._mom_init = False
            with torch.no_grad():
                self.data16.copy_(self.master.to(torch.bfloat16))
                self._materialize([(0, arena.total)])

    # -------------------------------------------------------------- geometry
    def shard(self, j, rank=None):
        (_, (lo, hi)) = self.buckets[j]
        per = (hi - lo) // self.world
        r = self.rank if rank is None else rank
        return lo + r * per, lo + (r + 1) * per

    def _pieces(self, a, b):
        """[a, b) split at tensor boundaries: (start, end, is_operand) runs."""
        out = []
        for t0, t1, op in self._tensors:
            s, e = max(a, t0), min(b, t1)
            if s < e:
                out.append((s, e, op))
        return out

    def _plan_bucket(self, j, slot_base):
        (_, (lo, hi)) = self.buckets[j]
        small = []  # per rank: list of (arena start, count, slot offset within the rank's row)
        for r in range(self.world):
            s0, s1 = self.shard(j, r)
            k, lst = 0, []
            for s, e, op in self._pieces(s0, s1):
                if not op:
                    lst.append((s, e - s, k))
                    k += e - s
            small.append(lst)
        M = max(sum(c for _, c, _ in lst) for lst in small)
        M = (M + 3) // 4 * 4
        repack = [i for i, p in enumerate(self.arena.params)
                  if lo <= self.arena.offsets[i] < hi and not self.op[i]
                  and hasattr(p, "_ddp_amd_pack")]
        return {"M": M, "slot_base": slot_base, "small": small, "repack": repack}

    def wire_bytes(self, j):
        """(reduce-scatter bytes, all-gather bytes) of bucket j per rank's input buffer."""
        (_, (lo, hi)) = self.buckets[j]
        return 4 * (hi - lo), 2 * (hi - lo) + 4 * self.world * self._plan[j]["M"]

    # -------------------------------------------------------------- GPU
    def _bind_operands(self):
        """Re-point every operand tensor's bf16 copy into the shadow arena (same offsets), then
        rebuild all operand copies from the (still replicated) fp32 masters."""
        a = self.arena
        for i, p in enumerate(a.params):
            if self.op[i]:
                spec = p._ddp_amd_pack.__self__
                spec.rebind_wc(self.data16[a.offsets[i]:a.offsets[i] + a.numels[i]])
        self.opt.repack()

    def _device_tables(self, j):
        items = self.shard_items(j, self.rank)
        dev = self.arena.data.device
        return torch.tensor(items, dtype=torch.int32, device=dev), len(items)

    def shard_items(self, j, rank):
        """Work items of ``rank``'s update launch for bucket j (optim.hip sgd_pack_kernel):
        {3, offset, count, slot offset | -1} over its shard (SGD + bf16 operand + small-tensor
        send slot), {4, offset, count, -} clearing the rest of the bucket's gradients."""
        (_, (lo, hi)) = self.buckets[j]
        plan = self._plan[j]
        s0, s1 = self.shard(j, rank)
        items = []
        mine = {s: k for s, _, k in plan["small"][rank]}
        for s, e, op in self._pieces(s0, s1):
            for c0 in range(s, e, 8192):
                c1 = min(e, c0 + 8192)
                items.append([3, c0, c1 - c0, -1 if op else mine[s] + (c0 - s)])
        for a0, a1 in ((lo, s0), (s1, hi)):
            for c0 in range(a0, a1, 65536):
                items.append([4, c0, min(a1, c0 + 65536) - c0, 0])
        return items

    def tail_segments(self):
        """Copy segments of the step tail (optim.hip shard_tail_kernel): {slot index, arena
        index, count, -} for every sharded bucket's gathered small-tensor values (emulated: this
        rank's own only — the other ranks' slots hold nothing)."""
        segs = []
        ranks = [self.rank] if self.emulated else range(self.world)
        for j in sorted(self.which):
            plan = self._plan[j]
            for r in ranks:
                row = plan["slot_base"] + r * plan["M"]
                for s, c, k in plan["small"][r]:
                    for c0 in range(0, c, 4096):
                        segs.append([row + k + c0, s + c0, min(4096, c - c0), 0])
        return segs

    def _tail_table(self):
        """Tail copy segments (device table) and the operands to re-pack."""
        segs, descs = self.tail_segments(), []
        for j in sorted(self.which):
            descs += [self.arena.params[i]._ddp_amd_pack() for i in self._plan[j]["repack"]]
        if len(descs) > 4:
            raise ValueError("more than 4 channel-padded operands to re-pack in the step tail")
        dev = self.arena.data.device
        self._tail = (torch.tensor(segs if segs else [[0, 0, 0, 0]], dtype=torch.int32,
                                   device=dev), len(segs), descs)

    def step(self, j, stream=None, counter=None, skip=None, standin=None):
        """Bucket j's reduce-scatter, shard SGD, grouped all-gather and unpack (on ``stream``).
        ``standin(kind, nbytes, ptr, n)``: replaces the collectives (emulated world)."""
        if not self.cuda:
            return self._step_cpu(j)
        from ..ops.common import native, stream_handle
        from .comm import AVG
        nat = native()
        (_, (lo, hi)) = self.buckets[j]
        plan = self._plan[j]
        s0, s1 = self.shard(j)
        per = s1 - s0
        a, opt = self.arena, self.opt
        g = opt.param_groups[0]
        cs = stream.cuda_stream if stream is not None else stream_handle()
        items, n_items = self._tables[j]
        gp, dp, sp = a.grad.data_ptr(), a.data.data_ptr(), self.data16.data_ptr()
        slot_row = self.slots.data_ptr() + 4 * (plan["slot_base"] + self.rank * plan["M"])
        slot_all = self.slots.data_ptr() + 4 * plan["slot_base"]
        if standin is not None:
            standin("reduce_scatter", 4 * (hi - lo), gp + 4 * lo, hi - lo)
        else:
            self.comm.comm.reduce_scatter(gp + 4 * lo, gp + 4 * s0, per, 0, AVG, cs)
        nat.sgd_pack(items.data_ptr(), n_items, opt._descs_ptr(), dp, gp,
                     opt.momentum_buffer.data_ptr(), float(g["lr"]), float(g["momentum"]),
                     float(g["weight_decay"]), float(opt._grad_scale_factor),
                     int(bool(g["nesterov"])), cs, zero_grad=1,
                     counter=int(counter[0]) if counter else 0,
                     delta=int(counter[1]) if counter else 0, skip=int(skip) if skip else 0,
                     shadow=sp, slot=slot_row)
        if standin is not None:
            standin("all_gather", 2 * (hi - lo) + 4 * self.world * plan["M"], slot_all, 0)
        else:
            self.comm.comm.all_gather2(sp + 2 * s0, sp + 2 * lo, per, 1, slot_row, slot_all,
                                       plan["M"], 0, cs)

    def tail(self, stream=None, done=0, signal=0, skip=None):
        """After the step's last bucket (any plan), on the same stream: every sharded bucket's
        gathered small tensors -> fp32 masters, operand re-packs, then (``signal``: device
        pointer) release-increment the step's flag; ``done``: a zeroed uint32 ticket."""
        if not self.cuda:
            return
        from ..ops.common import native, stream_handle
        cs = stream.cuda_stream if stream is not None else stream_handle()
        segs, n_segs, descs = self._tail
        native().shard_tail(segs.data_ptr(), n_segs, self.slots.data_ptr(),
                            self.arena.data.data_ptr(), descs, int(done), int(signal),
                            int(skip) if skip else 0, cs)

    @torch.no_grad()
    def gather_masters(self, stream=None):
        """All-gather the fp32 masters AND the momentum buffers of every sharded bucket
        (check_replicas, optimizer / checkpoint state_dict, an eager step after the replays):
        a rank updates both only on its own shard, so afterwards every rank holds the owners'
        values everywhere. On the CPU the model's parameters then hold the fp32 masters too
        (until the next step re-materialises the operands)."""
        if self.emulated:
            return
        for j in sorted(self.which):
            (_, (lo, hi)) = self.buckets[j]
            buf = self.arena.data if self.cuda else self.master
            mom = self.opt.momentum_buffer if self.cuda else self.momentum
            self.comm.all_gather_inplace(buf[lo:hi], stream=stream)
            self.comm.all_gather_inplace(mom[lo:hi], stream=stream)
        if not self.cuda:
            self.arena.data.copy_(self.master)

    # -------------------------------------------------------------- CPU twin
    def _materialize(self, ranges):
        """CPU: the model's parameters = what the GPU forward reads (bf16 operands widened,
        fp32 small tensors)."""
        for a0, a1 in ranges:
            for s, e, op in self._pieces(a0, a1):
                self.arena.data[s:e] = (self.data16[s:e].float() if op else self.master[s:e])

    @torch.no_grad()
    def _step_cpu(self, j):
        from .comm import AVG
        (_, (lo, hi)) = self.buckets[j]
        plan = self._plan[j]
        s0, s1 = self.shard(j)
        a, g = self.arena, self.opt.param_groups[0]
        lr, m, wd = float(g["lr"]), float(g["momentum"]), float(g["weight_decay"])
        nesterov, gs = bool(g["nesterov"]), float(self.opt._grad_scale_factor)
        self.comm.reduce_scatter_inplace(a.grad[lo:hi], AVG)
        # the GPU launch's per-element math (common.h sgd_update1 = torch.optim.SGD's, momentum
        # buffer = d on the first step == m*0 + d): d = g*scale + wd*p; b = m*b + d;
        # d = nesterov ? d + m*b : b; p -= lr*d
        p, gr, buf = self.master[s0:s1], a.grad[s0:s1], self.momentum[s0:s1]
        d = gr * gs if gs != 1.0 else gr.clone()
        if wd != 0:
            d.add_(p, alpha=wd)
        if m != 0:
            buf.mul_(m).add_(d)
            d = d.add(buf, alpha=m) if nesterov else buf
        p.add_(d, alpha=-lr)
        self.data16[s0:s1] = p.to(torch.bfloat16)
        row = self.slots[plan["slot_base"] + self.rank * plan["M"]:
                         plan["slot_base"] + (self.rank + 1) * plan["M"]]
        for s, c, k in plan["small"][self.rank]:
            row[k:k + c] = self.master[s:s + c]
        a.grad[lo:hi].zero_()
        # bf16 all-gather through an int32 view (two bf16 per word; shards are multiples of 4)
        self.comm.all_gather_inplace(self.data16[lo:hi].view(torch.int32))
        allrows = self.slots[plan["slot_base"]:plan["slot_base"] + self.world * plan["M"]]
        self.comm.all_gather_inplace(allrows)
        for r in range(self.world):
            base = r * plan["M"]
            for s, c, k in plan["small"][r]:
                self.master[s:s + c] = allrows[base + k:base + k + c]
        self._materialize([(lo, hi)])
