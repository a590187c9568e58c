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
