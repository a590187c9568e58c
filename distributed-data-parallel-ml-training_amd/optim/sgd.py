"""Fused multi-tensor SGD.

Reference parity: ``optim.SGD(params, lr=0.1, momentum=0.9, weight_decay=1e-4)``
(part1/main.py:124-125, part3/main.py:176-177): no dampening, no nesterov, momentum buffer
initialised to the first gradient. On the GPU one launch of ``sgd_kernel`` (csrc/kernels/optim.hip)
updates the whole flat parameter arena, followed by one launch that re-packs every conv weight
into the bf16 MFMA operand layouts the next forward consumes. On the CPU it is exactly
``torch.optim.SGD`` (the oracle).
"""
import torch

from .arena import arena_for


class FusedSGD(torch.optim.SGD):
    def __init__(self, params, lr=0.1, momentum=0.0, dampening=0.0, weight_decay=0.0,
                 nesterov=False, grad_scale=1.0):
        params = list(params)
        super().__init__(params, lr=lr, momentum=momentum, dampening=dampening,
                         weight_decay=weight_decay, nesterov=nesterov)
        self._grad_scale_factor = grad_scale
        self._fused = bool(params) and params[0].is_cuda
        if self._fused:
            if dampening != 0.0:
                raise ValueError("fused SGD supports dampening=0 only")
            if len(self.param_groups) != 1:
                raise ValueError("fused SGD supports a single param group")
            self.arena = arena_for(params)
            self.momentum_buffer = torch.zeros_like(self.arena.data)
        else:
            # CPU: plain torch.optim.SGD; the flat arena (if the DDP wrapper built one) serves the
            # element-range update of the ZeRO-1 path (step_elements)
            self.arena = getattr(params[0], "_ddp_amd_arena", None) if params else None

    def _packs(self):
        return [p._ddp_amd_pack() for p in self.arena.params if hasattr(p, "_ddp_amd_pack")]

    def repack(self):
        """Rebuild every bf16 conv-weight copy from the fp32 master weights (after the master
        weights were written outside the optimizer, e.g. a state rollback or checkpoint load)."""
        descs = self._packs()
        if descs and self.arena.data.is_cuda:
            from ..ops.common import native, stream_handle
            native().pack_conv_weights(descs, stream_handle())

    def register_in_backward(self):
        """SGD in the backward (engine/step.py TrainStep, one GPU): hand every conv weight whose
        bf16 copy has the master's index order to the kernel library, which applies its update
        in the WGRAD split-K finish that completes its gradient (conv_igemm.hip SgdFuse). Active
        until unregister_in_backward(); ``step(fused_taken=True)`` then skips the tensors whose
        finish took it (native sgd_fuse_taken)."""
        from ..ops.common import native
        a, g = self.arena, self.param_groups[0]
        nat = native()
        nat.sgd_fuse_register(0, clear=1)
        self._bwd_index = {}
        base_g, base_p = a.grad.data_ptr(), a.data.data_ptr()
        base_b = self.momentum_buffer.data_ptr()
        for i, p in enumerate(a.params):
            if not hasattr(p, "_ddp_amd_pack"):
                continue
            pp, wc, wt, K, Cr, C, R, S, krsc = p._ddp_amd_pack()
            if wt or not wc or not (krsc or R * S == 1) or pp != base_p + 4 * a.offsets[i]:
                continue
            dw = base_g + 4 * a.offsets[i]
            nat.sgd_fuse_register(dw, pp, base_b + 4 * a.offsets[i], wc, float(g["lr"]),
                                  float(g["momentum"]), float(g["weight_decay"]),
                                  float(self._grad_scale_factor), int(bool(g["nesterov"])))
            self._bwd_index[dw] = i
        nat.sgd_fuse_begin()

    def unregister_in_backward(self):
        from ..ops.common import native
        native().sgd_fuse_register(0, clear=1)

    def _fused_in_backward(self):
        """Parameter indices whose update a WGRAD finish applied since register_in_backward."""
        from ..ops.common import native
        idx = getattr(self, "_bwd_index", {})
        return frozenset(idx[d] for d in native().sgd_fuse_taken() if d in idx)

    def _master_in_backward(self):
        """Parameter indices whose fp32 master (and momentum) a backward pair's unsplit WGRAD
        epilogue updated: the step's launch re-packs only their bf16 operand copy."""
        from ..ops.common import native
        idx = getattr(self, "_bwd_index", {})
        return frozenset(idx[d] for d in native().sgd_fuse_taken_master() if d in idx)

    def _work_table(self, prange=None, exclude=frozenset(), pack_only=frozenset()):
        """Device work-item table of the fused SGD + re-pack kernel (rebuilt when the set of
        packed conv weights changes, e.g. after the model's fused plan is first built).
        ``prange = (i0, i1)`` restricts it to parameters i0 <= i < i1 (one DDP bucket: the
        pipelined step updates each bucket as soon as its all-reduce is done); ``exclude`` =
        parameter indices updated elsewhere (SGD in the backward); ``pack_only`` (a subset of
        ``exclude``) = those whose bf16 operand copy is still to be re-packed here (item 5)."""
        from ..ops.common import native
        a = self.arena
        key = tuple(self._packs())
        if getattr(self, "_table_key", None) != key:
            self._tables = {}
            self._table_key = key
            descs, per_param = [], [[] for _ in a.params]
            for i, p in enumerate(a.params):
                if not hasattr(p, "_ddp_amd_pack"):
                    continue
                pp, wc, wt, K, Cr, C, R, S, krsc = p._ddp_amd_pack()
                if pp != a.data.data_ptr() + 4 * a.offsets[i] or (R * S > 1 and bool(krsc) != a.krsc[i]):
                    raise RuntimeError("packed conv weight is not a view into the parameter arena")
                d = len(descs)
                descs.append([a.offsets[i], K, Cr, C, R, S, wc, wt, int(krsc), 0, 0, 0])
                n = a.numels[i]
                if not wt and C == Cr and (krsc or R * S == 1) and n % 4 == 0:
                    # bf16 copy in the master's own index order: elementwise items
                    for s0 in range(0, n, 8192):
                        per_param[i].append([2, s0, min(8192, n - s0), d])
                    continue
                TK, TC = native().sgd_tile_dims(R * S)
                for k0 in range(0, K, TK):
                    for c0 in range(0, C, TC):
                        per_param[i].append([1, d, k0, c0])
            chunk = 8192
            for i in range(len(a.params)):
                if per_param[i]:
                    continue
                o, n = a.offsets[i], a.numels[i]
                for s in range(0, n, chunk):
                    per_param[i].append([0, o + s, min(chunk, n - s), 0])
            self._per_param = per_param
            dev = a.data.device
            self._descs = torch.tensor(descs if descs else [[0] * 12], dtype=torch.int64, device=dev)
        rng = tuple(prange) if prange is not None else (0, len(a.params))
        t = self._tables.get((rng, exclude, pack_only))
        if t is None:
            keep = [i for i in range(*rng) if i not in exclude]
            packs = [i for i in range(*rng) if i in pack_only]
            for i in packs:
                if not self._per_param[i] or any(it[0] != 2 for it in self._per_param[i]):
                    raise RuntimeError(f"parameter {i}: no elementwise re-pack layout")
            # conv re-pack items first (the heavier tiles start early), then elementwise items
            sel = [it for i in keep for it in self._per_param[i] if it[0] != 0] + \
                  [[5] + it[1:] for i in packs for it in self._per_param[i]] + \
                  [it for i in keep for it in self._per_param[i] if it[0] == 0]
            if not sel and not exclude:
                raise ValueError(f"no parameters in range {rng}")
            items = (torch.tensor(sel, dtype=torch.int32, device=a.data.device) if sel
                     else None)
            t = (items, len(sel))
            self._tables[(rng, exclude, pack_only)] = t
        return t[0], t[1], self._descs

    def _elem_table(self, lo, hi):
        """Plain fp32 SGD items over arena elements [lo, hi) (no bf16 re-pack): the ZeRO-1
        shard update (parallel/zero.py)."""
        key = ("elems", lo, hi)
        t = getattr(self, "_elem_tables", {}).get(key)
        if t is None:
            chunk = 8192
            items = [[0, s0, min(chunk, hi - s0), 0] for s0 in range(lo, hi, chunk)]
            if not items:
                raise ValueError("empty element range")
            t = (torch.tensor(items, dtype=torch.int32, device=self.arena.data.device), len(items))
            self._elem_tables = getattr(self, "_elem_tables", {})
            self._elem_tables[key] = t
        return t

    @torch.no_grad()
    def step_elements(self, lo, hi, stream=None, zero_grad=False, counter=None, skip=None):
        """SGD (fp32 master + momentum only) on arena elements [lo, hi): one launch on the GPU,
        torch.optim.SGD's exact per-element math on the flat slices on the CPU."""
        g = self.param_groups[0]
        lr, m, wd = float(g["lr"]), float(g["momentum"]), float(g["weight_decay"])
        a = self.arena
        if not self._fused:
            p, gr = a.data[lo:hi], a.grad[lo:hi]
            d = gr.add(p, alpha=wd) if wd != 0 else gr
            if m != 0:
                if not hasattr(self, "_flat_buf"):
                    self._flat_buf = torch.zeros_like(a.data)
                    self._flat_init = torch.zeros(a.total, dtype=torch.bool)
                buf = self._flat_buf[lo:hi]
                if bool(self._flat_init[lo:hi].all()):
                    buf.mul_(m).add_(d)
                else:
                    buf.copy_(d)
                    self._flat_init[lo:hi] = True
                d = buf
            p.add_(d, alpha=-lr)
            if zero_grad:
                gr.zero_()
            return
        from ..ops.common import native, stream_handle
        s = stream.cuda_stream if stream is not None else stream_handle()
        items, n_items = self._elem_table(lo, hi)
        native().sgd_pack(items.data_ptr(), n_items, self._descs_ptr(), a.data.data_ptr(),
                          a.grad.data_ptr(), self.momentum_buffer.data_ptr(), lr, m, wd,
                          float(self._grad_scale_factor), int(bool(g["nesterov"])), s,
                          zero_grad=int(bool(zero_grad)),
                          counter=int(counter[0]) if counter else 0,
                          delta=int(counter[1]) if counter else 0,
                          skip=int(skip) if skip else 0)

    def _descs_ptr(self):
        return self._work_table()[2].data_ptr()

    def repack_params(self, i0, i1, stream=None):
        """Rebuild the bf16 operand copies of the conv weights among parameters [i0, i1)."""
        descs = [p._ddp_amd_pack() for p in self.arena.params[i0:i1] if hasattr(p, "_ddp_amd_pack")]
        if descs and self.arena.data.is_cuda:
            from ..ops.common import native, stream_handle
            native().pack_conv_weights(descs, stream.cuda_stream if stream is not None
                                       else stream_handle())

    def zero_grad(self, set_to_none=False):
        if self._fused:
            self.arena.zero_grad()  # kernels accumulate into the arena: always zero, never None
        else:
            super().zero_grad(set_to_none=set_to_none)

    @torch.no_grad()
    def step(self, closure=None, zero_grad=False, counter=None, skip=None, params=None,
             stream=None, fused_taken=False, signal=None):
        """One fused launch. ``params = (i0, i1)``: only parameters i0 <= i < i1 (arena order);
        ``stream``: launch on this torch stream instead of the current one. ``zero_grad=True`` also clears every gradient after its use (the
        next step then needs no zero_grad fill); ``counter=(int32 device ptr, delta)`` is
        advanced by the same launch (the on-device data cursor of engine/step.py); ``skip`` =
        device pointer of a uint32 error word: the update is skipped when it is non-zero.
        ``fused_taken=True``: skip the parameters whose update the backward already applied
        (register_in_backward). ``signal = (ticket ptr, flag ptr)``: the launch's last block to
        finish release-increments the uint32 flag (zeroed uint32 ticket)."""
        if not self._fused:
            out = super().step(closure)
            if zero_grad:
                super().zero_grad(set_to_none=False)
            return out
        from ..ops.common import native, stream_handle
        g = self.param_groups[0]
        s = stream.cuda_stream if stream is not None else stream_handle()
        a = self.arena
        exclude = pack_only = frozenset()
        if fused_taken:
            pack_only = self._master_in_backward()
            exclude = self._fused_in_backward() | pack_only
        items, n_items, descs = self._work_table(params, exclude, pack_only)
        if n_items == 0:  # every tensor was updated in the backward: only the data cursor
            if counter:
                native().counter_add(int(counter[0]), int(counter[1]), s)
            if signal:
                native().flag_signal(int(signal[1]), s)
            return None
        # one launch: SGD over every tensor + bf16 re-pack of every conv weight
        native().sgd_pack(items.data_ptr(), n_items, descs.data_ptr(), a.data.data_ptr(),
                          a.grad.data_ptr(), self.momentum_buffer.data_ptr(), float(g["lr"]),
                          float(g["momentum"]), float(g["weight_decay"]),
                          float(self._grad_scale_factor), int(bool(g["nesterov"])), s,
                          zero_grad=int(bool(zero_grad)),
                          counter=int(counter[0]) if counter else 0,
                          delta=int(counter[1]) if counter else 0,
                          skip=int(skip) if skip else 0,
                          done=int(signal[0]) if signal else 0,
                          signal=int(signal[1]) if signal else 0)
        return None

    def state_dict(self):
        sd = super().state_dict()
        if self._fused:
            # expose the momentum buffers in torch.optim.SGD's per-parameter layout
            a = self.arena
            for i, p in enumerate(a.params):
                    sd["state"][i] = {"momentum_buffer": a.shaped(self.momentum_buffer, i).contiguous()}
        return sd

    def load_state_dict(self, sd):
        if not self._fused:
            return super().load_state_dict(sd)
        a = self.arena
        st = sd.get("state", {})
        for i, p in enumerate(a.params):
            buf = st.get(i, st.get(str(i), {})).get("momentum_buffer")
            if buf is not None:
                a.shaped(self.momentum_buffer, i).copy_(buf.reshape(p.shape))
        for k in ("lr", "momentum", "weight_decay", "nesterov"):
            if sd.get("param_groups"):
                self.param_groups[0][k] = sd["param_groups"][0].get(k, self.param_groups[0][k])
