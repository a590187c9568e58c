"""VGG family (VGG-11/13/16/19) for 3x32x32 inputs and 10 classes.

Reference parity: part1/model.py:3-50 (identical copies in part2/part2a, part2/part2b, part3).
The module tree — ``layers`` (nn.Sequential of Conv2d(3x3,s1,p1,bias) / BatchNorm2d(
track_running_stats=False) / ReLU(inplace) / MaxPool2d(2,2)) and ``fc1`` (Linear(512, 10)) —
is kept exactly so that ``state_dict`` keys and shapes match the reference checkpoint layout
(``layers.{0,4,8,...}.{weight,bias}``, BN without running buffers, ``fc1.{weight,bias}``).

Execution:
* CPU tensors run the ATen modules unchanged (the numerical oracle, and the part1 CPU path).
* GPU tensors run the fused gfx950 path: each Conv->BN->ReLU(->MaxPool) group becomes one
  ``ConvBNAct`` autograd Function (ops/layers.py), activations stay NHWC bf16, the head is a
  fused small-Linear kernel. Inputs may be NCHW fp32 (converted on device) or the NHWC bf16
  batches produced by the on-device data pipeline (data/loader.py).
"""
import torch
import torch.nn as nn

_cfg = {
    'VGG11': [64, 'M', 128, 'M', 256, 256, 'M', 512, 512, 'M', 512, 512, 'M'],
    'VGG13': [64, 64, 'M', 128, 128, 'M', 256, 256, 'M', 512, 512, 'M', 512, 512, 'M'],
    'VGG16': [64, 64, 'M', 128, 128, 'M', 256, 256, 256, 'M', 512, 512, 512, 'M', 512, 512, 512, 'M'],
    'VGG19': [64, 64, 'M', 128, 128, 'M', 256, 256, 256, 256, 'M', 512, 512, 512, 512, 'M',
              512, 512, 512, 512, 'M'],
}

IN_CHANNELS_PADDED = 8  # first conv consumes 3 real + 5 zero channels on the MFMA path


def _make_layers(cfg):
    """Same module sequence (and therefore the same Sequential indices) as part1/model.py:11-27."""
    mods = []
    cin = 3
    for v in cfg:
        if v == 'M':
            mods.append(nn.MaxPool2d(kernel_size=2, stride=2))
            continue
        mods += [nn.Conv2d(cin, v, kernel_size=3, stride=1, padding=1, bias=True),
                 nn.BatchNorm2d(v, track_running_stats=False),
                 nn.ReLU(inplace=True)]
        cin = v
    return nn.Sequential(*mods)


class _VGG(nn.Module):
    """VGG module for 3x32x32 input, 10 classes."""

    def __init__(self, name, num_classes=10):
        super().__init__()
        self.name = name
        self.layers = _make_layers(_cfg[name])
        self.fc1 = nn.Linear(512, num_classes)
        self._plan = None

    # ------------------------------------------------------------ fused GPU plan
    def fused_plan(self):
        """Group the Sequential into ConvBNAct stages (built once per device)."""
        from ..ops.layers import ConvBNActSpec
        dev = self.fc1.weight.device
        if self._plan is not None and self._plan[0] == dev:
            return self._plan[1]
        mods = list(self.layers)
        stages, i, first = [], 0, True
        while i < len(mods):
            conv = mods[i]
            if not isinstance(conv, nn.Conv2d):
                raise RuntimeError(f"unexpected module {conv} at layers.{i}")
            bn, relu = mods[i + 1], mods[i + 2]
            assert isinstance(bn, nn.BatchNorm2d) and isinstance(relu, nn.ReLU)
            pool = i + 3 < len(mods) and isinstance(mods[i + 3], nn.MaxPool2d)
            spec = ConvBNActSpec(conv, bn, relu=True, pool=pool,
                                 cin_pad=IN_CHANNELS_PADDED if first else None)
            # this block's dgrad produces the gradient at the previous block's output: it
            # accumulates that block's BatchNorm-backward sums (ops.layers, BnBwdFuse)
            spec.prev = stages[-1] if stages else None
            if stages:
                stages[-1].next = spec
            stages.append(spec)
            first = False
            i += 4 if pool else 3
        self._plan = (dev, stages)
        return stages

    def packed_specs(self):
        return self.fused_plan() if self.fc1.weight.is_cuda else []

    def _features_fused(self, x):
        from ..ops.layers import conv_bn_act, to_nhwc_input
        from ..ops.common import step_scratch
        plan = self.fused_plan()
        step_scratch(x.device).zero()  # BN statistics / backward sums of every layer: one fill
        h = to_nhwc_input(x, IN_CHANNELS_PADDED)
        for spec in plan:
            h = conv_bn_act(h, spec)
        if h.shape[1] != 1 or h.shape[2] != 1:
            raise RuntimeError("VGG head expects 1x1 spatial features (32x32 input)")
        return h.view(h.shape[0], -1)  # NHWC with H=W=1: identical to the NCHW flatten

    def forward(self, x):
        if not x.is_cuda:
            y = self.layers(x)
            y = y.view(y.size(0), -1)
            return self.fc1(y)
        from ..ops.layers import linear_small
        return linear_small(self._features_fused(x), self.fc1)

    @torch.no_grad()
    def forward_metrics(self, x, labels, loss_acc, correct_acc):
        """Evaluation in one classifier kernel (GPU): loss_acc (fp32 scalar) += mean CE of the
        batch, correct_acc (int32 scalar) += number of argmax hits (reference test_model,
        part1/main.py:96-111). No logits tensor, no host sync per batch."""
        from ..ops.common import native, ptr, stream_handle
        h = self._features_fused(x)
        B, F = h.shape
        labels = labels.to(torch.int64).contiguous()
        native().linear_ce_fwd(ptr(h), ptr(self.fc1.weight), ptr(self.fc1.bias), ptr(labels), B, F,
                               self.fc1.weight.shape[0], 0, 0, ptr(loss_acc), ptr(correct_acc),
                               stream_handle())

    def forward_loss_split(self, x, labels, split, acc=None, transient=False):
        """``forward_loss`` cut after fused stage(s) ``split`` (GPU; an int or ascending list of
        stage indices): returns (loss, cuts) with cuts[k] = (h_k, leaf_k), h_k the output of the
        stages before split[k] and ``leaf_k = h_k.detach().requires_grad_()`` the input of the
        stages from split[k] on. ``loss.backward()`` produces the gradients of the stages from
        split[-1] (+ fc1) and ``h_k.backward(leaf_k.grad)`` for k = len-1 .. 0 those of each
        earlier segment — backward segments the DDP engine can put collectives between
        (engine/step.py SegmentedDDPStep)."""
        from ..ops.layers import conv_bn_act, to_nhwc_input, linear_cross_entropy
        from ..ops.common import step_scratch
        plan = self.fused_plan()
        splits = [split] if isinstance(split, int) else list(split)
        if not splits or splits != sorted(set(splits)) or not 0 < splits[0] or splits[-1] >= len(plan):
            raise ValueError(f"split stages must be ascending in 1..{len(plan) - 1}")
        step_scratch(x.device).zero()
        h = to_nhwc_input(x, IN_CHANNELS_PADDED)
        cuts, prev = [], 0
        for sp in splits + [len(plan)]:
            for spec in plan[prev:sp]:
                h = conv_bn_act(h, spec)
            if sp < len(plan):
                leaf = h.detach().requires_grad_(True)
                cuts.append((h, leaf))
                h = leaf
            prev = sp
        loss = linear_cross_entropy(h.view(h.shape[0], -1), self.fc1, labels, acc, transient,
                                    bn_prev=plan[-1])
        return loss, cuts

    def n_stages(self):
        """Number of fused Conv->BN->ReLU(->pool) stages (cut points for forward_loss_split)."""
        return sum(1 for v in _cfg[self.name] if v != 'M')

    def first_param_of_stage(self, i):
        """Parameter that starts fused stage ``i`` in ``parameters()`` order (its conv weight)."""
        return self.fused_plan()[i].conv.weight

    def forward_loss(self, x, labels, acc=None, transient=False):
        """``CrossEntropyLoss()(self(x), labels)`` with the classifier and the loss fused into one
        kernel on the GPU (engine/step.py uses it for the captured training step). ``acc`` (fp32
        scalar) additionally accumulates the loss across calls. The returned loss tensor is only
        valid until the next forward when ``transient`` (it then lives in the per-forward
        scratch and costs no fill launch)."""
        if not x.is_cuda:
            loss = nn.functional.cross_entropy(self.forward(x), labels)
            if acc is not None:
                acc.add_(loss.detach())
            return loss
        from ..ops.layers import linear_cross_entropy
        last = self.fused_plan()[-1]
        last.defer_to_head = True  # its BN + ReLU + pool may run inside the head's kernel
        try:
            h = self._features_fused(x)
        finally:
            last.defer_to_head = False
        return linear_cross_entropy(h, self.fc1, labels, acc, transient, bn_prev=last)


def VGG11():
    return _VGG('VGG11')


def VGG13():
    return _VGG('VGG13')


def VGG16():
    return _VGG('VGG16')


def VGG19():
    return _VGG('VGG19')
