"""ResNet-50 (torchvision-compatible module tree and state_dict keys) for the driver's
large-gradient config: synthetic ImageNet 3x224x224, 1000 classes, bucketed DDP on 8 MI355X
(BASELINE.json configs[4]; SURVEY.md §2.D "Extra ops for the driver's ResNet-50 config").

Not part of the CS744 reference itself. 53 convolutions (1x1 / 3x3 / 7x7, stride 1/2),
BatchNorm with running statistics (track_running_stats=True, eval uses them), bottleneck
residual adds, 3x3/s2 max-pool, global average pool, Linear 2048 -> 1000; 161 parameter
tensors, 25 557 032 parameters.

GPU execution: every conv+BN(+residual)+ReLU is one ConvBNAct Function (implicit-GEMM MFMA
conv with fused BN statistics + one streaming BN/add/ReLU pass), the classifier is the same
MFMA GEMM (1x1 conv), pooling uses the pool.hip kernels; CPU execution is plain ATen.
"""

import torch
import torch.nn as nn

# stem BatchNorm + ReLU + 3x3/s2 max-pool fused (no pre-pool activation in HBM); False: the
# separate bn_act + maxpool passes (test oracle)
STEM_POOL_FUSE = True


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride=stride, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, planes * self.expansion, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * self.expansion)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride
        self._specs = None

    def forward(self, x):  # CPU / ATen path
        identity = x
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        if self.downsample is not None:
            identity = self.downsample(x)
        return self.relu(out + identity)

    def specs(self):
        from ..ops.layers import ConvBNActSpec
        if self._specs is None:
            ds = None
            if self.downsample is not None:
                ds = ConvBNActSpec(self.downsample[0], self.downsample[1], relu=False)
            s1 = ConvBNActSpec(self.conv1, self.bn1, relu=True)
            s2 = ConvBNActSpec(self.conv2, self.bn2, relu=True)
            s3 = ConvBNActSpec(self.conv3, self.bn3, relu=True, residual=True)
            # conv2's / conv3's dgrad produce the gradient at bn1's / bn2's output: their
            # epilogues accumulate those BatchNorms' backward sums (ops/layers.py BnBwdFuse)
            s2.prev, s3.prev = s1, s2
            self._specs = (s1, s2, s3, ds)
        return self._specs

    def forward_fused(self, h):
        from ..ops.layers import conv_bn_act, conv_pre_bn, res_bn_fuse_ok, GradLink
        s1, s2, s3, sd = self.specs()
        # the block input feeds two branches; their gradients meet in a GradLink (the second
        # one accumulates from its dgrad epilogue) instead of an autograd add kernel
        link = GradLink() if (h.requires_grad and torch.is_grad_enabled()) else None
        out = conv_bn_act(h, s1, in_link=link)
        out = conv_bn_act(out, s2)
        if sd is not None:
            if res_bn_fuse_ok(s3):
                # the shortcut's BatchNorm runs inside bn3's passes (ops/layers.py RES_BN_FUSE)
                zd = conv_pre_bn(h, sd, in_link=link)
                return conv_bn_act(out, s3, residual=zd, res_bn=sd)
            identity = conv_bn_act(h, sd, in_link=link)
            return conv_bn_act(out, s3, residual=identity)
        return conv_bn_act(out, s3, residual=h, res_link=link)


class ResNet(nn.Module):
    def __init__(self, layers=(3, 4, 6, 3), num_classes=1000, zero_init_residual=False):
        super().__init__()
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(64, layers[0])
        self.layer2 = self._make_layer(128, layers[1], stride=2)
        self.layer3 = self._make_layer(256, layers[2], stride=2)
        self.layer4 = self._make_layer(512, layers[3], stride=2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512 * Bottleneck.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    nn.init.constant_(m.bn3.weight, 0)
        self._stem = None
        self._fc_spec = None

    def _make_layer(self, planes, blocks, stride=1):
        downsample = None
        if stride != 1 or self.inplanes != planes * Bottleneck.expansion:
            downsample = nn.Sequential(
                nn.Conv2d(self.inplanes, planes * Bottleneck.expansion, 1, stride=stride, bias=False),
                nn.BatchNorm2d(planes * Bottleneck.expansion))
        layers = [Bottleneck(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes * Bottleneck.expansion
        for _ in range(1, blocks):
            layers.append(Bottleneck(self.inplanes, planes))
        return nn.Sequential(*layers)

    def blocks(self):
        for layer in (self.layer1, self.layer2, self.layer3, self.layer4):
            yield from layer

    def _gpu_specs(self):
        from ..ops.layers import ConvBNActSpec, LinearGemmSpec
        if self._stem is None:
            self._stem = ConvBNActSpec(self.conv1, self.bn1, relu=True, cin_pad=8)
            # bn1 + relu + maxpool in one pass each way (bn_act.hip bn_pool3_*)
            self._stem.maxpool3 = STEM_POOL_FUSE
            self._fc_spec = LinearGemmSpec(self.fc)
            for b in self.blocks():
                b.specs()
        return self._stem, self._fc_spec

    def fused_plan(self):
        stem, fc = self._gpu_specs()
        out = [stem]
        for b in self.blocks():
            out += [s for s in b.specs() if s is not None]
        return out + [fc]

    def forward(self, x):
        if not x.is_cuda:
            x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
            x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
            return self.fc(torch.flatten(self.avgpool(x), 1))
        from ..ops.common import step_scratch
        from ..ops.layers import conv_bn_act, global_avg_pool, linear_gemm, to_nhwc_input
        stem, fc = self._gpu_specs()
        step_scratch(x.device).zero()
        if self.training:
            self._bump_batches_tracked()
        h = to_nhwc_input(x, 8)
        h = self._stem_forward(h, stem)
        for b in self.blocks():
            h = b.forward_fused(h)
        return linear_gemm(global_avg_pool(h), fc)

    @staticmethod
    def _stem_forward(h, stem):
        from ..ops.layers import conv_bn_act, max_pool
        if stem.maxpool3:
            return conv_bn_act(h, stem)
        return max_pool(conv_bn_act(h, stem), 3, 2, 1)

    # ------------------------------------------------------------ segmented backward (DDP)
    # Stages: 0 = stem (conv1 + bn1 + relu + maxpool), 1..16 = the bottleneck blocks in order.
    # A cut before stage s detaches the stage's input, so the backward runs in segments the
    # pipelined DDP step (engine/step.py SegmentedDDPStep) puts bucket all-reduces between.
    def n_stages(self):
        return 1 + len(list(self.blocks()))

    def first_param_of_stage(self, i):
        """Parameter that starts stage ``i`` in ``parameters()`` order (its first conv weight):
        a stage's parameters are contiguous in the flat arena."""
        if i == 0:
            return self.conv1.weight
        return list(self.blocks())[i - 1].conv1.weight

    def forward_loss_split(self, x, labels, split, acc=None, transient=False):
        """Mean CE loss of the fused GPU forward, cut before stage(s) ``split`` (int or
        ascending list in 1..n_stages-1): returns (loss, cuts), cuts[k] = (h_k, leaf_k) as in
        models/vgg.py ``forward_loss_split``. A cut block input that feeds both residual
        branches is a leaf: the two branch gradients meet in its ``.grad``."""
        from ..ops.common import step_scratch
        from ..ops.layers import cross_entropy, global_avg_pool, linear_gemm, to_nhwc_input
        stem, fc = self._gpu_specs()
        blocks = list(self.blocks())
        n = 1 + len(blocks)
        splits = [split] if isinstance(split, int) else list(split)
        if not splits or splits != sorted(set(splits)) or not 0 < splits[0] or splits[-1] >= n:
            raise ValueError(f"split stages must be ascending in 1..{n - 1}")
        step_scratch(x.device).zero()
        if self.training:
            self._bump_batches_tracked()
        h = to_nhwc_input(x, 8)
        cuts = []
        for st in range(n):
            if st in splits:
                leaf = h.detach().requires_grad_(True)
                cuts.append((h, leaf))
                h = leaf
            h = self._stem_forward(h, stem) if st == 0 else blocks[st - 1].forward_fused(h)
        loss = cross_entropy(linear_gemm(global_avg_pool(h), fc), labels)
        if acc is not None:
            acc.add_(loss.detach())
        return loss, cuts

    def _bump_batches_tracked(self):
        nbt = getattr(self, "_nbt", None)
        if nbt is None:
            nbt = [m.num_batches_tracked for m in self.modules()
                   if isinstance(m, nn.BatchNorm2d) and m.num_batches_tracked is not None]
            self._nbt = nbt
        if nbt:
            torch._foreach_add_(nbt, 1)


def resnet50(num_classes=1000):
    return ResNet((3, 4, 6, 3), num_classes)
