"""Bucket planning (DDP part 3): Python twin vs the native C++ planner, reference sizes."""
import pytest

from ddp_amd.models import VGG11
from ddp_amd.parallel import plan_buckets


def _vgg_layout(align=64):
    offs, nums, o = [], [], 0
    for p in VGG11().parameters():
        offs.append(o)
        nums.append(p.numel())
        o += (p.numel() + align - 1) // align * align
    return offs, nums


def test_reverse_order_and_caps():
    offs, nums = _vgg_layout()
    b = plan_buckets(offs, nums, 4, 25 << 20, 1 << 20)
    # every parameter exactly once, buckets contiguous and in reverse parameter order
    assert b[0][1] == len(nums)
    for (s0, e0, _, _), (s1, e1, _, _) in zip(b, b[1:]):
        assert e1 == s0
    assert b[-1][0] == 0
    for i, (s, e, off, cnt) in enumerate(b):
        cap = (1 << 20) if i == 0 else (25 << 20)
        # a bucket only exceeds its cap when it holds a single oversized parameter
        assert cnt * 4 <= cap + 256 * 4 or e - s == 1


def test_native_planner_matches_python(native_ext):
    offs, nums = _vgg_layout()
    for cap, first in [(25 << 20, 1 << 20), (4 << 20, 4 << 20), (1 << 30, 1 << 30), (1 << 10, 1 << 10)]:
        py = plan_buckets(offs, nums, 4, cap, first)
        nat = [tuple(x) for x in native_ext.plan_buckets(offs, nums, 4, cap, first)]
        assert py == nat
