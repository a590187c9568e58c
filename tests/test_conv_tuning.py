"""The measured conv tile / split-K table (ops/conv_tuning.json, written by tools/conv_tune.py)
is well-formed: every entry names a valid tile and split factor for a GEMM problem, and the
recorded winner was not slower than the cost-model choice it replaces."""
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TABLE = os.path.join(ROOT, "distributed-data-parallel-ml-training_amd", "ops", "conv_tuning.json")


@pytest.mark.skipif(not os.path.exists(TABLE), reason="no tuning table")
def test_tuning_table_well_formed():
    with open(TABLE) as f:
        t = json.load(f)
    keys = set()
    for e in t["entries"]:
        assert e["mode"] in (0, 1, 2, 3)
        if e["mode"] == 3:  # backward pair: tile = 0 separate / pair tile 1..4, splits / stages = DGRAD / WGRAD
            assert e["tile"] in (0, 1, 2, 3, 4, 5) and 1 <= e["splits"] <= 16 and 1 <= e["stages"] <= 128
        else:
            assert 0 <= e["tile"] <= 7
            # split-K slabs (splits x M x N fp32) must fit the 32 Mi-element workspace
            # (ops/common.py WORKSPACE_ELEMS); the stem WGRAD's 512-way split is the largest
            assert 1 <= e["splits"] <= 1024
            assert e["splits"] == 1 or e["splits"] * e["M"] * e["N"] <= 32 << 20
        assert min(e["M"], e["N"], e["K"]) > 0
        if "auto_us" in e:  # (hand-added entries from a dedicated sweep carry a "note" instead)
            assert e["us"] <= e["auto_us"] + 1e-6
        elif "step_ms" in e:  # tools/step_tune.py: timed inside the captured step
            assert e["mode"] == 3 and e["step_ms"] > 0 and e["H"] >= 1
        else:
            assert "note" in e
        keys.add((e["mode"], e["M"], e["N"], e["K"], e.get("H", 0)))
    # unique keys (pair entries are keyed by the layer's H too: different layers share GEMM dims)
    assert len(keys) == len(t["entries"])
    # the flagship VGG-11 b256 problems are covered (e.g. layers.18 fwd: M=256*4*4, N=512)
    assert (0, 256 * 16, 512, 9 * 512, 0) in keys
