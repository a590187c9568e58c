"""Part 1 — single-process VGG-11 training (reference: part1/main.py).

    python part1/main.py [--device auto|cpu|cuda] [--max-batches N] ...

Runs on the CPU (ATen, the reference configuration) or on one MI355X (gfx950 kernels).
Prints the reference lines: loss every 20 batches, the iteration 1-39 timing, the test summary.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from ddp_amd.engine.apps import main  # noqa: E402

if __name__ == "__main__":
    main("part1")
