#!/bin/bash
# round 4: the bench's own loss over steps 10..19 (lr 0.1 headline regime), run to run
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r4z12; mkdir -p $O
for i in 1 2 3 4 5 6; do
  timeout -k 10 200 python bench.py --steps 10 --warmup 10 --ref-window 0 > $O/run$i.log 2>&1 || { tail -5 $O/run$i.log; exit 1; }
  echo "run$i $(tail -1 $O/run$i.log | grep -oE '"(train_loss_mean|warmup_loss_sum)": [0-9.]+' | tr '\n' ' ')"
done
