cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/rnlr
for i in 1 2 3; do
 for LR in 0.01 0.1; do
  L=gpurun_out/rnlr/lr${LR}_$i.log
  timeout -k 10 200 python bench.py --model resnet50 --steps 30 --warmup 10 --ref-window 0 --lr $LR > $L 2>&1 || { tail -5 $L; exit 1; }
  echo "lr=$LR run$i $(python -c "import json; d=json.loads(open('$L').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['train_loss_mean'], d['warmup_loss_sum'])")"
 done
done
