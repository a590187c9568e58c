cd "$GRAFT_REPO_ROOT" || exit 2
for b in 32 256; do
for i in 1 2; do
for kb in 0 256 2048; do
  DDP_AMD_BN_FOLD_BWD_KB=$kb timeout -k 10 200 python bench.py --per-gpu-batch $b --steps 60 --warmup 10 > gpurun_out/f.log 2>&1 || { tail -3 gpurun_out/f.log; exit 1; }
  echo "B=$b KB=$kb $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/f.log)"
done; done; done
