cd "$GRAFT_REPO_ROOT" || exit 2
for b in 64 128 256; do
timeout -k 10 300 python bench.py --model resnet50 --per-gpu-batch $b --steps 10 --warmup 3 > gpurun_out/rb_$b.log 2>&1 || { tail -3 gpurun_out/rb_$b.log; exit 1; }
echo "B=$b $(grep -o '"value": [0-9.]*' gpurun_out/rb_$b.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/rb_$b.log)"
done
