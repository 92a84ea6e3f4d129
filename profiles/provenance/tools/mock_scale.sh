set -e
mkdir -p gpurun_out/mockscale
for n in 1 2 4 8; do
  timeout -k 10 200 python bench.py --gpus $n --backend mock --steps 100 --warmup 10 --identity-phase 0 --xgmi-patterns 0 > gpurun_out/mockscale/n$n.json 2>> gpurun_out/mockscale/stderr.log
  echo "done n=$n"
done
