# Starts the exporter with the DaemonSet's container args (deploy/kubernetes/daemonset.yaml)
# on a GPU box outside Kubernetes (rccl dir and pod-log dir under /tmp), scrapes it once,
# and prints the family list and the source status line.
set -u
D=/tmp/gpuexp-ds && mkdir -p $D/rccl $D/pods
timeout -k 5 40 python -m kubernetes_gpu_exporter_amd --backend=amdsmi --listen=127.0.0.1:18000 --path=/metrics \
  --interval=1 --enable-sentinel=true --enable-counters=true --series-profile=full --enable-rccl=true \
  --rccl-dir=$D/rccl --pod-logdir=$D/pods --log-level=info > $D/exporter.log 2>&1 &
P=$!
for i in $(seq 1 30); do sleep 1; curl -sf http://127.0.0.1:18000/readyz > /dev/null && break; done
sleep 3
curl -s http://127.0.0.1:18000/metrics > $D/metrics.txt
echo "families: $(grep -c '^# TYPE' $D/metrics.txt)  series: $(grep -vc '^#' $D/metrics.txt)"
grep '^# TYPE' $D/metrics.txt | awk '{print $3}' | tr '\n' ' '; echo
grep 'gpuexp_source_up' $D/metrics.txt
kill $P; wait $P
tail -5 $D/exporter.log
