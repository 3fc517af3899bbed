set -o pipefail
for w in default 262144 default 262144; do
  if [ $w = default ]; then unset HIPBLASLT_WORKSPACE_SIZE; else export HIPBLASLT_WORKSPACE_SIZE=$w; fi
  timeout -k 10 300 python bench.py --steps 8 --warmup 2 > gpurun_out/ws_$w.log 2>&1 || exit 1
  echo "ws=$w $(grep '^{' gpurun_out/ws_$w.log | cut -c80-140)"
done
