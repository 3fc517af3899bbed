set -o pipefail
for c in 4096 8192 16384 4096 8192 16384; do
  FTC_CE_CHUNK=$c timeout -k 10 300 python bench.py --steps 8 --warmup 2 > gpurun_out/ce_$c.log 2>&1 || exit 1
  echo "chunk $c $(grep '^{' gpurun_out/ce_$c.log | cut -c80-150) $(grep -o '"peak_mem_gb": [0-9.]*' gpurun_out/ce_$c.log)"
done
