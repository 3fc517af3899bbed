set -o pipefail
O=gpurun_out/tail_ab2; mkdir -p $O
P=finetune_controller_amd
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_kernels_gpu.py -k "rmsnorm or llama3_8b" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rb in 16 8; do
  cp $P/_C_rb$rb.so $P/_C.so
  timeout -k 10 120 python -u tools/bench_norm_tail.py > $O/micro_rb$rb.log 2>&1 || { tail $O/micro_rb$rb.log; exit 1; }
  echo "rb$rb: $(cat $O/micro_rb$rb.log | grep shape | tr '\n' ' ')"
done
cp $P/_C_rb8.so $P/_C.so
for r in 1 2 3; do
  for arm in fused off; do
    if [ $arm = off ]; then pre="finetune_controller_amd.ops.norm._TAIL_OFF=True"; else pre="finetune_controller_amd.ops.norm._TAIL_OFF=False"; fi
    timeout -k 10 300 python -u tools/run_patched.py $pre -- bench.py > $O/${arm}_r$r.log 2>&1 || { tail -20 $O/${arm}_r$r.log; exit 1; }
    echo "$arm r$r $(grep '^{' $O/${arm}_r$r.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
