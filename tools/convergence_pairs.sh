set -o pipefail
O=gpurun_out/conv2; mkdir -p $O/pairs $O/pairs1b
python tools/make_structured_tokens.py $O/pairs/tokens.npy --tokens 4000000 --vocab 512 --mode pairs > $O/pairs.log 2>&1 || exit 1
timeout -k 10 500 python -m finetune_controller_amd.train.cli --model llama3.2-1b --method full --batch-size 8 \
  --seq-len 2048 --max-steps 300 --lr 5e-4 --warmup-steps 30 --log-interval 25 --eval-every 100 --eval-holdout 0.02 \
  --dataset_path=$O/pairs --checkpoint_path=$O/pairs1b --no-resume > $O/pairs1b.log 2>&1 || { tail -20 $O/pairs1b.log; exit 1; }
grep -E "Epoch" $O/pairs1b.log | tail -16
cp $O/pairs1b/metrics.csv $O/pairs1b_metrics.csv; rm -rf $O/pairs $O/pairs1b
