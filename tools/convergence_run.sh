#!/bin/bash
# Does training on the GPU actually learn?  Structured synthetic corpus (tools/make_structured_tokens.py:
# copy / induction windows), the worker CLI end to end (native loader, HIP kernels, metrics.csv,
# held-out eval, checkpoints), then a kill-free resume: a second invocation continues from the newest
# checkpoint_step*.pt.  -> gpurun_out/conv/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/conv
mkdir -p $O/data $O/pairs $O/full1b $O/pairs1b $O/lora8b
python tools/make_structured_tokens.py $O/data/tokens.npy --tokens 6000000 --vocab 512 --chunk 64 > $O/data.log 2>&1 || exit 1
cat $O/data.log
# 1) Llama-3.2-1B full fine-tune from random init
timeout -k 10 500 python -m finetune_controller_amd.train.cli --model llama3.2-1b --method full --batch-size 8 \
  --seq-len 2048 --max-steps 500 --lr 5e-4 --warmup-steps 50 --log-interval 25 --eval-every 100 --eval-holdout 0.02 \
  --dataset_path=$O/data --checkpoint_path=$O/full1b --no-resume > $O/full1b.log 2>&1 || { tail -20 $O/full1b.log; exit 1; }
grep -E "Epoch" $O/full1b.log | tail -26
# 1b) the same model on repeated pairs (a a b b ...): only attention to the previous position predicts
#     the second token of a pair; ideal loss ln(512) / 2 = 3.12
python tools/make_structured_tokens.py $O/pairs/tokens.npy --tokens 4000000 --vocab 512 --mode pairs > $O/pairs.log 2>&1 || exit 1
timeout -k 10 500 python -m finetune_controller_amd.train.cli --model llama3.2-1b --method full --batch-size 8 \
  --seq-len 2048 --max-steps 300 --lr 5e-4 --warmup-steps 30 --log-interval 25 --eval-every 100 --eval-holdout 0.02 \
  --dataset_path=$O/pairs --checkpoint_path=$O/pairs1b --no-resume > $O/pairs1b.log 2>&1 || { tail -20 $O/pairs1b.log; exit 1; }
grep -E "Epoch" $O/pairs1b.log | tail -16
# 2) Llama-3-8B LoRA r16 all-linear, 61 steps with resume checkpoints at 30 and 60 ...
timeout -k 10 500 python -m finetune_controller_amd.train.cli --model llama3-8b --method lora --batch-size 4 \
  --seq-len 4096 --max-steps 61 --lr 2e-4 --warmup-steps 10 --schedule constant --log-interval 10 --save-every 30 \
  --dataset_path=$O/data --checkpoint_path=$O/lora8b > $O/lora8b_a.log 2>&1 || { tail -20 $O/lora8b_a.log; exit 1; }
grep -E "Epoch" $O/lora8b_a.log | tail -7
ls $O/lora8b
# ... then continued to 120 steps by a second process: it must resume from checkpoint_step60
timeout -k 10 500 python -m finetune_controller_amd.train.cli --model llama3-8b --method lora --batch-size 4 \
  --seq-len 4096 --max-steps 120 --lr 2e-4 --warmup-steps 10 --schedule constant --log-interval 10 --save-every 30 \
  --dataset_path=$O/data --checkpoint_path=$O/lora8b > $O/lora8b_b.log 2>&1 || { tail -20 $O/lora8b_b.log; exit 1; }
grep -iE "resum|Epoch" $O/lora8b_b.log | tail -8
cp $O/full1b/metrics.csv $O/full1b_metrics.csv 2>/dev/null; cp $O/lora8b/metrics.csv $O/lora8b_metrics.csv 2>/dev/null
rm -rf $O/data $O/pairs $O/pairs1b/*.safetensors $O/full1b/*.safetensors $O/lora8b/*.pt $O/lora8b/*.safetensors
exit 0
