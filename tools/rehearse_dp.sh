#!/bin/bash
# Rehearse the multi-rank bench path on a ONE-GPU box: N ranks share the card (FTC_SHARE_GPU=1), so
# the torchrun launch, rendezvous, parameter broadcast, bucketed backward-overlapped all-reduce,
# timing max-reduction and rank-0 JSON line all run exactly as on an 8-GPU node.  RCCL refuses two
# ranks on one device, so the collectives go through gloo (FTC_DIST_BACKEND=gloo) unless
# BACKEND=nccl is given.  Usage: [TAG=name] bash tools/rehearse_dp.sh [N=2] [extra bench args]
# -> gpurun_out/rehearse_dp{N}_{backend}[_TAG].log
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
N=${1:-2}; shift || true
mkdir -p gpurun_out
FTC_SHARE_GPU=1 FTC_DIST_BACKEND=${BACKEND:-gloo} timeout -k 10 ${REHEARSE_TIMEOUT:-400} \
  python -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus "$N" "$@" > gpurun_out/rehearse_dp${N}_${BACKEND:-gloo}${TAG:+_$TAG}.log 2>&1
rc=$?
tail -3 gpurun_out/rehearse_dp${N}_${BACKEND:-gloo}${TAG:+_$TAG}.log | cut -c1-400
exit $rc
