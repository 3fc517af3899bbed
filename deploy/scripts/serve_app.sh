#!/bin/bash
# Local API server (dev): in-process fakes unless the env says otherwise.
export STORE_BACKEND=${STORE_BACKEND:-memory} OBJECT_STORE=${OBJECT_STORE:-local:/tmp/ftc-objects} \
       KUBE_BACKEND=${KUBE_BACKEND:-fake} NAMESPACE=${NAMESPACE:-finetune} S3_BUCKET_NAME=${S3_BUCKET_NAME:-ftc} \
       AWS_SECRET_NAME=${AWS_SECRET_NAME:-none} DEV_LOCAL_JOB_MONITOR=${DEV_LOCAL_JOB_MONITOR:-true}
exec uvicorn finetune_controller_amd.controlplane.api.app:app_from_env --factory --host 0.0.0.0 --port "${PORT:-8000}" \
  --ws-per-message-deflate false "$@"
