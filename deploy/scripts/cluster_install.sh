#!/bin/bash
# Bootstrap an MI355X Kubernetes cluster for the fine-tune controller:
#   Kubeflow training-operator (PyTorchJob CRD), Kueue, namespace + queues, RBAC, config, services.
# Prerequisite: the AMD GPU operator (device plugin advertising amd.com/gpu) is installed.
set -euo pipefail
NS=${NS:-finetune}
TRAINING_OPERATOR_VERSION=${TRAINING_OPERATOR_VERSION:-v1.8.1}
KUEUE_VERSION=${KUEUE_VERSION:-v0.10.1}
HERE=$(cd "$(dirname "$0")/.." && pwd)

kubectl apply --server-side -k "github.com/kubeflow/training-operator.git/manifests/overlays/standalone?ref=${TRAINING_OPERATOR_VERSION}"
kubectl apply --server-side -f "https://github.com/kubernetes-sigs/kueue/releases/download/${KUEUE_VERSION}/manifests.yaml"
kubectl -n kueue-system rollout status deploy/kueue-controller-manager --timeout=300s

kubectl create namespace "$NS" --dry-run=client -o yaml | kubectl apply -f -
kubectl apply -f "$HERE/kueue/resource-flavors.yaml" -f "$HERE/kueue/cluster-queue.yaml"
sed "s/namespace: finetune/namespace: ${NS}/" "$HERE/kueue/local-queue.yaml" | kubectl apply -f -
sed "s/namespace: finetune/namespace: ${NS}/" "$HERE/k8s/rbac.yaml" | kubectl apply -f -
kubectl -n "$NS" create configmap ftc-devices --from-file=config.json="$HERE/config.example.json" \
  --dry-run=client -o yaml | kubectl apply -f -
if [ -f "$HERE/.env" ]; then
  kubectl -n "$NS" create secret generic ftc-env --from-env-file="$HERE/.env" --dry-run=client -o yaml | kubectl apply -f -
else
  echo "note: copy deploy/.env.example to deploy/.env and re-run to create the ftc-env secret"
fi
sed "s/namespace: finetune/namespace: ${NS}/" "$HERE/k8s/controlplane.yaml" | kubectl apply -f -
echo "installed into namespace ${NS}"
