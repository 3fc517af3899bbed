#!/bin/bash
# Bootstrap an MI355X Kubernetes cluster for the fine-tune controller:
#   Kubeflow training-operator (PyTorchJob CRD), Kueue, namespace + queues, RBAC, config, services.
# Prerequisite: the AMD GPU operator (device plugin advertising amd.com/gpu) is installed.
# Options (env): NS, TRAINING_OPERATOR_VERSION, KUEUE_VERSION,
#   INSTALL_MONGO=1   also deploy a single-node MongoDB (deploy/k8s/mongodb.yaml) for test clusters,
#                     with random credentials in the ftc-mongo Secret; MONGODB_URL is printed
#   KUEUE_EXAMPLE=mixed  install the mixed-pool cohort example (deploy/kueue/examples) instead of the
#                     single ClusterQueue
set -euo pipefail
NS=${NS:-finetune}
TRAINING_OPERATOR_VERSION=${TRAINING_OPERATOR_VERSION:-v1.8.1}
KUEUE_VERSION=${KUEUE_VERSION:-v0.10.1}
HERE=$(cd "$(dirname "$0")/.." && pwd)

kubectl apply --server-side -k "github.com/kubeflow/training-operator.git/manifests/overlays/standalone?ref=${TRAINING_OPERATOR_VERSION}"
kubectl apply --server-side -f "https://github.com/kubernetes-sigs/kueue/releases/download/${KUEUE_VERSION}/manifests.yaml"
kubectl -n kueue-system rollout status deploy/kueue-controller-manager --timeout=300s

kubectl create namespace "$NS" --dry-run=client -o yaml | kubectl apply -f -
if [ "${KUEUE_EXAMPLE:-}" = "mixed" ]; then
  kubectl apply -f "$HERE/kueue/examples/flavors.yaml" -f "$HERE/kueue/examples/cluster-queues.yaml"
  sed "s/namespace: finetune/namespace: ${NS}/" "$HERE/kueue/examples/local-queues.yaml" | kubectl apply -f -
  DEVICES="$HERE/kueue/examples/config.mixed.json"
else
  kubectl apply -f "$HERE/kueue/resource-flavors.yaml" -f "$HERE/kueue/cluster-queue.yaml"
  sed "s/namespace: finetune/namespace: ${NS}/" "$HERE/kueue/local-queue.yaml" | kubectl apply -f -
  DEVICES="$HERE/config.example.json"
fi
if [ "${INSTALL_MONGO:-0}" = "1" ]; then
  if ! kubectl -n "$NS" get secret ftc-mongo >/dev/null 2>&1; then
    kubectl -n "$NS" create secret generic ftc-mongo --from-literal=username=ftc \
      --from-literal=password="$(head -c 24 /dev/urandom | base64 | tr -d '/+=')"
  fi
  sed "s/namespace: finetune/namespace: ${NS}/" "$HERE/k8s/mongodb.yaml" | kubectl apply -f -
  kubectl -n "$NS" rollout status statefulset/ftc-mongodb --timeout=300s
  echo "MongoDB: MONGODB_URL=mongodb://ftc-mongodb.${NS}.svc:27017 (credentials: secret ftc-mongo)"
fi
sed "s/namespace: finetune/namespace: ${NS}/" "$HERE/k8s/rbac.yaml" | kubectl apply -f -
kubectl -n "$NS" create configmap ftc-devices --from-file=config.json="$DEVICES" \
  --dry-run=client -o yaml | kubectl apply -f -
if [ -f "$HERE/.env" ]; then
  kubectl -n "$NS" create secret generic ftc-env --from-env-file="$HERE/.env" --dry-run=client -o yaml | kubectl apply -f -
else
  echo "note: copy deploy/.env.example to deploy/.env and re-run to create the ftc-env secret"
fi
sed "s/namespace: finetune/namespace: ${NS}/" "$HERE/k8s/controlplane.yaml" | kubectl apply -f -
echo "installed into namespace ${NS}"
