#!/bin/bash
# Build the three images from the repository root.
set -euo pipefail
cd "$(dirname "$0")/../.."
REG=${REG:-ghcr.io/finetune-controller-amd}
TAG=${TAG:-latest}
docker build -f deploy/docker/Dockerfile.controlplane -t "$REG/controlplane:$TAG" .
docker build -f deploy/docker/Dockerfile.monitor -t "$REG/monitor:$TAG" .
docker build -f deploy/docker/Dockerfile.worker -t "$REG/worker-rocm:$TAG" .
