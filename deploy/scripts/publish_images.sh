#!/bin/bash
# Build and push the controller, monitor and MI355X worker images (the reference's publish_git.sh /
# publish_local.sh).  The tag is the git commit by default, so a cluster pins exactly what was tested.
#   REG=registry.example.com/ftc bash deploy/scripts/publish_images.sh            # tag = short SHA
#   TAG=v0.2.0 LATEST=1 bash deploy/scripts/publish_images.sh                     # also move :latest
#   DIRTY_OK=1 ...                                                                # allow a dirty tree
set -euo pipefail
cd "$(dirname "$0")/../.."
REG=${REG:-ghcr.io/finetune-controller-amd}
if [ -n "$(git status --porcelain)" ] && [ "${DIRTY_OK:-0}" != "1" ]; then
  echo "working tree has uncommitted changes (set DIRTY_OK=1 to publish anyway)" >&2
  exit 1
fi
TAG=${TAG:-$(git rev-parse --short=12 HEAD)}
REG=$REG TAG=$TAG bash deploy/scripts/build_images.sh
for img in controlplane monitor worker-rocm; do
  docker push "$REG/$img:$TAG"
  if [ "${LATEST:-0}" = "1" ]; then
    docker tag "$REG/$img:$TAG" "$REG/$img:latest"
    docker push "$REG/$img:latest"
  fi
done
echo "published $REG/{controlplane,monitor,worker-rocm}:$TAG"
