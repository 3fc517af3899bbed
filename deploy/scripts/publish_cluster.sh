#!/bin/bash
# In-cluster build (OpenShift BuildConfigs of deploy/openshift/buildconfigs.yaml): archive the committed
# tree and start one binary build per image -- the reference's publish_git.sh flow
# (/root/reference/scripts/publish_git.sh: `git archive` + `oc start-build --from-archive`).
#   NAMESPACE=ml bash deploy/scripts/publish_cluster.sh                  # all three images
#   NAMESPACE=ml IMAGES="ftc-worker-rocm" bash deploy/scripts/publish_cluster.sh
#   DRY_RUN=1 ...                                                        # print the oc commands only
set -euo pipefail
cd "$(dirname "$0")/../.."
if [ -z "${NAMESPACE:-}" ] && [ -f .env ]; then
  NAMESPACE=$(grep '^NAMESPACE=' .env | cut -d= -f2 || true)
fi
NAMESPACE=${NAMESPACE:-default}
IMAGES=${IMAGES:-"ftc-controlplane ftc-monitor ftc-worker-rocm"}
if [ -n "$(git status --porcelain)" ] && [ "${DIRTY_OK:-0}" != "1" ]; then
  echo "working tree has uncommitted changes: the build archives HEAD (set DIRTY_OK=1 to proceed)" >&2
  exit 1
fi
ARCHIVE=$(mktemp --suffix=.tar.gz)
trap 'rm -f "$ARCHIVE"' EXIT
git archive --format=tar HEAD | gzip > "$ARCHIVE"
run() { if [ "${DRY_RUN:-0}" = "1" ]; then echo "$*"; else "$@"; fi; }
run oc apply -n "$NAMESPACE" -f deploy/openshift/buildconfigs.yaml
for img in $IMAGES; do
  run oc start-build "$img" --from-archive="$ARCHIVE" --namespace="$NAMESPACE" --follow
done
echo "built $IMAGES in namespace $NAMESPACE from $(git rev-parse --short=12 HEAD)"
