#!/bin/bash
# Build images for several ROCm PyTorch bases (reference scripts/build_all_dockers.sh).
for BASE in "$@"; do
  bash "$(dirname "$0")/build_docker.sh" "imaginaire-amd:$(echo "$BASE" | tr '/:' '__')" "$BASE" || exit 1
done
