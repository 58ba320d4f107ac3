#!/bin/bash
# Run the image with every GPU of the node visible (reference scripts/start_local_docker.sh;
# ROCm exposes GPUs through /dev/kfd + /dev/dri instead of the NVIDIA runtime).
TAG=${1:-imaginaire-amd:latest}
docker run --rm -it --network host --ipc host --shm-size 64g \
  --device /dev/kfd --device /dev/dri --group-add video --security-opt seccomp=unconfined \
  -e HSA_ENABLE_IPC_MODE_LEGACY=0 -v "$(pwd)":/workspace/imaginaire_amd "$TAG" bash
