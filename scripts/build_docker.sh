#!/bin/bash
# Build the ROCm image (reference scripts/build_docker.sh). Usage: bash scripts/build_docker.sh [tag] [base]
TAG=${1:-imaginaire-amd:latest}
BASE=${2:-rocm/pytorch:latest}
docker build --build-arg BASE="$BASE" -t "$TAG" -f Dockerfile "$(dirname "$0")/.."
