# MI355X (gfx950) image (reference Dockerfile.base builds on NGC PyTorch + CUDA extensions).
# The base already ships PyTorch-ROCm, hipcc, MIOpen, hipBLASLt and RCCL.
ARG BASE=rocm/pytorch:latest
FROM ${BASE}
ENV PYTORCH_ROCM_ARCH=gfx950 HSA_ENABLE_IPC_MODE_LEGACY=0
RUN pip install --no-cache-dir pyyaml pillow scipy scikit-learn tensorboard imageio
WORKDIR /workspace/imaginaire_amd
COPY . .
RUN python -m imaginaire_amd._build
