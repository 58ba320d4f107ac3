#!/bin/bash
# Environment check + native build (reference scripts/install.sh: apt/conda/pip installs and three
# CUDA extension builds). ROCm images already carry PyTorch-ROCm, hipcc and the libraries; this
# script installs nothing from the network: it checks what is present, builds the gfx950
# extension in-tree and runs a CPU import check.
set -e
cd "$(dirname "$0")/.."
ROCM=${ROCM_PATH:-/opt/rocm}
[ -x "$ROCM/bin/hipcc" ] || { echo "hipcc not found under $ROCM"; exit 1; }
python - <<'PY'
import importlib, torch
print('torch', torch.__version__, 'hip', torch.version.hip)
assert torch.version.hip, 'a ROCm build of PyTorch is required'
for mod, why in [('numpy', 'core'), ('scipy', 'FID / face maps'), ('yaml', 'configs'),
                 ('PIL', 'image decode'), ('sklearn', 'PRDC / pix2pixHD clustering'),
                 ('tensorboard', 'optional: TensorBoard logging'),
                 ('imageio', 'optional: mp4 writing / native-video datasets')]:
    try:
        importlib.import_module(mod)
        print('  ok     ', mod)
    except ImportError:
        print('  missing', mod, '-', why)
PY
python -m imaginaire_amd._build "$@"
python -c "import imaginaire_amd.ops._ext as e; e.load(); print('imaginaire_amd._C loaded')"
