"""Convolution-library flags (reference utils/cudnn.py:10-22).

On ROCm ``torch.backends.cudnn`` drives MIOpen: ``benchmark=True`` runs
MIOpen's kernel search once per shape (results cached for the process).
"""
import torch.backends.cudnn as cudnn

from imaginaire_amd.utils.distributed import master_only_print as print


def init_cudnn(deterministic, benchmark):
    cudnn.deterministic = deterministic
    cudnn.benchmark = benchmark
    print('cudnn/MIOpen benchmark: {}'.format(benchmark))
    print('cudnn/MIOpen deterministic: {}'.format(deterministic))
