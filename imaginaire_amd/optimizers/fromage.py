"""Fromage optimizer (reference optimizers/fromage.py:11-44; Bernstein et al. 2020)."""
import math

import torch
from torch.optim.optimizer import Optimizer, required


class Fromage(Optimizer):
    def __init__(self, params, lr=required, momentum=0):
        defaults = dict(lr=lr, momentum=momentum)
        super().__init__(params, defaults)

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        for group in self.param_groups:
            for p in group['params']:
                if p.grad is None:
                    continue
                d_p = p.grad
                d_p_norm = p.grad.norm()
                p_norm = p.norm()
                if p_norm > 0.0 and d_p_norm > 0.0:
                    p.add_(d_p * (p_norm / d_p_norm), alpha=-group['lr'])
                else:
                    p.add_(d_p, alpha=-group['lr'])
                p.mul_(1 / math.sqrt(1 + group['lr'] ** 2))
        return loss
