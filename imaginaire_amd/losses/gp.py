"""Gradient penalty for discriminators.

The reference MUNIT trainer references ``criteria['gp']`` but never creates
it (trainers/munit.py:210-222, Appendix A: crashes when ``loss_weight.gp>0``).
This implements the WGAN-GP penalty with the interface that code expects:
``get_dis_inputs(real, fake)`` → random interpolates requiring grad, and
``__call__(inputs, outputs)`` → E[(‖∇D(x̂)‖₂ − 1)²].
"""
import torch
import torch.nn as nn


class GradientPenaltyLoss(nn.Module):
    def __init__(self, target=1.0):
        super().__init__()
        self.target = target

    @staticmethod
    def get_dis_inputs(real, fake):
        alpha = torch.rand(real.size(0), 1, 1, 1, device=real.device, dtype=real.dtype)
        x = alpha * real.detach() + (1 - alpha) * fake.detach()
        return x.requires_grad_(True)

    def forward(self, inputs, outputs):
        if isinstance(outputs, (list, tuple)):
            outputs = sum(o.float().sum() for o in outputs)
        else:
            outputs = outputs.float().sum()
        grad = torch.autograd.grad(outputs, inputs, create_graph=True)[0]
        norm = grad.float().reshape(grad.size(0), -1).norm(2, dim=1)
        return ((norm - self.target) ** 2).mean()
