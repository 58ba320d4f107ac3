"""Gaussian KL divergence (reference losses/kl.py:9-23): -0.5·Σ(1+logvar-μ²-e^logvar)."""
import torch
import torch.nn as nn


class GaussianKLLoss(nn.Module):
    def forward(self, mu, logvar=None):
        mu = mu.float()
        if logvar is None:
            logvar = torch.zeros_like(mu)
        logvar = logvar.float()
        return -0.5 * torch.sum(1 + logvar - mu.pow(2) - logvar.exp())
