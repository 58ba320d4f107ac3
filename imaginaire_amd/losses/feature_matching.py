"""Discriminator feature matching (reference losses/feature_matching.py:8-38)."""
import torch
import torch.nn as nn
import torch.nn.functional as F


class FeatureMatchingLoss(nn.Module):
    def __init__(self, criterion='l1'):
        super().__init__()
        if criterion == 'l1':
            self.criterion = F.l1_loss
        elif criterion in ('l2', 'mse'):
            self.criterion = F.mse_loss
        else:
            raise ValueError('Criterion %s is not recognized' % criterion)

    def forward(self, fake_features, real_features):
        num_d = len(fake_features)
        dis_weight = 1.0 / num_d
        loss = fake_features[0][0].new_zeros((), dtype=torch.float32)
        for i in range(num_d):
            for j in range(len(fake_features[i])):
                loss = loss + dis_weight * self.criterion(
                    fake_features[i][j], real_features[i][j].detach()).float()
        return loss
