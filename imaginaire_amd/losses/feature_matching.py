"""Discriminator feature matching (reference losses/feature_matching.py:8-38)."""
import torch
import torch.nn as nn
import torch.nn.functional as F

from imaginaire_amd.ops.loss import weighted_l1


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
        if self.criterion is F.l1_loss:
            # every (fake, real) feature pair in one multi-tensor L1 (k13 on the GPU)
            fs = [f for i in range(num_d) for f in fake_features[i]]
            rs = [r for i in range(num_d) for r in real_features[i]]
            return weighted_l1(fs, rs, [dis_weight] * len(fs))
        loss = fake_features[0][0].new_zeros((), dtype=torch.float32)
        for i in range(num_d):
            for j in range(len(fake_features[i])):
                loss = loss + dis_weight * self.criterion(
                    fake_features[i][j], real_features[i][j].detach()).float()
        return loss
