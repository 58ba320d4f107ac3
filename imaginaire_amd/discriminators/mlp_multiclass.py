"""MLP multi-class classifier (reference discriminators/mlp_multiclass.py:13-63)."""
import functools

import numpy as np
import torch.nn as nn

from imaginaire_amd.layers import LinearBlock


class Discriminator(nn.Module):
    def __init__(self, dis_cfg, data_cfg):
        super().__init__()
        num_input_channels = dis_cfg.input_dims
        num_labels = dis_cfg.num_labels
        num_layers = getattr(dis_cfg, 'num_layers', 5)
        num_filters = getattr(dis_cfg, 'num_filters', 512)
        activation_norm_type = getattr(dis_cfg, 'activation_norm_type', 'batch_norm')
        if activation_norm_type == 'batch_norm':
            activation_norm_type = 'batch'
        nonlinearity = getattr(dis_cfg, 'nonlinearity', 'leakyrelu')
        base_linear_block = functools.partial(LinearBlock,
                                              activation_norm_type=activation_norm_type,
                                              nonlinearity=nonlinearity, order='CNA')
        dropout_ratio = 0.1
        layers = [base_linear_block(num_input_channels, num_filters), nn.Dropout(dropout_ratio)]
        for _ in range(num_layers):
            dropout_ratio = float(np.min([dropout_ratio * 1.5, 0.5]))
            layers += [base_linear_block(num_filters, num_filters), nn.Dropout(dropout_ratio)]
        layers += [LinearBlock(num_filters, num_labels)]
        self.model = nn.Sequential(*layers)

    def forward(self, data):
        input_x = data['data']
        return {'results': self.model(input_x.reshape(input_x.size(0), -1))}
