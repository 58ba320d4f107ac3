"""Global residual discriminator (reference discriminators/residual.py:13-92)."""
import warnings

import torch
import torch.nn as nn

from imaginaire_amd.layers import Conv2dBlock, Res2dBlock
from imaginaire_amd.ops.pool import AvgPool2d


class ResDiscriminator(nn.Module):
    def __init__(self, image_channels=3, num_filters=64, max_num_filters=512,
                 first_kernel_size=1, num_layers=4, padding_mode='zeros',
                 activation_norm_type='', weight_norm_type='', aggregation='conv',
                 order='pre_act', anti_aliased=False, **kwargs):
        super().__init__()
        for key in kwargs:
            if key not in ('type', 'patch_wise', 'common', 'patch_dis'):
                warnings.warn("Discriminator argument {} is not used".format(key))
        conv_params = dict(padding_mode=padding_mode, activation_norm_type=activation_norm_type,
                           weight_norm_type=weight_norm_type, nonlinearity='leakyrelu')
        first_padding = (first_kernel_size - 1) // 2
        model = [Conv2dBlock(image_channels, num_filters, first_kernel_size, 1, first_padding,
                             **conv_params)]
        for _ in range(num_layers):
            num_filters_prev = num_filters
            num_filters = min(num_filters * 2, max_num_filters)
            model.append(Res2dBlock(num_filters_prev, num_filters, order=order, **conv_params))
            model.append(AvgPool2d(2, stride=2))
        if aggregation == 'pool':
            model += [torch.nn.AdaptiveAvgPool2d(1)]
        elif aggregation == 'conv':
            model += [Conv2dBlock(num_filters, num_filters, 4, 1, 0, nonlinearity='leakyrelu')]
        else:
            raise ValueError('The aggregation mode %s is not recognized' % aggregation)
        self.model = nn.Sequential(*model)
        self.classifier = nn.Linear(num_filters, 1)

    def forward(self, images):
        batch_size = images.size(0)
        features = self.model(images)
        outputs = self.classifier(features.reshape(batch_size, -1))
        return outputs, features, images
