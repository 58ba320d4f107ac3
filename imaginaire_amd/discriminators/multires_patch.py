"""Multi-resolution PatchGAN discriminators (reference discriminators/multires_patch.py:19-313).

The strided 4×4 convolutions run bias-free on MIOpen (NHWC bf16) with the
bias + leaky-ReLU applied by the fused HIP epilogue (k2) through Conv2dBlock.
"""
import functools
import os
import warnings

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from imaginaire_amd.layers import Conv2dBlock
from imaginaire_amd.layers.spectral_norm import extra_sn_power_iteration
from imaginaire_amd.utils.data import (get_paired_input_image_channel_number,
                                       get_paired_input_label_channel_number)
from imaginaire_amd.utils.distributed import master_only_print as print
from imaginaire_amd.ops import _ext
from imaginaire_amd.ops.conv import stack_nhwc
from imaginaire_amd.ops.resize import interpolate


class Discriminator(nn.Module):
    """Label ⊕ image multi-res patch discriminator (multires_patch.py:19-100)."""

    def __init__(self, dis_cfg, data_cfg):
        super().__init__()
        image_channels = get_paired_input_image_channel_number(data_cfg)
        num_labels = get_paired_input_label_channel_number(data_cfg)
        kernel_size = getattr(dis_cfg, 'kernel_size', 3)
        num_filters = getattr(dis_cfg, 'num_filters', 128)
        max_num_filters = getattr(dis_cfg, 'max_num_filters', 512)
        num_discriminators = getattr(dis_cfg, 'num_discriminators', 2)
        num_layers = getattr(dis_cfg, 'num_layers', 5)
        activation_norm_type = getattr(dis_cfg, 'activation_norm_type', 'none')
        weight_norm_type = getattr(dis_cfg, 'weight_norm_type', 'spectral')
        num_input_channels = image_channels + num_labels
        # D update: fake and real as ONE batch-concatenated pass (per-sample layers only; SN
        # iterations kept: see ``forward``). IMAGINAIRE_AMD_DIS_BATCH=0: A/B switch.
        self.batched = getattr(dis_cfg, 'batch_real_fake', True) and \
            activation_norm_type in ('none', '', 'instance') and \
            os.environ.get('IMAGINAIRE_AMD_DIS_BATCH', '1') != '0'
        self.model = MultiResPatchDiscriminator(num_discriminators, kernel_size,
                                                num_input_channels, num_filters, num_layers,
                                                max_num_filters, activation_norm_type,
                                                weight_norm_type)

    @staticmethod
    def _input(label, image):
        # GPU: label|image written once into a 64-channel-aligned bf16 NHWC buffer with its
        # zero tail marked — the first conv consumes it without re-padding, and the
        # downsampling for the coarser scales runs on the k12 kernel in bf16 (a 39-channel
        # Cityscapes label|image pair otherwise took an fp32 copy + fp32 bilinear per scale)
        if label.is_cuda and _ext.use_native(label):
            return stack_nhwc([[label, image]])
        return torch.cat((label, image), 1)

    def forward(self, data, net_G_output, real=True):
        output_x = dict()
        fake = net_G_output['fake_images']
        if real and self.batched and fake.shape == data['images'].shape and \
                not (torch.is_grad_enabled() and fake.requires_grad):
            # D update (fake detached): the reference's fake and real passes as one pass over
            # the concatenated batch; the real pass's spectral-norm power iteration runs first
            # (u / v advance as in the reference, both halves see the second σ — see
            # discriminators/spade.py). The G update keeps two passes: its real pass needs no
            # backward.
            extra_sn_power_iteration(self)
            real_img = data['images']
            if 'label' in data:
                label = data['label']
                if label.is_cuda and _ext.use_native(label):
                    x = stack_nhwc([[label, fake], [label, real_img]])
                else:
                    x = torch.cat((torch.cat((label, fake.to(real_img.dtype)), 1),
                                   torch.cat((label, real_img), 1)), 0)
            else:
                x = torch.cat((fake.to(real_img.dtype), real_img), 0)
            outs, feats, _ = self.model(x)
            n = fake.shape[0]
            output_x['fake_outputs'] = [o[:n] for o in outs]
            output_x['real_outputs'] = [o[n:] for o in outs]
            output_x['fake_features'] = [[f[:n] for f in fl] for fl in feats]
            output_x['real_features'] = [[f[n:] for f in fl] for fl in feats]
            return output_x
        if 'label' in data:
            fake_input_x = self._input(data['label'], net_G_output['fake_images'])
        else:
            fake_input_x = net_G_output['fake_images']
        output_x['fake_outputs'], output_x['fake_features'], _ = self.model(fake_input_x)
        if real:
            if 'label' in data:
                real_input_x = self._input(data['label'], data['images'])
            else:
                real_input_x = data['images']
            output_x['real_outputs'], output_x['real_features'], _ = self.model(real_input_x)
        return output_x


def _down2(x):
    return interpolate(x, scale_factor=0.5, mode='bilinear', align_corners=True,
                       recompute_scale_factor=True)


class MultiResPatchDiscriminator(nn.Module):
    def __init__(self, num_discriminators=3, kernel_size=3, num_image_channels=3,
                 num_filters=64, num_layers=4, max_num_filters=512, activation_norm_type='',
                 weight_norm_type='', **kwargs):
        super().__init__()
        for key in kwargs:
            if key != 'type' and key != 'patch_wise':
                warnings.warn("Discriminator argument {} is not used".format(key))
        self.discriminators = nn.ModuleList()
        for _ in range(num_discriminators):
            self.discriminators.append(NLayerPatchDiscriminator(
                kernel_size, num_image_channels, num_filters, num_layers, max_num_filters,
                activation_norm_type, weight_norm_type))

    def forward(self, input_x):
        input_list, output_list, features_list = [], [], []
        input_downsampled = input_x
        for net_discriminator in self.discriminators:
            input_list.append(input_downsampled)
            output, features = net_discriminator(input_downsampled)
            output_list.append(output)
            features_list.append(features)
            input_downsampled = _down2(input_downsampled)
        return output_list, features_list, input_list


class WeightSharedMultiResPatchDiscriminator(nn.Module):
    def __init__(self, num_discriminators=3, kernel_size=3, num_image_channels=3,
                 num_filters=64, num_layers=4, max_num_filters=512, activation_norm_type='',
                 weight_norm_type='', **kwargs):
        super().__init__()
        for key in kwargs:
            if key != 'type' and key != 'patch_wise':
                warnings.warn("Discriminator argument {} is not used".format(key))
        self.num_discriminators = num_discriminators
        self.discriminator = NLayerPatchDiscriminator(kernel_size, num_image_channels,
                                                      num_filters, num_layers, max_num_filters,
                                                      activation_norm_type, weight_norm_type)

    def forward(self, input_x):
        input_list, output_list, features_list = [], [], []
        input_downsampled = input_x
        for _ in range(self.num_discriminators):
            input_list.append(input_downsampled)
            output, features = self.discriminator(input_downsampled)
            output_list.append(output)
            features_list.append(features)
            input_downsampled = interpolate(input_downsampled, scale_factor=0.5,
                                            mode='bilinear', align_corners=True)
        return output_list, features_list, input_list


class NLayerPatchDiscriminator(nn.Module):
    def __init__(self, kernel_size, num_input_channels, num_filters, num_layers,
                 max_num_filters, activation_norm_type, weight_norm_type):
        super().__init__()
        self.num_layers = num_layers
        padding = int(np.floor((kernel_size - 1.0) / 2))
        base_conv2d_block = functools.partial(
            Conv2dBlock, kernel_size=kernel_size, padding=padding,
            weight_norm_type=weight_norm_type, activation_norm_type=activation_norm_type,
            nonlinearity='leakyrelu', order='CNA')
        layers = [[base_conv2d_block(num_input_channels, num_filters, stride=2)]]
        for n in range(num_layers):
            num_filters_prev = num_filters
            num_filters = min(num_filters * 2, max_num_filters)
            stride = 2 if n < (num_layers - 1) else 1
            layers += [[base_conv2d_block(num_filters_prev, num_filters, stride=stride)]]
        layers += [[Conv2dBlock(num_filters, 1, 3, 1, padding,
                                weight_norm_type=weight_norm_type)]]
        for n in range(len(layers)):
            setattr(self, 'layer' + str(n), nn.Sequential(*layers[n]))

    def forward(self, input_x):
        res = [input_x]
        for n in range(self.num_layers + 2):
            layer = getattr(self, 'layer' + str(n))
            res.append(layer(res[-1]))
        return res[-1], res[1:-1]
