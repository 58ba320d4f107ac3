"""pix2pixHD generator (reference generators/pix2pixHD.py:18-349).

GlobalGenerator (7×7 conv, strided downsampling convs, 'CNACN' residual
blocks, nearest-up convs, tanh) with optional coarse-to-fine LocalEnhancers
and the instance-wise feature Encoder. The encoder's per-instance average
pooling runs as one device segment-mean (ops/segment.py) instead of the
reference's host-synchronising Python loops.
"""
from functools import partial

import numpy as np
import torch
import torch.nn as nn
# nn.Upsample runs in fp32 under autocast; this one is the bf16 NHWC k12 resize
from imaginaire_amd.ops.resize import Upsample as NearestUpsample

from imaginaire_amd.layers import Conv2dBlock, Res2dBlock
from imaginaire_amd.ops.pool import AvgPool2d
from imaginaire_amd.ops.segment import instance_mean
from imaginaire_amd.utils.data import (get_paired_input_image_channel_number,
                                       get_paired_input_label_channel_number)
from imaginaire_amd.utils.distributed import master_only_print as print


class Generator(nn.Module):
    def __init__(self, gen_cfg, data_cfg):
        super().__init__()
        global_gen_cfg = gen_cfg.global_generator
        num_filters_global = getattr(global_gen_cfg, 'num_filters', 64)
        local_gen_cfg = getattr(gen_cfg, 'local_enhancer', None)
        self.num_local_enhancers = num_local_enhancers = \
            getattr(local_gen_cfg, 'num_enhancers', 1) if local_gen_cfg is not None else 0
        activation_norm_type = getattr(gen_cfg, 'activation_norm_type', 'instance')
        activation_norm_params = getattr(gen_cfg, 'activation_norm_params', None)
        weight_norm_type = getattr(gen_cfg, 'weight_norm_type', '')
        padding_mode = getattr(gen_cfg, 'padding_mode', 'reflect')
        base_conv_block = partial(Conv2dBlock, padding_mode=padding_mode,
                                  weight_norm_type=weight_norm_type,
                                  activation_norm_type=activation_norm_type,
                                  activation_norm_params=activation_norm_params,
                                  nonlinearity='relu')
        base_res_block = partial(Res2dBlock, padding_mode=padding_mode,
                                 weight_norm_type=weight_norm_type,
                                 activation_norm_type=activation_norm_type,
                                 activation_norm_params=activation_norm_params,
                                 nonlinearity='relu', order='CNACN')
        num_input_channels = get_paired_input_label_channel_number(data_cfg)
        self.concat_features = False
        self.contain_instance_map = data_cfg.input_labels[-1] == 'instance_maps'
        if hasattr(gen_cfg, 'enc') and self.contain_instance_map:
            num_feat_channels = getattr(gen_cfg.enc, 'num_feat_channels', 0)
            if num_feat_channels > 0:
                num_input_channels += num_feat_channels
                self.concat_features = True
                self.encoder = Encoder(gen_cfg.enc, data_cfg)
        global_model = GlobalGenerator(global_gen_cfg, data_cfg, num_input_channels,
                                       padding_mode, base_conv_block, base_res_block)
        if num_local_enhancers == 0:
            self.global_model = global_model
        else:
            global_model = global_model.model
            self.global_model = nn.Sequential(*[global_model[i]
                                                for i in range(len(global_model) - 1)])
        for n in range(num_local_enhancers):
            num_filters = num_filters_global // (2 ** (n + 1))
            output_img = (n == num_local_enhancers - 1)
            setattr(self, 'enhancer_%d' % n,
                    LocalEnhancer(local_gen_cfg, data_cfg, num_input_channels, num_filters,
                                  padding_mode, base_conv_block, base_res_block, output_img))
        self.downsample = AvgPool2d(3, stride=2, padding=[1, 1], count_include_pad=False)

    def forward(self, data, random_style=False):
        label = data['label']
        output = dict()
        if self.concat_features:
            features = self.encoder(data['images'], data['instance_maps'])
            label = torch.cat([label, features], dim=1)
            output['feature_maps'] = features
        input_downsampled = [label]
        for _ in range(self.num_local_enhancers):
            input_downsampled.append(self.downsample(input_downsampled[-1]))
        x = self.global_model(input_downsampled[-1])
        for n in range(self.num_local_enhancers):
            input_n = input_downsampled[self.num_local_enhancers - n - 1]
            x = getattr(self, 'enhancer_%d' % n)(x, input_n)
        output['fake_images'] = x
        return output

    def load_pretrained_network(self, pretrained_dict):
        model_dict = self.state_dict()
        not_initialized = set()
        for k, v in model_dict.items():
            kp = 'module.' + k.replace('global_model.', 'global_model.model.')
            if kp in pretrained_dict and v.size() == pretrained_dict[kp].size():
                model_dict[k] = pretrained_dict[kp]
            else:
                not_initialized.add('.'.join(k.split('.')[:2]))
        print('Not initialized:', sorted(not_initialized))
        self.load_state_dict(model_dict)

    def inference(self, data, **kwargs):
        output = self.forward(data, **kwargs)
        key = data['key']
        name = key['seg_maps'][0] if isinstance(key, dict) and 'seg_maps' in key else key
        return output['fake_images'], name


class LocalEnhancer(nn.Module):
    def __init__(self, gen_cfg, data_cfg, num_input_channels, num_filters, padding_mode,
                 base_conv_block, base_res_block, output_img=False):
        super().__init__()
        num_res_blocks = getattr(gen_cfg, 'num_res_blocks', 3)
        num_img_channels = get_paired_input_image_channel_number(data_cfg)
        model_downsample = [base_conv_block(num_input_channels, num_filters, 7, padding=3),
                            base_conv_block(num_filters, num_filters * 2, 3, stride=2,
                                            padding=1)]
        model_upsample = [base_res_block(num_filters * 2, num_filters * 2, 3, padding=1)
                          for _ in range(num_res_blocks)]
        model_upsample += [NearestUpsample(scale_factor=2),
                           base_conv_block(num_filters * 2, num_filters, 3, padding=1)]
        if output_img:
            model_upsample += [Conv2dBlock(num_filters, num_img_channels, 7, padding=3,
                                           padding_mode=padding_mode, nonlinearity='tanh')]
        self.model_downsample = nn.Sequential(*model_downsample)
        self.model_upsample = nn.Sequential(*model_upsample)

    def forward(self, output_coarse, input_fine):
        return self.model_upsample(self.model_downsample(input_fine) + output_coarse)


class GlobalGenerator(nn.Module):
    def __init__(self, gen_cfg, data_cfg, num_input_channels, padding_mode, base_conv_block,
                 base_res_block):
        super().__init__()
        num_img_channels = get_paired_input_image_channel_number(data_cfg)
        num_filters = getattr(gen_cfg, 'num_filters', 64)
        num_downsamples = getattr(gen_cfg, 'num_downsamples', 4)
        num_res_blocks = getattr(gen_cfg, 'num_res_blocks', 9)
        model = [base_conv_block(num_input_channels, num_filters, kernel_size=7, padding=3)]
        for i in range(num_downsamples):
            ch = num_filters * (2 ** i)
            model += [base_conv_block(ch, ch * 2, 3, padding=1, stride=2)]
        ch = num_filters * (2 ** num_downsamples)
        for _ in range(num_res_blocks):
            model += [base_res_block(ch, ch, 3, padding=1)]
        for i in reversed(range(num_downsamples)):
            ch = num_filters * (2 ** i)
            model += [NearestUpsample(scale_factor=2), base_conv_block(ch * 2, ch, 3, padding=1)]
        model += [Conv2dBlock(num_filters, num_img_channels, 7, padding=3,
                              padding_mode=padding_mode, nonlinearity='tanh')]
        self.model = nn.Sequential(*model)

    def forward(self, input):
        return self.model(input)


class Encoder(nn.Module):
    """Instance-wise feature encoder with K-means cluster buffers (pix2pixHD.py:277-349)."""

    def __init__(self, enc_cfg, data_cfg):
        super().__init__()
        label_nc = get_paired_input_label_channel_number(data_cfg)
        feat_nc = enc_cfg.num_feat_channels
        n_clusters = getattr(enc_cfg, 'num_clusters', 10)
        for i in range(label_nc):
            self.register_buffer('cluster_%d' % i,
                                 torch.zeros(n_clusters, feat_nc, dtype=torch.float32))
        num_img_channels = get_paired_input_image_channel_number(data_cfg)
        self.num_feat_channels = getattr(enc_cfg, 'num_feat_channels', 3)
        num_filters = getattr(enc_cfg, 'num_filters', 64)
        num_downsamples = getattr(enc_cfg, 'num_downsamples', 4)
        weight_norm_type = getattr(enc_cfg, 'weight_norm_type', 'none')
        activation_norm_type = getattr(enc_cfg, 'activation_norm_type', 'instance')
        padding_mode = getattr(enc_cfg, 'padding_mode', 'reflect')
        base_conv_block = partial(Conv2dBlock, padding_mode=padding_mode,
                                  weight_norm_type=weight_norm_type,
                                  activation_norm_type=activation_norm_type,
                                  nonlinearity='relu')
        model = [base_conv_block(num_img_channels, num_filters, 7, padding=3)]
        for i in range(num_downsamples):
            ch = num_filters * (2 ** i)
            model += [base_conv_block(ch, ch * 2, 3, stride=2, padding=1)]
        for i in reversed(range(num_downsamples)):
            ch = num_filters * (2 ** i)
            model += [NearestUpsample(scale_factor=2), base_conv_block(ch * 2, ch, 3, padding=1)]
        model += [Conv2dBlock(num_filters, self.num_feat_channels, 7, padding=3,
                              padding_mode=padding_mode, nonlinearity='tanh')]
        self.model = nn.Sequential(*model)

    def forward(self, input, instance_map):
        return instance_mean(self.model(input), instance_map)
