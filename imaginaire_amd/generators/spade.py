"""SPADE / GauGAN generator (reference generators/spade.py:22-563).

Architecture, config keys and parameter names follow the reference exactly so
reference checkpoints load unchanged: ``Generator`` (optional VAE style
encoder; random / encoded / frozen style codes; ``inference`` with
``keep_original_size``), ``SPADEGenerator`` (label downsampled to H/base,
``head_0`` → CBN/conv → Res2dBlocks with SPADE norms (order NACNAC, biases
[T, T, F]) → 4× nearest-up → multi-resolution tanh heads) and
``StyleEncoder``.

MI355X execution:
  * activations are channels-last (NHWC) bf16 end to end — MIOpen's bf16 NHWC
    convolutions are 10-60 % faster than NCHW on every SPADE shape
    (profiles/conv_layout_probe_mi355x.txt);
  * every SPADE/CBN norm + leaky-ReLU is one fused HIP kernel (k1) with the γ|β
    convolutions merged into one MIOpen call per norm;
  * the nearest-resized label map is computed once per resolution per forward.
"""
import functools
import math
import types

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
from imaginaire_amd.ops.resize import Upsample as NearestUpsample

from imaginaire_amd.layers import Conv2dBlock, LinearBlock, Res2dBlock
from imaginaire_amd.layers.activation_norm import LabelMapCache
from imaginaire_amd.utils.data import (get_crop_h_w, get_paired_input_image_channel_number,
                                       get_paired_input_label_channel_number)
from imaginaire_amd.utils.distributed import master_only_print as print


def _ns(cfg):
    """AttrDict / dict / namespace → mutable SimpleNamespace copy."""
    if cfg is None:
        return types.SimpleNamespace()
    if isinstance(cfg, types.SimpleNamespace):
        return types.SimpleNamespace(**vars(cfg))
    d = dict(cfg) if isinstance(cfg, dict) else dict(vars(cfg))
    for k, v in list(d.items()):
        if isinstance(v, dict):
            d[k] = _ns(v)
    return types.SimpleNamespace(**d)


class Generator(nn.Module):
    def __init__(self, gen_cfg, data_cfg):
        super().__init__()
        print('SPADE generator initialization.')
        image_channels = get_paired_input_image_channel_number(data_cfg)
        num_labels = get_paired_input_label_channel_number(data_cfg)
        crop_h, crop_w = get_crop_h_w(data_cfg.train.augmentations)
        out_image_small_side_size = crop_w if crop_w < crop_h else crop_h
        num_filters = getattr(gen_cfg, 'num_filters', 128)
        kernel_size = getattr(gen_cfg, 'kernel_size', 3)
        weight_norm_type = getattr(gen_cfg, 'weight_norm_type', 'spectral')
        cond_dims = 0
        style_dims = getattr(gen_cfg, 'style_dims', None)
        self.style_dims = style_dims
        if style_dims is not None:
            cond_dims += style_dims
            self.use_style = True
        else:
            self.use_style = False
        if hasattr(gen_cfg, 'attribute_dims'):
            self.use_attribute = True
            self.attribute_dims = gen_cfg.attribute_dims
            cond_dims += gen_cfg.attribute_dims
        else:
            self.use_attribute = False
        self.use_style_encoder = self.use_style or self.use_attribute
        skip_activation_norm = getattr(gen_cfg, 'skip_activation_norm', True)
        activation_norm_params = _ns(getattr(gen_cfg, 'activation_norm_params', None))
        if not hasattr(activation_norm_params, 'num_filters'):
            activation_norm_params.num_filters = 128
        if not hasattr(activation_norm_params, 'kernel_size'):
            activation_norm_params.kernel_size = 3
        if not hasattr(activation_norm_params, 'activation_norm_type'):
            activation_norm_params.activation_norm_type = 'sync_batch'
        if not hasattr(activation_norm_params, 'separate_projection'):
            activation_norm_params.separate_projection = False
        if not hasattr(activation_norm_params, 'activation_norm_params'):
            activation_norm_params.activation_norm_params = types.SimpleNamespace(affine=True)
        activation_norm_params.cond_dims = num_labels
        if not hasattr(activation_norm_params, 'weight_norm_type'):
            activation_norm_params.weight_norm_type = weight_norm_type
        global_adaptive_norm_type = getattr(gen_cfg, 'global_adaptive_norm_type', 'sync_batch')
        use_posenc_in_input_layer = getattr(gen_cfg, 'use_posenc_in_input_layer', True)
        self.spade_generator = SPADEGenerator(
            num_labels, out_image_small_side_size, image_channels, num_filters, kernel_size,
            cond_dims, activation_norm_params, weight_norm_type, global_adaptive_norm_type,
            skip_activation_norm, use_posenc_in_input_layer, self.use_style_encoder)
        if self.use_style:
            style_enc_cfg = _ns(getattr(gen_cfg, 'style_enc', None))
            if not hasattr(style_enc_cfg, 'num_filters'):
                style_enc_cfg.num_filters = 128
            if not hasattr(style_enc_cfg, 'kernel_size'):
                style_enc_cfg.kernel_size = 3
            if not hasattr(style_enc_cfg, 'freeze_random'):
                style_enc_cfg.freeze_random = False
            if not hasattr(style_enc_cfg, 'weight_norm_type'):
                style_enc_cfg.weight_norm_type = weight_norm_type
            style_enc_cfg.input_image_channels = image_channels
            style_enc_cfg.style_dims = style_dims
            self.style_encoder = StyleEncoder(style_enc_cfg)
        self.z = None
        self.base = self.spade_generator.base

    def _random_z(self, data):
        bs = data['label'].size(0)
        z = torch.randn(bs, self.style_dims, dtype=torch.float32, device=data['label'].device)
        if data['label'].dtype == torch.float16:
            z = z.half()
        return z

    def forward(self, data, random_style=False):
        mu = logvar = None
        if self.use_style_encoder:
            if random_style:
                z = self._random_z(data)
            else:
                mu, logvar, z = self.style_encoder(data['images'])
            if self.use_attribute:
                data['z'] = torch.cat((z, data['attributes'].squeeze(1)), dim=1)
            else:
                data['z'] = z
        output = self.spade_generator(data)
        if self.use_style_encoder:
            output['mu'] = mu
            output['logvar'] = logvar
        return output

    def inference(self, data, random_style=False, use_fixed_random_style=False,
                  keep_original_size=False):
        self.eval()
        self.spade_generator.eval()
        if self.use_style_encoder:
            if random_style:
                if self.z is None or not use_fixed_random_style:
                    self.z = self._random_z(data)
                z = self.z
            else:
                _, _, z = self.style_encoder(data['images'])
            data['z'] = z
        output = self.spade_generator(data)
        output_images = output['fake_images']
        if keep_original_size:
            height = int(data['original_h_w'][0][0])
            width = int(data['original_h_w'][0][1])
            output_images = F.interpolate(output_images, size=[height, width])
        key = data['key']
        if isinstance(key, dict):
            file_names = key.get('seg_maps', next(iter(key.values())))[0]
        else:
            file_names = key
        return output_images, file_names


class SPADEGenerator(nn.Module):
    def __init__(self, num_labels, out_image_small_side_size, image_channels, num_filters,
                 kernel_size, style_dims, activation_norm_params, weight_norm_type,
                 global_adaptive_norm_type, skip_activation_norm, use_posenc_in_input_layer,
                 use_style_encoder):
        super().__init__()
        self.use_style_encoder = use_style_encoder
        self.use_posenc_in_input_layer = use_posenc_in_input_layer
        self.out_image_small_side_size = out_image_small_side_size
        self.num_filters = num_filters
        padding = int(np.ceil((kernel_size - 1.0) / 2))
        nonlinearity = 'leakyrelu'
        base_res2d_block = functools.partial(
            Res2dBlock, kernel_size=kernel_size, padding=padding, bias=[True, True, False],
            weight_norm_type=weight_norm_type, activation_norm_type='spatially_adaptive',
            activation_norm_params=activation_norm_params,
            skip_activation_norm=skip_activation_norm, nonlinearity=nonlinearity,
            order='NACNAC')
        if self.use_style_encoder:
            self.fc_0 = LinearBlock(style_dims, 2 * style_dims, weight_norm_type=weight_norm_type,
                                    nonlinearity='relu', order='CAN')
            self.fc_1 = LinearBlock(2 * style_dims, 2 * style_dims,
                                    weight_norm_type=weight_norm_type, nonlinearity='relu',
                                    order='CAN')
            adaptive_norm_params = types.SimpleNamespace(
                cond_dims=2 * style_dims, activation_norm_type=global_adaptive_norm_type,
                weight_norm_type=activation_norm_params.weight_norm_type,
                separate_projection=activation_norm_params.separate_projection,
                activation_norm_params=types.SimpleNamespace(
                    affine=getattr(activation_norm_params.activation_norm_params, 'affine',
                                   True)))
            base_cbn2d_block = functools.partial(
                Conv2dBlock, kernel_size=kernel_size, stride=1, padding=padding, bias=True,
                weight_norm_type=weight_norm_type, activation_norm_type='adaptive',
                activation_norm_params=adaptive_norm_params, nonlinearity=nonlinearity,
                order='NAC')
        else:
            base_conv2d_block = functools.partial(
                Conv2dBlock, kernel_size=kernel_size, stride=1, padding=padding, bias=True,
                weight_norm_type=weight_norm_type, nonlinearity=nonlinearity, order='NAC')
        in_num_labels = num_labels + (2 if self.use_posenc_in_input_layer else 0)
        self.head_0 = Conv2dBlock(in_num_labels, 8 * num_filters, kernel_size=kernel_size,
                                  stride=1, padding=padding, weight_norm_type=weight_norm_type,
                                  activation_norm_type='none', nonlinearity=nonlinearity)
        F_ = num_filters
        if self.use_style_encoder:
            self.cbn_head_0 = base_cbn2d_block(8 * F_, 16 * F_)
        else:
            self.conv_head_0 = base_conv2d_block(8 * F_, 16 * F_)
        self.head_1 = base_res2d_block(16 * F_, 16 * F_)
        self.head_2 = base_res2d_block(16 * F_, 16 * F_)
        self.up_0a = base_res2d_block(16 * F_, 8 * F_)
        if self.use_style_encoder:
            self.cbn_up_0a = base_cbn2d_block(8 * F_, 8 * F_)
        else:
            self.conv_up_0a = base_conv2d_block(8 * F_, 8 * F_)
        self.up_0b = base_res2d_block(8 * F_, 8 * F_)
        self.up_1a = base_res2d_block(8 * F_, 4 * F_)
        if self.use_style_encoder:
            self.cbn_up_1a = base_cbn2d_block(4 * F_, 4 * F_)
        else:
            self.conv_up_1a = base_conv2d_block(4 * F_, 4 * F_)
        self.up_1b = base_res2d_block(4 * F_, 4 * F_)
        self.up_2a = base_res2d_block(4 * F_, 4 * F_)
        if self.use_style_encoder:
            self.cbn_up_2a = base_cbn2d_block(4 * F_, 4 * F_)
        else:
            self.conv_up_2a = base_conv2d_block(4 * F_, 4 * F_)
        self.up_2b = base_res2d_block(4 * F_, 2 * F_)
        self.conv_img256 = Conv2dBlock(2 * F_, image_channels, 5, stride=1, padding=2,
                                       weight_norm_type=weight_norm_type,
                                       activation_norm_type='none', nonlinearity=nonlinearity,
                                       order='ANC')
        self.base = 16
        if self.out_image_small_side_size == 512:
            self.up_3a = base_res2d_block(2 * F_, 1 * F_)
            self.up_3b = base_res2d_block(1 * F_, 1 * F_)
            self.conv_img512 = Conv2dBlock(1 * F_, image_channels, 5, stride=1, padding=2,
                                           weight_norm_type=weight_norm_type,
                                           activation_norm_type='none',
                                           nonlinearity=nonlinearity, order='ANC')
            self.base = 32
        if self.out_image_small_side_size == 1024:
            self.up_3a = base_res2d_block(2 * F_, 1 * F_)
            self.up_3b = base_res2d_block(1 * F_, 1 * F_)
            self.conv_img512 = Conv2dBlock(1 * F_, image_channels, 5, stride=1, padding=2,
                                           weight_norm_type=weight_norm_type,
                                           activation_norm_type='none',
                                           nonlinearity=nonlinearity, order='ANC')
            self.up_4a = base_res2d_block(F_, F_ // 2)
            self.up_4b = base_res2d_block(F_ // 2, F_ // 2)
            self.conv_img1024 = Conv2dBlock(F_ // 2, image_channels, 5, stride=1, padding=2,
                                            weight_norm_type=weight_norm_type,
                                            activation_norm_type='none',
                                            nonlinearity=nonlinearity, order='ANC')
            self.base = 64
        if self.out_image_small_side_size not in (256, 512, 1024):
            raise ValueError('Generation image size (%d, %d) not supported' %
                             (self.out_image_small_side_size, self.out_image_small_side_size))
        self.nearest_upsample2x = NearestUpsample(scale_factor=2, mode='nearest')
        xv, yv = torch.meshgrid([torch.arange(-1, 1.1, 2. / 15), torch.arange(-1, 1.1, 2. / 15)],
                                indexing='ij')
        self.register_buffer('xy', torch.cat((xv.unsqueeze(0), yv.unsqueeze(0)), 0).unsqueeze(0),
                             persistent=False)

    def forward(self, data):
        seg = data['label']
        if seg.dim() == 4 and seg.is_cuda:
            seg = seg.contiguous(memory_format=torch.channels_last)
        with LabelMapCache():
            return self._forward(data, seg)

    def _forward(self, data, seg):
        if self.use_style_encoder:
            z = data['z']
            z = self.fc_0(z)
            z = self.fc_1(z)
        sy = math.floor(seg.size()[2] * 1.0 / self.base)
        sx = math.floor(seg.size()[3] * 1.0 / self.base)
        in_seg = LabelMapCache.resize(seg, (sy, sx))
        if self.use_posenc_in_input_layer:
            in_xy = F.interpolate(self.xy.to(seg.dtype), size=[sy, sx], mode='bicubic')
            in_seg_xy = torch.cat((in_seg, in_xy.expand(in_seg.size()[0], 2, sy, sx)), 1)
        else:
            in_seg_xy = in_seg
        x = self.head_0(in_seg_xy)
        x = self.cbn_head_0(x, z) if self.use_style_encoder else self.conv_head_0(x)
        x = self.head_1(x, seg)
        x = self.head_2(x, seg)
        x = self.nearest_upsample2x(x)
        x = self.up_0a(x, seg)
        x = self.cbn_up_0a(x, z) if self.use_style_encoder else self.conv_up_0a(x)
        x = self.up_0b(x, seg)
        x = self.nearest_upsample2x(x)
        x = self.up_1a(x, seg)
        x = self.cbn_up_1a(x, z) if self.use_style_encoder else self.conv_up_1a(x)
        x = self.up_1b(x, seg)
        x = self.nearest_upsample2x(x)
        x = self.up_2a(x, seg)
        x = self.cbn_up_2a(x, z) if self.use_style_encoder else self.conv_up_2a(x)
        x = self.up_2b(x, seg)
        if self.out_image_small_side_size == 256 and x.is_cuda and \
                list(self.conv_img256.layers.keys())[:1] == ['nonlinearity']:
            # the head's leading activation commutes with the nearest upsampling: applied before
            # it, on a quarter of the pixels (the 2 x F-channel full-resolution map is the
            # largest activation of the generator)
            act = self.conv_img256.layers['nonlinearity']
            x = self.nearest_upsample2x(act(x))
            x = torch.tanh(self.conv_img256(x, skip_first_act=True))
        elif self.out_image_small_side_size == 256:
            x = self.nearest_upsample2x(x)
            x = torch.tanh(self.conv_img256(x))
        elif self.out_image_small_side_size == 512:
            x256 = self.nearest_upsample2x(self.conv_img256(x))
            x = self.up_3a(x, seg)
            x = self.up_3b(x, seg)
            x = self.nearest_upsample2x(x)
            x = torch.tanh(x256 + self.conv_img512(x))
        else:
            x256 = self.nearest_upsample2x(self.conv_img256(x))
            x = self.up_3a(x, seg)
            x = self.up_3b(x, seg)
            x = self.nearest_upsample2x(x)
            x512 = self.nearest_upsample2x(self.conv_img512(x))
            x = self.up_4a(x, seg)
            x = self.up_4b(x, seg)
            x = self.nearest_upsample2x(x)
            x = torch.tanh(x256 + x512 + self.conv_img1024(x))
        return {'fake_images': x}


class StyleEncoder(nn.Module):
    """VAE style encoder: 6 stride-2 convs → μ, log σ² (spade.py:496-563)."""

    def __init__(self, style_enc_cfg):
        super().__init__()
        input_image_channels = style_enc_cfg.input_image_channels
        num_filters = style_enc_cfg.num_filters
        kernel_size = style_enc_cfg.kernel_size
        padding = int(np.ceil((kernel_size - 1.0) / 2))
        style_dims = style_enc_cfg.style_dims
        weight_norm_type = style_enc_cfg.weight_norm_type
        base_conv2d_block = functools.partial(
            Conv2dBlock, kernel_size=kernel_size, stride=2, padding=padding,
            weight_norm_type=weight_norm_type, activation_norm_type='none',
            nonlinearity='leakyrelu')
        self.layer1 = base_conv2d_block(input_image_channels, num_filters)
        self.layer2 = base_conv2d_block(num_filters * 1, num_filters * 2)
        self.layer3 = base_conv2d_block(num_filters * 2, num_filters * 4)
        self.layer4 = base_conv2d_block(num_filters * 4, num_filters * 8)
        self.layer5 = base_conv2d_block(num_filters * 8, num_filters * 8)
        self.layer6 = base_conv2d_block(num_filters * 8, num_filters * 8)
        self.fc_mu = LinearBlock(num_filters * 8 * 4 * 4, style_dims)
        self.fc_var = LinearBlock(num_filters * 8 * 4 * 4, style_dims)
        self.freeze_random = style_enc_cfg.freeze_random
        self.eps = None

    def forward(self, input_x):
        if input_x.size(2) != 256 or input_x.size(3) != 256:
            input_x = F.interpolate(input_x, size=(256, 256), mode='bilinear')
        x = self.layer1(input_x)
        x = self.layer2(x)
        x = self.layer3(x)
        x = self.layer4(x)
        x = self.layer5(x)
        x = self.layer6(x)
        # flatten in NCHW order (matches the reference fc weight layout)
        x = x.contiguous().view(x.size(0), -1)
        mu = self.fc_mu(x)
        logvar = self.fc_var(x)
        std = torch.exp(0.5 * logvar)
        if self.eps is None or not self.freeze_random:
            eps = torch.randn_like(std)
            self.eps = eps
        else:
            eps = self.eps
        z = eps.mul(std) + mu
        return mu, logvar, z
