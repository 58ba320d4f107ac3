"""MUNIT generator (reference generators/munit.py:16-465).

Content encoder (shared with UNIT), style encoder (strided convs → global
average pool → 1×1 conv), AdaIN decoder whose adaptive norms run as fused
instance-norm + per-(n,c) modulation + ReLU HIP kernels, and the style MLP.
"""
import warnings
from types import SimpleNamespace

import torch
from torch import nn
# nn.Upsample runs in fp32 under autocast; this one is the bf16 NHWC k12 resize
from imaginaire_amd.ops.resize import Upsample as NearestUpsample

from imaginaire_amd.generators.unit import ContentEncoder, _kw, _name
from imaginaire_amd.layers.conv import NHWCConv2d
from imaginaire_amd.layers import Conv2dBlock, LinearBlock, Res2dBlock


class Generator(nn.Module):
    def __init__(self, gen_cfg, data_cfg):
        super().__init__()
        self.autoencoder_a = AutoEncoder(**_kw(gen_cfg))
        self.autoencoder_b = AutoEncoder(**_kw(gen_cfg))

    def forward(self, data, random_style=True, image_recon=True, latent_recon=True,
                cycle_recon=True, within_latent_recon=False):
        images_a, images_b = data['images_a'], data['images_b']
        out = dict()
        content_a, style_a = self.autoencoder_a.encode(images_a)
        content_b, style_b = self.autoencoder_b.encode(images_b)
        if image_recon:
            images_aa = self.autoencoder_a.decode(content_a, style_a)
            images_bb = self.autoencoder_b.decode(content_b, style_b)
            out.update(images_aa=images_aa, images_bb=images_bb)
        if random_style:
            style_a_rand = torch.randn_like(style_a)
            style_b_rand = torch.randn_like(style_b)
        else:
            style_a_rand, style_b_rand = style_a, style_b
        images_ba = self.autoencoder_a.decode(content_b, style_a_rand)
        images_ab = self.autoencoder_b.decode(content_a, style_b_rand)
        if latent_recon or cycle_recon:
            content_ba, style_ba = self.autoencoder_a.encode(images_ba)
            content_ab, style_ab = self.autoencoder_b.encode(images_ab)
            out.update(content_ba=content_ba, style_ba=style_ba, content_ab=content_ab,
                       style_ab=style_ab)
        if image_recon and within_latent_recon:
            content_aa, style_aa = self.autoencoder_a.encode(images_aa)
            content_bb, style_bb = self.autoencoder_b.encode(images_bb)
            out.update(content_aa=content_aa, style_aa=style_aa, content_bb=content_bb,
                       style_bb=style_bb)
        if cycle_recon:
            out.update(images_aba=self.autoencoder_a.decode(content_ab, style_a),
                       images_bab=self.autoencoder_b.decode(content_ba, style_b))
        out.update(content_a=content_a, content_b=content_b, style_a=style_a, style_b=style_b,
                   style_a_rand=style_a_rand, style_b_rand=style_b_rand, images_ba=images_ba,
                   images_ab=images_ab)
        return out

    def inference(self, data, a2b=True, random_style=True):
        if a2b:
            input_key, content_encode = 'images_a', self.autoencoder_a.content_encoder
            style_encode, decode = self.autoencoder_b.style_encoder, self.autoencoder_b.decode
        else:
            input_key, content_encode = 'images_b', self.autoencoder_b.content_encoder
            style_encode, decode = self.autoencoder_a.style_encoder, self.autoencoder_a.decode
        content = content_encode(data[input_key])
        if random_style:
            style = torch.randn(content.size(0), self.autoencoder_a.style_channels, 1, 1,
                                device=content.device)
            file_names = [_name(data, input_key)]
        else:
            style_key = 'images_b' if a2b else 'images_a'
            style = style_encode(data[style_key])
            file_names = [_name(data, input_key) + '_style_' + _name(data, style_key)]
        return decode(content, style), file_names


class AutoEncoder(nn.Module):
    def __init__(self, num_filters=64, max_num_filters=256, num_filters_mlp=256, latent_dim=8,
                 num_res_blocks=4, num_mlp_blocks=2, num_downsamples_style=4,
                 num_downsamples_content=2, num_image_channels=3, content_norm_type='instance',
                 style_norm_type='', decoder_norm_type='instance', weight_norm_type='',
                 decoder_norm_params=SimpleNamespace(affine=False), output_nonlinearity='',
                 pre_act=False, apply_noise=False, **kwargs):
        super().__init__()
        for key in kwargs:
            if key not in ('type', 'common'):
                warnings.warn("Generator argument '{}' is not used.".format(key))
        if isinstance(decoder_norm_params, dict):
            decoder_norm_params = SimpleNamespace(**decoder_norm_params)
        self.style_encoder = StyleEncoder(num_downsamples_style, num_image_channels, num_filters,
                                          latent_dim, 'reflect', style_norm_type,
                                          weight_norm_type, 'relu')
        self.content_encoder = ContentEncoder(num_downsamples_content, num_res_blocks,
                                              num_image_channels, num_filters, max_num_filters,
                                              'reflect', content_norm_type, weight_norm_type,
                                              'relu', pre_act)
        self.decoder = Decoder(num_downsamples_content, num_res_blocks,
                               self.content_encoder.output_dim, num_image_channels,
                               num_filters_mlp, 'reflect', decoder_norm_type,
                               decoder_norm_params, weight_norm_type, 'relu',
                               output_nonlinearity, pre_act, apply_noise)
        self.mlp = MLP(latent_dim, num_filters_mlp, num_filters_mlp, num_mlp_blocks, 'none',
                       'relu')
        self.style_channels = latent_dim

    def forward(self, images):
        content, style = self.encode(images)
        return self.decode(content, style)

    def encode(self, images):
        return self.content_encoder(images), self.style_encoder(images)

    def decode(self, content, style):
        return self.decoder(content, self.mlp(style))


class StyleEncoder(nn.Module):
    def __init__(self, num_downsamples, num_image_channels, num_filters, style_channels,
                 padding_mode, activation_norm_type, weight_norm_type, nonlinearity):
        super().__init__()
        conv_params = dict(padding_mode=padding_mode, activation_norm_type=activation_norm_type,
                           weight_norm_type=weight_norm_type, nonlinearity=nonlinearity,
                           inplace_nonlinearity=True)
        model = [Conv2dBlock(num_image_channels, num_filters, 7, 1, 3, **conv_params)]
        for _ in range(2):
            model += [Conv2dBlock(num_filters, 2 * num_filters, 4, 2, 1, **conv_params)]
            num_filters *= 2
        for _ in range(num_downsamples - 2):
            model += [Conv2dBlock(num_filters, num_filters, 4, 2, 1, **conv_params)]
        model += [nn.AdaptiveAvgPool2d(1)]
        model += [NHWCConv2d(num_filters, style_channels, 1, 1, 0)]
        self.model = nn.Sequential(*model)
        self.output_dim = num_filters

    def forward(self, x):
        return self.model(x)


class Decoder(nn.Module):
    def __init__(self, num_upsamples, num_res_blocks, num_filters, num_image_channels,
                 style_channels, padding_mode, activation_norm_type, activation_norm_params,
                 weight_norm_type, nonlinearity, output_nonlinearity, pre_act=False,
                 apply_noise=False):
        super().__init__()
        adain_params = SimpleNamespace(activation_norm_type=activation_norm_type,
                                       activation_norm_params=activation_norm_params,
                                       cond_dims=style_channels)
        conv_params = dict(padding_mode=padding_mode, nonlinearity=nonlinearity,
                           inplace_nonlinearity=True, apply_noise=apply_noise,
                           weight_norm_type=weight_norm_type, activation_norm_type='adaptive',
                           activation_norm_params=adain_params)
        order = 'pre_act' if pre_act else 'CNACNA'
        self.decoder = nn.ModuleList()
        for _ in range(num_res_blocks):
            self.decoder += [Res2dBlock(num_filters, num_filters, **conv_params, order=order)]
        for _ in range(num_upsamples):
            self.decoder += [NearestUpsample(scale_factor=2)]
            self.decoder += [Conv2dBlock(num_filters, num_filters // 2, 5, 1, 2, **conv_params)]
            num_filters //= 2
        self.decoder += [Conv2dBlock(num_filters, num_image_channels, 7, 1, 3,
                                     nonlinearity=output_nonlinearity,
                                     padding_mode=padding_mode)]

    def forward(self, x, style):
        for block in self.decoder:
            if getattr(block, 'conditional', False):
                x = block(x, style)
            else:
                x = block(x)
        return x


class MLP(nn.Module):
    def __init__(self, input_dim, output_dim, latent_dim, num_layers, norm, nonlinearity):
        super().__init__()
        model = [LinearBlock(input_dim, latent_dim, activation_norm_type=norm,
                             nonlinearity=nonlinearity)]
        for _ in range(num_layers - 2):
            model += [LinearBlock(latent_dim, latent_dim, activation_norm_type=norm,
                                  nonlinearity=nonlinearity)]
        model += [LinearBlock(latent_dim, output_dim, activation_norm_type=norm,
                              nonlinearity=nonlinearity)]
        self.model = nn.Sequential(*model)

    def forward(self, x):
        return self.model(x.reshape(x.size(0), -1))
