"""FUNIT generator (reference generators/funit.py:15-398): content encoder
(instance norm), style encoder, AdaIN decoder of Res2dBlocks + UpRes2dBlocks
whose adaptive norms are fused HIP kernels, style MLP."""
from functools import partial
from types import SimpleNamespace

import torch
from torch import nn

from imaginaire_amd.generators.unit import _kw
from imaginaire_amd.layers.conv import NHWCConv2d
from imaginaire_amd.layers import Conv2dBlock, LinearBlock, Res2dBlock, UpRes2dBlock
from imaginaire_amd.generators.unit import _names


class Generator(nn.Module):
    def __init__(self, gen_cfg, data_cfg):
        super().__init__()
        self.generator = FUNITTranslator(**_kw(gen_cfg))

    def forward(self, data):
        content_a = self.generator.content_encoder(data['images_content'])
        style_a = self.generator.style_encoder(data['images_content'])
        style_b = self.generator.style_encoder(data['images_style'])
        return dict(images_trans=self.generator.decode(content_a, style_b),
                    images_recon=self.generator.decode(content_a, style_a))

    def inference(self, data, keep_original_size=True):
        content_a = self.generator.content_encoder(data['images_content'])
        style_b = self.generator.style_encoder(data['images_style'])
        output_images = self.generator.decode(content_a, style_b)
        if keep_original_size:
            height, width = int(data['original_h_w'][0][0]), int(data['original_h_w'][0][1])
            output_images = torch.nn.functional.interpolate(output_images, size=[height, width])
        file_names = _names(data, 'images_content')
        return output_images, file_names


class FUNITTranslator(nn.Module):
    def __init__(self, num_filters=64, num_filters_mlp=256, style_dims=64, num_res_blocks=2,
                 num_mlp_blocks=3, num_downsamples_style=4, num_downsamples_content=2,
                 num_image_channels=3, weight_norm_type='', **kwargs):
        super().__init__()
        self.style_encoder = StyleEncoder(num_downsamples_style, num_image_channels, num_filters,
                                          style_dims, 'reflect', 'none', weight_norm_type, 'relu')
        self.content_encoder = ContentEncoder(num_downsamples_content, num_res_blocks,
                                              num_image_channels, num_filters, 'reflect',
                                              'instance', weight_norm_type, 'relu')
        self.decoder = Decoder(self.content_encoder.output_dim, num_filters_mlp,
                               num_image_channels, num_downsamples_content, 'reflect',
                               weight_norm_type, 'relu')
        self.mlp = MLP(style_dims, num_filters_mlp, num_filters_mlp, num_mlp_blocks, 'none',
                       'relu')

    def forward(self, images):
        content, style = self.encode(images)
        return self.decode(content, style)

    def encode(self, images):
        return self.content_encoder(images), self.style_encoder(images)

    def decode(self, content, style):
        return self.decoder(content, self.mlp(style))


class Decoder(nn.Module):
    def __init__(self, num_enc_output_channels, style_channels, num_image_channels=3,
                 num_upsamples=4, padding_type='reflect', weight_norm_type='none',
                 nonlinearity='relu'):
        super().__init__()
        adain_params = SimpleNamespace(activation_norm_type='instance',
                                       activation_norm_params=SimpleNamespace(affine=False),
                                       cond_dims=style_channels)
        base_res_block = partial(Res2dBlock, kernel_size=3, padding=1, padding_mode=padding_type,
                                 nonlinearity=nonlinearity, activation_norm_type='adaptive',
                                 activation_norm_params=adain_params,
                                 weight_norm_type=weight_norm_type)
        base_up_res_block = partial(UpRes2dBlock, kernel_size=5, padding=2,
                                    padding_mode=padding_type, weight_norm_type=weight_norm_type,
                                    activation_norm_type='adaptive',
                                    activation_norm_params=adain_params,
                                    skip_activation_norm='instance',
                                    skip_nonlinearity=nonlinearity, nonlinearity=nonlinearity,
                                    hidden_channels_equal_out_channels=True)
        dims = num_enc_output_channels
        self.decoder = nn.ModuleList()
        self.decoder += [base_res_block(dims, dims)]
        self.decoder += [base_res_block(dims, dims)]
        for _ in range(num_upsamples):
            self.decoder += [base_up_res_block(dims, dims // 2)]
            dims = dims // 2
        self.decoder += [Conv2dBlock(dims, num_image_channels, kernel_size=7, stride=1,
                                     padding=3, padding_mode='reflect', nonlinearity='tanh')]

    def forward(self, x, style):
        for block in self.decoder:
            x = block(x, style) if getattr(block, 'conditional', False) else block(x)
        return x


class StyleEncoder(nn.Module):
    def __init__(self, num_downsamples, image_channels, num_filters, style_channels,
                 padding_mode, activation_norm_type, weight_norm_type, nonlinearity):
        super().__init__()
        conv_params = dict(padding_mode=padding_mode, activation_norm_type=activation_norm_type,
                           weight_norm_type=weight_norm_type, nonlinearity=nonlinearity,
                           inplace_nonlinearity=True)
        model = [Conv2dBlock(image_channels, num_filters, 7, 1, 3, **conv_params)]
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


class ContentEncoder(nn.Module):
    def __init__(self, num_downsamples, num_res_blocks, image_channels, num_filters,
                 padding_mode, activation_norm_type, weight_norm_type, nonlinearity):
        super().__init__()
        conv_params = dict(padding_mode=padding_mode, activation_norm_type=activation_norm_type,
                           weight_norm_type=weight_norm_type, nonlinearity=nonlinearity,
                           inplace_nonlinearity=True, order='CNACNA')
        model = [Conv2dBlock(image_channels, num_filters, 7, 1, 3, **conv_params)]
        dims = num_filters
        for _ in range(num_downsamples):
            model += [Conv2dBlock(dims, dims * 2, 4, 2, 1, **conv_params)]
            dims *= 2
        for _ in range(num_res_blocks):
            model += [Res2dBlock(dims, dims, **conv_params)]
        self.model = nn.Sequential(*model)
        self.output_dim = dims

    def forward(self, x):
        return self.model(x)


class MLP(nn.Module):
    def __init__(self, input_dim, output_dim, latent_dim, num_layers, activation_norm_type,
                 nonlinearity):
        super().__init__()
        model = [LinearBlock(input_dim, latent_dim, activation_norm_type=activation_norm_type,
                             nonlinearity=nonlinearity)]
        for _ in range(num_layers - 3):
            model += [LinearBlock(latent_dim, latent_dim,
                                  activation_norm_type=activation_norm_type,
                                  nonlinearity=nonlinearity)]
        model += [LinearBlock(latent_dim, output_dim, activation_norm_type=activation_norm_type,
                              nonlinearity=nonlinearity)]
        self.model = nn.Sequential(*model)

    def forward(self, x):
        return self.model(x.reshape(x.size(0), -1))
