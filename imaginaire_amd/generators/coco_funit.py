"""COCO-FUNIT generator (reference generators/coco_funit.py:12-194): FUNIT
with a content-conditioned style code ``mlp(mlp_style([s, usb]) ⊙
mlp_content(mean(content)))`` and a learned universal style bias."""
import torch
from torch import nn

from imaginaire_amd.generators.funit import MLP, ContentEncoder, Decoder, StyleEncoder
from imaginaire_amd.generators.unit import _kw
from imaginaire_amd.generators.unit import _names


class Generator(nn.Module):
    def __init__(self, gen_cfg, data_cfg):
        super().__init__()
        self.generator = COCOFUNITTranslator(**_kw(gen_cfg))

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


class COCOFUNITTranslator(nn.Module):
    def __init__(self, num_filters=64, num_filters_mlp=256, style_dims=64, usb_dims=1024,
                 num_res_blocks=2, num_mlp_blocks=3, num_downsamples_style=4,
                 num_downsamples_content=2, num_image_channels=3, weight_norm_type='', **kwargs):
        super().__init__()
        self.style_encoder = StyleEncoder(num_downsamples_style, num_image_channels, num_filters,
                                          style_dims, 'reflect', 'none', weight_norm_type, 'relu')
        self.content_encoder = ContentEncoder(num_downsamples_content, num_res_blocks,
                                              num_image_channels, num_filters, 'reflect',
                                              'instance', weight_norm_type, 'relu')
        self.decoder = Decoder(self.content_encoder.output_dim, num_filters_mlp,
                               num_image_channels, num_downsamples_content, 'reflect',
                               weight_norm_type, 'relu')
        self.usb = torch.nn.Parameter(torch.randn(1, usb_dims))
        self.mlp = MLP(style_dims, num_filters_mlp, num_filters_mlp, num_mlp_blocks, 'none',
                       'relu')
        self.mlp_content = MLP(self.content_encoder.output_dim, style_dims, num_filters_mlp, 2,
                               'none', 'relu')
        self.mlp_style = MLP(style_dims + usb_dims, style_dims, num_filters_mlp, 2, 'none',
                             'relu')

    def forward(self, images):
        content, style = self.encode(images)
        return self.decode(content, style)

    def encode(self, images):
        return self.content_encoder(images), self.style_encoder(images)

    def decode(self, content, style):
        content_style_code = self.mlp_content(content.mean(3).mean(2))
        batch_size = style.size(0)
        usb = self.usb.repeat(batch_size, 1).to(style.dtype)
        style_in = self.mlp_style(torch.cat([style.reshape(batch_size, -1), usb], 1))
        coco_style = self.mlp(style_in * content_style_code)
        return self.decoder(content, coco_style)
