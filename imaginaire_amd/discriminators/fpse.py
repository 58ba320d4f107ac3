"""Feature-Pyramid Semantics-Embedding discriminator (reference discriminators/fpse.py:15-132)."""
import functools

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from imaginaire_amd.layers import Conv2dBlock
from imaginaire_amd.ops.pool import avg_pool2d
from imaginaire_amd.ops.resize import Upsample, upsample_add


class FPSEDiscriminator(nn.Module):
    def __init__(self, num_input_channels, num_labels, num_filters, kernel_size,
                 weight_norm_type, activation_norm_type):
        super().__init__()
        padding = int(np.ceil((kernel_size - 1.0) / 2))
        nl = 'leakyrelu'
        stride1 = functools.partial(Conv2dBlock, kernel_size=kernel_size, stride=1,
                                    padding=padding, weight_norm_type=weight_norm_type,
                                    activation_norm_type=activation_norm_type, nonlinearity=nl,
                                    order='CNA')
        down = functools.partial(Conv2dBlock, kernel_size=kernel_size, stride=2,
                                 padding=padding, weight_norm_type=weight_norm_type,
                                 activation_norm_type=activation_norm_type, nonlinearity=nl,
                                 order='CNA')
        latent = functools.partial(Conv2dBlock, kernel_size=1, stride=1,
                                   weight_norm_type=weight_norm_type,
                                   activation_norm_type=activation_norm_type, nonlinearity=nl,
                                   order='CNA')
        self.enc1 = down(num_input_channels, num_filters)
        self.enc2 = down(1 * num_filters, 2 * num_filters)
        self.enc3 = down(2 * num_filters, 4 * num_filters)
        self.enc4 = down(4 * num_filters, 8 * num_filters)
        self.enc5 = down(8 * num_filters, 8 * num_filters)
        self.lat2 = latent(2 * num_filters, 4 * num_filters)
        self.lat3 = latent(4 * num_filters, 4 * num_filters)
        self.lat4 = latent(8 * num_filters, 4 * num_filters)
        self.lat5 = latent(8 * num_filters, 4 * num_filters)
        self.upsample2x = Upsample(scale_factor=2, mode='bilinear', align_corners=False)
        self.final2 = stride1(4 * num_filters, 2 * num_filters)
        self.final3 = stride1(4 * num_filters, 2 * num_filters)
        self.final4 = stride1(4 * num_filters, 2 * num_filters)
        self.output = Conv2dBlock(num_filters * 2, 1, kernel_size=1)
        self.seg = Conv2dBlock(num_filters * 2, num_filters * 2, kernel_size=1)
        self.embedding = Conv2dBlock(num_labels, num_filters * 2, kernel_size=1)

    def _embedding_is_linear(self):
        layers = self.embedding.layers
        return list(layers.keys()) == ['conv'] and type(layers['conv']) is nn.Conv2d and \
            layers['conv'].kernel_size == (1, 1) and layers['conv'].stride == (1, 1)

    def forward(self, images, segmaps, seg_repeat=1):
        """``seg_repeat``: ``images`` holds that many stacked copies of the batch of
        ``segmaps`` (real and fake halves of a batched D pass): the label embedding is computed
        once and repeated at the (small) prediction resolutions."""
        feat11 = self.enc1(images)
        feat12 = self.enc2(feat11)
        feat13 = self.enc3(feat12)
        feat14 = self.enc4(feat13)
        feat15 = self.enc5(feat14)
        feat25 = self.lat5(feat15)
        # bilinear 2x up + lateral in one k12 pass (ops/resize.upsample_add)
        feat24 = upsample_add(feat25, self.lat4(feat14))
        feat23 = upsample_add(feat24, self.lat3(feat13))
        feat22 = upsample_add(feat23, self.lat2(feat12))
        feat32 = self.final2(feat22)
        feat33 = self.final3(feat23)
        feat34 = self.final4(feat24)
        pred2 = self.output(feat32)
        pred3 = self.output(feat33)
        pred4 = self.output(feat34)
        seg2 = self.seg(feat32)
        seg3 = self.seg(feat33)
        seg4 = self.seg(feat34)
        # avg_pool(conv1x1(s)) == conv1x1(avg_pool(s)) for the linear, bias-only embedding
        # block: pool the label map first so the 1x1 conv (and its weight gradient) runs at
        # half resolution and the full-resolution 2F-channel embedding is never materialised
        if self._embedding_is_linear():
            segembs = self.embedding(avg_pool2d(segmaps, kernel_size=2, stride=2))
        else:
            segembs = avg_pool2d(self.embedding(segmaps), kernel_size=2, stride=2)
        segembs2 = avg_pool2d(segembs, kernel_size=2, stride=2)
        segembs3 = avg_pool2d(segembs2, kernel_size=2, stride=2)
        segembs4 = avg_pool2d(segembs3, kernel_size=2, stride=2)
        if seg_repeat > 1:
            segembs2, segembs3, segembs4 = (e.repeat(seg_repeat, 1, 1, 1)
                                            for e in (segembs2, segembs3, segembs4))
        pred2 = pred2 + torch.mul(segembs2, seg2).sum(dim=1, keepdim=True)
        pred3 = pred3 + torch.mul(segembs3, seg3).sum(dim=1, keepdim=True)
        pred4 = pred4 + torch.mul(segembs4, seg4).sum(dim=1, keepdim=True)
        return pred2, pred3, pred4
