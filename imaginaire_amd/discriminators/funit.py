"""FUNIT projection discriminator (reference discriminators/funit.py:13-117)."""
import warnings

import torch
from torch import nn

from imaginaire_amd.layers import Conv2dBlock, Res2dBlock
from imaginaire_amd.ops.pool import AvgPool2d, ReflectionPad2d
from imaginaire_amd.discriminators.munit import _kw


class Discriminator(nn.Module):
    def __init__(self, dis_cfg, data_cfg):
        super().__init__()
        self.model = ResDiscriminator(**_kw(dis_cfg))

    def forward(self, data, net_G_output, recon=True):
        source_labels = data['labels_content']
        target_labels = data['labels_style']
        fake_out_trans, fake_features_trans = self.model(net_G_output['images_trans'],
                                                         target_labels)
        output = dict(fake_out_trans=fake_out_trans, fake_features_trans=fake_features_trans)
        real_out_style, real_features_style = self.model(data['images_style'], target_labels)
        output.update(dict(real_out_style=real_out_style,
                           real_features_style=real_features_style))
        if recon:
            fake_out_recon, fake_features_recon = self.model(net_G_output['images_recon'],
                                                             source_labels)
            output.update(dict(fake_out_recon=fake_out_recon,
                               fake_features_recon=fake_features_recon))
        return output


class ResDiscriminator(nn.Module):
    def __init__(self, image_channels=3, num_classes=119, num_filters=64, max_num_filters=1024,
                 num_layers=6, padding_mode='reflect', weight_norm_type='', **kwargs):
        super().__init__()
        for key in kwargs:
            if key != 'type':
                warnings.warn("Discriminator argument {} is not used".format(key))
        conv_params = dict(padding_mode=padding_mode, activation_norm_type='none',
                           weight_norm_type=weight_norm_type, bias=[True, True, True],
                           nonlinearity='leakyrelu', order='NACNAC')
        model = [Conv2dBlock(image_channels, num_filters, 7, 1, 3, padding_mode=padding_mode,
                             weight_norm_type=weight_norm_type)]
        for i in range(num_layers):
            num_filters_prev = num_filters
            num_filters = min(num_filters * 2, max_num_filters)
            model += [Res2dBlock(num_filters_prev, num_filters_prev, **conv_params),
                      Res2dBlock(num_filters_prev, num_filters, **conv_params)]
            if i != num_layers - 1:
                model += [ReflectionPad2d(1), AvgPool2d(3, stride=2)]
        self.model = nn.Sequential(*model)
        self.classifier = Conv2dBlock(num_filters, 1, 1, 1, 0, nonlinearity='leakyrelu',
                                      weight_norm_type=weight_norm_type, order='NACNAC')
        self.embedder = nn.Embedding(num_classes, num_filters)

    def forward(self, images, labels=None):
        features = self.model(images)
        outputs = self.classifier(features)
        features_1x1 = features.mean(3).mean(2)
        if labels is None:
            return features_1x1
        assert images.size(0) == labels.size(0)
        embeddings = self.embedder(labels.long().reshape(-1))
        outputs = outputs + torch.sum(embeddings * features_1x1, dim=1, keepdim=True).reshape(
            images.size(0), 1, 1, 1).to(outputs.dtype)
        return outputs, features_1x1
