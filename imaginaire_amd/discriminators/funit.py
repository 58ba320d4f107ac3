"""FUNIT projection discriminator (reference discriminators/funit.py:13-117).

The reference runs the ResDiscriminator once per image set: translation, style (real) and
reconstruction. Sets that go through the same backward are concatenated along the batch axis
and run as ONE pass instead (no batch-coupled layers: activation_norm_type is 'none'): in the
D update translation + style (both feed the D weight gradients), in the G update translation
+ reconstruction (gradient through both fakes), with the style set, which the G update only
reads for feature matching, in its own pass. One weight cast and one weight gradient per conv
instead of two or three, and two or three times the rows per GEMM at the 8x8..32x32 layers.
Spectral norm: the reference iterates each layer once per pass; the skipped passes' power
iterations run back to back first (``extra_sn_power_iteration``), so u / v advance exactly as
in the reference and only the σ that each set is normalised by shifts by one iteration (as in
discriminators/spade.py). ``dis.batch_real_fake: False`` restores the reference passes.
"""
import os
import warnings

import torch
from torch import nn

from imaginaire_amd.layers import Conv2dBlock, Res2dBlock
from imaginaire_amd.layers.spectral_norm import extra_sn_power_iteration
from imaginaire_amd.ops.pool import AvgPool2d, ReflectionPad2d
from imaginaire_amd.discriminators.munit import _kw


class Discriminator(nn.Module):
    def __init__(self, dis_cfg, data_cfg):
        super().__init__()
        kw = _kw(dis_cfg)
        # (IMAGINAIRE_AMD_DIS_BATCH=0: A/B switch to the reference passes)
        self.batched = bool(kw.pop('batch_real_fake', True)) and \
            os.environ.get('IMAGINAIRE_AMD_DIS_BATCH', '1') != '0'
        self.model = ResDiscriminator(**kw)

    def _passes(self, sets):
        """ResDiscriminator outputs of each (images, labels) set, the sets run as one
        batch-concatenated pass."""
        n = [im.shape[0] for im, _ in sets]
        for _ in range(len(sets) - 1):  # one per pass saved: see the module docstring
            extra_sn_power_iteration(self)
        dt = sets[0][0].dtype
        out, feat = self.model(torch.cat([im.to(dt) for im, _ in sets], 0),
                               torch.cat([lb for _, lb in sets], 0))
        return list(zip(out.split(n, 0), feat.split(n, 0)))

    def forward(self, data, net_G_output, recon=True):
        source_labels = data['labels_content']
        target_labels = data['labels_style']
        trans, style = net_G_output['images_trans'], data['images_style']
        rec = net_G_output['images_recon'] if recon else None
        same = trans.shape == style.shape and (rec is None or rec.shape == trans.shape)
        if self.batched and same:
            grad_fake = torch.is_grad_enabled() and trans.requires_grad
            if recon and grad_fake:  # G update: the two fakes together, the style set alone
                (fo_t, ff_t), (fo_r, ff_r) = self._passes(
                    [(trans, target_labels), (rec, source_labels)])
                ro_s, rf_s = self.model(style, target_labels)
            elif recon:
                (fo_t, ff_t), (ro_s, rf_s), (fo_r, ff_r) = self._passes(
                    [(trans, target_labels), (style, target_labels), (rec, source_labels)])
            else:  # D update: translation and style together
                (fo_t, ff_t), (ro_s, rf_s) = self._passes(
                    [(trans, target_labels), (style, target_labels)])
            output = dict(fake_out_trans=fo_t, fake_features_trans=ff_t, real_out_style=ro_s,
                          real_features_style=rf_s)
            if recon:
                output.update(dict(fake_out_recon=fo_r, fake_features_recon=ff_r))
            return output
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
