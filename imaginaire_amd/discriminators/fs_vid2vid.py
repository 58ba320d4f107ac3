"""(fs-)vid2vid discriminator (reference discriminators/fs_vid2vid.py:18-318).

Per-frame multi-scale patch D on [label (+ref label/image), image], an
optional raw-output branch, optional region discriminators (face / hand
crops, ``crop_func``) and ``num_scales`` temporal discriminators over frame
windows sub-sampled at strides tD**s.

MI355X change: real and fake go through each patch D as ONE batched forward
(concatenated along the batch axis) when the D has no batch-statistics
normalisation — half the kernel launches and twice the per-launch work. The
spectral-norm power iteration then runs once per call instead of twice
(same convention as discriminators/spade.py here).
"""
import importlib

import torch
import torch.nn.functional as F
from torch import nn

from imaginaire_amd.discriminators.multires_patch import NLayerPatchDiscriminator
from imaginaire_amd.model_utils.fs_vid2vid import get_fg_mask, pick_image
from imaginaire_amd.utils.data import (get_paired_input_image_channel_number,
                                       get_paired_input_label_channel_number)
from imaginaire_amd.utils.misc import get_nested_attr
from imaginaire_amd.ops.conv import stack_nhwc
from imaginaire_amd.ops.resize import interpolate


class Discriminator(nn.Module):
    def __init__(self, dis_cfg, data_cfg):
        super().__init__()
        self.data_cfg = data_cfg
        num_input_channels = get_paired_input_label_channel_number(data_cfg)
        if num_input_channels == 0:
            num_input_channels = getattr(data_cfg, 'label_channels', 1)
        num_img_channels = get_paired_input_image_channel_number(data_cfg)
        self.num_frames_D = data_cfg.num_frames_D
        self.num_scales = get_nested_attr(dis_cfg, 'temporal.num_scales', 0)
        num_netD_input_channels = num_input_channels + num_img_channels
        self.use_few_shot = 'few_shot' in data_cfg.type
        if self.use_few_shot:
            num_netD_input_channels *= 2
        self.net_D = MultiPatchDiscriminator(dis_cfg.image, num_netD_input_channels)
        self.add_dis_cfg = getattr(dis_cfg, 'additional_discriminators', None)
        if self.add_dis_cfg is not None:
            for name in self.add_dis_cfg:
                num_ch = num_img_channels * (2 if self.use_few_shot else 1)
                setattr(self, 'net_D_' + name,
                        MultiPatchDiscriminator(self.add_dis_cfg[name], num_ch))
        self.num_netDT_input_channels = num_img_channels * self.num_frames_D
        for n in range(self.num_scales):
            setattr(self, 'net_DT%d' % n,
                    MultiPatchDiscriminator(dis_cfg.temporal, self.num_netDT_input_channels))
        self.has_fg = getattr(data_cfg, 'has_foreground', False)

    def forward(self, data, net_G_output, past_frames):
        label, real_image = data['label'], data['image']
        if label.dim() == 5:
            label = label[:, -1]
        if self.use_few_shot:
            ref_idx = net_G_output.get('ref_idx', 0)
            ref_label = pick_image(data['ref_labels'], ref_idx)
            ref_image = pick_image(data['ref_images'], ref_idx)
            label = torch.cat([label, ref_label, ref_image], dim=1)
        fake_image = net_G_output['fake_images']
        output = dict()
        pred_real, pred_fake = self.discrminate_image(self.net_D, label, real_image, fake_image)
        output['indv'] = dict(pred_real=pred_real, pred_fake=pred_fake)
        if net_G_output.get('fake_raw_images') is not None:
            fg_mask = get_fg_mask(data['label'], self.has_fg)
            pred_real, pred_fake = self.discrminate_image(
                self.net_D, label, real_image * fg_mask,
                net_G_output['fake_raw_images'] * fg_mask)
            output['raw'] = dict(pred_real=pred_real, pred_fake=pred_fake)
        if self.add_dis_cfg is not None:
            for name in self.add_dis_cfg:
                mod, fn = self.add_dis_cfg[name].crop_func.split('::')
                crop_func = getattr(importlib.import_module(
                    mod.replace('imaginaire.', 'imaginaire_amd.', 1)), fn)
                real_crop = crop_func(self.data_cfg, real_image, label)
                fake_crop = crop_func(self.data_cfg, fake_image, label)
                if self.use_few_shot:
                    ref_crop = crop_func(self.data_cfg, ref_image, label)
                    if ref_crop is not None:
                        real_crop = torch.cat([real_crop, ref_crop], dim=1)
                        fake_crop = torch.cat([fake_crop, ref_crop], dim=1)
                if fake_crop is not None:
                    pred_real, pred_fake = self.discrminate_image(
                        getattr(self, 'net_D_' + name), None, real_crop, fake_crop)
                else:
                    pred_real = pred_fake = None
                output[name] = dict(pred_real=pred_real, pred_fake=pred_fake)
        past_frames, skipped_frames = get_all_skipped_frames(
            past_frames, [real_image, fake_image], self.num_scales, self.num_frames_D)
        for scale in range(self.num_scales):
            real_s, fake_s = [f[scale] for f in skipped_frames]
            pred_real, pred_fake = self.discriminate_video(real_s, fake_s, scale)
            output['temporal_%d' % scale] = dict(pred_real=pred_real, pred_fake=pred_fake)
        return output, past_frames

    def discrminate_image(self, net_D, real_A, real_B, fake_B):
        if real_A is not None and net_D.batchable and real_B.is_cuda and real_B.dim() == 4:
            # label|real and label|fake written once into one channel-padded NHWC buffer
            both = stack_nhwc([[real_A, real_B], [real_A, fake_B]])
            return net_D.forward_stacked(both, real_B.shape[0])
        if real_A is not None:
            real_AB = torch.cat([real_A, real_B], dim=1)
            fake_AB = torch.cat([real_A, fake_B.to(real_A.dtype)], dim=1)
        else:
            real_AB, fake_AB = real_B, fake_B
        return net_D.forward_pair(real_AB, fake_AB)

    def discriminate_video(self, real_B, fake_B, scale):
        if real_B is None:
            return None, None
        net_DT = getattr(self, 'net_DT%d' % scale)
        h, w = real_B.shape[-2:]
        real_B = real_B.reshape(-1, self.num_netDT_input_channels, h, w)
        fake_B = fake_B.reshape(-1, self.num_netDT_input_channels, h, w)
        return net_DT.forward_pair(real_B, fake_B)


def get_all_skipped_frames(past_frames, new_frames, t_scales, tD):
    new_past, skipped = [], []
    for past, new in zip(past_frames, new_frames):
        sk = None
        if t_scales > 0:
            past, sk = get_skipped_frames(past, new.unsqueeze(1), t_scales, tD)
        new_past.append(past)
        skipped.append(sk)
    return new_past, skipped


def get_skipped_frames(all_frames, frame, t_scales, tD):
    """Append ``frame`` to the history and cut windows of tD frames at strides
    tD**s (fs_vid2vid.py:225-256)."""
    all_frames = torch.cat([all_frames.detach(), frame], dim=1) if all_frames is not None \
        else frame
    skipped = [None] * t_scales
    for s in range(t_scales):
        t_step = tD ** s
        t_span = t_step * (tD - 1)
        if all_frames.size(1) > t_span:
            skipped[s] = all_frames[:, -(t_span + 1)::t_step].contiguous()
    max_prev = (tD ** (t_scales - 1)) * (tD - 1)
    if all_frames.size(1) > max_prev:
        all_frames = all_frames[:, -max_prev:]
    return all_frames, skipped


class MultiPatchDiscriminator(nn.Module):
    """``num_discriminators`` patch Ds on successively 2x-downsampled input
    (fs_vid2vid.py:259-318)."""

    def __init__(self, dis_cfg, num_input_channels):
        super().__init__()
        kernel_size = getattr(dis_cfg, 'kernel_size', 4)
        num_filters = getattr(dis_cfg, 'num_filters', 64)
        max_num_filters = getattr(dis_cfg, 'max_num_filters', 512)
        num_discriminators = getattr(dis_cfg, 'num_discriminators', 3)
        num_layers = getattr(dis_cfg, 'num_layers', 3)
        activation_norm_type = getattr(dis_cfg, 'activation_norm_type', 'none')
        weight_norm_type = getattr(dis_cfg, 'weight_norm_type', 'spectral_norm')
        self.batchable = activation_norm_type in ('none', 'instance')
        for i in range(num_discriminators):
            self.add_module('discriminator_%d' % i, NLayerPatchDiscriminator(
                kernel_size, num_input_channels, num_filters, num_layers, max_num_filters,
                activation_norm_type, weight_norm_type))

    def forward(self, input_x):
        outputs, features = [], []
        x = input_x
        for name, net in self.named_children():
            if not name.startswith('discriminator_'):
                continue
            out, feat = net(x)
            outputs.append(out)
            features.append(feat)
            x = interpolate(x, scale_factor=0.5, mode='bilinear', align_corners=True,
                              recompute_scale_factor=True)
        return dict(output=outputs, features=features)

    def forward_pair(self, real, fake):
        """(D(real), D(fake)) — one batched pass when the D has no batch stats."""
        if not self.batchable:
            return self.forward(real), self.forward(fake)
        return self.forward_stacked(torch.cat([real, fake.to(real.dtype)], 0), real.shape[0])

    def forward_stacked(self, inputs, n):
        """(D(real), D(fake)) of real / fake stacked along the batch (first ``n`` = real)."""
        both = self.forward(inputs)

        def split(o, part):
            return [t[:n] if part == 0 else t[n:] for t in o]
        pr = dict(output=split(both['output'], 0),
                  features=[split(f, 0) for f in both['features']])
        pf = dict(output=split(both['output'], 1),
                  features=[split(f, 1) for f in both['features']])
        return pr, pf
