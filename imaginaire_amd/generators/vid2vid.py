"""vid2vid generator (reference generators/vid2vid.py:21-481).

First frame: a SPADE decoder from a constant code (or the segmentation map)
through ``up_{num_layers..0}``. Later frames: the previous output is encoded
by ``down_*`` / ``res_*`` SPADE blocks, a flow network predicts flow + an
occlusion mask from the previous labels/images, and the warped previous frame
is fed to the last ``num_multi_spade_layers`` SPADE layers as an extra
condition (multi-SPADE combine) — same module tree / state-dict names as the
reference.

Fork delta: the fork comments out the learned temporal
flow network (vid2vid.py:338), which makes temporal training crash for plain
vid2vid. Here ``flow_network_temp`` is built as upstream does; wc-vid2vid
(which takes flow from the data) disables it via ``_use_learned_flow``.
"""
from functools import partial

import numpy as np
import torch
import torch.nn.functional as F
from torch import nn

from imaginaire_amd.generators.fs_vid2vid import LabelEmbedder
from imaginaire_amd.ops.pool import AvgPool2d
from imaginaire_amd.layers import Conv2dBlock, LinearBlock, Res2dBlock
from imaginaire_amd.model_utils.fs_vid2vid import extract_valid_pose_labels, resample
from imaginaire_amd.utils.data import (get_paired_input_image_channel_number,
                                       get_paired_input_label_channel_number)
from imaginaire_amd.utils.init_weight import weights_init
from imaginaire_amd.ops.resize import interpolate, Upsample


class BaseNetwork(nn.Module):
    def get_num_filters(self, num_downsamples):
        return min(self.max_num_filters, self.num_filters * (2 ** num_downsamples))


class Generator(BaseNetwork):
    _use_learned_flow = True

    def __init__(self, gen_cfg, data_cfg):
        super().__init__()
        self.gen_cfg = gen_cfg
        self.data_cfg = data_cfg
        self.num_frames_G = data_cfg.num_frames_G
        self.num_layers = num_layers = getattr(gen_cfg, 'num_layers', 7)
        self.num_downsamples_img = getattr(gen_cfg, 'num_downsamples_img', 4)
        self.num_filters = num_filters = getattr(gen_cfg, 'num_filters', 32)
        self.max_num_filters = getattr(gen_cfg, 'max_num_filters', 1024)
        self.kernel_size = kernel_size = getattr(gen_cfg, 'kernel_size', 3)
        padding = kernel_size // 2
        self.is_pose_data = hasattr(data_cfg, 'for_pose_dataset')
        if self.is_pose_data:
            pose_cfg = data_cfg.for_pose_dataset
            self.pose_type = getattr(pose_cfg, 'pose_type', 'both')
            self.remove_face_labels = getattr(pose_cfg, 'remove_face_labels', False)
        self.num_input_channels = num_input_channels = \
            get_paired_input_label_channel_number(data_cfg)
        num_img_channels = get_paired_input_image_channel_number(data_cfg)
        aug_cfg = data_cfg.val.augmentations
        if hasattr(aug_cfg, 'center_crop_h_w'):
            crop_h_w = aug_cfg.center_crop_h_w
        elif hasattr(aug_cfg, 'resize_h_w'):
            crop_h_w = aug_cfg.resize_h_w
        else:
            raise ValueError('Need to specify output size.')
        crop_h, crop_w = [int(v) for v in str(crop_h_w).split(',')]
        self.sh = crop_h // (2 ** num_layers)
        self.sw = crop_w // (2 ** num_layers)
        self.z_dim = getattr(gen_cfg, 'style_dims', 256)
        self.use_segmap_as_input = getattr(gen_cfg, 'use_segmap_as_input', False)

        self.emb_cfg = emb_cfg = getattr(gen_cfg, 'embed', None)
        self.use_embed = getattr(emb_cfg, 'use_embed', 'True')
        self.num_downsamples_embed = getattr(emb_cfg, 'num_downsamples', 5)
        if self.use_embed:
            self.label_embedding = LabelEmbedder(emb_cfg, num_input_channels)

        self.flow_cfg = flow_cfg = gen_cfg.flow
        self.spade_combine = getattr(flow_cfg, 'multi_spade_combine', True)
        self.num_multi_spade_layers = getattr(flow_cfg.multi_spade_combine, 'num_layers', 3)
        self.temporal_initialized = False
        self.generate_raw_output = False

        weight_norm_type = getattr(gen_cfg, 'weight_norm_type', 'spectral')
        activation_norm_type = gen_cfg.activation_norm_type
        activation_norm_params = gen_cfg.activation_norm_params
        if self.use_embed and not hasattr(activation_norm_params, 'num_filters'):
            activation_norm_params.num_filters = 0
        nonlinearity = 'leakyrelu'
        self.base_res_block = base_res_block = partial(
            Res2dBlock, kernel_size=kernel_size, padding=padding,
            weight_norm_type=weight_norm_type, activation_norm_type=activation_norm_type,
            activation_norm_params=activation_norm_params, nonlinearity=nonlinearity,
            order='NACNAC')
        for i in range(num_layers, -1, -1):
            activation_norm_params.cond_dims = self.get_cond_dims(i)
            activation_norm_params.partial = self.get_partial(i) \
                if hasattr(self, 'get_partial') else False
            setattr(self, 'up_%d' % i, base_res_block(self.get_num_filters(i + 1),
                                                       self.get_num_filters(i)))
        self.conv_img = Conv2dBlock(num_filters, num_img_channels, kernel_size,
                                    padding=padding, nonlinearity=nonlinearity, order='AC')
        top = min(self.max_num_filters, num_filters * (2 ** (self.num_layers + 1)))
        if self.use_segmap_as_input:
            self.fc = Conv2dBlock(num_input_channels, top, kernel_size=3, padding=1)
        else:
            self.fc = LinearBlock(self.z_dim, top * self.sh * self.sw)
        self.downsample = AvgPool2d(kernel_size=3, stride=2, padding=1)
        self.upsample = partial(interpolate, scale_factor=2)
        self.init_temporal_network()

    # ------------------------------------------------------------------ forward
    def _first_frame_code(self, label, z, bs, cond_maps_now):
        if self.use_segmap_as_input:
            x = self.fc(interpolate(label, size=(self.sh, self.sw)))
        else:
            if z is None:
                z = torch.zeros(bs, self.z_dim, dtype=label.dtype, device=label.device)
            x = self.fc(z).view(bs, -1, self.sh, self.sw)
        for i in range(self.num_layers, self.num_downsamples_img, -1):
            j = min(self.num_downsamples_embed, i)
            x = self.upsample(getattr(self, 'up_%d' % i)(x, *cond_maps_now[j]))
        return x

    def _encode_prev(self, img_prev, label_prev, cond_maps_now):
        x = self.down_first(img_prev[:, -1])
        cond_maps_prev = self.get_cond_maps(label_prev[:, -1], self.label_embedding)
        for i in range(self.num_downsamples_img + 1):
            j = min(self.num_downsamples_embed, i)
            x = getattr(self, 'down_%d' % i)(x, *cond_maps_prev[j])
            if i != self.num_downsamples_img:
                x = self.downsample(x)
        j = min(self.num_downsamples_embed, self.num_downsamples_img + 1)
        for i in range(self.num_res_blocks):
            cond = cond_maps_prev[j] if i < self.num_res_blocks // 2 else cond_maps_now[j]
            x = getattr(self, 'res_%d' % i)(x, *cond)
        return x

    def forward(self, data):
        label = data['label']
        label_prev, img_prev = data['prev_labels'], data['prev_images']
        is_first_frame = img_prev is None
        z = data.get('z', None) if isinstance(data, dict) else None
        bs, _, h, w = label.size()
        if self.is_pose_data:
            label, label_prev = extract_valid_pose_labels([label, label_prev], self.pose_type,
                                                          self.remove_face_labels)
        cond_maps_now = self.get_cond_maps(label, self.label_embedding)
        if is_first_frame:
            x_img = self._first_frame_code(label, z, bs, cond_maps_now)
        else:
            x_img = self._encode_prev(img_prev, label_prev, cond_maps_now)

        flow = mask = img_warp = None
        warp_prev = self.temporal_initialized and not is_first_frame and \
            label_prev.shape[1] == self.num_frames_G - 1
        if warp_prev:
            flow, mask = self._temporal_flow(data, label, label_prev, img_prev, bs, h, w)
            img_warp = resample(img_prev[:, -1], flow)
            if self.spade_combine:
                cond_maps_img = self.get_cond_maps(torch.cat([img_warp, mask], dim=1),
                                                   self.img_prev_embedding)
        x_raw_img = None
        for i in range(self.num_downsamples_img, -1, -1):
            j = min(i, self.num_downsamples_embed)
            cond_maps = list(cond_maps_now[j])
            if self.generate_raw_output:
                if i >= self.num_multi_spade_layers - 1:
                    x_raw_img = x_img
                if i < self.num_multi_spade_layers:
                    x_raw_img = self.one_up_conv_layer(x_raw_img, cond_maps, i)
            if warp_prev and self.spade_combine and i < self.num_multi_spade_layers:
                cond_maps += cond_maps_img[j]
            x_img = self.one_up_conv_layer(x_img, cond_maps, i)
        img_final = torch.tanh(self.conv_img(x_img))
        img_raw = None
        if self.spade_combine and self.generate_raw_output:
            img_raw = torch.tanh(self.conv_img(x_raw_img))
        if warp_prev and not self.spade_combine:
            img_raw = img_final
            img_final = img_final * mask + img_warp * (1 - mask)
        return dict(fake_images=img_final, fake_flow_maps=flow, fake_occlusion_masks=mask,
                    fake_raw_images=img_raw, warped_images=img_warp)

    def _temporal_flow(self, data, label, label_prev, img_prev, bs, h, w):
        label_concat = torch.cat([label_prev.reshape(bs, -1, h, w), label], dim=1)
        return self.flow_network_temp(label_concat, img_prev.reshape(bs, -1, h, w))

    def one_up_conv_layer(self, x, encoded_label, i):
        x = getattr(self, 'up_%d' % i)(x, *encoded_label)
        return self.upsample(x) if i != 0 else x

    def init_temporal_network(self, cfg_init=None):
        nd = self.num_downsamples_img
        self.num_res_blocks = int(np.ceil((self.num_layers - nd) / 2.0) * 2)
        num_img_channels = get_paired_input_image_channel_number(self.data_cfg)
        self.down_first = Conv2dBlock(num_img_channels, self.num_filters, self.kernel_size,
                                      padding=self.kernel_size // 2)
        if cfg_init is not None:
            self.down_first.apply(weights_init(cfg_init.type, cfg_init.gain))
        params = self.gen_cfg.activation_norm_params
        for i in range(nd + 1):
            params.cond_dims = self.get_cond_dims(i)
            layer = self.base_res_block(self.get_num_filters(i), self.get_num_filters(i + 1))
            if cfg_init is not None:
                layer.apply(weights_init(cfg_init.type, cfg_init.gain))
            setattr(self, 'down_%d' % i, layer)
        res_ch = self.get_num_filters(nd + 1)
        params.cond_dims = self.get_cond_dims(nd + 1)
        for i in range(self.num_res_blocks):
            layer = self.base_res_block(res_ch, res_ch)
            if cfg_init is not None:
                layer.apply(weights_init(cfg_init.type, cfg_init.gain))
            setattr(self, 'res_%d' % i, layer)
        flow_cfg = self.flow_cfg
        self.temporal_initialized = True
        self.generate_raw_output = getattr(flow_cfg, 'generate_raw_output', False) and \
            self.spade_combine
        if self._use_learned_flow:
            self.flow_network_temp = FlowGenerator(flow_cfg, self.data_cfg)
            if cfg_init is not None:
                self.flow_network_temp.apply(weights_init(cfg_init.type, cfg_init.gain))
        self.spade_combine = getattr(flow_cfg, 'multi_spade_combine', True)
        if self.spade_combine:
            self.img_prev_embedding = LabelEmbedder(flow_cfg.multi_spade_combine.embed,
                                                    num_img_channels + 1)
            if cfg_init is not None:
                self.img_prev_embedding.apply(weights_init(cfg_init.type, cfg_init.gain))

    def get_cond_dims(self, num_downs=0):
        if not self.use_embed:
            return [self.num_input_channels]
        num_filters = getattr(self.emb_cfg, 'num_filters', 32)
        num_downs = min(num_downs, self.num_downsamples_embed)
        ch = [min(self.max_num_filters, num_filters * (2 ** num_downs))]
        if num_downs < self.num_multi_spade_layers:
            ch = ch * 2
        return ch

    def get_cond_maps(self, label, embedder):
        if not self.use_embed:
            return [[label]] * (self.num_layers + 1)
        return [[m] for m in embedder(label)]


class FlowGenerator(BaseNetwork):
    """Temporal flow network over [prev labels, label] and prev images
    (reference vid2vid.py:390-481)."""

    def __init__(self, flow_cfg, data_cfg):
        super().__init__()
        num_input_channels = get_paired_input_label_channel_number(data_cfg)
        num_prev_img_channels = get_paired_input_image_channel_number(data_cfg)
        num_frames = data_cfg.num_frames_G
        self.num_filters = num_filters = getattr(flow_cfg, 'num_filters', 32)
        self.max_num_filters = getattr(flow_cfg, 'max_num_filters', 1024)
        num_downsamples = getattr(flow_cfg, 'num_downsamples', 5)
        kernel_size = getattr(flow_cfg, 'kernel_size', 3)
        padding = kernel_size // 2
        self.num_res_blocks = getattr(flow_cfg, 'num_res_blocks', 6)
        self.flow_output_multiplier = getattr(flow_cfg, 'flow_output_multiplier', 20)
        activation_norm_type = getattr(flow_cfg, 'activation_norm_type', 'sync_batch')
        weight_norm_type = getattr(flow_cfg, 'weight_norm_type', 'spectral')
        block = partial(Conv2dBlock, kernel_size=kernel_size, padding=padding,
                        weight_norm_type=weight_norm_type,
                        activation_norm_type=activation_norm_type, nonlinearity='leakyrelu')
        down_lbl = [block(num_input_channels * num_frames, num_filters)]
        down_img = [block(num_prev_img_channels * (num_frames - 1), num_filters)]
        for i in range(num_downsamples):
            down_lbl += [block(self.get_num_filters(i), self.get_num_filters(i + 1), stride=2)]
            down_img += [block(self.get_num_filters(i), self.get_num_filters(i + 1), stride=2)]
        ch = self.get_num_filters(num_downsamples)
        res_flow = [Res2dBlock(ch, ch, kernel_size, padding=padding,
                               weight_norm_type=weight_norm_type,
                               activation_norm_type=activation_norm_type, order='CNACN')
                    for _ in range(self.num_res_blocks)]
        up_flow = []
        for i in reversed(range(num_downsamples)):
            up_flow += [Upsample(scale_factor=2),
                        block(self.get_num_filters(i + 1), self.get_num_filters(i))]
        self.down_lbl = nn.Sequential(*down_lbl)
        self.down_img = nn.Sequential(*down_img)
        self.res_flow = nn.Sequential(*res_flow)
        self.up_flow = nn.Sequential(*up_flow)
        self.conv_flow = nn.Sequential(Conv2dBlock(num_filters, 2, kernel_size, padding=padding))
        self.conv_mask = nn.Sequential(Conv2dBlock(num_filters, 1, kernel_size, padding=padding,
                                                   nonlinearity='sigmoid'))

    def forward(self, label, img_prev):
        res = self.res_flow(self.down_lbl(label) + self.down_img(img_prev))
        flow_feat = self.up_flow(res)
        return self.conv_flow(flow_feat) * self.flow_output_multiplier, \
            self.conv_mask(flow_feat)
