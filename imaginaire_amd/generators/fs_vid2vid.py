"""Few-shot vid2vid generator (reference generators/fs_vid2vid.py:24-1176).

Structure (same modules / state-dict names as the reference):

* ``WeightGenerator`` encodes the K reference frames (optionally attention-
  combined) and turns the encoded features into per-sample SPADE / conv /
  embedding weights with small spectral-norm MLPs (``fc_*``);
* ``LabelEmbedder`` is an encoder(-decoder / U-Net) over the driving label
  whose layers may themselves be hyper (per-sample) convolutions;
* ``FlowGenerator`` predicts flow + occlusion mask to warp the reference
  and previous frames, which enter the SPADE stack through extra
  conditional inputs (``SPADE_combine``);
* the decoder is a stack of ``HyperRes2dBlock``s whose SPADE and conv
  weights come from the weight generator.

MI355X notes: every hyper convolution runs as ONE batched k10 MFMA launch over
the whole batch (grid z = sample; layers/conv.py HyperConv2d, ops/conv.py
conv2d_per_sample) instead of a per-sample loop; SPADE normalisation +
modulation + activation is the fused HIP kernel k1; warps use the k9 HIP kernel;
the reference-frame attention softmaxes its bf16 energy in place (no fp32 copy). The reference's ``num_downsamples_atn`` typo
(fs_vid2vid.py:903 vs 906) is fixed so K > 1 works.
"""
import copy
import os
from functools import partial

import numpy as np
import torch
import torch.nn.functional as F
from torch import nn

from imaginaire_amd.layers import (Conv2dBlock, HyperConv2dBlock, HyperRes2dBlock, LinearBlock,
                                   Res2dBlock)
from imaginaire_amd.ops.few_shot import softmax_pool
from imaginaire_amd.model_utils.fs_vid2vid import (extract_valid_pose_labels, pick_image,
                                                   resample)
from imaginaire_amd.utils.data import (get_paired_input_image_channel_number,
                                       get_paired_input_label_channel_number)
from imaginaire_amd.utils.distributed import master_only_print as print
from imaginaire_amd.utils.init_weight import weights_init

# IMAGINAIRE_AMD_FUSED_ATTN=0: the reference formulation of the few-shot attention (energy
# matrix, softmax over K*HW, bmm) instead of the fused scaled-dot-product path
_FUSED_ATTN = os.environ.get('IMAGINAIRE_AMD_FUSED_ATTN', '1') == '1'
from imaginaire_amd.utils.misc import get_and_setattr, get_nested_attr
from imaginaire_amd.ops.resize import interpolate, Upsample
from imaginaire_amd.ops import attention as fused_attention_ops


def _filters(num_filters, max_num_filters, n):
    return [min(max_num_filters, num_filters * (2 ** i)) for i in range(n)]


class Generator(nn.Module):
    def __init__(self, gen_cfg, data_cfg):
        super().__init__()
        self.gen_cfg = gen_cfg
        self.data_cfg = data_cfg
        self.num_frames_G = data_cfg.num_frames_G
        self.flow_cfg = flow_cfg = gen_cfg.flow
        self.is_pose_data = hasattr(data_cfg, 'for_pose_dataset')
        if self.is_pose_data:
            pose_cfg = data_cfg.for_pose_dataset
            self.pose_type = getattr(pose_cfg, 'pose_type', 'both')
            self.remove_face_labels = getattr(pose_cfg, 'remove_face_labels', False)

        num_img_channels = get_paired_input_image_channel_number(data_cfg)
        self.num_downsamples = num_downsamples = get_and_setattr(gen_cfg, 'num_downsamples', 5)
        conv_kernel_size = get_and_setattr(gen_cfg, 'kernel_size', 3)
        num_filters = get_and_setattr(gen_cfg, 'num_filters', 32)
        max_num_filters = getattr(gen_cfg, 'max_num_filters', 1024)
        self.max_num_filters = gen_cfg.max_num_filters = \
            min(max_num_filters, num_filters * (2 ** num_downsamples))
        nf = _filters(num_filters, self.max_num_filters, num_downsamples + 2)

        hyper_cfg = gen_cfg.hyper
        self.use_hyper_spade = hyper_cfg.is_hyper_spade
        self.use_hyper_conv = hyper_cfg.is_hyper_conv
        self.num_hyper_layers = getattr(hyper_cfg, 'num_hyper_layers', 4)
        if self.num_hyper_layers == -1:
            self.num_hyper_layers = num_downsamples
        gen_cfg.hyper.num_hyper_layers = self.num_hyper_layers
        self.weight_generator = WeightGenerator(gen_cfg, data_cfg)
        self.num_multi_spade_layers = getattr(flow_cfg.multi_spade_combine, 'num_layers', 3)
        self.generate_raw_output = getattr(flow_cfg, 'generate_raw_output', False)

        padding = conv_kernel_size // 2
        activation_norm_type = get_and_setattr(gen_cfg, 'activation_norm_type', 'sync_batch')
        weight_norm_type = get_and_setattr(gen_cfg, 'weight_norm_type', 'spectral')
        activation_norm_params = get_and_setattr(gen_cfg, 'activation_norm_params', None)
        # SPADE conditions per level: label embedding (+ warped ref, + warped prev)
        spade_in = [[nf[i]] if i >= self.num_multi_spade_layers else [nf[i]] * 3
                    for i in range(num_downsamples + 1)]
        order = getattr(gen_cfg.hyper, 'hyper_block_order', 'NAC')
        for i in reversed(range(num_downsamples + 1)):
            activation_norm_params.cond_dims = spade_in[i]
            setattr(self, 'up_%d' % i, HyperRes2dBlock(
                nf[i + 1], nf[i], conv_kernel_size, padding=padding,
                weight_norm_type=weight_norm_type, activation_norm_type=activation_norm_type,
                activation_norm_params=activation_norm_params, order=order * 2,
                is_hyper_conv=self.use_hyper_conv and i < self.num_hyper_layers,
                is_hyper_norm=self.use_hyper_spade and i < self.num_hyper_layers))
        self.conv_img = Conv2dBlock(num_filters, num_img_channels, conv_kernel_size,
                                    padding=padding, nonlinearity='leakyrelu', order='AC')
        self.upsample = partial(interpolate, scale_factor=2)

        self.warp_ref = getattr(flow_cfg, 'warp_ref', True)
        if self.warp_ref:
            self.flow_network_ref = FlowGenerator(flow_cfg, data_cfg, 2)
            self.ref_image_embedding = LabelEmbedder(flow_cfg.multi_spade_combine.embed,
                                                     num_img_channels + 1)
        self.temporal_initialized = False
        if getattr(gen_cfg, 'init_temporal', True):
            self.init_temporal_network()

    def forward(self, data):
        label = data['label']
        ref_labels, ref_images = data['ref_labels'], data['ref_images']
        prev_labels, prev_images = data['prev_labels'], data['prev_images']
        is_first_frame = prev_labels is None
        if self.is_pose_data:
            label, prev_labels = extract_valid_pose_labels(
                [label, prev_labels], self.pose_type, self.remove_face_labels)
            ref_labels = extract_valid_pose_labels(ref_labels, self.pose_type,
                                                   self.remove_face_labels, do_remove=False)
        x, encoded_label, conv_weights, norm_weights, atn, atn_vis, ref_idx = \
            self.weight_generator(ref_images, ref_labels, label, is_first_frame)
        flow, flow_mask, img_warp, cond_inputs = self.flow_generation(
            label, ref_labels, ref_images, prev_labels, prev_images, ref_idx)
        encoded_label = [[e] for e in encoded_label]
        if self.generate_raw_output:
            encoded_label_raw = [list(encoded_label[i])
                                 for i in range(self.num_multi_spade_layers)]
            x_raw = None
        encoded_label = self.SPADE_combine(encoded_label, cond_inputs)
        for i in range(self.num_downsamples, -1, -1):
            conv_weight = norm_weight = [None] * 3
            if self.use_hyper_conv and i < self.num_hyper_layers:
                conv_weight = conv_weights[i]
            if self.use_hyper_spade and i < self.num_hyper_layers:
                norm_weight = norm_weights[i]
            x = self.one_up_conv_layer(x, encoded_label, conv_weight, norm_weight, i)
            if self.generate_raw_output and i < self.num_multi_spade_layers:
                x_raw = self.one_up_conv_layer(x_raw, encoded_label_raw, conv_weight,
                                               norm_weight, i)
            else:
                x_raw = x
        img_raw = torch.tanh(self.conv_img(x_raw)) if self.generate_raw_output else None
        img_final = torch.tanh(self.conv_img(x))
        return dict(fake_images=img_final, fake_flow_maps=flow,
                    fake_occlusion_masks=flow_mask, fake_raw_images=img_raw,
                    warped_images=img_warp, attention_visualization=atn_vis, ref_idx=ref_idx)

    def one_up_conv_layer(self, x, encoded_label, conv_weight, norm_weight, i):
        x = getattr(self, 'up_%d' % i)(x, *encoded_label[i], conv_weights=conv_weight,
                                       norm_weights=norm_weight)
        return self.upsample(x) if i != 0 else x

    def init_temporal_network(self, cfg_init=None):
        flow_cfg = self.flow_cfg
        emb_cfg = flow_cfg.multi_spade_combine.embed
        self.temporal_initialized = True
        self.sep_prev_flownet = flow_cfg.sep_prev_flow or (self.num_frames_G != 2) or \
            not flow_cfg.warp_ref
        if self.sep_prev_flownet:
            self.flow_network_temp = FlowGenerator(flow_cfg, self.data_cfg, self.num_frames_G)
            if cfg_init is not None:
                self.flow_network_temp.apply(weights_init(cfg_init.type, cfg_init.gain))
        else:
            self.flow_network_temp = self.flow_network_ref
        self.sep_prev_embedding = emb_cfg.sep_warp_embed or not flow_cfg.warp_ref
        if self.sep_prev_embedding:
            num_img_channels = get_paired_input_image_channel_number(self.data_cfg)
            self.prev_image_embedding = LabelEmbedder(emb_cfg, num_img_channels + 1)
            if cfg_init is not None:
                self.prev_image_embedding.apply(weights_init(cfg_init.type, cfg_init.gain))
        else:
            self.prev_image_embedding = self.ref_image_embedding
        if self.warp_ref:
            if self.sep_prev_flownet:
                self.init_network_weights(self.flow_network_ref, self.flow_network_temp)
                print('Initialized temporal flow network with the reference one.')
            if self.sep_prev_embedding:
                self.init_network_weights(self.ref_image_embedding, self.prev_image_embedding)
                print('Initialized temporal embedding network with the reference one.')
            self.flow_temp_is_initalized = True

    @staticmethod
    def init_network_weights(net_src, net_dst):
        src = net_src.state_dict()
        dst = net_dst.state_dict()
        for k, v in src.items():
            if k in dst and dst[k].size() == v.size():
                dst[k] = v
        net_dst.load_state_dict(dst)

    def load_pretrained_network(self, pretrained_dict, prefix='module.'):
        model_dict = self.state_dict()
        missing = set()
        for k, v in model_dict.items():
            kp = prefix + k
            if kp in pretrained_dict and v.size() == pretrained_dict[kp].size():
                model_dict[k] = pretrained_dict[kp]
            else:
                missing.add('.'.join(k.split('.')[:2]))
        print('Pretrained network has fewer layers; not initialized: {}'.format(sorted(missing)))
        self.load_state_dict(model_dict)

    def reset(self):
        self.weight_generator.reset()

    def flow_generation(self, label, ref_labels, ref_images, prev_labels, prev_images, ref_idx):
        ref_label, ref_image = pick_image([ref_labels, ref_images], ref_idx)
        has_prev = prev_labels is not None and prev_labels.shape[1] == self.num_frames_G - 1
        flow, occ_mask, img_warp, cond_inputs = [None] * 2, [None] * 2, [None] * 2, [None] * 2
        if self.warp_ref:
            flow_ref, occ_ref = self.flow_network_ref(label, ref_label, ref_image)
            flow[0], occ_mask[0] = flow_ref, occ_ref
            img_warp[0] = resample(ref_image, flow_ref)[:, :3]
            cond_inputs[0] = torch.cat([img_warp[0], occ_mask[0]], dim=1)
        if self.temporal_initialized and has_prev:
            b, t, c, h, w = prev_labels.shape
            flow_prev, occ_prev = self.flow_network_temp(label, prev_labels.reshape(b, -1, h, w),
                                                         prev_images.reshape(b, -1, h, w))
            flow[1], occ_mask[1] = flow_prev, occ_prev
            img_warp[1] = resample(prev_images[:, -1], flow_prev)
            cond_inputs[1] = torch.cat([img_warp[1], occ_mask[1]], dim=1)
        return flow, occ_mask, img_warp, cond_inputs

    def SPADE_combine(self, encoded_label, cond_inputs):  # noqa: N802
        feats = [None, None]
        if cond_inputs[0] is not None:
            feats[0] = self.ref_image_embedding(cond_inputs[0])
        if cond_inputs[1] is not None:
            feats[1] = self.prev_image_embedding(cond_inputs[1])
        for i in range(self.num_multi_spade_layers):
            encoded_label[i] += [f[i] if f is not None else None for f in feats]
        return encoded_label

    def custom_init(self):
        print('Use custom initialization for the generator.')
        for k, m in self.named_modules():
            if 'weight_generator.ref_label_' in k and 'norm' in k:
                m.eps = 1e-1


class WeightGenerator(nn.Module):
    """Reference encoder -> per-sample SPADE / conv / embedding weights
    (reference fs_vid2vid.py:394-783)."""

    def __init__(self, gen_cfg, data_cfg):
        super().__init__()
        self.data_cfg = data_cfg
        self.embed_cfg = embed_cfg = gen_cfg.embed
        self.embed_arch = embed_cfg.arch
        num_filters = gen_cfg.num_filters
        self.max_num_filters = gen_cfg.max_num_filters
        self.num_downsamples = num_downsamples = gen_cfg.num_downsamples
        self.num_filters_each_layer = nf = _filters(num_filters, self.max_num_filters,
                                                    num_downsamples + 2)
        if getattr(embed_cfg, 'num_filters', 32) != num_filters:
            raise ValueError('Embedding network must have the same number of filters as '
                             'generator.')
        hyper_cfg = gen_cfg.hyper
        kernel_size = getattr(hyper_cfg, 'kernel_size', 3)
        activation_norm_type = getattr(hyper_cfg, 'activation_norm_type', 'sync_batch')
        weight_norm_type = getattr(hyper_cfg, 'weight_norm_type', 'spectral')
        self.conv_kernel_size = conv_kernel_size = gen_cfg.kernel_size
        self.embed_kernel_size = embed_kernel_size = getattr(gen_cfg.embed, 'kernel_size', 3)
        self.kernel_size = kernel_size = getattr(gen_cfg.activation_norm_params,
                                                 'kernel_size', 1)
        self.spade_in_channels = [nf[i] for i in range(num_downsamples + 1)]
        self.use_hyper_spade = hyper_cfg.is_hyper_spade
        self.use_hyper_embed = hyper_cfg.is_hyper_embed
        self.use_hyper_conv = hyper_cfg.is_hyper_conv
        self.num_hyper_layers = hyper_cfg.num_hyper_layers
        order = getattr(gen_cfg.hyper, 'hyper_block_order', 'NAC')
        self.conv_before_norm = order.find('C') < order.find('N')
        self.concat_ref_label = 'concat' in hyper_cfg.method_to_use_ref_labels
        self.mul_ref_label = 'mul' in hyper_cfg.method_to_use_ref_labels
        self.sh_fix = self.sw_fix = 32
        self.num_fc_layers = getattr(hyper_cfg, 'num_fc_layers', 2)

        num_input_channels = get_paired_input_label_channel_number(data_cfg)
        if num_input_channels == 0:
            num_input_channels = getattr(data_cfg, 'label_channels', 1)
        elif get_nested_attr(data_cfg, 'for_pose_dataset.pose_type', 'both') == 'open':
            num_input_channels -= 3
        data_cfg.num_input_channels = num_input_channels
        num_img_channels = get_paired_input_image_channel_number(data_cfg)
        num_ref_channels = num_img_channels + (num_input_channels if self.concat_ref_label
                                               else 0)
        conv_2d_block = partial(Conv2dBlock, kernel_size=kernel_size,
                                padding=(kernel_size // 2), weight_norm_type=weight_norm_type,
                                activation_norm_type=activation_norm_type,
                                nonlinearity='leakyrelu')
        self.ref_img_first = conv_2d_block(num_ref_channels, num_filters)
        if self.mul_ref_label:
            self.ref_label_first = conv_2d_block(num_input_channels, num_filters)
        for i in range(num_downsamples):
            in_ch, out_ch = nf[i], nf[i + 1]
            setattr(self, 'ref_img_down_%d' % i, conv_2d_block(in_ch, out_ch, stride=2))
            setattr(self, 'ref_img_up_%d' % i, conv_2d_block(out_ch, in_ch))
            if self.mul_ref_label:
                setattr(self, 'ref_label_down_%d' % i, conv_2d_block(in_ch, out_ch, stride=2))
                setattr(self, 'ref_label_up_%d' % i, conv_2d_block(out_ch, in_ch))

        if self.use_hyper_spade or self.use_hyper_conv:
            for i in range(self.num_hyper_layers):
                ch_in, ch_out = nf[i], nf[i + 1]
                conv_ks2, embed_ks2, spade_ks2 = conv_kernel_size ** 2, embed_kernel_size ** 2, \
                    kernel_size ** 2
                spade_in_ch = self.spade_in_channels[i]
                heads = []  # (name, fc input, fc output)
                if self.use_hyper_spade:
                    n0 = (spade_in_ch * spade_ks2 + 1) * (1 if self.conv_before_norm else 2)
                    n1 = (spade_in_ch * spade_ks2 + 1) * (1 if ch_in != ch_out else 2)
                    heads += [('fc_spade_0', ch_out, n0), ('fc_spade_1', ch_out, n1),
                              ('fc_spade_s', ch_out, n0)]
                    if self.use_hyper_embed:
                        heads += [('fc_spade_e', ch_out, ch_in * embed_ks2 + 1)]
                if self.use_hyper_conv:
                    heads += [('fc_conv_0', ch_in, ch_out * conv_ks2 + 1),
                              ('fc_conv_1', ch_in, ch_in * conv_ks2 + 1),
                              ('fc_conv_s', ch_in, ch_out + 1)]
                lin = partial(LinearBlock, weight_norm_type='spectral', nonlinearity='leakyrelu')
                for name, fc_in, fc_out in heads:
                    fc_in = fc_in if self.mul_ref_label else self.sh_fix * self.sw_fix
                    layers = [lin(fc_in, ch_out)]
                    layers += [lin(ch_out, ch_out) for _ in range(1, self.num_fc_layers)]
                    layers += [LinearBlock(ch_out, fc_out, weight_norm_type='spectral')]
                    setattr(self, '%s_%d' % (name, i), nn.Sequential(*layers))

        num_hyper_layers = self.num_hyper_layers if self.use_hyper_embed else 0
        self.label_embedding = LabelEmbedder(self.embed_cfg, num_input_channels,
                                             num_hyper_layers=num_hyper_layers)
        if hasattr(hyper_cfg, 'attention'):
            self.num_downsample_atn = get_and_setattr(hyper_cfg.attention, 'num_downsamples', 2)
            if data_cfg.initial_few_shot_K > 1:
                self.attention_module = AttentionModule(hyper_cfg.attention, data_cfg,
                                                        conv_2d_block, nf)
        else:
            self.num_downsample_atn = 0

    def forward(self, ref_image, ref_label, label, is_first_frame):
        b, k, c, h, w = ref_image.size()
        ref_image = ref_image.reshape(b * k, -1, h, w)
        if ref_label is not None:
            ref_label = ref_label.reshape(b * k, -1, h, w)
        x, encoded_ref, atn, atn_vis, ref_idx = self.encode_reference(ref_image, ref_label,
                                                                      label, k)
        if self.training or is_first_frame or k > 1:
            embedding_weights, norm_weights, conv_weights = [], [], []
            for i in range(self.num_hyper_layers):
                if self.use_hyper_spade:
                    feat = encoded_ref[min(len(encoded_ref) - 1, i + 1)]
                    ew, nw = self.get_norm_weights(feat, i)
                    embedding_weights.append(ew)
                    norm_weights.append(nw)
                if self.use_hyper_conv:
                    feat = encoded_ref[min(len(encoded_ref) - 1, i)]
                    conv_weights.append(self.get_conv_weights(feat, i))
            if not self.training:
                self.embedding_weights, self.conv_weights, self.norm_weights = \
                    embedding_weights, conv_weights, norm_weights
        else:
            embedding_weights, conv_weights, norm_weights = \
                self.embedding_weights, self.conv_weights, self.norm_weights
        encoded_label = self.label_embedding(
            label, weights=embedding_weights if self.use_hyper_embed else None)
        return x, encoded_label, conv_weights, norm_weights, atn, atn_vis, ref_idx

    def encode_reference(self, ref_image, ref_label, label, k):
        if self.concat_ref_label:
            x = self.ref_img_first(torch.cat([ref_image, ref_label], dim=1))
        elif self.mul_ref_label:
            x = self.ref_img_first(ref_image)
            x_label = self.ref_label_first(ref_label)
        else:
            x = self.ref_img_first(ref_image)
        atn = atn_vis = ref_idx = None
        for i in range(self.num_downsamples):
            x = getattr(self, 'ref_img_down_%d' % i)(x)
            if self.mul_ref_label:
                x_label = getattr(self, 'ref_label_down_%d' % i)(x_label)
            if k > 1 and i == self.num_downsample_atn - 1 and not _FUSED_ATTN:
                x, atn, atn_vis = self.attention_module(x, label, ref_label)
                if self.mul_ref_label:
                    x_label, _, _ = self.attention_module(x_label, None, None, atn)
                atn_sum = atn.reshape(label.shape[0], k, -1).sum(2)
                ref_idx = torch.argmax(atn_sum, dim=1)
            elif k > 1 and i == self.num_downsample_atn - 1:
                # one fused attention for the image (and label) features: no B x KHW x HW
                # matrix, the per-frame attention mass as a side output
                feats = [x, x_label] if self.mul_ref_label else [x]
                outs, atn_full = self.attention_module.fused(feats, label, ref_label)
                x = outs[0]
                if self.mul_ref_label:
                    x_label = outs[1]
                atn_vis = atn_full[-1:, 0:1]
                atn_sum = atn_full.reshape(label.shape[0], k, -1).float().sum(2)
                ref_idx = torch.argmax(atn_sum, dim=1)
        encoded_image_ref = [x]
        if self.mul_ref_label:
            encoded_ref_label = [x_label]
        for i in reversed(range(self.num_downsamples)):
            encoded_image_ref.append(getattr(self, 'ref_img_up_%d' % i)(encoded_image_ref[-1]))
            if self.mul_ref_label:
                encoded_ref_label.append(
                    getattr(self, 'ref_label_up_%d' % i)(encoded_ref_label[-1]))
        if self.mul_ref_label:
            encoded_ref = []
            for conv, conv_label in zip(encoded_image_ref, encoded_ref_label):
                # Σ_hw conv[b, c, hw] * softmax_c'(label)[b, c', hw]: k15 channel softmax +
                # per-sample k11 MFMA GEMM (ops/few_shot.py)
                prod = softmax_pool(conv, conv_label)
                encoded_ref.append(prod.unsqueeze(-1))
        else:
            encoded_ref = encoded_image_ref
        return x, encoded_ref[::-1], atn, atn_vis, ref_idx

    def _embed_input(self, x):
        if not self.mul_ref_label:
            x = F.adaptive_avg_pool2d(x, (self.sh_fix, self.sw_fix))
        return WeightReshaper().reshape_embed_input(x)

    def get_norm_weights(self, x, i):
        in_ch = self.num_filters_each_layer[i]
        out_ch = self.num_filters_each_layer[i + 1]
        spade_ch = self.spade_in_channels[i]
        eks, sks = self.embed_kernel_size, self.kernel_size
        b = x.size(0)
        rs = WeightReshaper()
        x = self._embed_input(x)
        embedding_weights = None
        if self.use_hyper_embed:
            fc_e = getattr(self, 'fc_spade_e_%d' % i)(x).reshape(b, -1)
            if 'decoder' in self.embed_arch:
                shape = [in_ch, out_ch, eks, eks]
                fc_e = fc_e[:, :-in_ch]
            else:
                shape = [out_ch, in_ch, eks, eks]
            embedding_weights = rs.reshape_weight(fc_e, shape)
        fc_0 = getattr(self, 'fc_spade_0_%d' % i)(x).reshape(b, -1)
        fc_1 = getattr(self, 'fc_spade_1_%d' % i)(x).reshape(b, -1)
        fc_s = getattr(self, 'fc_spade_s_%d' % i)(x).reshape(b, -1)
        if self.conv_before_norm:
            out_ch = in_ch
        norm_weights = [rs.reshape_weight(fc_0, [out_ch * 2, spade_ch, sks, sks]),
                        rs.reshape_weight(fc_1, [in_ch * 2, spade_ch, sks, sks]),
                        rs.reshape_weight(fc_s, [out_ch * 2, spade_ch, sks, sks])]
        return embedding_weights, norm_weights

    def get_conv_weights(self, x, i):
        in_ch = self.num_filters_each_layer[i]
        out_ch = self.num_filters_each_layer[i + 1]
        cks = self.conv_kernel_size
        b = x.size(0)
        rs = WeightReshaper()
        x = self._embed_input(x)
        fc_0 = getattr(self, 'fc_conv_0_%d' % i)(x).reshape(b, -1)
        fc_1 = getattr(self, 'fc_conv_1_%d' % i)(x).reshape(b, -1)
        fc_s = getattr(self, 'fc_conv_s_%d' % i)(x).reshape(b, -1)
        return [rs.reshape_weight(fc_0, [in_ch, out_ch, cks, cks]),
                rs.reshape_weight(fc_1, [in_ch, in_ch, cks, cks]),
                rs.reshape_weight(fc_s, [in_ch, out_ch, 1, 1])]

    def reset(self):
        self.embedding_weights = self.conv_weights = self.norm_weights = None


class WeightReshaper:
    """Split flat MLP outputs into [weight, bias] pairs (fs_vid2vid.py:786-883)."""

    def reshape_weight(self, x, weight_shape):
        if isinstance(weight_shape[0], list) and not isinstance(x, list):
            x = self.split_weights(x, self.sum_mul(weight_shape))
        if isinstance(x, list):
            return [self.reshape_weight(xi, wi) for xi, wi in zip(x, weight_shape)]
        shape = [x.size(0)] + list(weight_shape)
        bias_size = shape[1]
        n_w = int(np.prod(shape[1:]))
        if x.size(1) == n_w + bias_size:
            return [x[:, :-bias_size].reshape(shape), x[:, -bias_size:]]
        return [x.reshape(shape), None]

    def split_weights(self, weight, sizes):
        if isinstance(sizes, list):
            out, cur = [], 0
            for s in sizes:
                nxt = cur + self.sum(s)
                out.append(self.split_weights(weight[:, cur:nxt], s))
                cur = nxt
            assert cur == weight.size(1)
            return out
        return weight

    def reshape_embed_input(self, x):
        if isinstance(x, list):
            return [self.reshape_embed_input(xi) for xi in x]
        b, c = x.shape[:2]
        return x.reshape(b * c, -1)

    def sum(self, x):
        return sum(self.sum(xi) for xi in x) if isinstance(x, list) else x

    def sum_mul(self, x):
        assert isinstance(x, list)
        if not isinstance(x[0], list):
            return int(np.prod(x)) + x[0]
        return [self.sum_mul(xi) for xi in x]


class AttentionModule(nn.Module):
    """Dot-product attention from the driving label over the K reference
    frames (fs_vid2vid.py:886-969). The B x KHW x HW energy, softmax and
    feature mixing are two batched GEMMs (hipBLASLt)."""

    def __init__(self, atn_cfg, data_cfg, conv_2d_block, num_filters_each_layer):
        super().__init__()
        self.initial_few_shot_K = data_cfg.initial_few_shot_K
        num_input_channels = data_cfg.num_input_channels
        # the reference reads num_filters from the hyper cfg (default 32), which only
        # matches the key/query towers when the generator also uses 32 filters; the
        # towers' first layer must produce num_filters_each_layer[0] channels.
        num_filters = num_filters_each_layer[0]
        self.num_downsample_atn = getattr(atn_cfg, 'num_downsamples', 2)
        self.atn_query_first = conv_2d_block(num_input_channels, num_filters)
        self.atn_key_first = conv_2d_block(num_input_channels, num_filters)
        for i in range(self.num_downsample_atn):
            f_in, f_out = num_filters_each_layer[i], num_filters_each_layer[i + 1]
            setattr(self, 'atn_key_%d' % i, conv_2d_block(f_in, f_out, stride=2))
            setattr(self, 'atn_query_%d' % i, conv_2d_block(f_in, f_out, stride=2))

    def forward(self, in_features, label, ref_label, attention=None):
        b, c, h, w = in_features.size()
        k = self.initial_few_shot_K
        b = b // k
        if attention is None:
            atn_key = self.attention_encode(ref_label, 'atn_key')
            atn_query = self.attention_encode(label, 'atn_query')
            atn_key = atn_key.reshape(b, k, c, -1).permute(0, 1, 3, 2).reshape(b, -1, c)
            atn_query = atn_query.reshape(b, c, -1)
            energy = torch.bmm(atn_key, atn_query)
            if energy.is_cuda and energy.dtype == torch.bfloat16:
                # softmax over the K*HW reference positions on the bf16 energy itself (fp32
                # accumulation inside the kernel): autocast would otherwise widen the
                # B x KHW x HW matrix to fp32, softmax it in fp32 and narrow it back for the
                # next bmm — three passes over the largest tensor of the generator
                with torch.autocast('cuda', enabled=False):
                    attention = torch.softmax(energy, dim=1)
            else:
                attention = torch.softmax(energy, dim=1)
        feats = in_features.reshape(b, k, c, h * w).permute(0, 2, 1, 3).reshape(b, c, -1)
        out = torch.bmm(feats, attention).reshape(b, c, h, w)
        atn_vis = attention.reshape(b, k, h * w, h * w).sum(2).reshape(b, k, h, w)
        return out, attention, atn_vis[-1:, 0:1]

    def fused(self, features, label, ref_label):
        """The attention of :meth:`forward` applied to every tensor of ``features`` (each
        [B*K, C_i, H, W]) without materialising the B x KHW x HW attention matrix: one fused
        attention (the k16 HIP kernel, ops/attention.py; PyTorch SDPA off the GPU; scale 1,
        softmax over the K*HW reference positions) whose
        values are the features' channels plus K frame-indicator channels, so the same call
        also returns, per query position, the attention mass on each reference frame (the
        reference's ``attention.reshape(b, k, hw, hw).sum(2)``). Returns (outputs, atn_vis
        [B, K, H, W])."""
        import torch.nn.functional as F
        bk, c, h, w = features[0].shape
        k = self.initial_few_shot_K
        b = bk // k
        hw = h * w
        atn_key = self.attention_encode(ref_label, 'atn_key')
        atn_query = self.attention_encode(label, 'atn_query')
        ck = atn_key.shape[1]
        q = atn_query.reshape(b, ck, hw).transpose(1, 2)                       # [b, hw, ck]
        key = atn_key.reshape(b, k, ck, hw).permute(0, 1, 3, 2).reshape(b, k * hw, ck)
        vals = [f.reshape(b, k, f.shape[1], hw).permute(0, 1, 3, 2).reshape(b, k * hw, -1)
                for f in features]
        ind = torch.eye(k, device=q.device, dtype=vals[0].dtype).repeat_interleave(hw, 0)
        vals.append(ind.unsqueeze(0).expand(b, -1, -1))
        v = torch.cat(vals, 2)
        dt = torch.get_autocast_dtype('cuda') if q.is_cuda and torch.is_autocast_enabled('cuda') \
            else q.dtype
        if dt == torch.bfloat16 and fused_attention_ops.native_ok(q, key, v):
            # the k16 HIP kernel: online softmax over the K*HW keys, no attention matrix in HBM
            # (bf16 compute only: an fp32 run keeps the fp32 SDPA path and its dtype)
            o = fused_attention_ops.fused_attention(q, key, v, 1.0)
        else:
            # one head dim for q, k and v (zero columns change no dot product)
            d = max(ck, v.shape[2])
            d = (d + 7) // 8 * 8
            q = F.pad(q, (0, d - ck))
            key = F.pad(key, (0, d - ck))
            v = F.pad(v, (0, d - v.shape[2]))
            with torch.autocast('cuda', enabled=False):
                o = F.scaled_dot_product_attention(q.unsqueeze(1).to(dt), key.unsqueeze(1).to(dt),
                                                   v.unsqueeze(1).to(dt), scale=1.0).squeeze(1)
        outs, off = [], 0
        for f in features:
            cf = f.shape[1]
            outs.append(o[:, :, off:off + cf].transpose(1, 2).reshape(b, cf, h, w))
            off += cf
        atn_vis = o[:, :, off:off + k].transpose(1, 2).reshape(b, k, h, w)
        return outs, atn_vis

    def attention_encode(self, img, net_name):
        x = getattr(self, net_name + '_first')(img)
        for i in range(self.num_downsample_atn):
            x = getattr(self, '%s_%d' % (net_name, i))(x)
        return x


class FlowGenerator(nn.Module):
    """Flow + occlusion-mask predictor (fs_vid2vid.py:972-1069)."""

    def __init__(self, flow_cfg, data_cfg, num_frames):
        super().__init__()
        num_input_channels = data_cfg.num_input_channels or 1
        num_prev_img_channels = get_paired_input_image_channel_number(data_cfg)
        num_downsamples = getattr(flow_cfg, 'num_downsamples', 3)
        kernel_size = getattr(flow_cfg, 'kernel_size', 3)
        padding = kernel_size // 2
        num_blocks = getattr(flow_cfg, 'num_blocks', 6)
        num_filters = getattr(flow_cfg, 'num_filters', 32)
        max_num_filters = getattr(flow_cfg, 'max_num_filters', 1024)
        nf = _filters(num_filters, max_num_filters, num_downsamples + 1)
        self.flow_output_multiplier = getattr(flow_cfg, 'flow_output_multiplier', 20)
        self.sep_up_mask = getattr(flow_cfg, 'sep_up_mask', False)
        activation_norm_type = getattr(flow_cfg, 'activation_norm_type', 'sync_batch')
        weight_norm_type = getattr(flow_cfg, 'weight_norm_type', 'spectral')
        block = partial(Conv2dBlock, kernel_size=kernel_size, padding=padding,
                        weight_norm_type=weight_norm_type,
                        activation_norm_type=activation_norm_type, nonlinearity='leakyrelu')
        in_ch = num_input_channels * num_frames + num_prev_img_channels * (num_frames - 1)
        down = [block(in_ch, num_filters)]
        down += [block(nf[i], nf[i + 1], stride=2) for i in range(num_downsamples)]
        ch = nf[num_downsamples]
        res = [Res2dBlock(ch, ch, kernel_size, padding=padding,
                          weight_norm_type=weight_norm_type,
                          activation_norm_type=activation_norm_type, order='NACNAC')
               for _ in range(num_blocks)]
        up = []
        for i in reversed(range(num_downsamples)):
            up += [Upsample(scale_factor=2), block(nf[i + 1], nf[i])]
        self.down_flow = nn.Sequential(*down)
        self.res_flow = nn.Sequential(*res)
        self.up_flow = nn.Sequential(*up)
        if self.sep_up_mask:
            self.up_mask = nn.Sequential(*copy.deepcopy(up))
        self.conv_flow = nn.Sequential(Conv2dBlock(num_filters, 2, kernel_size, padding=padding))
        self.conv_mask = nn.Sequential(Conv2dBlock(num_filters, 1, kernel_size, padding=padding,
                                                   nonlinearity='sigmoid'))

    def forward(self, label, ref_label, ref_image):
        res = self.res_flow(self.down_flow(torch.cat([label, ref_label, ref_image], dim=1)))
        flow_feat = self.up_flow(res)
        flow = self.conv_flow(flow_feat) * self.flow_output_multiplier
        mask = self.conv_mask(self.up_mask(res) if self.sep_up_mask else flow_feat)
        return flow, mask


class LabelEmbedder(nn.Module):
    """Label encoder / encoder-decoder / U-Net with optional hyper convs
    (fs_vid2vid.py:1072-1176). Returns the per-level features fine->coarse."""

    def __init__(self, emb_cfg, num_input_channels, num_hyper_layers=0):
        super().__init__()
        num_filters = getattr(emb_cfg, 'num_filters', 32)
        max_num_filters = getattr(emb_cfg, 'max_num_filters', 1024)
        self.arch = getattr(emb_cfg, 'arch', 'encoderdecoder')
        self.num_downsamples = num_downsamples = getattr(emb_cfg, 'num_downsamples', 5)
        kernel_size = getattr(emb_cfg, 'kernel_size', 3)
        weight_norm_type = getattr(emb_cfg, 'weight_norm_type', 'spectral')
        activation_norm_type = getattr(emb_cfg, 'activation_norm_type', 'none')
        self.unet = 'unet' in self.arch
        self.has_decoder = 'decoder' in self.arch or self.unet
        self.num_hyper_layers = num_hyper_layers if num_hyper_layers != -1 else num_downsamples
        block = partial(HyperConv2dBlock, kernel_size=kernel_size, padding=kernel_size // 2,
                        weight_norm_type=weight_norm_type,
                        activation_norm_type=activation_norm_type, nonlinearity='leakyrelu')
        ch = _filters(num_filters, max_num_filters, num_downsamples + 1)
        self.conv_first = block(num_input_channels, num_filters, activation_norm_type='none')
        for i in range(num_downsamples):
            setattr(self, 'down_%d' % i, block(
                ch[i], ch[i + 1], stride=2,
                is_hyper_conv=(i < num_hyper_layers) and not self.has_decoder))
        if self.has_decoder:
            self.upsample = Upsample(scale_factor=2)
            for i in reversed(range(num_downsamples)):
                ch_i = ch[i + 1] * (2 if self.unet and i != num_downsamples - 1 else 1)
                setattr(self, 'up_%d' % i, block(ch_i, ch[i],
                                                 is_hyper_conv=(i < num_hyper_layers)))

    def forward(self, input, weights=None):
        if input is None:
            return None
        output = [self.conv_first(input)]
        for i in range(self.num_downsamples):
            layer = getattr(self, 'down_%d' % i)
            if i >= self.num_hyper_layers or self.has_decoder:
                output.append(layer(output[-1]))
            else:
                output.append(layer(output[-1], conv_weights=weights[i]))
        if not self.has_decoder:
            return output
        if not self.unet:
            output = [output[-1]]
        for i in reversed(range(self.num_downsamples)):
            inp = output[-1]
            if self.unet and i != self.num_downsamples - 1:
                inp = torch.cat([inp, output[i + 1]], dim=1)
            inp = self.upsample(inp)
            layer = getattr(self, 'up_%d' % i)
            output.append(layer(inp) if i >= self.num_hyper_layers
                          else layer(inp, conv_weights=weights[i]))
        if self.unet:
            output = output[self.num_downsamples:]
        return output[::-1]
