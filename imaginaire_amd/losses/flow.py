"""Flow-related losses (reference losses/flow.py:14-313).

``MaskedL1Loss`` (optionally normalised over the valid region) and
``FlowLoss``: GT flow + confidence for (reference→target) and
(previous→target) from the FlowNet2 stack (whose correlation / resample2d /
channelnorm ops are the HIP kernels k6-k8), flow L1, warp L1 and occlusion-
mask losses.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from imaginaire_amd.model_utils.fs_vid2vid import (get_face_mask, get_fg_mask, get_part_mask,
                                                   pick_image, resample)
from imaginaire_amd.registry import import_module


class MaskedL1Loss(nn.Module):
    def __init__(self, normalize_over_valid=False):
        super().__init__()
        self.criterion = nn.L1Loss()
        self.normalize_over_valid = normalize_over_valid

    def forward(self, input, target, mask):
        mask = mask.expand_as(input)
        loss = self.criterion(input * mask, target * mask)
        if self.normalize_over_valid:
            loss = loss * torch.numel(mask) / (torch.sum(mask) + 1e-6)
        return loss


class FlowLoss(nn.Module):
    """Flow supervision from a frozen FlowNet2 (reference losses/flow.py:42-313).

    GT flows (reference->target from RGB or, for pose data, DensePose maps;
    previous->target from the real previous frame once temporal training has
    started) + FlowNet2 confidence; losses: masked flow L1, warp L1 (plus
    body-part / foreground warp terms for pose data) and occlusion-mask
    losses. FlowNet2 runs bf16 when AMP is on (``fp16`` in the reference).
    """

    def __init__(self, cfg):
        super().__init__()
        self.cfg = cfg
        self.data_cfg = cfg.data
        self.criterion = nn.L1Loss()
        self.criterionMasked = MaskedL1Loss()
        flow_module = import_module(getattr(cfg.flow_network, 'type',
                                            'imaginaire_amd.third_party.flow_net.flow_net'))
        fp16 = str(getattr(cfg.trainer, 'amp', 'O0')) > 'O0'
        self.flowNet = flow_module.FlowNet(pretrained=True, fp16=fp16)
        self.warp_ref = getattr(cfg.gen.flow, 'warp_ref', False)
        self.pose_cfg = getattr(cfg.data, 'for_pose_dataset', None)
        self.for_pose_dataset = self.pose_cfg is not None
        self.has_fg = getattr(cfg.data, 'has_foreground', False)

    def _zero(self, ref):
        return torch.zeros((), device=ref.device)

    def forward(self, data, net_G_output, current_epoch):
        tgt_label, tgt_image = data['label'], data['image']
        fake_image = net_G_output['fake_images']
        warped_images = net_G_output['warped_images']
        flow = net_G_output['fake_flow_maps']
        occ_mask = net_G_output['fake_occlusion_masks']
        if self.warp_ref:
            ref_label, ref_image = pick_image([data['ref_labels'], data['ref_images']],
                                              net_G_output['ref_idx'])
        else:
            ref_label = ref_image = None
        flow_gt_prev = flow_gt_ref = conf_gt_prev = conf_gt_ref = None
        with torch.no_grad():
            if self.warp_ref:
                if self.for_pose_dataset:
                    flow_gt_ref, conf_gt_ref = self.flowNet(tgt_label[:, :3], ref_label[:, :3])
                else:
                    flow_gt_ref, conf_gt_ref = self.flowNet(tgt_image, ref_image)
            if current_epoch >= getattr(self.cfg, 'single_frame_epoch', 0) and \
                    data.get('real_prev_image') is not None:
                flow_gt_prev, conf_gt_prev = self.flowNet(tgt_image, data['real_prev_image'])
        flow_gt = [flow_gt_ref, flow_gt_prev]
        flow_conf_gt = [conf_gt_ref, conf_gt_prev]
        fg_mask, ref_fg_mask = get_fg_mask([tgt_label, ref_label], self.has_fg)
        loss_flow_L1, loss_flow_warp, body_mask_diff = self.compute_flow_losses(
            flow, warped_images, tgt_image, flow_gt, flow_conf_gt, fg_mask, tgt_label,
            ref_label)
        loss_mask = self.compute_mask_losses(occ_mask, fake_image, warped_images, tgt_label,
                                             tgt_image, fg_mask, ref_fg_mask, body_mask_diff)
        return loss_flow_L1, loss_flow_warp, loss_mask

    def compute_flow_losses(self, flow, warped_images, tgt_image, flow_gt, flow_conf_gt,
                            fg_mask, tgt_label, ref_label):
        loss_flow_L1 = self._zero(tgt_image)
        loss_flow_warp = self._zero(tgt_image)
        if isinstance(flow, list):
            for i in range(len(flow)):
                l1, lw = self.compute_flow_loss(flow[i], warped_images[i], tgt_image,
                                                flow_gt[i], flow_conf_gt[i], fg_mask)
                loss_flow_L1 = loss_flow_L1 + l1
                loss_flow_warp = loss_flow_warp + lw
        else:
            loss_flow_L1, loss_flow_warp = self.compute_flow_loss(
                flow, warped_images, tgt_image, flow_gt[-1], flow_conf_gt[-1], fg_mask)
        body_mask_diff = None
        if self.warp_ref:
            if self.for_pose_dataset:
                body_mask = get_part_mask(tgt_label[:, 2])
                warped_ref_body = resample(get_part_mask(ref_label[:, 2]), flow[0])
                loss_flow_warp = loss_flow_warp + self.criterion(warped_ref_body, body_mask)
                body_mask_diff = torch.sum((warped_ref_body - body_mask).abs(), dim=1,
                                           keepdim=True)
            if self.has_fg:
                fg, ref_fg = get_fg_mask([tgt_label, ref_label], True)
                loss_flow_warp = loss_flow_warp + self.criterion(resample(ref_fg, flow[0]), fg)
        return loss_flow_L1, loss_flow_warp, body_mask_diff

    def compute_flow_loss(self, flow, warped_image, tgt_image, flow_gt, flow_conf_gt, fg_mask):
        loss_flow_L1 = self._zero(tgt_image)
        loss_flow_warp = self._zero(tgt_image)
        if flow is not None and flow_gt is not None:
            loss_flow_L1 = self.criterionMasked(flow, flow_gt, flow_conf_gt * fg_mask)
        if warped_image is not None:
            loss_flow_warp = self.criterion(warped_image, tgt_image)
        return loss_flow_L1, loss_flow_warp

    def compute_mask_losses(self, occ_mask, fake_image, warped_image, tgt_label, tgt_image,
                            fg_mask, ref_fg_mask, body_mask_diff):
        loss_mask = self._zero(tgt_image)
        if isinstance(occ_mask, list):
            for i in range(len(occ_mask)):
                loss_mask = loss_mask + self.compute_mask_loss(occ_mask[i], warped_image[i],
                                                               tgt_image)
        else:
            loss_mask = loss_mask + self.compute_mask_loss(occ_mask, warped_image, tgt_image)
        if self.warp_ref:
            ref_occ_mask = occ_mask[0]
            dummy0 = torch.zeros_like(ref_occ_mask)
            dummy1 = torch.ones_like(ref_occ_mask)
            if self.for_pose_dataset:
                face_mask = F.avg_pool2d(get_face_mask(tgt_label[:, 2]).unsqueeze(1), 15,
                                         stride=1, padding=7)
                loss_mask = loss_mask + self.criterionMasked(ref_occ_mask, dummy0, face_mask)
                loss_mask = loss_mask + self.criterionMasked(fake_image, warped_image[0],
                                                             face_mask)
                loss_mask = loss_mask + self.criterionMasked(ref_occ_mask, dummy1,
                                                             body_mask_diff)
            if self.has_fg:
                fg_mask_diff = ((ref_fg_mask - fg_mask) > 0).float()
                loss_mask = loss_mask + self.criterionMasked(ref_occ_mask, dummy1, fg_mask_diff)
        return loss_mask

    def compute_mask_loss(self, occ_mask, warped_image, tgt_image):
        if occ_mask is None:
            return self._zero(tgt_image)
        dummy0 = torch.zeros_like(occ_mask)
        dummy1 = torch.ones_like(occ_mask)
        img_diff = torch.sum((warped_image - tgt_image).abs(), dim=1, keepdim=True)
        conf = torch.clamp(1 - img_diff, 0, 1)
        return self.criterionMasked(occ_mask, dummy0, conf) + \
            self.criterionMasked(occ_mask, dummy1, 1 - conf)
