"""FUNIT / COCO-FUNIT trainer (reference trainers/funit.py:17-162): GAN on
translation + reconstruction, L1 reconstruction, L1 feature matching on
pooled D features; FID averaged over style classes."""
import os

import numpy as np
import torch
from torch import nn

from imaginaire_amd.losses.l1 import L1Loss
from imaginaire_amd.evaluation import compute_fid
from imaginaire_amd.losses import GANLoss
from imaginaire_amd.trainers.base import BaseTrainer
from imaginaire_amd.trainers.munit import _weights_from
from imaginaire_amd.utils.distributed import is_master


class Trainer(BaseTrainer):
    rank_uniform_control_flow = True

    def _init_loss(self, cfg):
        self.criteria['gan'] = GANLoss(cfg.trainer.gan_mode)
        self.criteria['image_recon'] = L1Loss()
        self.criteria['feature_matching'] = L1Loss()
        self.weights.update(_weights_from(cfg.trainer.loss_weight))

    def gen_forward(self, data):
        out = self.net_G(data)
        dout = self.net_D(data, out)
        self._time_before_loss()
        gan = self.criteria['gan']
        self.gen_losses['gan'] = 0.5 * (gan(dout['fake_out_trans'], True, dis_update=False) +
                                        gan(dout['fake_out_recon'], True, dis_update=False))
        self.gen_losses['image_recon'] = self.criteria['image_recon'](out['images_recon'],
                                                                      data['images_content'])
        self.gen_losses['feature_matching'] = self.criteria['feature_matching'](
            dout['fake_features_trans'], dout['real_features_style'])
        return self._get_total_loss(gen_forward=True)

    def dis_forward(self, data):
        with torch.no_grad():
            out = self.net_G(data)
        out['images_trans'].requires_grad = True
        dout = self.net_D(data, out, recon=False)
        self._time_before_loss()
        self.dis_losses['gan'] = self.criteria['gan'](dout['real_out_style'], True) + \
            self.criteria['gan'](dout['fake_out_trans'], False)
        self.dis_losses['gp'] = torch.zeros((), device=self.device)
        return self._get_total_loss(gen_forward=False)

    def _get_visualizations(self, data):
        with torch.no_grad(), self.autocast():
            out = self.net_G(data)
            vis = [data['images_content'], data['images_style'], out['images_recon'],
                   out['images_trans']]
            if self.cfg.trainer.model_average:
                out = self.net_G.module.averaged_model(data)
                vis += [out['images_recon'], out['images_trans']]
            return vis

    def _compute_fid(self):
        if self.val_data_loader is None:
            return None
        self.net_G.eval()
        net = self.net_G.module.averaged_model if self.cfg.trainer.model_average else self.net_G
        dataset = self.val_data_loader.dataset
        num_test_classes = getattr(dataset, 'num_style_classes', 1)
        values = []
        for class_idx in range(num_test_classes):
            fid_path = self._get_save_path(os.path.join('fid', str(class_idx)), 'npy')
            if hasattr(dataset, 'set_sample_class_idx'):
                dataset.set_sample_class_idx(class_idx)
            with self.autocast():
                values.append(compute_fid(fid_path, self.val_data_loader, net, 'images_style',
                                          'images_trans'))
        self.net_G.train()
        if is_master():
            return float(np.mean(values))
        return None
