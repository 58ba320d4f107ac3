"""UNIT trainer (reference trainers/unit.py:14-229): GAN + image recon + cycle
recon + perceptual."""
import torch
from torch import nn

from imaginaire_amd.losses.l1 import L1Loss
from imaginaire_amd.losses import GANLoss, PerceptualLoss
from imaginaire_amd.trainers.munit import Trainer as MUNITTrainer, _weights_from


class Trainer(MUNITTrainer):
    def _init_loss(self, cfg):
        self.criteria['gan'] = GANLoss(cfg.trainer.gan_mode)
        self.criteria['image_recon'] = L1Loss()
        self.criteria['cycle_recon'] = L1Loss()
        if getattr(cfg.trainer.loss_weight, 'perceptual', 0) > 0:
            self.criteria['perceptual'] = PerceptualLoss(
                cfg=cfg, network=cfg.trainer.perceptual_mode,
                layers=cfg.trainer.perceptual_layers)
        self.weights.update(_weights_from(cfg.trainer.loss_weight))

    def gen_forward(self, data):
        cycle_recon = 'cycle_recon' in self.weights
        perceptual = 'perceptual' in self.weights
        out = self.net_G(data, cycle_recon=cycle_recon)
        dout = self.net_D(data, out, real=False)
        self._time_before_loss()
        gan = self.criteria['gan']
        self.gen_losses['gan_a'] = gan(dout['out_ba'], True, dis_update=False)
        self.gen_losses['gan_b'] = gan(dout['out_ab'], True, dis_update=False)
        self.gen_losses['gan'] = self.gen_losses['gan_a'] + self.gen_losses['gan_b']
        if perceptual:
            self.gen_losses['perceptual_a'] = self.criteria['perceptual'](out['images_ab'],
                                                                          data['images_a'])
            self.gen_losses['perceptual_b'] = self.criteria['perceptual'](out['images_ba'],
                                                                          data['images_b'])
            self.gen_losses['perceptual'] = self.gen_losses['perceptual_a'] + \
                self.gen_losses['perceptual_b']
        self.gen_losses['image_recon'] = \
            self.criteria['image_recon'](out['images_aa'], data['images_a']) + \
            self.criteria['image_recon'](out['images_bb'], data['images_b'])
        if cycle_recon:
            self.gen_losses['cycle_recon_aba'] = self.criteria['cycle_recon'](
                out['images_aba'], data['images_a'])
            self.gen_losses['cycle_recon_bab'] = self.criteria['cycle_recon'](
                out['images_bab'], data['images_b'])
            self.gen_losses['cycle_recon'] = self.gen_losses['cycle_recon_aba'] + \
                self.gen_losses['cycle_recon_bab']
        return self._get_total_loss(gen_forward=True)

    def dis_forward(self, data):
        with torch.no_grad():
            out = self.net_G(data, image_recon=False, cycle_recon=False)
        out['images_ba'].requires_grad = True
        out['images_ab'].requires_grad = True
        dout = self.net_D(data, out)
        self._time_before_loss()
        gan = self.criteria['gan']
        self.dis_losses['gan_a'] = gan(dout['out_a'], True) + gan(dout['out_ba'], False)
        self.dis_losses['gan_b'] = gan(dout['out_b'], True) + gan(dout['out_ab'], False)
        self.dis_losses['gan'] = self.dis_losses['gan_a'] + self.dis_losses['gan_b']
        return self._get_total_loss(gen_forward=False)

    def _get_visualizations(self, data):
        net = self.net_G.module.averaged_model if self.cfg.trainer.model_average else self.net_G
        with torch.no_grad(), self.autocast():
            out = net(data)
            return [data['images_a'], data['images_b'], out['images_aa'], out['images_bb'],
                    out['images_ab'], out['images_ba'], out['images_aba'], out['images_bab']]
