"""GAN objectives (reference losses/gan.py:12-132): non_saturated, least_square,
hinge (D uses the fused ``-mean(min(±x-1, 0))`` form), wasserstein; lists of
multi-scale outputs are averaged. On the GPU a whole list of discriminator outputs is one
multi-tensor k13b launch (``ops/loss.py: gan_loss_multi``) instead of per-output
relu / mean / neg kernels."""
import torch
import torch.nn as nn
import torch.nn.functional as F

from imaginaire_amd.ops import loss as loss_ops


def fuse_math_min_mean_pos(x):
    """-mean(min(x-1, 0)) == mean(relu(1-x))."""
    return F.relu(1 - x).float().mean()


def fuse_math_min_mean_neg(x):
    """-mean(min(-x-1, 0)) == mean(relu(1+x))."""
    return F.relu(1 + x).float().mean()


class GANLoss(nn.Module):
    def __init__(self, gan_mode, target_real_label=1.0, target_fake_label=0.0):
        super().__init__()
        self.real_label = target_real_label
        self.fake_label = target_fake_label
        self.gan_mode = gan_mode

    def forward(self, dis_output, t_real, dis_update=True):
        if isinstance(dis_output, list) and dis_output and \
                all(isinstance(d, torch.Tensor) for d in dis_output):
            if not dis_update:
                assert t_real, "The target should be real when updating the generator."
            kind, a, b = self._phi(t_real, dis_update)
            return loss_ops.gan_loss_multi(dis_output, kind, a, b, 1.0 / len(dis_output))
        if isinstance(dis_output, list):
            loss = 0
            for dis_output_i in dis_output:
                assert isinstance(dis_output_i, torch.Tensor)
                loss = loss + self.loss(dis_output_i, t_real, dis_update)
            return loss / len(dis_output)
        return self.loss(dis_output, t_real, dis_update)

    def loss(self, dis_output, t_real, dis_update=True):
        if not dis_update:
            assert t_real, "The target should be real when updating the generator."
        if self.gan_mode == 'non_saturated':
            target = self.get_target_tensor(dis_output, t_real)
            return F.binary_cross_entropy_with_logits(dis_output.float(), target)
        if self.gan_mode == 'least_square':
            target = self.get_target_tensor(dis_output, t_real)
            return 0.5 * F.mse_loss(dis_output.float(), target)
        if self.gan_mode == 'hinge':
            if dis_update:
                return fuse_math_min_mean_pos(dis_output) if t_real else \
                    fuse_math_min_mean_neg(dis_output)
            return -torch.mean(dis_output.float())
        if self.gan_mode == 'wasserstein':
            return -torch.mean(dis_output.float()) if t_real else torch.mean(dis_output.float())
        raise ValueError('Unexpected gan_mode {}'.format(self.gan_mode))

    def _phi(self, t_real, dis_update):
        """(kind, a, b) of the k13b loss for this mode / target (ops/loss.py)."""
        if self.gan_mode == 'non_saturated':
            return loss_ops.GAN_BCE, self.real_label if t_real else self.fake_label, 1.0
        if self.gan_mode == 'least_square':
            return loss_ops.GAN_LSQ, self.real_label if t_real else self.fake_label, 1.0
        if self.gan_mode == 'hinge':
            if dis_update:
                return loss_ops.GAN_RELU, 1.0, -1.0 if t_real else 1.0
            return loss_ops.GAN_LINEAR, 0.0, -1.0
        if self.gan_mode == 'wasserstein':
            return loss_ops.GAN_LINEAR, 0.0, -1.0 if t_real else 1.0
        raise ValueError('Unexpected gan_mode {}'.format(self.gan_mode))

    def get_target_tensor(self, dis_output, t_real):
        value = self.real_label if t_real else self.fake_label
        return torch.full_like(dis_output, value, dtype=torch.float32)
