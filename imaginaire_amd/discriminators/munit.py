"""MUNIT discriminator: per-domain multi-res patch (or residual) D
(reference discriminators/munit.py:11-99)."""
from torch import nn

from imaginaire_amd.discriminators.multires_patch import MultiResPatchDiscriminator
from imaginaire_amd.discriminators.residual import ResDiscriminator


def _kw(cfg):
    d = dict(cfg) if isinstance(cfg, dict) else dict(vars(cfg))
    d.pop('common', None)
    return d


class Discriminator(nn.Module):
    def __init__(self, dis_cfg, data_cfg):
        super().__init__()
        if getattr(dis_cfg, 'patch_wise', True):
            self.discriminator_a = MultiResPatchDiscriminator(**_kw(dis_cfg))
            self.discriminator_b = MultiResPatchDiscriminator(**_kw(dis_cfg))
        else:
            self.discriminator_a = ResDiscriminator(**_kw(dis_cfg))
            self.discriminator_b = ResDiscriminator(**_kw(dis_cfg))

    def forward(self, data, net_G_output, gan_recon=False, real=True):
        out_ab, fea_ab, _ = self.discriminator_b(net_G_output['images_ab'])
        out_ba, fea_ba, _ = self.discriminator_a(net_G_output['images_ba'])
        output = dict(out_ba=out_ba, out_ab=out_ab, fea_ba=fea_ba, fea_ab=fea_ab)
        if real:
            out_a, fea_a, _ = self.discriminator_a(data['images_a'])
            out_b, fea_b, _ = self.discriminator_b(data['images_b'])
            output.update(dict(out_a=out_a, out_b=out_b, fea_a=fea_a, fea_b=fea_b))
        if gan_recon:
            out_aa, fea_aa, _ = self.discriminator_a(net_G_output['images_aa'])
            out_bb, fea_bb, _ = self.discriminator_b(net_G_output['images_bb'])
            output.update(dict(out_aa=out_aa, out_bb=out_bb, fea_aa=fea_aa, fea_bb=fea_bb))
        return output
