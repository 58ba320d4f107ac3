"""MUNIT discriminator: per-domain multi-res patch (or residual) D
(reference discriminators/munit.py:11-99).

The reference runs each domain's discriminator once per image set (translated fake, real,
reconstruction). In the D update, where every set feeds the same weight gradients, the sets of
a domain run as ONE batch-concatenated pass (no batch-coupled layers: activation norm 'none' /
'instance'), as do the G update's translated + reconstructed fakes when ``gan_recon`` is on.
Spectral norm: the power iterations of the skipped passes run back to back first
(``extra_sn_power_iteration``), so u / v advance exactly as in the reference; each set is
normalised by the last σ (see discriminators/spade.py). ``dis.batch_real_fake: False``
restores the reference passes.
"""
import os

import torch
from torch import nn

from imaginaire_amd.discriminators.multires_patch import MultiResPatchDiscriminator
from imaginaire_amd.discriminators.residual import ResDiscriminator
from imaginaire_amd.layers.spectral_norm import extra_sn_power_iteration


def _kw(cfg):
    d = dict(cfg) if isinstance(cfg, dict) else dict(vars(cfg))
    d.pop('common', None)
    return d


class Discriminator(nn.Module):
    def __init__(self, dis_cfg, data_cfg):
        super().__init__()
        kw = _kw(dis_cfg)
        # (IMAGINAIRE_AMD_DIS_BATCH=0: A/B switch to the reference passes)
        self.batched = bool(kw.pop('batch_real_fake', True)) and \
            os.environ.get('IMAGINAIRE_AMD_DIS_BATCH', '1') != '0' and \
            kw.get('activation_norm_type', 'none') in ('none', '', 'instance', None)
        if getattr(dis_cfg, 'patch_wise', True):
            self.discriminator_a = MultiResPatchDiscriminator(**kw)
            self.discriminator_b = MultiResPatchDiscriminator(**kw)
        else:
            self.discriminator_a = ResDiscriminator(**kw)
            self.discriminator_b = ResDiscriminator(**kw)

    def _batched_forward(self, sets_a, sets_b):
        """(out, features) of every image set of each domain, each domain's sets run as one
        batch-concatenated pass; None when the sets do not qualify."""
        shapes = {tuple(t.shape) for t in sets_a + sets_b}
        if len(sets_a) < 2 or len(sets_a) != len(sets_b) or len(shapes) != 1:
            return None
        for _ in range(len(sets_a) - 1):  # one per pass saved: see the module docstring
            extra_sn_power_iteration(self)
        n = sets_a[0].shape[0]

        def take(x, i):
            if torch.is_tensor(x):
                return x[i * n:(i + 1) * n]
            if isinstance(x, (list, tuple)):
                return [take(e, i) for e in x]
            return x

        res = []
        for net, sets in ((self.discriminator_a, sets_a), (self.discriminator_b, sets_b)):
            dt = sets[0].dtype
            out, fea, _ = net(torch.cat([t.to(dt) for t in sets], 0))
            res.append([(take(out, i), take(fea, i)) for i in range(len(sets))])
        return res

    def forward(self, data, net_G_output, gan_recon=False, real=True):
        if self.batched:
            # a: fake ba, real a, recon aa; b: fake ab, real b, recon bb
            ka, kb = ['ba'], ['ab']
            sa, sb = [net_G_output['images_ba']], [net_G_output['images_ab']]
            if real:
                ka.append('a')
                kb.append('b')
                sa.append(data['images_a'])
                sb.append(data['images_b'])
            if gan_recon:
                ka.append('aa')
                kb.append('bb')
                sa.append(net_G_output['images_aa'])
                sb.append(net_G_output['images_bb'])
            res = self._batched_forward(sa, sb)
            if res is not None:
                output = {}
                for keys, rs in zip((ka, kb), res):
                    for k, (o, f) in zip(keys, rs):
                        output['out_' + k] = o
                        output['fea_' + k] = f
                return output
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
