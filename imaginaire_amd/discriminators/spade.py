"""SPADE discriminator: PatchGAN pyramid + FPSE (reference discriminators/spade.py:15-117).

In the D update real and fake are run as ONE batched forward (concatenated
along the batch axis) instead of two separate passes: the same network math (no
batch-coupled layers, activation_norm_type is 'none'), half the kernel launches
and twice the parallelism per conv. In the G update (gradient flows through the
fake branch only) the passes stay separate so the backward skips the real half.

``dis.batch_real_fake`` (default True) selects this. The reference's two sequential passes
run two spectral-norm power iterations per D call (the fake pass sees the σ refreshed by the
real pass, reference discriminators/spade.py:91-117); the batched D update runs the same two
iterations back to back before its one forward (``extra_sn_power_iteration``), so u / v evolve
exactly as in the reference and the only difference is that the real half is normalised by
the second σ instead of the first (bounded in tests/test_spade_dis_semantics_cpu.py).
``batch_real_fake: False`` restores the reference order exactly.
"""
import torch
import torch.nn as nn

from imaginaire_amd.discriminators.fpse import FPSEDiscriminator
from imaginaire_amd.ops.conv import mark_zero_tail
from imaginaire_amd.ops.resize import interpolate
from imaginaire_amd.discriminators.multires_patch import NLayerPatchDiscriminator
from imaginaire_amd.layers.spectral_norm import (extra_sn_power_iteration,
                                                 refresh_batched_spectral_norm)
from imaginaire_amd.ops import _ext
from imaginaire_amd.registry import canonical_module_name
from imaginaire_amd.utils.data import (get_paired_input_image_channel_number,
                                       get_paired_input_label_channel_number)


class _PatchInput(torch.autograd.Function):
    """``cat(label, image)`` of each (real / fake) half written into one zero-tailed,
    channel-padded NHWC buffer. The backward hands each input its channel slice of the
    gradient as a view: slice-assignment autograd (CopySlices) would first clone the whole
    [2B, 192, H, W] gradient (~200 MB per D call at 256 x 512, profiles/spade_step_op_sites_r3)."""

    @staticmethod
    def forward(ctx, cl, c, cp, npairs, *tensors):
        labels, images = tensors[:npairs], tensors[npairs:]
        lab, img = labels[0], images[0]
        n = [lb.shape[0] for lb in labels]
        dtype = img.dtype if img.is_floating_point() else lab.dtype
        out = torch.empty((sum(n), cp) + tuple(lab.shape[2:]), dtype=dtype, device=lab.device,
                          memory_format=torch.channels_last)
        o = 0
        native = out.is_cuda and _ext.use_native(out)
        for lb, im, k in zip(labels, images, n):
            if native:
                # one pass per half (label | image | zero tail) on the HIP concat kernel
                _ext.ext().nhwc_concat_into(
                    out[o:o + k], lb.to(dtype).contiguous(memory_format=torch.channels_last),
                    im.to(dtype).contiguous(memory_format=torch.channels_last))
            else:
                out[o:o + k, :cl] = lb
                out[o:o + k, cl:c] = im
            o += k
        if cp > c and not native:
            out[:, c:].zero_()
        ctx.conf = (cl, c, n, [t.dtype for t in tensors])
        return out

    @staticmethod
    def backward(ctx, grad):
        cl, c, n, dtypes = ctx.conf
        npairs = len(n)
        grads = []
        o = 0
        offs = []
        for k in n:
            offs.append(o)
            o += k
        for i in range(npairs):  # labels
            need = ctx.needs_input_grad[4 + i]
            grads.append(grad[offs[i]:offs[i] + n[i], :cl].to(dtypes[i]) if need else None)
        for i in range(npairs):  # images
            need = ctx.needs_input_grad[4 + npairs + i]
            grads.append(grad[offs[i]:offs[i] + n[i], cl:c].to(dtypes[npairs + i])
                         if need else None)
        return (None, None, None, None) + tuple(grads)


class Discriminator(nn.Module):
    def __init__(self, dis_cfg, data_cfg):
        super().__init__()
        image_channels = get_paired_input_image_channel_number(data_cfg)
        if canonical_module_name(data_cfg.type) == 'imaginaire_amd.datasets.paired_videos':
            num_labels = get_paired_input_label_channel_number(data_cfg, video=True)
        else:
            num_labels = get_paired_input_label_channel_number(data_cfg)
        kernel_size = getattr(dis_cfg, 'kernel_size', 3)
        num_filters = getattr(dis_cfg, 'num_filters', 128)
        max_num_filters = getattr(dis_cfg, 'max_num_filters', 512)
        num_discriminators = getattr(dis_cfg, 'num_discriminators', 2)
        num_layers = getattr(dis_cfg, 'num_layers', 5)
        activation_norm_type = getattr(dis_cfg, 'activation_norm_type', 'none')
        weight_norm_type = getattr(dis_cfg, 'weight_norm_type', 'spectral')
        num_input_channels = image_channels + num_labels
        self.batched = getattr(dis_cfg, 'batch_real_fake', True) and \
            activation_norm_type in ('none', '', 'instance') and \
            getattr(dis_cfg, 'fpse_activation_norm_type', 'none') in ('none', '', 'instance')
        self.discriminators = nn.ModuleList()
        for _ in range(num_discriminators):
            self.discriminators.append(NLayerPatchDiscriminator(
                kernel_size, num_input_channels, num_filters, num_layers, max_num_filters,
                activation_norm_type, weight_norm_type))
        fpse_kernel_size = getattr(dis_cfg, 'fpse_kernel_size', 3)
        fpse_activation_norm_type = getattr(dis_cfg, 'fpse_activation_norm_type', 'none')
        self.fpse_discriminator = FPSEDiscriminator(image_channels, num_labels, num_filters,
                                                    fpse_kernel_size, weight_norm_type,
                                                    fpse_activation_norm_type)

    @staticmethod
    def _patch_input(labels, images):
        """The PatchGAN input ``cat(label, image)`` (reference discriminators/spade.py:73-77)
        written ONCE into a channel-padded NHWC buffer (188 -> 192 channels on the COCO-Stuff
        recipe, zero tail): the convs and the bilinear pyramid consume it without the
        concat + pad copies; ``labels`` / ``images`` are lists (real and fake halves) stacked
        along the batch."""
        lab, img = labels[0], images[0]
        cl, ci = lab.shape[1], img.shape[1]
        c = cl + ci
        if not (lab.is_cuda and lab.dim() == 4):
            return torch.cat([torch.cat((lb, im), 1) for lb, im in zip(labels, images)], 0)
        cp = (c + 7) // 8 * 8 if c <= 64 else (c + 31) // 32 * 32
        out = _PatchInput.apply(cl, c, cp, len(labels), *labels, *images)
        if cp > c:
            mark_zero_tail(out, c)
        return out

    def _single_forward(self, input_label, input_image, input_x=None, seg_repeat=1):
        if input_x is None:
            input_x = self._patch_input([input_label], [input_image])
        features_list = []
        pred2, pred3, pred4 = self.fpse_discriminator(input_image, input_label, seg_repeat)
        output_list = [pred2, pred3, pred4]
        input_downsampled = input_x
        for net_discriminator in self.discriminators:
            output, features = net_discriminator(input_downsampled)
            output_list.append(output)
            features_list.append(features)
            input_downsampled = interpolate(
                input_downsampled, scale_factor=0.5, mode='bilinear', align_corners=True)
        return output_list, features_list

    def forward(self, data, net_G_output):
        output_x = dict()
        real, fake = data['images'], net_G_output['fake_images']
        # Batch real+fake only in the D update (fake detached; D weights need grads from both
        # halves). In the G update the real branch needs no backward at all: batched, the
        # conv backward would still compute it for the real half (~half of D's data-gradient
        # work), so the two passes run separately there, as in the reference.
        grad_through_fake = torch.is_grad_enabled() and fake.requires_grad
        if self.batched and real.shape == fake.shape and not grad_through_fake:
            # the reference's two sequential passes take two spectral-norm power iterations per
            # D call: run the second one now, so both halves see the refreshed σ and u / v
            # advance exactly as in the reference (dis.batch_real_fake=False: reference order)
            extra_sn_power_iteration(self)
            n = real.shape[0]
            fake = fake.to(real.dtype)
            images = torch.cat([real, fake], 0)
            label = data['label']
            # the label of both halves is the same tensor: FPSE embeds it once (seg_repeat)
            outs, feats = self._single_forward(
                label, images, input_x=self._patch_input([label, label], [real, fake]),
                seg_repeat=2)
            output_x['real_outputs'] = [o[:n] for o in outs]
            output_x['fake_outputs'] = [o[n:] for o in outs]
            output_x['real_features'] = [[f[:n] for f in fl] for fl in feats]
            output_x['fake_features'] = [[f[n:] for f in fl] for fl in feats]
            return output_x
        output_x['real_outputs'], output_x['real_features'] = \
            self._single_forward(data['label'], real)
        # second spectral-norm power iteration of this forward (the reference's fake pass
        # refreshes u, v, σ of every layer): one batched k5b pass instead of per-layer fallbacks
        refresh_batched_spectral_norm(self)
        output_x['fake_outputs'], output_x['fake_features'] = \
            self._single_forward(data['label'], fake)
        return output_x
