"""UNIT generator: shared-latent autoencoders (reference generators/unit.py:13-312)."""
import warnings

from torch import nn
# nn.Upsample runs in fp32 under autocast; this one is the bf16 NHWC k12 resize
from imaginaire_amd.ops.resize import Upsample as NearestUpsample

from imaginaire_amd.layers import Conv2dBlock, Res2dBlock


def _kw(cfg):
    return dict(cfg) if isinstance(cfg, dict) else dict(vars(cfg))


class Generator(nn.Module):
    def __init__(self, gen_cfg, data_cfg):
        super().__init__()
        self.autoencoder_a = AutoEncoder(**_kw(gen_cfg))
        self.autoencoder_b = AutoEncoder(**_kw(gen_cfg))

    def forward(self, data, image_recon=True, cycle_recon=True):
        images_a, images_b = data['images_a'], data['images_b']
        out = dict()
        content_a = self.autoencoder_a.content_encoder(images_a)
        content_b = self.autoencoder_b.content_encoder(images_b)
        if image_recon:
            out.update(images_aa=self.autoencoder_a.decoder(content_a),
                       images_bb=self.autoencoder_b.decoder(content_b))
        images_ba = self.autoencoder_a.decoder(content_b)
        images_ab = self.autoencoder_b.decoder(content_a)
        if cycle_recon:
            content_ba = self.autoencoder_a.content_encoder(images_ba)
            content_ab = self.autoencoder_b.content_encoder(images_ab)
            out.update(content_ba=content_ba, content_ab=content_ab,
                       images_aba=self.autoencoder_a.decoder(content_ab),
                       images_bab=self.autoencoder_b.decoder(content_ba))
        out.update(content_a=content_a, content_b=content_b, images_ba=images_ba,
                   images_ab=images_ab)
        return out

    def inference(self, data, a2b=True):
        if a2b:
            input_key, enc, dec = 'images_a', self.autoencoder_a.content_encoder, \
                self.autoencoder_b.decoder
        else:
            input_key, enc, dec = 'images_b', self.autoencoder_b.content_encoder, \
                self.autoencoder_a.decoder
        output_images = dec(enc(data[input_key]))
        return output_images, [_name(data, input_key)]


def _name(data, key):
    k = data.get('key', {})
    entry = k.get(key, k) if isinstance(k, dict) else k
    if isinstance(entry, dict) and 'sequence_name' in entry:
        return '%s/%s' % (entry['sequence_name'][0], entry['filename'][0])
    if isinstance(entry, (list, tuple)):
        return str(entry[0])
    return str(entry)


def _names(data, key):
    """Per-sample output names ``sequence/filename`` for a collated batch."""
    k = data.get('key', {})
    entry = k.get(key, k) if isinstance(k, dict) else k
    if isinstance(entry, dict) and 'sequence_name' in entry:
        return ['%s/%s' % (s, f) for s, f in zip(entry['sequence_name'], entry['filename'])]
    if isinstance(entry, (list, tuple)):
        return [str(e) for e in entry]
    return [str(entry)]


class AutoEncoder(nn.Module):
    def __init__(self, num_filters=64, max_num_filters=256, num_res_blocks=4,
                 num_downsamples_content=2, num_image_channels=3, content_norm_type='instance',
                 decoder_norm_type='instance', weight_norm_type='', output_nonlinearity='',
                 pre_act=False, apply_noise=False, **kwargs):
        super().__init__()
        for key in kwargs:
            if key not in ('type', 'common'):
                warnings.warn("Generator argument '{}' is not used.".format(key))
        self.content_encoder = ContentEncoder(num_downsamples_content, num_res_blocks,
                                              num_image_channels, num_filters, max_num_filters,
                                              'reflect', content_norm_type, weight_norm_type,
                                              'relu', pre_act)
        self.decoder = Decoder(num_downsamples_content, num_res_blocks,
                               self.content_encoder.output_dim, num_image_channels, 'reflect',
                               decoder_norm_type, weight_norm_type, 'relu', output_nonlinearity,
                               pre_act, apply_noise)

    def forward(self, images):
        return self.decoder(self.content_encoder(images))


class ContentEncoder(nn.Module):
    def __init__(self, num_downsamples, num_res_blocks, num_image_channels, num_filters,
                 max_num_filters, padding_mode, activation_norm_type, weight_norm_type,
                 nonlinearity, pre_act=False):
        super().__init__()
        conv_params = dict(padding_mode=padding_mode, activation_norm_type=activation_norm_type,
                           weight_norm_type=weight_norm_type, nonlinearity=nonlinearity)
        if not pre_act or (activation_norm_type != '' and activation_norm_type != 'none'):
            conv_params['inplace_nonlinearity'] = True
        order = 'pre_act' if pre_act else 'CNACNA'
        model = [Conv2dBlock(num_image_channels, num_filters, 7, 1, 3, **conv_params)]
        for _ in range(num_downsamples):
            num_filters_prev = num_filters
            num_filters = min(num_filters * 2, max_num_filters)
            model += [Conv2dBlock(num_filters_prev, num_filters, 4, 2, 1, **conv_params)]
        for _ in range(num_res_blocks):
            model += [Res2dBlock(num_filters, num_filters, **conv_params, order=order)]
        self.model = nn.Sequential(*model)
        self.output_dim = num_filters

    def forward(self, x):
        return self.model(x)


class Decoder(nn.Module):
    def __init__(self, num_upsamples, num_res_blocks, num_filters, num_image_channels,
                 padding_mode, activation_norm_type, weight_norm_type, nonlinearity,
                 output_nonlinearity, pre_act=False, apply_noise=False):
        super().__init__()
        conv_params = dict(padding_mode=padding_mode, nonlinearity=nonlinearity,
                           inplace_nonlinearity=True, apply_noise=apply_noise,
                           weight_norm_type=weight_norm_type,
                           activation_norm_type=activation_norm_type)
        order = 'pre_act' if pre_act else 'CNACNA'
        self.decoder = nn.ModuleList()
        for _ in range(num_res_blocks):
            self.decoder += [Res2dBlock(num_filters, num_filters, **conv_params, order=order)]
        for _ in range(num_upsamples):
            self.decoder += [NearestUpsample(scale_factor=2)]
            self.decoder += [Conv2dBlock(num_filters, num_filters // 2, 5, 1, 2, **conv_params)]
            num_filters //= 2
        self.decoder += [Conv2dBlock(num_filters, num_image_channels, 7, 1, 3,
                                     nonlinearity=output_nonlinearity,
                                     padding_mode=padding_mode)]

    def forward(self, x):
        for block in self.decoder:
            x = block(x)
        return x
