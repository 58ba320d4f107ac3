"""World-consistent vid2vid generator (reference generators/wc_vid2vid.py:19-359).

vid2vid plus (a) an optional frozen single-image SPADE model that renders
the first frame, (b) externally supplied flow + occlusion mask
(``data['flow']`` / ``data['mask']`` — the fork's data contract, SURVEY
Appendix A) instead of a learned temporal flow network, and (c) guidance
images splatted from the accumulated 3-D point cloud (device-resident
``SplatRenderer``) fed to SPADE as an extra (optionally partial-conv)
condition.

The fork forces ``unprojection = None`` (guidance off); here guidance is
used whenever the data carries unprojections and ``gen.guidance.enabled`` is
not false — with the fork's configs (no unprojections in the data) the
behaviour is identical.
"""
import numpy as np
import torch
import torch.nn.functional as F

from imaginaire_amd.generators.vid2vid import Generator as Vid2VidGenerator
from imaginaire_amd.model_utils.fs_vid2vid import resample
from imaginaire_amd.model_utils.wc_vid2vid.render import SplatRenderer
from imaginaire_amd.utils.visualization import tensor2im


class Generator(Vid2VidGenerator):
    _use_learned_flow = False  # flow comes from the data (fork contract)

    def __init__(self, gen_cfg, data_cfg):
        self.guidance_cfg = gen_cfg.guidance
        self.guidance_only_with_flow = getattr(self.guidance_cfg, 'only_with_flow', False)
        self.guidance_partial_conv = getattr(self.guidance_cfg, 'partial_conv', False)
        self.guidance_enabled = getattr(self.guidance_cfg, 'enabled', True)
        super().__init__(gen_cfg, data_cfg)
        self.renderer = SplatRenderer()
        self.reset_renderer()
        self.single_image_model = None
        self.single_image_model_z = None

    def _init_single_image_model(self, load_weights=True, locrank=0):
        if self.single_image_model is None and hasattr(self.gen_cfg, 'single_image_model'):
            from imaginaire_amd.config import Config
            from imaginaire_amd.utils.trainer import (get_model_optimizer_and_scheduler,
                                                      get_trainer)
            print('Using single image model...')
            cfg = Config(self.gen_cfg.single_image_model.config)
            if not hasattr(cfg, 'local_rank'):
                cfg.local_rank = locrank
            net_G, net_D, opt_G, opt_D, sch_G, sch_D = get_model_optimizer_and_scheduler(cfg)
            trainer = get_trainer(cfg, net_G, net_D, opt_G, opt_D, sch_G, sch_D, None, None)
            if load_weights:
                trainer.load_checkpoint(cfg, self.gen_cfg.single_image_model.checkpoint)
            m = net_G.module
            self.single_image_model = m.module if hasattr(m, 'averaged_model') else m
            self.single_image_model_z = None

    def reset_renderer(self, is_flipped_input=False):
        self.renderer.reset()
        self.is_flipped_input = bool(is_flipped_input[0]) if isinstance(
            is_flipped_input, (list, tuple, torch.Tensor)) else bool(is_flipped_input)
        self.renderer_num_forwards = 0
        self.single_image_model_z = None

    def renderer_update_point_cloud(self, image, point_info):
        if point_info is None or len(point_info) == 0:
            return
        if isinstance(image, torch.Tensor):
            image = tensor2im(image.detach())[0]
        if self.is_flipped_input:
            image = np.fliplr(image).copy()
        self.renderer.update_point_cloud(image, point_info)
        self.renderer_num_forwards += 1

    def get_guidance_images_and_masks(self, unprojection, device):
        resolution = 'w1024xh512'
        point_info = unprojection[resolution]
        w, h = [int(v[1:]) for v in resolution.split('x')]
        image, mask = self.renderer.render_image(point_info, w, h, return_mask=True)
        if self.is_flipped_input:
            image, mask = np.fliplr(image).copy(), np.fliplr(mask).copy()
        image = torch.from_numpy(image).permute(2, 0, 1).float().div(255).sub(0.5).mul(2)
        mask = torch.from_numpy(mask).permute(2, 0, 1).float().div(255)
        guidance = torch.cat((image, mask), dim=0).unsqueeze(0).to(device)
        return guidance, point_info

    def forward(self, data):
        self._init_single_image_model()
        label = data['label']
        unprojection = data.get('unprojection') if self.guidance_enabled else None
        label_prev, img_prev = data['prev_labels'], data['prev_images']
        is_first_frame = img_prev is None
        z = data.get('z')
        bs, _, h, w = label.size()
        flow = mask = img_warp = None
        warp_prev = self.temporal_initialized and not is_first_frame and \
            label_prev.shape[1] == self.num_frames_G - 1
        guidance, point_info = None, None
        if unprojection is not None:
            guidance, point_info = self.get_guidance_images_and_masks(unprojection, label.device)
        cond_maps_now = self.get_cond_maps(label, self.label_embedding)

        if self.single_image_model is not None and not warp_prev:
            if self.single_image_model_z is None:
                self.single_image_model_z = torch.randn(
                    bs, self.single_image_model.style_dims, device=label.device,
                    dtype=label.dtype)
            data['z'] = self.single_image_model_z
            self.single_image_model.eval()
            with torch.no_grad():
                img_final = self.single_image_model.spade_generator(data)['fake_images']
            img_final = img_final.detach()
            source = 'pretrained'
        else:
            if is_first_frame:
                x_img = self._first_frame_code(label, z, bs, cond_maps_now)
            else:
                x_img = self._encode_prev(img_prev, label_prev, cond_maps_now)
            if warp_prev:
                flow, mask = data['flow'], data['mask']
                img_warp = resample(img_prev[:, -1], flow)
                if self.spade_combine:
                    cond_maps_img = self.get_cond_maps(torch.cat([img_warp, mask], dim=1),
                                                       self.img_prev_embedding)
            for i in range(self.num_downsamples_img, -1, -1):
                j = min(i, self.num_downsamples_embed)
                cond_maps = list(cond_maps_now[j])
                if warp_prev:
                    if i < self.num_multi_spade_layers:
                        cond_maps += cond_maps_img[j]
                        cond_maps += [guidance]
                    elif not self.guidance_only_with_flow:
                        cond_maps += [guidance]
                x_img = self.one_up_conv_layer(x_img, cond_maps, i)
            img_final = torch.tanh(self.conv_img(x_img))
            source = 'in_training'
        self.renderer_update_point_cloud(img_final, point_info)
        return dict(fake_images=img_final, fake_flow_maps=flow, fake_occlusion_masks=mask,
                    fake_raw_images=None, warped_images=img_warp,
                    guidance_images_and_masks=guidance, fake_images_source=source)

    def _guidance_dims(self):
        return [3 if self.guidance_partial_conv else 4]

    def get_cond_dims(self, num_downs=0):
        if not self.use_embed:
            return [self.num_input_channels]
        num_filters = getattr(self.emb_cfg, 'num_filters', 32)
        num_downs = min(num_downs, self.num_downsamples_embed)
        ch = [min(self.max_num_filters, num_filters * (2 ** num_downs))]
        if num_downs < self.num_multi_spade_layers:
            ch = ch * 2 + self._guidance_dims()
        elif not self.guidance_only_with_flow:
            ch = ch + self._guidance_dims()
        return ch

    def get_partial(self, num_downs=0):
        partial = [False]
        if num_downs < self.num_multi_spade_layers:
            partial = partial * 2 + [self.guidance_partial_conv]
        elif not self.guidance_only_with_flow:
            partial = partial + [self.guidance_partial_conv]
        return partial
