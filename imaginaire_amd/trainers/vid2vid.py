"""vid2vid trainer (reference trainers/vid2vid.py:30-882).

Per iteration the trainer walks the sequence frame by frame: for each t it
builds ``data_t`` (current label/image + the last num_frames_G-1 labels and
*generated* frames), runs G, updates D on the detached output, then updates
G against the fresh D (image GAN + feature matching + multi-scale
perceptual + optional L1 + flow + temporal GAN over frame windows).
``single_frame_epoch`` / ``num_epochs_temporal_step`` grow the sequence
length exactly like the reference.

MI355X specifics: bf16 autocast instead of apex AMP; the per-frame D and G
backward passes go through the bucketed RCCL DDP (begin/finish per phase);
flow GT comes from the FlowNet2 stack on the k6/k7/k8 HIP kernels.

Flow loss: with ``cfg.flow_network`` the upstream FlowNet2 ``FlowLoss``
(Flow_L1 / Flow_Warp / Flow_Mask) is used; without it, the fork's variant —
masked L1 between the output and the warped previous output under
``data_t['mask']`` (trainers/vid2vid.py:149-153, 513-519).
"""
import os

import numpy as np
import torch

from imaginaire_amd.losses.l1 import L1Loss
from imaginaire_amd.evaluation.fid import compute_fid
from imaginaire_amd.losses import FeatureMatchingLoss, GANLoss, MaskedL1Loss, PerceptualLoss
from imaginaire_amd.model_utils.fs_vid2vid import (concat_frames, detach, get_fg_mask,
                                                   pre_process_densepose, resample)
from imaginaire_amd.trainers.base import BaseTrainer, _ddp_call
from imaginaire_amd.utils.distributed import is_master
from imaginaire_amd.utils.distributed import master_only_print as print
from imaginaire_amd.utils.meters import Meter
from imaginaire_amd.utils.misc import get_nested_attr, requires_grad, split_labels
from imaginaire_amd.utils.visualization import tensor2flow, tensor2im, tensor2label


def _imwrite(path, image):
    from PIL import Image
    os.makedirs(os.path.dirname(path) or '.', exist_ok=True)
    Image.fromarray(np.asarray(image)).save(path)


def _save_video(path, frames, fps):
    """mp4 via imageio when available, else a directory of frames."""
    try:
        import imageio
        imageio.mimsave(path, frames, fps=fps)
    except Exception:  # noqa: BLE001 (imageio/ffmpeg absent)
        root = os.path.splitext(path)[0] + '_frames'
        for i, f in enumerate(frames):
            _imwrite(os.path.join(root, '%04d.jpg' % i), f)


class Trainer(BaseTrainer):
    # one training iteration = the whole per-frame D / G update loop over the sequence: replayed
    # from one hipGraph per sequence length (captured again when the length changes, as the
    # batch shape does; tests/test_graph_families_gpu.py)
    graph_capturable = True

    @classmethod
    def rank_uniform(cls, cfg):
        """Rank-uniform unless the config adds the data-dependent discriminators: the
        reference's ``additional_discriminators`` (the pose recipes' hand / face crops,
        reference discriminators/fs_vid2vid.py:58-150) run only on batches whose labels hold
        that part, so ranks can differ in which D parameters get gradients. Without them every
        rank calls the same networks on every frame (the temporal D / flow nets follow the
        sequence length, which the epoch schedule sets identically on all ranks): DDP uses the
        rank-local unused mask and the multi-rank step is captured."""
        dis = getattr(cfg, 'dis', None)
        return getattr(dis, 'additional_discriminators', None) is None

    def __init__(self, cfg, net_G, net_D, opt_G, opt_D, sch_G, sch_D, train_data_loader,
                 val_data_loader):
        super().__init__(cfg, net_G, net_D, opt_G, opt_D, sch_G, sch_D, train_data_loader,
                         val_data_loader)
        self.sample_size = (getattr(cfg.trainer, 'num_videos_to_test', 64),
                            getattr(cfg.trainer, 'num_frames_per_video', 10))
        self.sequence_length = 1
        if not self.is_inference:
            self.train_dataset = self.train_data_loader.dataset
            self.sequence_length_max = min(getattr(cfg.data.train, 'max_sequence_length', 100),
                                           self.train_dataset.sequence_length_max)
        self.has_fg = getattr(cfg.data, 'has_foreground', False)
        self.net_G_output = self.data_prev = None

    # ----------------------------------------------------------------- losses
    def _assign_criteria(self, name, criterion, weight):
        self.criteria[name] = criterion
        self.weights[name] = weight

    def _init_loss(self, cfg):
        tcfg = cfg.trainer
        lw = tcfg.loss_weight
        self._assign_criteria('GAN', GANLoss(tcfg.gan_mode), lw.gan)
        self._assign_criteria('FeatureMatching', FeatureMatchingLoss(), lw.feature_matching)
        pl = tcfg.perceptual_loss
        self._assign_criteria('Perceptual', PerceptualLoss(
            cfg=cfg, network=pl.mode, layers=pl.layers, weights=pl.weights,
            num_scales=getattr(pl, 'num_scales', 1)), lw.perceptual)
        if getattr(lw, 'L1', 0) > 0:
            self._assign_criteria('L1', L1Loss(), lw.L1)
        self.add_dis_cfg = getattr(cfg.dis, 'additional_discriminators', None)
        if self.add_dis_cfg is not None:
            for name in self.add_dis_cfg:
                self.weights['GAN_' + name] = self.add_dis_cfg[name].loss_weight
                self.weights['FeatureMatching_' + name] = lw.feature_matching
        self.num_temporal_scales = get_nested_attr(cfg.dis, 'temporal.num_scales', 0)
        for s in range(self.num_temporal_scales):
            self.weights['GAN_T%d' % s] = lw.temporal_gan
            self.weights['FeatureMatching_T%d' % s] = lw.feature_matching
        self.use_flow = hasattr(cfg.gen, 'flow')
        self.flow_mode = None
        if self.use_flow:
            self.flow_mode = getattr(tcfg, 'flow_loss', 'flownet' if hasattr(cfg, 'flow_network')
                                     else 'masked_l1')
            if self.flow_mode == 'flownet':
                from imaginaire_amd.losses.flow import FlowLoss
                self.criteria['Flow'] = FlowLoss(cfg)
            else:
                self.criteria['Flow'] = MaskedL1Loss()
            self.weights['Flow'] = self.weights['Flow_L1'] = self.weights['Flow_Warp'] = \
                self.weights['Flow_Mask'] = lw.flow
        self._define_custom_losses()

    def _define_custom_losses(self):
        pass

    # -------------------------------------------------------- epoch schedule
    def _start_of_epoch(self, current_epoch):
        cfg = self.cfg
        if current_epoch < cfg.single_frame_epoch:
            self.train_dataset.sequence_length = 1
        elif current_epoch == cfg.single_frame_epoch:
            self.init_temporal_network()
        temp_epoch = current_epoch - cfg.single_frame_epoch
        if temp_epoch > 0:
            seq = cfg.data.train.initial_sequence_length * \
                (2 ** (temp_epoch // cfg.num_epochs_temporal_step))
            seq = min(seq, self.sequence_length_max)
            if seq > self.sequence_length:
                self.sequence_length = seq
                self.train_dataset.set_sequence_length(seq)
                print('------- Updating sequence length to %d -------' % seq)

    def init_temporal_network(self):
        self.tensorboard_init = False
        self.sequence_length = self.cfg.data.train.initial_sequence_length
        if not self.is_inference:
            self.train_dataset.set_sequence_length(self.sequence_length)
            print('------ Now start training %d frames -------' % self.sequence_length)

    def _start_of_iteration(self, data, current_iteration):
        data = self.pre_process(data)
        if self.amp_dtype is not None and not self.is_inference:
            # the label maps feed only bf16 convs: cast once per sequence instead of per conv
            # and per frame. The real frames stay fp32: they are also the L1 / warp /
            # perceptual targets and FlowNet2's ground-truth input (reference precision);
            # autocast casts them where they enter a conv.
            for key in ('label', 'few_shot_label'):
                v = data.get(key)
                if torch.is_tensor(v) and v.is_floating_point():
                    data[key] = v.to(self.amp_dtype)
        return data

    def pre_process(self, data):
        data_cfg = self.cfg.data
        if hasattr(data_cfg, 'for_pose_dataset') and \
                'pose_maps-densepose' in data_cfg.input_labels:
            data['label'] = pre_process_densepose(data_cfg.for_pose_dataset, data['label'],
                                                  self.is_inference)
        return data

    def post_process(self, data, net_G_output):
        return data, net_G_output

    # ------------------------------------------------------------- updates
    def gen_update(self, data):
        """One pass over the sequence with interleaved per-frame D and G steps."""
        reuse = getattr(self.cfg.trainer, 'reuse_gen_output', True)
        past_frames = [None, None]
        net_G_output = None
        data_prev = None
        for t in range(self.sequence_length):
            data_t = self.get_data_t(data, net_G_output, data_prev, t)
            data_prev = data_t
            with self.autocast():
                if reuse:
                    net_G_output = self.net_G(data_t)
                else:
                    with torch.no_grad():
                        net_G_output = self.net_G(data_t)
                data_t, net_G_output = self.post_process(data_t, net_G_output)
            net_G_output.setdefault('fake_images_source', 'in_training')
            if net_G_output['fake_images_source'] != 'pretrained':
                requires_grad(self.net_D, True)
                with self.autocast():
                    net_D_output, _ = self.net_D(data_t, detach(net_G_output), past_frames)
                self.get_dis_losses(net_D_output)
            if not reuse:
                with self.autocast():
                    net_G_output = self.net_G(data_t)
                    data_t, net_G_output = self.post_process(data_t, net_G_output)
                net_G_output.setdefault('fake_images_source', 'in_training')
            if net_G_output['fake_images_source'] != 'pretrained':
                requires_grad(self.net_D, False)
                with self.autocast():
                    net_D_output, past_frames = self.net_D(data_t, net_G_output, past_frames)
                self.get_gen_losses(data_t, net_G_output, net_D_output)
        if self.cfg.trainer.model_average:
            self.net_G.module.update_average()
        self._detach_losses()

    def dis_update(self, data):
        """D is updated inside ``gen_update`` frame by frame (reference behaviour)."""

    def _step(self, total_loss, net, opt):
        _ddp_call(net, 'begin')
        total_loss.backward()
        _ddp_call(net, 'finish')
        opt.step()

    def get_gen_losses(self, data_t, net_G_output, net_D_output):
        self.opt_G.zero_grad(set_to_none=True)
        with self.autocast():
            self.gen_losses['GAN'], self.gen_losses['FeatureMatching'] = \
                self.compute_GAN_losses(net_D_output['indv'], dis_update=False)
            self.gen_losses['Perceptual'] = self.criteria['Perceptual'](
                net_G_output['fake_images'], data_t['image'])
            if getattr(self.cfg.trainer.loss_weight, 'L1', 0) > 0:
                self.gen_losses['L1'] = self.criteria['L1'](net_G_output['fake_images'],
                                                            data_t['image'])
            if 'raw' in net_D_output:
                raw_gan, raw_fm = self.compute_GAN_losses(net_D_output['raw'], dis_update=False)
                fg_mask = get_fg_mask(data_t['label'], self.has_fg)
                raw_perc = self.criteria['Perceptual'](net_G_output['fake_raw_images'] * fg_mask,
                                                       data_t['image'] * fg_mask)
                self.gen_losses['GAN'] = self.gen_losses['GAN'] + raw_gan
                self.gen_losses['FeatureMatching'] = self.gen_losses['FeatureMatching'] + raw_fm
                self.gen_losses['Perceptual'] = self.gen_losses['Perceptual'] + raw_perc
            if self.add_dis_cfg is not None:
                for name in self.add_dis_cfg:
                    self.gen_losses['GAN_' + name], self.gen_losses['FeatureMatching_' + name] = \
                        self.compute_GAN_losses(net_D_output[name], dis_update=False)
            if self.use_flow:
                self._flow_losses(data_t, net_G_output)
            if self.cfg.trainer.loss_weight.temporal_gan > 0 and self.sequence_length > 1:
                for s in range(self.num_temporal_scales):
                    self.gen_losses['GAN_T%d' % s], self.gen_losses['FeatureMatching_T%d' % s] = \
                        self.compute_GAN_losses(net_D_output['temporal_%d' % s],
                                                dis_update=False)
            self._get_custom_gen_losses(data_t, net_G_output, net_D_output)
        total = torch.zeros((), device=self.device)
        for key, v in self.gen_losses.items():
            if key != 'total':
                total = total + v.float() * self.weights[key]
        self.gen_losses['total'] = total
        self._step(total, self.net_G, self.opt_G)

    def _flow_losses(self, data_t, net_G_output):
        if self.flow_mode == 'flownet':
            l1, warp, mask = self.criteria['Flow'](data_t, net_G_output, self.current_epoch)
            self.gen_losses['Flow_L1'], self.gen_losses['Flow_Warp'], \
                self.gen_losses['Flow_Mask'] = l1, warp, mask
        elif net_G_output['warped_images'] is not None and data_t.get('mask') is not None:
            self.gen_losses['Flow_L1'] = self.criteria['Flow'](
                net_G_output['fake_images'].float(), net_G_output['warped_images'].float(),
                data_t['mask'].float())
        else:
            self.gen_losses['Flow_L1'] = torch.zeros((), device=self.device)

    def _get_custom_gen_losses(self, data_t, net_G_output, net_D_output):
        pass

    def get_dis_losses(self, net_D_output):
        self.opt_D.zero_grad(set_to_none=True)
        with self.autocast():
            self.dis_losses['GAN'] = self.compute_GAN_losses(net_D_output['indv'],
                                                             dis_update=True)
            if 'raw' in net_D_output:
                self.dis_losses['GAN'] = self.dis_losses['GAN'] + self.compute_GAN_losses(
                    net_D_output['raw'], dis_update=True)
            if self.add_dis_cfg is not None:
                for name in self.add_dis_cfg:
                    self.dis_losses['GAN_' + name] = self.compute_GAN_losses(
                        net_D_output[name], dis_update=True)
            if self.cfg.trainer.loss_weight.temporal_gan > 0 and self.sequence_length > 1:
                for s in range(self.num_temporal_scales):
                    self.dis_losses['GAN_T%d' % s] = self.compute_GAN_losses(
                        net_D_output['temporal_%d' % s], dis_update=True)
            self._get_custom_dis_losses(net_D_output)
        total = torch.zeros((), device=self.device)
        for key, v in self.dis_losses.items():
            if key != 'total':
                total = total + v.float() * self.weights[key]
        self.dis_losses['total'] = total
        self._step(total, self.net_D, self.opt_D)

    def _get_custom_dis_losses(self, net_D_output):
        pass

    def compute_GAN_losses(self, net_D_output, dis_update):  # noqa: N802
        zero = torch.zeros((), device=self.device)
        if net_D_output['pred_fake'] is None:
            return zero if dis_update else [zero, zero]
        if dis_update:
            return self.criteria['GAN'](net_D_output['pred_fake']['output'], False,
                                        dis_update=True) + \
                self.criteria['GAN'](net_D_output['pred_real']['output'], True, dis_update=True)
        gan = self.criteria['GAN'](net_D_output['pred_fake']['output'], True, dis_update=False)
        fm = self.criteria['FeatureMatching'](net_D_output['pred_fake']['features'],
                                              net_D_output['pred_real']['features'])
        return gan, fm

    def get_data_t(self, data, net_G_output, data_prev, t):
        label = data['label'][:, t]
        image = data['images'][:, t]
        if data_prev is not None:
            n = self.cfg.data.num_frames_G
            prev_labels = concat_frames(data_prev['prev_labels'], data_prev['label'], n - 1)
            prev_images = concat_frames(data_prev['prev_images'],
                                        net_G_output['fake_images'].detach(), n - 1)
        else:
            prev_labels = prev_images = None
        return dict(label=label, image=image, prev_labels=prev_labels, prev_images=prev_images,
                    real_prev_image=data['images'][:, t - 1] if t > 0 else None)

    # ------------------------------------------------------------- inference
    def reset(self):
        self.net_G_output = self.data_prev = None
        self.t = 0
        self.test_in_model_average_mode = getattr(self, 'test_in_model_average_mode',
                                                  self.cfg.trainer.model_average)
        net = self.net_G.module.averaged_model if self.test_in_model_average_mode \
            else self.net_G.module
        if hasattr(net, 'reset'):
            net.reset()

    def create_sequence_output_dir(self, output_dir, key):
        seq_dir = '/'.join(key.split('/')[:-1])
        output_dir = os.path.join(output_dir, seq_dir)
        os.makedirs(output_dir, exist_ok=True)
        return output_dir, seq_dir.replace('/', '-')

    def test(self, test_data_loader, root_output_dir, inference_args):
        loader = test_data_loader
        for sequence_idx in range(loader.dataset.num_inference_sequences()):
            loader.dataset.set_inference_sequence_idx(sequence_idx)
            print('Seq id: %d, Seq length: %d' % (sequence_idx + 1, len(loader)))
            self.reset()
            self.sequence_length = len(loader)
            video = []
            for idx, data in enumerate(loader):
                key = data['key']['images'][0][0]
                if idx == 0:
                    output_dir, seq_name = self.create_sequence_output_dir(root_output_dir, key)
                    video_path = os.path.join(output_dir, '..', seq_name)
                data['img_name'] = key.split('/')[-1]
                data = self.start_of_iteration(data, current_iteration=-1)
                video.append(self.test_single(data, output_dir, inference_args))
            _save_video(video_path + '.mp4', video, fps=15)

    def test_single(self, data, output_dir=None, inference_args=None):
        if getattr(inference_args, 'finetune', False) and not getattr(self, 'has_finetuned',
                                                                       False):
            self.finetune(data, inference_args)
        net_G = self.net_G.module.averaged_model if getattr(
            self, 'test_in_model_average_mode', False) else self.net_G
        net_G.eval()
        data_t = self.get_data_t(data, self.net_G_output, self.data_prev, 0)
        if self.is_inference or self.sequence_length > 1:
            self.data_prev = data_t
        with torch.no_grad(), self.autocast():
            self.net_G_output = net_G(data_t)
        if output_dir is None:
            return self.net_G_output
        if getattr(inference_args, 'save_fake_only', False):
            image_grid = tensor2im(self.net_G_output['fake_images'])[0]
        else:
            vis = self.get_test_output_images(data)
            image_grid = np.hstack([np.vstack(im) for im in vis if im is not None])
        name = data['img_name'].split('.')[0] + '.jpg' if 'img_name' in data \
            else '%04d.jpg' % self.t
        _imwrite(os.path.join(output_dir, name), image_grid)
        self.t += 1
        return image_grid

    def get_test_output_images(self, data):
        return [self.visualize_label(data['label'][:, -1]), tensor2im(data['images'][:, -1]),
                tensor2im(self.net_G_output['fake_images'])]

    def gen_frames(self, data, use_model_average=False):
        net_G_output = None
        data_prev = None
        net_G = self.net_G.module.averaged_model if use_model_average else self.net_G
        all_info = {'inputs': [], 'outputs': []}
        first = None
        for t in range(self.sequence_length):
            data_t = self.get_data_t(data, net_G_output, data_prev, t)
            data_prev = data_t
            with torch.no_grad(), self.autocast():
                net_G_output = net_G(data_t)
            data_t, net_G_output = self.post_process(data_t, net_G_output)
            if t == 0:
                first = net_G_output
            all_info['inputs'].append(data_t)
            all_info['outputs'].append(net_G_output)
        return first, net_G_output, all_info

    # ---------------------------------------------------------- monitoring
    def _end_of_iteration(self, data, current_epoch, current_iteration):
        if not torch.distributed.is_initialized() and \
                current_iteration % self.cfg.logging_iter == 0:
            msg = '(epoch: %d, iters: %d) ' % (current_epoch, current_iteration)
            msg += ', '.join('%s: %.3f' % (k, float(v)) for k, v in self.gen_losses.items()
                             if k != 'total')
            msg += '\n' + ', '.join('%s: %.3f' % (k, float(v))
                                    for k, v in self.dis_losses.items() if k != 'total')
            print(msg)

    def _init_tensorboard(self):
        super()._init_tensorboard()
        self.regular_fid_meter = Meter('FID/regular')
        if self.cfg.trainer.model_average:
            self.average_fid_meter = Meter('FID/average')

    def write_metrics(self):
        self.sync_buffers()
        if self.cfg.trainer.model_average:
            res = self._compute_fid()
            if res is None or res[0] is None or res[1] is None:
                return
            self.regular_fid_meter.write(res[0])
            self.average_fid_meter.write(res[1])
            meters = [self.regular_fid_meter, self.average_fid_meter]
        else:
            fid = self._compute_fid()
            if fid is None:
                return
            self.regular_fid_meter.write(fid)
            meters = [self.regular_fid_meter]
        for m in meters:
            m.flush(self.current_iteration)

    def _compute_fid(self):
        if self.val_data_loader is None:
            return None
        self.net_G.eval()
        self.net_G_output = None
        few_shot = 'few_shot' in self.cfg.data.type
        self.test_in_model_average_mode = False
        regular = compute_fid(self._get_save_path('regular_fid', 'npy'), self.val_data_loader,
                              self, sample_size=self.sample_size, is_video=True,
                              few_shot_video=few_shot)
        print('Epoch {:05}, Iteration {:09}, Regular FID {}'.format(
            self.current_epoch, self.current_iteration, regular))
        if self.cfg.trainer.model_average:
            self.test_in_model_average_mode = True
            avg = compute_fid(self._get_save_path('average_fid', 'npy'), self.val_data_loader,
                              self, sample_size=self.sample_size, is_video=True,
                              few_shot_video=few_shot)
            print('Epoch {:05}, Iteration {:09}, Average FID {}'.format(
                self.current_epoch, self.current_iteration, avg))
            return regular, avg
        return regular

    def visualize_label(self, label):
        cfgdata = self.cfg.data
        if hasattr(cfgdata, 'for_pose_dataset'):
            from imaginaire_amd.utils.visualization.pose import tensor2pose
            return tensor2pose(self.cfg, label)
        if hasattr(cfgdata, 'input_labels') and 'seg_maps' in cfgdata.input_labels:
            num_labels = None
            for input_type in cfgdata.input_types:
                if 'seg_maps' in input_type:
                    num_labels = input_type['seg_maps'].num_channels
            return tensor2label(label, num_labels)
        if getattr(cfgdata, 'label_channels', 1) > 3:
            return tensor2im(label.sum(1, keepdim=True))
        return tensor2im(label)

    def save_image(self, path, data):
        self.net_G.eval()
        if self.cfg.trainer.model_average:
            self.net_G.module.averaged_model.eval()
        self.net_G_output = None
        first, last, all_info = self.gen_frames(data)
        if self.cfg.trainer.model_average:
            first_avg, last_avg, _ = self.gen_frames(data, use_model_average=True)
        lengths = self.train_data_loader.dataset.get_label_lengths()
        labels = split_labels(data['label'], lengths)
        vis_start, vis_end = [], []
        for key, value in labels.items():
            f = self.visualize_label if key == 'seg_maps' else tensor2im
            vis_start.append(f(value[:, -1]))
            vis_end.append(f(value[:, 0]))
        if is_master():
            vis = [*vis_start, tensor2im(data['images'][:, -1]), tensor2im(last['fake_images']),
                   tensor2im(last['fake_raw_images'])]
            if self.cfg.trainer.model_average:
                vis += [tensor2im(last_avg['fake_images']),
                        tensor2im(last_avg['fake_raw_images'])]
            if self.sequence_length > 1:
                vis_first = [*vis_end, tensor2im(data['images'][:, 0]),
                             tensor2im(first['fake_images']), tensor2im(first['fake_raw_images'])]
                if self.cfg.trainer.model_average:
                    vis_first += [tensor2im(first_avg['fake_images']),
                                  tensor2im(first_avg['fake_raw_images'])]
                if self.use_flow and last['fake_flow_maps'] is not None:
                    flows = [(tensor2flow(last['fake_flow_maps']),
                              tensor2im(last['fake_occlusion_masks'], normalize=False),
                              tensor2im(last['warped_images']))]
                    if self.flow_mode == 'flownet':
                        flow_gt, conf_gt = self.criteria['Flow'].flowNet(
                            data['images'][:, -1], data['images'][:, -2])
                        gt = [tensor2flow(flow_gt), tensor2im(conf_gt, normalize=False),
                              tensor2im(resample(data['images'][:, -1], flow_gt))]
                    else:
                        gt = [[np.zeros_like(x) for x in im] for im in flows[0]]
                    vis_first += gt
                    vis += list(flows[0])
                vis = [[np.vstack((a, b)) for a, b in zip(fi, li)]
                       for fi, li in zip(vis_first, vis) if li is not None and fi is not None]
            image_grid = np.hstack([np.vstack(im) for im in vis if im is not None])
            print('Save output images to {}'.format(path))
            _imwrite(path, image_grid)
            if self.sequence_length > 1:
                frames = [tensor2im(o['fake_images'])[0] for o in all_info['outputs']]
                _save_video(os.path.splitext(path)[0] + '.mp4', frames, fps=2)
        self.net_G.train()

    def finetune(self, data, inference_args):
        raise NotImplementedError('fine-tuning is defined for few-shot vid2vid')
