"""Few-shot vid2vid trainer (reference trainers/fs_vid2vid.py:24-292): the
vid2vid per-frame schedule plus reference (few-shot) frames in ``data_t``,
foreground masking of the raw output, and test-time fine-tuning on the
reference frames."""
import os

import numpy as np
import torch

from imaginaire_amd.model_utils.fs_vid2vid import (concat_frames, get_fg_mask,
                                                   pre_process_densepose, random_roll)
from imaginaire_amd.model_utils.pix2pixHD import get_optimizer_with_params
from imaginaire_amd.trainers.vid2vid import Trainer as Vid2VidTrainer
from imaginaire_amd.trainers.vid2vid import _imwrite, _save_video
from imaginaire_amd.utils.distributed import is_master
from imaginaire_amd.utils.distributed import master_only_print as print
from imaginaire_amd.utils.visualization import tensor2flow, tensor2im


class Trainer(Vid2VidTrainer):
    def pre_process(self, data):
        data_cfg = self.cfg.data
        if hasattr(data_cfg, 'for_pose_dataset') and \
                'pose_maps-densepose' in data_cfg.input_labels:
            pose_cfg = data_cfg.for_pose_dataset
            data['label'] = pre_process_densepose(pose_cfg, data['label'], self.is_inference)
            data['few_shot_label'] = pre_process_densepose(pose_cfg, data['few_shot_label'],
                                                           self.is_inference)
        return data

    def get_test_output_images(self, data):
        return [tensor2im(data['few_shot_images'][:, 0]),
                self.visualize_label(data['label'][:, -1]), tensor2im(data['images'][:, -1]),
                tensor2im(self.net_G_output['fake_images'])]

    def get_data_t(self, data, net_G_output, data_prev, t):
        label = data['label'][:, t] if 'label' in data else None
        image = data['images'][:, t]
        if data_prev is not None:
            n = self.cfg.data.num_frames_G
            prev_labels = concat_frames(data_prev['prev_labels'], data_prev['label'], n - 1)
            prev_images = concat_frames(data_prev['prev_images'],
                                        net_G_output['fake_images'].detach(), n - 1)
        else:
            prev_labels = prev_images = None
        data_t = dict(label=label, image=image, ref_labels=data.get('few_shot_label'),
                      ref_images=data['few_shot_images'], prev_labels=prev_labels,
                      prev_images=prev_images,
                      real_prev_image=data['images'][:, t - 1] if t > 0 else None)
        if 'landmarks_xy' in data:
            data_t['landmarks_xy'] = data['landmarks_xy'][:, t]
            data_t['ref_landmarks_xy'] = data['few_shot_landmarks_xy']
        return data_t

    def post_process(self, data, net_G_output):
        if self.has_fg:
            fg_mask = get_fg_mask(data['label'], self.has_fg)
            if net_G_output['fake_raw_images'] is not None:
                net_G_output['fake_raw_images'] = net_G_output['fake_raw_images'] * fg_mask
        return data, net_G_output

    def test(self, test_data_loader, root_output_dir, inference_args):
        self.reset()
        test_data_loader.dataset.set_sequence_length(0)
        test_data_loader.dataset.set_inference_sequence_idx(
            inference_args.driving_seq_index, inference_args.few_shot_seq_index,
            inference_args.few_shot_frame_index)
        video = []
        output_dir = os.path.join(root_output_dir, '%03d' % inference_args.driving_seq_index)
        os.makedirs(output_dir, exist_ok=True)
        for idx, data in enumerate(test_data_loader):
            data['img_name'] = data['key']['images'][0][0].split('/')[-1]
            data = self.start_of_iteration(data, current_iteration=-1)
            video.append(self.test_single(data, output_dir, inference_args))
        _save_video(output_dir + '.mp4', video, fps=15)

    def save_image(self, path, data):
        self.net_G.eval()
        if self.cfg.trainer.model_average:
            self.net_G.module.averaged_model.eval()
        self.net_G_output = None
        first, last, _ = self.gen_frames(data)
        if self.cfg.trainer.model_average:
            first_avg, last_avg, _ = self.gen_frames(data, use_model_average=True)

        def get_images(out, first_frame=True, avg=False):
            fi = 0 if first_frame else -1
            wi = 0 if first_frame else 1
            vis = [] if avg else [tensor2im(data['few_shot_images'][:, fi]),
                                  self.visualize_label(data['label'][:, fi]),
                                  tensor2im(data['images'][:, fi])]
            vis += [tensor2im(out['fake_images']), tensor2im(out['fake_raw_images'])]
            if not avg:
                vis += [tensor2im(out['warped_images'][wi]),
                        tensor2flow(out['fake_flow_maps'][wi]),
                        tensor2im(out['fake_occlusion_masks'][wi], normalize=False)]
            return vis
        if is_master():
            vis_first = get_images(first)
            if self.cfg.trainer.model_average:
                vis_first += get_images(first_avg, avg=True)
            if self.sequence_length > 1:
                vis_last = get_images(last, first_frame=False)
                if self.cfg.trainer.model_average:
                    vis_last += get_images(last_avg, first_frame=False, avg=True)
                vis = [[np.vstack((a, b)) for a, b in zip(fi, la)]
                       for fi, la in zip(vis_first, vis_last)
                       if fi is not None and la is not None]
            else:
                vis = vis_first
            image_grid = np.hstack([np.vstack(im) for im in vis if im is not None])
            print('Save output images to {}'.format(path))
            _imwrite(path, image_grid)
        self.net_G.train()

    def finetune(self, data, inference_args):
        """Few-shot test-time fine-tuning on the reference frames (fs_vid2vid.py:264-292)."""
        self.net_G, self.net_D, self.opt_G, self.opt_D = get_optimizer_with_params(
            self.cfg, self.net_G, self.net_D,
            param_names_start_with=['weight_generator.fc', 'conv_img', 'up'])
        data_ft = dict(data)
        ref_labels, ref_images = data_ft['few_shot_label'], data_ft['few_shot_images']
        iterations = getattr(inference_args, 'finetune_iter', 100)
        for it in range(1, iterations + 1):
            idx = np.random.randint(ref_labels.size(1))
            tgt_label, tgt_image = random_roll([ref_labels[:, idx], ref_images[:, idx]])
            data_ft['label'] = tgt_label.unsqueeze(1)
            data_ft['images'] = tgt_image.unsqueeze(1)
            self.gen_update(data_ft)
            self.dis_update(data_ft)
            if it % max(1, iterations // 10) == 0:
                print(it)
        self.has_finetuned = True
