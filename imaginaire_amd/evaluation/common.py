"""Inception activation extraction (reference evaluation/common.py:16-175).

Activations are gathered across ranks with an all-gather (RCCL) to rank 0.
The Inception-v3 pool features run in bf16 channels-last on MI355X when the
caller is under autocast.
"""
import torch
from torch.nn import functional as F

from imaginaire_amd.models.backbones import inception_v3
from imaginaire_amd.utils.distributed import (dist_all_gather_variable, get_rank, get_world_size,
                                              is_master)
from imaginaire_amd.utils.distributed import master_only_print as print
from imaginaire_amd.utils.misc import apply_imagenet_normalization, to_device

_INCEPTION = {}


def get_inception(device):
    key = str(device)
    if key not in _INCEPTION:
        net = inception_v3(pretrained=True).to(device).eval()
        if device.type == 'cuda':
            net = net.to(memory_format=torch.channels_last)
        _INCEPTION[key] = net
    return _INCEPTION[key]


def _device_of(data):
    for v in data.values() if isinstance(data, dict) else []:
        if isinstance(v, torch.Tensor):
            return v.device
    return torch.device('cuda' if torch.cuda.is_available() else 'cpu')


def _inception_features(inception, images):
    images = images.float().clamp(-1, 1)
    images = apply_imagenet_normalization(images[:, :3])
    images = F.interpolate(images, size=(299, 299), mode='bilinear', align_corners=True)
    if images.is_cuda:
        images = images.contiguous(memory_format=torch.channels_last)
    return inception.features(images).float()


@torch.no_grad()
def get_activations(data_loader, key_real, key_fake, generator=None, sample_size=None,
                    preprocess=None):
    device = torch.device('cuda', torch.cuda.current_device()) if torch.cuda.is_available() \
        else torch.device('cpu')
    inception = get_inception(device)
    world_size = get_world_size()
    batch_y = []
    for it, data in enumerate(data_loader):
        data = to_device(data, device)
        if preprocess is not None:
            data = preprocess(data)
        if generator is None:
            images = data[key_real]
        else:
            images = generator(data)[key_fake]
        batch_y.append(_inception_features(inception, images))
        if sample_size is not None and \
                data_loader.batch_size * world_size * (it + 1) >= sample_size:
            break
    batch_y = torch.cat(batch_y)
    batch_y = dist_all_gather_variable(batch_y)
    if is_master():
        batch_y = torch.cat(batch_y).cpu().numpy()
        if sample_size is not None:
            batch_y = batch_y[:sample_size]
        return batch_y
    return None


@torch.no_grad()
def get_video_activations(data_loader, key_real, key_fake, trainer=None, sample_size=None,
                          preprocess=None, few_shot=False):
    device = torch.device('cuda', torch.cuda.current_device()) if torch.cuda.is_available() \
        else torch.device('cpu')
    inception = get_inception(device)
    batch_y = []
    num_sequences = data_loader.dataset.num_inference_sequences()
    if sample_size is None:
        num_videos_to_test, num_frames_per_video = 10, 5
    else:
        num_videos_to_test, num_frames_per_video = sample_size
    if num_videos_to_test == -1:
        num_videos_to_test = num_sequences
    else:
        num_videos_to_test = min(num_videos_to_test, num_sequences)
    world_size = get_world_size()
    if num_videos_to_test < world_size:
        seq_to_run = [get_rank() % num_videos_to_test]
    else:
        num_videos_to_test = num_videos_to_test // world_size * world_size
        seq_to_run = range(get_rank(), num_videos_to_test, world_size)
    for sequence_idx in seq_to_run:
        data_loader = set_sequence_idx(few_shot, data_loader, sequence_idx)
        if trainer is not None:
            trainer.reset()
        for it, data in enumerate(data_loader):
            if it >= num_frames_per_video:
                break
            if trainer is not None:
                data = trainer.pre_process(data)
            elif preprocess is not None:
                data = preprocess(data)
            data = to_device(data, device)
            if trainer is None:
                images = data[key_real][:, -1]
            else:
                images = trainer.test_single(data)[key_fake]
            batch_y.append(_inception_features(inception, images))
    batch_y = torch.cat(batch_y)
    batch_y = dist_all_gather_variable(batch_y)
    if is_master():
        return torch.cat(batch_y).cpu().numpy()
    return None


def set_sequence_idx(few_shot, data_loader, sequence_idx):
    if few_shot:
        data_loader.dataset.set_inference_sequence_idx(sequence_idx, sequence_idx, 0)
    else:
        data_loader.dataset.set_inference_sequence_idx(sequence_idx)
    return data_loader
