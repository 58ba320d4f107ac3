"""Video-model utilities (reference model_utils/fs_vid2vid.py:14-865).

``resample`` (flow warp with bilinear sampling, border padding,
align_corners=True) runs on the HIP warp kernel (k9, ops/flow_warp.py) on
MI355X; the remaining helpers are small tensor manipulations.
"""
import random

import numpy as np
import torch
import torch.nn.functional as F

from imaginaire_amd.ops.flow_warp import flow_warp


def resample(image, flow):
    """Warp ``image`` by ``flow`` (pixels, [B,2,H,W]) — reference fs_vid2vid.py:14-38."""
    assert flow.shape[1] == 2
    return flow_warp(image, flow)


def get_grid(batchsize, size, minval=-1.0, maxval=1.0, device=None):
    if len(size) == 2:
        rows, cols = size
    elif len(size) == 3:
        deps, rows, cols = size
    else:
        raise ValueError('Dimension can only be 2 or 3.')
    x = torch.linspace(minval, maxval, cols, device=device).view(1, 1, 1, cols)
    x = x.expand(batchsize, 1, rows, cols)
    y = torch.linspace(minval, maxval, rows, device=device).view(1, 1, rows, 1)
    y = y.expand(batchsize, 1, rows, cols)
    t_grid = torch.cat([x, y], dim=1)
    if len(size) == 3:
        z = torch.linspace(minval, maxval, deps, device=device).view(1, 1, deps, 1, 1)
        z = z.expand(batchsize, 1, deps, rows, cols)
        t_grid = t_grid.unsqueeze(2).expand(batchsize, 2, deps, rows, cols)
        t_grid = torch.cat([t_grid, z], dim=1)
    return t_grid


def pick_image(images, idx):
    if type(images) == list:
        return [pick_image(r, idx) for r in images]
    if idx is None:
        return images[:, 0]
    if type(idx) == int:
        return images[:, idx]
    idx = idx.long().view(-1, 1, 1, 1, 1)
    return images.gather(1, idx.expand_as(images)[:, 0:1])[:, 0]


def concat_frames(prev, now, n_frames):
    """Append ``now`` to the sliding window ``prev`` keeping the last n_frames-1 entries."""
    now = now.unsqueeze(1)
    if prev is None:
        return now
    if prev.shape[1] == n_frames:
        prev = prev[:, 1:]
    return torch.cat([prev, now], dim=1)


def detach(output):
    if type(output) == dict:
        return {k: detach(v) for k, v in output.items()}
    if type(output) == list:
        return [detach(v) for v in output]
    if isinstance(output, torch.Tensor):
        return output.detach()
    return output


def crop_and_resize(img, coords, size=None, method='bilinear'):
    if isinstance(img, list):
        return [crop_and_resize(x, coords, size, method) for x in img]
    if img is None:
        return None
    min_y, max_y, min_x, max_x = coords
    img = img[..., min_y:max_y, min_x:max_x]
    if size is not None:
        if method == 'nearest':
            img = F.interpolate(img.reshape(-1, *img.shape[-3:]), size=size, mode='nearest')
        else:
            img = F.interpolate(img.reshape(-1, *img.shape[-3:]), size=size, mode='bilinear',
                                align_corners=False)
    return img


def random_roll(tensors):
    """Random cyclic shift (< 1/16 of the size, either direction) + random
    horizontal flip, applied identically to every tensor (fs_vid2vid.py:814-847)."""
    h, w = tensors[0].shape[2:]
    ny = np.random.choice([np.random.randint(h // 16), h - np.random.randint(h // 16)])
    nx = np.random.choice([np.random.randint(w // 16), w - np.random.randint(w // 16)])
    flip = np.random.rand() > 0.5
    return [roll(t, ny, nx, flip) for t in tensors]


def roll(t, ny, nx, flip):
    t = torch.roll(t, shifts=(int(ny), int(nx)), dims=(2, 3))
    return torch.flip(t, dims=[3]) if flip else t


def select_object(data, obj_indices=None):
    """Keep one person per frame in the OpenPose lists (fs_vid2vid.py:378-402)."""
    key = 'poses-openpose'
    if key in data:
        for i, people in enumerate(data[key]):
            data[key][i] = people[obj_indices[i] if obj_indices is not None else 0]
    return data


# ----------------------------------------------------------------- pose helpers
_PART_GROUPS = [[0], [1, 2], [3, 4], [5, 6], [7, 9, 8, 10], [11, 13, 12, 14],
                [15, 17, 16, 18], [19, 21, 20, 22], [23, 24]]


def _part_index(densepose_map):
    """DensePose part channel in [-1, 1] -> part id in [0, 24] (rounded)."""
    part = (densepose_map / 2 + 0.5) * 24
    assert (part >= 0).all() and (part < 25).all()
    return torch.round(part)


def combine_fg_mask(fg_mask, ref_fg_mask, has_fg):
    return ((fg_mask > 0) | (ref_fg_mask > 0)).float() if has_fg else 1


def get_fg_mask(densepose_map, has_fg):
    """Dilated (15x15) human mask from the DensePose part channel (fs_vid2vid.py:436-458)."""
    if isinstance(densepose_map, list):
        return [get_fg_mask(m, has_fg) for m in densepose_map]
    if not has_fg or densepose_map is None:
        return 1
    if densepose_map.dim() == 5:
        densepose_map = densepose_map[:, 0]
    mask = F.max_pool2d(densepose_map[:, 2:3], 15, stride=1, padding=7)
    return (mask > -1).float()


def get_part_mask(densepose_map):
    """One mask per body-part group (9 groups) (fs_vid2vid.py:461-493)."""
    reshape = densepose_map.dim() == 4
    if reshape:
        bo, t, h, w = densepose_map.shape
        densepose_map = densepose_map.reshape(-1, h, w)
    part = (densepose_map / 2 + 0.5) * 24
    assert (part >= 0).all() and (part < 25).all()
    masks = []
    for group in _PART_GROUPS:
        m = torch.zeros_like(part, dtype=torch.bool)
        for j in group:
            m |= (part > j - 0.1) & (part < j + 0.1)
        masks.append(m)
    mask = torch.stack(masks, 1).float()
    if reshape:
        mask = mask.reshape(bo, t, -1, h, w)
    return mask


def get_face_mask(densepose_map):
    """Face (parts 23, 24) mask (fs_vid2vid.py:496-519)."""
    part = (densepose_map / 2 + 0.5) * 24
    assert (part >= 0).all() and (part < 25).all()
    m = ((part > 22.9) & (part < 23.1)) | ((part > 23.9) & (part < 24.1))
    return m.float()


def extract_valid_pose_labels(pose_map, pose_type, remove_face_labels, do_remove=True):
    """Drop DensePose channels ('open') or blank the face region (fs_vid2vid.py:522-562)."""
    if pose_map is None:
        return pose_map
    if isinstance(pose_map, list):
        return [extract_valid_pose_labels(p, pose_type, remove_face_labels, do_remove)
                for p in pose_map]
    orig_dim = pose_map.dim()
    assert 3 <= orig_dim <= 5
    p = pose_map.reshape((1,) * (5 - orig_dim) + tuple(pose_map.shape))
    if pose_type == 'open':
        p = p[:, :, 3:]
    elif remove_face_labels and do_remove:
        dense, openp = p[:, :, :3], p[:, :, 3:]
        face = get_face_mask(p[:, :, 2]).unsqueeze(2)
        p = torch.cat([dense * (1 - face) - face, openp], dim=2)
    return p.reshape(p.shape[5 - orig_dim:])


def pre_process_densepose(pose_cfg, pose_map, is_infer=False):
    """Random body-part dropout, part channel [0,24]->[0,255], [0,1]->[-1,1]
    (fs_vid2vid.py:780-811)."""
    part_map = pose_map[:, :, 2] * 255
    assert (part_map >= 0).all() and (part_map < 25).all()
    drop = 0 if is_infer else getattr(pose_cfg, 'random_drop_prob', 0)
    if drop > 0:
        dense = pose_map[:, :, :3]
        for part_id in range(1, 25):
            if random.random() < drop:
                m = (part_map - part_id).abs() < 0.1
                dense[m.unsqueeze(2).expand_as(dense)] = 0
        pose_map[:, :, :3] = dense
    pose_map[:, :, 2] = pose_map[:, :, 2] * (255 / 24)
    return pose_map * 2 - 1


def remove_other_ppl(labels, densemasks):
    """Zero every person except the one overlapping OpenPose (fs_vid2vid.py:352-375)."""
    densemasks = densemasks[:, 0:1] * 255
    for idx in range(labels.shape[0]):
        label, densemask = labels[idx], densemasks[idx]
        openpose = label[3:]
        valid = (openpose[0] > 0) | (openpose[1] > 0) | (openpose[2] > 0)
        dp_valid = densemask[valid.unsqueeze(0)]
        if dp_valid.shape[0]:
            ind = torch.bincount(dp_valid.long().flatten()).argmax()
            label = label * (densemask == ind).float()
        labels[idx] = label
    return labels


def normalize_faces(keypoints, ref_keypoints, dist_scale_x=None, dist_scale_y=None):
    """Rescale each facial part of ``keypoints`` to the reference face's
    proportions (fs_vid2vid.py:565-628)."""
    if keypoints.shape[0] == 68:
        central = [8]
        part_list = [[0, 16], [1, 15], [2, 14], [3, 13], [4, 12], [5, 11], [6, 10], [7, 9, 8],
                     [17, 26], [18, 25], [19, 24], [20, 23], [21, 22], [27], [28], [29], [30],
                     [31, 35], [32, 34], [33], [36, 45], [37, 44], [38, 43], [39, 42],
                     [40, 47], [41, 46], [48, 54], [49, 53], [50, 52], [51], [55, 59],
                     [56, 58], [57], [60, 64], [61, 63], [62], [65, 67], [66]]
    elif keypoints.shape[0] == 126:
        central = [16]
        part_list = [[i] for i in range(126)]
    else:
        raise ValueError('Input keypoints type not supported.')
    face_cen = keypoints[central].mean(0)
    ref_face_cen = ref_keypoints[central].mean(0)

    def mean_dists(pts, cen):
        pc = pts.mean(0)
        dx = np.linalg.norm(pts - pc, axis=1).mean() + 1e-3
        dy = np.linalg.norm(pc - cen) + 1e-3
        return dx, dy
    if dist_scale_x is None:
        dist_scale_x = [None] * len(part_list)
        dist_scale_y = [None] * len(part_list)
    for i, idx in enumerate(part_list):
        pts = keypoints[idx]
        if dist_scale_x[i] is None:
            mx, my = mean_dists(pts, face_cen)
            rx, ry = mean_dists(ref_keypoints[idx], ref_face_cen)
            dist_scale_x[i], dist_scale_y[i] = rx / mx, ry / my
        pc = pts.mean(0)
        keypoints[idx] = (pts - pc) * dist_scale_x[i] + (pc - face_cen) * dist_scale_y[i] + \
            face_cen
    return keypoints, [dist_scale_x, dist_scale_y]


# ------------------------------------------------------------------ cropping
def get_face_bbox_for_data(keypoints, orig_img_size, scale, is_inference):
    """Face crop box from landmarks with train-time jitter (fs_vid2vid.py:148-193)."""
    min_y, max_y = int(keypoints[:, 1].min()), int(keypoints[:, 1].max())
    min_x, max_x = int(keypoints[:, 0].min()), int(keypoints[:, 0].max())
    x_cen, y_cen = (min_x + max_x) // 2, (min_y + max_y) // 2
    H, W = orig_img_size
    w = h = max_x - min_x
    if not is_inference:
        offset = np.random.uniform(-0.2, 0.2, 2)
        if scale is None:
            scale = list(np.random.uniform(0.8, 1.2, 2))
        w *= scale[0]
        h *= scale[1]
        x_cen += int(offset[0] * w)
        y_cen += int(offset[1] * h)
    x_cen = max(w, min(W - w, x_cen))
    y_cen = max(h * 1.25, min(H - h * 0.75, y_cen))
    min_x = x_cen - w
    min_y = y_cen - h * 1.25
    return [int(v) for v in (min_y, min_y + h * 2, min_x, min_x + w * 2)], scale


def crop_face_from_data(cfg, is_inference, data):
    """Crop target and reference frames around the face (fs_vid2vid.py:100-145)."""
    label = data.get('label')
    image = data['images']
    ref_labels = data.get('few_shot_label')
    ref_images = data['few_shot_images']
    h, w = [int(v) for v in cfg.output_h_w.split(',')]
    if 'common_attr' in data and 'crop_coords' in data['common_attr']:
        crop_coords, ref_crop_coords = data['common_attr']['crop_coords']
    else:
        ref_crop_coords, scale = get_face_bbox_for_data(
            data['few_shot_landmarks-dlib68_xy'][0], image.shape[-2:], None, is_inference)
        crop_coords, _ = get_face_bbox_for_data(data['landmarks-dlib68_xy'][0],
                                                image.shape[-2:], scale, is_inference)
    label, image = crop_and_resize([label, image], crop_coords, (h, w))
    ref_labels, ref_images = crop_and_resize([ref_labels, ref_images], ref_crop_coords, (h, w))
    data['images'], data['few_shot_images'] = image, ref_images
    if label is not None:
        data['label'], data['few_shot_label'] = label, ref_labels
    if is_inference:
        data.setdefault('common_attr', {})['crop_coords'] = crop_coords, ref_crop_coords
    return data


def get_person_bbox_for_data(pose_map, orig_img_size, scale=1.5, crop_aspect_ratio=1,
                             offset=None):
    """Body crop box from the non-zero DensePose region (fs_vid2vid.py:281-322)."""
    H, W = orig_img_size
    assert pose_map.dim() == 4
    nz = (pose_map[:, :3] > 0).nonzero(as_tuple=False)
    if nz.size(0) == 0:
        bw = int(H * crop_aspect_ratio // 2)
        return [0, H, W // 2 - bw, W // 2 + bw]
    ys, xs = nz[:, 2], nz[:, 3]
    y_min, y_max, x_min, x_max = ys.min().item(), ys.max().item(), xs.min().item(),         xs.max().item()
    y_cen, x_cen = int(y_min + y_max) // 2, int(x_min + x_max) // 2
    bh = int(min(H, max(H // 2, (y_max - y_min) * scale))) // 2
    bh = max(bh, int((x_max - x_min) * scale / crop_aspect_ratio) // 2)
    bw = int(bh * crop_aspect_ratio)
    if offset is not None:
        x_cen += int(offset[0] * bw)
        y_cen += int(offset[1] * bh)
    x_cen = max(bw, min(W - bw, x_cen))
    y_cen = max(bh, min(H - bh, y_cen))
    return [y_cen - bh, y_cen + bh, x_cen - bw, x_cen + bw]


def crop_person_from_data(cfg, is_inference, data):
    """Crop target and reference frames around the person (fs_vid2vid.py:196-278)."""
    label, image = data['label'], data['images']
    few_shot = 'few_shot_label' in data
    ref_labels = data.get('few_shot_label')
    ref_images = data.get('few_shot_images')
    out_h, out_w = [int(v) for v in cfg.output_h_w.split(',')]
    aspect = out_w / out_h
    if 'human_instance_maps' in data:
        label = remove_other_ppl(label, data['human_instance_maps'])
        if few_shot:
            ref_labels = remove_other_ppl(ref_labels, data['few_shot_human_instance_maps'])
    offset = ref_offset = None
    scale = ref_scale = 1.5
    if not is_inference:
        offset = np.clip(np.random.randn(2) * 0.05, -1, 1)
        ref_offset = np.clip(np.random.randn(2) * 0.02, -1, 1)
        scale = min(2, max(1, scale + np.random.randn() * 0.05))
        ref_scale = min(2, max(1, ref_scale + np.random.randn() * 0.02))
    if 'common_attr' in data:
        crop_coords, ref_crop_coords = data['common_attr']['crop_coords']
    else:
        crop_coords = get_person_bbox_for_data(label, image.shape[-2:], scale, aspect, offset)
        ref_crop_coords = get_person_bbox_for_data(ref_labels, image.shape[-2:], ref_scale,
                                                   aspect, ref_offset) if few_shot else None
    data['label'] = crop_and_resize(label, crop_coords, (out_h, out_w), 'nearest')
    data['images'] = crop_and_resize(image, crop_coords, (out_h, out_w))
    if few_shot:
        data['few_shot_label'] = crop_and_resize(ref_labels, ref_crop_coords, (out_h, out_w),
                                                 'nearest')
        data['few_shot_images'] = crop_and_resize(ref_images, ref_crop_coords, (out_h, out_w))
    data.pop('human_instance_maps', None)
    data.pop('few_shot_human_instance_maps', None)
    if is_inference:
        data['common_attr'] = {'crop_coords': (crop_coords, ref_crop_coords)}
    return data


def get_face_bbox_for_output(data_cfg, pose, crop_smaller=0):
    """Square face box in output space (fs_vid2vid.py:661-714)."""
    if pose.dim() == 3:
        pose = pose.unsqueeze(0)
    elif pose.dim() == 5:
        pose = pose[-1, -1:]
    _, _, h, w = pose.shape
    use_openpose = 'pose_maps-densepose' not in data_cfg.input_labels
    if use_openpose:
        num_ch = 0
        for input_type in data_cfg.input_types:
            if 'poses-openpose' in input_type:
                num_ch = input_type['poses-openpose'].num_channels
        if num_ch <= 3:
            raise ValueError('Not implemented yet.')
        face = (pose[:, -1] > 0).nonzero(as_tuple=False)
    else:
        face = (pose[:, 2] > 0.9).nonzero(as_tuple=False)
    ylen = xlen = h // 32 * 8
    if face.size(0):
        y, x = face[:, 1], face[:, 2]
        ys, ye, xs, xe = y.min().item(), y.max().item(), x.min().item(), x.max().item()
        if use_openpose:
            xc, yc = (xs + xe) // 2, (ys * 3 + ye * 2) // 5
            ylen = int((xe - xs) * 2.5)
        else:
            xc, yc = (xs + xe) // 2, (ys + ye) // 2
            ylen = int((ye - ys) * 1.25)
        ylen = xlen = min(w, max(32, ylen))
        yc = max(ylen // 2, min(h - 1 - ylen // 2, yc))
        xc = max(xlen // 2, min(w - 1 - xlen // 2, xc))
    else:
        yc, xc = h // 4, w // 2
    ys, ye, xs, xe = yc - ylen // 2, yc + ylen // 2, xc - xlen // 2, xc + xlen // 2
    if crop_smaller:
        ys, xs, ye, xe = ys + crop_smaller, xs + crop_smaller, ye - crop_smaller, \
            xe - crop_smaller
    return [ys, ye, xs, xe]


def crop_face_from_output(data_cfg, image, input_label, crop_smaller=0):
    """Crop + resize the face of every sample (fs_vid2vid.py:631-658)."""
    if isinstance(image, list):
        return [crop_face_from_output(data_cfg, im, input_label, crop_smaller) for im in image]
    face_size = image.shape[-2] // 32 * 8
    crops = []
    for i in range(input_label.size(0)):
        ys, ye, xs, xe = get_face_bbox_for_output(data_cfg, input_label[i:i + 1],
                                                  crop_smaller=crop_smaller)
        crops.append(F.interpolate(image[i:i + 1, -3:, ys:ye, xs:xe],
                                   size=(face_size, face_size), mode='bilinear',
                                   align_corners=True))
    return torch.cat(crops)


def get_hand_bbox_for_output(data_cfg, pose):
    """Boxes around the two one-hot OpenPose hand channels (fs_vid2vid.py:743-777)."""
    if pose.dim() == 3:
        pose = pose.unsqueeze(0)
    elif pose.dim() == 5:
        pose = pose[-1, -1:]
    _, _, h, w = pose.shape
    ylen = xlen = h // 64 * 8
    coords = []
    for i in range(2):
        if pose.shape[1] <= 6:
            raise ValueError('Not implemented yet.')
        hand = (pose[:, -3 if i == 0 else -2] == 1).nonzero(as_tuple=False)
        if hand.size(0):
            y, x = hand[:, 1], hand[:, 2]
            xc = (x.min().item() + x.max().item()) // 2
            yc = (y.min().item() + y.max().item()) // 2
            yc = max(ylen // 2, min(h - 1 - ylen // 2, yc))
            xc = max(xlen // 2, min(w - 1 - xlen // 2, xc))
            coords.append([yc - ylen // 2, yc + ylen // 2, xc - xlen // 2, xc + xlen // 2])
    return coords


def crop_hand_from_output(data_cfg, image, input_label):
    if isinstance(image, list):
        return [crop_hand_from_output(data_cfg, im, input_label) for im in image]
    crops = []
    for i in range(input_label.size(0)):
        for ys, ye, xs, xe in get_hand_bbox_for_output(data_cfg, input_label[i:i + 1]):
            crops.append(image[i:i + 1, -3:, ys:ye, xs:xe])
    return torch.cat(crops) if crops else None
