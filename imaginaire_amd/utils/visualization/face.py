"""Facial-landmark rendering and normalisation (reference utils/visualization/face.py:14-491).

Landmarks (68 dlib points, optionally + 15 synthesised upper-face points)
are grouped into facial parts, each part drawn as piece-wise quadratic
curves through consecutive point triples, producing the edge-map label
used by the few-shot face models. Optional per-part distance transforms
(L1 / taxicab, scipy instead of OpenCV) and sinusoidal positional encodings
extend the label map exactly as in the reference.
"""
import warnings
from math import pi

import numpy as np
import torch
from scipy.ndimage import distance_transform_cdt
from scipy.optimize import curve_fit
from scipy.signal import medfilt


def _face_options(cfgdata):
    face_cfg = getattr(cfgdata, 'for_face_dataset', None)
    if face_cfg is None:
        return False, False, False
    add_upper_face = getattr(face_cfg, 'add_upper_face', False)
    add_dist_map = getattr(face_cfg, 'add_distance_transform', False)
    add_pos_encode = add_dist_map and getattr(face_cfg, 'add_positional_encode', False)
    return add_upper_face, add_dist_map, add_pos_encode


def _part_list(add_upper_face):
    jaw = list(range(0, 17)) + ((list(range(68, 83)) + [0]) if add_upper_face else [])
    return [[jaw],                                                      # face contour
            [list(range(17, 22))],                                      # right eyebrow
            [list(range(22, 27))],                                      # left eyebrow
            [[28, 31], list(range(31, 36)), [35, 28]],                  # nose
            [[36, 37, 38, 39], [39, 40, 41, 36]],                       # right eye
            [[42, 43, 44, 45], [45, 46, 47, 42]],                       # left eye
            [list(range(48, 55)), [54, 55, 56, 57, 58, 59, 48],         # mouth
             list(range(60, 65)), [64, 65, 66, 67, 60]]]                # tongue


def _add_upper_face(keypoints):
    pts = keypoints[:, :17, :].astype(np.int32)
    baseline_y = (pts[:, 0:1, 1] + pts[:, -1:, 1]) / 2
    upper = pts[:, 1:-1, :].copy()
    upper[:, :, 1] = baseline_y + (baseline_y - upper[:, :, 1]) * 2 // 3
    return np.hstack((keypoints, upper[:, ::-1, :]))


def connect_face_keypoints(resize_h, resize_w, crop_h, crop_w, original_h, original_w,
                           is_flipped, cfgdata, keypoints):
    """[T, K, 2] landmarks -> list of T HxWxC float32 label maps in [0, 1]."""
    add_upper_face, add_dist_map, add_pos_encode = _face_options(cfgdata)
    parts = _part_list(add_upper_face)
    if add_upper_face:
        keypoints = _add_upper_face(keypoints)
    edge_len = 3
    bw = max(1, resize_h // 256)
    outputs = []
    for t in range(keypoints.shape[0]):
        im_edges = np.zeros((resize_h, resize_w, 1), np.uint8)
        dists = []
        im_pos = None
        for edge_list in parts:
            for e, edge in enumerate(edge_list):
                im_edge = np.zeros((resize_h, resize_w, 1), np.uint8)
                for i in range(0, max(1, len(edge) - 1), edge_len - 1):
                    sub = edge[i:i + edge_len]
                    cx, cy = interp_points(keypoints[t, sub, 0], keypoints[t, sub, 1])
                    draw_edge(im_edges, cx, cy, bw=bw)
                    if add_dist_map:
                        draw_edge(im_edge, cx, cy, bw=bw)
                if add_dist_map:
                    d = distance_transform_cdt(255 - im_edge[..., 0] > 0, metric='taxicab')
                    im_dist = np.clip(d / 3, 0, 255)
                    dists.append(im_dist[..., None])
                    if add_pos_encode and e == 0:
                        x = (im_dist.astype(np.float32) - 127.5) / 127.5
                        enc = []
                        for lv in range(10):
                            enc += [np.sin(pi * (2 ** lv) * x), np.cos(pi * (2 ** lv) * x)]
                        im_pos = np.stack(enc, -1)
        out = im_edges
        if add_dist_map:
            out = np.dstack([out] + dists)
        out = out.astype(np.float32) / 255.0
        if add_pos_encode and im_pos is not None:
            out = np.dstack((out, im_pos))
        outputs.append(out)
    return outputs


def normalize_and_connect_face_keypoints(cfg, is_inference, data):
    """Inference-time: normalise driving landmarks to the reference face,
    median-smooth them over time, then draw both into label maps."""
    assert is_inference
    resize_h, resize_w = data['images'][0].shape[-2:]
    keypoints = data['label'].numpy()[0]
    ref_keypoints = data['few_shot_label'].numpy()[0]
    dist_scales = prev = None
    if 'common_attr' in data and 'prev_data' in data['common_attr']:
        dist_scales = data['common_attr']['dist_scales']
        prev = data['common_attr']['prev_data']
    keypoints, dist_scales = normalize_face_keypoints(
        keypoints[0], ref_keypoints[0], dist_scales,
        momentum=getattr(cfg.for_face_dataset, 'normalize_momentum', 0.9))
    keypoints = keypoints[np.newaxis]
    ks = getattr(cfg.for_face_dataset, 'smooth_kernel_size', 5)
    window = keypoints if prev is None else np.vstack([prev, keypoints])[-ks:]
    if ks > 1 and window.shape[0] == ks:
        keypoints = smooth_face_keypoints(window, ks)
    data.setdefault('common_attr', {})
    data['common_attr']['dist_scales'] = dist_scales
    data['common_attr']['prev_data'] = window
    labels = []
    for kpt in (keypoints, ref_keypoints):
        lab = connect_face_keypoints(resize_h, resize_w, None, None, None, None, False, cfg,
                                     kpt)
        labels.append(torch.from_numpy(lab[0]).permute(2, 0, 1).unsqueeze(0))
    data['label'], data['few_shot_label'] = labels
    return data


def smooth_face_keypoints(concat_keypoints, ks):
    """Temporal median filter; zero (missing) points take the previous frame's value."""
    f = medfilt(concat_keypoints, kernel_size=[ks, 1, 1])
    if (f == 0).any():
        for t in range(1, f.shape[0]):
            cur = f[t]
            mx = np.maximum(cur, f[t - 1])
            cur[cur == 0] = mx[cur == 0]
            f[t] = cur
    return f[ks // 2: ks // 2 + 1]


_PARTS_68 = [[0, 16], [1, 15], [2, 14], [3, 13], [4, 12], [5, 11], [6, 10], [7, 9, 8],
             [17, 26], [18, 25], [19, 24], [20, 23], [21, 22], [27], [28], [29], [30],
             [31, 35], [32, 34], [33], [36, 45], [37, 44], [38, 43], [39, 42], [40, 47],
             [41, 46], [48, 54], [49, 53], [50, 52], [51], [55, 59], [56, 58], [57],
             [60, 64], [61, 63], [62], [65, 67], [66]]


def normalize_face_keypoints(keypoints, ref_keypoints, dist_scales=None, momentum=0.9):
    """Rescale each symmetric part pair of the driving face to the reference
    face's proportions, with temporal momentum on the scales."""
    if keypoints.shape[0] != 68:
        raise ValueError('Input keypoints type not supported.')
    face_cen = keypoints[[8]].mean(0)
    ref_face_cen = ref_keypoints[[8]].mean(0)

    def mean_dists(pts, cen):
        pc = pts.mean(0)
        return np.linalg.norm(pts - pc, axis=1).mean() + 1e-3, np.linalg.norm(pc - cen) + 1e-3
    sx, sy = [None] * len(_PARTS_68), [None] * len(_PARTS_68)
    px_prev, py_prev, img_scale = dist_scales if dist_scales is not None else (None, None, None)
    if img_scale is None:
        img_scale = (keypoints[:, 0].max() - keypoints[:, 0].min()) / \
            (ref_keypoints[:, 0].max() - ref_keypoints[:, 0].min())
    for i, idx in enumerate(_PARTS_68):
        pts = keypoints[idx]
        pts = pts[pts[:, 0] != 0]
        if not pts.shape[0]:
            continue
        mx, my = mean_dists(pts, face_cen)
        rx, ry = mean_dists(ref_keypoints[idx], ref_face_cen)
        sx[i] = rx / mx * img_scale
        sy[i] = ry / my * img_scale
        if px_prev is not None:
            sx[i] = px_prev[i] * momentum + sx[i] * (1 - momentum)
            sy[i] = py_prev[i] * momentum + sy[i] * (1 - momentum)
        pc = pts.mean(0)
        keypoints[idx] = (pts - pc) * sx[i] + (pc - face_cen) * sy[i] + face_cen
    return keypoints, [sx, sy, img_scale]


def npy_to_tensor(keypoints):
    return torch.from_numpy(keypoints).unsqueeze(0)


def get_dlib_landmarks_from_image(imgs, predictor_path='shape_predictor_68_face_landmarks.dat'):
    """dlib 68-point detector (optional dependency; raises if dlib is absent)."""
    import dlib
    from imaginaire_amd.utils.io import get_checkpoint
    predictor_path = get_checkpoint(predictor_path, url='1l9zT-AI1yKlfyAb_wl_RjLBSaiWQr8dr')
    if isinstance(imgs, torch.Tensor):
        imgs = np.transpose(((imgs + 1) / 2 * 255).byte().cpu().numpy(), (0, 2, 3, 1))
    detector = dlib.get_frontal_face_detector()
    predictor = dlib.shape_predictor(predictor_path)
    points = np.zeros([imgs.shape[0], 68, 2], dtype=int)
    for i in range(imgs.shape[0]):
        dets = detector(imgs[i], 1)
        if len(dets) > 0:
            shape = predictor(imgs[i], dets[0])
            for b in range(68):
                points[i, b] = shape.part(b).x, shape.part(b).y
    return points


def get_126_landmarks_from_image(imgs, landmarks_network):
    if isinstance(imgs, torch.Tensor):
        imgs = np.transpose(((imgs + 1) / 2 * 255).byte().cpu().numpy(), (0, 2, 3, 1))
    out = []
    for i in range(imgs.shape[0]):
        boxes, landmark = landmarks_network.get_face_boxes_and_landmarks(imgs[i])
        if len(landmark) > 1:
            sizes = [max(b[2] - b[0], b[1] - b[1]) for b in boxes]
            landmark = landmark[int(np.argmax(sizes))]
        elif len(landmark) == 1:
            landmark = landmark[0]
        else:
            landmark = np.zeros((126, 2), dtype=np.float32)
        out.append(landmark[np.newaxis])
    return np.vstack(out).astype(np.float32)


def convert_face_landmarks_to_image(cfgdata, landmarks, output_size, output_tensor=True,
                                    cpu_only=False):
    h, w = output_size
    labels = connect_face_keypoints(h, w, None, None, None, None, False, cfgdata, landmarks)
    if not output_tensor:
        return labels
    labels = torch.cat([torch.from_numpy(x).permute(2, 0, 1).unsqueeze(0) for x in labels])
    return labels if cpu_only or not torch.cuda.is_available() else labels.cuda()


def add_face_keypoints(label_map, image, keypoints):
    """Set the pixels of [-1, 1]-normalised keypoints to 1 in the label map."""
    if label_map is None:
        label_map = torch.zeros_like(image)[:, :1]
    h, w = image.shape[-2:]
    x = ((keypoints[:, :, 0] + 1) / 2 * w).long()
    y = ((keypoints[:, :, 1] + 1) / 2 * h).long()
    bs = torch.arange(label_map.shape[0], device=label_map.device).view(-1, 1).expand_as(x)
    label_map[bs, :, y, x] = 1
    return label_map


def draw_edge(im, x, y, bw=1, color=(255, 255, 255), draw_end_points=False):
    """Stamp a (2bw)x(2bw) brush at every (x, y) of the curve."""
    if x is None or not x.size:
        return
    h, w = im.shape[0], im.shape[1]
    for i in range(-bw, bw):
        for j in range(-bw, bw):
            set_color(im, np.clip(y + i, 0, h - 1), np.clip(x + j, 0, w - 1), color)
    if draw_end_points:
        ends_y, ends_x = np.array([y[0], y[-1]]), np.array([x[0], x[-1]])
        for i in range(-bw * 2, bw * 2):
            for j in range(-bw * 2, bw * 2):
                if i * i + j * j < 4 * bw * bw:
                    set_color(im, np.clip(ends_y + i, 0, h - 1), np.clip(ends_x + j, 0, w - 1),
                              color)


def set_color(im, yy, xx, color):
    if not isinstance(color, (list, tuple)):
        color = [color] * 3
    if im.ndim == 3 and im.shape[2] == 3:
        if (im[yy, xx] == 0).all():
            im[yy, xx, 0], im[yy, xx, 1], im[yy, xx, 2] = color[0], color[1], color[2]
        else:
            for c in range(3):
                im[yy, xx, c] = ((im[yy, xx, c].astype(float) + color[c]) / 2).astype(np.uint8)
    else:
        im[yy, xx] = color[0]


def func(x, a, b, c):
    return a * x ** 2 + b * x + c


def linear(x, a, b):
    return a * x + b


def interp_points(x, y):
    """Fit a line (2 points) or parabola (3 points) and sample it at integer x
    (or integer y when the curve is steeper in y)."""
    x, y = np.asarray(x, dtype=np.float64), np.asarray(y, dtype=np.float64)
    if np.abs(x[:-1] - x[1:]).max() < np.abs(y[:-1] - y[1:]).max():
        cy, cx = interp_points(y, x)
        return (None, None) if cy is None else (cx, cy)
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        try:
            if len(x) < 3:
                popt, _ = curve_fit(linear, x, y)
            else:
                popt, _ = curve_fit(func, x, y)
                if abs(popt[0]) > 1:
                    return None, None
        except Exception:  # noqa: BLE001 (degenerate fit)
            return None, None
    if x[0] > x[-1]:
        x, y = x[::-1], y[::-1]
    cx = np.linspace(x[0], x[-1], int(np.round(x[-1] - x[0])))
    cy = linear(cx, *popt) if len(x) < 3 else func(cx, *popt)
    return cx.astype(int), cy.astype(int)
