"""pix2pixHD utilities (reference model_utils/pix2pixHD.py:17-226): K-means
feature clustering per label (after all-gathering feature & instance maps),
instance edge maps and the partial-parameter fine-tune optimizer builder."""
import numpy as np
import torch

from imaginaire_amd.ops.segment import get_edges  # noqa: F401  (re-export)
from imaginaire_amd.utils.data import get_paired_input_label_channel_number
from imaginaire_amd.utils.distributed import dist_all_gather_tensor, is_master
from imaginaire_amd.utils.distributed import master_only_print as print
from imaginaire_amd.utils.trainer import (get_optimizer, get_optimizer_for_params,
                                          wrap_model_and_optimizer)


def cluster_features(cfg, train_data_loader, net_E, preprocess=None, small_ratio=0.0625,
                     is_cityscapes=True):
    from sklearn.cluster import KMeans
    label_nc = get_paired_input_label_channel_number(cfg.data)
    feat_nc = cfg.gen.enc.num_feat_channels
    n_clusters = getattr(cfg.gen.enc, 'num_clusters', 10)
    features = {label: np.zeros((0, feat_nc + 1)) for label in range(label_nc)}
    for data in train_data_loader:
        if preprocess is not None:
            data = preprocess(data)
        feat = encode_features(net_E, feat_nc, label_nc, data['images'], data['instance_maps'],
                               is_cityscapes)
        if is_master():
            for label in range(label_nc):
                features[label] = np.append(features[label], feat[label], axis=0)
    if is_master():
        for label in range(label_nc):
            feat = features[label]
            feat = feat[feat[:, -1] > small_ratio, :-1]
            if feat.shape[0]:
                n_clusters_l = min(feat.shape[0], n_clusters)
                kmeans = KMeans(n_clusters=n_clusters_l, random_state=0, n_init=10).fit(feat)
                n, d = kmeans.cluster_centers_.shape
                this_cluster = getattr(net_E, 'cluster_%d' % label)
                this_cluster[0:n, :] = torch.as_tensor(kmeans.cluster_centers_).float()


@torch.no_grad()
def encode_features(net_E, feat_nc, label_nc, image, inst, is_cityscapes=True):
    feat_map = net_E(image, inst)
    feature_map_gather = dist_all_gather_tensor(feat_map)
    inst_gathered = dist_all_gather_tensor(inst)
    feature = {i: np.zeros((0, feat_nc + 1)) for i in range(label_nc)}
    if not is_master():
        return feature
    all_feat_map = torch.cat(feature_map_gather, 0).float().cpu()
    all_inst_map = torch.cat(inst_gathered, 0).cpu()
    for n in range(all_feat_map.size(0)):
        fm = all_feat_map[n]
        inst_n = all_inst_map[n, 0].long()
        fh, fw = fm.shape[1:]
        for i in torch.unique(inst_n).tolist():
            label = (i if i < 1000 else i // 1000) if is_cityscapes else i
            if label >= label_nc:
                continue
            idx = (inst_n == i).nonzero()
            num = idx.size(0)
            y, x = idx[num // 2].tolist()
            val = np.zeros((1, feat_nc + 1))
            val[0, :feat_nc] = fm[:feat_nc, y, x].numpy()
            val[0, feat_nc] = float(num) / (fh * fw)
            feature[label] = np.append(feature[label], val, axis=0)
    return feature


def get_optimizer_with_params(cfg, net_G, net_D, param_names_start_with=(),
                              param_names_include=()):
    def get_train_params(net, starts, includes):
        params_to_train = []
        names = set()
        for key, value in net.named_parameters():
            key_s = key.replace('module.', '').replace('averaged_model.', '')
            do_train = False
            for p in starts:
                if key_s.startswith(p):
                    do_train = True
                    names.add(p)
            if not do_train:
                for p in includes:
                    if p in key_s:
                        do_train = True
                        names.add(key_s[:key_s.find(p) + len(p)])
            if do_train:
                params_to_train.append(value)
        print('Training layers: ', sorted(names))
        return params_to_train
    if param_names_start_with or param_names_include:
        params = get_train_params(net_G, param_names_start_with, param_names_include)
    else:
        params = net_G.parameters()
    opt_G = get_optimizer_for_params(cfg.gen_opt, params)
    opt_D = get_optimizer(cfg.dis_opt, net_D)
    return wrap_model_and_optimizer(cfg, net_G, net_D, opt_G, opt_D)
