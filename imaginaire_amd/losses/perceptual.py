"""Perceptual loss (reference losses/perceptual.py:15-358).

Frozen VGG-19 / VGG-16 / AlexNet / Inception-v3 / ResNet-50 / VGG-face
feature networks with per-layer weights, L1/L2, optional resize to 224,
instance-normalised features and multi-scale evaluation.

MI355X execution: the backbone is kept in bf16 channels-last when the trainer
runs mixed precision (the reference runs it in fp16 under apex O1), the
network is truncated after the deepest requested layer (the reference also
computes the unused tail), every conv+ReLU pair is one k10 MFMA launch with
the bias and ReLU in its epilogue, and the target branch runs under ``no_grad``.
"""
import torch
import torch.nn.functional as F
from torch import nn

from imaginaire_amd.models import backbones
from imaginaire_amd.ops import conv as nhwc_conv
from imaginaire_amd.utils.distributed import master_only_print as print
from imaginaire_amd.ops.loss import weighted_l1
from imaginaire_amd.utils.misc import apply_imagenet_normalization
from imaginaire_amd.ops.resize import interpolate
from imaginaire_amd.ops.pool import max_pool2d


class PerceptualLoss(nn.Module):
    def __init__(self, cfg, network='vgg19', layers='relu_4_1', weights=None, criterion='l1',
                 resize=False, resize_mode='bilinear', instance_normalized=False,
                 num_scales=1):
        super().__init__()
        if isinstance(layers, str):
            layers = [layers]
        if weights is None:
            weights = [1.] * len(layers)
        elif isinstance(weights, (float, int)):
            weights = [weights]
        assert len(layers) == len(weights), \
            'The number of layers (%s) must be equal to the number of weights (%s).' % (
                len(layers), len(weights))
        builders = {'vgg19': _vgg19, 'vgg16': _vgg16, 'alexnet': _alexnet,
                    'inception_v3': _inception_v3, 'resnet50': _resnet50,
                    'robust_resnet50': _robust_resnet50, 'vgg_face_dag': _vgg_face_dag}
        if network not in builders:
            raise ValueError('Network %s is not recognized' % network)
        self.model = builders[network](layers)
        self.num_scales = num_scales
        self.layers = layers
        self.weights = weights
        if criterion == 'l1':
            self.criterion = F.l1_loss
        elif criterion in ('l2', 'mse'):
            self.criterion = F.mse_loss
        else:
            raise ValueError('Criterion %s is not recognized' % criterion)
        self.resize = resize
        self.resize_mode = resize_mode
        self.instance_normalized = instance_normalized
        amp = getattr(cfg.trainer, 'amp', 'O0') if cfg is not None else 'O0'
        self.low_precision = amp in ('O1', 'O2', 'O3', 'bf16')
        print('Perceptual loss:\n\tMode: {}'.format(network))

    def _apply(self, fn, *args, **kwargs):
        out = super()._apply(fn, *args, **kwargs)
        return out

    def to_device_format(self):
        """Move the frozen backbone to bf16 channels-last (called by the trainer on GPU)."""
        if self.low_precision:
            self.model.to(dtype=torch.bfloat16)
        self.model.to(memory_format=torch.channels_last)

    def forward(self, inp, target):
        self.model.eval()
        inp, target = apply_imagenet_normalization(inp), apply_imagenet_normalization(target)
        inp, target = inp[:, :3], target[:, :3]
        if self.resize:
            inp = interpolate(inp, mode=self.resize_mode, size=(224, 224), align_corners=False)
            target = interpolate(target, mode=self.resize_mode, size=(224, 224),
                                   align_corners=False)
        dtype = next(self.model.parameters()).dtype
        loss = 0
        for scale in range(self.num_scales):
            input_features = self.model(inp.to(dtype))
            with torch.no_grad():
                target_features = self.model(target.to(dtype))
            if self.criterion is F.l1_loss and not self.instance_normalized:
                # all layers in one multi-tensor L1 (k13 on the GPU)
                loss = loss + weighted_l1([input_features[k] for k in self.layers],
                                          [target_features[k] for k in self.layers],
                                          self.weights)
            else:
                for layer, weight in zip(self.layers, self.weights):
                    input_feature = input_features[layer]
                    target_feature = target_features[layer].detach()
                    if self.instance_normalized:
                        input_feature = F.instance_norm(input_feature)
                        target_feature = F.instance_norm(target_feature)
                    loss = loss + weight * self.criterion(input_feature, target_feature).float()
            # the next scale sees the half-resolution pair (reference perceptual.py:126-131)
            if scale != self.num_scales - 1:
                inp = interpolate(inp, mode=self.resize_mode, scale_factor=0.5,
                                    align_corners=False, recompute_scale_factor=True)
                target = interpolate(target, mode=self.resize_mode, scale_factor=0.5,
                                       align_corners=False, recompute_scale_factor=True)
        return loss.float()


class _PerceptualNetwork(nn.Module):
    """Sequential feature network returning the requested named activations."""

    def __init__(self, network, layer_name_mapping, layers):
        super().__init__()
        assert isinstance(network, nn.Sequential), 'The network needs to be of type "nn.Sequential".'
        self.network = network
        self.layer_name_mapping = layer_name_mapping
        self.layers = layers
        idx = [i for i, n in layer_name_mapping.items() if n in layers]
        self.last_index = max(idx) if idx else len(network) - 1
        for param in self.parameters():
            param.requires_grad = False
            param._iamd_frozen = True  # never trained: ops/conv.py caches its k10 operand

    def forward(self, x):
        output = {}
        layers = list(self.network)
        i = 0
        while i < len(layers):
            layer = layers[i]
            nxt = layers[i + 1] if i + 1 < len(layers) else None
            if x.is_cuda and type(layer) is nn.Conv2d and type(nxt) is nn.ReLU and \
                    self.layer_name_mapping.get(i, None) not in self.layers and \
                    layer.padding_mode == 'zeros' and layer.groups == 1:
                # conv + ReLU as one k10 MFMA launch (bias + ReLU in the epilogue)
                x = nhwc_conv.conv2d_act(x, layer.weight, layer.bias, layer.stride,
                                         layer.padding, layer.dilation, 0.0)
                i += 1
            elif x.is_cuda and type(layer) is nn.Conv2d:
                x = nhwc_conv.conv2d(x, layer.weight, layer.bias, layer.stride, layer.padding,
                                     layer.dilation, layer.groups, layer.padding_mode)
            elif x.is_cuda and type(layer) is nn.MaxPool2d:
                x = max_pool2d(x, layer.kernel_size, layer.stride, layer.padding, layer.dilation,
                               layer.ceil_mode)
            else:
                x = layer(x)
            layer_name = self.layer_name_mapping.get(i, None)
            if layer_name in self.layers:
                output[layer_name] = x
            if i >= self.last_index:
                break
            i += 1
        return output


def _vgg19(layers):
    network = backbones.vgg19(pretrained=True).features
    mapping = {1: 'relu_1_1', 3: 'relu_1_2', 6: 'relu_2_1', 8: 'relu_2_2', 11: 'relu_3_1',
               13: 'relu_3_2', 15: 'relu_3_3', 17: 'relu_3_4', 20: 'relu_4_1', 22: 'relu_4_2',
               24: 'relu_4_3', 26: 'relu_4_4', 29: 'relu_5_1'}
    return _PerceptualNetwork(network, mapping, layers)


def _vgg16(layers):
    network = backbones.vgg16(pretrained=True).features
    mapping = {1: 'relu_1_1', 3: 'relu_1_2', 6: 'relu_2_1', 8: 'relu_2_2', 11: 'relu_3_1',
               13: 'relu_3_2', 15: 'relu_3_3', 18: 'relu_4_1', 20: 'relu_4_2', 22: 'relu_4_3',
               25: 'relu_5_1'}
    return _PerceptualNetwork(network, mapping, layers)


def _alexnet(layers):
    network = backbones.alexnet(pretrained=True).features
    mapping = {0: 'conv_1', 1: 'relu_1', 3: 'conv_2', 4: 'relu_2', 6: 'conv_3', 7: 'relu_3',
               8: 'conv_4', 9: 'relu_4', 10: 'conv_5', 11: 'relu_5'}
    return _PerceptualNetwork(network, mapping, layers)


def _inception_v3(layers):
    inception = backbones.inception_v3(pretrained=True)
    network = nn.Sequential(inception.Conv2d_1a_3x3, inception.Conv2d_2a_3x3,
                            inception.Conv2d_2b_3x3, nn.MaxPool2d(kernel_size=3, stride=2),
                            inception.Conv2d_3b_1x1, inception.Conv2d_4a_3x3,
                            nn.MaxPool2d(kernel_size=3, stride=2), inception.Mixed_5b,
                            inception.Mixed_5c, inception.Mixed_5d, inception.Mixed_6a,
                            inception.Mixed_6b, inception.Mixed_6c, inception.Mixed_6d,
                            inception.Mixed_6e, inception.Mixed_7a, inception.Mixed_7b,
                            inception.Mixed_7c, nn.AdaptiveAvgPool2d(output_size=(1, 1)))
    mapping = {3: 'pool_1', 6: 'pool_2', 14: 'mixed_6e', 18: 'pool_3'}
    return _PerceptualNetwork(network, mapping, layers)


def _resnet_seq(resnet50):
    return nn.Sequential(resnet50.conv1, resnet50.bn1, resnet50.relu, resnet50.maxpool,
                         resnet50.layer1, resnet50.layer2, resnet50.layer3, resnet50.layer4,
                         resnet50.avgpool)


def _resnet50(layers):
    network = _resnet_seq(backbones.resnet50(pretrained=True))
    mapping = {4: 'layer_1', 5: 'layer_2', 6: 'layer_3', 7: 'layer_4'}
    return _PerceptualNetwork(network, mapping, layers)


def _robust_resnet50(layers):
    # adversarially robust ResNet-50 weights (Madry lab) if available locally
    resnet50 = backbones.resnet50(pretrained=False)
    backbones.load_pretrained(resnet50, 'robust_resnet50')
    mapping = {4: 'layer_1', 5: 'layer_2', 6: 'layer_3', 7: 'layer_4'}
    return _PerceptualNetwork(_resnet_seq(resnet50), mapping, layers)


class _Flatten(nn.Module):
    def forward(self, x):
        return x.reshape(x.shape[0], -1)


def _vgg_face_dag(layers):
    network = backbones.vgg16(pretrained=False, num_classes=2622)
    backbones.load_pretrained(network, 'vgg_face_dag')
    mapping = {1: 'avgpool', 3: 'fc6', 4: 'relu_6', 6: 'fc7', 7: 'relu_7', 9: 'fc8'}
    seq = [network.features, network.avgpool, _Flatten()]
    seq += [network.classifier[i] for i in range(7)]
    return _PerceptualNetwork(nn.Sequential(*seq), mapping, layers)
