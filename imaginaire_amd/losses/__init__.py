from .gan import GANLoss
from .perceptual import PerceptualLoss
from .feature_matching import FeatureMatchingLoss
from .kl import GaussianKLLoss
from .flow import MaskedL1Loss, FlowLoss
from .l1 import L1Loss

__all__ = ['GANLoss', 'PerceptualLoss', 'FeatureMatchingLoss', 'GaussianKLLoss', 'MaskedL1Loss',
           'FlowLoss', 'L1Loss']
