"""FlowNet2 native ops in one namespace: Correlation (k6), Resample2d (k7), ChannelNorm (k8).

Each op (HIP autograd wrapper, functional form, module and fp32 PyTorch reference) lives at the
reference's module path under ``imaginaire_amd/third_party/{correlation,resample2d,channelnorm}``;
this module gathers them for the FlowNet2 networks and the kernel tests.
"""
from imaginaire_amd.third_party.channelnorm.channelnorm import (  # noqa: F401
    ChannelNorm, _ChannelNormFn, channelnorm, channelnorm_reference)
from imaginaire_amd.third_party.correlation.correlation import (  # noqa: F401
    Correlation, _CorrelationFn, correlation, correlation_out_size, correlation_reference)
from imaginaire_amd.third_party.resample2d.resample2d import (  # noqa: F401
    Resample2d, _Resample2dFn, resample2d, resample2d_reference)
