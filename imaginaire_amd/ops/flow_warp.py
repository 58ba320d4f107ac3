"""Optical-flow warp (k9, ``csrc/flow_warp.hip``).

Same result as the reference ``resample`` (model_utils/fs_vid2vid.py:14-38):
``F.grid_sample`` with bilinear interpolation, border padding and
``align_corners=True`` on a pixel grid shifted by the flow.
"""
import torch
import torch.nn.functional as F

from imaginaire_amd.ops import _ext


class _FlowWarpFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, image, flow):
        ctx.save_for_backward(image, flow)
        return _ext.ext().flow_warp_fwd(image, flow)

    @staticmethod
    def backward(ctx, dout):
        image, flow = ctx.saved_tensors
        dimg, dflow = _ext.ext().flow_warp_bwd(image, flow, dout.contiguous())
        dimg = dimg.to(image.dtype) if ctx.needs_input_grad[0] else None
        if dimg is not None and image.is_contiguous(memory_format=torch.channels_last) and \
                not image.is_contiguous():
            dimg = dimg.contiguous(memory_format=torch.channels_last)
        return dimg, (dflow.to(flow.dtype) if ctx.needs_input_grad[1] else None)


def flow_warp_reference(image, flow):
    b, c, h, w = image.size()
    x = torch.linspace(-1.0, 1.0, w, device=image.device).view(1, 1, 1, w).expand(b, 1, h, w)
    y = torch.linspace(-1.0, 1.0, h, device=image.device).view(1, 1, h, 1).expand(b, 1, h, w)
    grid = torch.cat([x, y], 1)
    flow = torch.cat([flow[:, 0:1] / ((w - 1.0) / 2.0), flow[:, 1:2] / ((h - 1.0) / 2.0)], 1)
    final_grid = (grid + flow.float()).permute(0, 2, 3, 1)
    return F.grid_sample(image.float(), final_grid, mode='bilinear', padding_mode='border',
                         align_corners=True).to(image.dtype)


def flow_warp(image, flow):
    if _ext.use_native(image):
        return _FlowWarpFn.apply(image, flow)
    return flow_warp_reference(image, flow)
