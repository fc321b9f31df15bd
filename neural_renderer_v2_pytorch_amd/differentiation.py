"""Soft rasterisation gradient (reference differentiation.py:6-40).

Forward is the identity on `images`; backward returns the incoming gradient for `images` and, for
`coordinates`, the neighbour-difference estimate of Differentiation.backward
(differentiation.py:12-36 with utils.pad_zeros / utils.maximum, utils.py:75-101), computed by the
HIP kernel nr_differentiation_backward.  Inside rasterize_core the same stencil is fused into the
rasterizer's backward kernel; this standalone Function serves direct callers of `differentiation`.
"""
import torch

from . import _lib


class Differentiation(torch.autograd.Function):
    @staticmethod
    def forward(ctx, images, coordinates):
        ctx.save_for_backward(images)
        return images

    @staticmethod
    def backward(ctx, gradients):
        images, = ctx.saved_tensors
        _lib.require_gpu(images, gradients)
        img = images.contiguous().float()
        g = gradients.contiguous().float()
        B, H, W, C = img.shape
        gxy = torch.empty((B, H, W, 2), dtype=torch.float32, device=img.device)
        with torch.cuda.device(img.device):
            _lib.check(_lib.lib().nr_differentiation_backward(_lib.ptr(img), _lib.ptr(g), _lib.ptr(gxy), B, H, W, C,
                                                              _lib.stream_of(img)), "nr_differentiation_backward")
        return gradients, gxy


def differentiation(images, coordinates):
    return Differentiation.apply(images, coordinates)
