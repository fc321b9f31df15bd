"""Soft rasterisation gradient (reference differentiation.py:6-40).

Forward is the identity on `images`; backward returns the incoming gradient for `images` and, for
`coordinates`, the neighbour-difference estimate of Differentiation.backward
(differentiation.py:12-36 with utils.pad_zeros / utils.maximum, utils.py:75-101).

* CUDA (HIP) tensors: the HIP kernel nr_differentiation_backward (one thread per pixel).  Inside
  rasterize_core the same stencil is fused into the rasterizer's backward kernel; this standalone
  Function serves direct callers of `differentiation`.
* CPU tensors: plain torch ops, as the reference's own Function runs on the CPU (BASELINE cfg1,
  tests_torch/test_differentiation.py).  This is part of the product's API surface, not a fallback
  for the GPU path: a CUDA input never takes it.
"""
import torch

from . import _lib


def _both_sides(t, axis):
    """A term of the neighbour pair (i, i+1) added to both of its pixels: [.., n-1, ..] ->
    [.., n, ..] with out[i] = t[i] (i <= n-2) + t[i-1] (i >= 1).  The reference forms this as
    pad_zeros(t, 'right') + pad_zeros(t, 'left') (differentiation.py:17-27, utils.py:75-88)."""
    shape = list(t.shape)
    shape[axis] = 1
    z = torch.zeros(shape, dtype=t.dtype, device=t.device)
    return torch.cat((t, z), axis) + torch.cat((z, t), axis)


def _select(r, l, eps=1e-4):
    """utils.maximum (utils.py:91-101): -r where r > l, else l; zero where |r - l| < eps, and zero
    where max(r, l) <= 0 (the later masks win, as in the reference's assignment order)."""
    out = torch.where(r > l, -r, l)
    out = torch.where(torch.abs(r - l) < eps, torch.zeros((), dtype=out.dtype), out)
    return torch.where(torch.max(r, l) <= 0, torch.zeros((), dtype=out.dtype), out)


def soft_gradient_cpu(images, grad):
    """[B, S, S, C] internal images and their upstream gradient -> [B, S, S, 2] (x, y) on the CPU,
    with the reference's float operation order (differentiation.py:15-29)."""
    step = 2. / images.shape[1]
    out = []
    for axis in (2, 1):  # x first, then y (differentiation.py:31)
        n = images.shape[axis]
        lo, hi = images.narrow(axis, 0, n - 1), images.narrow(axis, 1, n - 1)
        glo, ghi = grad.narrow(axis, 0, n - 1), grad.narrow(axis, 1, n - 1)
        r = -((lo - hi) * ghi).sum(-1) / step
        l = -((hi - lo) * glo).sum(-1) / step
        out.append(_select(_both_sides(r[..., None], axis), _both_sides(l[..., None], axis)))
    return torch.cat(out, -1)


class Differentiation(torch.autograd.Function):
    @staticmethod
    def forward(ctx, images, coordinates):
        ctx.save_for_backward(images)
        return images

    @staticmethod
    def backward(ctx, gradients):
        images, = ctx.saved_tensors
        if images.device.type == "cpu" and gradients.device.type == "cpu":
            return gradients, soft_gradient_cpu(images.float(), gradients.float())
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
