"""Fused camera prologue: Renderer.transform_vertices (reference renderer.py:27-38) as one HIP
launch each way (nr_camera_forward / nr_camera_backward, include/nr_raster.h) -- look_at
(look_at.py:5-44) followed by perspective (perspective.py:4-18) -- instead of the ~15 torch
launches of the composed ops and their autograd graph.

Gradients reach the vertices and the viewpoints (example4's camera fit, examples_pytorch/
example4.py:30-33).  The standalone look_at / look / perspective functions stay torch ops, like the
reference's; this module is what the Renderer runs for GPU tensors."""
import math

import torch

from . import _lib


def _width(angle):
    """tan(angle / 180 * 3.1416) in float32, as perspective.py:10-13 computes it."""
    a = torch.as_tensor(angle, dtype=torch.float32).detach().cpu()
    return float(torch.tan(a / 180. * 3.1416))


class _Cam:
    __slots__ = ("B", "V", "look_at", "perspective", "width", "at", "up")


def _args(cfg, vertices, eye):
    c = _lib.NrCameraArgs()
    c.batch_size, c.num_vertices = cfg.B, cfg.V
    c.vertices = vertices.data_ptr()
    c.v_batch_stride = 0 if vertices.shape[0] == 1 and cfg.B > 1 else cfg.V * 3
    if cfg.look_at:
        c.eye = eye.data_ptr()
        c.eye_batch_stride = 0 if eye.shape[0] == 1 else 3
        c.mode = _lib.NR_CAMERA_LOOK_AT
    else:
        c.mode = _lib.NR_CAMERA_NONE
    for j in range(3):
        c.at[j], c.up[j] = cfg.at[j], cfg.up[j]
    c.perspective = int(cfg.perspective)
    c.width = cfg.width
    return c


class CameraTransform(torch.autograd.Function):
    """vertices [1 or B, V, 3] (world), eye [1 or B, 3] -> projected vertices [B, V, 3]."""

    @staticmethod
    def forward(ctx, vertices, eye, cfg):
        out = torch.empty((cfg.B, cfg.V, 3), dtype=torch.float32, device=vertices.device)
        c = _args(cfg, vertices, eye)
        with torch.cuda.device(vertices.device):
            _lib.check(_lib.lib().nr_camera_forward(c, _lib.ptr(out), _lib.stream_of(vertices)), "nr_camera_forward")
        ctx.cfg = cfg
        ctx.save_for_backward(vertices, eye)
        return out

    @staticmethod
    def backward(ctx, grad_out):
        vertices, eye = ctx.saved_tensors
        cfg = ctx.cfg
        grad_out = grad_out.contiguous()
        dev = vertices.device
        gv = torch.empty_like(vertices) if ctx.needs_input_grad[0] else None
        ge = torch.empty_like(eye) if (ctx.needs_input_grad[1] and cfg.look_at) else None
        L = _lib.lib()
        ws = torch.empty(L.nr_camera_workspace_bytes(cfg.B) if ge is not None else 0, dtype=torch.uint8, device=dev)
        c = _args(cfg, vertices, eye)
        with torch.cuda.device(dev):
            _lib.check(L.nr_camera_backward(c, _lib.ptr(grad_out), _lib.ptr(gv), _lib.ptr(ge), _lib.ptr(ws), ws.numel(),
                                            _lib.stream_of(vertices)), "nr_camera_backward")
        return gv, ge, None


def camera_transform(vertices, viewpoints=None, perspective=True, angle=30., at=None, up=None):
    """look_at(vertices, viewpoints, at, up) (when viewpoints is given) then, with `perspective`,
    perspective(., angle): the result of the reference's composition, fused on the GPU.
    vertices [B, V, 3] (a batch-expanded view is read once); viewpoints [3], [1, 3] or [B, 3]."""
    assert vertices.ndim == 3
    _lib.require_gpu(vertices)
    dev = vertices.device
    cfg = _Cam()
    cfg.B, cfg.V = vertices.shape[0], vertices.shape[1]
    v = vertices.float()
    if v.shape[0] > 1 and v.stride(0) == 0:
        v = v[:1]  # one mesh for every item: read once, gradient summed over the items
    v = v.contiguous()
    cfg.look_at = viewpoints is not None
    cfg.perspective = bool(perspective)
    cfg.width = _width(angle) if perspective else 1.0
    cfg.at = [0., 0., 0.] if at is None else [float(x) for x in torch.as_tensor(at, dtype=torch.float32).reshape(3)]
    cfg.up = [0., 1., 0.] if up is None else [float(x) for x in torch.as_tensor(up, dtype=torch.float32).reshape(3)]
    if cfg.look_at:
        eye = viewpoints if torch.is_tensor(viewpoints) else torch.as_tensor(viewpoints, dtype=torch.float32)
        eye = eye.float().to(dev).reshape(-1, 3)
        if eye.shape[0] not in (1, cfg.B):
            raise AssertionError("viewpoints batch must be 1 or %d" % cfg.B)
        if eye.shape[0] > 1 and eye.stride(0) == 0:
            eye = eye[:1]
        eye = eye.contiguous()
    else:
        eye = torch.zeros((1, 3), dtype=torch.float32, device=dev)
    return CameraTransform.apply(v, eye, cfg)


def fusable(vertices, angle):
    """The fused path covers GPU float tensors whose viewing angle takes no gradient."""
    return (torch.is_tensor(vertices) and vertices.is_cuda and vertices.ndim == 3 and
            not (torch.is_tensor(angle) and angle.requires_grad) and
            (not torch.is_tensor(angle) or angle.numel() == 1) and not math.isnan(_width(angle)))
