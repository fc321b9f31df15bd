"""The reference's native module, re-bound to the MI355X library: a drop-in for the pybind11
extension `neural_renderer_torch.cuda.rasterize_cuda` (cuda/rasterize_cuda.cpp:93-99).

Same function names, argument order, in-place semantics and return values as the reference's
bindings, so the reference's own rasterize.py (which does
`from .cuda.rasterize_cuda import face_index_map_forward_safe, face_index_map_forward_unsafe,
compute_weight_map_c`, rasterize.py:5) runs unchanged on top of libnr_raster.so when this file is
installed as neural_renderer_torch/cuda/rasterize_cuda.py ("Level 1").

Error behaviour follows the reference's CHECK_INPUT (cuda/rasterize_cuda.cpp:5-7): a RuntimeError
for a tensor that is not on the GPU or not contiguous; a failed launch raises too (the reference
only printf'd it, rasterize_cuda_kernel.cu:385-388).  Launches go to the current torch stream.
"""
import torch

from . import _lib


def _check_input(name, t):
    if not (torch.is_tensor(t) and t.is_cuda):
        raise RuntimeError("%s must be a CUDA tensor" % name)
    if not t.is_contiguous():
        raise RuntimeError("%s must be contiguous" % name)


def face_index_map_forward_safe(faces, face_index, num_faces, image_size, near, far, draw_backside, eps,
                                depth_min_delta):
    """cuda/rasterize_cuda.cpp:55-65 -> rasterize_cuda_kernel.cu:362-390.  faces [B, F, 3, 3] f32,
    face_index int32 with B * S * S elements (written in place: every element, -1 = background).
    Returns face_index."""
    _check_input("faces", faces)
    _check_input("face_index", face_index)
    B = faces.shape[0]
    S = int(image_size)
    if face_index.dtype != torch.int32 or face_index.numel() != B * S * S:
        raise RuntimeError("face_index must be int32 with batch * image_size^2 elements")
    if faces.dtype != torch.float32:
        raise RuntimeError("faces must be float32")
    L = _lib.lib()
    ws = torch.empty(L.nr_workspace_bytes(B, int(num_faces), S), dtype=torch.uint8, device=faces.device)
    with torch.cuda.device(faces.device):
        _lib.check(L.nr_face_index_map_forward_safe(
            _lib.ptr(faces), _lib.ptr(face_index), B, int(num_faces), S, float(near), float(far), int(draw_backside),
            float(eps), float(depth_min_delta), _lib.ptr(ws), ws.numel(), _lib.stream_of(faces)),
            "face_index_map_forward_safe")
    return face_index


def face_index_map_forward_unsafe(faces, face_index_map, depth_map, lock, num_faces, image_size, near, far,
                                  draw_backside, eps):
    """cuda/rasterize_cuda.cpp:67-79: bound but dead in the reference (its z-buffer update is
    commented out, rasterize_cuda_kernel.cu:236-240, and rasterize.py:23-24 never calls it)."""
    raise NotImplementedError("face_index_map_forward_unsafe is dead code in the reference; "
                              "use face_index_map_forward_safe")


def compute_weight_map_c(faces, face_index_map, weight_map, num_faces, image_size):
    """cuda/rasterize_cuda.cpp:81-90 -> rasterize_cuda_kernel.cu:420-443.  face_index_map is the
    flat [B * S * S] int32 map, weight_map [B * S * S, 3] f32 (written in place; background
    pixels get 0, which is what the reference's caller-zeroed buffer holds).  Returns
    face_index_map, as the reference does (.cu:440)."""
    _check_input("faces", faces)
    _check_input("face_index_map", face_index_map)
    _check_input("weight_map", weight_map)
    S = int(image_size)
    n = face_index_map.numel()
    if n % (S * S) != 0 or weight_map.numel() != 3 * n:
        raise RuntimeError("face_index_map / weight_map sizes do not match image_size")
    with torch.cuda.device(faces.device):
        _lib.check(_lib.lib().nr_compute_weight_map(
            _lib.ptr(faces), _lib.ptr(face_index_map), _lib.ptr(weight_map), n // (S * S), int(num_faces), S,
            _lib.stream_of(faces)), "compute_weight_map_c")
    return face_index_map


def mask_foreground_forward(face_index, data_in, data_out, dim):
    """cuda/rasterize_cuda.cpp:35-43 -> .cu:312-335: data_out[p] = data_in[p] (dim floats) where
    face_index[p] >= 0; other elements untouched.  face_index [B, S, S].  Returns data_out."""
    for name, t in (("face_index", face_index), ("data_in", data_in), ("data_out", data_out)):
        _check_input(name, t)
    n = face_index.numel()
    with torch.cuda.device(face_index.device):
        _lib.check(_lib.lib().nr_mask_foreground_forward(
            _lib.ptr(face_index), _lib.ptr(data_in), _lib.ptr(data_out), n, int(dim),
            _lib.stream_of(face_index)), "mask_foreground_forward")
    return data_out


def mask_foreground_backward(face_index, grad_in, grad_out, dim):
    """cuda/rasterize_cuda.cpp:45-53 -> .cu:337-359: grad_in[p] = grad_out[p] where face_index[p]
    >= 0.  Covers every pixel (the reference's launch covers only a third of them, .cu:343; it is
    never called there).  Returns grad_in."""
    for name, t in (("face_index", face_index), ("grad_in", grad_in), ("grad_out", grad_out)):
        _check_input(name, t)
    n = face_index.numel()
    with torch.cuda.device(face_index.device):
        _lib.check(_lib.lib().nr_mask_foreground_backward(
            _lib.ptr(face_index), _lib.ptr(grad_in), _lib.ptr(grad_out), n, int(dim),
            _lib.stream_of(face_index)), "mask_foreground_backward")
    return grad_in
