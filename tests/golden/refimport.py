"""Import the reference neural_renderer_torch Python package from /root/reference for golden-vector
generation (this container only; /root/reference does not exist on the GPU box).

The package cannot be imported as-is here: it needs imageio (absent), chainer
(optimizers.py:6, absent) and its CUDA extension (rasterize.py:5, needs nvcc + a GPU).  So its
modules are loaded one by one under a synthetic package name with:
  * an `imageio` stand-in whose imread is PIL-backed,
  * a stand-in `<pkg>.cuda.rasterize_cuda` whose two used entry points run the CPU oracle
    restatement of the kernels (oracle/nr_oracle.c),
  * __init__.py and optimizers.py skipped.
Nothing is written under /root/reference (bytecode writing is disabled).
"""
import importlib.util
import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference/neural_renderer_torch"
PKG = "nrt_ref"

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import oracle  # noqa: E402


def _imageio_stub():
    from PIL import Image
    m = types.ModuleType("imageio")
    m.imread = lambda p: np.asarray(Image.open(p))

    def imwrite(p, a):
        a = np.asarray(a)
        if a.dtype != np.uint8:
            a = np.clip(a * 255, 0, 255).astype(np.uint8)
        Image.fromarray(a).save(p)
    m.imwrite = imwrite
    return m


def _cuda_stub():
    m = types.ModuleType(PKG + ".cuda.rasterize_cuda")

    def face_index_map_forward_safe(faces, face_index, num_faces, image_size, near, far, draw_backside,
                                    eps, depth_min_delta):
        out = oracle.face_index_map(faces, image_size, near, far, bool(draw_backside), depth_min_delta)
        face_index.copy_(torch.as_tensor(out).reshape(-1))
        return face_index

    def compute_weight_map_c(faces, face_index_map, weight_map, num_faces, image_size):
        B = faces.shape[0]
        fim = face_index_map.reshape(B, image_size, image_size)
        weight_map.copy_(torch.as_tensor(oracle.weight_map(faces, fim)).reshape(weight_map.shape))
        return face_index_map

    def face_index_map_forward_unsafe(*a, **k):
        raise RuntimeError("unused by the reference")

    m.face_index_map_forward_safe = face_index_map_forward_safe
    m.compute_weight_map_c = compute_weight_map_c
    m.face_index_map_forward_unsafe = face_index_map_forward_unsafe
    return m


def load():
    if PKG in sys.modules:
        return sys.modules[PKG]
    sys.dont_write_bytecode = True
    sys.modules.setdefault("imageio", _imageio_stub())
    pkg = types.ModuleType(PKG)
    pkg.__path__ = [REF]
    sys.modules[PKG] = pkg
    cuda = types.ModuleType(PKG + ".cuda")
    cuda.__path__ = []
    sys.modules[PKG + ".cuda"] = cuda
    stub = _cuda_stub()
    sys.modules[PKG + ".cuda.rasterize_cuda"] = stub
    cuda.rasterize_cuda = stub

    def _load(name):
        spec = importlib.util.spec_from_file_location(PKG + "." + name, os.path.join(REF, name + ".py"))
        mod = importlib.util.module_from_spec(spec)
        sys.modules[PKG + "." + name] = mod
        spec.loader.exec_module(mod)
        setattr(pkg, name, mod)
        return mod

    for name in ["rasterize_param", "lights", "utils", "differentiation", "look_at", "look",
                 "perspective", "load_obj", "save_obj", "rasterize"]:
        _load(name)
    # mirror the attribute layout of the reference __init__.py:1-12 that renderer.py imports from
    pkg.look_at = pkg.look_at.look_at
    pkg.look = pkg.look.look
    pkg.perspective = pkg.perspective.perspective
    for n in ["rasterize_silhouettes", "rasterize_rgba", "rasterize_rgb", "rasterize_depth"]:
        setattr(pkg, n, getattr(sys.modules[PKG + ".rasterize"], n))
    ren = _load("renderer")
    pkg.Renderer = ren.Renderer
    return pkg
