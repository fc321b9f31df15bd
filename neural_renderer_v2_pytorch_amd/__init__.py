"""neural_renderer_v2_pytorch_amd -- MI355X-native drop-in for neural_renderer_torch's rasterize path.

Public surface mirrors the reference's neural_renderer_torch/__init__.py:1-14 (minus Mesh and the
chainer-based Adam, which are outside the hot path).  Compute runs in hand-written HIP kernels for
gfx950 (csrc/nr_raster.hip) behind the C ABI of include/nr_raster.h; there is no CPU fallback.
"""
from .lights import AmbientLight, DirectionalLight, Light, SpecularLight
from .load_obj import load_obj
from .look import look
from .look_at import look_at
from .perspective import perspective
from .rasterize import rasterize_core, rasterize_depth, rasterize_rgb, rasterize_rgba, rasterize_silhouettes
from .rasterize_param import RasterizeHyperparam, RasterizeParam
from .renderer import Renderer
from .save_obj import save_obj
from .utils import create_textures, get_points_from_angles, imread, make_gif, to_gpu
from .differentiation import differentiation
from .camera import camera_transform

__version__ = '2.0.2+mi355x.1'
