"""Camera + dispatch API (reference renderer.py:7-75): same attributes, defaults and methods."""
import math

from . import camera
from .look import look
from .look_at import look_at
from .perspective import perspective
from .rasterize import rasterize_depth, rasterize_rgb, rasterize_rgba, rasterize_silhouettes
from .rasterize_param import RasterizeHyperparam, RasterizeParam


class Renderer(object):
    def __init__(self):
        # rendering
        self.image_size = 256
        self.anti_aliasing = True
        self.draw_backside = True
        self.background_color = None
        # camera
        self.perspective = True
        self.viewing_angle = 30
        self.viewpoints = [0, 0, -(1. / math.tan(math.radians(self.viewing_angle)) + 1)]
        self.camera_mode = 'look_at'
        self.camera_direction = [0, 0, 1]
        self.near = 0.1
        self.far = 100

    def transform_vertices(self, vertices, lights=None):
        # GPU tensors: look_at + perspective fused into one HIP launch each way (camera.py); 'look'
        # and CPU tensors take the reference's composition of torch ops below
        if self.camera_mode != 'look' and camera.fusable(vertices, self.viewing_angle):
            return camera.camera_transform(vertices, self.viewpoints if self.camera_mode == 'look_at' else None,
                                           perspective=self.perspective, angle=self.viewing_angle)
        if self.camera_mode == 'look_at':
            vertices = look_at(vertices, self.viewpoints)
        elif self.camera_mode == 'look':
            vertices = look(vertices, self.viewpoints, self.camera_direction)
        if self.perspective:
            vertices = perspective(vertices, angle=self.viewing_angle)
        return vertices

    def _hyper(self):
        return RasterizeHyperparam(image_size=self.image_size, near=self.near, far=self.far,
                                   anti_aliasing=self.anti_aliasing, draw_backside=self.draw_backside)

    def render_silhouettes(self, vertices, faces, backgrounds=None):
        vertices = self.transform_vertices(vertices)
        params = RasterizeParam(background_color=self.background_color, backgrounds=backgrounds)
        return rasterize_silhouettes(vertices, faces, params, self._hyper())

    def render(self, vertices, faces, vertices_t, faces_t, textures, backgrounds=None, lights=None):
        vertices = self.transform_vertices(vertices)
        params = RasterizeParam(vertices_textures=vertices_t, faces_textures=faces_t, textures=textures,
                                background_color=self.background_color, backgrounds=backgrounds, lights=lights)
        return rasterize_rgba(vertices, faces, params, self._hyper())

    def render_rgb(self, vertices, faces, vertices_t, faces_t, textures, backgrounds=None, lights=None):
        vertices = self.transform_vertices(vertices, lights)
        params = RasterizeParam(vertices_textures=vertices_t, faces_textures=faces_t, textures=textures,
                                background_color=self.background_color, backgrounds=backgrounds, lights=lights)
        return rasterize_rgb(vertices, faces, params, self._hyper())

    def render_depth(self, vertices, faces, backgrounds=None):
        vertices = self.transform_vertices(vertices)
        params = RasterizeParam(background_color=self.background_color, backgrounds=backgrounds)
        return rasterize_depth(vertices, faces, params, self._hyper())
