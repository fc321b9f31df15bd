"""Light records (reference lights.py:4-39): same classes, attributes and defaults.  rasterize_core
turns a list of them into per-item records for the HIP shading (NrRasterArgs.lights), built with
differentiable torch ops: gradients flow to the vertices through the normals and, through
nr_rasterize_backward_params, to the light colours, directions and specular exponents that
require them (pinned by the param_grads_* goldens)."""
import torch


class Light:
    def __init__(self, color):
        self.color = color

    def to(self, device):
        self.color = self.color.to(device)


class DirectionalLight(Light):
    def __init__(self, color, direction, backside=False):
        super().__init__(color)
        self.direction = direction
        self.backside = backside

    def to(self, device):
        super().to(device)
        self.direction = self.direction.to(device)


class AmbientLight(Light):
    def __init__(self, color):
        super().__init__(color)


class SpecularLight(Light):
    def __init__(self, color, alpha=None, backside=False):
        super().__init__(color)
        self.backside = backside
        self.alpha = alpha if alpha is not None else torch.ones(color.shape[0], dtype=torch.float32)

    def to(self, device):
        super().to(device)
        self.alpha = self.alpha.to(device)
