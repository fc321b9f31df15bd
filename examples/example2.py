"""Silhouette fitting: deform a mesh until its rendered silhouette matches a reference image.

The workload of the reference's examples_pytorch/example2.py:17-78, on this package: a teapot's
vertices are an nn.Parameter, the loss is the squared difference between the rendered silhouette
and the reference image (viewed from azimuth 90), and Adam steps the vertices.  Every render and
its backward run through the HIP rasterizer (Renderer.render_silhouettes -> rasterize_core).

    python examples/example2.py [--iters 300] [--frames DIR] [--gif out.gif]

Inputs default to tests/data/teapot.obj and tests/data/example2_ref.png (the reference example's
own data files).
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
import neural_renderer_v2_pytorch_amd as nr  # noqa: E402
from neural_renderer_v2_pytorch_amd.utils import imread, make_gif  # noqa: E402

DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'tests', 'data')
CAMERA_DISTANCE, ELEVATION, AZIMUTH = 2.732, 0, 90


class SilhouetteFit(torch.nn.Module):
    """example2.py:17-43: the mesh (vertices trainable), the reference silhouette, a Renderer."""

    def __init__(self, obj_file, ref_file, device):
        super().__init__()
        vertices, faces = nr.load_obj(obj_file)
        self.vertices = torch.nn.Parameter(torch.as_tensor(vertices[None]).to(device))
        self.faces = torch.as_tensor(faces).to(device)
        self.image_ref = torch.as_tensor(imread(ref_file).mean(-1)).to(device)
        self.renderer = nr.Renderer()

    def render(self, azimuth=AZIMUTH):
        self.renderer.viewpoints = nr.get_points_from_angles(CAMERA_DISTANCE, ELEVATION, azimuth)
        return self.renderer.render_silhouettes(self.vertices, self.faces)

    def forward(self):
        return torch.sum((self.render() - self.image_ref[None]) ** 2)


def optimize(model, iters, frames_dir=None):
    """example2.py:62-80: Adam over the vertices; returns the loss of every step."""
    opt = torch.optim.Adam(model.parameters())
    losses = []
    for i in range(iters):
        opt.zero_grad()
        loss = model()
        loss.backward()
        opt.step()
        losses.append(float(loss.detach()))
        if frames_dir:
            save_frame(model.render().detach()[0], '%s/_tmp_%04d.png' % (frames_dir, i))
    return losses


def save_frame(image, path):
    from PIL import Image
    a = image.cpu().numpy()
    lo, hi = a.min(), a.max()
    a = (a - lo) / (hi - lo) * 255 if hi > lo else a * 0
    Image.fromarray(a.astype(np.uint8)).save(path)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--obj', default=os.path.join(DATA, 'teapot.obj'))
    ap.add_argument('--ref', default=os.path.join(DATA, 'example2_ref.png'))
    ap.add_argument('--iters', type=int, default=300)
    ap.add_argument('--frames', default=None, help='directory for per-step frames (and the GIFs)')
    ap.add_argument('--gpu', type=int, default=0)
    args = ap.parse_args()
    model = SilhouetteFit(args.obj, args.ref, torch.device('cuda', args.gpu))
    if args.frames:
        os.makedirs(args.frames, exist_ok=True)
    losses = optimize(model, args.iters, args.frames)
    print('loss: first %.1f, last %.1f after %d steps' % (losses[0], losses[-1], len(losses)))
    if args.frames:
        make_gif(args.frames, os.path.join(args.frames, 'example2_opt.gif'))
        with torch.no_grad():  # example2.py:82-95: a turntable of the result
            for n, az in enumerate(range(0, 360, 4)):
                save_frame(model.render(az)[0], '%s/_tmp_%04d.png' % (args.frames, n))
        make_gif(args.frames, os.path.join(args.frames, 'example2_res.gif'))


if __name__ == '__main__':
    main()
