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


def optimize_graphed(model, iters):
    """optimize() with the whole step -- camera, rasterize, loss, backward, Adam -- captured once in a
    HIP graph (torch.cuda.CUDAGraph) and replayed: the same kernels without the per-launch host
    cost.  The viewpoint is held as a device tensor and Adam runs with capturable=True, so nothing
    in the step touches the host; returns the loss of every step."""
    dev = model.vertices.device
    model.renderer.viewpoints = torch.as_tensor(
        nr.get_points_from_angles(CAMERA_DISTANCE, ELEVATION, AZIMUTH), dtype=torch.float32, device=dev)
    opt = torch.optim.Adam(model.parameters(), capturable=True)

    def step():
        loss = torch.sum((model.renderer.render_silhouettes(model.vertices, model.faces) - model.image_ref[None]) ** 2)
        loss.backward()
        opt.step()
        return loss

    # warm-up on a side stream (state allocation, cached faces checks), then capture one step
    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    snapshot = model.vertices.detach().clone()
    with torch.cuda.stream(side):
        for _ in range(3):
            opt.zero_grad(set_to_none=True)
            step()
    torch.cuda.current_stream(dev).wait_stream(side)
    # undo the warm-up updates: the replays start from the initial mesh and a fresh Adam state
    with torch.no_grad():
        model.vertices.copy_(snapshot)
        for st in opt.state.values():
            for k, v in st.items():
                if torch.is_tensor(v):
                    v.zero_()
    opt.zero_grad(set_to_none=True)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        static_loss = step()
    losses = torch.empty(iters, device=dev)
    for i in range(iters):
        graph.replay()
        losses[i] = static_loss
    return losses.tolist()


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
    ap.add_argument('--graph', action='store_true', help='replay the step as a HIP graph (no frames)')
    args = ap.parse_args()
    model = SilhouetteFit(args.obj, args.ref, torch.device('cuda', args.gpu))
    if args.frames:
        os.makedirs(args.frames, exist_ok=True)
    losses = optimize_graphed(model, args.iters) if args.graph else optimize(model, args.iters, args.frames)
    print('loss: first %.1f, last %.1f after %d steps' % (losses[0], losses[-1], len(losses)))
    if args.frames:
        make_gif(args.frames, os.path.join(args.frames, 'example2_opt.gif'))
        with torch.no_grad():  # example2.py:82-95: a turntable of the result
            for n, az in enumerate(range(0, 360, 4)):
                save_frame(model.render(az)[0], '%s/_tmp_%04d.png' % (args.frames, n))
        make_gif(args.frames, os.path.join(args.frames, 'example2_res.gif'))


if __name__ == '__main__':
    main()
