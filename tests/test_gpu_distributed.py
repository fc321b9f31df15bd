"""The product's multi-rank path on the GPU: torch.distributed world size 2 (gloo: both ranks share
the one GPU of the test box -- RCCL refuses two ranks on one device; the driver's 8-GPU bench runs
the same code over RCCL), each rank rendering its shard of the batch through the HIP kernels.

One mesh and one texture atlas, shared by every item, seen from B viewpoints through
Renderer.render (fused camera + rasterize_rgba).  Each rank takes its items with
distributed.shard, renders and differentiates them, sums the shared mesh and texture gradients
with distributed.allreduce_shared_grads, and assembles the images with distributed.gather_images.
The gathered images must equal the single-process full-batch render bit for bit, and the summed
gradients must match its gradients within the gradient tolerance (the per-rank partial sums add
in a different order).  B = 6 (even shards) and B = 5 (3 + 2 items)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

GRAD_TOL = 1e-4


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _inputs(batch):
    import neural_renderer_v2_pytorch_amd as nr
    from neural_renderer_v2_pytorch_amd import synthetic
    v, f = synthetic.icosphere(3)
    vt, ft, tex = nr.create_textures(f.shape[0], texture_size=4)
    tex = np.random.RandomState(61).uniform(0, 1, tex.shape).astype(np.float32)
    eyes = synthetic.viewpoints(batch, seed_base=2100)
    g = np.random.RandomState(62).normal(size=(batch, 4, 64, 64)).astype(np.float32)
    return v, f, vt, ft, tex, eyes, g


def _render(dev, v, f, vt, ft, tex, eyes, g):
    """Renderer.render of the shared mesh from `eyes`; returns (images, mesh grad, texture grad)."""
    import neural_renderer_v2_pytorch_amd as nr
    B = eyes.shape[0]
    mesh = torch.as_tensor(v[None], device=dev).requires_grad_(True)
    atlas = torch.as_tensor(tex, device=dev).requires_grad_(True)
    ren = nr.Renderer()
    ren.image_size = 64
    ren.viewpoints = torch.as_tensor(eyes, device=dev)
    img = ren.render(mesh.expand(B, -1, -1), torch.as_tensor(f, device=dev),
                     torch.as_tensor(vt, device=dev)[None].expand(B, -1, -1), torch.as_tensor(ft, device=dev),
                     atlas[None].expand(B, -1, -1, -1))
    img.backward(torch.as_tensor(g, device=dev))
    return img.detach(), mesh, atlas


def _worker(rank, world_size, port, batch, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world_size)
    try:
        from neural_renderer_v2_pytorch_amd import _lib
        from neural_renderer_v2_pytorch_amd import distributed as ndist
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        v, f, vt, ft, tex, eyes, g = _inputs(batch)
        lo, hi = ndist.shard_range(batch, *ndist.world())
        local_eyes = ndist.shard(torch.as_tensor(eyes)).numpy()
        assert local_eyes.shape[0] == hi - lo
        img, mesh, atlas = _render(dev, v, f, vt, ft, tex, local_eyes, g[lo:hi])
        ndist.allreduce_shared_grads([mesh, atlas])
        full = ndist.gather_images(img)
        full_known = ndist.gather_images(img, batch_size=batch)
        torch.cuda.synchronize()
        np.savez(os.path.join(out_dir, "r%d.npz" % rank), images=full.cpu().numpy(),
                 images_known=full_known.cpu().numpy(), grad_mesh=mesh.grad.cpu().numpy(),
                 grad_atlas=atlas.grad.cpu().numpy(), lib=_lib.LIB_PATH)
    finally:
        dist.destroy_process_group()


def _close(a, b, what):
    scale = float(np.abs(b).max())
    bad = np.abs(a - b) > GRAD_TOL * scale + GRAD_TOL * np.abs(b)
    assert not bad.any(), "%s: %d elements off" % (what, int(bad.sum()))


@pytest.mark.parametrize("batch", [6, 5])
def test_world2_hip_path_matches_full_batch(tmp_path, dev, batch):
    mp.spawn(_worker, args=(2, _free_port(), batch, str(tmp_path)), nprocs=2, join=True)
    v, f, vt, ft, tex, eyes, g = _inputs(batch)
    img, mesh, atlas = _render(dev, v, f, vt, ft, tex, eyes, g)
    want = img.cpu().numpy()
    assert float(np.abs(mesh.grad.cpu().numpy()).sum()) > 0
    for r in range(2):
        got = np.load(str(tmp_path / ("r%d.npz" % r)))
        assert str(got["lib"]).endswith("libnr_raster.so")
        assert np.array_equal(got["images"], want), "rank %d gathered images" % r
        assert np.array_equal(got["images_known"], want), "rank %d gathered images (known batch)" % r
        _close(got["grad_mesh"], mesh.grad.cpu().numpy(), "rank %d shared mesh gradient" % r)
        _close(got["grad_atlas"], atlas.grad.cpu().numpy(), "rank %d shared texture gradient" % r)
