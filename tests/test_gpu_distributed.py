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


def _bench_args(batch):
    import argparse
    return argparse.Namespace(batch=batch, level=4, image_size=256, mode="rgbsd")


def _bench_worker(rank, world_size, port, out_dir, batch=64):
    """One rank of bench.py's N > 1 step: its own `batch` headline items, forward + backward, then the
    all_reduce of the shared atlas gradient that bench.step issues inside the timed region."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world_size)
    try:
        import bench
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        w = bench.workload(_bench_args(batch), rank, dev)
        assert w["shared"] == [w["tex"]]
        bench.step(w)
        torch.cuda.synchronize()
        np.savez(os.path.join(out_dir, "b%d.npz" % rank), grad_atlas=w["tex"].grad.cpu().numpy(),
                 grad_proj=w["proj"].grad.cpu().numpy(), g=w["g"].cpu().numpy())
    finally:
        dist.destroy_process_group()


def test_bench_step_allreduce_matches_128_items(tmp_path, dev):
    """bench.py's N > 1 step is the whole sharded step: two gloo ranks, 64 headline items each
    (bench.workload: items 0-63 and 64-127, one shared 288^2 atlas), each ending its step with the
    all_reduce(SUM) of the atlas gradient.  Both ranks' atlas gradients must equal the gradient of
    the same 128 items rendered and differentiated in one process (the reference's index_put_
    scatter summed over the global batch, rasterize.py:144-148, utils.py:104-114) within
    GRAD_TOL; each rank's projected-vertex gradients equal that process's for its items."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    mp.spawn(_bench_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    got = [np.load(str(tmp_path / ("b%d.npz" % r))) for r in range(2)]
    w = bench.workload(_bench_args(128), 0, dev)
    # bench.workload draws each rank's upstream gradient from the same seed: the 128-item run uses
    # the two ranks' gradients side by side
    w["g"] = torch.as_tensor(np.concatenate([got[0]["g"], got[1]["g"]]), device=dev)
    bench.step(w)  # no process group here: no all_reduce, one batched backward over 128 items
    want_atlas = w["tex"].grad.cpu().numpy()
    want_proj = w["proj"].grad.cpu().numpy()
    assert float(np.abs(want_atlas).sum()) > 0
    for r in range(2):
        _close(got[r]["grad_atlas"], want_atlas, "rank %d all-reduced atlas gradient" % r)
        _close(got[r]["grad_proj"], want_proj[64 * r:64 * (r + 1)], "rank %d projected-vertex gradient" % r)
    # a rank's own (un-reduced) gradient is not the global one: the all_reduce did the work
    single = bench.workload(_bench_args(64), 0, dev)
    bench.step(single)
    part = single["tex"].grad.cpu().numpy()
    assert np.abs(part - want_atlas).max() > 1e-2 * np.abs(want_atlas).max()


def test_bench_step_allreduce_8_ranks(tmp_path, dev):
    """cfg4's 8-rank form (batch=512 over 8 GPUs) rehearsed at 8 items per rank: eight gloo
    ranks on the box's one GPU run bench.py's N > 1 step (bench.workload: rank r renders items
    8r .. 8r + 7, one shared 288^2 atlas; the step ends with the all_reduce(SUM) of the atlas
    gradient).  Every rank's atlas gradient equals the gradient of the same 64 items rendered and
    differentiated in one process, and each rank's projected-vertex gradients equal that process's
    for its items (within GRAD_TOL).  The RCCL form needs 8 devices (RCCL refuses two ranks on one)."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    R, B = 8, 8
    mp.spawn(_bench_worker, args=(R, _free_port(), str(tmp_path), B), nprocs=R, join=True)
    got = [np.load(str(tmp_path / ("b%d.npz" % r))) for r in range(R)]
    w = bench.workload(_bench_args(R * B), 0, dev)
    w["g"] = torch.as_tensor(np.concatenate([got[r]["g"] for r in range(R)]), device=dev)
    bench.step(w)
    want_atlas = w["tex"].grad.cpu().numpy()
    want_proj = w["proj"].grad.cpu().numpy()
    assert float(np.abs(want_atlas).sum()) > 0
    for r in range(R):
        _close(got[r]["grad_atlas"], want_atlas, "rank %d of 8: all-reduced atlas gradient" % r)
        _close(got[r]["grad_proj"], want_proj[B * r:B * (r + 1)], "rank %d of 8: projected-vertex gradient" % r)


def _rccl_worker(rank, port, out_dir):
    """A world of one rank over the "nccl" backend (RCCL): bench.py's N > 1 process-group setup
    (bench.setup_dist's init_process_group with device_id), one headline step, and RCCL's
    all_reduce(SUM) and all_gather_into_tensor on its atlas gradient and images."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=rank, world_size=1, device_id=dev)
    try:
        import bench
        assert dist.get_backend() == "nccl"
        w = bench.workload(_bench_args(64), rank, dev)
        images = bench.step(w)
        grad = w["tex"].grad.clone()
        red = w["tex"].grad.clone()
        dist.all_reduce(red, op=dist.ReduceOp.SUM)
        out = torch.empty_like(images)
        dist.all_gather_into_tensor(out, images.detach().contiguous())
        torch.cuda.synchronize()
        np.savez(os.path.join(out_dir, "rccl.npz"), grad=grad.cpu().numpy(), red=red.cpu().numpy(),
                 same_images=bool(torch.equal(out, images.detach())))
    finally:
        dist.destroy_process_group()


def test_rccl_world1_collectives(tmp_path, dev):
    """RCCL (the "nccl" backend) on this box: a one-rank process group set up as bench.py sets up its
    ranks, one headline step, and the two collectives of the N > 1 path on its tensors -- the
    all_reduce leaves the atlas gradient unchanged (a sum over one rank) and the all_gather returns
    the images.  The box has one GPU and RCCL refuses two ranks on one device, so this is the RCCL
    runtime check; the two-rank exchange itself is covered over gloo above."""
    mp.spawn(_rccl_worker, args=(_free_port(), str(tmp_path)), nprocs=1, join=True)
    got = np.load(str(tmp_path / "rccl.npz"))
    assert float(np.abs(got["grad"]).sum()) > 0
    assert np.array_equal(got["red"], got["grad"])
    assert bool(got["same_images"])
