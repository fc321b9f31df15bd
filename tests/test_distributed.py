"""Batch sharding across ranks on CPU with gloo, world_size 2 and 8.

Each rank renders its shard of the batch (here with the CPU oracle standing in for the GPU, which
the sharding logic does not depend on), the shards are assembled with gather_images, and the
gradient of a mesh shared by all items is summed with allreduce_shared_grads.  Both must equal
the single-process full-batch result."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from neural_renderer_v2_pytorch_amd import distributed as ndist
from neural_renderer_v2_pytorch_amd import synthetic


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _scene(batch):
    """A shared mesh seen from `batch` viewpoints: vertices [V,3] (leaf) -> projected [B,V,3]."""
    v, f = synthetic.icosphere(1)
    base = torch.tensor(v * 0.6, dtype=torch.float32)
    shifts = torch.tensor([[0.07 * i - 0.1, 0.05 * (i % 2), 2.0 + 0.1 * i] for i in range(batch)],
                          dtype=torch.float32)
    return base, torch.as_tensor(f.astype(np.int32)), shifts


def _render(oracle, base, faces, shifts):
    v = base[None] + shifts[:, None, :]
    proj = torch.stack([v[..., 0] / v[..., 2], v[..., 1] / v[..., 2], v[..., 2]], -1)
    return oracle.rasterize_core(proj, faces, image_size=24, anti_aliasing=False, draw_rgb=False,
                                 draw_silhouettes=True, draw_depth=True)


def _loss(images, shifts):
    w = torch.linspace(-1.0, 1.0, images[0].numel()).reshape(images.shape[1:])
    return sum(((images[i] * w).sum() * (1.0 + 0.1 * float(shifts[i, 2]))) for i in range(images.shape[0]))


def _worker(rank, world_size, port, batch, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world_size)
    try:
        import build as oracle_build
        oracle_build.build()
        import oracle
        base, faces, shifts = _scene(batch)
        base.requires_grad_(True)
        local_shifts = ndist.shard(shifts)
        assert local_shifts.shape[0] == ndist.shard_range(batch, rank, world_size)[1] - \
            ndist.shard_range(batch, rank, world_size)[0]
        images = _render(oracle, base, faces, local_shifts)
        _loss(images, local_shifts).backward()
        ndist.allreduce_shared_grads([base])
        full = ndist.gather_images(images.detach())
        full_known = ndist.gather_images(images.detach(), batch_size=batch)
        np.savez(os.path.join(out_dir, "r%d.npz" % rank), images=full.numpy(), images_known=full_known.numpy(),
                 grad=base.grad.numpy())
    finally:
        dist.destroy_process_group()


def test_shard_range_covers_batch():
    for b in range(0, 11):
        for g in range(1, 9):
            rs = [ndist.shard_range(b, r, g) for r in range(g)]
            assert rs[0][0] == 0 and rs[-1][1] == b
            assert all(rs[i][1] == rs[i + 1][0] for i in range(g - 1))
            sizes = [e - s for s, e in rs]
            assert max(sizes) - min(sizes) <= 1


def test_single_process_is_identity():
    x = torch.randn(3, 4)
    assert ndist.gather_images(x) is x
    assert torch.equal(ndist.shard(x), x)


@pytest.mark.parametrize("batch", [4, 3])
def test_gloo_world2_matches_full_batch(tmp_path, oracle_mod, batch):
    mp.spawn(_worker, args=(2, _free_port(), batch, str(tmp_path)), nprocs=2, join=True)
    base, faces, shifts = _scene(batch)
    base.requires_grad_(True)
    images = _render(oracle_mod, base, faces, shifts)
    _loss(images, shifts).backward()
    for r in range(2):
        got = np.load(str(tmp_path / ("r%d.npz" % r)))
        assert np.array_equal(got["images"], images.detach().numpy())
        assert np.array_equal(got["images_known"], images.detach().numpy())
        np.testing.assert_allclose(got["grad"], base.grad.numpy(), rtol=1e-5, atol=1e-6)
    assert float(base.grad.abs().sum()) > 0


@pytest.mark.parametrize("batch", [16, 13])
def test_gloo_world8_matches_full_batch(tmp_path, oracle_mod, batch):
    """cfg4's form (one rank per GPU of an 8-GPU node) rehearsed with eight gloo
    ranks: each renders its shard (2 items each, or 1-2 for an uneven 13), the shared mesh's
    gradient is summed over the eight ranks and every rank assembles the whole batch in rank order;
    both equal the single-process full batch."""
    ws = 8
    mp.spawn(_worker, args=(ws, _free_port(), batch, str(tmp_path)), nprocs=ws, join=True)
    base, faces, shifts = _scene(batch)
    base.requires_grad_(True)
    images = _render(oracle_mod, base, faces, shifts)
    _loss(images, shifts).backward()
    for r in range(ws):
        got = np.load(str(tmp_path / ("r%d.npz" % r)))
        assert np.array_equal(got["images"], images.detach().numpy())
        assert np.array_equal(got["images_known"], images.detach().numpy())
        np.testing.assert_allclose(got["grad"], base.grad.numpy(), rtol=1e-5, atol=1e-6)
    assert float(base.grad.abs().sum()) > 0


def _group_worker(rank, world_size, port, out_dir):
    """Subgroup collectives and a rank with no gradient (distributed.py: world(group),
    allreduce_shared_grads' zero contribution)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world_size)
    try:
        group = dist.new_group([0, 2])  # every rank creates it, as torch requires
        res = {}
        if rank in (0, 2):
            grank, gws = ndist.world(group)
            assert gws == 2 and grank == (0 if rank == 0 else 1)
            batch = 5
            lo, hi = ndist.shard_range(batch, grank, gws)
            local = torch.arange(lo, hi, dtype=torch.float32)[:, None].repeat(1, 3)
            res["gathered"] = ndist.gather_images(local, group=group).numpy()
            res["gathered_known"] = ndist.gather_images(local, batch_size=batch, group=group).numpy()
        # a shared parameter whose grad is None on rank 1 (an empty shard): every rank still
        # enters the all_reduce and the sum is that of the ranks that had a gradient
        p = torch.zeros(4, requires_grad=True)
        if rank != 1:
            (p * float(rank + 1)).sum().backward()
        frozen = torch.ones(3)  # requires_grad False: skipped on every rank, .grad stays None
        ndist.allreduce_shared_grads([p, frozen, None])
        assert frozen.grad is None
        res["grad"] = p.grad.numpy()
        if rank == 1:  # not in `group`: a clear error instead of shard math with rank -1
            try:
                ndist.world(group)
            except ValueError:
                res["outside_raises"] = np.array(1)
            try:
                ndist.gather_images(torch.zeros(1, 3), group=group)
            except ValueError:
                res["gather_outside_raises"] = np.array(1)
        np.savez(os.path.join(out_dir, "g%d.npz" % rank), **res)
    finally:
        dist.destroy_process_group()


def test_gloo_subgroup_and_missing_grad(tmp_path):
    mp.spawn(_group_worker, args=(3, _free_port(), str(tmp_path)), nprocs=3, join=True)
    want = np.repeat(np.arange(5, dtype=np.float32)[:, None], 3, 1)
    for r in range(3):
        got = np.load(str(tmp_path / ("g%d.npz" % r)))
        np.testing.assert_array_equal(got["grad"], np.full(4, 1.0 + 3.0, np.float32))
        if r == 1:
            assert int(got["outside_raises"]) == 1 and int(got["gather_outside_raises"]) == 1
        if r != 1:
            np.testing.assert_array_equal(got["gathered"], want)
            np.testing.assert_array_equal(got["gathered_known"], want)
