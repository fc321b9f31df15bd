"""Parity of the HIP path (through the C ABI) with the reference, on the GPU.

Golden vectors: tests/golden/*.npz, produced by the reference implementation itself
(tests/golden/make_golden.py).  Large sizes are checked against the CPU oracle (oracle/).

Tolerances (north star: face_index_map bit-exact; fp32 tolerance elsewhere):
  * face_index_map, weight_map:   bit-exact
  * images (rgb, depth, sil):     |d| <= 1e-5 + 1e-5 |ref|
  * gradients (vertices, textures): |d| <= 1e-4 max|ref| + 1e-4 |ref| per element; float atomics
    sum in a different order than the reference's index_put_ scatter.
"""
import os
import numpy as np
import pytest
import torch

import neural_renderer_v2_pytorch_amd as nr
from neural_renderer_v2_pytorch_amd import rasterize as nrr
from neural_renderer_v2_pytorch_amd import synthetic
from neural_renderer_v2_pytorch_amd import _lib

pytestmark = pytest.mark.gpu

IMG_RTOL = IMG_ATOL = 1e-5
GRAD_TOL = 1e-4


def close_images(a, b, what):
    a = torch.as_tensor(a).detach().cpu().double()
    b = torch.as_tensor(b).detach().cpu().double()
    assert a.shape == b.shape, (what, a.shape, b.shape)
    err = (a - b).abs()
    bad = err > IMG_ATOL + IMG_RTOL * b.abs()
    assert not bad.any(), "%s: %d elements off, max |d| %g" % (what, int(bad.sum()), float(err.max()))


def close_grads(a, b, what):
    a = torch.as_tensor(a).detach().cpu().double()
    b = torch.as_tensor(b).detach().cpu().double()
    assert a.shape == b.shape, (what, a.shape, b.shape)
    scale = float(b.abs().max())
    err = (a - b).abs()
    bad = err > GRAD_TOL * scale + GRAD_TOL * b.abs()
    assert not bad.any(), "%s: %d of %d elements off, max |d| %g (scale %g)" % (
        what, int(bad.sum()), bad.numel(), float(err.max()), scale)


def flags_of(name):
    if "rgbsd" in name:
        return dict(draw_rgb=True, draw_silhouettes=True, draw_depth=True)
    if "rgba" in name:
        return dict(draw_rgb=True, draw_silhouettes=True, draw_depth=False)
    return dict(draw_rgb=True, draw_silhouettes=False, draw_depth=False)


@pytest.mark.parametrize("name", ["teapot_rgbsd_aa", "teapot_rgb_nobs", "teapot_rgba_aa", "ico_rgbsd_aa"])
def test_textured_scene(golden, dev, name):
    d = golden(name)
    B = d["proj"].shape[0]
    proj = torch.as_tensor(d["proj"], device=dev).requires_grad_(True)
    tex_leaf = torch.as_tensor(d["textures"], device=dev).requires_grad_(True)
    if int(d["shared_textures"]):
        tex = tex_leaf[None].expand(B, *tex_leaf.shape)
        vt = torch.as_tensor(d["vertices_textures"], device=dev)[None].expand(B, -1, -1)
    else:
        tex = tex_leaf
        vt = torch.as_tensor(d["vertices_textures"], device=dev)
    params = nr.RasterizeParam(vertices_textures=vt, faces_textures=torch.as_tensor(d["faces_textures"], device=dev),
                               textures=tex)
    hp = nr.RasterizeHyperparam(image_size=int(d["image_size"]), anti_aliasing=bool(d["anti_aliasing"]),
                                draw_backside=bool(d["draw_backside"]), **flags_of(name))
    img, fim = nrr.rasterize_core(proj, torch.as_tensor(d["faces"], device=dev), params, hp, return_face_index=True)
    assert torch.equal(fim.cpu(), torch.as_tensor(d["fim"])), "face_index_map not bit-exact"
    close_images(img, d["images"], name + " images")
    img.backward(torch.as_tensor(d["grad_up"], device=dev))
    close_grads(proj.grad, d["grad_proj"], name + " grad vertices")
    close_grads(tex_leaf.grad, d["grad_textures"], name + " grad textures")


@pytest.mark.parametrize("name", ["teapot_rgbsd_aa", "ico_rgbsd_aa"])
def test_textured_scene_unpacked_textures(golden, dev, name):
    """The same goldens with the texels sampled straight from the [B, 3, H, W] textures instead of
    the forward's RGBA-packed copy (NrRasterArgs.textures_packed = NULL): both layouts are exact."""
    try:
        nrr._TEX_PACK = False
        test_textured_scene(golden, dev, name)
    finally:
        nrr._TEX_PACK = True


def test_wrappers_match_core(golden, dev):
    """rasterize_rgba / rasterize_rgb set the draw flags on the passed hyperparams (rasterize.py:341-356)."""
    d = golden("teapot_rgba_aa")
    B = d["proj"].shape[0]
    proj = torch.as_tensor(d["proj"], device=dev)
    tex = torch.as_tensor(d["textures"], device=dev)[None].expand(B, -1, -1, -1)
    vt = torch.as_tensor(d["vertices_textures"], device=dev)[None].expand(B, -1, -1)
    params = nr.RasterizeParam(vertices_textures=vt, faces_textures=torch.as_tensor(d["faces_textures"], device=dev),
                               textures=tex)
    hp = nr.RasterizeHyperparam(image_size=int(d["image_size"]), anti_aliasing=True, draw_backside=False)
    img = nr.rasterize_rgba(proj, torch.as_tensor(d["faces"], device=dev), params, hp)
    assert (hp.draw_rgb, hp.draw_silhouettes, hp.draw_depth) == (True, True, False)
    assert hp.image_size == int(d["image_size"])
    close_images(img, d["images"], "rasterize_rgba")


def test_silhouettes_teapot(golden, dev):
    d = golden("teapot_sil")
    proj = torch.as_tensor(d["proj"], device=dev).requires_grad_(True)
    hp = nr.RasterizeHyperparam(image_size=256, anti_aliasing=False)
    img = nr.rasterize_silhouettes(proj, torch.as_tensor(d["faces"]), nr.RasterizeParam(), hp)
    assert torch.equal(img.detach().cpu(), torch.as_tensor(d["images"]))
    img.backward(torch.as_tensor(d["grad_up"], device=dev))
    close_grads(proj.grad, d["grad_proj"], "teapot silhouettes grad")
    fim = nrr.compute_face_index_map(torch.as_tensor(d["proj"], device=dev)[:, torch.as_tensor(d["faces"]).long()],
                                     nr.RasterizeHyperparam(image_size=256))
    assert torch.equal(fim.cpu(), torch.as_tensor(d["fim"]))
    w = nrr.compute_weight_map(torch.as_tensor(d["proj"], device=dev)[:, torch.as_tensor(d["faces"]).long()], fim)
    assert torch.equal(w.cpu(), torch.as_tensor(d["weight_map"])), "weight_map not bit-exact"


def test_renderer_silhouettes_teapot(golden, dev):
    """Renderer path (look_at + perspective fused on the GPU, then rasterize) against the
    reference's golden, which projected the vertices with the torch CPU composition.  Observed on
    an MI355X: no silhouette pixel flips and the vertex gradient's relative L1 error is 1.7e-8, so
    the bounds are the strict ones: a bit-exact image and the per-element gradient tolerance."""
    d = golden("teapot_sil")
    ren = nr.Renderer()
    ren.anti_aliasing = False
    ren.viewpoints = nr.get_points_from_angles(2.732, 0, 0)
    v = torch.as_tensor(d["vertices"], device=dev).requires_grad_(True)
    img = ren.render_silhouettes(v, torch.as_tensor(d["faces"], device=dev))
    flips = int((img.detach().cpu() != torch.as_tensor(d["images"])).sum())
    img.backward(torch.as_tensor(d["grad_up"], device=dev))
    g, ref = v.grad.cpu(), torch.as_tensor(d["grad_vertices"])
    l1 = float((g - ref).abs().sum() / ref.abs().sum())
    print("Renderer teapot: %d of %d silhouette pixels flip; grad L1 rel %.3g" % (flips, img.numel(), l1))
    assert flips == 0, flips
    close_grads(g, ref, "Renderer teapot grad vertices")


def test_depth_teapot(golden, dev):
    d = golden("teapot_depth")
    proj = torch.as_tensor(d["proj"], device=dev).requires_grad_(True)
    hp = nr.RasterizeHyperparam(image_size=256, anti_aliasing=False)
    img = nr.rasterize_depth(proj, torch.as_tensor(d["faces"], device=dev), nr.RasterizeParam(), hp)
    close_images(img, d["images"], "depth")
    img.backward(torch.as_tensor(d["grad_up"], device=dev))
    close_grads(proj.grad, d["grad_proj"], "depth grad")


def test_square_first_step_gradient(golden, dev):
    """test_backward_case1's scene: the IoU-loss gradient of the first step (reference: +-0.0617 in x/y,
    exactly 0 in z)."""
    d = golden("square_sil")
    from PIL import Image
    import os
    ref = 1 - np.asarray(Image.open(os.path.join(os.path.dirname(__file__), "data", "gradient.png")),
                         np.float32)[:, :, 0] / 255.
    ref = torch.as_tensor(ref, device=dev)
    v = torch.as_tensor(d["vertices"], device=dev).requires_grad_(True)
    hp = nr.RasterizeHyperparam(image_size=256, anti_aliasing=False)
    img = nr.rasterize_silhouettes(v[None], torch.as_tensor(d["faces"]), nr.RasterizeParam(), hp)[0]
    assert torch.equal(img.detach().cpu(), torch.as_tensor(d["images"][0]))
    iou = torch.sum(img * ref) / torch.sum(img + ref - img * ref)
    (1 - iou).backward()
    close_grads(v.grad, d["iou_grad"], "square iou grad")
    assert torch.all(v.grad[:, 2] == 0)


def test_backward_case1_convergence(dev):
    """tests_torch/test_rasterize.py:205-249: Adam(lr=0.005) on a 2-triangle square reaches
    1 - IoU < 0.01 within 350 steps (reference on CPU oracle: step 221)."""
    import os
    from PIL import Image
    vertices = np.array([[0.1, 0.1, 1.], [-0.1, 0.1, 1.], [-0.1, -0.1, 1.], [0.1, -0.1, 1.]], 'float32')
    faces = torch.as_tensor(np.array([[0, 1, 2], [0, 2, 3]], 'int32'), device=dev)
    ref = 1 - np.asarray(Image.open(os.path.join(os.path.dirname(__file__), "data", "gradient.png")),
                         np.float32)[:, :, 0] / 255.
    ref = torch.as_tensor(ref, device=dev)
    v = torch.nn.Parameter(torch.as_tensor(vertices, device=dev))
    opt = torch.optim.Adam([v], lr=0.005)
    for i in range(350):
        hp = nr.RasterizeHyperparam(image_size=256, anti_aliasing=False)
        img = nr.rasterize_silhouettes(v[None], faces, nr.RasterizeParam(), hp)[0]
        loss = 1 - torch.sum(img * ref) / torch.sum(img + ref - img * ref)
        opt.zero_grad()
        loss.backward()
        opt.step()
        if float(loss.detach()) < 0.01:
            assert abs(i - 221) <= 10, i
            return
    raise AssertionError("did not converge")


def test_car_rgba(golden, dev):
    """test_forward_case2 / test_save_obj scene (car 4e4987...): load_obj + Renderer.render, rgba."""
    import os
    d = golden("car1_rgba")
    obj = os.path.join(os.path.dirname(__file__), "data", "4e49873292196f02574b5684eaec43e9", "model.obj")
    v, f, vt, ft, tex = nr.load_obj(obj, load_textures=True)
    assert np.array_equal(v, d["vertices"]) and np.array_equal(f, d["faces"])
    assert np.array_equal(vt, d["vertices_textures"]) and np.array_equal(ft, d["faces_textures"])
    assert list(tex.shape) == list(d["textures_shape"])
    assert abs(tex.astype(np.float64).sum() - float(d["textures_sum"])) < 1e-6 * float(d["textures_sum"])
    ren = nr.Renderer()
    ren.draw_backside = False
    ren.viewpoints = nr.get_points_from_angles(2.5, 10, -90)
    proj = torch.as_tensor(d["proj"], device=dev)
    hp = nr.RasterizeHyperparam(image_size=256, draw_backside=False)
    params = nr.RasterizeParam(vertices_textures=torch.as_tensor(vt, device=dev)[None],
                               faces_textures=torch.as_tensor(ft, device=dev), textures=torch.as_tensor(tex, device=dev)[None])
    img = nr.rasterize_rgba(proj, torch.as_tensor(f, device=dev), params, hp)
    close_images(img, d["images"], "car rgba")
    # the reference's own golden PNG (tests_torch/data/4e49...png): alpha channel
    from PIL import Image
    png = np.asarray(Image.open(os.path.join(os.path.dirname(__file__), "data",
                                             "4e49873292196f02574b5684eaec43e9.png")), np.float32) / 255.
    alpha = img[0, 3].cpu().numpy()
    assert np.abs(alpha - png[:, :, 3]).mean() < 1e-4


def test_differentiation_golden(golden, dev):
    d = golden("diff_kat")
    for i in range(3):
        images = torch.as_tensor(d["images%d" % i], device=dev)
        coords = torch.zeros(images.shape[:3] + (2,), device=dev, requires_grad=True)
        y = nr.differentiation(images, coords)
        y.backward(torch.as_tensor(d["grad%d" % i], device=dev))
        close_images(coords.grad, d["grad_xy%d" % i], "differentiation %d" % i)


def test_differentiation_reference_procedure(dev):
    """tests_torch/test_differentiation.py:10-65, verbatim procedure on the GPU implementation."""
    r = np.random.RandomState(0)
    images = torch.as_tensor(r.normal(size=(10, 32, 32, 3)).astype('float32'), device=dev)
    x = np.tile(np.arange(32).astype('float32')[None, None, :, None], (10, 32, 1, 1))
    y = np.tile(np.arange(32).astype('float32')[None, :, None, None], (10, 1, 32, 1))
    coordinates = ((np.concatenate((x, y), axis=-1) / 31) * 2 - 1) * 31. / 32.
    noise = torch.as_tensor(r.normal(size=(10, 32, 32, 3)).astype('float32'), device=dev)
    step = 2 / 32.
    coordinates = torch.tensor(coordinates, device=dev, requires_grad=True)
    torch.sum(nr.differentiation(images, coordinates) * noise).backward()
    g = coordinates.grad
    for _ in range(100):
        yi, xi = r.randint(1, 31), r.randint(1, 31)
        pairs = []
        for axis in (1, 0):
            for sgn in (1, -1):
                im = images.clone()
                if axis == 1:
                    im[:, yi - sgn, xi] = images[:, yi, xi]
                    im[:, yi, xi] = images[:, yi + sgn, xi]
                else:
                    im[:, yi, xi - sgn] = images[:, yi, xi]
                    im[:, yi, xi] = images[:, yi, xi + sgn]
                gg = ((im - images) * noise).sum((1, 2, 3)) / step
                pairs.append(torch.min(gg, torch.zeros_like(gg)))
        gy = torch.max(pairs[0].abs(), pairs[1].abs())
        gx = torch.max(pairs[2].abs(), pairs[3].abs())
        assert torch.allclose(gy, g[:, yi, xi, 1].abs().to(gy.dtype), rtol=1e-4, atol=0)
        assert torch.allclose(gx, g[:, yi, xi, 0].abs().to(gx.dtype), rtol=1e-4, atol=0)


def test_edges_face_index(golden, dev):
    d = golden("edges")
    for i in range(3):
        faces = torch.as_tensor(d["faces%d" % i], device=dev)
        S = d["fim%d_1" % i].shape[1]
        for bs in (0, 1):
            hp = nr.RasterizeHyperparam(image_size=S, draw_backside=bool(bs))
            fim = nrr.compute_face_index_map(faces, hp)
            ref = torch.as_tensor(d["fim%d_%d" % (i, bs)])
            assert torch.equal(fim.cpu(), ref), "edges %d backside %d: %d px differ" % (
                i, bs, int((fim.cpu() != ref).sum()))
            w = nrr.compute_weight_map(faces, fim)
            np.testing.assert_array_equal(w.cpu().numpy(), d["weight%d_%d" % (i, bs)])


def _ico_batch(level, B, dev):
    v, f = synthetic.icosphere(level)
    vb = torch.as_tensor(synthetic.jittered(v, B))
    proj = synthetic.project(vb, torch.as_tensor(synthetic.viewpoints(B)))
    return proj, f


@pytest.mark.parametrize("S,level,B", [(512, 4, 2), (1000, 3, 1), (130, 4, 3), (1100, 2, 1)])
def test_face_index_large_vs_oracle(oracle_mod, dev, S, level, B):
    """Headline-size face-index map (ico-sphere 5120 faces, 512^2 internal) bit-exact against the
    brute-force CPU oracle; plus a non-multiple-of-tile size and a size past the LDS bin-mask path
    of k_face_setup (S > 1024)."""
    proj, f = _ico_batch(level, B, dev)
    fg = proj[:, torch.as_tensor(f).long()].contiguous()
    fim = nrr.compute_face_index_map(fg.to(dev), nr.RasterizeHyperparam(image_size=S))
    ref = oracle_mod.face_index_map(fg, S)
    assert np.array_equal(fim.cpu().numpy(), ref), int((fim.cpu().numpy() != ref).sum())


@pytest.mark.parametrize("S,F,seed", [(64, 1500, 0), (96, 3000, 1), (64, 400, 2)])
def test_face_index_dense_snapped_soup(oracle_mod, dev, S, F, seed):
    """Deep bins (tens of faces over every 8x8 block, so k_raster_fwd's edge cull runs) of triangles
    whose vertices sit exactly on pixel centres, many with an axis-aligned edge 1-2: along that
    edge's line the reference's c2 is exactly 0, so its edge tests (.cu:107-116) pass pixels outside
    the triangle, which may then win the z-test.  Bit-exact against the brute-force oracle, through
    both the fused path's setup (vertices) and the caller-gathered entry point."""
    r = np.random.RandomState(seed)
    B = 2
    centres = ((2 * np.arange(S) + 1 - S) / S).astype(np.float32)
    ix = r.randint(0, S, size=(B, F, 3))
    iy = r.randint(0, S, size=(B, F, 3))
    flat = r.rand(B, F) < 0.5
    iy[:, :, 2] = np.where(flat, iy[:, :, 1], iy[:, :, 2])           # edge 1-2 horizontal
    ix[:, :, 2] = np.where(~flat & (r.rand(B, F) < 0.5), ix[:, :, 1], ix[:, :, 2])  # or vertical
    # small triangles: the other corners within 6 pixels of corner 0
    ix[:, :, 1:] = np.clip(ix[:, :, :1] + (ix[:, :, 1:] % 13) - 6, 0, S - 1)
    iy[:, :, 1:] = np.clip(iy[:, :, :1] + (iy[:, :, 1:] % 13) - 6, 0, S - 1)
    if True:  # keep the horizontal / vertical edges after the clipping
        iy[:, :, 2] = np.where(flat, iy[:, :, 1], iy[:, :, 2])
    z = r.uniform(0.5, 5.0, size=(B, F, 3)).astype(np.float32)
    fg = np.stack([centres[ix], centres[iy], z], -1).astype(np.float32)  # [B, F, 3, 3]
    ref = oracle_mod.face_index_map(torch.as_tensor(fg), S)
    fim = nrr.compute_face_index_map(torch.as_tensor(fg, device=dev), nr.RasterizeHyperparam(image_size=S))
    assert np.array_equal(fim.cpu().numpy(), ref), int((fim.cpu().numpy() != ref).sum())
    # fused path: the same faces as a vertex list
    verts = torch.as_tensor(fg.reshape(B, F * 3, 3), device=dev)
    faces = torch.arange(F * 3, dtype=torch.int32, device=dev).reshape(F, 3)
    hp = nr.RasterizeHyperparam(image_size=S, anti_aliasing=False)
    hp.draw_rgb = False
    _, fim2 = nrr.rasterize_core(verts, faces, nr.RasterizeParam(), hp, return_face_index=True)
    assert np.array_equal(fim2.cpu().numpy(), ref), int((fim2.cpu().numpy() != ref).sum())


@pytest.mark.parametrize("zlevels", [0, 3])
def test_face_index_deep_stack_depth_cull(oracle_mod, dev, zlevels):
    """Bins of 1000+ small faces at random depths (zlevels > 0: only that many distinct depths, so
    many faces tie within depth_min_delta): the deep variant's deep-first order, its empty-bin skip,
    its dealt 4x4 quarters (per-pixel state in LDS across the staging rounds) and its wave-level depth
    cull (k_raster_fwd walk_block<..., ZCULL>, bins of >= 512 candidates) drop faces behind every
    pixel of a wave in the ballot; bit-exact against the brute-force oracle."""
    r = np.random.RandomState(7 + zlevels)
    S, F, B = 64, 4000, 2
    cx = r.uniform(-0.9, 0.9, size=(B, F, 1))
    cy = r.uniform(-0.9, 0.9, size=(B, F, 1))
    x = (cx + r.uniform(-0.12, 0.12, size=(B, F, 3))).astype(np.float32)
    y = (cy + r.uniform(-0.12, 0.12, size=(B, F, 3))).astype(np.float32)
    if zlevels:
        z = np.repeat(r.choice(np.linspace(1.0, 3.0, zlevels), size=(B, F, 1)), 3, axis=2).astype(np.float32)
    else:
        z = r.uniform(0.5, 5.0, size=(B, F, 3)).astype(np.float32)
    x[1] = np.abs(cx[1]) + 0.15 + (x[1] - cx[1])  # item 1: nothing in its left bins (empty, flagged)
    fg = np.stack([x, y, z], -1).astype(np.float32)
    ref = oracle_mod.face_index_map(torch.as_tensor(fg), S)
    verts = torch.as_tensor(fg.reshape(B, F * 3, 3), device=dev)
    faces = torch.arange(F * 3, dtype=torch.int32, device=dev).reshape(F, 3)
    hp = nr.RasterizeHyperparam(image_size=S, anti_aliasing=False)
    hp.draw_rgb = False
    _, fim = nrr.rasterize_core(verts, faces, nr.RasterizeParam(), hp, return_face_index=True)
    ntf, flags = _lib.last_launch("k_raster_fwd")
    # (not split, B % 8 != 0: the deep bins' quarters dealt to the waves, each deep bin walked by four
    # quadrant blocks)
    assert ntf == 1024 and flags & _lib.NR_LAUNCH_DEEP_FIRST and flags & _lib.NR_LAUNCH_DEALT_QUARTERS, (ntf, flags)
    assert flags & _lib.NR_LAUNCH_QUADRANTS, flags
    assert np.array_equal(fim.cpu().numpy(), ref), int((fim.cpu().numpy() != ref).sum())
    assert (ref[1] >= 0).any() and (ref[1] < 0).any()


@pytest.mark.parametrize("B", [1, 8])
def test_quadrant_split_over_cap_vs_oracle(oracle_mod, dev, B):
    """More deep bins per deep-first list than the quadrant split takes (NR_QS_CAP = 16): the deepest
    16 of each list are walked by four quadrant blocks each (ordered_bin part 3), the rest by one
    block with dealt quarters, and every quarter walk takes four faces per step (walk_quarter4); one
    list (B = 1, fused silhouettes + depth) and one list per XCD (B = 8, the face-index map alone, a
    forward that does not split); bit-exact against the brute-force oracle, with depth ties."""
    r = np.random.RandomState(31 + B)
    S, F = 192, 16000
    cx = r.uniform(-0.95, 0.95, size=(B, F, 1))
    cy = r.uniform(-0.95, 0.95, size=(B, F, 1))
    x = (cx + r.uniform(-0.12, 0.12, size=(B, F, 3))).astype(np.float32)
    y = (cy + r.uniform(-0.12, 0.12, size=(B, F, 3))).astype(np.float32)
    z = r.uniform(0.5, 5.0, size=(B, F, 3)).astype(np.float32)
    z[:, ::7] = np.float32(2.0)  # every seventh face flat at one depth: ties within depth_min_delta
    fg = np.stack([x, y, z], -1).astype(np.float32)
    ref = oracle_mod.face_index_map(torch.as_tensor(fg), S)
    if B == 1:
        verts = torch.as_tensor(fg.reshape(B, F * 3, 3), device=dev)
        faces = torch.arange(F * 3, dtype=torch.int32, device=dev).reshape(F, 3)
        hp = nr.RasterizeHyperparam(image_size=S, anti_aliasing=False)
        hp.draw_rgb = False
        _, fim = nrr.rasterize_core(verts, faces, nr.RasterizeParam(), hp, return_face_index=True)
    else:
        fim = nrr.compute_face_index_map(torch.as_tensor(fg, device=dev), nr.RasterizeHyperparam(image_size=S))
    ntf, flags = _lib.last_launch("k_raster_fwd")
    assert ntf == 1024 and flags & _lib.NR_LAUNCH_QUADRANTS and not flags & _lib.NR_LAUNCH_SPLIT, (ntf, flags)
    assert np.array_equal(fim.cpu().numpy(), ref), int((fim.cpu().numpy() != ref).sum())


def test_sparse_groups_cap_dense_fallback_vs_oracle(oracle_mod, dev):
    """A deep-first forward that does not split with more face groups than the sparse-group path takes
    (200k faces: 1042 groups of 192 > 1024, one forward thread per group): the setup writes the dense
    masks and the forward reads them whole, with the quadrant blocks and the four-face quarter walk;
    bit-exact against the brute-force oracle (and the same faces at 160k, 834 groups, through the sparse
    groups)."""
    r = np.random.RandomState(41)
    S = 64
    for F in (200000, 160000):
        cx = r.uniform(-0.9, 0.9, size=(1, F, 1))
        cy = r.uniform(-0.9, 0.9, size=(1, F, 1))
        x = (cx + r.uniform(-0.05, 0.05, size=(1, F, 3))).astype(np.float32)
        y = (cy + r.uniform(-0.05, 0.05, size=(1, F, 3))).astype(np.float32)
        z = r.uniform(0.5, 5.0, size=(1, F, 3)).astype(np.float32)
        fg = np.stack([x, y, z], -1).astype(np.float32)
        ref = oracle_mod.face_index_map(torch.as_tensor(fg), S)
        fim = nrr.compute_face_index_map(torch.as_tensor(fg, device=dev), nr.RasterizeHyperparam(image_size=S))
        ntf, flags = _lib.last_launch("k_raster_fwd")
        assert ntf == 1024 and flags & _lib.NR_LAUNCH_QUADRANTS, (F, ntf, flags)
        assert np.array_equal(fim.cpu().numpy(), ref), (F, int((fim.cpu().numpy() != ref).sum()))


def test_split_forward_capped_vs_oracle(oracle_mod, dev):
    """The split forward (fused, anti-aliased, B % 8 == 0): every bin holds 1000+ candidates, so each
    deep-first list's deep prefix is capped (a quarter of the items' bins may go to the 1024-thread
    launch) and the remaining deep bins run in the 256-thread launch on the side stream, in its
    multi-round static path; the face-index map is bit-exact against the oracle and the silhouette
    and depth images match the ones the unsplit forward of the same faces gives item by item."""
    r = np.random.RandomState(11)
    S, F, B = 64, 4000, 16
    cx = r.uniform(-0.9, 0.9, size=(B, F, 1))
    cy = r.uniform(-0.9, 0.9, size=(B, F, 1))
    x = (cx + r.uniform(-0.12, 0.12, size=(B, F, 3))).astype(np.float32)
    y = (cy + r.uniform(-0.12, 0.12, size=(B, F, 3))).astype(np.float32)
    z = r.uniform(0.5, 5.0, size=(B, F, 3)).astype(np.float32)
    fg = np.stack([x, y, z], -1).astype(np.float32)
    ref = oracle_mod.face_index_map(torch.as_tensor(fg), S)
    verts = torch.as_tensor(fg.reshape(B, F * 3, 3), device=dev)
    faces = torch.arange(F * 3, dtype=torch.int32, device=dev).reshape(F, 3)
    hp = nr.RasterizeHyperparam(image_size=S // 2, anti_aliasing=True)
    hp.draw_rgb = False
    img, fim = nrr.rasterize_core(verts, faces, nr.RasterizeParam(), hp, return_face_index=True)
    ntf, flags = _lib.last_launch("k_raster_fwd")
    assert ntf == 1024 and flags & _lib.NR_LAUNCH_SPLIT, (ntf, flags)
    assert np.array_equal(fim.cpu().numpy(), ref), int((fim.cpu().numpy() != ref).sum())
    # items 0-7 alone: B % 8 == 0 still, but no cap (Bcap = 8 = B): the same images
    img8, fim8 = nrr.rasterize_core(verts[:8].contiguous(), faces, nr.RasterizeParam(), hp, return_face_index=True)
    assert torch.equal(fim8, fim[:8]) and torch.equal(img8, img[:8])


def test_split_forward_from_exiting_threads(dev):
    """The split forward's side stream is per host thread and released when the thread ends
    (nr_raster.hip SideStreamTable): split forwards rendered from three worker threads that start,
    render and exit one after another, then again from this thread, all give the same images and
    face-index maps (the streams and events of the ended threads are destroyed, not reused)."""
    import threading
    r = np.random.RandomState(12)
    S, F, B = 64, 4000, 16
    cx = r.uniform(-0.9, 0.9, size=(B, F, 1))
    cy = r.uniform(-0.9, 0.9, size=(B, F, 1))
    x = (cx + r.uniform(-0.12, 0.12, size=(B, F, 3))).astype(np.float32)
    y = (cy + r.uniform(-0.12, 0.12, size=(B, F, 3))).astype(np.float32)
    z = r.uniform(0.5, 5.0, size=(B, F, 3)).astype(np.float32)
    verts = torch.as_tensor(np.stack([x, y, z], -1).reshape(B, F * 3, 3), device=dev)
    faces = torch.arange(F * 3, dtype=torch.int32, device=dev).reshape(F, 3)

    def render():
        hp = nr.RasterizeHyperparam(image_size=S // 2, anti_aliasing=True)
        hp.draw_rgb = False
        img, fim = nrr.rasterize_core(verts, faces, nr.RasterizeParam(), hp, return_face_index=True)
        flags = _lib.last_launch("k_raster_fwd")[1]
        torch.cuda.synchronize()
        return img.cpu(), fim.cpu(), flags

    want = render()
    assert want[2] & _lib.NR_LAUNCH_SPLIT
    got = []
    for _ in range(3):
        th = threading.Thread(target=lambda: got.append(render()))
        th.start()
        th.join()
    got.append(render())
    assert len(got) == 4
    for img, fim, flags in got:
        assert flags & _lib.NR_LAUNCH_SPLIT
        assert torch.equal(img, want[0]) and torch.equal(fim, want[1])


def test_headline_properties(dev):
    """Full headline config (B=64, 256^2 AA, ico 5120, rgb+sil+depth): size-independent properties."""
    B = 64
    proj, f = _ico_batch(4, B, dev)
    vt, ft, tex = nr.create_textures(f.shape[0], texture_size=4)
    tex = torch.rand(tex.shape, device=dev, generator=torch.Generator(device=dev).manual_seed(3), requires_grad=True)
    pv = proj.to(dev).requires_grad_(True)
    params = nr.RasterizeParam(vertices_textures=torch.as_tensor(vt, device=dev)[None].expand(B, -1, -1),
                               faces_textures=torch.as_tensor(ft, device=dev), textures=tex[None].expand(B, -1, -1, -1))
    img, fim = nrr.rasterize_core(pv, torch.as_tensor(f, device=dev), params, nr.RasterizeHyperparam(),
                                  return_face_index=True)
    assert img.shape == (B, 5, 256, 256)
    sil = img[:, 3]
    # silhouette = 2x2 average of the flipped (fim >= 0) mask
    m = (fim >= 0).float().flip(1, 2)
    m = (m[:, 0::2, 0::2] + m[:, 1::2, 0::2] + m[:, 0::2, 1::2] + m[:, 1::2, 1::2]) / 4
    assert torch.equal(sil, m)
    assert torch.isfinite(img).all()
    assert float(img[:, :3].min()) >= 0 and float(img[:, :3].max()) <= 1 + 1e-6
    # item independence: rendering item 5 alone gives the same item-5 output
    params1 = nr.RasterizeParam(vertices_textures=torch.as_tensor(vt, device=dev)[None],
                                faces_textures=torch.as_tensor(ft, device=dev), textures=tex[None])
    img1 = nrr.rasterize_core(pv[5:6].detach(), torch.as_tensor(f, device=dev), params1, nr.RasterizeHyperparam())
    assert torch.equal(img1[0], img[5].detach())
    g = torch.randn_like(img)
    img.backward(g)
    assert torch.isfinite(pv.grad).all() and torch.isfinite(tex.grad).all()
    # repeatability: same inputs -> same gradients up to float-atomic summation order
    # (not linearity: utils.maximum's |R - L| < 1e-4 threshold is not scale invariant)
    pv2 = proj.to(dev).requires_grad_(True)
    img2 = nrr.rasterize_core(pv2, torch.as_tensor(f, device=dev), params, nr.RasterizeHyperparam())
    assert torch.equal(img2, img)
    img2.backward(g)
    assert float((pv2.grad - pv.grad).abs().max()) <= 1e-4 * float(pv.grad.abs().max())


def oracle_batch(oracle_mod, proj, f, g, image_size=256, tex=None, vt=None, ft=None, items=None, chunk=8, **kw):
    """The CPU oracle over `items` of a batch (all by default), `chunk` items per call: (images,
    fim, grad vertices, grad of the shared texture).  The texture is one leaf expanded over every
    chunk, so its gradient accumulates over the items as the reference's expand backward sums the
    batch's index_put_ scatter (rasterize.py:144-148, utils.py:104-114)."""
    items = list(range(proj.shape[0])) if items is None else list(items)
    tx = tex.detach().cpu().clone().requires_grad_(True) if tex is not None else None
    imgs, fims, gvs = [], [], []
    for c in range(0, len(items), chunk):
        idx = items[c:c + chunk]
        pc = proj[idx].detach().cpu().clone().requires_grad_(True)
        extra = {}
        if tx is not None:
            extra = dict(vertices_textures=torch.as_tensor(vt)[None].expand(len(idx), -1, -1), faces_textures=ft,
                         textures=tx[None].expand(len(idx), -1, -1, -1))
        ref, internals = oracle_mod.rasterize_core(pc, f, image_size=image_size, return_internals=True, **extra, **kw)
        ref.backward(g[idx].cpu())
        imgs.append(ref.detach())
        fims.append(internals["fim"].numpy())
        gvs.append(pc.grad)
    return torch.cat(imgs), np.concatenate(fims), torch.cat(gvs), (tx.grad if tx is not None else None)


def test_headline_full_batch_vs_oracle(oracle_mod, dev):
    """The full headline batch (B=64, 256^2 AA, ico 5120, rgb+sil+depth, shared texture atlas),
    rendered and differentiated in one batched call, against the CPU oracle on all 64 items:
    face-index map bit-exact, images and per-item vertex gradients within the stated tolerances,
    and the shared texture's gradient -- the sum over the 64 items of the reference's index_put_
    scatter through to_map (rasterize.py:144-148, utils.py:104-114), which is what the headline
    bench produces -- against the oracle's sum.  Also asserts the kernel variants that ran (the
    fused 256-thread forward and the 2-pixel-per-lane backward, both with compile-time channels)."""
    B = 64
    proj, f = _ico_batch(4, B, dev)
    vt, ft, tex = nr.create_textures(f.shape[0], texture_size=4)
    tex_cpu = torch.rand(tex.shape, generator=torch.Generator().manual_seed(3))
    leaf = tex_cpu.to(dev).requires_grad_(True)
    pv = proj.to(dev).requires_grad_(True)
    params = nr.RasterizeParam(vertices_textures=torch.as_tensor(vt, device=dev)[None].expand(B, -1, -1),
                               faces_textures=torch.as_tensor(ft, device=dev), textures=leaf[None].expand(B, -1, -1, -1))
    img, fim = nrr.rasterize_core(pv, torch.as_tensor(f, device=dev), params, nr.RasterizeHyperparam(),
                                  return_face_index=True)
    assert _lib.last_launch("k_raster_fwd") == (256, _lib.NR_LAUNCH_FUSED_SHADE | _lib.NR_LAUNCH_STATIC_CHANNELS)
    g = torch.randn(img.shape, generator=torch.Generator().manual_seed(11))
    img.backward(g.to(dev))
    torch.cuda.synchronize()
    assert _lib.last_launch("k_raster_bwd") == (256, _lib.NR_LAUNCH_STATIC_CHANNELS | _lib.NR_LAUNCH_TWO_PX_PER_LANE)
    ref, rfim, rgv, rgt = oracle_batch(oracle_mod, proj, f, g, 256, tex_cpu, vt, ft)
    got = fim.cpu().numpy()
    for i in range(B):
        assert np.array_equal(got[i], rfim[i]), "item %d fim: %d px" % (i, int((got[i] != rfim[i]).sum()))
        close_images(img[i:i + 1], ref[i:i + 1], "item %d images" % i)
        close_grads(pv.grad[i:i + 1], rgv[i:i + 1], "item %d grad vertices" % i)
    assert int((rfim >= 0).sum()) > 0.2 * rfim.size
    close_grads(leaf.grad, rgt, "shared texture gradient (sum over 64 items)")


def test_sparse_face_index_forward_vs_oracle(oracle_mod, dev):
    """The forward whose face-index map stays internal (return_face_index=False, halo cache on)
    leaves the -1 entries of bins without candidate faces unwritten (NrRasterArgs.face_index_sparse);
    the backward must read none of them.  The map is filled with face id 0 before the forward, so a
    read of an unwritten entry would add face 0's gradient at a background pixel: images and
    gradients of 8 headline items (ico 5120, 256^2 AA, rgb + sil + depth, shared texture) against
    the oracle, and against the same render with the full map (return_face_index=True)."""
    B = 8
    proj, f = _ico_batch(4, B, dev)
    vt, ft, tex = nr.create_textures(f.shape[0], texture_size=4)
    tex_cpu = torch.rand(tex.shape, generator=torch.Generator().manual_seed(5))
    g = torch.randn((B, 5, 256, 256), generator=torch.Generator().manual_seed(6))
    out = {}
    for want_fim in (False, True):
        leaf = tex_cpu.to(dev).requires_grad_(True)
        pv = proj.to(dev).requires_grad_(True)
        params = nr.RasterizeParam(vertices_textures=torch.as_tensor(vt, device=dev)[None].expand(B, -1, -1),
                                   faces_textures=torch.as_tensor(ft, device=dev),
                                   textures=leaf[None].expand(B, -1, -1, -1))
        nrr._FIM_FILL = 0
        try:
            img = nrr.rasterize_core(pv, torch.as_tensor(f, device=dev), params, nr.RasterizeHyperparam(),
                                     return_face_index=want_fim)
        finally:
            nrr._FIM_FILL = None
        if want_fim:
            img = img[0]
        img.backward(g.to(dev))
        out[want_fim] = (img.detach(), pv.grad, leaf.grad)
    assert torch.equal(out[False][0], out[True][0])
    ref, rfim, rgv, rgt = oracle_batch(oracle_mod, proj, f, g, 256, tex_cpu, vt, ft)
    assert int((rfim < 0).sum()) > 0.5 * rfim.size  # most of the map is background
    for k in (False, True):
        close_images(out[k][0], ref, "images (full map %d)" % k)
        close_grads(out[k][1], rgv, "grad vertices (full map %d)" % k)
        close_grads(out[k][2], rgt, "grad textures (full map %d)" % k)


def test_tiny_depth_faces_vs_oracle(oracle_mod, dev):
    """Faces whose z + 1e-10 does not round to z (FACE_ZQ_EQ clear: the texture sampling divides by
    z + 1e-10 itself) beside faces where it does (the depth's w / z terms are reused), mixed within
    waves: every even vertex's z scaled by 2^-12 (near lowered to 1e-5), a 32-item batch through the
    fused C = 5 forward and backward, items 0 and 31 against the CPU oracle."""
    B = 32
    proj, f = _ico_batch(4, B, dev)
    proj = proj.clone()
    proj[:, 0::2, 2] *= 2.0 ** -12
    vt, ft, tex = nr.create_textures(f.shape[0], texture_size=4)
    tex_cpu = torch.rand(tex.shape, generator=torch.Generator().manual_seed(5))
    tex = tex_cpu.to(dev)
    pv = proj.to(dev).requires_grad_(True)
    params = nr.RasterizeParam(vertices_textures=torch.as_tensor(vt, device=dev)[None].expand(B, -1, -1),
                               faces_textures=torch.as_tensor(ft, device=dev), textures=tex[None].expand(B, -1, -1, -1))
    img, fim = nrr.rasterize_core(pv, torch.as_tensor(f, device=dev), params, nr.RasterizeHyperparam(near=1e-5),
                                  return_face_index=True)
    assert bool((fim >= 0).any())
    g = torch.randn(img.shape, generator=torch.Generator().manual_seed(12))
    img.backward(g.to(dev))
    for i in (0, B - 1):
        pc = proj[i:i + 1].clone().requires_grad_(True)
        ref, internals = oracle_mod.rasterize_core(pc, f, image_size=256, near=1e-5,
                                                   vertices_textures=torch.as_tensor(vt)[None], faces_textures=ft,
                                                   textures=tex_cpu[None], return_internals=True)
        ref.backward(g[i:i + 1])
        assert np.array_equal(fim[i].cpu().numpy(), internals["fim"][0].numpy()), "item %d fim" % i
        close_images(img[i:i + 1], ref, "item %d images" % i)
        close_grads(pv.grad[i:i + 1], pc.grad, "item %d grad vertices" % i)


@pytest.mark.parametrize("mode", ["sil", "depth", "rgba", "rgbsd"])
def test_fused_forward_shading_matches_separate_shade(dev, mode):
    """A 32-item batch at 256^2 AA takes the forward with shading fused into the face-index kernel
    (k_raster_fwd<256, true>: >= 8192 bins, shallow bins); a single item takes the 1024-thread
    face-index kernel plus k_shade_px.  Same images bit for bit, and the same per-item vertex
    gradients within the gradient tolerance (the halo cache is written by the fused epilogue in
    the batch and by k_shade_px alone)."""
    B = 32
    proj, f = _ico_batch(4, B, dev)
    ft_ = torch.as_tensor(f, device=dev)
    hp = nr.RasterizeHyperparam()
    hp.draw_rgb = mode in ("rgba", "rgbsd")
    hp.draw_silhouettes = mode in ("sil", "rgba", "rgbsd")
    hp.draw_depth = mode in ("depth", "rgbsd")
    params = nr.RasterizeParam()
    params1 = nr.RasterizeParam()
    if hp.draw_rgb:
        vt, ft, tex = nr.create_textures(f.shape[0], texture_size=4)
        tex = torch.rand(tex.shape, device=dev, generator=torch.Generator(device=dev).manual_seed(5))
        vt = torch.as_tensor(vt, device=dev)
        params = nr.RasterizeParam(vertices_textures=vt[None].expand(B, -1, -1), faces_textures=torch.as_tensor(ft, device=dev),
                                   textures=tex[None].expand(B, -1, -1, -1))
        params1 = nr.RasterizeParam(vertices_textures=vt[None], faces_textures=torch.as_tensor(ft, device=dev),
                                    textures=tex[None])
    pv = proj.to(dev).requires_grad_(True)
    img = nrr.rasterize_core(pv, ft_, params, hp)
    g = torch.randn(img.shape, generator=torch.Generator().manual_seed(13)).to(dev)
    img.backward(g)
    for i in (0, 17, 31):
        p1 = proj[i:i + 1].to(dev).requires_grad_(True)
        img1 = nrr.rasterize_core(p1, ft_, params1, hp)
        assert torch.equal(img1[0], img[i].detach()), "item %d images" % i
        img1.backward(g[i:i + 1])
        close_grads(pv.grad[i:i + 1], p1.grad, "item %d grad vertices" % i)


def test_empty_and_degenerate(dev):
    hp = nr.RasterizeHyperparam(image_size=16)
    v = torch.zeros((0, 3, 3), device=dev)
    f = torch.as_tensor([[0, 1, 2]], device=dev)
    out = nr.rasterize_silhouettes(v, f, nr.RasterizeParam(), hp)
    assert out.shape == (0, 16, 16)
    v = torch.rand((2, 5, 3), device=dev)
    out = nr.rasterize_depth(v, torch.zeros((0, 3), dtype=torch.int32), nr.RasterizeParam(),
                             nr.RasterizeHyperparam(image_size=10, anti_aliasing=False))
    assert out.shape == (2, 10, 10) and float(out.abs().max()) == 0
    with pytest.raises(IndexError):
        nr.rasterize_silhouettes(v, torch.as_tensor([[0, 1, 7]]), nr.RasterizeParam(), hp)


def test_empty_batch_textured(dev):
    """An rgb render of an empty shard (B=0): empty images; the batch-shared texture and the
    shared vertices_textures get zero gradients (nr_rasterize_backward's B == 0 path)."""
    vt, ft, tex = nr.create_textures(4, texture_size=2)
    tex_leaf = torch.as_tensor(tex, device=dev).requires_grad_(True)
    vt_leaf = torch.as_tensor(vt, device=dev).requires_grad_(True)
    v = torch.zeros((0, 4, 3), device=dev, requires_grad=True)
    f = torch.as_tensor([[0, 1, 2], [1, 2, 3], [0, 2, 3], [0, 1, 3]], device=dev)
    params = nr.RasterizeParam(vertices_textures=vt_leaf[None].expand(0, -1, -1),
                               faces_textures=torch.as_tensor(ft, device=dev),
                               textures=tex_leaf[None].expand(0, *tex_leaf.shape))
    hp = nr.RasterizeHyperparam(image_size=16)
    img = nr.rasterize_rgba(v, f, params, hp)
    assert img.shape == (0, 4, 16, 16)
    img.sum().backward()
    assert v.grad is not None and v.grad.shape == (0, 4, 3)
    assert tex_leaf.grad is not None and float(tex_leaf.grad.abs().max()) == 0


def test_expanded_texture_leaf_gets_per_item_grads(golden, dev):
    """textures = tex[None].expand(B, ...).requires_grad_() (the reference tests' idiom with the
    expanded view as the leaf): autograd gives that leaf one gradient per item, as the reference
    fills it.  Their sum is the shared-texture golden gradient, and item b's share is what item b
    rendered alone gives its texture."""
    d = golden("teapot_rgbsd_aa")
    assert int(d["shared_textures"])
    B = d["proj"].shape[0]
    proj = torch.as_tensor(d["proj"], device=dev)
    faces = torch.as_tensor(d["faces"], device=dev)
    ft = torch.as_tensor(d["faces_textures"], device=dev)
    g = torch.as_tensor(d["grad_up"], device=dev)
    tex = torch.as_tensor(d["textures"], device=dev)[None].expand(B, *d["textures"].shape).requires_grad_()
    assert tex.grad_fn is None and tex.stride(0) == 0
    vt = torch.as_tensor(d["vertices_textures"], device=dev)[None]

    def hp():
        return nr.RasterizeHyperparam(image_size=int(d["image_size"]), anti_aliasing=bool(d["anti_aliasing"]),
                                      draw_backside=bool(d["draw_backside"]), **flags_of("teapot_rgbsd_aa"))

    params = nr.RasterizeParam(vertices_textures=vt.expand(B, -1, -1), faces_textures=ft, textures=tex)
    img = nrr.rasterize_core(proj, faces, params, hp())
    close_images(img, d["images"], "expanded-leaf images")
    img.backward(g)
    assert tex.grad is not None and tex.grad.shape == tex.shape
    close_grads(tex.grad.sum(0), d["grad_textures"], "expanded-leaf grad textures (sum over items)")
    for b in range(B):
        t1 = torch.as_tensor(d["textures"], device=dev)[None].requires_grad_()
        one = nrr.rasterize_core(proj[b:b + 1], faces, nr.RasterizeParam(vertices_textures=vt, faces_textures=ft,
                                                                          textures=t1), hp())
        one.backward(g[b:b + 1])
        close_grads(tex.grad[b], t1.grad[0], "expanded-leaf grad textures, item %d" % b)


def test_reference_binding_module(golden, dev):
    """neural_renderer_v2_pytorch_amd.rasterize_cuda, driven the way the reference's own
    rasterize.py:27-38 and :67-77 drive its pybind module (flat -1-filled index buffer, zeroed
    weight buffer, in-place writes, aliased returns), reproduces the golden face-index and weight
    maps bit for bit."""
    from neural_renderer_v2_pytorch_amd import rasterize_cuda as rc
    d = golden("edges")
    for i in range(3):
        faces = torch.as_tensor(d["faces%d" % i], device=dev).contiguous()
        B, F = faces.shape[:2]
        for bs in (0, 1):
            S = d["fim%d_%d" % (i, bs)].shape[1]
            face_index = (torch.zeros((B, S, S), dtype=torch.int32).reshape((-1,)) - 1).to(dev)
            out = rc.face_index_map_forward_safe(faces, face_index, F, S, 0.1, 100.0, bs, 1e-8, 1e-4)
            assert out is face_index
            fim = out.reshape((B, S, S))
            assert np.array_equal(fim.cpu().numpy(), d["fim%d_%d" % (i, bs)])
            wm = torch.zeros((B * S * S, 3), dtype=torch.float32, device=dev)
            ret = rc.compute_weight_map_c(faces, fim.flatten(), wm, F, S)
            assert ret.numel() == B * S * S
            assert np.array_equal(wm.reshape(B, S, S, 3).cpu().numpy(), d["weight%d_%d" % (i, bs)])
            data = torch.randn((B, S, S, 3), device=dev)
            dst = torch.full_like(data, 7.0)
            assert rc.mask_foreground_forward(fim, data, dst, 3) is dst
            fg = (fim >= 0)[..., None]
            assert torch.equal(dst, torch.where(fg, data, torch.full_like(data, 7.0)))
            gin = torch.zeros_like(data)
            assert rc.mask_foreground_backward(fim, gin, data, 3) is gin
            assert torch.equal(gin, torch.where(fg, data, torch.zeros_like(data)))


def test_exact_division_shortcut(dev):
    """div_nr (the compiler's f32 division sequence without v_div_scale / v_div_fixup) equals IEEE
    a / b bit for bit over the operand range the kernels guard: |a|, |b| in [2^-81, 2^62] and
    [2^-20, 2^20] respectively, quotients normal, exponent gap < 96 (random mantissas, every
    exponent pair, and mantissas next to powers of two)."""
    from neural_renderer_v2_pytorch_amd import _lib
    g = torch.Generator(device=dev).manual_seed(5)
    n = 1 << 24
    ea = torch.randint(-81, 62, (n,), device=dev, generator=g).float()
    eb = torch.randint(-20, 20, (n,), device=dev, generator=g).float()
    ma = 1 + torch.rand(n, device=dev, generator=g)
    mb = 1 + torch.rand(n, device=dev, generator=g)
    # mantissas at the ends of the binade (all-ones / just above 1)
    edge = torch.rand(n, device=dev, generator=g) < 0.25
    ulp = torch.randint(0, 8, (n,), device=dev, generator=g).float() * 2.0 ** -23
    mb = torch.where(edge, torch.where(torch.rand(n, device=dev, generator=g) < 0.5, 2 - 2.0 ** -23 - ulp, 1 + ulp), mb)
    sa = torch.where(torch.rand(n, device=dev, generator=g) < 0.5, -1.0, 1.0)
    sb = torch.where(torch.rand(n, device=dev, generator=g) < 0.5, -1.0, 1.0)
    a = (sa * ma * torch.exp2(ea)).float().contiguous()
    b = (sb * mb * torch.exp2(eb)).float().contiguous()
    qf, qi = torch.empty_like(a), torch.empty_like(a)
    _lib.check(_lib.lib().nr_selftest_division(_lib.ptr(a), _lib.ptr(b), _lib.ptr(qf), _lib.ptr(qi), n,
                                               _lib.stream_of(a)), "nr_selftest_division")
    assert torch.equal(qi, a / b)  # the IEEE leg is torch's division too
    bad = (qf.view(torch.int32) != qi.view(torch.int32))
    assert not bad.any(), (int(bad.sum()), a[bad][:4].tolist(), b[bad][:4].tolist())


@pytest.mark.parametrize("aa,size,extras", [(True, 64, False), (False, 70, False), (True, 48, True)])
def test_halo_cache_matches_reshading(dev, aa, size, extras):
    """The backward's tile halos read from the forward's halo cache give the same gradients as
    re-shading them (NrRasterArgs.halo NULL); includes a size that is not a multiple of the tiles.
    The cache starts out as NaN: the forward writes no halo values for a bin without candidate faces,
    and the backward must read those as 0 (from the bin flags) and never an unwritten value."""
    B = 3
    proj, f = _ico_batch(3, B, dev)
    vt, ft, tex = nr.create_textures(f.shape[0], texture_size=4)
    tex = torch.rand(tex.shape, generator=torch.Generator().manual_seed(4)).to(dev)
    g = torch.randn((B, 5, size, size), generator=torch.Generator().manual_seed(6)).to(dev)
    grads = []
    for use in (True, False):
        nrr._HALO_CACHE = use
        nrr._HALO_FILL = float("nan")
        try:
            pv = proj.to(dev).requires_grad_(True)
            tx = tex.clone().requires_grad_(True)
            S = size * (2 if aa else 1)
            extra = {}
            if extras:  # lights and backgrounds change the halo's image values too
                extra = dict(backgrounds=torch.rand((B, 3, S, S), generator=torch.Generator().manual_seed(2)).to(dev),
                             lights=[nr.AmbientLight(torch.full((B, 3), 0.4, device=dev)),
                                     nr.SpecularLight(torch.full((B, 3), 0.5, device=dev))])
            params = nr.RasterizeParam(vertices_textures=torch.as_tensor(vt, device=dev)[None].expand(B, -1, -1),
                                       faces_textures=torch.as_tensor(ft, device=dev),
                                       textures=tx[None].expand(B, -1, -1, -1), **extra)
            img = nrr.rasterize_core(pv, torch.as_tensor(f, device=dev), params,
                                     nr.RasterizeHyperparam(image_size=size, anti_aliasing=aa))
            img.backward(g)
            grads.append((img.detach(), pv.grad, tx.grad))
        finally:
            nrr._HALO_CACHE = True
            nrr._HALO_FILL = None
    assert torch.equal(grads[0][0], grads[1][0])
    assert torch.isfinite(grads[0][1]).all() and torch.isfinite(grads[0][2]).all()
    close_grads(grads[0][1], grads[1][1], "grad vertices")
    close_grads(grads[0][2], grads[1][2], "grad textures")


def _fixture_lights(d, dev):
    """Our light classes from a golden fixture's light arrays (kind 0 ambient, 1 directional, 2 specular)."""
    out = []
    for i, k in enumerate(d["light_kind"]):
        col = torch.as_tensor(d["light_color"][i], device=dev)
        if k == 0:
            out.append(nr.AmbientLight(col))
        elif k == 1:
            out.append(nr.DirectionalLight(col, torch.as_tensor(d["light_direction"][i], device=dev),
                                           backside=bool(d["light_backside"][i])))
        else:
            out.append(nr.SpecularLight(col, alpha=torch.as_tensor(d["light_alpha"][i], device=dev),
                                        backside=bool(d["light_backside"][i])))
    return out


@pytest.mark.parametrize("name", ["teapot_lights", "ico_lights"])
def test_lights_golden(golden, dev, name):
    """Lit textured renders (rasterize.py:162-190 normal map, 252-283 light loop) against the
    reference's own images and gradients: the teapot scene of tests_torch/test_rasterize.py
    test_forward_case4 (three lights, no backside) and every light kind / option on an ico-sphere."""
    d = golden(name)
    B = d["proj"].shape[0]
    pv = torch.as_tensor(d["proj"], device=dev).requires_grad_(True)
    tex = torch.as_tensor(d["textures"], device=dev).requires_grad_(True)
    chans = d["images"].shape[1]
    params = nr.RasterizeParam(vertices_textures=torch.as_tensor(d["vertices_textures"], device=dev)[None].expand(B, -1, -1),
                               faces_textures=torch.as_tensor(d["faces_textures"], device=dev),
                               textures=tex[None].expand(B, -1, -1, -1), lights=_fixture_lights(d, dev))
    hp = nr.RasterizeHyperparam(image_size=int(d["image_size"]), anti_aliasing=bool(d["anti_aliasing"]),
                                draw_backside=bool(d["draw_backside"]), draw_silhouettes=chans == 5, draw_depth=chans == 5)
    img = nrr.rasterize_core(pv, torch.as_tensor(d["faces"], device=dev), params, hp)
    close_images(img, d["images"], name + " images")
    img.backward(torch.as_tensor(d["grad_up"], device=dev))
    close_grads(pv.grad, d["grad_proj"], name + " grad vertices")
    close_grads(tex.grad, d["grad_textures"], name + " grad textures")


@pytest.mark.parametrize("name", ["param_grads_items", "param_grads_shared"])
def test_param_grads_golden(golden, dev, name):
    """Gradients w.r.t. vertices_textures (per item, and shared by the batch through an expanded
    [1, Vt, 2] leaf) and w.r.t. every light parameter (colours, directions, the given specular
    exponent) against the reference's own autograd (rasterize.py:100-153, 246, 252-283), through
    nr_rasterize_backward_params."""
    d = golden(name)
    B = d["proj"].shape[0]
    pv = torch.as_tensor(d["proj"], device=dev).requires_grad_(True)
    tex = torch.as_tensor(d["textures"], device=dev).requires_grad_(True)
    vt = torch.as_tensor(d["vertices_textures"], device=dev).requires_grad_(True)
    lights = None
    if "light_kind" in d:
        lights = _fixture_lights(d, dev)
        for L, req in zip(lights, d["light_alpha_requires_grad"]):
            L.color.requires_grad_(True)
            if isinstance(L, nr.DirectionalLight):
                L.direction.requires_grad_(True)
            if isinstance(L, nr.SpecularLight):
                L.alpha.requires_grad_(bool(req))
    params = nr.RasterizeParam(vertices_textures=vt if vt.shape[0] == B else vt.expand(B, -1, -1),
                               faces_textures=torch.as_tensor(d["faces_textures"], device=dev),
                               textures=tex[None].expand(B, -1, -1, -1), lights=lights)
    hp = nr.RasterizeHyperparam(image_size=int(d["image_size"]), anti_aliasing=bool(d["anti_aliasing"]),
                                draw_backside=bool(d["draw_backside"]))
    img = nrr.rasterize_core(pv, torch.as_tensor(d["faces"], device=dev), params, hp)
    close_images(img, d["images"], name + " images")
    img.backward(torch.as_tensor(d["grad_up"], device=dev))
    close_grads(pv.grad, d["grad_proj"], name + " grad vertices")
    close_grads(tex.grad, d["grad_textures"], name + " grad textures")
    close_grads(vt.grad, d["grad_vertices_textures"], name + " grad vertices_textures")
    if lights is not None:
        close_grads(torch.stack([L.color.grad for L in lights]), d["grad_light_color"], name + " grad light colours")
        for i, L in enumerate(lights):
            if isinstance(L, nr.DirectionalLight):
                close_grads(L.direction.grad, d["grad_light_direction"][i], name + " grad light direction %d" % i)
        close_grads(torch.stack([L.alpha.grad for L in lights if isinstance(L, nr.SpecularLight) and L.alpha.requires_grad]),
                    d["grad_light_alpha"], name + " grad specular alpha")


@pytest.mark.parametrize("aa,size,lit", [(True, 40, False), (False, 50, True)])
def test_backgrounds_vs_oracle(oracle_mod, dev, aa, size, lit):
    """backgrounds blended with the chainer semantics (rasterize.py:574-577; the torch
    blend_backgrounds raises, so this is pinned by the oracle restatement only): images and the
    gradients of vertices, textures and the backgrounds themselves, with and without lights."""
    B = 2
    proj, f = _ico_batch(2, B, dev)
    vt, ft, tex = nr.create_textures(f.shape[0], texture_size=4)
    tex = torch.rand(tex.shape, generator=torch.Generator().manual_seed(8))
    S = size * (2 if aa else 1)
    bgs = torch.rand((B, 3, S, S), generator=torch.Generator().manual_seed(9))
    lights_cpu = [nr.AmbientLight(torch.full((B, 3), 0.3)),
                  nr.DirectionalLight(torch.full((B, 3), 0.6), torch.tensor([[0.3, -0.5, 0.81]] * B))] if lit else None
    g = torch.randn((B, 5, size, size), generator=torch.Generator().manual_seed(10))
    out = {}
    for where in ("gpu", "cpu"):
        d = dev if where == "gpu" else torch.device("cpu")
        pv = proj.to(d).clone().requires_grad_(True)
        tx = tex.to(d).clone().requires_grad_(True)
        bg = bgs.to(d).clone().requires_grad_(True)
        vts = torch.as_tensor(vt, device=d)[None].expand(B, -1, -1)
        lights = None
        if lit:
            lights = [nr.AmbientLight(lights_cpu[0].color.to(d)),
                      nr.DirectionalLight(lights_cpu[1].color.to(d), lights_cpu[1].direction.to(d))]
        if where == "gpu":
            params = nr.RasterizeParam(vertices_textures=vts, faces_textures=torch.as_tensor(ft, device=d),
                                       textures=tx[None].expand(B, -1, -1, -1), backgrounds=bg, lights=lights)
            img = nrr.rasterize_core(pv, torch.as_tensor(f, device=d), params,
                                     nr.RasterizeHyperparam(image_size=size, anti_aliasing=aa))
        else:
            img = oracle_mod.rasterize_core(pv, f, image_size=size, anti_aliasing=aa, vertices_textures=vts,
                                            faces_textures=ft, textures=tx[None].expand(B, -1, -1, -1),
                                            lights=lights, backgrounds=bg)
        img.backward(g.to(d))
        out[where] = (img.detach().cpu(), pv.grad.cpu(), tx.grad.cpu(), bg.grad.cpu())
    close_images(out["gpu"][0], out["cpu"][0], "images")
    for i, what in ((1, "vertices"), (2, "textures"), (3, "backgrounds")):
        close_grads(out["gpu"][i], out["cpu"][i], "grad " + what)


@pytest.mark.parametrize("per_item,ts", [(False, 2), (True, 8)])
def test_texture_repack_and_transpose_paths_vs_oracle(oracle_mod, dev, per_item, ts):
    """The texture repack and the texture-gradient transpose run inside k_face_setup /
    k_vertex_grad when they are small (a shared 36x36 atlas here) and as launches of their own when
    they are not (per-item 144x144 atlases, whose 8x8 texel tiles also exceed the backward's 4x4
    face window): images, vertex and texture gradients against the CPU oracle either way."""
    B = 2
    proj, f = _ico_batch(2, B, dev)
    vt, ft, tex = nr.create_textures(f.shape[0], texture_size=ts)
    shape = ((B,) if per_item else (1,)) + tex.shape
    tex = torch.rand(shape, generator=torch.Generator().manual_seed(21))
    g = torch.randn((B, 5, 48, 48), generator=torch.Generator().manual_seed(22))
    out = {}
    for where in ("gpu", "cpu"):
        d = dev if where == "gpu" else torch.device("cpu")
        pv = proj.to(d).clone().requires_grad_(True)
        tx = tex.to(d).clone().requires_grad_(True)
        texb = tx if per_item else tx.expand(B, -1, -1, -1)
        vts = torch.as_tensor(vt, device=d)[None].expand(B, -1, -1)
        if where == "gpu":
            params = nr.RasterizeParam(vertices_textures=vts, faces_textures=torch.as_tensor(ft, device=d), textures=texb)
            img = nrr.rasterize_core(pv, torch.as_tensor(f, device=d), params, nr.RasterizeHyperparam(image_size=48))
        else:
            img = oracle_mod.rasterize_core(pv, f, image_size=48, vertices_textures=vts, faces_textures=ft, textures=texb)
        img.backward(g.to(d))
        out[where] = (img.detach().cpu(), pv.grad.cpu(), tx.grad.cpu())
    close_images(out["gpu"][0], out["cpu"][0], "images")
    close_grads(out["gpu"][1], out["cpu"][1], "grad vertices")
    close_grads(out["gpu"][2], out["cpu"][2], "grad textures")


def test_partial_upstream_gradient_vs_oracle(oracle_mod, dev):
    """A loss on some channels and regions only (zero upstream gradient elsewhere): the backward
    leaves zero-contribution pixels out of its per-face gather; gradients against the oracle."""
    B = 2
    proj, f = _ico_batch(2, B, dev)
    vt, ft, tex = nr.create_textures(f.shape[0], texture_size=4)
    tex = torch.rand(tex.shape, generator=torch.Generator().manual_seed(31))
    g = torch.randn((B, 5, 40, 40), generator=torch.Generator().manual_seed(32))
    g[:, 0:3] = 0.0          # no loss on rgb
    g[:, :, :, 20:] = 0.0    # nor on the right half
    out = {}
    for where in ("gpu", "cpu"):
        d = dev if where == "gpu" else torch.device("cpu")
        pv = proj.to(d).clone().requires_grad_(True)
        tx = tex.to(d).clone().requires_grad_(True)
        vts = torch.as_tensor(vt, device=d)[None].expand(B, -1, -1)
        if where == "gpu":
            params = nr.RasterizeParam(vertices_textures=vts, faces_textures=torch.as_tensor(ft, device=d),
                                       textures=tx[None].expand(B, -1, -1, -1))
            img = nrr.rasterize_core(pv, torch.as_tensor(f, device=d), params, nr.RasterizeHyperparam(image_size=40))
        else:
            img = oracle_mod.rasterize_core(pv, f, image_size=40, vertices_textures=vts, faces_textures=ft,
                                            textures=tx[None].expand(B, -1, -1, -1))
        img.backward(g.to(d))
        out[where] = (pv.grad.cpu(), tx.grad.cpu())
    close_grads(out["gpu"][0], out["cpu"][0], "grad vertices")
    close_grads(out["gpu"][1], out["cpu"][1], "grad textures")


def test_background_color_is_black(dev):
    """background_color: the reference computes zeros * colour (rasterize.py:208-214), a black
    background; the parameter object gets the backgrounds tensor, as the reference sets it."""
    B = 1
    proj, f = _ico_batch(2, B, dev)
    vt, ft, tex = nr.create_textures(f.shape[0], texture_size=4)
    params = nr.RasterizeParam(vertices_textures=torch.as_tensor(vt, device=dev)[None],
                               faces_textures=torch.as_tensor(ft, device=dev),
                               textures=torch.rand((1,) + tex.shape, device=dev), background_color=[0.2, 0.5, 0.9])
    img = nr.rasterize_rgb(proj.to(dev), torch.as_tensor(f, device=dev), params, nr.RasterizeHyperparam(image_size=32))
    plain = nr.rasterize_rgb(proj.to(dev), torch.as_tensor(f, device=dev),
                             nr.RasterizeParam(vertices_textures=params.vertices_textures,
                                               faces_textures=params.faces_textures, textures=params.textures),
                             nr.RasterizeHyperparam(image_size=32))
    assert params.backgrounds is not None and float(params.backgrounds.abs().max()) == 0
    assert torch.equal(img, plain)


@pytest.mark.gpu
def test_example2_silhouette_fit(dev):
    """the reference's example2 workload (examples_pytorch/example2.py:17-78) run
    by examples/example2.py on the HIP path: Adam on the teapot's vertices against the example's
    reference silhouette.  The squared-error loss (10103 at step 0) must fall below 1 % of its
    start within the example's 300 steps (measured: 0.1 on an MI355X)."""
    import importlib.util
    path = os.path.join(os.path.dirname(__file__), '..', 'examples', 'example2.py')
    spec = importlib.util.spec_from_file_location('nr_example2', path)
    ex = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ex)
    model = ex.SilhouetteFit(os.path.join(ex.DATA, 'teapot.obj'), os.path.join(ex.DATA, 'example2_ref.png'), dev)
    losses = ex.optimize(model, 300)
    assert all(np.isfinite(losses))
    assert losses[0] > 5000
    assert losses[-1] < 0.01 * losses[0]


def test_example2_graphed_fit(dev):
    """The same fit with the whole step (camera, rasterize, loss, backward, Adam) captured once in a
    HIP graph and replayed (examples/example2.py optimize_graphed): it must converge as the eager
    loop does, from the same initial loss."""
    import importlib.util
    path = os.path.join(os.path.dirname(__file__), '..', 'examples', 'example2.py')
    spec = importlib.util.spec_from_file_location('nr_example2g', path)
    ex = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ex)
    model = ex.SilhouetteFit(os.path.join(ex.DATA, 'teapot.obj'), os.path.join(ex.DATA, 'example2_ref.png'), dev)
    losses = ex.optimize_graphed(model, 300)
    assert all(np.isfinite(losses))
    assert 5000 < losses[0] < 20000
    assert losses[-1] < 0.01 * losses[0]


@pytest.mark.parametrize("B,shared_v,eye_kind,persp", [(2, False, "items", True), (3, False, "items", True),
                                                        (4, True, "items", True), (2, False, "one", False),
                                                        (3, True, "one", True)])
def test_camera_transform_vs_torch(dev, B, shared_v, eye_kind, persp):
    """Fused look_at + perspective (nr_camera_forward / backward) against the reference's composition
    of torch ops (look_at.py:5-44 with per-item cross products, perspective.py:4-18) in float64 on
    the CPU: projected vertices and the gradients of vertices and viewpoints."""
    from neural_renderer_v2_pytorch_amd import camera
    r = np.random.RandomState(11 + B)
    V = 300
    v_np = r.normal(size=(1 if shared_v else B, V, 3)).astype(np.float32) * 0.5
    eyes_np = np.stack([nr.get_points_from_angles(2.732, r.uniform(-30, 30), r.uniform(0, 360))
                        for _ in range(B if eye_kind == "items" else 1)]).astype(np.float32)
    g_np = r.normal(size=(B, V, 3)).astype(np.float32)

    def run(v_leaf, e_leaf, fused):
        vv = v_leaf.expand(B, -1, -1) if shared_v else v_leaf
        ee = e_leaf if eye_kind == "items" else e_leaf[0]
        if fused:
            out = camera.camera_transform(vv, ee, perspective=persp, angle=30)
        else:
            out = nr.look_at(vv, ee, at=torch.zeros(3, dtype=vv.dtype),
                             up=torch.tensor([0., 1., 0.], dtype=vv.dtype))
            if persp:
                out = nr.perspective(out, angle=30.)
        out.backward(torch.as_tensor(g_np, dtype=out.dtype, device=out.device))
        return out

    v_g = torch.as_tensor(v_np, device=dev).requires_grad_(True)
    e_g = torch.as_tensor(eyes_np, device=dev).requires_grad_(True)
    out = run(v_g, e_g, True)
    v_c = torch.as_tensor(v_np, dtype=torch.float64).requires_grad_(True)
    e_c = torch.as_tensor(eyes_np, dtype=torch.float64).requires_grad_(True)
    ref = run(v_c, e_c, False)
    np.testing.assert_allclose(out.detach().cpu().numpy(), ref.detach().numpy(), rtol=1e-5, atol=1e-5)
    close_grads(v_g.grad, v_c.grad.float(), "camera grad vertices")
    close_grads(e_g.grad, e_c.grad.float(), "camera grad viewpoints")
    assert v_g.grad.shape == v_g.shape and e_g.grad.shape == e_g.shape


def test_renderer_camera_fit(dev):
    """example4 (examples_pytorch/example4.py:17-110): fit the camera position to a silhouette of the
    teapot through Renderer.render_silhouettes; gradients reach the viewpoints through the fused
    camera prologue.  The loss must drop well below its start within 150 Adam steps."""
    v, f = nr.load_obj(os.path.join(os.path.dirname(__file__), "data", "teapot.obj"))
    vertices = torch.as_tensor(v[None], device=dev)
    faces = torch.as_tensor(f, device=dev)
    ren = nr.Renderer()
    ren.image_size = 128
    ren.viewpoints = nr.get_points_from_angles(2.732, 30, -15)
    with torch.no_grad():
        target = ren.render_silhouettes(vertices, faces)
    cam = torch.nn.Parameter(torch.tensor([4., 6., -9.], device=dev))
    ren.viewpoints = cam
    opt = torch.optim.Adam([cam], lr=0.1)
    losses = []
    for _ in range(150):
        opt.zero_grad()
        loss = ((ren.render_silhouettes(vertices, faces) - target) ** 2).sum()
        loss.backward()
        assert cam.grad is not None and torch.isfinite(cam.grad).all()
        opt.step()
        losses.append(float(loss.detach()))
    assert losses[-1] < 0.3 * losses[0], (losses[0], losses[-1])


@pytest.mark.parametrize("B,s,level", [(3, 64, 3), (8, 64, 4)])
def test_hip_graph_capture_matches_eager(dev, B, s, level):
    """The fused forward + backward issues no host synchronisation (faces checks and adjacency are
    cached per tensor), so a whole step can be captured once in a HIP graph (torch.cuda.CUDAGraph)
    and replayed: the replayed images equal the eager ones bit for bit and the gradients agree
    within the gradient tolerance (float atomics).  The second case is a split forward (deep bins at
    1024 threads on the caller's stream, the rest at 256 on the library's side stream): the capture
    records its fork and join."""
    proj, f = _ico_batch(level, B, dev)
    faces = torch.as_tensor(f, device=dev)
    vt, ft, tex = nr.create_textures(f.shape[0], texture_size=4)
    tex = torch.as_tensor(np.random.RandomState(3).uniform(0, 1, tex.shape).astype(np.float32), device=dev)
    g = torch.as_tensor(np.random.RandomState(4).normal(size=(B, 5, s, s)).astype(np.float32), device=dev)
    pv = proj.detach().to(dev).requires_grad_(True)
    tx = tex.clone().requires_grad_(True)
    vt_d, ft_d = torch.as_tensor(vt, device=dev), torch.as_tensor(ft, device=dev)
    hp = nr.RasterizeHyperparam(image_size=s)

    def step():
        # the expand of the leaf texture is built per step, so no autograd node from outside the
        # capture stream stays alive (torch's graph-capture rule for leaves)
        params = nr.RasterizeParam(vertices_textures=vt_d[None].expand(B, -1, -1), faces_textures=ft_d,
                                   textures=tx[None].expand(B, -1, -1, -1))
        img = nrr.rasterize_core(pv, faces, params, hp)
        img.backward(g)
        return img

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(2):
            pv.grad = tx.grad = None
            eager = step().detach().clone()
    torch.cuda.current_stream().wait_stream(side)
    eager_gv, eager_gt = pv.grad.clone(), tx.grad.clone()
    pv.grad = tx.grad = None
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        img = step()
    if B % 8 == 0:
        assert _lib.last_launch("k_raster_fwd")[1] & _lib.NR_LAUNCH_SPLIT
    for _ in range(3):
        graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(img, eager)
    close_grads(pv.grad, eager_gv, "graph grad vertices")
    close_grads(tx.grad, eager_gt, "graph grad textures")


@pytest.mark.gpu
def test_backward_workspace_zeroed_by_forward(dev):
    """The forward's setup zeroes the backward's accumulators (NrRasterArgs.bwd_workspace): the
    gradients match a backward that zero-fills its own workspace, and a second backward through the
    same graph (retain_graph; the workspace is no longer zero) still adds the same gradients."""
    B = 3
    proj, f = _ico_batch(3, B, dev)
    faces = torch.as_tensor(f, device=dev)
    vt, ft, tex = nr.create_textures(f.shape[0], texture_size=4)
    tex = torch.as_tensor(np.random.RandomState(5).uniform(0, 1, tex.shape).astype(np.float32), device=dev)
    g = torch.as_tensor(np.random.RandomState(6).normal(size=(B, 5, 64, 64)).astype(np.float32), device=dev)
    out = {}
    for prezero in (False, True):
        nrr._BWD_PREZERO = prezero
        try:
            v = proj.detach().to(dev).requires_grad_(True)
            t = tex.detach().clone().requires_grad_(True)
            params = nr.RasterizeParam(vertices_textures=torch.as_tensor(vt, device=dev)[None].expand(B, -1, -1),
                                       faces_textures=torch.as_tensor(ft, device=dev), textures=t[None].expand(B, -1, -1, -1))
            img = nrr.rasterize_core(v, faces, params, nr.RasterizeHyperparam(image_size=64))
            img.backward(g, retain_graph=True)
            g1 = (v.grad.clone(), t.grad.clone())
            img.backward(g)
            out[prezero] = (g1, (v.grad.clone(), t.grad.clone()))
        finally:
            nrr._BWD_PREZERO = True
    for i in range(2):
        torch.testing.assert_close(out[True][0][i], out[False][0][i], rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(out[True][1][i], 2 * out[True][0][i], rtol=1e-5, atol=1e-6)


def test_two_meshes_alternating_in_one_hip_graph(dev):
    """Faces checks and adjacencies are cached per faces tensor in a small LRU (rasterize.py
    _TensorCache): a caller alternating two meshes pays the host-side checks once per mesh, never
    per call.  Proof that no call syncs with the host: after one eager step per mesh, a step that
    renders and differentiates mesh A, then mesh B, then A again is captured in ONE HIP graph
    (a device-to-host copy or a .cpu() inside the capture would raise) and replayed; the replayed
    images equal the eager ones bit for bit and the gradients agree within the tolerance."""
    s = 64
    meshes = []
    for level, B in ((3, 2), (2, 3)):
        proj, f = _ico_batch(level, B, dev)
        meshes.append((proj.detach().to(dev).requires_grad_(True), torch.as_tensor(f, device=dev)))
    g = [torch.randn((p.shape[0], 5, s, s), generator=torch.Generator().manual_seed(70 + i)).to(dev)
         for i, (p, _) in enumerate(meshes)]
    tex = torch.rand((3, 16, 16), generator=torch.Generator().manual_seed(72)).to(dev)

    def render(i):
        pv, faces = meshes[i]
        hp = nr.RasterizeHyperparam(image_size=s)
        hp.draw_rgb = False
        img = nrr.rasterize_core(pv, faces, nr.RasterizeParam(), hp)
        img.backward(g[i][:, :img.shape[1]])
        return img

    def step():
        return [render(0), render(1), render(0)]

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(2):
            for pv, _ in meshes:
                pv.grad = None
            eager = [x.detach().clone() for x in step()]
    torch.cuda.current_stream().wait_stream(side)
    eager_g = [pv.grad.clone() for pv, _ in meshes]
    for pv, _ in meshes:
        pv.grad = None
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        out = step()
    graph.replay()
    torch.cuda.synchronize()
    for a, b in zip(out, eager):
        assert torch.equal(a, b)
    for (pv, _), ge in zip(meshes, eager_g):
        close_grads(pv.grad, ge, "graph grad vertices")
    assert len(nrr._faces_checked.entries) >= 2 and len(nrr._adjacency.entries) >= 2


def test_car_renderer_render_batch(oracle_mod, dev):
    """The car (tests_torch/test_rasterize.py:43-81's scene) through Renderer.render at B = 4 views:
    the output equals rasterize_rgba of the Renderer's own camera transform bit for bit, and that
    render matches the oracle on the same projected vertices (face-index map bit-exact, images,
    vertex and texture gradients).  The fused camera itself is checked against the reference's
    torch composition in float64 by test_camera_transform_vs_torch."""
    from neural_renderer_v2_pytorch_amd import camera
    v, f, vt, ft, tex = nr.load_obj(os.path.join(os.path.dirname(__file__), "data", "4e49873292196f02574b5684eaec43e9",
                                                 "model.obj"), load_textures=True)
    B = 4
    eyes = torch.as_tensor(np.stack([nr.get_points_from_angles(2.5, 10 * i, -90 + 40 * i) for i in range(B)]),
                           dtype=torch.float32, device=dev)
    ren = nr.Renderer()
    ren.draw_backside = False
    ren.viewpoints = eyes
    mesh = torch.as_tensor(v[None], device=dev).requires_grad_(True)
    atlas = torch.as_tensor(tex, device=dev).requires_grad_(True)
    vt_d, ft_d, f_d = torch.as_tensor(vt, device=dev)[None].expand(B, -1, -1), torch.as_tensor(ft, device=dev), \
        torch.as_tensor(f, device=dev)
    img = ren.render(mesh.expand(B, -1, -1), f_d, vt_d, ft_d, atlas[None].expand(B, -1, -1, -1))
    assert img.shape == (B, 4, 256, 256)
    with torch.no_grad():
        proj = camera.camera_transform(mesh.expand(B, -1, -1), eyes, perspective=True, angle=30)
    hp = nr.RasterizeHyperparam(image_size=256, draw_backside=False)
    params = nr.RasterizeParam(vertices_textures=vt_d, faces_textures=ft_d, textures=atlas.detach()[None].expand(B, -1, -1, -1))
    assert torch.equal(nr.rasterize_rgba(proj, f_d, params, hp), img.detach())
    pv = proj.clone().requires_grad_(True)
    tx = atlas.detach().clone().requires_grad_(True)
    params = nr.RasterizeParam(vertices_textures=vt_d, faces_textures=ft_d, textures=tx[None].expand(B, -1, -1, -1))
    img2, fim = nrr.rasterize_core(pv, f_d, params, nr.RasterizeHyperparam(image_size=256, draw_backside=False,
                                                                          draw_depth=False), return_face_index=True)
    g = torch.randn(img2.shape, generator=torch.Generator().manual_seed(74))
    img2.backward(g.to(dev))
    pc = proj.cpu().clone().requires_grad_(True)
    tc = torch.as_tensor(tex).clone().requires_grad_(True)
    ref, internals = oracle_mod.rasterize_core(pc, f, image_size=256, draw_backside=False, draw_depth=False,
                                               vertices_textures=torch.as_tensor(vt)[None].expand(B, -1, -1),
                                               faces_textures=ft, textures=tc[None].expand(B, -1, -1, -1),
                                               return_internals=True)
    ref.backward(g)
    assert np.array_equal(fim.cpu().numpy(), internals["fim"].numpy())
    close_images(img2, ref, "car Renderer.render images")
    close_grads(pv.grad, pc.grad, "car grad projected vertices")
    close_grads(tx.grad, tc.grad, "car grad textures")


def test_pixel_centre_division(dev):
    """The kernels' pixel centre (nr_common.h pix_center: rcp_nr + div_nr of (2 i + 1 - S) by S) equals
    the IEEE f32 division bit for bit for every i in -2 .. S + 1 of every raster size S <= 16384; the
    host check (test_host.py::test_pixel_centre_is_exact_on_host) proves that division equal to the
    reference's double formula (rasterize_cuda_kernel.cu:76-77).  Through nr_selftest_division, whose
    fast leg is the same div_nr(a, b, rcp_nr(b))."""
    from neural_renderer_v2_pytorch_amd import _lib
    sizes = torch.arange(1, 16385, device=dev)
    lens = sizes + 4
    starts = torch.cumsum(lens, 0) - lens
    total = int(lens.sum())
    done = 0
    chunk = 1 << 25
    S_all = torch.repeat_interleave(sizes, lens)
    i_all = torch.arange(total, device=dev) - torch.repeat_interleave(starts, lens) - 2
    while done < total:
        n = min(chunk, total - done)
        S = S_all[done:done + n]
        a = (2 * i_all[done:done + n] + 1 - S).float().contiguous()
        b = S.float().contiguous()
        qf, qi = torch.empty_like(a), torch.empty_like(a)
        _lib.check(_lib.lib().nr_selftest_division(_lib.ptr(a), _lib.ptr(b), _lib.ptr(qf), _lib.ptr(qi), n,
                                                   _lib.stream_of(a)), "nr_selftest_division")
        assert torch.equal(qi, a / b)
        bad = qf.view(torch.int32) != qi.view(torch.int32)
        assert not bad.any(), (int(bad.sum()), a[bad][:4].tolist(), b[bad][:4].tolist())
        done += n
    assert done > 134000000


def test_shared_texture_windows_vs_oracle(oracle_mod, dev):
    """Texture windows shared by many faces (NrRasterArgs.face_hot): three groups of faces with
    identical texture-coordinate triples, each a flat-colour-material patch of load_obj.py:84-94
    ([0, p], [0, p + 1], [1, p + 1] in texel units), on a texture shared by the batch.  The backward
    sums those windows in private copies and adds them into the texture gradient after its main
    kernel (asserted from its launch record).  The atlas gradient matches the oracle's sum over the
    batch, equals the direct path's (face_hot off) within the tolerance, and a second backward
    through the same graph (its accumulators, the private copies among them, zeroed by the backward
    itself this time) adds the same gradient again."""
    B, s = 4, 64
    proj, f = _ico_batch(3, B, dev)
    faces = torch.as_tensor(f, device=dev)
    vt = np.array([[[0, p], [0, p + 1], [1, p + 1]] for p in (0, 2, 4)], np.float32).reshape(-1, 2)
    ft = np.stack([np.arange(3) + 3 * (i % 3) for i in range(f.shape[0])]).astype(np.int32)
    tex = np.random.RandomState(81).uniform(0, 1, (3, 8, 8)).astype(np.float32)
    g = torch.as_tensor(np.random.RandomState(82).normal(size=(B, 5, s, s)).astype(np.float32), device=dev)

    def run(min_faces):
        old = nrr._HOT_MIN_FACES
        nrr._HOT_MIN_FACES = min_faces
        try:
            v = proj.detach().to(dev).requires_grad_(True)
            t = torch.as_tensor(tex, device=dev).requires_grad_(True)
            params = nr.RasterizeParam(vertices_textures=torch.as_tensor(vt, device=dev)[None].expand(B, -1, -1),
                                       faces_textures=torch.as_tensor(ft, device=dev),
                                       textures=t[None].expand(B, -1, -1, -1))
            img = nrr.rasterize_core(v, faces, params, nr.RasterizeHyperparam(image_size=s))
            img.backward(g, retain_graph=True)
            launch = _lib.last_launch("k_raster_bwd")
            first = (v.grad.clone(), t.grad.clone())
            img.backward(g)
            return launch, first, (v.grad.clone(), t.grad.clone())
        finally:
            nrr._HOT_MIN_FACES = old
    launch, (gv, gt), (gv2, gt2) = run(32)
    assert launch[1] & _lib.NR_LAUNCH_HOT_WINDOWS
    launch0, (gv0, gt0), _ = run(0)
    assert not launch0[1] & _lib.NR_LAUNCH_HOT_WINDOWS
    assert float(gt.abs().sum()) > 0
    close_grads(gt, gt0, "shared windows vs direct: grad textures")
    close_grads(gv, gv0, "shared windows vs direct: grad vertices")
    close_grads(gt2, 2 * gt, "second backward: grad textures")
    _, _, rgv, rgt = oracle_batch(oracle_mod, proj, f, g, s, torch.as_tensor(tex), vt, ft)
    close_grads(gt, rgt, "shared windows: grad textures vs oracle")
    close_grads(gv, rgv, "shared windows: grad vertices vs oracle")


@pytest.mark.gpu
def test_shared_texture_windows_off_for_trainable_vt(oracle_mod, dev):
    """The shared-window grouping (face_hot) is computed on the host from the texture-coordinate
    table's values, so it is used only for a fixed table: with vertices_textures requiring a gradient
    (an optimiser moves it in place between steps, which a grouping cached per (storage, version), or
    captured in a graph, would not see) the backward takes the plain window flush.  Two steps with the
    table edited in place between them (under no_grad, as an optimiser step does): no hot-window
    launch either time, and the second step's texture gradient matches the oracle at the edited table
    (three of the formerly identical triples now diverge)."""
    B, s = 4, 64
    proj, f = _ico_batch(3, B, dev)
    faces = torch.as_tensor(f, device=dev)
    vt0 = np.array([[[0, p], [0, p + 1], [1, p + 1]] for p in (0, 2, 4)], np.float32).reshape(-1, 2)
    ft = np.stack([np.arange(3) + 3 * (i % 3) for i in range(f.shape[0])]).astype(np.int32)
    tex = np.random.RandomState(81).uniform(0, 1, (3, 8, 8)).astype(np.float32)
    g = torch.as_tensor(np.random.RandomState(82).normal(size=(B, 5, s, s)).astype(np.float32), device=dev)
    vtp = torch.as_tensor(vt0, device=dev).requires_grad_(True)
    for step in range(2):
        v = proj.detach().to(dev).requires_grad_(True)
        t = torch.as_tensor(tex, device=dev).requires_grad_(True)
        params = nr.RasterizeParam(vertices_textures=vtp[None].expand(B, -1, -1),
                                   faces_textures=torch.as_tensor(ft, device=dev),
                                   textures=t[None].expand(B, -1, -1, -1))
        img = nrr.rasterize_core(v, faces, params, nr.RasterizeHyperparam(image_size=s))
        img.backward(g)
        assert not _lib.last_launch("k_raster_bwd")[1] & _lib.NR_LAUNCH_HOT_WINDOWS
        if step == 0:
            with torch.no_grad():
                vtp[3:6] += torch.tensor([[0.5, 0.25], [0.75, 0.5], [1.25, 0.5]], device=dev)
            vtp.grad = None
    vt1 = vtp.detach().cpu().numpy()
    assert not np.array_equal(vt1, vt0)
    _, _, rgv, rgt = oracle_batch(oracle_mod, proj, f, g, s, torch.as_tensor(tex), vt1, ft)
    close_grads(t.grad, rgt, "trainable vt, edited table: grad textures vs oracle")
    close_grads(v.grad, rgv, "trainable vt, edited table: grad vertices vs oracle")
