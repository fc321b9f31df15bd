"""The CPU oracle, pinned (no GPU needed).

  * the face-index / weight kernels restated in C (oracle/nr_oracle.c) against the reference's own
    data: the alpha channel of tests_torch/data/4e49873292196f02574b5684eaec43e9.png (rendered by
    the reference on CUDA) and the test_backward_case1 convergence step;
  * the same kernels against an independent numpy restatement (vectorised over faces);
  * the oracle's torch restatement of rasterize_core's Python stages against the golden vectors that
    the reference implementation produced (tests/golden/make_golden.py).
"""
import os

import numpy as np
import pytest
import torch

from conftest import DATA


def test_car_alpha_matches_reference_png(golden):
    d = golden("car1_rgba")
    from PIL import Image
    png = np.asarray(Image.open(os.path.join(DATA, "4e49873292196f02574b5684eaec43e9.png")), np.float32) / 255.
    alpha = d["images"][0, 3]
    assert np.abs(alpha - png[:, :, 3]).mean() < 1e-5


def test_square_converges_like_reference(golden):
    d = golden("square_sil")
    assert int(d["converge_step"]) == 221
    g = d["iou_grad"]
    assert np.allclose(np.abs(g[:, :2]), 0.0617, atol=2e-4) and np.all(g[:, 2] == 0)


def _numpy_face_index(faces, S, near=0.1, far=100.0, draw_backside=True, delta=np.float32(1e-4)):
    """Independent restatement of rasterize_cuda_kernel.cu:52-153, vectorised over pixels, looping
    over faces in order (float32 numpy arithmetic; numpy never fuses multiply-adds)."""
    f32 = np.float32
    B, F = faces.shape[:2]
    i = np.arange(S)
    c = ((2. * i + 1 - S) / S).astype(f32)
    yp, xp = np.meshgrid(c, c, indexing="ij")
    out = np.full((B, S, S), -1, np.int32)
    with np.errstate(all="ignore"):
        for b in range(B):
            dmin = np.full((S, S), f32(far), f32)
            idx = np.full((S, S), -1, np.int32)
            for fn in range(F):
                x0, y0, z0, x1, y1, z1, x2, y2, z2 = [f32(v) for v in faces[b, fn].reshape(-1)]
                ok = ~((xp < x0) & (xp < x1) & (xp < x2))
                ok &= ~((x0 < xp) & (x1 < xp) & (x2 < xp))
                ok &= ~((yp < y0) & (yp < y1) & (yp < y2))
                ok &= ~((y0 < yp) & (y1 < yp) & (y2 < yp))
                if not draw_backside and (y2 - y0) * (x1 - x0) > (y1 - y0) * (x2 - x0):
                    continue
                c1 = (yp - y0) * (x1 - x0) - (y1 - y0) * (xp - x0)
                c2 = (yp - y1) * (x2 - x1) - (y2 - y1) * (xp - x1)
                c3 = (yp - y2) * (x0 - x2) - (y0 - y2) * (xp - x2)
                ok &= ~(c1 * c2 < 0) & ~(c2 * c3 < 0)
                det = x2 * (y0 - y1) + x0 * (y1 - y2) + x1 * (y2 - y0)
                if float(abs(det)) < 1e-8:
                    continue
                ok &= ~((dmin < z0) & (dmin < z1) & (dmin < z2))
                w0 = yp * (x2 - x1) + xp * (y1 - y2) + (x1 * y2 - x2 * y1)
                w1 = yp * (x0 - x2) + xp * (y2 - y0) + (x2 * y0 - x0 * y2)
                w2 = yp * (x1 - x0) + xp * (y0 - y1) + (x0 * y1 - x1 * y0)
                s = w0 + w1 + w2
                w0, w1, w2 = w0 / s, w1 / s, w2 / s
                zp = (1. / (w0 / z0 + w1 / z1 + w2 / z2).astype(np.float64)).astype(f32)
                ok &= ~((zp <= f32(near)) | (f32(far) <= zp))
                ok &= zp <= dmin - delta
                dmin = np.where(ok, zp, dmin)
                idx = np.where(ok, fn, idx)
            out[b] = idx
    return out


@pytest.mark.parametrize("i", [0, 1, 2])
def test_face_index_oracle_vs_numpy(golden, oracle_mod, i):
    d = golden("edges")
    faces = d["faces%d" % i]
    S = d["fim%d_1" % i].shape[1]
    for bs in (True, False):
        ref = _numpy_face_index(faces, S, draw_backside=bs)
        got = oracle_mod.face_index_map(faces, S, draw_backside=bs)
        assert np.array_equal(ref, got)
        assert np.array_equal(got, d["fim%d_%d" % (i, int(bs))])


def test_division_double_rounding_is_innocuous():
    """(float)(1.0 / (double)x) == 1.0f / x (reference .cu:139 computes zp in double)."""
    r = np.random.RandomState(0)
    x = np.concatenate([r.uniform(-10, 10, 200000), r.lognormal(0, 20, 200000)]).astype(np.float32)
    with np.errstate(all="ignore"):
        a = (1.0 / x.astype(np.float64)).astype(np.float32)
        b = np.float32(1) / x
    assert np.array_equal(a.view(np.int32), b.view(np.int32))


def _core(oracle_mod, d, name, grads=True):
    B = d["proj"].shape[0]
    proj = torch.as_tensor(d["proj"]).requires_grad_(True)
    tex_leaf = torch.as_tensor(d["textures"]).requires_grad_(True)
    if int(d["shared_textures"]):
        tex = tex_leaf[None].expand(B, *tex_leaf.shape)
        vt = torch.as_tensor(d["vertices_textures"])[None].expand(B, -1, -1)
    else:
        tex, vt = tex_leaf, torch.as_tensor(d["vertices_textures"])
    flags = dict(draw_rgb=True, draw_silhouettes="rgbsd" in name or "rgba" in name, draw_depth="rgbsd" in name)
    img, inter = oracle_mod.rasterize_core(proj, d["faces"], image_size=int(d["image_size"]),
                                           anti_aliasing=bool(d["anti_aliasing"]),
                                           draw_backside=bool(d["draw_backside"]), vertices_textures=vt,
                                           faces_textures=d["faces_textures"], textures=tex, return_internals=True,
                                           **flags)
    img.backward(torch.as_tensor(d["grad_up"]))
    return img, inter, proj.grad, tex_leaf.grad


@pytest.mark.parametrize("name", ["teapot_rgbsd_aa", "teapot_rgb_nobs", "teapot_rgba_aa", "ico_rgbsd_aa"])
def test_oracle_core_vs_reference(golden, oracle_mod, name):
    d = golden(name)
    img, inter, gp, gt = _core(oracle_mod, d, name)
    assert np.array_equal(inter["fim"].numpy(), d["fim"])
    assert np.array_equal(inter["weight_map"].numpy(), d["weight_map"])
    assert np.array_equal(img.detach().numpy(), d["images"]), float(np.abs(img.detach().numpy() - d["images"]).max())
    np.testing.assert_allclose(gp.numpy(), d["grad_proj"], rtol=1e-5, atol=1e-6 * np.abs(d["grad_proj"]).max())
    np.testing.assert_allclose(gt.numpy(), d["grad_textures"], rtol=1e-5, atol=1e-6 * np.abs(d["grad_textures"]).max())


def test_oracle_silhouettes_and_depth(golden, oracle_mod):
    for name, flags in (("teapot_sil", dict(draw_rgb=False, draw_silhouettes=True, draw_depth=False)),
                        ("teapot_depth", dict(draw_rgb=False, draw_silhouettes=False, draw_depth=True))):
        d = golden(name)
        proj = torch.as_tensor(d["proj"]).requires_grad_(True)
        img = oracle_mod.rasterize_core(proj, d["faces"], image_size=256, anti_aliasing=False, **flags)[:, 0]
        assert np.array_equal(img.detach().numpy(), d["images"])
        img.backward(torch.as_tensor(d["grad_up"]))
        np.testing.assert_allclose(proj.grad.numpy(), d["grad_proj"], rtol=1e-5,
                                   atol=1e-6 * np.abs(d["grad_proj"]).max())


def test_oracle_differentiation_vs_reference(golden, oracle_mod):
    d = golden("diff_kat")
    for i in range(3):
        got = oracle_mod.soft_grad_xy(torch.as_tensor(d["images%d" % i]), torch.as_tensor(d["grad%d" % i]))
        assert np.array_equal(got.numpy(), d["grad_xy%d" % i])


class _L:
    """A light with the reference Light attributes (lights.py:4-39), kind given by the class name."""

    def __init__(self, kind, color, direction, alpha, backside):
        self.__class__ = type(kind, (_L,), {})
        self.color, self.direction, self.alpha, self.backside = color, direction, alpha, bool(backside)


def fixture_lights(d, t=torch.as_tensor):
    names = {0: "AmbientLight", 1: "DirectionalLight", 2: "SpecularLight"}
    return [_L(names[int(k)], t(d["light_color"][i]), t(d["light_direction"][i]), t(d["light_alpha"][i]),
               d["light_backside"][i]) for i, k in enumerate(d["light_kind"])]


@pytest.mark.parametrize("name", ["teapot_lights", "ico_lights"])
def test_oracle_lights_vs_reference(golden, oracle_mod, name):
    """normal_map + light loop restatement against the reference's own lit renders and gradients
    (rasterize.py:162-190, 252-283)."""
    d = golden(name)
    B = d["proj"].shape[0]
    pv = torch.as_tensor(d["proj"]).requires_grad_(True)
    tex = torch.as_tensor(d["textures"]).requires_grad_(True)
    chans = d["images"].shape[1]
    img = oracle_mod.rasterize_core(pv, d["faces"], image_size=int(d["image_size"]),
                                    anti_aliasing=bool(d["anti_aliasing"]), draw_backside=bool(d["draw_backside"]),
                                    draw_silhouettes=chans == 5, draw_depth=chans == 5,
                                    vertices_textures=torch.as_tensor(d["vertices_textures"])[None].expand(B, -1, -1),
                                    faces_textures=d["faces_textures"], textures=tex[None].expand(B, -1, -1, -1),
                                    lights=fixture_lights(d))
    np.testing.assert_allclose(img.detach().numpy(), d["images"], rtol=1e-5, atol=1e-5)
    img.backward(torch.as_tensor(d["grad_up"]))
    for got, ref in ((pv.grad, d["grad_proj"]), (tex.grad, d["grad_textures"])):
        scale = np.abs(ref).max()
        np.testing.assert_allclose(got.numpy(), ref, rtol=1e-4, atol=1e-4 * scale)


@pytest.mark.parametrize("name", ["param_grads_items", "param_grads_shared"])
def test_oracle_param_grads_vs_reference(golden, oracle_mod, name):
    """Gradients w.r.t. vertices_textures (through sample_textures' uv interpolation and clamp,
    rasterize.py:111-121, and the gather at :246) and w.r.t. the light colours, directions and
    specular exponents (rasterize.py:252-283): the restatement against the reference's autograd."""
    d = golden(name)
    B = d["proj"].shape[0]
    pv = torch.as_tensor(d["proj"]).requires_grad_(True)
    tex = torch.as_tensor(d["textures"]).requires_grad_(True)
    vt = torch.as_tensor(d["vertices_textures"]).requires_grad_(True)
    lights = None
    if "light_kind" in d:
        leaf = lambda a: torch.as_tensor(a).clone().requires_grad_(True)  # noqa: E731
        lights = fixture_lights(d, t=leaf)
        for L, req in zip(lights, d["light_alpha_requires_grad"]):
            L.alpha.requires_grad_(bool(req))
    img = oracle_mod.rasterize_core(pv, d["faces"], image_size=int(d["image_size"]),
                                    anti_aliasing=bool(d["anti_aliasing"]), draw_backside=bool(d["draw_backside"]),
                                    vertices_textures=vt if vt.shape[0] == B else vt.expand(B, -1, -1),
                                    faces_textures=d["faces_textures"], textures=tex[None].expand(B, -1, -1, -1),
                                    lights=lights)
    np.testing.assert_allclose(img.detach().numpy(), d["images"], rtol=1e-5, atol=1e-5)
    img.backward(torch.as_tensor(d["grad_up"]))
    pairs = [(pv.grad, d["grad_proj"]), (tex.grad, d["grad_textures"]), (vt.grad, d["grad_vertices_textures"])]
    if lights is not None:
        pairs.append((torch.stack([L.color.grad for L in lights]), d["grad_light_color"]))
        pairs += [(L.direction.grad, d["grad_light_direction"][i]) for i, L in enumerate(lights)
                  if type(L).__name__ == "DirectionalLight"]
        pairs.append((torch.stack([L.alpha.grad for L in lights if L.alpha.requires_grad]), d["grad_light_alpha"]))
    for got, ref in pairs:
        np.testing.assert_allclose(got.numpy(), ref, rtol=1e-4, atol=1e-4 * np.abs(ref).max())
