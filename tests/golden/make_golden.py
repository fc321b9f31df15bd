"""Generate the golden vectors in tests/golden/*.npz by running the REFERENCE implementation.

Run in the build container only (needs /root/reference):   python tests/golden/make_golden.py

The reference Python package is imported through tests/golden/refimport.py (stubs for imageio,
chainer and the CUDA extension; the extension's two kernels are served by the CPU oracle
restatement).  Everything above the two kernels -- to_map, MaskForeground, the depth / coordinate /
texture maps, Differentiation, flip and anti-aliasing, Renderer / look_at / perspective, load_obj --
is the reference's own code, so these fixtures pin the oracle's Python restatement and the HIP
path independently of them.  The face-index / weight kernels themselves are pinned by the
reference's own data (tests/test_oracle_pins.py).

Each fixture holds inputs and expected outputs only (no reference source).
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, REPO)
import refimport  # noqa: E402
from neural_renderer_v2_pytorch_amd import synthetic  # noqa: E402

R = refimport.load()
rast = sys.modules["nrt_ref.rasterize"]
RP = sys.modules["nrt_ref.rasterize_param"]
DATA = os.path.join(REPO, "tests", "data")
TEAPOT = os.path.join(DATA, "teapot.obj")
CAR = os.path.join(DATA, "4e49873292196f02574b5684eaec43e9", "model.obj")


def save(name, **arrays):
    out = {}
    for k, v in arrays.items():
        if torch.is_tensor(v):
            v = v.detach().cpu().numpy()
        out[k] = np.asarray(v)
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **out)
    print("%-28s %8.1f KB  %s" % (name, os.path.getsize(path) / 1024, sorted(out)))


def internals(proj, faces, S, near=0.1, far=100.0, draw_backside=True):
    """face-index and weight maps through the reference's own rasterize.py:60-77 wrappers."""
    hp = RP.RasterizeHyperparam(image_size=S, near=near, far=far, draw_backside=draw_backside)
    fg = proj.detach()[:, torch.as_tensor(faces).long()]
    fim = rast.compute_face_index_map(fg, hp)
    w = rast.compute_weight_map(fg, fim)
    return fim, w


def flags_call(fn, proj, faces, params, hp):
    leaf = proj.detach().clone().requires_grad_(True)
    img = fn(leaf, torch.as_tensor(faces), params, hp)
    return leaf, img


def teapot_batch(slot=2, B=4):
    v, f = R.load_obj.load_obj(TEAPOT)
    vb = np.tile(v[None], (B, 1, 1)) * 0
    vb[slot] = v
    return vb.astype(np.float32), f


def scene_square():
    vertices = np.array([[0.1, 0.1, 1.], [-0.1, 0.1, 1.], [-0.1, -0.1, 1.], [0.1, -0.1, 1.]], 'float32')
    faces = np.array([[0, 1, 2], [0, 2, 3]], 'int32')
    ref = 1 - R.utils.imread(os.path.join(DATA, "gradient.png"))[:, :, 0]
    ref = torch.as_tensor(ref)
    v = torch.nn.Parameter(torch.tensor(vertices))  # a copy: Adam updates v in place
    opt = torch.optim.Adam([v], lr=0.005)
    first_grad = None
    first_img = None
    conv = -1
    for i in range(350):
        hp = RP.RasterizeHyperparam(image_size=256, anti_aliasing=False)
        img = R.rasterize_silhouettes(v[None], torch.as_tensor(faces), RP.RasterizeParam(), hp)[0]
        iou = torch.sum(img * ref) / torch.sum(img + ref - img * ref)
        loss = 1 - iou
        opt.zero_grad()
        loss.backward()
        if first_grad is None:
            first_grad = v.grad.clone()
            first_img = img.detach().clone()
        opt.step()
        if float(loss) < 0.01:
            conv = i
            break
    fim, w = internals(torch.as_tensor(vertices)[None], faces, 256)
    save("square_sil", vertices=vertices, faces=faces, fim=fim, weight_map=w, images=first_img[None],
         iou_grad=first_grad, converge_step=np.int32(conv))


def scene_teapot_sil():
    vb, f = teapot_batch()
    ren = R.Renderer()
    ren.anti_aliasing = False
    ren.viewpoints = R.utils.get_points_from_angles(2.732, 0, 0)
    vt = torch.as_tensor(vb).requires_grad_(True)
    proj = ren.transform_vertices(vt)
    img = ren.render_silhouettes(vt, torch.as_tensor(f))
    g = torch.as_tensor(np.random.RandomState(11).normal(size=img.shape).astype(np.float32))
    img.backward(g)
    leaf, img2 = flags_call(R.rasterize_silhouettes, proj, f, RP.RasterizeParam(),
                            RP.RasterizeHyperparam(image_size=256, anti_aliasing=False))
    img2.backward(g)
    fim, w = internals(proj, f, 256)
    save("teapot_sil", vertices=vb, faces=f, eye=np.asarray(ren.viewpoints, np.float32), proj=proj,
         fim=fim, weight_map=w, images=img, grad_up=g, grad_vertices=vt.grad, grad_proj=leaf.grad)


def scene_teapot_depth():
    vb, f = teapot_batch()
    ren = R.Renderer()
    ren.anti_aliasing = False
    ren.viewpoints = R.utils.get_points_from_angles(2, 30., 0)
    vt = torch.as_tensor(vb)
    proj = ren.transform_vertices(vt)
    leaf, img = flags_call(R.rasterize_depth, proj, f, RP.RasterizeParam(),
                           RP.RasterizeHyperparam(image_size=256, anti_aliasing=False))
    g = torch.as_tensor(np.random.RandomState(12).normal(size=img.shape).astype(np.float32))
    img.backward(g)
    save("teapot_depth", vertices=vb, faces=f, eye=np.asarray(ren.viewpoints, np.float32), proj=proj,
         images=img, grad_up=g, grad_proj=leaf.grad)


def _textured(name, proj, f, vt_np, ft_np, tex_np, image_size, aa, draw_backside, fn, shared_tex, seed):
    B = proj.shape[0]
    tex_leaf = torch.as_tensor(tex_np).requires_grad_(True)
    if shared_tex:
        textures = tex_leaf[None].expand((B,) + tex_leaf.shape)
        vts = torch.as_tensor(vt_np)[None].expand((B,) + vt_np.shape)
    else:
        textures = tex_leaf
        vts = torch.as_tensor(vt_np)
    params = RP.RasterizeParam(vertices_textures=vts, faces_textures=torch.as_tensor(ft_np), textures=textures)
    hp = RP.RasterizeHyperparam(image_size=image_size, anti_aliasing=aa, draw_backside=draw_backside)
    leaf, img = flags_call(fn, proj, f, params, hp)
    g = torch.as_tensor(np.random.RandomState(seed).normal(size=img.shape).astype(np.float32))
    img.backward(g)
    S = image_size * (2 if aa else 1)
    fim, w = internals(proj, f, S, draw_backside=draw_backside)
    save(name, proj=proj, faces=f, vertices_textures=vt_np, faces_textures=ft_np, textures=tex_np,
         shared_textures=np.int32(shared_tex), image_size=np.int32(image_size), anti_aliasing=np.int32(aa),
         draw_backside=np.int32(draw_backside), fim=fim, weight_map=w, images=img, grad_up=g,
         grad_proj=leaf.grad, grad_textures=tex_leaf.grad)


def rasterize_all(v, f, params, hp):
    hp.draw_rgb = hp.draw_silhouettes = hp.draw_depth = True
    return rast.rasterize_core(v, f, params, hp)


def scene_teapot_textured():
    v, f = R.load_obj.load_obj(TEAPOT)
    eyes = np.stack([R.utils.get_points_from_angles(2.732, 30, 30),
                     R.utils.get_points_from_angles(2.732, -20, 135)]).astype(np.float32)
    vb = torch.as_tensor(np.tile(v[None], (2, 1, 1)))
    proj = R.perspective(R.look_at(vb, torch.as_tensor(eyes)))
    vt, ft, tex = R.utils.create_textures(f.shape[0], texture_size=4)
    tex = np.random.RandomState(3).uniform(0, 1, tex.shape).astype(np.float32)
    _textured("teapot_rgbsd_aa", proj, f, vt, ft, tex, 64, True, True, rasterize_all, True, 21)
    _textured("teapot_rgb_nobs", proj, f, vt, ft, tex, 96, False, False, R.rasterize_rgb, True, 22)
    _textured("teapot_rgba_aa", proj, f, vt, ft, tex, 48, True, False, R.rasterize_rgba, True, 23)


def scene_ico():
    v, f = synthetic.icosphere(2)
    B = 3
    vb = synthetic.jittered(v, B)
    eyes = synthetic.viewpoints(B)
    # project per item (the reference look_at mis-crosses at batch size 3)
    proj = torch.cat([R.perspective(R.look_at(torch.as_tensor(vb[b:b + 1]), torch.as_tensor(eyes[b:b + 1])))
                      for b in range(B)], 0)
    vt, ft, tex = R.utils.create_textures(f.shape[0], texture_size=4)
    r = np.random.RandomState(4)
    tex = r.uniform(0, 1, (B,) + tex.shape).astype(np.float32)
    vt = np.tile(vt[None], (B, 1, 1))
    _textured("ico_rgbsd_aa", proj, f, vt, ft, tex, 40, True, True, rasterize_all, False, 24)


def scene_car():
    ren = R.Renderer()
    ren.draw_backside = False
    ren.viewpoints = R.utils.get_points_from_angles(2.5, 10, -90)
    v, f, vt, ft, tex = R.load_obj.load_obj(CAR, load_textures=True)
    vv = torch.as_tensor(v[None])
    img = ren.render(vv, torch.as_tensor(f), torch.as_tensor(vt[None]), torch.as_tensor(ft),
                     torch.as_tensor(tex[None]))
    proj = ren.transform_vertices(vv)
    t = tex.astype(np.float64)
    save("car1_rgba", vertices=v, faces=f, vertices_textures=vt, faces_textures=ft,
         textures_shape=np.asarray(tex.shape), textures_sum=np.float64(t.sum()),
         textures_sumsq=np.float64((t * t).sum()), eye=np.asarray(ren.viewpoints, np.float32), proj=proj,
         images=img)


def scene_diff_kat():
    out = {}
    for i, shape in enumerate([(3, 16, 16, 4), (2, 12, 20, 3), (1, 32, 32, 5)]):
        r = np.random.RandomState(30 + i)
        images = torch.as_tensor(r.normal(size=shape).astype(np.float32))
        if i == 2:  # silhouette-like piecewise-constant images exercise the |R-L| < eps and max <= 0 rules
            images = torch.as_tensor((r.uniform(size=shape) > 0.5).astype(np.float32))
        coords = torch.zeros(shape[:3] + (2,), requires_grad=True)
        g = torch.as_tensor(r.normal(size=shape).astype(np.float32))
        y = R.differentiation.differentiation(images, coords)
        y.backward(g)
        out["images%d" % i] = images
        out["grad%d" % i] = g
        out["grad_xy%d" % i] = coords.grad
    save("diff_kat", **out)


def scene_edges():
    """Adversarial face soups for the face-index kernel: pixel-aligned vertices (edge ties),
    near-coplanar overlaps inside depth_min_delta (order dependence), degenerate and huge faces,
    faces behind near / beyond far, NaN and inf coordinates."""
    out = {}
    for i, (B, F, S) in enumerate([(2, 300, 64), (1, 500, 50), (2, 64, 33)]):
        r = np.random.RandomState(40 + i)
        grid = (2 * r.randint(0, S, (B, F, 3, 2)) + 1 - S) / S              # pixel centres
        jit = r.uniform(-1.3, 1.3, (B, F, 3, 2))
        xy = np.where(r.uniform(size=(B, F, 1, 1)) < 0.5, grid, jit)
        z = np.repeat(r.choice([1.0, 1.00003, 1.00006, 1.0001, 1.5, 2.0], (B, F, 1, 1)), 3, 2)
        z = z + np.where(r.uniform(size=(B, F, 1, 1)) < 0.3, r.uniform(-0.2, 0.2, (B, F, 3, 1)), 0)
        faces = np.concatenate([xy, z], -1).astype(np.float32)
        faces[:, :8] = faces[:, :8] * 4                                       # huge faces
        faces[:, 8:12, 2] = 0.05                                               # before near
        faces[:, 12:16, 2] = 200.                                              # beyond far
        faces[:, 16:20, 1] = faces[:, 16:20, 0]                                # degenerate
        faces[:, 20, 0, 0] = np.nan
        faces[:, 21, 1, 2] = np.nan
        faces[:, 22, 2, 0] = np.inf
        faces[:, 23, 0, 1] = -np.inf
        for bs in (True, False):
            fim = torch.as_tensor(refimport.oracle.face_index_map(faces, S, 0.1, 100.0, bs, 1e-4))
            w = rast.compute_weight_map(torch.as_tensor(faces), fim)
            # reference python path for the face-index wrapper, as a cross-check of the stub
            hp = RP.RasterizeHyperparam(image_size=S, draw_backside=bs)
            fim2 = rast.compute_face_index_map(torch.as_tensor(faces), hp)
            assert torch.equal(fim, fim2)
            out["faces%d" % i] = faces
            out["fim%d_%d" % (i, bs)] = fim
            out["weight%d_%d" % (i, bs)] = w
    save("edges", **out)


def _light_arrays(lights):
    """Light objects -> plain arrays for the fixture: kind 0 ambient, 1 directional, 2 specular."""
    kinds, colors, dirs, alphas, backs = [], [], [], [], []
    for L in lights:
        kind = {"AmbientLight": 0, "DirectionalLight": 1, "SpecularLight": 2}[type(L).__name__]
        kinds.append(kind)
        colors.append(L.color.detach().numpy())
        dirs.append(L.direction.detach().numpy() if kind == 1 else np.zeros_like(L.color.detach().numpy()))
        alphas.append(L.alpha.detach().numpy() if kind == 2 else np.ones(L.color.shape[0], np.float32))
        backs.append(int(getattr(L, "backside", False)))
    return dict(light_kind=np.asarray(kinds, np.int32), light_color=np.stack(colors),
                light_direction=np.stack(dirs), light_alpha=np.stack(alphas), light_backside=np.asarray(backs, np.int32))


def _lit(name, ren_fn, proj, f, vt, ft, tex_np, lights, image_size, aa, draw_backside, seed, shared_tex=True):
    """A textured render with lights through the reference's rasterize_* (lights loop
    rasterize.py:252-283, compute_normal_map :162-190), forward and backward."""
    B = proj.shape[0]
    tex_leaf = torch.as_tensor(tex_np).requires_grad_(True)
    textures = tex_leaf[None].expand((B,) + tex_leaf.shape) if shared_tex else tex_leaf
    vts = torch.as_tensor(vt)[None].expand((B,) + vt.shape)
    params = RP.RasterizeParam(vertices_textures=vts, faces_textures=torch.as_tensor(ft), textures=textures,
                               lights=lights)
    hp = RP.RasterizeHyperparam(image_size=image_size, anti_aliasing=aa, draw_backside=draw_backside)
    leaf, img = flags_call(ren_fn, proj, f, params, hp)
    g = torch.as_tensor(np.random.RandomState(seed).normal(size=img.shape).astype(np.float32))
    img.backward(g)
    save(name, proj=proj, faces=f, vertices_textures=vt, faces_textures=ft, textures=tex_np,
         shared_textures=np.int32(shared_tex), image_size=np.int32(image_size), anti_aliasing=np.int32(aa),
         draw_backside=np.int32(draw_backside), images=img, grad_up=g, grad_proj=leaf.grad,
         grad_textures=tex_leaf.grad, **_light_arrays(lights))


def scene_lights():
    Lm = R.lights
    # tests_torch/test_rasterize.py:158-200 (test_forward_case4): teapot in slot 2 of 4, three lights,
    # no backside, render_rgb; here at 96^2 output, with a random texture atlas and the backward
    vb, f = teapot_batch()
    eye = R.utils.get_points_from_angles(2.732, 30, 30)
    proj = R.perspective(R.look_at(torch.as_tensor(vb), eye))
    vt, ft, tex = R.utils.create_textures(f.shape[0], texture_size=4)
    tex = np.random.RandomState(5).uniform(0, 1, tex.shape).astype(np.float32)
    c1 = torch.as_tensor([[0.47481096, 0.7131511, 0.4510043], [0.49120015, 0.161955, 0.71638113],
                          [0.32655084, 0.7805874, 0.7682426], [0.42193118, 0.90416473, 0.5267034]])
    d1 = torch.as_tensor([[0.328245, 0.8916046, 0.31189483], [0.99824226, 0.05838178, 0.00867782],
                          [0.35747865, 0.61983925, 0.6985467], [0.0393897, 0.6937492, 0.7191179]])
    c2 = torch.as_tensor([[0.2732121, 0.09439224, 0.38380036], [0.06487979, 0.02794903, 0.261018],
                          [0.28739947, 0.2996951, 0.42412606], [0.10019363, 0.26517034, 0.07372955]])
    c3 = torch.as_tensor([[0.32410273, 0.24369295, 0.3126097], [0.3456873, 0.24514836, 0.21663068],
                          [0.33004418, 0.25533527, 0.48039845], [0.29468802, 0.44377372, 0.10724097]])
    lights = [Lm.DirectionalLight(c1, d1), Lm.AmbientLight(c2), Lm.SpecularLight(c3)]
    _lit("teapot_lights", R.rasterize_rgb, proj, f, vt, ft, tex, lights, 96, True, False, 41)
    # every light kind and option (backside, specular alpha), all channels, per-item light values
    v, fi = synthetic.icosphere(2)
    B = 2
    vb = synthetic.jittered(v, B)
    eyes = synthetic.viewpoints(B)
    proj = torch.cat([R.perspective(R.look_at(torch.as_tensor(vb[b:b + 1]), torch.as_tensor(eyes[b:b + 1])))
                      for b in range(B)], 0)
    vt, ft, tex = R.utils.create_textures(fi.shape[0], texture_size=4)
    tex = np.random.RandomState(6).uniform(0, 1, tex.shape).astype(np.float32)
    r = np.random.RandomState(7)
    col = lambda: torch.as_tensor(r.uniform(0.1, 0.6, (B, 3)).astype(np.float32))
    dirn = lambda: torch.nn.functional.normalize(torch.as_tensor(r.normal(size=(B, 3)).astype(np.float32)), dim=1)
    lights = [Lm.AmbientLight(col()), Lm.DirectionalLight(col(), dirn()), Lm.DirectionalLight(col(), dirn(), backside=True),
              Lm.SpecularLight(col(), alpha=torch.as_tensor([2.5, 0.7])), Lm.SpecularLight(col(), backside=True)]
    _lit("ico_lights", rasterize_all, proj, fi, vt, ft, tex, lights, 40, True, True, 42)


def scene_param_grads():
    """Gradients w.r.t. the vertices_textures and the light parameters (colours, directions,
    specular exponents): the reference's autograd through sample_textures (rasterize.py:100-153,
    the faces_textures gather at :246) and the light loop (:252-283).  Two cases: per-item uv
    coordinates with every light kind, and uv coordinates shared by the batch (an expanded
    [1, Vt, 2] leaf) without lights."""
    Lm = R.lights
    v, fi = synthetic.icosphere(2)
    B = 2
    vb = synthetic.jittered(v, B)
    eyes = synthetic.viewpoints(B)
    proj = torch.cat([R.perspective(R.look_at(torch.as_tensor(vb[b:b + 1]), torch.as_tensor(eyes[b:b + 1])))
                      for b in range(B)], 0)
    vt, ft, tex = R.utils.create_textures(fi.shape[0], texture_size=4)
    tex = np.random.RandomState(8).uniform(0, 1, tex.shape).astype(np.float32)
    r = np.random.RandomState(9)
    # uv coordinates moved off the texel grid (a per-item jitter of up to a quarter texel)
    # (clipped so that the bilinear +1 neighbour stays inside the atlas, where the reference indexes)
    hw = np.asarray([tex.shape[2], tex.shape[1]], np.float32)
    vt_items = np.clip(vt[None] + r.uniform(-0.25, 0.25, (B,) + vt.shape), 0, hw - 1.01).astype(np.float32)
    col = lambda: torch.as_tensor(r.uniform(0.1, 0.6, (B, 3)).astype(np.float32)).requires_grad_(True)
    dirn = lambda: torch.nn.functional.normalize(torch.as_tensor(r.normal(size=(B, 3)).astype(np.float32)),
                                                 dim=1).detach().requires_grad_(True)
    alpha = torch.as_tensor([1.5, 0.8]).requires_grad_(True)
    lights = [Lm.AmbientLight(col()), Lm.DirectionalLight(col(), dirn()), Lm.DirectionalLight(col(), dirn(), backside=True),
              Lm.SpecularLight(col(), alpha=alpha), Lm.SpecularLight(col(), backside=True)]
    for case, (vts_np, lts) in {"param_grads_items": (vt_items, lights), "param_grads_shared": (vt_items[:1], None)}.items():
        tex_leaf = torch.as_tensor(tex).requires_grad_(True)
        vt_leaf = torch.as_tensor(vts_np).requires_grad_(True)
        vts = vt_leaf if vt_leaf.shape[0] == B else vt_leaf.expand((B,) + vt_leaf.shape[1:])
        params = RP.RasterizeParam(vertices_textures=vts, faces_textures=torch.as_tensor(ft),
                                   textures=tex_leaf[None].expand((B,) + tex_leaf.shape), lights=lts)
        hp = RP.RasterizeHyperparam(image_size=40, anti_aliasing=True, draw_backside=True)
        leaf, img = flags_call(rasterize_all, proj, fi, params, hp)
        g = torch.as_tensor(np.random.RandomState(43).normal(size=img.shape).astype(np.float32))
        img.backward(g)
        extra = {}
        if lts is not None:
            extra = _light_arrays(lts)
            extra["grad_light_color"] = np.stack([L.color.grad.numpy() for L in lts])
            extra["grad_light_direction"] = np.stack([L.direction.grad.numpy() if hasattr(L, "direction")
                                                      else np.zeros((B, 3), np.float32) for L in lts])
            # only the explicitly given exponent is a leaf (SpecularLight's default is a constant)
            extra["light_alpha_requires_grad"] = np.asarray([int(L.alpha.requires_grad) if hasattr(L, "alpha") else 0
                                                             for L in lts], np.int32)
            extra["grad_light_alpha"] = np.stack([L.alpha.grad.numpy() for L in lts
                                                  if hasattr(L, "alpha") and L.alpha.requires_grad])
        save(case, proj=proj, faces=fi, vertices_textures=vts_np, faces_textures=ft, textures=tex,
             image_size=np.int32(40), anti_aliasing=np.int32(1), draw_backside=np.int32(1), images=img, grad_up=g,
             grad_proj=leaf.grad, grad_textures=tex_leaf.grad, grad_vertices_textures=vt_leaf.grad, **extra)


if __name__ == "__main__":
    torch.manual_seed(0)
    todo = sys.argv[1:] or ["square", "teapot_sil", "teapot_depth", "teapot_textured", "ico", "car",
                            "diff_kat", "edges", "lights"]
    for name in todo:
        globals()["scene_" + name]()
