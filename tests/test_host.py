"""Host-side logic and the C ABI library (no GPU needed)."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

import neural_renderer_v2_pytorch_amd as nr
from neural_renderer_v2_pytorch_amd import _lib, synthetic
from conftest import DATA, ROOT


def test_look_at_kat():
    """tests_torch/test_look_at.py:10-26."""
    vertices = torch.as_tensor(np.array([1, 0, 0], 'float32'))[None, None, :]
    cases = [([1, 0, 1], [-np.sqrt(2) / 2, 0, np.sqrt(2) / 2]), ([0, 0, -10], [1, 0, 10]),
             ([-1, 1, 0], [0, np.sqrt(2) / 2, 3. / 2. * np.sqrt(2)])]
    for e, a in cases:
        out = nr.look_at(vertices, torch.as_tensor(np.array(e, 'float32')))
        np.testing.assert_allclose(out.flatten().numpy(), np.array(a), rtol=1e-6, atol=1e-6)


def test_perspective_kat():
    """tests_torch/test_perspective.py:10-16."""
    v = torch.as_tensor(np.array([1, 2, 10], 'float32'))[None, None, :]
    np.testing.assert_allclose(nr.perspective(v).flatten().numpy(),
                               np.asarray([np.sqrt(3) / 10, 2 * np.sqrt(3) / 10, 10], np.float32), rtol=1e-5)


def test_look_at_batch3_is_per_item():
    """The reference's dim-less torch.cross mixes items at batch size 3; ours is per item."""
    v = torch.randn(3, 7, 3)
    eyes = torch.as_tensor(synthetic.viewpoints(3))
    batched = nr.look_at(v, eyes)
    single = torch.cat([nr.look_at(v[i:i + 1], eyes[i:i + 1]) for i in range(3)])
    assert torch.allclose(batched, single, atol=1e-6)


def test_renderer_transform_matches_golden(golden):
    d = golden("teapot_sil")
    ren = nr.Renderer()
    ren.viewpoints = nr.get_points_from_angles(2.732, 0, 0)
    proj = ren.transform_vertices(torch.as_tensor(d["vertices"]))
    np.testing.assert_allclose(proj.numpy(), d["proj"], rtol=1e-6, atol=1e-6)


def test_load_obj_car_matches_reference(golden):
    d = golden("car1_rgba")
    v, f, vt, ft, tex = nr.load_obj(os.path.join(DATA, "4e49873292196f02574b5684eaec43e9", "model.obj"),
                                    load_textures=True)
    assert np.array_equal(v, d["vertices"]) and np.array_equal(f, d["faces"])
    assert np.array_equal(vt, d["vertices_textures"]) and np.array_equal(ft, d["faces_textures"])
    t = tex.astype(np.float64)
    assert list(tex.shape) == list(d["textures_shape"])
    assert abs(t.sum() - float(d["textures_sum"])) <= 1e-9 * float(d["textures_sum"])
    assert abs((t * t).sum() - float(d["textures_sumsq"])) <= 1e-9 * float(d["textures_sumsq"])


def test_load_obj_teapot(golden):
    v, f = nr.load_obj(os.path.join(DATA, "teapot.obj"))
    d = golden("teapot_sil")
    assert np.array_equal(v, d["vertices"][2]) and np.array_equal(f, d["faces"])


def test_save_load_roundtrip(tmp_path):
    v, f, vt, ft, tex = nr.load_obj(os.path.join(DATA, "4e49873292196f02574b5684eaec43e9", "model.obj"),
                                    load_textures=True)
    path = str(tmp_path / "m.obj")
    nr.save_obj(path, v, f, vt, ft, tex)
    v2, f2, vt2, ft2, tex2 = nr.load_obj(path, load_textures=True, normalization=False)
    assert np.allclose(v2, v, atol=1e-6) and np.array_equal(f2, f) and np.array_equal(ft2, ft)
    assert tex2.shape == tex.shape and np.abs(tex2 - tex).max() <= 1 / 255. + 1e-6


def test_create_textures_layout():
    vt, ft, tex = nr.create_textures(5120, texture_size=4)
    assert tex.shape == (3, 288, 288) and vt.shape == (5120 * 3, 2) and ft.shape == (5120, 3)
    assert vt.max() == 287 and vt.min() == 0


def test_synthetic_meshes():
    v, f = synthetic.icosphere(4)
    assert v.shape == (2562, 3) and f.shape == (5120, 3)
    v, f = synthetic.torus()
    assert v.shape == (25000, 3) and f.shape == (50000, 3)
    assert f.min() == 0 and f.max() == 24999


def test_library_exports_every_header_symbol():
    """The C-ABI library loads and exports exactly what include/nr_raster.h declares."""
    header = open(os.path.join(ROOT, "include", "nr_raster.h")).read()
    # the diagnostic build's counters (#ifdef NR_COUNT_TESTS) are declared for that build only
    diag = re.findall(r"^#ifdef NR_COUNT_TESTS\n(.*?)^#endif", header, re.M | re.S)
    header = re.sub(r"^#ifdef NR_COUNT_TESTS\n.*?^#endif", "", header, flags=re.M | re.S)
    decl = r"^\s*(?:NR_API\s+)?(?:const\s+)?\w+\s*\*?\s*(nr_\w+)\s*\("
    declared = set(re.findall(decl, header, re.M))
    assert declared == set(_lib.EXPORTS), declared ^ set(_lib.EXPORTS)
    assert set(re.findall(decl, "".join(diag), re.M)) == {"nr_count_read"}
    count_lib = os.path.join(_lib.LIB_DIR, "libnr_raster_count.so")
    assert hasattr(ctypes.CDLL(count_lib), "nr_count_read")
    assert not hasattr(ctypes.CDLL(_lib.LIB_PATH), "nr_count_read")
    L = ctypes.CDLL(_lib.LIB_PATH)
    for name in declared:
        assert hasattr(L, name), name
    assert _lib.lib().nr_version() == _lib.ABI_VERSION == 6
    assert _lib.lib().nr_hot_acc_bytes(0) == 0
    assert _lib.lib().nr_hot_acc_bytes(3) >= _lib.NR_HOT_COPIES * 3 * 64 * 4 + 3 * 8
    # the ctypes mirror of NrRasterArgs has the C layout
    assert _lib.lib().nr_raster_args_size() == ctypes.sizeof(_lib.NrRasterArgs)
    assert _lib.lib().nr_num_channels(7) == 5 and _lib.lib().nr_num_channels(2) == 1
    assert _lib.lib().nr_workspace_bytes(64, 5120, 512) >= 64 * 5120 * 8 + 64 * 64 * 160 * 4


def test_abi_rejects_bad_arguments():
    """Error behaviour without touching the GPU: argument validation runs before any launch."""
    L = _lib.lib()
    st = L.nr_face_index_map_forward_safe(None, None, 1, 10, 0, 0.1, 100., 1, 1e-8, 1e-4, None, 0, None)
    assert st == 1 and b"bad sizes" in L.nr_last_error()
    a = _lib.NrRasterArgs()
    a.batch_size, a.num_faces, a.num_vertices, a.image_size, a.draw_flags = 1, 1, 3, 8, 0
    assert L.nr_rasterize_forward(ctypes.byref(a), None, None) == 1
    assert b"nothing to draw" in L.nr_last_error()


def test_no_cpu_fallback():
    v = torch.rand(1, 3, 3)
    with pytest.raises(RuntimeError, match="GPU only"):
        nr.rasterize_silhouettes(v, torch.as_tensor([[0, 1, 2]]), nr.RasterizeParam(), nr.RasterizeHyperparam())


def test_differentiation_cpu_golden(golden):
    """BASELINE cfg1: the reference's Differentiation runs on CPU tensors (differentiation.py:6-36).
    The package's CPU branch against the golden KAT made by the reference itself, bit for bit."""
    d = golden("diff_kat")
    for i in range(3):
        images = torch.as_tensor(d["images%d" % i])
        coords = torch.zeros(images.shape[:3] + (2,), requires_grad=True)
        y = nr.differentiation(images, coords)
        assert y is images or torch.equal(y, images)
        y.backward(torch.as_tensor(d["grad%d" % i]))
        assert torch.equal(coords.grad, torch.as_tensor(d["grad_xy%d" % i])), i


def test_differentiation_cpu_reference_procedure():
    """tests_torch/test_differentiation.py:10-65 verbatim procedure, on CPU tensors (cfg1)."""
    r = np.random.RandomState(0)
    images = torch.as_tensor(r.normal(size=(10, 32, 32, 3)).astype('float32'))
    x = np.tile(np.arange(32).astype('float32')[None, None, :, None], (10, 32, 1, 1))
    y = np.tile(np.arange(32).astype('float32')[None, :, None, None], (10, 1, 32, 1))
    coordinates = ((np.concatenate((x, y), axis=-1) / 31) * 2 - 1) * 31. / 32.
    noise = torch.as_tensor(r.normal(size=(10, 32, 32, 3)).astype('float32'))
    step = 2 / 32.
    coordinates = torch.tensor(coordinates, requires_grad=True)
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


def test_cfg1_cpu_pipeline():
    """BASELINE cfg1 end to end on the CPU: teapot -> look_at -> perspective -> differentiation,
    with gradients reaching the vertices through the projection (the rasterizer itself is GPU only)."""
    v, f = nr.load_obj(os.path.join(DATA, "teapot.obj"))
    verts = torch.as_tensor(v[None]).requires_grad_(True)
    eye = torch.as_tensor(nr.get_points_from_angles(2.732, 0, 90), dtype=torch.float32)[None]
    proj = nr.perspective(nr.look_at(verts, eye))
    S = 16
    img = torch.zeros((1, S, S, 3))
    # a smooth image whose values depend on the projected vertices, then the soft gradient
    img = img + proj[:, :S * S, :].reshape(1, S, S, 3)
    coords = proj[:, :S * S, :2].reshape(1, S, S, 2)
    out = nr.differentiation(img, coords)
    (out * torch.linspace(-1, 1, out.numel()).reshape(out.shape)).sum().backward()
    assert verts.grad is not None and torch.isfinite(verts.grad).all() and float(verts.grad.abs().sum()) > 0


def test_product_never_imports_oracle():
    pkg = os.path.join(ROOT, "neural_renderer_v2_pytorch_amd")
    for dirpath, _, files in os.walk(pkg):
        for fn in files:
            if fn.endswith((".py", ".hip", ".h", ".cpp")):
                src = open(os.path.join(dirpath, fn)).read()
                assert not re.search(r"^\s*(import|from)\s+oracle", src, re.M), fn
                assert "libnr_oracle" not in src, fn


def test_reference_binding_module_checks_inputs():
    """rasterize_cuda mirrors the reference's CHECK_INPUT (cuda/rasterize_cuda.cpp:5-7): a CPU or
    non-contiguous tensor raises RuntimeError before any launch; the dead unsafe kernel is refused."""
    from neural_renderer_v2_pytorch_amd import rasterize_cuda as rc
    faces = torch.zeros((1, 2, 3, 3))
    fi = torch.zeros(16, dtype=torch.int32) - 1
    with pytest.raises(RuntimeError, match="must be a CUDA tensor"):
        rc.face_index_map_forward_safe(faces, fi, 2, 4, 0.1, 100., 1, 1e-8, 1e-4)
    with pytest.raises(RuntimeError, match="must be a CUDA tensor"):
        rc.compute_weight_map_c(faces, fi, torch.zeros(16, 3), 2, 4)
    with pytest.raises(NotImplementedError):
        rc.face_index_map_forward_unsafe(faces, fi, None, None, 2, 4, 0.1, 100., 1, 1e-8)


def test_make_gif(tmp_path):
    """utils.py:10-15: frames _tmp_*.png -> one looping GIF, frames removed."""
    from PIL import Image
    from neural_renderer_v2_pytorch_amd.utils import make_gif
    for i in range(3):
        Image.fromarray(np.full((8, 8), 80 * i, np.uint8)).save(str(tmp_path / ('_tmp_%04d.png' % i)))
    out = str(tmp_path / 'o.gif')
    make_gif(str(tmp_path), out)
    g = Image.open(out)
    assert g.n_frames == 3
    assert not list(tmp_path.glob('_tmp_*.png'))


def test_edge_cull_is_exact_on_host(tmp_path):
    """The forward's edge cull (csrc/nr_cull.h, the same header the kernel includes) compiled for
    the host: over random, pixel-snapped (c2 exactly 0 along an axis-aligned edge 1-2), tiny,
    degenerate and non-finite triangles, no culled 8x8 block has a pixel centre that passes the
    reference's edge tests (.cu:107-116) -- the face would have been walked for nothing, never
    missed. The check also culls about half the cases, so it is not vacuous."""
    import subprocess
    exe = str(tmp_path / "cull_check")
    subprocess.check_call(["g++", "-O2", "-ffp-contract=off", "-I" + os.path.join(ROOT, "neural_renderer_v2_pytorch_amd", "csrc"),
                           os.path.join(ROOT, "tests", "host", "cull_check.cpp"), "-o", exe])
    out = subprocess.run([exe, "2000000"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    m = re.match(r"checked (\d+) culled (\d+) passes-in-culled (\d+)", out.stdout)
    assert m and int(m.group(3)) == 0 and int(m.group(2)) > int(m.group(1)) // 4, out.stdout


def test_tensor_cache_lru():
    """rasterize._TensorCache: a small LRU keyed by (storage, version, ...); hits refresh an
    entry, the least recently used entry leaves first, and entries keep their source alive."""
    from neural_renderer_v2_pytorch_amd.rasterize import _TensorCache
    c = _TensorCache(size=2)
    a, b, d = torch.zeros(3), torch.ones(3), torch.full((3,), 2.0)
    ka, kb, kd = [(t.data_ptr(), t._version) for t in (a, b, d)]
    c.put(ka, a)
    c.put(kb, b)
    assert c.get(ka) is a       # refreshes a: b is now the oldest
    c.put(kd, d)
    assert c.get(kb) is None and c.get(ka) is a and c.get(kd) is d
    a.add_(1)                   # an in-place edit bumps the version: a new key
    assert c.get((a.data_ptr(), a._version)) is None


def test_pixel_centre_is_exact_on_host(tmp_path):
    """csrc/nr_pixel.h (the kernels' pixel centre without doubles: an f32 division, or a 2^-k scaling
    for a power-of-two raster) equals the reference's (float)((2.0 * i + 1 - S) / S)
    (rasterize_cuda_kernel.cu:76-77) bit for bit for every i of every raster size up to 16384."""
    import subprocess
    exe = str(tmp_path / "pixel_centre_check")
    subprocess.check_call(["g++", "-O2", "-ffp-contract=off", "-I" + os.path.join(ROOT, "neural_renderer_v2_pytorch_amd", "csrc"),
                           os.path.join(ROOT, "tests", "host", "pixel_centre_check.cpp"), "-o", exe])
    out = subprocess.run([exe, "16384"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    m = re.match(r"checked (\d+) mismatches (\d+)", out.stdout)
    assert m and int(m.group(2)) == 0 and int(m.group(1)) > 134000000, out.stdout
