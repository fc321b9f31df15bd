"""Host-side (Python + ctypes + torch dispatch) profile of the eager teapot B=4 step (cfg2), where the
step is bound by the host's launch path rather than the kernels.  usage (GPU box):
python tools/host_profile.py [steps]"""
import cProfile
import os
import pstats
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import bench_configs  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 300
_, step = None, None


def cfg2_step():
    import numpy as np
    import neural_renderer_v2_pytorch_amd as nr
    v, f = nr.load_obj(os.path.join(bench_configs.DATA, "teapot.obj"))
    B, s = 4, 256
    proj = bench_configs.scene(v, f, B, dev)
    vt, ft, tex = nr.create_textures(f.shape[0], texture_size=4)
    tex = torch.as_tensor(np.random.RandomState(3).uniform(0, 1, tex.shape).astype(np.float32), device=dev)
    tex.requires_grad_(True)
    vt_d, ft_d = torch.as_tensor(vt, device=dev), torch.as_tensor(ft, device=dev)
    faces = torch.as_tensor(f, device=dev)
    g = torch.randn((B, 5, s, s), device=dev)

    def step():
        proj.grad = tex.grad = None
        params = nr.RasterizeParam(vertices_textures=vt_d[None].expand(B, -1, -1), faces_textures=ft_d,
                                   textures=tex[None].expand(B, -1, -1, -1))
        nr.rasterize_core(proj, faces, params, nr.RasterizeHyperparam(image_size=s)).backward(g)
    return step


step = cfg2_step()
for _ in range(20):
    step()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(n):
    step()
t_host = (time.perf_counter() - t0) / n
torch.cuda.synchronize()
t_all = (time.perf_counter() - t0) / n
print("host enqueue %.3f ms/step, with the GPU %.3f ms/step" % (1e3 * t_host, 1e3 * t_all))
pr = cProfile.Profile()
pr.enable()
for _ in range(n):
    step()
pr.disable()
torch.cuda.synchronize()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(25)
