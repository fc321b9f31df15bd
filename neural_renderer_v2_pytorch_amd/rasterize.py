"""Rasterize API -- drop-in for neural_renderer_torch.rasterize (reference rasterize.py:1-365).

Public surface kept: rasterize_silhouettes / rasterize_rgba / rasterize_rgb / rasterize_depth
(rasterize.py:332-365), rasterize_core (:194-329), FaceIndexMap / compute_face_index_map (:14-64),
compute_weight_map (:67-77), RasterizeParam / RasterizeHyperparam.

What changed underneath: rasterize_core is one autograd Function, `Rasterize`, whose forward and
backward are two calls into the HIP library (csrc/nr_raster.hip through include/nr_raster.h):
no per-batch Python loops, no host<->device copies, no intermediate [B,S,S,*] maps in HBM.

Behavioural notes ("Drop-in boundary"):
  * like the reference, the wrappers set hyperparams.draw_* on the object they are given; unlike
    the reference, rasterize_core does NOT double hyperparams.image_size in place under
    anti-aliasing (rasterize.py:227-228 compounds on every reuse of the object);
  * lights (rasterize.py:252-283) are shaded on the GPU, forward and backward (gradients reach the
    vertices through the smooth normal map, and the light colours / directions / exponents);
  * backgrounds / background_color (rasterize.py:208-226, 286-288) blend with the semantics of
    neural_renderer_chainer/rasterize.py:574-577, since the torch blend_backgrounds raises
    AttributeError (rasterize.py:157); background_color gives zeros * colour = black, as both
    references compute it;
  * gradients flow to vertices, textures, vertices_textures, light parameters and backgrounds,
    as the reference's autograd gives them.
"""
import os

import torch

from . import _lib
from .rasterize_param import RasterizeParam, RasterizeHyperparam  # noqa: F401  (re-exported like the reference)


# ------------------------------------------------------------------------------------------------
# the face-index and weight kernels on their own (reference rasterize.py:14-77)
class FaceIndexMap(torch.nn.Module):
    """Z-buffered face index per internal pixel: [B, F, 3, 3] faces -> int32 [B, S, S]
    (-1 = background).  rasterize.py:14-57 / rasterize_cuda_kernel.cu:52-153."""

    def __init__(self, num_faces, image_size, near, far, draw_backside):
        super().__init__()
        self.num_faces = num_faces
        self.image_size = image_size
        self.near = near
        self.far = far
        self.draw_backside = draw_backside

    def forward(self, inputs, **kwargs):
        return self.forward_gpu_safe(inputs)

    def forward_gpu_safe(self, inputs):
        faces = inputs
        _lib.require_gpu(faces)
        faces = faces.detach().contiguous().float()
        B = faces.shape[0]
        S = int(self.image_size)
        fim = torch.empty((B, S, S), dtype=torch.int32, device=faces.device)
        ws = torch.empty(_lib.lib().nr_workspace_bytes(B, int(self.num_faces), S), dtype=torch.uint8,
                         device=faces.device)
        with torch.cuda.device(faces.device):
            _lib.check(_lib.lib().nr_face_index_map_forward_safe(
                _lib.ptr(faces), _lib.ptr(fim), B, int(self.num_faces), S, float(self.near), float(self.far),
                int(self.draw_backside), 1e-8, 1e-4, _lib.ptr(ws), ws.numel(), _lib.stream_of(faces)),
                "nr_face_index_map_forward_safe")
        return fim


def compute_face_index_map(faces, hyperparams):
    return FaceIndexMap(faces.shape[1], hyperparams.image_size, hyperparams.near, hyperparams.far,
                        hyperparams.draw_backside)(faces)


def compute_weight_map(faces, face_index_map):
    """Barycentric weights of the visible face per pixel, [B, S, S, 3] (rasterize.py:67-77)."""
    _lib.require_gpu(faces, face_index_map)
    faces = faces.detach().contiguous().float()
    fim = face_index_map.contiguous().to(torch.int32)
    B, F = faces.shape[:2]
    S = fim.shape[1]
    w = torch.empty((B, S, S, 3), dtype=torch.float32, device=faces.device)
    with torch.cuda.device(faces.device):
        _lib.check(_lib.lib().nr_compute_weight_map(_lib.ptr(faces), _lib.ptr(fim), _lib.ptr(w), B, F, S,
                                                    _lib.stream_of(faces)), "nr_compute_weight_map")
    return w


class MaskForeground(torch.autograd.Function):
    """utils.MaskForeground (utils.py:117-156): keep foreground pixels, zero elsewhere."""

    @staticmethod
    def forward(ctx, data_in, face_index_map):
        _lib.require_gpu(data_in, face_index_map)
        data_in = data_in.contiguous().float()
        fim = face_index_map.contiguous().to(torch.int32)
        out = torch.zeros_like(data_in)
        n = fim.numel()
        dim = data_in.numel() // max(n, 1)
        with torch.cuda.device(data_in.device):
            _lib.check(_lib.lib().nr_mask_foreground_forward(_lib.ptr(fim), _lib.ptr(data_in), _lib.ptr(out), n, dim,
                                                             _lib.stream_of(data_in)), "nr_mask_foreground_forward")
        ctx.save_for_backward(fim)
        ctx.dim = dim
        return out

    @staticmethod
    def backward(ctx, grad):
        fim, = ctx.saved_tensors
        grad = grad.contiguous()
        gin = torch.zeros_like(grad)
        with torch.cuda.device(grad.device):
            _lib.check(_lib.lib().nr_mask_foreground_backward(_lib.ptr(fim), _lib.ptr(gin), _lib.ptr(grad), fim.numel(),
                                                              ctx.dim, _lib.stream_of(grad)), "nr_mask_foreground_backward")
        return gin, None


def mask_foreground(data, face_index_map):
    return MaskForeground.apply(data, face_index_map)


# ------------------------------------------------------------------------------------------------
# the fused path
class _TensorCache:
    """Small LRU of results derived from device index tensors (the faces checks and the vertex
    adjacency), keyed by (storage address, version counter, shape, ...).  Each entry keeps its
    source tensor alive, so its storage -- hence the address in the key -- cannot be freed and
    reused by another tensor while the entry lives; the version counter catches in-place edits.
    A caller alternating a few meshes (several objects, or train / validation sets) keeps hitting:
    no device-to-host copy and no host sync per call, so such steps stay graph-capturable."""

    def __init__(self, size=8):
        import collections
        self.size = size
        self.entries = collections.OrderedDict()

    def get(self, key):
        hit = self.entries.get(key)
        if hit is not None:
            self.entries.move_to_end(key)
        return hit

    def put(self, key, value):
        self.entries[key] = value
        self.entries.move_to_end(key)
        while len(self.entries) > self.size:
            self.entries.popitem(last=False)


_faces_checked = _TensorCache()


def _faces_i32(faces, device, bound, what):
    """[F,3] int32 on `device`, indices checked like the reference's IndexError on out-of-range
    indices (rasterize.py:232, :246).  CPU index tensors are checked on the host before the copy;
    device-resident int32 ones once per (storage, version), so steady-state calls never sync."""
    f = faces if isinstance(faces, torch.Tensor) else torch.as_tensor(faces)
    if f.ndim != 2 or f.shape[1] != 3:
        raise AssertionError("%s must be [F, 3]" % what)
    if f.is_cuda and f.dtype == torch.int32 and f.device == device and f.is_contiguous():
        # the steady-state case (a device int32 index tensor reused every step): no conversion calls
        key = (f.data_ptr(), f._version, f.shape[0], bound, f.device)
        if f.numel() and _faces_checked.get(key) is None:
            lo, hi = int(f.min()), int(f.max())
            if lo < 0 or hi >= bound:
                raise IndexError("%s index out of range [0, %d): min %d max %d" % (what, bound, lo, hi))
            _faces_checked.put(key, f)
        return f
    if not f.is_cuda:
        if f.numel():
            lo, hi = int(f.min()), int(f.max())
            if lo < 0 or hi >= bound:
                raise IndexError("%s index out of range [0, %d): min %d max %d" % (what, bound, lo, hi))
        return f.to(dtype=torch.int32).contiguous().to(device, non_blocking=False)
    reuse = f.dtype == torch.int32 and f.is_contiguous() and f.device == device
    f = f.to(device=device, dtype=torch.int32).contiguous()
    key = (f.data_ptr(), f._version, f.shape[0], bound, f.device)
    if f.numel() and not (reuse and _faces_checked.get(key) is not None):
        lo, hi = int(f.min()), int(f.max())
        if lo < 0 or hi >= bound:
            raise IndexError("%s index out of range [0, %d): min %d max %d" % (what, bound, lo, hi))
        if reuse:
            _faces_checked.put(key, f)
    return f


_adjacency = _TensorCache()


def _vertex_adjacency(faces_i32, V):
    """CSR vertex -> face corners (3 f + k) for the backward's vertex gather, built on the host
    with a stable sort (deterministic summation order) and cached per (storage, version)."""
    key = (faces_i32.data_ptr(), faces_i32._version, faces_i32.shape[0], V, faces_i32.device)
    hit = _adjacency.get(key)
    if hit is not None:
        return hit[0], hit[1]
    import numpy as np
    flat = faces_i32.reshape(-1).cpu().numpy().astype(np.int64)
    order = np.argsort(flat, kind="stable").astype(np.int32)
    counts = np.bincount(flat, minlength=V)
    offsets = np.zeros(V + 1, np.int32)
    np.cumsum(counts, out=offsets[1:])
    off = torch.as_tensor(offsets, device=faces_i32.device)
    ent = torch.as_tensor(order, device=faces_i32.device)
    _adjacency.put(key, (off, ent, faces_i32))  # keep faces_i32 alive: its storage is the key
    return off, ent


_normal_adj = _TensorCache()
_hot_cache = _TensorCache()
# a texture window shared by at least this many faces gets private copies in the backward
# (NrRasterArgs.face_hot): every face of an OBJ's flat-colour material samples one 2x2 atlas patch
# (load_obj.py:84-94), so all the waves that render the material add into the same texels
_HOT_MIN_FACES = int(os.environ.get("NR_HOT_MIN_FACES", "32"))


def _face_hot(ft, vt_src, dev):
    """(face_hot [F] int32 on dev, num_hot) for a batch-shared texture-coordinate table vt_src
    [Vt, 2] and faces_textures ft [F, 3]: faces whose three texture coordinates are identical
    (bit for bit, so the backward computes the same texel window for all of them) form a group; the
    NR_HOT_MAX largest groups of at least _HOT_MIN_FACES faces get ids 0.., every other face -1.
    (None, 0) when no group qualifies.  Cached per (storage, version) of both tensors."""
    key = (ft.data_ptr(), ft._version, vt_src.data_ptr(), vt_src._version, tuple(ft.shape), tuple(vt_src.shape),
           _HOT_MIN_FACES, dev)
    hit = _hot_cache.get(key)
    if hit is not None:
        return hit[0], hit[1]
    if vt_src.is_cuda and torch.cuda.is_current_stream_capturing():
        return None, 0  # the grouping needs a host copy; the plain flush is exact without it
    import numpy as np
    if _HOT_MIN_FACES <= 0 or ft.shape[0] == 0:
        res = (None, 0)
    else:
        uv = vt_src.detach().float().cpu().numpy()[ft.long().cpu().numpy()]  # [F, 3, 2]
        rows = np.ascontiguousarray(uv.reshape(-1, 6)).view(np.int32)        # exact bits
        _, inv, cnt = np.unique(rows, axis=0, return_inverse=True, return_counts=True)
        inv = inv.reshape(-1)
        big = np.nonzero(cnt >= _HOT_MIN_FACES)[0]
        big = big[np.argsort(-cnt[big], kind="stable")][:_lib.NR_HOT_MAX]
        if len(big) == 0:
            res = (None, 0)
        else:
            ids = np.full(len(cnt), -1, np.int32)
            ids[big] = np.arange(len(big), dtype=np.int32)
            res = (torch.as_tensor(ids[inv], device=dev), len(big))
    _hot_cache.put(key, (res[0], res[1], ft, vt_src))  # keep the key tensors alive
    return res[0], res[1]


def _normal_adjacency(faces_i32, V):
    """CSR vertex -> its distinct faces, ascending (the one-hot [F, V] matrix of
    rasterize.py:173-179: a face counts once per vertex), cached per faces tensor."""
    key = (faces_i32.data_ptr(), faces_i32._version, faces_i32.shape[0], V, faces_i32.device)
    hit = _normal_adj.get(key)
    if hit is not None:
        return hit[0], hit[1]
    import numpy as np
    f = faces_i32.cpu().numpy().astype(np.int64)
    F = f.shape[0]
    pairs = np.unique(np.stack([f.reshape(-1), np.repeat(np.arange(F), 3)], 1), axis=0)  # sorted by (v, f)
    counts = np.bincount(pairs[:, 0], minlength=V)
    offsets = np.zeros(V + 1, np.int32)
    np.cumsum(counts, out=offsets[1:])
    off = torch.as_tensor(offsets, device=faces_i32.device)
    ent = torch.as_tensor(pairs[:, 1].astype(np.int32), device=faces_i32.device)
    _normal_adj.put(key, (off, ent, faces_i32))
    return off, ent


def _light_records(lights, B, dev):
    """lights (reference Light objects, lights.py:4-39, in list order) -> [L, B, NR_LIGHT_FLOATS]
    records for NrRasterArgs.lights: kind, backside, colour rgb, direction xyz / specular alpha.
    Built with differentiable torch ops, so the gradient Rasterize returns for the records (same
    layout, nr_rasterize_backward_params) reaches the light tensors that require it."""
    kinds = {"AmbientLight": _lib.NR_LIGHT_AMBIENT, "DirectionalLight": _lib.NR_LIGHT_DIRECTIONAL,
             "SpecularLight": _lib.NR_LIGHT_SPECULAR}

    def vec(t, n):
        return torch.as_tensor(t, dtype=torch.float32).to(dev).reshape(-1, n).expand(B, n)

    recs = []
    for L in lights:
        kind = next((k for c, k in kinds.items() if any(t.__name__ == c for t in type(L).__mro__)), None)
        if kind is None:
            raise TypeError("unknown light type %s" % type(L).__name__)
        head = torch.tensor([float(kind), float(bool(getattr(L, "backside", False)))], device=dev).expand(B, 2)
        if kind == _lib.NR_LIGHT_DIRECTIONAL:
            tail = vec(L.direction, 3)
        elif kind == _lib.NR_LIGHT_SPECULAR:
            tail = torch.cat([vec(L.alpha, 1), torch.zeros((B, 2), device=dev)], 1)
        else:
            tail = torch.zeros((B, 3), device=dev)
        recs.append(torch.cat([head, vec(L.color, 3), tail], 1))
    return torch.stack(recs).contiguous()


class _Cfg:
    __slots__ = ("image_size", "aa", "backside", "flags", "near", "far", "eps", "C", "V", "F", "tex_shared",
                 "tex_hw", "vt_shared", "Vt", "B", "tex_view", "want_fim")


def _args(cfg, vertices, faces, vt, ft, tex, fim, vt_bstride):
    """NrRasterArgs of one call: sizes, flags and the caller's tensors (the library's own buffers are
    set from the arena layout, _Layout.fill)."""
    a = _lib.NrRasterArgs()
    a.batch_size = cfg.B
    a.num_vertices = cfg.V
    a.num_faces = cfg.F
    a.image_size = cfg.image_size
    a.anti_aliasing = int(cfg.aa)
    a.draw_backside = int(cfg.backside)
    a.draw_flags = cfg.flags
    a.near = cfg.near
    a.far = cfg.far
    a.eps = cfg.eps
    a.depth_min_delta = 1e-4
    a.vertices = vertices.data_ptr()
    a.faces = faces.data_ptr()
    a.face_index = fim.data_ptr()
    if cfg.flags & _lib.NR_DRAW_RGB:
        a.vertices_textures = vt.data_ptr()
        a.vt_batch_stride = vt_bstride
        a.num_vertices_textures = cfg.Vt
        a.faces_textures = ft.data_ptr()
        tv = cfg.tex_view  # (data_ptr offset in elements, strides) of the [B, 3, H, W] view read
        a.textures = tex.data_ptr() + 4 * tv[0]
        a.tex_stride_b, a.tex_stride_c, a.tex_stride_p = tv[1], tv[2], tv[3]
        a.tex_height, a.tex_width = cfg.tex_hw
    return a


# the forward stores the backward's tile-border image values (NrRasterArgs.halo); False makes the
# backward re-shade its halos instead (same results; the parity tests cover both)
_HALO_CACHE = os.environ.get("NR_HALO_CACHE", "1") != "0"
# test hook: a value the halo cache is filled with before the forward (NaN in the parity tests, which
# so check that the backward reads only values the forward wrote, or infers from the bin flags)
_HALO_FILL = None
# test hook: a face id the face-index map is filled with before the forward (a valid id in the parity
# tests, so that a backward reading an entry the sparse forward left unwritten would show up in the
# gradients)
_FIM_FILL = None
# the forward packs the texels into RGBA rows that forward and backward sample (NrRasterArgs.
# textures_packed); False samples the [B, 3, H, W] textures directly (same results)
_TEX_PACK = os.environ.get("NR_TEX_PACK", "1") != "0"
# True: the forward allocates the backward's workspace and its setup launch zeroes the accumulators
# (NrRasterArgs.bwd_workspace); False: the backward allocates and zero-fills it (same results)
_BWD_PREZERO = os.environ.get("NR_BWD_PREZERO", "1") != "0"
# only small workspaces: there the separate zero fill is a latency-bound launch (headline: 12 MB,
# step 0.516 -> 0.505 ms); a large one is bandwidth-bound either way and only lengthens the setup
# (the car with its atlas gradient: 63 MB, setup 0.052 -> 0.063 ms, step no better).  The cost: a
# grad-enabled forward whose backward never runs (a render kept for logging, validation without
# no_grad) still allocates and zero-fills the workspace, and holds it as long as its graph lives.
_BWD_PREZERO_MAX = 32 << 20
_WS_ARENA_MAX = 16 << 20
_TEX_PACK_MAX_BYTES = 1 << 31


def _align(n):
    return (n + 255) & ~255


class _Layout:
    """The library's per-call buffers as byte offsets into ONE device allocation (the arena): face
    records, face uv records, the forward's bin workspace, the halo cache, the packed texels, the
    backward's pre-zeroed workspace and the light scratch.  The library takes raw pointers, so none of
    them needs a tensor of its own: one caching-allocator call per forward instead of up to eight.
    Computed once per configuration (sizes only) and cached."""
    __slots__ = ("nbytes", "frec", "fuv", "ws", "ws_bytes", "halo", "halo_bytes", "tex4", "bws", "bws_bytes",
                 "fnorm", "vnorm", "bwd_need", "hot", "num_hot")

    def __init__(self, L, cfg, uv_items, want_halo, want_bws, tex_grad, nl, num_hot=0):
        off = 0

        def take(n):
            nonlocal off
            o = off
            off += _align(n)
            return o
        B, F, V = cfg.B, cfg.F, cfg.V
        S = cfg.image_size * (2 if cfg.aa else 1)
        rgb = bool(cfg.flags & _lib.NR_DRAW_RGB)
        self.frec = take(B * F * 16 * 4)
        self.fuv = take(uv_items * F * 8 * 4) if rgb else None
        self.ws_bytes = L.nr_workspace_bytes(B, F, S)
        # the forward's bin workspace is read by the forward only: in the arena (which the graph keeps
        # alive until its backward) when small, else a temporary freed when the forward returns
        self.ws = take(self.ws_bytes) if self.ws_bytes <= _WS_ARENA_MAX else None
        self.halo = self.halo_bytes = None
        if want_halo:
            self.halo_bytes = L.nr_halo_bytes(B, cfg.image_size, int(cfg.aa), cfg.flags)
            self.halo = take(self.halo_bytes)
        self.tex4 = None
        if rgb and _TEX_PACK:
            H, W = cfg.tex_hw
            n = L.nr_texture_packed_bytes(1 if cfg.tex_shared else B, H, W)
            if n <= _TEX_PACK_MAX_BYTES:  # per-item atlases of hundreds of MB are sampled in place
                self.tex4 = take(n)
        self.bws = self.bws_bytes = None
        H, W = cfg.tex_hw
        tex_items = (1 if cfg.tex_shared else B) if (rgb and tex_grad) else 0
        # the backward's workspace for this configuration (its texture gradient follows tex_grad)
        self.bwd_need = L.nr_backward_workspace_bytes(B, F, V, tex_items, H, W, nl)
        # the shared windows' private copies (NrRasterArgs.hot_acc) right after the backward's
        # workspace, inside the span the forward zeroes
        self.num_hot = num_hot
        hot_bytes = L.nr_hot_acc_bytes(num_hot) if num_hot > 0 else 0
        self.hot = None
        if want_bws and self.bwd_need <= _BWD_PREZERO_MAX:
            self.bws = take(self.bwd_need)
            if hot_bytes:
                self.hot = take(hot_bytes)
            self.bws_bytes = off - self.bws
        elif hot_bytes:
            self.hot = take(hot_bytes)  # zeroed by the backward
        self.fnorm = self.vnorm = None
        if nl:
            self.fnorm, self.vnorm = take(B * F * 3 * 4), take(B * V * 4 * 4)
        self.nbytes = max(off, 256)

    def fill(self, a, base):
        """Point the NrRasterArgs buffers at the arena at device address `base`."""
        a.face_records = base + self.frec
        if self.fuv is not None:
            a.face_uv = base + self.fuv
        if self.ws is not None:
            a.workspace, a.workspace_bytes = base + self.ws, self.ws_bytes
        if self.halo is not None:
            a.halo = base + self.halo
        if self.tex4 is not None:
            a.textures_packed = base + self.tex4
        if self.bws is not None:
            a.bwd_workspace, a.bwd_workspace_bytes = base + self.bws, self.bws_bytes
        if self.hot is not None:
            a.hot_acc, a.num_hot = base + self.hot, self.num_hot
        if self.fnorm is not None:
            a.face_normals, a.vertex_normals = base + self.fnorm, base + self.vnorm


_layouts = {}


def _layout(L, cfg, uv_items, want_halo, want_bws, tex_grad, nl, num_hot=0):
    key = (cfg.B, cfg.F, cfg.V, cfg.image_size, cfg.aa, cfg.flags, cfg.tex_hw, cfg.tex_shared, uv_items,
           want_halo, want_bws, tex_grad, nl, _TEX_PACK, num_hot)
    lay = _layouts.get(key)
    if lay is None:
        if len(_layouts) > 64:
            _layouts.clear()
        lay = _layouts[key] = _Layout(L, cfg, uv_items, want_halo, want_bws, tex_grad, nl, num_hot)
    return lay


class Rasterize(torch.autograd.Function):
    """rasterize_core (rasterize.py:194-329) as one Function: vertices [B,V,3] (+ textures) ->
    images [B, C, s, s]; backward returns d/dvertices and d/dtextures."""

    @staticmethod
    def forward(ctx, vertices, textures, vertices_textures, faces, faces_textures, backgrounds, light_recs, cfg):
        dev = vertices.device
        ctx.vt_shape = vertices_textures.shape
        # a [1, Vt, 2] vt is shared by the batch: item stride 0 (NrRasterArgs.vt_batch_stride)
        vt_shared = vertices_textures.ndim == 3 and (vertices_textures.shape[0] == 1 or vertices_textures.stride(0) == 0)
        vt_bstride = 0 if vt_shared else (vertices_textures.stride(0) if vertices_textures.ndim == 3 else 0)
        B = cfg.B
        S = cfg.image_size * (2 if cfg.aa else 1)
        L = _lib.lib()
        if B == 0:
            # an empty shard (distributed.shard with B < world size): nothing to draw, and the
            # backward returns zero gradients for the batch-shared inputs
            ctx.cfg = cfg
            ctx.dev = dev
            ctx.shapes = (textures.shape, ctx.vt_shape, None if light_recs is None else light_recs.shape,
                          None if backgrounds is None else backgrounds.shape)
            fim = torch.empty((0, S, S), dtype=torch.int32, device=dev)
            ctx.mark_non_differentiable(fim)
            ctx.set_materialize_grads(False)
            return torch.empty((0, cfg.C, cfg.image_size, cfg.image_size), dtype=torch.float32, device=dev), fim
        rgb = bool(cfg.flags & _lib.NR_DRAW_RGB)
        grads = ctx.needs_input_grad[0] or ctx.needs_input_grad[1]
        uv_items = (1 if vt_bstride == 0 else B) if rgb else 0
        nl = light_recs.shape[0] if light_recs is not None else 0
        # shared texture windows (a texture and texture coordinates shared by the batch, texture gradient
        # wanted).  Only for a fixed texture-coordinate table: the grouping is computed on the host from
        # the table's values and cached per (storage, version), so a trainable vt (updated in place every
        # step, or inside a captured graph whose replays never re-run the host code) would keep a stale
        # grouping and send diverged windows' sums to one slot.  A cache miss during stream capture (its
        # host copy would raise) also goes without.
        face_hot, num_hot = None, 0
        if rgb and ctx.needs_input_grad[1] and not ctx.needs_input_grad[2] and cfg.tex_shared and vt_bstride == 0:
            face_hot, num_hot = _face_hot(faces_textures, vertices_textures[0] if vertices_textures.ndim == 3
                                          else vertices_textures, dev)
        lay = _layout(L, cfg, uv_items, _HALO_CACHE and grads, _BWD_PREZERO and grads,
                      ctx.needs_input_grad[1], nl, num_hot)
        arena = torch.empty(lay.nbytes, dtype=torch.uint8, device=dev)
        fim = torch.empty((B, S, S), dtype=torch.int32, device=dev)
        images = torch.empty((B, cfg.C, cfg.image_size, cfg.image_size), dtype=torch.float32, device=dev)
        a = _args(cfg, vertices, faces, vertices_textures, faces_textures, textures, fim, vt_bstride)
        lay.fill(a, arena.data_ptr())
        ws_tmp = None
        if lay.ws is None:  # a large bin workspace: a temporary (stream-ordered reuse once it is freed)
            ws_tmp = torch.empty(lay.ws_bytes, dtype=torch.uint8, device=dev)
            a.workspace, a.workspace_bytes = ws_tmp.data_ptr(), lay.ws_bytes
        if face_hot is not None:
            a.face_hot = face_hot.data_ptr()
            ctx.face_hot = face_hot  # alive until the backward
        if _FIM_FILL is not None:
            fim.fill_(_FIM_FILL)
        if _HALO_FILL is not None and lay.halo is not None:
            arena[lay.halo:lay.halo + lay.halo_bytes].view(torch.float32).fill_(_HALO_FILL)
        light = None
        if light_recs is not None:
            nadj = _normal_adjacency(faces, cfg.V)
            a.num_lights = nl
            a.lights = light_recs.data_ptr()
            a.normal_offsets, a.normal_faces = nadj[0].data_ptr(), nadj[1].data_ptr()
            light = (light_recs, nadj)  # keeps the CSR alive as long as the graph
        if backgrounds is not None and rgb:  # [B, 3, S, S] x-contiguous
            a.backgrounds = backgrounds.data_ptr()
            a.bg_stride_b, a.bg_stride_c, a.bg_stride_y = backgrounds.stride(0), backgrounds.stride(1), \
                backgrounds.stride(2)
        # the face-index map stays internal (not returned) and only the backward reads it, through the
        # halo cache's bin flags: empty bins need not write their -1 entries (NrRasterArgs.
        # face_index_sparse).  Not when the parameter-gradient pass (vertices_textures) reads them all.
        a.face_index_sparse = int(lay.halo is not None and not cfg.want_fim and backgrounds is None and
                                  light_recs is None and not (rgb and ctx.needs_input_grad[2]))
        with _lib.on_device(dev):
            _lib.check(L.nr_rasterize_forward(a, images.data_ptr(), _lib.stream_of(vertices)), "nr_rasterize_forward")
        if ws_tmp is not None:
            a.workspace, a.workspace_bytes = None, 0
            del ws_tmp
        # the backward's workspace was zeroed by the setup launch (NrRasterArgs.bwd_workspace): for the
        # first backward only (its accumulators are spent after it)
        ctx.prezeroed = lay.bws is not None
        ctx.arena = arena
        ctx.layout = lay
        ctx.args = a
        ctx.cfg = cfg
        ctx.light = light
        ctx.save_for_backward(vertices, textures, vertices_textures, faces, faces_textures, fim, backgrounds)
        ctx.mark_non_differentiable(fim)
        # no zero-filled gradient for the int32 face-index output (a 67 MB fill per backward at the
        # headline size otherwise)
        ctx.set_materialize_grads(False)
        return images, fim

    @staticmethod
    def backward(ctx, grad_images, _grad_fim):
        cfg = ctx.cfg
        if cfg.B == 0:
            tshape, vtshape, lshape, bshape = ctx.shapes
            dev = ctx.dev
            z = (lambda shp, i: torch.zeros(shp, dtype=torch.float32, device=dev) if ctx.needs_input_grad[i] else None)
            return (z((0, cfg.V, 3), 0), z(tshape, 1), z(vtshape, 2), None, None,
                    z(bshape, 5) if bshape is not None else None, z(lshape, 6) if lshape is not None else None, None)
        if grad_images is None:
            return None, None, None, None, None, None, None, None
        vertices, textures, vt, faces, ft, fim, backgrounds = ctx.saved_tensors
        grad_images = grad_images.contiguous()
        L = _lib.lib()
        dev = vertices.device
        a = ctx.args  # the forward's arguments: same inputs and arena (the forward has consumed them)
        a.workspace, a.workspace_bytes = None, 0  # the backward does not use the forward's bin workspace
        gv = torch.empty_like(vertices)
        gt = None
        rgb = bool(cfg.flags & _lib.NR_DRAW_RGB)
        want_tex = rgb and ctx.needs_input_grad[1]
        tex_items = 0
        H, W = cfg.tex_hw
        if want_tex:
            tex_items = 1 if cfg.tex_shared else cfg.B
            gt = torch.empty((tex_items, 3, H, W), dtype=torch.float32, device=dev)
        lay = ctx.layout
        need = lay.bwd_need
        prezeroed = ctx.prezeroed and lay.bws is not None
        ctx.prezeroed = False
        if prezeroed:
            ws_ptr = a.bwd_workspace  # the library checks it is the buffer the forward zeroed
            ws = None
        else:
            ws = torch.empty(need, dtype=torch.uint8, device=dev)
            ws_ptr = ws.data_ptr()
        adj = _vertex_adjacency(faces, cfg.V)
        a.vertex_offsets, a.vertex_faces = adj[0].data_ptr(), adj[1].data_ptr()
        gbg = None
        if backgrounds is not None and rgb:
            if ctx.needs_input_grad[5]:
                gbg = torch.empty((cfg.B, 3) + tuple(backgrounds.shape[2:]), dtype=torch.float32, device=dev)
            a.grad_backgrounds = gbg.data_ptr() if gbg is not None else None
        stream = _lib.stream_of(vertices)
        with _lib.on_device(dev):
            # workspace_zeroed = 1 only for the first backward after the forward zeroed it (no fill)
            _lib.check(L.nr_rasterize_backward(a, grad_images.data_ptr(), gv.data_ptr(),
                                               gt.data_ptr() if gt is not None else None, ws_ptr, need,
                                               int(prezeroed), stream), "nr_rasterize_backward")
        if gt is not None:
            # the Function's texture input is [B, 3, H, W], or the single [3, H, W] / [1, 3, H, W]
            # source of a shared texture (see rasterize_core): same element count as gt either way
            gt = gt.reshape(textures.shape)
        # vertices_textures and light parameters (rasterize.py:246, 252-283): a second, separate pass
        gvt = glt = None
        want_vt = rgb and ctx.needs_input_grad[2]
        want_lt = rgb and ctx.needs_input_grad[6] and ctx.light is not None
        if want_vt or want_lt:
            if want_vt:
                # the Function's vt input is [B, Vt, 2] per item, or the [1, Vt, 2] source of a shared one
                gvt = torch.empty(tuple(ctx.vt_shape), dtype=torch.float32, device=dev)
            if want_lt:
                glt = torch.empty_like(ctx.light[0])
            with _lib.on_device(dev):
                _lib.check(L.nr_rasterize_backward_params(a, grad_images.data_ptr(), _lib.ptr(gvt), _lib.ptr(glt),
                                                          stream), "nr_rasterize_backward_params")
        return (gv if ctx.needs_input_grad[0] else None), gt, gvt, None, None, gbg, glt, None


def _flags(hp):
    return ((_lib.NR_DRAW_RGB if hp.draw_rgb else 0) | (_lib.NR_DRAW_SILHOUETTES if hp.draw_silhouettes else 0) |
            (_lib.NR_DRAW_DEPTH if hp.draw_depth else 0))


def rasterize_core(vertices, faces, params: RasterizeParam, hyperparams: RasterizeHyperparam, return_face_index=False):
    """Render [B, C, s, s] images (channels rgb, silhouettes, depth in that order, those enabled
    by hyperparams.draw_*).  Same contract as rasterize.py:194-329."""
    assert vertices.ndim == 3
    assert vertices.shape[2] == 3
    faces_t = torch.as_tensor(faces)
    assert faces_t.ndim == 2
    assert faces_t.shape[1] == 3
    if hyperparams.draw_rgb:
        assert params.vertices_textures.ndim == 3
        assert params.vertices_textures.shape[2] == 2
        assert torch.as_tensor(params.faces_textures).ndim == 2
        assert params.faces_textures.shape[1] == 3
        assert params.textures.ndim == 4
        assert params.textures.shape[1] == 3
    if params.backgrounds is not None:  # shape contract of rasterize.py:216-225
        assert params.backgrounds.ndim == 4
        assert params.backgrounds.shape[0] == vertices.shape[0]
        assert params.backgrounds.shape[1] == 3
        side = hyperparams.image_size * (2 if hyperparams.anti_aliasing else 1)
        assert params.backgrounds.shape[2] == side and params.backgrounds.shape[3] == side
    if params.background_color is not None:
        # rasterize.py:208-214 (and chainer rasterize.py:649-655): zeros * colour, i.e. black
        side = hyperparams.image_size * (2 if hyperparams.anti_aliasing else 1)
        params.backgrounds = torch.zeros((vertices.shape[0], 3, side, side), dtype=torch.float32,
                                         device=vertices.device) * \
            torch.as_tensor(params.background_color, dtype=torch.float32, device=vertices.device)[None, :, None, None]
    flags = _flags(hyperparams)
    if flags == 0:
        raise Exception  # rasterize.py:309-310
    _lib.require_gpu(vertices)
    dev = vertices.device
    v = vertices if (vertices.dtype == torch.float32 and vertices.is_contiguous()) else vertices.float().contiguous()
    cfg = _Cfg()
    cfg.B, cfg.V = v.shape[0], v.shape[1]
    cfg.F = faces_t.shape[0]
    cfg.image_size = int(hyperparams.image_size)
    cfg.aa = bool(hyperparams.anti_aliasing)
    cfg.backside = bool(hyperparams.draw_backside)
    cfg.flags = flags
    cfg.near, cfg.far, cfg.eps = float(hyperparams.near), float(hyperparams.far), float(hyperparams.eps)
    cfg.C = (3 if flags & _lib.NR_DRAW_RGB else 0) + (1 if flags & _lib.NR_DRAW_SILHOUETTES else 0) + \
        (1 if flags & _lib.NR_DRAW_DEPTH else 0)  # nr_num_channels
    cfg.want_fim = bool(return_face_index)
    fi = _faces_i32(faces_t, dev, cfg.V, "faces")
    tex = vt = ft = None
    cfg.tex_shared = cfg.vt_shared = False
    cfg.tex_hw = (0, 0)
    cfg.tex_view = (0, 0, 0, 0)
    cfg.Vt = 0
    if hyperparams.draw_rgb:
        vt = params.vertices_textures
        tex = params.textures
        _lib.require_gpu(vt, tex)
        if vt.dtype != torch.float32:
            vt = vt.float()
        if vt.shape[0] not in (1, cfg.B):
            raise AssertionError("vertices_textures batch must be 1 or %d" % cfg.B)
        # the Function gets the [1, Vt, 2] source of a batch-shared vt (a slice of the expanded view,
        # so autograd returns its gradient once, summed over the items) or the per-item [B, Vt, 2]
        if vt.shape[0] == 1 or vt.stride(0) == 0:
            vt = vt[:1]
        if vt.stride(2) != 1 or vt.stride(1) != 2:
            vt = vt.contiguous()
        cfg.Vt = vt.shape[1]
        cfg.vt_shared = vt.shape[0] == 1 and cfg.B > 1
        ft = _faces_i32(params.faces_textures, dev, cfg.Vt, "faces_textures")
        if ft.shape[0] != cfg.F:
            raise AssertionError("faces_textures must have one row per face")
        if tex.dtype != torch.float32:
            tex = tex.float()
        if tex.shape[0] not in (1, cfg.B):
            raise AssertionError("textures batch must be 1 or %d" % cfg.B)
        H, W = tex.shape[2], tex.shape[3]
        if tex.shape[0] > 1 and tex.stride(0) != 0 and tex.stride(2) != W * tex.stride(3):
            tex = tex.contiguous()
        if tex.shape[0] > 1 and tex.stride(0) == 0 and tex.requires_grad and tex.grad_fn is None:
            # a batch-expanded view that is itself the gradient leaf (expand(...).requires_grad_()):
            # autograd gives such a leaf one gradient per item (t.grad[b] = item b's share), as the
            # reference fills it, so it is rendered as B per-item textures (a copy, this case only)
            tex = tex.contiguous()
        cfg.tex_hw = (H, W)
        cfg.tex_shared = tex.shape[0] == 1 or tex.stride(0) == 0
        if cfg.tex_shared:
            # one texture for every item.  A batch-expanded view (tex[None].expand(B, ...), the
            # reference tests' idiom) is handed to the Function as its [3, H, W] source so that the
            # texture gradient is returned once, not B times through expand's backward.
            if tex.shape[0] == 0:
                # an empty batch (B = 0) of an expanded view: its source takes the zero gradient
                base = tex._base if tex._is_view() else None
                tex = (base.reshape(1, 3, H, W) if base is not None and base.numel() == 3 * H * W
                       else torch.zeros((1, 3, H, W), dtype=torch.float32, device=dev))
            # item 0 of the view: [3, H, W] at the view's own data pointer, contiguous when its strides
            # are (H W, W, 1) (size-1 dimensions excepted) -- tested on the strides, without the view
            st = tex.stride()
            item_contig = st[1] == H * W and (H == 1 or st[2] == W) and (W == 1 or st[3] == 1)
            # the view's base takes the gradient in place of the view only when the gradient reaches
            # the caller's leaf through it: the view is not itself a leaf that requires grad
            # (that case was made per-item above), so its grad_fn, if any, is expand's of `base`
            base = tex._base if tex._is_view() else None
            if base is not None and tex.requires_grad and not base.requires_grad:
                base = None
            if (base is not None and base.numel() == 3 * H * W and base.is_contiguous()
                    and item_contig and tex.data_ptr() == base.data_ptr()):
                tex = base
            elif not item_contig:
                tex = tex[0].contiguous()[None]
            elif tex.shape[0] != 1:
                tex = tex[0][None]
            cfg.tex_view = (0, 0, H * W, 1)
        else:
            cfg.tex_view = (0, tex.stride(0), tex.stride(1), tex.stride(3))
    else:
        tex = torch.empty(0, device=dev)
    if vt is None:
        vt = torch.empty(0, device=dev)
        ft = torch.empty(0, dtype=torch.int32, device=dev)
    bg = light_recs = None
    if hyperparams.draw_rgb:
        # backgrounds / lights only change the rgb channels (rasterize.py:252-288); otherwise the
        # reference validates and ignores them
        if params.backgrounds is not None:
            bg = params.backgrounds
            _lib.require_gpu(bg)
            bg = bg.float()
            if bg.stride(3) != 1:
                bg = bg.contiguous()
        if params.lights is not None and len(params.lights) > 0:
            light_recs = _light_records(params.lights, cfg.B, dev)
    images, fim = Rasterize.apply(v, tex, vt, fi, ft, bg, light_recs, cfg)
    if return_face_index:
        return images, fim
    return images


def rasterize_silhouettes(vertices, faces, params: RasterizeParam, hyperparams: RasterizeHyperparam):
    hyperparams.draw_rgb = False
    hyperparams.draw_silhouettes = True
    hyperparams.draw_depth = False
    return rasterize_core(vertices, faces, params, hyperparams)[:, 0]


def rasterize_rgba(vertices, faces, params: RasterizeParam, hyperparams: RasterizeHyperparam):
    hyperparams.draw_rgb = True
    hyperparams.draw_silhouettes = True
    hyperparams.draw_depth = False
    return rasterize_core(vertices=vertices, faces=faces, params=params, hyperparams=hyperparams)


def rasterize_rgb(vertices, faces, params: RasterizeParam, hyperparams: RasterizeHyperparam):
    hyperparams.draw_rgb = True
    hyperparams.draw_silhouettes = False
    hyperparams.draw_depth = False
    return rasterize_core(vertices=vertices, faces=faces, params=params, hyperparams=hyperparams)


def rasterize_depth(vertices, faces, params: RasterizeParam, hyperparams: RasterizeHyperparam):
    hyperparams.draw_rgb = False
    hyperparams.draw_silhouettes = False
    hyperparams.draw_depth = True
    return rasterize_core(vertices=vertices, faces=faces, params=params, hyperparams=hyperparams)[:, 0]
