"""ctypes binding of the HIP library (include/nr_raster.h -> _lib/libnr_raster.so).

The library is loaded on first use.  There is no CPU fallback: if the shared object is missing or
a call fails, a RuntimeError is raised.  Build it with `python -c "import __graft_entry__ as g;
g.build()"` from the repository root (hipcc --offload-arch=gfx950).
"""
import ctypes
import os

import torch

LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib")
# NR_LIB_PATH: developer override used by the timing-variant scripts in tools/
LIB_PATH = os.environ.get("NR_LIB_PATH") or os.path.join(LIB_DIR, "libnr_raster.so")

NR_DRAW_RGB = 1
NR_DRAW_SILHOUETTES = 2
NR_DRAW_DEPTH = 4

# every symbol declared in include/nr_raster.h
EXPORTS = [
    "nr_last_error", "nr_version", "nr_workspace_bytes", "nr_face_index_map_forward_safe",
    "nr_compute_weight_map", "nr_mask_foreground_forward", "nr_mask_foreground_backward",
    "nr_differentiation_backward", "nr_num_channels", "nr_rasterize_forward", "nr_rasterize_backward",
    "nr_backward_workspace_bytes", "nr_profile_enable", "nr_profile_read",
    "nr_selftest_division", "nr_halo_bytes", "nr_raster_args_size", "nr_rasterize_backward_params",
    "nr_camera_forward", "nr_camera_backward", "nr_camera_workspace_bytes", "nr_texture_packed_bytes",
    "nr_last_launch", "nr_hot_acc_bytes",
]

ABI_VERSION = 6  # include/nr_raster.h NR_ABI_VERSION

NR_LAUNCH_FUSED_SHADE, NR_LAUNCH_STATIC_CHANNELS, NR_LAUNCH_TWO_PX_PER_LANE, NR_LAUNCH_DEEP_FIRST, NR_LAUNCH_SPLIT = 1, 2, 4, 8, 16
NR_LAUNCH_HOT_WINDOWS, NR_LAUNCH_DEALT_QUARTERS, NR_LAUNCH_QUADRANTS = 32, 64, 128
NR_HOT_MAX, NR_HOT_COPIES = 256, 32

c_int, c_float, c_void_p, c_size_t, c_ll = ctypes.c_int, ctypes.c_float, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_longlong


class NrRasterArgs(ctypes.Structure):
    _fields_ = [
        ("batch_size", c_int), ("num_vertices", c_int), ("num_faces", c_int), ("image_size", c_int),
        ("anti_aliasing", c_int), ("draw_backside", c_int), ("draw_flags", c_int),
        ("near", c_float), ("far", c_float), ("eps", c_float), ("depth_min_delta", c_float),
        ("vertices", c_void_p), ("faces", c_void_p),
        ("vertices_textures", c_void_p), ("vt_batch_stride", c_ll), ("num_vertices_textures", c_int),
        ("faces_textures", c_void_p), ("textures", c_void_p),
        ("tex_stride_b", c_ll), ("tex_stride_c", c_ll), ("tex_stride_p", c_ll),
        ("tex_height", c_int), ("tex_width", c_int),
        ("face_records", c_void_p), ("face_uv", c_void_p), ("face_index", c_void_p),
        ("workspace", c_void_p), ("workspace_bytes", c_size_t),
        ("vertex_offsets", c_void_p), ("vertex_faces", c_void_p), ("halo", c_void_p),
        ("num_lights", c_int), ("lights", c_void_p), ("face_normals", c_void_p), ("vertex_normals", c_void_p),
        ("normal_offsets", c_void_p), ("normal_faces", c_void_p),
        ("backgrounds", c_void_p), ("bg_stride_b", c_ll), ("bg_stride_c", c_ll), ("bg_stride_y", c_ll),
        ("grad_backgrounds", c_void_p), ("textures_packed", c_void_p),
        ("bwd_workspace", c_void_p), ("bwd_workspace_bytes", c_size_t), ("face_index_sparse", c_int),
        ("face_hot", c_void_p), ("num_hot", c_int), ("hot_acc", c_void_p),
    ]

NR_LIGHT_AMBIENT, NR_LIGHT_DIRECTIONAL, NR_LIGHT_SPECULAR, NR_LIGHT_FLOATS = 0, 1, 2, 8
NR_CAMERA_NONE, NR_CAMERA_LOOK_AT = 0, 1


class NrCameraArgs(ctypes.Structure):  # include/nr_raster.h
    _fields_ = [
        ("batch_size", c_int), ("num_vertices", c_int), ("vertices", c_void_p), ("v_batch_stride", c_ll),
        ("eye", c_void_p), ("eye_batch_stride", c_ll), ("mode", c_int), ("at", c_float * 3), ("up", c_float * 3),
        ("perspective", c_int), ("width", c_float),
    ]


_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError("neural_renderer_v2_pytorch_amd: HIP library %s is missing; build it with "
                           "__graft_entry__.build() (there is no CPU fallback)" % LIB_PATH)
    L = ctypes.CDLL(LIB_PATH)
    L.nr_last_error.restype = ctypes.c_char_p
    L.nr_last_error.argtypes = []
    L.nr_version.restype = c_int
    L.nr_workspace_bytes.restype = c_size_t
    L.nr_workspace_bytes.argtypes = [c_int, c_int, c_int]
    L.nr_num_channels.restype = c_int
    L.nr_num_channels.argtypes = [c_int]
    L.nr_face_index_map_forward_safe.argtypes = [c_void_p, c_void_p, c_int, c_int, c_int, c_float, c_float, c_int,
                                                 c_float, c_float, c_void_p, c_size_t, c_void_p]
    L.nr_compute_weight_map.argtypes = [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p]
    L.nr_mask_foreground_forward.argtypes = [c_void_p, c_void_p, c_void_p, c_ll, c_int, c_void_p]
    L.nr_mask_foreground_backward.argtypes = [c_void_p, c_void_p, c_void_p, c_ll, c_int, c_void_p]
    L.nr_differentiation_backward.argtypes = [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p]
    L.nr_rasterize_forward.argtypes = [ctypes.POINTER(NrRasterArgs), c_void_p, c_void_p]
    L.nr_rasterize_backward.argtypes = [ctypes.POINTER(NrRasterArgs), c_void_p, c_void_p, c_void_p, c_void_p,
                                        c_size_t, c_int, c_void_p]
    L.nr_rasterize_backward_params.argtypes = [ctypes.POINTER(NrRasterArgs), c_void_p, c_void_p, c_void_p, c_void_p]
    L.nr_camera_forward.argtypes = [ctypes.POINTER(NrCameraArgs), c_void_p, c_void_p]
    L.nr_camera_backward.argtypes = [ctypes.POINTER(NrCameraArgs), c_void_p, c_void_p, c_void_p, c_void_p, c_size_t,
                                     c_void_p]
    L.nr_texture_packed_bytes.restype = c_size_t
    L.nr_texture_packed_bytes.argtypes = [c_int, c_int, c_int]
    L.nr_camera_workspace_bytes.restype = c_size_t
    L.nr_camera_workspace_bytes.argtypes = [c_int]
    L.nr_backward_workspace_bytes.restype = c_size_t
    L.nr_backward_workspace_bytes.argtypes = [c_int, c_int, c_int, c_int, c_int, c_int, c_int]
    L.nr_raster_args_size.restype = c_size_t
    L.nr_raster_args_size.argtypes = []
    L.nr_hot_acc_bytes.restype = c_size_t
    L.nr_hot_acc_bytes.argtypes = [c_int]
    L.nr_halo_bytes.restype = c_size_t
    L.nr_halo_bytes.argtypes = [c_int, c_int, c_int, c_int]
    L.nr_selftest_division.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, c_ll, c_void_p]
    L.nr_last_launch.argtypes = [ctypes.c_char_p, ctypes.POINTER(c_int), ctypes.POINTER(c_int)]
    L.nr_profile_enable.argtypes = [c_int]
    L.nr_profile_read.argtypes = [ctypes.c_char_p, ctypes.POINTER(c_float)]
    for name in EXPORTS:
        if name not in ("nr_last_error", "nr_workspace_bytes", "nr_num_channels", "nr_backward_workspace_bytes",
                        "nr_halo_bytes", "nr_raster_args_size", "nr_camera_workspace_bytes",
                        "nr_texture_packed_bytes", "nr_hot_acc_bytes"):
            getattr(L, name).restype = c_int
    # a library of another ABI revision (an NR_LIB_PATH override, a stale build) would misread the
    # arguments (e.g. an older nr_rasterize_backward takes its stream where workspace_zeroed is now)
    if L.nr_version() != ABI_VERSION or L.nr_raster_args_size() != ctypes.sizeof(NrRasterArgs):
        raise RuntimeError("neural_renderer_v2_pytorch_amd: %s has ABI version %d with a %d-byte NrRasterArgs; this "
                           "binding needs version %d and %d bytes (rebuild with __graft_entry__.build())"
                           % (LIB_PATH, L.nr_version(), L.nr_raster_args_size(), ABI_VERSION,
                              ctypes.sizeof(NrRasterArgs)))
    _lib = L
    return L


def last_launch(kernel):
    """(threads per block, NR_LAUNCH_* flags) of the latest launch of `kernel` ("k_raster_fwd" or
    "k_raster_bwd") in this process: the variant the library actually ran."""
    t, f = c_int(), c_int()
    check(lib().nr_last_launch(kernel.encode(), ctypes.byref(t), ctypes.byref(f)), "nr_last_launch")
    return t.value, f.value


def check(status, what):
    if status != 0:
        raise RuntimeError("%s failed (status %d): %s" % (what, status, lib().nr_last_error().decode()))


def stream_of(t):
    """The raw hipStream_t of the current stream on t's device (what torch launches on)."""
    return ctypes.c_void_p(torch._C._cuda_getCurrentRawStream(t.device.index))


class on_device:
    """`with torch.cuda.device(dev)` that costs nothing when dev is already the current device
    (the usual case: the per-call exchange of the current device was a few microseconds of host
    time per launch call)."""
    __slots__ = ("idx", "prev")

    def __init__(self, dev):
        self.idx = dev.index

    def __enter__(self):
        cur = torch._C._cuda_getDevice()
        self.prev = None if cur == self.idx else torch.cuda._exchange_device(self.idx)

    def __exit__(self, *exc):
        if self.prev is not None:
            torch.cuda._exchange_device(self.prev)
        return False


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def require_gpu(*tensors):
    for t in tensors:
        if t is not None and (not torch.is_tensor(t) or not t.is_cuda):
            raise RuntimeError("neural_renderer_v2_pytorch_amd runs on the GPU only (no CPU fallback); "
                               "got a %s" % ("CPU tensor" if torch.is_tensor(t) else type(t).__name__))
