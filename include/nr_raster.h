/*
 * nr_raster.h -- C ABI of the MI355X (gfx950) rasterizer library libnr_raster.so.
 *
 * Plain pointers (device memory), sizes and a hipStream_t passed as void*.  No torch types.
 * Every entry point is asynchronous on `stream`, returns 0 on success and a nonzero
 * NR_ERR_* code on failure, with a message in nr_last_error() (thread-local).  The library never
 * allocates device memory: callers pass every output and the scratch workspace.
 *
 * Reference interfaces replaced (paths relative to /root/reference):
 *   pybind11 module neural_renderer_torch.cuda.rasterize_cuda  (cuda/rasterize_cuda.cpp:93-99)
 *     face_index_map_forward_safe  (.cpp:55-65 -> rasterize_cuda_kernel.cu:362-390, kernel :52-153)
 *                                   -> nr_face_index_map_forward_safe
 *     compute_weight_map_c         (.cpp:81-90 -> .cu:420-443, kernel :246-308)
 *                                   -> nr_compute_weight_map
 *     mask_foreground_forward      (.cpp:35-43 -> .cu:312-335)  -> nr_mask_foreground_forward
 *     mask_foreground_backward     (.cpp:45-53 -> .cu:337-359)  -> nr_mask_foreground_backward
 *     face_index_map_forward_unsafe (.cpp:67-79) -- dead code in the reference (its z-buffer
 *                                   update is commented out, .cu:236-240); not provided.
 *   python-level stages that had no native code in the reference, fused here:
 *     rasterize_core forward (rasterize.py:194-329: gather, face index, weight, coordinate, depth,
 *       texture and silhouette maps, channel merge, flip, 2x2 anti-aliasing)
 *                                   -> nr_rasterize_forward
 *     its autograd backward (Differentiation.backward differentiation.py:12-36, MaskForeground,
 *       to_map index backward, face gather backward)      -> nr_rasterize_backward
 *     Differentiation.backward on its own (differentiation.py:12-36)
 *                                   -> nr_differentiation_backward
 */
#ifndef NR_RASTER_H_
#define NR_RASTER_H_

#include <stddef.h>
#include <stdint.h>

#if defined(__GNUC__)
#define NR_API __attribute__((visibility("default")))
#else
#define NR_API
#endif

#ifdef __cplusplus
extern "C" {
#endif

enum {
    NR_OK = 0,
    NR_ERR_ARGS = 1,    /* invalid sizes / null pointers */
    NR_ERR_LAUNCH = 2,  /* a HIP launch failed */
    NR_ERR_WORKSPACE = 3 /* workspace too small */
};

/* Draw flags for nr_rasterize_forward / nr_rasterize_backward (RasterizeHyperparam.draw_*). */
enum { NR_DRAW_RGB = 1, NR_DRAW_SILHOUETTES = 2, NR_DRAW_DEPTH = 4 };

NR_API const char* nr_last_error(void);
NR_API int nr_version(void);
/* sizeof(NrRasterArgs), for bindings to check their mirror of the struct */
NR_API size_t nr_raster_args_size(void);

/* ABI version of this header: 6 (NrRasterArgs.face_hot / num_hot / hot_acc, nr_hot_acc_bytes; 5:
 * NrRasterArgs.face_index_sparse; 4: nr_last_launch; 3: workspace_zeroed of nr_rasterize_backward).
 * Bindings check it, and nr_raster_args_size(), before the first call. */
#define NR_ABI_VERSION 6

/* Scratch bytes needed by the face-index map for B items, F faces, S x S internal pixels
 * (per-face screen bounding boxes + coarse-bin face bitmasks). */
NR_API size_t nr_workspace_bytes(int batch_size, int num_faces, int image_size);

/* rasterize.py:27-38 / rasterize_cuda_kernel.cu:52-153.
 * faces: [B, F, 3, 3] f32 (screen x, y and depth z of each corner), face_index: [B, S, S] int32
 * (fully written; -1 = background).  Same arguments and meaning as the reference binding;
 * `eps` is accepted and unused exactly as in the reference kernel. */
NR_API int nr_face_index_map_forward_safe(const float* faces, int32_t* face_index, int batch_size, int num_faces,
                                   int image_size, float near, float far, int draw_backside, float eps,
                                   float depth_min_delta, void* workspace, size_t workspace_bytes,
                                   void* stream);

/* rasterize.py:67-77 / .cu:246-308.  weight_map: [B, S, S, 3] f32; background pixels are written
 * with 0 (the reference relies on a caller-zeroed buffer; here every element is written). */
NR_API int nr_compute_weight_map(const float* faces, const int32_t* face_index_map, float* weight_map,
                          int batch_size, int num_faces, int image_size, void* stream);

/* .cu:7-49: copy `dim` floats per pixel where face_index >= 0 (n = number of pixels). */
NR_API int nr_mask_foreground_forward(const int32_t* face_index, const float* data_in, float* data_out,
                               long long n, int dim, void* stream);
NR_API int nr_mask_foreground_backward(const int32_t* face_index, float* grad_in, const float* grad_out,
                                long long n, int dim, void* stream);

/* differentiation.py:12-36: grad_xy[B, H, W, 2] (x first) from the saved images[B, H, W, C] and
 * the incoming gradient grad[B, H, W, C]; step = 2 / H as in the reference. */
NR_API int nr_differentiation_backward(const float* images, const float* grad, float* grad_xy, int batch_size,
                                int height, int width, int channels, void* stream);

/* Arguments of the fused rasterize_core.  All pointers are device pointers; f32 unless noted.
 * Strides are in elements; a batch stride of 0 means "shared by every item" (a torch.expand). */
typedef struct NrRasterArgs {
    int batch_size;          /* B */
    int num_vertices;        /* V */
    int num_faces;           /* F */
    int image_size;          /* s: output size (RasterizeHyperparam.image_size) */
    int anti_aliasing;       /* internal S = 2s when set */
    int draw_backside;
    int draw_flags;          /* NR_DRAW_* */
    float near, far, eps;    /* eps: texture-coordinate clamp (RasterizeHyperparam.eps) */
    float depth_min_delta;   /* 1e-4 in the reference (rasterize.py:35) */
    const float* vertices;   /* [B, V, 3] contiguous, screen space (after look_at + perspective) */
    const int32_t* faces;    /* [F, 3] vertex indices, shared by every item */
    /* textures (only with NR_DRAW_RGB) */
    const float* vertices_textures; /* [Bvt, Vt, 2]; item stride vt_batch_stride (0 = shared) */
    long long vt_batch_stride;
    int num_vertices_textures;
    const int32_t* faces_textures;  /* [F, 3] */
    const float* textures;          /* [Bt, 3, H, W] with the strides below; (h, w) row-contiguous.
                                       Texture coordinates must stay inside the texture (within one
                                       texel past its edge, whose bilinear weight is 0), as the
                                       reference's to_map indexing requires (it raises IndexError);
                                       H and W below 2^23 (24-bit texel index arithmetic). */
    long long tex_stride_b, tex_stride_c, tex_stride_p; /* p = flat texel index h * W + w */
    int tex_height, tex_width;
    /* saved state, written by forward, read by backward */
    float* face_records;     /* [B, F, 16]: gathered faces (rasterize.py:232) + per-face reciprocals/flags */
    float* face_uv;          /* [Buv, F, 8] with Buv = (vt_batch_stride ? B : 1); only with RGB */
    int32_t* face_index;     /* [B, S, S] */
    void* workspace;         /* forward scratch, nr_workspace_bytes(B, F, S) */
    size_t workspace_bytes;
    /* backward only: CSR adjacency vertex -> face corners, built once per faces tensor.
     * vertex_faces[vertex_offsets[v] .. vertex_offsets[v+1]) lists 3 f + k for every faces[f, k] == v. */
    const int32_t* vertex_offsets; /* [V + 1] */
    const int32_t* vertex_faces;   /* [3 F] */
    /* optional halo cache, nr_halo_bytes() bytes (the tile-border image values, then one byte per
     * 32x32 bin and item: "the bin has a foreground pixel", which lets the backward skip background
     * tiles): when set, the forward stores the internal-image
     * values of the backward's tile borders there and the backward reads them instead of shading
     * its tile halos again; NULL = backward re-shades (same results). */
    float* halo;
    /* lights (rasterize.py:252-283, lights.py:4-39), only with NR_DRAW_RGB.  lights holds
     * [num_lights][B][NR_LIGHT_FLOATS] records in list order: kind (NR_LIGHT_*), backside, colour
     * r g b, then direction x y z (directional) or alpha (specular, slot 5).  The smooth normal
     * map (rasterize.py:162-190) needs: */
    int num_lights;
    const float* lights;
    float* face_normals;             /* [B, F, 3] scratch (forward) */
    float* vertex_normals;           /* [B, V, 4]: normalised normal + norm; written by the forward,
                                        read by the backward */
    const int32_t* normal_offsets;   /* [V + 1] CSR vertex -> its distinct faces (the reference's */
    const int32_t* normal_faces;     /*          one-hot [F, V] matrix, rasterize.py:173-179)     */
    /* backgrounds, only with NR_DRAW_RGB: [B, 3, S, S] at the internal size (x stride 1); the rgb of
     * background pixels is backgrounds[b, c, S-1-y, S-1-x] (the blend of
     * neural_renderer_chainer/rasterize.py:574-577; the torch blend_backgrounds raises) */
    const float* backgrounds;
    long long bg_stride_b, bg_stride_c, bg_stride_y;
    float* grad_backgrounds;         /* backward output [B, 3, S, S] contiguous, fully written; or NULL */
    /* optional, only with NR_DRAW_RGB: nr_texture_packed_bytes() of scratch that the forward fills
     * with the texels as RGBA rows [Bt, ceil4(H*W), 4] (Bt = tex_stride_b ? B : 1) and the forward and
     * backward then sample (one 16-B load per bilinear corner); kept by the caller from the forward
     * to the backward.  NULL = sample `textures` directly (same results). */
    float* textures_packed;
    /* optional, read by nr_rasterize_forward only: the backward's workspace
     * (nr_backward_workspace_bytes), allocated before the forward.  The forward zeroes its first
     * bwd_workspace_bytes bytes (the backward's accumulators) from the face-setup launch; the caller
     * may then pass workspace_zeroed = 1 to the ONE nr_rasterize_backward call that uses this
     * workspace next (after a backward its accumulators are no longer zero).  NULL = nothing zeroed. */
    void* bwd_workspace;
    size_t bwd_workspace_bytes;
    /* 1 = the caller reads face_index only inside the 32x32 bins that hold candidate faces (the
     * backward with a halo cache reads no other entry; a bin without candidates is -1 throughout): the
     * fused forward then leaves those bins' -1 entries unwritten (64 % of the headline's face-index
     * map).  Honoured only with the halo cache and the fused shading; nr_rasterize_backward_params
     * (which reads every entry) refuses such a forward state.  0 = face_index fully written. */
    int face_index_sparse;
    /* optional, backward only (NR_DRAW_RGB, a texture and texture coordinates shared by the batch):
     * texture windows that many faces share -- every face of an OBJ's flat-colour material samples
     * one 2x2 atlas patch (load_obj.py:84-94), so every wave that renders such a material would add
     * its window into the same texels.  face_hot[f] in [0, num_hot) names the shared window of face f
     * (faces with identical texture-coordinate triples share it), -1 for the rest; the backward then
     * adds those faces' window sums into one of NR_HOT_COPIES private copies per hot window in
     * hot_acc (nr_hot_acc_bytes(num_hot) bytes; zero at the start, like the backward's accumulators:
     * zeroed by the forward when it lies inside bwd_workspace, otherwise by nr_rasterize_backward
     * unless workspace_zeroed) and sums the copies into the texture gradient after its main kernel.
     * num_hot <= NR_HOT_MAX.  NULL / 0 = every window adds into the texture gradient directly (same
     * results up to the order of float additions). */
    const int32_t* face_hot;
    int num_hot;
    float* hot_acc;
} NrRasterArgs;

enum { NR_HOT_MAX = 256, NR_HOT_COPIES = 32 };
/* bytes of NrRasterArgs.hot_acc for num_hot shared windows */
NR_API size_t nr_hot_acc_bytes(int num_hot);

enum { NR_LIGHT_AMBIENT = 0, NR_LIGHT_DIRECTIONAL = 1, NR_LIGHT_SPECULAR = 2, NR_LIGHT_FLOATS = 8 };

/* Channels in output order: rgb (3), silhouettes (1), depth (1) -- those enabled by draw_flags. */
NR_API int nr_num_channels(int draw_flags);

/* rasterize.py:194-329 (without lights / backgrounds): images [B, C, s, s] contiguous.  Ordered on
 * `stream`; a deep-bin batch (B % 8 == 0) forks part of the forward onto the library's side stream and
 * joins it back with events before returning (NR_LAUNCH_SPLIT). */
NR_API int nr_rasterize_forward(const NrRasterArgs* args, float* images, void* stream);

/* Bytes of NrRasterArgs.textures_packed for texture_items textures of H x W texels. */
NR_API size_t nr_texture_packed_bytes(int texture_items, int tex_height, int tex_width);

/* Bytes of NrRasterArgs.halo for B items at output size s (internal 2s with anti-aliasing). */
NR_API size_t nr_halo_bytes(int batch_size, int image_size, int anti_aliasing, int draw_flags);

/* Scratch bytes of nr_rasterize_backward: per-face gradient records [B, F, 9], the texture
 * gradient accumulator [texture_items, H*W rounded up to 4, 4], and with lights the per-face
 * vertex-normal gradients [B, F, 9] and per-vertex normal gradients [B, V, 3]. */
NR_API size_t nr_backward_workspace_bytes(int batch_size, int num_faces, int num_vertices, int texture_items,
                                          int tex_height, int tex_width, int num_lights);

/* Backward of nr_rasterize_forward for upstream grad_images [B, C, s, s] (contiguous), given the
 * state the forward saved in `args`.  Writes grad_vertices [B, V, 3] and, with NR_DRAW_RGB and
 * grad_textures != NULL, grad_textures [Bt, 3, H, W] contiguous with Bt = (tex_stride_b ? B : 1)
 * (the batch total when the textures are shared).  Needs args->vertex_offsets/vertex_faces.
 * workspace_zeroed: per call, 1 when the caller guarantees the workspace's accumulators are zero
 * (the forward zeroed them through NrRasterArgs.bwd_workspace and no backward has used it since):
 * the backward then skips its own zero fill; 0 = the backward zero-fills (always correct).  With 1,
 * args->bwd_workspace must be `workspace` and args->bwd_workspace_bytes must cover the accumulators
 * (NR_ERR_ARGS otherwise).  A second backward over the same forward state must pass 0.  A texture
 * gradient takes at most 2^25 texels per texture and rows of at most 2^22 - 1 texels (NR_ERR_ARGS). */
NR_API int nr_rasterize_backward(const NrRasterArgs* args, const float* grad_images, float* grad_vertices,
                                 float* grad_textures, void* workspace, size_t workspace_bytes, int workspace_zeroed,
                                 void* stream);

/* The gradients that only the rgb channels carry and nr_rasterize_backward does not produce, for the
 * same forward state and upstream grad_images:
 *   grad_vertices_textures [Bvt, Vt, 2] (Bvt = vt_batch_stride ? B : 1; the batch total when shared):
 *     autograd of sample_textures' uv interpolation and clamps (rasterize.py:111-121) and of the
 *     faces_textures gather (rasterize.py:246);
 *   grad_lights [num_lights, B, NR_LIGHT_FLOATS], laid out like NrRasterArgs.lights: colour at 2..4,
 *     direction at 5..7 (directional) or exponent alpha at 5 (specular), zero elsewhere: autograd of
 *     the light loop (rasterize.py:252-283).
 * Either may be NULL; those given are fully written (zeroed, then accumulated).  Needs NR_DRAW_RGB. */
NR_API int nr_rasterize_backward_params(const NrRasterArgs* args, const float* grad_images,
                                        float* grad_vertices_textures, float* grad_lights, void* stream);

/* Camera prologue of Renderer.transform_vertices (renderer.py:27-38): look_at (look_at.py:5-44, with
 * the default at = (0, 0, 0) / up = (0, 1, 0) or the given ones) and/or perspective
 * (perspective.py:4-18), fused.  Cross products are per item (the reference's dim-less torch.cross
 * mixes items at B == 3, SURVEY section 8a hazards). */
enum { NR_CAMERA_NONE = 0, NR_CAMERA_LOOK_AT = 1 };
typedef struct NrCameraArgs {
    int batch_size;            /* B */
    int num_vertices;          /* V */
    const float* vertices;     /* [B, V, 3] world space; v_batch_stride 0 = one mesh for every item */
    long long v_batch_stride;
    const float* eye;          /* [B, 3] viewpoints; eye_batch_stride 0 = one eye for every item */
    long long eye_batch_stride;
    int mode;                  /* NR_CAMERA_* */
    float at[3], up[3];
    int perspective;           /* apply x / z / width, y / z / width */
    float width;               /* tan(angle / 180 * 3.1416) in f32, as perspective.py:10-13 computes it */
} NrCameraArgs;

/* out [B, V, 3] contiguous. */
NR_API int nr_camera_forward(const NrCameraArgs* args, float* out, void* stream);
/* Scratch bytes of nr_camera_backward (per-item eye-gradient sums). */
NR_API size_t nr_camera_workspace_bytes(int batch_size);
/* grad_out [B, V, 3] -> grad_vertices [Bv, V, 3] (Bv = v_batch_stride ? B : 1, the item sum for a
 * shared mesh) and grad_eye [Be, 3] (Be = eye_batch_stride ? B : 1); either may be NULL, those
 * given are fully written. */
NR_API int nr_camera_backward(const NrCameraArgs* args, const float* grad_out, float* grad_vertices,
                              float* grad_eye, void* workspace, size_t workspace_bytes, void* stream);

/* Diagnostics (no reference counterpart): the kernels replace some IEEE divisions by a shortened
 * form of the compiler's own division sequence inside a guarded operand range (DESIGN.md,
 * "Numerics").  This runs both forms on n operand pairs so tests can check they agree bit for bit. */
NR_API int nr_selftest_division(const float* a, const float* b, float* q_fast, float* q_ieee, long long n,
                                void* stream);

/* Measurement hook (bench.py's roofline leg; no reference counterpart).  With profiling on, the
 * library brackets each launch of its kernels with a pair of HIP events recorded on the launch
 * stream; nr_profile_read gives the mean duration in ms of the launches of `kernel` ("k_face_setup",
 * "k_raster_fwd", "k_shade", "k_raster_bwd", "k_vertex_grad", "k_tex_out", "k_tex_pack") recorded
 * since profiling was last enabled (up to the last 64), once the stream has been synchronised;
 * nr_profile_enable(1) while on starts a new measurement.  Process-wide state, meant for a single
 * measuring thread. */
NR_API int nr_profile_enable(int on);
NR_API int nr_profile_read(const char* kernel, float* ms);

/* Launch record (no reference counterpart; the tests use it to assert which kernel variant ran).
 * For the most recent launch of `kernel` ("k_raster_fwd" or "k_raster_bwd") in this process
 * (process-wide, like the profiling hook; torch issues a backward from its autograd thread): block_threads = threads per block (k_raster_fwd: 256 = four 16x16 quadrants per
 * 32x32 bin, 1024 = one wave per 8x8 block; k_raster_bwd: 256 = 2 pixels per lane, 512 = 1 pixel
 * per lane) and flags = NR_LAUNCH_* bits.  NR_ERR_ARGS when none was recorded. */
enum { NR_LAUNCH_FUSED_SHADE = 1, NR_LAUNCH_STATIC_CHANNELS = 2, NR_LAUNCH_TWO_PX_PER_LANE = 4,
       NR_LAUNCH_DEEP_FIRST = 8 /* k_raster_fwd: bins dispatched deepest first (k_bin_order) */,
       NR_LAUNCH_SPLIT = 16 /* k_raster_fwd: deep bins at 1024 threads, the rest at 256 on a side stream */,
       NR_LAUNCH_HOT_WINDOWS = 32 /* k_raster_bwd: shared texture windows into private copies (face_hot) */,
       NR_LAUNCH_DEALT_QUARTERS = 64 /* k_raster_fwd: deep bins' 4x4 quarters dealt to the waves (not split) */,
       NR_LAUNCH_QUADRANTS = 128 /* k_raster_fwd: deep bins walked by four blocks, one per 16x16 quadrant (not split) */ };
NR_API int nr_last_launch(const char* kernel, int* block_threads, int* flags);

#ifdef NR_COUNT_TESTS
/* Face-test counters, in the diagnostic build compiled with -DNR_COUNT_TESTS only
 * (_lib/libnr_raster_count.so, bench.py's face-test rate; SURVEY 8d's secondary bound, the reference's
 * brute force doing B*S^2*F tests per call, rasterize_cuda_kernel.cu:82-149).  Since the last reset,
 * out[0] = (pixel, face) pass tests the forward's walks evaluated (64 per face a wave walks over an 8x8
 * block, 16 over a 4x4 quarter), out[1] = faces walked (wave level), out[2] = deferred commit batches
 * (the division chain, run by a whole wave), out[3] = walks (8x8 blocks or quarters walked).  reset != 0
 * zeroes them after the read (device-wide counters: call with the device idle). */
NR_API int nr_count_read(unsigned long long* out4, int reset);
#endif

#ifdef __cplusplus
}
#endif
#endif /* NR_RASTER_H_ */
