// nr_raster.hip -- MI355X (gfx950 / CDNA4) differentiable mesh rasterizer.
//
// Hand-written HIP behind the C ABI of include/nr_raster.h.  Replaces the reference's CUDA
// extension (neural_renderer_torch/cuda/rasterize_cuda_kernel.cu) AND the torch glue around it in
// rasterize_core (neural_renderer_torch/rasterize.py:194-329), with the same results:
//   * face_index_map bit-exact: every pixel scans, in ascending face order, a superset of the faces
//     whose bounding box contains it, with the reference's float arithmetic unchanged
//     (rasterize_cuda_kernel.cu:82-149; no FMA contraction, IEEE division, double pixel centres);
//   * rgb / depth / silhouette values follow rasterize.py:80-153 operation for operation.
//
// Pipeline of one forward (3 launches: setup, raster, shade) -- see DESIGN.md for the data layout and rooflines:
//   k_face_setup     one block per (128 faces, item): gather the faces from vertices (rasterize.py:232),
//                    per-face screen bbox + face-level rejects, texture-uv gather, and the coarse-bin
//                    face bitmasks (32x32-pixel bins, bit f set when face f may touch the bin).
//   k_raster_fwd     one block per 32x32-pixel coarse bin: stages the bin's candidate faces in face
//                    order into LDS, each wave walks (ballot) the faces touching its pixels in order;
//                    writes the face-index map.
//   k_shade          one thread per output pixel: weights, texture, silhouette, depth, merged,
//                    flipped and 2x2-averaged into the [B, C, s, s] image.
//   backward         k_raster_bwd: one block per 32x16 pixels + 1-pixel halo: recomputes the internal
//                    image from fim, applies Differentiation.backward's stencil, and chains the
//                    coordinate / depth / texture gradients to vertices and textures with atomics.
//
// Source layout (one translation unit): nr_common.h (errors, profiling, geometry, exact division,
// per-pixel shading, XCD tile map), nr_fwd.h (setup + face-index raster), nr_shade.h (image epilogue,
// halo cache, standalone reference kernels), nr_bwd.h (backward), nr_camera.h (look_at + perspective),
// nr_host.h (argument checks); this file holds the extern "C" ABI.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <limits.h>
#include <math.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <cstdlib>
#include <string>

#include "nr_raster.h"


#pragma clang fp contract(off)

#include "nr_cull.h"
#include "nr_pixel.h"
#include "nr_common.h"
#include "nr_shade.h"
#include "nr_fwd.h"
#include "nr_bwd.h"
#include "nr_camera.h"
#include "nr_host.h"


// self-test of the exact division shortcut (nr_selftest_division): q_fast = div_nr(a, b, rcp_nr(b)),
// q_ieee = a / b as the compiler lowers it
__global__ void k_selftest_div(const float* __restrict__ a, const float* __restrict__ b, float* __restrict__ qf,
                               float* __restrict__ qi, long long n) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float x = a[i], y = b[i];
    qf[i] = div_nr(x, y, rcp_nr(y));
    qi[i] = x / y;
}

#ifdef NR_ABL_EXTRAK
// (timing builds) an empty dispatch: its cost in the step is one launch and drain
__global__ void k_abl_empty(int) {}
#endif

// ==================================================================================================
extern "C" {

const char* nr_last_error(void) { return g_err.c_str(); }
int nr_version(void) { return NR_ABI_VERSION; }
size_t nr_raster_args_size(void) { return sizeof(NrRasterArgs); }

int nr_num_channels(int draw_flags) {
    return ((draw_flags & NR_DRAW_RGB) ? 3 : 0) + ((draw_flags & NR_DRAW_SILHOUETTES) ? 1 : 0) +
           ((draw_flags & NR_DRAW_DEPTH) ? 1 : 0);
}

size_t nr_hot_acc_bytes(int num_hot) {
    if (num_hot <= 0) return 0;
    return align_up(hot_sums_floats(num_hot) * 4) + align_up((size_t)num_hot * 8);
}

size_t nr_workspace_bytes(int batch_size, int num_faces, int image_size) {
    const Geom g = make_geom(num_faces, image_size);
    return ws_bbox_bytes(batch_size, num_faces) + ws_mask_bytes(batch_size, g) + ws_order_bytes(batch_size, g);
}

// A side stream per (host thread, device) for the split forward, with its fork / join events; created
// on first use outside a stream capture (null: no split for this call).  The thread's table releases
// them when the thread ends (a worker pool's recycled threads do not accumulate streams).  No
// synchronisation there: hipStreamDestroy of a stream with queued work returns at once and releases it
// when the work is done, and a synchronising call from an exiting thread would invalidate another
// thread's graph capture in global capture mode; the destroys themselves run in this thread's relaxed
// capture mode for the same reason.  Errors are ignored (at process exit the runtime may be gone).
struct SideStream {
    hipStream_t s = nullptr;
    hipEvent_t fork = nullptr, join = nullptr;
};
struct SideStreamTable {
    SideStream tab[64];
    ~SideStreamTable() {
        bool any = false;
        for (const SideStream& x : tab) any = any || x.s || x.fork || x.join;
        if (!any) return;
        hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
        const bool exch = hipThreadExchangeStreamCaptureMode(&mode) == hipSuccess;
        for (SideStream& x : tab) {
            if (x.s) (void)hipStreamDestroy(x.s);
            if (x.fork) (void)hipEventDestroy(x.fork);
            if (x.join) (void)hipEventDestroy(x.join);
            x = SideStream{};
        }
        if (exch) (void)hipThreadExchangeStreamCaptureMode(&mode);
    }
};
#ifndef NR_SPLIT_BUCKET
#define NR_SPLIT_BUCKET 10
#endif
constexpr int SPLIT_BUCKET = NR_SPLIT_BUCKET;  // deep bins: >= 512 candidates
#ifndef NR_QS_CAP
#define NR_QS_CAP 16
#endif
constexpr int QS_CAP = NR_QS_CAP;  // deep bins per list walked by quadrant blocks (a forward that does not split)
SideStream* side_stream(hipStream_t st) {
    static thread_local SideStreamTable table;
    SideStream* tab = table.tab;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
    // the side stream lives on the current device: a caller's stream of another device gets no split
    hipDevice_t sdev = dev;
    if (st && hipStreamGetDevice(st, &sdev) != hipSuccess) return nullptr;
    if (sdev != dev) return nullptr;
    SideStream& x = tab[dev];
    if (!x.s) {
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
        if (hipEventCreateWithFlags(&x.fork, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&x.join, hipEventDisableTiming) != hipSuccess ||
            hipStreamCreateWithFlags(&x.s, hipStreamNonBlocking) != hipSuccess) {
            if (x.fork) (void)hipEventDestroy(x.fork);
            if (x.join) (void)hipEventDestroy(x.join);
            x = SideStream{};
            return nullptr;
        }
    }
    return &x;
}

// 1024-thread blocks of k_raster_fwd resident at once on one XCD of the current device: two per CU
// (32 waves and 2 x 62.6 KB of LDS), the CUs dealt evenly over the 8 XCDs
static int deep_slots_per_xcd() {
    static int cached[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 64;
    if (!cached[dev]) {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
        __atomic_store_n(&cached[dev], 2 * max(cus / 8, 1), __ATOMIC_RELAXED);
    }
    return __atomic_load_n(&cached[dev], __ATOMIC_RELAXED);
}

static int run_face_index(const float* vertices, const int32_t* faces_idx, float* face_records, int32_t* fim,
                          int B, int V, int F, int S, float near, float far, int draw_backside, float delta,
                          void* ws, size_t ws_bytes, hipStream_t st, const NrRasterArgs* ra, float* images,
                          TexPack pk, ZeroFill zf = ZeroFill{nullptr, 0}) {
    Geom g = make_geom(F, S);
    g.group = group_for(B, FWD_GROUP);
    g.B = B;
    int2* bbox = (int2*)ws;
    uint32_t* mask = (uint32_t*)((char*)ws + ws_bbox_bytes(B, F));
    uint8_t* bin_part = (uint8_t*)mask + ws_mask_bytes(B, g);
    int* bin_order = (int*)(bin_part + ws_part_bytes(B, g));
    if (B == 0) return NR_OK;
    // forward block size (k_raster_fwd notes): 256 threads when the grid alone fills the chip many
    // times over and the bins are shallow; 1024 when it does not, or when the bins are deep (F per bin
    // at the 32x32 bin granularity as the depth proxy)
    const long long blocks = (long long)g.nbins * B;
    const double faces_per_bin = (double)F / g.nbins;
    const int ntf = (blocks >= 8192 && faces_per_bin < 40.0) ? 256 : 1024;
    // deep bins (the car, the 50k torus): dispatch the bins deepest first (k_bin_order), from candidate
    // counts the setup adds up (its LDS bin-mask path); a list per XCD needs B % 8 == 0 or fits one block
    const long long order_list = (B % 8 == 0 ? B / 8 : B) * (long long)g.nbins;  // entries per k_bin_order block
    const bool ordered = F > 0 && ntf == 1024 && faces_per_bin >= 24.0 &&
                         (long long)g.nbins * (SETUP_FACES / 32) <= SETUP_LDS_WORDS && order_list <= ORDER_MAX_ENTRIES;
    // the setup's idle threads repack the textures when that takes them up to 32 texels each; with no
    // setup launch, or a texture too large for that, the repacking gets a launch of its own
    const long long setup_idle = (long long)((F + SETUP_FACES - 1) / SETUP_FACES) * B * (256 - SETUP_FACES);
    if (pk.out && (F == 0 || pk.n > 32 * setup_idle)) {
        ProfScope _p(P_TEXPACK, st, true);
        nr_launch(k_tex_pack, dim3((unsigned)((pk.n + 255) / 256)), dim3(256), 0, st, pk);
        const int e = check_launch("k_tex_pack");
        if (e) return e;
        pk.out = nullptr;
    }
    if (F == 0 && zf.p && hipMemsetAsync(zf.p, 0, (size_t)zf.n16 * 16, st) != hipSuccess)
        return check_launch("hipMemsetAsync");

    // k_shade's work fused into the forward's 256-thread variant (anti-aliasing, no lights or
    // backgrounds): the face-index map is not read back, and there is one launch fewer
    const Shade sh = ra ? make_shade(ra) : Shade{};
    // the deep-bin / small-grid 1024-thread variant shades too (its threads 0-255)
    const bool fuse = ra && ra->anti_aliasing && sh.nl == 0 && !sh.bg && vertices;
    // the split forward (below) when the batch is deep-first, fused and B % 8 == 0; otherwise a
    // deep-first forward reads its bins' mask words through sparse groups: the setup writes only the
    // (group, bin) pieces with candidates, and each forward block lists its bin's groups from the
    // setup's counts (for the 50k torus at 1024^2: 1024 bins x 1563 words of dense masks for ~10^4
    // non-empty pieces).  A split that finds no side stream falls back to the dense reads (the setup
    // wrote every piece)
    const int Bcap = B % 8 == 0 ? max(8, (B / 4 + 7) / 8 * 8) : 0;
    const bool want_split = ordered && fuse && B % 8 == 0 && Bcap <= B;
#ifndef NR_NO_SPARSE_GROUPS
    const bool sg = ordered && !want_split && setup_groups(g) <= 1024;
#else
    const bool sg = false;
#endif
    if (F > 0) {
        dim3 grid((F + SETUP_FACES - 1) / SETUP_FACES, B);
        const bool rgb = ra && (ra->draw_flags & NR_DRAW_RGB);
        const int uv_items = rgb ? (ra->vt_batch_stride ? B : 1) : 0;
        ProfScope _p(P_SETUP, st, true);
        const bool lit = rgb && ra->num_lights > 0;
        const size_t lds = (size_t)setup_lds_words(g.nbins) * 4;
        if (vertices)
            nr_launch(k_face_setup<true>, grid, dim3(256), lds, st, vertices, faces_idx, face_records, V, F, S,
                               draw_backside, bbox, mask, g.nbx, g.nbins, g.nwords,
                               rgb ? ra->vertices_textures : nullptr, rgb ? ra->vt_batch_stride : 0,
                               rgb ? ra->num_vertices_textures : 0, rgb ? ra->faces_textures : nullptr,
                               rgb ? ra->face_uv : nullptr, uv_items, lit ? ra->face_normals : nullptr, pk, zf,
                               ordered ? bin_part : nullptr, B % 8 == 0, sg ? 1 : 0);
        else
            nr_launch(k_face_setup<false>, grid, dim3(256), lds, st, nullptr, nullptr, face_records, V, F, S,
                               draw_backside, bbox, mask, g.nbx, g.nbins, g.nwords, nullptr, 0, 0, nullptr, nullptr, 0,
                               nullptr, pk, zf, ordered ? bin_part : nullptr, B % 8 == 0, sg ? 1 : 0);
        int e = check_launch("k_face_setup");
        if (e) return e;
        if (lit && V > 0) {
            const long long nv = (long long)B * V;
            nr_launch(k_vertex_normals, dim3((unsigned)((nv + 255) / 256)), dim3(256), 0, st, ra->face_normals,
                               ra->normal_offsets, ra->normal_faces, ra->vertex_normals, F, V, nv);
            e = check_launch("k_vertex_normals");
            if (e) return e;
        }
    }
    // split forward (deep-bin batches of B % 8 == 0 items, e.g. the car): the bins with >= 2^(SPLIT_BUCKET
    // - 1) candidates (a prefix of each deep-first list, at most Bcap / 8 * nbins of them) in the
    // 1024-thread variant on the caller's stream, the rest in the 256-thread variant on a side stream at
    // the same time: a shallow bin's 16 waves in the 1024-thread variant mostly wait for their block's
    // slowest wave, where the 256-thread variant deals its 16 8x8 blocks to 4 waves
    int* split_cnt = (int*)((char*)bin_order + align_up((size_t)B * g.nbins * 4));
    SideStream* side = nullptr;
#ifndef NR_NO_SPLIT
    if (want_split) side = side_stream(st);
#endif
    // the deep launch takes at most 7/8 of one XCD's slots for 1024-thread blocks per list (two per CU,
    // by their waves and LDS), so every deep bin is dispatched at once: a deep block waiting for a slot
    // starves behind the rest launch's 256-thread blocks, which take every CU space that frees up (at
    // 75 deep bins per list the last ones started at 430 us of a 535 us car forward,
    // profiles/r05_v56_car_fwd_wave_phases.txt); the bins past the cap go to the rest launch.  Car
    // forward 0.49-0.50 -> 0.44 ms at 56 per list (48: the same; 40: 0.57 ms, the bins it leaves to the
    // 256-thread launch then end last; 64: 0.46-0.48 ms; no cap: 0.50 ms; same-box A/Bs, 3 runs each,
    // gpurun_out/e7, e9)
    const int deep_cap = min(Bcap / 8 * g.nbins, deep_slots_per_xcd() * 7 / 8);
    // a deep-first forward that does not split (e.g. one item, the 50k torus): each list's bins of
    // >= 512 candidates (up to QS_CAP of them) are walked by four blocks each, one per 16x16 quadrant
    // (ordered_bin part 3), so the deepest bins, which set the span while most of the chip idles, spread
    // over four CUs
#ifndef NR_NO_QS
    const bool qs = ordered && !side;
#else
    const bool qs = false;
#endif
    const int lists = B % 8 == 0 ? 8 : 1;
    const unsigned qs_grid = (unsigned)((long long)g.nbins * B + (qs ? 3 * QS_CAP * lists : 0));
    if (ordered) {
        nr_launch(k_bin_order, dim3(lists), dim3(1024), 0, st, bin_part, setup_groups(g), bin_order, B,
                           g.nbins, (side || qs) ? split_cnt : nullptr, SPLIT_BUCKET, side ? deep_cap : QS_CAP);
        const int e = check_launch("k_bin_order");
        if (e) return e;
    }
    const int* order = ordered ? bin_order : nullptr;
    // per-bin foreground flags after the halo values (the backward skips background tiles)
    uint8_t* binfg = (ra && ra->halo) ? (uint8_t*)ra->halo + halo_flags_offset_bytes(B, S, sh.C) : nullptr;
    // empty bins leave their -1 face ids unwritten (NrRasterArgs.face_index_sparse): with the fused
    // shading nothing else in this launch reads them, and the backward skips those tiles by the flags
    const int sparse = (ra && ra->face_index_sparse && fuse && binfg) ? 1 : 0;
    {
        ProfScope _p(P_RASTER, st, side == nullptr);
        const int rs = vertices ? FACE_REC : 9;
        g_last_fwd.store(LaunchRec{ntf, (fuse ? NR_LAUNCH_FUSED_SHADE : 0) |
                                        (fuse && ntf == 256 && (sh.C == MAXC || sh.draw == static_draw(4)) ? NR_LAUNCH_STATIC_CHANNELS : 0) |
                                        (ordered ? NR_LAUNCH_DEEP_FIRST : 0) | (side ? NR_LAUNCH_SPLIT : 0) |
                                        (ordered && !side && ntf == 1024 ? NR_LAUNCH_DEALT_QUARTERS : 0) |
                                        (qs ? NR_LAUNCH_QUADRANTS : 0)});
        if (side) {
            // fork: the side stream waits for the setup and the order; join: the caller's stream waits
            // for the side stream's launch
            if (hipEventRecord(side->fork, st) != hipSuccess || hipStreamWaitEvent(side->s, side->fork, 0) != hipSuccess)
                return check_launch("hipEventRecord");
            // (a grid of exactly the cap's blocks: every block past a list's deep prefix exits at once, but
            // each still needs a 1024-thread slot to be dispatched in)
            // (the dealt-quarter variant with its four-faces-per-step walk here instead: car forward 0.427 ->
            // 0.434 ms, same-box A/B, gpurun_out/w4b: the deep launch takes more of the rest's wave slots)
            nr_launch((k_raster_fwd<1024, true>), dim3(8 * deep_cap), dim3(1024), 0, st, face_records, rs, bbox,
                               mask, F, g, near, far, delta, fim, sh, images, ra->halo, binfg, order, sparse, split_cnt, 1, nullptr);
            int e = check_launch("k_raster_fwd");
            if (e) return e;
            if (sh.C == MAXC)
                nr_launch((k_raster_fwd<256, true, MAXC>), dim3(g.nbins, B), dim3(256), 0, side->s, face_records, rs,
                                   bbox, mask, F, g, near, far, delta, fim, sh, images, ra->halo, binfg, order, sparse,
                                   split_cnt, 2, nullptr);
            else if (sh.draw == static_draw(4))  // rgba (the car): compile-time channels
                nr_launch((k_raster_fwd<256, true, 4>), dim3(g.nbins, B), dim3(256), 0, side->s, face_records, rs,
                                   bbox, mask, F, g, near, far, delta, fim, sh, images, ra->halo, binfg, order, sparse,
                                   split_cnt, 2, nullptr);
            else
                nr_launch((k_raster_fwd<256, true>), dim3(g.nbins, B), dim3(256), 0, side->s, face_records, rs, bbox,
                                   mask, F, g, near, far, delta, fim, sh, images, ra->halo, binfg, order, sparse, split_cnt, 2, nullptr);
            e = check_launch("k_raster_fwd");
            if (e) return e;
            if (hipEventRecord(side->join, side->s) != hipSuccess || hipStreamWaitEvent(st, side->join, 0) != hipSuccess)
                return check_launch("hipEventRecord");
        } else if (fuse && ntf == 1024 && ordered)  // deep bins, not split (e.g. one item): dealt quarters
            nr_launch((k_raster_fwd<1024, true, 0, true>), dim3(qs_grid),
                      dim3(1024), 0, st, face_records, rs, bbox, mask, F, g, near, far, delta, fim, sh, images, ra->halo,
                      binfg, order, sparse, split_cnt, qs ? 3 : 0, sg ? bin_part : nullptr);
        else if (fuse && ntf == 1024)
            nr_launch((k_raster_fwd<1024, true>), dim3(g.nbins, B), dim3(1024), 0, st, face_records, rs, bbox,
                               mask, F, g, near, far, delta, fim, sh, images, ra->halo, binfg, order, sparse, nullptr, 0, nullptr);
        else if (fuse && sh.C == MAXC)  // rgb + sil + depth: compile-time channels
            nr_launch((k_raster_fwd<256, true, MAXC>), dim3(g.nbins, B), dim3(256), 0, st, face_records, rs, bbox,
                               mask, F, g, near, far, delta, fim, sh, images, ra->halo, binfg, order, sparse, nullptr, 0, nullptr);
        else if (fuse && sh.draw == static_draw(4))  // rgba: compile-time channels
            nr_launch((k_raster_fwd<256, true, 4>), dim3(g.nbins, B), dim3(256), 0, st, face_records, rs, bbox,
                               mask, F, g, near, far, delta, fim, sh, images, ra->halo, binfg, order, sparse, nullptr, 0, nullptr);
        else if (fuse)
            nr_launch((k_raster_fwd<256, true>), dim3(g.nbins, B), dim3(256), 0, st, face_records, rs, bbox, mask,
                               F, g, near, far, delta, fim, sh, images, ra->halo, binfg, order, sparse, nullptr, 0, nullptr);
        else if (ntf == 256)
            nr_launch((k_raster_fwd<256, false>), dim3(g.nbins, B), dim3(256), 0, st, face_records, rs, bbox, mask,
                               F, g, near, far, delta, fim, sh, nullptr, nullptr, binfg, order, 0, nullptr, 0, nullptr);
        else if (ordered)
            nr_launch((k_raster_fwd<1024, false, 0, true>), dim3(qs_grid),
                      dim3(1024), 0, st, face_records, rs, bbox, mask, F, g, near, far, delta, fim, sh, nullptr, nullptr,
                      binfg, order, 0, split_cnt, qs ? 3 : 0, sg ? bin_part : nullptr);
        else
            nr_launch((k_raster_fwd<1024, false>), dim3(g.nbins, B), dim3(1024), 0, st, face_records, rs, bbox,
                               mask, F, g, near, far, delta, fim, sh, nullptr, nullptr, binfg, order, 0, nullptr, 0, nullptr);
    }
    int e = check_launch("k_raster_fwd");
    if (e || !ra || fuse) return e;
    const int s = ra->anti_aliasing ? S / 2 : S;
    {
        ProfScope _p(P_SHADE, st, true);
        if (((long long)s * s + 255) / 256 * B < 4096) {
            const dim3 grid((unsigned)(((long long)s * s + (ra->anti_aliasing ? 63 : 255)) / (ra->anti_aliasing ? 64 : 256)), B);
            switch ((sh.nl ? 1 : 0) | (sh.bg ? 2 : 0)) {
                case 0: nr_launch(k_shade_px<0>, grid, dim3(256), 0, st, face_records, fim, F, S, sh, ra->anti_aliasing, images, ra->halo); break;
                case 1: nr_launch(k_shade_px<1>, grid, dim3(256), 0, st, face_records, fim, F, S, sh, ra->anti_aliasing, images, ra->halo); break;
                case 2: nr_launch(k_shade_px<2>, grid, dim3(256), 0, st, face_records, fim, F, S, sh, ra->anti_aliasing, images, ra->halo); break;
                default: nr_launch(k_shade_px<3>, grid, dim3(256), 0, st, face_records, fim, F, S, sh, ra->anti_aliasing, images, ra->halo); break;
            }
            return check_launch("k_shade");
        }
        const dim3 grid((unsigned)(((long long)s * s + 255) / 256), B);
        switch ((sh.nl ? 1 : 0) | (sh.bg ? 2 : 0)) {
            case 0: nr_launch(k_shade<0>, grid, dim3(256), 0, st, face_records, fim, F, S, sh, ra->anti_aliasing, images, ra->halo); break;
            case 1: nr_launch(k_shade<1>, grid, dim3(256), 0, st, face_records, fim, F, S, sh, ra->anti_aliasing, images, ra->halo); break;
            case 2: nr_launch(k_shade<2>, grid, dim3(256), 0, st, face_records, fim, F, S, sh, ra->anti_aliasing, images, ra->halo); break;
            default: nr_launch(k_shade<3>, grid, dim3(256), 0, st, face_records, fim, F, S, sh, ra->anti_aliasing, images, ra->halo); break;
        }
    }
    return check_launch("k_shade");
}

int nr_face_index_map_forward_safe(const float* faces, int32_t* face_index, int batch_size, int num_faces,
                                   int image_size, float near, float far, int draw_backside, float eps,
                                   float depth_min_delta, void* workspace, size_t workspace_bytes, void* stream) {
    (void)eps;
    if (batch_size < 0 || num_faces < 0 || image_size <= 0 || image_size > 16384)
        return fail(NR_ERR_ARGS, "bad sizes B=%d F=%d S=%d", batch_size, num_faces, image_size);
    if (batch_size > 0 && (!face_index || (num_faces > 0 && !faces))) return fail(NR_ERR_ARGS, "null pointer");
    if (workspace_bytes < nr_workspace_bytes(batch_size, num_faces, image_size))
        return fail(NR_ERR_WORKSPACE, "workspace too small");
    return run_face_index(nullptr, nullptr, const_cast<float*>(faces), face_index, batch_size, 0, num_faces,
                          image_size, near, far, draw_backside, depth_min_delta, workspace, workspace_bytes,
                          (hipStream_t)stream, nullptr, nullptr, TexPack{});
}

int nr_compute_weight_map(const float* faces, const int32_t* face_index_map, float* weight_map, int batch_size,
                          int num_faces, int image_size, void* stream) {
    // the kernels' pixel centres are exact for S <= 16384 (nr_pixel.h), as in the other entry points
    if (batch_size < 0 || num_faces < 0 || image_size <= 0 || image_size > 16384)
        return fail(NR_ERR_ARGS, "bad sizes B=%d F=%d S=%d", batch_size, num_faces, image_size);
    const long long n = (long long)batch_size * image_size * image_size;
    if (n == 0) return NR_OK;
    nr_launch(k_weight_map, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, faces,
                       face_index_map, weight_map, num_faces, image_size, n);
    return check_launch("k_weight_map");
}

int nr_mask_foreground_forward(const int32_t* face_index, const float* data_in, float* data_out, long long n, int dim,
                               void* stream) {
    if (n < 0 || dim < 0) return fail(NR_ERR_ARGS, "bad sizes");
    if (n == 0) return NR_OK;
    nr_launch(k_mask_fg, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, face_index,
                       data_in, data_out, n, dim);
    return check_launch("k_mask_fg");
}

int nr_mask_foreground_backward(const int32_t* face_index, float* grad_in, const float* grad_out, long long n, int dim,
                                void* stream) {
    return nr_mask_foreground_forward(face_index, grad_out, grad_in, n, dim, stream);
}

int nr_differentiation_backward(const float* images, const float* grad, float* grad_xy, int batch_size, int height,
                                int width, int channels, void* stream) {
    if (batch_size < 0 || height <= 0 || width <= 0 || channels <= 0) return fail(NR_ERR_ARGS, "bad sizes");
    const long long n = (long long)batch_size * height * width;
    if (n == 0) return NR_OK;
    const float step = (float)(2. / height);
    nr_launch(k_diff_bwd, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, images, grad,
                       grad_xy, height, width, channels, step, n);
    return check_launch("k_diff_bwd");
}

int nr_rasterize_forward(const NrRasterArgs* a, float* images, void* stream) {
    int e = validate_raster(a, true);
    if (e) return e;
    if (!images && a->batch_size > 0) return fail(NR_ERR_ARGS, "null images");
    TexPack pk{};
    if ((a->draw_flags & NR_DRAW_RGB) && a->textures_packed && a->batch_size > 0) {
        const int tex_items = a->tex_stride_b ? a->batch_size : 1;
        pk.tex = a->textures;
        pk.sb = a->tex_stride_b;
        pk.sc = (int)a->tex_stride_c;
        pk.sp = (int)a->tex_stride_p;
        pk.HW = a->tex_height * a->tex_width;
        pk.HWp = (pk.HW + 3) & ~3;
        pk.out = reinterpret_cast<float4*>(a->textures_packed);
        pk.n = (long long)tex_items * pk.HWp;
    }
    // the backward's accumulators, zeroed by the setup's idle threads (no memset launch in the backward)
    ZeroFill zf{nullptr, 0};
    if (a->bwd_workspace && a->bwd_workspace_bytes > 0) {
        if (((uintptr_t)a->bwd_workspace & 15) || (a->bwd_workspace_bytes & 15))
            return fail(NR_ERR_ARGS, "bwd_workspace must be 16-byte aligned and sized");
        zf.p = reinterpret_cast<float4*>(a->bwd_workspace);
        zf.n16 = (long long)(a->bwd_workspace_bytes / 16);
    }
    const int S = a->anti_aliasing ? 2 * a->image_size : a->image_size;
    return run_face_index(a->vertices, a->faces, a->face_records, a->face_index, a->batch_size, a->num_vertices,
                          a->num_faces, S, a->near, a->far, a->draw_backside, a->depth_min_delta, a->workspace,
                          a->workspace_bytes, (hipStream_t)stream, a, images, pk, zf);
}

size_t nr_texture_packed_bytes(int texture_items, int tex_height, int tex_width) {
    if (texture_items <= 0 || tex_height <= 0 || tex_width <= 0) return 0;
    return (size_t)texture_items * ((((size_t)tex_height * tex_width) + 3) & ~size_t(3)) * 16;
}

size_t nr_halo_bytes(int batch_size, int image_size, int anti_aliasing, int draw_flags) {
    const int S = anti_aliasing ? 2 * image_size : image_size;
    if (batch_size <= 0 || image_size <= 0) return 0;
    const Geom g = make_geom(0, S);
    return (size_t)halo_flags_offset_bytes(batch_size, S, nr_num_channels(draw_flags)) +
           (((size_t)batch_size * g.nbins + 3) & ~size_t(3));
}

// backward workspace: [gF: B F 9 face-corner floats][g4: Bt HWp RGBA texel rows]
// [lights: gN: B F 9][gU: B V 3]; everything before gU starts at zero (one memset, or the forward's
// setup zeroed it: NrRasterArgs.bwd_workspace)
size_t nr_backward_workspace_bytes(int batch_size, int num_faces, int num_vertices, int texture_items,
                                   int tex_height, int tex_width, int num_lights) {
    const size_t hw = (size_t)tex_height * tex_width, hwp = (hw + 3) & ~size_t(3);
    size_t n = align_up((size_t)batch_size * num_faces * 9 * 4);
    if (texture_items > 0) n += align_up((size_t)texture_items * hwp * 16);
    if (num_lights > 0)
        n += align_up((size_t)batch_size * num_faces * 9 * 4) + align_up((size_t)batch_size * num_vertices * 3 * 4);
    return n;
}

int nr_rasterize_backward(const NrRasterArgs* a, const float* grad_images, float* grad_vertices, float* grad_textures,
                          void* workspace, size_t workspace_bytes, int workspace_zeroed, void* stream) {
    int e = validate_raster(a, false);
    if (e) return e;
    if (a->batch_size == 0) {
        // an empty batch still owes the caller its batch-shared gradient: a shared texture
        // (tex_stride_b == 0: one item) gets zeros; per-item textures and backgrounds have no items
        if ((a->draw_flags & NR_DRAW_RGB) && grad_textures && !a->tex_stride_b) {
            const size_t n = (size_t)3 * a->tex_height * a->tex_width * sizeof(float);
            if (n && hipMemsetAsync(grad_textures, 0, n, (hipStream_t)stream) != hipSuccess)
                return check_launch("hipMemsetAsync");
        }
        return NR_OK;
    }
    if (!grad_images || !grad_vertices) return fail(NR_ERR_ARGS, "null gradient buffers");
    if (a->num_faces > 0 && (!a->vertex_offsets || !a->vertex_faces))
        return fail(NR_ERR_ARGS, "missing vertex adjacency (vertex_offsets / vertex_faces)");
    const bool rgb = (a->draw_flags & NR_DRAW_RGB) && grad_textures;
    const bool lit = (a->draw_flags & NR_DRAW_RGB) && a->num_lights > 0;
    const int tex_items = rgb ? (a->tex_stride_b ? a->batch_size : 1) : 0;
    // texel indices of the backward's direct samples ride in a 32-bit field (nr_bwd.h POS_DIRECT)
    // (and a row at most DIRECT_OFF - 1 texels wide: the top-left index of a sample one row above the
    // texture, -W - 1 + x, must stay above -DIRECT_OFF to be encoded)
    if (rgb && ((long long)a->tex_height * a->tex_width > DIRECT_MAX_HW || a->tex_width >= DIRECT_OFF))
        return fail(NR_ERR_ARGS, "texture gradient: at most %d texels per texture and %d per row (got %d x %d)",
                    DIRECT_MAX_HW, DIRECT_OFF - 1, a->tex_height, a->tex_width);
    // shared texture windows into private copies (NrRasterArgs.face_hot): a texture and texture
    // coordinates shared by the batch
    // (the plain textured backward only: no lights, no backgrounds -- their instantiations have no
    // shared-window flush -- and rgb drawn)
    const bool hot = rgb && tex_items == 1 && a->face_hot && a->num_hot > 0 && !a->vt_batch_stride && !lit &&
                     !a->backgrounds;
    if (hot && (a->num_hot > NR_HOT_MAX || !a->hot_acc || ((uintptr_t)a->hot_acc & 15)))
        return fail(NR_ERR_ARGS, "face_hot: num_hot %d (at most %d) needs a 16-byte aligned hot_acc", a->num_hot, NR_HOT_MAX);
    const size_t need = nr_backward_workspace_bytes(a->batch_size, a->num_faces, a->num_vertices, tex_items,
                                                    a->tex_height, a->tex_width, lit ? a->num_lights : 0);
    if (need > 0 && (!workspace || workspace_bytes < need))
        return fail(NR_ERR_WORKSPACE, "backward workspace missing or too small");
    hipStream_t st = (hipStream_t)stream;
    const int S = a->anti_aliasing ? 2 * a->image_size : a->image_size;
    Geom g = make_geom(a->num_faces, S);
    const bool hot_texels = rgb && !a->tex_stride_b &&
                            (long long)a->tex_height * a->tex_width > BWD_HOT_TEXELS_PER_FACE * a->num_faces;
    g.group = group_for(a->batch_size, hot_texels ? BWD_GROUP_TEX : BWD_GROUP);
    const int HW = a->tex_height * a->tex_width;
    const int HWp = (HW + 3) & ~3;
    char* w = (char*)workspace;
    float* gF = (float*)w;
    w += align_up((size_t)a->batch_size * a->num_faces * 9 * 4);
    float* g4 = rgb ? (float*)w : nullptr;
    if (rgb) w += align_up((size_t)tex_items * HWp * 16);
    float* gN = lit ? (float*)w : nullptr;
    float* gU = lit ? (float*)(w + align_up((size_t)a->batch_size * a->num_faces * 9 * 4)) : nullptr;
    // gU is fully written by k_vnormal_bwd; the accumulators before it start at zero
    const size_t zero_bytes = lit ? (size_t)((char*)gU - (char*)workspace) : need;
    // ... unless the caller states, for this call, that the forward zeroed them (NrRasterArgs.bwd_workspace)
    const bool prezeroed = workspace_zeroed != 0;
    if (prezeroed && zero_bytes > 0 && (a->bwd_workspace != workspace || a->bwd_workspace_bytes < zero_bytes))
        return fail(NR_ERR_ARGS, "workspace_zeroed = 1 needs args->bwd_workspace == workspace with at least %zu bytes "
                                 "(the buffer the forward zeroed)", zero_bytes);
    if (zero_bytes > 0 && !prezeroed && hipMemsetAsync(workspace, 0, zero_bytes, st) != hipSuccess)
        return check_launch("hipMemsetAsync");
    if (hot) {
        // hot_acc starts at zero: the forward zeroed it when it lies inside the zeroed bwd_workspace
        const size_t hb = nr_hot_acc_bytes(a->num_hot);
        const char* hz = (const char*)a->hot_acc;
        const bool in_zeroed = prezeroed && hz >= (const char*)a->bwd_workspace &&
                               hz + hb <= (const char*)a->bwd_workspace + a->bwd_workspace_bytes;
        if (!in_zeroed && hipMemsetAsync(a->hot_acc, 0, hb, st) != hipSuccess) return check_launch("hipMemsetAsync");
    }
    BwdArgs ba;
    ba.face_records = a->face_records;
    ba.fim = a->face_index;
    ba.grad_images = grad_images;
    ba.grad_faces = gF;
    ba.grad_tex = g4;
    ba.halo = a->halo;
    ba.binfg = a->halo ? (const uint8_t*)a->halo + halo_flags_offset_bytes(a->batch_size, S, nr_num_channels(a->draw_flags))
                       : nullptr;
    ba.grad_normals = gN;
    ba.grad_bg = (a->draw_flags & NR_DRAW_RGB) && a->backgrounds ? a->grad_backgrounds : nullptr;
    ba.F = a->num_faces;
    ba.aa = a->anti_aliasing;
    ba.s = a->image_size;
    ba.HW = HW;
    ba.HWp = HWp;
    ba.step = (float)(2. / S);
    ba.inv_step = 1.f / ba.step;
    ba.step_pow2 = (S & (S - 1)) == 0;  // step = 2/S is then a power of two: x / step == x * (S / 2)
    ba.face_hot = hot ? a->face_hot : nullptr;
    ba.num_hot = hot ? a->num_hot : 0;
    ba.hot_acc = hot ? a->hot_acc : nullptr;
    Shade sh = make_shade(a);
    {
        ProfScope _p(P_BWD, st, !hot);
        const dim3 grid(((S + TW - 1) / TW) * ((S + BH - 1) / BH), a->batch_size);
        const bool silo = !(a->draw_flags & (NR_DRAW_RGB | NR_DRAW_DEPTH));  // lights / backgrounds need rgb
        switch ((lit ? 1 : 0) | (sh.bg ? 2 : 0) | (silo ? 4 : 0)) {
            case 0: launch_bwd<0>(grid, st, ba, g, sh); break;
            case 1: launch_bwd<1>(grid, st, ba, g, sh); break;
            case 2: launch_bwd<2>(grid, st, ba, g, sh); break;
            case 3: launch_bwd<3>(grid, st, ba, g, sh); break;
            default: launch_bwd<4>(grid, st, ba, g, sh); break;
        }
        e = check_launch("k_raster_bwd");
        if (e) return e;
        // the shared windows' private copies, summed (timed with k_raster_bwd, whose window flushes they
        // complete; bench.py counts their bytes there), before the texture-gradient output (k_vertex_grad
        // / k_tex_out) reads the accumulator
        if (hot) {
            nr_launch(k_hot_reduce, dim3((unsigned)a->num_hot), dim3(64), 0, st, a->hot_acc, a->num_hot, g4,
                               a->tex_width, a->tex_height);
            e = check_launch("k_hot_reduce");
            if (e) return e;
        }
    }
    const long long nv = (long long)a->batch_size * a->num_vertices;
    if (lit && nv > 0) {
        // lights: vertex-normal gradients -> face normals -> corner gradients (added into gF)
        nr_launch(k_vnormal_bwd, dim3((unsigned)((nv + 255) / 256)), dim3(256), 0, st, gN, a->vertex_offsets,
                           a->vertex_faces, a->vertex_normals, gU, a->num_faces, a->num_vertices, nv);
        e = check_launch("k_vnormal_bwd");
        if (e) return e;
        const long long nf = (long long)a->batch_size * a->num_faces;
        if (nf > 0) {
            nr_launch(k_fnormal_bwd, dim3((unsigned)((nf + 255) / 256)), dim3(256), 0, st, a->face_records,
                               a->faces, gU, gF, a->num_faces, a->num_vertices, nf);
            e = check_launch("k_fnormal_bwd");
            if (e) return e;
        }
    }
    TexOut to{};
    if (rgb) to = TexOut{g4, grad_textures, HW, HWp, (long long)tex_items * HW};
    // k_vertex_grad's blocks also carry the texture-gradient output when that is a few texels per
    // thread; otherwise (no vertices, or a large texture) it gets a launch of its own
    constexpr int VB = 256;  // small blocks: more of them in flight for this latency-bound gather
    // items on XCDs (k_vertex_grad): a multiple of 8 items
    const int xcd_items = a->batch_size % 8 == 0 && a->num_vertices > 0;
    const long long vblocks = xcd_items ? (long long)a->batch_size * ((a->num_vertices + VB - 1) / VB) : (nv + VB - 1) / VB;
    const long long vgrad_threads = vblocks * VB;
    // (up to 16 texels per thread: the car's texture-gradient output rides on its k_vertex_grad blocks,
    // 0.022 + 0.0135 -> 0.031 ms; at 8 it had a launch of its own; same-box A/B, gpurun_out/o28)
    const bool carry = nv > 0 && to.n <= 16 * vgrad_threads;
#ifdef NR_ABL_EXTRAK
    nr_launch(k_abl_empty, dim3(NR_ABL_EXTRAK), dim3(256), 0, st, 0);
#endif
#ifdef NR_ABL_NOVGRAD
    if (false) {
#else
    if (nv > 0) {
#endif
        {
            ProfScope _p(P_VGRAD, st, true);
            nr_launch(k_vertex_grad, dim3((unsigned)vblocks), dim3(VB), 0, st, gF, a->vertex_offsets,
                               a->vertex_faces, grad_vertices, a->num_faces, a->num_vertices, nv, carry ? to : TexOut{},
                               xcd_items);
        }
        e = check_launch("k_vertex_grad");
        if (e) return e;
    }
    if (to.out && to.n > 0 && !carry) {
        {
            ProfScope _p(P_TEXOUT, st, true);
            nr_launch(k_tex_out, dim3((unsigned)((to.n + 255) / 256)), dim3(256), 0, st, to);
        }
        e = check_launch("k_tex_out");
    }
    return e;
}

int nr_rasterize_backward_params(const NrRasterArgs* a, const float* grad_images, float* grad_vertices_textures,
                                 float* grad_lights, void* stream) {
    int e = validate_raster(a, false);
    if (e) return e;
    const bool rgb = (a->draw_flags & NR_DRAW_RGB) != 0;
    const bool uv = rgb && grad_vertices_textures, lgt = rgb && grad_lights && a->num_lights > 0;
    if ((grad_vertices_textures || grad_lights) && !rgb) return fail(NR_ERR_ARGS, "parameter gradients need NR_DRAW_RGB");
    if (a->face_index_sparse && (grad_vertices_textures || grad_lights))
        return fail(NR_ERR_ARGS, "parameter gradients read every face id: the forward must not use face_index_sparse");
    if (grad_lights && a->num_lights > 0 && !a->vertex_normals) return fail(NR_ERR_ARGS, "lights need vertex_normals");
    hipStream_t st = (hipStream_t)stream;
    const int B = a->batch_size;
    const long long gvt_bstride = (long long)a->num_vertices_textures * 2;
    if (uv) {
        const size_t n = (size_t)(a->vt_batch_stride ? B : 1) * gvt_bstride * sizeof(float);
        if (n && hipMemsetAsync(grad_vertices_textures, 0, n, st) != hipSuccess) return check_launch("hipMemsetAsync");
    }
    if (lgt) {
        const size_t n = (size_t)a->num_lights * B * NR_LIGHT_FLOATS * sizeof(float);
        if (n && hipMemsetAsync(grad_lights, 0, n, st) != hipSuccess) return check_launch("hipMemsetAsync");
    }
    if (B == 0 || a->num_faces == 0 || !(uv || lgt)) return NR_OK;
    if (!grad_images) return fail(NR_ERR_ARGS, "null grad_images");
    const int S = a->anti_aliasing ? 2 * a->image_size : a->image_size;
    BwdArgs ba = {};
    ba.face_records = a->face_records;
    ba.fim = a->face_index;
    ba.grad_images = grad_images;
    ba.F = a->num_faces;
    ba.aa = a->anti_aliasing;
    ba.s = a->image_size;
    const Shade sh = make_shade(a);  // the lights shade (cw) the uv gradient even without light gradients
    const dim3 grid((unsigned)(((long long)S * S + 255) / 256), B);
    if (uv && lgt)
        nr_launch((k_param_bwd<true, true>), grid, dim3(256), 0, st, ba, sh, S, a->faces_textures,
                           grad_vertices_textures, gvt_bstride, grad_lights);
    else if (uv)
        nr_launch((k_param_bwd<true, false>), grid, dim3(256), 0, st, ba, sh, S, a->faces_textures,
                           grad_vertices_textures, gvt_bstride, grad_lights);
    else
        nr_launch((k_param_bwd<false, true>), grid, dim3(256), 0, st, ba, sh, S, a->faces_textures,
                           grad_vertices_textures, gvt_bstride, grad_lights);
    return check_launch("k_param_bwd");
}

static int validate_camera(const NrCameraArgs* c) {
    if (!c) return fail(NR_ERR_ARGS, "null camera args");
    if (c->batch_size < 0 || c->num_vertices < 0) return fail(NR_ERR_ARGS, "bad sizes B=%d V=%d", c->batch_size, c->num_vertices);
    if (c->mode != NR_CAMERA_NONE && c->mode != NR_CAMERA_LOOK_AT) return fail(NR_ERR_ARGS, "bad camera mode %d", c->mode);
    if ((long long)c->batch_size * c->num_vertices > 0 && !c->vertices) return fail(NR_ERR_ARGS, "null vertices");
    if (c->mode == NR_CAMERA_LOOK_AT && c->batch_size > 0 && !c->eye) return fail(NR_ERR_ARGS, "null eye");
    return NR_OK;
}

size_t nr_camera_workspace_bytes(int batch_size) { return batch_size > 0 ? align_up((size_t)batch_size * 12 * 4) : 0; }

int nr_camera_forward(const NrCameraArgs* c, float* out, void* stream) {
    int e = validate_camera(c);
    if (e) return e;
    const long long n = (long long)c->batch_size * c->num_vertices;
    if (n == 0) return NR_OK;
    if (!out) return fail(NR_ERR_ARGS, "null output");
    nr_launch(k_camera_fwd, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, *c, out);
    return check_launch("k_camera_fwd");
}

int nr_camera_backward(const NrCameraArgs* c, const float* grad_out, float* grad_vertices, float* grad_eye,
                       void* workspace, size_t workspace_bytes, void* stream) {
    int e = validate_camera(c);
    if (e) return e;
    hipStream_t st = (hipStream_t)stream;
    const bool want_eye = grad_eye && c->mode == NR_CAMERA_LOOK_AT;
    const int neye = c->eye_batch_stride ? c->batch_size : 1;
    if (grad_eye && !want_eye) {  // no eye in the transform: zero gradient
        if (hipMemsetAsync(grad_eye, 0, (size_t)neye * 3 * 4, st) != hipSuccess) return check_launch("hipMemsetAsync");
        grad_eye = nullptr;
    }
    const long long nv = (long long)(c->v_batch_stride ? c->batch_size : 1) * c->num_vertices;
    if (c->batch_size == 0) {
        if (grad_vertices && nv > 0 && hipMemsetAsync(grad_vertices, 0, (size_t)nv * 12, st) != hipSuccess)
            return check_launch("hipMemsetAsync");
        if (want_eye && hipMemsetAsync(grad_eye, 0, (size_t)neye * 12, st) != hipSuccess) return check_launch("hipMemsetAsync");
        return NR_OK;
    }
    if (!grad_out && (grad_vertices || want_eye)) return fail(NR_ERR_ARGS, "null grad_out");
    float* acc = nullptr;
    if (want_eye) {
        if (!workspace || workspace_bytes < nr_camera_workspace_bytes(c->batch_size))
            return fail(NR_ERR_WORKSPACE, "camera workspace missing or too small");
        acc = (float*)workspace;
        if (hipMemsetAsync(acc, 0, (size_t)c->batch_size * 12 * 4, st) != hipSuccess) return check_launch("hipMemsetAsync");
    }
    if ((grad_vertices || acc) && nv > 0) {
        nr_launch(k_camera_bwd, dim3((unsigned)((nv + 255) / 256)), dim3(256), 0, st, *c, grad_out, grad_vertices, acc);
        e = check_launch("k_camera_bwd");
        if (e) return e;
    }
    if (want_eye) {
        if (nv == 0 && hipMemsetAsync(acc, 0, (size_t)c->batch_size * 12 * 4, st) != hipSuccess) return check_launch("hipMemsetAsync");
        nr_launch(k_camera_eye, dim3((unsigned)((neye + 63) / 64)), dim3(64), 0, st, *c, acc, grad_eye);
        e = check_launch("k_camera_eye");
    }
    return e;
}

int nr_selftest_division(const float* a, const float* b, float* q_fast, float* q_ieee, long long n, void* stream) {
    if (n < 0 || (n > 0 && (!a || !b || !q_fast || !q_ieee))) return fail(NR_ERR_ARGS, "bad arguments");
    if (n == 0) return NR_OK;
    nr_launch(k_selftest_div, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, a, b,
                       q_fast, q_ieee, n);
    return check_launch("k_selftest_div");
}

#ifdef NR_FWD_TIMING
// timing builds only: the fused forward's per-wave phase timestamps (g_fwd_t)
__attribute__((visibility("default"))) int nr_debug_fwd_timing(unsigned long long* out, size_t n) {
    if (n > (size_t)NR_FTIMING_MAX) n = NR_FTIMING_MAX;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fwd_t), n * sizeof(unsigned long long), 0, hipMemcpyDeviceToHost) != hipSuccess)
        return fail(NR_ERR_LAUNCH, "hipMemcpyFromSymbol failed");
    return NR_OK;
}
#endif
#ifdef NR_COUNT_DIRECT
__attribute__((visibility("default"))) int nr_debug_counts(unsigned long long* out) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ncount), 4 * sizeof(unsigned long long), 0, hipMemcpyDeviceToHost) != hipSuccess)
        return fail(NR_ERR_LAUNCH, "hipMemcpyFromSymbol failed");
    return NR_OK;
}
#endif
#ifdef NR_BWD_TIMING
// timing builds only: the backward's per-wave phase timestamps (g_bwd_t), n entries to host memory
__attribute__((visibility("default"))) int nr_debug_bwd_timing(unsigned long long* out, size_t n) {
    if (n > (size_t)NR_TIMING_MAX) n = NR_TIMING_MAX;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_bwd_t), n * sizeof(unsigned long long), 0, hipMemcpyDeviceToHost) != hipSuccess)
        return fail(NR_ERR_LAUNCH, "hipMemcpyFromSymbol failed");
    return NR_OK;
}
#endif

int nr_last_launch(const char* kernel, int* block_threads, int* flags) {
    if (!kernel || !block_threads || !flags) return fail(NR_ERR_ARGS, "null argument");
    const LaunchSlot* slot = strcmp(kernel, "k_raster_fwd") == 0 ? &g_last_fwd
                             : strcmp(kernel, "k_raster_bwd") == 0 ? &g_last_bwd : nullptr;
    if (!slot) return fail(NR_ERR_ARGS, "nr_last_launch: unknown kernel name %s", kernel);
    const LaunchRec r = slot->load();
    if (!r.threads) return fail(NR_ERR_ARGS, "nr_last_launch: no %s launch recorded in this process", kernel);
    *block_threads = r.threads;
    *flags = r.flags;
    return NR_OK;
}

int nr_profile_enable(int on) {
    if (on && !g_prof) {
        for (int k = 0; k < P_N; k++)
            for (int r = 0; r < PROF_RING; r++)
                for (int j = 0; j < 2; j++)
                    if (hipEventCreate(&g_prof_ev[k][r][j]) != hipSuccess) return fail(NR_ERR_LAUNCH, "hipEventCreate failed");
    } else if (!on && g_prof) {
        for (int k = 0; k < P_N; k++)
            for (int r = 0; r < PROF_RING; r++)
                for (int j = 0; j < 2; j++) (void)hipEventDestroy(g_prof_ev[k][r][j]);
    }
    // (re)enabling starts a new measurement: the ring's recorded launches are forgotten
    for (int k = 0; k < P_N; k++) g_prof_n[k] = 0;
    g_prof = on != 0;
    return NR_OK;
}

#ifdef NR_COUNT_TESTS
int nr_count_read(unsigned long long* out4, int reset) {
    if (!out4) return fail(NR_ERR_ARGS, "null argument");
    if (hipMemcpyFromSymbol(out4, HIP_SYMBOL(g_fwd_count), 4 * sizeof(unsigned long long)) != hipSuccess)
        return fail(NR_ERR_LAUNCH, "nr_count_read: hipMemcpyFromSymbol failed");
    if (reset) {
        const unsigned long long z[4] = {0, 0, 0, 0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_fwd_count), z, sizeof(z)) != hipSuccess)
            return fail(NR_ERR_LAUNCH, "nr_count_read: hipMemcpyToSymbol failed");
    }
    return NR_OK;
}
#endif

int nr_profile_read(const char* kernel, float* ms) {
    if (!kernel || !ms) return fail(NR_ERR_ARGS, "null argument");
    for (int k = 0; k < P_N; k++) {
        if (strcmp(kernel, kProfNames[k]) != 0) continue;
        if (!g_prof || g_prof_n[k] == 0) return fail(NR_ERR_ARGS, "%s: no profiled launch recorded", kernel);
        const int n = g_prof_n[k] < PROF_RING ? g_prof_n[k] : PROF_RING;
        double sum = 0.0;
        for (int r = 0; r < n; r++) {
            float e = 0.f;
            if (hipEventElapsedTime(&e, g_prof_ev[k][r][0], g_prof_ev[k][r][1]) != hipSuccess)
                return fail(NR_ERR_LAUNCH, "%s: hipEventElapsedTime failed", kernel);
            sum += e;
        }
        *ms = (float)(sum / n);
        return NR_OK;
    }
    return fail(NR_ERR_ARGS, "unknown kernel name %s", kernel);
}

}  // extern "C"
