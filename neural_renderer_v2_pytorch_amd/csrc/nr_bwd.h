// nr_bwd.h -- backward: k_raster_bwd, k_vertex_grad (lights), normal backward, k_param_bwd
// Part of nr_raster.hip (one translation unit); see that file and DESIGN.md.
#pragma once

#pragma clang fp contract(off)

namespace {

// ------------------------------------------------------------------------------------------------
// k_raster_bwd: one block per 32x16 pixels + 1-pixel halo; each wave owns a 16x8 block, 2 pixels per
// lane.
//   1. recompute the internal image I (all channels, bit-identical to the forward) and the upstream
//      gradient G of the block + halo into LDS (Differentiation saved the images; the flip/AA
//      backward is an index map and /4), and for the block's own pixels the gradient terms that do
//      not depend on the stencil (depth and texture-coordinate paths to z, bilinear weights);
//   2. the soft-gradient stencil (gx, gy) of Differentiation.backward from per-pair dot products (each
//      neighbour pair computed once, in LDS, for both its pixels), then the coordinate-map chain
//      rule -> a 9-float gradient of the gathered face (rasterize.py:232);
//   3. reduction without LDS float atomics (ds_add_f32 runs at ~3 cycles per lane on gfx950,
//      tools/ubench_lds_atomics.hip): each lane stages its two pixel records in LDS; the wave groups
//      its records by face (ballot match loop); for each face, lanes 0..47 own the 4x4 texel x RGB
//      window of the face and lanes 48..56 its 9 gradient floats, and sum over the face's records;
//   4. one global float atomic per lane and face: a whole face record and whole 4-texel RGBA rows,
//      i.e. a handful of 64-byte requests per (face, wave).
//   Texel contributions outside a face's 4x4 window (atlases with larger per-face texture regions)
//   go straight to global atomics in step 1.
constexpr int BH = 16;                        // block height
constexpr int HW_ = TW + 2, HH_ = BH + 2, HN = HW_ * HH_;
constexpr int NHALO = 2 * HW_ + 2 * BH;       // 100 halo pixels
constexpr int TWIN = 4;                       // texel window edge per face
// pos of a pixel without a window texel: tt - POS_NONE is 16..31 for every window texel tt, so the
// gather's footprint test (0x33 >> (d & 31)) & 1 rejects it with no separate check
constexpr int POS_NONE = -16;
// a texture sample outside its face's window (step 1: large atlases, e.g. ShapeNet image textures)
// keeps its top-left texel's flat index in `pos` as POS_DIRECT - 32 (index + DIRECT_OFF): again 16
// mod 32, so the gather rejects it too, and after the gather the wave adds it to the texel
// accumulator four samples per atomic instruction (step 5)
constexpr int POS_DIRECT = -48;
constexpr int DIRECT_OFF = 1 << 22;
constexpr int DIRECT_MAX_HW = 1 << 25;  // texels per texture with a gradient (nr_rasterize_backward checks)
__device__ __forceinline__ int direct_pos(int base) {
    return POS_DIRECT - 32 * min(max(base + DIRECT_OFF, 0), DIRECT_MAX_HW + DIRECT_OFF);
}
__device__ __forceinline__ int direct_base(int pos) { return ((POS_DIRECT - pos) >> 5) - DIRECT_OFF; }

// staged record: ay by ax bx | G_rgb[3] pos | gF[9] | pad (20 floats); with lights also dL/dnormal[3]
// and the weights w[3] at 17..22 (24 floats)
template <bool LIT> constexpr int srec() { return LIT ? 24 : 20; }
constexpr int BWD_LDS_IG = 2 * MAXC * HN * 4;
constexpr int BWD_LDS_HALO = 2 * MAXC * 128 * 4;  // halo staging (step 0), after the I / G planes
template <bool LIT> constexpr int bwd_lds() {
    return BWD_LDS_IG + BWD_LDS_HALO > 4 * 128 * srec<LIT>() * 4 ? BWD_LDS_IG + BWD_LDS_HALO : 4 * 128 * srec<LIT>() * 4;
}
static_assert(BWD_LDS_IG % 16 == 0, "halo staging alignment");

// per-wave phase timestamps (timing builds only, tools/bwd_timing.py): lane 0 of every wave of the
// 2-pixel variant records the shader clock at 8 points of its life
#ifdef NR_BWD_TIMING
constexpr long long NR_TIMING_MAX = 1 << 23;
constexpr int NR_BSLOTS = 10;  // per wave: 8 phase slots, then the wall clock (100 MHz, chip-wide) at entry and exit
__device__ unsigned long long g_bwd_t[NR_TIMING_MAX];
#define NR_TSTAMP(k)                                                                                       \
    do {                                                                                                   \
        const long long i_ = (((long long)blockIdx.y * gridDim.x + blockIdx.x) * (blockDim.x / 64) + (threadIdx.x >> 6)) * NR_BSLOTS + (k); \
        const unsigned long long t_ = clock64();                                                           \
        if ((threadIdx.x & 63) == 0 && i_ < NR_TIMING_MAX) g_bwd_t[i_] = t_;                                 \
    } while (0)
#else
#define NR_TSTAMP(k) \
    do {             \
    } while (0)
#endif
#ifdef NR_BWD_TIMING
#define NR_WSTAMP(k)                                                                                         \
    do {                                                                                                     \
        const long long i_ = (((long long)blockIdx.y * gridDim.x + blockIdx.x) * (blockDim.x / 64) + (threadIdx.x >> 6)) * NR_BSLOTS + (k); \
        const unsigned long long t_ = wall_clock64();                                                      \
        if ((threadIdx.x & 63) == 0 && i_ < NR_TIMING_MAX) g_bwd_t[i_] = t_;                                 \
    } while (0)
#else
#define NR_WSTAMP(k) \
    do {             \
    } while (0)
#endif

struct BwdArgs {
    const float* __restrict__ face_records;
    const int32_t* __restrict__ fim;
    const float* __restrict__ grad_images;
    float* __restrict__ grad_faces;   // [B, F, 9] face-corner accumulator
    // texture gradient: a zero-filled accumulator of RGBA rows [Bt, HWp, 4] (or null) that
    // k_vertex_grad / k_tex_out transpose into the [Bt, 3, H, W] output; a face's 4x4 window is 4
    // cache-line rows, a direct sample's 2x2 footprint two 32-B segments
    float* __restrict__ grad_tex;
    int HWp;
    const float* __restrict__ halo;   // halo cache written by the forward, or null (re-shade the halo)
    const uint8_t* __restrict__ binfg; // per (item, 32x32 bin) foreground flags after the halo values, or null
    float* __restrict__ grad_normals; // [B, F, 9] per-face corner vertex-normal gradients (lights)
    float* __restrict__ grad_bg;      // [B, 3, S, S] or null
    int F, aa, s, HW;
    float step, inv_step;
    int step_pow2;                     // x / step == x * inv_step exactly
    // shared texture windows (NrRasterArgs.face_hot): the window sums of a face with face_hot >= 0 go
    // to private copy (block % NR_HOT_COPIES) of its window in hot_acc, which k_hot_reduce adds into
    // grad_tex after the kernel; null: every window into grad_tex directly
    const int32_t* __restrict__ face_hot;
    int num_hot;
    float* __restrict__ hot_acc;
};
// hot_acc: [NR_HOT_COPIES][num_hot][16 texels][4] window sums, then [num_hot][2] window origins
__device__ __host__ inline size_t hot_sums_floats(int num_hot) { return (size_t)NR_HOT_COPIES * num_hot * 64; }

// upstream gradient of internal pixel (x, y): the flip / 2x2-mean backward is an index map and /4.
// gi: this item's [C, s, s] upstream gradient (32-bit offsets inside it)
// The MAXC loads are unconditional (channel min(c, C - 1), in bounds) and issued together: a load
// under the runtime `c < C` branch had its wait inside the branch, which serialised the channels'
// HBM round trips.  x / 4 == x * 0.25 exactly (power-of-two scale).
__device__ __forceinline__ void upstream_load(const BwdArgs& a, const float* __restrict__ gi, int C, int y, int x, int S,
                                              float* raw) {
    const int s = a.s;
    const int plane = a.aa ? s * s : S * S;
    // 24-bit multiplies (sizes < 2^24): a 64-bit v_mad_u64_u32 here reads an undefined high half
    // that the compiler's wait insertion treats as a use of an in-flight load's destination
    const int o = a.aa ? (int)__umul24((S - 1 - y) >> 1, s) + ((S - 1 - x) >> 1) : (int)__umul24(S - 1 - y, S) + (S - 1 - x);
#pragma unroll
    for (int c = 0; c < MAXC; c++) raw[c] = gi[min(c, C - 1) * plane + o];
}
__device__ __forceinline__ void upstream_scale(const BwdArgs& a, int C, const float* raw, float* G) {
    const float scale = a.aa ? 0.25f : 1.f;
#pragma unroll
    for (int c = 0; c < MAXC; c++) G[c] = c < C ? raw[c] * scale : 0.f;
}
__device__ __forceinline__ void upstream_grad(const BwdArgs& a, const float* __restrict__ gi, int C, int y, int x, int S,
                                              float* G) {
    float raw[MAXC];
    upstream_load(a, gi, C, y, x, S, raw);
    upstream_scale(a, C, raw, G);
}

__device__ __forceinline__ float upstream_one(const BwdArgs& a, const float* __restrict__ gi, int y, int x, int S, int c) {
    if (a.aa) {
        const int s = a.s;
        return gi[c * s * s + ((S - 1 - y) >> 1) * s + ((S - 1 - x) >> 1)] / 4.f;
    }
    return gi[c * S * S + (S - 1 - y) * S + (S - 1 - x)];
}

__device__ __forceinline__ float div_step(const BwdArgs& a, float x) { return a.step_pow2 ? x * a.inv_step : x / a.step; }

// sum_c d[c] g[c] in channel order, as pair_dot (nr_shade.h) forms it from its differences
__device__ __forceinline__ float diff_dot(const float* d, const float* g, int C) {
    float s = d[0] * g[0];
#pragma unroll
    for (int c = 1; c < MAXC; c++)
        if (c < C) s = s + d[c] * g[c];
    return s;
}
// Differentiation.backward's stencil at position i of n along one axis (axis_grad, nr_shade.h), from
// its two neighbour pairs' channel dot products: p = (dp . G(i + 1), dp . G(i)) of the pair (i, i + 1)
// and m = the same of the pair (i - 1, i), with dp = I(first) - I(second).  axis_grad's one-sided
// terms are these exactly: -pair_dot(Ip, I0, G0) = -sum (-dp) G0 = sum dp G0 (negation is exact and
// round-to-nearest is symmetric), and its (i - 1, i) terms are the left pair's; only the sign of an
// all-zero sum can differ, which no caller observes (pick_grad compares, and it is added to gF).  Each
// pair is computed once and serves both of its pixels (k_raster_bwd step 2).
__device__ __forceinline__ float stencil_pair(const BwdArgs& a, float2 p, float2 m, int i, int n) {
    const bool has_p = i <= n - 2, has_m = i >= 1;
    const float r_i = has_p ? div_step(a, -p.x) : 0.f;
    const float r_m = has_m ? div_step(a, -m.x) : 0.f;
    const float l_i = has_p ? div_step(a, p.y) : 0.f;
    const float l_m = has_m ? div_step(a, m.y) : 0.f;
    return pick_grad(r_i + r_m, l_m + l_i);
}

__device__ __forceinline__ float frcp(float x) { return __builtin_amdgcn_rcpf(x); }

// position (hy, hx) in the (BH + 2) x (TW + 2) tile frame of halo pixel t < NHALO: top row, bottom
// row, left column, right column
__device__ __forceinline__ void halo_pixel(int t, int& hy, int& hx) {
    if (t < HW_) { hy = 0; hx = t; }
    else if (t < 2 * HW_) { hy = HH_ - 1; hx = t - HW_; }
    else if (t < 2 * HW_ + BH) { hy = 1 + (t - 2 * HW_); hx = 0; }
    else { hy = 1 + (t - 2 * HW_ - BH); hx = HW_ - 1; }
}

// Values (v0, v1, v2, v3) held by every lane; lane l ends with v_c summed over the four lanes
// l & 15 + 16 k, where c = l >> 4.  v_permlane32_swap(A, B) leaves [A_lo | B_lo] and [A_hi | B_hi]
// (32-lane halves), so their sum is A summed over the halves in the low half and B in the high
// half; v_permlane16_swap does the same for 16-lane rows.
__device__ __forceinline__ float chunk_reduce_scatter(float v0, float v1, float v2, float v3) {
    const auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(v0), __float_as_uint(v2), false, false);
    const float b0 = __uint_as_float(p[0]) + __uint_as_float(p[1]);  // rows 0,1: v0; rows 2,3: v2
    const auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(v1), __float_as_uint(v3), false, false);
    const float b1 = __uint_as_float(q[0]) + __uint_as_float(q[1]);  // rows 0,1: v1; rows 2,3: v3
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(b0), __float_as_uint(b1), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);           // row c: v_c
}

#ifdef NR_COUNT_DIRECT
__device__ unsigned long long g_ncount[4];  // debug builds: windowed / direct samples, direct without a window
#endif
// per interior pixel state carried across the stencil's barrier
struct BwdPix {
    int fi;            // face index (-1: background or outside)
    float w[3];        // barycentric weights (compute_weight_map)
    float gz[3];       // d/dz of the face corners through the depth and texture-coordinate paths
    float grgb[3];     // upstream gradient of the rgb channels
    float ay, by, ax, bx;
    int pos;           // bilinear top-left texel relative to the face window: dx + 4 dy; POS_NONE none
    int wx, wy;        // face window origin (texels); INT_MIN when not windowed
    float gn[3];       // lights: dL/d(smooth normal)
};

// FEAT: 1 = lights, 2 = backgrounds, 4 = silhouettes only (separate instantiations keep the plain path lean)
// NPX: pixels per lane (2: 256 threads, a wave = 16x8 pixels; 1: 512 threads, a wave = 16x4 pixels,
// at 6 waves/SIMD)
// CC: the channel count as a compile-time constant (0: sh.C at run time).  With every channel present
// (rgb + sil + depth, C = MAXC) the per-channel `c < C` guards of the loads, the LDS staging and the
// stencil fold away, with their zero defaults and scalar branches; that instantiation is launched
// only with anti-aliasing and a power-of-two raster (both folded too).
// HOT: the shared-window flush (BwdArgs.face_hot) compiled in; its instantiations run only when the
// caller passes face_hot (its per-face id load and address select cost the headline's backward 4 %,
// 0.194 -> 0.202 ms, when compiled into the plain instantiation, gpurun_out/nh)
#ifdef NR_ABL_S1LOAD
__device__ float4* g_abl_prod;  // timing builds only: the per-pixel product planes (zeroed)
#endif
template <int FEAT, int NPX, int CC = 0, bool HOT = false>
__global__ __launch_bounds__(2 * NT / NPX) __attribute__((amdgpu_waves_per_eu((FEAT & 1) ? 3 : (NPX == 1 ? 6 : 4), 8))) void k_raster_bwd(BwdArgs a, Geom g, Shade sh_in) {
    constexpr bool LIT = (FEAT & 1) != 0, BG = (FEAT & 2) != 0, SILO = (FEAT & 4) != 0;
    // features this instantiation does not have become compile-time constants (the shared
    // shade_pixel then carries no light / background code or arguments)
    Shade sh = sh_in;
    if (!LIT) sh.nl = 0;
    if (!BG) sh.bg = nullptr;
    if (CC) {
        // CC = MAXC: rgb + sil + depth (the only 5-channel render); CC = 4: rgb + sil (rasterize_rgba,
        // Renderer.render); launched only with anti-aliasing and a power-of-two raster
        sh.draw = static_draw(CC);
        a.aa = 1;
        a.step_pow2 = 1;
    }
    constexpr int REC = srec<LIT>();
    __shared__ __attribute__((aligned(16))) float s_raw[bwd_lds<LIT>() / 4];
    // the tile's image and upstream gradient (+ halo) in LDS, (I_c, G_c) interleaved per pixel in three
    // planes: (I0 G0 I1 G1), (I2 G2 I3 G3), (I4 G4) -- a pixel's ten values are 3 LDS accesses
    // (ds_read_b128 x 2 + ds_read_b64) instead of 10 dword accesses; unused channels hold 0
    static_assert(MAXC == 5, "interleaved I/G planes");
    float4* s_ig01 = reinterpret_cast<float4*>(s_raw);
    float4* s_ig23 = s_ig01 + HN;
    float2* s_ig4 = reinterpret_cast<float2*>(s_ig23 + HN);
    static_assert(HN * (16 + 16 + 8) == BWD_LDS_IG, "I/G planes fill BWD_LDS_IG");
    auto store_ig = [&](int i, const float* I, const float* G) {
        s_ig01[i] = make_float4(I[0], G[0], I[1], G[1]);
        s_ig23[i] = make_float4(I[2], G[2], I[3], G[3]);
        s_ig4[i] = make_float2(I[4], G[4]);
    };
    auto load_ig = [&](int i, float* I, float* G) {
        const float4 a01 = s_ig01[i], a23 = s_ig23[i];
        const float2 a4 = s_ig4[i];
        I[0] = a01.x; G[0] = a01.y; I[1] = a01.z; G[1] = a01.w;
        I[2] = a23.x; G[2] = a23.y; I[3] = a23.z; G[3] = a23.w;
        I[4] = a4.x; G[4] = a4.y;
    };
    const int S = g.S;
    const int C = CC ? CC : sh.C;
    const bool rgb = !SILO && (sh.draw & NR_DRAW_RGB) != 0;
    const bool want_tex = rgb && a.grad_tex != nullptr;
    constexpr bool wlate = SILO;  // silhouettes only: weights after the stencil, sparse gather
    int b, tile_x, tile_y;
    block_item_tile(g.group, (S + TW - 1) / TW, (S + BH - 1) / BH, b, tile_x, tile_y);
    const int tx0 = tile_x * TW;
    const int ty0 = tile_y * BH;
    // a tile with no foreground pixel contributes nothing (every gradient term is per foreground
    // pixel; the halo only feeds foreground pixels' stencils): with the forward's bin flags it ends
    // here.  Backgrounds (BG) get gradient from background pixels, so that instantiation never skips.
    NR_WSTAMP(8);
    if (!BG && a.binfg && a.binfg[(long long)b * g.nbins + (ty0 / COARSE) * g.nbx + tx0 / COARSE] == 0) {
        NR_WSTAMP(9);
        return;
    }
    const int t = threadIdx.x;
    const int lane = t & 63, wid = t >> 6;
    const int bt = sh.tv.sb ? b : 0;
    // per-item bases (uniform, 64-bit); per-pixel offsets below are 32-bit
    const int32_t* __restrict__ fimb = a.fim + (long long)b * S * S;
    const float* __restrict__ gimb = a.grad_images + (long long)b * C * (a.aa ? a.s * a.s : S * S);
    const float* __restrict__ frb = a.face_records + (long long)b * a.F * FACE_REC;
    const float* __restrict__ fuvb = sh.face_uv + (sh.uv_bstride ? (long long)b * sh.uv_bstride : 0);
    float* __restrict__ gFb = a.grad_faces + (long long)b * a.F * 9;
    float* __restrict__ gtb = a.grad_tex ? a.grad_tex + (long long)bt * 4 * a.HWp : nullptr;
    // wave wid owns the 16x8 block at (16 (wid & 1), 8 (wid >> 1)); lane -> (lx, ly0) and (lx, ly0 + 4)
    // lanes 16 c .. 16 c + 15 (member chunk c of the gather, step 3) hold the pixels of parity class
    // (x & 1, y & 1) = (c & 1, c >> 1) of the wave's region (8 x 2 of them per pixel k, rows 4 apart):
    // a face's pixels split about evenly over the four chunks, so its member loop, which runs as
    // long as the fullest chunk, takes fewer steps than with one pixel row per chunk (CPU count on
    // the headline: 5.25 instead of 5.95 per face)
    const int lx = (wid & 1) * 16 + 2 * (lane & 7) + ((lane >> 4) & 1);
    const int ly0 = (wid >> 1) * (4 * NPX) + 2 * ((lane >> 3) & 1) + (lane >> 5);
    const int px = tx0 + lx;
    const float xp = pix_center(px, S);

    // halo ring from the forward's halo cache: asynchronous global -> LDS loads by waves 0 and 1
    // (lane t < NHALO carries halo pixel t, ring order of halo_pixel), landed before the barrier
    // (round 6: dealt to all four waves, 25 each, so that no wave waits at the barrier for two others'
    // moves: backward 0.2021-0.2033 against 0.1995-0.2029 ms, gpurun_out/hs; not kept)
    float(*s_hI)[128] = reinterpret_cast<float(*)[128]>(s_raw + BWD_LDS_IG / 4);
    float(*s_hG)[128] = reinterpret_cast<float(*)[128]>(s_raw + BWD_LDS_IG / 4 + MAXC * 128);
    // the halo pixel's bin flag: the forward writes no halo values for a bin without candidate faces
    // (all 0 there); backgrounds (BG) fill such bins with the background colour, and k_shade writes them
    int h_live = 1;
    auto halo_prefetch = [&]() {
        if (a.halo && t < 128) {
            int hy, hx;
            halo_pixel(t, hy, hx);
            const int hpy = ty0 - 1 + hy, hpx = tx0 - 1 + hx;
            const bool h_in = t < NHALO && hpy >= 0 && hpy < S && hpx >= 0 && hpx < S;
            if (!BG && a.binfg && h_in) h_live = a.binfg[(long long)b * g.nbins + (hpy / COARSE) * g.nbx + hpx / COARSE];
            int hoff = 0, hcs = 0;
            if (h_in) halo_locate(C, S, hpx, hpy, hoff, hcs);
            // opaque copies of the base pointers: keeps the compiler from sharing these address
            // computations with step 1's (which would stretch their live ranges over it)
            const float* hbase = a.halo;
            const float* gbase = a.grad_images;
            asm volatile("" : "+s"(hbase), "+s"(gbase));
            const float* hsrc = hbase + b * halo_item_floats(S, C) + hoff;
            const float* gsrc = gbase + (long long)b * C * (a.aa ? a.s * a.s : S * S);
            if (h_in) gsrc += a.aa ? ((S - 1 - hpy) >> 1) * a.s + ((S - 1 - hpx) >> 1) : (S - 1 - hpy) * S + (S - 1 - hpx);
            const int gplane = a.aa ? a.s * a.s : S * S;
#pragma unroll
            for (int c = 0; c < MAXC; c++) {
                if (c < C) {
                    __builtin_amdgcn_global_load_lds((const void*)(hsrc + c * hcs),
                                                     (void __attribute__((address_space(3)))*)(&s_hI[c][wid * 64]), 4, 0, 0);
                    __builtin_amdgcn_global_load_lds((const void*)(gsrc + c * gplane),
                                                     (void __attribute__((address_space(3)))*)(&s_hG[c][wid * 64]), 4, 0, 0);
                }
            }
        }
    };
    NR_TSTAMP(0);
#ifndef NR_ABL_NOSTENCIL
    halo_prefetch();  // in flight during step 1
#else
    (void)halo_prefetch;
#endif

    // ---- 1. image + upstream gradient (LDS), and the stencil-independent gradient terms ---------
    BwdPix P[NPX];
    float I2[NPX][MAXC], G2[NPX][MAXC];
    // every pixel's face id and upstream gradient loads first, unconditional (clamped in-bounds
    // coordinates) so they are all in flight together; the image-border mask is applied after
    int fiv[NPX];
#pragma unroll
    for (int k = 0; k < NPX; k++) {
        const int cy = min(ty0 + ly0 + 4 * k, S - 1), cx = min(px, S - 1);
        fiv[k] = fimb[(int)__umul24(cy, S) + cx];
        upstream_load(a, gimb, C, cy, cx, S, G2[k]);
    }
#pragma unroll
    for (int k = 0; k < NPX; k++) {
        const int py = ty0 + ly0 + 4 * k;
        const bool inside = px < S && py < S;
        BwdPix& q = P[k];
        q.fi = inside ? fiv[k] : -1;
        q.pos = POS_NONE;
        q.wx = q.wy = INT_MIN;
        q.w[0] = q.w[1] = q.w[2] = 0.f;
        q.gz[0] = q.gz[1] = q.gz[2] = 0.f;
        q.grgb[0] = q.grgb[1] = q.grgb[2] = 0.f;
        q.ay = q.by = q.ax = q.bx = 0.f;
        q.gn[0] = q.gn[1] = q.gn[2] = 0.f;
        float graw[MAXC];
#pragma unroll
        for (int c = 0; c < MAXC; c++) {
            graw[c] = G2[k][c];
            I2[k][c] = 0.f;
        }
        upstream_scale(a, inside ? C : 0, graw, G2[k]);
        if (BG && rgb && inside) {
            // background pixels: rgb = 0 * 0 + 1 * bg (chainer rasterize.py:576); grad of bg = (1 - fg) G
            const float fg = q.fi >= 0 ? 1.f : 0.f;
            if (q.fi < 0) {
                float bgc[3];
                background(sh, b, px, py, S, bgc);
#pragma unroll
                for (int c = 0; c < 3; c++) I2[k][c] = fg * 0.f + (1.f - fg) * bgc[c];
            }
            if (a.grad_bg) {
                float* gb = a.grad_bg + ((long long)b * 3) * S * S + (S - 1 - py) * S + (S - 1 - px);
#pragma unroll
                for (int c = 0; c < 3; c++) gb[c * S * S] = (1.f - fg) * G2[k][c];
            }
        }
    }
#pragma unroll
    for (int k = 0; k < NPX; k++) {
        const int py = ty0 + ly0 + 4 * k;
        BwdPix& q = P[k];
        if (q.fi < 0) continue;
        const float yp = pix_center(py, S);
        const float* G = G2[k];
        if (wlate) {  // silhouettes only: I is (fim >= 0); the weights after the stencil, where needed
            I2[k][0] = 1.f;
            continue;
        }
#if defined(NR_ABL_S1ZERO) || defined(NR_ABL_S1LOAD)
        // timing builds only (the bound of a backward that reads its per-pixel products instead of
        // recomputing them; values are placeholders, not gradients): S1ZERO recomputes nothing, S1LOAD
        // loads 48 B per foreground pixel from a lane-ordered buffer (3 coalesced float4 planes)
        {
            float4 v0 = make_float4(0.f, 0.f, 0.f, 0.f), v1 = v0, v2 = v0;
#ifdef NR_ABL_S1LOAD
            const size_t np = (size_t)gridDim.x * gridDim.y * blockDim.x * NPX;
            const size_t pi = (((size_t)blockIdx.y * gridDim.x + blockIdx.x) * blockDim.x + t) * NPX + k;
            v0 = g_abl_prod[pi];
            v1 = g_abl_prod[np + pi];
            v2 = g_abl_prod[2 * np + pi];
#endif
            const float fh = (float)(q.fi & 255) * (1.f / 255.f);
            q.w[0] = 0.3f + v0.x;
            q.w[1] = 0.3f + v0.y;
            q.w[2] = 0.4f + v0.z;
            I2[k][0] = fh + v0.w;
            I2[k][1] = 1.f - fh + v1.x;
            I2[k][2] = 0.5f * fh + v1.y;
            I2[k][3] = 1.f;
            I2[k][4] = 2.f + fh + v1.z;
            q.ay = 0.5f + v1.w;
            q.by = 0.5f + v2.x;
            q.ax = 0.25f + v2.y;
            q.bx = 0.75f + v2.z;
            q.grgb[0] = G[0];
            q.grgb[1] = G[1];
            q.grgb[2] = G[2];
#pragma unroll
            for (int j = 0; j < 3; j++) q.gz[j] = G[MAXC - 1] * 0.01f * q.w[j] + v2.w;
            if (want_tex) {
                q.wx = (q.fi % 72) * 4;
                q.wy = (q.fi / 72) * 4;
                q.pos = 5;
            }
            continue;
        }
#endif
        Face f = load_face_rec(frb + q.fi * FACE_REC);
        // the texture record with the face record: one round trip for both (unconditional, so that
        // no branch join needs its value: without rgb it reads the face record's first 32 bytes)
        const FaceUV fuv = load_face_uv(rgb ? fuvb + q.fi * 8 : frb + q.fi * FACE_REC);
        __builtin_amdgcn_sched_barrier(0);  // keeps the scheduler from sinking the uv load to its use
        // the exact shortened divisions (DESIGN.md "Numerics") as in the forward: bit-identical
        // values (v28: bwd 0.284 -> 0.279 ms; before the latency fixes of v27-v28 it measured even)
        const bool wfast = face_weights(xp, yp, f, q.w);
        const float* w = q.w;
        float dz[3];  // w_k / z_k, shared by the depth and (FACE_ZQ_EQ faces) the texture sampling
        face_dz(f, w, wfast, dz);
        float r = 0.f, gg = 0.f, bb = 0.f, dep = 0.f;
        if (rgb) {
            TexSample s;
            const float uvs[6] = {fuv.a.x, fuv.a.y, fuv.a.z, fuv.a.w, fuv.b.x, fuv.b.y};
            // lights: rgb = texture * cw, so the texture sees G * cw and cw sees G * texture
            float Gt[3] = {G[0], G[1], G[2]};
            float nrm[3], cw[3];
            if (LIT) {
                pixel_normal(sh, b, q.fi, w, nrm);
                light_weights(sh, b, nrm, cw);
#pragma unroll
                for (int c = 0; c < 3; c++) Gt[c] = G[c] * cw[c];
            }
            // bilinear: images = sum_i wt_i T_i -> textures (staged below) and weights (gw)
            float gw[4];
            sample_texture(f, w, wfast, fuv, sh.tv, bt, sh.eps, s, Gt, gw, dz);
            r = s.rgb[0];
            gg = s.rgb[1];
            bb = s.rgb[2];
            if (LIT) {
                const float gcw[3] = {G[0] * r, G[1] * gg, G[2] * bb};
                float cw2[3];
                light_weights(sh, b, nrm, cw2, gcw, q.gn);
                r = r * cw[0];
                gg = gg * cw[1];
                bb = bb * cw[2];
            }
            if (BG) {  // foreground: 1 * rgb + 0 * bg, as the forward computes it
                float bgc[3];
                background(sh, b, px, py, S, bgc);
                r = 1.f * r + 0.f * bgc[0];
                gg = 1.f * gg + 0.f * bgc[1];
                bb = 1.f * bb + 0.f * bgc[2];
            }
            q.ay = s.y1 - s.y;
            q.by = s.y - s.y0;
            q.ax = s.x1 - s.x;
            q.bx = s.x - s.x0;
            q.grgb[0] = Gt[0];
            q.grgb[1] = Gt[1];
            q.grgb[2] = Gt[2];
            if (want_tex) {
                const bool wok = fabsf(s.lo[0]) < 1e9f && fabsf(s.lo[1]) < 1e9f;
                const int ix0 = (int)s.x0, iy0 = (int)s.y0;
                if (wok) {
                    q.wx = (int)floorf(s.lo[0]);
                    q.wy = (int)floorf(s.lo[1]);
                }
                const int dx = ix0 - q.wx, dy = iy0 - q.wy;
                // all four corners inside the window and the texture (no row wrap).  Conservative: a
                // corner of zero weight outside them also sends the sample to the direct atomics below,
                // which handle any sample (it can only happen when x or y is a whole number at the
                // window's or the texture's last column / row)
                const bool fits = wok && (unsigned)dx <= (unsigned)(TWIN - 2) && (unsigned)dy <= (unsigned)(TWIN - 2) &&
                                  (unsigned)ix0 < (unsigned)(sh.tv.W - 1) && (unsigned)iy0 < (unsigned)(sh.tv.H - 1);
#ifdef NR_COUNT_DIRECT
                atomicAdd(&g_ncount[fits ? 0 : 1], 1ull);
                if (!fits && !wok) atomicAdd(&g_ncount[2], 1ull);
                {  // direct samples whose top-left texel a lower lane of the wave also samples directly
                    const unsigned long long dm = __ballot(!fits);
                    bool dup = false;
                    for (unsigned long long m = dm; m; m &= m - 1) {
                        const int j = __builtin_ctzll(m);
                        const int oj = __builtin_amdgcn_readlane(s.idx[0], j);
                        dup = dup || (j < (int)(threadIdx.x & 63) && oj == s.idx[0]);
                    }
                    if (!fits && dup) atomicAdd(&g_ncount[3], 1ull);
                }
#endif
                // window texel of the top-left corner (dx, dy in 0..2); outside the face window: the
                // top-left texel's flat index as sampled (row-major, unclamped), added in step 5
                q.pos = fits ? dx + 4 * dy : direct_pos((int)__mul24(iy0, sh.tv.W) + ix0);
            }
            // texture coordinates -> z.  Gradient-only terms (within the gradient tolerance, they feed
            // no comparison): fused multiply-adds, factored sums, and the face record's reciprocals
            // 1 / (z_k + 1e-10) in place of a v_rcp each.
            //   d pr_q / d zq_k = -dt w_k uv_kq / zq_k^2, d dt / d zq_k = dt^2 w_k / zq_k^2, so
            //   d/dzq_k = w_k / zq_k^2 (dt^2 g_dt - dt (gpr_0 u_k + gpr_1 v_k))
            const float g_x = __builtin_fmaf(gw[1] - gw[0], q.ay, (gw[3] - gw[2]) * q.by);
            const float g_y = __builtin_fmaf(gw[2] - gw[0], q.ax, (gw[3] - gw[1]) * q.bx);
            const float gp[2] = {g_x, g_y};
            float gpr[2];
#pragma unroll
            for (int j = 0; j < 2; j++) {
                // minimum(pc, hm) then maximum(pr, lo) backward (ties split the gradient)
                const float pc = s.pc[j], hm = s.hm[j], pr = s.pr[j], lo = s.lo[j];
                float gq = gp[j];
                gq = (pc == hm) ? gq * 0.5f : (pc > hm ? 0.f : gq);
                gq = (pr == lo) ? gq * 0.5f : (pr < lo ? 0.f : gq);
                gpr[j] = gq * s.dt;
            }
            const float g_dt = __builtin_fmaf(gpr[0], s.num[0], gpr[1] * s.num[1]);  // dt g_dt
            const float rq[3] = {f.rq0, f.rq1, f.rq2};
#pragma unroll
            for (int j = 0; j < 3; j++) {
                const float inner = __builtin_fmaf(-gpr[0], uvs[2 * j], __builtin_fmaf(-gpr[1], uvs[2 * j + 1], g_dt * s.dt));
                q.gz[j] = (w[j] * (rq[j] * rq[j])) * inner;
            }
        }
        if (sh.draw & NR_DRAW_DEPTH) {
            dep = depth_from_dz(dz, wfast);
            // depth channel gradient: selected from the registers with compile-time indices (a
            // runtime-indexed register array would go to scratch)
            const int dc = (rgb ? 3 : 0) + ((sh.draw & NR_DRAW_SILHOUETTES) ? 1 : 0);
            const float gd = dc == 4 ? G[4] : dc == 3 ? G[3] : dc == 1 ? G[1] : G[0];
            // d dep / d z_k = dep^2 w_k / z_k^2 (the record's 1 / z_k)
            const float e = gd * (dep * dep);
            const float rz[3] = {f.rz0, f.rz1, f.rz2};
#pragma unroll
            for (int j = 0; j < 3; j++) q.gz[j] = __builtin_fmaf(w[j] * (rz[j] * rz[j]), e, q.gz[j]);
        }
        // channel values in merge order (rgb, sil, depth), compile-time slots as in shade_pixel
        const bool R = rgb, Sl = (sh.draw & NR_DRAW_SILHOUETTES) != 0;
        I2[k][0] = R ? r : (Sl ? 1.f : dep);
        I2[k][1] = R ? gg : dep;
        I2[k][2] = bb;
        I2[k][3] = Sl ? 1.f : dep;
        I2[k][4] = dep;
    }
#ifndef NR_ABL_NOSTENCIL  // timing builds only: no LDS staging, halo or pair terms (placeholder stencil)
#pragma unroll
    for (int k = 0; k < NPX; k++) store_ig((ly0 + 4 * k + 1) * HW_ + (lx + 1), I2[k], G2[k]);
    // halo ring: image and upstream gradient only
    int hy, hx;
    halo_pixel(t, hy, hx);
    const int hpy = ty0 - 1 + hy, hpx = tx0 - 1 + hx;
    const bool h_in = t < NHALO && hpy >= 0 && hpy < S && hpx >= 0 && hpx < S;
    if (a.halo) {
        __builtin_amdgcn_s_waitcnt(0);  // this wave's LDS-DMA halo loads have landed
        // each lane t < NHALO moves the halo values it loaded itself (s_hI/s_hG slot t), so its own
        // vmcnt wait is enough: no barrier before the move
        if (t < NHALO) {
            float hI[MAXC], hG[MAXC];
#pragma unroll
            for (int c = 0; c < MAXC; c++) {
                hI[c] = c < C && h_in && h_live ? s_hI[c][t] : 0.f;
                hG[c] = c < C && h_in ? (a.aa ? s_hG[c][t] / 4.f : s_hG[c][t]) : 0.f;
            }
            store_ig(hy * HW_ + hx, hI, hG);
        }
    } else if (t < NHALO) {
        float hI[MAXC], hG[MAXC];
#pragma unroll
        for (int c = 0; c < MAXC; c++) hI[c] = hG[c] = 0.f;
        if (h_in) {
            const int hf = fimb[hpy * S + hpx];
            Face ff;
            FaceUV fu;
            load_shading_face(sh, frb, b, hf, ff, fu);
            shade_pixel(sh, b, hf, ff, fu, hpx, hpy, pix_center(hpx, S), pix_center(hpy, S), S, hI);
            upstream_grad(a, gimb, C, hpy, hpx, S, hG);
        }
        store_ig(hy * HW_ + hx, hI, hG);
    }
    NR_TSTAMP(1);
    __syncthreads();
    NR_TSTAMP(2);

    // ---- 2. Differentiation.backward stencil -> coordinate-map gradient ------------------------
    float gF[NPX][9];
    // Each neighbour pair's two channel dot products serve both of its pixels (stencil_pair): every
    // pixel computes the pair with its right and its lower neighbour, the tile's left halo column and
    // top halo row have theirs computed by lanes of waves 0 and 1, and after a barrier each foreground
    // pixel combines its four pairs -- half the dot products of a per-pixel stencil, the same values
    // (bwd 0.207 -> 0.204 ms with the 24-bit index multiplies, same-box A/B, 5 runs each)
    float2* s_px = reinterpret_cast<float2*>(s_raw + (BWD_LDS_IG + BWD_LDS_HALO) / 4);  // [HN]: pair (i, i + 1)
    float2* s_py = s_px + HN;                                                            // [HN]: pair (i, i + row)
    static_assert(BWD_LDS_IG + BWD_LDS_HALO + 2 * HN * 8 <= bwd_lds<LIT>(), "pair terms fit the block's LDS");
    // (the pixel's own I and G are this lane's registers, the values it staged: no LDS read for them)
    float2 own_px[NPX], own_py[NPX];
#pragma unroll
    for (int k = 0; k < NPX; k++) {
        const int li = (ly0 + 4 * k + 1) * HW_ + (lx + 1);
        float I0[MAXC], G0[MAXC], dx[MAXC], dy[MAXC], Gx[MAXC], Gy[MAXC], Ix[MAXC], Iy[MAXC];
        load_ig(li + 1, Ix, Gx);
        load_ig(li + HW_, Iy, Gy);
#pragma unroll
        for (int c = 0; c < MAXC; c++) {
            const bool u = c < C;
            I0[c] = u ? I2[k][c] : 0.f; G0[c] = u ? G2[k][c] : 0.f;
            dx[c] = u ? I0[c] - Ix[c] : 0.f; Gx[c] = u ? Gx[c] : 0.f;
            dy[c] = u ? I0[c] - Iy[c] : 0.f; Gy[c] = u ? Gy[c] : 0.f;
        }
        own_px[k] = make_float2(diff_dot(dx, Gx, C), diff_dot(dx, G0, C));
        own_py[k] = make_float2(diff_dot(dy, Gy, C), diff_dot(dy, G0, C));
        s_px[li] = own_px[k];
        s_py[li] = own_py[k];
    }
    {
        // the pairs whose first pixel is a halo pixel: left column rows 1..BH (wave 0), top row
        // columns 1..TW (wave 1)
        const bool lc = t < BH, tr = t >= 64 && t < 64 + TW;
        if (lc || tr) {
            const int li = lc ? (t + 1) * HW_ : t - 63, lj = lc ? li + 1 : li + HW_;
            float d[MAXC], Gi[MAXC], Gj[MAXC], Ii[MAXC], Ij[MAXC];
            load_ig(li, Ii, Gi);
            load_ig(lj, Ij, Gj);
#pragma unroll
            for (int c = 0; c < MAXC; c++) {
                const bool u = c < C;
                d[c] = u ? Ii[c] - Ij[c] : 0.f;
                Gi[c] = u ? Gi[c] : 0.f;
                Gj[c] = u ? Gj[c] : 0.f;
            }
            const float2 v = make_float2(diff_dot(d, Gj, C), diff_dot(d, Gi, C));
            if (lc) s_px[li] = v;
            else s_py[li] = v;
        }
    }
    __syncthreads();
#else
    float gF[NPX][9];
    (void)h_live;
#endif
#pragma unroll
    for (int k = 0; k < NPX; k++) {
        BwdPix& q = P[k];
#pragma unroll
        for (int j = 0; j < 9; j++) gF[k][j] = 0.f;
        if (q.fi < 0) continue;
        const int py = ty0 + ly0 + 4 * k;
#ifndef NR_ABL_NOSTENCIL
        const int li = (ly0 + 4 * k + 1) * HW_ + (lx + 1);
        const float gx = stencil_pair(a, own_px[k], s_px[li - 1], px, S);
        const float gy = stencil_pair(a, own_py[k], s_py[li - HW_], py, S);
#else
        const float gx = (I2[k][0] - I2[k][1]) * G2[k][0] * 7.f, gy = (I2[k][2] - I2[k][MAXC - 1]) * G2[k][1] * 5.f;
#endif
        if (wlate && (gx != 0.f || gy != 0.f)) {
            // silhouettes only: the stencil is zero away from silhouette edges, so only these pixels
            // fetch their face and weights (the same computation as in step 1)
            const Face f = load_face_rec(frb + q.fi * FACE_REC);
            face_weights(xp, pix_center(py, S), f, q.w);
        }
        // coordinate map: coord = sum_k w_k faces_xy[k]  (rasterize.py:91-97)
#pragma unroll
        for (int j = 0; j < 3; j++) {
            gF[k][3 * j + 0] = gx * q.w[j];
            gF[k][3 * j + 1] = gy * q.w[j];
            gF[k][3 * j + 2] = q.gz[j];
        }
    }
    NR_TSTAMP(3);
    __syncthreads();  // the staged records reuse the image / gradient LDS
    NR_TSTAMP(4);

    // ---- 3. stage this lane's two pixel records; group the wave's records by face --------------
    // slot of pixel k of lane l: 16 NPX (l >> 4) + 16 k + (l & 15), so member bit b (NPX 16-bit rows)
    // of chunk c is slot 16 NPX c + b; the first float4 holds the four bilinear corner weights
    // (ay ax, ay bx, by ax, by bx: the products the accumulation would form)
    float* rec = s_raw + wid * (64 * NPX * REC);
#pragma unroll
    for (int k = 0; k < NPX; k++) {
        float* r = rec + (16 * NPX * (lane >> 4) + 16 * k + (lane & 15)) * REC;
        reinterpret_cast<float4*>(r)[0] = make_float4(P[k].ay * P[k].ax, P[k].ay * P[k].bx, P[k].by * P[k].ax, P[k].by * P[k].bx);
        reinterpret_cast<float4*>(r)[1] = make_float4(P[k].grgb[0], P[k].grgb[1], P[k].grgb[2], __int_as_float(P[k].pos));
#pragma unroll
        for (int j = 0; j < 9; j++) r[8 + j] = gF[k][j];
        if (LIT) {
#pragma unroll
            for (int j = 0; j < 3; j++) {
                r[17 + j] = P[k].gn[j];
                r[20 + j] = P[k].w[j];
            }
        }
    }
    // output lane roles: texel t = lane & 15 of the face's 4x4 window (dx = t & 3, dy = t >> 2), member
    // chunk c = lane >> 4: lane (t, c) sums the 3 channel contributions to texel t (and, for t < 9,
    // face-gradient float t) over the face's records held by lanes 16 c .. 16 c + 15 (the wave's pixels
    // of parity class c); the 4 chunks are then added across lanes.
    const int tt = lane & 15, chunk = lane >> 4;
    const int tdx = tt & 3, tdy = tt >> 2;
    const int fsel = 8 + (tt < 9 ? tt : 0);
    const int nsel_w = 20 + (tt < 9 ? tt / 3 : 0), nsel_n = 17 + (tt < 9 ? tt % 3 : 0);
    float* __restrict__ gNb = LIT ? a.grad_normals + (long long)b * a.F * 9 : nullptr;
    // the second pixel's state (NPX == 1: none, never active)
    const int fi1 = NPX > 1 ? P[NPX - 1].fi : -1, wx1 = NPX > 1 ? P[NPX - 1].wx : 0, wy1 = NPX > 1 ? P[NPX - 1].wy : 0;
    // a pixel whose every contribution is zero stays out of the per-face gather (exact: it would add
    // zeros): silhouettes away from silhouette edges, where the stencil is zero, or any pixel whose
    // upstream gradient is zero (a loss on some channels or regions only)
    // (testing every pixel for an all-zero record cost the headline ~0.5 %: only silhouettes-only
    // renders, whose stencil is zero away from silhouette edges, do)
    bool nz[NPX];
#pragma unroll
    for (int k = 0; k < NPX; k++) {
        bool v = !wlate;
#pragma unroll
        for (int j = 0; j < 9; j++) v = v || gF[k][j] != 0.f;
        nz[k] = v;
    }
    const bool act0 = P[0].fi >= 0 && nz[0], act1 = fi1 >= 0 && nz[NPX - 1];
    unsigned long long p0 = __ballot(act0), p1 = __ballot(act1);
    NR_TSTAMP(5);
    // texel lanes: consecutive faces with the same texel window (e.g. every face of a flat-colour
    // material samples one 2x2 atlas patch, load_obj.py:84-94) accumulate into `pend` and flush once
    // per run, so such hot texels take one atomic per run instead of one per face
    float pend = 0.f;
    int pwx = INT_MIN, pwy = 0;
    int phid = -1;  // the pending window's shared-window id (face_hot), -1: into the texture gradient
    const bool hot_on = HOT && a.face_hot != nullptr;
    float* __restrict__ hacc = hot_on ? a.hot_acc + (size_t)((blockIdx.y * gridDim.x + blockIdx.x) & (NR_HOT_COPIES - 1)) * a.num_hot * 64 : nullptr;
    int* __restrict__ hpos = hot_on ? reinterpret_cast<int*>(a.hot_acc + hot_sums_floats(a.num_hot)) : nullptr;
#ifdef NR_BWD_TIMING
    int nfaces_dbg = 0;
#endif
    while (p0 | p1) {
#ifdef NR_BWD_TIMING
        nfaces_dbg++;
#endif
        // leader: lowest pending pixel; both candidates read without branches, selected on the scalar unit
        const bool from0 = p0 != 0ull;
        const int l0 = from0 ? __builtin_ctzll(p0) : 0, l1 = p1 ? __builtin_ctzll(p1) : 0;
        const int k0 = __builtin_amdgcn_readlane(P[0].fi, l0), k1 = __builtin_amdgcn_readlane(fi1, l1);
        const int x0w = __builtin_amdgcn_readlane(P[0].wx, l0), x1w = __builtin_amdgcn_readlane(wx1, l1);
        const int y0w = __builtin_amdgcn_readlane(P[0].wy, l0), y1w = __builtin_amdgcn_readlane(wy1, l1);
        const int key = from0 ? k0 : k1, wx = from0 ? x0w : x1w, wy = from0 ? y0w : y1w;
        const int hid = hot_on ? a.face_hot[key] : -1;
        // key >= 0, so fi == key implies an active pixel
        const unsigned long long m0 = __builtin_amdgcn_ballot_w64(P[0].fi == key) & p0;
        const unsigned long long m1 = __builtin_amdgcn_ballot_w64(fi1 == key) & p1;
        p0 &= ~m0;
        p1 &= ~m1;
        float a0 = 0.f, a1 = 0.f, a2 = 0.f, af = 0.f, an = 0.f;
        {
            // this lane's members: those of lanes 16 chunk .. 16 chunk + 15 (parity class `chunk`);
            // bits 0..15 from the first pixel of each lane, 16..31 from the second
            uint32_t mine = ((uint32_t)(m0 >> (16 * chunk)) & 0xffffu) | (((uint32_t)(m1 >> (16 * chunk)) & 0xffffu) << 16);
            const float* rbase = rec + 16 * NPX * chunk * REC;
            // one member's contribution: its loads issued together, accumulation predicated (no branch)
            auto member = [&](const float* r, bool on) {
                const float4 ra = reinterpret_cast<const float4*>(r)[0];  // corner weights w00 w01 w10 w11
                const float4 rb = reinterpret_cast<const float4*>(r)[1];  // G_r G_g G_b pos (G_r, G_g a register pair)
                const float rf = r[fsel];
                // whole rows in registers: otherwise the compiler splits the corner select below into
                // branches, each with its own half-row LDS read
                asm volatile("" ::"v"(ra.x), "v"(ra.y), "v"(ra.z), "v"(ra.w), "v"(rf));
                float rw = 0.f, rn = 0.f;
                if (LIT) {
                    rw = r[nsel_w];
                    rn = r[nsel_n];
                }
                // texel tt = tdx + 4 tdy is corner (d & 1, d >> 2) of the member's footprint when
                // d = tt - pos is 0, 1, 4 or 5 (dx, dy <= 2 rule out row wrap-around): bits 0, 1, 4, 5
                // of 0x33; d & 31 is 6..31 for every other d in -10..15 and for POS_NONE
                const int pos = __float_as_int(rb.w);
                const int d = tt - pos;
                const bool hit = on && __builtin_amdgcn_ubfe(0x33u, (unsigned)d, 1u);  // (0x33 >> (d & 31)) & 1
                const float wsel = (d & 4) ? ((d & 1) ? ra.w : ra.z) : ((d & 1) ? ra.y : ra.x);
                const float wt = hit ? wsel : 0.f;
                // fused multiply-adds (gradient sums; 3 of the step's 24 VALU: bwd 0.212 -> 0.207 ms)
                a0 = __builtin_fmaf(rb.x, wt, a0);
                a1 = __builtin_fmaf(rb.y, wt, a1);
                a2 = __builtin_fmaf(rb.z, wt, a2);
                af += on ? rf : 0.f;
                if (LIT) an += on ? rw * rn : 0.f;  // corner-normal gradient tt = 3 corner + axis
            };
            // one loop over both pixel rows (2- and 4-member steps measured slower)
#ifndef NR_ABL_NOGATHER  // timing builds only: no member loop
            for (; mine; mine &= mine - 1) member(rbase + __builtin_ctz(mine) * REC, true);
#else
            (void)rbase;
#endif
        }
        // reduce-scatter over the 4 member chunks (lanes t, t+16, t+32, t+48) with the gfx950 lane
        // swaps (VALU, no LDS round trip): lane (t, c) ends with the chunk total of value c
        const float v = chunk_reduce_scatter(a0, a1, a2, af);
        if (LIT) {  // the normal gradients: a plain sum over the 4 chunks, flushed by chunk 0
            const auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(an), __float_as_uint(an), false, false);
            const float h = __uint_as_float(p[0]) + __uint_as_float(p[1]);
            const auto q2 = __builtin_amdgcn_permlane16_swap(__float_as_uint(h), __float_as_uint(h), false, false);
            const float nt = __uint_as_float(q2[0]) + __uint_as_float(q2[1]);
            if (chunk == 0 && tt < 9 && nt != 0.f) unsafeAtomicAdd(gNb + key * 9 + tt, nt);
        }
        // ---- 4. flush this face: lane (t, c) writes channel c of texel t (c < 3) or face float t (c == 3)
        {
            // one atomic per lane, address selected without branches: face lanes add this face's
            // floats; texel lanes flush the pending window when the window changes
            const bool win = wx != INT_MIN;
            const bool sw = win && (wx != pwx || wy != pwy);
            const int x = pwx + tdx, y = pwy + tdy;
            const bool tex_lane = want_tex && chunk < 3 && sw && pwx != INT_MIN && x < sh.tv.W && y < sh.tv.H;
            const bool face_lane = chunk == 3 && tt < 9;
            const float fv = face_lane ? v : pend;
            float* tdst = phid >= 0 ? hacc + (phid * 16 + tt) * 4 + chunk : gtb + ((int)__umul24(y, sh.tv.W) + x) * 4 + chunk;
            float* dst = tex_lane ? tdst : gFb + key * 9 + tt;
            if (tex_lane && phid >= 0 && tt == 0 && chunk == 0) {  // the window's origin (every writer's is the same)
                hpos[2 * phid] = pwx;
                hpos[2 * phid + 1] = pwy;
            }
#ifdef NR_ABL_NOATOM  // timing builds only: no flush atomics
            if ((tex_lane || face_lane) && fv == 12345.f) unsafeAtomicAdd(dst, fv);
#elif defined(NR_ABL_NOTEXFLUSH)  // timing builds only: no texture-window flush atomics
            if (((tex_lane && fv == 12345.f) || face_lane) && fv != 0.f) unsafeAtomicAdd(dst, fv);
#elif defined(NR_ABL_NOGFFLUSH)  // timing builds only: no face-gradient flush atomics
            if ((tex_lane || (face_lane && fv == 12345.f)) && fv != 0.f) unsafeAtomicAdd(dst, fv);
#else
            if ((tex_lane || face_lane) && fv != 0.f) unsafeAtomicAdd(dst, fv);
#endif
            if (win) {
                pend = sw ? v : pend + v;
                pwx = wx;
                pwy = wy;
                if (sw) phid = hid;
            }
        }
    }
    {  // the last pending window
        const int x = pwx + tdx, y = pwy + tdy;
        const bool tex_lane = want_tex && chunk < 3 && pwx != INT_MIN && x < sh.tv.W && y < sh.tv.H;
        if (tex_lane && phid >= 0 && tt == 0 && chunk == 0) {
            hpos[2 * phid] = pwx;
            hpos[2 * phid + 1] = pwy;
        }
        if (tex_lane && pend != 0.f)
            unsafeAtomicAdd(phid >= 0 ? hacc + (phid * 16 + tt) * 4 + chunk : gtb + ((int)__umul24(y, sh.tv.W) + x) * 4 + chunk, pend);
    }
    // ---- 5. texture samples outside their face's window (POS_DIRECT): their texel gradients, 4
    // samples per atomic instruction.  Lane (sample u = lane >> 4, row = bit 3, column = bit 2,
    // channel = bits 0-1) adds G_ch * w(row, column) to texel (x0 + column, y0 + row) of RGBA row
    // storage, so one instruction covers two 32-B segments (the two texel pairs) per sample, where
    // one texel channel per lane and instruction put every lane in its own 64-B line (the memory-side
    // atomic units take a line per request: MI355X_MICROARCH.md "Global float atomics").  The
    // staged records still hold each sample's corner weights, G and position, so no state crosses
    // the gather loop; the wave's own record region is all it reads.
    if (want_tex) {
        unsigned long long d0 = 0ull, d1 = 0ull;
#pragma unroll
        for (int k = 0; k < NPX; k++) {
            const int pos = __float_as_int(rec[(16 * NPX * (lane >> 4) + 16 * k + (lane & 15)) * REC + 7]);
            const unsigned long long m = __ballot(pos <= POS_DIRECT);
            if (k == 0) d0 = m;
            else d1 = m;
        }
        const int row = (lane >> 3) & 1, col = (lane >> 2) & 1, ch = lane & 3;
        const int HW = sh.tv.H * sh.tv.W;
        while (d0 | d1) {
            // four samples (wave-uniform slots; -1 when the list runs out), picked on the scalar unit
            int sl[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const bool from0 = d0 != 0ull;
                const unsigned long long m = from0 ? d0 : d1;
                const int j = m ? __builtin_ctzll(m) : 0;
                sl[u] = m ? 16 * NPX * (j >> 4) + 16 * (from0 ? 0 : 1) + (j & 15) : -1;
                if (from0) d0 &= d0 - 1;
                else d1 &= d1 - 1;
            }
            const int u = lane >> 4;
            const int slot = u == 0 ? sl[0] : u == 1 ? sl[1] : u == 2 ? sl[2] : sl[3];
            const float* r = rec + max(slot, 0) * REC;
            const float4 ra = reinterpret_cast<const float4*>(r)[0];  // corner weights w00 w01 w10 w11
            const float4 rb = reinterpret_cast<const float4*>(r)[1];  // G_r G_g G_b pos
            const float wsel = row ? (col ? ra.w : ra.z) : (col ? ra.y : ra.x);
            const float gsel = ch == 0 ? rb.x : (ch == 1 ? rb.y : rb.z);
            const float v = gsel * wsel;
            // the texel index as sample_texture clamps it (a clamped corner has weight 0)
            const int idx = min(max(direct_base(__float_as_int(rb.w)) + col + row * sh.tv.W, 0), HW - 1);
#ifdef NR_ABL_NODIRECT  // timing builds only: no direct-sample atomics
            if (slot >= 0 && ch < 3 && v == 12345.f) unsafeAtomicAdd(gtb + idx * 4 + ch, v);
#else
            if (slot >= 0 && ch < 3 && v != 0.f) unsafeAtomicAdd(gtb + idx * 4 + ch, v);
#endif
        }
    }
    NR_TSTAMP(6);
    NR_WSTAMP(9);
#ifdef NR_BWD_TIMING
    {
        const long long i_ = (((long long)blockIdx.y * gridDim.x + blockIdx.x) * (blockDim.x / 64) + (threadIdx.x >> 6)) * NR_BSLOTS + 7;
        if (lane == 0 && i_ < NR_TIMING_MAX) g_bwd_t[i_] = (unsigned long long)nfaces_dbg;
    }
#endif
}

// the private copies of the shared texture windows (BwdArgs.face_hot) summed and added into the RGBA
// texture-gradient accumulator (item 0: a shared texture): block h = window h, lane (texel t = lane &
// 15, channel lane >> 4 < 3).  A window no face flushed has sums of 0 and adds nothing.
__global__ __launch_bounds__(64) void k_hot_reduce(const float* __restrict__ acc, int num_hot, float* __restrict__ gtb,
                                                   int W, int H) {
    const int h = blockIdx.x, tt = threadIdx.x & 15, ch = threadIdx.x >> 4;
    if (ch >= 3) return;
    const int* pos = reinterpret_cast<const int*>(acc + hot_sums_floats(num_hot));
    float s = 0.f;
#pragma unroll 8
    for (int c = 0; c < NR_HOT_COPIES; c++) s += acc[(((size_t)c * num_hot + h) * 16 + tt) * 4 + ch];
    const int x = pos[2 * h] + (tt & 3), y = pos[2 * h + 1] + (tt >> 2);
    if (s != 0.f && x >= 0 && y >= 0 && x < W && y < H) unsafeAtomicAdd(gtb + ((size_t)y * W + x) * 4 + ch, s);
}

// pixels per lane, per launch: 2 (256 threads) when the grid fills the chip many times over; 1 (512
// threads, 6 waves/SIMD instead of 4) for small grids, where the waves, not the per-face work, are
// short (teapot B=4: 0.041 -> 0.035 ms; torus 1024^2 B=1: 0.059 -> 0.048 ms; on the headline and the
// car the smaller wave regions mean more face flushes: 0.405 -> 0.417 and 0.73 -> 0.84 ms).
template <int FEAT, bool HOT>
void launch_bwd_v(dim3 grid, hipStream_t st, const BwdArgs& ba, const Geom& g, const Shade& sh) {
    const bool one = (long long)grid.x * grid.y < 8192;
    const int hotf = HOT ? NR_LAUNCH_HOT_WINDOWS : 0;
    if (one) {
        nr_launch((k_raster_bwd<FEAT, 1, 0, HOT>), grid, dim3(2 * NT), 0, st, ba, g, sh);
        g_last_bwd.store(LaunchRec{2 * NT, hotf});
    } else if (FEAT == 0 && sh.C == MAXC && ba.aa && ba.step_pow2) {
        nr_launch((k_raster_bwd<FEAT, 2, MAXC, HOT>), grid, dim3(NT), 0, st, ba, g, sh);
        g_last_bwd.store(LaunchRec{NT, NR_LAUNCH_STATIC_CHANNELS | NR_LAUNCH_TWO_PX_PER_LANE | hotf});
    } else if (FEAT == 0 && sh.draw == static_draw(4) && ba.aa && ba.step_pow2) {
        nr_launch((k_raster_bwd<FEAT, 2, 4, HOT>), grid, dim3(NT), 0, st, ba, g, sh);
        g_last_bwd.store(LaunchRec{NT, NR_LAUNCH_STATIC_CHANNELS | NR_LAUNCH_TWO_PX_PER_LANE | hotf});
    } else {
        nr_launch((k_raster_bwd<FEAT, 2, 0, HOT>), grid, dim3(NT), 0, st, ba, g, sh);
        g_last_bwd.store(LaunchRec{NT, NR_LAUNCH_TWO_PX_PER_LANE | hotf});
    }
}
// the shared-window instantiations exist for the plain textured backward (FEAT 0) only; the caller
// passes face_hot for no other (nr_rasterize_backward)
template <int FEAT>
void launch_bwd(dim3 grid, hipStream_t st, const BwdArgs& ba, const Geom& g, const Shade& sh) {
#ifdef NR_ABL_S1LOAD
    {  // timing builds only: a zeroed buffer of 3 float4 planes, one entry per (thread, pixel) of the grid
        static float4* buf = nullptr;
        static size_t have = 0;
        const size_t need = (size_t)grid.x * grid.y * NT * 2 * 3 * sizeof(float4);
        if (need > have) {
            if (buf) (void)hipFree(buf);
            if (hipMalloc(&buf, need) != hipSuccess || hipMemset(buf, 0, need) != hipSuccess ||
                hipMemcpyToSymbol(HIP_SYMBOL(g_abl_prod), &buf, sizeof(buf)) != hipSuccess || hipDeviceSynchronize() != hipSuccess)
                abort();
            have = need;
        }
    }
#endif
    if constexpr (FEAT == 0) {
        if (ba.face_hot) {
            launch_bwd_v<FEAT, true>(grid, st, ba, g, sh);
            return;
        }
    }
    launch_bwd_v<FEAT, false>(grid, st, ba, g, sh);
}

constexpr int VGRAD_UNROLL = 4;
// gathered-face gradient -> vertex gradient: gV[b, v] = sum over (f, k) with faces[f, k] = v of gF[b, f, k]
// (the index backward of rasterize.py:232), through a CSR adjacency built once per faces tensor.
// xcd_items (B % 8 == 0): the grid is 8 B / 8 item columns of bpi = ceil(V / blockDim.x) blocks, and
// block L works on item b = L % 8 + 8 m: workgroups are dealt to XCD L % 8, so every block of item b
// runs on XCD b % 8 and the item's gF rows (184 KB at the headline) come from HBM into one L2 once,
// not into each L2 that a block of the item lands on (40 -> ~15 MB of reads per launch)
__global__ void k_vertex_grad(const float* __restrict__ gF, const int32_t* __restrict__ off,
                              const int32_t* __restrict__ ent, float* __restrict__ gV, int F, int V, long long n,
                              TexOut to, int xcd_items) {
    if (to.out) {  // this block's slice of the texture-gradient output (the RGBA accumulator transposed)
        long long lo, hi;
        grid_slice(to.n, lo, hi);
        for (long long j = lo + threadIdx.x; j < hi; j += blockDim.x) tex_out_one(to, j);
    }
    int b, v;
    long long i;
    if (xcd_items) {
        const int bpi = (V + blockDim.x - 1) / blockDim.x;
        const int L = blockIdx.x, j = L >> 3;
        b = (L & 7) + 8 * (j / bpi);
        v = (j % bpi) * blockDim.x + threadIdx.x;
        if (v >= V) return;
        i = (long long)b * V + v;
        if (i >= n) return;
    } else {
        i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
        if (i >= n) return;
        b = (int)(i / V);
        v = (int)(i % V);
    }
    const float* base = gF + (long long)b * F * 9;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f;
    const int e0 = off[v], e1 = off[v + 1];
    // entries read VGRAD_UNROLL at a time (their row loads in flight together); the sums keep the
    // CSR order
    int e = e0;
    for (; e + VGRAD_UNROLL <= e1; e += VGRAD_UNROLL) {
        int en[VGRAD_UNROLL];
#pragma unroll
        for (int u = 0; u < VGRAD_UNROLL; u++) en[u] = ent[e + u];
        float3 rv[VGRAD_UNROLL];
#pragma unroll
        for (int u = 0; u < VGRAD_UNROLL; u++) {
            const float* r = base + (long long)en[u] * 3;
            rv[u] = make_float3(r[0], r[1], r[2]);
        }
#pragma unroll
        for (int u = 0; u < VGRAD_UNROLL; u++) {
            s0 += rv[u].x;
            s1 += rv[u].y;
            s2 += rv[u].z;
        }
    }
    for (; e < e1; e++) {
        const float* r = base + (long long)ent[e] * 3;  // entry = 3 f + k
        s0 += r[0];
        s1 += r[1];
        s2 += r[2];
    }
    gV[i * 3 + 0] = s0;
    gV[i * 3 + 1] = s1;
    gV[i * 3 + 2] = s2;
}

// vertex-normal backward (lights): gU[b, v] = d/du of F.normalize (rasterize.py:182) applied to the
// gradient of n[b, v], gathered over the vertex's face corners (the gather at rasterize.py:183)
__global__ void k_vnormal_bwd(const float* __restrict__ gN, const int32_t* __restrict__ off,
                              const int32_t* __restrict__ ent, const float* __restrict__ vnorm,
                              float* __restrict__ gU, int F, int V, long long n) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int b = (int)(i / V), v = (int)(i % V);
    const float* base = gN + (long long)b * F * 9;
    float g0 = 0.f, g1 = 0.f, g2 = 0.f;
    for (int e = off[v]; e < off[v + 1]; e++) {
        const float* r = base + ent[e] * 3;  // entry = 3 f + k
        g0 += r[0];
        g1 += r[1];
        g2 += r[2];
    }
    const float4 nv = reinterpret_cast<const float4*>(vnorm)[i];  // n = u / max(|u|, eps), |u|
    float* o = gU + i * 3;
    if (nv.w > 1e-12f) {
        // d(u / |u|)/du^T g = (g - n (n . g)) / |u|
        const float nd = (nv.x * g0 + nv.y * g1) + nv.z * g2;
        o[0] = (g0 - nv.x * nd) / nv.w;
        o[1] = (g1 - nv.y * nd) / nv.w;
        o[2] = (g2 - nv.z * nd) / nv.w;
    } else {
        o[0] = g0 / 1e-12f;
        o[1] = g1 / 1e-12f;
        o[2] = g2 / 1e-12f;
    }
}

// face-normal backward (lights): the face normal gets the gradients of its distinct vertices' sums
// (the one-hot matmul, rasterize.py:173-179), then n = a x b with a = v1 - v0, b = v2 - v1 gives
// dL/da = b x g, dL/db = g x a, added to the face's corner gradients gF (rasterize.py:166-170)
__global__ void k_fnormal_bwd(const float* __restrict__ face_records, const int32_t* __restrict__ fidx,
                              const float* __restrict__ gU, float* __restrict__ gF, int F, int V, long long n) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int b = (int)(i / F), f = (int)(i % F);
    const int v0 = fidx[f * 3], v1 = fidx[f * 3 + 1], v2 = fidx[f * 3 + 2];
    const float* ub = gU + (long long)b * V * 3;
    float g[3];
#pragma unroll
    for (int j = 0; j < 3; j++) {
        g[j] = ub[v0 * 3 + j];
        if (v1 != v0) g[j] += ub[v1 * 3 + j];
        if (v2 != v0 && v2 != v1) g[j] += ub[v2 * 3 + j];
    }
    const float* c = face_records + i * FACE_REC;
    const float a0 = c[3] - c[0], a1 = c[4] - c[1], a2 = c[5] - c[2];
    const float b0 = c[6] - c[3], b1 = c[7] - c[4], b2 = c[8] - c[5];
    const float da0 = b1 * g[2] - b2 * g[1], da1 = b2 * g[0] - b0 * g[2], da2 = b0 * g[1] - b1 * g[0];
    const float db0 = g[1] * a2 - g[2] * a1, db1 = g[2] * a0 - g[0] * a2, db2 = g[0] * a1 - g[1] * a0;
    float* o = gF + i * 9;
    o[0] -= da0;
    o[1] -= da1;
    o[2] -= da2;
    o[3] += da0 - db0;
    o[4] += da1 - db1;
    o[5] += da2 - db2;
    o[6] += db0;
    o[7] += db1;
    o[8] += db2;
}

// the RGBA texture-gradient accumulator -> [Bt, 3, H, W]
__global__ void k_tex_out(TexOut to) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < to.n) tex_out_one(to, i);
}

// ------------------------------------------------------------------------------------------------
// k_param_bwd: the gradients of the inputs that only the rgb channels see and that the main backward
// does not produce -- vertices_textures (UV) and the light parameters (LGT).  One thread per internal
// pixel (a wave = 64 pixels of one row); runs only when one of them is requested.
//   UV:  sample_textures (rasterize.py:111-121): x = min(max(pr, lo), hm) with pr = num * dt,
//        num = sum_k (w_k uv_k) / zq_k, lo = min_k uv_k, hm = max_k uv_k - eps.  The bilinear weight
//        gradient (as in k_raster_bwd) goes back through the two clamps (ties split in half, as
//        torch.maximum / torch.minimum do), to pr -> uv_k through (w_k / zq_k) dt, and to the
//        first-occurring arg-min / arg-max corner (torch's min(-2) / max(-2) backward).  Lanes of
//        one face are summed across the wave and the leader adds the 6 corner values to
//        grad_vt[faces_textures[f, k]] (the gather backward of rasterize.py:246).
//   LGT: the light loop (rasterize.py:252-283) with rgb = T cw, dL/dcw = G T: per light, the colour
//        gets s dL/dcw, a directional light's direction gets -n s'(raw) sum_c(dL/dcw_c col_c), a
//        specular exponent gets sum_c(dL/dcw_c col_c) s^alpha log(s) (0 where s == 0, alpha >= 0, as
//        torch's pow backward).  Wave sums, one atomic per wave and value into grad_lights, laid
//        out like the light records [L][B][NR_LIGHT_FLOATS] (colour 2..4, direction 5..7, alpha 5).
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

template <bool UV, bool LGT>
__global__ __launch_bounds__(256) void k_param_bwd(BwdArgs a, Shade sh, int S, const int32_t* __restrict__ ftex,
                                                   float* __restrict__ grad_vt, long long gvt_bstride,
                                                   float* __restrict__ grad_lights) {
    const int b = blockIdx.y;
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    const int lane = threadIdx.x & 63;
    const bool inside = p < S * S;
    const int y = inside ? p / S : 0, x = inside ? p - y * S : 0;
    const int fi = inside ? a.fim[(long long)b * S * S + p] : -1;
    const int bt = sh.tv.sb ? b : 0;
    float guv[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    float T[3] = {0.f, 0.f, 0.f}, G[MAXC], nrm[3] = {0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < MAXC; c++) G[c] = 0.f;
    if (fi >= 0) {
        const float* gimb = a.grad_images + (long long)b * sh.C * (a.aa ? a.s * a.s : S * S);
        upstream_grad(a, gimb, sh.C, y, x, S, G);
        Face f = load_face_rec(a.face_records + ((long long)b * a.F + fi) * FACE_REC);
        f.flags = 0;
        float w[3];
        face_weights(pix_center(x, S), pix_center(y, S), f, w);
        float Gt[3] = {G[0], G[1], G[2]};
        float cw[3];
        if (sh.nl) {
            pixel_normal(sh, b, fi, w, nrm);
            light_weights(sh, b, nrm, cw);
#pragma unroll
            for (int c = 0; c < 3; c++) Gt[c] = G[c] * cw[c];
        }
        const float* fuv = sh.face_uv + (sh.uv_bstride ? (long long)b * sh.uv_bstride : 0) + fi * 8;
        TexSample s;
        float gw[4];
        sample_texture(f, w, false, load_face_uv(fuv), sh.tv, bt, sh.eps, s, Gt, gw);
        T[0] = s.rgb[0];
        T[1] = s.rgb[1];
        T[2] = s.rgb[2];
        if (UV) {
            const float ay = s.y1 - s.y, by = s.y - s.y0, ax = s.x1 - s.x, bx = s.x - s.x0;
            const float gp[2] = {((-(gw[0] * ay) + gw[1] * ay) - gw[2] * by) + gw[3] * by,
                                 ((-(gw[0] * ax) - gw[1] * bx) + gw[2] * ax) + gw[3] * bx};
#pragma unroll
            for (int j = 0; j < 2; j++) {
                const float pc = s.pc[j], hm = s.hm[j], pr = s.pr[j], lo = s.lo[j];
                const float g = gp[j];
                const float to_pc = pc == hm ? g * 0.5f : (pc < hm ? g : 0.f);
                const float to_hm = pc == hm ? g * 0.5f : (pc > hm ? g : 0.f);
                const float to_pr = pr == lo ? to_pc * 0.5f : (pr > lo ? to_pc : 0.f);
                const float to_lo = pr == lo ? to_pc * 0.5f : (pr < lo ? to_pc : 0.f);
                const float gnum = to_pr * s.dt;
                const float u[3] = {fuv[j], fuv[2 + j], fuv[4 + j]};
                const int kmin = (u[1] < u[0] && !(u[2] < u[1])) ? 1 : ((u[2] < u[0] && u[2] < u[1]) ? 2 : 0);
                const int kmax = (u[1] > u[0] && !(u[2] > u[1])) ? 1 : ((u[2] > u[0] && u[2] > u[1]) ? 2 : 0);
#pragma unroll
                for (int k = 0; k < 3; k++)
                    guv[2 * k + j] = (gnum / s.zq[k]) * w[k] + (k == kmin ? to_lo : 0.f) + (k == kmax ? to_hm : 0.f);
            }
        }
    }
    if (UV) {
        // group the wave's lanes by face; the leader adds the face's 6 sums to its uv vertices
        const bool act = fi >= 0;
        unsigned long long pend = __ballot(act);
        float* gvb = grad_vt + (sh.uv_bstride ? (long long)b * gvt_bstride : 0);
        while (pend) {
            const int leader = __builtin_ctzll(pend);
            const int key = __builtin_amdgcn_readlane(fi, leader);
            const bool mem = act && fi == key;
            pend &= ~__ballot(mem);
#pragma unroll
            for (int q = 0; q < 6; q++) {
                const float v = wave_sum(mem ? guv[q] : 0.f);
                if (lane == leader && v != 0.f) unsafeAtomicAdd(gvb + ftex[key * 3 + q / 2] * 2 + (q & 1), v);
            }
        }
    }
    if (LGT) {
        const bool act = fi >= 0;
        const float gcw[3] = {G[0] * T[0], G[1] * T[1], G[2] * T[2]};
        for (int l = 0; l < sh.nl; l++) {
            const float* L = sh.lights + ((long long)l * sh.B + b) * NR_LIGHT_FLOATS;
            float* gl = grad_lights + ((long long)l * sh.B + b) * NR_LIGHT_FLOATS;
            const int kind = (int)L[0];
            const bool back = L[1] != 0.f;
            const float col[3] = {L[2], L[3], L[4]};
            float gc[3], gd[3] = {0.f, 0.f, 0.f}, ga = 0.f;
            if (kind == NR_LIGHT_AMBIENT) {
                gc[0] = gcw[0], gc[1] = gcw[1], gc[2] = gcw[2];
            } else {
                const bool dirl = kind == NR_LIGHT_DIRECTIONAL;
                const float d0 = dirl ? L[5] : 0.f, d1 = dirl ? L[6] : 0.f, d2 = dirl ? L[7] : 1.f;
                const float raw = ((-d0) * nrm[0] + (-d1) * nrm[1]) + (-d2) * nrm[2];
                const float sv = back ? fabsf(raw) : t_relu(raw);
                const float ds = back ? (raw > 0.f ? 1.f : (raw < 0.f ? -1.f : 0.f)) : (raw > 0.f ? 1.f : 0.f);
                const float gs = (gcw[0] * col[0] + gcw[1] * col[1]) + gcw[2] * col[2];
                if (dirl) {
#pragma unroll
                    for (int c = 0; c < 3; c++) gc[c] = sv * gcw[c];
                    gd[0] = gs * ds * (-nrm[0]);
                    gd[1] = gs * ds * (-nrm[1]);
                    gd[2] = gs * ds * (-nrm[2]);
                } else {
                    const float alpha = L[5];
                    const float pw = powf(sv, alpha);
#pragma unroll
                    for (int c = 0; c < 3; c++) gc[c] = pw * gcw[c];
                    ga = (sv == 0.f && alpha >= 0.f) ? 0.f : gs * (pw * logf(sv));
                }
            }
#pragma unroll
            for (int c = 0; c < 3; c++) {
                const float v = wave_sum(act ? gc[c] : 0.f);
                if (lane == 0 && v != 0.f) unsafeAtomicAdd(gl + 2 + c, v);
            }
            if (kind == NR_LIGHT_DIRECTIONAL) {
#pragma unroll
                for (int c = 0; c < 3; c++) {
                    const float v = wave_sum(act ? gd[c] : 0.f);
                    if (lane == 0 && v != 0.f) unsafeAtomicAdd(gl + 5 + c, v);
                }
            } else if (kind == NR_LIGHT_SPECULAR) {
                const float v = wave_sum(act ? ga : 0.f);
                if (lane == 0 && v != 0.f) unsafeAtomicAdd(gl + 5, v);
            }
        }
    }
}

}  // namespace
