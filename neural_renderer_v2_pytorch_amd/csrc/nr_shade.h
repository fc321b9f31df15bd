// nr_shade.h -- forward epilogue: halo cache, k_shade / k_shade_px, standalone weight-map / mask / Differentiation kernels
// Part of nr_raster.hip (one translation unit); see that file and DESIGN.md.
#pragma once

#pragma clang fp contract(off)

namespace {

// ------------------------------------------------------------------------------------------------
// Halo cache: the internal-image values of the pixels on the border rows / columns of the backward's
// 32x16 tiles, written by k_shade (which computes every internal pixel anyway) so that
// k_raster_bwd loads its 1-pixel tile halo (asynchronously, during its main work) instead of
// re-shading it.  Per item:
//   rows: [nty][2][C][S]        side 0 = row 16 ty, side 1 = row 16 ty + 15, every column
//   cols: [nty][C][16][ntx][2]  row y = 16 ty + r of column 32 tx (side 0) / 32 tx + 31 (side 1)
// Both parts are written in contiguous runs by a shade block (one output row = two internal rows).
constexpr int HALO_TW = 32, HALO_TH = 16;
__host__ __device__ __forceinline__ long long halo_item_floats(int S, int C) {
    const long long nty = (S + HALO_TH - 1) / HALO_TH, ntx = (S + HALO_TW - 1) / HALO_TW;
    return nty * 2 * C * (long long)S + nty * C * HALO_TH * ntx * 2;
}
// after the B items' halo values: one byte per (item, 32x32 bin), nonzero when the bin has a
// foreground pixel (written by the forward, read by the backward to skip background tiles)
__host__ __device__ __forceinline__ long long halo_flags_offset_bytes(int B, int S, int C) {
    return (long long)B * halo_item_floats(S, C) * 4;
}
// (24-bit multiplies: every factor here is below 2^24 and every offset below 2^31 for the rasters the
// library accepts; v_mul_lo_u32 would be quarter rate, and every shading wave forms these offsets)
__device__ __forceinline__ int halo_row_offset(int C, int S, int x, int y, int c) {
    return (int)__umul24(__umul24((unsigned)((y / HALO_TH) * 2 + ((y & (HALO_TH - 1)) != 0)), C) + c, S) + x;
}
__device__ __forceinline__ int halo_col_offset(int C, int S, int x, int y, int c) {
    const int nty = (S + HALO_TH - 1) / HALO_TH, ntx = (S + HALO_TW - 1) / HALO_TW;
    return (int)__umul24(__umul24(nty * 2, C), S) +
           (int)__umul24((__umul24((unsigned)(y / HALO_TH), C) + c) * HALO_TH + (y & (HALO_TH - 1)), 2 * ntx) +
           2 * (x / HALO_TW) + ((x & (HALO_TW - 1)) != 0);
}
// offset of channel 0 of tile-border pixel (x, y) and the stride between its channels
__device__ __forceinline__ void halo_locate(int C, int S, int x, int y, int& off, int& cstride) {
    const int ry = y & (HALO_TH - 1);
    if (ry == 0 || ry == HALO_TH - 1) {
        off = halo_row_offset(C, S, x, y, 0);
        cstride = S;
    } else {
        off = halo_col_offset(C, S, x, y, 0);
        cstride = HALO_TH * 2 * ((S + HALO_TW - 1) / HALO_TW);
    }
}
__device__ __forceinline__ void halo_store(float* __restrict__ halo, int b, int C, int S, int x, int y, const float* v) {
    float* base = halo + b * halo_item_floats(S, C);
    const int ry = y & (HALO_TH - 1), rx = x & (HALO_TW - 1);
    if (ry == 0 || ry == HALO_TH - 1) {
#pragma unroll
        for (int c = 0; c < MAXC; c++)
            if (c < C) base[halo_row_offset(C, S, x, y, c)] = v[c];
    }
    if (rx == 0 || rx == HALO_TW - 1) {
#pragma unroll
        for (int c = 0; c < MAXC; c++)
            if (c < C) base[halo_col_offset(C, S, x, y, c)] = v[c];
    }
}

// ------------------------------------------------------------------------------------------------
// One anti-aliased output pixel: the 2x2 average of the flipped image (rasterize.py:321-328).  The
// internal quad has top-left (iy, ix) and face ids fis = {a, b, c, d} with a = (iy+1, ix+1),
// b = (iy, ix+1), c = (iy+1, ix), d = (iy, ix); output (oi, oj) = ((S-2-iy)/2, (S-2-ix)/2).  Writes
// the C channels and the quad's backward-tile-border pixels to the halo cache.  Used by k_shade and by
// the forward's fused shading epilogue (k_raster_fwd<256, true>).
__device__ __forceinline__ void shade_quad(const Shade& sh, const float* __restrict__ frb, int b, int S, int iy, int ix,
                                           const int fis[4], float* __restrict__ images, float* __restrict__ halo) {
    const int s = S / 2;
    const int o = (int)__umul24((S - 2 - iy) >> 1, s) + ((S - 2 - ix) >> 1);
    float* ob = images + (long long)b * sh.C * s * s + o;
    const int ys[4] = {iy + 1, iy, iy + 1, iy}, xs[4] = {ix + 1, ix + 1, ix, ix};
    // the quad's two column and two row centres
    const float cx0 = pix_center(ix, S), cx1 = pix_center(ix + 1, S), cy0 = pix_center(iy, S), cy1 = pix_center(iy + 1, S);
    const float xps[4] = {cx1, cx1, cx0, cx0}, yps[4] = {cy1, cy0, cy1, cy0};
    float v[4][MAXC];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        Face f;
        FaceUV u;
        load_shading_face(sh, frb, b, fis[q], f, u);
        shade_pixel(sh, b, fis[q], f, u, xs[q], ys[q], xps[q], yps[q], S, v[q]);
    }
#pragma unroll
    for (int c = 0; c < MAXC; c++)
        if (c < sh.C) ob[c * s * s] = (((v[0][c] + v[1][c]) + v[2][c]) + v[3][c]) / 4.f;
    if (halo) {
        // this thread's 2x2 internal pixels on the backward's tile borders: rows iy (top border) /
        // iy + 1 (bottom border) as float2 pairs, columns ix (left) / ix + 1 (right)
        float* hb = halo + b * halo_item_floats(S, sh.C);
        const int C = sh.C;
        const int ry = iy & (HALO_TH - 1), rx = ix & (HALO_TW - 1);
        if (ry == 0 || ry == HALO_TH - 2) {
            const int top = ry == 0, y = top ? iy : iy + 1;
#pragma unroll
            for (int c = 0; c < MAXC; c++)
                if (c < C)
                    *reinterpret_cast<float2*>(hb + halo_row_offset(C, S, ix, y, c)) =
                        top ? make_float2(v[3][c], v[1][c]) : make_float2(v[2][c], v[0][c]);
        }
        if (rx == 0 || rx == HALO_TW - 2) {
            const int left = rx == 0, x = left ? ix : ix + 1;
#pragma unroll
            for (int c = 0; c < MAXC; c++) {
                if (c < C) {
                    hb[halo_col_offset(C, S, x, iy, c)] = left ? v[3][c] : v[1][c];
                    hb[halo_col_offset(C, S, x, iy + 1, c)] = left ? v[2][c] : v[0][c];
                }
            }
        }
    }
}

// shade_quad for a quad of background pixels without backgrounds: every value is 0
__device__ __forceinline__ void shade_quad_empty(const Shade& sh, int b, int S, int iy, int ix, float* __restrict__ images,
                                                 float* __restrict__ halo) {
    const int s = S / 2;
    const int o = (int)__umul24((S - 2 - iy) >> 1, s) + ((S - 2 - ix) >> 1);
    float* ob = images + (long long)b * sh.C * s * s + o;
#pragma unroll
    for (int c = 0; c < MAXC; c++)
        if (c < sh.C) ob[c * s * s] = 0.f;
    if (halo) {
        float* hb = halo + b * halo_item_floats(S, sh.C);
        const int C = sh.C;
        const int ry = iy & (HALO_TH - 1), rx = ix & (HALO_TW - 1);
        if (ry == 0 || ry == HALO_TH - 2) {
            const int y = ry == 0 ? iy : iy + 1;
#pragma unroll
            for (int c = 0; c < MAXC; c++)
                if (c < C) *reinterpret_cast<float2*>(hb + halo_row_offset(C, S, ix, y, c)) = make_float2(0.f, 0.f);
        }
        if (rx == 0 || rx == HALO_TW - 2) {
            const int x = rx == 0 ? ix : ix + 1;
#pragma unroll
            for (int c = 0; c < MAXC; c++) {
                if (c < C) {
                    hb[halo_col_offset(C, S, x, iy, c)] = 0.f;
                    hb[halo_col_offset(C, S, x, iy + 1, c)] = 0.f;
                }
            }
        }
    }
}

// ------------------------------------------------------------------------------------------------
// k_shade: the image channels from the face-index map, one thread per OUTPUT pixel (rasterize.py:
// 237-328): weights (compute_weight_map), texture sample, silhouette and depth for the 1 or 2x2
// internal pixels it covers, merged in rgb/sil/depth order, flipped, and 2x2-averaged with the
// reference's summation order.  Kept out of the rasteriser so that kernel stays lean (registers,
// occupancy); costs one extra read of the face-index map.
// 6 waves/SIMD: up to 80 VGPRs, no spills with the packed-texel path (7: a 2-dword spill, same time)
constexpr int SHADE_WPE = 6;
template <int FEAT>  // 1 = lights, 2 = backgrounds, as k_raster_bwd
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu((FEAT & 1) ? 1 : SHADE_WPE, 8))) void k_shade(const float* __restrict__ face_records, const int32_t* __restrict__ fim,
                                               int F, int S, Shade sh_in, int aa, float* __restrict__ images,
                                               float* __restrict__ halo) {
    Shade sh = sh_in;
    if (!(FEAT & 1)) sh.nl = 0;
    if (!(FEAT & 2)) sh.bg = nullptr;
    const int s = aa ? S / 2 : S;
    const int b = blockIdx.y;
    int blk = blockIdx.x, unused;
    xcd_tile(blockIdx.x, b, 1, gridDim.x, unused, blk);
    const int o = blk * blockDim.x + threadIdx.x;
    if (o >= s * s) return;
    const int oi = o / s, oj = o - oi * s;
    const float* frb = face_records + (long long)b * F * FACE_REC;
    const int32_t* fb = fim + (long long)b * S * S;
    float* ob = images + (long long)b * sh.C * s * s + o;
    if (!aa) {
        // permute to [B, C, S, S] and flip both axes (rasterize.py:315-316)
        const int y = S - 1 - oi, x = S - 1 - oj;
        const int fi = fb[y * S + x];
        Face f;
        FaceUV u;
        load_shading_face(sh, frb, b, fi, f, u);
        float v[MAXC];
        shade_pixel(sh, b, fi, f, u, x, y, pix_center(x, S), pix_center(y, S), S, v);
#pragma unroll
        for (int c = 0; c < MAXC; c++)
            if (c < sh.C) ob[c * s * s] = v[c];
        if (halo) halo_store(halo, b, sh.C, S, x, y, v);
        return;
    }
    // 2x2 average of the flipped image (rasterize.py:321-328): output (oi, oj) reads internal rows
    // iy, iy+1 and columns ix, ix+1 with a=(iy+1,ix+1) b=(iy,ix+1) c=(iy+1,ix) d=(iy,ix)
    const int iy = S - 2 - 2 * oi, ix = S - 2 - 2 * oj;
    const int2 f0 = *reinterpret_cast<const int2*>(fb + iy * S + ix);        // d, b
    const int2 f1 = *reinterpret_cast<const int2*>(fb + (iy + 1) * S + ix);  // c, a
    const int fis[4] = {f1.y, f0.y, f1.x, f0.x};
    shade_quad(sh, frb, b, S, iy, ix, fis, images, halo);
}

// ------------------------------------------------------------------------------------------------
// compute_weight_map (standalone entry point): one thread per pixel
// k_shade_px: the same as k_shade with one thread per INTERNAL pixel.  k_shade's thread shades its
// 2x2 quad in turn, each pixel a chain of three dependent loads (face-index map -> face / uv records
// -> texels), so a wave waits on 12 serialised load latencies; here the four pixels of an output
// pixel are four lanes of a DPP quad (lane q of the quad: q = 0 a=(iy+1,ix+1), 1 b=(iy,ix+1),
// 2 c=(iy+1,ix), 3 d=(iy,ix)), their chains run concurrently, and the 2x2 mean is summed with
// quad_perm broadcasts in the reference's order ((a + b) + c) + d (rasterize.py:321-328).  A block
// covers 64 consecutive output pixels of one output row.  Without anti-aliasing a thread is one
// output pixel.  Every internal pixel on a backward tile border stores itself to the halo cache.
// Measured: k_shade_px is faster only when the grid is small (teapot B=4: 0.0176 -> 0.0136 ms); on the
// headline the 2x2-per-thread k_shade wins (0.121 vs 0.164 ms: shading is VALU-bound there, and the
// per-pixel form repeats the per-thread overheads 4x), so it is picked by grid size (run_face_index).
template <int FEAT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu((FEAT & 1) ? 1 : 8, 8))) void k_shade_px(const float* __restrict__ face_records, const int32_t* __restrict__ fim,
                                                  int F, int S, Shade sh_in, int aa, float* __restrict__ images,
                                                  float* __restrict__ halo) {
    Shade sh = sh_in;
    if (!(FEAT & 1)) sh.nl = 0;
    if (!(FEAT & 2)) sh.bg = nullptr;
    const int s = aa ? S / 2 : S;
    const int b = blockIdx.y;
    const int t = threadIdx.x;
    const float* frb = face_records + (long long)b * F * FACE_REC;
    const int32_t* fb = fim + (long long)b * S * S;
    int o, x, y;
    if (aa) {
        o = blockIdx.x * 64 + (t >> 2);  // output pixel of this quad
        const int q = t & 3;
        const int oo = min(o, s * s - 1);
        const int oi = oo / s, oj = oo - oi * s;
        const int iy = S - 2 - 2 * oi, ix = S - 2 - 2 * oj;
        y = iy + ((q & 1) ? 0 : 1);
        x = ix + ((q & 2) ? 0 : 1);
    } else {
        o = blockIdx.x * 256 + t;
        const int oo = min(o, s * s - 1);
        const int oi = oo / s, oj = oo - oi * s;
        y = S - 1 - oi;
        x = S - 1 - oj;
    }
    const int fi = fb[y * S + x];
    Face f;
    FaceUV u;
    load_shading_face(sh, frb, b, fi, f, u);
    float v[MAXC];
    shade_pixel(sh, b, fi, f, u, x, y, pix_center(x, S), pix_center(y, S), S, v);
    const bool live = o < s * s;
    if (halo && live) halo_store(halo, b, sh.C, S, x, y, v);
    float* ob = images + (long long)b * sh.C * s * s + o;
    if (!aa) {
#pragma unroll
        for (int c = 0; c < MAXC; c++)
            if (c < sh.C && live) ob[c * s * s] = v[c];
        return;
    }
#pragma unroll
    for (int c = 0; c < MAXC; c++) {
        if (c < sh.C) {
            const int bits = __float_as_int(v[c]);
            const float va = __int_as_float(__builtin_amdgcn_mov_dpp(bits, 0x00, 0xf, 0xf, false));
            const float vb = __int_as_float(__builtin_amdgcn_mov_dpp(bits, 0x55, 0xf, 0xf, false));
            const float vc = __int_as_float(__builtin_amdgcn_mov_dpp(bits, 0xaa, 0xf, 0xf, false));
            const float vd = __int_as_float(__builtin_amdgcn_mov_dpp(bits, 0xff, 0xf, 0xf, false));
            if ((t & 3) == 0 && live) ob[c * s * s] = (((va + vb) + vc) + vd) / 4.f;
        }
    }
}

__global__ void k_weight_map(const float* __restrict__ faces, const int32_t* __restrict__ fim, float* __restrict__ wm,
                             int F, int S, long long n) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int fi = fim[i];
    float w[3] = {0.f, 0.f, 0.f};
    if (fi >= 0) {
        const long long ss = (long long)S * S;
        const int bn = (int)(i / ss);
        const int pn = (int)(i % ss);
        const Face f = load_face(faces + ((long long)bn * F + fi) * 9);
        face_weights(pix_center(pn % S, S), pix_center(pn / S, S), f, w);
    }
    wm[i * 3 + 0] = w[0];
    wm[i * 3 + 1] = w[1];
    wm[i * 3 + 2] = w[2];
}

__global__ void k_mask_fg(const int32_t* __restrict__ fi, const float* __restrict__ src, float* __restrict__ dst,
                          long long n, int dim) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || fi[i] < 0) return;
    for (int j = 0; j < dim; j++) dst[i * dim + j] = src[i * dim + j];
}

// ------------------------------------------------------------------------------------------------
// Differentiation.backward stencil (differentiation.py:12-36, utils.py:75-101)
//   r[i] = -(sum_c (I[i]-I[i+1]) G[i+1]) / step,  l[i] = -(sum_c (I[i+1]-I[i]) G[i]) / step
//   R[i] = r[i] + r[i-1], L[i] = l[i-1] + l[i] (missing terms 0), then maximum(R, L)
__device__ __forceinline__ float pair_dot(const float* a, const float* b, const float* g, int C) {
    float s = (a[0] - b[0]) * g[0];
#pragma unroll
    for (int c = 1; c < MAXC; c++)
        if (c < C) s = s + (a[c] - b[c]) * g[c];
    return s;
}

// arr[i] for a runtime i < MAXC without a runtime-indexed (scratch) access
__device__ __forceinline__ float pick(const float* arr, int i) {
    float v = arr[0];
#pragma unroll
    for (int c = 1; c < MAXC; c++) v = (i == c) ? arr[c] : v;
    return v;
}

__device__ __forceinline__ float pick_grad(float R, float L) {
    // utils.maximum: start from L; R > L -> -R; |R-L| < 1e-4 -> 0; max(R, L) <= 0 -> 0
    float out = (R > L) ? -R : L;
    if (fabsf(R - L) < 1e-4f) out = 0.f;
    if (fmaxf(R, L) <= 0.f) out = 0.f;
    return out;
}

// grad along one axis at position i of n, given the channel vectors of (i-1, i, i+1)
__device__ __forceinline__ float axis_grad(const float* Im, const float* I0, const float* Ip, const float* Gm,
                                           const float* G0, const float* Gp, int i, int n, int C, float step) {
    const bool has_p = i <= n - 2, has_m = i >= 1;
    const float r_i = has_p ? -pair_dot(I0, Ip, Gp, C) / step : 0.f;
    const float r_m = has_m ? -pair_dot(Im, I0, G0, C) / step : 0.f;
    const float l_i = has_p ? -pair_dot(Ip, I0, G0, C) / step : 0.f;
    const float l_m = has_m ? -pair_dot(I0, Im, Gm, C) / step : 0.f;
    return pick_grad(r_i + r_m, l_m + l_i);
}

__global__ void k_diff_bwd(const float* __restrict__ img, const float* __restrict__ grad, float* __restrict__ gxy, int H,
                           int W, int C, float step, long long n) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const long long hw = (long long)H * W;
    const int b = (int)(i / hw);
    const int p = (int)(i % hw);
    const int y = p / W, x = p % W;
    auto at = [&](const float* base, int yy, int xx, int c) -> float {
        return base[(((long long)b * H + yy) * W + xx) * C + c];
    };
    // generic-C pair dots without local arrays
    auto dot = [&](int ya, int xa, int yb, int xb, int yg, int xg) -> float {
        float s = (at(img, ya, xa, 0) - at(img, yb, xb, 0)) * at(grad, yg, xg, 0);
        for (int c = 1; c < C; c++) s = s + (at(img, ya, xa, c) - at(img, yb, xb, c)) * at(grad, yg, xg, c);
        return s;
    };
    float gx, gy;
    {
        const bool hp = x <= W - 2, hm = x >= 1;
        const float r_i = hp ? -dot(y, x, y, x + 1, y, x + 1) / step : 0.f;
        const float r_m = hm ? -dot(y, x - 1, y, x, y, x) / step : 0.f;
        const float l_i = hp ? -dot(y, x + 1, y, x, y, x) / step : 0.f;
        const float l_m = hm ? -dot(y, x, y, x - 1, y, x - 1) / step : 0.f;
        gx = pick_grad(r_i + r_m, l_m + l_i);
    }
    {
        const bool hp = y <= H - 2, hm = y >= 1;
        const float r_i = hp ? -dot(y, x, y + 1, x, y + 1, x) / step : 0.f;
        const float r_m = hm ? -dot(y - 1, x, y, x, y, x) / step : 0.f;
        const float l_i = hp ? -dot(y + 1, x, y, x, y, x) / step : 0.f;
        const float l_m = hm ? -dot(y, x, y - 1, x, y - 1, x) / step : 0.f;
        gy = pick_grad(r_i + r_m, l_m + l_i);
    }
    gxy[i * 2 + 0] = gx;
    gxy[i * 2 + 1] = gy;
}

}  // namespace
