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
#include <hip/hip_runtime.h>

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

namespace {

constexpr int TW = 32;             // tile width  (internal pixels)
constexpr int TH = 8;              // tile height
constexpr int NT = TW * TH;        // threads per raster block, one pixel each
constexpr int COARSE = 32;         // coarse bin edge (pixels) = forward block region; = TW, multiple of TH
constexpr int SETUP_FACES = 128;   // faces per setup block (4 bitmask words)
constexpr int SETUP_LDS_WORDS = 4096;  // bin-mask words built in LDS (up to 1024 bins, S <= 1024)
constexpr int MAXC = 5;            // max output channels

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

int check_launch(const char* what) {
    hipError_t e = hipPeekAtLastError();
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return fail(NR_ERR_LAUNCH, "%s: %s", what, hipGetErrorString(e));
    }
    return NR_OK;
}

// ---- measurement hook (nr_profile_enable / nr_profile_read) ----
enum { P_SETUP, P_RASTER, P_SHADE, P_BWD, P_VGRAD, P_TEXOUT, P_TEXPACK, P_N };
const char* const kProfNames[P_N] = {"k_face_setup", "k_raster_fwd", "k_shade",
                                     "k_raster_bwd", "k_vertex_grad", "k_tex_out", "k_tex_pack"};
bool g_prof = false;
hipEvent_t g_prof_ev[P_N][2];
bool g_prof_rec[P_N];

struct ProfScope {  // records the start/end events of one launch when profiling is on
    int k;
    hipStream_t st;
    ProfScope(int k_, hipStream_t s) : k(k_), st(s) {
        if (g_prof) (void)hipEventRecord(g_prof_ev[k][0], st);
    }
    ~ProfScope() {
        if (g_prof) {
            (void)hipEventRecord(g_prof_ev[k][1], st);
            g_prof_rec[k] = true;
        }
    }
};

struct Geom {
    int S, nbx, nby, nbins, nwords, tiles_x, tiles_y;
};

Geom make_geom(int F, int S) {
    Geom g;
    g.S = S;
    g.nbx = (S + COARSE - 1) / COARSE;
    g.nby = g.nbx;
    g.nbins = g.nbx * g.nby;
    g.nwords = (F + 31) / 32;
    g.tiles_x = (S + TW - 1) / TW;
    g.tiles_y = (S + TH - 1) / TH;
    return g;
}

size_t align_up(size_t x) { return (x + 255) & ~size_t(255); }

// workspace layout: [bbox int2 B*F][mask u32 B*nbins*nwords]
size_t ws_bbox_bytes(int B, int F) { return align_up((size_t)B * F * sizeof(int2)); }
size_t ws_mask_bytes(int B, const Geom& g) { return align_up((size_t)B * g.nbins * g.nwords * 4); }

// ------------------------------------------------------------------------------------------------
// device helpers

// rasterize_cuda_kernel.cu:76-77: pixel centre, computed in double, rounded to float
__device__ __forceinline__ float pix_center(int i, int S) { return (float)((2. * i + 1 - S) / S); }

// conservative range of pixel indices whose centre may lie in [lo, hi] (float compare).  Empty
// when lo > hi.  One pixel of margin on each side absorbs the float rounding of the centres.
__device__ __forceinline__ void pix_range(float lo, float hi, int S, int& i0, int& i1) {
    double a = ((double)lo * S + S - 1) * 0.5;
    double b = ((double)hi * S + S - 1) * 0.5;
    a = fmin(fmax(a, -2.0), (double)S + 2.0);
    b = fmin(fmax(b, -2.0), (double)S + 2.0);
    i0 = max((int)ceil(a) - 1, 0);
    i1 = min((int)floor(b) + 1, S - 1);
}

__device__ __forceinline__ int pack_range(int lo, int hi) { return (lo & 0xffff) | (hi << 16); }
// an empty range never overlaps anything: lo = 32767 > any pixel index, hi = -1
#define NR_EMPTY_RANGE ((int)0xffff7fff)
__device__ __forceinline__ int range_lo(int p) { return p & 0xffff; }
__device__ __forceinline__ int range_hi(int p) { return p >> 16; }

// A gathered face.  The fused path keeps 16-float face records (FACE_REC floats, 64 B, one aligned
// load of 4 x float4): the 9 corner coordinates, then per-face reciprocals for the exact division
// shortcut (rcp_nr(z_k), rcp_nr(z_k + 1e-10)) and the operand-range flags that allow it.  Faces
// handed over by the caller (face_index_map_forward_safe, compute_weight_map) are 9 floats and
// always take the plain IEEE divisions (flags = 0).
constexpr int FACE_REC = 16;
constexpr int FACE_FAST_XYZ = 1;  // x, y in {0} u [2^-20, 2^20], |z| in [2^-20, 2^20]
constexpr int FACE_FAST_ZQ = 2;   // |z + 1e-10| in [2^-20, 2^20]
struct Face {
    float x0, y0, z0, x1, y1, z1, x2, y2, z2;
    float rz0, rz1, rz2, rq0, rq1, rq2;
    int flags;
};

__device__ __forceinline__ Face load_face(const float* __restrict__ fr) {
    Face f;
    f.x0 = fr[0]; f.y0 = fr[1]; f.z0 = fr[2];
    f.x1 = fr[3]; f.y1 = fr[4]; f.z1 = fr[5];
    f.x2 = fr[6]; f.y2 = fr[7]; f.z2 = fr[8];
    f.rz0 = f.rz1 = f.rz2 = f.rq0 = f.rq1 = f.rq2 = 0.f;
    f.flags = 0;
    return f;
}

__device__ __forceinline__ Face load_face_rec(const float* __restrict__ fr) {
    const float4* p = reinterpret_cast<const float4*>(fr);
    const float4 a = p[0], b = p[1], c = p[2], d = p[3];
    Face f;
    f.x0 = a.x; f.y0 = a.y; f.z0 = a.z;
    f.x1 = a.w; f.y1 = b.x; f.z1 = b.y;
    f.x2 = b.z; f.y2 = b.w; f.z2 = c.x;
    f.rz0 = c.y; f.rz1 = c.z; f.rz2 = c.w;
    f.rq0 = d.x; f.rq1 = d.y; f.rq2 = d.z;
    f.flags = __float_as_int(d.w);
    return f;
}

__device__ __forceinline__ Face empty_face() {
    Face f = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    return f;
}

// torch.maximum / torch.minimum / min(-2) / max(-2) semantics: NaN propagates
__device__ __forceinline__ float t_max(float a, float b) { return (a != a || b != b) ? __builtin_nanf("") : (a > b ? a : b); }
__device__ __forceinline__ float t_min(float a, float b) { return (a != a || b != b) ? __builtin_nanf("") : (a < b ? a : b); }

// ---- exact division without the scaling / fix-up steps --------------------------------------
// gfx950 lowers an IEEE binary32 a / b to
//   v_div_scale(b), v_rcp, v_div_scale(a), r = fma(fma(-b, rcp, 1), rcp, rcp), q = a * r,
//   q = fma(fma(-b, q, a), r, q), v_div_fmas(fma(-b, q, a), r, q), v_div_fixup.
// v_div_scale leaves its operand unchanged and clears VCC, and v_div_fixup returns its input, unless
// an operand is zero / inf / NaN / denormal, the quotient or 1/b is denormal, the numerator is below
// 2^-103, or the exponents differ by 96 or more.  Outside those cases the sequence is exactly
// rcp_nr + div_nr below, so div_nr is bit-identical to a / b there, and a reciprocal shared by
// several divisions by the same b is computed once.  Callers guard the operand ranges (DESIGN.md
// "Numerics"); a zero numerator may come out as +0 where a / b gives -0, which no caller observes.
__device__ __forceinline__ float rcp_nr(float b) {
    const float r = __builtin_amdgcn_rcpf(b);
    return __builtin_fmaf(__builtin_fmaf(-b, r, 1.f), r, r);
}
__device__ __forceinline__ float div_nr(float a, float b, float r) {
    float q = a * r;
    q = __builtin_fmaf(__builtin_fmaf(-b, q, a), r, q);
    return __builtin_fmaf(__builtin_fmaf(-b, q, a), r, q);
}
// |x| in [2^-e, 2^e]
__device__ __forceinline__ bool in_range(float x, float lo, float hi) { return fabsf(x) >= lo && fabsf(x) <= hi; }
// coordinate / depth magnitudes for which the face-level guard below holds: 0 or [2^-20, 2^20]
__device__ __forceinline__ bool coord_ok(float x) { return x == 0.f || in_range(x, 0x1p-20f, 0x1p20f); }

// compute_weight_map_cuda_kernel (.cu:286-306).  Returns true when the weights are known to lie in
// {0} u [2^-84, 1] (the exact-division path was taken), which the texture and depth stages below
// need for their own shortcut.
__device__ __forceinline__ bool face_weights(float xp, float yp, const Face& f, float w[3]) {
    w[0] = yp * (f.x2 - f.x1) + xp * (f.y1 - f.y2) + (f.x1 * f.y2 - f.x2 * f.y1);
    w[1] = yp * (f.x0 - f.x2) + xp * (f.y2 - f.y0) + (f.x2 * f.y0 - f.x0 * f.y2);
    w[2] = yp * (f.x1 - f.x0) + xp * (f.y0 - f.y1) + (f.x0 * f.y1 - f.x1 * f.y0);
    float s = w[0] + w[1] + w[2];
    if (s < 0) {
        w[0] = -w[0];
        w[1] = -w[1];
        w[2] = -w[2];
    }
    w[0] = fmaxf(w[0], 0.f);
    w[1] = fmaxf(w[1], 0.f);
    w[2] = fmaxf(w[2], 0.f);
    s = w[0] + w[1] + w[2];
    // with FACE_FAST_XYZ every w is 0 or in [2^-80, 2^42] (DESIGN.md "Numerics")
    if ((f.flags & FACE_FAST_XYZ) && in_range(s, 0x1p-20f, 0x1p4f)) {
        const float r = rcp_nr(s);
#pragma unroll
        for (int j = 0; j < 3; j++) w[j] = fmaxf(fminf(div_nr(w[j], s, r), 1.f), 0.f);
        return true;
    }
#pragma unroll
    for (int j = 0; j < 3; j++) w[j] = fmaxf(fminf(w[j] / s, 1.f), 0.f);
    return false;
}

// 1 / x through div_nr's range (|x| in [2^-90, 2^90]), else IEEE
__device__ __forceinline__ float recip_exact(float x) {
    if (in_range(x, 0x1p-90f, 0x1p90f)) {
        const float r = rcp_nr(x);
        const float q = __builtin_fmaf(__builtin_fmaf(-x, r, 1.f), r, r);  // div_nr(1, x, r): 1 * r == r
        return __builtin_fmaf(__builtin_fmaf(-x, q, 1.f), r, q);
    }
    return 1.f / x;
}

struct TexView {
    const float* __restrict__ tex;
    long long sb;   // item stride (uniform 64-bit part)
    int sc, sp;     // channel / texel strides: one item's view spans < 2^31 elements (validate_raster)
    int H, W;
    // the same texels packed as RGBA rows [Bt][HWp] (NrRasterArgs.textures_packed), or null: one 16-B
    // load per bilinear corner, and 2 cache lines per pixel instead of 6 (3 channel planes x 2 rows)
    const float4* __restrict__ t4;
    int HWp;
};

__device__ __forceinline__ float texel(const TexView& t, int b, int c, int p) {
    return t.tex[(long long)b * t.sb + (c * t.sc + p * t.sp)];
}

// sample_textures (rasterize.py:100-153) for one foreground pixel, with the intermediates the
// backward needs.
struct TexSample {
    float zq[3];        // z_k + 1e-10
    float dt;           // 1 / sum(w/(z+1e-10) + 1e-10)
    float num[2];       // sum_k (w_k uv_k)/(z_k + 1e-10)
    float pr[2];        // num * dt (pre-clamp)
    float pc[2];        // after the lower clamp
    float hm[2];        // upper bound (max uv - eps)
    float lo[2];
    float x, y, x0, y0, x1, y1;
    int idx[4];
    float wt[4];
    float rgb[3];
};

// uv: the face's 8-float texture record (u0 v0 u1 v1 u2 v2, flag, -); flag 1 = every u, v in
// {0} u [2^-16, 2^20].  wfast: face_weights took its exact-division path.
// G (optional, backward): upstream gradient of the rgb channels; then gw[i] = sum_c G[c] T_i[c] for
// the 4 bilinear texels, from the texel values loaded here (no second load)
__device__ __forceinline__ void sample_texture(const Face& f, const float w[3], bool wfast, const float* __restrict__ uv,
                                               const TexView& tv, int bt, float eps, TexSample& s,
                                               const float* G = nullptr, float* gw = nullptr) {
    const float4 uva = reinterpret_cast<const float4*>(uv)[0], uvb = reinterpret_cast<const float4*>(uv)[1];
    const float uvs[6] = {uva.x, uva.y, uva.z, uva.w, uvb.x, uvb.y};
    const bool fast = wfast && (f.flags & FACE_FAST_ZQ) && __float_as_int(uvb.z) != 0;
    const float z[3] = {f.z0, f.z1, f.z2};
    const float rq[3] = {f.rq0, f.rq1, f.rq2};
    float st = 0.f;
#pragma unroll
    for (int k = 0; k < 3; k++) {
        s.zq[k] = z[k] + 1e-10f;
        const float t = (fast ? div_nr(w[k], s.zq[k], rq[k]) : w[k] / s.zq[k]) + 1e-10f;
        st = (k == 0) ? t : st + t;
    }
    s.dt = fast ? recip_exact(st) : 1.f / st;
#pragma unroll
    for (int j = 0; j < 2; j++) {
        const float u0 = uvs[j], u1 = uvs[2 + j], u2 = uvs[4 + j];
        if (fast)
            s.num[j] = (div_nr(w[0] * u0, s.zq[0], rq[0]) + div_nr(w[1] * u1, s.zq[1], rq[1])) +
                       div_nr(w[2] * u2, s.zq[2], rq[2]);
        else
            s.num[j] = ((w[0] * u0) / s.zq[0] + (w[1] * u1) / s.zq[1]) + (w[2] * u2) / s.zq[2];
        s.pr[j] = s.num[j] * s.dt;
        s.lo[j] = t_min(t_min(u0, u1), u2);
        s.hm[j] = t_max(t_max(u0, u1), u2) - eps;
        s.pc[j] = t_max(s.pr[j], s.lo[j]);
    }
    s.x = t_min(s.pc[0], s.hm[0]);
    s.y = t_min(s.pc[1], s.hm[1]);
    s.x0 = floorf(s.x);
    s.y0 = floorf(s.y);
    s.x1 = s.x0 + 1;
    s.y1 = s.y0 + 1;
    const int xi0 = (int)s.x0, yi0 = (int)s.y0, xi1 = (int)s.x1, yi1 = (int)s.y1;
    const int W = tv.W, HW = tv.H * tv.W;
    s.idx[0] = yi0 * W + xi0;
    s.idx[1] = yi0 * W + xi1;
    s.idx[2] = yi1 * W + xi0;
    s.idx[3] = yi1 * W + xi1;
#pragma unroll
    for (int i = 0; i < 4; i++) s.idx[i] = min(max(s.idx[i], 0), HW - 1);  // weight-0 overhang, SURVEY A9
    s.wt[0] = (s.y1 - s.y) * (s.x1 - s.x);
    s.wt[1] = (s.y1 - s.y) * (s.x - s.x0);
    s.wt[2] = (s.y - s.y0) * (s.x1 - s.x);
    s.wt[3] = (s.y - s.y0) * (s.x - s.x0);
    const float* tb = tv.tex + (long long)bt * tv.sb;
    int off[4];
    float4 q4[4];
    if (tv.t4) {
        const float4* t4b = tv.t4 + (long long)bt * tv.HWp;
#pragma unroll
        for (int i = 0; i < 4; i++) q4[i] = t4b[s.idx[i]];
    } else {
#pragma unroll
        for (int i = 0; i < 4; i++) off[i] = s.idx[i] * tv.sp;
    }
#pragma unroll
    for (int c = 0; c < 3; c++) {
        const float* tc = tb + c * tv.sc;
        float t0, t1, t2, t3;
        if (tv.t4) {
            t0 = c == 0 ? q4[0].x : (c == 1 ? q4[0].y : q4[0].z);
            t1 = c == 0 ? q4[1].x : (c == 1 ? q4[1].y : q4[1].z);
            t2 = c == 0 ? q4[2].x : (c == 1 ? q4[2].y : q4[2].z);
            t3 = c == 0 ? q4[3].x : (c == 1 ? q4[3].y : q4[3].z);
        } else {
            t0 = tc[off[0]], t1 = tc[off[1]], t2 = tc[off[2]], t3 = tc[off[3]];
        }
        s.rgb[c] = ((s.wt[0] * t0 + s.wt[1] * t1) + s.wt[2] * t2) + s.wt[3] * t3;
        if (G) {
            if (c == 0) {
                gw[0] = G[0] * t0;
                gw[1] = G[0] * t1;
                gw[2] = G[0] * t2;
                gw[3] = G[0] * t3;
            } else {
                gw[0] = gw[0] + G[c] * t0;
                gw[1] = gw[1] + G[c] * t1;
                gw[2] = gw[2] + G[c] * t2;
                gw[3] = gw[3] + G[c] * t3;
            }
        }
    }
}

// compute_depth_map (rasterize.py:80-88) for a foreground pixel
__device__ __forceinline__ float depth_value(const Face& f, const float w[3], bool wfast) {
    if (wfast) {  // weights in {0} u [2^-84, 1], |z| in [2^-20, 2^20]
        return recip_exact((div_nr(w[0], f.z0, f.rz0) + div_nr(w[1], f.z1, f.rz1)) + div_nr(w[2], f.z2, f.rz2));
    }
    return 1.f / ((w[0] / f.z0 + w[1] / f.z1) + w[2] / f.z2);
}

struct Shade {
    int draw;       // NR_DRAW_* flags
    int C;          // channels
    float eps;
    TexView tv;
    const float* __restrict__ face_uv;
    long long uv_bstride;  // F*8 or 0
    // lights (rgb only): records [nl][B][NR_LIGHT_FLOATS], vertex normals [B, V, 4], face corners
    int nl, B, V;
    const float* __restrict__ lights;
    const float* __restrict__ vnorm;
    const int32_t* __restrict__ fidx;
    // backgrounds (rgb only): [B, 3, S, S], x stride 1
    const float* __restrict__ bg;
    long long bg_sb;
    int bg_sc, bg_sy;
};

// torch.relu (NaN stays NaN)
__device__ __forceinline__ float t_relu(float x) { return x > 0.f ? x : (x != x ? x : 0.f); }

// smooth normal map at a pixel of face fi (rasterize.py:185-187): sum_k w_k n_k over the face's
// corner vertex normals, per component ((w0 n0 + w1 n1) + w2 n2)
__device__ __forceinline__ void pixel_normal(const Shade& sh, int b, int fi, const float w[3], float n[3]) {
    const float* vb = sh.vnorm + (long long)b * sh.V * 4;
    float c[3][3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const float4 v = *reinterpret_cast<const float4*>(vb + sh.fidx[fi * 3 + k] * 4);
        c[k][0] = v.x;
        c[k][1] = v.y;
        c[k][2] = v.z;
    }
#pragma unroll
    for (int j = 0; j < 3; j++) n[j] = (w[0] * c[0][j] + w[1] * c[1][j]) + w[2] * c[2][j];
}

// the light loop of rasterize.py:252-281 for one pixel: colour weights cw (starting from 0, lights
// added in list order); with gcw != nullptr, instead accumulate dL/dn into gn given dL/dcw = gcw
__device__ __forceinline__ void light_weights(const Shade& sh, int b, const float n[3], float cw[3],
                                              const float* gcw = nullptr, float* gn = nullptr) {
    cw[0] = cw[1] = cw[2] = 0.f;
    for (int l = 0; l < sh.nl; l++) {
        const float* L = sh.lights + ((long long)l * sh.B + b) * NR_LIGHT_FLOATS;
        const int kind = (int)L[0];
        const bool back = L[1] != 0.f;
        const float col[3] = {L[2], L[3], L[4]};
        if (kind == NR_LIGHT_AMBIENT) {
#pragma unroll
            for (int c = 0; c < 3; c++) cw[c] = cw[c] + col[c];
            continue;
        }
        // intensity = sum(-d * n) with d the light direction, or (0, 0, 1) for specular
        const float d0 = kind == NR_LIGHT_DIRECTIONAL ? L[5] : 0.f;
        const float d1 = kind == NR_LIGHT_DIRECTIONAL ? L[6] : 0.f;
        const float d2 = kind == NR_LIGHT_DIRECTIONAL ? L[7] : 1.f;
        const float raw = ((-d0) * n[0] + (-d1) * n[1]) + (-d2) * n[2];
        float s = back ? fabsf(raw) : t_relu(raw);
        const float alpha = L[5];
        float ds = back ? (raw > 0.f ? 1.f : (raw < 0.f ? -1.f : 0.f)) : (raw > 0.f ? 1.f : 0.f);  // d s / d raw
        if (kind == NR_LIGHT_SPECULAR) {
            const float p = powf(s, alpha);
            ds = ds * (alpha * powf(s, alpha - 1.f));  // torch pow backward: exponent * base^(exponent - 1)
            s = p;
        }
#pragma unroll
        for (int c = 0; c < 3; c++) cw[c] = cw[c] + s * col[c];
        if (gn) {
            const float gs = ((gcw[0] * col[0] + gcw[1] * col[1]) + gcw[2] * col[2]) * ds;
            gn[0] += gs * (-d0);
            gn[1] += gs * (-d1);
            gn[2] += gs * (-d2);
        }
    }
}

// background colour of internal pixel (x, y): backgrounds[b, c, S-1-y, S-1-x]
__device__ __forceinline__ void background(const Shade& sh, int b, int x, int y, int S, float bgc[3]) {
    const float* p = sh.bg + (long long)b * sh.bg_sb + (S - 1 - y) * sh.bg_sy + (S - 1 - x);
#pragma unroll
    for (int c = 0; c < 3; c++) bgc[c] = p[c * sh.bg_sc];
}

// All channels of one internal pixel (rasterize.py:295-310 merge order: rgb, sil, depth), written
// to compile-time slots of out[MAXC] (runtime-indexed register arrays would spill to scratch).
__device__ __forceinline__ void shade_pixel(const Shade& sh, int b, int fi, const Face& f, int x, int y, int S,
                                            float* out) {
    const bool R = (sh.draw & NR_DRAW_RGB) != 0, Sl = (sh.draw & NR_DRAW_SILHOUETTES) != 0;
    const float xp = pix_center(x, S), yp = pix_center(y, S);
    float r = 0.f, gg = 0.f, bb = 0.f, sil = 0.f, dep = 0.f;
    if (fi >= 0) {
        float w[3];
        const bool wfast = face_weights(xp, yp, f, w);
        if (R) {
            TexSample s;
            const float* fuv = sh.face_uv + (sh.uv_bstride ? (long long)b * sh.uv_bstride : 0) + fi * 8;
            sample_texture(f, w, wfast, fuv, sh.tv, sh.tv.sb ? b : 0, sh.eps, s);
            r = s.rgb[0];
            gg = s.rgb[1];
            bb = s.rgb[2];
            if (sh.nl) {  // rgb_map *= color_weight_map (rasterize.py:283)
                float n[3], cw[3];
                pixel_normal(sh, b, fi, w, n);
                light_weights(sh, b, n, cw);
                r = r * cw[0];
                gg = gg * cw[1];
                bb = bb * cw[2];
            }
        }
        sil = 1.f;
        if (sh.draw & NR_DRAW_DEPTH) dep = depth_value(f, w, wfast);
    }
    if (R && sh.bg) {  // fg * rgb + (1 - fg) * bg (chainer rasterize.py:576)
        float bgc[3];
        background(sh, b, x, y, S, bgc);
        const float fg = fi >= 0 ? 1.f : 0.f;
        r = fg * r + (1.f - fg) * bgc[0];
        gg = fg * gg + (1.f - fg) * bgc[1];
        bb = fg * bb + (1.f - fg) * bgc[2];
    }
    out[0] = R ? r : (Sl ? sil : dep);
    out[1] = R ? gg : dep;
    out[2] = bb;
    out[3] = Sl ? sil : dep;
    out[4] = dep;
}

// ------------------------------------------------------------------------------------------------
// XCD-aware block -> tile map.  Workgroups go round-robin to the 8 XCDs (linear id % 8) and each XCD
// has its own L2, so with the identity map horizontally adjacent tiles never share a cache, and the
// halo columns, upstream-gradient lines and face records they have in common are fetched once per
// XCD.  Two remaps (measured on the headline workload):
//   mode 1 (groups): runs of SW x SH neighbouring tiles go to one XCD back to back; groups
//          interleave over the XCDs.  Full tile rows (SW = nx, SH = 1) are the balanced case.
//   mode 2 (bands):  XCD x takes a band of ny / 8 whole tile rows of each item, the band rotating
//          with the item so every XCD sees every band over 8 items (balanced over the batch).
// Both fall back to the identity when the grid does not divide evenly (the linear id of item b
// starts at b * nx * ny, a multiple of 8 whenever the remap applies).
#ifndef NR_SWZ_MODE
#define NR_SWZ_MODE 2
#endif
#ifndef NR_SWZ_W
#define NR_SWZ_W 0  // 0: the full tile row
#endif
#ifndef NR_SWZ_H
#define NR_SWZ_H 1
#endif
#ifndef NR_FSWZ_MODE
#define NR_FSWZ_MODE 2
#endif
#ifndef NR_FSWZ_W
#define NR_FSWZ_W 0
#endif
#ifndef NR_SSWZ_MODE
#define NR_SSWZ_MODE 0
#endif
#ifndef NR_FSWZ_H
#define NR_FSWZ_H 1
#endif
template <int MODE, int SW_, int SH>
__device__ __forceinline__ void xcd_tile(int L, int b, int nx, int ny, int& tx, int& ty) {
    tx = L % nx;
    ty = L / nx;
    if (MODE == 1) {
        const int SW = SW_ > 0 ? SW_ : nx;
        const int per = SW * SH;
        const int ngx = nx / SW;
        if (per > 1 && nx % SW == 0 && ny % SH == 0 && (ngx * (ny / SH)) % 8 == 0) {
            const int j = L >> 3, xcd = L & 7;
            const int grp = (j / per) * 8 + xcd;
            const int q = j % per;
            tx = (grp % ngx) * SW + q % SW;
            ty = (grp / ngx) * SH + q / SW;
        }
    } else if (MODE == 2) {
        if (ny % 8 == 0) {
            const int j = L >> 3, xcd = L & 7;
            const int band = (xcd + b) & 7;
            tx = j % nx;
            ty = band * (ny >> 3) + j / nx;
        }
    }
}

// ------------------------------------------------------------------------------------------------
// block-wide exclusive scan of one int per thread (NW waves)
template <int NW = NT / 64>
__device__ __forceinline__ int block_scan(int v, int& total, int* lds4) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) lds4[wid] = x;
    __syncthreads();
    int base = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < NW; i++) {
        const int t = lds4[i];
        base += (i < wid) ? t : 0;
        tot += t;
    }
    __syncthreads();
    total = tot;
    return base + x - v;
}

// ------------------------------------------------------------------------------------------------
// Texture repacking, carried by other launches: textures [Bt, 3, H, W] (any strides) -> RGBA rows
// [Bt, HWp, 4] (alpha slot 0) before the sampling (k_face_setup's idle threads), and the [Bt, HWp, 4]
// gradient accumulator -> [Bt, 3, H, W] after the backward (k_vertex_grad's blocks).  Each block of
// the carrying grid takes one contiguous slice, so neither needs a launch of its own.
struct TexPack {
    const float* __restrict__ tex;
    long long sb;
    int sc, sp, HW, HWp;
    float4* __restrict__ out;  // null: nothing to pack
    long long n;               // Bt * HWp
};
struct TexOut {
    const float* __restrict__ g4;
    float* __restrict__ out;   // null: nothing to write
    int HW, HWp;
    long long n;               // Bt * HW
};
__device__ __forceinline__ void tex_pack_one(const TexPack& pk, long long i) {
    const long long bt = i / pk.HWp;
    const int p = (int)(i - bt * pk.HWp);
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (p < pk.HW) {
        const float* tb = pk.tex + bt * pk.sb + (long long)p * pk.sp;
        v = make_float4(tb[0], tb[pk.sc], tb[2 * (long long)pk.sc], 0.f);
    }
    pk.out[i] = v;
}
__device__ __forceinline__ void tex_out_one(const TexOut& to, long long i) {
    const long long bt = i / to.HW;
    const int p = (int)(i % to.HW);
    const float4 v = reinterpret_cast<const float4*>(to.g4)[bt * to.HWp + p];
    to.out[(bt * 3 + 0) * to.HW + p] = v.x;
    to.out[(bt * 3 + 1) * to.HW + p] = v.y;
    to.out[(bt * 3 + 2) * to.HW + p] = v.z;
}
// this block's slice [lo, hi) of n items spread over the whole grid
__device__ __forceinline__ void grid_slice(long long n, long long& lo, long long& hi) {
    const long long nb = (long long)gridDim.x * gridDim.y;
    const long long id = (long long)blockIdx.y * gridDim.x + blockIdx.x;
    const long long chunk = (n + nb - 1) / nb;
    lo = min(id * chunk, n);
    hi = min(lo + chunk, n);
}

// ------------------------------------------------------------------------------------------------
// k_face_setup: per (face group of 128, item)
//   GATHER: faces come from vertices[b, faces_idx[f, k]] (rasterize.py:232) and are written to
//           face_records; otherwise face_records already holds the gathered faces (the
//           face_index_map_forward_safe entry point receives them that way, rasterize.py:34).
template <bool GATHER>
__global__ __launch_bounds__(256) void k_face_setup(const float* __restrict__ vertices, const int32_t* __restrict__ faces_idx,
                                                    float* __restrict__ face_records, int V, int F, int S,
                                                    int draw_backside, int2* __restrict__ bbox,
                                                    uint32_t* __restrict__ mask, int nbx, int nbins, int nwords,
                                                    const float* __restrict__ vt, long long vt_bstride, int Vt,
                                                    const int32_t* __restrict__ faces_t, float* __restrict__ face_uv,
                                                    int uv_items, float* __restrict__ fnorm, TexPack pk) {
    __shared__ int2 s_bb[SETUP_FACES];
    // the block's face records, assembled per face and then written out coalesced (a record per lane
    // would store 64-B strided rows); the bin-mask words reuse the space afterwards
    constexpr int STAGE = SETUP_FACES * FACE_REC;
    __shared__ __attribute__((aligned(16))) float s_stage[STAGE > SETUP_LDS_WORDS ? STAGE : SETUP_LDS_WORDS];
    float* s_frec = s_stage;
    uint32_t* s_mask = reinterpret_cast<uint32_t*>(s_stage);
    const int b = blockIdx.y;
    const int f0 = blockIdx.x * SETUP_FACES;
    const int t = threadIdx.x;
    if (pk.out && t >= SETUP_FACES) {  // the threads the face phase leaves idle repack the textures
        long long lo, hi;
        grid_slice(pk.n, lo, hi);
        for (long long i = lo + (t - SETUP_FACES); i < hi; i += blockDim.x - SETUP_FACES) tex_pack_one(pk, i);
    }
    if (t < SETUP_FACES) {
        const int f = f0 + t;
        int2 bb = make_int2(NR_EMPTY_RANGE, NR_EMPTY_RANGE);
        if (f < F) {
            float c[9];
            if (GATHER) {
                const float* vb = vertices + (long long)b * V * 3;
#pragma unroll
                for (int k = 0; k < 3; k++) {
                    const int vi = faces_idx[f * 3 + k];
                    c[3 * k + 0] = vb[vi * 3 + 0];
                    c[3 * k + 1] = vb[vi * 3 + 1];
                    c[3 * k + 2] = vb[vi * 3 + 2];
                }
                // 16-float record: corners, rcp_nr(z_k), rcp_nr(z_k + 1e-10), range flags (see Face)
                bool fxyz = true, fzq = true;
#pragma unroll
                for (int k = 0; k < 3; k++) {
                    fxyz = fxyz && coord_ok(c[3 * k]) && coord_ok(c[3 * k + 1]) && in_range(c[3 * k + 2], 0x1p-20f, 0x1p20f);
                    fzq = fzq && in_range(c[3 * k + 2] + 1e-10f, 0x1p-20f, 0x1p20f);
                }
#ifdef NR_NO_FASTDIV
                const int flags = 0;  // timing build: IEEE divisions everywhere
#else
                const int flags = (fxyz ? FACE_FAST_XYZ : 0) | (fzq ? FACE_FAST_ZQ : 0);
#endif
                float4* rec = reinterpret_cast<float4*>(s_frec + t * FACE_REC);
                rec[0] = make_float4(c[0], c[1], c[2], c[3]);
                rec[1] = make_float4(c[4], c[5], c[6], c[7]);
                rec[2] = make_float4(c[8], rcp_nr(c[2]), rcp_nr(c[5]), rcp_nr(c[8]));
                rec[3] = make_float4(rcp_nr(c[2] + 1e-10f), rcp_nr(c[5] + 1e-10f), rcp_nr(c[8] + 1e-10f),
                                     __int_as_float(flags));
                if (fnorm) {
                    // face normal cross(v1 - v0, v2 - v1) (rasterize.py:166-170; torch.cross component order)
                    const float a0 = c[3] - c[0], a1 = c[4] - c[1], a2 = c[5] - c[2];
                    const float b0 = c[6] - c[3], b1 = c[7] - c[4], b2 = c[8] - c[5];
                    float* nf = fnorm + ((long long)b * F + f) * 3;
                    nf[0] = a1 * b2 - a2 * b1;
                    nf[1] = a2 * b0 - a0 * b2;
                    nf[2] = a0 * b1 - a1 * b0;
                }
            } else {
                const float* rec = face_records + ((long long)b * F + f) * 9;  // caller's [B, F, 3, 3]
#pragma unroll
                for (int k = 0; k < 9; k++) c[k] = rec[k];
            }
            const float x0 = c[0], y0 = c[1], x1 = c[3], y1 = c[4], x2 = c[6], y2 = c[7];
            bool ok = true;
#pragma unroll
            for (int k = 0; k < 9; k++) ok = ok && !(c[k] != c[k]);  // NaN faces are never accepted
            // face-level rejects of .cu:100-104 and .cu:118-121 (pixel independent)
            if (!draw_backside && (y2 - y0) * (x1 - x0) > (y1 - y0) * (x2 - x0)) ok = false;
            const float det = x2 * (y0 - y1) + x0 * (y1 - y2) + x1 * (y2 - y0);
            if ((double)fabsf(det) < 0.00000001) ok = false;
            if (ok) {
                int ix0, ix1, iy0, iy1;
                pix_range(fminf(fminf(x0, x1), x2), fmaxf(fmaxf(x0, x1), x2), S, ix0, ix1);
                pix_range(fminf(fminf(y0, y1), y2), fmaxf(fmaxf(y0, y1), y2), S, iy0, iy1);
                if (ix0 <= ix1 && iy0 <= iy1) bb = make_int2(pack_range(ix0, ix1), pack_range(iy0, iy1));
            }
            if (face_uv != nullptr && b < uv_items) {
                const float* vtb = vt + (long long)b * vt_bstride;
                float uv[6];
                bool uok = true;
#pragma unroll
                for (int k = 0; k < 3; k++) {
                    const int ti = faces_t[f * 3 + k];
                    uv[2 * k + 0] = vtb[(long long)ti * 2 + 0];
                    uv[2 * k + 1] = vtb[(long long)ti * 2 + 1];
                }
#pragma unroll
                for (int k = 0; k < 6; k++) uok = uok && (uv[k] == 0.f || in_range(uv[k], 0x1p-16f, 0x1p20f));
                // 8-float texture record: u0 v0 u1 v1 u2 v2, range flag (see sample_texture), pad
                float4* u = reinterpret_cast<float4*>(face_uv + ((long long)b * F + f) * 8);
                u[0] = make_float4(uv[0], uv[1], uv[2], uv[3]);
                u[1] = make_float4(uv[4], uv[5], __int_as_float(uok ? 1 : 0), 0.f);
            }
            bbox[(long long)b * F + f] = bb;
        }
        s_bb[t] = bb;
    }
    __syncthreads();
    {
        const int nf = min(SETUP_FACES, F - f0);
        if (GATHER) {
            float4* dst = reinterpret_cast<float4*>(face_records + ((long long)b * F + f0) * FACE_REC);
            const float4* src = reinterpret_cast<const float4*>(s_frec);
            for (int i = t; i < nf * (FACE_REC / 4); i += blockDim.x) dst[i] = src[i];
        }
        __syncthreads();
    }
    // coarse-bin bitmask words of this face group
    const int w0 = blockIdx.x * (SETUP_FACES / 32);
    const int nw = min(SETUP_FACES / 32, nwords - w0);
    if (nbins * (SETUP_FACES / 32) <= SETUP_LDS_WORDS) {
        // each face sets its bit in the (few) bins its pixel range touches (LDS ds_or), then the
        // block writes its words out
        for (int i = t; i < nbins * (SETUP_FACES / 32); i += blockDim.x) s_mask[i] = 0u;
        __syncthreads();
        if (t < SETUP_FACES) {
            const int2 bb = s_bb[t];
            const int x0 = range_lo(bb.x), x1 = range_hi(bb.x), y0 = range_lo(bb.y), y1 = range_hi(bb.y);
            if (x0 <= x1 && y0 <= y1) {
                const int nby = nbins / nbx;
                for (int by = y0 / COARSE; by <= min(y1 / COARSE, nby - 1); by++)
                    for (int bx = x0 / COARSE; bx <= min(x1 / COARSE, nbx - 1); bx++)
                        atomicOr(&s_mask[(by * nbx + bx) * (SETUP_FACES / 32) + (t >> 5)], 1u << (t & 31));
            }
        }
        __syncthreads();
        for (int p = t; p < nbins * nw; p += blockDim.x) {
            const int bin = p / nw, wi = p % nw;
            mask[((long long)b * nbins + bin) * nwords + w0 + wi] = s_mask[bin * (SETUP_FACES / 32) + wi];
        }
        return;
    }
    for (int p = t; p < nbins * nw; p += blockDim.x) {
        const int bin = p / nw, wi = p % nw;
        const int bx0 = (bin % nbx) * COARSE, by0 = (bin / nbx) * COARSE;
        const int bx1 = bx0 + COARSE - 1, by1 = by0 + COARSE - 1;
        uint32_t bits = 0;
#pragma unroll 8
        for (int j = 0; j < 32; j++) {
            const int2 bb = s_bb[wi * 32 + j];
            const bool hit = range_lo(bb.x) <= bx1 && range_hi(bb.x) >= bx0 && range_lo(bb.y) <= by1 &&
                             range_hi(bb.y) >= by0;
            bits |= (hit ? 1u : 0u) << j;
        }
        mask[((long long)b * nbins + bin) * nwords + w0 + wi] = bits;
    }
}

// ------------------------------------------------------------------------------------------------
// vertex normals (rasterize.py:171-182): u = sum of the normals of the vertex's distinct faces (the
// reference's one-hot [F, V] matmul), n = u / max(|u|, 1e-12) (F.normalize); stored as (n, |u|)
__global__ void k_vertex_normals(const float* __restrict__ fnorm, const int32_t* __restrict__ off,
                                 const int32_t* __restrict__ vfaces, float* __restrict__ vnorm, int F, int V, long long n) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int b = (int)(i / V), v = (int)(i % V);
    const float* fb = fnorm + (long long)b * F * 3;
    float u0 = 0.f, u1 = 0.f, u2 = 0.f;
    for (int e = off[v]; e < off[v + 1]; e++) {
        const float* nf = fb + vfaces[e] * 3;
        u0 += nf[0];
        u1 += nf[1];
        u2 += nf[2];
    }
    const float len = sqrtf((u0 * u0 + u1 * u1) + u2 * u2);
    const float d = fmaxf(len, 1e-12f);
    reinterpret_cast<float4*>(vnorm)[i] = make_float4(u0 / d, u1 / d, u2 / d, len);
}

// ------------------------------------------------------------------------------------------------
// k_raster_fwd<NTF>: one block per 32x32-pixel coarse bin (the bitmask granularity), split into 16
// 8x8 pixel blocks; NTF / 64 waves, each walking 16 / (NTF / 64) of the 8x8 blocks in turn.
//   1. the bin's bitmask words are expanded (block scan over popcounts) into the ordered list of
//      candidate faces;
//   2. up to FCAP candidates at a time are staged into LDS in ascending face order (one face per
//      thread, one global load stage);
//   3. per 8x8 block, the wave ballots which staged faces' float bounding boxes meet the block's
//      pixel-centre extent (an exact cull: such a face fails .cu:94-97 at every pixel of the block)
//      and walks the set bits in order (scalar loop), running the reference's per-face test for its
//      pixel -- every pixel therefore sees its candidate faces in ascending index order, as the
//      reference's sequential loop does (.cu:82-149), and the per-pixel state stays in registers
//      across rounds;
//   shading and the output image are computed by k_shade.
//   Block sizes (picked per launch, run_face_index): 256 threads = 4 waves, each walking the four 8x8
//   blocks of a 16x16 quadrant (most per-thread work, least fixed cost per pixel: best when the grid
//   has many bins of moderate depth, e.g. the headline); 1024 threads = 16 waves, one 8x8 block each
//   (the bin's walks run 4x wider: small batches, where the grid is a few blocks per CU, and dense
//   bins -- 300+ faces over one 8x8 block on a 50k-face torus -- no longer serialise on 4 waves).
//   LDS face record, structure of arrays (float4 i of staged face j at s_face[i * FCAP + j]: the
//   staging stores are lane-contiguous), 8 x float4:
//     0: xmin xmax ymin ymax | 1: bx by zmin id | 2: x0 y0 x1 y1 | 3: x2 y2 z0 z1
//     4: z2 A=x1-x0 B=y1-y0 C=x2-x1 | 5: D=y2-y1 E=x0-x2 F=y0-y2 k0 | 6: k1 k2 1/z0 1/z1 | 7: 1/z2 - - ok
//   (y1-y2 = -D etc. exactly, so w0 = (yp*C - xp*D) + k0 reproduces .cu:130 bit for bit)
constexpr int FREC = 8;  // float4 per staged face
template <int NTF> struct FwdCfg {
    static constexpr int NW = NTF / 64;                        // waves
    static constexpr int NSUB = (COARSE * COARSE) / NTF;       // 8x8 blocks (pixels) per thread
    static constexpr int CAND = NTF >= 1024 ? 1024 : 512;      // candidate ids expanded per round
    static constexpr int FCAP = NTF >= 1024 ? 256 : 128;       // faces staged per round
    static constexpr int LDS = FCAP * FREC * 16 + CAND * 4;
    static_assert(NSUB == 1 || NSUB == 2 || NSUB == 4, "forward block layout");
    // 8x8 block k of wave w: its origin (ox, oy) in the bin
    __device__ static __forceinline__ void block_of(int w, int k, int& ox, int& oy) {
        if (NSUB == 1) {         // 16 waves: wave w owns block (w & 3, w >> 2)
            ox = (w & 3) * 8;
            oy = (w >> 2) * 8;
        } else if (NSUB == 2) {  // 8 waves: a vertical pair of blocks in quadrant w >> 1
            ox = ((w >> 1) & 1) * 16 + (w & 1) * 8;
            oy = (w >> 2) * 16 + k * 8;
        } else {                 // 4 waves: the 16x16 quadrant w, walked as four 8x8 blocks
            ox = (w & 1) * 16 + (k & 1) * 8;
            oy = (w >> 1) * 16 + (k >> 1) * 8;
        }
    }
};

// the reference's per-face test sequence (.cu:94-148) for one staged face at one pixel; q0, q1 are
// the record's first two float4 (loaded ahead by the caller); FST = the SoA stride (FCAP)
template <int FST>
__device__ __forceinline__ void face_test(const float4* e, float4 q0, float4 q1, float xp, float yp, float near, float far,
                                          float delta, float& depth_min, int& best) {
#if defined(NR_ABLATE_FWD) && NR_ABLATE_FWD == 1
    best += (int)q0.x;  // timing build: no per-pixel test
    return;
#endif
    // The rejections of .cu:94-126 are independent of each other (none changes the state), so their
    // order is free: the depth-bound reject .cu:124-126 goes first, as it is the cheapest and lets a
    // whole wave skip a face hidden behind what its pixels already hold.
    if (depth_min < q1.z) return;
    // .cu:94-97 (min/max form, exact for non-NaN faces)
    if (xp < q0.x || xp > q0.y || yp < q0.z || yp > q0.w) return;
    const float4 q2 = e[2 * FST], q3 = e[3 * FST], q4 = e[4 * FST], q5 = e[5 * FST];
    const float x0 = q2.x, y0 = q2.y, x1 = q2.z, y1 = q2.w, x2 = q3.x, y2 = q3.y;
    // .cu:107-116
    const float c1 = (yp - y0) * q4.y - q4.z * (xp - x0);
    const float c2 = (yp - y1) * q4.w - q5.x * (xp - x1);
    if (c1 * c2 < 0) return;
    const float c3 = (yp - y2) * q5.y - q5.z * (xp - x2);
    if (c2 * c3 < 0) return;
#if defined(NR_ABLATE_FWD) && NR_ABLATE_FWD == 2
    best = __float_as_int(q1.w);  // timing build: no division block
    return;
#endif
    const float4 q6 = e[6 * FST];
    const float z0 = q3.z, z1 = q3.w, z2 = q4.x;
    // .cu:130-139
    float w0 = (yp * q4.w - xp * q5.x) + q5.w;
    float w1 = (yp * q5.y - xp * q5.z) + q6.x;
    float w2 = (yp * q4.y - xp * q4.z) + q6.y;
    const float ws = w0 + w1 + w2;
    float zp;
    const float4 q7 = e[7 * FST];
    if (__float_as_int(q7.w) && in_range(ws, 0x1p-20f, 0x1p20f)) {
        // face coordinates and depths within [2^-20, 2^20] (or 0) bound every operand below inside
        // div_nr's exact range (DESIGN.md "Numerics"); 1/z is staged per face
        const float rs = rcp_nr(ws);
        w0 = div_nr(w0, ws, rs);
        w1 = div_nr(w1, ws, rs);
        w2 = div_nr(w2, ws, rs);
        const float sum = div_nr(w0, z0, q6.z) + div_nr(w1, z1, q6.w) + div_nr(w2, z2, q7.x);
        if (in_range(sum, 0x1p-90f, 0x1p90f)) {
            const float r = rcp_nr(sum);
            zp = __builtin_fmaf(__builtin_fmaf(-sum, r, 1.f), r, r);  // div_nr(1, sum, r): 1 * r == r
            zp = __builtin_fmaf(__builtin_fmaf(-sum, zp, 1.f), r, zp);
        } else {
            zp = 1.f / sum;
        }
    } else {
        w0 /= ws;
        w1 /= ws;
        w2 /= ws;
        zp = 1.f / (w0 / z0 + w1 / z1 + w2 / z2);
    }
    if (zp <= near || far <= zp) return;
    if (zp <= depth_min - delta) {  // .cu:145-148
        depth_min = zp;
        best = __float_as_int(q1.w);
    }
}

template <int FST>
__device__ __forceinline__ void stage_face(float4* e, const float* __restrict__ c, int f, int2 bb) {
    const float x0 = c[0], y0 = c[1], z0 = c[2], x1 = c[3], y1 = c[4], z1 = c[5];
    const float x2 = c[6], y2 = c[7], z2 = c[8];
    e[0 * FST] = make_float4(fminf(fminf(x0, x1), x2), fmaxf(fmaxf(x0, x1), x2), fminf(fminf(y0, y1), y2),
                       fmaxf(fmaxf(y0, y1), y2));
    e[1 * FST] = make_float4(__int_as_float(bb.x), __int_as_float(bb.y), fminf(fminf(z0, z1), z2), __int_as_float(f));
    e[2 * FST] = make_float4(x0, y0, x1, y1);
    e[3 * FST] = make_float4(x2, y2, z0, z1);
    e[4 * FST] = make_float4(z2, x1 - x0, y1 - y0, x2 - x1);
    e[5 * FST] = make_float4(y2 - y1, x0 - x2, y0 - y2, x1 * y2 - x2 * y1);
    e[6 * FST] = make_float4(x2 * y0 - x0 * y2, x0 * y1 - x1 * y0, rcp_nr(z0), rcp_nr(z1));
    const bool ok = coord_ok(x0) && coord_ok(y0) && coord_ok(x1) && coord_ok(y1) && coord_ok(x2) && coord_ok(y2) &&
                    in_range(z0, 0x1p-20f, 0x1p20f) && in_range(z1, 0x1p-20f, 0x1p20f) &&
                    in_range(z2, 0x1p-20f, 0x1p20f);
    e[7 * FST] = make_float4(rcp_nr(z2), 0.f, 0.f, __int_as_float(ok ? 1 : 0));
}

#ifndef NR_FWD_WPE
#define NR_FWD_WPE 8
#endif
#ifndef NR_FWD_FORCE_NT
#define NR_FWD_FORCE_NT 0  // timing builds: 256 / 512 / 1024 threads for every launch
#endif
template <int NTF>
__global__ __launch_bounds__(NTF) __attribute__((amdgpu_waves_per_eu(NR_FWD_WPE, 8))) void k_raster_fwd(const float* __restrict__ face_records, int rs,
                                                  const int2* __restrict__ bbox, const uint32_t* __restrict__ mask,
                                                  int F, Geom g, float near, float far, float delta,
                                                  int32_t* __restrict__ fim) {
    using C = FwdCfg<NTF>;
    constexpr int NSUB = C::NSUB, FCAP = C::FCAP, CAND = C::CAND;
    __shared__ __attribute__((aligned(16))) unsigned char s_raw[C::LDS];
    __shared__ int s_scan[C::NW];
    float4* s_face = reinterpret_cast<float4*>(s_raw);
    int* s_cand = reinterpret_cast<int*>(s_raw + FCAP * FREC * 16);

    const int b = blockIdx.y;
    const int S = g.S;
    int bin_x, bin_y;
    xcd_tile<NR_FSWZ_MODE, NR_FSWZ_W, NR_FSWZ_H>(blockIdx.x, b, g.nbx, g.nby, bin_x, bin_y);
    const int bin = bin_y * g.nbx + bin_x;
    const int bx0 = bin_x * COARSE;
    const int by0 = bin_y * COARSE;
    const int t = threadIdx.x;
    const int lane = t & 63, wid = t >> 6;
    float xp[NSUB], yp[NSUB];
    float depth_min[NSUB];
    int best[NSUB];
    float xcl[NSUB], xch[NSUB], ycl[NSUB], ych[NSUB];
#pragma unroll
    for (int k = 0; k < NSUB; k++) {
        int ox, oy;
        C::block_of(wid, k, ox, oy);
        xcl[k] = pix_center(bx0 + ox, S);
        xch[k] = pix_center(bx0 + ox + 7, S);
        ycl[k] = pix_center(by0 + oy, S);
        ych[k] = pix_center(by0 + oy + 7, S);
        xp[k] = pix_center(bx0 + ox + (lane & 7), S);
        yp[k] = pix_center(by0 + oy + (lane >> 3), S);
        depth_min[k] = far;
        best[k] = -1;
    }

    const uint32_t* words = mask + ((long long)b * g.nbins + bin) * g.nwords;
    const int2* bbb = bbox + (long long)b * F;
    const float* frb = face_records + (long long)b * F * rs;
    int32_t* __restrict__ fimb = fim + (long long)b * S * S;

    for (int wbase = 0; wbase < g.nwords; wbase += NTF) {
        const int w = wbase + t;
        const uint32_t bits = (w < g.nwords) ? words[w] : 0u;
        int total;
        const int off = block_scan<C::NW>(__builtin_popcount(bits), total, s_scan);
        for (int cbase = 0; cbase < total; cbase += CAND) {
            // expand my word's set bits into the ordered candidate list
            int r = off;
            for (uint32_t m = bits; m; m &= m - 1, r++) {
                if (r < cbase) continue;
                if (r >= cbase + CAND) break;
                s_cand[r - cbase] = w * 32 + __builtin_ctz(m);
            }
            __syncthreads();
            const int nc = min(CAND, total - cbase);
            for (int j0 = 0; j0 < nc; j0 += FCAP) {
                const int n = min(FCAP, nc - j0);
                if (t < n) {
                    const int f = s_cand[j0 + t];
                    stage_face<FCAP>(s_face + t, frb + f * rs, f, bbb[f]);
                }
                __syncthreads();
#pragma unroll
                for (int k = 0; k < NSUB; k++) {
                    const float xc0 = xcl[k], xc1 = xch[k], yc0 = ycl[k], yc1 = ych[k];
                    for (int c0 = 0; c0 < n; c0 += 64) {
                        bool hit = false;
                        if (c0 + lane < n) {
                            const float4 q0 = s_face[c0 + lane];
                            hit = !(xc1 < q0.x || xc0 > q0.y || yc1 < q0.z || yc0 > q0.w);
                        }
                        // faces touching this wave's pixels, walked in ascending order
                        for (unsigned long long m = __ballot(hit); m; m &= m - 1) {
                            const float4* e = s_face + (c0 + __builtin_ctzll(m));
                            const float4 q0 = e[0], q1 = e[FCAP];
                            face_test<FCAP>(e, q0, q1, xp[k], yp[k], near, far, delta, depth_min[k], best[k]);
                        }
                    }
                }
                __syncthreads();
            }
        }
    }

#pragma unroll
    for (int k = 0; k < NSUB; k++) {
        int ox, oy;
        C::block_of(wid, k, ox, oy);
        const int px = bx0 + ox + (lane & 7), py = by0 + oy + (lane >> 3);
        if (px < S && py < S) fimb[py * S + px] = best[k];
    }
}

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
__device__ __forceinline__ int halo_row_offset(int C, int S, int x, int y, int c) {
    return (((y / HALO_TH) * 2 + ((y & (HALO_TH - 1)) != 0)) * C + c) * S + x;
}
__device__ __forceinline__ int halo_col_offset(int C, int S, int x, int y, int c) {
    const int nty = (S + HALO_TH - 1) / HALO_TH, ntx = (S + HALO_TW - 1) / HALO_TW;
    return nty * 2 * C * S + (((y / HALO_TH) * C + c) * HALO_TH + (y & (HALO_TH - 1))) * (2 * ntx) +
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
// k_shade: the image channels from the face-index map, one thread per OUTPUT pixel (rasterize.py:
// 237-328): weights (compute_weight_map), texture sample, silhouette and depth for the 1 or 2x2
// internal pixels it covers, merged in rgb/sil/depth order, flipped, and 2x2-averaged with the
// reference's summation order.  Kept out of the rasteriser so that kernel stays lean (registers,
// occupancy); costs one extra read of the face-index map.
template <int FEAT>  // 1 = lights, 2 = backgrounds, as k_raster_bwd
#ifndef NR_SHADE_WPE
#define NR_SHADE_WPE 6  // 6 waves/SIMD: up to 80 VGPRs, no spills with the packed-texel path (7: a 2-dword spill, same time)
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu((FEAT & 1) ? 1 : NR_SHADE_WPE, 8))) void k_shade(const float* __restrict__ face_records, const int32_t* __restrict__ fim,
                                               int F, int S, Shade sh_in, int aa, float* __restrict__ images,
                                               float* __restrict__ halo) {
    Shade sh = sh_in;
    if (!(FEAT & 1)) sh.nl = 0;
    if (!(FEAT & 2)) sh.bg = nullptr;
    const int s = aa ? S / 2 : S;
    const int b = blockIdx.y;
    int blk = blockIdx.x, unused;
    xcd_tile<NR_SSWZ_MODE, 1, 1>(blockIdx.x, b, 1, gridDim.x, unused, blk);
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
        Face f = empty_face();
        if (fi >= 0) f = load_face_rec(frb + fi * FACE_REC);
        float v[MAXC];
        shade_pixel(sh, b, fi, f, x, y, S, v);
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
    const int ys[4] = {iy + 1, iy, iy + 1, iy}, xs[4] = {ix + 1, ix + 1, ix, ix};
    float v[4][MAXC];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        Face f = empty_face();
        if (fis[q] >= 0) f = load_face_rec(frb + fis[q] * FACE_REC);
        shade_pixel(sh, b, fis[q], f, xs[q], ys[q], S, v[q]);
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
// per-pixel form repeats the per-thread overheads 4x).  NR_SHADE_PX: 0 never, 1 always, 2 by grid size.
#ifndef NR_SHADE_PX
#define NR_SHADE_PX 2
#endif
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
    Face f = empty_face();
    if (fi >= 0) f = load_face_rec(frb + fi * FACE_REC);
    float v[MAXC];
    shade_pixel(sh, b, fi, f, x, y, S, v);
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

// ------------------------------------------------------------------------------------------------
// k_raster_bwd: one block per 32x16 pixels + 1-pixel halo; each wave owns a 16x8 block, 2 pixels per
// lane.
//   1. recompute the internal image I (all channels, bit-identical to the forward) and the upstream
//      gradient G of the block + halo into LDS (Differentiation saved the images; the flip/AA
//      backward is an index map and /4), and for the block's own pixels the gradient terms that do
//      not depend on the stencil (depth and texture-coordinate paths to z, bilinear weights);
//   2. the soft-gradient stencil (gx, gy) of Differentiation.backward, then the coordinate-map chain
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
// staged record: ay by ax bx | pos G_rgb[3] | gF[9] | pad (20 floats); with lights also dL/dnormal[3]
// and the weights w[3] at 17..22 (24 floats)
template <bool LIT> constexpr int srec() { return LIT ? 24 : 20; }
constexpr int BWD_LDS_IG = 2 * MAXC * HN * 4;
constexpr int BWD_LDS_HALO = 2 * MAXC * 128 * 4;  // halo staging (step 0), after the I / G planes
template <bool LIT> constexpr int bwd_lds() {
#ifdef NR_BWD_LDS_SMALL
    return BWD_LDS_IG + BWD_LDS_HALO;  // timing builds with NR_ABLATE & 2 only (no record staging)
#endif
    return BWD_LDS_IG + BWD_LDS_HALO > 4 * 128 * srec<LIT>() * 4 ? BWD_LDS_IG + BWD_LDS_HALO : 4 * 128 * srec<LIT>() * 4;
}
static_assert(BWD_LDS_IG % 16 == 0, "halo staging alignment");
// experiment switch for timing builds (never set in the shipped library):
//   2 = no gradient accumulation (steps 3 and 4), 4 = no global atomics (step 4),
//   8 = no per-face gather (step 3's member loop), 16 = no halo shading, 64 = no stencil,
//   1024 = no direct texel atomics (texels outside a face's window)
#ifndef NR_ABLATE
#define NR_ABLATE 0
#endif
#ifndef NR_HALO_EARLY
#define NR_HALO_EARLY 1
#endif

struct BwdArgs {
    const float* __restrict__ face_records;
    const int32_t* __restrict__ fim;
    const float* __restrict__ grad_images;
    float* __restrict__ grad_faces;   // [B, F, 9]
    float* __restrict__ grad_tex4;    // [Bt, HWp, 4] or null
    const float* __restrict__ halo;   // halo cache written by the forward, or null (re-shade the halo)
    float* __restrict__ grad_normals; // [B, F, 9] per-face corner vertex-normal gradients (lights)
    float* __restrict__ grad_bg;      // [B, 3, S, S] or null
    int F, aa, s, HWp;
    float step, inv_step;
    int step_pow2;                     // x / step == x * inv_step exactly
};

// upstream gradient of internal pixel (x, y): the flip / 2x2-mean backward is an index map and /4.
// gi: this item's [C, s, s] upstream gradient (32-bit offsets inside it)
__device__ __forceinline__ void upstream_grad(const BwdArgs& a, const float* __restrict__ gi, int C, int y, int x, int S,
                                              float* G) {
    if (a.aa) {
        const int s = a.s;
        const int o = ((S - 1 - y) >> 1) * s + ((S - 1 - x) >> 1);
#pragma unroll
        for (int c = 0; c < MAXC; c++) G[c] = c < C ? gi[c * s * s + o] / 4.f : 0.f;
    } else {
        const int o = (S - 1 - y) * S + (S - 1 - x);
#pragma unroll
        for (int c = 0; c < MAXC; c++) G[c] = c < C ? gi[c * S * S + o] : 0.f;
    }
}

__device__ __forceinline__ float upstream_one(const BwdArgs& a, const float* __restrict__ gi, int y, int x, int S, int c) {
    if (a.aa) {
        const int s = a.s;
        return gi[c * s * s + ((S - 1 - y) >> 1) * s + ((S - 1 - x) >> 1)] / 4.f;
    }
    return gi[c * S * S + (S - 1 - y) * S + (S - 1 - x)];
}

__device__ __forceinline__ float div_step(const BwdArgs& a, float x) { return a.step_pow2 ? x * a.inv_step : x / a.step; }

__device__ __forceinline__ float stencil(const BwdArgs& a, const float* Im, const float* I0, const float* Ip,
                                         const float* Gm, const float* G0, const float* Gp, int i, int n, int C) {
    const bool has_p = i <= n - 2, has_m = i >= 1;
    const float r_i = has_p ? div_step(a, -pair_dot(I0, Ip, Gp, C)) : 0.f;
    const float r_m = has_m ? div_step(a, -pair_dot(Im, I0, G0, C)) : 0.f;
    const float l_i = has_p ? div_step(a, -pair_dot(Ip, I0, G0, C)) : 0.f;
    const float l_m = has_m ? div_step(a, -pair_dot(I0, Im, Gm, C)) : 0.f;
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

// per interior pixel state carried across the stencil's barrier
struct BwdPix {
    int fi;            // face index (-1: background or outside)
    float w[3];        // barycentric weights (compute_weight_map)
    float gz[3];       // d/dz of the face corners through the depth and texture-coordinate paths
    float grgb[3];     // upstream gradient of the rgb channels
    float ay, by, ax, bx;
    int pos;           // bilinear top-left texel relative to the face window: dx | dy << 8; -1 none
    int wx, wy;        // face window origin (texels); INT_MIN when not windowed
    float gn[3];       // lights: dL/d(smooth normal)
};

// FEAT: 1 = lights, 2 = backgrounds (separate instantiations keep the plain path lean)
// NPX: pixels per lane (2: 256 threads, a wave = 16x8 pixels; 1: 512 threads, a wave = 16x4 pixels)
#ifndef NR_BWD_WPE1
#define NR_BWD_WPE1 6
#endif
template <int FEAT, int NPX>
__global__ __launch_bounds__(2 * NT / NPX) __attribute__((amdgpu_waves_per_eu((FEAT & 1) ? 3 : (NPX == 1 ? NR_BWD_WPE1 : 4), 8))) void k_raster_bwd(BwdArgs a, Geom g, Shade sh_in) {
    constexpr bool LIT = (FEAT & 1) != 0, BG = (FEAT & 2) != 0;
    // features this instantiation does not have become compile-time constants (the shared
    // shade_pixel then carries no light / background code or arguments)
    Shade sh = sh_in;
    if (!LIT) sh.nl = 0;
    if (!BG) sh.bg = nullptr;
    constexpr int REC = srec<LIT>();
    __shared__ __attribute__((aligned(16))) float s_raw[bwd_lds<LIT>() / 4];
    float(*s_I)[HN] = reinterpret_cast<float(*)[HN]>(s_raw);
    float(*s_G)[HN] = reinterpret_cast<float(*)[HN]>(s_raw + MAXC * HN);
    const int b = blockIdx.y;
    const int S = g.S;
    const int C = sh.C;
    const bool rgb = (sh.draw & NR_DRAW_RGB) != 0;
    const bool want_tex = rgb && a.grad_tex4 != nullptr;
    int tile_x, tile_y;
    xcd_tile<NR_SWZ_MODE, NR_SWZ_W, NR_SWZ_H>(blockIdx.x, b, (S + TW - 1) / TW, (S + BH - 1) / BH, tile_x, tile_y);
    const int tx0 = tile_x * TW;
    const int ty0 = tile_y * BH;
    const int t = threadIdx.x;
    const int lane = t & 63, wid = t >> 6;
    const int bt = sh.tv.sb ? b : 0;
    // per-item bases (uniform, 64-bit); per-pixel offsets below are 32-bit
    const int32_t* __restrict__ fimb = a.fim + (long long)b * S * S;
    const float* __restrict__ gimb = a.grad_images + (long long)b * C * (a.aa ? a.s * a.s : S * S);
    const float* __restrict__ frb = a.face_records + (long long)b * a.F * FACE_REC;
    const float* __restrict__ fuvb = sh.face_uv + (sh.uv_bstride ? (long long)b * sh.uv_bstride : 0);
    float* __restrict__ gFb = a.grad_faces + (long long)b * a.F * 9;
    float* __restrict__ g4b = a.grad_tex4 ? a.grad_tex4 + (long long)bt * a.HWp * 4 : nullptr;
    // wave wid owns the 16x8 block at (16 (wid & 1), 8 (wid >> 1)); lane -> column lane & 15, rows lane >> 4 (+4)
    const int lx = (wid & 1) * 16 + (lane & 15);
    const int ly0 = (wid >> 1) * (4 * NPX) + (lane >> 4);
    const int px = tx0 + lx;
    const float xp = pix_center(px, S);

    // halo ring from the forward's halo cache: asynchronous global -> LDS loads by waves 0 and 1
    // (lane t < NHALO carries halo pixel t, ring order of halo_pixel), landed before the barrier
    float(*s_hI)[128] = reinterpret_cast<float(*)[128]>(s_raw + BWD_LDS_IG / 4);
    float(*s_hG)[128] = reinterpret_cast<float(*)[128]>(s_raw + BWD_LDS_IG / 4 + MAXC * 128);
    auto halo_prefetch = [&]() {
        if (a.halo && t < 128) {
            int hy, hx;
            halo_pixel(t, hy, hx);
            const int hpy = ty0 - 1 + hy, hpx = tx0 - 1 + hx;
            const bool h_in = t < NHALO && hpy >= 0 && hpy < S && hpx >= 0 && hpx < S;
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
#if NR_HALO_EARLY
    halo_prefetch();  // in flight during step 1
#endif

    // ---- 1. image + upstream gradient (LDS), and the stencil-independent gradient terms ---------
    BwdPix P[NPX];
    float I2[NPX][MAXC], G2[NPX][MAXC];
#pragma unroll
    for (int k = 0; k < NPX; k++) {
        const int py = ty0 + ly0 + 4 * k;
        const bool inside = px < S && py < S;
        BwdPix& q = P[k];
        q.fi = inside ? fimb[py * S + px] : -1;
        q.pos = -1;
        q.wx = q.wy = INT_MIN;
        q.w[0] = q.w[1] = q.w[2] = 0.f;
        q.gz[0] = q.gz[1] = q.gz[2] = 0.f;
        q.grgb[0] = q.grgb[1] = q.grgb[2] = 0.f;
        q.ay = q.by = q.ax = q.bx = 0.f;
        q.gn[0] = q.gn[1] = q.gn[2] = 0.f;
#pragma unroll
        for (int c = 0; c < MAXC; c++) I2[k][c] = G2[k][c] = 0.f;
        if (inside) upstream_grad(a, gimb, C, py, px, S, G2[k]);
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
        Face f = load_face_rec(frb + q.fi * FACE_REC);
#ifndef NR_BWD_FASTDIV
        f.flags = 0;  // IEEE divisions here: the shortcut's extra live values cost more than it saves
#endif
        bool wfast = false;
        if (NR_ABLATE & 512) {
            q.w[0] = f.x0, q.w[1] = f.y0, q.w[2] = f.z0;  // timing build: no weights
        } else {
            wfast = face_weights(xp, yp, f, q.w);
        }
        const float* w = q.w;
        float r = 0.f, gg = 0.f, bb = 0.f, dep = 0.f;
        if (rgb && !(NR_ABLATE & 128)) {
            TexSample s;
            const float* fuv = fuvb + q.fi * 8;
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
            sample_texture(f, w, wfast, fuv, sh.tv, bt, sh.eps, s, Gt, gw);
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
                // corners with nonzero weight inside the window and the texture (no row wrap)
                bool fits = wok;
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const float wt = ((i & 2) ? q.by : q.ay) * ((i & 1) ? q.bx : q.ax);
                    if (wt == 0.f) continue;
                    const int cx = dx + (i & 1), cy = dy + (i >> 1);
                    const int gx_ = ix0 + (i & 1), gy_ = iy0 + (i >> 1);
                    fits = fits && cx >= 0 && cx < TWIN && cy >= 0 && cy < TWIN && gx_ >= 0 && gy_ >= 0 &&
                           gx_ < sh.tv.W && gy_ < sh.tv.H;
                }
                if (fits) {
                    q.pos = dx | (dy << 8);
                } else {
                    // outside the face window: direct atomics (texel index as sampled)
#pragma unroll
                    for (int i = 0; i < 4; i++) {
                        float* gtg = g4b + s.idx[i] * 4;
#pragma unroll
                        for (int ch = 0; ch < 3; ch++) {
                            const float v = Gt[ch] * s.wt[i];
                            if (v != 0.f && !(NR_ABLATE & 1024)) unsafeAtomicAdd(gtg + ch, v);
                        }
                    }
                }
            }
            // texture coordinates -> z (gradient-only terms: reciprocal multiplies)
            const float ayv = q.ay, byv = q.by, axv = q.ax, bxv = q.bx;
            float g_x = -(gw[0] * ayv);
            g_x = g_x + gw[1] * ayv;
            g_x = g_x - gw[2] * byv;
            g_x = g_x + gw[3] * byv;
            float g_y = -(gw[0] * axv);
            g_y = g_y - gw[1] * bxv;
            g_y = g_y + gw[2] * axv;
            g_y = g_y + gw[3] * bxv;
            const float gp[2] = {g_x, g_y};
            float gpr[2];
#pragma unroll
            for (int j = 0; j < 2; j++) {
                // minimum(pc, hm) then maximum(pr, lo) backward (ties split the gradient)
                const float pc = s.pc[j], hm = s.hm[j], pr = s.pr[j], lo = s.lo[j];
                float gq = gp[j];
                gq = (pc == hm) ? gq * 0.5f : (pc > hm ? 0.f : gq);
                gq = (pr == lo) ? gq * 0.5f : (pr < lo ? 0.f : gq);
                gpr[j] = gq;
            }
            const float g_dt = gpr[0] * s.num[0] + gpr[1] * s.num[1];
            const float g_st = -g_dt * (s.dt * s.dt);
#pragma unroll
            for (int j = 0; j < 3; j++) {
                const float rz = frcp(s.zq[j]);
                float gzj = 0.f;
#pragma unroll
                for (int qq = 0; qq < 2; qq++) gzj += (-(gpr[qq] * s.dt)) * (w[j] * fuv[2 * j + qq]) * rz * rz;
                gzj += (-g_st) * w[j] * rz * rz;
                q.gz[j] = gzj;
            }
        }
        if ((sh.draw & NR_DRAW_DEPTH) && !(NR_ABLATE & 256)) {
            dep = depth_value(f, w, wfast);
            // depth channel gradient reloaded (cache hit) rather than a runtime-indexed register array
            const int dc = (rgb ? 3 : 0) + ((sh.draw & NR_DRAW_SILHOUETTES) ? 1 : 0);
            const float gd = upstream_one(a, gimb, py, px, S, dc);
            const float g_s = -gd * (dep * dep);
            const float z[3] = {f.z0, f.z1, f.z2};
#pragma unroll
            for (int j = 0; j < 3; j++) {
                const float rz = frcp(z[j]);
                q.gz[j] += (-g_s) * w[j] * rz * rz;
            }
        }
        // channel values in merge order (rgb, sil, depth), compile-time slots as in shade_pixel
        const bool R = rgb, Sl = (sh.draw & NR_DRAW_SILHOUETTES) != 0;
        I2[k][0] = R ? r : (Sl ? 1.f : dep);
        I2[k][1] = R ? gg : dep;
        I2[k][2] = bb;
        I2[k][3] = Sl ? 1.f : dep;
        I2[k][4] = dep;
    }
#pragma unroll
    for (int k = 0; k < NPX; k++) {
        const int li = (ly0 + 4 * k + 1) * HW_ + (lx + 1);
#pragma unroll
        for (int c = 0; c < MAXC; c++) {
            if (c < C) {
                s_I[c][li] = I2[k][c];
                s_G[c][li] = G2[k][c];
            }
        }
    }
#if !NR_HALO_EARLY
    halo_prefetch();
#endif
    // halo ring: image and upstream gradient only
    int hy, hx;
    halo_pixel(t, hy, hx);
    const int hpy = ty0 - 1 + hy, hpx = tx0 - 1 + hx;
    const bool h_in = t < NHALO && hpy >= 0 && hpy < S && hpx >= 0 && hpx < S;
    if (a.halo) {
        __builtin_amdgcn_s_waitcnt(0);  // this wave's LDS-DMA halo loads have landed
        __syncthreads();
        if (t < NHALO) {
            const int hl = hy * HW_ + hx;
#pragma unroll
            for (int c = 0; c < MAXC; c++) {
                if (c < C) {
                    s_I[c][hl] = h_in ? s_hI[c][t] : 0.f;
                    s_G[c][hl] = h_in ? (a.aa ? s_hG[c][t] / 4.f : s_hG[c][t]) : 0.f;
                }
            }
        }
    } else if (t < NHALO) {
        float hI[MAXC], hG[MAXC];
#pragma unroll
        for (int c = 0; c < MAXC; c++) hI[c] = hG[c] = 0.f;
        if (!(NR_ABLATE & 16) && h_in) {
            const int hf = fimb[hpy * S + hpx];
            Face ff = empty_face();
            if (hf >= 0) ff = load_face_rec(frb + hf * FACE_REC);
            shade_pixel(sh, b, hf, ff, hpx, hpy, S, hI);
            upstream_grad(a, gimb, C, hpy, hpx, S, hG);
        }
        const int hl = hy * HW_ + hx;
#pragma unroll
        for (int c = 0; c < MAXC; c++) {
            if (c < C) {
                s_I[c][hl] = hI[c];
                s_G[c][hl] = hG[c];
            }
        }
    }
    __syncthreads();

    // ---- 2. Differentiation.backward stencil -> coordinate-map gradient ------------------------
    float gF[NPX][9];
#pragma unroll
    for (int k = 0; k < NPX; k++) {
        const BwdPix& q = P[k];
#pragma unroll
        for (int j = 0; j < 9; j++) gF[k][j] = 0.f;
        if (q.fi < 0) continue;
        const int py = ty0 + ly0 + 4 * k;
        const int li = (ly0 + 4 * k + 1) * HW_ + (lx + 1);
        // centre values re-read from LDS (not kept in registers across the barrier)
        float I0[MAXC], G0[MAXC], Im[MAXC], Ip[MAXC], Gm[MAXC], Gp[MAXC];
#pragma unroll
        for (int c = 0; c < MAXC; c++) {
            const bool u = c < C;
            I0[c] = u ? s_I[c][li] : 0.f; G0[c] = u ? s_G[c][li] : 0.f;
            Im[c] = u ? s_I[c][li - 1] : 0.f; Ip[c] = u ? s_I[c][li + 1] : 0.f;
            Gm[c] = u ? s_G[c][li - 1] : 0.f; Gp[c] = u ? s_G[c][li + 1] : 0.f;
        }
        const float gx = (NR_ABLATE & 64) ? Im[0] : stencil(a, Im, I0, Ip, Gm, G0, Gp, px, S, C);
#pragma unroll
        for (int c = 0; c < MAXC; c++) {
            const bool u = c < C;
            Im[c] = u ? s_I[c][li - HW_] : 0.f; Ip[c] = u ? s_I[c][li + HW_] : 0.f;
            Gm[c] = u ? s_G[c][li - HW_] : 0.f; Gp[c] = u ? s_G[c][li + HW_] : 0.f;
        }
        const float gy = (NR_ABLATE & 64) ? Ip[0] : stencil(a, Im, I0, Ip, Gm, G0, Gp, py, S, C);
        // coordinate map: coord = sum_k w_k faces_xy[k]  (rasterize.py:91-97)
#pragma unroll
        for (int j = 0; j < 3; j++) {
            gF[k][3 * j + 0] = gx * q.w[j];
            gF[k][3 * j + 1] = gy * q.w[j];
            gF[k][3 * j + 2] = q.gz[j];
        }
    }
    if (NR_ABLATE & 2) {
#pragma unroll
        for (int k = 0; k < NPX; k++)
#pragma unroll
            for (int j = 0; j < 9; j++) asm volatile("" ::"v"(gF[k][j]));
        return;
    }
    __syncthreads();  // the staged records reuse the image / gradient LDS

    // ---- 3. stage this lane's two pixel records; group the wave's records by face --------------
    float* rec = s_raw + wid * (64 * NPX * REC);
#pragma unroll
    for (int k = 0; k < NPX; k++) {
        float* r = rec + (k * 64 + lane) * REC;
        reinterpret_cast<float4*>(r)[0] = make_float4(P[k].ay, P[k].by, P[k].ax, P[k].bx);
        reinterpret_cast<float4*>(r)[1] = make_float4(__int_as_float(P[k].pos), P[k].grgb[0], P[k].grgb[1], P[k].grgb[2]);
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
    // face-gradient float t) over the face's records whose pixel lies in row c of the wave's 16x4
    // sub-blocks; the 4 chunks are then added across lanes.
    const int tt = lane & 15, chunk = lane >> 4;
    const int tdx = tt & 3, tdy = tt >> 2;
    const int fsel = 8 + (tt < 9 ? tt : 0);
    const int nsel_w = 20 + (tt < 9 ? tt / 3 : 0), nsel_n = 17 + (tt < 9 ? tt % 3 : 0);
    float* __restrict__ gNb = LIT ? a.grad_normals + (long long)b * a.F * 9 : nullptr;
    // the second pixel's state (NPX == 1: none, never active)
    const int fi1 = NPX > 1 ? P[NPX - 1].fi : -1, wx1 = NPX > 1 ? P[NPX - 1].wx : 0, wy1 = NPX > 1 ? P[NPX - 1].wy : 0;
    const bool act0 = P[0].fi >= 0, act1 = fi1 >= 0;
    unsigned long long p0 = __ballot(act0), p1 = __ballot(act1);
    // texel lanes: consecutive faces with the same texel window (e.g. every face of a flat-colour
    // material samples one 2x2 atlas patch, load_obj.py:84-94) accumulate into `pend` and flush once
    // per run, so such hot texels take one atomic per run instead of one per face
    float pend = 0.f;
    int pwx = INT_MIN, pwy = 0;
    while (p0 | p1) {
        // leader: lowest pending pixel; both candidates read without branches, selected on the scalar unit
        const bool from0 = p0 != 0ull;
        const int l0 = from0 ? __builtin_ctzll(p0) : 0, l1 = p1 ? __builtin_ctzll(p1) : 0;
        const int k0 = __builtin_amdgcn_readlane(P[0].fi, l0), k1 = __builtin_amdgcn_readlane(fi1, l1);
        const int x0w = __builtin_amdgcn_readlane(P[0].wx, l0), x1w = __builtin_amdgcn_readlane(wx1, l1);
        const int y0w = __builtin_amdgcn_readlane(P[0].wy, l0), y1w = __builtin_amdgcn_readlane(wy1, l1);
        const int key = from0 ? k0 : k1, wx = from0 ? x0w : x1w, wy = from0 ? y0w : y1w;
        // key >= 0, so fi == key implies an active pixel
        const unsigned long long m0 = __builtin_amdgcn_ballot_w64(P[0].fi == key) & p0;
        const unsigned long long m1 = __builtin_amdgcn_ballot_w64(fi1 == key) & p1;
        p0 &= ~m0;
        p1 &= ~m1;
        float a0 = 0.f, a1 = 0.f, a2 = 0.f, af = 0.f, an = 0.f;
        if (!(NR_ABLATE & 8)) {
            // this lane's members: row `chunk` of each 16x4 sub-block (lanes 16 chunk .. 16 chunk + 15);
            // bits 0..15 from the first pixel of each lane, 16..31 from the second
            uint32_t mine = ((uint32_t)(m0 >> (16 * chunk)) & 0xffffu) | (((uint32_t)(m1 >> (16 * chunk)) & 0xffffu) << 16);
            const float* rbase = rec + 16 * chunk * REC;
            // one member's contribution: its loads issued together, accumulation predicated (no branch)
            auto member = [&](int bit, bool on) {
                const float* r = rbase + (((bit >> 4) * 64) + (bit & 15)) * REC;
                const float4 ra = reinterpret_cast<const float4*>(r)[0];  // ay by ax bx
                const float4 rb = reinterpret_cast<const float4*>(r)[1];  // pos G_r G_g G_b
                const float rf = r[fsel];
                float rw = 0.f, rn = 0.f;
                if (LIT) {
                    rw = r[nsel_w];
                    rn = r[nsel_n];
                }
                const int pos = __float_as_int(rb.x);
                const int cx = tdx - (pos & 0xff), cy = tdy - (pos >> 8);
                const bool hit = on && pos >= 0 && cx >= 0 && cx <= 1 && cy >= 0 && cy <= 1;
                const float wt = hit ? (cy & 1 ? ra.y : ra.x) * (cx & 1 ? ra.w : ra.z) : 0.f;
                a0 += rb.y * wt;
                a1 += rb.z * wt;
                a2 += rb.w * wt;
                af += on ? rf : 0.f;
                if (LIT) an += on ? rw * rn : 0.f;  // corner-normal gradient tt = 3 corner + axis
            };
            // one loop over both pixel rows (2- and 4-member steps measured slower)
            for (; mine; mine &= mine - 1) member(__builtin_ctz(mine), true);
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
        if (NR_ABLATE & 4) {
            asm volatile("" ::"v"(v));
        } else {
            // one atomic per lane, address selected without branches: face lanes add this face's
            // floats; texel lanes flush the pending window when the window changes
            const bool win = wx != INT_MIN;
            const bool sw = win && (wx != pwx || wy != pwy);
            const int x = pwx + tdx, y = pwy + tdy;
            const bool tex_lane = want_tex && chunk < 3 && sw && pwx != INT_MIN && x < sh.tv.W && y < sh.tv.H;
            const bool face_lane = chunk == 3 && tt < 9;
            const float fv = face_lane ? v : pend;
            float* dst = tex_lane ? g4b + (y * sh.tv.W + x) * 4 + chunk : gFb + key * 9 + tt;
            if ((tex_lane || face_lane) && fv != 0.f) unsafeAtomicAdd(dst, fv);
            if (win) {
                pend = sw ? v : pend + v;
                pwx = wx;
                pwy = wy;
            }
        }
    }
    if (!(NR_ABLATE & 4)) {  // the last pending window
        const int x = pwx + tdx, y = pwy + tdy;
        if (want_tex && chunk < 3 && pwx != INT_MIN && x < sh.tv.W && y < sh.tv.H && pend != 0.f)
            unsafeAtomicAdd(g4b + (y * sh.tv.W + x) * 4 + chunk, pend);
    }
}

// pixels per lane, per launch: 2 (256 threads) when the grid fills the chip many times over; 1 (512
// threads, 6 waves/SIMD instead of 4) for small grids, where the waves, not the per-face work, are
// short (teapot B=4: 0.041 -> 0.035 ms; torus 1024^2 B=1: 0.059 -> 0.048 ms; on the headline and the
// car the smaller wave regions mean more face flushes: 0.405 -> 0.417 and 0.73 -> 0.84 ms).
// NR_BWD_NPX: 0 by grid size, 1 / 2 forced (timing builds).
#ifndef NR_BWD_NPX
#define NR_BWD_NPX 0
#endif
template <int FEAT>
void launch_bwd(dim3 grid, hipStream_t st, const BwdArgs& ba, const Geom& g, const Shade& sh) {
    const bool one = NR_BWD_NPX == 1 || (NR_BWD_NPX == 0 && (long long)grid.x * grid.y < 8192);
    if (one)
        hipLaunchKernelGGL((k_raster_bwd<FEAT, 1>), grid, dim3(2 * NT), 0, st, ba, g, sh);
    else
        hipLaunchKernelGGL((k_raster_bwd<FEAT, 2>), grid, dim3(NT), 0, st, ba, g, sh);
}

// gathered-face gradient -> vertex gradient: gV[b, v] = sum over (f, k) with faces[f, k] = v of gF[b, f, k]
// (the index backward of rasterize.py:232), through a CSR adjacency built once per faces tensor.
__global__ void k_vertex_grad(const float* __restrict__ gF, const int32_t* __restrict__ off,
                              const int32_t* __restrict__ ent, float* __restrict__ gV, int F, int V, long long n,
                              TexOut to) {
    if (to.out) {  // this block's slice of the texture-gradient transpose
        long long lo, hi;
        grid_slice(to.n, lo, hi);
        for (long long j = lo + threadIdx.x; j < hi; j += blockDim.x) tex_out_one(to, j);
    }
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int b = (int)(i / V), v = (int)(i % V);
    const float* base = gF + (long long)b * F * 9;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f;
    for (int e = off[v]; e < off[v + 1]; e++) {
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

// [Bt, HWp, 4] accumulation layout -> [Bt, 3, H, W]
__global__ void k_tex_out(TexOut to) {  // standalone form (no vertex gradient to carry it)
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
        sample_texture(f, w, false, fuv, sh.tv, bt, sh.eps, s, Gt, gw);
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

// ------------------------------------------------------------------------------------------------
// Camera prologue: Renderer.transform_vertices = look_at (look_at.py:5-44)
// followed by perspective (perspective.py:4-18), forward and backward, in place of the ~15 torch
// launches each way.  One thread per (item, vertex); every thread rebuilds its item's rotation from
// the eye (a few dozen flops, cheaper than a dependent launch).
struct Cam {
    float r[3][3];  // rows x, y, z axes
    float z_u[3], x_u[3], y_u[3];  // the unnormalised axes (at - eye, up x z, z x x)
};

// F.normalize(v) = v / max(|v|, 1e-12) (torch.nn.functional.normalize, dim=1)
__device__ __forceinline__ float cam_norm(const float v[3]) { return sqrtf((v[0] * v[0] + v[1] * v[1]) + v[2] * v[2]); }
__device__ __forceinline__ void cam_normalize(const float v[3], float o[3]) {
    const float n = fmaxf(cam_norm(v), 1e-12f);
    o[0] = v[0] / n, o[1] = v[1] / n, o[2] = v[2] / n;
}
__device__ __forceinline__ void cam_cross(const float a[3], const float b[3], float o[3]) {
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
}
// the look_at axes for eye e (cross products per item: the reference's dim-less torch.cross crosses
// along the batch axis at B == 3, a hazard not replicated)
__device__ __forceinline__ void cam_build(const NrCameraArgs& c, const float e[3], Cam& m) {
#pragma unroll
    for (int j = 0; j < 3; j++) m.z_u[j] = c.at[j] - e[j];
    cam_normalize(m.z_u, m.r[2]);
    cam_cross(c.up, m.r[2], m.x_u);
    cam_normalize(m.x_u, m.r[0]);
    cam_cross(m.r[2], m.r[0], m.y_u);
    cam_normalize(m.y_u, m.r[1]);
}
// backward of o = normalize(u): du = (g - o (o . g)) / |u| (|u| > eps), else g / eps
__device__ __forceinline__ void cam_normalize_bwd(const float u[3], const float o[3], const float g[3], float du[3]) {
    const float n = cam_norm(u);
    if (n > 1e-12f) {
        const float d = (o[0] * g[0] + o[1] * g[1]) + o[2] * g[2];
#pragma unroll
        for (int j = 0; j < 3; j++) du[j] = (g[j] - o[j] * d) / n;
    } else {
#pragma unroll
        for (int j = 0; j < 3; j++) du[j] = g[j] / 1e-12f;
    }
}

__device__ __forceinline__ void cam_eye(const NrCameraArgs& c, int b, float e[3]) {
    const float* ep = c.eye + (long long)b * c.eye_batch_stride;
    e[0] = ep[0], e[1] = ep[1], e[2] = ep[2];
}

__global__ void k_camera_fwd(NrCameraArgs c, float* __restrict__ out) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long long)c.batch_size * c.num_vertices) return;
    const int b = (int)(i / c.num_vertices), v = (int)(i - (long long)b * c.num_vertices);
    const float* vp = c.vertices + (long long)b * c.v_batch_stride + v * 3;
    float p[3] = {vp[0], vp[1], vp[2]};
    if (c.mode == NR_CAMERA_LOOK_AT) {
        float e[3];
        cam_eye(c, b, e);
        Cam m;
        cam_build(c, e, m);
        const float d[3] = {p[0] - e[0], p[1] - e[1], p[2] - e[2]};
#pragma unroll
        for (int k = 0; k < 3; k++) p[k] = (d[0] * m.r[k][0] + d[1] * m.r[k][1]) + d[2] * m.r[k][2];
    }
    if (c.perspective) {  // x / z / width, y / z / width (perspective.py:15-16)
        p[0] = p[0] / p[2] / c.width;
        p[1] = p[1] / p[2] / c.width;
    }
    out[i * 3 + 0] = p[0];
    out[i * 3 + 1] = p[1];
    out[i * 3 + 2] = p[2];
}

// camera-space gradient g' of vertex (b, v) from the projected-space gradient g
__device__ __forceinline__ void cam_point_bwd(const NrCameraArgs& c, const float* __restrict__ go, int b, int v,
                                              const Cam& m, const float e[3], float gq[3], float d[3]) {
    const float* vp = c.vertices + (long long)b * c.v_batch_stride + v * 3;
    const float* g = go + ((long long)b * c.num_vertices + v) * 3;
    d[0] = vp[0], d[1] = vp[1], d[2] = vp[2];
    if (c.mode == NR_CAMERA_LOOK_AT) d[0] -= e[0], d[1] -= e[1], d[2] -= e[2];
    float q[3] = {d[0], d[1], d[2]};
    if (c.mode == NR_CAMERA_LOOK_AT) {
#pragma unroll
        for (int k = 0; k < 3; k++) q[k] = (d[0] * m.r[k][0] + d[1] * m.r[k][1]) + d[2] * m.r[k][2];
    }
    gq[0] = g[0], gq[1] = g[1], gq[2] = g[2];
    if (c.perspective) {  // p = (q / z) / w: dq = dp / w / z, dz -= (dp / w) q / z^2
        const float a0 = g[0] / c.width, a1 = g[1] / c.width;
        gq[0] = a0 / q[2];
        gq[1] = a1 / q[2];
        gq[2] = g[2] - (a0 * q[0] + a1 * q[1]) / (q[2] * q[2]);
    }
}

// grad_vertices = R^T g' per vertex (summed over the items for a batch-shared mesh, in item order);
// with grad_eye, each wave also sums its items' sum_v g' (3) and sum_v g' (v - eye)^T (9) into acc[B][12]
__global__ void k_camera_bwd(NrCameraArgs c, const float* __restrict__ go, float* __restrict__ gv,
                             float* __restrict__ acc) {
    const bool shared = c.v_batch_stride == 0;
    const int nb = shared ? 1 : c.batch_size;
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = i < (long long)nb * c.num_vertices;
    const int b0 = live ? (int)(i / c.num_vertices) : 0, v = live ? (int)(i - (long long)b0 * c.num_vertices) : 0;
    float out[3] = {0.f, 0.f, 0.f};
    for (int bb = 0; bb < (shared ? c.batch_size : 1); bb++) {
        const int b = shared ? bb : b0;
        float e[3] = {0.f, 0.f, 0.f};
        Cam m;
        if (c.mode == NR_CAMERA_LOOK_AT) {
            cam_eye(c, b, e);
            cam_build(c, e, m);
        }
        float gq[3] = {0.f, 0.f, 0.f}, d[3] = {0.f, 0.f, 0.f};
        if (live) cam_point_bwd(c, go, b, v, m, e, gq, d);
        if (c.mode == NR_CAMERA_LOOK_AT) {
#pragma unroll
            for (int j = 0; j < 3; j++) out[j] += (gq[0] * m.r[0][j] + gq[1] * m.r[1][j]) + gq[2] * m.r[2][j];
        } else {
#pragma unroll
            for (int j = 0; j < 3; j++) out[j] += gq[j];
        }
        if (acc && c.mode == NR_CAMERA_LOOK_AT) {
            // items differ across a wave only at item boundaries (shared meshes loop over b uniformly)
            const int bl = __builtin_amdgcn_readfirstlane(b);
            const bool same = __builtin_amdgcn_ballot_w64(b != bl) == 0ull;
            float part[12];
#pragma unroll
            for (int k = 0; k < 3; k++) part[k] = gq[k];
#pragma unroll
            for (int k = 0; k < 3; k++)
#pragma unroll
                for (int j = 0; j < 3; j++) part[3 + 3 * k + j] = gq[k] * d[j];
            if (same) {
#pragma unroll
                for (int q = 0; q < 12; q++) {
                    const float sv = wave_sum(part[q]);
                    if ((threadIdx.x & 63) == 0 && sv != 0.f) unsafeAtomicAdd(acc + bl * 12 + q, sv);
                }
            } else if (live) {
#pragma unroll
                for (int q = 0; q < 12; q++)
                    if (part[q] != 0.f) unsafeAtomicAdd(acc + b * 12 + q, part[q]);
            }
        }
    }
    if (gv && live) {
        gv[i * 3 + 0] = out[0];
        gv[i * 3 + 1] = out[1];
        gv[i * 3 + 2] = out[2];
    }
}

// eye gradient per item from acc = (s = sum g', M = sum g' (v - eye)^T): the translation gives -R^T s,
// the rotation rows get dR = M and go back through normalize / cross to z_u = at - eye.  A shared eye
// (batch stride 0) sums its items in order.
__global__ void k_camera_eye(NrCameraArgs c, const float* __restrict__ acc, float* __restrict__ ge) {
    const bool shared = c.eye_batch_stride == 0;
    const int n = shared ? 1 : c.batch_size;
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    float tot[3] = {0.f, 0.f, 0.f};
    for (int bb = 0; bb < (shared ? c.batch_size : 1); bb++) {
        const int b = shared ? bb : t;
        const float* A = acc + b * 12;
        float e[3];
        cam_eye(c, b, e);
        Cam m;
        cam_build(c, e, m);
        float gr[3][3];
#pragma unroll
        for (int k = 0; k < 3; k++)
#pragma unroll
            for (int j = 0; j < 3; j++) gr[k][j] = A[3 + 3 * k + j];
        // y = normalize(z x x)
        float gyu[3], t3[3];
        cam_normalize_bwd(m.y_u, m.r[1], gr[1], gyu);
        cam_cross(m.r[0], gyu, t3);  // d z += x x gyu
        float gz[3] = {gr[2][0] + t3[0], gr[2][1] + t3[1], gr[2][2] + t3[2]};
        cam_cross(gyu, m.r[2], t3);  // d x += gyu x z
        float gx[3] = {gr[0][0] + t3[0], gr[0][1] + t3[1], gr[0][2] + t3[2]};
        // x = normalize(up x z): d z += gxu x up
        float gxu[3];
        cam_normalize_bwd(m.x_u, m.r[0], gx, gxu);
        cam_cross(gxu, c.up, t3);
        gz[0] += t3[0], gz[1] += t3[1], gz[2] += t3[2];
        // z = normalize(at - eye)
        float gzu[3];
        cam_normalize_bwd(m.z_u, m.r[2], gz, gzu);
#pragma unroll
        for (int j = 0; j < 3; j++) {
            const float direct = (A[0] * m.r[0][j] + A[1] * m.r[1][j]) + A[2] * m.r[2][j];
            tot[j] += -direct - gzu[j];
        }
    }
    ge[t * 3 + 0] = tot[0];
    ge[t * 3 + 1] = tot[1];
    ge[t * 3 + 2] = tot[2];
}

// textures [Bt, 3, H, W] (any strides) -> RGBA rows [Bt, HWp, 4] (alpha slot 0), read by the sampling
__global__ void k_tex_pack(TexPack pk) {  // standalone form (no face setup to carry it)
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < pk.n) tex_pack_one(pk, i);
}

int validate_raster(const NrRasterArgs* a, bool need_workspace) {
    if (!a) return fail(NR_ERR_ARGS, "null args");
    if (a->batch_size < 0 || a->num_faces < 0 || a->num_vertices < 0 || a->image_size <= 0)
        return fail(NR_ERR_ARGS, "bad sizes B=%d F=%d V=%d s=%d", a->batch_size, a->num_faces, a->num_vertices,
                    a->image_size);
    const int S = a->anti_aliasing ? 2 * a->image_size : a->image_size;
    if (S > 16384) return fail(NR_ERR_ARGS, "image too large (%d internal pixels per side)", S);
    if (nr_num_channels(a->draw_flags) == 0) return fail(NR_ERR_ARGS, "nothing to draw");
    if (a->batch_size > 0 && a->num_faces > 0 && (!a->vertices || !a->faces || !a->face_records))
        return fail(NR_ERR_ARGS, "null vertices/faces/face_records");
    if (a->batch_size > 0 && !a->face_index) return fail(NR_ERR_ARGS, "null face_index");
    if (a->draw_flags & NR_DRAW_RGB) {
        if (!a->vertices_textures || !a->faces_textures || !a->textures || !a->face_uv)
            return fail(NR_ERR_ARGS, "rgb requested without textures");
        if (a->tex_height <= 0 || a->tex_width <= 0) return fail(NR_ERR_ARGS, "bad texture size");
        if (a->num_lights < 0) return fail(NR_ERR_ARGS, "negative light count");
        if (a->num_lights > 0 && (!a->lights || !a->vertex_normals || !a->face_normals || !a->normal_offsets ||
                                  !a->normal_faces))
            return fail(NR_ERR_ARGS, "lights need lights / face_normals / vertex_normals / normal CSR buffers");
        const long long span = 2 * std::llabs(a->tex_stride_c) +
                               ((long long)a->tex_height * a->tex_width - 1) * std::llabs(a->tex_stride_p) + 1;
        if (span >= (1ll << 31)) return fail(NR_ERR_ARGS, "texture item spans 2^31 elements or more");
    }
    const Geom g = make_geom(a->num_faces, S);
    const size_t need = ws_bbox_bytes(a->batch_size, a->num_faces) + ws_mask_bytes(a->batch_size, g);
    if (need_workspace && need > 0 && (!a->workspace || a->workspace_bytes < need))
        return fail(NR_ERR_WORKSPACE, "workspace missing or too small");
    return NR_OK;
}

Shade make_shade(const NrRasterArgs* a) {
    Shade sh;
    sh.draw = a->draw_flags;
    sh.C = nr_num_channels(a->draw_flags);
    sh.eps = a->eps;
    sh.tv.tex = a->textures;
    sh.tv.sb = a->tex_stride_b;
    sh.tv.sc = (int)a->tex_stride_c;
    sh.tv.sp = (int)a->tex_stride_p;
    sh.tv.H = a->tex_height;
    sh.tv.W = a->tex_width;
    sh.tv.t4 = reinterpret_cast<const float4*>(a->textures_packed);
    sh.tv.HWp = (a->tex_height * a->tex_width + 3) & ~3;
    sh.face_uv = a->face_uv;
    sh.uv_bstride = a->vt_batch_stride ? (long long)a->num_faces * 8 : 0;
    const bool rgb = (a->draw_flags & NR_DRAW_RGB) != 0;
    sh.nl = rgb ? a->num_lights : 0;
    sh.B = a->batch_size;
    sh.V = a->num_vertices;
    sh.lights = a->lights;
    sh.vnorm = a->vertex_normals;
    sh.fidx = a->faces;
    sh.bg = rgb ? a->backgrounds : nullptr;
    sh.bg_sb = a->bg_stride_b;
    sh.bg_sc = (int)a->bg_stride_c;
    sh.bg_sy = (int)a->bg_stride_y;
    return sh;
}

}  // namespace

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

// ==================================================================================================
extern "C" {

const char* nr_last_error(void) { return g_err.c_str(); }
int nr_version(void) { return 2; }
size_t nr_raster_args_size(void) { return sizeof(NrRasterArgs); }

int nr_num_channels(int draw_flags) {
    return ((draw_flags & NR_DRAW_RGB) ? 3 : 0) + ((draw_flags & NR_DRAW_SILHOUETTES) ? 1 : 0) +
           ((draw_flags & NR_DRAW_DEPTH) ? 1 : 0);
}

size_t nr_workspace_bytes(int batch_size, int num_faces, int image_size) {
    const Geom g = make_geom(num_faces, image_size);
    return ws_bbox_bytes(batch_size, num_faces) + ws_mask_bytes(batch_size, g);
}

static int run_face_index(const float* vertices, const int32_t* faces_idx, float* face_records, int32_t* fim,
                          int B, int V, int F, int S, float near, float far, int draw_backside, float delta,
                          void* ws, size_t ws_bytes, hipStream_t st, const NrRasterArgs* ra, float* images,
                          TexPack pk) {
    const Geom g = make_geom(F, S);
    int2* bbox = (int2*)ws;
    uint32_t* mask = (uint32_t*)((char*)ws + ws_bbox_bytes(B, F));
    if (B == 0) return NR_OK;
    // the setup's idle threads repack the textures when that takes them a few texels each; with no
    // setup launch, or a texture too large for that, the repacking gets a launch of its own
    const long long setup_idle = (long long)((F + SETUP_FACES - 1) / SETUP_FACES) * B * (256 - SETUP_FACES);
    if (pk.out && (F == 0 || pk.n > 8 * setup_idle)) {
        ProfScope _p(P_TEXPACK, st);
        hipLaunchKernelGGL(k_tex_pack, dim3((unsigned)((pk.n + 255) / 256)), dim3(256), 0, st, pk);
        const int e = check_launch("k_tex_pack");
        if (e) return e;
        pk.out = nullptr;
    }
    if (F > 0) {
        dim3 grid((F + SETUP_FACES - 1) / SETUP_FACES, B);
        const bool rgb = ra && (ra->draw_flags & NR_DRAW_RGB);
        const int uv_items = rgb ? (ra->vt_batch_stride ? B : 1) : 0;
        ProfScope _p(P_SETUP, st);
        const bool lit = rgb && ra->num_lights > 0;
        if (vertices)
            hipLaunchKernelGGL(k_face_setup<true>, grid, dim3(256), 0, st, vertices, faces_idx, face_records, V, F, S,
                               draw_backside, bbox, mask, g.nbx, g.nbins, g.nwords,
                               rgb ? ra->vertices_textures : nullptr, rgb ? ra->vt_batch_stride : 0,
                               rgb ? ra->num_vertices_textures : 0, rgb ? ra->faces_textures : nullptr,
                               rgb ? ra->face_uv : nullptr, uv_items, lit ? ra->face_normals : nullptr, pk);
        else
            hipLaunchKernelGGL(k_face_setup<false>, grid, dim3(256), 0, st, nullptr, nullptr, face_records, V, F, S,
                               draw_backside, bbox, mask, g.nbx, g.nbins, g.nwords, nullptr, 0, 0, nullptr, nullptr, 0,
                               nullptr, pk);
        int e = check_launch("k_face_setup");
        if (e) return e;
        if (lit && V > 0) {
            const long long nv = (long long)B * V;
            hipLaunchKernelGGL(k_vertex_normals, dim3((unsigned)((nv + 255) / 256)), dim3(256), 0, st, ra->face_normals,
                               ra->normal_offsets, ra->normal_faces, ra->vertex_normals, F, V, nv);
            e = check_launch("k_vertex_normals");
            if (e) return e;
        }
    }
    {
        ProfScope _p(P_RASTER, st);
        // block size (k_raster_fwd notes): 256 threads when the grid alone fills the chip many times
        // over and the bins are shallow; 1024 when it does not, or when the bins are deep (F per bin
        // at the 32x32 bin granularity as the depth proxy)
        const long long blocks = (long long)g.nbins * B;
        const double faces_per_bin = (double)F / g.nbins;
        const int ntf = NR_FWD_FORCE_NT ? NR_FWD_FORCE_NT : ((blocks >= 8192 && faces_per_bin < 40.0) ? 256 : 1024);
        const int rs = vertices ? FACE_REC : 9;
        if (ntf == 256)
            hipLaunchKernelGGL(k_raster_fwd<256>, dim3(g.nbins, B), dim3(256), 0, st, face_records, rs, bbox, mask, F, g,
                               near, far, delta, fim);
        else if (ntf == 512)
            hipLaunchKernelGGL(k_raster_fwd<512>, dim3(g.nbins, B), dim3(512), 0, st, face_records, rs, bbox, mask, F, g,
                               near, far, delta, fim);
        else
            hipLaunchKernelGGL(k_raster_fwd<1024>, dim3(g.nbins, B), dim3(1024), 0, st, face_records, rs, bbox, mask, F, g,
                               near, far, delta, fim);
    }
    int e = check_launch("k_raster_fwd");
    if (e || !ra) return e;
    const int s = ra->anti_aliasing ? S / 2 : S;
    {
        ProfScope _p(P_SHADE, st);
        const Shade sh = make_shade(ra);
        if (NR_SHADE_PX == 1 || (NR_SHADE_PX == 2 && ((long long)s * s + 255) / 256 * B < 4096)) {
            const dim3 grid((unsigned)(((long long)s * s + (ra->anti_aliasing ? 63 : 255)) / (ra->anti_aliasing ? 64 : 256)), B);
            switch ((sh.nl ? 1 : 0) | (sh.bg ? 2 : 0)) {
                case 0: hipLaunchKernelGGL(k_shade_px<0>, grid, dim3(256), 0, st, face_records, fim, F, S, sh, ra->anti_aliasing, images, ra->halo); break;
                case 1: hipLaunchKernelGGL(k_shade_px<1>, grid, dim3(256), 0, st, face_records, fim, F, S, sh, ra->anti_aliasing, images, ra->halo); break;
                case 2: hipLaunchKernelGGL(k_shade_px<2>, grid, dim3(256), 0, st, face_records, fim, F, S, sh, ra->anti_aliasing, images, ra->halo); break;
                default: hipLaunchKernelGGL(k_shade_px<3>, grid, dim3(256), 0, st, face_records, fim, F, S, sh, ra->anti_aliasing, images, ra->halo); break;
            }
            return check_launch("k_shade");
        }
        const dim3 grid((unsigned)(((long long)s * s + 255) / 256), B);
        switch ((sh.nl ? 1 : 0) | (sh.bg ? 2 : 0)) {
            case 0: hipLaunchKernelGGL(k_shade<0>, grid, dim3(256), 0, st, face_records, fim, F, S, sh, ra->anti_aliasing, images, ra->halo); break;
            case 1: hipLaunchKernelGGL(k_shade<1>, grid, dim3(256), 0, st, face_records, fim, F, S, sh, ra->anti_aliasing, images, ra->halo); break;
            case 2: hipLaunchKernelGGL(k_shade<2>, grid, dim3(256), 0, st, face_records, fim, F, S, sh, ra->anti_aliasing, images, ra->halo); break;
            default: hipLaunchKernelGGL(k_shade<3>, grid, dim3(256), 0, st, face_records, fim, F, S, sh, ra->anti_aliasing, images, ra->halo); break;
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
    if (batch_size < 0 || num_faces < 0 || image_size <= 0) return fail(NR_ERR_ARGS, "bad sizes");
    const long long n = (long long)batch_size * image_size * image_size;
    if (n == 0) return NR_OK;
    hipLaunchKernelGGL(k_weight_map, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, faces,
                       face_index_map, weight_map, num_faces, image_size, n);
    return check_launch("k_weight_map");
}

int nr_mask_foreground_forward(const int32_t* face_index, const float* data_in, float* data_out, long long n, int dim,
                               void* stream) {
    if (n < 0 || dim < 0) return fail(NR_ERR_ARGS, "bad sizes");
    if (n == 0) return NR_OK;
    hipLaunchKernelGGL(k_mask_fg, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, face_index,
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
    hipLaunchKernelGGL(k_diff_bwd, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, images, grad,
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
    const int S = a->anti_aliasing ? 2 * a->image_size : a->image_size;
    return run_face_index(a->vertices, a->faces, a->face_records, a->face_index, a->batch_size, a->num_vertices,
                          a->num_faces, S, a->near, a->far, a->draw_backside, a->depth_min_delta, a->workspace,
                          a->workspace_bytes, (hipStream_t)stream, a, images, pk);
}

size_t nr_texture_packed_bytes(int texture_items, int tex_height, int tex_width) {
    if (texture_items <= 0 || tex_height <= 0 || tex_width <= 0) return 0;
    return (size_t)texture_items * ((((size_t)tex_height * tex_width) + 3) & ~size_t(3)) * 16;
}

size_t nr_halo_bytes(int batch_size, int image_size, int anti_aliasing, int draw_flags) {
    const int S = anti_aliasing ? 2 * image_size : image_size;
    if (batch_size <= 0 || image_size <= 0) return 0;
    return (size_t)batch_size * halo_item_floats(S, nr_num_channels(draw_flags)) * sizeof(float);
}

size_t nr_backward_workspace_bytes(int batch_size, int num_faces, int num_vertices, int texture_items,
                                   int tex_height, int tex_width, int num_lights) {
    const size_t hwp = ((size_t)tex_height * tex_width + 3) & ~size_t(3);
    size_t n = align_up((size_t)batch_size * num_faces * 9 * 4) + align_up((size_t)texture_items * hwp * 16);
    if (num_lights > 0)
        n += align_up((size_t)batch_size * num_faces * 9 * 4) + align_up((size_t)batch_size * num_vertices * 3 * 4);
    return n;
}

int nr_rasterize_backward(const NrRasterArgs* a, const float* grad_images, float* grad_vertices, float* grad_textures,
                          void* workspace, size_t workspace_bytes, void* stream) {
    int e = validate_raster(a, false);
    if (e) return e;
    if (a->batch_size == 0) return NR_OK;
    if (!grad_images || !grad_vertices) return fail(NR_ERR_ARGS, "null gradient buffers");
    if (a->num_faces > 0 && (!a->vertex_offsets || !a->vertex_faces))
        return fail(NR_ERR_ARGS, "missing vertex adjacency (vertex_offsets / vertex_faces)");
    const bool rgb = (a->draw_flags & NR_DRAW_RGB) && grad_textures;
    const bool lit = (a->draw_flags & NR_DRAW_RGB) && a->num_lights > 0;
    const int tex_items = rgb ? (a->tex_stride_b ? a->batch_size : 1) : 0;
    const size_t need = nr_backward_workspace_bytes(a->batch_size, a->num_faces, a->num_vertices, tex_items,
                                                    a->tex_height, a->tex_width, lit ? a->num_lights : 0);
    if (need > 0 && (!workspace || workspace_bytes < need))
        return fail(NR_ERR_WORKSPACE, "backward workspace missing or too small");
    hipStream_t st = (hipStream_t)stream;
    const int S = a->anti_aliasing ? 2 * a->image_size : a->image_size;
    const Geom g = make_geom(a->num_faces, S);
    float* gF = (float*)workspace;
    const size_t gF_bytes = align_up((size_t)a->batch_size * a->num_faces * 9 * 4);
    float* g4 = (float*)((char*)workspace + gF_bytes);
    const int HW = a->tex_height * a->tex_width;
    const int HWp = (HW + 3) & ~3;
    const size_t g4_bytes = align_up((size_t)tex_items * (((size_t)HW + 3) & ~size_t(3)) * 16);
    float* gN = lit ? (float*)((char*)workspace + gF_bytes + g4_bytes) : nullptr;
    float* gU = lit ? (float*)((char*)workspace + 2 * gF_bytes + g4_bytes) : nullptr;
    // gU is fully written by k_vnormal_bwd; the accumulators before it start at zero
    const size_t zero_bytes = lit ? 2 * gF_bytes + g4_bytes : need;
    if (zero_bytes > 0 && hipMemsetAsync(workspace, 0, zero_bytes, st) != hipSuccess) return check_launch("hipMemsetAsync");
    BwdArgs ba;
    ba.face_records = a->face_records;
    ba.fim = a->face_index;
    ba.grad_images = grad_images;
    ba.grad_faces = gF;
    ba.grad_tex4 = rgb ? g4 : nullptr;
    ba.halo = a->halo;
    ba.grad_normals = gN;
    ba.grad_bg = (a->draw_flags & NR_DRAW_RGB) && a->backgrounds ? a->grad_backgrounds : nullptr;
    ba.F = a->num_faces;
    ba.aa = a->anti_aliasing;
    ba.s = a->image_size;
    ba.HWp = HWp;
    ba.step = (float)(2. / S);
    ba.inv_step = 1.f / ba.step;
    ba.step_pow2 = (S & (S - 1)) == 0;  // step = 2/S is then a power of two: x / step == x * (S / 2)
    Shade sh = make_shade(a);
    {
        ProfScope _p(P_BWD, st);
        const dim3 grid(((S + TW - 1) / TW) * ((S + BH - 1) / BH), a->batch_size);
        switch ((lit ? 1 : 0) | (sh.bg ? 2 : 0)) {
            case 0: launch_bwd<0>(grid, st, ba, g, sh); break;
            case 1: launch_bwd<1>(grid, st, ba, g, sh); break;
            case 2: launch_bwd<2>(grid, st, ba, g, sh); break;
            default: launch_bwd<3>(grid, st, ba, g, sh); break;
        }
    }
    e = check_launch("k_raster_bwd");
    if (e) return e;
    const long long nv = (long long)a->batch_size * a->num_vertices;
    if (lit && nv > 0) {
        // lights: vertex-normal gradients -> face normals -> corner gradients (added into gF)
        hipLaunchKernelGGL(k_vnormal_bwd, dim3((unsigned)((nv + 255) / 256)), dim3(256), 0, st, gN, a->vertex_offsets,
                           a->vertex_faces, a->vertex_normals, gU, a->num_faces, a->num_vertices, nv);
        e = check_launch("k_vnormal_bwd");
        if (e) return e;
        const long long nf = (long long)a->batch_size * a->num_faces;
        if (nf > 0) {
            hipLaunchKernelGGL(k_fnormal_bwd, dim3((unsigned)((nf + 255) / 256)), dim3(256), 0, st, a->face_records,
                               a->faces, gU, gF, a->num_faces, a->num_vertices, nf);
            e = check_launch("k_fnormal_bwd");
            if (e) return e;
        }
    }
    TexOut to{};
    if (rgb) {
        to.g4 = g4;
        to.out = grad_textures;
        to.HW = HW;
        to.HWp = HWp;
        to.n = (long long)tex_items * HW;
    }
    // k_vertex_grad's blocks also carry the texture-gradient transpose when that is a few texels per
    // thread; otherwise (no vertices, or a large texture) it gets a launch of its own
    const long long vgrad_threads = (nv + 255) / 256 * 256;
    const bool carry = nv > 0 && to.n <= 8 * vgrad_threads;
    if (nv > 0) {
        {
            ProfScope _p(P_VGRAD, st);
            hipLaunchKernelGGL(k_vertex_grad, dim3((unsigned)((nv + 255) / 256)), dim3(256), 0, st, gF, a->vertex_offsets,
                               a->vertex_faces, grad_vertices, a->num_faces, a->num_vertices, nv, carry ? to : TexOut{});
        }
        e = check_launch("k_vertex_grad");
        if (e) return e;
    }
    if (to.out && to.n > 0 && !carry) {
        {
            ProfScope _p(P_TEXOUT, st);
            hipLaunchKernelGGL(k_tex_out, dim3((unsigned)((to.n + 255) / 256)), dim3(256), 0, st, to);
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
        hipLaunchKernelGGL((k_param_bwd<true, true>), grid, dim3(256), 0, st, ba, sh, S, a->faces_textures,
                           grad_vertices_textures, gvt_bstride, grad_lights);
    else if (uv)
        hipLaunchKernelGGL((k_param_bwd<true, false>), grid, dim3(256), 0, st, ba, sh, S, a->faces_textures,
                           grad_vertices_textures, gvt_bstride, grad_lights);
    else
        hipLaunchKernelGGL((k_param_bwd<false, true>), grid, dim3(256), 0, st, ba, sh, S, a->faces_textures,
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
    hipLaunchKernelGGL(k_camera_fwd, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, *c, out);
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
        hipLaunchKernelGGL(k_camera_bwd, dim3((unsigned)((nv + 255) / 256)), dim3(256), 0, st, *c, grad_out, grad_vertices, acc);
        e = check_launch("k_camera_bwd");
        if (e) return e;
    }
    if (want_eye) {
        if (nv == 0 && hipMemsetAsync(acc, 0, (size_t)c->batch_size * 12 * 4, st) != hipSuccess) return check_launch("hipMemsetAsync");
        hipLaunchKernelGGL(k_camera_eye, dim3((unsigned)((neye + 63) / 64)), dim3(64), 0, st, *c, acc, grad_eye);
        e = check_launch("k_camera_eye");
    }
    return e;
}

int nr_selftest_division(const float* a, const float* b, float* q_fast, float* q_ieee, long long n, void* stream) {
    if (n < 0 || (n > 0 && (!a || !b || !q_fast || !q_ieee))) return fail(NR_ERR_ARGS, "bad arguments");
    if (n == 0) return NR_OK;
    hipLaunchKernelGGL(k_selftest_div, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, a, b,
                       q_fast, q_ieee, n);
    return check_launch("k_selftest_div");
}

int nr_profile_enable(int on) {
    if (on && !g_prof) {
        for (int k = 0; k < P_N; k++)
            for (int j = 0; j < 2; j++)
                if (hipEventCreate(&g_prof_ev[k][j]) != hipSuccess) return fail(NR_ERR_LAUNCH, "hipEventCreate failed");
    } else if (!on && g_prof) {
        for (int k = 0; k < P_N; k++)
            for (int j = 0; j < 2; j++) (void)hipEventDestroy(g_prof_ev[k][j]);
    }
    if (!on || !g_prof)
        for (int k = 0; k < P_N; k++) g_prof_rec[k] = false;
    g_prof = on != 0;
    return NR_OK;
}

int nr_profile_read(const char* kernel, float* ms) {
    if (!kernel || !ms) return fail(NR_ERR_ARGS, "null argument");
    for (int k = 0; k < P_N; k++) {
        if (strcmp(kernel, kProfNames[k]) != 0) continue;
        if (!g_prof || !g_prof_rec[k]) return fail(NR_ERR_ARGS, "%s: no profiled launch recorded", kernel);
        if (hipEventElapsedTime(ms, g_prof_ev[k][0], g_prof_ev[k][1]) != hipSuccess)
            return fail(NR_ERR_LAUNCH, "%s: hipEventElapsedTime failed", kernel);
        return NR_OK;
    }
    return fail(NR_ERR_ARGS, "unknown kernel name %s", kernel);
}

}  // extern "C"
