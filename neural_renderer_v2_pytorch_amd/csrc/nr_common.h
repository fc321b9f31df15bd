// nr_common.h -- errors, profiling hook, geometry, the exact-division helpers, per-pixel shading (weights, texture sample, depth, lights, backgrounds), XCD tile map, block scan, texture repack helpers
// Part of nr_raster.hip (one translation unit); see that file and DESIGN.md.
#pragma once

#pragma clang fp contract(off)

namespace {

constexpr int TW = 32;             // tile width  (internal pixels)
constexpr int TH = 8;              // tile height
constexpr int NT = TW * TH;        // threads per raster block, one pixel each
constexpr int COARSE = 32;         // coarse bin edge (pixels) = forward block region; = TW, multiple of TH
// faces per setup block (SETUP_FACES / 32 bitmask words); 192: 27 blocks per item at 5120 faces, one
// round of blocks on the chip (128: 0.023 -> 0.020 ms)
constexpr int SETUP_FACES = 192;
static_assert(SETUP_FACES % 32 == 0 && SETUP_FACES <= 256, "setup block layout");
constexpr int SETUP_LDS_WORDS = 12288;  // bin-mask words built in LDS (dynamic LDS, 48 KB: 2048 bins, S <= 1448, at 192 faces)
// dynamic LDS words of a k_face_setup launch: the staged face records, or the block's mask words of
// every bin when those fit SETUP_LDS_WORDS (else the setup tests every (bin, word) from global memory)
inline int setup_lds_words(int nbins) {
    const int m = nbins * (SETUP_FACES / 32);
    const int stage = SETUP_FACES * 16;  // FACE_REC
    return (m <= SETUP_LDS_WORDS && m > stage) ? m : stage;
}
constexpr int MAXC = 5;            // max output channels
// the draw flags of a compile-time channel count (the instantiations with static channels): 5 = rgb +
// silhouettes + depth, 4 = rgb + silhouettes (rgba)
__host__ __device__ constexpr int static_draw(int cc) {
    return cc == 5 ? (NR_DRAW_RGB | NR_DRAW_SILHOUETTES | NR_DRAW_DEPTH) : (NR_DRAW_RGB | NR_DRAW_SILHOUETTES);
}

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
// a ring of start/end event pairs per kernel: nr_profile_read averages the launches recorded since
// profiling was (re)enabled, up to the last PROF_RING of them
constexpr int PROF_RING = 64;
hipEvent_t g_prof_ev[P_N][PROF_RING][2];
int g_prof_n[P_N];

// launch record (nr_last_launch): block size and NR_LAUNCH_* flags of the latest raster launches in
// this process (process-wide: torch runs a backward on its autograd device thread), so tests can
// assert the variant that actually ran.  One 64-bit word per kernel, stored and loaded with relaxed
// atomics: a reader sees one whole record; with several threads rendering at once it is one of
// their latest, not a particular thread's (a diagnostic)
struct LaunchRec {
    int threads = 0, flags = 0;
};
struct LaunchSlot {
    unsigned long long w = 0;
    void store(LaunchRec r) {
        __atomic_store_n(&w, ((unsigned long long)(unsigned)r.flags << 32) | (unsigned)r.threads, __ATOMIC_RELAXED);
    }
    LaunchRec load() const {
        const unsigned long long v = __atomic_load_n(&w, __ATOMIC_RELAXED);
        return LaunchRec{(int)(unsigned)(v & 0xffffffffu), (int)(unsigned)(v >> 32)};
    }
};
LaunchSlot g_last_fwd, g_last_bwd;

// A launch's start / stop events for the next nr_launch of this thread (armed by a ProfScope of a single
// launch): hipExtLaunchKernel stamps them from the kernel's own dispatch, where a pair of hipEventRecord
// markers around the launch measured the headline's kernels 5-7 % longer than a rocprofv3 trace of the
// same run on some boxes (round 6)
thread_local hipEvent_t t_launch_ev[2] = {nullptr, nullptr};
template <typename F, typename... Args>
void nr_launch(F kernel, dim3 grid, dim3 block, uint32_t lds, hipStream_t st, Args... args) {
    if (t_launch_ev[0]) {
        hipEvent_t a = t_launch_ev[0], b = t_launch_ev[1];
        t_launch_ev[0] = t_launch_ev[1] = nullptr;
        hipExtLaunchKernelGGL(kernel, grid, block, lds, st, a, b, 0u, args...);
    } else {
        hipLaunchKernelGGL(kernel, grid, block, lds, st, args...);
    }
}
// Profiles the launches in its scope when profiling is on.  single: the scope holds one kernel
// launch (nr_launch), which records its own start / stop; otherwise a pair of event markers brackets
// the scope (the split forward's two streams, the backward with its window reduction)
struct ProfScope {
    int k, slot;
    hipStream_t st;
    bool single;
    ProfScope(int k_, hipStream_t s, bool single_ = false) : k(k_), slot(g_prof_n[k_] % PROF_RING), st(s), single(single_) {
        if (!g_prof) return;
        if (single) {
            t_launch_ev[0] = g_prof_ev[k][slot][0];
            t_launch_ev[1] = g_prof_ev[k][slot][1];
        } else {
            (void)hipEventRecord(g_prof_ev[k][slot][0], st);
        }
    }
    ~ProfScope() {
        if (!g_prof) return;
        if (single) {
            const bool launched = t_launch_ev[0] == nullptr;
            t_launch_ev[0] = t_launch_ev[1] = nullptr;
            if (launched) g_prof_n[k]++;
        } else {
            (void)hipEventRecord(g_prof_ev[k][slot][1], st);
            g_prof_n[k]++;
        }
    }
};

struct Geom {
    int S, nbx, nby, nbins, nwords, tiles_x, tiles_y;
    int group;  // item-interleave group of the raster launches (block_item_tile); 0: per-item bands
    int B;      // items (the ordered forward's lists; set by run_face_index)
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
    g.group = 0;
    g.B = 0;
    return g;
}

size_t align_up(size_t x) { return (x + 255) & ~size_t(255); }

// workspace layout: [bbox int2 B*F][mask u32 B*nbins*nwords][per-face-group bin candidate counts u8
// B*groups*nbins][bin order i32 B*nbins][split counts] (the last three: deep-bin dispatch order,
// run_face_index; groups = the setup's face groups of SETUP_FACES)
size_t ws_bbox_bytes(int B, int F) { return align_up((size_t)B * F * sizeof(int2)); }
size_t ws_mask_bytes(int B, const Geom& g) { return align_up((size_t)B * g.nbins * g.nwords * 4); }
__host__ __device__ inline int setup_groups(const Geom& g) { return (g.nwords + SETUP_FACES / 32 - 1) / (SETUP_FACES / 32); }
size_t ws_part_bytes(int B, const Geom& g) { return align_up((size_t)B * setup_groups(g) * g.nbins); }
size_t ws_order_bytes(int B, const Geom& g) { return ws_part_bytes(B, g) + align_up((size_t)B * g.nbins * 4) + 256; }

// ------------------------------------------------------------------------------------------------
// device helpers

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
#ifdef NR_REC48
// timing builds only: 48-B records (corners and flags; the six reciprocals recomputed where a record is
// loaded), the record DESIGN.md section 9 item 5 modelled
constexpr int FACE_REC = 12;
#else
constexpr int FACE_REC = 16;
#endif
constexpr int FACE_FAST_XYZ = 1;  // x, y in {0} u [2^-20, 2^20], |z| in [2^-20, 2^20]
constexpr int FACE_FAST_ZQ = 2;   // |z + 1e-10| in [2^-20, 2^20]
constexpr int FACE_ZQ_EQ = 4;     // z + 1e-10 == z for every corner (|z| >= ~2^-6): w / (z + 1e-10) == w / z
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

#ifdef NR_REC48
__device__ __forceinline__ float face_rcp(float x);
__device__ __forceinline__ Face load_face_rec(const float* __restrict__ fr) {
    const float4* p = reinterpret_cast<const float4*>(fr);
    const float4 a = p[0], b = p[1], c = p[2];
    Face f;
    f.x0 = a.x; f.y0 = a.y; f.z0 = a.z;
    f.x1 = a.w; f.y1 = b.x; f.z1 = b.y;
    f.x2 = b.z; f.y2 = b.w; f.z2 = c.x;
    f.rz0 = face_rcp(f.z0); f.rz1 = face_rcp(f.z1); f.rz2 = face_rcp(f.z2);
    f.rq0 = face_rcp(f.z0 + 1e-10f); f.rq1 = face_rcp(f.z1 + 1e-10f); f.rq2 = face_rcp(f.z2 + 1e-10f);
    f.flags = __float_as_int(c.y);
    return f;
}
#else
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
#endif

__device__ __forceinline__ Face empty_face() {
    Face f = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    return f;
}


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
// rasterize_cuda_kernel.cu:76-77: pixel centre (float)((2.0 * i + 1 - S) / S), bit for bit: the f32
// division of nr_pixel.h, as the exact shortened sequence (numerator and S are integers of at most 15
// bits, inside div_nr's exact range; checked for every pixel of every S <= 16384 on the GPU), or an
// exact scaling when S is a power of two (measured: headline forward 0.169 -> 0.163 ms against the
// division alone).  pix_center_div: the division without the branch, where the branch would hold
// several centres live across it (the forward's static walk: 45 spilled registers)
__device__ __forceinline__ float pix_center_div(int i, int S) {
    const float s = (float)S;
    return div_nr((float)(2 * i + 1 - S), s, rcp_nr(s));
}
__device__ __forceinline__ float pix_center(int i, int S) {
    // a power-of-two S (uniform branch): the quotient is exact, a scaling by 2^-log2(S)
    if ((S & (S - 1)) == 0) return __builtin_ldexpf((float)(2 * i + 1 - S), -__builtin_ctz((unsigned)S));
    return pix_center_div(i, S);
}
// lanes (of the active ones) where a >= b or a, b unordered, i.e. !(a < b) / where a <= b or
// unordered, i.e. !(a > b): the comparison's own lane mask (llvm.amdgcn.fcmp, predicates UGE = 11,
// ULE = 13), with no per-lane boolean in between
__device__ __forceinline__ unsigned long long lane_mask_uge(float a, float b) { return __builtin_amdgcn_fcmpf(a, b, 11); }
__device__ __forceinline__ unsigned long long lane_mask_ule(float a, float b) { return __builtin_amdgcn_fcmpf(a, b, 13); }
// lane l's value of v, wave-uniform (an SGPR)
__device__ __forceinline__ float lane_value(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
// the maximum of v over the wave's 64 lanes (all active), wave-uniform; NaN lanes are ignored unless
// every lane is NaN.  A row_shr max chain leaves each 16-lane row's maximum in its lane 15 (a lane
// whose DPP source is outside its row keeps its own value).
__device__ __forceinline__ float wave_max(float v) {
    float r = v;
#define NR_MAX_SHR(ctrl) r = fmaxf(r, __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(r), __float_as_int(r), ctrl, 0xf, 0xf, false)))
    NR_MAX_SHR(0x111);  // row_shr:1
    NR_MAX_SHR(0x112);  // row_shr:2
    NR_MAX_SHR(0x114);  // row_shr:4
    NR_MAX_SHR(0x118);  // row_shr:8
#undef NR_MAX_SHR
    return fmaxf(fmaxf(lane_value(r, 15), lane_value(r, 31)), fmaxf(lane_value(r, 47), lane_value(r, 63)));
}

// |x| in [2^-e, 2^e]
__device__ __forceinline__ bool in_range(float x, float lo, float hi) { return fabsf(x) >= lo && fabsf(x) <= hi; }
// coordinate / depth magnitudes for which the face-level guard below holds: 0 or [2^-20, 2^20]
__device__ __forceinline__ bool coord_ok(float x) { return x == 0.f || in_range(x, 0x1p-20f, 0x1p20f); }
// the face record's reciprocals: rcp_nr inside the exact-division range (the only values the exact
// paths read, under the face's range flags), the IEEE 1 / x outside it (1 / 0 = inf, as v_rcp; the
// backward's gradient terms use these for every face)
__device__ __forceinline__ float face_rcp(float x) { return in_range(x, 0x1p-20f, 0x1p20f) ? rcp_nr(x) : 1.f / x; }

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

// The face's 8-float texture record (u0 v0 u1 v1 u2 v2, flag, -); flag 1 = every u, v in
// {0} u [2^-16, 2^20].  Callers load it together with the face record (both depend only on the face
// id), so the two are one memory round trip, not two.
struct FaceUV {
    float4 a, b;
};
__device__ __forceinline__ FaceUV load_face_uv(const float* __restrict__ uv) {
    FaceUV u;
    u.a = reinterpret_cast<const float4*>(uv)[0];
    u.b = reinterpret_cast<const float4*>(uv)[1];
    return u;
}

// wfast: face_weights took its exact-division path.
// G (optional, backward): upstream gradient of the rgb channels; then gw[i] = sum_c G[c] T_i[c] for
// the 4 bilinear texels, from the texel values loaded here (no second load)
// dz (optional): w_k / z_k from face_dz; on a FACE_ZQ_EQ face these are the w_k / (z_k + 1e-10) the
// sampling needs, bit for bit, and its own three divisions are skipped
__device__ __forceinline__ void sample_texture(const Face& f, const float w[3], bool wfast, const FaceUV& uvr,
                                               const TexView& tv, int bt, float eps, TexSample& s,
                                               const float* G = nullptr, float* gw = nullptr, const float* dz = nullptr) {
    const float4 uva = uvr.a, uvb = uvr.b;
    const float uvs[6] = {uva.x, uva.y, uva.z, uva.w, uvb.x, uvb.y};
    const bool fast = wfast && (f.flags & FACE_FAST_ZQ) && __float_as_int(uvb.z) != 0;
    const float z[3] = {f.z0, f.z1, f.z2};
    const float rq[3] = {f.rq0, f.rq1, f.rq2};
    float tq[3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        s.zq[k] = z[k] + 1e-10f;
        tq[k] = dz ? dz[k] : 0.f;
    }
    if (!dz || !(f.flags & FACE_ZQ_EQ)) {  // skipped when every lane's face has z + 1e-10 == z
#pragma unroll
        for (int k = 0; k < 3; k++) tq[k] = fast ? div_nr(w[k], s.zq[k], rq[k]) : w[k] / s.zq[k];
    }
    float st = 0.f;
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const float t = tq[k] + 1e-10f;
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
        // torch.minimum / maximum and min(-2) / max(-2) as gfx950's NaN-propagating v_minimum3_f32 /
        // v_maximum3_f32 (one instruction each).  Against (a < b ? a : b) with NaN propagation they differ only in the sign of a
        // zero result when the operands are +0 and -0, which leaves every value sample_texture yields
        // unchanged: floor(-0) = -0, x - floor(x) = +0 and 1 - x = 1 either way, and the gradient
        // paths compare these values (sign-blind).
        s.lo[j] = __builtin_elementwise_minimum(__builtin_elementwise_minimum(u0, u1), u2);
        s.hm[j] = __builtin_elementwise_maximum(__builtin_elementwise_maximum(u0, u1), u2) - eps;
        s.pc[j] = __builtin_elementwise_maximum(s.pr[j], s.lo[j]);
    }
    s.x = __builtin_elementwise_minimum(s.pc[0], s.hm[0]);
    s.y = __builtin_elementwise_minimum(s.pc[1], s.hm[1]);
    s.x0 = floorf(s.x);
    s.y0 = floorf(s.y);
    s.x1 = s.x0 + 1;
    s.y1 = s.y0 + 1;
    const int xi0 = (int)s.x0, yi0 = (int)s.y0, xi1 = (int)s.x1, yi1 = (int)s.y1;
    const int W = tv.W, HW = tv.H * tv.W;
    // 24-bit multiplies (full rate; v_mul_lo_u32 is quarter rate): exact for |row| < 2^23 and W < 2^23,
    // i.e. for any sample inside a texture or one texel past it (the clamp below handles the overhang)
    const int r0 = __mul24(yi0, W), r1 = __mul24(yi1, W);
    s.idx[0] = r0 + xi0;
    s.idx[1] = r0 + xi1;
    s.idx[2] = r1 + xi0;
    s.idx[3] = r1 + xi1;
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
        for (int i = 0; i < 4; i++) {
#ifdef NR_ABL_NOTEX  // timing builds only: no texel loads (constant texels)
            q4[i] = make_float4(0.25f * i, 0.5f, 0.75f, 0.f);
            (void)t4b;
#else
            q4[i] = t4b[s.idx[i]];
#endif
        }
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
        if (G) {  // gradient-only terms: fused multiply-adds (within the gradient tolerance)
            if (c == 0) {
                gw[0] = G[0] * t0;
                gw[1] = G[0] * t1;
                gw[2] = G[0] * t2;
                gw[3] = G[0] * t3;
            } else {
                gw[0] = __builtin_fmaf(G[c], t0, gw[0]);
                gw[1] = __builtin_fmaf(G[c], t1, gw[1]);
                gw[2] = __builtin_fmaf(G[c], t2, gw[2]);
                gw[3] = __builtin_fmaf(G[c], t3, gw[3]);
            }
        }
    }
}

// w_k / z_k of a foreground pixel (the exact shortened division on the fast path: weights in
// {0} u [2^-84, 1], |z| in [2^-20, 2^20]), shared by the depth and, on FACE_ZQ_EQ faces, the texture
// sampling.  The shortened form can give +0 where IEEE gives -0 for a zero weight; both callers add
// these terms to nonzero ones.
__device__ __forceinline__ void face_dz(const Face& f, const float w[3], bool wfast, float dz[3]) {
    if (wfast) {
        dz[0] = div_nr(w[0], f.z0, f.rz0);
        dz[1] = div_nr(w[1], f.z1, f.rz1);
        dz[2] = div_nr(w[2], f.z2, f.rz2);
    } else {
        dz[0] = w[0] / f.z0;
        dz[1] = w[1] / f.z1;
        dz[2] = w[2] / f.z2;
    }
}
// compute_depth_map (rasterize.py:80-88) for a foreground pixel, from face_dz's terms
__device__ __forceinline__ float depth_from_dz(const float dz[3], bool wfast) {
    const float sum = (dz[0] + dz[1]) + dz[2];
    return wfast ? recip_exact(sum) : 1.f / sum;
}
__device__ __forceinline__ float depth_value(const Face& f, const float w[3], bool wfast) {
    float dz[3];
    face_dz(f, w, wfast, dz);
    return depth_from_dz(dz, wfast);
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
__device__ __forceinline__ bool shade_needs_face(const Shade& sh) { return (sh.draw & (NR_DRAW_RGB | NR_DRAW_DEPTH)) != 0; }

// A zero record: the address the shading loads read for pixels that need no face.
__device__ float k_zero_rec[FACE_REC] = {};  // never written (a global, so the loads stay global_load)

// The face record and (rgb) texture record of pixel face id fi, loaded together and without a branch:
// a load under a branch has its wait at the branch join, which serialises the pixels' round trips.
// Pixels that need no face (background, or a render without rgb / depth) read k_zero_rec; shade_pixel
// ignores their values.
__device__ __forceinline__ void load_shading_face(const Shade& sh, const float* __restrict__ frb, int b, int fi, Face& f,
                                                  FaceUV& u) {
    const bool need = fi >= 0 && shade_needs_face(sh);
    f = load_face_rec(need ? frb + fi * FACE_REC : k_zero_rec);
    u = load_face_uv(need && (sh.draw & NR_DRAW_RGB)
                         ? sh.face_uv + (sh.uv_bstride ? (long long)b * sh.uv_bstride : 0) + fi * 8
                         : k_zero_rec);
}

// (xp, yp): the pixel centre of (x, y) (pix_center), computed by the caller, which often shares them
// between pixels (shade_quad: two columns and two rows)
__device__ __forceinline__ void shade_pixel(const Shade& sh, int b, int fi, const Face& f, const FaceUV& fuv, int x, int y,
                                            float xp, float yp, int S, float* out) {
    const bool R = (sh.draw & NR_DRAW_RGB) != 0, Sl = (sh.draw & NR_DRAW_SILHOUETTES) != 0;
    float r = 0.f, gg = 0.f, bb = 0.f, sil = 0.f, dep = 0.f;
    if (fi >= 0) sil = 1.f;
    // the weights (and the face record) only feed rgb and depth: a silhouettes-only render skips them
    if (fi >= 0 && shade_needs_face(sh)) {
        float w[3];
        const bool wfast = face_weights(xp, yp, f, w);
        float dz[3];
        face_dz(f, w, wfast, dz);
        if (R) {
            TexSample s;
            sample_texture(f, w, wfast, fuv, sh.tv, sh.tv.sb ? b : 0, sh.eps, s, nullptr, nullptr, dz);
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
        if (sh.draw & NR_DRAW_DEPTH) dep = depth_from_dz(dz, wfast);
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
// XCD.  Bands: XCD x takes a band of ny / 8 whole tile rows of each item, the band rotating with the
// item so every XCD sees every band over 8 items (balanced over the batch; measured against groups
// of neighbouring tiles and interleaved full rows in DESIGN.md).  The identity when ny is not a
// multiple of 8 (the linear id of item b starts at b * nx * ny, a multiple of 8 whenever it applies).
__device__ __forceinline__ void xcd_tile(int L, int b, int nx, int ny, int& tx, int& ty) {
    tx = L % nx;
    ty = L / nx;
    if (ny % 8 == 0) {
        const int j = L >> 3, xcd = L & 7;
        const int band = (xcd + b) & 7;
        tx = j % nx;
        ty = band * (ny >> 3) + j / nx;
    }
}

// The (item, tile) of a raster block.  group 0: item = blockIdx.y, tile by xcd_tile (bands per XCD,
// rotating with the item).  group G > 0 (G % 8 == 0, B % G == 0): items interleaved in groups of G:
// the linear block id L = blockIdx.y gridDim.x + blockIdx.x (the dispatch order) runs over groups of
// G items, and within a group over the tiles in row-major order with the item fastest (item = group
// G + L % G).  Workgroups go to XCD L % 8 = item % 8, so an XCD keeps its items' face records in its
// own L2.  The tiles run centre-out: rows from the middle row outwards, and each row's tiles from its
// middle outwards, so a centred object's foreground tiles (whose waves live ~7x longer than a
// background tile's) start first and the kernel ends on the border rows' background tiles instead of
// a tail of foreground tiles that started late (row-major order: headline fwd 0.148 -> 0.141 ms, the
// backward unchanged; same-box A/B).  Smaller groups put fewer items on the same tile at once, which
// matters to the backward's atomics into a shared texture's hot texels.  (group_for picks G on the host.)
__device__ __forceinline__ int centre_out(int k, int n) {
    const int d = (k + 1) >> 1;  // k = 0, 1, 2, 3, ... -> n/2, n/2 - 1, n/2 + 1, n/2 - 2, ...: a permutation of 0..n-1
    return (n >> 1) + ((k & 1) ? -d : d);
}
__device__ __forceinline__ void block_item_tile(int G, int nx, int ny, int& b, int& tx, int& ty) {
    if (G > 0) {
        const int L = blockIdx.y * gridDim.x + blockIdx.x;
        const int per = G * gridDim.x;  // blocks per group
        const int grp = L / per, r = L - grp * per;
        b = grp * G + r % G;
        const int t = r / G;
        tx = centre_out(t % nx, nx);
        ty = centre_out(t / nx, ny);
        return;
    }
    b = blockIdx.y;
    xcd_tile(blockIdx.x, b, nx, ny, tx, ty);
}
// The (item, bin) of a forward block from the deep-first dispatch order (k_bin_order): with B a
// multiple of 8, list x (items = x mod 8) is read by the blocks dealt to XCD x (L % 8 = x), so an
// item's bins stay on one XCD as with block_item_tile; otherwise one list for the whole grid.  part:
// 0 = the whole list, 1 = its deep prefix [0, split[x]), 2 = the rest (the split launches of
// run_face_index).  Returns -1 past the block's part (the block ends), 1 when the entry carries
// ORDER_EMPTY (no candidate face: the block skips the bin-mask scan), else 0.
constexpr int ORDER_EMPTY = 1 << 30;
// part 3 (quadrant split, a forward that does not split its list over two launches): the first
// split[x] entries of list x (its bins of >= 512 candidates, deepest first) are each walked by four
// blocks, one per 16x16 quadrant (quad 0-3: x half quad & 1, y half quad >> 1), the rest by one block
// each (quad -1); the grid holds 3 cap blocks per list more than the list, the surplus exits
// (QS: part 3 compiled in -- the dealt-quarter variant, the only one launched with it)
template <bool QS>
__device__ __forceinline__ int ordered_bin(const int* __restrict__ order, const int* __restrict__ split, int part, int B,
                                           int nbins, int nbx, int& b, int& tx, int& ty, int& quad) {
    const int L = blockIdx.y * gridDim.x + blockIdx.x;
    const bool per_xcd = B % 8 == 0;
    const int x = per_xcd ? (L & 7) : 0;
    const int n = per_xcd ? (B >> 3) * nbins : B * nbins;
    int r = per_xcd ? (L >> 3) : L;
    int hi = n;
    quad = -1;
    if (part == 1) hi = split[x];
    else if (part == 2) r += split[x];
    else if (QS && part == 3) {
        const int d = split[x];
        if (r < 4 * d) {
            quad = r & 3;
            r >>= 2;
        } else {
            r -= 3 * d;
        }
    }
    if (r >= hi) return -1;
    const int oe = order[x * n + r];
    const int e = oe & (ORDER_EMPTY - 1);
    b = e / nbins;
    const int bin = e - b * nbins;
    ty = bin / nbx;
    tx = bin - ty * nbx;
    return (oe & ORDER_EMPTY) ? 1 : 0;
}
// the interleave group for B items and a preferred group size: the preference when it divides B, else
// all B items; 0 (per-item bands) when B is not a multiple of 8
inline int group_for(int B, int pref) {
    if (pref <= 0 || B % 8 != 0) return 0;
    return B % pref == 0 ? pref : B;
}
constexpr int FWD_GROUP = 64;
constexpr int BWD_GROUP = 64;
// a shared image atlas (more than BWD_HOT_TEXELS_PER_FACE texels per face, e.g. an OBJ's materials,
// where every face of a flat-colour material samples one 2x2 patch): fewer items on a tile at once,
// so fewer waves flush the same hot texels together (the car: 0.41 ms at 16 items, 0.53 ms at 64).
// A create_textures-style atlas (one 4x4 window per face, ~16 texels per face) has no such texels
// and takes the whole batch (headline backward 0.200 -> 0.194 ms at 64; same-box A/B, r4p / r4q).
constexpr int BWD_GROUP_TEX = 16;
constexpr long long BWD_HOT_TEXELS_PER_FACE = 32;

// ------------------------------------------------------------------------------------------------
// block-wide exclusive scan of one int per thread (NW waves)
template <int NW = NT / 64>
__device__ __forceinline__ int block_scan(int v, int& total, int* lds4) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    // inclusive wave scan with DPP (VALU lane shifts, no LDS round trips): row_shr 1, 2, 4, 8 within
    // the 16-lane rows (bound_ctrl: lanes shifted in from outside the row read 0), then row_bcast:15
    // adds row r's last lane to row r + 1 and row_bcast:31 lane 31 to rows 2 and 3
    int x = v;
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, true);  // row_shr:1
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, true);  // row_shr:2
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, true);  // row_shr:4
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, true);  // row_shr:8
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
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
// Texture repacking, carried by another launch: textures [Bt, 3, H, W] (any strides) -> RGBA rows
// [Bt, HWp, 4] (alpha slot 0) before the sampling (k_face_setup's idle threads).  Each block of the
// carrying grid takes one contiguous slice, so the repacking needs no launch of its own.
struct TexPack {
    const float* __restrict__ tex;
    long long sb;
    int sc, sp, HW, HWp;
    float4* __restrict__ out;  // null: nothing to pack
    long long n;               // Bt * HWp
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
// The backward's texture-gradient accumulator (RGBA rows [Bt, HWp, 4]: the per-face window flushes and
// the direct samples) transposed into the [Bt, 3, H, W] gradient, carried by k_vertex_grad's blocks
// (or k_tex_out)
struct TexOut {
    const float* __restrict__ g4;
    float* __restrict__ out;   // null: nothing to write
    int HW, HWp;
    long long n;  // Bt * HW
};
__device__ __forceinline__ void tex_out_one(const TexOut& to, long long i) {
    const long long bt = i / to.HW;
    const int p = (int)(i % to.HW);
    const float4 v = reinterpret_cast<const float4*>(to.g4)[bt * to.HWp + p];
    to.out[(bt * 3 + 0) * to.HW + p] = v.x;
    to.out[(bt * 3 + 1) * to.HW + p] = v.y;
    to.out[(bt * 3 + 2) * to.HW + p] = v.z;
}
// this block's slice [lo, hi) of n items spread over the whole grid
// the backward's accumulators, zeroed by the forward's face setup (NrRasterArgs.bwd_workspace)
struct ZeroFill {
    float4* __restrict__ p;  // null: nothing to zero
    long long n16;           // 16-byte units
};

__device__ __forceinline__ void grid_slice(long long n, long long& lo, long long& hi) {
    const long long nb = (long long)gridDim.x * gridDim.y;
    const long long id = (long long)blockIdx.y * gridDim.x + blockIdx.x;
    const long long chunk = (n + nb - 1) / nb;
    lo = min(id * chunk, n);
    hi = min(lo + chunk, n);
}

// this block's slice of the zero fill, by all its threads, as its last work (the stores would
// otherwise count in the vmcnt waits of the block's loads)
__device__ __forceinline__ void zero_fill(const ZeroFill& zf) {
    if (!zf.p) return;
    long long lo, hi;
    grid_slice(zf.n16, lo, hi);
    for (long long i = lo + threadIdx.x; i < hi; i += blockDim.x) zf.p[i] = make_float4(0.f, 0.f, 0.f, 0.f);
}

}  // namespace
